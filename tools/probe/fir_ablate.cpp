// Probe: time the MFMA FIR (through the C-ABI) with parts of the kernel compiled out
// (NSH_FIR_ABLATE mask, see nsh_fir_mfma.hip). Built by fir_ablate.sh, one binary per mask.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "nsh_hip.h"
#define CK(x) do { if ((x) != 0) { printf("FAIL %s: %s\n", #x, nsh_last_error()); return 1; } } while (0)
int main(int argc, char** argv)
{
    const long n = 1L << 25;
    std::vector<float> taps(127);
    for (int i = 0; i < 127; ++i) taps[i] = 0.01f * (float)((i * 37) % 17 - 8);
    void *x, *y, *h0, *h1, *s, *plan, *e0, *e1;
    CK(nsh_malloc(0, n * 8, &x)); CK(nsh_malloc(0, n * 8, &y));
    CK(nsh_malloc(0, 126 * 8, &h0)); CK(nsh_malloc(0, 126 * 8, &h1));
    CK(nsh_stream_create(0, &s));
    CK(nsh_synth_cf32((float*)x, n, 0, 0, s));
    CK(nsh_memset_async(h0, 0, 126 * 8, s));
    CK(nsh_fir_plan_create(0, taps.data(), 127, 1, NSH_FIR_MFMA, &plan));
    CK(nsh_event_create(&e0)); CK(nsh_event_create(&e1));
    std::vector<float> t;
    for (int r = 0; r < 13; ++r) {
        CK(nsh_event_record(e0, s));
        for (int i = 0; i < 5; ++i) CK(nsh_fir_ccf(plan, (float*)x, (float*)h0, (float*)h1, (float*)y, n, s));
        CK(nsh_event_record(e1, s));
        CK(nsh_event_sync(e1));
        float ms; CK(nsh_event_elapsed_ms(e0, e1, &ms));
        if (r) t.push_back(ms / 5);
    }
    std::sort(t.begin(), t.end());
    printf("ablate %s: median %.1f us  min %.1f us  (%.0f GB/s at min)\n", argc > 1 ? argv[1] : "?",
           t[t.size() / 2] * 1e3, t[0] * 1e3, 16.0 * n / (t[0] * 1e-3) / 1e9);
    return 0;
}
