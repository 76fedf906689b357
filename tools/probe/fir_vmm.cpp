// Probe: FIR kernel time on plain hipMalloc memory vs on the VMM double-mapped ring
// (nsh_ring_alloc), same sizes as one bench launch (2^25 samples).
#include <cstdio>
#include <vector>
#include <algorithm>
#include "nsh_hip.h"
#define CK(x) do { if ((x) != 0) { printf("FAIL %s: %s\n", #x, nsh_last_error()); return 1; } } while (0)
static int timeit(const char* name, void* plan, float* x, float* y, float* h0, float* h1, long n, void* s, void* e0, void* e1)
{
    std::vector<float> t;
    for (int r = 0; r < 13; ++r) {
        CK(nsh_event_record(e0, s));
        for (int i = 0; i < 5; ++i) CK(nsh_fir_ccf(plan, x, h0, h1, y, n, s));
        CK(nsh_event_record(e1, s));
        CK(nsh_event_sync(e1));
        float ms; CK(nsh_event_elapsed_ms(e0, e1, &ms));
        if (r) t.push_back(ms / 5);
    }
    std::sort(t.begin(), t.end());
    printf("%-28s median %.1f us  min %.1f us\n", name, t[t.size() / 2] * 1e3, t[0] * 1e3);
    return 0;
}
int main()
{
    const long n = 1L << 25;
    std::vector<float> taps(127, 0.01f);
    void *x, *y, *h0, *h1, *s, *plan, *e0, *e1, *rx, *ry;
    size_t ax, ay; int dmx, dmy;
    CK(nsh_malloc(0, n * 8, &x)); CK(nsh_malloc(0, n * 8, &y));
    CK(nsh_malloc(0, 126 * 8, &h0)); CK(nsh_malloc(0, 126 * 8, &h1));
    CK(nsh_ring_alloc(0, 8 * n * 8, &rx, &ax, &dmx)); // 2 GiB rings like the bench's input
    CK(nsh_ring_alloc(0, n * 8, &ry, &ay, &dmy));
    printf("rings: %zu B (double mapped %d), %zu B (%d)\n", ax, dmx, ay, dmy);
    CK(nsh_stream_create(0, &s));
    CK(nsh_synth_cf32((float*)x, n, 0, 0, s));
    CK(nsh_synth_cf32((float*)rx, 8 * n, 0, 0, s));
    CK(nsh_memset_async(h0, 0, 126 * 8, s));
    CK(nsh_fir_plan_create(0, taps.data(), 127, 1, NSH_FIR_MFMA, &plan));
    CK(nsh_event_create(&e0)); CK(nsh_event_create(&e1));
    float* X = (float*)x; float* Y = (float*)y; float* RX = (float*)rx; float* RY = (float*)ry;
    if (timeit("malloc -> malloc", plan, X, Y, (float*)h0, (float*)h1, n, s, e0, e1)) return 1;
    if (timeit("ring -> malloc", plan, RX, Y, (float*)h0, (float*)h1, n, s, e0, e1)) return 1;
    if (timeit("malloc -> ring", plan, X, RY, (float*)h0, (float*)h1, n, s, e0, e1)) return 1;
    if (timeit("ring -> ring", plan, RX, RY, (float*)h0, (float*)h1, n, s, e0, e1)) return 1;
    if (timeit("ring+3/8 -> ring", plan, RX + 2 * 3 * n, RY, (float*)h0, (float*)h1, n, s, e0, e1)) return 1;
    if (timeit("ring(2nd map) -> ring", plan, RX + 2 * (ax / 8 - n / 2), RY, (float*)h0, (float*)h1, n, s, e0, e1)) return 1;
    if (timeit("malloc -> malloc again", plan, X, Y, (float*)h0, (float*)h1, n, s, e0, e1)) return 1;
    return 0;
}
