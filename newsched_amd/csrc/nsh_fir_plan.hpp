// Internal FIR plan shared by nsh_fir.hip (direct form, dispatch) and nsh_fir_mfma.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <string>
#include <vector>

struct nsh_fir_plan {
    int dev = 0;
    int L = 0;            // taps
    int Lp = 0;           // taps rounded up to a multiple of 8 (zero padded) for DIRECT
    int D = 1;            // decimation
    int algo = 0;         // resolved nsh_fir_algo
    std::vector<float> taps_host;
    float* taps_dev = nullptr;
    // MFMA form: Q tap blocks of 32, S = 2Q k-steps of 16; B fragments in lane order,
    // [part(3)][kstep(S)][lane(64)][8] bf16.
    int Q = 0;
    int S = 0;
    void* frag_dev = nullptr;
    // 16-phase form (v_mfma_f32_16x16x32_bf16): QH tap blocks of 16, (QH+1)/2 k-steps of
    // 32; [part(3)][kstep][lane(64)][8] bf16.
    int QH = 0;
    void* frag16_dev = nullptr;
    // decimating polyphase form (D = 2, 4): per phase QHD tap blocks of 16,
    // [phase][part(3)][kstep][lane][8] + [phase][part][lane][4] tail, bf16.
    int QHD = 0;
    void* fragd_dev = nullptr;
    void* fragd8_dev = nullptr; // fp16x2 polyphase fragments (k_fir_mfma11), taps scaled by 2^sh8
    // scaled fp16x2 form (decim 1, default): taps * 2^sh8 split into two fp16 terms,
    // [part(2)][kstep(S)][lane(64)][8]; null when the taps' range does not allow it.
    void* frag8_dev = nullptr;
    // k_fir_mfma12: the same scaled fp16x2 taps reversed, as 8 shifted copies per plane,
    // [part(2)][shift(8)][32Q + 24] fp16 (a lane's 8 taps of a k-step = one aligned 16-B read)
    void* frag12_dev = nullptr;
    int sh8 = 0;
    // exact fp32 form (k_fir_f32mfma, NSH_FIR_MFMA_F32): QF tap blocks of 16, the reversed taps
    // as 4 shifted copies [4][16 QF + 16] fp32
    int QF = 0;
    void* tf32_dev = nullptr;
    void* tf32q_dev = nullptr; // the exact-fp32 tile taps of k_fir_mfma12 / k_fir_mfma11, same layout
    int QFT = 0;               // their tap blocks: 2Q - 1 (k_fir_mfma12), D (QHD - 1) + 1 (k_fir_mfma11)
    void* casc = nullptr; // NSH_FIR_PFFT: a one-stage nsh_fir_cascade plan (k_fir_pfft)
    bool force_x3 = false; // NSH_FIR_MFMA_BF16X3: always the bf16x3 six-product kernel
    int variant = 0;      // MFMA kernel tuning variant (0 = default)
    int wg_per_cu = 0;    // decim-1 fp16x2 kernel: workgroups per CU over the launch (0 = auto)
    int n_cu = 0;         // the device's CU count, queried once (0 = not yet)
    std::string kernel;   // the kernel nsh_fir_ccf launches (rocprof name without namespace)
};

std::string nsh_fir_mfma_kernel_name(const nsh_fir_plan* p);
// legacy/nsh_fir_legacy.hip (make LEGACY=1) defines these; nsh_fir_mfma.hip has weak stubs
bool nsh_fir_legacy_built();
int nsh_fir_legacy_prepare(nsh_fir_plan* p);
int nsh_fir_legacy_run(const nsh_fir_plan* p, const float2* in, const float2* hist_in, float2* hist_out, float2* out,
                       int64_t n_out, hipStream_t s);
std::string nsh_fir_legacy_kernel_name(const nsh_fir_plan* p);

bool nsh_fir_mfma_supported(const nsh_fir_plan* p);
bool nsh_fir_mfma16_supported(const nsh_fir_plan* p);
int nsh_fir_mfma_prepare(nsh_fir_plan* p);
int nsh_fir_mfma_run(const nsh_fir_plan* p, const float2* in, const float2* hist_in, float2* hist_out,
                     float2* out, int64_t n_out, hipStream_t s);
int nsh_fir_mfma16_run(const nsh_fir_plan* p, const float2* in, const float2* hist_in, float2* hist_out,
                       float2* out, int64_t n_out, hipStream_t s);
bool nsh_fir_f32_supported(const nsh_fir_plan* p);
int nsh_fir_f32_prepare(nsh_fir_plan* p);
int nsh_fir_f32_run(const nsh_fir_plan* p, const float2* in, const float2* hist_in, float2* hist_out, float2* out,
                    int64_t n_out, hipStream_t s);
bool nsh_fir_cascade2_ok(const nsh_fir_plan* p1, const nsh_fir_plan* p2);
int nsh_fir_cascade2_run(const nsh_fir_plan* p1, const nsh_fir_plan* p2, const float2* in, const float2* h1i, float2* h1o,
                         const float2* h2i, float2* h2o, float2* out, int64_t n_out, hipStream_t s);
