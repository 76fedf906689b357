// Internal FIR plan shared by nsh_fir.hip (direct form, dispatch) and nsh_fir_mfma.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <mutex>
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
    // k_fir_mfma12 (decim 1): Q tap blocks of 32, S = 2Q k-steps of 16; the taps scaled by 2^sh8
    // and split into two fp16 terms, reversed, as NSH_V12_COPIES shifted copies per plane
    // (a lane's 8 taps of a k-step = two aligned 8-B reads)
    int Q = 0;
    int S = 0;
    void* frag12_dev = nullptr;
    // decimating polyphase form (k_fir_mfma11, D = 2, 4): per phase QHD tap blocks of 16, fp16x2
    // fragments [phase][part(2)][kstep][lane][8] + [phase][part][lane][4] tail, taps scaled by 2^sh8
    int QHD = 0;
    void* fragd8_dev = nullptr;
    int sh8 = 0;
    // exact fp32 form (k_fir_f32mfma, NSH_FIR_MFMA_F32): QF tap blocks of 16, the reversed taps
    // as 4 shifted copies [4][16 QF + 16] fp32
    int QF = 0;
    void* tf32_dev = nullptr;
    void* tf32q_dev = nullptr; // the exact-fp32 tile taps of k_fir_mfma12 / k_fir_mfma11, same layout
    int QFT = 0;               // their tap blocks: 2Q - 1 (k_fir_mfma12), D (QHD - 1) + 1 (k_fir_mfma11)
    // k_fir_mfma12's exact queue, one per stream the plan runs on (the chunks it hands to
    // k_fir_exact12: device words [count, done, entries...], nsh_fir_mfma.hip); launches on one
    // stream are ordered, so each stream's queue is empty again when its next launch starts
    struct xqueue {
        hipStream_t s;
        unsigned* d;      // two sets of `stride` words: launch k on this stream uses set k & 1
        int64_t stride;
        uint64_t launches;
    };
    mutable std::mutex xq_mu;
    mutable std::vector<xqueue> xq;
    void* casc = nullptr; // NSH_FIR_PFFT: a one-stage nsh_fir_cascade plan (k_fir_pfft)
    int dec_walk = 0;     // decim 2 / 4: bit D set = the lockstep walk (k_fir_mfma13), else k_fir_mfma11
    int walk_wgpc = 2;    // k_fir_mfma13: workgroups per CU (the lockstep row is 8 x n_cu x this / 8 wide)
    int n_cu = 0;         // the device's CU count, queried once (0 = not yet)
    std::string kernel;   // the kernel nsh_fir_ccf launches (rocprof name without namespace)
};

std::string nsh_fir_mfma_kernel_name(const nsh_fir_plan* p);
bool nsh_fir_mfma_supported(const nsh_fir_plan* p);
int nsh_fir_mfma_prepare(nsh_fir_plan* p);
int nsh_fir_mfma_run(const nsh_fir_plan* p, const float2* in, const float2* hist_in, float2* hist_out,
                     float2* out, int64_t n_out, hipStream_t s);
bool nsh_fir_f32_supported(const nsh_fir_plan* p);
int nsh_fir_f32_prepare(nsh_fir_plan* p);
int nsh_fir_f32_run(const nsh_fir_plan* p, const float2* in, const float2* hist_in, float2* hist_out, float2* out,
                    int64_t n_out, hipStream_t s);
