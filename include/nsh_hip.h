/*
 * nsh_hip.h -- C-ABI of libnsh_hip.so, the MI355X (gfx950) kernel shim behind the
 * newsched block-execution path.
 *
 * Plain C, POD arguments only (device pointers as void* or float*, sizes as size_t/int64_t,
 * streams and events as opaque void*). No C++ or torch types cross this boundary, so the
 * newsched C++17 host (meson or otherwise) links it directly, and Python reaches it with
 * ctypes.
 *
 * Every entry point returns 0 on success or a nonzero hipError_t-style code; it never
 * throws. The text of the last failure on the calling thread is in nsh_last_error().
 * The C++ wrappers (gr::hip_buffer, gr::hip::* blocks) turn nonzero codes into
 * std::runtime_error, because WORK_ERROR would spin forever in the reference executor
 * (schedulers/mt/lib/graph_executor.cpp:102-131).
 *
 * Reference interfaces each group replaces (paths relative to the reference tree):
 *   streams/events     cudaStreamCreate per buffer/block (runtime/lib/cudabuffer.cu:37,
 *                      blocklib/cuda/lib/copy.cpp:33) and cudaStreamSynchronize per work()
 *                      (copy.cpp:58, cudabuffer.cu:175) -> one stream per GPU partition,
 *                      event-ordered edges, no host syncs in steady state.
 *   ring memory        cuda_buffer's 2x cudaMalloc + mirror copies (cudabuffer.cu:27-35,
 *                      :116-176) -> one HIP-VMM allocation mapped twice back to back.
 *   nsh_memcpy_async   cuda_buffer::post_write H2D/D2H copies (cudabuffer.cu:129-157) and
 *                      copy_items (cudabuffer.cu:179-183, a host memcpy on device memory).
 *   nsh_copy           apply_copy_kernel (blocklib/cuda/lib/copy.cu:6-33), one launch per
 *                      1024-sample vector (copy.cpp:49-57) -> one launch per work().
 *   nsh_mul_const_*    multiply_const_kernel (blocklib/cuda/lib/multiply_const.cu:1-18, ff
 *                      only) and the CPU multiply_const<T>::work (blocklib/blocks/lib/
 *                      multiply_const.cpp:17-46, VOLK 32fc_s32fc / 32f_s32f).
 *   nsh_add_cc, nsh_mul_cc, nsh_fir_*, nsh_fft1024_c2c, nsh_channelizer1024
 *                      no reference counterpart; GNU Radio semantics.
 */
#ifndef NSH_HIP_H
#define NSH_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NSH_ABI_VERSION 1

/* ---- errors / device ---------------------------------------------------------- */
int nsh_abi_version(void);
const char* nsh_last_error(void);          /* thread-local; "" when no error */
int nsh_get_device_count(int* count);
int nsh_set_device(int dev);
int nsh_device_info(int dev, int* n_cu, int* clock_khz, size_t* hbm_bytes, char* arch, int arch_len);
int nsh_device_sync(void);
/* PCI bus id of `dev` ("dddd:bb:dd.f"): identifies a physical GPU across processes whose
 * device ordinals differ (per-rank HIP_VISIBLE_DEVICES makes every rank device 0). */
int nsh_device_pci_id(int dev, char* buf, int len);
/* *device = the GPU whose memory `ptr` points into (hipPointerGetAttributes, device memory
 * only: VMM rings and hipMalloc), else -1 (NULL, pinned or pageable host memory). The rccl
 * transport checks every buffer with it before handing it to librccl, so a wrong pointer is a
 * thrown error of the edge instead of a fault inside an RCCL kernel. */
int nsh_pointer_device(const void* ptr, int* device);

/* ---- streams and events (opaque hipStream_t / hipEvent_t) ---------------------- */
int nsh_stream_create(int dev, void** stream);
int nsh_stream_destroy(void* stream);
int nsh_stream_sync(void* stream);
/* 0: every operation on the stream has finished; 1: not yet; -1: error (hipStreamQuery, no wait). */
int nsh_stream_query(void* stream);
int nsh_event_create(void** event);
int nsh_event_destroy(void* event);
int nsh_event_record(void* event, void* stream);
int nsh_event_query(void* event);          /* 0 complete, 1 not ready, <0 error */
int nsh_event_sync(void* event);
int nsh_event_elapsed_ms(void* start, void* stop, float* ms);
int nsh_stream_wait_event(void* stream, void* event);
/* Times the NEXT kernel launched by this library on the calling thread (e.g. the FIR kernel of
 * the next nsh_fir_ccf / nsh_fir_cascade_ccf): the launch records start_event when the kernel
 * begins and stop_event when it ends, as part of its own dispatch (hipExtLaunchKernel), instead
 * of two event records around the call -- two fewer stream packets per timed launch. Events from
 * nsh_event_create. The setting is consumed by that one launch; (NULL, NULL) clears it. Replaces
 * the per-work() cudaEventRecord pairs a CUDA block would use for kernel timing (the reference
 * blocks do not time their kernels). */
int nsh_time_next_launch(void* start_event, void* stop_event);
/* (Every kernel entry point takes an armed pair with its launch and drops it, unrecorded, if it
 * returns without launching: the stream kernels, fft / channelizer, synth, FIR and cascade.)
 * Launches on the calling thread so far that recorded a pair set by nsh_time_next_launch (a pair
 * spanning several launches of one entry point counts each launch that records one of its two
 * events). A caller that armed a pair compares the count before and after the call it meant to
 * time: unchanged means no launch took the pair (the call launched nothing; the pair was dropped
 * unrecorded when the entry point returned). gr::schedulers::scheduler_hip's kernel timing. */
int nsh_timed_launches(uint64_t* count);
/* The shader clock while other work runs: one wave on `stream` (meant to be a second stream beside
 * the measured kernel's) reads the SQ cycle counter and the 100 MHz real-time counter, sleeps for
 * real_ticks (<= 2^32) ticks of the latter, reads both again and writes {cycles, ticks} to out_dev
 * (2 x uint64, device memory): MHz = 100 * cycles / ticks. The wave's end is bounded by the real-
 * time counter and by an iteration cap. A measurement helper (bench.py records the clock each
 * timed leg ran at); no reference counterpart. */
int nsh_clock_sample(void* out_dev, int64_t real_ticks, void* stream);

/* ---- memory ----------------------------------------------------------------------- */
enum nsh_copy_kind { NSH_H2D = 0, NSH_D2H = 1, NSH_D2D = 2, NSH_DEFAULT = 3 };
int nsh_malloc(int dev, size_t bytes, void** ptr);
int nsh_free(void* ptr);
int nsh_host_alloc(size_t bytes, void** ptr);       /* pinned, device-visible */
int nsh_host_free(void* ptr);
int nsh_memcpy_async(void* dst, const void* src, size_t bytes, int kind, void* stream);
int nsh_memset_async(void* ptr, int value, size_t bytes, void* stream);

/* Device ring for gr::hip_buffer: one physical allocation of *actual_bytes (>= min_bytes,
 * rounded to the VMM granularity) mapped twice back to back, so [base, base+2*actual)
 * aliases [base, base+actual) -- read_ptr()/write_ptr() spans are always contiguous and
 * no mirror copy is ever made. *double_mapped = 0 means VMM was unavailable and a plain
 * allocation was returned; the caller must then cap spans at the wrap point. */
int nsh_ring_alloc(int dev, size_t min_bytes, void** base, size_t* actual_bytes, int* double_mapped);
int nsh_ring_free(void* base);

/* Inter-process device memory: the "p2p" transport of gr::domain_adapter_remote (a flowgraph
 * edge between two processes whose rings are device memory). The receiving process exports a
 * nsh_malloc'd landing area (nsh_ipc_mem_export -> NSH_IPC_HANDLE_BYTES opaque bytes sent over
 * the edge's control socket); the sending process maps it on its own device
 * (nsh_ipc_mem_open) and writes it with a stream-ordered nsh_memcpy_async (same GPU: a local
 * D2D copy; different GPUs: a peer write over xGMI). Replaces the reference's direct
 * peer-buffer access between domains, which exists only inside one process
 * (runtime/include/gnuradio/domain_adapter_direct.hpp:156-172); the reference has no
 * cross-process edge. */
#define NSH_IPC_HANDLE_BYTES 64
int nsh_ipc_mem_export(void* dev_ptr, void* handle_out);
int nsh_ipc_mem_open(int dev, const void* handle, void** ptr);
int nsh_ipc_mem_close(void* ptr);

/* ---- stream kernels (n counts complex samples unless the name ends in _ff) --------- */
int nsh_copy(const void* in, void* out, size_t bytes, void* stream);
int nsh_mul_const_cc(const float* in, float* out, int64_t n, float k_re, float k_im, void* stream);
int nsh_mul_const_ff(const float* in, float* out, int64_t n, float k, void* stream);
/* m multiply_const_cc stages fused into one pass: k holds m (re,im) pairs, applied in
 * order with the same per-stage float rounding as m separate launches. */
int nsh_mul_const_chain_cc(const float* in, float* out, int64_t n, const float* k_host, int m, void* stream);
int nsh_add_cc(const float* a, const float* b, float* out, int64_t n, void* stream);
int nsh_mul_cc(const float* a, const float* b, float* out, int64_t n, void* stream);
/* multiply_const_vcc: items of vlen complex samples, y[i][j] = x[i][j] * k[j], k_dev a device
 * array of vlen (re,im) pairs (GNU Radio's vector-constant multiply; the reference has only the
 * scalar multiply_const<T> over n_items*vlen, blocklib/blocks/lib/multiply_const.cpp:33-46). */
int nsh_mul_const_vcc(const float* in, float* out, const float* k_dev, int vlen, int64_t nitems, void* stream);

/* Counter-based synthetic stream: x[i] = (u(2i), u(2i+1)),
 * u(j) = 24-bit uniform in [-1,1) from splitmix64(seed ^ j), j counted from first_index*2. */
int nsh_synth_cf32(float* out, int64_t n, uint64_t first_index, uint64_t seed, void* stream);

/* ---- FIR (fir_filter_ccf, optionally decimating) ----------------------------------
 * y[m] = sum_{k<ntaps} h[k] * x[m*decim - k], x complex fp32, h real fp32. The block keeps
 * its own (ntaps-1)-sample history because the reference block API has none
 * (runtime/include/gnuradio/sync_block.hpp:36-86). Per call:
 *   in       : n_out*decim input samples (device)
 *   hist_in  : ntaps-1 samples that precede in[0] (device; zeros at stream start; NULL = zeros,
 *              which saves the stream-start memset)
 *   hist_out : receives the ntaps-1 samples that precede the NEXT call's in[0]
 *              (must not alias hist_in -- ping-pong two buffers; NULL is an error, returned
 *              before any launch, except for NSH_FIR_PFFT plans, which then skip it)
 * NULL in / out or a NULL plan return an error before any launch.
 * algo: NSH_FIR_AUTO picks by measurement (MFMA for decim 1, 2, 4 with finite
 * taps, PFFT for decim 8 and 16, else DIRECT); NSH_FIR_DIRECT is the fp32 VALU direct form
 * (decim 1, 2, 4, 8); NSH_FIR_MFMA is the split-precision Toeplitz form on the matrix
 * cores: decim 1 on 32-sample blocks, ntaps <= 161, fp16x2 at a per-chunk power-of-two scale
 * with three products (k_fir_mfma12); decim 2 and 4 as the polyphase fp16x2 form
 * (k_fir_mfma11). In both, a 2048-input chunk whose samples (with its halo) are finite but span
 * more than the split holds takes the exact-fp32 matrix tile of NSH_FIR_MFMA_F32 (fp32 products
 * and sums; the decimators filter it undecimated and keep every decim-th output), and one
 * holding inf/NaN the fp32 direct form (exact IEEE semantics) -- at decim 1 in a second kernel
 * the call enqueues right after the first on the same stream (k_fir_exact12 filters the chunks
 * k_fir_mfma12 queued; it returns at once when none were), at decim 2 and 4 inside the same
 * launch. A plan may be used on several streams (each has its own queue of such chunks); its
 * first call on a stream, or a call with more chunks than any before on that stream, allocates
 * that queue (the latter after synchronizing the stream);
 * NSH_FIR_MFMA16 (3) and NSH_FIR_MFMA_BF16X3 (4) name bf16x3 kernels retired in round 4: plan
 * creation refuses them; NSH_FIR_MFMA_F32 is the exact-fp32 Toeplitz form on the fp32-input matrix instructions
 * (decim 1, ntaps <= 257, finite taps; no operand split: fp32 products and sums, chunks with
 * inf/NaN through the fp32 direct form in the same launch). NSH_FIR_PFFT (decim 8 and 16; AUTO
 * picks it there when ceil((ntaps-1)/decim) <= 256 and the taps are finite): the polyphase-FFT
 * overlap-save kernel of nsh_fir_cascade_ccf with one stage (k_fir_pfft2<16> / k_fir_pfft<8,1>; within fp32
 * transform rounding of the direct form, frame-relative, see nsh_fir_cascade_ccf below); decim 16
 * is only available as PFFT. */
enum nsh_fir_algo {
    NSH_FIR_AUTO = 0,
    NSH_FIR_DIRECT = 1,
    NSH_FIR_MFMA = 2,
    NSH_FIR_MFMA16 = 3,
    NSH_FIR_MFMA_BF16X3 = 4,
    NSH_FIR_MFMA_F32 = 5,
    NSH_FIR_PFFT = 6
};
int nsh_fir_plan_create(int dev, const float* taps_host, int ntaps, int decim, int algo, void** plan);
int nsh_fir_plan_destroy(void* plan);
int nsh_fir_plan_algo(void* plan);          /* the algorithm AUTO resolved to */
const char* nsh_fir_plan_kernel(void* plan); /* the kernel nsh_fir_ccf launches, e.g. "k_fir_mfma12<5>" */
int nsh_fir_ccf(void* plan, const float* in, const float* hist_in, float* hist_out,
                float* out, int64_t n_out, void* stream);

/* Decimating FIR chain in one pass (the fused form of nstages fir_filter_ccf(h_s, D_s) blocks in
 * a chain; BASELINE config C5 = 4 x fir_filter_ccf(firwin(127, 0.45), 2); replaces nstages
 * nsh_fir_ccf calls and the intermediate streams). The chain composes into one decimating filter
 *   y[m] = sum_n heq[n] x[m D - n],   D = prod D_s,   heq = h_1 * (h_2 up D_1) * (h_3 up D_1 D_2) ...
 * (composed in double at plan creation), computed by polyphase-FFT overlap-save
 * (k_fir_pfft2<16> / k_fir_pfft<8,1>; ceil((len(heq) - 1) / D) <= 256). Per call: in = n_out * D
 * samples; hist_in / hist_out = nsh_fir_cascade_hist_len(plan) = len(heq) - 1 input samples, as
 * for nsh_fir_ccf (NULL hist_in reads as zeros; hist_out may be NULL; no aliasing). A chain whose
 * stages all start from zero history is equivalent to this plan from a zero history.
 * Accuracy (not bit-identical to the staged chain): fp32 transform rounding, relative to each
 * 512-row frame's input level rather than to each output -- per output
 *   |y - y_chain| <= 1e-5 |y_chain| + 1e-6 max|x over the output's frame window| sum|heq|
 * (C5 on the synthetic stream: 2.2e-7 of max|y| against the oracle's double-accumulated chain;
 * north-star tolerance 1e-5). So quiet outputs that share a frame (8192 inputs at D = 16) with a
 * much louder burst are accurate to the burst's level, not their own
 * (tests/test_gpu_pfft.py::test_c5_mixed_amplitude_frame_relative_bound).
 * Frames holding inf/NaN are computed by the staged chain itself (fp32 direct form, stage by
 * stage over the frame's window): their NaN and inf outputs are the chain's exactly (a one-stage
 * plan: the direct form on its taps; a chain whose first stage has decimation 1: the direct form
 * on heq, which can give +-inf where the chain's inf - inf gives NaN). */
int nsh_fir_cascade_plan_create(int dev, const float* const* taps_host, const int* ntaps, const int* decims,
                                int nstages, void** plan);
int nsh_fir_cascade_plan_destroy(void* plan);
int nsh_fir_cascade_decim(void* plan);         /* D = prod D_s */
int nsh_fir_cascade_hist_len(void* plan);      /* len(heq) - 1 */
const char* nsh_fir_cascade_kernel(void* plan); /* "k_fir_pfft2<16>" (D = 16; "k_fir_pfft<16,1>" with NSH_PFFT_FORM=1), "k_fir_pfft<8,1>" */
int nsh_fir_cascade_ccf(void* plan, const float* in, const float* hist_in, float* hist_out, float* out,
                        int64_t n_out, void* stream);

/* ---- FFT (fft_vcc, 1024-point, unnormalised both ways) ------------------------------
 * frames of 1024 complex samples; inverse=1 computes sum_k X[k] e^{+2 pi i kn/1024}
 * (= 1024 * numpy.fft.ifft). nsh_channelizer1024 fuses fft -> multiply by w[1024]
 * (complex, device) -> ifft in one pass over HBM. */
int nsh_fft1024_c2c(const float* in, float* out, int64_t nframes, int inverse, void* stream);
int nsh_channelizer1024(const float* in, float* out, const float* w, int64_t nframes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NSH_HIP_H */
