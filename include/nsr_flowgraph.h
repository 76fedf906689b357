/*
 * nsr_flowgraph.h -- C-ABI of libnewsched.so's flowgraph runners: the BASELINE
 * configurations built from the C++ runtime (gr::flowgraph + scheduler_hip / scheduler_mt
 * + hip_buffer + gr::hip blocks), for bench.py, smoke() and the Python tests. The blocks
 * and buffers themselves are C++ (newsched_amd/runtime, schedulers, blocklib); this header
 * only exposes whole-flowgraph entry points with POD arguments.
 *
 * Returns 0 on success, nonzero on failure (text in nsr_last_error()); never throws.
 */
#ifndef NSR_FLOWGRAPH_H
#define NSR_FLOWGRAPH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* nsr_last_error(void);

/* C3 measurement flowgraph on GPU `dev` (one scheduler_hip domain):
 *   nop_source -> nop_head(n) -> [hip_buffer ring of 2n items, PRELOADED with the synthetic
 *   stream x[first_index .. first_index+n) before any run] -> hip::fir_filter_ccf(taps, algo)
 *   -> [hip_buffer D2D, 2*out_buf_bytes] -> null_sink
 * nop_source/nop_head produce items without touching memory (reference blocklib/blocks/
 * include/gnuradio/blocklib/blocks/nop_source.hpp, nop_head.hpp), so each run streams the
 * HBM-resident input through the FIR's work() calls exactly once. With first_index > 0 the
 * FIR starts with the ntaps-1 preceding samples as history (a time shard's halo,
 * regenerated from the counter-based source). n must be a multiple of 256. */
int nsr_fir_bench_create(int dev, const float* taps, int ntaps, int algo, int64_t n, uint64_t first_index,
                         uint64_t seed, size_t out_buf_bytes, int timing, void** handle);
int nsr_fir_bench_run(void* handle); /* one run (start + wait); rethrown work() errors -> rc */
/* `count` runs back to back (each a complete fg->run(): start, every work(), drain), looped in C. */
int nsr_fir_bench_runs(void* handle, int64_t count);
/* Items per run = batches * n from the next run on (nop_head::set_length): one run then streams the
 * resident n-sample input `batches` times through the FIR as one continuous stream (the ring holds
 * x twice, so every batch reads x; the FIR's history carries across batches as in any stream) --
 * one launch per batch, queued back to back on the partition stream. Default 1. */
int nsr_fir_bench_set_batches(void* handle, int64_t batches);
/* Cumulative over every timed launch since create (callers take differences around the runs
 * they time): summed FIR kernel time from HIP events that each timed launch records as part of
 * its dispatch on the partition stream (nsh_time_next_launch), the timed launches, their output
 * samples, and the algorithm the plan resolved to. */
int nsr_fir_bench_stats(void* handle, double* kernel_ms, uint64_t* launches, uint64_t* samples, int* algo);
/* Time every stride-th FIR launch from now on (default 1: every launch). A timed launch costs
 * its event pair's stream packets (~7 us per launch measured, tools/probe/stream_gap.py). */
int nsr_fir_bench_set_timing_stride(void* handle, int stride);
/* The FIR kernel the bench's block launches (after its first run), e.g. "k_fir_mfma12<5>". */
const char* nsr_fir_bench_kernel(void* handle);
/* The last `count` FIR outputs of the last run (interleaved re,im fp32) -> host. */
int nsr_fir_bench_tail(void* handle, int64_t count, float* out_host);
int nsr_fir_bench_destroy(void* handle);

/* The other single-GPU BASELINE configurations as measurement flowgraphs, built like the C3
 * bench: nop_source -> nop_head(n) -> [hip_buffer ring of 2n samples, PRELOADED with the synthetic
 * stream x[first_index ..)] -> chain -> [hip_buffer] -> null_sink in one scheduler_hip domain, with
 * the scheduler's kernel timing on (scheduler_hip::set_kernel_timing: every launching work() call
 * records its own HIP event pair). kind:
 *   NSR_CHAIN_MUL_CONST_CC  params = m (re, im) constants -> m x hip::multiply_const_cc (C2: m = 4;
 *                           scheduler_hip fuses them into one launch per work())
 *   NSR_CHAIN_CHANNELIZER   params = 1024 (re, im) weights W -> hip::fft_vcc(1024) ->
 *                           hip::multiply_const_vcc(W) -> hip::fft_vcc(1024, inverse) (C4; fused into
 *                           the channelizer); items are 1024-sample vectors, n a multiple of 2^18
 *   NSR_CHAIN_FIR           params = taps -> hip::fir_filter_ccf(taps, decim) (the decimators)
 * n counts complex samples per batch (a multiple of 256 items). */
enum nsr_chain_kind { NSR_CHAIN_MUL_CONST_CC = 1, NSR_CHAIN_CHANNELIZER = 2, NSR_CHAIN_FIR = 3 };
int nsr_chain_bench_create(int dev, int kind, const float* params, int nparams, int decim, int64_t n,
                           uint64_t first_index, uint64_t seed, size_t out_buf_bytes, void** handle);
int nsr_chain_bench_run(void* handle);
int nsr_chain_bench_set_batches(void* handle, int64_t batches); /* as nsr_fir_bench_set_batches */
/* Cumulative since create, for the block with the most kernel time (the fused block): summed
 * kernel ms, timed launches, output samples, its alias; *n_launching_blocks = blocks that launched. */
int nsr_chain_bench_stats(void* handle, double* kernel_ms, uint64_t* launches, uint64_t* samples, char* block,
                          int len, int* n_launching_blocks);
int nsr_chain_bench_tail(void* handle, int64_t count, float* out_host); /* last `count` output samples */
int nsr_chain_bench_destroy(void* handle);

/* BASELINE config C1 on the CPU (the reference's bm_copy flowgraph, schedulers/mt/bench/bm_copy.cpp:
 * 143-154): null_source -> head(n) -> blocks::copy -> null_sink on scheduler_mt (thread per block,
 * vmcircbuf edges of 2 * fixed_buf_size bytes). *seconds = wall time of fg->run(). */
int nsr_c1_run(int64_t n, size_t fixed_buf_size, double* seconds, int* threads);

/* C5 pipeline leg (BASELINE config 5): synth_source(first_index, n) -> 4 x
 * hip::fir_filter_ccf(taps, decim) -> null_sink, domain-partitioned over n_groups processes
 * (n_groups in {1, 2, 4}; group g runs stages [4g/G, 4(g+1)/G) in a scheduler_hip domain on
 * `dev`, plus the source (g = 0) / the sink (g = G-1); the other groups' domains are
 * remote_domain placeholders). Every process of one pipeline calls this with the same
 * arguments except `group` and `dev`. Rendezvous: every process of the pipeline passes the
 * same `rendezvous_dir` (a directory on this node, empty before the job; needed for
 * n_groups > 1) and the same `nonce` (job id): the receiving end of crossing i listens on a
 * kernel-chosen port on 127.0.0.1 and publishes it there as crossing<i>, the sending end waits
 * for that entry; handshakes with the wrong role or nonce, and sockets connected to
 * themselves, are refused (domain_adapter_remote.hpp).
 * transport: "auto" (RCCL when both rings are device memory on GPUs with different PCI bus
 * ids, else the TCP socket, staged through pinned memory) | "rccl" (fail otherwise) |
 * "socket". buf_bytes: scheduler_hip fixed_buf_size. n must be a multiple of decim^4.
 * Reference: graph_utils.cpp:11-205 (partition), domain_adapter_direct.hpp:236-257. */
int nsr_c5_create(int group, int n_groups, int dev, const float* taps, int ntaps, int decim, int64_t n,
                  uint64_t first_index, uint64_t seed, const char* rendezvous_dir, uint64_t nonce,
                  const char* transport, size_t buf_bytes, void** handle);
int nsr_c5_run(void* handle);
/* The transports this process's crossings negotiated, e.g. "send1:rccl,recv0:rccl". */
int nsr_c5_transport(void* handle, char* buf, int len);
/* The librccl file this process's rccl crossings bound (dladdr of ncclSend), "" if none. */
int nsr_rccl_library(char* buf, int len);
/* The rccl transport's library binding run in one process (domain_adapter_remote::rccl_self_test):
 * the crossings' dlopen/dlsym table, a 1-rank communicator on `dev`, grouped ncclSend + ncclRecv
 * of `bytes` from src to dst to `peer` (0 = self) on `stream`, drained and async-error checked.
 * src / dst must be device memory of `dev` (refused before any RCCL call otherwise). Replaces
 * nothing in the reference (its crossing is in-process, domain_adapter_direct.hpp:156-172): it
 * checks the real librccl ABI (ncclUniqueId size, ncclCommInitRank order, ncclInt8 = 0) on a
 * one-GPU box before a multi-GPU run depends on it. */
int nsr_rccl_self_test(int dev, const void* src, void* dst, size_t bytes, void* stream, int peer);
/* The last `count` outputs of the last run -> host (only the process of group n_groups-1). */
int nsr_c5_tail(void* handle, int64_t count, float* out_host);
int nsr_c5_destroy(void* handle);

/* CPU baseline: the reference scheduler_mt CPU path restated -- thread per block,
 * vmcircbuf edges of 2*fixed_buf_size bytes (reference default 32768):
 *   vector_source(x[0..nx), repeat) -> head(n) -> blocks::fir_filter_ccf -> null_sink
 * *seconds = wall time of fg->run() (threads already created). */
int nsr_cpu_fir_run(const float* taps, int ntaps, const float* x, int64_t nx, int64_t n, size_t fixed_buf_size,
                    double* seconds, int* threads);  /* *threads: scheduler_mt threads the run used */
/* The same blocks::fir_filter_ccf arithmetic with no scheduler: n outputs in `chunk`-sample calls of
 * fir_filter_ccf::filter() (what work() runs on a 4096-item scheduler_mt chunk), input read
 * cyclically from x[0..nx) (nx a multiple of chunk), on the calling thread. *seconds = wall time;
 * isa = the vector ISA the CPU blocks dispatched to (blocks::cpu_isa()). Splits the flowgraph
 * baseline's time per work() call into FIR arithmetic and scheduler hand-off. */
int nsr_cpu_fir_work_only(const float* taps, int ntaps, const float* x, int64_t nx, int64_t n, int chunk, double* seconds,
                          char* isa, int len);

#ifdef __cplusplus
}
#endif
#endif /* NSR_FLOWGRAPH_H */
