// libnsh_hip.so: HBM-bound stream kernels -- copy, multiply_const (cc/ff, fused chain),
// add_cc, multiply_cc and the counter-based synthetic source.
//
// One launch per work() call over all n items (the reference launches one kernel per
// 1024-sample vector and synchronises each work(): blocklib/cuda/lib/copy.cpp:49-58).
// 16 B per lane per access (global_load/store_dwordx4 = two complex samples), grid-stride
// over a grid sized for 256 CUs. Pointers that are only 8-byte aligned (an odd item
// offset in a ring) take the 8-byte path; results are identical either way.
//
// Complex products use separate rounded multiplies and one rounded add/sub, no FMA
// contraction: (ar*kr - ai*ki, ar*ki + ai*kr), the std::complex<float> / VOLK generic
// formula (reference blocklib/blocks/lib/multiply_const.cpp:33-46 ->
// volk_32fc_s32fc_multiply_32fc). With k = 1+0j this is bit-exact identity, which is what
// the reference's own tests pin (schedulers/mt/test/qa_scheduler_mt.cpp:79-135,
// qa_block_grouping.cpp:15-66).
#include "nsh_common.hpp"

#include <vector>

// hipcc contracts a*b - c*d into an FMA by default (also through the inlined bodies of
// __fmul_rn/__fsub_rn); the reference formula rounds each product, so the library is
// built with -ffp-contract=off (Makefile) and FMAs are written explicitly where wanted.

namespace {

constexpr int kBlock = 256;

// Native clang vectors (the nontemporal builtins reject HIP_vector_type wrappers).
typedef float nf4 __attribute__((ext_vector_type(4)));
typedef unsigned nu4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_nt(const float4* p)
{
    const nf4 v = __builtin_nontemporal_load(reinterpret_cast<const nf4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_nt(float4* p, float4 v)
{
    nf4 w = { v.x, v.y, v.z, v.w };
    __builtin_nontemporal_store(w, reinterpret_cast<nf4*>(p));
}

// Blocked grid-stride: each workgroup step covers kUnroll x kBlock float4s, all loads issued
// before the first store (4 x 16 B in flight per lane); the grid is sized to ~64 Ki
// workgroups so every CU has many waves in flight (tools/probe/copy_variants.hip:
// nontemporal, unroll 4, large grid = the measured copy ceiling).
constexpr int kUnroll = 4;
inline unsigned tile_grid(int64_t n_vec)
{
    int64_t g = (n_vec + (int64_t)kBlock * kUnroll - 1) / ((int64_t)kBlock * kUnroll);
    const int64_t cap = 65536;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (unsigned)g;
}
template <class F>
__device__ __forceinline__ void tiles_unary(const float4* __restrict__ in, float4* __restrict__ out, int64_t nv, F f)
{
    const int64_t step = (int64_t)gridDim.x * kBlock * kUnroll;
    for (int64_t base = (int64_t)blockIdx.x * kBlock * kUnroll + threadIdx.x; base < nv; base += step) {
        float4 v[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t i = base + (int64_t)u * kBlock;
            if (i < nv) v[u] = ld_nt(in + i);
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t i = base + (int64_t)u * kBlock;
            if (i < nv) st_nt(out + i, f(v[u]));
        }
    }
}
template <class F>
__device__ __forceinline__ void tiles_binary(const float4* __restrict__ a, const float4* __restrict__ b,
                                             float4* __restrict__ out, int64_t nv, F f)
{
    const int64_t step = (int64_t)gridDim.x * kBlock * kUnroll;
    for (int64_t base = (int64_t)blockIdx.x * kBlock * kUnroll + threadIdx.x; base < nv; base += step) {
        float4 x[kUnroll], y[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t i = base + (int64_t)u * kBlock;
            if (i < nv) {
                x[u] = ld_nt(a + i);
                y[u] = ld_nt(b + i);
            }
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t i = base + (int64_t)u * kBlock;
            if (i < nv) st_nt(out + i, f(x[u], y[u]));
        }
    }
}

__device__ __forceinline__ float2 cmul(float2 a, float2 k)
{
    return make_float2(__fsub_rn(__fmul_rn(a.x, k.x), __fmul_rn(a.y, k.y)),
                       __fadd_rn(__fmul_rn(a.x, k.y), __fmul_rn(a.y, k.x)));
}

struct op_mulc {
    float2 k;
    __device__ float2 operator()(float2 a) const { return cmul(a, k); }
};
template <int M>
struct op_chain {
    float2 k[M];
    __device__ float2 operator()(float2 a) const
    {
#pragma unroll
        for (int i = 0; i < M; ++i) a = cmul(a, k[i]);
        return a;
    }
};
struct op_chain_dyn {
    float2 k[16];
    int m;
    __device__ float2 operator()(float2 a) const
    {
        for (int i = 0; i < m; ++i) a = cmul(a, k[i]);
        return a;
    }
};

// Unary complex map, 2 samples (16 B) per lane per step.
template <class Op>
__global__ __launch_bounds__(kBlock) void k_map_c_v4(const float4* __restrict__ in,
                                                     float4* __restrict__ out,
                                                     int64_t n_vec,
                                                     Op op)
{
    tiles_unary(in, out, n_vec, [&](float4 v) {
        const float2 a = op(make_float2(v.x, v.y));
        const float2 b = op(make_float2(v.z, v.w));
        return make_float4(a.x, a.y, b.x, b.y);
    });
}
template <class Op>
__global__ __launch_bounds__(kBlock) void k_map_c_v2(const float2* __restrict__ in,
                                                     float2* __restrict__ out,
                                                     int64_t n,
                                                     Op op)
{
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        out[i] = op(in[i]);
}

template <class Op>
int launch_map_c(const float* in, float* out, int64_t n, Op op, hipStream_t s, const char* what)
{
    if (n <= 0) return 0;
    const bool a16 = ((uintptr_t)in % 16 == 0) && ((uintptr_t)out % 16 == 0);
    if (a16) {
        const int64_t nv = n / 2;
        if (nv > 0) {
            nsh::launch(k_map_c_v4<Op>, dim3(tile_grid(nv)), dim3(kBlock), 0, s,
                               (const float4*)in, (float4*)out, nv, op);
            NSH_CK_LAUNCH(what);
        }
        if (n & 1) {
            nsh::launch(k_map_c_v2<Op>, dim3(1), dim3(kBlock), 0, s,
                               (const float2*)in + (n - 1), (float2*)out + (n - 1), (int64_t)1, op);
            NSH_CK_LAUNCH(what);
        }
    } else {
        nsh::launch(k_map_c_v2<Op>, dim3(nsh::stream_grid(n, kBlock)), dim3(kBlock), 0, s,
                           (const float2*)in, (float2*)out, n, op);
        NSH_CK_LAUNCH(what);
    }
    return 0;
}

// Binary complex maps (add_cc, multiply_cc).
// y[i] = x[i] * k[i mod vlen] (multiply_const_vcc); cmul's rounding, as fft -> w -> ifft in
// k_chan1024, so the scheduler's channelizer fusion is bit-identical to the separate blocks.
template <bool POW2>
__global__ __launch_bounds__(kBlock) void k_mulc_vec(const float2* __restrict__ in, float2* __restrict__ out,
                                                     const float2* __restrict__ k, int vlen, int64_t n)
{
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        const int j = POW2 ? (int)(i & (int64_t)(vlen - 1)) : (int)(i % vlen);
        out[i] = cmul(in[i], k[j]);
    }
}

template <int OP>
__device__ __forceinline__ float2 bin(float2 a, float2 b)
{
    if constexpr (OP == 0)
        return make_float2(__fadd_rn(a.x, b.x), __fadd_rn(a.y, b.y));
    else
        return cmul(a, b);
}
template <int OP>
__global__ __launch_bounds__(kBlock) void k_bin_v4(const float4* __restrict__ a,
                                                   const float4* __restrict__ b,
                                                   float4* __restrict__ out,
                                                   int64_t n_vec)
{
    tiles_binary(a, b, out, n_vec, [](float4 x, float4 y) {
        const float2 p = bin<OP>(make_float2(x.x, x.y), make_float2(y.x, y.y));
        const float2 q = bin<OP>(make_float2(x.z, x.w), make_float2(y.z, y.w));
        return make_float4(p.x, p.y, q.x, q.y);
    });
}
template <int OP>
__global__ __launch_bounds__(kBlock) void k_bin_v2(const float2* __restrict__ a,
                                                   const float2* __restrict__ b,
                                                   float2* __restrict__ out,
                                                   int64_t n)
{
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        out[i] = bin<OP>(a[i], b[i]);
}
template <int OP>
int launch_bin(const float* a, const float* b, float* out, int64_t n, hipStream_t s, const char* what)
{
    if (n <= 0) return 0;
    const bool a16 = ((uintptr_t)a % 16 == 0) && ((uintptr_t)b % 16 == 0) && ((uintptr_t)out % 16 == 0);
    if (a16) {
        const int64_t nv = n / 2;
        if (nv > 0) {
            nsh::launch(k_bin_v4<OP>, dim3(tile_grid(nv)), dim3(kBlock), 0, s,
                               (const float4*)a, (const float4*)b, (float4*)out, nv);
            NSH_CK_LAUNCH(what);
        }
        if (n & 1) {
            nsh::launch(k_bin_v2<OP>, dim3(1), dim3(kBlock), 0, s, (const float2*)a + (n - 1),
                               (const float2*)b + (n - 1), (float2*)out + (n - 1), (int64_t)1);
            NSH_CK_LAUNCH(what);
        }
    } else {
        nsh::launch(k_bin_v2<OP>, dim3(nsh::stream_grid(n, kBlock)), dim3(kBlock), 0, s,
                           (const float2*)a, (const float2*)b, (float2*)out, n);
        NSH_CK_LAUNCH(what);
    }
    return 0;
}

// Byte copy, 16 B per lane (copy.cu:6-17 restated once per work() instead of per vector).
__global__ __launch_bounds__(kBlock) void k_copy_v4(const float4* __restrict__ in, float4* __restrict__ out, int64_t nv)
{
    tiles_unary(in, out, nv, [](float4 v) { return v; }); // bits moved as-is (no arithmetic)
}

// f32 scalar map (multiply_const_ff), 4 floats per lane.
__global__ __launch_bounds__(kBlock) void k_mulc_f_v4(const float4* __restrict__ in, float4* __restrict__ out, int64_t nv, float k)
{
    tiles_unary(in, out, nv, [k](float4 v) {
        return make_float4(__fmul_rn(v.x, k), __fmul_rn(v.y, k), __fmul_rn(v.z, k), __fmul_rn(v.w, k));
    });
}
__global__ __launch_bounds__(kBlock) void k_mulc_f_v1(const float* __restrict__ in, float* __restrict__ out, int64_t n, float k)
{
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) out[i] = __fmul_rn(in[i], k);
}

// ---- synthetic source ----------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ float u24(uint64_t seed, uint64_t j)
{
    const uint64_t z = splitmix64(seed ^ j);
    return (float)(int)(z >> 40) * (1.0f / 8388608.0f) - 1.0f; // exact: 24-bit grid on [-1,1)
}
__global__ __launch_bounds__(kBlock) void k_synth(float2* __restrict__ out, int64_t n, uint64_t first, uint64_t seed)
{
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        const uint64_t g = 2 * (first + (uint64_t)i);
        out[i] = make_float2(u24(seed, g), u24(seed, g + 1));
    }
}

} // namespace

extern "C" {

int nsh_copy(const void* in, void* out, size_t bytes, void* stream)
{
    nsh::launch_events_guard timing_guard; // an armed event pair never outlives this call
    if (bytes && (!in || !out)) return nsh::fail_msg("nsh_copy: null pointer");
    if (bytes == 0) return 0;
    hipStream_t s = nsh::S(stream);
    if ((uintptr_t)in % 16 == 0 && (uintptr_t)out % 16 == 0 && bytes >= 16) {
        const int64_t nv = (int64_t)(bytes / 16);
        nsh::launch(k_copy_v4, dim3(tile_grid(nv)), dim3(kBlock), 0, s, (const float4*)in, (float4*)out, nv);
        NSH_CK_LAUNCH("nsh_copy");
        const size_t done = (size_t)nv * 16;
        if (done < bytes)
            NSH_CK(hipMemcpyAsync((char*)out + done, (const char*)in + done, bytes - done, hipMemcpyDeviceToDevice, s));
        return 0;
    }
    NSH_CK(hipMemcpyAsync(out, in, bytes, hipMemcpyDeviceToDevice, s));
    return 0;
}

int nsh_mul_const_cc(const float* in, float* out, int64_t n, float k_re, float k_im, void* stream)
{
    nsh::launch_events_guard timing_guard; // an armed event pair never outlives this call
    if (n > 0 && (!in || !out)) return nsh::fail_msg("nsh_mul_const_cc: null pointer");
    return launch_map_c(in, out, n, op_mulc{ make_float2(k_re, k_im) }, nsh::S(stream), "nsh_mul_const_cc");
}

int nsh_mul_const_ff(const float* in, float* out, int64_t n, float k, void* stream)
{
    nsh::launch_events_guard timing_guard; // an armed event pair never outlives this call
    if (n > 0 && (!in || !out)) return nsh::fail_msg("nsh_mul_const_ff: null pointer");
    if (n <= 0) return 0;
    hipStream_t s = nsh::S(stream);
    if ((uintptr_t)in % 16 == 0 && (uintptr_t)out % 16 == 0) {
        const int64_t nv = n / 4;
        if (nv) {
            nsh::launch(k_mulc_f_v4, dim3(tile_grid(nv)), dim3(kBlock), 0, s,
                               (const float4*)in, (float4*)out, nv, k);
            NSH_CK_LAUNCH("nsh_mul_const_ff");
        }
        if (n % 4) {
            nsh::launch(k_mulc_f_v1, dim3(1), dim3(kBlock), 0, s, in + nv * 4, out + nv * 4, n % 4, k);
            NSH_CK_LAUNCH("nsh_mul_const_ff");
        }
        return 0;
    }
    nsh::launch(k_mulc_f_v1, dim3(nsh::stream_grid(n, kBlock)), dim3(kBlock), 0, s, in, out, n, k);
    NSH_CK_LAUNCH("nsh_mul_const_ff");
    return 0;
}

int nsh_mul_const_chain_cc(const float* in, float* out, int64_t n, const float* k_host, int m, void* stream)
{
    nsh::launch_events_guard timing_guard; // an armed event pair never outlives this call
    if (n > 0 && (!in || !out || (m > 0 && !k_host))) return nsh::fail_msg("nsh_mul_const_chain_cc: null pointer");
    hipStream_t s = nsh::S(stream);
    if (m <= 0) return nsh_copy(in, out, (size_t)n * 8, stream);
    if (m > 16) return nsh::fail_msg("nsh_mul_const_chain_cc: at most 16 fused stages");
    auto K = [&](int i) { return make_float2(k_host[2 * i], k_host[2 * i + 1]); };
    switch (m) {
    case 1: return launch_map_c(in, out, n, op_mulc{ K(0) }, s, "nsh_mul_const_chain_cc");
    case 2: return launch_map_c(in, out, n, op_chain<2>{ { K(0), K(1) } }, s, "nsh_mul_const_chain_cc");
    case 4: return launch_map_c(in, out, n, op_chain<4>{ { K(0), K(1), K(2), K(3) } }, s, "nsh_mul_const_chain_cc");
    default: {
        op_chain_dyn op{};
        op.m = m;
        for (int i = 0; i < m; ++i) op.k[i] = K(i);
        return launch_map_c(in, out, n, op, s, "nsh_mul_const_chain_cc");
    }
    }
}

int nsh_add_cc(const float* a, const float* b, float* out, int64_t n, void* stream)
{
    nsh::launch_events_guard timing_guard; // an armed event pair never outlives this call
    if (n > 0 && (!a || !b || !out)) return nsh::fail_msg("nsh_add_cc: null pointer");
    return launch_bin<0>(a, b, out, n, nsh::S(stream), "nsh_add_cc");
}

int nsh_mul_cc(const float* a, const float* b, float* out, int64_t n, void* stream)
{
    nsh::launch_events_guard timing_guard; // an armed event pair never outlives this call
    if (n > 0 && (!a || !b || !out)) return nsh::fail_msg("nsh_mul_cc: null pointer");
    return launch_bin<1>(a, b, out, n, nsh::S(stream), "nsh_mul_cc");
}

int nsh_mul_const_vcc(const float* in, float* out, const float* k_dev, int vlen, int64_t nitems, void* stream)
{
    nsh::launch_events_guard timing_guard; // an armed event pair never outlives this call
    if (nitems > 0 && (!in || !out || !k_dev)) return nsh::fail_msg("nsh_mul_const_vcc: null pointer");
    if (vlen <= 0 || nitems < 0) return nsh::fail_msg("nsh_mul_const_vcc: bad vlen or item count");
    const int64_t n = nitems * (int64_t)vlen;
    if (n == 0) return 0;
    hipStream_t s = nsh::S(stream);
    const unsigned grid = nsh::stream_grid(n, kBlock);
    if ((vlen & (vlen - 1)) == 0)
        nsh::launch(k_mulc_vec<true>, dim3(grid), dim3(kBlock), 0, s, (const float2*)in, (float2*)out,
                           (const float2*)k_dev, vlen, n);
    else
        nsh::launch(k_mulc_vec<false>, dim3(grid), dim3(kBlock), 0, s, (const float2*)in, (float2*)out,
                           (const float2*)k_dev, vlen, n);
    NSH_CK_LAUNCH("nsh_mul_const_vcc");
    return 0;
}

int nsh_synth_cf32(float* out, int64_t n, uint64_t first_index, uint64_t seed, void* stream)
{
    nsh::launch_events_guard timing_guard; // an armed event pair never outlives this call
    if (n > 0 && !out) return nsh::fail_msg("nsh_synth_cf32: null pointer");
    if (n <= 0) return 0;
    nsh::launch(k_synth, dim3(nsh::stream_grid(n, kBlock)), dim3(kBlock), 0, nsh::S(stream),
                       (float2*)out, n, first_index, seed);
    NSH_CK_LAUNCH("nsh_synth_cf32");
    return 0;
}

} // extern "C"
