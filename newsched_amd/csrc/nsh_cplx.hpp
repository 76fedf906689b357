// Complex arithmetic on packed (re, im) pairs and wave reductions shared by the FFT-based
// kernels (nsh_fft.hip, nsh_fir_pfft.hip). gfx950 only.
#pragma once
#include <hip/hip_runtime.h>

namespace nsh {

// A complex value is a packed pair (re, im): adds are one v_pk_add_f32, a twiddle multiply is
// one v_pk_mul_f32 + one v_pk_fma_f32 with the swizzles/negations as operand modifiers. (Written
// on HIP's float2 struct, the compiler packed the same arithmetic itself but built the operand
// pairs with ~380 v_mov per channelizer frame, a third of its VALU issue.)
typedef float cf __attribute__((ext_vector_type(2)));

// a * w with a fused second product: re = fma(-a.y, w.y, a.x w.x), im = fma(a.y, w.x, a.x w.y)
__device__ __forceinline__ cf cmulw(cf a, cf w)
{
    return __builtin_elementwise_fma(a.yy, cf{ -w.y, w.x }, a.xx * w);
}
// a * w as two packed instructions with the operand swap and the one negation as VOP3P
// modifiers: v_pk_mul (w.x broadcast) + v_pk_fma (a swapped, its low half negated, w.y broadcast).
// Written in C (cmulw) the compiler materialises (-w.y, w.x) with a v_xor + v_mov per use when w
// is loaded or loop-carried; s_nop 0 covers the packed-math read-after-write wait it would insert.
// re = fma(-a.y, w.y, w.x a.x), im = fma(a.x, w.y, w.x a.y)
__device__ __forceinline__ cf cmul_asm(cf a, cf w)
{
    cf d;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]\n\ts_nop 0\n\t"
        "v_pk_fma_f32 %0, %2, %1, %0 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]\n\ts_nop 0"
        : "=&v"(d)
        : "v"(w), "v"(a));
    return d;
}
// a * conj(w): re = fma(a.y, w.y, a.x w.x), im = fma(a.y, w.x, -a.x w.y)
__device__ __forceinline__ cf cmulc(cf a, cf w)
{
    return __builtin_elementwise_fma(a.yy, w.yx, a.xx * cf{ w.x, -w.y });
}
// multiply by -i (forward) or +i (inverse)
template <bool INV>
__device__ __forceinline__ cf rot(cf a)
{
    return INV ? cf{ -a.y, a.x } : cf{ a.y, -a.x };
}

// In-place DFT4 of (a, b, c, d): X_k = sum_n x_n W_4^{nk}, W_4 = e^{-+i pi/2}.
template <bool INV>
__device__ __forceinline__ void dft4(cf& a, cf& b, cf& c, cf& d)
{
    const cf s0 = a + c, d0 = a - c;
    const cf s1 = b + d, t = b - d;
    a = s0 + s1;
    c = s0 - s1;
    // d0 -+ i t as one packed fma each: t swapped by op_sel, (1, -1) = 1.0 with neg_hi; a
    // multiply by 1 is exact, so this rounds exactly as d0 + rot(t) (the compiler emitted rot()
    // as a v_xor + v_mov pair before each add)
    const cf pm = INV ? cf{ -1.f, 1.f } : cf{ 1.f, -1.f };
    b = __builtin_elementwise_fma(t.yx, pm, d0);
    d = __builtin_elementwise_fma(t.yx, -pm, d0);
}

// In-place DFT8, natural order in and out: X[k] = E[k] + W_8^k O[k], X[k + 4] = E[k] - W_8^k O[k]
template <bool INV>
__device__ __forceinline__ void dft8(cf (&v)[8])
{
    constexpr float R2 = 0.70710678118654757f;
    dft4<INV>(v[0], v[2], v[4], v[6]); // E[0..3] in v[0], v[2], v[4], v[6]
    dft4<INV>(v[1], v[3], v[5], v[7]); // O[0..3] in v[1], v[3], v[5], v[7]
    const cf w1 = cf{ R2, INV ? R2 : -R2 }, w3 = cf{ -R2, INV ? R2 : -R2 };
    const cf o1 = cmulw(v[3], w1), o2 = rot<INV>(v[5]), o3 = cmulw(v[7], w3);
    const cf e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6], o0 = v[1];
    v[0] = e0 + o0;
    v[4] = e0 - o0;
    v[1] = e1 + o1;
    v[5] = e1 - o1;
    v[2] = e2 + o2;
    v[6] = e2 - o2;
    v[3] = e3 + o3;
    v[7] = e3 - o3;
}

// Wave-wide unsigned max, uniform result: DPP within each 16-lane row (quad_perm xor 1, xor 2,
// row_ror 4, 8: VALU, no LDS) then the four row results by v_readlane.
__device__ __forceinline__ unsigned wave_umax(unsigned v)
{
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false));  // quad_perm [1,0,3,2]
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false));  // quad_perm [2,3,0,1]
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false)); // row_ror:4
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false)); // row_ror:8
    const unsigned a = (unsigned)__builtin_amdgcn_readlane((int)v, 0), b = (unsigned)__builtin_amdgcn_readlane((int)v, 16);
    const unsigned c = (unsigned)__builtin_amdgcn_readlane((int)v, 32), d = (unsigned)__builtin_amdgcn_readlane((int)v, 48);
    return max(max(a, b), max(c, d));
}

} // namespace nsh
