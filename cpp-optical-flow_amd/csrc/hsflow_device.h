// hsflow_device.h -- device helpers shared by the Jacobi kernels (K2 tiles and
// their persistent dataflow form in hsflow_kernels.hip).  Every variant builds
// the per-pixel operation sequence of hornSchunck.cpp:56-74 from these same
// functions, so they all give bit-identical (u, v).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hsflow {

// ------------------------------------------------------------------ packing
__device__ __forceinline__ uint32_t pack_grad(int ix, int iy, int it) {
    return ((uint32_t)ix & 0x7FFu) | (((uint32_t)iy & 0x7FFu) << 11) |
           (((uint32_t)it & 0x1FFu) << 22);
}
__device__ __forceinline__ void unpack_grad(uint32_t p, float &ix, float &iy,
                                            float &it) {
    // v_bfe_i32 sign-extends; the builtin is typed unsigned, so cast back to
    // int before converting (else v_cvt_f32_u32 turns -1 into 4.29e9)
    ix = (float)(int)__builtin_amdgcn_sbfe(p, 0, 11);
    iy = (float)(int)__builtin_amdgcn_sbfe(p, 11, 11);
    it = (float)(int)__builtin_amdgcn_sbfe(p, 22, 9);
}

// Cross-lane shifts by one lane over the whole wavefront: DPP wave_shr:1 /
// wave_shl:1 (GFX9-family DPP, kept on gfx950).  They fuse into the consuming
// v_add_f32 as a DPP source modifier: pure VALU, no LDS crossbar traffic.
// Lanes shifted in from outside the wave read 0 (bound_ctrl); those results
// only ever land in the region's halo columns, which are never stored.
__device__ __forceinline__ float from_left(float x) {  // lane l <- lane l-1
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x138, 0xF, 0xF, true));
}
__device__ __forceinline__ float from_right(float x) {  // lane l <- lane l+1
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x130, 0xF, 0xF, true));
}

// Keep the compiler from CSE-ing an address computation across the
// iteration loop (that would pin RH extra VGPRs for the whole solve).
__device__ __forceinline__ int launder(int x) {
    asm volatile("" : "+v"(x));
    return x;
}
typedef float f2v __attribute__((ext_vector_type(2)));
typedef uint32_t u2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v launder_v2(f2v x) {
    asm volatile("" : "+v"(x));
    return x;
}
__device__ __forceinline__ uint32_t launder_u(uint32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}
__device__ __forceinline__ float launder_f(float x) {
    asm volatile("" : "+v"(x));
    return x;
}

// The same decode for a column pair in fewer instructions (K4's per-row
// set-up): Ix and Iy by the float-magic form, one v_bitop3 per column and
// one packed op per pair instead of a v_bfe and a v_cvt per column.  The
// field's sign bit is flipped (so the field reads as Ix + 1024, 0..2047)
// and the exponent of 2^23 set in one masked xor; the float is then 2^23 +
// Ix + 1024 exactly (Iy: its field stays at bit 11, 2^23 + (Iy + 1024) 2^11,
// scaled back by an exact fma), and subtracting the constant leaves Ix
// exactly.  A zero word (the buffer loads' out-of-range value) still
// decodes to 0 in every field.  It keeps the bfe/cvt pair (its field
// overlaps the exponent bits).
__device__ __forceinline__ void unpack_grad_pair(uint32_t pe, uint32_t po, f2v &ix, f2v &iy,
                                                 f2v &it) {
    const f2v fx = {__uint_as_float((pe & 0x7FFu) ^ 0x4B000400u),
                     __uint_as_float((po & 0x7FFu) ^ 0x4B000400u)};
    const f2v fy = {__uint_as_float((pe & 0x3FF800u) ^ 0x4B200000u),
                     __uint_as_float((po & 0x3FF800u) ^ 0x4B200000u)};
    const f2v bx = {-(8388608.f + 1024.f), -(8388608.f + 1024.f)};
    const f2v sy = {1.f / 2048.f, 1.f / 2048.f};
    const f2v by = {-(4096.f + 1024.f), -(4096.f + 1024.f)};
    ix = fx + bx;
    iy = __builtin_elementwise_fma(fy, sy, by);
    it = f2v{(float)(int)__builtin_amdgcn_sbfe(pe, 22, 9),
              (float)(int)__builtin_amdgcn_sbfe(po, 22, 9)};
}

// Horizontal window sums of two columns per lane (e = even, o = odd column),
// any window 2..9.  The window of column c is [c - A, c + AR].  Lane offset j
// contributes P = e + o, e alone, o alone or nothing; the sum is evaluated
// from both ends inwards, one fused DPP add per lane spanned:
//   accL = c(-m); accL = L(accL) + c(j) for j = -m+1..-1   (L: lane l <- l-1)
//   accR = c(+m'); accR = R(accR) + c(j) for j = m'-1..1    (R: lane l <- l+1)
//   sum  = (L(accL) + c(0)) + R(accR)
// For w = 5 this is ((P(l-1) + P(l)) + e(l+1)) and ((o(l-1) + P(l)) + P(l+1)),
// for w = 3 (o(l-1) + P(l)) and (P(l) + e(l+1)).  The association depends only
// on the column's parity, so every blocking depth gives identical bits.
template <int A, int AR>
struct HWin {
    // contribution of lane offset j to the window of an even (odd = 0) or odd
    // column: 0 none, 1 e, 2 o, 3 P
    static constexpr int kind(int j, int odd) {
        const int ce = 2 * j - odd, co = 2 * j + 1 - odd;  // offsets of e, o
        const bool ie = ce >= -A && ce <= AR, io = co >= -A && co <= AR;
        return (ie ? 1 : 0) | (io ? 2 : 0);
    }
    static constexpr int left(int odd) {  // lanes spanned to the left
        int m = 0;
        while (kind(-(m + 1), odd) != 0) ++m;
        return m;
    }
    static constexpr int right(int odd) {
        int m = 0;
        while (kind(m + 1, odd) != 0) ++m;
        return m;
    }
};

template <int A, int AR, int ODD>
__device__ __forceinline__ float hwin(float e, float o, float P) {
    using H = HWin<A, AR>;
    constexpr int mL = H::left(ODD), mR = H::right(ODD);
    auto c = [&](int j) {
        const int k = H::kind(j, ODD);
        return k == 3 ? P : (k == 1 ? e : o);
    };
    float s = c(0);
    if constexpr (mL > 0) {
        float acc = c(-mL);
#pragma unroll
        for (int j = -mL + 1; j <= -1; ++j) acc = from_left(acc) + c(j);
        s = from_left(acc) + s;
    }
    if constexpr (mR > 0) {
        float acc = c(mR);
#pragma unroll
        for (int j = mR - 1; j >= 1; --j) acc = from_right(acc) + c(j);
        s = s + from_right(acc);
    }
    return launder_f(s);
}

// both columns of both fields; statements of u and v interleave after
// scheduling, so each DPP read of a just-written VGPR has independent work
// as its wait state
template <int W>
__device__ __forceinline__ void hsum_c2(float ue, float uo, float ve, float vo, float &hue,
                                        float &huo, float &hve, float &hvo) {
    constexpr int A = W - W / 2 - 1, AR = W / 2;
    const float pu = ue + uo;
    const float pv = ve + vo;
    if constexpr (W == 5) {
        // the same sums as hwin, hand-interleaved (this order keeps the
        // 10-row w = 5 kernel within 128 VGPRs without spills)
        const float au = from_left(pu) + pu;
        const float av = from_left(pv) + pv;
        const float bu = from_left(uo) + pu;
        const float bv = from_left(vo) + pv;
        hue = launder_f(au + from_right(ue));
        hve = launder_f(av + from_right(ve));
        huo = launder_f(bu + from_right(pu));
        hvo = launder_f(bv + from_right(pv));
    } else if constexpr (W == 3) {
        hue = launder_f(from_left(uo) + pu);
        hve = launder_f(from_left(vo) + pv);
        huo = launder_f(pu + from_right(ue));
        hvo = launder_f(pv + from_right(ve));
    } else {
        hue = hwin<A, AR, 0>(ue, uo, pu);
        hve = hwin<A, AR, 0>(ve, vo, pv);
        huo = hwin<A, AR, 1>(ue, uo, pu);
        hvo = hwin<A, AR, 1>(ve, vo, pv);
    }
}

// Per-pixel Jacobi operator in normalised form, set up once per pass
// (hornSchunck.cpp:63-68 rearranged): s = 1/sqrt(alpha^2 + Ix^2 + Iy^2),
// X = Ix s, Y = Iy s, T = It s; one column pair (even, odd) at a time.
// Every multiply-add of the Jacobi arithmetic is an explicit fused
// multiply-add and every other product and sum a plain operation, so no
// compiler contraction choice (-ffp-contract, which may differ between two
// instantiations of the same source) can change a bit: K2, K4 and K4's
// parallelogram segments all round alike.
__device__ __forceinline__ float fmaf_x(float a, float b, float c) {
    return __builtin_fmaf(a, b, c);
}
__device__ __forceinline__ f2v fma2(f2v a, f2v b, f2v c) {
    return __builtin_elementwise_fma(a, b, c);
}

// alpha^2 of a lane's column pair: alpha^2 inside the image, 1 outside.  A
// column outside the image reads zero gradients, so its operator is
// X = Y = T = 0 * rsq(alpha^2): 0 for any alpha but 0 * inf = NaN at
// alpha = 0, and that NaN would reach the image through the next
// iteration's window sums (the reference never computes those columns:
// hornSchunck.cpp:60-61 pads with zeros).  With 1 there they stay exactly
// 0; columns inside the image keep the caller's alpha^2 (same bits).
__device__ __forceinline__ f2v alpha2_cols(float alpha2, bool ce, bool co) {
    return f2v{ce ? alpha2 : 1.f, co ? alpha2 : 1.f};
}

__device__ __forceinline__ void op_setup(f2v alpha2, float ixe, float iye, float ite,
                                         float ixo, float iyo, float ito, f2v &X, f2v &Y,
                                         f2v &T) {
    const float se = __builtin_amdgcn_rsqf(fmaf_x(iye, iye, fmaf_x(ixe, ixe, alpha2.x)));
    const float so = __builtin_amdgcn_rsqf(fmaf_x(iyo, iyo, fmaf_x(ixo, ixo, alpha2.y)));
    X = f2v{ixe * se, ixo * so};
    Y = f2v{iye * se, iyo * so};
    T = f2v{ite * se, ito * so};
}

// One Jacobi update of a column pair from its window sums (su, sv):
// ubar = su / w^2, k = X ubar + Y vbar + T, u' = ubar - X k, v' = vbar - Y k
// (hornSchunck.cpp:60-73 with c = k s).
__device__ __forceinline__ void op_update(f2v su, f2v sv, f2v invv, f2v X, f2v Y, f2v T,
                                          f2v &nu, f2v &nv) {
    const f2v ub = su * invv, vb = sv * invv;
    const f2v k = fma2(X, ub, fma2(Y, vb, T));
    nu = fma2(-X, k, ub);
    nv = fma2(-Y, k, vb);
}

// The same update from the window means themselves (ub, vb).  Windows 3
// and 5 (K2 and K4) form the mean inside the vertical sum: the core that
// two neighbouring rows share (w = 5: M = Q + Q, four rows; w = 3: the pair
// sum Q) is scaled once, c M, and each row's mean is one fused
// multiply-add with its remaining row h, ub = fma(h, c, c M) -- one packed
// op per row and field fewer than S = h + M, ub = S c (a lone K4 wave's
// time follows its packed-op count: profiles/r06_k4_nomul_ab.txt).
__device__ __forceinline__ void op_update_mean(f2v ub, f2v vb, f2v X, f2v Y, f2v T, f2v &nu,
                                               f2v &nv) {
    const f2v k = fma2(X, ub, fma2(Y, vb, T));
    nu = fma2(-X, k, ub);
    nv = fma2(-Y, k, vb);
}

}  // namespace hsflow
