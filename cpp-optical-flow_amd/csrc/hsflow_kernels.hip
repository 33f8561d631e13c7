// hsflow_kernels.hip -- CDNA4 (gfx950) kernels of the Horn-Schunck hot path.
//
// Replaces the numeric body of HornSchunckOF/hornSchunck.cpp:19-75 (the
// reference runs it as ~15 OpenCV full-image float64 passes per iteration,
// SURVEY.md §2.1).
//
//  K1  hs_gradients_kernel   hornSchunck.cpp:19-41, once per pair.
//      Sobel Ix, Iy on I0 (reflect-101) and It = I1 - I0.  For 8-bit-valued
//      inputs these are small integers (|Ix|,|Iy| <= 1020, |It| <= 255) and
//      are packed EXACTLY into one 32-bit word (11+11+9 bit two's
//      complement), so a Jacobi pass streams 4 B of gradients per pixel
//      instead of 12.  Non-integral inputs set a per-pair flag; the Jacobi
//      kernels then read that pair's f32 gradient planes.
//  K1f hs_gradients_f32_kernel  those f32 planes, for the flagged pairs only
//      (K1 writes them for every pair only when the gradients API takes them).
//
//  K2  hs_jacobi_wg_kernel   hornSchunck.cpp:56-74, windows 3..9: one pass
//      of KB Jacobi iterations on register-resident 128-column tiles (eight
//      stacked waves per workgroup, boundary rows exchanged through LDS,
//      temporal halo KB*(W-1) rows and columns).  Runs the passes K4 does
//      not (launches too small to fill the chip with K4 segments, other
//      windows and depths, a shorter last pass).  K4 (hsflow_strips.hip)
//      streams the full-depth passes of windows 3 and 5 and gives the same
//      bits.
//
//  K2w hs_jacobi_kernel      windows 1 and 2: one wave per 64-column region.
//  K2g hs_jacobi_generic_kernel  any window up to HSFLOW_MAX_WINDOW, one
//      iteration per launch (windows > 9).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <atomic>
#include <type_traits>

#include "hsflow_internal.h"
#include "hsflow_device.h"


namespace hsflow {


__device__ __forceinline__ int reflect101(int p, int len) {
    // OpenCV borderInterpolate(BORDER_REFLECT_101) for |overshoot| <= 1.
    if (len == 1) return 0;
    p = p < 0 ? -p : p;
    return p >= len ? 2 * (len - 1) - p : p;
}

// K1 arithmetic type: double for CV_64FC1 frames (hornSchunck.cpp:23-28 take
// the Sobel sums in float64; each gradient is rounded to f32 once), float
// otherwise (exact for 8-bit-valued frames either way)
template <typename T> struct GradMath { using type = float; };
template <> struct GradMath<double> { using type = double; };

// ----------------------------------------------------------------------- K1
// Sobel dx, dy (ksize 3, reflect-101) and dt at pixel (r, c) of one pair,
// hornSchunck.cpp:27-28 and :39; exact for 8-bit-valued data.  Shared by K1
// and K1f so the f32 planes hold the same values whichever kernel writes them.
template <typename T, typename F>
__device__ __forceinline__ void sobel_at(const T *a, const T *b, int rows, int cols, int r,
                                         int c, F &dx, F &dy, F &dt, F &z_0, F &nxt) {
    const int rm = reflect101(r - 1, rows), rp = reflect101(r + 1, rows);
    const int cm = reflect101(c - 1, cols), cp = reflect101(c + 1, cols);
    const T *pm = a + (size_t)rm * cols, *p0 = a + (size_t)r * cols,
            *pp = a + (size_t)rp * cols;
    const F m_m = (F)pm[cm], m_0 = (F)pm[c], m_p = (F)pm[cp];
    const F z_m = (F)p0[cm], z_p = (F)p0[cp];
    const F p_m = (F)pp[cm], p_0 = (F)pp[c], p_p = (F)pp[cp];
    z_0 = (F)p0[c];
    nxt = (F)b[(size_t)r * cols + c];
    dx = (m_p - m_m) + (F)2 * (z_p - z_m) + (p_p - p_m);
    dy = (p_m - m_m) + (F)2 * (p_0 - m_0) + (p_p - m_p);
    dt = nxt - z_0;
}

// K1: packed exact gradients and the per-pair integrality flag; with PLANES
// also the f32 gradient planes (the gradients API hands them out).  Without
// PLANES the planes are written by K1f for the flagged pairs only -- the
// only pairs whose Jacobi passes read them -- which takes 12 of K1's 24 B
// per pixel of f32 frames off every solve.
// One thread per column pair (c, c + 1) and kK1Rows rows, walking down with
// the three I0 rows of its 3 x 4 neighbourhood in registers (each row
// loaded once: 4 I0 and 2 I1 loads per pixel pair and row, against 20 with
// a pixel per thread re-reading its 3 x 3 window); the arithmetic is
// sobel_at's, term for term.  Block 64 x 4 threads = 128 columns x 4 kK1Rows
// rows; grid (ceil(cols/128), ceil(rows/(4 kK1Rows)), batch).
constexpr int kK1Rows = 8;
template <typename T, bool PLANES>
__global__ __launch_bounds__(256) void hs_gradients_kernel(
    const T *__restrict__ I0, const T *__restrict__ I1, int rows, int cols,
    uint32_t *__restrict__ gpack, float *__restrict__ gx, float *__restrict__ gy,
    float *__restrict__ gt, uint32_t *__restrict__ flags) {
    using F = typename GradMath<T>::type;
    const int c = 2 * (blockIdx.x * 64 + threadIdx.x);
    const int r0 = (blockIdx.y * 4 + threadIdx.y) * kK1Rows;
    const size_t plane = (size_t)rows * cols;
    bool bad = false;
    if (c < cols && r0 < rows) {
        const T *a = I0 + blockIdx.z * plane, *b = I1 + blockIdx.z * plane;
        const bool two = c + 1 < cols;
        // the neighbourhood's columns: c - 1, c, c + 1, c + 2 (reflect-101)
        const int x0 = reflect101(c - 1, cols), x2 = reflect101(c + 1, cols);
        const int x3 = reflect101(c + 2, cols);
        auto ld = [&](int r, F (&q)[4]) {
            const T *p = a + (size_t)reflect101(r, rows) * cols;
            q[0] = (F)p[x0];
            q[1] = (F)p[c];
            q[2] = (F)p[x2];
            q[3] = (F)p[x3];
        };
        F pm[4], p0[4], pp[4];
        ld(r0 - 1, pm);
        ld(r0, p0);
        const int r1 = min(rows, r0 + kK1Rows);
        for (int r = r0; r < r1; ++r) {
            ld(r + 1, pp);
            const size_t o = blockIdx.z * plane + (size_t)r * cols + c;
            const T *bn = b + (size_t)r * cols + c;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (k == 1 && !two) break;
                // column c + k: left k, centre k + 1, right k + 2 of the rows
                const F m_m = pm[k], m_0 = pm[k + 1], m_p = pm[k + 2];
                const F z_m = p0[k], z_0 = p0[k + 1], z_p = p0[k + 2];
                const F p_m = pp[k], p_0 = pp[k + 1], p_p = pp[k + 2];
                const F nxt = (F)bn[k];
                const F dx = (m_p - m_m) + (F)2 * (z_p - z_m) + (p_p - p_m);
                const F dy = (p_m - m_m) + (F)2 * (p_0 - m_0) + (p_p - m_p);
                const F dt = nxt - z_0;
                if constexpr (PLANES) {
                    gx[o + k] = (float)dx;
                    gy[o + k] = (float)dy;
                    gt[o + k] = (float)dt;
                }
                // packed form is exact iff both frames are integers in [0, 255]
                bad |= !(z_0 == rint(z_0) && nxt == rint(nxt) && z_0 >= (F)0 &&
                         z_0 <= (F)255 && nxt >= (F)0 && nxt <= (F)255);
                gpack[o + k] = pack_grad((int)dx, (int)dy, (int)dt);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                pm[k] = p0[k];
                p0[k] = pp[k];
            }
        }
    }
    if constexpr (std::is_same<T, uint8_t>::value) {
        // 8-bit frames are always integral: the flag is a plain 0, stored
        // by one thread of the pair (no zeroing memset before K1)
        if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && threadIdx.y == 0)
            flags[blockIdx.z] = 0u;
    } else if (__any(bad) && (threadIdx.x & 63) == 0) {
        atomicOr(&flags[blockIdx.z], 1u);
    }
}

// K1f: the f32 gradient planes of the pairs K1 flagged as non-integral;
// the other pairs' workgroups return at once.  Grid (kK1fBlocks, batch),
// 256 threads, grid-stride over the pair's pixels.
constexpr int kK1fBlocks = 256;
template <typename T>
__global__ __launch_bounds__(256) void hs_gradients_f32_kernel(
    const T *__restrict__ I0, const T *__restrict__ I1, int rows, int cols,
    float *__restrict__ gx, float *__restrict__ gy, float *__restrict__ gt,
    const uint32_t *__restrict__ flags) {
    using F = typename GradMath<T>::type;
    if (flags[blockIdx.y] == 0u) return;  // whole workgroup: uniform
    const size_t plane = (size_t)rows * cols;
    const T *a = I0 + blockIdx.y * plane, *b = I1 + blockIdx.y * plane;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < plane;
         i += (size_t)gridDim.x * 256) {
        const int r = (int)(i / (size_t)cols), c = (int)(i - (size_t)r * cols);
        F dx, dy, dt, z_0, nxt;
        sobel_at(a, b, rows, cols, r, c, dx, dy, dt, z_0, nxt);
        const size_t o = blockIdx.y * plane + i;
        gx[o] = (float)dx;
        gy[o] = (float)dy;
        gt[o] = (float)dt;
    }
}

// ----------------------------------------------------------------------- K2

// Horizontal window sum over lanes [l - A, l + W-1-A] (A = anchor).  The
// summation order is fixed per W, so every blocking depth gives the same bits.
template <int W> __device__ __forceinline__ float hsum(float x);

// Two independent fields (u and v) in lockstep, statement by statement, so
// each DPP read of a just-written VGPR has the other field's instruction as
// its wait state instead of an s_nop.
template <int W>
__device__ __forceinline__ void hsum2(float x, float y, float &hx, float &hy) {
    if constexpr (W == 5) {
        const float ax = from_left(x) + x;
        const float ay = from_left(y) + y;
        const float bx = from_left(ax) + from_right(ax);
        const float by = from_left(ay) + from_right(ay);
        const float cx = from_right(x);
        const float cy = from_right(y);
        hx = bx + from_right(cx);
        hy = by + from_right(cy);
    } else if constexpr (W == 3) {
        const float ax = from_left(x) + x;
        const float ay = from_left(y) + y;
        hx = ax + from_right(x);
        hy = ay + from_right(y);
    } else {
        hx = hsum<W>(x);
        hy = hsum<W>(y);
    }
}

template <int W> __device__ __forceinline__ float hsum(float x) {
    constexpr int A = W - W / 2 - 1, AR = W - 1 - A;
    if constexpr (W == 1) {
        return x;
    } else if constexpr (W == 3) {
        return (from_left(x) + x) + from_right(x);
    } else if constexpr (W == 5) {
        // a(l) = x(l-1) + x(l);  hs = (a(l-1) + a(l+1)) + x(l+2)
        const float a = from_left(x) + x;
        return (from_left(a) + from_right(a)) + from_right(from_right(x));
    } else {
        float s = x, m = x, r = x;
#pragma unroll
        for (int d = 0; d < A; ++d) {
            m = from_left(m);
            s += m;
        }
#pragma unroll
        for (int d = 0; d < AR; ++d) {
            r = from_right(r);
            s += r;
        }
        return s;
    }
}


// One wavefront's work on one region: rows [r0, r0 + RH) x the 64 columns
// starting at gc - lane; KB iterations; writes region rows [HL, HL + nout)
// (nout <= RH - HL - HR) of the lanes [HL, 64 - HR).
template <int W, int KB, int RH, bool PACKED>
__device__ __forceinline__ void jacobi_region(const JacobiArgs &p, size_t pbase,
                                              int plane_bytes, int lane, int gc, int r0,
                                              int nout, int nout_cols = 64) {
    constexpr int A = W - W / 2 - 1;  // anchor (hornSchunck.cpp:54)
    constexpr int AR = W - 1 - A;     // taps right/below of the anchor
    constexpr int HL = KB * A, HR = KB * AR;
    constexpr int OX = 64 - HL - HR;
    static_assert(OX > 0 && RH - HL - HR > 0, "halo too deep for the region");
    static_assert(RH <= 64, "row mask is 64 bits");
    const int cols = p.cols;
    const bool col_in = (unsigned)gc < (unsigned)cols;
    // bit r set <=> region row r lies inside the image (wave-uniform)
    uint64_t rowmask = 0;
#pragma unroll
    for (int r = 0; r < RH; ++r)
        rowmask |= (uint64_t)((unsigned)(r0 + r) < (unsigned)p.rows) << r;

    // Buffer descriptors over this pair's planes: a byte offset >= the
    // plane size reads 0 / drops the store, so the halo outside the image
    // (u = v = 0, BORDER_CONSTANT) needs no branches.
    constexpr int kOOB = 0x7FFFFFF0;
    const auto u_rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(p.u_in ? p.u_in + pbase : p.u_out + pbase), 0, p.u_in ? plane_bytes : 0,
        0x00020000);
    const auto v_rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(p.v_in ? p.v_in + pbase : p.v_out + pbase), 0, p.v_in ? plane_bytes : 0,
        0x00020000);

    float u[RH], v[RH];
    uint32_t g[PACKED ? RH : 1];
    float gxr[PACKED ? 1 : RH], gyr[PACKED ? 1 : RH], gtr[PACKED ? 1 : RH];
    {
        const auto g_rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(p.gpack + pbase), 0, PACKED ? plane_bytes : 0, 0x00020000);
        const auto gx_rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(p.gx + pbase), 0, PACKED ? 0 : plane_bytes, 0x00020000);
        const auto gy_rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(p.gy + pbase), 0, PACKED ? 0 : plane_bytes, 0x00020000);
        const auto gt_rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(p.gt + pbase), 0, PACKED ? 0 : plane_bytes, 0x00020000);
        const int off0 = (r0 * cols + gc) * 4;
#pragma unroll
        for (int r = 0; r < RH; ++r) {
            const bool in = col_in && ((rowmask >> r) & 1ull);
            const int off = in ? off0 + r * cols * 4 : kOOB;
            u[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(u_rs, off, 0, 0));
            v[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(v_rs, off, 0, 0));
            if constexpr (PACKED) {
                g[r] = __builtin_amdgcn_raw_buffer_load_b32(g_rs, off, 0, 0);
            } else {
                gxr[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gx_rs, off, 0, 0));
                gyr[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gy_rs, off, 0, 0));
                gtr[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gt_rs, off, 0, 0));
            }
        }
    }

    const float alpha2 = p.alpha2, inv = p.inv_w2;
    for (int it = 0; it < p.iters; ++it) {
        // rings of horizontal sums (hu, hv) and, for W = 5, of vertical pair
        // sums q(y) = h(y) + h(y+1); all indices are compile-time
        float hu[W], hv[W], qu[W], qv[W];
#pragma unroll
        for (int r = 0; r < RH; ++r) {
            hsum2<W>(u[r], v[r], hu[r % W], hv[r % W]);
            if constexpr (W == 5) {
                if (r >= 1) {
                    qu[(r - 1) % W] = hu[(r - 1) % W] + hu[r % W];
                    qv[(r - 1) % W] = hv[(r - 1) % W] + hv[r % W];
                }
            }
            const int y = r - AR;  // output row whose window ends at row r
            if (y >= A) {
                float su, sv;
                if constexpr (W == 5) {
                    // (h(y-2) + h(y-1)) + (h(y) + h(y+1)) + h(y+2)
                    su = (qu[(y - 2) % W] + qu[y % W]) + hu[(y + 2) % W];
                    sv = (qv[(y - 2) % W] + qv[y % W]) + hv[(y + 2) % W];
                } else {
                    su = hu[(y - A) % W];
                    sv = hv[(y - A) % W];
#pragma unroll
                    for (int d = 1; d < W; ++d) {
                        su += hu[(y - A + d) % W];
                        sv += hv[(y - A + d) % W];
                    }
                }
                const float ub = su * inv, vb = sv * inv;
                float ix, iy, itv;
                if constexpr (PACKED) {
                    // unpack every iteration: hoisting the loop-invariant
                    // Ix, Iy, It, 1/D out of the loop costs 4 VGPRs per row
                    unpack_grad(launder_u(g[y]), ix, iy, itv);
                } else {
                    ix = launder_f(gxr[y]);
                    iy = launder_f(gyr[y]);
                    itv = launder_f(gtr[y]);
                }
                // hornSchunck.cpp:63-73
                const float den = alpha2 + ix * ix + iy * iy;
                const float num = ix * ub + iy * vb + itv;
                const float cc = num * __builtin_amdgcn_rcpf(den);
                const bool in = col_in && ((rowmask >> y) & 1ull);
                u[y] = in ? ub - ix * cc : 0.f;
                v[y] = in ? vb - iy * cc : 0.f;
            }
            // Keep rows in program order: otherwise the scheduler hoists every
            // row's horizontal sums (they only read the previous iteration)
            // and the live set explodes past 256 VGPRs.
            __builtin_amdgcn_sched_barrier(0);
        }
    }

    {
        const auto uo_rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p.u_out + pbase), 0,
                                                             plane_bytes, 0x00020000);
        const auto vo_rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p.v_out + pbase), 0,
                                                             plane_bytes, 0x00020000);
        const bool st_lane = lane >= HL && lane < HL + OX && (lane - HL) < nout_cols && col_in;
        const int off0 = launder(((r0 + HL) * cols + gc) * 4);
#pragma unroll
        for (int r = HL; r < RH - HR; ++r) {
            const bool in = st_lane && (r - HL) < nout && ((rowmask >> r) & 1ull);
            const int off = in ? off0 + (r - HL) * cols * 4 : kOOB;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(u[r]), uo_rs, off, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[r]), vo_rs, off, 0, 0);
        }
    }
}

// Region heights (rows held in VGPRs per wavefront).
constexpr int kRowsPacked = 48;
constexpr int kRowsF32 = 24;
constexpr bool kb_ok_packed(int W, int KB) { return KB * (W - 1) <= 32; }
constexpr bool kb_ok_f32(int W, int KB) { return KB * (W - 1) <= 16; }

// f32-gradient path (pairs whose inputs are not 8-bit integers): 5 VGPRs per
// region row, so it walks the packed tile in 24-row regions and the kernel's
// register budget (the max over both branches) stays that of the packed path.
template <int W, int KB>
__device__ __forceinline__ void jacobi_tile_f32(const JacobiArgs p, size_t pbase,
                                                         int plane_bytes, int lane, int gc,
                                                         int out_r0, int nout) {
    if constexpr (kb_ok_f32(W, KB)) {
        constexpr int HL = KB * (W - W / 2 - 1);
        constexpr int OYF = kRowsF32 - KB * (W - 1);
        for (int o = 0; o < nout; o += OYF)
            jacobi_region<W, KB, kRowsF32, false>(p, pbase, plane_bytes, lane, gc,
                                                  out_r0 + o - HL, min(OYF, nout - o));
    }
}

template <int W, int KB>
__global__ __launch_bounds__(256) void hs_jacobi_kernel(const JacobiArgs p) {
    constexpr int HL = KB * (W - W / 2 - 1);
    constexpr int OX = 64 - KB * (W - 1), OY = kRowsPacked - KB * (W - 1);
    // XCD-aware block order.  Workgroups are dealt round-robin over the 8
    // XCDs (linear id % 8 share an L2); remap so each XCD walks a contiguous
    // run of tile rows and the halo rows/columns neighbouring regions re-read
    // hit its L2.  Any bijection is correct; this one only changes speed.
    const int nblk = gridDim.x * gridDim.y;
    const int lin = blockIdx.y * gridDim.x + blockIdx.x;
    const int q = nblk >> 3, rem = nblk & 7, xcd = lin & 7;
    const int logical = xcd * q + min(xcd, rem) + (lin >> 3);
    const int pair = logical / gridDim.x;
    const int lane = threadIdx.x & 63;
    // wave-uniform tile index (readfirstlane: keep tile maths in SGPRs)
    const int tile = (logical - pair * gridDim.x) * 4 +
                     __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (tile >= p.tiles_x * p.tiles_y) return;
    const int ty = tile / p.tiles_x, tx = tile - ty * p.tiles_x;
    const size_t pbase = (size_t)pair * (size_t)p.rows * (size_t)p.cols;
    const int plane_bytes = p.rows * p.cols * 4;
    const int gc = tx * OX - HL + lane;  // this lane's image column
    const uint32_t flag = p.flags != nullptr ? p.flags[pair] : 0u;
    if (flag != 0u) {
        jacobi_tile_f32<W, KB>(p, pbase, plane_bytes, lane, gc, ty * OY, OY);
        return;
    }
    jacobi_region<W, KB, kRowsPacked, true>(p, pbase, plane_bytes, lane, gc, ty * OY - HL,
                                            OY);
}

// ------------------------------------------------------------------- K2 v2
// Workgroup-stacked, two-columns-per-lane variant (windows 3 and 5, the
// reference's 5 and the north-star's 3).
//
//  * A workgroup of NW waves covers a 128-column x NW*RW-row region; wave w
//    owns slab rows [w*RW, (w+1)*RW), lane l owns columns 2l (e) and 2l+1 (o).
//    Two columns per lane halve the horizontal halo share (KB(W-1) of 128
//    instead of 64) and the cross-lane work per pixel.
//  * The vertical window reaches A rows into the slab above and AR rows into
//    the slab below.  Instead of recomputing those rows (temporal halo per
//    wave), the stacked waves exchange their boundary rows through LDS once
//    per iteration (double-buffered by iteration parity: one barrier per
//    iteration).  Only the workgroup's outer rows carry a temporal halo.
//  * Same per-pixel arithmetic as K2 except the horizontal sum association,
//    which depends only on the column's parity within the region (region
//    origins are even for every KB), so every KB gives identical bits.


// workgroup-kernel geometry per window: slab rows per wave (deeper register
// rings for wider windows) and double-buffered slab exchange while two
// workgroups' W-1 boundary rows fit in LDS
constexpr int wg_rows(int W) { return W <= 5 ? 10 : (W <= 7 ? 8 : 7); }
constexpr bool wg_double_buffer(int W) { return W <= 5; }
// T plane in LDS (w = 5, 12-row slabs): frees 2 VGPRs per row for taller
// slabs; the exchange is single-buffered so two workgroups still fit a CU
// (32 KB exchange + 48 KB T plane each)
// Any slab taller than the all-register height wg_rows(W) keeps T in LDS.
// (w = 3 keeps the double-buffered exchange: 2 boundary rows, 32 KB + 44 KB.)
constexpr bool wg_tlds(int W, int RW) { return RW > wg_rows(W); }
constexpr int wg_nbuf(int W, int RW) {
    return (wg_double_buffer(W) && !(W >= 4 && wg_tlds(W, RW))) ? 2 : 1;
}
// slab height of the T-in-LDS variant (two workgroups per CU must fit the
// 160 KB LDS: exchange + 8 RW rows x 512 B of T); 0 = none
constexpr int wg_rows_tl(int W) {
    return (W == 3 || W == 4 || W == 5) ? 11 : (W == 6 ? 10 : 0);
}

template <int W, int KB, int RW, int NW, int SB, bool EDGE, bool X2, bool G32, bool ROWE,
          int PAR>
__device__ __forceinline__ void wg_body_p(const JacobiArgs &p,
                                          float2 (&xch)[wg_nbuf(W, RW)][NW][W - 1][2][64],
                                          float2 *tpl, int tx, int ty, int wv, int lane,
                                          size_t pbase, int plane_bytes);

// A wave whose slab lies wholly outside the image: its rows are u = v = 0
// in every iteration (BORDER_CONSTANT), so it publishes zero boundary sums
// once (both exchange buffers) and then only takes the workgroup's barriers
// -- the same sequence as wg_body_p's iterations (one per iteration, and a
// second after each but the last when the exchange is single-buffered).
// It stores nothing: no row of it is in the image.
template <int W, int RW, int NW>
__device__ __forceinline__ void wg_zero_wave(const JacobiArgs &p,
                                             float2 (&xch)[wg_nbuf(W, RW)][NW][W - 1][2][64],
                                             int wv, int lane) {
#pragma unroll
    for (int b = 0; b < wg_nbuf(W, RW); ++b)
#pragma unroll
        for (int k = 0; k < W - 1; ++k) {
            xch[b][wv][k][0][lane] = make_float2(0.f, 0.f);
            xch[b][wv][k][1][lane] = make_float2(0.f, 0.f);
        }
    const int n_it = p.iters;
    for (int it = 0; it < n_it; ++it) {
        __syncthreads();
        if (wg_nbuf(W, RW) == 1 && it + 1 < n_it) __syncthreads();
    }
}

// One wave's slab, specialised on the parity of its first image row (the
// order of the vertical sums follows image-row parity, see wg_body_p): a
// whole body per parity, so no register state lives across the two.
template <int W, int KB, int RW, int NW, int SB, bool EDGE, bool X2, bool G32,
          bool ROWE = true>
__device__ __forceinline__ void wg_body(const JacobiArgs &p,
                                        float2 (&xch)[wg_nbuf(W, RW)][NW][W - 1][2][64], float2 *tpl,
                                        int tx, int ty, int wv, int lane, size_t pbase,
                                        int plane_bytes) {
    constexpr int A = W - W / 2 - 1, AR = W - 1 - A;
    constexpr int OY = NW * RW - KB * A - KB * AR;
    const int r0 = ty * OY - KB * A + wv * RW;
    if ((W == 3 || W == 5) && (r0 & 1))
        wg_body_p<W, KB, RW, NW, SB, EDGE, X2, G32, ROWE, 1>(p, xch, tpl, tx, ty, wv, lane, pbase,
                                                            plane_bytes);
    else
        wg_body_p<W, KB, RW, NW, SB, EDGE, X2, G32, ROWE, 0>(p, xch, tpl, tx, ty, wv, lane, pbase,
                                                            plane_bytes);
}

template <int W, int KB, int RW, int NW, int SB>
__device__ __forceinline__ void wg_tile(const JacobiArgs &p,
                                        float2 (&xch)[wg_nbuf(W, RW)][NW][W - 1][2][64],
                                        float2 *tpl, int logical);

// 4 waves per SIMD (<= 128 VGPRs): two 8-wave workgroups per CU
constexpr int kK2Waves = 4;
template <int W, int KB, int RW, int NW, int SB>
__global__ __launch_bounds__(NW * 64, kK2Waves) void hs_jacobi_wg_kernel(const JacobiArgs p) {
    constexpr int A = W - W / 2 - 1, AR = W - 1 - A;
    constexpr int HL = KB * A, HR = KB * AR;  // temporal halo, rows
    // column halo rounded up to even: region origins stay even for every KB,
    // so a column's parity (which fixes its summation order) never changes
    constexpr int HLc = HL + (HL & 1), HRc = HR + (HR & 1);
    constexpr int RX = 128, RY = NW * RW;
    constexpr int OX = RX - HLc - HRc, OY = RY - HL - HR;
    constexpr int NB = A + AR;  // boundary rows a wave publishes per iteration
    static_assert(OX > 0 && OY > 0 && (OX % 2) == 0, "geometry");
    static_assert(RW <= 64, "row mask is 64 bits");
    // [parity][wave][boundary row][field u/v][lane] of (even, odd) columns
    __shared__ float2 xch[wg_nbuf(W, RW)][NW][NB][2][64];
    __shared__ float2 tpl[wg_tlds(W, RW) ? NW * RW * 64 : 1];

    // XCD-aware workgroup order (see hs_jacobi_kernel)
    const int nblk = gridDim.x * gridDim.y;
    const int lin = blockIdx.y * gridDim.x + blockIdx.x;
    const int qn = nblk >> 3, rem = nblk & 7, xcd = lin & 7;
    wg_tile<W, KB, RW, NW, SB>(p, xch, tpl, xcd * qn + min(xcd, rem) + (lin >> 3));
}

// One tile (logical index: pair-major, then the tile order) of the
// workgroup kernel: pick the body variant and run it.
template <int W, int KB, int RW, int NW, int SB>
__device__ __forceinline__ void wg_tile(const JacobiArgs &p,
                                        float2 (&xch)[wg_nbuf(W, RW)][NW][W - 1][2][64],
                                        float2 *tpl, int logical) {
    constexpr int A = W - W / 2 - 1, AR = W - 1 - A;
    constexpr int HL = KB * A, HR = KB * AR;
    constexpr int HLc = HL + (HL & 1), HRc = HR + (HR & 1);
    constexpr int RX = 128, RY = NW * RW;
    constexpr int OX = RX - HLc - HRc, OY = RY - HL - HR;
    const int ntile = p.tiles_x * p.tiles_y;
    const int pair = logical / ntile;
    const int tile = logical - pair * ntile;
    if (pair >= p.batch) return;  // whole workgroup: uniform
    // tiles of a pair in row-major order
    const int ty = tile / p.tiles_x;
    const int tx = tile - ty * p.tiles_x;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int cols = p.cols;
    const size_t pbase = (size_t)pair * (size_t)p.rows * (size_t)cols;
    const int plane_bytes = p.rows * cols * 4;

    // interior workgroup: region + halo entirely inside the image, so no
    // border masks (wave-uniform; the masked body handles the rest).
    // For an even image width every lane's column pair (even first column)
    // is 8-byte aligned and lies wholly inside or wholly outside the image,
    // so it moves as one 8-byte word (fully coalesced 512 B per wave
    // instruction instead of two half-line stride-2 dword accesses).  Odd
    // widths take per-column dword accesses.  Pairs K1 flagged as
    // non-integral read the f32 gradient planes instead of the packed words
    // (same tiles, same operator, any blocking depth).
    //
    // The body is chosen per wave (all take the same barriers): a wave whose
    // slab lies wholly outside the image only publishes zeros (its rows are
    // u = v = 0 every iteration); a wave wholly inside needs no row zeroing
    // (the per-row selects cost a whole tile row 18 % at 1080p, where every
    // slab is wholly inside or outside); only a slab that straddles the
    // top or bottom edge runs the row-zeroing body.
    const int r0w = ty * OY - HL + wv * RW;  // image row of this wave's slab row 0
    if (r0w + RW <= 0 || r0w >= p.rows) {
        wg_zero_wave<W, RW, NW>(p, xch, wv, lane);
        return;
    }
    const bool w_in = r0w >= 0 && r0w + RW <= p.rows;
    const bool interior = tx * OX - HLc >= 0 && tx * OX - HLc + RX <= cols && w_in;
    const bool g32 = p.flags != nullptr && p.flags[pair] != 0u;
    if (g32) {
        if ((cols & 1) == 0)
            wg_body<W, KB, RW, NW, SB, true, true, true>(p, xch, tpl, tx, ty, wv, lane, pbase,
                                                         plane_bytes);
        else
            wg_body<W, KB, RW, NW, SB, true, false, true>(p, xch, tpl, tx, ty, wv, lane, pbase,
                                                          plane_bytes);
        return;
    }
    if ((cols & 1) == 0) {
        if (interior)
            wg_body<W, KB, RW, NW, SB, false, true, false>(p, xch, tpl, tx, ty, wv, lane, pbase,
                                                           plane_bytes);
        else if (W <= 7 && w_in)
            // left/right border tiles: every slab row inside the image
            wg_body<W, KB, RW, NW, SB, true, true, false, false>(p, xch, tpl, tx, ty, wv,
                                                                 lane, pbase, plane_bytes);
        else
            wg_body<W, KB, RW, NW, SB, true, true, false>(p, xch, tpl, tx, ty, wv, lane, pbase,
                                                          plane_bytes);
    } else {
        wg_body<W, KB, RW, NW, SB, true, false, false>(p, xch, tpl, tx, ty, wv, lane, pbase,
                                                       plane_bytes);
    }
}

template <int W, int KB, int RW, int NW, int SB, bool EDGE, bool X2, bool G32, bool ROWE,
          int PAR>
__device__ __forceinline__ void wg_body_p(const JacobiArgs &p,
                                          float2 (&xch)[wg_nbuf(W, RW)][NW][W - 1][2][64],
                                          float2 *tpl, int tx, int ty, int wv, int lane,
                                          size_t pbase, int plane_bytes) {
    // distinct markers at both ends keep the compiler from hoisting or
    // sinking the two parity bodies' identical load and store code into the
    // shared path (which costs ~50 spilled VGPRs at 11-row slabs)
    asm volatile("; slab parity %0 begin" ::"n"(PAR));
    constexpr int A = W - W / 2 - 1, AR = W - 1 - A;
    constexpr int HL = KB * A, HR = KB * AR;
    constexpr int HLc = HL + (HL & 1), HRc = HR + (HR & 1);
    constexpr int RX = 128;
    constexpr int OX = RX - HLc - HRc, OY = NW * RW - HL - HR;
    constexpr int NB = A + AR;
    const int cols = p.cols;
    const int gce = tx * OX - HLc + 2 * lane;  // this lane's even image column
    const int r0 = ty * OY - HL + wv * RW;    // image row of slab row 0
    const bool ce = (unsigned)gce < (unsigned)cols;
    const bool co = (unsigned)(gce + 1) < (unsigned)cols;
    // window-mean factor of this lane's columns: 1/w^2 inside the image, 0 outside
    const f2v colm = {ce ? p.inv_w2 : 0.f, co ? p.inv_w2 : 0.f};
    const int ce_i = ce ? 1 : 0, co_i = co ? 1 : 0;
    // Border tiles zero the columns outside the image either by per-lane
    // selects after the update (SEL: w >= 8, whose factor form spills) or by
    // the window-mean factor 0 there.  The factor form needs the operator of
    // those columns to be 0, not NaN: alpha^2 per column, 1 outside the
    // image (hsflow_device.h alpha2_cols; w = 6 then spills 8 bytes, still
    // fewer than with the selects).  Interior tiles have no column outside.
    constexpr bool SEL = EDGE && W >= 8;
    const f2v a2c = (EDGE && !SEL) ? alpha2_cols(p.alpha2, ce, co) : f2v{p.alpha2, p.alpha2};
    uint64_t rowmask = 0;
#pragma unroll
    for (int r = 0; r < RW; ++r)
        rowmask |= (uint64_t)((unsigned)(r0 + r) < (unsigned)p.rows) << r;

    constexpr int kOOB = 0x7FFFFFF0;
    const int nbytes = plane_bytes;
    const auto u_rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(p.u_in ? p.u_in + pbase : p.u_out + pbase), 0, p.u_in ? nbytes : 0,
        0x00020000);
    const auto v_rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(p.v_in ? p.v_in + pbase : p.v_out + pbase), 0, p.v_in ? nbytes : 0,
        0x00020000);
    const auto gp_rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p.gpack + pbase), 0,
                                                         G32 ? 0 : nbytes, 0x00020000);
    const auto gx_rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p.gx + pbase), 0,
                                                         G32 ? nbytes : 0, 0x00020000);
    const auto gy_rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p.gy + pbase), 0,
                                                         G32 ? nbytes : 0, 0x00020000);
    const auto gt_rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p.gt + pbase), 0,
                                                         G32 ? nbytes : 0, 0x00020000);

    // (even, odd) column pairs as 2-wide vectors: the identical per-column
    // arithmetic issues as packed FP32 (v_pk_add/mul/fma_f32), one
    // instruction for both columns (on gfx950 a wave64 VALU op costs ~4 SIMD
    // cycles and v_pk_*_f32 ~4.6 for twice the work: scripts/ubench).
    //
    // The per-pixel Jacobi operator is the same every iteration, so it is
    // set up once per launch in normalised form:
    //   s = 1/sqrt(alpha^2 + Ix^2 + Iy^2);  X = Ix s, Y = Iy s, T = It s
    //   u' = ubar - X (X ubar + Y vbar + T),  v' = vbar - Y (...)
    // which is hornSchunck.cpp:63-73 rearranged (c = (Ix ubar + Iy vbar +
    // It)/D): 6 packed ops per column pair and no unpack / rcp per iteration.
    constexpr bool TL = wg_tlds(W, RW);
    f2v U[RW], V[RW], X[RW], Y[RW], T[TL ? 1 : RW];
    float2 *tw = tpl + (TL ? wv * RW * 64 + lane : 0);  // this lane's T rows
    {
        const int off0 = (r0 * cols + gce) * 4;
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            float ixe, iye, ite, ixo, iyo, ito;
            if constexpr (X2) {
                const int o = (!EDGE || (((rowmask >> r) & 1ull) && ce))
                                  ? off0 + r * cols * 4 : kOOB;
                const u2v a = __builtin_amdgcn_raw_buffer_load_b64(u_rs, o, 0, 0);
                const u2v b = __builtin_amdgcn_raw_buffer_load_b64(v_rs, o, 0, 0);
                U[r] = f2v{__uint_as_float(a.x), __uint_as_float(a.y)};
                V[r] = f2v{__uint_as_float(b.x), __uint_as_float(b.y)};
                if constexpr (G32) {
                    const u2v gx2 = __builtin_amdgcn_raw_buffer_load_b64(gx_rs, o, 0, 0);
                    const u2v gy2 = __builtin_amdgcn_raw_buffer_load_b64(gy_rs, o, 0, 0);
                    const u2v gt2 = __builtin_amdgcn_raw_buffer_load_b64(gt_rs, o, 0, 0);
                    ixe = __uint_as_float(gx2.x); ixo = __uint_as_float(gx2.y);
                    iye = __uint_as_float(gy2.x); iyo = __uint_as_float(gy2.y);
                    ite = __uint_as_float(gt2.x); ito = __uint_as_float(gt2.y);
                } else {
                    const u2v g = __builtin_amdgcn_raw_buffer_load_b64(gp_rs, o, 0, 0);
                    unpack_grad(g.x, ixe, iye, ite);
                    unpack_grad(g.y, ixo, iyo, ito);
                }
            } else {
                const bool rin = (rowmask >> r) & 1ull;
                const int oe = (rin && ce) ? off0 + r * cols * 4 : kOOB;
                const int oo = (rin && co) ? off0 + r * cols * 4 + 4 : kOOB;
                U[r].x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(u_rs, oe, 0, 0));
                U[r].y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(u_rs, oo, 0, 0));
                V[r].x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(v_rs, oe, 0, 0));
                V[r].y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(v_rs, oo, 0, 0));
                if constexpr (G32) {
                    ixe = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gx_rs, oe, 0, 0));
                    ixo = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gx_rs, oo, 0, 0));
                    iye = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gy_rs, oe, 0, 0));
                    iyo = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gy_rs, oo, 0, 0));
                    ite = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gt_rs, oe, 0, 0));
                    ito = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gt_rs, oo, 0, 0));
                } else {
                    unpack_grad(__builtin_amdgcn_raw_buffer_load_b32(gp_rs, oe, 0, 0), ixe,
                                iye, ite);
                    unpack_grad(__builtin_amdgcn_raw_buffer_load_b32(gp_rs, oo, 0, 0), ixo,
                                iyo, ito);
                }
            }
            if constexpr (TL) {
                f2v Tr;
                op_setup(a2c, ixe, iye, ite, ixo, iyo, ito, X[r], Y[r], Tr);
                tw[r * 64] = make_float2(Tr.x, Tr.y);
            } else {
                op_setup(a2c, ixe, iye, ite, ixo, iyo, ito, X[r], Y[r], T[r]);
            }
        }
    }

    const float inv = p.inv_w2;
    const f2v invv = {inv, inv};
    auto t_row = [&](int y) -> f2v {
        if constexpr (TL) {
            const float2 t = tw[y * 64];
            return f2v{t.x, t.y};
        } else {
            return T[y];
        }
    };
    // horizontal sums of slab row t (own data)
    auto hrow = [&](int t, f2v &hu, f2v &hv) {
        float a, b, c, d;
        hsum_c2<W>(U[t].x, U[t].y, V[t].x, V[t].y, a, b, c, d);
        hu = f2v{a, b};
        hv = f2v{c, d};
    };

    const int n_it = p.iters;
    // The vertical sums follow the parity of the image row (PAR = parity
    // of slab row 0), so every slab height, blocking depth and kernel
    // adds in the same order.  w = 5: pair sums Q(t) = h(t) + h(t+1) at
    // odd rows t, cores M(y) = Q(y-1) + Q(y+1) at even rows y, shared by
    // two outputs: S(y) = h(y-2) + M(y), S(y+1) = M(y) + h(y+3).
    // w = 3: Q at even rows, S(y) = h(y-1) + Q(y), S(y+1) = Q(y) + h(y+2).
    // 2 (w = 5) and 1.5 (w = 3) adds per row and field instead of 3 and 2.
    constexpr bool SHARED = W == 3 || W == 5;
    // output descriptors and this lane's store offset: the last iteration
    // stores each row as soon as it is final (the stores drain under the
    // rest of the sweep instead of holding the workgroup slot after it)
    const auto uo_rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p.u_out + pbase), 0,
                                                         nbytes, 0x00020000);
    const auto vo_rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p.v_out + pbase), 0,
                                                         nbytes, 0x00020000);
    const bool st_lane = lane >= HLc / 2 && lane < (HLc + OX) / 2;
    // u', v' are streamed out with the nt policy in launches that fill the
    // chip (+0.7 % at 1080p x 8, +-0 at 4K x 2 against default-policy stores;
    // sc0 +0.2 %; sc1 -4 % / -2 %) and write-through (sc1) in the others
    // (p.write_through: a single 1080p pair +9 %, 720p x 2 +4 %, KITTI +3 %;
    // profiles/r03_store_policy_ab.txt) -- their lines leave the L2 at once
    // instead of at the kernel boundary.  A wave-uniform branch per row.
    auto store_row = [&](int r, int vo_e, int vo_o) {
        const int wr = wv * RW + r;  // workgroup region row (wave-uniform)
        if (!(wr >= HL && wr < HL + OY && ((rowmask >> r) & 1ull))) return;
        const int so = (r0 + r) * cols * 4;
        auto st = [&](auto aux_c) {
            constexpr int AUX = decltype(aux_c)::value;
            if constexpr (X2) {
                __builtin_amdgcn_raw_buffer_store_b64(
                    u2v{__float_as_uint(U[r].x), __float_as_uint(U[r].y)}, uo_rs, vo_e, so, AUX);
                __builtin_amdgcn_raw_buffer_store_b64(
                    u2v{__float_as_uint(V[r].x), __float_as_uint(V[r].y)}, vo_rs, vo_e, so, AUX);
            } else {
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(U[r].x), uo_rs, vo_e, so, AUX);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(U[r].y), uo_rs, vo_o, so, AUX);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(V[r].x), vo_rs, vo_e, so, AUX);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(V[r].y), vo_rs, vo_o, so, AUX);
            }
        };
        if (p.write_through)
            st(std::integral_constant<int, 16>{});
        else
            st(std::integral_constant<int, 2>{});
    };
    auto iteration = [&](int it, auto last_c) {
        constexpr bool LAST = decltype(last_c)::value;
        int vo_e = 0, vo_o = 0;
        if constexpr (LAST) {
            const int c4 = launder(gce * 4);
            vo_e = (st_lane && ce) ? c4 : kOOB;
            vo_o = (st_lane && co) ? c4 + 4 : kOOB;
        }
        const int par = wg_nbuf(W, RW) == 2 ? (it & 1) : 0;
        // 1. horizontal sums of the boundary rows first, published for the
        //    neighbouring slabs: rows 0..AR-1 feed the wave above, rows
        //    RW-A..RW-1 the wave below.  Exchanging sums (not raw rows)
        //    means no wave recomputes another slab's rows.
        f2v htu[AR > 0 ? AR : 1], htv[AR > 0 ? AR : 1], hbu[A > 0 ? A : 1], hbv[A > 0 ? A : 1];
#pragma unroll
        for (int k = 0; k < AR; ++k) {
            hrow(k, htu[k], htv[k]);
            xch[par][wv][k][0][lane] = make_float2(htu[k].x, htu[k].y);
            xch[par][wv][k][1][lane] = make_float2(htv[k].x, htv[k].y);
        }
#pragma unroll
        for (int k = 0; k < A; ++k) {
            hrow(RW - A + k, hbu[k], hbv[k]);
            xch[par][wv][AR + k][0][lane] = make_float2(hbu[k].x, hbu[k].y);
            xch[par][wv][AR + k][1][lane] = make_float2(hbv[k].x, hbv[k].y);
        }
        __syncthreads();

        // 2. sweep slab rows t = -A .. RW+AR-1 through a ring of horizontal
        //    sums (hu, hv) and vertical pair sums q(t) = h(t) + h(t+1)
        // Rows beyond the workgroup region (above wave 0, below wave NW-1)
        // may hold anything finite or not: their influence moves A (AR)
        // rows per iteration, so after KB iterations it has reached only
        // the HL (HR) halo rows, which are never stored; at the image border
        // those rows are re-zeroed every iteration (EDGE).  So the reads are
        // unconditional, from a clamped slab (no branches, no zero fill).
        const int wa = wv > 0 ? wv - 1 : 0, wb = wv < NW - 1 ? wv + 1 : NW - 1;
        f2v hu[W], hv[W], qu[W], qv[W], mu, mv;
        // T plane in LDS: interior tiles read it one output row ahead, so
        // the LDS latency of row y+1's operator hides under row y's update
        // (w = 5: +0.7 % at 1080p x 8 and 4K x 2, same box, bit-identical;
        // the tall w = 6 and w = 3 slabs have no VGPR left for it: they
        // spill 8 and 84 B per lane with it)
        constexpr bool TPF = TL && !EDGE && W == 5;
        f2v tnext = f2v{0.f, 0.f};
        if constexpr (TPF) tnext = t_row(0);
#pragma unroll
        for (int rr = 0; rr < RW + NB; ++rr) {
            const int t = rr - A;
            const int sl = (t + 2 * W) % W;
            if (t < 0) {  // the slab above's bottom rows
                const float2 a = xch[par][wa][AR + (t + A)][0][lane];
                const float2 b = xch[par][wa][AR + (t + A)][1][lane];
                hu[sl] = f2v{a.x, a.y};
                hv[sl] = f2v{b.x, b.y};
            } else if (t >= RW) {  // the slab below's top rows
                const float2 a = xch[par][wb][t - RW][0][lane];
                const float2 b = xch[par][wb][t - RW][1][lane];
                hu[sl] = f2v{a.x, a.y};
                hv[sl] = f2v{b.x, b.y};
            } else if (t < AR) {
                hu[sl] = htu[t];
                hv[sl] = htv[t];
            } else if (t >= RW - A) {
                hu[sl] = hbu[t - (RW - A)];
                hv[sl] = hbv[t - (RW - A)];
            } else {
                hrow(t, hu[sl], hv[sl]);
            }
            // window-mean factors of this lane's columns (0 outside the
            // image in border tiles)
            const f2v cf = (EDGE && !SEL) ? launder_v2(colm) : invv;
            // pair sum Q(t-1) (w = 5: t-1 odd; w = 3: t-1 even, kept as
            // c Q, the core two rows' means share; else every row)
            if (rr >= 1 && (!SHARED || ((PAR + t - 1 + 2 * W) & 1) == (W == 5 ? 1 : 0))) {
                const int sp = (t - 1 + 2 * W) % W;
                if constexpr (W == 3) {
                    qu[sp] = (hu[sp] + hu[sl]) * cf;
                    qv[sp] = (hv[sp] + hv[sl]) * cf;
                } else {
                    qu[sp] = hu[sp] + hu[sl];
                    qv[sp] = hv[sp] + hv[sl];
                }
            }
            const int y = t - AR;  // slab row whose window ends at t
            if (y >= 0) {
                // w = 3, 5: the window means (ub, vb) straight from the
                // scaled core, one fma per row (op_update_mean); other
                // windows: pair tree over rows y-A .. y+AR,
                // ((q(y-A) + q(y-A+2)) + ...) [+ h(y+AR) for odd W]
                f2v su, sv;
                const bool yev = ((PAR + y + 2 * W) & 1) == 0;  // image row y even
                if constexpr (W == 5) {
                    const int s0 = (y - 2 + 2 * W) % W, s1 = (y - 1 + 2 * W) % W,
                              s2 = (y + 1 + 2 * W) % W, s3 = (y + 2 + 2 * W) % W;
                    if (yev) {  // mean(y): h(y-2) and c M(y), M(y) = Q(y-1) + Q(y+1)
                        mu = (qu[s1] + qu[s2]) * cf;
                        mv = (qv[s1] + qv[s2]) * cf;
                        su = fma2(hu[s0], cf, mu);
                        sv = fma2(hv[s0], cf, mv);
                    } else {  // mean(y): c M(y-1), M(y-1) = Q(y-2) + Q(y), and h(y+2)
                        if (y == 0) {  // core M(-1) not formed by row -1
                            mu = (qu[s0] + qu[(y + 2 * W) % W]) * cf;
                            mv = (qv[s0] + qv[(y + 2 * W) % W]) * cf;
                        }
                        su = fma2(hu[s3], cf, mu);
                        sv = fma2(hv[s3], cf, mv);
                    }
                } else if constexpr (W == 3) {
                    const int s0 = (y - 1 + 2 * W) % W, s1 = (y + 2 * W) % W,
                              s2 = (y + 1 + 2 * W) % W;
                    if (yev) {  // mean(y): h(y-1) and c Q(y)
                        su = fma2(hu[s0], cf, qu[s1]);
                        sv = fma2(hv[s0], cf, qv[s1]);
                    } else {  // mean(y): c Q(y-1) and h(y+1)
                        su = fma2(hu[s2], cf, qu[s0]);
                        sv = fma2(hv[s2], cf, qv[s0]);
                    }
                } else {
                    su = qu[(y - A + 2 * W) % W];
                    sv = qv[(y - A + 2 * W) % W];
#pragma unroll
                    for (int pq = 1; pq < W / 2; ++pq) {
                        const int sq = (y - A + 2 * pq + 2 * W) % W;
                        su = su + qu[sq];
                        sv = sv + qv[sq];
                    }
                    if constexpr (W & 1) {
                        const int sh = (y + AR + 2 * W) % W;
                        su = su + hu[sh];
                        sv = sv + hv[sh];
                    }
                }
                // (su, sv): window sums, or for w = 3, 5 already the means
                auto update = [&](f2v factor, f2v T_y, f2v &nu_, f2v &nv_) {
                    if constexpr (SHARED)
                        op_update_mean(su, sv, X[y], Y[y], T_y, nu_, nv_);
                    else
                        op_update(su, sv, factor, X[y], Y[y], T_y, nu_, nv_);
                };
                f2v nu, nv;
                if constexpr (SEL) {
                    // outside the image u = v = 0 (BORDER_CONSTANT); per-lane
                    // selects (see SEL)
                    update(invv, t_row(y), nu, nv);
                    const bool rin = (rowmask >> y) & 1ull;
                    const bool ie = rin & (launder(ce_i) != 0);
                    const bool io = rin & (launder(co_i) != 0);
                    nu.x = ie ? nu.x : 0.f;
                    nu.y = io ? nu.y : 0.f;
                    nv.x = ie ? nv.x : 0.f;
                    nv.y = io ? nv.y : 0.f;
                } else if constexpr (EDGE) {
                    // Outside the image u = v = 0 (BORDER_CONSTANT).  Columns:
                    // the window mean is taken with factor 0 there and the
                    // gradients read there are 0 (out-of-range loads), so the
                    // update yields 0 (every value in the region is finite)
                    // without per-lane masks.  Rows (wave-uniform): select.
                    update(cf, t_row(y), nu, nv);
                    if (ROWE && !((rowmask >> y) & 1ull)) {
                        nu = f2v{0.f, 0.f};
                        nv = f2v{0.f, 0.f};
                    }
                } else if constexpr (TPF) {
                    const f2v tcur = tnext;
                    if (y + 1 < RW) tnext = t_row(y + 1);
                    // keep the read of row y+1 here: only LDS reads may not
                    // be moved across (VALU, SALU, VMEM and DS writes may)
                    __builtin_amdgcn_sched_barrier(0x67E);
                    update(invv, tcur, nu, nv);
                } else {
                    update(invv, t_row(y), nu, nv);
                }
                U[y] = nu;
                V[y] = nv;
                if constexpr (LAST) store_row(y, vo_e, vo_o);
            }
            if ((rr % SB) == SB - 1) __builtin_amdgcn_sched_barrier(0);
        }
        // single-buffered exchange: the neighbours' reads of this iteration
        // must finish before the next iteration's publish overwrites them
        if constexpr (!LAST && wg_nbuf(W, RW) == 1) __syncthreads();
    };
    int it = 0;
    for (; it + 1 < n_it; ++it) iteration(it, std::false_type{});
    if (it < n_it) iteration(it, std::true_type{});

    asm volatile("; slab parity %0 sweep end" ::"n"(PAR));
    // no iteration ran (iters = 0): the loaded state is the output
    if (n_it == 0) {
        const int c4 = launder(gce * 4);
        const int vo_e = (st_lane && ce) ? c4 : kOOB;
        const int vo_o = (st_lane && co) ? c4 + 4 : kOOB;
#pragma unroll
        for (int r = 0; r < RW; ++r) store_row(r, vo_e, vo_o);
    }
    asm volatile("; slab parity %0 end" ::"n"(PAR));
}

// ---------------------------------------------------------------------- K2g
__global__ __launch_bounds__(256) void hs_jacobi_generic_kernel(const JacobiArgs p,
                                                                int W) {
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const int r = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int pair = blockIdx.z;
    if (r >= p.rows || c >= p.cols) return;
    const int A = W - W / 2 - 1;
    const size_t plane = (size_t)p.rows * p.cols;
    const size_t pbase = (size_t)pair * plane;
    float su = 0.f, sv = 0.f;
    if (p.u_in) {
        for (int i = 0; i < W; ++i) {
            const int yy = r + i - A;
            if ((unsigned)yy >= (unsigned)p.rows) continue;
            float hu = 0.f, hv = 0.f;
            for (int j = 0; j < W; ++j) {
                const int xx = c + j - A;
                if ((unsigned)xx >= (unsigned)p.cols) continue;
                hu += p.u_in[pbase + (size_t)yy * p.cols + xx];
                hv += p.v_in[pbase + (size_t)yy * p.cols + xx];
            }
            su += hu;
            sv += hv;
        }
    }
    const size_t o = pbase + (size_t)r * p.cols + c;
    float ix, iy, itv;
    if (p.flags != nullptr && p.flags[pair] != 0u) {
        ix = p.gx[o];
        iy = p.gy[o];
        itv = p.gt[o];
    } else {
        unpack_grad(p.gpack[o], ix, iy, itv);
    }
    const float ub = su * p.inv_w2, vb = sv * p.inv_w2;
    const float den = p.alpha2 + ix * ix + iy * iy;
    const float num = ix * ub + iy * vb + itv;
    const float cc = num * __builtin_amdgcn_rcpf(den);
    p.u_out[o] = ub - ix * cc;
    p.v_out[o] = vb - iy * cc;
}

// ------------------------------------------------------------------ launchers
template <typename T>
static void launch_gradients_t(const void *I0, const void *I1, int rows, int cols, int batch,
                               uint32_t *gpack, float *gx, float *gy, float *gt,
                               uint32_t *flags, bool planes, hipStream_t s) {
    dim3 blk(64, 4, 1), grd((cols + 127) / 128, (rows + 4 * kK1Rows - 1) / (4 * kK1Rows), batch);
    const T *a = (const T *)I0, *b = (const T *)I1;
    if (planes) {
        hipLaunchKernelGGL((hs_gradients_kernel<T, true>), grd, blk, 0, s, a, b, rows, cols,
                           gpack, gx, gy, gt, flags);
        return;
    }
    hipLaunchKernelGGL((hs_gradients_kernel<T, false>), grd, blk, 0, s, a, b, rows, cols, gpack,
                       gx, gy, gt, flags);
    // 8-bit frames are always integral: no pair is ever flagged
    if constexpr (!std::is_same<T, uint8_t>::value)
        hipLaunchKernelGGL(hs_gradients_f32_kernel<T>, dim3(kK1fBlocks, batch), dim3(256), 0, s,
                           a, b, rows, cols, gx, gy, gt, flags);
}

hipError_t launch_gradients(const void *I0, const void *I1, int dtype_in, int rows,
                            int cols, int batch, uint32_t *gpack, float *gx, float *gy,
                            float *gt, uint32_t *flags, bool planes, hipStream_t s) {
    if (dtype_in == 0)
        launch_gradients_t<uint8_t>(I0, I1, rows, cols, batch, gpack, gx, gy, gt, flags, planes,
                                    s);
    else if (dtype_in == 2)  // HSFLOW_F64 (CV_64FC1 frames)
        launch_gradients_t<double>(I0, I1, rows, cols, batch, gpack, gx, gy, gt, flags, planes,
                                   s);
    else if (dtype_in == 3)  // HSFLOW_F16 (config 5 inputs)
        launch_gradients_t<_Float16>(I0, I1, rows, cols, batch, gpack, gx, gy, gt, flags,
                                     planes, s);
    else
        launch_gradients_t<float>(I0, I1, rows, cols, batch, gpack, gx, gy, gt, flags, planes,
                                  s);
    return hipGetLastError();
}

template <int W, int KB>
static hipError_t launch_jacobi_t(JacobiArgs a, hipStream_t s) {
    constexpr int OX = 64 - KB * (W - 1), OY = kRowsPacked - KB * (W - 1);
    a.tiles_x = (a.cols + OX - 1) / OX;
    a.tiles_y = (a.rows + OY - 1) / OY;
    const long ntiles = (long)a.tiles_x * a.tiles_y;
    dim3 grd((unsigned)((ntiles + 3) / 4), (unsigned)a.batch, 1);
    hipLaunchKernelGGL((hs_jacobi_kernel<W, KB>), grd, dim3(256), 0, s, a);
    return hipGetLastError();
}

// windows 3..9; w = 1, 2 keep the per-wave kernel (a 1-column halo makes
// it fast already: 920 k Mpix*iter/s at w = 2), wider windows the generic one
static bool uses_wg_kernel(int W) { return W >= 3 && W <= 9; }

// Temporal-blocking depth per window (overridable through
// hsflow_set_iters_per_launch).  The workgroup kernel (W = 3, 5) takes
// KB in {1..6, 8} for packed and f32 gradients alike; its halo KB(W-1)
// must leave at least half the 128 x 64 region as output.  The per-wave
// kernel keeps the older limits (f32 regions are 24 rows).
int default_kb(int W) {
    // measured on MI355X (scripts/sweep.py, profiles/README.md): the extra
    // halo work of deeper blocking is cheaper than the HBM pass it saves up
    // to KB(W-1) = 24 for W = 5 and 16 for W = 3 (10/12/16 measured, no gain)
    if (uses_wg_kernel(W)) {
        // about 24 halo rows per launch (measured optimum at w = 5: KB 6)
        switch (W) {
        case 3: return 8;
        case 4: return 8;
        case 5: return 6;
        case 6: return 5;
        case 7: return 4;
        default: return 3;  // 8, 9
        }
    }
    if (W < 1 || W > 9) return 1;
    for (int kb : {8, 4, 2})
        if (kb_ok_f32(W, kb)) return kb;
    return 1;
}

bool kb_supported(int W, int KB, bool need_f32) {
    if (uses_wg_kernel(W))
        return ((KB >= 1 && KB <= 6) || KB == 8) && KB * (W - 1) <= 32;
    if (W < 1 || W > 9) return KB == 1;
    if (KB != 1 && KB != 2 && KB != 4 && KB != 8) return false;
    return need_f32 ? kb_ok_f32(W, KB) : kb_ok_packed(W, KB);
}

// compute units of the current device (cached per device id; relaxed atomics:
// concurrent solves from several host threads may fill an entry together,
// with the same value)
int device_cus() {
    static std::atomic<int> per_dev[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int cus = per_dev[dev].load(std::memory_order_relaxed);
    if (cus == 0) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                hipSuccess || cus <= 0)
            cus = 256;
        per_dev[dev].store(cus, std::memory_order_relaxed);
    }
    return cus;
}

// workgroups of a workgroup-kernel launch with RW-row slabs (NW waves)
static long wg_tiles(const JacobiArgs &a, int W, int KB, int RW, int NW = 8) {
    const int HL = KB * (W - W / 2 - 1), HR = KB * (W / 2);
    const int ox = 128 - (HL + (HL & 1)) - (HR + (HR & 1));
    const int oy = NW * RW - KB * (W - 1);
    return (long)((a.cols + ox - 1) / ox) * ((a.rows + oy - 1) / oy) * a.batch;
}

// Slab rows the busiest SIMD sweeps per iteration: workgroups per CU (the
// launch spread evenly) x waves per SIMD of one workgroup x slab rows.  A
// launch that cannot fill the chip ends when its busiest SIMD does.
static long wg_simd_rows(const JacobiArgs &a, int W, int KB, int RW, int NW) {
    const long cus = device_cus();
    const long per_cu = (wg_tiles(a, W, KB, RW, NW) + cus - 1) / cus;
    return per_cu * (NW / 4) * RW;
}

// Blocking depth for a launch that does not fill the chip.  KB = 6 is the
// measured optimum at w = 5 when a launch has several rounds of workgroups;
// when one round does not even fill the 2 x CUs slots (a single 1080p pair:
// 380 workgroups), a pass costs one workgroup lifetime whatever the tile
// count, so fewer, longer passes win: KB = 8 (its 460 workgroups still fit
// one round) -- 1080p pair 0.957 -> 0.833 ms, 720p 0.586 -> 0.519 ms, the
// KITTI 375 x 1242 pair at 100 it 0.209 -> 0.187 ms; a 4K pair (1258
// workgroups) keeps KB 6 (4.08 vs 4.37 ms).  `batch` counts every pair in
// flight (a batch split over side streams runs its halves concurrently).
int fill_kb(int W, int kb, int rows, int cols, int batch) {
    if (W != 5 || kb != 6 || !uses_wg_kernel(W) || rows <= 0 || cols <= 0 || batch <= 0)
        return kb;
    JacobiArgs a{};
    a.rows = rows;
    a.cols = cols;
    a.batch = batch;
    const long slots = 2L * device_cus();
    if (wg_tiles(a, 5, 6, wg_rows_tl(5)) >= slots) return kb;
    const long t8 = std::max(wg_tiles(a, 5, 8, wg_rows_tl(5)), wg_tiles(a, 5, 8, wg_rows(5)));
    return t8 <= slots ? 8 : kb;
}

bool fill_limited(int W, int KB, bool strip, int rows, int cols, int batch, int strip_rows) {
    if (rows <= 0 || cols <= 0 || batch <= 0) return false;
    JacobiArgs a{};
    a.rows = rows;
    a.cols = cols;
    a.batch = batch;
    if (strip) {  // K4: under 3/4 of the wave slots (a 4K pair: 962 of 2048),
                  // counted with the segment height the launch uses
        int nseg = 0, nstrips = 0;
        strip_seg_rows(W, KB, rows, cols, batch, 1, &nseg, &nstrips,
                       strip_rows > 0 ? strip_rows : 84);
        return (long)nseg * nstrips * batch * 4 < 8L * device_cus() * 3;
    }
    // K2: one round of 8-wave tiles (a single 1080p pair: 460 for 512 slots)
    if (W < 3 || W > 9) return false;
    return wg_tiles(a, W, KB, wg_rows(W)) <= 2L * device_cus();
}

template <int W, int KB, int RW, int NW, int SB>
static hipError_t launch_jacobi_wg(JacobiArgs a, hipStream_t s) {
    constexpr int HL = KB * (W - W / 2 - 1), HR = KB * (W / 2);
    constexpr int OX = 128 - (HL + (HL & 1)) - (HR + (HR & 1));
    constexpr int OY = NW * RW - KB * (W - 1);
    a.tiles_x = (a.cols + OX - 1) / OX;
    a.tiles_y = (a.rows + OY - 1) / OY;
    const long ntiles = (long)a.tiles_x * a.tiles_y;
    dim3 grd((unsigned)ntiles, (unsigned)a.batch, 1);
    hipLaunchKernelGGL((hs_jacobi_wg_kernel<W, KB, RW, NW, SB>), grd, dim3(NW * 64), 0, s,
                       a);
    return hipGetLastError();
}


template <int W, int KB>
static hipError_t launch_jacobi_wgv(JacobiArgs a, hipStream_t s) {
    if constexpr (KB * (W - 1) > 32) {  // kb_supported() rejects these
        (void)a;
        (void)s;
        return hipErrorInvalidValue;
    } else {
    // 8 waves x 10 slab rows (80 x 128 region, 128 VGPRs, no spills).
    // Same-box A/B on MI355X (scripts/ab_bench.sh), W = 5, KB = 6:
    // 8 rows 820k / 941k, 9 rows 850k / 995k, 10 rows 863k / 1026k
    // Mpix*iter/s at 1080p / 4K (the taller slab shrinks the share of
    // temporal-halo rows).  Also slower: 16 waves x 8 rows (one workgroup
    // per CU).  SB = 16 > rows swept: no scheduling barriers inside the
    // sweep, so the scheduler interleaves rows and fills the DPP
    // read-after-write wait states.
    // Taller slabs with the T plane in LDS (wg_rows_tl): w = 5, 11 rows
    // (88 x 128 region), single-buffered exchange: same box, 1080p x 8 /
    // 4K x 2, 1.011 M / 1.072 M -> 1.032 M / 1.089 M Mpix*iter/s (12 rows
    // spill).  Used for w = 5 and w = 6 (8 -> 10 rows: 1080p 782 k -> 859 k,
    // 4K 793 k -> 891 k); at w = 3 and w = 4 they measure equal to the
    // all-register slabs.
    // Fill-limited KB 8 launches (a single 1080p pair: 460 8-wave tiles for
    // 512 slots, so two workgroups, 40 slab rows, on the busiest SIMD):
    // 16-wave workgroups of 8-row slabs (128-row regions, one per CU: 128 KB
    // of exchange buffers) cover 1080p in 240 tiles, 32 rows per SIMD.  Taken
    // when the busiest SIMD sweeps fewer rows that way.  Same box, one pair,
    // 300 it: 1080p w 5 0.825 -> 0.790 ms, w 3 0.717 -> 0.700 ms, bit-identical;
    // 720p x 2 and KITTI keep the 8-wave tiles (scripts/lab/geom_ab.sh,
    // profiles/r03_k2_geometry_ab.txt).
    if constexpr ((W == 3 || W == 5) && KB == 8) {
        if (wg_simd_rows(a, W, KB, 8, 16) < wg_simd_rows(a, W, KB, wg_rows(W), 8))
            return launch_jacobi_wg<W, KB, 8, 16, 16>(a, s);
    }
    constexpr int RT = (W == 5 || W == 6) ? wg_rows_tl(W) : 0;
    if constexpr (RT > 0 && KB * (W - 1) < 8 * RT / 2) {
        bool on = true;
        {
            // Taller slabs mean fewer workgroups: keep them only while the
            // launch still fills one round of 2 workgroups per CU (single
            // 1080p pair at w = 5: 323 vs 380 workgroups for 512 slots,
            // 515 k vs 569 k Mpix*iter/s with the all-register slabs).
            const long slots = 2L * device_cus();
            const long t_tall = wg_tiles(a, W, KB, RT), t_reg = wg_tiles(a, W, KB, wg_rows(W));
            if (t_tall < slots && t_reg > t_tall) on = false;
        }
        if (on) return launch_jacobi_wg<W, KB, RT, 8, 16>(a, s);
    }
    return launch_jacobi_wg<W, KB, wg_rows(W), 8, 16>(a, s);
    }
}

template <int W>
static hipError_t launch_jacobi_w(JacobiArgs a, int KB, hipStream_t s) {
    if constexpr (W >= 3 && W <= 9) {  // K2 workgroup tiles
        switch (KB) {
        case 1: return launch_jacobi_wgv<W, 1>(a, s);
        case 2: return launch_jacobi_wgv<W, 2>(a, s);
        case 3: return launch_jacobi_wgv<W, 3>(a, s);
        case 4: return launch_jacobi_wgv<W, 4>(a, s);
        case 5: return launch_jacobi_wgv<W, 5>(a, s);
        case 6: return launch_jacobi_wgv<W, 6>(a, s);
        case 8: return launch_jacobi_wgv<W, 8>(a, s);
        default: return hipErrorInvalidValue;
        }
    } else {  // windows 1, 2: per-wave regions
        switch (KB) {
        case 1: return launch_jacobi_t<W, 1>(a, s);
        case 2:
            if constexpr (kb_ok_packed(W, 2)) return launch_jacobi_t<W, 2>(a, s);
            break;
        case 4:
            if constexpr (kb_ok_packed(W, 4)) return launch_jacobi_t<W, 4>(a, s);
            break;
        case 8:
            if constexpr (kb_ok_packed(W, 8)) return launch_jacobi_t<W, 8>(a, s);
            break;
        default: break;
        }
        return hipErrorInvalidValue;
    }
}

// One Jacobi pass of a.iters (<= KB) iterations.  Pairs flagged by K1 as
// non-integral take the f32-gradient path inside the same launch; the caller
// must then pick KB with kb_supported(W, KB, true).
hipError_t launch_jacobi(JacobiArgs a, int W, int KB, hipStream_t s) {
    switch (W) {
    case 1: return launch_jacobi_w<1>(a, KB, s);
    case 2: return launch_jacobi_w<2>(a, KB, s);
    case 3: return launch_jacobi_w<3>(a, KB, s);
    case 4: return launch_jacobi_w<4>(a, KB, s);
    case 5: return launch_jacobi_w<5>(a, KB, s);
    case 6: return launch_jacobi_w<6>(a, KB, s);
    case 7: return launch_jacobi_w<7>(a, KB, s);
    case 8: return launch_jacobi_w<8>(a, KB, s);
    case 9: return launch_jacobi_w<9>(a, KB, s);
    default: {
        if (a.iters != 1) return hipErrorInvalidValue;
        dim3 grd((a.cols + 63) / 64, (a.rows + 3) / 4, a.batch);
        hipLaunchKernelGGL(hs_jacobi_generic_kernel, grd, dim3(256), 0, s, a, W);
        return hipGetLastError();
    }
    }
}

}  // namespace hsflow
