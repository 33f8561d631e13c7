// hsflow_stream.hip -- K3: streaming (2.5-D temporally blocked) Jacobi pass
// over hornSchunck.cpp:56-74.
//
// K2 (hsflow_kernels.hip) loads a 128 x 80 tile, runs KB iterations on it in
// VGPRs and stores the interior: every iteration recomputes a KB(W-1)-row
// temporal halo above and below (1.76x work at W = 5, KB = 6), and a
// workgroup's load phase and compute phase do not overlap.  K3 removes the
// vertical halo and streams memory under the compute:
//
//  * A workgroup owns one 128-column strip (lane l: columns 2l, 2l+1, as in
//    K2) of a horizontal segment of H output rows, and walks it top to
//    bottom one row per step.  The KB iterations of the pass are KB pipeline
//    STAGES: stage k holds ring buffers of the horizontal sums (and vertical
//    pair sums) of the last W rows of iteration k-1 and emits iteration k of
//    the row AR rows behind its newest input.  Only the horizontal halo
//    (KB(W-1) columns) and the pipeline fill/drain at the segment ends are
//    redundant (1.23x + ~KB(W-1)/H at W = 5, KB = 6).
//  * The S waves of the workgroup split the stages (KB/S each).  Wave 0 loads
//    row r + 2 of (u, v, gradients) while it works on row r (the loads are
//    in flight for two steps), sets up the row's normalised operator
//    (X, Y, T) once, and publishes it in an LDS ring that every stage reads
//    at its own lag.  A wave hands its last stage's output row to the next
//    wave through a double-buffered LDS slot; the next wave consumes it one
//    step later, so the stages of one step are independent across waves and
//    one s_barrier per step orders everything.  The last wave stores.
//  * Outside the image u = v = 0 (BORDER_CONSTANT, hornSchunck.cpp:60-61):
//    the window mean is taken as sum * m with m = 1/w^2 inside the image and
//    0 outside (per-lane column mask, per-step row mask), and the gradients
//    read there are 0, so the update yields 0 without selects.
//  * Same per-pixel operation sequence as K2 (hsflow_device.h: hsum_c2, the
//    vertical pair tree, op_setup, op_update): bit-identical results, so the
//    two kernels can split the passes of one solve.
//
// Even image widths only (8-byte column-pair memory ops); odd widths and a
// short last pass (fewer than KB iterations) take K2.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "hsflow_device.h"
#include "hsflow_internal.h"

// Build-time experiment switches (measured alternatives):
#ifndef K3_PF  // load distance in rows (0: default 2)
#define K3_PF 0
#endif
#ifndef K3_DECOUPLE  // 1: every stage boundary is a one-step hand-off
#define K3_DECOUPLE 0
#endif
#ifndef K3_LATE_OPS  // 1: read each stage's operator row just before it
#define K3_LATE_OPS 1
#endif

namespace hsflow {

template <int W, int KB, int S>
struct K3Geo {
    static constexpr int A = W - W / 2 - 1, AR = W - 1 - A;
    static constexpr int KPW = KB / S;  // stages per wave
    static constexpr int HL = KB * A, HR = KB * AR;
    static constexpr int HLc = HL + (HL & 1), HRc = HR + (HR & 1);
    static constexpr int OX = 128 - HLc - HRc;  // output columns per strip
    // Stage k (1..KB) consumes the row its predecessor emitted in the same
    // step when both are in one wave, and the row emitted one step earlier
    // across a wave boundary (K3_DECOUPLE: at every boundary).  Input row
    // lag D(k) and output row lag LAG(k) behind the newest loaded row:
    static constexpr int D(int k) {
        return K3_DECOUPLE ? (AR + 1) * (k - 1) : AR * (k - 1) + (k - 1) / KPW;
    }
    static constexpr int LAG(int k) { return D(k) + AR; }
    // Operator ring rows: every stage reads its output row's (X, Y, T) from
    // the ring, except the very last one, which reuses the row stage KB-1
    // read GAP steps earlier (register delay line) -- the ring then spans
    // only up to LAG(KB-1).
    static constexpr int LMAX = KB >= 2 ? LAG(KB - 1) : LAG(KB);
    static constexpr int R = LMAX + 1;
    // steps between stage KB-1's read of a row and stage KB's use of it
    static constexpr int GAP = KB >= 2 ? LAG(KB) - LAG(KB - 1) : 1;
    static constexpr int P = (W % 2 == 0) ? W : 2 * W;  // unroll period
    // load distance in rows (5 rows measured no faster than 2 and costs 18
    // VGPRs; K3_PF overrides for experiments)
    static constexpr int PF = (K3_PF > 0 && P % K3_PF == 0) ? K3_PF : 2;
    static_assert(KB % S == 0, "stages split evenly over the waves");
    static_assert(OX > 0 && OX % 2 == 0, "halo too wide for a 128-column strip");
    static_assert(P % PF == 0 && P % 2 == 0, "period");
};

constexpr int k3_mod(int a, int m) { return ((a % m) + m) % m; }

template <int W, int KB, int S>
struct K3Lds {
    using G = K3Geo<W, KB, S>;
    float2 xyt[G::R][3][64];               // operator ring: X, Y, T per row
    float2 lnk[S > 1 ? S - 1 : 1][2][2][64];  // [link][parity][u/v][lane]
};

// One wave's share of the pass: stages J*KPW+1 .. (J+1)*KPW.
template <int W, int KB, int S, bool G32, bool RE, int J>
__device__ __forceinline__ void k3_role(const JacobiArgs &p, K3Lds<W, KB, S> &L, int lane,
                                        int pair, int strip, int seg) {
    using G = K3Geo<W, KB, S>;
    constexpr int A = G::A, AR = G::AR, KPW = G::KPW, P = G::P, PF = G::PF, R = G::R;
    constexpr bool kDelay = (J == S - 1) && KB >= 2;  // last stage uses the delay line
    constexpr int kOOB = 0x7FFFFFF0;
    const int rows = p.rows, cols = p.cols;
    const int y0 = seg * p.seg_rows;
    const int y1 = min(y0 + p.seg_rows, rows);
    const int H = y1 - y0;
    const int r0 = y0 - A * KB;                 // image row of relative row 0
    const int nload = H + (W - 1) * KB;         // rows stage 1 needs
    const int st0 = A * KB + G::LAG(KB);        // first storing step
    const int nsteps = st0 + H;
    const int gce = strip * G::OX - G::HLc + 2 * lane;  // even column of this lane
    const bool ce = (unsigned)gce < (unsigned)cols;     // even width: pair in or out
    const size_t pbase = (size_t)pair * (size_t)rows * (size_t)cols;
    // diagnostics (HSFLOW_ABLATE): 2 = no memory traffic, 4 = no step barrier
    const int plane_bytes = p.ablate == 2 ? 0 : rows * cols * 4;
    const float inv = p.inv_w2;
    // window-mean factor: 1/w^2 inside the image, 0 outside
    const f2v colm = ce ? f2v{inv, inv} : f2v{0.f, 0.f};

    // rings of horizontal sums and vertical pair sums, per local stage, and
    // each stage's last output row (the next stage's input one step later)
    f2v hu[KPW][W], hv[KPW][W], qu[KPW][W], qv[KPW][W], ou[KPW], ov[KPW], mu[KPW], mv[KPW];
#pragma unroll
    for (int i = 0; i < KPW; ++i) {
        ou[i] = ov[i] = mu[i] = mv[i] = f2v{0.f, 0.f};
#pragma unroll
        for (int w = 0; w < W; ++w) hu[i][w] = hv[i][w] = qu[i][w] = qv[i][w] = f2v{0.f, 0.f};
    }
    // last stage's operator rows: AR+1 deep shift register
    constexpr int GAP = G::GAP;
    f2v DX[GAP], DY[GAP], DT[GAP];
#pragma unroll
    for (int d = 0; d < GAP; ++d) DX[d] = DY[d] = DT[d] = f2v{0.f, 0.f};

    // wave 0: load queue of PF rows
    u2v qU[PF], qV[PF], qG[PF], qX[G32 ? PF : 1], qY[G32 ? PF : 1], qT[G32 ? PF : 1];
    __amdgpu_buffer_rsrc_t u_rs, v_rs, g_rs, gx_rs, gy_rs, gt_rs;
    if constexpr (J == 0) {
        u_rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(p.u_in ? p.u_in + pbase : p.u_out + pbase), 0, p.u_in ? plane_bytes : 0,
            0x00020000);
        v_rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(p.v_in ? p.v_in + pbase : p.v_out + pbase), 0, p.v_in ? plane_bytes : 0,
            0x00020000);
        g_rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p.gpack + pbase), 0,
                                                 G32 ? 0 : plane_bytes, 0x00020000);
        gx_rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p.gx + pbase), 0,
                                                  G32 ? plane_bytes : 0, 0x00020000);
        gy_rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p.gy + pbase), 0,
                                                  G32 ? plane_bytes : 0, 0x00020000);
        gt_rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p.gt + pbase), 0,
                                                  G32 ? plane_bytes : 0, 0x00020000);
    }
    auto issue_load = [&](int rel, int slot) {
        const int row = r0 + rel;
        const bool ok = rel < nload && (unsigned)row < (unsigned)rows && ce;
        const int off = ok ? (row * cols + gce) * 4 : kOOB;
        qU[slot] = __builtin_amdgcn_raw_buffer_load_b64(u_rs, off, 0, 0);
        qV[slot] = __builtin_amdgcn_raw_buffer_load_b64(v_rs, off, 0, 0);
        if constexpr (G32) {
            qX[slot] = __builtin_amdgcn_raw_buffer_load_b64(gx_rs, off, 0, 0);
            qY[slot] = __builtin_amdgcn_raw_buffer_load_b64(gy_rs, off, 0, 0);
            qT[slot] = __builtin_amdgcn_raw_buffer_load_b64(gt_rs, off, 0, 0);
        } else {
            qG[slot] = __builtin_amdgcn_raw_buffer_load_b64(g_rs, off, 0, 0);
        }
    };
    if constexpr (J == 0) {
#pragma unroll
        for (int i = 0; i < PF; ++i) issue_load(i, i);
    }

    // last wave: output descriptors and lane mask
    const bool st_lane = lane >= G::HLc / 2 && lane < (G::HLc + G::OX) / 2 && ce;
    const auto uo_rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p.u_out + pbase), 0,
                                                         plane_bytes, 0x00020000);
    const auto vo_rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p.v_out + pbase), 0,
                                                         plane_bytes, 0x00020000);

    // operator rows of step s's stages (K3_LATE_OPS: each read just before
    // its stage; else all issued first in the step)
    f2v Xk[KPW], Yk[KPW], Tk[KPW];
#if !K3_LATE_OPS
    auto fetch_ops = [&](int s1) {
        const int rb = s1 % R;
#pragma unroll
        for (int i = 0; i < KPW; ++i) {
            const int k = J * KPW + i + 1;
            if (!(kDelay && k == KB)) {
                int ys = rb - G::LAG(k);
                ys += ys < 0 ? R : 0;
                const float2 x2 = L.xyt[ys][0][lane];
                const float2 y2 = L.xyt[ys][1][lane];
                const float2 t2 = L.xyt[ys][2][lane];
                Xk[i] = f2v{x2.x, x2.y};
                Yk[i] = f2v{y2.x, y2.y};
                Tk[i] = f2v{t2.x, t2.y};
            }
        }
    };
#endif

    for (int sb = 0; sb < nsteps; sb += P) {
#pragma unroll
        for (int ph = 0; ph < P; ++ph) {
            const int s = sb + ph;
            if (s >= nsteps) break;
            const int rbase = s % R;  // ring slot of relative row s
#if !K3_LATE_OPS
            fetch_ops(s);
#endif
            if constexpr (kDelay) {
                Xk[KPW - 1] = DX[GAP - 1];
                Yk[KPW - 1] = DY[GAP - 1];
                Tk[KPW - 1] = DT[GAP - 1];
            }
            // first stage's input row
            f2v in_u, in_v;
            if constexpr (J == 0) {
                // row s arrives: operator set-up, ring publish, next load
                const int slot = ph % PF;
                float ixe, iye, ite, ixo, iyo, ito;
                if constexpr (G32) {
                    ixe = __uint_as_float(qX[slot].x); ixo = __uint_as_float(qX[slot].y);
                    iye = __uint_as_float(qY[slot].x); iyo = __uint_as_float(qY[slot].y);
                    ite = __uint_as_float(qT[slot].x); ito = __uint_as_float(qT[slot].y);
                } else {
                    unpack_grad(qG[slot].x, ixe, iye, ite);
                    unpack_grad(qG[slot].y, ixo, iyo, ito);
                }
                f2v X, Y, T;
                op_setup(p.alpha2, ixe, iye, ite, ixo, iyo, ito, X, Y, T);
                L.xyt[rbase][0][lane] = make_float2(X.x, X.y);
                L.xyt[rbase][1][lane] = make_float2(Y.x, Y.y);
                L.xyt[rbase][2][lane] = make_float2(T.x, T.y);
                in_u = f2v{__uint_as_float(qU[slot].x), __uint_as_float(qU[slot].y)};
                in_v = f2v{__uint_as_float(qV[slot].x), __uint_as_float(qV[slot].y)};
                issue_load(s + PF, slot);
            } else {
                // the previous wave's last stage, written one step ago
                const int par = (ph + 1) & 1;
                const float2 a = L.lnk[J - 1][par][0][lane];
                const float2 b = L.lnk[J - 1][par][1][lane];
                in_u = f2v{a.x, a.y};
                in_v = f2v{b.x, b.y};
            }
            // Every stage runs every step: during the pipeline fill a stage
            // works on rows before its needed range (ring slots and operator
            // rows not yet written); those outputs never enter a needed
            // row's window (each stage's needed inputs are exactly the
            // previous stage's needed outputs) and are never stored.
            f2v nu[KPW], nv[KPW];
#pragma unroll
            for (int i = 0; i < KPW; ++i) {
                const int k = J * KPW + i + 1;  // global stage index
                const f2v xu = i == 0 ? in_u : (K3_DECOUPLE ? ou[i - 1] : nu[i - 1]);
                const f2v xv = i == 0 ? in_v : (K3_DECOUPLE ? ov[i - 1] : nv[i - 1]);
                // relative input row t = s - D(k); ring slots by t mod W
                const int sl = k3_mod(ph - G::D(k), W);
                const int sp = k3_mod(ph - G::D(k) - 1, W);
                {
                    float a, b, c, d;
                    hsum_c2<W>(xu.x, xu.y, xv.x, xv.y, a, b, c, d);
                    hu[i][sl] = f2v{a, b};
                    hv[i][sl] = f2v{c, d};
                }
                // Relative row r equals image row r0 + r with r0 even
                // (launch_k3), so the vertical sums follow image-row parity
                // exactly as in K2 (hsflow_kernels.hip, wg_body_p): w = 5
                // pair sums at odd rows and shared cores at even rows, w = 3
                // pair sums at even rows.  sb is a multiple of the even P.
                const int tph = ph - G::D(k);  // input row, relative to sb
                if ((W != 3 && W != 5) || k3_mod(tph - 1, 2) == (W == 5 ? 1 : 0)) {
                    qu[i][sp] = hu[i][sp] + hu[i][sl];
                    qv[i][sp] = hv[i][sp] + hv[i][sl];
                }
                // output row y = t - AR
                const int yph = ph - G::LAG(k);
                const bool yev = k3_mod(yph, 2) == 0;
                f2v su, sv;
                if constexpr (W == 5) {
                    const int s0 = k3_mod(yph - 2, W), s1 = k3_mod(yph - 1, W),
                              s2 = k3_mod(yph + 1, W), s3 = k3_mod(yph + 2, W);
                    if (yev) {  // S(y) = h(y-2) + (Q(y-1) + Q(y+1))
                        mu[i] = qu[i][s1] + qu[i][s2];
                        mv[i] = qv[i][s1] + qv[i][s2];
                        su = hu[i][s0] + mu[i];
                        sv = hv[i][s0] + mv[i];
                    } else {  // S(y) = (Q(y-2) + Q(y)) + h(y+2), core of row y-1
                        su = mu[i] + hu[i][s3];
                        sv = mv[i] + hv[i][s3];
                    }
                } else if constexpr (W == 3) {
                    const int s0 = k3_mod(yph - 1, W), s1 = k3_mod(yph, W),
                              s2 = k3_mod(yph + 1, W);
                    if (yev) {  // S(y) = h(y-1) + Q(y)
                        su = hu[i][s0] + qu[i][s1];
                        sv = hv[i][s0] + qv[i][s1];
                    } else {  // S(y) = Q(y-1) + h(y+1)
                        su = qu[i][s0] + hu[i][s2];
                        sv = qv[i][s0] + hv[i][s2];
                    }
                } else {
                    // other windows: pair tree over rows y-A .. y+AR
                    su = qu[i][k3_mod(yph - A, W)];
                    sv = qv[i][k3_mod(yph - A, W)];
#pragma unroll
                    for (int pq = 1; pq < W / 2; ++pq) {
                        const int sq = k3_mod(yph - A + 2 * pq, W);
                        su = su + qu[i][sq];
                        sv = sv + qv[i][sq];
                    }
                    if constexpr (W & 1) {
                        const int sh = k3_mod(yph + AR, W);
                        su = su + hu[i][sh];
                        sv = sv + hv[i][sh];
                    }
                }
#if K3_LATE_OPS
                if (!(kDelay && k == KB)) {
                    int ys = rbase - G::LAG(k);
                    ys += ys < 0 ? R : 0;
                    const float2 x2 = L.xyt[ys][0][lane];
                    const float2 y2 = L.xyt[ys][1][lane];
                    const float2 t2 = L.xyt[ys][2][lane];
                    Xk[i] = f2v{x2.x, x2.y};
                    Yk[i] = f2v{y2.x, y2.y};
                    Tk[i] = f2v{t2.x, t2.y};
                }
#endif
                f2v m = colm;
                if constexpr (RE) {
                    const int yabs = r0 + s - G::LAG(k);
                    if ((unsigned)yabs >= (unsigned)rows) m = f2v{0.f, 0.f};
                }
                op_update(su, sv, m, Xk[i], Yk[i], Tk[i], nu[i], nv[i]);
            }
#pragma unroll
            for (int i = 0; i < KPW; ++i) {
                ou[i] = nu[i];
                ov[i] = nv[i];
            }
            if constexpr (kDelay) {
                // stage KB-1's row this step is stage KB's row AR+1 steps on
#pragma unroll
                for (int d = GAP - 1; d > 0; --d) {
                    DX[d] = DX[d - 1];
                    DY[d] = DY[d - 1];
                    DT[d] = DT[d - 1];
                }
                if constexpr (KPW >= 2) {
                    DX[0] = Xk[KPW - 2];
                    DY[0] = Yk[KPW - 2];
                    DT[0] = Tk[KPW - 2];
                } else {  // stage KB-1 is in the previous wave: read it here
                    int ys = rbase - G::LAG(KB - 1);
                    ys += ys < 0 ? R : 0;
                    const float2 x2 = L.xyt[ys][0][lane];
                    const float2 y2 = L.xyt[ys][1][lane];
                    const float2 t2 = L.xyt[ys][2][lane];
                    DX[0] = f2v{x2.x, x2.y};
                    DY[0] = f2v{y2.x, y2.y};
                    DT[0] = f2v{t2.x, t2.y};
                }
            }
            if constexpr (J < S - 1) {
                const int par = ph & 1;
                L.lnk[J][par][0][lane] = make_float2(ou[KPW - 1].x, ou[KPW - 1].y);
                L.lnk[J][par][1][lane] = make_float2(ov[KPW - 1].x, ov[KPW - 1].y);
            } else {
                if (s >= st0) {
                    const int row = y0 + (s - st0);
                    const int o = st_lane ? (row * cols + gce) * 4 : kOOB;
                    __builtin_amdgcn_raw_buffer_store_b64(
                        u2v{__float_as_uint(ou[KPW - 1].x), __float_as_uint(ou[KPW - 1].y)},
                        uo_rs, o, 0, 0);
                    __builtin_amdgcn_raw_buffer_store_b64(
                        u2v{__float_as_uint(ov[KPW - 1].x), __float_as_uint(ov[KPW - 1].y)},
                        vo_rs, o, 0, 0);
                }
            }
            // LDS-only step barrier (a __syncthreads fence would also wait for
            // wave 0's loads in flight)
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
            if (p.ablate != 4) __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

template <int W, int KB, int S, bool G32, bool RE, int J = 0>
__device__ __forceinline__ void k3_dispatch(const JacobiArgs &p, K3Lds<W, KB, S> &L, int wv,
                                            int lane, int pair, int strip, int seg) {
    if constexpr (J < S) {
        if (wv == J)
            k3_role<W, KB, S, G32, RE, J>(p, L, lane, pair, strip, seg);
        else
            k3_dispatch<W, KB, S, G32, RE, J + 1>(p, L, wv, lane, pair, strip, seg);
    }
}

template <int W, int KB, int S>
__global__ __launch_bounds__(S * 64, 4) void hs_jacobi_stream_kernel(const JacobiArgs p) {
    using G = K3Geo<W, KB, S>;
    __shared__ K3Lds<W, KB, S> L;
    // XCD-aware workgroup order (see hs_jacobi_kernel): each XCD walks a
    // contiguous run of (pair, segment, strip), so neighbouring strips' halo
    // columns and neighbouring segments' overlap rows meet in its L2
    const int nblk = gridDim.x;
    const int lin = blockIdx.x;
    const int qn = nblk >> 3, rem = nblk & 7, xcd = lin & 7;
    const int logical = xcd * qn + min(xcd, rem) + (lin >> 3);
    const int per_pair = p.tiles_x * p.tiles_y;
    const int pair = logical / per_pair;
    const int t = logical - pair * per_pair;
    const int seg = t / p.tiles_x, strip = t - seg * p.tiles_x;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const bool g32 = p.flags != nullptr && p.flags[pair] != 0u;
    // segments whose streamed rows leave the image need the per-step row mask
    const int y0 = seg * p.seg_rows, y1 = min(y0 + p.seg_rows, p.rows);
    const bool re = y0 - G::A * KB < 0 || y1 + G::AR * KB > p.rows;
    if (g32) {
        k3_dispatch<W, KB, S, true, true>(p, L, wv, lane, pair, strip, seg);
    } else if (re) {
        k3_dispatch<W, KB, S, false, true>(p, L, wv, lane, pair, strip, seg);
    } else {
        k3_dispatch<W, KB, S, false, false>(p, L, wv, lane, pair, strip, seg);
    }
}

// ------------------------------------------------------------------ launcher
template <int W, int KB, int S>
static hipError_t launch_k3(JacobiArgs a, hipStream_t s) {
    using G = K3Geo<W, KB, S>;
    a.tiles_x = (a.cols + G::OX - 1) / G::OX;  // strips
    // Segment height: one round of resident workgroups when the
    // batch is small, else whole-strip segments.  HSFLOW_SEG overrides.
    static const int seg_env = [] {
        const char *e = getenv("HSFLOW_SEG");
        return e ? atoi(e) : 0;
    }();
    int seg = seg_env;
    if (seg <= 0) {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess)
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        // resident workgroups per CU (LDS and VGPR limited)
        static const int per_cu = [] {
            int n = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                    &n, reinterpret_cast<const void *>(&hs_jacobi_stream_kernel<W, KB, S>),
                    S * 64, 0) != hipSuccess || n <= 0)
                n = 4;
            return n;
        }();
        const long slots = (long)per_cu * cus;
        const long strips = (long)a.tiles_x * a.batch;
        long nseg = strips >= slots ? 1 : slots / strips;
        if (nseg < 1) nseg = 1;
        seg = (int)((a.rows + nseg - 1) / nseg);
        if (seg < 32) seg = 32;
    }
    // even segment starts: with an even A * KB every relative row has the
    // parity of its image row (the vertical summation order depends on it)
    static_assert((G::A * KB) % 2 == 0, "relative rows keep image-row parity");
    seg += seg & 1;
    a.seg_rows = seg;
    a.tiles_y = (a.rows + seg - 1) / seg;
    const long nwg = (long)a.tiles_x * a.tiles_y * a.batch;
    hipLaunchKernelGGL((hs_jacobi_stream_kernel<W, KB, S>), dim3((unsigned)nwg), dim3(S * 64),
                       0, s, a);
    return hipGetLastError();
}

bool k3_supported(int W, int KB, int cols) {
    if (cols & 1) return false;
    return (W == 5 && KB == 6) || (W == 3 && KB == 8);
}

hipError_t launch_jacobi_stream(JacobiArgs a, int W, int KB, hipStream_t s) {
    if (a.iters != KB || (a.cols & 1)) return hipErrorInvalidValue;
    static const int S_env = [] {
        const char *e = getenv("HSFLOW_K3_WAVES");
        return e ? atoi(e) : 0;
    }();
    if (W == 5 && KB == 6) {
        if (S_env == 2) return launch_k3<5, 6, 2>(a, s);
        if (S_env == 6) return launch_k3<5, 6, 6>(a, s);
        return launch_k3<5, 6, 3>(a, s);
    }
    if (W == 3 && KB == 8) {
        if (S_env == 2) return launch_k3<3, 8, 2>(a, s);
        return launch_k3<3, 8, 4>(a, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace hsflow
