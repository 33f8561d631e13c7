// hsflow_strips.hip -- K4, the streaming Jacobi pass (hornSchunck.cpp:56-74).
//
// One wavefront owns a 128-column strip of one pair (lane l: columns 2l and
// 2l+1 of the strip, as in K2) and a segment of N output rows of it.  It
// streams the segment's rows once per pass -- even segments top to bottom,
// odd ones bottom to top (strip_body's `dir`; written below for the
// downward stream) -- and runs the pass's KB Jacobi iterations as KB
// time-skewed stages in registers:
//
//   time step t: row t of the input state (u, v) and its packed gradients
//     arrive (loaded D steps earlier);  stage 1 updates row t - AR to
//     iteration 1 (its window rows t - W + 1 .. t are complete), stage 2
//     updates row t - 2 AR to iteration 2 from stage 1's rows, ...,
//     stage KB writes row t - KB AR of iteration KB.
//
// Each stage keeps only the vertical-sum state of its input rows (4 packed
// values per field for w = 5, 3 for w = 3); the per-pixel operator
// (X, Y, T, set up once per row) is kept for the KB AR rows the stages are
// apart.  So a pass moves each row of u, v and the gradients through HBM
// once, with no vertical temporal halo inside a segment (only its first
// KB (W - 1) rows are recomputed by the neighbouring segment), no LDS, no
// barriers and no load phase: every wave is independent and its loads run
// D rows ahead of its arithmetic.  Horizontally the strip has K2's halo
// (KB A columns on the left, KB AR on the right, rounded up to even).
//
// The per-pixel operation sequence is K2's (hsflow_kernels.hip): the same
// horizontal sums (hsum_c2, association by column parity), the same
// vertical sums by image-row parity (w = 5: pair sums Q at odd rows, cores
// M at even rows; w = 3: Q at even rows), the same window means formed from
// the scaled core (one fma per row) and the same normalised update
// (op_setup / op_update_mean), so K4 and K2 give identical bits for every
// pass, and a solve may mix them (K2 runs the passes K4 does not cover).
//
// Outside the image u = v = 0 (BORDER_CONSTANT, hornSchunck.cpp:60-61):
// columns through the window-mean factor (0 outside, as in K2's border
// body), rows by a wave-uniform select.  Rows of a stage that precede its
// first complete window (the segment's start-up) are finite garbage that
// only ever reaches rows the segment does not store.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "hsflow_internal.h"
#include "hsflow_device.h"

// no implicit contraction anywhere in K4: the arithmetic's fused
// multiply-adds are explicit (hsflow_device.h), so every instantiation
// rounds exactly as K2 does whatever the compiler's contraction choices
// (a parallelogram-segment variant differed from K2 by 1 ulp in a few rows
// until they were explicit: scripts/k4pg/README.md)
#pragma clang fp contract(off)

namespace hsflow {

namespace {

constexpr int kOOB = 0x7FFFFFF0;

// ---- vertical sums, streamed (one field; f2v = the lane's column pair) ----
// K2's association (by image-row parity), w = 5: Q(t) = h(t) + h(t+1) at
// odd t; M(y) = Q(y-1) + Q(y+1) at even y; S(y) = h(y-2) + M(y) for even y,
// M(y-1) + h(y+2) for odd y.  w = 3: Q(t) = h(t) + h(t+1) at even t;
// S(y) = h(y-1) + Q(y) for even y, Q(y-1) + h(y+1) for odd y.  Rows stream
// downwards: the arrival of h(t) completes the window of y = t - AR.
// Segments alternate direction (strip_body's `dir`): upwards the same state
// machine runs with the row parity flipped (round 3 measured a separately
// written upward stream 4 % slower; this one shares the downward code, and
// the alternation makes neighbouring segments read their shared halo rows
// at the same time -- 4K x 2 +2.1 %, profiles/r05_k4_alt_dir_ab.txt).
//
// Each arrival returns the completed row's window MEAN (c = the lane's
// window-mean factors): the shared core is scaled once and the row's mean
// is fma(h, c, c core) (hsflow_device.h op_update_mean; K2 does the same).
//
// w = 5.  State before an even arrival t: e0 = h(t-4), e1 = h(t-2),
// q = Q(t-3), x = h(t-1); before an odd arrival: x = c M(t-3).
struct VS5 {
    f2v e0, e1, q, x;
};
template <int PT>  // PT: parity of the arriving image row t
__device__ __forceinline__ f2v vs_arrive(VS5 &s, f2v h, f2v c) {
    if constexpr (PT == 0) {
        const f2v qn = s.x + h;  // Q(t-1) = h(t-1) + h(t)
        const f2v m = s.q + qn;  // M(t-2) = Q(t-3) + Q(t-1)
        const f2v mc = m * c;
        const f2v ub = fma2(s.e0, c, mc);  // mean(t-2): h(t-4) and M(t-2)
        s.e0 = s.e1;
        s.e1 = h;
        s.q = qn;
        s.x = mc;
        return ub;
    } else {
        const f2v ub = fma2(h, c, s.x);  // mean(t-2): M(t-3) and h(t)
        s.x = h;
        return ub;
    }
}
// w = 3.  State before an odd arrival t: h1 = h(t-1), h2 = h(t-2); before
// an even arrival: q = c Q(t-2).
struct VS3 {
    f2v h1, h2, q;
};
template <int PT>
__device__ __forceinline__ f2v vs_arrive(VS3 &s, f2v h, f2v c) {
    if constexpr (PT == 1) {
        const f2v qc = (s.h1 + h) * c;     // c Q(t-1), Q(t-1) = h(t-1) + h(t)
        const f2v ub = fma2(s.h2, c, qc);  // mean(t-1): h(t-2) and Q(t-1)
        s.q = qc;
        s.h2 = h;
        return ub;
    } else {
        const f2v ub = fma2(h, c, s.q);  // mean(t-1): Q(t-2) and h(t)
        s.h1 = h;
        return ub;
    }
}

template <int W> struct VSOf;
template <> struct VSOf<3> { using type = VS3; };
template <> struct VSOf<5> { using type = VS5; };

template <bool G32> struct RowIn;
template <> struct RowIn<false> {  // packed exact integer gradients
    f2v u, v;
    u2v g;
};
template <> struct RowIn<true> {  // f32 gradient planes (non-integral inputs)
    f2v u, v, gx, gy, gt;
};

struct Rsrc {
    __amdgpu_buffer_rsrc_t u, v, g, gx, gy, gt, uo, vo;
};

template <bool X2>
__device__ __forceinline__ f2v ld2(__amdgpu_buffer_rsrc_t r, int vo_e, int vo_o, int so) {
    if constexpr (X2) {
        const u2v a = __builtin_amdgcn_raw_buffer_load_b64(r, vo_e, so, 0);
        return f2v{__uint_as_float(a.x), __uint_as_float(a.y)};
    } else {
        return f2v{__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, vo_e, so, 0)),
                   __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, vo_o, so, 0))};
    }
}

template <bool X2, bool G32>
__device__ __forceinline__ void load_row(RowIn<G32> &d, const Rsrc &rs, int vo_e, int vo_o,
                                         int so) {
    d.u = ld2<X2>(rs.u, vo_e, vo_o, so);
    d.v = ld2<X2>(rs.v, vo_e, vo_o, so);
    if constexpr (G32) {
        d.gx = ld2<X2>(rs.gx, vo_e, vo_o, so);
        d.gy = ld2<X2>(rs.gy, vo_e, vo_o, so);
        d.gt = ld2<X2>(rs.gt, vo_e, vo_o, so);
    } else if constexpr (X2) {
        d.g = __builtin_amdgcn_raw_buffer_load_b64(rs.g, vo_e, so, 0);
    } else {
        d.g = u2v{__builtin_amdgcn_raw_buffer_load_b32(rs.g, vo_e, so, 0),
                  __builtin_amdgcn_raw_buffer_load_b32(rs.g, vo_o, so, 0)};
    }
}

// op_setup (hsflow_device.h) for the column pair in packed FP32: the same
// operations per column -- fma(Ix, Ix, alpha^2), fma(Iy, Iy, .), rsq, three
// products -- so the same bits, in half the instructions
template <bool G32>
__device__ __forceinline__ void row_op(f2v a2, const RowIn<G32> &d, f2v &X, f2v &Y,
                                       f2v &T) {
    f2v ix, iy, it;
    if constexpr (G32) {
        ix = d.gx;
        iy = d.gy;
        it = d.gt;
    } else {
        unpack_grad_pair(d.g.x, d.g.y, ix, iy, it);
    }
    const f2v den = fma2(iy, iy, fma2(ix, ix, a2));
    const f2v sc = {__builtin_amdgcn_rsqf(den.x), __builtin_amdgcn_rsqf(den.y)};
    X = ix * sc;
    Y = iy * sc;
    T = it * sc;
}

template <int W>
__device__ __forceinline__ void hrow(f2v u, f2v v, f2v &hu, f2v &hv) {
    if constexpr (W == 5) {
        // hsum_c2's sums without its launder statements (empty asm, which
        // the hazard recogniser pads with s_nops; K4's registers do not
        // need them): the same operations, the same bits
        const float pu = u.x + u.y, pv = v.x + v.y;
        const float au = from_left(pu) + pu, av = from_left(pv) + pv;
        const float bu = from_left(u.y) + pu, bv = from_left(v.y) + pv;
        hu = f2v{au + from_right(u.x), bu + from_right(pu)};
        hv = f2v{av + from_right(v.x), bv + from_right(pv)};
    } else {
        float a, b, c, d;
        hsum_c2<W>(u.x, u.y, v.x, v.y, a, b, c, d);
        hu = f2v{a, b};
        hv = f2v{c, d};
    }
}

}  // namespace

// Segment body: rows [a, b) of strip columns [c0, c0 + 128) of one pair,
// streamed downwards.  U = unroll period (multiple of the operator ring
// KB*AR, of 2 and of D).
template <int W, int KB, int D, int U, bool X2, bool G32, bool WT>
__device__ __forceinline__ void strip_body(const JacobiArgs &p, size_t pbase, int plane_bytes,
                                           int c0, int a, int b, int dir) {
    constexpr int A = W - W / 2 - 1, AR = W / 2;
    static_assert(A == AR, "K4 is built for odd windows");
    constexpr int L = KB * AR;  // operator ring: the rows t - AR .. t - KB AR
    static_assert(U % L == 0 && U % 2 == 0 && U % D == 0, "unroll period");
    using VS = typename VSOf<W>::type;
    constexpr int HLc = KB * A + ((KB * A) & 1), HRc = KB * AR + ((KB * AR) & 1);
    const int lane = threadIdx.x & 63;
    const int cols = p.cols, rows = p.rows;
    const int gce = c0 + 2 * lane;  // this lane's even image column
    const bool ce = (unsigned)gce < (unsigned)cols;
    const bool co = (unsigned)(gce + 1) < (unsigned)cols;
    // window-mean factor of this lane's columns: 1/w^2 inside the image, 0
    // outside (there the loaded gradients are 0 too, so the update is 0)
    const f2v colm = {ce ? p.inv_w2 : 0.f, co ? p.inv_w2 : 0.f};
    // alpha^2 per column, 1 outside the image (hsflow_device.h alpha2_cols)
    const f2v a2c = alpha2_cols(p.alpha2, ce, co);
    const int c4 = gce * 4;
    // per-lane load offsets (the row goes in soffset); X2: one 8-byte word
    // per column pair, wholly inside or outside the image (even width)
    const int ld_e = ce ? c4 : kOOB;
    const int ld_o = co ? c4 + 4 : kOOB;
    const bool st_lane = lane >= HLc / 2 && lane < (128 - HRc) / 2;
    const int st_e = (st_lane && ce) ? c4 : kOOB;
    const int st_o = (st_lane && co) ? c4 + 4 : kOOB;

    Rsrc rs;
    rs.u = __builtin_amdgcn_make_buffer_rsrc((void *)(p.u_in ? p.u_in + pbase : p.u_out + pbase),
                                             0, p.u_in ? plane_bytes : 0, 0x00020000);
    rs.v = __builtin_amdgcn_make_buffer_rsrc((void *)(p.v_in ? p.v_in + pbase : p.v_out + pbase),
                                             0, p.v_in ? plane_bytes : 0, 0x00020000);
    rs.g = __builtin_amdgcn_make_buffer_rsrc((void *)(p.gpack + pbase), 0,
                                             G32 ? 0 : plane_bytes, 0x00020000);
    rs.gx = __builtin_amdgcn_make_buffer_rsrc((void *)(p.gx + pbase), 0, G32 ? plane_bytes : 0,
                                              0x00020000);
    rs.gy = __builtin_amdgcn_make_buffer_rsrc((void *)(p.gy + pbase), 0, G32 ? plane_bytes : 0,
                                              0x00020000);
    rs.gt = __builtin_amdgcn_make_buffer_rsrc((void *)(p.gt + pbase), 0, G32 ? plane_bytes : 0,
                                              0x00020000);
    rs.uo = __builtin_amdgcn_make_buffer_rsrc((void *)(p.u_out + pbase), 0, plane_bytes,
                                              0x00020000);
    rs.vo = __builtin_amdgcn_make_buffer_rsrc((void *)(p.v_out + pbase), 0, plane_bytes,
                                              0x00020000);

    // The stream: rows a - KB A .. b - 1 + KB AR, downwards (dir = 1) from
    // an even first row (segment starts are even, and so is KB A) or upwards
    // (dir = -1) from an odd first row -- one more row streamed when b - 1 +
    // KB AR is even.  Upwards the arrival of h(t) completes the window of
    // t + AR, and K2's parity-ordered sums come out of the same state
    // machine with the row parity flipped (the adds are commutative, the
    // association is the same); an odd first row flips the parity of every
    // arriving row, so the compile-time pattern below serves both
    // directions.  Step k of a stream always handles the same stage and
    // ring slots; only row indices depend on the direction.
    const int t_first = dir > 0 ? a - KB * A : ((b - 1 + KB * AR) | 1);
    const int nsteps = dir > 0 ? b - a + KB * (A + AR) : t_first - (a - KB * A) + 1;
    // Rows outside the image read 0 through the buffer range check, which
    // covers voffset + soffset (gfx950; scripts/ubench/soffset_range.hip):
    // the row's byte offset goes in soffset, 2^31 for rows above the image
    // (no VALU work and no branches per load; a per-lane offset stays
    // constant).  Offsets stay below 2^32: voffset < 2^31, soffset <= 2^31.
    // Rows below the image take 2^31 as well: their own byte offset can pass
    // 2^31 for planes near the 2^29-pixel cap, and voffset kOOB + such an
    // soffset would wrap past 2^32 back into the plane (one wave-uniform
    // compare per row).
    const int row_bytes = cols * 4;
    auto row_off = [&](int r) {
        return (unsigned)r < (unsigned)rows ? r * row_bytes : (int)0x80000000;
    };
    auto issue = [&](RowIn<G32> &d, int r) { load_row<X2, G32>(d, rs, ld_e, ld_o, row_off(r)); };

    RowIn<G32> buf[D];
#pragma unroll
    for (int k = 0; k < D; ++k) issue(buf[k], t_first + dir * k);

    const f2v z = {0.f, 0.f};
    f2v OX[L], OY[L], OT[L];
#pragma unroll
    for (int k = 0; k < L; ++k) OX[k] = OY[k] = OT[k] = z;
    VS su[KB], sv[KB];
#pragma unroll
    for (int j = 0; j < KB; ++j) {
        if constexpr (W == 5) {
            su[j] = VS{z, z, z, z};
            sv[j] = VS{z, z, z, z};
        } else {
            su[j] = VS{z, z, z};
            sv[j] = VS{z, z, z};
        }
    }

    // one unrolled block of U time steps from row tb (even); ROWE: some
    // stage row of the block may lie outside the image (top / bottom
    // segments).  FILL = f > 0: the stream's f-th block, in the pipeline
    // fill, where stage j (0-based) receives no row it needs before its
    // step 2 AR j (its window's first needed input): it starts there (its
    // vertical-sum state depends on the last W arrivals alone, so the
    // skipped steps leave no trace in any row a later stage or a store
    // uses; identical bits).  Σ_j 2 AR j of its KB (N + KB (W - 1)) stage
    // steps: 60 of 648 at w 5, KB 6, N 84.  (Also skipping the operator
    // update of the next 2 AR steps, whose rows are not needed either, gave
    // 1-ulp differences in a segment's first rows on the GPU, not kept.)
    static_assert(2 * AR * KB == 2 * U, "the pipeline fill is two blocks");
    // PLAIN: every row the block loads lies inside the image and every row
    // it stores inside the segment, so the offsets are the rows' own (one
    // scalar add per row from the block's base, no compare / select: the
    // interior blocks of every stream; round 6, a single 4K pair's lone
    // waves issue every instruction, SALU included)
    const int drb = dir * row_bytes;
    auto block = [&](int tb, auto rowe_c, auto fill_c, auto plain_c) {
        constexpr bool ROWE = decltype(rowe_c)::value;
        constexpr int FILL = decltype(fill_c)::value;
        constexpr bool PLAIN = decltype(plain_c)::value;
        // byte offset of the block's first stage-KB row (PLAIN blocks)
        const int ob = PLAIN ? (tb - dir * (KB * AR)) * row_bytes : 0;
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int t = tb + dir * k;
            // 1. this row's input (loaded D steps ago), then the load of
            //    the row D steps ahead into the freed slot
            const RowIn<G32> cur = buf[k % D];
            if constexpr (PLAIN)
                load_row<X2, G32>(buf[k % D], rs, ld_e, ld_o, ob + (k + KB * AR + D) * drb);
            else
                issue(buf[k % D], t + dir * D);
            // 2. level-0 horizontal sums of row t
            f2v hu, hv;
            hrow<W>(cur.u, cur.v, hu, hv);
            // 3. the stages: stage j (1-based) receives row t - (j-1) AR of
            //    iteration j-1 and updates row t - j AR to iteration j
#pragma unroll
            for (int j = 0; j < KB; ++j) {
                const int y = t - dir * ((j + 1) * AR);
                // step within the fill (compile-time after unrolling)
                const int kf = FILL > 0 ? (FILL - 1) * U + k : 1 << 20;
                if (kf < 2 * AR * j) break;  // nor any later stage
                // image-row parity of the arriving row t - j AR (tb even;
                // upwards: flipped, tb odd -- the same pattern)
                const int pt = (k + j * AR) & 1;
                f2v ub, vb;
                if (pt == 0) {
                    ub = vs_arrive<0>(su[j], hu, colm);
                    vb = vs_arrive<0>(sv[j], hv, colm);
                } else {
                    ub = vs_arrive<1>(su[j], hu, colm);
                    vb = vs_arrive<1>(sv[j], hv, colm);
                }
                const int sl = ((k - (j + 1) * AR) % L + L) % L;  // operator slot of row y
                f2v nu, nv;
                op_update_mean(ub, vb, OX[sl], OY[sl], OT[sl], nu, nv);
                if constexpr (ROWE) {
                    if ((unsigned)y >= (unsigned)rows) {  // rows outside the image: 0
                        nu = z;
                        nv = z;
                    }
                }
                if (j + 1 < KB) {
                    hrow<W>(nu, nv, hu, hv);
                } else {
                    // every step issues its two stores (out-of-segment rows
                    // at an out-of-range offset, dropped): the compiler then
                    // counts them in its vmcnt waits, which keep the loads
                    // of the D rows ahead in flight
                    const bool sin = y >= a && y < b;
                    const int so =
                        PLAIN ? ob + k * drb : (sin ? y * row_bytes : (int)0x80000000);
                    const int oe = st_e;
                    // nt, or write-through (sc1) in launches that leave most
                    // of the chip idle (WT, from p.write_through: a 4K pair
                    // +8.5 %; 4K x 2 -2 %, 1080p x 8 -4 % with sc1).  A
                    // template parameter: a run-time branch here cost the
                    // full-chip launches 3 % (profiles/r03_store_policy_ab.txt)
                    {
                        constexpr int AUX = WT ? 16 : 2;
                        if constexpr (X2) {
                            __builtin_amdgcn_raw_buffer_store_b64(
                                u2v{__float_as_uint(nu.x), __float_as_uint(nu.y)}, rs.uo, oe, so,
                                AUX);
                            __builtin_amdgcn_raw_buffer_store_b64(
                                u2v{__float_as_uint(nv.x), __float_as_uint(nv.y)}, rs.vo, oe, so,
                                AUX);
                        } else {
                            const int oo = st_o;
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(nu.x), rs.uo, oe,
                                                                  so, AUX);
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(nu.y), rs.uo, oo,
                                                                  so, AUX);
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(nv.x), rs.vo, oe,
                                                                  so, AUX);
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(nv.y), rs.vo, oo,
                                                                  so, AUX);
                        }
                    }
                }
            }
            // 4. operator of row t, into the slot stage KB has just read
            row_op<G32>(a2c, cur, OX[k % L], OY[k % L], OT[k % L]);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    // three loops, so the blocks whose stage rows all lie inside the image
    // run a body without row zeroing (one body per loop: a two-body loop
    // makes the allocator spill); the rarely used variants take one loop
    // (the block's stage rows are [tb - KB AR, tb + U - 1 - AR])
    // (every stream is at least 3 blocks: N + KB (W - 1) >= 3 U)
    using F0 = std::integral_constant<int, 0>;
    // a block's stage rows: t - dir (j + 1) AR over its U steps and KB stages
    auto inside = [&](int tb) {
        const int e = tb + dir * (U - 1);
        const int lo = dir > 0 ? tb - KB * AR : e + AR;
        const int hi = dir > 0 ? e - AR : tb + KB * AR;
        return lo >= 0 && hi < rows;
    };
    // ... and PLAIN (above): its loads D rows ahead inside the image, its
    // stage-KB rows inside [a, b) (false only near the stream's ends)
    auto within = [&](int r0, int r1, int lo, int hi) {
        return (r0 < r1 ? r0 : r1) >= lo && (r0 < r1 ? r1 : r0) < hi;
    };
    auto plain = [&](int tb) {
        const int e = tb + dir * (U - 1);
        return inside(tb) && within(tb + dir * D, e + dir * D, 0, rows) &&
               within(tb - dir * (KB * AR), e - dir * (KB * AR), a, b);
    };
    const int nblk = (nsteps + U - 1) / U;
    int tb = t_first, ib = 2;
    using NP = std::false_type;
    block(tb, std::true_type{}, std::integral_constant<int, 1>{}, NP{});
    tb += dir * U;
    block(tb, std::true_type{}, std::integral_constant<int, 2>{}, NP{});
    tb += dir * U;
    if constexpr (X2 && !G32) {
        for (; ib < nblk && !inside(tb); tb += dir * U, ++ib)
            block(tb, std::true_type{}, F0{}, NP{});
        for (; ib < nblk && plain(tb); tb += dir * U, ++ib)
            block(tb, std::false_type{}, F0{}, std::true_type{});
    }
    for (; ib < nblk; tb += dir * U, ++ib) block(tb, std::true_type{}, F0{}, NP{});
}

// ---------------------------------------------------------------- kernel
// One wave per (pair, segment, strip); 64-thread workgroups, 8 per CU (two
// waves per SIMD: up to 256 VGPRs).  Logical order: pair, segment, strip
// (strips fastest), so the strips that share halo columns run side by side;
// the XCD-aware remap gives each XCD a contiguous run of them (its L2
// serves the shared halo columns and the rows two segments both read).
template <int W, int KB, int D, int U, int WPE, bool WT>
__global__ __launch_bounds__(64, WPE) void hs_jacobi_strip_kernel(const JacobiArgs p) {
    const int nblk = gridDim.x;
    const int lin = blockIdx.x;
    const int qn = nblk >> 3, rem = nblk & 7, xcd = lin & 7;
    const int logical = xcd * qn + min(xcd, rem) + (lin >> 3);
    const int nstrips = p.tiles_x, nseg = p.tiles_y;
    const int per_pair = nstrips * nseg;
    const int pair = logical / per_pair;
    if (pair >= p.batch) return;
    const int r = logical - pair * per_pair;
    const int seg = r / nstrips, sx = r - seg * nstrips;
    constexpr int A = W - W / 2 - 1, AR = W / 2;
    constexpr int HLc = KB * A + ((KB * A) & 1), HRc = KB * AR + ((KB * AR) & 1);
    constexpr int OX = 128 - HLc - HRc;
    const int c0 = sx * OX - HLc;
    const int a = seg * p.seg_rows;
    const int b = min(p.rows, a + p.seg_rows);  // segments end inside the image
    const size_t pbase = (size_t)pair * (size_t)p.rows * (size_t)p.cols;
    const int plane_bytes = p.rows * p.cols * 4;
    const bool g32 = p.flags != nullptr && p.flags[pair] != 0u;
    // segments alternate direction (even: down, odd: up), so the 2 KB (W - 1)
    // rows two neighbours share are read by both at their starts (an L2 hit
    // for one of them) or both at their ends, instead of one at its start
    // and the other at its end, a whole stream apart
    const int dir = (seg & 1) ? -1 : 1;
    if (g32) {
        if ((p.cols & 1) == 0)
            strip_body<W, KB, D, U, true, true, WT>(p, pbase, plane_bytes, c0, a, b, dir);
        else
            strip_body<W, KB, D, U, false, true, WT>(p, pbase, plane_bytes, c0, a, b, dir);
    } else {
        if ((p.cols & 1) == 0)
            strip_body<W, KB, D, U, true, false, WT>(p, pbase, plane_bytes, c0, a, b, dir);
        else
            strip_body<W, KB, D, U, false, false, WT>(p, pbase, plane_bytes, c0, a, b, dir);
    }
}

// ------------------------------------------------------------- launcher
namespace {
// D rows of prefetch, U = KB AR steps per unrolled block, WPE waves per SIMD
// the register budget is sized for (w = 5, KB 4: 3 waves, <= 168 VGPRs)
template <int W, int KB> struct StripCfg;
template <> struct StripCfg<5, 6> { static constexpr int D = 3, U = 12, WPE = 2; };
template <> struct StripCfg<5, 5> { static constexpr int D = 5, U = 10, WPE = 2; };
template <> struct StripCfg<5, 4> { static constexpr int D = 2, U = 8, WPE = 3; };
template <> struct StripCfg<3, 8> { static constexpr int D = 2, U = 8, WPE = 2; };

template <int W, int KB>
void launch_cfg(const JacobiArgs &a, dim3 grd, bool wt, hipStream_t s) {
    using C = StripCfg<W, KB>;
    if (wt)
        hipLaunchKernelGGL((hs_jacobi_strip_kernel<W, KB, C::D, C::U, C::WPE, true>), grd,
                           dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL((hs_jacobi_strip_kernel<W, KB, C::D, C::U, C::WPE, false>), grd,
                           dim3(64), 0, s, a);
}
}  // namespace

// w = 5 at KB 6 (the default depth) and the shallower 5 and 4 (fewer
// registers per wave: more waves per SIMD for launches that fill part of
// the chip), w = 3 at KB 8
bool strip_supported(int W, int KB) {
    return (W == 5 && KB >= 4 && KB <= 6) || (W == 3 && KB == 8);
}

// Segment rows for a launch.  Each wave streams N rows plus the KB (W - 1)
// halo rows its stages need: tall segments waste little work and re-read
// few rows, short ones give more waves.  Cost model (fitted to same-box
// sweeps): a wave alone on its SIMD takes ~0.45 us per
// streamed row, two waves sharing a SIMD ~0.75 us each; a launch's waves
// come in rounds of 2 per SIMD (the last round at 1 per SIMD if it has at
// most one wave per SIMD); the pass cannot beat its row loads (1.5 KB per
// wave-row) at ~5 TB/s.  Candidates: N >= 48 (w = 5: N >= 12) with N + KB
// (W - 1) a multiple of the unroll period, up to 240 rows.  `override_rows` > 0
// forces N (rounded up to the period).
int strip_seg_rows(int W, int KB, int rows, int cols, int batch, int slots, int *nseg_out,
                   int *nstrips_out, int override_rows) {
    const int A = W - W / 2 - 1, AR = W / 2;
    const int HLc = KB * A + ((KB * A) & 1), HRc = KB * AR + ((KB * AR) & 1);
    const int ox = 128 - HLc - HRc;
    const int U = KB * AR;  // the unroll period (StripCfg)
    const int nstrips = (cols + ox - 1) / ox;
    const long strips = (long)nstrips * batch;
    const int halo = KB * (W - 1);
    auto aligned = [&](int n) {  // smallest n' >= n with (n' + halo) % U == 0, n' even
        while ((n + halo) % U != 0 || (n & 1)) ++n;
        return n;
    };
    int best_n = aligned(override_rows > 0 ? override_rows : 84);
    // w = 5 (KB 6): 84-row segments measured best on every launch that fills
    // one round of wave slots with them (same box, N 48..240: 1080p x 8, 4K
    // x 2, and 8K, where the model below would take 168 rows and one round
    // of waves: 1.13 M against 1.14-1.15 M Mpix*iter/s at 84, alternated on
    // one box).  A single pair whose 84-row waves do not fill one round
    // takes the model's height (round 5, scripts/kernel_choice_sweep.py,
    // profiles/r05_kernel_choice_sweep*.txt: config 5's 8K level-0 band at
    // N = 4, 1176 rows, 48-row segments 16 % faster than 84; it keeps 84 for
    // a 4K pair).  Batches do not follow the model (its heights lost 3-30 %
    // on 1080p x 3..7, whose halves run concurrently on the side streams)
    if (override_rows <= 0 && W == 5 && KB == 6 && batch > 1) {
        // a batch: the tallest of 84, 72, 60, 48 rows whose waves fill 0.6 of
        // the slots (same sweep: 1080p x 3 48 rows, 10 % faster than K2;
        // x 4 60 rows, 11 % faster than 84; x 5..8 and 4K x 2 keep 84)
        for (const int n : {84, 72, 60, 48}) {
            const int na = aligned(n);
            if (strips * ((rows + na - 1) / na) * 10 >= (long)slots * 6 || na == aligned(48)) {
                override_rows = na;
                break;
            }
        }
        best_n = override_rows;
    } else if (override_rows <= 0 && W == 5 && KB == 6 &&
               strips * ((rows + best_n - 1) / best_n) >= slots) {
        override_rows = best_n;
    }
    if (override_rows <= 0) {
        const long simds = slots / 2 > 0 ? slots / 2 : 1;
        double best = -1.0;
        // w = 5 also below 48 rows while every wave runs alone on its SIMD
        // (round 6: a 1440p pair at 36 rows, 1000 waves, 15 % faster than
        // at 48 -- profiles/r06_kb_sweep.txt); others from 48
        const int n0 = (W == 5 && KB == 6) ? 12 : 48;
        for (int n = aligned(n0); n <= 240; n = aligned(n + 1)) {
            const long w = strips * ((rows + n - 1) / n);
            if (n < 48 && w > simds) continue;
            const long rounds = (w + slots - 1) / slots;
            const long last = w - (rounds - 1) * slots;
            const int steps = n + halo;
            const double compute = (double)(rounds - 1) * steps * 0.75 +
                                   (double)steps * (last <= simds ? 0.45 : 0.75);
            const double mem = (double)w * steps * 1536.0 / 5e12 * 1e6;
            const double t = compute > mem ? compute : mem;
            if (best < 0 || t < best - 1e-9) {
                best = t;
                best_n = n;
            }
            if (n >= rows) break;  // taller segments only repeat this one
        }
    }
    *nseg_out = (rows + best_n - 1) / best_n;
    *nstrips_out = nstrips;
    return best_n;
}

// K4 pays when its waves fill a good part of the chip with tall segments:
// at least 0.45 of the wave slots with 84-row segments (same-box sweeps: a
// 4K pair, 37 strips x 26 segments = 962 waves, runs K4 5 % faster than
// K2; two 1080p pairs, 38 x 13 = 494 waves, and a single one, 247, run K2's
// tiles 30 % faster), or (w = 5, a single pair) at least 0.35 with 60-row
// or 48-row segments (round 5: config 5's 8K level-0 band at N = 8, 640 x
// 7680, 814 waves at 60 rows, runs K4 8 % faster than K2; a 1176 x 3840
// band 16 %; a 1440p pair, 750 waves at 48 rows, 12 %; a 1080p pair, 437
// at 48, stays on K2), or (w = 5, a batch) at least 0.6
// with 48-row segments (1080p x 3: 1311 waves, K4 10 % faster than K2;
// 1080p x 2, 874, and 720p x 4, 780, stay on K2).
bool strip_fills(int W, int KB, int rows, int cols, int batch, int slots) {
    int nseg = 0, nstrips = 0;
    strip_seg_rows(W, KB, rows, cols, batch, slots, &nseg, &nstrips, 84);
    if ((long)nseg * nstrips * batch * 20 >= (long)slots * 9) return true;  // >= 0.45
    if (W != 5 || KB != 6) return false;
    if (batch > 1) {  // a batch whose 48-row waves fill 0.6 of the slots
        strip_seg_rows(W, KB, rows, cols, batch, slots, &nseg, &nstrips, 48);
        return (long)nseg * nstrips * batch * 10 >= (long)slots * 6;
    }
    for (const int n : {60, 48}) {  // a single pair: >= 0.35 at 60 or 48 rows
        strip_seg_rows(W, KB, rows, cols, batch, slots, &nseg, &nstrips, n);
        if ((long)nseg * nstrips * batch * 20 >= (long)slots * 7) return true;
    }
    return false;
}

// One K4 pass of `a.batch` pairs in segments of `seg_rows` rows (the
// caller's choice: strip_seg_rows over every pair in flight).
hipError_t launch_jacobi_strip(JacobiArgs a, int W, int KB, int seg_rows, hipStream_t s) {
    int nseg = 0, nstrips = 0;
    a.seg_rows = strip_seg_rows(W, KB, a.rows, a.cols, a.batch, 1, &nseg, &nstrips,
                                seg_rows > 0 ? seg_rows : 84);
    a.tiles_x = nstrips;
    a.tiles_y = nseg;
    const long waves = (long)nstrips * nseg * a.batch;
    if (waves <= 0 || waves > 0x7FFFFFFFL) return hipErrorInvalidValue;
    dim3 grd((unsigned)waves, 1, 1);
    const bool wt = a.write_through != 0;
    if (W == 5 && KB == 6)
        launch_cfg<5, 6>(a, grd, wt, s);
    else if (W == 5 && KB == 5)
        launch_cfg<5, 5>(a, grd, wt, s);
    else if (W == 5 && KB == 4)
        launch_cfg<5, 4>(a, grd, wt, s);
    else if (W == 3 && KB == 8)
        launch_cfg<3, 8>(a, grd, wt, s);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace hsflow
