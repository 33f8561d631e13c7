"""Round-3 experiment, retired (profiles/r03_k4_experiments.jsonl):
writes scratch/strips_<name>.hip = the product K4 file plus K5, two
cooperating waves per strip segment (A = loads + stages 1..SA, B = stages
SA+1..KB, LDS hand-off, one barrier per step, <= 128 VGPRs: 4 waves per
SIMD), launched for w 5 / KB 6.  Bit-identical to K4/K2; 7 % slower.
    python scripts/k5_coop_experiment.py <name> [b2] [pf]
then build it against the product objects (scratch/Makefile X=<name>) and
load it through HSFLOW_LIB."""
import sys
opts = set(sys.argv[2:])
out_name = sys.argv[1] if len(sys.argv) > 1 else "k5"
src = open("cpp-optical-flow_amd/csrc/hsflow_strips.hip").read()
K5 = r'''
// ---------------------------------------------------------------- K5
// Two waves per (pair, segment, strip): wave A streams the rows in, sets
// up the operator and runs stages 1..SA; wave B runs stages SA+1..KB and
// stores.  A hands B, per step, the level-SA row's horizontal sums and the
// operator of row t - SA AR through LDS; one barrier per step (A after its
// step, B before its own, so A's step t+1 overlaps B's step t).  <= 128
// VGPRs per wave: 4 waves per SIMD.
template <int W, int KB, int SA, int D, int U, bool X2, bool G32>
__device__ __forceinline__ void coop_body(const JacobiArgs &p, size_t pbase, int plane_bytes,
                                          int c0, int a, int b, f2v (*s_op)[3][64],
                                          f2v (*s_h)[2][64]) {
    constexpr int A = W - W / 2 - 1, AR = W / 2;
    constexpr int LA = SA * AR;
    constexpr int R = 12;
    static_assert(U % LA == 0 && U % R == 0 && U % 2 == 0 && U % D == 0, "unroll period");
    static_assert(2 * AR * KB == 2 * U, "the pipeline fill is two blocks");
    using VS = typename VSOf<W>::type;
    constexpr int HLc = KB * A + ((KB * A) & 1), HRc = KB * AR + ((KB * AR) & 1);
    const int role = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int cols = p.cols, rows = p.rows;
    const int gce = c0 + 2 * lane;
    const bool ce = (unsigned)gce < (unsigned)cols;
    const bool co = (unsigned)(gce + 1) < (unsigned)cols;
    const f2v colm = {ce ? p.inv_w2 : 0.f, co ? p.inv_w2 : 0.f};
    const int c4 = gce * 4;
    const int t_first = a - KB * A;
    const int t_last = b - 1 + KB * AR;
    const int row_bytes = cols * 4;
    const f2v z = {0.f, 0.f};
    using F0 = std::integral_constant<int, 0>;
    using F1 = std::integral_constant<int, 1>;
    using F2 = std::integral_constant<int, 2>;
    // the LDS operator ring starts at 0 (rows a stage reads before A wrote
    // them only reach rows nobody needs; zero keeps them finite)
    for (int i = threadIdx.x; i < R * 3 * 64; i += 128) (&s_op[0][0][0])[i] = z;
    __syncthreads();
    if (role == 0) {
        const int ld_e = ce ? c4 : kOOB;
        const int ld_o = co ? c4 + 4 : kOOB;
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
        const float alpha2 = p.alpha2;
        auto row_off = [&](int r) { return r >= 0 ? r * row_bytes : (int)0x80000000; };
        auto issue = [&](RowIn<G32> &d, int r) { load_row<X2, G32>(d, rs, ld_e, ld_o, row_off(r)); };
        RowIn<G32> buf[D];
#pragma unroll
        for (int k = 0; k < D; ++k) issue(buf[k], t_first + k);
        f2v OX[LA], OY[LA], OT[LA];
#pragma unroll
        for (int k = 0; k < LA; ++k) OX[k] = OY[k] = OT[k] = z;
        VS su[SA], sv[SA];
#pragma unroll
        for (int j = 0; j < SA; ++j) {
            su[j] = VS{z, z, z, z};
            sv[j] = VS{z, z, z, z};
        }
        auto block = [&](int tb, auto rowe_c, auto fill_c) {
            constexpr bool ROWE = decltype(rowe_c)::value;
            constexpr int FILL = decltype(fill_c)::value;
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int t = tb + k;
                const RowIn<G32> cur = buf[k % D];
                issue(buf[k % D], t + D);
                f2v hu, hv;
                hrow<W>(cur.u, cur.v, hu, hv);
#pragma unroll
                for (int j = 0; j < SA; ++j) {
                    const int y = t - (j + 1) * AR;
                    const int kf = FILL > 0 ? (FILL - 1) * U + k : 1 << 20;
                    if (kf < 2 * AR * j) break;
                    const int pt = (k + j * AR) & 1;
                    f2v Su, Sv;
                    if (pt == 0) {
                        Su = vs_arrive<0>(su[j], hu);
                        Sv = vs_arrive<0>(sv[j], hv);
                    } else {
                        Su = vs_arrive<1>(su[j], hu);
                        Sv = vs_arrive<1>(sv[j], hv);
                    }
                    const int sl = ((k - (j + 1) * AR) % LA + LA) % LA;
                    f2v nu, nv;
                    op_update(Su, Sv, colm, OX[sl], OY[sl], OT[sl], nu, nv);
                    if constexpr (ROWE) {
                        if ((unsigned)y >= (unsigned)rows) {
                            nu = z;
                            nv = z;
                        }
                    }
                    hrow<W>(nu, nv, hu, hv);
                }
                s_h[k & 1][0][lane] = hu;
                s_h[k & 1][1][lane] = hv;
                const int so = k % LA;                  // row t - LA
                const int ro = ((k - LA) % R + R) % R;  // its LDS slot
                s_op[ro][0][lane] = OX[so];
                s_op[ro][1][lane] = OY[so];
                s_op[ro][2][lane] = OT[so];
                row_op<G32>(alpha2, cur, OX[so], OY[so], OT[so]);
                __syncthreads();
            }
        };
        int tb = t_first;
        block(tb, std::true_type{}, F1{});
        tb += U;
        block(tb, std::true_type{}, F2{});
        tb += U;
        if constexpr (X2 && !G32) {
            for (; tb <= t_last && tb - KB * AR < 0; tb += U) block(tb, std::true_type{}, F0{});
            for (; tb <= t_last && tb + U - 1 - AR < rows; tb += U)
                block(tb, std::false_type{}, F0{});
        }
        for (; tb <= t_last; tb += U) block(tb, std::true_type{}, F0{});
    } else {
        const bool st_lane = lane >= HLc / 2 && lane < (128 - HRc) / 2;
        const int st_e = (st_lane && ce) ? c4 : kOOB;
        const int st_o = (st_lane && co) ? c4 + 4 : kOOB;
        __amdgpu_buffer_rsrc_t uo = __builtin_amdgcn_make_buffer_rsrc((void *)(p.u_out + pbase), 0,
                                                                      plane_bytes, 0x00020000);
        __amdgpu_buffer_rsrc_t vo = __builtin_amdgcn_make_buffer_rsrc((void *)(p.v_out + pbase), 0,
                                                                      plane_bytes, 0x00020000);
        constexpr int SB = KB - SA;
        VS su[SB], sv[SB];
#pragma unroll
        for (int j = 0; j < SB; ++j) {
            su[j] = VS{z, z, z, z};
            sv[j] = VS{z, z, z, z};
        }
        auto block = [&](int tb, auto rowe_c, auto fill_c) {
            constexpr bool ROWE = decltype(rowe_c)::value;
            constexpr int FILL = decltype(fill_c)::value;
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int t = tb + k;
                __syncthreads();
                f2v hu = s_h[k & 1][0][lane], hv = s_h[k & 1][1][lane];
#pragma unroll
                for (int j = SA; j < KB; ++j) {
                    const int y = t - (j + 1) * AR;
                    const int kf = FILL > 0 ? (FILL - 1) * U + k : 1 << 20;
                    if (kf < 2 * AR * j) break;
                    const int pt = (k + j * AR) & 1;
                    f2v Su, Sv;
                    if (pt == 0) {
                        Su = vs_arrive<0>(su[j - SA], hu);
                        Sv = vs_arrive<0>(sv[j - SA], hv);
                    } else {
                        Su = vs_arrive<1>(su[j - SA], hu);
                        Sv = vs_arrive<1>(sv[j - SA], hv);
                    }
                    const int ro = ((k - (j + 1) * AR) % R + R) % R;
                    f2v nu, nv;
                    op_update(Su, Sv, colm, s_op[ro][0][lane], s_op[ro][1][lane],
                              s_op[ro][2][lane], nu, nv);
                    if constexpr (ROWE) {
                        if ((unsigned)y >= (unsigned)rows) {
                            nu = z;
                            nv = z;
                        }
                    }
                    if (j + 1 < KB) {
                        hrow<W>(nu, nv, hu, hv);
                    } else {
                        const bool sin = y >= a && y < b;
                        const int so = sin ? y * row_bytes : (int)0x80000000;
                        if constexpr (X2) {
                            __builtin_amdgcn_raw_buffer_store_b64(
                                u2v{__float_as_uint(nu.x), __float_as_uint(nu.y)}, uo, st_e, so, 2);
                            __builtin_amdgcn_raw_buffer_store_b64(
                                u2v{__float_as_uint(nv.x), __float_as_uint(nv.y)}, vo, st_e, so, 2);
                        } else {
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(nu.x), uo, st_e, so, 2);
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(nu.y), uo, st_o, so, 2);
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(nv.x), vo, st_e, so, 2);
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(nv.y), vo, st_o, so, 2);
                        }
                    }
                }
            }
        };
        int tb = t_first;
        block(tb, std::true_type{}, F1{});
        tb += U;
        block(tb, std::true_type{}, F2{});
        tb += U;
        if constexpr (X2 && !G32) {
            for (; tb <= t_last && tb - KB * AR < 0; tb += U) block(tb, std::true_type{}, F0{});
            for (; tb <= t_last && tb + U - 1 - AR < rows; tb += U)
                block(tb, std::false_type{}, F0{});
        }
        for (; tb <= t_last; tb += U) block(tb, std::true_type{}, F0{});
    }
}

template <int W, int KB, int SA, int D, int U>
__global__ __launch_bounds__(128, 4) void hs_jacobi_coop_kernel(const JacobiArgs p) {
    __shared__ f2v s_op[12][3][64];
    __shared__ f2v s_h[2][2][64];
    const int nblk = gridDim.x;
    const int lin = blockIdx.x;
    const int qn = nblk >> 3, rem = nblk & 7, xcd = lin & 7;
    const int logical = xcd * qn + min(xcd, rem) + (lin >> 3);
    const int nstrips = p.tiles_x, nseg = p.tiles_y;
    const int per_pair = nstrips * nseg;
    const int pair = logical / per_pair;
    if (pair >= p.batch) return;  // the whole workgroup
    const int r = logical - pair * per_pair;
    const int seg = r / nstrips, sx = r - seg * nstrips;
    constexpr int A = W - W / 2 - 1, AR = W / 2;
    constexpr int HLc = KB * A + ((KB * A) & 1), HRc = KB * AR + ((KB * AR) & 1);
    constexpr int OX = 128 - HLc - HRc;
    const int c0 = sx * OX - HLc;
    const int a = seg * p.seg_rows;
    const int b = min(p.rows, a + p.seg_rows);
    const size_t pbase = (size_t)pair * (size_t)p.rows * (size_t)p.cols;
    const int plane_bytes = p.rows * p.cols * 4;
    const bool g32 = p.flags != nullptr && p.flags[pair] != 0u;
    if (g32) {
        if ((p.cols & 1) == 0)
            coop_body<W, KB, SA, D, U, true, true>(p, pbase, plane_bytes, c0, a, b, s_op, s_h);
        else
            coop_body<W, KB, SA, D, U, false, true>(p, pbase, plane_bytes, c0, a, b, s_op, s_h);
    } else {
        if ((p.cols & 1) == 0)
            coop_body<W, KB, SA, D, U, true, false>(p, pbase, plane_bytes, c0, a, b, s_op, s_h);
        else
            coop_body<W, KB, SA, D, U, false, false>(p, pbase, plane_bytes, c0, a, b, s_op, s_h);
    }
}
'''
marker = "// ------------------------------------------------------------- launcher"
assert marker in src
src = src.replace(marker, K5 + "\n" + marker, 1)
old = """        using C = StripCfg<5, 6>;
        hipLaunchKernelGGL((hs_jacobi_strip_kernel<5, 6, C::D, C::U>), grd, dim3(64), 0, s, a);"""
assert old in src
src = src.replace(old, """        hipLaunchKernelGGL((hs_jacobi_coop_kernel<5, 6, 2, 3, 12>), grd, dim3(128), 0, s, a);""")
if "pf" in opts:
    a = """        constexpr int SB = KB - SA;
        VS su[SB], sv[SB];"""
    assert a in src
    src = src.replace(a, """        constexpr int SB = KB - SA;
        VS su[SB], sv[SB];
        // each stage's operator for the next step, read one step ahead
        f2v PX[SB], PY[SB], PT[SB];
#pragma unroll
        for (int j = 0; j < SB; ++j) PX[j] = PY[j] = PT[j] = z;""")
    a = """                    const int ro = ((k - (j + 1) * AR) % R + R) % R;
                    f2v nu, nv;
                    op_update(Su, Sv, colm, s_op[ro][0][lane], s_op[ro][1][lane],
                              s_op[ro][2][lane], nu, nv);"""
    assert a in src
    src = src.replace(a, """                    // row t + 1 - (j + 1) AR: written by A at a step <= t - 1
                    const int rn = ((k + 1 - (j + 1) * AR) % R + R) % R;
                    f2v nu, nv;
                    op_update(Su, Sv, colm, PX[j - SA], PY[j - SA], PT[j - SA], nu, nv);
                    PX[j - SA] = s_op[rn][0][lane];
                    PY[j - SA] = s_op[rn][1][lane];
                    PT[j - SA] = s_op[rn][2][lane];""")
if "b2" in opts:
    src = src.replace("""                row_op<G32>(alpha2, cur, OX[so], OY[so], OT[so]);
                __syncthreads();""", """                row_op<G32>(alpha2, cur, OX[so], OY[so], OT[so]);
                if (k & 1) __syncthreads();""")
    src = src.replace("""                const int t = tb + k;
                __syncthreads();
                f2v hu = s_h[k & 1][0][lane], hv = s_h[k & 1][1][lane];""", """                const int t = tb + k;
                if (!(k & 1)) __syncthreads();
                f2v hu = s_h[k & 3][0][lane], hv = s_h[k & 3][1][lane];""")
    src = src.replace("""                s_h[k & 1][0][lane] = hu;
                s_h[k & 1][1][lane] = hv;""", """                s_h[k & 3][0][lane] = hu;
                s_h[k & 3][1][lane] = hv;""")
    src = src.replace("f2v (*s_h)[2][64]) {", "f2v (*s_h)[2][64]) {  // [4] slots")
    src = src.replace("__shared__ f2v s_h[2][2][64];", "__shared__ f2v s_h[4][2][64];")
    src = src.replace("__shared__ f2v s_op[12][3][64];", "__shared__ f2v s_op[12][3][64];  // + 4 KB of s_h")
open(f"scratch/strips_{out_name}.hip", "w").write(src)
