"""K4 lab variants: the product hsflow_strips.hip with textual patches, each
linked with the product's other objects into cpp-optical-flow_amd/lab/
libhsflow_<name>.so (not tracked; travels to the GPU box with the tree).

    python scripts/lab/k4_variants.py build NAME [NAME ...]   # here (hipcc)
    python scripts/lab/k4_variants.py probe NAME [NAME ...]   # GPU box

Variants (timing questions about K4's issue limit):
  base      the product source unchanged (the A/B reference build)
  nop16     +16 `s_nop 0` per time step: does an instruction that is not
            VALU cost the wave issue time (the K4 loop carries ~16 nops and
            ~25 SALU per step)?
  rawoff    loads and stores with the unclamped row offset r * row_bytes (no
            compare / select per row): the most SALU trimming can give
            (timing only; edge rows read garbage)
  short     each segment streams KB AR rows less (timing only): what a
            parallelogram segment's stage-steps cost without its exchange
  oldunpack the per-column v_bfe/v_cvt unpack of the gradients (round 4)
  haloL2    halo rows read as the nearest segment row (timing only): the
            cost of the segments' halo re-reads
  d4        4 rows of prefetch instead of 3 at w = 5
`probe` runs 1080p x 8 and 4K x 2 solves (K4_SHAPES=4k1,1080p1,...: other shapes) (hipGraph replays after a 0.15 s
pre-warm) with each build in its own process, alternating the order twice,
and prints Mpix*iter/s per build."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "cpp-optical-flow_amd")
LAB = os.path.join(PKG, "lab")
SRC = os.path.join(PKG, "csrc", "hsflow_strips.hip")
# the product build of hsflow_strips.hip (cpp-optical-flow_amd/Makefile STRIPS_FLAGS)
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-fno-slp-vectorize",
         "-mllvm", "-amdgpu-sched-strategy=max-ilp"]

PATCHES = {
    "base": [],
    "nop16": [("            __builtin_amdgcn_sched_barrier(0);\n",
               "            asm volatile(\"s_nop 0\\n s_nop 0\\n s_nop 0\\n s_nop 0\\n"
               " s_nop 0\\n s_nop 0\\n s_nop 0\\n s_nop 0\\n s_nop 0\\n s_nop 0\\n"
               " s_nop 0\\n s_nop 0\\n s_nop 0\\n s_nop 0\\n s_nop 0\\n s_nop 0\");\n"
               "            __builtin_amdgcn_sched_barrier(0);\n")],
    "rawoff": [("        return (unsigned)r < (unsigned)rows ? r * row_bytes : (int)0x80000000;",
                "        return r * row_bytes;"),
               ("                    const int so = sin ? y * row_bytes : (int)0x80000000;",
                "                    const int so = y * row_bytes; (void)sin;")],
    # the stream ends KB AR steps early, so no stage works on rows below its
    # segment (timing only: the last rows of every segment are wrong) -- the
    # stage-steps of a parallelogram segment without its exchange traffic
    "short": [("    const int t_last = b - 1 + KB * AR;", "    const int t_last = b - 1;")],
    # no scheduling barrier between time steps: the scheduler may interleave
    # step t's later stages with step t+1's earlier ones (more independent
    # work in flight per wave, more live registers)
    "nosb": [("            __builtin_amdgcn_sched_barrier(0);\n        }\n    };",
              "        }\n    };")],
    # round 4's per-column unpack of the packed gradients (v_bfe + v_cvt
    # for each of the six fields) instead of unpack_grad_pair
    "oldunpack": [("        unpack_grad_pair(d.g.x, d.g.y, ix, iy, it);",
                   "        float ixe, iye, ite, ixo, iyo, ito;\n"
                   "        unpack_grad(d.g.x, ixe, iye, ite);\n"
                   "        unpack_grad(d.g.y, ixo, iyo, ito);\n"
                   "        ix = f2v{ixe, ixo};\n        iy = f2v{iye, iyo};\n"
                   "        it = f2v{ite, ito};")],
    # timing only: rows outside the segment [a, b) load the nearest segment
    # row instead (wrong values; the halo rows' HBM/MALL reads become L2
    # hits of rows the wave just read): what the halo re-read costs, the
    # most an alternating stream direction could win back
    "haloL2": [("    auto issue = [&](RowIn<G32> &d, int r) { load_row<X2, G32>(d, rs, ld_e, ld_o, row_off(r)); };",
                "    auto issue = [&](RowIn<G32> &d, int r) {\n"
                "        load_row<X2, G32>(d, rs, ld_e, ld_o, row_off(r < a ? a : (r >= b ? b - 1 : r)));\n"
                "    };")],
    # timing only: with the alternating directions, rows beyond the END of
    # each stream (below b downwards, above a upwards) load the nearest
    # segment row instead: what the end-boundary halo reads still cost
    "haloEnd": [("    auto issue = [&](RowIn<G32> &d, int r) { load_row<X2, G32>(d, rs, ld_e, ld_o, row_off(r)); };",
                 "    auto issue = [&](RowIn<G32> &d, int r) {\n"
                 "        const int rr = dir > 0 ? (r >= b ? b - 1 : r) : (r < a ? a : r);\n"
                 "        load_row<X2, G32>(d, rs, ld_e, ld_o, row_off(rr));\n"
                 "    };")],
    # progress-ranked wave priority: a wave in the first quarter of its
    # stream runs at priority 3, the last quarter at 0, so a SIMD's lagging
    # wave is issued first (waves that start together stay together, and
    # the end-boundary neighbours read their shared rows closer in time)
    "prio": [("        constexpr int FILL = decltype(fill_c)::value;\n",
              "        constexpr int FILL = decltype(fill_c)::value;\n"
              "        {\n"
              "            const int q = ((tb - t_first) * dir) * 4 / nsteps;\n"
              "            if (q <= 0) __builtin_amdgcn_s_setprio(3);\n"
              "            else if (q == 1) __builtin_amdgcn_s_setprio(2);\n"
              "            else if (q == 2) __builtin_amdgcn_s_setprio(1);\n"
              "            else __builtin_amdgcn_s_setprio(0);\n"
              "        }\n")],
    # 4 rows of prefetch at w = 5 (the stream's loads run a row further
    # ahead; +6 VGPRs)
    "d4": [("template <> struct StripCfg<5, 6> { static constexpr int D = 3, U = 12; };",
            "template <> struct StripCfg<5, 6> { static constexpr int D = 4, U = 12; };")],
    # a barrier every second step only
    # launch bounds of one wave per SIMD (the single-pair launches run ~1
    # wave per SIMD anyway): the allocator may use 512 registers
    "lb1": [("__launch_bounds__(64, 2) void hs_jacobi_strip_kernel",
             "__launch_bounds__(64, 1) void hs_jacobi_strip_kernel")],
    "d4lb1": [("__launch_bounds__(64, 2) void hs_jacobi_strip_kernel",
               "__launch_bounds__(64, 1) void hs_jacobi_strip_kernel"),
              ("template <> struct StripCfg<5, 6> { static constexpr int D = 3, U = 12; };",
               "template <> struct StripCfg<5, 6> { static constexpr int D = 4, U = 12; };")],
    "d6lb1": [("__launch_bounds__(64, 2) void hs_jacobi_strip_kernel",
               "__launch_bounds__(64, 1) void hs_jacobi_strip_kernel"),
              ("template <> struct StripCfg<5, 6> { static constexpr int D = 3, U = 12; };",
               "template <> struct StripCfg<5, 6> { static constexpr int D = 6, U = 12; };")],
    # timing only (wrong values): the stage chain of a time step cut in two
    # -- stages KB/2.. take the level-(KB/2) sums of the PREVIOUS step -- so
    # a lone wave has two independent dependency chains per step: is the
    # single-pair launch latency-bound on the serial stage chain?
    "split": [('    auto block = [&](int tb, auto rowe_c, auto fill_c, auto plain_c) {\n', "    f2v chu = {0.f, 0.f}, chv = {0.f, 0.f};\n" + '    auto block = [&](int tb, auto rowe_c, auto fill_c, auto plain_c) {\n'),
              ('                if (kf < 2 * AR * j) break;  // nor any later stage\n', '                if (kf < 2 * AR * j) break;  // nor any later stage\n' + "                if (j == KB / 2) { const f2v a0 = hu, a1 = hv; hu = chu; hv = chv; chu = a0; chv = a1; }\n")],
    "split3": [('    auto block = [&](int tb, auto rowe_c, auto fill_c, auto plain_c) {\n', "    f2v chu = {0.f, 0.f}, chv = {0.f, 0.f}, dhu = {0.f, 0.f}, dhv = {0.f, 0.f};\n" + '    auto block = [&](int tb, auto rowe_c, auto fill_c, auto plain_c) {\n'),
               ('                if (kf < 2 * AR * j) break;  // nor any later stage\n', '                if (kf < 2 * AR * j) break;  // nor any later stage\n' + "                if (j == 2) { const f2v a0 = hu, a1 = hv; hu = chu; hv = chv; chu = a0; chv = a1; }\n"
                         "                if (j == 4) { const f2v a0 = hu, a1 = hv; hu = dhu; hv = dhv; dhu = a0; dhv = a1; }\n")],
    # timing only: no memory traffic (every load / store out of range, the
    # same instructions), loads only out of range, stores only
    "nomem": [('        return (unsigned)r < (unsigned)rows ? r * row_bytes : (int)0x80000000;', "        return (int)0x80000000; (void)r;"),
              ('                    const int so = sin ? y * row_bytes : (int)0x80000000;', "                    const int so = (int)0x80000000; (void)sin;")],
    "noload": [('        return (unsigned)r < (unsigned)rows ? r * row_bytes : (int)0x80000000;', "        return (int)0x80000000; (void)r;")],
    "nostore": [('                    const int so = sin ? y * row_bytes : (int)0x80000000;', "                    const int so = (int)0x80000000; (void)sin;")],
    # issue cost of one more instruction per time step, by type (timing
    # calibration of a lone wave): 16 independent v_mov, 16 v_pk_add_f32,
    # 16 s_mov per step, results unused
    "valu16": [('            __builtin_amdgcn_sched_barrier(0);\n', '            { int d0_, d1_, d2_, d3_; asm volatile("v_mov_b32 %0, 0\\nv_mov_b32 %1, 1\\nv_mov_b32 %2, 2\\nv_mov_b32 %3, 3\\nv_mov_b32 %0, 4\\nv_mov_b32 %1, 5\\nv_mov_b32 %2, 6\\nv_mov_b32 %3, 7\\nv_mov_b32 %0, 8\\nv_mov_b32 %1, 9\\nv_mov_b32 %2, 10\\nv_mov_b32 %3, 11\\nv_mov_b32 %0, 12\\nv_mov_b32 %1, 13\\nv_mov_b32 %2, 14\\nv_mov_b32 %3, 15" : "=v"(d0_), "=v"(d1_), "=v"(d2_), "=v"(d3_)); }\n            __builtin_amdgcn_sched_barrier(0);\n')],
    "pk16": [('            __builtin_amdgcn_sched_barrier(0);\n', '            { f2v d0_, d1_, d2_, d3_; asm volatile("v_pk_add_f32 %0, %4, %4\\nv_pk_add_f32 %1, %4, %4\\nv_pk_add_f32 %2, %4, %4\\nv_pk_add_f32 %3, %4, %4\\nv_pk_add_f32 %0, %4, %4\\nv_pk_add_f32 %1, %4, %4\\nv_pk_add_f32 %2, %4, %4\\nv_pk_add_f32 %3, %4, %4\\nv_pk_add_f32 %0, %4, %4\\nv_pk_add_f32 %1, %4, %4\\nv_pk_add_f32 %2, %4, %4\\nv_pk_add_f32 %3, %4, %4\\nv_pk_add_f32 %0, %4, %4\\nv_pk_add_f32 %1, %4, %4\\nv_pk_add_f32 %2, %4, %4\\nv_pk_add_f32 %3, %4, %4" : "=v"(d0_), "=v"(d1_), "=v"(d2_), "=v"(d3_) : "v"(colm)); }\n            __builtin_amdgcn_sched_barrier(0);\n')],
    "salu16": [('            __builtin_amdgcn_sched_barrier(0);\n', '            { int d0_, d1_, d2_, d3_; asm volatile("s_mov_b32 %0, 0\\ns_mov_b32 %1, 1\\ns_mov_b32 %2, 2\\ns_mov_b32 %3, 3\\ns_mov_b32 %0, 4\\ns_mov_b32 %1, 5\\ns_mov_b32 %2, 6\\ns_mov_b32 %3, 7\\ns_mov_b32 %0, 8\\ns_mov_b32 %1, 9\\ns_mov_b32 %2, 10\\ns_mov_b32 %3, 11\\ns_mov_b32 %0, 12\\ns_mov_b32 %1, 13\\ns_mov_b32 %2, 14\\ns_mov_b32 %3, 15" : "=s"(d0_), "=s"(d1_), "=s"(d2_), "=s"(d3_)); }\n            __builtin_amdgcn_sched_barrier(0);\n')],
    # launches of lone waves (write-through ones, under 3/4 of the wave
    # slots) ask for 40 KB of LDS per wave they do not use: at most 4
    # workgroups per CU, so the dispatcher cannot put two of the launch's
    # waves on one SIMD while another SIMD idles
    "lds40": [("hs_jacobi_strip_kernel<W, KB, C::D, C::U, C::WPE, true>), grd,\n                           dim3(64), 0, s, a);",
               "hs_jacobi_strip_kernel<W, KB, C::D, C::U, C::WPE, true>), grd,\n                           dim3(64), 40960, s, a);")],
    # timing record (lab only): each wave of a K4 launch stores its start
    # and end (s_memrealtime, 100 MHz), its hardware id (XCC, SE, CU, SIMD)
    # and its segment / strip into a module array that
    # hsflow_lab_k4_stamps() copies out (the last K4 launch's waves)
    "stamp": [("#pragma clang fp contract(off)\n",
               "#pragma clang fp contract(off)\n"
               "__device__ unsigned long long g_k4_stamps[16384 * 4];\n"
               "extern \"C\" int hsflow_lab_k4_stamps(void *host, int n) {\n"
               "    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_k4_stamps),\n"
               "                                    (size_t)n * 32, 0, hipMemcpyDeviceToHost);\n"
               "}\n"),
              ("    const int dir = (seg & 1) ? -1 : 1;\n    if (g32) {",
               "    const int dir = (seg & 1) ? -1 : 1;\n"
               "    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();\n"
               "    if (g32) {"),
              ("            strip_body<W, KB, D, U, false, false, WT>(p, pbase, plane_bytes, c0, a, b, dir);\n    }\n}",
               "            strip_body<W, KB, D, U, false, false, WT>(p, pbase, plane_bytes, c0, a, b, dir);\n    }\n"
               "    {\n"
               "        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();\n"
               "        unsigned hw = 0, xcc = 0;\n"
               "        asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\" : \"=s\"(hw));\n"
               "        asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)\" : \"=s\"(xcc));\n"
               "        if ((threadIdx.x & 63) == 0 && lin < 16384) {\n"
               "            g_k4_stamps[4 * lin] = t_start;\n"
               "            g_k4_stamps[4 * lin + 1] = t_end;\n"
               "            g_k4_stamps[4 * lin + 2] = ((unsigned long long)xcc << 32) | hw;\n"
               "            g_k4_stamps[4 * lin + 3] = ((unsigned long long)seg << 32) | (unsigned)sx;\n"
               "        }\n"
               "    }\n"
               "}")],
    # timing only (wrong values): the update without the two window-mean
    # products per stage (12 fewer packed multiplies per time step): does
    # a lone wave's time follow its instruction count?
    "nomul": [("                op_update(Su, Sv, colm, OX[sl], OY[sl], OT[sl], nu, nv);",
               "                {\n"
               "                    const f2v k_ = fma2(OX[sl], Su, fma2(OY[sl], Sv, OT[sl]));\n"
               "                    nu = fma2(-OX[sl], k_, Su);\n"
               "                    nv = fma2(-OY[sl], k_, Sv);\n"
               "                }")],
    # timing only (wrong values): the horizontal sums as plain adds (the
    # same count, no cross-lane DPP operand): what the DPP form costs
    "nodpp": [("    hsum_c2<W>(u.x, u.y, v.x, v.y, a, b, c, d);",
               "    {\n"
               "        const float pu = u.x + u.y, pv = v.x + v.y;\n"
               "        const float au = launder_f(pu + u.y), av = launder_f(pv + v.y);\n"
               "        const float bu = launder_f(u.x + pu), bv = launder_f(v.x + pv);\n"
               "        a = launder_f(au + u.x); c = launder_f(av + v.x);\n"
               "        b = launder_f(bu + pu); d = launder_f(bv + pv);\n"
               "    }")],
    # timing only (wrong at the image's side columns): the window-mean
    # factor uniform over the wave, so the compiler can take it from an SGPR
    # pair (op_sel_hi) instead of a VGPR pair in the packed multiply-adds
    "csgpr": [("    const f2v colm = {ce ? p.inv_w2 : 0.f, co ? p.inv_w2 : 0.f};",
               "    const f2v colm = {p.inv_w2, p.inv_w2};")],
    # timing record (lab only): lane 0 of every wave stores the shader
    # clock (s_memtime) at the start of each unrolled block of its stream
    # and at its end, slots [lin][0..15] of a module array that
    # hsflow_lab_k4_bstamps() copies out (the last K4 launch's waves)
    "bstamp": [("#pragma clang fp contract(off)\n",
                "#pragma clang fp contract(off)\n"
                "__device__ unsigned long long g_k4_bstamps[16384 * 16];\n"
                "extern \"C\" int hsflow_lab_k4_bstamps(void *host, int n) {\n"
                "    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_k4_bstamps),\n"
                "                                    (size_t)n * 128, 0, hipMemcpyDeviceToHost);\n"
                "}\n"),
               ("    auto block = [&](int tb, auto rowe_c, auto fill_c, auto plain_c) {\n",
                "    auto block = [&](int tb, auto rowe_c, auto fill_c, auto plain_c) {\n"
                "        {\n"
                "            const int bi_ = (tb - t_first) * dir / U;\n"
                "            const unsigned long long ts_ = __builtin_amdgcn_s_memtime();\n"
                "            if (lane == 0 && blockIdx.x < 16384 && bi_ < 15)\n"
                "                g_k4_bstamps[blockIdx.x * 16 + bi_] = ts_;\n"
                "        }\n"),
               ("    for (; ib < nblk; tb += dir * U, ++ib) block(tb, std::true_type{}, F0{}, NP{});\n}",
                "    for (; ib < nblk; tb += dir * U, ++ib) block(tb, std::true_type{}, F0{}, NP{});\n"
                "    {\n"
                "        const unsigned long long ts_ = __builtin_amdgcn_s_memtime();\n"
                "        if (lane == 0 && blockIdx.x < 16384) g_k4_bstamps[blockIdx.x * 16 + 15] = ts_ | ((unsigned long long)nblk << 56);\n"
                "    }\n"
                "}")],
    # the pipeline fill's two blocks as iterations of the row-zeroing loop
    # body (every stage runs from the stream's first step, as before round
    # 5's fill skipping; the same bits): the fill then runs code the wave
    # re-uses instead of ~24 steps of straight-line code fetched once per
    # wave -- is the fill's slowness at full chip instruction fetch?
    "nofill": [("    block(tb, std::true_type{}, std::integral_constant<int, 1>{}, NP{});\n"
                "    tb += dir * U;\n"
                "    block(tb, std::true_type{}, std::integral_constant<int, 2>{}, NP{});\n"
                "    tb += dir * U;\n",
                "    for (int f_ = 0; f_ < 2; ++f_, tb += dir * U)\n"
                "        block(tb, std::true_type{}, F0{}, NP{});\n")],
    # the waves dispatched after one per SIMD (blockIdx.x >= 1024, the
    # second wave of a SIMD in a full-chip launch) start their stream 6 or
    # 12 us late, so the two waves' fills (memory-bound, 2.5x the steady
    # step time when every wave of the chip fills at once) do not overlap
    "stag4": [("    const int dir = (seg & 1) ? -1 : 1;\n",
                "    const int dir = (seg & 1) ? -1 : 1;\n"
                "    if (blockIdx.x >= 1024) {\n"
                "        const long t0_ = wall_clock64();\n"
                "        while (wall_clock64() - t0_ < 400) __builtin_amdgcn_s_sleep(8);\n"
                "    }\n")],
    "stag8": [("    const int dir = (seg & 1) ? -1 : 1;\n",
                "    const int dir = (seg & 1) ? -1 : 1;\n"
                "    if (blockIdx.x >= 1024) {\n"
                "        const long t0_ = wall_clock64();\n"
                "        while (wall_clock64() - t0_ < 800) __builtin_amdgcn_s_sleep(8);\n"
                "    }\n")],
    "stag12": [("    const int dir = (seg & 1) ? -1 : 1;\n",
                "    const int dir = (seg & 1) ? -1 : 1;\n"
                "    if (blockIdx.x >= 1024) {\n"
                "        const long t0_ = wall_clock64();\n"
                "        while (wall_clock64() - t0_ < 1200) __builtin_amdgcn_s_sleep(8);\n"
                "    }\n")],
    "stag16": [("    const int dir = (seg & 1) ? -1 : 1;\n",
                "    const int dir = (seg & 1) ? -1 : 1;\n"
                "    if (blockIdx.x >= 1024) {\n"
                "        const long t0_ = wall_clock64();\n"
                "        while (wall_clock64() - t0_ < 1600) __builtin_amdgcn_s_sleep(8);\n"
                "    }\n")],
    # prefetch depth 4 / 6 rows at w = 5 with one wave per SIMD's register
    # budget (the lone-wave launches: 4K pair), current source
    "d4w1": [("template <> struct StripCfg<5, 6> { static constexpr int D = 3, U = 12, WPE = 2; };",
               "template <> struct StripCfg<5, 6> { static constexpr int D = 4, U = 12, WPE = 1; };")],
    "d6w1": [("template <> struct StripCfg<5, 6> { static constexpr int D = 3, U = 12, WPE = 2; };",
               "template <> struct StripCfg<5, 6> { static constexpr int D = 6, U = 12, WPE = 1; };")],
    # the operator set-up of row t first in the step (into temporaries,
    # written to its ring slot after stage KB has read it): independent
    # work ahead of the stage chain for the scheduler to interleave
    "ropfirst": [("            // 2. level-0 horizontal sums of row t\n",
                  "            f2v rX_, rY_, rT_;\n"
                  "            row_op<G32>(a2c, cur, rX_, rY_, rT_);\n"
                  "            // 2. level-0 horizontal sums of row t\n"),
                 ("            row_op<G32>(a2c, cur, OX[k % L], OY[k % L], OT[k % L]);\n",
                  "            OX[k % L] = rX_;\n            OY[k % L] = rY_;\n            OT[k % L] = rT_;\n")],
    # a scheduling barrier after the third stage of each time step: the
    # operator set-up's instructions stay in the region of stages 4-6, where
    # the post-RA scheduler uses them as wait-state fillers (1910 -> 1883
    # instructions per 12 interior steps)
    "sbmid": [("                if (j + 1 < KB) {\n                    hrow<W>(nu, nv, hu, hv);\n",
               "                if (j == 2) __builtin_amdgcn_sched_barrier(0);\n"
               "                if (j + 1 < KB) {\n                    hrow<W>(nu, nv, hu, hv);\n")],
    "sb2": [("            __builtin_amdgcn_sched_barrier(0);\n        }\n    };",
             "            if (k % 2 == 1) __builtin_amdgcn_sched_barrier(0);\n        }\n    };")],
}


# variants that are another variant's source compiled with other scheduler
# options: name -> (source variant, extra hipcc flags)
FLAG_VARIANTS = {
    "ilp": ("base", ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]),
    "ropfirstilp": ("ropfirst", ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]),
    "split3ilp": ("split3", ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]),
    "iilp": ("base", ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]),
    "split3iilp": ("split3", ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]),
}


# variants that stack other variants' patches: name -> patch names
COMBOS = {"nofillbs": ["nofill", "bstamp"], "d6w1bs": ["d6w1", "bstamp"]}


def build(name):
    os.makedirs(LAB, exist_ok=True)
    src = open(SRC).read()
    base, extra = FLAG_VARIANTS.get(name, (name, []))
    for pname in COMBOS.get(base, [base]):
        for old, new in PATCHES[pname]:
            assert old in src, (name, old)
            src = src.replace(old, new)
    path = os.path.join(PKG, "csrc", f"_lab_strips_{name}.hip")
    with open(path, "w") as f:
        f.write(src)
    obj = os.path.join(LAB, f"strips_{name}.o")
    try:
        subprocess.check_call(["/opt/rocm/bin/hipcc", *FLAGS, *extra, "-c", path, "-o", obj])
    finally:
        os.remove(path)
    objs = [os.path.join(PKG, "build", f) for f in sorted(os.listdir(os.path.join(PKG, "build")))
            if f.endswith(".o") and f != "hsflow_strips.o"]
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", "-o",
                           os.path.join(LAB, f"libhsflow_{name}.so"), *objs, obj,
                           "-Wl,-rpath,/opt/rocm/lib"])
    print("built", name, flush=True)


CHILD = r'''
import os, sys, time, json
sys.path.insert(0, %(pkg)r)
import hsflow
hsflow.LIB_PATH = %(lib)r
import numpy as np, torch
out = {}
SHAPES = {"1080p8": (8, 1080, 1920, 300), "4k2": (2, 2160, 3840, 500),
          "4k1": (1, 2160, 3840, 500), "1080p1": (1, 1080, 1920, 300),
          "1080p8w3": (8, 1080, 1920, 300, 3), "1440p1": (1, 1440, 2560, 300)}
for tag in os.environ.get("K4_SHAPES", "1080p8,4k2").split(","):
    batch, rows, cols, iters, win = (SHAPES[tag] + (5,))[:5]
    ps = [hsflow.synth_pair(1000 + i, rows, cols) for i in range(batch)]
    I0 = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
    I1 = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
    u = torch.empty((batch, rows, cols), dtype=torch.float32, device="cuda"); v = torch.empty_like(u)
    ws = hsflow.alloc_workspace(rows, cols, batch)
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        hsflow.flow_device(I0, I1, win, iters, 1.0, u, v, ws, s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with hsflow.max_streams_as(2), torch.cuda.graph(g, capture_error_mode="thread_local"):
        hsflow.flow_device(I0, I1, win, iters, 1.0, u, v, ws, torch.cuda.current_stream())
    t = time.perf_counter(); n = 0
    while time.perf_counter() - t < 0.15:
        g.replay(); n += 1
        if n %% 4 == 0: torch.cuda.synchronize()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): g.replay()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    out[tag] = {"ms": round(ms, 4), "Mpix_iter_s": round(batch * rows * cols * iters / ms / 1e3),
                "u_sum": float(u.double().sum())}
print("RESULT " + json.dumps(out), flush=True)
'''


def probe(names):
    res = {n: [] for n in names}
    order = list(names) + list(reversed(names))
    for n in order:
        lib = os.path.join(LAB, f"libhsflow_{n}.so")
        code = CHILD % {"pkg": PKG, "lib": lib}
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                           timeout=240)
        line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")]
        if r.returncode != 0 or not line:
            print(n, "FAILED", r.returncode, r.stderr[-2000:], flush=True)
            return 1
        res[n].append(json.loads(line[0][7:]))
        print(n, line[0][7:], flush=True)
    print(json.dumps({n: {k: max(x[k]["Mpix_iter_s"] for x in v) for k in v[0]}
                      for n, v in res.items()}), flush=True)
    return 0


if __name__ == "__main__":
    cmd, names = sys.argv[1], sys.argv[2:]
    if cmd == "build":
        for n in names:
            build(n)
    else:
        sys.exit(probe(names))
