// hsflow_internal.h -- shared between the kernels and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <atomic>
#include <vector>

namespace hsflow {

// Arguments of one Jacobi launch (hornSchunck.cpp:56-74 x `iters`).
struct JacobiArgs {
    int rows, cols, batch;
    int iters;             // iterations fused in this launch (<= KB)
    int tiles_x, tiles_y;  // filled by the launcher
    float alpha2;          // pow(alpha, 2)            (hornSchunck.cpp:68)
    float inv_w2;          // 1 / pow(windowSize, 2)   (hornSchunck.cpp:53)
    const float *u_in, *v_in;  // nullptr -> initial state u = v = 0 (:49-50)
    float *u_out, *v_out;
    const uint32_t *gpack;     // packed exact integer gradients
    const float *gx, *gy, *gt; // f32 gradients (non-integral inputs)
    const uint32_t *flags;     // per pair: 0 -> gpack valid, else f32 planes
    int seg_rows;              // K4 strip kernel: output rows per segment
    int write_through;         // store u', v' write-through (sc1) instead of nt: launches
                               // that do not fill the chip (fill_limited)
};

// K1 (+ K1f): packed gradients and flags; the f32 planes for every pair
// when `planes` (the gradients API), else only for the flagged pairs
hipError_t launch_gradients(const void *I0, const void *I1, int dtype_in, int rows,
                            int cols, int batch, uint32_t *gpack, float *gx, float *gy,
                            float *gt, uint32_t *flags, bool planes, hipStream_t s);
hipError_t launch_jacobi(JacobiArgs a, int W, int KB, hipStream_t s);
// config 5 pyramid (hsflow_pyramid.hip); dtype as HSFLOW_U8/F32/F16
hipError_t launch_pyrdown(const void *src, int dtype, int rows, int cols, int batch,
                          float *dst, const uint32_t *flags, hipStream_t s);
// GPU input path (hsflow_input.hip): dense BGR u8 planes -> gray u8
hipError_t launch_bgr2gray(const uint8_t *bgr, int rows, int cols, int batch,
                           uint8_t *gray, hipStream_t s);
hipError_t launch_upflow(const float *uc, const float *vc, int rc, int cc, float *u,
                         float *v, int rows, int cols, int batch, hipStream_t s);
// K4 (hsflow_strips.hip): the streaming pass for the (window, KB) pairs it
// is built for; `slots` = waves the chip holds at its occupancy
bool strip_supported(int W, int KB);
hipError_t launch_jacobi_strip(JacobiArgs a, int W, int KB, int seg_rows, hipStream_t s);
int strip_seg_rows(int W, int KB, int rows, int cols, int batch, int slots, int *nseg,
                   int *nstrips, int override_rows);
bool strip_fills(int W, int KB, int rows, int cols, int batch, int slots);
// compute units of the current device (cached per device)
int device_cus();
int default_kb(int W);
// default_kb adjusted for launches that do not fill one round of slots
int fill_kb(int W, int kb, int rows, int cols, int batch);
bool kb_supported(int W, int KB, bool need_f32);
// the solve's launches leave most of the chip idle (all pairs in flight):
// their outputs are stored write-through (JacobiArgs::write_through);
// strip_rows = the K4 segment height the launches use (0: 84)
bool fill_limited(int W, int KB, bool strip, int rows, int cols, int batch, int strip_rows);

// ---- host I/O of the host-buffer entry points (hsflow_hostio.cpp) ----
// threads of the host copy pool (the caller included)
int host_pool_width();
// hsflow_set_output_hugepages: advise MADV_HUGEPAGE on f64 outputs (1, default)
extern std::atomic<int> g_output_hugepages;
// n dense device f32 planes -> host rows (f64 when `f64`, else f32; row step
// `step`).  f32: DMA copies straight into the rows.  f64: through `stage`
// (n * rows * cols floats, pinned) in row chunks, each widened by the pool
// as soon as it has arrived.  Returns when every row is in place (the
// stream has drained).
hipError_t download_planes_pipelined(const float *const *src, void *const *dst, int n, int rows,
                                     int cols, bool f64, size_t step, float *stage,
                                     std::vector<hipEvent_t> &events, hipStream_t s);

}  // namespace hsflow
