// hsflow_internal.h -- shared between the kernels and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace hsflow {

// Diagnostic environment switches (HSFLOW_K2_TL, HSFLOW_ABLATE, ...) exist
// only in the probe build (`make probe` -> libhsflow_probe.so, compiled with
// -DHSFLOW_PROBE).  The product library never reads the environment, so no
// variable can change the work a caller (or bench.py) times.
#ifdef HSFLOW_PROBE
constexpr bool kProbeBuild = true;
#else
constexpr bool kProbeBuild = false;
#endif
inline int probe_env(const char *name, int dflt) {
#ifdef HSFLOW_PROBE
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
#else
    (void)name;
    return dflt;
#endif
}

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
    int ablate;                // probe build only (HSFLOW_ABLATE): 1 = no
                               // iterations (memory only), 2 = no memory
                               // traffic (descriptors of size 0); always 0
                               // in the product library
    int band_w;                // K2 workgroup kernel: tile-column band width
                               // of the tile order (0 = row-major; launcher)
#ifdef HSFLOW_DEV_TRACE
    long trace_base;           // development builds: first trace record of
                               // this launch (-1: off)
#endif
};

hipError_t launch_gradients(const void *I0, const void *I1, int dtype_in, int rows,
                            int cols, int batch, uint32_t *gpack, float *gx, float *gy,
                            float *gt, uint32_t *flags, hipStream_t s);
hipError_t launch_jacobi(JacobiArgs a, int W, int KB, hipStream_t s);
// config 5 pyramid (hsflow_pyramid.hip); dtype as HSFLOW_U8/F32/F16
hipError_t launch_pyrdown(const void *src, int dtype, int rows, int cols, int batch,
                          float *dst, const uint32_t *flags, hipStream_t s);
// GPU input path (hsflow_input.hip): dense BGR u8 planes -> gray u8
hipError_t launch_bgr2gray(const uint8_t *bgr, int rows, int cols, int batch,
                           uint8_t *gray, hipStream_t s);
hipError_t launch_upflow(const float *uc, const float *vc, int rc, int cc, float *u,
                         float *v, int rows, int cols, int batch, hipStream_t s);
int default_kb(int W);
// default_kb adjusted for launches that do not fill one round of slots
int fill_kb(int W, int kb, int rows, int cols, int batch);
bool kb_supported(int W, int KB, bool need_f32);

}  // namespace hsflow
