/*
 * hsflow.h -- C ABI of libhsflow.so, the MI355X-native Horn-Schunck solver.
 *
 * Drop-in boundary.  The reference (liuyang9609/Cpp-Optical-Flow) exposes
 * its hot path as a header-style C++ class compiled into the caller
 * (HornSchunckOF/hornSchunck.cpp:8-76, pulled in by main.cpp:8):
 *
 *   hornSchunck(int windowSize, int maxIterations, double alpha)   :13-17
 *   void getGradients(cv::Mat prev, cv::Mat next,
 *                     cv::Mat& gx, cv::Mat& gy, cv::Mat& gt)       :19-41
 *   void getFlow(cv::Mat prev, cv::Mat next, cv::Mat& u, cv::Mat& v) :43-75
 *
 * Its FFI surface is therefore C++/cv::Mat; the functions below are the
 * plain-pointer entry points that surface lowers onto (include/hornSchunck.hpp
 * is the cv::Mat adapter with the reference's exact signatures; INTEGRATION.md
 * shows the binding).  No torch or OpenCV types cross this boundary.
 *
 * Semantics (identical to the reference, computed in fp32 on the GPU):
 *   Ix, Iy = 3x3 Sobel of I0 (reflect-101 border), It = I1 - I0;
 *   u = v = 0; repeat `iters` times:
 *     ubar, vbar = windowSize x windowSize box mean (zero border, anchor
 *                  windowSize - windowSize/2 - 1)
 *     c = (Ix ubar + Iy vbar + It) / (alpha^2 + Ix^2 + Iy^2)
 *     u = ubar - Ix c;  v = vbar - Iy c
 * Parity: max|u - u_ref| / max|u_ref| <= 1e-4 against the float64 reference.
 *
 * Threading: a context is used by one host thread at a time.  Host-buffer
 * calls are blocking (as the reference is).  *_device calls are
 * stream-ordered, never synchronise the host and never allocate, so they may
 * be captured into a hipGraph.
 */
#ifndef HSFLOW_H
#define HSFLOW_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HSFLOW_VERSION 20000 /* 2.0.0: separate row steps for I0 and I1 */

/* Status codes (0 ok, <0 error).  The reference has no codes: OpenCV throws
 * cv::Exception (e.g. size mismatch in multiply, hornSchunck.cpp:63-70);
 * the cv::Mat adapter maps every non-zero status to an exception. */
enum {
    HSFLOW_OK = 0,
    HSFLOW_ERR_ARG = -1,   /* null pointer, bad size/window/dtype/stride     */
    HSFLOW_ERR_HIP = -2,   /* HIP runtime error; see hsflow_last_error()      */
    HSFLOW_ERR_OOM = -3,   /* device allocation failed                        */
    HSFLOW_ERR_NODEV = -4, /* no HIP device / device index out of range       */
    HSFLOW_ERR_SIZE = -5   /* prev/next sizes differ (main.cpp:71-73)         */
};

/* Element types.  U8 = CV_8UC1, F32 = CV_32FC1, F64 = CV_64FC1,
 * F16 = CV_16FC1 (config 5 inputs; input only). */
enum { HSFLOW_U8 = 0, HSFLOW_F32 = 1, HSFLOW_F64 = 2, HSFLOW_F16 = 3 };

/* Largest windowSize accepted (hornSchunck.cpp:53 allows any; OpenCV would
 * take a few seconds per iteration at this size already). */
#define HSFLOW_MAX_WINDOW 63

typedef struct hsflow_ctx hsflow_ctx;

int hsflow_version(void);
const char *hsflow_status_string(int status);

/* Build flags of the loaded library: 0 for every build (the diagnostic
 * build of v2.0 is retired; the library reads no environment variable). */
int hsflow_build_flags(void);

/* Context = device + stream + cached device buffers (grow-only). */
int hsflow_create(hsflow_ctx **ctx, int device);
void hsflow_destroy(hsflow_ctx *ctx);
const char *hsflow_last_error(const hsflow_ctx *ctx);
/* The HIP stream the host-buffer calls run on (hipStream_t as void*). */
void *hsflow_stream(hsflow_ctx *ctx);

/* ---- host-buffer, blocking: the reference's two methods ---------------- */

/* hornSchunck::getFlow (hornSchunck.cpp:43-75).  I0/I1: rows x cols, element
 * type dtype_in, row steps in BYTES, one per frame (cv::Mat::step of
 * imagePrev and imageNext; non-continuous ROIs ok, the two may differ).
 * u/v: rows x cols of dtype_out (HSFLOW_F64 = what the reference returns,
 * CV_64FC1, or HSFLOW_F32), row step out_step bytes.  Frames are uploaded as
 * they are; CV_64FC1 frames get their Sobel sums in float64 on the device
 * (hornSchunck.cpp:23-28), each gradient rounded to f32 once. */
int hsflow_flow(hsflow_ctx *ctx, const void *I0, const void *I1, int dtype_in,
                int rows, int cols, size_t in_step0, size_t in_step1, int window,
                int iters, double alpha, void *u, void *v, int dtype_out,
                size_t out_step);

/* Frame-parallel getFlow over several GPUs of this node from ONE process,
 * for C/C++ callers that do not run one process per GPU (the multi-rank
 * form is cpp-optical-flow_amd/frame_parallel.py over torch.distributed).
 * Pair j -- host frames I0[j], I1[j] (rows x cols, dtype_in, row steps
 * in_step0 / in_step1), host outputs u[j], v[j] (dtype_out, out_step) -- is
 * solved on devices[j % n_devices], each listed device by its own host
 * thread, context and stream, exactly as hsflow_flow (same bits).  A device
 * may be listed twice (two streams on one GPU).  Blocking; returns the
 * first error, its message in hsflow_last_error(NULL).  The per-device
 * contexts are kept by the library across calls (no allocation or device
 * synchronisation per call once warm); a context whose call failed is
 * destroyed, not reused.  Concurrent calls that list the same device slot
 * are serialised on that slot only. */
int hsflow_flow_multi(const int *devices, int n_devices, int batch,
                      const void *const *I0, const void *const *I1, int dtype_in, int rows,
                      int cols, size_t in_step0, size_t in_step1, int window, int iters,
                      double alpha, void *const *u, void *const *v, int dtype_out,
                      size_t out_step);

/* Destroys every context hsflow_flow_multi keeps (device buffers, pinned
 * stages, streams); the next multi call creates them again.  Waits for
 * multi calls in progress. */
void hsflow_flow_multi_release(void);

/* hornSchunck::getGradients (hornSchunck.cpp:19-41): gx, gy, gt. */
int hsflow_gradients(hsflow_ctx *ctx, const void *I0, const void *I1, int dtype_in,
                     int rows, int cols, size_t in_step0, size_t in_step1, void *gx,
                     void *gy, void *gt, int dtype_out, size_t out_step);

/* ---- device pointers, stream-ordered ------------------------------------
 * A batch is `batch` (1..65535) independent frame pairs stored back to back:
 * I0[b][rows][cols], dense (pitch = cols elements), likewise u, v.
 * Inputs are U8, F16, F32 or F64.  Outputs are f32.  `stream` is a hipStream_t
 * (NULL = the default stream of the CURRENT device: then the caller must
 * make the buffers' device current); a non-null stream's own device runs the
 * call, whatever device is current.  `workspace` is device memory of at least
 * hsflow_workspace_bytes(rows, cols, batch) bytes, 256-byte aligned. */
size_t hsflow_workspace_bytes(int rows, int cols, int batch);

/* Full solve: gradients + `iters` Jacobi iterations from u = v = 0. */
int hsflow_flow_device(const void *I0, const void *I1, int dtype_in, int rows,
                       int cols, int batch, int window, int iters, float alpha,
                       float *u, float *v, void *workspace, size_t workspace_bytes,
                       void *stream);

/* The two phases separately (bench / profiling / warm starts):
 * gradients into the workspace (optionally also to gx/gy/gt, may be NULL)... */
int hsflow_gradients_device(const void *I0, const void *I1, int dtype_in, int rows,
                            int cols, int batch, float *gx, float *gy, float *gt,
                            void *workspace, size_t workspace_bytes, void *stream);
/* ...then `iters` Jacobi iterations from the gradients in the workspace,
 * starting from (u, v) when warm_start != 0, else from zero. */
int hsflow_jacobi_device(int rows, int cols, int batch, int window, int iters,
                         float alpha, int warm_start, float *u, float *v,
                         void *workspace, size_t workspace_bytes, void *stream);

/* Iterations fused per Jacobi launch (temporal blocking depth) the library
 * picks for this shape; 0 = automatic (default).  Results are bit-identical
 * for every depth.  Process-wide; not thread-safe against running solves. */
int hsflow_set_iters_per_launch(int k);
int hsflow_iters_per_launch(int rows, int cols, int batch, int window);

/* Kernel of the Jacobi passes (one launch per pass of iters_per_launch
 * iterations): 0 = automatic (default: K4 streaming strips where built --
 * windowSize 3 and 5 at their default depth -- K2 register tiles
 * elsewhere), 2 = K2 everywhere, 4 = K4 where built.  Every choice gives
 * identical bits.  Process-wide; not thread-safe against running solves. */
int hsflow_set_jacobi_kernel(int k);

/* Rows per segment of the K4 streaming passes (each wave streams one
 * segment of one 128-column strip); 0 = automatic (default, a cost model of
 * waves per SIMD and row loads).  Results are bit-identical for every
 * choice.  Process-wide; not thread-safe against running solves. */
int hsflow_set_strip_rows(int seg_rows);

/* Name of the kernel that runs the full-depth Jacobi passes of a solve of
 * this shape under the current settings ("hs_jacobi_strip_kernel",
 * "hs_jacobi_wg_kernel", "hs_jacobi_kernel" or "hs_jacobi_generic_kernel");
 * a static string.  For profiles and the bench's roofline record. */
const char *hsflow_jacobi_kernel_name(int rows, int cols, int batch, int window);

/* Rows per K4 segment that a solve of this shape uses under the current
 * settings (hsflow_set_strip_rows, else the automatic choice); 0 when its
 * full-depth passes do not run K4.  For profiles and tests. */
int hsflow_strip_seg_rows(int rows, int cols, int batch, int window);

/* Batches of >= 2 pairs are split over side streams (forked from and joined
 * back to the caller's stream with events) so that concurrent Jacobi
 * launches overlap.  0 = automatic (default): 2 streams for eager calls, no
 * split while the caller's stream is being captured (on ROCm 7.2 a stream
 * forked inside a capture from a capturing stream other than the capture's
 * origin crashes hipStreamEndCapture, and the library cannot tell the
 * origin apart); n >= 1 = up to n streams always (n >= 2 under capture only
 * when the caller captures on the origin stream itself).  Process-wide.
 * hsflow_max_streams returns the current setting. */
int hsflow_set_max_streams(int n);
int hsflow_max_streams(void);

/* Huge-page advice on f64 outputs of the host-buffer calls (hsflow_flow,
 * hsflow_flow_bgr, hsflow_flow_pyramid, hsflow_flow_multi with
 * dtype_out = HSFLOW_F64): before widening the downloaded f32 rows into
 * the caller's CV_64FC1 planes, the library advises MADV_HUGEPAGE over the
 * whole 2 MB extents inside each plane's rows and faults their pages in
 * while the device solve runs (a fresh 4K output: 18.5 ms of 4 KB faults on
 * one thread, ~1.2 ms as 2 MB pages).  The advice STAYS on the caller's
 * allocation after the call (khugepaged may later collapse other parts of
 * it into huge pages); it changes no byte, and memory already resident
 * keeps its pages.  on = 1 (default) advises, 0 does not (the pages are
 * still faulted in ahead, at 4 KB).  Process-wide; returns the previous
 * setting. */
int hsflow_set_output_hugepages(int on);

/* Stream-ordered download of `bytes` from device memory to pinned host
 * memory (hipHostMalloc / torch pin_memory), issued so the runtime moves it
 * with its DMA engines (~46 GB/s over PCIe Gen5) instead of a blit kernel:
 * a download of batch k then overlaps the Jacobi passes of batch k+1 on
 * other streams without taking their workgroup slots (main.cpp:99-104
 * consumes u, v on the host). */
int hsflow_download_device(void *dst, const void *src, size_t bytes, void *stream);

/* ---- coarse-to-fine warm start (north_star config 5) ---------------------
 * The reference's HS has no pyramid; the repository's own multi-resolution
 * code is the precedent (BMOpticalFlow/.../OpticalFlow/MultiResolution.cpp:
 * 9-97 Pyramider, OpticalFlow.cpp:197-210 Add_VectorOffset).  Level l is
 * ceil(rows / 2^l) x ceil(cols / 2^l), made from level l-1 by the 5-tap
 * kernel (2,5,4,5,2)/18 per axis (a = 0.4), stride 2, reflect-101; levels of
 * integer-valued pairs are rounded half-up to integers.  The coarsest level
 * starts from u = v = 0, every finer one from u = 2 u_coarse(y/2, x/2)
 * (likewise v); each level runs `iters` Jacobi iterations of the getFlow
 * loop (hornSchunck.cpp:56-74) on its own gradients.  levels = 1 is
 * hsflow_flow_device exactly. */
#define HSFLOW_MAX_LEVELS 8

/* Size of pyramid level `level` (0 = full size). */
int hsflow_pyramid_level_size(int rows, int cols, int level, int *level_rows,
                              int *level_cols);
size_t hsflow_pyramid_workspace_bytes(int rows, int cols, int batch, int levels);
int hsflow_flow_pyramid_device(const void *I0, const void *I1, int dtype_in, int rows,
                               int cols, int batch, int levels, int window, int iters,
                               float alpha, float *u, float *v, void *workspace,
                               size_t workspace_bytes, void *stream);
/* Host-buffer, blocking form (same conventions as hsflow_flow). */
int hsflow_flow_pyramid(hsflow_ctx *ctx, const void *I0, const void *I1, int dtype_in,
                        int rows, int cols, size_t in_step0, size_t in_step1, int levels,
                        int window, int iters, double alpha, void *u, void *v,
                        int dtype_out, size_t out_step);

/* The pyramid's pieces, for callers that schedule the levels themselves
 * (e.g. cpp-optical-flow_amd/row_bands.py, one 8K pair split over GPUs):
 * levels 1..levels-1 of both frames into caller planes I0_levels[l-1],
 * I1_levels[l-1] (dense f32, batch x level size), rounding decided per pair
 * exactly as hsflow_flow_pyramid_device does; `workspace` as for
 * hsflow_workspace_bytes(rows, cols, batch)... */
int hsflow_pyramid_build_device(const void *I0, const void *I1, int dtype_in, int rows,
                                int cols, int batch, int levels, float *const *I0_levels,
                                float *const *I1_levels, void *workspace,
                                size_t workspace_bytes, void *stream);
/* ...and the warm start of a finer level: u = 2 uc(y/2, x/2), v likewise
 * (rows x cols from rc x cc, dense, batch planes). */
int hsflow_upflow_device(const float *uc, const float *vc, int rc, int cc, float *u,
                         float *v, int rows, int cols, int batch, void *stream);

/* ---- host utilities on the path to the hot loop ------------------------ */

/* main.cpp:13-14 cv::cvtColor(BGR2GRAY) for 8-bit BGR, OpenCV 4.x 15-bit
 * fixed point: Y = (9798 R + 19235 G + 3735 B + 16384) >> 15. */
int hsflow_bgr_to_gray(const uint8_t *bgr, int rows, int cols, size_t bgr_step,
                       uint8_t *gray, size_t gray_step);

/* The same conversion on the device (stream-ordered): `batch` dense BGR
 * planes [batch][rows][cols][3] -> dense gray [batch][rows][cols]. */
int hsflow_bgr_to_gray_device(const uint8_t *bgr, int rows, int cols, int batch,
                              uint8_t *gray, void *stream);

/* main.cpp:50-51 + :13-14 + :97-98 in one call: two decoded 8-bit BGR frames
 * (row steps bgr_step0, bgr_step1 bytes) are uploaded as BGR, converted on
 * the GPU and solved (hornSchunck::getFlow); u/v as in hsflow_flow. */
int hsflow_flow_bgr(hsflow_ctx *ctx, const uint8_t *bgr0, const uint8_t *bgr1, int rows,
                    int cols, size_t bgr_step0, size_t bgr_step1, int window, int iters,
                    double alpha, void *u, void *v, int dtype_out, size_t out_step);

/* Deterministic synthetic frame pair: I0 = smoothed hash noise
 * around 128 (integer-valued 0..255), I1 = I0's texture shifted by
 * (dy, dx) = (qdy/4, qdx/4) px with integer bilinear weights.  Outputs are
 * rows x cols f32 (dense) and/or u8 (either pointer may be NULL). */
int hsflow_synth_pair(uint64_t seed, int rows, int cols, int qdy, int qdx,
                      float *I0, float *I1, uint8_t *I0_u8, uint8_t *I1_u8);

#ifdef __cplusplus
}
#endif
#endif /* HSFLOW_H */
