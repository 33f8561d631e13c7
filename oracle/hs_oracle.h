/*
 * hs_oracle.h -- CPU float64 restatement of the reference Horn-Schunck path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker and the
 * "port" CPU baseline.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product path (libhsflow.so) never links
 * or calls it.
 *
 * Reference being restated (liuyang9609/Cpp-Optical-Flow, HornSchunckOF/):
 *   hornSchunck.cpp:19-41  getGradients  (convertTo f64, Sobel x/y, It = I1-I0)
 *   hornSchunck.cpp:43-75  getFlow       (zeros, box kernel, Jacobi loop)
 *   main.cpp:11-26         preprocess    (cv::cvtColor BGR2GRAY, OpenCV 4.x 15-bit)
 *   plotFlow.cpp:24-88     plotBresenhamLine (headless; imshow omitted)
 * The arithmetic lives in OpenCV 4.4.0 (HornSchunckOF/OpenCVx64d.props:6-11),
 * which is not vendored; the OpenCV semantics restated here are:
 *   Sobel ksize 3, BORDER_DEFAULT = reflect-101; filter2D correlation with
 *   anchor (w-w/2-1), BORDER_CONSTANT 0, sum of k*src in kernel row-major
 *   order; cvtColor Y = (9798 R + 19235 G + 3735 B + 16384) >> 15.
 * Pinned by the reference's own output artifacts (the two arrow plots in
 * HornSchunckOF/img/resimage/), see tests/test_oracle_golden.py.
 */
#ifndef HS_ORACLE_H
#define HS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* main.cpp:13-14 -> cv::cvtColor(COLOR_BGR2GRAY) on 8-bit BGR pixels. */
void hso_bgr_to_gray(const uint8_t *bgr, int rows, int cols, size_t row_stride,
                     uint8_t *gray);

/* hornSchunck.cpp:19-41.  I0/I1 are rows*cols float64 (already convertTo'd),
 * outputs rows*cols float64, all dense row-major. */
void hso_gradients(const double *I0, const double *I1, int rows, int cols,
                   double *gx, double *gy, double *gt);

/* hornSchunck.cpp:43-75, op by op: one full-array pass per OpenCV call and
 * fresh temporaries per iteration (the reference's structure; used as the
 * CPU baseline).  nthreads<=1 -> single thread (as the reference). */
void hso_flow(const double *I0, const double *I1, int rows, int cols,
              int window, int iters, double alpha, double *u, double *v,
              int nthreads);

/* Same maths as hso_flow with u,v given as the initial state (warm start);
 * hso_flow == hso_flow_from(u=v=0).  Used for the iteration-continuation
 * tests.  gx/gy/gt are the precomputed gradients. */
void hso_jacobi(const double *gx, const double *gy, const double *gt,
                int rows, int cols, int window, int iters, double alpha,
                double *u, double *v, int nthreads);

/* ---- config 5: coarse-to-fine pyramid warm start ----
 * HornSchunckOF has no pyramid; the design precedent is the repository's
 * BM module: Pyramider (BMOpticalFlow/.../OpticalFlow/MultiResolution.cpp:
 * 9-97: 5-tap kernel w = (a/2, 1/2, a, 1/2, a/2)/sum, a = 0.4, i.e.
 * (2,5,4,5,2)/18, stride 2, level size ceil(n / 2^l), mirrored border) and
 * Add_VectorOffset (OpticalFlow.cpp:197-210: u_l(x,y) += 2 u_{l+1}(x/2,y/2)).
 * The mirror border (ImgVector::get_mirror, not vendored) is taken as
 * reflect-101.  Levels of an integer-valued pair (every pixel of both
 * frames an integer in [0, 255]) are rounded half-up to integers, as an
 * 8-bit pyrDown would:  L = floor((S + 162) / 324), S = sum w_m w_n I;
 * other pairs keep S / 324. */

/* One level down: src rows x cols -> dst ceil(rows/2) x ceil(cols/2). */
void hso_pyrdown(const double *src, int rows, int cols, int round_int, double *dst);

/* 1 if every pixel of both frames is an integer in [0, 255]. */
int hso_integer_pair(const double *I0, const double *I1, size_t n);

/* Coarse to fine over `levels` levels (1 = hso_flow): at the coarsest level
 * u = v = 0; each finer level starts from u = 2 u_coarse(y/2, x/2) (same for
 * v) and runs `iters` Jacobi iterations of hornSchunck.cpp:56-74 on its own
 * gradients.  u, v: rows x cols (level 0). */
void hso_flow_pyramid(const double *I0, const double *I1, int rows, int cols,
                      int levels, int window, int iters, double alpha, double *u,
                      double *v, int nthreads);

/* plotFlow.cpp:68-88 without namedWindow/imshow.  Draws into `bgr`
 * (rows x cols x 3, dense) in place. */
void hso_plot_bresenham(uint8_t *bgr, int rows, int cols, const double *u,
                        const double *v, int delta, float scale, int outlier);

#ifdef __cplusplus
}
#endif
#endif
