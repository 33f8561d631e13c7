/*
 * hs_oracle.c -- CPU float64 restatement of HornSchunckOF (see hs_oracle.h).
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker and the "port" CPU baseline.
 * Nothing in the product (libhsflow.so, include/, cpp-optical-flow_amd/)
 * links, loads or calls this file.
 *
 * Structure mirrors the reference call by call (one full-array pass per
 * OpenCV primitive, fresh temporaries every Jacobi iteration) so that timing
 * it is a fair stand-in for the reference's CPU path, which cannot be built
 * here (needs OpenCV 4.4.0, absent from the image).
 */
#include "hs_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* OpenCV borderInterpolate(p, len, BORDER_REFLECT_101) for |overshoot| <= len. */
static int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) {
        if (p < 0) p = -p;
        if (p >= len) p = 2 * (len - 1) - p;
    }
    return p;
}

/* main.cpp:13-14 -- cv::cvtColor(src, dst, COLOR_BGR2GRAY) for CV_8UC3.
 * OpenCV 4.x uses 15-bit fixed point with round-half-up (the probe in
 * SURVEY.md §4.3 shows only this variant reproduces the reference plots). */
void hso_bgr_to_gray(const uint8_t *bgr, int rows, int cols, size_t row_stride,
                     uint8_t *gray) {
    for (int r = 0; r < rows; ++r) {
        const uint8_t *p = bgr + (size_t)r * row_stride;
        for (int c = 0; c < cols; ++c) {
            unsigned B = p[3 * c + 0], G = p[3 * c + 1], R = p[3 * c + 2];
            gray[(size_t)r * cols + c] =
                (uint8_t)((9798u * R + 19235u * G + 3735u * B + 16384u) >> 15);
        }
    }
}

/* hornSchunck.cpp:19-41. */
void hso_gradients(const double *I0, const double *I1, int rows, int cols,
                   double *gx, double *gy, double *gt) {
    /* :27  Sobel(prev, gradX, -1, 1, 0, 3): x-derivative [-1 0 1] smoothed by
     *      [1 2 1] over rows; border reflect-101.
     * :28  Sobel(prev, gradY, -1, 0, 1, 3): the transpose. */
    for (int r = 0; r < rows; ++r) {
        int rm = reflect101(r - 1, rows), rp = reflect101(r + 1, rows);
        for (int c = 0; c < cols; ++c) {
            int cm = reflect101(c - 1, cols), cp = reflect101(c + 1, cols);
#define P(y, x) I0[(size_t)(y) * cols + (x)]
            double dx = 1.0 * (P(rm, cp) - P(rm, cm)) + 2.0 * (P(r, cp) - P(r, cm)) +
                        1.0 * (P(rp, cp) - P(rp, cm));
            double dy = 1.0 * (P(rp, cm) - P(rm, cm)) + 2.0 * (P(rp, c) - P(rm, c)) +
                        1.0 * (P(rp, cp) - P(rm, cp));
#undef P
            gx[(size_t)r * cols + c] = dx;
            gy[(size_t)r * cols + c] = dy;
        }
    }
    /* :39  gradT = imageNextNorm - imagePrevNorm */
    size_t n = (size_t)rows * cols;
    for (size_t i = 0; i < n; ++i) gt[i] = I1[i] - I0[i];
}

/* filter2D(src, dst, CV_64F, ones(w,w)/w^2, anchor(a,a), 0, BORDER_CONSTANT)
 * (hornSchunck.cpp:53-54, 60-61).  Correlation; taps summed in kernel
 * row-major order as s += k*src; out-of-image taps read 0. */
static void box_filter(const double *src, double *dst, int rows, int cols, int w,
                       double k, int nthreads) {
    const int a = w - (w / 2) - 1;
    (void)nthreads;
#pragma omp parallel for num_threads(nthreads) if (nthreads > 1) schedule(static)
    for (int y = 0; y < rows; ++y) {
        for (int x = 0; x < cols; ++x) {
            double s = 0.0;
            for (int i = 0; i < w; ++i) {
                int yy = y + i - a;
                if (yy < 0 || yy >= rows) continue; /* k*0 adds nothing */
                const double *row = src + (size_t)yy * cols;
                for (int j = 0; j < w; ++j) {
                    int xx = x + j - a;
                    if (xx < 0 || xx >= cols) continue;
                    s += k * row[xx];
                }
            }
            dst[(size_t)y * cols + x] = s;
        }
    }
}

#define ELEMWISE(expr)                                                              \
    do {                                                                            \
        _Pragma("omp parallel for num_threads(nthreads) if (nthreads > 1) schedule(static)") \
        for (long i = 0; i < (long)n; ++i) { expr; }                                \
    } while (0)

/* hornSchunck.cpp:56-74 from a given (u, v). */
void hso_jacobi(const double *gx, const double *gy, const double *gt, int rows,
                int cols, int window, int iters, double alpha, double *u, double *v,
                int nthreads) {
    const size_t n = (size_t)rows * cols;
    /* :53  kernel = ones(w,w,CV_64FC1) / pow(w,2) */
    const double k = 1.0 / pow((double)window, 2.0);
    const double alpha2 = pow(alpha, 2.0);
    if (nthreads < 1) nthreads = 1;
    for (int it = 0; it < iters; ++it) {
        /* :57  nine fresh cv::Mat per iteration */
        double *uAvg = (double *)malloc(n * sizeof(double));
        double *vAvg = (double *)malloc(n * sizeof(double));
        double *gXuAvg = (double *)malloc(n * sizeof(double));
        double *gYvAvg = (double *)malloc(n * sizeof(double));
        double *gXgX = (double *)malloc(n * sizeof(double));
        double *gYgY = (double *)malloc(n * sizeof(double));
        double *num = (double *)malloc(n * sizeof(double));
        double *den = (double *)malloc(n * sizeof(double));
        double *upd = (double *)malloc(n * sizeof(double));
        double *uUpd = (double *)malloc(n * sizeof(double));
        double *vUpd = (double *)malloc(n * sizeof(double));
        /* :60-61 */
        box_filter(u, uAvg, rows, cols, window, k, nthreads);
        box_filter(v, vAvg, rows, cols, window, k, nthreads);
        /* :63-66 */
        ELEMWISE(gXuAvg[i] = gx[i] * uAvg[i]);
        ELEMWISE(gYvAvg[i] = gy[i] * vAvg[i]);
        ELEMWISE(gXgX[i] = gx[i] * gx[i]);
        ELEMWISE(gYgY[i] = gy[i] * gy[i]);
        /* :68  MatExpr temporaries (A + B) + C and (s + D) + E, then divide */
        ELEMWISE(num[i] = gXuAvg[i] + gYvAvg[i]);
        ELEMWISE(num[i] = num[i] + gt[i]);
        ELEMWISE(den[i] = alpha2 + gXgX[i]);
        ELEMWISE(den[i] = den[i] + gYgY[i]);
        ELEMWISE(upd[i] = num[i] / den[i]);
        /* :69-70 */
        ELEMWISE(uUpd[i] = gx[i] * upd[i]);
        ELEMWISE(vUpd[i] = gy[i] * upd[i]);
        /* :72-73 */
        ELEMWISE(u[i] = uAvg[i] - uUpd[i]);
        ELEMWISE(v[i] = vAvg[i] - vUpd[i]);
        free(uAvg); free(vAvg); free(gXuAvg); free(gYvAvg); free(gXgX);
        free(gYgY); free(num); free(den); free(upd); free(uUpd); free(vUpd);
    }
}

/* hornSchunck.cpp:43-75. */
void hso_flow(const double *I0, const double *I1, int rows, int cols, int window,
              int iters, double alpha, double *u, double *v, int nthreads) {
    const size_t n = (size_t)rows * cols;
    double *gx = (double *)malloc(n * sizeof(double));
    double *gy = (double *)malloc(n * sizeof(double));
    double *gt = (double *)malloc(n * sizeof(double));
    hso_gradients(I0, I1, rows, cols, gx, gy, gt); /* :46 */
    memset(u, 0, n * sizeof(double));              /* :49 */
    memset(v, 0, n * sizeof(double));              /* :50 */
    hso_jacobi(gx, gy, gt, rows, cols, window, iters, alpha, u, v, nthreads);
    free(gx); free(gy); free(gt);
}

/* ---- config 5 pyramid (see hs_oracle.h) ------------------------------- */
static const double kPyrW[5] = {2.0, 5.0, 4.0, 5.0, 2.0}; /* a = 0.4, x 9 / 0.5 */

void hso_pyrdown(const double *src, int rows, int cols, int round_int, double *dst) {
    const int r2 = (rows + 1) / 2, c2 = (cols + 1) / 2;
    for (int y = 0; y < r2; ++y)
        for (int x = 0; x < c2; ++x) {
            /* MultiResolution.cpp:80-87: ym = 2y + m - 2, xn = 2x + n - 2 */
            double S = 0.0;
            for (int m = 0; m < 5; ++m) {
                const double *row = src + (size_t)reflect101(2 * y + m - 2, rows) * cols;
                double h = 0.0;
                for (int n = 0; n < 5; ++n) h += kPyrW[n] * row[reflect101(2 * x + n - 2, cols)];
                S += kPyrW[m] * h;
            }
            dst[(size_t)y * c2 + x] = round_int ? floor((S + 162.0) / 324.0) : S / 324.0;
        }
}

int hso_integer_pair(const double *I0, const double *I1, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        const double a = I0[i], b = I1[i];
        if (a != floor(a) || b != floor(b) || a < 0 || a > 255 || b < 0 || b > 255)
            return 0;
    }
    return 1;
}

void hso_flow_pyramid(const double *I0, const double *I1, int rows, int cols,
                      int levels, int window, int iters, double alpha, double *u,
                      double *v, int nthreads) {
    if (levels < 1) levels = 1;
    if (levels > 16) levels = 16;
    const int rnd = hso_integer_pair(I0, I1, (size_t)rows * cols);
    int R[16], C[16];
    double *P0[16], *P1[16], *U[16], *V[16];
    R[0] = rows; C[0] = cols;
    P0[0] = (double *)I0; P1[0] = (double *)I1;
    for (int l = 1; l < levels; ++l) {
        R[l] = (R[l - 1] + 1) / 2;
        C[l] = (C[l - 1] + 1) / 2;
        P0[l] = (double *)malloc((size_t)R[l] * C[l] * sizeof(double));
        P1[l] = (double *)malloc((size_t)R[l] * C[l] * sizeof(double));
        hso_pyrdown(P0[l - 1], R[l - 1], C[l - 1], rnd, P0[l]);
        hso_pyrdown(P1[l - 1], R[l - 1], C[l - 1], rnd, P1[l]);
    }
    for (int l = levels - 1; l >= 0; --l) {
        const size_t n = (size_t)R[l] * C[l];
        U[l] = l ? (double *)malloc(n * sizeof(double)) : u;
        V[l] = l ? (double *)malloc(n * sizeof(double)) : v;
        if (l == levels - 1) {
            memset(U[l], 0, n * sizeof(double));
            memset(V[l], 0, n * sizeof(double));
        } else { /* OpticalFlow.cpp:205-206 */
            for (int y = 0; y < R[l]; ++y)
                for (int x = 0; x < C[l]; ++x) {
                    const size_t c = (size_t)(y / 2) * C[l + 1] + x / 2;
                    U[l][(size_t)y * C[l] + x] = 2.0 * U[l + 1][c];
                    V[l][(size_t)y * C[l] + x] = 2.0 * V[l + 1][c];
                }
            free(U[l + 1]);
            free(V[l + 1]);
        }
        double *gx = (double *)malloc(n * sizeof(double));
        double *gy = (double *)malloc(n * sizeof(double));
        double *gt = (double *)malloc(n * sizeof(double));
        hso_gradients(P0[l], P1[l], R[l], C[l], gx, gy, gt);
        hso_jacobi(gx, gy, gt, R[l], C[l], window, iters, alpha, U[l], V[l], nthreads);
        free(gx); free(gy); free(gt);
    }
    for (int l = 1; l < levels; ++l) {
        free(P0[l]);
        free(P1[l]);
    }
}

/* ---- plotFlow.cpp, headless ------------------------------------------- */

static int sgn(int x) { return x < 0 ? -1 : (x > 0 ? 1 : 0); } /* :24-28 */

/* plotFlow.cpp:24-32  note: writes [0]=r,[1]=g,[2]=b into BGR memory, and only when
 * 0 <= x < rows-1 and 0 <= y < cols-1 (the reference's off-by-one kept). */
static void set_pixel(uint8_t *img, int rows, int cols, int x, int y, int r, int g,
                      int b) {
    if ((x < rows - 1) & (x >= 0)) {
        if ((y < cols - 1) & (y >= 0)) {
            uint8_t *p = img + ((size_t)x * cols + y) * 3;
            p[0] = (uint8_t)r;
            p[1] = (uint8_t)g;
            p[2] = (uint8_t)b;
        }
    }
}

/* plotFlow.cpp:34-41 */
static void move_lateral(int *x, int *y, double *R, int sx, int sy, int dx, int dy) {
    *x += sx;
    *R += dy;
    if (*R >= dx) {
        *y += sy;
        *R -= dx;
    }
}

/* plotFlow.cpp:43-66 */
static void bresenham(uint8_t *img, int rows, int cols, int x0, int y0, int x1,
                      int y1, int r, int g, int b) {
    int dX = x1 - x0, dY = y1 - y0;
    int sX = sgn(dX), sY = sgn(dY);
    dX = abs(dX);
    dY = abs(dY);
    int dist = dX > dY ? dX : dY;
    double R = dist / 2; /* integer division, then widened */
    int x = x0, y = y0;
    if (dX > dY) {
        for (int i = 0; i < dist; ++i) {
            set_pixel(img, rows, cols, x, y, r, g, b);
            move_lateral(&x, &y, &R, sX, sY, dX, dY);
        }
    } else {
        for (int i = 0; i < dist; ++i) {
            set_pixel(img, rows, cols, x, y, r, g, b);
            move_lateral(&y, &x, &R, sY, sX, dY, dX);
        }
    }
}

/* plotFlow.cpp:68-88 (namedWindow/imshow/imwrite left to the caller). */
void hso_plot_bresenham(uint8_t *bgr, int rows, int cols, const double *u,
                        const double *v, int delta, float scale, int outlier) {
    for (int x1 = 0; x1 < rows; x1 += delta) {
        for (int y1 = 0; y1 < cols; y1 += delta) {
            double uu = u[(size_t)x1 * cols + y1], vv = v[(size_t)x1 * cols + y1];
            int x2 = (int)(x1 + (uu * scale)); /* u is added to the ROW index */
            int y2 = (int)(y1 + (vv * scale));
            if (outlier > 0) {
                if ((uu < outlier) & (vv < outlier) & (uu > -1 * outlier) &
                    (vv > -1 * outlier))
                    bresenham(bgr, rows, cols, x1, y1, x2, y2, 0, 255, 0);
            } else {
                bresenham(bgr, rows, cols, x1, y1, x2, y2, 0, 255, 0);
            }
            set_pixel(bgr, rows, cols, x2, y2, 0, 0, 255);
        }
    }
}
