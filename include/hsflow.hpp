// hsflow.hpp -- header-only C++ host layer over the C ABI (hsflow.h),
// OpenCV-free.  Mirrors the reference's operator class
// HornSchunckOF/hornSchunck.cpp:8-76 on plain image views:
//
//   hsflow::HornSchunck hs(windowSize, maxIterations, alpha);   // :13-17
//   hs.getGradients(prev, next, gx, gy, gt);                      // :19-41
//   hs.getFlow(prev, next, u, v);                                  // :43-75
//
// Same public fields, same argument meaning, outputs float64 row-major
// (what CV_64FC1 holds).  Errors throw hsflow::Error (the reference throws
// cv::Exception from inside OpenCV).  Copies share one device context, so a
// copy-initialised object (main.cpp:97) reuses the cached device buffers.
// Link: -lhsflow (cpp-optical-flow_amd/libhsflow.so).
#pragma once

#include <cmath>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "hsflow.h"

namespace hsflow {

class Error : public std::runtime_error {
  public:
    Error(int status, const std::string &msg)
        : std::runtime_error("hsflow: " + msg + " (" + hsflow_status_string(status) + ")"),
          status_(status) {}
    int status() const { return status_; }

  private:
    int status_;
};

// One single-channel image: U8 (CV_8UC1), F32 (CV_32FC1) or F64 (CV_64FC1);
// `step` = bytes between rows (cv::Mat::step), so ROIs need no copy.
struct ImageView {
    const void *data = nullptr;
    int rows = 0, cols = 0;
    size_t step = 0;
    int type = HSFLOW_U8;
};

inline ImageView view(const uint8_t *p, int rows, int cols, size_t step = 0) {
    return {p, rows, cols, step ? step : (size_t)cols, HSFLOW_U8};
}
inline ImageView view(const float *p, int rows, int cols, size_t step = 0) {
    return {p, rows, cols, step ? step : (size_t)cols * 4, HSFLOW_F32};
}
inline ImageView view(const double *p, int rows, int cols, size_t step = 0) {
    return {p, rows, cols, step ? step : (size_t)cols * 8, HSFLOW_F64};
}

// RAII device context (device, stream, cached buffers).
class Context {
  public:
    explicit Context(int device = 0) {
        int rc = hsflow_create(&ctx_, device);
        if (rc != HSFLOW_OK) throw Error(rc, hsflow_last_error(nullptr));
    }
    ~Context() { hsflow_destroy(ctx_); }
    Context(const Context &) = delete;
    Context &operator=(const Context &) = delete;
    hsflow_ctx *get() const { return ctx_; }
    void check(int rc) const {
        if (rc != HSFLOW_OK) throw Error(rc, hsflow_last_error(ctx_));
    }

  private:
    hsflow_ctx *ctx_ = nullptr;
};

class HornSchunck {
  public:
    // hornSchunck.cpp:10-11 -- public, same names
    int windowSize, maxIterations;
    double alpha;

    // hornSchunck.cpp:13-17
    HornSchunck(int inpWindowSize, int inpMaxIterations, double inpAlpha, int device = 0)
        : windowSize(inpWindowSize), maxIterations(inpMaxIterations), alpha(inpAlpha),
          device_(device) {}

    // hornSchunck.cpp:19-41 -> Ix, Iy, It as rows*cols float64
    void getGradients(const ImageView &imagePrev, const ImageView &imageNext,
                      std::vector<double> &gradX, std::vector<double> &gradY,
                      std::vector<double> &gradT) {
        check_pair(imagePrev, imageNext);
        const size_t n = (size_t)imagePrev.rows * imagePrev.cols;
        gradX.resize(n);
        gradY.resize(n);
        gradT.resize(n);
        getGradientsInto(imagePrev, imageNext, gradX.data(), gradY.data(), gradT.data(),
                         HSFLOW_F64, (size_t)imagePrev.cols * 8);
    }

    // hornSchunck.cpp:43-75 -> u, v as rows*cols float64 (reallocated, like
    // the reference's u = cv::Mat::zeros(...) at :49-50)
    void getFlow(const ImageView &imagePrev, const ImageView &imageNext,
                 std::vector<double> &u, std::vector<double> &v) {
        check_pair(imagePrev, imageNext);
        const size_t n = (size_t)imagePrev.rows * imagePrev.cols;
        u.resize(n);
        v.resize(n);
        getFlowInto(imagePrev, imageNext, u.data(), v.data(), HSFLOW_F64,
                    (size_t)imagePrev.cols * 8);
    }

    // Raw form for callers that own output rows (cv::Mat adapter): dtype_out
    // HSFLOW_F64 or HSFLOW_F32, out_step in bytes.  Each frame keeps its own
    // row step; frames of different element types are both widened to
    // float64 first, as hornSchunck.cpp:23-24 converts each with convertTo.
    void getFlowInto(const ImageView &imagePrev, const ImageView &imageNext, void *u,
                     void *v, int dtype_out, size_t out_step) {
        check_pair(imagePrev, imageNext);
        std::vector<double> ha, hb;
        const ImageView a = common_type(imagePrev, imageNext, ha);
        const ImageView b = common_type(imageNext, imagePrev, hb);
        Context &c = ctx();
        c.check(hsflow_flow(c.get(), a.data, b.data, a.type, a.rows, a.cols, a.step, b.step,
                            windowSize, maxIterations, alpha, u, v, dtype_out, out_step));
    }
    void getGradientsInto(const ImageView &imagePrev, const ImageView &imageNext, void *gx,
                          void *gy, void *gt, int dtype_out, size_t out_step) {
        check_pair(imagePrev, imageNext);
        std::vector<double> ha, hb;
        const ImageView a = common_type(imagePrev, imageNext, ha);
        const ImageView b = common_type(imageNext, imagePrev, hb);
        Context &c = ctx();
        c.check(hsflow_gradients(c.get(), a.data, b.data, a.type, a.rows, a.cols, a.step,
                                 b.step, gx, gy, gt, dtype_out, out_step));
    }

  private:
    int device_;
    std::shared_ptr<Context> ctx_;

    Context &ctx() {
        if (!ctx_) ctx_ = std::make_shared<Context>(device_);
        return *ctx_;
    }
    static void check_pair(const ImageView &a, const ImageView &b) {
        if (!a.data || !b.data) throw Error(HSFLOW_ERR_ARG, "empty image");
        if (a.rows != b.rows || a.cols != b.cols)
            throw Error(HSFLOW_ERR_SIZE, "Image sizes are different");
    }
    static double half_to_double(uint16_t h) {  // IEEE binary16 (CV_16F)
        const int e = (h >> 10) & 31, f = h & 1023;
        const double s = (h & 0x8000) ? -1.0 : 1.0;
        if (e == 0) return s * std::ldexp((double)f, -24);
        if (e == 31) return f ? std::nan("") : s * HUGE_VAL;
        return s * std::ldexp((double)(f | 1024), e - 25);
    }
    // `m` as it enters the ABI: unchanged when both frames share an element
    // type, else widened to a dense float64 copy held in `hold`.
    static ImageView common_type(const ImageView &m, const ImageView &other,
                                 std::vector<double> &hold) {
        if (m.type == other.type) return m;
        hold.resize((size_t)m.rows * m.cols);
        for (int r = 0; r < m.rows; ++r) {
            const char *row = (const char *)m.data + (size_t)r * m.step;
            double *d = hold.data() + (size_t)r * m.cols;
            for (int c = 0; c < m.cols; ++c) {
                switch (m.type) {
                case HSFLOW_U8: d[c] = ((const uint8_t *)row)[c]; break;
                case HSFLOW_F32: d[c] = ((const float *)row)[c]; break;
                case HSFLOW_F64: d[c] = ((const double *)row)[c]; break;
                case HSFLOW_F16: d[c] = half_to_double(((const uint16_t *)row)[c]); break;
                default: throw Error(HSFLOW_ERR_ARG, "unsupported element type");
                }
            }
        }
        return {hold.data(), m.rows, m.cols, (size_t)m.cols * 8, HSFLOW_F64};
    }
};

// compute(I0, I1, alpha, nIter) -> (u, v): the north-star convenience form.
inline void compute(const ImageView &I0, const ImageView &I1, double alpha, int nIter,
                    std::vector<double> &u, std::vector<double> &v, int windowSize = 5) {
    HornSchunck(windowSize, nIter, alpha).getFlow(I0, I1, u, v);
}

// Frame-parallel getFlow over several GPUs from one process
// (hsflow_flow_multi): pair j (prev[j], next[j], all one size, type and row
// steps) on devices[j % devices.size()]; u[j], v[j] receive CV_64FC1-style
// rows x cols doubles (resized here).
inline void flowMulti(const std::vector<int> &devices, const std::vector<ImageView> &prev,
                      const std::vector<ImageView> &next, int windowSize, int maxIterations,
                      double alpha, std::vector<std::vector<double>> &u,
                      std::vector<std::vector<double>> &v) {
    if (prev.size() != next.size()) throw Error(HSFLOW_ERR_ARG, "prev/next counts differ");
    const size_t n = prev.size();
    u.resize(n);
    v.resize(n);
    if (n == 0) return;
    const ImageView &a = prev[0], &b = next[0];
    std::vector<const void *> I0(n), I1(n);
    std::vector<void *> pu(n), pv(n);
    for (size_t j = 0; j < n; ++j) {
        if (prev[j].rows != a.rows || prev[j].cols != a.cols || prev[j].type != a.type ||
            prev[j].step != a.step || next[j].rows != a.rows || next[j].cols != a.cols ||
            next[j].type != a.type || next[j].step != b.step)
            throw Error(HSFLOW_ERR_SIZE, "pairs differ in size, type or row step");
        I0[j] = prev[j].data;
        I1[j] = next[j].data;
        u[j].assign((size_t)a.rows * a.cols, 0.0);
        v[j].assign((size_t)a.rows * a.cols, 0.0);
        pu[j] = u[j].data();
        pv[j] = v[j].data();
    }
    const int rc = hsflow_flow_multi(devices.data(), (int)devices.size(), (int)n, I0.data(),
                                     I1.data(), a.type, a.rows, a.cols, a.step, b.step,
                                     windowSize, maxIterations, alpha, pu.data(), pv.data(),
                                     HSFLOW_F64, (size_t)a.cols * sizeof(double));
    if (rc != HSFLOW_OK) throw Error(rc, hsflow_last_error(nullptr));
}

}  // namespace hsflow
