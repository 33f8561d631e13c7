// hornSchunck.hpp -- drop-in replacement for HornSchunckOF/hornSchunck.cpp.
//
// The reference's main.cpp does `#include "hornSchunck.cpp"` (main.cpp:8)
// and then
//     hornSchunck hs = hornSchunck(windowSize, maxIterations, alpha); // :97
//     hs.getFlow(imagePrev, imageNext, u, v);                         // :98
// Replace that include with `#include "hornSchunck.hpp"` and link
// -lhsflow: the class below has the reference's exact public surface
// (hornSchunck.cpp:8-17 fields and ctor, :19 getGradients, :43 getFlow),
// takes cv::Mat by value, honours ROI steps, and returns CV_64FC1 u, v
// (plotFlow.cpp:72-75 reads them with at<double>).  The numerics run on the
// MI355X through libhsflow.so; errors surface as cv::Exception (CV_Error),
// as they would from inside OpenCV.
//
// Compiled only where OpenCV is available (the reference's own dependency);
// the OpenCV-free layer it wraps is hsflow.hpp.
#pragma once

#if __has_include(<opencv2/core.hpp>)
#include <opencv2/core.hpp>

#include "hsflow.hpp"

class hornSchunck {
  public:
    int windowSize, maxIterations;
    double alpha;

    hornSchunck(int inpWindowSize, int inpMaxIterations, double inpAlpha)
        : windowSize(inpWindowSize), maxIterations(inpMaxIterations), alpha(inpAlpha),
          impl_(inpWindowSize, inpMaxIterations, inpAlpha) {}

    void getGradients(cv::Mat imagePrev, cv::Mat imageNext, cv::Mat &gradX, cv::Mat &gradY,
                      cv::Mat &gradT) {
        cv::Mat ha, hb;  // converted copies for depths the ABI does not take
        const hsflow::ImageView a = as_view(imagePrev, ha), b = as_view(imageNext, hb);
        gradX.create(imagePrev.rows, imagePrev.cols, CV_64FC1);
        gradY.create(imagePrev.rows, imagePrev.cols, CV_64FC1);
        gradT.create(imagePrev.rows, imagePrev.cols, CV_64FC1);
        if (gradX.step != gradY.step || gradX.step != gradT.step)
            CV_Error(cv::Error::StsInternal, "gradient steps differ");
        try {
            impl_.getGradientsInto(a, b, gradX.data, gradY.data, gradT.data, HSFLOW_F64,
                                   gradX.step);
        } catch (const hsflow::Error &e) {
            CV_Error(cv::Error::StsError, e.what());
        }
    }

    void getFlow(cv::Mat imagePrev, cv::Mat imageNext, cv::Mat &u, cv::Mat &v) {
        sync_params();
        cv::Mat ha, hb;
        const hsflow::ImageView a = as_view(imagePrev, ha), b = as_view(imageNext, hb);
        // hornSchunck.cpp:49-50 and :72-73 assign MatExprs (Mat::zeros, then
        // uAvg - uUpdateConst) to u, v; OpenCV evaluates a MatExpr into the
        // destination through create(), so an existing CV_64FC1 buffer of the
        // right size is written in place (headers sharing it see the result)
        // and anything else is reallocated.  create() here does the same.
        u.create(imagePrev.rows, imagePrev.cols, CV_64FC1);
        v.create(imagePrev.rows, imagePrev.cols, CV_64FC1);
        if (u.step != v.step) CV_Error(cv::Error::StsInternal, "u/v steps differ");
        try {
            impl_.getFlowInto(a, b, u.data, v.data, HSFLOW_F64, u.step);
        } catch (const hsflow::Error &e) {
            CV_Error(cv::Error::StsError, e.what());
        }
    }

  private:
    hsflow::HornSchunck impl_;

    void sync_params() {  // the public fields may be edited between calls
        impl_.windowSize = windowSize;
        impl_.maxIterations = maxIterations;
        impl_.alpha = alpha;
    }
    // A view of m for the C ABI; depths the ABI does not take are converted
    // into `holder` first, exactly as hornSchunck.cpp:23-24 converts every
    // input with convertTo(CV_64FC1).
    static hsflow::ImageView as_view(const cv::Mat &m, cv::Mat &holder) {
        if (m.empty()) CV_Error(cv::Error::StsBadArg, "empty image");
        if (m.channels() != 1)
            CV_Error(cv::Error::StsBadArg, "hornSchunck expects single-channel images "
                                           "(main.cpp:11-26 converts BGR to gray first)");
        const cv::Mat *src = &m;
        int type;
        switch (m.depth()) {
        case CV_8U: type = HSFLOW_U8; break;
        case CV_16F: type = HSFLOW_F16; break;
        case CV_32F: type = HSFLOW_F32; break;
        case CV_64F: type = HSFLOW_F64; break;
        default:  // CV_8S, CV_16U, CV_16S, CV_32S
            m.convertTo(holder, CV_64FC1);
            src = &holder;
            type = HSFLOW_F64;
        }
        hsflow::ImageView v;
        v.data = src->data;
        v.rows = src->rows;
        v.cols = src->cols;
        v.step = src->step;
        v.type = type;
        return v;
    }
};

#endif  // __has_include(<opencv2/core.hpp>)
