// TEST DOUBLE -- not OpenCV.  OpenCV is absent from this image, so this
// header implements only the cv::Mat surface that include/hornSchunck.hpp
// (our cv::Mat adapter) touches, with OpenCV 4.x's type codes and error
// conventions, to compile and run the adapter in tests/test_cv_adapter.py.
// It is never used to build anything from the reference.
#pragma once
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#define CV_8U 0
#define CV_8S 1
#define CV_16U 2
#define CV_16S 3
#define CV_32S 4
#define CV_32F 5
#define CV_64F 6
#define CV_16F 7
#define CV_MAKETYPE(depth, cn) ((depth) + (((cn)-1) << 3))
#define CV_8UC1 CV_MAKETYPE(CV_8U, 1)
#define CV_8UC3 CV_MAKETYPE(CV_8U, 3)
#define CV_16UC1 CV_MAKETYPE(CV_16U, 1)
#define CV_16FC1 CV_MAKETYPE(CV_16F, 1)
#define CV_32FC1 CV_MAKETYPE(CV_32F, 1)
#define CV_64FC1 CV_MAKETYPE(CV_64F, 1)

namespace cv {
namespace Error {
enum { StsError = -2, StsInternal = -3, StsBadArg = -5, StsUnsupportedFormat = -210 };
}
struct Exception : std::runtime_error {
    int code;
    Exception(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

inline size_t elem_size1(int depth) {
    static const size_t s[8] = {1, 1, 2, 2, 4, 4, 8, 2};
    return s[depth & 7];
}

class Mat {
  public:
    int rows = 0, cols = 0;
    size_t step = 0;
    unsigned char *data = nullptr;

    Mat() = default;
    Mat(int r, int c, int type) { create(r, c, type); }
    Mat(int r, int c, int type, void *ext, size_t st)  // external data, like cv::Mat
        : rows(r), cols(c), step(st), data((unsigned char *)ext), type_(type) {}
    int type() const { return type_; }
    int depth() const { return type_ & 7; }
    int channels() const { return (type_ >> 3) + 1; }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    void create(int r, int c, int type) {
        if (buf_ && r == rows && c == cols && type == type_) return;
        rows = r;
        cols = c;
        type_ = type;
        step = (size_t)c * channels() * elem_size1(depth());
        buf_ = std::make_shared<std::vector<unsigned char>>((size_t)r * step);
        data = buf_->data();
    }
    // the adapter converts single-channel integer depths to CV_64FC1
    void convertTo(Mat &dst, int rtype) const {
        if (rtype != CV_64FC1 || channels() != 1) throw Exception(Error::StsError, "stub");
        dst.create(rows, cols, CV_64FC1);
        for (int r = 0; r < rows; ++r) {
            const unsigned char *s = data + (size_t)r * step;
            double *d = (double *)(dst.data + (size_t)r * dst.step);
            for (int c = 0; c < cols; ++c) switch (depth()) {
                case CV_8S: d[c] = ((const int8_t *)s)[c]; break;
                case CV_16U: d[c] = ((const uint16_t *)s)[c]; break;
                case CV_16S: d[c] = ((const int16_t *)s)[c]; break;
                case CV_32S: d[c] = ((const int32_t *)s)[c]; break;
                default: throw Exception(Error::StsError, "stub: depth");
                }
        }
    }
    template <typename T> T &at(int r, int c) { return ((T *)(data + (size_t)r * step))[c]; }

  private:
    int type_ = 0;
    std::shared_ptr<std::vector<unsigned char>> buf_;
};
}  // namespace cv

#define CV_Error(code, msg) throw cv::Exception((code), (msg))
