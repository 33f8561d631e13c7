// The reference's main.cpp:97-98 call sequence through include/hornSchunck.hpp
// (the cv::Mat drop-in), on synthetic u8 frames in several cv::Mat forms.
// Writes u, v of each case as raw float64 to <out>_<case>.bin; tests compare
// them with the Python host API.  Exit code 0, or 10 + case on a wrong error.
#include <cstdio>
#include <vector>

#include "hornSchunck.hpp"

static void dump(const char *out, const char *tag, const cv::Mat &u, const cv::Mat &v) {
    char path[512];
    std::snprintf(path, sizeof path, "%s_%s.bin", out, tag);
    FILE *f = std::fopen(path, "wb");
    for (int r = 0; r < u.rows; ++r) std::fwrite(u.data + r * u.step, 8, u.cols, f);
    for (int r = 0; r < v.rows; ++r) std::fwrite(v.data + r * v.step, 8, v.cols, f);
    std::fclose(f);
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const int rows = 90, cols = 130;
    std::vector<uint8_t> a(rows * cols), b(rows * cols);
    hsflow_synth_pair(1000, rows, cols, -3, 6, nullptr, nullptr, a.data(), b.data());
    cv::Mat prev(rows, cols, CV_8UC1, a.data(), cols), next(rows, cols, CV_8UC1, b.data(), cols);

    cv::Mat u, v;
    hornSchunck hs = hornSchunck(5, 100, 1);           // main.cpp:97
    hs.getFlow(prev, next, u, v);                       // main.cpp:98
    if (u.type() != CV_64FC1 || u.rows != rows || u.cols != cols) return 10;
    dump(argv[1], "u8", u, v);

    // ROI of a wider frame (non-continuous rows)
    std::vector<uint8_t> wa(rows * (cols + 9)), wb(rows * (cols + 9));
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < cols; ++c) {
            wa[r * (cols + 9) + c] = a[r * cols + c];
            wb[r * (cols + 9) + c] = b[r * cols + c];
        }
    cv::Mat rp(rows, cols, CV_8UC1, wa.data(), cols + 9), rn(rows, cols, CV_8UC1, wb.data(), cols + 9);
    hs.getFlow(rp, rn, u, v);
    dump(argv[1], "roi", u, v);

    // ROI prev with a contiguous next: each frame keeps its own row step
    hs.getFlow(rp, next, u, v);
    dump(argv[1], "roi_mixed", u, v);

    // frames of different depths (u8 prev, CV_32FC1 next), each converted
    // on its own as hornSchunck.cpp:23-24 does
    cv::Mat n32(rows, cols, CV_32FC1);
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < cols; ++c) n32.at<float>(r, c) = b[r * cols + c];
    hs.getFlow(prev, n32, u, v);
    dump(argv[1], "mixed_depth", u, v);

    // Output aliasing: u = Mat::zeros(...) and u = uAvg - uUpdateConst
    // (hornSchunck.cpp:49-50, 72) are MatExpr assignments, which OpenCV
    // evaluates into the destination with create() -- an existing CV_64FC1
    // buffer of the right size is written in place, so a header sharing it
    // sees the result.  The adapter keeps that behaviour.
    cv::Mat alias = u;
    hs.getFlow(prev, next, u, v);
    if (alias.data != u.data) return 11;
    dump(argv[1], "alias", alias, v);

    // CV_16UC1 frames: converted with convertTo(CV_64FC1) (hornSchunck.cpp:23-24)
    cv::Mat p16(rows, cols, CV_16UC1), n16(rows, cols, CV_16UC1);
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < cols; ++c) {
            p16.at<uint16_t>(r, c) = a[r * cols + c];
            n16.at<uint16_t>(r, c) = b[r * cols + c];
        }
    hs.getFlow(p16, n16, u, v);
    dump(argv[1], "u16", u, v);

    // public fields edited between calls are honoured (hornSchunck.cpp:10-11)
    hs.maxIterations = 7;
    hs.windowSize = 3;
    hs.getFlow(prev, next, u, v);
    dump(argv[1], "w3n7", u, v);

    cv::Mat gx, gy, gt;
    hs.getGradients(prev, next, gx, gy, gt);
    dump(argv[1], "grad_xy", gx, gy);

    // errors surface as cv::Exception, as from inside OpenCV
    int caught = 0;
    try {
        cv::Mat small(rows - 1, cols, CV_8UC1, a.data(), cols);
        hs.getFlow(prev, small, u, v);
    } catch (const cv::Exception &) { caught |= 1; }
    try {
        std::vector<uint8_t> c3(rows * cols * 3);
        cv::Mat bgr(rows, cols, CV_8UC3, c3.data(), cols * 3);
        hs.getFlow(bgr, bgr, u, v);
    } catch (const cv::Exception &) { caught |= 2; }
    try {
        hs.getFlow(cv::Mat(), cv::Mat(), u, v);
    } catch (const cv::Exception &) { caught |= 4; }
    if (caught != 7) return 20 + caught;
    std::printf("ok\n");
    return 0;
}
