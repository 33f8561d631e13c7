// hs_main.cpp -- the reference's HornSchunckOF/main.cpp driver flow on the
// MI355X solver, without OpenCV (PGM/PPM in, YAML + PPM out).
//
//   hs_main <prev.{pgm,ppm}> <next.{pgm,ppm}> <savePath> [windowSize maxIterations alpha]
//   hs_main <video.y4m> <prevFrame> <nextFrame> <savePath> [windowSize maxIterations alpha]
//
// main.cpp:53-59   the video branch (VideoCapture + CAP_PROP_POS_FRAMES seek)
//                  over YUV4MPEG2, the decoder-free raw container; gray =
//                  luma, video range expanded to 0..255 (frames.Y4MVideo)
// main.cpp:50-51   read the two frames (PPM = 8-bit RGB, PGM = 8-bit gray)
// main.cpp:65-73   empty / size-mismatch checks -> return -1
// main.cpp:84      preprocess: BGR -> gray, OpenCV 4.x 15-bit (hsflow_bgr_to_gray)
// main.cpp:94-98   hornSchunck(5, 100, 1).getFlow(prev, next, u, v)
// main.cpp:99-102  <savePath>uMatrixHS.txt / vMatrixHS.txt in cv::FileStorage
//                  YAML layout ("u matrix" / "v matrix", !!opencv-matrix, dt: d)
// main.cpp:103-104 plotFlow(prev raw).plotBresenhamLine(u, v, 20, 20, 5) ->
//                  <savePath>hsbresenhamLineFlow.ppm (headless: no imshow)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "../include/hsflow.hpp"

namespace {

struct Image {
    int rows = 0, cols = 0, channels = 0;  // channels 1 (gray) or 3 (BGR)
    std::vector<uint8_t> px;
};

bool read_pnm(const std::string &path, Image &im) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::string magic;
    f >> magic;
    if (magic != "P5" && magic != "P6") return false;
    auto next_int = [&](int &x) {
        f >> std::ws;
        while (f.peek() == '#') {
            std::string line;
            std::getline(f, line);
            f >> std::ws;
        }
        f >> x;
    };
    int w, h, mx;
    next_int(w);
    next_int(h);
    next_int(mx);
    f.get();
    if (mx != 255 || w <= 0 || h <= 0) return false;
    im.rows = h;
    im.cols = w;
    im.channels = magic == "P5" ? 1 : 3;
    im.px.resize((size_t)w * h * im.channels);
    f.read((char *)im.px.data(), (std::streamsize)im.px.size());
    if (!f) return false;
    if (im.channels == 3)  // PPM stores RGB; imread gives BGR
        for (size_t i = 0; i < im.px.size(); i += 3) std::swap(im.px[i], im.px[i + 2]);
    return true;
}

// YUV4MPEG2 frame `index` as gray (see frames.py Y4MVideo for the rule)
bool read_y4m_frame(const std::string &path, long index, Image &im) {
    std::ifstream f(path, std::ios::binary);
    if (!f || index < 0) return false;
    std::string head;
    std::getline(f, head);
    if (head.rfind("YUV4MPEG2", 0) != 0) return false;
    std::istringstream hs(head);
    std::string tok, cs = "420jpeg";
    int w = 0, h = 0;
    bool full = false;
    while (hs >> tok) {
        if (tok[0] == 'W') w = std::atoi(tok.c_str() + 1);
        else if (tok[0] == 'H') h = std::atoi(tok.c_str() + 1);
        else if (tok[0] == 'C') cs = tok.substr(1);
        else if (tok == "XCOLORRANGE=FULL") full = true;
    }
    if (w <= 0 || h <= 0) return false;
    size_t chroma = 0;
    if (cs.rfind("mono", 0) != 0) {
        int sx = 2, sy = 2;
        if (cs.rfind("444", 0) == 0) sx = sy = 1;
        else if (cs.rfind("422", 0) == 0) sy = 1;
        else if (cs.rfind("411", 0) == 0) { sx = 4; sy = 1; }
        chroma = 2 * (size_t)((w + sx - 1) / sx) * (size_t)((h + sy - 1) / sy);
    }
    const size_t luma = (size_t)w * h;
    for (long i = 0;; ++i) {  // frame headers may carry parameters: walk them
        std::string fh;
        if (!std::getline(f, fh) || fh.rfind("FRAME", 0) != 0) return false;
        if (i == index) break;
        f.seekg((std::streamoff)(luma + chroma), std::ios::cur);
    }
    im.rows = h;
    im.cols = w;
    im.channels = 1;
    im.px.resize(luma);
    f.read((char *)im.px.data(), (std::streamsize)luma);
    if (!f) return false;
    if (!full)
        for (auto &y : im.px) {
            const int g = ((int)y - 16) * 255 + 109;
            const int q = g >= 0 ? g / 219 : -((-g + 218) / 219);
            y = (uint8_t)std::min(255, std::max(0, q));
        }
    return true;
}

bool ends_with(const std::string &s, const char *suf) {
    const size_t n = std::strlen(suf);
    return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

bool write_ppm_bgr(const std::string &path, const Image &im) {
    std::ofstream f(path, std::ios::binary);
    if (!f) return false;
    f << "P6\n" << im.cols << " " << im.rows << "\n255\n";
    std::vector<uint8_t> rgb(im.px);
    for (size_t i = 0; i < rgb.size(); i += 3) std::swap(rgb[i], rgb[i + 2]);
    f.write((const char *)rgb.data(), (std::streamsize)rgb.size());
    return (bool)f;
}

// cv::FileStorage text form of a double (OpenCV 4.x persistence: integral
// values print as "%d.", others "%.16e"; NaN/Inf as .Nan/.Inf/-.Inf)
std::string fs_double(double x) {
    char buf[64];
    if (std::isnan(x)) return ".Nan";
    if (std::isinf(x)) return x > 0 ? ".Inf" : "-.Inf";
    const double r = std::nearbyint(x);
    if (r == x && std::fabs(x) < 2147483647.0)
        std::snprintf(buf, sizeof buf, "%d.", (int)r);
    else
        std::snprintf(buf, sizeof buf, "%.16e", x);
    return buf;
}

bool write_fs_matrix(const std::string &path, const char *name, const std::vector<double> &m,
                     int rows, int cols) {
    std::ofstream f(path);
    if (!f) return false;
    f << "%YAML:1.0\n---\n" << name << ": !!opencv-matrix\n   rows: " << rows
      << "\n   cols: " << cols << "\n   dt: d\n   data: [ ";
    size_t line = 0;
    for (size_t i = 0; i < m.size(); ++i) {
        std::string s = fs_double(m[i]);
        if (i + 1 < m.size()) s += ", ";
        if (line + s.size() > 70) {
            f << "\n       ";
            line = 0;
        }
        f << s;
        line += s.size();
    }
    f << " ]\n";
    return (bool)f;
}

// ---- plotFlow.cpp:24-88, headless --------------------------------------
void set_pixel(Image &im, int x, int y, int r, int g, int b) {
    if ((x < im.rows - 1) & (x >= 0))
        if ((y < im.cols - 1) & (y >= 0)) {
            uint8_t *p = &im.px[((size_t)x * im.cols + y) * 3];
            p[0] = (uint8_t)r;  // [0]=r,[1]=g,[2]=b into BGR memory, as plotFlow.cpp:27-29
            p[1] = (uint8_t)g;
            p[2] = (uint8_t)b;
        }
}

int sgn(int x) { return x < 0 ? -1 : (x > 0 ? 1 : 0); }

void bresenham(Image &im, int x0, int y0, int x1, int y1, int r, int g, int b) {
    int dX = x1 - x0, dY = y1 - y0;
    const int sX = sgn(dX), sY = sgn(dY);
    dX = std::abs(dX);
    dY = std::abs(dY);
    const int dist = std::max(dX, dY);
    double R = dist / 2;  // integer division (plotFlow.cpp:51)
    int x = x0, y = y0;
    for (int i = 0; i < dist; ++i) {
        set_pixel(im, x, y, r, g, b);
        if (dX > dY) {
            x += sX;
            R += dY;
            if (R >= dX) {
                y += sY;
                R -= dX;
            }
        } else {
            y += sY;
            R += dX;
            if (R >= dY) {
                x += sX;
                R -= dY;
            }
        }
    }
}

void plot_bresenham_line(Image &im, const std::vector<double> &u, const std::vector<double> &v,
                         int delta, float scale, int outlier) {
    for (int x1 = 0; x1 < im.rows; x1 += delta)
        for (int y1 = 0; y1 < im.cols; y1 += delta) {
            const double uu = u[(size_t)x1 * im.cols + y1], vv = v[(size_t)x1 * im.cols + y1];
            const int x2 = (int)(x1 + (uu * scale));  // u moves the ROW (reference quirk)
            const int y2 = (int)(y1 + (vv * scale));
            if (outlier > 0) {
                if ((uu < outlier) & (vv < outlier) & (uu > -1 * outlier) & (vv > -1 * outlier))
                    bresenham(im, x1, y1, x2, y2, 0, 255, 0);
            } else {
                bresenham(im, x1, y1, x2, y2, 0, 255, 0);
            }
            set_pixel(im, x2, y2, 0, 0, 255);
        }
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 4) {
        std::cout << "usage: hs_main prev.{pgm,ppm} next.{pgm,ppm} savePath "
                     "[windowSize maxIterations alpha]\n"
                     "       hs_main video.y4m prevFrame nextFrame savePath "
                     "[windowSize maxIterations alpha]\n";
        return 0;
    }
    // main.cpp:48-64: image pair or two frames of a video by index
    const bool video = ends_with(argv[1], ".y4m");
    if (video && argc < 5) {
        std::cout << "No image or video input given! Please try again!" << std::endl;
        return 0;
    }
    const int a0 = video ? 5 : 4;  // first optional argument
    const std::string savePath = argv[a0 - 1];
    const int windowSize = argc > a0 ? std::atoi(argv[a0]) : 5;          // main.cpp:94
    const int maxIterations = argc > a0 + 1 ? std::atoi(argv[a0 + 1]) : 100;  // main.cpp:95
    const double alpha = argc > a0 + 2 ? std::atof(argv[a0 + 2]) : 1.0;       // main.cpp:96

    Image prevRaw, nextRaw;
    const bool ok = video ? read_y4m_frame(argv[1], std::atol(argv[2]), prevRaw) &&
                                read_y4m_frame(argv[1], std::atol(argv[3]), nextRaw)
                          : read_pnm(argv[1], prevRaw) && read_pnm(argv[2], nextRaw);
    if (!ok) {
        std::cout << "Can't read the images. Please check the path." << std::endl;
        return -1;
    }
    if (prevRaw.rows != nextRaw.rows || prevRaw.cols != nextRaw.cols) {
        std::cout << "Image sizes are different. Please provide images of same size."
                  << std::endl;
        return -1;
    }
    // main.cpp:11-26 preprocess
    auto to_gray = [](const Image &im) {
        std::vector<uint8_t> g((size_t)im.rows * im.cols);
        if (im.channels == 3)
            hsflow_bgr_to_gray(im.px.data(), im.rows, im.cols, (size_t)im.cols * 3, g.data(),
                               (size_t)im.cols);
        else
            g = im.px;
        return g;
    };
    const std::vector<uint8_t> prev = to_gray(prevRaw), next = to_gray(nextRaw);

    std::vector<double> u, v;
    try {
        hsflow::HornSchunck hs = hsflow::HornSchunck(windowSize, maxIterations, alpha);
        hs.getFlow(hsflow::view(prev.data(), prevRaw.rows, prevRaw.cols),
                   hsflow::view(next.data(), nextRaw.rows, nextRaw.cols), u, v);
    } catch (const hsflow::Error &e) {
        std::cerr << e.what() << std::endl;
        return 1;
    }
    write_fs_matrix(savePath + "uMatrixHS.txt", "u matrix", u, prevRaw.rows, prevRaw.cols);
    write_fs_matrix(savePath + "vMatrixHS.txt", "v matrix", v, prevRaw.rows, prevRaw.cols);

    Image canvas;
    canvas.rows = prevRaw.rows;
    canvas.cols = prevRaw.cols;
    canvas.channels = 3;
    canvas.px.resize((size_t)canvas.rows * canvas.cols * 3);
    for (size_t i = 0; i < (size_t)canvas.rows * canvas.cols; ++i)
        for (int c = 0; c < 3; ++c)
            canvas.px[i * 3 + c] =
                prevRaw.channels == 3 ? prevRaw.px[i * 3 + c] : prevRaw.px[i];
    plot_bresenham_line(canvas, u, v, 20, 20.0f, 5);
    write_ppm_bgr(savePath + "hsbresenhamLineFlow.ppm", canvas);
    std::cout << "Saved HS Algorithm Results in " + savePath << std::endl;
    return 0;
}
