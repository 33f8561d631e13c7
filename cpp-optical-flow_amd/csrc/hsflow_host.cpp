// hsflow_host.cpp -- host-side utilities of libhsflow.so on the path into the
// hot loop: the reference's BGR->gray pre-processing (main.cpp:13-14) and the
// deterministic synthetic frame-pair generator used by bench.py.

#include <stdint.h>

#include <algorithm>
#include <vector>

#include "../../include/hsflow.h"

namespace {

inline uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

inline int64_t floor_div(int64_t a, int64_t b) {
    int64_t q = a / b;
    return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}

}  // namespace

extern "C" int hsflow_bgr_to_gray(const uint8_t *bgr, int rows, int cols,
                                  size_t bgr_step, uint8_t *gray, size_t gray_step) {
    if (!bgr || !gray || rows < 1 || cols < 1 || bgr_step < (size_t)cols * 3 ||
        gray_step < (size_t)cols)
        return HSFLOW_ERR_ARG;
    for (int r = 0; r < rows; ++r) {
        const uint8_t *p = bgr + (size_t)r * bgr_step;
        uint8_t *g = gray + (size_t)r * gray_step;
        for (int c = 0; c < cols; ++c) {
            const uint32_t B = p[3 * c], G = p[3 * c + 1], R = p[3 * c + 2];
            g[c] = (uint8_t)((9798u * R + 19235u * G + 3735u * B + 16384u) >> 15);
        }
    }
    return HSFLOW_OK;
}

// Texture T(r, c) on the whole integer plane:
//   n(r, c) = top byte of splitmix64(splitmix64(seed) ^ (r << 32 | c))
//   S = 7x7 box sum of n;  T = clamp(128 + floor((S - 6248) * 5 / 64), 0, 255)
// I0 = T;  I1(r, c) = bilinear T at (r - qdy/4, c - qdx/4), integer weights
// in quarters, rounded half up: (sum w*T + 8) >> 4.
extern "C" int hsflow_synth_pair(uint64_t seed, int rows, int cols, int qdy, int qdx,
                                 float *I0, float *I1, uint8_t *I0_u8, uint8_t *I1_u8) {
    if (rows < 1 || cols < 1 || qdy < -64 || qdy > 64 || qdx < -64 || qdx > 64)
        return HSFLOW_ERR_ARG;
    const int64_t qy = -qdy, qx = -qdx;
    // texture box [ty0, ty1) x [tx0, tx1) needed by I0 and I1
    const int64_t ty0 = std::min<int64_t>(0, floor_div(qy, 4));
    const int64_t ty1 = std::max<int64_t>(rows, floor_div(4 * (int64_t)(rows - 1) + qy, 4) + 2);
    const int64_t tx0 = std::min<int64_t>(0, floor_div(qx, 4));
    const int64_t tx1 = std::max<int64_t>(cols, floor_div(4 * (int64_t)(cols - 1) + qx, 4) + 2);
    const int R = 3;
    const int64_t nh = ty1 - ty0 + 2 * R, nw = tx1 - tx0 + 2 * R;
    const uint64_t smix = splitmix64(seed);
    // horizontal 7-sums of the noise, then vertical
    std::vector<int32_t> hs((size_t)nh * (tx1 - tx0));
    std::vector<int32_t> row((size_t)nw);
    for (int64_t i = 0; i < nh; ++i) {
        const int64_t r = ty0 - R + i;
        for (int64_t j = 0; j < nw; ++j) {
            const int64_t c = tx0 - R + j;
            const uint64_t key = ((uint64_t)(uint32_t)(int32_t)r << 32) | (uint32_t)(int32_t)c;
            row[j] = (int32_t)(splitmix64(smix ^ key) >> 56);
        }
        int32_t acc = 0;
        for (int j = 0; j < 2 * R + 1; ++j) acc += row[j];
        const int64_t w = tx1 - tx0;
        for (int64_t j = 0; j < w; ++j) {
            hs[(size_t)i * w + j] = acc;
            if (j + 2 * R + 1 < nw) acc += row[j + 2 * R + 1] - row[j];
        }
    }
    const int64_t th = ty1 - ty0, tw = tx1 - tx0;
    std::vector<uint8_t> T((size_t)th * tw);
    for (int64_t j = 0; j < tw; ++j) {
        int32_t acc = 0;
        for (int i = 0; i < 2 * R + 1; ++i) acc += hs[(size_t)i * tw + j];
        for (int64_t i = 0; i < th; ++i) {
            const int64_t t = 128 + floor_div((int64_t)(acc - 6248) * 5, 64);
            T[(size_t)i * tw + j] = (uint8_t)std::min<int64_t>(255, std::max<int64_t>(0, t));
            if (i + 2 * R + 1 < nh) acc += hs[(size_t)(i + 2 * R + 1) * tw + j] - hs[(size_t)i * tw + j];
        }
    }
    auto tex = [&](int64_t r, int64_t c) -> int32_t {
        return T[(size_t)(r - ty0) * tw + (c - tx0)];
    };
    for (int r = 0; r < rows; ++r) {
        const int64_t y4 = 4 * (int64_t)r + qy;
        const int64_t y0 = floor_div(y4, 4), fy = y4 - 4 * y0;
        for (int c = 0; c < cols; ++c) {
            const int64_t x4 = 4 * (int64_t)c + qx;
            const int64_t x0 = floor_div(x4, 4), fx = x4 - 4 * x0;
            const int32_t a = tex(r, c);
            const int32_t num = (int32_t)((4 - fy) * (4 - fx) * tex(y0, x0) +
                                          (4 - fy) * fx * tex(y0, x0 + 1) +
                                          fy * (4 - fx) * tex(y0 + 1, x0) +
                                          fy * fx * tex(y0 + 1, x0 + 1));
            const int32_t b = (num + 8) >> 4;
            const size_t o = (size_t)r * cols + c;
            if (I0) I0[o] = (float)a;
            if (I1) I1[o] = (float)b;
            if (I0_u8) I0_u8[o] = (uint8_t)a;
            if (I1_u8) I1_u8[o] = (uint8_t)b;
        }
    }
    return HSFLOW_OK;
}
