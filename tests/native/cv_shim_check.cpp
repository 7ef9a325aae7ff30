// CPU check of include/orbgpu_cv.hpp (the ORBextractor drop-in) against ABI test doubles and a mock
// OpenCV core (tests/native/mock_cv), so the shim is compiled and run without OpenCV or a GPU; the
// extraction itself is compared with the oracle in tests/test_extract_gpu.py.  Checked:
//   * constructor: the orb_params_t it passes, the scale getters (include/ORBextractor.h:61-83);
//   * operator() (src/ORBextractor.cc:1557-1682): the lapping area forwarded, keypoints converted
//     field by field, descriptors as an n x 32 matrix, monoIndex returned, the ORB_ERR_CAPACITY retry
//     with the needed count, an empty image returning -1;
//   * failures never throw (orbgpu_status.hpp): a library error, a second capacity shortfall, a handle
//     that cannot be created (scale getters from the host restatement of src/ORBextractor.cc:474-500)
//     and a failed pyramid download each give the reference's result for a frame without corners
//     (no keypoints, descriptors released, monoIndex 0) or empty levels, with the code reported;
//   * mvImagePyramid (read by Frame::ComputeStereoMatches as mvImagePyramid[octave],
//     src/Frame.cc:1126,1249,1268,1275): downloaded on the first operator[] after an extraction and
//     not again until the next one; each level a view at (19, 19) inside its padded plane, so the
//     19-pixel border is readable at negative offsets.
#include <cmath>
#include <cstdio>
#include <vector>

#include "orbgpu_cv.hpp"

static int g_fail = 0;
#define CHECK(c)                                                     \
    do {                                                             \
        if (!(c)) {                                                  \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                \
        }                                                            \
    } while (0)

// ---- ABI test doubles ---------------------------------------------------------------------------------
static orb_params_t g_params;
static int g_nfound = 37, g_extract_calls = 0, g_downloads = 0, g_last_cap = 0, g_lap[2];
static bool g_fail_next = false, g_fail_create = false, g_fail_level = false, g_grow = false;
static int g_handle_obj;

static int level_w(int l) { return (int)std::lround(640 / std::pow(1.2, l)); }
static int level_h(int l) { return (int)std::lround(480 / std::pow(1.2, l)); }

extern "C" {
const char* orb_last_error(void) { return "mock failure"; }
int orb_extractor_create(const orb_params_t* p, int, int, int, orb_extractor_t* out) {
    if (g_fail_create) return ORB_ERR_DEVICE;
    g_params = *p;
    *out = (orb_extractor_t)&g_handle_obj;
    return ORB_OK;
}
int orb_extractor_destroy(orb_extractor_t) { return ORB_OK; }
int orb_extractor_scales(orb_extractor_t, float* s, float* is, float* s2, float* is2, int32_t* per) {
    for (int l = 0; l < g_params.nlevels; ++l) {
        const float f = std::pow(g_params.scale_factor, (float)l);
        s[l] = f, is[l] = 1.f / f, s2[l] = f * f, is2[l] = 1.f / (f * f), per[l] = 100 + l;
    }
    return ORB_OK;
}
int orb_extract(orb_extractor_t, const uint8_t* image, int w, int h, int stride, int lx0, int lx1,
                orb_keypoint_t* kps, uint8_t* desc, int cap, int* n) {
    ++g_extract_calls;
    g_last_cap = cap, g_lap[0] = lx0, g_lap[1] = lx1;
    if (g_fail_next) { g_fail_next = false; return ORB_ERR_DEVICE; }
    if (!image || w != 640 || h != 480 || stride != 640) return ORB_ERR_ARG;
    if (g_grow) g_nfound = cap + 1;  // never enough room
    *n = g_nfound;
    if (cap < g_nfound) return ORB_ERR_CAPACITY;
    for (int i = 0; i < g_nfound; ++i) {
        kps[i] = orb_keypoint_t{1.5f * i, 2.5f * i, 31.f, (float)i, 0.25f * i, i % 8, -1};
        for (int b = 0; b < 32; ++b) desc[i * 32 + b] = (uint8_t)(i * 7 + b);
    }
    return g_nfound > 5 ? g_nfound - 5 : 0;  // monoIndex
}
int orb_extractor_level(orb_extractor_t, int frame, int l, const uint8_t**, int* w, int* h, int* pitch) {
    if (g_fail_level || frame != 0 || l < 0 || l >= g_params.nlevels) return ORB_ERR_ARG;
    *w = level_w(l), *h = level_h(l), *pitch = *w + 38;
    return ORB_OK;
}
int orb_extractor_level_download(orb_extractor_t, int, int l, uint8_t* p) {
    ++g_downloads;
    const int pw = level_w(l) + 38, ph = level_h(l) + 38;
    for (int r = 0; r < ph; ++r)
        for (int c = 0; c < pw; ++c) p[(size_t)r * pw + c] = (uint8_t)(l * 31 + r * 7 + c + g_extract_calls);
    return ORB_OK;
}
}

int main() {
    orbgpu::ORBextractor ex(1000, 1.2f, 8, 20, 7);
    CHECK(g_params.nfeatures == 1000 && g_params.scale_factor == 1.2f && g_params.nlevels == 8 &&
          g_params.ini_th_fast == 20 && g_params.min_th_fast == 7);
    CHECK(ex.GetLevels() == 8 && ex.GetScaleFactor() == 1.2f);
    CHECK(ex.GetScaleFactors().size() == 8 && ex.GetScaleFactors()[3] == std::pow(1.2f, 3.f));
    CHECK(ex.GetInverseScaleSigmaSquares()[2] == 1.f / (std::pow(1.2f, 2.f) * std::pow(1.2f, 2.f)));
    CHECK(ex.mvImagePyramid.size() == 8);

    cv::Mat img(480, 640, CV_8U);
    std::vector<cv::KeyPoint> kps;
    cv::Mat desc;
    std::vector<int> lap = {100, 400};

    // capacity retry: the needed count is reported and the call repeated with it
    g_nfound = 2 * 1000 + 64 * 8 + 3;
    int mono = ex(img, cv::Mat(), kps, desc, lap);
    CHECK(g_extract_calls == 2 && g_last_cap == g_nfound);
    CHECK(mono == g_nfound - 5 && (int)kps.size() == g_nfound && desc.rows == g_nfound && desc.cols == 32);
    CHECK(g_lap[0] == 100 && g_lap[1] == 400);

    g_nfound = 37;
    const int calls0 = g_extract_calls;
    mono = ex(img, cv::Mat(), kps, desc, lap);
    CHECK(g_extract_calls == calls0 + 1 && mono == 32 && kps.size() == 37 && desc.rows == 37);
    CHECK(kps[5].pt.x == 7.5f && kps[5].pt.y == 12.5f && kps[5].size == 31.f && kps[5].angle == 5.f &&
          kps[5].response == 1.25f && kps[5].octave == 5 && kps[5].class_id == -1);
    CHECK(desc.at(4, 3) == (uint8_t)(4 * 7 + 3) && desc.at(36, 31) == (uint8_t)(36 * 7 + 31));

    // pyramid: nothing downloaded until read, all levels on the first read, then cached
    CHECK(g_downloads == 0);
    const cv::Mat& l3 = ex.mvImagePyramid[3];
    CHECK(g_downloads == 8);
    CHECK(l3.cols == level_w(3) && l3.rows == level_h(3));
    const int stamp = g_extract_calls;
    CHECK(l3.at(0, 0) == (uint8_t)(3 * 31 + 19 * 7 + 19 + stamp));  // view origin at (19, 19)
    CHECK(l3.data[-19 * (long)l3.step - 19] == (uint8_t)(3 * 31 + stamp));  // border readable
    const int nRows = ex.mvImagePyramid[0].rows;  // src/Frame.cc:1126
    CHECK(nRows == 480 && g_downloads == 8);
    cv::Mat IL = ex.mvImagePyramid[2].rowRange(10, 21).colRange(30, 41);  // src/Frame.cc:1249
    CHECK(IL.rows == 11 && IL.cols == 11 && IL.at(0, 0) == (uint8_t)(2 * 31 + 29 * 7 + 49 + stamp));
    CHECK(g_downloads == 8);
    const orbgpu::ORBextractor& cex = ex;
    CHECK(cex.mvImagePyramid[7].cols == level_w(7) && g_downloads == 8);

    // the next extraction makes the pyramid stale again
    ex(img, cv::Mat(), kps, desc, lap);
    CHECK(g_downloads == 8);
    CHECK(ex.mvImagePyramid[1].at(0, 0) == (uint8_t)(31 + 19 * 7 + 19 + g_extract_calls));
    CHECK(g_downloads == 16);

    // no keypoints: the descriptor matrix is released
    g_nfound = 0;
    mono = ex(img, cv::Mat(), kps, desc, lap);
    CHECK(mono == 0);
    CHECK(kps.empty() && desc.empty());

    // empty image and library errors
    CHECK(ex(cv::Mat(), cv::Mat(), kps, desc, lap) == -1);
    g_nfound = 37;
    ex(img, cv::Mat(), kps, desc, lap);
    CHECK(kps.size() == 37 && orbgpu::LastShimError() == ORB_OK);
    const long fails0 = orbgpu::ShimFailureCount();
    bool threw = false;
    try {
        g_fail_next = true;
        CHECK(ex(img, cv::Mat(), kps, desc, lap) == 0 && kps.empty() && desc.empty());
        CHECK(orbgpu::LastShimError() == ORB_ERR_DEVICE &&
              orbgpu::LastShimMessage().find("mock failure") != std::string::npos);
        orbgpu::ClearShimError();
        g_grow = true;  // the capacity retry falls short again
        CHECK(ex(img, cv::Mat(), kps, desc, lap) == 0 && kps.empty() && desc.empty());
        CHECK(orbgpu::LastShimError() == ORB_ERR_CAPACITY);
        g_grow = false;
        g_nfound = 37;
        orbgpu::ClearShimError();
        CHECK(ex(img, cv::Mat(), kps, desc, lap) == 32 && kps.size() == 37 && orbgpu::LastShimError() == ORB_OK);
        g_fail_level = true;  // pyramid download fails: empty levels
        CHECK(ex.mvImagePyramid[2].empty() && ex.mvImagePyramid.size() == 8);
        CHECK(orbgpu::LastShimError() == ORB_ERR_ARG);
        g_fail_level = false;
        // a handle that cannot be created
        g_fail_create = true;
        orbgpu::ClearShimError();
        orbgpu::ORBextractor bad(1200, 1.2f, 8, 20, 7);
        CHECK(orbgpu::LastShimError() == ORB_ERR_DEVICE);
        float s = 1.0f;
        const double sf = 1.2f;
        for (int l = 0; l < 8; ++l) {  // src/ORBextractor.cc:474-500
            if (l) s = (float)(s * sf);
            CHECK(bad.GetScaleFactors()[l] == s && bad.GetScaleSigmaSquares()[l] == (l ? s * s : 1.0f));
            CHECK(bad.GetInverseScaleFactors()[l] == 1.0f / s);
        }
        const int calls = g_extract_calls;
        orbgpu::ClearShimError();
        CHECK(bad(img, cv::Mat(), kps, desc, lap) == 0 && kps.empty() && desc.empty());
        CHECK(g_extract_calls == calls && orbgpu::LastShimError() != ORB_OK);
        CHECK(bad.mvImagePyramid[0].empty());
        g_fail_create = false;
    } catch (...) {
        threw = true;
    }
    CHECK(!threw);
    CHECK(orbgpu::ShimFailureCount() >= fails0 + 5);

    if (g_fail) return 1;
    std::printf("OK cv_shim_check\n");
    return 0;
}
