// GPU check of include/orbgpu_cv.hpp (the ORBextractor drop-in) linked to the real liborbgpu.so, with
// the minimal OpenCV stand-in of tests/native/mock_cv (OpenCV is absent from this image).  Each
// extraction is compared with the oracle (oracle/_build/liborb_oracle.so, test infrastructure) on the
// same image:
//   * operator() (src/ORBextractor.cc:1557-1682): keypoints field by field, descriptors, monoIndex, for
//     mono ({0, 1000}), stereo ({0, 0}) and an odd lapping area, at 640x480 and 752x480, and with the
//     initialisation extractor's 5 x nFeatures (src/Tracking.cc:659-665);
//   * the getters against the oracle's scale tables (include/ORBextractor.h:61-81);
//   * mvImagePyramid[l] (read by Frame::ComputeStereoMatches, src/Frame.cc:1126,1249): every byte of the
//     padded plane a ROI can reach (the view and its 19-pixel REFLECT_101 border) equals the oracle's;
//   * an empty image returns -1.
// Input: images written by tests/test_shims_gpu.py.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "orbgpu_cv.hpp"
#include "shim_records.h"

extern "C" {
typedef struct oracle_orb_s oracle_orb_t;
oracle_orb_t* oracle_orb_create(int nfeatures, float scale_factor, int nlevels, int ini_th, int min_th);
void oracle_orb_destroy(oracle_orb_t* h);
void oracle_orb_params(oracle_orb_t* h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2,
                       int* n_per_level, int* umax);
int oracle_orb_extract(oracle_orb_t* h, const uint8_t* img, int w, int hgt, int stride, int lap0, int lap1, void* kps,
                       uint8_t* desc, int cap, int* n_out);
void oracle_orb_level_dims(oracle_orb_t* h, int level, int* w, int* hh, int* pw, int* ph);
void oracle_orb_level_copy(oracle_orb_t* h, int level, uint8_t* out);
}

static int g_fail = 0;
#define CHECK(c)                                                     \
    do {                                                             \
        if (!(c)) {                                                  \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                \
        }                                                            \
    } while (0)

static void run_case(const std::vector<uint8_t>& img, int w, int h, int nfeatures, int lap0, int lap1) {
    const float sf = 1.2f;
    const int nl = 8;
    orbgpu::ORBextractor ex(nfeatures, sf, nl, 20, 7, 1280, 720);
    oracle_orb_t* ref = oracle_orb_create(nfeatures, sf, nl, 20, 7);
    // getters
    std::vector<float> s(nl), is(nl), s2(nl), is2(nl);
    std::vector<int> per(nl), umax(16);
    oracle_orb_params(ref, s.data(), is.data(), s2.data(), is2.data(), per.data(), umax.data());
    CHECK(ex.GetLevels() == nl && ex.GetScaleFactor() == sf);
    CHECK(ex.GetScaleFactors() == s && ex.GetInverseScaleFactors() == is);
    CHECK(ex.GetScaleSigmaSquares() == s2 && ex.GetInverseScaleSigmaSquares() == is2);
    // operator()
    cv::Mat image(h, w, CV_8U);
    std::memcpy(image.data, img.data(), img.size());
    std::vector<cv::KeyPoint> kps;
    cv::Mat desc;
    std::vector<int> lap{lap0, lap1};
    const int mono = ex(image, cv::Mat(), kps, desc, lap);
    const int cap = 8 * nfeatures + 1024;
    std::vector<orb_keypoint_t> rk(cap);
    std::vector<uint8_t> rd((size_t)cap * 32);
    int rn = 0;
    const int rmono = oracle_orb_extract(ref, img.data(), w, h, w, lap0, lap1, rk.data(), rd.data(), cap, &rn);
    int kp_bad = 0, desc_bad = 0;
    CHECK((int)kps.size() == rn && mono == rmono);
    for (int i = 0; i < rn && i < (int)kps.size(); ++i) {
        const cv::KeyPoint& a = kps[i];
        const orb_keypoint_t& b = rk[i];
        if (a.pt.x != b.x || a.pt.y != b.y || a.size != b.size || a.angle != b.angle || a.response != b.response ||
            a.octave != b.octave || a.class_id != b.class_id)
            ++kp_bad;
        if (std::memcmp(desc.data + (size_t)i * desc.step, &rd[32 * (size_t)i], 32) != 0) ++desc_bad;
    }
    CHECK(desc.rows == rn && desc.cols == 32);
    // mvImagePyramid: the view and the 19-pixel ring around it
    int pyr_bad = 0;
    for (int l = 0; l < nl; ++l) {
        int lw, lh, pw, ph;
        oracle_orb_level_dims(ref, l, &lw, &lh, &pw, &ph);
        std::vector<uint8_t> plane((size_t)pw * ph);
        oracle_orb_level_copy(ref, l, plane.data());
        const cv::Mat& v = ex.mvImagePyramid[l];
        CHECK(v.cols == lw && v.rows == lh);
        for (int y = -19; y < lh + 19; ++y)
            for (int x = -19; x < lw + 19; ++x)
                if (v.data[(long)y * (long)v.step + x] != plane[(size_t)(y + 19) * pw + (x + 19)]) ++pyr_bad;
    }
    std::printf("%dx%d nFeatures %d lapping {%d,%d}: %d keypoints, monoIndex %d (oracle %d, %d); %d keypoints, %d "
                "descriptors, %d pyramid bytes differ\n",
                w, h, nfeatures, lap0, lap1, (int)kps.size(), mono, rn, rmono, kp_bad, desc_bad, pyr_bad);
    CHECK(kp_bad == 0 && desc_bad == 0 && pyr_bad == 0 && rn > 100);
    // an empty image: -1, as src/ORBextractor.cc:1561-1562
    cv::Mat empty;
    std::vector<cv::KeyPoint> k2;
    cv::Mat d2;
    CHECK(ex(empty, cv::Mat(), k2, d2, lap) == -1);
    oracle_orb_destroy(ref);
}

int main(int argc, char** argv) {
    Records r;
    if (argc < 2 || !r.Load(argv[1])) {
        std::printf("usage: %s images.bin\n", argv[0]);
        return 2;
    }
    try {
        const auto a = r.Get<uint8_t>("img640");
        const auto b = r.Get<uint8_t>("img752");
        run_case(a, 640, 480, 1000, 0, 1000);   // monocular Frame (src/Frame.cc:380)
        run_case(b, 752, 480, 1200, 0, 0);      // stereo Frame (src/Frame.cc:136-138)
        run_case(b, 752, 480, 1200, 100, 400);  // a lapping area: keypoints split front / back
        run_case(a, 640, 480, 5000, 0, 1000);   // the initialisation extractor, 5 x nFeatures
    } catch (const std::exception& e) {
        std::printf("FAIL exception: %s\n", e.what());
        return 1;
    }
    if (orbgpu::LastShimError() != ORB_OK) {  // failures do not throw: every call must have succeeded
        std::printf("FAIL shim error %d: %s\n", orbgpu::LastShimError(), orbgpu::LastShimMessage().c_str());
        return 1;
    }
    if (g_fail) {
        std::printf("%d checks failed\n", g_fail);
        return 1;
    }
    std::printf("OK cv_shim_gpu\n");
    return 0;
}
