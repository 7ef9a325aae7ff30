/*
 * orbgpu_cv.hpp -- header-only C++ drop-in for ORB_SLAM3::ORBextractor on top of the C ABI
 * (orbgpu.h).  Same public interface as the reference class (include/ORBextractor.h:43-109):
 * constructor (nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST), operator()(image, mask,
 * keypoints, descriptors, vLappingArea) returning monoIndex, the scale getters and the public
 * mvImagePyramid.  Include it instead of ORBextractor.h and alias the type:
 *
 *     #include "orbgpu_cv.hpp"
 *     namespace ORB_SLAM3 { using ORBextractor = orbgpu::ORBextractor; }
 *
 * Needs OpenCV (core) and liborbgpu.so at link time.  mvImagePyramid is downloaded on first
 * access after each extraction: only Frame::ComputeStereoMatches reads it (src/Frame.cc:1126,
 * 1249,1268,1275, always through operator[]), so tracking without stereo never pays the copy and
 * the caller compiles unchanged.  The levels are views into padded planes, like the reference's
 * (src/ORBextractor.cc:1695-1697).  The device writes each level plus a 3-pixel border; the download
 * (orb_extractor_level_download) fills the rest of the 19-pixel ring on the host by the REFLECT_101
 * rule of the reference's copyMakeBorder (:1712-1716, 1734-1736), so every byte reachable through the
 * view's ROI equals the reference's padded plane.
 */
#ifndef ORBGPU_CV_HPP
#define ORBGPU_CV_HPP

#include <stdexcept>
#include <string>
#include <vector>

#include <opencv2/core/core.hpp>

#include "orbgpu.h"

namespace orbgpu {

class ORBextractor;

// std::vector<cv::Mat>-like view of the last frame's pyramid that downloads it from the device on
// the first operator[] after an extraction (the reference member is a plain vector, include/
// ORBextractor.h:83; its readers use only operator[], size() and iteration).
class LazyPyramid {
public:
    explicit LazyPyramid(ORBextractor* owner) : owner_(owner) {}
    cv::Mat& operator[](size_t l);
    const cv::Mat& operator[](size_t l) const { return const_cast<LazyPyramid*>(this)->operator[](l); }
    size_t size() const { return levels_.size(); }
    void resize(size_t n) { levels_.resize(n); }
    std::vector<cv::Mat>::iterator begin();
    std::vector<cv::Mat>::iterator end() { return levels_.end(); }

private:
    friend class ORBextractor;
    ORBextractor* owner_;
    std::vector<cv::Mat> levels_;
};

class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST,
                 int maxWidth = 1280, int maxHeight = 720)
        : nfeatures_(nfeatures), scaleFactor_(scaleFactor), nlevels_(nlevels) {
        orb_params_t p{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST};
        if (orb_extractor_create(&p, maxWidth, maxHeight, 1, &h_) != ORB_OK)
            throw std::runtime_error(std::string("orb_extractor_create: ") + orb_last_error());
        mvScaleFactor_.resize(nlevels);
        mvInvScaleFactor_.resize(nlevels);
        mvLevelSigma2_.resize(nlevels);
        mvInvLevelSigma2_.resize(nlevels);
        std::vector<int32_t> per(nlevels);
        orb_extractor_scales(h_, mvScaleFactor_.data(), mvInvScaleFactor_.data(), mvLevelSigma2_.data(),
                             mvInvLevelSigma2_.data(), per.data());
        mvImagePyramid.resize(nlevels);
    }
    // mvImagePyramid refers back to this object
    ORBextractor(ORBextractor&&) = delete;
    ~ORBextractor() { orb_extractor_destroy(h_); }
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    // src/ORBextractor.cc:1557-1682.  Returns monoIndex, or -1 for an empty image.
    int operator()(cv::InputArray _image, cv::InputArray /*_mask (ignored upstream)*/,
                   std::vector<cv::KeyPoint>& _keypoints, cv::OutputArray _descriptors,
                   std::vector<int>& vLappingArea) {
        if (_image.empty()) return -1;
        cv::Mat image = _image.getMat();
        CV_Assert(image.type() == CV_8UC1);
        int cap = 2 * nfeatures_ + 64 * nlevels_;
        for (int attempt = 0; attempt < 2; ++attempt) {
            kps_.resize(cap);
            desc_.create(cap, 32, CV_8U);
            int n = 0;
            int rc = orb_extract(h_, image.data, image.cols, image.rows, (int)image.step, vLappingArea[0],
                                 vLappingArea[1], kps_.data(), desc_.data, cap, &n);
            if (rc == ORB_ERR_CAPACITY) { cap = n; continue; }
            if (rc < 0) throw std::runtime_error(std::string("orb_extract: ") + orb_last_error());
            _keypoints.resize(n);
            for (int i = 0; i < n; ++i) {
                const orb_keypoint_t& k = kps_[i];
                _keypoints[i] = cv::KeyPoint(k.x, k.y, k.size, k.angle, k.response, k.octave, k.class_id);
            }
            if (n == 0) _descriptors.release();
            else desc_.rowRange(0, n).copyTo(_descriptors);
            pyramidStale_ = true;
            return rc;
        }
        throw std::runtime_error("orb_extract: capacity retry failed");
    }

    int inline GetLevels() { return nlevels_; }
    float inline GetScaleFactor() { return (float)scaleFactor_; }
    std::vector<float> inline GetScaleFactors() { return mvScaleFactor_; }
    std::vector<float> inline GetInverseScaleFactors() { return mvInvScaleFactor_; }
    std::vector<float> inline GetScaleSigmaSquares() { return mvLevelSigma2_; }
    std::vector<float> inline GetInverseScaleSigmaSquares() { return mvInvLevelSigma2_; }

    // Download the pyramid of the last frame into mvImagePyramid.  mvImagePyramid[l] calls this
    // itself; an explicit call only moves the copy to a chosen point.
    void SyncPyramid() {
        if (!pyramidStale_) return;
        for (int l = 0; l < nlevels_; ++l) {
            int w = 0, h = 0, pitch = 0;
            if (orb_extractor_level(h_, 0, l, nullptr, &w, &h, &pitch) != ORB_OK)
                throw std::runtime_error(std::string("orb_extractor_level: ") + orb_last_error());
            padded_[l].create(h + 38, w + 38, CV_8U);
            orb_extractor_level_download(h_, 0, l, padded_[l].data);
            mvImagePyramid.levels_[l] = padded_[l](cv::Rect(19, 19, w, h));
        }
        pyramidStale_ = false;
    }

    LazyPyramid mvImagePyramid{this};

    // the underlying handle, for the device-side consumers of the pyramid (orb_compute_stereo_matches)
    orb_extractor_t handle() const { return h_; }

private:
    orb_extractor_t h_ = nullptr;
    int nfeatures_;
    double scaleFactor_;
    int nlevels_;
    bool pyramidStale_ = true;
    std::vector<orb_keypoint_t> kps_;
    cv::Mat desc_;
    cv::Mat padded_[12];
    std::vector<float> mvScaleFactor_, mvInvScaleFactor_, mvLevelSigma2_, mvInvLevelSigma2_;
};

inline cv::Mat& LazyPyramid::operator[](size_t l) {
    owner_->SyncPyramid();
    return levels_[l];
}
inline std::vector<cv::Mat>::iterator LazyPyramid::begin() {
    owner_->SyncPyramid();
    return levels_.begin();
}

}  // namespace orbgpu

#endif  // ORBGPU_CV_HPP
