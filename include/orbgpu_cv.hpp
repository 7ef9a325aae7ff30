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
 *
 * Failures (orbgpu_status.hpp): nothing here throws on a library failure.  A handle that cannot be
 * created leaves the scale getters on the host's restatement of the reference's tables
 * (src/ORBextractor.cc:474-500) and every extraction failing; a failed extraction returns what the
 * reference returns for an image without corners (no keypoints, descriptors released, monoIndex 0); a
 * failed pyramid download leaves empty levels.  orbgpu::LastShimError() reports each.
 */
#ifndef ORBGPU_CV_HPP
#define ORBGPU_CV_HPP

#include <string>
#include <vector>

#include <opencv2/core/core.hpp>

#include "orbgpu.h"
#include "orbgpu_status.hpp"

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
        if (detail::Failed(orb_extractor_create(&p, maxWidth, maxHeight, 1, &h_), "orb_extractor_create")) h_ = nullptr;
        const int nl = nlevels > 0 ? nlevels : 0;
        mvScaleFactor_.resize(nl);
        mvInvScaleFactor_.resize(nl);
        mvLevelSigma2_.resize(nl);
        mvInvLevelSigma2_.resize(nl);
        std::vector<int32_t> per(nl);
        if (!h_ || detail::Failed(orb_extractor_scales(h_, mvScaleFactor_.data(), mvInvScaleFactor_.data(),
                                                       mvLevelSigma2_.data(), mvInvLevelSigma2_.data(), per.data()),
                                  "orb_extractor_scales"))
            HostScales();
        mvImagePyramid.resize(nl);
    }
    // mvImagePyramid refers back to this object
    ORBextractor(ORBextractor&&) = delete;
    ~ORBextractor() {
        if (h_) orb_extractor_destroy(h_);
    }
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    // src/ORBextractor.cc:1557-1682.  Returns monoIndex, or -1 for an empty image.
    int operator()(cv::InputArray _image, cv::InputArray /*_mask (ignored upstream)*/,
                   std::vector<cv::KeyPoint>& _keypoints, cv::OutputArray _descriptors,
                   std::vector<int>& vLappingArea) {
        if (_image.empty()) return -1;
        cv::Mat image = _image.getMat();
        CV_Assert(image.type() == CV_8UC1);
        pyramidStale_ = true;
        int cap = 2 * nfeatures_ + 64 * nlevels_;
        for (int attempt = 0; attempt < 2; ++attempt) {
            kps_.resize(cap);
            desc_.create(cap, 32, CV_8U);
            int n = 0;
            int rc = h_ ? orb_extract(h_, image.data, image.cols, image.rows, (int)image.step, vLappingArea[0],
                                      vLappingArea[1], kps_.data(), desc_.data, cap, &n)
                        : ORB_ERR_ARG;
            if (rc == ORB_ERR_CAPACITY && attempt == 0 && n > cap) { cap = n; continue; }
            if (detail::Failed(rc, h_ ? "orb_extract" : "orb_extract (no extractor handle)")) break;
            _keypoints.resize(n);
            for (int i = 0; i < n; ++i) {
                const orb_keypoint_t& k = kps_[i];
                _keypoints[i] = cv::KeyPoint(k.x, k.y, k.size, k.angle, k.response, k.octave, k.class_id);
            }
            if (n == 0) _descriptors.release();
            else desc_.rowRange(0, n).copyTo(_descriptors);
            return rc;
        }
        // the reference's result for an image without corners
        _keypoints.clear();
        _descriptors.release();
        return 0;
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
        pyramidStale_ = false;
        for (int l = 0; l < nlevels_ && l < 12; ++l) {
            int w = 0, h = 0, pitch = 0;
            bool ok = !detail::Failed(h_ ? orb_extractor_level(h_, 0, l, nullptr, &w, &h, &pitch) : ORB_ERR_ARG,
                                      "orb_extractor_level");
            if (ok) {
                padded_[l].create(h + 38, w + 38, CV_8U);
                ok = !detail::Failed(orb_extractor_level_download(h_, 0, l, padded_[l].data), "orb_extractor_level_download");
            }
            if (!ok) {
                for (auto& m : mvImagePyramid.levels_) m = cv::Mat();  // no pyramid: empty levels
                return;
            }
            mvImagePyramid.levels_[l] = padded_[l](cv::Rect(19, 19, w, h));
        }
    }

    LazyPyramid mvImagePyramid{this};

    // the underlying handle, for the device-side consumers of the pyramid (orb_compute_stereo_matches)
    orb_extractor_t handle() const { return h_; }

private:
    // src/ORBextractor.cc:474-500 (scaleFactor is a double member; the tables are float)
    void HostScales() {
        const int nl = (int)mvScaleFactor_.size();
        for (int i = 0; i < nl; ++i) {
            mvScaleFactor_[i] = i == 0 ? 1.0f : (float)(mvScaleFactor_[i - 1] * scaleFactor_);
            mvLevelSigma2_[i] = i == 0 ? 1.0f : mvScaleFactor_[i] * mvScaleFactor_[i];
        }
        for (int i = 0; i < nl; ++i) {
            mvInvScaleFactor_[i] = 1.0f / mvScaleFactor_[i];
            mvInvLevelSigma2_[i] = 1.0f / mvLevelSigma2_[i];
        }
    }

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
