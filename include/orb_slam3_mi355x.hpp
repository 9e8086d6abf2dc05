// orb_slam3_mi355x.hpp — C++ host interface over the C ABI (orb_mi355x.h),
// mirroring ORB_SLAM3::ORBextractor (reference include/ORBextractor.h:43-109)
// and ORB_SLAM3::ORBmatcher (include/ORBmatcher.h:36-103) with the same names,
// argument meaning and error behaviour, but without OpenCV types: keypoints
// are orb_keypoint (layout-identical to cv::KeyPoint), descriptors a
// row-major N x 32 byte buffer (cv::Mat CV_8U N x 32), images 8UC1 pointers.
// INTEGRATION.md shows the cv::Mat glue a maintainer adds.
#pragma once
#include <cstdint>
#include <functional>
#include <stdexcept>
#include <utility>
#include <vector>

#include "orb_mi355x.h"

namespace ORB_SLAM3_MI355X {

typedef orb_keypoint KeyPoint;

struct Descriptors {                       // cv::Mat(N, 32, CV_8U), continuous
    int rows = 0;
    std::vector<uint8_t> data;
    const uint8_t* row(int i) const { return data.data() + 32 * (size_t)i; }
};

class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    // ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int device = 0)
        : nlevels_(nlevels), scaleFactor_(scaleFactor) {
        orbx_params p{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, 0, 1, 0};
        h_ = orbx_create(&p, device);
        if (!h_) throw std::runtime_error("orbx_create: bad parameters or no HIP device");
        scale_.resize(nlevels); inv_scale_.resize(nlevels); sigma2_.resize(nlevels); inv_sigma2_.resize(nlevels);
        orbx_get_tables(h_, scale_.data(), inv_scale_.data(), sigma2_.data(), inv_sigma2_.data(), nullptr, nullptr);
    }
    ~ORBextractor() { orbx_destroy(h_); }
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    // int operator()(InputArray image, InputArray mask, vector<KeyPoint>& keypoints,
    //                OutputArray descriptors, vector<int>& vLappingArea)
    // Returns monoIndex, or -1 for an empty image (ORBextractor.cc:1090-1091).
    int operator()(const uint8_t* image, int cols, int rows, size_t step, const void* /*mask: ignored*/,
                   std::vector<KeyPoint>& keypoints, Descriptors& descriptors, const std::vector<int>& vLappingArea) {
        if (!image || cols <= 0 || rows <= 0) return -1;
        const int cap = orbx_max_keypoints(h_, cols, rows);
        if (cap < 0) throw std::runtime_error("orbx_max_keypoints failed");
        keypoints.resize(cap);
        descriptors.data.resize((size_t)cap * 32);
        int n = 0, mono = 0;
        const int rc = orbx_extract(h_, image, cols, rows, step, vLappingArea.at(0), vLappingArea.at(1),
                                    keypoints.data(), descriptors.data.data(), cap, &n, &mono);
        if (rc != ORB_OK) throw std::runtime_error("orbx_extract failed");
        keypoints.resize(n);
        descriptors.rows = n;
        descriptors.data.resize((size_t)n * 32);
        return mono;
    }

    // operator() on several images of one size in one call (orbx_extract_batch),
    // e.g. the left and right images of a stereo frame; returns the monoIndex
    // of each image.  images[f] has row step steps[f]; laps[f] = its vLappingArea.
    std::vector<int> ExtractBatch(const std::vector<const uint8_t*>& images, const std::vector<size_t>& steps,
                                  int cols, int rows, const std::vector<std::pair<int, int>>& laps,
                                  std::vector<std::vector<KeyPoint>>& keypoints,
                                  std::vector<Descriptors>& descriptors) {
        const int nf = (int)images.size();
        if (nf == 0) return {};
        const int cap = orbx_max_keypoints(h_, cols, rows);
        if (cap < 0) throw std::runtime_error("orbx_max_keypoints failed");
        std::vector<KeyPoint> kps((size_t)nf * cap);
        std::vector<uint8_t> desc((size_t)nf * cap * 32);
        std::vector<int32_t> lap(2 * (size_t)nf), n(nf), mono(nf);
        for (int f = 0; f < nf; ++f) { lap[2 * f] = laps.at(f).first; lap[2 * f + 1] = laps.at(f).second; }
        const int rc = orbx_extract_batch(h_, nf, images.data(), steps.data(), cols, rows, lap.data(), kps.data(),
                                          desc.data(), cap, n.data(), mono.data());
        if (rc != ORB_OK) throw std::runtime_error("orbx_extract_batch failed");
        keypoints.assign(nf, {});
        descriptors.assign(nf, {});
        for (int f = 0; f < nf; ++f) {
            keypoints[f].assign(kps.begin() + (size_t)f * cap, kps.begin() + (size_t)f * cap + n[f]);
            descriptors[f].rows = n[f];
            descriptors[f].data.assign(desc.begin() + (size_t)f * cap * 32, desc.begin() + ((size_t)f * cap + n[f]) * 32);
        }
        return std::vector<int>(mono.begin(), mono.end());
    }

    int GetLevels() const { return nlevels_; }
    float GetScaleFactor() const { return scaleFactor_; }
    std::vector<float> GetScaleFactors() const { return scale_; }
    std::vector<float> GetInverseScaleFactors() const { return inv_scale_; }
    std::vector<float> GetScaleSigmaSquares() const { return sigma2_; }
    std::vector<float> GetInverseScaleSigmaSquares() const { return inv_sigma2_; }

    // mvImagePyramid[level] of the last image (host copy)
    std::vector<uint8_t> ImagePyramid(int level, int* cols, int* rows) const {
        int w = 0, h = 0;
        if (orbx_get_level(h_, level, nullptr, 0, &w, &h) != ORB_OK) throw std::runtime_error("orbx_get_level");
        std::vector<uint8_t> out((size_t)w * h);
        orbx_get_level(h_, level, out.data(), w, &w, &h);
        if (cols) *cols = w;
        if (rows) *rows = h;
        return out;
    }

    orbx_handle* handle() const { return h_; }

private:
    orbx_handle* h_ = nullptr;
    int nlevels_;
    float scaleFactor_;
    std::vector<float> scale_, inv_scale_, sigma2_, inv_sigma2_;
};

// Frame::ComputeStereoMatches (src/Frame.cc:811-981) for a rectified pair whose
// images were the last inputs of `left` / `right`: fills mvuRight / mvDepth
// (-1 where unmatched).  mb = baseline, mbf = baseline * fx.
inline void ComputeStereoMatches(const ORBextractor& left, const ORBextractor& right,
                                 const std::vector<KeyPoint>& mvKeys, const Descriptors& mDescriptors,
                                 const std::vector<KeyPoint>& mvKeysRight, const Descriptors& mDescriptorsRight,
                                 float mb, float mbf, std::vector<float>& mvuRight, std::vector<float>& mvDepth) {
    mvuRight.assign(mvKeys.size(), -1.0f);
    mvDepth.assign(mvKeys.size(), -1.0f);
    const int rc = orbs_compute_stereo_matches(left.handle(), right.handle(), mvKeys.data(), (int)mvKeys.size(),
                                               mDescriptors.data.data(), mvKeysRight.data(), (int)mvKeysRight.size(),
                                               mDescriptorsRight.data.data(), mb, mbf, mvuRight.data(),
                                               mvDepth.data());
    if (rc != ORB_OK) throw std::runtime_error("ComputeStereoMatches failed");
}

class ORBmatcher {
public:
    static const int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;

    explicit ORBmatcher(float nnratio = 0.6f, bool checkOri = true) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

    static int DescriptorDistance(const uint8_t* a, const uint8_t* b) { return orbm_descriptor_distance(a, b); }

    // int SearchForInitialization(Frame &F1, Frame &F2, vector<cv::Point2f> &vbPrevMatched,
    //                             vector<int> &vnMatches12, int windowSize=10)
    int SearchForInitialization(const orbm_frame& F1, const orbm_frame& F2, std::vector<float>& vbPrevMatchedXY,
                                std::vector<int>& vnMatches12, int windowSize = 10) const {
        vnMatches12.assign(F1.n, -1);
        const int nm = orbm_search_for_initialization(&F1, &F2, vbPrevMatchedXY.data(), windowSize, mfNNratio,
                                                      mbCheckOrientation, vnMatches12.data());
        if (nm < 0) throw std::runtime_error("SearchForInitialization failed");
        return nm;
    }

    // int SearchByBoW(KeyFrame *pKF, Frame &F, vector<MapPoint*> &vpMapPointMatches)
    int SearchByBoW(const orbm_frame& KF, const orbm_featvec& KFfv, const std::vector<uint8_t>& kfMapPointValid,
                    const orbm_frame& F, const orbm_featvec& Ffv, std::vector<int>& vMatchesKFIdx) const {
        vMatchesKFIdx.assign(F.n, -1);
        const int nm = orbm_search_by_bow(&KF, &KFfv, kfMapPointValid.data(), &F, &Ffv, mfNNratio,
                                          mbCheckOrientation, vMatchesKFIdx.data());
        if (nm < 0) throw std::runtime_error("SearchByBoW failed");
        return nm;
    }

    // The relocalisation loop (Tracking.cc:3641-3648): SearchByBoW(KF_i, F) for
    // every candidate in one launch; returns the per-candidate counts and fills
    // vvMatchesKFIdx[i] like the single form.
    std::vector<int> SearchByBoW(const std::vector<const orbm_frame*>& KFs, const std::vector<const orbm_featvec*>& KFfvs,
                                 const std::vector<const uint8_t*>& kfMapPointValid, const orbm_frame& F,
                                 const orbm_featvec& Ffv, std::vector<std::vector<int>>& vvMatchesKFIdx) const {
        const int nkf = (int)KFs.size();
        std::vector<int32_t> match((size_t)nkf * F.n), counts(nkf);
        const int rc = orbm_search_by_bow_many(nkf, KFs.data(), KFfvs.data(), kfMapPointValid.data(), &F, &Ffv,
                                               mfNNratio, mbCheckOrientation, match.data(), counts.data());
        if (rc != ORB_OK) throw std::runtime_error("SearchByBoW (many) failed");
        vvMatchesKFIdx.assign(nkf, {});
        for (int i = 0; i < nkf; ++i)
            vvMatchesKFIdx[i].assign(match.begin() + (size_t)i * F.n, match.begin() + (size_t)(i + 1) * F.n);
        return std::vector<int>(counts.begin(), counts.end());
    }

    // int SearchByProjection(Frame &F, const vector<MapPoint*> &vpMapPoints, const float th=3, ...)
    int SearchByProjection(const orbm_frame& F, const orbm_mappoints& mps, std::vector<int>& owner,
                           const std::vector<uint8_t>& blocked, float th = 3, bool bFarPoints = false,
                           float thFarPoints = 50.0f) const {
        const int nm = orbm_search_by_projection_mps(&F, &mps, th, bFarPoints, thFarPoints, mfNNratio, owner.data(),
                                                     blocked.data());
        if (nm < 0) throw std::runtime_error("SearchByProjection failed");
        return nm;
    }

    // int SearchByProjection(Frame &CurrentFrame, const Frame &LastFrame, const float th, const bool bMono)
    // The caller projects the last frame's points (Tcw * X); bForwardMode: 0 none, 1 forward, 2 backward.
    int SearchByProjection(const orbm_frame& CurrentFrame, const std::vector<uint8_t>& valid,
                           const std::vector<float>& u, const std::vector<float>& v, const std::vector<float>& ur,
                           const std::vector<int32_t>& lastOctave, const std::vector<float>& lastAngle,
                           const std::vector<uint8_t>& hasObs, const uint8_t* lastDescriptors, float th,
                           int motionMode, std::vector<int>& owner, const std::vector<uint8_t>& blocked) const {
        const int nm = orbm_search_by_projection_last(&CurrentFrame, (int)valid.size(), valid.data(), u.data(),
                                                      v.data(), ur.data(), lastOctave.data(), lastAngle.data(),
                                                      hasObs.data(), lastDescriptors, th, motionMode,
                                                      mbCheckOrientation, owner.data(), blocked.data());
        if (nm < 0) throw std::runtime_error("SearchByProjection(F, LastFrame) failed");
        return nm;
    }

    // int SearchByProjection(Frame &CurrentFrame, KeyFrame* pKF, const set<MapPoint*> &sAlreadyFound,
    //                        const float th, const int ORBdist)
    int SearchByProjection(const orbm_frame& CurrentFrame, const std::vector<uint8_t>& valid,
                           const std::vector<float>& u, const std::vector<float>& v,
                           const std::vector<int32_t>& predictedLevel, const std::vector<float>& kfAngle,
                           const uint8_t* mapPointDescriptors, float th, int ORBdist, std::vector<int>& owner) const {
        const int nm = orbm_search_by_projection_kf(&CurrentFrame, (int)valid.size(), valid.data(), u.data(), v.data(),
                                                    predictedLevel.data(), kfAngle.data(), mapPointDescriptors, th,
                                                    ORBdist, mbCheckOrientation, owner.data());
        if (nm < 0) throw std::runtime_error("SearchByProjection(F, KF) failed");
        return nm;
    }

    // int SearchByProjection(KeyFrame* pKF, Sophus::Sim3<float> &Scw, const vector<MapPoint*> &vpPoints,
    //                        vector<MapPoint*> &vpMatched, int th, float ratioHamming=1.0)
    // (and the vpPointsKFs variant: vpMatchedKF[idx] = vpPointsKFs[vMatched[idx]] for new matches)
    int SearchByProjection(const orbm_frame& KF, const std::vector<uint8_t>& valid, const std::vector<float>& u,
                           const std::vector<float>& v, const std::vector<int32_t>& predictedLevel,
                           const uint8_t* mapPointDescriptors, std::vector<int>& vMatched, int th,
                           float ratioHamming = 1.0f) const {
        const int nm = orbm_search_by_projection_sim3(&KF, (int)valid.size(), valid.data(), u.data(), v.data(),
                                                      predictedLevel.data(), mapPointDescriptors, (float)th,
                                                      ratioHamming, vMatched.data());
        if (nm < 0) throw std::runtime_error("SearchByProjection(KF, Sim3) failed");
        return nm;
    }

    // int SearchByBoW(KeyFrame *pKF1, KeyFrame* pKF2, vector<MapPoint*> &vpMatches12)
    int SearchByBoW(const orbm_frame& KF1, const orbm_featvec& fv1, const std::vector<uint8_t>& valid1,
                    const orbm_frame& KF2, const orbm_featvec& fv2, const std::vector<uint8_t>& valid2,
                    std::vector<int>& vMatches12) const {
        vMatches12.assign(KF1.n, -1);
        const int nm = orbm_search_by_bow_kf(&KF1, &fv1, valid1.data(), &KF2, &fv2, valid2.data(), mfNNratio,
                                             mbCheckOrientation, vMatches12.data());
        if (nm < 0) throw std::runtime_error("SearchByBoW(KF1, KF2) failed");
        return nm;
    }

    // int SearchForTriangulation(KeyFrame *pKF1, KeyFrame* pKF2, vector<pair<size_t, size_t> > &vMatchedPairs,
    //                            const bool bOnlyStereo, const bool bCoarse = false)
    int SearchForTriangulation(const orbm_frame& KF1, const orbm_featvec& fv1, const std::vector<uint8_t>& hasMP1,
                               const orbm_frame& KF2, const orbm_featvec& fv2, const std::vector<uint8_t>& hasMP2,
                               const float F12[9], float epx, float epy, const std::vector<float>& levelSigma2_2,
                               std::vector<std::pair<size_t, size_t>>& vMatchedPairs, bool bOnlyStereo,
                               bool bCoarse = false) const {
        std::vector<int32_t> m12(KF1.n, -1);
        const int nm = orbm_search_for_triangulation(&KF1, &fv1, hasMP1.data(), &KF2, &fv2, hasMP2.data(), F12, epx,
                                                     epy, levelSigma2_2.data(), bOnlyStereo, bCoarse,
                                                     mbCheckOrientation, 1, m12.data());
        if (nm < 0) throw std::runtime_error("SearchForTriangulation failed");
        vMatchedPairs.clear();
        for (int i = 0; i < KF1.n; ++i)
            if (m12[i] >= 0) vMatchedPairs.emplace_back((size_t)i, (size_t)m12[i]);
        return nm;
    }

    // The same for KannalaBrandt8 / two-camera keyframes: `check(idx1, idx2)` is
    // the reference's per-candidate geometry (epipole test + the selected camera
    // pair's epipolarConstrain, src/ORBmatcher.cc:1014-1076), e.g. a lambda over
    // pKF1/pKF2 calling pCamera1->epipolarConstrain(pCamera2, kp1, kp2, R12, t12, ...).
    int SearchForTriangulation(const orbm_frame& KF1, const orbm_featvec& fv1, const std::vector<uint8_t>& hasMP1,
                               const orbm_frame& KF2, const orbm_featvec& fv2, const std::vector<uint8_t>& hasMP2,
                               const std::function<bool(int, int)>& check,
                               std::vector<std::pair<size_t, size_t>>& vMatchedPairs, bool bOnlyStereo) const {
        std::vector<int32_t> m12(KF1.n, -1);
        auto tramp = [](void* ctx, int i1, int i2) -> int {
            return (*static_cast<const std::function<bool(int, int)>*>(ctx))(i1, i2) ? 1 : 0;
        };
        const int nm = orbm_search_for_triangulation_checked(&KF1, &fv1, hasMP1.data(), &KF2, &fv2, hasMP2.data(),
                                                             bOnlyStereo, mbCheckOrientation, tramp,
                                                             const_cast<std::function<bool(int, int)>*>(&check),
                                                             m12.data());
        if (nm < 0) throw std::runtime_error("SearchForTriangulation (checked) failed");
        vMatchedPairs.clear();
        for (int i = 0; i < KF1.n; ++i)
            if (m12[i] >= 0) vMatchedPairs.emplace_back((size_t)i, (size_t)m12[i]);
        return nm;
    }

    // int SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*> &vpMatches12, const Sophus::Sim3f &S12,
    //                  const float th) -- new mutual matches only (vNewMatches12[i1] = KF2 feature or -1)
    int SearchBySim3(const orbm_frame& KF1, const orbm_frame& KF2, const std::vector<uint8_t>& valid1,
                     const std::vector<float>& u1, const std::vector<float>& v1, const std::vector<int32_t>& level1,
                     const uint8_t* desc1, const std::vector<uint8_t>& valid2, const std::vector<float>& u2,
                     const std::vector<float>& v2, const std::vector<int32_t>& level2, const uint8_t* desc2,
                     float th, std::vector<int>& vNewMatches12) const {
        vNewMatches12.assign(KF1.n, -1);
        const int nf = orbm_search_by_sim3(&KF1, &KF2, valid1.data(), u1.data(), v1.data(), level1.data(), desc1,
                                           valid2.data(), u2.data(), v2.data(), level2.data(), desc2, th,
                                           vNewMatches12.data());
        if (nf < 0) throw std::runtime_error("SearchBySim3 failed");
        return nf;
    }

    // int Fuse(KeyFrame* pKF, const vector<MapPoint *> &vpMapPoints, const float th=3.0, const bool bRight=false)
    // -- the matching; the caller replaces / adds in index order from vBestIdx.
    static int Fuse(const orbm_frame& KF, const std::vector<float>& invLevelSigma2, const std::vector<uint8_t>& valid,
                    const std::vector<float>& u, const std::vector<float>& v, const std::vector<float>& ur,
                    const std::vector<int32_t>& level, const uint8_t* desc, std::vector<int>& vBestIdx,
                    std::vector<int>& vBestDist, float th = 3.0f) {
        vBestIdx.resize(valid.size());
        vBestDist.resize(valid.size());
        const int nf = orbm_fuse(&KF, invLevelSigma2.data(), (int)valid.size(), valid.data(), u.data(), v.data(),
                                 ur.data(), level.data(), desc, th, 1, vBestIdx.data(), vBestDist.data());
        if (nf < 0) throw std::runtime_error("Fuse failed");
        return nf;
    }

    // int Fuse(KeyFrame* pKF, Sophus::Sim3f &Scw, const vector<MapPoint*> &vpPoints, float th,
    //          vector<MapPoint *> &vpReplacePoint) -- the matching, as above
    static int Fuse(const orbm_frame& KF, const std::vector<uint8_t>& valid, const std::vector<float>& u,
                    const std::vector<float>& v, const std::vector<int32_t>& level, const uint8_t* desc, float th,
                    std::vector<int>& vBestIdx, std::vector<int>& vBestDist) {
        vBestIdx.resize(valid.size());
        vBestDist.resize(valid.size());
        const int nf = orbm_fuse_sim3(&KF, (int)valid.size(), valid.data(), u.data(), v.data(), level.data(), desc,
                                      th, vBestIdx.data(), vBestDist.data());
        if (nf < 0) throw std::runtime_error("Fuse(KF, Sim3) failed");
        return nf;
    }

    float mfNNratio;
    bool mbCheckOrientation;
};

}  // namespace ORB_SLAM3_MI355X
