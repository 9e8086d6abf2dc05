/**
 * Drop-in bodies of the ORB_SLAM3::ORBmatcher searches on the Tracking
 * thread's per-frame path, over the MI355X C ABI (include/orb_mi355x.h):
 *
 *   SearchForInitialization(F1, F2, ...)        src/ORBmatcher.cc:648-763
 *   SearchByBoW(KeyFrame*, Frame&, ...)         src/ORBmatcher.cc:223-425
 *   SearchByProjection(Frame&, MapPoints, ...)  src/ORBmatcher.cc:43-221
 *   SearchByProjection(Frame&, const Frame&, ..) src/ORBmatcher.cc:1676-1887
 *
 * Delete those four bodies from the reference's src/ORBmatcher.cc and add this
 * file to the library sources; the class declaration (include/ORBmatcher.h:36-103)
 * is unchanged.  The adapter reads the map under the reference's own locks
 * (MapPoint accessors), does the per-point pose math (Sophus) on the host
 * exactly as the reference writes it, hands flat snapshots to the device, and
 * writes MapPoint pointers back from the returned indices.
 *
 * Both camera set-ups of the reference are handled: a pinhole / rectified
 * frame (Nleft == -1: mvKeysUn, the stereo gate on mvuRight) and a fisheye
 * stereo frame (Nleft != -1: keypoints indexed as [mvKeys; mvKeysRight],
 * Frame.cc:1069-1071, with the right camera's grid, stereo partners and
 * projections, ORBmatcher.cc:131-209, :1794-1860).
 *
 * The other ten search / Fuse bodies (the mapping and loop-closing threads and
 * relocalisation's projection) are in ORBmatcher_mapping.cc; the helpers both
 * files share are in ORBmatcher_adapter.h.
 *
 * tests/test_adapter.py compiles this file (g++ -fsyntax-only) against the
 * reference's unmodified ORBmatcher.h / Frame.h / KeyFrame.h / MapPoint.h and
 * their includes, with declaration-only stand-ins for the third-party headers
 * the image lacks (OpenCV, Eigen, Sophus, g2o, boost serialization, Pangolin;
 * tests/native/decl/); the extractor adapter next to it is compiled against
 * the reference header and run on the GPU (tests/test_gpu_adapter.py); the ABI
 * calls here are those of tests/native/cpp_api_test.cpp, which runs on the GPU.
 */
#include "ORBmatcher_adapter.h"

#include <vector>

using namespace std;

namespace ORB_SLAM3
{

using namespace mi355x_adapter;

int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, vector<cv::Point2f>& vbPrevMatched,
                                        vector<int>& vnMatches12, int windowSize)
{
    vnMatches12 = vector<int>(F1.mvKeysUn.size(), -1);
    vector<cv::KeyPoint> s1, s2;
    orbm_frame f1 = view(F1, -1, s1), f2 = view(F2, -1, s2);     // monocular initialization: mvKeysUn
    static_assert(sizeof(cv::Point2f) == 2 * sizeof(float), "Point2f is two floats");
    const int n = orbm_search_for_initialization(&f1, &f2, reinterpret_cast<float*>(vbPrevMatched.data()),
                                                 windowSize, mfNNratio, mbCheckOrientation ? 1 : 0,
                                                 vnMatches12.data());
    check(n, "SearchForInitialization");
    return n;   // vbPrevMatched updated in place as :753-756 does
}

int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches)
{
    const vector<MapPoint*> vpMapPointsKF = pKF->GetMapPointMatches();
    vpMapPointMatches = vector<MapPoint*>(F.N, static_cast<MapPoint*>(NULL));
    vector<uint8_t> valid(vpMapPointsKF.size());
    for (size_t i = 0; i < vpMapPointsKF.size(); ++i)
        valid[i] = vpMapPointsKF[i] && !vpMapPointsKF[i]->isBad();   // :262-268
    FeatVecCSR kfv(pKF->mFeatVec), fv(F.mFeatVec);
    // keypoints for the rotation check (:290-292, :349-351): the keyframe's
    // mvKeysUn, or its [mvKeys; mvKeysRight] when it has a second camera; the
    // frame's combined array when it is a fisheye stereo frame
    vector<cv::KeyPoint> skf, sf;
    orbm_frame kf = view(*pKF, pKF->mpCamera2 ? pKF->NLeft : -1, skf), f = view(F, F.Nleft, sf);
    vector<int32_t> match(F.N, -1);
    const int n = F.Nleft == -1
                      ? orbm_search_by_bow(&kf, &kfv.c, valid.data(), &f, &fv.c, mfNNratio,
                                           mbCheckOrientation ? 1 : 0, match.data())
                      : orbm_search_by_bow_fisheye(&kf, &kfv.c, valid.data(), &f, &fv.c, F.Nleft, mfNNratio,
                                                   mbCheckOrientation ? 1 : 0, match.data());
    check(n, "SearchByBoW");
    for (int i = 0; i < F.N; ++i)
        if (match[i] >= 0) vpMapPointMatches[i] = vpMapPointsKF[match[i]];
    return n;
}

int ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints, const float th,
                                   const bool bFarPoints, const float thFarPoints)
{
    const int n = (int)vpMapPoints.size();
    const bool fisheye = F.Nleft != -1;
    // MapPoint snapshot (the fields :50-75 and, for a fisheye frame, the right
    // camera's :131-140 read, under the MapPoint's locks)
    vector<float> px(n), py(n), pxr(n), vcos(n), depth(n);
    vector<int32_t> level(n);
    vector<uint8_t> in_view(n), has_obs(n), desc((size_t)n * 32);
    vector<float> rx, ry, rcos;
    vector<int32_t> rlevel;
    vector<uint8_t> rin_view;
    if (fisheye) {
        rx.resize(n); ry.resize(n); rcos.resize(n); rlevel.resize(n); rin_view.resize(n);
    }
    for (int i = 0; i < n; ++i) {
        MapPoint* pMP = vpMapPoints[i];
        const bool bad = pMP->isBad();
        in_view[i] = pMP->mbTrackInView && !bad;
        px[i] = pMP->mTrackProjX; py[i] = pMP->mTrackProjY; pxr[i] = pMP->mTrackProjXR;
        level[i] = pMP->mnTrackScaleLevel; vcos[i] = pMP->mTrackViewCos; depth[i] = pMP->mTrackDepth;
        has_obs[i] = pMP->Observations() > 0;
        if (fisheye) {
            rin_view[i] = pMP->mbTrackInViewR && !bad;
            rx[i] = pMP->mTrackProjXR; ry[i] = pMP->mTrackProjYR;
            rlevel[i] = pMP->mnTrackScaleLevelR; rcos[i] = pMP->mTrackViewCosR;
        }
        if (in_view[i] || (fisheye && rin_view[i])) {
            const cv::Mat d = pMP->GetDescriptor();
            std::copy(d.data, d.data + 32, desc.begin() + (size_t)i * 32);
        }
    }
    orbm_mappoints mps{n, px.data(), py.data(), pxr.data(), level.data(), vcos.data(), depth.data(),
                       in_view.data(), has_obs.data(), desc.data()};
    // slots that already hold a MapPoint: opaque owner, blocked when observed (:86-88, :155-157)
    vector<int32_t> owner(F.N, -1);
    vector<uint8_t> blocked(F.N, 0);
    for (int i = 0; i < F.N; ++i)
        if (F.mvpMapPoints[i]) { owner[i] = -2; blocked[i] = F.mvpMapPoints[i]->Observations() > 0; }
    vector<cv::KeyPoint> store;
    orbm_frame f = view(F, F.Nleft, store);
    int nm;
    if (!fisheye) {
        nm = orbm_search_by_projection_mps(&f, &mps, th, bFarPoints ? 1 : 0, thFarPoints, mfNNratio, owner.data(),
                                           blocked.data());
    } else {
        // left camera, then the right camera's grid by local index; a match
        // also claims its stereo partner (mvLeftToRightMatch / mvRightToLeftMatch)
        orbm_mappoints_right mpr{rin_view.data(), rx.data(), ry.data(), rlevel.data(), rcos.data()};
        nm = orbm_search_by_projection_mps_fisheye(&f, F.Nleft, F.mvLeftToRightMatch.data(),
                                                   F.mvRightToLeftMatch.data(), &mps, &mpr, th, bFarPoints ? 1 : 0,
                                                   thFarPoints, mfNNratio, owner.data(), blocked.data());
    }
    check(nm, "SearchByProjection(F, MapPoints)");
    for (int i = 0; i < F.N; ++i)
        if (owner[i] >= 0) F.mvpMapPoints[i] = vpMapPoints[owner[i]];
    return nm;
}

int ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono)
{
    const bool fisheye = CurrentFrame.Nleft != -1;
    // the pose math of :1686-1720 (and :1794-1796 for the right camera), per
    // last-frame point, unchanged
    const Sophus::SE3f Tcw = CurrentFrame.GetPose();
    const Eigen::Vector3f twc = Tcw.inverse().translation();
    const Sophus::SE3f Tlw = LastFrame.GetPose();
    const Eigen::Vector3f tlc = Tlw * twc;
    const bool bForward = tlc(2) > CurrentFrame.mb && !bMono;
    const bool bBackward = -tlc(2) > CurrentFrame.mb && !bMono;
    Sophus::SE3f Trl;
    if (fisheye) Trl = CurrentFrame.GetRelativePoseTrl();

    const int n = LastFrame.N;
    vector<uint8_t> valid(n, 0), has_obs(n, 0), desc((size_t)n * 32, 0);
    vector<float> u(n, 0.f), v(n, 0.f), ur(n, 0.f), vr(n, 0.f), angle(n, 0.f);
    vector<int32_t> octave(n, 0);
    for (int i = 0; i < n; ++i) {
        MapPoint* pMP = LastFrame.mvpMapPoints[i];
        if (!pMP || LastFrame.mvbOutlier[i]) continue;
        const Eigen::Vector3f x3Dc = Tcw * pMP->GetWorldPos();
        const float invzc = 1.0 / x3Dc(2);
        if (invzc < 0) continue;
        const Eigen::Vector2f uv = CurrentFrame.mpCamera->project(x3Dc);
        if (uv(0) < CurrentFrame.mnMinX || uv(0) > CurrentFrame.mnMaxX) continue;
        if (uv(1) < CurrentFrame.mnMinY || uv(1) > CurrentFrame.mnMaxY) continue;
        valid[i] = 1;
        u[i] = uv(0); v[i] = uv(1);
        // the last frame's keypoint of point i (:1721-1722, :1775-1777)
        const bool right_kp = LastFrame.Nleft != -1 && i >= LastFrame.Nleft;
        const cv::KeyPoint& kpo = right_kp ? LastFrame.mvKeysRight[i - LastFrame.Nleft] : LastFrame.mvKeys[i];
        const cv::KeyPoint& kpa = LastFrame.Nleft == -1 ? LastFrame.mvKeysUn[i] : kpo;
        octave[i] = kpo.octave;
        angle[i] = kpa.angle;
        if (fisheye) {
            // the right camera's projection (:1795-1796: the reference projects
            // with mpCamera)
            const Eigen::Vector3f x3Dr = Trl * x3Dc;
            const Eigen::Vector2f uvr = CurrentFrame.mpCamera->project(x3Dr);
            ur[i] = uvr(0); vr[i] = uvr(1);
        } else {
            ur[i] = uv(0) - CurrentFrame.mbf * invzc;   // :1763
        }
        // a slot this point claims blocks later points iff it is observed (:1747-1749)
        has_obs[i] = pMP->Observations() > 0;
        const cv::Mat d = pMP->GetDescriptor();
        std::copy(d.data, d.data + 32, desc.begin() + (size_t)i * 32);
    }
    vector<int32_t> owner(CurrentFrame.N, -1);
    vector<uint8_t> blocked(CurrentFrame.N, 0);
    for (int i = 0; i < CurrentFrame.N; ++i)
        if (CurrentFrame.mvpMapPoints[i]) {
            owner[i] = -2;
            blocked[i] = CurrentFrame.mvpMapPoints[i]->Observations() > 0;
        }
    vector<cv::KeyPoint> store;
    orbm_frame cur = view(CurrentFrame, CurrentFrame.Nleft, store);
    const int mode = bForward ? 1 : (bBackward ? 2 : 0);
    const int nm = !fisheye
                       ? orbm_search_by_projection_last(&cur, n, valid.data(), u.data(), v.data(), ur.data(),
                                                        octave.data(), angle.data(), has_obs.data(), desc.data(), th,
                                                        mode, mbCheckOrientation ? 1 : 0, owner.data(), blocked.data())
                       : orbm_search_by_projection_last_fisheye(&cur, CurrentFrame.Nleft, n, valid.data(), u.data(),
                                                                v.data(), ur.data(), vr.data(), octave.data(),
                                                                angle.data(), has_obs.data(), desc.data(), th, mode,
                                                                mbCheckOrientation ? 1 : 0, owner.data(),
                                                                blocked.data());
    check(nm, "SearchByProjection(F, LastFrame)");
    for (int i = 0; i < CurrentFrame.N; ++i)
        if (owner[i] >= 0) CurrentFrame.mvpMapPoints[i] = LastFrame.mvpMapPoints[owner[i]];
    return nm;
}

}  // namespace ORB_SLAM3
