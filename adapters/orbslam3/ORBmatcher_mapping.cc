/**
 * Drop-in bodies of the ORB_SLAM3::ORBmatcher searches off the Tracking
 * thread's per-frame path, over the MI355X C ABI (include/orb_mi355x.h):
 *
 *   SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist)
 *                                   src/ORBmatcher.cc:1889-2010  (Tracking::Relocalization, Tracking.cc:3726,3740)
 *   SearchByProjection(KeyFrame*, Sim3, vpPoints, vpMatched, th, ratioHamming)
 *                                   :427-532   (LoopClosing.cc:2133,2178)
 *   SearchByProjection(KeyFrame*, Sim3, vpPoints, vpPointsKFs, vpMatched, vpMatchedKF, th, ratioHamming)
 *                                   :534-646   (LoopClosing.cc:662,755,777)
 *   SearchByBoW(KeyFrame*, KeyFrame*, vpMatches12)
 *                                   :765-905   (LoopClosing.cc)
 *   SearchForTriangulation(pKF1, pKF2, vMatchedPairs, bOnlyStereo, bCoarse)
 *                                   :907-1146  (LocalMapping.cc:466)
 *   SearchBySim3(pKF1, pKF2, vpMatches12, S12, th)
 *                                   :1457-1674 (LoopClosing.cc:964)
 *   Fuse(pKF, vpMapPoints, th, bRight)
 *                                   :1148-1331 (LocalMapping.cc:772-803)
 *   Fuse(pKF, Scw, vpPoints, th, vpReplacePoint)
 *                                   :1340-1455 (LoopClosing)
 *   DescriptorDistance(a, b)        :2058-2074
 *
 * With ORBmatcher_searches.cc (the four per-frame searches) every Search* and
 * Fuse body of src/ORBmatcher.cc is replaced; the reference file keeps only the
 * constructor, RadiusByViewingCos, ComputeThreeMaxima and the TH_* constants.
 * The class declaration (include/ORBmatcher.h:36-103) is unchanged.
 *
 * Division of work, as in the per-frame searches: the per-point geometry
 * (Sophus / Eigen poses, the camera's project(), IsInImage, the distance
 * invariance, the viewing angle, PredictScale) runs here on the host exactly
 * as the reference writes it, reading the map under the reference's own locks;
 * the flat snapshot goes to the device, which does every window and Hamming
 * search and the rotation filters; the results are written back here.  Map
 * mutations (Fuse's Replace / AddObservation) stay here, in the reference's
 * index order, and a point whose state an earlier decision changed is
 * re-snapshotted and re-searched before its own decision (Fuse below), so the
 * result is the reference's sequential one.
 *
 * Camera set-ups: the pinhole / rectified keyframe (NLeft == -1), and the
 * fisheye stereo keyframe (NLeft != -1): searches that read mGrid without
 * bRight see the left keypoints only (left_grid_view), Fuse(..., bRight) sees
 * the right camera (camera_view), SearchByBoW(KF, KF) skips the indices past
 * mvKeysUn (:799-801, :816-818) through its validity masks, and
 * SearchForTriangulation between KannalaBrandt8 or two-camera keyframes takes
 * the reference's own epipolarConstrain per candidate through
 * orbm_search_for_triangulation_checked.
 *
 * tests/test_adapter.py compiles this file (g++ -fsyntax-only -Wall -Wextra)
 * against the reference's unmodified headers, like ORBmatcher_searches.cc.
 */
#include "ORBmatcher_adapter.h"
#include "ORBmatcher_tails.h"

#include <set>
#include <tuple>
#include <utility>
#include <vector>

using namespace std;

namespace ORB_SLAM3
{

using namespace mi355x_adapter;

using mi355x_tails::PointRows;

namespace
{
// ---- SearchByProjection(KeyFrame*, Sim3, ...) :446-486 / :558-604 and
// Fuse(KeyFrame*, Sim3, ...) :1372-1411: the candidate geometry of one point.
// project_with_camera: pKF->mpCamera->project (:463, :1385); otherwise the
// pinhole formula the vpPointsKFs variant writes out (:573-578).
bool sim3_point(KeyFrame* pKF, MapPoint* pMP, const Sophus::SE3f& Tcw, const Eigen::Vector3f& Ow,
                bool project_with_camera, float& u, float& v, int& level)
{
    // Get 3D Coords.
    Eigen::Vector3f p3Dw = pMP->GetWorldPos();
    // Transform into Camera Coords.
    Eigen::Vector3f p3Dc = Tcw * p3Dw;
    // Depth must be positive
    if (p3Dc(2) < 0.0) return false;
    if (project_with_camera) {
        const Eigen::Vector2f uv = pKF->mpCamera->project(p3Dc);
        u = uv(0);
        v = uv(1);
    } else {
        const float invz = 1 / p3Dc(2);
        const float x = p3Dc(0) * invz;
        const float y = p3Dc(1) * invz;
        u = pKF->fx * x + pKF->cx;
        v = pKF->fy * y + pKF->cy;
    }
    // Point must be inside the image
    if (!pKF->IsInImage(u, v)) return false;
    // Depth must be inside the scale invariance region of the point
    const float maxDistance = pMP->GetMaxDistanceInvariance();
    const float minDistance = pMP->GetMinDistanceInvariance();
    Eigen::Vector3f PO = p3Dw - Ow;
    const float dist = PO.norm();
    if (dist < minDistance || dist > maxDistance) return false;
    // Viewing angle must be less than 60 deg
    Eigen::Vector3f Pn = pMP->GetNormal();
    if (PO.dot(Pn) < 0.5 * dist) return false;
    level = pMP->PredictScale(dist, pKF);
    return true;
}

// Both Sim3 projections (:427-646): the shared body.  vpMatchedKF / vpPointsKFs
// are null for the first form.
int sim3_projection(KeyFrame* pKF, Sophus::Sim3f& Scw, const vector<MapPoint*>& vpPoints,
                    const vector<KeyFrame*>* vpPointsKFs, vector<MapPoint*>& vpMatched,
                    vector<KeyFrame*>* vpMatchedKF, int th, float ratioHamming, bool project_with_camera)
{
    Sophus::SE3f Tcw = Sophus::SE3f(Scw.rotationMatrix(), Scw.translation() / Scw.scale());
    Eigen::Vector3f Ow = Tcw.inverse().translation();
    // Set of MapPoints already found in the KeyFrame
    set<MapPoint*> spAlreadyFound(vpMatched.begin(), vpMatched.end());
    spAlreadyFound.erase(static_cast<MapPoint*>(NULL));

    const size_t n = vpPoints.size();
    PointRows pr(n);
    for (size_t i = 0; i < n; ++i) {
        MapPoint* pMP = vpPoints[i];
        // Discard Bad MapPoints and already found
        if (pMP->isBad() || spAlreadyFound.count(pMP)) continue;
        int level = 0;
        if (!sim3_point(pKF, pMP, Tcw, Ow, project_with_camera, pr.u[i], pr.v[i], level)) continue;
        pr.valid[i] = 1;
        pr.level[i] = level;
        copy_descriptor(pMP, pr.desc, i);
    }
    // slots: -1 = vpMatched[idx] NULL, -2 = occupied; the device writes the
    // point index into the slots it fills, in the reference's point order
    vector<int32_t> matched = mi355x_tails::slot_states(vpMatched);
    vector<cv::KeyPoint> store;
    orbm_frame kf = left_grid_view(*pKF, pKF->NLeft, store);
    check(kf.n == (int32_t)vpMatched.size() ? 0 : ORB_ERR_PARAM, "SearchByProjection(KF, Sim3): vpMatched size");
    const int nm = orbm_search_by_projection_sim3(&kf, (int)n, pr.valid.data(), pr.u.data(), pr.v.data(),
                                                  pr.level.data(), pr.desc.data(), (float)th, ratioHamming,
                                                  matched.data());
    check(nm, "SearchByProjection(KF, Sim3)");
    mi355x_tails::slot_writeback(matched, vpPoints, vpPointsKFs, vpMatched, vpMatchedKF);
    return nm;
}

// ---- SearchForTriangulation's per-candidate geometry (:1004-1069) for the
// keyframes whose epipolar test the device does not run.
struct TriCtx {
    KeyFrame *k1, *k2;
    Eigen::Vector2f ep;
    bool coarse;
    Eigen::Matrix3f R12, Rll, Rlr, Rrl, Rrr;
    Eigen::Vector3f t12, tll, tlr, trl, trr;
};

const cv::KeyPoint& tri_kp(KeyFrame* k, size_t idx)
{
    return (k->NLeft == -1) ? k->mvKeysUn[idx]
                            : (idx < (size_t)k->NLeft) ? k->mvKeys[idx] : k->mvKeysRight[idx - k->NLeft];
}

int tri_check(void* p, int i1, int i2)
{
    TriCtx& c = *static_cast<TriCtx*>(p);
    KeyFrame* pKF1 = c.k1;
    KeyFrame* pKF2 = c.k2;
    const size_t idx1 = (size_t)i1, idx2 = (size_t)i2;
    const bool bStereo1 = (!pKF1->mpCamera2 && pKF1->mvuRight[idx1] >= 0);
    const bool bStereo2 = (!pKF2->mpCamera2 && pKF2->mvuRight[idx2] >= 0);
    const cv::KeyPoint& kp1 = tri_kp(pKF1, idx1);
    const cv::KeyPoint& kp2 = tri_kp(pKF2, idx2);
    const bool bRight1 = (pKF1->NLeft == -1 || idx1 < (size_t)pKF1->NLeft) ? false : true;
    const bool bRight2 = (pKF2->NLeft == -1 || idx2 < (size_t)pKF2->NLeft) ? false : true;
    if (!bStereo1 && !bStereo2 && !pKF1->mpCamera2) {
        const float distex = c.ep(0) - kp2.pt.x;
        const float distey = c.ep(1) - kp2.pt.y;
        if (distex * distex + distey * distey < 100 * pKF2->mvScaleFactors[kp2.octave]) return 0;
    }
    GeometricCamera* pCamera1 = pKF1->mpCamera;
    GeometricCamera* pCamera2 = pKF2->mpCamera;
    Eigen::Matrix3f R12 = c.R12;
    Eigen::Vector3f t12 = c.t12;
    if (pKF1->mpCamera2 && pKF2->mpCamera2) {
        if (bRight1 && bRight2) {
            R12 = c.Rrr; t12 = c.trr; pCamera1 = pKF1->mpCamera2; pCamera2 = pKF2->mpCamera2;
        } else if (bRight1 && !bRight2) {
            R12 = c.Rrl; t12 = c.trl; pCamera1 = pKF1->mpCamera2; pCamera2 = pKF2->mpCamera;
        } else if (!bRight1 && bRight2) {
            R12 = c.Rlr; t12 = c.tlr; pCamera1 = pKF1->mpCamera; pCamera2 = pKF2->mpCamera2;
        } else {
            R12 = c.Rll; t12 = c.tll; pCamera1 = pKF1->mpCamera; pCamera2 = pKF2->mpCamera;
        }
    }
    return (c.coarse || pCamera1->epipolarConstrain(pCamera2, kp1, kp2, R12, t12, pKF1->mvLevelSigma2[kp1.octave],
                                                     pKF2->mvLevelSigma2[kp2.octave]))
               ? 1
               : 0;
}

bool is_pinhole(GeometricCamera* cam) { return cam && cam->GetType() == GeometricCamera::CAM_PINHOLE; }

// ---- Fuse(pKF, vpMapPoints, th, bRight) :1180-1240: one point's row.
bool fuse_point(KeyFrame* pKF, MapPoint* pMP, const Sophus::SE3f& Tcw, const Eigen::Vector3f& Ow,
                GeometricCamera* pCamera, float& u, float& v, float& ur, int& level)
{
    if (!pMP || pMP->isBad() || pMP->IsInKeyFrame(pKF)) return false;
    Eigen::Vector3f p3Dw = pMP->GetWorldPos();
    Eigen::Vector3f p3Dc = Tcw * p3Dw;
    // Depth must be positive
    if (p3Dc(2) < 0.0f) return false;
    const float invz = 1 / p3Dc(2);
    const Eigen::Vector2f uv = pCamera->project(p3Dc);
    // Point must be inside the image
    if (!pKF->IsInImage(uv(0), uv(1))) return false;
    u = uv(0);
    v = uv(1);
    ur = uv(0) - pKF->mbf * invz;
    const float maxDistance = pMP->GetMaxDistanceInvariance();
    const float minDistance = pMP->GetMinDistanceInvariance();
    Eigen::Vector3f PO = p3Dw - Ow;
    const float dist3D = PO.norm();
    // Depth must be inside the scale pyramid of the image
    if (dist3D < minDistance || dist3D > maxDistance) return false;
    // Viewing angle must be less than 60 deg
    Eigen::Vector3f Pn = pMP->GetNormal();
    if (PO.dot(Pn) < 0.5 * dist3D) return false;
    level = pMP->PredictScale(dist3D, pKF);
    return true;
}
}  // namespace

int ORBmatcher::DescriptorDistance(const cv::Mat& a, const cv::Mat& b)
{
    return orbm_descriptor_distance(a.data, b.data);
}

int ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>& sAlreadyFound,
                                   const float th, const int ORBdist)
{
    const Sophus::SE3f Tcw = CurrentFrame.GetPose();
    Eigen::Vector3f Ow = Tcw.inverse().translation();
    const vector<MapPoint*> vpMPs = pKF->GetMapPointMatches();
    const size_t n = vpMPs.size();
    PointRows pr(n);
    vector<float> kf_angle(n, 0.f);
    for (size_t i = 0; i < n; ++i) {
        MapPoint* pMP = vpMPs[i];
        if (!pMP || pMP->isBad() || sAlreadyFound.count(pMP)) continue;
        // Project (:1913-1922)
        Eigen::Vector3f x3Dw = pMP->GetWorldPos();
        Eigen::Vector3f x3Dc = Tcw * x3Dw;
        const Eigen::Vector2f uv = CurrentFrame.mpCamera->project(x3Dc);
        if (uv(0) < CurrentFrame.mnMinX || uv(0) > CurrentFrame.mnMaxX) continue;
        if (uv(1) < CurrentFrame.mnMinY || uv(1) > CurrentFrame.mnMaxY) continue;
        // Compute predicted scale level (:1924-1934)
        Eigen::Vector3f PO = x3Dw - Ow;
        float dist3D = PO.norm();
        const float maxDistance = pMP->GetMaxDistanceInvariance();
        const float minDistance = pMP->GetMinDistanceInvariance();
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        pr.valid[i] = 1;
        pr.u[i] = uv(0);
        pr.v[i] = uv(1);
        pr.level[i] = pMP->PredictScale(dist3D, &CurrentFrame);
        copy_descriptor(pMP, pr.desc, i);
        // the keyframe keypoint's angle of the rotation check (:1972): mvKeysUn[i]
        // (for a fisheye keyframe's right slots, past mvKeysUn, the right keypoint)
        kf_angle[i] = i < pKF->mvKeysUn.size() ? pKF->mvKeysUn[i].angle
                                               : pKF->mvKeysRight[i - (size_t)pKF->NLeft].angle;
    }
    // -1: mvpMapPoints[i2] NULL (a candidate), -2: occupied (:1949-1950)
    vector<int32_t> owner = mi355x_tails::slot_states(CurrentFrame.mvpMapPoints);
    vector<cv::KeyPoint> store;
    orbm_frame f = left_grid_view(CurrentFrame, CurrentFrame.Nleft, store);
    const int nm = orbm_search_by_projection_kf(&f, (int)n, pr.valid.data(), pr.u.data(), pr.v.data(), pr.level.data(),
                                                kf_angle.data(), pr.desc.data(), th, ORBdist,
                                                mbCheckOrientation ? 1 : 0, owner.data());
    check(nm, "SearchByProjection(F, KF)");
    mi355x_tails::slot_writeback<MapPoint, KeyFrame*>(owner, vpMPs, nullptr, CurrentFrame.mvpMapPoints, nullptr);
    return nm;
}

int ORBmatcher::SearchByProjection(KeyFrame* pKF, Sophus::Sim3f& Scw, const vector<MapPoint*>& vpPoints,
                                   vector<MapPoint*>& vpMatched, int th, float ratioHamming)
{
    return sim3_projection(pKF, Scw, vpPoints, nullptr, vpMatched, nullptr, th, ratioHamming, true);
}

int ORBmatcher::SearchByProjection(KeyFrame* pKF, Sophus::Sim3<float>& Scw, const std::vector<MapPoint*>& vpPoints,
                                   const std::vector<KeyFrame*>& vpPointsKFs, std::vector<MapPoint*>& vpMatched,
                                   std::vector<KeyFrame*>& vpMatchedKF, int th, float ratioHamming)
{
    return sim3_projection(pKF, Scw, vpPoints, &vpPointsKFs, vpMatched, &vpMatchedKF, th, ratioHamming, false);
}

int ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12)
{
    const vector<MapPoint*> vpMapPoints1 = pKF1->GetMapPointMatches();
    const vector<MapPoint*> vpMapPoints2 = pKF2->GetMapPointMatches();
    vpMatches12 = vector<MapPoint*>(vpMapPoints1.size(), static_cast<MapPoint*>(NULL));
    // a feature takes part iff its MapPoint is set and good (:803-808,
    // :822-827) and, for a two-camera keyframe, its index lies within
    // mvKeysUn (:799-801, :816-818)
    auto in_range = [](KeyFrame* k, const vector<MapPoint*>& mps) {
        return k->NLeft == -1 ? mps.size() : k->mvKeysUn.size();
    };
    const vector<uint8_t> valid1 = mi355x_tails::bow_kf_mask(vpMapPoints1, in_range(pKF1, vpMapPoints1));
    const vector<uint8_t> valid2 = mi355x_tails::bow_kf_mask(vpMapPoints2, in_range(pKF2, vpMapPoints2));
    FeatVecCSR fv1(pKF1->mFeatVec), fv2(pKF2->mFeatVec);
    vector<cv::KeyPoint> s1, s2;
    orbm_frame k1 = view(*pKF1, pKF1->NLeft, s1), k2 = view(*pKF2, pKF2->NLeft, s2);
    vector<int32_t> m12(vpMapPoints1.size(), -1);
    const int nm = orbm_search_by_bow_kf(&k1, &fv1.c, valid1.data(), &k2, &fv2.c, valid2.data(), mfNNratio,
                                         mbCheckOrientation ? 1 : 0, m12.data());
    check(nm, "SearchByBoW(KF, KF)");
    mi355x_tails::matches_writeback(m12, vpMapPoints2, vpMatches12);
    return nm;
}

int ORBmatcher::SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, vector<pair<size_t, size_t> >& vMatchedPairs,
                                       const bool bOnlyStereo, const bool bCoarse)
{
    // Compute epipole in second image (:913-943, unchanged)
    Sophus::SE3f T1w = pKF1->GetPose();
    Sophus::SE3f T2w = pKF2->GetPose();
    Sophus::SE3f Tw2 = pKF2->GetPoseInverse();
    Eigen::Vector3f Cw = pKF1->GetCameraCenter();
    Eigen::Vector3f C2 = T2w * Cw;
    Eigen::Vector2f ep = pKF2->mpCamera->project(C2);
    Sophus::SE3f T12;
    Sophus::SE3f Tll, Tlr, Trl, Trr;
    Eigen::Matrix3f R12;
    Eigen::Vector3f t12;
    if (!pKF1->mpCamera2 && !pKF2->mpCamera2) {
        T12 = T1w * Tw2;
        R12 = T12.rotationMatrix();
        t12 = T12.translation();
    } else {
        Sophus::SE3f Tr1w = pKF1->GetRightPose();
        Sophus::SE3f Twr2 = pKF2->GetRightPoseInverse();
        Tll = T1w * Tw2;
        Tlr = T1w * Twr2;
        Trl = Tr1w * Tw2;
        Trr = Tr1w * Twr2;
    }

    const int N1 = pKF1->N, N2 = pKF2->N;
    vector<uint8_t> has1(N1), has2(N2);
    for (int i = 0; i < N1; ++i) has1[i] = pKF1->GetMapPoint(i) != NULL;
    for (int i = 0; i < N2; ++i) has2[i] = pKF2->GetMapPoint(i) != NULL;
    FeatVecCSR fv1(pKF1->mFeatVec), fv2(pKF2->mFeatVec);
    vector<int32_t> m12(N1, -1);
    int nm;
    if (!pKF1->mpCamera2 && !pKF2->mpCamera2 && is_pinhole(pKF1->mpCamera) && is_pinhole(pKF2->mpCamera)) {
        // Pinhole::epipolarConstrain's fundamental matrix (Pinhole.cpp:109-112),
        // the same expression on the same operands, once for the pair; the
        // device runs the epipole and epipolar-line tests per candidate
        Eigen::Matrix3f t12x = Sophus::SO3f::hat(t12);
        Eigen::Matrix3f K1 = pKF1->mpCamera->toK_();
        Eigen::Matrix3f K2 = pKF2->mpCamera->toK_();
        Eigen::Matrix3f F12 = K1.transpose().inverse() * t12x * R12 * K2.inverse();
        float F[9];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) F[3 * r + c] = F12(r, c);
        vector<cv::KeyPoint> s1, s2;
        orbm_frame k1 = view(*pKF1, -1, s1), k2 = view(*pKF2, -1, s2);
        nm = orbm_search_for_triangulation(&k1, &fv1.c, has1.data(), &k2, &fv2.c, has2.data(), F, ep(0), ep(1),
                                           pKF2->mvLevelSigma2.data(), bOnlyStereo ? 1 : 0, bCoarse ? 1 : 0,
                                           mbCheckOrientation ? 1 : 0, 1, m12.data());
    } else {
        // KannalaBrandt8 / two-camera keyframes: the reference's own geometry per
        // candidate, candidates ranked on the device (best first)
        TriCtx ctx;
        ctx.k1 = pKF1;
        ctx.k2 = pKF2;
        ctx.ep = ep;
        ctx.coarse = bCoarse;
        ctx.R12 = R12;
        ctx.t12 = t12;
        ctx.Rll = Tll.rotationMatrix(); ctx.Rlr = Tlr.rotationMatrix();
        ctx.Rrl = Trl.rotationMatrix(); ctx.Rrr = Trr.rotationMatrix();
        ctx.tll = Tll.translation(); ctx.tlr = Tlr.translation();
        ctx.trl = Trl.translation(); ctx.trr = Trr.translation();
        vector<cv::KeyPoint> s1, s2;
        orbm_frame k1 = view(*pKF1, pKF1->NLeft, s1), k2 = view(*pKF2, pKF2->NLeft, s2);
        nm = orbm_search_for_triangulation_checked(&k1, &fv1.c, has1.data(), &k2, &fv2.c, has2.data(),
                                                   bOnlyStereo ? 1 : 0, mbCheckOrientation ? 1 : 0, tri_check, &ctx,
                                                   m12.data());
    }
    check(nm, "SearchForTriangulation");
    vMatchedPairs.reserve(nm);
    mi355x_tails::triangulation_pairs(m12, vMatchedPairs);
    return nm;
}

int ORBmatcher::SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12,
                             const Sophus::Sim3f& S12, const float th)
{
    const float& fx = pKF1->fx;
    const float& fy = pKF1->fy;
    const float& cx = pKF1->cx;
    const float& cy = pKF1->cy;
    // Camera 1 & 2 from world
    Sophus::SE3f T1w = pKF1->GetPose();
    Sophus::SE3f T2w = pKF2->GetPose();
    // Transformation between cameras
    Sophus::Sim3f S21 = S12.inverse();

    const vector<MapPoint*> vpMapPoints1 = pKF1->GetMapPointMatches();
    const int N1 = vpMapPoints1.size();
    const vector<MapPoint*> vpMapPoints2 = pKF2->GetMapPointMatches();
    const int N2 = vpMapPoints2.size();
    vector<bool> vbAlreadyMatched1, vbAlreadyMatched2;
    mi355x_tails::sim3_already_matched(vpMatches12, pKF2, N2, vbAlreadyMatched1, vbAlreadyMatched2);
    // one direction's candidate geometry (:1496-1530 and :1572-1606): both
    // project with pKF1's intrinsics, as the reference does
    auto side = [&](const vector<MapPoint*>& mps, const vector<bool>& already, const Sophus::SE3f& Tw,
                    const Sophus::Sim3f& S, KeyFrame* pKFto, PointRows& pr) {
        for (size_t i = 0; i < mps.size(); ++i) {
            MapPoint* pMP = mps[i];
            if (!pMP || already[i]) continue;
            if (pMP->isBad()) continue;
            Eigen::Vector3f p3Dw = pMP->GetWorldPos();
            Eigen::Vector3f p3Dcf = Tw * p3Dw;
            Eigen::Vector3f p3Dct = S * p3Dcf;
            // Depth must be positive
            if (p3Dct(2) < 0.0) continue;
            const float invz = 1.0 / p3Dct(2);
            const float x = p3Dct(0) * invz;
            const float y = p3Dct(1) * invz;
            const float u = fx * x + cx;
            const float v = fy * y + cy;
            // Point must be inside the image
            if (!pKFto->IsInImage(u, v)) continue;
            const float maxDistance = pMP->GetMaxDistanceInvariance();
            const float minDistance = pMP->GetMinDistanceInvariance();
            const float dist3D = p3Dct.norm();
            // Depth must be inside the scale invariance region
            if (dist3D < minDistance || dist3D > maxDistance) continue;
            pr.valid[i] = 1;
            pr.u[i] = u;
            pr.v[i] = v;
            pr.level[i] = pMP->PredictScale(dist3D, pKFto);
            copy_descriptor(pMP, pr.desc, i);
        }
    };
    PointRows p1(N1), p2(N2);
    side(vpMapPoints1, vbAlreadyMatched1, T1w, S21, pKF2, p1);   // KF1 -> KF2
    side(vpMapPoints2, vbAlreadyMatched2, T2w, S12, pKF1, p2);   // KF2 -> KF1
    vector<cv::KeyPoint> s1, s2;
    orbm_frame k1 = left_grid_view(*pKF1, pKF1->NLeft, s1), k2 = left_grid_view(*pKF2, pKF2->NLeft, s2);
    check(k1.n == N1 && k2.n == N2 ? 0 : ORB_ERR_PARAM, "SearchBySim3: keyframe sizes");
    vector<int32_t> m12(N1, -1);
    const int nFound = orbm_search_by_sim3(&k1, &k2, p1.valid.data(), p1.u.data(), p1.v.data(), p1.level.data(),
                                           p1.desc.data(), p2.valid.data(), p2.u.data(), p2.v.data(),
                                           p2.level.data(), p2.desc.data(), th, m12.data());
    check(nFound, "SearchBySim3");
    // Check agreement (:1653-1671): the device returns the new mutual matches
    mi355x_tails::matches_writeback(m12, vpMapPoints2, vpMatches12);
    return nFound;
}

int ORBmatcher::Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, const float th, const bool bRight)
{
    GeometricCamera* pCamera;
    Sophus::SE3f Tcw;
    Eigen::Vector3f Ow;
    if (bRight) {
        Tcw = pKF->GetRightPose();
        Ow = pKF->GetRightCameraCenter();
        pCamera = pKF->mpCamera2;
    } else {
        Tcw = pKF->GetPose();
        Ow = pKF->GetCameraCenter();
        pCamera = pKF->mpCamera;
    }
    const size_t n = vpMapPoints.size();
    PointRows pr(n);
    for (size_t i = 0; i < n; ++i) {
        int level = 0;
        if (!fuse_point(pKF, vpMapPoints[i], Tcw, Ow, pCamera, pr.u[i], pr.v[i], pr.ur[i], level)) continue;
        pr.valid[i] = 1;
        pr.level[i] = level;
        copy_descriptor(vpMapPoints[i], pr.desc, i);
    }
    // the camera's keypoints, descriptors and mvuRight as :1258-1270 read them
    vector<float> ur_store;
    orbm_frame kf = camera_view(*pKF, bRight && pKF->NLeft != -1, ur_store);
    const int slot0 = (bRight && pKF->NLeft != -1) ? pKF->NLeft : 0;   // :1296
    vector<int32_t> best(n, -1), bdist(n, 0);
    check(orbm_fuse(&kf, pKF->mvInvLevelSigma2.data(), (int)n, pr.valid.data(), pr.u.data(), pr.v.data(),
                    pr.ur.data(), pr.level.data(), pr.desc.data(), th, 1, best.data(), bdist.data()),
          "Fuse");

    // The replace / add decisions (:1311-1328), in index order, with the
    // re-snapshot and single-row re-search of touched points (ORBmatcher_tails.h)
    auto row = [&](MapPoint* pMP, float& u, float& v, float& ur, int& level, uint8_t* d) {
        if (!fuse_point(pKF, pMP, Tcw, Ow, pCamera, u, v, ur, level)) return false;
        const cv::Mat md = pMP->GetDescriptor();
        std::copy(md.data, md.data + 32, d);
        return true;
    };
    auto search1 = [&](float u, float v, float ur, int level, const uint8_t* d) {
        const uint8_t one = 1;
        int32_t b = -1, bd = 0;
        check(orbm_fuse(&kf, pKF->mvInvLevelSigma2.data(), 1, &one, &u, &v, &ur, &level, d, th, 1, &b, &bd), "Fuse");
        return (int)b;
    };
    return mi355x_tails::fuse_decisions(pKF, vpMapPoints, slot0, pr, best, row, search1);
}

int ORBmatcher::Fuse(KeyFrame* pKF, Sophus::Sim3f& Scw, const vector<MapPoint*>& vpPoints, float th,
                     vector<MapPoint*>& vpReplacePoint)
{
    // Decompose Scw
    Sophus::SE3f Tcw = Sophus::SE3f(Scw.rotationMatrix(), Scw.translation() / Scw.scale());
    Eigen::Vector3f Ow = Tcw.inverse().translation();
    // Set of MapPoints already found in the KeyFrame (fixed for the call: :1352)
    const set<MapPoint*> spAlreadyFound = pKF->GetMapPoints();
    const size_t n = vpPoints.size();
    PointRows pr(n);
    for (size_t i = 0; i < n; ++i) {
        MapPoint* pMP = vpPoints[i];
        // Discard Bad MapPoints and already found
        if (pMP->isBad() || spAlreadyFound.count(pMP)) continue;
        int level = 0;
        if (!sim3_point(pKF, pMP, Tcw, Ow, true, pr.u[i], pr.v[i], level)) continue;
        pr.valid[i] = 1;
        pr.level[i] = level;
        copy_descriptor(pMP, pr.desc, i);
    }
    vector<float> ur_store;
    orbm_frame kf = camera_view(*pKF, false, ur_store);   // mGrid, mvKeysUn[idx].octave (:1419-1421)
    vector<int32_t> best(n, -1), bdist(n, 0);
    check(orbm_fuse_sim3(&kf, (int)n, pr.valid.data(), pr.u.data(), pr.v.data(), pr.level.data(), pr.desc.data(), th,
                         best.data(), bdist.data()),
          "Fuse(KF, Sim3)");
    // The replace / add decisions (:1439-1449), in index order (ORBmatcher_tails.h)
    return mi355x_tails::fuse_sim3_decisions(pKF, vpPoints, best, vpReplacePoint);
}

}  // namespace ORB_SLAM3
