/**
 * The ordering and map-mutation tails of the drop-in ORBmatcher bodies
 * (ORBmatcher_mapping.cc): what the host does with the device's per-point
 * results -- slot write-backs, the Fuse replace / add decisions with their
 * re-snapshot of touched points, the SearchByBoW(KF, KF) and SearchBySim3
 * masks, the SearchForTriangulation pairs.  Templates over the map types, so
 * the adapter instantiates them with ORB_SLAM3::KeyFrame / MapPoint and
 * tests/native/adapter_tails_test.cpp runs the very same code with functional
 * mock types against the reference's serial loops restated over the oracle
 * (tests/test_gpu_adapter_tails.py).  No reference or OpenCV header here.
 *
 * A map type needs what the reference's own loops call on it:
 *   MP: isBad(), Observations(), Replace(MP*), AddObservation(KF*, int),
 *       GetIndexInKeyFrame(KF*) -> std::tuple<int, int>
 *   KF: GetMapPoint(size_t) -> MP*, AddMapPoint(MP*, size_t)
 */
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <set>
#include <tuple>
#include <utility>
#include <vector>

namespace mi355x_tails
{

// The device searches' per-point inputs (orbm_fuse, orbm_fuse_sim3,
// orbm_search_by_projection_sim3 / _kf, orbm_search_by_sim3): one row a point.
struct PointRows {
    std::vector<uint8_t> valid, desc;
    std::vector<float> u, v, ur;
    std::vector<int32_t> level;
    explicit PointRows(size_t n) : valid(n, 0), desc(n * 32, 0), u(n, 0.f), v(n, 0.f), ur(n, 0.f), level(n, 0) {}
};

// Fuse(pKF, vpMapPoints, th, bRight): the replace / add decisions
// (src/ORBmatcher.cc:1311-1328) in the reference's index order, from the
// device's best slot per point (`best`, camera-local, -1 = none: bestDist >
// TH_LOW or no candidate) computed on the snapshot `pr`.  A decision changes
// the points it touches (Replace makes one bad and recomputes the survivor's
// descriptor, normal and depth; AddObservation puts the point in pKF), so a
// later occurrence of a touched point is snapshotted again at its turn --
// `row(pMP, u, v, ur, level, desc)` is the reference's geometry (:1180-1240),
// false when it rejects the point -- and searched again through
// `search1(u, v, ur, level, desc)` (one device row) when its row changed.
// Untouched points keep their snapshot: no decision changes them.  slot0: the
// right camera's offset into the keyframe's slots (:1296).  Returns nFused.
template <class KF, class MP, class RowFn, class Search1Fn>
int fuse_decisions(KF* pKF, const std::vector<MP*>& vpMapPoints, int slot0, const PointRows& pr,
                   const std::vector<int32_t>& best, RowFn row, Search1Fn search1)
{
    std::set<MP*> touched;
    int nFused = 0;
    for (size_t i = 0; i < vpMapPoints.size(); ++i) {
        MP* pMP = vpMapPoints[i];
        int bestIdx = best[i];
        if (pMP && touched.count(pMP)) {
            float u = 0.f, v = 0.f, ur = 0.f;
            int level = 0;
            uint8_t d[32] = {};
            const bool ok = row(pMP, u, v, ur, level, d);
            const bool same = ok == (pr.valid[i] != 0) &&
                              (!ok || (u == pr.u[i] && v == pr.v[i] && ur == pr.ur[i] && level == pr.level[i] &&
                                       std::equal(d, d + 32, pr.desc.begin() + i * 32)));
            if (!same) bestIdx = ok ? search1(u, v, ur, level, d) : -1;
        }
        // If there is already a MapPoint replace otherwise add new measurement
        if (bestIdx < 0) continue;
        bestIdx += slot0;
        MP* pMPinKF = pKF->GetMapPoint(bestIdx);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) {
                if (pMPinKF->Observations() > pMP->Observations())
                    pMP->Replace(pMPinKF);
                else
                    pMPinKF->Replace(pMP);
                touched.insert(pMP);
                touched.insert(pMPinKF);
            }
        } else {
            pMP->AddObservation(pKF, bestIdx);
            pKF->AddMapPoint(pMP, bestIdx);
            touched.insert(pMP);
        }
        nFused++;
    }
    return nFused;
}

// Fuse(pKF, Scw, vpPoints, th, vpReplacePoint): the decisions of :1439-1449 in
// index order.  No decision here changes another point's inputs (no Replace;
// the already-found set is fixed for the call, :1352), only the keyframe's
// slots, which are read at each decision.
template <class KF, class MP>
int fuse_sim3_decisions(KF* pKF, const std::vector<MP*>& vpPoints, const std::vector<int32_t>& best,
                        std::vector<MP*>& vpReplacePoint)
{
    int nFused = 0;
    for (size_t i = 0; i < vpPoints.size(); ++i) {
        const int bestIdx = best[i];
        if (bestIdx < 0) continue;
        MP* pMP = vpPoints[i];
        MP* pMPinKF = pKF->GetMapPoint(bestIdx);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) vpReplacePoint[i] = pMPinKF;
        } else {
            pMP->AddObservation(pKF, bestIdx);
            pKF->AddMapPoint(pMP, bestIdx);
        }
        nFused++;
    }
    return nFused;
}

// The device's slot states of a slot array: -1 = NULL (a candidate), -2 =
// occupied (SearchByProjection(KF, Sim3) vpMatched :502-503 / :618-619,
// SearchByProjection(F, KF) mvpMapPoints :1949-1950).
template <class MP> std::vector<int32_t> slot_states(const std::vector<MP*>& slots)
{
    std::vector<int32_t> s(slots.size());
    for (size_t k = 0; k < slots.size(); ++k) s[k] = slots[k] ? -2 : -1;
    return s;
}

// A slot the device filled (its point index >= 0) takes that point, and for
// the vpPointsKFs form of SearchByProjection(KF, Sim3) (:534-646) its
// keyframe too (vpMatchedKF[bestIdx] = vpPointsKFs[iMP], :631-632).  Slots
// the device left (-1 / -2) keep what they held.
template <class MP, class KFp>
void slot_writeback(const std::vector<int32_t>& matched, const std::vector<MP*>& vpPoints,
                    const std::vector<KFp>* vpPointsKFs, std::vector<MP*>& slots, std::vector<KFp>* slotKFs)
{
    for (size_t k = 0; k < slots.size(); ++k)
        if (matched[k] >= 0) {
            slots[k] = vpPoints[matched[k]];
            if (slotKFs) (*slotKFs)[k] = (*vpPointsKFs)[matched[k]];
        }
}

// SearchByBoW(KF1, KF2): a feature takes part iff its MapPoint is set and
// good (:803-808, :822-827) and its index lies within the keyframe's
// mvKeysUn (`n_in_range`; :799-801, :816-818 for a two-camera keyframe).
template <class MP> std::vector<uint8_t> bow_kf_mask(const std::vector<MP*>& mps, size_t n_in_range)
{
    std::vector<uint8_t> m(mps.size(), 0);
    for (size_t i = 0; i < mps.size(); ++i) m[i] = mps[i] && !mps[i]->isBad() && i < n_in_range;
    return m;
}

// vpMatches12 from the device's KF1 -> KF2 feature indices (:892-902), and
// SearchBySim3's new mutual matches (:1653-1671) the same way.
template <class MP>
void matches_writeback(const std::vector<int32_t>& m12, const std::vector<MP*>& vpMapPoints2,
                       std::vector<MP*>& vpMatches12)
{
    for (size_t i = 0; i < m12.size(); ++i)
        if (m12[i] >= 0) vpMatches12[i] = vpMapPoints2[m12[i]];
}

// SearchBySim3's already-matched flags (:1477-1492): KF1 features whose
// vpMatches12 entry is set, and the KF2 features those points occupy.
template <class MP, class KF>
void sim3_already_matched(const std::vector<MP*>& vpMatches12, KF* pKF2, int N2, std::vector<bool>& am1,
                          std::vector<bool>& am2)
{
    am1.assign(vpMatches12.size(), false);
    am2.assign(N2, false);
    for (size_t i = 0; i < vpMatches12.size(); i++) {
        MP* pMP = vpMatches12[i];
        if (pMP) {
            am1[i] = true;
            const int idx2 = std::get<0>(pMP->GetIndexInKeyFrame(pKF2));
            if (idx2 >= 0 && idx2 < N2) am2[idx2] = true;
        }
    }
}

// SearchForTriangulation's output (:1138-1145): the pairs in KF1 index order.
inline void triangulation_pairs(const std::vector<int32_t>& m12, std::vector<std::pair<size_t, size_t> >& pairs)
{
    pairs.clear();
    for (size_t i = 0; i < m12.size(); i++)
        if (m12[i] >= 0) pairs.push_back(std::make_pair(i, (size_t)m12[i]));
}

}  // namespace mi355x_tails
