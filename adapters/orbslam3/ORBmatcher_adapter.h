/**
 * Shared pieces of the ORBmatcher drop-in bodies (ORBmatcher_searches.cc,
 * ORBmatcher_mapping.cc): the Frame / KeyFrame views the C ABI
 * (include/orb_mi355x.h) takes, the FeatureVector as CSR, and the status check.
 */
#pragma once

#include "ORBmatcher.h"
#include "KeyFrame.h"
#include "MapPoint.h"
#include "orb_mi355x.h"

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

namespace ORB_SLAM3
{
namespace mi355x_adapter
{
static_assert(sizeof(cv::KeyPoint) == sizeof(orb_keypoint), "cv::KeyPoint is the 28-byte orb_keypoint");

// The keypoints a frame's matchers index: mvKeysUn, or for a fisheye stereo
// frame (nleft != -1) mvKeys followed by mvKeysRight (Frame.cc:1069-1071,
// AssignFeaturesToGrid :401-415); `store` keeps the combined copy alive.
template <class F> inline const cv::KeyPoint* keys_of(const F& f, int nleft, std::vector<cv::KeyPoint>& store, int& n)
{
    if (nleft == -1) {
        n = (int)f.mvKeysUn.size();
        return f.mvKeysUn.data();
    }
    store.assign(f.mvKeys.begin(), f.mvKeys.end());
    store.insert(store.end(), f.mvKeysRight.begin(), f.mvKeysRight.end());
    n = (int)store.size();
    return store.data();
}

// A Frame / KeyFrame as the matchers read it (Frame.h:223-290).
template <class F> inline orbm_frame view(const F& f, int nleft, std::vector<cv::KeyPoint>& store)
{
    orbm_frame v;
    int n = 0;
    v.kps = reinterpret_cast<const orb_keypoint*>(keys_of(f, nleft, store, n));
    v.n = (int32_t)n;
    v.desc = f.mDescriptors.data;
    v.min_x = f.mnMinX; v.max_x = f.mnMaxX; v.min_y = f.mnMinY; v.max_y = f.mnMaxY;
    v.grid_inv_w = f.mfGridElementWidthInv;
    v.grid_inv_h = f.mfGridElementHeightInv;
    v.u_right = nleft != -1 || f.mvuRight.empty() ? nullptr : f.mvuRight.data();
    v.scale_factors = f.mvScaleFactors.data();
    v.nlevels = (int32_t)f.mvScaleFactors.size();
    return v;
}

// The left-camera grid of a frame or keyframe with all N feature slots: the
// searches that call GetFeaturesInArea(x, y, r) without bRight read mGrid,
// whose cells hold mvKeysUn (NLeft == -1) or the left mvKeys by index
// (KeyFrame.cc:728-743, Frame.cc:401-415), while their index arrays
// (GetMapPointMatches, mvpMapPoints) span all N slots.  For NLeft != -1 the
// right slots get a position outside the grid bounds, so the library's grid
// (which drops such features, as PosInGrid does: Frame.cc:725-735) holds the
// left keypoints only; their descriptors stay rows NLeft.. of mDescriptors.
template <class F> inline orbm_frame left_grid_view(const F& f, int nleft, std::vector<cv::KeyPoint>& store)
{
    if (nleft == -1) return view(f, -1, store);
    orbm_frame v = view(f, nleft, store);   // [mvKeys; mvKeysRight]
    for (size_t i = (size_t)nleft; i < store.size(); ++i) {
        store[i].pt.x = f.mnMinX - 1.0e6f;
        store[i].pt.y = f.mnMinY - 1.0e6f;
    }
    return v;
}

// One camera of a keyframe as its own frame (Fuse(pKF, ..., bRight)): the
// camera's keypoints (mvKeysUn; mvKeys or mvKeysRight when NLeft != -1), its
// descriptor rows, and mvuRight indexed by the camera-local index as the
// reference reads it (ORBmatcher.cc:1262-1266; entries past the end of
// mvuRight, which the reference would read out of bounds for a right camera
// with more keypoints than the left, read as -1 here).
inline orbm_frame camera_view(const KeyFrame& k, bool right, std::vector<float>& ur_store)
{
    orbm_frame v;
    const std::vector<cv::KeyPoint>& keys = k.NLeft == -1 ? k.mvKeysUn : (right ? k.mvKeysRight : k.mvKeys);
    v.kps = reinterpret_cast<const orb_keypoint*>(keys.data());
    v.n = (int32_t)keys.size();
    v.desc = k.mDescriptors.data + (right ? (size_t)k.NLeft * 32 : 0);
    v.min_x = k.mnMinX; v.max_x = k.mnMaxX; v.min_y = k.mnMinY; v.max_y = k.mnMaxY;
    v.grid_inv_w = k.mfGridElementWidthInv;
    v.grid_inv_h = k.mfGridElementHeightInv;
    if (k.mvuRight.size() >= keys.size()) {
        v.u_right = k.mvuRight.data();
    } else {
        ur_store.assign(keys.size(), -1.0f);
        std::copy(k.mvuRight.begin(), k.mvuRight.end(), ur_store.begin());
        v.u_right = ur_store.data();
    }
    v.scale_factors = k.mvScaleFactors.data();
    v.nlevels = (int32_t)k.mvScaleFactors.size();
    return v;
}

// DBoW2::FeatureVector (std::map<NodeId, std::vector<unsigned int>>) as CSR
struct FeatVecCSR {
    std::vector<uint32_t> nodes, idx;
    std::vector<int32_t> off;
    orbm_featvec c;
    explicit FeatVecCSR(const DBoW2::FeatureVector& fv)
    {
        off.push_back(0);
        for (const auto& kv : fv) {
            nodes.push_back(kv.first);
            idx.insert(idx.end(), kv.second.begin(), kv.second.end());
            off.push_back((int32_t)idx.size());
        }
        c.nnodes = (int32_t)nodes.size();
        c.node_ids = nodes.data();
        c.offsets = off.data();
        c.idx = idx.data();
    }
};

inline void check(int rc, const char* what)
{
    if (rc < 0) throw std::runtime_error(std::string("ORBmatcher: ") + what + " failed");
}

inline void copy_descriptor(MapPoint* pMP, std::vector<uint8_t>& desc, size_t row)
{
    const cv::Mat d = pMP->GetDescriptor();
    std::copy(d.data, d.data + 32, desc.begin() + row * 32);
}
}  // namespace mi355x_adapter
}  // namespace ORB_SLAM3
