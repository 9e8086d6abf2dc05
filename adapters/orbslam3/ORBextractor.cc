/**
 * Drop-in body of ORB_SLAM3::ORBextractor (reference src/ORBextractor.cc)
 * over the MI355X C ABI (include/orb_mi355x.h).
 *
 * Compiles against the reference's UNMODIFIED include/ORBextractor.h:43-109:
 * the device handle lives in a registry keyed by the extractor object instead
 * of a new member, so Frame, Tracking, LocalMapping and LoopClosing rebuild
 * without any header change.  Replace src/ORBextractor.cc by this file, add
 * this repository's include/ to the include path and link
 * orb_slam3_vio_fixes_amd/liborb_mi355x.so.
 *
 * Semantics follow the reference line for line at the boundary:
 *   ctor tables           src/ORBextractor.cc:409-469 (read back from the device plan)
 *   operator()            src/ORBextractor.cc:1086-1168 (returns monoIndex, -1 on empty input :1090-1091)
 *   mvImagePyramid        include/ORBextractor.h:83, read by Frame::ComputeStereoMatches (src/Frame.cc:818-923)
 * The mask argument is ignored: the reference never reads it either.
 * ComputePyramid / ComputeKeyPointsOctTree / DistributeOctTree /
 * ComputeKeyPointsOld and ExtractorNode::DivideNode stay declared by the
 * header and are never called: the device pipeline replaces all of them.
 */
#include "ORBextractor.h"
#include "orb_mi355x.h"

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

using namespace cv;
using namespace std;

static_assert(sizeof(KeyPoint) == sizeof(orb_keypoint), "cv::KeyPoint is the 28-byte orb_keypoint");

namespace ORB_SLAM3
{

namespace
{
// One device handle per extractor object.  The reference header's inline
// destructor cannot release it; ORB-SLAM3 creates its extractors once per
// System (src/Tracking.cc:596-603), so the handles live for the process.
struct Entry {
    orbx_handle* h = nullptr;
    bool host_pyramid = true;   // refresh mvImagePyramid after every extraction
};
std::mutex g_mutex;
std::unordered_map<const ORBextractor*, Entry> g_handles;

Entry entry_of(const ORBextractor* e)
{
    std::lock_guard<std::mutex> lock(g_mutex);
    auto it = g_handles.find(e);
    if (it == g_handles.end()) throw std::runtime_error("ORBextractor: no MI355X handle");
    return it->second;
}

int device_ordinal()
{
    // ORB_MI355X_DEVICE selects the GPU of this process (one process per GPU)
    const char* s = std::getenv("ORB_MI355X_DEVICE");
    return s ? std::atoi(s) : 0;
}

bool host_pyramid_default()
{
    // ORB_MI355X_HOST_PYRAMID=0: no host copies of the levels by default
    const char* s = std::getenv("ORB_MI355X_HOST_PYRAMID");
    return !(s && s[0] == '0');
}
}  // namespace

// The device handle of an extractor object: Frame::ComputeStereoMatches
// passes the left and right extractors' handles to orbs_compute_stereo_matches
// (INTEGRATION.md §4).
orbx_handle* ORBextractorDeviceHandle(const ORBextractor* e)
{
    return entry_of(e).h;
}

// mvImagePyramid is read only by the host Frame::ComputeStereoMatches
// (src/Frame.cc:818-923).  While this is on (the default, so an unmodified
// Frame.cc keeps working) every extraction also downloads the levels (one
// copy inside orbx_extract's captured graph, orbx_set_host_pyramid) and
// refreshes the eight cv::Mats from pinned host memory; switch it off for
// the extractors of a monocular / RGB-D system, or when stereo matching runs
// on the device (orbs_compute_stereo_matches).  Off, the
// levels are released so a stale pyramid is never read.
void ORBextractorSetHostPyramid(ORBextractor* e, bool on)
{
    std::lock_guard<std::mutex> lock(g_mutex);
    auto it = g_handles.find(e);
    if (it == g_handles.end()) throw std::runtime_error("ORBextractor: no MI355X handle");
    it->second.host_pyramid = on;
    orbx_set_host_pyramid(it->second.h, on ? 1 : 0);
}

ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST, int _minThFAST)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels), iniThFAST(_iniThFAST),
      minThFAST(_minThFAST)
{
    orbx_params p;
    p.nfeatures = _nfeatures;
    p.scale_factor = _scaleFactor;
    p.nlevels = _nlevels;
    p.ini_th_fast = _iniThFAST;
    p.min_th_fast = _minThFAST;
    p.blur_variant = 0;   // OpenCV >= 4.5 GaussianBlur kernel
    p.fma_sampling = 1;   // the reference's -O3 -march=native build contracts the rBRIEF sampling (App. A.6)
    p.reserved = 0;
    orbx_handle* h = orbx_create(&p, device_ordinal());
    if (!h) throw std::runtime_error("ORBextractor: orbx_create failed (parameters or no MI355X)");

    // the constructor's tables, computed by the device plan with the
    // reference's float/double expressions (:413-469)
    mvScaleFactor.resize(nlevels);
    mvInvScaleFactor.resize(nlevels);
    mvLevelSigma2.resize(nlevels);
    mvInvLevelSigma2.resize(nlevels);
    mnFeaturesPerLevel.resize(nlevels);
    umax.resize(16);   // HALF_PATCH_SIZE + 1
    if (orbx_get_tables(h, mvScaleFactor.data(), mvInvScaleFactor.data(), mvLevelSigma2.data(),
                        mvInvLevelSigma2.data(), mnFeaturesPerLevel.data(), umax.data()) != ORB_OK) {
        orbx_destroy(h);
        throw std::runtime_error("ORBextractor: orbx_get_tables failed");
    }
    mvImagePyramid.resize(nlevels);

    std::lock_guard<std::mutex> lock(g_mutex);
    Entry en;
    en.h = h;
    en.host_pyramid = host_pyramid_default();
    // the levels come back inside orbx_extract's graph (one copy into pinned
    // memory), so refreshing mvImagePyramid is a host memcpy per row
    orbx_set_host_pyramid(h, en.host_pyramid ? 1 : 0);
    g_handles[this] = en;
}

int ORBextractor::operator()(InputArray _image, InputArray _mask, vector<KeyPoint>& _keypoints,
                             OutputArray _descriptors, std::vector<int>& vLappingArea)
{
    (void)_mask;
    if (_image.empty())
        return -1;
    Mat image = _image.getMat();
    if (image.type() != CV_8UC1)
        throw std::runtime_error("ORBextractor: image must be CV_8UC1");   // assert at :1094
    const Entry en = entry_of(this);
    orbx_handle* h = en.h;

    const int cap = orbx_max_keypoints(h, image.cols, image.rows);
    if (cap < 0)
        throw std::runtime_error("ORBextractor: unsupported image size");
    _keypoints.resize(cap);
    Mat desc(std::max(cap, 1), 32, CV_8U);
    int n = 0, mono = 0;
    const int rc = orbx_extract(h, image.data, image.cols, image.rows, image.step[0], vLappingArea[0],
                                vLappingArea[1], reinterpret_cast<orb_keypoint*>(_keypoints.data()), desc.data,
                                cap, &n, &mono);
    if (rc != ORB_OK)
        throw std::runtime_error("ORBextractor: orbx_extract failed, status " + std::to_string(rc));
    _keypoints.resize(n);

    // descriptors as the reference leaves them (:1107-1113): released when
    // there are no keypoints, else an n x 32 CV_8U matrix
    if (n == 0)
        _descriptors.release();
    else
        desc.rowRange(0, n).copyTo(_descriptors);   // creates the n x 32 CV_8U output

    // mvImagePyramid (host copies of the device levels; level 0 is the input)
    if (!en.host_pyramid) {
        for (Mat& m : mvImagePyramid) m.release();
        return mono;
    }
    for (int level = 0; level < nlevels; ++level) {
        int w = 0, hh = 0;
        if (orbx_get_level(h, level, nullptr, 0, &w, &hh) != ORB_OK)
            throw std::runtime_error("ORBextractor: orbx_get_level failed");
        mvImagePyramid[level].create(hh, w, CV_8U);
        if (orbx_get_level(h, level, mvImagePyramid[level].data, mvImagePyramid[level].step[0], &w, &hh) != ORB_OK)
            throw std::runtime_error("ORBextractor: orbx_get_level failed");
    }
    return mono;
}

}  // namespace ORB_SLAM3
