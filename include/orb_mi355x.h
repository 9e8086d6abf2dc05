/*
 * orb_mi355x.h — C ABI of the MI355X-native ORB front-end and Hamming matcher.
 *
 * Drop-in boundary for the hot path of vdoom/ORB_SLAM3_VIO_FIXES
 * (paths are relative to the reference tree):
 *   ORBextractor  include/ORBextractor.h:43-109, src/ORBextractor.cc:409-1195
 *   ORBmatcher    include/ORBmatcher.h:36-103,  src/ORBmatcher.cc:43-763,1676-2074
 *   Frame grid    src/Frame.cc:385-416,657-735
 *   DBoW2         Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1126-1259
 *
 * Plain pointers and sizes only.  Nothing throws across this boundary; every
 * entry point returns an integer status (ORB_OK = 0, negatives below) unless
 * documented otherwise.  All functions without "_device" take and return
 * HOST memory; "_device" entry points take device pointers already resident
 * in HBM and an optional hipStream_t (passed as void*, NULL = default stream).
 */
#ifndef ORB_MI355X_H
#define ORB_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (mirrors ORBextractor::operator() -1 on empty input,
 *      src/ORBextractor.cc:1090-1091) ---- */
#define ORB_OK              0
#define ORB_ERR_EMPTY      (-1)  /* empty image                          */
#define ORB_ERR_CAPACITY   (-2)  /* output capacity too small; *n_out = required */
#define ORB_ERR_PARAM      (-3)  /* bad type / size / parameter           */
#define ORB_ERR_DEVICE     (-4)  /* HIP runtime error or no device        */
#define ORB_ERR_UNSUPPORTED (-5) /* configuration outside the restated semantics */

/* cv::KeyPoint layout, 28 bytes (OpenCV core/types.hpp; used as
 * std::vector<cv::KeyPoint> throughout Frame.h). */
typedef struct orb_keypoint {
    float x, y;        /* pt */
    float size;
    float angle;
    float response;
    int32_t octave;
    int32_t class_id;
} orb_keypoint;

/* ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST,
 * int minThFAST)  (include/ORBextractor.h:49-50).  The two knobs select the
 * platform-dependent semantics of the reference build. */
typedef struct orbx_params {
    int32_t nfeatures;
    float   scale_factor;
    int32_t nlevels;
    int32_t ini_th_fast;
    int32_t min_th_fast;
    int32_t blur_variant;   /* 0 = OpenCV>=4.5 error-diffused kernel [18,34,48,56,..] (default),
                               1 = legacy rounded kernel [18,34,49,55,..] */
    int32_t fma_sampling;   /* 1 = fused sampling (reference -O3 -march=native on an FMA host,
                               default), 0 = unfused */
    int32_t reserved;
} orbx_params;

typedef struct orbx_handle orbx_handle;

/* ---------------- extractor ---------------- */

/* ORBextractor::ORBextractor (src/ORBextractor.cc:409-469).  device = HIP
 * ordinal.  Returns NULL on bad params / no device. */
orbx_handle* orbx_create(const orbx_params* params, int device);
void         orbx_destroy(orbx_handle* h);

/* Getters of include/ORBextractor.h:61-81 (GetLevels, GetScaleFactors,
 * GetInverseScaleFactors, GetScaleSigmaSquares, GetInverseScaleSigmaSquares)
 * plus the per-level feature budget and the IC_Angle umax table.  Each array
 * argument may be NULL; sized nlevels (umax: 16). */
int orbx_get_tables(const orbx_handle* h, float* scale, float* inv_scale,
                    float* sigma2, float* inv_sigma2, int32_t* features_per_level,
                    int32_t* umax);

/* Upper bound on keypoints one image of w x h can produce (capacity hint). */
int orbx_max_keypoints(orbx_handle* h, int w, int h_);

/* ORBextractor::operator() (src/ORBextractor.cc:1086-1168) on one 8UC1 host
 * image.  lap0/lap1 = vLappingArea.  Writes *n_out keypoints and *n_out x 32
 * descriptor bytes; *mono_index_out = the return value of the reference
 * (monoIndex).  Returns ORB_OK, ORB_ERR_EMPTY, ORB_ERR_CAPACITY (then *n_out
 * = required), ORB_ERR_PARAM or ORB_ERR_DEVICE. */
int orbx_extract(orbx_handle* h, const uint8_t* img, int w, int h_, size_t step,
                 int lap0, int lap1, orb_keypoint* kps, uint8_t* desc, int cap,
                 int* n_out, int* mono_index_out);

/* operator() on nframes host images of one size at once (the left and right
 * images of a stereo frame, which Frame.cc:122-125,222 extract on two
 * threads, or a window of frames): one upload, one batched pipeline, one
 * download.  imgs[f] with row step steps[f] (steps NULL: w); lap[2f], lap[2f+1]
 * = frame f's vLappingArea (lap NULL: {0, 1000}).  Frame f's outputs:
 * kps[f*cap ...], desc[(f*cap ...) * 32], n_out[f], mono_out[f] (may be NULL).
 * Returns ORB_OK, ORB_ERR_EMPTY (an empty image), ORB_ERR_CAPACITY (some
 * n_out[f] > cap: that frame is not copied), ORB_ERR_PARAM or ORB_ERR_DEVICE.
 * Every frame's pyramid stays on the device (orbx_get_batch_level) until the
 * next extraction call on this handle. */
int orbx_extract_batch(orbx_handle* h, int nframes, const uint8_t* const* imgs, const size_t* steps, int w, int h_,
                       const int32_t* lap, orb_keypoint* kps, uint8_t* desc, int cap, int32_t* n_out,
                       int32_t* mono_out);

/* mvImagePyramid[level] (include/ORBextractor.h:83) of the LAST image
 * extracted by orbx_extract (host copy).  dst may be NULL to query w/h. */
int orbx_get_level(orbx_handle* h, int level, uint8_t* dst, size_t dst_step,
                   int* w, int* h_);

/* mvImagePyramid for the host at the cost of one extra copy: with enable != 0
 * every later orbx_extract on the handle also downloads levels 1.. of its
 * image (one device-to-host copy inside its captured graph) next to the
 * pinned copy of its input, and orbx_get_level then reads them from host
 * memory (a memcpy per row) instead of copying each level from the device.
 * For an adapter that keeps the public mvImagePyramid of
 * include/ORBextractor.h:83 filled for the host Frame::ComputeStereoMatches
 * (src/Frame.cc:818-923).  Not part of the reference interface. */
int orbx_set_host_pyramid(orbx_handle* h, int enable);

/* mvImagePyramid[level] of frame `frame` of the LAST batch call
 * (orbx_extract_batch or orbx_extract_batch_device) on this handle: the
 * per-image pyramid each of the reference's extractor objects exposes
 * (include/ORBextractor.h:83), read by Frame::ComputeStereoMatches
 * (src/Frame.cc:818-923) for the left and right image of a stereo frame
 * extracted in one call.  Level 0 is read from the batch's input frames (for
 * orbx_extract_batch_device: the caller's buffer, which must still be live).
 * ORB_ERR_PARAM when no batch is current (any orbx_extract or plan rebuild
 * ends it).  Waits for an orbx_extract_batch_device batch's work on its
 * stream before copying.  dst may be NULL to query w/h. */
int orbx_get_batch_level(orbx_handle* h, int frame, int level, uint8_t* dst, size_t dst_step,
                         int* w, int* h_);

/* Batched, HBM-resident path: nframes images of w x h, frame f at
 * d_frames + f*frame_stride, rows row_step apart.  Outputs per frame f:
 * d_kps[f*cap ...], d_desc[(f*cap ...)*32], d_n[f], d_mono[f].
 * cap must be >= orbx_max_keypoints(h, w, h_).  Asynchronous on `stream`. */
int orbx_extract_batch_device(orbx_handle* h, int nframes, const uint8_t* d_frames,
                              size_t frame_stride, size_t row_step, int w, int h_,
                              int lap0, int lap1, orb_keypoint* d_kps, uint8_t* d_desc,
                              int cap, int32_t* d_n, int32_t* d_mono, void* stream);

/* Per-stage debug/parity hooks for the last orbx_extract call (host copies).
 * stage 0: per-level FAST candidates (vToDistributeKeys, ORBextractor.cc:794-872)
 * stage 1: per-level DistributeOctTree output (ORBextractor.cc:877-890, before
 *          orientation).  Keypoints are written level after level; counts[l]
 *          receives the per-level count. */
int orbx_debug_stage(orbx_handle* h, int stage, orb_keypoint* kps, int cap,
                     int32_t* counts);

/* Exhaustive check of the device compile of the descriptor's scalar math
 * (test infrastructure; tests/test_gpu_math.py compares the hashes with the
 * oracle's orbo_debug_math, which uses the system libm like the reference):
 * what 0 = glibc sincosf on every float bit pattern in [begin, end) (radians),
 * what 1 = the angle conversion, sincosf and the 512 rBRIEF sampling offsets
 * of every float degree angle in [begin, end) (ORBextractor.cc:107-146),
 * what 2 = fastAtan2 on integer moment pairs (ORBextractor.cc:76-103).
 * hashes[(i - begin) >> chunk_log2] receives sum e_i (2 i + 1) mod 2^64
 * (csrc/orb_math.h: math_mix). */
int orbx_debug_math(int device, int what, long long begin, long long end, int chunk_log2, int fused,
                    unsigned long long* hashes);

/* Device std::sort check (test infrastructure, not part of the reference
 * interface): k_quadtree's emulation of DistributeOctTree's
 * sort(vPrevSizeAndPointerToNode, compareNodes) (src/ORBextractor.cc:538-553,
 * :700; libstdc++ introsort) run on the device over narrays arrays of
 * (count, UL.x) pairs, one workgroup per array.  Array i is elements
 * [off[i], off[i+1]) of cnt / x0, at most 4000 long.  perm[off[i] + j] =
 * the original index (within array i) of the element the sort puts at j;
 * fallback[i] = 1 where the depth limit sent the array to the sequential port
 * (the heap-sort case).  Returns ORB_OK, ORB_ERR_PARAM or ORB_ERR_DEVICE. */
/* The fused FAST pre-test of k_pyr_stream (test hook, not part of the
 * reference interface): for frame `frame` of the last orbx_extract_batch_device
 * call and level `level`, the bitmap of the pixels passing the compass test of
 * ORBextractor's FAST(iniThFAST) candidates (bit x & 7 of byte x >> 3 of row
 * y; defined inside the union of the level's FAST windows, rows win[0]..win[1],
 * columns win[2]..win[3]); win[4] / win[5] receive the bytes per row and the
 * rows dst must hold (dst may be NULL to query win).  ORB_ERR_UNSUPPORTED when
 * that call's FAST pass did not take its candidates from the pre-test. */
int orbx_debug_pretest(orbx_handle* h, int frame, int level, uint8_t* dst, size_t dst_step, int32_t* win);

/* The extraction plan of a w x h image on this handle (built if needed; test
 * hook, not part of the reference interface): info[0..7] = k_pyr_stream usable,
 * fused pre-test on, level-0 chunk rows, steps, LDS bytes, step entries, FAST
 * cells per frame, every window <= 64 x 64 px.  Returns ORB_OK or an error. */
int orbx_debug_plan_info(orbx_handle* h, int w, int h_, int32_t* info, int n);

int orbx_debug_sort(int device, int narrays, const int32_t* off, const int32_t* cnt, const int32_t* x0,
                    int32_t* perm, int32_t* fallback);

/* Per-stage HIP-event timing of subsequent orbx_extract* calls (on the stream
 * they run on).  orbx_get_profile sums, over the recorded calls, the stage
 * times in ms: [0] pyramid, [1] FAST cells, [2] quadtree, [3] describe
 * (orientation + rBRIEF), [4] assemble; returns the number of calls and clears
 * the record.  Not part of the reference interface. */
int orbx_set_profiling(orbx_handle* h, int enable);
int orbx_get_profile(orbx_handle* h, float* stage_ms, int nstages);

/* orbx_extract_batch_device splits a batch into up to `nsub` frame ranges
 * (each >= 16 frames) run on private streams that fork from and join back into
 * the caller's stream; results are identical for every nsub.  With profiling
 * on, each range is one recorded call.  Default 1.  Not part of the reference
 * interface. */
int orbx_set_streams(orbx_handle* h, int nsub);

/* Pyramid kernel of subsequent extractions (results identical for every
 * choice): 0 auto (k_pyr_stream for batches of >= 32 frames, k_pyramid row
 * bands below that), 1 k_pyramid, 2 k_pyr_stream (one workgroup sliding down
 * each frame) whenever the image size allows it.  orbx_pyramid_kernel returns
 * the kernel (1 or 2) the last extraction on the handle ran, 0 before any.
 * Not part of the reference interface. */
int orbx_set_pyramid_mode(orbx_handle* h, int mode);
int orbx_pyramid_kernel(orbx_handle* h);

/* Alternative kernel forms for parity tests and A/B runs (test hooks, not part
 * of the reference interface; process-wide, read when a call is issued).
 * Every form gives identical results; the defaults (0) are the measured
 * fastest, and the alternatives are also the forms a size falls back to when
 * the default's LDS tables do not fit.
 *   ORB_OPT_PROJ_FORM    projection searches: 0 fused single launch
 *                        (brute-force top-K + last-block fixpoint resolve,
 *                        frames <= 4096 keypoints, <= 8192 queries; else 3),
 *                        1 top-K + serial resolve, 2 single-wave search,
 *                        3 top-K + speculative resolve, 4 the fused form
 *                        without its in-block LDS grid (every window scans
 *                        the whole frame), 5 the fused form as two
 *                        launches (phase 1; phase 2 in one block)
 *   ORB_OPT_BOW_FORM     map-wide SearchByBoW: 0 lane per keyframe feature
 *                        (k_bowk_*) when the map carries its totals, 1 k_bow
 *   ORB_OPT_BOWK_BIG     0 auto, 1 no big-node resolve form (every frame node
 *                        in the 256-thread form)
 *   ORB_OPT_PYR_CNT_END  k_pyr_stream's step counters at the top of its LDS
 *                        allocation instead of inside the table image
 *   ORB_OPT_PYR_PRETEST  1: FAST's iniThFAST compass pre-test fused into
 *                        k_pyr_stream (a candidate bitmap k_fast_cells reads;
 *                        measured slower)
 *   ORB_OPT_SFI_FORM     host SearchForInitialization: 0 fused single launch
 *                        (frames <= 4096 keypoints, nnratio >= 0.2; else 1),
 *                        1 grid + top-K + serial resolve, 2 fused without
 *                        its in-block LDS grid, 3 fused as two launches
 *   ORB_OPT_HOST_OUT     single-launch host calls (fused projection and
 *                        initialization searches, SearchByBoW): 0 result
 *                        block written by the kernel into pinned host memory,
 *                        then a completion word the call spins on (no stream
 *                        synchronisation); 1 the same block, the call
 *                        synchronises the stream; 2 a device block copied
 *                        back by one device-to-host copy
 *   ORB_OPT_UPLOAD       host calls' inputs: 0 one kernel reading the pinned
 *                        staging buffer (k_pull), 1 hipMemcpyAsync
 *   ORB_OPT_FAST_CAND_CAP  FAST's per-cell candidate list: 0 the capacity the
 *                        LDS budget leaves (a cell with more candidates is
 *                        scored densely), n > 0 at most n - 1 entries (1:
 *                        every cell through the dense form)
 *   ORB_OPT_BOW_TRACE    diagnostics: n > 0 makes the n-th
 *                        orbm_search_by_bow_dframe call after it is set print
 *                        its small-node waves' checkpoints to stderr
 *   ORB_OPT_QT_FORM      DistributeOctTree: 0 one 4-wave workgroup per (frame,
 *                        level), 1 one wave per (frame, level) with the keys
 *                        in registers (levels of more than 1,536 keys go to
 *                        the 4-wave form in a fixup launch), n >= 2: the
 *                        one-wave form with a key capacity of n - 2 (levels
 *                        beyond it take the fixup path)
 * The two k_pyr_stream options are read when a handle builds its plan (the
 * first extraction of a size).
 * orb_debug_set_option returns ORB_OK or ORB_ERR_PARAM; get returns the value
 * (-1 for an unknown option). */
enum {
    ORB_OPT_PROJ_FORM = 0,
    ORB_OPT_BOW_FORM = 1,
    ORB_OPT_BOWK_BIG = 2,
    ORB_OPT_PYR_CNT_END = 3,
    ORB_OPT_PYR_PRETEST = 4,
    ORB_OPT_SFI_FORM = 5,
    ORB_OPT_HOST_OUT = 6,
    ORB_OPT_UPLOAD = 7,
    ORB_OPT_FAST_CAND_CAP = 8,
    ORB_OPT_BOW_TRACE = 9,
    ORB_OPT_QT_FORM = 10,
    ORB_OPT_COUNT = 11
};
int orb_debug_set_option(int option, int value);
int orb_debug_get_option(int option);

/* Pipeline control for work overlapped with extraction: subsequent
 * extractions on the handle record `event` (a hipEvent_t, NULL = none) on
 * their stream when stage `stage` ends: 0 start, 1 pyramid, 2 FAST cells,
 * 3 quadtree, 4 describe, 5 assemble (with sub-batch streams, after each
 * range).  A caller can thus start other work on another stream once the
 * extraction's VALU-heavy stages are done.  Not part of the reference
 * interface. */
int orbx_set_stage_event(orbx_handle* h, int stage, void* event);

/* ---------------- stereo ---------------- */

/* Frame::ComputeStereoMatches (src/Frame.cc:811-981) for one rectified pair:
 * `left` / `right` are the extractors whose last orbx_extract inputs were the
 * left / right images (their mvImagePyramid, read on the device); kl/dl and
 * kr/dr their keypoints (mvKeys, mvKeysRight) and descriptors; mb = baseline
 * (m), mbf = baseline * fx.  uright / depth (nl floats each) receive
 * mvuRight / mvDepth, -1 where no match.  The reference reads vDistIdx[0] of an
 * empty list when nothing matches; here that case leaves every entry at -1. */
int orbs_compute_stereo_matches(orbx_handle* left, orbx_handle* right,
                                const orb_keypoint* kl, int nl, const uint8_t* dl,
                                const orb_keypoint* kr, int nr, const uint8_t* dr,
                                float mb, float mbf, float* uright, float* depth);

/* Batched, HBM-resident form: pairs i = 0..npairs-1 are frames left0+i and
 * right0+i of the last orbx_extract_batch_device call on h (whose frame buffer
 * must still hold them); d_kps/d_desc/d_n/cap are that call's outputs.
 * d_uright/d_depth/d_sad are [npairs][cap] (d_sad: the correlation distance of
 * kept matches before the median cut, -1 otherwise). */
int orbs_compute_stereo_matches_batch_device(orbx_handle* h, int npairs, int left0, int right0,
                                             const orb_keypoint* d_kps, const uint8_t* d_desc,
                                             const int32_t* d_n, int cap, float mb, float mbf,
                                             float* d_uright, float* d_depth, int32_t* d_sad,
                                             void* stream);

/* cv::BFMatcher(NORM_HAMMING).knnMatch(query, train, matches, 2) as used by
 * Frame::ComputeStereoFishEyeMatches (src/Frame.cc:1144): idx/dist are
 * [nq][2] (host), the two nearest train rows per query in (distance, index)
 * order, -1 where fewer than two train rows exist. */
int orbs_knn_match2(const uint8_t* query, int nq, const uint8_t* train, int nt,
                    int32_t* idx, int32_t* dist, int device);

/* Batched, HBM-resident fisheye stereo candidates (Frame.cc:1126-1156): for
 * pair p, the lapping-area rows [mono, n) of frame left0+p (queries) against
 * those of frame right0+p (train) from the outputs of one
 * orbx_extract_batch_device call; d_idx/d_dist [npairs][cap][2] and
 * d_l2r [npairs][cap] (absolute right row passing Lowe's ratio, -1 otherwise)
 * are indexed by absolute left row.  The triangulation check of each candidate
 * (KannalaBrandt8::TriangulateMatches, :1155) stays with the caller. */
int orbs_fisheye_stereo_candidates_batch_device(int npairs, int left0, int right0, const uint8_t* d_desc,
                                                const int32_t* d_n, const int32_t* d_mono, int cap,
                                                double ratio, int32_t* d_idx, int32_t* d_dist,
                                                int32_t* d_l2r, void* stream);

/* ---------------- matcher ---------------- */

/* ORBmatcher::DescriptorDistance / DBoW2::FORB::distance
 * (src/ORBmatcher.cc:2058-2074, FORB.cpp:81-100). */
int orbm_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* A Frame as the matchers see it (Frame.h): N keypoints (mvKeysUn), N x 32
 * descriptors, image bounds and grid factors (Frame.h:250-251,287-290).
 * The library builds the 64 x 48 cell grid itself (Frame.cc:385-416). */
typedef struct orbm_frame {
    int32_t n;
    const orb_keypoint* kps;
    const uint8_t* desc;
    float min_x, max_x, min_y, max_y;
    float grid_inv_w, grid_inv_h;
    const float* u_right;        /* mvuRight (N) or NULL (mono: all -1) */
    const float* scale_factors;  /* mvScaleFactors (nlevels) or NULL */
    int32_t nlevels;
} orbm_frame;

/* ORBmatcher(nnratio, checkOri).SearchForInitialization(F1, F2, vbPrevMatched,
 * vnMatches12, windowSize)  (src/ORBmatcher.cc:648-763).  prev_xy: N1 x 2
 * in/out.  matches12: N1 out.  Returns nmatches (>= 0) or a negative status. */
int orbm_search_for_initialization(const orbm_frame* f1, const orbm_frame* f2,
                                   float* prev_xy, int window, float nnratio,
                                   int check_ori, int32_t* matches12);

/* Batched device form used by the throughput bench: pairs (F[t], F[t+1]) of
 * consecutive frames of an orbx_extract_batch_device output, prev = F[t]'s own
 * keypoint positions (Tracking.cc:2459-2461).  d_matches: npairs x cap,
 * d_nmatches: npairs.  Grid factors as in orbm_frame. */
int orbm_search_for_initialization_batch_device(
    int nframes, const orb_keypoint* d_kps, const uint8_t* d_desc, const int32_t* d_n,
    int cap, float min_x, float max_x, float min_y, float max_y, float grid_inv_w,
    float grid_inv_h, int window, float nnratio, int check_ori, int32_t* d_matches,
    int32_t* d_nmatches, void* stream);

/* FeatureVector (DBoW2 FeatureVector.h:24-25) as CSR: nnodes node ids in
 * ascending order, offsets[nnodes+1] into idx[] (feature indices ascending). */
typedef struct orbm_featvec {
    int32_t nnodes;
    const uint32_t* node_ids;
    const int32_t* offsets;
    const uint32_t* idx;
} orbm_featvec;

/* ORBmatcher(nnratio, checkOri).SearchByBoW(KeyFrame*, Frame&, matches)
 * (src/ORBmatcher.cc:223-425), monocular/rectified case (F.Nleft == -1,
 * !pKF->mpCamera2).  kf_mp_valid[i] = (pMP != NULL && !pMP->isBad()) for KF
 * feature i.  match_f[F.N] out = KF feature index matched to each F feature
 * or -1.  Returns nmatches. */
int orbm_search_by_bow(const orbm_frame* kf, const orbm_featvec* kf_fv,
                       const uint8_t* kf_mp_valid, const orbm_frame* f,
                       const orbm_featvec* f_fv, float nnratio, int check_ori,
                       int32_t* match_f);

/* A keyframe map resident in HBM for map-wide SearchByBoW (relocalization:
 * Tracking.cc:3641-3648 runs one SearchByBoW(KF_i, F) per candidate).  All
 * pointers are DEVICE pointers.  Keyframe i owns features
 * [kp_off[i], kp_off[i+1]) of kps/desc/valid and FeatureVector nodes
 * [fv_node_off[i], fv_node_off[i+1]) of fv_node; its CSR offsets are the
 * (nnodes_i + 1) entries of fv_off starting at fv_node_off[i] + i, relative to
 * fv_idx + fv_idx_off[i]. */
typedef struct orbm_kf_map_device {
    int32_t nkf;
    const orb_keypoint* kps;
    const uint8_t* desc;
    const uint8_t* valid;        /* MapPoint != NULL && !isBad() */
    const int64_t* kp_off;       /* nkf + 1 */
    const uint32_t* fv_node;
    const int32_t* fv_off;
    const uint32_t* fv_idx;
    const int64_t* fv_node_off;  /* nkf + 1 */
    const int64_t* fv_idx_off;   /* nkf */
    /* host-side totals of the map (0 = unknown: the node-per-wave kernel runs):
     * fv_node_off[nkf] and the FeatureVector entries of all keyframes.  With
     * both set the search runs a lane per keyframe feature (k_bowk_*). */
    int64_t n_nodes_total;
    int64_t n_fv_total;
    /* optional (NULL = gathered from desc): the descriptors in FeatureVector
     * order, n_fv_total x 32, row fv_idx_off[i] + p = desc row kp_off[i] +
     * fv_idx[fv_idx_off[i] + p]; built once per map by orbm_kf_map_fv_desc.  A
     * (keyframe, node)'s features are then contiguous, so the map-wide search
     * streams them instead of gathering 32-B rows across the keyframe. */
    const uint8_t* fv_desc;
    /* optional (NULL = gathered from kps): the keypoint angles in FeatureVector
     * order, n_fv_total floats, row as fv_desc; built once per map by
     * orbm_kf_map_fv_angle.  The rotation filter of the map-wide search then
     * reads 4 contiguous bytes per match instead of a 28-B keypoint row. */
    const float* fv_angle;
} orbm_kf_map_device;

/* Fills d_fv_desc (n_fv_total x 32 device bytes) for map->fv_desc.
 * Asynchronous on `stream`.  Returns ORB_OK or an error. */
int orbm_kf_map_fv_desc(const orbm_kf_map_device* map, uint8_t* d_fv_desc, void* stream);

/* Fills d_fv_angle (n_fv_total device floats) for map->fv_angle.
 * Asynchronous on `stream`.  Returns ORB_OK or an error. */
int orbm_kf_map_fv_angle(const orbm_kf_map_device* map, float* d_fv_angle, void* stream);

/* SearchByBoW(KF_i, F) for nkf host keyframes against one frame in one launch:
 * the relocalisation loop over candidates (src/Tracking.cc:3641-3648).
 * kfs[i], kfvs[i], kf_valid[i] as in orbm_search_by_bow; match_f: nkf x f->n
 * (row i = candidate i's vpMapPointMatches as KF feature indices, -1 = none),
 * counts: nkf.  Returns ORB_OK or an error. */
int orbm_search_by_bow_many(int nkf, const orbm_frame* const* kfs, const orbm_featvec* const* kfvs,
                            const uint8_t* const* kf_valid, const orbm_frame* f, const orbm_featvec* ffv, float nnratio,
                            int check_ori, int32_t* match_f, int32_t* counts);

/* SearchByBoW(KF_i, F) for every keyframe of the map against one frame; f and
 * ffv hold DEVICE pointers.  d_match: nkf x f->n (KF feature index or -1),
 * d_nmatches: nkf.  A keyframe holds fewer than 2^26 features.  Asynchronous
 * on `stream`. */
int orbm_search_by_bow_batch_device(const orbm_kf_map_device* map, const orbm_frame* f,
                                    const orbm_featvec* ffv, float nnratio, int check_ori,
                                    int32_t* d_match, int32_t* d_nmatches, void* stream);

/* The batched device searches (orbm_search_by_bow_batch_device,
 * orbm_search_for_initialization_batch_device) keep their scratch between
 * calls, one set per (device, stream) of the calling thread; at most 16 sets
 * stay allocated (the least recently used one is freed once its own stream has
 * finished its last use of it -- an event wait on that stream, not a device
 * synchronisation).  This frees the calling thread's sets for `stream` on the
 * current device (all = 1: every set of the thread, on any device) the same
 * way.  Call it before destroying a stream these calls used.  Returns ORB_OK,
 * or ORB_ERR_DEVICE if a set's stream reported an error (that set is kept). */
int orbm_release_scratch(void* stream, int all);

/* Test hook: statistics of the calling thread's last projection or
 * initialization search that took the fused form (ORB_OPT_PROJ_FORM 0,
 * ORB_OPT_SFI_FORM 0), 12 ints: fixpoint rounds, exact
 * rescans, the last block's phase-1 and phase-2 shader clocks (s_memtime
 * ticks), its wave 0's grid-build and top-K selection clocks, the block's
 * lifetime in 100 MHz ticks (s_memrealtime), phase 2's table setup clocks,
 * and phase 2's decision passes, rescans, claim-table rebuilds and outputs. */
int orbm_debug_proj_stats(int32_t* out12);

/* Map points projected into F (the fields ORBmatcher reads from MapPoint,
 * MapPoint.h mTrackProjX/Y/XR, mnTrackScaleLevel, mTrackViewCos, mbTrackInView,
 * isBad(), GetDescriptor(), Observations()). */
typedef struct orbm_mappoints {
    int32_t n;
    const float* proj_x;
    const float* proj_y;
    const float* proj_xr;
    const int32_t* level;
    const float* view_cos;
    const float* track_depth;
    const uint8_t* in_view;     /* mbTrackInView && !isBad() */
    const uint8_t* has_obs;     /* Observations() > 0 */
    const uint8_t* desc;        /* n x 32 */
} orbm_mappoints;

/* SearchByProjection(Frame&, vector<MapPoint*>, th, bFarPoints, thFarPoints)
 * (src/ORBmatcher.cc:43-213) for F.Nleft == -1.  owner[F.N] in/out: -1 = no
 * MapPoint, <= -2 = a pre-existing MapPoint (opaque), >= 0 = index into mps
 * set by this call.  blocked[F.N] in: the pre-existing MapPoint has
 * Observations() > 0.  Returns nmatches. */
int orbm_search_by_projection_mps(const orbm_frame* f, const orbm_mappoints* mps,
                                  float th, int far_points, float th_far,
                                  float nnratio, int32_t* owner, const uint8_t* blocked);

/* SearchByProjection(Frame& Current, const Frame& Last, th, bMono)
 * (src/ORBmatcher.cc:1676-1887) for CurrentFrame.Nleft == -1.  The pose math
 * is done by the caller: for each last-frame point i, valid[i] (pMP && !outlier
 * && invzc >= 0 && inside bounds), u,v (projection), ur (u - mbf*invzc),
 * last_octave[i], has_obs[i] and descriptor.  mode: 0 = neither, 1 = bForward,
 * 2 = bBackward.  owner/blocked as above (indices into the last frame).
 * Returns nmatches. */
int orbm_search_by_projection_last(const orbm_frame* cur, int nlast,
                                   const uint8_t* valid, const float* u, const float* v,
                                   const float* ur, const int32_t* last_octave,
                                   const float* last_angle, const uint8_t* has_obs,
                                   const uint8_t* last_desc, float th, int mode,
                                   int check_ori,
                                   int32_t* owner, const uint8_t* blocked);

/* ---------------- frames resident in HBM (the Tracking thread's searches) ----------------
 *
 * The reference runs its per-frame searches on the Frame it just extracted
 * (Tracking::TrackReferenceKeyFrame: Frame::ComputeBoW, then SearchByBoW(KF, F),
 * Tracking.cc:2720-2730; TrackWithMotionModel: SearchByProjection(F, LastFrame),
 * :2886; TrackLocalMap: SearchByProjection(F, local points), :3413), against
 * keyframes whose keypoints, descriptors and FeatureVector never change once
 * built (KeyFrame.cc:98-107).  An orbm_dframe holds such a frame or keyframe in
 * HBM, so a search call moves only its per-call inputs (MapPoint validity,
 * projected points) and its result across PCIe: the inputs are read by the
 * search kernel itself from pinned memory, the result comes back the same way,
 * one launch per call.  The upload forms above stay for callers that hold
 * host arrays only.  A dframe is immutable between updates; updating or
 * destroying it while a search on it runs (on another thread) is the caller's
 * race, as is destroying a keyframe the reference is still reading. */
typedef struct orbm_dframe orbm_dframe;

/* An empty dframe on HIP device `device`.  NULL on error. */
orbm_dframe* orbm_dframe_create(int device);
void orbm_dframe_destroy(orbm_dframe* df);

/* The frame f (host arrays: keypoints, descriptors, u_right / scale factors
 * when set, bounds and grid factors) and its FeatureVector fv (NULL: none;
 * the BoW search needs one) copied into HBM.  Synchronous.  Returns ORB_OK,
 * ORB_ERR_PARAM or ORB_ERR_DEVICE. */
int orbm_dframe_upload(orbm_dframe* df, const orbm_frame* f, const orbm_featvec* fv);

/* The last image orbx_extract extracted on h (Frame::ExtractORB,
 * Frame.cc:418-425) as the dframe's keypoints and descriptors, copied device
 * to device (no PCIe); geom supplies the bounds, grid factors, u_right and
 * scale factors (its kps / desc / n are ignored); fv as in orbm_dframe_upload
 * (Frame::ComputeBoW runs after the extraction: orbm_dframe_set_featvec can
 * add it later).  Asynchronous on the null stream, ordered before every later
 * search.  ORB_ERR_PARAM when h holds no single-image extraction. */
int orbm_dframe_from_extractor(orbm_dframe* df, orbx_handle* h, const orbm_frame* geom, const orbm_featvec* fv);

/* Replaces the dframe's FeatureVector (Frame::ComputeBoW / KeyFrame::ComputeBoW). */
int orbm_dframe_set_featvec(orbm_dframe* df, const orbm_featvec* fv);

/* Keypoint count of the dframe (>= 0), or ORB_ERR_PARAM. */
int orbm_dframe_count(const orbm_dframe* df);

/* The searches of orbm_search_by_bow, orbm_search_by_projection_last,
 * orbm_search_by_projection_mps and orbm_search_for_initialization on
 * dframes: same arguments otherwise, identical results. */
int orbm_search_by_bow_dframe(const orbm_dframe* kf, const uint8_t* kf_mp_valid, const orbm_dframe* f,
                              float nnratio, int check_ori, int32_t* match_f);
int orbm_search_by_projection_last_dframe(const orbm_dframe* cur, int nlast, const uint8_t* valid, const float* u,
                                          const float* v, const float* ur, const int32_t* last_octave,
                                          const float* last_angle, const uint8_t* has_obs,
                                          const uint8_t* last_desc, float th, int mode, int check_ori,
                                          int32_t* owner, const uint8_t* blocked);
int orbm_search_by_projection_mps_dframe(const orbm_dframe* f, const orbm_mappoints* mps, float th, int far_points,
                                         float th_far, float nnratio, int32_t* owner, const uint8_t* blocked);
int orbm_search_for_initialization_dframe(const orbm_dframe* f1, const orbm_dframe* f2, float* prev_xy, int window,
                                          float nnratio, int check_ori, int32_t* matches12);

/* ---------------- fisheye stereo frames (Frame::Nleft != -1) ----------------
 * The frame is the combined keypoint array [mvKeys (nleft); mvKeysRight] with
 * f->n = N descriptor rows; the library builds mGrid over the left keypoints
 * and mGridRight over the right ones by local index (Frame.cc:385-416).  The
 * stereo gate on mvuRight does not apply (f->u_right is ignored). */

/* The right-camera fields ORBmatcher reads from MapPoint (MapPoint.h
 * mbTrackInViewR, mTrackProjXR / YR, mnTrackScaleLevelR, mTrackViewCosR). */
typedef struct orbm_mappoints_right {
    const uint8_t* in_view;     /* mbTrackInViewR && !isBad() */
    const float* proj_x;
    const float* proj_y;
    const int32_t* level;       /* -1: not predicted */
    const float* view_cos;
} orbm_mappoints_right;

/* SearchByBoW(KeyFrame*, Frame&, matches) (src/ORBmatcher.cc:223-425) for
 * F.Nleft = f_nleft >= 0: separate left / right best matches per KF feature
 * (:296-323, :357-386).  Arguments otherwise as orbm_search_by_bow. */
int orbm_search_by_bow_fisheye(const orbm_frame* kf, const orbm_featvec* kf_fv, const uint8_t* kf_valid,
                               const orbm_frame* f, const orbm_featvec* f_fv, int f_nleft, float nnratio,
                               int check_ori, int32_t* match_f);

/* SearchByProjection(Frame&, vector<MapPoint*>, th, bFarPoints, thFarPoints)
 * (src/ORBmatcher.cc:43-213) for F.Nleft = nleft >= 0: left search, then the
 * right camera (its radius carries no th factor, :147), stereo partners set
 * through l2r = mvLeftToRightMatch [nleft] and r2l = mvRightToLeftMatch
 * [N - nleft]; mps->in_view is mbTrackInView && !isBad(), mps->proj_xr is not
 * read.  owner / blocked as orbm_search_by_projection_mps. */
int orbm_search_by_projection_mps_fisheye(const orbm_frame* f, int nleft, const int32_t* l2r, const int32_t* r2l,
                                          const orbm_mappoints* mps, const orbm_mappoints_right* mps_r, float th,
                                          int far_points, float th_far, float nnratio, int32_t* owner,
                                          const uint8_t* blocked);

/* SearchByProjection(Frame& Current, const Frame& Last, th, bMono)
 * (src/ORBmatcher.cc:1676-1887) for CurrentFrame.Nleft = nleft >= 0: ur / vr
 * are each point's projection into the right camera (GetRelativePoseTrl *
 * Tcw * X, :1795-1796); the right search runs when the left candidate list
 * was not empty.  last_octave / last_angle are the last frame's (combined)
 * keypoints.  Other arguments as orbm_search_by_projection_last. */
int orbm_search_by_projection_last_fisheye(const orbm_frame* cur, int nleft, int nlast, const uint8_t* valid,
                                           const float* u, const float* v, const float* ur, const float* vr,
                                           const int32_t* last_octave, const float* last_angle,
                                           const uint8_t* has_obs, const uint8_t* last_desc, float th, int mode,
                                           int check_ori, int32_t* owner, const uint8_t* blocked);

/* ---------------- vocabulary (DBoW2 TemplatedVocabulary<FORB>) ---------------- */

/* A k-ary vocabulary tree laid out breadth first: node 0 = root; children of
 * node i are first_child[i] .. first_child[i]+nchild[i]-1 (nchild 0 = leaf).
 * node_desc: nnodes x 32, word_id/weight per node (leaves). */
typedef struct orbv_vocab {
    int32_t nnodes;
    int32_t depth_levels;       /* m_L */
    const int32_t* first_child;
    const int32_t* nchild;
    const uint8_t* node_desc;
    const int32_t* word_id;
    const double* weight;
    /* NULL: the children of node i are first_child[i] .. first_child[i]+nchild[i]-1;
     * otherwise they are child_idx[first_child[i] + j], j < nchild[i], in the
     * order of Node::children (a loaded text vocabulary, whose ids are line
     * numbers). */
    const int32_t* child_idx;
} orbv_vocab;

/* TemplatedVocabulary::transform(feature, word_id, weight, &nid, levelsup)
 * (TemplatedVocabulary.h:1217-1259) for n descriptors: out word ids, weights
 * and the node id at level m_L - levelsup.  GPU when device >= 0. */
int orbv_transform(const orbv_vocab* voc, int n, const uint8_t* desc, int levelsup,
                   int32_t* word_id, double* weight, int32_t* node_id, int device);

/* orbv_transform with the vocabulary and the descriptors resident in HBM:
 * every array of voc and d_desc / d_word_id / d_weight / d_node_id are
 * DEVICE pointers (e.g. the vocabulary a multi-GPU job broadcast once over
 * RCCL, orb_slam3_vio_fixes_amd/sharding.py).  Asynchronous on `stream`. */
int orbv_transform_device(const orbv_vocab* voc, int n, const uint8_t* d_desc, int levelsup,
                          int32_t* d_word_id, double* d_weight, int32_t* d_node_id, void* stream);

/* ---------------- mapping matchers ---------------- */

/* ORBmatcher::Fuse(pKF, vpMapPoints, th, bRight = false) (src/ORBmatcher.cc:1148-1331)
 * for a pinhole keyframe (NLeft == -1): the matching of every map point.  The
 * caller does the per-point geometry of :1183-1240 on the host (Tcw * P,
 * depth > 0, IsInImage, ur = u - bf / z, distance invariance, viewing angle,
 * PredictScale) and passes valid[i] = false for NULL, bad or already-in-KF
 * points.  kf: mvKeysUn, descriptors, grid bounds, mvuRight (or NULL),
 * mvScaleFactors; inv_level_sigma2: mvInvLevelSigma2.  best_idx[i] receives
 * the keyframe keypoint the point fuses with (bestDist <= TH_LOW) or -1,
 * best_dist[i] its distance.  The replace / add decisions (:1311-1328) depend
 * on the map state and stay with the caller, in index order.  fma = 1
 * reproduces the reference build's contraction of the chi-square sums.
 * Returns the number of points with a keypoint. */
int orbm_fuse(const orbm_frame* kf, const float* inv_level_sigma2, int nmp, const uint8_t* valid, const float* u,
              const float* v, const float* ur, const int32_t* level, const uint8_t* desc, float th, int fma,
              int32_t* best_idx, int32_t* best_dist);

/* ORBmatcher::SearchForTriangulation(pKF1, pKF2, vMatchedPairs, bOnlyStereo,
 * bCoarse) (src/ORBmatcher.cc:907-1146) for pinhole keyframes.  F12 is the
 * 3x3 fundamental matrix row-major exactly as Pinhole::epipolarConstrain
 * computes it (K1^-T [t12]x R12 K2^-1, Pinhole.cpp:109-112), ep the epipole of
 * KF1's centre in KF2 (pKF2->mpCamera->project(T2w * Cw)); both are host
 * geometry.  has_mp: GetMapPoint(i) != NULL.  matches12[N1] out (the pairs of
 * vMatchedPairs are (i, matches12[i]) for matches12[i] >= 0).  Returns the
 * number of matches. */
int orbm_search_for_triangulation(const orbm_frame* kf1, const orbm_featvec* fv1, const uint8_t* has_mp1,
                                  const orbm_frame* kf2, const orbm_featvec* fv2, const uint8_t* has_mp2,
                                  const float* F12, float ep_x, float ep_y, const float* level_sigma2_2,
                                  int only_stereo, int coarse, int check_ori, int fma, int32_t* matches12);

/* SearchForTriangulation for keyframes whose epipolar test only the host can
 * run: KannalaBrandt8 keyframes and two-camera (NLeft != -1) keyframes
 * (ORBmatcher.cc:1014-1076 -> GeometricCamera::epipolarConstrain, for
 * KannalaBrandt8 a Newton unprojection + Eigen JacobiSVD triangulation,
 * KannalaBrandt8.cpp:306-380).  The GPU ranks, for every KF1 feature without a
 * MapPoint (and stereo when only_stereo) in a node both FeatureVectors hold,
 * the KF2 candidates of that node (no MapPoint, stereo filter, distance <=
 * TH_LOW) by (distance ascending, node position descending); check(ctx, idx1,
 * idx2) is the reference's per-candidate geometry (the epipole test of
 * :1014-1021 when it applies, then epipolarConstrain with the camera pair and
 * relative pose the reference selects at :1023-1062) and must be a pure
 * function; the match of idx1 is the first candidate it accepts, which is the
 * candidate the reference's loop keeps.  Then the rotation filter (check_ori),
 * as in orbm_search_for_triangulation.  Returns nmatches. */
typedef int (*orbm_tri_check_fn)(void* ctx, int idx1, int idx2);
int orbm_search_for_triangulation_checked(const orbm_frame* kf1, const orbm_featvec* fv1, const uint8_t* has_mp1,
                                          const orbm_frame* kf2, const orbm_featvec* fv2, const uint8_t* has_mp2,
                                          int only_stereo, int check_ori, orbm_tri_check_fn check, void* ctx,
                                          int32_t* matches12);

/* MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:329-405) for
 * npoints points at once: point p's observed descriptors (the order of its
 * observation map, gathered by the caller) are rows off[p] .. off[p+1]-1 of
 * desc; best[p] receives the index (within the point's rows) of the
 * descriptor with the least median Hamming distance to the others (first on
 * ties), -1 for a point without descriptors.  GPU device `device`. */
int orbm_compute_distinctive_descriptors(int npoints, const int32_t* off, const uint8_t* desc, int32_t* best,
                                         int device);

/* ---------------- relocalisation / loop-closing matchers ---------------- */

/* ORBmatcher(nnratio, checkOri).SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2,
 * vpMatches12) (src/ORBmatcher.cc:765-905) for keyframes with NLeft == -1.
 * valid1 / valid2[i] = (GetMapPointMatches()[i] != NULL && !isBad()).
 * matches12[kf1->n] out: the KF2 feature whose MapPoint becomes
 * vpMatches12[i1], or -1 (NULL).  Returns nmatches. */
int orbm_search_by_bow_kf(const orbm_frame* kf1, const orbm_featvec* fv1, const uint8_t* valid1,
                          const orbm_frame* kf2, const orbm_featvec* fv2, const uint8_t* valid2,
                          float nnratio, int check_ori, int32_t* matches12);

/* SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, sAlreadyFound, th,
 * ORBdist) (src/ORBmatcher.cc:1889-2010) for CurrentFrame.Nleft == -1.  The
 * caller does the per-point geometry of :1906-1934 (Tcw * X, the
 * [mnMinX, mnMaxX] x [mnMinY, mnMaxY] bounds, the distance invariance,
 * PredictScale) for the keyframe's map points i < nq: valid[i] = (pMP && !bad
 * && !sAlreadyFound.count(pMP) && all checks pass), u, v, level, the point's
 * descriptor and kf_angle[i] = pKF->mvKeysUn[i].angle.  owner[f->n] in/out:
 * -1 = CurrentFrame.mvpMapPoints[i2] is NULL, any other value = occupied;
 * slots matched here receive the keyframe index i (cleared again by the
 * rotation filter).  Returns nmatches. */
int orbm_search_by_projection_kf(const orbm_frame* f, int nq, const uint8_t* valid, const float* u,
                                 const float* v, const int32_t* level, const float* kf_angle, const uint8_t* desc,
                                 float th, int orb_dist, int check_ori, int32_t* owner);

/* SearchByProjection(KeyFrame* pKF, Sim3 Scw, vpPoints, vpMatched, th,
 * ratioHamming) (src/ORBmatcher.cc:427-532) and the vpPointsKFs variant
 * (:534-646) for a pinhole keyframe.  Caller geometry (:446-486): valid[i] =
 * (!isBad && !spAlreadyFound.count && depth >= 0 && IsInImage && distance
 * invariance && viewing angle), u, v, level = PredictScale(dist, pKF), the
 * point's descriptor.  matched[kf->n] in/out: -1 = vpMatched[idx] NULL, any
 * other value = occupied; slots matched here receive the point index (the
 * variant sets vpMatchedKF[idx] = vpPointsKFs[matched[idx]]).  Returns
 * nmatches. */
int orbm_search_by_projection_sim3(const orbm_frame* kf, int nq, const uint8_t* valid, const float* u,
                                   const float* v, const int32_t* level, const uint8_t* desc, float th,
                                   float ratio_hamming, int32_t* matched);

/* SearchBySim3(pKF1, pKF2, vpMatches12, S12, th) (src/ORBmatcher.cc:1457-1674)
 * for pinhole keyframes.  Caller geometry: for KF1's map points (kf1->n
 * entries) valid1 (pMP && !already matched && !bad && depth >= 0 && inside
 * KF2 && distance invariance), u1/v1 = projection into KF2 by S21 * T1w,
 * level1 = PredictScale(dist3D, pKF2), mdesc1 = GetDescriptor(); for KF2's
 * map points the same into KF1 (S12 * T2w).  matches12[kf1->n] out: the KF2
 * feature of every NEW mutual match (i1 -> idx2 -> i1, :1658-1671), else -1
 * (vpMatches12[i1] keeps its value).  Returns nFound. */
int orbm_search_by_sim3(const orbm_frame* kf1, const orbm_frame* kf2, const uint8_t* valid1, const float* u1,
                        const float* v1, const int32_t* level1, const uint8_t* mdesc1, const uint8_t* valid2,
                        const float* u2, const float* v2, const int32_t* level2, const uint8_t* mdesc2, float th,
                        int32_t* matches12);

/* Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (src/ORBmatcher.cc:1340-1455)
 * for a pinhole keyframe: the matching of every point.  Caller geometry as
 * for orbm_search_by_projection_sim3 (with spAlreadyFound = pKF->GetMapPoints()).
 * best_idx[i] = the keyframe keypoint (bestDist <= TH_LOW) or -1, best_dist[i]
 * its distance; the replace / add decisions (:1439-1449) read the map and
 * stay with the caller, in index order.  Returns the number of points with a
 * keypoint (nFused). */
int orbm_fuse_sim3(const orbm_frame* kf, int nmp, const uint8_t* valid, const float* u, const float* v,
                   const int32_t* level, const uint8_t* desc, float th, int32_t* best_idx, int32_t* best_dist);

/* ---------------- vocabulary side ---------------- */

/* TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1338-1424): the
 * DBoW2 text format ("k L scoring weighting" header, then one node per line:
 * parent, is-leaf, 32 descriptor bytes, weight).  Node ids are line numbers,
 * word ids follow the order of the leaf lines, and -- as in the reference --
 * the empty read after a final newline appends one non-leaf child of the root
 * with weight 0 (its descriptor is undefined in the reference, 0 here).
 * Returns NULL on failure (*err: ORB_ERR_EMPTY unreadable, ORB_ERR_PARAM bad
 * header or a parent index out of range). */
typedef struct orbv_text_vocab orbv_text_vocab;
orbv_text_vocab* orbv_load_text(const char* path, int32_t* err);
/* Pointers into the loaded vocabulary (valid until orbv_free_text); fills
 * child_idx.  k, scoring (0 L1 .. 5 dot product), weighting (0 TF-IDF, 1 TF,
 * 2 IDF, 3 binary) and the word count as in the header / file. */
int orbv_text_vocab_view(const orbv_text_vocab* v, orbv_vocab* view, int32_t* k, int32_t* scoring,
                         int32_t* weighting, int32_t* nwords);
void orbv_free_text(orbv_text_vocab* v);

/* TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup)
 * (TemplatedVocabulary.h:1126-1194) assembled from the per-descriptor word,
 * weight and node id of orbv_transform: BowVector as (word, value) pairs in
 * word order, normalised as `scoring` requires; FeatureVector as CSR (nodes
 * ascending, feature indices ascending).  Capacities: n entries each, fv_off
 * n + 1. */
int orbv_bow_assemble(int scoring, int weighting, int n, const int32_t* word_id, const double* weight,
                      const int32_t* node_id, int32_t* bow_words, double* bow_values, int32_t* nbow,
                      int32_t* fv_nodes, int32_t* fv_off, int32_t* fv_idx, int32_t* nfv);
/* GeneralScoring::score for two BowVectors (ScoringObject.cpp): scoring 0 L1,
 * 1 L2, 2 chi-square, 3 KL, 4 Bhattacharyya, 5 dot product. */
double orbv_score(int scoring, const int32_t* w1, const double* v1, int n1, const int32_t* w2, const double* v2,
                  int n2);

/* ---------------- keyframe database ---------------- */

/* Device-resident snapshot of KeyFrameDatabase (src/KeyFrameDatabase.cc) for
 * relocalisation.  Keyframes are 0..nkf-1: per-keyframe BowVectors as CSR
 * (bow_off[nkf+1]; words ascending, L1-normalised values), the inverted file
 * mvInvertedFile as CSR by word (inv_off[nwords+1], keyframes in list order),
 * per-keyframe GetBestCovisibilityKeyFrames(10) as CSR and map ids. */
typedef struct orbk_db orbk_db;
orbk_db* orbk_db_create(int device);
void orbk_db_destroy(orbk_db* db);
int orbk_db_upload(orbk_db* db, int nkf, const int32_t* bow_off, const int32_t* bow_words, const double* bow_vals,
                   int nwords, const int32_t* inv_off, const int32_t* inv_kf, const int32_t* cov_off,
                   const int32_t* cov_kf, const int32_t* kf_map);
/* KeyFrameDatabase::DetectRelocalizationCandidates(F, pMap) (:733-845) for the
 * query BowVector (words ascending).  reloc_score[nkf] is every keyframe's
 * mRelocScore: the scored ones are overwritten, and -- as in the reference --
 * neighbours that share words without being scored contribute their current
 * (previous-query) value.  Writes up to cap keyframe indices in the
 * reference's order; returns their count or an error < 0. */
int orbk_detect_relocalization_candidates(orbk_db* db, const int32_t* q_words, const double* q_vals, int nq,
                                          int32_t map_id, float* reloc_score, int32_t* cand, int cap);

#ifdef __cplusplus
}
#endif

#endif /* ORB_MI355X_H */
