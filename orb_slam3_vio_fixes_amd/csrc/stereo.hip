// stereo.hip — Frame::ComputeStereoMatches (reference src/Frame.cc:811-981) on
// the GPU pyramids of the extractor.
//
// Three launches per batch of rectified pairs:
//   k_stereo_rows    one workgroup per pair: the row table of the right
//                    keypoints' bands (Frame.cc:821-838) as CSR lists built
//                    with LDS counters (list order is irrelevant, see below).
//   k_stereo_match   one wave per left keypoint: its row's candidates,
//                    octave window and disparity range, the lexicographic
//                    (Hamming distance, right index) minimum below TH_HIGH --
//                    what the reference's in-index-order first-minimum scan
//                    returns; then the 11-position 11x11 L1 correlation on the
//                    keypoint's pyramid level (patch and strip staged in LDS,
//                    lanes over (offset, row)), parabola fit, depth.
//   k_stereo_prune   one workgroup per pair: the (SAD, index) list sorted in
//                    LDS (bitonic), median, and the 1.5*1.4*median cut
//                    (Frame.cc:967-980).
// Everything runs on device data the extractor left in HBM: level 0 is the
// caller's frame, levels >= 1 the handle's pyramid slab.
#include "../../include/orb_mi355x.h"
#include "common.h"
#include "plan.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <vector>

namespace orbmi {

constexpr int kStThHigh = 100, kStThLow = 50;     // ORBmatcher.cc:35-36
constexpr int kWin = 5, kSlide = 5;               // Frame.cc:904, :910

// Pyramid levels of one side for every pair of the launch.
struct PyrView {
    const uint8_t* l0;          // level 0 of pair 0's frame
    long long l0_fstride;       // bytes between consecutive pairs' level-0 images
    int l0_pitch;
    const uint8_t* pyr;         // levels >= 1 slab of pair 0's frame
    long long pyr_fstride;
    const LevelDev* lv;         // device level table (w, h, pitch, off)
};

__device__ __forceinline__ const uint8_t* level_row(const PyrView& v, int pair, int level, int y) {
    if (level == 0) return v.l0 + pair * v.l0_fstride + (long long)y * v.l0_pitch;
    const LevelDev& d = v.lv[level];
    return v.pyr + pair * v.pyr_fstride + d.off + (long long)y * d.pitch;
}

struct StereoArgs {
    PyrView L, R;
    const orb_keypoint* kl;     // pair p: kl + p * kstride
    const uint8_t* dl;          // pair p: dl + p * kstride * 32
    const int32_t* nl;          // pair p: nl[p]
    const orb_keypoint* kr;
    const uint8_t* dr;
    const int32_t* nr;
    long long kstride;
    float scale[kMaxLevels], inv_scale[kMaxLevels];
    float mb, mbf;
    float* uright;              // pair p: + p * ostride
    float* depth;
    int* sad;                   // correlation distance of accepted matches, -1 otherwise
    long long ostride;
    // row table (Frame.cc:821-838): pair p, row y -> right indices
    // row_list[p * list_stride + row_off[p * (rows + 1) + y] ...]
    int* row_off;
    int* row_list;
    int rows;                   // level-0 image rows
    long long list_stride;
};

__device__ __forceinline__ int hamming_st(const uint4 a0, const uint4 a1, const uint8_t* b) {
    const uint4 b0 = *(const uint4*)b, b1 = *(const uint4*)(b + 16);
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// Row band of a right keypoint (Frame.cc:830-834).
__device__ __forceinline__ void row_band(const StereoArgs& a, const orb_keypoint& kp, int& lo, int& hi) {
    const float r = 2.0f * a.scale[kp.octave];
    hi = (int)ceilf(kp.y + r);
    lo = (int)floorf(kp.y - r);
}

// grid (pairs) x 256, dynamic LDS = (rows + 1) ints: the row table.  Lists hold
// every right keypoint whose band covers the row, in arbitrary order (the
// match kernel takes the lexicographic (distance, index) minimum, which is
// what the reference's in-index-order first-minimum scan returns).
__global__ __launch_bounds__(256) void k_stereo_rows(StereoArgs a) {
    extern __shared__ int rc[];
    __shared__ int tmp[16];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int nr = a.nr[p];
    const orb_keypoint* KR = a.kr + p * a.kstride;
    for (int y = tid; y <= a.rows; y += blockDim.x) rc[y] = 0;
    __syncthreads();
    for (int i = tid; i < nr; i += blockDim.x) {
        int lo, hi;
        row_band(a, KR[i], lo, hi);
        for (int y = max(lo, 0); y <= min(hi, a.rows - 1); ++y) atomicAdd(&rc[y], 1);
    }
    __syncthreads();
    block_excl_scan(rc, a.rows + 1, tmp);
    int* off = a.row_off + (long long)p * (a.rows + 1);
    for (int y = tid; y <= a.rows; y += blockDim.x) off[y] = rc[y];
    __syncthreads();
    int* list = a.row_list + p * a.list_stride;
    for (int i = tid; i < nr; i += blockDim.x) {
        int lo, hi;
        row_band(a, KR[i], lo, hi);
        for (int y = max(lo, 0); y <= min(hi, a.rows - 1); ++y) list[atomicAdd(&rc[y], 1)] = i;
    }
}

// grid (ceil(max nl / 4), pairs) x 256: one wave per left keypoint
__global__ __launch_bounds__(256) void k_stereo_match(StereoArgs a) {
    __shared__ uint8_t patch[4][11 * 11 + 11 * 21];
    __shared__ int part[4][128];
    const int p = blockIdx.y, lane = lane_id(), wv = wave_id();
    const int iL = blockIdx.x * 4 + wv;
    const int nl = a.nl[p];
    if (iL >= nl) return;
    const orb_keypoint kpL = a.kl[p * a.kstride + iL];
    float* ur_out = a.uright + p * a.ostride;
    float* dp_out = a.depth + p * a.ostride;
    int* sad_out = a.sad + p * a.ostride;
    float uR_res = -1.0f, depth_res = -1.0f;
    int sad_res = -1;
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    const int row = (int)vL;                                       // vRowIndices[vL] (:856)
    const float minD = 0.f, maxD = a.mbf / a.mb;                   // :841-843
    const float minU = uL - maxD, maxU = uL - minD;
    if (maxU >= 0 && row >= 0 && row < a.rows) {
        // best right candidate: (dist, iR) lexicographic minimum below TH_HIGH (:867-893)
        const uint8_t* dL = a.dl + (p * a.kstride + iL) * 32;
        const uint4 q0 = *(const uint4*)dL, q1 = *(const uint4*)(dL + 16);
        const orb_keypoint* KR = a.kr + p * a.kstride;
        const uint8_t* DR = a.dr + p * a.kstride * 32;
        const int* off = a.row_off + (long long)p * (a.rows + 1);
        const int* list = a.row_list + p * a.list_stride;
        const int c0 = off[row], c1 = off[row + 1];
        uint32_t best = ((uint32_t)kStThHigh << 16) | 0xffffu;
        for (int c = c0 + lane; c < c1; c += kWave) {
            const int iR = list[c];
            const orb_keypoint kpR = KR[iR];
            if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
            if (!(kpR.x >= minU && kpR.x <= maxU)) continue;
            const int dist = hamming_st(q0, q1, DR + (long long)iR * 32);
            if (dist < kStThHigh) best = min(best, ((uint32_t)dist << 16) | (uint32_t)iR);
        }
        best = wave_min(best, 0xffffffffu);
        const int bestDist = (int)(best >> 16), bestIdxR = (int)(best & 0xffff);
        if (bestDist < (kStThHigh + kStThLow) / 2) {               // :896
            // sub-pixel match by correlation (:898-933)
            const float uR0 = KR[bestIdxR].x;
            const float sf = a.inv_scale[levelL];
            const float scaleduL = roundf(kpL.x * sf), scaledvL = roundf(kpL.y * sf);
            const float scaleduR0 = roundf(uR0 * sf);
            const float iniu = scaleduR0 + kSlide - kWin, endu = scaleduR0 + kSlide + kWin + 1;
            if (!(iniu < 0 || endu >= a.R.lv[levelL].w)) {
                // stage the 11x11 left patch and the 11x21 right strip, then
                // lanes take (offset, row) items: 11 abs differences each
                const int yl0 = (int)scaledvL - kWin, xl0 = (int)scaleduL - kWin;
                const int xr0 = (int)scaleduR0 - kSlide - kWin;
                uint8_t* PL = patch[wv];
                uint8_t* PR = PL + 121;
                for (int i = lane; i < 121 + 231; i += kWave) {
                    if (i < 121) {
                        const int y = i / 11, x = i - y * 11;
                        PL[i] = level_row(a.L, p, levelL, yl0 + y)[xl0 + x];
                    } else {
                        const int j = i - 121, y = j / 21, x = j - y * 21;
                        PR[j] = level_row(a.R, p, levelL, yl0 + y)[xr0 + x];
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                for (int i = lane; i < 121; i += kWave) {
                    const int k = i / 11, y = i - k * 11;       // offset index, row
                    int s = 0;
#pragma unroll
                    for (int x = 0; x < 11; ++x) s += abs((int)PL[y * 11 + x] - (int)PR[y * 21 + k + x]);
                    part[wv][i] = s;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                float dist = 0.f;
                if (lane <= 2 * kSlide) {
                    int s = 0;
#pragma unroll
                    for (int y = 0; y < 11; ++y) s += part[wv][lane * 11 + y];
                    dist = (float)s;                               // cv::norm(NORM_L1): exact
                }
                float dists[2 * kSlide + 1];
#pragma unroll
                for (int k = 0; k <= 2 * kSlide; ++k) dists[k] = __shfl(dist, k, kWave);
                int bestSad = INT_MAX, bestinc = 0;
#pragma unroll
                for (int k = 0; k <= 2 * kSlide; ++k)
                    if (dists[k] < (float)bestSad) { bestSad = (int)dists[k]; bestinc = k - kSlide; }
                if (bestinc != -kSlide && bestinc != kSlide) {      // :935-936
                    const float d1 = dists[kSlide + bestinc - 1], d2 = dists[kSlide + bestinc];
                    const float d3 = dists[kSlide + bestinc + 1];
                    const float deltaR = (d1 - d3) / (2.0f * (d1 + d3 - 2.0f * d2));
                    if (!(deltaR < -1 || deltaR > 1)) {
                        float bestuR = a.scale[levelL] * ((float)scaleduR0 + (float)bestinc + deltaR);
                        float disparity = uL - bestuR;
                        if (disparity >= minD && disparity < maxD) {  // :953-964
                            if (disparity <= 0) {
                                disparity = (float)0.01;
                                bestuR = (float)((double)uL - 0.01);
                            }
                            depth_res = a.mbf / disparity;
                            uR_res = bestuR;
                            sad_res = bestSad;
                        }
                    }
                }
            }
        }
    }
    if (lane == 0) {
        ur_out[iL] = uR_res;
        dp_out[iL] = depth_res;
        sad_out[iL] = sad_res;
    }
}

// grid (pairs) x 256, dynamic LDS = pow2 >= nl keys: the outlier cut (:967-980)
__global__ __launch_bounds__(256) void k_stereo_prune(StereoArgs a, int np2) {
    extern __shared__ uint32_t keys[];
    __shared__ int cnt;
    const int p = blockIdx.x, tid = threadIdx.x;
    const int nl = a.nl[p];
    const int* sad = a.sad + p * a.ostride;
    if (tid == 0) cnt = 0;
    __syncthreads();
    for (int i = tid; i < np2; i += blockDim.x) keys[i] = 0xffffffffu;
    __syncthreads();
    for (int i = tid; i < nl; i += blockDim.x)
        if (sad[i] >= 0) keys[atomicAdd(&cnt, 1)] = ((uint32_t)sad[i] << 16) | (uint32_t)i;
    __syncthreads();
    const int n = cnt;
    if (n == 0) return;                 // the reference reads vDistIdx[0] here (undefined)
    // bitonic sort of (SAD, index) ascending == std::sort of the pairs
    for (int k = 2; k <= np2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < np2; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint32_t x = keys[i], y = keys[ixj];
                    const bool up = (i & k) == 0;
                    if ((x > y) == up) { keys[i] = y; keys[ixj] = x; }
                }
            }
            __syncthreads();
        }
    const float median = (float)(int)(keys[n / 2] >> 16);
    const float thDist = 1.5f * 1.4f * median;
    float* ur = a.uright + p * a.ostride;
    float* dp = a.depth + p * a.ostride;
    // the reference walks down from the largest and stops at the first below thDist
    for (int j = tid; j < n; j += blockDim.x) {
        const int s = (int)(keys[j] >> 16);
        if (!((float)s < thDist)) {
            const int i = (int)(keys[j] & 0xffff);
            ur[i] = -1.0f;
            dp[i] = -1.0f;
        }
    }
}

// ---------------------------------------------------------------------------
// Frame::ComputeStereoFishEyeMatches (Frame.cc:1126-1166): brute-force
// BFMatcher(NORM_HAMMING).knnMatch(k = 2) of the left lapping-area
// descriptors against the right ones and Lowe's 0.7 ratio.  One query per
// thread (its 32 B in registers), train descriptors streamed through LDS in
// tiles of 256 (broadcast reads); the per-thread top-2 insertion is OpenCV's
// batchDistance rule (strict '<' against the 2nd best, equal distances keep
// index order).  The Kannala-Brandt triangulation of the candidates stays on
// the host.
// ---------------------------------------------------------------------------
struct KnnArgs {
    const uint8_t* q;           // pair p: q + p * stride * 32, rows [q0[p], qn[p])
    const uint8_t* t;
    const int32_t* q0;
    const int32_t* qn;
    const int32_t* t0;
    const int32_t* tn;
    long long stride;           // rows per pair (cap)
    double ratio;
    int32_t* idx;               // [pair][stride][2], absolute train rows, -1 if none
    int32_t* dist;              // [pair][stride][2]
    int32_t* l2r;               // [pair][stride]: ratio-passing candidate or -1
};

__global__ __launch_bounds__(256) void k_knn2(KnnArgs a) {
    __shared__ uint4 tile[256][2];
    const int p = blockIdx.y, tid = threadIdx.x;
    const int q0 = a.q0[p], qn = a.qn[p], t0 = a.t0[p], tn = a.tn[p];
    const int nt = max(0, tn - t0);
    const int q = q0 + blockIdx.x * 256 + tid;
    int32_t* idx = a.idx + p * a.stride * 2;
    int32_t* dst = a.dist + p * a.stride * 2;
    int32_t* l2r = a.l2r + p * a.stride;
    if (blockIdx.x == 0)                       // rows outside the lapping area
        for (int i = tid; i < q0; i += 256) {
            idx[2 * i] = idx[2 * i + 1] = -1;
            dst[2 * i] = dst[2 * i + 1] = -1;
            l2r[i] = -1;
        }
    if (q0 + (int)blockIdx.x * 256 >= qn) return;          // block-uniform
    const bool act = q < qn;
    uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
    if (act) {
        const uint4* qp = (const uint4*)(a.q + (p * a.stride + q) * 32);
        a0 = qp[0];
        a1 = qp[1];
    }
    int d1 = INT_MAX, d2 = INT_MAX, i1 = -1, i2 = -1;
    const uint4* tp = (const uint4*)(a.t + (p * a.stride + t0) * 32);
    for (int base = 0; base < nt; base += 256) {
        __syncthreads();
        if (base + tid < nt) {
            tile[tid][0] = tp[2 * (base + tid)];
            tile[tid][1] = tp[2 * (base + tid) + 1];
        }
        __syncthreads();
        const int m = min(256, nt - base);
        if (act)
            for (int j = 0; j < m; ++j) {
                const uint4 b0 = tile[j][0], b1 = tile[j][1];
                const int d = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) +
                              __popc(a0.w ^ b0.w) + __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) +
                              __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
                if (d < d2) {
                    if (d1 > d) { d2 = d1; i2 = i1; d1 = d; i1 = base + j; }
                    else { d2 = d; i2 = base + j; }
                }
            }
    }
    if (act) {
        idx[2 * q] = i1 >= 0 ? i1 + t0 : -1;
        idx[2 * q + 1] = i2 >= 0 ? i2 + t0 : -1;
        dst[2 * q] = i1 >= 0 ? d1 : -1;
        dst[2 * q + 1] = i2 >= 0 ? d2 : -1;
        // (*it).size() >= 2 && (*it)[0].distance < (*it)[1].distance * 0.7 (:1151), in double
        l2r[q] = (i2 >= 0 && (double)d1 < (double)d2 * a.ratio) ? i1 + t0 : -1;
    }
}

static PyrView pyr_view(const orbx_handle* h, const uint8_t* l0, long long l0_fstride, int l0_pitch, int first) {
    PyrView v;
    v.l0 = l0 + first * l0_fstride;
    v.l0_fstride = l0_fstride;
    v.l0_pitch = l0_pitch;
    v.pyr = h->plan.d_pyr + first * h->plan.pyr_bytes;
    v.pyr_fstride = h->plan.pyr_bytes;
    v.lv = h->plan.d_lv;
    return v;
}

// Sizes of the row table for `npairs` pairs of `rows` rows and <= max_nr right keypoints.
static void row_table_sizes(const orbx_handle* h, int npairs, int rows, int max_nr, size_t& off_ints,
                            long long& list_stride) {
    const int band = (int)(4.0f * h->scale[h->plan.L - 1]) + 3;    // ceil(y+r) - floor(y-r) + 1 <= 2r + 2
    off_ints = (size_t)npairs * (rows + 1);
    list_stride = (long long)max_nr * band;
}

static int launch_stereo(StereoArgs& a, const orbx_handle* h, int npairs, int max_nl, hipStream_t st) {
    for (int l = 0; l < h->plan.L; ++l) {
        a.scale[l] = h->scale[l];
        a.inv_scale[l] = h->inv_scale[l];
    }
    ORB_LAUNCH(k_stereo_rows, dim3(npairs), dim3(256), (a.rows + 1) * sizeof(int), st, a);
    if (max_nl > 0)
        ORB_LAUNCH(k_stereo_match, dim3((max_nl + 3) / 4, npairs), dim3(256), 0, st, a);
    int np2 = 1;
    while (np2 < std::max(1, max_nl)) np2 <<= 1;
    ORB_LAUNCH(k_stereo_prune, dim3(npairs), dim3(256), np2 * sizeof(uint32_t), st, a, np2);
    ORB_CHECK(hipGetLastError());
    return ORB_OK;
}

template <typename T>
struct SBuf {
    T* p = nullptr;
    ~SBuf() { if (p) (void)hipFree(p); }
    int alloc(size_t n) { return hipMalloc(&p, std::max<size_t>(1, n) * sizeof(T)) == hipSuccess ? ORB_OK : ORB_ERR_DEVICE; }
};

}  // namespace orbmi

using namespace orbmi;

extern "C" {

int orbs_compute_stereo_matches_batch_device(orbx_handle* h, int npairs, int left0, int right0,
                                             const orb_keypoint* d_kps, const uint8_t* d_desc, const int32_t* d_n,
                                             int cap, float mb, float mbf, float* d_uright, float* d_depth,
                                             int32_t* d_sad, void* stream) {
    if (!h || npairs <= 0 || !d_kps || !d_desc || !d_n || !d_uright || !d_depth || !d_sad) return ORB_ERR_PARAM;
    if (!h->last_frames || left0 < 0 || right0 < 0 || left0 + npairs > h->last_B || right0 + npairs > h->last_B)
        return ORB_ERR_PARAM;
    if (cap < h->plan.out_total || cap > 65536 || !(mb > 0.f)) return ORB_ERR_PARAM;
    if (hipSetDevice(h->device) != hipSuccess) return ORB_ERR_DEVICE;
    StereoArgs a;
    a.L = pyr_view(h, h->last_frames, h->last_fstride, h->last_pitch0, left0);
    a.R = pyr_view(h, h->last_frames, h->last_fstride, h->last_pitch0, right0);
    a.kl = d_kps + (long long)left0 * cap;
    a.dl = d_desc + (long long)left0 * cap * 32;
    a.nl = d_n + left0;
    a.kr = d_kps + (long long)right0 * cap;
    a.dr = d_desc + (long long)right0 * cap * 32;
    a.nr = d_n + right0;
    a.kstride = cap;
    a.mb = mb;
    a.mbf = mbf;
    a.uright = d_uright;
    a.depth = d_depth;
    a.sad = d_sad;
    a.ostride = cap;
    a.rows = h->plan.lv[0].h;
    size_t off_ints;
    row_table_sizes(h, npairs, a.rows, cap, off_ints, a.list_stride);
    const size_t need = (off_ints + (size_t)npairs * a.list_stride) * sizeof(int);
    if (need > h->st_scratch_bytes) {
        if (h->st_scratch) (void)hipFree(h->st_scratch);
        h->st_scratch = nullptr;
        h->st_scratch_bytes = 0;
        ORB_CHECK(hipMalloc(&h->st_scratch, need));
        h->st_scratch_bytes = need;
    }
    a.row_off = (int*)h->st_scratch;
    a.row_list = a.row_off + off_ints;
    return launch_stereo(a, h, npairs, cap, (hipStream_t)stream);
}

int orbs_compute_stereo_matches(orbx_handle* left, orbx_handle* right, const orb_keypoint* kl, int nl,
                                const uint8_t* dl, const orb_keypoint* kr, int nr, const uint8_t* dr, float mb,
                                float mbf, float* uright, float* depth) {
    if (!left || !right || nl < 0 || nr < 0 || (nl && (!kl || !dl || !uright || !depth)) || (nr && (!kr || !dr)))
        return ORB_ERR_PARAM;
    if (!left->have_last || !right->have_last || left->device != right->device) return ORB_ERR_PARAM;
    if (left->last_w != right->last_w || left->last_h != right->last_h || left->plan.L != right->plan.L)
        return ORB_ERR_PARAM;
    if (!(mb > 0.f) || nr > 65536) return ORB_ERR_PARAM;
    if (nl == 0) return ORB_OK;
    if (hipSetDevice(left->device) != hipSuccess) return ORB_ERR_DEVICE;
    SBuf<orb_keypoint> bkl, bkr;
    SBuf<uint8_t> bdl, bdr;
    SBuf<int32_t> bn, bsad;
    SBuf<float> bur, bdp;
    if (bkl.alloc(nl) || bkr.alloc(nr) || bdl.alloc((size_t)nl * 32) || bdr.alloc((size_t)nr * 32) || bn.alloc(2) ||
        bsad.alloc(nl) || bur.alloc(nl) || bdp.alloc(nl))
        return ORB_ERR_DEVICE;
    const int32_t ns[2] = {nl, nr};
    ORB_CHECK(hipMemcpy(bkl.p, kl, nl * sizeof(orb_keypoint), hipMemcpyHostToDevice));
    if (nr) ORB_CHECK(hipMemcpy(bkr.p, kr, nr * sizeof(orb_keypoint), hipMemcpyHostToDevice));
    ORB_CHECK(hipMemcpy(bdl.p, dl, (size_t)nl * 32, hipMemcpyHostToDevice));
    if (nr) ORB_CHECK(hipMemcpy(bdr.p, dr, (size_t)nr * 32, hipMemcpyHostToDevice));
    ORB_CHECK(hipMemcpy(bn.p, ns, sizeof(ns), hipMemcpyHostToDevice));
    StereoArgs a;
    // the single-image path keeps level 0 in plan.d_in (pitch in_pitch)
    a.L = pyr_view(left, left->plan.d_in, 0, (int)left->plan.in_pitch, 0);
    a.R = pyr_view(right, right->plan.d_in, 0, (int)right->plan.in_pitch, 0);
    a.kl = bkl.p;
    a.dl = bdl.p;
    a.nl = bn.p;
    a.kr = bkr.p;
    a.dr = bdr.p;
    a.nr = bn.p + 1;
    a.kstride = 0;
    a.mb = mb;
    a.mbf = mbf;
    a.uright = bur.p;
    a.depth = bdp.p;
    a.sad = bsad.p;
    a.ostride = 0;
    a.rows = left->plan.lv[0].h;
    size_t off_ints;
    row_table_sizes(left, 1, a.rows, nr, off_ints, a.list_stride);
    SBuf<int> btab;
    if (btab.alloc(off_ints + a.list_stride)) return ORB_ERR_DEVICE;
    a.row_off = btab.p;
    a.row_list = btab.p + off_ints;
    const int rc = launch_stereo(a, left, 1, nl, 0);
    if (rc) return rc;
    ORB_CHECK(hipMemcpy(uright, bur.p, nl * sizeof(float), hipMemcpyDeviceToHost));
    ORB_CHECK(hipMemcpy(depth, bdp.p, nl * sizeof(float), hipMemcpyDeviceToHost));
    return ORB_OK;
}

int orbs_knn_match2(const uint8_t* query, int nq, const uint8_t* train, int nt, int32_t* idx, int32_t* dist,
                    int device) {
    if (nq < 0 || nt < 0 || (nq && (!query || !idx || !dist)) || (nt && !train)) return ORB_ERR_PARAM;
    if (nq == 0) return ORB_OK;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return ORB_ERR_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return ORB_ERR_DEVICE;
    const long long stride = std::max(nq, nt);
    SBuf<uint8_t> bq, bt;
    SBuf<int32_t> bi, bd, bl, bn;
    if (bq.alloc(stride * 32) || bt.alloc(stride * 32) || bi.alloc(stride * 2) || bd.alloc(stride * 2) ||
        bl.alloc(stride) || bn.alloc(4))
        return ORB_ERR_DEVICE;
    const int32_t ns[4] = {0, nq, 0, nt};
    ORB_CHECK(hipMemcpy(bq.p, query, (size_t)nq * 32, hipMemcpyHostToDevice));
    if (nt) ORB_CHECK(hipMemcpy(bt.p, train, (size_t)nt * 32, hipMemcpyHostToDevice));
    ORB_CHECK(hipMemcpy(bn.p, ns, sizeof(ns), hipMemcpyHostToDevice));
    KnnArgs a{bq.p, bt.p, bn.p, bn.p + 1, bn.p + 2, bn.p + 3, stride, 0.7, bi.p, bd.p, bl.p};
    ORB_LAUNCH(k_knn2, dim3((nq + 255) / 256, 1), dim3(256), 0, 0, a);
    ORB_CHECK(hipGetLastError());
    ORB_CHECK(hipMemcpy(idx, bi.p, (size_t)nq * 2 * sizeof(int32_t), hipMemcpyDeviceToHost));
    ORB_CHECK(hipMemcpy(dist, bd.p, (size_t)nq * 2 * sizeof(int32_t), hipMemcpyDeviceToHost));
    return ORB_OK;
}

int orbs_fisheye_stereo_candidates_batch_device(int npairs, int left0, int right0, const uint8_t* d_desc,
                                                const int32_t* d_n, const int32_t* d_mono, int cap, double ratio,
                                                int32_t* d_idx, int32_t* d_dist, int32_t* d_l2r, void* stream) {
    if (npairs <= 0 || left0 < 0 || right0 < 0 || !d_desc || !d_n || !d_mono || cap <= 0 || !d_idx || !d_dist ||
        !d_l2r)
        return ORB_ERR_PARAM;
    // left pair p: rows [mono[left0+p], n[left0+p]) of frame left0+p; right likewise
    KnnArgs a;
    a.q = d_desc + (long long)left0 * cap * 32;
    a.t = d_desc + (long long)right0 * cap * 32;
    a.q0 = d_mono + left0;
    a.qn = d_n + left0;
    a.t0 = d_mono + right0;
    a.tn = d_n + right0;
    a.stride = cap;
    a.ratio = ratio;
    a.idx = d_idx;
    a.dist = d_dist;
    a.l2r = d_l2r;
    ORB_LAUNCH(k_knn2, dim3((cap + 255) / 256, npairs), dim3(256), 0, (hipStream_t)stream, a);
    ORB_CHECK(hipGetLastError());
    return ORB_OK;
}

}  // extern "C"
