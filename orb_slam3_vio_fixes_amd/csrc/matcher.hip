// matcher.hip — MI355X-native ORBmatcher searches, Frame grid and DBoW2 descent.
//
// Replaces ORB_SLAM3::ORBmatcher (reference src/ORBmatcher.cc:43-763,
// 1676-2074), Frame::AssignFeaturesToGrid / GetFeaturesInArea (Frame.cc:385-416,
// 657-735) and TemplatedVocabulary::transform (TemplatedVocabulary.h:1217-1259).
//
// Every search has a serial dependency in the reference (a query skips frame
// features that an EARLIER query already took), so each search runs as one
// wavefront per (query set, frame): queries are visited in reference order by
// the whole wave, the candidates of one query are spread over the 64 lanes,
// Hamming distances use v_xor + v_bcnt on 8 dwords, and the best / second-best
// selection is a lexicographic (distance, candidate order) wave reduction that
// reproduces the reference's sequential `if (d < best) ... else if (d < best2)`.
// Candidate order is GetFeaturesInArea's: grid cells column-major (ix outer,
// iy inner), feature index ascending inside a cell.  The grid is a per-frame
// array of feature indices sorted by (ix*48+iy, index) built by a bitonic sort
// in LDS; scanning that array in order and testing the cell range and the
// |dx| < r, |dy| < r window yields exactly the reference's candidate list.
#include "../../include/orb_mi355x.h"
#include "common.h"
#include "orb_math.h"

#include <algorithm>
#include <atomic>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <list>
#include <map>
#include <memory>
#include <vector>

namespace orbmi {

// Host-API uploads are coalesced (h2d below): every other GPU operation of
// this file flushes the pending copy first.
static hipError_t flush_uploads();
#define KLAUNCH(K, G, B, S, ST, ...) do { (void)flush_uploads(); ORB_LAUNCH(K, G, B, S, ST, ##__VA_ARGS__); } while (0)

constexpr int kGridCols = 64, kGridRows = 48;        // Frame.h:44-45
constexpr int kThHigh = 100, kThLow = 50, kHisto = 30;   // ORBmatcher.cc:35-37

struct GridParams { float min_x, min_y, inv_w, inv_h; };

// Frame::PosInGrid (Frame.cc:725-735)
__device__ __forceinline__ int grid_cell(const orb_keypoint& k, const GridParams& g) {
    const int gx = (int)roundf((k.x - g.min_x) * g.inv_w);
    const int gy = (int)roundf((k.y - g.min_y) * g.inv_h);
    if (gx < 0 || gx >= kGridCols || gy < 0 || gy >= kGridRows) return -1;
    return gx * kGridRows + gy;
}

__device__ __forceinline__ int hamming32(const uint4 a0, const uint4 a1, const uint8_t* b) {
    const uint4 b0 = *(const uint4*)b, b1 = *(const uint4*)(b + 16);
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ __forceinline__ void wave_sync_m() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------------------
// k_grid: AssignFeaturesToGrid for a batch of frames.  Output per frame: the
// feature indices sorted by (cell, index), packed (cell << 16 | index), and
// their count (features outside the grid are dropped, as PosInGrid does).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_grid(const orb_keypoint* __restrict__ kps, const int* __restrict__ n,
                                              int cap, GridParams g, uint32_t* __restrict__ sorted,
                                              int* __restrict__ count, int sort_cap,
                                              uint32_t* __restrict__ l0sorted, int* __restrict__ l0count) {
    extern __shared__ __attribute__((aligned(16))) uint32_t keys[];
    const int f = blockIdx.x, tid = threadIdx.x;
    const int nf = min(n[f], cap);
    for (int i = tid; i < sort_cap; i += blockDim.x) {
        uint32_t v = 0xffffffffu;
        if (i < nf) {
            const int c = grid_cell(kps[(long long)f * cap + i], g);
            if (c >= 0) v = ((uint32_t)c << 16) | (uint32_t)i;
        }
        keys[i] = v;
    }
    __syncthreads();
    for (int k = 2; k <= sort_cap; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < sort_cap; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint32_t a = keys[i], b = keys[ixj];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) { keys[i] = b; keys[ixj] = a; }
                }
            }
            __syncthreads();
        }
    int valid = 0;
    for (int i = tid; i < sort_cap; i += blockDim.x) {
        const uint32_t v = keys[i];
        if (v != 0xffffffffu) { sorted[(long long)f * cap + i] = v; ++valid; }
    }
    valid = wave_sum(valid);
    __shared__ int wsum[4];
    if (lane_id() == 0) wsum[wave_id()] = valid;
    __syncthreads();
    if (tid == 0) count[f] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    // the octave-0 subsequence (SearchForInitialization queries level 0 only, ORBmatcher.cc:664-668)
    if (l0sorted && wave_id() == 0) {
        const int tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        int nl = 0;
        for (int base = 0; base < tot; base += kWave) {
            const int i = base + lane_id();
            bool keep = false;
            uint32_t v = 0;
            if (i < tot) { v = keys[i]; keep = kps[(long long)f * cap + (v & 0xffff)].octave == 0; }
            const uint64_t m = __ballot(keep);
            if (keep) l0sorted[(long long)f * cap + nl + mask_rank(m)] = v;
            nl += __popcll(m);
        }
        if (lane_id() == 0) l0count[f] = nl;
    }
}

// k_grid_cs: the same grid order by a counting sort, one frame per block:
// per-cell counts (LDS atomics), their exclusive scan (= the cell-start table
// of k_cell_start below), atomic placement, then an insertion sort of each
// cell's few entries restores index order inside the cell.  cellstart may be
// NULL; l0sorted / l0count as in k_grid.
constexpr int kGridCells = 64 * 48;

static size_t grid_cs_lds(int cap) { return (size_t)(2 * kGridCells + 1) * 4 + (size_t)cap * 6 + 64; }

__global__ __launch_bounds__(256) void k_grid_cs(const orb_keypoint* __restrict__ kps, const int* __restrict__ n,
                                                 int cap, GridParams g, uint32_t* __restrict__ sorted,
                                                 int* __restrict__ count, int* __restrict__ cellstart,
                                                 uint32_t* __restrict__ l0sorted, int* __restrict__ l0count) {
    extern __shared__ __attribute__((aligned(16))) int glds[];
    __shared__ int tmp[8];
    int* start = glds;                                   // kGridCells + 1
    int* cursor = start + kGridCells + 1;                // kGridCells
    uint32_t* out = (uint32_t*)(cursor + kGridCells);    // cap
    short* cellof = (short*)(out + cap);                 // cap
    const int f = blockIdx.x, tid = threadIdx.x, T = blockDim.x;
    const int nf = min(n[f], cap);
    const orb_keypoint* K = kps + (long long)f * cap;
    for (int c = tid; c < kGridCells; c += T) start[c] = 0;
    __syncthreads();
    for (int i = tid; i < nf; i += T) {
        const int c = grid_cell(K[i], g);
        cellof[i] = (short)c;
        if (c >= 0) atomicAdd(&start[c], 1);
    }
    __syncthreads();
    const int total = block_excl_scan(start, kGridCells, tmp);
    if (tid == 0) start[kGridCells] = total;
    for (int c = tid; c < kGridCells; c += T) cursor[c] = start[c];
    __syncthreads();
    for (int i = tid; i < nf; i += T) {
        const int c = cellof[i];
        if (c >= 0) out[atomicAdd(&cursor[c], 1)] = ((uint32_t)c << 16) | (uint32_t)i;
    }
    __syncthreads();
    for (int c = tid; c < kGridCells; c += T) {          // index order inside each cell
        const int b = start[c], e = start[c + 1];
        for (int x = b + 1; x < e; ++x) {
            const uint32_t v = out[x];
            int y = x - 1;
            while (y >= b && out[y] > v) { out[y + 1] = out[y]; --y; }
            out[y + 1] = v;
        }
    }
    __syncthreads();
    for (int j = tid; j < total; j += T) sorted[(long long)f * cap + j] = out[j];
    if (tid == 0) count[f] = total;
    if (cellstart)
        for (int c = tid; c <= kGridCells; c += T) cellstart[(long long)f * (kGridCells + 1) + c] = start[c];
    // the octave-0 subsequence (SearchForInitialization queries level 0 only, ORBmatcher.cc:664-668)
    if (l0sorted && wave_id() == 0) {
        int nl = 0;
        for (int base = 0; base < total; base += kWave) {
            const int i = base + lane_id();
            bool keep = false;
            uint32_t v = 0;
            if (i < total) { v = out[i]; keep = K[v & 0xffff].octave == 0; }
            const uint64_t m = __ballot(keep);
            if (keep) l0sorted[(long long)f * cap + nl + mask_rank(m)] = v;
            nl += __popcll(m);
        }
        if (lane_id() == 0) l0count[f] = nl;
    }
}

// GetFeaturesInArea cell range (Frame.cc:661-689); false = empty.
struct CellRange { int x0, x1, y0, y1; };
__device__ __forceinline__ bool cell_range(float x, float y, float r, const GridParams& g, CellRange& cr) {
    cr.x0 = max(0, (int)floorf((x - g.min_x - r) * g.inv_w));
    if (cr.x0 >= kGridCols) return false;
    cr.x1 = min(kGridCols - 1, (int)ceilf((x - g.min_x + r) * g.inv_w));
    if (cr.x1 < 0) return false;
    cr.y0 = max(0, (int)floorf((y - g.min_y - r) * g.inv_h));
    if (cr.y0 >= kGridRows) return false;
    cr.y1 = min(kGridRows - 1, (int)ceilf((y - g.min_y + r) * g.inv_h));
    if (cr.y1 < 0) return false;
    return true;
}

// ---------------------------------------------------------------------------
// Cell-start table of a grid order: cs[c] = first position of `gsorted` whose
// cell is >= c, c in [0, 3072].  The candidates of GetFeaturesInArea
// (ix outer, iy inner, index order inside a cell) are then, per grid column
// gx in [x0, x1], the contiguous run [cs[gx*48 + y0], cs[gx*48 + y1 + 1]) of
// the grid order, and the runs concatenated in column order ARE the
// reference's candidate list -- no scan over the whole frame per query.
// ---------------------------------------------------------------------------
constexpr int kCells = kGridCols * kGridRows;

__global__ __launch_bounds__(256) void k_cell_start(const uint32_t* __restrict__ gsorted,
                                                    const int* __restrict__ gcount, int cap, int* __restrict__ cs) {
    const int f = blockIdx.x;
    const uint32_t* gs = gsorted + (long long)f * cap;
    const int gn = gcount[f];
    int* out = cs + (long long)f * (kCells + 1);
    for (int c = threadIdx.x; c <= kCells; c += blockDim.x) {
        const uint32_t key = (uint32_t)c << 16;
        int lo = 0, hi = gn;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (gs[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        out[c] = lo;
    }
}

// Lane l holds the run of grid column x0 + l (the grid has 64 columns, so one
// wave covers every column range): its start `lo` in the grid order and its
// offset `off` in the concatenated candidate list; `total` = list length.
struct AreaRuns { int lo, off, total; };

__device__ __forceinline__ AreaRuns area_runs(const int* cs, const CellRange& cr) {
    const int lane = lane_id();
    int lo = 0, len = 0;
    if (lane <= cr.x1 - cr.x0) {
        const int c = (cr.x0 + lane) * kGridRows;
        lo = cs[c + cr.y0];
        len = cs[c + cr.y1 + 1] - lo;
    }
    int inc = len;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const int t = __shfl_up(inc, o, kWave);
        if (lane >= o) inc += t;
    }
    return AreaRuns{lo, inc - len, __shfl(inc, kWave - 1, kWave)};
}

// Grid-order position of candidate t (0 <= t < total): the run s is the last
// lane with off_s <= t (offsets are non-decreasing).  Every lane takes part.
__device__ __forceinline__ int area_pos(const AreaRuns& r, int t) {
    int s = 0;
#pragma unroll
    for (int step = kWave / 2; step > 0; step >>= 1) {
        const int o = __shfl(r.off, s + step, kWave);
        if (o <= t) s += step;
    }
    return __shfl(r.lo, s, kWave) + (t - __shfl(r.off, s, kWave));
}

// Running best / second-best over a candidate stream in reference order.
struct Best2 {
    int best, best2, idx, lvl, lvl2;
};

// Merge one wave chunk (candidate of this lane: dist d (INT_MAX = none), feature
// index fi, level lv; lanes in stream order) into the running state with the
// exact semantics of the sequential loop
//   if (d < best) {best2 = best; lvl2 = lvl; best = d; lvl = lv; idx = fi;}
//   else if (d < best2) {best2 = d; lvl2 = lv;}
__device__ __forceinline__ void merge_chunk(Best2& st, int d, int fi, int lv) {
    // chunk minimum and its first lane (DPP reduction, readlane broadcasts)
    const int m = wave_min(d, INT_MAX);
    if (m == INT_MAX) return;
    const uint64_t at = __ballot(d == m);
    const int first = __ffsll((long long)at) - 1;
    const int fi_m = __builtin_amdgcn_readlane(fi, first), lv_m = __builtin_amdgcn_readlane(lv, first);
    // chunk second: min over lanes other than `first`, with its first lane
    const int d2 = lane_id() == first ? INT_MAX : d;
    const int m2 = wave_min(d2, INT_MAX);
    int lv_m2 = -1;
    if (m2 != INT_MAX) {
        const uint64_t at2 = __ballot(d2 == m2);
        lv_m2 = __builtin_amdgcn_readlane(lv, __ffsll((long long)at2) - 1);
    }
    // sequential merge: the chunk's elements come after the running ones.
    // New best: strictly smaller chunk min replaces; the old best becomes a
    // second candidate.  The second-smallest of the union with the level of
    // the element the sequential loop would have recorded.
    if (m < st.best) {
        // old best is pushed to second unless the chunk's own second is smaller
        int nb2 = st.best, nl2 = st.lvl;
        if (m2 < nb2) { nb2 = m2; nl2 = lv_m2; }
        st.best2 = nb2; st.lvl2 = nl2;
        st.best = m; st.lvl = lv_m; st.idx = fi_m;
    } else {
        // chunk min m >= best: it competes for second (first lane of m first)
        if (m < st.best2) { st.best2 = m; st.lvl2 = lv_m; }
    }
}

__host__ __device__ __forceinline__ int rot_bin(float a1, float a2) {
    float rot = a1 - a2;
    if (rot < 0.0f) rot += 360.0f;
    int bin = (int)roundf(rot * (1.0f / kHisto));
    if (bin == kHisto) bin = 0;
    return bin;
}

// hist[b] += 1 for every active lane's bin b (b < 0: none), one LDS atomic
// per distinct bin of the wave: the matches of a keyframe share one or two
// rotation bins, and 64 same-address LDS atomics serialise
__device__ __forceinline__ void hist_add_wave(int* hist, int b) {
    for (uint64_t act = __ballot(b >= 0); act;) {
        const int l = __ffsll((long long)act) - 1;
        const int b0 = __builtin_amdgcn_readlane(b, l);
        const uint64_t m = __ballot(b == b0) & act;
        if (lane_id() == l) atomicAdd(&hist[b0], __popcll(m));
        act &= ~m;
    }
}

// ComputeThreeMaxima (ORBmatcher.cc:2012-2053)
__host__ __device__ __forceinline__ void three_maxima(const int* h, int& i1, int& i2, int& i3) {
    int m1 = 0, m2 = 0, m3 = 0;
    i1 = i2 = i3 = -1;
    for (int i = 0; i < kHisto; ++i) {
        const int s = h[i];
        if (s > m1) { m3 = m2; m2 = m1; m1 = s; i3 = i2; i2 = i1; i1 = i; }
        else if (s > m2) { m3 = m2; m2 = s; i3 = i2; i2 = i; }
        else if (s > m3) { m3 = s; i3 = i; }
    }
    if (m2 < 0.1f * (float)m1) { i2 = -1; i3 = -1; }
    else if (m3 < 0.1f * (float)m1) { i3 = -1; }
}

// The same from a whole wave (every lane active; every lane gets the result):
// the serial scan's strict comparisons in ascending bin order rank the nonzero
// bins by (count descending, bin ascending), so the three are three wave maxima
// of count << 8 | (255 - bin) -- three DPP reductions instead of a 30-step
// chain of dependent LDS reads on one lane.
__device__ __forceinline__ void three_maxima_wave(const int* h, int& i1, int& i2, int& i3) {
    const int l = lane_id();
    const int c = l < kHisto ? h[l] : 0;
    uint32_t key = c > 0 ? ((uint32_t)c << 8) | (uint32_t)(255 - l) : 0u;
    uint32_t k[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        k[t] = ~wave_min(~key, 0xffffffffu);
        if (key == k[t]) key = 0u;
    }
    const int m1 = (int)(k[0] >> 8), m2 = (int)(k[1] >> 8), m3 = (int)(k[2] >> 8);
    i1 = k[0] ? 255 - (int)(k[0] & 0xff) : -1;
    i2 = k[1] ? 255 - (int)(k[1] & 0xff) : -1;
    i3 = k[2] ? 255 - (int)(k[2] & 0xff) : -1;
    if (m2 < 0.1f * (float)m1) { i2 = -1; i3 = -1; }
    else if (m3 < 0.1f * (float)m1) { i3 = -1; }
}

// ---------------------------------------------------------------------------
// SearchForInitialization (ORBmatcher.cc:648-763) in two kernels.
//
// The only order dependence is the skip rule `if (vMatchedDistance[i2] <=
// dist) continue;` (:687-688): the best and second-best of F1 feature i1 are
// the first two elements, in (distance, candidate order), of its candidates
// that survive that rule under the state left by i1-1.  k_sfi_topk computes,
// for every level-0 F1 feature in parallel, its candidate count and its
// kTopK smallest (distance, order) pairs (k_sfi_topk_st / k_sfi_topk).
// k_sfi_resolve then walks F1 in order with one wave per frame pair; each
// step filters <= kTopK entries
// against vMatchedDistance.  When fewer than two entries survive and the list
// was truncated, the wave re-scans the full candidate list (exact fallback).
// ---------------------------------------------------------------------------
constexpr int kTopK = 8;
constexpr uint32_t kNoKey = 0xffffffffu;

struct SfiArgs {
    const orb_keypoint* kps;
    const uint8_t* desc;
    const int* n;
    int cap;
    const uint32_t* gsorted;   // per frame: level-0 features in grid order (k_grid l0 list)
    const int* gcount;
    const int* pair_f1;      // per pair: frame index of F1 / F2
    const int* pair_f2;
    const float* prev_in;    // [pair][cap][2] or null (= F1 keypoint positions)
    float* prev_out;         // [pair][cap][2] or null
    GridParams g;
    float window, ratio;
    int check_ori;
    uint32_t* topk;          // [pair][cap][kTopK]  (rotation bin << 25 | dist << 16 | F2 feature), in (dist, grid order)
    int* ncand;              // [pair][cap]  (-1: not a query)
    int32_t* matches;        // [pair][cap]
    int32_t* nmatches;       // [pair]
};

// the K smallest keys seen so far, ascending (keys are unique): with
// k0 <= k1 <= ..., the new k_t is med3(k_{t-1}, k_t, key) -- independent ops
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
template <int K>
__device__ __forceinline__ void topk_push(uint32_t (&kk)[K], uint32_t key) {
    uint32_t n[K];
    n[0] = min(kk[0], key);
#pragma unroll
    for (int t = 1; t < K; ++t) n[t] = umed3(kk[t - 1], kk[t], key);
#pragma unroll
    for (int t = 0; t < K; ++t) kk[t] = n[t];
}

__device__ __forceinline__ void query_pos(const SfiArgs& a, int pr, int i1, const orb_keypoint& k1, float& px,
                                          float& py) {
    px = k1.x; py = k1.y;
    if (a.prev_in) {
        px = a.prev_in[((long long)pr * a.cap + i1) * 2];
        py = a.prev_in[((long long)pr * a.cap + i1) * 2 + 1];
    }
}

// distance of level-0 list entry j (F2's level-0 features in grid order:
// GetFeaturesInArea(.., level1, level1) with level1 = 0 keeps octave 0 only,
// :668) to query i1 if it is a candidate, else INT_MAX
__device__ __forceinline__ int cand_dist(const int* list, int j, const CellRange& cr, float px, float py, float r,
                                         const orb_keypoint* K2, const uint8_t* D2, uint4 q0, uint4 q1) {
    const int v = list[j];
    const int cell = v >> 16, gx = cell / kGridRows, gy = cell - gx * kGridRows;
    if (gx < cr.x0 || gx > cr.x1 || gy < cr.y0 || gy > cr.y1) return INT_MAX;
    const int fi = v & 0xffff;
    const orb_keypoint k2 = K2[fi];
    if (!(fabsf(k2.x - px) < r && fabsf(k2.y - py) < r)) return INT_MAX;
    return hamming32(q0, q1, D2 + (long long)fi * 32);
}

// The queries [qbeg + wave * qpw, + qpw) of pair pr against an F2 level-0 list
// of any length (read from global memory): each lane keeps the kTopK smallest
// keys (distance << 16 | list position) of the candidates at positions lane,
// lane + 64, ... in registers (one min and kTopK - 1 med3 per candidate), then
// kTopK rounds of wave minimum over the lanes' heads draw the query's kTopK
// smallest -- every key of the query's top-K is in its own lane's top-K.  No
// LDS, so frames of any keypoint count (16-bit list positions) take it.
__device__ void sfi_topk_lanes(const SfiArgs& a, int pr, int qbeg, int qpw) {
    const int lane = lane_id(), wv = wave_id();
    const int f1 = a.pair_f1[pr], f2 = a.pair_f2[pr];
    const int n1 = min(a.n[f1], a.cap);
    const int* list = (const int*)(a.gsorted + (long long)f2 * a.cap);
    const int nl = a.gcount[f2];
    const orb_keypoint* K1 = a.kps + (long long)f1 * a.cap;
    const orb_keypoint* K2 = a.kps + (long long)f2 * a.cap;
    const uint8_t* D1 = a.desc + (long long)f1 * a.cap * 32;
    const uint8_t* D2 = a.desc + (long long)f2 * a.cap * 32;
    const float r = a.window;
    for (int t = 0; t < qpw; ++t) {
        const int i1 = qbeg + wv * qpw + t;
        if (i1 >= n1) break;
        uint32_t* tk = a.topk + ((long long)pr * a.cap + i1) * kTopK;
        int* nc = a.ncand + (long long)pr * a.cap + i1;
        const orb_keypoint k1 = K1[i1];
        float px, py;
        query_pos(a, pr, i1, k1, px, py);
        CellRange cr;
        if (k1.octave > 0 || !cell_range(px, py, r, a.g, cr)) {
            if (lane == 0) *nc = -1;
            continue;
        }
        const uint4 q0 = *(const uint4*)(D1 + (long long)i1 * 32), q1 = *(const uint4*)(D1 + (long long)i1 * 32 + 16);
        uint32_t kk[kTopK];
#pragma unroll
        for (int k = 0; k < kTopK; ++k) kk[k] = kNoKey;
        int cnt = 0;
        for (int base = 0; base < nl; base += kWave) {
            const int j = base + lane;
            const int d = j < nl ? cand_dist(list, j, cr, px, py, r, K2, D2, q0, q1) : INT_MAX;
            cnt += __popcll(__ballot(d != INT_MAX));
            if (d != INT_MAX) topk_push(kk, ((uint32_t)d << 16) | (uint32_t)j);
        }
        const int rounds = min(cnt, kTopK);
        uint32_t mine = kNoKey;   // lane k < kTopK: the k-th draw
        for (int k = 0; k < rounds; ++k) {
            const uint32_t mn = wave_min(kk[0], 0xffffffffu);
            if (kk[0] == mn) {
#pragma unroll
                for (int q = 0; q + 1 < kTopK; ++q) kk[q] = kk[q + 1];
                kk[kTopK - 1] = kNoKey;
            }
            if (lane == k) mine = mn;
        }
        // out: rotation bin, distance and F2 feature index (the list position
        // only ordered the ties), one store per draw
        if (lane < kTopK) {
            uint32_t o = kNoKey;
            if (mine != kNoKey) {
                const uint32_t fi = (uint32_t)list[mine & 0xffffu] & 0xffffu;
                const uint32_t bn = a.check_ori ? (uint32_t)rot_bin(k1.angle, K2[fi].angle) : 0u;
                o = (bn << 25) | (mine & 0xffff0000u) | fi;
            }
            tk[lane] = o;
        }
        if (lane == 0) *nc = cnt;
    }
}

// k_sfi_topk_st: the top-K lists with F2's level-0 features staged in
// LDS once per block of 64 queries (cell, position and descriptor in grid
// order: 44 bytes each), so a query's candidate scan reads only LDS, and the
// K smallest keys are drawn from registers (a lane holds the keys of its list
// positions lane, lane + 64, ...; kStIt positions at most, longer lists take
// sfi_topk_lanes).  Rounds stop after min(count, K) draws.
#ifndef ORB_SFI_QSTAGE
#define ORB_SFI_QSTAGE 1   // k_sfi_topk_st stages its 64 queries in LDS with the F2 list
#endif
constexpr int kStIt = 4;                  // level-0 lists of <= 256 features
constexpr int kStQ = 64;                  // queries per block
__global__ __launch_bounds__(256) void k_sfi_topk_st(SfiArgs a) {
    extern __shared__ __attribute__((aligned(16))) int lds[];
    uint4* d2s = (uint4*)lds;                                   // 2 * kStIt * 64 (descriptor halves)
    float2* xy2 = (float2*)(d2s + 2 * kStIt * kWave);           // kStIt * 64
    int* list = (int*)(xy2 + kStIt * kWave);                    // kStIt * 64
    float* an2 = (float*)(list + kStIt * kWave);                // kStIt * 64
#if ORB_SFI_QSTAGE
    // the block's 64 queries: descriptor halves, (position, angle, octave)
    uint4* qd = (uint4*)(an2 + kStIt * kWave);                  // 2 * kStQ
    float4* qk = (float4*)(qd + 2 * kStQ);                      // kStQ
#endif
    const int pr = blockIdx.x, lane = lane_id(), wv = wave_id(), tid = threadIdx.x;
    const int f1 = a.pair_f1[pr], f2 = a.pair_f2[pr];
    const int n1 = min(a.n[f1], a.cap);
    const int q0 = blockIdx.y * kStQ;
    const orb_keypoint* K1 = a.kps + (long long)f1 * a.cap;
    __shared__ int s_any;
    if (tid == 0) s_any = 0;
    __syncthreads();
    if (tid < kStQ && q0 + tid < n1 && K1[q0 + tid].octave == 0) s_any = 1;
    __syncthreads();
    if (!s_any) {
        if (tid < kStQ && q0 + tid < n1) a.ncand[(long long)pr * a.cap + q0 + tid] = -1;
        return;
    }
    const orb_keypoint* K2 = a.kps + (long long)f2 * a.cap;
    const uint8_t* D1 = a.desc + (long long)f1 * a.cap * 32;
    const uint8_t* D2 = a.desc + (long long)f2 * a.cap * 32;
    const int nl = a.gcount[f2];
    if (nl > kStIt * kWave) {             // a long level-0 list: per-lane top-K from global memory
        sfi_topk_lanes(a, pr, q0, kStQ / 4);
        return;
    }
    {
#if ORB_SFI_QSTAGE
        // (a query's keypoint, position and descriptor were three dependent
        // global round trips at the head of every query of a wave's 16):
        // loaded here, in flight with the F2 list's loads, stored after them
        const bool qs = tid < kStQ && q0 + tid < n1;
        orb_keypoint qk1{};
        uint4 qd0{}, qd1{};
        if (qs) {
            qk1 = K1[q0 + tid];
            qd0 = *(const uint4*)(D1 + (long long)(q0 + tid) * 32);
            qd1 = *(const uint4*)(D1 + (long long)(q0 + tid) * 32 + 16);
        }
#endif
        const uint32_t* gs = a.gsorted + (long long)f2 * a.cap;
        for (int j = tid; j < nl; j += 256) {
            const int v = (int)gs[j], fi = v & 0xffff;
            list[j] = v;
            xy2[j] = make_float2(K2[fi].x, K2[fi].y);
            an2[j] = K2[fi].angle;
            d2s[2 * j] = *(const uint4*)(D2 + (long long)fi * 32);
            d2s[2 * j + 1] = *(const uint4*)(D2 + (long long)fi * 32 + 16);
        }
#if ORB_SFI_QSTAGE
        if (qs) {
            float px, py;
            query_pos(a, pr, q0 + tid, qk1, px, py);
            qk[tid] = make_float4(px, py, qk1.angle, __int_as_float(qk1.octave));
            qd[2 * tid] = qd0;
            qd[2 * tid + 1] = qd1;
        }
#endif
    }
    __syncthreads();
    const float r = a.window;
    for (int t = 0; t < kStQ / 4; ++t) {
        const int i1 = q0 + wv * (kStQ / 4) + t;
        if (i1 >= n1) break;
        uint32_t* tk = a.topk + ((long long)pr * a.cap + i1) * kTopK;
        int* nc = a.ncand + (long long)pr * a.cap + i1;
#if ORB_SFI_QSTAGE
        const float4 kq = qk[i1 - q0];
        const float px = kq.x, py = kq.y;
        struct { float angle; int octave; } k1{kq.z, __float_as_int(kq.w)};
#else
        const orb_keypoint k1 = K1[i1];
        float px, py;
        query_pos(a, pr, i1, k1, px, py);
#endif
        CellRange cr;
        if (k1.octave > 0 || !cell_range(px, py, r, a.g, cr)) {
            if (lane == 0) *nc = -1;
            continue;
        }
#if ORB_SFI_QSTAGE
        const uint4 qa = qd[2 * (i1 - q0)], qb = qd[2 * (i1 - q0) + 1];
#else
        const uint4 qa = *(const uint4*)(D1 + (long long)i1 * 32), qb = *(const uint4*)(D1 + (long long)i1 * 32 + 16);
#endif
        uint32_t kv[kStIt];
        int cnt = 0;
#pragma unroll
        for (int it = 0; it < kStIt; ++it) {
            const int j = it * kWave + lane;
            kv[it] = kNoKey;
            if (j < nl) {
                const int v = list[j];
                const int cell = v >> 16, gx = cell / kGridRows, gy = cell - gx * kGridRows;
                const float2 p2 = xy2[j];
                if (gx >= cr.x0 && gx <= cr.x1 && gy >= cr.y0 && gy <= cr.y1 && fabsf(p2.x - px) < r &&
                    fabsf(p2.y - py) < r) {
                    const uint4 b0 = d2s[2 * j], b1 = d2s[2 * j + 1];
                    const int d = __popc(qa.x ^ b0.x) + __popc(qa.y ^ b0.y) + __popc(qa.z ^ b0.z) +
                                  __popc(qa.w ^ b0.w) + __popc(qb.x ^ b1.x) + __popc(qb.y ^ b1.y) +
                                  __popc(qb.z ^ b1.z) + __popc(qb.w ^ b1.w);
                    kv[it] = ((uint32_t)d << 16) | (uint32_t)j;
                }
            }
            cnt += __popcll(__ballot(kv[it] != kNoKey));
        }
        const int rounds = min(cnt, kTopK);
        uint32_t mine = kNoKey;   // lane k < kTopK: the k-th draw
        for (int k = 0; k < rounds; ++k) {
            uint32_t mn = kv[0];
#pragma unroll
            for (int it = 1; it < kStIt; ++it) mn = min(mn, kv[it]);
            mn = wave_min(mn, 0xffffffffu);
#pragma unroll
            for (int it = 0; it < kStIt; ++it)
                if (kv[it] == mn) kv[it] = kNoKey;
            if (lane == k) mine = mn;
        }
        // out: rotation bin, distance and F2 feature index (the list position
        // only ordered the ties), one store per draw
        if (lane < kTopK) {
            uint32_t o = kNoKey;
            if (mine != kNoKey) {
                const int j = (int)(mine & 0xffffu);
                const uint32_t bn = a.check_ori ? (uint32_t)rot_bin(k1.angle, an2[j]) : 0u;
                o = (bn << 25) | (mine & 0xffff0000u) | ((uint32_t)list[j] & 0xffffu);
            }
            tk[lane] = o;
        }
        if (lane == 0) *nc = cnt;
    }
}

// One block per pair: the serial pass runs on wave 0; the four waves stage
// what it reads into LDS first (the pair's level-0 list, the query list) and
// finish the orientation filter and the outputs after it.  The top-K lists
// stay in global memory: lanes 8t..8t+7 of the wave hold the keys of query
// j0 + t of a run of 8 queries (one gather per run), the next run is in
// flight while this one is walked, and query t's step ballots only its own
// lanes -- its keys are already in (distance, grid order) and carry the F2
// feature and the rotation bin.  The serial state (matched distance and
// F2 -> F1 match, packed) and the matches live in LDS: ~17 bytes per
// keypoint, so the block does not hold off the extraction's blocks it runs
// beside.
constexpr int kSfiThreads = 256;
#ifndef ORB_SFI_PRIO
#define ORB_SFI_PRIO 1
#endif
#ifndef ORB_SFI_SPEC
#define ORB_SFI_SPEC 1   // speculative 8-query runs (0: the serial step-per-query walk)
#endif
#ifndef ORB_SFI_CONFL
#define ORB_SFI_CONFL 3  // the run's conflict scan as unrolled readlanes, each query's stop by a DPP group OR, a conflict only where a claim kills a read entry (2: any read of a claimed feature; 1: by a ballot; 0: a loop over the accepting queries)
#endif
#ifndef ORB_SFI_DEPTH
#define ORB_SFI_DEPTH 3  // runs of keys in registers: the current one and the next ones in flight
#endif
constexpr int kSfiDepth = ORB_SFI_DEPTH;
#ifndef ORB_SFI_STAGE
#define ORB_SFI_STAGE 256   // queries whose top-K keys are staged in LDS before the walk (32 B each)
#endif
constexpr int kSfiStage = ORB_SFI_STAGE;
#ifndef ORB_SFI_STAGE2
#define ORB_SFI_STAGE2 256  // F2 level-0 list entries staged in LDS for the exact rescans (44 B each)
#endif
constexpr int kSfiStage2 = ORB_SFI_STAGE2;
// LDS of k_sfi_resolve: the state (9 B a keypoint), the staged keys, the
// staged F2 list (entry, position, descriptor)
__host__ __device__ inline size_t sfi_lds_base(int cap) { return ((size_t)cap * 9 + 128 + 15) / 16 * 16; }
__host__ __device__ inline size_t sfi_lds_bytes(int cap) {
    return sfi_lds_base(cap) + (size_t)kSfiStage * kTopK * 4 + (size_t)kSfiStage2 * (32 + 8 + 4);
}
static_assert(kSfiDepth >= 2, "the current run and at least one in flight");
constexpr uint32_t kMdNone = 0xffff0000u;    // md21: no match yet (distance field 0xffff)
#ifdef ORB_SFI_COUNT
// walk statistics (tools/sfi_counts.py): rounds, rounds that committed fewer
// than 8 queries, exact rescans, queries, committed claims
// and shader cycles per walk phase (g_sfi_cnt[8..15]: decide, conflict
// scan, commit, in-place state update, rescan, run advance, prologue, the
// whole block)
__device__ unsigned long long g_sfi_cnt[16];
extern "C" int orbm_debug_sfi_counts(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sfi_cnt), sizeof(g_sfi_cnt)) != hipSuccess) return -4;
    if (reset) {
        static unsigned long long z[16];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_sfi_cnt), z, sizeof(z)) != hipSuccess) return -4;
    }
    return 0;
}
// (counts in registers, flushed once a block: same-address global atomics per
// step from every block had been the stamps' largest cost)
#define SFI_CNT(k, v)                                                  \
    do {                                                               \
        switch (k) {                                                   \
            case 0: sfi_c0 += (v); break;                              \
            case 1: sfi_c1 += (v); break;                              \
            case 2: sfi_c2 += (v); break;                              \
            case 3: sfi_c3 += (v); break;                              \
            default: sfi_c4 += (v); break;                             \
        }                                                              \
    } while (0)
#define SFI_TS(k)                                                      \
    do {                                                               \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();    \
        const unsigned long long d_ = t_ - sfi_tl;                     \
        sfi_tl = t_;                                                   \
        switch (k) {                                                   \
            case 0: sfi_a0 += d_; break;                               \
            case 1: sfi_a1 += d_; break;                               \
            case 2: sfi_a2 += d_; break;                               \
            case 3: sfi_a3 += d_; break;                               \
            case 4: sfi_a4 += d_; break;                               \
            case 5: sfi_a5 += d_; break;                               \
            default: sfi_a6 += d_; break;                              \
        }                                                              \
    } while (0)
#else
#define SFI_CNT(k, v) do { } while (0)
#define SFI_TS(k) do { } while (0)
#endif
// minimum over each aligned group of 8 lanes, in every lane of the group:
// quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror
__device__ __forceinline__ uint32_t grp8_min(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, false));
    return v;
}
// M12L: the F1 -> F2 matches live in LDS during the walk and go out once,
// coalesced, at the end (a global store in the walk made the next step wait
// for it: gfx9 counts stores in vmcnt, and the compiler's waits at the loop
// head drained them every step)
template <bool M12L>
__global__ __launch_bounds__(kSfiThreads) void k_sfi_resolve(SfiArgs a) {
    extern __shared__ __attribute__((aligned(16))) int lds[];
    const int pr = blockIdx.x, lane = lane_id(), tid = threadIdx.x;
#ifdef ORB_SFI_COUNT
    // (separate scalars: an array captured by the walk's lambda went to scratch)
    unsigned long long sfi_c0 = 0, sfi_c1 = 0, sfi_c2 = 0, sfi_c3 = 0, sfi_c4 = 0;
    unsigned long long sfi_a0 = 0, sfi_a1 = 0, sfi_a2 = 0, sfi_a3 = 0, sfi_a4 = 0, sfi_a5 = 0, sfi_a6 = 0;
    const unsigned long long sfi_t0 = __builtin_amdgcn_s_memtime();
    unsigned long long sfi_tl = sfi_t0;
#endif
    const int f1 = a.pair_f1[pr], f2 = a.pair_f2[pr];
    const int n1 = min(a.n[f1], a.cap), n2 = min(a.n[f2], a.cap);
    const orb_keypoint* K1 = a.kps + (long long)f1 * a.cap;
    const orb_keypoint* K2 = a.kps + (long long)f2 * a.cap;
    const uint8_t* D1 = a.desc + (long long)f1 * a.cap * 32;
    const uint8_t* D2 = a.desc + (long long)f2 * a.cap * 32;
    // LDS: the serial state, the query list and the rotation bins (9 bytes a
    // keypoint); F2's level-0 list (read only by exact rescans) and the
    // matches (written by the walk, read after the block's barrier) stay in
    // global memory
    uint32_t* md21 = (uint32_t*)lds;              // cap: matched distance << 16 | (F1 match + 1)
    int* hist = (int*)(md21 + a.cap);             // 32 (hist[31]: the final match count)
    int* qlist = hist + 32;                       // cap: query i1 | (more than kTopK candidates) << 31
    int8_t* bin1 = (int8_t*)(qlist + a.cap);      // cap
    // the first kSfiStage queries' keys (staged by all four waves before the
    // walk: the walk then does no global load for them)
    uint32_t* skeys = (uint32_t*)((uint8_t*)lds + sfi_lds_base(a.cap));
    uint4* s2desc = (uint4*)(skeys + kSfiStage * kTopK);          // [kSfiStage2][2]
    float2* s2xy = (float2*)(s2desc + 2 * kSfiStage2);             // [kSfiStage2]
    int* s2list = (int*)(s2xy + kSfiStage2);                       // [kSfiStage2]
    int32_t* const m12g = a.matches + (long long)pr * a.cap;
    int32_t* m12 = M12L ? (int32_t*)(s2list + kSfiStage2) : m12g;   // [cap] in LDS (M12L)
    const int* list = (const int*)(a.gsorted + (long long)f2 * a.cap);
    const uint32_t* topk = a.topk + (long long)pr * a.cap * kTopK;
    const int* ncand = a.ncand + (long long)pr * a.cap;
    const int nl = a.gcount[f2];
    // (4 count loads a thread in flight: a load-store loop waited on each)
    for (int i0 = tid; i0 < n1; i0 += 4 * kSfiThreads) {
        int c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) c[u] = i0 + u * kSfiThreads < n1 ? ncand[i0 + u * kSfiThreads] : 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + u * kSfiThreads;
            if (i < n1) {
                qlist[i] = c[u];
                m12[i] = -1;
                bin1[i] = -1;
            }
        }
    }
    for (int i = tid; i < n2; i += kSfiThreads) md21[i] = kMdNone;
    if (tid < 32) hist[tid] = 0;
    __syncthreads();
    if (tid < kWave) {
        // compact the queries in F1 order (in place: a round reads its 64
        // counts before it writes, and writes only below its own reads)
        int nq = 0;
        for (int base = 0; base < n1; base += kWave) {
            const int i = base + lane;
            const int c = i < n1 ? qlist[i] : -1;
            const uint64_t m = __ballot(c > 0);
            if (c > 0) qlist[nq + mask_rank(m)] = i | (c > kTopK ? (int)0x80000000 : 0);
            nq += __popcll(m);
        }
        if (lane == 0) hist[31] = nq;                // (hist[31] is zeroed again below)
    }
    __syncthreads();
#ifndef ORB_SFI_ABL
#define ORB_SFI_ABL 0   // timing ablation (tools only; wrong results): 1 = no walk, 2 = no rescan work, 3 = no conflict scan
#endif
    const int nq = ORB_SFI_ABL == 1 ? 0 : hist[31];
    const int nst = min(nq, kSfiStage);
    // a staged query's whole top-K row (32 B) by one thread, its two 16-byte
    // loads in flight (an element per thread was 8 dependent round trips each)
    static_assert(kTopK == 8, "a top-K row is two uint4");
    for (int q = tid; q < nst; q += kSfiThreads) {
        const uint4* row = (const uint4*)(topk + (long long)(qlist[q] & 0x7fffffff) * kTopK);
        const uint4 r0 = row[0], r1 = row[1];
        ((uint4*)skeys)[2 * q] = r0;
        ((uint4*)skeys)[2 * q + 1] = r1;
    }
    // F2's level-0 list for the exact rescans (entry, position, descriptor):
    // a rescan then reads LDS, not three dependent global loads per candidate
    const int nl2 = min(nl, kSfiStage2);
    for (int e = tid; e < nl2; e += kSfiThreads) {
        const int v = list[e], fi = v & 0xffff;
        s2list[e] = v;
        s2xy[e] = make_float2(K2[fi].x, K2[fi].y);
        s2desc[2 * e] = *(const uint4*)(D2 + (long long)fi * 32);
        s2desc[2 * e + 1] = *(const uint4*)(D2 + (long long)fi * 32 + 16);
    }
    __syncthreads();
    if (tid == 0) hist[31] = 0;
    if (tid < kWave) {
#if ORB_SFI_PRIO
        // the serial walk is one latency-bound wave beside the extraction's
        // waves on its SIMD: it issues first
        __builtin_amdgcn_s_setprio(3);
#endif
#if ORB_SFI_SPEC
        // Speculative runs of 8 queries (the approach of k_proj_resolve_spec):
        // lane 8t + k holds key k of query j0 + t; every query of the run
        // decides against the state at the run's start, and the longest
        // prefix of queries whose decision no earlier claim of the run can
        // change is committed at once.  A query's decision reads its list up
        // to its second live entry (all of it when fewer than two are live), and
        // the state only ever blocks more entries (a claim lowers
        // vMatchedDistance), so an earlier claim of an F2 feature outside that
        // part leaves the decision exactly as the serial walk takes it; so
        // does a claim inside it that leaves the entry live (ORB_SFI_CONFL 3:
        // its distance above the entry's).  Committed claims are written in
        // parallel: two of one F2 feature in a prefix are a steal, the later
        // claim's distance strictly smaller, so an LDS min keeps it.  A query whose
        // truncated list cannot decide is rescanned exactly by the wave after
        // the prefix is committed; a conflicting one is re-decided next round.
        int nm = 0;
        const float r = a.window;
        const int grp = lane >> 3, kk = lane & 7;
        // per query tp of a run: 0 for the lanes of later queries, else a bit
        // above any feature index (their entries cannot conflict with tp's claim)
        uint32_t sfi_pen[7];
#pragma unroll
        for (int tp = 0; tp < 7; ++tp) sfi_pen[tp] = grp > tp ? 0u : (ORB_SFI_CONFL == 3 ? 1u : 0x100000u);
        SFI_CNT(3, nq);
        SFI_TS(6);
        // the walk in two instantiations: every query's keys staged (no global
        // load in the loop at all, so no wait at its head drains one), or not
        auto walk = [&](auto all_staged_c) {
        constexpr bool kAllStaged = decltype(all_staged_c)::value;
        auto run_keys = [&](int j0) -> uint32_t {
            const int j = j0 + grp;
            if constexpr (kAllStaged) return j < nq ? skeys[j * kTopK + kk] : kNoKey;
            return j < nst ? skeys[j * kTopK + kk]
                           : (j < nq ? topk[(long long)(qlist[j] & 0x7fffffff) * kTopK + kk] : kNoKey);
        };
        // keys of the staged queries come from LDS (walk 84.8 -> 78.7 us
        // alone); past them the next kSfiDepth - 1 runs' keys are in flight
        // while a round runs (the register rotation waits for the newest load
        // every round, so deeper prefetch does not help: 82 / 82 / 85 / 90 us
        // at 3 / 4 / 6 / 8 runs)
        uint32_t kr[kSfiDepth];
#pragma unroll
        for (int i = 0; i < kSfiDepth; ++i) kr[i] = nq > 8 * i ? run_keys(8 * i) : kNoKey;
        int j0 = 0;
        while (j0 < nq) {
            const uint32_t kcur = kr[0];
            const int nrun = min(8, nq - j0);
            const int qe = grp < nrun ? qlist[j0 + grp] : 0;
            const bool many = qe < 0;
            const bool kval = kcur != kNoKey;
            const int kd = (int)((kcur >> 16) & 0x1ffu);
            const int kfi = kval ? (int)(kcur & 0xffffu) : 0;
            const int i1 = qe & 0x7fffffff;
            uint32_t st = md21[kfi];
            // queries t0.. of the run are undecided; after a committed prefix the
            // lanes' states are brought up to date in registers and the rest of
            // the run is decided again in place (no new state read, no key shift)
            int t0 = 0, P = 0;
            bool ok = true;
            while (t0 < nrun) {
                const bool active = grp >= t0 && grp < nrun;
                const bool live = kval && !((int)(st >> 16) <= kd);
                // the query's first two live entries by 8-lane DPP minima of
                // (entry | distance | F2 feature) words (no LDS-routed shuffle):
                // the winner's fields and state reach every lane of its group
                const uint32_t wl = live ? ((uint32_t)kk << 25) | ((uint32_t)kd << 16) | (uint32_t)kfi : 0xffffffffu;
                const uint32_t w1 = grp8_min(wl);
                const int p1 = w1 == 0xffffffffu ? 8 : (int)(w1 >> 25);
                const uint32_t w2 = grp8_min(kk != p1 ? wl : 0xffffffffu);
                const int p2 = w2 == 0xffffffffu ? 8 : (int)(w2 >> 25);
                ok = p2 < 8 || !many;
                const int best = p1 < 8 ? (int)((w1 >> 16) & 0x1ffu) : INT_MAX;
                const int bi = (int)(w1 & 0xffffu);
                const uint32_t stb = grp8_min(kk == p1 ? st : 0xffffffffu);
                const uint32_t kb = grp8_min(kk == p1 ? kcur : 0xffffffffu);
                const int best2 = p2 < 8 ? (int)((w2 >> 16) & 0x1ffu) : INT_MAX;
                const bool acc = ok && active && best <= kThLow && (float)best < (float)best2 * a.ratio;
                // an earlier claim on an entry this query's decision reads stops it
                const bool reads = kval && kk <= p2;
                SFI_TS(0);
                uint64_t confl = 0;
                bool gconf = false;
#if ORB_SFI_CONFL
                // the claims of queries 0..6 of the run as 7 independent
                // readlanes, each lane comparing its entry with those of the
                // earlier queries (a loop over the accepting queries was a
                // SALU -> readlane -> compare -> SALU chain per claim: 850 of a
                // step's ~2,100 cycles, profiles/r06/README.md)
                if (ORB_SFI_ABL != 3) {
#if ORB_SFI_CONFL == 3
                    // Only a claim that KILLS an entry a later query reads
                    // changes that query's decision: a claim of distance best
                    // on the lane's feature kills it iff best <= kd (a claim
                    // with best > kd leaves it live, as at the run's start: the
                    // claim lowered the state from above best to best).  So a
                    // later query may steal an earlier claim of the same run in
                    // the same prefix (the smaller distance wins: ds_min below).
                    // With C = bi * 2048 + best and L = kfi * 2048 + kd,
                    // u = L - C lies in [0, 512) iff kfi == bi and best <= kd
                    // (|kfi - bi| >= 1 puts u at least 2048 - 511 away);
                    // v_alignbit(pen, u, 9) is 0 iff that holds and pen is 0.
                    const uint32_t ca = acc ? ((uint32_t)bi << 11) | (uint32_t)best : 0x7fffffffu;
                    const uint32_t Lk = ((uint32_t)kfi << 11) | (uint32_t)kd;
                    uint32_t x[7];
#pragma unroll
                    for (int tp = 0; tp < 7; ++tp)
                        x[tp] = __builtin_amdgcn_alignbit(sfi_pen[tp],
                                                          Lk - (uint32_t)__builtin_amdgcn_readlane((int)ca, 8 * tp), 9);
#else
                    const int bia = acc ? bi : 0xffff0;                 // group-uniform: the query's claim
                    // hit iff some (kfi ^ claim of an earlier query) is 0: one
                    // v_xor3 a query (the lane's penalty for queries not before
                    // it) and a v_min3 tree, all VALU -- no SALU mask per claim
                    uint32_t x[7];
#pragma unroll
                    for (int tp = 0; tp < 7; ++tp)
                        x[tp] = (uint32_t)kfi ^ (uint32_t)__builtin_amdgcn_readlane(bia, 8 * tp) ^ sfi_pen[tp];
#endif
                    const uint32_t m = umin3(umin3(x[0], x[1], x[2]), umin3(x[3], x[4], x[5]), x[6]);
#if ORB_SFI_CONFL >= 2
                    // the query's conflict as an 8-lane DPP OR (no 64-bit
                    // per-lane shift of a ballot, no divergent branch)
                    gconf = grp8_min((reads && m == 0u) ? 0u : 1u) == 0u;
#else
                    confl = __ballot(reads && m == 0u);
#endif
                }
#else
                for (uint64_t am = ORB_SFI_ABL == 3 ? 0 : __ballot(acc && kk == 0); am; am &= am - 1) {
                    const int l = __ffsll((long long)am) - 1;           // lane 8t' of a claiming query
                    const int cb = __builtin_amdgcn_readlane(bi, l);
                    confl |= __ballot(reads && kfi == cb && lane >= l + 8);
                }
#endif
                SFI_TS(1);
#if ORB_SFI_CONFL >= 2
                (void)confl;
                const bool stop = (active & (gconf | !ok)) | (grp >= nrun);
#else
                const bool stop = (active && (((confl >> (8 * grp)) & 0xffull) != 0 || !ok)) || grp >= nrun;
#endif
                const uint64_t sm = __ballot(stop && kk == 0);
                P = sm ? (__ffsll((long long)sm) - 1) >> 3 : 8;
                const bool commit = acc && grp < P && kk == 0;
                const int prev = (int)(stb & 0xffffu) - 1;
                const uint32_t nst_v = ((uint32_t)best << 16) | (uint32_t)(i1 + 1);
                // a claim writes only the state and the query's rotation bin:
                // the matches (md21 holds every F2 feature's final F1 match) and
                // the rotation histogram (every query claims at most once, and
                // bin1 keeps a stolen query's bin) are rebuilt after the walk
                (void)prev;
                if (commit) {
#if ORB_SFI_CONFL == 3
                    atomicMin(&md21[bi], nst_v);   // two claims of one feature in a prefix: the later, smaller one
#else
                    md21[bi] = nst_v;
#endif
                    if (a.check_ori) bin1[i1] = (int8_t)(kb >> 25);
                }
                // (the match count is taken from m12 after the walk: no per-step
                // ballots for it)
                const uint64_t cmask = __ballot(commit);
                SFI_CNT(4, __popcll(cmask));
                // the next reads see these writes (one wave: its LDS operations
                // complete in order; the asm keeps the compiler from hoisting
                // later reads above the stores)
                asm volatile("" ::: "memory");
                SFI_TS(2);
                if (P >= nrun) break;
                // the committed claims into the lanes' states (what md21 now holds)
                for (uint64_t cm = cmask; cm; cm &= cm - 1) {
                    const int l = __ffsll((long long)cm) - 1;
                    const int cb = __builtin_amdgcn_readlane(bi, l);
                    const uint32_t cv = (uint32_t)__builtin_amdgcn_readlane((int)nst_v, l);
                    st = kfi == cb ? min(st, cv) : st;
                }
                SFI_TS(3);
                t0 = P;
                if (ORB_SFI_ABL == 2 && __builtin_amdgcn_readlane((int)ok, 8 * P) == 0) {
                    t0 = P + 1;
                } else if (__builtin_amdgcn_readlane((int)ok, 8 * P) == 0) {
                // query j0 + P cannot decide from its truncated list: exact
                // full candidate scan under the state after the prefix
                const int qx = __builtin_amdgcn_readlane(qe, 8 * P);
                const int q1 = qx & 0x7fffffff;
                const orb_keypoint k1 = K1[q1];
                float px, py;
                query_pos(a, pr, q1, k1, px, py);
                CellRange cr;
                cell_range(px, py, r, a.g, cr);
                const uint4 d0 = *(const uint4*)(D1 + (long long)q1 * 32);
                const uint4 d1 = *(const uint4*)(D1 + (long long)q1 * 32 + 16);
                Best2 bs{INT_MAX, INT_MAX, -1, 0, 0};
                for (int base = 0; base < nl; base += kWave) {
                    const int jj = base + lane;
                    int d = INT_MAX, fi = -1;
                    if (jj < nl2) {                            // the staged part of the list
                        const int v = s2list[jj];
                        const int cell = v >> 16, gx = cell / kGridRows, gy = cell - gx * kGridRows;
                        fi = v & 0xffff;
                        const float2 xy = s2xy[jj];
                        if (gx >= cr.x0 && gx <= cr.x1 && gy >= cr.y0 && gy <= cr.y1 && fabsf(xy.x - px) < r &&
                            fabsf(xy.y - py) < r) {
                            const uint4 b0 = s2desc[2 * jj], b1 = s2desc[2 * jj + 1];
                            d = __popc(d0.x ^ b0.x) + __popc(d0.y ^ b0.y) + __popc(d0.z ^ b0.z) + __popc(d0.w ^ b0.w) +
                                __popc(d1.x ^ b1.x) + __popc(d1.y ^ b1.y) + __popc(d1.z ^ b1.z) + __popc(d1.w ^ b1.w);
                        }
                        if (d != INT_MAX && (int)(md21[fi] >> 16) <= d) d = INT_MAX;
                    } else if (jj < nl) {
                        d = cand_dist(list, jj, cr, px, py, r, K2, D2, d0, d1);
                        fi = list[jj] & 0xffff;
                        if (d != INT_MAX && (int)(md21[fi] >> 16) <= d) d = INT_MAX;
                    }
                    merge_chunk(bs, d, fi, 0);
                }
                if (bs.idx >= 0 && bs.best <= kThLow && (float)bs.best < (float)bs.best2 * a.ratio) {
                    const int pv = (int)(md21[bs.idx] & 0xffffu) - 1;
                    const uint32_t nv = ((uint32_t)bs.best << 16) | (uint32_t)(q1 + 1);
                    (void)pv;
                    if (lane == 0) {
                        md21[bs.idx] = nv;
                        if (a.check_ori) bin1[q1] = (int8_t)rot_bin(k1.angle, K2[bs.idx].angle);
                    }
                    asm volatile("" ::: "memory");
                    st = kfi == bs.idx ? nv : st;
                }
                SFI_CNT(2, 1);
                t0 = P + 1;
                // drain the rescan's loads here (a rescan is rare): a load left
                // pending on some path made the compiler wait for memory at the
                // head of every step
                __builtin_amdgcn_s_waitcnt(0);
                SFI_TS(4);
                }
                SFI_CNT(1, 1);
            }
            const int adv = nrun;
            SFI_CNT(0, 1);
            (void)P; (void)ok;
            j0 += adv;
            // the next runs' keys: shifted by the queries done (a whole run in
            // the usual case), the run after them loaded
            if (adv == 8) {
#pragma unroll
                for (int i = 0; i + 1 < kSfiDepth; ++i) kr[i] = kr[i + 1];
            } else {
                const int src = lane + 8 * adv;
                uint32_t sh[kSfiDepth];
#pragma unroll
                for (int i = 0; i < kSfiDepth; ++i) sh[i] = (uint32_t)__shfl((int)kr[i], src & 63, kWave);
#pragma unroll
                for (int i = 0; i + 1 < kSfiDepth; ++i) kr[i] = src < 64 ? sh[i] : sh[i + 1];
            }
            kr[kSfiDepth - 1] = j0 + 8 * (kSfiDepth - 1) < nq ? run_keys(j0 + 8 * (kSfiDepth - 1)) : kNoKey;
            SFI_TS(5);
        }
        };
        if (nq <= kSfiStage) walk(std::true_type{});
        else walk(std::false_type{});
#else
        int nm = 0, hreg = 0;   // lane b: the rotation histogram's bin b
        const float r = a.window;
        const int grp = lane >> 3;
        // run of 8 queries from j0: lane 8t + k holds key k of query j0 + t
        auto run_keys = [&](int j0) -> uint32_t {
            const int j = j0 + grp;
            return j < nq ? topk[(long long)(qlist[j] & 0x7fffffff) * kTopK + (lane & 7)] : kNoKey;
        };
        uint32_t kcur = nq > 0 ? run_keys(0) : kNoKey;
        uint32_t knxt = nq > 8 ? run_keys(8) : kNoKey;
        // runs as a loop nest: inside a run no step reads the run in flight,
        // so the compiler's wait counts never stall a step on that load (a
        // flat loop with the swap inside made every step wait for it)
        for (int j0 = 0; j0 < nq; j0 += 8) {
          if (j0 > 0) {
            kcur = knxt;
            knxt = j0 + 8 < nq ? run_keys(j0 + 8) : kNoKey;
          }
          // per run, everything but the state: lane 8t + k's key fields and
          // state address, lane t's query entry (read per step by readlane)
          const bool kval = kcur != kNoKey;
          const int kd = (int)((kcur >> 16) & 0x1ffu);
          const int kfi = kval ? (int)(kcur & 0xffffu) : 0;
          const int qv = lane < 8 && j0 + lane < nq ? qlist[j0 + lane] : 0;
          const int jend = min(j0 + 8, nq);
          for (int j = j0; j < jend; ++j) {
            const int t = j - j0;
            const int qe = __builtin_amdgcn_readlane(qv, t);
            const int i1 = qe & 0x7fffffff;
            const bool many = qe < 0;
            int best = INT_MAX, best2 = INT_MAX, bi = -1, prev = -1, bn = 0;
            bool ok = false;
            {
                // one LDS read per step: the state of each lane's candidate
                // (query t's lanes count), which for the winner is also its
                // previous match
                const uint32_t st = md21[kfi];
                const bool live = kval && !((int)(st >> 16) <= kd);
                uint64_t m = __ballot(live) & (0xffull << (8 * t));
                const int nlive = __popcll(m);
                if (nlive >= 2 || !many) {
                    ok = true;
                    if (nlive >= 1) {
                        // the ballot is uniform: readlane, not an LDS-routed shuffle
                        const int l0 = __ffsll((long long)m) - 1;
                        best = __builtin_amdgcn_readlane(kd, l0);
                        bi = __builtin_amdgcn_readlane(kfi, l0);
                        prev = (int)((uint32_t)__builtin_amdgcn_readlane((int)st, l0) & 0xffffu) - 1;
                        bn = (int)((uint32_t)__builtin_amdgcn_readlane((int)kcur, l0) >> 25);
                        m &= m - 1;
                        if (m) best2 = __builtin_amdgcn_readlane(kd, __ffsll((long long)m) - 1);
                    }
                }
            }
            if (!ok) {   // exact fallback: full candidate scan under the current state
                const orb_keypoint k1 = K1[i1];
                float px, py;
                query_pos(a, pr, i1, k1, px, py);
                CellRange cr;
                cell_range(px, py, r, a.g, cr);
                const uint4 q0 = *(const uint4*)(D1 + (long long)i1 * 32);
                const uint4 q1 = *(const uint4*)(D1 + (long long)i1 * 32 + 16);
                Best2 st{INT_MAX, INT_MAX, -1, 0, 0};
                for (int base = 0; base < nl; base += kWave) {
                    const int jj = base + lane;
                    int d = INT_MAX, fi = -1;
                    if (jj < nl) {
                        d = cand_dist(list, jj, cr, px, py, r, K2, D2, q0, q1);
                        fi = list[jj] & 0xffff;
                        if (d != INT_MAX && (int)(md21[fi] >> 16) <= d) d = INT_MAX;
                    }
                    merge_chunk(st, d, fi, 0);
                }
                best = st.best; best2 = st.best2; bi = st.idx;
                if (bi >= 0) {
                    prev = (int)(md21[bi] & 0xffffu) - 1;
                    bn = a.check_ori ? rot_bin(k1.angle, K2[bi].angle) : 0;
                }
            }
            if (best <= kThLow && (float)best < (float)best2 * a.ratio) {
                if (prev >= 0) --nm;
                if (lane == 0) {
                    if (prev >= 0) m12[prev] = -1;
                    m12[i1] = bi;
                    md21[bi] = ((uint32_t)best << 16) | (uint32_t)(i1 + 1);
                    if (a.check_ori) bin1[i1] = (int8_t)bn;
                }
                if (a.check_ori && lane == bn) ++hreg;
                ++nm;
                // Only this wave touches the state and one wave's LDS
                // operations complete in order, so the next step's reads see
                // these writes without a wait; the compiler keeps the order
                // (the indices may alias) and the asm keeps it from moving
                // the next step's loads above the stores.
                asm volatile("" ::: "memory");
            }
          }
        }
#if !ORB_SFI_SPEC
        if (lane < 32) hist[lane] = hreg;   // bins 0..29; hist[31] = 0 counts the matches below
#endif
#endif
        (void)nm;
    }
    __syncthreads();
#if ORB_SFI_SPEC
    // the walk's outcome from its state: F1 feature i matched iff some F2
    // feature's final claim is i (vnMatches12 / vnMatches21 agree at the end
    // of ORBmatcher.cc:700-735), and rotHist[b] counts every claim ever made
    // in bin b (:729-735 push back before any later steal)
    for (int j = tid; j < n2; j += kSfiThreads) {
        const int w = (int)(md21[j] & 0xffffu);
        if (w) m12[w - 1] = j;
    }
    if (a.check_ori) {
        int hb = 0;   // lane b < 30 of each wave: its count of bin b
        for (int i0 = (tid & ~(kWave - 1)); i0 < n1; i0 += kSfiThreads) {
            const int b = i0 + lane < n1 ? (int)bin1[i0 + lane] : -1;
            for (uint64_t bm = __ballot(b >= 0); bm; ) {
                const int l = __ffsll((long long)bm) - 1;
                const int bb = __builtin_amdgcn_readlane(b, l);
                const uint64_t same = __ballot(b == bb);
                if (lane == bb) hb += __popcll(same & bm);
                bm &= ~same;
            }
        }
        if (lane < 30 && hb) atomicAdd(&hist[lane], hb);
    }
    __syncthreads();
#endif
    // nmatches = the F1 features left matched (every claim matched one, every
    // steal unmatched one), after the rotation filter (ORBmatcher.cc:738-758)
    int i1x = -1, i2x = -1, i3x = -1;
    if (a.check_ori) three_maxima_wave(hist, i1x, i2x, i3x);   // bins 0..29
    int nmk = 0;
    for (int i = tid; i < n1; i += kSfiThreads) {
        if (m12[i] < 0) continue;
        const int b = a.check_ori ? (int)bin1[i] : -1;
        if (b >= 0 && b != i1x && b != i2x && b != i3x) m12[i] = -1;
        else ++nmk;
    }
    nmk = wave_sum(nmk);
    if (lane == 0 && nmk) atomicAdd(&hist[31], nmk);
    __syncthreads();
    const int nm = hist[31];
    if (a.prev_out) {
        for (int i = tid; i < n1; i += kSfiThreads) {
            float px, py;
            query_pos(a, pr, i, K1[i], px, py);
            const int m = m12[i];
            if (m >= 0) { px = K2[m].x; py = K2[m].y; }
            a.prev_out[((long long)pr * a.cap + i) * 2] = px;
            a.prev_out[((long long)pr * a.cap + i) * 2 + 1] = py;
        }
    }
    if (M12L)
        for (int i = tid; i < n1; i += kSfiThreads) m12g[i] = m12[i];
    if (tid == 0) a.nmatches[pr] = nm;
#ifdef ORB_SFI_COUNT
    const unsigned long long sfi_t[8] = {sfi_a0, sfi_a1, sfi_a2, sfi_a3, sfi_a4, sfi_a5, sfi_a6,
                                         __builtin_amdgcn_s_memtime() - sfi_t0};
    const unsigned long long sfi_c[5] = {sfi_c0, sfi_c1, sfi_c2, sfi_c3, sfi_c4};
    if (tid == 0) {
        for (int k = 0; k < 5; ++k) atomicAdd(&g_sfi_cnt[k], sfi_c[k]);
        for (int k = 0; k < 8; ++k) atomicAdd(&g_sfi_cnt[8 + k], sfi_t[k]);
    }
#endif
}

constexpr size_t kLdsMax = 160 * 1024;

// Frames up to ~15,600 keypoints (the resolve's 9 bytes of LDS a keypoint and its ~19 KB of staging);
// beyond that ORB_ERR_UNSUPPORTED before any launch.
static int launch_sfi(SfiArgs& a, int npairs, hipStream_t st) {
    const size_t lds_res = sfi_lds_bytes(a.cap);
    if (lds_res > kLdsMax) return ORB_ERR_UNSUPPORTED;
    if (a.cap > 65535) return ORB_ERR_UNSUPPORTED;   // 16-bit feature fields of the keys and the state
    // staged form; a block whose F2 level-0 list is longer than its
    // registers take runs the per-lane form from global memory
    KLAUNCH(k_sfi_topk_st, dim3(npairs, (a.cap + kStQ - 1) / kStQ), dim3(256),
            (size_t)kStIt * kWave * (32 + 8 + 4 + 4) + (ORB_SFI_QSTAGE ? (size_t)kStQ * (32 + 16) : 0), st, a);
    const size_t lds_m12 = lds_res + (size_t)a.cap * 4;
    if (lds_m12 <= kLdsMax)
        KLAUNCH(k_sfi_resolve<true>, dim3(npairs), dim3(kSfiThreads), lds_m12, st, a);
    else
        KLAUNCH(k_sfi_resolve<false>, dim3(npairs), dim3(kSfiThreads), lds_res, st, a);
    return ORB_OK;
}

// ---------------------------------------------------------------------------
// k_bow: ORBmatcher::SearchByBoW(KeyFrame*, Frame&) (ORBmatcher.cc:223-425),
// mono branch, one wave per (keyframe, frame) pair: merge-join of the two
// FeatureVectors by node id; per KF feature with a valid MapPoint, best/second
// over the frame features of the node that are not yet matched.
// With f_valid set it is SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2)
// (:765-905): the second keyframe plays the frame, its features need a valid
// MapPoint (:824-830), the acceptance is strict (`bestDist1 < TH_LOW`, :848)
// and out12 receives vpMatches12 by KF1 feature.  The two forms record the
// rotation bin of a match on opposite sides (:352 bestIdxF, :864 idx1); every
// match is a one-to-one pair, so filtering by either side is the same.
// ---------------------------------------------------------------------------
struct BowArgs {
    // keyframes (one per pair), concatenated: kf i owns features
    // [kp_off[i], kp_off[i+1]) and FeatureVector nodes [node_off[i], node_off[i+1]);
    // its CSR offsets start at fv_off[node_off[i] + i] (nnodes_i + 1 entries, relative
    // to idx_off[i]).
    const orb_keypoint* kf_kps;
    const uint8_t* kf_desc;
    const uint8_t* kf_valid;
    const long long* kp_off;
    const uint32_t* kf_node;
    const int* kf_off;
    const uint32_t* kf_idx;
    const long long* node_off;
    const long long* idx_off;
    const uint8_t* kf_fvdesc;   // optional: KF descriptors in FeatureVector order (orbm_kf_map_device::fv_desc)
    const float* kf_fvangle;    // optional: KF keypoint angles in FeatureVector order (::fv_angle)
    // frame (shared by all pairs)
    const orb_keypoint* f_kps;  const uint8_t* f_desc;  int f_n;
    const uint32_t* f_node;  const int* f_off;  const uint32_t* f_idx;  int f_nnodes;
    float ratio;
    int check_ori;
    int npairs;
    int32_t* match;      // [pair][f_n]  (-1 before k_bow)
    int32_t* nmatches;   // [pair]       (0 before k_bow)
    const uint8_t* f_valid;   // KF-KF form: pKF2 MapPoint != NULL && !isBad(), else NULL
    int32_t* out12;           // KF-KF form: [KF1 features] KF2 feature or -1, else NULL
    int f_nleft = -1;         // the frame's Nleft (-1: mono / rectified)
    unsigned* fin_ticket = nullptr;   // single pair: k_bow's last block runs the final (k_bow_final's body)
    int32_t* host_out = nullptr;      // ... and then copies match[f_n] + nmatches there (pinned host memory)
    int* done = nullptr;              // ... and writes seq into this word (signal_done)
    int seq = 0;
    int reset_after = 0;              // ... and leaves match / nmatches / fin_ticket as it found them
                                      // (-1 / 0 / 0: persistent scratch of the dframe form)
    int single_nodes = -1;            // >= 0: one pair whose offsets all start at 0 (kp_off, node_off,
                                      // idx_off), with this many KF nodes: the kernels skip those loads
    unsigned* tstart = nullptr;       // dframe form: the first block's start (s_memrealtime, 100 MHz;
                                      // 0xffffffff before the launch, reset by the last block), and
                                      // host_out[f_n + 1 ..] = node phase, final phase (10 ns ticks)
    int kv_lds = 0;                   // dframe form: kf_valid (host-mapped, 16-B padded) staged in
                                      // LDS by every block, this many bytes (0: read in place)
    unsigned* wtrace = nullptr;       // ORB_OPT_BOW_TRACE (diagnostics): per small-node wave, 16 words of
                                      // s_memrealtime checkpoints (bow_nodes_body)
};

// One wave per (pair, vocabulary node) the two FeatureVectors share: the
// reference's merge-join (:239-402) visits each node both FeatureVectors hold
// exactly once, and a node's matching reads and writes only that node's
// features, so nodes are independent.  Inside the node the KF features run in
// order; the F features sit on the lanes (chunk c, lane l) with their
// "already matched" flags in a per-lane bit mask (chunks >= 64 of a node with
// more than 4096 frame features read the flag from `match` itself: only this
// wave touches the node's features).
// Frame nodes of at most kBowRegChunks chunks run in k_bow's small-node blocks with their F
// descriptors in registers; larger ones (a vocabulary's skew puts hundreds of
// features in a few nodes) run in its large-node blocks, which stage the node's F
// descriptors in LDS once and share them between the block's keyframes.
constexpr int kBowMaskChunks = 64;
#ifndef ORB_BOWF_DROP4
#define ORB_BOWF_DROP4 1   // 3.955 vs 4.02-4.04 ms per C5 query on one box
#endif

constexpr int kBowRegChunks = 2;        // frame-feature chunks held in registers per node
#ifndef ORB_BOW_TRANS
#define ORB_BOW_TRANS 4      // transposed register-chunk nodes: frame features < this x KF features
#endif
static_assert(kBowRegChunks == 2, "bow_node's claim selects between two register chunks");
constexpr int kBowLdsNodes = 4096;      // frame FeatureVector nodes staged in LDS (dynamic size)
constexpr int kBowBigCap = 512;         // large-node blocks: node positions staged in LDS
constexpr int kBowBigPairs = 4;         // large-node blocks: keyframes per block (one per wave)

constexpr int kBowKvLds = 16384;        // dframe form: KF validity bytes staged in LDS
static size_t bow_kv_bytes(int kv) { return ((size_t)kv + 15) & ~size_t(15); }
static size_t bow_lds(int f_nnodes, int kv = 0) {
    return bow_kv_bytes(kv) + (f_nnodes <= kBowLdsNodes ? (size_t)(2 * f_nnodes + 1) * 4 : 0);
}

// Best / second over a BoW node's frame features for one KF feature.  A
// candidate is the key dist << 22 | position (unique; ordered like the
// reference's stream: the first position of the smallest distance is the best,
// and bestDist2 is the second smallest distance of the multiset).  Each lane
// folds its chunks into a local (smallest, second) pair; two DPP minima finish:
// the chunk-independent work has no serial dependency between chunks.
__device__ __forceinline__ void key_push(int& lo, int& hi, int key) {
    hi = min(hi, max(lo, key));
    lo = min(lo, key);
}
// A wave-uniform 64-bit value in SGPRs (the compiler cannot prove a ballot's
// result uniform once it is merged with other values).
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32;
}
// The median of three (v_med3_i32): with k1 <= k2 <= k3 the sorted three
// smallest of {k1, k2, k3, key} are (min(k1, key), med3(k1, key, k2), med3(k2, key, k3)).
__device__ __forceinline__ int med3i(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }
// kSecond: the caller reads best2 (only when best can pass TH_LOW: no claim is
// possible otherwise, so the second reduction is skipped).
template <bool kSecond>
__device__ __forceinline__ Best2 key_best2(int lo, int hi) {
    Best2 st{256, 256, -1, 0, 0};
    const int m = wave_min(lo, INT_MAX);
    if (m == INT_MAX) return st;
    st.best = m >> 22; st.idx = m & ((1 << 22) - 1);
    if (kSecond && st.best <= kThLow) {
        const int m2 = wave_min(lane_id() == (m & (kWave - 1)) ? hi : lo, INT_MAX);
        st.best2 = m2 == INT_MAX ? 256 : m2 >> 22;
    }
    return st;
}

// The merge-join step of one (pair, node): KF node ia of pair pr against the
// frame node's positions [fb, fe).  kLds: positions < kBowBigCap come from the
// block's LDS copy (s_fd descriptor bytes 0-15 at [pos], 16-31 at
// [kBowBigCap + pos]; s_fi frame index | invalid << 31);
// otherwise the first kBowRegChunks chunks are loaded into registers.  Anything
// past either reads global memory.
template <bool kLds, bool kFish>
__device__ __forceinline__ void bow_node(const BowArgs& a, int pr, int ia, int fb, int fe,
                                         const uint4* s_fd, const int* s_fi, uint4* s_q,
                                         unsigned* tr = nullptr, int coop_w = -1) {
    const int lane = lane_id();
    const bool one = a.single_nodes >= 0;            // one pair at offset 0: no offset loads in the chain
    const long long kpo = one ? 0 : a.kp_off[pr];
    const uint8_t* KD = a.kf_desc + kpo * 32;
    extern __shared__ __attribute__((aligned(16))) int bow_smem[];
    // the dframe form's validity bytes come from the block's LDS copy: read in
    // place they are host memory, one PCIe round trip per lane-distinct line
    const uint8_t* KV = a.kv_lds > 0 ? (const uint8_t*)bow_smem : a.kf_valid + kpo;
    const int* ko = a.kf_off + (one ? 0 : a.node_off[pr] + pr);
    const uint32_t* ki = a.kf_idx + (one ? 0 : a.idx_off[pr]);
    fb = __builtin_amdgcn_readfirstlane(fb);     // wave-uniform (read from LDS by the caller): keeps
    fe = __builtin_amdgcn_readfirstlane(fe);     // the node's loops scalar
    const int nf = fe - fb;
    const int nch = (nf + kWave - 1) / kWave;
    int32_t* match = a.match + (long long)pr * a.f_n;
    constexpr bool fish = kFish;                     // the frame is fisheye stereo (f_nleft >= 0)
    constexpr int kReg = kLds ? 0 : kBowRegChunks;
    const int nlds = kLds ? min(nch, kBowBigCap / kWave) : 0;   // chunks [0, nlds) in LDS
    uint4 fr0[kBowRegChunks], fr1[kBowRegChunks];
    int fir[kBowRegChunks];
    int mcl[kBowRegChunks] = {-1, -1};               // register chunks: this lane's claim (KF feature)
    uint64_t taken = 0;                              // bit c: (chunk c, this lane) is matched / invalid
    if constexpr (!kLds) {
#pragma unroll
        for (int c = 0; c < kBowRegChunks; ++c) {
            fr0[c] = make_uint4(0, 0, 0, 0); fr1[c] = fr0[c]; fir[c] = -1;
            const int q = fb + c * kWave + lane;
            if (c < nch && q < fe) {
                const int fi = (int)a.f_idx[q];
                fir[c] = fi;
                fr0[c] = *(const uint4*)(a.f_desc + (long long)fi * 32);
                fr1[c] = *(const uint4*)(a.f_desc + (long long)fi * 32 + 16);
            }
        }
#pragma unroll
        for (int c = 0; c < kBowRegChunks; ++c) {
            if (fir[c] < 0) taken |= 1ull << c;                               // past the node's end
            else if (a.f_valid && !a.f_valid[fir[c]]) taken |= 1ull << c;
        }
    }
    for (int c = kReg; c < nch && c < kBowMaskChunks; ++c) {
        const int pos = c * kWave + lane;
        if (pos >= nf) taken |= 1ull << c;
        else if (c < nlds) { if (s_fi[pos] < 0) taken |= 1ull << c; }
        else if (a.f_valid && !a.f_valid[(int)a.f_idx[fb + pos]]) taken |= 1ull << c;
    }
    int nm = 0;
    // the node's KF features, 64 at a time, prefetched lane-parallel (index,
    // MapPoint validity, descriptor, angle) and visited in order by readlane
    const int pe = ko[ia + 1];
    // Register-chunk nodes with many KF features for their frame features run
    // transposed (a lane per KF feature): per KF feature that costs one pass
    // over the free positions' descriptors in a lane instead of two wave-wide
    // reductions (~85 VALU cycles a frame position against ~400 a KF feature).
    // tk0 / tk1: the taken / invalid flags of chunks 0 / 1 as wave-uniform masks.
    const bool trans = !kLds && !kFish && nch <= kBowRegChunks && nf < ORB_BOW_TRANS * (pe - ko[ia]);
    // coop_w >= 0 (single pair: a block per KF node, every wave here with the
    // same node): a transposed node's positions are split over the block's
    // four waves for the lists, wave 0 merges them and walks; other nodes are
    // wave 0's alone.  sq0: wave 0's area (the frame descriptors), the other
    // waves' areas take their lists, wave 3's also the flags after a walk.
    const bool coop = coop_w >= 0;
    if (coop && coop_w > 0 && !trans) return;
    uint4* const sq0 = coop ? s_q - coop_w * 4 * kWave : s_q;
    uint64_t tk0 = ~0ull, tk1 = ~0ull;
    if (!kLds && trans) {
        tk0 = uniform64(__ballot(taken & 1));
        tk1 = uniform64(__ballot((taken >> 1) & 1));
        if (coop_w <= 0) {
#pragma unroll
            for (int c = 0; c < kBowRegChunks; ++c) {
                s_q[c * 2 * kWave + lane] = fr0[c];
                s_q[c * 2 * kWave + kWave + lane] = fr1[c];
            }
        }
        if (coop) {
            __syncthreads();
        } else {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    for (int pbase = ko[ia]; pbase < pe; pbase += kWave) {
      const int pl = pbase + lane;
      int my_ikf = 0, my_ok = 0;
      uint4 mq0 = make_uint4(0, 0, 0, 0), mq1 = mq0;
      if (pl < pe) {
          my_ikf = (int)ki[pl];
          my_ok = KV[my_ikf];
          mq0 = *(const uint4*)(KD + (long long)my_ikf * 32);
          mq1 = *(const uint4*)(KD + (long long)my_ikf * 32 + 16);
      }
      if (tr && lane == 0 && pbase == ko[ia]) {
          tr[3] = (unsigned)__builtin_amdgcn_s_memrealtime();
          tr[5] = (unsigned)(pe - pbase);
          tr[6] = (unsigned)nf;
      }
      if constexpr (!kLds && !kFish) {
        if (trans) {
          // Lane per KF feature: each lane keeps the three smallest keys over
          // the node's free frame positions (uniform position, descriptor by a
          // broadcast LDS read: no cross-lane reduction per pair), then the
          // decisions run in KF order on those lists.  A claim earlier in the
          // node removes one position: a feature's best / second are the first
          // two of its list still free, exact while at least two remain (keys
          // smaller than its third are all in the list; an INT_MAX entry means
          // the list already holds every candidate).  A list with fewer than
          // two left is recomputed lanes-over-positions against the flags.
          int k1 = INT_MAX, k2 = INT_MAX, k3 = INT_MAX;
          if (tr) {
              const unsigned ok = (unsigned)__ballot(my_ok != 0) + (unsigned)(mq0.x & 0);   // waits for the loads
              if (lane == 0 && pbase == ko[ia] && ok != 1u) tr[9] = (unsigned)__builtin_amdgcn_s_memrealtime();
          }
          {
              // every position of the node in order, four per iteration (their
              // LDS reads together, then the math); a taken position's key is
              // INT_MAX (a wave-uniform test)
              auto step = [&](const uint4& f0, const uint4& f1, int p) {
                  const int d = __popc(mq0.x ^ f0.x) + __popc(mq0.y ^ f0.y) + __popc(mq0.z ^ f0.z) +
                                __popc(mq0.w ^ f0.w) + __popc(mq1.x ^ f1.x) + __popc(mq1.y ^ f1.y) +
                                __popc(mq1.z ^ f1.z) + __popc(mq1.w ^ f1.w);
                  const bool tkp = (((p < kWave ? tk0 : tk1) >> (p & (kWave - 1))) & 1) != 0;
                  const int key = tkp ? INT_MAX : ((d << 22) | p);
                  k3 = med3i(k2, key, k3);
                  k2 = med3i(k1, key, k2);
                  k1 = min(k1, key);
              };
              const int pb0 = coop ? (nf * coop_w) >> 2 : 0, pb1 = coop ? (nf * (coop_w + 1)) >> 2 : nf;
              for (int p0 = pb0; p0 < pb1; p0 += 4) {
                  uint4 f0[4], f1[4];
#pragma unroll
                  for (int u = 0; u < 4; ++u) {
                      const int p = min(p0 + u, pb1 - 1);
                      const uint4* sf = sq0 + (p >> 6) * 2 * kWave + (p & (kWave - 1));
                      f0[u] = sf[0];
                      f1[u] = sf[kWave];
                  }
#pragma unroll
                  for (int u = 0; u < 4; ++u)
                      if (p0 + u < pb1) step(f0[u], f1[u], p0 + u);
              }
          }
          if (coop) {
              // the other waves' lists into wave 0's (each list sorted; keys distinct)
              if (coop_w > 0) {
                  int* L = (int*)s_q;
                  L[lane] = k1;
                  L[kWave + lane] = k2;
                  L[2 * kWave + lane] = k3;
              }
              __syncthreads();
              if (coop_w > 0) {
                  __syncthreads();                         // wave 0's walk done: its flags
                  const uint64_t* T = (const uint64_t*)(sq0 + 3 * 4 * kWave + kWave);
                  tk0 = uniform64(T[0]);
                  tk1 = uniform64(T[1]);
                  continue;
              }
#pragma unroll
              for (int w = 1; w < 4; ++w) {
                  const int* L = (const int*)(sq0 + w * 4 * kWave);
#pragma unroll
                  for (int r = 0; r < 3; ++r) {
                      const int key = L[r * kWave + lane];
                      k3 = med3i(k2, key, k3);
                      k2 = med3i(k1, key, k2);
                      k1 = min(k1, key);
                  }
              }
          }
          constexpr int kPos = (1 << 22) - 1;
          // the claimed position of a best / second pair, or -1 (:848 / :327, ratio)
          auto decide = [&](int r0, int r1) -> int {
              const int best = r0 == INT_MAX ? 256 : r0 >> 22;
              const int best2 = r1 == INT_MAX ? 256 : r1 >> 22;
              const bool low = a.f_valid ? best < kThLow : best <= kThLow;
              return (low && (float)best < a.ratio * (float)best2) ? (r0 & kPos) : -1;
          };
          // Lane-parallel, per list: its three positions (0xff: none), which of
          // them are taken (tb), and whether each pair it can present as (best,
          // second) -- (1,2) with nothing or only the third taken, (1,3) with
          // the second taken, (2,3) with the first -- passes the thresholds.
          // From these every feature's decision at the current flags is one
          // table lookup (cur: claimed position, kNone, kShort: list ran short).  A
          // feature that does not claim changes nothing, and its decision can
          // only change after a claim before it: the ordered walk visits only
          // the claiming (and short) features, re-deciding the rest after each
          // claim -- steps = claims, not KF features.
          auto p8 = [&](int k) { return k == INT_MAX ? 0xff : (k & kPos); };
          const int q1 = p8(k1), q2 = p8(k2), q3 = p8(k3);
          const int okb = (decide(k1, k2) >= 0 ? 1 : 0) | (decide(k1, k3) >= 0 ? 2 : 0) |
                          (decide(k2, k3) >= 0 ? 4 : 0);
          auto tk_has = [&](int q) -> int {                // lane-parallel: position q taken (0xff: never)
              const uint64_t m = q < kWave ? tk0 : (q < 2 * kWave ? tk1 : 0ull);
              return (int)((m >> (q & (kWave - 1))) & 1);
          };
          int tb = tk_has(q1) | tk_has(q2) << 1 | tk_has(q3) << 2;
          // the decision for each taken-state tb of the list, a byte each (0xff
          // none, 0xfe short): tb 0 / 4 -> (1,2), 1 -> (2,3), 2 -> (1,3)
          constexpr int kNone = 0xff, kShort = 0xfe;
          uint64_t lut = (uint64_t)kShort << 24 | (uint64_t)kShort << 40 | (uint64_t)kShort << 48 |
                         (uint64_t)kShort << 56;           // states 3, 5, 6, 7
          {
              const uint64_t e12 = (okb & 1) ? (uint64_t)q1 : (uint64_t)kNone;
              const uint64_t e23 = (okb & 4) ? (uint64_t)q2 : (uint64_t)kNone;
              const uint64_t e13 = (okb & 2) ? (uint64_t)q1 : (uint64_t)kNone;
              lut |= e12 | e23 << 8 | e13 << 16 | e12 << 32;
          }
          auto cur_of = [&]() -> int { return (int)((lut >> (tb * 8)) & 0xff); };
          int cur = cur_of();
          if (tr && lane == 0 && pbase == ko[ia]) tr[7] = (unsigned)__builtin_amdgcn_s_memrealtime();
          const uint64_t okm = uniform64(__ballot(my_ok != 0));
          uint64_t todo = okm & uniform64(__ballot(cur != kNone));
          unsigned nsteps = 0, nshort = 0, nclaim = 0;
          while (todo) {
              const int u = __ffsll((long long)todo) - 1;
              int pos = __builtin_amdgcn_readlane(cur, u);
              if (tr) { ++nsteps; nshort += pos == kShort; nclaim += pos < kShort; }
              if (pos == kNone) pos = -1;
              if (pos == kShort) {                         // list ran short: lanes over positions
                  uint4 q0, q1;
                  q0.x = __builtin_amdgcn_readlane(mq0.x, u); q0.y = __builtin_amdgcn_readlane(mq0.y, u);
                  q0.z = __builtin_amdgcn_readlane(mq0.z, u); q0.w = __builtin_amdgcn_readlane(mq0.w, u);
                  q1.x = __builtin_amdgcn_readlane(mq1.x, u); q1.y = __builtin_amdgcn_readlane(mq1.y, u);
                  q1.z = __builtin_amdgcn_readlane(mq1.z, u); q1.w = __builtin_amdgcn_readlane(mq1.w, u);
                  int lo = INT_MAX, hi = INT_MAX;
#pragma unroll
                  for (int c = 0; c < kBowRegChunks; ++c) {
                      if (c >= nch) break;
                      const int d = __popc(q0.x ^ fr0[c].x) + __popc(q0.y ^ fr0[c].y) + __popc(q0.z ^ fr0[c].z) +
                                    __popc(q0.w ^ fr0[c].w) + __popc(q1.x ^ fr1[c].x) + __popc(q1.y ^ fr1[c].y) +
                                    __popc(q1.z ^ fr1[c].z) + __popc(q1.w ^ fr1[c].w);
                      const int tbit = (int)(((c ? tk1 : tk0) >> lane) & 1);
                      key_push(lo, hi, ((d << 22) | (c * kWave + lane)) | (-tbit & INT_MAX));
                  }
                  const int r0 = wave_min(lo, INT_MAX);
                  const int r1 = wave_min(lane == (r0 & (kWave - 1)) ? hi : lo, INT_MAX);
                  pos = decide(r0, r1);
              }
              uint64_t later = todo & (todo - 1);          // the features after u
              if (pos >= 0) {
                  const int ikf = __builtin_amdgcn_readlane(my_ikf, u);
                  if (pos < kWave) {
                      tk0 |= 1ull << pos;
                      mcl[0] = lane == pos ? ikf : mcl[0];
                  } else {
                      tk1 |= 1ull << (pos - kWave);
                      mcl[1] = lane == pos - kWave ? ikf : mcl[1];
                  }
                  ++nm;
                  tb |= (q1 == pos ? 1 : 0) | (q2 == pos ? 2 : 0) | (q3 == pos ? 4 : 0);
                  cur = cur_of();
                  const uint64_t after = u == kWave - 1 ? 0ull : (~0ull << (u + 1));
                  later = okm & after & uniform64(__ballot(cur != kNone));
              }
              todo = later;
          }
          if (tr && lane == 0 && pbase == ko[ia]) { tr[12] = nsteps; tr[13] = nshort; tr[14] = nclaim; }
          if (coop) {
              uint64_t* T = (uint64_t*)(sq0 + 3 * 4 * kWave + kWave);
              if (lane == 0) { T[0] = tk0; T[1] = tk1; }
              __syncthreads();
          }
          if (tr && lane == 0 && pbase == ko[ia]) tr[8] = (unsigned)__builtin_amdgcn_s_memrealtime();
          continue;
        }
      }
      if constexpr (!kLds) {
          // wave-private LDS copy: one KF descriptor is then two broadcast LDS
          // reads instead of eight v_readlane (the small-node path is VALU-bound)
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // previous block's reads done
          __builtin_amdgcn_wave_barrier();
          s_q[lane] = mq0;
          s_q[kWave + lane] = mq1;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      for (uint64_t rem = __ballot(my_ok != 0); rem; rem &= rem - 1) {
        const int src = __ffsll((long long)rem) - 1;
        const int ikf = __builtin_amdgcn_readlane(my_ikf, src);
        uint4 q0, q1;
        if constexpr (!kLds) {
            q0 = s_q[src];
            q1 = s_q[kWave + src];
        } else {
            q0.x = __builtin_amdgcn_readlane(mq0.x, src); q0.y = __builtin_amdgcn_readlane(mq0.y, src);
            q0.z = __builtin_amdgcn_readlane(mq0.z, src); q0.w = __builtin_amdgcn_readlane(mq0.w, src);
            q1.x = __builtin_amdgcn_readlane(mq1.x, src); q1.y = __builtin_amdgcn_readlane(mq1.y, src);
            q1.z = __builtin_amdgcn_readlane(mq1.z, src); q1.w = __builtin_amdgcn_readlane(mq1.w, src);
        }
        // left (or only) track; right track when the frame is fisheye stereo (:296-323)
        int klo = INT_MAX, khi = INT_MAX, rlo = INT_MAX, rhi = INT_MAX;
        // branch-free (INT_MAX keys are no-ops; both tracks always pushed, so no
        // reference to a track is ever selected at run time)
        auto push_key = [&](int key, bool right) {
            if constexpr (kFish) {
                key_push(klo, khi, right ? INT_MAX : key);
                key_push(rlo, rhi, right ? key : INT_MAX);
            } else {
                key_push(klo, khi, key);
            }
        };
        auto push = [&](int d, int pos, bool right) { push_key(d == INT_MAX ? INT_MAX : (d << 22) | pos, right); };
        // key of a distance, INT_MAX when the lane's chunk-c bit is taken (arithmetic, no branch)
        auto key_of = [&](int d, int pos, int c) {
            const int tb = (int)((taken >> c) & 1);
            return ((d << 22) | pos) | (-tb & INT_MAX);
        };
        auto dist_reg = [&](const uint4& f0, const uint4& f1) {
            return __popc(q0.x ^ f0.x) + __popc(q0.y ^ f0.y) + __popc(q0.z ^ f0.z) + __popc(q0.w ^ f0.w) +
                   __popc(q1.x ^ f1.x) + __popc(q1.y ^ f1.y) + __popc(q1.z ^ f1.z) + __popc(q1.w ^ f1.w);
        };
        if constexpr (!kLds) {
#pragma unroll
            for (int c = 0; c < kBowRegChunks; ++c) {            // register chunks
                if (c >= nch) break;
                push_key(key_of(dist_reg(fr0[c], fr1[c]), c * kWave + lane, c), fish && fir[c] >= a.f_nleft);
            }
        } else {
            // LDS chunks (large-node blocks): positions past the node's end are taken, so
            // whatever the staging area holds there is never a candidate
#pragma unroll 2
            for (int c = 0; c < nlds; ++c) {
                const int pos = c * kWave + lane;
                const uint4 f0 = s_fd[pos], f1 = s_fd[kBowBigCap + pos];
                push_key(key_of(dist_reg(f0, f1), pos, c), fish && (s_fi[pos] & 0x7fffffff) >= a.f_nleft);
            }
        }
        for (int c = kLds ? nlds : kReg; c < nch; ++c) {     // global memory
            int d = INT_MAX, fi = -1;
            const int pos = c * kWave + lane;
            {
                if (pos < nf) fi = (int)a.f_idx[fb + pos];
                if (c < kBowMaskChunks) {
                    if (!((taken >> c) & 1)) d = hamming32(q0, q1, a.f_desc + (long long)fi * 32);
                } else if (pos < nf) {
                    if (match[fi] < 0 && (!a.f_valid || a.f_valid[fi]))
                        d = hamming32(q0, q1, a.f_desc + (long long)fi * 32);
                }
            }
            push(d, pos, fish && fi >= a.f_nleft);
        }
        const Best2 st = key_best2<true>(klo, khi);
        const Best2 sr = fish ? key_best2<false>(rlo, rhi) : Best2{256, 256, -1, 0, 0};   // ratio not applied
        auto claim = [&](int pos) {                  // pos: position in the node's F list
            const bool mine = lane == (pos & (kWave - 1));
            if ((pos >> 6) < kBowMaskChunks && mine) taken |= 1ull << (pos >> 6);
            // register chunks: the owning lane keeps the claim and the node's
            // matches go out as one coalesced store per chunk at its end; elsewhere
            // the frame index comes from the LDS copy or global memory.  (The
            // rotation bin of a match is k_bow_final's: it needs only the angles.)
            if (!kLds && pos < kBowRegChunks * kWave) {
                if (mine) {
                    if (pos < kWave) mcl[0] = ikf;
                    else mcl[kBowRegChunks - 1] = ikf;
                }
            } else {
                const int fi = (kLds && pos < kBowBigCap) ? (s_fi[pos] & 0x7fffffff) : (int)a.f_idx[fb + pos];
                if (lane == 0) match[fi] = ikf;
            }
            ++nm;
            if (nch > kBowMaskChunks) {              // the flag lives in `match` (global memory)
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
        };
        const bool low = a.f_valid ? st.best < kThLow : st.best <= kThLow;     // :848 / :327
        if (low && (float)st.best < a.ratio * (float)st.best2) claim(st.idx);
        if (fish && low && sr.best <= kThLow) claim(sr.idx);                   // :357-386, ratio ignored
      }
    }
    if constexpr (!kLds) {
#pragma unroll
        for (int c = 0; c < kBowRegChunks; ++c)
            if (mcl[c] >= 0) match[fir[c]] = mcl[c];
    }
    if (lane == 0 && nm) atomicAdd(&a.nmatches[pr], nm);
}

// Small frame nodes: each wave owns a contiguous run of KF nodes (all pairs
// flattened), one pair search per run, the pair advanced incrementally (KF
// nodes of consecutive keyframes are adjacent).
__device__ __forceinline__ void bow_nodes_body(const BowArgs& a, int bid, int nblocks, uint4* s_q) {
    extern __shared__ __attribute__((aligned(16))) int bow_smem[];
    // dynamic LDS: [staged KF validity][frame node ids][offsets]
    uint32_t* s_fnode = (uint32_t*)bow_smem + ((a.kv_lds + 15) >> 4) * 4;
    int* s_foff = (int*)s_fnode + a.f_nnodes;
    const bool lds_f = a.f_nnodes <= kBowLdsNodes;
    {
        // the staged validity (host memory) and the frame node table (HBM) in
        // one pass: each thread's reads of all three go out together
        const int n16 = (a.kv_lds + 15) >> 4, nn = lds_f ? a.f_nnodes + 1 : 0;
        for (int i = threadIdx.x; i < max(n16, nn); i += blockDim.x) {
            uint4 kv = make_uint4(0, 0, 0, 0);
            uint32_t fnd = 0;
            int fo = 0;
            if (i < n16) kv = ((const uint4*)a.kf_valid)[i];
            if (i < nn - 1) fnd = a.f_node[i];
            if (i < nn) fo = a.f_off[i];
            if (i < n16) ((uint4*)bow_smem)[i] = kv;
            if (i < nn - 1) s_fnode[i] = fnd;
            if (i < nn) s_foff[i] = fo;
        }
    }
    __syncthreads();
    if (a.tstart && threadIdx.x == 0) atomicMax(a.tstart + 1, (unsigned)__builtin_amdgcn_s_memrealtime());
    const uint32_t* fnode = lds_f ? s_fnode : a.f_node;
    const int* foff = lds_f ? s_foff : a.f_off;
    const bool one = a.single_nodes >= 0;
    const long long total = one ? a.single_nodes : a.node_off[a.npairs];
    // a single pair: a block per KF node, its four waves on it together (the
    // transposed nodes' lists split four ways); else a wave per KF node
    const bool coop = one;
    const long long nw = coop ? nblocks : (long long)nblocks * 4, w = coop ? bid : (long long)bid * 4 + wave_id();
    const long long per = (total + nw - 1) / nw;
    const long long g0 = w * per, g1 = min(total, g0 + per);
    if (g0 >= g1) return;
    unsigned* tr = a.wtrace ? a.wtrace + ((long long)bid * 4 + wave_id()) * 16 : nullptr;
    if (tr && lane_id() == 0) {
        tr[0] = a.tstart ? a.tstart[0] : 0u;
        tr[1] = (unsigned)__builtin_amdgcn_s_memrealtime();
        tr[10] = (unsigned)__builtin_amdgcn_s_memtime();
    }
    int pr = 0;
    if (!one) {
        int lo = 0, hi = a.npairs;                       // last pr with node_off[pr] <= g0
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (a.node_off[mid] <= g0) lo = mid;
            else hi = mid;
        }
        pr = lo;
    }
    long long pr_end = one ? total : a.node_off[pr + 1];
    for (long long g = g0; g < g1; ++g) {
        while (g >= pr_end) { ++pr; pr_end = a.node_off[pr + 1]; }
        const long long pr_base = one ? 0 : a.node_off[pr];
        const uint32_t na = a.kf_node[g];
        int fl = 0, fh = a.f_nnodes;                     // lower_bound of na in F's node ids
        while (fl < fh) {
            const int mid = (fl + fh) >> 1;
            if (fnode[mid] < na) fl = mid + 1;
            else fh = mid;
        }
        if (fl >= a.f_nnodes || fnode[fl] != na) continue;
        const int fb = foff[fl], fe = foff[fl + 1];
        if (fe - fb > kBowRegChunks * kWave) continue;  // a large-node block's
        if (tr && lane_id() == 0) tr[2] = (unsigned)__builtin_amdgcn_s_memrealtime();
        const int cw = coop ? wave_id() : -1;
        if (a.f_nleft >= 0) bow_node<false, true>(a, pr, (int)(g - pr_base), fb, fe, nullptr, nullptr, s_q, tr, cw);
        else bow_node<false, false>(a, pr, (int)(g - pr_base), fb, fe, nullptr, nullptr, s_q, tr, cw);
    }
    if (tr && lane_id() == 0) {
        tr[4] = (unsigned)__builtin_amdgcn_s_memrealtime();
        tr[11] = (unsigned)__builtin_amdgcn_s_memtime();
    }
    if (a.tstart && lane_id() == 0) atomicMax(a.tstart + 2, (unsigned)__builtin_amdgcn_s_memrealtime());
}

// Large frame nodes: block = kBowBigPairs consecutive keyframes; for each frame
// node of more than kBowRegChunks chunks the block stages the node's F
// descriptors in LDS, then wave w finds the node in keyframe w's FeatureVector.
// Block bid = (keyframe group, slot): the group's large nodes are dealt
// round-robin over `slots` blocks (one slot per large node for a single pair,
// where the host knows the frame's node sizes; one slot for a map).
__device__ __forceinline__ void bow_big_body(const BowArgs& a, int bid, int slots, uint4* s_fd, int* s_fi) {
    const int slot = bid % slots;
    const int pr = (bid / slots) * kBowBigPairs + wave_id();
    long long k0 = 0, k1 = 0;
    if (pr < a.npairs) {
        if (a.single_nodes >= 0) { k0 = 0; k1 = a.single_nodes; }
        else { k0 = a.node_off[pr]; k1 = a.node_off[pr + 1]; }
    }
    int nbig = 0;
    for (int fl = 0; fl < a.f_nnodes; ++fl) {
        const int fb = a.f_off[fl], fe = a.f_off[fl + 1];
        if (fe - fb <= kBowRegChunks * kWave) continue;              // uniform over the block
        if (nbig++ % slots != slot) continue;
        __syncthreads();                                             // previous node's readers done
        const int ns = min(fe - fb, kBowBigCap);
        for (int p = threadIdx.x; p < ns; p += blockDim.x) {
            const int fi = (int)a.f_idx[fb + p];
            const uint4* src = (const uint4*)(a.f_desc + (long long)fi * 32);
            s_fd[p] = src[0];
            s_fd[kBowBigCap + p] = src[1];
            s_fi[p] = fi | ((a.f_valid && !a.f_valid[fi]) ? (int)0x80000000u : 0);
        }
        __syncthreads();
        const uint32_t na = a.f_node[fl];
        long long lo = k0, hi = k1;                                  // lower_bound in KF pr's nodes
        while (lo < hi) {
            const long long mid = (lo + hi) >> 1;
            if (a.kf_node[mid] < na) lo = mid + 1;
            else hi = mid;
        }
        if (lo < k1 && a.kf_node[lo] == na) {
            if (a.f_nleft >= 0) bow_node<true, true>(a, pr, (int)(lo - k0), fb, fe, s_fd, s_fi, nullptr);
            else bow_node<true, false>(a, pr, (int)(lo - k0), fb, fe, s_fd, s_fi, nullptr);
        }
    }
}

// One launch for both: blocks [0, big_blocks) take the large nodes (latency-
// bound serial chains), the rest the small ones (VALU-bound), so the two
// co-schedule on the CUs.  Small-node blocks use s_fd as four wave-private
// descriptor areas (4 * 64 uint4 each: the KF descriptors of 64 features, or a
// transposed node's frame descriptors).
__device__ void bow_final_body(const BowArgs& a, int pr, int* hist, int* drop_p, uint8_t* sbin, int nbins,
                               int32_t* hcopy = nullptr);
// The end of a host call's kernel (the last block, every thread): each wave's
// result stores complete, then one lane releases them at system scope and
// writes the call's sequence number into the word the host polls.
__device__ __forceinline__ void signal_done(int* flag, int seq) {
    if (!flag) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The last-arriver hand-off of the single-launch kernels (the split-K recipe
// of cdna_hip_programming.md): every wave drains its stores, ONE lane releases
// at agent scope (a buffer_wbl2 per block, not one per thread as
// __threadfence() in every thread costs) and draws a relaxed agent-scope
// ticket; the block drawing the last one acquires and reads everyone's
// results.  flag: one int of the block's LDS.  Every thread calls it.
__device__ __forceinline__ bool last_arriver(unsigned* ticket, int* flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // keep: the fence's own wait can be dropped
        const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = t == gridDim.x - 1;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *flag = last;
    }
    __syncthreads();
    return *flag != 0;
}
static_assert(2 * kBowBigCap >= 4 * 4 * kWave, "s_fd holds the small-node waves' descriptor areas");
static_assert(kBowBigCap >= 41, "s_fi holds the fused final's histogram, drop count and last-arriver flag");
__global__ __launch_bounds__(256) void k_bow(BowArgs a, int big_blocks, int big_slots) {
    __shared__ uint4 s_fd[2 * kBowBigCap];
    __shared__ int s_fi[kBowBigCap];
    if (a.tstart && threadIdx.x == 0) atomicMin(a.tstart, (unsigned)__builtin_amdgcn_s_memrealtime());
    if (a.kv_lds > 0 && (int)blockIdx.x < big_blocks) {   // (small-node blocks stage it with their table)
        extern __shared__ __attribute__((aligned(16))) int bow_smem[];
        const int n16 = (a.kv_lds + 15) >> 4;
        for (int i = threadIdx.x; i < n16; i += blockDim.x) ((uint4*)bow_smem)[i] = ((const uint4*)a.kf_valid)[i];
        __syncthreads();
    }
    if ((int)blockIdx.x < big_blocks) bow_big_body(a, blockIdx.x, big_slots, s_fd, s_fi);
    else bow_nodes_body(a, blockIdx.x - big_blocks, gridDim.x - big_blocks, s_fd + wave_id() * 4 * kWave);
    if (a.fin_ticket) {
        // a single pair: the last block to finish runs the rotation filter on
        // every block's matches (the match rows, nmatches and the LDS are free)
        if (!last_arriver(a.fin_ticket, s_fi + 40)) return;
        const unsigned t_arrive = (unsigned)__builtin_amdgcn_s_memrealtime();
        const bool fused_copy = a.host_out && a.check_ori && ORB_BOWF_DROP4;
        bow_final_body(a, 0, s_fi, s_fi + 32, (uint8_t*)s_fd, (int)sizeof(s_fd), fused_copy ? a.host_out : nullptr);
        if (a.tstart && threadIdx.x == 0) {
            const unsigned t0 = *a.tstart;
            a.host_out[a.f_n + 1] = (int)(t_arrive - t0);
            a.host_out[a.f_n + 2] = (int)((unsigned)__builtin_amdgcn_s_memrealtime() - t_arrive);
            a.host_out[a.f_n + 3] = (int)(a.tstart[1] - t0);    // the last block past its table load
            a.host_out[a.f_n + 4] = (int)(a.tstart[2] - t0);    // the last wave past its nodes
            a.tstart[0] = 0xffffffffu;
            a.tstart[1] = 0u;
            a.tstart[2] = 0u;
        }
        if (a.host_out) {
            __syncthreads();
            if (!fused_copy)
                for (int i = threadIdx.x; i < a.f_n; i += blockDim.x) {
                    a.host_out[i] = a.match[i];
                    if (a.reset_after) a.match[i] = -1;
                }
            if (threadIdx.x == 0) {
                a.host_out[a.f_n] = a.nmatches[0];
                if (a.reset_after) {
                    a.nmatches[0] = 0;
                    *a.fin_ticket = 0u;
                }
            }
            signal_done(a.done, a.seq);
        }
    }
}

// Rotation-consistency filter (:404-422 / :884-902) and the KF-KF output, one
// workgroup per pair.  Every match of either track enters the reference's
// histogram with the bin of (KF angle - F angle), so the bins are computed
// here, lane-parallel over the frame features, instead of in the serial loop.
constexpr int kBowFinalBins = 16384;    // frame features whose bin k_bow_final keeps in LDS

// hist: 32 ints, drop: 1 int, sbin: nbins bytes of LDS (the bin of each match,
// one gather of the KF angle).  hcopy (the single-pair kernel, with check_ori):
// the filtered row also goes there in the same pass (and, with reset_after, the
// row is left at -1), instead of a separate copy pass.
__device__ void bow_final_body(const BowArgs& a, int pr, int* hist, int* drop_p, uint8_t* sbin, int nbins,
                               int32_t* hcopy) {
    const int tid = threadIdx.x, nt = blockDim.x;
    int32_t* match = a.match + (long long)pr * a.f_n;
    int& drop = *drop_p;
    if (a.check_ori) {
        const orb_keypoint* KK = a.kf_kps + (a.single_nodes >= 0 ? 0 : a.kp_off[pr]);
        if (tid < 32) hist[tid] = 0;
        if (tid == 0) drop = 0;
        __syncthreads();
        // four rows in flight per thread: their match loads, then their angle
        // gathers, then the bins (one dependent load chain per four matches)
        constexpr int kU = 4;
        for (int i0 = tid; i0 < a.f_n; i0 += kU * nt) {
            int m[kU];
            float ka[kU], fa[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) m[u] = i0 + u * nt < a.f_n ? match[i0 + u * nt] : -1;
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                ka[u] = m[u] >= 0 ? KK[m[u]].angle : 0.f;
                fa[u] = m[u] >= 0 ? a.f_kps[i0 + u * nt].angle : 0.f;
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int i = i0 + u * nt;
                const int b = m[u] >= 0 ? rot_bin(ka[u], fa[u]) : -1;
                hist_add_wave(hist, b);
                if (b >= 0 && i < nbins) sbin[i] = (uint8_t)b;
            }
        }
        __syncthreads();
        int i1, i2, i3;
        three_maxima_wave(hist, i1, i2, i3);
        int d = 0;
#if ORB_BOWF_DROP4
        // four rows' match loads in flight per thread
        for (int i0 = tid; i0 < a.f_n; i0 += 4 * nt) {
            int m[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) m[u] = i0 + u * nt < a.f_n ? match[i0 + u * nt] : -1;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = i0 + u * nt;
                if (hcopy && i < a.f_n) {
                    bool keep = m[u] >= 0;
                    if (keep) {
                        const int b = i < nbins ? sbin[i] : rot_bin(KK[m[u]].angle, a.f_kps[i].angle);
                        keep = b == i1 || b == i2 || b == i3;
                        d += !keep;
                    }
                    hcopy[i] = keep ? m[u] : -1;
                    if (m[u] >= 0 && (a.reset_after || !keep)) match[i] = -1;
                    continue;
                }
                if (m[u] < 0) continue;
                const int b = i < nbins ? sbin[i] : rot_bin(KK[m[u]].angle, a.f_kps[i].angle);
                if (b == i1 || b == i2 || b == i3) continue;
                match[i] = -1;
                ++d;
            }
        }
#else
        for (int i = tid; i < a.f_n; i += nt) {
            const int m = match[i];
            if (m < 0) continue;
            const int b = i < nbins ? sbin[i] : rot_bin(KK[m].angle, a.f_kps[i].angle);
            if (b == i1 || b == i2 || b == i3) continue;
            match[i] = -1;
            ++d;
        }
#endif
        d = wave_sum(d);
        if (lane_id() == 0 && d) atomicAdd(&drop, d);
        __syncthreads();
        if (tid == 0) a.nmatches[pr] -= drop;
    }
    if (a.out12) {
        __syncthreads();
        const long long kpo = a.kp_off[pr];
        const int kn1 = (int)(a.kp_off[pr + 1] - kpo);
        int32_t* o12 = a.out12 + kpo;
        for (int i = tid; i < kn1; i += nt) o12[i] = -1;
        __syncthreads();
        for (int i = tid; i < a.f_n; i += nt)
            if (match[i] >= 0) o12[match[i]] = i;
    }
}

__global__ __launch_bounds__(256) void k_bow_final(BowArgs a) {
    __shared__ int hist[32];
    __shared__ int drop;
    __shared__ uint8_t sbin[kBowFinalBins];
    bow_final_body(a, blockIdx.x, hist, &drop, sbin, kBowFinalBins);
}

// The per-call state of k_bow in one launch (instead of memsets).
__global__ __launch_bounds__(256) void k_bow_init(BowArgs a) {
    const long long nmf = (long long)a.npairs * a.f_n, stride = (long long)gridDim.x * blockDim.x;
    const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    for (long long i = t0; i < nmf; i += stride) a.match[i] = -1;
    for (long long i = t0; i < a.npairs; i += stride) a.nmatches[i] = 0;
}

// big_slots: blocks per keyframe group for the large frame nodes (their count
// when the host holds the frame's FeatureVector, else 1); kf_nodes: the KF
// FeatureVector nodes in all when the host knows them (a single pair: one
// wave per node, for latency), else -1.
// With a.fin_ticket (one pair, match / nmatches initialised by the caller)
// the call is the one k_bow launch.
static int launch_bow(BowArgs& a, int npairs, hipStream_t st, int big_slots = 1, long long kf_nodes = -1) {
    a.npairs = npairs;
    if (a.fin_ticket && npairs != 1) return ORB_ERR_PARAM;
    if (!a.fin_ticket) {
        const long long nmf = (long long)npairs * a.f_n;
        const int ib = (int)std::min<long long>(4096, std::max<long long>(1, (nmf + 1023) / 1024));
        KLAUNCH(k_bow_init, dim3(ib), dim3(256), 0, st, a);
    }
    // (one pair: a block per KF node, bow_nodes_body's cooperative form)
    const long long want = kf_nodes >= 0 ? (a.single_nodes >= 0 ? kf_nodes : (kf_nodes + 3) / 4) : (long long)npairs * 8;
    const int blocks = (int)std::min<long long>(65535, std::max<long long>(1, want));
    big_slots = std::max(1, big_slots);
    const int big_blocks = (npairs + kBowBigPairs - 1) / kBowBigPairs * big_slots;
    KLAUNCH(k_bow, dim3(big_blocks + blocks), dim3(256), bow_lds(a.f_nnodes, a.kv_lds), st, a, big_blocks,
            big_slots);
    if (!a.fin_ticket) KLAUNCH(k_bow_final, dim3(npairs), dim3(256), 0, st, a);
    return hipGetLastError() == hipSuccess ? ORB_OK : ORB_ERR_DEVICE;
}

// ---------------------------------------------------------------------------
// Map-wide SearchByBoW(KF_i, F) (mono frame, ORBmatcher.cc:223-425) with a
// lane per KEYFRAME feature.  In k_bow a wave walks one (keyframe, node)'s KF
// features serially and spends two wave reductions per KF feature; a node of
// 40 frame features then keeps 24 of 64 lanes idle.  Here:
//   k_bowk_map     (pair, KF node) g -> frame node fl, KF feature count; a
//                  slot range in fl's bucket by one atomic
//   k_bowk_scan    bucket starts (buckets padded to 64 slots)
//   k_bowk_fill    slot -> global KF feature index (or none: no valid MapPoint)
//   k_bowk_expand  the frame's descriptors as +-1 int8 rows in node order
//   k_bowk_topk_mfma  one wave per 32 slots of one frame node: each slot's KF
//                  feature keeps the kBowK smallest keys (distance << 16 |
//                  position in the frame node) over ALL the node's frame
//                  features, the distances as int8 dot products on
//                  v_mfma_i32_32x32x32_i8
//   k_bowk_resolve_lane  one thread per g: the reference's serial walk over the
//                  node's KF features.  A frame feature is "taken" when an earlier KF
//                  feature of the same (pair, node) claimed it; best / second
//                  of a KF feature are the first two untaken keys of its list,
//                  exact because every frame feature off the list has a larger
//                  key.  With one untaken key, the last listed distance bounds
//                  the second from below, which decides the ratio test unless
//                  best >= ratio * that bound; only then (or with no untaken
//                  key of an incomplete list while a claim is still possible)
//                  is the node rescanned exactly, lane-parallel.
// k_bow_final (rotation filter, counts) follows unchanged.
// ---------------------------------------------------------------------------
#ifndef ORB_BOWK_K
#define ORB_BOWK_K 4
#endif
constexpr int kBowK = ORB_BOWK_K;
static_assert(kBowK == 2 || kBowK == 4, "a slot's list is one 8- or 16-byte load");
typedef uint32_t bowk_list __attribute__((ext_vector_type(kBowK)));
// the lane resolve's LDS bitmap: 16 words (512 positions) a thread, odd pitch
constexpr int kBowLaneWords = 16, kBowLanePitch = 17;

struct BowKArgs {
    BowArgs b;
    long long G;           // (pair, KF node) entries
    int* g_fl;             // [G] frame node of g, -1 if F does not hold it
    int* g_off;            // [G] offset of g's KF features in the node's bucket
    int* g_pr;             // [G] pair of g
    unsigned long long* bgcount;   // [f_nnodes][nsub] (zeroed): lo KF features, hi g entries; after
                                   // k_bowk_scan the exclusive prefixes of both within the node
    int nsub;                      // sub-counters per frame node (pair & (nsub - 1)): spreads the atomics
    int* node_n;                   // [f_nnodes + 1] KF features per frame node; [f_nnodes]: any node the
                                   // big-node resolve form takes (written by k_bowk_scan)
    int* bstart;           // [f_nnodes + 1] bucket starts, padded to 64 slots
    uint32_t* slot_src;    // [slots] global KF feature (kp_off[pr] + ikf), ~0: none
    bowk_list* lists;      // [slots] kBowK smallest keys, ascending, ~0: none
    int* gstart;           // [f_nnodes + 1] their starts
    int* g_rank;           // [G] rank of g among its frame node's entries
    int* perm;             // [G] g entries ordered by frame node
    int* chunk_node;       // [slots / 32] frame node of every 32-slot chunk
    uint32_t* slot_pos;    // [slots] FeatureVector position (row of kf_fvdesc) when kf_fvdesc is set
    uint16_t* claim;       // [slots] the resolve's claim (frame feature index, 0xffff: none) for
                           // k_bowk_final, or NULL: claims go straight to the match rows (then k_bow_final)
};

// A g's slots run from an 8-aligned offset of its bucket (buckets start at
// multiples of 64) over its KF features rounded up to 8, the tail slots
// holding no feature: the resolve reads and writes a g's slots 8 at a time
// with aligned vector accesses.
__device__ __forceinline__ int kf_run(int nkf) { return (nkf + 7) & ~7; }

// One block per pair (its KF nodes g are contiguous: no search for the pair
// of g), the frame's node ids staged in LDS for the lower_bound of each KF
// node when they fit (~100 nodes at levelsup 4)
constexpr int kBowMapStage = 2048;
__global__ __launch_bounds__(256) void k_bowk_map(BowKArgs k) {
    __shared__ uint32_t s_fnode[kBowMapStage];
    const BowArgs& a = k.b;
    const int pr = blockIdx.x;
    const int nfn = a.f_nnodes;
    const bool st = nfn <= kBowMapStage;
    if (st)
        for (int i = threadIdx.x; i < nfn; i += blockDim.x) s_fnode[i] = a.f_node[i];
    __syncthreads();
    const uint32_t* fnode = st ? s_fnode : a.f_node;
    const long long g0 = a.node_off[pr], g1 = a.node_off[pr + 1];
    const int* ko = a.kf_off + g0 + pr;
    for (long long g = g0 + threadIdx.x; g < g1; g += blockDim.x) {
        const int ia = (int)(g - g0);
        const int nkf = ko[ia + 1] - ko[ia];
        const uint32_t na = a.kf_node[g];
        int fl = 0, fh = nfn;                        // lower_bound of na in F's node ids
        while (fl < fh) {
            const int mid = (fl + fh) >> 1;
            if (fnode[mid] < na) fl = mid + 1;
            else fh = mid;
        }
        k.g_pr[g] = pr;
        if (fl < nfn && fnode[fl] == na && nkf > 0) {
            k.g_fl[g] = fl;
            // one atomic for both counters (a pair holds a frame node at most once, so
            // nothing aggregates in the block), on one of nsub words of the node: ~10k
            // same-address atomics per node serialised at L2 (0.22 ms) otherwise
            const unsigned long long o =
                atomicAdd(k.bgcount + (long long)fl * k.nsub + (pr & (k.nsub - 1)),
                          (1ull << 32) | (unsigned long long)kf_run(nkf));
            k.g_off[g] = (int)(uint32_t)o;
            k.g_rank[g] = (int)(o >> 32);
        } else {
            k.g_fl[g] = -1;
        }
    }
}

__global__ __launch_bounds__(1024) void k_bowk_scan(BowKArgs k) {
    extern __shared__ int sc_s[];                    // [2 n]: padded KF features, then g entries per node
    const int n = k.b.f_nnodes;
    // the node's sub-counters -> exclusive prefixes in place, totals to LDS
    if (k.nsub == kWave) {                           // a wave per node, a lane per sub-counter
        const int nw = blockDim.x / kWave, lane = lane_id();
        for (int i = wave_id(); i < n; i += nw) {
            unsigned long long* c = k.bgcount + (long long)i * kWave;
            const unsigned long long v = c[lane];
            const int lo = (int)(uint32_t)v, hi = (int)(v >> 32);
            const int ilo = wave_incl_scan(lo), ihi = wave_incl_scan(hi);
            c[lane] = ((unsigned long long)(uint32_t)(ihi - hi) << 32) | (uint32_t)(ilo - lo);
            if (lane == kWave - 1) {
                sc_s[i] = (ilo + kWave - 1) / kWave * kWave;
                sc_s[n + i] = ihi;
                k.node_n[i] = ilo;
            }
        }
    } else {
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const unsigned long long v = k.bgcount[i];
            k.bgcount[i] = 0;
            k.node_n[i] = (int)(uint32_t)v;
            sc_s[i] = ((int)(uint32_t)v + kWave - 1) / kWave * kWave;
            sc_s[n + i] = (int)(v >> 32);
        }
    }
    __syncthreads();
    // any node with entries that the big-node resolve form takes (> 512 features)
    __shared__ int s_big;
    if (threadIdx.x == 0) s_big = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        if (sc_s[n + i] > 0 && k.b.f_off[i + 1] - k.b.f_off[i] > 32 * kBowLaneWords) s_big = 1;
    __syncthreads();
    if (threadIdx.x == 0) k.node_n[n] = s_big;
    __shared__ int tmp[1024 / kWave + 1];
    const int total = block_excl_scan(sc_s, n, tmp);
    for (int i = threadIdx.x; i < n; i += blockDim.x) k.bstart[i] = sc_s[i];
    if (threadIdx.x == 0) k.bstart[n] = total;
    __syncthreads();
    const int gtotal = block_excl_scan(sc_s + n, n, tmp);
    for (int i = threadIdx.x; i < n; i += blockDim.x) k.gstart[i] = sc_s[n + i];
    if (threadIdx.x == 0) k.gstart[n] = gtotal;
}

// the frame node of every 32-slot chunk of the buckets (a table lookup
// instead of a binary search over bstart per top-4 wave)
__global__ __launch_bounds__(256) void k_bowk_chunks(BowKArgs k) {
    const int fl = blockIdx.x;
    const int c0 = k.bstart[fl] / 32, c1 = k.bstart[fl + 1] / 32;
    for (int c = c0 + threadIdx.x; c < c1; c += blockDim.x) k.chunk_node[c] = fl;
    // the bucket's padding slots hold no keyframe feature (instead of a memset
    // of every slot)
    const int p0 = k.bstart[fl] + k.node_n[fl], p1 = k.bstart[fl + 1];
    for (int p = p0 + threadIdx.x; p < p1; p += blockDim.x) k.slot_src[p] = 0xffffffffu;
}

// One block per pair: every thread over the pair's KF features in
// FeatureVector order (contiguous), each feature's node found by a search of
// the node offsets staged in LDS together with the node's slot base (a wave
// per node left 60 % of its lanes idle on ~38-feature nodes).  Pairs with
// more nodes than the stage take them a wave per node.
constexpr int kBowFillStage = 1024;
#ifndef ORB_BOWKFILL_U
#define ORB_BOWKFILL_U 4   // k_bowk_fill: features a thread in flight
#endif
__global__ __launch_bounds__(256) void k_bowk_fill(BowKArgs k) {
    __shared__ int s_ko[kBowFillStage + 1];
    __shared__ int s_base[kBowFillStage];
    const BowArgs& a = k.b;
    const int pr = blockIdx.x;
    const long long g0 = a.node_off[pr];
    const int nn = (int)(a.node_off[pr + 1] - g0);
    const int* ko = a.kf_off + g0 + pr;
    const uint32_t* ki = a.kf_idx + a.idx_off[pr];
    const long long kpo = a.kp_off[pr];
    auto slot_base = [&](int ia) -> int {            // slot of the node's feature p: base + p; -1: no frame node
        const long long g = g0 + ia;
        const int fl = k.g_fl[g];
        if (fl < 0) return -1;
        // the sub-counter's prefix within the node; the final offset stays in
        // g_off for the resolve
        const unsigned long long sb = k.bgcount[(long long)fl * k.nsub + (pr & (k.nsub - 1))];
        const int off = k.g_off[g] + (int)(uint32_t)sb;
        k.g_off[g] = off;
        k.perm[k.gstart[fl] + k.g_rank[g] + (int)(sb >> 32)] = (int)g;
        return k.bstart[fl] + off - ko[ia];
    };
    const uint32_t fvo = (uint32_t)a.idx_off[pr];
    auto put = [&](int base, int p) {
        const long long gk = kpo + (long long)ki[p];
        k.slot_src[base + p] = a.kf_valid[gk] ? (uint32_t)gk : 0xffffffffu;
        if (a.kf_fvdesc) k.slot_pos[base + p] = fvo + (uint32_t)p;
    };
    if (nn > kBowFillStage) {
        for (int ia = wave_id(); ia < nn; ia += blockDim.x / kWave) {
            int base = 0;
            if (lane_id() == 0) base = slot_base(ia);
            base = __shfl(base, 0, kWave);
            if (base < 0) continue;
            for (int p = ko[ia] + lane_id(); p < ko[ia + 1]; p += kWave) put(base, p);
            const int pe = ko[ia] + kf_run(ko[ia + 1] - ko[ia]);       // the run's tail: no feature
            if (ko[ia + 1] + lane_id() < pe) k.slot_src[base + ko[ia + 1] + lane_id()] = 0xffffffffu;
        }
        return;
    }
    for (int ia = threadIdx.x; ia <= nn; ia += blockDim.x) {
        s_ko[ia] = ko[ia];
        if (ia < nn) {
            const int b = slot_base(ia);
            s_base[ia] = b;
            if (b >= 0) {                                              // the run's tail: no feature
                const int p0 = ko[ia], p1 = ko[ia + 1];
                for (int p = p1; p < p0 + kf_run(p1 - p0); ++p) k.slot_src[b + p] = 0xffffffffu;
            }
        }
    }
    __syncthreads();
    const int p0 = s_ko[0], p1 = s_ko[nn];
    // four features in flight per thread: their FeatureVector indices, then
    // their MapPoint flags, then the stores (one dependent load chain per four)
    constexpr int kU = ORB_BOWKFILL_U;
    const int bd = blockDim.x;
    for (int q = p0 + threadIdx.x; q < p1; q += kU * bd) {
        int bs[kU];
        uint32_t kv[kU];
        uint8_t vv[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int p = q + u * bd;
            int lo = 0, hi = nn;                     // last ia with s_ko[ia] <= p (empty nodes skipped)
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (s_ko[mid] <= p) lo = mid;
                else hi = mid;
            }
            bs[u] = p < p1 ? s_base[lo] : -1;
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) kv[u] = bs[u] >= 0 ? ki[q + u * bd] : 0u;
#pragma unroll
        for (int u = 0; u < kU; ++u) vv[u] = bs[u] >= 0 ? a.kf_valid[kpo + (long long)kv[u]] : (uint8_t)0;
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (bs[u] < 0) continue;
            const int p = q + u * bd;
            k.slot_src[bs[u] + p] = vv[u] ? (uint32_t)(kpo + (long long)kv[u]) : 0xffffffffu;
            if (a.kf_fvdesc) k.slot_pos[bs[u] + p] = fvo + (uint32_t)p;
        }
    }
}

// (topk_push, the sorted insertion of the kBowK smallest keys: above, with SearchForInitialization)

// The same lists with the distances on the matrix cores.  A descriptor's 256
// bits as +-1 int8 make Hamming distance a dot product, dot = 256 - 2 ham,
// so a (32 frame features) x (32 keyframe features) tile of a node is eight
// v_mfma_i32_32x32x32_i8 (K = 32 bits each), exact in i32.  Operand maps
// (checked by tools/mfma_i8_probe.hip): lane l feeds A row l & 31 and B
// column l & 31 with the 16-element k-slice 16 (l >> 5) .. +15 of each K = 32
// block; C holds column l & 31, rows (reg & 3) + 8 (reg >> 2) + 4 (l >> 5).
// Here A = frame features (rows, expanded once per query by k_bowk_expand),
// B = the wave's 32 keyframe features (columns); each lane pushes its 16
// accumulator rows into its column's top-4, and lanes l, l ^ 32 (the other
// 16 rows of every tile) merge at the end.
typedef int bowk_v4i __attribute__((ext_vector_type(4)));
typedef int bowk_v16i __attribute__((ext_vector_type(16)));

// 16 bits (bit e -> byte e) as +-1 int8: four bytes per nibble spread
// (per nibble: bit i -> byte i as 4 (bfe, v_mul_u32_u24, and), then one v_perm
// picking byte 0x01 (selector 4) or 0xff (selector 0) -- no quarter-rate
// v_mul_lo_u32)
__device__ __forceinline__ bowk_v4i bits_pm1(uint32_t x16) {
    bowk_v4i o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t nib = (x16 >> (4 * q)) & 0xfu;
        const uint32_t sel = (nib * 0x00810204u) & 0x04040404u;   // nibble bit i -> byte i, value 4
        o[q] = (int)__builtin_amdgcn_perm(0x01010101u, 0xffffffffu, sel);
    }
    return o;
}

// the frame's node positions p (f_idx order: a node's features are
// contiguous) as +-1 int8, [position][dword s][half h] 16-byte slices, so a
// node's tile is one contiguous read with no index indirection
__global__ __launch_bounds__(256) void k_bowk_expand(const uint8_t* __restrict__ f_desc,
                                                     const uint32_t* __restrict__ f_idx, const int* __restrict__ npos,
                                                     bowk_v4i* __restrict__ fexp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;   // (position, dword, half)
    if (i >= *npos * 16) return;
    const int p = i >> 4, s = (i >> 1) & 7, h = i & 1;
    const uint32_t d = ((const uint32_t*)(f_desc + (long long)f_idx[p] * 32))[s];
    fexp[i] = bits_pm1(d >> (16 * h));
}

// a key without the lane half's row offset: (256 - acc) << 15 == ham << 16
// (acc = 256 - 2 ham), plus the uniform part of the row.  Plain 24-bit
// arithmetic (|acc| <= 256, acc * -32768 and the sum fit 24 x 24 -> 32 bits).
// It must stay visible to
// the compiler: acc is an MFMA result, and the hazard recognizer inserts the
// MFMA -> VALU read wait states only for instructions it can see.  Round 2
// wrote this as an inline-asm v_mad_i32_i24 reading the accumulator directly;
// with the accumulators in VGPRs (the compiler's VGPR-destination MFMA form)
// the asm read them before the MFMA had written them back and lost matches
// (8 of 2125), which an AGPR pin (a compiler-visible v_accvgpr_read first)
// had hidden.
__device__ __forceinline__ uint32_t bowk_key(int acc, int neg, int kb) {
    return (uint32_t)(__mul24(acc, neg) + kb);
}

// The block's 4 waves (128 keyframe slots) share their frame node's tiles:
// the block copies each 32-feature tile of the node-ordered expansion into
// LDS once (8 KB, double-buffered), so an A fragment is a ds_read_b128, not a
// re-read of the 8x larger expanded descriptors from L2 by every wave.  The
// copy is software-pipelined: tile t+2 is loaded into registers while tile t
// is on the matrix cores, and lands in LDS after the next barrier (a barrier
// that orders LDS only, so the load in flight is not drained by it).  A wave
// whose slots lie in another node than the block's first reads its tiles
// from fexp.
__device__ __forceinline__ void bowk_lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
#ifndef ORB_BOWK_AGPR_PIN
#define ORB_BOWK_AGPR_PIN 0
#endif
#ifndef ORB_BOWK_WPE
#define ORB_BOWK_WPE 3   // A/B per C5 query: 3.98 at 3, 4.02-4.09 at 4-5 on one box (B stays in VGPRs); 6 and 7 slower
#endif
// NSET keyframe column sets of 32 per wave (a wave's 32 NSET slots lie in one
// bucket: buckets are padded to 64): with NSET = 2 every A fragment read from
// LDS feeds two MFMAs and one set's MFMA chain overlaps the other set's
// top-4 epilogue inside the wave.
template <int NSET>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NSET == 1 ? ORB_BOWK_WPE : 2)))
void k_bowk_topk_mfma(BowKArgs k, const bowk_v4i* __restrict__ fexp) {
    // [buffer][row * 17 + 2 s + h]: the odd row pitch (272 B) keeps a
    // ds_read_b128 of 32 rows at one (s, h) off a single bank group
    __shared__ bowk_v4i s_a[2][32 * 17];
    // byte -> its 8 bits as +-1 int8 (bit e -> byte e): a keyframe descriptor's
    // B operand is 2 table reads per 16 bits (4 VALU ops) instead of 4 nibble
    // spreads (16 VALU ops)
    __shared__ uint2 s_pm1[256];
    {
        const uint32_t t = threadIdx.x;   // blockDim = 256: one entry each
        const uint32_t sel = ((t & 0xfu) * 0x00810204u) & 0x04040404u, seh = ((t >> 4) * 0x00810204u) & 0x04040404u;
        s_pm1[t] = make_uint2(__builtin_amdgcn_perm(0x01010101u, 0xffffffffu, sel),
                              __builtin_amdgcn_perm(0x01010101u, 0xffffffffu, seh));
    }
    __syncthreads();
    const BowArgs& a = k.b;
    constexpr int kWS = 32 * NSET;                   // slots per wave
    const long long slotb = (long long)blockIdx.x * 4 * kWS;
    const long long slot0 = slotb + (long long)wave_id() * kWS;
    const int total = __builtin_amdgcn_readfirstlane(k.bstart[a.f_nnodes]);
    if (slotb >= total) return;                      // the whole block
    auto node_of = [&](long long slot) {             // last fl with bstart[fl] <= slot
        return __builtin_amdgcn_readfirstlane(k.chunk_node[slot >> 5]);
    };
    const int flb = node_of(slotb);
    const int fbb = __builtin_amdgcn_readfirstlane(a.f_off[flb]);
    const int nfb = __builtin_amdgcn_readfirstlane(a.f_off[flb + 1]) - fbb;
    const bool live = slot0 < total;                 // buckets are padded to 64: a wave's slots never straddle
    const int fl = live ? (slot0 == slotb ? flb : node_of(slot0)) : flb;
    const bool shared_node = fl == flb;
    const int fb = __builtin_amdgcn_readfirstlane(a.f_off[fl]);
    const int nf = __builtin_amdgcn_readfirstlane(a.f_off[fl + 1]) - fb;
    const int lane = lane_id(), col = lane & 31, h = lane >> 5;
    bowk_v4i B[NSET][8];
#pragma unroll
    for (int c = 0; c < NSET; ++c) {
        const uint32_t src = live ? k.slot_src[slot0 + 32 * c + col] : 0xffffffffu;
        uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (src != 0xffffffffu) {
            // a (keyframe, node)'s slots are consecutive FeatureVector rows: with the
            // map's fv_desc the wave's 32 descriptors are one contiguous 1 KB read
            const uint8_t* kd = a.kf_fvdesc ? a.kf_fvdesc + (long long)k.slot_pos[slot0 + 32 * c + col] * 32
                                            : a.kf_desc + (long long)src * 32;
            const uint4 q0 = *(const uint4*)kd;
            const uint4 q1 = *(const uint4*)(kd + 16);
            d[0] = q0.x; d[1] = q0.y; d[2] = q0.z; d[3] = q0.w; d[4] = q1.x; d[5] = q1.y; d[6] = q1.z; d[7] = q1.w;
        }
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2) {
            const uint2 lo = s_pm1[__builtin_amdgcn_ubfe(d[s2], 16 * h, 8)];
            const uint2 hi = s_pm1[__builtin_amdgcn_ubfe(d[s2], 16 * h + 8, 8)];
            B[c][s2] = bowk_v4i{(int)lo.x, (int)lo.y, (int)hi.x, (int)hi.y};
        }
    }
    uint32_t kk[NSET][kBowK];
#pragma unroll
    for (int c = 0; c < NSET; ++c)
#pragma unroll
        for (int t = 0; t < kBowK; ++t) kk[c][t] = 0xffffffffu;
    // -32768 in a VGPR and the key base in an SGPR, both opaque to the
    // compiler (empty asm on constants, no MFMA operand involved): a key is
    // then a v_mul_i32_i24 and an add (as many VALU ops as round 2's
    // v_accvgpr_read + inline v_mad) instead of a shift, a subtract and an add
    int neg = -32768, kbase = 256 << 15;
    asm volatile("" : "+v"(neg));
    asm volatile("" : "+s"(kbase));
    // a 32x32 tile per set: its 16 accumulator rows of this lane into the
    // column's top-4 (keys without + 4 h: the order of one lane's keys is the same)
    auto tile_mfma = [&](const bowk_v4i* ar, int t0, int nfx) {
        bowk_v16i acc[NSET];
#pragma unroll
        for (int c = 0; c < NSET; ++c) acc[c] = bowk_v16i{};
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2) {
            const bowk_v4i A = ar[2 * s2];
#pragma unroll
            for (int c = 0; c < NSET; ++c) acc[c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, B[c][s2], acc[c], 0, 0, 0);
        }
#if ORB_BOWK_AGPR_PIN
        // build knob: accumulators forced into AGPRs (round 2's workaround for
        // the inline-asm key above; see bowk_key)
#pragma unroll
        for (int c = 0; c < NSET; ++c) asm volatile("" : "+a"(acc[c]));
#endif
        const int kb = kbase + t0;
        if (t0 + 32 <= nfx) {
#pragma unroll
            for (int c = 0; c < NSET; ++c)
#pragma unroll
                for (int g = 0; g < 16; ++g) {
                    // the row's key base opaque in an SGPR: one v_mad_i32_i24 per key
                    // (the compiler otherwise folds the row constant into a
                    // v_mul_i32_i24 + v_add3_u32 pair)
                    int cg = kb + (g & 3) + 8 * (g >> 2);
                    asm volatile("" : "+s"(cg));
                    topk_push(kk[c], bowk_key(acc[c][g], neg, cg));
                }
        } else {
            const int lim = nfx - t0 - 4 * h;        // rows (g & 3) + 8 (g >> 2) below it exist
            const int lim0 = nfx - t0;               // the h = 0 half's bound, wave-uniform
#pragma unroll
            for (int c = 0; c < NSET; ++c)
#pragma unroll
                for (int g = 0; g < 16; ++g) {
                    // a row no lane holds is skipped by a scalar branch (a node's
                    // last tile is on average half empty)
                    if ((g & 3) + 8 * (g >> 2) >= lim0) continue;
                    int cg = kb + (g & 3) + 8 * (g >> 2);
                    asm volatile("" : "+s"(cg));
                    const uint32_t key = bowk_key(acc[c][g], neg, cg);
                    topk_push(kk[c], (g & 3) + 8 * (g >> 2) < lim ? key : 0xffffffffu);
                }
        }
    };
    // block-uniform loop over the block node's tiles: every thread reaches
    // every barrier; the staged tile serves the waves of that node
    const int ntb = (nfb + 31) / 32;
    const int srow = threadIdx.x >> 3, ss = threadIdx.x & 7;   // staging: row, dword (both halves)
    bowk_v4i p0, p1;
    auto fetch = [&](int tile) {
        const bowk_v4i* g = fexp + (long long)(fbb + min(tile * 32 + srow, nfb - 1)) * 16 + 2 * ss;
        p0 = g[0];
        p1 = g[1];
    };
    auto put = [&](int buf) {
        s_a[buf][srow * 17 + 2 * ss] = p0;
        s_a[buf][srow * 17 + 2 * ss + 1] = p1;
    };
    if (ntb > 0) { fetch(0); put(0); }
    if (ntb > 1) fetch(1);
    for (int tile = 0; tile < ntb; ++tile) {
        bowk_lds_barrier();                          // tile's buffer written; the other one free
        if (tile + 1 < ntb) {
            put((tile + 1) & 1);
            if (tile + 2 < ntb) fetch(tile + 2);
        }
        if (live && shared_node) tile_mfma(&s_a[tile & 1][col * 17 + h], tile * 32, nf);
    }
    if (live && !shared_node) {
        for (int t0 = 0; t0 < nf; t0 += 32) {
            const int fr = min(t0 + col, nf - 1);
            tile_mfma(fexp + (long long)(fb + fr) * 16 + h, t0, nf);
        }
    }
    if (!live) return;
#pragma unroll
    for (int c = 0; c < NSET; ++c) {
        uint32_t (&q)[kBowK] = kk[c];
#pragma unroll
        for (int t = 0; t < kBowK; ++t) q[t] = q[t] == 0xffffffffu ? q[t] : q[t] + 4u * (uint32_t)h;
        uint32_t other[kBowK];
#pragma unroll
        for (int t = 0; t < kBowK; ++t) other[t] = (uint32_t)__shfl_xor((int)q[t], 32, kWave);
#pragma unroll
        for (int t = 0; t < kBowK; ++t) topk_push(q, other[t]);
        if (h == 0) {
            bowk_list o;
#pragma unroll
            for (int t = 0; t < kBowK; ++t) o[t] = q[t];
            k.lists[slot0 + 32 * c + col] = o;
        }
    }
}

// One thread per g, the g entries ordered by frame node (neighbouring lanes
// walk nodes of one size: little divergence).  The positions of the node
// claimed so far in this walk are bits of a thread-private LDS bitmap (17
// words a thread: the odd pitch spreads the threads over the banks); nodes of
// more than 512 features read "taken" from the match row instead (only this
// thread writes the node's entries of it).
// The walk's memory traffic is kept off its critical path: a thread's slots
// and lists are read 8 steps at a time, the frame-feature indices of the
// block's first node come from an LDS copy, and every step issues exactly one
// store (a claim to `match`, otherwise to a scratch word).
constexpr int kBowFidxStage = 1024;
// Exact rescans (a list that cannot decide) are done by the whole wave: the
// walk runs in wave-uniform steps (the wave's longest walk), and at each step
// the lanes needing a rescan are served one after the other with the node's
// features spread over the 64 lanes (the rescanning lane's claimed positions
// read from its LDS bitmap, or its match row for large nodes), instead of a
// serial loop over the whole node by the one lane while the wave waits.
// BIG = false: 256-thread blocks, nodes of <= 512 features (17 words of LDS
// bitmap a thread); with big_pitch > 0 the larger nodes are left to the BIG
// form (one wave a block, a bitmap of big_pitch words a thread covering every
// frame position), whose few long walks set the kernel's tail: their "taken"
// checks then cost an LDS read, not two dependent global loads into the
// match row.  big_pitch = 0: the 256-thread form takes every node (match-row
// checks above 512 features).
template <bool BIG, bool ALL_LDS>
__global__ __launch_bounds__(256) void k_bowk_resolve_lane(BowKArgs k, int big_pitch) {
    extern __shared__ uint32_t taken_dyn[];                        // BIG: blockDim x big_pitch words
    __shared__ uint32_t taken_st[BIG ? 1 : 256 * kBowLanePitch];
    __shared__ uint16_t s_fidx[BIG ? 1 : kBowFidxStage];
    const BowArgs& a = k.b;
    if (BIG && k.node_n[a.f_nnodes] == 0) return;                  // no node for this form
    const int ntot = k.gstart[a.f_nnodes];
    const int tb = blockIdx.x * blockDim.x;
    if (tb >= ntot) return;                                        // the whole block
    const int fl0 = k.g_fl[k.perm[tb]];
    const int fb0 = a.f_off[fl0], nf0 = a.f_off[fl0 + 1] - fb0;
    const bool st0 = !BIG && nf0 <= kBowFidxStage;
    if (st0)
        for (int p = threadIdx.x; p < nf0; p += blockDim.x) s_fidx[p] = (uint16_t)a.f_idx[fb0 + p];
    __syncthreads();
    const int t = tb + threadIdx.x;
    const int lane = lane_id();
    if (tb + (int)threadIdx.x - lane >= ntot) return;              // the whole wave
    const int kSmall = 32 * kBowLaneWords;
    const int pitch = BIG ? big_pitch : kBowLanePitch;
    bool have = t < ntot;
    long long base = 0, kpo = 0;
    int fb = 0, nf = 0, nkf = 0, pr = 0, fl = -1;
    if (have) {
        const int flt = k.g_fl[k.perm[t]];
        const int nft = a.f_off[flt + 1] - a.f_off[flt];
        have = BIG ? nft > kSmall : (big_pitch == 0 || nft <= kSmall);
    }
    if (BIG && !__ballot(have)) return;                            // the whole wave
    if (have) {
        const long long g = k.perm[t];
        fl = k.g_fl[g];
        pr = k.g_pr[g];
        const int ia = (int)(g - a.node_off[pr]);
        const int* ko = a.kf_off + a.node_off[pr] + pr;
        base = (long long)k.bstart[fl] + k.g_off[g];
        fb = a.f_off[fl];
        nf = a.f_off[fl + 1] - fb;
        kpo = a.kp_off[pr];
        nkf = ko[ia + 1] - ko[ia];
    }
    const bool complete = nf <= kBowK, lds_bits = BIG || nf <= kSmall;
    const bool lds_fidx = have && st0 && fl == fl0;
    int32_t* match = a.match + (long long)pr * a.f_n;
    const uint32_t* fidx = a.f_idx + fb;
    int32_t* sink;                                                 // scratch (g_rank is k_bowk_fill's)
    uint32_t* const taken_s = BIG ? taken_dyn : taken_st;
    uint32_t* taken = taken_s + threadIdx.x * pitch;
    if (BIG) {
        if (have)
            for (int i = 0; i < (nf + 31) / 32; ++i) taken[i] = 0;
    } else {
#pragma unroll
        for (int i = 0; i < kBowLaneWords; ++i) taken[i] = 0;
    }
    const int nkf_max = -wave_min(-nkf, 0);
    // wave-uniform: every lane's frame indices come from the block's LDS copy
    const bool wave_lds_fidx = __ballot(have && !lds_fidx) == 0;
    // the walk is branch-free per lane (selects, not exec-mask round trips
    // between the vector and the scalar unit, which stalled its issue ~58 % of
    // the time): the taken checks read the bitmap at clamped positions, the
    // bitmap update and the claim store run for every lane with a neutral
    // value, and the only branch per step is the wave's rescan test
    constexpr bool all_lds = BIG || ALL_LDS;                       // every lane's bitmap in LDS (big_pitch > 0)
    const int nfc = max(nf, 1) - 1;
    sink = k.g_rank + min(t, ntot - 1);
    int nm = 0;
    // a thread's slots are contiguous: its walk reads them kChunk at a time
    // (kChunk lists = one 128-B line), not one 16-B piece of a line per step,
    // which refetched every line ~8 times from HBM once the 64 streams of a
    // wave no longer fit the cache between steps
#ifndef ORB_BOWK_RES_CHUNK
#define ORB_BOWK_RES_CHUNK 8
#endif
    constexpr int kChunk = ORB_BOWK_RES_CHUNK;
    const int nkc = max(nkf, 1) - 1;
    static_assert(kChunk == 8, "a chunk is one aligned 8-slot run");
    for (int j0 = 0; j0 < nkf_max; j0 += kChunk) {
        uint32_t sv[kChunk];
        bowk_list Lv[kChunk];
        uint32_t cw[kChunk / 2] = {0u, 0u, 0u, 0u};   // the chunk's claims, u16 each
        {
            // inside the lane's own run (past its end: its last chunk again, unused)
            const int jb = min(j0, nkc & ~7);
            const uint4 s0 = *(const uint4*)(k.slot_src + base + jb), s1 = *(const uint4*)(k.slot_src + base + jb + 4);
            sv[0] = s0.x; sv[1] = s0.y; sv[2] = s0.z; sv[3] = s0.w; sv[4] = s1.x; sv[5] = s1.y; sv[6] = s1.z; sv[7] = s1.w;
#pragma unroll
            for (int c = 0; c < kChunk; ++c) Lv[c] = k.lists[base + jb + c];
        }
#pragma unroll
        for (int c = 0; c < kChunk; ++c) {
            const bool act = j0 + c < nkf;
            const uint32_t s = act ? sv[c] : 0xffffffffu;
            const bowk_list L = Lv[c];
            const bool valid = s != 0xffffffffu;                         // a valid MapPoint (:255-260)
            uint32_t keys[kBowK];
#pragma unroll
            for (int q = 0; q < kBowK; ++q) keys[q] = L[q];
            uint32_t e1 = 0xffffffffu, e2 = 0xffffffffu;
            bool tk[kBowK];
            if constexpr (all_lds) {
#pragma unroll
                for (int q = 0; q < kBowK; ++q) {
                    const int f = min((int)(keys[q] & 0xffff), nfc);
                    tk[q] = (taken[f >> 5] >> (f & 31)) & 1u;
                }
            } else {
#pragma unroll
                for (int q = 0; q < kBowK; ++q) {
                    const int f = min((int)(keys[q] & 0xffff), nfc);
                    tk[q] = lds_bits ? ((taken[f >> 5] >> (f & 31)) & 1u) : (have && match[fidx[f]] >= 0);
                }
            }
#pragma unroll
            for (int q = kBowK - 1; q >= 0; --q) {                       // first two untaken keys (:275-276)
                const bool u = keys[q] != 0xffffffffu && !tk[q];
                e2 = u ? e1 : e2;
                e1 = u ? keys[q] : e1;
            }
            const int dlast = (int)(keys[kBowK - 1] >> 16);
            const bool h1 = e1 != 0xffffffffu, h2 = e2 != 0xffffffffu;
            int best = h1 ? (int)(e1 >> 16) : 256;
            int bpos = h1 ? (int)(e1 & 0xffff) : 0;
            // with one untaken key, dlast bounds the second from below: decided
            // when even dlast passes the ratio test
            const bool bound_ok = a.ratio > 0.f && (float)best < a.ratio * (float)dlast;
            int best2 = h2 ? (int)(e2 >> 16) : ((h1 && !complete && best <= kThLow && bound_ok) ? dlast : 256);
            const bool exact = complete || (h1 ? (h2 || best > kThLow || bound_ok) : dlast > kThLow);
            // the reference's node loop (:266-292) for each lane that needs it,
            // the node's features over the wave's lanes
            uint64_t need = __ballot(valid && !exact);
            while (need) {
                const int i = __builtin_ctzll(need);
                need &= need - 1;
                const uint32_t si = (uint32_t)__builtin_amdgcn_readlane((int)s, i);
                const int nfi = __builtin_amdgcn_readlane(nf, i), fbi = __builtin_amdgcn_readlane(fb, i);
                const int pri = __builtin_amdgcn_readlane(pr, i);
                const uint32_t* tki = taken_s + (threadIdx.x - lane + i) * pitch;
                const int32_t* mi = a.match + (long long)pri * a.f_n;
                const bool lbi = BIG || nfi <= kSmall;
                const uint8_t* kd = a.kf_desc + (long long)si * 32;
                const uint4 q0 = *(const uint4*)kd, q1 = *(const uint4*)(kd + 16);
                uint32_t m1 = (uint32_t)INT_MAX, m2 = (uint32_t)INT_MAX;   // wave_min works on ints
                for (int f = lane; f < nfi; f += kWave) {
                    const uint32_t fi = a.f_idx[fbi + f];
                    if (lbi ? ((tki[f >> 5] >> (f & 31)) & 1u) : mi[fi] >= 0) continue;
                    const uint32_t key = ((uint32_t)hamming32(q0, q1, a.f_desc + (long long)fi * 32) << 16) | (uint32_t)f;
                    m2 = min(m2, max(m1, key));
                    m1 = min(m1, key);
                }
                // first and second minima over the lanes (keys < 2^25: positive ints)
                const int a1 = wave_min((int)m1, INT_MAX);
                const int own = (m1 == (uint32_t)a1) ? (int)m2 : (int)m1;
                const int a2 = wave_min(own, INT_MAX);
                if (lane == i) {
                    best = a1 == INT_MAX ? 256 : (a1 >> 16);
                    best2 = a2 == INT_MAX ? 256 : (a2 >> 16);
                    bpos = a1 == INT_MAX ? 0 : (a1 & 0xffff);
                }
            }
            const bool claim = valid && best <= kThLow && (float)best < a.ratio * (float)best2;   // :327-329
            bpos = min(bpos, nfc);
            uint32_t fi;
            if (wave_lds_fidx) fi = s_fidx[min(bpos, kBowFidxStage - 1)];
            else fi = lds_fidx ? s_fidx[min(bpos, kBowFidxStage - 1)] : fidx[claim ? bpos : 0];
            if (k.claim) {
                // the claim beside the slot, stored 8 at a time below
                cw[c >> 1] |= (claim ? fi : 0xffffu) << (16 * (c & 1));
            } else {
                int32_t* dst = claim ? match + fi : sink;
                *dst = claim ? (int32_t)((long long)s - kpo) : 0;
            }
            if constexpr (all_lds) {
                taken[bpos >> 5] |= (claim ? 1u : 0u) << (bpos & 31);
            } else if (claim && lds_bits) {
                taken[bpos >> 5] |= 1u << (bpos & 31);
            }
            nm += claim;
        }
        // one aligned 16-B store per lane per chunk: a store of 64 lanes' claims
        // touches 64 lines, and one per step (or a scattered 4-B store into the
        // match rows) cost the walk ~0.9 ms of its ~1.6 on the C5 map
        if (k.claim && j0 < nkf) *(uint4*)(k.claim + base + j0) = make_uint4(cw[0], cw[1], cw[2], cw[3]);
    }
    if (nm && !k.claim) atomicAdd(&a.nmatches[pr], nm);
}

// The match rows from the resolve's claims, with the rotation filter
// (:404-422) and the counts: one block per pair, its row and the match bins
// in LDS.  Like k_bowk_fill, every thread takes the pair's KF features in
// FeatureVector order (contiguous), each one's run base found by a search of
// the node offsets staged in LDS, four features' loads in flight per thread;
// the keyframe angles come from the map's FeatureVector-order copy
// (contiguous too) when it has one; the row is written once, coalesced.
constexpr int kBowkRow = 8192;          // frame features of the LDS row (the all-LDS resolve's bound)
constexpr int kBowkFinalStage = 256;    // KF nodes whose run bases are staged in LDS
#ifndef ORB_BOWKF_U
#define ORB_BOWKF_U 4
#endif
__global__ __launch_bounds__(256) void k_bowk_final(BowKArgs k) {
    extern __shared__ int s_row[];                       // [f_n] KF feature | rotation bin << 26, or -1
    __shared__ int s_ko[kBowkFinalStage + 1];
    __shared__ int s_base[kBowkFinalStage];
    __shared__ int hist[32];
    __shared__ int s_cnt;
    const BowArgs& a = k.b;
    const int pr = blockIdx.x, tid = threadIdx.x, nt = blockDim.x, lane = lane_id();
    for (int i = tid; i < a.f_n; i += nt) s_row[i] = -1;
    if (tid < 32) hist[tid] = 0;
    if (tid == 0) s_cnt = 0;
    const long long g0 = a.node_off[pr];
    const int nn = (int)(a.node_off[pr + 1] - g0);
    const int* ko = a.kf_off + g0 + pr;
    const long long io = a.idx_off[pr], kpo = a.kp_off[pr];
    const uint32_t* ki = a.kf_idx + io;
    auto run_base = [&](int ia) -> int {              // slot of the node's feature p: base + p; -1: no frame node
        const int fl = k.g_fl[g0 + ia];
        return fl < 0 ? -1 : k.bstart[fl] + k.g_off[g0 + ia] - ko[ia];
    };
    // claim c (0xffff: none) of KF feature row p; the bins counted per wave by
    // bin value (a keyframe's matches share one or two bins: one LDS atomic per
    // distinct bin, not 64 serialised same-address atomics)
    auto take = [&](int c, int p) {
        int b = -1;
        if (c != 0xffff) {
            const int ikf = (int)ki[p];
            if (a.check_ori) {
                const float ka = a.kf_fvangle ? a.kf_fvangle[io + p] : a.kf_kps[kpo + ikf].angle;
                b = rot_bin(ka, a.f_kps[c].angle);
            }
            s_row[c] = ikf | (max(b, 0) << 26);
        }
        hist_add_wave(hist, b);
    };
    const bool staged = nn <= kBowkFinalStage;
    if (staged)
        for (int ia = tid; ia <= nn; ia += nt) {
            s_ko[ia] = ko[ia];
            if (ia < nn) s_base[ia] = run_base(ia);
        }
    __syncthreads();
    if (staged) {
        // every thread over the pair's KF features in FeatureVector order (as
        // k_bowk_fill), ORB_BOWKF_U claims in flight per thread
        const int p0 = s_ko[0], p1 = s_ko[nn];
        constexpr int kU = ORB_BOWKF_U;
        for (int q = p0 + tid; q < p1; q += kU * nt) {
            // every load of the four rows that does not need a claim first, then
            // the frame angles of the claimed ones: two dependent rounds
            int cs[kU], ik[kU];
            float ka[kU], fa[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int p = q + u * nt;
                int lo = 0, hi = nn;                     // last ia with s_ko[ia] <= p
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (s_ko[mid] <= p) lo = mid;
                    else hi = mid;
                }
                const int b = p < p1 ? s_base[lo] : -1;
                const int pc = min(p, p1 - 1);
                cs[u] = b >= 0 ? (int)k.claim[b + p] : 0xffff;
                ik[u] = (int)ki[pc];
                ka[u] = a.kf_fvangle ? a.kf_fvangle[io + pc] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                fa[u] = 0.f;
                if (a.check_ori && cs[u] != 0xffff) {
                    fa[u] = a.f_kps[cs[u]].angle;
                    if (!a.kf_fvangle) ka[u] = a.kf_kps[kpo + ik[u]].angle;
                }
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                int b = -1;
                if (cs[u] != 0xffff) {
                    if (a.check_ori) b = rot_bin(ka[u], fa[u]);
                    s_row[cs[u]] = ik[u] | (max(b, 0) << 26);
                }
                hist_add_wave(hist, b);
            }
        }
    } else {
        for (int ia = wave_id(); ia < nn; ia += nt / kWave) {   // a wave per KF node
            const int b = run_base(ia);
            if (b < 0) continue;
            for (int p = ko[ia] + lane; p < ko[ia + 1]; p += kWave) take(k.claim[b + p], p);
        }
    }
    __syncthreads();
    int i1 = -1, i2 = -1, i3 = -1;
    if (a.check_ori) three_maxima_wave(hist, i1, i2, i3);
    int32_t* match = a.match + (long long)pr * a.f_n;
    int cnt = 0;
    for (int i = tid; i < a.f_n; i += nt) {
        const int e = s_row[i];
        int m = e < 0 ? -1 : (e & 0x3ffffff);
        if (m >= 0 && a.check_ori) {
            const int b = e >> 26;
            if (b != i1 && b != i2 && b != i3) m = -1;
        }
        cnt += m >= 0;
        match[i] = m;
    }
    cnt = wave_sum(cnt);
    if (lane == 0 && cnt) atomicAdd(&s_cnt, cnt);
    __syncthreads();
    if (tid == 0) a.nmatches[pr] = s_cnt;
}

// ---------------------------------------------------------------------------
// k_proj: the projection searches with a serial claim on the target's slots,
// one wave per target, queries in reference order, the candidates of a query
// spread over the lanes (cell-start runs, in GetFeaturesInArea order).
//   mode 0  SearchByProjection(Frame&, vector<MapPoint*>) (ORBmatcher.cc:43-213),
//           best + second best with their levels, F.Nleft == -1.
//   mode 1  "best only" searches (strict `dist < bestDist` from 256, accept
//           bestDist <= accept):
//     SearchByProjection(Frame&, const Frame&) (:1676-1887): win 0/1/2,
//       skip a slot whose MapPoint has observations, mvuRight gate, TH_HIGH,
//       rotation filter;
//     SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist)
//       (:1889-2010): win 0 (levels pl-1 .. pl+1), skip any occupied slot,
//       ORBdist, rotation filter;
//     SearchByProjection(KeyFrame*, Sim3, vpPoints, vpMatched, th,
//       ratioHamming) and its vpPointsKFs twin (:427-646): win 3 (levels
//       pl-1 .. pl, :509), skip any matched slot, TH_LOW * ratioHamming.
// ---------------------------------------------------------------------------
struct ProjArgs {
    int mode;                 // 0 = map points, 1 = best-only searches
    const orb_keypoint* kps; const uint8_t* desc; int n; const float* u_right; const float* scale;
    const uint32_t* gsorted; const int* gcount; const int* cellstart;
    GridParams g;
    int nq;
    const float* qx; const float* qy; const float* qxr;
    const int32_t* qlevel; const float* qviewcos; const float* qdepth;
    const uint8_t* qvalid; const uint8_t* qhas_obs; const uint8_t* qdesc; const float* qangle;
    float th, th_far, ratio;
    int far_points, last_mode, check_ori;
    int skip_any;             // any occupied slot is skipped (vpMatched[idx] / mvpMapPoints[i2] != NULL)
    float accept;             // mode 1: bestDist <= accept
    int32_t* owner; const uint8_t* blocked;
    int32_t* nmatches;
};

// The query's search window: radius, level range and cell range; false = no
// candidate list (invalid, far point, or an empty cell range).
struct ProjQuery { float x, y, r; int minL, maxL; CellRange cr; };

__device__ __forceinline__ bool proj_query(const ProjArgs& a, int i, ProjQuery& q) {
    if (!a.qvalid[i]) return false;
    q.x = a.qx[i]; q.y = a.qy[i];
    if (a.mode == 0) {
        if (a.far_points && a.qdepth[i] > a.th_far) return false;
        const int lvl = a.qlevel[i];
        float r = a.qviewcos[i] > 0.998f ? 2.5f : 4.0f;      // RadiusByViewingCos
        if (a.th != 1.0f) r *= a.th;
        q.r = r * a.scale[lvl];
        q.minL = lvl - 1; q.maxL = lvl;
    } else {
        const int oct = a.qlevel[i];
        q.r = a.th * a.scale[oct];
        if (a.last_mode == 1) { q.minL = oct; q.maxL = -1; }
        else if (a.last_mode == 2) { q.minL = 0; q.maxL = oct; }
        else if (a.last_mode == 3) { q.minL = oct - 1; q.maxL = oct; }
        else { q.minL = oct - 1; q.maxL = oct + 1; }
    }
    return cell_range(q.x, q.y, q.r, a.g, q.cr);
}

// Static candidate test (window, level range, stereo gate) of feature fi.
__device__ __forceinline__ bool proj_static(const ProjArgs& a, int i, const ProjQuery& q, int fi, int& lv) {
    const orb_keypoint k = a.kps[fi];
    lv = k.octave;
    if ((q.minL > 0) || (q.maxL >= 0)) {
        if (k.octave < q.minL) return false;
        if (q.maxL >= 0 && k.octave > q.maxL) return false;
    }
    if (!(fabsf(k.x - q.x) < q.r && fabsf(k.y - q.y) < q.r)) return false;
    if (a.u_right && a.u_right[fi] > 0 && fabsf(a.qxr[i] - a.u_right[fi]) > q.r) return false;
    return true;
}

// The slot holds a MapPoint the search must skip (:88-90, :1747-1749, :504, :1952).
__device__ __forceinline__ bool proj_blocked(const ProjArgs& a, const int* owner, int fi) {
    const int o = owner[fi];
    if (o == -1) return false;
    if (a.skip_any) return true;
    return o <= -2 ? a.blocked[fi] != 0 : a.qhas_obs[o] != 0;
}

// Exact scan of query i's whole candidate list under the current slot state.
__device__ Best2 proj_scan(const ProjArgs& a, int i, const ProjQuery& q, const int* cs, const int* owner) {
    const uint4 q0 = *(const uint4*)(a.qdesc + (long long)i * 32);
    const uint4 q1 = *(const uint4*)(a.qdesc + (long long)i * 32 + 16);
    const AreaRuns ar = area_runs(cs, q.cr);
    Best2 st{256, 256, -1, -1, -1};
    for (int base = 0; base < ar.total; base += kWave) {
        const int t = base + lane_id();
        const int j = area_pos(ar, min(t, ar.total - 1));
        int d = INT_MAX, fi = -1, lv = -1;
        if (t < ar.total) {
            fi = (int)(a.gsorted[j] & 0xffff);
            if (proj_static(a, i, q, fi, lv) && !proj_blocked(a, owner, fi))
                d = hamming32(q0, q1, a.desc + (long long)fi * 32);
        }
        merge_chunk(st, d, fi, lv);
    }
    return st;
}

// Acceptance (mode 0: :123-139; mode 1: :1770, :1966, :523).
__device__ __forceinline__ bool proj_accept(const ProjArgs& a, const Best2& st) {
    if (a.mode == 0) return st.best <= kThHigh && !(st.lvl == st.lvl2 && (float)st.best > a.ratio * (float)st.best2);
    return st.idx >= 0 && (float)st.best <= a.accept;
}

__device__ __forceinline__ void proj_claim(const ProjArgs& a, const Best2& st, int i, int* owner, int* hist, int* hent,
                                           int& nm, int& nh) {
    if (lane_id() == 0) owner[st.idx] = i;
    ++nm;
    if (a.mode == 1 && a.check_ori) {
        const int bn = rot_bin(a.qangle[i], a.kps[st.idx].angle);
        if (lane_id() == 0) { hist[bn]++; hent[nh] = (bn << 16) | st.idx; }
        ++nh;
    }
}

// Rotation filter of the mode-1 searches: entries in push order; every entry
// in a rejected bin clears its slot and decrements (:1864-1884, :1988-2007).
__device__ __forceinline__ void proj_rot_filter(const ProjArgs& a, const int* hist, const int* hent, int nh,
                                                int* owner, int& nm) {
    int i1, i2, i3;
    three_maxima_wave(hist, i1, i2, i3);
    __syncthreads();
    int drop = 0;
    for (int e = lane_id(); e < nh; e += kWave) {
        const int bn = hent[e] >> 16;
        if (bn == i1 || bn == i2 || bn == i3) continue;
        owner[hent[e] & 0xffff] = -1;
        ++drop;
    }
    nm -= wave_sum(drop);
}

// Single-wave form (slot state in global memory): the fallback when the slot
// table or the query list does not fit in LDS.
__global__ __launch_bounds__(64) void k_proj(ProjArgs a) {
    extern __shared__ __attribute__((aligned(16))) int lds[];
    const int lane = lane_id();
    int* hist = lds;                          // 32
    int* cs = lds + 32;                       // kCells + 1: cell-start table
    int* hent = cs + kCells + 1;              // rotation histogram entries in push order: (bin << 16) | slot
    for (int i = lane; i < 32; i += kWave) hist[i] = 0;
    for (int i = lane; i <= kCells; i += kWave) cs[i] = a.cellstart[i];
    __syncthreads();
    int nm = 0, nh = 0;
    for (int i = 0; i < a.nq; ++i) {
        ProjQuery q;
        if (!proj_query(a, i, q)) continue;
        const Best2 st = proj_scan(a, i, q, cs, a.owner);
        if (proj_accept(a, st)) proj_claim(a, st, i, a.owner, hist, hent, nm, nh);
        __syncthreads();
    }
    if (a.mode == 1 && a.check_ori) proj_rot_filter(a, hist, hent, nh, a.owner, nm);
    if (lane == 0) a.nmatches[0] = nm;
}

static size_t proj_lds(int nq) { return (size_t)(32 + kCells + 1 + nq + 1) * 4 + 64; }

// ---- fisheye stereo frames (Frame::Nleft != -1) ---------------------------
// Slots [0, nleft) are the left keypoints (mvKeys), [nleft, n) the right ones
// (mvKeysRight); each camera has its own grid order and cell-start table, the
// right one by local index (Frame.cc:385-416).  One wave, queries in order, the
// left search then the right one per query (ORBmatcher.cc:61-210 / :1695-1859).
struct FishArgs {
    int nleft;
    const uint32_t *gs_l, *gs_r;
    const int *cs_l, *cs_r;
    const int32_t *l2r, *r2l;                      // mvLeftToRightMatch / mvRightToLeftMatch (mode 0)
    const uint8_t* rvalid;                         // mode 0: mbTrackInViewR && !isBad()
    const float *rqx, *rqy;                        // right-camera projections
    const int32_t* rlevel;                         // mode 0: mnTrackScaleLevelR
    const float* rviewcos;                         // mode 0: mTrackViewCosR
};

// Exact scan of one camera's candidate list (grid order gs / cell starts cs,
// slot = local index + off); *nstatic = the GetFeaturesInArea list length.
__device__ Best2 proj_scan_cam(const ProjArgs& a, int i, const ProjQuery& q, const uint32_t* gs, const int* cs,
                               int off, int& nstatic) {
    const uint4 q0 = *(const uint4*)(a.qdesc + (long long)i * 32);
    const uint4 q1 = *(const uint4*)(a.qdesc + (long long)i * 32 + 16);
    const AreaRuns ar = area_runs(cs, q.cr);
    Best2 st{256, 256, -1, -1, -1};
    int ns = 0;
    for (int base = 0; base < ar.total; base += kWave) {
        const int t = base + lane_id();
        const int j = area_pos(ar, min(t, ar.total - 1));
        int d = INT_MAX, fi = -1, lv = -1;
        bool stat = false;
        if (t < ar.total) {
            fi = (int)(gs[j] & 0xffff) + off;
            stat = proj_static(a, i, q, fi, lv);
            if (stat && !proj_blocked(a, a.owner, fi)) d = hamming32(q0, q1, a.desc + (long long)fi * 32);
        }
        ns += __popcll(__ballot(stat));
        merge_chunk(st, d, fi, lv);
    }
    nstatic = ns;
    return st;
}

__device__ __forceinline__ void proj_window(const ProjArgs& a, int oct, ProjQuery& q) {
    if (a.last_mode == 1) { q.minL = oct; q.maxL = -1; }
    else if (a.last_mode == 2) { q.minL = 0; q.maxL = oct; }
    else { q.minL = oct - 1; q.maxL = oct + 1; }
}

__global__ __launch_bounds__(64) void k_proj_fisheye(ProjArgs a, FishArgs fa) {
    extern __shared__ __attribute__((aligned(16))) int lds[];
    const int lane = lane_id();
    int* hist = lds;                          // 32
    int* hent = lds + 32;                     // 2 nq: (bin << 16) | slot in push order
    for (int k = lane; k < 32; k += kWave) hist[k] = 0;
    __syncthreads();
    int nm = 0, nh = 0;
    auto ori_push = [&](int i, int slot) {
        const int bn = rot_bin(a.qangle[i], a.kps[slot].angle);
        if (lane == 0) { hist[bn]++; hent[nh] = (bn << 16) | slot; }
        ++nh;
    };
    auto set_owner = [&](int slot, int i) { if (lane == 0) a.owner[slot] = i; };
    for (int i = 0; i < a.nq; ++i) {
        const bool lv = a.qvalid[i] != 0;
        const bool rv = a.mode == 0 ? fa.rvalid[i] != 0 : lv;
        if (!lv && !rv) continue;
        if (a.mode == 0 && a.far_points && a.qdepth[i] > a.th_far) continue;
        bool go_right = true;
        if (lv) {
            ProjQuery q;
            q.x = a.qx[i]; q.y = a.qy[i];
            const int lvl = a.qlevel[i];
            if (a.mode == 0) {
                float r = a.qviewcos[i] > 0.998f ? 2.5f : 4.0f;
                if (a.th != 1.0f) r *= a.th;
                q.r = r * a.scale[lvl];
                q.minL = lvl - 1; q.maxL = lvl;
            } else {
                q.r = a.th * a.scale[lvl];
                proj_window(a, lvl, q);
            }
            int ns = 0;
            Best2 st{256, 256, -1, -1, -1};
            if (cell_range(q.x, q.y, q.r, a.g, q.cr)) st = proj_scan_cam(a, i, q, fa.gs_l, fa.cs_l, 0, ns);
            if (a.mode == 0) {
                if (ns > 0 && st.best <= kThHigh) {                                   // :123-139
                    if (st.lvl == st.lvl2 && (float)st.best > a.ratio * (float)st.best2) {
                        go_right = false;                                             // `continue` (:126)
                    } else {
                        set_owner(st.idx, i);
                        if (fa.l2r[st.idx] != -1) { set_owner(fa.l2r[st.idx] + fa.nleft, i); ++nm; }
                        ++nm;
                    }
                }
            } else {
                if (ns == 0) go_right = false;                                        // :1735-1736
                else if (st.best <= kThHigh) {                                        // :1770-1792
                    set_owner(st.idx, i);
                    ++nm;
                    if (a.check_ori) ori_push(i, st.idx);
                }
            }
            __syncthreads();
        }
        if (!go_right || !rv) continue;
        ProjQuery q;
        q.x = fa.rqx[i]; q.y = fa.rqy[i];
        if (a.mode == 0) {                                                            // :144-150
            const int lvl = fa.rlevel[i];
            if (lvl == -1) continue;
            q.r = (fa.rviewcos[i] > 0.998f ? 2.5f : 4.0f) * a.scale[lvl];
            q.minL = lvl - 1; q.maxL = lvl;
        } else {                                                                      // :1798-1811
            const int oct = a.qlevel[i];
            q.r = a.th * a.scale[oct];
            proj_window(a, oct, q);
        }
        if (!cell_range(q.x, q.y, q.r, a.g, q.cr)) continue;
        int ns = 0;
        const Best2 st = proj_scan_cam(a, i, q, fa.gs_r, fa.cs_r, fa.nleft, ns);
        if (st.best > kThHigh) continue;
        if (a.mode == 0) {                                                            // :193-208
            if (st.lvl == st.lvl2 && (float)st.best > a.ratio * (float)st.best2) continue;
            const int partner = fa.r2l[st.idx - fa.nleft];
            if (partner != -1) { set_owner(partner, i); ++nm; }
            set_owner(st.idx, i);
            ++nm;
        } else {                                                                      // :1836-1857
            set_owner(st.idx, i);
            ++nm;
            if (a.check_ori) ori_push(i, st.idx);
        }
        __syncthreads();
    }
    if (a.mode == 1 && a.check_ori) proj_rot_filter(a, hist, hent, nh, a.owner, nm);
    if (lane == 0) a.nmatches[0] = nm;
}

// ---- two-phase form ------------------------------------------------------
// Phase 1 (k_proj_topk, every query in parallel, one wave each): the static
// candidates whose distance can still decide the outcome (d <= bound: mode 1
// bestDist <= accept; mode 0 the best <= TH_HIGH, and a second best only
// while ratio * d < TH_HIGH can fail the ratio test), and the kProjK smallest
// of them in (distance, candidate order), packed
//   x = d << 24 | level << 16 | slot,  y = rotation bin of (query, slot);
// cnt = how many there are (-1: no list).  Phase 2 (k_proj_resolve, one
// wave): queries in reference order against the slot state in LDS; the first
// (and second) unblocked entries of the list ARE the reference's best (and
// second best) because every unlisted candidate sorts after them; when a
// truncated list runs dry the wave rescans the query exactly.
constexpr int kProjK = 8;

__global__ __launch_bounds__(256) void k_proj_topk(ProjArgs a, int bound, uint2* __restrict__ topk,
                                                   int* __restrict__ cnt) {
    const int i = blockIdx.x * 4 + wave_id(), lane = lane_id();
    if (i >= a.nq) return;
    ProjQuery q;
    if (!proj_query(a, i, q)) {
        if (lane == 0) cnt[i] = -1;
        return;
    }
    const uint4 q0 = *(const uint4*)(a.qdesc + (long long)i * 32);
    const uint4 q1 = *(const uint4*)(a.qdesc + (long long)i * 32 + 16);
    const float qang = (a.mode == 1 && a.check_ori) ? a.qangle[i] : 0.0f;
    const AreaRuns ar = area_runs(a.cellstart, q.cr);
    int run = INT_MAX;                        // lanes < kProjK: running list, sort key (d << 16 | order)
    uint32_t run_e = 0xffffffffu;             //                 and its packed entry
    int total = 0;
    for (int base = 0; base < ar.total; base += kWave) {
        const int t = base + lane;
        const int j = area_pos(ar, min(t, ar.total - 1));
        int key = INT_MAX;
        uint32_t ent = 0xffffffffu;
        if (t < ar.total) {
            const int fi = (int)(a.gsorted[j] & 0xffff);
            int lv;
            if (proj_static(a, i, q, fi, lv)) {
                const int d = hamming32(q0, q1, a.desc + (long long)fi * 32);
                if (d <= bound) {
                    key = (d << 16) | t;
                    ent = ((uint32_t)d << 24) | ((uint32_t)(lv & 0xff) << 16) | (uint32_t)fi;
                }
            }
        }
        total += __popcll(__ballot(key != INT_MAX));
        // kProjK smallest of (running list) U (this chunk); keys are distinct
        int prev = -1, nrun = INT_MAX;
        uint32_t nrun_e = 0xffffffffu;
        for (int r = 0; r < kProjK; ++r) {
            const int xa = key > prev ? key : INT_MAX;
            const int xb = (lane < kProjK && run > prev) ? run : INT_MAX;
            const int x = min(xa, xb);
            const uint32_t xe = xa <= xb ? ent : run_e;
            int m = x;
            m = wave_min(m, INT_MAX);
            if (m == INT_MAX) break;
            const int src = __ffsll((long long)__ballot(x == m)) - 1;
            const uint32_t me = (uint32_t)__builtin_amdgcn_readlane((int)xe, src);
            if (lane == r) { nrun = m; nrun_e = me; }
            prev = m;
        }
        run = nrun; run_e = nrun_e;
    }
    if (lane < kProjK) {
        uint32_t bin = 0;
        if (run_e != 0xffffffffu && a.mode == 1 && a.check_ori) bin = (uint32_t)rot_bin(qang, a.kps[run_e & 0xffff].angle);
        topk[(long long)i * kProjK + lane] = make_uint2(run_e, bin);
    }
    if (lane == 0) cnt[i] = total;
}

// LDS layout of k_proj_resolve: hist[32] | own[n] | hent[nq] | bl[n] bytes
// (slot blocked now) | has_obs[nq] bytes.
static size_t proj_resolve_lds(int n, int nq) { return (size_t)(32 + n + nq + 1) * 4 + (size_t)n + nq + 64; }

// Compiler-only ordering between one wave's LDS accesses: DS instructions of a
// wave execute in order, so a later ds_read sees an earlier ds_write.
__device__ __forceinline__ void lds_order() { __asm__ __volatile__("" ::: "memory"); }

constexpr int kResQ = kWave / kProjK;             // queries per lane group load (8)
constexpr int kResBlk = kResQ * 8;                // queries per prefetched block (64)

// The lists of block `blk` (64 queries): lane (grp, k) holds entry k of query
// blk*64 + u*8 + grp in slot u.  Loads are unconditional (in bounds) so the
// whole block is in flight at once.
__device__ __forceinline__ void res_load(const ProjArgs& a, const uint2* topk, const int* cnt, int blk,
                                         uint2 (&E)[8], int (&C)[8], int (&HO)[8]) {
    const int grp = lane_id() / kProjK, k = lane_id() % kProjK;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int qi = min(blk * kResBlk + u * kResQ + grp, a.nq - 1);
        C[u] = cnt[qi];
        E[u] = topk[(long long)qi * kProjK + k];
        HO[u] = a.skip_any ? 1 : a.qhas_obs[qi];
    }
}

__global__ __launch_bounds__(64) void k_proj_resolve(ProjArgs a, const uint2* __restrict__ topk,
                                                     const int* __restrict__ cnt) {
    extern __shared__ __attribute__((aligned(16))) int lds[];
    const int lane = lane_id();
    int* hist = lds;                          // 32 (final filter only; counted in registers)
    int* own = lds + 32;                      // n: slot owner (-1 free, <= -2 pre-existing, >= 0 query)
    int* hent = own + a.n;                    // nq
    uint8_t* bl = (uint8_t*)(hent + a.nq + 1);    // n: slot is skipped by the search now
    uint8_t* hob = bl + a.n;                      // nq
    uint2 EA[8], EB[8];
    int CA[8], CB[8], HA[8], HB[8];
    const int nblk = (a.nq + kResBlk - 1) / kResBlk;
    if (nblk) res_load(a, topk, cnt, 0, EA, CA, HA);     // in flight during the init
#pragma unroll 8
    for (int i = lane; i < a.n; i += kWave) own[i] = a.owner[i];
    if (a.skip_any) {
#pragma unroll 8
        for (int i = lane; i < a.n; i += kWave) bl[i] = own[i] != -1;
    } else {
#pragma unroll 8
        for (int i = lane; i < a.nq; i += kWave) hob[i] = a.qhas_obs[i];
#pragma unroll 8
        for (int i = lane; i < a.n; i += kWave) {
            const int o = own[i];
            bl[i] = o == -1 ? 0 : (o <= -2 ? a.blocked[i] : a.qhas_obs[o]);
        }
    }
    __syncthreads();
    int nm = 0, nh = 0, hcount = 0;           // lane b < 30 counts rotation bin b
    const int grp = lane / kProjK, k = lane % kProjK;
    // the per-query decisions read these scalars only (SGPRs, no argument reloads)
    const int mode = a.mode, skip_any = a.skip_any, ori = a.mode == 1 && a.check_ori, nq = a.nq;
    const float ratio = a.ratio, accept = a.accept;
    auto accept_st = [&](const Best2& st) {
        if (mode == 0) return st.best <= kThHigh && !(st.lvl == st.lvl2 && (float)st.best > ratio * (float)st.best2);
        return st.idx >= 0 && (float)st.best <= accept;
    };
    // Per group of 8 queries (always register slot 0; the slots shift after
    // each group so ONE rolled copy of the body runs: a serial wave must not
    // stream through unrolled code): one LDS read of every listed slot's
    // blocked flag (lane (grp, k) = entry k of query grp), then the queries in
    // order with the group's own claims tracked in registers -- a claim by
    // query i blocks its slot for later queries iff skip_any or has_obs[i].
    for (int blk = 0; blk < nblk; ++blk) {
        if (blk + 1 < nblk) res_load(a, topk, cnt, blk + 1, EB, CB, HB);
#pragma unroll 1
        for (int u = 0; u < 8; ++u) {
            const int base = blk * kResBlk + u * kResQ;
            const int nj = min(kResQ, nq - base);
            const uint2 e0 = EA[0];
            const int c0 = CA[0], h0 = HA[0];
#pragma unroll
            for (int v = 0; v < 7; ++v) { EA[v] = EA[v + 1]; CA[v] = CA[v + 1]; HA[v] = HA[v + 1]; }
            if (nj <= 0) continue;
            const int slot = (int)(e0.x & 0xffff);
            bool avail = k < min(c0, kProjK) && bl[slot] == 0;
            for (int jq = 0; jq < nj; ++jq) {
                const int i = base + jq;
                const int ci = __builtin_amdgcn_readlane(c0, jq * kProjK);
                if (ci <= 0) continue;
                const uint64_t fm = __ballot(grp == jq && avail);
                Best2 st{256, 256, -1, -1, -1};
                int bin = 0;
                bool exact = true;
                if (fm) {
                    const int l1 = __ffsll((long long)fm) - 1;
                    const uint32_t e1 = (uint32_t)__builtin_amdgcn_readlane((int)e0.x, l1);
                    bin = __builtin_amdgcn_readlane((int)e0.y, l1);
                    st.best = (int)(e1 >> 24); st.lvl = (int)((e1 >> 16) & 0xff); st.idx = (int)(e1 & 0xffff);
                    const uint64_t fm2 = fm & (fm - 1);
                    if (fm2) {
                        const uint32_t e2 = (uint32_t)__builtin_amdgcn_readlane((int)e0.x, __ffsll((long long)fm2) - 1);
                        st.best2 = (int)(e2 >> 24); st.lvl2 = (int)((e2 >> 16) & 0xff);
                    } else if (mode == 0 && ci > kProjK) {
                        exact = false;
                    }
                } else if (ci > kProjK) {
                    exact = false;
                }
                if (!exact) {                  // a truncated list ran dry: exact rescan
                    ProjQuery q;
                    proj_query(a, i, q);
                    wave_sync_m();
                    st = proj_scan(a, i, q, a.cellstart, own);
                    if (st.idx >= 0 && ori) bin = rot_bin(a.qangle[i], a.kps[st.idx].angle);
                }
                if (accept_st(st)) {
                    const int blocks = skip_any ? 1 : __builtin_amdgcn_readlane(h0, jq * kProjK);
                    if (lane == 0) {
                        own[st.idx] = i;
                        bl[st.idx] = (uint8_t)blocks;
                    }
                    if (blocks) avail = avail && slot != st.idx;
                    ++nm;
                    if (ori) {
                        if (lane == 0) hent[nh] = (bin << 16) | st.idx;
                        hcount += lane == bin;
                        ++nh;
                    }
                    lds_order();
                }
            }
        }
#pragma unroll
        for (int v = 0; v < 8; ++v) { EA[v] = EB[v]; CA[v] = CB[v]; HA[v] = HB[v]; }
    }
    if (a.mode == 1 && a.check_ori) {
        if (lane < 32) hist[lane] = hcount;
        __syncthreads();
        proj_rot_filter(a, hist, hent, nh, own, nm);
    }
    __syncthreads();
    for (int i = lane; i < a.n; i += kWave) a.owner[i] = own[i];
    if (lane == 0) a.nmatches[0] = nm;
}

// Speculative form of phase 2 (the default): one wave, lane = query of a
// 64-query block.  Each round every unresolved lane decides against the slot
// state at the round's start.  A lane's decision is the reference's when no
// earlier lane of the round claims, blocking, a slot on its list (an earlier
// non-blocking claim changes no one's candidates), so the longest prefix of
// lanes without such an overlap commits: overlaps are found with a per-slot
// mark (ds_min of the claiming lane); repeated claims of one slot resolve to
// the last lane through the same table (the later query owns it, as in the
// serial loop).
// The first lane after the prefix starts the next round; if its truncated list
// ran dry the wave rescans it exactly at that point.  Every round commits at
// least its first lane.  Candidate lists of different queries rarely share a
// slot within the decision bound, so a block usually commits in one round.
// LDS: the k_proj_resolve layout + mark[n].
static size_t proj_spec_lds(int n, int nq) { return proj_resolve_lds(n, nq) + (size_t)n * 4 + 16; }

__global__ __launch_bounds__(64) void k_proj_resolve_spec(ProjArgs a, const uint2* __restrict__ topk,
                                                          const int* __restrict__ cnt) {
    extern __shared__ __attribute__((aligned(16))) int lds[];
    const int lane = lane_id();
    int* hist = lds;                          // 32
    int* own = lds + 32;                      // n
    int* hent = own + a.n;                    // nq
    int* mark = hent + a.nq + 1;              // n: first lane of the round claiming the slot (64: none)
    uint8_t* bl = (uint8_t*)(mark + a.n);     // n
    for (int i = lane; i < 32; i += kWave) hist[i] = 0;
#pragma unroll 8
    for (int i = lane; i < a.n; i += kWave) {
        const int o = a.owner[i];
        own[i] = o;
        mark[i] = kWave;
        bl[i] = o == -1 ? 0 : (a.skip_any ? 1 : (o <= -2 ? a.blocked[i] : a.qhas_obs[o]));
    }
    __syncthreads();
    const int mode = a.mode, skip_any = a.skip_any, ori = a.mode == 1 && a.check_ori, nq = a.nq;
    const float ratio = a.ratio, accept = a.accept;
    const uint64_t lt = (1ull << lane) - 1;                                // lanes below this one
    int nm = 0, nh = 0;
    const int nblk = (nq + kWave - 1) / kWave;
    for (int blk = 0; blk < nblk; ++blk) {
        const int i = blk * kWave + lane;
        const bool inq = i < nq;
        const int ci = inq ? cnt[i] : -1;
        uint2 E[kProjK];
#pragma unroll
        for (int k = 0; k < kProjK; ++k) E[k] = inq ? topk[(long long)i * kProjK + k] : make_uint2(0xffffffffu, 0);
        const int hob = skip_any ? 1 : (inq ? a.qhas_obs[i] : 0);
        const int nl = min(ci, kProjK);                                    // listed entries
        bool done = ci <= 0;
        while (__ballot(!done)) {
            // tentative decision under the round's starting state
            Best2 st{256, 256, -1, -1, -1};
            int bin = 0, nav = 0;
#pragma unroll
            for (int k = 0; k < kProjK; ++k) {
                if (k < nl) {
                    const int s = (int)(E[k].x & 0xffff);
                    if (!bl[s]) {
                        if (nav == 0) {
                            st.best = (int)(E[k].x >> 24); st.lvl = (int)((E[k].x >> 16) & 0xff); st.idx = s;
                            bin = (int)E[k].y;
                        } else if (nav == 1) {
                            st.best2 = (int)(E[k].x >> 24); st.lvl2 = (int)((E[k].x >> 16) & 0xff);
                        }
                        ++nav;
                    }
                }
            }
            const bool exact = ci <= kProjK || nav >= 2 || (mode == 1 && nav == 1);
            bool acc;
            if (mode == 0) acc = st.best <= kThHigh && !(st.lvl == st.lvl2 && (float)st.best > ratio * (float)st.best2);
            else acc = st.idx >= 0 && (float)st.best <= accept;
            acc = acc && !done && exact;
            const bool blocking = acc && hob;
            if (blocking) atomicMin(&mark[st.idx], lane);
            lds_order();
            bool conflict = false;
#pragma unroll
            for (int k = 0; k < kProjK; ++k)
                if (k < nl && mark[(int)(E[k].x & 0xffff)] < lane) conflict = true;
            const uint64_t bad = __ballot(!done && (conflict || !exact));
            const int p = bad ? __ffsll((long long)bad) - 1 : kWave;
            lds_order();
            if (blocking) mark[st.idx] = kWave;
            const bool commit = !done && lane < p;
            const bool cl = commit && acc;
            // repeated claims of a slot in the prefix: the last lane (the later
            // query) owns it, as in the serial loop
            if (cl) atomicMin(&mark[st.idx], kWave - 1 - lane);
            lds_order();
            if (cl && mark[st.idx] == kWave - 1 - lane) { own[st.idx] = i; bl[st.idx] = (uint8_t)hob; }
            lds_order();
            if (cl) mark[st.idx] = kWave;
            const uint64_t cm = __ballot(cl);
            if (ori) {
                if (cl) {
                    hent[nh + __popcll(cm & lt)] = (bin << 16) | st.idx;
                    atomicAdd(&hist[bin], 1);
                }
                nh += __popcll(cm);
            }
            nm += __popcll(cm);
            done = done || commit;
            lds_order();
            if (p < kWave) {
                // lane p's list ran dry (or overlapped): with every earlier lane
                // committed, a dry list is rescanned exactly now
                const bool dry = (bad >> p) & 1 && __builtin_amdgcn_readlane((int)(!exact), p);
                if (dry) {
                    const int qi = blk * kWave + p;
                    ProjQuery q;
                    proj_query(a, qi, q);
                    wave_sync_m();
                    const Best2 sx = proj_scan(a, qi, q, a.cellstart, own);
                    bool ax;
                    if (mode == 0) ax = sx.best <= kThHigh && !(sx.lvl == sx.lvl2 && (float)sx.best > ratio * (float)sx.best2);
                    else ax = sx.idx >= 0 && (float)sx.best <= accept;
                    if (ax) {
                        const int hq = __builtin_amdgcn_readlane(hob, p);
                        if (lane == 0) { own[sx.idx] = qi; bl[sx.idx] = (uint8_t)hq; }
                        ++nm;
                        if (ori) {
                            const int bx = rot_bin(a.qangle[qi], a.kps[sx.idx].angle);
                            if (lane == 0) { hent[nh] = (bx << 16) | sx.idx; hist[bx]++; }
                            ++nh;
                        }
                    }
                    if (lane == p) done = true;
                    lds_order();
                }
            }
        }
    }
    if (ori) {
        __syncthreads();
        proj_rot_filter(a, hist, hent, nh, own, nm);
    }
    __syncthreads();
    for (int i = lane; i < a.n; i += kWave) a.owner[i] = own[i];
    if (lane == 0) a.nmatches[0] = nm;
}

// ---- fused single-launch form (the host APIs' default) --------------------
// k_proj_fused: a whole projection search in ONE launch, no grid build.
//
// Phase 1, one wave per query, every query in parallel: its kProjK smallest
// candidates by (distance, GetFeaturesInArea order) from a brute-force pass
// over the frame's keypoints.  A keypoint is in the query's GetFeaturesInArea
// list iff its PosInGrid cell lies in the cell range the window visits and it
// passes the window / level / stereo tests (Frame.cc:661-708 visit the cells
// ix outer, iy inner, and a cell's keypoints in index order), so its list
// position is (cell = gx * 48 + gy, index) -- a 32-bit key d << 24 | cell << 12
// | index for frames of <= 4096 keypoints.  Only candidates that can still
// decide the query are kept (d <= bound, as k_proj_topk); cnt = how many.
//
// Phase 2, in the LAST block to finish phase 1 (a ticket counter): the serial
// claim loop over all queries at once, as a fixpoint.  T[s] = the first query
// that claims slot s blocking (-1: blocked before the search, INT_MAX: never);
// query j's decision reads only whether T[s] < j for its listed slots -- the
// claims of EARLIER queries -- so recomputing every decision from the previous
// round's T leaves the earliest wrong decision right after each round (a
// Jacobi iteration of a recursion well-founded in query order), and two equal
// consecutive rounds are the serial loop's outcome.  A decision its truncated
// list cannot make (fewer unblocked entries than it needs) is made by a wave's
// exact brute-force scan under the round's T.  Then: nmatches = accepted
// decisions, owner[s] = the last query accepted on s (a later claim of a slot
// its earlier claimer left unblocked overwrites it, as the serial loop does),
// and the rotation filter clears the slot of every claim in a rejected bin.
#ifndef ORB_PROJ_TPRE
#define ORB_PROJ_TPRE 1   // phase-2 decisions read their list's claim words up front
#endif
constexpr int kFusedThreads = 1024;
constexpr int kFusedQpt = 8;                        // queries per thread in phase 2 (nq <= 8192)
constexpr int kFusedMaxN = 4096;                    // 12-bit keypoint index in the order key
constexpr int kFusedMaxQ = kFusedThreads * kFusedQpt;
#ifndef ORB_PROJ_WIN
#define ORB_PROJ_WIN 0   // phase-2 fixpoint window of queries (0: every query each round; 1024 measured slower: 13 rounds instead of 6 at ~5.5 k cycles each, phase 2 138 k vs 108 k cycles, profiles/r06/README.md)
#endif
constexpr int kProjWin = ORB_PROJ_WIN;
constexpr uint32_t kFusedNone = 0xffffffffu;

// byte offsets of k_proj_fused's phase-2 tables, every table 16-byte aligned
// (the lists are read as 16-byte words)
struct ProjLds { size_t T, D, dry, hist, misc, pre, Cs, Ls, total; };
__host__ __device__ inline ProjLds proj_lds_layout(int n, int nq, bool lds_lists) {
    auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
    ProjLds o{};
    size_t at = 0;
    o.T = at;    at += al((size_t)n * 4);
    o.D = at;    at += al((size_t)nq * 4);
    o.dry = at;  at += al((size_t)nq * 4);
    o.hist = at; at += 32 * 4;
    o.misc = at; at += 16 * 4;
    o.pre = at;  at += al((size_t)n);
    o.Cs = at;   if (lds_lists) at += al((size_t)nq * 4);
    o.Ls = at;   if (lds_lists) at += (size_t)nq * kProjK * 4;
    o.total = al(at);
    return o;
}
__host__ __device__ inline size_t proj_fused_lds(int n, int nq, bool lds_lists) {
    return proj_lds_layout(n, nq, lds_lists).total;
}

// The frame's grid in each block's LDS (no grid-build launch): gcs[c] = start
// of cell c in gent (c in [0, kCells]), gent = cell << 12 | keypoint index, by
// cell (the order inside a cell is free: a candidate's key carries its list
// position).  oct >= 0 keeps the keypoints of that octave only.  Every thread
// of the block calls it; tmp holds blockDim / 64 + 1 ints.  A query's window
// then enumerates only the keypoints of its cell range instead of the frame.
constexpr int kGridInts = kCells + 1;
__host__ __device__ inline size_t lds_grid_bytes(int n) { return (size_t)(kGridInts + (n > 1 ? n : 1) + 32) * 4; }

__device__ void lds_grid_build(const orb_keypoint* kps, int n, const GridParams& g, int oct, int* gcs,
                               uint32_t* gent, int* tmp) {
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int c = tid; c < kGridInts; c += nt) gcs[c] = 0;
    __syncthreads();
    constexpr int kPer = kFusedMaxN / kFusedThreads;
    int cell[kPer], rank[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        const int i = tid + u * nt;
        cell[u] = -1;
        if (i < n && (oct < 0 || kps[i].octave == oct)) cell[u] = grid_cell(kps[i], g);
        rank[u] = cell[u] >= 0 ? atomicAdd(&gcs[cell[u]], 1) : 0;
    }
    __syncthreads();
    block_excl_scan(gcs, kGridInts, tmp);
#pragma unroll
    for (int u = 0; u < kPer; ++u)
        if (cell[u] >= 0) gent[gcs[cell[u]] + rank[u]] = ((uint32_t)cell[u] << 12) | (uint32_t)(tid + u * nt);
    __syncthreads();
}

// A frame's grid built once (k_grid_prebuild, the dframe searches): the
// cell starts and entries of lds_grid_build, kGridInts + n ints contiguous,
// copied into the block's LDS instead of rebuilt.
__device__ void lds_grid_load(const int* __restrict__ pg, int n, int* gcs) {
    const int tot = kGridInts + max(1, n);
    // in 16-byte pieces when source and LDS share their alignment (one read a
    // thread for a thousand-point frame: one HBM round trip, not four)
    const int hs = (int)((16 - ((uintptr_t)pg & 15)) & 15) >> 2, hd = (int)((16 - ((uintptr_t)gcs & 15)) & 15) >> 2;
    if (hs == hd && ((uintptr_t)pg & 3) == 0) {
        const int body = (tot - hs) >> 2;
        const uint4* src = (const uint4*)(pg + hs);
        uint4* dst = (uint4*)(gcs + hs);
        for (int c = threadIdx.x; c < body; c += blockDim.x) dst[c] = src[c];
        const int t0 = hs + body * 4;
        if ((int)threadIdx.x < hs) gcs[threadIdx.x] = pg[threadIdx.x];
        if ((int)threadIdx.x < tot - t0) gcs[t0 + threadIdx.x] = pg[t0 + threadIdx.x];
    } else {
        for (int c = threadIdx.x; c < tot; c += blockDim.x) gcs[c] = pg[c];
    }
    __syncthreads();
}

__global__ __launch_bounds__(kFusedThreads) void k_grid_prebuild(const orb_keypoint* kps, int n, GridParams g,
                                                                  int oct, int* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) int gl[];
    int* gcs = gl;
    uint32_t* gent = (uint32_t*)(gcs + kGridInts);
    lds_grid_build(kps, n, g, oct, gcs, gent, (int*)(gent + max(1, n)));
    const int tot = kGridInts + max(1, n);
    for (int c = threadIdx.x; c < tot; c += blockDim.x) out[c] = gl[c];
}

// A window's cell columns on the lanes: lane c < ncol holds column cr.x0 + c's
// run [start, start + cnt) of gent and its exclusive offset in the window's
// list; total = the list length (wave-uniform).
struct WinCols { int ncol, total, start, excl; };
__device__ __forceinline__ WinCols win_cols(const int* gcs, const CellRange& cr) {
    WinCols w;
    const int lane = lane_id();
    w.ncol = cr.x1 - cr.x0 + 1;
    int cnt = 0;
    w.start = 0;
    if (lane < w.ncol) {
        const int c0 = (cr.x0 + lane) * kGridRows;
        w.start = gcs[c0 + cr.y0];
        cnt = gcs[c0 + cr.y1 + 1] - w.start;
    }
    const int incl = wave_incl_scan(cnt);
    w.excl = incl - cnt;
    w.total = __builtin_amdgcn_readlane(incl, kWave - 1);
    return w;
}
// the entry at window list position p (< total)
__device__ __forceinline__ uint32_t win_entry(const WinCols& w, const uint32_t* gent, int p) {
    int st = 0, ex = 0;
    for (int c = 0; c < w.ncol; ++c) {
        const int e = __builtin_amdgcn_readlane(w.excl, c);
        if (p >= e) { ex = e; st = __builtin_amdgcn_readlane(w.start, c); }
    }
    return gent[st + p - ex];
}

// The kProjK (or 2 for a rescan) smallest 32-bit keys of query i's candidates
// with d <= bound, skipping (T != nullptr) slots blocked before query j; lane
// r < K holds the r-th key and its packed entry d << 24 | (lvl | bin << 3) << 16
// | slot.  Returns the number of such candidates.
template <int K>
__device__ int fused_select(const ProjArgs& a, int i, const ProjQuery& q, int bound, const int* T, int j,
                            const int* gcs, const uint32_t* gent, uint32_t& run, uint32_t& run_e) {
    const int lane = lane_id();
    const uint4 q0 = *(const uint4*)(a.qdesc + (long long)i * 32);
    const uint4 q1 = *(const uint4*)(a.qdesc + (long long)i * 32 + 16);
    const float qang = (a.mode == 1 && a.check_ori) ? a.qangle[i] : 0.0f;
    run = kFusedNone;
    run_e = kFusedNone;
    int total = 0;
    // x, y, octave of the next chunk's keypoints are in flight while this
    // chunk is tested (the scan is a chain of L2 round trips otherwise)
    const float* kf = (const float*)a.kps;
    const int kw = (int)(sizeof(orb_keypoint) / 4);
    // the list to scan: the window's cells of the LDS grid, or the whole frame
    WinCols w{};
    int len = a.n;
    if (gcs) {
        w = win_cols(gcs, q.cr);
        len = w.total;
    }
    auto kload = [&](int base, int& f, float& x, float& y, int& o) {
        const int p = min(base + lane, max(len - 1, 0));
        f = gcs ? (int)(win_entry(w, gent, p) & 0xfff) : p;
        x = kf[(long long)f * kw + 0];
        y = kf[(long long)f * kw + 1];
        o = ((const int*)kf)[(long long)f * kw + 5];
    };
    float nx = 0.f, ny = 0.f;
    int no = 0, nf = 0;
    if (len > 0) kload(0, nf, nx, ny, no);
    for (int base = 0; base < len; base += kWave) {
        const float kx = nx, ky = ny;
        const int ko = no, fi = nf;
        if (base + kWave < len) kload(base + kWave, nf, nx, ny, no);
        uint32_t key = kFusedNone, ent = kFusedNone;
        if (base + lane < len) {
            // PosInGrid (Frame.cc:725-735) and the cell range the window visits
            const int gx = (int)roundf((kx - a.g.min_x) * a.g.inv_w);
            const int gy = (int)roundf((ky - a.g.min_y) * a.g.inv_h);
            const bool in_cells = gx >= q.cr.x0 && gx <= q.cr.x1 && gy >= q.cr.y0 && gy <= q.cr.y1 &&
                                  gx < kGridCols && gy < kGridRows && gx >= 0 && gy >= 0;
            // proj_static: level range, window, stereo gate
            bool ok = in_cells;
            if ((q.minL > 0) || (q.maxL >= 0)) ok = ok && ko >= q.minL && !(q.maxL >= 0 && ko > q.maxL);
            ok = ok && fabsf(kx - q.x) < q.r && fabsf(ky - q.y) < q.r;
            if (ok && a.u_right && a.u_right[fi] > 0 && fabsf(a.qxr[i] - a.u_right[fi]) > q.r) ok = false;
            if (ok && (!T || T[fi] >= j)) {
                const int d = hamming32(q0, q1, a.desc + (long long)fi * 32);
                if (d <= bound) {
                    const int c = gx * kGridRows + gy;
                    key = ((uint32_t)d << 24) | ((uint32_t)c << 12) | (uint32_t)fi;
                    ent = ((uint32_t)d << 24) | ((uint32_t)(ko & 7) << 16) | (uint32_t)fi;
                }
            }
        }
        const uint64_t has = __ballot(key != kFusedNone);
        if (!has) continue;
        total += __popcll(has);
        // K smallest of (running list) U (this chunk); keys are distinct
        uint32_t prev = 0, nrun = kFusedNone, nrun_e = kFusedNone;
        bool first = true;
        for (int r = 0; r < K; ++r) {
            const uint32_t xa = (first || key > prev) ? key : kFusedNone;
            const uint32_t xb = (lane < K && (first || run > prev)) ? run : kFusedNone;
            const uint32_t x = min(xa, xb);
            const uint32_t xe = xa <= xb ? ent : run_e;
            const uint32_t m = wave_min(x, kFusedNone);
            if (m == kFusedNone) break;
            const int src = __ffsll((long long)__ballot(x == m)) - 1;
            const uint32_t me = (uint32_t)__builtin_amdgcn_readlane((int)xe, src);
            if (lane == r) { nrun = m; nrun_e = me; }
            prev = m;
            first = false;
        }
        run = nrun;
        run_e = nrun_e;
    }
    if (lane < K && run_e != kFusedNone && a.mode == 1 && a.check_ori) {
        const uint32_t bin = (uint32_t)rot_bin(qang, a.kps[run_e & 0xfff].angle);
        run_e |= bin << 19;                           // (lvl | bin << 3) << 16
    }
    return total;
}

// A decision: -1 none, else slot | blocking << 12 | bin << 13.
__device__ __forceinline__ int fused_accept(const ProjArgs& a, int best, int lvl, int best2, int lvl2) {
    if (a.mode == 0) return best <= kThHigh && !(lvl == lvl2 && (float)best > a.ratio * (float)best2);
    return (float)best <= a.accept;
}

// The per-call inputs of a dframe search (orbm_*_dframe): phase 1 reads its
// query's rows straight from pinned host memory through the device mapping
// (one launch, no upload kernel), and every block copies its share of the
// whole input run into a device mirror before the last-arriver hand-off, so
// the last block's phase 2 -- which reads every slot and rescans queries --
// reads HBM.  delta = mirror address - mapped address of the run.
struct Mirror {
    const uint4* src = nullptr;
    uint4* dst = nullptr;
    long long n16 = 0, delta = 0;
};
__device__ __forceinline__ void mirror_share(const Mirror& m) {
    if (!m.src) return;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < m.n16; i += stride) m.dst[i] = m.src[i];
}
template <class T> __device__ __forceinline__ T* mirrored(T* p, long long delta) {
    return p ? (T*)((char*)p + delta) : p;
}

__global__ __launch_bounds__(kFusedThreads) void k_proj_fused(ProjArgs a, int bound, uint32_t* __restrict__ lists,
                                                               int* __restrict__ cnt, unsigned* __restrict__ ticket,
                                                               const int32_t* __restrict__ owner_in,
                                                               int32_t* __restrict__ out, int lds_lists,
                                                               int use_grid, int part, int* done, int seq,
                                                               Mirror mir, const int* __restrict__ pgrid) {
    extern __shared__ __attribute__((aligned(16))) int fl[];
    const int n = a.n, nq = a.nq, tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
    // the frame's grid after the phase-2 tables (used by phase 1 and the rescans)
    int* gcs = nullptr;
    uint32_t* gent = nullptr;
    if (use_grid) {
        gcs = fl + proj_fused_lds(n, nq, lds_lists != 0) / 4;
        gent = (uint32_t*)(gcs + kGridInts);
        if (pgrid) lds_grid_load(pgrid, n, gcs);
        else lds_grid_build(a.kps, n, a.g, -1, gcs, gent, (int*)(gent + max(1, n)));
    }
    const unsigned long long tg = __builtin_amdgcn_s_memtime();
    unsigned long long tsel = 0;
    const ProjLds lo = proj_lds_layout(n, nq, lds_lists != 0);
    uint8_t* const fb = (uint8_t*)fl;
    int* T = (int*)(fb + lo.T);
    int* D = (int*)(fb + lo.D);
    int* dry = (int*)(fb + lo.dry);
    int* hist = (int*)(fb + lo.hist);
    int* misc = (int*)(fb + lo.misc);   // 0 last-block flag, 1 first changed query, 2 ndry, 3 nm, 4 dropped
    uint8_t* pre = fb + lo.pre;
    int* Cs = (int*)(fb + lo.Cs);
    uint32_t* Ls = (uint32_t*)(fb + lo.Ls);
    // ---- phase 1: one wave per query (part 0: all of it in this launch with
    // a ticket; part 1: phase 1 only; part 2: one block, phase 2 only)
    if (part != 2) {
        const int i = blockIdx.x * (kFusedThreads / kWave) + wv;
        if (i < nq) {
            ProjQuery q;
            if (!proj_query(a, i, q)) {
                if (lane == 0) cnt[i] = -1;
            } else {
                uint32_t run, run_e;
                const unsigned long long ts = __builtin_amdgcn_s_memtime();
                const int total = fused_select<kProjK>(a, i, q, bound, nullptr, 0, gcs, gent, run, run_e);
                tsel = __builtin_amdgcn_s_memtime() - ts;
                if (lane < kProjK) lists[(long long)i * kProjK + lane] = run_e;
                // the count with the query's "blocking claim" flag (bit 30): phase 2
                // reads no per-query global array
                const int hob = a.skip_any ? 1 : a.qhas_obs[i] != 0;
                if (lane == 0) cnt[i] = min(total, (1 << 30) - 1) | (hob << 30);
            }
        }
        mirror_share(mir);
    }
    if (part == 1) return;
    // ---- the last block to finish phase 1 runs phase 2
    if (part == 0 && !last_arriver(ticket, &misc[0])) return;
    if (mir.src) {             // phase 2 reads the per-call inputs from their HBM mirror
        const long long d = mir.delta;
        a.qx = mirrored(a.qx, d); a.qy = mirrored(a.qy, d); a.qxr = mirrored(a.qxr, d);
        a.qlevel = mirrored(a.qlevel, d); a.qviewcos = mirrored(a.qviewcos, d); a.qdepth = mirrored(a.qdepth, d);
        a.qvalid = mirrored(a.qvalid, d); a.qhas_obs = mirrored(a.qhas_obs, d); a.qdesc = mirrored(a.qdesc, d);
        a.qangle = mirrored(a.qangle, d); a.blocked = mirrored(a.blocked, d);
        owner_in = mirrored(owner_in, d);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const int mode = a.mode, skip_any = a.skip_any, ori = a.mode == 1 && a.check_ori;
    int rounds = 0, ndry_total = 0;
    for (int s = tid; s < n; s += kFusedThreads) {
        const int o = owner_in[s];
        const bool b = o != -1 && (skip_any || (o <= -2 ? a.blocked[s] != 0 : a.qhas_obs[o] != 0));
        pre[s] = b;
        T[s] = b ? -1 : INT_MAX;
    }
    for (int j = tid; j < nq; j += kFusedThreads) D[j] = -2;           // "no decision yet"
    if (lds_lists) {
        for (int j = tid; j < nq; j += kFusedThreads) Cs[j] = cnt[j];
        for (int e = tid; e < nq * (kProjK / 4); e += kFusedThreads) ((uint4*)Ls)[e] = ((const uint4*)lists)[e];
    }
    if (tid < 32) hist[tid] = 0;
    if (tid < 8) misc[tid] = 0;
    if (tid == 0) misc[1] = nq;
    __syncthreads();
    const unsigned long long t2 = __builtin_amdgcn_s_memtime();
    const uint4* Lsrc = lds_lists ? (const uint4*)Ls : (const uint4*)lists;
    const int* Csrc = lds_lists ? Cs : cnt;
    int settled = 0;          // queries below it decided the same in the last two rounds: final
    // The fixpoint runs over a window of queries [settled, wend) at a time:
    // the claims of the queries before the window are final, so a window
    // converges in the rounds of its own dependency chains, and a round
    // evaluates at most kProjWin queries instead of every unsettled one (6
    // whole-list rounds at 3,000 queries were ~3 list evaluations a thread
    // each).  ORB_PROJ_WIN 0: one window of every query (the round-5 form).
    const int win = kProjWin > 0 ? kProjWin : nq;
    int wend = min(nq, win);
    unsigned long long c_dec = 0, c_res = 0, c_reb = 0, tc = __builtin_amdgcn_s_memtime();
    for (int round = 0; round <= nq; ++round) {
        // decisions under this round's T, queries in [settled, wend) only (an
        // earlier query's decision reads only claims of queries before it,
        // all final).  Groups of 4 queries per thread: 8 lists in registers
        // at once spill
        int chg = INT_MAX;        // the thread's first changed query (one LDS atomic per wave below)
#pragma unroll 1
        for (int u0 = 0; u0 < kFusedQpt; u0 += 4) {
        if (tid + u0 * kFusedThreads >= wend) break;
        if (tid + (u0 + 3) * kFusedThreads < settled) continue;
        uint4 LA[4], LB[4];
        int C[4], H[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int jj = tid + (u0 + u) * kFusedThreads;
            const int j = min(jj, max(nq - 1, 0));
            const int cr = (jj < wend && jj >= settled) ? Csrc[j] : -1;
            C[u] = cr < 0 ? -1 : (cr & ((1 << 30) - 1));
            H[u] = cr < 0 ? 0 : (cr >> 30) & 1;
            LA[u] = Lsrc[(long long)j * 2];
            LB[u] = Lsrc[(long long)j * 2 + 1];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = tid + (u0 + u) * kFusedThreads;
            if (j >= wend || j < settled) continue;
            const uint32_t L[kProjK] = {LA[u].x, LA[u].y, LA[u].z, LA[u].w, LB[u].x, LB[u].y, LB[u].z, LB[u].w};
            int dec = -1;
            if (C[u] > 0) {
                int best = 256, lvl = -1, slot = -1, bin = 0, best2 = 256, lvl2 = -1, nav = 0;
#if ORB_PROJ_TPRE
                // the list's 8 claim words read up front, unconditionally (an
                // index clamped into the table): 8 LDS reads in flight instead of
                // one behind each data-dependent branch
                int tv[kProjK];
#pragma unroll
                for (int k = 0; k < kProjK; ++k) tv[k] = T[min((int)(L[k] & 0xfff), max(n - 1, 0))];
#endif
#pragma unroll
                for (int k = 0; k < kProjK; ++k) {
                    const uint32_t e = L[k];
                    if (k >= C[u] || e == kFusedNone) continue;
                    const int s = (int)(e & 0xfff);
#if ORB_PROJ_TPRE
                    if (tv[k] < j) continue;
#else
                    if (T[s] < j) continue;
#endif
                    if (nav == 0) {
                        best = (int)(e >> 24); lvl = (int)((e >> 16) & 7); bin = (int)((e >> 19) & 31); slot = s;
                    } else if (nav == 1) {
                        best2 = (int)(e >> 24); lvl2 = (int)((e >> 16) & 7);
                    }
                    ++nav;
                }
                const bool exact = C[u] <= kProjK || nav >= 2 || (mode == 1 && nav >= 1);
                if (!exact) {
                    dec = -3;                                            // made by an exact rescan below
                    dry[atomicAdd(&misc[2], 1)] = j;
                } else if (slot >= 0 && fused_accept(a, best, lvl, best2, lvl2)) {
                    dec = slot | (H[u] << 12) | (bin << 13);
                }
            }
            if (dec != -3) {
                if (dec != D[j]) chg = min(chg, j);
                D[j] = dec;
            }
        }
        }
        chg = wave_min(chg, INT_MAX);
        if (lane == 0 && chg < INT_MAX) atomicMin(&misc[1], chg);
        __syncthreads();
        { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); c_dec += t_ - tc; tc = t_; }
        // exact rescans of the decisions a truncated list could not make: one wave each
        const int ndry = misc[2];
        ++rounds;
        ndry_total += ndry;
        for (int t = wv; t < ndry; t += kFusedThreads / kWave) {
            const int j = dry[t];
            ProjQuery q;
            proj_query(a, j, q);
            uint32_t run, run_e;
            fused_select<2>(a, j, q, bound, T, j, gcs, gent, run, run_e);
            const uint32_t e1 = (uint32_t)__builtin_amdgcn_readlane((int)run_e, 0);
            const uint32_t e2 = (uint32_t)__builtin_amdgcn_readlane((int)run_e, 1);
            int dec = -1;
            if (e1 != kFusedNone) {
                const int best = (int)(e1 >> 24), lvl = (int)((e1 >> 16) & 7);
                const int best2 = e2 != kFusedNone ? (int)(e2 >> 24) : 256, lvl2 = e2 != kFusedNone ? (int)((e2 >> 16) & 7) : -1;
                if (fused_accept(a, best, lvl, best2, lvl2)) {
                    const int hob = skip_any ? 1 : a.qhas_obs[j] != 0;
                    dec = (int)(e1 & 0xfff) | (hob << 12) | (int)(((e1 >> 19) & 31) << 13);
                }
            }
            if (lane == 0) {
                if (dec != D[j]) atomicMin(&misc[1], j);
                D[j] = dec;
            }
        }
        __syncthreads();
        { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); c_res += t_ - tc; tc = t_; }
        const int first_changed = misc[1];
        __syncthreads();
        if (first_changed >= wend) {      // the window is final
            if (wend >= nq) break;
            settled = wend;
            wend = min(nq, wend + win);
        } else {
            settled = first_changed;
        }
        // T from this round's decisions: the first blocking claim of each slot
        for (int s = tid; s < n; s += kFusedThreads) T[s] = pre[s] ? -1 : INT_MAX;
        if (tid == 0) { misc[1] = nq; misc[2] = 0; }
        __syncthreads();
        for (int j = tid; j < nq; j += kFusedThreads) {
            const int dec = D[j];
            if (dec >= 0 && (dec >> 12 & 1)) atomicMin(&T[dec & 0xfff], j);
        }
        __syncthreads();
        { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); c_reb += t_ - tc; tc = t_; }
    }
    // ---- outputs: the last claimer of each slot, nmatches, rotation filter
    for (int s = tid; s < n; s += kFusedThreads) T[s] = -1;
    __syncthreads();
    int nacc = 0;
    for (int j = tid; j < nq; j += kFusedThreads) {
        const int dec = D[j];
        if (dec < 0) continue;
        ++nacc;
        atomicMax(&T[dec & 0xfff], j);
        if (ori) hist_add_wave(hist, (dec >> 13) & 31);
    }
    nacc = wave_sum(nacc);
    if (lane == 0) atomicAdd(&misc[3], nacc);
    __syncthreads();
    if (ori) {
        __shared__ int tm[3];
        if (wv == 0) {
            int x1, x2, x3;
            three_maxima_wave(hist, x1, x2, x3);
            if (lane == 0) { tm[0] = x1; tm[1] = x2; tm[2] = x3; }
        }
        for (int s = tid; s < n; s += kFusedThreads) pre[s] = 0;          // reused: slot cleared
        __syncthreads();
        int drop = 0;
        for (int j = tid; j < nq; j += kFusedThreads) {
            const int dec = D[j];
            if (dec < 0) continue;
            const int b = (dec >> 13) & 31;
            if (b == tm[0] || b == tm[1] || b == tm[2]) continue;
            pre[dec & 0xfff] = 1;
            ++drop;
        }
        drop = wave_sum(drop);
        if (lane == 0) atomicAdd(&misc[4], drop);
        __syncthreads();
    }
    for (int s = tid; s < n; s += kFusedThreads) {
        const int last = T[s];
        out[1 + s] = (ori && pre[s]) ? -1 : (last >= 0 ? last : owner_in[s]);
    }
    if (tid == 0) {
        out[0] = misc[3] - misc[4];
        *ticket = 0u;                                                   // reusable
        // statistics after the owner row (orbm_debug_proj_stats): rounds, exact
        // rescans, phase-1 and phase-2 shader clocks of the last block
        out[n + 1] = rounds;
        out[n + 2] = ndry_total;
        out[n + 3] = (int)min(t1 - t0, 0x7fffffffull);
        out[n + 4] = (int)min(__builtin_amdgcn_s_memtime() - t1, 0x7fffffffull);
        // wave 0's grid build and selection, the whole block in 100 MHz ticks
        // (calibrates the shader clock), phase 2's table setup
        out[n + 5] = (int)min(tg - t0, 0x7fffffffull);
        out[n + 6] = (int)min(tsel, 0x7fffffffull);
        out[n + 7] = (int)min(__builtin_amdgcn_s_memrealtime() - rt0, 0x7fffffffull);
        out[n + 8] = (int)min(t2 - t1, 0x7fffffffull);
        // phase 2 by step: decision passes, rescans, T rebuilds, the outputs
        out[n + 9] = (int)min(c_dec, 0x7fffffffull);
        out[n + 10] = (int)min(c_res, 0x7fffffffull);
        out[n + 11] = (int)min(c_reb, 0x7fffffffull);
        out[n + 12] = (int)min(__builtin_amdgcn_s_memtime() - tc, 0x7fffffffull);
    }
    signal_done(done, seq);
}

// Largest distance that can still decide a query (see k_proj_topk).
static int proj_bound(const ProjArgs& a) {
    if (a.mode == 1) return a.accept < 0 ? -1 : (int)std::min(255.0f, std::floor(a.accept));
    int b = kThHigh;
    for (int d = kThHigh + 1; d <= 255; ++d)
        if (a.ratio <= 0.0f || a.ratio * (float)d < (float)kThHigh) b = d;
    return b;
}

// ---------------------------------------------------------------------------
// k_transform: TemplatedVocabulary::transform per descriptor
// (TemplatedVocabulary.h:1217-1259): greedy descent, first child wins ties;
// one thread per descriptor (the tree lives in L2 / Infinity Cache).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_transform(const int* __restrict__ first_child, const int* __restrict__ nchild,
                                                   const int* __restrict__ child_idx,
                                                   const uint8_t* __restrict__ node_desc,
                                                   const int* __restrict__ word_id, const double* __restrict__ weight,
                                                   int n, const uint8_t* __restrict__ desc, int nid_level,
                                                   int32_t* __restrict__ wid_out, double* __restrict__ w_out,
                                                   int32_t* __restrict__ nid_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 q0 = *(const uint4*)(desc + (long long)i * 32), q1 = *(const uint4*)(desc + (long long)i * 32 + 16);
    int fin = 0, level = 0, nid = 0;
    do {
        ++level;
        const int c0 = first_child[fin], nc = nchild[fin];
        const int b0 = child_idx ? child_idx[c0] : c0;
        int best = hamming32(q0, q1, node_desc + (long long)b0 * 32), bid = b0;
        for (int j = 1; j < nc; ++j) {
            const int c = child_idx ? child_idx[c0 + j] : c0 + j;
            const int d = hamming32(q0, q1, node_desc + (long long)c * 32);
            if (d < best) { best = d; bid = c; }
        }
        fin = bid;
        if (level == nid_level) nid = fin;
    } while (nchild[fin] != 0);
    wid_out[i] = word_id[fin];
    w_out[i] = weight[fin];
    nid_out[i] = nid;
}


// ---------------------------------------------------------------------------
// Mapping-thread matchers, pinhole keyframes
// (NLeft == -1, no mpCamera2).  The float expressions follow the reference
// build's contraction (GCC -O3 -march=native, probed in this container):
// a*b + c*d + e*f -> fma(e, f, fma(a, b, c*d)); x*f0 + y*f1 + f2 ->
// fma(x, f0, y*f1) + f2.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float sq2(float a, float b, int fma) { return fma ? __builtin_fmaf(a, a, b * b) : a * a + b * b; }
__device__ __forceinline__ float lin2(float x, float a, float y, float b, float c, int fma) {
    return fma ? __builtin_fmaf(x, a, y * b) + c : x * a + y * b + c;
}

// k_fuse: Fuse(pKF, vpMapPoints, th) (ORBmatcher.cc:1148-1331) -- the keypoint
// each map point would fuse with; one wave per map point (the matching of a
// point reads none of the others' results).  chi2 = 0, accept = TH_LOW is the
// matching of Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (:1340-1455);
// chi2 = 0, accept = TH_HIGH one direction of SearchBySim3 (:1496-1573,
// :1576-1653).  All take the first candidate at the least distance
// (`dist < bestDist`) among the levels pl-1 .. pl.
struct FuseArgs {
    const orb_keypoint* kps;
    const uint8_t* desc;
    const float* u_right;       // mvuRight or NULL
    const float* scale;         // mvScaleFactors
    const float* inv_sigma2;    // mvInvLevelSigma2
    GridParams g;
    const uint32_t* gsorted;
    const int* gcount;
    const int* cellstart;
    int nmp;
    const uint8_t* valid;
    const float *u, *v, *ur;
    const int32_t* level;       // PredictScale
    const uint8_t* mdesc;       // GetDescriptor()
    float th;
    int fma;
    int chi2;                   // 1: the reprojection-error gate of :1267-1280
    int accept;                 // bestDist <= accept
    int32_t* best_idx;
    int32_t* best_dist;
};

__global__ __launch_bounds__(256) void k_fuse(FuseArgs a) {
    const int i = blockIdx.x * 4 + wave_id(), lane = lane_id();
    if (i >= a.nmp) return;
    int out_idx = -1, out_dist = 256;
    if (a.valid[i]) {
        const int pl = a.level[i];
        const float r = a.th * a.scale[pl];                        // :1242
        const float x = a.u[i], y = a.v[i];
        CellRange cr;
        if (cell_range(x, y, r, a.g, cr)) {
            const uint4 q0 = *(const uint4*)(a.mdesc + (long long)i * 32);
            const uint4 q1 = *(const uint4*)(a.mdesc + (long long)i * 32 + 16);
            const AreaRuns ar = area_runs(a.cellstart, cr);
            uint32_t best = 0xffffffffu;            // (dist << 20) | position in GetFeaturesInArea order
            for (int base = 0; base < ar.total; base += kWave) {
                const int t = base + lane;
                const int j = area_pos(ar, min(t, ar.total - 1));
                if (t >= ar.total) continue;
                const int fi = (int)(a.gsorted[j] & 0xffff);
                const orb_keypoint k = a.kps[fi];
                if (!(fabsf(k.x - x) < r && fabsf(k.y - y) < r)) continue;          // KeyFrame.cc:741
                const int kl = k.octave;
                if (kl < pl - 1 || kl > pl) continue;                               // :1262-1265
                if (a.chi2) {
                    const float ex = x - k.x, ey = y - k.y;
                    if (a.u_right && a.u_right[fi] >= 0) {                          // :1267-1280
                        const float er = a.ur[i] - a.u_right[fi];
                        const float e2 = a.fma ? __builtin_fmaf(er, er, __builtin_fmaf(ex, ex, ey * ey))
                                               : ex * ex + ey * ey + er * er;
                        if ((double)(e2 * a.inv_sigma2[kl]) > 7.8) continue;
                    } else {
                        const float e2 = sq2(ex, ey, a.fma);
                        if ((double)(e2 * a.inv_sigma2[kl]) > 5.99) continue;
                    }
                }
                const int d = hamming32(q0, q1, a.desc + (long long)fi * 32);
                best = min(best, ((uint32_t)d << 20) | (uint32_t)t);
            }
            best = wave_min(best, 0xffffffffu);
            if (best != 0xffffffffu && (int)(best >> 20) <= a.accept) {
                out_dist = (int)(best >> 20);
                out_idx = (int)(a.gsorted[area_pos(ar, (int)(best & 0xfffff))] & 0xffff);
            }
        }
    }
    if (lane == 0) {
        a.best_idx[i] = out_idx;
        a.best_dist[i] = out_idx >= 0 ? out_dist : -1;
    }
}

// SearchBySim3's agreement check (ORBmatcher.cc:1655-1671): i1 -> idx2 -> i1.
__global__ __launch_bounds__(256) void k_sim3_agree(const int32_t* __restrict__ m1, int n1,
                                                    const int32_t* __restrict__ m2, int32_t* __restrict__ m12,
                                                    int32_t* __restrict__ nfound) {
    __shared__ int cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    int c = 0;
    for (int i = threadIdx.x; i < n1; i += blockDim.x) {
        const int idx2 = m1[i];
        const bool ok = idx2 >= 0 && m2[idx2] == i;
        m12[i] = ok ? idx2 : -1;
        c += ok;
    }
    atomicAdd(&cnt, c);
    __syncthreads();
    if (threadIdx.x == 0) nfound[0] = cnt;
}

// k_tri: SearchForTriangulation(pKF1, pKF2, ...) (ORBmatcher.cc:907-1146).
// vbMatched2 is never set in the reference, so every KF1 feature is matched
// independently: one wave per (KF1 feature, shared vocabulary node) item.
// Inside a node the reference keeps the LAST candidate at the minimum
// distance among those passing the checks (`dist > bestDist` skips, equal
// distances overwrite), i.e. the lexicographic (min distance, max position).
struct TriArgs {
    const orb_keypoint *k1, *k2;
    const uint8_t *d1, *d2;
    const float *ur1, *ur2;     // mvuRight or NULL
    const uint8_t *mp1, *mp2;   // GetMapPoint(idx) != NULL
    const float* scale2;        // pKF2->mvScaleFactors
    const float* sigma2_2;      // pKF2->mvLevelSigma2
    const int32_t* item_i1;     // items: KF1 feature, range of its node's KF2 features
    const int32_t* item_b;
    const int32_t* item_e;
    const uint32_t* fv2_idx;
    int nitems;
    float F[9];                 // F12 row-major (Eigen F12(r, c) = F[3 r + c])
    float ep_x, ep_y;
    int only_stereo, coarse, fma, check_ori;
    int32_t* item_match;        // KF2 feature or -1
    int32_t* item_bin;
};

__global__ __launch_bounds__(256) void k_tri(TriArgs a) {
    const int t = blockIdx.x * 4 + wave_id(), lane = lane_id();
    if (t >= a.nitems) return;
    const int i1 = a.item_i1[t];
    int res = -1;
    const bool st1 = a.ur1 && a.ur1[i1] >= 0;
    if (!a.mp1[i1] && (!a.only_stereo || st1)) {
        const orb_keypoint kp1 = a.k1[i1];
        const uint4 q0 = *(const uint4*)(a.d1 + (long long)i1 * 32), q1 = *(const uint4*)(a.d1 + (long long)i1 * 32 + 16);
        // epipolar line of kp1 in image 2 (Pinhole::epipolarConstrain, Pinhole.cpp:115-117)
        const float la = lin2(kp1.x, a.F[0], kp1.y, a.F[3], a.F[6], a.fma);
        const float lb = lin2(kp1.x, a.F[1], kp1.y, a.F[4], a.F[7], a.fma);
        const float lc = lin2(kp1.x, a.F[2], kp1.y, a.F[5], a.F[8], a.fma);
        uint32_t best = 0xffffffffu;                // (dist << 16) | (0xffff - position)
        for (int j = a.item_b[t] + lane; j < a.item_e[t]; j += kWave) {
            const int i2 = (int)a.fv2_idx[j];
            if (a.mp2[i2]) continue;
            const bool st2 = a.ur2 && a.ur2[i2] >= 0;
            if (a.only_stereo && !st2) continue;
            const int dist = hamming32(q0, q1, a.d2 + (long long)i2 * 32);
            if (dist > kThLow) continue;
            const orb_keypoint kp2 = a.k2[i2];
            if (!st1 && !st2) {                                                   // :1014-1021
                const float ex = a.ep_x - kp2.x, ey = a.ep_y - kp2.y;
                if (sq2(ex, ey, a.fma) < 100 * a.scale2[kp2.octave]) continue;
            }
            bool ok = a.coarse != 0;
            if (!ok) {                                                            // Pinhole.cpp:119-128
                const float num = lin2(la, kp2.x, lb, kp2.y, lc, a.fma);
                const float den = sq2(la, lb, a.fma);
                if (den != 0) ok = (double)(num * num / den) < 3.84 * (double)a.sigma2_2[kp2.octave];
            }
            if (ok) best = min(best, ((uint32_t)dist << 16) | (uint32_t)(0xffff - (j - a.item_b[t])));
        }
        best = wave_min(best, 0xffffffffu);
        if (best != 0xffffffffu) res = (int)a.fv2_idx[a.item_b[t] + (0xffff - (int)(best & 0xffff))];
        if (lane == 0 && res >= 0) a.item_bin[t] = rot_bin(kp1.angle, a.k2[res].angle);
    }
    if (lane == 0) a.item_match[t] = res;
}

// k_tri_cands: the checked form's candidate ranking.  Per item (KF1 feature
// without a MapPoint, its shared node), every KF2 candidate of the node with
// no MapPoint, the stereo filter passed and dist <= TH_LOW, written to the
// item's segment as key = dist << 16 | (0xffff - node position) and the KF2
// index (ballot compaction, unordered; the host sorts the short lists).
__global__ __launch_bounds__(256) void k_tri_cands(TriArgs a, const int32_t* __restrict__ seg_off,
                                                   int32_t* __restrict__ seg_cnt, uint32_t* __restrict__ ent_key,
                                                   int32_t* __restrict__ ent_i2) {
    const int t = blockIdx.x * 4 + wave_id(), lane = lane_id();
    if (t >= a.nitems) return;
    const int i1 = a.item_i1[t];
    const bool st1 = a.ur1 && a.ur1[i1] >= 0;
    int n = 0;
    if (!a.mp1[i1] && (!a.only_stereo || st1)) {
        const uint4 q0 = *(const uint4*)(a.d1 + (long long)i1 * 32), q1 = *(const uint4*)(a.d1 + (long long)i1 * 32 + 16);
        const int base = seg_off[t];
        for (int j0 = a.item_b[t]; j0 < a.item_e[t]; j0 += kWave) {
            const int j = j0 + lane;
            bool ok = false;
            int i2 = 0, dist = 0;
            if (j < a.item_e[t]) {
                i2 = (int)a.fv2_idx[j];
                const bool st2 = a.ur2 && a.ur2[i2] >= 0;
                if (!a.mp2[i2] && (!a.only_stereo || st2)) {
                    dist = hamming32(q0, q1, a.d2 + (long long)i2 * 32);
                    ok = dist <= kThLow;
                }
            }
            const uint64_t m = __ballot(ok);
            if (ok) {
                const int o = base + n + __popcll(m & ((1ull << lane) - 1));
                ent_key[o] = ((uint32_t)dist << 16) | (uint32_t)(0xffff - (j - a.item_b[t]));
                ent_i2[o] = i2;
            }
            n += __popcll(m);
        }
    }
    if (lane == 0) seg_cnt[t] = n;
}

// rotation-consistency filter and vMatches12 (:1106-1144), one workgroup
__global__ __launch_bounds__(256) void k_tri_final(TriArgs a, int n1, int32_t* matches12, int32_t* nmatches) {
    __shared__ int hist[kHisto];
    __shared__ int keep[3];
    __shared__ int cnt;
    const int tid = threadIdx.x;
    if (tid < kHisto) hist[tid] = 0;
    if (tid == 0) cnt = 0;
    __syncthreads();
    for (int i = tid; i < n1; i += 256) matches12[i] = -1;
    if (a.check_ori)
        for (int t = tid; t < a.nitems; t += 256)
            if (a.item_match[t] >= 0) atomicAdd(&hist[a.item_bin[t]], 1);
    __syncthreads();
    if (tid < kWave) {
        int i1 = -1, i2 = -1, i3 = -1;
        if (a.check_ori) three_maxima_wave(hist, i1, i2, i3);
        if (tid == 0) { keep[0] = i1; keep[1] = i2; keep[2] = i3; }
    }
    __syncthreads();
    for (int t = tid; t < a.nitems; t += 256) {
        const int m = a.item_match[t];
        if (m < 0) continue;
        if (a.check_ori) {
            const int b = a.item_bin[t];
            if (b != keep[0] && b != keep[1] && b != keep[2]) continue;
        }
        matches12[a.item_i1[t]] = m;
        atomicAdd(&cnt, 1);
    }
    __syncthreads();
    if (tid == 0) nmatches[0] = cnt;
}


// k_distinctive: MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:329-405)
// for many points; one wave per point.  Row i's median (vDists[0.5 (N-1)]
// after sorting) is the smallest m with #{j : d_ij <= m} > (N-1)/2, found by
// bisection over [0, 256] with the distances recomputed from the LDS copy of
// the point's descriptors; the first row with the least median wins.
constexpr int kDistinctiveLds = 256;   // descriptors per point held in LDS

__global__ __launch_bounds__(64) void k_distinctive(int npoints, const int32_t* off, const uint8_t* desc,
                                                    int32_t* best_out) {
    __shared__ uint4 sd[kDistinctiveLds][2];
    const int p = blockIdx.x, lane = lane_id();
    if (p >= npoints) return;
    const int b = off[p], n = off[p + 1] - b;
    if (n <= 0) {
        if (lane == 0) best_out[p] = -1;
        return;
    }
    const uint8_t* D = desc + (long long)b * 32;
    const bool lds = n <= kDistinctiveLds;
    if (lds)
        for (int i = lane; i < n; i += kWave) {
            sd[i][0] = *(const uint4*)(D + (long long)i * 32);
            sd[i][1] = *(const uint4*)(D + (long long)i * 32 + 16);
        }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    auto row = [&](int i, uint4& a0, uint4& a1) {
        if (lds) { a0 = sd[i][0]; a1 = sd[i][1]; }
        else { a0 = *(const uint4*)(D + (long long)i * 32); a1 = *(const uint4*)(D + (long long)i * 32 + 16); }
    };
    const int k = (int)(0.5 * (n - 1));                       // vDists[0.5*(N-1)]
    uint32_t best = 0xffffffffu;                               // (median << 16) | row
    for (int i = lane; i < n; i += kWave) {
        uint4 a0, a1;
        row(i, a0, a1);
        int lo = 0, hi = 256;                                  // smallest m with count(d <= m) >= k + 1
        while (lo < hi) {
            const int m = (lo + hi) >> 1;
            int c = 0;
            for (int j = 0; j < n; ++j) {
                uint4 b0, b1;
                row(j, b0, b1);
                const int d = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
                              __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
                c += d <= m;
            }
            if (c >= k + 1) hi = m;
            else lo = m + 1;
        }
        best = min(best, ((uint32_t)lo << 16) | (uint32_t)i);
    }
    best = wave_min(best, 0xffffffffu);
    if (lane == 0) best_out[p] = (int)(best & 0xffff);
}

// ---------------------------------------------------------------------------
// host helpers
// ---------------------------------------------------------------------------
// Per-host-thread bump arenas for the synchronous host APIs: device memory
// and pinned staging, reset at the start of every call (the previous call has
// completed: each ends with a synchronous download).  A call that outgrows
// the arena takes an extra chunk; the next reset coalesces the chunks into
// one, so steady-state calls never allocate.  Arenas live until process exit
// (no destructors: the HIP runtime may already be gone at thread teardown).
struct Arena {
    bool pinned = false;
    std::vector<std::pair<char*, size_t>> chunks;
    size_t cur = 0, off = 0;
    size_t capacity() const { size_t c = 0; for (auto& ch : chunks) c += ch.second; return c; }
    bool grow(size_t bytes) {
        char* q = nullptr;
        const size_t sz = std::max(bytes, std::max<size_t>(size_t(4) << 20, capacity()));
        if (pinned ? hipHostMalloc((void**)&q, sz, hipHostMallocDefault) != hipSuccess
                   : hipMalloc((void**)&q, sz) != hipSuccess)
            return false;
        chunks.emplace_back(q, sz);
        cur = chunks.size() - 1;
        off = 0;
        return true;
    }
    void* get(size_t bytes) {
        bytes = (std::max<size_t>(bytes, 1) + 255) & ~size_t(255);
        if (chunks.empty() || off + bytes > chunks[cur].second)
            if (!grow(bytes)) return nullptr;
        void* r = chunks[cur].first + off;
        off += bytes;
        return r;
    }
    void reset() {
        if (chunks.size() > 1) {
            const size_t tot = capacity();
            for (auto& ch : chunks) (void)(pinned ? hipHostFree(ch.first) : hipFree(ch.first));
            chunks.clear();
            (void)grow(tot);
        }
        cur = 0;
        off = 0;
    }
};

static Arena& dev_arena() { static thread_local Arena* a = new Arena(); return *a; }
static Arena& host_stage() {
    static thread_local Arena* a = [] { Arena* x = new Arena(); x->pinned = true; return x; }();
    return *a;
}

// H2D through pinned staging, asynchronous on the null stream and coalesced:
// DBuf::put takes its device block and its staging block in lockstep from the
// two bump arenas, so the uploads of one call are contiguous on both sides and
// go as ONE copy (each hipMemcpyAsync costs microseconds of API time, and a
// host API uploads a dozen arrays).  The pending run is issued before any other
// GPU operation (KLAUNCH, memsets, downloads, direct copies, arena reset).
struct PendingUpload { char* dst = nullptr; char* src = nullptr; size_t len = 0; };
static PendingUpload& pending_upload() { static thread_local PendingUpload p; return p; }
static size_t round256(size_t b) { return (b + 255) & ~size_t(255); }
// The run goes up by k_pull, a kernel reading the pinned staging through its
// device mapping, not by hipMemcpyAsync: a copy-engine transfer followed by a
// dependent kernel costs ~30 us of hand-off on this box, a kernel followed by a
// kernel ~5 us (tools/latency_floor.hip: upload + kernel + completion 41 vs
// 22 us).  ORB_OPT_UPLOAD 1 selects hipMemcpyAsync.
__global__ __launch_bounds__(256) void k_pull(const uint4* __restrict__ src, uint4* __restrict__ dst, long long n16,
                                              int tail) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
    if (blockIdx.x == 0 && (int)threadIdx.x < tail)
        ((uint8_t*)(dst + n16))[threadIdx.x] = ((const uint8_t*)(src + n16))[threadIdx.x];
}
hipError_t pull_to_device(void* dst, const void* src, size_t len, hipStream_t st) {
    if (!len) return hipSuccess;
    void* src_d = nullptr;
    if (debug_opt(ORB_OPT_UPLOAD) == 1 || hipHostGetDevicePointer(&src_d, const_cast<void*>(src), 0) != hipSuccess ||
        !src_d || ((uintptr_t)dst | (uintptr_t)src_d) % 16)
        return hipMemcpyAsync(dst, src, len, hipMemcpyHostToDevice, st);
    const long long n16 = (long long)(len / 16);
    const int blocks = (int)std::min<long long>(1024, std::max<long long>(1, (n16 + 255) / 256));
    // (ORB_LAUNCH's LDS guard; this function speaks hipError_t)
    if (!lds_fits(reinterpret_cast<const void*>(k_pull), 0)) return hipErrorInvalidConfiguration;
    hipLaunchKernelGGL(k_pull, dim3(blocks), dim3(256), 0, st, (const uint4*)src_d, (uint4*)dst, n16, (int)(len % 16));
    return hipGetLastError();
}
static hipError_t flush_uploads() {
    PendingUpload& p = pending_upload();
    if (!p.len) return hipSuccess;
    const PendingUpload q = p;
    p = PendingUpload{};
    return pull_to_device(q.dst, q.src, q.len, 0);
}
// A run still pending at the next call's reset was never used by a GPU
// operation: it is dropped (issuing it now would race the reused staging).
static void arena_reset() { pending_upload() = PendingUpload{}; dev_arena().reset(); host_stage().reset(); }

static hipError_t h2d(void* dst, const void* src, size_t bytes) {
    if (!bytes) return hipSuccess;
    char* st = (char*)host_stage().get(bytes);
    if (!st) return hipErrorOutOfMemory;
    std::memcpy(st, src, bytes);
    PendingUpload& p = pending_upload();
    if (p.len && (char*)dst == p.dst + round256(p.len) && st == p.src + round256(p.len)) {
        p.len = (size_t)((char*)dst - p.dst) + bytes;          // extends the run (gaps are arena padding)
        return hipSuccess;
    }
    const hipError_t e = flush_uploads();
    p.dst = (char*)dst; p.src = st; p.len = bytes;
    return e;
}
// D2H through pinned staging (synchronous).
static hipError_t d2h(void* dst, const void* src, size_t bytes) {
    if (!bytes) return hipSuccess;
    if (const hipError_t e = flush_uploads(); e != hipSuccess) return e;
    void* st = host_stage().get(bytes);
    if (!st) return hipErrorOutOfMemory;
    hipError_t e = hipMemcpyAsync(st, src, bytes, hipMemcpyDeviceToHost, 0);
    if (e == hipSuccess) e = hipStreamSynchronize(0);
    if (e == hipSuccess) std::memcpy(dst, st, bytes);
    return e;
}

// The word a host call's kernel writes last (system scope) and the host polls
// instead of synchronising the stream: a sequence number per call, pinned and
// mapped, one per host thread.
struct DoneWord {
    int* h = nullptr;
    int* d = nullptr;
    int seq = 0;
};
static DoneWord& done_word() {
    static thread_local DoneWord w = [] {
        DoneWord x;
        if (hipHostMalloc((void**)&x.h, 64, hipHostMallocPortable) != hipSuccess ||
            hipHostGetDevicePointer((void**)&x.d, x.h, 0) != hipSuccess) {
            x.h = x.d = nullptr;
        } else {
            *(volatile int*)x.h = 0;
        }
        return x;
    }();
    return w;
}

// The result block of a single-launch host call.  ORB_OPT_HOST_OUT 0 (default):
// the kernel writes it straight into pinned host memory (the staging arena,
// mapped into the device's address space) and then a completion word the host
// spins on; 1: the same block, but the call synchronises the stream; 2: device
// memory brought back by one d2h.
struct OutBlock {
    int32_t* d = nullptr;      // what the kernel writes
    int32_t* h = nullptr;      // host view (zero-copy) or nullptr
    size_t n = 0;
    int* flag = nullptr;       // ORB_OPT_HOST_OUT 0: the completion word the kernel writes last (device view)
    int seq = 0;
    // host_only: the block is pinned host memory in every mode (mode 2 acts
    // as 0: the dframe searches' kernels always write their result there)
    int alloc(size_t cnt, bool host_only = false) {
        n = std::max<size_t>(1, cnt);
        int mode = debug_opt(ORB_OPT_HOST_OUT);
        if (host_only && mode == 2) mode = 0;
        flag = nullptr;
        if (mode != 2) {
            h = (int32_t*)host_stage().get(n * sizeof(int32_t));
            if (!h || hipHostGetDevicePointer((void**)&d, h, 0) != hipSuccess) return ORB_ERR_DEVICE;
            if (mode != 1) {
                DoneWord& w = done_word();
                if (!w.h) return ORB_ERR_DEVICE;
                flag = w.d;
                w.seq = (w.seq + 1) & 0x7fffffff;    // never 0 (the word's initial value)
                if (!w.seq) w.seq = 1;
                seq = w.seq;
            }
            return ORB_OK;
        }
        h = nullptr;
        d = (int32_t*)dev_arena().get(n * sizeof(int32_t));
        return d ? ORB_OK : ORB_ERR_DEVICE;
    }
    // after the launch: the block's words [0, cnt) into dst
    hipError_t fetch(int32_t* dst, size_t cnt) const {
        if (!h) return d2h(dst, d, cnt * sizeof(int32_t));
        if (flag) {
            // spin on the word; every 256 reads ask the stream whether it ended
            // without writing it (a fault) -- then its error is the result
            const volatile int* w = done_word().h;
            for (unsigned spin = 1; *w != seq; ++spin) {
                if ((spin & 255) == 0) {
                    const hipError_t q = hipStreamQuery(0);
                    if (q != hipErrorNotReady) {
                        if (*w == seq) break;
                        return q == hipSuccess ? hipErrorUnknown : q;
                    }
                }
            }
            std::atomic_thread_fence(std::memory_order_acquire);   // the block was released before the word
        } else if (const hipError_t e = hipStreamSynchronize(0); e != hipSuccess) {
            return e;
        }
        std::memcpy(dst, h, cnt * sizeof(int32_t));
        return hipSuccess;
    }
};

// A device buffer of the current host-API call (arena-backed).
template <typename T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    int alloc(size_t cnt) {
        if (p && cnt <= n) return ORB_OK;
        p = (T*)dev_arena().get(std::max<size_t>(1, cnt) * sizeof(T));
        if (!p) return ORB_ERR_DEVICE;
        n = cnt;
        return ORB_OK;
    }
    int put(const T* src, size_t cnt, hipStream_t = 0) {
        int rc = alloc(cnt);
        if (rc) return rc;
        return h2d(p, src, cnt * sizeof(T)) == hipSuccess ? ORB_OK : ORB_ERR_DEVICE;
    }
};

// A persistent device buffer (the asynchronous batch APIs' workspaces).
template <typename T>
struct PBuf {
    T* p = nullptr;
    size_t n = 0;
    PBuf() = default;
    PBuf(const PBuf&) = delete;
    PBuf& operator=(const PBuf&) = delete;
    ~PBuf() {
        if (p) (void)hipFree(p);
    }
    int alloc(size_t cnt) {
        if (cnt <= n) return ORB_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        if (hipMalloc(&p, std::max<size_t>(1, cnt) * sizeof(T)) != hipSuccess) return ORB_ERR_DEVICE;
        n = cnt;
        return ORB_OK;
    }
    int put(const T* src, size_t cnt, hipStream_t st = 0) {
        int rc = alloc(cnt);
        if (rc) return rc;
        if (flush_uploads() != hipSuccess) return ORB_ERR_DEVICE;
        if (cnt && hipMemcpyAsync(p, src, cnt * sizeof(T), hipMemcpyHostToDevice, st) != hipSuccess) return ORB_ERR_DEVICE;
        return ORB_OK;
    }
};

static int pow2_at_least(int n) { int p = 64; while (p < n) p <<= 1; return p; }

// Device scratch that batched launches keep between calls (grown on demand),
// one set per (device, stream, kind) of the calling thread -- two searches
// issued on different streams, or for different GPUs, must not share buffers
// -- most recently used first.  Each use ends with an event recorded on the
// set's stream (scratch_used), so a set is freed only after ITS stream's last
// use of it has finished (hipEventSynchronize of that event: no device-wide
// synchronisation, no stall of the other streams).  At most kScratchSets stay
// allocated (hardware queues x scratch kinds with room to spare); a call on a
// further stream frees the least recently used set that way.
// orbm_release_scratch frees a stream's sets at once; a caller must do so
// before destroying a stream it used here, or a new stream at the same address
// would inherit the buffers unordered against the old stream's work.
struct ScratchBase {
    virtual ~ScratchBase() = default;
};
constexpr size_t kScratchSets = 16;
struct ScratchEntry {
    int dev;
    hipStream_t st;
    const void* kind;
    std::unique_ptr<ScratchBase> s;
    hipEvent_t ev;              // recorded after the set's last use (nullptr: never used)
};
static std::list<ScratchEntry>& scratch_sets() {
    static thread_local std::list<ScratchEntry>* l = new std::list<ScratchEntry>();   // never destroyed at exit
    return *l;
}
// Frees a set once its stream's last use of it has completed; false (and the
// set kept, leaked rather than freed under running work) if that wait fails.
static bool scratch_free(ScratchEntry& e) {
    if (e.ev) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        if (cur != e.dev && hipSetDevice(e.dev) != hipSuccess) return false;
        const hipError_t w = hipEventSynchronize(e.ev);
        if (w == hipSuccess) (void)hipEventDestroy(e.ev);
        if (cur != e.dev) (void)hipSetDevice(cur);
        if (w != hipSuccess) return false;
        e.ev = nullptr;
    }
    e.s.reset();
    return true;
}
template <class S>
static S* stream_scratch(hipStream_t st) {
    static const char kind = 0;                      // one address per scratch type
    auto& L = scratch_sets();
    int dev = 0;
    (void)hipGetDevice(&dev);
    for (auto it = L.begin(); it != L.end(); ++it)
        if (it->dev == dev && it->st == st && it->kind == &kind) {
            L.splice(L.begin(), L, it);
            return static_cast<S*>(L.front().s.get());
        }
    if (L.size() >= kScratchSets) {
        if (!scratch_free(L.back())) return nullptr;
        L.pop_back();
    }
    L.push_front(ScratchEntry{dev, st, &kind, std::make_unique<S>(), nullptr});
    return static_cast<S*>(L.front().s.get());
}
// After a call's launches on `st`: the front set (the one stream_scratch just
// returned) records its stream's progress.
static int scratch_used(hipStream_t st) {
    ScratchEntry& e = scratch_sets().front();
    if (!e.ev && hipEventCreateWithFlags(&e.ev, hipEventDisableTiming) != hipSuccess) {
        e.ev = nullptr;
        return ORB_ERR_DEVICE;
    }
    return hipEventRecord(e.ev, st) == hipSuccess ? ORB_OK : ORB_ERR_DEVICE;
}

static GridParams grid_params(const orbm_frame* f) {
    return GridParams{f->min_x, f->min_y, f->grid_inv_w, f->grid_inv_h};
}

// Upload one frame and build its grid order on the device.
struct DevFrame {
    DBuf<orb_keypoint> kps;
    DBuf<uint8_t> desc;
    DBuf<int> n;
    DBuf<uint32_t> sorted;
    DBuf<int> count;
    DBuf<int> cs;               // cell-start table (k_cell_start)
    DBuf<float> ur, scale;
    int upload(const orbm_frame* f, bool grid, hipStream_t st) {
        int rc;
        const int nn = std::max(1, f->n);
        if ((rc = kps.alloc(nn)) || (rc = desc.alloc((size_t)nn * 32)) || (rc = n.put(&f->n, 1, st))) return rc;
        if (f->n) {
            if (h2d(kps.p, f->kps, f->n * sizeof(orb_keypoint)) != hipSuccess ||
                h2d(desc.p, f->desc, (size_t)f->n * 32) != hipSuccess)
                return ORB_ERR_DEVICE;
        }
        if (f->u_right && (rc = ur.put(f->u_right, f->n, st))) return rc;
        if (f->scale_factors && (rc = scale.put(f->scale_factors, f->nlevels, st))) return rc;
        return grid ? build_grid(f, st) : ORB_OK;
    }
    // the frame's grid order and cell-start table (AssignFeaturesToGrid)
    int build_grid(const orbm_frame* f, hipStream_t st) {
        int rc;
        const int nn = std::max(1, f->n);
        if ((rc = sorted.alloc(nn)) || (rc = count.alloc(1)) || (rc = cs.alloc(kCells + 1))) return rc;
        if (grid_cs_lds(nn) <= 160 * 1024) {
            KLAUNCH(k_grid_cs, dim3(1), dim3(256), grid_cs_lds(nn), st, kps.p, n.p, nn,
                               grid_params(f), sorted.p, count.p, cs.p, (uint32_t*)nullptr, (int*)nullptr);
        } else {
            const int sc = pow2_at_least(nn);
            KLAUNCH(k_grid, dim3(1), dim3(256), sc * sizeof(uint32_t), st, kps.p, n.p, nn,
                               grid_params(f), sorted.p, count.p, sc, (uint32_t*)nullptr, (int*)nullptr);
            KLAUNCH(k_cell_start, dim3(1), dim3(256), 0, st, sorted.p, count.p, nn, cs.p);
        }
        return ORB_OK;
    }
};

// the last fused projection search's statistics (orbm_debug_proj_stats)
static int32_t* proj_stats() { static thread_local int32_t st[12] = {}; return st; }

// Start of a synchronous host-API call: a device must be present; the call's
// arenas start empty.
static int device_ok() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return ORB_ERR_DEVICE;
    arena_reset();
    return ORB_OK;
}

// the map's descriptors in FeatureVector order, one block per keyframe
__global__ __launch_bounds__(256) void k_fv_desc(const uint8_t* __restrict__ desc, const long long* __restrict__ kp_off,
                                                 const int* __restrict__ fv_off, const uint32_t* __restrict__ fv_idx,
                                                 const long long* __restrict__ node_off,
                                                 const long long* __restrict__ idx_off, uint8_t* __restrict__ out) {
    const int i = blockIdx.x;
    const long long nn = node_off[i + 1] - node_off[i];
    const int n = fv_off[node_off[i] + i + nn];        // the keyframe's FeatureVector entries
    const long long io = idx_off[i], ko = kp_off[i];
    for (int q = threadIdx.x; q < 2 * n; q += blockDim.x) {   // 16-byte halves
        const int p = q >> 1, h = q & 1;
        ((uint4*)out)[(io + p) * 2 + h] = ((const uint4*)desc)[(ko + fv_idx[io + p]) * 2 + h];
    }
}

// the map's keypoint angles in FeatureVector order, one block per keyframe
__global__ __launch_bounds__(256) void k_fv_angle(const orb_keypoint* __restrict__ kps, const long long* __restrict__ kp_off,
                                                  const int* __restrict__ fv_off, const uint32_t* __restrict__ fv_idx,
                                                  const long long* __restrict__ node_off,
                                                  const long long* __restrict__ idx_off, float* __restrict__ out) {
    const int i = blockIdx.x;
    const long long nn = node_off[i + 1] - node_off[i];
    const int n = fv_off[node_off[i] + i + nn];
    const long long io = idx_off[i], ko = kp_off[i];
    for (int p = threadIdx.x; p < n; p += blockDim.x) out[io + p] = kps[ko + fv_idx[io + p]].angle;
}

// ---------------------------------------------------------------------------
// k_sfi_fused: SearchForInitialization(F1, F2, ...) (ORBmatcher.cc:648-763)
// in ONE launch for the host API, no grid build (the k_proj_fused pattern).
//
// Phase 1, one wave per F1 keypoint of octave 0: its kTopK smallest F2
// candidates by (distance, GetFeaturesInArea order) from a brute-force pass
// over F2 (octave 0, in a visited cell, |dx| < window, |dy| < window), only
// distances that can still decide (d <= bound: a best above TH_LOW is
// rejected anyway, and a second above TH_LOW / ratio cannot fail the ratio
// test).  Phase 2, last block: the serial loop's only order dependence is the
// skip rule `vMatchedDistance[i2] <= dist` (:687-688), where vMatchedDistance
// of slot s seen by query j is the distance of the LATEST claim on s by a
// query before j (a steal needs a strictly smaller distance, so that is also
// the smallest).  Recomputing every decision from the previous round's claims
// (per-slot claim lists sorted by query) leaves the earliest wrong decision
// right after each round; two equal rounds are the serial outcome.  Then the
// last claimer of each slot keeps it (earlier ones were stolen: vnMatches12 =
// -1), nmatches = claimed slots, the rotation histogram counts every accepted
// claim (stolen ones too, as rotHist does) and unmatches the kept matches of
// rejected bins, and vbPrevMatched takes the matched F2 positions.
// ---------------------------------------------------------------------------
struct SfiFusedArgs {
    const orb_keypoint* k1; const uint8_t* d1; int n1;
    const orb_keypoint* k2; const uint8_t* d2; int n2;
    const float* prev;                          // [n1][2]
    GridParams g;
    float window, ratio;
    int check_ori, bound;
};

// LDS: D[n1] | dry[n1] | ccnt[n2 + 1] | cstart[n2 + 1] | claims[n1] | hist[32] | misc[8] | scan tmp[32]
__host__ __device__ inline size_t sfi_fused_lds(int n1, int n2) { return (size_t)(3 * n1 + 2 * (n2 + 1) + 72) * 4; }

// K smallest candidate keys of F1 keypoint i (d << 24 | cell << 12 | F2 index),
// skipping (cl != nullptr) candidates a claim before query j blocks; lane r < K
// holds the r-th key and its entry d << 24 | bin << 16 | slot.  Returns the
// number of candidates within the bound.
template <int K>
__device__ int sfi_select(const SfiFusedArgs& a, int i, const CellRange& cr, float px, float py, const int* ccnt,
                          const int* cstart, const int* claims, int j, const int* gcs, const uint32_t* gent,
                          uint32_t& run, uint32_t& run_e) {
    const int lane = lane_id();
    const uint4 q0 = *(const uint4*)(a.d1 + (long long)i * 32);
    const uint4 q1 = *(const uint4*)(a.d1 + (long long)i * 32 + 16);
    const float r = a.window;
    const float* kf = (const float*)a.k2;
    const int kw = (int)(sizeof(orb_keypoint) / 4);
    WinCols w{};
    int len = a.n2;
    if (gcs) {
        w = win_cols(gcs, cr);
        len = w.total;
    }
    auto kload = [&](int base, int& f, float& x, float& y, int& o) {
        const int p = min(base + lane, max(len - 1, 0));
        f = gcs ? (int)(win_entry(w, gent, p) & 0xfff) : p;
        x = kf[(long long)f * kw + 0];
        y = kf[(long long)f * kw + 1];
        o = ((const int*)kf)[(long long)f * kw + 5];
    };
    run = kFusedNone;
    run_e = kFusedNone;
    int total = 0;
    float nx = 0.f, ny = 0.f;
    int no = 0, nf = 0;
    if (len > 0) kload(0, nf, nx, ny, no);
    for (int base = 0; base < len; base += kWave) {
        const float kx = nx, ky = ny;
        const int ko = no, fi = nf;
        if (base + kWave < len) kload(base + kWave, nf, nx, ny, no);
        uint32_t key = kFusedNone, ent = kFusedNone;
        if (base + lane < len && ko == 0) {
            const int gx = (int)roundf((kx - a.g.min_x) * a.g.inv_w);
            const int gy = (int)roundf((ky - a.g.min_y) * a.g.inv_h);
            if (gx >= cr.x0 && gx <= cr.x1 && gy >= cr.y0 && gy <= cr.y1 && gx >= 0 && gx < kGridCols && gy >= 0 &&
                gy < kGridRows && fabsf(kx - px) < r && fabsf(ky - py) < r) {
                const int d = hamming32(q0, q1, a.d2 + (long long)fi * 32);
                bool usable = d <= a.bound;
                if (usable && claims) {
                    // vMatchedDistance[fi] before query j: the latest claim before j
                    int md = INT_MAX;
                    for (int c = cstart[fi], ce = c + ccnt[fi]; c < ce; ++c) {
                        const int cl = claims[c];
                        if ((cl >> 8) >= j) break;
                        md = cl & 0xff;
                    }
                    usable = md > d;
                }
                if (usable) {
                    key = ((uint32_t)d << 24) | ((uint32_t)(gx * kGridRows + gy) << 12) | (uint32_t)fi;
                    ent = ((uint32_t)d << 24) | (uint32_t)fi;
                }
            }
        }
        const uint64_t has = __ballot(key != kFusedNone);
        if (!has) continue;
        total += __popcll(has);
        uint32_t prev = 0, nrun = kFusedNone, nrun_e = kFusedNone;
        bool first = true;
        for (int rr = 0; rr < K; ++rr) {
            const uint32_t xa = (first || key > prev) ? key : kFusedNone;
            const uint32_t xb = (lane < K && (first || run > prev)) ? run : kFusedNone;
            const uint32_t x = min(xa, xb);
            const uint32_t xe = xa <= xb ? ent : run_e;
            const uint32_t m = wave_min(x, kFusedNone);
            if (m == kFusedNone) break;
            const int src = __ffsll((long long)__ballot(x == m)) - 1;
            const uint32_t me = (uint32_t)__builtin_amdgcn_readlane((int)xe, src);
            if (lane == rr) { nrun = m; nrun_e = me; }
            prev = m;
            first = false;
        }
        run = nrun;
        run_e = nrun_e;
    }
    if (lane < K && run_e != kFusedNone && a.check_ori)
        run_e |= (uint32_t)rot_bin(a.k1[i].angle, a.k2[run_e & 0xfff].angle) << 16;
    return total;
}

// accept (:701-703): bestDist <= TH_LOW and bestDist < bestDist2 * nnratio
__device__ __forceinline__ bool sfi_accept(int best, int best2, float ratio) {
    return best <= kThLow && (float)best < (float)best2 * ratio;
}

__global__ __launch_bounds__(kFusedThreads) void k_sfi_fused(SfiFusedArgs a, uint32_t* __restrict__ lists,
                                                              int* __restrict__ cnt, unsigned* __restrict__ ticket,
                                                              int32_t* __restrict__ out, int use_grid, int part,
                                                              int* done, int seq, Mirror mir,
                                                              const int* __restrict__ pgrid) {
    extern __shared__ __attribute__((aligned(16))) int sl[];
    const int n1 = a.n1, n2 = a.n2, tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
    // F2's level-0 grid after the phase-2 tables (phase 1 and the rescans)
    int* gcs = nullptr;
    uint32_t* gent = nullptr;
    if (use_grid) {
        gcs = sl + sfi_fused_lds(n1, n2) / 4;
        gent = (uint32_t*)(gcs + kGridInts);
        if (pgrid) lds_grid_load(pgrid, n2, gcs);
        else lds_grid_build(a.k2, n2, a.g, 0, gcs, gent, (int*)(gent + max(1, n2)));
    }
    const unsigned long long tg = __builtin_amdgcn_s_memtime();
    unsigned long long tsel = 0;
    int* D = sl;                                // decision: -1 none, else slot | d << 12 | bin << 20
    int* dry = D + n1;
    int* ccnt = dry + n1;                       // claims per slot
    int* cstart = ccnt + n2 + 1;                // their segment starts
    int* claims = cstart + n2 + 1;              // j << 8 | d, by slot, ascending j
    int* hist = claims + n1;
    int* misc = hist + 32;                      // 0 last block, 1 first changed, 2 ndry, 3 fill, 4 nm, 5 dropped
    // ---- phase 1 (part 0: both phases in this launch with a ticket; part 1:
    // phase 1 only; part 2: one block, phase 2 only)
    if (part != 2) {
        const int i = blockIdx.x * (kFusedThreads / kWave) + wv;
        if (i < n1) {
            const float px = a.prev[2 * i], py = a.prev[2 * i + 1];
            CellRange cr;
            if (a.k1[i].octave != 0 || !cell_range(px, py, a.window, a.g, cr)) {
                if (lane == 0) cnt[i] = -1;
            } else {
                uint32_t run, run_e;
                const unsigned long long ts = __builtin_amdgcn_s_memtime();
                const int total = sfi_select<kTopK>(a, i, cr, px, py, nullptr, nullptr, nullptr, 0, gcs, gent, run, run_e);
                tsel = __builtin_amdgcn_s_memtime() - ts;
                if (lane < kTopK) lists[(long long)i * kTopK + lane] = run_e;
                if (lane == 0) cnt[i] = total;
            }
        }
        mirror_share(mir);
    }
    if (part == 1) return;
    if (part == 0 && !last_arriver(ticket, &misc[0])) return;
    if (mir.src) a.prev = mirrored(a.prev, mir.delta);   // phase 2: prev from its HBM mirror
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    // ---- phase 2: fixpoint over all queries
    for (int j = tid; j < n1; j += kFusedThreads) D[j] = -2;
    for (int s = tid; s <= n2; s += kFusedThreads) { ccnt[s] = 0; cstart[s] = 0; }
    if (tid < 32) hist[tid] = 0;
    if (tid < 8) misc[tid] = 0;
    if (tid == 0) misc[1] = n1;
    __syncthreads();
    const float ratio = a.ratio;
    const int* cl = nullptr;                    // no claims in round 0
    int settled = 0, rounds = 0, ndry_total = 0;
    const unsigned long long t2 = __builtin_amdgcn_s_memtime();
    unsigned long long c_dec = 0, c_res = 0, c_reb = 0, tc = t2;
    for (int round = 0; round <= n1; ++round) {
        int chg = INT_MAX;                       // the thread's first changed query
        for (int j = tid; j < n1; j += kFusedThreads) {
            if (j < settled) continue;
            const int c = cnt[j];
            int dec = -1;
            if (c > 0) {
                const uint4 LA = ((const uint4*)lists)[(long long)j * 2], LB = ((const uint4*)lists)[(long long)j * 2 + 1];
                const uint32_t L[kTopK] = {LA.x, LA.y, LA.z, LA.w, LB.x, LB.y, LB.z, LB.w};
                int best = INT_MAX, slot = -1, bin = 0, best2 = INT_MAX, nav = 0, dlast = 0;
#pragma unroll
                for (int k = 0; k < kTopK; ++k) {
                    const uint32_t e = L[k];
                    if (k >= c || e == kFusedNone) continue;
                    const int s = (int)(e & 0xfff), d = (int)(e >> 24);
                    dlast = d;
                    if (cl) {
                        int md = INT_MAX;
                        for (int q = cstart[s], qe = q + ccnt[s]; q < qe; ++q) {
                            const int x = cl[q];
                            if ((x >> 8) >= j) break;
                            md = x & 0xff;
                        }
                        if (md <= d) continue;                          // :687-688
                    }
                    if (nav == 0) { best = d; slot = s; bin = (int)((e >> 16) & 31); }
                    else if (nav == 1) best2 = d;
                    ++nav;
                }
                // a truncated list decides when two usable entries are listed, or
                // one that fails TH_LOW, or one the unlisted rest (every distance
                // >= the last listed one) cannot reject by the ratio
                const bool exact = c <= kTopK || nav >= 2 ||
                                   (nav == 1 && (best > kThLow || (float)best < (float)dlast * ratio));
                if (!exact) {
                    dec = -3;
                    dry[atomicAdd(&misc[2], 1)] = j;
                } else if (slot >= 0 && sfi_accept(best, best2, ratio)) {
                    dec = slot | (best << 12) | (bin << 20);
                }
            }
            if (dec != -3) {
                if (dec != D[j]) chg = min(chg, j);
                D[j] = dec;
            }
        }
        chg = wave_min(chg, INT_MAX);            // one LDS atomic per wave
        if (lane == 0 && chg < INT_MAX) atomicMin(&misc[1], chg);
        __syncthreads();
        { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); c_dec += t_ - tc; tc = t_; }
        const int ndry = misc[2];
        ++rounds;
        ndry_total += ndry;
        for (int t = wv; t < ndry; t += kFusedThreads / kWave) {
            const int j = dry[t];
            const float px = a.prev[2 * j], py = a.prev[2 * j + 1];
            CellRange cr;
            cell_range(px, py, a.window, a.g, cr);
            uint32_t run, run_e;
            sfi_select<2>(a, j, cr, px, py, ccnt, cstart, cl, j, gcs, gent, run, run_e);
            const uint32_t e1 = (uint32_t)__builtin_amdgcn_readlane((int)run_e, 0);
            const uint32_t e2 = (uint32_t)__builtin_amdgcn_readlane((int)run_e, 1);
            int dec = -1;
            if (e1 != kFusedNone) {
                const int best = (int)(e1 >> 24), best2 = e2 != kFusedNone ? (int)(e2 >> 24) : INT_MAX;
                if (sfi_accept(best, best2, ratio)) dec = (int)(e1 & 0xfff) | (best << 12) | (int)(((e1 >> 16) & 31) << 20);
            }
            if (lane == 0) {
                if (dec != D[j]) atomicMin(&misc[1], j);
                D[j] = dec;
            }
        }
        __syncthreads();
        { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); c_res += t_ - tc; tc = t_; }
        const int first_changed = misc[1];
        __syncthreads();
        if (first_changed >= n1 && round > 0) break;
        settled = first_changed;
        // the claim lists of this round's decisions, by slot and ascending query
        for (int s = tid; s <= n2; s += kFusedThreads) { ccnt[s] = 0; cstart[s] = 0; }
        if (tid == 0) { misc[1] = n1; misc[2] = 0; misc[3] = 0; }
        __syncthreads();
        for (int j = tid; j < n1; j += kFusedThreads)      // counts, then the segment starts in place
            if (D[j] >= 0) atomicAdd(&cstart[D[j] & 0xfff], 1);
        __syncthreads();
        block_excl_scan(cstart, n2, misc + 8);              // (ends in a barrier)
        for (int j = tid; j < n1; j += kFusedThreads) {     // fill; ccnt ends as the counts
            const int dec = D[j];
            if (dec < 0) continue;
            const int s = dec & 0xfff;
            claims[cstart[s] + atomicAdd(&ccnt[s], 1)] = (j << 8) | ((dec >> 12) & 0xff);
        }
        __syncthreads();
        for (int s = tid; s < n2; s += kFusedThreads) {     // insertion sort of each slot's few claims by query
            const int b = cstart[s], m = ccnt[s];
            for (int x = b + 1; x < b + m; ++x) {
                const int v = claims[x];
                int y = x - 1;
                while (y >= b && claims[y] > v) { claims[y + 1] = claims[y]; --y; }
                claims[y + 1] = v;
            }
        }
        cl = claims;
        __syncthreads();
        { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); c_reb += t_ - tc; tc = t_; }
    }
    // ---- outputs (with the final claim lists: the rounds ended on a fixpoint)
    // every accepted claim enters the histogram; the last claimer of a slot keeps it
    int nacc = 0;
    for (int j = tid; j < n1; j += kFusedThreads) {
        const int dec = D[j];
        if (dec < 0) continue;
        if (a.check_ori) hist_add_wave(hist, (dec >> 20) & 31);
    }
    for (int s = tid; s < n2; s += kFusedThreads) nacc += ccnt[s] > 0;
    nacc = wave_sum(nacc);
    if (lane == 0) atomicAdd(&misc[4], nacc);
    __syncthreads();
    __shared__ int tm[3];
    if (wv == 0) {
        int x1 = -1, x2 = -1, x3 = -1;
        if (a.check_ori) three_maxima_wave(hist, x1, x2, x3);
        if (lane == 0) { tm[0] = x1; tm[1] = x2; tm[2] = x3; }
    }
    __syncthreads();
    int drop = 0;
    int32_t* m12 = out + 1;
    float* pout = (float*)(out + 1 + n1);
    for (int j = tid; j < n1; j += kFusedThreads) {
        const int dec = D[j];
        int m = -1;
        if (dec >= 0) {
            const int s = dec & 0xfff;
            const bool last = (claims[cstart[s] + ccnt[s] - 1] >> 8) == j;
            if (last) {
                const int b = (dec >> 20) & 31;
                if (a.check_ori && b != tm[0] && b != tm[1] && b != tm[2]) ++drop;
                else m = s;
            }
        }
        m12[j] = m;
        pout[2 * j] = m >= 0 ? a.k2[m].x : a.prev[2 * j];
        pout[2 * j + 1] = m >= 0 ? a.k2[m].y : a.prev[2 * j + 1];
    }
    drop = wave_sum(drop);
    if (lane == 0) atomicAdd(&misc[5], drop);
    __syncthreads();
    if (tid == 0) {
        out[0] = misc[4] - misc[5];
        *ticket = 0u;
        // statistics after the outputs, as k_proj_fused's (orbm_debug_proj_stats)
        int32_t* st = out + 1 + 3 * n1;
        st[0] = rounds;
        st[1] = ndry_total;
        st[2] = (int)min(t1 - t0, 0x7fffffffull);
        st[3] = (int)min(__builtin_amdgcn_s_memtime() - t1, 0x7fffffffull);
        st[4] = (int)min(tg - t0, 0x7fffffffull);
        st[5] = (int)min(tsel, 0x7fffffffull);
        st[6] = (int)min(__builtin_amdgcn_s_memrealtime() - rt0, 0x7fffffffull);
        st[7] = (int)min(t2 - t1, 0x7fffffffull);
        st[8] = (int)min(c_dec, 0x7fffffffull);
        st[9] = (int)min(c_res, 0x7fffffffull);
        st[10] = (int)min(c_reb, 0x7fffffffull);
        st[11] = (int)min(__builtin_amdgcn_s_memtime() - tc, 0x7fffffffull);
    }
    signal_done(done, seq);
}

}  // namespace orbmi


// ---------------------------------------------------------------------------
// Frames resident in HBM (orbm_dframe_*, include/orb_mi355x.h).
// ---------------------------------------------------------------------------
struct orbm_dframe {
    int device = 0;
    int n = 0, cap_k = 0, cap_d = 0;        // keypoints; allocated keypoint rows / descriptor bytes
    orb_keypoint* kps = nullptr;
    uint8_t* desc = nullptr;
    float* ur = nullptr;                    // mvuRight (n) when the frame has one
    float* scale = nullptr;                 // mvScaleFactors (nlevels)
    int ur_cap = 0, scale_cap = 0, nlevels = 0;
    bool has_ur = false, has_scale = false;
    orbmi::GridParams g{};
    float max_x = 0.f, max_y = 0.f;
    // FeatureVector CSR (fv_nnodes < 0: none yet)
    int fv_nnodes = -1, fv_total = 0, fv_big = 0, fv_cap_node = 0, fv_cap_off = 0, fv_cap_idx = 0;
    uint32_t* fv_node = nullptr;
    int32_t* fv_off = nullptr;
    uint32_t* fv_idx = nullptr;
    // k_bow's single-pair offsets: kp_off {0, n}, node_off {0, fv_nnodes}, idx_off {0}
    long long* offs = nullptr;
    // the frame's grid prebuilt for the fused searches (k_grid_prebuild):
    // [0] every keypoint, [1] octave 0 (SearchForInitialization's F2); null
    // when the frame exceeds the fused forms' kFusedMaxN keypoints
    int* grid[2] = {nullptr, nullptr};
    int grid_cap[2] = {0, 0};
    ~orbm_dframe() {
        void* ps[] = {kps, desc, ur, scale, fv_node, fv_off, fv_idx, offs, grid[0], grid[1]};
        for (void* q : ps)
            if (q) (void)hipFree(q);
    }
};

namespace orbmi {

// grows a device array to at least cnt elements (contents not kept)
template <class T> static int grow_dev(T*& p, int& cap, size_t cnt) {
    cnt = std::max<size_t>(1, cnt);
    if (p && (size_t)cap >= cnt) return ORB_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc((void**)&p, cnt * sizeof(T)) != hipSuccess) return ORB_ERR_DEVICE;
    cap = (int)cnt;
    return ORB_OK;
}

// the two prebuilt grids of a dframe whose keypoints are in place (stream 0,
// ordered before every later search)
static int df_grids(orbm_dframe* df) {
    if (df->n > kFusedMaxN) {                      // (the fused forms refuse such a frame)
        for (int k = 0; k < 2; ++k) {
            if (df->grid[k]) (void)hipFree(df->grid[k]);
            df->grid[k] = nullptr;
            df->grid_cap[k] = 0;
        }
        return ORB_OK;
    }
    for (int k = 0; k < 2; ++k) {
        int rc;
        if ((rc = grow_dev(df->grid[k], df->grid_cap[k], (size_t)kGridInts + std::max(1, df->n)))) return rc;
        if (!df->grid[k]) return ORB_ERR_DEVICE;
        KLAUNCH(k_grid_prebuild, dim3(1), dim3(kFusedThreads), lds_grid_bytes(df->n), 0, df->kps, df->n, df->g,
                k ? 0 : -1, df->grid[k]);
    }
    return hipGetLastError() == hipSuccess ? ORB_OK : ORB_ERR_DEVICE;
}

static int df_offsets(orbm_dframe* df) {
    if (!df->offs && hipMalloc((void**)&df->offs, 8 * sizeof(long long)) != hipSuccess) return ORB_ERR_DEVICE;
    const long long o[5] = {0, df->n, 0, std::max(0, df->fv_nnodes), 0};
    return hipMemcpy(df->offs, o, sizeof(o), hipMemcpyHostToDevice) == hipSuccess ? ORB_OK : ORB_ERR_DEVICE;
}

// bounds, grid factors, u_right and scale factors of an orbm_frame
static int df_geometry(orbm_dframe* df, const orbm_frame* f, int n) {
    df->g = grid_params(f);
    df->max_x = f->max_x;
    df->max_y = f->max_y;
    df->has_ur = f->u_right != nullptr;
    df->has_scale = f->scale_factors != nullptr && f->nlevels > 0;
    df->nlevels = std::max(0, f->nlevels);
    int rc;
    if (df->has_ur) {
        if ((rc = grow_dev(df->ur, df->ur_cap, n))) return rc;
        if (n && hipMemcpy(df->ur, f->u_right, (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess) return ORB_ERR_DEVICE;
    }
    if (df->has_scale) {
        if ((rc = grow_dev(df->scale, df->scale_cap, df->nlevels))) return rc;
        if (hipMemcpy(df->scale, f->scale_factors, (size_t)df->nlevels * 4, hipMemcpyHostToDevice) != hipSuccess)
            return ORB_ERR_DEVICE;
    }
    return ORB_OK;
}

static int df_featvec(orbm_dframe* df, const orbm_featvec* fv) {
    if (!fv) return ORB_OK;
    if (fv->nnodes < 0 || (fv->nnodes && (!fv->node_ids || !fv->offsets || !fv->idx))) return ORB_ERR_PARAM;
    const int nn = fv->nnodes, tot = nn ? fv->offsets[nn] : 0;
    for (int i = 0; i < nn; ++i)
        if (fv->offsets[i + 1] < fv->offsets[i]) return ORB_ERR_PARAM;
    for (int i = 0; i < tot; ++i)
        if (fv->idx[i] >= (uint32_t)df->n) return ORB_ERR_PARAM;
    int rc;
    if ((rc = grow_dev(df->fv_node, df->fv_cap_node, nn)) || (rc = grow_dev(df->fv_off, df->fv_cap_off, nn + 1)) ||
        (rc = grow_dev(df->fv_idx, df->fv_cap_idx, tot)))
        return rc;
    if ((nn && hipMemcpy(df->fv_node, fv->node_ids, (size_t)nn * 4, hipMemcpyHostToDevice) != hipSuccess) ||
        hipMemcpy(df->fv_off, fv->offsets, (size_t)(nn + 1) * 4, hipMemcpyHostToDevice) != hipSuccess ||
        (tot && hipMemcpy(df->fv_idx, fv->idx, (size_t)tot * 4, hipMemcpyHostToDevice) != hipSuccess))
        return ORB_ERR_DEVICE;
    df->fv_nnodes = nn;
    df->fv_total = tot;
    df->fv_big = 0;                  // k_bow's large frame nodes (bow_big_nodes)
    for (int i = 0; i < nn; ++i) df->fv_big += fv->offsets[i + 1] - fv->offsets[i] > kBowRegChunks * kWave;
    return df_offsets(df);
}

// Per-thread, per-device state of the dframe searches that their kernels
// leave as they found it: the last-arriver ticket (0) and k_bow's match row
// (-1) and count (0).  A call that fails marks it dirty; the next one
// re-initialises it.
struct DfScratch {
    int dev = -1;
    unsigned* ticket = nullptr;
    int32_t* match = nullptr;              // [match_cap] then nmatches
    size_t match_cap = 0;
    bool dirty = true;
};
static DfScratch* df_scratch(int dev, size_t nmatch) {
    static thread_local std::vector<DfScratch>* v = new std::vector<DfScratch>();   // never destroyed at exit
    DfScratch* S = nullptr;
    for (auto& x : *v)
        if (x.dev == dev) S = &x;
    if (!S) {
        v->push_back(DfScratch{});
        S = &v->back();
        S->dev = dev;
    }
    if (!S->ticket && hipMalloc((void**)&S->ticket, 256) != hipSuccess) { S->ticket = nullptr; return nullptr; }
    if (!S->match || nmatch > S->match_cap) {
        if (S->match) (void)hipFree(S->match);
        S->match = nullptr;
        S->match_cap = 0;
        const size_t cap = std::max<size_t>(4096, nmatch);
        if (hipMalloc((void**)&S->match, (cap + 1) * 4) != hipSuccess) return nullptr;
        S->match_cap = cap;
        S->dirty = true;
    }
    if (S->dirty) {
        if (hipMemset(S->ticket, 0, 256) != hipSuccess || hipMemset(S->ticket + 1, 0xff, 4) != hipSuccess ||
            hipMemset(S->ticket + 2, 0, 8) != hipSuccess ||
            hipMemset(S->match, 0xff, S->match_cap * 4) != hipSuccess ||
            hipMemset(S->match + S->match_cap, 0, 4) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
            return nullptr;
        S->dirty = false;
    }
    return S;
}

// The per-call inputs of a dframe search, packed into one run of the pinned
// staging arena (16-byte aligned pieces): the kernel reads them through the
// run's device mapping and mirrors the run into HBM for its phase 2 (Mirror).
struct ZRun {
    char* h = nullptr;      // pinned staging
    char* m = nullptr;      // its device mapping
    char* dev = nullptr;    // the HBM mirror
    size_t len = 0, cap = 0;
    int begin(size_t total, bool mirror) {
        cap = (std::max<size_t>(16, total) + 255) & ~size_t(255);
        h = (char*)host_stage().get(cap);
        if (!h || hipHostGetDevicePointer((void**)&m, h, 0) != hipSuccess || !m) return ORB_ERR_DEVICE;
        if (mirror && !(dev = (char*)dev_arena().get(cap))) return ORB_ERR_DEVICE;
        len = 0;
        return ORB_OK;
    }
    static size_t piece(size_t bytes) { return (bytes + 15) & ~size_t(15); }
    template <class T> const T* add(const T* src, size_t cnt) {
        const size_t b = cnt * sizeof(T);
        char* q = h + len;
        if (b) std::memcpy(q, src, b);
        const T* r = (const T*)(m + len);
        len += piece(b);
        return r;
    }
    Mirror mirror() const {
        Mirror x;
        if (!dev) return x;
        x.src = (const uint4*)m;
        x.dst = (uint4*)dev;
        x.n16 = (long long)(len / 16);
        x.delta = (long long)((uintptr_t)dev - (uintptr_t)m);
        return x;
    }
};

// The device of a dframe search (every dframe on one device), current on return.
static int df_device(std::initializer_list<const orbm_dframe*> dfs) {
    int dev = -1;
    for (const orbm_dframe* d : dfs) {
        if (!d) return ORB_ERR_PARAM;
        if (dev >= 0 && d->device != dev) return ORB_ERR_PARAM;
        dev = d->device;
    }
    if (hipSetDevice(dev) != hipSuccess) return ORB_ERR_DEVICE;
    arena_reset();
    return ORB_OK;
}

// The fused projection search on a dframe (k_proj_fused, part 0, inputs
// read zero-copy and mirrored): run_proj's fused form with the frame in HBM.
static int run_proj_dframe(ProjArgs& a, const orbm_dframe* f, ZRun& z, const int32_t* owner_m, int32_t* owner) {
    const int n = f->n;
    if (n > kFusedMaxN || a.nq > kFusedMaxQ || f->nlevels > 8 || proj_fused_lds(n, a.nq, false) > kCuLds)
        return ORB_ERR_UNSUPPORTED;
    DfScratch* S = df_scratch(f->device, 0);
    if (!S) return ORB_ERR_DEVICE;
    a.kps = f->kps; a.desc = f->desc; a.n = n; a.u_right = f->has_ur ? f->ur : nullptr; a.scale = f->scale;
    a.g = f->g; a.owner = nullptr; a.nmatches = nullptr;
    const size_t gb = lds_grid_bytes(n);
    const int use_grid = proj_fused_lds(n, a.nq, false) + gb <= kCuLds;
    const int lds_lists = proj_fused_lds(n, a.nq, true) + (use_grid ? gb : 0) <= kCuLds;
    const size_t lds = proj_fused_lds(n, a.nq, lds_lists != 0) + (use_grid ? gb : 0);
    uint32_t* lists = (uint32_t*)dev_arena().get((size_t)std::max(1, a.nq) * kProjK * 4);
    int* cnt = (int*)dev_arena().get((size_t)std::max(1, a.nq) * 4);
    OutBlock out;
    if (!lists || !cnt || out.alloc((size_t)n + 13, true)) return ORB_ERR_DEVICE;
    const int nblk = std::max(1, (a.nq + kFusedThreads / kWave - 1) / (kFusedThreads / kWave));
    S->dirty = true;                   // until the kernel has reset the ticket
    KLAUNCH(k_proj_fused, dim3(nblk), dim3(kFusedThreads), lds, 0, a, proj_bound(a), lists, cnt, S->ticket, owner_m,
            out.d, lds_lists, use_grid, 0, out.flag, out.seq, z.mirror(), use_grid ? f->grid[0] : nullptr);
    ORB_CHECK(hipGetLastError());
    std::vector<int32_t> res((size_t)n + 13);
    ORB_CHECK(out.fetch(res.data(), res.size()));
    S->dirty = false;
    if (n) std::memcpy(owner, res.data() + 1, (size_t)n * sizeof(int32_t));
    std::memcpy(proj_stats(), res.data() + n + 1, 12 * sizeof(int32_t));
    return res[0];
}

}  // namespace orbmi

using namespace orbmi;

static std::atomic<int> g_debug_opt[ORB_OPT_COUNT];

int orbmi::debug_opt(int option) {
    return option >= 0 && option < ORB_OPT_COUNT ? g_debug_opt[option].load(std::memory_order_relaxed) : 0;
}

extern "C" {

int orb_debug_set_option(int option, int value) {
    if (option < 0 || option >= ORB_OPT_COUNT) return ORB_ERR_PARAM;
    g_debug_opt[option].store(value, std::memory_order_relaxed);
    return ORB_OK;
}

int orbm_release_scratch(void* stream, int all) {
    if (device_ok() != ORB_OK) return ORB_ERR_DEVICE;
    auto& L = scratch_sets();
    int dev = 0;
    (void)hipGetDevice(&dev);
    int rc = ORB_OK;
    for (auto it = L.begin(); it != L.end();) {
        if (all || (it->dev == dev && it->st == (hipStream_t)stream)) {
            if (!scratch_free(*it)) {               // its stream's work did not finish cleanly: keep it
                rc = ORB_ERR_DEVICE;
                ++it;
                continue;
            }
            it = L.erase(it);
        } else {
            ++it;
        }
    }
    return rc;
}

int orb_debug_get_option(int option) {
    return option >= 0 && option < ORB_OPT_COUNT ? g_debug_opt[option].load(std::memory_order_relaxed) : -1;
}


int orbm_debug_proj_stats(int32_t* out12) {
    if (!out12) return ORB_ERR_PARAM;
    std::memcpy(out12, proj_stats(), 12 * sizeof(int32_t));
    return ORB_OK;
}

int orbm_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    // host inline utility (Frame.cc:886, MapPoint.cc:377 call it on single pairs)
    int d = 0;
    for (int i = 0; i < 32; ++i) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

int orbm_search_for_initialization(const orbm_frame* f1, const orbm_frame* f2, float* prev_xy, int window,
                                   float nnratio, int check_ori, int32_t* matches12) {
    if (!f1 || !f2 || !prev_xy || !matches12) return ORB_ERR_PARAM;
    if (device_ok()) return ORB_ERR_DEVICE;
    if (f1->n > 0xffff || f2->n > 0xffff) return ORB_ERR_UNSUPPORTED;
    // fused single launch: one coalesced upload, one launch, one download of
    // [nmatches, matches12[n1], prev_xy[n1][2]]
    const int sform = debug_opt(ORB_OPT_SFI_FORM);
    if ((sform == 0 || sform == 2 || sform == 3) && f1->n <= kFusedMaxN && f2->n <= kFusedMaxN && nnratio >= 0.2f &&
        sfi_fused_lds(f1->n, f2->n) <= kCuLds) {
        SfiFusedArgs a{};
        DBuf<orb_keypoint> k1, k2; DBuf<uint8_t> d1, d2; DBuf<float> pv;
        DBuf<uint32_t> lists; DBuf<int> cnt; DBuf<unsigned> ticket; OutBlock out;
        const unsigned zero = 0;
        const int n1 = f1->n, n2 = f2->n;
        int rc;
        if ((rc = k1.put(f1->kps, n1)) || (rc = d1.put(f1->desc, (size_t)n1 * 32)) || (rc = k2.put(f2->kps, n2)) ||
            (rc = d2.put(f2->desc, (size_t)n2 * 32)) || (rc = pv.put(prev_xy, (size_t)2 * n1)) ||
            (rc = ticket.put(&zero, 1)) || (rc = lists.alloc((size_t)std::max(1, n1) * kTopK)) ||
            (rc = cnt.alloc(std::max(1, n1))) || (rc = out.alloc((size_t)13 + 3 * n1)))
            return rc;
        a.k1 = k1.p; a.d1 = d1.p; a.n1 = n1; a.k2 = k2.p; a.d2 = d2.p; a.n2 = n2; a.prev = pv.p;
        a.g = grid_params(f2); a.window = (float)window; a.ratio = nnratio; a.check_ori = check_ori;
        // a best above TH_LOW is rejected; a second d with (float)d * ratio > TH_LOW
        // cannot fail the ratio test of an accepted best
        int bound = kThLow;
        while (bound < 255 && (float)(bound + 1) * nnratio <= (float)kThLow) ++bound;
        a.bound = bound;
        const int nblk = std::max(1, (n1 + kFusedThreads / kWave - 1) / (kFusedThreads / kWave));
        // F2's level-0 grid in LDS (form 2: none, every window scans F2)
        const size_t gb = lds_grid_bytes(n2);
        const int use_grid = sform != 2 && sfi_fused_lds(n1, n2) + gb <= kCuLds;
        const size_t lds = sfi_fused_lds(n1, n2) + (use_grid ? gb : 0);
        if (sform == 3) {      // phase 1, then phase 2 as a one-block launch (no ticket)
            KLAUNCH(k_sfi_fused, dim3(nblk), dim3(kFusedThreads), lds, 0, a, lists.p, cnt.p, ticket.p, out.d,
                    use_grid, 1, (int*)nullptr, 0, Mirror{}, (const int*)nullptr);
            KLAUNCH(k_sfi_fused, dim3(1), dim3(kFusedThreads), lds, 0, a, lists.p, cnt.p, ticket.p, out.d, use_grid, 2,
                    out.flag, out.seq, Mirror{}, (const int*)nullptr);
        } else {
            KLAUNCH(k_sfi_fused, dim3(nblk), dim3(kFusedThreads), lds, 0, a, lists.p, cnt.p, ticket.p, out.d,
                    use_grid, 0, out.flag, out.seq, Mirror{}, (const int*)nullptr);
        }
        ORB_CHECK(hipGetLastError());
        std::vector<int32_t> res((size_t)13 + 3 * n1);
        ORB_CHECK(out.fetch(res.data(), res.size()));
        std::memcpy(proj_stats(), res.data() + 1 + 3 * n1, 12 * sizeof(int32_t));
        if (n1) {
            std::memcpy(matches12, res.data() + 1, (size_t)n1 * sizeof(int32_t));
            std::memcpy(prev_xy, res.data() + 1 + n1, (size_t)n1 * 2 * sizeof(float));
        }
        return res[0];
    }
    // both frames share one [2][cap] layout
    const int cap = std::max(1, std::max(f1->n, f2->n));
    DBuf<orb_keypoint> kps; DBuf<uint8_t> desc; DBuf<int> n; DBuf<uint32_t> sorted; DBuf<int> count;
    DBuf<int> pf; DBuf<float> prev_in, prev_out; DBuf<int32_t> m; DBuf<int32_t> nm;
    DBuf<uint32_t> topk; DBuf<int> ncand;
    int rc;
    if ((rc = kps.alloc(2 * cap)) || (rc = desc.alloc((size_t)2 * cap * 32)) || (rc = sorted.alloc(2 * cap)) ||
        (rc = count.alloc(2)) || (rc = m.alloc(cap)) || (rc = nm.alloc(1)) || (rc = prev_out.alloc((size_t)2 * cap)) ||
        (rc = topk.alloc((size_t)cap * kTopK)) || (rc = ncand.alloc(cap)))
        return rc;
    const int ns[2] = {f1->n, f2->n};
    const int pfs[2] = {0, 1};
    if ((rc = n.put(ns, 2)) || (rc = pf.put(pfs, 2))) return rc;
    std::vector<float> pv((size_t)2 * cap, 0.f);
    std::memcpy(pv.data(), prev_xy, sizeof(float) * 2 * f1->n);
    if ((rc = prev_in.put(pv.data(), pv.size()))) return rc;
    if (f1->n) {
        ORB_CHECK(h2d(kps.p, f1->kps, f1->n * sizeof(orb_keypoint)));
        ORB_CHECK(h2d(desc.p, f1->desc, (size_t)f1->n * 32));
    }
    if (f2->n) {
        ORB_CHECK(h2d(kps.p + cap, f2->kps, f2->n * sizeof(orb_keypoint)));
        ORB_CHECK(h2d(desc.p + (size_t)cap * 32, f2->desc, (size_t)f2->n * 32));
    }
    const GridParams g = grid_params(f2);
    const int sc = pow2_at_least(cap);
    DBuf<uint32_t> l0s; DBuf<int> l0c;
    if ((rc = l0s.alloc((size_t)2 * cap)) || (rc = l0c.alloc(2))) return rc;
    if (grid_cs_lds(cap) <= 160 * 1024)
        KLAUNCH(k_grid_cs, dim3(2), dim3(256), grid_cs_lds(cap), 0, kps.p, n.p, cap, g, sorted.p, count.p,
                           (int*)nullptr, l0s.p, l0c.p);
    else
        KLAUNCH(k_grid, dim3(2), dim3(256), sc * sizeof(uint32_t), 0, kps.p, n.p, cap, g, sorted.p,
                           count.p, sc, l0s.p, l0c.p);
    SfiArgs a;
    a.kps = kps.p; a.desc = desc.p; a.n = n.p; a.cap = cap; a.gsorted = l0s.p; a.gcount = l0c.p;
    a.pair_f1 = pf.p; a.pair_f2 = pf.p + 1; a.prev_in = prev_in.p; a.prev_out = prev_out.p;
    a.g = g; a.window = (float)window; a.ratio = nnratio; a.check_ori = check_ori;
    a.matches = m.p; a.nmatches = nm.p; a.topk = topk.p; a.ncand = ncand.p;
    if ((rc = launch_sfi(a, 1, 0))) return rc;
    ORB_CHECK(hipGetLastError());
    int32_t res = 0;
    ORB_CHECK(d2h(&res, nm.p, 4));
    if (f1->n) {
        ORB_CHECK(d2h(matches12, m.p, f1->n * 4));
        ORB_CHECK(d2h(prev_xy, prev_out.p, f1->n * 8));
    }
    return res;
}

int orbm_search_for_initialization_batch_device(int nframes, const orb_keypoint* d_kps, const uint8_t* d_desc,
                                                const int32_t* d_n, int cap, float min_x, float max_x, float min_y,
                                                float max_y, float grid_inv_w, float grid_inv_h, int window,
                                                float nnratio, int check_ori, int32_t* d_matches, int32_t* d_nmatches,
                                                void* stream) {
    (void)max_x; (void)max_y;
    if (nframes < 2 || cap <= 0 || cap > 0xffff) return ORB_ERR_PARAM;
    hipStream_t st = (hipStream_t)stream;
    struct Scratch : ScratchBase { PBuf<uint32_t> sorted, topk, l0s; PBuf<int> count, pf, ncand, l0c; int pf_frames = 0; };
    Scratch* Sp = stream_scratch<Scratch>(st);
    if (!Sp) return ORB_ERR_DEVICE;
    Scratch& S = *Sp;
    PBuf<uint32_t>&sorted = S.sorted, &topk = S.topk, &l0s = S.l0s;
    PBuf<int>&count = S.count, &pf = S.pf, &ncand = S.ncand, &l0c = S.l0c;
    int& pf_frames = S.pf_frames;
    int rc;
    if ((rc = sorted.alloc((size_t)nframes * cap)) || (rc = count.alloc(nframes)) ||
        (rc = topk.alloc((size_t)nframes * cap * kTopK)) || (rc = ncand.alloc((size_t)nframes * cap)) ||
        (rc = l0s.alloc((size_t)nframes * cap)) || (rc = l0c.alloc(nframes)))
        return rc;
    if (pf_frames < nframes) {
        std::vector<int> idx(nframes);
        for (int i = 0; i < nframes; ++i) idx[i] = i;
        if ((rc = pf.put(idx.data(), nframes, st))) return rc;
        ORB_CHECK(hipStreamSynchronize(st));           // (idx is pageable and leaves scope)
        pf_frames = nframes;
    }
    const GridParams g{min_x, min_y, grid_inv_w, grid_inv_h};
    const int sc = pow2_at_least(cap);
    if (grid_cs_lds(cap) <= 160 * 1024)
        KLAUNCH(k_grid_cs, dim3(nframes), dim3(256), grid_cs_lds(cap), st, d_kps, d_n, cap, g, sorted.p,
                           count.p, (int*)nullptr, l0s.p, l0c.p);
    else
        KLAUNCH(k_grid, dim3(nframes), dim3(256), sc * sizeof(uint32_t), st, d_kps, d_n, cap, g,
                           sorted.p, count.p, sc, l0s.p, l0c.p);
    SfiArgs a;
    a.kps = d_kps; a.desc = d_desc; a.n = d_n; a.cap = cap; a.gsorted = l0s.p; a.gcount = l0c.p;
    a.pair_f1 = pf.p; a.pair_f2 = pf.p + 1; a.prev_in = nullptr; a.prev_out = nullptr;
    a.g = g; a.window = (float)window; a.ratio = nnratio; a.check_ori = check_ori;
    a.matches = d_matches; a.nmatches = d_nmatches; a.topk = topk.p; a.ncand = ncand.p;
    if ((rc = launch_sfi(a, nframes - 1, st))) return rc;
    ORB_CHECK(hipGetLastError());
    return scratch_used(st);
}

// Frame nodes the large-node blocks take (host FeatureVector).
static int bow_big_nodes(const orbm_featvec* fv) {
    int n = 0;
    for (int i = 0; i < fv->nnodes; ++i) n += fv->offsets[i + 1] - fv->offsets[i] > kBowRegChunks * kWave;
    return n;
}

static int bow_host(const orbm_frame* kf, const orbm_featvec* kfv, const uint8_t* kf_valid, const orbm_frame* f,
                    const orbm_featvec* ffv, int f_nleft, float nnratio, int check_ori, int32_t* match_f) {
    if (!kf || !kfv || !kf_valid || !f || !ffv || !match_f) return ORB_ERR_PARAM;
    if (device_ok()) return ORB_ERR_DEVICE;
    int rc;
    DBuf<orb_keypoint> kk, fk; DBuf<uint8_t> kd, fd, kvv; DBuf<uint32_t> kn, ki, fn, fi; DBuf<int> ko, fo;
    DBuf<long long> kpo, nodo, idxo; DBuf<int32_t> m;
    const long long kp_off[2] = {0, kf->n}, node_off[2] = {0, kfv->nnodes}, idx_off[1] = {0};
    if ((rc = kk.put(kf->kps, kf->n)) || (rc = kd.put(kf->desc, (size_t)kf->n * 32)) || (rc = kvv.put(kf_valid, kf->n)) ||
        (rc = kn.put(kfv->node_ids, kfv->nnodes)) || (rc = ko.put(kfv->offsets, kfv->nnodes + 1)) ||
        (rc = ki.put(kfv->idx, kfv->offsets[kfv->nnodes])) || (rc = fk.put(f->kps, f->n)) ||
        (rc = fd.put(f->desc, (size_t)f->n * 32)) || (rc = fn.put(ffv->node_ids, ffv->nnodes)) ||
        (rc = fo.put(ffv->offsets, ffv->nnodes + 1)) || (rc = fi.put(ffv->idx, ffv->offsets[ffv->nnodes])) ||
        (rc = kpo.put(kp_off, 2)) || (rc = nodo.put(node_off, 2)) || (rc = idxo.put(idx_off, 1)))
        return rc;
    // match[n] = -1 and nmatches = 0 go up with the inputs, and come back as one
    // download; the last k_bow block runs the rotation filter (one launch)
    // (the zero-copy modes: the last block copies the finished row and count
    // into the pinned result block)
    std::vector<int32_t> init((size_t)f->n + 1, -1);
    init[f->n] = 0;
    const unsigned zero = 0;
    DBuf<unsigned> ticket;
    OutBlock out;
    if ((rc = ticket.put(&zero, 1)) || (rc = m.put(init.data(), init.size())) || (rc = out.alloc(init.size())))
        return rc;
    if (!out.h) out.d = m.p;          // ORB_OPT_HOST_OUT 2: the row itself comes back by d2h
    BowArgs a{};
    a.kf_kps = kk.p; a.kf_desc = kd.p; a.kf_valid = kvv.p; a.kp_off = kpo.p;
    a.kf_node = kn.p; a.kf_off = ko.p; a.kf_idx = ki.p; a.node_off = nodo.p; a.idx_off = idxo.p;
    a.f_kps = fk.p; a.f_desc = fd.p; a.f_n = f->n; a.f_node = fn.p; a.f_off = fo.p; a.f_idx = fi.p;
    a.f_nnodes = ffv->nnodes; a.ratio = nnratio; a.check_ori = check_ori; a.match = m.p; a.nmatches = m.p + f->n;
    a.f_nleft = f_nleft; a.fin_ticket = ticket.p;
    a.single_nodes = kfv->nnodes;      // (kp_off, node_off, idx_off above all start at 0)
    if (out.h) { a.host_out = out.d; a.done = out.flag; a.seq = out.seq; }
    if ((rc = launch_bow(a, 1, 0, bow_big_nodes(ffv), kfv->nnodes))) return rc;
    ORB_CHECK(out.fetch(init.data(), init.size()));
    if (f->n) std::memcpy(match_f, init.data(), (size_t)f->n * 4);
    return init[f->n];
}

int orbm_search_by_bow(const orbm_frame* kf, const orbm_featvec* kfv, const uint8_t* kf_valid, const orbm_frame* f,
                       const orbm_featvec* ffv, float nnratio, int check_ori, int32_t* match_f) {
    return bow_host(kf, kfv, kf_valid, f, ffv, -1, nnratio, check_ori, match_f);
}

int orbm_search_by_bow_fisheye(const orbm_frame* kf, const orbm_featvec* kfv, const uint8_t* kf_valid,
                               const orbm_frame* f, const orbm_featvec* ffv, int f_nleft, float nnratio,
                               int check_ori, int32_t* match_f) {
    if (!f || f_nleft < 0 || f_nleft > f->n) return ORB_ERR_PARAM;
    return bow_host(kf, kfv, kf_valid, f, ffv, f_nleft, nnratio, check_ori, match_f);
}

int orbm_search_by_bow_many(int nkf, const orbm_frame* const* kfs, const orbm_featvec* const* kfvs,
                            const uint8_t* const* kf_valid, const orbm_frame* f, const orbm_featvec* ffv, float nnratio,
                            int check_ori, int32_t* match_f, int32_t* counts) {
    if (nkf < 0 || (nkf && (!kfs || !kfvs || !kf_valid)) || !f || !ffv || !match_f || !counts) return ORB_ERR_PARAM;
    for (int i = 0; i < nkf; ++i)
        if (!kfs[i] || !kfvs[i] || !kf_valid[i] || kfs[i]->n < 0) return ORB_ERR_PARAM;
    if (nkf == 0) return ORB_OK;
    if (device_ok()) return ORB_ERR_DEVICE;
    // the candidates packed like orbm_kf_map_device: features, FeatureVector
    // nodes and per-keyframe CSR offsets concatenated
    std::vector<long long> kp_off(nkf + 1, 0), node_off(nkf + 1, 0), idx_off(nkf, 0);
    long long nidx = 0;
    for (int i = 0; i < nkf; ++i) {
        kp_off[i + 1] = kp_off[i] + kfs[i]->n;
        node_off[i + 1] = node_off[i] + kfvs[i]->nnodes;
        idx_off[i] = nidx;
        nidx += kfvs[i]->nnodes ? kfvs[i]->offsets[kfvs[i]->nnodes] : 0;
    }
    const long long nkp = kp_off[nkf], nnode = node_off[nkf];
    std::vector<orb_keypoint> kk((size_t)std::max(1LL, nkp));
    std::vector<uint8_t> kd((size_t)std::max(1LL, nkp) * 32), kv((size_t)std::max(1LL, nkp));
    std::vector<uint32_t> kn((size_t)std::max(1LL, nnode)), ki((size_t)std::max(1LL, nidx));
    std::vector<int> ko((size_t)(nnode + nkf));
    for (int i = 0; i < nkf; ++i) {
        const orbm_frame* kf = kfs[i];
        const orbm_featvec* fv = kfvs[i];
        std::copy(kf->kps, kf->kps + kf->n, kk.begin() + kp_off[i]);
        if (kf->n) {
            std::memcpy(kd.data() + kp_off[i] * 32, kf->desc, (size_t)kf->n * 32);
            std::memcpy(kv.data() + kp_off[i], kf_valid[i], (size_t)kf->n);
        }
        std::copy(fv->node_ids, fv->node_ids + fv->nnodes, kn.begin() + node_off[i]);
        for (int j = 0; j <= fv->nnodes; ++j) ko[(size_t)(node_off[i] + i + j)] = fv->nnodes ? fv->offsets[j] : 0;
        const int ni = fv->nnodes ? fv->offsets[fv->nnodes] : 0;
        std::copy(fv->idx, fv->idx + ni, ki.begin() + idx_off[i]);
    }
    int rc;
    DBuf<orb_keypoint> dk, fk; DBuf<uint8_t> dd, dv, fd; DBuf<uint32_t> dn, di, fn, fi; DBuf<int> dof, fo;
    DBuf<long long> dkpo, dnodo, didxo; DBuf<int32_t> out;
    const int fidx = ffv->nnodes ? ffv->offsets[ffv->nnodes] : 0;
    const int zero = 0;
    if ((rc = dk.put(kk.data(), kk.size())) || (rc = dd.put(kd.data(), kd.size())) || (rc = dv.put(kv.data(), kv.size())) ||
        (rc = dn.put(kn.data(), kn.size())) || (rc = dof.put(ko.data(), ko.size())) || (rc = di.put(ki.data(), ki.size())) ||
        (rc = dkpo.put(kp_off.data(), kp_off.size())) || (rc = dnodo.put(node_off.data(), node_off.size())) ||
        (rc = didxo.put(idx_off.data(), idx_off.size())) || (rc = fk.put(f->kps, f->n)) ||
        (rc = fd.put(f->desc, (size_t)f->n * 32)) || (rc = fn.put(ffv->node_ids, ffv->nnodes)) ||
        (rc = fo.put(ffv->nnodes ? ffv->offsets : &zero, ffv->nnodes + 1)) || (rc = fi.put(ffv->idx, fidx)) ||
        (rc = out.alloc((size_t)nkf * f->n + nkf)))
        return rc;
    BowArgs a{};
    a.kf_kps = dk.p; a.kf_desc = dd.p; a.kf_valid = dv.p; a.kp_off = dkpo.p;
    a.kf_node = dn.p; a.kf_off = dof.p; a.kf_idx = di.p; a.node_off = dnodo.p; a.idx_off = didxo.p;
    a.f_kps = fk.p; a.f_desc = fd.p; a.f_n = f->n; a.f_node = fn.p; a.f_off = fo.p; a.f_idx = fi.p;
    a.f_nnodes = ffv->nnodes; a.ratio = nnratio; a.check_ori = check_ori;
    a.match = out.p; a.nmatches = out.p + (size_t)nkf * f->n;
    if ((rc = launch_bow(a, nkf, 0, bow_big_nodes(ffv), nnode))) return rc;
    std::vector<int32_t> res((size_t)nkf * f->n + nkf);
    ORB_CHECK(d2h(res.data(), out.p, res.size() * sizeof(int32_t)));
    std::memcpy(match_f, res.data(), (size_t)nkf * f->n * sizeof(int32_t));
    std::memcpy(counts, res.data() + (size_t)nkf * f->n, (size_t)nkf * sizeof(int32_t));
    return ORB_OK;
}

// G: (pair, KF node) entries of the map, nfv: its FeatureVector entries (host
// totals of the resident map: scratch is sized without reading the device).
static int launch_bow_kf(BowArgs& a, int npairs, long long G, long long nfv, hipStream_t st) {
    struct Scratch : ScratchBase {
        PBuf<int> g_fl, g_off, g_pr, bstart, gstart, g_rank, perm, chunk_node, node_n;
        PBuf<unsigned long long> bgcount;
        PBuf<uint32_t> slot_src, slot_pos;
        PBuf<uint16_t> claim;
        PBuf<bowk_list> lists;
        PBuf<bowk_v4i> fexp;
    };
    Scratch* Sp = stream_scratch<Scratch>(st);
    if (!Sp) return ORB_ERR_DEVICE;
    Scratch& S = *Sp;
    PBuf<int>&g_fl = S.g_fl, &g_off = S.g_off, &g_pr = S.g_pr, &bstart = S.bstart, &gstart = S.gstart,
        &g_rank = S.g_rank, &perm = S.perm, &chunk_node = S.chunk_node, &node_n = S.node_n;
    PBuf<unsigned long long>& bgcount = S.bgcount;
    PBuf<uint32_t>&slot_src = S.slot_src, &slot_pos = S.slot_pos;
    PBuf<uint16_t>& claim = S.claim;
    PBuf<bowk_list>& lists = S.lists;
    PBuf<bowk_v4i>& fexp = S.fexp;
    const int nsub = a.f_nnodes <= 1024 ? 64 : 1;
    a.npairs = npairs;
    // every g's run rounded up to 8 slots, every bucket to 64
    const long long slots = nfv + 7 * G + (long long)kWave * a.f_nnodes;
    // the resolve form: every thread's claimed positions in an LDS bitmap when a
    // bitmap over every frame position fits 64 threads' LDS (nodes of > 512
    // features then take the BIG form); its claims then go beside the slots and
    // k_bowk_final builds the rows
    const int words = (a.f_n + 31) / 32, bp = a.f_n > 32 * kBowLaneWords ? (words | 1) : 0;
    const size_t big_lds = (size_t)64 * bp * sizeof(uint32_t);
    const bool all_lds = big_lds <= 64 * 1024 && !debug_opt(ORB_OPT_BOWK_BIG);
    const int big_pitch = all_lds ? bp : 0;
    // (k_bowk_final packs a KF feature index, < 2^26 by the C ABI's contract,
    // with its bin; the map's FeatureVector total bounds it where the host
    // knows it: a larger map takes k_bow_final)
    const bool claims = all_lds && a.f_n <= kBowkRow && !a.out12 && !a.f_valid && nfv < (1LL << 26);
    // every LDS-sized launch of the sequence checked before the first is
    // queued: a refusal half-way would leave queued work on scratch that
    // scratch_used() below would not cover
    if (!lds_fits(reinterpret_cast<const void*>(&k_bowk_scan), (size_t)2 * a.f_nnodes * sizeof(int)) ||
        (big_pitch && !lds_fits(reinterpret_cast<const void*>(&k_bowk_resolve_lane<true, true>), big_lds)) ||
        (claims && !lds_fits(reinterpret_cast<const void*>(&k_bowk_final), (size_t)a.f_n * 4)))
        return ORB_ERR_UNSUPPORTED;
    int rc;
    if ((rc = g_fl.alloc(G)) || (rc = g_off.alloc(G)) || (rc = g_pr.alloc(G)) || (rc = bgcount.alloc((size_t)a.f_nnodes * nsub)) ||
        (rc = bstart.alloc(a.f_nnodes + 1)) || (rc = slot_src.alloc(slots)) || (rc = lists.alloc(slots)) ||
        (rc = gstart.alloc(a.f_nnodes + 1)) || (rc = g_rank.alloc(G)) ||
        (rc = perm.alloc(G)) || (rc = fexp.alloc((size_t)std::max(1, a.f_n) * 16)) ||
        (rc = chunk_node.alloc(slots / 32 + 1)) || (rc = node_n.alloc(a.f_nnodes + 1)) || (a.kf_fvdesc && (rc = slot_pos.alloc(slots))) ||
        (claims && (rc = claim.alloc(slots))))
        return rc;
    BowKArgs k;
    k.b = a; k.G = G; k.g_fl = g_fl.p; k.g_off = g_off.p; k.g_pr = g_pr.p; k.bgcount = bgcount.p; k.nsub = nsub; k.node_n = node_n.p; k.bstart = bstart.p;
    k.slot_src = slot_src.p; k.lists = lists.p;
    k.gstart = gstart.p; k.g_rank = g_rank.p; k.perm = perm.p; k.chunk_node = chunk_node.p;
    k.slot_pos = slot_pos.p;
    k.claim = claims ? claim.p : nullptr;
    ORB_CHECK(flush_uploads());
    ORB_CHECK(hipMemsetAsync(bgcount.p, 0, (size_t)a.f_nnodes * nsub * sizeof(unsigned long long), st));
    if (!claims) {                                   // (k_bowk_final writes every row and count)
        const long long nmf = (long long)npairs * a.f_n;
        const int ib = (int)std::min<long long>(4096, std::max<long long>(1, (nmf + 1023) / 1024));
        KLAUNCH(k_bow_init, dim3(ib), dim3(256), 0, st, a);
    }
    const unsigned gb = (unsigned)((G + 255) / 256);
    KLAUNCH(k_bowk_map, dim3(npairs), dim3(256), 0, st, k);
    KLAUNCH(k_bowk_scan, dim3(1), dim3(1024), (size_t)2 * a.f_nnodes * sizeof(int), st, k);
    KLAUNCH(k_bowk_fill, dim3(npairs), dim3(256), 0, st, k);
    KLAUNCH(k_bowk_chunks, dim3(a.f_nnodes), dim3(256), 0, st, k);
    KLAUNCH(k_bowk_expand, dim3((unsigned)((16 * a.f_n + 255) / 256)), dim3(256), 0, st, a.f_desc, a.f_idx,
            a.f_off + a.f_nnodes, fexp.p);
    // (measured and dropped, DESIGN.md §5: the VALU top-4 pass, two 32-column
    // keyframe sets per MFMA wave, a wave-walk resolve)
    // (measured and dropped in round 4: persistent blocks over the whole grid,
    // 3.1-3.2 ms; blocks of 2 / 4 consecutive items with the next item's
    // descriptors prefetched, 2.88 / 2.78 vs 2.51 ms)
    KLAUNCH(k_bowk_topk_mfma<1>, dim3((unsigned)((slots + 127) / 128)), dim3(256), 0, st, k, fexp.p);
    if (all_lds) {
        KLAUNCH((k_bowk_resolve_lane<false, true>), dim3(gb), dim3(256), 0, st, k, big_pitch);
        if (big_pitch)
            KLAUNCH((k_bowk_resolve_lane<true, true>), dim3((unsigned)((G + 63) / 64)), dim3(64), big_lds, st, k,
                    big_pitch);
    } else {
        KLAUNCH((k_bowk_resolve_lane<false, false>), dim3(gb), dim3(256), 0, st, k, 0);
    }
    if (claims) KLAUNCH(k_bowk_final, dim3(npairs), dim3(256), (size_t)a.f_n * 4, st, k);
    else KLAUNCH(k_bow_final, dim3(npairs), dim3(256), 0, st, a);
    if (hipGetLastError() != hipSuccess) return ORB_ERR_DEVICE;
    return scratch_used(st);
}

int orbm_kf_map_fv_desc(const orbm_kf_map_device* map, uint8_t* d_fv_desc, void* stream) {
    if (!map || !d_fv_desc || map->nkf < 0) return ORB_ERR_PARAM;
    if (map->nkf == 0) return ORB_OK;
    hipStream_t st = (hipStream_t)stream;
    KLAUNCH(k_fv_desc, dim3(map->nkf), dim3(256), 0, st, map->desc, (const long long*)map->kp_off, map->fv_off,
            map->fv_idx, (const long long*)map->fv_node_off, (const long long*)map->fv_idx_off, d_fv_desc);
    return hipGetLastError() == hipSuccess ? ORB_OK : ORB_ERR_DEVICE;
}

int orbm_kf_map_fv_angle(const orbm_kf_map_device* map, float* d_fv_angle, void* stream) {
    if (!map || !d_fv_angle || map->nkf < 0) return ORB_ERR_PARAM;
    if (map->nkf == 0) return ORB_OK;
    hipStream_t st = (hipStream_t)stream;
    KLAUNCH(k_fv_angle, dim3(map->nkf), dim3(256), 0, st, map->kps, (const long long*)map->kp_off, map->fv_off,
            map->fv_idx, (const long long*)map->fv_node_off, (const long long*)map->fv_idx_off, d_fv_angle);
    return hipGetLastError() == hipSuccess ? ORB_OK : ORB_ERR_DEVICE;
}

int orbm_search_by_bow_batch_device(const orbm_kf_map_device* map, const orbm_frame* f, const orbm_featvec* ffv,
                                    float nnratio, int check_ori, int32_t* d_match, int32_t* d_nmatches, void* stream) {
    if (!map || !f || !ffv || !d_match || !d_nmatches || map->nkf < 0) return ORB_ERR_PARAM;
    if (map->nkf == 0) return ORB_OK;
    BowArgs a{};
    a.kf_kps = map->kps; a.kf_desc = map->desc; a.kf_valid = map->valid; a.kp_off = (const long long*)map->kp_off;
    a.kf_node = map->fv_node; a.kf_off = map->fv_off; a.kf_idx = map->fv_idx;
    a.node_off = (const long long*)map->fv_node_off; a.idx_off = (const long long*)map->fv_idx_off;
    a.kf_fvdesc = map->n_fv_total < 0xffffffffll ? map->fv_desc : nullptr;
    a.kf_fvangle = map->fv_angle;
    a.f_kps = f->kps; a.f_desc = f->desc; a.f_n = f->n; a.f_node = ffv->node_ids; a.f_off = ffv->offsets;
    a.f_idx = ffv->idx; a.f_nnodes = ffv->nnodes; a.ratio = nnratio; a.check_ori = check_ori;
    a.match = d_match; a.nmatches = d_nmatches;
    // the lane-per-KF-feature search (k_bowk_*) when the map carries its totals
    // (6.7 vs 7.1 ms per 10k-keyframe query); ORB_OPT_BOW_FORM
    // 1 selects k_bow (A/B, tests)
    // (k_bowk_scan holds two ints per frame node in LDS: 20,000 nodes = 160 KB
    // less its static scratch; beyond that k_bow runs)
    if (map->n_nodes_total > 0 && map->n_fv_total > 0 && f->n <= 0xffff && ffv->nnodes > 0 &&
        ffv->nnodes <= 20000 && debug_opt(ORB_OPT_BOW_FORM) != 1)
        return launch_bow_kf(a, map->nkf, map->n_nodes_total, map->n_fv_total, (hipStream_t)stream);
    return launch_bow(a, map->nkf, (hipStream_t)stream);
}

// The projection searches' device part.  df holds the uploaded frame (no grid
// yet).  Default: the fused single-launch form (k_proj_fused) when the frame
// has <= 4096 keypoints of <= 8 levels and <= 8192 queries -- one coalesced
// upload, one launch, one download of [nmatches, owner[n]].  Otherwise (or
// ORB_OPT_PROJ_FORM 1 / 2 / 3: serial phase 2 / single wave / two-phase
// speculative) the grid is built and the multi-kernel forms run.
static int run_proj(ProjArgs& a, const orbm_frame* f, DevFrame& df, int32_t* owner, const uint8_t* blocked) {
    int rc;
    DBuf<int32_t> own, nm; DBuf<uint8_t> blk;
    if ((rc = own.put(owner, std::max(1, f->n))) || (rc = blk.put(blocked, std::max(1, f->n)))) return rc;
    a.kps = df.kps.p; a.desc = df.desc.p; a.n = f->n; a.u_right = f->u_right ? df.ur.p : nullptr;
    a.scale = df.scale.p; a.g = grid_params(f); a.owner = own.p; a.blocked = blk.p;
    const int form = debug_opt(ORB_OPT_PROJ_FORM);
    if ((form == 0 || form == 4 || form == 5) && f->n <= kFusedMaxN && a.nq <= kFusedMaxQ && f->nlevels <= 8 &&
        proj_fused_lds(f->n, a.nq, false) <= kCuLds) {
        // the frame's grid in LDS (form 4: none, every window scans the frame),
        // then the lists in LDS for phase 2 when they fit (else read from L2 each round)
        const size_t gb = lds_grid_bytes(f->n);
        const int use_grid = form != 4 && proj_fused_lds(f->n, a.nq, false) + gb <= kCuLds;
        const int lds_lists = proj_fused_lds(f->n, a.nq, true) + (use_grid ? gb : 0) <= kCuLds;
        const size_t lds = proj_fused_lds(f->n, a.nq, lds_lists != 0) + (use_grid ? gb : 0);
        DBuf<uint32_t> lists; DBuf<int> cnt; DBuf<unsigned> ticket; OutBlock out;
        const unsigned zero = 0;
        if ((rc = ticket.put(&zero, 1)) || (rc = lists.alloc((size_t)std::max(1, a.nq) * kProjK)) ||
            (rc = cnt.alloc(std::max(1, a.nq))) || (rc = out.alloc((size_t)f->n + 13)))
            return rc;
        a.nmatches = nullptr;
        const int nblk = std::max(1, (a.nq + kFusedThreads / kWave - 1) / (kFusedThreads / kWave));
        if (form == 5) {       // phase 1, then phase 2 as a one-block launch (no ticket)
            KLAUNCH(k_proj_fused, dim3(nblk), dim3(kFusedThreads), lds, 0, a, proj_bound(a), lists.p, cnt.p,
                    ticket.p, own.p, out.d, lds_lists, use_grid, 1, (int*)nullptr, 0, Mirror{}, (const int*)nullptr);
            KLAUNCH(k_proj_fused, dim3(1), dim3(kFusedThreads), lds, 0, a, proj_bound(a), lists.p, cnt.p, ticket.p,
                    own.p, out.d, lds_lists, use_grid, 2, out.flag, out.seq, Mirror{}, (const int*)nullptr);
        } else {
            KLAUNCH(k_proj_fused, dim3(nblk), dim3(kFusedThreads), lds, 0, a, proj_bound(a), lists.p, cnt.p,
                    ticket.p, own.p, out.d, lds_lists, use_grid, 0, out.flag, out.seq, Mirror{}, (const int*)nullptr);
        }
        ORB_CHECK(hipGetLastError());
        std::vector<int32_t> res((size_t)f->n + 13);
        ORB_CHECK(out.fetch(res.data(), res.size()));
        if (f->n) std::memcpy(owner, res.data() + 1, (size_t)f->n * sizeof(int32_t));
        std::memcpy(proj_stats(), res.data() + f->n + 1, 12 * sizeof(int32_t));
        return res[0];
    }
    if ((rc = df.build_grid(f, 0)) || (rc = nm.alloc(1))) return rc;
    a.gsorted = df.sorted.p; a.gcount = df.count.p; a.cellstart = df.cs.p; a.nmatches = nm.p;
    // two-phase form unless its LDS slot table does not fit; phase 2 speculative
    // unless its table does not fit.  For testing, ORB_OPT_PROJ_FORM 2 forces
    // the single-wave form and 1 the serial phase 2.
    const size_t lds2 = proj_resolve_lds(a.n, a.nq), lds3 = proj_spec_lds(a.n, a.nq);
    if (lds2 <= 160 * 1024 && form != 2) {
        DBuf<uint2> topk; DBuf<int> cnt;
        if ((rc = topk.alloc((size_t)std::max(1, a.nq) * kProjK)) || (rc = cnt.alloc(std::max(1, a.nq)))) return rc;
        if (a.nq) KLAUNCH(k_proj_topk, dim3((a.nq + 3) / 4), dim3(256), 0, 0, a, proj_bound(a), topk.p, cnt.p);
        if (lds3 <= 160 * 1024 && form != 1)
            KLAUNCH(k_proj_resolve_spec, dim3(1), dim3(64), lds3, 0, a, topk.p, cnt.p);
        else
            KLAUNCH(k_proj_resolve, dim3(1), dim3(64), lds2, 0, a, topk.p, cnt.p);
    } else {
        const size_t lds = proj_lds(a.nq);
        if (lds > 160 * 1024) return ORB_ERR_UNSUPPORTED;
        KLAUNCH(k_proj, dim3(1), dim3(64), lds, 0, a);
    }
    ORB_CHECK(hipGetLastError());
    int32_t res = 0;
    ORB_CHECK(d2h(&res, nm.p, 4));
    if (f->n) ORB_CHECK(d2h(owner, own.p, f->n * 4));
    return res;
}

int orbm_search_by_projection_mps(const orbm_frame* f, const orbm_mappoints* mps, float th, int far_points,
                                  float th_far, float nnratio, int32_t* owner, const uint8_t* blocked) {
    if (!f || !mps || !owner || !blocked || !f->scale_factors) return ORB_ERR_PARAM;
    if (device_ok()) return ORB_ERR_DEVICE;
    if (f->n > 0xffff) return ORB_ERR_UNSUPPORTED;
    DevFrame df;
    int rc = df.upload(f, false, 0);
    if (rc) return rc;
    const int nq = mps->n;
    DBuf<float> qx, qy, qxr, vc, dp; DBuf<int32_t> lv; DBuf<uint8_t> iv, ho, qd;
    if ((rc = qx.put(mps->proj_x, nq)) || (rc = qy.put(mps->proj_y, nq)) || (rc = qxr.put(mps->proj_xr, nq)) ||
        (rc = lv.put(mps->level, nq)) || (rc = vc.put(mps->view_cos, nq)) || (rc = dp.put(mps->track_depth, nq)) ||
        (rc = iv.put(mps->in_view, nq)) || (rc = ho.put(mps->has_obs, nq)) || (rc = qd.put(mps->desc, (size_t)nq * 32)))
        return rc;
    ProjArgs a{};
    a.mode = 0; a.nq = nq; a.qx = qx.p; a.qy = qy.p; a.qxr = qxr.p; a.qlevel = lv.p; a.qviewcos = vc.p;
    a.qdepth = dp.p; a.qvalid = iv.p; a.qhas_obs = ho.p; a.qdesc = qd.p; a.qangle = nullptr;
    a.th = th; a.th_far = th_far; a.ratio = nnratio; a.far_points = far_points; a.last_mode = 0; a.check_ori = 0;
    return run_proj(a, f, df, owner, blocked);
}

int orbm_search_by_projection_last(const orbm_frame* cur, int nlast, const uint8_t* valid, const float* u,
                                   const float* v, const float* ur, const int32_t* last_octave,
                                   const float* last_angle, const uint8_t* has_obs, const uint8_t* last_desc,
                                   float th, int mode, int check_ori, int32_t* owner, const uint8_t* blocked) {
    if (!cur || !valid || !u || !v || !ur || !last_octave || !last_angle || !has_obs || !last_desc || !owner ||
        !blocked || !cur->scale_factors)
        return ORB_ERR_PARAM;
    if (device_ok()) return ORB_ERR_DEVICE;
    if (cur->n > 0xffff) return ORB_ERR_UNSUPPORTED;
    DevFrame df;
    int rc = df.upload(cur, false, 0);
    if (rc) return rc;
    DBuf<float> qx, qy, qxr, qa; DBuf<int32_t> lv; DBuf<uint8_t> iv, ho, qd;
    if ((rc = qx.put(u, nlast)) || (rc = qy.put(v, nlast)) || (rc = qxr.put(ur, nlast)) ||
        (rc = lv.put(last_octave, nlast)) || (rc = qa.put(last_angle, nlast)) || (rc = iv.put(valid, nlast)) ||
        (rc = ho.put(has_obs, nlast)) || (rc = qd.put(last_desc, (size_t)nlast * 32)))
        return rc;
    ProjArgs a{};
    a.mode = 1; a.nq = nlast; a.qx = qx.p; a.qy = qy.p; a.qxr = qxr.p; a.qlevel = lv.p; a.qviewcos = nullptr;
    a.qdepth = nullptr; a.qvalid = iv.p; a.qhas_obs = ho.p; a.qdesc = qd.p; a.qangle = qa.p;
    a.th = th; a.th_far = 0; a.ratio = 0; a.far_points = 0; a.last_mode = mode; a.check_ori = check_ori;
    a.skip_any = 0; a.accept = (float)kThHigh;                                   // :1770
    return run_proj(a, cur, df, owner, blocked);
}

int orbv_transform(const orbv_vocab* voc, int n, const uint8_t* desc, int levelsup, int32_t* word_id,
                   double* weight, int32_t* node_id, int device) {
    if (!voc || n < 0 || !desc || !word_id || !weight || !node_id) return ORB_ERR_PARAM;
    if (device < 0) return ORB_ERR_PARAM;     // the product path runs on the GPU only
    if (voc->nnodes < 2 || voc->nchild[0] == 0) return ORB_ERR_EMPTY;   // no words (TemplatedVocabulary::empty)
    if (hipSetDevice(device) != hipSuccess) return ORB_ERR_DEVICE;
    arena_reset();
    if (n == 0) return ORB_OK;
    int rc;
    DBuf<int> fc, nc, wid, ci; DBuf<uint8_t> nd, dd; DBuf<double> wt, wo; DBuf<int32_t> wio, nio;
    if (voc->child_idx) {
        int nchild_total = 0;
        for (int i = 0; i < voc->nnodes; ++i) nchild_total = std::max(nchild_total, voc->first_child[i] + voc->nchild[i]);
        if ((rc = ci.put(voc->child_idx, nchild_total))) return rc;
    }
    if ((rc = fc.put(voc->first_child, voc->nnodes)) || (rc = nc.put(voc->nchild, voc->nnodes)) ||
        (rc = nd.put(voc->node_desc, (size_t)voc->nnodes * 32)) || (rc = wid.put(voc->word_id, voc->nnodes)) ||
        (rc = wt.put(voc->weight, voc->nnodes)) || (rc = dd.put(desc, (size_t)n * 32)) || (rc = wo.alloc(n)) ||
        (rc = wio.alloc(n)) || (rc = nio.alloc(n)))
        return rc;
    const int nid_level = voc->depth_levels - levelsup;
    KLAUNCH(k_transform, dim3((n + 255) / 256), dim3(256), 0, 0, fc.p, nc.p, voc->child_idx ? ci.p : nullptr,
                       nd.p, wid.p, wt.p, n, dd.p,
                       nid_level, wio.p, wo.p, nio.p);
    ORB_CHECK(hipGetLastError());
    ORB_CHECK(d2h(word_id, wio.p, n * 4));
    ORB_CHECK(d2h(weight, wo.p, n * 8));
    ORB_CHECK(d2h(node_id, nio.p, n * 4));
    return ORB_OK;
}

int orbv_transform_device(const orbv_vocab* voc, int n, const uint8_t* d_desc, int levelsup, int32_t* d_word_id,
                          double* d_weight, int32_t* d_node_id, void* stream) {
    if (!voc || n < 0 || (n && (!d_desc || !d_word_id || !d_weight || !d_node_id))) return ORB_ERR_PARAM;
    if (!voc->first_child || !voc->nchild || !voc->node_desc || !voc->word_id || !voc->weight) return ORB_ERR_PARAM;
    if (voc->nnodes < 2) return ORB_ERR_EMPTY;
    if (n == 0) return ORB_OK;
    const int nid_level = voc->depth_levels - levelsup;
    ORB_LAUNCH(k_transform, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, voc->first_child,
                       voc->nchild, voc->child_idx, voc->node_desc, voc->word_id, voc->weight, n, d_desc, nid_level,
                       d_word_id, d_weight, d_node_id);
    ORB_CHECK(hipGetLastError());
    return ORB_OK;
}

int orbm_fuse(const orbm_frame* kf, const float* inv_level_sigma2, int nmp, const uint8_t* valid, const float* u,
              const float* v, const float* ur, const int32_t* level, const uint8_t* desc, float th, int fma,
              int32_t* best_idx, int32_t* best_dist) {
    if (!kf || !inv_level_sigma2 || !kf->scale_factors || nmp < 0 || !best_idx || !best_dist) return ORB_ERR_PARAM;
    if (nmp && (!valid || !u || !v || !ur || !level || !desc)) return ORB_ERR_PARAM;
    if (nmp == 0) return 0;
    int rc;
    if ((rc = device_ok())) return rc;
    for (int i = 0; i < nmp; ++i)
        if (valid[i] && (level[i] < 0 || level[i] >= kf->nlevels)) return ORB_ERR_PARAM;
    DevFrame df;
    if ((rc = df.upload(kf, true, 0))) return rc;
    DBuf<float> is2, bu, bv, bur; DBuf<uint8_t> bval, bd; DBuf<int32_t> blv, bi, bdist;
    if ((rc = is2.put(inv_level_sigma2, kf->nlevels)) || (rc = bu.put(u, nmp)) || (rc = bv.put(v, nmp)) ||
        (rc = bur.put(ur, nmp)) || (rc = bval.put(valid, nmp)) || (rc = bd.put(desc, (size_t)nmp * 32)) ||
        (rc = blv.put(level, nmp)) || (rc = bi.alloc(nmp)) || (rc = bdist.alloc(nmp)))
        return rc;
    FuseArgs a{};
    a.kps = df.kps.p; a.desc = df.desc.p; a.u_right = kf->u_right ? df.ur.p : nullptr; a.scale = df.scale.p;
    a.inv_sigma2 = is2.p; a.g = grid_params(kf); a.gsorted = df.sorted.p; a.gcount = df.count.p;
    a.cellstart = df.cs.p; a.nmp = nmp;
    a.valid = bval.p; a.u = bu.p; a.v = bv.p; a.ur = bur.p; a.level = blv.p; a.mdesc = bd.p; a.th = th; a.fma = fma;
    a.chi2 = 1; a.accept = kThLow;                                               // :1311
    a.best_idx = bi.p; a.best_dist = bdist.p;
    KLAUNCH(k_fuse, dim3((nmp + 3) / 4), dim3(256), 0, 0, a);
    ORB_CHECK(hipGetLastError());
    ORB_CHECK(d2h(best_idx, bi.p, nmp * sizeof(int32_t)));
    ORB_CHECK(d2h(best_dist, bdist.p, nmp * sizeof(int32_t)));
    int n = 0;
    for (int i = 0; i < nmp; ++i) n += best_idx[i] >= 0;
    return n;
}

// Items of SearchForTriangulation: every KF1 feature of a node both
// FeatureVectors hold (the merge of :962-1100), with that node's KF2 range.
static void tri_items(const orbm_featvec* fv1, const orbm_featvec* fv2, std::vector<int32_t>& it_i1,
                      std::vector<int32_t>& it_b, std::vector<int32_t>& it_e) {
    int a = 0, b = 0;
    while (a < fv1->nnodes && b < fv2->nnodes) {
        if (fv1->node_ids[a] == fv2->node_ids[b]) {
            for (int j = fv1->offsets[a]; j < fv1->offsets[a + 1]; ++j) {
                it_i1.push_back((int32_t)fv1->idx[j]);
                it_b.push_back(fv2->offsets[b]);
                it_e.push_back(fv2->offsets[b + 1]);
            }
            ++a;
            ++b;
        } else if (fv1->node_ids[a] < fv2->node_ids[b]) {
            ++a;
        } else {
            ++b;
        }
    }
}

int orbm_search_for_triangulation(const orbm_frame* kf1, const orbm_featvec* fv1, const uint8_t* has_mp1,
                                  const orbm_frame* kf2, const orbm_featvec* fv2, const uint8_t* has_mp2,
                                  const float* F12, float ep_x, float ep_y, const float* level_sigma2_2,
                                  int only_stereo, int coarse, int check_ori, int fma, int32_t* matches12) {
    if (!kf1 || !kf2 || !fv1 || !fv2 || !has_mp1 || !has_mp2 || !F12 || !level_sigma2_2 || !matches12 ||
        !kf2->scale_factors)
        return ORB_ERR_PARAM;
    int rc;
    if ((rc = device_ok())) return rc;
    std::vector<int32_t> it_i1, it_b, it_e;
    tri_items(fv1, fv2, it_i1, it_b, it_e);
    const int nitems = (int)it_i1.size();
    DevFrame f1, f2;
    if ((rc = f1.upload(kf1, false, 0)) || (rc = f2.upload(kf2, false, 0))) return rc;
    DBuf<uint8_t> m1, m2; DBuf<float> s2; DBuf<int32_t> bi1, bb, be, bm, bbin, out, nm; DBuf<uint32_t> fidx;
    const int n2idx = fv2->nnodes ? fv2->offsets[fv2->nnodes] : 0;
    if ((rc = m1.put(has_mp1, std::max(1, kf1->n))) || (rc = m2.put(has_mp2, std::max(1, kf2->n))) ||
        (rc = s2.put(level_sigma2_2, kf2->nlevels)) || (rc = bi1.put(it_i1.data(), nitems)) ||
        (rc = bb.put(it_b.data(), nitems)) || (rc = be.put(it_e.data(), nitems)) ||
        (rc = fidx.put(fv2->idx, n2idx)) || (rc = bm.alloc(std::max(1, nitems))) ||
        (rc = bbin.alloc(std::max(1, nitems))) || (rc = out.alloc(std::max(1, kf1->n))) || (rc = nm.alloc(1)))
        return rc;
    TriArgs ta;
    ta.k1 = f1.kps.p; ta.k2 = f2.kps.p; ta.d1 = f1.desc.p; ta.d2 = f2.desc.p;
    ta.ur1 = kf1->u_right ? f1.ur.p : nullptr; ta.ur2 = kf2->u_right ? f2.ur.p : nullptr;
    ta.mp1 = m1.p; ta.mp2 = m2.p; ta.scale2 = f2.scale.p; ta.sigma2_2 = s2.p;
    ta.item_i1 = bi1.p; ta.item_b = bb.p; ta.item_e = be.p; ta.fv2_idx = fidx.p; ta.nitems = nitems;
    for (int k = 0; k < 9; ++k) ta.F[k] = F12[k];
    ta.ep_x = ep_x; ta.ep_y = ep_y; ta.only_stereo = only_stereo; ta.coarse = coarse; ta.fma = fma;
    ta.check_ori = check_ori; ta.item_match = bm.p; ta.item_bin = bbin.p;
    if (nitems) KLAUNCH(k_tri, dim3((nitems + 3) / 4), dim3(256), 0, 0, ta);
    KLAUNCH(k_tri_final, dim3(1), dim3(256), 0, 0, ta, kf1->n, out.p, nm.p);
    ORB_CHECK(hipGetLastError());
    int32_t n = 0;
    if (kf1->n) ORB_CHECK(d2h(matches12, out.p, kf1->n * sizeof(int32_t)));
    ORB_CHECK(d2h(&n, nm.p, sizeof(int32_t)));
    return n;
}

int orbm_search_for_triangulation_checked(const orbm_frame* kf1, const orbm_featvec* fv1, const uint8_t* has_mp1,
                                          const orbm_frame* kf2, const orbm_featvec* fv2, const uint8_t* has_mp2,
                                          int only_stereo, int check_ori, orbm_tri_check_fn check, void* ctx,
                                          int32_t* matches12) {
    if (!kf1 || !kf2 || !fv1 || !fv2 || !has_mp1 || !has_mp2 || !check || !matches12) return ORB_ERR_PARAM;
    int rc;
    if ((rc = device_ok())) return rc;
    std::vector<int32_t> it_i1, it_b, it_e;
    tri_items(fv1, fv2, it_i1, it_b, it_e);
    const int nitems = (int)it_i1.size();
    std::vector<int32_t> seg(nitems + 1, 0);
    for (int t = 0; t < nitems; ++t) seg[t + 1] = seg[t] + (it_e[t] - it_b[t]);
    const int total = seg[nitems];
    for (int i = 0; i < kf1->n; ++i) matches12[i] = -1;
    std::vector<int32_t> res(1 + nitems + 2 * (size_t)total);       // [unused | counts | keys | KF2 indices]
    if (nitems) {
        DevFrame f1, f2;
        if ((rc = f1.upload(kf1, false, 0)) || (rc = f2.upload(kf2, false, 0))) return rc;
        DBuf<uint8_t> m1, m2; DBuf<int32_t> bi1, bb, be, bseg, out; DBuf<uint32_t> fidx;
        const int n2idx = fv2->nnodes ? fv2->offsets[fv2->nnodes] : 0;
        if ((rc = m1.put(has_mp1, std::max(1, kf1->n))) || (rc = m2.put(has_mp2, std::max(1, kf2->n))) ||
            (rc = bi1.put(it_i1.data(), nitems)) || (rc = bb.put(it_b.data(), nitems)) ||
            (rc = be.put(it_e.data(), nitems)) || (rc = bseg.put(seg.data(), nitems + 1)) ||
            (rc = fidx.put(fv2->idx, n2idx)) || (rc = out.alloc(res.size())))
            return rc;
        TriArgs ta{};
        ta.k1 = f1.kps.p; ta.k2 = f2.kps.p; ta.d1 = f1.desc.p; ta.d2 = f2.desc.p;
        ta.ur1 = kf1->u_right ? f1.ur.p : nullptr; ta.ur2 = kf2->u_right ? f2.ur.p : nullptr;
        ta.mp1 = m1.p; ta.mp2 = m2.p; ta.item_i1 = bi1.p; ta.item_b = bb.p; ta.item_e = be.p;
        ta.fv2_idx = fidx.p; ta.nitems = nitems; ta.only_stereo = only_stereo;
        KLAUNCH(k_tri_cands, dim3((nitems + 3) / 4), dim3(256), 0, 0, ta, bseg.p, out.p + 1,
                (uint32_t*)(out.p + 1 + nitems), out.p + 1 + nitems + total);
        ORB_CHECK(hipGetLastError());
        ORB_CHECK(d2h(res.data(), out.p, res.size() * sizeof(int32_t)));
    }
    // the caller's geometric check in (distance, last position) order: the
    // first candidate it accepts is the reference's surviving bestIdx2
    // (accepted distances never increase and equal ones overwrite, :1010-1076)
    const int32_t* cnt = res.data() + 1;
    const uint32_t* key = (const uint32_t*)(res.data() + 1 + nitems);
    const int32_t* i2s = res.data() + 1 + nitems + total;
    int nmatches = 0, hist[kHisto] = {0};
    std::vector<int32_t> bins(nitems, -1);
    std::vector<std::pair<uint32_t, int32_t>> cand;
    for (int t = 0; t < nitems; ++t) {
        cand.clear();
        for (int e = seg[t]; e < seg[t] + cnt[t]; ++e) cand.emplace_back(key[e], i2s[e]);
        std::sort(cand.begin(), cand.end());
        const int i1 = it_i1[t];
        for (const auto& c : cand) {
            if (!check(ctx, i1, c.second)) continue;
            matches12[i1] = c.second;
            ++nmatches;
            if (check_ori) {
                bins[t] = rot_bin(kf1->kps[i1].angle, kf2->kps[c.second].angle);
                ++hist[bins[t]];
            }
            break;
        }
    }
    if (check_ori) {
        int k1, k2, k3;
        three_maxima(hist, k1, k2, k3);
        for (int t = 0; t < nitems; ++t)
            if (bins[t] >= 0 && bins[t] != k1 && bins[t] != k2 && bins[t] != k3) { matches12[it_i1[t]] = -1; --nmatches; }
    }
    return nmatches;
}

int orbm_compute_distinctive_descriptors(int npoints, const int32_t* off, const uint8_t* desc, int32_t* best,
                                         int device) {
    if (npoints < 0 || (npoints && (!off || !best))) return ORB_ERR_PARAM;
    if (npoints == 0) return ORB_OK;
    const int total = off[npoints];
    if (off[0] != 0 || total < 0 || (total && !desc)) return ORB_ERR_PARAM;
    for (int p = 0; p < npoints; ++p)
        if (off[p + 1] < off[p] || off[p + 1] - off[p] > 65535) return ORB_ERR_PARAM;
    if (hipSetDevice(device) != hipSuccess) return ORB_ERR_DEVICE;
    arena_reset();
    int rc;
    DBuf<int32_t> bo, bb; DBuf<uint8_t> bd;
    if ((rc = bo.put(off, (size_t)npoints + 1)) || (rc = bd.put(desc, (size_t)total * 32)) || (rc = bb.alloc(npoints)))
        return rc;
    KLAUNCH(k_distinctive, dim3(npoints), dim3(64), 0, 0, npoints, bo.p, bd.p, bb.p);
    ORB_CHECK(hipGetLastError());
    ORB_CHECK(d2h(best, bb.p, npoints * sizeof(int32_t)));
    return ORB_OK;
}


// ---------------- loop-closing / relocalisation matchers ----------------

int orbm_search_by_bow_kf(const orbm_frame* kf1, const orbm_featvec* fv1, const uint8_t* valid1,
                          const orbm_frame* kf2, const orbm_featvec* fv2, const uint8_t* valid2, float nnratio,
                          int check_ori, int32_t* matches12) {
    if (!kf1 || !fv1 || !valid1 || !kf2 || !fv2 || !valid2 || !matches12) return ORB_ERR_PARAM;
    if (kf1->n < 0 || kf2->n < 0) return ORB_ERR_PARAM;
    int rc;
    if ((rc = device_ok())) return rc;
    DBuf<orb_keypoint> kk, fk; DBuf<uint8_t> kd, fd, kvv, fvv; DBuf<uint32_t> kn, ki, fn, fi; DBuf<int> ko, fo;
    DBuf<long long> kpo, nodo, idxo; DBuf<int32_t> m, nm, o12;
    const long long kp_off[2] = {0, kf1->n}, node_off[2] = {0, fv1->nnodes}, idx_off[1] = {0};
    const int n1idx = fv1->nnodes ? fv1->offsets[fv1->nnodes] : 0;
    const int n2idx = fv2->nnodes ? fv2->offsets[fv2->nnodes] : 0;
    static const int zero = 0;
    if ((rc = kk.put(kf1->kps, kf1->n)) || (rc = kd.put(kf1->desc, (size_t)kf1->n * 32)) ||
        (rc = kvv.put(valid1, kf1->n)) || (rc = kn.put(fv1->node_ids, fv1->nnodes)) ||
        (rc = ko.put(fv1->nnodes ? fv1->offsets : &zero, fv1->nnodes + 1)) || (rc = ki.put(fv1->idx, n1idx)) ||
        (rc = fk.put(kf2->kps, kf2->n)) || (rc = fd.put(kf2->desc, (size_t)kf2->n * 32)) ||
        (rc = fvv.put(valid2, kf2->n)) || (rc = fn.put(fv2->node_ids, fv2->nnodes)) ||
        (rc = fo.put(fv2->nnodes ? fv2->offsets : &zero, fv2->nnodes + 1)) || (rc = fi.put(fv2->idx, n2idx)) ||
        (rc = kpo.put(kp_off, 2)) || (rc = nodo.put(node_off, 2)) || (rc = idxo.put(idx_off, 1)) ||
        (rc = m.alloc(std::max(1, kf2->n))) || (rc = nm.alloc(1)) || (rc = o12.alloc(std::max(1, kf1->n))))
        return rc;
    BowArgs a{};
    a.kf_kps = kk.p; a.kf_desc = kd.p; a.kf_valid = kvv.p; a.kp_off = kpo.p;
    a.kf_node = kn.p; a.kf_off = ko.p; a.kf_idx = ki.p; a.node_off = nodo.p; a.idx_off = idxo.p;
    a.f_kps = fk.p; a.f_desc = fd.p; a.f_n = kf2->n; a.f_node = fn.p; a.f_off = fo.p; a.f_idx = fi.p;
    a.f_nnodes = fv2->nnodes; a.ratio = nnratio; a.check_ori = check_ori; a.match = m.p; a.nmatches = nm.p;
    a.f_valid = fvv.p; a.out12 = o12.p;
    if ((rc = launch_bow(a, 1, 0, bow_big_nodes(fv2), fv1->nnodes))) return rc;
    int32_t res = 0;
    ORB_CHECK(d2h(&res, nm.p, 4));
    if (kf1->n) ORB_CHECK(d2h(matches12, o12.p, kf1->n * 4));
    return res;
}

// Shared by the two "best only" projection searches with a claim on any
// occupied slot (mode 1 of k_proj).
static int proj_best_only(const orbm_frame* f, int nq, const uint8_t* valid, const float* u, const float* v,
                          const int32_t* level, const float* angle, const uint8_t* desc, float th, int win,
                          float accept, int check_ori, int32_t* owner) {
    if (!f || nq < 0 || !owner || !f->scale_factors) return ORB_ERR_PARAM;
    if (nq && (!valid || !u || !v || !level || !desc || (check_ori && !angle))) return ORB_ERR_PARAM;
    int rc;
    if ((rc = device_ok())) return rc;
    if (f->n > 0xffff) return ORB_ERR_UNSUPPORTED;
    for (int i = 0; i < nq; ++i)
        if (valid[i] && (level[i] < 0 || level[i] >= f->nlevels)) return ORB_ERR_PARAM;
    if (nq == 0) return 0;
    orbm_frame fn = *f;
    fn.u_right = nullptr;                       // no stereo gate in these searches
    DevFrame df;
    if ((rc = df.upload(&fn, false, 0))) return rc;
    DBuf<float> qx, qy, qa; DBuf<int32_t> lv; DBuf<uint8_t> iv, qd;
    if ((rc = qx.put(u, nq)) || (rc = qy.put(v, nq)) || (rc = lv.put(level, nq)) || (rc = iv.put(valid, nq)) ||
        (rc = qd.put(desc, (size_t)nq * 32)))
        return rc;
    if (check_ori && (rc = qa.put(angle, nq))) return rc;
    std::vector<uint8_t> blocked(std::max(1, f->n), 1);
    ProjArgs a{};
    a.mode = 1; a.nq = nq; a.qx = qx.p; a.qy = qy.p; a.qxr = nullptr; a.qlevel = lv.p; a.qvalid = iv.p;
    a.qhas_obs = nullptr; a.qdesc = qd.p; a.qangle = check_ori ? qa.p : nullptr;
    a.th = th; a.last_mode = win; a.check_ori = check_ori; a.skip_any = 1; a.accept = accept;
    return run_proj(a, &fn, df, owner, blocked.data());
}

int orbm_search_by_projection_kf(const orbm_frame* f, int nq, const uint8_t* valid, const float* u,
                                 const float* v, const int32_t* level, const float* kf_angle, const uint8_t* desc,
                                 float th, int orb_dist, int check_ori, int32_t* owner) {
    // GetFeaturesInArea(.., nPredictedLevel-1, nPredictedLevel+1) (:1939), bestDist <= ORBdist (:1966)
    return proj_best_only(f, nq, valid, u, v, level, kf_angle, desc, th, 0, (float)orb_dist, check_ori, owner);
}

int orbm_search_by_projection_sim3(const orbm_frame* kf, int nq, const uint8_t* valid, const float* u,
                                   const float* v, const int32_t* level, const uint8_t* desc, float th,
                                   float ratio_hamming, int32_t* matched) {
    // levels pl-1 .. pl (:509), bestDist <= TH_LOW * ratioHamming (:523), no rotation filter
    return proj_best_only(kf, nq, valid, u, v, level, nullptr, desc, th, 3, (float)kThLow * ratio_hamming, 0,
                          matched);
}

// One "independent best" pass (k_fuse without the chi-square gate) of nq
// points against the keyframe kf, into device buffers bi / bd.
static int best_in_area(const orbm_frame* kf, DevFrame& df, int nq, const uint8_t* valid, const float* u,
                        const float* v, const int32_t* level, const uint8_t* desc, float th, int accept,
                        DBuf<int32_t>& bi, DBuf<int32_t>& bd, DBuf<uint8_t>& bval, DBuf<float>& bu,
                        DBuf<float>& bv, DBuf<int32_t>& blv, DBuf<uint8_t>& bdesc) {
    int rc;
    if ((rc = bu.put(u, nq)) || (rc = bv.put(v, nq)) || (rc = bval.put(valid, nq)) ||
        (rc = bdesc.put(desc, (size_t)nq * 32)) || (rc = blv.put(level, nq)) || (rc = bi.alloc(nq)) ||
        (rc = bd.alloc(nq)))
        return rc;
    FuseArgs a{};
    a.kps = df.kps.p; a.desc = df.desc.p; a.u_right = nullptr; a.scale = df.scale.p; a.inv_sigma2 = nullptr;
    a.g = grid_params(kf); a.gsorted = df.sorted.p; a.gcount = df.count.p; a.cellstart = df.cs.p; a.nmp = nq;
    a.valid = bval.p; a.u = bu.p; a.v = bv.p; a.ur = nullptr; a.level = blv.p; a.mdesc = bdesc.p; a.th = th;
    a.fma = 0; a.chi2 = 0; a.accept = accept; a.best_idx = bi.p; a.best_dist = bd.p;
    KLAUNCH(k_fuse, dim3((nq + 3) / 4), dim3(256), 0, 0, a);
    ORB_CHECK(hipGetLastError());
    return ORB_OK;
}

static int check_levels(int nq, const uint8_t* valid, const int32_t* level, int nlevels) {
    for (int i = 0; i < nq; ++i)
        if (valid[i] && (level[i] < 0 || level[i] >= nlevels)) return ORB_ERR_PARAM;
    return ORB_OK;
}

int orbm_fuse_sim3(const orbm_frame* kf, int nmp, const uint8_t* valid, const float* u, const float* v,
                   const int32_t* level, const uint8_t* desc, float th, int32_t* best_idx, int32_t* best_dist) {
    if (!kf || !kf->scale_factors || nmp < 0 || !best_idx || !best_dist) return ORB_ERR_PARAM;
    if (nmp && (!valid || !u || !v || !level || !desc)) return ORB_ERR_PARAM;
    if (nmp == 0) return 0;
    int rc;
    if ((rc = device_ok()) || (rc = check_levels(nmp, valid, level, kf->nlevels))) return rc;
    if (kf->n > 0xffff) return ORB_ERR_UNSUPPORTED;
    DevFrame df;
    if ((rc = df.upload(kf, true, 0))) return rc;
    DBuf<int32_t> bi, bd, blv; DBuf<uint8_t> bval, bdesc; DBuf<float> bu, bv;
    if ((rc = best_in_area(kf, df, nmp, valid, u, v, level, desc, th, kThLow, bi, bd, bval, bu, bv, blv, bdesc)))
        return rc;                                                               // :1437
    ORB_CHECK(d2h(best_idx, bi.p, nmp * sizeof(int32_t)));
    ORB_CHECK(d2h(best_dist, bd.p, nmp * sizeof(int32_t)));
    int n = 0;
    for (int i = 0; i < nmp; ++i) n += best_idx[i] >= 0;
    return n;
}

int orbm_search_by_sim3(const orbm_frame* kf1, const orbm_frame* kf2, const uint8_t* valid1, const float* u1,
                        const float* v1, const int32_t* level1, const uint8_t* mdesc1, const uint8_t* valid2,
                        const float* u2, const float* v2, const int32_t* level2, const uint8_t* mdesc2, float th,
                        int32_t* matches12) {
    if (!kf1 || !kf2 || !kf1->scale_factors || !kf2->scale_factors || !matches12 || kf1->n < 0 || kf2->n < 0)
        return ORB_ERR_PARAM;
    const int n1 = kf1->n, n2 = kf2->n;
    if (n1 && (!valid1 || !u1 || !v1 || !level1 || !mdesc1)) return ORB_ERR_PARAM;
    if (n2 && (!valid2 || !u2 || !v2 || !level2 || !mdesc2)) return ORB_ERR_PARAM;
    int rc;
    if ((rc = device_ok())) return rc;
    if (n1 > 0xffff || n2 > 0xffff) return ORB_ERR_UNSUPPORTED;
    // KF1's points are predicted in KF2's pyramid and vice versa (:1534, :1614)
    if ((rc = check_levels(n1, valid1, level1, kf2->nlevels)) || (rc = check_levels(n2, valid2, level2, kf1->nlevels)))
        return rc;
    if (n1 == 0) return 0;
    DevFrame f1, f2;
    if ((rc = f1.upload(kf1, true, 0)) || (rc = f2.upload(kf2, true, 0))) return rc;
    DBuf<int32_t> b1, d1, l1, b2, d2, l2, out, nf; DBuf<uint8_t> va1, de1, va2, de2; DBuf<float> x1, y1, x2, y2;
    // KF1 -> KF2 (:1496-1573) and KF2 -> KF1 (:1576-1653), bestDist <= TH_HIGH
    if ((rc = best_in_area(kf2, f2, n1, valid1, u1, v1, level1, mdesc1, th, kThHigh, b1, d1, va1, x1, y1, l1, de1)))
        return rc;
    if ((rc = b2.alloc(std::max(1, n2)))) return rc;
    if (n2) {
        if ((rc = best_in_area(kf1, f1, n2, valid2, u2, v2, level2, mdesc2, th, kThHigh, b2, d2, va2, x2, y2, l2,
                               de2)))
            return rc;
    } else {
        ORB_CHECK(flush_uploads());
        ORB_CHECK(hipMemset(b2.p, 0xff, sizeof(int32_t)));
    }
    if ((rc = out.alloc(n1)) || (rc = nf.alloc(1))) return rc;
    KLAUNCH(k_sim3_agree, dim3(1), dim3(256), 0, 0, b1.p, n1, b2.p, out.p, nf.p);
    ORB_CHECK(hipGetLastError());
    int32_t res = 0;
    ORB_CHECK(d2h(matches12, out.p, n1 * sizeof(int32_t)));
    ORB_CHECK(d2h(&res, nf.p, sizeof(int32_t)));
    return res;
}


// ---------------- fisheye stereo frames ----------------

// One grid order + cell-start table over cnt keypoints at kps_dev (one frame).
static int grid_one(const orb_keypoint* kps_dev, const int* n_dev, int cnt, GridParams g, DBuf<uint32_t>& sorted,
                    DBuf<int>& count, DBuf<int>& cs) {
    int rc;
    const int nn = std::max(1, cnt);
    if ((rc = sorted.alloc(nn)) || (rc = count.alloc(1)) || (rc = cs.alloc(kCells + 1))) return rc;
    if (grid_cs_lds(nn) <= 160 * 1024) {
        KLAUNCH(k_grid_cs, dim3(1), dim3(256), grid_cs_lds(nn), 0, kps_dev, n_dev, nn, g, sorted.p,
                           count.p, cs.p, (uint32_t*)nullptr, (int*)nullptr);
    } else {
        const int sc = pow2_at_least(nn);
        KLAUNCH(k_grid, dim3(1), dim3(256), sc * sizeof(uint32_t), 0, kps_dev, n_dev, nn, g, sorted.p,
                           count.p, sc, (uint32_t*)nullptr, (int*)nullptr);
        KLAUNCH(k_cell_start, dim3(1), dim3(256), 0, 0, sorted.p, count.p, nn, cs.p);
    }
    return hipGetLastError() == hipSuccess ? ORB_OK : ORB_ERR_DEVICE;
}

// Upload the combined frame and build the left / right grids; run k_proj_fisheye.
static int run_fisheye(ProjArgs& a, FishArgs& fa, const orbm_frame* f, int nleft, int32_t* owner,
                       const uint8_t* blocked) {
    int rc;
    orbm_frame fn = *f;
    fn.u_right = nullptr;                       // no mvuRight gate for Nleft != -1 (:92, :1751)
    DevFrame df;
    if ((rc = df.upload(&fn, false, 0))) return rc;
    const int ns[2] = {nleft, f->n - nleft};
    DBuf<int> dn; DBuf<uint32_t> gl, gr; DBuf<int> cl, cr, csl, csr;
    if ((rc = dn.put(ns, 2))) return rc;
    const GridParams g = grid_params(f);
    if ((rc = grid_one(df.kps.p, dn.p, nleft, g, gl, cl, csl)) ||
        (rc = grid_one(df.kps.p + nleft, dn.p + 1, f->n - nleft, g, gr, cr, csr)))
        return rc;
    DBuf<int32_t> own, nm; DBuf<uint8_t> blk;
    if ((rc = own.put(owner, std::max(1, f->n))) || (rc = blk.put(blocked, std::max(1, f->n))) || (rc = nm.alloc(1)))
        return rc;
    a.kps = df.kps.p; a.desc = df.desc.p; a.n = f->n; a.u_right = nullptr; a.scale = df.scale.p; a.g = g;
    a.owner = own.p; a.blocked = blk.p; a.nmatches = nm.p;
    fa.nleft = nleft; fa.gs_l = gl.p; fa.gs_r = gr.p; fa.cs_l = csl.p; fa.cs_r = csr.p;
    const size_t lds = (size_t)(32 + 2 * a.nq + 1) * 4 + 64;
    if (lds > 160 * 1024) return ORB_ERR_UNSUPPORTED;
    KLAUNCH(k_proj_fisheye, dim3(1), dim3(64), lds, 0, a, fa);
    ORB_CHECK(hipGetLastError());
    int32_t res = 0;
    ORB_CHECK(d2h(&res, nm.p, 4));
    if (f->n) ORB_CHECK(d2h(owner, own.p, f->n * 4));
    return res;
}

int orbm_search_by_projection_mps_fisheye(const orbm_frame* f, int nleft, const int32_t* l2r, const int32_t* r2l,
                                          const orbm_mappoints* mps, const orbm_mappoints_right* mr, float th,
                                          int far_points, float th_far, float nnratio, int32_t* owner,
                                          const uint8_t* blocked) {
    if (!f || !mps || !mr || !owner || !blocked || !f->scale_factors || !l2r || !r2l) return ORB_ERR_PARAM;
    if (nleft < 0 || nleft > f->n || f->n > 0xffff) return ORB_ERR_PARAM;
    int rc;
    if ((rc = device_ok())) return rc;
    const int nq = mps->n, nr = f->n - nleft;
    for (int i = 0; i < nq; ++i) {
        if (mps->in_view[i] && (mps->level[i] < 0 || mps->level[i] >= f->nlevels)) return ORB_ERR_PARAM;
        if (mr->in_view[i] && (mr->level[i] < -1 || mr->level[i] >= f->nlevels)) return ORB_ERR_PARAM;
    }
    DBuf<float> qx, qy, vc, dp, rx, ry, rvc; DBuf<int32_t> lv, rlv, dl2r, dr2l; DBuf<uint8_t> iv, ho, qd, riv;
    if ((rc = qx.put(mps->proj_x, nq)) || (rc = qy.put(mps->proj_y, nq)) || (rc = lv.put(mps->level, nq)) ||
        (rc = vc.put(mps->view_cos, nq)) || (rc = dp.put(mps->track_depth, nq)) || (rc = iv.put(mps->in_view, nq)) ||
        (rc = ho.put(mps->has_obs, nq)) || (rc = qd.put(mps->desc, (size_t)nq * 32)) ||
        (rc = rx.put(mr->proj_x, nq)) || (rc = ry.put(mr->proj_y, nq)) || (rc = rlv.put(mr->level, nq)) ||
        (rc = rvc.put(mr->view_cos, nq)) || (rc = riv.put(mr->in_view, nq)) ||
        (rc = dl2r.put(l2r, std::max(1, nleft))) || (rc = dr2l.put(r2l, std::max(1, nr))))
        return rc;
    ProjArgs a{};
    a.mode = 0; a.nq = nq; a.qx = qx.p; a.qy = qy.p; a.qxr = nullptr; a.qlevel = lv.p; a.qviewcos = vc.p;
    a.qdepth = dp.p; a.qvalid = iv.p; a.qhas_obs = ho.p; a.qdesc = qd.p; a.qangle = nullptr;
    a.th = th; a.th_far = th_far; a.ratio = nnratio; a.far_points = far_points; a.last_mode = 0; a.check_ori = 0;
    FishArgs fa{};
    fa.l2r = dl2r.p; fa.r2l = dr2l.p; fa.rvalid = riv.p; fa.rqx = rx.p; fa.rqy = ry.p; fa.rlevel = rlv.p;
    fa.rviewcos = rvc.p;
    return run_fisheye(a, fa, f, nleft, owner, blocked);
}

int orbm_search_by_projection_last_fisheye(const orbm_frame* cur, int nleft, int nlast, const uint8_t* valid,
                                           const float* u, const float* v, const float* ur, const float* vr,
                                           const int32_t* last_octave, const float* last_angle,
                                           const uint8_t* has_obs, const uint8_t* last_desc, float th, int mode,
                                           int check_ori, int32_t* owner, const uint8_t* blocked) {
    if (!cur || !owner || !blocked || !cur->scale_factors || nlast < 0) return ORB_ERR_PARAM;
    if (nlast && (!valid || !u || !v || !ur || !vr || !last_octave || !last_angle || !has_obs || !last_desc))
        return ORB_ERR_PARAM;
    if (nleft < 0 || nleft > cur->n || cur->n > 0xffff) return ORB_ERR_PARAM;
    int rc;
    if ((rc = device_ok())) return rc;
    for (int i = 0; i < nlast; ++i)
        if (valid[i] && (last_octave[i] < 0 || last_octave[i] >= cur->nlevels)) return ORB_ERR_PARAM;
    DBuf<float> qx, qy, rx, ry, qa; DBuf<int32_t> lv; DBuf<uint8_t> iv, ho, qd;
    if ((rc = qx.put(u, nlast)) || (rc = qy.put(v, nlast)) || (rc = rx.put(ur, nlast)) || (rc = ry.put(vr, nlast)) ||
        (rc = lv.put(last_octave, nlast)) || (rc = qa.put(last_angle, nlast)) || (rc = iv.put(valid, nlast)) ||
        (rc = ho.put(has_obs, nlast)) || (rc = qd.put(last_desc, (size_t)nlast * 32)))
        return rc;
    ProjArgs a{};
    a.mode = 1; a.nq = nlast; a.qx = qx.p; a.qy = qy.p; a.qxr = nullptr; a.qlevel = lv.p; a.qvalid = iv.p;
    a.qhas_obs = ho.p; a.qdesc = qd.p; a.qangle = qa.p; a.th = th; a.last_mode = mode; a.check_ori = check_ori;
    a.skip_any = 0; a.accept = (float)kThHigh;
    FishArgs fa{};
    fa.rqx = rx.p; fa.rqy = ry.p;
    return run_fisheye(a, fa, cur, nleft, owner, blocked);
}

orbm_dframe* orbm_dframe_create(int device) {
    int ndev = 0;
    if (device < 0 || hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) return nullptr;
    orbm_dframe* df = new (std::nothrow) orbm_dframe();
    if (df) df->device = device;
    return df;
}

void orbm_dframe_destroy(orbm_dframe* df) {
    if (!df) return;
    if (hipSetDevice(df->device) == hipSuccess) (void)hipDeviceSynchronize();   // no search may still read it
    delete df;
}

int orbm_dframe_count(const orbm_dframe* df) { return df ? df->n : ORB_ERR_PARAM; }

int orbm_dframe_upload(orbm_dframe* df, const orbm_frame* f, const orbm_featvec* fv) {
    if (!df || !f || f->n < 0 || (f->n && (!f->kps || !f->desc))) return ORB_ERR_PARAM;
    if (hipSetDevice(df->device) != hipSuccess) return ORB_ERR_DEVICE;
    int rc;
    if ((rc = grow_dev(df->kps, df->cap_k, f->n)) || (rc = grow_dev(df->desc, df->cap_d, (size_t)f->n * 32))) return rc;
    df->n = f->n;
    if (f->n && (hipMemcpy(df->kps, f->kps, (size_t)f->n * sizeof(orb_keypoint), hipMemcpyHostToDevice) != hipSuccess ||
                 hipMemcpy(df->desc, f->desc, (size_t)f->n * 32, hipMemcpyHostToDevice) != hipSuccess))
        return ORB_ERR_DEVICE;
    df->fv_nnodes = -1;
    if ((rc = df_geometry(df, f, f->n)) || (rc = df_offsets(df)) || (rc = df_grids(df))) return rc;
    return df_featvec(df, fv);
}

int orbm_dframe_from_extractor(orbm_dframe* df, orbx_handle* h, const orbm_frame* geom, const orbm_featvec* fv) {
    if (!df || !h || !geom) return ORB_ERR_PARAM;
    const orb_keypoint* sk = nullptr;
    const uint8_t* sd = nullptr;
    int n = 0, dev = 0;
    if (extractor_last_outputs(h, &sk, &sd, &n, &dev) != ORB_OK || dev != df->device) return ORB_ERR_PARAM;
    if (hipSetDevice(df->device) != hipSuccess) return ORB_ERR_DEVICE;
    int rc;
    if ((rc = grow_dev(df->kps, df->cap_k, n)) || (rc = grow_dev(df->desc, df->cap_d, (size_t)n * 32))) return rc;
    df->n = n;
    // device to device by the copy kernel (k_pull) on the null stream: the
    // extraction has completed (orbx_extract returned after synchronising)
    if (n && (pull_to_device(df->kps, sk, (size_t)n * sizeof(orb_keypoint), 0) != hipSuccess ||
              pull_to_device(df->desc, sd, (size_t)n * 32, 0) != hipSuccess))
        return ORB_ERR_DEVICE;
    df->fv_nnodes = -1;
    if ((rc = df_geometry(df, geom, n)) || (rc = df_offsets(df)) || (rc = df_grids(df))) return rc;
    return df_featvec(df, fv);
}

int orbm_dframe_set_featvec(orbm_dframe* df, const orbm_featvec* fv) {
    if (!df || !fv) return ORB_ERR_PARAM;
    if (hipSetDevice(df->device) != hipSuccess) return ORB_ERR_DEVICE;
    return df_featvec(df, fv);
}

int orbm_search_by_bow_dframe(const orbm_dframe* kf, const uint8_t* kf_mp_valid, const orbm_dframe* f,
                              float nnratio, int check_ori, int32_t* match_f) {
    if (!kf || !f || !match_f || kf->fv_nnodes < 0 || f->fv_nnodes < 0 || (kf->n && !kf_mp_valid))
        return ORB_ERR_PARAM;
    int rc;
    if ((rc = df_device({kf, f}))) return rc;
    DfScratch* S = df_scratch(f->device, (size_t)std::max(1, f->n));
    if (!S) return ORB_ERR_DEVICE;
    ZRun z;
    OutBlock out;
    if ((rc = z.begin(kf->n, false)) || (rc = out.alloc((size_t)f->n + 5, true))) return rc;
    const uint8_t* kv = z.add(kf_mp_valid, kf->n);     // read by k_bow through the mapping
    BowArgs a{};
    a.kf_kps = kf->kps; a.kf_desc = kf->desc; a.kf_valid = kv; a.kp_off = kf->offs;
    a.kf_node = kf->fv_node; a.kf_off = kf->fv_off; a.kf_idx = kf->fv_idx; a.node_off = kf->offs + 2;
    a.idx_off = kf->offs + 4;
    a.f_kps = f->kps; a.f_desc = f->desc; a.f_n = f->n; a.f_node = f->fv_node; a.f_off = f->fv_off;
    a.f_idx = f->fv_idx; a.f_nnodes = f->fv_nnodes; a.ratio = nnratio; a.check_ori = check_ori;
    a.match = S->match; a.nmatches = S->match + S->match_cap; a.f_nleft = -1; a.fin_ticket = S->ticket;
    a.host_out = out.d; a.done = out.flag; a.seq = out.seq; a.reset_after = 1;
    a.tstart = S->ticket + 1;
    a.single_nodes = kf->fv_nnodes;
    if (kf->n <= kBowKvLds) a.kv_lds = kf->n;
    // ORB_OPT_BOW_TRACE = n: the n-th call after it is set prints its per-wave
    // checkpoints to stderr (diagnostics)
    static int trace_opt = 0, ncall = 0;
    const int trace_call = orbmi::debug_opt(ORB_OPT_BOW_TRACE);
    if (trace_call != trace_opt) { trace_opt = trace_call; ncall = 0; }
    unsigned* wtrace = nullptr;
    const int nwtr = (int)(kf->fv_nnodes * 4);               // (16 words a wave, four waves a node)
    const bool tracing = trace_call > 0 && ++ncall == trace_call;
    if (tracing) {
        if (hipMalloc(&wtrace, (size_t)nwtr * 16 * 4) != hipSuccess ||
            hipMemset(wtrace, 0, (size_t)nwtr * 16 * 4) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
            return ORB_ERR_DEVICE;
        a.wtrace = wtrace;
    }
    S->dirty = true;                   // until the kernel has reset its scratch
    if ((rc = launch_bow(a, 1, 0, f->fv_big, kf->fv_nnodes))) return rc;
    std::vector<int32_t> res((size_t)f->n + 5);
    ORB_CHECK(out.fetch(res.data(), res.size()));
    if (tracing) {
        std::vector<unsigned> t((size_t)nwtr * 16);
        if (hipMemcpy(t.data(), wtrace, t.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return ORB_ERR_DEVICE;
        (void)hipFree(wtrace);
        fprintf(stderr, "bow trace: wave start search issued end nkf nf loads-done top3-done decided "
                        "(10 ns from the first block)\n");
        for (int w = 0; w < nwtr; ++w) {
            const unsigned* r = t.data() + (size_t)w * 16;
            if (!r[1]) continue;
            auto rel = [&](unsigned x) { return x ? (long)(x - r[0]) : -1L; };
            const double mhz = r[4] > r[1] ? 100.0 * (double)(r[11] - r[10]) / (double)(r[4] - r[1]) : 0.0;
            fprintf(stderr, "bow trace: %d %ld %ld %ld %ld %u %u %ld %ld %ld clk %.0f MHz steps %u short %u claims %u\n",
                    w, rel(r[1]), rel(r[2]), rel(r[3]), rel(r[4]), r[5], r[6], rel(r[9]), rel(r[7]), rel(r[8]), mhz,
                    r[12], r[13], r[14]);
        }
    }
    S->dirty = false;
    if (f->n) std::memcpy(match_f, res.data(), (size_t)f->n * 4);
    // orbm_debug_proj_stats (10 ns ticks from the first block's start): [6]
    // the last arrival, [7] the final phase, [8] the last block past its frame
    // node table, [9] the last wave past its nodes
    int32_t* st = proj_stats();
    std::fill(st, st + 12, 0);
    st[6] = res[f->n + 1];
    st[7] = res[f->n + 2];
    st[8] = res[f->n + 3];
    st[9] = res[f->n + 4];
    return res[f->n];
}

int orbm_search_for_initialization_dframe(const orbm_dframe* f1, const orbm_dframe* f2, float* prev_xy, int window,
                                          float nnratio, int check_ori, int32_t* matches12) {
    if (!f1 || !f2 || !prev_xy || !matches12) return ORB_ERR_PARAM;
    int rc;
    if ((rc = df_device({f1, f2}))) return rc;
    const int n1 = f1->n, n2 = f2->n;
    if (n1 > kFusedMaxN || n2 > kFusedMaxN || nnratio < 0.2f || sfi_fused_lds(n1, n2) > kCuLds)
        return ORB_ERR_UNSUPPORTED;
    DfScratch* S = df_scratch(f1->device, 0);
    if (!S) return ORB_ERR_DEVICE;
    ZRun z;
    OutBlock out;
    if ((rc = z.begin((size_t)8 * n1, true)) || (rc = out.alloc((size_t)13 + 3 * n1, true))) return rc;
    SfiFusedArgs a{};
    a.k1 = f1->kps; a.d1 = f1->desc; a.n1 = n1; a.k2 = f2->kps; a.d2 = f2->desc; a.n2 = n2;
    a.prev = z.add(prev_xy, (size_t)2 * n1);
    a.g = f2->g; a.window = (float)window; a.ratio = nnratio; a.check_ori = check_ori;
    int bound = kThLow;
    while (bound < 255 && (float)(bound + 1) * nnratio <= (float)kThLow) ++bound;
    a.bound = bound;
    uint32_t* lists = (uint32_t*)dev_arena().get((size_t)std::max(1, n1) * kTopK * 4);
    int* cnt = (int*)dev_arena().get((size_t)std::max(1, n1) * 4);
    if (!lists || !cnt) return ORB_ERR_DEVICE;
    const int nblk = std::max(1, (n1 + kFusedThreads / kWave - 1) / (kFusedThreads / kWave));
    const size_t gb = lds_grid_bytes(n2);
    const int use_grid = sfi_fused_lds(n1, n2) + gb <= kCuLds;
    const size_t lds = sfi_fused_lds(n1, n2) + (use_grid ? gb : 0);
    S->dirty = true;
    KLAUNCH(k_sfi_fused, dim3(nblk), dim3(kFusedThreads), lds, 0, a, lists, cnt, S->ticket, out.d, use_grid, 0,
            out.flag, out.seq, z.mirror(), use_grid ? f2->grid[1] : nullptr);
    ORB_CHECK(hipGetLastError());
    std::vector<int32_t> res((size_t)13 + 3 * n1);
    ORB_CHECK(out.fetch(res.data(), res.size()));
    S->dirty = false;
    std::memcpy(proj_stats(), res.data() + 1 + 3 * n1, 12 * sizeof(int32_t));
    if (n1) {
        std::memcpy(matches12, res.data() + 1, (size_t)n1 * sizeof(int32_t));
        std::memcpy(prev_xy, res.data() + 1 + n1, (size_t)n1 * 2 * sizeof(float));
    }
    return res[0];
}

int orbm_search_by_projection_mps_dframe(const orbm_dframe* f, const orbm_mappoints* mps, float th, int far_points,
                                         float th_far, float nnratio, int32_t* owner, const uint8_t* blocked) {
    if (!f || !mps || !owner || !blocked || !f->has_scale || mps->n < 0) return ORB_ERR_PARAM;
    const int nq = mps->n;
    if (nq && (!mps->proj_x || !mps->proj_y || !mps->proj_xr || !mps->level || !mps->view_cos || !mps->track_depth ||
               !mps->in_view || !mps->has_obs || !mps->desc))
        return ORB_ERR_PARAM;
    int rc;
    if ((rc = df_device({f}))) return rc;
    if (f->n > 0xffff) return ORB_ERR_UNSUPPORTED;
    for (int i = 0; i < nq; ++i)
        if (mps->in_view[i] && (mps->level[i] < 0 || mps->level[i] >= f->nlevels)) return ORB_ERR_PARAM;
    const size_t nn = (size_t)std::max(1, f->n);
    ZRun z;
    if ((rc = z.begin((size_t)nq * (4 * 6 + 2 + 32) + 6 * 16 + nn * 5 + 32, true))) return rc;
    ProjArgs a{};
    a.mode = 0; a.nq = nq;
    a.qdesc = z.add(mps->desc, (size_t)nq * 32);
    a.qx = z.add(mps->proj_x, nq); a.qy = z.add(mps->proj_y, nq); a.qxr = z.add(mps->proj_xr, nq);
    a.qlevel = z.add(mps->level, nq); a.qviewcos = z.add(mps->view_cos, nq); a.qdepth = z.add(mps->track_depth, nq);
    a.qvalid = z.add(mps->in_view, nq); a.qhas_obs = z.add(mps->has_obs, nq); a.qangle = nullptr;
    const int32_t* own = z.add(owner, (size_t)f->n);
    a.blocked = z.add(blocked, (size_t)f->n);
    a.th = th; a.th_far = th_far; a.ratio = nnratio; a.far_points = far_points; a.last_mode = 0; a.check_ori = 0;
    return run_proj_dframe(a, f, z, own, owner);
}

int orbm_search_by_projection_last_dframe(const orbm_dframe* cur, int nlast, const uint8_t* valid, const float* u,
                                          const float* v, const float* ur, const int32_t* last_octave,
                                          const float* last_angle, const uint8_t* has_obs,
                                          const uint8_t* last_desc, float th, int mode, int check_ori,
                                          int32_t* owner, const uint8_t* blocked) {
    if (!cur || !owner || !blocked || !cur->has_scale || nlast < 0) return ORB_ERR_PARAM;
    if (nlast && (!valid || !u || !v || !ur || !last_octave || !last_angle || !has_obs || !last_desc))
        return ORB_ERR_PARAM;
    int rc;
    if ((rc = df_device({cur}))) return rc;
    if (cur->n > 0xffff) return ORB_ERR_UNSUPPORTED;
    for (int i = 0; i < nlast; ++i)
        if (valid[i] && (last_octave[i] < 0 || last_octave[i] >= cur->nlevels)) return ORB_ERR_PARAM;
    const size_t nn = (size_t)std::max(1, cur->n);
    ZRun z;
    if ((rc = z.begin((size_t)nlast * (4 * 5 + 2 + 32) + 6 * 16 + nn * 5 + 32, true))) return rc;
    ProjArgs a{};
    a.mode = 1; a.nq = nlast;
    a.qdesc = z.add(last_desc, (size_t)nlast * 32);
    a.qx = z.add(u, nlast); a.qy = z.add(v, nlast); a.qxr = z.add(ur, nlast);
    a.qlevel = z.add(last_octave, nlast); a.qangle = z.add(last_angle, nlast);
    a.qvalid = z.add(valid, nlast); a.qhas_obs = z.add(has_obs, nlast);
    a.qviewcos = nullptr; a.qdepth = nullptr;
    const int32_t* own = z.add(owner, (size_t)cur->n);
    a.blocked = z.add(blocked, (size_t)cur->n);
    a.th = th; a.th_far = 0; a.ratio = 0; a.far_points = 0; a.last_mode = mode; a.check_ori = check_ori;
    a.skip_any = 0; a.accept = (float)kThHigh;                                   // :1770
    return run_proj_dframe(a, cur, z, own, owner);
}

}  // extern "C"
