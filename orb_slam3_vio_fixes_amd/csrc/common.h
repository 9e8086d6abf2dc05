// common.h — HIP helpers shared by the extractor and matcher translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orb_mi355x.h"

#include <unordered_map>

#define ORB_CHECK(call)                                  \
    do {                                                 \
        hipError_t e_ = (call);                          \
        if (e_ != hipSuccess) return ORB_ERR_DEVICE;     \
    } while (0)

// Every product launch: refused with ORB_ERR_UNSUPPORTED when static + dynamic
// LDS exceed a CU (orbmi::lds_fits), otherwise hipLaunchKernelGGL.
#define ORB_LAUNCH(K, G, B, S, ST, ...)                                                  \
    do {                                                                                 \
        if (!::orbmi::lds_fits(reinterpret_cast<const void*>(K), (size_t)(S)))           \
            return ORB_ERR_UNSUPPORTED;                                                  \
        hipLaunchKernelGGL(K, G, B, S, ST, ##__VA_ARGS__);                               \
    } while (0)

namespace orbmi {

constexpr int kWave = 64;
constexpr size_t kCuLds = 160 * 1024;       // LDS of one CU: a workgroup's ceiling (MI355X_MICROARCH.md)

// Launch-time LDS guard: a kernel's static LDS (hipFuncGetAttributes, once per
// kernel and thread) plus the launch's dynamic LDS must fit one CU, or the
// launch is refused before it reaches the device (an over-subscribed launch
// faults the GPU instead of failing cleanly).  A failed attribute query is not
// cached: the launch is refused and the next one asks again.
inline bool lds_fits(const void* kernel, size_t dyn) {
    static thread_local std::unordered_map<const void*, size_t>* cache = new std::unordered_map<const void*, size_t>();
    size_t st = 0;
    const auto it = cache->find(kernel);
    if (it != cache->end()) {
        st = it->second;
    } else {
        hipFuncAttributes at{};
        if (hipFuncGetAttributes(&at, kernel) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        st = at.sharedSizeBytes;
        cache->emplace(kernel, st);
    }
    return dyn + st <= kCuLds;
}

// The last orbx_extract's keypoints / descriptors in HBM (extractor.hip), for
// the matcher's device-resident frames (orbm_dframe_from_extractor).
int extractor_last_outputs(orbx_handle* h, const orb_keypoint** kps, const uint8_t** desc, int* n, int* device);

// orb_debug_set_option's process-wide table (matcher.hip): alternative kernel
// forms for parity tests; every product default is 0
int debug_opt(int option);

// Host -> device copy of a pinned host buffer by a kernel reading it through
// its device mapping (matcher.hip; hipMemcpyAsync when the buffer is not
// mapped, misaligned, or ORB_OPT_UPLOAD is 1).  Stream-ordered, capturable.
hipError_t pull_to_device(void* dst, const void* src_pinned, size_t len, hipStream_t st);

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }
// wave index within the block, made wave-uniform (SGPR) so per-wave indexing
// of global tables compiles to scalar loads
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// Wave-wide minimum in registers (DPP): quad permutes and row rotations give
// every lane its row-of-16 minimum, row_bcast:15 / row_bcast:31 (gfx9 DPP)
// fold the rows into lane 63, read back as a wave-uniform value.  Lanes of
// rows a broadcast does not write keep `old` = the identity.  No LDS traffic,
// unlike __shfl_xor (ds_bpermute).
template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_mov(int v, int id) {
    return __builtin_amdgcn_update_dpp(id, v, CTRL, ROWS, 0xf, false);
}

template <typename T>
__device__ __forceinline__ T dpp_min2(T v, int x) {
    const T o = __builtin_bit_cast(T, x);
    return o < v ? o : v;
}

template <typename T>
__device__ __forceinline__ T wave_min(T v, T id) {
    const int ii = __builtin_bit_cast(int, id);
    v = dpp_min2(v, dpp_mov<0xb1, 0xf>(__builtin_bit_cast(int, v), ii));    // quad_perm [1,0,3,2]
    v = dpp_min2(v, dpp_mov<0x4e, 0xf>(__builtin_bit_cast(int, v), ii));    // quad_perm [2,3,0,1]
    v = dpp_min2(v, dpp_mov<0x124, 0xf>(__builtin_bit_cast(int, v), ii));   // row_ror:4
    v = dpp_min2(v, dpp_mov<0x128, 0xf>(__builtin_bit_cast(int, v), ii));   // row_ror:8
    v = dpp_min2(v, dpp_mov<0x142, 0xa>(__builtin_bit_cast(int, v), ii));   // row_bcast:15 -> rows 1, 3
    v = dpp_min2(v, dpp_mov<0x143, 0xc>(__builtin_bit_cast(int, v), ii));   // row_bcast:31 -> rows 2, 3
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), kWave - 1));
}

// Wave-wide sum by the same DPP steps as wave_min (identity 0 for the lanes a
// broadcast does not write): six dependent VALU ops instead of six
// ds_bpermute round trips through the LDS unit.
__device__ __forceinline__ int wave_sum_dpp(int v) {
    v += dpp_mov<0xb1, 0xf>(v, 0);    // quad_perm [1,0,3,2]
    v += dpp_mov<0x4e, 0xf>(v, 0);    // quad_perm [2,3,0,1]
    v += dpp_mov<0x124, 0xf>(v, 0);   // row_ror:4
    v += dpp_mov<0x128, 0xf>(v, 0);   // row_ror:8
    v += dpp_mov<0x142, 0xa>(v, 0);   // row_bcast:15 -> rows 1, 3
    v += dpp_mov<0x143, 0xc>(v, 0);   // row_bcast:31 -> rows 2, 3
    return __builtin_amdgcn_readlane(v, kWave - 1);
}

// Inclusive prefix sum over the wave by DPP (row_shr within rows of 16, then
// the row broadcasts), no LDS traffic; every lane of the wave active.
__device__ __forceinline__ int wave_incl_scan_dpp(int v) {
    v += dpp_mov<0x111, 0xf>(v, 0);   // row_shr:1
    v += dpp_mov<0x112, 0xf>(v, 0);   // row_shr:2
    v += dpp_mov<0x114, 0xf>(v, 0);   // row_shr:4
    v += dpp_mov<0x118, 0xf>(v, 0);   // row_shr:8
    v += dpp_mov<0x142, 0xa>(v, 0);   // row_bcast:15 -> rows 1, 3
    v += dpp_mov<0x143, 0xc>(v, 0);   // row_bcast:31 -> rows 2, 3
    return v;
}

// Position of this lane among the set bits of `mask` below it.
__device__ __forceinline__ int mask_rank(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

__device__ __forceinline__ int wave_incl_scan(int v) {
    const int l = lane_id();
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const int t = __shfl_up(v, o, kWave);
        if (l >= o) v += t;
    }
    return v;
}

// Exclusive scan, in place, of n ints in LDS (any n); every thread of the
// block must call it; `tmp` holds >= blockDim.x/64 + 1 ints.  Returns the total.
__device__ int block_excl_scan(int* a, int n, int* tmp) {
    const int T = blockDim.x, t = threadIdx.x;
    const int per = (n + T - 1) / T;
    const int b = min(n, t * per), e = min(n, b + per);
    int s = 0;
    for (int i = b; i < e; ++i) s += a[i];
    const int incl = wave_incl_scan_dpp(s);   // (DPP: no ds_bpermute round trips)
    if (lane_id() == kWave - 1) tmp[wave_id()] = incl;
    __syncthreads();
    if (t == 0) {
        int acc = 0;
        for (int w = 0; w < T / kWave; ++w) { const int x = tmp[w]; tmp[w] = acc; acc += x; }
        tmp[T / kWave] = acc;
    }
    __syncthreads();
    int run = tmp[wave_id()] + incl - s;
    for (int i = b; i < e; ++i) { const int x = a[i]; a[i] = run; run += x; }
    const int total = tmp[T / kWave];
    __syncthreads();
    return total;
}

// Three exclusive scans in place (a[0..na), b[0..nb), c[0..nc)) with one set
// of barriers; tot receives the three totals.  tmp: >= 3 * (waves + 1) ints.
__device__ inline void block_excl_scan3(int* a, int na, int* b, int nb, int* c, int nc, int* tmp, int (&tot)[3]) {
    const int T = blockDim.x, t = threadIdx.x, W = T / kWave;
    int* arr[3] = {a, b, c};
    const int n[3] = {na, nb, nc};
    int sum[3], incl[3], lo[3], hi[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int per = (n[j] + T - 1) / T;
        lo[j] = min(n[j], t * per);
        hi[j] = min(n[j], lo[j] + per);
        int s = 0;
        for (int i = lo[j]; i < hi[j]; ++i) s += arr[j][i];
        sum[j] = s;
        incl[j] = wave_incl_scan_dpp(s);
        if (lane_id() == kWave - 1) tmp[j * (W + 1) + wave_id()] = incl[j];
    }
    __syncthreads();
    if (t < 3) {
        int acc = 0;
        for (int w = 0; w < W; ++w) { const int x = tmp[t * (W + 1) + w]; tmp[t * (W + 1) + w] = acc; acc += x; }
        tmp[t * (W + 1) + W] = acc;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        int run = tmp[j * (W + 1) + wave_id()] + incl[j] - sum[j];
        for (int i = lo[j]; i < hi[j]; ++i) { const int x = arr[j][i]; arr[j][i] = run; run += x; }
        tot[j] = tmp[j * (W + 1) + W];
    }
    __syncthreads();
}

}  // namespace orbmi
