// common.h — HIP helpers shared by the extractor and matcher translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ORB_CHECK(call)                                  \
    do {                                                 \
        hipError_t e_ = (call);                          \
        if (e_ != hipSuccess) return ORB_ERR_DEVICE;     \
    } while (0)

namespace orbmi {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }
// wave index within the block, made wave-uniform (SGPR) so per-wave indexing
// of global tables compiles to scalar loads
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
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
    const int incl = wave_incl_scan(s);
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

}  // namespace orbmi
