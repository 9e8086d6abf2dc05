// Micro-benchmark of k_resize layouts: 256 frames 752x480 -> 627x400 (level 1
// of C2) timed with HIP events; prints us per launch per variant.
// build: hipcc --offload-arch=gfx950 -O3 tools/resize_bench.hip -o tools/_resize_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef uint16_t u16u __attribute__((aligned(1)));

struct P {
    const uint8_t* src; long long sfs; int sp, sh;
    uint8_t* dst; long long dfs; int dp, dw, dh;
    const int2* xt; const int2* yt; int xmax;
};

__device__ __forceinline__ uint32_t px(const P& a, const uint8_t* S0, const uint8_t* S1, int b0, int b1, int dx) {
    const int2 tx = a.xt[dx];
    const int sx = tx.x, a0 = (short)(tx.y & 0xffff), a1 = tx.y >> 16;
    int h0, h1;
    if (dx < a.xmax) { h0 = S0[sx] * a0 + S0[sx + 1] * a1; h1 = S1[sx] * a0 + S1[sx + 1] * a1; }
    else { h0 = S0[sx] * 2048; h1 = S1[sx] * 2048; }
    return (uint32_t)((((b0 * (h0 >> 4)) >> 16) + ((b1 * (h1 >> 4)) >> 16) + 2) >> 2) & 0xff;
}

// V0: one row per wave, lanes over dx (the current shipped form)
__global__ __launch_bounds__(256) void v0(P a) {
    const int dy = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (dy >= a.dh) return;
    const int f = blockIdx.y;
    const uint8_t* S = a.src + f * a.sfs;
    uint8_t* D = a.dst + f * a.dfs + (long long)dy * a.dp;
    const int2 ty = a.yt[dy];
    const int r0 = min(max(ty.x, 0), a.sh - 1), r1 = min(max(ty.x + 1, 0), a.sh - 1);
    const int b0 = (short)(ty.y & 0xffff), b1 = ty.y >> 16;
    const uint8_t* S0 = S + (long long)r0 * a.sp;
    const uint8_t* S1 = S + (long long)r1 * a.sp;
    for (int dx = threadIdx.x & 63; dx < a.dw; dx += 64) D[dx] = (uint8_t)px(a, S0, S1, b0, b1, dx);
}

// V0U: V0 with U iterations' loads issued together (2 serial latencies per U)
template <int U>
__global__ __launch_bounds__(256) void v0u(P a) {
    const int dy = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (dy >= a.dh) return;
    const int f = blockIdx.y;
    const uint8_t* S = a.src + f * a.sfs;
    uint8_t* D = a.dst + f * a.dfs + (long long)dy * a.dp;
    const int2 ty = a.yt[dy];
    const int r0 = min(max(ty.x, 0), a.sh - 1), r1 = min(max(ty.x + 1, 0), a.sh - 1);
    const int b0 = (short)(ty.y & 0xffff), b1 = ty.y >> 16;
    const uint8_t* S0 = S + (long long)r0 * a.sp;
    const uint8_t* S1 = S + (long long)r1 * a.sp;
    const int lane = threadIdx.x & 63;
    for (int base = 0; base < a.dw; base += 64 * U) {
        int2 tx[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int dx = base + u * 64 + lane;
            tx[u] = a.xt[min(dx, a.dw - 1)];
        }
        int t00[U], t01[U], t10[U], t11[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int dx = base + u * 64 + lane;
            const int sx = tx[u].x, sx1 = dx < a.xmax ? sx + 1 : sx;
            t00[u] = S0[sx]; t01[u] = S0[sx1]; t10[u] = S1[sx]; t11[u] = S1[sx1];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int dx = base + u * 64 + lane;
            const int a0 = (short)(tx[u].y & 0xffff), a1 = tx[u].y >> 16;
            int h0, h1;
            if (dx < a.xmax) { h0 = t00[u] * a0 + t01[u] * a1; h1 = t10[u] * a0 + t11[u] * a1; }
            else { h0 = t00[u] * 2048; h1 = t10[u] * 2048; }
            if (dx < a.dw) D[dx] = (uint8_t)((((b0 * (h0 >> 4)) >> 16) + ((b1 * (h1 >> 4)) >> 16) + 2) >> 2);
        }
    }
}

// V1: 4 px per thread, byte taps, dword store; block 64x4
template <bool U16>
__global__ __launch_bounds__(256) void v1(P a) {
    const int dy = blockIdx.y * 4 + threadIdx.y;
    const int dx0 = 4 * (blockIdx.x * 64 + threadIdx.x);
    if (dy >= a.dh || dx0 >= a.dw) return;
    const long long f = blockIdx.z;
    const uint8_t* S = a.src + f * a.sfs;
    uint8_t* D = a.dst + f * a.dfs + (long long)dy * a.dp;
    const int2 ty = a.yt[dy];
    const int r0 = min(max(ty.x, 0), a.sh - 1), r1 = min(max(ty.x + 1, 0), a.sh - 1);
    const int b0 = (short)(ty.y & 0xffff), b1 = ty.y >> 16;
    const uint8_t* S0 = S + (long long)r0 * a.sp;
    const uint8_t* S1 = S + (long long)r1 * a.sp;
    const int n = min(4, a.dw - dx0);
    uint32_t out = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (k < n) {
            const int dx = dx0 + k;
            uint32_t v;
            if (U16 && dx < a.xmax) {
                const int2 tx = a.xt[dx];
                const int sx = tx.x, a0 = (short)(tx.y & 0xffff), a1 = tx.y >> 16;
                const uint32_t p0 = *(const u16u*)(S0 + sx), p1 = *(const u16u*)(S1 + sx);
                const int h0 = (int)(p0 & 0xff) * a0 + (int)(p0 >> 8) * a1, h1 = (int)(p1 & 0xff) * a0 + (int)(p1 >> 8) * a1;
                v = (uint32_t)((((b0 * (h0 >> 4)) >> 16) + ((b1 * (h1 >> 4)) >> 16) + 2) >> 2) & 0xff;
            } else {
                v = px(a, S0, S1, b0, b1, dx);
            }
            out |= v << (8 * k);
        }
    if (n == 4) *(uint32_t*)(D + dx0) = out;
    else for (int k = 0; k < n; ++k) D[dx0 + k] = (uint8_t)(out >> (8 * k));
}

// V2: LDS-staged source rows.  Block = 256 threads, TR output rows of one frame;
// stage the needed source rows (dwordx4 loads) then compute 4 px per thread.
template <int TR>
__global__ __launch_bounds__(256) void v2(P a) {
    __shared__ __attribute__((aligned(16))) uint8_t rows[(2 * TR + 4) * 1024];
    const int y0 = blockIdx.x * TR;
    const int f = blockIdx.y;
    const uint8_t* S = a.src + (long long)f * a.sfs;
    const int ylast = min(y0 + TR, a.dh) - 1;
    const int sr0 = min(max(a.yt[y0].x, 0), a.sh - 1);
    const int sr1 = min(max(a.yt[ylast].x + 1, 0), a.sh - 1);
    const int nr = sr1 - sr0 + 1;
    const int rw16 = (a.sp + 15) >> 4;     // 16-B chunks per source row (pitch multiple of 16 assumed)
    const int rp = rw16 * 16;
    for (int i = threadIdx.x; i < nr * rw16; i += 256) {
        const int r = i / rw16, c = i - r * rw16;
        ((uint4*)(rows + r * rp))[c] = ((const uint4*)(S + (long long)(sr0 + r) * a.sp))[c];
    }
    __syncthreads();
    const int ng = (a.dw + 3) >> 2;
    for (int i = threadIdx.x; i < TR * ng; i += 256) {
        const int ry = i / ng, g = i - ry * ng;
        const int dy = y0 + ry;
        if (dy >= a.dh) break;
        const int2 ty = a.yt[dy];
        const int r0 = min(max(ty.x, 0), a.sh - 1) - sr0, r1 = min(max(ty.x + 1, 0), a.sh - 1) - sr0;
        const int b0 = (short)(ty.y & 0xffff), b1 = ty.y >> 16;
        const uint8_t* S0 = rows + r0 * rp;
        const uint8_t* S1 = rows + r1 * rp;
        const int dx0 = 4 * g, n = min(4, a.dw - dx0);
        uint32_t out = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k < n) out |= px(a, S0, S1, b0, b1, dx0 + k) << (8 * k);
        uint8_t* D = a.dst + (long long)f * a.dfs + (long long)dy * a.dp;
        if (n == 4) *(uint32_t*)(D + dx0) = out;
        else for (int k = 0; k < n; ++k) D[dx0 + k] = (uint8_t)(out >> (8 * k));
    }
}

// V3: LDS-staged source rows AND x table (contiguous 16-B loads only); 4 px
// per thread from LDS bytes; dword stores.
template <int TR>
__global__ __launch_bounds__(256) void v3(P a) {
    __shared__ __attribute__((aligned(16))) uint8_t rows[(2 * TR + 4) * 1024];
    __shared__ __attribute__((aligned(16))) int2 xs[2048];
    const int y0 = blockIdx.x * TR;
    const int f = blockIdx.y;
    const uint8_t* S = a.src + (long long)f * a.sfs;
    const int ylast = min(y0 + TR, a.dh) - 1;
    const int sr0 = min(max(a.yt[y0].x, 0), a.sh - 1);
    const int sr1 = min(max(a.yt[ylast].x + 1, 0), a.sh - 1);
    const int nr = sr1 - sr0 + 1;
    const int rw16 = (a.sp + 15) >> 4;
    const int rp = rw16 * 16;
    for (int i = threadIdx.x; i < nr * rw16; i += 256) {
        const int r = i / rw16, c = i - r * rw16;
        ((uint4*)(rows + r * rp))[c] = ((const uint4*)(S + (long long)(sr0 + r) * a.sp))[c];
    }
    for (int i = threadIdx.x; i < (a.dw + 1) / 2; i += 256) ((int4*)xs)[i] = ((const int4*)a.xt)[i];
    __syncthreads();
    const int ng = (a.dw + 3) >> 2;
    for (int i = threadIdx.x; i < TR * ng; i += 256) {
        const int ry = i / ng, g = i - ry * ng;
        const int dy = y0 + ry;
        if (dy >= a.dh) break;
        const int2 ty = a.yt[dy];
        const int r0 = min(max(ty.x, 0), a.sh - 1) - sr0, r1 = min(max(ty.x + 1, 0), a.sh - 1) - sr0;
        const int b0 = (short)(ty.y & 0xffff), b1 = ty.y >> 16;
        const uint8_t* S0 = rows + r0 * rp;
        const uint8_t* S1 = rows + r1 * rp;
        const int dx0 = 4 * g, n = min(4, a.dw - dx0);
        uint32_t out = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k < n) {
                const int dx = dx0 + k;
                const int2 tx = xs[dx];
                const int sx = tx.x, a0 = (short)(tx.y & 0xffff), a1 = tx.y >> 16;
                int h0, h1;
                if (dx < a.xmax) { h0 = S0[sx] * a0 + S0[sx + 1] * a1; h1 = S1[sx] * a0 + S1[sx + 1] * a1; }
                else { h0 = S0[sx] * 2048; h1 = S1[sx] * 2048; }
                out |= ((uint32_t)((((b0 * (h0 >> 4)) >> 16) + ((b1 * (h1 >> 4)) >> 16) + 2) >> 2) & 0xff) << (8 * k);
            }
        uint8_t* D = a.dst + (long long)f * a.dfs + (long long)dy * a.dp;
        if (n == 4) *(uint32_t*)(D + dx0) = out;
        else for (int k = 0; k < n; ++k) D[dx0 + k] = (uint8_t)(out >> (8 * k));
    }
}

// V4: LDS-staged rows + x table, lanes over consecutive dx (v0 pattern), byte stores
template <int TR>
__global__ __launch_bounds__(256) void v4(P a) {
    __shared__ __attribute__((aligned(16))) uint8_t rows[(2 * TR + 4) * 1024];
    __shared__ __attribute__((aligned(16))) int2 xs[2048];
    const int y0 = blockIdx.x * TR;
    const int f = blockIdx.y;
    const uint8_t* S = a.src + (long long)f * a.sfs;
    const int ylast = min(y0 + TR, a.dh) - 1;
    const int sr0 = min(max(a.yt[y0].x, 0), a.sh - 1);
    const int sr1 = min(max(a.yt[ylast].x + 1, 0), a.sh - 1);
    const int nr = sr1 - sr0 + 1;
    const int rw16 = (a.sp + 15) >> 4;
    const int rp = rw16 * 16;
    for (int i = threadIdx.x; i < nr * rw16; i += 256) {
        const int r = i / rw16, c = i - r * rw16;
        ((uint4*)(rows + r * rp))[c] = ((const uint4*)(S + (long long)(sr0 + r) * a.sp))[c];
    }
    for (int i = threadIdx.x; i < (a.dw + 1) / 2; i += 256) ((int4*)xs)[i] = ((const int4*)a.xt)[i];
    __syncthreads();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int ry = w; ry < TR; ry += 4) {
        const int dy = y0 + ry;
        if (dy >= a.dh) break;
        const int2 ty = a.yt[dy];
        const int r0 = min(max(ty.x, 0), a.sh - 1) - sr0, r1 = min(max(ty.x + 1, 0), a.sh - 1) - sr0;
        const int b0 = (short)(ty.y & 0xffff), b1 = ty.y >> 16;
        const uint8_t* S0 = rows + r0 * rp;
        const uint8_t* S1 = rows + r1 * rp;
        uint8_t* D = a.dst + (long long)f * a.dfs + (long long)dy * a.dp;
        for (int dx = lane; dx < a.dw; dx += 64) {
            const int2 tx = xs[dx];
            const int sx = tx.x, a0 = (short)(tx.y & 0xffff), a1 = tx.y >> 16;
            int h0, h1;
            if (dx < a.xmax) { h0 = S0[sx] * a0 + S0[sx + 1] * a1; h1 = S1[sx] * a0 + S1[sx + 1] * a1; }
            else { h0 = S0[sx] * 2048; h1 = S1[sx] * 2048; }
            D[dx] = (uint8_t)((((b0 * (h0 >> 4)) >> 16) + ((b1 * (h1 >> 4)) >> 16) + 2) >> 2);
        }
    }
}

// V5: v0 with the x taps/weights computed in registers (no table load)
__global__ __launch_bounds__(256) void v5(P a, double scale_x, int sw) {
    const int dy = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (dy >= a.dh) return;
    const int f = blockIdx.y;
    const uint8_t* S = a.src + f * a.sfs;
    uint8_t* D = a.dst + f * a.dfs + (long long)dy * a.dp;
    const int2 ty = a.yt[dy];
    const int r0 = min(max(ty.x, 0), a.sh - 1), r1 = min(max(ty.x + 1, 0), a.sh - 1);
    const int b0 = (short)(ty.y & 0xffff), b1 = ty.y >> 16;
    const uint8_t* S0 = S + (long long)r0 * a.sp;
    const uint8_t* S1 = S + (long long)r1 * a.sp;
    for (int dx = threadIdx.x & 63; dx < a.dw; dx += 64) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)floorf(fx); fx -= sx;
        int a0 = (int)rintf((1.f - fx) * 2048), a1 = (int)rintf(fx * 2048);
        if (sx < 0) { sx = 0; a0 = 2048; a1 = 0; }
        int h0, h1;
        if (dx < a.xmax) { h0 = S0[sx] * a0 + S0[sx + 1] * a1; h1 = S1[sx] * a0 + S1[sx + 1] * a1; }
        else { h0 = S0[sx] * 2048; h1 = S1[sx] * 2048; }
        D[dx] = (uint8_t)((((b0 * (h0 >> 4)) >> 16) + ((b1 * (h1 >> 4)) >> 16) + 2) >> 2);
    }
}

// V6: v5 with both horizontal taps of a source row in one unaligned 2-byte load
__global__ __launch_bounds__(256) void v6(P a, double scale_x, int sw) {
    const int dy = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (dy >= a.dh) return;
    const int f = blockIdx.y;
    const uint8_t* S = a.src + f * a.sfs;
    uint8_t* D = a.dst + f * a.dfs + (long long)dy * a.dp;
    const int2 ty = a.yt[dy];
    const int r0 = min(max(ty.x, 0), a.sh - 1), r1 = min(max(ty.x + 1, 0), a.sh - 1);
    const int b0 = (short)(ty.y & 0xffff), b1 = ty.y >> 16;
    const uint8_t* S0 = S + (long long)r0 * a.sp;
    const uint8_t* S1 = S + (long long)r1 * a.sp;
    for (int dx = threadIdx.x & 63; dx < a.dw; dx += 64) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)floorf(fx); fx -= sx;
        int a0 = (int)rintf((1.f - fx) * 2048), a1 = (int)rintf(fx * 2048);
        if (sx < 0) { sx = 0; a0 = 2048; a1 = 0; }
        int h0, h1;
        if (dx < a.xmax) {
            const uint32_t p0 = *(const u16u*)(S0 + sx), p1 = *(const u16u*)(S1 + sx);
            h0 = (int)(p0 & 0xff) * a0 + (int)(p0 >> 8) * a1; h1 = (int)(p1 & 0xff) * a0 + (int)(p1 >> 8) * a1;
        } else { h0 = S0[sx] * 2048; h1 = S1[sx] * 2048; }
        D[dx] = (uint8_t)((((b0 * (h0 >> 4)) >> 16) + ((b1 * (h1 >> 4)) >> 16) + 2) >> 2);
    }
}

// V7: v5, two output rows per wave (rows dy and dy + dh/2 share nothing; just more work per wave)
__global__ __launch_bounds__(256) void v7(P a, double scale_x, int sw) {
    const int dy = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (dy >= a.dh) return;
    const int f = blockIdx.y;
    const uint8_t* S = a.src + f * a.sfs;
    uint8_t* D = a.dst + f * a.dfs + (long long)dy * a.dp;
    const int2 ty = a.yt[dy];
    const int r0 = min(max(ty.x, 0), a.sh - 1), r1 = min(max(ty.x + 1, 0), a.sh - 1);
    const int b0 = (short)(ty.y & 0xffff), b1 = ty.y >> 16;
    const uint8_t* S0 = S + (long long)r0 * a.sp;
    const uint8_t* S1 = S + (long long)r1 * a.sp;
    for (int dx = threadIdx.x & 63; dx < a.dw; dx += 64) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)floorf(fx); fx -= sx;
        int a0 = (int)rintf((1.f - fx) * 2048), a1 = (int)rintf(fx * 2048);
        if (sx < 0) { sx = 0; a0 = 2048; a1 = 0; }
        const bool in = dx < a.xmax;
        const int sx1 = in ? sx + 1 : sx;
        const int p00 = S0[sx], p01 = S0[sx1], p10 = S1[sx], p11 = S1[sx1];
        const int h0 = in ? p00 * a0 + p01 * a1 : p00 * 2048;
        const int h1 = in ? p10 * a0 + p11 * a1 : p10 * 2048;
        const uint32_t v = (uint32_t)((((b0 * (h0 >> 4)) >> 16) + ((b1 * (h1 >> 4)) >> 16) + 2) >> 2) & 0xff;
        // pack 4 neighbouring lanes' bytes: lanes 4q..4q+3 -> lane 4q stores a dword
        const uint32_t v1 = __shfl_down(v, 1, 64), v2 = __shfl_down(v, 2, 64), v3 = __shfl_down(v, 3, 64);
        const int lane = threadIdx.x & 63;
        if ((lane & 3) == 0) {
            if (dx + 3 < a.dw) *(uint32_t*)(D + dx) = v | (v1 << 8) | (v2 << 16) | (v3 << 24);
            else { D[dx] = v; if (dx + 1 < a.dw) D[dx + 1] = v1; if (dx + 2 < a.dw) D[dx + 2] = v2; }
        }
    }
}

// V8: v4 (LDS-staged source rows, coalesced lanes) with computed x taps
template <int TR>
__global__ __launch_bounds__(256) void v8(P a, double scale_x, int sw) {
    __shared__ __attribute__((aligned(16))) uint8_t rows[(2 * TR + 4) * 1024];
    const int y0 = blockIdx.x * TR;
    const int f = blockIdx.y;
    const uint8_t* S = a.src + (long long)f * a.sfs;
    const int ylast = min(y0 + TR, a.dh) - 1;
    const int sr0 = min(max(a.yt[y0].x, 0), a.sh - 1);
    const int sr1 = min(max(a.yt[ylast].x + 1, 0), a.sh - 1);
    const int nr = sr1 - sr0 + 1;
    const int rw16 = (a.sp + 15) >> 4;
    const int rp = rw16 * 16;
    for (int i = threadIdx.x; i < nr * rw16; i += 256) {
        const int r = i / rw16, c = i - r * rw16;
        ((uint4*)(rows + r * rp))[c] = ((const uint4*)(S + (long long)(sr0 + r) * a.sp))[c];
    }
    __syncthreads();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int ry = w; ry < TR; ry += 4) {
        const int dy = y0 + ry;
        if (dy >= a.dh) break;
        const int2 ty = a.yt[dy];
        const int r0 = min(max(ty.x, 0), a.sh - 1) - sr0, r1 = min(max(ty.x + 1, 0), a.sh - 1) - sr0;
        const int b0 = (short)(ty.y & 0xffff), b1 = ty.y >> 16;
        const uint8_t* S0 = rows + r0 * rp;
        const uint8_t* S1 = rows + r1 * rp;
        uint8_t* D = a.dst + (long long)f * a.dfs + (long long)dy * a.dp;
        for (int dx = lane; dx < a.dw; dx += 64) {
            float fx = (float)((dx + 0.5) * scale_x - 0.5);
            int sx = (int)floorf(fx); fx -= sx;
            int a0 = (int)rintf((1.f - fx) * 2048), a1 = (int)rintf(fx * 2048);
            if (sx < 0) { sx = 0; a0 = 2048; a1 = 0; }
            int h0, h1;
            if (dx < a.xmax) { h0 = S0[sx] * a0 + S0[sx + 1] * a1; h1 = S1[sx] * a0 + S1[sx + 1] * a1; }
            else { h0 = S0[sx] * 2048; h1 = S1[sx] * 2048; }
            D[dx] = (uint8_t)((((b0 * (h0 >> 4)) >> 16) + ((b1 * (h1 >> 4)) >> 16) + 2) >> 2);
        }
    }
}

// V9: v5 with two consecutive output rows per wave sharing the middle source row
__global__ __launch_bounds__(256) void v9(P a, double scale_x, int sw) {
    const int dy = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2;
    if (dy >= a.dh) return;
    const int f = blockIdx.y;
    const uint8_t* S = a.src + f * a.sfs;
    const bool two = dy + 1 < a.dh;
    const int2 ta = a.yt[dy], tb = a.yt[two ? dy + 1 : dy];
    const int ra0 = min(max(ta.x, 0), a.sh - 1), ra1 = min(max(ta.x + 1, 0), a.sh - 1);
    const int rb0 = min(max(tb.x, 0), a.sh - 1), rb1 = min(max(tb.x + 1, 0), a.sh - 1);
    const int ab0 = (short)(ta.y & 0xffff), ab1 = ta.y >> 16, bb0 = (short)(tb.y & 0xffff), bb1 = tb.y >> 16;
    const uint8_t *A0 = S + (long long)ra0 * a.sp, *A1 = S + (long long)ra1 * a.sp;
    const uint8_t *B0 = S + (long long)rb0 * a.sp, *B1 = S + (long long)rb1 * a.sp;
    const bool share = rb0 == ra1;
    uint8_t* DA = a.dst + f * a.dfs + (long long)dy * a.dp;
    uint8_t* DB = DA + a.dp;
    for (int dx = threadIdx.x & 63; dx < a.dw; dx += 64) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)floorf(fx); fx -= sx;
        int a0 = (int)rintf((1.f - fx) * 2048), a1 = (int)rintf(fx * 2048);
        if (sx < 0) { sx = 0; a0 = 2048; a1 = 0; }
        const bool in = dx < a.xmax;
        const int sx1 = in ? sx + 1 : sx;
        const int c0 = in ? a0 : 2048, c1 = in ? a1 : 0;
        const int hA0 = A0[sx] * c0 + A0[sx1] * c1;
        const int hA1 = A1[sx] * c0 + A1[sx1] * c1;
        DA[dx] = (uint8_t)((((ab0 * (hA0 >> 4)) >> 16) + ((ab1 * (hA1 >> 4)) >> 16) + 2) >> 2);
        if (two) {
            const int hB0 = share ? hA1 : B0[sx] * c0 + B0[sx1] * c1;
            const int hB1 = B1[sx] * c0 + B1[sx1] * c1;
            DB[dx] = (uint8_t)((((bb0 * (hB0 >> 4)) >> 16) + ((bb1 * (hB1 >> 4)) >> 16) + 2) >> 2);
        }
    }
}

int main() {
    const int B = 256, sw = 752, sh = 480, dw = 627, dh = 400;
    const int sp = 768, dp = 640;
    std::vector<int2> xt(dw), yt(dh);
    const double sx_ = (double)sw / dw, sy_ = (double)sh / dh;
    int xmax = dw;
    for (int x = 0; x < dw; ++x) {
        float fx = (float)((x + 0.5) * sx_ - 0.5); int s = (int)floorf(fx); fx -= s;
        if (s >= sw - 1 && xmax == dw) xmax = x;
        int a0 = (int)rintf((1.f - fx) * 2048), a1 = (int)rintf(fx * 2048);
        xt[x] = make_int2(s, (a0 & 0xffff) | (a1 << 16));
    }
    for (int y = 0; y < dh; ++y) {
        float fy = (float)((y + 0.5) * sy_ - 0.5); int s = (int)floorf(fy); fy -= s;
        int b0 = (int)rintf((1.f - fy) * 2048), b1 = (int)rintf(fy * 2048);
        yt[y] = make_int2(s, (b0 & 0xffff) | (b1 << 16));
    }
    uint8_t *src, *dst, *ref; int2 *dxt, *dyt;
    CK(hipMalloc(&src, (size_t)B * sp * sh)); CK(hipMalloc(&dst, (size_t)B * dp * dh)); CK(hipMalloc(&ref, (size_t)B * dp * dh));
    CK(hipMalloc(&dxt, dw * 8)); CK(hipMalloc(&dyt, dh * 8));
    std::vector<uint8_t> h((size_t)B * sp * sh);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint8_t)((i * 2654435761u) >> 13);
    CK(hipMemcpy(src, h.data(), h.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dxt, xt.data(), dw * 8, hipMemcpyHostToDevice)); CK(hipMemcpy(dyt, yt.data(), dh * 8, hipMemcpyHostToDevice));
    P a{src, (long long)sp * sh, sp, sh, dst, (long long)dp * dh, dp, dw, dh, dxt, dyt, xmax};
    P r = a; r.dst = ref;
    hipLaunchKernelGGL(v0, dim3((dh + 3) / 4, B), dim3(256), 0, 0, r);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<uint8_t> o((size_t)B * dp * dh), ro((size_t)B * dp * dh);
    CK(hipMemcpy(ro.data(), ref, ro.size(), hipMemcpyDeviceToHost));
    auto run = [&](const char* name, auto launch) -> int {
        CK(hipMemset(dst, 0, (size_t)B * dp * dh));
        launch(); CK(hipDeviceSynchronize());
        CK(hipMemcpy(o.data(), dst, o.size(), hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (int f = 0; f < B; ++f) for (int y = 0; y < dh; ++y) for (int x = 0; x < dw; ++x) {
            size_t i = ((size_t)f * dh + y) * dp + x; bad += o[i] != ro[i]; }
        const int it = 50;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; ++i) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / it;
        const double bytes = (double)B * (sw * sh + dw * dh);
        printf("%-12s %8.1f us  %6.0f GB/s  mismatches %zu\n", name, us, bytes / us * 1e-3, bad);
        return 0;
    };
    run("v0_row_wave", [&] { hipLaunchKernelGGL(v0, dim3((dh + 3) / 4, B), dim3(256), 0, 0, a); });
    run("v0u2", [&] { hipLaunchKernelGGL(v0u<2>, dim3((dh + 3) / 4, B), dim3(256), 0, 0, a); });
    run("v0u4", [&] { hipLaunchKernelGGL(v0u<4>, dim3((dh + 3) / 4, B), dim3(256), 0, 0, a); });
    run("v0u8", [&] { hipLaunchKernelGGL(v0u<8>, dim3((dh + 3) / 4, B), dim3(256), 0, 0, a); });
    run("v0u16", [&] { hipLaunchKernelGGL(v0u<16>, dim3((dh + 3) / 4, B), dim3(256), 0, 0, a); });
    run("v1_bytes", [&] { hipLaunchKernelGGL(v1<false>, dim3(((dw + 3) / 4 + 63) / 64, (dh + 3) / 4, B), dim3(64, 4), 0, 0, a); });
    run("v1_u16", [&] { hipLaunchKernelGGL(v1<true>, dim3(((dw + 3) / 4 + 63) / 64, (dh + 3) / 4, B), dim3(64, 4), 0, 0, a); });
    run("v4_tr4", [&] { hipLaunchKernelGGL(v4<4>, dim3((dh + 3) / 4, B), dim3(256), 0, 0, a); });
    run("v4_tr8", [&] { hipLaunchKernelGGL(v4<8>, dim3((dh + 7) / 8, B), dim3(256), 0, 0, a); });
    run("v4_tr16", [&] { hipLaunchKernelGGL(v4<16>, dim3((dh + 15) / 16, B), dim3(256), 0, 0, a); });
    run("v5_xcalc", [&] { hipLaunchKernelGGL(v5, dim3((dh + 3) / 4, B), dim3(256), 0, 0, a, sx_, sw); });
    run("v8_lds_calc4", [&] { hipLaunchKernelGGL(v8<4>, dim3((dh + 3) / 4, B), dim3(256), 0, 0, a, sx_, sw); });
    run("v8_lds_calc8", [&] { hipLaunchKernelGGL(v8<8>, dim3((dh + 7) / 8, B), dim3(256), 0, 0, a, sx_, sw); });
    run("v9_2rows", [&] { hipLaunchKernelGGL(v9, dim3((dh + 7) / 8, B), dim3(256), 0, 0, a, sx_, sw); });
    run("v6_u16", [&] { hipLaunchKernelGGL(v6, dim3((dh + 3) / 4, B), dim3(256), 0, 0, a, sx_, sw); });
    run("v7_dwstore", [&] { hipLaunchKernelGGL(v7, dim3((dh + 3) / 4, B), dim3(256), 0, 0, a, sx_, sw); });
    run("v3_tr4", [&] { hipLaunchKernelGGL(v3<4>, dim3((dh + 3) / 4, B), dim3(256), 0, 0, a); });
    run("v3_tr8", [&] { hipLaunchKernelGGL(v3<8>, dim3((dh + 7) / 8, B), dim3(256), 0, 0, a); });
    run("v3_tr16", [&] { hipLaunchKernelGGL(v3<16>, dim3((dh + 15) / 16, B), dim3(256), 0, 0, a); });
    run("v2_lds_tr4", [&] { hipLaunchKernelGGL(v2<4>, dim3((dh + 3) / 4, B), dim3(256), 0, 0, a); });
    run("v2_lds_tr8", [&] { hipLaunchKernelGGL(v2<8>, dim3((dh + 7) / 8, B), dim3(256), 0, 0, a); });
    run("v2_lds_tr16", [&] { hipLaunchKernelGGL(v2<16>, dim3((dh + 15) / 16, B), dim3(256), 0, 0, a); });
    return 0;
}
