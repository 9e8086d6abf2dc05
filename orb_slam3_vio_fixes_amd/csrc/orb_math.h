// orb_math.h — bit-exact scalar semantics shared by host and device code.
//
// Everything here reproduces a platform detail the reference binary depends
// on.  Compiled with -ffp-contract=off; every fused
// multiply-add below is an explicit fma()/fmaf().
#pragma once
#include <stdint.h>
#include <math.h>
#include <string.h>

#if defined(__HIPCC__)
#define ORB_HD __host__ __device__ __forceinline__
#else
#define ORB_HD inline
#endif

namespace orbmi {

// cvRound(float): ties to even under the default rounding mode.
ORB_HD int cv_round(float v) { return (int)rintf(v); }

ORB_HD uint32_t f32_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

// ---------------------------------------------------------------------------
// glibc 2.35 sincosf, FMA variant (x86_64 multiarch __sincosf_fma, selected by
// the ifunc on every FMA/AVX2 host).  The reference calls sincosf@PLT from
// computeOrbDescriptor (ORBextractor.cc:111-112).  Restated from the
// disassembly of the system libm (table at .rodata: sign[4], hpi_inv*2^24,
// hpi, c0, c1, s1, c2, s2, c3, s3, c4) and checked exhaustively against it in
// tests/test_math_host.py for every float in [0, 2*pi].  Valid for |y| < 120
// (descriptor angles are in [0, 2*pi)); larger inputs return NaN.
// ---------------------------------------------------------------------------
struct SinCosTab { double sgn[4], hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4; };

ORB_HD void glibc_sincosf(float y, float* sinp, float* cosp) {
    const SinCosTab t0 = {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
                          0x1p+0, -0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, 0x1.55553e1068f19p-5,
                          0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13,
                          0x1.99343027bf8c3p-16};
    const SinCosTab t1 = {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
                          -0x1p+0, 0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, -0x1.55553e1068f19p-5,
                          0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13,
                          -0x1.99343027bf8c3p-16};
    // Branch-free restatement (the device schedules it among independent
    // work): for |y| < pi/4 the reduction below gives n = 0 and xr = y exactly,
    // i.e. glibc's first branch; the tiny and out-of-range cases are selects.
    const double x = (double)y;
    const uint32_t top = (f32_bits(y) >> 20) & 0x7ff;
    const double r = x * t0.hpi_inv;
    const int n = top < 0x42f ? ((int32_t)r + 0x800000) >> 24 : 0;
    const double xr = fma(-(double)n, t0.hpi, x);
    // t0.sgn[n & 3] = {1, -1, -1, 1}[n & 3], as a select: an indexed table
    // read becomes a device memory load (and a vmcnt wait) in the kernels
    const double sg = ((n + 1) & 2) ? -1.0 : 1.0;
    const SinCosTab& p = (n & 2) ? t1 : t0;
    const double xs = xr * sg, x2 = xr * xr;
    const double x3 = x2 * xs;
    const double x4 = x2 * x2;
    const double s1p = fma(x2, p.s3, p.s2);
    const double c2p = fma(x2, p.c4, p.c3);
    const double c1p = fma(x2, p.c1, p.c0);
    const double x5 = x2 * x3;
    const double x6 = x2 * x4;
    const double sv = fma(x3, p.s1, xs);
    const double cv = fma(x4, p.c2, c1p);
    const float so = (float)fma(s1p, x5, sv);
    const float co = (float)fma(c2p, x6, cv);
    float sn = (n & 1) ? co : so, cs = (n & 1) ? so : co;
    if (top < 0x398) { sn = y; cs = 1.0f; }                 // |y| < 2^-12
    if (top >= 0x42f) { sn = NAN; cs = NAN; }               // |y| >= 120 (not reached)
    *sinp = sn;
    *cosp = cs;
}

// cv::fastAtan2 (OpenCV 4.x atan_f32), degrees; no contraction (A.4).
ORB_HD float fast_atan2_deg(float y, float x) {
    const float k = (float)(180 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    const float ax = fabsf(x), ay = fabsf(y);
    // both octant cases as selects (same operations, no branch)
    const bool xbig = ax >= ay;
    const float c = (xbig ? ay : ax) / ((xbig ? ax : ay) + (float)2.220446049250313e-16);
    const float c2 = c * c;
    float a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    a = xbig ? a : 90.f - a;
    a = x < 0 ? 180.f - a : a;
    a = y < 0 ? 360.f - a : a;
    return a;
}

// Sampling offsets of one rBRIEF point (computeOrbDescriptor's GET_VALUE,
// ORBextractor.cc:115-118): row = x sin + y cos, column = x cos - y sin, in
// the fused form GCC emits for the reference's -O3 -march=native build on an
// FMA host (A.6), or unfused.  Used by k_describe and by the exhaustive device
// check (orbx_debug_math, tests/test_gpu_math.py).
ORB_HD void brief_offset(float x, float y, float sb, float ca, bool fused, int& r, int& c) {
    if (fused) {
        r = cv_round(__builtin_fmaf(x, sb, y * ca));
        c = cv_round(__builtin_fmaf(x, ca, -(y * sb)));
    } else {
        r = cv_round(x * sb + y * ca);
        c = cv_round(x * ca - y * sb);
    }
}

// The angle conversion of computeOrbDescriptor (ORBextractor.cc:110).
ORB_HD float deg_to_rad(float deg) { return deg * (float)(3.14159265358979323846 / 180.f); }

// Hashes of the exhaustive math check (orbx_debug_math on the device, the
// oracle's orbo_debug_math with the system libm on the host).  Element i of
// [begin, end) goes to chunk (i - begin) >> chunk_log2; a chunk's hash is
// sum_i e_i * (2 i + 1) mod 2^64 over its elements.
ORB_HD uint64_t math_mix(uint32_t e, uint64_t i) { return (uint64_t)e * (2 * i + 1); }
ORB_HD uint32_t lowbias32(uint32_t v) {
    v ^= v >> 16; v *= 0x7feb352du; v ^= v >> 15; v *= 0x846ca68bu; v ^= v >> 16;
    return v;
}
// what 2 (fastAtan2): index -> (y, x) integer moments: every pair of
// [-2048, 2048]^2 first, then pseudo-random pairs over +-1.5e6 (|m10|, |m01|
// of a radius-15 disc of bytes stay below 1.2e6)
constexpr uint64_t kAtanGrid = 4097ull * 4097ull;
ORB_HD void atan_pair(uint64_t i, float& y, float& x) {
    if (i < kAtanGrid) {
        y = (float)((int)(i / 4097) - 2048);
        x = (float)((int)(i % 4097) - 2048);
    } else {
        y = (float)((int)(lowbias32((uint32_t)(2 * i)) % 3000001u) - 1500000);
        x = (float)((int)(lowbias32((uint32_t)(2 * i + 1)) % 3000001u) - 1500000);
    }
}
// what 1: one degree angle's 512 sampling offsets folded into one word
ORB_HD uint32_t offsets_word(uint32_t acc, int k, int r, int c) {
    return acc + ((uint32_t)(r & 0xff) | ((uint32_t)(c & 0xff) << 8)) * ((uint32_t)k * 0x9E3779B1u | 1u);
}

// ---------------------------------------------------------------------------
// libstdc++ std::sort (introsort, _S_threshold = 16, median-of-3 to first,
// unguarded partition, heap-sort fallback at depth 2*lg(n), final insertion
// sort), restated for a POD array so the device reproduces the exact
// permutation std::sort gives for DistributeOctTree's unstable sort of
// (count, node) pairs under compareNodes (ORBextractor.cc:538-553, :700).
// Checked against std::sort with heavy ties in tests/test_math_host.py.
// ---------------------------------------------------------------------------
struct SortRec { int cnt; int x0; int pos; };

ORB_HD bool node_less(const SortRec& a, const SortRec& b) {
    if (a.cnt < b.cnt) return true;
    if (a.cnt > b.cnt) return false;
    return a.x0 < b.x0;
}
ORB_HD void rec_swap(SortRec* a, SortRec* b) { SortRec t = *a; *a = *b; *b = t; }
ORB_HD int ilg(int n) { int l = 0; while (n >>= 1) ++l; return l; }

ORB_HD void push_heap_(SortRec* f, int hole, int top, SortRec v) {
    int parent = (hole - 1) / 2;
    while (hole > top && node_less(f[parent], v)) {
        f[hole] = f[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    f[hole] = v;
}
ORB_HD void adjust_heap_(SortRec* f, int hole, int len, SortRec v) {
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (node_less(f[child], f[child - 1])) child--;
        f[hole] = f[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        f[hole] = f[child - 1];
        hole = child - 1;
    }
    push_heap_(f, hole, top, v);
}
ORB_HD void heap_sort_(SortRec* f, int len) {
    if (len >= 2) {                                   // __make_heap
        for (int parent = (len - 2) / 2;; --parent) {
            adjust_heap_(f, parent, len, f[parent]);
            if (parent == 0) break;
        }
    }
    for (int last = len; last > 1;) {                 // __sort_heap
        --last;
        SortRec v = f[last];
        f[last] = f[0];
        adjust_heap_(f, 0, last, v);
    }
}
ORB_HD void median_to_first_(SortRec* r, SortRec* a, SortRec* b, SortRec* c) {
    if (node_less(*a, *b)) {
        if (node_less(*b, *c)) rec_swap(r, b);
        else if (node_less(*a, *c)) rec_swap(r, c);
        else rec_swap(r, a);
    } else if (node_less(*a, *c)) rec_swap(r, a);
    else if (node_less(*b, *c)) rec_swap(r, c);
    else rec_swap(r, b);
}
ORB_HD SortRec* unguarded_partition_(SortRec* first, SortRec* last, SortRec* pivot) {
    while (true) {
        while (node_less(*first, *pivot)) ++first;
        --last;
        while (node_less(*pivot, *last)) --last;
        if (!(first < last)) return first;
        rec_swap(first, last);
        ++first;
    }
}
ORB_HD void unguarded_linear_insert_(SortRec* last) {
    SortRec v = *last;
    SortRec* next = last - 1;
    while (node_less(v, *next)) { *last = *next; last = next; --next; }
    *last = v;
}
ORB_HD void insertion_sort_(SortRec* first, SortRec* last) {
    if (first == last) return;
    for (SortRec* i = first + 1; i != last; ++i) {
        if (node_less(*i, *first)) {
            SortRec v = *i;
            for (SortRec* p = i; p != first; --p) *p = *(p - 1);
            *first = v;
        } else {
            unguarded_linear_insert_(i);
        }
    }
}
// Iterative form of __introsort_loop.  The recursion (right part, then loop
// on the left part) only ever touches disjoint ranges, so any processing order
// of the pending ranges yields the same permutation; each range keeps the
// depth budget the recursion would give it.  `stk` holds >= 2*lg(n)+4 frames
// (the device passes an LDS buffer so nothing spills to scratch).
struct SortFrame { int f, l, depth; };

ORB_HD void std_sort(SortRec* first, int n, SortFrame* stk) {
    if (n <= 1) return;
    int sp = 0;
    stk[sp++] = {0, n, ilg(n) * 2};
    while (sp) {
        const SortFrame fr = stk[--sp];
        SortRec* f = first + fr.f;
        SortRec* l = first + fr.l;
        int depth = fr.depth;
        if (l - f <= 16) continue;
        if (depth == 0) { heap_sort_(f, (int)(l - f)); continue; }
        --depth;
        SortRec* mid = f + (l - f) / 2;
        median_to_first_(f, f + 1, mid, l - 1);
        SortRec* cut = unguarded_partition_(f + 1, l, f);
        stk[sp++] = {fr.f, (int)(cut - first), depth};
        stk[sp++] = {(int)(cut - first), fr.l, depth};
    }
    // __final_insertion_sort
    if (n > 16) {
        insertion_sort_(first, first + 16);
        for (SortRec* i = first + 16; i != first + n; ++i) unguarded_linear_insert_(i);
    } else {
        insertion_sort_(first, first + n);
    }
}


// ---------------------------------------------------------------------------
// The same permutation from data-parallel steps (k_quadtree).  One step of
// __introsort_loop on [f, l): median of three to first, then
// __unguarded_partition restated by ranks.  With L = ascending positions in
// [f+1, l) holding x >= pivot (!(x < pivot)) and R = descending positions in
// [f, l) holding x <= pivot, the scanners' k-th stops are L[k] and R[k] as
// long as L[k] < R[k] (each scanner only passes unexamined originals), the
// first k* with L[k*] >= R[k*] ends the loop at min(L[k*], R[k*-1]) (R[-1] = l:
// the left scanner runs into the value the last swap left at R[k*-1]), and the
// swaps are the pairs (L[k], R[k]), k < k*, all disjoint.  Every leaf range
// (<= 16 elements) ends up holding exactly its own elements, so the final
// insertion pass is a stable insertion sort per leaf (k_quadtree places each
// leaf's records at their stable ranks, 16 lanes a leaf: the same permutation).
// partition_ranks is the sequential statement (host check); the kernel
// computes L, R and k* with ballots.
// ---------------------------------------------------------------------------
ORB_HD int partition_ranks(SortRec* a, int f, int l, int* Lp, int* Rp) {
    median_to_first_(a + f, a + f + 1, a + f + (l - f) / 2, a + l - 1);
    const SortRec pv = a[f];
    int cl = 0, cr = 0;
    for (int p = f + 1; p < l; ++p) {
        if (!node_less(a[p], pv)) Lp[f + cl++] = p;
        if (!node_less(pv, a[p])) Rp[f + cr++] = p;          // ascending; R[k] = Rp[f + cr - 1 - k]
    }
    auto R = [&](int k) { return k < cr ? Rp[f + cr - 1 - k] : f; };
    int ks = 0;
    while (ks < cl && ks <= cr && Lp[f + ks] < R(ks)) ++ks;
    const int lk = ks < cl ? Lp[f + ks] : 0x7fffffff;
    const int rk = ks == 0 ? l : R(ks - 1);
    const int cut = lk < rk ? lk : rk;
    for (int k = 0; k < ks; ++k) rec_swap(a + Lp[f + k], a + R(k));
    return cut;
}

// Sequential statement of k_quadtree's level-synchronous driver: returns
// false where the reference would heap-sort a range (depth limit reached),
// in which case the caller falls back to std_sort on the original array.
ORB_HD bool std_sort_levels(SortRec* a, int n, int* Lp, int* Rp, SortFrame* qa, SortFrame* qb, SortFrame* leaves) {
    if (n <= 1) return true;
    int na = 0, nleaf = 0;
    if (n > 16) qa[na++] = {0, n, ilg(n) * 2};
    else leaves[nleaf++] = {0, n, 0};
    while (na) {
        int nb = 0;
        for (int r = 0; r < na; ++r) {
            const SortFrame fr = qa[r];
            if (fr.depth == 0) return false;
            const int cut = partition_ranks(a, fr.f, fr.l, Lp, Rp);
            const SortFrame kids[2] = {{fr.f, cut, fr.depth - 1}, {cut, fr.l, fr.depth - 1}};
            for (const SortFrame& k : kids) {
                if (k.l - k.f > 16) qb[nb++] = k;
                else leaves[nleaf++] = k;
            }
        }
        for (int r = 0; r < nb; ++r) qa[r] = qb[r];
        na = nb;
    }
    for (int i = 0; i < nleaf; ++i) insertion_sort_(a + leaves[i].f, a + leaves[i].l);
    return true;
}

}  // namespace orbmi
