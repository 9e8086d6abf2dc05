// extractor.hip — MI355X-native ORBextractor (gfx950).
//
// Replaces ORB_SLAM3::ORBextractor (reference include/ORBextractor.h:43-109,
// src/ORBextractor.cc:409-1195) behind the C ABI of include/orb_mi355x.h.
//
// Per batch of same-size frames the path is five launches, all batched over
// frames (one grid dimension indexes the frame):
//   k_pyr_stream   ComputePyramid: one workgroup per frame slides down it once
//                  with LDS row rings (k_pyramid row bands for small batches)
//   k_fast_cells   one wave per 2 FAST cells: LDS-staged ROI, compass
//                  pre-test, FAST-9 scores, cell-local 3x3 NMS at iniThFAST /
//                  minThFAST, ballot compaction
//   k_quadtree     one workgroup per (frame, level): DistributeOctTree as
//                  data-parallel passes over the node list + exact std::sort
//   k_describe     one wave per run of keypoint slots: raw patch in registers,
//                  IC_Angle moments, the 7x7 fixed-point blur of the 37x37
//                  patch only (horizontal pass on v_mfma_i32_16x16x64_i8),
//                  glibc-exact sincosf, 256 rBRIEF tests
//   k_assemble     per frame: scaling, lapping partition (monoIndex), output
// Everything is integer/bitwise and bit-exact against the reference.
#include "../../include/orb_mi355x.h"
#include "common.h"
#include "orb_math.h"
#include "host_gather.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <type_traits>
#include <thread>
#include <vector>

namespace orbmi {

constexpr int kHalfPatch = 15;
constexpr int kEdge = 19;
constexpr int kMinSubFrames = 16;   // smallest frame range worth its own stream

__constant__ __attribute__((aligned(16))) int8_t c_pattern[1024];
static const int8_t h_pattern[1024] = {
#include "brief_pattern.inc"
};

}  // namespace orbmi

#include "plan.h"

namespace orbmi {

static int cv_round_d(double v) { return (int)std::nearbyint(v); }
static int cv_floor_f(float v) { int i = (int)v; return i - (i > v); }
static int cv_ceil_f(float v) { int i = (int)v; return i + (i < v); }
static short sat_short(float v) {
    const int i = (int)std::nearbyintf(v);
    return (short)std::min(32767, std::max(-32768, i));
}

// ORBextractor::ORBextractor tables (ORBextractor.cc:414-468).
static void init_tables(orbx_handle* h) {
    const int L = h->prm.nlevels;
    const double sf = (double)h->prm.scale_factor;
    h->scale.assign(L, 1.f); h->sigma2.assign(L, 1.f);
    h->inv_scale.assign(L, 1.f); h->inv_sigma2.assign(L, 1.f);
    for (int i = 1; i < L; ++i) {
        h->scale[i] = (float)(h->scale[i - 1] * sf);
        h->sigma2[i] = h->scale[i] * h->scale[i];
    }
    for (int i = 0; i < L; ++i) { h->inv_scale[i] = 1.f / h->scale[i]; h->inv_sigma2[i] = 1.f / h->sigma2[i]; }
    h->nfeat.assign(L, 0);
    const float factor = (float)(1.0f / sf);
    float per = h->prm.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)L));
    int sum = 0;
    for (int l = 0; l < L - 1; ++l) {
        h->nfeat[l] = cv_round(per);
        sum += h->nfeat[l];
        per *= factor;
    }
    h->nfeat[L - 1] = std::max(h->prm.nfeatures - sum, 0);
    h->umax.assign(kHalfPatch + 1, 0);
    const int vmax = cv_floor_f(kHalfPatch * std::sqrt(2.f) / 2 + 1);
    const int vmin = cv_ceil_f(kHalfPatch * std::sqrt(2.f) / 2);
    const double hp2 = kHalfPatch * kHalfPatch;
    for (int v = 0; v <= vmax; ++v) h->umax[v] = cv_round_d(std::sqrt(hp2 - v * v));
    for (int v = kHalfPatch, v0 = 0; v >= vmin; --v) {
        while (h->umax[v0] == h->umax[v0 + 1]) ++v0;
        h->umax[v] = v0;
        ++v0;
    }
}

static int round_up(int x, int m) { return (x + m - 1) / m * m; }

// ---------------------------------------------------------------------------
// k_pyramid plan: column/row tap tables in the form the kernel reads, and the
// launch groups with their band tables.
// ---------------------------------------------------------------------------
constexpr int kLdsMax = 160 * 1024;          // LDS of one CU: a workgroup's ceiling
constexpr int kPyrLdsBudget = 64 * 1024;   // per workgroup: 2 workgroups of 256 threads per CU

static int pyr_lds_pitch(int w) { return round_up(w + 4, 16); }

// Bands of one group (la, lb) with R rows of level lb per band; returns the
// LDS bytes (A + B) and fills `band` ([nb][lb-la+1] int4 {n0, n1, p0, p1}).
static int pyr_bands(const Plan& P, const std::vector<int2>& yt, int la, int lb, int R, std::vector<int4>& band,
                     int& lds_a, int& lds_b, int& lds_x, int& lds_y) {
    const int nl = lb - la + 1, hb = P.lv[lb].h;
    const int nb = (hb + R - 1) / R;
    band.assign((size_t)nb * nl, make_int4(0, 0, 0, 0));
    auto B = [&](int b, int l) -> int4& { return band[(size_t)b * nl + (l - la)]; };
    for (int b = 0; b < nb; ++b) B(b, lb) = make_int4(b * R, std::min(hb, (b + 1) * R), 0, 0);
    for (int l = lb; l > la; --l) {
        const int h = P.lv[l].h;
        // every row of a written level is computed by some band: close the
        // gaps between the bands' ranges and reach both edges
        B(0, l).x = 0;
        B(nb - 1, l).y = h;
        for (int b = 0; b + 1 < nb; ++b) B(b, l).y = std::max(B(b, l).y, B(b + 1, l).x);
        // rows of level l-1 those rows read (clamped row taps)
        for (int b = 0; b < nb; ++b) {
            const int2 t0 = yt[P.lv[l].ytab + B(b, l).x], t1 = yt[P.lv[l].ytab + B(b, l).y - 1];
            B(b, l - 1).x = t0.x & 0xffff;
            B(b, l - 1).y = (t1.x >> 16) + 1;
        }
        // owned rows: what the previous band did not compute
        for (int b = 0; b < nb; ++b) {
            B(b, l).z = b == 0 ? 0 : std::max(B(b, l).x, B(b - 1, l).y);
            B(b, l).w = B(b, l).y;
        }
    }
    lds_x = lds_y = 0;
    for (int l = la + 1; l <= lb; ++l) {
        int rows = 0;
        for (int b = 0; b < nb; ++b) rows = std::max(rows, B(b, l).y - B(b, l).x);
        lds_x = std::max(lds_x, round_up(P.lv[l].w, 4) * 8);
        lds_y = std::max(lds_y, rows * 8);
    }
    lds_a = lds_b = 0;
    for (int l = la; l < lb; ++l) {
        int rows = 0;
        for (int b = 0; b < nb; ++b) rows = std::max(rows, B(b, l).y - B(b, l).x);
        int& dst = ((l - la) & 1) ? lds_b : lds_a;
        dst = std::max(dst, rows * pyr_lds_pitch(P.lv[l].w));
    }
    return lds_a + lds_b + lds_x + lds_y;
}

static int pyr_group_lds(const PyrGroup& g) { return g.lds_a + g.lds_b + g.lds_x + g.lds_y; }

// Tap tables and launch groups of k_pyramid.  Groups: greedily the longest
// run of levels (at most 4) whose bands of >= 8 top-level rows fit the LDS
// budget.
static void build_pyramid(Plan& P, const std::vector<int2>& tab, std::vector<int4>& bands, std::vector<int>& xs,
                          std::vector<uint32_t>& xw, std::vector<int2>& yt) {
    const int L = P.L;
    for (int l = 1; l < L; ++l) {
        LevelDev& d = P.lv[l];
        const LevelDev& s = P.lv[l - 1];
        d.xtab = (int)xs.size();
        for (int dx = 0; dx < round_up(d.w, 4); ++dx) {
            const int2 e = tab[P.tab_off[l] + std::min(dx, d.w - 1)];
            xs.push_back(e.x);
            xw.push_back((uint32_t)e.y);
        }
        d.ytab = (int)yt.size();
        for (int dy = 0; dy < d.h; ++dy) {
            const int2 e = tab[P.tab_off[l] + d.w + dy];
            const int r0 = std::min(std::max(e.x, 0), s.h - 1), r1 = std::min(std::max(e.x + 1, 0), s.h - 1);
            yt.push_back(make_int2(r0 | (r1 << 16), e.y));
        }
    }
    P.pgroups.clear();
    std::vector<int4> bt;
    int la = 0;
    while (la < L - 1) {
        PyrGroup g{};
        bool ok = false;
        for (int span = 4; span >= 1 && !ok; --span) {
            const int lb = std::min(L - 1, la + span);
            for (int R : {32, 24, 16, 12, 8, 6, 4, 2, 1}) {
                if (R < 8 && span > 1) break;
                int a, b, x, y;
                if (pyr_bands(P, yt, la, lb, R, bt, a, b, x, y) <= kPyrLdsBudget || (span == 1 && R == 1)) {
                    g.la = la; g.lb = lb; g.R = R;
                    ok = true;
                    break;
                }
            }
        }
        pyr_bands(P, yt, g.la, g.lb, g.R, bt, g.lds_a, g.lds_b, g.lds_x, g.lds_y);
        g.nb = (int)(bt.size() / (size_t)(g.lb - g.la + 1));
        g.band_off = (long long)bands.size();
        bands.insert(bands.end(), bt.begin(), bt.end());
        P.pgroups.push_back(g);
        la = g.lb;
    }
}

constexpr int kPyrStreamMinFrames = 32;   // below this a frame per CU leaves the chip idle: row bands
constexpr int kPsRun = 4;                 // k_pyr_stream: output rows per run (one lane, one column group)
// The FAST pre-test at iniThFAST fused into k_pyr_stream (candidate bitmap ->
// k_fast_cells<..., BM = true>) is exact but off by default: same-box A/B
//  put pyramid + FAST at 0.507 ms with it against 0.475 ms
// without -- the pre-test's VALU work moves ~1:1 into the pyramid, which
// issues it at lower efficiency (one 1024-thread workgroup per CU) than
// k_fast_cells does.  orb_debug_set_option(ORB_OPT_PYR_PRETEST, 1) selects it
// when a plan is built (tests, A/B).
#ifndef ORB_PYR_K0
#define ORB_PYR_K0 0
#endif
#ifndef ORB_ASM_THREADS
#define ORB_ASM_THREADS 256   // k_assemble: threads per frame's workgroup
#endif

// k_pyr_stream layout for level-0 chunks of K0 rows: runs the step schedule
// (level l computes at step s every row whose two source rows of level l-1
// were visible at the start of step s, i.e. written at a step < s; chunk c of
// level 0 is written at step c; with the fused FAST pre-test, level m's
// pre-test at step s takes every window row y whose row y + 3 was visible)
// and sizes each level's ring to the rows that must coexist: those written at
// a step and every row still to be read at that step or later.  Fills PS
// (except the table offsets) and `steps` (PS.E entries per step: [0] the
// step's wave-items, [l] level l's resize, [L + m] level m's pre-test);
// returns the LDS bytes of the rings.
static long long pyr_stream_schedule(const Plan& P, const std::vector<int2>& rows_tab, int K0, int R, bool pretest,
                                     PyrStream& PS, std::vector<int4>& steps) {
    const int L = P.L, h0 = P.lv[0].h;
    PS.K0 = K0;
    PS.nchunks = (h0 + K0 - 1) / K0;
    PS.pretest = pretest;
    PS.E = pretest ? 2 * L : L;
    std::vector<int> next(L, 0), vis(L, 0), ptn(L, 0);
    for (int m = 0; m < L; ++m) ptn[m] = PS.pt_y0[m];
    struct Span { int rd_lo, wr_lo, wr_hi; };
    std::vector<std::vector<Span>> hist(L);
    steps.clear();
    int s = 0;
    for (;; ++s) {
        bool done = true;
        for (int l = 1; l < L; ++l) done &= next[l] >= P.lv[l].h;
        if (pretest)
            for (int m = 0; m < L; ++m) done &= ptn[m] >= PS.pt_y1[m];
        if (done) break;
        if (s > 4 * h0 + 64) return -1;                  // no progress (cannot happen for valid tables)
        vis[0] = std::min(s * K0, h0);
        std::vector<int4> row(PS.E, make_int4(0, 0, 0, 0));
        int wtotal = 0;
        std::vector<Span> sp(L, Span{INT32_MAX, 0, 0});
        // level 0: chunk s written at this step
        if (s < PS.nchunks) sp[0].wr_lo = s * K0, sp[0].wr_hi = std::min(h0, (s + 1) * K0);
        for (int l = 1; l < L; ++l) {
            const int hl = P.lv[l].h, ng = (P.lv[l].w + 3) / 4;
            const int lo = next[l];
            int hi = lo;
            while (hi < hl && (rows_tab[P.lv[l].ytab + hi].x >> 16) < vis[l - 1]) ++hi;
            if (hi > lo) sp[l - 1].rd_lo = std::min(sp[l - 1].rd_lo, rows_tab[P.lv[l].ytab + lo].x & 0xffff);
            sp[l].wr_lo = lo, sp[l].wr_hi = hi;
            const int runs = (hi - lo + R - 1) / R;           // runs of <= R rows per column group
            const int wi = (runs * ng + kWave - 1) / kWave;
            row[l] = make_int4(lo, hi - lo, wtotal, ng | (runs << 16));
            wtotal += wi;
            next[l] = hi;
        }
        if (pretest)
            for (int m = 0; m < L; ++m) {
                const int lo = ptn[m];
                int hi = lo;
                while (hi < PS.pt_y1[m] && hi + 3 < vis[m]) ++hi;
                if (hi > lo) sp[m].rd_lo = std::min(sp[m].rd_lo, lo - 3);
                const int wi = ((hi - lo) * PS.pt_ngx[m] + kWave - 1) / kWave;
                row[L + m] = make_int4(lo, hi - lo, wtotal, PS.pt_ngx[m]);
                wtotal += wi;
                ptn[m] = hi;
            }
        row[0] = make_int4(wtotal, 0, 0, 0);
        steps.insert(steps.end(), row.begin(), row.end());
        for (int l = 1; l < L; ++l) vis[l] = next[l];
        for (int m = 0; m < L; ++m) hist[m].push_back(sp[m]);
    }
    PS.nsteps = s;
    long long bytes = 0;
    const int nring = pretest ? L : L - 1;               // the last level's rows only feed the pre-test
    for (int m = 0; m < nring; ++m) {
        int need = 1, fut = INT32_MAX;
        for (int t = s - 1; t >= 0; --t) {                // minimum row read at step >= t
            fut = std::min(fut, hist[m][t].rd_lo);
            const Span& x = hist[m][t];
            if (x.wr_hi > x.wr_lo) need = std::max(need, x.wr_hi - std::min(fut, x.wr_lo));
        }
        PS.ring_rows[m] = std::min(need, P.lv[m].h);
        PS.ring_pitch[m] = round_up(P.lv[m].w + 12, 16);
        bytes += (long long)PS.ring_rows[m] * PS.ring_pitch[m];
    }
    return bytes;
}

// Column records of level l (>= 1) for k_pyr_stream: per group
// of 4 output columns the weights (16 a0 | 16 a1 << 16) of each output, the
// v_perm selectors that place (S[sx] << 8, S[sx+1] << 8) in a u16 pair from
// the 3 dwords at the group's first tap dword bd, and bd | window flags << 16
// (outputs 0-2 take their taps from dwords 0:1, output 3 from 0:1 or 1:2).
// Layout W[4 ng], S[4 ng], BF[ng].  False when a tap span or weight is outside
// what that selection handles (scale factors near 2).
static bool pyr_col_records(const Plan& P, const std::vector<int2>& tab, int l, std::vector<uint32_t>& rec) {
    const LevelDev& d = P.lv[l];
    const int ng = (d.w + 3) / 4, ws = P.lv[l - 1].w;
    rec.assign((size_t)9 * ng, 0u);
    for (int g = 0; g < ng; ++g) {
        const int sx0 = tab[P.tab_off[l] + std::min(4 * g, d.w - 1)].x;
        const int bd = sx0 >> 2;
        uint32_t flags = 0;
        for (int c = 0; c < 4; ++c) {
            const int2 e = tab[P.tab_off[l] + std::min(4 * g + c, d.w - 1)];
            const int a0 = (short)(e.y & 0xffff), a1 = e.y >> 16;
            const int o = e.x - 4 * bd;
            if (a0 < 0 || a0 > 2048 || a1 < 0 || a1 > 2048 || o < 0 || o > 10 || e.x + 1 > ws) return false;
            if (c < 3 && o > 6) return false;
            const int win = c == 3 && o >= 4, op = o - 4 * win;
            rec[4 * g + c] = (uint32_t)(16 * a0) | ((uint32_t)(16 * a1) << 16);
            rec[4 * ng + 4 * g + c] = 0x0cu | ((uint32_t)op << 8) | (0x0cu << 16) | ((uint32_t)(op + 1) << 24);
            flags |= (uint32_t)win << c;
        }
        rec[8 * ng + g] = (uint32_t)bd | (flags << 16);
    }
    return true;
}

// The k_pyr_stream plan: table image (column records, row records) and
// rings in one LDS image of at most 160 KiB, with the largest level-0 chunk
// (<= 32 rows) that fits -- with the fused FAST pre-test if any chunk size
// leaves room for its rings (7 rows of every level), else without; PS.ok stays
// false when the size is not supported (more than kPsMaxLevels levels,
// weights or tap spans outside what the kernel's byte selection handles, or no
// chunk size fits).  Table image (dwords, 16-byte aligned sections):
//   [nsteps]            per-step wave-item counters (zeros)
//   [L] uint4 level A   {column records dw, row records dw, HBM offset, pitch}
//   [L] uint4 level B   {ring dw | ring pitch dw << 16, ring rows | pre-test
//                        16-px group origin << 8 | bitmap pitch << 16,
//                        bitmap offset, 0}
//   [nsteps][E] uint4   step entries (pyr_stream_schedule)
//   per level l >= 1: column records W[4 ng] S[4 ng] BF[ng], row records
//                        uint2 {source ring dw r0 | r1 << 16, b0 | b1 << 16}
static void build_pyr_stream(Plan& P, const std::vector<int2>& tab, std::vector<uint32_t>& img,
                             std::vector<int4>& steps) {
    PyrStream PS;
    P.ps = PS;
    const int L = P.L;
    if (L < 2 || L > kPsMaxLevels) return;
    // per level l >= 1: the row table of k_pyramid form (clamped rows) for the schedule
    std::vector<int2> rows_tab;
    std::vector<LevelDev> lv = P.lv;
    for (int l = 1; l < L; ++l) {
        const LevelDev& s = P.lv[l - 1];
        lv[l].ytab = (int)rows_tab.size();
        for (int dy = 0; dy < P.lv[l].h; ++dy) {
            const int2 e = tab[P.tab_off[l] + P.lv[l].w + dy];
            const int r0 = std::min(std::max(e.x, 0), s.h - 1), r1 = std::min(std::max(e.x + 1, 0), s.h - 1);
            const int b0 = (short)(e.y & 0xffff), b1 = e.y >> 16;
            if (b0 < 0 || b0 > 2048 || b1 < 0 || b1 > 2048) return;
            rows_tab.push_back(make_int2(r0 | (r1 << 16), e.y));
        }
    }
    // the fused pre-test covers the union of the level's FAST windows, in
    // groups of 16 pixels (columns 16 g - 4 .. 16 g + 19 of a ring row must
    // exist: the windows lie >= 19 px inside the level); the bitmap path of
    // k_fast_cells reads windows of <= 64 columns
    bool pt_ok = P.bm_ok && debug_opt(ORB_OPT_PYR_PRETEST) == 1;
    for (int m = 0; m < L && pt_ok; ++m) {
        PS.pt_y0[m] = P.win_y0[m]; PS.pt_y1[m] = P.win_y1[m];
        PS.pt_gx0[m] = P.win_x0[m] >> 4;
        PS.pt_ngx[m] = ((P.win_x1[m] + 15) >> 4) - PS.pt_gx0[m];
        pt_ok = PS.pt_gx0[m] >= 1 && PS.pt_gx0[m] < 256 && 16 * (PS.pt_gx0[m] + PS.pt_ngx[m]) + 4 <= P.lv[m].w + 12 &&
                PS.pt_y0[m] >= 3 && PS.pt_y1[m] + 3 <= P.lv[m].h && PS.pt_y1[m] > PS.pt_y0[m];
    }
    Plan Q = P;                       // the schedule reads lv[l].ytab of the row table above
    Q.lv = lv;
    int K0 = 0;
    int rec_dw = 0;                   // column and row records
    for (int l = 1; l < L; ++l) {
        const int ng = (P.lv[l].w + 3) / 4;
        rec_dw += round_up(9 * ng, 4) + round_up(2 * P.lv[l].h, 4);
    }
    // ORB_PYR_K0 (build flag, A/B): force the level-0 chunk rows (0: the largest that fits)
    const int k0_env = ORB_PYR_K0, run_rows = kPsRun;
    const int nq16 = (P.lv[0].w + 15) / 16;
    int tab_dw = 0;
    for (int pass = pt_ok ? 0 : 1; pass < 2 && !K0; ++pass) {
        const bool pretest = pass == 0;
        for (int k : {32, 24, 16, 12, 8, 6, 4}) {
            if (k0_env > 0 && k != k0_env) continue;
            if (k * nq16 > 2 * 1024) continue;                 // two 16-byte chunk loads per thread at most
            std::vector<int4> st;
            PyrStream T = PS;
            const long long rb = pyr_stream_schedule(Q, rows_tab, k, run_rows, pretest, T, st);
            const int td = round_up(T.nsteps, 4) + 8 * L + 4 * T.nsteps * T.E + rec_dw;
            if (rb < 0 || 4LL * td + rb > 160 * 1024) continue;
            K0 = k;
            tab_dw = td;
            PS = T;
            steps = st;
            break;
        }
    }
    if (K0 == 0) return;
    // LDS image: counters, level tables, step table, records, then the rings
    img.assign(tab_dw, 0u);
    PS.cnt_dw = 0;
    PS.lev_u4 = round_up(PS.nsteps, 4) / 4;
    PS.steps_u4 = PS.lev_u4 + 2 * L;
    std::memcpy(&img[4 * PS.steps_u4], steps.data(), steps.size() * sizeof(int4));
    int dw = 4 * (PS.steps_u4 + PS.nsteps * PS.E);
    for (int l = 1; l < L; ++l) {
        const int ng = (P.lv[l].w + 3) / 4;
        PS.ng[l] = ng;
        PS.rec_dw[l] = dw;
        dw += round_up(9 * ng, 4);
        PS.yt_dw[l] = dw;
        dw += round_up(2 * P.lv[l].h, 4);
    }
    int rdw = tab_dw;
    const int nring = PS.pretest ? L : L - 1;
    for (int m = 0; m < nring; ++m) {
        PS.ring_dw[m] = rdw;
        rdw += PS.ring_rows[m] * PS.ring_pitch[m] / 4;
    }
    if (rdw >= 65536) return;                              // row records hold 16-bit dword offsets
    for (int m = 0; m < nring; ++m)
        if (PS.ring_rows[m] >= 256 || PS.ring_pitch[m] / 4 >= 65536) return;   // 8-bit ring rows in level table B
    // ORB_OPT_PYR_CNT_END (test hook, orb_debug_set_option): the per-step
    // counters after the rings, at the top of the allocation, outside the copied
    // table image (the kernel zeroes them there); the default keeps them at dword
    // 0 of the image
    if (debug_opt(ORB_OPT_PYR_CNT_END)) {
        PS.cnt_dw = rdw;
        rdw += round_up(PS.nsteps, 4);
    }
    if (4LL * rdw > 160 * 1024) return;
    for (int l = 0; l < L; ++l) {
        const LevelDev& d = P.lv[l];
        uint32_t* A = &img[4 * (PS.lev_u4 + l)];
        uint32_t* Bv = &img[4 * (PS.lev_u4 + L + l)];
        if (l >= 1) {
            A[0] = (uint32_t)PS.rec_dw[l];
            A[1] = (uint32_t)PS.yt_dw[l];
            A[2] = (uint32_t)d.off;
            A[3] = (uint32_t)d.pitch;
        }
        if (l < nring) {
            Bv[0] = (uint32_t)PS.ring_dw[l] | ((uint32_t)(PS.ring_pitch[l] / 4) << 16);
            Bv[1] = (uint32_t)PS.ring_rows[l] | ((uint32_t)PS.pt_gx0[l] << 8) | ((uint32_t)d.bm_pitch << 16);
            Bv[2] = (uint32_t)d.bm_off;
        }
    }
    for (int l = 1; l < L; ++l) {
        const LevelDev& d = P.lv[l];
        const int ng = PS.ng[l];
        std::vector<uint32_t> rec;
        if (!pyr_col_records(P, tab, l, rec)) return;
        for (int g = 0; g < ng; ++g)
            if ((int)(rec[8 * ng + g] & 0xffff) + 2 >= PS.ring_pitch[l - 1] / 4) return;
        std::copy(rec.begin(), rec.end(), img.begin() + PS.rec_dw[l]);
        for (int dy = 0; dy < d.h; ++dy) {
            const int2 e = rows_tab[lv[l].ytab + dy];
            const int r0 = e.x & 0xffff, r1 = e.x >> 16, m = l - 1;
            const uint32_t o0 = (uint32_t)(PS.ring_dw[m] + (r0 % PS.ring_rows[m]) * PS.ring_pitch[m] / 4);
            const uint32_t o1 = (uint32_t)(PS.ring_dw[m] + (r1 % PS.ring_rows[m]) * PS.ring_pitch[m] / 4);
            uint32_t* r = &img[PS.yt_dw[l] + 2 * dy];
            r[0] = o0 | (o1 << 16);
            r[1] = (uint32_t)e.y;
        }
    }
    PS.tab_u4 = tab_dw / 4;
    PS.lds_bytes = 4 * rdw;
    PS.ok = true;
    P.ps = PS;
}

// Builds the size-dependent plan into P; returns ORB_OK or an error.  The
// caller (build_plan) releases P on any error, so a failed size never leaves a
// plan that a later call with the same size would take for a built one.
static void qt_lds_split(const Plan& P, size_t& lds, size_t& gstride);

static int build_plan_into(orbx_handle* hd, Plan& P, int w, int h, int maxB) {
    if (w > 4096 + 16 || h > 4096 + 16) return ORB_ERR_UNSUPPORTED;   // 12-bit key coordinates
    const int L = hd->prm.nlevels;
    P.L = L;
    P.lv.assign(L, LevelDev{});
    std::vector<int2> tab;
    P.xmax.assign(L, 0);
    P.tab_off.assign(L, 0);
    long long poff = 0;
    int cellsum = 0, slotsum = 0, outsum = 0;
    P.win_y0.assign(L, INT32_MAX); P.win_y1.assign(L, 0); P.win_x0.assign(L, INT32_MAX); P.win_x1.assign(L, 0);
    P.bm_ok = true;
    long long bmoff = 0;
    for (int l = 0; l < L; ++l) {
        LevelDev& d = P.lv[l];
        // ComputePyramid sizes (ORBextractor.cc:1174-1175)
        d.w = cv_round((float)w * hd->inv_scale[l]);
        d.h = cv_round((float)h * hd->inv_scale[l]);
        // A level of 33..66 px on a side has no FAST cells in the reference
        // (nCols or nRows = 0 at ORBextractor.cc:798-799: the cell loops do not
        // run) and gives no keypoints; one of <= 32 px makes DistributeOctTree
        // divide by maxY - minY <= 0 and size a vector from the result
        // (:559-565), which the reference does not survive: refused here.
        if (d.w - 2 * (kEdge - 3) < 1 || d.h - 2 * (kEdge - 3) < 1) return ORB_ERR_UNSUPPORTED;
        // 12 bytes of slack past the level's last pixel
        d.pitch = round_up(d.w + 12, 64);
        d.off = l == 0 ? 0 : poff;
        if (l > 0) poff += (long long)d.pitch * d.h;
        d.scale = hd->scale[l];
        d.patch = (int)(31 * hd->scale[l]);
        if (l > 0) {
            // cv::resize coefficient tables (imgproc resize.cpp)
            const LevelDev& s = P.lv[l - 1];
            const double sx_inv = (double)d.w / s.w, sy_inv = (double)d.h / s.h;
            const double scx = 1. / sx_inv, scy = 1. / sy_inv;
            // At an exact 2x reduction in both directions cv::resize switches
            // INTER_LINEAR to INTER_AREA (resize.cpp: is_area_fast, iscale 2),
            // whose fast path is (a + b + c + d + 2) >> 2 over each 2x2 block
            // (ResizeAreaFastVec).  The fixed-point linear taps below are then
            // all 1024 (fx = fy = 0.5, sx = 2 dx, sy = 2 dy, never clamped) and
            // give (1024 * ((1024 (a + b)) >> 4)) >> 16 = a + b per source row:
            // ((a + b) + (c + d) + 2) >> 2, the same value, so the linear
            // kernels serve that case unchanged (tests/test_gpu_configs.py
            // checks every level against the 2x2 block average).
            P.tab_off[l] = (long long)tab.size();
            int xmax = d.w;
            for (int dx = 0; dx < d.w; ++dx) {
                float fx = (float)((dx + 0.5) * scx - 0.5);
                int sx = cv_floor_f(fx);
                fx -= sx;
                if (sx < 0) { fx = 0.f; sx = 0; }
                if (sx + 1 >= s.w) {
                    xmax = std::min(xmax, dx);
                    if (sx >= s.w - 1) { fx = 0.f; sx = s.w - 1; }
                }
                const int a0 = sat_short((1.f - fx) * 2048.f), a1 = sat_short(fx * 2048.f);
                tab.push_back(make_int2(sx, (a0 & 0xffff) | (a1 << 16)));
            }
            for (int dy = 0; dy < d.h; ++dy) {
                float fy = (float)((dy + 0.5) * scy - 0.5);
                int sy = cv_floor_f(fy);
                fy -= sy;
                const int b0 = sat_short((1.f - fy) * 2048.f), b1 = sat_short(fy * 2048.f);
                tab.push_back(make_int2(sy, (b0 & 0xffff) | (b1 << 16)));
            }
            P.xmax[l] = xmax;
        }
        // ComputeKeyPointsOctTree cell grid (ORBextractor.cc:785-822)
        const int minBX = kEdge - 3, minBY = minBX;
        const int maxBX = d.w - kEdge + 3, maxBY = d.h - kEdge + 3;
        const float width = (float)(maxBX - minBX), height = (float)(maxBY - minBY);
        const int nCols = (int)(width / 35.f), nRows = (int)(height / 35.f);
        // (nCols or nRows = 0: no cells; the reference's cell sizes are then
        // a division by zero that nothing reads)
        const int wCell = nCols ? (int)std::ceil(width / nCols) : 0, hCell = nRows ? (int)std::ceil(height / nRows) : 0;
        const int cap = ((wCell + 1) / 2) * ((hCell + 1) / 2);
        d.cell_base = cellsum;
        d.slot_base = slotsum;
        int nc = 0;
        for (int i = 0; i < nRows; ++i) {
            const float iniY = (float)(minBY + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBY - 3) continue;
            if (maxY > maxBY) maxY = (float)maxBY;
            for (int j = 0; j < nCols; ++j) {
                const float iniX = (float)(minBX + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBX - 6) continue;
                if (maxX > maxBX) maxX = (float)maxBX;
                CellDev c;
                c.level = l;
                c.x0 = (int)iniX; c.y0 = (int)iniY;
                c.cols = (int)maxX - c.x0; c.rows = (int)maxY - c.y0;
                c.slot_off = slotsum;
                c.cap = cap;
                c.pitch = l == 0 ? 0 : P.lv[l].pitch;
                c.roi_off = l == 0 ? 0 : (int)(P.lv[l].off + (long long)c.y0 * P.lv[l].pitch + (c.x0 & ~3));
                // the FAST window (the ROI less its 3-px border): union per level
                P.win_y0[l] = std::min(P.win_y0[l], c.y0 + 3);
                P.win_y1[l] = std::max(P.win_y1[l], c.y0 + c.rows - 3);
                P.win_x0[l] = std::min(P.win_x0[l], c.x0 + 3);
                P.win_x1[l] = std::max(P.win_x1[l], c.x0 + c.cols - 3);
                P.bm_ok &= c.cols - 6 <= 64 && c.rows - 6 <= 64;
                slotsum += cap;
                P.cells.push_back(c);
                // + 16: the pre-test reads up to 2 dwords past the last row's window
                P.roi_max = std::max(P.roi_max, 4 * c.rows * (((c.x0 & 3) + c.cols + 3) >> 2) + 16);
                P.roi_rows_max = std::max(P.roi_rows_max, c.rows);
                P.roi_nd_max = std::max(P.roi_nd_max, ((c.x0 & 3) + c.cols + 3) >> 2);
                P.win_max = std::max(P.win_max, (std::max(0, c.cols - 6) + 2) * (std::max(0, c.rows - 6) + 2));
                P.win_pix_max = std::max(P.win_pix_max, std::max(0, c.cols - 6) * std::max(0, c.rows - 6));
                // k_fast_cells' candidates hold (row, column) in 7 bits each (< 70 px: wCell < 2 * 35)
                if (c.cols - 6 >= 128 || c.rows - 6 >= 128) return ORB_ERR_UNSUPPORTED;
                {   // k_fast_cells' pre-test items of this cell: window rows x aligned dword pairs
                    const int ww = std::max(0, c.cols - 6), X0 = (c.x0 & 3) + 3, j0 = X0 >> 2;
                    const int ndw = ww ? ((X0 + ww - 1) >> 2) - j0 + 1 : 0;
                    P.item_max = std::max(P.item_max, std::max(0, c.rows - 6) * ((ndw + 1) >> 1));
                }
                ++nc;
            }
        }
        d.ncells = nc;
        cellsum += nc;
        // pre-test bitmap rows: one bit per pixel, 16 bytes of slack (k_fast_cells
        // reads 4 dwords from the dword holding a window row's first bit)
        d.bm_pitch = round_up((d.w + 7) / 8 + 16, 16);
        d.bm_off = bmoff;
        bmoff += (long long)d.bm_pitch * d.h;
        if (P.item_max >= 65536) return ORB_ERR_UNSUPPORTED;   // 16-bit item indices in k_fast_cells' list
        d.slot_total = slotsum - d.slot_base;
        P.max_level_cells = std::max(P.max_level_cells, nc);
        // DistributeOctTree sizing (ORBextractor.cc:559-561)
        d.qW = maxBX - minBX;
        d.qH = maxBY - minBY;
        d.N = hd->nfeat[l];
        d.nIni = (int)std::round((float)(maxBX - minBX) / (maxBY - minBY));
        // nIni = 0 is harmless only without keys (the reference indexes
        // vpIniNodes[x / inf] = [0] of an empty vector otherwise, :583-584)
        if (d.nIni < 0 || (d.nIni == 0 && nc > 0)) return ORB_ERR_UNSUPPORTED;
        d.hX = d.nIni ? (float)(maxBX - minBX) / d.nIni : 0.f;
        d.out_base = outsum;
        d.out_cap = std::max(d.N + 3, 4 * d.nIni);
        outsum += d.out_cap;
        P.max_out_cap = std::max(P.max_out_cap, d.out_cap);
    }
    std::vector<int4> pband;
    std::vector<int> pxs;
    std::vector<uint32_t> pxw;
    std::vector<int2> pyt;
    build_pyramid(P, tab, pband, pxs, pxw, pyt);
    std::vector<uint32_t> psimg;
    std::vector<int4> pssteps;
    build_pyr_stream(P, tab, psimg, pssteps);
    for (const PyrGroup& g : P.pgroups)
        if (pyr_group_lds(g) > 160 * 1024) return ORB_ERR_UNSUPPORTED;   // a level row beyond ~80 KB
    P.pyr_bytes = poff;
    P.bm_bytes = round_up((int)std::min<long long>(bmoff, 1ll << 30), 256);
    P.ncells = cellsum;
    P.slot_total = slotsum;
    P.out_total = outsum;
    // k_assemble holds a flag per output slot of a frame in LDS (dynamic) next
    // to its static lvl_start[kMaxLevels + 1] and tmp[16]: up to ~40,000
    // features a frame (Tracking's largest extractor is 5 x nFeatures)
    if ((size_t)outsum * 4 + 64 + (size_t)(4 * kMaxLevels + 1 + ORB_ASM_THREADS / 64 + 1) * 4 > (size_t)kLdsMax) return ORB_ERR_UNSUPPORTED;
    P.in_pitch = (size_t)round_up(w, 64);

    const size_t B = (size_t)maxB;
    ORB_CHECK(hipMalloc(&P.d_pyr, std::max<size_t>(1, B * P.pyr_bytes)));
    if (P.ps.ok && P.ps.pretest) ORB_CHECK(hipMalloc(&P.d_bm, B * P.bm_bytes));
    ORB_CHECK(hipMalloc(&P.d_in, P.in_pitch * h));
    ORB_CHECK(hipMalloc(&P.d_tab, std::max<size_t>(1, tab.size()) * sizeof(int2)));
    ORB_CHECK(hipMalloc(&P.d_lv, L * sizeof(LevelDev)));
    ORB_CHECK(hipMalloc(&P.d_cells, P.cells.size() * sizeof(CellDev)));
    ORB_CHECK(hipMalloc(&P.d_cell_count, B * P.ncells * sizeof(int)));
    ORB_CHECK(hipMalloc(&P.d_cell_keys, B * P.slot_total * sizeof(uint32_t)));
    ORB_CHECK(hipMalloc(&P.d_key_scr, B * P.slot_total * sizeof(uint32_t)));
    ORB_CHECK(hipMalloc(&P.d_knode, B * P.slot_total * sizeof(int)));
    ORB_CHECK(hipMalloc(&P.d_kq, B * P.slot_total));
    ORB_CHECK(hipMalloc(&P.d_qt_key, B * P.out_total * sizeof(uint32_t)));
    {
        size_t qlds, qgs;
        qt_lds_split(P, qlds, qgs);
        if (qgs) ORB_CHECK(hipMalloc(&P.d_qt_gscr, B * L * qgs));
    }
    ORB_CHECK(hipMalloc(&P.d_qt_n, B * L * sizeof(int)));
    ORB_CHECK(hipMalloc(&P.d_qt_ovf, B * L * sizeof(int)));
    ORB_CHECK(hipMalloc(&P.d_angle, B * P.out_total * sizeof(float)));
    ORB_CHECK(hipMalloc(&P.d_sdesc, B * P.out_total * 32));
    P.host_cap = P.out_total;
    ORB_CHECK(hipMalloc(&P.d_kps, P.host_cap * sizeof(orb_keypoint)));
    ORB_CHECK(hipMalloc(&P.d_desc, (size_t)P.host_cap * 32));
    ORB_CHECK(hipMalloc(&P.d_n, sizeof(int32_t)));
    ORB_CHECK(hipMalloc(&P.d_mono, sizeof(int32_t)));
    if (!tab.empty()) ORB_CHECK(hipMemcpy(P.d_tab, tab.data(), tab.size() * sizeof(int2), hipMemcpyHostToDevice));
    ORB_CHECK(hipMalloc(&P.d_pband, std::max<size_t>(1, pband.size()) * sizeof(int4)));
    ORB_CHECK(hipMalloc(&P.d_pxs, std::max<size_t>(1, pxs.size()) * sizeof(int)));
    ORB_CHECK(hipMalloc(&P.d_pxw, std::max<size_t>(1, pxw.size()) * sizeof(uint32_t)));
    ORB_CHECK(hipMalloc(&P.d_pyt, std::max<size_t>(1, pyt.size()) * sizeof(int2)));
    if (!pband.empty())
        ORB_CHECK(hipMemcpy(P.d_pband, pband.data(), pband.size() * sizeof(int4), hipMemcpyHostToDevice));
    if (!pxs.empty()) {
        ORB_CHECK(hipMemcpy(P.d_pxs, pxs.data(), pxs.size() * sizeof(int), hipMemcpyHostToDevice));
        ORB_CHECK(hipMemcpy(P.d_pxw, pxw.data(), pxw.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        ORB_CHECK(hipMemcpy(P.d_pyt, pyt.data(), pyt.size() * sizeof(int2), hipMemcpyHostToDevice));
    }
    if (P.ps.ok) {
        ORB_CHECK(hipMalloc(&P.d_ps_tab, psimg.size() * sizeof(uint32_t)));
        ORB_CHECK(hipMemcpy(P.d_ps_tab, psimg.data(), psimg.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    ORB_CHECK(hipMemcpy(P.d_lv, P.lv.data(), L * sizeof(LevelDev), hipMemcpyHostToDevice));
    ORB_CHECK(hipMemcpy(P.d_cells, P.cells.data(), P.cells.size() * sizeof(CellDev), hipMemcpyHostToDevice));
    {
        std::vector<uint8_t> sl(P.out_total);
        for (int l = 0; l < L; ++l)
            for (int o = 0; o < P.lv[l].out_cap; ++o) sl[P.lv[l].out_base + o] = (uint8_t)l;
        ORB_CHECK(hipMalloc(&P.d_slot_level, std::max<size_t>(1, sl.size())));
        ORB_CHECK(hipMemcpy(P.d_slot_level, sl.data(), sl.size(), hipMemcpyHostToDevice));
    }
    // the size keys last: only a complete plan answers the cache check
    P.w = w; P.h = h; P.maxB = maxB;
    return ORB_OK;
}

static int build_plan(orbx_handle* hd, int w, int h, int maxB) {
    Plan& P = hd->plan;
    if (P.w == w && P.h == h && P.maxB >= maxB && P.L == hd->prm.nlevels) return ORB_OK;
    P.release();
    ++hd->plan_epoch;                                        // captured graphs point at the old buffers
    // the pyramids of earlier calls lived in the released buffers
    hd->have_last = false;
    hd->x_pyr_valid = false;
    hd->last_frames = nullptr;
    hd->last_B = 0;
    const int rc = build_plan_into(hd, P, w, h, maxB);
    if (rc != ORB_OK) P.release();
    return rc;
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ int round_up_d(int x, int m) { return (x + m - 1) / m * m; }

// ---------------------------------------------------------------------------
// k_pyramid: ComputePyramid (ORBextractor.cc:1170-1195) for levels la+1..lb
// of every frame in one launch, cv::resize INTER_LINEAR 8UC1.
//
// A workgroup owns a band of rows of every level of the group.  It stages the
// rows of level la its band needs in LDS with 16-byte coalesced loads, then
// builds each next level from the previous one in LDS (two ping-pong
// buffers), writing the rows it owns to HBM and keeping the rows the next
// level reads (its own plus a few halo rows the neighbouring band also
// computes) in LDS.  Each HBM row of a level is written once; level la is read
// once plus the halo.  One thread makes 4 consecutive outputs of a row: the
// frame-invariant column taps come from the plan tables (one 16-byte load
// each for the 4 source columns and the 4 weight pairs), the horizontal pass
// is one v_dot2_u32_u16 per row tap (pixel pair x weight pair), the vertical
// one OpenCV's (b * (h >> 4)) >> 16 as a v_mul_hi_u32 by b << 16.
//
// Workgroup -> (frame, band) is XCD-aware: the bands of one frame run on one
// XCD (workgroups are dealt round-robin over the 8 XCDs), so the halo rows
// two bands share are L2 hits.
// ---------------------------------------------------------------------------
struct PyrArgs {
    const uint8_t* src;         // level la of frame 0
    long long src_fstride;
    int src_pitch, load_mode;   // 16 / 4 / 1: widest aligned load of a row of level la
    uint8_t* pyr;               // levels >= 1 of frame 0
    long long pyr_fstride;
    const LevelDev* lv;
    const int4* band;           // [nb][lb-la+1] {n0, n1, p0, p1}
    const int* xs;
    const uint32_t* xw;
    const int2* yt;
    int la, lb, nb, nframes, lds_b;
    int lds_x, lds_y;           // offsets of the staged column / row tap tables
};

__global__ __launch_bounds__(256) void k_pyramid(PyrArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t pyr_lds[];
    const int wg = blockIdx.x;
    const int f = (wg / 8 / a.nb) * 8 + (wg & 7), b = (wg / 8) % a.nb;
    if (f >= a.nframes) return;
    const int tid = threadIdx.x, nl = a.lb - a.la + 1;
    typedef __attribute__((address_space(4))) const LevelDev* ConstLevels;
    const ConstLevels lv = (ConstLevels)a.lv;
    const int4* bd = a.band + (long long)b * nl;
    // 1. rows [n0, n1) of level la -> buffer A
    {
        const int4 nb0 = bd[0];
        const int w = lv[a.la].w, P = round_up_d(w + 4, 16);
        const uint8_t* src = a.src + f * a.src_fstride + (long long)nb0.x * a.src_pitch;
        const int rows = nb0.y - nb0.x;
        if (a.load_mode == 16) {
            const int nq = (w + 15) >> 4, n = rows * nq;
            const float inv = 1.0f / (float)nq;
            int i = tid;
            for (; i + 3 * 256 < n; i += 4 * 256) {   // four 16-byte loads in flight per thread
                uint4 v[4];
                int r[4], q[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int ii = i + k * 256;
                    r[k] = (int)(((float)ii + 0.5f) * inv);
                    q[k] = ii - r[k] * nq;
                    v[k] = *(const uint4*)(src + (long long)r[k] * a.src_pitch + 16 * q[k]);
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) *(uint4*)(pyr_lds + r[k] * P + 16 * q[k]) = v[k];
            }
            for (; i < n; i += 256) {
                const int r = (int)(((float)i + 0.5f) * inv), q = i - r * nq;
                *(uint4*)(pyr_lds + r * P + 16 * q) = *(const uint4*)(src + (long long)r * a.src_pitch + 16 * q);
            }
        } else if (a.load_mode == 4) {
            const int nq = (w + 3) >> 2, n = rows * nq;
            const float inv = 1.0f / (float)nq;
            for (int i = tid; i < n; i += 256) {
                const int r = (int)(((float)i + 0.5f) * inv), q = i - r * nq;
                *(uint32_t*)(pyr_lds + r * P + 4 * q) = *(const uint32_t*)(src + (long long)r * a.src_pitch + 4 * q);
            }
        } else {
            const int n = rows * w;
            const float inv = 1.0f / (float)w;
            for (int i = tid; i < n; i += 256) {
                const int r = (int)(((float)i + 0.5f) * inv), q = i - r * w;
                pyr_lds[r * P + q] = src[(long long)r * a.src_pitch + q];
            }
        }
    }
    __syncthreads();
    // 2. each next level from the previous one
    for (int l = a.la + 1; l <= a.lb; ++l) {
        const int k = l - a.la;
        const int4 sb = bd[k - 1], db = bd[k];
        const uint8_t* S = pyr_lds + ((k - 1) & 1 ? a.lds_b : 0);
        uint8_t* Dl = pyr_lds + (k & 1 ? a.lds_b : 0);
        const int sP = round_up_d(lv[l - 1].w + 4, 16);
        const int w = lv[l].w, dP = round_up_d(w + 4, 16), pitch = lv[l].pitch;
        const bool keep = l < a.lb;
        uint8_t* G = a.pyr + f * a.pyr_fstride + lv[l].off;
        const int ng = (w + 3) >> 2, nrows = db.y - db.x, n = nrows * ng;
        // this level's tap tables -> LDS (a dependent global load per item
        // would leave every item waiting on L2 latency)
        int* xs = (int*)(pyr_lds + a.lds_x);
        uint32_t* xw = (uint32_t*)(xs + 4 * ng);
        int2* yt = (int2*)(pyr_lds + a.lds_y);
        {
            const uint4* gx = (const uint4*)(a.xs + lv[l].xtab);
            const uint4* gw = (const uint4*)(a.xw + lv[l].xtab);
            const int2* gy = a.yt + lv[l].ytab + db.x;
            for (int i = tid; i < ng; i += 256) {
                ((uint4*)xs)[i] = gx[i];
                ((uint4*)xw)[i] = gw[i];
            }
            for (int i = tid; i < nrows; i += 256) yt[i] = gy[i];
        }
        __syncthreads();
        const float inv = 1.0f / (float)ng;
#pragma unroll 2
        for (int i = tid; i < n; i += 256) {
            const int r = (int)(((float)i + 0.5f) * inv), g = i - (int)__umul24(r, ng);
            const int row = db.x + r;
            const int2 ty = yt[r];
            const uint32_t B0 = (ty.y & 0xffff) << 16, B1 = ((uint32_t)ty.y >> 16) << 16;
            const uint8_t* S0 = S + __umul24((ty.x & 0xffff) - sb.x, sP);
            const uint8_t* S1 = S + __umul24((ty.x >> 16) - sb.x, sP);
            const int4 sx = *(const int4*)(xs + 4 * g);
            const uint4 wt = *(const uint4*)(xw + 4 * g);
            const int sxa[4] = {sx.x, sx.y, sx.z, sx.w};
            const uint32_t wta[4] = {wt.x, wt.y, wt.z, wt.w};
            uint32_t out = 0;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint32_t p0 = (uint32_t)S0[sxa[c]] | ((uint32_t)S0[sxa[c] + 1] << 16);
                const uint32_t p1 = (uint32_t)S1[sxa[c]] | ((uint32_t)S1[sxa[c] + 1] << 16);
                const uint32_t h0 = __builtin_amdgcn_udot2(as_u16x2(p0), as_u16x2(wta[c]), 0u, false);
                const uint32_t h1 = __builtin_amdgcn_udot2(as_u16x2(p1), as_u16x2(wta[c]), 0u, false);
                const uint32_t v = (__umulhi(B0, h0 >> 4) + __umulhi(B1, h1 >> 4) + 2) >> 2;
                out |= v << (8 * c);
            }
            if (keep) *(uint32_t*)(Dl + __umul24(r, dP) + 4 * g) = out;
            // a level is < 2^24 bytes (4112 x 4112 at most)
            if (row >= db.z && row < db.w) *(uint32_t*)(G + (__umul24(row, pitch) + 4 * g)) = out;
        }
        __syncthreads();
    }
}

// Compass pre-test, 4 pixels per lane: a 9-pixel arc of the 16-ring always
// covers two ring-adjacent compass pixels -- one of {U, D} and one of {L, R} --
// so a brighter corner at threshold t has min(max(U,D), max(L,R)) > v + t and
// a darker one max(min(U,D), min(L,R)) < v - t (ORB_FAST_COMPASS_AND; round 2
// tested the looser 2nd largest / 2nd smallest of the four).  Pixels failing both at min(iniTh, minTh) are corners at no
// threshold used; their score stays 0, which the NMS treats exactly like a
// non-corner (s_t(q) = 0).  Bytes are split into u16 pairs (pixels 0/2 and
// 1/3) and tested with packed u16 min/max; the flags are the signs of packed
// differences, gathered into one flag byte per pixel.  (A planar u16 ROI --
// even and odd columns de-interleaved at landing, no splitting here -- was
// measured slower: 0.575 vs 0.510 ms, twice the LDS reads per item.)

#ifndef ORB_FAST_LERP
#define ORB_FAST_LERP 1   // k_fast_cells' pre-test in bytes by v_lerp_u8 (0: packed u16 pairs)
#endif
#ifndef ORB_FAST_COMPASS_AND
#define ORB_FAST_COMPASS_AND 1   // pre-test: one vertical AND one horizontal compass pixel past the threshold
#endif
// Flags as signs: (C + t) - L2 and (S2 + t) - C as packed u16 differences;
// every value is < 2^10, so the i16 sign bit is exactly the bright / dark test.
__device__ __forceinline__ void compass_signs(uint32_t c, uint32_t u, uint32_t d, uint32_t l, uint32_t r,
                                              u16x2 tt, uint32_t& bneg, uint32_t& dneg) {
    const u16x2 C = as_u16x2(c), U = as_u16x2(u), D = as_u16x2(d), L = as_u16x2(l), R = as_u16x2(r);
    const u16x2 m1 = __builtin_elementwise_min(U, D), M1 = __builtin_elementwise_max(U, D);
    const u16x2 m2 = __builtin_elementwise_min(L, R), M2 = __builtin_elementwise_max(L, R);
    const u16x2 X = __builtin_elementwise_min(M1, M2), Y = __builtin_elementwise_max(m1, m2);
#if ORB_FAST_COMPASS_AND
    // every 9-arc holds two ring-adjacent compass pixels, one of {U, D} and
    // one of {L, R}: a bright corner has min(max(U,D), max(L,R)) > v + t, a
    // dark one max(min(U,D), min(L,R)) < v - t -- tighter than the 2nd
    // largest / 2nd smallest of the four (which also passes U, D alone) and
    // two packed ops cheaper; a failing direction still has strength - 1 < t
    bneg = as_u32((C + tt) - X);
    dneg = as_u32((Y + tt) - C);
#else
    const u16x2 L2 = __builtin_elementwise_max(X, Y), S2 = __builtin_elementwise_min(X, Y);
    bneg = as_u32((C + tt) - L2);
    dneg = as_u32((S2 + tt) - C);
#endif
}

// pairs (pixels 0, 2) and (1, 3) of a dword -> one flag byte per pixel (bit 7), pixel order
__device__ __forceinline__ uint32_t sign_bytes(uint32_t p02, uint32_t p13) {
    return __builtin_amdgcn_perm(p13, p02, 0x07030501u) & 0x80808080u;
}

// byte-flag mask of item pixels [s, e) (0 <= s, e <= 8): byte k of the (lo, hi) pair = pixel k
__device__ __forceinline__ uint64_t item_byte_mask(int s, int e) {
    const uint64_t hi = e >= 8 ? ~0ull : ((1ull << (8 * e)) - 1ull);
    const uint64_t lo = s >= 8 ? ~0ull : ((1ull << (8 * s)) - 1ull);
    return hi & ~lo & 0x8080808080808080ull;
}

__device__ __forceinline__ uint32_t lo_bytes(uint32_t x) { return x & 0x00ff00ffu; }
// u16 pair (x.b1, x.b3) in one v_perm (a shift and a mask otherwise)
__device__ __forceinline__ uint32_t hi_bytes(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0c030c01u); }

// The compass pre-test on four pixels at once, in bytes (ORB_FAST_LERP).
// v_lerp_u8 averages bytes with a 9-bit sum, so with the complement of the
// centre, h = lerp(X, ~C, 1) = 128 + floor((X - C) / 2) per byte, and a second
// lerp against a complemented constant puts "h >= T" in bit 7 of each byte.
// X > C + t  =>  h >= 128 + floor((t + 1) / 2)  (= tb), and
// X < C - t  =>  h <= 128 + floor((-t - 1) / 2) (= td1 - 1): necessary
// conditions (the halving admits X - C = t for odd t + 1 and -t for odd t), so
// a cleared flag still proves the direction's strength - 1 < t, as the u16
// form's.  ntb = ~tb, ntd = ~td1 per byte.  Flags: bit 7 of byte k = pixel k.
struct LerpTh { uint32_t ntb, ntd; };
__device__ __forceinline__ LerpTh lerp_thresholds(int t) {
    const uint32_t tb = min(128 + ((t + 1) >> 1), 255), td1 = 129 - ((t + 2) >> 1);
    return LerpTh{~(tb * 0x01010101u), ~(td1 * 0x01010101u)};
}
__device__ __forceinline__ void compass_lerp(uint32_t c, uint32_t u, uint32_t d, uint32_t l, uint32_t r,
                                             LerpTh th, uint32_t& bright, uint32_t& darkx) {
    const uint32_t nc = ~c, one = 0x01010101u;
    const uint32_t hu = __builtin_amdgcn_lerp(u, nc, one), hd = __builtin_amdgcn_lerp(d, nc, one);
    const uint32_t hl = __builtin_amdgcn_lerp(l, nc, one), hr = __builtin_amdgcn_lerp(r, nc, one);
    const uint32_t bu = __builtin_amdgcn_lerp(hu, th.ntb, one), bd = __builtin_amdgcn_lerp(hd, th.ntb, one);
    const uint32_t bl = __builtin_amdgcn_lerp(hl, th.ntb, one), br = __builtin_amdgcn_lerp(hr, th.ntb, one);
    const uint32_t gu = __builtin_amdgcn_lerp(hu, th.ntd, one), gd = __builtin_amdgcn_lerp(hd, th.ntd, one);
    const uint32_t gl = __builtin_amdgcn_lerp(hl, th.ntd, one), gr = __builtin_amdgcn_lerp(hr, th.ntd, one);
    bright = (bu | bd) & (bl | br);              // bit 7: one of U, D and one of L, R brighter
    darkx = (gu & gd) | (gl & gr);               // bit 7 CLEAR: one of U, D and one of L, R darker
}
// u16 pair of bytes (hi.bs1 | lo.bs0 selectors 0-3: lo, 4-7: hi) in one v_perm
template <uint32_t SEL>
__device__ __forceinline__ uint32_t pair_bytes(uint32_t hi, uint32_t lo) { return __builtin_amdgcn_perm(hi, lo, SEL); }
// ---------------------------------------------------------------------------
// k_pyr_stream: ComputePyramid (ORBextractor.cc:1170-1195) of one frame per
// 1024-thread workgroup, cv::resize INTER_LINEAR 8UC1, as a
// software pipeline that slides down the frame once.
//
// Step s: chunk s of level 0 (K0 rows, prefetched into registers with 16-byte
// loads during step s-1) lands in level 0's LDS ring, and every level l >= 1
// computes the rows whose two source rows of level l-1 were in its ring by
// the end of step s-1, writing each row to HBM and (levels < L-1) into its own
// ring.  All levels of a step are independent, so a step is one flat list of
// wave-items (64 column groups of 4 outputs; levels padded to whole waves)
// followed by ONE barrier.  Nothing is recomputed and level 0 is read from HBM
// exactly once; ring sizes come from the host's run of the same schedule.
//
// Per item: 3 dwords of each source row (the 4 outputs' taps lie within 12
// bytes of the first tap's dword), the (S[sx], S[sx+1]) pair of output c by
// one v_perm with a host-made selector (window D0:D1 or D1:D2 by a flag bit),
// h = a0*S[sx] + a1*S[sx+1] by v_dot2_u32_u16 with weights pre-scaled by 16 so
// that (16h) & ~0xff = (h >> 4) << 8, and OpenCV's (b * (h >> 4)) >> 16 as
// v_mul_hi_u32_u24(b << 8, (h >> 4) << 8).
// ---------------------------------------------------------------------------

struct PyrStreamArgs {
    const uint8_t* src;         // level 0 of frame 0
    long long src_fstride;
    int src_pitch, load_mode;   // 16 / 4 / 1
    uint8_t* pyr;               // levels >= 1 of frame 0
    long long pyr_fstride;
    const uint4* tab;           // LDS table image
    int tab_u4, lev_u4, steps_u4;   // table image size; level and step tables inside it (uint4 units)
    int L, E, nsteps, nchunks, K0, h0, w0, nframes;
    int ring0_dw, ring0_rows, ring0_pitch;
    int cnt_dw;                 // per-step wave-item counters (nsteps dwords)
    int pretest;                // the fused FAST pre-test at ini_th (E = 2L)
    int ini_th;
    uint8_t* bm;                // pre-test bitmaps of frame 0 (LevelDev::bm_off / bm_pitch layout)
    long long bm_fstride;
};

// Workgroup barrier that orders LDS only: __syncthreads()' workgroup fence
// also waits for every outstanding global load and store (vmcnt(0)), which
// would drain the next chunk's prefetch and the step's HBM writes each step.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ uint32_t mulhi_u24(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)(a & 0xffffffu) * (uint64_t)(b & 0xffffffu)) >> 32);
}

// y % n for 0 <= y < 2^16, 1 <= n < 256 by a float reciprocal: (y + 0.5) / n
// lies >= 1 / (2n) from every integer, far beyond the reciprocal's error
__device__ __forceinline__ int small_mod(int y, int n, float inv_n) {
    return y - (int)__umul24((uint32_t)(((float)y + 0.5f) * inv_n), (uint32_t)n);
}

// The compass pre-test (above) of 16 consecutive pixels of a ring row at
// threshold t: c[0..3] the pixels' dwords, cm / c4 the dwords left / right of
// them, u / d the dwords 3 rows up / down.  Bit k of the result: pixel k passes
// in some direction (bright or dark) -- a FAST candidate at t.
__device__ __forceinline__ uint32_t pretest16(uint32_t cm, const uint4& c, uint32_t c4, const uint4& u,
                                              const uint4& d, u16x2 tt) {
    const uint32_t cw[6] = {cm, c.x, c.y, c.z, c.w, c4};
    const uint32_t uw[4] = {u.x, u.y, u.z, u.w}, dw[4] = {d.x, d.y, d.z, d.w};
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t left = cw[k], cur = cw[k + 1], right = cw[k + 2];
        uint32_t b0, k0, b1, k1;
        // pixels (0, 2): left (-3, -1), right (3, 5); pixels (1, 3): left (-2, 0), right (4, 6)
        compass_signs(lo_bytes(cur), lo_bytes(uw[k]), lo_bytes(dw[k]), hi_bytes(left),
                      pair_bytes<0x0c050c03u>(right, cur), tt, b0, k0);
        compass_signs(hi_bytes(cur), hi_bytes(uw[k]), hi_bytes(dw[k]), pair_bytes<0x0c040c02u>(cur, left),
                      lo_bytes(right), tt, b1, k1);
        const uint32_t f = sign_bytes(b0 | k0, b1 | k1);           // byte j: pixel j passes (bit 7)
        bits |= __builtin_amdgcn_udot4(f >> 7, 0x08040201u, 0u, false) << (4 * k);
    }
    return bits;
}

// PRE: the fused iniThFAST pre-test (a test hook, ORB_OPT_PYR_PRETEST; the
// release path launches k_pyr_stream<false>, which carries none of its code)
template <bool PRE>
__global__ __launch_bounds__(1024) void k_pyr_stream(PyrStreamArgs a) {
    extern __shared__ uint4 ps_lds[];
    uint32_t* lds = (uint32_t*)ps_lds;
    const int f = blockIdx.x;
    if (f >= a.nframes) return;
    const int tid = threadIdx.x, lane = lane_id();
    for (int i = tid; i < a.tab_u4; i += 1024) ps_lds[i] = a.tab[i];
    if (a.cnt_dw >= 4 * a.tab_u4)                    // counters outside the image (ORB_OPT_PYR_CNT_END)
        for (int i = tid; i < a.nsteps; i += 1024) lds[a.cnt_dw + i] = 0;
    lds_barrier();
    // lane l: level l's tables A {column records dw, row records dw, HBM
    // offset, pitch} and B {ring dw | ring pitch dw << 16, ring rows | pre-test
    // group origin << 8 | bitmap pitch << 16, bitmap offset, -}
    const uint4 lva = ps_lds[a.lev_u4 + min(lane, a.L - 1)];
    const uint4 lvb = ps_lds[a.lev_u4 + a.L + min(lane, a.L - 1)];
    const uint8_t* src = a.src + f * a.src_fstride;
    uint8_t* pyr = a.pyr + f * a.pyr_fstride;
    uint8_t* bm = a.bm + f * a.bm_fstride;
    const int nq = (a.w0 + 15) >> 4;
    const float inv_nq = 1.0f / (float)nq;
    const u16x2 tt = {(unsigned short)a.ini_th, (unsigned short)a.ini_th};
    uint4 pre0 = make_uint4(0, 0, 0, 0), pre1 = pre0;
    // chunk c of level 0 -> registers (two 16-byte pieces per thread at most)
#define PS_FETCH(c)                                                                            \
    do {                                                                                       \
        const int r0_ = (c) * a.K0, n_ = min(a.K0, a.h0 - r0_) * nq;                           \
        if (tid < n_) {                                                                        \
            const int r_ = (int)(((float)tid + 0.5f) * inv_nq), q_ = tid - r_ * nq;            \
            pre0 = *(const uint4*)(src + (long long)(r0_ + r_) * a.src_pitch + 16 * q_);       \
        }                                                                                      \
        if (tid + 1024 < n_) {                                                                 \
            const int i_ = tid + 1024;                                                         \
            const int r_ = (int)(((float)i_ + 0.5f) * inv_nq), q_ = i_ - r_ * nq;              \
            pre1 = *(const uint4*)(src + (long long)(r0_ + r_) * a.src_pitch + 16 * q_);       \
        }                                                                                      \
    } while (0)
    // chunk c -> level 0's ring
    auto land = [&](int c, uint4 v0, uint4 v1) {
        const int r0 = c * a.K0, rows = min(a.K0, a.h0 - r0);
        const int base = r0 % a.ring0_rows;
        if (a.load_mode == 16) {
            const int n = rows * nq;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int i = tid + k * 1024;
                if (i < n) {
                    const int r = (int)(((float)i + 0.5f) * inv_nq), q = i - r * nq;
                    int slot = base + r;
                    if (slot >= a.ring0_rows) slot -= a.ring0_rows;
                    ps_lds[(a.ring0_dw + slot * (a.ring0_pitch >> 2)) / 4 + q] = k ? v1 : v0;
                }
            }
        } else if (a.load_mode == 4) {
            const int nd = (a.w0 + 3) >> 2, n = rows * nd;
            const float inv = 1.0f / (float)nd;
            for (int i = tid; i < n; i += 1024) {
                const int r = (int)(((float)i + 0.5f) * inv), q = i - r * nd;
                int slot = base + r;
                if (slot >= a.ring0_rows) slot -= a.ring0_rows;
                lds[a.ring0_dw + slot * (a.ring0_pitch >> 2) + q] =
                    *(const uint32_t*)(src + (long long)(r0 + r) * a.src_pitch + 4 * q);
            }
        } else {
            const int n = rows * a.w0;
            const float inv = 1.0f / (float)a.w0;
            uint8_t* l8 = (uint8_t*)lds;
            for (int i = tid; i < n; i += 1024) {
                const int r = (int)(((float)i + 0.5f) * inv), q = i - r * a.w0;
                int slot = base + r;
                if (slot >= a.ring0_rows) slot -= a.ring0_rows;
                l8[4 * a.ring0_dw + slot * a.ring0_pitch + q] = src[(long long)(r0 + r) * a.src_pitch + q];
            }
        }
    };
    if (a.load_mode == 16) PS_FETCH(0);
    for (int s = 0; s < a.nsteps; ++s) {
        if (s < a.nchunks) {
            land(s, pre0, pre1);
            if (a.load_mode == 16 && s + 1 < a.nchunks) PS_FETCH(s + 1);
        }
        // lane e >= 1 holds entry e of this step {first row, rows, first
        // wave-item, ng | runs << 16 (resize) / groups (pre-test)}: e < L the
        // resize of level e, e >= L the pre-test of level e - L; lane 0 {the
        // step's wave-items}
        const uint4 se = ps_lds[a.steps_u4 + s * a.E + min(lane, a.E - 1)];
        const int W = __builtin_amdgcn_readfirstlane((int)se.x);
        for (int it = 0; it <= W; ++it) {      // bounded: a wave never takes more than W items
            // wave-items are taken from a per-step LDS counter: waves that drew
            // cheap items take more, so the step ends when the work does.  The
            // counters are zeroes of the copied table image (dword 0 on); with
            // ORB_OPT_PYR_CNT_END they sit at the top of the allocation and are
            // zeroed above.  (Round 2 blamed a failing end-of-LDS layout on the
            // hardware; tests/test_gpu_configs.py runs that layout, zeroed,
            // bit-exact -- see DESIGN.md on the cause.)
            int jj = 0;
            if (lane == 0) jj = atomicAdd((int*)&lds[a.cnt_dw + s], 1);
            const int j = __builtin_amdgcn_readfirstlane(jj);
            if (j >= W) break;
            const int e = __builtin_popcountll(__ballot(lane >= 1 && lane < a.E && (int)se.z <= j));
            const int lo = __builtin_amdgcn_readlane((int)se.x, e), nrows = __builtin_amdgcn_readlane((int)se.y, e);
            const int wst = __builtin_amdgcn_readlane((int)se.z, e), ngr = __builtin_amdgcn_readlane((int)se.w, e);
            const int local = (j - wst) * kWave + lane;
            if (PRE && e >= a.L) {
                // pre-test of level m: lane = (row, 16-pixel group) of the step's rows
                const int m = e - a.L;
                const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)lvb.x, m);
                const uint32_t b1 = (uint32_t)__builtin_amdgcn_readlane((int)lvb.y, m);
                const uint32_t boff = (uint32_t)__builtin_amdgcn_readlane((int)lvb.z, m);
                const int rdw = b0 & 0xffff, pdw = b0 >> 16, rr = b1 & 0xff, gx0 = (b1 >> 8) & 0xff, bp = b1 >> 16;
                const int row = (int)(((float)local + 0.5f) * __builtin_amdgcn_rcpf((float)ngr));
                const int g = local - (int)__umul24((uint32_t)row, (uint32_t)ngr);
                if (row < nrows) {
                    const int y = lo + row, gg = gx0 + g;
                    const int sc = small_mod(y, rr, __builtin_amdgcn_rcpf((float)rr));
                    const int su = sc >= 3 ? sc - 3 : sc - 3 + rr, sd = sc + 3 < rr ? sc + 3 : sc + 3 - rr;
                    const int bc = rdw + (int)__umul24((uint32_t)sc, (uint32_t)pdw) + 4 * gg;
                    const uint4 c = ps_lds[bc >> 2];
                    const uint32_t cm = lds[bc - 1], c4 = lds[bc + 4];
                    const uint4 u = ps_lds[(rdw + (int)__umul24((uint32_t)su, (uint32_t)pdw)) / 4 + gg];
                    const uint4 d = ps_lds[(rdw + (int)__umul24((uint32_t)sd, (uint32_t)pdw)) / 4 + gg];
                    const uint32_t bits = pretest16(cm, c, c4, u, d, tt);
                    *(uint16_t*)(bm + boff + (uint32_t)y * (uint32_t)bp + 2 * gg) = (uint16_t)bits;
                }
                continue;
            }
            const int l = e;
            const int rec = __builtin_amdgcn_readlane((int)lva.x, l), ytd = __builtin_amdgcn_readlane((int)lva.y, l);
            const uint32_t loff = (uint32_t)__builtin_amdgcn_readlane((int)lva.z, l);
            const uint32_t lpitch = (uint32_t)__builtin_amdgcn_readlane((int)lva.w, l);
            const uint32_t rb0 = (uint32_t)__builtin_amdgcn_readlane((int)lvb.x, l);
            const int rr = __builtin_amdgcn_readlane((int)lvb.y, l) & 0xff;
            const bool ring_out = l < a.L - 1 || (PRE && a.pretest);   // the last level's rows feed only the pre-test
            const int runs = ngr >> 16, ng = ngr & 0xffff;
            const int run = (int)(((float)local + 0.5f) * __builtin_amdgcn_rcpf((float)ng));
            const int g = local - (int)__umul24(run, ng);
            if (run < runs) {
                // rows [y0, y1) of the step's nrows, split into `runs` nearly equal runs
                const float inv_runs = __builtin_amdgcn_rcpf((float)runs);
                const int y0 = lo + (int)(((float)__umul24(run, nrows) + 0.5f) * inv_runs);
                const int y1 = lo + (int)(((float)__umul24(run + 1, nrows) + 0.5f) * inv_runs);
                const int nr = y1 - y0;
                const uint4 wt = ps_lds[(rec >> 2) + g];
                const uint4 sl = ps_lds[(rec >> 2) + ng + g];
                const uint32_t bf = lds[rec + 8 * ng + g];
                const uint32_t bd = bf & 0xffff;
                const bool hi3 = (bf >> 19) & 1;        // output 3's taps in D1:D2 (outputs 0-2: D0:D1)
                // horizontal pass of one source row: the perm puts each tap pixel
                // in the high byte of its u16, so with weights 16a the dot product
                // is 4096 h and its upper half-word is OpenCV's h >> 4
                auto hrow = [&](const uint32_t (&d)[3], uint32_t (&hv)[4]) {
                    const uint32_t d0 = d[0], d1 = d[1], d2 = d[2];
                    hv[0] = __builtin_amdgcn_udot2(as_u16x2(__builtin_amdgcn_perm(d1, d0, sl.x)), as_u16x2(wt.x), 0u, false);
                    hv[1] = __builtin_amdgcn_udot2(as_u16x2(__builtin_amdgcn_perm(d1, d0, sl.y)), as_u16x2(wt.y), 0u, false);
                    hv[2] = __builtin_amdgcn_udot2(as_u16x2(__builtin_amdgcn_perm(d1, d0, sl.z)), as_u16x2(wt.z), 0u, false);
                    hv[3] = __builtin_amdgcn_udot2(as_u16x2(__builtin_amdgcn_perm(hi3 ? d2 : d1, hi3 ? d1 : d0, sl.w)),
                                                   as_u16x2(wt.w), 0u, false);
                };
                // every LDS read of the run first (row records, then both source
                // rows of every output row), so the run waits on LDS latency twice
                uint2 yr[kPsRun];
#pragma unroll
                for (int q = 0; q < kPsRun; ++q) yr[q] = ((const uint2*)lds)[(ytd >> 1) + y0 + min(q, nr - 1)];
                uint32_t D[kPsRun][2][3];
#pragma unroll
                for (int q = 0; q < kPsRun; ++q)
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        const uint32_t* Rp = lds + (t ? yr[q].x >> 16 : yr[q].x & 0xffff) + bd;
                        D[q][t][0] = Rp[0]; D[q][t][1] = Rp[1]; D[q][t][2] = Rp[2];
                    }
                // the run's ring slots: y0 % rr once, then consecutive with wrap
                int slot = ring_out ? small_mod(y0, rr, __builtin_amdgcn_rcpf((float)rr)) : 0;
                uint32_t hA[4], hB[4];
#pragma unroll
                for (int q = 0; q < kPsRun; ++q) {
                    if (q < nr) {
                        const uint32_t o0 = yr[q].x & 0xffff, o1 = yr[q].x >> 16;
                        // the top source row is usually the previous row's bottom one
                        if (q > 0 && o0 == (yr[q - 1].x >> 16)) {
#pragma unroll
                            for (int c = 0; c < 4; ++c) hA[c] = hB[c];
                        } else {
                            hrow(D[q][0], hA);
                        }
                        if (o1 == o0) {
#pragma unroll
                            for (int c = 0; c < 4; ++c) hB[c] = hA[c];
                        } else {
                            hrow(D[q][1], hB);
                        }
                        // OpenCV's ((b0 * (h0 >> 4)) >> 16) + ((b1 * (h1 >> 4)) >> 16) + 2) >> 2
                        const uint32_t b0 = yr[q].y & 0xffff, b1 = yr[q].y >> 16;
                        uint32_t out = 0;
#pragma unroll
                        for (int c = 0; c < 4; ++c) {
                            const uint32_t x0 = __umul24(b0, hA[c] >> 16), x1 = __umul24(b1, hB[c] >> 16);
                            out |= (((x0 >> 16) + (x1 >> 16) + 2) >> 2) << (8 * c);
                        }
                        if (ring_out) lds[(rb0 & 0xffff) + __umul24((uint32_t)slot, rb0 >> 16) + g] = out;
                        *(uint32_t*)(pyr + loff + (uint32_t)(y0 + q) * lpitch + 4 * g) = out;
                        if (++slot == rr) slot = 0;
                    }
                }
            }
        }
        lds_barrier();
    }
#undef PS_FETCH
}

// ---------------------------------------------------------------------------
// k_fast_cells: FAST-9/16 with 3x3 NMS per cell ROI, exact reformulation of
// cv::FAST on the ROI: score s(p) = max over the 16 arcs of
// 9 contiguous ring pixels of the arc's min |difference| - 1; corner at t iff
// s(p) >= t; NMS keeps p iff s(p) > s_t(q) for its 8 neighbours inside the
// cell's detection window.  One wave per cell, 4 cells per block.
// ---------------------------------------------------------------------------
struct FastArgs {
    const uint8_t* in;      // level 0 of every frame
    long long in_fstride;
    int in_pitch;
    const uint8_t* pyr;     // levels >= 1
    long long pyr_fstride;
    const LevelDev* lv;
    const CellDev* cells;
    int ncells;
    int cell_begin, cell_end;   // this launch's range of every frame's cells (a level range)
    int nframes;
    int* cell_count;        // [B][ncells]
    uint32_t* cell_keys;    // [B][slot_total]
    int slot_total;
    int ini_th, min_th;
    int roi_max, win_max;   // LDS per wave
    int kmask_bytes;        // NMS ballots of the separate output pass (0 with ORB_FAST_FUSED_OUT)
    int cand_bytes;         // u16 candidate list of cand_cap entries
    int cand_cap;           // a cell whose candidates exceed it takes the dense path (fast_dense_cell)
    int ilist_bytes;      // u32 list of the pre-test items holding a candidate (ORB_FAST_EMIT 1;
                            // 0 with ORB_FAST_ILIST_IN_MAP: the list lives in the score map's bytes)
    const uint8_t* bm;      // k_pyr_stream's iniThFAST pre-test bitmaps of frame 0 (k_fast_cells<..., true>)
    long long bm_fstride;
};

// Arc strength of one direction on the raw ring values: max over the 16 arcs
// of 9 contiguous ring pixels of min(x ^ m), m = 0 (brighter ring: the arc's
// min x) or 0xff (darker ring: 255 - the arc's max x).  With d = v - x,
// cv::FAST's score is max(A, B) - 1 for B = strength(0) - v and
// A = strength(0xff) - (255 - v).
// v_min3 / v_max3 by hand: the shared pairwise minima of the arc windows keep
// the compiler from forming them (it emitted 45 two-input v_min per score)
__device__ __forceinline__ int vmin3(int a, int b, int c) {
    int d;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ int vmax3(int a, int b, int c) {
    int d;
    asm("v_max3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ int arc_strength(const int (&x)[16], int m) {
    int w[16], w3[16], a9[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = x[k] ^ m;
#pragma unroll
    for (int k = 0; k < 16; ++k) w3[k] = vmin3(w[k], w[(k + 1) & 15], w[(k + 2) & 15]);
#pragma unroll
    for (int k = 0; k < 16; ++k) a9[k] = vmin3(w3[k], w3[(k + 3) & 15], w3[(k + 6) & 15]);
    int a = vmax3(a9[0], a9[1], a9[2]);
#pragma unroll
    for (int k = 3; k < 15; k += 2) a = vmax3(a, a9[k], a9[k + 1]);
    return max(a, a9[15]);
}

// a * b + c for a, b < 2^24 in one full-rate v_mad_u32_u24: with __umul24
// the compiler, unable to bound a min() result, fuses the product and the add
// into a quarter-rate v_mad_u64_u32
__device__ __forceinline__ uint32_t mad24(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// RP > 0: the ROI pitch is the compile-time RP dwords (every ring read an
// immediate offset from one base); 0: the runtime stride
template <int RP>
__device__ __forceinline__ void fast_ring(const uint8_t* roi, int stride, int r, int c, int& v, int (&x)[16]) {
    if (RP) stride = 4 * RP;
    const uint8_t* p = roi + (RP ? r * (4 * RP) + c : (int)mad24((uint32_t)r, (uint32_t)stride, (uint32_t)c));
    v = p[0];
    x[0] = p[3 * stride];
    x[1] = p[3 * stride + 1];
    x[2] = p[2 * stride + 2];
    x[3] = p[stride + 3];
    x[4] = p[3];
    x[5] = p[-stride + 3];
    x[6] = p[-2 * stride + 2];
    x[7] = p[-3 * stride + 1];
    x[8] = p[-3 * stride];
    x[9] = p[-3 * stride - 1];
    x[10] = p[-2 * stride - 2];
    x[11] = p[-stride - 3];
    x[12] = p[-3];
    x[13] = p[stride - 3];
    x[14] = p[2 * stride - 2];
    x[15] = p[3 * stride - 1];
}

// Score of one direction (dark = 0: brighter ring, 1: darker ring) minus one.
// A pixel whose compass pre-test at the pass threshold t fails in a direction
// has that direction's strength - 1 < t, so dropping it changes no score >= t,
// and scores < t act as 0 in the NMS at t: the candidate's score is the max
// over its passing directions only (exact for the NMS at t).
__device__ __forceinline__ int fast_dir_score(const int (&x)[16], int v, int dark) {
    const int m = dark ? 0xff : 0;
    return arc_strength(x, m) - (v ^ m) - 1;
}

// NMS on the zero-padded score map (pitch ww+2): p survives at threshold t iff
// s(p) >= max(t, 1) and s(p) > s_t(q) for its 8 neighbours, s_t(q) = s(q) if
// s(q) >= t else 0; the zero border stands for pixels outside the window.
__device__ __forceinline__ bool nms_keep(const uint8_t* sc, int sp, int r, int c, int t, int& s) {
    const uint8_t* p = sc + mad24((uint32_t)(r + 1), (uint32_t)sp, (uint32_t)(c + 1));
    s = p[0];
    if (s < max(t, 1)) return false;
    const int q[8] = {p[-sp - 1], p[-sp], p[-sp + 1], p[-1], p[1], p[sp - 1], p[sp], p[sp + 1]};
    bool keep = true;
#pragma unroll
    for (int k = 0; k < 8; ++k) keep &= s > (q[k] >= t ? q[k] : 0);
    return keep;
}

constexpr int kCandIdx = 0x3fff, kCandBright = 0x4000, kCandDark = 0x8000;

#ifdef ORB_FAST_TIMING
// phase profile of k_fast_cells (tools/fast_phases.py): shader cycles per phase
__device__ unsigned long long g_fast_t[1024][16];   // spread: no contended atomics
#define FAST_T(k)                                                            \
    do {                                                                     \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();          \
        const unsigned long long d_ = t_ - tlast;                            \
        tlast = t_;                                                          \
        switch (k) {                                                         \
            case 0: t0 += d_; break;                                         \
            case 1: t1 += d_; break;                                         \
            case 2: t2 += d_; break;                                         \
            case 3: t3 += d_; break;                                         \
            case 5: t5 += d_; break;                                         \
            case 6: t6 += d_; break;                                         \
            case 7: t7 += d_; break;                                         \
            case 10: t10 += d_; break;                                       \
            default: t9 += d_; break;                                        \
        }                                                                    \
    } while (0)
#else
#define FAST_T(k) do { } while (0)
#endif

// each wave of k_fast_cells owns its cells and its LDS region: wave-level sync only
__device__ __forceinline__ void fast_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// XCD-aware block order (ORB_XCD_REMAP): the hardware deals the blocks of a
// launch round-robin over the 8 XCDs (linear id L to XCD L % 8).  Over a grid
// of `per` units x B frames, XCD x is given frames x, x + 8, x + 16, ...
// (the XCD whose L2 k_pyr_stream wrote them through: one block per frame),
// each frame's units in order, so a frame's neighbouring cells or patches --
// which share ROI rows and cache lines -- meet in one L2.  Identity when B is
// not a multiple of 8.
#ifndef ORB_XCD_REMAP
#define ORB_XCD_REMAP 1
#endif
__device__ __forceinline__ void xcd_remap(int per, int B, int& unit, int& frame) {
    const int L = (int)blockIdx.x + per * (int)blockIdx.y;
    if (!ORB_XCD_REMAP || (B & 7)) { unit = blockIdx.x; frame = blockIdx.y; return; }
    const int x = L & 7, k = L >> 3;
    const int fl = k / per;
    unit = k - fl * per;
    frame = 8 * fl + x;
}

// row/column of linear window index i (ww <= 4096): exact via a float reciprocal
__device__ __forceinline__ int div_row(int i, float inv_ww) { return (int)(((float)i + 0.5f) * inv_ww); }

#ifndef ORB_FAST_RC
#define ORB_FAST_RC 1   // candidate entries hold (row, column) as 7-bit fields (0: the window's linear index)
#endif
// A candidate's 14-bit window position: row | column << 7 (windows are < 70
// px a side: wCell = ceil(width / floor(width / 35)) < 70; the plan checks
// < 128), so it decodes in two ops instead of a float-reciprocal division
constexpr int kCandColStep = ORB_FAST_RC ? 128 : 1;
__device__ __forceinline__ int cand_enc(int r, int c, int ww) {
    return ORB_FAST_RC ? (r | (c << 7)) : (int)__umul24((uint32_t)r, (uint32_t)ww) + c;
}
__device__ __forceinline__ void cand_dec(int i, float inv_ww, int ww, int& r, int& c) {
    if (ORB_FAST_RC) {
        r = i & 127;
        c = i >> 7;
    } else {
        r = div_row(i, inv_ww);
        c = i - (int)__umul24((uint32_t)r, (uint32_t)ww);
    }
}

#ifndef ORB_FAST_CELLS_PER_WAVE
// 2 with one-wave blocks (FAST 0.321-0.325 -> 0.315-0.320 ms in four same-box
// A/B pairs; 8 cells: 0.35 ms)
#define ORB_FAST_CELLS_PER_WAVE 2
#endif
constexpr int kCellsPerWave = ORB_FAST_CELLS_PER_WAVE;
#ifndef ORB_FAST_WPB
// waves per k_fast_cells block: each wave owns its cells and its LDS region,
// so one-wave blocks free their LDS the moment their wave ends instead of
// waiting for the slowest of four (FAST 0.345 -> 0.327 ms, same-box A/B)
#define ORB_FAST_WPB 1
#endif
constexpr int kFastWpb = ORB_FAST_WPB;
#ifndef ORB_FAST_PRE2
#define ORB_FAST_PRE2 0
#endif
#ifndef ORB_FAST_EMIT
#define ORB_FAST_EMIT 1   // 1: items list + one expansion pass; 0: per-round bit loops (round 2)
#endif
#ifndef ORB_FAST_FIXED_PITCH
#define ORB_FAST_FIXED_PITCH 1   // ROIs of <= 13 dwords land at a compile-time LDS pitch (11 or 13)
#endif
#ifndef ORB_FAST_KEEPLIST
#define ORB_FAST_KEEPLIST 1   // the NMS list keeps only candidates scoring >= max(t, 1)
#endif
#if ORB_FAST_RESET && ORB_FAST_KEEPLIST
#error "ORB_FAST_RESET needs every scored candidate in the list (ORB_FAST_KEEPLIST=0)"
#endif
#ifndef ORB_FAST_DIAG
#define ORB_FAST_DIAG 1   // diagonal-pair filter on the candidate list before scoring
#endif
#ifndef ORB_FAST_FUSED_OUT
#define ORB_FAST_FUSED_OUT 1   // survivors written inside the NMS loop (0: a separate output pass)
#endif
#ifndef ORB_FAST_RESET
#define ORB_FAST_RESET 0   // 1: score map zeroed once per wave, each cell resets its own entries (measured slower: 0.418-0.420 vs 0.408-0.413 ms)
#endif
#ifndef ORB_FAST_ILIST_IN_MAP
// the pre-test's item list lives in the score map's bytes (the list is read
// out before the map is zeroed and scored; 1 KB less LDS a wave at 752x480,
// 16 -> 17-18 waves a CU)
#define ORB_FAST_ILIST_IN_MAP 1
#endif
#if ORB_FAST_ILIST_IN_MAP && ORB_FAST_RESET
#error "ORB_FAST_RESET keeps the score map zero between cells: the item list cannot live in it"
#endif
#ifndef ORB_FAST_PIPE
#define ORB_FAST_PIPE 0   // 1: pre-test LDS reads one round ahead (ORB_FAST_EMIT 1)
#endif
#ifndef ORB_FAST_INC
#define ORB_FAST_INC 0    // 1: pre-test item (row, pair) advanced by a carry per round (measured: time neutral, VALU per wave 1,686 -> 1,749); 0: divided per round
#endif
#ifndef ORB_FAST_CELLOFF
#define ORB_FAST_CELLOFF 1   // ROI address from the cell record alone (0: through the level table)
#endif
#ifndef ORB_QT_LEVEL_MAJOR
#define ORB_QT_LEVEL_MAJOR 1
#endif
#ifndef ORB_FAST_ABL
#define ORB_FAST_ABL 0   // timing ablations (tools only; wrong results): 1 scores, 2 compaction, 3 compass, 4 L2-resident ROIs
#endif
// The candidate list is sized for the typical cell, not the worst one: a cell
// whose pre-test leaves more candidates than FastArgs::cand_cap is scored
// densely instead (every window pixel, both directions, straight into the
// score map; the NMS then walks the window in row-major order), which needs no
// list at all.  The cap comes from an LDS budget of ORB_FAST_WAVES_CU waves a
// CU (the 8.7 KB worst-case list capped k_fast_cells at 17-18 waves a CU).
#ifndef ORB_FAST_WAVES_CU
#define ORB_FAST_WAVES_CU 24
#endif
constexpr bool kFastDense = ORB_FAST_FUSED_OUT && ORB_FAST_EMIT == 1 && !ORB_FAST_RESET && ORB_FAST_ILIST_IN_MAP;

// A cell's ROI lands in LDS row-major at its own pitch of nd dwords (dense:
// the banks of the pre-test's row reads spread as before).  It is fetched as
// rows of PDW >= nd dwords, lane i + 64 j holding row (i + 64 j) / PDW, dword
// (i + 64 j) % PDW: lanes past nd re-read dword nd - 1 and rows past the ROI
// its last row (identical values to identical places), so the NV loads per
// lane issue back to back, branch-free, with a clamp and a multiply-add of
// address math each (the float-reciprocal split of a linear index cost ~14
// VALU per load).
// Global-address-space views: image pointers that reach a loop through
// readlanes lose their address space, and flat loads also count in lgkmcnt
// (the next LDS wait would drain a prefetch); a uniform base plus a 32-bit
// offset also gives the saddr form of global_load.
typedef __attribute__((address_space(1))) const uint8_t* GlobalBytes;
typedef __attribute__((address_space(1))) const uint32_t* GlobalWords;

struct RoiFetch {
    const uint8_t* src;     // ROI row 0, dword 0 (level row y0, column x0 & ~3)
    int pitch, nd, rows;
};

// Addresses as 32-bit offsets from the cell's uniform row-0 pointer (one
// v_mad_u32_u24 per load: a 64-bit product per load was two quarter-rate
// v_mad_u64_u32, and the landing's r * nd a quarter-rate v_mul_lo_u32).
#ifndef ORB_FAST_ROWLOAD
#define ORB_FAST_ROWLOAD 2   // lane r fetches ROI row r (16-dword, 16-load forms; one address per lane): 2 in 16-byte groups (FAST 264.5-265.3 -> 260.4-261.7 us), 1 dword by dword (268.7-268.8 -> 265.1-266.1 us, VGPRs 95 -> 78; profiles/r05/fast_rowload_*); 0: the spread
#endif
template <int PDW, int NV>
__device__ __forceinline__ void roi_issue(const RoiFetch& rf, uint32_t (&v)[NV]) {
    static_assert(kWave % PDW == 0, "rows of a load round are whole");
    const int lane = lane_id();
#if ORB_FAST_ROWLOAD
    if constexpr (PDW == 16 && NV == 16) {
        // rows <= 64 in this form (NV * 64 / PDW); the dword offsets are immediates
        const GlobalWords p = (GlobalWords)((GlobalBytes)rf.src + (uint32_t)min(lane, rf.rows - 1) * (uint32_t)rf.pitch);
#if ORB_FAST_ROWLOAD == 2
        // whole groups of 4 dwords as one 16-byte load each (4 line requests
        // a lane instead of nd); the group holding the ROI's end dword by dword
#pragma unroll
        for (int g = 0; g < NV / 4; ++g) {
            if (4 * g + 3 < rf.nd) {
#pragma unroll
                for (int k = 0; k < 4; ++k) v[4 * g + k] = p[4 * g + k];
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (4 * g + k < rf.nd) v[4 * g + k] = p[4 * g + k];
            }
        }
#else
#pragma unroll
        for (int k = 0; k < NV; ++k)
            if (k < rf.nd) v[k] = p[k];
#endif
        return;
    }
#endif
    const uint32_t col = 4u * (uint32_t)min(lane % PDW, rf.nd - 1);
    const GlobalBytes base = (GlobalBytes)rf.src;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const uint32_t r = (uint32_t)min(lane / PDW + j * (kWave / PDW), rf.rows - 1);
        v[j] = *(GlobalWords)(base + mad24(r, (uint32_t)rf.pitch, col));
    }
}

template <int PDW, int NV, int RP>
__device__ __forceinline__ void roi_land(const RoiFetch& rf, const uint32_t (&v)[NV], uint32_t* roi) {
    const int lane = lane_id();
#if ORB_FAST_ROWLOAD
    if constexpr (PDW == 16 && NV == 16) {
        if (lane < rf.rows) {
            uint32_t* q = roi + mad24((uint32_t)lane, (uint32_t)(RP ? RP : rf.nd), 0u);
#pragma unroll
            for (int k = 0; k < NV; ++k)
                if (k < rf.nd) q[k] = v[k];
        }
        return;
    }
#endif
    const uint32_t d = (uint32_t)min(lane % PDW, rf.nd - 1);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const uint32_t r = (uint32_t)min(lane / PDW + j * (kWave / PDW), rf.rows - 1);
        // (r * RP by v_mad_u32_u24: the compiler's r * RP was a quarter-rate
        // v_mul_lo_u32 per landed dword, r being a min() it cannot bound)
        if (RP) roi[mad24(r, (uint32_t)RP, d)] = v[j];
        else roi[mad24(r, (uint32_t)rf.nd, d)] = v[j];
    }
}

#if !defined(ORB_FAST_WPE) && ORB_FAST_WAVES_CU % 4 == 0
#define ORB_FAST_WPE (ORB_FAST_WAVES_CU / 4)   // registers for the LDS budget's occupancy (79 VGPRs, no spills)
#endif
#ifdef ORB_FAST_WPE
#define FAST_WPE_ATTR __attribute__((amdgpu_waves_per_eu(ORB_FAST_WPE)))
#else
#define FAST_WPE_ATTR
#endif
// RP: the LDS pitch of a landed ROI in dwords, fixed at compile time (every
// row offset of the pre-test, the ring and the diagonal reads an immediate),
// or 0 for each cell's own nd

// The iniThFAST candidates of a cell's window from k_pyr_stream's bitmap
// (k_fast_cells<..., BM = true>): lane r holds window row r's bitmap dwords
// (the 3 dwords from the one holding the window's first column: a window is
// <= 64 columns, so its bits lie within 96), issued one cell ahead like the ROI.
struct BmFetch {
    const uint8_t* row0;    // the bitmap row of window row 0, dword-aligned at the window's first column
    int pitch, sh, ww, wh;
};
__device__ __forceinline__ void bm_issue(const BmFetch& bf, uint32_t (&w)[3]) {
    const int r = min(lane_id(), max(bf.wh - 1, 0));
    const GlobalWords p = (GlobalWords)(bf.row0 + (uint32_t)r * (uint32_t)bf.pitch);
    w[0] = p[0]; w[1] = p[1]; w[2] = p[2];
}

template <int PDW, int NV, int RP, bool BM>
__global__ __launch_bounds__(256) FAST_WPE_ATTR void k_fast_cells(FastArgs a) {
    static_assert(!BM || ORB_FAST_DIAG, "bitmap candidates get their compass directions in the diagonal filter");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = lane_id(), wv = wave_id();
    uint8_t* roi = smem + wv * (a.roi_max + a.win_max + a.cand_bytes + a.kmask_bytes + a.ilist_bytes);   // multiples of 16
    uint8_t* sc = roi + a.roi_max;                            // padded score map, <= win_max bytes
    uint16_t* cand = (uint16_t*)(sc + a.win_max);             // <= win_pix_max entries
    uint64_t* kmask = (uint64_t*)(sc + a.win_max + a.cand_bytes);   // NMS ballots, one per 64 candidates
    uint32_t* ilist = ORB_FAST_ILIST_IN_MAP ? (uint32_t*)sc   // items holding candidates
                                            : (uint32_t*)(sc + a.win_max + a.cand_bytes + a.kmask_bytes);
#ifdef ORB_FAST_TIMING
    const unsigned long long t_start = __builtin_amdgcn_s_memtime();
#endif
    // work items it = frame * ncells + cell
    int bunit, bframe;
    xcd_remap((int)gridDim.x, (int)gridDim.y, bunit, bframe);
    bunit = __builtin_amdgcn_readfirstlane(bunit);
    bframe = __builtin_amdgcn_readfirstlane(bframe);
    const int c_begin = a.cell_begin + (bunit * kFastWpb + wv) * kCellsPerWave;
    const int it0 = bframe * a.ncells + c_begin, step = 1;
    const int it_end = bframe * a.ncells + min(c_begin + kCellsPerWave, a.cell_end);
    // the plan tables are read-only here: constant address space -> scalar loads
    typedef __attribute__((address_space(4))) const LevelDev* ConstLevels;
    typedef __attribute__((address_space(4))) const CellDev* ConstCells;
    const ConstLevels lvc = (ConstLevels)a.lv;
    const ConstCells cells = (ConstCells)a.cells;
    auto cell_at = [&](int it) {
        const int i = it - bframe * a.ncells;   // frame = bframe: no division
        CellDev r;
        r.level = cells[i].level; r.x0 = cells[i].x0; r.y0 = cells[i].y0; r.cols = cells[i].cols;
        r.rows = cells[i].rows; r.slot_off = cells[i].slot_off; r.cap = cells[i].cap;
        r.roi_off = cells[i].roi_off; r.pitch = cells[i].pitch;
        return r;
    };
    auto fetch_of = [&](const CellDev& c, int it) {
        const int f = bframe;
        RoiFetch rf;
#if ORB_FAST_CELLOFF
        if (c.level == 0) {
            rf.pitch = a.in_pitch;
            rf.src = a.in + f * a.in_fstride + (long long)c.y0 * rf.pitch + (c.x0 & ~3);
        } else {
            rf.pitch = c.pitch;
            rf.src = a.pyr + f * a.pyr_fstride + c.roi_off;
        }
#else
        if (c.level == 0) { rf.src = a.in + f * a.in_fstride; rf.pitch = a.in_pitch; }
        else { rf.src = a.pyr + f * a.pyr_fstride + lvc[c.level].off; rf.pitch = lvc[c.level].pitch; }
        rf.src += (long long)c.y0 * rf.pitch + (c.x0 & ~3);
#endif
        rf.nd = max(1, ((c.x0 & 3) + c.cols + 3) >> 2);
        rf.rows = max(1, c.rows);
#if ORB_FAST_ABL == 4
        rf.src = a.in + (c.x0 & ~3);   // ablation: every ROI from frame 0's first rows, L2-resident (timing only)
        rf.pitch = a.in_pitch;
#endif
        return rf;
    };
    auto bm_of = [&](const CellDev& c) {
        BmFetch bf;
        const int xs = c.x0 + 3;
        bf.pitch = lvc[c.level].bm_pitch;
        bf.row0 = a.bm + bframe * a.bm_fstride + lvc[c.level].bm_off + (long long)(c.y0 + 3) * bf.pitch + 4 * (xs >> 5);
        bf.sh = xs & 31;
        bf.ww = max(0, c.cols - 6);
        bf.wh = max(0, c.rows - 6);
        return bf;
    };
    // cell descriptors (scalar loads) run two cells ahead, ROI (and bitmap) loads one cell ahead
    uint32_t v[NV];
    uint32_t bmw[3] = {0u, 0u, 0u};
    CellDev c{}, cn{};
    RoiFetch rf{};
    BmFetch bfc{};
    if (it0 < it_end) {
        c = cell_at(it0);
        rf = fetch_of(c, it0);
        roi_issue<PDW, NV>(rf, v);
        if (BM) {
            bfc = bm_of(c);
            bm_issue(bfc, bmw);
        }
    }
    if (it0 + step < it_end) cn = cell_at(it0 + step);
#ifdef ORB_FAST_TIMING
    unsigned long long t0 = 0, t1 = 0, t2 = 0, t3 = 0, t5 = 0, t6 = 0, t7 = 0, t9 = 0, t10 = 0;
    unsigned long long tlast = t_start;
#endif
    auto land = [&](const uint32_t (&vv)[NV], const RoiFetch& r) { roi_land<PDW, NV, RP>(r, vv, (uint32_t*)roi); };
    // one cell from its landed ROI
    auto process = [&](const CellDev& cur, const RoiFetch& rfc, const BmFetch& bfw, const uint32_t (&bw)[3], int it) {
        const int f = bframe;
        const int rstride = (RP ? RP : rfc.nd) * 4;
        const int shift = cur.x0 & 3;
        const uint8_t* R = roi + shift;
        const int ww = max(0, cur.cols - 6), wh = max(0, cur.rows - 6);
        const int sp = ww + 2, npad = sp * (wh + 2);
#if ORB_FAST_RESET
        (void)npad;   // the map is all zero here: zeroed once, and each cell resets the entries it wrote
#elif !ORB_FAST_ILIST_IN_MAP
        // 16 bytes per lane per store (sc is 16-byte aligned, win_max a multiple of 16)
        for (int i = lane; i < (npad + 15) / 16; i += kWave) ((uint4*)sc)[i] = make_uint4(0u, 0u, 0u, 0u);
        fast_wave_sync();
#endif
        if (it == it0) FAST_T(10); else FAST_T(0);
        const float inv_ww = ww ? 1.0f / (float)ww : 0.f;
        const int X0 = shift + 3, j0 = X0 >> 2;
        const int ndw = ww ? ((X0 + ww - 1) >> 2) - j0 + 1 : 0;
        const int ndp = (ndw + 1) >> 1;                   // items: pairs of aligned dwords
        const int nitems = wh * ndp;
        // (an approximate reciprocal is exact here: (i + 0.5) / ndp < wh lies
        // >= 1 / (2 ndp) from an integer, while v_rcp's 1 ulp and the product's
        // rounding err by < wh * 2^-21, smaller whenever nitems < 2^20)
        const float inv_ndp = ndp ? __builtin_amdgcn_rcpf((float)ndp) : 0.f;
        const uint32_t* roi32 = (const uint32_t*)roi;
        const int rs4 = rstride >> 2;
        // byte-flag masks of the first and the last item of a row (the only
        // partial ones: X0 - 4 j0 is in [0, 3])
        uint64_t m_first = 0, m_last = 0;
        if (ndp) {
            const int cxf = 4 * j0 - X0, cxl = 4 * (j0 + 2 * (ndp - 1)) - X0;
            m_first = item_byte_mask(min(max(-cxf, 0), 8), min(max(ww - cxf, 0), 8));
            m_last = item_byte_mask(min(max(-cxl, 0), 8), min(max(ww - cxl, 0), 8));
        }
        // The dense form of a cell from pass p0 on: the exact score s(p) of
        // every window pixel (max of both directions, 0 below 1) in the map,
        // then the NMS of each remaining pass over the window in row-major
        // order -- the reference's definition itself, for the cells whose
        // candidates overflow the list.  Returns the survivors of the deciding
        // pass (written like the list form's).
        auto dense_cell = [&](int p0) -> int {
            fast_wave_sync();   // the item list (in the map's bytes) is read out
            for (int i = lane; i < (npad + 15) / 16; i += kWave) ((uint4*)sc)[i] = make_uint4(0u, 0u, 0u, 0u);
            fast_wave_sync();
            const int npix = ww * wh;
            for (int q0 = 0; q0 < npix; q0 += kWave) {
                const int q = q0 + lane;
                if (q < npix) {
                    const int r = div_row(q, inv_ww), cc = q - (int)__umul24((uint32_t)r, (uint32_t)ww);
                    int v, x[16];
                    fast_ring<RP>(R, rstride, r + 3, cc + 3, v, x);
                    const int sv = max(max(fast_dir_score(x, v, 0), fast_dir_score(x, v, 1)), 0);
                    sc[mad24((uint32_t)(r + 1), (uint32_t)sp, (uint32_t)(cc + 1))] = (uint8_t)sv;
                }
            }
            fast_wave_sync();
            uint32_t* outp = a.cell_keys + (long long)f * a.slot_total + cur.slot_off;
            int n = 0;
            for (int pass = p0; pass < 2; ++pass) {
                const int t = pass == 0 ? a.ini_th : a.min_th;
                n = 0;
                for (int q0 = 0; q0 < npix; q0 += kWave) {
                    const int q = q0 + lane;
                    bool keep = false;
                    uint32_t key = 0;
                    if (q < npix) {
                        const int r = div_row(q, inv_ww), cc = q - (int)__umul24((uint32_t)r, (uint32_t)ww);
                        int sv;
                        keep = nms_keep(sc, sp, r, cc, t, sv);
                        key = (uint32_t)(cur.x0 + cc + 3 - (kEdge - 3)) | ((uint32_t)(cur.y0 + r + 3 - (kEdge - 3)) << 12) |
                              ((uint32_t)sv << 24);
                    }
                    const uint64_t m = __ballot(keep);
                    if (keep) {
                        const int pos = n + mask_rank(m);
                        if (pos < cur.cap) outp[pos] = key;
                    }
                    n += __popcll(m);
                }
                if (n > 0) break;
            }
            fast_wave_sync();
            return n;
        };
        int dense_from = -1;    // pass at which the candidates overflowed the list
        // FAST(ROI, iniThFAST) and, only if that leaves no corner, FAST(ROI,
        // minThFAST) (ORBextractor.cc:826-846).  Each pass pre-tests at its own
        // threshold, so the iniTh pass scores far fewer pixels; scores stored by
        // the first pass stay exact for the second (its candidates are a superset).
        int ncand = 0, cnt = 0;
        for (int pass = 0; pass < 2; ++pass) {
            const int t = pass == 0 ? a.ini_th : a.min_th;
            // 1. compass pre-test on (row, aligned dword) items: candidates in
            //    row-major order tagged with their passing directions (~4% of
            //    pixels pass, ~8% of items hold one, so the compaction writes
            //    loop over the set bits instead of visiting all four bytes)
            const u16x2 tt = {(unsigned short)t, (unsigned short)t};
#if ORB_FAST_LERP
            const LerpTh lth = lerp_thresholds(t);
#endif
            ncand = 0;
            // one item: flag bytes (byte k = item pixel k) and its window index
            // item (row r, dword pair k) -> flag bytes; ok: the item exists
            auto pretest_rk = [&](bool ok, int r, int k, uint32_t& bl, uint32_t& bh, uint32_t& dl, uint32_t& dh,
                                  int& idx0) {
#if ORB_FAST_LERP
                {   // branch-free: the caller clamps a missing item onto the last one, ok = 0 clears its flags
#else
                bl = bh = dl = dh = 0;
                idx0 = 0;
                if (ok) {
#endif
                    const int j = j0 + 2 * k;
                    const uint32_t* row = roi32 + __umul24(r + 3, rs4) + j;
                    const uint32_t cm = row[-1], c0 = row[0], c1 = row[1], c2 = row[2];
                    const uint32_t u0 = row[-3 * rs4], u1 = row[1 - 3 * rs4];
                    const uint32_t d0 = row[3 * rs4], d1 = row[1 + 3 * rs4];
#if ORB_FAST_LERP
                    uint64_t vm = k == 0 ? m_first : (k == ndp - 1 ? m_last : 0x8080808080808080ull);
                    if (!ok) vm = 0;
                    const uint32_t vl = (uint32_t)vm, vh = (uint32_t)(vm >> 32);
                    uint32_t br0, dx0, br1, dx1;
                    // the pixels 3 left / 3 right of each dword's 4: one v_alignbyte each
                    compass_lerp(c0, u0, d0, __builtin_amdgcn_alignbyte(c0, cm, 1), __builtin_amdgcn_alignbyte(c1, c0, 3),
                                 lth, br0, dx0);
                    compass_lerp(c1, u1, d1, __builtin_amdgcn_alignbyte(c1, c0, 1), __builtin_amdgcn_alignbyte(c2, c1, 3),
                                 lth, br1, dx1);
                    bl = br0 & vl;
                    bh = br1 & vh;
                    dl = ~dx0 & vl;
                    dh = ~dx1 & vh;
                    idx0 = cand_enc(r, 4 * j - X0, ww);
                    (void)tt;
#else
                    // u16 pairs of the pixels 3 left / 3 right of pixels (0, 2) and
                    // (1, 3) of dwords c0, c1: one v_perm each, four shared with C
                    const uint32_t c0l = lo_bytes(c0), c0h = hi_bytes(c0), c1l = lo_bytes(c1), c1h = hi_bytes(c1);
                    const uint32_t lf0l = hi_bytes(cm), lf0h = pair_bytes<0x0c040c02u>(c0, cm);
                    const uint32_t rt0l = pair_bytes<0x0c050c03u>(c1, c0), rt0h = c1l;
                    const uint32_t lf1l = c0h, lf1h = pair_bytes<0x0c040c02u>(c1, c0);
                    const uint32_t rt1l = pair_bytes<0x0c050c03u>(c2, c1), rt1h = lo_bytes(c2);
                    uint32_t b0, k0, b1, k1, b2, k2, b3, k3;
#if ORB_FAST_ABL == 3
                    // ablation: one compass evaluation stands in for all four (timing only)
                    compass_signs(c0l, lo_bytes(u0), lo_bytes(d0), lf0l, rt0l, tt, b0, k0);
                    b1 = b2 = b3 = b0; k1 = k2 = k3 = k0;
#else
                    compass_signs(c0l, lo_bytes(u0), lo_bytes(d0), lf0l, rt0l, tt, b0, k0);
                    compass_signs(c0h, hi_bytes(u0), hi_bytes(d0), lf0h, rt0h, tt, b1, k1);
                    compass_signs(c1l, lo_bytes(u1), lo_bytes(d1), lf1l, rt1l, tt, b2, k2);
                    compass_signs(c1h, hi_bytes(u1), hi_bytes(d1), lf1h, rt1h, tt, b3, k3);
#endif
                    const uint64_t vm = k == 0 ? m_first : (k == ndp - 1 ? m_last : 0x8080808080808080ull);
                    const uint32_t vl = (uint32_t)vm, vh = (uint32_t)(vm >> 32);
                    bl = sign_bytes(b0, b1) & vl;
                    bh = sign_bytes(b2, b3) & vh;
                    dl = sign_bytes(k0, k1) & vl;
                    dh = sign_bytes(k2, k3) & vh;
                    idx0 = cand_enc(r, 4 * j - X0, ww);
#endif
                }
            };
            auto pretest = [&](int it, uint32_t& bl, uint32_t& bh, uint32_t& dl, uint32_t& dh, int& idx0) {
#if ORB_FAST_LERP
                const int itc = min(it, nitems - 1);
#else
                const int itc = it;
#endif
                const int r = div_row(itc, inv_ndp);
                pretest_rk(it < nitems, r, itc - (int)__umul24(r, ndp), bl, bh, dl, dh, idx0);
            };
#if ORB_FAST_PIPE
            // the same pre-test split at its LDS reads, so the reads of round
            // r + 1 are in flight while round r is evaluated (the ilist store
            // between them would otherwise keep the compiler from hoisting)
            struct PreIn {
                uint32_t cm, c0, c1, c2, u0, u1, d0, d1;
                int k;
            };
            auto pre_load = [&](int it, PreIn& q) {
                const int itc = min(it, nitems - 1);
                const int r = div_row(itc, inv_ndp);
                q.k = itc - (int)__umul24(r, ndp);
                const uint32_t* row = roi32 + __umul24(r + 3, rs4) + (j0 + 2 * q.k);
                q.cm = row[-1]; q.c0 = row[0]; q.c1 = row[1]; q.c2 = row[2];
                q.u0 = row[-3 * rs4]; q.u1 = row[1 - 3 * rs4];
                q.d0 = row[3 * rs4]; q.d1 = row[1 + 3 * rs4];
            };
            auto pre_eval = [&](const PreIn& q, bool ok, uint32_t& bl, uint32_t& bh, uint32_t& dl, uint32_t& dh) {
                const uint32_t c0l = lo_bytes(q.c0), c0h = hi_bytes(q.c0), c1l = lo_bytes(q.c1), c1h = hi_bytes(q.c1);
                const uint32_t lf0l = hi_bytes(q.cm), lf0h = pair_bytes<0x0c040c02u>(q.c0, q.cm);
                const uint32_t rt0l = pair_bytes<0x0c050c03u>(q.c1, q.c0), rt0h = c1l;
                const uint32_t lf1l = c0h, lf1h = pair_bytes<0x0c040c02u>(q.c1, q.c0);
                const uint32_t rt1l = pair_bytes<0x0c050c03u>(q.c2, q.c1), rt1h = lo_bytes(q.c2);
                uint32_t b0, k0, b1, k1, b2, k2, b3, k3;
                compass_signs(c0l, lo_bytes(q.u0), lo_bytes(q.d0), lf0l, rt0l, tt, b0, k0);
                compass_signs(c0h, hi_bytes(q.u0), hi_bytes(q.d0), lf0h, rt0h, tt, b1, k1);
                compass_signs(c1l, lo_bytes(q.u1), lo_bytes(q.d1), lf1l, rt1l, tt, b2, k2);
                compass_signs(c1h, hi_bytes(q.u1), hi_bytes(q.d1), lf1h, rt1h, tt, b3, k3);
                uint64_t vm = q.k == 0 ? m_first : (q.k == ndp - 1 ? m_last : 0x8080808080808080ull);
                if (!ok) vm = 0;
                const uint32_t vl = (uint32_t)vm, vh = (uint32_t)(vm >> 32);
                bl = sign_bytes(b0, b1) & vl;
                bh = sign_bytes(b2, b3) & vh;
                dl = sign_bytes(k0, k1) & vl;
                dh = sign_bytes(k2, k3) & vh;
            };
#endif
            // candidates of one item per lane, appended in row-major order
            auto emit = [&](uint32_t bl, uint32_t bh, uint32_t dl, uint32_t dh, int idx0) {
                uint32_t pl = bl | dl, ph = bh | dh;
                const int pc = __popc(pl) + __popc(ph);
                // lane-exclusive prefixes of the per-lane counts (<= 8) by bit ballots
                const uint64_t q0 = __ballot(pc & 1), q1 = __ballot(pc & 2), q2 = __ballot(pc & 4),
                               q3 = __ballot(pc & 8);
                const int tot = __popcll(q0) + 2 * __popcll(q1) + 4 * __popcll(q2) + 8 * __popcll(q3);
                int pos = ncand + mask_rank(q0) + 2 * mask_rank(q1) + 4 * mask_rank(q2) + 8 * mask_rank(q3);
#if ORB_FAST_ABL == 2
                pl = ph = 0;   // ablation: no candidate writes (timing only)
                if (pc) cand[pos] = (uint16_t)idx0;
#endif
                while (pl) {
                    const int bb = __builtin_ctz(pl);
                    pl &= pl - 1;
                    const uint32_t fl = (((bl >> bb) & 1u) << 14) | (((dl >> bb) & 1u) << 15);
                    cand[pos++] = (uint16_t)((uint32_t)(idx0 + kCandColStep * (bb >> 3)) | fl);
                }
                while (ph) {
                    const int bb = __builtin_ctz(ph);
                    ph &= ph - 1;
                    const uint32_t fl = (((bh >> bb) & 1u) << 14) | (((dh >> bb) & 1u) << 15);
                    cand[pos++] = (uint16_t)((uint32_t)(idx0 + kCandColStep * (4 + (bb >> 3))) | fl);
                }
                ncand += tot;
            };
            if (BM && pass == 0) {
                // 1'. the iniThFAST candidates from k_pyr_stream's pre-test bitmap:
                //     lane r = window row r, its bits placed by a funnel shift,
                //     row-major order by a wave prefix sum of the rows' counts.
                //     Their passing directions are decided below (1c, from the
                //     ring), so every candidate is tagged with both.
                const int r = lane;
                const uint64_t lo64 = ((uint64_t)bw[1] << 32) | bw[0];
                uint64_t m64 = bfw.sh ? (lo64 >> bfw.sh) | ((uint64_t)bw[2] << (64 - bfw.sh)) : lo64;
                if (ww < 64) m64 &= (1ull << ww) - 1ull;
                if (r >= wh) m64 = 0;
                const int pc = __popcll(m64);
                const int incl = wave_incl_scan_dpp(pc);
                if (kFastDense && __builtin_amdgcn_readlane(incl, kWave - 1) > a.cand_cap) {
                    dense_from = pass;
                    break;
                }
                int pos = incl - pc;
                const int base = cand_enc(r, 0, ww) | kCandBright | kCandDark;
                while (m64) {
                    const int cb = __builtin_ctzll(m64);
                    m64 &= m64 - 1;
                    cand[pos++] = (uint16_t)(base + kCandColStep * cb);
                }
                ncand = __builtin_amdgcn_readlane(incl, kWave - 1);
            } else {
#if ORB_FAST_EMIT == 1
            // 1a. items holding a candidate go to the wave's item list, one
            //     ballot per round (at iniTh ~20 % of the items, ~3 pixels
            //     each): item index | bright mask << 16 | dark mask << 24, bit
            //     k = item pixel k (byte flags folded by one v_dot4 per half)
            int nlist = 0;
#if ORB_FAST_PIPE
            PreIn pq{};
            if (nitems > 0) pre_load(lane, pq);
#endif
#if ORB_FAST_INC
            // the lane's item (row rr, pair kk) advanced by 64 items a round
            // (a carry instead of a float-reciprocal division per round); lanes
            // past the end take the last item (branch-free, flags cleared)
            int rr = 0, kk = 0, rl = 0, kl = 0, sr = 0, sk = 0;
            if (nitems > 0) {
                rr = div_row(lane, inv_ndp);
                kk = lane - (int)__umul24(rr, ndp);
                rl = div_row(nitems - 1, inv_ndp);
                kl = nitems - 1 - (int)__umul24(rl, ndp);
                sr = div_row(kWave, inv_ndp);
                sk = kWave - (int)__umul24(sr, ndp);
            }
#endif
            for (int base = 0; base < nitems; base += kWave) {
                uint32_t bl, bh, dl, dh;
#if ORB_FAST_PIPE
                const PreIn cq = pq;
                if (base + kWave < nitems) pre_load(base + kWave + lane, pq);
                pre_eval(cq, base + lane < nitems, bl, bh, dl, dh);
#elif ORB_FAST_INC
                {
                    const bool ok = base + lane < nitems;
                    int i0;
                    pretest_rk(ok, ok ? rr : rl, ok ? kk : kl, bl, bh, dl, dh, i0);
                    (void)i0;
                    kk += sk;
                    rr += sr;
                    if (kk >= ndp) { kk -= ndp; ++rr; }
                }
#else
                int i0;
                pretest(base + lane, bl, bh, dl, dh, i0);
#endif
                // flag bytes (bit 7 only) -> 8-bit masks, still scaled by 128
                // (the shift folds into the list entry's)
                const uint32_t mb = __builtin_amdgcn_udot4(bh, 0x80402010u, __builtin_amdgcn_udot4(bl, 0x08040201u, 0u, false),
                                                           false);
                const uint32_t md = __builtin_amdgcn_udot4(dh, 0x80402010u, __builtin_amdgcn_udot4(dl, 0x08040201u, 0u, false),
                                                           false);
                const bool has = (mb | md) != 0u;
                const uint64_t bal = __ballot(has);
                if (has) ilist[nlist + mask_rank(bal)] = (uint32_t)(base + lane) | (mb << 9) | (md << 17);
                nlist += __popcll(bal);
            }
            fast_wave_sync();
            if (kFastDense && 8 * nlist > a.cand_cap) {
                // at most 8 pixels an item: count them exactly only when that
                // bound does not already fit the list
                int np = 0;
                for (int b0 = 0; b0 < nlist; b0 += kWave) {
                    const uint32_t e = b0 + lane < nlist ? ilist[b0 + lane] : 0u;
                    np += __popc(((e >> 16) & 0xffu) | (e >> 24));
                }
                if (wave_sum_dpp(np) > a.cand_cap) {
                    dense_from = pass;
                    break;
                }
            }
            // 1b. the listed items' pixels -> the candidate list, row-major
            //     (items in order, pixels in order within an item)
            for (int b0 = 0; b0 < nlist; b0 += kWave) {
                const uint32_t e = b0 + lane < nlist ? ilist[b0 + lane] : 0u;
                const uint32_t mb = (e >> 16) & 0xffu, md = e >> 24;
                uint32_t m = mb | md;
                const int pc = __popc(m);
                const uint64_t q0 = __ballot(pc & 1), q1 = __ballot(pc & 2), q2 = __ballot(pc & 4),
                               q3 = __ballot(pc & 8);
                const int tot = __popcll(q0) + 2 * __popcll(q1) + 4 * __popcll(q2) + 8 * __popcll(q3);
                int pos = ncand + mask_rank(q0) + 2 * mask_rank(q1) + 4 * mask_rank(q2) + 8 * mask_rank(q3);
                if (m) {
                    const int itm = (int)(e & 0xffffu);
                    const int r = div_row(itm, inv_ndp);
                    const int k = itm - (int)mad24((uint32_t)r, (uint32_t)ndp, 0u);
                    const int idx0 = cand_enc(r, 4 * (j0 + 2 * k) - X0, ww);
                    while (m) {
                        const int bb = __builtin_ctz(m);
                        m &= m - 1;
                        cand[pos++] = (uint16_t)((uint32_t)(idx0 + kCandColStep * bb) | (((mb >> bb) & 1u) << 14) |
                                                 (((md >> bb) & 1u) << 15));
                    }
                }
                ncand += tot;
            }
#elif ORB_FAST_PRE2
            // two items per lane per round: both items' LDS reads and compass
            // chains in flight together
            for (int base = 0; base < nitems; base += 2 * kWave) {
                uint32_t bl, bh, dl, dh, bl2, bh2, dl2, dh2;
                int i0, i2;
                pretest(base + lane, bl, bh, dl, dh, i0);
                pretest(base + kWave + lane, bl2, bh2, dl2, dh2, i2);
                emit(bl, bh, dl, dh, i0);
                emit(bl2, bh2, dl2, dh2, i2);
            }
#else
            for (int base = 0; base < nitems; base += kWave) {
                uint32_t bl, bh, dl, dh;
                int i0;
                pretest(base + lane, bl, bh, dl, dh, i0);
                emit(bl, bh, dl, dh, i0);
            }
#endif
            }
            fast_wave_sync();
            if (pass == 0) FAST_T(1); else FAST_T(5);
#if ORB_FAST_DIAG
            // 1c. a second necessary condition, on the candidates only: a 9-arc
            //     also holds two ring-adjacent diagonal pixels (ring positions
            //     2, 6, 10, 14: one of each opposite pair), so a direction
            //     survives only if min(max(x2,x10), max(x6,x14)) > v + t
            //     (bright) / max(min(x2,x10), min(x6,x14)) < v - t (dark).  A
            //     dropped direction has strength - 1 < t: its score acts as 0
            //     at t, like a pixel the compass test dropped.  The list is
            //     compacted in place, in order (~40 % of the candidates go)
            {
                int n2 = 0;
                for (int q0 = 0; q0 < ncand; q0 += kWave) {
                    const int q = q0 + lane;
                    uint32_t e2 = 0;
                    bool keep = false;
                    if (q < ncand) {
                        const int e = cand[q];
                        int r, cc;
                        cand_dec(e & kCandIdx, inv_ww, ww, r, cc);
                        const uint8_t* p = R + (RP ? (r + 3) * rstride + cc + 3
                                                   : (int)mad24((uint32_t)(r + 3), (uint32_t)rstride, (uint32_t)(cc + 3)));
                        const int v = p[0];
                        const int x2 = p[2 * rstride + 2], x6 = p[-2 * rstride + 2];
                        const int x10 = p[-2 * rstride - 2], x14 = p[2 * rstride - 2];
                        bool bo = (e & kCandBright) && min(max(x2, x10), max(x6, x14)) > v + t;
                        bool dk = (e & kCandDark) && max(min(x2, x10), min(x6, x14)) < v - t;
                        if (BM && pass == 0) {
                            // bitmap candidates: the compass directions (ring positions 0,
                            // 4, 8, 12) here, as the pre-test would have tagged them
                            const int xu = p[-3 * rstride], xd = p[3 * rstride], xl = p[-3], xr = p[3];
                            bo = bo && min(max(xu, xd), max(xl, xr)) > v + t;
                            dk = dk && max(min(xu, xd), min(xl, xr)) < v - t;
                        }
                        keep = bo || dk;
                        e2 = (uint32_t)(e & kCandIdx) | (bo ? (uint32_t)kCandBright : 0u) | (dk ? (uint32_t)kCandDark : 0u);
                    }
                    const uint64_t m = __ballot(keep);
                    if (keep) cand[n2 + mask_rank(m)] = (uint16_t)e2;
                    n2 += __popcll(m);
                }
                ncand = n2;
                fast_wave_sync();
            }
#endif
#if ORB_FAST_ILIST_IN_MAP
            // the map zeroed here, over the item list, in each pass: the minThFAST
            // pass rescores every pixel the first pass scored (its candidates are
            // a superset), so nothing of the first pass's map is needed
            for (int i = lane; i < (npad + 15) / 16; i += kWave) ((uint4*)sc)[i] = make_uint4(0u, 0u, 0u, 0u);
            fast_wave_sync();
#endif
            // 2. FAST score of the candidates (the dark direction too for the rare
            //    pixels passing both pre-tests).  ORB_FAST_KEEPLIST: the list
            //    keeps only scores >= max(t, 1) -- the NMS at t keeps nothing
            //    else, and the map holds every score for the neighbour reads --
            //    compacted in place, in order (~1/3 of the candidates remain)
#if ORB_FAST_KEEPLIST
            {
                const int tk = max(t, 1);
                int n3 = 0;
                for (int q0 = 0; q0 < ncand; q0 += kWave) {
                    const int q = q0 + lane;
                    bool keep = false;
                    int e = 0;
                    if (q < ncand) {
                        e = cand[q];
                        int r, cc;
                        cand_dec(e & kCandIdx, inv_ww, ww, r, cc);
                        int v, x[16];
                        fast_ring<RP>(R, rstride, r + 3, cc + 3, v, x);
                        int sv = fast_dir_score(x, v, (e & kCandBright) ? 0 : 1);
                        if ((e & kCandBright) && (e & kCandDark)) sv = max(sv, fast_dir_score(x, v, 1));
                        sv = max(sv, 0);
                        sc[mad24((uint32_t)(r + 1), (uint32_t)sp, (uint32_t)(cc + 1))] = (uint8_t)sv;
                        keep = sv >= tk;
                    }
                    const uint64_t m = __ballot(keep);
                    if (keep) cand[n3 + mask_rank(m)] = (uint16_t)e;
                    n3 += __popcll(m);
                }
                ncand = n3;
            }
#else
            for (int q = lane; q < ncand; q += kWave) {
                const int e = cand[q], i = e & kCandIdx;
                int r, cc;
                cand_dec(i, inv_ww, ww, r, cc);
#if ORB_FAST_ABL == 1
                int sv = (e * 37) & 63;   // ablation: no ring reads / arc scores (timing only)
#else
                int v, x[16];
                fast_ring<RP>(R, rstride, r + 3, cc + 3, v, x);
                int sv = fast_dir_score(x, v, (e & kCandBright) ? 0 : 1);
                if ((e & kCandBright) && (e & kCandDark)) sv = max(sv, fast_dir_score(x, v, 1));
#endif
                sc[mad24((uint32_t)(r + 1), (uint32_t)sp, (uint32_t)(cc + 1))] = (uint8_t)max(sv, 0);
            }
#endif
            fast_wave_sync();
            if (pass == 0) FAST_T(2); else FAST_T(6);
            // 3. NMS at this pass's threshold.  ORB_FAST_FUSED_OUT: the
            //    survivors go out in the same loop (the candidate list is
            //    row-major, so ballot order is the reference's order; a pass
            //    with no survivor writes nothing, so writing speculatively in
            //    the iniTh pass is exact); otherwise keep the ballots for step 4
            cnt = 0;
            const int nchunk = (ncand + kWave - 1) / kWave;
#if ORB_FAST_FUSED_OUT
            uint32_t* outp = a.cell_keys + (long long)f * a.slot_total + cur.slot_off;
#endif
            for (int k = 0; k < nchunk; ++k) {
                const int q = k * kWave + lane;
                bool keep = false;
#if ORB_FAST_FUSED_OUT
                uint32_t key = 0;
                if (q < ncand) {
                    int r, cc;
                    cand_dec(cand[q] & kCandIdx, inv_ww, ww, r, cc);
                    int sv;
                    keep = nms_keep(sc, sp, r, cc, t, sv);
                    // key coordinates relative to minBorder (ORBextractor.cc:865-866 add j*wCell, i*hCell)
                    key = (uint32_t)(cur.x0 + cc + 3 - (kEdge - 3)) | ((uint32_t)(cur.y0 + r + 3 - (kEdge - 3)) << 12) |
                          ((uint32_t)sv << 24);
                }
                const uint64_t m = __ballot(keep);
                if (keep) {
                    const int pos = cnt + mask_rank(m);
                    if (pos < cur.cap) outp[pos] = key;
                }
#else
                if (q < ncand) {
                    int r, cc, sv;
                    cand_dec(cand[q] & kCandIdx, inv_ww, ww, r, cc);
                    keep = nms_keep(sc, sp, r, cc, t, sv);
                }
                const uint64_t m = __ballot(keep);
                if (lane == 0) kmask[k] = m;
#endif
                cnt += __popcll(m);
            }
            fast_wave_sync();
            if (pass == 0) FAST_T(3); else FAST_T(7);
            if (cnt > 0) break;
        }
        if (kFastDense && dense_from >= 0) cnt = dense_cell(dense_from);
#if ORB_FAST_FUSED_OUT
        const int written = cnt;
#else
        // 4. survivors of the deciding pass, row-major
        uint32_t* out = a.cell_keys + (long long)f * a.slot_total + cur.slot_off;
        int written = 0;
        if (cnt > 0) {
            const int nchunk = (ncand + kWave - 1) / kWave;
            for (int k = 0; k < nchunk; ++k) {
                const bool keep = (kmask[k] >> lane) & 1;
                const uint64_t m = __ballot(keep);
                if (keep) {
                    const int pos = written + mask_rank(m);
                    if (pos < cur.cap) {
                        int r, cc;
                        cand_dec(cand[k * kWave + lane] & kCandIdx, inv_ww, ww, r, cc);
                        // key coordinates relative to minBorder (ORBextractor.cc:865-866 add j*wCell, i*hCell)
                        const uint32_t x = (uint32_t)(cur.x0 + cc + 3 - (kEdge - 3));
                        const uint32_t y = (uint32_t)(cur.y0 + r + 3 - (kEdge - 3));
                        out[pos] = x | (y << 12) | ((uint32_t)sc[(r + 1) * sp + cc + 1] << 24);
                    }
                }
                written += __popcll(m);
            }
        }
#endif
        if (lane == 0) a.cell_count[it] = min(written, cur.cap);
#if ORB_FAST_RESET
        // back to an all-zero map: the deciding pass's candidates cover every
        // entry either pass wrote (a pixel passing the pre-test at iniTh
        // passes it at minThFAST < iniThFAST)
        for (int q = lane; q < ncand; q += kWave) {
            int r, cc;
            cand_dec(cand[q] & kCandIdx, inv_ww, ww, r, cc);
            sc[mad24((uint32_t)(r + 1), (uint32_t)sp, (uint32_t)(cc + 1))] = 0;
        }
#endif
        fast_wave_sync();
        FAST_T(9);
    };
#if ORB_FAST_RESET
    for (int i = lane; i < a.win_max / 4; i += kWave) ((uint32_t*)sc)[i] = 0u;
#endif
    for (int it = it0; it < it_end; it += step) {
        // land the prefetched ROI in LDS, then prefetch the next cell's ROI
        land(v, rf);
        const CellDev cur = c;
        const RoiFetch rcur = rf;
        const BmFetch bcur = bfc;
        uint32_t bw[3] = {bmw[0], bmw[1], bmw[2]};
        if (it + step < it_end) {
            c = cn;
            rf = fetch_of(c, it + step);
            roi_issue<PDW, NV>(rf, v);
            if (BM) {
                bfc = bm_of(c);
                bm_issue(bfc, bmw);
            }
        }
        if (it + 2 * step < it_end) cn = cell_at(it + 2 * step);
        process(cur, rcur, bcur, bw, it);
    }
#ifdef ORB_FAST_TIMING
    if (lane == 0) {
        const unsigned long long tv[11] = {t0, t1, t2, t3, __builtin_amdgcn_s_memtime() - t_start, t5, t6, t7,
                                           1ull, t9, t10};
#pragma unroll
        for (int k = 0; k < 11; ++k)
            atomicAdd(&g_fast_t[(bunit * 4 + wv + bframe * 61) & 1023][k], tv[k]);
    }
#endif
}

#ifdef ORB_FAST_TIMING
extern "C" int orbx_debug_fast_timing(unsigned long long* out, int reset) {
    static unsigned long long h[1024][16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_fast_t), sizeof(h)) != hipSuccess) return -4;
    for (int k = 0; k < 16; ++k) {
        out[k] = 0;
        for (int i = 0; i < 1024; ++i) out[k] += h[i][k];
    }
    if (reset) {
        static unsigned long long z[1024][16];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_fast_t), z, sizeof(z)) != hipSuccess) return -4;
    }
    return 0;
}
#endif

// ---------------------------------------------------------------------------
// k_quadtree: ORBextractor::DistributeOctTree (ORBextractor.cc:555-779) for
// one (frame, level) per workgroup.
//
// The std::list becomes an array in list order rebuilt by scans.  One step
// divides a set of nodes given in processing order; the rebuilt list is the
// children blocks (n4,n3,n2,n1, non-empty only) in REVERSE processing order
// followed by the undivided nodes in their old order -- exactly what the
// reference's push_front + erase produce (:633-679, :703-744).  Children with
// >1 key are queued (n1..n4, processing order) like vSizeAndPointerToNode.
// Outer passes divide every node that still holds >1 key; the last rounds
// (:689-754) sort the queue with the libstdc++ std::sort port and divide from
// the largest down until the list holds N nodes.  Keys never move: each key
// carries the list index of its node, remapped after every step.  A node keeps
// its max-response key, the first in vToDistributeKeys order on ties
// (:757-776).
// ---------------------------------------------------------------------------
struct QtArgs {
    const LevelDev* lv;
    const int* cell_count;
    const uint32_t* cell_keys;
    uint32_t* key_scr;
    int* knode;
    uint8_t* kq;
    int ncells_total, slot_total;
    uint32_t* qt_key;   // [B][out_total]
    int* qt_n;          // [B][L]
    int out_total, L;
    int lds_bytes;          // dynamic LDS of the launch
    uint8_t* gscr;          // k_quadtree<true>: [B][L] node arrays of levels beyond the LDS
    long long gscr_stride;
    int* qt_ovf;            // [B][L]: k_quadtree_w left the level to k_quadtree (more keys than kcap)
    int fixup;              // k_quadtree: only the levels whose qt_ovf is set
    int qw_nc, qw_kcap;     // k_quadtree_w: node capacity of the LDS layout; key capacity (<= 64 KPL)
};

// Bytes of a level's node arrays (NC = out_cap + 8 nodes: the list never
// grows past N + 3 or 4 nIni, see qt_divide) and cell offsets; the layout
// k_quadtree carves.
__host__ __device__ inline size_t qt_scratch_bytes(int NC, int ncells) {
    auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
    const size_t n = (size_t)NC;
    size_t b = al((size_t)(ncells + 1) * 4);
    b += 2 * al(n * 8) + 2 * al(n * 4) + 2 * al(n) + 2 * al(n * 16);
    b += 7 * al(n * 4) + al(n * sizeof(SortRec)) + al(80 * sizeof(SortFrame)) + 2 * al(64);
    return b;
}

// double-buffered arrays are picked by a select, never by a dynamic index:
// an indexed pointer array would live in scratch and every access through it
// would become a flat memory op
template <class T> __device__ __forceinline__ T* qsel(T* const (&arr)[2], int i) { return i ? arr[1] : arr[0]; }

struct QtLds {
    int* off;
    short4* rect[2];
    int* cnt[2];
    uint8_t* nomore[2];
    int* ccnt;      // 4 per node
    int* newpos;    // 4 per node
    int* keep;      // new index of an undivided node
    int* div;       // node divides in this step
    int* ord;       // processing order (node indices)
    int* rne;       // per rank: #non-empty children (scanned)
    int* rgt;       // per rank: #children with >1 key (scanned)
    int* nd;        // per node: undivided (scanned)
    int* expand;    // queue of list indices (processing order)
    SortRec* srt;
    SortFrame* stk; // introsort stack
    int* tmp;       // scan scratch
    int* misc;
};

__device__ __forceinline__ int quadrant(uint32_t key, short4 r) {
    const int x = key & 0xfff, y = (key >> 12) & 0xfff;
    const int hx = (int)ceilf((float)(r.z - r.x) / 2), hy = (int)ceilf((float)(r.w - r.y) / 2);
    const bool left = x < r.x + hx, top = y < r.y + hy;
    return left ? (top ? 0 : 2) : (top ? 1 : 3);
}

// ExtractorNode::DivideNode child boundaries (ORBextractor.cc:480-508).
__device__ __forceinline__ short4 child_rect(short4 r, int q) {
    const int hx = (int)ceilf((float)(r.z - r.x) / 2), hy = (int)ceilf((float)(r.w - r.y) / 2);
    const short mx = (short)(r.x + hx), my = (short)(r.y + hy);
    switch (q) {
        case 0: return make_short4(r.x, r.y, mx, my);
        case 1: return make_short4(mx, r.y, r.z, my);
        case 2: return make_short4(r.x, my, mx, r.w);
        default: return make_short4(mx, my, r.z, r.w);
    }
}

// One __introsort_loop step on [f, l) by a whole wave: partition_ranks
// (orb_math.h) with the L / R lists built by ballots.
#ifndef ORB_QT_KCELL
#define ORB_QT_KCELL 0   // 1: the gather finds a key's cell by a table written per cell instead of a binary search (same-box A/B: quadtree 86-88 vs 83-87 us, no gain)
#endif
#ifndef ORB_QT_OFFLOAD4
#define ORB_QT_OFFLOAD4 1   // k_quadtree's cell-count loads 4 a thread in flight
#endif
#ifndef ORB_SORT_LEAF16
#define ORB_SORT_LEAF16 0   // 1: a leaf's records read at once (same-box A/B: no gain, profiles/r06/README.md)
#endif
#ifndef ORB_SORT_REGMED
#define ORB_SORT_REGMED 0   // 1: median of three from one round of reads by lanes 0-3 (no gain measured)
#endif
__device__ __forceinline__ SortRec rec_lane(const SortRec& r, int l) {
    return SortRec{__builtin_amdgcn_readlane(r.cnt, l), __builtin_amdgcn_readlane(r.x0, l),
                   __builtin_amdgcn_readlane(r.pos, l)};
}
__device__ int wave_partition(SortRec* a, int f, int l, int* Lp, int* Rp) {
    const int lane = lane_id();
#if ORB_SORT_REGMED
    // median_to_first_(a + f, a + f + 1, a + mid, a + l - 1) with the four
    // records read at once (lanes 0-3) and the choice made in registers:
    // ranges here hold > 16 records, so f + 1 < mid < l - 1
    SortRec pv;
    {
        const int mid = f + (l - f) / 2;
        const int src = lane == 1 ? f + 1 : (lane == 2 ? mid : (lane == 3 ? l - 1 : f));
        const SortRec mine = a[src];
        const SortRec r0 = rec_lane(mine, 0), A = rec_lane(mine, 1), B = rec_lane(mine, 2), C = rec_lane(mine, 3);
        int mp;   // the position median_to_first_ swaps with f
        if (node_less(A, B)) {
            if (node_less(B, C)) mp = mid;
            else if (node_less(A, C)) mp = l - 1;
            else mp = f + 1;
        } else if (node_less(A, C)) mp = f + 1;
        else if (node_less(B, C)) mp = l - 1;
        else mp = mid;
        pv = mp == mid ? B : (mp == f + 1 ? A : C);
        fast_wave_sync();   // every lane has read before lane 0 writes
        if (lane == 0) {
            a[f] = pv;
            a[mp] = r0;
        }
        fast_wave_sync();
    }
#else
    if (lane == 0) median_to_first_(a + f, a + f + 1, a + f + (l - f) / 2, a + l - 1);
    fast_wave_sync();
    const SortRec pv = a[f];
#endif
    int cl = 0, cr = 0;
    for (int base = f + 1; base < l; base += kWave) {
        const int p = base + lane;
        bool ge = false, le = false;
        if (p < l) {
            const SortRec x = a[p];
            ge = !node_less(x, pv);
            le = !node_less(pv, x);
        }
        const uint64_t mg = __ballot(ge), ml = __ballot(le);
        if (ge) Lp[f + cl + mask_rank(mg)] = p;
        if (le) Rp[f + cr + mask_rank(ml)] = p;
        cl += __popcll(mg);
        cr += __popcll(ml);
    }
    fast_wave_sync();
    const int kmax = min(cl, cr + 1);
    int ks = 0;
    for (int base = 0; base < kmax; base += kWave) {
        const int k = base + lane;
        bool pr = false;
        if (k < kmax) pr = Lp[f + k] < (k < cr ? Rp[f + cr - 1 - k] : f);
        ks += __popcll(__ballot(pr));            // the predicate holds on a prefix
    }
    const int lk = ks < cl ? Lp[f + ks] : 0x7fffffff;
    const int rk = ks == 0 ? l : (ks - 1 < cr ? Rp[f + cr - ks] : f);
    const int cut = min(lk, rk);
    for (int k = lane; k < ks; k += kWave) {
        const int i = Lp[f + k], j = Rp[f + cr - 1 - k];
        const SortRec x = a[i], y = a[j];
        a[i] = y;
        a[j] = x;
    }
    fast_wave_sync();
    return cut;
}

// std::sort(a, a + m) under compareNodes by the whole workgroup: levels of
// disjoint ranges partitioned by one wave each, then every leaf (<= 16
// records) put in stable order by 16 lanes, each placing one record at its
// rank -- the permutation the final insertion sort gives (std_sort_levels,
// orb_math.h, states it sequentially and is checked against std::sort on the
// host).  Where the reference would heap-sort (depth limit),
// the original array is restored and sorted by the sequential port.
__device__ void block_std_sort(SortRec* a, int m, SortRec* backup, int* Lp, int* Rp, SortFrame* qa, SortFrame* qb,
                               int* leaves, int* ctl, SortFrame* stk) {
    const int tid = threadIdx.x, T = blockDim.x, lane = lane_id(), wv = wave_id(), nw = T / kWave;
    if (m <= 1) return;
    for (int i = tid; i < m; i += T) backup[i] = a[i];
    if (tid == 0) {
        ctl[0] = 0; ctl[1] = 0; ctl[2] = 0; ctl[3] = 0;
        if (m > 16) { qa[0] = SortFrame{0, m, ilg(m) * 2}; ctl[0] = 1; }
        else { leaves[0] = m; ctl[3] = 1; }                // leaf = (f << 16) | l
    }
    __syncthreads();
    while (true) {
        const int na = ctl[0];
        if (na == 0 || ctl[2]) break;
        for (int r = wv; r < na; r += nw) {
            const SortFrame fr = qa[r];
            if (fr.depth == 0) {
                if (lane == 0) ctl[2] = 1;
                continue;
            }
            const int cut = wave_partition(a, fr.f, fr.l, Lp, Rp);
            if (lane == 0) {
                const SortFrame kids[2] = {SortFrame{fr.f, cut, fr.depth - 1}, SortFrame{cut, fr.l, fr.depth - 1}};
                for (int c = 0; c < 2; ++c) {
                    if (kids[c].l - kids[c].f > 16) qb[atomicAdd(&ctl[1], 1)] = kids[c];
                    else leaves[atomicAdd(&ctl[3], 1)] = (kids[c].f << 16) | kids[c].l;
                }
            }
        }
        __syncthreads();
        if (tid == 0) { ctl[0] = ctl[1]; ctl[1] = 0; }
        SortFrame* t = qa; qa = qb; qb = t;
        __syncthreads();
    }
    if (ctl[2]) {
        for (int i = tid; i < m; i += T) a[i] = backup[i];
        __syncthreads();
        if (tid == 0) std_sort(a, m, stk);
        __syncthreads();
        return;
    }
    // leaves (<= 16 records, never crossed by the final insertion pass):
    // insertion sort under a strict weak order is the stable sort, so record
    // j of a leaf goes to #{less} + #{equivalent before j} -- 16 lanes per
    // leaf, four leaves per wave, instead of a serial insertion sort by one
    // thread per leaf (~20 % of the sort)
    const int nleaf = ctl[3];
    for (int L0 = wv * 4; L0 < nleaf; L0 += nw * 4) {
        const int leaf = L0 + (lane >> 4), sub = lane & 15;
        int f = 0, len = 0, rank = 0;
        SortRec x{};
        if (leaf < nleaf) {
            f = leaves[leaf] >> 16;
            len = (leaves[leaf] & 0xffff) - f;
        }
        if (sub < len) {
            x = a[f + sub];
#if ORB_SORT_LEAF16
            // the leaf's <= 16 records read at once (16 reads in flight, not a
            // chain of len dependent round trips)
            SortRec y[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) y[j] = a[f + min(j, len - 1)];
#pragma unroll
            for (int j = 0; j < 16; ++j)
                rank += j < len && (node_less(y[j], x) || (j < sub && !node_less(x, y[j])));
#else
            for (int j = 0; j < len; ++j) {
                const SortRec y = a[f + j];
                rank += node_less(y, x) || (j < sub && !node_less(x, y));
            }
#endif
        }
        fast_wave_sync();
        if (sub < len) a[f + rank] = x;
        fast_wave_sync();
    }
    __syncthreads();
}

// orbx_debug_sort: block_std_sort -- k_quadtree's device std::sort under
// compareNodes (ORBextractor.cc:538-553, :700) -- on many arrays, one
// workgroup each, so the exact permutation can be compared with the host's
// std::sort on adversarial inputs (tests/test_gpu_sort.py).  LDS: the array
// and its backup, the partition lists, the range queues and leaves, ctl, the
// sequential port's stack.
constexpr int kDbgSortMax = 4000;
__host__ __device__ inline size_t dbg_sort_lds(int m) {
    auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
    return 2 * al(m * sizeof(SortRec)) + 2 * al(m * sizeof(int)) + 2 * al((m / 17 + 2) * sizeof(SortFrame)) +
           al((m + 2) * sizeof(int)) + al(4 * sizeof(int)) + al(80 * sizeof(SortFrame));
}
__global__ __launch_bounds__(256) void k_debug_sort(const int* __restrict__ off, const int* __restrict__ cnt,
                                                    const int* __restrict__ x0, int* __restrict__ perm,
                                                    int* __restrict__ fallback) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int o = off[blockIdx.x], m = off[blockIdx.x + 1] - o;
    uint8_t* p = smem;
    auto take = [&](size_t bytes) { uint8_t* q = p; p += (bytes + 15) & ~size_t(15); return q; };
    SortRec* a = (SortRec*)take(m * sizeof(SortRec));
    SortRec* backup = (SortRec*)take(m * sizeof(SortRec));
    int* Lp = (int*)take(m * sizeof(int));
    int* Rp = (int*)take(m * sizeof(int));
    SortFrame* qa = (SortFrame*)take((m / 17 + 2) * sizeof(SortFrame));
    SortFrame* qb = (SortFrame*)take((m / 17 + 2) * sizeof(SortFrame));
    int* leaves = (int*)take((m + 2) * sizeof(int));
    int* ctl = (int*)take(4 * sizeof(int));
    SortFrame* stk = (SortFrame*)take(80 * sizeof(SortFrame));
    for (int i = threadIdx.x; i < m; i += blockDim.x) a[i] = SortRec{cnt[o + i], x0[o + i], i};
    if (threadIdx.x == 0) ctl[2] = 0;
    __syncthreads();
    block_std_sort(a, m, backup, Lp, Rp, qa, qb, leaves, ctl, stk);
    for (int i = threadIdx.x; i < m; i += blockDim.x) perm[o + i] = a[i].pos;
    if (threadIdx.x == 0) fallback[blockIdx.x] = ctl[2];
}

#ifndef ORB_QT_B
#define ORB_QT_B 4
#endif
constexpr int kQtB = ORB_QT_B;   // keys per thread per round of the quadtree's key passes

// Divide s.ord[0..m) (ccnt/kq already computed for them, s.div set for every
// node); rebuild the list into buffer cur^1; remap the keys.  Returns the new
// size; *nexp receives the queue length.
__device__ int qt_divide(QtLds& s, int& cur, int size, int m, const int K, int* knode, const uint8_t* kq,
                         int* nexp) {
    const int tid = threadIdx.x, T = blockDim.x;
    for (int r = tid; r < m; r += T) {
        const int i = s.ord[r];
        int ne = 0, gt = 0;
        for (int q = 0; q < 4; ++q) { ne += s.ccnt[4 * i + q] > 0; gt += s.ccnt[4 * i + q] > 1; }
        s.rne[r] = ne;
        s.rgt[r] = gt;
    }
    for (int i = tid; i < size; i += T) s.nd[i] = s.div[i] ? 0 : 1;
    __syncthreads();
    int tot3[3];
    block_excl_scan3(s.rne, m, s.rgt, m, s.nd, size, s.tmp, tot3);
    const int totNE = tot3[0], totGT = tot3[1];
    const int nx = cur ^ 1;
    const short4* R = qsel(s.rect, cur);
    const int* C = qsel(s.cnt, cur);
    for (int r = tid; r < m; r += T) {
        const int i = s.ord[r];
        int ne = 0;
        for (int q = 0; q < 4; ++q) ne += s.ccnt[4 * i + q] > 0;
        const int start = totNE - s.rne[r] - ne;   // reverse processing order
        int w = 0;
        for (int q = 3; q >= 0; --q) {
            const int c = s.ccnt[4 * i + q];
            if (c > 0) {
                const int np = start + w++;
                s.newpos[4 * i + q] = np;
                qsel(s.rect, nx)[np] = child_rect(R[i], q);
                qsel(s.cnt, nx)[np] = c;
                qsel(s.nomore, nx)[np] = c == 1;
            }
        }
        int e = s.rgt[r];
        for (int q = 0; q < 4; ++q)
            if (s.ccnt[4 * i + q] > 1) s.expand[e++] = s.newpos[4 * i + q];
    }
    for (int i = tid; i < size; i += T) {
        if (s.div[i]) continue;
        const int np = totNE + s.nd[i];
        s.keep[i] = np;
        qsel(s.rect, nx)[np] = R[i];
        qsel(s.cnt, nx)[np] = C[i];
        qsel(s.nomore, nx)[np] = qsel(s.nomore, cur)[i];
    }
    __syncthreads();
    {
        int* __restrict__ kn = knode;
        const uint8_t* __restrict__ kqi = kq;
        for (int k0 = tid; k0 < K; k0 += kQtB * T) {
            int n[kQtB], q[kQtB];
#pragma unroll
            for (int b = 0; b < kQtB; ++b) {
                const int k = k0 + b * T;
                n[b] = k < K ? kn[k] : 0;
                q[b] = k < K ? kqi[k] : 0;
            }
#pragma unroll
            for (int b = 0; b < kQtB; ++b) {
                const int k = k0 + b * T;
                if (k < K) kn[k] = s.div[n[b]] ? s.newpos[4 * n[b] + q[b]] : s.keep[n[b]];
            }
        }
    }
    __syncthreads();
    cur = nx;
    *nexp = totGT;
    return totNE + (size - m);
}

// Count keys per child quadrant for every node with s.div set.
__device__ void qt_count(QtLds& s, int cur, int size, const int K, const uint32_t* keys, const int* knode,
                         uint8_t* kq) {
    const int tid = threadIdx.x, T = blockDim.x;
    for (int i = tid; i < 4 * size; i += T) s.ccnt[i] = 0;
    __syncthreads();
    const short4* R = qsel(s.rect, cur);
    // kQtB keys per thread per round, every load of the round in flight at once
    const int* __restrict__ kn = knode;
    const uint32_t* __restrict__ ks = keys;
    uint8_t* __restrict__ kqo = kq;
    for (int k0 = tid; k0 < K; k0 += kQtB * T) {
        int n[kQtB];
        uint32_t key[kQtB];
#pragma unroll
        for (int b = 0; b < kQtB; ++b) {
            const int k = k0 + b * T;
            n[b] = k < K ? kn[k] : 0;
            key[b] = k < K ? ks[k] : 0u;
        }
#pragma unroll
        for (int b = 0; b < kQtB; ++b) {
            const int k = k0 + b * T;
            if (k < K && s.div[n[b]]) {
                const int q = quadrant(key[b], R[n[b]]);
                kqo[k] = (uint8_t)q;
                atomicAdd(&s.ccnt[4 * n[b] + q], 1);
            }
        }
    }
    __syncthreads();
}

#ifdef ORB_QT_TIMING
// phase profile of k_quadtree (tools/fast_phases.py --quadtree): per level,
// shader cycles per phase summed over blocks, the longest block, pass counts
__device__ unsigned long long g_qt_t[16][16];
#define QT_T(k)                                                              \
    do {                                                                     \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();          \
        if (tid == 0) atomicAdd(&g_qt_t[l][k], t_ - qt_last);                \
        qt_last = t_;                                                        \
    } while (0)
extern "C" int orbx_debug_qt_timing(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_qt_t), sizeof(g_qt_t)) != hipSuccess) return -4;
    if (reset) {
        static unsigned long long z[16][16];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_qt_t), z, sizeof(z)) != hipSuccess) return -4;
    }
    return 0;
}
#else
#define QT_T(k) do { } while (0)
#endif

// GS: a level whose node arrays exceed the launch's LDS (N beyond ~1,600 a
// level: Tracking's 5 x nFeatures initialization extractor) keeps them in a
// global scratch slice instead; the instantiation is only launched when a
// plan has such a level, so the LDS form keeps its ds_* instructions.
#ifndef ORB_QT_THREADS
#define ORB_QT_THREADS 256   // threads of a k_quadtree block (one (frame, level) tree)
#endif
template <bool GS>
__global__ __launch_bounds__(ORB_QT_THREADS) void k_quadtree(QtArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
#if ORB_QT_LEVEL_MAJOR
    // grid (frames, levels): every frame's level 0 (the largest trees) dispatches first
    const int l = blockIdx.y, f = blockIdx.x, tid = threadIdx.x, T = blockDim.x;
#else
    const int l = blockIdx.x, f = blockIdx.y, tid = threadIdx.x, T = blockDim.x;
#endif
    if (a.fixup && !a.qt_ovf[f * a.L + l]) return;   // k_quadtree_w distributed this level
    const LevelDev lv = a.lv[l];
    const int NC = lv.out_cap + 8;
#ifdef ORB_QT_TIMING
    const unsigned long long qt_t0 = __builtin_amdgcn_s_memtime();
    unsigned long long qt_last = qt_t0;
    int qt_outer = 0, qt_lastr = 0;
#endif
    QtLds s;
    {
        uint8_t* p = smem;
        if (GS && qt_scratch_bytes(NC, lv.ncells) > (size_t)a.lds_bytes)
            p = a.gscr + ((long long)f * a.L + l) * a.gscr_stride;
        auto take = [&](size_t bytes) { uint8_t* q = p; p += (bytes + 15) & ~size_t(15); return q; };
        s.off = (int*)take((lv.ncells + 1) * sizeof(int));
        s.rect[0] = (short4*)take(NC * sizeof(short4));
        s.rect[1] = (short4*)take(NC * sizeof(short4));
        s.cnt[0] = (int*)take(NC * sizeof(int));
        s.cnt[1] = (int*)take(NC * sizeof(int));
        s.nomore[0] = take(NC);
        s.nomore[1] = take(NC);
        s.ccnt = (int*)take(4 * NC * sizeof(int));
        s.newpos = (int*)take(4 * NC * sizeof(int));
        s.keep = (int*)take(NC * sizeof(int));
        s.div = (int*)take(NC * sizeof(int));
        s.ord = (int*)take(NC * sizeof(int));
        s.rne = (int*)take(NC * sizeof(int));
        s.rgt = (int*)take(NC * sizeof(int));
        s.nd = (int*)take(NC * sizeof(int));
        s.expand = (int*)take(NC * sizeof(int));
        s.srt = (SortRec*)take(NC * sizeof(SortRec));
        s.stk = (SortFrame*)take(80 * sizeof(SortFrame));
        s.tmp = (int*)take(16 * sizeof(int));
        s.misc = (int*)take(16 * sizeof(int));
    }
    const int* ccount = a.cell_count + (long long)f * a.ncells_total + lv.cell_base;
    const uint32_t* cslots = a.cell_keys + (long long)f * a.slot_total + lv.slot_base;
    const long long kb = (long long)f * a.slot_total + lv.slot_base;
    uint32_t* keys = a.key_scr + kb;
    int* knode = a.knode + kb;
    uint8_t* kq = a.kq + kb;
    uint32_t* out = a.qt_key + (long long)f * a.out_total + lv.out_base;

    // 1. vToDistributeKeys: cells in (row, col) order, row-major inside a cell (:805-872)
#if ORB_QT_OFFLOAD4
    // the cell counts with 4 loads a thread in flight (a load-store loop
    // waited on each load: three serial round trips to L2 at 700 cells)
    for (int i0 = tid; i0 < lv.ncells; i0 += 4 * T) {
        int v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = i0 + u * T < lv.ncells ? ccount[i0 + u * T] : 0;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i0 + u * T < lv.ncells) s.off[i0 + u * T] = v[u];
    }
#else
    for (int i = tid; i < lv.ncells; i += T) s.off[i] = ccount[i];
#endif
    __syncthreads();
    const int K = block_excl_scan(s.off, lv.ncells, s.tmp);
    const int cap = lv.ncells ? lv.slot_total / lv.ncells : 0;
    if (K == 0) {
        QT_T(0);
        if (tid == 0) a.qt_n[f * a.L + l] = 0;
        return;
    }
    // 1+2. keys in vToDistributeKeys order, each with its initial node's bin
    // (:559-601, vpIniNodes[kp.pt.x / hX]) -- one flat pass: key k's cell by a
    // binary search of the cell offsets in LDS, kQtB keys per thread in flight
    const int nIni = lv.nIni;
    int* bcnt = s.rne;
    int* bpos = s.rgt;
    for (int i = tid; i < nIni; i += T) bcnt[i] = 0;
    __syncthreads();
    {
        const uint32_t* __restrict__ src = cslots;
        uint32_t* __restrict__ dst = keys;
        int* __restrict__ kn = knode;
        const int nc = lv.ncells;
        // key k's cell: written per cell into the (still free) ccnt / newpos
        // bytes, one LDS read a key instead of a ~10-step binary search of the
        // offsets (levels whose keys do not fit those bytes keep the search)
        uint16_t* const kcell = (uint16_t*)s.ccnt;
        const bool direct = ORB_QT_KCELL && K <= 16 * NC && nc <= 65536;
        if (direct) {
            for (int c = tid; c < nc; c += T) {
                const int e = c + 1 < nc ? s.off[c + 1] : K;
                for (int j = s.off[c]; j < e; ++j) kcell[j] = (uint16_t)c;
            }
            __syncthreads();
        }
        for (int k0 = tid; k0 < K; k0 += kQtB * T) {
            int c[kQtB];
#pragma unroll
            for (int q = 0; q < kQtB; ++q) {
                const int k = min(k0 + q * T, K - 1);
                if (direct) {
                    c[q] = kcell[k];
                    continue;
                }
                int lo = 0, hi = nc;                   // off[lo] <= k < off[hi] (off[nc] = K)
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (s.off[mid] <= k) lo = mid;
                    else hi = mid;
                }
                c[q] = lo;
            }
            uint32_t v[kQtB];
#pragma unroll
            for (int q = 0; q < kQtB; ++q) {
                const int k = min(k0 + q * T, K - 1);
                v[q] = src[c[q] * cap + (k - s.off[c[q]])];
            }
#pragma unroll
            for (int q = 0; q < kQtB; ++q) {
                const int k = k0 + q * T;
                if (k < K) {
                    dst[k] = v[q];
                    const int bn = (int)((float)(v[q] & 0xfff) / lv.hX);
                    kn[k] = bn;
                    atomicAdd(&bcnt[bn], 1);
                }
            }
        }
    }
    __syncthreads();
    QT_T(0);
    if (tid == 0) {
        int n = 0;
        for (int i = 0; i < nIni; ++i) {
            bpos[i] = -1;
            if (bcnt[i] == 0) continue;
            bpos[i] = n;
            s.rect[0][n] = make_short4((short)(int)(lv.hX * (float)i), 0, (short)(int)(lv.hX * (float)(i + 1)),
                                       (short)lv.qH);
            s.cnt[0][n] = bcnt[i];
            s.nomore[0][n] = bcnt[i] == 1;
            ++n;
        }
        s.misc[0] = n;
    }
    __syncthreads();
    // bins to list positions: the identity unless a bin is empty
    if (s.misc[0] != nIni)
        for (int k = tid; k < K; k += T) knode[k] = bpos[knode[k]];
    int size = s.misc[0];
    int cur = 0;
    const int N = lv.N;
    __syncthreads();
    QT_T(1);

    // 3. outer passes (:610-689)
    int nexp = 0;
    bool last = false;
    while (true) {
        const int prev = size;
        for (int i = tid; i < size; i += T) s.div[i] = s.nd[i] = qsel(s.nomore, cur)[i] ? 0 : 1;
        __syncthreads();
        const int m = block_excl_scan(s.nd, size, s.tmp);
        for (int i = tid; i < size; i += T)
            if (s.div[i]) s.ord[s.nd[i]] = i;
        __syncthreads();
#ifdef ORB_QT_TIMING
        ++qt_outer;
        QT_T(5);
#endif
        qt_count(s, cur, size, K, keys, knode, kq);
        QT_T(6);
        size = qt_divide(s, cur, size, m, K, knode, kq, &nexp);
        QT_T(7);
        if (size >= N || size == prev) break;
        if (size + nexp * 3 > N) { last = true; break; }
    }
    QT_T(2);
    // 4. last rounds (:692-753)
    while (last) {
        const int prev = size;
        const int m = nexp;
        for (int j = tid; j < m; j += T) {
            const int i = s.expand[j];
            s.srt[j] = SortRec{qsel(s.cnt, cur)[i], (int)qsel(s.rect, cur)[i].x, i};
        }
        for (int i = tid; i < size; i += T) s.div[i] = 0;
        __syncthreads();
        QT_T(15);
        // ccnt / newpos / ord are free until qt_count below
        block_std_sort(s.srt, m, (SortRec*)s.ccnt, s.newpos, s.newpos + NC, (SortFrame*)(s.newpos + 2 * NC),
                       (SortFrame*)(s.newpos + 3 * NC), s.ord, s.misc + 4, s.stk);
        for (int j = tid; j < m; j += T) s.div[s.srt[j].pos] = 1;
        __syncthreads();
        QT_T(12);
        qt_count(s, cur, size, K, keys, knode, kq);
        QT_T(13);
        // processing rank r = m-1-j; stop after the first rank at which the list reaches N
        for (int r = tid; r < m; r += T) {
            const int i = s.srt[m - 1 - r].pos;
            int ne = 0;
            for (int q = 0; q < 4; ++q) ne += s.ccnt[4 * i + q] > 0;
            s.rne[r] = ne - 1;
        }
        if (tid == 0) s.misc[1] = m;
        __syncthreads();
        block_excl_scan(s.rne, m, s.tmp);
        for (int r = tid; r < m; r += T) {
            const int i = s.srt[m - 1 - r].pos;
            int ne = 0;
            for (int q = 0; q < 4; ++q) ne += s.ccnt[4 * i + q] > 0;
            if (size + s.rne[r] + ne - 1 >= N) atomicMin(&s.misc[1], r + 1);
        }
        __syncthreads();
        const int mp = s.misc[1];
        for (int r = tid; r < m; r += T) {
            const int i = s.srt[m - 1 - r].pos;
            if (r < mp) s.ord[r] = i;
            else s.div[i] = 0;
        }
        __syncthreads();
        QT_T(15);
        size = qt_divide(s, cur, size, mp, K, knode, kq, &nexp);
        QT_T(14);
#ifdef ORB_QT_TIMING
        ++qt_lastr;
#endif
        if (size >= N || size == prev) break;
    }
    QT_T(3);
    // 5. retain the best key per node (:757-776)
    int* best = s.ccnt;
    for (int i = tid; i < size; i += T) best[i] = 0;
    __syncthreads();
    for (int k0 = tid; k0 < K; k0 += kQtB * T) {
        int n[kQtB];
        uint32_t key[kQtB];
#pragma unroll
        for (int b = 0; b < kQtB; ++b) {
            const int k = k0 + b * T;
            n[b] = k < K ? knode[k] : 0;
            key[b] = k < K ? keys[k] : 0u;
        }
#pragma unroll
        for (int b = 0; b < kQtB; ++b) {
            const int k = k0 + b * T;
            if (k < K) atomicMax(&best[n[b]], (int)(((key[b] >> 24) << 23) | (0x7FFFFF - k)));
        }
    }
    __syncthreads();
    const int nout = min(size, lv.out_cap);
    for (int i = tid; i < nout; i += T) out[i] = keys[0x7FFFFF - (best[i] & 0x7FFFFF)];
    if (tid == 0) a.qt_n[f * a.L + l] = nout;
#ifdef ORB_QT_TIMING
    QT_T(4);
    if (tid == 0) {
        atomicMax(&g_qt_t[l][8], __builtin_amdgcn_s_memtime() - qt_t0);
        atomicAdd(&g_qt_t[l][9], (unsigned long long)qt_outer);
        atomicAdd(&g_qt_t[l][10], (unsigned long long)qt_lastr);
        atomicAdd(&g_qt_t[l][11], 1ull);
    }
#endif
}

// ---------------------------------------------------------------------------
// k_quadtree_w: the same DistributeOctTree steps (ORBextractor.cc:555-779) for
// one (frame, level) by ONE wave, with the keys in registers.
//
// k_quadtree spends 82-103 us per 256 frames at 3 % VALU issue: its keys live
// in global memory, so every pass over them (gather, quadrant count, remap,
// retain) is a round trip to L2 per 1,024 keys, and each pass has a dozen
// block barriers between its four waves.  A level of C2 holds 300-1,500 keys
// and at most ~230 nodes, which one wave holds comfortably: lane l keeps the
// run of keys l KPL .. l KPL + KPL - 1 (vToDistributeKeys order: cell by cell,
// so a lane's keys mostly share a node) and each key's list index (bits 0-15;
// its quadrant in bits 16+ between the count and the remap).  Per-key passes
// are branch-free register work plus LDS reads of the key's node, and their
// LDS atomics are aggregated over a lane's run (a target word that stays the
// same accumulates in a register; the first passes have 2-8 nodes, so
// per-key atomics were thousands of same-address conflicts).  Per-node passes
// walk the list in 64-node chunks with ballots and DPP scans;
// synchronisation is the wave's own.  Node arrays stay in LDS, indexed by
// list position, double buffered across a rebuild.  nomore is cnt == 1 (a
// node never changes its count), so it is not stored.  A level with more than
// qw_kcap keys sets its overflow flag and is left to k_quadtree, launched
// after this kernel in fixup mode (only flagged levels run there).
// ---------------------------------------------------------------------------
#ifndef ORB_QW_KPL
#define ORB_QW_KPL 24   // keys per lane: levels of up to 1,536 keys (235 VGPRs; 32 spills 50)
#endif
constexpr int kQwKpl = ORB_QW_KPL;
#ifndef ORB_QW_WAVES
#define ORB_QW_WAVES 2   // 8 waves a CU (2,048 (frame, level) waves over 256 CUs)
#endif
constexpr size_t kQwLdsMax = 64 * 1024;   // larger layouts (Tracking's 5 x nFeatures extractor) keep k_quadtree

struct QwLds {
    short4* rect[2];
    int* cnt[2];
    uint32_t* cc;   // per node: quadrant counts (q0 | q1 << 16, q2 | q3 << 16)
    int* nb;        // per node: first child (divided) or new index (kept); initial bins: list position
    uint8_t* dv;    // per node: divides in this step
    int* ord;       // processing order of the dividing nodes
    int* queue;     // vSizeAndPointerToNode: children with > 1 key, processing order (list indices)
    SortRec* srt;
    uint32_t* mg;   // per node: its split point in the keys' guarded format (qw_guard)
    uint32_t* dum;  // one word per lane: the no-op target of the run-aggregated atomics
    uint8_t* u;     // shared by the gather, the divide's scans and the sort
};
__host__ __device__ inline size_t qw_al(size_t b) { return (b + 15) & ~size_t(15); }
// the union region: the gather (cell offsets, key cells), the divide's three
// scans, block_std_sort's scratch
__host__ __device__ inline size_t qw_union_bytes(int NC, int ncells, int kcap) {
    const size_t n = (size_t)NC;
    const size_t g = qw_al((size_t)(ncells + 1) * 4) + qw_al((size_t)kcap * 2);
    const size_t d = 3 * qw_al(n * 4);
    const size_t s = qw_al(n * sizeof(SortRec)) + 2 * qw_al(n * 4) + 2 * qw_al((n / 17 + 2) * sizeof(SortFrame)) +
                     qw_al((n + 2) * 4) + qw_al(16) + qw_al(80 * sizeof(SortFrame));
    return g > d ? (g > s ? g : s) : (d > s ? d : s);
}
__host__ __device__ inline size_t qw_lds_bytes(int NC, int ncells, int kcap) {
    const size_t n = (size_t)NC;
    return 2 * qw_al(n * 8) + 2 * qw_al(n * 4) + qw_al(n * 8) + qw_al(n * 4) + qw_al(n) + 2 * qw_al(n * 4) +
           qw_al(n * sizeof(SortRec)) + qw_al(n * 4) + qw_al(kWave * 4) + qw_union_bytes(NC, ncells, kcap);
}

// keys of a per-key pass in groups of kQwGrp: a compiler fence between
// groups keeps it from hoisting every key's LDS reads at once (spills)
#ifndef ORB_QW_GRP
#define ORB_QW_GRP 8
#endif
#define QW_GROUP_FENCE(j) do { if (((j) + 1) % ORB_QW_GRP == 0) asm volatile("" ::: "memory"); } while (0)

// Keys in registers in a guarded format: x | 1 << 12 | y << 13 | 1 << 25.
// With a node's split point (mx, my) as mx | my << 13, one subtraction
// compares both coordinates: bit 12 of the difference is x >= mx, bit 25 is
// y >= my (the guard bits absorb the borrows), so ExtractorNode::DivideNode's
// child (:511-525) is bit 12 | bit 25 >> 24 -- no unpacking a compiler could
// hoist out of the passes (it kept every key's x and y live: spills).
__device__ __forceinline__ uint32_t qw_guard(uint32_t key) {
    return (key & 0xfffu) | ((key & 0xfff000u) << 1) | 0x2001000u;
}
__device__ __forceinline__ uint32_t qw_unguard(uint32_t g, uint32_t resp) {
    return (g & 0xfffu) | ((g >> 1) & 0xfff000u) | (resp << 24);
}
__device__ __forceinline__ uint32_t qw_split(short4 r) {
    const int hx = (int)ceilf((float)(r.z - r.x) / 2), hy = (int)ceilf((float)(r.w - r.y) / 2);
    return (uint32_t)(r.x + hx) | ((uint32_t)(r.y + hy) << 13);
}
__device__ __forceinline__ int qw_quadrant(uint32_t g, uint32_t split) {
    const uint32_t d = g - split;
    return (int)(((d >> 12) & 1u) | ((d >> 24) & 2u));
}

__device__ __forceinline__ int qw_cc(const uint32_t* cc, int i, int q) {
    return (int)((cc[2 * i + (q >> 1)] >> (16 * (q & 1))) & 0xffffu);
}

// One step of a lane's run-aggregated LDS add: while the target word w stays
// the same the increments accumulate in acc; a changed target flushes the run
// into the previous word, every other step adds 0 to the lane's own dum word
// (no branch, no same-address conflict).  pw starts at kNoWord; qw_add_end
// flushes the last run.
constexpr uint32_t kNoWord = 0xffffffffu;
__device__ __forceinline__ void qw_add(uint32_t* base, uint32_t* mine, uint32_t w, uint32_t inc, uint32_t& pw,
                                       uint32_t& acc) {
    const bool flush = w != pw;
    atomicAdd(flush && pw != kNoWord ? base + pw : mine, flush ? acc : 0u);
    acc = flush ? inc : acc + inc;
    pw = w;
}
__device__ __forceinline__ void qw_add_end(uint32_t* base, uint32_t pw, uint32_t acc) {
    if (pw != kNoWord) atomicAdd(base + pw, acc);
}

// Divide ord[0..m) (counts in cc, dv set for exactly those nodes), rebuild the
// list into buffer cur ^ 1 (children blocks n4..n1 in REVERSE processing
// order, then the kept nodes in their old order: push_front + erase,
// ORBextractor.cc:633-679, :703-744), queue the children with > 1 key in
// processing order, remap the keys.  Returns the new size.
template <int KPL>
__device__ int qw_divide(QwLds& s, int& cur, int size, int m, uint32_t (&nq)[KPL], int NC, int& nexp) {
    const int lane = lane_id();
    int* rne = (int*)s.u;     // per rank: inclusive scan of the non-empty children
    int* rgt = rne + NC;      // per rank: exclusive scan of the children with > 1 key
    int* ndx = rgt + NC;      // per node: kept nodes before it
    int cne = 0, cgt = 0;
    for (int base = 0; base < m; base += kWave) {
        const int r = base + lane;
        int ne = 0, gt = 0;
        if (r < m) {
            const int i = s.ord[r];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int c = qw_cc(s.cc, i, q);
                ne += c > 0;
                gt += c > 1;
            }
        }
        const int ine = wave_incl_scan_dpp(ne), igt = wave_incl_scan_dpp(gt);
        if (r < m) {
            rne[r] = cne + ine;
            rgt[r] = cgt + igt - gt;
        }
        cne += __builtin_amdgcn_readlane(ine, kWave - 1);
        cgt += __builtin_amdgcn_readlane(igt, kWave - 1);
    }
    int cnd = 0;
    for (int base = 0; base < size; base += kWave) {
        const int i = base + lane;
        const bool kept = i < size && !s.dv[i];
        const uint64_t b = __ballot(kept);
        if (kept) ndx[i] = cnd + mask_rank(b);
        cnd += __popcll(b);
    }
    const int totNE = cne;
    const int nx = cur ^ 1;
    const short4* R = qsel(s.rect, cur);
    const int* C = qsel(s.cnt, cur);
    short4* Rn = qsel(s.rect, nx);
    int* Cn = qsel(s.cnt, nx);
    for (int r = lane; r < m; r += kWave) {
        const int i = s.ord[r];
        const short4 ri = R[i];
        int c[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) c[q] = qw_cc(s.cc, i, q);
        const int start = totNE - rne[r];
        int w = start;
        int pos[4];
#pragma unroll
        for (int q = 3; q >= 0; --q) {
            pos[q] = w;
            if (c[q] > 0) {
                Rn[w] = child_rect(ri, q);
                Cn[w] = c[q];
                ++w;
            }
        }
        s.nb[i] = start;
        int e = rgt[r];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (c[q] > 1) s.queue[e++] = pos[q];
    }
    for (int i = lane; i < size; i += kWave) {
        if (s.dv[i]) continue;
        const int np = totNE + ndx[i];
        s.nb[i] = np;
        Rn[np] = R[i];
        Cn[np] = C[i];
    }
    fast_wave_sync();
    // keys: a divided node's child q sits at first child + its non-empty
    // siblings q' > q (n4 first); a kept node moved to nb
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        const int n = (int)(nq[j] & 0xffffu), q = (int)(nq[j] >> 16);
        const int d = s.dv[n], b = s.nb[n];
        const uint32_t w0 = s.cc[2 * n], w1 = s.cc[2 * n + 1];
        const int above = (q < 3 && (w1 >> 16) != 0u) + (q < 2 && (w1 & 0xffffu) != 0u) + (q < 1 && (w0 >> 16) != 0u);
        nq[j] = (uint32_t)(b + (d ? above : 0));
        QW_GROUP_FENCE(j);
    }
    fast_wave_sync();
    cur = nx;
    nexp = cgt;
    return totNE + (size - m);
}

// Quadrant counts of every node with dv set; every key keeps its quadrant in
// nq bits 16+ (read by qw_divide only for keys of dividing nodes).
template <int KPL>
__device__ void qw_count(QwLds& s, int cur, int size, const uint32_t (&key)[KPL], uint32_t (&nq)[KPL]) {
    const int lane = lane_id();
    const short4* R = qsel(s.rect, cur);
    for (int i = lane; i < size; i += kWave) {
        s.cc[2 * i] = 0u;
        s.cc[2 * i + 1] = 0u;
        s.mg[i] = qw_split(R[i]);
    }
    fast_wave_sync();
    uint32_t pw = kNoWord, acc = 0u;
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        const int n = (int)nq[j];
        const int d = s.dv[n];
        const int q = qw_quadrant(key[j], s.mg[n]);
        nq[j] = (uint32_t)n | ((uint32_t)q << 16);
        qw_add(s.cc, s.dum + lane, 2u * (uint32_t)n + (uint32_t)(q >> 1), d ? 1u << (16 * (q & 1)) : 0u, pw, acc);
        QW_GROUP_FENCE(j);
    }
    qw_add_end(s.cc, pw, acc);
    fast_wave_sync();
}

template <int KPL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(ORB_QW_WAVES))) void k_quadtree_w(QtArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int f = blockIdx.x, l = blockIdx.y, lane = threadIdx.x;
    const LevelDev lv = a.lv[l];
    const int NC = a.qw_nc;
#ifdef ORB_QT_TIMING
    const int tid = lane;
    const unsigned long long qt_t0 = __builtin_amdgcn_s_memtime();
    unsigned long long qt_last = qt_t0;
    int qt_outer = 0, qt_lastr = 0;
#endif
    QwLds s;
    {
        uint8_t* p = smem;
        auto take = [&](size_t bytes) { uint8_t* q = p; p += qw_al(bytes); return q; };
        s.rect[0] = (short4*)take(NC * 8);
        s.rect[1] = (short4*)take(NC * 8);
        s.cnt[0] = (int*)take(NC * 4);
        s.cnt[1] = (int*)take(NC * 4);
        s.cc = (uint32_t*)take(NC * 8);
        s.nb = (int*)take(NC * 4);
        s.dv = take(NC);
        s.ord = (int*)take(NC * 4);
        s.queue = (int*)take(NC * 4);
        s.srt = (SortRec*)take(NC * sizeof(SortRec));
        s.mg = (uint32_t*)take(NC * 4);
        s.dum = (uint32_t*)take(kWave * 4);
        s.u = p;
    }
    const int nc = lv.ncells;
    const int* ccount = a.cell_count + (long long)f * a.ncells_total + lv.cell_base;
    const uint32_t* cslots = a.cell_keys + (long long)f * a.slot_total + lv.slot_base;
    uint32_t* out = a.qt_key + (long long)f * a.out_total + lv.out_base;

    // 1. vToDistributeKeys (:805-872): cell offsets by one scan, lane l over a
    // contiguous run of cells; then the cell of every key, and the keys
    int* off = (int*)s.u;
    uint16_t* kcell = (uint16_t*)(s.u + qw_al((size_t)(nc + 1) * 4));
    for (int cb = 0; cb < nc; cb += 16 * kWave) {   // 16 loads a lane in flight (a load-store loop waited on each)
        int v[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int c = cb + t * kWave + lane;
            v[t] = c < nc ? ccount[c] : 0;
        }
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int c = cb + t * kWave + lane;
            if (c < nc) off[c] = v[t];
        }
    }
    fast_wave_sync();
    const int per = (nc + kWave - 1) / kWave;
    const int c0 = min(nc, lane * per), c1 = min(nc, c0 + per);
    int sum = 0;
    for (int c = c0; c < c1; ++c) sum += off[c];
    const int incl = wave_incl_scan_dpp(sum);
    const int K = __builtin_amdgcn_readlane(incl, kWave - 1);
    if (K > a.qw_kcap) {
        if (lane == 0) a.qt_ovf[f * a.L + l] = 1;
        return;
    }
    if (lane == 0) a.qt_ovf[f * a.L + l] = 0;
    if (K == 0) {
        if (lane == 0) a.qt_n[f * a.L + l] = 0;
        return;
    }
    {
        int run = incl - sum;
        for (int c = c0; c < c1; ++c) {
            const int x = off[c];
            off[c] = run;
            run += x;
        }
        if (lane == 0) off[nc] = K;
    }
    fast_wave_sync();
    // key k's cell at (k % KPL) * 64 + k / KPL: lane l reads its run's j-th
    // cell at j * 64 + l (a straight index would put lanes l and l + 4 in one bank)
    for (int c = c0; c < c1; ++c)
        for (int j = off[c], e = off[c + 1]; j < e; ++j) kcell[(j % KPL) * kWave + j / KPL] = (uint16_t)c;
    fast_wave_sync();
    const int cap = lv.slot_total / nc;
    const int k0 = lane * KPL;   // this lane's run of keys
    uint32_t key[KPL], nq[KPL];  // key: guarded x, y (qw_guard)
    uint32_t rs[(KPL + 3) / 4];  // responses, 4 bytes a register
    {
        int src[KPL];
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            const int k = k0 + j;
            const int c = k < K ? (int)kcell[j * kWave + lane] : 0;
            src[j] = k < K ? c * cap + (k - off[c]) : -1;
        }
#pragma unroll
        for (int j = 0; j < KPL; ++j) key[j] = src[j] >= 0 ? cslots[src[j]] : 0u;
#pragma unroll
        for (int j = 0; j < (KPL + 3) / 4; ++j) rs[j] = 0u;
#pragma unroll
        for (int j = 0; j < KPL; ++j) rs[j / 4] |= (key[j] >> 24) << (8 * (j % 4));
#pragma unroll
        for (int j = 0; j < KPL; ++j) key[j] = qw_guard(key[j]);
    }
    fast_wave_sync();   // off / kcell (the union region) are dead from here
    QT_T(0);
#ifndef ORB_QW_ABL
#define ORB_QW_ABL 0   // timing ablation (tools only; wrong results): return after phase 1 gather, 2 init, 3 outer, 4 last rounds
#endif
#define QW_ABL_RETURN(p)                                           \
    do {                                                           \
        if (ORB_QW_ABL == (p)) {                                   \
            if (lane == 0) a.qt_n[f * a.L + l] = 0;                \
            if (lane == 0 && key[0] == 12345u) out[0] = nq[0];     \
            return;                                                \
        }                                                          \
    } while (0)
    if (ORB_QW_ABL == 1)
        for (int j = 0; j < KPL; ++j) nq[j] = 0;
    QW_ABL_RETURN(1);

    // 2. the initial nodes (:559-601): key k in bin x / hX (vpIniNodes), empty
    // bins dropped, the rest in bin order; nomore = one key.  Keys k >= K (the
    // register slots past the level's keys) sit in the dummy node NC - 1:
    // never in the list, never dividing, remapped onto itself.
    const int nIni = lv.nIni;
    const int dummy = NC - 1;
    int* bcnt = s.cnt[1];
    for (int i = lane; i < nIni; i += kWave) bcnt[i] = 0;
    if (lane == 0) {
        s.dv[dummy] = 0;
        s.nb[dummy] = dummy;
    }
    fast_wave_sync();
    {
        uint32_t pw = kNoWord, acc = 0u;
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            const bool ok = k0 + j < K;
            const int bn = ok ? (int)((float)(key[j] & 0xfff) / lv.hX) : 0;
            nq[j] = ok ? (uint32_t)bn : (uint32_t)dummy;
            qw_add((uint32_t*)bcnt, s.dum + lane, (uint32_t)bn, ok ? 1u : 0u, pw, acc);
        }
        qw_add_end((uint32_t*)bcnt, pw, acc);
    }
    fast_wave_sync();
    int size = 0;
    for (int base = 0; base < nIni; base += kWave) {
        const int i = base + lane;
        const int c = i < nIni ? bcnt[i] : 0;
        const uint64_t b = __ballot(c > 0);
        if (c > 0) {
            const int pos = size + mask_rank(b);
            s.nb[i] = pos;
            s.rect[0][pos] = make_short4((short)(int)(lv.hX * (float)i), 0, (short)(int)(lv.hX * (float)(i + 1)),
                                         (short)lv.qH);
            s.cnt[0][pos] = c;
        }
        size += __popcll(b);
    }
    fast_wave_sync();
    if (size != nIni) {
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            nq[j] = (uint32_t)s.nb[nq[j]];
            QW_GROUP_FENCE(j);
        }
        fast_wave_sync();
    }
    int cur = 0;
    const int N = lv.N;
    QT_T(1);
    QW_ABL_RETURN(2);

    // 3. outer passes (:610-689): every node with > 1 key divides, in list order
    int nexp = 0;
    bool last = false;
    while (true) {
        const int prev = size;
        int m = 0;
        const int* C = qsel(s.cnt, cur);
        for (int base = 0; base < size; base += kWave) {
            const int i = base + lane;
            const bool d = i < size && C[i] > 1;
            const uint64_t b = __ballot(d);
            if (i < size) s.dv[i] = d;
            if (d) s.ord[m + mask_rank(b)] = i;
            m += __popcll(b);
        }
        fast_wave_sync();
#ifdef ORB_QT_TIMING
        ++qt_outer;
        QT_T(5);
#endif
        qw_count<KPL>(s, cur, size, key, nq);
        QT_T(6);
        size = qw_divide<KPL>(s, cur, size, m, nq, NC, nexp);
        QT_T(7);
        if (size >= N || size == prev) break;
        if (size + nexp * 3 > N) {
            last = true;
            break;
        }
    }
    QW_ABL_RETURN(3);
    // 4. last rounds (:692-753): the queue sorted by (count, UL.x) with the
    // libstdc++ std::sort port, divided from the largest until the list holds N
    while (last) {
        const int prev = size;
        const int m = nexp;
        {
            const short4* R = qsel(s.rect, cur);
            const int* C = qsel(s.cnt, cur);
            for (int j = lane; j < m; j += kWave) {
                const int i = s.queue[j];
                s.srt[j] = SortRec{C[i], (int)R[i].x, i};
            }
            for (int i = lane; i < size; i += kWave) s.dv[i] = 0;
        }
        fast_wave_sync();
        QT_T(15);
        {
            uint8_t* p = s.u;
            auto take = [&](size_t bytes) { uint8_t* q = p; p += qw_al(bytes); return q; };
            SortRec* backup = (SortRec*)take(NC * sizeof(SortRec));
            int* Lp = (int*)take(NC * 4);
            int* Rp = (int*)take(NC * 4);
            SortFrame* qa = (SortFrame*)take((NC / 17 + 2) * sizeof(SortFrame));
            SortFrame* qb = (SortFrame*)take((NC / 17 + 2) * sizeof(SortFrame));
            int* leaves = (int*)take((NC + 2) * 4);
            int* ctl = (int*)take(16);
            SortFrame* stk = (SortFrame*)take(80 * sizeof(SortFrame));
            block_std_sort(s.srt, m, backup, Lp, Rp, qa, qb, leaves, ctl, stk);
        }
        for (int j = lane; j < m; j += kWave) s.dv[s.srt[j].pos] = 1;
        fast_wave_sync();
        QT_T(12);
        qw_count<KPL>(s, cur, size, key, nq);
        QT_T(13);
        // processing rank r = m-1-j; stop after the first rank at which the list reaches N
        int mp = m, carry = 0;
        for (int base = 0; base < m; base += kWave) {
            const int r = base + lane;
            int d = 0;
            if (r < m) {
                const int i = s.srt[m - 1 - r].pos;
#pragma unroll
                for (int q = 0; q < 4; ++q) d += qw_cc(s.cc, i, q) > 0;
                d -= 1;
            }
            const int inc = wave_incl_scan_dpp(d);
            const uint64_t hit = __ballot(r < m && size + carry + inc >= N);
            if (hit) {
                mp = base + (int)__builtin_ctzll(hit) + 1;
                break;
            }
            carry += __builtin_amdgcn_readlane(inc, kWave - 1);
        }
        for (int r = lane; r < m; r += kWave) {
            const int i = s.srt[m - 1 - r].pos;
            if (r < mp) s.ord[r] = i;
            else s.dv[i] = 0;
        }
        fast_wave_sync();
        QT_T(15);
        size = qw_divide<KPL>(s, cur, size, mp, nq, NC, nexp);
        QT_T(14);
#ifdef ORB_QT_TIMING
        ++qt_lastr;
#endif
        if (size >= N || size == prev) break;
    }
    QT_T(3);
    QW_ABL_RETURN(4);
    // 5. retain the best key per node (:757-776): max response, the first in
    // vToDistributeKeys order on ties (key k scores (response << 23) | (2^23 -
    // 1 - k), distinct per key); the winner writes its node's slot
    int* best = (int*)s.cc;
    for (int i = lane; i < size; i += kWave) best[i] = 0;
    fast_wave_sync();
    {
        uint32_t pw = kNoWord;
        int acc = 0;
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            const uint32_t resp = (rs[j / 4] >> (8 * (j % 4))) & 0xffu;
            const int v = (int)((resp << 23) | (uint32_t)(0x7FFFFF - (k0 + j)));
            const uint32_t w = nq[j];
            const bool flush = w != pw;
            atomicMax(flush && pw != kNoWord ? best + pw : (int*)(s.dum + lane), flush ? acc : 0);
            acc = flush ? v : max(acc, v);
            pw = w;
            QW_GROUP_FENCE(j);
        }
        atomicMax(best + pw, acc);
    }
    fast_wave_sync();
    const int nout = min(size, lv.out_cap);   // (the dummy node is >= size)
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        const int n = (int)nq[j];
        const uint32_t resp = (rs[j / 4] >> (8 * (j % 4))) & 0xffu;
        if (n < nout && best[n] == (int)((resp << 23) | (uint32_t)(0x7FFFFF - (k0 + j)))) out[n] = qw_unguard(key[j], resp);
        QW_GROUP_FENCE(j);
    }
    if (lane == 0) a.qt_n[f * a.L + l] = nout;
#ifdef ORB_QT_TIMING
    QT_T(4);
    if (lane == 0) {
        atomicMax(&g_qt_t[l][8], __builtin_amdgcn_s_memtime() - qt_t0);
        atomicAdd(&g_qt_t[l][9], (unsigned long long)qt_outer);
        atomicAdd(&g_qt_t[l][10], (unsigned long long)qt_lastr);
        atomicAdd(&g_qt_t[l][11], 1ull);
    }
#endif
}

// ---------------------------------------------------------------------------
// k_describe: computeOrientation/IC_Angle (ORBextractor.cc:76-103,471-478) and
// computeOrbDescriptor (:107-146) with the level blur folded in.
//
// The reference blurs every full level (GaussianBlur 7x7, sigma 2,
// REFLECT_101 on a clone(), :1132-1133) and samples it.  Here one wave per
// keypoint stages the 43x43 raw patch around the keypoint in LDS (reflected
// at the level border exactly like the full-level blur would see it), reads
// the IC_Angle disc (radius 15) from it, blurs the 37x37 centre with the same
// fixed-point separable kernel and evaluates the 256 tests on
// it: the blurred level never goes to HBM.  Lane l evaluates tests 4l..4l+3.
// The horizontal pass is stored column-major, so a sample's 7 vertical taps
// are 7 consecutive u16: two ds_read2_b32 and four v_dot2 per sample instead
// of 7 scattered u16 reads (54 % bank-conflict cycles in round 1; the kernel
// time did not change: it is VALU/latency-bound).
// ---------------------------------------------------------------------------
constexpr int kRaw = 43, kRawP = 48, kBl = 37;
// column-major horizontal-pass buffer: hbT[col][row], a column's 43 rows plus
// pad (u16 units; ORB_DESC_HBT / 2 dwords per column)
#ifndef ORB_DESC_HBT
#define ORB_DESC_HBT 44
#endif
constexpr int kHbT = ORB_DESC_HBT;
static_assert(kHbT >= 44 && kHbT % 2 == 0, "a column holds 43 rows plus the 7-tap read's pad, in whole dwords");
#ifndef ORB_DESC_SLOTS
#define ORB_DESC_SLOTS 8   // 16 -> 8: 257-259 vs 263-267 us (twice as many waves, 4 frames an XCD at a time; profiles/r05/README.md)
#endif
#ifndef ORB_DESC_ABL
#define ORB_DESC_ABL 0   // timing ablation (tools only; wrong results): 1 = every patch load hits one L2-resident patch
#endif
constexpr int kDescSlots = ORB_DESC_SLOTS;   // keypoint slots per wave
#ifndef ORB_DESC_WPB
// waves per k_describe block (each wave owns its slots and its LDS buffers):
// one-wave blocks free their LDS when their wave ends (describe 0.325 -> 0.30
// ms); with the matching placed after the pyramid stage (bench --sfi-after 1)
#define ORB_DESC_WPB 1
#endif
constexpr int kDescWpb = ORB_DESC_WPB;

struct DescArgs {
    const uint8_t* in;
    long long in_fstride;
    int in_pitch;
    const uint8_t* pyr;
    long long pyr_fstride;
    const LevelDev* lv;
    const uint32_t* qt_key;
    const int* qt_n;
    float* angle;
    uint8_t* sdesc;
    int out_total, L;
    const uint8_t* slot_level;      // level of each of the out_total per-frame slots
    long long nslots;               // frames * out_total
    int fma;
    int kern[7];
    int umax[16];
};

// One keypoint slot of the flat (frame, quadtree output) space: qt_key, angle
// and sdesc are all indexed by the slot.
struct DescKp {
    const uint8_t* img;
    int pitch, w, h;
    uint32_t key;
};

// The wave's run of slots is resolved once, lane j holding slot s_begin + j
// (validity, key, level geometry), so the keypoint loop reads everything from
// registers (readlane) and no dependent load chain stands between a keypoint
// and the prefetch of the next one's patch.
struct DescLane {
    uint64_t img;
    int pitch, w, h;
    uint32_t key;
};

__device__ __forceinline__ bool desc_lane(const DescArgs& a, long long s, DescLane& k) {
    const int f = (int)(s / a.out_total);
    const int o = (int)(s - (long long)f * a.out_total);
    const int l = a.slot_level[o];
    const LevelDev& lv = a.lv[l];
    if (o - lv.out_base >= a.qt_n[f * a.L + l]) return false;
    k.img = (uint64_t)(l == 0 ? a.in + f * a.in_fstride : a.pyr + f * a.pyr_fstride + lv.off);
    k.pitch = l == 0 ? a.in_pitch : lv.pitch;
    k.w = lv.w;
    k.h = lv.h;
    k.key = a.qt_key[s];
    return true;
}

__device__ __forceinline__ DescKp desc_pick(const DescLane& k, int j) {
    DescKp d;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)k.img, j);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(k.img >> 32), j);
    d.img = (const uint8_t*)(((uint64_t)hi << 32) | lo);
    d.pitch = __builtin_amdgcn_readlane(k.pitch, j);
    d.w = __builtin_amdgcn_readlane(k.w, j);
    d.h = __builtin_amdgcn_readlane(k.h, j);
    d.key = (uint32_t)__builtin_amdgcn_readlane((int)k.key, j);
    return d;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int refl101(int p, int n) { return p < 0 ? -p : (p >= n ? 2 * n - 2 - p : p); }

// The 43 x 43 raw patch whose top-left level pixel is (x0, y0), row pitch 48 in
// LDS.  Interior patches move as 12 aligned dwords per row: patch_issue puts
// all 516 dword loads of one patch in flight into registers (the caller does
// this one keypoint ahead), patch_land writes them to LDS.  Patches touching
// the level border take reflected byte loads (patch_border).
constexpr int kPDw = kRawP / 4, kPN = kRaw * kPDw, kPV = (kPN + kWave - 1) / kWave;   // 12, 516, 9

__device__ __forceinline__ bool patch_interior(int w, int h, int x0, int y0) {
    return y0 >= 0 && y0 + kRaw <= h && x0 >= 0 && (x0 & ~3) + kRawP <= w;
}

__device__ __forceinline__ void patch_issue(const uint8_t* img, int pitch, int x0, int y0, uint32_t (&v)[kPV]) {
    const int lane = lane_id(), base = x0 & ~3;
    const GlobalBytes g = (GlobalBytes)img;
#pragma unroll
    for (int j = 0; j < kPV; ++j) {
        const int i = lane + j * kWave;
        if (i < kPN) {
            const int r = i / kPDw, d = i - r * kPDw;
#if ORB_DESC_ABL == 1
            v[j] = *(GlobalWords)(g + (long long)r * pitch + 4 * d);   // ablation: one L2-resident patch (timing only)
#else
            v[j] = *(GlobalWords)(g + (long long)(y0 + r) * pitch + base + 4 * d);
#endif
        }
    }
}

__device__ __forceinline__ void patch_land(const uint32_t (&v)[kPV], uint8_t* raw) {
    const int lane = lane_id();
#pragma unroll
    for (int j = 0; j < kPV; ++j) {
        const int i = lane + j * kWave;
        if (i < kPN) ((uint32_t*)raw)[i] = v[j];
    }
}

#ifndef ORB_DESC_ROWLOAD
#define ORB_DESC_ROWLOAD 1   // lane r loads patch row r as three 16-byte loads (one address per lane, no div/mod): describe 281-285 -> 261-267 us (profiles/r05/desc_rowload_*); 0: the 516-dword spread
#endif
// The row form: lane r < 43 holds row r's 12 dwords (3 x 16 B from a 4-byte
// aligned address), lands them as 3 x ds_write_b128 at raw + 48 r.
constexpr int kPR = 12;
// xs: the 4-byte aligned first column; rows outside [0, h) reflected (REFLECT_101)
__device__ __forceinline__ void patch_issue_rows(const uint8_t* img, int pitch, int h, int xs, int y0,
                                                 uint32_t (&v)[kPR]) {
    const int lane = lane_id();
    if (lane < kRaw) {
        // 12 consecutive dwords (the load vectorizer makes them dwordx4 loads)
#if ORB_DESC_ABL == 1
        const GlobalWords p = (GlobalWords)(img + (long long)lane * pitch);   // ablation: one L2-resident patch (timing only)
        (void)h; (void)xs; (void)y0;
#else
        const GlobalWords p = (GlobalWords)(img + (long long)refl101(y0 + lane, h) * pitch + xs);
#endif
#pragma unroll
        for (int k = 0; k < kPR; ++k) v[k] = p[k];
    }
}
__device__ __forceinline__ void patch_land_rows(const uint32_t (&v)[kPR], uint8_t* raw) {
    const int lane = lane_id();
    if (lane < kRaw) {
        uint4* q = (uint4*)(raw + lane * kRawP);
        q[0] = make_uint4(v[0], v[1], v[2], v[3]);
        q[1] = make_uint4(v[4], v[5], v[6], v[7]);
        q[2] = make_uint4(v[8], v[9], v[10], v[11]);
    }
}
// Left-border landing: the row was loaded from column 0 and the patch starts at
// x0 in [-3, -1]; the row goes in one dword later, and the first dword holds
// the reflected columns -1, -2, -3 = pixels 1, 2, 3 at bytes 3, 2, 1, so the
// patch reads from byte 4 + x0 like an interior one from x0 & 3
__device__ __forceinline__ void patch_land_rows_left(const uint32_t (&v)[kPR], uint8_t* raw) {
    const int lane = lane_id();
    if (lane < kRaw) {
        uint4* q = (uint4*)(raw + lane * kRawP);
        q[0] = make_uint4(__builtin_amdgcn_perm(v[0], v[0], 0x01020300u), v[0], v[1], v[2]);
        q[1] = make_uint4(v[3], v[4], v[5], v[6]);
        q[2] = make_uint4(v[7], v[8], v[9], v[10]);
    }
}
#ifndef ORB_DESC_BORDER_ROWS
#define ORB_DESC_BORDER_ROWS 1   // border patches by prefetched row loads where the columns allow (0: all by reflected byte loads)
#endif
// How the patch whose top-left level pixel is (x0, y0) is fetched: 1 row
// loads from x0 & ~3, 2 row loads from column 0 (left border, x0 in [-3, -1]),
// 3 row loads from x0 & ~3 with the one or two columns past the right border
// (w, w + 1 = pixels w - 2, w - 3) rewritten in LDS after landing, 0
// reflected byte loads (patch_border).  Rows outside the level are reflected
// per lane in modes 1-3; a row load may read past the level width but stays
// inside the row pitch, and no loaded byte of a column >= w is used.
__device__ __forceinline__ int patch_mode(int w, int h, int pitch, int x0, int y0) {
#if ORB_DESC_BORDER_ROWS && ORB_DESC_ROWLOAD
    if (y0 < 1 - h || y0 + kRaw > 2 * h - 1) return 0;
    if (x0 >= 0) {
        if ((x0 & ~3) + kRawP > pitch) return 0;
        if (x0 + kRaw <= w) return 1;
        return x0 + kRaw <= w + 2 ? 3 : 0;
    }
    return x0 >= -3 && x0 + kRaw <= w && kRawP <= pitch ? 2 : 0;
#else
    (void)pitch;
    return patch_interior(w, h, x0, y0) ? 1 : 0;
#endif
}
#if ORB_DESC_ROWLOAD
constexpr int kPVN = kPR;
#define DESC_PATCH_ISSUE patch_issue_rows
#define DESC_PATCH_LAND patch_land_rows
#else
constexpr int kPVN = kPV;
#define DESC_PATCH_ISSUE patch_issue
#define DESC_PATCH_LAND patch_land
#endif

#ifndef ORB_DESC_BORDER_BATCH
#define ORB_DESC_BORDER_BATCH 10   // reflected byte loads in flight per lane (0: the round-3 loop, one at a time)
#endif
__device__ __forceinline__ void patch_border(const uint8_t* img, int pitch, int w, int h, int x0, int y0,
                                             uint8_t* raw) {
#if ORB_DESC_BORDER_BATCH
    // 29 bytes per lane in batches whose loads are all in flight before the
    // first LDS store (one memory round trip per batch, not per byte)
    constexpr int kB = ORB_DESC_BORDER_BATCH, kN = (kRaw * kRaw + kWave - 1) / kWave;
    const int lane = lane_id();
#pragma unroll 1
    for (int j0 = 0; j0 < kN; j0 += kB) {   // (rolled: unrolled, the lane-invariant offsets get hoisted out of the keypoint loop and spill)
        uint32_t v[kB];
        int o[kB];
#pragma unroll
        for (int j = 0; j < kB; ++j) {
            const int i = min(lane + (j0 + j) * kWave, kRaw * kRaw - 1);   // past the patch: repeats its last byte
            const int r = i / kRaw, c = i - r * kRaw;
            o[j] = r * kRawP + c;
            v[j] = (j0 + j < kN) ? ((GlobalBytes)img)[(long long)refl101(y0 + r, h) * pitch + refl101(x0 + c, w)] : 0u;
        }
#pragma unroll
        for (int j = 0; j < kB; ++j)
            if (j0 + j < kN) raw[o[j]] = (uint8_t)v[j];
    }
#else
    for (int i = lane_id(); i < kRaw * kRaw; i += kWave) {
        const int r = i / kRaw, c = i - r * kRaw;
        raw[r * kRawP + c] = ((GlobalBytes)img)[(long long)refl101(y0 + r, h) * pitch + refl101(x0 + c, w)];
    }
#endif
}

#ifdef ORB_DESC_TIMING
// phase profile of k_describe (tools/fast_phases.py --describe): shader cycles per phase
__device__ unsigned long long g_desc_t[1024][8];
#define DESC_T(var)                                                          \
    do {                                                                     \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();          \
        var += t_ - tlast;                                                   \
        tlast = t_;                                                          \
    } while (0)
extern "C" int orbx_debug_desc_timing(unsigned long long* out, int reset) {
    static unsigned long long h[1024][8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_desc_t), sizeof(h)) != hipSuccess) return -4;
    for (int k = 0; k < 8; ++k) {
        out[k] = 0;
        for (int i = 0; i < 1024; ++i) out[k] += h[i][k];
    }
    if (reset) {
        static unsigned long long z[1024][8];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_desc_t), z, sizeof(z)) != hipSuccess) return -4;
    }
    return 0;
}
#else
#define DESC_T(var) do { } while (0)
#endif

#ifndef ORB_DESC_WAVES
#define ORB_DESC_WAVES 4
#endif
#ifndef ORB_DESC_PF2
#define ORB_DESC_PF2 0   // 1: two patches in flight per wave (measured slower: describe 0.352-0.362 -> 0.369-0.372 ms)
#endif
#ifndef ORB_DESC_ICM_REG
#define ORB_DESC_ICM_REG 1   // IC_Angle disc masks held in 9 VGPRs (0: made per use from umax)
#endif
#ifndef ORB_DESC_PATF
#define ORB_DESC_PATF 0   // 1: pattern points converted to float once per wave
#endif
#ifndef ORB_DESC_HDOT4
#define ORB_DESC_HDOT4 1   // horizontal pass by v_dot4_u32_u8 (0: packed-u16 pairs, round 2)
#endif
#ifndef ORB_Q_UNROLL
// rBRIEF test groups unrolled: all 8 samples of a lane in one block (122 VGPRs,
// still 4 waves a SIMD): describe 261-264 -> 245 us (profiles/r05/README.md)
#define ORB_Q_UNROLL 4
#endif
#ifndef ORB_DESC_HMFMA
#define ORB_DESC_HMFMA 1   // horizontal pass on the matrix cores (v_mfma_i32_16x16x64_i8); 0: v_dot4 per row
#endif
// The horizontal pass as a product on the matrix cores: H[r][x] = sum_t w_t
// raw[r][x + t] is (the raw patch, its rows realigned by the column shift sh)
// x (a 64 x 37 banded matrix, w_t at row x + t of column x).
// v_mfma_i32_16x16x64_i8 takes i8 operands, so the pixels go in as p ^ 0x80 =
// p - 128 and every output starts from 128 * sum(w) (all 7 taps of an output
// lie inside the row); the taps are < 128 (checked on the host).  Integer and
// exact: H is the ufixedpoint16 sum of the dot4 form.  M = 43 rows as the
// 16-row blocks at rows 0, 16, 28 (the last overlaps: rows 28..31 are written
// twice with equal values, row 43 lands in the column pad), N = 37 outputs as
// the 16-column blocks at 0, 16, 22 (likewise), K = 64 (bytes 43.. meet zero
// weights), so every lane's store is in bounds and unpredicated.  Operand maps
// (as the 32x32x32 form, tools/mfma_i8_probe.hip): lane l feeds A row (l & 15)
// and B column (l & 15) with the 16-byte k-slice 16 (l >> 4); result rows
// 4 (l >> 4) + i, column l & 15.  The band is 12 VGPRs made once per wave.
constexpr int kHmNb = 3;
typedef int v4i_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int hm_row0(int mb) { return mb == 0 ? 0 : (mb == 1 ? 16 : 28); }
__device__ __forceinline__ int hm_col0(int nb) { return nb == 0 ? 0 : (nb == 1 ? 16 : 22); }
template <bool FMA>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ORB_DESC_WAVES))) void k_describe(DescArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t raw_s[kDescWpb][kRaw * kRawP];
    __shared__ __attribute__((aligned(16))) uint16_t hb_s[kDescWpb][(kBl + 1) * kHbT];
    const int lane = lane_id(), wv = wave_id();
#if ORB_DESC_HMFMA
    // lane's 16 band bytes: byte e = w[16 (l >> 4) + e - n], i.e. the 7 taps as
    // a 56-bit little-endian word T shifted by d = 16 (l >> 4) - n bytes
    v4i_t Bm[kHmNb];
    {
        uint64_t T = 0;
#pragma unroll
        for (int q = 0; q < 7; ++q) T |= (uint64_t)((uint32_t)a.kern[q] & 0xffu) << (8 * q);
#pragma unroll
        for (int nb = 0; nb < kHmNb; ++nb) {
            const int d = 16 * (lane >> 4) - (hm_col0(nb) + (lane & 15));
            uint64_t lo = 0, hi = 0;
            if (d >= 0) {
                if (d < 7) lo = T >> (8 * d);
            } else {
                const int s = -8 * d;
                if (s < 64) { lo = T << s; hi = T >> (64 - s); }
                else if (s < 128) hi = T << (s - 64);
            }
            Bm[nb] = v4i_t{(int)(uint32_t)lo, (int)(uint32_t)(lo >> 32), (int)(uint32_t)hi, (int)(uint32_t)(hi >> 32)};
        }
    }
    const int hbias = 128 * (a.kern[0] + a.kern[1] + a.kern[2] + a.kern[3] + a.kern[4] + a.kern[5] + a.kern[6]);
#endif
    // lane's 4 tests = 16 consecutive pattern bytes, kept packed in registers
    const uint4 patv = ((const uint4*)c_pattern)[lane];
    // wait for the pattern here: a use inside the keypoint loop would get a
    // conservative vmcnt(0) that also drains the patch prefetch
    asm volatile("" ::"v"(patv.x), "v"(patv.y), "v"(patv.z), "v"(patv.w));
    const uint32_t patw[4] = {patv.x, patv.y, patv.z, patv.w};
#if ORB_DESC_PATF
    // the lane's 8 pattern points as floats, made once (4 VALU per sample in the loop otherwise)
    float pfx[8], pfy[8];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            pfx[2 * q + e] = (float)(int)(int8_t)(patw[q] >> (16 * e));
            pfy[2 * q + e] = (float)(int)(int8_t)(patw[q] >> (16 * e + 8));
        }
#endif
    uint8_t* raw = raw_s[wv];
    uint16_t* hb = hb_s[wv];
    // symmetric 7-tap kernel: k0 = k6, k1 = k5, k2 = k4
    const uint32_t k0 = a.kern[0], k1 = a.kern[1], k2 = a.kern[2], k3 = a.kern[3];
    // u16 weight pairs of the vertical taps v0..v6 over 4 dwords whose first
    // tap is at the low half of the first (v0v1 v2v3 v4v5 v6-)
    const uint32_t W0e = k0 | (k1 << 16), W1e = k2 | (k3 << 16), W2e = k2 | (k1 << 16), W3e = k0;
#if ORB_DESC_HDOT4
    // horizontal taps w = (k0 k1 k2 k3 k2 k1 k0) as bytes for v_dot4 on the
    // words al[j], al[j+1], al[j+2] of an output at byte offset b = 0..3:
    // b 0: (w0..w3)(w4 w5 w6 -); 1: (- w0 w1 w2)(w3..w6); 2: (- - w0 w1)(w2..w5)(w6 - - -);
    // 3: (- - - w0)(w1..w4)(w5 w6 - -)
    const uint32_t hw[10] = {k0 | (k1 << 8) | (k2 << 16) | (k3 << 24), k2 | (k1 << 8) | (k0 << 16),
                             (k0 << 8) | (k1 << 16) | (k2 << 24), k3 | (k2 << 8) | (k1 << 16) | (k0 << 24),
                             (k0 << 16) | (k1 << 24), k2 | (k3 << 8) | (k2 << 16) | (k1 << 24), k0,
                             k0 << 24, k1 | (k2 << 8) | (k3 << 16) | (k2 << 24), k1 | (k0 << 8)};
#endif
    // umax in SGPRs: a lane-indexed a.umax[v] compiles to a vector load from
    // the kernarg segment whose vmcnt wait would also drain the patch prefetch
    int um_s[kHalfPatch + 1];
#pragma unroll
    for (int v = 0; v <= kHalfPatch; ++v) um_s[v] = __builtin_amdgcn_readfirstlane(a.umax[v]);
    // IC_Angle disc masks for the h-pass lanes: lane r holds patch row r
    // (v = r - 21); byte b of its aligned word j is column 4j + b (u = 4j + b - 21)
#if ORB_DESC_ICM_REG
    uint32_t icm[9];
    {
        const int av = lane >= 21 ? lane - 21 : 21 - lane;
        int um = -1;
#pragma unroll
        for (int k = 0; k <= kHalfPatch; ++k)
            if (av == k) um = um_s[k];
        if (lane >= kRaw) um = -1;
#pragma unroll
        for (int j = 1; j <= 9; ++j) {
            uint32_t m = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int u = 4 * j + b - 21;
                if (u >= -um && u <= um) m |= 0xffu << (8 * b);
            }
            icm[j - 1] = m;
        }
    }
#else
    // the lane's disc half-width (-1: no disc row) for masks made per use
    int um_l = -1;
    {
        const int av = lane >= 21 ? lane - 21 : 21 - lane;
#pragma unroll
        for (int k = 0; k <= kHalfPatch; ++k)
            if (av == k) um_l = um_s[k];
        if (lane >= kRaw) um_l = -1;
    }
    // bytes of 128 + umax (0x7f: no disc row), so (um_rep - |u|) has bit 7
    // set per byte exactly where |u| <= umax, with no borrow across bytes
    const uint32_t um_rep = (uint32_t)((um_l + 128) & 0xff) * 0x01010101u;
#endif
    // this wave's run of kDescSlots slots; the next valid slot's patch is
    // always in flight while the current one is described
    // grid (runs of 4 * kDescSlots slots of a frame, frames), XCD-aware order
    int bunit, bframe;
    xcd_remap((int)gridDim.x, (int)gridDim.y, bunit, bframe);
    const int lb = (bunit * kDescWpb + wv) * kDescSlots;           // frame-local slot
    const long long s_begin = (long long)bframe * a.out_total + lb;
    const int nrun = max(0, min(kDescSlots, a.out_total - lb));
    DescLane mine{};
    const bool valid = lane < nrun && desc_lane(a, s_begin + lane, mine);
    uint64_t todo = __ballot(valid);
    // two patches in flight (ORB_DESC_PF2): the current keypoint's, landed at
    // the top of its iteration, and the next one's; the register set freed by
    // the landing takes the keypoint after that, so the sets alternate and the
    // loop body is instantiated once per set
    uint32_t pv[kPVN];
#if ORB_DESC_PF2
    uint32_t pv2[kPVN];
#endif
    DescKp cur{}, nxt{};
    int jc = -1, jn = -1;
#ifdef ORB_DESC_TIMING
    const unsigned long long t_start = __builtin_amdgcn_s_memtime();
    unsigned long long tlast = t_start, d0 = 0, d1 = 0, d2 = 0, d3 = 0, d4 = 0, d5 = 0, dk = 0;
#endif
    auto take = [&](int& j, DescKp& k, uint32_t (&v)[kPVN]) {      // the next valid slot, its patch issued
        j = -1;
        if (!todo) return;
        j = __builtin_ctzll(todo);
        todo &= todo - 1;
        k = desc_pick(mine, j);
        const int x0 = (int)(k.key & 0xfff) + (kEdge - 3) - 21, y0 = (int)((k.key >> 12) & 0xfff) + (kEdge - 3) - 21;
#if ORB_DESC_ROWLOAD
        const int md = patch_mode(k.w, k.h, k.pitch, x0, y0);
        if (md) patch_issue_rows(k.img, k.pitch, k.h, md == 2 ? 0 : (x0 & ~3), y0, v);
#else
        if (patch_interior(k.w, k.h, x0, y0)) DESC_PATCH_ISSUE(k.img, k.pitch, x0, y0, v);
#endif
    };
    take(jc, cur, pv);
#if ORB_DESC_PF2
    take(jn, nxt, pv2);
#endif
    auto body = [&](uint32_t (&pvl)[kPVN]) {
        const long long s = s_begin + jc;
        const uint32_t key = cur.key;
        const int cx = (int)(key & 0xfff) + (kEdge - 3), cy = (int)((key >> 12) & 0xfff) + (kEdge - 3);
        // 1. raw 43x43 patch centred on (cx, cy), REFLECT_101 at the level border
        int sh = 0;
#if ORB_DESC_ROWLOAD
        const int md = patch_mode(cur.w, cur.h, cur.pitch, cx - 21, cy - 21);
        if (md == 1) {
            DESC_PATCH_LAND(pvl, raw);
            sh = (cx - 21) & 3;
        } else if (md == 2) {
            patch_land_rows_left(pvl, raw);
            sh = 4 + (cx - 21);
        } else if (md == 3) {
            DESC_PATCH_LAND(pvl, raw);
            sh = (cx - 21) & 3;
            // columns w (and w + 1) of the row: bytes P, P + 1 of the loaded
            // row (P = w - (x0 & ~3) <= 46) take pixels w - 2, w - 3
            if (lane < kRaw) {
                uint8_t* rr = raw + lane * kRawP;
                const int P = cur.w - ((cx - 21) & ~3);
                const uint8_t a2 = rr[P - 2], a3 = rr[P - 3];
                rr[P] = a2;
                if (P + 1 < kRawP) rr[P + 1] = a3;
            }
        } else {
            patch_border(cur.img, cur.pitch, cur.w, cur.h, cx - 21, cy - 21, raw);
        }
#else
        if (patch_interior(cur.w, cur.h, cx - 21, cy - 21)) {
            DESC_PATCH_LAND(pvl, raw);
            sh = (cx - 21) & 3;
        } else {
            patch_border(cur.img, cur.pitch, cur.w, cur.h, cx - 21, cy - 21, raw);
        }
#endif
        // refill the landed set: the keypoint after the next one (PF2), or
        // the next one (one patch in flight during this keypoint)
        int jnn = -1;
        DescKp nn{};
#if ORB_DESC_PF2
        take(jnn, nn, pvl);
#else
        take(jn, nxt, pvl);
#endif
        wave_sync();
        DESC_T(d0);
#ifdef ORB_DESC_TIMING
        ++dk;
#endif
        int m10 = 0, m01 = 0;
        float ang_deg, sb, ca;
        DESC_T(d1);
        // 3. horizontal pass (ufixedpoint16): lane r holds raw row r in registers
        //    (3 x ds_read_b128 + v_alignbyte for the column shift), splits it
        //    into u16 pixel pairs starting at even (E) and odd (O) columns and
        //    makes two outputs per packed-u16 op (every partial sum fits 16 bits:
        //    the kernel sums to <= 257); outputs 2m, 2m+1 go out as one dword
        // all 64 lanes run it (lanes past the patch repeat row 42 and rewrite
        // identical values), so the angle chain below shares its basic block
        // and is scheduled among the h-pass ops
        {
            const int rr = min(lane, kRaw - 1);
            const uint4* rowp = (const uint4*)(raw + rr * kRawP);
            const uint4 q0 = rowp[0], q1 = rowp[1], q2 = rowp[2];
            const uint32_t wd[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
            uint32_t al[11];
#pragma unroll
            for (int j = 0; j < 11; ++j) al[j] = __builtin_amdgcn_alignbyte(wd[j + 1], wd[j], (uint32_t)sh);
            // 2. IC_Angle (ORBextractor.cc:76-103) on this row of the unblurred
            //    disc: sum I and sum (u + 15) I by byte dot products, then
            //    m10 = sum u I, m01 = v sum I (integer, order-free)
            {
                uint32_t s1 = 0, sw = 0;
#pragma unroll
                for (int j = 1; j <= 9; ++j) {
                    uint32_t wgt = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const int u = 4 * j + b - 21;
                        if (u >= -kHalfPatch && u <= kHalfPatch) wgt |= (uint32_t)(u + kHalfPatch) << (8 * b);
                    }
#if ORB_DESC_ICM_REG
                    const uint32_t px = al[j] & icm[j - 1];
#else
                    // bytes with |u| <= umax(v): SWAR (um | 0x80) - |u| keeps bit 7 exactly there
                    uint32_t au = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const int u = 4 * j + b - 21;
                        au |= (uint32_t)(u < 0 ? -u : u) << (8 * b);
                    }
                    const uint32_t ge = ((um_rep - au) & 0x80808080u) >> 7;
                    const uint32_t px = al[j] & ((ge << 8) - ge);
#endif
                    s1 = __builtin_amdgcn_udot4(px, 0x01010101u, s1, false);
                    sw = __builtin_amdgcn_udot4(px, wgt, sw, false);
                }
                m10 = (int)sw - kHalfPatch * (int)s1;
                m01 = (lane - 21) * (int)s1;
            }
            m10 = wave_sum_dpp(m10);
            m01 = wave_sum_dpp(m01);
            ang_deg = fast_atan2_deg((float)m01, (float)m10);
            glibc_sincosf(deg_to_rad(ang_deg), &sb, &ca);
            const u16x2 K0 = {(unsigned short)k0, (unsigned short)k0}, K1 = {(unsigned short)k1, (unsigned short)k1};
            const u16x2 K2 = {(unsigned short)k2, (unsigned short)k2}, K3 = {(unsigned short)k3, (unsigned short)k3};
            // E(k) = (p[2k], p[2k+1]), O(k) = (p[2k+1], p[2k+2]); two halves of
            // the row keep at most ~26 pairs live
            auto Ep = [&](int k) {
                return as_u16x2(__builtin_amdgcn_perm(0u, al[k >> 1], (k & 1) ? 0x0c030c02u : 0x0c010c00u));
            };
            auto Op = [&](int k) {
                return (k & 1) ? as_u16x2(__builtin_amdgcn_perm(al[(k >> 1) + 1], al[k >> 1], 0x0c040c03u))
                               : as_u16x2(__builtin_amdgcn_perm(0u, al[k >> 1], 0x0c020c01u));
            };
            auto half = [&](auto mlo_c, auto mhi_c) {
                constexpr int mlo = decltype(mlo_c)::value, mhi = decltype(mhi_c)::value;
                u16x2 E[mhi - mlo + 3], O[mhi - mlo + 2];
#pragma unroll
                for (int k = 0; k < mhi - mlo + 3; ++k) E[k] = Ep(mlo + k);
#pragma unroll
                for (int k = 0; k < mhi - mlo + 2; ++k) O[k] = Op(mlo + k);
#pragma unroll
                for (int m = 0; m < mhi - mlo; ++m) {
                    const u16x2 h = K0 * (E[m] + E[m + 3]) + K1 * (O[m] + O[m + 2]) + K2 * (E[m + 1] + E[m + 2]) +
                                    K3 * O[m + 1];
                    // columns 2(mlo+m) and 2(mlo+m)+1 of this row (the last pair's
                    // second column, 37, lands in the pad)
                    hb[(2 * (mlo + m)) * kHbT + rr] = h.x;
                    hb[(2 * (mlo + m) + 1) * kHbT + rr] = h.y;
                }
            };
#if ORB_DESC_HMFMA
            (void)half;
            {
                const v4i_t bias = {hbias, hbias, hbias, hbias};
                // slice 3 (k >= 48) meets zero weights: it takes slice 2's bytes
                const int ks = 16 * min(lane >> 4, 2);
                const uint32_t shb = (uint32_t)sh;
#pragma unroll
                for (int mb = 0; mb < 3; ++mb) {
                    // the slice's 16 bytes from byte ks + sh of the row: one
                    // 16-byte read, the next dword (slice 2: bytes 48.. meet zero
                    // weights, so its own last dword) and 4 v_alignbyte
                    const int row = min(hm_row0(mb) + (lane & 15), kRaw - 1);
                    const uint8_t* rp = raw + row * kRawP + ks;
                    const uint4 q = *(const uint4*)rp;
                    const uint32_t q4 = *(const uint32_t*)(rp + (ks < 32 ? 16 : 12));
                    const v4i_t A = {(int)(__builtin_amdgcn_alignbyte(q.y, q.x, shb) ^ 0x80808080u),
                                     (int)(__builtin_amdgcn_alignbyte(q.z, q.y, shb) ^ 0x80808080u),
                                     (int)(__builtin_amdgcn_alignbyte(q.w, q.z, shb) ^ 0x80808080u),
                                     (int)(__builtin_amdgcn_alignbyte(q4, q.w, shb) ^ 0x80808080u)};
                    const int r0 = hm_row0(mb) + 4 * (lane >> 4);
#pragma unroll
                    for (int nb = 0; nb < kHmNb; ++nb) {
                        const v4i_t acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, Bm[nb], bias, 0, 0, 0);
                        // rows r0..r0+3 of column x as u16
                        const int x = hm_col0(nb) + (lane & 15);
                        const uint32_t lo = __builtin_amdgcn_perm((uint32_t)acc[1], (uint32_t)acc[0], 0x05040100u);
                        const uint32_t hi = __builtin_amdgcn_perm((uint32_t)acc[3], (uint32_t)acc[2], 0x05040100u);
                        if ((kHbT / 2) % 2 == 0) {
                            *(uint2*)(hb + x * kHbT + r0) = make_uint2(lo, hi);
                        } else {
                            // odd dword pitch: the pair is 4-byte aligned only (ds_write2_b32)
                            uint32_t* d32 = (uint32_t*)(hb + x * kHbT + r0);
                            d32[0] = lo;
                            d32[1] = hi;
                        }
                    }
                }
            }
#elif ORB_DESC_HDOT4
            // output x = 4 j + b takes raw columns x .. x + 6: bytes b.. of
            // al[j], al[j + 1] and (b >= 2) al[j + 2], one v_dot4_u32_u8 per
            // word with the 7 weights placed at the matching bytes (every sum
            // <= 257 * 255 < 2^16, the u16 of ufixedpoint16); no pair
            // unpacking, 2.5 dot4 per output
            (void)half;
#pragma unroll
            for (int x = 0; x < kBl; ++x) {
                const int j = x >> 2, b = x & 3;
                uint32_t h;
                if (b == 0) h = __builtin_amdgcn_udot4(al[j + 1], hw[1], __builtin_amdgcn_udot4(al[j], hw[0], 0u, false), false);
                else if (b == 1) h = __builtin_amdgcn_udot4(al[j + 1], hw[3], __builtin_amdgcn_udot4(al[j], hw[2], 0u, false), false);
                else if (b == 2)
                    h = __builtin_amdgcn_udot4(al[j + 2], hw[6], __builtin_amdgcn_udot4(al[j + 1], hw[5],
                                               __builtin_amdgcn_udot4(al[j], hw[4], 0u, false), false), false);
                else
                    h = __builtin_amdgcn_udot4(al[j + 2], hw[9], __builtin_amdgcn_udot4(al[j + 1], hw[8],
                                               __builtin_amdgcn_udot4(al[j], hw[7], 0u, false), false), false);
                hb[x * kHbT + rr] = (uint16_t)h;
            }
#else
            half(std::integral_constant<int, 0>{}, std::integral_constant<int, 10>{});
            __builtin_amdgcn_sched_barrier(0);
            half(std::integral_constant<int, 10>{}, std::integral_constant<int, (kBl + 1) / 2>{});
#endif
        }
        DESC_T(d2);
        wave_sync();
        DESC_T(d3);
        // 4. rBRIEF tests: the vertical pass (ufixedpoint32 + rounding) evaluated
        //    only at the 512 sample points, hb rows R..R+6 at blurred column C,
        //    blurred centre (18, 18)
        int nib = 0;
#pragma unroll ORB_Q_UNROLL
        for (int q = 0; q < 4; ++q) {
            int val[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
#if ORB_DESC_PATF
                const float x = pfx[2 * q + e], y = pfy[2 * q + e];
#else
                const float x = (float)(int)(int8_t)(patw[q] >> (16 * e));
                const float y = (float)(int)(int8_t)(patw[q] >> (16 * e + 8));
#endif
                int r, c;
                brief_offset(x, y, sb, ca, FMA, r, c);
                // the 7 vertical taps are rows 18+r .. 24+r of column 18+c:
                // contiguous u16 from index s0, inside the 4 dwords from the
                // even index at or below s0; for an odd s0 the dwords are
                // realigned by 16 bits (v_alignbit), so one set of dot2 weights
                // serves both parities
                const int s0 = (int)__umul24(18 + c, kHbT) + 18 + r;
                const uint32_t* dw = (const uint32_t*)hb + (s0 >> 1);
                const uint32_t D0 = dw[0], D1 = dw[1], D2 = dw[2], D3 = dw[3];
                const uint32_t sh = (uint32_t)(s0 & 1) << 4;
                const uint32_t E0 = __builtin_amdgcn_alignbit(D1, D0, sh), E1 = __builtin_amdgcn_alignbit(D2, D1, sh);
                const uint32_t E2 = __builtin_amdgcn_alignbit(D3, D2, sh), E3 = __builtin_amdgcn_alignbit(0u, D3, sh);
                const uint32_t acc = __builtin_amdgcn_udot2(
                    as_u16x2(E3), as_u16x2(W3e),
                    __builtin_amdgcn_udot2(
                        as_u16x2(E2), as_u16x2(W2e),
                        __builtin_amdgcn_udot2(as_u16x2(E1), as_u16x2(W1e),
                                               __builtin_amdgcn_udot2(as_u16x2(E0), as_u16x2(W0e), 0u, false),
                                               false),
                        false),
                    false);
                val[e] = (int)min(255u, (acc + 32768u) >> 16);   // saturate_cast<uchar>
            }
            nib |= (val[0] < val[1]) << q;
        }
        DESC_T(d4);
        const int hi = __shfl_down(nib, 1, kWave);
        uint8_t* d = a.sdesc + s * 32;
        if ((lane & 1) == 0) d[lane >> 1] = (uint8_t)(nib | (hi << 4));
        if (lane == 0) a.angle[s] = ang_deg;
        jc = jn;
        cur = nxt;
#if ORB_DESC_PF2
        jn = jnn;
        nxt = nn;
#else
        (void)jnn; (void)nn;
#endif
        wave_sync();
        DESC_T(d5);
    };
    while (jc >= 0) {
        body(pv);
#if ORB_DESC_PF2
        if (jc < 0) break;
        body(pv2);
#endif
    }
#ifdef ORB_DESC_TIMING
    if (lane == 0) {
        const unsigned long long tv[8] = {d0, d1, d2, d3, d4, d5, dk, __builtin_amdgcn_s_memtime() - t_start};
#pragma unroll
        for (int k = 0; k < 8; ++k) atomicAdd(&g_desc_t[(bunit * 4 + wv + bframe * 61) & 1023][k], tv[k]);
    }
#endif
}

// ---------------------------------------------------------------------------
// k_debug_math: the device compile of k_describe's scalar math over whole
// input domains, as chunk hashes (orbx_debug_math; host side: the oracle with
// the system libm, tests/test_gpu_math.py).  One workgroup per chunk.
//   what 0: glibc_sincosf on every float bit pattern i (radians)
//   what 1: deg_to_rad + glibc_sincosf + the 512 brief_offset()s of every
//           float degree angle i
//   what 2: fast_atan2_deg on the integer moment pairs atan_pair(i)
// ---------------------------------------------------------------------------
template <int WHAT>
__global__ __launch_bounds__(256) void k_debug_math(long long begin, long long end, int chunk_log2, int fused,
                                                    unsigned long long* hashes) {
    __shared__ unsigned long long part[4];
    const long long nchunks = ((end - begin) + (1ll << chunk_log2) - 1) >> chunk_log2;
    for (long long ck = blockIdx.x; ck < nchunks; ck += gridDim.x) {
        const long long c0 = begin + (ck << chunk_log2), c1 = min(end, c0 + (1ll << chunk_log2));
        unsigned long long acc = 0;
        for (long long i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
            uint32_t e;
            if (WHAT == 0) {
                float s, c;
                glibc_sincosf(__builtin_bit_cast(float, (uint32_t)i), &s, &c);
                e = f32_bits(s) ^ (f32_bits(c) * 0x9E3779B9u);
            } else if (WHAT == 1) {
                float sb, ca;
                glibc_sincosf(deg_to_rad(__builtin_bit_cast(float, (uint32_t)i)), &sb, &ca);
                e = 0;
                for (int k = 0; k < 512; ++k) {
                    int r, c;
                    brief_offset((float)c_pattern[2 * k], (float)c_pattern[2 * k + 1], sb, ca, fused != 0, r, c);
                    e = offsets_word(e, k, r, c);
                }
            } else {
                float y, x;
                atan_pair((uint64_t)i, y, x);
                e = f32_bits(fast_atan2_deg(y, x));
            }
            acc += math_mix(e, (uint64_t)i);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, kWave);
        if (lane_id() == 0) part[wave_id()] = acc;
        __syncthreads();
        if (threadIdx.x == 0) hashes[ck] = part[0] + part[1] + part[2] + part[3];
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// k_assemble: ORBextractor::operator() output loop (ORBextractor.cc:1105-1167):
// levels in order, keypoints in quadtree list order; pt *= scale for level>0;
// x in [lap0, lap1] goes to the tail in reverse, others to the head; returns
// monoIndex.  One workgroup per frame.
// ---------------------------------------------------------------------------
struct AsmArgs {
    const LevelDev* lv;
    const uint32_t* qt_key;
    const int* qt_n;
    const float* angle;
    const uint8_t* sdesc;
    int out_total, L;
    float lap0, lap1;
    orb_keypoint* kps;
    uint8_t* desc;
    int cap;
    int32_t* n_out;
    int32_t* mono_out;
};

__global__ __launch_bounds__(ORB_ASM_THREADS) void k_assemble(AsmArgs a) {
    __shared__ int lvl_start[kMaxLevels + 1];
    __shared__ int lvl_base[kMaxLevels];
    __shared__ float lvl_scale[kMaxLevels];
    __shared__ float lvl_patch[kMaxLevels];
    __shared__ int tmp[ORB_ASM_THREADS / kWave + 1];   // block_excl_scan: a word a wave + the total
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    int* inlap = (int*)smem;                    // per keypoint, scanned
    const int f = blockIdx.x, tid = threadIdx.x, T = blockDim.x;
    // the level starts by one DPP scan of the levels' counts (their loads in
    // flight together: a thread-0 loop waited on each), and the level fields
    // the keypoints need, in LDS
    if (tid < kWave) {
        const int c = tid < a.L ? a.qt_n[f * a.L + tid] : 0;
        const int incl = wave_incl_scan_dpp(c);
        if (tid < a.L) {
            lvl_start[tid] = incl - c;
            lvl_base[tid] = a.lv[tid].out_base;
            lvl_scale[tid] = a.lv[tid].scale;
            lvl_patch[tid] = (float)a.lv[tid].patch;
        }
        if (tid == a.L - 1) lvl_start[a.L] = incl;
        if (a.L == 0 && tid == 0) lvl_start[0] = 0;
    }
    __syncthreads();
    const int total = lvl_start[a.L];
    // the last level whose start is <= g (empty levels share their start with
    // the next one): a fixed 5-step search (kMaxLevels = 32), so the keypoint
    // loops below unroll (a data-dependent while loop kept them rolled and put
    // their per-keypoint arrays in scratch)
    static_assert(kMaxLevels == 32, "5 search steps");
    const int L = a.L;
    auto locate = [&](int g, int& l, int& p) {
        l = 0;
#pragma unroll
        for (int step = 16; step >= 1; step >>= 1)
            if (l + step < L && g >= lvl_start[l + step]) l += step;
        p = g - lvl_start[l];
    };
    const long long fo = (long long)f * a.out_total;
    constexpr int kU = 4;   // keypoints a thread in flight
    auto xkey = [&](int g, int& l) {
        int p;
        locate(min(g, total - 1), l, p);
        return a.qt_key[fo + lvl_base[l] + p];
    };
    auto flag = [&](int g, int l, uint32_t key) {
        float x = (float)((int)(key & 0xfff) + (kEdge - 3));
        if (l != 0) x *= lvl_scale[l];
        if (g < total) inlap[g] = (x >= a.lap0 && x <= a.lap1) ? 1 : 0;
    };
    for (int g0 = tid; g0 < total; g0 += kU * T) {
        int l0, l1, l2, l3;
        const uint32_t q0 = xkey(g0, l0), q1 = xkey(g0 + T, l1), q2 = xkey(g0 + 2 * T, l2), q3 = xkey(g0 + 3 * T, l3);
        flag(g0, l0, q0);
        flag(g0 + T, l1, q1);
        flag(g0 + 2 * T, l2, q2);
        flag(g0 + 3 * T, l3, q3);
    }
    __syncthreads();
    // keep the flags: recompute them after the scan from the scanned values
    const int nlap = block_excl_scan(inlap, total, tmp);
    // four keypoints' loads issued before any of their stores (named values,
    // not arrays: an array indexed in a rolled loop went to scratch)
    struct KpIn {
        uint32_t key;
        float ang;
        uint4 d0, d1;
        int l, g;
    };
    auto load = [&](int g) {
        KpIn k;
        k.g = g;
        int p;
        locate(min(g, total - 1), k.l, p);
        const long long src = fo + lvl_base[k.l] + p;
        k.key = a.qt_key[src];
        k.ang = a.angle[src];
        const uint4* s4 = (const uint4*)(a.sdesc + src * 32);
        k.d0 = s4[0];
        k.d1 = s4[1];
        return k;
    };
    auto store = [&](const KpIn& k) {
        if (k.g >= total) return;
        const int l = k.l;
        float x = (float)((int)(k.key & 0xfff) + (kEdge - 3));
        float y = (float)((int)((k.key >> 12) & 0xfff) + (kEdge - 3));
        if (l != 0) { x *= lvl_scale[l]; y *= lvl_scale[l]; }
        const bool in = x >= a.lap0 && x <= a.lap1;
        const int before_lap = inlap[k.g];
        const int dst = in ? total - 1 - before_lap : k.g - before_lap;
        orb_keypoint kp;
        kp.x = x; kp.y = y;
        kp.size = lvl_patch[l];
        kp.angle = k.ang;
        kp.response = (float)(k.key >> 24);
        kp.octave = l;
        kp.class_id = -1;
        if (dst < a.cap) {
            a.kps[(long long)f * a.cap + dst] = kp;
            uint4* d4 = (uint4*)(a.desc + ((long long)f * a.cap + dst) * 32);
            d4[0] = k.d0;
            d4[1] = k.d1;
        }
    };
    static_assert(kU == 4, "four named keypoints");
    for (int g0 = tid; g0 < total; g0 += kU * T) {
        const KpIn k0 = load(g0), k1 = load(g0 + T), k2 = load(g0 + 2 * T), k3 = load(g0 + 3 * T);
        store(k0);
        store(k1);
        store(k2);
        store(k3);
    }
    if (tid == 0) {
        a.n_out[f] = total;
        a.mono_out[f] = total - nlap;
    }
}

// ---------------------------------------------------------------------------
// Host orchestration
// ---------------------------------------------------------------------------
// k_quadtree's launch LDS (the largest level that fits kLdsMax) and the
// global slice size of the levels that do not (0: none)
#ifndef ORB_QT_GLOBAL_NODES
#define ORB_QT_GLOBAL_NODES 0   // 1: every level's node arrays in global scratch (no LDS: co-residency A/B)
#endif
static void qt_lds_split(const Plan& P, size_t& lds, size_t& gstride) {
    lds = 0;
    gstride = 0;
    for (const LevelDev& d : P.lv) {
        const size_t b = qt_scratch_bytes(d.out_cap + 8, d.ncells);
        if (b <= (size_t)kLdsMax && !ORB_QT_GLOBAL_NODES) lds = std::max(lds, b);
        else gstride = std::max(gstride, (b + 255) & ~size_t(255));
    }
}

// k_fast_cells launch geometry of a range of every frame's cells
struct FastGroup {
    int roi_max = 0, rows_max = 0, nd_max = 0, win_max = 0, win_pix_max = 0, item_max = 0;
};
static FastGroup fast_group(const Plan& P, int cb, int ce) {
    FastGroup G;
    for (int i = cb; i < ce; ++i) {
        const CellDev& c = P.cells[i];
        const int nd = ((c.x0 & 3) + c.cols + 3) >> 2, ww = std::max(0, c.cols - 6), wh = std::max(0, c.rows - 6);
        // + 16: the pre-test reads up to 2 dwords past the last row's window
        G.roi_max = std::max(G.roi_max, 4 * c.rows * nd + 16);
        G.rows_max = std::max(G.rows_max, c.rows);
        G.nd_max = std::max(G.nd_max, nd);
        G.win_max = std::max(G.win_max, (ww + 2) * (wh + 2));
        G.win_pix_max = std::max(G.win_pix_max, ww * wh);
        const int X0 = (c.x0 & 3) + 3, j0 = X0 >> 2, ndw = ww ? ((X0 + ww - 1) >> 2) - j0 + 1 : 0;
        G.item_max = std::max(G.item_max, wh * ((ndw + 1) >> 1));
    }
    return G;
}
// fetch row width (dwords) and loads per lane: <16, 12> takes ROIs of at most
// 16 dwords by 48 rows (W = 35 cells are < 70 px: nd <= 19 and rows < 76
// always fit <32, 40>); rp: the fixed LDS pitch of the ROIs (dwords), 0: per cell
static void (*fast_kernel(const FastGroup& G, bool want_bm, int& rp, bool& bm))(FastArgs) {
    const int ndm = G.nd_max, rm = G.rows_max;
    rp = 0;
    // bitmap (BM) forms exist for ROIs of <= 64 rows and <= 16 dwords
    bm = want_bm && rm <= 64 && ndm <= 16;
#if ORB_FAST_FIXED_PITCH
    if (ndm <= 11 && rm <= 64) {
        rp = 11;
        return rm <= 48 ? (bm ? k_fast_cells<16, 12, 11, true> : k_fast_cells<16, 12, 11, false>)
                        : (bm ? k_fast_cells<16, 16, 11, true> : k_fast_cells<16, 16, 11, false>);
    }
    if (ndm <= 13 && rm <= 64) {
        rp = 13;
        return rm <= 48 ? (bm ? k_fast_cells<16, 12, 13, true> : k_fast_cells<16, 12, 13, false>)
                        : (bm ? k_fast_cells<16, 16, 13, true> : k_fast_cells<16, 16, 13, false>);
    }
#endif
    if (ndm <= 16 && rm <= 48) return bm ? k_fast_cells<16, 12, 0, true> : k_fast_cells<16, 12, 0, false>;
    if (ndm <= 16 && rm <= 64) return bm ? k_fast_cells<16, 16, 0, true> : k_fast_cells<16, 16, 0, false>;
    if (ndm <= 16 && rm <= 80) return k_fast_cells<16, 20, 0, false>;
    if (ndm <= 32 && rm <= 48) return k_fast_cells<32, 24, 0, false>;
    if (ndm <= 32 && rm <= 80) return k_fast_cells<32, 40, 0, false>;
    return nullptr;
}
static void fast_lds_layout(const FastGroup& G, int rp, FastArgs& fa) {
    fa.roi_max = (std::max(G.roi_max, 4 * G.rows_max * rp + 16) + 15) & ~15;
    const int il = ORB_FAST_EMIT == 1 ? (4 * G.item_max + 15) & ~15 : 0;
    fa.win_max = (std::max(G.win_max, ORB_FAST_ILIST_IN_MAP ? il : 0) + 15) & ~15;
    // NMS ballots only for the separate output pass
    fa.kmask_bytes = ORB_FAST_FUSED_OUT ? 0 : ((G.win_pix_max + kWave - 1) / kWave * 8 + 15) & ~15;
    // the list's capacity: what the LDS budget of ORB_FAST_WAVES_CU waves a CU
    // leaves after the ROI and the map (>= 256 entries), never more than a
    // window; ORB_OPT_FAST_CAND_CAP n > 0 (test hook) caps it at n - 1
    int cap = G.win_pix_max;
    if (kFastDense) {
        const int budget = (int)(kCuLds / ORB_FAST_WAVES_CU) & ~15;
        cap = std::min(cap, std::max(256, (budget - fa.roi_max - fa.win_max) / 2));
        const int opt = debug_opt(ORB_OPT_FAST_CAND_CAP);
        if (opt > 0) cap = std::min(cap, opt - 1);
    }
    fa.cand_cap = cap;
    fa.cand_bytes = std::max(16, (2 * cap + 15) & ~15);
    fa.ilist_bytes = ORB_FAST_ILIST_IN_MAP ? 0 : il;
}
static size_t fast_wave_lds(const FastArgs& fa) {
    return (size_t)(fa.roi_max + fa.win_max + fa.cand_bytes + fa.kmask_bytes + fa.ilist_bytes);
}
#ifndef ORB_FAST_LDS_PAD
#define ORB_FAST_LDS_PAD 0   // occupancy probe (tools only): extra LDS per block
#endif
// Frames [f0, f0+B) of the batch: every per-frame work buffer is addressed
// through pointers offset by f0, so disjoint frame ranges can run on separate
// streams without sharing scratch.
static int run_pipeline(orbx_handle* hd, int f0, int B, const uint8_t* d_frames, long long fstride, int pitch0,
                        float lap0, float lap1, orb_keypoint* d_kps, uint8_t* d_desc, int cap, int32_t* d_n,
                        int32_t* d_mono, hipStream_t st) {
    const Plan& P0 = hd->plan;
    const int L = P0.L;
    Plan P;                         // shallow view: host tables + offset device pointers (never released)
    P.lv = P0.lv; P.cells = P0.cells; P.pyr_bytes = P0.pyr_bytes; P.ncells = P0.ncells;
    P.slot_total = P0.slot_total; P.out_total = P0.out_total; P.roi_rows_max = P0.roi_rows_max; P.roi_max = P0.roi_max;
    P.roi_nd_max = P0.roi_nd_max; P.win_max = P0.win_max; P.max_level_cells = P0.max_level_cells;
    P.max_out_cap = P0.max_out_cap; P.xmax = P0.xmax; P.tab_off = P0.tab_off; P.L = L; P.pgroups = P0.pgroups;
    P.d_tab = P0.d_tab; P.d_lv = P0.d_lv; P.d_cells = P0.d_cells; P.d_slot_level = P0.d_slot_level;
    const long long F = f0;
    P.d_pyr = P0.d_pyr + F * P0.pyr_bytes;
    P.d_bm = P0.d_bm ? P0.d_bm + F * P0.bm_bytes : nullptr;
    P.d_cell_count = P0.d_cell_count + F * P0.ncells;
    P.d_cell_keys = P0.d_cell_keys + F * P0.slot_total;
    P.d_key_scr = P0.d_key_scr + F * P0.slot_total;
    P.d_knode = P0.d_knode + F * P0.slot_total;
    P.d_kq = P0.d_kq + F * P0.slot_total;
    P.d_qt_key = P0.d_qt_key + F * P0.out_total;
    P.d_qt_n = P0.d_qt_n + F * L;
    P.d_qt_ovf = P0.d_qt_ovf + F * L;
    P.d_angle = P0.d_angle + F * P0.out_total;
    P.d_sdesc = P0.d_sdesc + F * P0.out_total * 32;
    d_frames += F * fstride;
    d_kps += F * cap;
    d_desc += F * cap * 32;
    d_n += F;
    d_mono += F;
    std::vector<hipEvent_t> marks;
    int stage_no = 0;
    auto mark = [&]() {
        // caller's pipeline events (orbx_set_stage_event): recorded after stage k
        hipEvent_t ue = hd->stage_ev[std::min(stage_no++, 5)];
        if (ue) (void)hipEventRecord(ue, st);
        if (!hd->profiling) return;
        if (hd->ev_next >= hd->ev_pool.size()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return;
            hd->ev_pool.push_back(e);
        }
        hipEvent_t e = hd->ev_pool[hd->ev_next++];
        (void)hipEventRecord(e, st);
        marks.push_back(e);
    };
    mark();
    // pyramid
    const int pm = hd->pyr_mode;
    const bool use_stream = P0.ps.ok && (pm == 2 || (pm == 0 && B >= kPyrStreamMinFrames));
    hd->pyr_last = use_stream ? 2 : 1;
    if (use_stream) {
        const PyrStream& S = P0.ps;
        PyrStreamArgs pa;
        pa.src = d_frames; pa.src_fstride = fstride; pa.src_pitch = pitch0;
        const uintptr_t al = (uintptr_t)d_frames | (uintptr_t)pitch0 | (uintptr_t)(B > 1 ? fstride : 0);
        pa.load_mode = (al & 15) == 0 ? 16 : ((al & 3) == 0 ? 4 : 1);
        pa.pyr = P.d_pyr; pa.pyr_fstride = P.pyr_bytes;
        pa.tab = P0.d_ps_tab;
        pa.tab_u4 = S.tab_u4; pa.lev_u4 = S.lev_u4; pa.steps_u4 = S.steps_u4; pa.L = L; pa.E = S.E;
        pa.nsteps = S.nsteps; pa.nchunks = S.nchunks; pa.K0 = S.K0;
        pa.h0 = P.lv[0].h; pa.w0 = P.lv[0].w; pa.nframes = B;
        pa.ring0_dw = S.ring_dw[0]; pa.ring0_rows = S.ring_rows[0]; pa.ring0_pitch = S.ring_pitch[0];
        pa.cnt_dw = S.cnt_dw;
        pa.pretest = S.pretest;
        pa.ini_th = std::min(std::max(hd->prm.ini_th_fast, 0), 255);
        pa.bm = P.d_bm; pa.bm_fstride = P0.bm_bytes;
        ORB_LAUNCH(S.pretest ? k_pyr_stream<true> : k_pyr_stream<false>, dim3(B), dim3(1024), S.lds_bytes, st, pa);
    } else {
        for (const PyrGroup& g : P.pgroups) {
            PyrArgs pa;
            if (g.la == 0) {
                pa.src = d_frames; pa.src_fstride = fstride; pa.src_pitch = pitch0;
            } else {
                pa.src = P.d_pyr + P.lv[g.la].off; pa.src_fstride = P.pyr_bytes; pa.src_pitch = P.lv[g.la].pitch;
            }
            const uintptr_t al = (uintptr_t)pa.src | (uintptr_t)pa.src_pitch | (uintptr_t)(B > 1 ? pa.src_fstride : 0);
            pa.load_mode = (al & 15) == 0 ? 16 : ((al & 3) == 0 ? 4 : 1);
            pa.pyr = P.d_pyr; pa.pyr_fstride = P.pyr_bytes;
            pa.lv = P.d_lv; pa.band = P0.d_pband + g.band_off;
            pa.xs = P0.d_pxs; pa.xw = P0.d_pxw; pa.yt = P0.d_pyt;
            pa.la = g.la; pa.lb = g.lb; pa.nb = g.nb; pa.nframes = B; pa.lds_b = g.lds_a;
            pa.lds_x = g.lds_a + g.lds_b; pa.lds_y = pa.lds_x + g.lds_x;
            const unsigned nwg = (unsigned)((B + 7) / 8 * 8 * g.nb);
            ORB_LAUNCH(k_pyramid, dim3(nwg), dim3(256), pyr_group_lds(g), st, pa);
        }
    }
    mark();
    int kern[7];
    {
        // every tap < 128: k_describe's matrix-core horizontal pass takes them as i8
        static const int ked[7] = {18, 34, 48, 56, 48, 34, 18}, kleg[7] = {18, 34, 49, 55, 49, 34, 18};
        for (int t = 0; t < 7; ++t) kern[t] = hd->prm.blur_variant == 1 ? kleg[t] : ked[t];
    }
    // FAST cells
    FastArgs fa;
    fa.in = d_frames; fa.in_fstride = fstride; fa.in_pitch = pitch0;
    fa.pyr = P.d_pyr; fa.pyr_fstride = P.pyr_bytes;
    fa.lv = P.d_lv; fa.cells = P.d_cells; fa.ncells = P.ncells;
    fa.cell_count = P.d_cell_count; fa.cell_keys = P.d_cell_keys; fa.slot_total = P.slot_total;
    fa.ini_th = std::min(std::max(hd->prm.ini_th_fast, 0), 255);
    fa.min_th = std::min(std::max(hd->prm.min_th_fast, 0), 255);
    // the iniThFAST candidates come from k_pyr_stream's fused pre-test when it
    // ran (BM forms); otherwise k_fast_cells pre-tests the landed ROI itself
    bool bm = use_stream && P0.ps.pretest && P.d_bm;
    fa.bm_fstride = P0.bm_bytes;
    // A wave's LDS is sized for the largest cell of the plan and sets
    // k_fast_cells' occupancy: 17-18 waves a CU at 752x480 (8.7 KB a wave;
    // 16 -> 14 -> 12 waves a CU cost 6 % and 21 %).  Launching the tall-celled levels 5-7
    // apart (the rest at 20 waves a CU) was measured: alone they are a 55 us
    // tail, on a side stream their long waves slow the main launch
    // (profiles/r04/fast_occupancy).
    {
        const FastGroup G = fast_group(P0, 0, P0.ncells);
        int rp = 0;
        void (*kfast)(FastArgs) = fast_kernel(G, bm, rp, bm);
        if (!kfast) return ORB_ERR_UNSUPPORTED;
        // the bitmap is the candidate source only if a bitmap form was chosen
        // (fast_kernel falls back to the ROI pre-test beyond 64 rows)
        hd->bm_last = bm;
        fa.bm = bm ? P.d_bm : nullptr;
        fast_lds_layout(G, rp, fa);
        fa.cell_begin = 0;
        fa.cell_end = P0.ncells;
        const size_t flds = fast_wave_lds(fa) * kFastWpb + ORB_FAST_LDS_PAD;
        fa.nframes = B;
        const dim3 fgrid((P0.ncells + kFastWpb * kCellsPerWave - 1) / (kFastWpb * kCellsPerWave), B);
        if (P0.ncells > 0)                        // (every level under 67 px: no FAST cells at all)
            ORB_LAUNCH(kfast, fgrid, dim3(kWave * kFastWpb), flds, st, fa);
    }
    mark();
    // quadtree
    QtArgs qa;
    qa.lv = P.d_lv; qa.cell_count = P.d_cell_count; qa.cell_keys = P.d_cell_keys;
    qa.key_scr = P.d_key_scr; qa.knode = P.d_knode; qa.kq = P.d_kq;
    qa.ncells_total = P.ncells; qa.slot_total = P.slot_total;
    qa.qt_key = P.d_qt_key; qa.qt_n = P.d_qt_n; qa.out_total = P.out_total; qa.L = L;
    {
        size_t qlds, qgs;
        qt_lds_split(P0, qlds, qgs);
        qa.lds_bytes = (int)qlds;
        qa.gscr = P0.d_qt_gscr ? P0.d_qt_gscr + F * L * (long long)qgs : nullptr;
        qa.gscr_stride = (long long)qgs;
        if (qgs && !qa.gscr) return ORB_ERR_DEVICE;
#if ORB_QT_LEVEL_MAJOR
        const dim3 qg(B, L);
#else
        const dim3 qg(L, B);
#endif
        qa.qt_ovf = P.d_qt_ovf;
        qa.fixup = 0;
        // k_quadtree (4 waves per (frame, level)) by default; ORB_OPT_QT_FORM
        // >= 1 selects k_quadtree_w (one wave per (frame, level)) where the
        // plan keeps every level's node arrays in LDS and the one-wave layout
        // fits kQwLdsMax.  Same-box A/B: the one-wave form is
        // no faster on the 256-frame batch (96-105 vs 92-101 us; its level-0
        // wave is a 170k-cycle latency chain) and slower on one frame (70 vs
        // 50 us), and C2 frames reach 1,612 level-0 keys, past its register
        // capacity (the fixup path)
        const int form = debug_opt(ORB_OPT_QT_FORM);
        int ncm = 0, ncells_m = 0;
        for (const LevelDev& d : P0.lv) {
            ncm = std::max(ncm, d.out_cap + 8);
            ncells_m = std::max(ncells_m, d.ncells);
        }
        const int kcap = form >= 2 ? std::min(form - 2, 64 * kQwKpl) : 64 * kQwKpl;
        const size_t qwl = qw_lds_bytes(ncm, ncells_m, 64 * kQwKpl);   // (key cells at swizzled slots of all 64 KPL)
        if (form >= 1 && !qgs && qwl <= kQwLdsMax && ncells_m < 65536) {
            qa.qw_nc = ncm;
            qa.qw_kcap = kcap;
            ORB_LAUNCH(k_quadtree_w<kQwKpl>, dim3(B, L), dim3(kWave), qwl, st, qa);
            // the levels with more keys than kcap (flagged), by k_quadtree
            qa.fixup = 1;
            ORB_LAUNCH(k_quadtree<false>, qg, dim3(ORB_QT_THREADS), qlds, st, qa);
        } else {
            ORB_LAUNCH(qgs ? k_quadtree<true> : k_quadtree<false>, qg, dim3(ORB_QT_THREADS), qlds, st, qa);
        }
    }
    mark();
    // describe
    DescArgs da;
    da.in = d_frames; da.in_fstride = fstride; da.in_pitch = pitch0;
    da.pyr = P.d_pyr; da.pyr_fstride = P.pyr_bytes;
    for (int t = 0; t < 7; ++t) da.kern[t] = kern[t];
    da.lv = P.d_lv; da.qt_key = P.d_qt_key; da.qt_n = P.d_qt_n;
    da.angle = P.d_angle; da.sdesc = P.d_sdesc; da.out_total = P.out_total; da.L = L;
    da.fma = hd->prm.fma_sampling != 0;
    for (int v = 0; v < 16; ++v) da.umax[v] = hd->umax[v];
    da.slot_level = P.d_slot_level;
    da.nslots = (long long)B * P.out_total;
    const dim3 dgrid((unsigned)((P.out_total + kDescWpb * kDescSlots - 1) / (kDescWpb * kDescSlots)), (unsigned)B);
    ORB_LAUNCH(da.fma ? k_describe<true> : k_describe<false>, dgrid, dim3(kWave * kDescWpb), 0, st, da);
    mark();
    // assemble
    AsmArgs aa;
    aa.lv = P.d_lv; aa.qt_key = P.d_qt_key; aa.qt_n = P.d_qt_n; aa.angle = P.d_angle; aa.sdesc = P.d_sdesc;
    aa.out_total = P.out_total; aa.L = L; aa.lap0 = lap0; aa.lap1 = lap1;
    aa.kps = d_kps; aa.desc = d_desc; aa.cap = cap; aa.n_out = d_n; aa.mono_out = d_mono;
    ORB_LAUNCH(k_assemble, dim3(B), dim3(ORB_ASM_THREADS), (size_t)P.out_total * 4 + 64, st, aa);
    mark();
    if (hd->profiling) hd->ev_calls.push_back(marks);
    ORB_CHECK(hipGetLastError());
    return ORB_OK;
}

// Frames [fb, fb+B) of a batch whose base pointers are given (frame fb also
// uses scratch/pyramid slot fb, so separate runs of one batch never share
// slots).  Splits the range into hd->nsub frame ranges on private non-blocking
// streams that fork from and join back into the caller's stream.  The quadtree,
// pyramid and assemble kernels are latency bound (one block per frame-level,
// barrier heavy); running them beside the VALU-bound FAST/describe kernels
// of the other range fills the CUs they leave idle.
static int run_batched(orbx_handle* hd, int fb, int B, const uint8_t* d_frames, long long fstride, int pitch0,
                       float lap0, float lap1, orb_keypoint* d_kps, uint8_t* d_desc, int cap, int32_t* d_n,
                       int32_t* d_mono, hipStream_t st) {
    const int S = std::min(hd->nsub, std::max(1, B / kMinSubFrames));
    if (S <= 1)
        return run_pipeline(hd, fb, B, d_frames, fstride, pitch0, lap0, lap1, d_kps, d_desc, cap, d_n, d_mono, st);
    while ((int)hd->sub_streams.size() < S) {
        hipStream_t s;
        hipEvent_t e;
        ORB_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        ORB_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        hd->sub_streams.push_back(s);
        hd->sub_done.push_back(e);
    }
    if (!hd->fork_ev) ORB_CHECK(hipEventCreateWithFlags(&hd->fork_ev, hipEventDisableTiming));
    ORB_CHECK(hipEventRecord(hd->fork_ev, st));
    int f0 = fb;
    for (int i = 0; i < S; ++i) {
        const int nb = B / S + (i < B % S ? 1 : 0);
        ORB_CHECK(hipStreamWaitEvent(hd->sub_streams[i], hd->fork_ev, 0));
        const int rc = run_pipeline(hd, f0, nb, d_frames, fstride, pitch0, lap0, lap1, d_kps, d_desc, cap, d_n,
                                    d_mono, hd->sub_streams[i]);
        if (rc) return rc;
        ORB_CHECK(hipEventRecord(hd->sub_done[i], hd->sub_streams[i]));
        f0 += nb;
    }
    for (int i = 0; i < S; ++i) ORB_CHECK(hipStreamWaitEvent(st, hd->sub_done[i], 0));
    return ORB_OK;
}

}  // namespace orbmi

using namespace orbmi;

extern "C" {

orbx_handle* orbx_create(const orbx_params* p, int device) {
    if (!p || p->nlevels < 1 || p->nlevels > kMaxLevels || !(p->scale_factor > 1.f) || p->nfeatures < 0)
        return nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return nullptr;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    static bool pattern_loaded[64] = {false};
    if (!pattern_loaded[device]) {
        if (hipMemcpyToSymbol(HIP_SYMBOL(c_pattern), h_pattern, sizeof(h_pattern)) != hipSuccess) return nullptr;
        pattern_loaded[device] = true;
    }
    orbx_handle* h = new orbx_handle();
    h->prm = *p;
    h->device = device;
    init_tables(h);
    return h;
}

void orbx_destroy(orbx_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    h->plan.release();
    for (hipEvent_t e : h->ev_pool) (void)hipEventDestroy(e);
    for (hipEvent_t e : h->sub_done) (void)hipEventDestroy(e);
    for (hipStream_t s : h->sub_streams) (void)hipStreamDestroy(s);
    if (h->fork_ev) (void)hipEventDestroy(h->fork_ev);
    if (h->batch_done) (void)hipEventDestroy(h->batch_done);
    if (h->st_scratch) (void)hipFree(h->st_scratch);
    if (h->hb_dev) (void)hipFree(h->hb_dev);
    if (h->hb_pin) (void)hipHostFree(h->hb_pin);
    if (h->x_exec) (void)hipGraphExecDestroy(h->x_exec);
    if (h->x_stream) (void)hipStreamDestroy(h->x_stream);
    if (h->x_pin) (void)hipHostFree(h->x_pin);
    delete h;
}

int orbx_get_tables(const orbx_handle* h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2,
                    int32_t* fpl, int32_t* umax) {
    if (!h) return ORB_ERR_PARAM;
    for (int l = 0; l < h->prm.nlevels; ++l) {
        if (scale) scale[l] = h->scale[l];
        if (inv_scale) inv_scale[l] = h->inv_scale[l];
        if (sigma2) sigma2[l] = h->sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = h->inv_sigma2[l];
        if (fpl) fpl[l] = h->nfeat[l];
    }
    if (umax) for (int v = 0; v <= kHalfPatch; ++v) umax[v] = h->umax[v];
    return ORB_OK;
}

int orbx_max_keypoints(orbx_handle* h, int w, int hh) {
    if (!h) return ORB_ERR_PARAM;
    (void)hipSetDevice(h->device);
    const int maxB = std::max(1, h->plan.maxB);
    int rc = build_plan(h, w, hh, maxB);
    if (rc) return rc;
    return h->plan.out_total;
}

int orbx_extract_batch_device(orbx_handle* h, int nframes, const uint8_t* d_frames, size_t frame_stride,
                              size_t row_step, int w, int hh, int lap0, int lap1, orb_keypoint* d_kps,
                              uint8_t* d_desc, int cap, int32_t* d_n, int32_t* d_mono, void* stream) {
    if (!h || nframes <= 0 || !d_frames) return ORB_ERR_PARAM;
    if (w <= 0 || hh <= 0) return ORB_ERR_EMPTY;
    if (hipSetDevice(h->device) != hipSuccess) return ORB_ERR_DEVICE;
    int rc = build_plan(h, w, hh, std::max(nframes, h->plan.maxB));
    if (rc) return rc;
    if (cap < h->plan.out_total) return ORB_ERR_CAPACITY;
    h->last_frames = d_frames;
    h->last_fstride = (long long)frame_stride;
    h->last_pitch0 = (int)row_step;
    h->last_B = nframes;
    h->have_last = false;          // pyramid slot 0 now holds this batch's frame 0
    h->x_pyr_valid = false;
    rc = run_batched(h, 0, nframes, d_frames, (long long)frame_stride, (int)row_step, (float)lap0, (float)lap1,
                     d_kps, d_desc, cap, d_n, d_mono, (hipStream_t)stream);
    if (rc) return rc;
    // orbx_get_batch_level waits for this (the caller's stream may be a
    // non-blocking one the null-stream copy is not ordered after)
    if (!h->batch_done) ORB_CHECK(hipEventCreateWithFlags(&h->batch_done, hipEventDisableTiming));
    ORB_CHECK(hipEventRecord(h->batch_done, (hipStream_t)stream));
    return ORB_OK;
}

int orbx_extract_batch(orbx_handle* h, int nframes, const uint8_t* const* imgs, const size_t* steps, int w, int hh,
                       const int32_t* lap, orb_keypoint* kps, uint8_t* desc, int cap, int32_t* n_out,
                       int32_t* mono_out) {
    if (!h || nframes <= 0 || !imgs || !kps || !desc || !n_out || cap < 0) return ORB_ERR_PARAM;
    if (w <= 0 || hh <= 0) return ORB_ERR_EMPTY;                     // ORBextractor.cc:1090-1091
    for (int f = 0; f < nframes; ++f)
        if (!imgs[f]) return ORB_ERR_EMPTY;
    if (hipSetDevice(h->device) != hipSuccess) return ORB_ERR_DEVICE;
    int rc = build_plan(h, w, hh, std::max(nframes, h->plan.maxB));
    if (rc) return rc;
    const int ot = h->plan.out_total;                                // device slots per frame
    const size_t pitch = ((size_t)w + 63) & ~size_t(63), fbytes = pitch * hh;
    const size_t in_b = (size_t)nframes * fbytes, kp_b = (size_t)nframes * ot * sizeof(orb_keypoint),
                 de_b = (size_t)nframes * ot * 32, nm_b = (size_t)nframes * 2 * sizeof(int32_t);
    const size_t o_kp = (in_b + 255) & ~size_t(255), o_de = o_kp + ((kp_b + 255) & ~size_t(255)),
                 o_nm = o_de + ((de_b + 255) & ~size_t(255)), total = o_nm + nm_b;
    if (h->hb_dev_bytes < total) {
        if (h->hb_dev) (void)hipFree(h->hb_dev);
        h->hb_dev = nullptr; h->hb_dev_bytes = 0;
        if (hipMalloc(&h->hb_dev, total) != hipSuccess) return ORB_ERR_DEVICE;
        h->hb_dev_bytes = total;
    }
    if (h->hb_pin_bytes < total) {
        if (h->hb_pin) (void)hipHostFree(h->hb_pin);
        h->hb_pin = nullptr; h->hb_pin_bytes = 0;
        if (hipHostMalloc(&h->hb_pin, total, hipHostMallocDefault) != hipSuccess) return ORB_ERR_DEVICE;
        h->hb_pin_bytes = total;
    }
    uint8_t* dev = (uint8_t*)h->hb_dev;
    uint8_t* pin = (uint8_t*)h->hb_pin;
    // one upload: the frames gathered into pinned memory at a common pitch (a
    // few host threads for larger batches: the gather is the host-side cost)
    (void)gather_frames(pin, pitch, fbytes, imgs, steps, w, hh, nframes);
    ORB_CHECK(hipMemcpyAsync(dev, pin, in_b, hipMemcpyHostToDevice, 0));
    orb_keypoint* d_kps = (orb_keypoint*)(dev + o_kp);
    uint8_t* d_desc = dev + o_de;
    int32_t* d_nm = (int32_t*)(dev + o_nm);                          // n[nframes] | mono[nframes]
    // consecutive frames with the same vLappingArea run as one batch
    for (int f0 = 0; f0 < nframes;) {
        const int l0 = lap ? lap[2 * f0] : 0, l1 = lap ? lap[2 * f0 + 1] : 1000;
        int f1 = f0 + 1;
        while (f1 < nframes && (!lap || (lap[2 * f1] == l0 && lap[2 * f1 + 1] == l1))) ++f1;
        rc = run_batched(h, f0, f1 - f0, dev, (long long)fbytes, (int)pitch, (float)l0, (float)l1, d_kps, d_desc,
                         ot, d_nm, d_nm + nframes, 0);
        if (rc) return rc;
        f0 = f1;
    }
    h->last_frames = dev;
    h->have_last = false;          // pyramid slot 0 now holds this batch's frame 0
    h->x_pyr_valid = false;
    h->last_fstride = (long long)fbytes;
    h->last_pitch0 = (int)pitch;
    h->last_B = nframes;
    // one download of everything, then per-frame copies out of pinned memory
    ORB_CHECK(hipMemcpyAsync(pin + o_kp, dev + o_kp, total - o_kp, hipMemcpyDeviceToHost, 0));
    ORB_CHECK(hipStreamSynchronize(0));
    const int32_t* nm = (const int32_t*)(pin + o_nm);
    const orb_keypoint* hk = (const orb_keypoint*)(pin + o_kp);
    const uint8_t* hd = pin + o_de;
    bool over = false;
    for (int f = 0; f < nframes; ++f) {
        const int n = nm[f];
        n_out[f] = n;
        if (mono_out) mono_out[f] = nm[nframes + f];
        if (n > cap) { over = true; continue; }
        std::memcpy(kps + (size_t)f * cap, hk + (size_t)f * ot, (size_t)n * sizeof(orb_keypoint));
        std::memcpy(desc + (size_t)f * cap * 32, hd + (size_t)f * ot * 32, (size_t)n * 32);
    }
    return over ? ORB_ERR_CAPACITY : ORB_OK;
}

// orbx_extract's launch-bound sequence (upload, ~12 dependent kernels, four
// downloads) as one hipGraph, captured per (size, lapping, plan epoch, staging
// buffer) and replayed; the host copies the image into the pinned staging
// buffer and reads the outputs back from it after one synchronisation.
static int extract_graph(orbx_handle* h, const uint8_t* img, int w, int hh, size_t step, int lap0, int lap1,
                         orb_keypoint* kps, uint8_t* desc, int cap, int* n_out, int* mono_out) {
    Plan& P = h->plan;
    const size_t in_b = (size_t)P.in_pitch * hh, kp_b = (size_t)P.host_cap * sizeof(orb_keypoint),
                 de_b = (size_t)P.host_cap * 32;
    const size_t o_kp = (in_b + 255) & ~size_t(255), o_de = o_kp + ((kp_b + 255) & ~size_t(255)),
                 o_nm = o_de + ((de_b + 255) & ~size_t(255)), o_py = o_nm + 256,
                 total = o_py + (h->host_pyr ? (size_t)P.pyr_bytes : 0);
    h->x_pyr_valid = false;
    if (h->x_pin_bytes < total) {
        if (h->x_pin) (void)hipHostFree(h->x_pin);
        h->x_pin = nullptr; h->x_pin_bytes = 0;
        if (hipHostMalloc(&h->x_pin, total, hipHostMallocDefault) != hipSuccess) return ORB_ERR_DEVICE;
        h->x_pin_bytes = total;
        ++h->x_pin_gen;
    }
    if (!h->x_stream && hipStreamCreateWithFlags(&h->x_stream, hipStreamNonBlocking) != hipSuccess)
        return ORB_ERR_DEVICE;
    uint8_t* pin = (uint8_t*)h->x_pin;
    const long long key[7] = {w, hh, lap0, lap1, h->plan_epoch, h->x_pin_gen, (h->host_pyr ? 1 : 0) + 2LL * debug_opt(ORB_OPT_FAST_CAND_CAP)};
    if (!h->x_exec || !std::equal(key, key + 7, h->x_key)) {
        if (h->x_exec) (void)hipGraphExecDestroy(h->x_exec);
        h->x_exec = nullptr;
        hipStream_t st = h->x_stream;
        if (hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed) != hipSuccess) return ORB_ERR_DEVICE;
        bool ok = hipMemcpyAsync(P.d_in, pin, in_b, hipMemcpyHostToDevice, st) == hipSuccess;
        ok = ok && run_pipeline(h, 0, 1, P.d_in, (long long)in_b, (int)P.in_pitch, (float)lap0, (float)lap1, P.d_kps,
                                P.d_desc, P.host_cap, P.d_n, P.d_mono, st) == ORB_OK;
        ok = ok && hipMemcpyAsync(pin + o_kp, P.d_kps, kp_b, hipMemcpyDeviceToHost, st) == hipSuccess;
        ok = ok && hipMemcpyAsync(pin + o_de, P.d_desc, de_b, hipMemcpyDeviceToHost, st) == hipSuccess;
        ok = ok && hipMemcpyAsync(pin + o_nm, P.d_n, 4, hipMemcpyDeviceToHost, st) == hipSuccess;
        ok = ok && hipMemcpyAsync(pin + o_nm + 4, P.d_mono, 4, hipMemcpyDeviceToHost, st) == hipSuccess;
        // mvImagePyramid for the host (orbx_set_host_pyramid): levels 1.. of
        // this image in one copy; level 0 is the input already in pin
        if (h->host_pyr)
            ok = ok && hipMemcpyAsync(pin + o_py, P.d_pyr, (size_t)P.pyr_bytes, hipMemcpyDeviceToHost, st) == hipSuccess;
        hipGraph_t g = nullptr;
        const bool ended = hipStreamEndCapture(st, &g) == hipSuccess;
        if (ok && ended && g) ok = hipGraphInstantiate(&h->x_exec, g, nullptr, nullptr, 0) == hipSuccess;
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
        if (!ok || !ended || !h->x_exec) { h->x_exec = nullptr; return ORB_ERR_UNSUPPORTED; }
        std::copy(key, key + 7, h->x_key);
    }
    for (int y = 0; y < hh; ++y) std::memcpy(pin + (size_t)y * P.in_pitch, img + (size_t)y * step, w);
    ORB_CHECK(hipGraphLaunch(h->x_exec, h->x_stream));
    ORB_CHECK(hipStreamSynchronize(h->x_stream));
    const int32_t n = *(const int32_t*)(pin + o_nm), mono = *(const int32_t*)(pin + o_nm + 4);
    h->x_pyr_valid = h->host_pyr;
    h->x_pyr_off = o_py;
    if (n_out) *n_out = n;
    if (mono_out) *mono_out = mono;
    h->have_last = true;
    h->last_n = n;
    h->last_w = w; h->last_h = hh;
    h->last_frames = nullptr;      // pyramid slot 0 now holds this image
    h->last_B = 0;
    if (n > cap) return ORB_ERR_CAPACITY;
    if (n > 0) {
        std::memcpy(kps, pin + o_kp, (size_t)n * sizeof(orb_keypoint));
        std::memcpy(desc, pin + o_de, (size_t)n * 32);
    }
    return ORB_OK;
}

int orbx_extract(orbx_handle* h, const uint8_t* img, int w, int hh, size_t step, int lap0, int lap1,
                 orb_keypoint* kps, uint8_t* desc, int cap, int* n_out, int* mono_out) {
    if (!h) return ORB_ERR_PARAM;
    if (!img || w <= 0 || hh <= 0) return ORB_ERR_EMPTY;      // ORBextractor.cc:1090-1091
    if (hipSetDevice(h->device) != hipSuccess) return ORB_ERR_DEVICE;
    h->have_last = false;          // until this extraction's outputs are complete
    int rc = build_plan(h, w, hh, std::max(1, h->plan.maxB));
    if (rc) return rc;
    Plan& P = h->plan;
    // the graph path unless per-stage profiling is on (its events are recorded
    // per call) or capture is unavailable (then the direct launches below)
    if (!h->profiling) {
        rc = extract_graph(h, img, w, hh, step, lap0, lap1, kps, desc, cap, n_out, mono_out);
        if (rc != ORB_ERR_UNSUPPORTED) return rc;
    }
    h->x_pyr_valid = false;
    ORB_CHECK(hipMemcpy2D(P.d_in, P.in_pitch, img, step, w, hh, hipMemcpyHostToDevice));
    rc = run_pipeline(h, 0, 1, P.d_in, (long long)P.in_pitch * hh, (int)P.in_pitch, (float)lap0, (float)lap1, P.d_kps,
                      P.d_desc, P.host_cap, P.d_n, P.d_mono, 0);
    if (rc) return rc;
    int32_t n = 0, mono = 0;
    ORB_CHECK(hipMemcpy(&n, P.d_n, 4, hipMemcpyDeviceToHost));
    ORB_CHECK(hipMemcpy(&mono, P.d_mono, 4, hipMemcpyDeviceToHost));
    if (n_out) *n_out = n;
    if (mono_out) *mono_out = mono;
    h->have_last = true;
    h->last_n = n;
    h->last_w = w; h->last_h = hh;
    h->last_frames = nullptr;      // pyramid slot 0 now holds this image
    h->last_B = 0;
    if (n > cap) return ORB_ERR_CAPACITY;
    if (n > 0) {
        ORB_CHECK(hipMemcpy(kps, P.d_kps, n * sizeof(orb_keypoint), hipMemcpyDeviceToHost));
        ORB_CHECK(hipMemcpy(desc, P.d_desc, (size_t)n * 32, hipMemcpyDeviceToHost));
    }
    return ORB_OK;
}

// The last orbx_extract's outputs in HBM, for orbm_dframe_from_extractor
// (matcher.hip): valid until the next extraction call on h.
extern "C++" int orbmi::extractor_last_outputs(orbx_handle* h, const orb_keypoint** kps, const uint8_t** desc,
                                               int* n, int* device) {
    if (!h || !h->have_last || h->last_n > h->plan.host_cap) return ORB_ERR_PARAM;
    *kps = h->plan.d_kps;
    *desc = h->plan.d_desc;
    *n = h->last_n;
    *device = h->device;
    return ORB_OK;
}

int orbx_set_profiling(orbx_handle* h, int enable) {
    if (!h) return ORB_ERR_PARAM;
    h->profiling = enable != 0;
    h->ev_calls.clear();
    h->ev_next = 0;
    return ORB_OK;
}

int orbx_set_pyramid_mode(orbx_handle* h, int mode) {
    if (!h || mode < 0 || mode > 2) return ORB_ERR_PARAM;
    h->pyr_mode = mode;
    h->x_key[4] = -1;                       // the captured single-image graph holds the old choice
    return ORB_OK;
}

int orbx_pyramid_kernel(orbx_handle* h) { return h ? h->pyr_last : 0; }

int orbx_set_host_pyramid(orbx_handle* h, int enable) {
    if (!h) return ORB_ERR_PARAM;
    h->host_pyr = enable != 0;
    h->x_pyr_valid = false;
    return ORB_OK;
}

int orbx_set_stage_event(orbx_handle* h, int stage, void* event) {
    if (!h || stage < 0 || stage > 5) return ORB_ERR_PARAM;
    h->stage_ev[stage] = (hipEvent_t)event;
    h->x_key[4] = -1;                       // a captured single-image graph holds the old events
    return ORB_OK;
}

int orbx_set_streams(orbx_handle* h, int nsub) {
    if (!h || nsub < 1 || nsub > 16) return ORB_ERR_PARAM;
    h->nsub = nsub;
    return ORB_OK;
}

int orbx_get_profile(orbx_handle* h, float* stage_ms, int nstages) {
    if (!h || !stage_ms) return ORB_ERR_PARAM;
    for (int i = 0; i < nstages; ++i) stage_ms[i] = 0.f;
    int calls = 0;
    for (auto& m : h->ev_calls) {
        if (m.size() < 2) continue;
        ORB_CHECK(hipEventSynchronize(m.back()));
        for (size_t i = 0; i + 1 < m.size() && (int)i < nstages; ++i) {
            float ms = 0.f;
            ORB_CHECK(hipEventElapsedTime(&ms, m[i], m[i + 1]));
            stage_ms[i] += ms;
        }
        ++calls;
    }
    h->ev_calls.clear();
    h->ev_next = 0;
    return calls;
}

int orbx_get_level(orbx_handle* h, int level, uint8_t* dst, size_t dst_step, int* w, int* hh) {
    if (!h || !h->have_last || level < 0 || level >= h->plan.L) return ORB_ERR_PARAM;
    const Plan& P = h->plan;
    const LevelDev& d = P.lv[level];
    if (w) *w = d.w;
    if (hh) *hh = d.h;
    if (!dst) return ORB_OK;
    const size_t sp = level == 0 ? P.in_pitch : (size_t)d.pitch;
    if (h->x_pyr_valid) {          // the host copy the graph made (orbx_set_host_pyramid)
        const uint8_t* src = (const uint8_t*)h->x_pin + (level == 0 ? 0 : h->x_pyr_off + d.off);
        for (int y = 0; y < d.h; ++y) std::memcpy(dst + (size_t)y * dst_step, src + (size_t)y * sp, d.w);
        return ORB_OK;
    }
    (void)hipSetDevice(h->device);
    const uint8_t* src = level == 0 ? P.d_in : P.d_pyr + d.off;
    ORB_CHECK(hipMemcpy2D(dst, dst_step, src, sp, d.w, d.h, hipMemcpyDeviceToHost));
    return ORB_OK;
}

int orbx_debug_math(int device, int what, long long begin, long long end, int chunk_log2, int fused,
                    unsigned long long* hashes) {
    if (what < 0 || what > 2 || begin < 0 || end <= begin || chunk_log2 < 8 || chunk_log2 > 30 || !hashes)
        return ORB_ERR_PARAM;
    if (what != 2 && end > (1ll << 32)) return ORB_ERR_PARAM;
    if (hipSetDevice(device) != hipSuccess) return ORB_ERR_DEVICE;
    if (what == 1) {   // the pattern table lives in constant memory (orbx_create loads it per device)
        ORB_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_pattern), h_pattern, sizeof(h_pattern)));
    }
    const long long nchunks = ((end - begin) + (1ll << chunk_log2) - 1) >> chunk_log2;
    // (the guard before the allocation: nothing to free on a refusal)
    const void* kd = what == 0 ? reinterpret_cast<const void*>(&k_debug_math<0>)
                               : what == 1 ? reinterpret_cast<const void*>(&k_debug_math<1>)
                                           : reinterpret_cast<const void*>(&k_debug_math<2>);
    if (!lds_fits(kd, 0)) return ORB_ERR_UNSUPPORTED;
    unsigned long long* d = nullptr;
    ORB_CHECK(hipMalloc(&d, nchunks * sizeof(unsigned long long)));
    const dim3 grid((unsigned)std::min<long long>(nchunks, 8192));
    if (what == 0) hipLaunchKernelGGL(k_debug_math<0>, grid, dim3(256), 0, 0, begin, end, chunk_log2, fused, d);
    else if (what == 1) hipLaunchKernelGGL(k_debug_math<1>, grid, dim3(256), 0, 0, begin, end, chunk_log2, fused, d);
    else hipLaunchKernelGGL(k_debug_math<2>, grid, dim3(256), 0, 0, begin, end, chunk_log2, fused, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(hashes, d, nchunks * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? ORB_OK : ORB_ERR_DEVICE;
}

int orbx_debug_sort(int device, int narrays, const int32_t* off, const int32_t* cnt, const int32_t* x0,
                    int32_t* perm, int32_t* fallback) {
    if (narrays < 0 || (narrays && (!off || !perm || !fallback))) return ORB_ERR_PARAM;
    if (narrays == 0) return ORB_OK;
    int maxm = 0;
    for (int i = 0; i < narrays; ++i) {
        const int m = off[i + 1] - off[i];
        if (m < 0 || m > kDbgSortMax || off[i] < 0) return ORB_ERR_PARAM;
        maxm = std::max(maxm, m);
    }
    const long long tot = off[narrays];
    if (tot && (!cnt || !x0)) return ORB_ERR_PARAM;
    if (hipSetDevice(device) != hipSuccess) return ORB_ERR_DEVICE;
    int *d_off = nullptr, *d_buf = nullptr;
    const size_t nb = (size_t)std::max(1LL, tot);
    auto done = [&](int rc) {
        if (d_off) (void)hipFree(d_off);
        if (d_buf) (void)hipFree(d_buf);
        return rc;
    };
    if (hipMalloc(&d_off, (narrays + 1) * sizeof(int)) != hipSuccess ||
        hipMalloc(&d_buf, (3 * nb + narrays) * sizeof(int)) != hipSuccess)
        return done(ORB_ERR_DEVICE);
    int* d_cnt = d_buf;
    int* d_x0 = d_buf + nb;
    int* d_perm = d_buf + 2 * nb;
    int* d_fb = d_buf + 3 * nb;
    if (hipMemcpy(d_off, off, (narrays + 1) * sizeof(int), hipMemcpyHostToDevice) != hipSuccess ||
        (tot && (hipMemcpy(d_cnt, cnt, tot * sizeof(int), hipMemcpyHostToDevice) != hipSuccess ||
                 hipMemcpy(d_x0, x0, tot * sizeof(int), hipMemcpyHostToDevice) != hipSuccess)))
        return done(ORB_ERR_DEVICE);
    if (!lds_fits(reinterpret_cast<const void*>(&k_debug_sort), dbg_sort_lds(maxm))) return done(ORB_ERR_UNSUPPORTED);
    hipLaunchKernelGGL(k_debug_sort, dim3(narrays), dim3(256), dbg_sort_lds(maxm), 0, d_off, d_cnt, d_x0, d_perm, d_fb);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return done(ORB_ERR_DEVICE);
    if ((tot && hipMemcpy(perm, d_perm, tot * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) ||
        hipMemcpy(fallback, d_fb, narrays * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
        return done(ORB_ERR_DEVICE);
    return done(ORB_OK);
}

int orbx_get_batch_level(orbx_handle* h, int frame, int level, uint8_t* dst, size_t dst_step, int* w, int* hh) {
    if (!h || !h->last_frames || frame < 0 || frame >= h->last_B || level < 0 || level >= h->plan.L)
        return ORB_ERR_PARAM;
    const Plan& P = h->plan;
    const LevelDev& d = P.lv[level];
    if (w) *w = d.w;
    if (hh) *hh = d.h;
    if (!dst) return ORB_OK;
    (void)hipSetDevice(h->device);
    const uint8_t* src = level == 0 ? h->last_frames + (long long)frame * h->last_fstride
                                    : P.d_pyr + (long long)frame * P.pyr_bytes + d.off;
    const size_t sp = level == 0 ? (size_t)h->last_pitch0 : (size_t)d.pitch;
    if (h->batch_done) ORB_CHECK(hipEventSynchronize(h->batch_done));
    ORB_CHECK(hipMemcpy2D(dst, dst_step, src, sp, d.w, d.h, hipMemcpyDeviceToHost));
    return ORB_OK;
}

int orbx_debug_plan_info(orbx_handle* h, int w, int hh, int32_t* info, int n) {
    if (!h || !info || n < 1) return ORB_ERR_PARAM;
    (void)hipSetDevice(h->device);
    const int rc = build_plan(h, w, hh, std::max(1, h->plan.maxB));
    if (rc != ORB_OK) return rc;
    const PyrStream& S = h->plan.ps;
    const int32_t v[8] = {S.ok, S.pretest, S.K0, S.nsteps, S.lds_bytes, S.E, h->plan.ncells, h->plan.bm_ok};
    for (int i = 0; i < n && i < 8; ++i) info[i] = v[i];
    return ORB_OK;
}

int orbx_debug_pretest(orbx_handle* h, int frame, int level, uint8_t* dst, size_t dst_step, int32_t* win) {
    if (!h || !h->last_frames || frame < 0 || frame >= h->last_B || level < 0 || level >= h->plan.L)
        return ORB_ERR_PARAM;
    const Plan& P = h->plan;
    if (!h->bm_last || !P.d_bm) return ORB_ERR_UNSUPPORTED;
    const LevelDev& d = P.lv[level];
    if (win) {
        win[0] = P.win_y0[level]; win[1] = P.win_y1[level]; win[2] = P.win_x0[level]; win[3] = P.win_x1[level];
        win[4] = (d.w + 7) / 8; win[5] = d.h;
    }
    if (!dst) return ORB_OK;
    (void)hipSetDevice(h->device);
    if (h->batch_done) ORB_CHECK(hipEventSynchronize(h->batch_done));
    ORB_CHECK(hipMemcpy2D(dst, dst_step, P.d_bm + (long long)frame * P.bm_bytes + d.bm_off, (size_t)d.bm_pitch,
                          (size_t)(d.w + 7) / 8, d.h, hipMemcpyDeviceToHost));
    return ORB_OK;
}

int orbx_debug_stage(orbx_handle* h, int stage, orb_keypoint* kps, int cap, int32_t* counts) {
    if (!h || !h->have_last) return ORB_ERR_PARAM;
    (void)hipSetDevice(h->device);
    const Plan& P = h->plan;
    int off = 0;
    if (stage == 0) {
        std::vector<int> cc(P.ncells);
        std::vector<uint32_t> keys(P.slot_total);
        ORB_CHECK(hipMemcpy(cc.data(), P.d_cell_count, cc.size() * 4, hipMemcpyDeviceToHost));
        ORB_CHECK(hipMemcpy(keys.data(), P.d_cell_keys, keys.size() * 4, hipMemcpyDeviceToHost));
        for (int l = 0; l < P.L; ++l) {
            const LevelDev& d = P.lv[l];
            int nl = 0;
            for (int c = d.cell_base; c < d.cell_base + d.ncells; ++c)
                for (int j = 0; j < cc[c]; ++j, ++nl, ++off) {
                    const uint32_t k = keys[P.cells[c].slot_off + j];
                    if (off < cap) kps[off] = orb_keypoint{(float)(k & 0xfff), (float)((k >> 12) & 0xfff), 7.f,
                                                           -1.f, (float)(k >> 24), 0, -1};
                }
            if (counts) counts[l] = nl;
        }
    } else {
        std::vector<int> qn(P.L);
        std::vector<uint32_t> keys(P.out_total);
        ORB_CHECK(hipMemcpy(qn.data(), P.d_qt_n, qn.size() * 4, hipMemcpyDeviceToHost));
        ORB_CHECK(hipMemcpy(keys.data(), P.d_qt_key, keys.size() * 4, hipMemcpyDeviceToHost));
        for (int l = 0; l < P.L; ++l) {
            const LevelDev& d = P.lv[l];
            if (counts) counts[l] = qn[l];
            for (int p = 0; p < qn[l]; ++p, ++off) {
                const uint32_t k = keys[d.out_base + p];
                if (off < cap)
                    kps[off] = orb_keypoint{(float)((k & 0xfff) + kEdge - 3), (float)(((k >> 12) & 0xfff) + kEdge - 3),
                                            (float)d.patch, -1.f, (float)(k >> 24), l, -1};
            }
        }
    }
    return off <= cap ? off : ORB_ERR_CAPACITY;
}

}  // extern "C"
