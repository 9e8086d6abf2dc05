// =============================================================================
// oracle/orb_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the hot path of vdoom/ORB_SLAM3_VIO_FIXES (ORBextractor,
// the ORBmatcher searches, the Frame grid and the DBoW2 descent), written for
// this repository.  It is the CHECKER the HIP library is compared against in
// tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Nothing in
// the product (orb_slam3_vio_fixes_amd/) links, loads or calls it.
//
// PARITY STATUS: "parity unpinned" at the OpenCV boundary.  The reference path
// needs OpenCV (cv::FAST, cv::resize, cv::GaussianBlur, cv::fastAtan2), which is
// absent from the image; the reference holds no golden vectors, fixtures or
// known-answer tests for this path, and building it against
// stand-in headers is not allowed.  The OpenCV primitives below are restated
// from OpenCV 4.x semantics.  What IS pinned: the
// constructor tables against the survey's evaluation of the reference
// (Appendix B), the rBRIEF table (SHA-256 of the reference's integers), glibc
// sincosf (the oracle calls the system libm, exactly what the reference calls).
//
// Every function cites the reference file:line it follows (paths relative to
// the reference tree).  Compile with -ffp-contract=off: the only fused
// operations are the explicit fmaf() of the descriptor sampling (A.6).
// =============================================================================
#include "../include/orb_mi355x.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <list>
#include <thread>
#include <vector>

namespace {

const int kPatchSize = 31;      // ORBextractor.cc:71
const int kHalfPatch = 15;      // ORBextractor.cc:72
const int kEdge = 19;           // ORBextractor.cc:73
const float kCellW = 35.f;      // ORBextractor.cc:785
const int kThHigh = 100, kThLow = 50, kHisto = 30;   // ORBmatcher.cc:35-37
const int kGridCols = 64, kGridRows = 48;            // Frame.h:44-45

const int kPattern[256 * 4] = {
#include "../orb_slam3_vio_fixes_amd/csrc/brief_pattern.inc"
};

// ---- OpenCV scalar helpers (core/fast_math.hpp) -----------------------------
inline int cv_round(double v) { return (int)std::nearbyint(v); }   // ties-to-even
inline int cv_round(float v) { return (int)std::nearbyintf(v); }
inline int cv_floor(double v) { int i = (int)v; return i - (i > v); }
inline int cv_floor(float v) { int i = (int)v; return i - (i > v); }
inline int cv_ceil(float v) { int i = (int)v; return i + (i < v); }
inline short sat_short(float v) {
    int i = cv_round(v);
    return (short)std::min(32767, std::max(-32768, i));
}
inline int refl101(int p, int len) {            // borderInterpolate BORDER_REFLECT_101
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}

struct Img {
    int w = 0, h = 0;
    std::vector<uint8_t> px;
    void alloc(int ww, int hh) { w = ww; h = hh; px.assign((size_t)ww * hh, 0); }
    uint8_t* row(int y) { return px.data() + (size_t)y * w; }
    const uint8_t* row(int y) const { return px.data() + (size_t)y * w; }
};

// cv::resize(src, dst, dsize, 0, 0, INTER_LINEAR) for CV_8UC1, OpenCV 4.x generic
// path (imgproc/resize.cpp: hal::resize coefficient tables, HResizeLinear,
// VResizeLinear<uchar,int,short,FixedPtCast<..>,VResizeLinearVec_32s8u>).
// Called at ORBextractor.cc:1183.
int resize_linear(const Img& s, Img& d) {
    if (d.w == s.w && d.h == s.h) { d.px = s.px; return 0; }
    const double inv_sx = (double)d.w / s.w, inv_sy = (double)d.h / s.h;
    const double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
    // At an exact 2x reduction in both directions OpenCV switches to INTER_AREA
    // (resize.cpp: is_area_fast && iscale_x == 2 && iscale_y == 2), whose fast
    // path for 8UC1 is (a + b + c + d + 2) >> 2 per 2x2 block
    // (ResizeAreaFastVec::operator()).  The linear fixed point below reproduces
    // it exactly there: every weight is 1024 (fx = fy = 0.5, sx = 2 dx,
    // sy = 2 dy, no clamping), so a row gives (1024 * ((1024 (a + b)) >> 4)) >> 16
    // = a + b and the output ((a + b) + (c + d) + 2) >> 2.  No separate area
    // path is needed (tests/test_oracle_tables.py checks the block average).
    std::vector<int> xo(d.w), xa(2 * d.w), yo(d.h), yb(2 * d.h);
    int xmax = d.w;
    for (int dx = 0; dx < d.w; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0.f; sx = 0; }
        if (sx + 1 >= s.w) {
            xmax = std::min(xmax, dx);
            if (sx >= s.w - 1) { fx = 0.f; sx = s.w - 1; }
        }
        xo[dx] = sx;
        xa[2 * dx] = sat_short((1.f - fx) * 2048.f);
        xa[2 * dx + 1] = sat_short(fx * 2048.f);
    }
    for (int dy = 0; dy < d.h; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor(fy);
        fy -= sy;
        yo[dy] = sy;
        yb[2 * dy] = sat_short((1.f - fy) * 2048.f);
        yb[2 * dy + 1] = sat_short(fy * 2048.f);
    }
    std::vector<int> h0(d.w), h1(d.w);
    auto hrow = [&](int sy, std::vector<int>& out) {
        const uint8_t* S = s.row(sy);
        for (int dx = 0; dx < d.w; ++dx) {
            int sx = xo[dx];
            out[dx] = dx < xmax ? S[sx] * xa[2 * dx] + S[sx + 1] * xa[2 * dx + 1]
                                : S[sx] * 2048;
        }
    };
    for (int dy = 0; dy < d.h; ++dy) {
        int r0 = std::min(std::max(yo[dy], 0), s.h - 1);
        int r1 = std::min(std::max(yo[dy] + 1, 0), s.h - 1);
        hrow(r0, h0);
        hrow(r1, h1);
        const int b0 = yb[2 * dy], b1 = yb[2 * dy + 1];
        uint8_t* D = d.row(dy);
        for (int dx = 0; dx < d.w; ++dx)
            D[dx] = (uint8_t)((((b0 * (h0[dx] >> 4)) >> 16) + ((b1 * (h1[dx] >> 4)) >> 16) + 2) >> 2);
    }
    return 0;
}

// cv::FAST(img, kps, threshold, true) == FAST_t<16> + cornerScore<16>
// (features2d/src/fast.cpp), restated literally with its 3-row score ring.
// Called at ORBextractor.cc:826,845 on a cell ROI.
struct Cand { int x, y, score; };

int corner_score16(const uint8_t* p, const int* off, int thr) {
    int d[25];
    const int v = p[0];
    for (int k = 0; k < 25; ++k) d[k] = v - p[off[k]];
    int a0 = thr;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min(d[k + 1], std::min(d[k + 2], d[k + 3]));
        if (a <= a0) continue;
        for (int m = 4; m <= 8; ++m) a = std::min(a, d[k + m]);
        a0 = std::max(a0, std::min(a, d[k]));
        a0 = std::max(a0, std::min(a, d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = std::max(d[k + 1], std::max(d[k + 2], d[k + 3]));
        b = std::max(b, std::max(d[k + 4], d[k + 5]));
        if (b >= b0) continue;
        for (int m = 6; m <= 8; ++m) b = std::max(b, d[k + m]);
        b0 = std::min(b0, std::max(b, d[k]));
        b0 = std::min(b0, std::max(b, d[k + 9]));
    }
    return -b0 - 1;
}

void fast9(const uint8_t* base, int step, int rows, int cols, int thr, std::vector<Cand>& out) {
    out.clear();
    static const int ring[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                                    {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};
    int off[25];
    for (int k = 0; k < 16; ++k) off[k] = ring[k][0] + ring[k][1] * step;
    for (int k = 16; k < 25; ++k) off[k] = off[k - 16];
    thr = std::min(std::max(thr, 0), 255);
    if (rows < 7 || cols < 7) return;
    std::vector<uint8_t> sbuf(3 * (size_t)cols, 0);
    std::vector<int> cpos(3 * (size_t)(cols + 1), 0);
    uint8_t* sb[3] = {&sbuf[0], &sbuf[cols], &sbuf[2 * (size_t)cols]};
    int* cp[3] = {&cpos[1], &cpos[cols + 2], &cpos[2 * (size_t)cols + 3]};
    for (int i = 3; i < rows - 2; ++i) {
        const uint8_t* p = base + (size_t)i * step + 3;
        uint8_t* cur = sb[(i - 3) % 3];
        int* corners = cp[(i - 3) % 3];
        std::memset(cur, 0, cols);
        int nc = 0;
        if (i < rows - 3) {
            for (int j = 3; j < cols - 3; ++j, ++p) {
                const int v = p[0];
                int brighter = 0, darker = 0;   // longest runs over the wrapped ring
                int run_b = 0, run_d = 0;
                for (int k = 0; k < 25; ++k) {
                    const int x = p[off[k]];
                    if (x < v - thr) { if (++run_d > 8) darker = 1; } else run_d = 0;
                    if (x > v + thr) { if (++run_b > 8) brighter = 1; } else run_b = 0;
                }
                if (darker || brighter) {
                    corners[nc++] = j;
                    cur[j] = (uint8_t)corner_score16(p, off, thr);
                }
            }
        }
        corners[-1] = nc;
        if (i == 3) continue;
        const uint8_t* prev = sb[(i - 4 + 3) % 3];
        const uint8_t* pprev = sb[(i - 5 + 3) % 3];
        const int* pc = cp[(i - 4 + 3) % 3];
        for (int k = 0; k < pc[-1]; ++k) {
            const int j = pc[k];
            const int sc = prev[j];
            if (sc > prev[j + 1] && sc > prev[j - 1] && sc > pprev[j - 1] && sc > pprev[j] &&
                sc > pprev[j + 1] && sc > cur[j - 1] && sc > cur[j] && sc > cur[j + 1])
                out.push_back({j, i - 1, sc});
        }
    }
}

// Gaussian kernel of cv::GaussianBlur(Size(7,7), 2, 2) in 8-bit fixed point
// (OpenCV >= 4.5 getGaussianKernelBitExact + error diffusion, or the older
// plainly rounded kernel).  SURVEY.md A.5.
const int kBlurED[7] = {18, 34, 48, 56, 48, 34, 18};
const int kBlurLegacy[7] = {18, 34, 49, 55, 49, 34, 18};

// GaussianBlur(workingMat, workingMat, Size(7,7), 2, 2, BORDER_REFLECT_101) on a
// clone() of the level (ORBextractor.cc:1132-1133): GaussianBlurFixedPoint,
// horizontal ufixedpoint16 pass, vertical ufixedpoint32 pass, round and
// saturate to u8 (the legacy kernel sums to 257, so 255-regions overflow).
void blur7(const Img& s, Img& d, const int* k) {
    d.alloc(s.w, s.h);
    std::vector<uint32_t> hbuf((size_t)s.w * s.h);
    for (int y = 0; y < s.h; ++y)
        for (int x = 0; x < s.w; ++x) {
            uint32_t acc = 0;
            for (int t = 0; t < 7; ++t) acc += k[t] * s.row(y)[refl101(x + t - 3, s.w)];
            hbuf[(size_t)y * s.w + x] = acc;
        }
    for (int y = 0; y < s.h; ++y)
        for (int x = 0; x < s.w; ++x) {
            uint32_t acc = 0;
            for (int t = 0; t < 7; ++t) acc += k[t] * hbuf[(size_t)refl101(y + t - 3, s.h) * s.w + x];
            d.row(y)[x] = (uint8_t)std::min(255u, (acc + 32768u) >> 16);   // saturate_cast<uchar>
        }
}

// cv::fastAtan2 (OpenCV 4.x core/mathfuncs_core: atan_f32), degrees, no FMA.
float fast_atan2_deg(float y, float x) {
    const float k = (float)(180 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    const float ax = std::fabs(x), ay = std::fabs(y);
    float a;
    if (ax >= ay) {
        const float c = ay / (ax + (float)2.220446049250313e-16);
        const float c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        const float c = ax / (ay + (float)2.220446049250313e-16);
        const float c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// IC_Angle (ORBextractor.cc:76-103).
float ic_angle(const Img& im, float px, float py, const std::vector<int>& umax) {
    const int cx = cv_round(px), cy = cv_round(py);
    const uint8_t* c = im.row(cy) + cx;
    const int step = im.w;
    int m01 = 0, m10 = 0;
    for (int u = -kHalfPatch; u <= kHalfPatch; ++u) m10 += u * c[u];
    for (int v = 1; v <= kHalfPatch; ++v) {
        int vs = 0;
        for (int u = -umax[v]; u <= umax[v]; ++u) {
            const int up = c[u + v * step], dn = c[u - v * step];
            vs += up - dn;
            m10 += u * (up + dn);
        }
        m01 += v * vs;
    }
    return fast_atan2_deg((float)m01, (float)m10);
}

// computeOrbDescriptor (ORBextractor.cc:107-146).  (a, b) come from glibc's
// sincosf exactly as in the reference binary; the sampling offsets use the
// fused form GCC emits for -O3 -march=native on an FMA host (A.6).
void orb_descriptor(const Img& blurred, float px, float py, float angle_deg, bool fused,
                    uint8_t* out) {
    const float ang = angle_deg * (float)(3.14159265358979323846 / 180.f);
    float b, a;
    sincosf(ang, &b, &a);
    const uint8_t* c = blurred.row(cv_round(py)) + cv_round(px);
    const int step = blurred.w;
    auto sample = [&](int idx) -> int {
        const float x = (float)kPattern[2 * idx], y = (float)kPattern[2 * idx + 1];
        int r, q;
        if (fused) {
            r = cv_round(std::fmaf(x, b, y * a));
            q = cv_round(std::fmaf(x, a, -(y * b)));
        } else {
            r = cv_round(x * b + y * a);
            q = cv_round(x * a - y * b);
        }
        return c[r * step + q];
    };
    for (int byte = 0; byte < 32; ++byte) {
        int val = 0;
        for (int bit = 0; bit < 8; ++bit) {
            const int t = byte * 16 + bit * 2;
            val |= (sample(t) < sample(t + 1)) << bit;
        }
        out[byte] = (uint8_t)val;
    }
}

// ---- ORBextractor ------------------------------------------------------------
struct KP { float x, y, size, angle, response; int octave, class_id; };

struct QNode {                       // ExtractorNode (ORBextractor.h:30-41)
    std::vector<KP> keys;
    int ulx = 0, uly = 0, urx = 0, ury = 0, blx = 0, bly = 0, brx = 0, bry = 0;
    std::list<QNode>::iterator self;
    bool no_more = false;
};

// ExtractorNode::DivideNode (ORBextractor.cc:480-536).
void split4(const QNode& p, QNode& a, QNode& b, QNode& c, QNode& d) {
    const int hx = (int)std::ceil((float)(p.urx - p.ulx) / 2);
    const int hy = (int)std::ceil((float)(p.bry - p.uly) / 2);
    a.ulx = p.ulx; a.uly = p.uly; a.urx = p.ulx + hx; a.ury = p.uly;
    a.blx = p.ulx; a.bly = p.uly + hy; a.brx = p.ulx + hx; a.bry = p.uly + hy;
    b.ulx = a.urx; b.uly = a.ury; b.urx = p.urx; b.ury = p.ury;
    b.blx = a.brx; b.bly = a.bry; b.brx = p.urx; b.bry = p.uly + hy;
    c.ulx = a.blx; c.uly = a.bly; c.urx = a.brx; c.ury = a.bry;
    c.blx = p.blx; c.bly = p.bly; c.brx = a.brx; c.bry = p.bly;
    d.ulx = c.urx; d.uly = c.ury; d.urx = b.brx; d.ury = b.bry;
    d.blx = c.brx; d.bly = c.bry; d.brx = p.brx; d.bry = p.bry;
    for (const KP& k : p.keys) {
        if (k.x < a.urx) (k.y < a.bry ? a : c).keys.push_back(k);
        else (k.y < a.bry ? b : d).keys.push_back(k);
    }
    for (QNode* n : {&a, &b, &c, &d})
        if (n->keys.size() == 1) n->no_more = true;
}

typedef std::pair<int, QNode*> SizedNode;
// compareNodes (ORBextractor.cc:538-553)
bool node_less(SizedNode& l, SizedNode& r) {
    if (l.first != r.first) return l.first < r.first;
    return l.second->ulx < r.second->ulx;
}

// ORBextractor::DistributeOctTree (ORBextractor.cc:555-779).
std::vector<KP> distribute(const std::vector<KP>& in, int minX, int maxX, int minY, int maxY, int N) {
    const int nIni = (int)std::round((float)(maxX - minX) / (maxY - minY));
    const float hX = (float)(maxX - minX) / nIni;
    std::list<QNode> nodes;
    std::vector<QNode*> roots(nIni);
    for (int i = 0; i < nIni; ++i) {
        QNode n;
        n.ulx = (int)(hX * (float)i); n.uly = 0;
        n.urx = (int)(hX * (float)(i + 1)); n.ury = 0;
        n.blx = n.ulx; n.bly = maxY - minY;
        n.brx = n.urx; n.bry = maxY - minY;
        nodes.push_back(n);
        roots[i] = &nodes.back();
    }
    for (const KP& k : in) roots[(size_t)(k.x / hX)]->keys.push_back(k);
    for (auto it = nodes.begin(); it != nodes.end();) {
        if (it->keys.size() == 1) { it->no_more = true; ++it; }
        else if (it->keys.empty()) it = nodes.erase(it);
        else ++it;
    }
    std::vector<SizedNode> grow;
    // push the non-empty children to the list front; the ones with >1 key are
    // queued for expansion (ORBextractor.cc:636-676 / 706-742)
    auto adopt = [&](QNode (&ch)[4], int* nexp) {
        for (QNode& c : ch) {
            if (c.keys.empty()) continue;
            nodes.push_front(c);
            if (c.keys.size() > 1) {
                if (nexp) ++*nexp;
                grow.push_back(SizedNode((int)c.keys.size(), &nodes.front()));
                nodes.front().self = nodes.begin();
            }
        }
    };
    bool done = false;
    while (!done) {
        const int before = (int)nodes.size();
        int nexp = 0;
        grow.clear();
        for (auto it = nodes.begin(); it != nodes.end();) {
            if (it->no_more) { ++it; continue; }
            QNode ch[4];
            split4(*it, ch[0], ch[1], ch[2], ch[3]);
            adopt(ch, &nexp);
            it = nodes.erase(it);
        }
        if ((int)nodes.size() >= N || (int)nodes.size() == before) {
            done = true;
        } else if ((int)nodes.size() + nexp * 3 > N) {
            while (!done) {
                const int before2 = (int)nodes.size();
                std::vector<SizedNode> prev = grow;
                grow.clear();
                std::sort(prev.begin(), prev.end(), node_less);
                for (int j = (int)prev.size() - 1; j >= 0; --j) {
                    QNode ch[4];
                    split4(*prev[j].second, ch[0], ch[1], ch[2], ch[3]);
                    adopt(ch, nullptr);
                    nodes.erase(prev[j].second->self);
                    if ((int)nodes.size() >= N) break;
                }
                if ((int)nodes.size() >= N || (int)nodes.size() == before2) done = true;
            }
        }
    }
    std::vector<KP> out;
    out.reserve(nodes.size());
    for (QNode& n : nodes) {
        const KP* best = &n.keys[0];
        for (size_t k = 1; k < n.keys.size(); ++k)
            if (n.keys[k].response > best->response) best = &n.keys[k];
        out.push_back(*best);
    }
    return out;
}

struct Extractor {
    orbx_params prm{};
    std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
    std::vector<int> nfeat, umax;
    std::vector<Img> pyr;
    std::vector<std::vector<KP>> stage_cand, stage_qt;

    // ORBextractor::ORBextractor (ORBextractor.cc:409-469)
    explicit Extractor(const orbx_params& p) : prm(p) {
        const int L = p.nlevels;
        const double sf = (double)p.scale_factor;
        scale.resize(L); sigma2.resize(L); inv_scale.resize(L); inv_sigma2.resize(L);
        scale[0] = 1.f; sigma2[0] = 1.f;
        for (int i = 1; i < L; ++i) {
            scale[i] = (float)(scale[i - 1] * sf);
            sigma2[i] = scale[i] * scale[i];
        }
        for (int i = 0; i < L; ++i) { inv_scale[i] = 1.f / scale[i]; inv_sigma2[i] = 1.f / sigma2[i]; }
        nfeat.resize(L);
        const float factor = (float)(1.0f / sf);
        float per = p.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)L));
        int sum = 0;
        for (int l = 0; l < L - 1; ++l) {
            nfeat[l] = cv_round(per);
            sum += nfeat[l];
            per *= factor;
        }
        nfeat[L - 1] = std::max(p.nfeatures - sum, 0);
        umax.assign(kHalfPatch + 1, 0);
        const int vmax = cv_floor(kHalfPatch * std::sqrt(2.f) / 2 + 1);
        const int vmin = cv_ceil(kHalfPatch * std::sqrt(2.f) / 2);
        const double hp2 = kHalfPatch * kHalfPatch;
        for (int v = 0; v <= vmax; ++v) umax[v] = cv_round(std::sqrt(hp2 - v * v));
        for (int v = kHalfPatch, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
    }

    int err = 0;   // keypoints(): a size the reference does not survive

    // ComputePyramid (ORBextractor.cc:1170-1195)
    int pyramid(const uint8_t* img, int w, int h, size_t step) {
        pyr.assign(prm.nlevels, Img());
        for (int l = 0; l < prm.nlevels; ++l) {
            const float s = inv_scale[l];
            const int lw = cv_round((float)w * s), lh = cv_round((float)h * s);
            // a level of <= 32 px on a side: DistributeOctTree divides by
            // maxY - minY <= 0 and sizes a vector from it (ORBextractor.cc:
            // 559-565), which the reference does not survive
            if (lw - 2 * (kEdge - 3) < 1 || lh - 2 * (kEdge - 3) < 1) return ORB_ERR_UNSUPPORTED;
            pyr[l].alloc(lw, lh);
            if (l == 0) {
                for (int y = 0; y < h; ++y) std::memcpy(pyr[0].row(y), img + (size_t)y * step, w);
            } else {
                int rc = resize_linear(pyr[l - 1], pyr[l]);
                if (rc) return rc;
            }
        }
        return 0;
    }

    // ComputeKeyPointsOctTree (ORBextractor.cc:781-896)
    void keypoints(std::vector<std::vector<KP>>& all) {
        all.assign(prm.nlevels, {});
        stage_cand.assign(prm.nlevels, {});
        std::vector<Cand> cell;
        for (int l = 0; l < prm.nlevels; ++l) {
            const Img& im = pyr[l];
            const int minBX = kEdge - 3, minBY = minBX;
            const int maxBX = im.w - kEdge + 3, maxBY = im.h - kEdge + 3;
            std::vector<KP>& cand = stage_cand[l];
            const float width = (float)(maxBX - minBX), height = (float)(maxBY - minBY);
            const int nCols = (int)(width / kCellW), nRows = (int)(height / kCellW);
            // nCols or nRows = 0 (a level of 33..66 px): the cell loops below
            // do not run; the reference's cell sizes are then a division by
            // zero nothing reads (kept out of the integer conversion here)
            const int wCell = nCols ? (int)std::ceil(width / nCols) : 0;
            const int hCell = nRows ? (int)std::ceil(height / nRows) : 0;
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
                    const int y0 = (int)iniY, x0 = (int)iniX;
                    const uint8_t* roi = im.row(y0) + x0;
                    const int rr = (int)maxY - y0, cc = (int)maxX - x0;
                    fast9(roi, im.w, rr, cc, prm.ini_th_fast, cell);
                    if (cell.empty()) fast9(roi, im.w, rr, cc, prm.min_th_fast, cell);
                    for (const Cand& c : cell) {
                        KP k{(float)c.x, (float)c.y, 7.f, -1.f, (float)c.score, 0, -1};
                        k.x += j * wCell;
                        k.y += i * hCell;
                        cand.push_back(k);
                    }
                }
            }
            std::vector<KP>& kp = all[l];
            // nIni = 0 with keys indexes an empty vpIniNodes (:583-584): refused
            const int nIni = (int)std::round((float)(maxBX - minBX) / (maxBY - minBY));
            if (nIni < 0 || (nIni == 0 && !cand.empty())) { err = ORB_ERR_UNSUPPORTED; return; }
            kp = distribute(cand, minBX, maxBX, minBY, maxBY, nfeat[l]);
            const int patch = (int)(kPatchSize * scale[l]);
            for (KP& k : kp) {
                k.x += minBX;
                k.y += minBY;
                k.octave = l;
                k.size = (float)patch;
            }
        }
        stage_qt = all;
        for (int l = 0; l < prm.nlevels; ++l)
            for (KP& k : all[l]) k.angle = ic_angle(pyr[l], k.x, k.y, umax);
    }

    // ORBextractor::operator() (ORBextractor.cc:1086-1168)
    int run(const uint8_t* img, int w, int h, size_t step, int lap0, int lap1, std::vector<KP>& out,
            std::vector<uint8_t>& desc, int& mono) {
        if (!img || w <= 0 || h <= 0) return ORB_ERR_EMPTY;
        int rc = pyramid(img, w, h, step);
        if (rc) return rc;
        std::vector<std::vector<KP>> all;
        err = 0;
        keypoints(all);
        if (err) return err;
        int n = 0;
        for (auto& v : all) n += (int)v.size();
        out.assign(n, KP{});
        desc.assign((size_t)n * 32, 0);
        const int* kern = prm.blur_variant == 1 ? kBlurLegacy : kBlurED;
        int head = 0, tail = n - 1;
        for (int l = 0; l < prm.nlevels; ++l) {
            if (all[l].empty()) continue;
            Img bl;
            blur7(pyr[l], bl, kern);
            const float s = scale[l];
            for (KP k : all[l]) {
                uint8_t d[32];
                orb_descriptor(bl, k.x, k.y, k.angle, prm.fma_sampling != 0, d);
                if (l != 0) { k.x *= s; k.y *= s; }
                int dst;
                if (k.x >= (float)lap0 && k.x <= (float)lap1) dst = tail--;
                else dst = head++;
                out[dst] = k;
                std::memcpy(&desc[(size_t)dst * 32], d, 32);
            }
        }
        mono = head;
        return 0;
    }
};

// ---- ORBmatcher ----------------------------------------------------------------

// DescriptorDistance (ORBmatcher.cc:2058-2074): SWAR popcount per 32-bit word.
int hamming(const uint8_t* a, const uint8_t* b) {
    int dist = 0;
    for (int i = 0; i < 8; ++i) {
        uint32_t x, y;
        std::memcpy(&x, a + 4 * i, 4);
        std::memcpy(&y, b + 4 * i, 4);
        uint32_t v = x ^ y;
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
    }
    return dist;
}

// Frame grid: AssignFeaturesToGrid / PosInGrid / GetFeaturesInArea
// (Frame.cc:385-416, 725-735, 657-723).
struct Grid {
    const orbm_frame* f;
    std::vector<int> cell[kGridCols][kGridRows];
    explicit Grid(const orbm_frame* fr) : f(fr) {
        for (int i = 0; i < f->n; ++i) {
            const orb_keypoint& k = f->kps[i];
            const int gx = (int)std::round((k.x - f->min_x) * f->grid_inv_w);
            const int gy = (int)std::round((k.y - f->min_y) * f->grid_inv_h);
            if (gx < 0 || gx >= kGridCols || gy < 0 || gy >= kGridRows) continue;
            cell[gx][gy].push_back(i);
        }
    }
    std::vector<int> area(float x, float y, float r, int minL, int maxL) const {
        std::vector<int> res;
        const int cx0 = std::max(0, (int)std::floor((x - f->min_x - r) * f->grid_inv_w));
        if (cx0 >= kGridCols) return res;
        const int cx1 = std::min(kGridCols - 1, (int)std::ceil((x - f->min_x + r) * f->grid_inv_w));
        if (cx1 < 0) return res;
        const int cy0 = std::max(0, (int)std::floor((y - f->min_y - r) * f->grid_inv_h));
        if (cy0 >= kGridRows) return res;
        const int cy1 = std::min(kGridRows - 1, (int)std::ceil((y - f->min_y + r) * f->grid_inv_h));
        if (cy1 < 0) return res;
        const bool levels = (minL > 0) || (maxL >= 0);
        for (int ix = cx0; ix <= cx1; ++ix)
            for (int iy = cy0; iy <= cy1; ++iy)
                for (int i : cell[ix][iy]) {
                    const orb_keypoint& k = f->kps[i];
                    if (levels) {
                        if (k.octave < minL) continue;
                        if (maxL >= 0 && k.octave > maxL) continue;
                    }
                    if (std::fabs(k.x - x) < r && std::fabs(k.y - y) < r) res.push_back(i);
                }
        return res;
    }
};

// ComputeThreeMaxima (ORBmatcher.cc:2012-2053)
void three_maxima(const std::vector<int>* hist, int& i1, int& i2, int& i3) {
    int m1 = 0, m2 = 0, m3 = 0;
    i1 = i2 = i3 = -1;
    for (int i = 0; i < kHisto; ++i) {
        const int s = (int)hist[i].size();
        if (s > m1) { m3 = m2; m2 = m1; m1 = s; i3 = i2; i2 = i1; i1 = i; }
        else if (s > m2) { m3 = m2; m2 = s; i3 = i2; i2 = i; }
        else if (s > m3) { m3 = s; i3 = i; }
    }
    if (m2 < 0.1f * (float)m1) { i2 = -1; i3 = -1; }
    else if (m3 < 0.1f * (float)m1) { i3 = -1; }
}

int rot_bin(float a1, float a2) {
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)std::round(rot * (1.0f / kHisto));
    if (bin == kHisto) bin = 0;
    return bin;
}

}  // namespace

// =============================================================================
// C entry points: orbo_* mirror the product's orbx_* / orbm_* / orbv_*.
// =============================================================================
extern "C" {

struct orbo_state { Extractor* ex; };

void* orbo_create(const orbx_params* p) {
    if (!p || p->nlevels < 1 || p->nlevels > 32 || p->scale_factor <= 1.f || p->nfeatures < 0) return nullptr;
    return new Extractor(*p);
}
void orbo_destroy(void* h) { delete static_cast<Extractor*>(h); }

int orbo_get_tables(void* h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2,
                    int32_t* nfeat, int32_t* umax) {
    Extractor* e = static_cast<Extractor*>(h);
    for (int l = 0; l < e->prm.nlevels; ++l) {
        if (scale) scale[l] = e->scale[l];
        if (inv_scale) inv_scale[l] = e->inv_scale[l];
        if (sigma2) sigma2[l] = e->sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = e->inv_sigma2[l];
        if (nfeat) nfeat[l] = e->nfeat[l];
    }
    if (umax) for (int v = 0; v <= kHalfPatch; ++v) umax[v] = e->umax[v];
    return 0;
}

int orbo_extract(void* h, const uint8_t* img, int w, int hh, size_t step, int lap0, int lap1,
                 orb_keypoint* kps, uint8_t* desc, int cap, int* n_out, int* mono_out) {
    Extractor* e = static_cast<Extractor*>(h);
    std::vector<KP> out;
    std::vector<uint8_t> d;
    int mono = 0;
    int rc = e->run(img, w, hh, step, lap0, lap1, out, d, mono);
    if (rc) return rc;
    const int n = (int)out.size();
    if (n_out) *n_out = n;
    if (mono_out) *mono_out = mono;
    if (n > cap) return ORB_ERR_CAPACITY;
    static_assert(sizeof(KP) == sizeof(orb_keypoint), "KeyPoint layout");
    if (n) {   // (an empty vector's data() may be null: UBSan, tests/test_sanitizers.py)
        std::memcpy(kps, out.data(), sizeof(KP) * n);
        std::memcpy(desc, d.data(), (size_t)n * 32);
    }
    return 0;
}

int orbo_get_level(void* h, int level, uint8_t* dst, size_t dst_step, int* w, int* hh) {
    Extractor* e = static_cast<Extractor*>(h);
    if (level < 0 || level >= (int)e->pyr.size()) return ORB_ERR_PARAM;
    const Img& im = e->pyr[level];
    if (w) *w = im.w;
    if (hh) *hh = im.h;
    if (dst)
        for (int y = 0; y < im.h; ++y) std::memcpy(dst + (size_t)y * dst_step, im.row(y), im.w);
    return 0;
}

int orbo_debug_stage(void* h, int stage, orb_keypoint* kps, int cap, int32_t* counts) {
    Extractor* e = static_cast<Extractor*>(h);
    const auto& src = stage == 0 ? e->stage_cand : e->stage_qt;
    int off = 0;
    for (size_t l = 0; l < src.size(); ++l) {
        if (counts) counts[l] = (int)src[l].size();
        for (const KP& k : src[l]) {
            if (off < cap) std::memcpy(&kps[off], &k, sizeof(KP));
            ++off;
        }
    }
    return off <= cap ? off : ORB_ERR_CAPACITY;
}

// Standalone primitives, exposed for property tests.
int orbo_resize(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh) {
    Img s, d;
    s.alloc(sw, sh);
    std::memcpy(s.px.data(), src, (size_t)sw * sh);
    d.alloc(dw, dh);
    int rc = resize_linear(s, d);
    if (!rc) std::memcpy(dst, d.px.data(), (size_t)dw * dh);
    return rc;
}
int orbo_fast(const uint8_t* img, int w, int hh, int thr, int32_t* xys, int cap) {
    std::vector<Cand> out;
    fast9(img, w, hh, w, thr, out);
    for (size_t i = 0; i < out.size() && (int)i < cap; ++i) {
        xys[3 * i] = out[i].x; xys[3 * i + 1] = out[i].y; xys[3 * i + 2] = out[i].score;
    }
    return (int)out.size();
}
int orbo_blur(const uint8_t* src, int w, int hh, int variant, uint8_t* dst) {
    Img s, d;
    s.alloc(w, hh);
    std::memcpy(s.px.data(), src, (size_t)w * hh);
    blur7(s, d, variant == 1 ? kBlurLegacy : kBlurED);
    std::memcpy(dst, d.px.data(), (size_t)w * hh);
    return 0;
}
float orbo_fast_atan2(float y, float x) { return fast_atan2_deg(y, x); }

// Host side of the exhaustive device math check (include/orb_mi355x.h:
// orbx_debug_math; tests/test_gpu_math.py): the same chunk hashes from the
// system libm's sincosf (what the reference binary calls), this oracle's
// fastAtan2 and its sampling formula (orb_descriptor above).  The hash and
// the moment-pair enumeration are restated here, not shared with the product.
static inline uint32_t dm_lowbias32(uint32_t v) {
    v ^= v >> 16; v *= 0x7feb352du; v ^= v >> 15; v *= 0x846ca68bu; v ^= v >> 16;
    return v;
}
static inline uint32_t dm_bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
static inline float dm_float(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

static uint32_t dm_element(int what, uint64_t i, int fused) {
    if (what == 0) {
        float s, c;
        sincosf(dm_float((uint32_t)i), &s, &c);
        return dm_bits(s) ^ (dm_bits(c) * 0x9E3779B9u);
    }
    if (what == 1) {
        // the pattern as float columns and the word weights, once: the loop
        // below then vectorises (the -O3 -march builds, liborb_oracle_v3.so)
        static const struct Cols {
            float x[512], y[512];
            uint32_t w[512];
            Cols() {
                for (int k = 0; k < 512; ++k) {
                    x[k] = (float)kPattern[2 * k];
                    y[k] = (float)kPattern[2 * k + 1];
                    w[k] = (uint32_t)k * 0x9E3779B1u | 1u;
                }
            }
        } P;
        const float ang = dm_float((uint32_t)i) * (float)(3.14159265358979323846 / 180.f);
        float b, a;
        sincosf(ang, &b, &a);
        // cvRound of |v| < 2^22 as (v + 1.5*2^23) - 1.5*2^23: the same
        // ties-to-even result, in a form the compiler vectorises
        const float M = 12582912.f;
        auto rnd = [M](float v) { return (int)((v + M) - M); };
        uint32_t e = 0;
        if (fused) {
            for (int k = 0; k < 512; ++k) {
                const int r = rnd(std::fmaf(P.x[k], b, P.y[k] * a));
                const int q = rnd(std::fmaf(P.x[k], a, -(P.y[k] * b)));
                e += ((uint32_t)(r & 0xff) | ((uint32_t)(q & 0xff) << 8)) * P.w[k];
            }
        } else {
            for (int k = 0; k < 512; ++k) {
                const int r = rnd(P.x[k] * b + P.y[k] * a);
                const int q = rnd(P.x[k] * a - P.y[k] * b);
                e += ((uint32_t)(r & 0xff) | ((uint32_t)(q & 0xff) << 8)) * P.w[k];
            }
        }
        return e;
    }
    float y, x;
    if (i < 4097ull * 4097ull) {
        y = (float)((int)(i / 4097) - 2048);
        x = (float)((int)(i % 4097) - 2048);
    } else {
        y = (float)((int)(dm_lowbias32((uint32_t)(2 * i)) % 3000001u) - 1500000);
        x = (float)((int)(dm_lowbias32((uint32_t)(2 * i + 1)) % 3000001u) - 1500000);
    }
    return dm_bits(fast_atan2_deg(y, x));
}

// Degree angles below 2^-36 (float bits < kTinyDeg): the radian angle is
// below 2^-41, where sincosf returns (angle, 1.0f) exactly, so every product
// x*b, y*b is below 2^-36 in magnitude: fmaf(x, b, y*1) rounds to y and
// fmaf(x, 1, -(y*b)) to x for the nonzero integers of the pattern, and to a
// value of magnitude < 0.5 (cvRound 0) for a zero one; the unfused forms
// likewise.  Every such angle has the offsets (r, c) = (y, x).  The host
// takes that word instead of evaluating ~7.6e8 angles whose products are
// subnormal (microcode assists: ~30x slower); orbo_debug_math checks it
// against the full evaluation at both ends of the range before using it.
static const uint32_t kTinyDeg = 0x2d800000u;   // 2^-36
static uint32_t dm_tiny_word() {
    uint32_t e = 0;
    for (int k = 0; k < 512; ++k)
        e += ((uint32_t)(kPattern[2 * k + 1] & 0xff) | ((uint32_t)(kPattern[2 * k] & 0xff) << 8)) *
             ((uint32_t)k * 0x9E3779B1u | 1u);
    return e;
}

int orbo_debug_math(int what, long long begin, long long end, int chunk_log2, int fused, int nthreads,
                    unsigned long long* hashes) {
    if (what < 0 || what > 2 || begin < 0 || end <= begin || chunk_log2 < 8 || chunk_log2 > 30 || !hashes ||
        nthreads < 1)
        return -1;
    const uint32_t tiny = dm_tiny_word();
    // fused bit 1: evaluate the tiny range too (tests/test_oracle_math.py)
    if (what == 1 && (dm_element(1, 1, fused & 1) != tiny || dm_element(1, kTinyDeg - 1, fused & 1) != tiny ||
                      dm_element(1, 0, fused & 1) != tiny))
        return -2;
    const long long nchunks = ((end - begin) + (1ll << chunk_log2) - 1) >> chunk_log2;
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
        th.emplace_back([=] {
            for (long long ck = t; ck < nchunks; ck += nthreads) {
                const long long c0 = begin + (ck << chunk_log2), c1 = std::min(end, c0 + (1ll << chunk_log2));
                unsigned long long acc = 0;
                for (long long i = c0; i < c1; ++i) {
                    const uint32_t e = (what == 1 && !(fused & 2) && i < (long long)kTinyDeg)
                                           ? tiny : dm_element(what, (uint64_t)i, fused & 1);
                    acc += (unsigned long long)e * (2 * (uint64_t)i + 1);
                }
                hashes[ck] = acc;
            }
        });
    for (auto& x : th) x.join();
    return 0;
}

int orbo_descriptor_distance(const uint8_t* a, const uint8_t* b) { return hamming(a, b); }

// ORBmatcher::SearchForInitialization (ORBmatcher.cc:648-763)
int orbo_search_for_initialization(const orbm_frame* f1, const orbm_frame* f2, float* prev,
                                   int window, float ratio, int check_ori, int32_t* m12) {
    Grid g2(f2);
    int nm = 0;
    std::vector<int> hist[kHisto];
    std::vector<int> mdist(f2->n, INT32_MAX), m21(f2->n, -1);
    for (int i = 0; i < f1->n; ++i) m12[i] = -1;
    for (int i1 = 0; i1 < f1->n; ++i1) {
        const orb_keypoint& k1 = f1->kps[i1];
        if (k1.octave > 0) continue;
        std::vector<int> cand = g2.area(prev[2 * i1], prev[2 * i1 + 1], (float)window, k1.octave, k1.octave);
        if (cand.empty()) continue;
        const uint8_t* d1 = f1->desc + (size_t)i1 * 32;
        int best = INT32_MAX, best2 = INT32_MAX, bi = -1;
        for (int i2 : cand) {
            const int dist = hamming(d1, f2->desc + (size_t)i2 * 32);
            if (mdist[i2] <= dist) continue;
            if (dist < best) { best2 = best; best = dist; bi = i2; }
            else if (dist < best2) best2 = dist;
        }
        if (best <= kThLow && best < (float)best2 * ratio) {
            if (m21[bi] >= 0) { m12[m21[bi]] = -1; --nm; }
            m12[i1] = bi;
            m21[bi] = i1;
            mdist[bi] = best;
            ++nm;
            if (check_ori) hist[rot_bin(f1->kps[i1].angle, f2->kps[bi].angle)].push_back(i1);
        }
    }
    if (check_ori) {
        int a, b, c;
        three_maxima(hist, a, b, c);
        for (int i = 0; i < kHisto; ++i) {
            if (i == a || i == b || i == c) continue;
            for (int i1 : hist[i])
                if (m12[i1] >= 0) { m12[i1] = -1; --nm; }
        }
    }
    for (int i1 = 0; i1 < f1->n; ++i1)
        if (m12[i1] >= 0) {
            prev[2 * i1] = f2->kps[m12[i1]].x;
            prev[2 * i1 + 1] = f2->kps[m12[i1]].y;
        }
    return nm;
}

// ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) (ORBmatcher.cc:223-425), mono.
int orbo_search_by_bow(const orbm_frame* kf, const orbm_featvec* kfv, const uint8_t* kf_valid,
                       const orbm_frame* f, const orbm_featvec* ffv, float ratio, int check_ori,
                       int32_t* match) {
    for (int i = 0; i < f->n; ++i) match[i] = -1;
    std::vector<int> hist[kHisto];
    int nm = 0, a = 0, b = 0;
    while (a < kfv->nnodes && b < ffv->nnodes) {
        const uint32_t na = kfv->node_ids[a], nb = ffv->node_ids[b];
        if (na == nb) {
            for (int p = kfv->offsets[a]; p < kfv->offsets[a + 1]; ++p) {
                const int ikf = (int)kfv->idx[p];
                if (!kf_valid[ikf]) continue;
                const uint8_t* dk = kf->desc + (size_t)ikf * 32;
                int best = 256, best2 = 256, bi = -1;
                for (int q = ffv->offsets[b]; q < ffv->offsets[b + 1]; ++q) {
                    const int jf = (int)ffv->idx[q];
                    if (match[jf] >= 0) continue;
                    const int dist = hamming(dk, f->desc + (size_t)jf * 32);
                    if (dist < best) { best2 = best; best = dist; bi = jf; }
                    else if (dist < best2) best2 = dist;
                }
                if (best <= kThLow && (float)best < ratio * (float)best2) {
                    match[bi] = ikf;
                    if (check_ori) hist[rot_bin(kf->kps[ikf].angle, f->kps[bi].angle)].push_back(bi);
                    ++nm;
                }
            }
            ++a; ++b;
        } else if (na < nb) {
            a = (int)(std::lower_bound(kfv->node_ids + a, kfv->node_ids + kfv->nnodes, nb) - kfv->node_ids);
        } else {
            b = (int)(std::lower_bound(ffv->node_ids + b, ffv->node_ids + ffv->nnodes, na) - ffv->node_ids);
        }
    }
    if (check_ori) {
        int i1, i2, i3;
        three_maxima(hist, i1, i2, i3);
        for (int i = 0; i < kHisto; ++i) {
            if (i == i1 || i == i2 || i == i3) continue;
            for (int j : hist[i]) { match[j] = -1; --nm; }
        }
    }
    return nm;
}


// The relocalisation loop over candidates (Tracking.cc:3641-3648: one
// SearchByBoW(KF_i, F) per candidate) over a whole keyframe map laid out like
// orbm_kf_map_device but in host memory; keyframes are independent, so they are
// spread over nthreads.  match: nkf x f->n, nm: nkf.
int orbo_search_by_bow_map(int nkf, const orb_keypoint* kps, const uint8_t* desc, const uint8_t* valid,
                           const int64_t* kp_off, const uint32_t* fv_node, const int32_t* fv_off,
                           const uint32_t* fv_idx, const int64_t* fv_node_off, const int64_t* fv_idx_off,
                           const orbm_frame* f, const orbm_featvec* ffv, float ratio, int check_ori, int nthreads,
                           int32_t* match, int32_t* nm) {
    if (nkf < 0 || !f || !ffv) return -3;
    auto one = [&](int i) {
        orbm_frame kf{};
        kf.n = (int32_t)(kp_off[i + 1] - kp_off[i]);
        kf.kps = kps + kp_off[i];
        kf.desc = desc + kp_off[i] * 32;
        orbm_featvec fv{};
        fv.nnodes = (int32_t)(fv_node_off[i + 1] - fv_node_off[i]);
        fv.node_ids = fv_node + fv_node_off[i];
        fv.offsets = fv_off + fv_node_off[i] + i;
        fv.idx = fv_idx + fv_idx_off[i];
        nm[i] = orbo_search_by_bow(&kf, &fv, valid + kp_off[i], f, ffv, ratio, check_ori,
                                   match + (size_t)i * f->n);
    };
    const int nt = std::max(1, std::min(nthreads, nkf));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (int i = t; i < nkf; i += nt) one(i);
        });
    for (auto& x : th) x.join();
    return 0;
}

// ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th, bFarPoints, thFarPoints)
// (ORBmatcher.cc:43-213, the F.Nleft == -1 branch) + RadiusByViewingCos (:215-221).
int orbo_search_by_projection_mps(const orbm_frame* f, const orbm_mappoints* mp, float th, int far_points,
                                  float th_far, float ratio, int32_t* owner, const uint8_t* blocked) {
    Grid g(f);
    int nm = 0;
    const bool factor = th != 1.0;
    // slot "has a MapPoint with Observations() > 0" (ORBmatcher.cc:88-90)
    auto slot_blocked = [&](int idx) {
        const int o = owner[idx];
        if (o == -1) return false;
        if (o <= -2) return blocked[idx] != 0;
        return mp->has_obs[o] != 0;
    };
    for (int i = 0; i < mp->n; ++i) {
        if (!mp->in_view[i]) continue;
        if (far_points && mp->track_depth[i] > th_far) continue;
        const int lvl = mp->level[i];
        float r = mp->view_cos[i] > 0.998 ? 2.5f : 4.0f;
        if (factor) r *= th;
        const float rs = r * f->scale_factors[lvl];
        std::vector<int> cand = g.area(mp->proj_x[i], mp->proj_y[i], rs, lvl - 1, lvl);
        if (cand.empty()) continue;
        const uint8_t* dm = mp->desc + (size_t)i * 32;
        int best = 256, bl = -1, best2 = 256, bl2 = -1, bi = -1;
        for (int idx : cand) {
            if (slot_blocked(idx)) continue;
            if (f->u_right && f->u_right[idx] > 0) {
                const float er = std::fabs(mp->proj_xr[i] - f->u_right[idx]);
                if (er > rs) continue;
            }
            const int dist = hamming(dm, f->desc + (size_t)idx * 32);
            if (dist < best) {
                best2 = best; best = dist; bl2 = bl; bl = f->kps[idx].octave; bi = idx;
            } else if (dist < best2) {
                bl2 = f->kps[idx].octave; best2 = dist;
            }
        }
        if (best <= kThHigh) {
            if (bl == bl2 && best > ratio * best2) continue;
            if (bl != bl2 || best <= ratio * best2) {
                owner[bi] = i;
                ++nm;
            }
        }
    }
    return nm;
}

// ORBmatcher::SearchByProjection(Frame& Current, const Frame& Last, th, bMono)
// (ORBmatcher.cc:1676-1887, CurrentFrame.Nleft == -1); projection done by the caller.
int orbo_search_by_projection_last(const orbm_frame* cur, int nlast, const uint8_t* valid, const float* u,
                                   const float* v, const float* ur, const int32_t* last_octave,
                                   const float* last_angle, const uint8_t* has_obs, const uint8_t* last_desc,
                                   float th, int mode, int check_ori, int32_t* owner, const uint8_t* blocked) {
    Grid g(cur);
    int nm = 0;
    std::vector<int> hist[kHisto];
    auto slot_blocked = [&](int idx) {
        const int o = owner[idx];
        if (o == -1) return false;
        if (o <= -2) return blocked[idx] != 0;
        return has_obs[o] != 0;
    };
    for (int i = 0; i < nlast; ++i) {
        if (!valid[i]) continue;
        const int oct = last_octave[i];
        const float radius = th * cur->scale_factors[oct];
        std::vector<int> cand;
        if (mode == 1) cand = g.area(u[i], v[i], radius, oct, -1);
        else if (mode == 2) cand = g.area(u[i], v[i], radius, 0, oct);
        else cand = g.area(u[i], v[i], radius, oct - 1, oct + 1);
        if (cand.empty()) continue;
        const uint8_t* dm = last_desc + (size_t)i * 32;
        int best = 256, bi = -1;
        for (int i2 : cand) {
            if (slot_blocked(i2)) continue;
            if (cur->u_right && cur->u_right[i2] > 0) {
                const float er = std::fabs(ur[i] - cur->u_right[i2]);
                if (er > radius) continue;
            }
            const int dist = hamming(dm, cur->desc + (size_t)i2 * 32);
            if (dist < best) { best = dist; bi = i2; }
        }
        if (best <= kThHigh) {
            owner[bi] = i;
            ++nm;
            if (check_ori) hist[rot_bin(last_angle[i], cur->kps[bi].angle)].push_back(bi);
        }
    }
    if (check_ori) {
        int a, b, c;
        three_maxima(hist, a, b, c);
        for (int k = 0; k < kHisto; ++k) {
            if (k == a || k == b || k == c) continue;
            for (int j : hist[k]) { owner[j] = -1; --nm; }
        }
    }
    return nm;
}

// TemplatedVocabulary::transform(feature, word_id, weight, &nid, levelsup)
// (TemplatedVocabulary.h:1217-1259): greedy descent, first child wins ties.
int orbo_transform(const orbv_vocab* voc, int n, const uint8_t* desc, int levelsup, int32_t* word_id,
                   double* weight, int32_t* node_id) {
    const int nid_level = voc->depth_levels - levelsup;
    for (int i = 0; i < n; ++i) {
        const uint8_t* d = desc + (size_t)i * 32;
        int nid = 0;
        if (nid_level <= 0) nid = 0;
        int fin = 0, level = 0;
        do {
            ++level;
            // nodes = m_nodes[final_id].children; first child wins ties (:1236-1249)
            const int c0 = voc->first_child[fin], nc = voc->nchild[fin];
            auto child = [&](int j) { return voc->child_idx ? voc->child_idx[c0 + j] : c0 + j; };
            int best_id = child(0);
            double best = hamming(d, voc->node_desc + (size_t)best_id * 32);
            for (int j = 1; j < nc; ++j) {
                const int c = child(j);
                const double dd = hamming(d, voc->node_desc + (size_t)c * 32);
                if (dd < best) { best = dd; best_id = c; }
            }
            fin = best_id;
            if (level == nid_level) nid = fin;
        } while (voc->nchild[fin] != 0);
        word_id[i] = voc->word_id[fin];
        weight[i] = voc->weight[fin];
        node_id[i] = nid;
    }
    return 0;
}

// Frame::ComputeStereoMatches (src/Frame.cc:811-981) for a rectified pair whose
// left/right images were the last inputs of the extractors hl/hr (their
// mvImagePyramid).  kl/kr are the extractors' keypoints (mvKeys, mvKeysRight),
// scale/inv_scale the level tables.  uright/depth receive mvuRight/mvDepth.
int orbo_compute_stereo_matches(void* hl, void* hr, const orb_keypoint* kl, int nl, const uint8_t* dl,
                                const orb_keypoint* kr, int nr, const uint8_t* dr, const float* scale,
                                const float* inv_scale, float mb, float mbf, float* uright, float* depth) {
    const Extractor* el = static_cast<const Extractor*>(hl);
    const Extractor* er = static_cast<const Extractor*>(hr);
    for (int i = 0; i < nl; ++i) uright[i] = depth[i] = -1.0f;                       // :813-814
    const int thOrbDist = (kThHigh + kThLow) / 2;                                    // :816
    const int nRows = el->pyr[0].h;                                                  // :818
    std::vector<std::vector<int>> rows(nRows);                                       // :821
    for (int iR = 0; iR < nr; ++iR) {                                                // :828-838
        const float kpY = kr[iR].y;
        const float r = 2.0f * scale[kr[iR].octave];
        const int maxr = (int)std::ceil(kpY + r);
        const int minr = (int)std::floor(kpY - r);
        for (int yi = minr; yi <= maxr; ++yi)
            if (yi >= 0 && yi < nRows) rows[yi].push_back(iR);
    }
    const float minZ = mb, minD = 0, maxD = mbf / minZ;                              // :841-843
    std::vector<std::pair<int, int>> dist_idx;                                        // :846
    for (int iL = 0; iL < nl; ++iL) {
        const orb_keypoint& kpL = kl[iL];
        const int levelL = kpL.octave;
        const float vL = kpL.y, uL = kpL.x;
        const std::vector<int>& cand = rows[(size_t)vL];                             // :856
        if (cand.empty()) continue;
        const float minU = uL - maxD, maxU = uL - minD;                              // :861-862
        if (maxU < 0) continue;
        int bestDist = kThHigh;                                                      // :867-868
        int bestIdxR = 0;
        for (int iR : cand) {                                                        // :873-893
            const orb_keypoint& kpR = kr[iR];
            if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
            const float uR = kpR.x;
            if (uR >= minU && uR <= maxU) {
                const int dist = hamming(dl + (size_t)iL * 32, dr + (size_t)iR * 32);
                if (dist < bestDist) { bestDist = dist; bestIdxR = iR; }
            }
        }
        if (bestDist >= thOrbDist) continue;                                         // :896
        // sub-pixel match by 11-position L1 correlation at the keypoint's level (:898-933)
        const float uR0 = kr[bestIdxR].x;
        const float sf = inv_scale[kpL.octave];
        const float scaleduL = std::round(kpL.x * sf), scaledvL = std::round(kpL.y * sf);
        const float scaleduR0 = std::round(uR0 * sf);
        const int w = 5, L = 5;
        const Img& IL = el->pyr[kpL.octave];
        const Img& IR = er->pyr[kpL.octave];
        const float iniu = scaleduR0 + L - w, endu = scaleduR0 + L + w + 1;
        if (iniu < 0 || endu >= IR.w) continue;
        int bestSad = INT32_MAX, bestincR = 0;
        float dists[2 * L + 1];
        const int yl0 = (int)scaledvL - w, xl0 = (int)scaleduL - w;
        for (int incR = -L; incR <= L; ++incR) {
            const int xr0 = (int)scaleduR0 + incR - w;
            int sad = 0;
            for (int y = 0; y < 2 * w + 1; ++y)
                for (int x = 0; x < 2 * w + 1; ++x)
                    sad += std::abs((int)IL.row(yl0 + y)[xl0 + x] - (int)IR.row(yl0 + y)[xr0 + x]);
            const float dist = (float)(double)sad;                                   // cv::norm(NORM_L1) -> double
            if (dist < bestSad) { bestSad = (int)dist; bestincR = incR; }
            dists[L + incR] = dist;
        }
        if (bestincR == -L || bestincR == L) continue;                               // :935-936
        const float d1 = dists[L + bestincR - 1], d2 = dists[L + bestincR], d3 = dists[L + bestincR + 1];
        const float deltaR = (d1 - d3) / (2.0f * (d1 + d3 - 2.0f * d2));             // :943
        if (deltaR < -1 || deltaR > 1) continue;
        float bestuR = scale[kpL.octave] * ((float)scaleduR0 + (float)bestincR + deltaR);   // :949
        float disparity = uL - bestuR;
        if (disparity >= minD && disparity < maxD) {                                 // :953-964
            if (disparity <= 0) {
                disparity = 0.01;
                bestuR = uL - 0.01;
            }
            depth[iL] = mbf / disparity;
            uright[iL] = bestuR;
            dist_idx.push_back(std::make_pair(bestSad, iL));
        }
    }
    if (dist_idx.empty()) return 0;      // the reference reads vDistIdx[0] here (undefined)
    std::sort(dist_idx.begin(), dist_idx.end());                                     // :968-971
    const float median = dist_idx[dist_idx.size() / 2].first;
    const float thDist = 1.5f * 1.4f * median;
    for (int i = (int)dist_idx.size() - 1; i >= 0; --i) {                           // :973-980
        if (dist_idx[i].first < thDist) break;
        uright[dist_idx[i].second] = -1;
        depth[dist_idx[i].second] = -1;
    }
    return 0;
}

// cv::BFMatcher(NORM_HAMMING).knnMatch(query, train, matches, 2) as called by
// Frame::ComputeStereoFishEyeMatches (src/Frame.cc:1144; BFmatcher :43):
// per query the two nearest train rows, OpenCV batchDistance's insertion
// (strict '<' against the current 2nd best, equal distances keep index
// order).  idx/dist are [nq][2], -1 where fewer than two train rows exist.
int orbo_knn_match2(const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* idx, int32_t* dist) {
    for (int i = 0; i < nq; ++i) {
        int bi[2] = {-1, -1};
        int bd[2] = {INT32_MAX, INT32_MAX};
        for (int j = 0; j < nt; ++j) {
            const int d = hamming(q + (size_t)i * 32, t + (size_t)j * 32);
            if (d < bd[1]) {
                int k = 0;
                for (k = 0; k >= 0 && bd[k] > d; --k) { bi[k + 1] = bi[k]; bd[k + 1] = bd[k]; }
                bi[k + 1] = j;
                bd[k + 1] = d;
            }
        }
        for (int k = 0; k < 2; ++k) {
            idx[2 * i + k] = bi[k];
            dist[2 * i + k] = bi[k] >= 0 ? bd[k] : -1;
        }
    }
    return 0;
}

// KeyFrameDatabase::DetectRelocalizationCandidates (src/KeyFrameDatabase.cc:733-845)
// over a snapshot of the database: per-KF BowVectors (CSR, words ascending),
// the inverted file (CSR by word, list order), per-KF
// GetBestCovisibilityKeyFrames(10) (CSR), per-KF map id.  reloc_score is the
// mRelocScore member of every KF: read for neighbours that share words but
// were not scored in this query (the reference reads their stale value) and
// overwritten for the scored ones.  Returns the number of candidates.
int orbo_detect_relocalization_candidates(const int32_t* q_words, const double* q_vals, int nq, int nkf,
                                          const int32_t* bow_off, const int32_t* bow_words, const double* bow_vals,
                                          int nwords, const int32_t* inv_off, const int32_t* inv_kf,
                                          const int32_t* cov_off, const int32_t* cov_kf, const int32_t* kf_map,
                                          int32_t map_id, float* reloc_score, int32_t* cand, int cap) {
    std::vector<int> reloc_query(nkf, 0), reloc_words(nkf, 0);
    const int qid = 1;
    std::list<int> sharing;                                                          // :735-757
    for (int r = 0; r < nq; ++r) {
        const int w = q_words[r];
        if (w < 0 || w >= nwords) return ORB_ERR_PARAM;
        for (int e = inv_off[w]; e < inv_off[w + 1]; ++e) {
            const int kf = inv_kf[e];
            if (reloc_query[kf] != qid) {
                reloc_words[kf] = 0;
                reloc_query[kf] = qid;
                sharing.push_back(kf);
            }
            reloc_words[kf]++;
        }
    }
    if (sharing.empty()) return 0;
    int maxCommonWords = 0;                                                          // :762-767
    for (int kf : sharing) maxCommonWords = std::max(maxCommonWords, reloc_words[kf]);
    const int minCommonWords = maxCommonWords * 0.8f;
    std::list<std::pair<float, int>> score_match;                                   // :771-787
    for (int kf : sharing) {
        if (reloc_words[kf] > minCommonWords) {
            // L1Scoring::score (ScoringObject.cpp): common words in order
            double sc = 0;
            int i = 0, j = bow_off[kf];
            const int j1 = bow_off[kf + 1];
            while (i < nq && j < j1) {
                if (q_words[i] == bow_words[j]) {
                    const double vi = q_vals[i], wi = bow_vals[j];
                    sc += std::fabs(vi - wi) - std::fabs(vi) - std::fabs(wi);
                    ++i;
                    ++j;
                } else if (q_words[i] < bow_words[j]) {
                    ++i;
                } else {
                    ++j;
                }
            }
            const float si = (float)(-sc / 2.0);
            reloc_score[kf] = si;
            score_match.push_back(std::make_pair(si, kf));
        }
    }
    if (score_match.empty()) return 0;
    std::list<std::pair<float, int>> acc_match;                                     // :792-819
    float bestAccScore = 0;
    for (auto& it : score_match) {
        const int kfi = it.second;
        float bestScore = it.first, accScore = bestScore;
        int best_kf = kfi;
        for (int e = cov_off[kfi]; e < cov_off[kfi + 1]; ++e) {
            const int kf2 = cov_kf[e];
            if (reloc_query[kf2] != qid) continue;
            accScore += reloc_score[kf2];
            if (reloc_score[kf2] > bestScore) {
                best_kf = kf2;
                bestScore = reloc_score[kf2];
            }
        }
        acc_match.push_back(std::make_pair(accScore, best_kf));
        if (accScore > bestAccScore) bestAccScore = accScore;
    }
    const float minScoreToRetain = 0.75f * bestAccScore;                            // :822-842
    std::vector<char> added(nkf, 0);
    int n = 0;
    for (auto& it : acc_match) {
        if (it.first > minScoreToRetain) {
            const int kf = it.second;
            if (kf_map[kf] != map_id) continue;
            if (!added[kf]) {
                if (n < cap) cand[n] = kf;
                ++n;
                added[kf] = 1;
            }
        }
    }
    return n;
}

// ORBmatcher::Fuse(pKF, vpMapPoints, th) (src/ORBmatcher.cc:1148-1331), the
// matching of each point (pinhole keyframe); geometry from the caller, fma =
// the reference build's contraction (e2 = fma(er, er, fma(ex, ex, ey*ey))).
int orbo_fuse(const orbm_frame* kf, const float* inv_sigma2, int nmp, const uint8_t* valid, const float* u,
              const float* v, const float* ur, const int32_t* level, const uint8_t* desc, float th, int fma,
              int32_t* best_idx, int32_t* best_dist) {
    Grid grid(kf);
    int nf = 0;
    for (int i = 0; i < nmp; ++i) {
        best_idx[i] = -1;
        best_dist[i] = -1;
        if (!valid[i]) continue;
        const int pl = level[i];
        const float radius = th * kf->scale_factors[pl];                             // :1242
        const std::vector<int> cand = grid.area(u[i], v[i], radius, -1, -1);
        if (cand.empty()) continue;
        int bestDist = 256, bestIdx = -1;
        for (int idx : cand) {                                                       // :1255-1308
            const orb_keypoint& kp = kf->kps[idx];
            const int kl = kp.octave;
            if (kl < pl - 1 || kl > pl) continue;
            const float ex = u[i] - kp.x, ey = v[i] - kp.y;
            if (kf->u_right && kf->u_right[idx] >= 0) {
                const float er = ur[i] - kf->u_right[idx];
                const float e2 = fma ? std::fmaf(er, er, std::fmaf(ex, ex, ey * ey)) : ex * ex + ey * ey + er * er;
                if (e2 * inv_sigma2[kl] > 7.8) continue;
            } else {
                const float e2 = fma ? std::fmaf(ex, ex, ey * ey) : ex * ex + ey * ey;
                if (e2 * inv_sigma2[kl] > 5.99) continue;
            }
            const int dist = hamming(desc + (size_t)i * 32, kf->desc + (size_t)idx * 32);
            if (dist < bestDist) { bestDist = dist; bestIdx = idx; }
        }
        if (bestDist <= kThLow) {
            best_idx[i] = bestIdx;
            best_dist[i] = bestDist;
            ++nf;
        }
    }
    return nf;
}

// ORBmatcher::SearchForTriangulation (src/ORBmatcher.cc:907-1146), pinhole
// keyframes: F12 row-major, ep = epipole of KF1's centre in KF2.
int orbo_search_for_triangulation(const orbm_frame* kf1, const orbm_featvec* fv1, const uint8_t* has_mp1,
                                  const orbm_frame* kf2, const orbm_featvec* fv2, const uint8_t* has_mp2,
                                  const float* F, float ep_x, float ep_y, const float* sigma2_2, int only_stereo,
                                  int coarse, int check_ori, int fma, int32_t* matches12) {
    auto lin = [&](float x, float a, float y, float b, float c) {
        return fma ? std::fmaf(x, a, y * b) + c : x * a + y * b + c;
    };
    auto sq = [&](float a, float b) { return fma ? std::fmaf(a, a, b * b) : a * a + b * b; };
    int nmatches = 0;
    std::vector<char> matched2(kf2->n, 0);                 // vbMatched2: never set in the reference
    for (int i = 0; i < kf1->n; ++i) matches12[i] = -1;
    std::vector<int> hist[kHisto];
    int a = 0, b = 0;
    while (a < fv1->nnodes && b < fv2->nnodes) {
        if (fv1->node_ids[a] == fv2->node_ids[b]) {
            for (int p = fv1->offsets[a]; p < fv1->offsets[a + 1]; ++p) {
                const int idx1 = (int)fv1->idx[p];
                if (has_mp1[idx1]) continue;
                const bool st1 = kf1->u_right && kf1->u_right[idx1] >= 0;
                if (only_stereo && !st1) continue;
                const orb_keypoint& kp1 = kf1->kps[idx1];
                int bestDist = kThLow, bestIdx2 = -1;
                for (int q = fv2->offsets[b]; q < fv2->offsets[b + 1]; ++q) {
                    const int idx2 = (int)fv2->idx[q];
                    if (matched2[idx2] || has_mp2[idx2]) continue;
                    const bool st2 = kf2->u_right && kf2->u_right[idx2] >= 0;
                    if (only_stereo && !st2) continue;
                    const int dist = hamming(kf1->desc + (size_t)idx1 * 32, kf2->desc + (size_t)idx2 * 32);
                    if (dist > kThLow || dist > bestDist) continue;
                    const orb_keypoint& kp2 = kf2->kps[idx2];
                    if (!st1 && !st2) {
                        const float distex = ep_x - kp2.x, distey = ep_y - kp2.y;
                        if (sq(distex, distey) < 100 * kf2->scale_factors[kp2.octave]) continue;
                    }
                    bool ok = coarse != 0;
                    if (!ok) {                                                       // Pinhole.cpp:115-128
                        const float la = lin(kp1.x, F[0], kp1.y, F[3], F[6]);
                        const float lb = lin(kp1.x, F[1], kp1.y, F[4], F[7]);
                        const float lc = lin(kp1.x, F[2], kp1.y, F[5], F[8]);
                        const float num = lin(la, kp2.x, lb, kp2.y, lc);
                        const float den = sq(la, lb);
                        if (den != 0) ok = num * num / den < 3.84 * sigma2_2[kp2.octave];
                    }
                    if (ok) { bestIdx2 = idx2; bestDist = dist; }
                }
                if (bestIdx2 >= 0) {
                    matches12[idx1] = bestIdx2;
                    ++nmatches;
                    if (check_ori) hist[rot_bin(kp1.angle, kf2->kps[bestIdx2].angle)].push_back(idx1);
                }
            }
            ++a;
            ++b;
        } else if (fv1->node_ids[a] < fv2->node_ids[b]) {
            a = (int)(std::lower_bound(fv1->node_ids + a, fv1->node_ids + fv1->nnodes, fv2->node_ids[b]) - fv1->node_ids);
        } else {
            b = (int)(std::lower_bound(fv2->node_ids + b, fv2->node_ids + fv2->nnodes, fv1->node_ids[a]) - fv2->node_ids);
        }
    }
    if (check_ori) {
        int i1, i2, i3;
        three_maxima(hist, i1, i2, i3);
        for (int i = 0; i < kHisto; ++i) {
            if (i == i1 || i == i2 || i == i3) continue;
            for (int idx1 : hist[i]) { matches12[idx1] = -1; --nmatches; }
        }
    }
    return nmatches;
}

// SearchForTriangulation with the per-candidate geometry delegated to
// check(ctx, idx1, idx2) (the epipole test + GeometricCamera::epipolarConstrain
// of src/ORBmatcher.cc:1014-1076): the reference loop itself, the callback in
// place of the two tests.
int orbo_search_for_triangulation_checked(const orbm_frame* kf1, const orbm_featvec* fv1, const uint8_t* has_mp1,
                                          const orbm_frame* kf2, const orbm_featvec* fv2, const uint8_t* has_mp2,
                                          int only_stereo, int check_ori, int (*check)(void*, int, int), void* ctx,
                                          int32_t* matches12) {
    int nmatches = 0;
    for (int i = 0; i < kf1->n; ++i) matches12[i] = -1;
    std::vector<int> hist[kHisto];
    int a = 0, b = 0;
    while (a < fv1->nnodes && b < fv2->nnodes) {
        if (fv1->node_ids[a] == fv2->node_ids[b]) {
            for (int p = fv1->offsets[a]; p < fv1->offsets[a + 1]; ++p) {
                const int idx1 = (int)fv1->idx[p];
                if (has_mp1[idx1]) continue;
                const bool st1 = kf1->u_right && kf1->u_right[idx1] >= 0;
                if (only_stereo && !st1) continue;
                int bestDist = kThLow, bestIdx2 = -1;
                for (int q = fv2->offsets[b]; q < fv2->offsets[b + 1]; ++q) {
                    const int idx2 = (int)fv2->idx[q];
                    if (has_mp2[idx2]) continue;                       // vbMatched2 is never set
                    const bool st2 = kf2->u_right && kf2->u_right[idx2] >= 0;
                    if (only_stereo && !st2) continue;
                    const int dist = hamming(kf1->desc + (size_t)idx1 * 32, kf2->desc + (size_t)idx2 * 32);
                    if (dist > kThLow || dist > bestDist) continue;
                    if (check(ctx, idx1, idx2)) { bestIdx2 = idx2; bestDist = dist; }
                }
                if (bestIdx2 >= 0) {
                    matches12[idx1] = bestIdx2;
                    ++nmatches;
                    if (check_ori) hist[rot_bin(kf1->kps[idx1].angle, kf2->kps[bestIdx2].angle)].push_back(idx1);
                }
            }
            ++a;
            ++b;
        } else if (fv1->node_ids[a] < fv2->node_ids[b]) {
            a = (int)(std::lower_bound(fv1->node_ids + a, fv1->node_ids + fv1->nnodes, fv2->node_ids[b]) - fv1->node_ids);
        } else {
            b = (int)(std::lower_bound(fv2->node_ids + b, fv2->node_ids + fv2->nnodes, fv1->node_ids[a]) - fv2->node_ids);
        }
    }
    if (check_ori) {
        int i1, i2, i3;
        three_maxima(hist, i1, i2, i3);
        for (int i = 0; i < kHisto; ++i) {
            if (i == i1 || i == i2 || i == i3) continue;
            for (int idx1 : hist[i]) { matches12[idx1] = -1; --nmatches; }
        }
    }
    return nmatches;
}

// MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:368-397) per point
// of a CSR batch: the N x N distance matrix, each row sorted, the median at
// 0.5 * (N - 1), the first row with the least median.
int orbo_compute_distinctive_descriptors(int npoints, const int32_t* off, const uint8_t* desc, int32_t* best) {
    for (int p = 0; p < npoints; ++p) {
        const int b = off[p];
        const size_t N = (size_t)(off[p + 1] - b);
        if (N == 0) { best[p] = -1; continue; }
        std::vector<float> dist(N * N);
        for (size_t i = 0; i < N; ++i) {
            dist[i * N + i] = 0;
            for (size_t j = i + 1; j < N; ++j) {
                const int d = hamming(desc + (size_t)(b + i) * 32, desc + (size_t)(b + j) * 32);
                dist[i * N + j] = d;
                dist[j * N + i] = d;
            }
        }
        int bestMedian = INT32_MAX, bestIdx = 0;
        for (size_t i = 0; i < N; ++i) {
            std::vector<int> v(dist.begin() + i * N, dist.begin() + (i + 1) * N);
            std::sort(v.begin(), v.end());
            const int median = v[(size_t)(0.5 * (N - 1))];
            if (median < bestMedian) { bestMedian = median; bestIdx = (int)i; }
        }
        best[p] = bestIdx;
    }
    return 0;
}


// ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vpMatches12)
// (src/ORBmatcher.cc:765-905), NLeft == -1.  valid = MapPoint != NULL && !isBad.
int orbo_search_by_bow_kf(const orbm_frame* k1, const orbm_featvec* fv1, const uint8_t* valid1,
                          const orbm_frame* k2, const orbm_featvec* fv2, const uint8_t* valid2, float ratio,
                          int check_ori, int32_t* m12) {
    for (int i = 0; i < k1->n; ++i) m12[i] = -1;
    std::vector<char> matched2(k2->n, 0);
    std::vector<int> hist[kHisto];
    int nm = 0;
    int a = 0, b = 0;
    while (a < fv1->nnodes && b < fv2->nnodes) {
        if (fv1->node_ids[a] == fv2->node_ids[b]) {
            for (int p = fv1->offsets[a]; p < fv1->offsets[a + 1]; ++p) {
                const int idx1 = (int)fv1->idx[p];
                if (!valid1[idx1]) continue;                                        // :804-808
                const uint8_t* d1 = k1->desc + (size_t)idx1 * 32;
                int best1 = 256, bestIdx2 = -1, best2 = 256;
                for (int q = fv2->offsets[b]; q < fv2->offsets[b + 1]; ++q) {
                    const int idx2 = (int)fv2->idx[q];
                    if (matched2[idx2] || !valid2[idx2]) continue;                  // :826-830
                    const int dist = hamming(d1, k2->desc + (size_t)idx2 * 32);
                    if (dist < best1) { best2 = best1; best1 = dist; bestIdx2 = idx2; }
                    else if (dist < best2) best2 = dist;
                }
                if (best1 < kThLow) {                                               // :848
                    if ((float)best1 < ratio * (float)best2) {
                        m12[idx1] = bestIdx2;
                        matched2[bestIdx2] = 1;
                        if (check_ori) hist[rot_bin(k1->kps[idx1].angle, k2->kps[bestIdx2].angle)].push_back(idx1);
                        ++nm;
                    }
                }
            }
            ++a;
            ++b;
        } else if (fv1->node_ids[a] < fv2->node_ids[b]) {
            a = (int)(std::lower_bound(fv1->node_ids + a, fv1->node_ids + fv1->nnodes, fv2->node_ids[b]) - fv1->node_ids);
        } else {
            b = (int)(std::lower_bound(fv2->node_ids + b, fv2->node_ids + fv2->nnodes, fv1->node_ids[a]) - fv2->node_ids);
        }
    }
    if (check_ori) {
        int i1, i2, i3;
        three_maxima(hist, i1, i2, i3);
        for (int i = 0; i < kHisto; ++i) {
            if (i == i1 || i == i2 || i == i3) continue;
            for (int idx1 : hist[i]) { m12[idx1] = -1; --nm; }
        }
    }
    return nm;
}

// ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, sAlreadyFound,
// th, ORBdist) (src/ORBmatcher.cc:1889-2010), Nleft == -1; geometry from the
// caller.  owner: -1 = mvpMapPoints[i2] NULL, else occupied.
int orbo_search_by_projection_kf(const orbm_frame* f, int nq, const uint8_t* valid, const float* u, const float* v,
                                 const int32_t* level, const float* kf_angle, const uint8_t* desc, float th,
                                 int orb_dist, int check_ori, int32_t* owner) {
    Grid g(f);
    int nm = 0;
    std::vector<int> hist[kHisto];
    for (int i = 0; i < nq; ++i) {
        if (!valid[i]) continue;
        const int pl = level[i];
        const float radius = th * f->scale_factors[pl];                             // :1937
        const std::vector<int> cand = g.area(u[i], v[i], radius, pl - 1, pl + 1);   // :1939
        if (cand.empty()) continue;
        int bestDist = 256, bestIdx2 = -1;
        for (int i2 : cand) {
            if (owner[i2] != -1) continue;                                          // :1952
            const int dist = hamming(desc + (size_t)i * 32, f->desc + (size_t)i2 * 32);
            if (dist < bestDist) { bestDist = dist; bestIdx2 = i2; }
        }
        if (bestDist <= orb_dist && bestIdx2 >= 0) {                                // :1966
            owner[bestIdx2] = i;
            ++nm;
            if (check_ori) hist[rot_bin(kf_angle[i], f->kps[bestIdx2].angle)].push_back(bestIdx2);
        }
    }
    if (check_ori) {
        int i1, i2, i3;
        three_maxima(hist, i1, i2, i3);
        for (int k = 0; k < kHisto; ++k) {
            if (k == i1 || k == i2 || k == i3) continue;
            for (int j : hist[k]) { owner[j] = -1; --nm; }
        }
    }
    return nm;
}

// ORBmatcher::SearchByProjection(KeyFrame* pKF, Sim3 Scw, vpPoints, vpMatched, th,
// ratioHamming) (src/ORBmatcher.cc:427-532; the vpPointsKFs twin :534-646 matches
// identically); geometry from the caller.  matched: -1 = NULL, else occupied.
int orbo_search_by_projection_sim3(const orbm_frame* kf, int nq, const uint8_t* valid, const float* u,
                                   const float* v, const int32_t* level, const uint8_t* desc, float th,
                                   float ratio_hamming, int32_t* matched) {
    Grid g(kf);
    int nm = 0;
    for (int i = 0; i < nq; ++i) {
        if (!valid[i]) continue;
        const int pl = level[i];
        const float radius = th * kf->scale_factors[pl];                            // :489
        const std::vector<int> cand = g.area(u[i], v[i], radius, -1, -1);          // :491
        if (cand.empty()) continue;
        int bestDist = 256, bestIdx = -1;
        for (int idx : cand) {
            if (matched[idx] != -1) continue;                                       // :504
            const int kl = kf->kps[idx].octave;
            if (kl < pl - 1 || kl > pl) continue;                                   // :509
            const int dist = hamming(desc + (size_t)i * 32, kf->desc + (size_t)idx * 32);
            if (dist < bestDist) { bestDist = dist; bestIdx = idx; }
        }
        if ((float)bestDist <= (float)kThLow * ratio_hamming && bestIdx >= 0) {     // :523
            matched[bestIdx] = i;
            ++nm;
        }
    }
    return nm;
}

namespace {
// one direction of SearchBySim3 / the matching of Fuse(Sim3): first least
// distance over the levels pl-1 .. pl of KeyFrame::GetFeaturesInArea.
int best_in_area(const Grid& g, const orbm_frame* kf, float x, float y, int pl, const uint8_t* d, float th,
                 int& bestDist) {
    const float radius = th * kf->scale_factors[pl];
    const std::vector<int> cand = g.area(x, y, radius, -1, -1);
    bestDist = INT_MAX;
    int bestIdx = -1;
    for (int idx : cand) {
        const int kl = kf->kps[idx].octave;
        if (kl < pl - 1 || kl > pl) continue;
        const int dist = hamming(d, kf->desc + (size_t)idx * 32);
        if (dist < bestDist) { bestDist = dist; bestIdx = idx; }
    }
    return bestIdx;
}
}  // namespace

// ORBmatcher::SearchBySim3 (src/ORBmatcher.cc:1457-1674), pinhole keyframes,
// projections and predicted levels from the caller.  m12: new mutual matches.
int orbo_search_by_sim3(const orbm_frame* kf1, const orbm_frame* kf2, const uint8_t* valid1, const float* u1,
                        const float* v1, const int32_t* level1, const uint8_t* mdesc1, const uint8_t* valid2,
                        const float* u2, const float* v2, const int32_t* level2, const uint8_t* mdesc2, float th,
                        int32_t* m12) {
    Grid g1(kf1), g2(kf2);
    std::vector<int> vnMatch1(kf1->n, -1), vnMatch2(kf2->n, -1);
    for (int i1 = 0; i1 < kf1->n; ++i1) {                                           // :1496-1573
        if (!valid1[i1]) continue;
        int bd;
        const int bi = best_in_area(g2, kf2, u1[i1], v1[i1], level1[i1], mdesc1 + (size_t)i1 * 32, th, bd);
        if (bd <= kThHigh) vnMatch1[i1] = bi;
    }
    for (int i2 = 0; i2 < kf2->n; ++i2) {                                           // :1576-1653
        if (!valid2[i2]) continue;
        int bd;
        const int bi = best_in_area(g1, kf1, u2[i2], v2[i2], level2[i2], mdesc2 + (size_t)i2 * 32, th, bd);
        if (bd <= kThHigh) vnMatch2[i2] = bi;
    }
    int nFound = 0;
    for (int i1 = 0; i1 < kf1->n; ++i1) {                                           // :1658-1671
        m12[i1] = -1;
        const int idx2 = vnMatch1[i1];
        if (idx2 >= 0 && vnMatch2[idx2] == i1) { m12[i1] = idx2; ++nFound; }
    }
    return nFound;
}

// ORBmatcher::Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (src/ORBmatcher.cc:1340-1455),
// the matching of each point; geometry from the caller.
int orbo_fuse_sim3(const orbm_frame* kf, int nmp, const uint8_t* valid, const float* u, const float* v,
                   const int32_t* level, const uint8_t* desc, float th, int32_t* best_idx, int32_t* best_dist) {
    Grid g(kf);
    int nf = 0;
    for (int i = 0; i < nmp; ++i) {
        best_idx[i] = -1;
        best_dist[i] = -1;
        if (!valid[i]) continue;
        int bd;
        const int bi = best_in_area(g, kf, u[i], v[i], level[i], desc + (size_t)i * 32, th, bd);
        if (bd <= kThLow) { best_idx[i] = bi; best_dist[i] = bd; ++nf; }            // :1437
    }
    return nf;
}


// ---- fisheye stereo frames (Nleft != -1) ------------------------------------
// The frame is the combined keypoint array [mvKeys (Nleft); mvKeysRight] with N
// descriptor rows; mGrid holds the left keypoints, mGridRight the right ones by
// local index (Frame.cc:385-416), queried with bRight (Frame.cc:657-723).
namespace {
orbm_frame sub_frame(const orbm_frame* f, int b, int e) {
    orbm_frame s = *f;
    s.n = e - b;
    s.kps = f->kps + b;
    s.desc = f->desc + (size_t)b * 32;
    s.u_right = nullptr;
    return s;
}
float radius_by_viewing_cos(float c) { return c > 0.998 ? 2.5f : 4.0f; }   // ORBmatcher.cc:215-221
}  // namespace

// ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) (ORBmatcher.cc:223-425) with
// F.Nleft = nleft (>= 0): left and right best/second over each node's frame
// features (:296-323); the right match is taken only inside the left's
// `bestDist1 <= TH_LOW` and ignores the ratio (`|| true`, :357-359).
int orbo_search_by_bow_fisheye(const orbm_frame* kf, const orbm_featvec* kfv, const uint8_t* kf_valid,
                               const orbm_frame* f, const orbm_featvec* ffv, int nleft, float ratio, int check_ori,
                               int32_t* match) {
    for (int i = 0; i < f->n; ++i) match[i] = -1;
    std::vector<int> hist[kHisto];
    int nm = 0, a = 0, b = 0;
    while (a < kfv->nnodes && b < ffv->nnodes) {
        const uint32_t na = kfv->node_ids[a], nb = ffv->node_ids[b];
        if (na == nb) {
            for (int p = kfv->offsets[a]; p < kfv->offsets[a + 1]; ++p) {
                const int ikf = (int)kfv->idx[p];
                if (!kf_valid[ikf]) continue;
                const uint8_t* dk = kf->desc + (size_t)ikf * 32;
                int b1 = 256, bi = -1, b2 = 256, b1r = 256, bir = -1, b2r = 256;
                for (int q = ffv->offsets[b]; q < ffv->offsets[b + 1]; ++q) {
                    const int jf = (int)ffv->idx[q];
                    if (match[jf] >= 0) continue;
                    const int dist = hamming(dk, f->desc + (size_t)jf * 32);
                    if (jf < nleft && dist < b1) { b2 = b1; b1 = dist; bi = jf; }
                    else if (jf < nleft && dist < b2) b2 = dist;
                    if (jf >= nleft && dist < b1r) { b2r = b1r; b1r = dist; bir = jf; }
                    else if (jf >= nleft && dist < b2r) b2r = dist;
                }
                if (b1 <= kThLow) {
                    if ((float)b1 < ratio * (float)b2) {
                        match[bi] = ikf;
                        if (check_ori) hist[rot_bin(kf->kps[ikf].angle, f->kps[bi].angle)].push_back(bi);
                        ++nm;
                    }
                    if (b1r <= kThLow) {
                        match[bir] = ikf;
                        if (check_ori) hist[rot_bin(kf->kps[ikf].angle, f->kps[bir].angle)].push_back(bir);
                        ++nm;
                    }
                }
            }
            ++a; ++b;
        } else if (na < nb) {
            a = (int)(std::lower_bound(kfv->node_ids + a, kfv->node_ids + kfv->nnodes, nb) - kfv->node_ids);
        } else {
            b = (int)(std::lower_bound(ffv->node_ids + b, ffv->node_ids + ffv->nnodes, na) - ffv->node_ids);
        }
    }
    if (check_ori) {
        int i1, i2, i3;
        three_maxima(hist, i1, i2, i3);
        for (int i = 0; i < kHisto; ++i) {
            if (i == i1 || i == i2 || i == i3) continue;
            for (int j : hist[i]) { match[j] = -1; --nm; }
        }
    }
    return nm;
}

// ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th, bFarPoints,
// thFarPoints) (ORBmatcher.cc:43-213) with F.Nleft = nleft: left search on
// mGrid, then the right camera on mGridRight (:144-210; its radius has no th
// factor), stereo partners via mvLeftToRightMatch / mvRightToLeftMatch; a
// left best failing the ratio test skips the point's right search (:125-126).
int orbo_search_by_projection_mps_fisheye(const orbm_frame* f, int nleft, const int32_t* l2r, const int32_t* r2l,
                                          const orbm_mappoints* mp, const orbm_mappoints_right* mr, float th,
                                          int far_points, float th_far, float ratio, int32_t* owner,
                                          const uint8_t* blocked) {
    const orbm_frame fl = sub_frame(f, 0, nleft), fr = sub_frame(f, nleft, f->n);
    Grid gl(&fl), gr(&fr);
    int nm = 0;
    const bool factor = th != 1.0;
    auto slot_blocked = [&](int idx) {
        const int o = owner[idx];
        if (o == -1) return false;
        if (o <= -2) return blocked[idx] != 0;
        return mp->has_obs[o] != 0;
    };
    for (int i = 0; i < mp->n; ++i) {
        if (!mp->in_view[i] && !mr->in_view[i]) continue;
        if (far_points && mp->track_depth[i] > th_far) continue;
        const uint8_t* dm = mp->desc + (size_t)i * 32;
        if (mp->in_view[i]) {
            const int lvl = mp->level[i];
            float r = radius_by_viewing_cos(mp->view_cos[i]);
            if (factor) r *= th;
            const std::vector<int> cand = gl.area(mp->proj_x[i], mp->proj_y[i], r * f->scale_factors[lvl], lvl - 1, lvl);
            if (!cand.empty()) {
                int best = 256, bl = -1, best2 = 256, bl2 = -1, bi = -1;
                for (int idx : cand) {
                    if (slot_blocked(idx)) continue;
                    const int dist = hamming(dm, f->desc + (size_t)idx * 32);
                    if (dist < best) { best2 = best; best = dist; bl2 = bl; bl = f->kps[idx].octave; bi = idx; }
                    else if (dist < best2) { bl2 = f->kps[idx].octave; best2 = dist; }
                }
                if (best <= kThHigh) {
                    if (bl == bl2 && best > ratio * best2) continue;
                    if (bl != bl2 || best <= ratio * best2) {
                        owner[bi] = i;
                        if (l2r[bi] != -1) { owner[l2r[bi] + nleft] = i; ++nm; }
                        ++nm;
                    }
                }
            }
        }
        if (mr->in_view[i]) {
            const int lvl = mr->level[i];
            if (lvl != -1) {
                const float r = radius_by_viewing_cos(mr->view_cos[i]);
                const std::vector<int> cand = gr.area(mr->proj_x[i], mr->proj_y[i], r * f->scale_factors[lvl], lvl - 1, lvl);
                if (cand.empty()) continue;
                int best = 256, bl = -1, best2 = 256, bl2 = -1, bi = -1;
                for (int idx : cand) {
                    if (slot_blocked(idx + nleft)) continue;
                    const int dist = hamming(dm, f->desc + (size_t)(idx + nleft) * 32);
                    if (dist < best) { best2 = best; best = dist; bl2 = bl; bl = f->kps[idx + nleft].octave; bi = idx; }
                    else if (dist < best2) { bl2 = f->kps[idx + nleft].octave; best2 = dist; }
                }
                if (best <= kThHigh) {
                    if (bl == bl2 && best > ratio * best2) continue;
                    if (r2l[bi] != -1) { owner[r2l[bi]] = i; ++nm; }
                    owner[bi + nleft] = i;
                    ++nm;
                }
            }
        }
    }
    return nm;
}

// ORBmatcher::SearchByProjection(Frame& Current, const Frame& Last, th, bMono)
// (ORBmatcher.cc:1676-1887) with CurrentFrame.Nleft = nleft: after the left
// search (reached only when its candidate list is not empty) the point is
// searched again in the right camera (projection ur/vr from the caller,
// GetRelativePoseTrl, :1794-1859) with the same octave window.
int orbo_search_by_projection_last_fisheye(const orbm_frame* cur, int nleft, int nlast, const uint8_t* valid,
                                           const float* u, const float* v, const float* ur, const float* vr,
                                           const int32_t* last_octave, const float* last_angle,
                                           const uint8_t* has_obs, const uint8_t* last_desc, float th, int mode,
                                           int check_ori, int32_t* owner, const uint8_t* blocked) {
    const orbm_frame fl = sub_frame(cur, 0, nleft), fr = sub_frame(cur, nleft, cur->n);
    Grid gl(&fl), gr(&fr);
    int nm = 0;
    std::vector<int> hist[kHisto];
    auto slot_blocked = [&](int idx) {
        const int o = owner[idx];
        if (o == -1) return false;
        if (o <= -2) return blocked[idx] != 0;
        return has_obs[o] != 0;
    };
    auto area = [&](const Grid& g, float x, float y, float radius, int oct) {
        if (mode == 1) return g.area(x, y, radius, oct, -1);
        if (mode == 2) return g.area(x, y, radius, 0, oct);
        return g.area(x, y, radius, oct - 1, oct + 1);
    };
    for (int i = 0; i < nlast; ++i) {
        if (!valid[i]) continue;
        const int oct = last_octave[i];
        const float radius = th * cur->scale_factors[oct];
        const uint8_t* dm = last_desc + (size_t)i * 32;
        std::vector<int> cand = area(gl, u[i], v[i], radius, oct);
        if (cand.empty()) continue;
        int best = 256, bi = -1;
        for (int i2 : cand) {
            if (slot_blocked(i2)) continue;
            const int dist = hamming(dm, cur->desc + (size_t)i2 * 32);
            if (dist < best) { best = dist; bi = i2; }
        }
        if (best <= kThHigh) {
            owner[bi] = i;
            ++nm;
            if (check_ori) hist[rot_bin(last_angle[i], cur->kps[bi].angle)].push_back(bi);
        }
        cand = area(gr, ur[i], vr[i], radius, oct);
        best = 256;
        bi = -1;
        for (int i2 : cand) {
            if (slot_blocked(i2 + nleft)) continue;
            const int dist = hamming(dm, cur->desc + (size_t)(i2 + nleft) * 32);
            if (dist < best) { best = dist; bi = i2; }
        }
        if (best <= kThHigh) {
            owner[bi + nleft] = i;
            ++nm;
            if (check_ori) hist[rot_bin(last_angle[i], cur->kps[bi + nleft].angle)].push_back(bi + nleft);
        }
    }
    if (check_ori) {
        int a, b, c;
        three_maxima(hist, a, b, c);
        for (int k = 0; k < kHisto; ++k) {
            if (k == a || k == b || k == c) continue;
            for (int j : hist[k]) { owner[j] = -1; --nm; }
        }
    }
    return nm;
}

}  // extern "C"
