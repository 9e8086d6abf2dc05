// Sanitizer driver (tests/test_sanitizers.py; SURVEY.md §5 "ASan/TSan on the
// CPU reference build"): the host code of the path that runs without a
// device, built twice by tests/native/Makefile --
//   bin/san_driver   -fsanitize=address,undefined -fno-sanitize-recover=all
//   bin/tsan_driver  -fsanitize=thread
// and linked from the sources themselves:
//   * oracle/orb_oracle.cpp (the CPU checker): extraction of synthetic frames
//     at the configs' sizes and lapping areas, then every matcher entry point
//     on the results (SearchForInitialization, SearchByBoW, both projections,
//     Fuse, SearchByBoW(KF, KF), Sim3 / KF projections, knnMatch, the
//     distinctive descriptor);
//   * orb_slam3_vio_fixes_amd/csrc/vocab.cpp (product host code): the text
//     vocabulary parser on every file of <dir> (well-formed, truncated and
//     malformed files written by the test), BowVector / FeatureVector
//     assembly and the six scores;
//   * orb_slam3_vio_fixes_amd/csrc/host_gather.h (product host code):
//     orbx_extract_batch's threaded gather of the frames into one buffer.
// mode "all" runs everything on one thread; "threads" runs the oracle
// extraction on 4 threads with a handle each and the gather over 8 threads
// (the TSan build).  A sanitizer report aborts with a non-zero exit.
//
//   san_driver <all|threads> <vocab dir>
#include "orb_mi355x.h"
#include "../../orb_slam3_vio_fixes_amd/csrc/host_gather.h"

#include <dirent.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* orbo_create(const orbx_params* p);
void orbo_destroy(void* h);
int orbo_extract(void* h, const uint8_t* img, int w, int hh, size_t step, int lap0, int lap1, orb_keypoint* kps,
                 uint8_t* desc, int cap, int* n_out, int* mono_out);
int orbo_get_tables(void* h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2, int32_t* nfeat,
                    int32_t* umax);
int orbo_search_for_initialization(const orbm_frame* f1, const orbm_frame* f2, float* prev, int window, float ratio,
                                   int check_ori, int32_t* m12);
int orbo_search_by_bow(const orbm_frame* kf, const orbm_featvec* kfv, const uint8_t* kf_valid, const orbm_frame* f,
                       const orbm_featvec* ffv, float ratio, int check_ori, int32_t* match);
int orbo_search_by_projection_mps(const orbm_frame* f, const orbm_mappoints* mp, float th, int far_points,
                                  float th_far, float ratio, int32_t* owner, const uint8_t* blocked);
int orbo_search_by_projection_last(const orbm_frame* cur, int nlast, const uint8_t* valid, const float* u,
                                   const float* v, const float* ur, const int32_t* last_octave,
                                   const float* last_angle, const uint8_t* has_obs, const uint8_t* last_desc,
                                   float th, int mode, int check_ori, int32_t* owner, const uint8_t* blocked);
int orbo_fuse(const orbm_frame* kf, const float* inv_sigma2, int nmp, const uint8_t* valid, const float* u,
              const float* v, const float* ur, const int32_t* level, const uint8_t* desc, float th, int fma,
              int32_t* best_idx, int32_t* best_dist);
int orbo_search_by_bow_kf(const orbm_frame* k1, const orbm_featvec* fv1, const uint8_t* valid1,
                          const orbm_frame* k2, const orbm_featvec* fv2, const uint8_t* valid2, float ratio,
                          int check_ori, int32_t* m12);
int orbo_search_by_projection_kf(const orbm_frame* f, int nq, const uint8_t* valid, const float* u, const float* v,
                                 const int32_t* level, const float* kf_angle, const uint8_t* desc, float th,
                                 int orb_dist, int check_ori, int32_t* owner);
int orbo_search_by_projection_sim3(const orbm_frame* kf, int nq, const uint8_t* valid, const float* u,
                                   const float* v, const int32_t* level, const uint8_t* desc, float th,
                                   float ratio_hamming, int32_t* matched);
int orbo_search_by_sim3(const orbm_frame* kf1, const orbm_frame* kf2, const uint8_t* valid1, const float* u1,
                        const float* v1, const int32_t* level1, const uint8_t* mdesc1, const uint8_t* valid2,
                        const float* u2, const float* v2, const int32_t* level2, const uint8_t* mdesc2, float th,
                        int32_t* m12);
int orbo_fuse_sim3(const orbm_frame* kf, int nmp, const uint8_t* valid, const float* u, const float* v,
                   const int32_t* level, const uint8_t* desc, float th, int32_t* best_idx, int32_t* best_dist);
int orbo_knn_match2(const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* idx, int32_t* dist);
int orbo_compute_distinctive_descriptors(int npoints, const int32_t* off, const uint8_t* desc, int32_t* best);
}

namespace {

void fail(const char* what, int rc)
{
    std::fprintf(stderr, "%s returned %d\n", what, rc);
    std::exit(3);
}

// splitmix64: deterministic synthetic data
struct Rng {
    uint64_t s;
    uint64_t next()
    {
        uint64_t z = (s += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    }
    int uni(int n) { return (int)(next() % (uint64_t)n); }
    float unif() { return (float)((next() >> 40) * (1.0 / 16777216.0)); }
};

// rectangles and blobs on a ramp plus noise, with a flat patch (the minThFAST
// fallback) and saturated pixels
std::vector<uint8_t> image(int w, int h, uint64_t seed)
{
    Rng r{seed};
    std::vector<uint8_t> im((size_t)w * h);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) im[(size_t)y * w + x] = (uint8_t)((x * 97 / w + y * 61 / h) + r.uni(7));
    for (int k = 0; k < 160; ++k) {
        const int x0 = r.uni(w), y0 = r.uni(h), rw = 4 + r.uni(60), rh = 4 + r.uni(60), v = r.uni(256);
        for (int y = y0; y < std::min(h, y0 + rh); ++y)
            for (int x = x0; x < std::min(w, x0 + rw); ++x) im[(size_t)y * w + x] = (uint8_t)v;
    }
    for (int y = h / 3; y < h / 3 + 50 && y < h; ++y)
        for (int x = w / 2; x < w / 2 + 70 && x < w; ++x) im[(size_t)y * w + x] = 128;
    return im;
}

struct Frame {
    std::vector<orb_keypoint> k;
    std::vector<uint8_t> d;
    int w = 0, h = 0;
    std::vector<float> scale;
    orbm_frame view() const
    {
        orbm_frame f{};
        f.n = (int32_t)k.size();
        f.kps = k.data();
        f.desc = d.data();
        f.min_x = 0.f; f.max_x = (float)w; f.min_y = 0.f; f.max_y = (float)h;
        f.grid_inv_w = 64.0f / (float)w;
        f.grid_inv_h = 48.0f / (float)h;
        f.scale_factors = scale.data();
        f.nlevels = (int32_t)scale.size();
        return f;
    }
};

Frame extract(void* ex, int w, int h, uint64_t seed, int lap0, int lap1)
{
    const std::vector<uint8_t> im = image(w, h, seed);
    Frame f;
    f.w = w; f.h = h;
    const int cap = 20000;
    f.k.resize(cap);
    f.d.resize((size_t)cap * 32);
    int n = 0, mono = 0;
    const int rc = orbo_extract(ex, im.data(), w, h, (size_t)w, lap0, lap1, f.k.data(), f.d.data(), cap, &n, &mono);
    if (rc) fail("orbo_extract", rc);
    f.k.resize(n);
    f.d.resize((size_t)n * 32);
    f.scale.resize(8);
    if (orbo_get_tables(ex, f.scale.data(), nullptr, nullptr, nullptr, nullptr, nullptr)) fail("orbo_get_tables", -1);
    return f;
}

orbx_params params(int nfeatures)
{
    orbx_params p{};
    p.nfeatures = nfeatures; p.scale_factor = 1.2f; p.nlevels = 8; p.ini_th_fast = 20; p.min_th_fast = 7;
    p.blur_variant = 0; p.fma_sampling = 1;
    return p;
}

// FeatureVector CSR of per-feature node ids (ascending nodes, ascending features)
struct FV {
    std::vector<uint32_t> nodes, idx;
    std::vector<int32_t> off;
    orbm_featvec c{};
    FV(int n, int nnodes, Rng& r)
    {
        std::vector<std::vector<uint32_t>> by(nnodes);
        for (int i = 0; i < n; ++i) by[r.uni(nnodes)].push_back((uint32_t)i);
        off.push_back(0);
        for (int q = 0; q < nnodes; ++q) {
            if (by[q].empty()) continue;
            nodes.push_back((uint32_t)q);
            idx.insert(idx.end(), by[q].begin(), by[q].end());
            off.push_back((int32_t)idx.size());
        }
        c.nnodes = (int32_t)nodes.size();
        c.node_ids = nodes.data();
        c.offsets = off.data();
        c.idx = idx.data();
    }
};

void matchers(const Frame& A, const Frame& B)
{
    Rng r{77};
    const orbm_frame fa = A.view(), fb = B.view();
    const int na = fa.n, nb = fb.n;
    // SearchForInitialization
    std::vector<float> prev(2 * (size_t)na);
    for (int i = 0; i < na; ++i) { prev[2 * i] = A.k[i].x; prev[2 * i + 1] = A.k[i].y; }
    std::vector<int32_t> m12(std::max(1, na));
    int rc = orbo_search_for_initialization(&fa, &fb, prev.data(), 100, 0.9f, 1, m12.data());
    if (rc < 0) fail("orbo_search_for_initialization", rc);
    // SearchByBoW(KF, F) and (KF, KF)
    FV fva(na, 40, r), fvb(nb, 40, r);
    std::vector<uint8_t> va(std::max(1, na)), vb(std::max(1, nb));
    for (auto& x : va) x = r.uni(10) != 0;
    for (auto& x : vb) x = r.uni(10) != 0;
    std::vector<int32_t> mb(std::max(1, nb));
    if ((rc = orbo_search_by_bow(&fa, &fva.c, va.data(), &fb, &fvb.c, 0.7f, 1, mb.data())) < 0)
        fail("orbo_search_by_bow", rc);
    if ((rc = orbo_search_by_bow_kf(&fa, &fva.c, va.data(), &fb, &fvb.c, vb.data(), 0.75f, 1, m12.data())) < 0)
        fail("orbo_search_by_bow_kf", rc);
    // projected points: A's keypoints with noise, descriptors with flipped bits
    const int nq = std::min(na, 800);
    std::vector<float> u(nq), v(nq), ur(nq), vc(nq), dp(nq), ang(nq);
    std::vector<int32_t> lv(nq);
    std::vector<uint8_t> iv(nq), ho(nq), qd((size_t)nq * 32);
    for (int i = 0; i < nq; ++i) {
        u[i] = A.k[i].x + (r.unif() - 0.5f) * 4;
        v[i] = A.k[i].y + (r.unif() - 0.5f) * 4;
        ur[i] = u[i] - r.unif() * 40;
        vc[i] = 0.99f + r.unif() * 0.01f;
        dp[i] = r.unif() * 100;
        ang[i] = A.k[i].angle;
        lv[i] = A.k[i].octave;
        iv[i] = r.uni(10) != 0;
        ho[i] = r.uni(3) != 0;
        for (int b = 0; b < 32; ++b) qd[(size_t)i * 32 + b] = A.d[(size_t)i * 32 + b] ^ (uint8_t)(r.uni(16) == 0);
    }
    orbm_mappoints mp{nq, u.data(), v.data(), ur.data(), lv.data(), vc.data(), dp.data(), iv.data(), ho.data(),
                      qd.data()};
    std::vector<int32_t> owner(std::max(1, nb), -1);
    const std::vector<uint8_t> blocked(std::max(1, nb), 0);
    if ((rc = orbo_search_by_projection_mps(&fb, &mp, 3.0f, 1, 50.0f, 0.8f, owner.data(), blocked.data())) < 0)
        fail("orbo_search_by_projection_mps", rc);
    std::fill(owner.begin(), owner.end(), -1);
    if ((rc = orbo_search_by_projection_last(&fb, nq, iv.data(), u.data(), v.data(), ur.data(), lv.data(), ang.data(),
                                             ho.data(), qd.data(), 7.0f, 1, 1, owner.data(), blocked.data())) < 0)
        fail("orbo_search_by_projection_last", rc);
    std::fill(owner.begin(), owner.end(), -1);
    if ((rc = orbo_search_by_projection_kf(&fb, nq, iv.data(), u.data(), v.data(), lv.data(), ang.data(), qd.data(),
                                           10.0f, 100, 1, owner.data())) < 0)
        fail("orbo_search_by_projection_kf", rc);
    std::vector<int32_t> matched(std::max(1, nb), -1);
    if ((rc = orbo_search_by_projection_sim3(&fb, nq, iv.data(), u.data(), v.data(), lv.data(), qd.data(), 10.0f,
                                             1.0f, matched.data())) < 0)
        fail("orbo_search_by_projection_sim3", rc);
    // Fuse (both forms)
    std::vector<float> inv_s2(8);
    for (int l = 0; l < 8; ++l) inv_s2[l] = 1.0f / (B.scale[l] * B.scale[l]);
    std::vector<int32_t> best(std::max(1, nq)), bdist(std::max(1, nq));
    if ((rc = orbo_fuse(&fb, inv_s2.data(), nq, iv.data(), u.data(), v.data(), ur.data(), lv.data(), qd.data(), 3.0f,
                        1, best.data(), bdist.data())) < 0)
        fail("orbo_fuse", rc);
    if ((rc = orbo_fuse_sim3(&fb, nq, iv.data(), u.data(), v.data(), lv.data(), qd.data(), 3.0f, best.data(),
                             bdist.data())) < 0)
        fail("orbo_fuse_sim3", rc);
    // SearchBySim3 with the same rows both ways
    const int n1 = std::min(na, nb);
    orbm_frame f1 = fa, f2 = fb;
    f1.n = n1; f2.n = n1;
    std::vector<uint8_t> v1(std::max(1, n1));
    std::vector<int32_t> l1(std::max(1, n1));
    std::vector<float> u1(std::max(1, n1)), w1(std::max(1, n1));
    for (int i = 0; i < n1; ++i) {
        v1[i] = r.uni(5) != 0;
        u1[i] = B.k[i].x + (r.unif() - 0.5f) * 3;
        w1[i] = B.k[i].y + (r.unif() - 0.5f) * 3;
        l1[i] = B.k[i].octave;
    }
    std::vector<int32_t> s12(std::max(1, n1), -1);
    if ((rc = orbo_search_by_sim3(&f1, &f2, v1.data(), u1.data(), w1.data(), l1.data(), A.d.data(), v1.data(),
                                  u1.data(), w1.data(), l1.data(), B.d.data(), 7.5f, s12.data())) < 0)
        fail("orbo_search_by_sim3", rc);
    // knnMatch(k = 2) and the distinctive descriptor
    std::vector<int32_t> idx(2 * (size_t)std::max(1, na)), dist(2 * (size_t)std::max(1, na));
    if ((rc = orbo_knn_match2(A.d.data(), na, B.d.data(), nb, idx.data(), dist.data())) < 0)
        fail("orbo_knn_match2", rc);
    std::vector<int32_t> off;
    for (int p = 0; p * 7 <= na; ++p) off.push_back(std::min(na, p * 7));
    if (off.back() != na) off.push_back(na);
    std::vector<int32_t> dbest(off.size());
    if ((rc = orbo_compute_distinctive_descriptors((int)off.size() - 1, off.data(), A.d.data(), dbest.data())) < 0)
        fail("orbo_compute_distinctive_descriptors", rc);
}

void vocab_files(const std::string& dir)
{
    DIR* d = opendir(dir.c_str());
    if (!d) fail("opendir", -1);
    int files = 0, loaded = 0;
    Rng r{5};
    while (dirent* e = readdir(d)) {
        const std::string name = e->d_name;
        if (name.size() < 5 || name.substr(name.size() - 4) != ".txt") continue;
        ++files;
        int32_t err = 0;
        orbv_text_vocab* tv = orbv_load_text((dir + "/" + name).c_str(), &err);
        if (!tv) continue;
        ++loaded;
        orbv_vocab view{};
        int32_t k = 0, scoring = 0, weighting = 0, nwords = 0;
        if (orbv_text_vocab_view(tv, &view, &k, &scoring, &weighting, &nwords)) fail("orbv_text_vocab_view", -1);
        // BowVector / FeatureVector assembly of random words, and the scores
        const int n = 300;
        std::vector<int32_t> wid(n), nid(n), bw(n), fvn(n), fvo(n + 1), fvi(n);
        std::vector<double> wt(n), bv(n);
        for (int i = 0; i < n; ++i) {
            wid[i] = nwords ? r.uni(nwords) : 0;
            nid[i] = r.uni(50);
            wt[i] = r.unif();
        }
        int32_t nbow = 0, nfv = 0;
        for (int sc = 0; sc < 6; ++sc) {
            if (orbv_bow_assemble(sc, weighting, n, wid.data(), wt.data(), nid.data(), bw.data(), bv.data(), &nbow,
                                  fvn.data(), fvo.data(), fvi.data(), &nfv))
                fail("orbv_bow_assemble", -1);
            (void)orbv_score(sc, bw.data(), bv.data(), nbow, bw.data(), bv.data(), nbow / 2);
        }
        orbv_free_text(tv);
    }
    closedir(d);
    std::printf("vocabulary files %d, loaded %d\n", files, loaded);
}

void gather(int nframes, int w, int h)
{
    std::vector<std::vector<uint8_t>> imgs(nframes);
    std::vector<const uint8_t*> ptrs(nframes);
    std::vector<size_t> steps(nframes);
    for (int f = 0; f < nframes; ++f) {
        steps[f] = (size_t)w + (size_t)(f % 3) * 16;
        imgs[f].assign(steps[f] * h, (uint8_t)f);
        ptrs[f] = imgs[f].data();
    }
    const size_t pitch = ((size_t)w + 63) & ~size_t(63), fbytes = pitch * h;
    std::vector<uint8_t> dst((size_t)nframes * fbytes, 0xff);
    const int th = orbmi::gather_frames(dst.data(), pitch, fbytes, ptrs.data(), steps.data(), w, h, nframes);
    for (int f = 0; f < nframes; ++f)
        for (int y = 0; y < h; y += 37)
            if (dst[f * fbytes + y * pitch + (w - 1)] != (uint8_t)f) fail("gather_frames", f);
    std::printf("gather %d frames on %d threads\n", nframes, th);
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s <all|threads> <vocab dir>\n", argv[0]);
        return 2;
    }
    const std::string mode = argv[1];
    if (mode == "all") {
        // C2 / C1 (752x480, 1000, {0,1000}), C4 (512x512, 1500, {0,511}), C3's natural order
        const orbx_params p1 = params(1000), p4 = params(1500), p3 = params(1200);
        void* e1 = orbo_create(&p1);
        void* e4 = orbo_create(&p4);
        void* e3 = orbo_create(&p3);
        if (!e1 || !e4 || !e3) fail("orbo_create", -1);
        const Frame a = extract(e1, 752, 480, 1, 0, 1000), b = extract(e1, 752, 480, 2, 0, 1000);
        const Frame c = extract(e4, 512, 512, 3, 0, 511), s = extract(e3, 752, 480, 4, 0, 0);
        std::printf("keypoints %zu %zu %zu %zu\n", a.k.size(), b.k.size(), c.k.size(), s.k.size());
        matchers(a, b);
        matchers(c, c);
        // an empty image and a flat one
        std::vector<uint8_t> flat((size_t)752 * 480, 128);
        std::vector<orb_keypoint> kp(4000);
        std::vector<uint8_t> dd((size_t)4000 * 32);
        int n = 0, mono = 0;
        if (orbo_extract(e1, flat.data(), 752, 480, 752, 0, 1000, kp.data(), dd.data(), 4000, &n, &mono) || n != 0)
            fail("flat image", n);
        orbo_destroy(e1);
        orbo_destroy(e4);
        orbo_destroy(e3);
        vocab_files(argv[2]);
        gather(64, 752, 480);
    } else if (mode == "threads") {
        // the CPU baseline's model: a pool of threads, an oracle handle each
        std::vector<std::thread> th;
        std::vector<size_t> counts(4);
        for (int t = 0; t < 4; ++t)
            th.emplace_back([t, &counts] {
                const orbx_params p = params(1000);
                void* e = orbo_create(&p);
                if (!e) fail("orbo_create", -1);
                const Frame f = extract(e, 752, 480, 10 + t, 0, 1000);
                counts[t] = f.k.size();
                orbo_destroy(e);
            });
        for (auto& x : th) x.join();
        std::printf("threads: keypoints %zu %zu %zu %zu\n", counts[0], counts[1], counts[2], counts[3]);
        gather(128, 752, 480);
    } else {
        return 2;
    }
    return 0;
}
