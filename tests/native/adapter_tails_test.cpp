// The drop-in ORBmatcher mapping bodies' host tails (adapters/orbslam3/
// ORBmatcher_tails.h, the code ORBmatcher_mapping.cc instantiates with the
// reference's KeyFrame / MapPoint) executed with functional mock map types:
// the device searches through the product's C ABI, the tails on the mocks,
// against the reference's own serial loops restated over the same mocks with
// the CPU oracle's per-point searches (tests/test_gpu_adapter_tails.py).
//
//   adapter_tails_test <product.so> <oracle.so> <trials> [prefix of the first library, default orbm]
//
// Per trial a fresh randomised map (a keyframe of ~1000 oracle-extracted
// keypoints, slots partly occupied, some occupants bad; candidate points with
// duplicates, points already in the keyframe, bad and null points, points
// whose geometry rejects them) is built twice from one seed; one copy goes
// through the adapter path, the other through the serial loop, and every
// observable is compared: keyframe slots, every point's bad flag, replacement,
// observations and descriptor / level, and the returned counts.  Bodies:
//   Fuse(pKF, vpMapPoints, th, bRight)   ORBmatcher.cc:1148-1331 (left and right slots)
//   Fuse(pKF, Scw, vpPoints, th, vpReplacePoint)              :1340-1455
//   SearchByProjection(KF, Sim3, ...) both forms              :427-646
//   SearchByProjection(F, KF, sAlreadyFound, th, ORBdist)     :1889-2010
//   SearchByBoW(KF, KF)                                       :765-905
//   SearchBySim3                                              :1457-1674
//   SearchForTriangulation (pinhole)                          :907-1146
//   DescriptorDistance                                        :2058-2074
// Prints one JSON line; exit 0 iff every comparison holds.
#include "orb_mi355x.h"
#include "../../adapters/orbslam3/ORBmatcher_tails.h"

#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

namespace {

// ---------------------------------------------------------------- the C ABI
struct Api {
    int (*fuse)(const orbm_frame*, const float*, int, const uint8_t*, const float*, const float*, const float*,
                const int32_t*, const uint8_t*, float, int, int32_t*, int32_t*);
    int (*fuse_sim3)(const orbm_frame*, int, const uint8_t*, const float*, const float*, const int32_t*,
                     const uint8_t*, float, int32_t*, int32_t*);
    int (*proj_sim3)(const orbm_frame*, int, const uint8_t*, const float*, const float*, const int32_t*,
                     const uint8_t*, float, float, int32_t*);
    int (*proj_kf)(const orbm_frame*, int, const uint8_t*, const float*, const float*, const int32_t*, const float*,
                   const uint8_t*, float, int, int, int32_t*);
    int (*bow_kf)(const orbm_frame*, const orbm_featvec*, const uint8_t*, const orbm_frame*, const orbm_featvec*,
                  const uint8_t*, float, int, int32_t*);
    int (*sim3)(const orbm_frame*, const orbm_frame*, const uint8_t*, const float*, const float*, const int32_t*,
                const uint8_t*, const uint8_t*, const float*, const float*, const int32_t*, const uint8_t*, float,
                int32_t*);
    int (*tri)(const orbm_frame*, const orbm_featvec*, const uint8_t*, const orbm_frame*, const orbm_featvec*,
               const uint8_t*, const float*, float, float, const float*, int, int, int, int, int32_t*);
    int (*dist)(const uint8_t*, const uint8_t*);
};

void* need(void* lib, const std::string& name)
{
    void* p = dlsym(lib, name.c_str());
    if (!p) { std::fprintf(stderr, "no symbol %s\n", name.c_str()); std::exit(2); }
    return p;
}

Api load(const char* path, const std::string& pre)
{
    void* L = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!L) { std::fprintf(stderr, "dlopen %s: %s\n", path, dlerror()); std::exit(2); }
    Api a;
    a.fuse = (decltype(a.fuse))need(L, pre + "_fuse");
    a.fuse_sim3 = (decltype(a.fuse_sim3))need(L, pre + "_fuse_sim3");
    a.proj_sim3 = (decltype(a.proj_sim3))need(L, pre + "_search_by_projection_sim3");
    a.proj_kf = (decltype(a.proj_kf))need(L, pre + "_search_by_projection_kf");
    a.bow_kf = (decltype(a.bow_kf))need(L, pre + "_search_by_bow_kf");
    a.sim3 = (decltype(a.sim3))need(L, pre + "_search_by_sim3");
    a.tri = (decltype(a.tri))need(L, pre + "_search_for_triangulation");
    a.dist = (decltype(a.dist))need(L, pre + "_descriptor_distance");
    return a;
}

Api g_dev, g_ora;
int g_fail = 0;
std::string g_log;

void expect(bool ok, const char* what, int trial)
{
    if (ok) return;
    ++g_fail;
    if (g_log.size() < 2000) g_log += std::string(what) + " (trial " + std::to_string(trial) + "); ";
}

void check_rc(int rc, const char* what)
{
    if (rc < 0) { std::fprintf(stderr, "%s returned %d\n", what, rc); std::exit(3); }
}

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
    bool p(float q) { return unif() < q; }
};

// ---------------------------------------------------------------- the mocks
struct MockKF;
// MapPoint (MapPoint.h): observations, bad flag, replacement, descriptor; the
// geometry a Fuse row reads (projection, level) kept as fields, recomputed by
// Replace the way ComputeDistinctiveDescriptors / UpdateNormalAndDepth change
// the survivor (a deterministic function of its new observations).
struct MockMP {
    int id = 0;
    bool bad = false, geom_ok = true;
    MockMP* replaced = nullptr;
    std::map<MockKF*, int> obs;
    uint8_t desc[32] = {};
    float u = 0.f, v = 0.f, ur = -1.f;
    int level = 0;
    bool isBad() const { return bad; }
    int Observations() const { return (int)obs.size(); }
    bool IsInKeyFrame(MockKF* k) const { return obs.count(k) != 0; }
    std::tuple<int, int> GetIndexInKeyFrame(MockKF* k) const
    {
        const auto it = obs.find(k);
        return it == obs.end() ? std::make_tuple(-1, -1) : std::make_tuple(it->second, -1);
    }
    void AddObservation(MockKF* k, int idx)
    {
        if (!obs.count(k)) obs[k] = idx;      // MapPoint::AddObservation keeps an existing entry
    }
    void Replace(MockMP* p);                  // MapPoint::Replace (MapPoint.cc)
};

struct MockKF {
    int id = 0;
    std::vector<MockMP*> slots;
    MockMP* GetMapPoint(size_t i) const { return slots[i]; }
    void AddMapPoint(MockMP* p, size_t i) { slots[i] = p; }
};

void MockMP::Replace(MockMP* p)
{
    if (p->id == id) return;
    const std::map<MockKF*, int> o = obs;
    obs.clear();
    bad = true;
    replaced = p;
    for (const auto& kv : o) {
        if (!p->IsInKeyFrame(kv.first)) {
            kv.first->slots[kv.second] = p;          // ReplaceMapPointMatch
            p->AddObservation(kv.first, kv.second);
        } else {
            kv.first->slots[kv.second] = nullptr;    // EraseMapPointMatch
        }
    }
    // ComputeDistinctiveDescriptors / UpdateNormalAndDepth of the survivor
    const int n = p->Observations();
    for (int b = 0; b < 32; ++b) p->desc[b] ^= (uint8_t)((n * 37 + b) & (n % 3 ? 0x11 : 0x0));
    p->level = (p->level + (n % 2)) % 8;
}

// ---------------------------------------------------------------- the frames
struct Frame {
    std::vector<orb_keypoint> k;
    std::vector<uint8_t> d;
    std::vector<float> scale, sigma2, inv_sigma2, ur;
    orbm_frame view() const
    {
        orbm_frame f{};
        f.n = (int32_t)k.size();
        f.kps = k.data();
        f.desc = d.data();
        f.min_x = 0.f; f.max_x = 752.f; f.min_y = 0.f; f.max_y = 480.f;
        f.grid_inv_w = 64.0f / 752.f;
        f.grid_inv_h = 48.0f / 480.f;
        f.u_right = ur.empty() ? nullptr : ur.data();
        f.scale_factors = scale.data();
        f.nlevels = (int32_t)scale.size();
        return f;
    }
};

// keypoints on a jittered lattice with random octaves / angles, descriptors random
Frame make_frame(uint64_t seed, int n)
{
    Rng r{seed};
    Frame f;
    for (int l = 0; l < 8; ++l) {
        const float s = l ? f.scale.back() * 1.2f : 1.0f;
        f.scale.push_back(s);
        f.sigma2.push_back(s * s);
        f.inv_sigma2.push_back(1.0f / (s * s));
    }
    for (int i = 0; i < n; ++i) {
        orb_keypoint kp{};
        kp.x = 20.f + r.unif() * 712.f;
        kp.y = 20.f + r.unif() * 440.f;
        kp.octave = r.uni(4);
        kp.size = 31.f * f.scale[kp.octave];
        kp.angle = r.unif() * 360.f;
        kp.response = (float)r.uni(60);
        kp.class_id = -1;
        f.k.push_back(kp);
        for (int b = 0; b < 32; ++b) f.d.push_back((uint8_t)r.uni(256));
        f.ur.push_back(r.p(0.3f) ? kp.x - r.unif() * 40.f : -1.f);
    }
    return f;
}

// ---------------------------------------------------------------- a world
// One keyframe (slots [0, nl) on the left frame, [nl, nl + nr) on the right
// frame), other keyframes the points are observed in, and the candidate list.
struct World {
    std::vector<std::unique_ptr<MockMP>> mps;
    std::vector<std::unique_ptr<MockKF>> kfs;
    MockKF* kf = nullptr;
    std::vector<MockMP*> cand;
    MockMP* add(int id)
    {
        mps.emplace_back(new MockMP());
        mps.back()->id = id;
        return mps.back().get();
    }
};

// near keypoint j of `f`: a projection with noise and the descriptor with a few bits flipped
void near_kp(MockMP* p, const Frame& f, int j, Rng& r)
{
    p->u = f.k[j].x + (r.unif() - 0.5f) * 3.f;
    p->v = f.k[j].y + (r.unif() - 0.5f) * 3.f;
    p->ur = r.p(0.5f) ? p->u - (f.k[j].x - (f.ur[j] >= 0 ? f.ur[j] : f.k[j].x - 10.f)) : -1.f;
    p->level = f.k[j].octave;
    for (int b = 0; b < 32; ++b) p->desc[b] = f.d[(size_t)j * 32 + b] ^ (uint8_t)(r.p(0.06f) ? 1 << r.uni(8) : 0);
}

std::unique_ptr<World> make_world(uint64_t seed, const Frame& L, const Frame& R)
{
    Rng r{seed};
    std::unique_ptr<World> w(new World());
    const int nl = (int)L.k.size(), nr = (int)R.k.size();
    for (int i = 0; i < 6; ++i) {
        w->kfs.emplace_back(new MockKF());
        w->kfs.back()->id = i;
        w->kfs.back()->slots.assign(nl + nr, nullptr);
    }
    w->kf = w->kfs[0].get();
    int id = 1;
    // occupants of the keyframe's slots: observed there and in 0-3 other keyframes
    for (int s = 0; s < nl + nr; ++s) {
        if (!r.p(0.3f)) continue;
        MockMP* p = w->add(id++);
        const Frame& f = s < nl ? L : R;
        near_kp(p, f, s < nl ? s : s - nl, r);
        p->obs[w->kf] = s;
        w->kf->slots[s] = p;
        for (int k = 1 + r.uni(4); k < 5; k += 1 + r.uni(3)) {
            const int os = r.uni(nl + nr);
            if (!w->kfs[k]->slots[os]) { w->kfs[k]->slots[os] = p; p->obs[w->kfs[k].get()] = os; }
        }
        if (r.p(0.08f)) p->bad = true;
    }
    // candidates
    for (int i = 0; i < 700; ++i) {
        const float q = r.unif();
        if (q < 0.05f) { w->cand.push_back(nullptr); continue; }
        if (q < 0.17f && !w->cand.empty()) {                 // a duplicate of an earlier candidate
            w->cand.push_back(w->cand[r.uni((int)w->cand.size())]);
            continue;
        }
        if (q < 0.27f) {                                      // a point already in the keyframe
            MockMP* o = w->kf->slots[r.uni(nl + nr)];
            if (o) { w->cand.push_back(o); continue; }
        }
        MockMP* p = w->add(id++);
        const bool right = r.p(0.35f);
        const Frame& f = right ? R : L;
        near_kp(p, f, r.uni(right ? nr : nl), r);
        for (int k = 1 + r.uni(5); k < 6; k += 1 + r.uni(4)) {
            const int os = r.uni(nl + nr);
            if (!w->kfs[k]->slots[os]) { w->kfs[k]->slots[os] = p; p->obs[w->kfs[k].get()] = os; }
        }
        if (r.p(0.04f)) p->bad = true;
        if (r.p(0.04f)) p->geom_ok = false;
        w->cand.push_back(p);
    }
    return w;
}

// every observable of a world: slots, points' flags, replacements,
// observations, descriptors and levels, as ids
std::string state(const World& w)
{
    std::string s;
    for (const auto& k : w.kfs)
        for (MockMP* p : k->slots) s += std::to_string(p ? p->id : 0) + ",";
    for (const auto& p : w.mps) {
        s += "|" + std::to_string(p->id) + (p->bad ? "b" : "g") + std::to_string(p->replaced ? p->replaced->id : 0) +
             ":" + std::to_string(p->level) + ":";
        std::map<int, int> by_id;                    // (the obs map is keyed by address: compare by keyframe id)
        for (const auto& kv : p->obs) by_id[kv.first->id] = kv.second;
        for (const auto& kv : by_id) s += std::to_string(kv.first) + "@" + std::to_string(kv.second) + ";";
        for (int b = 0; b < 32; ++b) s += std::to_string(p->desc[b]) + ".";
    }
    return s;
}

// the geometry of a Fuse row (fuse_point): rejects null, bad, in-keyframe
// points and those the projection / distance / angle gates would drop
bool fuse_row(MockKF* kf, MockMP* p, float& u, float& v, float& ur, int& level, uint8_t* d)
{
    if (!p || p->isBad() || p->IsInKeyFrame(kf) || !p->geom_ok) return false;
    u = p->u; v = p->v; ur = p->ur; level = p->level;
    std::memcpy(d, p->desc, 32);
    return true;
}

// ------------------------------------------------ Fuse(pKF, vpMapPoints, th, bRight)
// the adapter: the batched device search on the snapshot, then fuse_decisions
int fuse_adapter(World& w, const Frame& cam, int slot0, float th)
{
    const size_t n = w.cand.size();
    mi355x_tails::PointRows pr(n);
    for (size_t i = 0; i < n; ++i) {
        int level = 0;
        if (!fuse_row(w.kf, w.cand[i], pr.u[i], pr.v[i], pr.ur[i], level, &pr.desc[i * 32])) continue;
        pr.valid[i] = 1;
        pr.level[i] = level;
    }
    const orbm_frame f = cam.view();
    std::vector<int32_t> best(n, -1), bd(n, 0);
    check_rc(g_dev.fuse(&f, cam.inv_sigma2.data(), (int)n, pr.valid.data(), pr.u.data(), pr.v.data(), pr.ur.data(),
                        pr.level.data(), pr.desc.data(), th, 1, best.data(), bd.data()),
             "orbm_fuse");
    auto row = [&](MockMP* p, float& u, float& v, float& ur, int& level, uint8_t* d) {
        return fuse_row(w.kf, p, u, v, ur, level, d);
    };
    auto search1 = [&](float u, float v, float ur, int level, const uint8_t* d) {
        const uint8_t one = 1;
        int32_t b = -1, x = 0;
        check_rc(g_dev.fuse(&f, cam.inv_sigma2.data(), 1, &one, &u, &v, &ur, &level, d, th, 1, &b, &x), "orbm_fuse");
        return (int)b;
    };
    return mi355x_tails::fuse_decisions(w.kf, w.cand, slot0, pr, best, row, search1);
}

// the reference's serial loop (ORBmatcher.cc:1160-1331): each point's row and
// window search at its own turn (the oracle's search of one row), then the
// replace / add decision
int fuse_serial(World& w, const Frame& cam, int slot0, float th)
{
    const orbm_frame f = cam.view();
    int nFused = 0;
    for (MockMP* pMP : w.cand) {
        float u, v, ur;
        int level;
        uint8_t d[32];
        if (!fuse_row(w.kf, pMP, u, v, ur, level, d)) continue;
        const uint8_t one = 1;
        int32_t bestIdx = -1, x = 0;
        check_rc(g_ora.fuse(&f, cam.inv_sigma2.data(), 1, &one, &u, &v, &ur, &level, d, th, 1, &bestIdx, &x),
                 "orbo_fuse");
        if (bestIdx < 0) continue;
        bestIdx += slot0;
        MockMP* pMPinKF = w.kf->GetMapPoint(bestIdx);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) {
                if (pMPinKF->Observations() > pMP->Observations())
                    pMP->Replace(pMPinKF);
                else
                    pMPinKF->Replace(pMP);
            }
        } else {
            pMP->AddObservation(w.kf, bestIdx);
            w.kf->AddMapPoint(pMP, bestIdx);
        }
        nFused++;
    }
    return nFused;
}

// ------------------------------------------------ Fuse(pKF, Scw, vpPoints, th, vpReplacePoint)
int fuse_sim3_run(World& w, const Frame& cam, const Api& api, bool serial, std::vector<MockMP*>& rep)
{
    const size_t n = w.cand.size();
    // the already-found set is fixed for the call (:1352)
    std::vector<uint8_t> valid(n, 0), desc(n * 32, 0);
    std::vector<float> u(n, 0.f), v(n, 0.f);
    std::vector<int32_t> level(n, 0);
    for (size_t i = 0; i < n; ++i) {
        MockMP* p = w.cand[i];
        float ur;
        int lv = 0;
        if (!fuse_row(w.kf, p, u[i], v[i], ur, lv, &desc[i * 32])) continue;
        valid[i] = 1;
        level[i] = lv;
    }
    const orbm_frame f = cam.view();
    std::vector<int32_t> best(n, -1), bd(n, 0);
    rep.assign(n, nullptr);
    if (!serial) {
        check_rc(api.fuse_sim3(&f, (int)n, valid.data(), u.data(), v.data(), level.data(), desc.data(), 4.0f,
                               best.data(), bd.data()),
                 "fuse_sim3");
        return mi355x_tails::fuse_sim3_decisions(w.kf, w.cand, best, rep);
    }
    int nFused = 0;                               // :1372-1449, one row at its turn
    for (size_t i = 0; i < n; ++i) {
        if (!valid[i]) continue;
        const uint8_t one = 1;
        int32_t bestIdx = -1, x = 0;
        check_rc(api.fuse_sim3(&f, 1, &one, &u[i], &v[i], &level[i], &desc[i * 32], 4.0f, &bestIdx, &x), "fuse_sim3");
        if (bestIdx < 0) continue;
        MockMP* pMP = w.cand[i];
        MockMP* pMPinKF = w.kf->GetMapPoint(bestIdx);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) rep[i] = pMPinKF;
        } else {
            pMP->AddObservation(w.kf, bestIdx);
            w.kf->AddMapPoint(pMP, bestIdx);
        }
        nFused++;
    }
    return nFused;
}

// ------------------------------------------------ the index-map bodies
struct Rows {
    std::vector<uint8_t> valid, desc;
    std::vector<float> u, v;
    std::vector<int32_t> level;
    std::vector<float> angle;
};
Rows rows_of(const std::vector<MockMP*>& pts, Rng& r)
{
    Rows q;
    const size_t n = pts.size();
    q.valid.assign(n, 0); q.desc.assign(n * 32, 0); q.u.assign(n, 0.f); q.v.assign(n, 0.f); q.level.assign(n, 0);
    q.angle.assign(n, 0.f);
    for (size_t i = 0; i < n; ++i) {
        MockMP* p = pts[i];
        q.angle[i] = r.unif() * 360.f;
        if (!p || p->isBad() || !p->geom_ok) continue;
        q.valid[i] = 1;
        q.u[i] = p->u; q.v[i] = p->v; q.level[i] = p->level;
        std::memcpy(&q.desc[i * 32], p->desc, 32);
    }
    return q;
}

std::string ids(const std::vector<MockMP*>& v)
{
    std::string s;
    for (MockMP* p : v) s += std::to_string(p ? p->id : 0) + ",";
    return s;
}

void index_bodies(World& w, const Frame& L, const Frame& R, int trial, Rng& r)
{
    const orbm_frame fl = L.view(), fr = R.view();
    const int nl = fl.n;
    // SearchByProjection(KF, Sim3) both forms: vpMatched partly occupied
    {
        std::vector<MockMP*> pts(w.cand.begin(), w.cand.end());
        const Rows q = rows_of(pts, r);
        std::vector<MockKF*> ptsKF(pts.size());
        for (size_t i = 0; i < pts.size(); ++i) ptsKF[i] = w.kfs[1 + r.uni(5)].get();
        std::vector<MockMP*> m0(nl, nullptr);
        for (int s = 0; s < nl; ++s)
            if (r.p(0.1f)) m0[s] = w.kf->slots[s] ? w.kf->slots[s] : w.mps[r.uni((int)w.mps.size())].get();
        std::vector<MockKF*> k0(nl, nullptr);
        std::string out[2];
        for (int side = 0; side < 2; ++side) {
            const Api& api = side ? g_ora : g_dev;
            std::vector<MockMP*> vpMatched = m0;
            std::vector<MockKF*> vpMatchedKF = k0;
            std::vector<int32_t> matched = mi355x_tails::slot_states(vpMatched);
            check_rc(api.proj_sim3(&fl, (int)pts.size(), q.valid.data(), q.u.data(), q.v.data(), q.level.data(),
                                   q.desc.data(), 10.0f, 1.0f, matched.data()),
                     "search_by_projection_sim3");
            mi355x_tails::slot_writeback(matched, pts, &ptsKF, vpMatched, &vpMatchedKF);
            out[side] = ids(vpMatched);
            for (MockKF* k : vpMatchedKF) out[side] += std::to_string(k ? k->id : -1) + ",";
        }
        expect(out[0] == out[1], "SearchByProjection(KF, Sim3)", trial);
    }
    // SearchByProjection(F, KF): the frame's slots partly occupied
    {
        std::vector<MockMP*> pts(w.kf->slots.begin(), w.kf->slots.begin() + nl);   // the keyframe's points
        const Rows q = rows_of(pts, r);
        std::vector<MockMP*> f0(R.k.size(), nullptr);
        for (size_t s = 0; s < f0.size(); ++s)
            if (r.p(0.1f)) f0[s] = w.mps[r.uni((int)w.mps.size())].get();
        std::string out[2];
        int nm[2];
        for (int side = 0; side < 2; ++side) {
            const Api& api = side ? g_ora : g_dev;
            std::vector<MockMP*> slots = f0;
            std::vector<int32_t> owner = mi355x_tails::slot_states(slots);
            nm[side] = api.proj_kf(&fr, (int)pts.size(), q.valid.data(), q.u.data(), q.v.data(), q.level.data(),
                                   q.angle.data(), q.desc.data(), 10.0f, 100, 1, owner.data());
            check_rc(nm[side], "search_by_projection_kf");
            mi355x_tails::slot_writeback<MockMP, MockKF*>(owner, pts, nullptr, slots, nullptr);
            out[side] = ids(slots);
        }
        expect(out[0] == out[1] && nm[0] == nm[1], "SearchByProjection(F, KF)", trial);
    }
    // SearchByBoW(KF, KF): masks from the points (null / bad / past mvKeysUn)
    {
        std::vector<MockMP*> mp1(w.kf->slots.begin(), w.kf->slots.begin() + nl);
        std::vector<MockMP*> mp2(w.kfs[1]->slots.begin(), w.kfs[1]->slots.begin() + (int)R.k.size());
        const std::vector<uint8_t> v1 = mi355x_tails::bow_kf_mask(mp1, mp1.size());
        const std::vector<uint8_t> v2 = mi355x_tails::bow_kf_mask(mp2, mp2.size() - 40);   // a two-camera keyframe
        std::vector<uint32_t> nodes1, idx1, nodes2, idx2;
        std::vector<int32_t> off1{0}, off2{0};
        for (int q = 0; q < 40; ++q) {
            nodes1.push_back(q); nodes2.push_back(q);
            for (int i = q; i < nl; i += 40) idx1.push_back(i);
            for (int i = q; i < (int)R.k.size(); i += 40) idx2.push_back(i);
            off1.push_back((int32_t)idx1.size());
            off2.push_back((int32_t)idx2.size());
        }
        const orbm_featvec fv1{40, nodes1.data(), off1.data(), idx1.data()}, fv2{40, nodes2.data(), off2.data(),
                                                                                  idx2.data()};
        // keyframe 2's descriptors: keyframe 1's of the same index, bits flipped, so matches exist
        Frame K2 = R;
        for (size_t i = 0; i < K2.k.size() && i < (size_t)nl; ++i)
            for (int b = 0; b < 32; ++b) K2.d[i * 32 + b] = L.d[i * 32 + b] ^ (uint8_t)(r.p(0.05f) ? 4 : 0);
        const orbm_frame fk2 = K2.view();
        std::string out[2];
        for (int side = 0; side < 2; ++side) {
            const Api& api = side ? g_ora : g_dev;
            std::vector<int32_t> m12(nl, -1);
            check_rc(api.bow_kf(&fl, &fv1, v1.data(), &fk2, &fv2, v2.data(), 0.75f, 1, m12.data()), "bow_kf");
            std::vector<MockMP*> vpMatches12(nl, nullptr);
            mi355x_tails::matches_writeback(m12, mp2, vpMatches12);
            out[side] = ids(vpMatches12);
        }
        expect(out[0] == out[1], "SearchByBoW(KF, KF)", trial);
        // SearchForTriangulation on the same pair (has-MapPoint masks, pairs)
        std::vector<uint8_t> h1(nl), h2(K2.k.size());
        for (int i = 0; i < nl; ++i) h1[i] = w.kf->GetMapPoint(i) != nullptr;
        for (size_t i = 0; i < h2.size(); ++i) h2[i] = w.kfs[1]->GetMapPoint(i) != nullptr;
        const float F[9] = {0.f, 0.f, 0.f, 0.f, 0.f, -1.f, 0.f, 1.f, 0.f};    // horizontal epipolar lines
        std::vector<std::pair<size_t, size_t> > pairs[2];
        for (int side = 0; side < 2; ++side) {
            const Api& api = side ? g_ora : g_dev;
            std::vector<int32_t> m12(nl, -1);
            check_rc(api.tri(&fl, &fv1, h1.data(), &fk2, &fv2, h2.data(), F, 1.0e6f, 1.0e6f, K2.sigma2.data(), 0, 0,
                             1, 1, m12.data()),
                     "search_for_triangulation");
            mi355x_tails::triangulation_pairs(m12, pairs[side]);
        }
        expect(pairs[0] == pairs[1], "SearchForTriangulation", trial);
    }
    // SearchBySim3: vpMatches12 partly set, the already-matched flags through GetIndexInKeyFrame
    {
        MockKF* k2 = w.kfs[1].get();
        const int N1 = nl, N2 = (int)R.k.size();
        std::vector<MockMP*> mp1(w.kf->slots.begin(), w.kf->slots.begin() + N1);
        std::vector<MockMP*> mp2(k2->slots.begin(), k2->slots.begin() + N2);
        std::vector<MockMP*> m0(N1, nullptr);
        for (int i = 0; i < N1; ++i)
            if (r.p(0.05f)) m0[i] = mp2[r.uni(N2)];
        std::vector<bool> am1, am2;
        mi355x_tails::sim3_already_matched(m0, k2, N2, am1, am2);
        Rows q1 = rows_of(mp1, r), q2 = rows_of(mp2, r);
        for (int i = 0; i < N1; ++i) if (am1[i]) q1.valid[i] = 0;
        for (int i = 0; i < N2; ++i) if (am2[i]) q2.valid[i] = 0;
        std::string out[2];
        for (int side = 0; side < 2; ++side) {
            const Api& api = side ? g_ora : g_dev;
            std::vector<int32_t> m12(N1, -1);
            check_rc(api.sim3(&fl, &fr, q1.valid.data(), q1.u.data(), q1.v.data(), q1.level.data(), q1.desc.data(),
                              q2.valid.data(), q2.u.data(), q2.v.data(), q2.level.data(), q2.desc.data(), 7.5f,
                              m12.data()),
                     "search_by_sim3");
            std::vector<MockMP*> vpMatches12 = m0;
            mi355x_tails::matches_writeback(m12, mp2, vpMatches12);
            out[side] = ids(vpMatches12);
        }
        expect(out[0] == out[1], "SearchBySim3", trial);
    }
    // DescriptorDistance
    for (int i = 0; i < 64 && i < nl; ++i)
        expect(g_dev.dist(&L.d[i * 32], &R.d[i * 32]) == g_ora.dist(&L.d[i * 32], &R.d[i * 32]), "DescriptorDistance",
               trial);
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc != 4 && argc != 5) {
        std::fprintf(stderr, "usage: %s <product.so> <oracle.so> <trials> [prefix]\n", argv[0]);
        return 2;
    }
    // (prefix orbo: the oracle on both sides, a CPU check of the harness itself)
    g_dev = load(argv[1], argc == 5 ? argv[4] : "orbm");
    g_ora = load(argv[2], "orbo");
    const int trials = std::max(1, std::atoi(argv[3]));
    int fused = 0, replaced = 0, rescans = 0, fused_sim3 = 0;
    for (int t = 0; t < trials; ++t) {
        const Frame L = make_frame(1000 + t, 900 + 13 * t), R = make_frame(5000 + t, 700 + 7 * t);
        // Fuse on the left camera (slot0 0) and on the right one (slot0 = NLeft)
        for (int right = 0; right < 2; ++right) {
            std::unique_ptr<World> a = make_world(77 + 31 * t, L, R), b = make_world(77 + 31 * t, L, R);
            const Frame& cam = right ? R : L;
            const int slot0 = right ? (int)L.k.size() : 0;
            const float th = right ? 3.0f : 5.0f;
            const int na = fuse_adapter(*a, cam, slot0, th), nb = fuse_serial(*b, cam, slot0, th);
            expect(na == nb, right ? "Fuse(bRight) count" : "Fuse count", t);
            expect(state(*a) == state(*b), right ? "Fuse(bRight) map state" : "Fuse map state", t);
            fused += na;
            for (const auto& p : a->mps) replaced += p->replaced != nullptr;
            // how often a touched point came back (the re-snapshot path)
            std::map<MockMP*, int> seen;
            for (MockMP* p : a->cand) rescans += p && seen[p]++ > 0;
        }
        // Fuse(Sim3): device + tail vs the serial loop on the oracle
        {
            std::unique_ptr<World> a = make_world(91 + 17 * t, L, R), b = make_world(91 + 17 * t, L, R);
            std::vector<MockMP*> ra, rb;
            const int na = fuse_sim3_run(*a, L, g_dev, false, ra), nb = fuse_sim3_run(*b, L, g_ora, true, rb);
            std::string sa, sb;
            for (MockMP* p : ra) sa += std::to_string(p ? p->id : 0) + ",";
            for (MockMP* p : rb) sb += std::to_string(p ? p->id : 0) + ",";
            expect(na == nb && sa == sb && state(*a) == state(*b), "Fuse(Sim3)", t);
            fused_sim3 += na;
        }
        {
            std::unique_ptr<World> w = make_world(123 + t, L, R);
            Rng r{999 + (uint64_t)t};
            index_bodies(*w, L, R, t, r);
        }
    }
    std::printf("{\"trials\": %d, \"failures\": %d, \"fused\": %d, \"replaced\": %d, \"repeated_candidates\": %d, "
                "\"fused_sim3\": %d, \"log\": \"%s\"}\n",
                trials, g_fail, fused, replaced, rescans, fused_sim3, g_log.c_str());
    return g_fail ? 1 : 0;
}
