// Per-call latency of the Tracking thread's matcher calls through a C ABI, as
// a C++ caller (the drop-in adapters) sees it: no Python in the timed loop.
//
//   matcher_latency <library.so> <prefix> <input dir> <reps> [opt=value,...]
//
// The optional last argument sets orb_debug_set_option values first (the
// product's A/B forms, e.g. 6=1 for zero-copy result blocks).
// <prefix> "orbm" times the MI355X library (include/orb_mi355x.h); "orbo" the
// same entry points of the CPU oracle (oracle/liborb_oracle.so, one thread:
// the reference's own per-call model) -- test infrastructure, run by
// bench.py's host_api.matchers block (the product) and its CPU-baseline leg
// (the oracle).  The searches and sizes:
//   SearchForInitialization(F1, F2, prev = F1's positions, window 100, 0.9, checkOri)
//                                             Tracking.cc:2459-2492, ORBmatcher.cc:648-763
//   SearchByProjection(F, LastFrame, th 7, motion model)   Tracking.cc:2886-2894, ORBmatcher.cc:1676-1887
//   SearchByProjection(F, local map points, th 3)          Tracking.cc:3413, ORBmatcher.cc:43-221
//   SearchByBoW(KF, F, 0.7, checkOri)                      Tracking.cc:2730, ORBmatcher.cc:223-425
// With the product (<prefix> orbm) each search is also timed in its dframe form
// (orbm_*_dframe: the frames resident in HBM -- the current frame as
// orbx_extract leaves it, the keyframe since its creation -- so a call moves
// only its per-call inputs and result), as <search>_dframe.
// Inputs are raw arrays written by bench.py (host_api_matchers) into <input
// dir>; every call starts from the same in/out arrays.  Prints one JSON line
// of per-call times (median and mean, microseconds) and writes each search's
// last outputs next to the inputs (<prefix>_<search>.bin) for the parity check.
#include "orb_mi355x.h"

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <string>
#include <vector>

namespace {

std::string g_dir;

template <class T> std::vector<T> load(const std::string& name)
{
    std::ifstream f(g_dir + "/" + name, std::ios::binary | std::ios::ate);
    if (!f) { std::fprintf(stderr, "missing %s\n", name.c_str()); std::exit(2); }
    const size_t bytes = (size_t)f.tellg();
    std::vector<T> v(bytes / sizeof(T) + (bytes % sizeof(T) ? 1 : 0));
    f.seekg(0);
    f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)bytes);
    return v;
}

template <class T> void save(const std::string& name, const T* p, size_t n)
{
    std::ofstream f(g_dir + "/" + name, std::ios::binary);
    f.write(reinterpret_cast<const char*>(p), (std::streamsize)(n * sizeof(T)));
}

std::map<std::string, double> read_meta()
{
    std::map<std::string, double> m;
    std::ifstream f(g_dir + "/meta.txt");
    std::string k;
    double v;
    while (f >> k >> v) m[k] = v;
    return m;
}

void* sym(void* lib, const std::string& prefix, const char* suffix)
{
    const std::string name = prefix + suffix;
    void* p = dlsym(lib, name.c_str());
    if (!p) { std::fprintf(stderr, "no symbol %s\n", name.c_str()); std::exit(2); }
    return p;
}

struct Stat { double median_us, mean_us; };

template <class F> Stat timed(int reps, F&& call)
{
    for (int i = 0; i < 10; ++i) call();
    std::vector<double> t(reps);
    for (int i = 0; i < reps; ++i) {
        const auto a = std::chrono::steady_clock::now();
        call();
        t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    }
    double s = 0;
    for (double x : t) s += x;
    std::sort(t.begin(), t.end());
    return Stat{t[t.size() / 2], s / reps};
}

void check(int rc, const char* what)
{
    if (rc < 0) { std::fprintf(stderr, "%s failed: %d\n", what, rc); std::exit(3); }
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc != 5 && argc != 6) {
        std::fprintf(stderr, "usage: %s <library.so> <orbm|orbo> <input dir> <reps> [opt=value,...]\n", argv[0]);
        return 2;
    }
    void* lib = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!lib) { std::fprintf(stderr, "dlopen: %s\n", dlerror()); return 2; }
    const std::string pre = argv[2];
    if (argc == 6) {
        typedef int (*SetFn)(int, int);
        SetFn set = (SetFn)dlsym(lib, "orb_debug_set_option");
        if (!set) { std::fprintf(stderr, "no orb_debug_set_option\n"); return 2; }
        for (const char* p = argv[5]; *p;) {
            int o = 0, v = 0, used = 0;
            if (std::sscanf(p, "%d=%d%n", &o, &v, &used) != 2 || set(o, v) != 0) {
                std::fprintf(stderr, "bad option list %s\n", argv[5]);
                return 2;
            }
            p += used;
            if (*p == ',') ++p;
        }
    }
    g_dir = argv[3];
    const int reps = std::max(1, std::atoi(argv[4]));
    auto meta = read_meta();
    const float W = (float)meta["W"], H = (float)meta["H"];

    const auto k1 = load<orb_keypoint>("f1_kps.bin"), k2 = load<orb_keypoint>("f2_kps.bin");
    const auto d1 = load<uint8_t>("f1_desc.bin"), d2 = load<uint8_t>("f2_desc.bin");
    const auto scale = load<float>("scale.bin");
    const int n1 = (int)meta["n1"], n2 = (int)meta["n2"];
    auto frame = [&](const std::vector<orb_keypoint>& k, const std::vector<uint8_t>& d, int n) {
        orbm_frame f{};
        f.n = n; f.kps = k.data(); f.desc = d.data();
        f.min_x = 0.f; f.max_x = W; f.min_y = 0.f; f.max_y = H;
        f.grid_inv_w = 64.0f / W; f.grid_inv_h = 48.0f / H;
        f.u_right = nullptr; f.scale_factors = scale.data(); f.nlevels = (int32_t)meta["nlevels"];
        return f;
    };
    const orbm_frame F1 = frame(k1, d1, n1), F2 = frame(k2, d2, n2);
    std::string json = "{";
    // the dframe forms (product only)
    const bool dfm = pre == "orbm";
    typedef orbm_dframe* (*DfCreate)(int);
    typedef int (*DfUpload)(orbm_dframe*, const orbm_frame*, const orbm_featvec*);
    DfCreate df_create = dfm ? (DfCreate)sym(lib, pre, "_dframe_create") : nullptr;
    DfUpload df_upload = dfm ? (DfUpload)sym(lib, pre, "_dframe_upload") : nullptr;
    orbm_dframe *D1 = nullptr, *D2 = nullptr;
    if (dfm) {
        D1 = df_create(0);
        D2 = df_create(0);
        if (!D1 || !D2) { std::fprintf(stderr, "orbm_dframe_create failed\n"); return 3; }
        check(df_upload(D1, &F1, nullptr), "orbm_dframe_upload");
        check(df_upload(D2, &F2, nullptr), "orbm_dframe_upload");
    }
    // the product's last fused projection search: rounds, rescans, phase clocks
    typedef int (*StatFn)(int32_t*);
    StatFn statfn = (StatFn)dlsym(lib, "orbm_debug_proj_stats");
    std::string extra;
    auto stats = [&](const char* name) {
        int32_t st[12];
        if (!statfn || statfn(st) != 0) return;
        char b[600];
        std::snprintf(b, sizeof b, ", \"%s_stats\": {\"rounds\": %d, \"rescans\": %d, \"phase1_clk\": %d, "
                      "\"phase2_clk\": %d, \"grid_clk\": %d, \"select_clk\": %d, \"block_10ns\": %d, "
                      "\"p2_setup_clk\": %d, \"p2_decide_clk\": %d, \"p2_rescan_clk\": %d, \"p2_rebuild_clk\": %d, "
                      "\"p2_out_clk\": %d}", name, st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7], st[8], st[9],
                      st[10], st[11]);
        extra += b;
    };
    auto put = [&](const char* name, const Stat& s) {
        char b[160];
        std::snprintf(b, sizeof b, "%s\"%s\": {\"median_us\": %.2f, \"mean_us\": %.2f}", json.size() > 1 ? ", " : "",
                      name, s.median_us, s.mean_us);
        json += b;
    };

    // SearchForInitialization (monocular initialisation, consecutive frames)
    {
        typedef int (*Fn)(const orbm_frame*, const orbm_frame*, float*, int, float, int, int32_t*);
        Fn fn = (Fn)sym(lib, pre, "_search_for_initialization");
        std::vector<float> prev0(2 * (size_t)n1), prev(2 * (size_t)n1);
        for (int i = 0; i < n1; ++i) { prev0[2 * i] = k1[i].x; prev0[2 * i + 1] = k1[i].y; }
        std::vector<int32_t> m12(std::max(1, n1));
        int nm = 0;
        const Stat s = timed(reps, [&] {
            std::memcpy(prev.data(), prev0.data(), prev0.size() * sizeof(float));
            nm = fn(&F1, &F2, prev.data(), 100, 0.9f, 1, m12.data());
            check(nm, "SearchForInitialization");
        });
        put("search_for_initialization", s);
        stats("search_for_initialization");
        m12.push_back(nm);
        save(pre + "_sfi.bin", m12.data(), m12.size());
        if (dfm) {
            typedef int (*DFn)(const orbm_dframe*, const orbm_dframe*, float*, int, float, int, int32_t*);
            DFn dfn = (DFn)sym(lib, pre, "_search_for_initialization_dframe");
            std::vector<int32_t> dm12(std::max(1, n1));
            const Stat sd = timed(reps, [&] {
                std::memcpy(prev.data(), prev0.data(), prev0.size() * sizeof(float));
                nm = dfn(D1, D2, prev.data(), 100, 0.9f, 1, dm12.data());
                check(nm, "SearchForInitialization(dframe)");
            });
            put("search_for_initialization_dframe", sd);
            stats("search_for_initialization_dframe");
            dm12.resize(n1);
            dm12.push_back(nm);
            save(pre + "_sfi_dframe.bin", dm12.data(), dm12.size());
        }
    }
    // SearchByProjection(F, LastFrame): the last frame's points projected into F2
    {
        typedef int (*Fn)(const orbm_frame*, int, const uint8_t*, const float*, const float*, const float*,
                          const int32_t*, const float*, const uint8_t*, const uint8_t*, float, int, int, int32_t*,
                          const uint8_t*);
        Fn fn = (Fn)sym(lib, pre, "_search_by_projection_last");
        const int nl = (int)meta["nlast"];
        const auto valid = load<uint8_t>("last_valid.bin"), hobs = load<uint8_t>("last_hobs.bin");
        const auto desc = load<uint8_t>("last_desc.bin");
        const auto u = load<float>("last_u.bin"), v = load<float>("last_v.bin"), ur = load<float>("last_ur.bin");
        const auto ang = load<float>("last_ang.bin");
        const auto oct = load<int32_t>("last_oct.bin");
        std::vector<int32_t> owner(std::max(1, n2));
        const std::vector<uint8_t> blocked(std::max(1, n2), 0);
        int nm = 0;
        const Stat s = timed(reps, [&] {
            std::fill(owner.begin(), owner.end(), -1);
            nm = fn(&F2, nl, valid.data(), u.data(), v.data(), ur.data(), oct.data(), ang.data(), hobs.data(),
                    desc.data(), 7.0f, 0, 1, owner.data(), blocked.data());
            check(nm, "SearchByProjection(F, LastFrame)");
        });
        put("search_by_projection_last", s);
        stats("search_by_projection_last");
        owner.resize(n2);
        owner.push_back(nm);
        save(pre + "_last.bin", owner.data(), owner.size());
        if (dfm) {
            typedef int (*DFn)(const orbm_dframe*, int, const uint8_t*, const float*, const float*, const float*,
                               const int32_t*, const float*, const uint8_t*, const uint8_t*, float, int, int,
                               int32_t*, const uint8_t*);
            DFn dfn = (DFn)sym(lib, pre, "_search_by_projection_last_dframe");
            std::vector<int32_t> down(std::max(1, n2));
            const Stat sd = timed(reps, [&] {
                std::fill(down.begin(), down.end(), -1);
                nm = dfn(D2, nl, valid.data(), u.data(), v.data(), ur.data(), oct.data(), ang.data(), hobs.data(),
                         desc.data(), 7.0f, 0, 1, down.data(), blocked.data());
                check(nm, "SearchByProjection(dframe, LastFrame)");
            });
            put("search_by_projection_last_dframe", sd);
            stats("search_by_projection_last_dframe");
            down.resize(n2);
            down.push_back(nm);
            save(pre + "_last_dframe.bin", down.data(), down.size());
        }
    }
    // SearchByProjection(F, local map points) (TrackLocalMap)
    {
        typedef int (*Fn)(const orbm_frame*, const orbm_mappoints*, float, int, float, float, int32_t*, const uint8_t*);
        Fn fn = (Fn)sym(lib, pre, "_search_by_projection_mps");
        const int nq = (int)meta["nmps"];
        const auto x = load<float>("mps_x.bin"), y = load<float>("mps_y.bin"), xr = load<float>("mps_xr.bin");
        const auto vc = load<float>("mps_vcos.bin"), dp = load<float>("mps_depth.bin");
        const auto lv = load<int32_t>("mps_lvl.bin");
        const auto iv = load<uint8_t>("mps_inview.bin"), ho = load<uint8_t>("mps_hobs.bin");
        const auto desc = load<uint8_t>("mps_desc.bin");
        orbm_mappoints mp{nq, x.data(), y.data(), xr.data(), lv.data(), vc.data(), dp.data(), iv.data(), ho.data(),
                          desc.data()};
        std::vector<int32_t> owner(std::max(1, n2));
        const std::vector<uint8_t> blocked(std::max(1, n2), 0);
        int nm = 0;
        const Stat s = timed(reps, [&] {
            std::fill(owner.begin(), owner.end(), -1);
            nm = fn(&F2, &mp, 3.0f, 0, 50.0f, 0.8f, owner.data(), blocked.data());
            check(nm, "SearchByProjection(F, MapPoints)");
        });
        put("search_by_projection_mps", s);
        stats("search_by_projection_mps");
        owner.resize(n2);
        owner.push_back(nm);
        save(pre + "_mps.bin", owner.data(), owner.size());
        if (dfm) {
            typedef int (*DFn)(const orbm_dframe*, const orbm_mappoints*, float, int, float, float, int32_t*,
                               const uint8_t*);
            DFn dfn = (DFn)sym(lib, pre, "_search_by_projection_mps_dframe");
            std::vector<int32_t> down(std::max(1, n2));
            const Stat sd = timed(reps, [&] {
                std::fill(down.begin(), down.end(), -1);
                nm = dfn(D2, &mp, 3.0f, 0, 50.0f, 0.8f, down.data(), blocked.data());
                check(nm, "SearchByProjection(dframe, MapPoints)");
            });
            put("search_by_projection_mps_dframe", sd);
            stats("search_by_projection_mps_dframe");
            down.resize(n2);
            down.push_back(nm);
            save(pre + "_mps_dframe.bin", down.data(), down.size());
        }
    }
    // SearchByBoW(KF, F): the keyframe = frame 1, the frame = frame 2
    {
        typedef int (*Fn)(const orbm_frame*, const orbm_featvec*, const uint8_t*, const orbm_frame*,
                          const orbm_featvec*, float, int, int32_t*);
        Fn fn = (Fn)sym(lib, pre, "_search_by_bow");
        const auto n1n = load<uint32_t>("fv1_nodes.bin"), n1i = load<uint32_t>("fv1_idx.bin");
        const auto n1o = load<int32_t>("fv1_off.bin");
        const auto n2n = load<uint32_t>("fv2_nodes.bin"), n2i = load<uint32_t>("fv2_idx.bin");
        const auto n2o = load<int32_t>("fv2_off.bin");
        const auto valid = load<uint8_t>("kf_valid.bin");
        const orbm_featvec fv1{(int32_t)meta["fv1_nodes"], n1n.data(), n1o.data(), n1i.data()};
        const orbm_featvec fv2{(int32_t)meta["fv2_nodes"], n2n.data(), n2o.data(), n2i.data()};
        std::vector<int32_t> match(std::max(1, n2));
        int nm = 0;
        const Stat s = timed(reps, [&] {
            nm = fn(&F1, &fv1, valid.data(), &F2, &fv2, 0.7f, 1, match.data());
            check(nm, "SearchByBoW(KF, F)");
        });
        put("search_by_bow", s);
        match.resize(n2);
        match.push_back(nm);
        save(pre + "_bow.bin", match.data(), match.size());
        if (dfm) {
            typedef int (*DFn)(const orbm_dframe*, const uint8_t*, const orbm_dframe*, float, int, int32_t*);
            DFn dfn = (DFn)sym(lib, pre, "_search_by_bow_dframe");
            check(df_upload(D1, &F1, &fv1), "orbm_dframe_upload");      // the keyframe with its FeatureVector
            check(df_upload(D2, &F2, &fv2), "orbm_dframe_upload");      // the frame after Frame::ComputeBoW
            std::vector<int32_t> dmatch(std::max(1, n2));
            const Stat sd = timed(reps, [&] {
                nm = dfn(D1, valid.data(), D2, 0.7f, 1, dmatch.data());
                check(nm, "SearchByBoW(dframe)");
            });
            put("search_by_bow_dframe", sd);
            stats("search_by_bow_dframe");      // [6] node phase, [7] final phase (10 ns ticks)
            dmatch.resize(n2);
            dmatch.push_back(nm);
            save(pre + "_bow_dframe.bin", dmatch.data(), dmatch.size());
        }
    }
    json += extra + "}";
    std::printf("%s\n", json.c_str());
    return 0;
}
