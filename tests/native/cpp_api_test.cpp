// C++ host interface test (GPU): include/orb_slam3_mi355x.hpp over the C ABI.
// Extracts a raw 8UC1 image given on the command line, matches it against a
// second one, and prints counts + an FNV-1a hash of keypoints and descriptors
// for tests/test_gpu_cpp_api.py to compare with the oracle.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/orb_slam3_mi355x.hpp"

static uint64_t fnv(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 1099511628211ull; }
    return h;
}

int main(int argc, char** argv) {
    if (argc < 5) { std::fprintf(stderr, "usage: img1.raw img2.raw cols rows\n"); return 2; }
    const int cols = std::atoi(argv[3]), rows = std::atoi(argv[4]);
    std::vector<uint8_t> im[2];
    for (int i = 0; i < 2; ++i) {
        im[i].resize((size_t)cols * rows);
        FILE* f = std::fopen(argv[1 + i], "rb");
        if (!f || std::fread(im[i].data(), 1, im[i].size(), f) != im[i].size()) return 3;
        std::fclose(f);
    }
    ORB_SLAM3_MI355X::ORBextractor ex(1000, 1.2f, 8, 20, 7);
    std::vector<ORB_SLAM3_MI355X::KeyPoint> k[2];
    ORB_SLAM3_MI355X::Descriptors d[2];
    int mono[2];
    const std::vector<int> lap = {0, 1000};
    for (int i = 0; i < 2; ++i) mono[i] = ex(im[i].data(), cols, rows, cols, nullptr, k[i], d[i], lap);
    if (ex(nullptr, 0, 0, 0, nullptr, k[0], d[0], lap) != -1) return 4;   // empty image -> -1
    for (int i = 0; i < 2; ++i) mono[i] = ex(im[i].data(), cols, rows, cols, nullptr, k[i], d[i], lap);
    orbm_frame f[2];
    for (int i = 0; i < 2; ++i)
        f[i] = orbm_frame{(int32_t)k[i].size(), k[i].data(), d[i].data.data(), 0.f, (float)cols, 0.f, (float)rows,
                          64.f / (float)cols, 48.f / (float)rows, nullptr, nullptr, 0};
    std::vector<float> prev;
    for (auto& kp : k[0]) { prev.push_back(kp.x); prev.push_back(kp.y); }
    std::vector<int> m12;
    ORB_SLAM3_MI355X::ORBmatcher matcher(0.9f, true);
    const int nm = matcher.SearchForInitialization(f[0], f[1], prev, m12, 100);
    // SearchByBoW(KF1, KF2) with FeatureVectors node(i) = i % 16 on both sides, every MapPoint valid
    std::vector<uint32_t> nodes[2], idx[2];
    std::vector<int32_t> offs[2];
    std::vector<uint8_t> valid[2];
    orbm_featvec fv[2];
    for (int i = 0; i < 2; ++i) {
        const int n = (int)k[i].size();
        for (int nd = 0; nd < 16; ++nd) {
            const int before = (int)idx[i].size();
            for (int j = nd; j < n; j += 16) idx[i].push_back((uint32_t)j);
            if ((int)idx[i].size() > before) { nodes[i].push_back(nd); offs[i].push_back(before); }
        }
        offs[i].push_back((int)idx[i].size());
        valid[i].assign(n, 1);
        fv[i] = orbm_featvec{(int32_t)nodes[i].size(), nodes[i].data(), offs[i].data(), idx[i].data()};
    }
    std::vector<int> b12;
    ORB_SLAM3_MI355X::ORBmatcher loop_matcher(0.75f, true);
    const int nb = loop_matcher.SearchByBoW(f[0], fv[0], valid[0], f[1], fv[1], valid[1], b12);
    // ExtractBatch == the single calls
    {
        std::vector<std::vector<ORB_SLAM3_MI355X::KeyPoint>> kb;
        std::vector<ORB_SLAM3_MI355X::Descriptors> db;
        const std::vector<int> mb = ex.ExtractBatch({im[0].data(), im[1].data()}, {(size_t)cols, (size_t)cols}, cols,
                                                    rows, {{0, 1000}, {0, 1000}}, kb, db);
        for (int i = 0; i < 2; ++i)
            if (mb[i] != mono[i] || kb[i].size() != k[i].size() || db[i].data != d[i].data ||
                std::memcmp(kb[i].data(), k[i].data(), k[i].size() * sizeof(orb_keypoint)) != 0)
                return 5;
    }
    // SearchByBoW over candidates == the single form
    {
        std::vector<int> single, unused;
        ORB_SLAM3_MI355X::ORBmatcher m(0.75f, true);
        const int ns = m.SearchByBoW(f[0], fv[0], valid[0], f[1], fv[1], single);
        std::vector<std::vector<int>> many;
        const std::vector<int> cnt = m.SearchByBoW({&f[0], &f[0]}, {&fv[0], &fv[0]}, {valid[0].data(), valid[0].data()},
                                                   f[1], fv[1], many);
        if (cnt.size() != 2 || cnt[0] != ns || cnt[1] != ns || many[0] != single || many[1] != single) return 6;
    }
    // SearchForTriangulation with an accept-all check == the pinhole form with bCoarse and the epipole out of reach
    {
        const std::vector<uint8_t> no_mp0(k[0].size(), 0), no_mp1(k[1].size(), 0);
        const std::vector<float> sig2(8, 1.f);
        const float F12[9] = {0, 0, 0, 0, 0, 0, 0, 0, 1};
        std::vector<float> sc(8, 1.f);
        orbm_frame g1 = f[1];
        g1.scale_factors = sc.data();
        g1.nlevels = 8;
        std::vector<std::pair<size_t, size_t>> pa, pb;
        ORB_SLAM3_MI355X::ORBmatcher m(0.6f, true);
        const int na = m.SearchForTriangulation(f[0], fv[0], no_mp0, g1, fv[1], no_mp1, F12, -1e6f, -1e6f, sig2, pa,
                                                false, true);
        const int nb2 = m.SearchForTriangulation(f[0], fv[0], no_mp0, g1, fv[1], no_mp1,
                                                 [](int, int) { return true; }, pb, false);
        if (na != nb2 || pa != pb || na <= 0) return 7;
    }
    std::printf("%zu %d %016llx %016llx %zu %d %d %016llx %d %016llx\n", k[0].size(), mono[0],
                (unsigned long long)fnv(k[0].data(), k[0].size() * sizeof(orb_keypoint)),
                (unsigned long long)fnv(d[0].data.data(), d[0].data.size()), k[1].size(), mono[1], nm,
                (unsigned long long)fnv(m12.data(), m12.size() * sizeof(int)), nb,
                (unsigned long long)fnv(b12.data(), b12.size() * sizeof(int)));
    return 0;
}
