// C++ host interface test (GPU): include/orb_slam3_mi355x.hpp over the C ABI.
// Extracts a raw 8UC1 image given on the command line, matches it against a
// second one, and prints counts + an FNV-1a hash of keypoints and descriptors
// for tests/test_gpu_cpp_api.py to compare with the oracle.
#include <cstdio>
#include <cstdlib>
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
    std::printf("%zu %d %016llx %016llx %zu %d %d %016llx %d %016llx\n", k[0].size(), mono[0],
                (unsigned long long)fnv(k[0].data(), k[0].size() * sizeof(orb_keypoint)),
                (unsigned long long)fnv(d[0].data.data(), d[0].data.size()), k[1].size(), mono[1], nm,
                (unsigned long long)fnv(m12.data(), m12.size() * sizeof(int)), nb,
                (unsigned long long)fnv(b12.data(), b12.size() * sizeof(int)));
    return 0;
}
