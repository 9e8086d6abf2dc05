// Drives the drop-in extractor adapter (adapters/orbslam3/ORBextractor.cc,
// compiled against the reference's unmodified include/ORBextractor.h) the way
// Frame::ExtractORB does (src/Frame.cc:418-425): ORBextractor(nfeatures, 1.2,
// 8, 20, 7), then operator()(image, mask, keypoints, descriptors,
// vLappingArea).  Test infrastructure for tests/test_gpu_adapter.py; built by
// __graft_entry__.build() where the reference tree is present.
//
// usage: adapter_extractor <image.u8> <w> <h> <nfeatures> <lap0> <lap1> <outdir> [reps]
// writes to outdir: meta.txt ("n mono desc_rows desc_cols desc_empty
// empty_ret"), kps.bin (n x 28 B cv::KeyPoint), desc.bin (n x 32 B),
// level<i>.bin (rows cols, then the level's bytes row by row) and, with
// reps > 0, time.txt ("ms_per_call_host_pyramid ms_per_call_no_pyramid").
#include "ORBextractor.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

namespace ORB_SLAM3 {
void ORBextractorSetHostPyramid(ORBextractor* e, bool on);
}

static double time_calls(ORB_SLAM3::ORBextractor& ex, const cv::Mat& img, std::vector<int>& lap, int reps) {
    std::vector<cv::KeyPoint> k;
    cv::Mat d, mask;
    ex(img, mask, k, d, lap);   // warm (plan, graph capture)
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) ex(img, mask, k, d, lap);
    const auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::milli>(t1 - t0).count() / reps;
}

int main(int argc, char** argv) {
    if (argc < 8) {
        std::fprintf(stderr, "usage: %s image.u8 w h nfeatures lap0 lap1 outdir [reps]\n", argv[0]);
        return 2;
    }
    const int w = std::atoi(argv[2]), h = std::atoi(argv[3]), nf = std::atoi(argv[4]);
    std::vector<int> lap = {std::atoi(argv[5]), std::atoi(argv[6])};
    const std::string out = argv[7];
    const int reps = argc > 8 ? std::atoi(argv[8]) : 0;
    cv::Mat img(h, w, CV_8U);
    FILE* f = std::fopen(argv[1], "rb");
    if (!f || std::fread(img.data, 1, (size_t)w * h, f) != (size_t)w * h) return 3;
    std::fclose(f);

    ORB_SLAM3::ORBextractor ex(nf, 1.2f, 8, 20, 7);
    std::vector<cv::KeyPoint> kps;
    cv::Mat desc, mask;
    const int mono = ex(img, mask, kps, desc, lap);
    // an empty image: -1, outputs untouched (src/ORBextractor.cc:1090-1091)
    std::vector<cv::KeyPoint> k2;
    cv::Mat d2, empty;
    const int empty_ret = ex(empty, mask, k2, d2, lap);

    FILE* m = std::fopen((out + "/meta.txt").c_str(), "w");
    std::fprintf(m, "%d %d %d %d %d %d\n", (int)kps.size(), mono, desc.rows, desc.cols, desc.empty() ? 1 : 0,
                 empty_ret);
    std::fclose(m);
    FILE* fk = std::fopen((out + "/kps.bin").c_str(), "wb");
    if (!kps.empty()) std::fwrite(kps.data(), sizeof(cv::KeyPoint), kps.size(), fk);
    std::fclose(fk);
    FILE* fd = std::fopen((out + "/desc.bin").c_str(), "wb");
    for (int r = 0; r < desc.rows; ++r) std::fwrite(desc.data + (size_t)r * desc.step[0], 1, 32, fd);
    std::fclose(fd);
    for (size_t l = 0; l < ex.mvImagePyramid.size(); ++l) {
        const cv::Mat& L = ex.mvImagePyramid[l];
        FILE* fl = std::fopen((out + "/level" + std::to_string(l) + ".bin").c_str(), "wb");
        const int hdr[2] = {L.rows, L.cols};
        std::fwrite(hdr, sizeof(int), 2, fl);
        for (int r = 0; r < L.rows; ++r) std::fwrite(L.data + (size_t)r * L.step[0], 1, L.cols, fl);
        std::fclose(fl);
    }
    if (reps > 0) {
        const double with = time_calls(ex, img, lap, reps);
        ORB_SLAM3::ORBextractorSetHostPyramid(&ex, false);
        const double without = time_calls(ex, img, lap, reps);
        bool released = true;
        for (const cv::Mat& L : ex.mvImagePyramid) released = released && L.empty();
        FILE* ft = std::fopen((out + "/time.txt").c_str(), "w");
        std::fprintf(ft, "%.6f %.6f %d\n", with, without, released ? 1 : 0);
        std::fclose(ft);
    }
    return 0;
}
