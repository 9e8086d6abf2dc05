// host_gather.h — the host side of orbx_extract_batch (extractor.hip): the
// frames of a batch gathered from the caller's images into one pinned buffer
// at a common pitch, the one upload's source.  Plain C++ (no HIP), so the
// sanitizer builds of tests/native (ASan/UBSan, TSan) run it without a device.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

namespace orbmi {

// Frame f's rows (row step steps[f], or w when steps is null) into
// dst + f * fbytes at row pitch `pitch`.  Batches of >= 32 frames are split
// over up to 8 threads (>= 16 frames each); a worker that cannot be started
// (std::system_error must not cross the C ABI) leaves its frames to the
// calling thread.  Returns the number of threads that ran.
inline int gather_frames(uint8_t* dst, size_t pitch, size_t fbytes, const uint8_t* const* imgs, const size_t* steps,
                         int w, int hh, int nframes) {
    auto gather = [&](int f0, int f1) {
        for (int f = f0; f < f1; ++f) {
            const size_t st = steps ? steps[f] : (size_t)w;
            for (int y = 0; y < hh; ++y) std::memcpy(dst + f * fbytes + y * pitch, imgs[f] + y * st, (size_t)w);
        }
    };
    const int nth = std::min(8, nframes / 16);
    std::vector<std::thread> th;
    int done = 0;
    if (nth > 1) {
        try {
            for (int t = 0; t < nth - 1; ++t) {
                const int a0 = (int)((long long)nframes * t / nth), a1 = (int)((long long)nframes * (t + 1) / nth);
                th.emplace_back(gather, a0, a1);
                done = a1;
            }
        } catch (...) {
        }
    }
    gather(done, nframes);
    for (auto& x : th) x.join();
    return (int)th.size() + 1;
}

}  // namespace orbmi
