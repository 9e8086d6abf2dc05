// kfdb.hip — KeyFrameDatabase::DetectRelocalizationCandidates
// (reference src/KeyFrameDatabase.cc:733-845) over a device-resident snapshot
// of the keyframe database.
//
// One query = three small copies in (query, mRelocScore snapshot), five
// launches, one compact record list out:
//   k_kfdb_count   one workgroup per query word: walks that word's inverted
//                  list, counts the shared words of every keyframe, keeps its
//                  first encounter (query-word rank, list position) -- the
//                  order in which the reference appends keyframes to
//                  lKFsSharingWords -- and the maximum count;
//   k_kfdb_select  keyframes above (int)(0.8f * max) compacted into records;
//   k_kfdb_score   one thread per record: the L1Scoring::score merge (double,
//                  common words in order, the query in LDS) -> mRelocScore;
//   k_kfdb_neigh   each record's GetBestCovisibilityKeyFrames(10) with their
//                  mRelocScore after scoring (the stale value for neighbours
//                  that share words without being scored, as the reference
//                  reads it) and whether they share a word.
// The host sorts the records into the reference's list order and runs the
// ordered accumulation and the 0.75 * best filter with its set (:792-842).
#include "../../include/orb_mi355x.h"
#include "common.h"

#include <algorithm>
#include <cstring>
#include <vector>

// One keyframe that shares enough words with the query, with everything the
// host's ordered covisibility pass needs (KeyFrameDatabase.cc:792-819).
struct Rec {
    unsigned long long first;    // (query-word rank << 32) | position in that word's list
    int32_t kf;
    float score;
    int32_t nb_kf[10];           // GetBestCovisibilityKeyFrames(10), -1 padded
    float nb_score[10];          // their mRelocScore after this query's scoring
    int32_t nb_shares;           // bit j: neighbour j shares a word with the query
    int32_t pad;
};

struct orbk_db {
    int device = 0;
    int nkf = 0, nwords = 0;
    int32_t *bow_off = nullptr, *bow_words = nullptr, *inv_off = nullptr, *inv_kf = nullptr;
    double* bow_vals = nullptr;
    std::vector<int32_t> kf_map;
    int32_t *cov_off_d = nullptr, *cov_kf_d = nullptr;
    // per-query scratch
    int32_t* cnt = nullptr;
    unsigned long long* first = nullptr;
    int32_t *qw = nullptr, *sel = nullptr;
    double* qv = nullptr;
    float* rs = nullptr;                 // mRelocScore snapshot of the query
    int32_t* ctl = nullptr;              // [0] max common words, [1] selected count
    struct Rec* rec = nullptr;           // per selected keyframe, compacted
    int q_cap = 0;

    void release() {
        void* ps[] = {bow_off, bow_words, inv_off, inv_kf, bow_vals, cnt, first, qw, sel, qv, rs, ctl, rec,
                      cov_off_d, cov_kf_d};
        for (void* p : ps)
            if (p) (void)hipFree(p);
        bow_off = bow_words = inv_off = inv_kf = cnt = qw = sel = nullptr;
        bow_vals = qv = nullptr;
        first = nullptr;
        rs = nullptr;
        ctl = nullptr;
        rec = nullptr;
        cov_off_d = cov_kf_d = nullptr;
        q_cap = 0;
    }
};

namespace orbmi {

__global__ __launch_bounds__(256) void k_kfdb_reset(int nkf, int32_t* cnt, unsigned long long* first) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < nkf) {
        cnt[i] = 0;
        first[i] = ~0ull;
    }
}

__global__ __launch_bounds__(256) void k_kfdb_count(const int32_t* qw, const int32_t* inv_off, const int32_t* inv_kf,
                                                    int32_t* cnt, unsigned long long* first, int32_t* ctl) {
    const int r = blockIdx.x;
    const int w = qw[r];
    const int e0 = inv_off[w], e1 = inv_off[w + 1];
    for (int e = e0 + threadIdx.x; e < e1; e += 256) {
        const int kf = inv_kf[e];
        const int c = atomicAdd(&cnt[kf], 1) + 1;
        atomicMax(&ctl[0], c);
        atomicMin(&first[kf], ((unsigned long long)r << 32) | (unsigned long long)(e - e0));
    }
}

// keyframes with more than (int)(max * 0.8f) shared words (:762-780)
__global__ __launch_bounds__(256) void k_kfdb_select(int nkf, const int32_t* cnt, const unsigned long long* first,
                                                     int32_t* ctl, int32_t* sel, Rec* rec) {
    const int kf = blockIdx.x * 256 + threadIdx.x;
    if (kf >= nkf) return;
    const int minCommonWords = ctl[0] * 0.8f;
    if (cnt[kf] > minCommonWords) {
        const int t = atomicAdd(&ctl[1], 1);
        sel[t] = kf;
        rec[t].first = first[kf];
        rec[t].kf = kf;
    }
}

// LDS holds up to kQ query entries; longer queries read from global memory
constexpr int kQ = 1024;

// L1Scoring::score (ScoringObject.cpp) per selected keyframe
__global__ __launch_bounds__(256) void k_kfdb_score(const int32_t* ctl, const int32_t* sel, int nq, const int32_t* qw,
                                                    const double* qv, const int32_t* bow_off,
                                                    const int32_t* bow_words, const double* bow_vals, float* rs,
                                                    Rec* rec) {
    __shared__ int32_t sw[kQ];
    __shared__ double sv[kQ];
    const int nsel = ctl[1];
    if ((int)blockIdx.x * 256 >= nsel) return;
    const bool lds = nq <= kQ;
    if (lds)
        for (int i = threadIdx.x; i < nq; i += 256) {
            sw[i] = qw[i];
            sv[i] = qv[i];
        }
    __syncthreads();
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= nsel) return;
    const int32_t* W1 = lds ? sw : qw;
    const double* V1 = lds ? sv : qv;
    const int kf = sel[t];
    int i = 0, j = bow_off[kf];
    const int j1 = bow_off[kf + 1];
    double s = 0;
    while (i < nq && j < j1) {
        const int a = W1[i], b = bow_words[j];
        if (a == b) {
            const double vi = V1[i], wi = bow_vals[j];
            s += fabs(vi - wi) - fabs(vi) - fabs(wi);
            ++i;
            ++j;
        } else if (a < b) {
            ++i;
        } else {
            ++j;
        }
    }
    const float si = (float)(-s / 2.0);
    rec[t].score = si;
    rs[kf] = si;                                  // pKFi->mRelocScore = si
}

// neighbour values after scoring (stale mRelocScore for unscored sharers)
__global__ __launch_bounds__(256) void k_kfdb_neigh(const int32_t* ctl, const int32_t* cov_off, const int32_t* cov_kf,
                                                    const int32_t* cnt, const float* rs, Rec* rec) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= ctl[1]) return;
    Rec& r = rec[t];
    const int e0 = cov_off[r.kf], ne = min(10, cov_off[r.kf + 1] - e0);
    int sh = 0;
    for (int j = 0; j < 10; ++j) {
        const int kf2 = j < ne ? cov_kf[e0 + j] : -1;
        r.nb_kf[j] = kf2;
        r.nb_score[j] = kf2 >= 0 ? rs[kf2] : 0.f;
        if (kf2 >= 0 && cnt[kf2] > 0) sh |= 1 << j;
    }
    r.nb_shares = sh;
}

template <typename T>
static int dput(T*& dst, const T* src, size_t n) {
    if (dst) (void)hipFree(dst);
    dst = nullptr;
    ORB_CHECK(hipMalloc(&dst, std::max<size_t>(1, n) * sizeof(T)));
    if (n) ORB_CHECK(hipMemcpy(dst, src, n * sizeof(T), hipMemcpyHostToDevice));
    return ORB_OK;
}

}  // namespace orbmi

using namespace orbmi;

extern "C" {

orbk_db* orbk_db_create(int device) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return nullptr;
    orbk_db* db = new orbk_db();
    db->device = device;
    return db;
}

void orbk_db_destroy(orbk_db* db) {
    if (!db) return;
    (void)hipSetDevice(db->device);
    db->release();
    delete db;
}

int orbk_db_upload(orbk_db* db, int nkf, const int32_t* bow_off, const int32_t* bow_words, const double* bow_vals,
                   int nwords, const int32_t* inv_off, const int32_t* inv_kf, const int32_t* cov_off,
                   const int32_t* cov_kf, const int32_t* kf_map) {
    if (!db || nkf < 0 || nwords < 0 || !bow_off || !inv_off || !cov_off || (nkf && !kf_map)) return ORB_ERR_PARAM;
    if (hipSetDevice(db->device) != hipSuccess) return ORB_ERR_DEVICE;
    db->release();
    db->nkf = nkf;
    db->nwords = nwords;
    int rc;
    const size_t nb = bow_off[nkf], ni = inv_off[nwords];
    if ((rc = dput(db->bow_off, bow_off, (size_t)nkf + 1)) || (rc = dput(db->bow_words, bow_words, nb)) ||
        (rc = dput(db->bow_vals, bow_vals, nb)) || (rc = dput(db->inv_off, inv_off, (size_t)nwords + 1)) ||
        (rc = dput(db->inv_kf, inv_kf, ni)))
        return rc;
    for (int k = 0; k < nkf; ++k)
        if (cov_off[k + 1] - cov_off[k] > 10) return ORB_ERR_PARAM;        // GetBestCovisibilityKeyFrames(10)
    db->kf_map.assign(kf_map, kf_map + nkf);
    if ((rc = dput(db->cov_off_d, cov_off, (size_t)nkf + 1)) || (rc = dput(db->cov_kf_d, cov_kf, (size_t)cov_off[nkf])))
        return rc;
    ORB_CHECK(hipMalloc(&db->rs, std::max(1, nkf) * sizeof(float)));
    ORB_CHECK(hipMalloc(&db->ctl, 2 * sizeof(int32_t)));
    ORB_CHECK(hipMalloc(&db->rec, std::max(1, nkf) * sizeof(Rec)));
    ORB_CHECK(hipMalloc(&db->cnt, std::max(1, nkf) * sizeof(int32_t)));
    ORB_CHECK(hipMalloc(&db->first, std::max(1, nkf) * sizeof(unsigned long long)));
    ORB_CHECK(hipMalloc(&db->sel, std::max(1, nkf) * sizeof(int32_t)));
    return ORB_OK;
}

int orbk_detect_relocalization_candidates(orbk_db* db, const int32_t* q_words, const double* q_vals, int nq,
                                          int32_t map_id, float* reloc_score, int32_t* cand, int cap) {
    if (!db || nq < 0 || (nq && (!q_words || !q_vals)) || !reloc_score || (cap > 0 && !cand)) return ORB_ERR_PARAM;
    if (nq == 0 || db->nkf == 0) return 0;
    for (int r = 0; r < nq; ++r)
        if (q_words[r] < 0 || q_words[r] >= db->nwords || (r && q_words[r] <= q_words[r - 1])) return ORB_ERR_PARAM;
    if (hipSetDevice(db->device) != hipSuccess) return ORB_ERR_DEVICE;
    if (nq > db->q_cap) {
        if (db->qw) (void)hipFree(db->qw);
        if (db->qv) (void)hipFree(db->qv);
        db->qw = nullptr;
        db->qv = nullptr;
        ORB_CHECK(hipMalloc(&db->qw, nq * sizeof(int32_t)));
        ORB_CHECK(hipMalloc(&db->qv, nq * sizeof(double)));
        db->q_cap = nq;
    }
    const int nkf = db->nkf;
    hipStream_t st = 0;
    ORB_CHECK(hipMemcpyAsync(db->qw, q_words, nq * sizeof(int32_t), hipMemcpyHostToDevice, st));
    ORB_CHECK(hipMemcpyAsync(db->qv, q_vals, nq * sizeof(double), hipMemcpyHostToDevice, st));
    ORB_CHECK(hipMemcpyAsync(db->rs, reloc_score, nkf * sizeof(float), hipMemcpyHostToDevice, st));
    ORB_CHECK(hipMemsetAsync(db->ctl, 0, 2 * sizeof(int32_t), st));
    const dim3 g((nkf + 255) / 256);
    ORB_LAUNCH(k_kfdb_reset, g, dim3(256), 0, st, nkf, db->cnt, db->first);
    ORB_LAUNCH(k_kfdb_count, dim3(nq), dim3(256), 0, st, db->qw, db->inv_off, db->inv_kf, db->cnt, db->first,
                       db->ctl);
    ORB_LAUNCH(k_kfdb_select, g, dim3(256), 0, st, nkf, db->cnt, db->first, db->ctl, db->sel, db->rec);
    ORB_LAUNCH(k_kfdb_score, g, dim3(256), 0, st, db->ctl, db->sel, nq, db->qw, db->qv, db->bow_off,
                       db->bow_words, db->bow_vals, db->rs, db->rec);
    ORB_LAUNCH(k_kfdb_neigh, g, dim3(256), 0, st, db->ctl, db->cov_off_d, db->cov_kf_d, db->cnt, db->rs,
                       db->rec);
    ORB_CHECK(hipGetLastError());
    int32_t ctl[2];
    ORB_CHECK(hipMemcpy(ctl, db->ctl, sizeof(ctl), hipMemcpyDeviceToHost));
    const int nsel = ctl[1];
    if (ctl[0] == 0 || nsel == 0) return 0;               // nothing shares a word / nothing scored
    std::vector<Rec> rec(nsel);
    ORB_CHECK(hipMemcpy(rec.data(), db->rec, nsel * sizeof(Rec), hipMemcpyDeviceToHost));
    // lScoreAndMatch in lKFsSharingWords order (:740-787)
    std::sort(rec.begin(), rec.end(), [](const Rec& x, const Rec& y) { return x.first < y.first; });
    for (const Rec& r : rec) reloc_score[r.kf] = r.score;
    // covisibility accumulation (:792-819)
    std::vector<std::pair<float, int>> acc;
    acc.reserve(nsel);
    float bestAccScore = 0;
    for (const Rec& r : rec) {
        float bestScore = r.score, accScore = bestScore;
        int best_kf = r.kf;
        for (int j = 0; j < 10; ++j) {
            if (r.nb_kf[j] < 0 || !((r.nb_shares >> j) & 1)) continue;
            accScore += r.nb_score[j];
            if (r.nb_score[j] > bestScore) {
                best_kf = r.nb_kf[j];
                bestScore = r.nb_score[j];
            }
        }
        acc.emplace_back(accScore, best_kf);
        if (accScore > bestAccScore) bestAccScore = accScore;
    }
    const float minScoreToRetain = 0.75f * bestAccScore;                          // :822-842
    std::vector<char> added(nkf, 0);
    int n = 0;
    for (auto& a : acc) {
        if (a.first > minScoreToRetain) {
            const int kf = a.second;
            if (db->kf_map[kf] != map_id) continue;
            if (!added[kf]) {
                if (n < cap) cand[n] = kf;
                ++n;
                added[kf] = 1;
            }
        }
    }
    return n;
}

}  // extern "C"
