// vocab.cpp — DBoW2 vocabulary side of the path,
// host code of the product library:
//   * the text vocabulary format: TemplatedVocabulary::loadFromTextFile
//     (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1424) into the
//     orbv_vocab layout the GPU descent (orbv_transform) reads;
//   * BowVector / FeatureVector assembly of transform(features, v, fv,
//     levelsup) (:1126-1194) from the per-descriptor (word, weight, node) the
//     GPU descent returns, with BowVector::addWeight / addIfNotExist /
//     normalize (BowVector.cpp) and FeatureVector::addFeature;
//   * the six ScoringObject scores (ScoringObject.cpp).
// The loader is a byte-level parser (the reference uses getline + stringstream,
// ~20 s for ORBvoc.txt) that reproduces the stream semantics on well-formed and
// truncated lines, including the reference's treatment of a trailing newline.
#include "../../include/orb_mi355x.h"

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

struct orbv_text_vocab {
    int k = 0, L = 0, scoring = 0, weighting = 0, nwords = 0;
    std::vector<int32_t> first_child, nchild, child_idx, word_id;
    std::vector<uint8_t> desc;
    std::vector<double> weight;
};

namespace {

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; }

// One line read like `std::stringstream ss(line); ss >> a >> b ...`: once an
// extraction fails the stream stays failed and every later target gets 0
// (C++11 num_get).  Tokens are whitespace-delimited.
struct LineStream {
    const char* p;
    const char* e;
    bool failed = false;
    LineStream(const char* b, const char* end) : p(b), e(end) {}
    bool token(const char*& tb, const char*& te) {
        while (p < e && is_space(*p)) ++p;
        if (p >= e) return false;
        tb = p;
        while (p < e && !is_space(*p)) ++p;
        te = p;
        return true;
    }
    long get_int() {
        if (failed) return 0;
        const char *tb, *te;
        if (!token(tb, te)) { failed = true; return 0; }
        std::string t(tb, te);
        char* end = nullptr;
        errno = 0;
        const long v = std::strtol(t.c_str(), &end, 10);
        if (end == t.c_str() || *end != '\0' || errno) { failed = true; return 0; }
        return v;
    }
    double get_double() {
        if (failed) return 0.0;
        const char *tb, *te;
        if (!token(tb, te)) { failed = true; return 0.0; }
        std::string t(tb, te);
        char* end = nullptr;
        const double v = std::strtod(t.c_str(), &end);
        if (end == t.c_str() || *end != '\0') { failed = true; return 0.0; }
        return v;
    }
    // F::fromString of the next L tokens (FORB.cpp:117-133): bytes whose
    // extraction fails keep the value of the freshly created cv::Mat, which
    // is undefined in the reference; they are 0 here.
    void get_desc(uint8_t* d) {
        std::string joined;
        for (int i = 0; i < 32; ++i) {
            const char *tb, *te;
            if (!failed && token(tb, te)) joined.append(tb, te);
            else failed = true;
            joined.push_back(' ');
        }
        LineStream ds(joined.data(), joined.data() + joined.size());
        for (int i = 0; i < 32; ++i) {
            const long n = ds.get_int();
            d[i] = ds.failed ? 0 : (uint8_t)(unsigned char)n;
        }
    }
};

}  // namespace

extern "C" {

orbv_text_vocab* orbv_load_text(const char* path, int32_t* err) {
    auto fail = [&](int32_t code) -> orbv_text_vocab* {
        if (err) *err = code;
        return nullptr;
    };
    if (!path) return fail(ORB_ERR_PARAM);
    FILE* f = std::fopen(path, "rb");
    if (!f) return fail(ORB_ERR_EMPTY);
    std::string buf;
    {
        char tmp[1 << 16];
        size_t r;
        while ((r = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.append(tmp, r);
        std::fclose(f);
    }
    // lines as std::getline yields them while !eof(): every '\n'-terminated
    // segment, plus the remainder -- an empty remainder after a final '\n'
    // is still read once (getline hits EOF and returns "") and becomes a node
    // (parent 0, not a leaf, weight 0), exactly as in the reference loop
    std::vector<std::pair<size_t, size_t>> lines;
    size_t b = 0;
    while (true) {
        const size_t nl = buf.find('\n', b);
        if (nl == std::string::npos) { lines.emplace_back(b, buf.size()); break; }
        lines.emplace_back(b, nl);
        b = nl + 1;
    }
    orbv_text_vocab* v = new orbv_text_vocab();
    {
        LineStream hs(buf.data() + lines[0].first, buf.data() + lines[0].second);
        v->k = (int)hs.get_int();
        v->L = (int)hs.get_int();
        v->scoring = (int)hs.get_int();
        v->weighting = (int)hs.get_int();
    }
    if (v->k < 0 || v->k > 20 || v->L < 1 || v->L > 10 || v->scoring < 0 || v->scoring > 5 || v->weighting < 0 ||
        v->weighting > 3) {
        delete v;
        return fail(ORB_ERR_PARAM);                        // "This is not a correct text file!"
    }
    // the header line without a '\n' is the whole file: the node loop never runs
    const size_t nnodes = lines.size() == 1 ? 1 : lines.size();
    std::vector<int32_t> parent(nnodes, 0);
    std::vector<std::vector<int32_t>> children(nnodes);
    v->desc.assign(nnodes * 32, 0);
    v->weight.assign(nnodes, 0.0);
    v->word_id.assign(nnodes, 0);                          // Node(): word_id(0)
    for (size_t nid = 1; nid < nnodes; ++nid) {
        LineStream ls(buf.data() + lines[nid].first, buf.data() + lines[nid].second);
        const long pid = ls.get_int();
        if (pid < 0 || (size_t)pid >= nid) {               // the reference indexes m_nodes[pid] unchecked
            delete v;
            return fail(ORB_ERR_PARAM);
        }
        parent[nid] = (int32_t)pid;
        children[pid].push_back((int32_t)nid);
        const long is_leaf = ls.get_int();
        ls.get_desc(&v->desc[nid * 32]);
        v->weight[nid] = ls.get_double();
        if (is_leaf > 0) v->word_id[nid] = v->nwords++;
    }
    v->first_child.assign(nnodes, 0);
    v->nchild.assign(nnodes, 0);
    for (size_t i = 0; i < nnodes; ++i) {
        v->first_child[i] = (int32_t)v->child_idx.size();
        v->nchild[i] = (int32_t)children[i].size();
        v->child_idx.insert(v->child_idx.end(), children[i].begin(), children[i].end());
    }
    if (err) *err = ORB_OK;
    return v;
}

int orbv_text_vocab_view(const orbv_text_vocab* v, orbv_vocab* view, int32_t* k, int32_t* scoring,
                         int32_t* weighting, int32_t* nwords) {
    if (!v || !view) return ORB_ERR_PARAM;
    view->nnodes = (int32_t)v->nchild.size();
    view->depth_levels = v->L;
    view->first_child = v->first_child.data();
    view->nchild = v->nchild.data();
    view->node_desc = v->desc.data();
    view->word_id = v->word_id.data();
    view->weight = v->weight.data();
    view->child_idx = v->child_idx.data();
    if (k) *k = v->k;
    if (scoring) *scoring = v->scoring;
    if (weighting) *weighting = v->weighting;
    if (nwords) *nwords = v->nwords;
    return ORB_OK;
}

void orbv_free_text(orbv_text_vocab* v) { delete v; }

int orbv_bow_assemble(int scoring, int weighting, int n, const int32_t* word_id, const double* weight,
                      const int32_t* node_id, int32_t* bow_words, double* bow_values, int32_t* nbow,
                      int32_t* fv_nodes, int32_t* fv_off, int32_t* fv_idx, int32_t* nfv) {
    if (n < 0 || scoring < 0 || scoring > 5 || weighting < 0 || weighting > 3) return ORB_ERR_PARAM;
    if (n && (!word_id || !weight || !node_id)) return ORB_ERR_PARAM;
    if (!bow_words || !bow_values || !nbow || !fv_nodes || !fv_off || !fv_idx || !nfv) return ORB_ERR_PARAM;
    std::map<int32_t, double> v;                           // BowVector
    std::map<int32_t, std::vector<int32_t>> fv;            // FeatureVector
    const bool tf = weighting == 0 || weighting == 1;      // TF_IDF, TF: addWeight; IDF, BINARY: addIfNotExist
    for (int i = 0; i < n; ++i) {
        if (weight[i] > 0) {                               // not stopped (:1161)
            if (tf) v[word_id[i]] += weight[i];
            else v.emplace(word_id[i], weight[i]);
            fv[node_id[i]].push_back(i);
        }
    }
    const bool must = scoring != 5;                        // DotProductScoring does not normalise
    const bool l2 = scoring == 1;
    if (tf && !v.empty() && !must) {
        const double nd = (double)v.size();
        for (auto& kv : v) kv.second /= nd;
    }
    if (must) {                                            // BowVector::normalize
        double norm = 0.0;
        if (!l2) {
            for (auto& kv : v) norm += std::fabs(kv.second);
        } else {
            for (auto& kv : v) norm += kv.second * kv.second;
            norm = std::sqrt(norm);
        }
        if (norm > 0.0)
            for (auto& kv : v) kv.second /= norm;
    }
    int j = 0;
    for (auto& kv : v) { bow_words[j] = kv.first; bow_values[j] = kv.second; ++j; }
    *nbow = j;
    int m = 0, off = 0;
    for (auto& kv : fv) {
        fv_nodes[m] = kv.first;
        fv_off[m] = off;
        for (int32_t idx : kv.second) fv_idx[off++] = idx;
        ++m;
    }
    fv_off[m] = off;
    *nfv = m;
    return ORB_OK;
}

double orbv_score(int scoring, const int32_t* w1, const double* v1, int n1, const int32_t* w2, const double* v2,
                  int n2) {
    static const double LOG_EPS = std::log(DBL_EPSILON);
    double score = 0;
    int i = 0, j = 0;
    // the lower_bound jumps of the reference visit the common words in order;
    // KL also adds every v1 entry absent from v2
    while (i < n1 && j < n2) {
        const double vi = v1[i], wi = v2[j];
        if (w1[i] == w2[j]) {
            switch (scoring) {
                case 0: score += std::fabs(vi - wi) - std::fabs(vi) - std::fabs(wi); break;
                case 1: case 5: score += vi * wi; break;
                case 2: if (vi + wi != 0.0) score += vi * wi / (vi + wi); break;
                case 3: if (vi != 0 && wi != 0) score += vi * std::log(vi / wi); break;
                case 4: score += std::sqrt(vi * wi); break;
            }
            ++i;
            ++j;
        } else if (w1[i] < w2[j]) {
            if (scoring == 3) { score += vi * (std::log(vi) - LOG_EPS); ++i; }
            else i = (int)(std::lower_bound(w1 + i, w1 + n1, w2[j]) - w1);
        } else {
            j = (int)(std::lower_bound(w2 + j, w2 + n2, w1[i]) - w2);
        }
    }
    switch (scoring) {
        case 0: return -score / 2.0;
        case 1: return score >= 1 ? 1.0 : 1.0 - std::sqrt(1.0 - score);
        case 2: return 2. * score;
        case 3:
            for (; i < n1; ++i)
                if (v1[i] != 0) score += v1[i] * (std::log(v1[i]) - LOG_EPS);
            return score;
        default: return score;
    }
}

}  // extern "C"
