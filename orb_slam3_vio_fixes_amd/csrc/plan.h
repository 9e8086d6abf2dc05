// plan.h — extractor plan and handle (shared by extractor.hip and stereo.hip).
#pragma once
#include "../../include/orb_mi355x.h"
#include "common.h"

#include <vector>

namespace orbmi {

constexpr int kMaxLevels = 32;

// ---------------------------------------------------------------------------
// Plan: everything that depends only on (params, w, h), computed once on the
// host with the reference's own float/double expressions.
// ---------------------------------------------------------------------------
struct LevelDev {
    int w, h, pitch;
    long long off;      // byte offset of the level inside one frame's pyramid slab (l >= 1)
    float scale;
    int patch;          // int(PATCH_SIZE * scale)  (ORBextractor.cc:880)
    // quadtree (DistributeOctTree arguments, ORBextractor.cc:877-878)
    int qW, qH, N, nIni;
    float hX;
    int cell_base, ncells, slot_base, slot_total;   // cells / key slots of this level
    int out_base, out_cap;                          // quadtree output slots
    // k_pyramid tables (l >= 1): column taps at xtab (padded to a multiple of
    // 4 columns), row taps at ytab
    int xtab, ytab;
    // the fused pre-test's candidate bitmap (k_pyr_stream -> k_fast_cells): one
    // bit per pixel (bit x & 7 of byte x >> 3 of a row), rows of bm_pitch bytes
    // at bm_off of the frame's bitmap slab
    long long bm_off;
    int bm_pitch;
};

// One launch of k_pyramid: levels la+1..lb from level la, in nb bands of
// rows per frame (band b owns rows of every level it writes; the rows it
// needs below are recomputed as a halo).  band_off indexes the device band
// table: int4 {n0, n1, p0, p1} per (band, level la..lb).
struct PyrGroup {
    int la, lb, nb, R;
    long long band_off;
    int lds_a, lds_b, lds_x, lds_y;   // LDS: two level buffers, column taps, row taps
};

// k_pyr_stream: one workgroup per frame slides down the frame once, keeping
// a ring of the most recent rows of every level but the last in LDS (no halo
// recompute, level 0 read once).  Host-side layout of its LDS image.
constexpr int kPsMaxLevels = 16;
struct PyrStream {
    bool ok = false;
    int K0 = 0, nchunks = 0, nsteps = 0;   // level-0 rows per chunk; chunks; pipeline steps
    int tab_u4 = 0;                        // table image (uint4 units) = the first bytes of LDS
    int lev_u4 = 0, steps_u4 = 0;          // level table {rec_dw, yt_dw} [L]; step table [nsteps][L]
    int lds_bytes = 0;
    int ring_rows[kPsMaxLevels] = {}, ring_pitch[kPsMaxLevels] = {};   // levels 0..L-2
    int ring_dw[kPsMaxLevels] = {};        // LDS dword offset of each ring
    int rec_dw[kPsMaxLevels] = {};         // level l >= 1: column records W[ng] uint4, S[ng] uint4, BF[ng] u32
    int yt_dw[kPsMaxLevels] = {};          // level l >= 1: row records uint4 per row
    int ng[kPsMaxLevels] = {};             // column groups of 4 per level
    int cnt_dw = 0;                        // per-step wave-item counters (LDS dword offset)
    // fused FAST pre-test at iniThFAST (k_fast_cells then reads the bitmap):
    // per level the window rows [pt_y0, pt_y1) and 16-pixel groups
    // [pt_gx0, pt_gx0 + pt_ngx); E step entries per step (2L with it, L without)
    bool pretest = false;
    int E = 0;
    int pt_y0[kPsMaxLevels] = {}, pt_y1[kPsMaxLevels] = {}, pt_gx0[kPsMaxLevels] = {}, pt_ngx[kPsMaxLevels] = {};
};

struct CellDev {
    int level;
    int x0, y0, cols, rows;   // ROI in level coordinates (ORBextractor.cc:807-826)
    int slot_off, cap;        // key slots (u32) relative to the frame's slot slab
    // levels >= 1: the ROI's first dword (row y0, column x0 & ~3) as a byte
    // offset in the frame's pyramid slab, and the level pitch, so k_fast_cells
    // addresses it from the cell record alone (no dependent level-table load
    // before its first ROI load); level 0 (the caller's image) uses its pitch
    int roi_off, pitch;
};

struct Plan {
    int w = 0, h = 0, L = 0, maxB = 0;
    std::vector<LevelDev> lv;
    std::vector<CellDev> cells;
    long long pyr_bytes = 0;
    int ncells = 0, slot_total = 0, out_total = 0;
    int roi_max = 0, roi_rows_max = 0, roi_nd_max = 0, win_max = 0, max_level_cells = 0, max_out_cap = 0;
    int win_pix_max = 0;             // largest FAST window (cols-6)*(rows-6): candidate list entries
    int item_max = 0;                // most FAST pre-test items of a cell (k_fast_cells item list; < 65536)
    std::vector<int> win_y0, win_y1, win_x0, win_x1;   // per level: union of the FAST windows
    bool bm_ok = false;              // every window <= 64 x 64 px (k_fast_cells' bitmap path)
    long long bm_bytes = 0;          // one frame's pre-test bitmap (k_pyr_stream with ps.pretest)
    std::vector<int> xmax;           // per level
    std::vector<long long> tab_off;  // per level: offset (int2 units) of the x table, y table follows
    std::vector<PyrGroup> pgroups;   // k_pyramid launches
    PyrStream ps;                    // k_pyr_stream layout (ps.ok: usable for this size)
    // device
    uint8_t *d_pyr = nullptr, *d_in = nullptr;
    int2* d_tab = nullptr;
    LevelDev* d_lv = nullptr;
    CellDev* d_cells = nullptr;
    int* d_cell_count = nullptr;
    uint32_t *d_cell_keys = nullptr, *d_key_scr = nullptr;
    int* d_knode = nullptr;
    uint8_t* d_kq = nullptr;
    uint32_t* d_qt_key = nullptr;
    int* d_qt_n = nullptr;
    int* d_qt_ovf = nullptr;         // [maxB][L] k_quadtree_w overflow flags (levels left to k_quadtree)
    float* d_angle = nullptr;
    uint8_t* d_sdesc = nullptr;
    uint8_t* d_slot_level = nullptr;
    int4* d_pband = nullptr;         // k_pyramid band tables
    int* d_pxs = nullptr;            // k_pyramid column taps: source column
    uint32_t* d_pxw = nullptr;       //   and weights a0 | a1 << 16
    int2* d_pyt = nullptr;           // k_pyramid row taps: sy0 | sy1 << 16 (clamped), b0 | b1 << 16
    uint4* d_ps_tab = nullptr;       // k_pyr_stream LDS table image
    uint8_t* d_bm = nullptr;         // [maxB][bm_bytes] pre-test bitmaps (ps.pretest)
    uint8_t* d_qt_gscr = nullptr;    // [maxB][L][stride] k_quadtree node arrays of levels beyond the LDS
    // single-image host path outputs
    orb_keypoint* d_kps = nullptr;
    uint8_t* d_desc = nullptr;
    int32_t *d_n = nullptr, *d_mono = nullptr;
    int host_cap = 0;
    size_t in_pitch = 0;

    void release() {
        void* ps[] = {d_pyr, d_in, d_tab, d_lv, d_cells, d_cell_count, d_cell_keys, d_key_scr,
                      d_knode, d_kq, d_qt_key, d_qt_n, d_angle, d_sdesc, d_kps, d_desc, d_n, d_mono,
                      d_slot_level, d_pband, d_pxs, d_pxw, d_pyt, d_ps_tab, d_bm, d_qt_gscr, d_qt_ovf};
        for (void* p : ps)
            if (p) (void)hipFree(p);
        *this = Plan();
    }
};

}  // namespace orbmi

struct orbx_handle {
    orbx_params prm{};
    int device = 0;
    std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
    std::vector<int> nfeat, umax;
    orbmi::Plan plan;
    bool have_last = false;
    int last_w = 0, last_h = 0;
    int last_n = 0;                  // keypoints of the last orbx_extract (in plan.d_kps / d_desc)
    // optional per-stage HIP-event timing (orbx_set_profiling)
    bool profiling = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::vector<hipEvent_t>> ev_calls;
    size_t ev_next = 0;
    // sub-batch streams (orbx_set_streams)
    int nsub = 1;
    // pyramid kernel choice (orbx_set_pyramid_mode) and the last one run
    int pyr_mode = 0, pyr_last = 0;
    bool bm_last = false;            // the last extraction's FAST candidates came from the fused pre-test
    // caller events recorded after pipeline stages (orbx_set_stage_event)
    hipEvent_t stage_ev[6] = {};
    std::vector<hipStream_t> sub_streams;
    std::vector<hipEvent_t> sub_done;
    hipEvent_t fork_ev = nullptr;
    hipEvent_t batch_done = nullptr;   // recorded after orbx_extract_batch_device's work on its stream
    // frames of the last orbx_extract_batch_device call (level 0 of its
    // pyramid; levels >= 1 stay in plan.d_pyr until the next call)
    const uint8_t* last_frames = nullptr;
    long long last_fstride = 0;
    int last_pitch0 = 0, last_B = 0;
    // device scratch of the stereo matcher (stereo.hip), grown on demand
    void* st_scratch = nullptr;
    size_t st_scratch_bytes = 0;
    // orbx_extract_batch (host images): staged frames on the device, the batch
    // outputs, and the pinned staging both ways; grown on demand
    void* hb_dev = nullptr;
    size_t hb_dev_bytes = 0;
    void* hb_pin = nullptr;
    size_t hb_pin_bytes = 0;
    // orbx_extract as one captured hipGraph (upload, pipeline, downloads) per
    // (size, lapping, plan epoch, staging buffer); build_plan bumps the epoch
    int plan_epoch = 0;
    hipStream_t x_stream = nullptr;
    hipGraphExec_t x_exec = nullptr;
    long long x_key[7] = {0, 0, 0, 0, -1, 0, 0};
    void* x_pin = nullptr;
    size_t x_pin_bytes = 0;
    int x_pin_gen = 0;
    bool host_pyr = false;           // orbx_set_host_pyramid: the graph also downloads levels 1.. to x_pin
    bool x_pyr_valid = false;        // x_pin holds the last orbx_extract's pyramid (level 0 = its input)
    size_t x_pyr_off = 0;            // levels 1.. in x_pin (at the plan's per-frame pyramid layout)
};
