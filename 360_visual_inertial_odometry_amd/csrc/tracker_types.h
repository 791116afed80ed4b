// tracker_types.h — kernel argument blocks of the ERP tracker (tracker.hip), shared with the host
// side (tracker_host.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vio360 {

constexpr int TRK_MAX_LEVELS = 8;

struct PyrLevelPair {  // one pyramid level of both frames (same geometry)
    uint8_t* p0;
    uint8_t* p1;
    int w, h, pitch;
};

struct LkLevel {
    const uint8_t* prev;
    const uint8_t* curr;
    int w, h, pitch;
};

struct LkArgs {
    LkLevel lv[TRK_MAX_LEVELS];
    int levels;  // top level index (maxLevel after buildOpticalFlowPyramid's size check)
    const float* pts;
    float* next;
    uint8_t* status;
    float* err;
    int n, win, max_iters;
    float min_eig;
    double eps2;
    float* bear1;  // [n][3] or null: the bearing of each tracked point (tracker pipeline: RANSAC's input)
};

struct RansacArgs {
    const float* p0;       // [n][2] previous points
    const float* p1;       // [n][2] tracked points
    const uint8_t* status; // [n] (mode 1)
    int n, W, H, mode;     // mode 0: every point enters RANSAC; 1: status/polar/boundary filter first
    float polar_ratio;
    int margin;
    int* gidx;             // [n] compacted -> input index
    int* n_good;           // device scalar
    float* b0;             // [n][3] bearings of the compacted points
    float* b1;
    const float* bear0;    // [n][3] or null: every input point's bearings already formed (tracker pipeline: the
    const float* bear1;    // LK launch); the compaction then copies them instead of evaluating the trigonometry
    int32_t* samples;      // [iters][3]
    const uint32_t* raw;   // [RS_RAW] tempered mt19937 words of `seed` (ransac_raw_kernel)
    int iters;
    uint32_t seed;
    float thresh;
    float* cmin;           // device scalar: the inlier test's cosine bound for thresh (ransac_cos_bound)
    int* count;            // [iters]
    float* rot;            // [iters][9] each hypothesis' rotation (ransac_hyp), read back for the best
    uint8_t* kept;         // [n] output mask in input order
    int* n_in;             // device scalar
};

struct GfArgs {
    const uint8_t* img;
    int W, H, pitch;
    // mask: explicit u8 (mask != null), else analytic region + optional disc bitmask
    const uint8_t* mask;
    int mask_pitch;
    int top_rows, bottom_start, margin;
    const uint32_t* disc_bits;
    int disc_words;  // 32-bit words per row
    double quality, min_dist;
    int max_corners;
    uint32_t* max_ord;              // device scalar (ordered-int max of the masked eig map)
    float* eig;                     // [H][W] min-eigenvalue map, written by pass 1, read by pass 2
    unsigned long long* cand;       // [cand_cap]
    unsigned long long* cand_sorted;
    unsigned int* n_cand;           // device scalar
    unsigned int cand_cap;
    int cell, gw, gh;
    uint32_t* grid_global;          // non-null when the selection grid does not fit LDS
    float* corners;                 // [max_corners][2]
    int* n_out;                     // device scalar
    // top-K fast path: histogram of candidate responses, the strongest candidates compacted and
    // sorted; `incomplete` is raised when the greedy pass needs candidates beyond them
    unsigned int* hist;             // [GF_BUCKETS]
    unsigned long long* topk;       // [topk_cap]
    unsigned long long* topk_sorted;
    unsigned int* n_top;            // device scalar
    int* cut;                       // device scalar: [0] cut bucket [1] everything selected
    unsigned int topk_cap, topk_target;
    int* incomplete;                // device scalar
    // local-maximum path (analytic mask: polar rows / side margins / discs; no explicit mask):
    // pass 1 (mask independent, side stream) keeps per LM_TX x LM_TY tile the 3x3 local maxima of
    // the eigenvalue map inside the static region (fixed slots of LM_CAP keys) and the tile's
    // maximum over that region; the map itself is never written
    unsigned long long* lmax;       // [n_tiles][LM_CAP]
    unsigned int* lmax_n;           // [n_tiles] local maxima of the tile (> LM_CAP: overflow)
    uint32_t* tile_max;             // [n_tiles] ordered-int max over the tile's static region (0: none)
    uint8_t* tile_dirty;            // [n_tiles] a disc covers part of the tile's static region
    uint32_t* tile_kmax;            // [n_tiles] histogram bucket of the tile's strongest local maximum
    int tiles_x, tiles_y;
    int* lmax_over;                 // device scalar: some tile overflowed its slots
    unsigned int* n_flat;           // device scalar: fill counter of the flattened candidate list
    // gftt_select_kernel over the presorted prefix of every local maximum (launch_gftt_presel): disc test
    // and the threshold's upper bound in its pre-filter, `incomplete` when the prefix cannot decide
    int presel;
    uint32_t* smax;       // ordered-int max of the tiles' static-region maxima: gftt_lm_hist_kernel reduces it when
                          // non-null (the presort), the presel pass reads it (its threshold bound)
    unsigned int* clear;  // gftt_lmax_kernel: words zeroed by its first workgroup (the presort's histogram)
    int clear_n;
    // device-side hand-off of the presort's result to the presel pass (no cross-stream event wait between them):
    // every workgroup of the presort's sort kernel adds 1 to *done after its stores (agent-scope release); the
    // presel pass polls *wait_ctr until it reaches wait_target (a per-run generation x the sort's grid), then
    // acquires; on a time-out it reports `incomplete` and the host runs the exact tail after syncing both streams
    unsigned int* done;
    const unsigned int* wait_ctr;
    unsigned int wait_target;
};

constexpr int LM_TX = 64, LM_TY = 32, LM_CAP = 1024;

constexpr int GF_BUCKETS = 2048;    // float bits >> 20 of a positive response
constexpr int kPresortWords = GF_BUCKETS + 8;  // the presort's histogram + scalars
constexpr int kPresortClear = GF_BUCKETS + 6;  // cleared per run (word 6: the monotonic hand-off counter)
// top-K buffer: the strongest candidates (>= 16 x max_corners of them when the buckets allow) sorted
// for the greedy selection; a selection that runs dry falls back to the full candidate sort
constexpr unsigned int GF_TOPK_CAP = 16384;
// dynamic LDS of the greedy selection (grid of 3 slots x 4 B per min-distance cell, + 4 B chain head per
// cell), next to its ~20.4 KB of static LDS (the presel stage buffer included) within the CU's 160 KB;
// larger grids live in global memory
constexpr size_t GF_SELECT_LDS_MAX = 136 * 1024;

struct DiscArgs {
    const float* pts;       // [n][2]
    const uint8_t* kept;    // [n] or null (every point)
    const int* src_index;   // null: point k = pts[k]
    const int* n_pts_dev;   // device scalar: number of points, or null (grid = point count)
    uint32_t* bits;
    int words, W, H, radius;
    const int* halfw;       // [radius+1]
};

hipError_t launch_pyr_down(const PyrLevelPair& s, const PyrLevelPair& d, int frames, hipStream_t st);
// work riding in extra workgroups of the LK launch (tracker pipeline, off LK's critical path and
// without a cross-stream wait): the RANSAC draws' raw mt19937 words, the GFTT counters / histogram /
// top-K reset and the disc bitmap clear (null pointers: none)
struct LkAux {
    uint32_t* raw;
    uint32_t seed;
    float thresh;  // RANSAC angle threshold: its cosine bound into *cmin (beside the raw draws)
    float* cmin;
    unsigned int* hist;
    unsigned long long* topk;
    unsigned int topk_cap;
    int* scal;
    uint32_t* disc;
    size_t disc_words;  // total 32-bit words of the bitmap
    const float* pts;   // the previous points' bearings (RANSAC's input) into bear0 [n][3] (null: none)
    float* bear0;
    int n, W, H;
};
hipError_t launch_lk(const LkArgs& a, hipStream_t st, const LkAux* aux = nullptr);
// the tempered mt19937 stream of a seed (independent of the points: may run on another stream)
hipError_t launch_ransac_raw(uint32_t seed, uint32_t* raw, hipStream_t st);
size_t ransac_raw_words();
// gen_samples: hypotheses drawn on device from r.raw (launch_ransac_raw of r.seed must precede)
hipError_t launch_ransac(const RansacArgs& r, bool gen_samples, hipStream_t st);
hipError_t launch_disc_mask(const DiscArgs& d, int max_pts, hipStream_t st);
// tracker pipeline: sampler (with the input compaction), hypotheses, then selection + discs in one launch
hipError_t launch_ransac_pipeline(const RansacArgs& r, const DiscArgs& d, hipStream_t st);
// fast path (top-K) and the exact fallback over every candidate (used when `incomplete` is raised)
// presort (side stream, after pass 1, before the disc mask): histogram, top-K cut and sort of EVERY local
// maximum of the static region (g: the pass-1 arguments with the presort's hist / topk / n_top / cut and a
// zero max_ord, no disc bitmap); presel: the greedy pass over that prefix with the disc test (g: the full
// arguments with presel = 1 and the presort's cut)
hipError_t launch_gftt_presort(const GfArgs& g, hipStream_t st);
hipError_t launch_gftt_presel(const GfArgs& g, const unsigned long long* keys, const unsigned int* n_keys,
                              hipStream_t st);
hipError_t launch_gftt_eig(const GfArgs& g, hipStream_t st);  // the min-eigenvalue map (needs img, W, H, pitch, eig)
hipError_t launch_gftt(const GfArgs& g, void* sort_tmp, size_t sort_tmp_bytes, hipStream_t st);  // after the map
hipError_t launch_gftt_full(const GfArgs& g, unsigned int count, void* sort_tmp, size_t sort_tmp_bytes,
                            hipStream_t st);  // sorts the first `count` candidates (n_cand read back)
hipError_t launch_gftt_reset(const GfArgs& g, int* scal, hipStream_t st);
// local-maximum path: pass 1 (mask independent) and everything after the mask is known
hipError_t launch_gftt_lmax(const GfArgs& g, hipStream_t st);
hipError_t launch_gftt_after_lmax(const GfArgs& g, void* sort_tmp, size_t sort_tmp_bytes, hipStream_t st);
// exact fallback of the local-maximum path: flatten the surviving candidates, then launch_gftt_full
hipError_t launch_gftt_flatten(const GfArgs& g, hipStream_t st);
size_t gftt_sort_tmp_bytes(unsigned int cap);
hipError_t gftt_select_set_lds(size_t bytes);

}  // namespace vio360
