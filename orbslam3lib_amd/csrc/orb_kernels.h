// orb_kernels.h -- launch-argument structs shared by orb_kernels.hip and orb_runtime.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace orbgpu {

constexpr int kMaxLevels = 16;
constexpr int kMinBorder = 16;   // EDGE_THRESHOLD - 3 (ORBextractor_old.cc:791)
constexpr int kEdge = 19;        // EDGE_THRESHOLD (:75)

// XCD-aware block order (cdna_hip_programming.md T1, bijective form): the dispatcher places
// block b on XCD b % 8, so a grid walked in (b % 8, b / 8) order gives every XCD one
// contiguous range of work -- neighbouring cells / tiles of one image then share that XCD's L2
// instead of being fetched once per XCD.  Speed only: any placement stays correct.
__device__ inline int xcd_remap(int orig, int nwg) {
    const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// Per-level geometry, computed on the host (orb_runtime.cpp) from the reference formulas.
struct LevelGeom {
    int w, h, pitch;           // plane size; pitch in bytes (level 0: the input's row stride)
    long long img_stride;      // bytes between images for this level's plane
    int bpitch;                // blurred plane pitch (multiple of 64)
    long long bimg_stride;     // bytes between images for the blurred plane
    int nCols, nRows, wCell, hCell, maxBX, maxBY;  // cell grid (:787-805)
    int ncells, cell_cap;      // cells in this level, key capacity per cell
    int cell_first;            // flattened index of this level's first cell
    long long cellkey_off;     // offset (in keys) of this level's cell-key region in an image
    int cellcnt_off;           // offset (in cells) of this level's counts in an image
    int cand_cap;              // ncells * cell_cap
    int N;                     // mnFeaturesPerLevel[level]
    int W, H;                  // octree extents maxBorder - minBorder
    int kp_cap;                // octree output capacity
    int kp_off;                // offset (in keypoints) in an image's level-keypoint region
    int oct_cap;               // node capacity of the octree workspace
    long long oct_off;         // byte offset of this level's octree workspace in an image
    float scale;               // mvScaleFactor[level]
    int patch;                 // (int)(PATCH_SIZE * scale) (:882)
    int tiles_x, tiles_y, tile_first;  // blur tiling (128 x 32)
    int xtab_off, ytab_off, simd_end;  // resize tables (levels >= 1)
    int area2;                 // exact 2x downscale: OpenCV switches to INTER_AREA (2x2 mean)
    // k_blur_resize (levels >= 1): ownership of this level's output rows / column quads by the
    // 128 x 32 blur tiles of level l - 1 (int views of rtab): band_row[b] = first output row whose
    // first source row is >= 32 b (tiles_y(l-1) + 1 entries), tile_quad[j] = first quad whose first
    // source column is >= 128 j (tiles_x(l-1) + 1 entries)
    int band_row_off, tile_quad_off;
    int od_blocks, od_first;   // orientation/descriptor blocks for this level
    int tpitch;                // k_pyr_tail: LDS row pitch of this level (levels >= tail0 - 1)
};

struct BatchArgs {
    int nlevels, nimages;
    int img0;                        // first image of this launch (sub-batches on parallel streams)
    int ini_th, min_th;
    LevelGeom lv[kMaxLevels];
    uint8_t* lvl_base[kMaxLevels];   // plane base of image 0 (level 0 = the input buffer)
    uint8_t* blur_base[kMaxLevels];
    const int4* rtab;                // resize tables (x: {sx,sx1,a0,a1}, y: {sy0,sy1,b0,b1})
    uint32_t* cellkeys;              // [img][cand region]
    long long cellkeys_img_stride;   // keys
    int32_t* cellcnt;                // [img][cells]
    int cellcnt_img_stride;
    uint8_t* octws;                  // [img][octree workspace]
    long long octws_img_stride;
    uint32_t* lvlkey;                // [img][level kps] packed key
    float* lvlangle;                 // [img][level kps]
    uint8_t* lvldesc;                // [img][level kps][32]
    int lvlkp_img_stride;            // keypoints
    int32_t* lvlcnt;                 // [img][kMaxLevels]
    int32_t* status;                 // [img][kMaxLevels]
    void* out_kps;                   // orbgpu_keypoint [img][out_cap]
    uint8_t* out_desc;               // [img][out_cap][32]
    int out_cap;
    int32_t* out_n;                  // [img]
    int32_t* out_mono;               // [img]
    const int32_t* laps;             // [img][2]
    int total_cells, total_tiles, total_od_blocks;
    int fast_tab_off;  // rtab index of k_fast_cells' per-cell records (2 int4 per flattened cell)
    int od_tab_off;    // rtab index of k_orient_desc's per-block records {level, block, 0, 0}
    int fast_n48;  // k_fast_cells records [0, fast_n48) run the 48-byte FAST tile,
    int fast_n64;  // [fast_n48, fast_n64) the 64-byte one, the rest the 80-byte one (records are
                   // grouped by tile, levels in order inside each group)
    // k_fast_cells' small-list path (48- and 64-byte tiles): queued overflow cells [img][fast_qcap] as
    // (image, cell), counters [2 * img0] per launch (queued, finished overflow workgroups);
    // fast_small: -1 for launches of more than kFastMergeMaxImages images, 0 never, 1 always
    // (diagnostics); fast_ovf_all (diagnostics): every small-path cell goes to the overflow pass
    int2* fast_ovf;
    int* fast_ovf_cnt;
    int fast_qcap;  // queue entries per image: the 48- and 64-byte tiles' cells
    int fast_small, fast_ovf_all;
    unsigned long long* octdbg;      // diagnostic: [img][kMaxLevels][8] phase clocks, or null
    int oct_lds_nodes;               // node capacity of k_octree's dynamic LDS (0: all global)
    int oct_lds_bytes;
    int oct_nq_off;                  // byte offset of the per-key labels in that LDS
    // levels [oct_split, nlevels) run in a second k_octree launch of kOctSmallThreads-thread
    // workgroups with their own, smaller LDS layout (more workgroups per CU for the short levels)
    int oct_split;
    int oct_split_min_images;        // below this many images per launch: every level at 512 threads
    int oct2_threads;                // 128 or 256
    int oct2_lds_nodes, oct2_lds_bytes, oct2_nq_off, oct2_lds_keys;
    int oct_may_retry;               // some level can exceed the LDS instantiation of k_octree
    int oct_force_retry;             // diagnostics: every level through the generic instantiation
    int oct_pyr_max;                 // deepest count pyramid of k_octree (0: label passes only)
    // k_pyr_tail: levels [tail0, nlevels) and the blurs of [tail0 - 1, nlevels) in one launch
    // (tail0 = nlevels + 1: no tail, k_blur_resize for every level and k_blur for the last)
    int tail0;
    int tail_lds, tail_buf1, tail_tab, tail_maxq, tail_maxrows;  // its LDS layout (bytes / entries)
    int tail_min;              // launches of fewer images take the per-level path (host only)
    int fuse_out;              // no image of the batch has a lapping area: k_orient_desc writes the
                               // assembled outputs and counts, k_finalize does not run
};

struct MatchArgs {
    const uint8_t* desc;      // out_desc
    const int32_t* out_n;
    const int32_t* out_mono;
    int out_cap;
    int stereo_only;
    int32_t* idx1;
    int32_t* dist1;
    int32_t* idx2;
    int32_t* dist2;           // [pair][out_cap]
    int32_t* nq;              // [pair]
    int pair0;                // first pair of this launch
    uint2* part;              // [kKnnSplitSlots][out_cap] partial top-2 keys of split launches, or null
    uint32_t* cnt;            // split launches: per (pair, query block) arrival counters (zero between
                              // launches), so the last split workgroup merges; null: k_knn2_merge does
    int cnt_slots;            // counters allocated at cnt (launch_knn2_pairs checks the grid fits)
};
#ifndef KNN_SPLIT
// round 5, C4 step (one pair, tools/c4_time.py): 4 splits 126.6-126.9 us, 8 splits 125.2-125.5,
// 16 splits 126.6-126.9
#define KNN_SPLIT 8
#endif
constexpr int kKnnMaxSplit = KNN_SPLIT;     // train-row splits of a launch with few pairs
constexpr int kKnnSplitSlots = KNN_SPLIT;   // pairs x splits the partial buffer holds (1 pair: KNN_SPLIT splits)
// queries per k_knn2_mfma_pairs workgroup (orb_kernels.hip); the grid's x extent is
// ceil(out_cap / kKnnQueries) query blocks per pair
constexpr int kKnnQueries = 256;
// arrival counters of the fused split merge: one per (pair of the launch, query block); a split
// launch has at most kKnnSplitSlots / 2 pairs (orb_runtime.cpp), sized for kKnnSplitSlots
__host__ inline size_t knn2_counter_slots(int out_cap) {
    return (size_t)kKnnSplitSlots * (size_t)((out_cap + kKnnQueries - 1) / kKnnQueries);
}

// Frame::ComputeStereoMatches over a batch's device-resident results (orb_stereo.hip).
struct StereoArgs {
    const void* kps;                 // out_kps: orbgpu_keypoint [img][out_cap]
    const uint8_t* desc;             // out_desc: [img][out_cap][32]
    const int32_t* out_n;            // [img]
    int out_cap;
    int nlevels, H0;                 // levels, rows of level 0
    const uint8_t* lvl_base[kMaxLevels];  // unblurred pyramid (mvImagePyramid), image 0
    long long limg_stride[kMaxLevels];
    int lw[kMaxLevels], lh[kMaxLevels], lpitch[kMaxLevels];
    float scale[kMaxLevels], inv_scale[kMaxLevels];  // mvScaleFactors / mvInvScaleFactors
    float mbf, mb;                   // Frame::mbf, Frame::mb
    int32_t* row_start;              // [pair][H0 + 1] right keypoints by row (CSR)
    int32_t* row_idx;                // [pair][out_cap]
    float* u_right;                  // [pair][out_cap] mvuRight
    float* depth;                    // [pair][out_cap] mvDepth
    int32_t* sad;                    // [pair][out_cap] accepted SAD distance, -1 if none
    int pair0;                       // first pair of this launch
};

// Frame::ComputeStereoFishEyeMatches over a batch (orb_fisheye.hip): pair p = left image 2p,
// right image 2p+1, on the stereo-row kNN2 of orbgpu_match_stereo_batch(stereo_only = 1).
struct FisheyeArgs {
    const void* kps;                 // out_kps: orbgpu_keypoint [img][out_cap]
    const int32_t* out_n;            // [img]
    const int32_t* out_mono;         // [img]
    int out_cap;
    const int32_t* idx1;             // [pair][out_cap] kNN2 best train row (stereo rows)
    const int32_t* dist1;            // [pair][out_cap]
    float cam_l[8], cam_r[8];        // KannalaBrandt8 mvParameters: fx fy cx cy k0 k1 k2 k3
    float prec_l, prec_r;            // KannalaBrandt8::precision
    float R12[9], t12[3];            // Frame::mRlr (row-major), Frame::mtlr
    float sigma2[kMaxLevels];        // mvLevelSigma2
    int32_t* l2r;                    // [pair][out_cap] mvLeftToRightMatch
    int32_t* r2l;                    // [pair][out_cap] mvRightToLeftMatch (pre-set to -1)
    float* depth;                    // [pair][out_cap] mvDepth
    float* p3d;                      // [pair][out_cap][3] mvStereo3Dpoints
    int32_t* counts;                 // [pair][2] nMatches, descMatches (pre-set to 0)
    int pair0;                       // first pair of this launch
};
hipError_t launch_fisheye(const FisheyeArgs& f, int npairs, hipStream_t s);

// Frame::UndistortKeyPoints + AssignFeaturesToGrid over a batch's keypoints (orb_frame.hip).
constexpr int kGridCols = 64, kGridRows = 48;  // FRAME_GRID_COLS / ROWS (Frame.h:46-47)
struct GridArgs {
    const void* kps;       // out_kps: orbgpu_keypoint [img][out_cap]
    const int32_t* out_n;  // [img]
    int out_cap;
    int undistort;         // mDistCoef(0) != 0 (Frame.cc:765)
    float K[4];            // fx fy cx cy
    double k[14];          // OpenCV distortion vector (k1 k2 p1 p2 k3, rest 0)
    float bounds[4];       // mnMinX mnMaxX mnMinY mnMaxY
    float grid_inv[2];     // mfGridElementWidthInv / HeightInv
    float* xy_un;          // [img][out_cap][2] mvKeysUn positions
    int32_t* cell;         // [img][out_cap] posX * 48 + posY or -1
    int32_t* cell_start;   // [img][64 * 48 + 1]
    int32_t* cell_idx;     // [img][out_cap]
    int img0;
};

// Octree workspace layout for one (image, level) with n_cap keys and node capacity C.  The node
// state lives in LDS when C <= kOctLdsNodes, otherwise in the `nodemem` part of this block.
constexpr int kOctLdsNodes = 1024;
constexpr int kOdKpBlock = 8;  // keypoints per k_orient_desc pass (256 threads, 32 lanes per keypoint)
// keypoints per k_orient_desc workgroup by default: 3 passes of kOdKpBlock.  Round 5, chunked
// moments, single stream per 512 images: 1 pass 553 us, 2 passes 483, 3 passes 463, 4 passes 467;
// headline at 3 vs 2 passes +0.2 to +2.3% (bench A/B, 3 rounds).  Contexts of a few images take 1
// (orb_runtime.cpp set_geometry).
constexpr int kOdBlockKps = 3 * kOdKpBlock;

constexpr int kOctLdsKeys = 16384;  // per-key node labels (u16) kept in LDS up to this many keys
constexpr int kFastMergeMaxImages = 4;  // launches this small run the 48/64 FAST cells as one launch
// candidate list of the small-list k_fast_cells<48> / <64> (orb_kernels.hip), split over the waves
template <int CP>
constexpr int kFastSmallList() { return CP == 48 ? 512 : 1280; }
constexpr int kFastOvfBlocks = 32;      // workgroups of k_fast_cells_ovf
constexpr int kOctSmallThreads = 256;  // default workgroup size of the short-level k_octree launch
constexpr int kOctSmallMinImages = 32;  // launches with fewer images keep the 512-thread shape
// default dynamic LDS of that launch: a 640x480 level 0's node state (~38 KB) plus its depth-5
// count pyramid (10.9 KB) and path tables (2.1 KB); 3 workgroups per CU with the static part
constexpr int kOctSmallLds = 51 * 1024;

// LDS layout of one k_octree launch
struct OctCfg {
    int nq_off;     // byte offset of the per-key labels
    int lds_nodes;  // node capacity in LDS
    int lds_keys;   // labels kept in LDS up to this many keys (global workspace above)
    int lds_bytes;  // dynamic LDS of the launch (the count pyramid takes what the level leaves)
};

struct OctLayout {
    long long keys, nq, nodemem, total;
};

__host__ __device__ inline long long oct_align(long long x) { return (x + 255) & ~255LL; }

// Bytes of node state per node (orb_octree.h oct_nodemem_carve: cntA / cntB 16, nodesA / nodesB
// 16 each, divrank 4, childpos 8, five u16 arrays 10) -- the one figure both the LDS layouts and
// the workspace below size from; orb_octree.h asserts that the carve adds up to it.
constexpr int kOctNodeMemPerNode = 86;
__host__ __device__ constexpr size_t oct_nodemem_bytes(int C) { return (size_t)C * kOctNodeMemPerNode + 64; }

__host__ __device__ inline OctLayout oct_layout(int n_cap, int C) {
    OctLayout L;
    long long o = 0;
    L.keys = o; o = oct_align(o + 4LL * n_cap);
    L.nq = o; o = oct_align(o + 2LL * n_cap);  // used when n exceeds kOctLdsKeys
    L.nodemem = o;
    // used when C exceeds the LDS capacity (k_octree_retry).  Round 3 grew OctNode from 12 to 16
    // bytes while this reserved the old 78 B per node: levels with their node state here (above
    // ~1000 features per level, e.g. 1920x1080 with 8200 features) wrote 8 B per node into the
    // next level's keys, which that level's workgroup was using at the same time (round 6)
    o = oct_align(o + (long long)oct_nodemem_bytes(C));
    L.total = o;
    return L;
}

// Kernel launchers (orb_kernels.hip).  Each returns hipGetLastError() of its launch.
// k_blur / k_blur_resize tile: kBlurTW x kBlurTH outputs of the blur (kBlurTH a multiple of 16:
// 8 row groups of kBlurTH / 8 rows, an even count, in the vertical pass)
#ifndef BLUR_TH
#define BLUR_TH 32
#endif
constexpr int kBlurTW = 128, kBlurTH = BLUR_TH;
static_assert(kBlurTH % 16 == 0, "blur tile height");
constexpr int kBrMaxQuads = 40;  // k_blur_resize: level-l column quads / rows one blur tile owns
constexpr int kBrMaxRows = kBlurTH + 2;
// The blur of level l - 1 and the resize to level l in one launch (every level except the last
// blur, which launch_blur_level does).
hipError_t launch_blur_resize(const BatchArgs& a, int level, hipStream_t s);
hipError_t launch_blur_level(const BatchArgs& a, int level, hipStream_t s);
hipError_t launch_level_linear(const BatchArgs& a, int level, hipStream_t s);  // scale steps > 2
constexpr int kTailPad = 16;          // k_pyr_tail: left pad of an LDS row (>= 3 reflected columns)
constexpr int kTailLdsMax = 160 * 1024;  // the LDS one workgroup may hold on gfx950
constexpr int kTailMinImages = 128;     // k_pyr_tail only for launches of >= this many images
hipError_t launch_pyr_tail(const BatchArgs& a, hipStream_t s);
// FAST cells of the levels that run the `tile`-byte LDS tile (48, 64 or kCellMax = 80):
// fast_cell_range gives their flattened cell range, launch_fast_cells launches nothing if empty
void fast_cell_range(const BatchArgs& a, int tile, int* c0, int* c1);
hipError_t launch_fast_cells(const BatchArgs& a, int tile, hipStream_t s);
hipError_t launch_octree(const BatchArgs& a, hipStream_t s);
hipError_t launch_orient_desc(const BatchArgs& a, hipStream_t s);
hipError_t launch_finalize(const BatchArgs& a, hipStream_t s);
hipError_t launch_knn2_pairs(const MatchArgs& m, int npairs, hipStream_t s);
hipError_t launch_stereo(const StereoArgs& s, int npairs, hipStream_t st);  // orb_stereo.hip
hipError_t launch_undistort_grid(const GridArgs& g, int nimages, hipStream_t st);  // orb_frame.hip
void grid_dist_table(const float* dist, int ndist, double k[14]);
void image_bounds_host(int cols, int rows, const float K[4], const float* dist, int ndist, float bounds[4]);

// Wire formats (orb_io.hip): side-by-side Y8 ingest and the IDL SoA egress.
struct SbsArgs {
    const uint8_t* src;     // nframes frames of h rows x stride bytes, frame_bytes apart
    long long frame_bytes;
    int stride, w, h, nframes;  // w = one eye's width (the frame is 2w wide)
    uint8_t* dst;           // batch input: image 2f = left, 2f + 1 = right, [h][w] each
};
struct SoaArgs {
    const void* kps;        // out_kps [img][out_cap] (28 B)
    const int32_t* out_n;
    int out_cap, nimages, img0;
    int32_t *x, *y, *angle, *level;  // [img][out_cap]
    const int32_t *nq, *idx1, *dist1, *dist2;  // kNN results [pair][out_cap]
    int16_t *idx16, *d1_16, *d2_16;
};
// ORBmatcher::SearchByProjection over device-resident frames (orb_sbp.hip).
struct MapPointIn {  // orbgpu_map_point (72 B)
    float proj_x, proj_y, proj_xr, view_cos, depth;
    int32_t level, flags;
    uint8_t desc[32];
    float proj_yr, view_cos_r;  // right camera of a two-camera frame
    int32_t level_r;
};
constexpr int kMpInView = 1, kMpBad = 2, kMpHasObs = 4, kMpInViewR = 8;
struct SbpCand {  // k_sbp_candidates -> k_sbp_resolve: 4 lowest (distance, window position)
    int32_t idx[4];
    int32_t key[4];   // dist | octave << 16
    int32_t n;        // candidates after the filters; -1: map point skipped
    int32_t flags;    // the map point's flags (kMpHasObs decides whether its keypoint is taken)
    int32_t idxR[4];  // the same for the right-camera window (two-camera frames)
    int32_t keyR[4];
    int32_t nR;       // -1: no right-camera search
};
struct SbpArgs {
    const MapPointIn* mps;    // all frames' map points, frame f = [mp_off[f], mp_off[f + 1])
    const int32_t* mp_off;
    SbpCand* cand;            // [mp]
    const void* kps;          // out_kps
    const int32_t* out_n;
    int out_cap;
    const float* xy_un;       // grid buffers (orbgpu_undistort_grid_batch)
    const int32_t* cell_start;
    const int32_t* cell_idx;
    const uint8_t* desc;      // out_desc
    const float* uright;      // [frame][out_cap] mvuRight or nullptr (pinhole frames)
    const uint8_t* kp_block;  // [frame][2 * out_cap] pre-call occupant with observations, or nullptr
    const int32_t* l2r;       // [frame][out_cap] mvLeftToRightMatch (two-camera frames) or nullptr
    const int32_t* r2l;       // [frame][out_cap] mvRightToLeftMatch or nullptr
    int two_cam;              // Nleft != -1: frame f = images 2f (left) and 2f + 1 (right)
    int image_step, img0;     // frame f = batch image (img0 + f) * image_step; img0 = first frame
    float bounds[4], grid_inv[2];
    float scale[kMaxLevels];
    int nlevels;
    float th, nnratio, th_far;
    int far_points, factor;
    int32_t* match;           // [frame][2 * out_cap]: left keypoints, then right ones
    int32_t* nmatches;        // [frame]
};
size_t sbp_resolve_lds_bytes(int out_cap, int two_cam);
hipError_t launch_sbp(const SbpArgs& a, int nframes, int max_mps, hipStream_t st);

hipError_t launch_sbs_split(const SbsArgs& a, hipStream_t st);
hipError_t launch_pack_soa(const SoaArgs& a, int npairs, hipStream_t st);
// orbgpu_export_batch (orb_io.hip k_pack_export): the produced rows of a batch, packed
struct ExportArgs {
    const void* kps;          // out_kps [img][out_cap] (28 B)
    const uint8_t* desc;      // out_desc [img][out_cap][32]
    const int32_t* out_n;     // [img] (>= 0: the host checked)
    const int32_t* out_mono;  // [img]
    const int32_t* nq;        // [pair]
    const int32_t *idx1, *dist1, *idx2, *dist2;  // [pair][out_cap]
    int out_cap, nimages, npairs;
    void* dst;                // device buffer, 4-byte aligned
};
hipError_t launch_pack_export(const ExportArgs& a, hipStream_t st);
hipError_t launch_knn2_plain(const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* i1,
                             int32_t* d1, int32_t* i2, int32_t* d2, hipStream_t s);

}  // namespace orbgpu
