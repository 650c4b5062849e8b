// orb_runtime.cpp -- host runtime and C ABI (include/orbgpu.h) of liborbgpu.so.
//
// Owns one HIP stream and every device buffer of a context (allocated once per geometry,
// never inside a launch sequence), computes the per-level geometry and the OpenCV resize
// tables on the host with the reference's own float/double formulas, and enqueues the kernels
// of orb_kernels.hip.  There is no CPU compute path: every result comes from the device.
#include <hip/hip_runtime.h>
#include <link.h>

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/orbgpu.h"
#include "orb_fast_cell.h"
#include "orb_kernels.h"
#include "orb_octree.h"

using namespace orbgpu;

namespace {

thread_local std::string g_err;

constexpr size_t kGraphCacheSize = 4;  // captured batch sequences kept per context

// chunk streams a batch of n images is split over (whole stereo pairs per chunk)
inline int kChunksFor(int n) { return n >= 256 ? 2 : 3; }

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

// Measurement knobs (launch shapes, stream counts, kernel variants, phase clocks) are read only
// when ORBGPU_DIAGNOSTICS=1 is set as well: a stray ORBGPU_* variable in a deployment never
// changes the product's kernel path.  orbgpu_diagnostic_knobs reports the ones in effect.
const char* const kDiagKnobs[] = {"ORBGPU_OD_ITERS",      "ORBGPU_OCT_SMALL_LDS", "ORBGPU_OCT_SMALL_THREADS",
                                  "ORBGPU_OCT_SPLIT",     "ORBGPU_OCT_GENERIC",   "ORBGPU_OCT_PYR",
                                  "ORBGPU_FAST_PITCH",    "ORBGPU_STREAMS",       "ORBGPU_ISOLATE",
                                  "ORBGPU_STAGGER",       "ORBGPU_OCT_STAMPS",    "ORBGPU_GRAPH",
                                  "ORBGPU_KNN_NOSPLIT",   "ORBGPU_NO_TAIL",       "ORBGPU_TAIL_MIN",
                                  "ORBGPU_NO_FUSE_OUT",   "ORBGPU_FAST_SMALL",    "ORBGPU_FAST_OVF_ALL"};

bool diagnostics_on() {
    const char* g = getenv("ORBGPU_DIAGNOSTICS");
    return g && std::strcmp(g, "1") == 0;
}

const char* diag_env(const char* name) { return diagnostics_on() ? getenv(name) : nullptr; }

// torch bundles its own libamdhip64 (loaded by path, so a copy of the same soname from /opt/rocm
// that liborbgpu mapped first does not satisfy it): two HIP runtimes in one process then each own
// the device, and torch's sees none.  Entry points that start device work refuse that state with
// ORBGPU_ERR_RUNTIME instead of letting the other runtime fail silently later.  The object list
// is only rescanned when the process has loaded something since the last check (dlpi_adds).
int check_single_hip_runtime() {
    struct Scan { unsigned long long adds; std::vector<std::string> paths; };
    // shared by every context and thread (one per eye in the headset): the cached verdict and
    // its message are read and rescanned under one lock
    static std::mutex mu;
    static unsigned long long checked_adds = ~0ull;
    static int verdict = 0;
    static std::string msg;
    Scan sc{0, {}};
    dl_iterate_phdr([](dl_phdr_info* i, size_t, void* d) -> int {
        static_cast<Scan*>(d)->adds = i->dlpi_adds;
        return 1;  // the counter is the same in every entry: stop at the first
    }, &sc);
    std::lock_guard<std::mutex> lk(mu);
    if (sc.adds != checked_adds) {
        dl_iterate_phdr([](dl_phdr_info* i, size_t, void* d) -> int {
            const char* nm = i->dlpi_name;
            if (!nm || !*nm) return 0;
            const char* base = std::strrchr(nm, '/');
            base = base ? base + 1 : nm;
            if (std::strncmp(base, "libamdhip64.so", 14) == 0) static_cast<Scan*>(d)->paths.push_back(nm);
            return 0;
        }, &sc);
        checked_adds = sc.adds;
        verdict = sc.paths.size() > 1 ? ORBGPU_ERR_RUNTIME : 0;
        std::string paths;
        for (const auto& q : sc.paths) paths += (paths.empty() ? "" : ", ") + q;
        msg = "two HIP runtimes are mapped into this process (" + paths +
              "): import torch before loading liborbgpu.so, so that both bind to one runtime";
    }
    if (verdict) g_err = msg;  // every refusal, cached or fresh, on every thread
    return verdict;
}

#define HIP_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return fail(ORBGPU_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

enum Stage { ST_RESIZE, ST_BLUR, ST_FAST48, ST_FAST, ST_FAST_TOP, ST_OCTREE, ST_ORIENT, ST_FINAL, ST_KNN,
             ST_STEREO, ST_GRID, ST_SBS, ST_SOA, ST_SBP, ST_FISHEYE, ST_TAIL, ST_COUNT };
// names as rocprofv3 shows the kernels (templates with their argument)
const char* kStageNames[ST_COUNT] = {"k_blur_resize",    "k_blur",   "k_fast_cells<48>", "k_fast_cells<64>",
                                     "k_fast_cells<80>", "k_octree", "k_orient_desc",    "k_finalize",
                                     "k_knn2",           "k_stereo",  "k_undistort_grid",
                                     "k_sbs_split",      "k_pack_soa",       "k_sbp",
                                     "k_fisheye_stereo", "k_pyr_tail"};

// hipMalloc / hipFree on one thread while another thread captures a stream into a graph fails
// the allocation and invalidates the capture on this HIP (measured: two contexts run from two
// threads, test_two_threads_two_contexts_concurrently), whatever the capture mode.  Device
// allocations and graph captures of every context therefore take this one process-wide lock.
std::recursive_mutex& alloc_capture_mutex() {
    static std::recursive_mutex mu;  // recursive: context creation holds it around its allocations
    return mu;
}

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int ensure(size_t n) {
        if (n <= bytes) return 0;
        std::lock_guard<std::recursive_mutex> lk(alloc_capture_mutex());
        if (p) hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, n) != hipSuccess) return -1;
        bytes = n;
        return 0;
    }
    void release() {
        std::lock_guard<std::recursive_mutex> lk(alloc_capture_mutex());
        if (p) hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

inline int round_up(int x, int a) { return (x + a - 1) / a * a; }
inline long long round_up_ll(long long x, long long a) { return (x + a - 1) / a * a; }
inline int cv_round_f(float v) { return (int)std::lrintf(v); }
inline int cv_round_d(double v) { return (int)std::lrint(v); }
inline int cv_floor_f(float v) { return (int)std::floor(v); }
inline short sat_short(float v) {
    int i = cv_round_f(v);
    return (short)std::min(std::max(i, (int)SHRT_MIN), (int)SHRT_MAX);
}

struct Pending {
    int stage;
    hipEvent_t a, b;
};

// Device-to-host copy on the context's own stream, waited for before the call returns (the
// callers ran ctx_sync first, so the stream is idle and the copy sees every result).  Never a
// null-stream hipMemcpy: that would also order against other contexts' and torch's work.
#define D2H(dst, src, bytes)                                                               \
    do {                                                                                   \
        HIP_TRY(hipMemcpyAsync((dst), (src), (bytes), hipMemcpyDeviceToHost, c->stream));  \
        HIP_TRY(hipStreamSynchronize(c->stream));                                          \
    } while (0)

}  // namespace

struct orbgpu_ctx {
    orbgpu_params prm{};
    int device = 0;
    hipStream_t stream = nullptr;
    std::vector<hipStream_t> sub;  // sub-batch streams (sub[0] == stream)
    int max_w = 0, max_h = 0, max_images = 0;
    // ORBextractor tables (ORBextractor_old.cc:416-447)
    std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
    std::vector<int> nper;
    // geometry of the current image size
    int gw = -1, gh = -1;
    BatchArgs A{};
    std::vector<int4> rtab_host;
    long long pyr_img = 0, blur_img = 0, cellkeys_img = 0, octws_img = 0;
    int cellcnt_img = 0, lvlkp_img = 0, out_cap = 0;
    // device buffers
    DevBuf input, pyr, blur, rtab, cellkeys, cellcnt, octws, lvlkey, lvlangle, lvldesc, lvlcnt,
        status, outkps, outdesc, outn, outmono, laps, midx1, mdist1, midx2, mdist2, mnq, mpart, scratch,
        octdbg, fastovf, strow, stidx, stur, stdepth, stsad, gxy, gcell, gstart, gidx, sbs, soa, m16,
        sbpmp, sbpoff, sbpcand, sbpblk, sbpmatch, sbpnm, sbplr, fel2r, fer2l, fedepth, fep3d, fecnt;
    float grid_bounds[4] = {0, 0, 0, 0}, grid_inv[2] = {0, 0};  // of the last undistort_grid
    int sbp_frames = 0, sbp_step = 1, sbp_two_cam = 0;
    int soa_images = 0, soa_pairs = 0;  // coverage of the last orbgpu_pack_soa
    int grid_images = 0;   // images of the last orbgpu_undistort_grid_batch
    int stereo_pairs = 0;  // pairs of the last orbgpu_stereo_matches_batch
    int fisheye_pairs = 0;  // pairs of the last orbgpu_fisheye_stereo_batch
    int input_images = 0;   // images currently sized for in `input`
    hipEvent_t fork = nullptr;
    hipEvent_t ext_done = nullptr;  // work on a caller's stream (rejoin)
    // double-buffered input (orbgpu_upload_images_async): batch k reads slot in_slot while the copy
    // stream fills the other slot for batch k + 1; slot_free[j] = sub stream j's work enqueued before
    // the current batch began (everything that read the other slot), slot_ready = the async copy
    DevBuf input2;
    int in_slot = 0, pending_slot = -1;
    hipStream_t copy = nullptr;
    hipEvent_t slot_ready = nullptr;
    std::vector<hipEvent_t> slot_free;
    std::vector<hipEvent_t> join;  // one per sub stream
    // stages launched once over the whole batch on the main stream (join before, fork after), so
    // their per-launch duration is their own; off by default: each join / fork costs ~30 us of
    // idle GPU per step (ORBGPU_ISOLATE=<stage bit mask> turns it on)
    unsigned isolate_mask = 0;
    bool serialize = false;  // profiling: every stage isolated
    bool oct_stamps = false; // ORBGPU_OCT_STAMPS (read once at create): octree phase clocks
    // scale factors above 2: k_blur_resize's staged window does not hold a resize step's taps, so
    // the pyramid is k_level_linear per level, then k_blur per level (no k_pyr_tail)
    bool generic_pyr = false;
    // the captured launch sequences of one-stream batches (run_batch / run_batch_match), keyed by
    // {images, width, height, input slot, match pairs, stereo rows only}: one exec per key, so
    // alternating input slots (async uploads) or match variants replay instead of recapturing
    bool streams_forced = false;  // ORBGPU_STREAMS (diagnostics): every sub stream is a chunk
    bool use_graph = true;   // ORBGPU_GRAPH=0 launches every kernel directly (A/B)
    struct GraphRec { int key[7]; hipGraphExec_t exec; unsigned long long used; };
    std::vector<GraphRec> graphs;
    unsigned long long graph_tick = 0;
    bool knn_nosplit = false;  // ORBGPU_KNN_NOSPLIT (read once at create): no split kNN2 launches
    bool no_fuse_out = false;  // ORBGPU_NO_FUSE_OUT: k_finalize assembles even without lapping areas
    int fast_small = -1;       // ORBGPU_FAST_SMALL: the small-list FAST kernel never (0) / always (1)
    bool fast_ovf_all = false;  // ORBGPU_FAST_OVF_ALL: every small-list cell through the overflow pass
    bool last_fused = false;   // the last batch's outputs were assembled by k_orient_desc
    std::vector<int32_t> laps_host;  // lapping areas currently in `laps` (device), per image
    bool need_fork = true;           // the main stream holds work the sub streams must wait for
    bool stagger = true;             // ORBGPU_STAGGER=0: the chunks start every layout in lockstep
    bool restagger = false;          // the next batch re-staggers the chunks (after serialized runs)
    std::vector<hipEvent_t> stagger_ev;
    struct ChunkRec { int img0, n; hipStream_t st; };
    std::vector<ChunkRec> last_chunks;
    int last_images = 0, last_w = 0, last_h = 0, last_pairs = 0;
    // profiling: bit s of prof_mask brackets stage s launches with HIP events
    unsigned prof_mask = 0;
    std::vector<Pending> pending;
    std::vector<hipEvent_t> event_pool;
    double stage_ms[ST_COUNT] = {};
    long long stage_n[ST_COUNT] = {};
};

namespace {

void build_tables(orbgpu_ctx* c) {
    const int L = c->prm.nlevels;
    const double scaleFactor = (double)c->prm.scale_factor;  // double member (ORBextractor_old.h:98)
    c->scale.assign(L, 0.f);
    c->sigma2.assign(L, 0.f);
    c->inv_scale.assign(L, 0.f);
    c->inv_sigma2.assign(L, 0.f);
    c->scale[0] = 1.0f;
    c->sigma2[0] = 1.0f;
    for (int i = 1; i < L; i++) {
        c->scale[i] = (float)(c->scale[i - 1] * scaleFactor);
        c->sigma2[i] = c->scale[i] * c->scale[i];
    }
    for (int i = 0; i < L; i++) {
        c->inv_scale[i] = 1.0f / c->scale[i];
        c->inv_sigma2[i] = 1.0f / c->sigma2[i];
    }
    c->nper.assign(L, 0);
    const int nfeatures = c->prm.nfeatures;
    float factor = (float)(1.0f / scaleFactor);
    float nDesired = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)L));
    int sum = 0;
    for (int l = 0; l < L - 1; l++) {
        c->nper[l] = cv_round_f(nDesired);
        sum += c->nper[l];
        nDesired *= factor;
    }
    c->nper[L - 1] = std::max(nfeatures - sum, 0);
}

// OpenCV cv::resize INTER_LINEAR coefficient tables (resize.cpp, fixed point, ksize 2), host-side.
// Returns true when OpenCV would take the INTER_AREA 2x path instead.
bool resize_tables(int sw, int sh, int dw, int dh, std::vector<int4>& xt, std::vector<int4>& yt) {
    double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    int iscale_x = cv_round_d(scale_x), iscale_y = cv_round_d(scale_y);
    bool area_fast = std::abs(scale_x - iscale_x) < DBL_EPSILON &&
                     std::abs(scale_y - iscale_y) < DBL_EPSILON && iscale_x == 2 && iscale_y == 2;
    xt.resize(dw);
    yt.resize(dh);
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor_f(fx);
        fx -= sx;
        if (sx < 0) fx = 0, sx = 0;
        if (sx + 1 >= sw && sx >= sw - 1) fx = 0, sx = sw - 1;
        const short a0 = sat_short((1.f - fx) * 2048), a1 = sat_short(fx * 2048);
        xt[dx] = make_int4(sx, std::min(sx + 1, sw - 1), a0, a1);
    }
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor_f(fy);
        fy -= sy;
        const short b0 = sat_short((1.f - fy) * 2048), b1 = sat_short(fy * 2048);
        yt[dy] = make_int4(std::min(std::max(sy, 0), sh - 1), std::min(std::max(sy + 1, 0), sh - 1),
                           b0, b1);
    }
    return area_fast;
}

int simd_end(int width) {  // VResizeLinearVec_32s8u coverage (oracle pins the same rule)
    int x = 0;
    for (; x <= width - 16; x += 16) {}
    for (; x <= width - 8; x += 8) {}
    return x;
}

int alloc_all(orbgpu_ctx* c, int n_images) {
    const size_t ni = (size_t)std::max(n_images, 1);
    int r = 0;
    r |= c->pyr.ensure(ni * c->pyr_img + 256);
    r |= c->blur.ensure(ni * c->blur_img + 256);
    r |= c->rtab.ensure(sizeof(int4) * (c->rtab_host.size() + 1));
    r |= c->cellkeys.ensure(ni * c->cellkeys_img * 4 + 256);
    r |= c->cellcnt.ensure(ni * c->cellcnt_img * 4 + 256);
    r |= c->octws.ensure(ni * c->octws_img + 256);
    r |= c->lvlkey.ensure(ni * c->lvlkp_img * 4 + 256);
    r |= c->lvlangle.ensure(ni * c->lvlkp_img * 4 + 256);
    r |= c->lvldesc.ensure(ni * c->lvlkp_img * 32 + 256);
    r |= c->lvlcnt.ensure(ni * kMaxLevels * 4);
    r |= c->status.ensure(ni * kMaxLevels * 4);
    r |= c->outkps.ensure(ni * c->out_cap * sizeof(orbgpu_keypoint) + 256);
    r |= c->outdesc.ensure(ni * c->out_cap * 32 + 256);
    r |= c->outn.ensure(ni * 4);
    r |= c->outmono.ensure(ni * 4);
    r |= c->laps.ensure(ni * 8);
    const size_t np = (ni + 1) / 2;
    r |= c->midx1.ensure(np * c->out_cap * 4 + 256);
    r |= c->mdist1.ensure(np * c->out_cap * 4 + 256);
    r |= c->midx2.ensure(np * c->out_cap * 4 + 256);
    r |= c->mdist2.ensure(np * c->out_cap * 4 + 256);
    r |= c->mnq.ensure(np * 4 + 64);
    {  // FAST overflow queue [img][fast_qcap] (image, cell) and two counters per image slot (zeroed
       // once: k_fast_cells_ovf's last workgroup resets its launch's pair)
        void* before = c->fastovf.p;
        const size_t ent = ni * (size_t)std::max(c->A.fast_qcap, 1) * 8;
        r |= c->fastovf.ensure(ent + ni * 8 + 256);
        if (!r && c->fastovf.p != before && hipMemset(c->fastovf.p, 0, c->fastovf.bytes) != hipSuccess) r = -1;
    }
    {  // split kNN2 partials, then the arrival counters of the fused merge (zeroed once: the last
       // workgroup of each query block resets its counter)
        void* before = c->mpart.p;
        const size_t cnt_bytes = knn2_counter_slots(c->out_cap) * 4;
        r |= c->mpart.ensure((size_t)kKnnSplitSlots * c->out_cap * 8 + 256 + cnt_bytes);
        if (!r && c->mpart.p != before && hipMemset(c->mpart.p, 0, c->mpart.bytes) != hipSuccess) r = -1;
    }
    return r ? fail(ORBGPU_ERR_HIP, "hipMalloc failed (device memory)") : 0;
}

int ctx_sync(orbgpu_ctx* c, bool with_copy = false);

// Graph execs are launched on c->stream: the last launch of one may still run when it is
// destroyed, so the stream drains first.
void drop_graph(orbgpu_ctx* c) {
    if (c->graphs.empty()) return;
    hipStreamSynchronize(c->stream);
    for (auto& g : c->graphs) hipGraphExecDestroy(g.exec);
    c->graphs.clear();
}

// Level geometry for a w x h image (input row stride = w in the batch buffer).
int set_geometry(orbgpu_ctx* c, int w, int h) {
    if (c->gw == w && c->gh == h) return 0;
    if (c->gw >= 0)  // the tables and buffers below are still read by the last batch's kernels
        if (int e = ctx_sync(c, true)) return e;
    drop_graph(c);  // its launches carry the old geometry and buffers
    const int L = c->prm.nlevels;
    BatchArgs& A = c->A;
    A = BatchArgs{};
    A.nlevels = L;
    A.ini_th = c->prm.ini_th_fast;
    A.min_th = c->prm.min_th_fast;
    c->rtab_host.clear();
    long long pyr_off[kMaxLevels] = {}, blur_off[kMaxLevels] = {};
    long long pyr = 0, blr = 0, ck = 0, ows = 0;
    int cc = 0, kpo = 0, cell_first = 0, tile_first = 0, od_first = 0;
    // keypoints per k_orient_desc workgroup (orb_kernels.h kOdBlockKps; ORBGPU_OD_ITERS: passes of
    // kOdKpBlock instead, for A/B).  A context that never holds more than a few images (the
    // latency shape) takes one pass per workgroup: more, shorter workgroups for its few keypoints
    // (C4 step 124.3 us at one pass, 125.4 at two, 126.4 at three)
    const char* odi = diag_env("ORBGPU_OD_ITERS");
    const int od_per_block = odi ? kOdKpBlock * std::max(1, atoi(odi))
                                 : c->max_images <= kFastMergeMaxImages ? kOdKpBlock : kOdBlockKps;
    for (int l = 0; l < L; ++l) {
        LevelGeom& G = A.lv[l];
        G.w = cv_round_f((float)w * c->inv_scale[l]);   // ComputePyramid :1336
        G.h = cv_round_f((float)h * c->inv_scale[l]);
        if (G.w < 2 * kEdge + 4 || G.h < 2 * kEdge + 4)
            return fail(ORBGPU_ERR_INVALID, "pyramid level " + std::to_string(l) + " too small");
        G.bpitch = round_up(G.w, 64);
        if (l == 0) {
            G.pitch = w;
            G.img_stride = (long long)w * h;
        } else {
            G.pitch = G.bpitch;
            pyr_off[l] = pyr;
            pyr += round_up_ll((long long)G.pitch * G.h, 256);
        }
        blur_off[l] = blr;
        blr += round_up_ll((long long)G.bpitch * G.h, 256);
        // cell grid (ComputeKeyPointsOctTree :787-805)
        G.maxBX = G.w - kEdge + 3;
        G.maxBY = G.h - kEdge + 3;
        const float width = (float)(G.maxBX - kMinBorder), height = (float)(G.maxBY - kMinBorder);
        G.nCols = (int)(width / 35.f);
        G.nRows = (int)(height / 35.f);
        if (G.nCols < 1 || G.nRows < 1)
            return fail(ORBGPU_ERR_INVALID, "pyramid level " + std::to_string(l) + " has no cells");
        G.wCell = (int)std::ceil(width / G.nCols);
        G.hCell = (int)std::ceil(height / G.nRows);
        if (G.wCell > 69 || G.hCell > 69) return fail(ORBGPU_ERR_INVALID, "cell too large");
        G.ncells = G.nCols * G.nRows;
        // (a multiple of 4: k_octree reads a cell's keys as 16-byte chunks)
        G.cell_cap = (((G.wCell + 1) / 2) * ((G.hCell + 1) / 2) + 3) & ~3;
        G.cell_first = cell_first;
        cell_first += G.ncells;
        G.cellkey_off = ck;
        G.cand_cap = G.ncells * G.cell_cap;
        ck += round_up_ll(G.cand_cap, 64);
        G.cellcnt_off = cc;
        cc += round_up(G.ncells, 16);
        // octree
        G.N = c->nper[l];
        G.W = G.maxBX - kMinBorder;
        G.H = G.maxBY - kMinBorder;
        const int nIni = std::max(1, (int)std::round((float)G.W / (float)G.H));
        // live octree nodes never exceed max(N + 3, 4 * nIni) (orb_octree.h)
        G.oct_cap = std::max(G.N + 3, 4 * nIni) + 8;
        G.kp_cap = G.oct_cap;
        G.kp_off = kpo;
        kpo += round_up(G.kp_cap, 16);
        G.oct_off = ows;
        ows += oct_layout(G.cand_cap, G.oct_cap).total;
        G.scale = c->scale[l];
        G.patch = (int)(31 * c->scale[l]);
        G.tiles_x = (G.w + kBlurTW - 1) / kBlurTW;  // k_blur tile kBlurTW x kBlurTH
        G.tiles_y = (G.h + kBlurTH - 1) / kBlurTH;
        G.tile_first = tile_first;
        tile_first += G.tiles_x * G.tiles_y;
        G.od_blocks = std::max(1, (G.N + 16 + od_per_block - 1) / od_per_block);  // k_orient_desc blocks
        G.od_first = od_first;
        od_first += G.od_blocks;
        G.area2 = 0;
        if (l >= 1) {
            const LevelGeom& S = A.lv[l - 1];
            std::vector<int4> xt, yt;
            G.area2 = resize_tables(S.w, S.h, G.w, G.h, xt, yt) ? 1 : 0;
            G.xtab_off = (int)c->rtab_host.size();
            c->rtab_host.insert(c->rtab_host.end(), xt.begin(), xt.end());
            G.ytab_off = (int)c->rtab_host.size();
            c->rtab_host.insert(c->rtab_host.end(), yt.begin(), yt.end());
            G.simd_end = simd_end(G.w);
            // k_blur_resize ownership: output row dy / column quad q belongs to the blur tile of
            // level l - 1 holding its first source row / column (monotone in dy / q)
            auto push_ints = [&](const std::vector<int>& v) {
                const int off = 4 * (int)c->rtab_host.size();
                for (size_t i = 0; i < v.size(); i += 4)
                    c->rtab_host.push_back(make_int4(v[i], i + 1 < v.size() ? v[i + 1] : 0,
                                                     i + 2 < v.size() ? v[i + 2] : 0, i + 3 < v.size() ? v[i + 3] : 0));
                return off;
            };
            std::vector<int> band(S.tiles_y + 1), tq(S.tiles_x + 1);
            const int nquads = (G.w + 3) / 4;
            for (int b = 0, dy = 0; b <= S.tiles_y; ++b) {
                while (dy < G.h && (b == S.tiles_y || (G.area2 ? 2 * dy : yt[dy].x) < kBlurTH * b)) ++dy;
                band[b] = b == S.tiles_y ? G.h : dy;
            }
            for (int j = 0, q = 0; j <= S.tiles_x; ++j) {
                while (q < nquads && (j == S.tiles_x || (G.area2 ? 8 * q : xt[4 * q].x) < kBlurTW * j)) ++q;
                tq[j] = j == S.tiles_x ? nquads : q;
            }
            for (int b = 0; b < S.tiles_y; ++b)
                if (band[b + 1] - band[b] > kBrMaxRows) return fail(ORBGPU_ERR_INVALID, "resize band table");
            for (int j = 0; j < S.tiles_x; ++j)
                if (tq[j + 1] - tq[j] > kBrMaxQuads) return fail(ORBGPU_ERR_INVALID, "resize quad table");
            G.band_row_off = push_ints(band);
            G.tile_quad_off = push_ints(tq);
        }
    }
    // k_pyr_tail: the smallest t >= 2 such that level t - 1 and level t (and level t's resize
    // tables) fit one workgroup's LDS together; the tail then makes levels t .. L-1 and blurs
    // t - 1 .. L-1 (ORBGPU_NO_TAIL under diagnostics: per-level launches only).  Its pad columns
    // and row reflection take one REFLECT_101 step, exact for levels of >= 4 px: every level
    // passed the 2 * kEdge + 4 check above.
    for (int l = 0; l < L; ++l) A.lv[l].tpitch = round_up(A.lv[l].w + 28, 16);
    A.tail0 = L + 1;
    c->generic_pyr = c->prm.scale_factor > 2.0f;
    if (!diag_env("ORBGPU_NO_TAIL") && !c->generic_pyr)
        for (int t = 2; t <= L; ++t) {
            const LevelGeom& S0 = A.lv[t - 1];
            const long long b0 = round_up_ll((long long)S0.tpitch * S0.h, 16);
            const long long b1 = t < L ? round_up_ll((long long)A.lv[t].tpitch * A.lv[t].h, 16) : 0;
            const int maxq = t < L ? (A.lv[t].w + 3) / 4 : 0, maxrows = t < L ? A.lv[t].h : 0;
            const long long tab = (long long)maxq * (16 + 16 + 4) + (long long)maxrows * 16;
            if (b0 + b1 + tab + 16 <= kTailLdsMax && (S0.w + 3) / 4 <= 1024) {  // one resize quad per thread
                A.tail0 = t;
                A.tail_buf1 = (int)b0;
                A.tail_tab = (int)(b0 + b1);
                A.tail_maxq = maxq;
                A.tail_maxrows = maxrows;
                A.tail_lds = (int)round_up_ll(b0 + b1 + tab, 16);
                break;
            }
        }
    // the tail runs for launches of at least tail_min images (one 1024-thread workgroup per image
    // makes levels tail0 .. L-1 serially: 46 us for one pair, where the per-level launches take
    // ~20 us; with hundreds of images the tail's single pass wins)
    A.tail_min = kTailMinImages;
    if (const char* e = diag_env("ORBGPU_TAIL_MIN")) A.tail_min = std::max(0, atoi(e));
    c->pyr_img = round_up_ll(pyr, 256);
    c->blur_img = round_up_ll(blr, 256);
    c->cellkeys_img = ck;
    c->cellcnt_img = cc;
    c->octws_img = round_up_ll(ows, 256);
    c->lvlkp_img = kpo;
    c->out_cap = kpo;
    // k_octree dynamic LDS: the largest node capacity that fits kOctLdsNodes (levels above it
    // keep their node state in the global workspace) and room for the cell offsets.
    int lds_nodes = 0, max_cells = 0;
    for (int l = 0; l < L; ++l) {
        if (A.lv[l].oct_cap <= kOctLdsNodes) lds_nodes = std::max(lds_nodes, A.lv[l].oct_cap);
        max_cells = std::max(max_cells, A.lv[l].ncells);
    }
    A.oct_lds_nodes = lds_nodes;
    A.oct_nq_off = ((int)oct_nodemem_bytes(std::max(lds_nodes, 1)) + 15) & ~15;
    A.oct_lds_bytes = std::max(A.oct_nq_off + 2 * kOctLdsKeys, std::min(4 * max_cells, 65536));
    A.oct_lds_bytes = (A.oct_lds_bytes + 15) & ~15;
    // Levels [oct_split, L) run as a second k_octree launch of smaller workgroups (kOctSmallThreads)
    // with an LDS layout of kOctSmallLds: node state + cell offsets of those levels, then labels
    // for as many keys as fit (the global workspace above that).  More workgroups fit a CU, which
    // is what the node phases' serial latency needs.  oct_split = the first level from which on
    // the node state leaves room for >= 1024 labels (0 for 640x480-class pyramids: every level).
    {
        const char* eb = diag_env("ORBGPU_OCT_SMALL_LDS");
        const int budget = eb ? atoi(eb) : kOctSmallLds;
        const char* et = diag_env("ORBGPU_OCT_SMALL_THREADS");
        A.oct2_threads = et && atoi(et) == 128 ? 128 : kOctSmallThreads;
        auto layout = [&](int s0) {
            int n2 = 0, c2 = 0;
            for (int l = s0; l < L; ++l) {
                if (A.lv[l].oct_cap <= kOctLdsNodes) n2 = std::max(n2, A.lv[l].oct_cap);
                c2 = std::max(c2, A.lv[l].ncells);
            }
            A.oct2_lds_nodes = n2;
            A.oct2_nq_off = std::max(((int)oct_nodemem_bytes(std::max(n2, 1)) + 15) & ~15, (4 * c2 + 15) & ~15);
            A.oct2_lds_keys = std::max(0, (budget - A.oct2_nq_off) / 2);
            A.oct2_lds_bytes = (A.oct2_nq_off + 2 * A.oct2_lds_keys + 15) & ~15;
            return A.oct2_lds_keys >= 1024;
        };
        // Default: every level in the small shape when all of them fit it (640x480-class
        // pyramids), else every level in the 512-thread shape: a partial split runs the two
        // launches back to back and measured slower (C5: 90 vs 98 Mfeatures/s).  Launches of
        // fewer than kOctSmallMinImages images stay in the 512-thread shape too (latency, not
        // occupancy, bounds them: C4 0.31 vs 0.26 ms per pair).  ORBGPU_OCT_SPLIT forces a split.
        if (const char* e = diag_env("ORBGPU_OCT_SPLIT")) {
            A.oct_split = std::max(0, std::min(L, atoi(e)));
            if (A.oct_split < L && !layout(A.oct_split)) A.oct_split = L;
            A.oct_split_min_images = 0;
        } else {
            A.oct_split = layout(0) ? 0 : L;
            A.oct_split_min_images = kOctSmallMinImages;
        }
    }
    // a level misses k_octree (labels in LDS or in the workspace) only if its node capacity or
    // its cell offsets do not fit LDS; then k_octree_retry redoes it with generic pointers
    A.oct_may_retry = 0;
    for (int l = 0; l < L; ++l) {
        const LevelGeom& G = A.lv[l];
        if (G.oct_cap > lds_nodes || G.ncells > A.oct_nq_off / 4) A.oct_may_retry = 1;
        if (l >= A.oct_split && (G.oct_cap > A.oct2_lds_nodes || G.ncells > A.oct2_nq_off / 4)) A.oct_may_retry = 1;
    }
    A.oct_force_retry = diag_env("ORBGPU_OCT_GENERIC") ? 1 : 0;  // diagnostics / tests
    // ORBGPU_OCT_PYR=<d>: cap the count pyramid's depth (0: the label-pass formulation only)
    A.oct_pyr_max = kOctPyrMaxD;
    if (const char* e = diag_env("ORBGPU_OCT_PYR")) A.oct_pyr_max = std::max(0, std::min(kOctPyrMaxD, atoi(e)));
    if (A.oct_force_retry) A.oct_may_retry = 1;
    A.total_cells = cell_first;
    // FAST LDS tiles: each level takes the smallest tile its cell ROIs (+3 alignment bytes) fit:
    // 48 bytes, else 64, else 80.  Cells grow as the levels shrink (fewer, wider cells) but not
    // monotonically in both directions (640x480: level 6's cells are 51 rows tall, level 7's 42),
    // so the tiers are chosen per level.
    auto fits = [&](int l, int P) { return A.lv[l].wCell + 9 <= P && A.lv[l].hCell + 6 <= P; };
    int tier[kMaxLevels];
    int min_tier = 0;
    if (const char* fp = diag_env("ORBGPU_FAST_PITCH")) {  // diagnostics: force the larger tiles
        const int P = atoi(fp);
        min_tier = P == kCellMax ? 2 : P == kCellPitchSmall ? 1 : 0;
    }
    for (int l = 0; l < L; ++l) {
        const int t = fits(l, kCellPitchTiny) ? 0 : fits(l, kCellPitchSmall) ? 1 : 2;
        tier[l] = std::max(t, min_tier);
    }
    // k_fast_cells per-cell records, two int4 per cell: {level, iniX, iniY, rows | cols << 16} and
    // {cell-count index, cell-key index, skip, 0} (the cell loop's :807-821 geometry), grouped by
    // tier.  One scalar load replaces each workgroup's level search and cell-grid divisions.
    A.fast_tab_off = (int)c->rtab_host.size();
    int tier_end[3] = {0, 0, 0}, nrec = 0;
    for (int t = 0; t < 3; ++t) {
        for (int l = 0; l < L; ++l) {
            if (tier[l] != t) continue;
            const LevelGeom& G = A.lv[l];
            for (int cell = 0; cell < G.ncells; ++cell) {
                const int ci = cell / G.nCols, cj = cell % G.nCols;
                const int iniY = kMinBorder + ci * G.hCell, iniX = kMinBorder + cj * G.wCell;
                const int skip = (iniY >= G.maxBY - 3 || iniX >= G.maxBX - 6) ? 1 : 0;  // :812, :821
                const int rows = skip ? 0 : std::min(iniY + G.hCell + 6, G.maxBY) - iniY;
                const int cols = skip ? 0 : std::min(iniX + G.wCell + 6, G.maxBX) - iniX;
                c->rtab_host.push_back(make_int4(l, iniX, iniY, rows | (cols << 16)));
                c->rtab_host.push_back(make_int4(G.cellcnt_off + cell,
                                                 (int)(G.cellkey_off + (long long)cell * G.cell_cap), skip, 0));
                ++nrec;
            }
        }
        tier_end[t] = nrec;
    }
    A.fast_n48 = tier_end[0];
    A.fast_n64 = tier_end[1];
    A.fast_qcap = tier_end[1];  // the 48- and 64-byte tiles' cells share one queue per launch
    A.total_tiles = tile_first;
    A.total_od_blocks = od_first;
    A.od_tab_off = (int)c->rtab_host.size();
    for (int l = 0; l < L; ++l)
        for (int b = 0; b < A.lv[l].od_blocks; ++b) c->rtab_host.push_back(make_int4(l, b, 0, 0));
    for (int l = 0; l < L; ++l) {
        if (l > 0) A.lv[l].img_stride = c->pyr_img;
        A.lv[l].bimg_stride = c->blur_img;
    }
    int r = alloc_all(c, c->max_images);
    if (r) return r;
    HIP_TRY(hipMemcpyAsync(c->rtab.p, c->rtab_host.data(), sizeof(int4) * c->rtab_host.size(),
                           hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));  // pageable source
    c->need_fork = true;
    for (int l = 0; l < L; ++l) {
        A.lvl_base[l] = l == 0 ? nullptr : c->pyr.as<uint8_t>() + pyr_off[l];
        A.blur_base[l] = c->blur.as<uint8_t>() + blur_off[l];
    }
    A.rtab = c->rtab.as<int4>();
    A.cellkeys = c->cellkeys.as<uint32_t>();
    A.cellkeys_img_stride = c->cellkeys_img;
    A.cellcnt = c->cellcnt.as<int32_t>();
    A.cellcnt_img_stride = c->cellcnt_img;
    A.octws = c->octws.as<uint8_t>();
    A.octws_img_stride = c->octws_img;
    A.lvlkey = c->lvlkey.as<uint32_t>();
    A.lvlangle = c->lvlangle.as<float>();
    A.lvldesc = c->lvldesc.as<uint8_t>();
    A.lvlkp_img_stride = c->lvlkp_img;
    A.lvlcnt = c->lvlcnt.as<int32_t>();
    A.status = c->status.as<int32_t>();
    A.out_kps = c->outkps.p;
    A.out_desc = c->outdesc.as<uint8_t>();
    A.out_cap = c->out_cap;
    A.out_n = c->outn.as<int32_t>();
    A.out_mono = c->outmono.as<int32_t>();
    A.laps = c->laps.as<int32_t>();
    A.fast_ovf = c->fastovf.as<int2>();
    A.fast_ovf_cnt = reinterpret_cast<int*>(c->fastovf.as<uint8_t>() + (size_t)std::max(c->max_images, 1) *
                                                                           std::max(A.fast_qcap, 1) * 8);
    A.fast_small = c->fast_small;
    A.fast_ovf_all = c->fast_ovf_all ? 1 : 0;
    c->gw = w;
    c->gh = h;
    return 0;
}

hipEvent_t take_event(orbgpu_ctx* c) {
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
}

template <class F>
int timed(orbgpu_ctx* c, int stage, hipStream_t s, F&& launch) {
    hipEvent_t a = nullptr, b = nullptr;
    const bool prof = (c->prof_mask >> stage) & 1u;
    if (prof) {
        a = take_event(c);
        b = take_event(c);
        hipEventRecord(a, s);
    }
    hipError_t e = launch();
    if (e != hipSuccess)
        return fail(ORBGPU_ERR_HIP, std::string(kStageNames[stage]) + ": " + hipGetErrorString(e));
    if (prof) {
        hipEventRecord(b, s);
        c->pending.push_back({stage, a, b});
    }
    return 0;
}

// Makes stream s wait for everything already enqueued on the context's other streams.
int join_all(orbgpu_ctx* c, hipStream_t s) {
    for (size_t k = 0; k < c->sub.size() && k < c->join.size(); ++k) {
        if (c->sub[k] == s) continue;
        HIP_TRY(hipEventRecord(c->join[k], c->sub[k]));
        HIP_TRY(hipStreamWaitEvent(s, c->join[k], 0));
    }
    return 0;
}

// After work was enqueued on a caller's stream s (not one of the context's own): the context's
// streams wait for it before they touch the buffers again (the next batch overwrites what it reads).
int rejoin(orbgpu_ctx* c, hipStream_t s) {
    for (hipStream_t t : c->sub)
        if (t == s) return 0;
    HIP_TRY(hipEventRecord(c->ext_done, s));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ext_done, 0));
    c->need_fork = true;
    return 0;
}

// Waits for the work of this context's own streams (the chunk streams, and the copy stream when
// with_copy) -- never the whole device: two contexts driven from two threads (one extractor per
// eye, Frame.cc:142-145) or torch work beside them do not wait for each other.  Work enqueued on
// a caller's stream is covered through rejoin(), which every such entry point calls.
int ctx_sync(orbgpu_ctx* c, bool with_copy) {
    HIP_TRY(hipSetDevice(c->device));
    for (hipStream_t s : c->sub) HIP_TRY(hipStreamSynchronize(s));
    if (with_copy && c->copy) HIP_TRY(hipStreamSynchronize(c->copy));
    return 0;
}

// True when p points into device memory (hipMalloc / torch CUDA tensors): the device entry
// points refuse host pointers instead of faulting on them.  A failed query leaves a sticky
// error for hipGetLastError, which the launchers read: clear it.
bool device_ptr(const void* p) {
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged;
}

// A per-image count the device wrote: k_finalize stores -5 (octree workspace overflow) or -2
// (output capacity) instead of a count; map them to the status the caller gets.
int count_status(int32_t nk) {
    if (nk == -5) return fail(ORBGPU_ERR_OVERFLOW, "device workspace overflow (octree)");
    if (nk < 0) return fail(ORBGPU_ERR_CAPACITY, "context output capacity exceeded");
    return 0;
}

void resolve_pending(orbgpu_ctx* c) {
    for (auto& p : c->pending) {
        float ms = 0;
        if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            c->stage_ms[p.stage] += ms;
            c->stage_n[p.stage] += 1;
        }
        c->event_pool.push_back(p.a);
        c->event_pool.push_back(p.b);
    }
    c->pending.clear();
}

DevBuf& in_buf(orbgpu_ctx* c, int slot) { return slot ? c->input2 : c->input; }
uint8_t* cur_input(orbgpu_ctx* c) { return in_buf(c, c->in_slot).as<uint8_t>(); }

int ensure_input(orbgpu_ctx* c, int n_images, int w, int h, int slot = -1) {
    if (n_images < 1 || n_images > c->max_images)
        return fail(ORBGPU_ERR_CAPACITY, "n_images exceeds the context's max_images");
    if (w > c->max_w || h > c->max_h) return fail(ORBGPU_ERR_CAPACITY, "image larger than context max");
    if (in_buf(c, slot < 0 ? c->in_slot : slot).ensure((size_t)c->max_images * c->max_w * c->max_h + 256))
        return fail(ORBGPU_ERR_HIP, "hipMalloc failed (input)");
    return 0;
}

// Up to k chunk streams (never more than max_images / 2), each with its join event and, once the
// async upload exists, its slot_free event; created under the allocation / capture lock.  A new
// stream changes the chunk layout, so the batch that asked for it forks from the main stream.
int ensure_sub_streams(orbgpu_ctx* c, int k) {
    k = std::min(k, std::max(1, c->max_images / 2));
    if ((int)c->sub.size() >= k) return 0;
    std::lock_guard<std::recursive_mutex> lk(alloc_capture_mutex());
    HIP_TRY(hipSetDevice(c->device));
    while ((int)c->sub.size() < k) {
        hipStream_t st;
        hipEvent_t jn, fr = nullptr;
        HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        if (hipEventCreateWithFlags(&jn, hipEventDisableTiming) != hipSuccess ||
            (c->copy && hipEventCreateWithFlags(&fr, hipEventDisableTiming) != hipSuccess)) {
            hipStreamDestroy(st);
            return fail(ORBGPU_ERR_HIP, "hipEventCreate failed");
        }
        c->sub.push_back(st);
        c->join.push_back(jn);
        if (fr) c->slot_free.push_back(fr);
    }
    return 0;
}

// A synchronous upload / ingest replaces whatever an async upload staged for the next batch.
int drop_pending_upload(orbgpu_ctx* c) {
    if (c->pending_slot < 0) return 0;
    HIP_TRY(hipStreamSynchronize(c->copy));
    c->pending_slot = -1;
    return 0;
}

}  // namespace

// =============================================================================================
extern "C" {

const char* orbgpu_last_error(void) { return g_err.c_str(); }

int orbgpu_diagnostic_knobs(char* buf, size_t cap) {
    std::string out;
    int n = 0;
    for (const char* k : kDiagKnobs)
        if (const char* v = diag_env(k)) {
            out += (out.empty() ? "" : ";") + std::string(k) + "=" + v;
            ++n;
        }
    if (buf && cap) {
        const size_t m = std::min(cap - 1, out.size());
        std::memcpy(buf, out.data(), m);
        buf[m] = 0;
    }
    return n;
}
int orbgpu_abi_version(void) { return ORBGPU_ABI_VERSION; }
int orbgpu_num_stages(void) { return ST_COUNT; }
const char* orbgpu_stage_name(int s) { return (s >= 0 && s < ST_COUNT) ? kStageNames[s] : ""; }

int orbgpu_create(const orbgpu_params* p, int device, int max_width, int max_height,
                  int max_images, orbgpu_ctx** out) {
    if (!p || !out) return fail(ORBGPU_ERR_INVALID, "null argument");
    *out = nullptr;
    if (p->nlevels < 1 || p->nlevels > kMaxLevels || p->nfeatures < 0 || !(p->scale_factor > 1.0f) ||
        max_width <= 0 || max_height <= 0 || max_images <= 0 || max_width >= 4096 + 16 ||
        max_height >= 4096 + 16)
        return fail(ORBGPU_ERR_INVALID, "invalid ORB parameters or sizes");
    if (int e = check_single_hip_runtime()) return e;
    // streams, events and buffers are created under the allocation / capture lock (another
    // thread's context may be capturing a graph)
    std::lock_guard<std::recursive_mutex> create_lk(alloc_capture_mutex());
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(ORBGPU_ERR_NO_DEVICE, "no HIP device");
    if (device == ORBGPU_DEVICE_CURRENT && hipGetDevice(&device) != hipSuccess)
        return fail(ORBGPU_ERR_NO_DEVICE, "hipGetDevice failed");
    if (device < 0 || device >= ndev) return fail(ORBGPU_ERR_NO_DEVICE, "bad device ordinal");
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        return fail(ORBGPU_ERR_NO_DEVICE, std::string("device is not gfx950: ") + prop.gcnArchName);
    HIP_TRY(hipSetDevice(device));
    orbgpu_ctx* c = new orbgpu_ctx();
    c->prm = *p;
    c->device = device;
    c->max_w = max_width;
    c->max_h = max_height;
    c->max_images = max_images;
    build_tables(c);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return fail(ORBGPU_ERR_HIP, "hipStreamCreate failed");
    }
    c->sub.push_back(c->stream);
    {
        // 2 or 3 chunk streams (with the copy stream of orbgpu_upload_images_async, 3 or 4 of the 4
        // hardware queues a process gets, GPU_MAX_HW_QUEUES = 4; a 5th stream shares a queue and
        // the ingest copy then serialises with the kernels: 3.16 vs 1.75 ms per 128-pair step).
        // Round 4, C2 at 256 pairs: 2 streams 503-508 Mfeatures/s, 3 streams 485-492, 4 streams
        // 467-500, 1 stream 469 (tools/stagger_ab.sh); a token ring that lets one chunk at a time
        // run its pyramid + FAST while the others run octree / orientation / matching: 498 at 2
        // streams, 477-486 at 3 (the stages do not overlap better than side by side)
        // A context that can never hold more than one stereo pair (the single-pair / one-eye
        // extractor) gets one stream: chunks are whole pairs, and every stream takes one of the
        // process's hardware queues, which a second context (the other eye's thread) needs for its
        // own work not to queue behind this one's.
        const char* e = diag_env("ORBGPU_STREAMS");
        // the chunk streams the largest batch takes (kChunksFor); run_batch_impl adds the third
        // stream of a smaller batch when one first asks for it (ensure_sub_streams), so a context
        // sized for >= 256 images that never runs a small batch holds 2 streams, not an idle third
        c->streams_forced = e != nullptr;
        const int ns = std::max(1, std::min({8, e ? atoi(e) : kChunksFor(max_images), max_images / 2}));
        for (int k = 1; k < ns; ++k) {
            hipStream_t st;
            if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) break;
            c->sub.push_back(st);
        }
        bool ok = hipEventCreateWithFlags(&c->fork, hipEventDisableTiming) == hipSuccess &&
                  hipEventCreateWithFlags(&c->ext_done, hipEventDisableTiming) == hipSuccess;
        for (size_t k = 0; ok && k < c->sub.size(); ++k) {
            hipEvent_t ev;
            ok = hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess;
            if (ok) c->join.push_back(ev);
        }
        if (!ok) {
            orbgpu_destroy(c);
            return fail(ORBGPU_ERR_HIP, "hipEventCreate failed");
        }
        const char* iso = diag_env("ORBGPU_ISOLATE");  // stage bit mask (diagnostics)
        if (iso) c->isolate_mask = (unsigned)strtoul(iso, nullptr, 0);
        const char* sg = diag_env("ORBGPU_STAGGER");
        if (sg) c->stagger = atoi(sg) != 0;
        c->oct_stamps = diag_env("ORBGPU_OCT_STAMPS") != nullptr;
        if (const char* g = diag_env("ORBGPU_GRAPH")) c->use_graph = atoi(g) != 0;
        c->knn_nosplit = diag_env("ORBGPU_KNN_NOSPLIT") != nullptr;
        c->no_fuse_out = diag_env("ORBGPU_NO_FUSE_OUT") != nullptr;
        if (const char* f = diag_env("ORBGPU_FAST_SMALL")) c->fast_small = atoi(f) != 0 ? 1 : 0;
        c->fast_ovf_all = diag_env("ORBGPU_FAST_OVF_ALL") != nullptr;
    }
    int r = ensure_input(c, 1, max_width, max_height);
    if (!r) r = set_geometry(c, max_width, max_height);
    if (r) {
        orbgpu_destroy(c);
        return r;
    }
    *out = c;
    return ORBGPU_OK;
}

int orbgpu_get_device(const orbgpu_ctx* c) { return c ? c->device : fail(ORBGPU_ERR_INVALID, "null ctx"); }

int orbgpu_destroy(orbgpu_ctx* c) {
    if (!c) return ORBGPU_OK;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    resolve_pending(c);
    if (c->copy) hipStreamSynchronize(c->copy);
    std::lock_guard<std::recursive_mutex> destroy_lk(alloc_capture_mutex());  // frees and destroys
    for (auto e : c->event_pool) hipEventDestroy(e);
    DevBuf* bufs[] = {&c->input, &c->input2, &c->pyr,     &c->blur,   &c->rtab,    &c->cellkeys, &c->cellcnt,
                      &c->octws,   &c->lvlkey,  &c->lvlangle, &c->lvldesc, &c->lvlcnt, &c->status,
                      &c->outkps,  &c->outdesc, &c->outn,   &c->outmono, &c->laps,     &c->midx1,
                      &c->mdist1,  &c->midx2,   &c->mdist2, &c->mnq,     &c->mpart,   &c->scratch, &c->octdbg, &c->fastovf,
                      &c->strow,  &c->stidx, &c->stur,    &c->stdepth,  &c->stsad,
                      &c->gxy,     &c->gcell,  &c->gstart, &c->gidx,    &c->sbs,      &c->soa,
                      &c->m16,     &c->sbpmp,  &c->sbpoff, &c->sbpcand, &c->sbpblk,  &c->sbpmatch,
                      &c->sbpnm,   &c->sbplr,  &c->fel2r,  &c->fer2l,   &c->fedepth, &c->fep3d,
                      &c->fecnt};
    for (DevBuf* b : bufs) b->release();
    drop_graph(c);
    for (size_t k = 1; k < c->sub.size(); ++k) hipStreamDestroy(c->sub[k]);
    if (c->fork) hipEventDestroy(c->fork);
    if (c->ext_done) hipEventDestroy(c->ext_done);
    if (c->slot_ready) hipEventDestroy(c->slot_ready);
    for (auto e : c->slot_free) hipEventDestroy(e);
    if (c->copy) hipStreamDestroy(c->copy);
    for (hipEvent_t e : c->stagger_ev) hipEventDestroy(e);
    for (auto e : c->join) hipEventDestroy(e);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
    return ORBGPU_OK;
}

int orbgpu_get_scale_tables(const orbgpu_ctx* c, float* scale, float* inv_scale, float* sigma2,
                            float* inv_sigma2, int32_t* fpl) {
    if (!c) return fail(ORBGPU_ERR_INVALID, "null ctx");
    for (int l = 0; l < c->prm.nlevels; ++l) {
        if (scale) scale[l] = c->scale[l];
        if (inv_scale) inv_scale[l] = c->inv_scale[l];
        if (sigma2) sigma2[l] = c->sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = c->inv_sigma2[l];
        if (fpl) fpl[l] = c->nper[l];
    }
    return ORBGPU_OK;
}

uint8_t* orbgpu_device_input(orbgpu_ctx* c) { return c ? cur_input(c) : nullptr; }

int orbgpu_upload_images(orbgpu_ctx* c, const uint8_t* images, int n, int w, int h, int stride) {
    if (!c || !images) return fail(ORBGPU_ERR_INVALID, "null argument");
    if (w <= 0 || h <= 0) return fail(ORBGPU_ERR_EMPTY_IMAGE, "empty image");
    if (stride < w) return fail(ORBGPU_ERR_INVALID, "stride < width");
    int r = ensure_input(c, n, w, h);
    if (r) return r;
    HIP_TRY(hipSetDevice(c->device));
    if ((r = drop_pending_upload(c))) return r;
    r = join_all(c, c->stream);  // sub streams may still read the previous images
    if (r) return r;
    HIP_TRY(hipMemcpy2DAsync(cur_input(c), w, images, stride, w, (size_t)h * n, hipMemcpyHostToDevice,
                             c->stream));
    c->need_fork = true;
    return ORBGPU_OK;
}

int orbgpu_upload_images_async(orbgpu_ctx* c, const uint8_t* images, int n, int w, int h, int stride) {
    if (!c || !images) return fail(ORBGPU_ERR_INVALID, "null argument");
    if (w <= 0 || h <= 0) return fail(ORBGPU_ERR_EMPTY_IMAGE, "empty image");
    if (stride < w) return fail(ORBGPU_ERR_INVALID, "stride < width");
    if (c->pending_slot >= 0) return fail(ORBGPU_ERR_INVALID, "an async upload is already staged (run a batch first)");
    const int slot = 1 - c->in_slot;
    int r = ensure_input(c, n, w, h, slot);
    if (r) return r;
    HIP_TRY(hipSetDevice(c->device));
    if (!c->copy) {  // under the allocation / capture lock: another thread may be capturing a graph
        std::lock_guard<std::recursive_mutex> lk(alloc_capture_mutex());
        HIP_TRY(hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&c->slot_ready, hipEventDisableTiming));
        while (c->slot_free.size() < c->sub.size()) {
            hipEvent_t e;
            HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            c->slot_free.push_back(e);
        }
    }
    // the slot was last read by work enqueued before the current batch began (slot_free)
    for (size_t k = 0; k < c->slot_free.size(); ++k) HIP_TRY(hipStreamWaitEvent(c->copy, c->slot_free[k], 0));
    HIP_TRY(hipMemcpy2DAsync(in_buf(c, slot).p, w, images, stride, w, (size_t)h * n, hipMemcpyHostToDevice,
                             c->copy));
    HIP_TRY(hipEventRecord(c->slot_ready, c->copy));
    c->pending_slot = slot;
    return ORBGPU_OK;
}

int orbgpu_host_alloc(size_t bytes, void** ptr) {
    if (!ptr) return fail(ORBGPU_ERR_INVALID, "null argument");
    *ptr = nullptr;
    std::lock_guard<std::recursive_mutex> lk(alloc_capture_mutex());
    HIP_TRY(hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault));
    return ORBGPU_OK;
}

int orbgpu_host_free(void* ptr) {
    std::lock_guard<std::recursive_mutex> lk(alloc_capture_mutex());
    if (ptr) HIP_TRY(hipHostFree(ptr));
    return ORBGPU_OK;
}

// MatchArgs over the context's last batch: pair p = images 2p (query) and 2p + 1 (train)
static MatchArgs stereo_match_args(orbgpu_ctx* c, int stereo_only) {
    MatchArgs m;
    m.desc = c->outdesc.as<uint8_t>();
    m.out_n = c->outn.as<int32_t>();
    m.out_mono = c->outmono.as<int32_t>();
    m.out_cap = c->out_cap;
    m.stereo_only = stereo_only;
    m.idx1 = c->midx1.as<int32_t>();
    m.dist1 = c->mdist1.as<int32_t>();
    m.idx2 = c->midx2.as<int32_t>();
    m.dist2 = c->mdist2.as<int32_t>();
    m.nq = c->mnq.as<int32_t>();
    m.part = nullptr;
    m.cnt = reinterpret_cast<uint32_t*>(c->mpart.as<uint8_t>() + (size_t)kKnnSplitSlots * c->out_cap * 8 + 256);
    m.cnt_slots = (int)knn2_counter_slots(c->out_cap);
    m.pair0 = 0;
    return m;
}

// The batch's kernels; match_pairs > 0 appends the stereo kNN2 of pairs [0, match_pairs) when the
// batch runs as one captured graph (*matched = true: one submission for extraction and match).
static int run_batch_impl(orbgpu_ctx* c, int n, int w, int h, const int32_t* laps, void* stream,
                          int match_pairs, int stereo_only, bool* matched) {
    if (matched) *matched = false;
    if (!c) return fail(ORBGPU_ERR_INVALID, "null ctx");
    if (int e = check_single_hip_runtime()) return e;
    if (w <= 0 || h <= 0) return fail(ORBGPU_ERR_EMPTY_IMAGE, "empty image");
    int r = ensure_input(c, n, w, h);
    if (r) return r;
    HIP_TRY(hipSetDevice(c->device));
    r = set_geometry(c, w, h);
    if (r) return r;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    // the lapping areas change rarely (per camera): upload them only when they differ from the
    // copy already on the device, after every stream has finished reading the old one
    {
        std::vector<int32_t> want((size_t)n * 2, 0);
        if (laps) std::memcpy(want.data(), laps, (size_t)n * 8);
        if (want != c->laps_host) {
            r = join_all(c, s);
            if (r) return r;
            HIP_TRY(hipMemcpyAsync(c->laps.p, want.data(), (size_t)n * 8, hipMemcpyHostToDevice, s));
            HIP_TRY(hipStreamSynchronize(s));  // `want` is pageable host memory
            c->laps_host.swap(want);
            c->need_fork = true;
        }
    }
    BatchArgs A = c->A;
    A.nimages = n;
    A.img0 = 0;
    A.octdbg = nullptr;
    // no image with a lapping area a keypoint can fall in (every x is >= minBorderX = 16): every
    // keypoint is mono and k_orient_desc writes the assembled outputs itself (no k_finalize)
    A.fuse_out = 1;
    for (int i = 0; i < n; ++i) {
        const int l0 = c->laps_host[2 * i], l1 = c->laps_host[2 * i + 1];
        if (l1 >= kMinBorder && l0 <= l1) A.fuse_out = 0;
    }
    if (c->no_fuse_out) A.fuse_out = 0;
    c->last_fused = A.fuse_out != 0;  // orbgpu_get_level_keypoints reads the outputs then
    if (c->oct_stamps) {  // diagnostic build of the octree phase clocks
        const size_t bytes = (size_t)n * kMaxLevels * 8 * 8;
        if (!c->octdbg.ensure(bytes)) {
            hipMemsetAsync(c->octdbg.p, 0, bytes, s);
            A.octdbg = c->octdbg.as<unsigned long long>();
        }
    }
    // an async upload staged the next batch in the other input slot: read it once the copy lands
    // (each chunk stream waits on the copy alone, so the chunks keep their steady-state offsets);
    // first note what every stream has enqueued so far -- the readers of the slot we leave
    bool slot_switch = false;
    if (c->pending_slot >= 0) {
        c->in_slot = c->pending_slot;
        c->pending_slot = -1;
        slot_switch = true;
    }
    for (size_t k = 0; k < c->sub.size() && k < c->slot_free.size(); ++k)
        HIP_TRY(hipEventRecord(c->slot_free[k], c->sub[k]));
    A.lvl_base[0] = cur_input(c);
    A.lv[0].img_stride = (long long)w * h;
    // Sub-batches (whole stereo pairs) on parallel streams: the stages have complementary
    // bottlenecks (octree latency, FAST VALU, blur/resize HBM), so their phases overlap.
    struct Chunk { int img0, n; hipStream_t st; };
    std::vector<Chunk> chunks;
    // chunks per batch: batches of >= 128 pairs take 2 (each chunk fills the GPU); smaller ones
    // 3 (C5's 16 1080p pairs: 161 vs 154 Mfeatures/s); ORBGPU_STREAMS forces the stream count
    const int kmax = c->streams_forced ? (int)c->sub.size() : kChunksFor(n);
    if (!stream && (n % 2) == 0 && !c->streams_forced)
        if (int e_ = ensure_sub_streams(c, std::min(kmax, n / 2))) return e_;
    const int K = (!stream && (n % 2) == 0) ? std::min({(int)c->sub.size(), kmax, n / 2}) : 1;
    // a different sub-batch layout than last time may put an image on another stream: drain first
    if (!c->last_chunks.empty() && ((int)c->last_chunks.size() != K || c->last_images != n))
        if (int e_ = ctx_sync(c)) return e_;
    const bool relayout = c->last_chunks.empty() || (int)c->last_chunks.size() != K || c->last_images != n;
    if (K > 1) {
        // sub stream k > 0 waits for the main stream only when the main stream holds work it
        // depends on (a new layout, uploaded images, new lapping areas): in the steady state
        // every chunk's chain of steps stays on its own stream, so the streams keep the offset
        // they were given at the first step (stagger below) instead of restarting in lockstep
        const bool fork = relayout || c->need_fork;
        if (fork) HIP_TRY(hipEventRecord(c->fork, s));
        for (int k = 0; k < K; ++k) {
            const int p0 = (int)((long long)k * (n / 2) / K), p1 = (int)((long long)(k + 1) * (n / 2) / K);
            if (p1 > p0) {
                if (k > 0 && fork) HIP_TRY(hipStreamWaitEvent(c->sub[k], c->fork, 0));
                chunks.push_back({2 * p0, 2 * (p1 - p0), c->sub[k]});
            }
        }
        c->need_fork = false;
    } else {
        chunks.push_back({0, n, s});
    }
    if (slot_switch)
        for (const Chunk& ch : chunks) HIP_TRY(hipStreamWaitEvent(ch.st, c->slot_ready, 0));
    // first step of a layout: chunk k starts after chunk k-1 finished its pyramid + blur, so the
    // chunks run different stages (memory-, VALU- and latency-bound ones) at the same time
    // (also after serialized profiling runs, which leave every chunk stream joined: without a new
    // stagger the chunks would run each stage side by side from then on)
    const bool stagger = (relayout || c->restagger) && c->stagger && chunks.size() > 1 && !c->serialize;
    if (stagger) c->restagger = false;
    while (stagger && c->stagger_ev.size() < chunks.size()) {
        hipEvent_t ev;
        HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        c->stagger_ev.push_back(ev);
    }
    auto each = [&](int stage, auto launch) -> int {
        if (chunks.size() > 1 && (c->serialize || ((c->isolate_mask >> stage) & 1u))) {
            for (size_t k = 1; k < chunks.size(); ++k) {
                HIP_TRY(hipEventRecord(c->join[k], chunks[k].st));
                HIP_TRY(hipStreamWaitEvent(chunks[0].st, c->join[k], 0));
            }
            BatchArgs B = A;  // whole batch
            int rr = timed(c, stage, chunks[0].st, [&] { return launch(B, chunks[0].st); });
            if (rr) return rr;
            HIP_TRY(hipEventRecord(c->fork, chunks[0].st));
            for (size_t k = 1; k < chunks.size(); ++k) HIP_TRY(hipStreamWaitEvent(chunks[k].st, c->fork, 0));
            return 0;
        }
        for (const Chunk& ch : chunks) {
            BatchArgs B = A;
            B.img0 = ch.img0;
            B.nimages = ch.n;
            int rr = timed(c, stage, ch.st, [&] { return launch(B, ch.st); });
            if (rr) return rr;
        }
        return 0;
    };
    // the kernel sequence of this batch (every launch goes to the chunk streams)
    auto launch_all = [&]() -> int {
        int r = 0;
        // k_blur_resize makes levels 1 .. last_br - 1; k_pyr_tail the rest (or k_blur the last blur)
        int chunk_images = 0;
        for (const Chunk& ch : chunks) chunk_images = std::max(chunk_images, ch.n);
        if (c->serialize || chunks.size() == 1) chunk_images = n;
        const bool tail = A.tail0 <= A.nlevels && chunk_images >= A.tail_min;
        const int last_br = tail ? A.tail0 : A.nlevels;
        if (c->generic_pyr) {  // scale steps above 2: every level from HBM, then every blur
            for (int l = 1; l < A.nlevels; ++l) {
                r = each(ST_RESIZE, [&](const BatchArgs& B, hipStream_t st) { return launch_level_linear(B, l, st); });
                if (r) return r;
            }
            for (int l = 0; l < A.nlevels; ++l) {
                r = each(ST_BLUR, [&](const BatchArgs& B, hipStream_t st) { return launch_blur_level(B, l, st); });
                if (r) return r;
            }
        } else if (stagger) {
            // chunk-major: chunk k's first kernel waits for chunk k-1's pyramid + blur
            for (size_t k = 0; k < chunks.size(); ++k) {
                const Chunk& ch = chunks[k];
                BatchArgs B = A;
                B.img0 = ch.img0;
                B.nimages = ch.n;
                if (k > 0) HIP_TRY(hipStreamWaitEvent(ch.st, c->stagger_ev[k - 1], 0));
                for (int l = 1; l < last_br; ++l)
                    if ((r = timed(c, ST_RESIZE, ch.st, [&] { return launch_blur_resize(B, l, ch.st); }))) return r;
                if (tail) {
                    if ((r = timed(c, ST_TAIL, ch.st, [&] { return launch_pyr_tail(B, ch.st); }))) return r;
                } else {
                    const int lt = A.nlevels - 1;
                    if ((r = timed(c, ST_BLUR, ch.st, [&] { return launch_blur_level(B, lt, ch.st); }))) return r;
                }
                HIP_TRY(hipEventRecord(c->stagger_ev[k], ch.st));
            }
        } else {
            // level l - 1's blur and level l in one pass over level l - 1, then the last level's blur
            for (int l = 1; l < last_br; ++l) {
                r = each(ST_RESIZE, [&](const BatchArgs& B, hipStream_t st) { return launch_blur_resize(B, l, st); });
                if (r) return r;
            }
            if (tail) {
                if ((r = each(ST_TAIL, [](const BatchArgs& B, hipStream_t st) { return launch_pyr_tail(B, st); }))) return r;
            } else {
                const int lt = A.nlevels - 1;
                if ((r = each(ST_BLUR, [&](const BatchArgs& B, hipStream_t st) { return launch_blur_level(B, lt, st); }))) return r;
            }
        }
        {   // the FAST tiles as one group: one join / fork around all of them when isolated
            const int tiles[3] = {kCellPitchTiny, kCellPitchSmall, kCellMax};
            const int stages[3] = {ST_FAST48, ST_FAST, ST_FAST_TOP};
            bool any[3], iso = false;
            for (int t = 0; t < 3; ++t) {
                int c0, c1;
                fast_cell_range(A, tiles[t], &c0, &c1);
                any[t] = c1 > c0;
                iso = iso || (any[t] && chunks.size() > 1 && (c->serialize || ((c->isolate_mask >> stages[t]) & 1u)));
            }
            if (iso) {
                for (size_t k = 1; k < chunks.size(); ++k) {
                    HIP_TRY(hipEventRecord(c->join[k], chunks[k].st));
                    HIP_TRY(hipStreamWaitEvent(chunks[0].st, c->join[k], 0));
                }
            }
            for (int t = 0; t < 3; ++t) {
                if (!any[t]) continue;
                for (const Chunk& ch : chunks) {
                    BatchArgs B = A;
                    if (!iso) {
                        B.img0 = ch.img0;
                        B.nimages = ch.n;
                    }
                    const hipStream_t st = ch.st;
                    const int tile = tiles[t];
                    if ((r = timed(c, stages[t], st, [&] { return launch_fast_cells(B, tile, st); }))) return r;
                    if (iso) break;  // whole batch on the main stream
                }
            }
            if (iso) {
                HIP_TRY(hipEventRecord(c->fork, chunks[0].st));
                for (size_t k = 1; k < chunks.size(); ++k) HIP_TRY(hipStreamWaitEvent(chunks[k].st, c->fork, 0));
            }
        }
        if ((r = each(ST_OCTREE, [](const BatchArgs& B, hipStream_t st) { return launch_octree(B, st); }))) return r;
        if ((r = each(ST_ORIENT, [](const BatchArgs& B, hipStream_t st) { return launch_orient_desc(B, st); }))) return r;
        if (!A.fuse_out)
            if ((r = each(ST_FINAL, [](const BatchArgs& B, hipStream_t st) { return launch_finalize(B, st); }))) return r;
        return 0;
    };
    // One stream, no caller stream, no instrumentation (the single-pair / latency shape, e.g.
    // orbgpu_extract_stereo): the ~15 launches are captured once into a hipGraph and replayed
    // while the batch shape and input slot stay the same -- one submission instead of ~15.
    const bool graphable = chunks.size() == 1 && !stream && c->prof_mask == 0 && c->use_graph &&
                           !c->oct_stamps;
    const bool with_match = graphable && match_pairs > 0 && 2 * match_pairs <= n && c->out_cap <= 65535;
    auto launch_match = [&]() -> int {
        MatchArgs m = stereo_match_args(c, stereo_only);
        m.part = match_pairs * 2 <= kKnnSplitSlots && !c->knn_nosplit ? c->mpart.as<uint2>() : nullptr;
        HIP_TRY(launch_knn2_pairs(m, match_pairs, s));
        return 0;
    };
    if (graphable) {
        const int key[7] = {n, w, h, c->in_slot, with_match ? match_pairs : 0, with_match ? stereo_only : 0, A.fuse_out};
        orbgpu_ctx::GraphRec* rec = nullptr;
        for (auto& g : c->graphs)
            if (std::memcmp(key, g.key, sizeof key) == 0) rec = &g;
        if (!rec) {
            if (c->graphs.size() >= kGraphCacheSize) {  // evict the least recently launched exec
                size_t lru = 0;
                for (size_t k = 1; k < c->graphs.size(); ++k)
                    if (c->graphs[k].used < c->graphs[lru].used) lru = k;
                HIP_TRY(hipStreamSynchronize(c->stream));  // its last launch may still run
                hipGraphExecDestroy(c->graphs[lru].exec);
                c->graphs.erase(c->graphs.begin() + lru);
            }
            hipGraphExec_t ex = nullptr;
            hipError_t ei = hipSuccess;
            {
                std::lock_guard<std::recursive_mutex> lk(alloc_capture_mutex());  // no allocation mid-capture
                HIP_TRY(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
                int rr = launch_all();
                if (!rr && with_match) rr = launch_match();
                hipGraph_t g = nullptr;
                const hipError_t ec = hipStreamEndCapture(s, &g);
                if (rr || ec != hipSuccess) {
                    if (g) hipGraphDestroy(g);
                    return rr ? rr : fail(ORBGPU_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ec));
                }
                ei = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
                hipGraphDestroy(g);
            }
            if (ei != hipSuccess)
                return fail(ORBGPU_ERR_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ei));
            orbgpu_ctx::GraphRec nr{};
            std::memcpy(nr.key, key, sizeof key);
            nr.exec = ex;
            c->graphs.push_back(nr);
            rec = &c->graphs.back();
        }
        rec->used = ++c->graph_tick;
        HIP_TRY(hipGraphLaunch(rec->exec, s));
    } else if ((r = launch_all())) {
        return r;
    }
    c->last_chunks.clear();
    for (const Chunk& ch : chunks) c->last_chunks.push_back({ch.img0, ch.n, ch.st});
    c->last_images = n;
    c->last_w = w;
    c->last_h = h;
    if (with_match) {
        c->last_pairs = match_pairs;
        if (matched) *matched = true;
    }
    // a caller's stream: the context's streams wait for it before they touch this batch's
    // buffers again (the next async upload overwrites the input slot this batch read)
    if (stream && (r = rejoin(c, s))) return r;
    return ORBGPU_OK;
}

int orbgpu_run_batch(orbgpu_ctx* c, int n, int w, int h, const int32_t* laps, void* stream) {
    return run_batch_impl(c, n, w, h, laps, stream, 0, 0, nullptr);
}

int orbgpu_run_batch_match(orbgpu_ctx* c, int n, int w, int h, const int32_t* laps, int stereo_rows_only,
                           void* stream) {
    if (!c) return fail(ORBGPU_ERR_INVALID, "null ctx");
    if (n < 2 || (n % 2) != 0) return fail(ORBGPU_ERR_INVALID, "run_batch_match needs whole stereo pairs");
    bool matched = false;
    int r = run_batch_impl(c, n, w, h, laps, stream, n / 2, stereo_rows_only ? 1 : 0, &matched);
    if (r || matched) return r;
    return orbgpu_match_stereo_batch(c, n / 2, stereo_rows_only, stream);
}

int orbgpu_synchronize(orbgpu_ctx* c) {
    if (!c) return fail(ORBGPU_ERR_INVALID, "null ctx");
    if (int e_ = ctx_sync(c, true)) return e_;
    resolve_pending(c);
    if (c->oct_stamps && c->octdbg.p && c->last_images > 0) {
        const int n = c->last_images, L = c->prm.nlevels;
        std::vector<unsigned long long> d((size_t)n * kMaxLevels * 8);
        D2H(d.data(), c->octdbg.p, d.size() * 8);
        for (int l = 0; l < L; ++l) {
            double acc[8] = {};
            for (int i = 0; i < n; ++i)
                for (int k = 0; k < 8; ++k) acc[k] += (double)d[((size_t)i * kMaxLevels + l) * 8 + k];
            fprintf(stderr, "octree L%d us: init %.1f choose %.1f barrier %.1f sort %.1f rebuild %.1f relabel(pyramid: gather+histogram) %.1f best(pyramid: sums) %.1f rounds %.1f\n",
                    l, acc[0] / n / 100, acc[1] / n / 100, acc[2] / n / 100, acc[3] / n / 100,
                    acc[4] / n / 100, acc[5] / n / 100, acc[6] / n / 100, acc[7] / n);
        }
    }
    return ORBGPU_OK;
}

int orbgpu_download_counts(orbgpu_ctx* c, int n, int32_t* nk, int32_t* nm) {
    if (!c) return fail(ORBGPU_ERR_INVALID, "null ctx");
    if (n > c->last_images) return fail(ORBGPU_ERR_INVALID, "more images than the last batch");
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (int e_ = ctx_sync(c)) return e_;
    if (nk) D2H(nk, c->outn.p, (size_t)n * 4);
    if (nm) D2H(nm, c->outmono.p, (size_t)n * 4);
    return ORBGPU_OK;
}

int orbgpu_candidate_counts(orbgpu_ctx* c, int n, int32_t* counts) {
    if (!c || !counts) return fail(ORBGPU_ERR_INVALID, "null argument");
    if (n > c->last_images) return fail(ORBGPU_ERR_INVALID, "more images than the last batch");
    HIP_TRY(hipSetDevice(c->device));
    if (int e_ = ctx_sync(c)) return e_;
    std::vector<int32_t> cc((size_t)n * c->cellcnt_img);
    if (!cc.empty())
        D2H(cc.data(), c->cellcnt.p, cc.size() * 4);
    const BatchArgs& A = c->A;
    for (int i = 0; i < n; ++i) {
        long long s = 0;
        for (int l = 0; l < A.nlevels; ++l)
            for (int k = 0; k < A.lv[l].ncells; ++k) s += cc[(size_t)i * c->cellcnt_img + A.lv[l].cellcnt_off + k];
        counts[i] = (int32_t)s;
    }
    return ORBGPU_OK;
}

int orbgpu_download_result(orbgpu_ctx* c, int img, orbgpu_keypoint* kps, uint8_t* desc, int cap,
                           int* n, int* n_mono) {
    if (!c || img < 0 || img >= c->last_images) return fail(ORBGPU_ERR_INVALID, "bad image index");
    if (int e_ = ctx_sync(c)) return e_;
    int32_t nk = 0, nm = 0;
    D2H(&nk, c->outn.as<int32_t>() + img, 4);
    D2H(&nm, c->outmono.as<int32_t>() + img, 4);
    if (int e = count_status(nk)) return e;
    if (n) *n = nk;
    if (n_mono) *n_mono = nm;
    if (nk > cap) return fail(ORBGPU_ERR_CAPACITY, "caller capacity too small");
    if (kps && nk)
        D2H(kps, c->outkps.as<orbgpu_keypoint>() + (size_t)img * c->out_cap,
                          sizeof(orbgpu_keypoint) * nk);
    if (desc && nk)
        D2H(desc, c->outdesc.as<uint8_t>() + (size_t)img * c->out_cap * 32, 32 * (size_t)nk);
    return ORBGPU_OK;
}

int orbgpu_extract(orbgpu_ctx* c, const uint8_t* image, int w, int h, int stride, int lap0,
                   int lap1, orbgpu_keypoint* kps, uint8_t* desc, int cap, int* n, int* n_mono) {
    if (!c) return fail(ORBGPU_ERR_INVALID, "null ctx");
    if (!image || w <= 0 || h <= 0) return fail(ORBGPU_ERR_EMPTY_IMAGE, "empty image");  // :1092
    int r = orbgpu_upload_images(c, image, 1, w, h, stride);
    if (r) return r;
    int32_t laps[2] = {lap0, lap1};
    r = orbgpu_run_batch(c, 1, w, h, laps, nullptr);
    if (r) return r;
    return orbgpu_download_result(c, 0, kps, desc, cap, n, n_mono);
}

int orbgpu_extract_stereo(orbgpu_ctx* c, const uint8_t* left, const uint8_t* right, int w, int h,
                          int stride, const int lap_left[2], const int lap_right[2],
                          orbgpu_keypoint* kl, uint8_t* dl, int* nl, int* ml, orbgpu_keypoint* kr,
                          uint8_t* dr, int* nr, int* mr, int cap) {
    if (!c) return fail(ORBGPU_ERR_INVALID, "null ctx");
    if (!left || !right || w <= 0 || h <= 0) return fail(ORBGPU_ERR_EMPTY_IMAGE, "empty image");
    int r = ensure_input(c, 2, w, h);
    if (r) return r;
    if (stride < w) return fail(ORBGPU_ERR_INVALID, "stride < width");
    HIP_TRY(hipSetDevice(c->device));
    if ((r = drop_pending_upload(c))) return r;
    r = join_all(c, c->stream);  // sub streams of an earlier batch may still read the input
    if (r) return r;
    c->need_fork = true;
    HIP_TRY(hipMemcpy2DAsync(cur_input(c), w, left, stride, w, h, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpy2DAsync(cur_input(c) + (size_t)w * h, w, right, stride, w, h,
                             hipMemcpyHostToDevice, c->stream));
    int32_t laps[4] = {lap_left ? lap_left[0] : 0, lap_left ? lap_left[1] : 0,
                       lap_right ? lap_right[0] : 0, lap_right ? lap_right[1] : 0};
    r = orbgpu_run_batch(c, 2, w, h, laps, nullptr);
    if (r) return r;
    r = orbgpu_download_result(c, 0, kl, dl, cap, nl, ml);
    if (r) return r;
    return orbgpu_download_result(c, 1, kr, dr, cap, nr, mr);
}

int orbgpu_get_pyramid_level(orbgpu_ctx* c, int img, int level, int blurred, uint8_t* dst,
                             int dst_stride, int* width, int* height) {
    if (!c || img < 0 || img >= c->last_images || level < 0 || level >= c->prm.nlevels)
        return fail(ORBGPU_ERR_INVALID, "bad image/level");
    if (int e_ = ctx_sync(c)) return e_;
    const LevelGeom& G = c->A.lv[level];
    if (width) *width = G.w;
    if (height) *height = G.h;
    if (!dst) return ORBGPU_OK;
    if (dst_stride < G.w) return fail(ORBGPU_ERR_INVALID, "dst_stride < level width");
    const uint8_t* src;
    int pitch;
    if (blurred) {
        src = c->A.blur_base[level] + (size_t)img * c->blur_img;
        pitch = G.bpitch;
    } else if (level == 0) {
        src = cur_input(c) + (size_t)img * c->last_w * c->last_h;
        pitch = c->last_w;
    } else {
        src = c->A.lvl_base[level] + (size_t)img * c->pyr_img;
        pitch = G.pitch;
    }
    HIP_TRY(hipMemcpy2DAsync(dst, dst_stride, src, pitch, G.w, G.h, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return ORBGPU_OK;
}

int orbgpu_get_level_keypoints(orbgpu_ctx* c, int img, orbgpu_keypoint* kps, uint8_t* desc, int cap,
                               int32_t* counts) {
    if (!c || img < 0 || img >= c->last_images) return fail(ORBGPU_ERR_INVALID, "bad image index");
    if (int e_ = ctx_sync(c)) return e_;
    const int L = c->prm.nlevels;
    std::vector<int32_t> cnt(kMaxLevels), st(kMaxLevels);
    D2H(cnt.data(), c->lvlcnt.as<int32_t>() + img * kMaxLevels, 4 * kMaxLevels);
    D2H(st.data(), c->status.as<int32_t>() + img * kMaxLevels, 4 * kMaxLevels);
    int off = 0;
    for (int l = 0; l < L; ++l) {
        if (st[l]) return fail(ORBGPU_ERR_OVERFLOW, "octree status " + std::to_string(st[l]));
        const LevelGeom& G = c->A.lv[l];
        const int m = cnt[l];
        counts[l] = m;
        if (off + m > cap) return fail(ORBGPU_ERR_CAPACITY, "caller capacity too small");
        std::vector<uint32_t> keys(m);
        std::vector<float> ang(m);
        const size_t base = (size_t)img * c->lvlkp_img + G.kp_off;
        if (m) {
            D2H(keys.data(), c->lvlkey.as<uint32_t>() + base, 4 * m);
            if (c->last_fused) {  // k_orient_desc wrote the assembled rows (all mono, level order) only
                const size_t row = (size_t)img * c->out_cap + off;
                std::vector<orbgpu_keypoint> ok(m);
                D2H(ok.data(), c->outkps.as<orbgpu_keypoint>() + row, sizeof(orbgpu_keypoint) * m);
                for (int i = 0; i < m; ++i) ang[i] = ok[i].angle;
                if (desc) D2H(desc + 32 * (size_t)off, c->outdesc.as<uint8_t>() + row * 32, 32 * (size_t)m);
            } else {
                D2H(ang.data(), c->lvlangle.as<float>() + base, 4 * m);
                if (desc)
                    D2H(desc + 32 * (size_t)off, c->lvldesc.as<uint8_t>() + base * 32, 32 * (size_t)m);
            }
        }
        for (int i = 0; i < m; ++i) {
            orbgpu_keypoint& k = kps[off + i];
            k.x = (float)((keys[i] & 0xFFF) + kMinBorder);
            k.y = (float)(((keys[i] >> 12) & 0xFFF) + kMinBorder);
            k.size = (float)G.patch;
            k.angle = ang[i];
            k.response = (float)(keys[i] >> 24);
            k.octave = l;
            k.class_id = -1;
        }
        off += m;
    }
    return ORBGPU_OK;
}

int orbgpu_match_knn2(orbgpu_ctx* c, const uint8_t* q, int nq, const uint8_t* t, int nt,
                      int32_t* i1, int32_t* d1, int32_t* i2, int32_t* d2) {
    if (!c || nq < 0 || nt < 0 || (nq && !q) || (nt && !t)) return fail(ORBGPU_ERR_INVALID, "bad args");
    if (nt > 65535) return fail(ORBGPU_ERR_INVALID, "train set larger than 65535 rows");
    if (nq == 0) return ORBGPU_OK;
    HIP_TRY(hipSetDevice(c->device));
    const size_t need = 32 * (size_t)(nq + nt) + 16 * (size_t)nq + 1024;
    if (c->scratch.ensure(need)) return fail(ORBGPU_ERR_HIP, "hipMalloc failed (match scratch)");
    uint8_t* dq = c->scratch.as<uint8_t>();
    uint8_t* dt = dq + 32 * (size_t)nq;
    int32_t* o = reinterpret_cast<int32_t*>(dt + 32 * (size_t)nt + 256 - ((32 * (size_t)(nq + nt)) & 255));
    HIP_TRY(hipMemcpyAsync(dq, q, 32 * (size_t)nq, hipMemcpyHostToDevice, c->stream));
    if (nt) HIP_TRY(hipMemcpyAsync(dt, t, 32 * (size_t)nt, hipMemcpyHostToDevice, c->stream));
    int r = timed(c, ST_KNN, c->stream, [&] {
        return launch_knn2_plain(dq, nq, dt, nt, o, o + nq, o + 2 * nq, o + 3 * nq, c->stream);
    });
    if (r) return r;
    std::vector<int32_t> h(4 * (size_t)nq);
    HIP_TRY(hipMemcpyAsync(h.data(), o, 16 * (size_t)nq, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int i = 0; i < nq; ++i) {
        if (i1) i1[i] = h[i];
        if (d1) d1[i] = h[nq + i];
        if (i2) i2[i] = h[2 * nq + i];
        if (d2) d2[i] = h[3 * nq + i];
    }
    return ORBGPU_OK;
}

int orbgpu_export_descriptors(orbgpu_ctx* c, int img, int row0, uint8_t* dst, int cap, int* n_rows, void* stream) {
    if (!c || img < 0 || img >= c->last_images || row0 < 0 || (cap > 0 && !dst))
        return fail(ORBGPU_ERR_INVALID, "bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    if (cap > 0 && !device_ptr(dst)) return fail(ORBGPU_ERR_INVALID, "device_dst is not device memory");
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    int r = join_all(c, s);  // the descriptors come from the chunk streams
    if (r) return r;
    int32_t nk = 0;  // the count decides the copy size: read it once the batch is done
    HIP_TRY(hipMemcpyAsync(&nk, c->outn.as<int32_t>() + img, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (int e = count_status(nk)) return e;
    const int n = nk > row0 ? nk - row0 : 0;
    if (n_rows) *n_rows = n;
    if (n > cap) return fail(ORBGPU_ERR_CAPACITY, "caller capacity too small");
    if (n)
        HIP_TRY(hipMemcpyAsync(dst, c->outdesc.as<uint8_t>() + ((size_t)img * c->out_cap + row0) * 32, 32 * (size_t)n,
                               hipMemcpyDeviceToDevice, s));
    return rejoin(c, s);
}

int orbgpu_ingest_images(orbgpu_ctx* c, const uint8_t* device_images, int n, int w, int h, int stride,
                         void* stream) {
    if (!c || !device_images) return fail(ORBGPU_ERR_INVALID, "null argument");
    if (w <= 0 || h <= 0) return fail(ORBGPU_ERR_EMPTY_IMAGE, "empty image");
    if (stride < w) return fail(ORBGPU_ERR_INVALID, "stride < width");
    int r = ensure_input(c, n, w, h);
    if (r) return r;
    HIP_TRY(hipSetDevice(c->device));
    if (!device_ptr(device_images)) return fail(ORBGPU_ERR_INVALID, "device_images is not device memory");
    if ((r = drop_pending_upload(c))) return r;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    if ((r = join_all(c, s))) return r;  // the chunk streams may still read the previous images
    HIP_TRY(hipMemcpy2DAsync(cur_input(c), w, device_images, stride, w, (size_t)h * n, hipMemcpyDeviceToDevice, s));
    c->need_fork = true;
    return rejoin(c, s);
}

// the packed layout's largest size (every image at the context's row capacity): no device access
size_t orbgpu_export_batch_bytes(const orbgpu_ctx* c, int n_images, int n_pairs) {
    if (!c || n_images < 0 || n_pairs < 0) return 0;
    const size_t cap = (size_t)c->out_cap;
    return 8 * (size_t)n_images + 4 * (size_t)n_pairs + cap * (sizeof(orbgpu_keypoint) + 32) * (size_t)n_images +
           16 * cap * (size_t)n_pairs;
}

int orbgpu_export_batch(orbgpu_ctx* c, int n_images, int n_pairs, void* device_dst, size_t dst_bytes,
                        size_t* used, void* stream) {
    if (!c || n_images < 0 || n_images > c->last_images || n_pairs < 0 || n_pairs > c->last_pairs ||
        2 * n_pairs > n_images)
        return fail(ORBGPU_ERR_INVALID, "bad image / pair count");
    if (used) *used = 0;
    if (n_images == 0) return ORBGPU_OK;
    HIP_TRY(hipSetDevice(c->device));
    if (device_dst && !device_ptr(device_dst)) return fail(ORBGPU_ERR_INVALID, "device_dst is not device memory");
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    int r = join_all(c, s);  // the outputs come from the chunk streams
    if (r) return r;
    // the produced rows size the layout: read the counts once the batch (and its match) is done
    std::vector<int32_t> cnt((size_t)n_images + n_pairs);
    HIP_TRY(hipMemcpyAsync(cnt.data(), c->outn.p, 4 * (size_t)n_images, hipMemcpyDeviceToHost, s));
    if (n_pairs) HIP_TRY(hipMemcpyAsync(cnt.data() + n_images, c->mnq.p, 4 * (size_t)n_pairs, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    size_t need = 4 * (2 * (size_t)n_images + n_pairs);
    for (int i = 0; i < n_images; ++i) {
        if (int e = count_status(cnt[i])) return e;  // -5 / -2 status words are not row counts
        need += (sizeof(orbgpu_keypoint) + 32) * (size_t)cnt[i];
    }
    for (int p = 0; p < n_pairs; ++p) need += 16 * (size_t)std::max(cnt[n_images + p], 0);
    if (used) *used = need;
    if (!device_dst) return rejoin(c, s);  // size query
    if (dst_bytes < need) return fail(ORBGPU_ERR_CAPACITY, "export buffer too small");
    if (reinterpret_cast<uintptr_t>(device_dst) % 4) return fail(ORBGPU_ERR_INVALID, "device_dst not 4-byte aligned");
    ExportArgs x;
    x.kps = c->outkps.p;
    x.desc = c->outdesc.as<uint8_t>();
    x.out_n = c->outn.as<int32_t>();
    x.out_mono = c->outmono.as<int32_t>();
    x.nq = c->mnq.as<int32_t>();
    x.idx1 = c->midx1.as<int32_t>();
    x.dist1 = c->mdist1.as<int32_t>();
    x.idx2 = c->midx2.as<int32_t>();
    x.dist2 = c->mdist2.as<int32_t>();
    x.out_cap = c->out_cap;
    x.nimages = n_images;
    x.npairs = n_pairs;
    x.dst = device_dst;
    HIP_TRY(launch_pack_export(x, s));
    return rejoin(c, s);
}

int orbgpu_match_knn2_device(orbgpu_ctx* c, const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* i1,
                             int32_t* d1, int32_t* i2, int32_t* d2, void* stream) {
    if (!c || nq < 0 || nt < 0 || (nq && (!q || !i1 || !d1 || !i2 || !d2)) || (nt && !t))
        return fail(ORBGPU_ERR_INVALID, "bad args");
    if (nt > 65535) return fail(ORBGPU_ERR_INVALID, "train set larger than 65535 rows");
    if (nq == 0) return ORBGPU_OK;
    HIP_TRY(hipSetDevice(c->device));
    for (const void* p : {(const void*)q, (const void*)i1, (const void*)d1, (const void*)i2, (const void*)d2})
        if (!device_ptr(p)) return fail(ORBGPU_ERR_INVALID, "query / outputs must be device memory");
    if (nt && !device_ptr(t)) return fail(ORBGPU_ERR_INVALID, "train must be device memory");
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    int r = timed(c, ST_KNN, s, [&] { return launch_knn2_plain(q, nq, t, nt, i1, d1, i2, d2, s); });
    if (r) return r;
    return rejoin(c, s);
}

int orbgpu_match_stereo_batch(orbgpu_ctx* c, int n_pairs, int stereo_only, void* stream) {
    if (!c || n_pairs < 1 || 2 * n_pairs > c->last_images) return fail(ORBGPU_ERR_INVALID, "bad pair count");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    MatchArgs m = stereo_match_args(c, stereo_only);  // the split path (<= 4 pairs) sets m.part below
    uint2* split_part = n_pairs * 2 <= kKnnSplitSlots && !c->knn_nosplit ? c->mpart.as<uint2>() : nullptr;
    if (c->out_cap > 65535) return fail(ORBGPU_ERR_INVALID, "matcher supports < 65536 rows per image");
    // follow the extraction's sub-batches so each chunk matches right after it is extracted
    bool chunked = !stream && !c->last_chunks.empty();
    for (const auto& ch : c->last_chunks) chunked &= (ch.img0 % 2) == 0 && (ch.n % 2) == 0;
    if (chunked && c->last_chunks.size() > 1 &&
        (c->serialize || ((c->isolate_mask >> ST_KNN) & 1u))) {  // one launch over all pairs
        hipStream_t s0 = c->last_chunks[0].st;
        for (size_t k = 1; k < c->last_chunks.size(); ++k) {
            HIP_TRY(hipEventRecord(c->join[k], c->last_chunks[k].st));
            HIP_TRY(hipStreamWaitEvent(s0, c->join[k], 0));
        }
        m.pair0 = 0;
        m.part = split_part;
        int r = timed(c, ST_KNN, s0, [&] { return launch_knn2_pairs(m, n_pairs, s0); });
        if (r) return r;
        HIP_TRY(hipEventRecord(c->fork, s0));
        for (size_t k = 1; k < c->last_chunks.size(); ++k)
            HIP_TRY(hipStreamWaitEvent(c->last_chunks[k].st, c->fork, 0));
    } else if (chunked) {
        for (const auto& ch : c->last_chunks) {
            const int p0 = ch.img0 / 2, np = std::min(ch.n / 2, n_pairs - p0);
            if (np <= 0) continue;
            MatchArgs mm = m;
            mm.pair0 = p0;
            if (c->last_chunks.size() == 1) mm.part = split_part;  // one launch: the slots are its own
            int r = timed(c, ST_KNN, ch.st, [&] { return launch_knn2_pairs(mm, np, ch.st); });
            if (r) return r;
        }
    } else {
        m.pair0 = 0;
        m.part = split_part;
        int r = join_all(c, s);  // the extraction may have run on the chunk streams
        if (r) return r;
        r = timed(c, ST_KNN, s, [&] { return launch_knn2_pairs(m, n_pairs, s); });
        if (r) return r;
        if ((r = rejoin(c, s))) return r;
    }
    c->last_pairs = n_pairs;
    return ORBGPU_OK;
}

int orbgpu_download_matches(orbgpu_ctx* c, int pair, int32_t* i1, int32_t* d1, int32_t* i2,
                            int32_t* d2, int cap, int* nq) {
    if (!c || pair < 0 || pair >= c->last_pairs) return fail(ORBGPU_ERR_INVALID, "bad pair");
    if (int e_ = ctx_sync(c)) return e_;
    int32_t n = 0;
    D2H(&n, c->mnq.as<int32_t>() + pair, 4);
    if (nq) *nq = n;
    if (n > cap) return fail(ORBGPU_ERR_CAPACITY, "caller capacity too small");
    const size_t o = (size_t)pair * c->out_cap;
    if (n) {
        if (i1) D2H(i1, c->midx1.as<int32_t>() + o, 4 * (size_t)n);
        if (d1) D2H(d1, c->mdist1.as<int32_t>() + o, 4 * (size_t)n);
        if (i2) D2H(i2, c->midx2.as<int32_t>() + o, 4 * (size_t)n);
        if (d2) D2H(d2, c->mdist2.as<int32_t>() + o, 4 * (size_t)n);
    }
    return ORBGPU_OK;
}

int orbgpu_stereo_matches_batch(orbgpu_ctx* c, int n_pairs, float mbf, float mb, void* stream) {
    if (!c || n_pairs < 1 || 2 * n_pairs > c->last_images) return fail(ORBGPU_ERR_INVALID, "bad pair count");
    if (!(mb > 0.f) || !(mbf > 0.f)) return fail(ORBGPU_ERR_INVALID, "mbf and mb must be positive");
    HIP_TRY(hipSetDevice(c->device));
    const BatchArgs& A = c->A;
    const int H0 = A.lv[0].h;
    const size_t np = (size_t)n_pairs;
    if (c->strow.ensure(np * (H0 + 1) * 4 + 256) || c->stidx.ensure(np * c->out_cap * 4 + 256) ||
        c->stur.ensure(np * c->out_cap * 4 + 256) || c->stdepth.ensure(np * c->out_cap * 4 + 256) ||
        c->stsad.ensure(np * c->out_cap * 4 + 256))
        return fail(ORBGPU_ERR_HIP, "hipMalloc failed (stereo buffers)");
    StereoArgs S{};
    S.kps = c->outkps.p;
    S.desc = c->outdesc.as<uint8_t>();
    S.out_n = c->outn.as<int32_t>();
    S.out_cap = c->out_cap;
    S.nlevels = A.nlevels;
    S.H0 = H0;
    for (int l = 0; l < A.nlevels; ++l) {
        S.lvl_base[l] = l == 0 ? cur_input(c) : A.lvl_base[l];
        S.limg_stride[l] = l == 0 ? (long long)A.lv[0].w * A.lv[0].h : A.lv[l].img_stride;
        S.lw[l] = A.lv[l].w;
        S.lh[l] = A.lv[l].h;
        S.lpitch[l] = l == 0 ? A.lv[0].w : A.lv[l].pitch;
        S.scale[l] = c->scale[l];
        S.inv_scale[l] = c->inv_scale[l];
    }
    S.mbf = mbf;
    S.mb = mb;
    S.row_start = c->strow.as<int32_t>();
    S.row_idx = c->stidx.as<int32_t>();
    S.u_right = c->stur.as<float>();
    S.depth = c->stdepth.as<float>();
    S.sad = c->stsad.as<int32_t>();
    // follow the extraction's sub-batches (each chunk's pairs right after their extraction)
    bool chunked = !stream && !c->last_chunks.empty();
    for (const auto& ch : c->last_chunks) chunked &= (ch.img0 % 2) == 0 && (ch.n % 2) == 0;
    if (chunked) {
        for (const auto& ch : c->last_chunks) {
            const int p0 = ch.img0 / 2, npp = std::min(ch.n / 2, n_pairs - p0);
            if (npp <= 0) continue;
            StereoArgs SS = S;
            SS.pair0 = p0;
            int r = timed(c, ST_STEREO, ch.st, [&] { return launch_stereo(SS, npp, ch.st); });
            if (r) return r;
        }
    } else {
        hipStream_t s = stream ? (hipStream_t)stream : c->stream;
        S.pair0 = 0;
        int r = join_all(c, s);  // the extraction may have run on the chunk streams
        if (r) return r;
        r = timed(c, ST_STEREO, s, [&] { return launch_stereo(S, n_pairs, s); });
        if (r) return r;
        if ((r = rejoin(c, s))) return r;
    }
    c->stereo_pairs = n_pairs;
    return ORBGPU_OK;
}

int orbgpu_download_stereo(orbgpu_ctx* c, int pair, float* u_right, float* depth, int32_t* sad, int cap,
                           int* n) {
    if (!c || pair < 0 || pair >= c->stereo_pairs) return fail(ORBGPU_ERR_INVALID, "bad pair");
    HIP_TRY(hipSetDevice(c->device));
    if (int e_ = ctx_sync(c)) return e_;
    int32_t nl = 0;
    D2H(&nl, c->outn.as<int32_t>() + 2 * pair, 4);
    if (int e = count_status(nl)) return e;
    if (n) *n = nl;
    if (nl > cap) return fail(ORBGPU_ERR_CAPACITY, "caller capacity too small");
    const size_t o = (size_t)pair * c->out_cap;
    if (nl) {
        if (u_right) D2H(u_right, c->stur.as<float>() + o, 4 * (size_t)nl);
        if (depth) D2H(depth, c->stdepth.as<float>() + o, 4 * (size_t)nl);
        if (sad) D2H(sad, c->stsad.as<int32_t>() + o, 4 * (size_t)nl);
    }
    return ORBGPU_OK;
}

// ---- Frame::ComputeStereoFishEyeMatches (orb_fisheye.hip) -------------------------------------
int orbgpu_fisheye_stereo_batch(orbgpu_ctx* c, int n_pairs, const orbgpu_kb8_rig* rig, void* stream) {
    if (!c || !rig || n_pairs < 1 || 2 * n_pairs > c->last_images) return fail(ORBGPU_ERR_INVALID, "bad pair count");
    for (int k = 0; k < 2; ++k)
        if (!(rig->cam_left[k] != 0.f) || !(rig->cam_right[k] != 0.f))
            return fail(ORBGPU_ERR_INVALID, "zero focal length");
    // BFMatchORB of the stereo rows (Frame.cc:1164), then the triangulation on the same streams
    if (int r = orbgpu_match_stereo_batch(c, n_pairs, 1, stream)) return r;
    HIP_TRY(hipSetDevice(c->device));
    const size_t np = (size_t)n_pairs, oc = (size_t)c->out_cap;
    if (c->fel2r.ensure(np * oc * 4 + 256) || c->fer2l.ensure(np * oc * 4 + 256) ||
        c->fedepth.ensure(np * oc * 4 + 256) || c->fep3d.ensure(np * oc * 12 + 256) || c->fecnt.ensure(np * 8 + 256))
        return fail(ORBGPU_ERR_HIP, "hipMalloc failed (fisheye buffers)");
    FisheyeArgs F{};
    F.kps = c->outkps.p;
    F.out_n = c->outn.as<int32_t>();
    F.out_mono = c->outmono.as<int32_t>();
    F.out_cap = c->out_cap;
    F.idx1 = c->midx1.as<int32_t>();
    F.dist1 = c->mdist1.as<int32_t>();
    for (int k = 0; k < 8; ++k) {
        F.cam_l[k] = rig->cam_left[k];
        F.cam_r[k] = rig->cam_right[k];
    }
    F.prec_l = rig->precision_left;
    F.prec_r = rig->precision_right;
    for (int k = 0; k < 9; ++k) F.R12[k] = rig->R12[k];
    for (int k = 0; k < 3; ++k) F.t12[k] = rig->t12[k];
    for (int l = 0; l < kMaxLevels; ++l) F.sigma2[l] = l < c->A.nlevels ? c->sigma2[l] : 0.f;
    F.l2r = c->fel2r.as<int32_t>();
    F.r2l = c->fer2l.as<int32_t>();
    F.depth = c->fedepth.as<float>();
    F.p3d = c->fep3d.as<float>();
    F.counts = c->fecnt.as<int32_t>();
    auto run = [&](int p0, int npp, hipStream_t st) {
        HIP_TRY(hipMemsetAsync(F.r2l + (size_t)p0 * oc, 0xFF, (size_t)npp * oc * 4, st));  // -1
        HIP_TRY(hipMemsetAsync(F.counts + 2 * (size_t)p0, 0, (size_t)npp * 8, st));
        FisheyeArgs FF = F;
        FF.pair0 = p0;
        return timed(c, ST_FISHEYE, st, [&] { return launch_fisheye(FF, npp, st); });
    };
    bool chunked = !stream && !c->last_chunks.empty();
    for (const auto& ch : c->last_chunks) chunked &= (ch.img0 % 2) == 0 && (ch.n % 2) == 0;
    if (chunked) {
        for (const auto& ch : c->last_chunks) {
            const int p0 = ch.img0 / 2, npp = std::min(ch.n / 2, n_pairs - p0);
            if (npp <= 0) continue;
            if (int r = run(p0, npp, ch.st)) return r;
        }
    } else {
        hipStream_t s = stream ? (hipStream_t)stream : c->stream;
        int r = join_all(c, s);
        if (r) return r;
        if ((r = run(0, n_pairs, s))) return r;
        if ((r = rejoin(c, s))) return r;
    }
    c->fisheye_pairs = n_pairs;
    return ORBGPU_OK;
}

int orbgpu_download_fisheye(orbgpu_ctx* c, int pair, int32_t* l2r, int32_t* r2l, float* depth, float* p3d, int cap,
                            int* n_left, int* n_right, int* n_matches) {
    if (!c || pair < 0 || pair >= c->fisheye_pairs) return fail(ORBGPU_ERR_INVALID, "bad pair");
    HIP_TRY(hipSetDevice(c->device));
    if (int e_ = ctx_sync(c)) return e_;
    int32_t n[2] = {0, 0}, cnt[2] = {0, 0};
    D2H(n, c->outn.as<int32_t>() + 2 * pair, 8);
    D2H(cnt, c->fecnt.as<int32_t>() + 2 * pair, 8);
    if (int e = count_status(n[0])) return e;
    if (int e = count_status(n[1])) return e;
    if (n_left) *n_left = n[0];
    if (n_right) *n_right = n[1];
    if (n_matches) *n_matches = cnt[0];
    if (n[0] > cap || n[1] > cap) return fail(ORBGPU_ERR_CAPACITY, "caller capacity too small");
    const size_t o = (size_t)pair * c->out_cap;
    if (n[0]) {
        if (l2r) D2H(l2r, c->fel2r.as<int32_t>() + o, 4 * (size_t)n[0]);
        if (depth) D2H(depth, c->fedepth.as<float>() + o, 4 * (size_t)n[0]);
        if (p3d) D2H(p3d, c->fep3d.as<float>() + 3 * o, 12 * (size_t)n[0]);
    }
    if (n[1] && r2l) D2H(r2l, c->fer2l.as<int32_t>() + o, 4 * (size_t)n[1]);
    return ORBGPU_OK;
}

// ---- wire formats (orb_io.hip) ---------------------------------------------------------------
uint8_t* orbgpu_device_sbs_input(orbgpu_ctx* c) {
    if (!c) return nullptr;
    if (hipSetDevice(c->device) != hipSuccess) return nullptr;
    const size_t frames = (size_t)(c->max_images / 2 > 0 ? c->max_images / 2 : 1);
    if (c->sbs.ensure(frames * c->max_h * 2 * (size_t)c->max_w + 256)) {
        fail(ORBGPU_ERR_HIP, "hipMalloc failed (sbs staging)");
        return nullptr;
    }
    return c->sbs.as<uint8_t>();
}

static int check_sbs(orbgpu_ctx* c, int n, int w, int h, int stride) {
    if (w <= 0 || h <= 0) return fail(ORBGPU_ERR_EMPTY_IMAGE, "empty image");
    if (stride < 2 * w) return fail(ORBGPU_ERR_INVALID, "stride < 2 * width (side-by-side frame)");
    if (n < 1) return fail(ORBGPU_ERR_INVALID, "bad frame count");
    return ensure_input(c, 2 * n, w, h);
}

int orbgpu_ingest_sbs(orbgpu_ctx* c, const uint8_t* frames, int n, int w, int h, int stride, void* stream) {
    if (!c || !frames) return fail(ORBGPU_ERR_INVALID, "null argument");
    int r = check_sbs(c, n, w, h, stride);
    if (r) return r;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    if ((r = drop_pending_upload(c))) return r;
    r = join_all(c, s);  // sub streams may still read the previous images
    if (r) return r;
    SbsArgs a{frames, (long long)h * stride, stride, w, h, n, cur_input(c)};
    r = timed(c, ST_SBS, s, [&] { return launch_sbs_split(a, s); });
    if (r) return r;
    c->need_fork = true;
    // a caller's stream: the next batch (forked from the context's stream) waits for the split
    return rejoin(c, s);
}

int orbgpu_upload_sbs(orbgpu_ctx* c, const uint8_t* frames, int n, int w, int h, int stride) {
    if (!c || !frames) return fail(ORBGPU_ERR_INVALID, "null argument");
    int r = check_sbs(c, n, w, h, stride);
    if (r) return r;
    HIP_TRY(hipSetDevice(c->device));
    const size_t bytes = (size_t)n * h * stride;
    if (c->sbs.ensure(bytes + 256)) return fail(ORBGPU_ERR_HIP, "hipMalloc failed (sbs staging)");
    r = join_all(c, c->stream);
    if (r) return r;
    // 2W bytes of each of the n*h rows: never reads the padding after the last row's pixels
    HIP_TRY(hipMemcpy2DAsync(c->sbs.p, stride, frames, stride, 2 * (size_t)w, (size_t)n * h,
                             hipMemcpyHostToDevice, c->stream));
    return orbgpu_ingest_sbs(c, c->sbs.as<uint8_t>(), n, w, h, stride, nullptr);
}

int orbgpu_pack_soa(orbgpu_ctx* c, int n_images, int n_pairs, void* stream) {
    if (!c || n_images < 0 || n_images > c->last_images || n_pairs < 0 || n_pairs > c->last_pairs)
        return fail(ORBGPU_ERR_INVALID, "bad image/pair count");
    HIP_TRY(hipSetDevice(c->device));
    const size_t cap = (size_t)c->out_cap;
    if (c->soa.ensure((size_t)c->max_images * cap * 16 + 256) ||
        c->m16.ensure((size_t)(c->max_images / 2 + 1) * cap * 6 + 256))
        return fail(ORBGPU_ERR_HIP, "hipMalloc failed (soa buffers)");
    const size_t plane = (size_t)c->max_images * cap;
    const size_t mplane = (size_t)(c->max_images / 2 + 1) * cap;
    SoaArgs a{};
    a.kps = c->outkps.p;
    a.out_n = c->outn.as<int32_t>();
    a.out_cap = c->out_cap;
    a.nimages = n_images;
    a.img0 = 0;
    a.x = c->soa.as<int32_t>();
    a.y = a.x + plane;
    a.angle = a.y + plane;
    a.level = a.angle + plane;
    a.nq = c->mnq.as<int32_t>();
    a.idx1 = c->midx1.as<int32_t>();
    a.dist1 = c->mdist1.as<int32_t>();
    a.dist2 = c->mdist2.as<int32_t>();
    a.idx16 = c->m16.as<int16_t>();
    a.d1_16 = a.idx16 + mplane;
    a.d2_16 = a.d1_16 + mplane;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    int r = join_all(c, s);  // the chunk streams produced the keypoints and matches
    if (r) return r;
    r = timed(c, ST_SOA, s, [&] { return launch_pack_soa(a, n_pairs, s); });
    if (r) return r;
    c->soa_images = n_images;
    c->soa_pairs = n_pairs;
    c->need_fork = true;  // the next batch's chunk streams must not overwrite what this reads
    return ORBGPU_OK;
}

int orbgpu_download_soa(orbgpu_ctx* c, int image, int32_t* x, int32_t* y, int32_t* angle, int32_t* level,
                        uint8_t* orb, int cap, int* count, int* mono) {
    if (!c || image < 0 || image >= c->soa_images) return fail(ORBGPU_ERR_INVALID, "bad image");
    HIP_TRY(hipSetDevice(c->device));
    if (int e_ = ctx_sync(c)) return e_;
    int32_t nm[2] = {0, 0};
    D2H(&nm[0], c->outn.as<int32_t>() + image, 4);
    D2H(&nm[1], c->outmono.as<int32_t>() + image, 4);
    if (int e = count_status(nm[0])) return e;
    if (count) *count = nm[0];
    if (mono) *mono = nm[1];
    if (nm[0] > cap) return fail(ORBGPU_ERR_CAPACITY, "caller capacity too small");
    const size_t n = (size_t)nm[0];
    if (!n) return ORBGPU_OK;
    const size_t plane = (size_t)c->max_images * c->out_cap, o = (size_t)image * c->out_cap;
    int32_t* dst[4] = {x, y, angle, level};
    for (int k = 0; k < 4; ++k)
        if (dst[k]) D2H(dst[k], c->soa.as<int32_t>() + k * plane + o, 4 * n);
    if (orb) D2H(orb, c->outdesc.as<uint8_t>() + o * 32, 32 * n);
    return ORBGPU_OK;
}

int orbgpu_download_matches16(orbgpu_ctx* c, int pair, int16_t* indices, int16_t* dist1, int16_t* dist2,
                              int cap, int* nq) {
    if (!c || pair < 0 || pair >= c->soa_pairs) return fail(ORBGPU_ERR_INVALID, "bad pair");
    HIP_TRY(hipSetDevice(c->device));
    if (int e_ = ctx_sync(c)) return e_;
    int32_t n = 0;
    D2H(&n, c->mnq.as<int32_t>() + pair, 4);
    if (nq) *nq = n;
    if (n > cap) return fail(ORBGPU_ERR_CAPACITY, "caller capacity too small");
    if (!n) return ORBGPU_OK;
    const size_t mplane = (size_t)(c->max_images / 2 + 1) * c->out_cap, o = (size_t)pair * c->out_cap;
    int16_t* dst[3] = {indices, dist1, dist2};
    for (int k = 0; k < 3; ++k)
        if (dst[k]) D2H(dst[k], c->m16.as<int16_t>() + k * mplane + o, 2 * (size_t)n);
    return ORBGPU_OK;
}

int orbgpu_extract_features(orbgpu_ctx* c, const uint8_t* image, int image_len, int width, int height,
                            int stride, int threshold, int lap_l0, int lap_l1, int lap_r0, int lap_r1,
                            int* count_l, int32_t* x_l, int32_t* y_l, int32_t* angle_l, int32_t* level_l,
                            uint8_t* orb_l, int* count_r, int32_t* x_r, int32_t* y_r, int32_t* angle_r,
                            int32_t* level_r, uint8_t* orb_r, int kp_cap, int* mono_l, int* mono_r,
                            int16_t* indices, int16_t* dist1, int16_t* dist2, int match_cap) {
    (void)threshold;  // the DSP ignores it too (orbslam_dsp.cpp:1003-1087): the ctx's FAST thresholds apply
    if (!c || !image) return fail(ORBGPU_ERR_INVALID, "null argument");
    if ((long long)image_len < (long long)stride * (height - 1) + 2LL * width)
        return fail(ORBGPU_ERR_INVALID, "image_len smaller than the side-by-side frame");
    int r = orbgpu_upload_sbs(c, image, 1, width, height, stride);
    if (r) return r;
    const int32_t laps[4] = {lap_l0, lap_l1, lap_r0, lap_r1};
    r = orbgpu_run_batch(c, 2, width, height, laps, nullptr);
    if (!r) r = orbgpu_match_stereo_batch(c, 1, 1, nullptr);
    if (!r) r = orbgpu_pack_soa(c, 2, 1, nullptr);
    if (!r) r = orbgpu_download_soa(c, 0, x_l, y_l, angle_l, level_l, orb_l, kp_cap, count_l, mono_l);
    if (!r) r = orbgpu_download_soa(c, 1, x_r, y_r, angle_r, level_r, orb_r, kp_cap, count_r, mono_r);
    int nq = 0;
    if (!r) r = orbgpu_download_matches16(c, 0, indices, dist1, dist2, match_cap, &nq);
    return r;
}

namespace {

// Shared by the pinhole and two-camera entry points (orb_sbp.hip).
int sbp_run(orbgpu_ctx* c, int n_frames, int image_step, int two_cam, int use_uright,
            const orbgpu_map_point* mps, const int32_t* mp_offsets, const int32_t* l2r, const int32_t* r2l,
            int lr_stride, const uint8_t* kp_block, int kp_stride, float th, float nnratio, int far_points,
            float th_far, void* stream) {
    static_assert(sizeof(orbgpu_map_point) == sizeof(MapPointIn), "map point layout");
    if (!c || !mp_offsets || n_frames < 1) return fail(ORBGPU_ERR_INVALID, "null argument");
    const int images_needed = (n_frames - 1) * image_step + (two_cam ? 2 : 1);
    if (image_step < 1 || images_needed > c->grid_images)
        return fail(ORBGPU_ERR_INVALID, "frames must lie in the last orbgpu_undistort_grid_batch");
    if (use_uright && (image_step != 2 || n_frames > c->stereo_pairs))
        return fail(ORBGPU_ERR_INVALID, "mvuRight needs image_step 2 and a stereo_matches_batch over the pairs");
    if (sbp_resolve_lds_bytes(c->out_cap, two_cam) > 160 * 1024)
        return fail(ORBGPU_ERR_CAPACITY, "keypoint capacity above the matcher's LDS budget");
    if ((kp_block && kp_stride < 1) || ((l2r || r2l) && lr_stride < 1))
        return fail(ORBGPU_ERR_INVALID, "stride");
    const int total = mp_offsets[n_frames];
    int max_mps = 0;
    for (int f = 0; f < n_frames; ++f) {
        if (mp_offsets[f + 1] < mp_offsets[f] || mp_offsets[0] != 0) return fail(ORBGPU_ERR_INVALID, "mp_offsets");
        max_mps = std::max(max_mps, mp_offsets[f + 1] - mp_offsets[f]);
    }
    if (total > 0 && !mps) return fail(ORBGPU_ERR_INVALID, "null map points");
    HIP_TRY(hipSetDevice(c->device));
    const size_t cap = (size_t)c->out_cap, ncap = two_cam ? 2 * cap : cap;
    if (c->sbpmp.ensure((size_t)total * sizeof(MapPointIn) + 256) ||
        c->sbpoff.ensure((size_t)(n_frames + 1) * 4 + 256) ||
        c->sbpcand.ensure((size_t)total * sizeof(SbpCand) + 256) ||
        c->sbpmatch.ensure((size_t)n_frames * ncap * 4 + 256) || c->sbpnm.ensure((size_t)n_frames * 4 + 256) ||
        (kp_block && c->sbpblk.ensure((size_t)n_frames * ncap + 256)) ||
        ((l2r || r2l) && c->sbplr.ensure((size_t)n_frames * cap * 8 + 256)))
        return fail(ORBGPU_ERR_HIP, "hipMalloc failed (projection search)");
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    int r = join_all(c, s);  // keypoints, grid and mvuRight come from the chunk streams
    if (r) return r;
    // host inputs are pageable: copy, then wait so the caller may reuse them on return
    if (total) HIP_TRY(hipMemcpyAsync(c->sbpmp.p, mps, (size_t)total * sizeof(MapPointIn), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->sbpoff.p, mp_offsets, (size_t)(n_frames + 1) * 4, hipMemcpyHostToDevice, s));
    if (kp_block) {
        HIP_TRY(hipMemsetAsync(c->sbpblk.p, 0, (size_t)n_frames * ncap, s));
        HIP_TRY(hipMemcpy2DAsync(c->sbpblk.p, ncap, kp_block, kp_stride, std::min((size_t)kp_stride, ncap),
                                 n_frames, hipMemcpyHostToDevice, s));
    }
    int32_t* dl2r = c->sbplr.as<int32_t>();
    int32_t* dr2l = dl2r ? dl2r + (size_t)n_frames * cap : nullptr;
    const size_t lrw = std::min((size_t)lr_stride, cap) * 4;
    if (l2r) {
        HIP_TRY(hipMemsetAsync(dl2r, 0xFF, (size_t)n_frames * cap * 4, s));
        HIP_TRY(hipMemcpy2DAsync(dl2r, cap * 4, l2r, (size_t)lr_stride * 4, lrw, n_frames, hipMemcpyHostToDevice, s));
    }
    if (r2l) {
        HIP_TRY(hipMemsetAsync(dr2l, 0xFF, (size_t)n_frames * cap * 4, s));
        HIP_TRY(hipMemcpy2DAsync(dr2l, cap * 4, r2l, (size_t)lr_stride * 4, lrw, n_frames, hipMemcpyHostToDevice, s));
    }
    SbpArgs a{};
    a.mps = c->sbpmp.as<MapPointIn>();
    a.mp_off = c->sbpoff.as<int32_t>();
    a.cand = c->sbpcand.as<SbpCand>();
    a.kps = c->outkps.p;
    a.out_n = c->outn.as<int32_t>();
    a.out_cap = c->out_cap;
    a.xy_un = c->gxy.as<float>();
    a.cell_start = c->gstart.as<int32_t>();
    a.cell_idx = c->gidx.as<int32_t>();
    a.desc = c->outdesc.as<uint8_t>();
    a.uright = use_uright ? c->stur.as<float>() : nullptr;
    a.kp_block = kp_block ? c->sbpblk.as<uint8_t>() : nullptr;
    a.l2r = l2r ? dl2r : nullptr;
    a.r2l = r2l ? dr2l : nullptr;
    a.two_cam = two_cam;
    a.image_step = image_step;
    a.img0 = 0;
    std::memcpy(a.bounds, c->grid_bounds, sizeof a.bounds);
    std::memcpy(a.grid_inv, c->grid_inv, sizeof a.grid_inv);
    for (int l = 0; l < kMaxLevels; ++l) a.scale[l] = l < c->prm.nlevels ? c->scale[l] : 1.0f;
    a.nlevels = c->prm.nlevels;
    a.th = th;
    a.nnratio = nnratio;
    a.th_far = th_far;
    a.far_points = far_points != 0;
    a.factor = th != 1.0;  // bFactor (:48)
    a.match = c->sbpmatch.as<int32_t>();
    a.nmatches = c->sbpnm.as<int32_t>();
    r = timed(c, ST_SBP, s, [&] { return launch_sbp(a, n_frames, max_mps, s); });
    if (r) return r;
    HIP_TRY(hipStreamSynchronize(s));  // the pageable uploads above
    c->sbp_frames = n_frames;
    c->sbp_step = image_step;
    c->sbp_two_cam = two_cam;
    c->need_fork = true;
    return ORBGPU_OK;
}

}  // namespace

int orbgpu_search_by_projection_batch(orbgpu_ctx* c, int n_frames, int image_step, int use_uright,
                                      const orbgpu_map_point* mps, const int32_t* mp_offsets,
                                      const uint8_t* kp_block, int kp_stride, float th, float nnratio,
                                      int far_points, float th_far, void* stream) {
    return sbp_run(c, n_frames, image_step, 0, use_uright, mps, mp_offsets, nullptr, nullptr, 0, kp_block,
                   kp_stride, th, nnratio, far_points, th_far, stream);
}

int orbgpu_search_by_projection_stereo(orbgpu_ctx* c, int n_pairs, const orbgpu_map_point* mps,
                                       const int32_t* mp_offsets, const int32_t* left_to_right,
                                       const int32_t* right_to_left, int lr_stride, const uint8_t* kp_block,
                                       int kp_stride, float th, float nnratio, int far_points, float th_far,
                                       void* stream) {
    return sbp_run(c, n_pairs, 2, 1, 0, mps, mp_offsets, left_to_right, right_to_left, lr_stride, kp_block,
                   kp_stride, th, nnratio, far_points, th_far, stream);
}

int orbgpu_download_projection_matches(orbgpu_ctx* c, int frame, int32_t* match, int cap, int* n_kp,
                                       int* nmatches) {
    if (!c || frame < 0 || frame >= c->sbp_frames) return fail(ORBGPU_ERR_INVALID, "bad frame");
    HIP_TRY(hipSetDevice(c->device));
    if (int e_ = ctx_sync(c)) return e_;
    int32_t nk[2] = {0, 0}, nm = 0;
    const size_t img = (size_t)frame * c->sbp_step;
    D2H(nk, c->outn.as<int32_t>() + img, c->sbp_two_cam ? 8 : 4);
    D2H(&nm, c->sbpnm.as<int32_t>() + frame, 4);
    if (int e = count_status(nk[0])) return e;
    if (c->sbp_two_cam)
        if (int e = count_status(nk[1])) return e;
    if (!c->sbp_two_cam) nk[1] = 0;
    const int n = nk[0] + nk[1];
    if (n_kp) *n_kp = n;
    if (nmatches) *nmatches = nm;
    if (n > cap) return fail(ORBGPU_ERR_CAPACITY, "caller capacity too small");
    const size_t ncap = c->sbp_two_cam ? 2 * (size_t)c->out_cap : (size_t)c->out_cap;
    if (match && n)
        D2H(match, c->sbpmatch.as<int32_t>() + (size_t)frame * ncap, 4 * (size_t)n);
    return ORBGPU_OK;
}

int orbgpu_image_bounds(int cols, int rows, const float K[4], const float* dist, int ndist, float bounds[4]) {
    if (!K || !bounds || (ndist > 0 && !dist) || ndist < 0) return fail(ORBGPU_ERR_INVALID, "null argument");
    image_bounds_host(cols, rows, K, dist, ndist, bounds);
    return ORBGPU_OK;
}

int orbgpu_undistort_grid_batch(orbgpu_ctx* c, int n, const float K[4], const float* dist, int ndist,
                                void* stream) {
    if (!c || !K || (ndist > 0 && !dist) || ndist < 0) return fail(ORBGPU_ERR_INVALID, "null argument");
    if (n < 1 || n > c->last_images) return fail(ORBGPU_ERR_INVALID, "bad image count");
    if (!(K[0] != 0.f) || !(K[1] != 0.f)) return fail(ORBGPU_ERR_INVALID, "fx and fy must be nonzero");
    HIP_TRY(hipSetDevice(c->device));
    const size_t ni = (size_t)n, cap = (size_t)c->out_cap;
    if (c->gxy.ensure(ni * cap * 8 + 256) || c->gcell.ensure(ni * cap * 4 + 256) ||
        c->gstart.ensure(ni * (kGridCols * kGridRows + 1) * 4 + 256) || c->gidx.ensure(ni * cap * 4 + 256))
        return fail(ORBGPU_ERR_HIP, "hipMalloc failed (grid buffers)");
    GridArgs g{};
    g.kps = c->outkps.p;
    g.out_n = c->outn.as<int32_t>();
    g.out_cap = c->out_cap;
    g.undistort = ndist > 0 && dist[0] != 0.0f;
    for (int i = 0; i < 4; ++i) g.K[i] = K[i];
    grid_dist_table(dist, ndist, g.k);
    image_bounds_host(c->A.lv[0].w, c->A.lv[0].h, K, dist, ndist, g.bounds);
    g.grid_inv[0] = static_cast<float>(kGridCols) / (g.bounds[1] - g.bounds[0]);  // Frame.cc:107-108
    g.grid_inv[1] = static_cast<float>(kGridRows) / (g.bounds[3] - g.bounds[2]);
    g.xy_un = c->gxy.as<float>();
    g.cell = c->gcell.as<int32_t>();
    g.cell_start = c->gstart.as<int32_t>();
    g.cell_idx = c->gidx.as<int32_t>();
    bool chunked = !stream && !c->last_chunks.empty();
    if (chunked) {
        for (const auto& ch : c->last_chunks) {
            const int nn = std::min(ch.n, n - ch.img0);
            if (nn <= 0) continue;
            GridArgs gg = g;
            gg.img0 = ch.img0;
            int r = timed(c, ST_GRID, ch.st, [&] { return launch_undistort_grid(gg, nn, ch.st); });
            if (r) return r;
        }
    } else {
        hipStream_t s = stream ? (hipStream_t)stream : c->stream;
        g.img0 = 0;
        int r = join_all(c, s);  // the extraction may have run on the chunk streams
        if (r) return r;
        r = timed(c, ST_GRID, s, [&] { return launch_undistort_grid(g, n, s); });
        if (r) return r;
        if ((r = rejoin(c, s))) return r;
    }
    c->grid_images = n;
    std::memcpy(c->grid_bounds, g.bounds, sizeof g.bounds);
    std::memcpy(c->grid_inv, g.grid_inv, sizeof g.grid_inv);
    return ORBGPU_OK;
}

int orbgpu_download_grid(orbgpu_ctx* c, int image, float* xy_un, int32_t* cell, int32_t* cell_start,
                         int32_t* cell_idx, int cap, int* n) {
    if (!c || image < 0 || image >= c->grid_images) return fail(ORBGPU_ERR_INVALID, "bad image");
    HIP_TRY(hipSetDevice(c->device));
    if (int e_ = ctx_sync(c)) return e_;
    int32_t nk = 0;
    D2H(&nk, c->outn.as<int32_t>() + image, 4);
    nk = std::max(nk, 0);
    if (n) *n = nk;
    if (nk > cap) return fail(ORBGPU_ERR_CAPACITY, "caller capacity too small");
    const size_t o = (size_t)image * c->out_cap;
    const size_t G = kGridCols * kGridRows + 1;
    if (xy_un && nk) D2H(xy_un, c->gxy.as<float>() + 2 * o, 8 * (size_t)nk);
    if (cell && nk) D2H(cell, c->gcell.as<int32_t>() + o, 4 * (size_t)nk);
    if (cell_start) D2H(cell_start, c->gstart.as<int32_t>() + (size_t)image * G, 4 * G);
    if (cell_idx && nk) D2H(cell_idx, c->gidx.as<int32_t>() + o, 4 * (size_t)nk);
    return ORBGPU_OK;
}

int orbgpu_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    int dist = 0;
    for (int i = 0; i < 8; ++i) {
        uint32_t pa, pb;
        std::memcpy(&pa, a + 4 * i, 4);
        std::memcpy(&pb, b + 4 * i, 4);
        dist += __builtin_popcount(pa ^ pb);
    }
    return dist;
}

int orbgpu_set_profiling(orbgpu_ctx* c, int enable) {
    if (!c) return fail(ORBGPU_ERR_INVALID, "null ctx");
    // enable: 0 = off, 1 = every stage, otherwise (1u << 31) | [1u << 30] | stage mask: the
    // selected stages; bit 30 also runs every stage as one whole-batch launch (serial timing)
    const unsigned e = (unsigned)enable;
    c->prof_mask = e == 0 ? 0u : e == 1 ? 0xFFFFFFFFu : (e & 0x3FFFFFFFu);
    const bool was_serial = c->serialize;
    c->serialize = e != 0 && e != 1 && (e & (1u << 30));
    if (was_serial && !c->serialize) c->restagger = true;
    return ORBGPU_OK;
}

int orbgpu_stage_times(orbgpu_ctx* c, double* ms, int64_t* launches, int max_stages) {
    if (!c) return fail(ORBGPU_ERR_INVALID, "null ctx");
    resolve_pending(c);
    for (int s = 0; s < ST_COUNT && s < max_stages; ++s) {
        if (ms) ms[s] = c->stage_ms[s];
        if (launches) launches[s] = c->stage_n[s];
    }
    return ST_COUNT;
}

int orbgpu_reset_stage_times(orbgpu_ctx* c) {
    if (!c) return fail(ORBGPU_ERR_INVALID, "null ctx");
    resolve_pending(c);
    for (int s = 0; s < ST_COUNT; ++s) c->stage_ms[s] = 0, c->stage_n[s] = 0;
    return ORBGPU_OK;
}

}  // extern "C"
