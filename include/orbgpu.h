/* orbgpu.h -- C ABI of the MI355X ORB front-end (liborbgpu.so).
 *
 * Plain C: pointers, sizes, int status codes, no torch / OpenCV / HIP types in signatures
 * (streams travel as void*).  One context per stream/thread; no globals.
 *
 * Each entry point names the reference interface it replaces (paths relative to the
 * Lynx-MR/orbslam3lib root, cpp/ = app/src/main/cpp/):
 *   - ORBextractor ctor + operator()      cpp/include/ORBextractor_old.h:51-59,
 *                                         cpp/src/ORBextractor_old.cc:411-471, 1088-1191
 *   - stereo operator()(AHardwareBuffer*) cpp/include/ORBextractor.h:52-57 /
 *                                         cpp/src/ORBextractor.cc:118-165
 *   - FastRPC extractFeatures/bfMatchStereo  cpp/inc/orbslam3.idl:15-21 (impl
 *                                         dsp/src/orbslam_dsp.cpp:866-1087)
 *   - LynxHardwareAccelerator::{ctor,ExtractORB,BFMatchORB,dtor}
 *                                         cpp/include/LynxHardwareAcceleration/
 *                                         LynxHardwareAccelerator.h:45-51
 *   - ORBmatcher::DescriptorDistance      cpp/include/ORBmatcher.h:44, cpp/src/ORBmatcher.cc:2107
 *   - cv::BFMatcher(NORM_HAMMING).knnMatch(k=2)  cpp/src/Frame.cc:45,1227
 *   - mvImagePyramid (public member)      cpp/include/ORBextractor_old.h:80
 *   - Frame::ComputeStereoMatches         cpp/include/Frame.h:119, cpp/src/Frame.cc:827-997
 *   - ORBmatcher::SearchByProjection (Frame&, vector<MapPoint*>)  cpp/src/ORBmatcher.cc:44-214
 *   - Frame::UndistortKeyPoints / ComputeImageBounds / AssignFeaturesToGrid
 *                                         cpp/src/Frame.cc:405-436, 741-825
 */
#ifndef ORBGPU_H_
#define ORBGPU_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORBGPU_ABI_VERSION 2  /* 2: packed orbgpu_export_batch, ORBGPU_DEVICE_CURRENT */

/* Status codes (the DSP path returned 1/3/7 and callers ignored them; we never exit()). */
enum {
    ORBGPU_OK = 0,
    ORBGPU_ERR_EMPTY_IMAGE = -1,  /* reference operator() returns -1 on an empty image (:1092) */
    ORBGPU_ERR_CAPACITY = -2,     /* caller buffer / context capacity too small */
    ORBGPU_ERR_INVALID = -3,      /* bad argument */
    ORBGPU_ERR_HIP = -4,          /* HIP runtime error (see orbgpu_last_error) */
    ORBGPU_ERR_OVERFLOW = -5,     /* device-side workspace overflow (keys / nodes) */
    ORBGPU_ERR_NO_DEVICE = -6,    /* no usable gfx950 device */
    ORBGPU_ERR_RUNTIME = -7       /* two HIP runtimes mapped into the process (import torch first) */
};

/* The 5 ORB parameters of the ORBextractor ctor / Settings.cc:443-451. */
typedef struct {
    int32_t nfeatures;
    float scale_factor;
    int32_t nlevels;
    int32_t ini_th_fast;
    int32_t min_th_fast;
} orbgpu_params;

/* cv::KeyPoint field layout (28 B): pt.x, pt.y, size, angle, response, octave, class_id. */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orbgpu_keypoint;

typedef struct orbgpu_ctx orbgpu_ctx;

/* Build a context for images up to max_width x max_height and batches of up to max_images
 * images.  Allocates all device memory once (nothing is allocated per call).  device = HIP
 * ordinal, or ORBGPU_DEVICE_CURRENT: the calling thread's current HIP device (hipGetDevice), so a
 * multi-camera process places each extractor on the GPU it selected before constructing it (the
 * C++ facades pass it); orbgpu_get_device reports the ordinal a context uses.
 * Replaces the ORBextractor ctor + LynxHardwareAccelerator ctor (orbslam3_open).
 * ORBGPU_ERR_INVALID for nlevels outside [1, 16], scale_factor not above 1 (any value above 1,
 * as ORBextractor; steps above 2 build the pyramid level by level from HBM), negative nfeatures
 * or sizes outside (0, 4112), or a pyramid level under 42 px (at the first batch of that size);
 * ORBGPU_ERR_NO_DEVICE without a HIP device. */
#define ORBGPU_DEVICE_CURRENT (-1)
int orbgpu_create(const orbgpu_params* params, int device, int max_width, int max_height,
                  int max_images, orbgpu_ctx** out_ctx);
int orbgpu_get_device(const orbgpu_ctx* ctx); /* the context's HIP ordinal (ORBGPU_ERR_INVALID: null) */
int orbgpu_destroy(orbgpu_ctx* ctx); /* orbslam3_close */

/* Scale tables exactly as the ORBextractor getters return them (GetScaleFactors, ...). */
int orbgpu_get_scale_tables(const orbgpu_ctx* ctx, float* scale, float* inv_scale,
                            float* sigma2, float* inv_sigma2, int32_t* features_per_level);

/* ORBextractor::operator()(image, mask, keypoints, descriptors, vLappingArea) on one host
 * image (u8, row stride `stride`).  Writes *n keypoints (cv::KeyPoint layout) and n x 32 B
 * descriptors (row i <-> keypoint i), mono first / lapping-area keypoints from the back;
 * *n_mono = return value of the reference (monoIndex).  cap = capacity of kps/desc. */
int orbgpu_extract(orbgpu_ctx* ctx, const uint8_t* image, int width, int height, int stride,
                   int lap0, int lap1, orbgpu_keypoint* kps, uint8_t* desc, int cap, int* n,
                   int* n_mono);

/* Stereo form (ORBextractor.h:52-57 / IDL extractFeatures): left and right images in one call,
 * both on the device together. */
int orbgpu_extract_stereo(orbgpu_ctx* ctx, const uint8_t* left, const uint8_t* right, int width,
                          int height, int stride, const int lap_left[2], const int lap_right[2],
                          orbgpu_keypoint* kps_left, uint8_t* desc_left, int* n_left,
                          int* mono_left, orbgpu_keypoint* kps_right, uint8_t* desc_right,
                          int* n_right, int* mono_right, int cap);

/* ---- device-resident batch API (the throughput path) --------------------------------------
 * Images live in the context's HBM input buffer: [n_images][height][width] u8 (pitch = width).
 * orbgpu_upload_images copies host pixels in (PCIe; not part of the timed hot path).
 * orbgpu_run_batch runs the whole front-end for n_images images on `stream` (void* hipStream_t,
 * NULL = the context's own stream) and leaves keypoints/descriptors/counts in HBM.
 * laps: n_images x {lap0, lap1}, host pointer (copied into the launch arguments). */
int orbgpu_upload_images(orbgpu_ctx* ctx, const uint8_t* images, int n_images, int width,
                         int height, int stride);
uint8_t* orbgpu_device_input(orbgpu_ctx* ctx); /* device pointer of the input buffer */
/* Streaming ingest (C3: one frame pair after another, LynxHardwareAccelerator.cpp:121-123 copies
 * each frame in): stage the NEXT batch's pixels while the current batch computes.  The copy runs
 * on the context's copy stream into the second input buffer, after every kernel that read that
 * buffer; the next orbgpu_run_batch reads it once the copy has landed.  `images` should be pinned
 * (orbgpu_host_alloc) for the copy to run asynchronously at full PCIe rate.  One staged upload at
 * a time (ORBGPU_ERR_INVALID otherwise). */
int orbgpu_upload_images_async(orbgpu_ctx* ctx, const uint8_t* images, int n_images, int width,
                               int height, int stride);
/* Page-locked host memory for the async upload (hipHostMalloc / hipHostFree). */
int orbgpu_host_alloc(size_t bytes, void** ptr);
int orbgpu_host_free(void* ptr);
int orbgpu_run_batch(orbgpu_ctx* ctx, int n_images, int width, int height, const int32_t* laps,
                     void* stream);
/* Copy image i's results to the host (after orbgpu_synchronize or on the same stream). */
int orbgpu_download_result(orbgpu_ctx* ctx, int image, orbgpu_keypoint* kps, uint8_t* desc,
                           int cap, int* n, int* n_mono);
/* Per-image keypoint counts and mono counts of the last batch (host arrays of n_images). */
int orbgpu_download_counts(orbgpu_ctx* ctx, int n_images, int32_t* n, int32_t* n_mono);
/* Per-image number of cell keypoints that entered DistributeOctTree (vToDistributeKeys summed
 * over the levels) in the last batch: the octree's input size, for instrumentation. */
int orbgpu_candidate_counts(orbgpu_ctx* ctx, int n_images, int32_t* counts);
int orbgpu_synchronize(orbgpu_ctx* ctx);

/* Pyramid level `level` of batch image `image` (mvImagePyramid[level]), optionally blurred
 * (the GaussianBlur'd working copy, ORBextractor_old.cc:1146-1147). */
int orbgpu_get_pyramid_level(orbgpu_ctx* ctx, int image, int level, int blurred, uint8_t* dst,
                             int dst_stride, int* width, int* height);

/* Level keypoints before assembly (level coordinates, octree order, with angle) and their
 * descriptors: for per-stage parity tests.  counts[nlevels]. */
int orbgpu_get_level_keypoints(orbgpu_ctx* ctx, int image, orbgpu_keypoint* kps, uint8_t* desc,
                               int cap, int32_t* counts);

/* ---- Hamming matching ---------------------------------------------------------------------
 * cv::BFMatcher(NORM_HAMMING).knnMatch(query, train, matches, 2): for each query row the best
 * and second-best train rows (lexicographic (distance, index): lowest index wins ties);
 * idx = -1 / dist = INT32_MAX when absent (nt < 2).  Host pointers, n x 32 B each. */
int orbgpu_match_knn2(orbgpu_ctx* ctx, const uint8_t* query, int nq, const uint8_t* train, int nt,
                      int32_t* idx1, int32_t* dist1, int32_t* idx2, int32_t* dist2);
/* Device-pointer forms for multi-GPU exchange (C5 cross-camera BFMatch, SURVEY §8e: the
 * descriptors go from this context's HBM straight into a collective's buffer and back into the
 * matcher; nothing touches the host):
 *   orbgpu_export_descriptors: rows [row0, n) of batch image `image` -> device_dst (cap_rows x 32 B),
 *     *n_rows = rows copied (host); device-to-device on `stream` (NULL = the context's stream),
 *     ordered after the batch that produced them;
 *   orbgpu_match_knn2_device: orbgpu_match_knn2 with query / train / outputs in device memory
 *     (idx1, dist1, idx2, dist2: int32 [nq] each), on `stream`. */
int orbgpu_export_descriptors(orbgpu_ctx* ctx, int image, int row0, uint8_t* device_dst, int cap_rows,
                              int* n_rows, void* stream);
int orbgpu_match_knn2_device(orbgpu_ctx* ctx, const uint8_t* d_query, int nq, const uint8_t* d_train, int nt,
                             int32_t* d_idx1, int32_t* d_dist1, int32_t* d_idx2, int32_t* d_dist2, void* stream);

/* The C4 ingest-rank path (frames ingested on one GPU, every result handed back to
 * one caller, as LynxHardwareAccelerator.cpp:146-204 returns each frame's keypoints, descriptors
 * and matches to its caller), device memory throughout so a collective can move both ends:
 *   orbgpu_ingest_images: n images already in device memory (e.g. a scatter's receive buffer;
 *     rows of `stride` bytes) -> the context's input buffer, device to device on `stream`; the
 *     next orbgpu_run_batch / run_batch_match reads them;
 *   orbgpu_export_batch: the last batch's results of images [0, n_images) and stereo pairs
 *     [0, n_pairs) -> one device buffer (e.g. a gather's send buffer, 4-byte aligned), device to
 *     device on `stream`, ordered after the batch.  Only the rows produced are packed:
 *       int32 count[n_images], int32 mono[n_images], int32 n_queries[n_pairs],
 *       then for each image i: orbgpu_keypoint kps[count[i]], uint8 desc[count[i]][32],
 *       then for each pair p: int32 idx1[n_queries[p]], dist1[..], idx2[..], dist2[..]
 *       (the last match call's).
 *     *used = the layout's size in bytes.  The counts size it, so the call waits for the batch;
 *     device_dst = NULL only reports *used (the size query before a collective's allocation).
 *     A count the device replaced by a status (octree workspace overflow, output capacity) is
 *     returned as that status (ORBGPU_ERR_OVERFLOW / ORBGPU_ERR_CAPACITY) and nothing is packed.
 *     orbgpu_export_batch_bytes: the largest such layout (every image at the context's row
 *     capacity), with no device access. */
int orbgpu_ingest_images(orbgpu_ctx* ctx, const uint8_t* device_images, int n_images, int width,
                         int height, int stride, void* stream);
size_t orbgpu_export_batch_bytes(const orbgpu_ctx* ctx, int n_images, int n_pairs);
int orbgpu_export_batch(orbgpu_ctx* ctx, int n_images, int n_pairs, void* device_dst, size_t dst_bytes,
                        size_t* used, void* stream);

/* Batch stereo matching on device-resident results of the last orbgpu_run_batch: pair p
 * matches image 2p (query) against image 2p+1 (train), rows [mono..n) of each when
 * stereo_rows_only != 0 (Frame::ComputeStereoFishEyeMatches, Frame.cc:1142-1148) or all rows.
 * Results stay in HBM; fetch with orbgpu_download_matches. */
int orbgpu_match_stereo_batch(orbgpu_ctx* ctx, int n_pairs, int stereo_rows_only, void* stream);
/* orbgpu_run_batch followed by orbgpu_match_stereo_batch over all n_images / 2 pairs, as ONE
 * submission when the batch runs as one captured graph (the latency shape: the accelerator
 * session's stereo frame, LynxHardwareAccelerator.cpp:133-204, which extracts both eyes and
 * runs BFMatchORB's kNN2 in one device pass); otherwise exactly the two calls.  n_images even. */
int orbgpu_run_batch_match(orbgpu_ctx* ctx, int n_images, int width, int height, const int32_t* laps,
                           int stereo_rows_only, void* stream);
int orbgpu_download_matches(orbgpu_ctx* ctx, int pair, int32_t* idx1, int32_t* dist1,
                            int32_t* idx2, int32_t* dist2, int cap, int* nq);

/* ---- stereo matching ----------------------------------------------------------------------
 * Frame::ComputeStereoMatches (cpp/src/Frame.cc:827-997, called from the stereo Frame ctor
 * :161 and FrameAHB.cc:129) on the device-resident results of the last orbgpu_run_batch:
 * pair p = left image 2p (mvKeys), right image 2p+1 (mvKeysRight), rectified pinhole stereo.
 * mbf = baseline * fx, mb = baseline (Frame::mbf, Frame::mb).  Per left keypoint: mvuRight and
 * mvDepth (-1 = no stereo match), and the accepted SAD distance (-1 = none; also set for
 * matches the median rule rejects).  Results stay in HBM; fetch with orbgpu_download_stereo. */
int orbgpu_stereo_matches_batch(orbgpu_ctx* ctx, int n_pairs, float mbf, float mb, void* stream);
int orbgpu_download_stereo(orbgpu_ctx* ctx, int pair, float* u_right, float* depth, int32_t* sad,
                           int cap, int* n);

/* ---- fisheye stereo ------------------------------------------------------------------------
 * Frame::ComputeStereoFishEyeMatches (cpp/src/Frame.cc:1142-1201, called from the two-camera
 * Frame ctor :1121 and FrameAHB.cc:320) on the device-resident results of the last
 * orbgpu_run_batch: pair p = left image 2p (mvKeys), right image 2p+1 (mvKeysRight).  Runs the
 * stereo-row kNN2 (BFMatchORB, :1164 = orbgpu_match_stereo_batch with stereo_rows_only = 1; its
 * result stays readable through orbgpu_download_matches), then per left stereo row: dist1 == 0
 * skipped, dist1 < 70 triangulated with KannalaBrandt8::TriangulateMatches
 * (CameraModels/KannalaBrandt8.cpp:300-366; sigmas = mvLevelSigma2 of the two octaves) and
 * accepted when the depth > 1e-4.  Parity with the reference is unpinned (Eigen's JacobiSVD
 * order and FMA use, the Android libm's atan2f / tanf): see DESIGN.md and tests/test_fisheye.py. */
typedef struct {
    float cam_left[8], cam_right[8];   /* KannalaBrandt8 mvParameters: fx fy cx cy k0 k1 k2 k3 */
    float precision_left, precision_right;  /* KannalaBrandt8::precision (1e-6 by default) */
    float R12[9];                      /* Frame::mRlr, row-major */
    float t12[3];                      /* Frame::mtlr */
} orbgpu_kb8_rig;
int orbgpu_fisheye_stereo_batch(orbgpu_ctx* ctx, int n_pairs, const orbgpu_kb8_rig* rig, void* stream);
/* Per pair: mvLeftToRightMatch [n_left], mvRightToLeftMatch [n_right] (-1 = none), mvDepth
 * [n_left] (-1 = none), mvStereo3Dpoints [n_left][3] (0 where none), nMatches. */
int orbgpu_download_fisheye(orbgpu_ctx* ctx, int pair, int32_t* l2r, int32_t* r2l, float* depth, float* p3d,
                            int cap, int* n_left, int* n_right, int* n_matches);

/* ---- ORBmatcher::SearchByProjection (cpp/src/ORBmatcher.cc:44-214, pinhole frames) ---------
 * Tracking's local-map search: every map point predicted in view is matched against the frame
 * keypoints in a window around its projection (Frame::GetFeaturesInArea, Frame.cc:673-735, on the
 * grid of orbgpu_undistort_grid_batch), best/second-best Hamming with TH_HIGH = 100 and the
 * nnratio test; the keypoint is then taken (later map points skip it when the taker has
 * observations).  Frames are batch images f * image_step (image_step 2: the left eye of stereo
 * pair f, whose mvuRight from orbgpu_stereo_matches_batch is used when use_uright != 0;
 * image_step 1: monocular frames, mvuRight all -1).
 * A map point carries the MapPoint state the function reads: */
typedef struct {
    float proj_x, proj_y;  /* mTrackProjX, mTrackProjY */
    float proj_xr;         /* mTrackProjXR */
    float view_cos;        /* mTrackViewCos */
    float depth;           /* mTrackDepth */
    int32_t level;         /* mnTrackScaleLevel, in [0, nlevels) (others are skipped) */
    int32_t flags;         /* ORBGPU_MP_* */
    uint8_t desc[32];      /* GetDescriptor() */
    float proj_yr;         /* mTrackProjYR     (two-camera frames) */
    float view_cos_r;      /* mTrackViewCosR   (two-camera frames) */
    int32_t level_r;       /* mnTrackScaleLevelR (two-camera frames) */
} orbgpu_map_point;
#define ORBGPU_MP_IN_VIEW 1    /* mbTrackInView */
#define ORBGPU_MP_BAD 2        /* isBad() */
#define ORBGPU_MP_HAS_OBS 4    /* Observations() > 0 */
#define ORBGPU_MP_IN_VIEW_R 8  /* mbTrackInViewR (two-camera frames) */
/* mps: all frames' map points, frame f's in [mp_offsets[f], mp_offsets[f + 1]) (host arrays).
 * kp_block (optional, [n_frames][kp_stride] u8): 1 where F.mvpMapPoints[k] is already set to a
 * point with observations before the call.  th / nnratio / far_points / th_far as the reference.
 * orbgpu_download_projection_matches: match[k] = index (within the frame's map points) of the
 * point assigned to keypoint k by this call, -1 if none; *nmatches = the reference's return. */
int orbgpu_search_by_projection_batch(orbgpu_ctx* ctx, int n_frames, int image_step, int use_uright,
                                      const orbgpu_map_point* mps, const int32_t* mp_offsets,
                                      const uint8_t* kp_block, int kp_stride, float th, float nnratio,
                                      int far_points, float th_far, void* stream);
/* Two-camera frames (Nleft != -1, the fisheye rig; ORBmatcher.cc:59-214): frame f = left image
 * 2f + right image 2f + 1, both gridded by orbgpu_undistort_grid_batch with no distortion
 * coefficients (the grid is built on the raw positions, Frame.cc:405-436, and the bounds are the
 * image, :798-825).  left_to_right / right_to_left ([n_pairs][lr_stride], -1 = none; NULL: all
 * -1) are Frame::mvLeftToRightMatch / mvRightToLeftMatch.  kp_block and the downloaded match
 * array cover Nleft + Nright keypoints: the left ones, then the right ones (the reference's
 * mvpMapPoints indexing). */
int orbgpu_search_by_projection_stereo(orbgpu_ctx* ctx, int n_pairs, const orbgpu_map_point* mps,
                                       const int32_t* mp_offsets, const int32_t* left_to_right,
                                       const int32_t* right_to_left, int lr_stride, const uint8_t* kp_block,
                                       int kp_stride, float th, float nnratio, int far_points, float th_far,
                                       void* stream);
int orbgpu_download_projection_matches(orbgpu_ctx* ctx, int frame, int32_t* match, int cap, int* n_kp,
                                       int* nmatches);

/* ---- wire formats ---------------------------------------------------------------------------
 * Ingest of side-by-side stereo Y8 frames (the headset's 2W x H AHardwareBuffer,
 * ORBextractor.cc:131-143; DSP split orbslam_dsp.cpp:643-648): frame f's left half (columns
 * [0, W)) becomes batch image 2f, its right half (columns [W, 2W)) image 2f + 1.  Frames are
 * height rows of `stride` bytes (stride >= 2W), height * stride bytes apart.
 *   orbgpu_upload_sbs: host frames (PCIe into a staging buffer, then the split kernel);
 *   orbgpu_ingest_sbs: frames already in device memory (e.g. the staging buffer returned by
 *   orbgpu_device_sbs_input, sized for max_images / 2 frames of stride 2 * max_width), on
 *   `stream` -- the zero-copy path. */
uint8_t* orbgpu_device_sbs_input(orbgpu_ctx* ctx);
int orbgpu_upload_sbs(orbgpu_ctx* ctx, const uint8_t* frames, int n_frames, int width, int height,
                      int stride);
int orbgpu_ingest_sbs(orbgpu_ctx* ctx, const uint8_t* device_frames, int n_frames, int width,
                      int height, int stride, void* stream);

/* Egress in the FastRPC result layout (cpp/inc/orbslam3.idl:15-19): per image int32 X, Y (the
 * level-0 coordinates truncated to int), angle ((cos8 & 0xFF) | (sin8 & 0xFF) << 8 with
 * cos8/sin8 = rint(64 cos / 64 sin) of the keypoint angle: what LynxHardwareAccelerator.cpp:
 * 174-178 decodes), level (octave) and the N x 32 B descriptors; per stereo pair the kNN result
 * as int16 indices / distances1 / distances2 (distances clamped to 32767; absent = -1 / 32767).
 * orbgpu_pack_soa converts the first n_images images and n_pairs pairs of the last batch on the
 * device (device-resident SoA), the download functions copy one image / pair out. */
int orbgpu_pack_soa(orbgpu_ctx* ctx, int n_images, int n_pairs, void* stream);
int orbgpu_download_soa(orbgpu_ctx* ctx, int image, int32_t* x, int32_t* y, int32_t* angle,
                        int32_t* level, uint8_t* orb, int cap, int* count, int* mono);
int orbgpu_download_matches16(orbgpu_ctx* ctx, int pair, int16_t* indices, int16_t* dist1,
                              int16_t* dist2, int cap, int* n_queries);

/* orbslam3_extractFeatures (orbslam3.idl:15-19, impl orbslam_dsp.cpp:1003-1087) in one call: one
 * side-by-side frame in, both eyes extracted (lapping areas {l0, l1} / {r0, r1}), the stereo
 * rows ([mono, n) of each eye, Frame.cc:1142-1148) kNN2-matched left -> right, everything out in
 * the SoA layout above.  `threshold` is accepted and ignored, as the DSP does; the context's
 * FAST thresholds apply.  *count_* is the exact keypoint count (the DSP's host wrapper subtracts
 * one from its count, LynxHardwareAccelerator.cpp:158-159; a caller of this ABI must not). */
int orbgpu_extract_features(orbgpu_ctx* ctx, const uint8_t* image, int image_len, int width,
                            int height, int stride, int threshold, int lap_l0, int lap_l1,
                            int lap_r0, int lap_r1, int* count_l, int32_t* x_l, int32_t* y_l,
                            int32_t* angle_l, int32_t* level_l, uint8_t* orb_l, int* count_r,
                            int32_t* x_r, int32_t* y_r, int32_t* angle_r, int32_t* level_r,
                            uint8_t* orb_r, int kp_cap, int* mono_l, int* mono_r, int16_t* indices,
                            int16_t* dist1, int16_t* dist2, int match_cap);

/* ---- Frame post-processing ----------------------------------------------------------------
 * Frame::UndistortKeyPoints (cpp/src/Frame.cc:763-796; cv::undistortPoints with P = K, 5
 * iterations in double) and Frame::AssignFeaturesToGrid + PosInGrid (:405-436, 741-751; 64 x 48
 * cells, Frame.h:46-47) for the first n_images images of the last orbgpu_run_batch.
 * K = {fx, fy, cx, cy}; dist = {k1, k2, p1, p2[, k3]} (ndist 0, 4 or 5; k1 == 0: no undistortion,
 * as :765).  The grid spans Frame::ComputeImageBounds (:798-825) of the batch image size, which
 * orbgpu_image_bounds returns ({mnMinX, mnMaxX, mnMinY, mnMaxY}, host computation).
 * Per image: undistorted positions (mvKeysUn.pt), the cell of each keypoint (posX * 48 + posY,
 * -1 outside the grid) and the cells as CSR lists (cell_start[64*48 + 1], cell_idx: keypoint
 * indices ascending within a cell = mGrid[posX][posY]). */
int orbgpu_image_bounds(int cols, int rows, const float K[4], const float* dist, int ndist, float bounds[4]);
int orbgpu_undistort_grid_batch(orbgpu_ctx* ctx, int n_images, const float K[4], const float* dist,
                                int ndist, void* stream);
int orbgpu_download_grid(orbgpu_ctx* ctx, int image, float* xy_un, int32_t* cell, int32_t* cell_start,
                         int32_t* cell_idx, int cap, int* n);

/* ORBmatcher::DescriptorDistance on two 32-byte descriptors (host, no device work). */
int orbgpu_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* ---- instrumentation ----------------------------------------------------------------------
 * enable = 1: every kernel launch of run_batch/match_stereo_batch is bracketed by HIP events on
 * its stream; enable = (1 << 31) | mask: only the stages whose bit is set; 0: off.  Adding
 * (1 << 30) also launches every stage once over the whole batch (no sub-batch overlap), so each
 * launch's duration is that kernel's alone.
 * orbgpu_stage_times returns the summed milliseconds and launch counts per stage since the last
 * reset.  Stage names via orbgpu_stage_name. */
int orbgpu_set_profiling(orbgpu_ctx* ctx, int enable);
int orbgpu_num_stages(void);
const char* orbgpu_stage_name(int stage);
int orbgpu_stage_times(orbgpu_ctx* ctx, double* ms, int64_t* launches, int max_stages);
int orbgpu_reset_stage_times(orbgpu_ctx* ctx);

/* Measurement knobs (ORBGPU_STREAMS, ORBGPU_OCT_SPLIT, ORBGPU_FAST_PITCH, ...) change launch
 * shapes and kernel variants; the library reads them only when ORBGPU_DIAGNOSTICS=1 is also set.
 * Writes the knobs in effect as "NAME=value;..." (NUL-terminated, truncated to cap) and returns
 * their count: 0 in a deployment. */
int orbgpu_diagnostic_knobs(char* buf, size_t cap);

const char* orbgpu_last_error(void);
int orbgpu_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ORBGPU_H_ */
