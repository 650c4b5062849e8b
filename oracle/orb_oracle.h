// orb_oracle.h -- TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference CPU ORB front-end (Lynx-MR/orbslam3lib,
// app/src/main/cpp/src/ORBextractor_old.cc) and of the OpenCV 4.2.0 primitives it calls
// (cv::resize INTER_LINEAR, cv::FAST TYPE_9_16 + nonmax, cv::GaussianBlur 7x7 sigma 2,
// cv::fastAtan2, cv::BFMatcher NORM_HAMMING knn).  OpenCV is not present in this image, so
// the OpenCV parts are restated from its published algorithm; the choices that OpenCV's
// build configuration leaves open are pinned as named constants below.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code,
// and only as the checker.  The product (liborbgpu.so) never links or calls it.
//
// Parity status: PARTIALLY PINNED.  The reference ships no tests/fixtures for this path and its
// CPU extractor cannot be built here (OpenCV 4.2 is fetched at configure time, Android headers,
// syntax error at ORBextractor_old.cc:477).  Pinned from the reference: the rBRIEF table (sha256),
// umax, level sizes, per-level feature split.  The OpenCV internals are restated (unpinned
// against OpenCV itself) and cross-checked by independent brute-force restatements in tests/.
#pragma once
#include <cstddef>
#include <cstdint>

extern "C" {

// cv::KeyPoint field layout (28 bytes).
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} oracle_kp;

// Pinned OpenCV-4.2 choices:
//  * resize vertical pass: 128-bit-SIMD body (VResizeLinearVec_32s8u) for x < simd_end(width),
//    scalar FixedPtCast tail after it.                     -> oracle_resize_simd_end()
//  * GaussianBlur 7x7 sigma=2 fixed-point kernel with error diffusion: {18,34,48,56,48,34,18}/256
//  * cos/sin in computeOrbDescriptor: (float)cos((double)angle)
//  * no FMA contraction anywhere (-ffp-contract=off)
int oracle_resize_simd_end(int width);
void oracle_blur_kernel(int32_t k[7]);

// Full ORBextractor::operator() (ORBextractor_old.cc:1088-1191) on one image.
// Returns monoIndex (or -1 on empty image, -2 on capacity overflow).  *n_out = N keypoints.
int oracle_extract(int nfeatures, float scale_factor, int nlevels, int ini_th, int min_th,
                   const uint8_t* img, int w, int h, int stride, int lap0, int lap1,
                   oracle_kp* kps, uint8_t* desc, int cap, int* n_out);

// Same, but per level, before assembly: keypoints in level coordinates in octree order with
// orientation, and their descriptors.  lvl_count[nlevels]; kps/desc packed level after level.
int oracle_extract_levels(int nfeatures, float scale_factor, int nlevels, int ini_th, int min_th,
                          const uint8_t* img, int w, int h, int stride,
                          oracle_kp* kps, uint8_t* desc, int cap, int* lvl_count);

// Pyramid level sizes (canonical ComputePyramid, ORBextractor_old.cc:1333-1339).
void oracle_level_sizes(float scale_factor, int nlevels, int w, int h, int* lw, int* lh);
// Whole pyramid, levels packed tightly (pitch = width) one after another into out.
int oracle_pyramid(float scale_factor, int nlevels, const uint8_t* img, int w, int h, int stride,
                   uint8_t* out);
// cv::resize(src, dst, Size(dw,dh), 0, 0, INTER_LINEAR) on CV_8UC1.
void oracle_resize(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh,
                   int dstride);
// cv::GaussianBlur(src, dst, Size(7,7), 2, 2, BORDER_REFLECT_101) on CV_8UC1, tight pitch.
void oracle_gaussian_blur(const uint8_t* src, int w, int h, uint8_t* dst);
// cv::FAST(roi, kps, th, true) on an ROI (x0,y0,cols,rows) of an image with row stride.
int oracle_fast(const uint8_t* img, int stride, int x0, int y0, int cols, int rows, int th,
                oracle_kp* kps, int cap);
// FAST score of one pixel as the nonmax buffer would hold it (cornerScore<16>), th-clamped.
int oracle_corner_score(const uint8_t* img, int stride, int x, int y, int th);
// Per-level keypoints BEFORE the octree (cell loop of ComputeKeyPointsOctTree, :807-874),
// coordinates relative to (minBorderX, minBorderY) exactly as vToDistributeKeys holds them.
int oracle_level_candidates(const uint8_t* lvl, int w, int h, int ini_th, int min_th,
                            oracle_kp* kps, int cap);
// DistributeOctTree (ORBextractor_old.cc:557-781) on a candidate list.
int oracle_distribute_octree(const oracle_kp* keys, int n, int minX, int maxX, int minY, int maxY,
                             int N, oracle_kp* out, int cap);
float oracle_fast_atan2(float y, float x);
float oracle_ic_angle(const uint8_t* img, int stride, int x, int y);
void oracle_orb_descriptor(const uint8_t* blurred, int stride, float x, float y, float angle,
                           uint8_t* desc32);
void oracle_umax(int* umax16);
void oracle_features_per_level(int nfeatures, float scale_factor, int nlevels, int* out);
void oracle_scale_factors(float scale_factor, int nlevels, float* scale, float* inv_scale,
                          float* sigma2, float* inv_sigma2);
// ORBmatcher::DescriptorDistance (ORBmatcher.cc:2107-2123).
int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b);
// cv::BFMatcher(NORM_HAMMING).knnMatch(q, t, m, 2) -> per query (idx1,d1,idx2,d2); idx=-1 absent.
/* Measurement switch (tests only): 1 evaluates the descriptor's cos / sin as (float)cos((double)a)
 * instead of the reference's float overloads; 0 (default) follows the reference. */
void oracle_set_trig_double(int on);
/* Frames-parallel pool: n_images frames (pitch w) over nthreads threads; total keypoints. */
long long oracle_extract_many(int nfeatures, float scale_factor, int nlevels, int ini_th, int min_th,
                              const uint8_t* imgs, int n_images, int w, int h, int nthreads, int32_t* counts);
void oracle_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* idx1, int32_t* d1,
                 int32_t* idx2, int32_t* d2);
// Reference-ordered sort (std::sort + compareNodes, ORBextractor_old.cc:540-555,702) on
// (size, ULx) pairs; writes the permutation of input indices.
void oracle_sort_nodes(const int32_t* size, const int32_t* ulx, int n, int32_t* perm);

// Frame::ComputeStereoMatches (Frame.cc:827-997) on one rectified stereo frame: row-band Hamming
// search (TH_HIGH / (TH_HIGH+TH_LOW)/2), 11x11 SAD over +-5 px on the unblurred pyramid level of
// the left keypoint, parabola sub-pixel fit, median-SAD outlier rejection.  Outputs mvuRight and
// mvDepth (-1 = unmatched) and the accepted SAD distances (-1 = none).
void oracle_stereo_matches(const oracle_kp* kpsL, int nL, const uint8_t* descL, const oracle_kp* kpsR,
                           int nR, const uint8_t* descR, const uint8_t* const* pyrL,
                           const uint8_t* const* pyrR, const int* lw, const int* lh, int nlevels,
                           const float* scale, const float* inv_scale, float mbf, float mb,
                           float* uRight, float* depth, int32_t* sad);

// Frame::UndistortKeyPoints (Frame.cc:763-796; cv::undistortPoints, 5 fixed-point iterations in
// double, P = K), Frame::ComputeImageBounds (:798-825) and Frame::AssignFeaturesToGrid +
// PosInGrid (:405-436, 741-751) on a 64 x 48 grid.  K = fx fy cx cy, dist = k1 k2 p1 p2 [k3].
void oracle_undistort_points(const float* xy, int n, const float K[4], const float* dist, int ndist, float* out);
void oracle_image_bounds(int cols, int rows, const float K[4], const float* dist, int ndist, float bounds[4]);
void oracle_assign_grid(const float* xy_un, int n, const float bounds[4], int32_t* cell, int32_t* cell_start,
                        int32_t* cell_idx);

// The orbslam3.idl:15-19 result layout of n keypoints: X/Y = (int) of the coordinates (the DSP's
// truncation, orbslam_dsp.cpp:447-453), angle = (cos8 & 0xFF) | (sin8 & 0xFF) << 8 with
// cos8/sin8 = rint(64 * the descriptor rotation's (float)cos/sin((double)(angle * factorPI)))
// (decoded by LynxHardwareAccelerator.cpp:174-178), level = octave.
void oracle_pack_soa(const oracle_kp* kps, int n, int32_t* x, int32_t* y, int32_t* angle, int32_t* level);

// ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFarPoints)
// (ORBmatcher.cc:44-214) for a pinhole frame (Nleft == -1), with Frame::GetFeaturesInArea
// (Frame.cc:673-735) over the 64 x 48 grid of oracle_assign_grid and RadiusByViewingCos
// (:216-222).  A map point is the MapPoint state the function reads (mbTrackInView,
// mTrackProjX/Y/XR, mTrackViewCos, mTrackDepth, mnTrackScaleLevel, isBad, Observations() > 0,
// GetDescriptor()).  kp_block[k] = 1 when F.mvpMapPoints[k] is set with Observations() > 0 before
// the call (NULL: none); uRight = F.mvuRight (NULL: all -1, a monocular frame).  match[k] = the
// index of the map point assigned to keypoint k by this call (the last one), -1 otherwise.
// Returns nmatches.
typedef struct {
    float proj_x, proj_y, proj_xr, view_cos, depth;
    int32_t level;  // mnTrackScaleLevel
    int32_t flags;  // ORACLE_MP_* bits
    uint8_t desc[32];
    float proj_yr, view_cos_r;  // mTrackProjYR, mTrackViewCosR (two-camera frames)
    int32_t level_r;            // mnTrackScaleLevelR
} oracle_map_point;
#define ORACLE_MP_IN_VIEW 1
#define ORACLE_MP_BAD 2
#define ORACLE_MP_HAS_OBS 4
#define ORACLE_MP_IN_VIEW_R 8
int oracle_search_by_projection(const oracle_map_point* mps, int nmp, const float* xy_un, const int32_t* octave,
                                const uint8_t* desc, const float* uRight, int n, const float bounds[4],
                                const int32_t* cell_start, const int32_t* cell_idx, const float* scale,
                                int nlevels, const uint8_t* kp_block, float th, float nnratio,
                                int far_points, float th_far, int32_t* match);

// The two-camera form (Nleft != -1, ORBmatcher.cc:59-214): left keypoints [0, nl) and right
// keypoints [nl, nl + nr) with their own grids (built on the raw positions, as
// AssignFeaturesToGrid does for Nleft != -1, Frame.cc:405-436), mvLeftToRightMatch /
// mvRightToLeftMatch (NULL: all -1).  The left branch has no mvuRight test; the right branch
// uses mTrackProjXR/YR, mTrackViewCosR (no th factor) and mnTrackScaleLevelR.  kp_block and
// match cover nl + nr keypoints.
int oracle_search_by_projection2(const oracle_map_point* mps, int nmp, const float* xyL, const int32_t* octL,
                                 const uint8_t* descL, int nl, const int32_t* csL, const int32_t* ciL,
                                 const float* xyR, const int32_t* octR, const uint8_t* descR, int nr,
                                 const int32_t* csR, const int32_t* ciR, const float bounds[4],
                                 const int32_t* l2r, const int32_t* r2l, const float* scale, int nlevels,
                                 const uint8_t* kp_block, float th, float nnratio, int far_points,
                                 float th_far, int32_t* match);

// Frame::ComputeStereoFishEyeMatches (Frame.cc:1142-1201) on one frame's stereo-row kNN2
// (orb_fisheye.cpp; parity unpinned, see there).  idx1 / dist1: [nL - monoL]; cam*: KannalaBrandt8
// mvParameters; R12 row-major (mRlr), t12 (mtlr); sigma2: mvLevelSigma2.  Outputs: l2r [nL],
// r2l [nR], depth [nL], p3d [nL][3]; per stereo row: code (1 dist 0, 2 dist >= 70, 3 index,
// 4 parallax, 5 z1, 6 z2, 7 reprojection 1, 8 reprojection 2, 9 depth <= 1e-4, 10 accepted) and
// margins [5] (cos parallax, z1, z2, err1 - bound1, err2 - bound2; NaN where not reached).
// Returns nMatches.
int oracle_fisheye_stereo(const oracle_kp* kpsL, int nL, int monoL, const oracle_kp* kpsR, int nR, int monoR,
                          const int32_t* idx1, const int32_t* dist1, const float* camL, const float* camR,
                          float precL, float precR, const float* R12, const float* t12, const float* sigma2,
                          int32_t* l2r, int32_t* r2l, float* depth, float* p3d, int32_t* code, double* margins);

}  // extern "C"
