// orb_frame.hip -- per-keypoint Frame post-processing after extraction, on the
// device-resident keypoints of a batch: Frame::UndistortKeyPoints (cpp/src/Frame.cc:763-796,
// cv::undistortPoints with P = K) and Frame::AssignFeaturesToGrid + PosInGrid (:405-436,
// 741-751, FRAME_GRID_COLS x ROWS = 64 x 48, Frame.h:46-47).
//
// k_undistort_grid: one workgroup per image.  Each keypoint is undistorted in double with the
// operation order of OpenCV 4.2's cvUndistortPointsInternal (5 iterations, TermCriteria COUNT;
// the identity tilt / rectification products are exact and folded), placed in its grid cell,
// and the cells are built as CSR lists whose entries are in ascending keypoint order, like the
// push_back order of mGrid[posX][posY]: counts (LDS atomics) -> exclusive scan -> a stable
// scatter in chunks of 256 keypoints (rank among the earlier keypoints of the chunk in the same
// cell + the cell's running cursor).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_kernels.h"

namespace orbgpu {

namespace {
struct Kp {
    float x, y, size, angle, response;
    int32_t octave, class_id;
};
}  // namespace

__host__ __device__ inline void undistort_point_d(float px, float py, const float K[4], const double k[14],
                                                  float* ox, float* oy) {
    const double fx = K[0], fy = K[1], cx = K[2], cy = K[3];
    const double ifx = 1. / fx, ify = 1. / fy;
    double x = px, y = py;
    const double u = x, v = y;
    x = (x - cx) * ifx;
    y = (y - cy) * ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        if (icdist < 0) {
            x = (u - cx) * ifx;
            y = (v - cy) * ify;
            break;
        }
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    const double xx = fx * x + 0. * y + cx;
    const double yy = 0. * x + fy * y + cy;
    const double ww = 1. / (0. * x + 0. * y + 1.);
    *ox = (float)(xx * ww);
    *oy = (float)(yy * ww);
}

constexpr int kGridCells = kGridCols * kGridRows;

__global__ __launch_bounds__(256) void k_undistort_grid(GridArgs g) {
    __shared__ int32_t cur[kGridCells];
    __shared__ int32_t part[256];
    __shared__ int32_t sc[256];
    const int img = g.img0 + blockIdx.x;
    const int n = max(g.out_n[img], 0);
    const Kp* kp = reinterpret_cast<const Kp*>(g.kps) + (long long)img * g.out_cap;
    float* xy = g.xy_un + (long long)img * g.out_cap * 2;
    int32_t* cell = g.cell + (long long)img * g.out_cap;
    int32_t* start = g.cell_start + (long long)img * (kGridCells + 1);
    int32_t* idx = g.cell_idx + (long long)img * g.out_cap;
    const int tid = threadIdx.x;
    for (int c = tid; c < kGridCells; c += 256) cur[c] = 0;
    __syncthreads();
    const float wInv = g.grid_inv[0], hInv = g.grid_inv[1];
    for (int i = tid; i < n; i += 256) {
        float ux = kp[i].x, uy = kp[i].y;
        if (g.undistort) undistort_point_d(ux, uy, g.K, g.k, &ux, &uy);
        xy[2 * i] = ux;
        xy[2 * i + 1] = uy;
        const int posX = (int)roundf((ux - g.bounds[0]) * wInv);
        const int posY = (int)roundf((uy - g.bounds[2]) * hInv);
        const bool in = !(posX < 0 || posX >= kGridCols || posY < 0 || posY >= kGridRows);
        const int c = in ? posX * kGridRows + posY : -1;
        cell[i] = c;
        if (in) atomicAdd(&cur[c], 1);
    }
    __syncthreads();
    // exclusive scan of the 3072 counts: 12 per thread, then the 256 chunk sums on one wave
    constexpr int per = kGridCells / 256;
    int s = 0;
    for (int k = 0; k < per; ++k) s += cur[tid * per + k];
    part[tid] = s;
    __syncthreads();
    if (tid < 64) {
        int v[4], run = 0;
        for (int k = 0; k < 4; ++k) v[k] = part[4 * tid + k];
        const int tot = v[0] + v[1] + v[2] + v[3];
        int x = tot;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (tid >= o) x += y;
        }
        run = x - tot;
        for (int k = 0; k < 4; ++k) {
            part[4 * tid + k] = run;
            run += v[k];
        }
    }
    __syncthreads();
    int run = part[tid];
    for (int k = 0; k < per; ++k) {
        const int c = tid * per + k;
        const int v = cur[c];
        start[c] = run;
        cur[c] = run;  // the cell's cursor
        run += v;
    }
    if (tid == 255) start[kGridCells] = run;
    __syncthreads();
    for (int base = 0; base < n; base += 256) {
        const int i = base + tid;
        const int c = i < n ? cell[i] : -1;
        sc[tid] = c;
        __syncthreads();
        int pos = -1;
        if (c >= 0) {
            int r = 0;
            for (int j = 0; j < tid; ++j) r += sc[j] == c;
            pos = cur[c] + r;
        }
        __syncthreads();
        if (c >= 0) {
            idx[pos] = i;
            atomicAdd(&cur[c], 1);
        }
        __syncthreads();
    }
}

void grid_dist_table(const float* dist, int ndist, double k[14]) {
    for (int i = 0; i < 14; ++i) k[i] = 0;
    for (int i = 0; i < ndist && i < 5; ++i) k[i] = dist[i];
}

void image_bounds_host(int cols, int rows, const float K[4], const float* dist, int ndist, float b[4]) {
    if (ndist > 0 && dist[0] != 0.0f) {
        double k[14];
        grid_dist_table(dist, ndist, k);
        const float c[8] = {0.0f, 0.0f, (float)cols, 0.0f, 0.0f, (float)rows, (float)cols, (float)rows};
        float u[8];
        for (int i = 0; i < 4; ++i) undistort_point_d(c[2 * i], c[2 * i + 1], K, k, &u[2 * i], &u[2 * i + 1]);
        b[0] = u[4] < u[0] ? u[4] : u[0];  // std::min(mat(0,0), mat(2,0)), Frame.cc:813-816
        b[1] = u[2] < u[6] ? u[6] : u[2];  // std::max(mat(1,0), mat(3,0))
        b[2] = u[3] < u[1] ? u[3] : u[1];
        b[3] = u[5] < u[7] ? u[7] : u[5];
    } else {
        b[0] = 0.0f;
        b[1] = (float)cols;
        b[2] = 0.0f;
        b[3] = (float)rows;
    }
}

hipError_t launch_undistort_grid(const GridArgs& g, int nimages, hipStream_t st) {
    if (nimages <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_undistort_grid, dim3(nimages), dim3(256), 0, st, g);
    return hipGetLastError();
}

}  // namespace orbgpu
