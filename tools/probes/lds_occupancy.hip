// lds_occupancy.hip -- how many 256-thread workgroups with D bytes of dynamic LDS (plus 112 static)
// run at once on a CU: each workgroup spins ~50 us, 256 * k workgroups are launched for k = 1..6,
// and the launch time steps up when k passes the resident count.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void k_spin(int* out, long long cycles) {
    extern __shared__ int dyn[];
    __shared__ int stat[28];
    const long long t0 = wall_clock64();
    dyn[threadIdx.x] = (int)threadIdx.x;
    if (threadIdx.x < 28) stat[threadIdx.x] = 1;
    __syncthreads();
    while (wall_clock64() - t0 < cycles) {
    }
    if (threadIdx.x == 0) out[blockIdx.x] = dyn[5] + stat[3];
}

int main(int argc, char** argv) {
    int* out;
    if (hipMalloc(&out, 256 * 64 * sizeof(int)) != hipSuccess) return 1;
    const int sizes[] = {30000, 36000, 40704, 40816, 40960, 41472, 52224};
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int s : sizes) {
        (void)hipFuncSetAttribute((const void*)k_spin, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
        printf("dyn %6d:", s);
        for (int k = 1; k <= 6; ++k) {
            hipLaunchKernelGGL(k_spin, dim3(256 * k), dim3(256), s, 0, out, 5000LL);  // warm-up, 50 us at 100 MHz
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(a, 0);
            hipLaunchKernelGGL(k_spin, dim3(256 * k), dim3(256), s, 0, out, 5000LL);
            (void)hipEventRecord(b, 0);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            printf("  k=%d %6.1f us", k, ms * 1e3);
        }
        printf("\n");
    }
    return 0;
}
