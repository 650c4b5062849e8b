// wave_simd.hip -- which SIMD each wave of a 256-thread workgroup lands on (HW_ID bits 5:4), for
// workgroups resident together on one CU: histogram of wave 0's SIMD over 1024 workgroups, and
// of every wave's SIMD by its index in the workgroup.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(256) void k_simd(unsigned* out, long long cycles) {
    extern __shared__ int dyn[];
    const long long t0 = wall_clock64();
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
    dyn[threadIdx.x] = 1;
    __syncthreads();
    while (wall_clock64() - t0 < cycles) {
    }
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = hw;
}

int main() {
    const int nb = 1024;
    unsigned* d;
    if (hipMalloc(&d, nb * 4 * sizeof(unsigned)) != hipSuccess) return 1;
    for (int lds : {40704, 52224}) {
        hipLaunchKernelGGL(k_simd, dim3(nb), dim3(256), lds, 0, d, 3000LL);
        (void)hipDeviceSynchronize();
        unsigned h[nb * 4];
        (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        int hist[4][4] = {};
        for (int b = 0; b < nb; ++b)
            for (int w = 0; w < 4; ++w) hist[w][(h[b * 4 + w] >> 4) & 3]++;
        printf("lds %d: wave index -> SIMD histogram\n", lds);
        for (int w = 0; w < 4; ++w) printf("  wave %d: %4d %4d %4d %4d\n", w, hist[w][0], hist[w][1], hist[w][2], hist[w][3]);
        printf("  raw hw_id of wg 0..7 wave 0: ");
        for (int b = 0; b < 8; ++b) printf("%08x ", h[b * 4]);
        printf("\n");
    }
    return 0;
}
