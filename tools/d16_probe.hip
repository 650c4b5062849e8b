// Probe: does ds_read_u8_d16_hi keep the low half written by a ds_read_u8 to the same VGPR that
// is still in flight (both reads issued back to back, one wait)?  Prints mismatches.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out, int wait_between) {
    __shared__ unsigned char T[256];
    T[threadIdx.x] = (unsigned char)(threadIdx.x * 7 + 1);
    __syncthreads();
    const unsigned base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)T;
    const unsigned a = base + threadIdx.x, b = base + ((threadIdx.x + 17) & 255);
    unsigned r;
    if (wait_between)
        asm volatile("ds_read_u8 %0, %1\n s_waitcnt lgkmcnt(0)\n ds_read_u8_d16_hi %0, %2\n s_waitcnt lgkmcnt(0)"
                     : "=&v"(r) : "v"(a), "v"(b) : "memory");
    else
        asm volatile("ds_read_u8 %0, %1\n ds_read_u8_d16_hi %0, %2\n s_waitcnt lgkmcnt(0)"
                     : "=&v"(r) : "v"(a), "v"(b) : "memory");
    out[threadIdx.x] = r;
}
int main() {
    unsigned* d;
    unsigned h[256];
    hipMalloc(&d, 1024);
    for (int w = 0; w < 2; ++w) {
        hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, d, w);
        hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < 256; ++i) {
            const unsigned want = ((i * 7 + 1) & 255) | ((((((i + 17) & 255) * 7) + 1) & 255) << 16);
            if (h[i] != want) {
                if (bad < 4) printf("wait=%d lane %d got %08x want %08x\n", w, i, h[i], want);
                ++bad;
            }
        }
        printf("wait_between=%d mismatches %d\n", w, bad);
    }
    return 0;
}
