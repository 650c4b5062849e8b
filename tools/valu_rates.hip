// valu_rates.hip -- measured issue cost of the VALU instructions the FAST / pyramid kernels lean
// on (gfx950): SIMD cycles per wave64 instruction with 8 waves per SIMD and 8 independent
// chains per wave.  Build: hipcc --offload-arch=gfx950 -O3 -o valu_rates tools/valu_rates.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define OP_KERNEL(NAME, ASM)                                                              \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, int iters, uint32_t s) {   \
        uint32_t v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ s,   \
                 v5 = v0 + s, v6 = v0 * 11, v7 = v0 * 13;                                 \
        const uint32_t k = s * 0x01010101u;                                               \
        for (int i = 0; i < iters; ++i) {                                                 \
            _Pragma("unroll") for (int r = 0; r < 4; ++r) {                                \
                asm volatile(ASM : "+v"(v0) : "v"(k));                                    \
                asm volatile(ASM : "+v"(v1) : "v"(k));                                    \
                asm volatile(ASM : "+v"(v2) : "v"(k));                                    \
                asm volatile(ASM : "+v"(v3) : "v"(k));                                    \
                asm volatile(ASM : "+v"(v4) : "v"(k));                                    \
                asm volatile(ASM : "+v"(v5) : "v"(k));                                    \
                asm volatile(ASM : "+v"(v6) : "v"(k));                                    \
                asm volatile(ASM : "+v"(v7) : "v"(k));                                    \
            }                                                                             \
        }                                                                                 \
        out[blockIdx.x * 256 + threadIdx.x] = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;      \
    }

OP_KERNEL(k_add_u32, "v_add_u32 %0, %0, %1")
OP_KERNEL(k_max_u32, "v_max_u32 %0, %0, %1")
OP_KERNEL(k_max3_u32, "v_max3_u32 %0, %0, %1, %0")
OP_KERNEL(k_pk_max_u16, "v_pk_max_u16 %0, %0, %1")
OP_KERNEL(k_pk_sub_u16, "v_pk_sub_u16 %0, %0, %1 clamp")
OP_KERNEL(k_pk_maximum3_f16, "v_pk_maximum3_f16 %0, %0, %1, %0")
OP_KERNEL(k_perm_b32, "v_perm_b32 %0, %0, %1, %1")
OP_KERNEL(k_alignbyte_b32, "v_alignbyte_b32 %0, %0, %1, 2")
OP_KERNEL(k_lerp_u8, "v_lerp_u8 %0, %0, %1, %1")
OP_KERNEL(k_bitop3_b32, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0xc8")
OP_KERNEL(k_dot4_u32_u8, "v_dot4_u32_u8 %0, %0, %1, %0")
OP_KERNEL(k_pk_mad_u16, "v_pk_mad_u16 %0, %0, %1, %0")
OP_KERNEL(k_mov_dpp, "v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf")
OP_KERNEL(k_mul_f32, "v_mul_f32 %0, %0, %1")
OP_KERNEL(k_mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %0")
OP_KERNEL(k_add3_u32, "v_add3_u32 %0, %0, %1, %0")
OP_KERNEL(k_sad_u8, "v_sad_u8 %0, %0, %1, %0")
OP_KERNEL(k_sub_u32, "v_sub_u32 %0, %0, %1")
OP_KERNEL(k_and_b32, "v_and_b32 %0, %0, %1")
OP_KERNEL(k_or_b32, "v_or_b32 %0, %0, %1")
OP_KERNEL(k_xor_b32, "v_xor_b32 %0, %0, %1")
OP_KERNEL(k_lshlrev_b32, "v_lshlrev_b32 %0, 1, %0")
OP_KERNEL(k_lshrrev_b32, "v_lshrrev_b32 %0, 1, %0")
OP_KERNEL(k_cndmask_b32, "v_cndmask_b32 %0, %0, %1, vcc")
OP_KERNEL(k_cmp_gt_u32, "v_cmp_gt_u32 vcc, %0, %1")
OP_KERNEL(k_max_i32, "v_max_i32 %0, %0, %1")
OP_KERNEL(k_min_u32, "v_min_u32 %0, %0, %1")
OP_KERNEL(k_max_f32, "v_max_f32 %0, %0, %1")
OP_KERNEL(k_add_f32, "v_add_f32 %0, %0, %1")
OP_KERNEL(k_fma_f32, "v_fma_f32 %0, %0, %1, %0")
OP_KERNEL(k_max3_f32, "v_max3_f32 %0, %0, %1, %0")
OP_KERNEL(k_med3_u32, "v_med3_u32 %0, %0, %1, %0")
OP_KERNEL(k_and_or_b32, "v_and_or_b32 %0, %0, %1, %0")
OP_KERNEL(k_or3_b32, "v_or3_b32 %0, %0, %1, %0")
OP_KERNEL(k_lshl_add_u32, "v_lshl_add_u32 %0, %0, 1, %1")
OP_KERNEL(k_lshl_or_b32, "v_lshl_or_b32 %0, %0, 1, %1")
OP_KERNEL(k_mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
OP_KERNEL(k_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
OP_KERNEL(k_bfe_u32, "v_bfe_u32 %0, %0, %1, 8")
OP_KERNEL(k_bcnt_u32, "v_bcnt_u32_b32 %0, %0, %1")
OP_KERNEL(k_cvt_f32_u32, "v_cvt_f32_u32 %0, %0")
OP_KERNEL(k_mov_b32, "v_mov_b32 %0, %1")
OP_KERNEL(k_add_dpp, "v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf")
OP_KERNEL(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")
OP_KERNEL(k_pk_max_f16, "v_pk_max_f16 %0, %0, %1")
OP_KERNEL(k_max_u16, "v_max_u16 %0, %0, %1")
OP_KERNEL(k_mul_hi_u32_u24, "v_mul_hi_u32_u24 %0, %0, %1")
OP_KERNEL(k_cvt_pk_u8_f32, "v_cvt_pk_u8_f32 %0, %1, 1, %0")
OP_KERNEL(k_readfirstlane, "v_mbcnt_lo_u32_b32 %0, %0, %1")

// 64-bit operands (register pairs): packed f32 and f64
#define OP_KERNEL64(NAME, ASM)                                                            \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, int iters, uint32_t s) {   \
        uint64_t v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 ^ s,   \
                 v5 = v0 + s, v6 = v0 * 11, v7 = v0 * 13;                                 \
        const uint64_t k = s * 0x0101010101010101ull;                                     \
        for (int i = 0; i < iters; ++i) {                                                 \
            _Pragma("unroll") for (int r = 0; r < 4; ++r) {                                \
                asm volatile(ASM : "+v"(v0) : "v"(k));                                    \
                asm volatile(ASM : "+v"(v1) : "v"(k));                                    \
                asm volatile(ASM : "+v"(v2) : "v"(k));                                    \
                asm volatile(ASM : "+v"(v3) : "v"(k));                                    \
                asm volatile(ASM : "+v"(v4) : "v"(k));                                    \
                asm volatile(ASM : "+v"(v5) : "v"(k));                                    \
                asm volatile(ASM : "+v"(v6) : "v"(k));                                    \
                asm volatile(ASM : "+v"(v7) : "v"(k));                                    \
            }                                                                             \
        }                                                                                 \
        out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7); \
    }
OP_KERNEL64(k_pk_mul_f32, "v_pk_mul_f32 %0, %0, %1")
OP_KERNEL64(k_pk_add_f32, "v_pk_add_f32 %0, %0, %1")
OP_KERNEL64(k_mul_f64, "v_mul_f64 %0, %0, %1")
OP_KERNEL64(k_pk_fma_f32, "v_pk_fma_f32 %0, %0, %1, %0")

typedef void (*kfn)(uint32_t*, int, uint32_t);

int main() {
    struct { const char* name; kfn f; } ks[] = {
        {"v_add_u32", k_add_u32}, {"v_max_u32", k_max_u32}, {"v_max3_u32", k_max3_u32},
        {"v_pk_max_u16", k_pk_max_u16}, {"v_pk_sub_u16 clamp", k_pk_sub_u16},
        {"v_pk_maximum3_f16", k_pk_maximum3_f16}, {"v_perm_b32", k_perm_b32},
        {"v_alignbyte_b32", k_alignbyte_b32}, {"v_lerp_u8", k_lerp_u8}, {"v_bitop3_b32", k_bitop3_b32},
        {"v_dot4_u32_u8", k_dot4_u32_u8}, {"v_pk_mad_u16", k_pk_mad_u16}, {"v_mov_b32_dpp wave_shr", k_mov_dpp},
        {"v_mul_f32", k_mul_f32}, {"v_mad_u32_u24", k_mad_u32_u24}, {"v_add3_u32", k_add3_u32},
        {"v_sad_u8", k_sad_u8}, {"v_pk_mul_f32", k_pk_mul_f32}, {"v_pk_add_f32", k_pk_add_f32},
        {"v_mul_f64", k_mul_f64}, {"v_pk_fma_f32", k_pk_fma_f32}, {"v_sub_u32", k_sub_u32}, {"v_and_b32", k_and_b32}, {"v_or_b32", k_or_b32}, {"v_xor_b32", k_xor_b32}, {"v_lshlrev_b32", k_lshlrev_b32}, {"v_lshrrev_b32", k_lshrrev_b32}, {"v_cndmask_b32", k_cndmask_b32}, {"v_cmp_gt_u32", k_cmp_gt_u32}, {"v_max_i32", k_max_i32}, {"v_min_u32", k_min_u32}, {"v_max_f32", k_max_f32}, {"v_add_f32", k_add_f32}, {"v_fma_f32", k_fma_f32}, {"v_max3_f32", k_max3_f32}, {"v_med3_u32", k_med3_u32}, {"v_and_or_b32", k_and_or_b32}, {"v_or3_b32", k_or3_b32}, {"v_lshl_add_u32", k_lshl_add_u32}, {"v_lshl_or_b32", k_lshl_or_b32}, {"v_mul_u32_u24", k_mul_u32_u24}, {"v_mul_lo_u32", k_mul_lo_u32}, {"v_bfe_u32", k_bfe_u32}, {"v_bcnt_u32_b32", k_bcnt_u32}, {"v_cvt_f32_u32", k_cvt_f32_u32}, {"v_mov_b32", k_mov_b32}, {"v_add_u32_dpp row_shr", k_add_dpp}, {"v_pk_add_u16", k_pk_add_u16}, {"v_pk_max_f16", k_pk_max_f16}, {"v_max_u16", k_max_u16}, {"v_mul_hi_u32_u24", k_mul_hi_u32_u24}, {"v_cvt_pk_u8_f32", k_cvt_pk_u8_f32}, {"v_mbcnt_lo_u32_b32", k_readfirstlane}};
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const int blocks = cus * 8;  // 8 blocks of 4 waves per CU = 8 waves per SIMD
    const int iters = 4000;
    uint32_t* out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    printf("{\"cus\": %d, \"waves_per_simd\": 8, \"rows\": [\n", cus);
    for (size_t i = 0; i < sizeof(ks) / sizeof(ks[0]); ++i) {
        hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(256), 0, 0, out, 10, 3u);
        hipDeviceSynchronize();
        hipEventRecord(a, 0);
        hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(256), 0, 0, out, iters, 3u);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        // wave-instructions per SIMD: 8 waves x iters x 32
        const double per_simd = 8.0 * iters * 32;
        const double ns_per = ms * 1e6 / per_simd;
        printf("  {\"op\": \"%s\", \"ms\": %.3f, \"ns_per_wave_instr_per_simd\": %.4f}%s\n", ks[i].name, ms, ns_per,
               i + 1 < sizeof(ks) / sizeof(ks[0]) ? "," : "");
    }
    printf("]}\n");
    hipFree(out);
    return 0;
}
