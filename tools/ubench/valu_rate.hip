// Microbenchmark (diagnostic, not product code): issue cost of the VALU
// instructions the PNG and JPEG kernels use, on gfx950, for 1, 2 and 4 waves per SIMD.
// Each wave runs 8 independent chains of one instruction; cycles per
// instruction per wave from s_memtime.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHAINS(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

#define DEF_KERNEL(NAME, ASM)                                                            \
    __global__ void NAME(uint32_t *out, uint64_t *cyc, int iters)                       \
    {                                                                                    \
        uint32_t v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 + 11, \
                 v5 = v0 + 13, v6 = v0 ^ 17, v7 = v0 ^ 19, k = blockIdx.x | 0x01030507u; \
        uint64_t t0 = __builtin_amdgcn_s_memtime();                                      \
        for (int i = 0; i < iters; i++) {                                                \
            _Pragma("unroll") for (int r = 0; r < 8; r++) {                              \
                _Pragma("unroll") for (int q = 0; q < 1; q++) {                          \
                    asm volatile(ASM : "+v"(v0) : "v"(k));                               \
                    asm volatile(ASM : "+v"(v1) : "v"(k));                               \
                    asm volatile(ASM : "+v"(v2) : "v"(k));                               \
                    asm volatile(ASM : "+v"(v3) : "v"(k));                               \
                    asm volatile(ASM : "+v"(v4) : "v"(k));                               \
                    asm volatile(ASM : "+v"(v5) : "v"(k));                               \
                    asm volatile(ASM : "+v"(v6) : "v"(k));                               \
                    asm volatile(ASM : "+v"(v7) : "v"(k));                               \
                }                                                                        \
            }                                                                            \
        }                                                                                \
        uint64_t t1 = __builtin_amdgcn_s_memtime();                                      \
        out[blockIdx.x * 64 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;      \
        if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                 \
    }

DEF_KERNEL(k_add, "v_add_u32 %0, %0, %1")
DEF_KERNEL(k_pk_add, "v_pk_add_u16 %0, %0, %1")
DEF_KERNEL(k_pk_min, "v_pk_min_u16 %0, %0, %1")
DEF_KERNEL(k_pk_sub, "v_pk_sub_i16 %0, %0, %1")
DEF_KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %1")
DEF_KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %0, 7, %1")
DEF_KERNEL(k_and_or, "v_and_or_b32 %0, %0, %1, %1")
DEF_KERNEL(k_alignbit, "v_alignbit_b32 %0, %0, %1, 16")
DEF_KERNEL(k_sad, "v_sad_u16 %0, %0, %1, %1")
DEF_KERNEL(k_min3, "v_min3_u32 %0, %0, %1, %1")
DEF_KERNEL(k_bfe, "v_bfe_u32 %0, %0, %1, 8")
DEF_KERNEL(k_dpp_wshr, "v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf")
DEF_KERNEL(k_dpp_rshr, "v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf")
DEF_KERNEL(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
DEF_KERNEL(k_mad24, "v_mad_i32_i24 %0, %0, %1, %1")
DEF_KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %0, 4, %1")
DEF_KERNEL(k_dot2, "v_dot2_i32_i16 %0, %0, %1, 0")
DEF_KERNEL(k_pk_mul, "v_pk_mul_lo_u16 %0, %0, %1")
DEF_KERNEL(k_med3, "v_med3_i32 %0, %0, %1, %1")
DEF_KERNEL(k_dpp_add_wshr, "v_add_u32_dpp %0, %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf")
// encoding size against operation: the same add as VOP3 (8 bytes), VOP2 with
// a literal (8 bytes), VOP2 with an inline constant; a VOP1; a VOP2 shift
DEF_KERNEL(k_add_e64, "v_add_u32_e64 %0, %0, %1")
DEF_KERNEL(k_add_lit, "v_add_u32_e32 %0, 0x1234, %0")
DEF_KERNEL(k_add_inl, "v_add_u32_e32 %0, 7, %0")
DEF_KERNEL(k_sat_pk, "v_sat_pk_u8_i16 %0, %0")
DEF_KERNEL(k_ashr, "v_ashrrev_i32_e32 %0, 3, %0")
DEF_KERNEL(k_mul24_e32, "v_mul_i32_i24_e32 %0, %1, %0")
DEF_KERNEL(k_mul24_lit, "v_mul_i32_i24_e32 %0, 0x968, %0")

typedef void (*KFn)(uint32_t *, uint64_t *, int);
int main()
{
    struct T { const char *name; KFn f; } tests[] = {
        {"v_add_u32", k_add}, {"v_pk_add_u16", k_pk_add}, {"v_pk_min_u16", k_pk_min}, {"v_pk_sub_i16", k_pk_sub},
        {"v_perm_b32", k_perm}, {"v_lshl_or_b32", k_lshl_or}, {"v_and_or_b32", k_and_or},
        {"v_alignbit_b32", k_alignbit}, {"v_sad_u16", k_sad}, {"v_min3_u32", k_min3}, {"v_bfe_u32", k_bfe},
        {"v_mov_dpp wave_shr:1", k_dpp_wshr}, {"v_mov_dpp row_shr:1", k_dpp_rshr},
        {"v_add_dpp wave_shr:1", k_dpp_add_wshr}, {"v_mul_lo_u32", k_mul_lo}, {"v_mad_i32_i24", k_mad24},
        {"v_lshl_add_u32", k_lshl_add}, {"v_dot2_i32_i16", k_dot2}, {"v_pk_mul_lo_u16", k_pk_mul}, {"v_med3_i32", k_med3},
        {"v_add_u32_e64 (VOP3)", k_add_e64}, {"v_add_u32 literal", k_add_lit}, {"v_add_u32 inline", k_add_inl},
        {"v_sat_pk_u8_i16 (VOP1)", k_sat_pk}, {"v_ashrrev_i32 (VOP2)", k_ashr}, {"v_mul_i32_i24_e32", k_mul24_e32},
        {"v_mul_i32_i24 literal", k_mul24_lit}};
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 2000;
    uint32_t *out;
    uint64_t *cyc;
    hipMalloc(&out, 64 * 64 * cus * sizeof(uint32_t));
    hipMalloc(&cyc, 64 * cus * sizeof(uint64_t));
    printf("instruction, cycles/instr/wave at 1 wave/SIMD (4/CU), 2 waves/SIMD (8/CU), 4 waves/SIMD (16/CU)\n");
    for (auto &t : tests) {
        printf("%-24s", t.name);
        for (int per_cu : {4, 8, 16}) {
            const int blocks = per_cu * cus;
            hipLaunchKernelGGL(t.f, dim3(blocks), dim3(64), 0, 0, out, cyc, 10);
            hipLaunchKernelGGL(t.f, dim3(blocks), dim3(64), 0, 0, out, cyc, iters);
            hipDeviceSynchronize();
            std::vector<uint64_t> h(blocks);
            hipMemcpy(h.data(), cyc, blocks * sizeof(uint64_t), hipMemcpyDeviceToHost);
            double s = 0;
            for (auto c : h) s += double(c);
            printf("  %6.2f", s / blocks / (double(iters) * 64));
        }
        printf("\n");
    }
    return 0;
}
