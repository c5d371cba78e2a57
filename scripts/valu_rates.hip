// valu_rates.hip — throughput of the VALU instructions the composite and multi-band kernels issue
// (gfx950): every CU full of waves (8 per SIMD), 8 independent chains per lane, one opcode per run.
// Prints cycles per wave-instruction per SIMD, using s_memtime (shader clock) read in-kernel.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/valu_rates.hip -o /tmp/valu_rates
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                         \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

constexpr int kIters = 4096;

// OP: asm template over one register %0 (in/out) and two read-only operands %1 %2
#define BODY8(ASM)                                                                                   \
    asm volatile(ASM : "+v"(r0) : "v"(a), "v"(b));                                                  \
    asm volatile(ASM : "+v"(r1) : "v"(a), "v"(b));                                                  \
    asm volatile(ASM : "+v"(r2) : "v"(a), "v"(b));                                                  \
    asm volatile(ASM : "+v"(r3) : "v"(a), "v"(b));                                                  \
    asm volatile(ASM : "+v"(r4) : "v"(a), "v"(b));                                                  \
    asm volatile(ASM : "+v"(r5) : "v"(a), "v"(b));                                                  \
    asm volatile(ASM : "+v"(r6) : "v"(a), "v"(b));                                                  \
    asm volatile(ASM : "+v"(r7) : "v"(a), "v"(b));

#define KERNEL(NAME, ASM)                                                                            \
    __global__ void __launch_bounds__(256) NAME(unsigned* out, unsigned long long* clk, unsigned s) { \
        unsigned r0 = s + threadIdx.x, r1 = r0 * 3, r2 = r0 * 5, r3 = r0 * 7, r4 = r0 ^ 9, r5 = r0 + 11, \
                 r6 = r0 * 13, r7 = r0 ^ 15;                                                         \
        unsigned a = s * 17 + threadIdx.x, b = s ^ 0x1234567u;                                       \
        asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cmp_gt_u32 s[20:21], %1, %0" :: "v"(a), "v"(r3) : "vcc", "s20", "s21");                                 \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                  \
        for (int i = 0; i < kIters; i++) { BODY8(ASM) }                                              \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                  \
        out[blockIdx.x * 256 + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;                 \
        if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;                                             \
    }

KERNEL(k_add_u32, "v_add_u32 %0, %0, %1")
KERNEL(k_fma_f32, "v_fma_f32 %0, %0, %1, %2")
KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %2")
KERNEL(k_dot2_u16, "v_dot2_u32_u16 %0, %1, %2, %0")
KERNEL(k_cvt_pk_u8, "v_cvt_pk_u8_f32 %0, %1, 1, %0")
KERNEL(k_cvt_f32_u32, "v_cvt_f32_u32 %0, %0")
KERNEL(k_rndne, "v_rndne_f32 %0, %0")
KERNEL(k_med3, "v_med3_f32 %0, %0, %1, %2")
KERNEL(k_mul_u24, "v_mul_u32_u24 %0, %0, %1")
KERNEL(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %2")
KERNEL(k_bfe, "v_bfe_u32 %0, %0, 15, 5")
KERNEL(k_sdwa, "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD")
KERNEL(k_cvt_ubyte, "v_cvt_f32_ubyte1 %0, %0")
KERNEL(k_pk_mad_u16, "v_pk_mad_u16 %0, %0, %1, %2")
KERNEL(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
KERNEL(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %0, 3, %1")
KERNEL(k_dot4_u8, "v_dot4_u32_u8 %0, %1, %2, %0")
KERNEL(k_sad_u8, "v_sad_u8 %0, %1, %2, %0")
KERNEL(k_mul_f32, "v_mul_f32 %0, %0, %1")
KERNEL(k_cvt_i32_f32, "v_cvt_i32_f32 %0, %0")

KERNEL(k_cnd_e32, "v_cndmask_b32_e32 %0, %0, %1, vcc")
KERNEL(k_lshr, "v_lshrrev_b32 %0, 3, %0")
KERNEL(k_lshl, "v_lshlrev_b32 %0, 3, %0")
KERNEL(k_and, "v_and_b32 %0, %0, %1")
KERNEL(k_or, "v_or_b32 %0, %0, %1")
KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
KERNEL(k_sub_u32, "v_sub_u32 %0, %0, %1")
KERNEL(k_mov, "v_mov_b32 %0, %1")
KERNEL(k_add_f32, "v_add_f32 %0, %0, %1")
KERNEL(k_sub_f32, "v_sub_f32 %0, %0, %1")
KERNEL(k_fmac, "v_fmac_f32 %0, %1, %2")
KERNEL(k_max_f32, "v_max_f32 %0, %0, %1")
KERNEL(k_min_i32, "v_min_i32 %0, %0, %1")
KERNEL(k_max_u32, "v_max_u32 %0, %0, %1")
KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %2")
KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %0, 8, %1")
KERNEL(k_or3, "v_or3_b32 %0, %0, %1, %2")
KERNEL(k_alignbyte, "v_alignbyte_b32 %0, %0, %1, 1")
KERNEL(k_bfi, "v_bfi_b32 %0, %0, %1, %2")
KERNEL(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
KERNEL(k_mul_hi_u24, "v_mul_hi_u32_u24 %0, %0, %1")
KERNEL(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")
KERNEL(k_pk_mul_lo_u16, "v_pk_mul_lo_u16 %0, %0, %1")
KERNEL(k_pk_fma_f16, "v_pk_fma_f16 %0, %0, %1, %2")
KERNEL(k_dot2_f32_f16, "v_dot2_f32_f16 %0, %1, %2, %0")
KERNEL(k_dot2c_f32_f16, "v_dot2c_f32_f16 %0, %1, %2")
KERNEL(k_cvt_f32_ubyte0, "v_cvt_f32_ubyte0 %0, %0")
KERNEL(k_cvt_u32_f32, "v_cvt_u32_f32 %0, %0")
KERNEL(k_mad_u16, "v_mad_u16 %0, %0, %1, %2")
KERNEL(k_min3_f32, "v_min3_f32 %0, %0, %1, %2")
KERNEL(k_fma_mix, "v_fma_mix_f32 %0, %0, %1, %2 op_sel_hi:[0,0,0]")
KERNEL(k_cvt_pkrtz, "v_cvt_pkrtz_f16_f32 %0, %0, %1")
KERNEL(k_mac_legacy, "v_mul_legacy_f32 %0, %0, %1")
KERNEL(k_readlane_like, "v_mbcnt_lo_u32_b32 %0, %1, %0")
KERNEL(k_sad_u16, "v_sad_u16 %0, %1, %2, %0")
KERNEL(k_msad, "v_msad_u8 %0, %1, %2, %0")
KERNEL(k_lerp, "v_lerp_u8 %0, %1, %2, %0")
KERNEL(k_cvt_f16_u16, "v_cvt_f16_u16 %0, %0")
KERNEL(k_add_u16, "v_add_u16 %0, %0, %1")
KERNEL(k_mul_u16, "v_mul_lo_u16 %0, %0, %1")
KERNEL(k_fma_f16, "v_fma_f16 %0, %0, %1, %2")
KERNEL(k_mul_f16, "v_mul_f16 %0, %0, %1")
KERNEL(k_pk_max_u16, "v_pk_max_u16 %0, %0, %1")
KERNEL(k_xad, "v_xad_u32 %0, %0, %1, %2")
KERNEL(k_add_co, "v_add_co_u32 %0, vcc, %0, %1")

KERNEL(k_cnd_sgpr, "v_cndmask_b32_e64 %0, %0, %1, s[20:21]")
KERNEL(k_cnd_mix3, "v_cndmask_b32_e32 %0, %0, %1, vcc\n\tv_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %2\n\tv_xor_b32 %0, %0, %1")
KERNEL(k_add_mix4, "v_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %2\n\tv_xor_b32 %0, %0, %1")
KERNEL(k_cmp_cnd, "v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32_e32 %0, %0, %2, vcc")
KERNEL(k_cmp_only, "v_cmp_gt_u32 vcc, %0, %1\n\tv_add_u32 %0, %0, %2")
KERNEL(k_perm_mix, "v_perm_b32 %0, %0, %1, %2\n\tv_add_u32 %0, %0, %1")
KERNEL(k_bfe_vop2, "v_lshrrev_b32 %0, 15, %0\n\tv_and_b32 %0, 31, %0")

// 64-bit packed-f32 ops need register pairs
#define KERNEL64(NAME, ASM)                                                                           \
    __global__ void __launch_bounds__(256) NAME(unsigned* out, unsigned long long* clk, unsigned s) { \
        typedef float f2 __attribute__((ext_vector_type(2)));                                         \
        f2 r[8];                                                                                      \
        for (int k = 0; k < 8; k++) r[k] = f2{(float)(s + threadIdx.x + k), (float)k};               \
        f2 a = {1.0001f, 0.9999f}, b = {0.5f, 0.25f};                                                 \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                   \
        for (int i = 0; i < kIters; i++) {                                                            \
            _Pragma("unroll") for (int k = 0; k < 8; k++) asm volatile(ASM : "+v"(r[k]) : "v"(a), "v"(b)); \
        }                                                                                             \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                   \
        float x = 0;                                                                                  \
        for (int k = 0; k < 8; k++) x += r[k].x + r[k].y;                                             \
        out[blockIdx.x * 256 + threadIdx.x] = (unsigned)x;                                            \
        if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;                                              \
    }
KERNEL64(k_pk_fma_f32, "v_pk_fma_f32 %0, %0, %1, %2")
KERNEL64(k_pk_mul_f32, "v_pk_mul_f32 %0, %0, %1")
KERNEL64(k_pk_add_f32, "v_pk_add_f32 %0, %0, %1")

typedef void (*kfn)(unsigned*, unsigned long long*, unsigned);
struct K {
    const char* name;
    kfn f;
};

int main() {
    const K ks[] = {{"v_add_u32", k_add_u32},     {"v_fma_f32", k_fma_f32},       {"v_mul_f32", k_mul_f32},
                    {"v_perm_b32", k_perm},       {"v_dot2_u32_u16", k_dot2_u16}, {"v_cvt_pk_u8_f32", k_cvt_pk_u8},
                    {"v_cvt_f32_u32", k_cvt_f32_u32}, {"v_cvt_i32_f32", k_cvt_i32_f32}, {"v_rndne_f32", k_rndne},
                    {"v_med3_f32", k_med3},       {"v_mul_u32_u24", k_mul_u24},   {"v_mad_u32_u24", k_mad_u24},
                    {"v_bfe_u32", k_bfe},         {"v_add_u32_sdwa", k_sdwa},     {"v_cvt_f32_ubyte1", k_cvt_ubyte},
                    {"v_pk_mad_u16", k_pk_mad_u16}, {"v_cndmask_b32", k_cndmask}, {"v_and_or_b32", k_and_or},
                    {"v_lshl_add_u32", k_lshl_add}, {"v_dot4_u32_u8", k_dot4_u8}, {"v_sad_u8", k_sad_u8},
                    {"v_pk_fma_f32", k_pk_fma_f32}, {"v_pk_mul_f32", k_pk_mul_f32}, {"v_pk_add_f32", k_pk_add_f32}, {"v_cndmask_b32_e32", k_cnd_e32}, {"v_lshrrev_b32", k_lshr}, {"v_lshlrev_b32", k_lshl}, {"v_and_b32", k_and}, {"v_or_b32", k_or}, {"v_xor_b32", k_xor}, {"v_sub_u32", k_sub_u32}, {"v_mov_b32", k_mov}, {"v_add_f32", k_add_f32}, {"v_sub_f32", k_sub_f32}, {"v_fmac_f32", k_fmac}, {"v_max_f32", k_max_f32}, {"v_min_i32", k_min_i32}, {"v_max_u32", k_max_u32}, {"v_add3_u32", k_add3}, {"v_lshl_or_b32", k_lshl_or}, {"v_or3_b32", k_or3}, {"v_alignbyte_b32", k_alignbyte}, {"v_bfi_b32", k_bfi}, {"v_mul_lo_u32", k_mul_lo}, {"v_mul_hi_u32_u24", k_mul_hi_u24}, {"v_pk_add_u16", k_pk_add_u16}, {"v_pk_mul_lo_u16", k_pk_mul_lo_u16}, {"v_pk_fma_f16", k_pk_fma_f16}, {"v_dot2_f32_f16", k_dot2_f32_f16}, {"v_dot2c_f32_f16", k_dot2c_f32_f16}, {"v_cvt_f32_ubyte0", k_cvt_f32_ubyte0}, {"v_cvt_u32_f32", k_cvt_u32_f32}, {"v_mad_u16", k_mad_u16}, {"v_min3_f32", k_min3_f32}, {"v_fma_mix_f32", k_fma_mix}, {"v_cvt_pkrtz_f16_f32", k_cvt_pkrtz}, {"v_mul_legacy_f32", k_mac_legacy}, {"v_mbcnt_lo_u32_b32", k_readlane_like}, {"v_sad_u16", k_sad_u16}, {"v_msad_u8", k_msad}, {"v_lerp_u8", k_lerp}, {"v_cvt_f16_u16", k_cvt_f16_u16}, {"v_add_u16", k_add_u16}, {"v_mul_lo_u16", k_mul_u16}, {"v_fma_f16", k_fma_f16}, {"v_mul_f16", k_mul_f16}, {"v_pk_max_u16", k_pk_max_u16}, {"v_xad_u32", k_xad}, {"v_add_co_u32", k_add_co}, {"k_cnd_sgpr", k_cnd_sgpr}, {"k_cnd_mix3", k_cnd_mix3}, {"k_add_mix4", k_add_mix4}, {"k_cmp_cnd", k_cmp_cnd}, {"k_cmp_only", k_cmp_only}, {"k_perm_mix", k_perm_mix}, {"k_bfe_vop2", k_bfe_vop2}};
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    for (int waves_per_simd : {8, 1}) {
        const int blocks = cus * waves_per_simd;  // 4 waves per block = one per SIMD
        unsigned* out;
        unsigned long long* clk;
        CHK(hipMalloc(&out, (size_t)blocks * 256 * 4));
        CHK(hipMalloc(&clk, (size_t)blocks * 8));
        unsigned long long* h = (unsigned long long*)malloc((size_t)blocks * 8);
        printf("waves per SIMD %d (%d CUs)\n", waves_per_simd, cus);
        for (const K& k : ks) {
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, clk, 1u);  // warm
            CHK(hipDeviceSynchronize());
            hipEvent_t e0, e1;
            CHK(hipEventCreate(&e0));
            CHK(hipEventCreate(&e1));
            CHK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, clk, 2u);
            CHK(hipEventRecord(e1, 0));
            CHK(hipEventSynchronize(e1));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            CHK(hipMemcpy(h, clk, (size_t)blocks * 8, hipMemcpyDeviceToHost));
            double mean = 0;
            for (int i = 0; i < blocks; i++) mean += (double)h[i];
            mean /= blocks;
            // per SIMD: waves_per_simd waves, each kIters * 8 instructions, over `mean` shader cycles
            // (s_memtime ticks at the shader clock)
            const double per = mean / ((double)kIters * 8 * waves_per_simd);
            printf("  %-20s %7.3f cyc/wave-instr/SIMD  (kernel %.3f ms, %.0f cycles per wave)\n", k.name, per, ms, mean);
            CHK(hipEventDestroy(e0));
            CHK(hipEventDestroy(e1));
        }
        CHK(hipFree(out));
        CHK(hipFree(clk));
        free(h);
    }
    return 0;
}
