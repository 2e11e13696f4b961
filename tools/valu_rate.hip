// Microbenchmark: issue cost of individual wave64 VALU instructions on gfx950
// (16 independent accumulators per lane, 4 / 16 waves per SIMD).  Calibrates
// the aligner's instruction budget; not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int OP>
__global__ __launch_bounds__(256) void k(int32_t *out, int32_t n, int32_t s0) {
    int32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
            a7 = a0 + 7, a8 = a0 + 8, a9 = a0 + 9, a10 = a0 + 10, a11 = a0 + 11, a12 = a0 + 12, a13 = a0 + 13,
            a14 = a0 + 14, a15 = a0 + 15;
    int32_t b = threadIdx.x * 3, c = threadIdx.x * 5;
    asm volatile("v_cmp_gt_i32 vcc, %0, %1" : : "v"(a0), "v"(b) : "vcc");
    for (int it = 0; it < n; ++it) {
#define ST(i) \
    if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 1) asm volatile("v_max_i32 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 2) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##i) : "v"(b) : "vcc"); \
    if (OP == 3) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a##i) : "v"(b)); \
    if (OP == 4) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(a##i) : "v"(b)); \
    if (OP == 5) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 6) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 7) asm volatile("v_max_u16 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 8) asm volatile("v_add_u16 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 9) asm volatile("v_sub_u16 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 10) asm volatile("v_cmp_eq_u16_e64 s[4:5], %0, %1" : : "v"(a##i), "v"(b) : "s4", "s5"); \
    if (OP == 11) asm volatile("v_cmp_eq_u32_e64 s[4:5], %0, %1" : : "v"(a##i), "v"(b) : "s4", "s5"); \
    if (OP == 12) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c)); \
    if (OP == 13) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c)); \
    if (OP == 14) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 15) asm volatile("v_sub_u32_e64 %0, %0, %1 clamp" : "+v"(a##i) : "v"(b)); \
    if (OP == 16) asm volatile("v_add_u32_e64 %0, %0, %1 clamp" : "+v"(a##i) : "v"(b)); \
    if (OP == 17) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c)); \
    if (OP == 18) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c)); \
    if (OP == 19) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c)); \
    if (OP == 20) asm volatile("v_max_i32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a##i) : "v"(b)); \
    if (OP == 21) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a##i) : "v"(b)); \
    if (OP == 22) asm volatile("v_add_u32 %0, 7, %0" : "+v"(a##i) : "v"(b)); \
    if (OP == 23) asm volatile("v_max_i32 %0, 0, %0" : "+v"(a##i) : "v"(b)); \
    if (OP == 24) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 25) asm volatile("v_max_u16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(a##i) : "v"(b)); \
    if (OP == 26) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a##i) : "v"(b) : "vcc"); \
    if (OP == 27) asm volatile("v_sub_i32 %0, %0, %1 clamp" : "+v"(a##i) : "v"(b)); \
    if (OP == 28) asm volatile("v_add_i32 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 29) asm volatile("v_ashrrev_i32 %0, %1, %0" : "+v"(a##i) : "v"(b)); \
    if (OP == 30) asm volatile("v_pk_sub_u16 %0, %0, %1 clamp" : "+v"(a##i) : "v"(b)); \
    if (OP == 31) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 32) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 33) asm volatile("v_pk_sub_i16 %0, 0, %0" : "+v"(a##i)); \
    if (OP == 34) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe4" : "+v"(a##i) : "v"(b), "v"(c)); \
    if (OP == 35) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a0) : "v"(b)); \
    if (OP == 36) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a0) : "v"(b)); \
    if (OP == 37) asm volatile("v_pk_max_u16 %0, %0, %1\n s_nop 0" : "+v"(a##i) : "v"(b)); \
    if (OP == 38) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c)); \
    if (OP == 39) asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c)); \
    if (OP == 40) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c)); \
    if (OP == 41) asm volatile("v_lshl_or_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c)); \
    if (OP == 42) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 43) asm volatile("v_pk_mul_lo_u16 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 44) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 45) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 46) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 47) asm volatile("v_min_i32 %0, %0, %1" : "+v"(a##i) : "v"(b)); \
    if (OP == 48) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##i) : "v"(b));
        R16(ST)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] =
        a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ a8 ^ a9 ^ a10 ^ a11 ^ a12 ^ a13 ^ a14 ^ a15;
}

template <int OP>
void run(int32_t *out, int blocks, int n) { hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, n, 3); }

static const char *NAMES[] = {"v_add_u32 vv", "v_max_i32 vv", "v_cndmask vcc (set)", "v_lshlrev_b32", "v_lshrrev_b32", "v_or_b32", "v_xor_b32", "v_max_u16", "v_add_u16", "v_sub_u16", "v_cmp_eq_u16 e64", "v_cmp_eq_u32 e64", "v_perm_b32", "v_mad_u32_u24", "v_mul_u32_u24", "v_sub_u32 clamp", "v_add_u32 clamp", "v_and_or_b32", "v_or3_b32", "v_bfi_b32", "v_max_i32 dpp", "v_mov_b32 dpp", "v_add_u32 inline", "v_max_i32 inline", "v_pk_max_u16", "v_max_u16 sdwa hi", "v_cndmask_b32 e64 vcc", "v_sub_i32 clamp", "v_add_i32", "v_ashrrev_i32", "v_pk_sub_u16 clamp", "v_pk_add_u16", "v_pk_min_u16", "v_pk_sub_i16 0-x", "v_bitop3_b32", "v_pk_max_u16 DEP", "v_max_u32 DEP", "v_pk_max_u16+s_nop0", "v_max3_u32", "v_med3_u32", "v_add3_u32", "v_lshl_or_b32", "v_pk_max_i16", "v_pk_mul_lo_u16", "v_max_u32", "v_sub_u32", "v_and_b32", "v_min_i32", "v_add_u32 (again)"};

int main() {
    int32_t *out;
    (void)hipMalloc(&out, 256 * 4096 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int n = 20000;
    void (*fns[])(int32_t *, int, int) = {run<0>, run<1>, run<2>, run<3>, run<4>, run<5>, run<6>, run<7>, run<8>, run<9>, run<10>, run<11>, run<12>, run<13>, run<14>, run<15>, run<16>, run<17>, run<18>, run<19>, run<20>, run<21>, run<22>, run<23>, run<24>, run<25>, run<26>, run<27>, run<28>, run<29>, run<30>, run<31>, run<32>, run<33>, run<34>, run<35>, run<36>, run<37>, run<38>, run<39>, run<40>, run<41>, run<42>, run<43>, run<44>, run<45>, run<46>, run<47>, run<48>};
    for (int op = 0; op < 49; ++op) {
        for (int blocks : {4096}) {
            fns[op](out, blocks, n);
            (void)hipEventRecord(e0);
            fns[op](out, blocks, n);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double winst = blocks * 4.0 * n * 16.0;
            printf("%-22s waves/SIMD %4.1f  %8.3f ms  %.2f cycles/wave-inst/SIMD @2.4GHz\n", NAMES[op],
                   blocks * 4.0 / 1024.0, ms, 1024.0 * 2.4e9 * (ms * 1e-3) / winst);
        }
    }
    return 0;
}
