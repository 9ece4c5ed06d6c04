// valu_rate.hip -- issue cost of the integer VALU instructions the SRTP
// kernels are built from, on MI355X: 8 independent accumulators per lane,
// 16 waves per CU, inline asm so the instruction is exactly the one named.
// Prints cycles per wave-instruction per SIMD (clock from s_memtime).
// Timing only.  hipcc -O3 --offload-arch=gfx950 tools/valu_rate.hip -o tools/valu_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define R8(OP)                                                                 \
    asm volatile(OP " %0, %0, %8, %9\n\t" OP " %1, %1, %8, %9\n\t"             \
                 OP " %2, %2, %8, %9\n\t" OP " %3, %3, %8, %9\n\t"             \
                 OP " %4, %4, %8, %9\n\t" OP " %5, %5, %8, %9\n\t"             \
                 OP " %6, %6, %8, %9\n\t" OP " %7, %7, %8, %9"                 \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), \
                   "+v"(a6), "+v"(a7)                                          \
                 : "v"(x), "v"(y))
#define R8S(OP, SFX)                                                           \
    asm volatile(OP " %0, %0, %8, %9 " SFX "\n\t" OP " %1, %1, %8, %9 " SFX "\n\t" \
                 OP " %2, %2, %8, %9 " SFX "\n\t" OP " %3, %3, %8, %9 " SFX "\n\t" \
                 OP " %4, %4, %8, %9 " SFX "\n\t" OP " %5, %5, %8, %9 " SFX "\n\t" \
                 OP " %6, %6, %8, %9 " SFX "\n\t" OP " %7, %7, %8, %9 " SFX      \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), \
                   "+v"(a6), "+v"(a7)                                          \
                 : "v"(x), "v"(y))
#define R8_2(OP)                                                               \
    asm volatile(OP " %0, %0, %8\n\t" OP " %1, %1, %8\n\t"                     \
                 OP " %2, %2, %8\n\t" OP " %3, %3, %8\n\t"                     \
                 OP " %4, %4, %8\n\t" OP " %5, %5, %8\n\t"                     \
                 OP " %6, %6, %8\n\t" OP " %7, %7, %8"                         \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), \
                   "+v"(a6), "+v"(a7)                                          \
                 : "v"(x))
#define R8_2S(OP, SFX)                                                         \
    asm volatile(OP " %0, %0, %8 " SFX "\n\t" OP " %1, %1, %8 " SFX "\n\t"     \
                 OP " %2, %2, %8 " SFX "\n\t" OP " %3, %3, %8 " SFX "\n\t"     \
                 OP " %4, %4, %8 " SFX "\n\t" OP " %5, %5, %8 " SFX "\n\t"     \
                 OP " %6, %6, %8 " SFX "\n\t" OP " %7, %7, %8 " SFX            \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), \
                   "+v"(a6), "+v"(a7)                                          \
                 : "v"(x))
#define R8_1(OP, S)                                                            \
    asm volatile(OP " %0, %0 " S "\n\t" OP " %1, %1 " S "\n\t"                 \
                 OP " %2, %2 " S "\n\t" OP " %3, %3 " S "\n\t"                 \
                 OP " %4, %4 " S "\n\t" OP " %5, %5 " S "\n\t"                 \
                 OP " %6, %6 " S "\n\t" OP " %7, %7 " S                        \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), \
                   "+v"(a6), "+v"(a7))

template <int K>
__global__ __launch_bounds__(1024) void k_rate(uint32_t *out, int iters,
                                               uint64_t *clk)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3,
             a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = blockIdx.x | 0x10203, y = 0x05040100;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            if (K == 0) R8_2("v_xor_b32");
            if (K == 1) R8_2("v_add_u32");
            if (K == 2) R8("v_perm_b32");
            if (K == 3) R8S("v_bitop3_b32", "bitop3:0x96");
            if (K == 4) R8("v_add3_u32");
            if (K == 5) R8("v_alignbit_b32");
            if (K == 6) R8_2("v_or_b32");
            if (K == 7) R8("v_lshl_or_b32");
            if (K == 8) R8("v_and_or_b32");
            if (K == 9) R8_1("v_mov_b32_dpp", "quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf");
            if (K == 10) R8("v_or3_b32");
            if (K == 11) R8_2("v_lshlrev_b32");
            if (K == 12) R8("v_xad_u32");
            if (K == 13) R8("v_lshl_add_u32");
            if (K == 14) R8_2("v_and_b32");
            if (K == 15) R8("v_bfi_b32");
            if (K == 16) R8_2("v_xor_b32_e64");
            if (K == 18) R8_2("v_sub_u32");
            if (K == 19) R8_1("v_mov_b32_sdwa", "dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2");
            if (K == 20) R8_1("v_mov_b32_sdwa", "dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0");
            if (K == 21) R8_1("v_permlane32_swap_b32", "");
            if (K == 22) R8_1("v_permlane16_swap_b32", "");
            if (K == 23) R8("v_bfe_u32");
            if (K == 24) R8_1("v_mov_b32_dpp", "row_shr:1 row_mask:0xf bank_mask:0xf");
            if (K == 25) R8_2("v_xor_b32_dpp");
            // packed 16-bit and 24-bit forms (round 5: byte moves at full rate?)
            if (K == 26) R8("v_pk_mad_u16");
            if (K == 27) R8_2S("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]");
            if (K == 28) R8_2("v_pk_lshlrev_b16");
            if (K == 29) R8_2("v_lshrrev_b32");
            if (K == 30) R8("v_mad_u32_u24");
            if (K == 31) R8("v_dot4_u32_u8");
            if (K == 32) R8("v_alignbyte_b32");
            if (K == 33) R8_2("v_pk_mul_lo_u16");
            if (K == 34) R8S("v_pk_mad_u16", "op_sel:[1,0,0] op_sel_hi:[0,1,1]");
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] =
        a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0)
        clk[blockIdx.x] = t1 - t0;
}

static const char *NAMES[] = { "v_xor_b32", "v_add_u32", "v_perm_b32",
                               "v_bitop3_b32", "v_add3_u32", "v_alignbit_b32",
                               "v_or_b32", "v_lshl_or_b32", "v_and_or_b32",
                               "v_mov_b32_dpp", "v_or3_b32", "v_lshlrev_b32",
                               "v_xad_u32", "v_lshl_add_u32", "v_and_b32",
                               "v_bfi_b32", "v_xor_b32_e64", "unused",
                               "v_sub_u32", "sdwa mov b2->b1", "sdwa mov b0->b1",
                               "permlane32_swap", "permlane16_swap", "v_bfe_u32",
                               "dpp row_shr", "v_xor_b32_dpp", "v_pk_mad_u16",
                               "pk_add_u16 swap", "v_pk_lshlrev_b16",
                               "v_lshrrev_b32", "v_mad_u32_u24",
                               "v_dot4_u32_u8", "v_alignbyte_b32",
                               "v_pk_mul_lo_u16", "pk_mad_u16 opsel" };

template <int K>
static void one(uint32_t *out, uint64_t *clk)
{
    const int iters = 2000;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_rate<K>), dim3(256), dim3(1024), 0, 0, out, iters,
                       clk);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k_rate<K>), dim3(256), dim3(1024), 0, 0, out, iters,
                       clk);
    (void)hipEventRecord(e1);
    (void)hipDeviceSynchronize();
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    uint64_t c[256];
    (void)hipMemcpy(c, clk, sizeof c, hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < 256; i++)
        m += (double)c[i];
    m /= 256;
    // 16 waves per CU = 4 per SIMD; per SIMD: 4 * iters * 32 instructions
    const double ni = 4.0 * iters * 32;   // wave-instructions per SIMD
    printf("%-16s %.2f memtime ticks per wave-instruction per SIMD; %.3f ms "
           "wall = %.3f ns per wave-instruction per SIMD (%.2f cycles at "
           "2.4 GHz)\n", NAMES[K], m / ni, ms, ms * 1e6 / ni,
           ms * 1e6 / ni * 2.4);
}

int main()
{
    uint32_t *out;
    uint64_t *clk;
    if (hipMalloc(&out, 256 * 1024 * 4) || hipMalloc(&clk, 256 * 8))
        return 1;
    one<0>(out, clk);
    one<1>(out, clk);
    one<2>(out, clk);
    one<3>(out, clk);
    one<4>(out, clk);
    one<5>(out, clk);
    one<6>(out, clk);
    one<7>(out, clk);
    one<8>(out, clk);
    one<9>(out, clk);
    one<10>(out, clk);
    one<11>(out, clk);
    one<12>(out, clk);
    one<13>(out, clk);
    one<14>(out, clk);
    one<15>(out, clk);
    one<16>(out, clk);
    one<18>(out, clk);
    one<19>(out, clk);
    one<20>(out, clk);
    one<21>(out, clk);
    one<22>(out, clk);
    one<23>(out, clk);
    one<24>(out, clk);
    one<26>(out, clk);
    one<27>(out, clk);
    one<28>(out, clk);
    one<29>(out, clk);
    one<30>(out, clk);
    one<31>(out, clk);
    one<32>(out, clk);
    one<33>(out, clk);
    one<34>(out, clk);
    return 0;
}
