// issue_rate.hip -- how many shader cycles one SIMD needs per wave64
// instruction for the instruction shapes the SRTP kernels are made of, at 2
// and 4 waves per SIMD: 2-source vs 3-source VALU, sources that change every
// instruction, and VALU mixed with LDS reads.  Timing only.
//   hipcc -O3 --offload-arch=gfx950 tools/issue_rate.hip -o tools/issue_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define V8 "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)

template <int K>
__device__ __forceinline__ void body(uint32_t &a0, uint32_t &a1, uint32_t &a2,
                                     uint32_t &a3, uint32_t &a4, uint32_t &a5,
                                     uint32_t &a6, uint32_t &a7, uint32_t x,
                                     uint32_t y, uint32_t lds)
{
    if (K == 0)   // 2-source VOP2
        asm volatile("v_xor_b32 %0, %0, %8\n v_xor_b32 %1, %1, %8\n v_xor_b32 %2, %2, %8\n v_xor_b32 %3, %3, %8\n"
                     "v_xor_b32 %4, %4, %8\n v_xor_b32 %5, %5, %8\n v_xor_b32 %6, %6, %8\n v_xor_b32 %7, %7, %8"
                     : V8 : "v"(x));
    if (K == 1)   // 3-source, two fixed sources
        asm volatile("v_bitop3_b32 %0, %0, %8, %9 bitop3:0x96\n v_bitop3_b32 %1, %1, %8, %9 bitop3:0x96\n"
                     "v_bitop3_b32 %2, %2, %8, %9 bitop3:0x96\n v_bitop3_b32 %3, %3, %8, %9 bitop3:0x96\n"
                     "v_bitop3_b32 %4, %4, %8, %9 bitop3:0x96\n v_bitop3_b32 %5, %5, %8, %9 bitop3:0x96\n"
                     "v_bitop3_b32 %6, %6, %8, %9 bitop3:0x96\n v_bitop3_b32 %7, %7, %8, %9 bitop3:0x96"
                     : V8 : "v"(x), "v"(y));
    if (K == 2)   // 3-source, all sources distinct and changing (as in AES / SHA-1)
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n v_bitop3_b32 %3, %3, %4, %5 bitop3:0x96\n"
                     "v_bitop3_b32 %6, %6, %7, %0 bitop3:0x96\n v_bitop3_b32 %1, %1, %2, %3 bitop3:0x96\n"
                     "v_bitop3_b32 %4, %4, %5, %6 bitop3:0x96\n v_bitop3_b32 %7, %7, %0, %1 bitop3:0x96\n"
                     "v_bitop3_b32 %2, %2, %3, %4 bitop3:0x96\n v_bitop3_b32 %5, %5, %6, %7 bitop3:0x96"
                     : V8);
    if (K == 3)   // v_perm, fixed selector
        asm volatile("v_perm_b32 %0, %0, %8, %9\n v_perm_b32 %1, %1, %8, %9\n v_perm_b32 %2, %2, %8, %9\n"
                     "v_perm_b32 %3, %3, %8, %9\n v_perm_b32 %4, %4, %8, %9\n v_perm_b32 %5, %5, %8, %9\n"
                     "v_perm_b32 %6, %6, %8, %9\n v_perm_b32 %7, %7, %8, %9"
                     : V8 : "v"(x), "v"(y));
    if (K == 4)   // 2-source VOP2 with distinct changing sources
        asm volatile("v_xor_b32 %0, %0, %1\n v_xor_b32 %2, %2, %3\n v_xor_b32 %4, %4, %5\n v_xor_b32 %6, %6, %7\n"
                     "v_xor_b32 %1, %1, %2\n v_xor_b32 %3, %3, %4\n v_xor_b32 %5, %5, %6\n v_xor_b32 %7, %7, %0"
                     : V8);
    if (K == 5)   // v_alignbit with changing sources (a rotate)
        asm volatile("v_alignbit_b32 %0, %0, %0, 27\n v_alignbit_b32 %1, %1, %1, 27\n v_alignbit_b32 %2, %2, %2, 27\n"
                     "v_alignbit_b32 %3, %3, %3, 27\n v_alignbit_b32 %4, %4, %4, 27\n v_alignbit_b32 %5, %5, %5, 27\n"
                     "v_alignbit_b32 %6, %6, %6, 27\n v_alignbit_b32 %7, %7, %7, 27"
                     : V8);
    if (K == 6)   // v_add3 with changing sources
        asm volatile("v_add3_u32 %0, %0, %1, %2\n v_add3_u32 %3, %3, %4, %5\n v_add3_u32 %6, %6, %7, %0\n"
                     "v_add3_u32 %1, %1, %2, %3\n v_add3_u32 %4, %4, %5, %6\n v_add3_u32 %7, %7, %0, %1\n"
                     "v_add3_u32 %2, %2, %3, %4\n v_add3_u32 %5, %5, %6, %7"
                     : V8);
    if (K == 7) {   // AES-like: 4 ds_read_b32 + 4 address perms + 2 xor3 per group of 4 (x2)
        uint32_t t0, t1, t2, t3;
        asm volatile("v_perm_b32 %4, %0, %12, %13\n v_perm_b32 %5, %1, %12, %13\n"
                     "v_perm_b32 %6, %2, %12, %13\n v_perm_b32 %7, %3, %12, %13\n"
                     "v_and_b32 %4, 0xfffc, %4\n v_and_b32 %5, 0xfffc, %5\n"
                     "v_and_b32 %6, 0xfffc, %6\n v_and_b32 %7, 0xfffc, %7\n"
                     "ds_read_b32 %4, %4\n ds_read_b32 %5, %5\n ds_read_b32 %6, %6\n ds_read_b32 %7, %7\n"
                     "v_bitop3_b32 %8, %8, %9, %10 bitop3:0x96\n v_bitop3_b32 %9, %9, %10, %11 bitop3:0x96\n"
                     "v_bitop3_b32 %10, %10, %11, %8 bitop3:0x96\n v_bitop3_b32 %11, %11, %8, %9 bitop3:0x96\n"
                     "s_waitcnt lgkmcnt(0)\n"
                     "v_bitop3_b32 %0, %4, %5, %0 bitop3:0x96\n v_bitop3_b32 %1, %6, %7, %1 bitop3:0x96\n"
                     "v_bitop3_b32 %2, %4, %7, %2 bitop3:0x96\n v_bitop3_b32 %3, %5, %6, %3 bitop3:0x96"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3),
                       "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(lds), "v"(y));
    }
}

// overlap probe (round 4): LDS-only, VALU-only and both, in one wave or in
// different waves of a SIMD -- does an LDS read stream overlap a VALU
// stream, or do the two add up?
#define LDS8(a, b)                                                              \
    asm volatile("ds_read_b32 %0, %8\n ds_read_b32 %1, %8 offset:4096\n"       \
                 "ds_read_b32 %2, %8 offset:8192\n ds_read_b32 %3, %8 offset:12288\n" \
                 "ds_read_b32 %4, %8 offset:16384\n ds_read_b32 %5, %8 offset:20480\n" \
                 "ds_read_b32 %6, %8 offset:24576\n ds_read_b32 %7, %8 offset:28672\n" \
                 "s_waitcnt lgkmcnt(0)"                                         \
                 : "=&v"(b[0]), "=&v"(b[1]), "=&v"(b[2]), "=&v"(b[3]),          \
                   "=&v"(b[4]), "=&v"(b[5]), "=&v"(b[6]), "=&v"(b[7])           \
                 : "v"(a))
template <int K>
__device__ __forceinline__ void body2(uint32_t &a0, uint32_t &a1, uint32_t &a2,
                                      uint32_t &a3, uint32_t &a4, uint32_t &a5,
                                      uint32_t &a6, uint32_t &a7, uint32_t addr)
{
    uint32_t b[8];
    const bool lw = (threadIdx.x >> 6) & 1;   // K == 11: odd waves read LDS
    if (K == 8 || K == 10 || (K == 11 && lw)) {
        LDS8(addr, b);
        a0 ^= b[0] + b[1] + b[2] + b[3] + b[4] + b[5] + b[6] + b[7];
    }
    if (K == 9 || K == 10 || (K == 11 && !lw))
        body<2>(a0, a1, a2, a3, a4, a5, a6, a7, 0, 0, 0);
}

// instructions per body() call
static const int NI[] = { 8, 8, 8, 8, 8, 8, 8, 20, 8, 8, 16, 8 };
static const char *NAMES[] = { "v_xor_b32 (2 src, fixed x)",
                               "v_bitop3 (3 src, 2 fixed)",
                               "v_bitop3 (3 src, all changing)",
                               "v_perm (fixed selector)",
                               "v_xor_b32 (2 src, changing)",
                               "v_alignbit rotate",
                               "v_add3 (changing)",
                               "AES-like mix (12 VALU + 4 ds_read_b32 + 4 VALU)",
                               "LDS only: 8 ds_read_b32 (+8 VALU to consume)",
                               "VALU only: 8 v_bitop3",
                               "both in every wave: 8 LDS + 8+8 VALU",
                               "odd waves LDS (+8 VALU), even waves VALU" };

template <int K>
__global__ __launch_bounds__(1024) void k_rate(uint32_t *out, int iters,
                                               uint64_t *clk)
{
    __shared__ uint32_t s[16384];
    for (int i = threadIdx.x; i < 16384; i += blockDim.x)
        s[i] = i * 2654435761u;
    __syncthreads();
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3,
             a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = blockIdx.x | 0x10203, y = 0x0c0c0504u;
    uint32_t lds = (uint32_t)(uintptr_t)s;
    // K >= 8: lane l reads copy l & 31 of a 128-B row (the T-table layout)
    const uint32_t addr = lds + ((threadIdx.x * 2654435761u >> 24) & 31) * 128 +
                          (threadIdx.x & 31) * 4;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < 8; r++)
            if constexpr (K >= 8)
                body2<K>(a0, a1, a2, a3, a4, a5, a6, a7, addr);
            else
                body<K>(a0, a1, a2, a3, a4, a5, a6, a7, x, y, lds);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] =
        a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0)
        clk[blockIdx.x] = t1 - t0;
}

template <int K>
static void one(uint32_t *out, uint64_t *clk, int threads)
{
    const int iters = 1000;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_rate<K>), dim3(256), dim3(threads), 0, 0, out,
                       iters, clk);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k_rate<K>), dim3(256), dim3(threads), 0, 0, out,
                       iters, clk);
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
    const int wps = threads / 256;   // waves per SIMD
    const double ni = (double)wps * iters * 8 * NI[K];
    printf("%-48s %d waves/SIMD: %.3f ns per wave-instruction per SIMD "
           "(wall), %.2f s_memtime ticks, %.3f ms\n", NAMES[K], wps,
           ms * 1e6 / ni, m / ni, ms);
}

template <int K>
static void both(uint32_t *out, uint64_t *clk)
{
    one<K>(out, clk, 256);
    one<K>(out, clk, 512);
    one<K>(out, clk, 1024);
}

int main()
{
    uint32_t *out;
    uint64_t *clk;
    if (hipMalloc(&out, 256 * 1024 * 4) || hipMalloc(&clk, 256 * 8))
        return 1;
    both<0>(out, clk);
    both<1>(out, clk);
    both<2>(out, clk);
    both<3>(out, clk);
    both<4>(out, clk);
    both<5>(out, clk);
    both<6>(out, clk);
    both<7>(out, clk);
    both<8>(out, clk);
    both<9>(out, clk);
    both<10>(out, clk);
    both<11>(out, clk);
    return 0;
}
