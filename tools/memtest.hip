// memtest.hip -- which lane <-> packet access shape can the SRTP kernels
// stream at?  Copies (loads + stores, 16 B per lane per instruction) the
// bench arena (2^20 packets, 1424-byte slots, 22 full 64-byte chunks per
// packet) with one wave per 64 packets, in several lane patterns:
//   lane   : lane l touches packet l only (16 B of it per instruction)
//   quad   : lanes 4m..4m+3 cover 64 contiguous bytes of one packet
//   spread : lanes m, m+16, m+32, m+48 cover 64 contiguous bytes
//   oct    : lanes 8m..8m+7 cover 128 contiguous bytes (2 chunks)
//   linear : the wave sweeps its 64 packets' span, 1 KiB per instruction
// PF = chunk steps of loads kept in flight.  Timing only.
//   hipcc -O3 --offload-arch=gfx950 tools/memtest.hip -o tools/memtest
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t SLOT = 1424, NCH = 22;

// address of (step s, instruction k) for lane l of the wave whose first
// packet is p0: returns the byte offset of the 16-B piece
template <int MODE>
__device__ __forceinline__ uint64_t piece(uint32_t p0, uint32_t l, uint32_t s,
                                          uint32_t k)
{
    if (MODE == 0)   // lane: packet l, quad k of chunk s
        return (uint64_t)(p0 + l) * SLOT + 64 * s + 16 * k;
    if (MODE == 1)   // quad: packet 16k + l/4, quad l%4 of chunk s
        return (uint64_t)(p0 + 16 * k + (l >> 2)) * SLOT + 64 * s + 16 * (l & 3);
    if (MODE == 2)   // spread: packet 16k + l%16, quad l/16
        return (uint64_t)(p0 + 16 * k + (l & 15)) * SLOT + 64 * s + 16 * (l >> 4);
    if (MODE == 6)   // lane, 64-B aligned segments of packet l
        return (((uint64_t)(p0 + l) * SLOT + 63) & ~63ull) + 64 * s + 16 * k;
    if (MODE == 7)   // quad, 64-B aligned segments
        return (((uint64_t)(p0 + 16 * k + (l >> 2)) * SLOT + 63) & ~63ull) +
               64 * s + 16 * (l & 3);
    if (MODE == 5)   // unit64: lane l = 64-B unit (64 s + l) of the span
        return (uint64_t)p0 * SLOT + 64 * (64 * s + l) + 16 * k;
    if (MODE == 4)   // linear: the wave's 64-packet span, 1 KiB per instruction
        return (uint64_t)p0 * SLOT + 1024 * (4 * s + k) + 16 * l;
    // oct: chunk pair s/2 .. 8 packets per instruction, 8 instructions per
    // pair; step s covers instructions 4(s&1)..4(s&1)+3
    const uint32_t ki = 4 * (s & 1) + k;
    return (uint64_t)(p0 + 8 * ki + (l >> 3)) * SLOT + 128 * (s >> 1) +
           16 * (l & 7);
}

template <int MODE, int PF>
__global__ __launch_bounds__(512) void k_copy(const uint8_t *in, uint8_t *out,
                                               uint32_t n)
{
    const uint32_t l = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * (blockDim.x / 64);
    for (uint32_t w = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
         64 * w < n; w += nw) {
        const uint32_t p0 = 64 * w;
        u32x4 ring[PF][4];
#pragma unroll
        for (int j = 0; j < PF; j++)
#pragma unroll
            for (int k = 0; k < 4; k++)
                ring[j][k] = *(const u32x4 *)(in + piece<MODE>(p0, l, j, k));
        for (uint32_t s = 0; s < NCH; s++) {
            u32x4 cur[4];
#pragma unroll
            for (int k = 0; k < 4; k++)
                cur[k] = ring[0][k];
#pragma unroll
            for (int j = 0; j + 1 < PF; j++)
#pragma unroll
                for (int k = 0; k < 4; k++)
                    ring[j][k] = ring[j + 1][k];
            if (s + PF < NCH) {
#pragma unroll
                for (int k = 0; k < 4; k++)
                    ring[PF - 1][k] =
                        *(const u32x4 *)(in + piece<MODE>(p0, l, s + PF, k));
            }
#pragma unroll
            for (int k = 0; k < 4; k++)
                *(u32x4 *)(out + piece<MODE>(p0, l, s, k)) = cur[k] ^ 0x5a5a5a5au;
        }
    }
}

template <int MODE, int PF>
static float run(const uint8_t *in, uint8_t *out, uint32_t n, int wgs)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int it = 0; it < 5; it++) {
        hipEventRecord(a);
        hipLaunchKernelGGL((k_copy<MODE, PF>), dim3(wgs), dim3(512), 0, 0, in,
                           out, n);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best)
            best = ms;
    }
    return best;
}

// read-only: MODE patterns, XOR-accumulated, one 16-B store per lane at end
template <int MODE, int PF>
__global__ __launch_bounds__(512) void k_read(const uint8_t *in, uint8_t *out,
                                               uint32_t n)
{
    const uint32_t l = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * (blockDim.x / 64);
    u32x4 acc = { 0, 0, 0, 0 };
    for (uint32_t w = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
         64 * w < n; w += nw) {
        const uint32_t p0 = 64 * w;
        u32x4 ring[PF][4];
#pragma unroll
        for (int j = 0; j < PF; j++)
#pragma unroll
            for (int k = 0; k < 4; k++)
                ring[j][k] = *(const u32x4 *)(in + piece<MODE>(p0, l, j, k));
        for (uint32_t s = 0; s < NCH; s++) {
#pragma unroll
            for (int k = 0; k < 4; k++)
                acc ^= ring[0][k];
#pragma unroll
            for (int j = 0; j + 1 < PF; j++)
#pragma unroll
                for (int k = 0; k < 4; k++)
                    ring[j][k] = ring[j + 1][k];
            if (s + PF < NCH) {
#pragma unroll
                for (int k = 0; k < 4; k++)
                    ring[PF - 1][k] =
                        *(const u32x4 *)(in + piece<MODE>(p0, l, s + PF, k));
            }
        }
    }
    *(u32x4 *)(out + 16 * (blockIdx.x * blockDim.x + threadIdx.x)) = acc;
}

template <int MODE, int PF>
static float runr(const uint8_t *in, uint8_t *out, uint32_t n, int wgs)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int it = 0; it < 5; it++) {
        hipEventRecord(a);
        hipLaunchKernelGGL((k_read<MODE, PF>), dim3(wgs), dim3(512), 0, 0, in,
                           out, n);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best)
            best = ms;
    }
    return best;
}

// 256-byte bursts per packet: 16 instructions per burst, loaded together
// (MODE 0: lane l = packet l; MODE 1: quad pattern, 16 packets x 64 B per
// instruction), then stored; NB bursts per packet
constexpr uint32_t NB = 5;
template <int MODE>
__device__ __forceinline__ uint64_t bpiece(uint32_t p0, uint32_t l, uint32_t s,
                                           uint32_t k)
{
    if (MODE == 0)
        return (uint64_t)(p0 + l) * SLOT + 256 * s + 16 * k;
    return (uint64_t)(p0 + 16 * (k & 3) + (l >> 2)) * SLOT + 256 * s +
           16 * (4 * (k >> 2) + (l & 3));
}

template <int MODE, int PF>
__global__ __launch_bounds__(512) void k_burst(const uint8_t *in, uint8_t *out,
                                                uint32_t n)
{
    const uint32_t l = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * (blockDim.x / 64);
    for (uint32_t w = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
         64 * w < n; w += nw) {
        const uint32_t p0 = 64 * w;
        u32x4 ring[PF][16];
#pragma unroll
        for (int j = 0; j < PF; j++)
#pragma unroll
            for (int k = 0; k < 16; k++)
                ring[j][k] = *(const u32x4 *)(in + bpiece<MODE>(p0, l, j, k));
        for (uint32_t s = 0; s < NB; s++) {
            u32x4 cur[16];
#pragma unroll
            for (int k = 0; k < 16; k++)
                cur[k] = ring[0][k];
#pragma unroll
            for (int j = 0; j + 1 < PF; j++)
#pragma unroll
                for (int k = 0; k < 16; k++)
                    ring[j][k] = ring[j + 1][k];
            if (s + PF < NB) {
#pragma unroll
                for (int k = 0; k < 16; k++)
                    ring[PF - 1][k] =
                        *(const u32x4 *)(in + bpiece<MODE>(p0, l, s + PF, k));
            }
#pragma unroll
            for (int k = 0; k < 16; k++)
                *(u32x4 *)(out + bpiece<MODE>(p0, l, s, k)) = cur[k] ^ 0x5a5a5a5au;
        }
    }
}

template <int MODE, int PF>
static float runb(const uint8_t *in, uint8_t *out, uint32_t n, int wgs)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int it = 0; it < 5; it++) {
        hipEventRecord(a);
        hipLaunchKernelGGL((k_burst<MODE, PF>), dim3(wgs), dim3(512), 0, 0, in,
                           out, n);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best)
            best = ms;
    }
    return best;
}

int main(int argc, char **argv)
{
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
    const size_t bytes = (size_t)n * SLOT;
    uint8_t *in, *out;
    if (hipMalloc(&in, bytes) || hipMalloc(&out, bytes))
        return 1;
    // argv[3] = 1: in place (the SRTP kernels protect in place)
    if (argc > 3 && atoi(argv[3]) == 1)
        out = in;
    hipMemset(in, 1, bytes);
    const double algo = (double)n * NCH * 64 * 2;
    const char *names[] = { "lane", "quad", "spread", "oct", "linear" };
    const int wl = argc > 2 ? atoi(argv[2]) : 0;
    for (int wgs : { 128, 256, 1024 }) {
        if (wl && wgs != wl)
            continue;
        float t[5][3] = {};
        t[4][0] = run<4, 1>(in, out, n, wgs);
        t[4][1] = run<4, 2>(in, out, n, wgs);
        t[4][2] = run<4, 4>(in, out, n, wgs);
        t[0][0] = run<0, 1>(in, out, n, wgs);
        t[0][1] = run<0, 2>(in, out, n, wgs);
        t[0][2] = run<0, 4>(in, out, n, wgs);
        t[1][0] = run<1, 1>(in, out, n, wgs);
        t[1][1] = run<1, 2>(in, out, n, wgs);
        t[1][2] = run<1, 4>(in, out, n, wgs);
        t[2][0] = run<2, 1>(in, out, n, wgs);
        t[2][1] = run<2, 2>(in, out, n, wgs);
        t[2][2] = run<2, 4>(in, out, n, wgs);
        t[3][0] = run<3, 1>(in, out, n, wgs);
        t[3][1] = run<3, 2>(in, out, n, wgs);
        t[3][2] = run<3, 4>(in, out, n, wgs);
        const double ab = (double)n * NB * 256 * 2;
        const float b0 = runb<0, 1>(in, out, n, wgs), b1 = runb<1, 1>(in, out, n, wgs);
        const float b2 = runb<0, 2>(in, out, n, wgs), b3 = runb<1, 2>(in, out, n, wgs);
        printf("wgs %4d burst256 lane PF1 %.2f TB/s PF2 %.2f | quad PF1 %.2f TB/s PF2 %.2f\n",
               wgs, ab / b0 / 1e9, ab / b2 / 1e9, ab / b1 / 1e9, ab / b3 / 1e9);
        {
            const double ar = (double)n * NCH * 64;
            printf("wgs %4d read-only lane PF4 %.2f TB/s | quad PF4 %.2f | oct PF4 %.2f | linear PF4 %.2f\n", wgs,
                   ar / runr<0, 4>(in, out, n, wgs) / 1e9, ar / runr<1, 4>(in, out, n, wgs) / 1e9,
                   ar / runr<3, 4>(in, out, n, wgs) / 1e9, ar / runr<4, 4>(in, out, n, wgs) / 1e9);
            printf("wgs %4d aligned copy lane PF1 %.2f PF4 %.2f | quad PF1 %.2f PF4 %.2f\n", wgs,
                   2 * ar / run<6, 1>(in, out, n, wgs) / 1e9, 2 * ar / run<6, 4>(in, out, n, wgs) / 1e9,
                   2 * ar / run<7, 1>(in, out, n, wgs) / 1e9, 2 * ar / run<7, 4>(in, out, n, wgs) / 1e9);
            printf("wgs %4d read-only aligned lane PF4 %.2f | quad PF4 %.2f\n", wgs,
                   ar / runr<6, 4>(in, out, n, wgs) / 1e9, ar / runr<7, 4>(in, out, n, wgs) / 1e9);
            printf("wgs %4d unit64 copy PF1 %.2f TB/s PF2 %.2f PF4 %.2f\n", wgs,
                   2 * ar / run<5, 1>(in, out, n, wgs) / 1e9, 2 * ar / run<5, 2>(in, out, n, wgs) / 1e9,
                   2 * ar / run<5, 4>(in, out, n, wgs) / 1e9);
        }
        for (int m = 0; m < 5; m++)
            printf("wgs %4d %-6s PF1 %.3f ms (%.2f TB/s)  PF2 %.3f ms (%.2f)  "
                   "PF4 %.3f ms (%.2f)\n",
                   wgs, names[m], t[m][0], algo / t[m][0] / 1e9, t[m][1],
                   algo / t[m][1] / 1e9, t[m][2], algo / t[m][2] / 1e9);
    }
    return 0;
}
