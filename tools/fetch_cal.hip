// fetch_cal.hip -- calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE against
// known byte counts for the access shapes the SRTP kernels use (VERDICT r03
// item 7: the headline's FETCH_SIZE read below the kernel's minimum read
// bytes).  2^20 packets x 1424-byte slots (1.49 GB, far past the 256 MB
// MALL), 22 full 64-byte chunks per packet, one wave per 64 packets:
//   k_rd_lane   lane l reads packet l, 16 B per lane per instruction
//   k_rd_quad   lanes 4m..4m+3 read 64 contiguous bytes of one packet
//   k_rd_linear the wave sweeps its packets' span, 1 KiB per instruction
//   k_cp_quad   quad loads + 64-B-aligned quad stores (the headline
//               kernel's steady state) into a second arena
//   k_cp_quad_ip the same in place, k_cp_lane_ip per-lane 16-B pieces in
//               place (the per-lane-key kernel's shape)
// Each kernel runs once after one untimed warmup launch of all; the known
// bytes per launch are printed.  Run the counters in separate passes:
//   rocprofv3 --pmc FETCH_SIZE -- tools/fetch_cal
//   rocprofv3 --pmc WRITE_SIZE -- tools/fetch_cal
//   hipcc -O3 --offload-arch=gfx950 tools/fetch_cal.hip -o tools/fetch_cal
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t SLOT = 1424, NCH = 22;

template <int MODE>
__device__ __forceinline__ uint64_t piece(uint32_t p0, uint32_t l, uint32_t s,
                                          uint32_t k)
{
    if (MODE == 0)
        return (uint64_t)(p0 + l) * SLOT + 64 * s + 16 * k;
    if (MODE == 1)
        return (uint64_t)(p0 + 16 * k + (l >> 2)) * SLOT + 64 * s + 16 * (l & 3);
    if (MODE == 2)   // quad, 64-B aligned segments
        return (((uint64_t)(p0 + 16 * k + (l >> 2)) * SLOT + 63) & ~63ull) +
               64 * s + 16 * (l & 3);
    return (uint64_t)p0 * SLOT + 1024 * (4 * s + k) + 16 * l;
}

template <int MODE>
__device__ void rd(const uint8_t *in, uint8_t *out, uint32_t n)
{
    const uint32_t l = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * (blockDim.x / 64);
    u32x4 acc = { 0, 0, 0, 0 };
    for (uint32_t w = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
         64 * w < n; w += nw)
        for (uint32_t s = 0; s < NCH; s++)
#pragma unroll
            for (int k = 0; k < 4; k++)
                acc ^= *(const u32x4 *)(in + piece<MODE>(64 * w, l, s, k));
    if (acc[0] == 0x12345678u && acc[1] == 0x9abcdef0u)   // keeps the loads
        *(u32x4 *)(out + 16 * (blockIdx.x * blockDim.x + threadIdx.x)) = acc;
}

__global__ __launch_bounds__(512) void k_rd_lane(const uint8_t *in, uint8_t *out, uint32_t n) { rd<0>(in, out, n); }
__global__ __launch_bounds__(512) void k_rd_quad(const uint8_t *in, uint8_t *out, uint32_t n) { rd<1>(in, out, n); }
__global__ __launch_bounds__(512) void k_rd_linear(const uint8_t *in, uint8_t *out, uint32_t n) { rd<3>(in, out, n); }

template <int MODE>
__device__ void cp(const uint8_t *in, uint8_t *out, uint32_t n)
{
    const uint32_t l = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * (blockDim.x / 64);
    for (uint32_t w = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
         64 * w < n; w += nw)
        for (uint32_t s = 0; s + 1 < NCH; s++)
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint64_t o = piece<MODE>(64 * w, l, s, k);
                *(u32x4 *)(out + o) = *(const u32x4 *)(in + o) ^ 0x5a5a5a5au;
            }
}

// copies of 21 chunks per packet: aligned quads out of place and in place
// (the SRTP kernels protect in place), per-lane 16-B pieces in place
__global__ __launch_bounds__(512) void k_cp_quad(const uint8_t *in, uint8_t *out, uint32_t n) { cp<2>(in, out, n); }
__global__ __launch_bounds__(512) void k_cp_quad_ip(const uint8_t *in, uint8_t *out, uint32_t n) { cp<2>(in, out, n); }
__global__ __launch_bounds__(512) void k_cp_lane_ip(const uint8_t *in, uint8_t *out, uint32_t n) { cp<0>(in, out, n); }

int main()
{
    const uint32_t n = 1u << 20;
    const size_t bytes = (size_t)n * SLOT + 64;
    uint8_t *in, *out;
    if (hipMalloc(&in, bytes) || hipMalloc(&out, bytes))
        return 1;
    hipMemset(in, 1, bytes);
    hipMemset(out, 0, bytes);
    const dim3 g(1024), b(512);
    for (int pass = 0; pass < 2; pass++) {
        hipLaunchKernelGGL(k_rd_lane, g, b, 0, 0, in, out, n);
        hipLaunchKernelGGL(k_rd_quad, g, b, 0, 0, in, out, n);
        hipLaunchKernelGGL(k_rd_linear, g, b, 0, 0, in, out, n);
        hipLaunchKernelGGL(k_cp_quad, g, b, 0, 0, in, out, n);
        hipLaunchKernelGGL(k_cp_quad_ip, g, b, 0, 0, in, in, n);
        hipLaunchKernelGGL(k_cp_lane_ip, g, b, 0, 0, in, in, n);
        if (hipDeviceSynchronize() != hipSuccess)
            return 2;
    }
    printf("{\"read_bytes_per_launch\": %llu, \"cp_bytes_each_way\": %llu}\n",
           (unsigned long long)n * NCH * 64,
           (unsigned long long)n * (NCH - 1) * 64);
    return 0;
}
