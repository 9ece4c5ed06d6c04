// lds128_rate.hip -- ds_read_b128 throughput per CU for k_gcm's GHASH
// lookups (GhPos8, srtp_dev_common.h: 8 per-position tables of 256 16-byte
// entries, entry b of table t at (b*8 + t)*16, lane L reads table
// st ^ (L & 7) at step st, b random) against a conflict-free b128 pattern
// (16 lanes of a group on 16 distinct 4-bank granules) and the b32 T-table
// pattern, at 2 waves per SIMD (512 lanes per CU, as k_gcm).  Each lane
// keeps 8 reads in flight and chains the next index from the data read, as
// GHASH's Horner steps do.  Timing only (DESIGN.md §4 k_gcm budget).
//   hipcc -O3 --offload-arch=gfx950 tools/lds128_rate.hip -o tools/lds128_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(512) void k_lds(uint32_t *out, int iters,
                                             uint32_t salt)
{
    __shared__ u32x4 s[2048];   // 32 KiB, as the GHASH tables
    for (int i = threadIdx.x; i < 2048; i += blockDim.x)
        s[i] = u32x4{ (uint32_t)i * 2654435761u ^ salt, (uint32_t)i,
                      (uint32_t)i * 40503u, salt };
    __syncthreads();
    const uint32_t L = threadIdx.x & 63, r = L & 7;
    uint32_t x[8];
#pragma unroll
    for (int k = 0; k < 8; k++)
        x[k] = (threadIdx.x * 7 + k * 131) * 2654435761u;
    u32x4 acc = { 0, 0, 0, 0 };
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            uint32_t e;
            if (MODE == 0)        // conflict-free: granule = (L & 15) + 16 j
                e = (L & 15) | ((x[k] >> 8) & 0x7f0u);
            else if (MODE == 1)   // GhPos8: table k ^ r, entry random
                e = ((x[k] >> 8) & 0xffu) * 8 + ((uint32_t)k ^ r);
            else                  // the same, both lane halves on one table set
                e = ((x[k] >> 8) & 0xfeu) * 8 + ((uint32_t)k ^ (L & 15)) % 16;
            const u32x4 v = s[e & 2047u];
            x[k] ^= v.x;
            acc ^= v;
        }
    }
    uint32_t res = acc.x ^ acc.y ^ acc.z ^ acc.w;
#pragma unroll
    for (int k = 0; k < 8; k++)
        res ^= x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = res;
}

template <int MODE>
static void one(uint32_t *out, const char *name)
{
    const int iters = 4000, threads = 512;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_lds<MODE>), dim3(256), dim3(threads), 0, 0, out,
                       iters, 1u);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k_lds<MODE>), dim3(256), dim3(threads), 0, 0, out,
                       iters, 2u);
    (void)hipEventRecord(e1);
    (void)hipDeviceSynchronize();
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double per_cu = (double)(threads / 64) * iters * 8;   // wave-instr
    printf("%-34s %d waves/CU: %.3f ns per ds_read_b128 per CU\n", name,
           threads / 64, ms * 1e6 / per_cu);
}

int main()
{
    uint32_t *out;
    if (hipMalloc(&out, 256 * 512 * 4))
        return 1;
    one<0>(out, "b128 conflict-free");
    one<1>(out, "b128 GhPos8 (k_gcm)");
    one<2>(out, "b128 16 tables, one parity");
    return 0;
}
