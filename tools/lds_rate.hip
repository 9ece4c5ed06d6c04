// lds_rate.hip -- LDS read throughput per CU for the AES T-table access
// pattern of k_icm_hmac / k_gcm (32 copies of a 1 KiB table row-interleaved:
// byte address x*256 + (lane & 31)*4 [+128 for the odd table], x random per
// lane) against the linear pattern, at 2 and 4 waves per SIMD.  Each lane
// keeps 8 reads in flight and chains the next address from the data read,
// as the AES rounds do.  Timing only.
//   hipcc -O3 --offload-arch=gfx950 tools/lds_rate.hip -o tools/lds_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int MODE>
__global__ __launch_bounds__(1024) void k_lds(uint32_t *out, int iters,
                                              uint32_t salt)
{
    __shared__ uint32_t s[32768];   // 128 KiB, as the four T-tables
    for (int i = threadIdx.x; i < 32768; i += blockDim.x)
        s[i] = (uint32_t)i * 2654435761u ^ salt;
    __syncthreads();
    const uint32_t c = (threadIdx.x & 31) * 4;
    uint32_t x[8];
#pragma unroll
    for (int k = 0; k < 8; k++)
        x[k] = (threadIdx.x * 7 + k * 131) * 2654435761u;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            uint32_t a;
            if (MODE == 0)        // linear: lane l reads dword l of a row
                a = ((x[k] & 0x1f00u) | (threadIdx.x & 63) * 4) & 0xfffcu;
            else if (MODE == 1)   // T-table: random row, copy lane & 31
                a = (x[k] & 0xff00u) | c | ((k & 1) << 7);
            else                  // T-table rows in all of 128 KiB
                a = ((x[k] & 0x1ff00u) | c | ((k & 1) << 7)) & 0x1ffffu;
            x[k] ^= *(const uint32_t *)((const char *)s + a);
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++)
        r ^= x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int MODE>
static void one(uint32_t *out, int threads, const char *name)
{
    const int iters = 2000;
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
    printf("%-28s %2d waves/CU: %.3f ns per ds_read_b32 per CU "
           "(%.2f cycles at 2.1 GHz)\n", name, threads / 64,
           ms * 1e6 / per_cu, ms * 1e6 / per_cu * 2.1);
}

int main()
{
    uint32_t *out;
    if (hipMalloc(&out, 256 * 1024 * 4))
        return 1;
    for (int t : { 512, 1024 }) {
        if (t == 512) {
            one<0>(out, 512, "linear");
            one<1>(out, 512, "T-table 64 KiB rows");
            one<2>(out, 512, "T-table 128 KiB rows");
        } else {
            one<0>(out, 1024, "linear");
            one<1>(out, 1024, "T-table 64 KiB rows");
            one<2>(out, 1024, "T-table 128 KiB rows");
        }
    }
    return 0;
}
