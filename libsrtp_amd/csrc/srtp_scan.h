// srtp_scan.h -- the device pre-pass's own scans and stable sort (no
// hipCUB): used by srtp_prepass.hip for the chain form of the index
// pre-pass (srtp/srtp.c:2038-2081 and crypto/replay/rdbx.c:112-145 in batch
// form: the advances of a stream's packets, summed in stream order).
//
//  * scan_run: inclusive or exclusive scan of 64-bit values with + or max,
//    optionally segmented by runs of equal keys (the reference walks every
//    stream's packets separately; a stable sort by stream makes each stream
//    one run).  Three launches: per-tile aggregates, one workgroup scanning
//    the tile aggregates, per-tile scan with the tile's carry.
//  * radix_sort: stable LSD radix sort of (key, value) pairs by the low
//    end_bit bits of the key; every pass is a per-tile digit histogram, a
//    scan of the histograms (scan_run) and a stable scatter.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srtp_scan {

constexpr int TILE_THREADS = 256;
constexpr int TILE_ITEMS = 4;                       // per thread, blocked
constexpr int TILE = TILE_THREADS * TILE_ITEMS;     // 1024 items per tile
constexpr uint32_t NOKEY = 0xffffffffu;

enum { OP_SUM = 0, OP_MAX = 1 };

template <int OP>
__device__ __forceinline__ uint64_t op2(uint64_t a, uint64_t b)
{
    if (OP == OP_SUM)
        return a + b;
    return a > b ? a : b;
}

// aggregate of a run of items: first / last key, whether all items share
// one key, the value of the last run (items of the last key at the end)
struct Agg {
    uint32_t fk, lk;
    uint32_t single, has;
    uint64_t v;
};

template <int OP>
__device__ __forceinline__ Agg combine(const Agg &a, const Agg &b)
{
    if (!a.has)
        return b;
    if (!b.has)
        return a;
    Agg r;
    const bool join = b.single && a.lk == b.fk;
    r.fk = a.fk;
    r.lk = b.lk;
    r.single = a.single && join;
    r.has = 1;
    r.v = join ? op2<OP>(a.v, b.v) : b.v;
    return r;
}

__device__ __forceinline__ Agg agg_of(uint32_t k, uint64_t v)
{
    Agg r;
    r.fk = r.lk = k;
    r.single = 1;
    r.has = 1;
    r.v = v;
    return r;
}

__device__ __forceinline__ Agg agg_none()
{
    Agg r;
    r.fk = r.lk = NOKEY;
    r.single = 1;
    r.has = 0;
    r.v = 0;
    return r;
}

template <int OP>
__device__ __forceinline__ Agg agg_shfl_up(const Agg &a, int d)
{
    Agg r;
    r.fk = (uint32_t)__shfl_up((int)a.fk, d);
    r.lk = (uint32_t)__shfl_up((int)a.lk, d);
    r.single = (uint32_t)__shfl_up((int)a.single, d);
    r.has = (uint32_t)__shfl_up((int)a.has, d);
    r.v = (uint64_t)__shfl_up((long long)a.v, d);
    return r;
}

// exclusive scan of one Agg per thread over the block: inclusive scans of
// the four waves by shuffles, the wave totals through LDS (two barriers;
// a Hillis-Steele pass over 256 threads in LDS took 16); returns the
// thread's exclusive prefix, *total = the block's
template <int OP, int NT = TILE_THREADS>
__device__ Agg block_exclusive(Agg mine, Agg *total)
{
    constexpr int NW = NT / 64;
    __shared__ Agg s_w[NW];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    Agg incl = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const Agg o = agg_shfl_up<OP>(incl, d);   // an earlier lane
        if (lane >= d)
            incl = combine<OP>(o, incl);
    }
    Agg lex = agg_shfl_up<OP>(incl, 1);
    if (lane == 0)
        lex = agg_none();
    if (lane == 63)
        s_w[wv] = incl;
    __syncthreads();
    Agg wex = agg_none(), tot = agg_none();
#pragma unroll
    for (int w = 0; w < NW; w++) {
        if (w == wv)
            wex = tot;
        tot = combine<OP>(tot, s_w[w]);
    }
    *total = tot;
    __syncthreads();   // s_w is free again
    return combine<OP>(wex, lex);
}

// Traits: key(i) (NOKEY-free; unsegmented scans return 0), val(i),
// store(i, v)
template <int OP, class S>
__global__ __launch_bounds__(TILE_THREADS) void k_scan_up(S s, uint32_t n,
                                                          Agg *agg)
{
    const uint32_t base = blockIdx.x * TILE + threadIdx.x * TILE_ITEMS;
    Agg a = agg_none();
#pragma unroll
    for (int k = 0; k < TILE_ITEMS; k++)
        if (base + k < n)
            a = combine<OP>(a, agg_of(s.key(base + k), s.val(base + k)));
    Agg tot;
    (void)block_exclusive<OP>(a, &tot);
    if (threadIdx.x == 0)
        agg[blockIdx.x] = tot;
}

// one workgroup of 1024 threads: exclusive carry of every tile
template <int OP>
__global__ __launch_bounds__(1024) void k_scan_mid(Agg *agg, uint32_t ntiles)
{
    constexpr uint32_t T = 1024;   // the launch's block size
    const uint32_t t = threadIdx.x;
    const uint32_t per = (ntiles + T - 1) / T;
    const uint32_t a0 = t * per < ntiles ? t * per : ntiles;
    const uint32_t a1 = a0 + per < ntiles ? a0 + per : ntiles;
    Agg run = agg_none();
    for (uint32_t i = a0; i < a1; i++)
        run = combine<OP>(run, agg[i]);
    Agg tot;
    Agg c = block_exclusive<OP, T>(run, &tot);
    for (uint32_t i = a0; i < a1; i++) {
        const Agg me = agg[i];
        agg[i] = c;   // exclusive carry of tile i
        c = combine<OP>(c, me);
    }
}

template <int OP, bool EXCL, class S>
__global__ __launch_bounds__(TILE_THREADS) void k_scan_down(S s, uint32_t n,
                                                            const Agg *carry)
{
    const uint32_t base = blockIdx.x * TILE + threadIdx.x * TILE_ITEMS;
    uint32_t key[TILE_ITEMS];
    uint64_t val[TILE_ITEMS];
    Agg a = agg_none();
#pragma unroll
    for (int k = 0; k < TILE_ITEMS; k++) {
        key[k] = NOKEY;
        val[k] = 0;
        if (base + k < n) {
            key[k] = s.key(base + k);
            val[k] = s.val(base + k);
            a = combine<OP>(a, agg_of(key[k], val[k]));
        }
    }
    Agg tot;
    Agg run = combine<OP>(carry[blockIdx.x], block_exclusive<OP>(a, &tot));
#pragma unroll
    for (int k = 0; k < TILE_ITEMS; k++) {
        if (base + k >= n)
            break;
        const Agg me = agg_of(key[k], val[k]);
        if (EXCL)
            s.store(base + k, run.has && run.lk == key[k] ? run.v : 0);
        run = combine<OP>(run, me);
        if (!EXCL)
            s.store(base + k, run.v);
    }
}

// agg: ceil(n / TILE) entries of scratch
template <int OP, bool EXCL, class S>
hipError_t scan_run(S s, uint32_t n, Agg *agg, hipStream_t st)
{
    if (!n)
        return hipSuccess;
    const uint32_t nt = (n + TILE - 1) / TILE;
    hipLaunchKernelGGL((k_scan_up<OP, S>), dim3(nt), dim3(TILE_THREADS), 0, st,
                       s, n, agg);
    hipLaunchKernelGGL((k_scan_mid<OP>), dim3(1), dim3(1024), 0, st, agg, nt);
    hipLaunchKernelGGL((k_scan_down<OP, EXCL, S>), dim3(nt),
                       dim3(TILE_THREADS), 0, st, s, n, agg);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// stable LSD radix sort
struct HistScan {   // the digit histograms, digit-major: h[d * ntiles + t]
    uint32_t *h;
    __device__ uint32_t key(uint32_t) const { return 0; }
    __device__ uint64_t val(uint32_t i) const { return h[i]; }
    __device__ void store(uint32_t i, uint64_t v) const { h[i] = (uint32_t)v; }
};

__global__ __launch_bounds__(TILE_THREADS) void k_rs_hist(
    const uint32_t *key, uint32_t n, uint32_t shift, uint32_t mask,
    uint32_t ntiles, uint32_t *hist)
{
    __shared__ uint32_t s_c[256];
    s_c[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * TILE;
    for (uint32_t k = threadIdx.x; k < TILE; k += TILE_THREADS)
        if (base + k < n)
            atomicAdd(&s_c[(key[base + k] >> shift) & mask], 1u);
    __syncthreads();
    if (threadIdx.x <= mask)
        hist[threadIdx.x * ntiles + blockIdx.x] = s_c[threadIdx.x];
}

// stable: tile item j = r * 256 + thread, rounds r in order; inside a round
// the lanes of a wave with one digit are ranked by lane, waves by index
__global__ __launch_bounds__(TILE_THREADS) void k_rs_scatter(
    const uint32_t *key, const uint32_t *val, uint32_t n, uint32_t shift,
    uint32_t mask, uint32_t bits, uint32_t ntiles, const uint32_t *hist,
    uint32_t *key_out, uint32_t *val_out)
{
    __shared__ uint32_t s_base[256];                      // running, per digit
    __shared__ uint32_t s_w[TILE_THREADS / 64][256];      // this round, per wave
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    s_base[t] = t <= mask ? hist[t * ntiles + blockIdx.x] : 0;
    for (uint32_t x = t; x < (TILE_THREADS / 64) * 256; x += TILE_THREADS)
        (&s_w[0][0])[x] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * TILE;
    for (int r = 0; r < TILE_ITEMS; r++) {
        const uint32_t i = base + r * TILE_THREADS + t;
        const bool live = i < n;
        const uint32_t k = live ? key[i] : 0;
        const uint32_t d = (k >> shift) & mask;
        uint64_t peers = __ballot(live);
        for (uint32_t b = 0; b < bits; b++) {
            const uint64_t v = __ballot(live && ((d >> b) & 1));
            peers &= ((d >> b) & 1) ? v : ~v;
        }
        const uint32_t below =
            (uint32_t)__popcll((unsigned long long)(peers & ((1ull << lane) - 1)));
        if (live && below == 0)
            s_w[w][d] = (uint32_t)__popcll((unsigned long long)peers);
        __syncthreads();
        if (live) {
            uint32_t pos = s_base[d] + below;
            for (uint32_t u = 0; u < w; u++)
                pos += s_w[u][d];
            key_out[pos] = k;
            val_out[pos] = val[i];
        }
        __syncthreads();
        if (t <= mask) {
            uint32_t add = 0;
            for (uint32_t u = 0; u < TILE_THREADS / 64; u++) {
                add += s_w[u][t];
                s_w[u][t] = 0;
            }
            s_base[t] += add;
        }
        __syncthreads();
    }
}

// sorts (k0, v0) by the low end_bit key bits into (k1, v1), stably; k0 / v0
// are clobbered.  hist: 256 * ceil(n / TILE) words, agg: scan_run scratch
// for that many items.
inline hipError_t radix_sort(uint32_t *k0, uint32_t *v0, uint32_t *k1,
                             uint32_t *v1, uint32_t n, int end_bit,
                             uint32_t *hist, Agg *agg, hipStream_t st)
{
    if (!n)
        return hipSuccess;
    int passes = (end_bit + 7) / 8;
    if (passes < 1)
        passes = 1;
    if (!(passes & 1))
        passes++;   // odd: the last pass lands in (k1, v1)
    const int bits = (end_bit + passes - 1) / passes;
    const uint32_t nt = (n + TILE - 1) / TILE;
    uint32_t *ks = k0, *vs = v0, *kd = k1, *vd = v1;
    for (int p = 0; p < passes; p++) {
        const uint32_t shift = (uint32_t)(p * bits);
        const uint32_t mask = bits >= 8 ? 0xffu : ((1u << bits) - 1);
        hipLaunchKernelGGL(k_rs_hist, dim3(nt), dim3(TILE_THREADS), 0, st, ks,
                           n, shift, mask, nt, hist);
        hipError_t e = scan_run<OP_SUM, true>(HistScan{ hist },
                                              (mask + 1) * nt, agg, st);
        if (e != hipSuccess)
            return e;
        hipLaunchKernelGGL(k_rs_scatter, dim3(nt), dim3(TILE_THREADS), 0, st,
                           ks, vs, n, shift, mask, (uint32_t)bits, nt, hist,
                           kd, vd);
        uint32_t *tk = ks, *tv = vs;
        ks = kd;
        vs = vd;
        kd = tk;
        vd = tv;
    }
    return hipGetLastError();
}

}   // namespace srtp_scan
