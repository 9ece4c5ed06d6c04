// ws_probe.hip -- does splitting the AES (LDS-bound) and SHA-1 (VALU-bound)
// halves of the ICM+HMAC work across different waves of a CU overlap them
// better than every wave doing both in turn?  Compute only (no HBM): each
// wave runs U work units; a unit = the keystream of 4 counter blocks (one
// 64-byte chunk) and/or one SHA-1 compression, as in k_icm_wave.
//   mode 0: every wave: AES chunk then SHA-1 chunk, U times
//   mode 1: even waves 2U AES chunks, odd waves 2U SHA-1 chunks
//   mode 2: AES only (U units), mode 3: SHA-1 only (U units)
// Timing only.  hipcc -O3 --offload-arch=gfx950 -I libsrtp_amd/csrc
//   -I include tools/ws_probe.hip -o tools/ws_probe
#include "srtp_dev_common.h"
#include <stdio.h>

namespace {
// ---------------------------------------------------------------------------
// Fused counter-mode keystream + SHA-1 compression (probe).  AES is
// bound by LDS table reads, SHA-1 by dependent VALU chains; waves that run
// one and then the other lock into phase (all waiting on the LDS, then all
// on the VALU) and the two never overlap.  Here ONE instruction stream
// interleaves them: the 4 counter blocks are encrypted one after the other,
// each AES round split into an issue stage (16 table reads in flight, within
// the 15-deep LGKM counter) and a combine stage, and a slice of SHA-1 rounds
// runs between the two, covering the table-read latency.
struct Sha1Run {
    uint32_t a, b, c, d, e;
};

template <int T0, int T1>
DEV void sha1_rounds(Sha1Run &s, uint32_t (&w)[16])
{
#pragma unroll
    for (int t = T0; t < T1; t++) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = rotl(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^
                          w[t & 15],
                      1);
            w[t & 15] = wt;
        }
        uint32_t f, k;
        if (t < 20) {
            f = __builtin_amdgcn_bitop3_b32(s.b, s.c, s.d, 0xCA);   // b?c:d
            k = 0x5a827999u;
        } else if (t < 40) {
            f = xor3(s.b, s.c, s.d);
            k = 0x6ed9eba1u;
        } else if (t < 60) {
            f = maj3(s.b, s.c, s.d);
            k = 0x8f1bbcdcu;
        } else {
            f = xor3(s.b, s.c, s.d);
            k = 0xca62c1d6u;
        }
        const uint32_t tmp = rotl(s.a, 5) + f + s.e + k + wt;
        s.e = s.d;
        s.d = s.c;
        s.c = rotl(s.b, 30);
        s.b = s.a;
        s.a = tmp;
    }
}

// per-block AES state of the fused loop
struct AesStep {
    uint32_t s[4];
    uint32_t lk[16];
};

// stage STG of the counter-mode encryption of block JB (TAB4 tables):
//   0: the round-1 T3 term (1 read)      1: round-2 terms of column 0 (4)
//   2: round-2 state, issue round 3     r: combine round r, issue round r+1
//   NR: combine the final round into ks
template <int STG, int NR, class KEY>
DEV void ctr_stage(AesStep &A, uint32_t jb, const CtrCache &C, const KEY &rk,
                   const AesLds &T, uint32_t (&ks)[4])
{
    if constexpr (STG == 0) {
        A.lk[0] = lds_rd(T, C.a3 ^ jb);
    } else if constexpr (STG == 1) {
        const uint32_t u0 = C.k1 ^ A.lk[0];
        A.lk[0] = tl<0, 0>(T, u0);
        A.lk[1] = tl<1, 1>(T, u0);
        A.lk[2] = tl<2, 2>(T, u0);
        A.lk[3] = tl<3, 3>(T, u0);
    } else {
        if constexpr (STG == 2) {
            A.s[0] = C.k2[0] ^ A.lk[0];
            A.s[1] = C.k2[1] ^ A.lk[3];
            A.s[2] = C.k2[2] ^ A.lk[2];
            A.s[3] = C.k2[3] ^ A.lk[1];
        } else if constexpr (STG < NR) {
            // combine round STG (issued at stage STG - 1)
            uint32_t n[4];
#pragma unroll
            for (int q = 0; q < 4; q++)
                n[q] = xor3(xor3(A.lk[4 * q], A.lk[4 * ((q + 1) & 3) + 1],
                                 A.lk[4 * ((q + 2) & 3) + 2]),
                            A.lk[4 * ((q + 3) & 3) + 3], rk(4 * (STG - 1) + q));
#pragma unroll
            for (int q = 0; q < 4; q++)
                A.s[q] = n[q];
        }
        if constexpr (STG < NR - 1) {
            // issue round STG + 1: lk[4q + k] = T_k[byte k of column q]
#pragma unroll
            for (int q = 0; q < 4; q++) {
                A.lk[4 * q + 0] = tl<0, 0>(T, A.s[q]);
                A.lk[4 * q + 1] = tl<1, 1>(T, A.s[q]);
                A.lk[4 * q + 2] = tl<2, 2>(T, A.s[q]);
                A.lk[4 * q + 3] = tl<3, 3>(T, A.s[q]);
            }
        } else if constexpr (STG == NR - 1) {
            // issue the final round: S at byte k taken from T_(k+2 mod 4)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                A.lk[4 * q + 0] = tl<2, 0>(T, A.s[q]);
                A.lk[4 * q + 1] = tl<3, 1>(T, A.s[q]);
                A.lk[4 * q + 2] = tl<0, 2>(T, A.s[q]);
                A.lk[4 * q + 3] = tl<1, 3>(T, A.s[q]);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; q++)
                ks[q] = xor3(__builtin_amdgcn_perm(A.lk[4 * ((q + 1) & 3) + 1],
                                                   A.lk[4 * q], 0x0c0c0500u),
                             __builtin_amdgcn_perm(A.lk[4 * ((q + 3) & 3) + 3],
                                                   A.lk[4 * ((q + 2) & 3) + 2],
                                                   0x07020c0cu),
                             rk(4 * NR + q));
        }
    }
}

// step K of NK: AES stage K % (NR+1) of block K / (NR+1), then the K-th
// slice of the 80 SHA-1 rounds
template <int K, int NK, int NR, class KEY>
DEV void fused_steps(AesStep &A, const uint32_t (&jb)[4], const CtrCache &C,
                     const KEY &rk, const AesLds &T, uint32_t (&ks)[4][4],
                     Sha1Run &sh, uint32_t (&w)[16])
{
    if constexpr (K < NK) {
        constexpr int STG = K % (NR + 1), BLK = K / (NR + 1);
        ctr_stage<STG, NR>(A, jb[BLK], C, rk, T, ks[BLK]);
        sha1_rounds<80 * K / NK, 80 * (K + 1) / NK>(sh, w);
#ifndef FUSED_NO_SCHED_BARRIER
        __builtin_amdgcn_sched_barrier(0);
#endif
        fused_steps<K + 1, NK, NR>(A, jb, C, rk, T, ks, sh, w);
    }
}

// ks <- keystream of the 4 counter blocks jb (cached epoch), and
// hst <- SHA1-compress(hst, w), interleaved
template <int NR, class KEY>
DEV void ctr4_sha1(uint32_t (&ks)[4][4], const uint32_t (&jb)[4],
                   const CtrCache &C, const KEY &rk, const AesLds &T,
                   uint32_t hst[5], uint32_t (&w)[16])
{
    AesStep A;
    Sha1Run sh{ hst[0], hst[1], hst[2], hst[3], hst[4] };
    fused_steps<0, 4 * (NR + 1), NR>(A, jb, C, rk, T, ks, sh, w);
    hst[0] += sh.a;
    hst[1] += sh.b;
    hst[2] += sh.c;
    hst[3] += sh.d;
    hst[4] += sh.e;
}

}   // namespace

template <int MODE, int THREADS>
__global__ __launch_bounds__(THREADS) void k_probe(uint32_t *out, uint32_t U,
                                                   uint32_t seed)
{
    __shared__ u32x4 s_tab[AES_TAB4_BYTES / 16];
    load_aes_tables<true>(s_tab);
    __syncthreads();
    const AesLds T = make_aes_lds(s_tab);
    UniKey<10> rk;
#pragma unroll
    for (int i = 0; i < 44; i++)
        rk.rk[i] = seed * (i + 1);
    const uint32_t wid = threadIdx.x >> 6;
    uint32_t c[4] = { threadIdx.x * 7u, blockIdx.x, seed, 0 };
    const CtrCache C = ctr_cache<10, true>(c, rk, T);
    uint32_t hst[5] = { 1, 2, 3, 4, (uint32_t)threadIdx.x };
    uint32_t acc = 0;
    const bool doaes = MODE == 0 || MODE == 2 || (MODE == 1 && !(wid & 1));
    const bool dosha = MODE == 0 || MODE == 3 || (MODE == 1 && (wid & 1));
    const uint32_t n = MODE == 1 ? 2 * U : U;
    if (MODE == 5) {   // fused: keystream + SHA-1 interleaved in one stream
        uint32_t w[16];
#pragma unroll
        for (int k = 0; k < 16; k++)
            w[k] = k * 0x01010101u + threadIdx.x;
        for (uint32_t u = 0; u < n; u++) {
            uint32_t ks[4][4];
            const uint32_t jb[4] = { ((4 * u) & 0xffu) << 8,
                                     ((4 * u + 1) & 0xffu) << 8,
                                     ((4 * u + 2) & 0xffu) << 8,
                                     ((4 * u + 3) & 0xffu) << 8 };
            ctr4_sha1<10>(ks, jb, C, rk, T, hst, w);
#pragma unroll
            for (int k = 0; k < 16; k++)
                w[k] = ks[k >> 2][k & 3] + u + k;
        }
        out[blockIdx.x * blockDim.x + threadIdx.x] = hst[0] ^ hst[4];
        return;
    }
    for (uint32_t u = 0; u < n; u++) {
        uint32_t ks[4][4] = {};
        if (doaes) {
#pragma unroll
            for (int g = 0; g < 4; g += 2) {
                const uint32_t jb[2] = { ((4 * u + g) & 0xffu) << 8,
                                         ((4 * u + g + 1) & 0xffu) << 8 };
                aes_ctr<2, 10, true>(
                    *reinterpret_cast<uint32_t(*)[2][4]>(&ks[g]), jb, C, rk, T);
            }
            acc ^= ks[0][0] ^ ks[1][1] ^ ks[2][2] ^ ks[3][3];
        }
        if (dosha) {
            uint32_t w[16];
#pragma unroll
            for (int k = 0; k < 16; k++)
                w[k] = ks[k >> 2][k & 3] + u + k;
            sha1_compress(hst, w);
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc ^ hst[0] ^ hst[4];
}

template <int MODE, int THREADS>
static float run(uint32_t *out, uint32_t U)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int it = 0; it < 7; it++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL((k_probe<MODE, THREADS>), dim3(256), dim3(THREADS),
                           0, 0, out, U, 12345u);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best)
            best = ms;
    }
    return best;
}

int main()
{
    uint32_t *out;
    if (hipMalloc(&out, 256 * 1024 * 4))
        return 1;
    // the bench's work per CU: 4096 packets x 22 chunks = 1408 chunk-waves;
    // U per wave = 1408 / waves per CU
#define ROW(T)                                                                 \
    {                                                                          \
        const uint32_t U = 1408 / (T / 64);                                    \
        printf("threads %4d U %3u: both %.3f ms  split %.3f ms  aes-only "    \
               "%.3f ms  sha-only %.3f ms  fused %.3f ms\n",                   \
               T, U, run<0, T>(out, U), run<1, T>(out, U), run<2, T>(out, U),  \
               run<3, T>(out, U), run<5, T>(out, U));                          \
    }
    ROW(256)
    ROW(512)
    ROW(768)
    ROW(1024)
    return 0;
}
