// srtp_dev_common.h -- CDNA4 (gfx950) device building blocks shared by the
// SRTP kernels (srtp_icm.hip, srtp_gcm.hip, srtp_gpu.hip).
//
//   AES (T-table) crypto/cipher/aes.c:2102-2130 semantics, AES-ICM counter
//   caching (aes_icm.c:236-414), SHA-1 compression (crypto/hash/sha1.c:91-212),
//   GHASH (aes_gcm_ossl.c via OpenSSL EVP semantics), and the lane-quad
//   cooperative memory helpers.
//
//  * AES is T-table based.  The table entries of every byte value live in
//    LDS replicated 32 times so that lane l always hits bank (l & 31): a
//    ds_read_b32 wave instruction is conflict-free for ANY byte values.
//    The LDS address of a lookup is formed by ONE v_perm_b32 (byte k of the
//    state word -> bits 15:8, the lane's copy offset -> bits 7:0).
//  * GHASH (GCM) uses Shoup's 8-bit table M[b] = b*H, 16 B per entry: for
//    uniform keys as 8 per-position tables M[b]*x^(8t) in LDS (GhPos8), for
//    per-lane keys each key's 4-bit table in global memory (GhNib4).
//  * v_bitop3_b32 (gfx950) gives 3-input XOR and majority in one op.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <type_traits>

#include "srtp_dev.h"
#include "srtp_rtp_hdr.h"

#define DEV __device__ __forceinline__

namespace {

// ---------------------------------------------------------------------------
// small integer helpers
DEV uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
DEV uint32_t bswap(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x00010203u); }
DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);   // symmetric table
}
DEV uint32_t maj3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);   // symmetric table
}

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// LDS T-tables.  Tk[x] = rotl(T0[x], 8k), T0[x] = (2s, s, s, 3s) bytes LE,
// s = S[x].  Every table is replicated 32 times so that lane l always reads
// copy l & 31: a ds_read_b32 of 32 lanes touches 32 distinct banks whatever
// the byte values are (never bank-conflicted).  Byte address of Tk[x] for
// lane l:  (k >> 1) << 16 | x << 8 | (k & 1) << 7 | (l & 31) << 2
// i.e. [0, 64K) holds (T0, T1) rows, [64K, 128K) (T2, T3) rows.  The address
// of a lookup is ONE v_perm_b32: byte K of the state word -> bits 15:8, the
// lane's template (table bits + copy offset) -> bytes 0 and 2.
//   TAB4 = true : all four tables (128 KiB); a MixColumns column is
//                 xor3(xor3(T0,T1,T2), T3, rk) = 2 VALU
//   TAB4 = false: T0, T1 only (64 KiB, leaves LDS for the GHASH table);
//                 T2/T3 are rotations: xor3(T0,T1,rk) ^ rotl16(T0' ^ T1')
constexpr int AES_TAB2_BYTES = 256 * 32 * 8;           // 64 KiB
constexpr int AES_TAB4_BYTES = 2 * AES_TAB2_BYTES;     // 128 KiB

// T0[x] = (2s, s, s, 3s) bytes little-endian, s = S[x]: the FIPS-197 5.1.1
// S-box (inverse in GF(2^8), then the affine map) computed on the device, so
// no kernel depends on an uploaded table (the reference transcribes its
// tables, crypto/cipher/aes.c:67-342).
DEV uint32_t gf_mul(uint32_t a, uint32_t b)   // mod x^8 + x^4 + x^3 + x + 1
{
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        r ^= (0u - (b & 1u)) & a;
        b >>= 1;
        a = (a << 1) ^ ((0u - (a >> 7)) & 0x11bu);
    }
    return r;
}

DEV uint32_t aes_t0(uint32_t x)
{
    const uint32_t x2 = gf_mul(x, x), x3 = gf_mul(x2, x), x6 = gf_mul(x3, x3),
                   x12 = gf_mul(x6, x6), x15 = gf_mul(x12, x3),
                   x30 = gf_mul(x15, x15), x60 = gf_mul(x30, x30),
                   x120 = gf_mul(x60, x60), x240 = gf_mul(x120, x120),
                   inv = gf_mul(gf_mul(x240, x12), x2);   // x^254
    const uint32_t r = inv | (inv << 8);
    const uint32_t s = (inv ^ (r >> 7) ^ (r >> 6) ^ (r >> 5) ^ (r >> 4) ^ 0x63u) & 0xffu;
    const uint32_t s2 = ((s << 1) ^ ((0u - (s >> 7)) & 0x11bu)) & 0xffu;
    return s2 | (s << 8) | (s << 16) | ((s2 ^ s) << 24);
}

// The replicated tables from the T0 row s_t0 (written and synchronised
// before): 16-byte stores, the 4 dwords of a store 4 copies of one entry
template <bool TAB4>
DEV void fill_aes_tables(void *lds, const uint32_t *s_t0)
{
    u32x4 *d = (u32x4 *)lds;
    constexpr int N = (TAB4 ? AES_TAB4_BYTES : AES_TAB2_BYTES) / 16;
    for (int e = threadIdx.x; e < N; e += blockDim.x) {
        const int tab = ((e >> 12) << 1) | ((e >> 3) & 1);
        const uint32_t v = rotl(s_t0[(e >> 4) & 255], 8 * tab);
        d[e] = u32x4{ v, v, v, v };
    }
}

// Fills the replicated tables; every thread of the block must call it.  The
// caller synchronises the block before the first lookup.
template <bool TAB4>
DEV void load_aes_tables(void *lds, uint32_t *s_t0)   // s_t0: 1 KiB of LDS
{
    for (int x = threadIdx.x; x < 256; x += blockDim.x)
        s_t0[x] = aes_t0((uint32_t)x);
    __syncthreads();
    fill_aes_tables<TAB4>(lds, s_t0);
}

template <bool TAB4>
DEV void load_aes_tables(void *lds)
{
    __shared__ uint32_t s_t0[256];
    load_aes_tables<TAB4>(lds, s_t0);
}

struct AesLds {
    const char *lds;
    uint32_t L[2];   // lane templates of tables (0,1) and (2,3): bytes 0, 2
};

DEV AesLds make_aes_lds(const void *lds)
{
    AesLds T;
    T.lds = (const char *)lds;
    const uint32_t c = (threadIdx.x & 31) * 4;   // the lane's table copy
    T.L[0] = c;
    T.L[1] = 0x10000u | c;
    return T;
}

// address of T_TAB[byte K of w] for an even TAB; odd tables sit +128 bytes
// further (the ds_read immediate offset)
// Byte 1 is already at bits 15:8: (w & 0xff00) | template is one
// v_bitop3_b32, a full-rate VALU op on gfx950, where v_perm_b32 is
// half-rate (tools/valu_rate.hip: 1.15 vs 1.9 ns per wave-instruction per
// SIMD); the other bytes need the permute.
template <int TAB, int K>
DEV uint32_t ta(const AesLds &T, uint32_t w)
{
    if constexpr (K == 1)
        return __builtin_amdgcn_bitop3_b32(w, 0x0000ff00u, T.L[TAB >> 1], 0xEA);
    return __builtin_amdgcn_perm(w, T.L[TAB >> 1], 0x0c020000u | ((4u + K) << 8));
}

DEV uint32_t lds_rd(const AesLds &T, uint32_t a)
{
    return *(const uint32_t *)(T.lds + a);
}

template <int TAB, int K>
DEV uint32_t tl(const AesLds &T, uint32_t w)
{
    return *(const uint32_t *)(T.lds + ta<TAB, K>(T, w) + (TAB & 1) * 128);
}

// T2 / T3 lookups: direct with four tables, else T0 / T1 to be rotated
template <bool TAB4, int K>
DEV uint32_t tl2(const AesLds &T, uint32_t w) { return tl<TAB4 ? 2 : 0, K>(T, w); }
template <bool TAB4, int K>
DEV uint32_t tl3(const AesLds &T, uint32_t w) { return tl<TAB4 ? 3 : 1, K>(T, w); }

// one MixColumns output column from its four lookups (c, d as returned by
// tl2 / tl3) and the round key word
template <bool TAB4>
DEV uint32_t mixcol(uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                    uint32_t rk)
{
    if (TAB4)
        return xor3(xor3(a, b, c), d, rk);
    return xor3(a, b, rk) ^ rotl(c ^ d, 16);
}

template <bool TAB4>
DEV uint32_t rot2(uint32_t x) { return TAB4 ? x : rotl(x, 16); }

// ---------------------------------------------------------------------------
// key material access: uniform (scalar loads, SGPRs) or per lane (VGPRs)
template <int NR>
struct LaneKey {
    uint32_t rk[4 * (NR + 1)];
    uint32_t slot = 0xffffffffu;   // the slot rk holds (reload(): ~0 none)
    DEV void load(const srtp_dev_key_t *k)
    {
#pragma unroll
        for (int i = 0; i < 4 * (NR + 1); i++)
            rk[i] = k->rk[i];
    }
    // the schedule of slot s, fetched only when the lane's previous packet
    // used another key: a lane's packets often share a stream (a stream's
    // packets in one batch, or configs[3]'s round-robin layout under the
    // persistent grid's stride), and the 176-704-byte gather per packet is
    // then a latency the lane need not pay again
    DEV void reload(const srtp_dev_key_t *keys, uint32_t s)
    {
        if (s == slot)
            return;
        load(keys + s);
        slot = s;
    }
    DEV uint32_t operator()(int i) const { return rk[i]; }
};

// The schedule is read once at kernel entry, before any store, into SGPRs:
// left as loads at the use sites, the compiler must assume the packet stores
// may alias the key table and re-fetches 11 dwordx4 per AES block through
// the vector memory path (measured: ~1000 VMEM reads per wave).
template <int NR>
struct UniKey {
    uint32_t rk[4 * (NR + 1)];
    DEV void load(const srtp_dev_key_t *k)
    {
#pragma unroll
        for (int i = 0; i < 4 * (NR + 1); i++)
            rk[i] = __builtin_amdgcn_readfirstlane(k->rk[i]);
    }
    DEV uint32_t operator()(int i) const { return rk[i]; }
};

// Rounds R0 .. NR-1 and the final round of NB independent blocks, advanced
// round by round together (the NB*16 table reads of a round are issued back
// to back).  State: little-endian words, column c = bytes 4c..4c+3.
//   col_q = T0[s_q.b0] ^ T1[s_q+1.b1] ^ T2[s_q+2.b2] ^ T3[s_q+3.b3] ^ rk
// Final round: S[x] is byte r of T(r+2 mod 4)[x], so row r of the output
// column is taken from that table (TAB4), or byte 1 of T0 / byte 2 of T1.
template <int NB, int NR, bool TAB4, class KEY>
DEV void aes_rounds(uint32_t (&s)[NB][4], const KEY &rk, const AesLds &T,
                    int r0)
{
#pragma unroll
    for (int r = r0; r < NR; r++) {
        uint32_t a[NB][4], b[NB][4], c[NB][4], d[NB][4];
#pragma unroll
        for (int j = 0; j < NB; j++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                a[j][q] = tl<0, 0>(T, s[j][q]);
                b[j][q] = tl<1, 1>(T, s[j][q]);
                c[j][q] = tl2<TAB4, 2>(T, s[j][q]);
                d[j][q] = tl3<TAB4, 3>(T, s[j][q]);
            }
#pragma unroll
        for (int j = 0; j < NB; j++)
#pragma unroll
            for (int q = 0; q < 4; q++)
                s[j][q] = mixcol<TAB4>(a[j][q], b[j][(q + 1) & 3],
                                       c[j][(q + 2) & 3], d[j][(q + 3) & 3],
                                       rk(4 * r + q));
    }
    uint32_t a[NB][4], b[NB][4], c[NB][4], d[NB][4];
#pragma unroll
    for (int j = 0; j < NB; j++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (TAB4) {
                a[j][q] = tl<2, 0>(T, s[j][q]);   // S at byte 0
                b[j][q] = tl<3, 1>(T, s[j][q]);   // S at byte 1
                c[j][q] = tl<0, 2>(T, s[j][q]);   // S at byte 2
                d[j][q] = tl<1, 3>(T, s[j][q]);   // S at byte 3
            } else {
                a[j][q] = tl<0, 0>(T, s[j][q]);   // S at byte 1
                b[j][q] = tl<1, 1>(T, s[j][q]);   // S at byte 2
                c[j][q] = tl<0, 2>(T, s[j][q]);
                d[j][q] = tl<1, 3>(T, s[j][q]);
            }
        }
    const uint32_t LO = TAB4 ? 0x0c0c0500u : 0x0c0c0601u;
    const uint32_t HI = TAB4 ? 0x07020c0cu : 0x06010c0cu;
#pragma unroll
    for (int j = 0; j < NB; j++)
#pragma unroll
        for (int q = 0; q < 4; q++)
            s[j][q] = xor3(__builtin_amdgcn_perm(b[j][(q + 1) & 3], a[j][q], LO),
                           __builtin_amdgcn_perm(d[j][(q + 3) & 3],
                                                 c[j][(q + 2) & 3], HI),
                           rk(4 * NR + q));
}

// full AES encryption of NB blocks
template <int NB, int NR, bool TAB4, class KEY>
DEV void aes_blocks(uint32_t (&s)[NB][4], const KEY &rk, const AesLds &T)
{
#pragma unroll
    for (int j = 0; j < NB; j++)
#pragma unroll
        for (int c = 0; c < 4; c++)
            s[j][c] ^= rk(c);
    aes_rounds<NB, NR, TAB4>(s, rk, T, 1);
}

template <int NR, bool TAB4, class KEY>
DEV void aes_block(uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3,
                   const KEY &rk, const AesLds &T)
{
    uint32_t s[1][4] = { { s0, s1, s2, s3 } };
    aes_blocks<1, NR, TAB4>(s, rk, T);
    s0 = s[0][0];
    s1 = s[0][1];
    s2 = s[0][2];
    s3 = s[0][3];
}

// ---------------------------------------------------------------------------
// Counter-mode caching.  Both SRTP counter modes vary only the last bytes of
// the counter block within a packet: ICM the 16-bit block counter in bytes
// 14..15 (aes_icm.c:266-282, the IV's bytes 14..15 are zero), GCM the 32-bit
// BE counter in bytes 12..15 (inc32).  For the blocks of one "epoch" (all
// bytes but byte 15 fixed -- 256 blocks = 4 KiB of payload) the state after
// round 1 differs only in column 0, through one T3 lookup on byte 15, and
// after round 2 every column differs only through one lookup on that column.
// So rounds 1 and 2 cost 1 + 4 table reads per block instead of 32.
struct CtrCache {
    uint32_t a3;      // LDS address of T3[byte 15 of (ctr ^ rk0)] for jlo = 0
    uint32_t k1;      // round-1 column 0 without its T3 term
    uint32_t k2[4];   // round-2 columns without their column-0 term
};

// c: the counter block with byte 15 = 0 (little-endian words)
template <int NR, bool TAB4, class KEY>
DEV CtrCache ctr_cache(const uint32_t c[4], const KEY &rk, const AesLds &T)
{
    const uint32_t s0 = c[0] ^ rk(0), s1 = c[1] ^ rk(1), s2 = c[2] ^ rk(2),
                   s3 = c[3] ^ rk(3);
    CtrCache C;
    C.a3 = ta<TAB4 ? 3 : 1, 3>(T, s3) | 128u;
    C.k1 = xor3(tl<0, 0>(T, s0), tl<1, 1>(T, s1), rk(4)) ^
           rot2<TAB4>(tl2<TAB4, 2>(T, s2));
    const uint32_t u1 = mixcol<TAB4>(tl<0, 0>(T, s1), tl<1, 1>(T, s2),
                                     tl2<TAB4, 2>(T, s3), tl3<TAB4, 3>(T, s0),
                                     rk(5));
    const uint32_t u2 = mixcol<TAB4>(tl<0, 0>(T, s2), tl<1, 1>(T, s3),
                                     tl2<TAB4, 2>(T, s0), tl3<TAB4, 3>(T, s1),
                                     rk(6));
    const uint32_t u3 = mixcol<TAB4>(tl<0, 0>(T, s3), tl<1, 1>(T, s0),
                                     tl2<TAB4, 2>(T, s1), tl3<TAB4, 3>(T, s2),
                                     rk(7));
    C.k2[0] = xor3(tl<1, 1>(T, u1), rk(8),
                   rot2<TAB4>(tl2<TAB4, 2>(T, u2)) ^
                       rot2<TAB4>(tl3<TAB4, 3>(T, u3)));
    C.k2[1] = xor3(tl<0, 0>(T, u1), tl<1, 1>(T, u2), rk(9)) ^
              rot2<TAB4>(tl2<TAB4, 2>(T, u3));
    C.k2[2] = xor3(tl<0, 0>(T, u2), tl<1, 1>(T, u3), rk(10)) ^
              rot2<TAB4>(tl3<TAB4, 3>(T, u1));
    C.k2[3] = xor3(tl<0, 0>(T, u3), rk(11),
                   rot2<TAB4>(tl2<TAB4, 2>(T, u1)) ^
                       rot2<TAB4>(tl3<TAB4, 3>(T, u2)));
    return C;
}

// NB counter blocks of the cached epoch; jb[j] = (byte 15 of block j) << 8
template <int NB, int NR, bool TAB4, class KEY>
DEV void aes_ctr(uint32_t (&s)[NB][4], const uint32_t (&jb)[NB],
                 const CtrCache &C, const KEY &rk, const AesLds &T)
{
    uint32_t u0[NB];
#pragma unroll
    for (int j = 0; j < NB; j++)
        u0[j] = C.k1 ^ rot2<TAB4>(lds_rd(T, C.a3 ^ jb[j]));
    uint32_t a[NB], b[NB], c[NB], d[NB];
#pragma unroll
    for (int j = 0; j < NB; j++) {
        a[j] = tl<0, 0>(T, u0[j]);
        b[j] = tl<1, 1>(T, u0[j]);
        c[j] = tl2<TAB4, 2>(T, u0[j]);
        d[j] = tl3<TAB4, 3>(T, u0[j]);
    }
#pragma unroll
    for (int j = 0; j < NB; j++) {
        s[j][0] = C.k2[0] ^ a[j];
        s[j][1] = C.k2[1] ^ rot2<TAB4>(d[j]);
        s[j][2] = C.k2[2] ^ rot2<TAB4>(c[j]);
        s[j][3] = C.k2[3] ^ b[j];
    }
    aes_rounds<NB, NR, TAB4>(s, rk, T, 3);
}

// ---------------------------------------------------------------------------
// SHA-1 compression (FIPS 180-4), W[] big-endian message words (clobbered)
DEV void sha1_compress(uint32_t h[5], uint32_t w[16])
{
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
    for (int t = 0; t < 80; t++) {
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
            f = (b & c) | (~b & d);
            k = 0x5a827999u;
        } else if (t < 40) {
            f = xor3(b, c, d);
            k = 0x6ed9eba1u;
        } else if (t < 60) {
            f = maj3(b, c, d);
            k = 0x8f1bbcdcu;
        } else {
            f = xor3(b, c, d);
            k = 0xca62c1d6u;
        }
        uint32_t tmp = rotl(a, 5) + f + e + k + wt;
        e = d;
        d = c;
        c = rotl(b, 30);
        b = a;
        a = tmp;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
}

// ---------------------------------------------------------------------------
// byte-precise stores for packet tails
DEV void store_bytes(uint8_t *p, uint32_t w, int n)
{
    // w little-endian: byte 0 first
    if (n >= 4) {
        if (((uintptr_t)p & 3) == 0) {
            *(uint32_t *)p = w;
            return;
        }
    }
    for (int i = 0; i < n && i < 4; i++)
        p[i] = (uint8_t)(w >> (8 * i));
}

// The first n bytes of the little-endian words w at p (an authentication
// tag): whole words as dword stores when p is 4-byte aligned (the usual
// case: a tag follows a 4-byte-aligned RTP payload end), the rest byte by
// byte.  A 10-byte HMAC-SHA1-80 tag is then 3 store instructions instead of
// 10 partial-line stores per lane.
template <int NW>
DEV void store_tag(uint8_t *p, const uint32_t (&w)[NW], uint32_t n)
{
    const bool al = ((uintptr_t)p & 3) == 0;
#pragma unroll
    for (int j = 0; j < NW; j++) {
        const int r = (int)n - 4 * j;
        if (r <= 0)
            break;
        if (r >= 4 && al) {
            *(uint32_t *)(p + 4 * j) = w[j];
            continue;
        }
#pragma unroll
        for (int b = 0; b < 4; b++)
            if (b < r)
                p[4 * j + b] = (uint8_t)(w[j] >> (8 * b));
    }
}

// OR of the differences between the n tag bytes at p and those of w (zero
// when equal; every byte is read, constant time in the data)
template <int NW>
DEV uint32_t tag_diff(const uint8_t *p, const uint32_t (&w)[NW], uint32_t n)
{
    const bool al = ((uintptr_t)p & 3) == 0;
    uint32_t diff = 0;
#pragma unroll
    for (int j = 0; j < NW; j++) {
        const int r = (int)n - 4 * j;
        if (r <= 0)
            break;
        if (r >= 4 && al) {
            diff |= *(const uint32_t *)(p + 4 * j) ^ w[j];
            continue;
        }
#pragma unroll
        for (int b = 0; b < 4; b++)
            if (b < r)
                diff |= (uint32_t)(p[4 * j + b] ^ (uint8_t)(w[j] >> (8 * b)));
    }
    return diff;
}

typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));
typedef uint32_t u32x3a4 __attribute__((ext_vector_type(3), aligned(4)));

DEV void store_words_partial(uint8_t *p, const uint32_t *w, int nbytes)
{
    // store the first nbytes (0..16) of 4 LE words at p (p 4-byte aligned):
    // the whole words in one store instruction, then the bytes left
    const int nw = nbytes >> 2;
    if (nw == 4)
        *(u32x4a4 *)p = u32x4a4{ w[0], w[1], w[2], w[3] };
    else if (nw == 3)
        *(u32x3a4 *)p = u32x3a4{ w[0], w[1], w[2] };
    else if (nw == 2)
        *(u32x2a4 *)p = u32x2a4{ w[0], w[1] };
    else if (nw == 1)
        *(uint32_t *)p = w[0];
    if ((nbytes & 3) == 0 || nw == 4)
        return;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if (i != nw)
            continue;
        store_bytes(p + 4 * i, w[i], nbytes & 3);
    }
}

// select word t of the keystream shifted right by s words:
// out[t] = (t >= s) ? cur[t - s] : prev[t - s + 4]
DEV void ks_shift(const uint32_t prev[4], const uint32_t cur[4], uint32_t s,
                  uint32_t out[4])
{
    uint32_t w[8] = { prev[0], prev[1], prev[2], prev[3],
                      cur[0],  cur[1],  cur[2],  cur[3] };
    bool b1 = (s & 2) != 0, b0 = (s & 1) != 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
        uint32_t x = b1 ? w[t + 2] : w[t + 4];
        uint32_t y = b1 ? w[t + 1] : w[t + 3];
        out[t] = b0 ? y : x;
    }
}

// SHA message word at absolute byte offset o for a message whose data part
// is L bytes and is followed by the 4-byte ROC and the 0x80 terminator.
DEV uint32_t tail_word(uint32_t data_be, int rem, uint32_t roc)
{
    // rem = L - o
    if (rem >= 4)
        return data_be;
    if (rem > 0) {
        uint32_t keep = ~(0xffffffffu >> (8 * rem));
        return (data_be & keep) | (roc >> (8 * rem));
    }
    int k = -rem;   // byte offset into ROC(4) || 80 00 00 00
    uint64_t e = ((uint64_t)roc << 32) | 0x80000000u;
    if (k >= 8)
        return 0;
    return (uint32_t)((e << (8 * k)) >> 32);
}

// ---------------------------------------------------------------------------
// Wave-cooperative steady state (uniform-key batches).  One lane per packet
// makes every wave instruction touch 64 packets 1424 B apart: measured on
// MI355X (tools/memtest.hip) such a copy streams at 2.2-2.7 TB/s, and the
// stores are the worse half -- a 64-B chunk of a packet is rarely 64-B
// aligned, so every aligned 64-B segment is written in two pieces ~1 us
// apart.  Here the four lanes of a lane-quad move 64 contiguous bytes of ONE
// packet per instruction, and stores are whole aligned 64-B segments:
//   * lane L owns packet 16*(L&3) + (L>>2) of the wave's 64, so quad m holds
//     packets m, 16+m, 32+m, 48+m and every exchange stays inside the quad;
//   * load instruction j: lanes 4m..4m+3 read chunk b (64 B) of packet
//     16j+m; a 4x4 transpose of 16-B elements (DPP quad_perm + selects)
//     hands each lane its own packet's chunk;
//   * the output of chunk b-1 and b, funnel-shifted by the packet's 16-B
//     misalignment r0, is aligned segment b; transposed back, instruction j
//     stores segment b of packet 16j+m as 64 contiguous aligned bytes.
// Measured copy rates of these shapes: quad loads 4.9 TB/s read-only,
// quad + aligned copy 3.6-3.8 TB/s, vs 2.4 / 2.65 for lane-per-packet.
template <int CTRL>
DEV uint32_t qperm(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}

// m ? a : b on all lanes (a bit-select: written as a ternary the compiler
// turns the DPP operand into an exec-masked branch, and a DPP read from a
// lane that is masked off returns 0)
DEV uint32_t bsel(uint32_t m, uint32_t a, uint32_t b)
{
    return __builtin_amdgcn_bitop3_b32(a, b, m, 0xE4);
}

typedef const u32x4 __attribute__((address_space(1))) *gcptr;
typedef u32x4 __attribute__((address_space(1))) *gptr;

template <int J>
DEV uint64_t qbcast64(uint64_t v)   // value of lane (L & ~3) + J
{
    constexpr int C = J | (J << 2) | (J << 4) | (J << 6);
    const uint32_t lo = qperm<C>((uint32_t)v), hi = qperm<C>((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Y[t] of lane j (in its quad) = X[j] of lane t: 4x4 transpose of 16-B
// elements inside each lane quad, in two 2x2 stages
DEV void quad_transpose(u32x4 (&x)[4])
{
    const uint32_t q = threadIdx.x & 3;
    const uint32_t j1 = 0u - ((q >> 1) & 1), j0 = 0u - (q & 1);   // masks
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const uint32_t x0 = x[0][c], x1 = x[1][c], x2 = x[2][c], x3 = x[3][c];
        const uint32_t p0 = qperm<0x4E>(x0), p1 = qperm<0x4E>(x1),
                       p2 = qperm<0x4E>(x2), p3 = qperm<0x4E>(x3);
        const uint32_t z0 = bsel(j1, p2, x0), z2 = bsel(j1, x2, p0);
        const uint32_t z1 = bsel(j1, p3, x1), z3 = bsel(j1, x3, p1);
        const uint32_t r0 = qperm<0xB1>(z0), r1 = qperm<0xB1>(z1),
                       r2 = qperm<0xB1>(z2), r3 = qperm<0xB1>(z3);
        x[0][c] = bsel(j0, r1, z0);
        x[1][c] = bsel(j0, z1, r0);
        x[2][c] = bsel(j0, r3, z2);
        x[3][c] = bsel(j0, z3, r2);
    }
}

// aligned segment = quads [4 - r0, 8 - r0) of prev ++ cur
DEV void seg_funnel(const u32x4 (&prev)[4], const u32x4 (&cur)[4], uint32_t r0,
                    u32x4 (&seg)[4])
{
    const uint32_t a = 0u - ((r0 >> 1) & 1), c = 0u - (r0 & 1);   // masks
    u32x4 e[5];   // e[k + 1] = C[4 - 2a + k], k = -1..3
#pragma unroll
    for (int u = 0; u < 4; u++) {
        e[0][u] = bsel(a, prev[1][u], prev[3][u]);
        e[1][u] = bsel(a, prev[2][u], cur[0][u]);
        e[2][u] = bsel(a, prev[3][u], cur[1][u]);
        e[3][u] = bsel(a, cur[0][u], cur[2][u]);
        e[4][u] = bsel(a, cur[1][u], cur[3][u]);
    }
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int u = 0; u < 4; u++)
            seg[t][u] = bsel(c, e[t][u], e[t + 1][u]);
}

// per-lane targets of the cooperative loads / stores: for j = 0..3 the
// packet owned by lane (L & ~3) + j
struct CoopPtr {
    const uint8_t *in[4];    // + 16 * (L & 3): this lane's quad of a chunk
    uint8_t *seg[4];         // aligned segment 0 base + 16 * (L & 3)
};

// ---------------------------------------------------------------------------
// GHASH: X held as big-endian words (x^0 = bit 31 of x0).  The device arena
// keeps each key's Shoup 8-bit table M[b] = b * H (16 B per entry, bit 7 of
// b = x^0) with the nibbles of the entry index swapped: entry q holds
// M[ghash_nswap(q)].  Its first 16 entries are then M[v << 4] = v * H (bit 3
// of v = x^0) -- the 4-bit table, 256 contiguous bytes, that the per-lane
// form (GhNib4) reads.
__host__ __device__ __forceinline__ uint32_t ghash_nswap(uint32_t b)
{
    return ((b & 15u) << 4) | (b >> 4);
}

// multiplies a GHASH value by x^8: the byte shifted out of word 3 (x^128..
// x^135) is folded back by x^128 = 1 + x + x^2 + x^7 (as in ghash_mul)
DEV u32x4 ghash_mulx8(u32x4 z)
{
    const uint32_t o = z.w << 24;
    u32x4 r;
    r.w = __builtin_amdgcn_alignbit(z.z, z.w, 8);
    r.z = __builtin_amdgcn_alignbit(z.y, z.z, 8);
    r.y = __builtin_amdgcn_alignbit(z.x, z.y, 8);
    r.x = xor3(xor3(z.x >> 8, o, o >> 1), o >> 2, o >> 7);
    return r;
}

// Per-position tables for uniform-key GHASH (32 KiB after the four AES
// tables, 160 KiB in all): table t holds M_t[b] = M[b] * x^(8t), t = 0..7
// (M = Shoup's table, byte position 0), entry b of table t at base +
// (b * 8 + t) * 16.  X * H is then
//   sum over bytes 0..7 of M_k[X_k]  +  x^64 * sum over bytes 8..15 of
//   M_(k-8)[X_k]
// -- 16 lookups and XORs, one multiply by x^64 (a 64-bit fold), instead of
// Shoup's 16 shift-and-reduce steps.  Bank spread: lane L walks the bytes
// of each half in the order s ^ r, r = L & 7 (its X halves are byte-permuted
// once per multiply), so the 16 lanes of a ds_read_b128 group read 8
// different tables at every step; two lanes share a table and conflict only
// when their entries have the same parity.
struct GhPos8 {
    const char *lds;   // LDS base (address 0)
    uint32_t tmpl0;    // table base | (r << 4): the table of step 0
    uint32_t sel;      // v_perm selector: LE byte i <- byte i ^ (r & 3)
    uint32_t swap;     // r & 4: swap the two words of a half
    DEV void init(const char *l, uint32_t base, uint32_t lane)
    {
        const uint32_t r = lane & 7, q = r & 3;
        lds = l;
        tmpl0 = base | (r << 4);
        sel = (0u ^ q) | ((1u ^ q) << 8) | ((2u ^ q) << 16) | ((3u ^ q) << 24);
        swap = r & 4;
    }
    // the 8 lookups of one half (words a, b = bytes 0..3, 4..7) into acc
    DEV void half(uint32_t a, uint32_t b, u32x4 &acc) const
    {
        a = __builtin_amdgcn_perm(0u, a, sel);
        b = __builtin_amdgcn_perm(0u, b, sel);
        const uint32_t w0 = swap ? b : a, w1 = swap ? a : b;
        u32x4 e[8];
#pragma unroll
        for (int st = 0; st < 8; st++) {
            const uint32_t w = st < 4 ? w0 : w1;
            const int k = st & 3;   // BE byte of w
            const uint32_t f = k == 3 ? (w << 7) : (w >> (17 - 8 * k));
            e[st] = *(const u32x4 *)(lds + __builtin_amdgcn_bitop3_b32(
                                               f, 0x7f80u,
                                               tmpl0 ^ ((uint32_t)st << 4), 0xEA));
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t t0 = xor3(e[0][u], e[1][u], e[2][u]);
            const uint32_t t1 = xor3(e[3][u], e[4][u], e[5][u]);
            const uint32_t t2 = xor3(e[6][u], e[7][u], acc[u]);
            acc[u] = xor3(t0, t1, t2);
        }
    }
};

// Z = X * H by Horner over the bytes of X, last byte first (Shoup's 8-bit
// table M[b] = b * H).  Each step multiplies Z by x^8: the byte leaving Z
// (coefficients x^128..x^135) would be reduced at once by
// x^128 = 1 + x + x^2 + x^7; here it is shifted into a fifth word o
// instead, and every 4 steps the 32 collected coefficients x^128..x^159
// (o bit j <-> x^(159-j)) are folded back in one go:
//   word 0 ^= o ^ o>>1 ^ o>>2 ^ o>>7,  word 1 ^= o<<31 ^ o<<30 ^ o<<25
// (6 shifts per 4 steps instead of 4 per step: the shifts are half-rate
// VALU on gfx950, tools/valu_rate.hip).
template <class TAB>
DEV void ghash_mul(uint32_t x[4], const TAB &T)
{
    u32x4 z = T.get(x[3], 3);
    uint32_t o = 0;
#pragma unroll
    for (int k = 14; k >= 0; k--) {
        u32x4 mv = T.get(x[k >> 2], k & 3);
        o = __builtin_amdgcn_alignbit(z.w, o, 8);
        u32x4 nz;
        nz.w = __builtin_amdgcn_alignbit(z.z, z.w, 8) ^ mv.w;
        nz.z = __builtin_amdgcn_alignbit(z.y, z.z, 8) ^ mv.z;
        nz.y = __builtin_amdgcn_alignbit(z.x, z.y, 8) ^ mv.y;
        nz.x = (z.x >> 8) ^ mv.x;
        z = nz;
        if (k % 4 == 3 || k == 0) {
            z.x = xor3(xor3(z.x, o, o >> 1), o >> 2, o >> 7);
            z.y = xor3(z.y, o << 31, o << 30) ^ (o << 25);
            o = 0;
        }
    }
    x[0] = z.x;
    x[1] = z.y;
    x[2] = z.z;
    x[3] = z.w;
}

// Per-lane keys: X * H by Horner over the 32 nibbles of X with the key's
// 4-bit table (GhNib4) in global memory, 256 bytes a key.  With 64k keys
// the 8-bit tables (4 KiB each, 256 MiB in all) missed in L2 on almost
// every lookup (116x the algorithmic read bytes); a 4-bit table is four
// 64-byte lines that stay cached for a packet's multiplies.  The 32 lookups
// depend only on X, so they go out in groups of 4 ahead of the shifts; the
// bits shifted out collect in o and fold back every 8 steps, as in
// ghash_mul above.
struct GhNib4 {
    const u32x4 *t;   // the key's 16 entries v * H
    DEV u32x4 nib(uint32_t v) const { return t[v]; }
    DEV void load(const uint32_t *arena, uint32_t gslot)
    {
        t = (const u32x4 *)(arena + 1024 * (size_t)gslot);
    }
};

// ... copied into the lane's own 256 bytes of LDS (the per-lane k_gcm):
// lane-private, so no barrier; entry v at (v + rot) mod 16, rot = lane mod
// 16, so that the 16 lanes of a ds_read_b128 group asking for the same v
// read different banks.  Copied again only when the lane's key changes.
typedef __attribute__((address_space(3))) u32x4 *LdsQuad;
struct GhNib4L {
    LdsQuad t;
    uint32_t rot;
    uint32_t slot;   // the GHASH slot the copy holds (~0: none)
    DEV u32x4 nib(uint32_t v) const { return t[(v + rot) & 15u]; }
    DEV void load(const uint32_t *arena, uint32_t gslot)
    {
        if (gslot == slot)
            return;
        const u32x4 *src = (const u32x4 *)(arena + 1024 * (size_t)gslot);
        u32x4 v[16];
#pragma unroll
        for (uint32_t e = 0; e < 16; e++)
            v[e] = src[e];
#pragma unroll
        for (uint32_t e = 0; e < 16; e++)
            t[(e + rot) & 15u] = v[e];
        slot = gslot;
    }
};

template <class NT>
DEV void ghash_mul_nib(uint32_t x[4], const NT &T)
{
    u32x4 z = { 0, 0, 0, 0 };   // (shifting the zero start is harmless)
    uint32_t o = 0;
    // a rolled loop: unrolled, the 32 lookups all go out at once and the
    // per-lane kernel (256 VGPRs already) spills
#pragma unroll 1
    for (int q = 7; q >= 0; q--) {   // nibbles 4q .. 4q + 3 (word q / 2)
        const uint32_t w = q >= 6 ? x[3] : q >= 4 ? x[2] : q >= 2 ? x[1] : x[0];
        const uint32_t hi = (q & 1) ? 0u : 16u;
        u32x4 e[4];
#pragma unroll
        for (int s = 0; s < 4; s++)
            e[s] = T.nib((w >> (hi + 12 - 4 * s)) & 15u);
#pragma unroll
        for (int s = 3; s >= 0; s--) {
            o = __builtin_amdgcn_alignbit(z.w, o, 4);
            u32x4 nz;
            nz.w = __builtin_amdgcn_alignbit(z.z, z.w, 4) ^ e[s].w;
            nz.z = __builtin_amdgcn_alignbit(z.y, z.z, 4) ^ e[s].z;
            nz.y = __builtin_amdgcn_alignbit(z.x, z.y, 4) ^ e[s].y;
            nz.x = (z.x >> 4) ^ e[s].x;
            z = nz;
        }
        if ((q & 1) == 0) {   // 8 shifts since the last fold
            z.x = xor3(xor3(z.x, o, o >> 1), o >> 2, o >> 7);
            z.y = xor3(z.y, o << 31, o << 30) ^ (o << 25);
            o = 0;
        }
    }
    x[0] = z.x;
    x[1] = z.y;
    x[2] = z.z;
    x[3] = z.w;
}

DEV void ghash_mul(uint32_t x[4], const GhNib4 &T) { ghash_mul_nib(x, T); }
DEV void ghash_mul(uint32_t x[4], const GhNib4L &T) { ghash_mul_nib(x, T); }

DEV void ghash_mul(uint32_t x[4], const GhPos8 &T)
{
    u32x4 lo = { 0, 0, 0, 0 }, hi = { 0, 0, 0, 0 };
    T.half(x[0], x[1], lo);
    T.half(x[2], x[3], hi);
    // hi * x^64: words move down two places; the 64 bits leaving word 3
    // (x^128..x^191, O = hi.z:hi.w at x^0..x^63) fold back as
    // O * (1 + x + x^2 + x^7), which stays below x^71
    const uint32_t a = hi.z, b = hi.w;
    x[0] = xor3(xor3(lo.x, a, a >> 1), a >> 2, a >> 7);
    x[1] = xor3(xor3(lo.y, b, __builtin_amdgcn_alignbit(a, b, 1)),
                __builtin_amdgcn_alignbit(a, b, 2),
                __builtin_amdgcn_alignbit(a, b, 7));
    x[2] = xor3(xor3(lo.z, hi.x, b << 31), b << 30, b << 25);
    x[3] = lo.w ^ hi.y;
}

struct GlobalKey {
    const srtp_dev_key_t *k;
    DEV uint32_t operator()(int i) const { return k->rk[i]; }
};

DEV u32x4 load_partial(const uint8_t *p, int nbytes)
{
    // load up to 16 bytes from a 4-byte aligned p, zero beyond nbytes
    u32x4 v = { 0, 0, 0, 0 };
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int n = nbytes - 4 * i;
        if (n >= 4) {
            v[i] = *(const uint32_t *)(p + 4 * i);
        } else if (n > 0) {
            uint32_t w = 0;
            for (int b = 0; b < n; b++)
                w |= (uint32_t)p[4 * i + b] << (8 * b);
            v[i] = w;
        }
    }
    return v;
}

}   // namespace
