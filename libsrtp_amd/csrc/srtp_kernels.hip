// srtp_kernels.hip -- CDNA4 (gfx950) kernels for the SRTP RTP hot path.
//
// Replaces, on the GPU, the per-packet crypto that libsrtp's srtp_protect /
// srtp_unprotect run through the cipher/auth vtables:
//   AES-ICM   crypto/cipher/aes_icm.c:236-414  (+ aes.c:2102-2130)
//   HMAC-SHA1 crypto/hash/hmac.c:157-229, crypto/hash/sha1.c:91-463
//   AES-GCM   crypto/cipher/aes_gcm_ossl.c:214-389 (OpenSSL EVP semantics)
// driven as in srtp/srtp.c:2493-2818 (protect), 2820-3172 (unprotect),
// 2088-2267 / 2276-2491 (AEAD).
//
// Mapping (DESIGN.md "Kernels"):
//  * one LANE per packet.  SHA-1 is a serial 80-round chain per 64-byte
//    block and HMAC chains ~23 blocks per 1400-byte packet, so packets -- not
//    blocks -- are the parallel unit; every lane runs the same instruction
//    stream when packet lengths match (no divergence, no cross-lane traffic).
//  * AES is T-table based.  The (T0,T1) pair of every byte value lives in
//    LDS replicated 32 times so that lane l always hits bank pair 2*(l&31):
//    a ds_read_b64 wave instruction is conflict-free for ANY byte values.
//    The LDS address of a lookup is formed by ONE v_perm_b32 (byte k of the
//    state word -> bits 15:8, the lane's copy offset -> bits 7:0).  T2/T3 are
//    rotations: col = T0[a]^T1[b]^rot16(T0[c]^T1[d])^rk.
//  * GHASH (GCM) uses Shoup's 8-bit table M[b] = b*H, 16 B per entry, in LDS
//    replicated 16 times (ds_read_b128 lane groups are 16 lanes), after the
//    AES table; the x^8 reduction is computed in VALU.
//  * v_bitop3_b32 (gfx950) gives 3-input XOR and majority in one op.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
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
constexpr int GH_LDS_BYTES = 256 * 16 * 16;            // 64 KiB

__device__ uint32_t g_t0[256];   // T0[x], little-endian word

template <bool TAB4>
DEV void load_aes_tables(void *lds)
{
    // 16-byte stores: the 4 dwords of a store are 4 copies of one entry
    u32x4 *d = (u32x4 *)lds;
    constexpr int N = (TAB4 ? AES_TAB4_BYTES : AES_TAB2_BYTES) / 16;
    for (int e = threadIdx.x; e < N; e += blockDim.x) {
        const int tab = ((e >> 12) << 1) | ((e >> 3) & 1);
        const uint32_t v = rotl(g_t0[(e >> 4) & 255], 8 * tab);
        d[e] = u32x4{ v, v, v, v };
    }
}

struct AesLds {
    const char *lds;
    uint32_t L[2];   // lane templates of tables (0,1) and (2,3): bytes 0, 2
};

DEV AesLds make_aes_lds(const void *lds)
{
    AesLds T;
    T.lds = (const char *)lds;
    const uint32_t c = (threadIdx.x & 31) * 4;
    T.L[0] = c;
    T.L[1] = 0x10000u | c;
    return T;
}

// address of T_TAB[byte K of w] for an even TAB; odd tables sit +128 bytes
// further (the ds_read immediate offset)
template <int TAB, int K>
DEV uint32_t ta(const AesLds &T, uint32_t w)
{
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
    DEV void load(const srtp_dev_key_t *k)
    {
#pragma unroll
        for (int i = 0; i < 4 * (NR + 1); i++)
            rk[i] = k->rk[i];
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

DEV void store_words_partial(uint8_t *p, const uint32_t *w, int nbytes)
{
    // store the first nbytes (0..16) of 4 LE words at p (p 4-byte aligned)
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int n = nbytes - 4 * i;
        if (n >= 4)
            *(uint32_t *)(p + 4 * i) = w[i];
        else if (n > 0)
            store_bytes(p + 4 * i, w[i], n);
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
// AES-ICM + HMAC-SHA1 protect / unprotect: one lane per packet.
struct IcmArgs {
    const uint8_t *in;
    const uint64_t *in_off;
    uint8_t *out;
    const uint64_t *out_off;
    const srtp_dev_meta_t *meta;
    const srtp_dev_key_t *keys;
    uint8_t *auth_ok;
    const uint32_t *abort;   // device pre-pass fell back: do nothing
    uint32_t n;
    uint32_t uni;   // uniform key slot
};

#ifndef ICM_NB
#define ICM_NB 2   // AES blocks interleaved per round in the steady state
#endif
#ifndef ICM_COOP
#define ICM_COOP 1   // wave-cooperative coalesced loads / aligned stores
#endif

// per-packet constants of the chunk loop
struct IcmPkt {
    const uint8_t *in;
    uint8_t *out;
    uint32_t L;        // end of the authenticated region (header + payload)
    uint32_t hw;       // header words (enc_start / 4)
    uint32_t s;        // hw & 3: keystream word shift inside a 16-byte quad
    uint32_t qoff;     // hw >> 2: quads before the first keystream block
    uint32_t nq;       // quads holding data
    uint32_t nb;       // 64-byte chunks (incl. the SHA-1 tail)
    uint32_t bclean;   // first chunk past the header
    uint32_t P;        // payload bytes
    uint32_t roc;
    bool conf;
    uint32_t cb[4];    // counter block, block counter (bytes 14..15) zero
};

// One 64-byte chunk b of a packet in its general form: header words that
// are not encrypted, quads past the end of the data, the partial last quad
// (kept in tailq, stored once after the chunk loop: a byte-wise store here,
// unrolled per quad, costs ~65 VGPRs), and the ROC / terminator / length
// words of the SHA-1 message tail (sha1.c srtp_sha1_final).  Full AES for
// the keystream blocks that any payload byte uses.
template <int NR, bool TAB4, bool AUTH, bool PROTECT, class KEY>
DEV void icm_chunk(uint32_t b, const IcmPkt &p, const KEY &rk,
                   const AesLds &T, uint32_t ks_prev[4], uint32_t hst[5],
                   uint32_t tailq[4], u32x4 (&oq)[4])
{
    const uint32_t q0 = 4 * b;
    const uint8_t *ip = p.in + 16 * q0;
    uint8_t *op = p.out + 16 * q0;
    u32x4 v[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        v[t] = u32x4{ 0, 0, 0, 0 };
        if (q0 + t < p.nq)
            v[t] = *(const u32x4 *)(ip + 16 * t);
    }
    uint32_t ks[4][4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const uint32_t jj = q0 + t - p.qoff;
        ks[t][0] = p.cb[0];
        ks[t][1] = p.cb[1];
        ks[t][2] = p.cb[2];
        ks[t][3] = p.cb[3] ^ ((jj >> 8) << 16) ^ ((jj & 0xffu) << 24);
    }
    if constexpr (NR > 0) {
        if (p.conf) {
#pragma unroll
            for (int g = 0; g < 4; g += ICM_NB) {
                const int jf = (int)(q0 + g) - (int)p.qoff;
                if (jf + ICM_NB - 1 >= 0 && 16 * jf < (int)p.P)
                    aes_blocks<ICM_NB, NR, TAB4>(
                        *reinterpret_cast<uint32_t(*)[ICM_NB][4]>(&ks[g]), rk,
                        T);
            }
        }
    }
    if (NR == 0 || !p.conf) {
#pragma unroll
        for (int t = 0; t < 4; t++)
            ks[t][0] = ks[t][1] = ks[t][2] = ks[t][3] = 0;
    }
    uint32_t wv[16];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const uint32_t q = q0 + t;
        uint32_t kk[4];
        ks_shift(ks_prev, ks[t], p.s, kk);
        if (b < p.bclean) {
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (4 * q + u < p.hw)
                    kk[u] = 0;   // header words are never encrypted
        }
        uint32_t o[4] = { v[t].x ^ kk[0], v[t].y ^ kk[1], v[t].z ^ kk[2],
                          v[t].w ^ kk[3] };
        oq[t] = u32x4{ o[0], o[1], o[2], o[3] };
        if (16 * q + 16 <= p.L) {
            *(u32x4 *)(op + 16 * t) = u32x4{ o[0], o[1], o[2], o[3] };
        } else if (16 * q < p.L) {
            // the one partial quad: stored after the loop
#pragma unroll
            for (int u = 0; u < 4; u++)
                tailq[u] = o[u];
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            wv[4 * t + u] = bswap(PROTECT ? o[u] : v[t][u]);
            ks_prev[u] = ks[t][u];
        }
    }
    if (AUTH) {
        if (64 * b + 64 > p.L) {
            // message tail: ROC, the 0x80 terminator, zero padding and
            // the bit length (sha1.c srtp_sha1_final)
#pragma unroll
            for (int g = 0; g < 16; g++)
                wv[g] = tail_word(wv[g], (int)p.L - (int)(64 * b + 4 * g),
                                  p.roc);
            if (b == p.nb - 1) {
                wv[14] = 0;
                wv[15] = (64 + p.L + 4) * 8;
            }
        }
        sha1_compress(hst, wv);
    }
}

// A payload chunk in the steady state: four full 16-byte quads, no header
// word, no message tail, all keystream blocks in the cached counter epoch,
// and the keystream word shift S (= header words mod 4) a compile-time
// constant, so aligning the keystream to the quads is register renaming.
// The chunk's data v was loaded ICM_PF chunks earlier (icm_steady_run).
template <int S, int NR, bool TAB4, bool AUTH, bool PROTECT, class KEY>
DEV void icm_steady(uint32_t b, const IcmPkt &p, const u32x4 (&v)[4],
                    const CtrCache &C, const KEY &rk, const AesLds &T,
                    uint32_t ks_prev[4], uint32_t hst[5])
{
    uint8_t *op = p.out + 64 * b;
    uint32_t ks[4][4];
#ifdef ICM_EXP_NOAES   // timing experiment only: no keystream
    if constexpr (false) {
#else
    if constexpr (NR > 0) {
#endif
        if (p.conf) {
            const uint32_t jb0 = ((4 * b - p.qoff) & 0xffu) << 8;
#pragma unroll
            for (int g = 0; g < 4; g += ICM_NB) {
                uint32_t jb[ICM_NB];
#pragma unroll
                for (int j = 0; j < ICM_NB; j++)
                    jb[j] = jb0 + ((uint32_t)(g + j) << 8);
                aes_ctr<ICM_NB, NR, TAB4>(
                    *reinterpret_cast<uint32_t(*)[ICM_NB][4]>(&ks[g]), jb, C,
                    rk, T);
            }
        } else {
#pragma unroll
            for (int t = 0; t < 4; t++)
                ks[t][0] = ks[t][1] = ks[t][2] = ks[t][3] = 0;
        }
    } else {
#pragma unroll
        for (int t = 0; t < 4; t++)
            ks[t][0] = ks[t][1] = ks[t][2] = ks[t][3] = 0;
    }
    uint32_t wv[16];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        u32x4 o;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t k = u >= S ? ks[t][u - S]
                                      : (t ? ks[t - 1][u - S + 4]
                                           : ks_prev[u - S + 4]);
            o[u] = v[t][u] ^ k;
        }
        *(u32x4 *)(op + 16 * t) = o;
#pragma unroll
        for (int u = 0; u < 4; u++)
            wv[4 * t + u] = bswap(PROTECT ? o[u] : v[t][u]);
    }
#pragma unroll
    for (int u = 0; u < 4; u++)
        ks_prev[u] = ks[3][u];
#ifdef ICM_EXP_NOSHA   // timing experiment only: fold instead of compress
    if (AUTH)
        hst[0] ^= xor3(wv[0], wv[5], wv[10]) ^ wv[15];
#else
    if (AUTH)
        sha1_compress(hst, wv);
#endif
}

#ifndef ICM_PF
#define ICM_PF 1   // chunks of packet data loaded ahead of their use
#endif

DEV void load_chunk(u32x4 (&v)[4], const uint8_t *ip)
{
#pragma unroll
    for (int t = 0; t < 4; t++)
        v[t] = *(const u32x4 *)(ip + 16 * t);
}

// The steady chunks [b, e) with the packet data loaded ICM_PF chunks ahead:
// one lane's loads are 16-byte pieces of its own packet (64 lanes, 64
// cache lines per wave instruction), so the HBM latency is hidden only if
// loads stay in flight across the AES + SHA-1 work of whole chunks.
template <int S, int NR, bool TAB4, bool AUTH, bool PROTECT, class KEY>
DEV void icm_steady_run(uint32_t &b, uint32_t e, const IcmPkt &p,
                        const CtrCache &C, const KEY &rk, const AesLds &T,
                        uint32_t ks_prev[4], uint32_t hst[5])
{
    u32x4 ring[ICM_PF][4];
#pragma unroll
    for (int k = 0; k < ICM_PF; k++)
        if (b + k < e)
            load_chunk(ring[k], p.in + 64 * (b + k));
    for (; b < e; b++) {
        u32x4 cur[4];
#pragma unroll
        for (int t = 0; t < 4; t++)
            cur[t] = ring[0][t];
#pragma unroll
        for (int k = 0; k + 1 < ICM_PF; k++)
#pragma unroll
            for (int t = 0; t < 4; t++)
                ring[k][t] = ring[k + 1][t];
        if (b + ICM_PF < e)
            load_chunk(ring[ICM_PF - 1], p.in + 64 * (b + ICM_PF));
        icm_steady<S, NR, TAB4, AUTH, PROTECT>(b, p, cur, C, rk, T, ks_prev,
                                               hst);
    }
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

// keystream of chunk b (4 counter blocks of the cached epoch)
template <int NR, bool TAB4, class KEY>
DEV void coop_keystream(uint32_t b, const IcmPkt &p, const CtrCache &C,
                        const KEY &rk, const AesLds &T, uint32_t (&ks)[4][4])
{
#ifdef ICM_EXP_NOAES   // timing experiment only: no keystream
    if constexpr (false) {
#else
    if constexpr (NR > 0) {
#endif
        if (p.conf) {
            const uint32_t jb0 = ((4 * b - p.qoff) & 0xffu) << 8;
#pragma unroll
            for (int g = 0; g < 4; g += ICM_NB) {
                uint32_t jb[ICM_NB];
#pragma unroll
                for (int j = 0; j < ICM_NB; j++)
                    jb[j] = jb0 + ((uint32_t)(g + j) << 8);
                aes_ctr<ICM_NB, NR, TAB4>(
                    *reinterpret_cast<uint32_t(*)[ICM_NB][4]>(&ks[g]), jb, C,
                    rk, T);
            }
            return;
        }
    }
#pragma unroll
    for (int t = 0; t < 4; t++)
        ks[t][0] = ks[t][1] = ks[t][2] = ks[t][3] = 0;
}

// One cooperative chunk b.  ks holds chunk b's keystream on entry and, when
// NEXT, chunk b+1's on exit: the AES of chunk b+1 and the SHA-1 compression
// of chunk b are independent and sit in one basic block, so the scheduler
// fills the LDS latency of the table rounds with SHA-1 VALU work.
template <bool NEXT, int S, int NR, bool TAB4, bool AUTH, bool PROTECT,
          class KEY>
DEV void coop_step(uint32_t b, const IcmPkt &p, const CtrCache &C,
                   const KEY &rk, const AesLds &T, uint32_t ks_prev[4],
                   uint32_t hst[5], u32x4 (&prev)[4], const CoopPtr &cp,
                   uint32_t r0, u32x4 (&nx)[4], uint32_t (&ks)[4][4])
{
    u32x4 v[4];
#pragma unroll
    for (int j = 0; j < 4; j++)
        v[j] = nx[j];
    if (NEXT) {
#pragma unroll
        for (int j = 0; j < 4; j++)
#ifdef ICM_EXP_L2   // timing experiment only: re-read 2 chunks (cache hits)
            nx[j] = *(gcptr)(cp.in[j] + 64 * (1 + ((b + 1) & 1)));
#else
            nx[j] = *(gcptr)(cp.in[j] + 64 * (b + 1));
#endif
    }
    quad_transpose(v);
    u32x4 o[4];
    uint32_t wv[16];
#pragma unroll
    for (int t = 0; t < 4; t++) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t k = u >= S ? ks[t][u - S]
                                      : (t ? ks[t - 1][u - S + 4]
                                           : ks_prev[u - S + 4]);
            o[t][u] = v[t][u] ^ k;
            wv[4 * t + u] = bswap(PROTECT ? o[t][u] : v[t][u]);
        }
    }
#pragma unroll
    for (int u = 0; u < 4; u++)
        ks_prev[u] = ks[3][u];
    u32x4 sg[4];
    seg_funnel(prev, o, r0, sg);
#pragma unroll
    for (int t = 0; t < 4; t++)
        prev[t] = o[t];
    quad_transpose(sg);
#pragma unroll
    for (int j = 0; j < 4; j++)
#ifdef ICM_EXP_L2
        *(gptr)(cp.seg[j] + 64 * (1 + (b & 1))) = sg[j];
#else
        *(gptr)(cp.seg[j] + 64 * b) = sg[j];
#endif
    if (NEXT)
        coop_keystream<NR, TAB4>(b + 1, p, C, rk, T, ks);
#ifdef ICM_EXP_NOSHA   // timing experiment only: fold instead of compress
    if (AUTH)
        hst[0] ^= xor3(wv[0], wv[5], wv[10]) ^ wv[15];
#else
    if (AUTH)
        sha1_compress(hst, wv);
#endif
}

template <int S, int NR, bool TAB4, bool AUTH, bool PROTECT, class KEY>
DEV void icm_coop_run(uint32_t &b, uint32_t e, const IcmPkt &p,
                      const CtrCache &C, const KEY &rk, const AesLds &T,
                      uint32_t ks_prev[4], uint32_t hst[5], u32x4 (&prev)[4],
                      const CoopPtr &cp, uint32_t r0)
{
    u32x4 nx[4];
#pragma unroll
    for (int j = 0; j < 4; j++)
        nx[j] = *(gcptr)(cp.in[j] + 64 * b);
    uint32_t ks[4][4];
    coop_keystream<NR, TAB4>(b, p, C, rk, T, ks);
    for (; b + 1 < e; b++)
        coop_step<true, S, NR, TAB4, AUTH, PROTECT>(b, p, C, rk, T, ks_prev,
                                                    hst, prev, cp, r0, nx, ks);
    coop_step<false, S, NR, TAB4, AUTH, PROTECT>(b, p, C, rk, T, ks_prev, hst,
                                                 prev, cp, r0, nx, ks);
    b++;
    // quads 4e - r0 .. 4e - 1 (the head of segment e) are not stored yet
#pragma unroll
    for (int t = 1; t < 4; t++)
        if (4 - (int)r0 <= t)
            *(u32x4 *)(p.out + 16 * (4 * e - 4 + t)) = prev[t];
}

// all 64 lanes active and in the same steady state: the cooperative path
DEV bool wave_uniform(uint32_t x)
{
    return __builtin_amdgcn_ballot_w64(x == (uint32_t)__builtin_amdgcn_readfirstlane(x)) ==
           ~0ull;
}

// one packet, front to back: header chunks, steady payload chunks, tail
// chunks, partial quad, outer hash, tag (srtp.c:2694-2818 protect,
// 2987-3093 unprotect: the tag is compared, the caller decides)
template <int NR, bool TAB4, bool AUTH, bool PROTECT, bool UNIFORM, class KEY>
DEV void icm_packet(const IcmArgs &A, uint32_t i, const AesLds &T, KEY &rk)
{
    const srtp_dev_meta_t m = A.meta[i];
    constexpr uint32_t VID = (NR == 0 ? 0u : 8u + 2u * ((NR - 8) / 2)) +
                             (AUTH ? 1u : 0u);
    if (SRTP_META_STATUS(m.info) || SRTP_META_VARIANT(m.info) != VID)
        return;
    const uint32_t slot = UNIFORM ? A.uni : m.key;
    const srtp_dev_key_t *key = A.keys + slot;
    if constexpr (!UNIFORM && NR > 0)
        rk.load(key);

    IcmPkt p;
    p.in = A.in + A.in_off[i];
    p.out = A.out + A.out_off[i];
    const uint32_t enc_start = SRTP_META_ENC_START(m.info);
    p.L = m.len;
    p.hw = enc_start >> 2;
    p.s = p.hw & 3;
    p.qoff = p.hw >> 2;
    p.P = p.L - enc_start;
    p.roc = m.roc;
    p.conf = NR != 0 && key->conf != 0;
    p.nq = (p.L + 15) >> 4;
    p.nb = AUTH ? ((p.L + 12) >> 6) + 1 : ((p.nq + 3) >> 2);
    p.bclean = (p.qoff + 4) >> 2;

    // counter block (little-endian words), block counter j in bytes 14..15
    // (aes_icm.c:236-258 IV formation, srtp.c:2694-2707)
    const uint32_t w0 = *(const uint32_t *)p.in;
    const uint32_t seq = bswap(w0) & 0xffffu;
    p.cb[0] = key->salt[0];
    p.cb[1] = key->salt[1] ^ *(const uint32_t *)(p.in + 8);   // SSRC bytes
    p.cb[2] = key->salt[2] ^ bswap(m.roc);
    p.cb[3] = key->salt[3] ^ (seq >> 8) ^ ((seq & 0xffu) << 8);

    uint32_t hst[5];
#pragma unroll
    for (int k = 0; k < 5; k++)
        hst[k] = AUTH ? key->ipad[k] : 0;

    uint32_t ks_prev[4] = { 0, 0, 0, 0 };
    uint32_t tailq[4] = { 0, 0, 0, 0 };
    u32x4 prev[4];   // output quads of the last chunk done
    uint32_t b = 0;
    for (; b < p.bclean && b < p.nb; b++)
        icm_chunk<NR, TAB4, AUTH, PROTECT>(b, p, rk, T, ks_prev, hst, tailq,
                                           prev);

    // steady chunks: full chunks whose blocks j = 4b+t-qoff stay in counter
    // epoch 0 (j <= 255, 4 KiB of payload)
    uint32_t se = p.L >> 6;
    se = se < ((256 + p.qoff) >> 2) ? se : ((256 + p.qoff) >> 2);
    if (b < se) {
        CtrCache C{};
        if constexpr (NR > 0) {
            if (p.conf)
                C = ctr_cache<NR, TAB4>(p.cb, rk, T);
        }
        bool coop = false;
        if constexpr (UNIFORM && ICM_COOP) {
            // every lane of the wave active, 16-B aligned and in the same
            // steady range / keystream shift: the cooperative path
            const uint32_t al =
                (uint32_t)(((uintptr_t)p.in | (uintptr_t)p.out) & 15);
            coop = wave_uniform(b) && wave_uniform(se) && wave_uniform(p.s) &&
                   wave_uniform(p.conf ? 1u : 0u) &&
                   __builtin_amdgcn_ballot_w64(al == 0) == ~0ull;
        }
        if (coop) {
            const uint64_t lq = 16 * (threadIdx.x & 3);
            const uint64_t pin = (uint64_t)(uintptr_t)p.in;
            const uint64_t seg0 = (uint64_t)(uintptr_t)p.out & ~63ull;
            const uint32_t r0 = (uint32_t)(((uintptr_t)p.out >> 4) & 3);
            CoopPtr cp;
            cp.in[0] = (const uint8_t *)(uintptr_t)(qbcast64<0>(pin) + lq);
            cp.in[1] = (const uint8_t *)(uintptr_t)(qbcast64<1>(pin) + lq);
            cp.in[2] = (const uint8_t *)(uintptr_t)(qbcast64<2>(pin) + lq);
            cp.in[3] = (const uint8_t *)(uintptr_t)(qbcast64<3>(pin) + lq);
            cp.seg[0] = (uint8_t *)(uintptr_t)(qbcast64<0>(seg0) + lq);
            cp.seg[1] = (uint8_t *)(uintptr_t)(qbcast64<1>(seg0) + lq);
            cp.seg[2] = (uint8_t *)(uintptr_t)(qbcast64<2>(seg0) + lq);
            cp.seg[3] = (uint8_t *)(uintptr_t)(qbcast64<3>(seg0) + lq);
            switch (p.s) {
            case 0:
                icm_coop_run<0, NR, TAB4, AUTH, PROTECT>(
                    b, se, p, C, rk, T, ks_prev, hst, prev, cp, r0);
                break;
            case 1:
                icm_coop_run<1, NR, TAB4, AUTH, PROTECT>(
                    b, se, p, C, rk, T, ks_prev, hst, prev, cp, r0);
                break;
            case 2:
                icm_coop_run<2, NR, TAB4, AUTH, PROTECT>(
                    b, se, p, C, rk, T, ks_prev, hst, prev, cp, r0);
                break;
            default:
                icm_coop_run<3, NR, TAB4, AUTH, PROTECT>(
                    b, se, p, C, rk, T, ks_prev, hst, prev, cp, r0);
                break;
            }
        } else {
            switch (p.s) {
            case 0:
                icm_steady_run<0, NR, TAB4, AUTH, PROTECT>(b, se, p, C, rk, T,
                                                           ks_prev, hst);
                break;
            case 1:
                icm_steady_run<1, NR, TAB4, AUTH, PROTECT>(b, se, p, C, rk, T,
                                                           ks_prev, hst);
                break;
            case 2:
                icm_steady_run<2, NR, TAB4, AUTH, PROTECT>(b, se, p, C, rk, T,
                                                           ks_prev, hst);
                break;
            default:
                icm_steady_run<3, NR, TAB4, AUTH, PROTECT>(b, se, p, C, rk, T,
                                                           ks_prev, hst);
                break;
            }
        }
    }
    for (; b < p.nb; b++)
        icm_chunk<NR, TAB4, AUTH, PROTECT>(b, p, rk, T, ks_prev, hst, tailq,
                                           prev);
    if (p.L & 15)
        store_words_partial(p.out + (p.L & ~15u), tailq, (int)(p.L & 15));

    const uint32_t tag_len = key->tag_len;
    const uint32_t mki_size = key->mki_size;
    const uint32_t L = p.L;
    uint8_t *out = p.out;
    if (!AUTH) {
        if (PROTECT && mki_size) {
            for (uint32_t u = 0; u < mki_size; u++)
                out[L + u] = key->mki[u];
        }
        if (!PROTECT)
            A.auth_ok[i] = 1;
        return;
    }

    // outer hash: SHA1(opad || inner)  (hmac.c:181-229)
    uint32_t ow[16];
#pragma unroll
    for (int k = 0; k < 5; k++)
        ow[k] = hst[k];
    ow[5] = 0x80000000u;
#pragma unroll
    for (int k = 6; k < 15; k++)
        ow[k] = 0;
    ow[15] = (64 + 20) * 8;
    uint32_t oh[5];
#pragma unroll
    for (int k = 0; k < 5; k++)
        oh[k] = key->opad[k];
    sha1_compress(oh, ow);

    if (PROTECT) {
        for (uint32_t u = 0; u < mki_size; u++)
            out[L + u] = key->mki[u];
        uint8_t *tp = out + L + mki_size;
        for (uint32_t u = 0; u < tag_len; u++)
            tp[u] = (uint8_t)(oh[u >> 2] >> (24 - 8 * (u & 3)));
    } else {
        const uint8_t *tp = p.in + L + mki_size;
        uint32_t diff = 0;
        for (uint32_t u = 0; u < tag_len; u++)
            diff |= (uint32_t)(tp[u] ^ (uint8_t)(oh[u >> 2] >> (24 - 8 * (u & 3))));
        A.auth_ok[i] = diff == 0;
    }
}

// Uniform-key batches: all four T-tables (128 KiB of LDS, one workgroup of
// 1024 lanes per CU = 4 waves per SIMD, <= 128 VGPRs), the AES schedule in
// SGPRs.  Per-lane keys: (T0, T1) only, 512 lanes, the schedule in VGPRs.
// Persistent: the grid is sized to the CUs and each workgroup walks the
// batch, so the tables are loaded once per CU.
#ifndef ICM_UNI_THREADS
#define ICM_UNI_THREADS 512
#endif

#ifndef ICM_UNI_TAB4
#define ICM_UNI_TAB4 1
#endif
#ifndef ICM_UNI_WGS_PER_CU
#define ICM_UNI_WGS_PER_CU 1
#endif
constexpr int ICM_THREADS_UNI = ICM_UNI_THREADS;
constexpr int ICM_THREADS_LANE = 512;

template <int NR, bool AUTH, bool PROTECT, bool UNIFORM>
__global__ __launch_bounds__(UNIFORM ? ICM_THREADS_UNI : ICM_THREADS_LANE)
void k_icm_hmac(IcmArgs A)
{
    constexpr bool TAB4 = UNIFORM && ICM_UNI_TAB4;
    constexpr int NRK = NR ? NR : 1;
    constexpr int LDSB = NR ? (TAB4 ? AES_TAB4_BYTES : AES_TAB2_BYTES) : 16;
    __shared__ u32x4 s_tab[LDSB / 16];
    if (A.abort && *A.abort)
        return;
    if (NR)
        load_aes_tables<TAB4>(s_tab);
    __syncthreads();
    const AesLds T = make_aes_lds(s_tab);

    typename std::conditional<UNIFORM, UniKey<NRK>, LaneKey<NRK>>::type rk;
    if (UNIFORM && NR)
        rk.load(A.keys + A.uni);
    // lane L of a wave takes packet 16 * (L & 3) + (L >> 2) of the wave's 64
    // (the cooperative path exchanges data inside lane quads)
    const uint32_t stride = gridDim.x * blockDim.x;
    const uint32_t L = threadIdx.x & 63;
    const uint32_t first = blockIdx.x * blockDim.x + (threadIdx.x & ~63u) +
                           16 * (L & 3) + (L >> 2);
    for (uint32_t i = first; i < A.n; i += stride)
        icm_packet<NR, TAB4, AUTH, PROTECT, UNIFORM>(A, i, T, rk);
}

// ---------------------------------------------------------------------------
// GHASH: Shoup 8-bit table, X held as big-endian words (x^0 = bit 31 of x0)
template <bool LDSM>
struct GhTab {
    const char *lds;          // LDS base of the replicated table (+64K)
    uint32_t lane16;          // (lane & 15) * 16 | 0x10000
    const u32x4 *g;           // global table (per-lane key variant)
    DEV u32x4 get(uint32_t w, int k) const;
};

template <>
DEV u32x4 GhTab<true>::get(uint32_t w, int k) const
{
    // byte k of BE word w (k = 0 is the most significant byte)
    uint32_t sel = 0x0c020000u | ((4u + 3u - (uint32_t)k) << 8);
    uint32_t a = __builtin_amdgcn_perm(w, lane16, sel);
    return *(const u32x4 *)(lds + a);
}

template <>
DEV u32x4 GhTab<false>::get(uint32_t w, int k) const
{
    uint32_t idx = (w >> (24 - 8 * k)) & 0xffu;
    return g[idx];
}

template <bool LDSM>
DEV void ghash_mul(uint32_t x[4], const GhTab<LDSM> &T)
{
    // Z = X * H by Horner over the bytes, last byte first
    u32x4 z = T.get(x[3], 3);
#pragma unroll
    for (int k = 14; k >= 0; k--) {
        uint32_t r = z.w & 0xffu;
        uint32_t red = xor3(r << 24, r << 23, r << 22) ^ (r << 17);
        u32x4 mv = T.get(x[k >> 2], k & 3);
        u32x4 nz;
        nz.w = __builtin_amdgcn_alignbit(z.z, z.w, 8) ^ mv.w;
        nz.z = __builtin_amdgcn_alignbit(z.y, z.z, 8) ^ mv.z;
        nz.y = __builtin_amdgcn_alignbit(z.x, z.y, 8) ^ mv.y;
        nz.x = xor3(z.x >> 8, red, mv.x);
        z = nz;
    }
    x[0] = z.x;
    x[1] = z.y;
    x[2] = z.z;
    x[3] = z.w;
}

struct GcmArgs {
    const uint8_t *in;
    const uint64_t *in_off;
    uint8_t *out;
    const uint64_t *out_off;
    const srtp_dev_meta_t *meta;
    const srtp_dev_key_t *keys;
    const uint32_t *ghash;   // 1024 words per GCM key
    uint8_t *auth_ok;
    const uint32_t *abort;   // device pre-pass fell back: do nothing
    uint32_t n;
    uint32_t uni;
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

#ifndef GCM_PF
#define GCM_PF 2   // 64-byte payload chunks loaded ahead of their use
#endif

DEV void load_chunk4(u32x4 (&v)[4], const uint8_t *ip)
{
#pragma unroll
    for (int t = 0; t < 4; t++)
        v[t] = *(const u32x4a4 *)(ip + 16 * t);
}

// One GCM packet (srtp.c:2088-2267 protect / 2276-2491 unprotect through
// aes_gcm_ossl.c: IV = (00 00 || SSRC || ROC || SEQ) ^ salt, AAD = header,
// CTR from inc32(J0), tag = E(J0) ^ GHASH).  The payload runs in 64-byte
// chunks of four CTR blocks whose counters stay in the cached epoch
// (j + 2 <= 255: the first 4 KiB), data loaded GCM_PF chunks ahead; the
// rest block by block with full AES.
template <int NR, bool PROTECT, bool UNIFORM, class KEY>
DEV void gcm_packet(const GcmArgs &A, uint32_t i, const AesLds &T,
                    GhTab<UNIFORM> G, KEY &rk)
{
    const srtp_dev_meta_t m = A.meta[i];
    constexpr uint32_t VID = 16u + 2u * ((NR - 8) / 2);
    if (SRTP_META_STATUS(m.info) || SRTP_META_VARIANT(m.info) != VID)
        return;
    const uint32_t slot = UNIFORM ? A.uni : m.key;
    const srtp_dev_key_t *key = A.keys + slot;
    if constexpr (!UNIFORM) {
        rk.load(key);
        G.g = (const u32x4 *)(A.ghash + 1024 * key->ghash_slot);
    }

    const uint8_t *in = A.in + A.in_off[i];
    uint8_t *out = A.out + A.out_off[i];
    const uint32_t enc_start = SRTP_META_ENC_START(m.info);
    const uint32_t tag_len = key->tag_len;
    const uint32_t mki_size = key->mki_size;
    const uint32_t P = m.len - enc_start;       // plaintext / ciphertext bytes

    // IV = (00 00 || SSRC || ROC || SEQ) ^ salt12   (srtp.c:1925-1959)
    const uint32_t w0 = bswap(*(const uint32_t *)in);
    const uint32_t ssrc = bswap(*(const uint32_t *)(in + 8));
    const uint32_t seq = w0 & 0xffffu;
    const uint32_t iv0 = (ssrc >> 16) ^ bswap(key->salt[0]);
    const uint32_t iv1 = ((ssrc << 16) | (m.roc >> 16)) ^ bswap(key->salt[1]);
    const uint32_t iv2 = ((m.roc << 16) | seq) ^ bswap(key->salt[2]);
    const uint32_t c0 = bswap(iv0), c1 = bswap(iv1), c2 = bswap(iv2);

    uint32_t x[4] = { 0, 0, 0, 0 };   // GHASH accumulator (BE words)

    // AAD = the RTP header (enc_start bytes), copied as-is when out != in
    const bool copy_hdr = in != out;
    for (uint32_t q = 0; 16 * q < enc_start; q++) {
        u32x4 v = *(const u32x4 *)(in + 16 * q);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            uint32_t wi = 4 * q + u;
            uint32_t vu = v[u];
            if (4 * wi >= enc_start)
                vu = 0;
            else if (copy_hdr)
                *(uint32_t *)(out + 4 * wi) = vu;
            x[u] ^= bswap(vu);
        }
        ghash_mul(x, G);
    }

    const uint32_t nblk = (P + 15) >> 4;
    const uint8_t *pin = in + enc_start;
    uint8_t *pout = out + enc_start;
    uint32_t j = 0;
    // full chunks in the cached counter epoch: block 4c+3 has j + 2 <= 255
    uint32_t nfc = P >> 6;
    nfc = nfc < 63 ? nfc : 63;
    if (nfc) {
        const uint32_t cc[4] = { c0, c1, c2, 0u };   // BE32(j+2) < 256
        const CtrCache C = ctr_cache<NR, false>(cc, rk, T);
        u32x4 ring[GCM_PF][4];
#pragma unroll
        for (int k = 0; k < GCM_PF; k++)
            if ((uint32_t)k < nfc)
                load_chunk4(ring[k], pin + 64 * k);
        for (uint32_t c = 0; c < nfc; c++) {
            u32x4 cur[4];
#pragma unroll
            for (int t = 0; t < 4; t++)
                cur[t] = ring[0][t];
#pragma unroll
            for (int k = 0; k + 1 < GCM_PF; k++)
#pragma unroll
                for (int t = 0; t < 4; t++)
                    ring[k][t] = ring[k + 1][t];
            if (c + GCM_PF < nfc)
                load_chunk4(ring[GCM_PF - 1], pin + 64 * (c + GCM_PF));
            uint32_t ks[4][4];
#pragma unroll
            for (int g = 0; g < 4; g += 2) {
                const uint32_t jb[2] = { (4 * c + g + 2) << 8,
                                         (4 * c + g + 3) << 8 };
                aes_ctr<2, NR, false>(
                    *reinterpret_cast<uint32_t(*)[2][4]>(&ks[g]), jb, C, rk, T);
            }
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const u32x4 o = { cur[t].x ^ ks[t][0], cur[t].y ^ ks[t][1],
                                  cur[t].z ^ ks[t][2], cur[t].w ^ ks[t][3] };
                *(u32x4a4 *)(pout + 64 * c + 16 * t) = o;
                const u32x4 ctv = PROTECT ? o : cur[t];
                x[0] ^= bswap(ctv.x);
                x[1] ^= bswap(ctv.y);
                x[2] ^= bswap(ctv.z);
                x[3] ^= bswap(ctv.w);
                ghash_mul(x, G);
            }
        }
        j = 4 * nfc;
    }
    for (; j < nblk; j++) {
        const int rem = (int)P - (int)(16 * j);
        u32x4 v;
        if (rem >= 16)
            v = *(const u32x4a4 *)(pin + 16 * j);
        else
            v = load_partial(pin + 16 * j, rem);
        uint32_t k0 = c0, k1 = c1, k2 = c2, k3 = bswap(j + 2);
        aes_block<NR, false>(k0, k1, k2, k3, rk, T);
        u32x4 o = { v.x ^ k0, v.y ^ k1, v.z ^ k2, v.w ^ k3 };
        u32x4 ctv = PROTECT ? o : v;
        if (rem < 16) {   // zero-pad the last ciphertext block for GHASH
#pragma unroll
            for (int u = 0; u < 4; u++) {
                int nb = rem - 4 * u;
                if (nb <= 0)
                    ctv[u] = 0;
                else if (nb < 4)
                    ctv[u] &= 0xffffffffu >> (8 * (4 - nb));
            }
        }
        x[0] ^= bswap(ctv.x);
        x[1] ^= bswap(ctv.y);
        x[2] ^= bswap(ctv.z);
        x[3] ^= bswap(ctv.w);
        ghash_mul(x, G);
        if (rem >= 16) {
            *(u32x4a4 *)(pout + 16 * j) = o;
        } else {
            uint32_t oa[4] = { o.x, o.y, o.z, o.w };
            store_words_partial(pout + 16 * j, oa, rem);
        }
    }
    // length block: [len(A)]64 || [len(C)]64 in bits
    x[1] ^= enc_start * 8;
    x[3] ^= P * 8;
    ghash_mul(x, G);
    // tag = E(J0) ^ S
    uint32_t e0 = c0, e1 = c1, e2 = c2, e3 = bswap(1u);
    aes_block<NR, false>(e0, e1, e2, e3, rk, T);
    uint32_t tagw[4] = { bswap(x[0]) ^ e0, bswap(x[1]) ^ e1, bswap(x[2]) ^ e2,
                         bswap(x[3]) ^ e3 };   // little-endian words of tag
    if (PROTECT) {
        uint8_t *tp = pout + P;
        for (uint32_t u = 0; u < tag_len; u++)
            tp[u] = (uint8_t)(tagw[u >> 2] >> (8 * (u & 3)));
        for (uint32_t u = 0; u < mki_size; u++)
            tp[tag_len + u] = key->mki[u];
    } else {
        const uint8_t *tp = pin + P;
        uint32_t diff = 0;
        for (uint32_t u = 0; u < tag_len; u++)
            diff |= (uint32_t)(tp[u] ^ (uint8_t)(tagw[u >> 2] >> (8 * (u & 3))));
        A.auth_ok[i] = diff == 0;
    }
}

// (T0, T1) in LDS plus, for uniform keys, the GHASH table replicated 16x
// (128 KiB: one 512-lane workgroup per CU); persistent grid.
#ifndef GCM_THREADS_N
#define GCM_THREADS_N 512
#endif
constexpr int GCM_THREADS = GCM_THREADS_N;

template <int NR, bool PROTECT, bool UNIFORM>
__global__ __launch_bounds__(GCM_THREADS) void k_gcm(GcmArgs A)
{
    __shared__ u32x4 s_tab[(AES_TAB2_BYTES + (UNIFORM ? GH_LDS_BYTES : 0)) / 16];
    if (A.abort && *A.abort)
        return;
    load_aes_tables<false>(s_tab);
    if (UNIFORM) {
        const u32x4 *src =
            (const u32x4 *)(A.ghash + 1024 * A.keys[A.uni].ghash_slot);
        u32x4 *dst = (u32x4 *)((char *)s_tab + AES_TAB2_BYTES);
        for (int e = threadIdx.x; e < 256 * 16; e += blockDim.x)
            dst[e] = src[e >> 4];
    }
    __syncthreads();
    const char *lds = (const char *)s_tab;
    const AesLds T = make_aes_lds(s_tab);

    typename std::conditional<UNIFORM, UniKey<NR>, LaneKey<NR>>::type rk;
    if (UNIFORM)
        rk.load(A.keys + A.uni);
    GhTab<UNIFORM> G;
    G.lds = lds + AES_TAB2_BYTES - 0x10000;   // the 0x10000 comes from lane16
    G.lane16 = ((threadIdx.x & 15) * 16) | 0x10000u;
    G.g = nullptr;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < A.n;
         i += stride)
        gcm_packet<NR, PROTECT, UNIFORM>(A, i, T, G, rk);
}

// ---------------------------------------------------------------------------
// Restore kernel for speculative unprotect: XORs the keystream the
// speculative pass used back over [enc_start, len) so the ciphertext of a
// packet that must be re-run is intact again (CTR decryption is an XOR).
// Rare path: byte-granular, runtime round count.
struct GlobalKey {
    const srtp_dev_key_t *k;
    DEV uint32_t operator()(int i) const { return k->rk[i]; }
};

template <int NR>
DEV void undo_one(const srtp_dev_key_t *key, const srtp_dev_meta_t &m,
                  uint8_t *p, const AesLds &T)
{
    GlobalKey rk{ key };
    const uint32_t enc_start = SRTP_META_ENC_START(m.info);
    const uint32_t P = m.len - enc_start;
    const uint32_t w0 = bswap(*(const uint32_t *)p);
    const uint32_t seq = w0 & 0xffffu;
    uint32_t c0, c1, c2, c3base;
    const bool gcm = key->family == SRTP_DEV_GCM;
    if (gcm) {
        const uint32_t ssrc = bswap(*(const uint32_t *)(p + 8));
        c0 = bswap((ssrc >> 16) ^ bswap(key->salt[0]));
        c1 = bswap(((ssrc << 16) | (m.roc >> 16)) ^ bswap(key->salt[1]));
        c2 = bswap(((m.roc << 16) | seq) ^ bswap(key->salt[2]));
        c3base = 0;
    } else {
        c0 = key->salt[0];
        c1 = key->salt[1] ^ *(const uint32_t *)(p + 8);
        c2 = key->salt[2] ^ bswap(m.roc);
        c3base = key->salt[3] ^ (seq >> 8) ^ ((seq & 0xffu) << 8);
    }
    for (uint32_t j = 0; 16 * j < P; j++) {
        uint32_t x0 = c0, x1 = c1, x2 = c2, x3;
        if (gcm)
            x3 = bswap(j + 2);
        else
            x3 = c3base ^ ((j >> 8) << 16) ^ ((j & 0xffu) << 24);
        aes_block<NR, false>(x0, x1, x2, x3, rk, T);
        uint32_t ks[4] = { x0, x1, x2, x3 };
        for (uint32_t b = 0; b < 16 && 16 * j + b < P; b++)
            p[enc_start + 16 * j + b] ^= (uint8_t)(ks[b >> 2] >> (8 * (b & 3)));
    }
}

__global__ __launch_bounds__(256) void k_undo(uint8_t *arena,
                                              const uint64_t *off,
                                              const srtp_dev_meta_t *meta,
                                              const srtp_dev_key_t *keys,
                                              uint32_t n)
{
    __shared__ u32x4 s_tab[AES_TAB2_BYTES / 16];
    load_aes_tables<false>(s_tab);
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const srtp_dev_meta_t m = meta[i];
    if (SRTP_META_STATUS(m.info))
        return;
    const srtp_dev_key_t *key = keys + m.key;
    if (!key->conf || key->family == SRTP_DEV_NULL)
        return;
    const AesLds T = make_aes_lds(s_tab);
    uint8_t *p = arena + off[i];
    if (key->rounds == 10)
        undo_one<10>(key, m, p, T);
    else if (key->rounds == 12)
        undo_one<12>(key, m, p, T);
    else
        undo_one<14>(key, m, p, T);
}

// ---------------------------------------------------------------------------
// SRTCP (srtp.c:4304-4544 protect, 4546-4837 unprotect): one lane per packet.
// RTCP is a low-rate control channel, so this is the plain byte-wise form of
// the RTP kernel's pieces: AES-ICM keystream over [8, P), the E|index trailer
// at P, MKI, HMAC-SHA1 over [0, P + 4).

// HMAC-SHA1 over msg[0, L) (hmac.c:157-229; no ROC suffix for SRTCP)
DEV void hmac_sha1_bytes(const srtp_dev_key_t *key, const uint8_t *msg,
                         uint32_t L, uint32_t oh[5])
{
    uint32_t h[5];
    for (int k = 0; k < 5; k++)
        h[k] = key->ipad[k];
    const uint32_t nb = (L + 1 + 8 + 63) / 64;   // data, 0x80, 64-bit length
    const uint32_t bits = (64 + L) * 8;          // the ipad block counts
    for (uint32_t b = 0; b < nb; b++) {
        uint32_t w[16];
        for (int t = 0; t < 16; t++) {
            uint32_t v = 0;
            for (int u = 0; u < 4; u++) {
                const uint32_t o = 64 * b + 4 * t + u;
                const uint32_t c = o < L ? msg[o] : (o == L ? 0x80u : 0u);
                v = (v << 8) | c;
            }
            w[t] = v;
        }
        if (b == nb - 1)
            w[15] = bits;
        sha1_compress(h, w);
    }
    uint32_t ow[16];
    for (int k = 0; k < 5; k++)
        ow[k] = h[k];
    ow[5] = 0x80000000u;
    for (int k = 6; k < 15; k++)
        ow[k] = 0;
    ow[15] = (64 + 20) * 8;
    for (int k = 0; k < 5; k++)
        oh[k] = key->opad[k];
    sha1_compress(oh, ow);
}

// AES-ICM over p[8, P): counter = salt ^ (0^4 || SSRC || be48(idx)) with the
// 16-bit block counter in bytes 14..15 (srtp.c:4470-4478, aes_icm.c:236-414)
template <int NR>
DEV void rtcp_icm(const srtp_dev_key_t *key, uint32_t idx, uint8_t *p,
                  uint32_t P, const AesLds &T)
{
    GlobalKey rk{ key };
    const uint32_t ssrc_le = (uint32_t)p[4] | (uint32_t)p[5] << 8 |
                             (uint32_t)p[6] << 16 | (uint32_t)p[7] << 24;
    const uint32_t c0 = key->salt[0];
    const uint32_t c1 = key->salt[1] ^ ssrc_le;
    const uint32_t c2 = key->salt[2] ^ bswap(idx >> 16);
    const uint32_t c3base = key->salt[3] ^ bswap(idx << 16);
    for (uint32_t j = 0; 8 + 16 * j < P; j++) {
        uint32_t x0 = c0, x1 = c1, x2 = c2;
        uint32_t x3 = c3base ^ ((j >> 8) << 16) ^ ((j & 0xffu) << 24);
        aes_block<NR, false>(x0, x1, x2, x3, rk, T);
        const uint32_t ks[4] = { x0, x1, x2, x3 };
        for (uint32_t b = 0; b < 16 && 8 + 16 * j + b < P; b++)
            p[8 + 16 * j + b] ^= (uint8_t)(ks[b >> 2] >> (8 * (b & 3)));
    }
}

DEV void rtcp_crypt(const srtp_dev_key_t *key, uint32_t idx, uint8_t *p,
                    uint32_t P, const AesLds &T)
{
    if (key->rounds == 10)
        rtcp_icm<10>(key, idx, p, P, T);
    else if (key->rounds == 12)
        rtcp_icm<12>(key, idx, p, P, T);
    else
        rtcp_icm<14>(key, idx, p, P, T);
}

// ---- AEAD SRTCP (srtp.c:3894-4300): AES-GCM with a bit-serial GHASH --------
// X <- X * H in GF(2^128), GCM bit order (SP 800-38D 6.3); 64-bit BE halves
DEV void gf128_mul(uint64_t &xh, uint64_t &xl, uint64_t hh, uint64_t hl)
{
    uint64_t zh = 0, zl = 0, vh = hh, vl = hl;
    for (int i = 0; i < 128; i++) {
        const uint64_t bit = i < 64 ? (xh >> (63 - i)) & 1u : (xl >> (127 - i)) & 1u;
        const uint64_t m = 0 - bit;
        zh ^= vh & m;
        zl ^= vl & m;
        const uint64_t lsb = vl & 1u;
        vl = (vl >> 1) | (vh << 63);
        vh = (vh >> 1) ^ ((0 - lsb) & 0xe100000000000000ull);
    }
    xh = zh;
    xl = zl;
}

struct Ghash {
    uint64_t xh, xl, hh, hl;
    uint8_t buf[16];
    uint32_t fill;
    DEV void put(uint8_t b)
    {
        buf[fill++] = b;
        if (fill == 16)
            flush();
    }
    DEV void flush()   // absorb the (zero-padded) pending block
    {
        if (!fill)
            return;
        for (uint32_t u = fill; u < 16; u++)
            buf[u] = 0;
        uint64_t a = 0, b = 0;
        for (int u = 0; u < 8; u++) {
            a = (a << 8) | buf[u];
            b = (b << 8) | buf[8 + u];
        }
        xh ^= a;
        xl ^= b;
        gf128_mul(xh, xl, hh, hl);
        fill = 0;
    }
};

// the GCM counter block IV12 || be32(ctr) through AES
template <int NR>
DEV void gcm_block(const srtp_dev_key_t *key, const uint8_t iv[12],
                   uint32_t ctr, uint32_t ks[4], const AesLds &T)
{
    GlobalKey rk{ key };
    uint32_t x[4];
    for (int w = 0; w < 3; w++)
        x[w] = (uint32_t)iv[4 * w] | (uint32_t)iv[4 * w + 1] << 8 |
               (uint32_t)iv[4 * w + 2] << 16 | (uint32_t)iv[4 * w + 3] << 24;
    x[3] = bswap(ctr);
    aes_block<NR, false>(x[0], x[1], x[2], x[3], rk, T);
    for (int w = 0; w < 4; w++)
        ks[w] = x[w];
}

template <int NR>
DEV void rtcp_gcm(const srtp_dev_key_t *key, const srtp_dev_meta_t &m,
                  uint8_t *p, uint8_t *auth_ok, uint32_t i, bool protect,
                  const AesLds &T)
{
    const uint32_t P = m.len, TL = key->tag_len, E = m.info & 1u;
    uint8_t *tr = p + P + TL;
    if (protect) {
        const uint32_t v = (E << 31) | m.roc;
        tr[0] = (uint8_t)(v >> 24);
        tr[1] = (uint8_t)(v >> 16);
        tr[2] = (uint8_t)(v >> 8);
        tr[3] = (uint8_t)v;
    }
    // IV = salt ^ (00 00 || SSRC || 00 00 || be32(index))  (srtp.c:3894-3930)
    const uint8_t *salt = (const uint8_t *)key->salt;
    uint8_t iv[12];
    for (int u = 0; u < 12; u++)
        iv[u] = salt[u];
    for (int u = 0; u < 4; u++) {
        iv[2 + u] ^= p[4 + u];
        iv[8 + u] ^= (uint8_t)(m.roc >> (24 - 8 * u));
    }
    Ghash G;
    G.xh = G.xl = 0;
    G.hh = (uint64_t)key->h[0] << 32 | key->h[1];
    G.hl = (uint64_t)key->h[2] << 32 | key->h[3];
    G.fill = 0;
    // AAD: header (E set) or the whole RTCP packet, then the trailer
    const uint32_t A1 = E ? 8u : P;
    for (uint32_t u = 0; u < A1; u++)
        G.put(p[u]);
    for (uint32_t u = 0; u < 4; u++)
        G.put(tr[u]);
    G.flush();
    const uint32_t C = E ? P - 8 : 0;
    uint32_t ks[4];
    for (uint32_t j = 0; 16 * j < C; j++) {
        gcm_block<NR>(key, iv, j + 2, ks, T);
        for (uint32_t b = 0; b < 16 && 16 * j + b < C; b++) {
            uint8_t *q = p + 8 + 16 * j + b;
            const uint8_t k8 = (uint8_t)(ks[b >> 2] >> (8 * (b & 3)));
            if (protect) {
                *q ^= k8;
                G.put(*q);
            } else {
                G.put(*q);   // GHASH runs over the ciphertext
            }
        }
    }
    G.flush();
    G.xh ^= (uint64_t)(A1 + 4) * 8;   // len(A) || len(C) in bits
    G.xl ^= (uint64_t)C * 8;
    gf128_mul(G.xh, G.xl, G.hh, G.hl);
    gcm_block<NR>(key, iv, 1, ks, T);   // E_K(J0)
    uint8_t tag[16];
    for (int u = 0; u < 16; u++) {
        const uint64_t half = u < 8 ? G.xh : G.xl;
        tag[u] = (uint8_t)(half >> (56 - 8 * (u & 7))) ^
                 (uint8_t)(ks[u >> 2] >> (8 * (u & 3)));
    }
    if (protect) {
        for (uint32_t u = 0; u < TL; u++)
            p[P + u] = tag[u];
        for (uint32_t u = 0; u < key->mki_size; u++)
            tr[4 + u] = key->mki[u];
        return;
    }
    uint32_t diff = 0;
    for (uint32_t u = 0; u < TL; u++)
        diff |= p[P + u] ^ tag[u];
    auth_ok[i] = (uint8_t)(diff == 0);
    if (diff)
        return;
    for (uint32_t j = 0; 16 * j < C; j++) {
        gcm_block<NR>(key, iv, j + 2, ks, T);
        for (uint32_t b = 0; b < 16 && 16 * j + b < C; b++)
            p[8 + 16 * j + b] ^= (uint8_t)(ks[b >> 2] >> (8 * (b & 3)));
    }
}

__global__ __launch_bounds__(256) void k_rtcp(uint8_t *arena,
                                              const uint64_t *off,
                                              const srtp_dev_meta_t *meta,
                                              const srtp_dev_key_t *keys,
                                              uint8_t *auth_ok, uint32_t n,
                                              int protect)
{
    __shared__ u32x4 s_tab[AES_TAB2_BYTES / 16];
    load_aes_tables<false>(s_tab);
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const srtp_dev_meta_t m = meta[i];
    if (SRTP_META_STATUS(m.info))
        return;
    const srtp_dev_key_t *key = keys + m.key;
    const AesLds T = make_aes_lds(s_tab);
    uint8_t *p = arena + off[i];
    if (key->family == SRTP_DEV_GCM) {
        if (key->rounds == 10)
            rtcp_gcm<10>(key, m, p, auth_ok, i, protect != 0, T);
        else
            rtcp_gcm<14>(key, m, p, auth_ok, i, protect != 0, T);
        return;
    }
    const uint32_t E = m.info & 1u;
    const bool enc = E && key->family == SRTP_DEV_ICM;
    const uint32_t tag_len = key->tag_len, mki_size = key->mki_size;
    if (protect) {
        const uint32_t P = m.len;
        const uint32_t tr = (E << 31) | m.roc;
        p[P] = (uint8_t)(tr >> 24);
        p[P + 1] = (uint8_t)(tr >> 16);
        p[P + 2] = (uint8_t)(tr >> 8);
        p[P + 3] = (uint8_t)tr;
        if (enc)
            rtcp_crypt(key, m.roc, p, P, T);
        for (uint32_t u = 0; u < mki_size; u++)
            p[P + 4 + u] = key->mki[u];
        if (key->auth) {
            uint32_t oh[5];
            hmac_sha1_bytes(key, p, P + 4, oh);
            uint8_t *tp = p + P + 4 + mki_size;
            for (uint32_t u = 0; u < tag_len; u++)
                tp[u] = (uint8_t)(oh[u >> 2] >> (24 - 8 * (u & 3)));
        }
    } else {
        const uint32_t A = m.len;   // authenticated bytes, trailer included
        uint32_t ok = 1;
        if (key->auth) {
            uint32_t oh[5];
            hmac_sha1_bytes(key, p, A, oh);
            const uint8_t *tp = p + A + mki_size;
            uint32_t diff = 0;   // constant time (datatypes.c:407-420)
            for (uint32_t u = 0; u < tag_len; u++)
                diff |= tp[u] ^ ((oh[u >> 2] >> (24 - 8 * (u & 3))) & 0xffu);
            ok = diff == 0;
        }
        auth_ok[i] = (uint8_t)ok;
        if (ok && enc)
            rtcp_crypt(key, m.roc, p, A - 4, T);
    }
}

// ---------------------------------------------------------------------------
// header parse for the device-resident API (srtp_validate_rtp_header,
// srtp.c:307-336; header length 96-125)
__global__ void k_parse(const uint8_t *in, const uint64_t *in_off,
                        const uint32_t *in_len, srtp_dev_hdr_t *hdr, uint32_t n)
{
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint64_t off = in_off[i];
    hdr[i] = srtp_parse_rtp(in + off, off, in_len[i]);
}

// ---------------------------------------------------------------------------
// host-side table construction
uint8_t sbox_host[256];

uint8_t gmul(uint8_t a, uint8_t b)
{
    uint8_t r = 0;
    while (b) {
        if (b & 1)
            r ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return r;
}

void build_ttab_host(uint32_t *t)
{
    // S-box from GF(2^8) inverse + affine map (FIPS-197 5.1.1)
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        for (int y = 1; x && y < 256; y++)
            if (gmul((uint8_t)x, (uint8_t)y) == 1) {
                inv = (uint8_t)y;
                break;
            }
        uint8_t s = inv, r = inv;
        for (int k = 0; k < 4; k++) {
            r = (uint8_t)((r << 1) | (r >> 7));
            s ^= r;
        }
        sbox_host[x] = s ^ 0x63;
    }
    for (int x = 0; x < 256; x++) {
        uint32_t s = sbox_host[x];
        uint32_t t0 = gmul((uint8_t)s, 2) | (s << 8) | (s << 16) |
                      ((uint32_t)gmul((uint8_t)s, 3) << 24);
        t[x] = t0;
    }
}

}   // namespace

// ===========================================================================
// thin C-ABI FFI (srtp_dev.h)

static thread_local char g_err[256];

static int fail(hipError_t e, const char *what)
{
    snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
    return -1;
}

#define HIPCHK(x)                                                              \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess)                                                  \
            return fail(e_, #x);                                               \
    } while (0)

struct srtp_gpu {
    hipStream_t stream;
    srtp_dev_key_t *d_keys;
    uint32_t key_cap;
    uint32_t *d_ghash;
    uint32_t ghash_cap;
    hipEvent_t ev0, ev1;
    int timing;
    float last_ms;
    void *pp;   // device pre-pass state (srtp_prepass.hip)
    int ncu;    // compute units (persistent grids)
};

// variant mask bits: which kernel instantiations the batch needs
//   bit (family*8 + rounds_code*2 + auth) with rounds_code 0:null 1:10 2:12 3:14
#define VBIT(fam, rc, au) (1u << ((fam) * 8 + (rc) * 2 + (au)))

template <int NR, bool AUTH, bool PROT>
static int launch_icm(srtp_gpu_t *g, const srtp_gpu_batch_t *b,
                      hipStream_t st)
{
    IcmArgs A;
    A.in = b->in;
    A.in_off = b->in_off;
    A.out = b->out;
    A.out_off = b->out_off;
    A.meta = b->meta;
    A.keys = g->d_keys;
    A.auth_ok = b->auth_ok;
    A.abort = b->abort;
    A.n = (uint32_t)b->n;
    A.uni = b->uniform_key;
    // persistent grid: one 1024-lane workgroup per CU (128 KiB of tables)
    // for uniform keys, two 512-lane workgroups per CU otherwise
    if (b->uniform_key != 0xffffffffu) {
        const size_t wgs = (b->n + ICM_THREADS_UNI - 1) / ICM_THREADS_UNI;
        const size_t cap = (size_t)g->ncu * ICM_UNI_WGS_PER_CU;
        hipLaunchKernelGGL((k_icm_hmac<NR, AUTH, PROT, true>),
                           dim3((unsigned)(wgs < cap ? wgs : cap)),
                           dim3(ICM_THREADS_UNI), 0, st, A);
    } else {
        const size_t wgs = (b->n + ICM_THREADS_LANE - 1) / ICM_THREADS_LANE;
        const size_t cap = 2 * (size_t)g->ncu;
        hipLaunchKernelGGL((k_icm_hmac<NR, AUTH, PROT, false>),
                           dim3((unsigned)(wgs < cap ? wgs : cap)),
                           dim3(ICM_THREADS_LANE), 0, st, A);
    }
    HIPCHK(hipGetLastError());
    return 0;
}

template <int NR, bool PROT>
static int launch_gcm(srtp_gpu_t *g, const srtp_gpu_batch_t *b, hipStream_t st)
{
    GcmArgs A;
    A.in = b->in;
    A.in_off = b->in_off;
    A.out = b->out;
    A.out_off = b->out_off;
    A.meta = b->meta;
    A.keys = g->d_keys;
    A.ghash = g->d_ghash;
    A.auth_ok = b->auth_ok;
    A.abort = b->abort;
    A.n = (uint32_t)b->n;
    A.uni = b->uniform_key;
    // persistent grid: one workgroup per CU (128 KiB of tables) for uniform
    // keys, two otherwise (64 KiB)
    const bool uni = b->uniform_key != 0xffffffffu;
    const size_t wgs = (b->n + GCM_THREADS - 1) / GCM_THREADS;
    const size_t cap = (size_t)g->ncu * (uni ? 1 : 2);
    const dim3 grid((unsigned)(wgs < cap ? wgs : cap)), block(GCM_THREADS);
    if (uni)
        hipLaunchKernelGGL((k_gcm<NR, PROT, true>), grid, block, 0, st, A);
    else
        hipLaunchKernelGGL((k_gcm<NR, PROT, false>), grid, block, 0, st, A);
    HIPCHK(hipGetLastError());
    return 0;
}

template <bool PROT>
static int run_dir(srtp_gpu_t *g, const srtp_gpu_batch_t *b, hipStream_t st)
{
    uint32_t m = b->mask;
    int rc = 0;
    // ICM / null family
    if (m & VBIT(SRTP_DEV_NULL, 0, 0)) rc |= launch_icm<0, false, PROT>(g, b, st);
    if (m & VBIT(SRTP_DEV_NULL, 0, 1)) rc |= launch_icm<0, true, PROT>(g, b, st);
    if (m & VBIT(SRTP_DEV_ICM, 1, 0)) rc |= launch_icm<10, false, PROT>(g, b, st);
    if (m & VBIT(SRTP_DEV_ICM, 1, 1)) rc |= launch_icm<10, true, PROT>(g, b, st);
    if (m & VBIT(SRTP_DEV_ICM, 2, 0)) rc |= launch_icm<12, false, PROT>(g, b, st);
    if (m & VBIT(SRTP_DEV_ICM, 2, 1)) rc |= launch_icm<12, true, PROT>(g, b, st);
    if (m & VBIT(SRTP_DEV_ICM, 3, 0)) rc |= launch_icm<14, false, PROT>(g, b, st);
    if (m & VBIT(SRTP_DEV_ICM, 3, 1)) rc |= launch_icm<14, true, PROT>(g, b, st);
    if (m & VBIT(SRTP_DEV_GCM, 1, 0)) rc |= launch_gcm<10, PROT>(g, b, st);
    if (m & VBIT(SRTP_DEV_GCM, 3, 0)) rc |= launch_gcm<14, PROT>(g, b, st);
    return rc;
}


extern "C" {

const char *srtp_gpu_last_error(void) { return g_err; }

void **srtp_gpu_pp_slot(srtp_gpu_t *g) { return &g->pp; }
void *srtp_gpu_stream_of(srtp_gpu_t *g) { return (void *)g->stream; }

int srtp_gpu_available(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        return 0;
    return n > 0;
}

static int g_table_ready = -1;

int srtp_gpu_open(srtp_gpu_t **gp)
{
    *gp = NULL;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) {
        snprintf(g_err, sizeof g_err, "no HIP device (%s)",
                 hipGetErrorString(e));
        return -1;
    }
    int dev = -1;
    HIPCHK(hipGetDevice(&dev));
    if (g_table_ready != dev) {
        uint32_t t[256];
        build_ttab_host(t);
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_t0), t, sizeof t));
        g_table_ready = dev;
    }
    srtp_gpu_t *g = (srtp_gpu_t *)calloc(1, sizeof(srtp_gpu_t));
    HIPCHK(hipDeviceGetAttribute(&g->ncu, hipDeviceAttributeMultiprocessorCount,
                                 dev));
    if (g->ncu <= 0)
        g->ncu = 256;
    HIPCHK(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreate(&g->ev0));
    HIPCHK(hipEventCreate(&g->ev1));
    *gp = g;
    return 0;
}

void srtp_gpu_close(srtp_gpu_t *g)
{
    if (!g)
        return;
    (void)hipStreamSynchronize(g->stream);
    srtp_gpu_pp_free(g->pp);
    (void)hipFree(g->d_keys);
    (void)hipFree(g->d_ghash);
    (void)hipEventDestroy(g->ev0);
    (void)hipEventDestroy(g->ev1);
    (void)hipStreamDestroy(g->stream);
    free(g);
}

static int grow(void **p, uint32_t *cap, uint32_t need, size_t elem)
{
    if (need <= *cap)
        return 0;
    uint32_t nc = *cap ? *cap : 16;
    while (nc < need)
        nc *= 2;
    void *np = NULL;
    HIPCHK(hipMalloc(&np, (size_t)nc * elem));
    if (*p) {
        HIPCHK(hipMemcpy(np, *p, (size_t)(*cap) * elem, hipMemcpyDeviceToDevice));
        HIPCHK(hipFree(*p));
    }
    *p = np;
    *cap = nc;
    return 0;
}

int srtp_gpu_set_key(srtp_gpu_t *g, uint32_t slot, const srtp_dev_key_t *k,
                     const uint32_t *ghash_tab)
{
    if (grow((void **)&g->d_keys, &g->key_cap, slot + 1, sizeof(srtp_dev_key_t)))
        return -1;
    HIPCHK(hipMemcpyAsync(g->d_keys + slot, k, sizeof *k,
                          hipMemcpyHostToDevice, g->stream));
    if (ghash_tab) {
        if (grow((void **)&g->d_ghash, &g->ghash_cap, k->ghash_slot + 1,
                 1024 * sizeof(uint32_t)))
            return -1;
        HIPCHK(hipMemcpyAsync(g->d_ghash + 1024 * (size_t)k->ghash_slot,
                              ghash_tab, 4096, hipMemcpyHostToDevice,
                              g->stream));
    }
    HIPCHK(hipStreamSynchronize(g->stream));
    return 0;
}

int srtp_gpu_run(srtp_gpu_t *g, int op, const srtp_gpu_batch_t *b)
{
    if (b->n == 0)
        return 0;
    hipStream_t st = (hipStream_t)b->stream;   // NULL = the null stream
    if (g->timing)
        HIPCHK(hipEventRecord(g->ev0, st));
    int rc = op == 0 ? run_dir<true>(g, b, st) : run_dir<false>(g, b, st);
    if (g->timing) {
        HIPCHK(hipEventRecord(g->ev1, st));
        HIPCHK(hipEventSynchronize(g->ev1));
        HIPCHK(hipEventElapsedTime(&g->last_ms, g->ev0, g->ev1));
    }
    return rc;
}

int srtp_gpu_undo(srtp_gpu_t *g, size_t n, uint8_t *arena,
                  const uint64_t *off, const srtp_dev_meta_t *meta,
                  void *stream)
{
    if (!n)
        return 0;
    hipStream_t st = (hipStream_t)stream;   // NULL = the null stream
    hipLaunchKernelGGL(k_undo, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       st, arena, off, meta, g->d_keys, (uint32_t)n);
    HIPCHK(hipGetLastError());
    return 0;
}

int srtp_gpu_rtcp(srtp_gpu_t *g, int op, size_t n, uint8_t *arena,
                  const uint64_t *off, const srtp_dev_meta_t *meta,
                  uint8_t *auth_ok, void *stream)
{
    if (!n)
        return 0;
    hipStream_t st = (hipStream_t)stream;   // NULL = the null stream
    hipLaunchKernelGGL(k_rtcp, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       st, arena, off, meta, g->d_keys, auth_ok, (uint32_t)n,
                       op == 0 ? 1 : 0);
    HIPCHK(hipGetLastError());
    return 0;
}

int srtp_gpu_parse(srtp_gpu_t *g, size_t n, const uint8_t *in,
                   const uint64_t *in_off, const uint32_t *in_len,
                   srtp_dev_hdr_t *hdr_out, void *stream)
{
    if (!n)
        return 0;
    hipStream_t st = (hipStream_t)stream;   // NULL = the null stream
    hipLaunchKernelGGL(k_parse, dim3((unsigned)((n + 255) / 256)), dim3(256),
                       0, st, in, in_off, in_len, hdr_out, (uint32_t)n);
    HIPCHK(hipGetLastError());
    return 0;
}

void *srtp_gpu_malloc(size_t bytes)
{
    void *p = NULL;
    if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess)
        return NULL;
    return p;
}

void srtp_gpu_free(void *p)
{
    if (p)
        (void)hipFree(p);
}

void *srtp_gpu_host_alloc(size_t bytes)
{
    void *p = NULL;
    if (hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocDefault) !=
        hipSuccess)
        return NULL;
    return p;
}

void srtp_gpu_host_free(void *p)
{
    if (p)
        (void)hipHostFree(p);
}

int srtp_gpu_h2d(srtp_gpu_t *g, void *dst, const void *src, size_t n,
                 void *stream)
{
    if (!n)
        return 0;
    hipStream_t st = (hipStream_t)stream;   // NULL = the null stream
    HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st));
    return 0;
}

int srtp_gpu_d2h(srtp_gpu_t *g, void *dst, const void *src, size_t n,
                 void *stream)
{
    if (!n)
        return 0;
    hipStream_t st = (hipStream_t)stream;   // NULL = the null stream
    HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, st));
    return 0;
}

int srtp_gpu_sync(srtp_gpu_t *g, void *stream)
{
    hipStream_t st = (hipStream_t)stream;   // NULL = the null stream
    HIPCHK(hipStreamSynchronize(st));
    return 0;
}

double srtp_gpu_last_kernel_ms(srtp_gpu_t *g) { return g->last_ms; }
void srtp_gpu_set_timing(srtp_gpu_t *g, int on) { g->timing = on; }

}   // extern "C"
