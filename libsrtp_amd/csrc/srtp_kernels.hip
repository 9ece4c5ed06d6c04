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
// LDS tables.  One static array: [0, 64K) AES (T0,T1) x 32 copies,
// [64K, 128K) GHASH M8 x 16 copies (GCM kernels only).
constexpr int AES_LDS_BYTES = 256 * 32 * 8;
constexpr int GH_LDS_BYTES = 256 * 16 * 16;

__device__ uint2 g_ttab[256];   // (T0[x], T1[x]) little-endian words

// LDS image of the AES tables, 64 KiB: for byte value x the 256-byte row
// x holds T0[x] 32 times (bytes 0..127) then T1[x] 32 times (128..255).
// Lane l reads copy (l & 31): a ds_read_b32 of 32 lanes touches 32 distinct
// banks whatever the byte values are, i.e. it is never bank-conflicted.
DEV void load_aes_table(uint2 *lds2)
{
    uint32_t *lds = (uint32_t *)lds2;
    for (int e = threadIdx.x; e < 256 * 64; e += blockDim.x) {
        uint2 t = g_ttab[e >> 6];
        lds[e] = (e & 32) ? t.y : t.x;
    }
}

struct AesLds {
    const char *lds;
    uint32_t l0;   // (lane & 31) * 4        -> T0 copy of this lane
    uint32_t l1;   // (lane & 31) * 4 | 128  -> T1 copy of this lane
};

DEV AesLds make_aes_lds(const void *lds)
{
    AesLds T;
    T.lds = (const char *)lds;
    T.l0 = (threadIdx.x & 31) * 4;
    T.l1 = T.l0 | 128u;
    return T;
}

// byte K of w -> address bits 15:8, the lane's copy offset -> bits 7:0: one
// v_perm_b32 per lookup
template <int K>
DEV uint32_t t0(const AesLds &T, uint32_t w)
{
    uint32_t a = __builtin_amdgcn_perm(w, T.l0, 0x0c0c0000u | ((4u + K) << 8));
    return *(const uint32_t *)(T.lds + a);
}

template <int K>
DEV uint32_t t1(const AesLds &T, uint32_t w)
{
    uint32_t a = __builtin_amdgcn_perm(w, T.l1, 0x0c0c0000u | ((4u + K) << 8));
    return *(const uint32_t *)(T.lds + a);
}

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

// AES encryption of one block held as little-endian words (column c =
// bytes 4c..4c+3).  Round: col_c = T0[s_c.b0] ^ T1[s_c+1.b1]
//                                ^ rot16(T0[s_c+2.b2] ^ T1[s_c+3.b3]) ^ rk
// with T2 = rot16(T0), T3 = rot16(T1).  16 ds_read_b32 + 32 VALU per round.
template <int NR, class KEY>
DEV void aes_block(uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3,
                   const KEY &rk, const AesLds &T)
{
    s0 ^= rk(0);
    s1 ^= rk(1);
    s2 ^= rk(2);
    s3 ^= rk(3);
#pragma unroll
    for (int r = 1; r < NR; r++) {
        uint32_t a0 = t0<0>(T, s0), a1 = t0<0>(T, s1), a2 = t0<0>(T, s2),
                 a3 = t0<0>(T, s3);
        uint32_t b0 = t1<1>(T, s0), b1 = t1<1>(T, s1), b2 = t1<1>(T, s2),
                 b3 = t1<1>(T, s3);
        uint32_t c0 = t0<2>(T, s0), c1 = t0<2>(T, s1), c2 = t0<2>(T, s2),
                 c3 = t0<2>(T, s3);
        uint32_t d0 = t1<3>(T, s0), d1 = t1<3>(T, s1), d2 = t1<3>(T, s2),
                 d3 = t1<3>(T, s3);
        uint32_t n0 = xor3(a0, b1, rk(4 * r + 0)) ^ rotl(c2 ^ d3, 16);
        uint32_t n1 = xor3(a1, b2, rk(4 * r + 1)) ^ rotl(c3 ^ d0, 16);
        uint32_t n2 = xor3(a2, b3, rk(4 * r + 2)) ^ rotl(c0 ^ d1, 16);
        uint32_t n3 = xor3(a3, b0, rk(4 * r + 3)) ^ rotl(c1 ^ d2, 16);
        s0 = n0;
        s1 = n1;
        s2 = n2;
        s3 = n3;
    }
    // final round: S[x] is byte 1 of T0[x] and byte 2 of T1[x]
    uint32_t a0 = t0<0>(T, s0), a1 = t0<0>(T, s1), a2 = t0<0>(T, s2),
             a3 = t0<0>(T, s3);
    uint32_t b0 = t1<1>(T, s0), b1 = t1<1>(T, s1), b2 = t1<1>(T, s2),
             b3 = t1<1>(T, s3);
    uint32_t c0 = t0<2>(T, s0), c1 = t0<2>(T, s1), c2 = t0<2>(T, s2),
             c3 = t0<2>(T, s3);
    uint32_t d0 = t1<3>(T, s0), d1 = t1<3>(T, s1), d2 = t1<3>(T, s2),
             d3 = t1<3>(T, s3);
    const uint32_t LO = 0x0c0c0601u, HI = 0x06010c0cu;
    uint32_t n0 = xor3(__builtin_amdgcn_perm(b1, a0, LO),
                       __builtin_amdgcn_perm(d3, c2, HI), rk(4 * NR + 0));
    uint32_t n1 = xor3(__builtin_amdgcn_perm(b2, a1, LO),
                       __builtin_amdgcn_perm(d0, c3, HI), rk(4 * NR + 1));
    uint32_t n2 = xor3(__builtin_amdgcn_perm(b3, a2, LO),
                       __builtin_amdgcn_perm(d1, c0, HI), rk(4 * NR + 2));
    uint32_t n3 = xor3(__builtin_amdgcn_perm(b0, a3, LO),
                       __builtin_amdgcn_perm(d2, c1, HI), rk(4 * NR + 3));
    s0 = n0;
    s1 = n1;
    s2 = n2;
    s3 = n3;
}

// NB independent blocks advanced round by round together: the NB*16 table
// reads of a round are issued back to back, so one wave keeps NB times the
// LDS requests in flight across the ~100-cycle read latency of a round.
template <int NB, int NR, class KEY>
DEV void aes_blocks(uint32_t (&s)[NB][4], const KEY &rk, const AesLds &T)
{
#pragma unroll
    for (int j = 0; j < NB; j++)
#pragma unroll
        for (int c = 0; c < 4; c++)
            s[j][c] ^= rk(c);
#pragma unroll
    for (int r = 1; r < NR; r++) {
        uint32_t a[NB][4], b[NB][4], c[NB][4], d[NB][4];
#pragma unroll
        for (int j = 0; j < NB; j++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                a[j][q] = t0<0>(T, s[j][q]);
                b[j][q] = t1<1>(T, s[j][q]);
                c[j][q] = t0<2>(T, s[j][q]);
                d[j][q] = t1<3>(T, s[j][q]);
            }
#pragma unroll
        for (int j = 0; j < NB; j++)
#pragma unroll
            for (int q = 0; q < 4; q++)
                s[j][q] = xor3(a[j][q], b[j][(q + 1) & 3], rk(4 * r + q)) ^
                          rotl(c[j][(q + 2) & 3] ^ d[j][(q + 3) & 3], 16);
    }
    const uint32_t LO = 0x0c0c0601u, HI = 0x06010c0cu;
    uint32_t a[NB][4], b[NB][4], c[NB][4], d[NB][4];
#pragma unroll
    for (int j = 0; j < NB; j++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
            a[j][q] = t0<0>(T, s[j][q]);
            b[j][q] = t1<1>(T, s[j][q]);
            c[j][q] = t0<2>(T, s[j][q]);
            d[j][q] = t1<3>(T, s[j][q]);
        }
#pragma unroll
    for (int j = 0; j < NB; j++)
#pragma unroll
        for (int q = 0; q < 4; q++)
            s[j][q] = xor3(__builtin_amdgcn_perm(b[j][(q + 1) & 3], a[j][q], LO),
                           __builtin_amdgcn_perm(d[j][(q + 3) & 3],
                                                 c[j][(q + 2) & 3], HI),
                           rk(4 * NR + q));
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

#ifndef ICM_WAVES_PER_SIMD
#define ICM_WAVES_PER_SIMD 1
#endif
#ifndef ICM_NB
#define ICM_NB 2   // AES blocks interleaved per round in the steady state
#endif

// One 64-byte chunk b of a packet in its general form: header words that
// are not encrypted, quads past the end of the data, the partial last quad
// (kept in tailq, stored once after the chunk loop: a byte-wise store here,
// unrolled per quad, costs ~65 VGPRs), and the ROC / terminator / length
// words of the SHA-1 message tail (sha1.c srtp_sha1_final).
template <int NR, bool AUTH, bool PROTECT, class KEY>
DEV void icm_chunk(uint32_t b, const uint8_t *in, uint8_t *out, uint32_t L,
                   uint32_t hw, uint32_t s, uint32_t qoff, uint32_t nq,
                   uint32_t nb, uint32_t bclean, bool conf, uint32_t roc,
                   const uint32_t cb[4], const KEY &rk, const AesLds &T,
                   uint32_t ks_prev[4], uint32_t hst[5], uint32_t tailq[4])
{
    const uint32_t q0 = 4 * b;
    const uint8_t *ip = in + 16 * q0;
    uint8_t *op = out + 16 * q0;
    u32x4 v[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        v[t] = u32x4{ 0, 0, 0, 0 };
        if (q0 + t < nq)
            v[t] = *(const u32x4 *)(ip + 16 * t);
    }
    uint32_t ks[4][4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const uint32_t jj = q0 + t - qoff;
        ks[t][0] = cb[0];
        ks[t][1] = cb[1];
        ks[t][2] = cb[2];
        ks[t][3] = cb[3] ^ ((jj >> 8) << 16) ^ ((jj & 0xffu) << 24);
    }
    if (conf) {
#pragma unroll
        for (int g = 0; g < 4; g += ICM_NB)
            aes_blocks<ICM_NB, NR ? NR : 1>(
                *reinterpret_cast<uint32_t(*)[ICM_NB][4]>(&ks[g]), rk, T);
    } else {
#pragma unroll
        for (int t = 0; t < 4; t++)
            ks[t][0] = ks[t][1] = ks[t][2] = ks[t][3] = 0;
    }
    uint32_t wv[16];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const uint32_t q = q0 + t;
        uint32_t kk[4];
        ks_shift(ks_prev, ks[t], s, kk);
        if (b < bclean) {
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (4 * q + u < hw)
                    kk[u] = 0;   // header words are never encrypted
        }
        uint32_t o[4] = { v[t].x ^ kk[0], v[t].y ^ kk[1], v[t].z ^ kk[2],
                          v[t].w ^ kk[3] };
        if (16 * q + 16 <= L) {
            *(u32x4 *)(op + 16 * t) = u32x4{ o[0], o[1], o[2], o[3] };
        } else if (16 * q < L) {
            // the one partial quad: stored after the loop (a byte-wise
            // store here, unrolled per quad, costs ~65 VGPRs)
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
        if (64 * b + 64 > L) {
            // message tail: ROC, the 0x80 terminator, zero padding and
            // the bit length (sha1.c srtp_sha1_final)
#pragma unroll
            for (int g = 0; g < 16; g++)
                wv[g] = tail_word(wv[g], (int)L - (int)(64 * b + 4 * g),
                                  roc);
            if (b == nb - 1) {
                wv[14] = 0;
                wv[15] = (64 + L + 4) * 8;
            }
        }
        sha1_compress(hst, wv);
    }
}

// AES-ICM + HMAC-SHA1 protect / unprotect: one lane per packet.
template <int NR, bool AUTH, bool PROTECT, bool UNIFORM>
__global__ __launch_bounds__(512, ICM_WAVES_PER_SIMD) void k_icm_hmac(IcmArgs A)
{
    __shared__ uint2 s_tab[256 * 32];
    if (A.abort && *A.abort)
        return;
    if (NR)
        load_aes_table(s_tab);
    __syncthreads();
    const AesLds T = make_aes_lds(s_tab);

    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.n)
        return;
    const srtp_dev_meta_t m = A.meta[i];
    constexpr uint32_t VID = (NR == 0 ? 0u : 8u + 2u * ((NR - 8) / 2)) +
                             (AUTH ? 1u : 0u);
    if (SRTP_META_STATUS(m.info) || SRTP_META_VARIANT(m.info) != VID)
        return;
    const uint32_t slot = UNIFORM ? A.uni : m.key;
    const srtp_dev_key_t *key = A.keys + slot;

    typename std::conditional<UNIFORM, UniKey<NR ? NR : 1>,
                              LaneKey<NR ? NR : 1>>::type rk;
    if (NR)
        rk.load(key);

    const uint8_t *in = A.in + A.in_off[i];
    uint8_t *out = A.out + A.out_off[i];
    const uint32_t enc_start = SRTP_META_ENC_START(m.info);
    const uint32_t L = m.len;                 // end of auth'd region
    const uint32_t hw = enc_start >> 2, s = hw & 3, qoff = hw >> 2;
    const bool conf = NR != 0 && key->conf != 0;

    // counter block (little-endian words), block counter j in bytes 14..15
    const uint32_t w0 = *(const uint32_t *)in;
    const uint32_t seq = bswap(w0) & 0xffffu;
    uint32_t cb[4];
    cb[0] = key->salt[0];
    cb[1] = key->salt[1] ^ *(const uint32_t *)(in + 8);   // SSRC bytes
    cb[2] = key->salt[2] ^ bswap(m.roc);
    cb[3] = key->salt[3] ^ (seq >> 8) ^ ((seq & 0xffu) << 8);

    uint32_t hst[5];
#pragma unroll
    for (int k = 0; k < 5; k++)
        hst[k] = AUTH ? key->ipad[k] : 0;

    uint32_t ks_prev[4] = { 0, 0, 0, 0 };
    const uint32_t nq = (L + 15) >> 4;             // quads holding data
    const uint32_t nb = AUTH ? ((L + 12) >> 6) + 1 : ((nq + 3) >> 2);
    const uint32_t bclean = (qoff + 4) >> 2;       // first chunk past header

    // One code path for every 64-byte chunk (header, payload, tail): the
    // header / tail / padding handling sits in branches that are not taken
    // in the steady state, so the loop keeps the register footprint of the
    // plain payload chunk (<= 128 VGPRs -> 4 waves per SIMD).  Keystream
    // blocks over header quads or past the payload are computed and masked
    // or never stored.
    uint32_t tailq[4] = { 0, 0, 0, 0 };
    // header chunks, then the payload chunks (branch-free: no header word,
    // no tail, full 16-byte loads and stores), then the tail chunks
    const uint32_t nfull = L >> 6;
    uint32_t b = 0;
    for (; b < bclean && b < nb; b++)
        icm_chunk<NR, AUTH, PROTECT>(b, in, out, L, hw, s, qoff, nq, nb, bclean,
                                     conf, m.roc, cb, rk, T, ks_prev, hst,
                                     tailq);
    for (; b < nfull; b++) {
        const uint8_t *ip = in + 64 * b;
        uint8_t *op = out + 64 * b;
        u32x4 v[4];
#pragma unroll
        for (int t = 0; t < 4; t++)
            v[t] = *(const u32x4 *)(ip + 16 * t);
        uint32_t ks[4][4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const uint32_t jj = 4 * b + t - qoff;
            ks[t][0] = cb[0];
            ks[t][1] = cb[1];
            ks[t][2] = cb[2];
            ks[t][3] = cb[3] ^ ((jj >> 8) << 16) ^ ((jj & 0xffu) << 24);
        }
        if (conf) {
#pragma unroll
            for (int g = 0; g < 4; g += ICM_NB)
                aes_blocks<ICM_NB, NR ? NR : 1>(
                    *reinterpret_cast<uint32_t(*)[ICM_NB][4]>(&ks[g]), rk, T);
        } else {
#pragma unroll
            for (int t = 0; t < 4; t++)
                ks[t][0] = ks[t][1] = ks[t][2] = ks[t][3] = 0;
        }
        uint32_t wv[16];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            uint32_t kk[4];
            ks_shift(ks_prev, ks[t], s, kk);
            u32x4 o = { v[t].x ^ kk[0], v[t].y ^ kk[1], v[t].z ^ kk[2],
                        v[t].w ^ kk[3] };
            *(u32x4 *)(op + 16 * t) = o;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                wv[4 * t + u] = bswap(PROTECT ? o[u] : v[t][u]);
                ks_prev[u] = ks[t][u];
            }
        }
        if (AUTH)
            sha1_compress(hst, wv);
    }
    for (; b < nb; b++)
        icm_chunk<NR, AUTH, PROTECT>(b, in, out, L, hw, s, qoff, nq, nb, bclean,
                                     conf, m.roc, cb, rk, T, ks_prev, hst,
                                     tailq);
    if (L & 15)
        store_words_partial(out + (L & ~15u), tailq, (int)(L & 15));

    const uint32_t tag_len = key->tag_len;
    const uint32_t mki_size = key->mki_size;
    if (!AUTH) {
        if (PROTECT && mki_size) {
            for (uint32_t u = 0; u < mki_size; u++)
                out[L + u] = key->mki[u];
        }
        if (!PROTECT)
            A.auth_ok[i] = 1;
        return;
    }

    // outer hash: SHA1(opad || inner)
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
        const uint8_t *tp = in + L + mki_size;
        uint32_t diff = 0;
        for (uint32_t u = 0; u < tag_len; u++)
            diff |= (uint32_t)(tp[u] ^ (uint8_t)(oh[u >> 2] >> (24 - 8 * (u & 3))));
        A.auth_ok[i] = diff == 0;
    }
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

template <int NR, bool PROTECT, bool UNIFORM>
__global__ __launch_bounds__(512) void k_gcm(GcmArgs A)
{
    __shared__ uint2 s_tab[(AES_LDS_BYTES + (UNIFORM ? GH_LDS_BYTES : 0)) / 8];
    if (A.abort && *A.abort)
        return;
    load_aes_table(s_tab);
    if (UNIFORM) {
        const u32x4 *src =
            (const u32x4 *)(A.ghash + 1024 * A.keys[A.uni].ghash_slot);
        u32x4 *dst = (u32x4 *)((char *)s_tab + AES_LDS_BYTES);
        for (int e = threadIdx.x; e < 256 * 16; e += blockDim.x)
            dst[e] = src[e >> 4];
    }
    __syncthreads();
    const char *lds = (const char *)s_tab;
    const AesLds T = make_aes_lds(s_tab);

    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.n)
        return;
    const srtp_dev_meta_t m = A.meta[i];
    constexpr uint32_t VID = 16u + 2u * ((NR - 8) / 2);
    if (SRTP_META_STATUS(m.info) || SRTP_META_VARIANT(m.info) != VID)
        return;
    const uint32_t slot = UNIFORM ? A.uni : m.key;
    const srtp_dev_key_t *key = A.keys + slot;
    typename std::conditional<UNIFORM, UniKey<NR>, LaneKey<NR>>::type rk;
    rk.load(key);

    GhTab<UNIFORM> G;
    G.lds = lds + AES_LDS_BYTES - 0x10000;   // the 0x10000 comes from lane16
    G.lane16 = ((threadIdx.x & 15) * 16) | 0x10000u;
    G.g = (const u32x4 *)(A.ghash + 1024 * key->ghash_slot);

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
    for (uint32_t j = 0; j < nblk; j++) {
        const int rem = (int)P - (int)(16 * j);
        u32x4 v;
        if (rem >= 16)
            v = *(const u32x4a4 *)(pin + 16 * j);
        else
            v = load_partial(pin + 16 * j, rem);
        uint32_t k0 = c0, k1 = c1, k2 = c2, k3 = bswap(j + 2);
        aes_block<NR>(k0, k1, k2, k3, rk, T);
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
    aes_block<NR>(e0, e1, e2, e3, rk, T);
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
        aes_block<NR>(x0, x1, x2, x3, rk, T);
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
    __shared__ uint2 s_tab[256 * 32];
    load_aes_table(s_tab);
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

void build_ttab_host(uint2 *t)
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
        uint32_t t1 = (t0 << 8) | (t0 >> 24);
        t[x] = make_uint2(t0, t1);
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
    dim3 grid((unsigned)((b->n + 511) / 512)), block(512);
    if (b->uniform_key != 0xffffffffu)
        hipLaunchKernelGGL((k_icm_hmac<NR, AUTH, PROT, true>), grid, block, 0,
                           st, A);
    else
        hipLaunchKernelGGL((k_icm_hmac<NR, AUTH, PROT, false>), grid, block, 0,
                           st, A);
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
    dim3 grid((unsigned)((b->n + 511) / 512)), block(512);
    if (b->uniform_key != 0xffffffffu)
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
        uint2 t[256];
        build_ttab_host(t);
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_ttab), t, sizeof t));
        g_table_ready = dev;
    }
    srtp_gpu_t *g = (srtp_gpu_t *)calloc(1, sizeof(srtp_gpu_t));
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
