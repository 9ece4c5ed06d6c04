// srtp_one.hip -- k_one: ONE packet by one workgroup, for the drop-in
// per-call path (srtp_protect / srtp_unprotect of a single packet,
// srtp/srtp.c:2493-2818 and 2820-3172; the AEAD forms 2088-2267 and
// 2276-2491).  The batch kernels give each packet one lane, so a lone packet
// would take one lane's 88 dependent AES blocks and 23 SHA-1 compressions
// (≈ 110 µs for 1412 bytes, profiles/r06/i_pipelined_percall_e2e/kt_percall);
// here the 256 lanes of a workgroup share it:
//
//   * the packet comes straight from (and goes back to) a pinned, mapped
//     host buffer the host copied it into -- no separate H2D / D2H copies;
//   * AES-ICM / AES-GCM keystream: one CTR block per lane (aes_icm.c:236-414,
//     the GCM counter inc32(J0) + j), XORed into the LDS image;
//   * HMAC-SHA1 (hmac.c:157-229, sha1.c:91-463): the lanes expand every
//     block's message schedule W[0..79] + K in parallel into LDS, then one
//     lane runs the 80 rounds of each compression -- the chain is serial by
//     definition;
//   * GHASH (aes_gcm_ossl.c's EVP GCM): 8 Horner chains with H^8 over
//     per-position tables in LDS (one_ghash), E(J0) by another lane;
//   * unprotect verifies the tag first and decrypts only an authentic
//     packet (srtp.c:2994-3053 before 3091-3101), so a rejected packet's
//     bytes are never touched;
//   * the verdict and a done flag go to the pinned buffer last, so the host
//     spins on host memory instead of synchronising the stream.
#include <stdio.h>
#include <stdlib.h>

#include "srtp_dev_common.h"
#include "srtp_gpu_int.h"

namespace {

constexpr uint32_t ONE_THREADS = 256;
constexpr uint32_t ONE_SCHED_BLOCKS = (SRTP_ONE_MAX + 4 + 9 + 63) / 64 + 1;

// the bytes of block j of keystream XORed into img[es + 16 j, es + P)
DEV void xor_block(uint8_t *img, uint32_t es, uint32_t P, uint32_t j,
                   const uint32_t ks[4])
{
    const uint32_t o = 16 * j;
    if (o + 16 <= P) {   // es is a multiple of 4: whole words
        uint32_t *w = (uint32_t *)(img + es + o);
#pragma unroll
        for (int u = 0; u < 4; u++)
            w[u] ^= ks[u];
        return;
    }
    for (uint32_t b = 0; o + b < P; b++)
        img[es + o + b] ^= (uint8_t)(ks[b >> 2] >> (8 * (b & 3)));
}

// the ICM counter block of packet keystream block j (make_pkt's cb, the
// 16-bit block counter in bytes 14..15)
DEV void icm_ctr(const srtp_dev_key_t *key, const uint8_t *img, uint32_t roc,
                 uint32_t j, uint32_t x[4])
{
    const uint32_t seq = bswap(*(const uint32_t *)img) & 0xffffu;
    x[0] = key->salt[0];
    x[1] = key->salt[1] ^ *(const uint32_t *)(img + 8);   // SSRC bytes
    x[2] = key->salt[2] ^ bswap(roc);
    x[3] = key->salt[3] ^ (seq >> 8) ^ ((seq & 0xffu) << 8) ^
           ((j >> 8) << 16) ^ ((j & 0xffu) << 24);
}

// the GCM counter block IV || be32(ctr) (gcm_packet's c0..c2)
DEV void gcm_ctr(const srtp_dev_key_t *key, const uint8_t *img, uint32_t roc,
                 uint32_t ctr, uint32_t x[4])
{
    const uint32_t w0 = bswap(*(const uint32_t *)img);
    const uint32_t ssrc = bswap(*(const uint32_t *)(img + 8));
    const uint32_t seq = w0 & 0xffffu;
    x[0] = bswap((ssrc >> 16) ^ bswap(key->salt[0]));
    x[1] = bswap(((ssrc << 16) | (roc >> 16)) ^ bswap(key->salt[1]));
    x[2] = bswap(((roc << 16) | seq) ^ bswap(key->salt[2]));
    x[3] = bswap(ctr);
}

template <int NR>
DEV void aes_enc(const srtp_dev_key_t *key, uint32_t x[4], const AesLds &T)
{
    GlobalKey rk{ key };
    aes_block<NR, false>(x[0], x[1], x[2], x[3], rk, T);
}

DEV void aes_any(const srtp_dev_key_t *key, uint32_t x[4], const AesLds &T)
{
    if (key->rounds == 10)
        aes_enc<10>(key, x, T);
    else if (key->rounds == 12)
        aes_enc<12>(key, x, T);
    else
        aes_enc<14>(key, x, T);
}

// message word t of SHA-1 block b over img[0, L) || be32(roc), padded, the
// ipad block counted in the length (hmac_sha1_bytes' layout)
DEV uint32_t sha_word(const uint8_t *img, uint32_t L, uint32_t roc,
                      uint32_t nb, uint32_t b, uint32_t t)
{
    const uint32_t M = L + 4;
    if (b == nb - 1 && t == 15)
        return (64 + M) * 8;
    if (b == nb - 1 && t == 14)
        return 0;
    uint32_t v = 0;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint32_t o = 64 * b + 4 * t + u;
        const uint32_t c = o < L   ? img[o]
                           : o < M ? (roc >> (24 - 8 * (o - L))) & 0xffu
                                   : (o == M ? 0x80u : 0u);
        v = (v << 8) | c;
    }
    return v;
}

// W_t + K_t, t = 0..79, of one SHA-1 block from its 16 message words
// (sha1.c's schedule and round constants)
DEV void sha1_wk(const uint32_t *m16, uint32_t *wk)
{
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; t++)
        w[t] = m16[t];
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
        const uint32_t k = t < 20   ? 0x5a827999u
                           : t < 40 ? 0x6ed9eba1u
                           : t < 60 ? 0x8f1bbcdcu
                                    : 0xca62c1d6u;
        wk[t] = wt + k;
    }
}

// x + y + z in one v_add3_u32 (left to itself the compiler splits the
// round's sum into three adds to start it early, which a lone wave pays for
// in issue slots)
DEV uint32_t add3(uint32_t x, uint32_t y, uint32_t z)
{
    uint32_t r;
    asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
    return r;
}

// the 80 rounds of one compression from W_t + K_t (sha1_compress without
// the schedule): five VALU per round on the chain's lane -- f as one
// v_bitop3 (Ch = 0xCA, parity, majority), e + W_t + K_t, rotl 5, one add3,
// rotl 30
DEV void sha1_rounds_wk(uint32_t h[5], const u32x4 (&wk)[20])
{
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
    for (int t = 0; t < 80; t++) {
        const uint32_t x = wk[t >> 2][t & 3];
        uint32_t f;
        if (t < 20)
            f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA);   // b ? c : d
        else if (t < 40 || t >= 60)
            f = xor3(b, c, d);
        else
            f = maj3(b, c, d);
        const uint32_t tmp = add3(rotl(a, 5), f, e + x);
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

// HMAC-SHA1 tag of img[0, L) || be32(roc).  The lanes build every block's
// padded big-endian message words in LDS in parallel, then every block's
// W_t + K_t (one lane per block; the schedule depends on the message
// only); thread 0 then runs the chain with each block's 80 words in
// registers (twenty 16-byte LDS loads, the next block's issued before the
// current one's rounds).  The digest (big-endian words) in oh, thread 0 only.
DEV void one_hmac(const srtp_dev_key_t *key, const uint8_t *img, uint32_t L,
                  uint32_t roc, uint32_t *msg, uint32_t *wk, uint32_t oh[5],
                  uint8_t *prof = nullptr)
{
    const uint32_t nb = (L + 4 + 9 + 63) / 64;
    for (uint32_t x = threadIdx.x; x < 16 * nb; x += blockDim.x)
        msg[x] = sha_word(img, L, roc, nb, x >> 4, x & 15);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x)
        sha1_wk(msg + 16 * b, wk + 80 * b);
    __syncthreads();
    // one lane runs the chain: ~5 cycles per instruction of a lone wave,
    // at its issue floor, so the schedule's instructions are off it (the
    // same chain on the scalar unit, rotates as two SALU shifts, took 59
    // against 38 us with the schedule in the chain: twice the instructions)
    if (threadIdx.x != 0)
        return;
    if (prof)
        *(uint64_t *)(prof) = __builtin_amdgcn_s_memrealtime();
    uint32_t h[5];
    for (int k = 0; k < 5; k++)
        h[k] = key->ipad[k];
    // two register sets, A and B, alternate (no copies between blocks)
    const u32x4 *mv = (const u32x4 *)wk;
    u32x4 A[20], B[20];
#pragma unroll
    for (int q = 0; q < 20; q++)
        A[q] = mv[q];
    for (uint32_t b = 0; b < nb; b += 2) {
        if (b + 1 < nb)
#pragma unroll
            for (int q = 0; q < 20; q++)
                B[q] = mv[20 * (b + 1) + q];
        sha1_rounds_wk(h, A);
        if (b + 1 >= nb)
            break;
        if (b + 2 < nb)
#pragma unroll
            for (int q = 0; q < 20; q++)
                A[q] = mv[20 * (b + 2) + q];
        sha1_rounds_wk(h, B);
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

// X <- X * x in GF(2^128), GCM bit order (x^0 = bit 31 of word 0)
DEV void gf_mulx(uint32_t v[4])
{
    const uint32_t c = v[3] & 1u;
    v[3] = (v[3] >> 1) | (v[2] << 31);
    v[2] = (v[2] >> 1) | (v[1] << 31);
    v[1] = (v[1] >> 1) | (v[0] << 31);
    v[0] = (v[0] >> 1) ^ (c ? 0xe1000000u : 0u);
}

// LDS layout past the (T0, T1) tables: GhPos8's per-position tables need
// bases on 32-KiB boundaries of the one LDS object they are addressed from
constexpr uint32_t ONE_POS_H = AES_TAB2_BYTES;             // tables of H
constexpr uint32_t ONE_POS_HK = AES_TAB2_BYTES + 32768;    // ... of H^K
constexpr uint32_t ONE_LDS_BIG = AES_TAB2_BYTES + 65536;

// GhPos8's tables from a Shoup table M: entry b of table t = M[b] * x^(8t)
DEV void one_pos_tables(const u32x4 *M, u32x4 *dst)
{
    for (uint32_t b = threadIdx.x; b < 256; b += blockDim.x) {
        u32x4 z = M[b];
#pragma unroll
        for (int t = 0; t < 8; t++) {
            dst[b * 8 + t] = z;
            z = ghash_mulx8(z);
        }
    }
}

// GHASH of the AAD img[0, A) and the ciphertext img[A, A + C), length block
// last (gcm_packet's order): Y = sum over blocks j < n of X_j * H^(n - j).
// A lone lane's multiply through Shoup's table is 16 dependent LDS reads
// (~0.6 us); through the per-position tables of k_gcm's uniform form
// (GhPos8) its 16 reads are independent (~0.1 us).  So: H's per-position
// tables from its Shoup table; H^K by K - 1 multiplies on one lane; H^K's
// Shoup table (XORs of its 8 basis values H^K * x^i) and per-position
// tables; then ONE_GH_LANES chains -- lane r takes blocks j = r (mod K) by
// Horner with H^K, Z_r = sum_i X_(r+iK) H^(K(m-i)), then Y_r = Z_r *
// H^(n - j_last) (at most K multiplies by H) -- and Y is the XOR of the Y_r.
// blk: the zero-padded big-endian blocks, built by all lanes; lds: the LDS
// object holding the per-position tables; x: BE words, thread 0 only.
constexpr uint32_t ONE_GH_LANES = 8;
DEV void one_ghash(const char *lds, const u32x4 *tab, u32x4 *tabk, u32x4 *pw,
                   const uint8_t *img, uint32_t A, uint32_t C, u32x4 *blk,
                   uint32_t x[4])
{
    const uint32_t na = (A + 15) / 16, nc = (C + 15) / 16, n = na + nc + 1;
    for (uint32_t q = threadIdx.x; q < 4 * n; q += blockDim.x) {
        const uint32_t j = q >> 2, u = q & 3;
        uint32_t v = 0;
        if (j + 1 == n) {   // [len(A)]64 || [len(C)]64 in bits
            v = u == 1 ? A * 8 : u == 3 ? C * 8 : 0u;
        } else {
            const uint32_t base = j < na ? 16 * j : A + 16 * (j - na);
            const uint32_t lim = j < na ? A : A + C;
            for (int b = 0; b < 4; b++) {
                const uint32_t o = base + 4 * u + b;
                v = (v << 8) | (o < lim ? img[o] : 0u);
            }
        }
        ((uint32_t *)blk)[q] = v;
    }
    one_pos_tables(tab, (u32x4 *)(lds + ONE_POS_H));
    __syncthreads();
    const uint32_t t = threadIdx.x, K = ONE_GH_LANES;
    GhPos8 GH;
    GH.init(lds, ONE_POS_H, t);
    if (t == 0) {   // H^K, then the basis of its table: H^K * x^i, i = 0..7
        const u32x4 h1 = tab[0x80];   // M[0x80] = H
        uint32_t v[4] = { h1.x, h1.y, h1.z, h1.w };
        for (uint32_t k = 1; k < K; k++)
            ghash_mul(v, GH);
        for (int i = 0; i < 8; i++) {
            pw[K + i] = u32x4{ v[0], v[1], v[2], v[3] };
            gf_mulx(v);
        }
    }
    __syncthreads();
    for (uint32_t e = t; e < 256; e += blockDim.x) {   // entry b: bit 7 = x^0
        u32x4 acc = { 0, 0, 0, 0 };
        for (int i = 0; i < 8; i++)
            if (e & (0x80u >> i))
                acc ^= pw[K + i];
        tabk[e] = acc;
    }
    __syncthreads();
    one_pos_tables(tabk, (u32x4 *)(lds + ONE_POS_HK));
    __syncthreads();
    if (t < K) {
        GhPos8 GK;
        GK.init(lds, ONE_POS_HK, t);
        uint32_t z[4] = { 0, 0, 0, 0 };
        uint32_t last = t;
        for (uint32_t j = t; j < n; j += K) {
            if (j != t)
                ghash_mul(z, GK);
            const u32x4 c = blk[j];
            z[0] ^= c.x;
            z[1] ^= c.y;
            z[2] ^= c.z;
            z[3] ^= c.w;
            last = j;
        }
        if (t < n)
            for (uint32_t k = 0; k < n - last; k++)
                ghash_mul(z, GH);
        else
            z[0] = z[1] = z[2] = z[3] = 0;
        pw[2 * K + 8 + t] = u32x4{ z[0], z[1], z[2], z[3] };
    }
    __syncthreads();
    if (t == 0) {
        u32x4 y = { 0, 0, 0, 0 };
        for (uint32_t r = 0; r < K; r++)
            y ^= pw[2 * K + 8 + r];
        x[0] = y.x;
        x[1] = y.y;
        x[2] = y.z;
        x[3] = y.w;
    }
}

struct OneArgs {
    uint8_t *buf;                 // pinned host buffer (device address)
    const srtp_dev_key_t *keys;
    const uint32_t *ghash;        // the GHASH table arena
    srtp_dev_meta_t m;
    uint32_t len;                 // bytes of the packet in buf
    int op;                       // 0 protect, 1 unprotect
    int prof;                     // SRTP_ONE_PROFILE: phase timestamps
};

// SRTP_ONE_PROFILE=1: thread 0 stamps the 100 MHz real-time counter at the
// phase boundaries into the staging buffer past the done word
#define ONE_STAMP(k)                                                           \
    do {                                                                       \
        if (a.prof && threadIdx.x == 0)                                        \
            ((uint64_t *)(a.buf + SRTP_ONE_FLAG + 8))[k] =                     \
                __builtin_amdgcn_s_memrealtime();                              \
    } while (0)

__global__ __launch_bounds__(ONE_THREADS) void k_one(OneArgs a)
{
    // (T0, T1) 64 KiB, then GCM: the per-position GHASH tables of H and
    // H^K (32 KiB each) / ICM: the SHA-1 W_t + K_t
    __shared__ u32x4 s_tab[ONE_LDS_BIG / 16];
    __shared__ uint32_t s_t0[256];                   // the T0 row
    __shared__ u32x4 s_img[SRTP_ONE_MAX / 16 + 1];   // the packet
    __shared__ u32x4 s_gh[256];                      // GCM: M[b] = b * H
    __shared__ u32x4 s_ghk[256];                     // ... and b * H^K
    __shared__ u32x4 s_pw[40];                       // H^1..K, basis, Y_r
    __shared__ uint32_t s_msg[ONE_SCHED_BLOCKS * 16];   // SHA-1 / GHASH input
    __shared__ uint32_t s_tag[5], s_ok;
    uint8_t *img = (uint8_t *)s_img;
    const srtp_dev_key_t *key = a.keys + a.m.key;
    const uint32_t tid = threadIdx.x;
    const bool gcm = key->family == SRTP_DEV_GCM;
    ONE_STAMP(0);
    // the T0 row, then the packet's words (4-byte: buf is the staging
    // buffer's start) and GCM's Shoup table loaded into registers while the
    // replicated tables fill, then into LDS: the PCIe / L2 latency of the
    // loads overlaps the table build
    for (uint32_t x = tid; x < 256; x += blockDim.x)
        s_t0[x] = aes_t0(x);
    __syncthreads();
    ONE_STAMP(1);
    constexpr uint32_t NWT = (SRTP_ONE_MAX / 4 + ONE_THREADS - 1) / ONE_THREADS;
    const uint32_t nw = (a.len + 3) / 4;
    uint32_t pkw[NWT];
#pragma unroll
    for (uint32_t k = 0; k < NWT; k++)
        if (tid + ONE_THREADS * k < nw)
            pkw[k] = ((const uint32_t *)a.buf)[tid + ONE_THREADS * k];
    u32x4 ghv = { 0, 0, 0, 0 };
    if (gcm)
        ghv = ((const u32x4 *)(a.ghash + 1024 * key->ghash_slot))[tid];
    fill_aes_tables<false>(s_tab, s_t0);
#pragma unroll
    for (uint32_t k = 0; k < NWT; k++)
        if (tid + ONE_THREADS * k < nw)
            ((uint32_t *)img)[tid + ONE_THREADS * k] = pkw[k];
    if (gcm)   // the arena's entry tid is M[ghash_nswap(tid)]
        s_gh[ghash_nswap(tid)] = ghv;
    __syncthreads();
    ONE_STAMP(2);
    const AesLds T = make_aes_lds(s_tab);
    const uint32_t es = SRTP_META_ENC_START(a.m.info), L = a.m.len;
    const uint32_t P = L - es;
    const uint32_t tag_len = key->tag_len, mki = key->mki_size;
    const bool conf = key->family != SRTP_DEV_NULL && key->rounds != 0 &&
                      (gcm || key->conf != 0);
    const bool protect = a.op == 0;
    uint32_t out_end = L;   // bytes written back
    bool ok = true;

    if (gcm) {
        // keystream blocks j (counter j + 2) by lane; E(J0) by lane 255
        uint32_t ks[4] = { 0, 0, 0, 0 }, ej[4] = { 0, 0, 0, 0 };
        const uint32_t nbk = (P + 15) / 16;
        for (uint32_t j = tid; j < nbk; j += blockDim.x) {
            gcm_ctr(key, img, a.m.roc, j + 2, ks);
            aes_any(key, ks, T);
            if (protect)
                xor_block(img, es, P, j, ks);
            else if (j + blockDim.x >= nbk)
                break;   // kept in registers (one block per lane or fewer)
        }
        if (tid == blockDim.x - 1) {
            gcm_ctr(key, img, a.m.roc, 1, ej);
            aes_any(key, ej, T);
            for (int u = 0; u < 4; u++)
                s_tag[u] = ej[u];
        }
        __syncthreads();
        ONE_STAMP(3);
        ONE_STAMP(4);   // (GCM: no schedule phase; "chain" is the GHASH)
        {
            uint32_t x[4];
            one_ghash((const char *)s_tab, s_gh, s_ghk, s_pw, img, es, P,
                      (u32x4 *)s_msg, x);
            ONE_STAMP(5);
            if (tid == 0) {
            uint32_t tw[4] = { bswap(x[0]) ^ s_tag[0], bswap(x[1]) ^ s_tag[1],
                               bswap(x[2]) ^ s_tag[2], bswap(x[3]) ^ s_tag[3] };
            if (protect) {
                store_tag(img + L, tw, tag_len);
                for (uint32_t u = 0; u < mki; u++)
                    img[L + tag_len + u] = key->mki[u];
            } else {
                s_ok = tag_diff(img + L, tw, tag_len) == 0;
            }
            }
        }
        __syncthreads();
        if (!protect) {
            ok = s_ok != 0;
            // decrypt only an authentic packet (a lane holds its block's
            // keystream when there are no more blocks than lanes)
            if (ok)
                for (uint32_t j = tid; j < nbk; j += blockDim.x) {
                    if (nbk > blockDim.x) {
                        gcm_ctr(key, img, a.m.roc, j + 2, ks);
                        aes_any(key, ks, T);
                    }
                    xor_block(img, es, P, j, ks);
                }
        } else {
            out_end = L + tag_len + mki;
        }
    } else {
        const bool auth = key->auth != 0;
        const uint32_t nbk = conf ? (P + 15) / 16 : 0;
        if (protect) {
            for (uint32_t j = tid; j < nbk; j += blockDim.x) {
                uint32_t ks[4];
                icm_ctr(key, img, a.m.roc, j, ks);
                aes_any(key, ks, T);
                xor_block(img, es, P, j, ks);
            }
            __syncthreads();
            ONE_STAMP(3);
            if (tid == 0)
                for (uint32_t u = 0; u < mki; u++)
                    img[L + u] = key->mki[u];
            if (auth) {
                uint32_t oh[5];
                one_hmac(key, img, L, a.m.roc, s_msg, (uint32_t *)((char *)s_tab + ONE_POS_H), oh,
                         a.prof ? a.buf + SRTP_ONE_FLAG + 8 + 8 * 4 : nullptr);
                ONE_STAMP(5);
                if (tid == 0) {
                    uint32_t tw[5];
                    for (int k = 0; k < 5; k++)
                        tw[k] = bswap(oh[k]);
                    store_tag(img + L + mki, tw, tag_len);
                }
            }
            out_end = L + mki + (auth ? tag_len : 0);
        } else {
            if (auth) {
                uint32_t oh[5];
                one_hmac(key, img, L, a.m.roc, s_msg, (uint32_t *)((char *)s_tab + ONE_POS_H), oh);
                if (tid == 0) {
                    uint32_t tw[5];
                    for (int k = 0; k < 5; k++)
                        tw[k] = bswap(oh[k]);
                    s_ok = tag_diff(img + L + mki, tw, tag_len) == 0;
                }
                __syncthreads();
                ok = s_ok != 0;
            }
            if (ok)
                for (uint32_t j = tid; j < nbk; j += blockDim.x) {
                    uint32_t ks[4];
                    icm_ctr(key, img, a.m.roc, j, ks);
                    aes_any(key, ks, T);
                    xor_block(img, es, P, j, ks);
                }
        }
    }
    __syncthreads();
    ONE_STAMP(6);
    // the result back into the pinned buffer (a rejected packet: nothing),
    // then the verdict word and the done flag, visible to the host in order
    const uint32_t ow = ok ? (out_end + 3) / 4 : 0;
    for (uint32_t w = tid; w < ow; w += blockDim.x)
        ((uint32_t *)a.buf)[w] = ((const uint32_t *)img)[w];
    __threadfence_system();
    __syncthreads();
    ONE_STAMP(7);
    if (tid == 0)
        __hip_atomic_store((uint32_t *)(a.buf + SRTP_ONE_FLAG),
                           0x100u | (ok ? 1u : 0u), __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

}   // namespace

extern "C" {

// the pinned staging buffer of the per-call path (allocated on first use):
// SRTP_ONE_MAX bytes of packet, then the verdict / done word
uint8_t *srtp_gpu_one_buf(srtp_gpu_t *g)
{
    if (!g->one_h) {
        void *h = nullptr;
        if (hipHostMalloc(&h, SRTP_ONE_FLAG + 128, hipHostMallocMapped) !=
            hipSuccess)
            return nullptr;
        void *d = nullptr;
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
            (void)hipHostFree(h);
            return nullptr;
        }
        g->one_h = (uint8_t *)h;
        g->one_d = (uint8_t *)d;
    }
    return g->one_h;
}

int srtp_gpu_one(srtp_gpu_t *g, int op, uint32_t len, const srtp_dev_meta_t *m,
                 void *stream, int *ok)
{
    if (!g->one_h || len > SRTP_ONE_MAX || m->len + SRTP_ONE_TRAILER > SRTP_ONE_MAX)
        return srtp_gpu_fail(hipErrorInvalidValue, "srtp_gpu_one");
    hipStream_t st = stream ? (hipStream_t)stream : g->stream;
    volatile uint32_t *flag = (volatile uint32_t *)(g->one_h + SRTP_ONE_FLAG);
    *flag = 0;
    OneArgs a;
    a.buf = g->one_d;
    a.keys = g->d_keys;
    a.ghash = g->d_ghash;
    a.m = *m;
    a.len = len;
    a.op = op;
    static const int prof = [] {
        const char *e = getenv("SRTP_ONE_PROFILE");
        return e && *e == '1' ? 1 : 0;
    }();
    a.prof = prof;
    hipLaunchKernelGGL(k_one, dim3(1), dim3(ONE_THREADS), 0, st, a);
    HIPCHK(hipGetLastError());
    // the kernel's done flag in host memory; the stream is asked now and
    // then, so a failed launch cannot spin forever
    for (uint32_t k = 1;; k++) {
        const uint32_t v = *flag;
        if (v & 0x100u) {
            *ok = (int)(v & 1u);
            if (prof) {   // phase times in microseconds (100 MHz counter)
                static int shown = 0;
                const uint64_t *t =
                    (const uint64_t *)(g->one_h + SRTP_ONE_FLAG + 8);
                if (shown++ < 12)
                    fprintf(stderr, "k_one op %d: load %.1f tables %.1f "
                            "crypt %.1f sched %.1f chain %.1f tail %.1f "
                            "fence %.1f us\n", op, (t[1] - t[0]) / 100.0,
                            (t[2] - t[1]) / 100.0, (t[3] - t[2]) / 100.0,
                            (t[4] - t[3]) / 100.0, (t[5] - t[4]) / 100.0,
                            (t[6] - t[5]) / 100.0, (t[7] - t[6]) / 100.0);
            }
            return 0;
        }
        if ((k & 4095) == 0) {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipSuccess) {
                const uint32_t w = *flag;
                if (!(w & 0x100u))
                    return srtp_gpu_fail(hipErrorLaunchFailure, "k_one flag");
                *ok = (int)(w & 1u);
                return 0;
            }
            if (q != hipErrorNotReady)
                return srtp_gpu_fail(q, "k_one");
        }
        __builtin_ia32_pause();
    }
}

}   // extern "C"
