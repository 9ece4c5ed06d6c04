// srtp_gpu.hip -- the thin extern "C" FFI (srtp_dev.h) between the C host
// engine and the HIP kernels: device context, key table, kernel dispatch,
// plus the small kernels (speculative-unprotect undo, SRTCP, header parse).
// The RTP crypto kernels live in srtp_icm.hip and srtp_gcm.hip
// (srtp_gpu_int.h).
#include <stdio.h>
#include <stdlib.h>

#include "srtp_dev_common.h"
#include "srtp_gpu_int.h"

namespace {

// ---------------------------------------------------------------------------
// Restore kernel for speculative unprotect: XORs the keystream the
// speculative pass used back over [enc_start, len) so the ciphertext of a
// packet that must be re-run (or is rejected) is intact again (CTR
// decryption is an XOR).  One packet by a whole wave: lane l takes CTR
// blocks l, l + 64, ...
// (a 1400-byte packet is 88 blocks: two AES steps per lane instead of 88
// dependent ones on one lane)
template <int NR>
DEV void undo_wave(const srtp_dev_key_t *key, const srtp_dev_meta_t &m,
                   uint8_t *p, const AesLds &T, uint32_t lane)
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
    for (uint32_t j = lane; 16 * j < P; j += 64) {
        uint32_t x0 = c0, x1 = c1, x2 = c2, x3;
        if (gcm)
            x3 = bswap(j + 2);
        else
            x3 = c3base ^ ((j >> 8) << 16) ^ ((j & 0xffu) << 24);
        aes_block<NR, false>(x0, x1, x2, x3, rk, T);
        const uint32_t ks[4] = { x0, x1, x2, x3 };
        for (uint32_t b = 0; b < 16 && 16 * j + b < P; b++)
            p[enc_start + 16 * j + b] ^= (uint8_t)(ks[b >> 2] >> (8 * (b & 3)));
    }
}

// header-extension / cryptex packets (k_xrtp, below): undo of an unprotect
DEV uint8_t xrtp_unprotect(const srtp_dev_key_t *keys, const srtp_dev_meta_t &m,
                           const uint8_t *src, uint8_t *p, bool undo,
                           const AesLds &T);

// The packets to undo, compacted (wave-aggregated atomic): most batches
// have few or none
__global__ __launch_bounds__(256) void k_undo_list(const srtp_dev_meta_t *meta,
                                                   uint32_t n, uint32_t *list,
                                                   uint32_t *count)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool todo = i < n && !SRTP_META_STATUS(meta[i].info);
    const uint64_t bal = __ballot(todo);
    if (!bal)
        return;
    const uint32_t lane = threadIdx.x & 63, lead = __ffsll((long long)bal) - 1;
    uint32_t base = 0;
    if (lane == lead)
        base = atomicAdd(count, (uint32_t)__popcll(bal));
    base = __shfl(base, lead);
    if (todo)
        list[base + __popcll(bal & ((1ull << lane) - 1))] = i;
}

// ... then one wave per listed packet; the
// blocks past the list leave before building the tables
__global__ __launch_bounds__(256) void k_undo_wave(uint8_t *arena,
                                                   const uint64_t *off,
                                                   const srtp_dev_meta_t *meta,
                                                   const srtp_dev_key_t *keys,
                                                   const uint32_t *list,
                                                   const uint32_t *count)
{
    __shared__ u32x4 s_tab[AES_TAB2_BYTES / 16];
    const uint32_t cnt = *count;
    const uint32_t wpb = blockDim.x >> 6;
    if (blockIdx.x * wpb >= cnt)
        return;
    load_aes_tables<false>(s_tab);
    __syncthreads();
    const AesLds T = make_aes_lds(s_tab);
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t w = blockIdx.x * wpb + (threadIdx.x >> 6); w < cnt;
         w += gridDim.x * wpb) {
        const uint32_t i = list[w];
        const srtp_dev_meta_t m = meta[i];
        const srtp_dev_key_t *key = keys + m.key;
        uint8_t *p = arena + off[i];
        if (SRTP_META_VARIANT(m.info) == SRTP_VARIANT_X) {
            if (lane == 0)
                xrtp_unprotect(keys, m, p, p, true, T);
            continue;
        }
        if (!key->conf || key->family == SRTP_DEV_NULL)
            continue;
        if (key->rounds == 10)
            undo_wave<10>(key, m, p, T, lane);
        else if (key->rounds == 12)
            undo_wave<12>(key, m, p, T, lane);
        else
            undo_wave<14>(key, m, p, T, lane);
    }
}

// ---------------------------------------------------------------------------
// SRTCP (srtp.c:4304-4544 protect, 4546-4837 unprotect): one lane per packet.
// RTCP is a low-rate control channel, so this is the plain byte-wise form of
// the RTP kernel's pieces: AES-ICM keystream over [8, P), the E|index trailer
// at P, MKI, HMAC-SHA1 over [0, P + 4).

// HMAC-SHA1 over msg[0, L) || tail[0, nt) (hmac.c:157-229; SRTCP has no
// tail, SRTP's is the big-endian ROC)
DEV void hmac_sha1_bytes(const srtp_dev_key_t *key, const uint8_t *msg,
                         uint32_t L, uint32_t oh[5],
                         const uint8_t *tail = nullptr, uint32_t nt = 0)
{
    uint32_t h[5];
    for (int k = 0; k < 5; k++)
        h[k] = key->ipad[k];
    const uint32_t M = L + nt;
    const uint32_t nb = (M + 1 + 8 + 63) / 64;   // data, 0x80, 64-bit length
    const uint32_t bits = (64 + M) * 8;          // the ipad block counts
    for (uint32_t b = 0; b < nb; b++) {
        uint32_t w[16];
        for (int t = 0; t < 16; t++) {
            uint32_t v = 0;
            for (int u = 0; u < 4; u++) {
                const uint32_t o = 64 * b + 4 * t + u;
                const uint32_t c = o < L   ? msg[o]
                                   : o < M ? tail[o - L]
                                           : (o == M ? 0x80u : 0u);
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
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    srtp_dev_meta_t m = {};
    if (i < n)
        m = meta[i];
    const bool todo = i < n && !SRTP_META_STATUS(m.info);
    // most blocks have nothing to undo (every packet authenticated): they
    // leave before building the tables
    if (!__syncthreads_or(todo))
        return;
    load_aes_tables<false>(s_tab);
    __syncthreads();
    if (!todo)
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
                        const uint32_t *in_len, srtp_dev_hdr_t *hdr,
                        uint32_t *xinfo, uint32_t n)
{
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint64_t off = in_off[i];
    const srtp_dev_hdr_t h = srtp_parse_rtp(in + off, off, in_len[i]);
    hdr[i] = h;
    if (xinfo)
        xinfo[i] = srtp_rtp_xinfo(in + off, h);
}

// ---------------------------------------------------------------------------
// Single-buffer operations of the crypto-kernel API (srtp_gpu_raw): one
// workgroup; AES-CTR blocks across the lanes, GHASH / SHA-1 on lane 0 (the
// API moves one buffer per call: a handful of blocks).
struct RawDev {
    int op;
    const srtp_dev_key_t *key;
    const uint8_t *src;
    uint8_t *dst;
    uint32_t len, nlead, aad_len, tag_len;
    uint8_t ctr[16], lead[16], iv[12];
    const uint8_t *aad;
    uint8_t *res;   // [0,16) keystream of the last ICM block, [16] GCM ok
};

template <int NR>
DEV void raw_icm(const RawDev &A, const AesLds &T)
{
    GlobalKey rk{ A.key };
    const uint32_t body = A.len > A.nlead ? A.len - A.nlead : 0;
    const uint32_t nb = (body + 15) / 16;
    if (threadIdx.x == 0)
        for (uint32_t b = 0; b < A.nlead && b < A.len; b++)
            A.dst[b] = A.src[b] ^ A.lead[b];
    uint32_t c[4];
    for (int w = 0; w < 4; w++)
        c[w] = (uint32_t)A.ctr[4 * w] | (uint32_t)A.ctr[4 * w + 1] << 8 |
               (uint32_t)A.ctr[4 * w + 2] << 16 | (uint32_t)A.ctr[4 * w + 3] << 24;
    const uint32_t c16 = (uint32_t)A.ctr[14] << 8 | A.ctr[15];
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) {
        const uint32_t k = (c16 + j) & 0xffffu;   // the caller checked 0xffff
        uint32_t x0 = c[0], x1 = c[1], x2 = c[2];
        uint32_t x3 = (c[3] & 0xffffu) | (k >> 8) << 16 | (k & 0xffu) << 24;
        aes_block<NR, false>(x0, x1, x2, x3, rk, T);
        const uint32_t ks[4] = { x0, x1, x2, x3 };
        const uint32_t o = A.nlead + 16 * j;
        for (uint32_t b = 0; b < 16 && o + b < A.len; b++)
            A.dst[o + b] = A.src[o + b] ^ (uint8_t)(ks[b >> 2] >> (8 * (b & 3)));
        if (j == nb - 1)
            for (uint32_t b = 0; b < 16; b++)
                A.res[b] = (uint8_t)(ks[b >> 2] >> (8 * (b & 3)));
    }
}

// GHASH(aad || data || lengths) and E_K(J0): the 16-byte tag before
// truncation (SP 800-38D 7.1-7.2)
template <int NR>
DEV void raw_gcm_tag(const RawDev &A, const uint8_t *data, uint8_t tag[16],
                     const AesLds &T)
{
    Ghash G;
    G.xh = G.xl = 0;
    G.hh = (uint64_t)A.key->h[0] << 32 | A.key->h[1];
    G.hl = (uint64_t)A.key->h[2] << 32 | A.key->h[3];
    G.fill = 0;
    for (uint32_t u = 0; u < A.aad_len; u++)
        G.put(A.aad[u]);
    G.flush();
    for (uint32_t u = 0; u < A.len; u++)
        G.put(data[u]);
    G.flush();
    G.xh ^= (uint64_t)A.aad_len * 8;
    G.xl ^= (uint64_t)A.len * 8;
    gf128_mul(G.xh, G.xl, G.hh, G.hl);
    uint32_t ks[4];
    gcm_block<NR>(A.key, A.iv, 1, ks, T);
    for (int u = 0; u < 16; u++) {
        const uint64_t half = u < 8 ? G.xh : G.xl;
        tag[u] = (uint8_t)(half >> (56 - 8 * (u & 7))) ^
                 (uint8_t)(ks[u >> 2] >> (8 * (u & 3)));
    }
}

template <int NR>
DEV void raw_gcm(const RawDev &A, bool seal, const AesLds &T)
{
    if (!seal && threadIdx.x == 0) {   // verify before the buffer changes
        uint8_t tag[16];
        raw_gcm_tag<NR>(A, A.src, tag, T);
        uint32_t diff = 0;
        for (uint32_t u = 0; u < A.tag_len; u++)
            diff |= tag[u] ^ A.src[A.len + u];
        A.res[16] = diff == 0;
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; 16 * j < A.len; j += blockDim.x) {
        uint32_t ks[4];
        gcm_block<NR>(A.key, A.iv, j + 2, ks, T);
        for (uint32_t b = 0; b < 16 && 16 * j + b < A.len; b++)
            A.dst[16 * j + b] =
                A.src[16 * j + b] ^ (uint8_t)(ks[b >> 2] >> (8 * (b & 3)));
    }
    __syncthreads();
    if (seal && threadIdx.x == 0) {
        uint8_t tag[16];
        raw_gcm_tag<NR>(A, A.dst, tag, T);
        for (uint32_t u = 0; u < A.tag_len; u++)
            A.dst[A.len + u] = tag[u];
    }
}

__global__ __launch_bounds__(256) void k_raw(RawDev A)
{
    __shared__ u32x4 s_tab[AES_TAB2_BYTES / 16];
    load_aes_tables<false>(s_tab);
    __syncthreads();
    const AesLds T = make_aes_lds(s_tab);
    if (A.op == SRTP_RAW_HMAC) {
        if (threadIdx.x == 0) {
            uint32_t oh[5];
            hmac_sha1_bytes(A.key, A.src, A.len, oh);
            for (int u = 0; u < 20; u++)
                A.dst[u] = (uint8_t)(oh[u >> 2] >> (24 - 8 * (u & 3)));
        }
        return;
    }
    const uint32_t nr = A.key->rounds;
    if (A.op == SRTP_RAW_ICM) {
        if (nr == 10)
            raw_icm<10>(A, T);
        else if (nr == 12)
            raw_icm<12>(A, T);
        else
            raw_icm<14>(A, T);
        return;
    }
    const bool seal = A.op == SRTP_RAW_GCM_SEAL;
    if (nr == 10)
        raw_gcm<10>(A, seal, T);
    else
        raw_gcm<14>(A, seal, T);
}

// ---------------------------------------------------------------------------
// RFC 6904 header-extension encryption and RFC 9335 cryptex.  Streams with
// either feature send every packet here (SRTP_VARIANT_X): one lane per
// packet, byte-wise, any family and key size.  It follows srtp_protect
// (srtp.c:2642-2818) / srtp_protect_aead (2163-2267) and srtp_unprotect
// (2984-3106) / srtp_unprotect_aead (2360-2423) from the header copy on; the
// host pre-pass did the rest (index, replay, key limit, cryptex_err and the
// header-length parse errors).  These are uncommon per-stream options, so
// this path is written for exactness, not rate.

DEV void aes_rt(const srtp_dev_key_t *k, uint32_t x[4], const AesLds &T)
{
    GlobalKey rk{ k };
    if (k->rounds == 10)
        aes_block<10, false>(x[0], x[1], x[2], x[3], rk, T);
    else if (k->rounds == 12)
        aes_block<12, false>(x[0], x[1], x[2], x[3], rk, T);
    else
        aes_block<14, false>(x[0], x[1], x[2], x[3], rk, T);
}

// the keystream of one SRTP counter mode, consumed a byte at a time (the
// reference's srtp_cipher_output / encrypt calls continue one stream)
struct Kstream {
    const srtp_dev_key_t *key;
    uint32_t c[4];      // counter block, little-endian words
    uint32_t ks[4];
    uint32_t j, pos;    // next block number, bytes of ks used
    bool gcm, null;

    // AES-ICM, IV 0^4 || SSRC || ROC || SEQ || 0^2 xor the salt, 16-bit
    // block counter in bytes 14..15 (srtp.c:2694-2707, aes_icm.c:236-282);
    // the null cipher's keystream is zero
    DEV void icm(const srtp_dev_key_t *k, const uint8_t *hdr, uint32_t roc)
    {
        key = k;
        gcm = false;
        null = k->family == SRTP_DEV_NULL;
        const uint32_t seq = (uint32_t)hdr[2] << 8 | hdr[3];
        c[0] = k->salt[0];
        c[1] = k->salt[1] ^ ((uint32_t)hdr[8] | (uint32_t)hdr[9] << 8 |
                             (uint32_t)hdr[10] << 16 | (uint32_t)hdr[11] << 24);
        c[2] = k->salt[2] ^ bswap(roc);
        c[3] = k->salt[3] ^ (seq >> 8) ^ ((seq & 0xffu) << 8);
        j = 0;
        pos = 16;
    }

    // AES-GCM counter blocks IV || be32(2 + i), IV = salt ^ (00 00 || SSRC ||
    // ROC || SEQ) (RFC 7714 8.1, srtp.c:1896-1950)
    DEV void aead(const srtp_dev_key_t *k, const uint8_t *hdr, uint32_t roc)
    {
        key = k;
        gcm = true;
        null = false;
        const uint8_t *salt = (const uint8_t *)k->salt;
        uint8_t iv[12];
        for (int u = 0; u < 12; u++)
            iv[u] = salt[u];
        for (int u = 0; u < 4; u++) {
            iv[2 + u] ^= hdr[8 + u];
            iv[6 + u] ^= (uint8_t)(roc >> (24 - 8 * u));
        }
        iv[10] ^= hdr[2];
        iv[11] ^= hdr[3];
        for (int w = 0; w < 3; w++)
            c[w] = (uint32_t)iv[4 * w] | (uint32_t)iv[4 * w + 1] << 8 |
                   (uint32_t)iv[4 * w + 2] << 16 | (uint32_t)iv[4 * w + 3] << 24;
        c[3] = 0;
        j = 2;
        pos = 16;
    }

    DEV void block(uint32_t b, uint32_t out[4], const AesLds &T) const
    {
        out[0] = c[0];
        out[1] = c[1];
        out[2] = c[2];
        out[3] = gcm ? bswap(b)
                     : c[3] ^ (((b >> 8) & 0xffu) << 16) ^ ((b & 0xffu) << 24);
        if (null)
            out[0] = out[1] = out[2] = out[3] = 0;
        else
            aes_rt(key, out, T);
    }

    DEV uint8_t next(const AesLds &T)
    {
        if (pos == 16) {
            block(j++, ks, T);
            pos = 0;
        }
        const uint8_t b = (uint8_t)(ks[pos >> 2] >> (8 * (pos & 3)));
        pos++;
        return b;
    }
};

// RTP header geometry: CSRC count, X bit, fixed + CSRC length, extension
// end, and the enc_start of a packet without cryptex
struct XGeo {
    uint32_t cc, x, hl, xend;
};

DEV XGeo xgeo(const uint8_t *p)
{
    XGeo g;
    g.cc = p[0] & 15u;
    g.x = (p[0] >> 4) & 1u;
    g.hl = 12 + 4 * g.cc;
    g.xend = g.x ? g.hl + 4 + 4 * ((uint32_t)p[g.hl + 2] << 8 | p[g.hl + 3])
                 : g.hl;
    return g;
}

// the encrypted byte ranges in keystream order: cryptex takes the CSRCs,
// the extension data and the payload (srtp.c:135-226, the in-place form
// moves the extension header word out of the way; the not-in-place form
// encrypts the CSRCs first), otherwise the payload after the header
DEV uint32_t xsegs(const XGeo &g, bool crx, uint32_t L, uint32_t lo[3],
                   uint32_t hi[3])
{
    if (!crx) {
        lo[0] = g.xend;
        hi[0] = L;
        return 1;
    }
    lo[0] = 12;
    hi[0] = g.hl;
    lo[1] = g.hl + 4;
    hi[1] = g.xend;
    lo[2] = g.xend;
    hi[2] = L;
    return 3;
}

DEV bool xtn_selected(const srtp_dev_key_t *k, uint32_t id)
{
    return (k->xids[id >> 5] >> (id & 31u)) & 1u;   // srtp.c:1776-1797
}

// srtp_process_header_encryption (srtp.c:1802-1894): walk the RFC 8285
// elements of the extension at p + xo (one-byte 0xBEDE or two-byte 0x100x
// profile), consuming the extension keystream per element (header bytes
// included); with `apply` XOR the data of the selected IDs.  Padding bytes
// are skipped without keystream; a one-byte ID 15 ends the walk.  Element
// header bytes are never encrypted, so the walk is the same both ways.
// false = parse error.
DEV bool xtn_walk(const srtp_dev_key_t *k, const srtp_dev_key_t *keys,
                  uint8_t *p, uint32_t xo, uint32_t xend, uint32_t roc,
                  bool apply, const AesLds &T)
{
    const uint32_t prof = (uint32_t)p[xo] << 8 | p[xo + 1];
    const bool one = prof == 0xBEDEu;
    if (!one && (prof & 0xfff0u) != 0x1000u)
        return false;
    Kstream K;
    K.icm(keys + k->xslot, p, roc);
    uint32_t d = xo + 4;
    while (one ? d < xend : d + 1 < xend) {
        uint32_t id, len;
        const uint32_t hb = one ? 1u : 2u;
        if (one) {
            id = p[d] >> 4;
            len = (p[d] & 15u) + 1;
        } else {
            id = p[d];
            len = p[d + 1];
        }
        d += hb;
        if (d + len > xend)
            return false;
        if (one && id == 15)
            break;
        if (apply) {
            const bool sel = (one || len > 0) && xtn_selected(k, id);
            for (uint32_t u = 0; u < hb; u++)
                K.next(T);
            for (uint32_t u = 0; u < len; u++) {
                const uint8_t b = K.next(T);
                if (sel)
                    p[d + u] ^= b;
            }
        }
        d += len;
        while (d < xend && p[d] == 0)
            d++;
    }
    return true;
}

// GHASH(aad || ciphertext || lengths) ^ E_K(J0) over the packet's AAD
// ranges and encrypted ranges (which already hold ciphertext)
DEV void xrtp_gcm_tag(const srtp_dev_key_t *k, const Kstream &K,
                      const uint8_t *p, const XGeo &g, bool crx,
                      const uint32_t lo[3], const uint32_t hi[3], uint32_t ns,
                      uint8_t tag[16], const AesLds &T)
{
    Ghash G;
    G.xh = G.xl = 0;
    G.hh = (uint64_t)k->h[0] << 32 | k->h[1];
    G.hl = (uint64_t)k->h[2] << 32 | k->h[3];
    G.fill = 0;
    // AAD: the header up to enc_start; with cryptex the fixed header and
    // the extension header word (srtp.c:2234-2241, 2391-2398)
    uint32_t alen;
    if (crx) {
        for (uint32_t u = 0; u < 12; u++)
            G.put(p[u]);
        for (uint32_t u = 0; u < 4; u++)
            G.put(p[g.hl + u]);
        alen = 16;
    } else {
        for (uint32_t u = 0; u < g.xend; u++)
            G.put(p[u]);
        alen = g.xend;
    }
    G.flush();
    uint32_t clen = 0;
    for (uint32_t s = 0; s < ns; s++) {
        for (uint32_t u = lo[s]; u < hi[s]; u++)
            G.put(p[u]);
        clen += hi[s] - lo[s];
    }
    G.flush();
    G.xh ^= (uint64_t)alen * 8;
    G.xl ^= (uint64_t)clen * 8;
    gf128_mul(G.xh, G.xl, G.hh, G.hl);
    uint32_t e[4];
    K.block(1, e, T);   // E_K(J0)
    for (int u = 0; u < 16; u++) {
        const uint64_t half = u < 8 ? G.xh : G.xl;
        tag[u] = (uint8_t)(half >> (56 - 8 * (u & 7))) ^
                 (uint8_t)(e[u >> 2] >> (8 * (u & 3)));
    }
}

DEV void roc_be(uint32_t roc, uint8_t r[4])
{
    r[0] = (uint8_t)(roc >> 24);
    r[1] = (uint8_t)(roc >> 16);
    r[2] = (uint8_t)(roc >> 8);
    r[3] = (uint8_t)roc;
}

DEV uint8_t xrtp_protect(const srtp_dev_key_t *keys, const srtp_dev_meta_t &m,
                         const uint8_t *src, uint8_t *p, const AesLds &T)
{
    const srtp_dev_key_t *k = keys + m.key;
    const uint32_t L = m.len;
    if (src != p)
        for (uint32_t u = 0; u < L; u++)
            p[u] = src[u];
    const XGeo g = xgeo(p);
    const bool inplace = (m.info & SRTP_XI_INPLACE) != 0;
    const bool crx = (k->xflags & SRTP_XF_CRYPTEX) &&
                     (k->xflags & SRTP_XF_CONF) && g.x;
    if (g.x && (k->xflags & SRTP_XF_XTN)) {
        // not in place, cryptex encrypts the caller's plaintext extension
        // (srtp.c:2766-2768, 2245-2246): only the walk's verdict remains
        if (!xtn_walk(k, keys, p, g.hl, g.xend, m.roc, !(crx && !inplace), T))
            return SRTP_XR_PARSE;
    }
    if (crx) {   // srtp_cryptex_protect (srtp.c:195-208)
        const uint32_t prof = (uint32_t)p[g.hl] << 8 | p[g.hl + 1];
        if (prof == 0xBEDEu) {
            p[g.hl] = 0xC0;
            p[g.hl + 1] = 0xDE;
        } else if (prof == 0x1000u) {
            p[g.hl] = 0xC2;
            p[g.hl + 1] = 0xDE;
        } else {
            return SRTP_XR_PARSE;
        }
    }
    uint32_t lo[3], hi[3];
    const uint32_t ns = xsegs(g, crx, L, lo, hi);
    const uint32_t mki = k->mki_size, TL = k->tag_len;
    Kstream K;
    if (k->family == SRTP_DEV_GCM) {
        K.aead(k, p, m.roc);
        for (uint32_t s = 0; s < ns; s++)
            for (uint32_t u = lo[s]; u < hi[s]; u++)
                p[u] ^= K.next(T);
        uint8_t tag[16];
        xrtp_gcm_tag(k, K, p, g, crx, lo, hi, ns, tag, T);
        for (uint32_t u = 0; u < TL; u++)
            p[L + u] = tag[u];
        for (uint32_t u = 0; u < mki; u++)
            p[L + TL + u] = k->mki[u];
    } else {
        if (k->conf && k->family == SRTP_DEV_ICM) {
            K.icm(k, p, m.roc);
            for (uint32_t s = 0; s < ns; s++)
                for (uint32_t u = lo[s]; u < hi[s]; u++)
                    p[u] ^= K.next(T);
        }
        for (uint32_t u = 0; u < mki; u++)
            p[L + u] = k->mki[u];
        if (k->auth) {   // HMAC over the packet, then the ROC (srtp.c:2785-2815)
            uint8_t r[4];
            roc_be(m.roc, r);
            uint32_t oh[5];
            hmac_sha1_bytes(k, p, L, oh, r, 4);
            for (uint32_t u = 0; u < TL; u++)
                p[L + mki + u] = (uint8_t)(oh[u >> 2] >> (24 - 8 * (u & 3)));
        }
    }
    return SRTP_XR_OK | SRTP_XR_WROTE | (crx ? SRTP_XR_CRYPTEX : 0);
}

// unprotect: verify on the input, then write the output.  `undo` re-applies
// a run's transform to its output (XOR is its own inverse; the profile goes
// back to the cryptex one) so a speculative run at a wrong index can be
// taken back (k_undo_wave).
DEV uint8_t xrtp_unprotect(const srtp_dev_key_t *keys, const srtp_dev_meta_t &m,
                           const uint8_t *src, uint8_t *p, bool undo,
                           const AesLds &T)
{
    const srtp_dev_key_t *k = keys + m.key;
    const uint32_t L = m.len;
    const XGeo g = xgeo(src);
    const bool inplace = (m.info & SRTP_XI_INPLACE) != 0;
    const uint32_t prof = g.x ? ((uint32_t)src[g.hl] << 8 | src[g.hl + 1]) : 0;
    // srtp_cryptex_unprotect_init (srtp.c:237-265): by the profile on the
    // wire
    const bool crx = undo ? (m.info & SRTP_XI_CRYPTEX) != 0
                          : (k->xflags & SRTP_XF_CRYPTEX) && g.x &&
                                (prof == 0xC0DEu || prof == 0xC2DEu);
    const bool gcm = k->family == SRTP_DEV_GCM;
    uint32_t lo[3], hi[3];
    const uint32_t ns = xsegs(g, crx, L, lo, hi);
    Kstream K;
    if (gcm)
        K.aead(k, src, m.roc);
    else
        K.icm(k, src, m.roc);
    if (!undo) {
        const uint32_t mki = k->mki_size, TL = k->tag_len;
        uint32_t diff = 0;
        if (gcm) {
            uint8_t tag[16];
            xrtp_gcm_tag(k, K, src, g, crx, lo, hi, ns, tag, T);
            for (uint32_t u = 0; u < TL; u++)
                diff |= tag[u] ^ src[L + u];
        } else if (k->auth) {
            uint8_t r[4];
            roc_be(m.roc, r);
            uint32_t oh[5];
            hmac_sha1_bytes(k, src, L, oh, r, 4);
            for (uint32_t u = 0; u < TL; u++)
                diff |= src[L + mki + u] ^
                        ((oh[u >> 2] >> (24 - 8 * (u & 3))) & 0xffu);
        }
        if (diff)
            return 0;
        // the extension walk runs on the still-cryptex profile and fails
        // (srtp.c:3073-3080, 2409-2418)
        if (g.x && (k->xflags & SRTP_XF_XTN) &&
            (crx || !xtn_walk(k, keys, const_cast<uint8_t *>(src), g.hl,
                              g.xend, m.roc, false, T)))
            return SRTP_XR_OK | SRTP_XR_PARSE;
        if (src != p)
            for (uint32_t u = 0; u < L; u++)
                p[u] = src[u];
    }
    if (g.x && (k->xflags & SRTP_XF_XTN) && !crx)
        xtn_walk(k, keys, p, g.hl, g.xend, m.roc, true, T);
    if (gcm || (k->conf && k->family == SRTP_DEV_ICM)) {
        for (uint32_t s = 0; s < ns; s++)
            for (uint32_t u = lo[s]; u < hi[s]; u++)
                p[u] ^= K.next(T);
    } else if (crx && !inplace && k->family != SRTP_DEV_NULL) {
        // not in place, srtp_cryptex_unprotect decrypts the CSRCs whether
        // or not the payload is encrypted (srtp.c:274-284)
        for (uint32_t u = lo[0]; u < hi[0]; u++)
            p[u] ^= K.next(T);
    }
    if (crx) {   // srtp_cryptex_unprotect_cleanup (srtp.c:290-305)
        const uint32_t cur = (uint32_t)p[g.hl] << 8 | p[g.hl + 1];
        if (!undo && cur == 0xC0DEu) {
            p[g.hl] = 0xBE;
            p[g.hl + 1] = 0xDE;
        } else if (!undo && cur == 0xC2DEu) {
            p[g.hl] = 0x10;
            p[g.hl + 1] = 0x00;
        } else if (undo && cur == 0xBEDEu) {
            p[g.hl] = 0xC0;
            p[g.hl + 1] = 0xDE;
        } else if (undo && cur == 0x1000u) {
            p[g.hl] = 0xC2;
            p[g.hl + 1] = 0xDE;
        }
    }
    return SRTP_XR_OK | SRTP_XR_WROTE | (crx ? SRTP_XR_CRYPTEX : 0);
}

__global__ __launch_bounds__(256) void k_xrtp(const uint8_t *in,
                                              const uint64_t *in_off,
                                              uint8_t *out,
                                              const uint64_t *out_off,
                                              const srtp_dev_meta_t *meta,
                                              const srtp_dev_key_t *keys,
                                              uint8_t *res,
                                              const uint32_t *abort,
                                              uint32_t n, int protect)
{
    __shared__ u32x4 s_tab[AES_TAB2_BYTES / 16];
    load_aes_tables<false>(s_tab);
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || (abort && *abort))
        return;
    const srtp_dev_meta_t m = meta[i];
    if (SRTP_META_STATUS(m.info) || SRTP_META_VARIANT(m.info) != SRTP_VARIANT_X)
        return;
    const AesLds T = make_aes_lds(s_tab);
    const uint8_t *src = in + in_off[i];
    uint8_t *dst = out + out_off[i];
    const uint8_t r = protect ? xrtp_protect(keys, m, src, dst, T)
                              : xrtp_unprotect(keys, m, src, dst, false, T);
    if (res)
        res[i] = r;
}

// ---------------------------------------------------------------------------
// Session-key derivation for many keys at once (srtp_gpu_kdf): one lane per
// session key.  The SRTP KDF (srtp.c:1070-1142) is AES-ICM keyed by the
// master key with the master salt as offset and the label in byte 7;
// srtp_stream_init_keys (srtp.c:1233-1607) draws the cipher key, salt and
// HMAC key from it, and the cipher / auth init turn them into the AES
// schedule (aes.c key expansion, FIPS-197 5.2), the HMAC ipad / opad SHA-1
// midstates (hmac.c:76-120) and, for AES-GCM, H = E_K(0) and the GHASH
// table.  The host decides every policy question (labels, lengths, which
// records) and the GPU does the arithmetic: a mass (re)key of 64k streams
// is one launch instead of 64k host derivations and uploads.

DEV uint32_t kdf_subword(uint32_t t, const uint32_t *sb)
{
    return sb[t & 0xffu] | sb[(t >> 8) & 0xffu] << 8 |
           sb[(t >> 16) & 0xffu] << 16 | sb[t >> 24] << 24;
}

template <int NR>
struct ArrKey {
    uint32_t rk[4 * (NR + 1)];
    DEV uint32_t operator()(int i) const { return rk[i]; }
};

// AES key expansion: little-endian words of the key bytes (the layout of
// srtp_dev_key_t.rk), RotWord / SubWord / Rcon on those
template <int NR>
DEV void kdf_expand(const uint8_t *key, ArrKey<NR> &K, const uint32_t *sb)
{
    constexpr int NK = NR - 6, NW = 4 * (NR + 1);
#pragma unroll
    for (int i = 0; i < NK; i++)
        K.rk[i] = (uint32_t)key[4 * i] | (uint32_t)key[4 * i + 1] << 8 |
                  (uint32_t)key[4 * i + 2] << 16 | (uint32_t)key[4 * i + 3] << 24;
    uint32_t rc = 1;
#pragma unroll
    for (int i = NK; i < NW; i++) {
        uint32_t t = K.rk[i - 1];
        if (i % NK == 0) {
            t = kdf_subword((t >> 8) | (t << 24), sb) ^ rc;
            rc = ((rc << 1) ^ ((rc >> 7) * 0x1bu)) & 0xffu;
        } else if (NK > 6 && i % NK == 4) {
            t = kdf_subword(t, sb);
        }
        K.rk[i] = K.rk[i - NK] ^ t;
    }
}

// `len` bytes of PRF output for `label` (srtp.c:1104-1142): counter block =
// offset ^ (label at byte 7), 16-bit block counter in bytes 14..15
template <int NR>
DEV void kdf_prf(const ArrKey<NR> &K, const uint8_t *salt, uint32_t label,
                 uint8_t *out, uint32_t len, const AesLds &T)
{
    for (uint32_t j = 0; 16 * j < len; j++) {
        uint8_t c[16];
        for (int u = 0; u < 14; u++)
            c[u] = salt[u];
        c[7] ^= (uint8_t)label;
        c[14] = (uint8_t)(j >> 8);
        c[15] = (uint8_t)j;
        uint32_t x[4];
        for (int w = 0; w < 4; w++)
            x[w] = (uint32_t)c[4 * w] | (uint32_t)c[4 * w + 1] << 8 |
                   (uint32_t)c[4 * w + 2] << 16 | (uint32_t)c[4 * w + 3] << 24;
        aes_block<NR, false>(x[0], x[1], x[2], x[3], K, T);
        for (uint32_t b = 0; b < 16 && 16 * j + b < len; b++)
            out[16 * j + b] = (uint8_t)(x[b >> 2] >> (8 * (b & 3)));
    }
}

// Shoup's table M[b] = b * H of the big-endian H words v (clobbered): powers
// by halving (v * x = v >> 1, ^ 0xe1 on carry), then sums
// (host_crypto.c hc_ghash_table), stored in the arena's layout: M[b] at
// entry ghash_nswap(b) (srtp_dev_common.h)
DEV void ghash_shoup(uint32_t v[4], uint32_t *tab)
{
    for (int w = 0; w < 4; w++)
        tab[w] = 0;
    for (uint32_t bit = 0x80; bit; bit >>= 1) {
        for (int w = 0; w < 4; w++)
            tab[4 * ghash_nswap(bit) + w] = v[w];
        const uint32_t lsb = v[3] & 1u;
        v[3] = (v[3] >> 1) | (v[2] << 31);
        v[2] = (v[2] >> 1) | (v[1] << 31);
        v[1] = (v[1] >> 1) | (v[0] << 31);
        v[0] = (v[0] >> 1) ^ ((0u - lsb) & 0xe1000000u);
    }
    for (uint32_t b = 1; b < 256; b++) {
        const uint32_t low = b & (0u - b);
        if (b == low)
            continue;
        for (int w = 0; w < 4; w++)
            tab[4 * ghash_nswap(b) + w] = tab[4 * ghash_nswap(low) + w] ^
                                          tab[4 * ghash_nswap(b ^ low) + w];
    }
}

// the cipher half of the record: schedule of the derived key, H, GHASH
template <int NR>
DEV void kdf_cipher(const srtp_kdf_job_t &J, const uint8_t *ek,
                    srtp_dev_key_t *o, uint32_t *ghash, const uint32_t *sb,
                    const AesLds &T)
{
    ArrKey<NR> K;
    kdf_expand<NR>(ek, K, sb);
#pragma unroll
    for (int i = 0; i < 4 * (NR + 1); i++)
        o->rk[i] = K.rk[i];
    if (!(J.flags & (SRTP_KDF_GCM_H | SRTP_KDF_GHASH)))
        return;
    uint32_t x[4] = { 0, 0, 0, 0 };
    aes_block<NR, false>(x[0], x[1], x[2], x[3], K, T);
    uint32_t v[4];   // H as big-endian words
    for (int w = 0; w < 4; w++) {
        v[w] = bswap(x[w]);
        o->h[w] = v[w];
    }
    if (!(J.flags & SRTP_KDF_GHASH))
        return;
    ghash_shoup(v, ghash + 1024 * (size_t)J.key.ghash_slot);
}

template <int NRK>
DEV void kdf_one(const srtp_kdf_job_t &J, srtp_dev_key_t *keys,
                 uint32_t *ghash, const uint32_t *sb, const AesLds &T)
{
    ArrKey<NRK> P;
    kdf_expand<NRK>(J.kdf_key, P, sb);
    uint8_t ek[32], sa[16], ak[20];
    for (int u = 0; u < 16; u++)
        sa[u] = 0;
    kdf_prf<NRK>(P, J.kdf_salt, J.lab_enc, ek, J.enc_len, T);
    kdf_prf<NRK>(P, J.kdf_salt, J.lab_salt, sa, J.salt_len, T);
    kdf_prf<NRK>(P, J.kdf_salt, J.lab_auth, ak, J.auth_len, T);
    if (J.flags & SRTP_KDF_SALT_TAIL) {
        sa[J.salt_len] = J.salt_tail[0];
        sa[J.salt_len + 1] = J.salt_tail[1];
    }
    srtp_dev_key_t *o = keys + J.slot;
    // the host's fields, then the derived ones
    const uint32_t *src = (const uint32_t *)&J.key;
    uint32_t *dst = (uint32_t *)o;
    for (uint32_t w = 0; w < sizeof(srtp_dev_key_t) / 4; w++)
        dst[w] = src[w];
    for (int w = 0; w < 4; w++)
        o->salt[w] = (uint32_t)sa[4 * w] | (uint32_t)sa[4 * w + 1] << 8 |
                     (uint32_t)sa[4 * w + 2] << 16 | (uint32_t)sa[4 * w + 3] << 24;
    if (J.enc_len == 16)
        kdf_cipher<10>(J, ek, o, ghash, sb, T);
    else if (J.enc_len == 24)
        kdf_cipher<12>(J, ek, o, ghash, sb, T);
    else if (J.enc_len == 32)
        kdf_cipher<14>(J, ek, o, ghash, sb, T);
    if (J.flags & SRTP_KDF_HMAC) {
        // SHA-1 midstates of (K ^ ipad) and (K ^ opad), K zero padded
        for (int pass = 0; pass < 2; pass++) {
            const uint32_t pad = pass ? 0x5c5c5c5cu : 0x36363636u;
            uint32_t w[16];
            for (int t = 0; t < 16; t++) {
                uint32_t v = 0;
                for (int u = 0; u < 4; u++) {
                    const uint32_t b = 4 * t + u;
                    v = (v << 8) | (b < J.auth_len ? ak[b] : 0u);
                }
                w[t] = v ^ pad;
            }
            uint32_t h[5] = { 0x67452301u, 0xefcdab89u, 0x98badcfeu,
                              0x10325476u, 0xc3d2e1f0u };
            sha1_compress(h, w);   // adds the chaining value itself
            for (int k = 0; k < 5; k++) {
                if (pass)
                    o->opad[k] = h[k];
                else
                    o->ipad[k] = h[k];
            }
        }
    }
}

// GHASH tables of imported key records (srtp_gpu_put_keys): one lane per
// slot whose flag is set, from the record's H
__global__ __launch_bounds__(256) void k_ghash_build(const srtp_dev_key_t *keys,
                                                     const uint8_t *flag,
                                                     uint32_t n, uint32_t *ghash)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !flag[i])
        return;
    uint32_t v[4] = { keys[i].h[0], keys[i].h[1], keys[i].h[2], keys[i].h[3] };
    ghash_shoup(v, ghash + 1024 * (size_t)keys[i].ghash_slot);
}

__global__ __launch_bounds__(256) void k_kdf(const srtp_kdf_job_t *jobs,
                                             uint32_t n, srtp_dev_key_t *keys,
                                             uint32_t *ghash)
{
    __shared__ u32x4 s_tab[AES_TAB2_BYTES / 16];
    __shared__ uint32_t s_sb[256];
    for (int x = threadIdx.x; x < 256; x += blockDim.x)
        s_sb[x] = (aes_t0((uint32_t)x) >> 8) & 0xffu;   // S[x]
    load_aes_tables<false>(s_tab);
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const AesLds T = make_aes_lds(s_tab);
    const srtp_kdf_job_t &J = jobs[i];
    if (J.kdf_len == 16)
        kdf_one<10>(J, keys, ghash, s_sb, T);
    else if (J.kdf_len == 24)
        kdf_one<12>(J, keys, ghash, s_sb, T);
    else
        kdf_one<14>(J, keys, ghash, s_sb, T);
}

}   // namespace

// ===========================================================================
// thin C-ABI FFI (srtp_dev.h)

static thread_local char g_err[256];

int srtp_gpu_fail(hipError_t e, const char *what)
{
    snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
    return -1;
}

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
    A.rec = b->rec;
    A.rec_idx = b->rec_idx;
    A.range = b->rec_range;
    A.fused = b->fused != nullptr;
    if (A.fused)
        A.fz = *(const IcmFused *)b->fused;
    A.ch = IcmChain{};
    if (b->inorder)
        A.ch = *(const IcmChain *)b->inorder;
    static const bool stg = [] {
        const char *e = getenv("SRTP_ICM_STG");
        return !(e && e[0] == '0');
    }();
    A.stg = stg;
    if (A.rec) {
        // key buckets: the wave-aligned groups with a key per wave, then
        // the streams with few packets with a key per lane
        IcmArgs Ln = A;
        Ln.range = A.range + 2;
        return launch_icm_km<NR, KM_WAVE>(A, AUTH, PROT, g->ncu, st) |
               launch_icm_km<NR, KM_LANE>(Ln, AUTH, PROT, g->ncu, st);
    }
    if (A.uni != 0xffffffffu)
        return launch_icm_km<NR, KM_UNI>(A, AUTH, PROT, g->ncu, st);
    return launch_icm_km<NR, KM_LANE>(A, AUTH, PROT, g->ncu, st);
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
    A.rec = b->rec;
    A.rec_idx = b->rec_idx;
    A.range = b->rec_range;
    A.fused = b->fused != nullptr;
    if (A.fused)
        A.fz = *(const IcmFused *)b->fused;
    A.ch = IcmChain{};
    if (b->inorder)
        A.ch = *(const IcmChain *)b->inorder;
    return launch_gcm_nr<NR>(A, PROT, g->ncu, st);
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
    if (m & (1u << SRTP_VARIANT_X)) {
        // header-extension encryption / cryptex streams (k_xrtp)
        const uint32_t n = (uint32_t)b->n;
        hipLaunchKernelGGL(k_xrtp, dim3((n + 255) / 256), dim3(256), 0, st,
                           b->in, b->in_off, b->out, b->out_off, b->meta,
                           (const srtp_dev_key_t *)g->d_keys, b->auth_ok,
                           b->abort, n, PROT ? 1 : 0);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess)
            rc |= srtp_gpu_fail(e, "k_xrtp launch");
    }
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
    (void)hipFree(g->d_raw);
    (void)hipFree(g->d_undo);
    if (g->one_h)
        (void)hipHostFree(g->one_h);
    for (int k = 0; k < SRTP_GPU_MARKS; k++)
        if (g->marks[k])
            (void)hipEventDestroy(g->marks[k]);
    for (int k = 0; k < 2; k++)
        if (g->aux[k])
            (void)hipStreamDestroy(g->aux[k]);
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
    uint32_t dev_tab[1024];   // the arena's layout: M[b] at ghash_nswap(b)
    if (ghash_tab) {
        if (grow((void **)&g->d_ghash, &g->ghash_cap, k->ghash_slot + 1,
                 1024 * sizeof(uint32_t)))
            return -1;
        for (uint32_t b = 0; b < 256; b++)
            memcpy(dev_tab + 4 * ghash_nswap(b), ghash_tab + 4 * b, 16);
        HIPCHK(hipMemcpyAsync(g->d_ghash + 1024 * (size_t)k->ghash_slot,
                              dev_tab, 4096, hipMemcpyHostToDevice,
                              g->stream));
    }
    HIPCHK(hipStreamSynchronize(g->stream));
    return 0;
}

int srtp_gpu_get_keys(srtp_gpu_t *g, uint32_t n, srtp_dev_key_t *dst)
{
    if (!n)
        return 0;
    if (n > g->key_cap) {
        snprintf(g_err, sizeof g_err, "srtp_gpu_get_keys: %u slots of %u",
                 n, g->key_cap);
        return -1;
    }
    HIPCHK(hipMemcpyAsync(dst, g->d_keys, (size_t)n * sizeof *dst,
                          hipMemcpyDeviceToHost, g->stream));
    HIPCHK(hipStreamSynchronize(g->stream));
    return 0;
}

int srtp_gpu_put_keys(srtp_gpu_t *g, uint32_t n, const srtp_dev_key_t *src,
                      const uint8_t *ghash_flag)
{
    if (!n)
        return 0;
    if (grow((void **)&g->d_keys, &g->key_cap, n, sizeof(srtp_dev_key_t)))
        return -1;
    HIPCHK(hipMemcpyAsync(g->d_keys, src, (size_t)n * sizeof *src,
                          hipMemcpyHostToDevice, g->stream));
    uint32_t gmax = 0;
    for (uint32_t i = 0; i < n; i++)
        if (ghash_flag[i] && src[i].ghash_slot + 1 > gmax)
            gmax = src[i].ghash_slot + 1;
    if (gmax) {
        if (grow((void **)&g->d_ghash, &g->ghash_cap, gmax,
                 1024 * sizeof(uint32_t)))
            return -1;
        uint8_t *d = NULL;
        HIPCHK(hipMalloc((void **)&d, n));
        hipError_t e = hipMemcpyAsync(d, ghash_flag, n, hipMemcpyHostToDevice,
                                      g->stream);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_ghash_build, dim3((n + 255) / 256), dim3(256),
                               0, g->stream, g->d_keys, d, n,
                               (uint32_t *)g->d_ghash);
            e = hipGetLastError();
        }
        if (e == hipSuccess)
            e = hipStreamSynchronize(g->stream);
        (void)hipFree(d);
        if (e != hipSuccess)
            return srtp_gpu_fail(e, "k_ghash_build");
        return 0;
    }
    HIPCHK(hipStreamSynchronize(g->stream));
    return 0;
}

int srtp_gpu_kdf(srtp_gpu_t *g, const srtp_kdf_job_t *jobs, size_t n)
{
    if (!n)
        return 0;
    uint32_t kmax = 0, gmax = 0;
    int any_gh = 0;
    for (size_t i = 0; i < n; i++) {
        if (jobs[i].slot + 1 > kmax)
            kmax = jobs[i].slot + 1;
        if (jobs[i].flags & SRTP_KDF_GHASH) {
            any_gh = 1;
            if (jobs[i].key.ghash_slot + 1 > gmax)
                gmax = jobs[i].key.ghash_slot + 1;
        }
    }
    if (grow((void **)&g->d_keys, &g->key_cap, kmax, sizeof(srtp_dev_key_t)))
        return -1;
    if (any_gh && grow((void **)&g->d_ghash, &g->ghash_cap, gmax,
                       1024 * sizeof(uint32_t)))
        return -1;
    srtp_kdf_job_t *d = NULL;
    HIPCHK(hipMalloc((void **)&d, n * sizeof *d));
    hipError_t e = hipMemcpyAsync(d, jobs, n * sizeof *d,
                                  hipMemcpyHostToDevice, g->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_kdf, dim3((unsigned)((n + 255) / 256)), dim3(256),
                           0, g->stream, d, (uint32_t)n, g->d_keys,
                           (uint32_t *)g->d_ghash);
        e = hipGetLastError();
    }
    if (e == hipSuccess)
        e = hipStreamSynchronize(g->stream);
    (void)hipFree(d);
    if (e != hipSuccess)
        return srtp_gpu_fail(e, "k_kdf");
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
    // the elapsed time is read when asked for (srtp_gpu_last_kernel_ms,
    // after the batch): waiting for ev1 here would hold back the launches
    // that follow the crypto kernel by a host round trip
    if (g->timing) {
        HIPCHK(hipEventRecord(g->ev1, st));
        g->ms_pending = 1;
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
    if (n > g->undo_cap) {
        // in-flight work may still read the old list: hipFree waits for it
        (void)hipFree(g->d_undo);
        g->d_undo = nullptr;
        g->undo_cap = 0;
        HIPCHK(hipMalloc((void **)&g->d_undo, (n + 1) * 4));
        g->undo_cap = n;
    }
    uint32_t *count = g->d_undo + n;
    HIPCHK(hipMemsetAsync(count, 0, 4, st));
    hipLaunchKernelGGL(k_undo_list, dim3((unsigned)((n + 255) / 256)),
                       dim3(256), 0, st, meta, (uint32_t)n, g->d_undo, count);
    size_t blocks = 2 * (size_t)g->ncu, need = (n + 3) / 4;
    blocks = blocks < need ? blocks : need;
    hipLaunchKernelGGL(k_undo_wave, dim3((unsigned)blocks), dim3(256), 0, st,
                       arena, off, meta, g->d_keys, g->d_undo, count);
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
                   srtp_dev_hdr_t *hdr_out, uint32_t *xinfo_out, void *stream)
{
    if (!n)
        return 0;
    hipStream_t st = (hipStream_t)stream;   // NULL = the null stream
    hipLaunchKernelGGL(k_parse, dim3((unsigned)((n + 255) / 256)), dim3(256),
                       0, st, in, in_off, in_len, hdr_out, xinfo_out,
                       (uint32_t)n);
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

int srtp_gpu_memset(void *dst, int v, size_t n, void *stream)
{
    if (!n)
        return 0;
    HIPCHK(hipMemsetAsync(dst, v, n, (hipStream_t)stream));
    return 0;
}

int srtp_gpu_sync(srtp_gpu_t *g, void *stream)
{
    hipStream_t st = (hipStream_t)stream;   // NULL = the null stream
    HIPCHK(hipStreamSynchronize(st));
    return 0;
}

// events of the host-batch staging pipeline (srtp_host.c
// batch_device_fast): slot k marks "chunk k's copy is done" on a stream
int srtp_gpu_mark(srtp_gpu_t *g, int slot, void *stream)
{
    if (slot < 0 || slot >= SRTP_GPU_MARKS)
        return srtp_gpu_fail(hipErrorInvalidValue, "mark slot");
    if (!g->marks[slot])
        HIPCHK(hipEventCreateWithFlags(&g->marks[slot], hipEventDisableTiming));
    HIPCHK(hipEventRecord(g->marks[slot], (hipStream_t)stream));
    return 0;
}

int srtp_gpu_mark_stream_wait(srtp_gpu_t *g, void *stream, int slot)
{
    if (slot < 0 || slot >= SRTP_GPU_MARKS || !g->marks[slot])
        return srtp_gpu_fail(hipErrorInvalidValue, "mark slot");
    HIPCHK(hipStreamWaitEvent((hipStream_t)stream, g->marks[slot], 0));
    return 0;
}

void *srtp_gpu_aux_stream(srtp_gpu_t *g, int k)
{
    if (k < 0 || k >= 2)
        return nullptr;
    if (!g->aux[k] &&
        hipStreamCreateWithFlags(&g->aux[k], hipStreamNonBlocking) != hipSuccess) {
        g->aux[k] = nullptr;
        return nullptr;
    }
    return g->aux[k];
}

int srtp_gpu_mark_wait(srtp_gpu_t *g, int slot)
{
    if (slot < 0 || slot >= SRTP_GPU_MARKS || !g->marks[slot])
        return srtp_gpu_fail(hipErrorInvalidValue, "mark slot");
    HIPCHK(hipEventSynchronize(g->marks[slot]));
    return 0;
}

double srtp_gpu_last_kernel_ms(srtp_gpu_t *g)
{
    if (g->ms_pending) {
        g->ms_pending = 0;
        if (hipEventSynchronize(g->ev1) != hipSuccess ||
            hipEventElapsedTime(&g->last_ms, g->ev0, g->ev1) != hipSuccess)
            g->last_ms = 0;
    }
    return g->last_ms;
}
void srtp_gpu_set_timing(srtp_gpu_t *g, int on) { g->timing = on; }


int srtp_gpu_raw(srtp_gpu_t *g, srtp_gpu_raw_t *r)
{
    // scratch layout: key | src (+ tag) | dst (+ tag) | aad | results
    const size_t ksz = (sizeof(srtp_dev_key_t) + 255) & ~(size_t)255;
    const size_t dsz = (r->len + 16 + 255) & ~(size_t)255;
    const size_t asz = (r->aad_len + 255) & ~(size_t)255;
    const size_t need = ksz + 2 * dsz + asz + 256;
    if (r->len > 0xffffff00u || r->aad_len > 0xffffff00u)
        return srtp_gpu_fail(hipErrorInvalidValue, "raw: buffer too large");
    if (need > g->raw_cap) {
        (void)hipFree(g->d_raw);
        g->d_raw = nullptr;
        g->raw_cap = 0;
        HIPCHK(hipMalloc((void **)&g->d_raw, need));
        g->raw_cap = need;
    }
    uint8_t *dk = g->d_raw, *ds = dk + ksz, *dd = ds + dsz, *da = dd + dsz,
            *dr = da + asz;
    hipStream_t st = g->stream;
    HIPCHK(hipMemcpyAsync(dk, r->key, sizeof(srtp_dev_key_t),
                          hipMemcpyHostToDevice, st));
    const size_t in_len =
        r->len + (r->op == SRTP_RAW_GCM_OPEN ? r->tag_len : 0);
    if (in_len)
        HIPCHK(hipMemcpyAsync(ds, r->src, in_len, hipMemcpyHostToDevice, st));
    if (r->aad_len)
        HIPCHK(hipMemcpyAsync(da, r->aad, r->aad_len, hipMemcpyHostToDevice,
                              st));
    HIPCHK(hipMemsetAsync(dr, 0, 32, st));
    RawDev A = {};
    A.op = r->op;
    A.key = (const srtp_dev_key_t *)dk;
    A.src = ds;
    A.dst = dd;
    A.len = (uint32_t)r->len;
    A.nlead = r->nlead;
    A.aad_len = (uint32_t)r->aad_len;
    A.tag_len = r->tag_len;
    memcpy(A.ctr, r->ctr, 16);
    memcpy(A.lead, r->lead, 16);
    memcpy(A.iv, r->iv, 12);
    A.aad = da;
    A.res = dr;
    hipLaunchKernelGGL(k_raw, dim3(1), dim3(256), 0, st, A);
    HIPCHK(hipGetLastError());
    const size_t out_len =
        r->op == SRTP_RAW_HMAC
            ? 20
            : r->len + (r->op == SRTP_RAW_GCM_SEAL ? r->tag_len : 0);
    if (out_len)
        HIPCHK(hipMemcpyAsync(r->dst, dd, out_len, hipMemcpyDeviceToHost, st));
    uint8_t res[32];
    HIPCHK(hipMemcpyAsync(res, dr, 32, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    memcpy(r->ks_last, res, 16);
    r->ok = res[16];
    return 0;
}

}   // extern "C"
