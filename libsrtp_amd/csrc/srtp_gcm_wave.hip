// srtp_gcm_wave.hip -- k_gcm_wave: AES-GCM seal / open for uniform-key
// batches on the lane-quad cooperative memory path (BASELINE configs[2]).
//
// Reference semantics: srtp_protect_aead / srtp_unprotect_aead
// (srtp/srtp.c:2088-2267, 2276-2491) through libsrtp's OpenSSL EVP backend
// (crypto/cipher/aes_gcm_ossl.c:214-389): IV = (00 00 || SSRC || ROC || SEQ)
// ^ salt12 (srtp.c:1925-1959), AAD = the RTP header, CTR from inc32(J0),
// GHASH over AAD || ciphertext || lengths, tag = E(J0) ^ GHASH, 8 or 16
// bytes after the ciphertext.
//
// k_gcm (srtp_gcm.hip) runs one lane per packet and moves payload-relative
// 16-byte pieces: its stores straddle cache lines and its loads touch 64
// packets per instruction, and that memory path alone took 1.66 of its
// 2.44 ms per 2^20 x 1400 B launch (AES and GHASH switched off).  Here a wave
// takes a GROUP of 64 consecutive packets of one shape (length, header size,
// 16-byte aligned, payload inside the first counter epoch) and walks them in
// packet-relative 64-byte chunks with the memory path of the ICM kernel:
// lane quads load 64 contiguous bytes of one packet, stores are whole
// 64-byte aligned segments (lane-quad transposes + funnel, srtp_dev_common.h).
// The keystream is shifted into the packet's word grid (header words mod 4)
// and GHASH consumes the ciphertext blocks one quad behind, across that
// shift.  Groups that do not qualify are flagged for k_gcm, which runs next.
#include "srtp_dev_common.h"
#include "srtp_gpu_int.h"

#ifndef GCMW_THREADS
#define GCMW_THREADS 512   // 8 waves per CU (tables take 128 KiB of LDS)
#endif

namespace {

typedef const uint8_t __attribute__((address_space(1))) *gbyte_cptr;
typedef uint8_t __attribute__((address_space(1))) *gbyte_ptr;

DEV u32x4 gload16(const uint8_t *base, uint32_t off)
{
    return *(const u32x4 __attribute__((address_space(1))) *)(
        (gbyte_cptr)base + off);
}

DEV void gstore16(uint8_t *base, uint32_t off, u32x4 v)
{
    *(u32x4 __attribute__((address_space(1))) *)((gbyte_ptr)base + off) = v;
}

// readfirstlane of an unsigned word (the builtin returns int: widening its
// result directly would sign-extend)
DEV uint32_t rfl(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}

// coop offsets: for j = 0..3 packet (L & ~3) + j's value, + 16 * (L & 3).
// DPP reads another lane's register: call it where every lane of the quad
// is active (uniform control flow), never under a per-lane predicate.
DEV void coop_offs(uint32_t own, uint32_t (&o)[4])
{
    const uint32_t lq16 = 16 * (threadIdx.x & 3);
    o[0] = qperm<0x00>(own) + lq16;
    o[1] = qperm<0x55>(own) + lq16;
    o[2] = qperm<0xAA>(own) + lq16;
    o[3] = qperm<0xFF>(own) + lq16;
}

struct GcmWaveArgs {
    GcmArgs A;
    uint8_t *rest;   // per group: 1 = left to k_gcm
    uint32_t *any;   // set to seq when some group was left
    uint32_t seq;
};

// per-lane constants of one packet in the chunk loop
struct GwPkt {
    uint32_t di;     // input offset from ibase
    uint32_t dob;    // output segment 0 offset from obase
    uint32_t r0;     // (out >> 4) & 3
    uint32_t r0s;    // r0 of packet (L & ~3) + j at bits 2j+1:2j
};

// the group's uniform shape
struct GwShape {
    uint32_t L;      // bytes of header + payload
    uint32_t hw;     // header words
    uint32_t nblk;   // ciphertext blocks
    uint32_t nb;     // 64-byte chunks covering [0, L)
};

// x <- (x ^ block) * H, block = 4 little-endian words of the byte stream
DEV void gh_absorb(uint32_t (&x)[4], uint32_t w0, uint32_t w1, uint32_t w2,
                   uint32_t w3, const GhTab<true> &G)
{
    x[0] ^= bswap(w0);
    x[1] ^= bswap(w1);
    x[2] ^= bswap(w2);
    x[3] ^= bswap(w3);
    ghash_mul(x, G);
}

// packet word 4q+u of the GHASH byte stream: zero past L (the last word
// keeps its L & 3 bytes)
DEV uint32_t gh_mask(uint32_t w, uint32_t wi, uint32_t L)
{
    const uint32_t lo = 4 * wi;
    if (lo + 4 <= L)
        return w;
    if (lo >= L)
        return 0;
    return w & (0xffffffffu >> (8 * (4 - (L & 3))));
}

// keystream of chunk b: counter blocks j = 4b + t - qoff (counter j + 2,
// cached epoch); blocks before the payload are zero
template <int NR>
DEV void gw_keystream(uint32_t b, uint32_t qoff, const CtrCache &C,
                      const UniKey<NR> &rk, const AesLds &T,
                      uint32_t (&ks)[4][4])
{
    const int j0 = (int)(4 * b) - (int)qoff;
    if (j0 + 3 < 0) {
#pragma unroll
        for (int t = 0; t < 4; t++)
            ks[t][0] = ks[t][1] = ks[t][2] = ks[t][3] = 0;
        return;
    }
#pragma unroll
    for (int g = 0; g < 4; g += 2) {
        const uint32_t jb[2] = { ((uint32_t)(j0 + g + 2) & 0xffu) << 8,
                                 ((uint32_t)(j0 + g + 3) & 0xffu) << 8 };
        aes_ctr<2, NR, false>(*reinterpret_cast<uint32_t(*)[2][4]>(&ks[g]), jb,
                              C, rk, T);
    }
    if (j0 < 0) {
#pragma unroll
        for (int t = 0; t < 3; t++)
            if (j0 + t < 0)
                ks[t][0] = ks[t][1] = ks[t][2] = ks[t][3] = 0;
    }
}

// The chunk loop (S = header words mod 4, compile-time).  Per quad Q of the
// packet, in order: AAD block Q (Q < qoff, or the last, masked one at Q ==
// qoff), then the ciphertext block that ENDS in quad Q (S > 0: the block
// starting at word 4(Q-1)+S; S = 0: quad Q itself).
template <int S, int NR, bool PROTECT>
DEV void gw_chunks(const GwPkt &p, const GwShape &sh, const uint8_t *ibase,
                   uint8_t *obase, const CtrCache &C, const UniKey<NR> &rk,
                   const AesLds &T, const GhTab<true> &G, uint32_t (&x)[4],
                   uint32_t &tailw)
{
    const uint32_t L = sh.L, qoff = sh.hw >> 2;
    const uint32_t nq = (L + 15) >> 4;   // quads holding data
    const uint32_t nfq = L >> 4;         // full data quads (stored in loop)
    const uint32_t lq = threadIdx.x & 3;
    const uint32_t d = L & 15;
    uint32_t ks_prev[4] = { 0, 0, 0, 0 };
    uint32_t cprev[4] = { 0, 0, 0, 0 };   // GHASH words of the previous quad
    u32x4 prev[4];
#pragma unroll
    for (int t = 0; t < 4; t++)
        prev[t] = u32x4{ 0, 0, 0, 0 };
    u32x4 nx[4];
    {
        uint32_t io[4];
        coop_offs(p.di, io);
#pragma unroll
        for (int j = 0; j < 4; j++)
            nx[j] = gload16(ibase, lq < nq ? io[j] : io[j] - 16 * lq);
    }
    for (uint32_t b = 0; b < sh.nb; b++) {
        uint32_t di = p.di, dob = p.dob;
        asm volatile("" : "+v"(di), "+v"(dob));
        uint32_t ks[4][4];
        gw_keystream<NR>(b, qoff, C, rk, T, ks);
        u32x4 v[4];
#pragma unroll
        for (int j = 0; j < 4; j++)
            v[j] = nx[j];
        if (b + 1 < sh.nb) {
            // quads past the data read the packet's first quad instead
            uint32_t io[4];
            coop_offs(di, io);
            const uint32_t sk = 4 * (b + 1) + lq < nq ? 64 * (b + 1) : 0u;
#pragma unroll
            for (int j = 0; j < 4; j++)
                nx[j] = gload16(ibase, io[j] + sk);
        }
        quad_transpose(v);
        u32x4 o[4];
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t k = u >= S ? ks[t][u - S]
                                          : (t ? ks[t - 1][u - S + 4]
                                               : ks_prev[u - S + 4]);
                o[t][u] = v[t][u] ^ k;
            }
#pragma unroll
        for (int u = 0; u < 4; u++)
            ks_prev[u] = ks[3][u];
        // the partial last quad: whole words now, the last partial word
        // with the tag
        if (b == (nfq >> 2) && d) {
            const uint32_t tt = nfq & 3;
            uint32_t pq[4];
#pragma unroll
            for (int u = 0; u < 4; u++)
                pq[u] = tt == 0   ? o[0][u]
                        : tt == 1 ? o[1][u]
                        : tt == 2 ? o[2][u]
                                  : o[3][u];
            uint8_t *dst = obase + dob + 16 * (nfq + p.r0);
#pragma unroll
            for (int u = 0; u < 3; u++)
                if ((uint32_t)(4 * u + 4) <= d)
                    *(uint32_t *)(dst + 4 * u) = pq[u];
            tailw = (d >> 2) == 0   ? pq[0]
                    : (d >> 2) == 1 ? pq[1]
                    : (d >> 2) == 2 ? pq[2]
                                    : pq[3];
        }
        // aligned segment b = quads [4b - r0, 4b + 4 - r0) of the packet
        u32x4 sg[4];
        seg_funnel(prev, o, p.r0, sg);
        quad_transpose(sg);
        uint32_t so[4];
        coop_offs(dob, so);
        const bool all = 4 * b >= 3 && 4 * b + 4 <= nfq;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int q = (int)(4 * b + lq) - (int)((p.r0s >> (2 * j)) & 3u);
            if (all || (q >= 0 && q < (int)nfq))
                gstore16(obase, so[j] + 64 * b, sg[j]);
        }
        // GHASH over AAD || ciphertext, one quad behind across the shift S
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const uint32_t Q = 4 * b + t;
            uint32_t c[4];
#pragma unroll
            for (int u = 0; u < 4; u++)
                c[u] = gh_mask(PROTECT ? o[t][u] : v[t][u], 4 * Q + u, L);
            if (Q < qoff) {
                gh_absorb(x, c[0], c[1], c[2], c[3], G);   // AAD block
            } else if (Q == qoff && S) {
                gh_absorb(x, c[0], S > 1 ? c[1] : 0u, S > 2 ? c[2] : 0u, 0u,
                          G);                              // last AAD block
            }
            if (S == 0) {
                if (Q >= qoff && Q - qoff < sh.nblk)
                    gh_absorb(x, c[0], c[1], c[2], c[3], G);
            } else {
                if (Q > qoff && Q - 1 - qoff < sh.nblk) {
                    uint32_t e[4];
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        e[u] = u + S < 4 ? cprev[(u + S) & 3] : c[(u + S) & 3];
                    gh_absorb(x, e[0], e[1], e[2], e[3], G);
                }
            }
#pragma unroll
            for (int u = 0; u < 4; u++)
                cprev[u] = c[u];
        }
#pragma unroll
        for (int t = 0; t < 4; t++)
            prev[t] = o[t];
    }
    // the last ciphertext block when its second quad lies past the chunks
    // (its words there are past L: zero)
    if (S) {
        const uint32_t Q = 4 * sh.nb;
        if (Q > qoff && Q - 1 - qoff < sh.nblk) {
            uint32_t e[4];
#pragma unroll
            for (int u = 0; u < 4; u++)
                e[u] = u + S < 4 ? cprev[(u + S) & 3] : 0u;
            gh_absorb(x, e[0], e[1], e[2], e[3], G);
        }
    }
    // segment nb: its quads below 4 * nb (r0 of them) are the packet's last
    u32x4 sg[4];
    const u32x4 z[4] = { { 0, 0, 0, 0 }, { 0, 0, 0, 0 }, { 0, 0, 0, 0 },
                         { 0, 0, 0, 0 } };
    seg_funnel(prev, z, p.r0, sg);
    quad_transpose(sg);
    uint32_t so[4];
    coop_offs(p.dob, so);
    const uint32_t b = sh.nb;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int q = (int)(4 * b + lq) - (int)((p.r0s >> (2 * j)) & 3u);
        if (q >= 0 && q < (int)nfq && q < (int)(4 * b))
            gstore16(obase, so[j] + 64 * b, sg[j]);
    }
}

// bytes [0, n) of the little-endian word stream x[] (n uniform) stored at
// dst (4-byte aligned): dwords, then a short and a byte
template <int NW>
DEV void store_stream(uint8_t *dst, const uint32_t (&x)[NW], uint32_t n)
{
#pragma unroll
    for (int k = 0; k < NW; k++) {
        const uint32_t lo = 4 * k;
        if (lo + 4 <= n) {
            *(uint32_t *)(dst + lo) = x[k];
        } else if (lo < n) {
            const uint32_t r = n - lo;
            if (r >= 2)
                *(uint16_t *)(dst + lo) = (uint16_t)x[k];
            if (r & 1)
                dst[lo + (r & 2)] = (uint8_t)(x[k] >> (8 * (r & 2)));
        }
    }
}

template <int NR, bool PROTECT>
__global__ __launch_bounds__(GCMW_THREADS) void k_gcm_wave(GcmWaveArgs W)
{
    const GcmArgs &A = W.A;
    __shared__ u32x4 s_tab[(AES_TAB2_BYTES + GH_LDS_BYTES) / 16];
    if (A.abort && *A.abort)
        return;
    load_aes_tables<false>(s_tab);
    const srtp_dev_key_t *key = A.keys + A.uni;
    {
        const u32x4 *src = (const u32x4 *)(A.ghash + 1024 * key->ghash_slot);
        u32x4 *dst = (u32x4 *)((char *)s_tab + AES_TAB2_BYTES);
        for (int e = threadIdx.x; e < 256 * 16; e += blockDim.x)
            dst[e] = src[e >> 4];
    }
    __syncthreads();
    const AesLds T = make_aes_lds(s_tab);
    GhTab<true> G;
    G.lds = (const char *)s_tab + AES_TAB2_BYTES - 0x10000;   // see lane16
    G.lane16 = ((threadIdx.x & 15) * 16) | 0x10000u;
    G.g = nullptr;
    UniKey<NR> rk;
    rk.load(key);
    const uint32_t tag_len = rfl(key->tag_len);
    const bool key_ok = rfl(key->mki_size) == 0 &&
                        (tag_len == 8 || tag_len == 16);
    constexpr uint32_t VID = 16u + 2u * ((NR - 8) / 2);

    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lq = lane & 3;
    const uint32_t ngroups = (A.n + 63) >> 6;
    const uint32_t wpb = blockDim.x >> 6;
    for (uint32_t g = blockIdx.x * wpb + (threadIdx.x >> 6); g < ngroups;
         g += gridDim.x * wpb) {
        // lane L takes packet 16 * (L & 3) + (L >> 2) of the group
        const uint32_t i = 64 * g + 16 * lq + (lane >> 2);
        srtp_dev_meta_t m = { 0, 0, 0xffffffffu, 0 };
        uint64_t ioff = 0, ooff = 0;
        if (i < A.n) {
            m = A.meta[i];
            ioff = A.in_off[i];
            ooff = A.out_off[i];
        }
        const uint64_t ia = (uint64_t)(uintptr_t)A.in + ioff;
        const uint64_t oa = (uint64_t)(uintptr_t)A.out + ooff;
        const uint32_t L = rfl(m.len);
        const uint32_t es = rfl(m.info) & 0xffffu;
        const uint64_t ib =
            (((uint64_t)rfl((uint32_t)(ia >> 32)) << 32) | rfl((uint32_t)ia)) -
            0x80000000ull;
        const uint64_t ob = ((((uint64_t)rfl((uint32_t)(oa >> 32)) << 32) |
                              rfl((uint32_t)oa)) &
                             ~63ull) -
                            0x80000000ull;
        const uint64_t di = ia - ib, dob = (oa & ~63ull) - ob;
        const bool ok = i < A.n && SRTP_META_STATUS(m.info) == 0 &&
                        SRTP_META_VARIANT(m.info) == VID && m.len == L &&
                        SRTP_META_ENC_START(m.info) == es &&
                        ((ia | oa) & 15) == 0 && di < 0xffff0000ull &&
                        dob < 0xffff0000ull;
        // payload inside the counter epoch: counters j + 2 <= 255
        const bool take = key_ok && es >= 12 && L >= es && L - es <= 16 * 254 &&
                          __builtin_amdgcn_ballot_w64(ok) == ~0ull;
        if (lane == 0) {
            W.rest[g] = take ? 0 : 1;
            if (!take)
                *W.any = W.seq;
        }
        if (!take)
            continue;

        const uint8_t *ibase = (const uint8_t *)(uintptr_t)ib;
        uint8_t *obase = (uint8_t *)(uintptr_t)ob;
        GwPkt p;
        p.r0 = (uint32_t)(oa >> 4) & 3u;
        p.di = (uint32_t)di;
        p.dob = (uint32_t)dob;
        p.r0s = qperm<0x00>(p.r0) | (qperm<0x55>(p.r0) << 2) |
                (qperm<0xAA>(p.r0) << 4) | (qperm<0xFF>(p.r0) << 6);
        GwShape sh;
        sh.L = L;
        sh.hw = es >> 2;
        sh.nblk = (L - es + 15) >> 4;
        sh.nb = (L + 63) >> 6;

        // IV = (00 00 || SSRC || ROC || SEQ) ^ salt12   (srtp.c:1925-1959)
        const srtp_dev_key_t *kp = key;
        asm volatile("" : "+s"(kp));
        const uint8_t *pin = (const uint8_t *)(uintptr_t)ia;
        const uint32_t w0 = bswap(*(const uint32_t *)pin);
        const uint32_t ssrc = bswap(*(const uint32_t *)(pin + 8));
        const uint32_t seq = w0 & 0xffffu;
        const uint32_t iv0 = (ssrc >> 16) ^ bswap(rfl(kp->salt[0]));
        const uint32_t iv1 = ((ssrc << 16) | (m.roc >> 16)) ^ bswap(rfl(kp->salt[1]));
        const uint32_t iv2 = ((m.roc << 16) | seq) ^ bswap(rfl(kp->salt[2]));
        const uint32_t c0 = bswap(iv0), c1 = bswap(iv1), c2 = bswap(iv2);
        const uint32_t cc[4] = { c0, c1, c2, 0u };   // BE32(j + 2) < 256
        const CtrCache C = ctr_cache<NR, false>(cc, rk, T);

        uint32_t x[4] = { 0, 0, 0, 0 };   // GHASH accumulator (BE words)
        uint32_t tailw = 0;
        switch (sh.hw & 3) {
        case 0:
            gw_chunks<0, NR, PROTECT>(p, sh, ibase, obase, C, rk, T, G, x, tailw);
            break;
        case 1:
            gw_chunks<1, NR, PROTECT>(p, sh, ibase, obase, C, rk, T, G, x, tailw);
            break;
        case 2:
            gw_chunks<2, NR, PROTECT>(p, sh, ibase, obase, C, rk, T, G, x, tailw);
            break;
        default:
            gw_chunks<3, NR, PROTECT>(p, sh, ibase, obase, C, rk, T, G, x, tailw);
            break;
        }
        // length block [len(A)]64 || [len(C)]64 in bits, tag = E(J0) ^ S
        x[1] ^= es * 8;
        x[3] ^= (L - es) * 8;
        ghash_mul(x, G);
        uint32_t e0 = c0, e1 = c1, e2 = c2, e3 = bswap(1u);
        aes_block<NR, false>(e0, e1, e2, e3, rk, T);
        const uint32_t tw[4] = { bswap(x[0]) ^ e0, bswap(x[1]) ^ e1,
                                 bswap(x[2]) ^ e2, bswap(x[3]) ^ e3 };
        if (PROTECT) {
            // the tag at L (srtp.c:2252-2264), merged with the packet's last
            // partial data word: window words from byte 4 * (L / 4)
            const uint32_t e = L & 3;
            uint32_t win[5];
#pragma unroll
            for (int k = 0; k < 5; k++) {
                const uint32_t hi = k < 4 ? tw[k] : 0u;
                const uint32_t lo = k ? tw[k - 1] : 0u;
                win[k] = e ? (uint32_t)((((uint64_t)hi << 32) | lo) >> (32 - 8 * e))
                           : hi;
            }
            if (e)
                win[0] |= tailw & (0xffffffffu >> (32 - 8 * e));
            store_stream<5>((uint8_t *)(uintptr_t)(oa + (L & ~3u)), win,
                            e + tag_len);
        } else {
            // the plaintext's last partial word
            const uint32_t e = L & 3;
            if (e) {
                const uint32_t win[1] = { tailw };
                store_stream<1>((uint8_t *)(uintptr_t)(oa + (L & ~3u)), win, e);
            }
            // constant-time compare with the packet's tag
            const uint8_t *tp = pin + L;
            uint32_t diff = 0;
            for (uint32_t u = 0; u < tag_len; u++)
                diff |= (uint32_t)(tp[u] ^ (uint8_t)(tw[u >> 2] >> (8 * (u & 3))));
            A.auth_ok[i] = diff == 0;
        }
    }
}

}   // namespace

template <int NR>
int launch_gcm_wave_nr(srtp_gpu_t *g, GcmArgs &A, bool prot, hipStream_t st)
{
    const size_t ngroups = (A.n + 63) / 64;
    if (g->rest_cap < ngroups) {
        if (g->d_rest)
            HIPCHK(hipFree(g->d_rest));
        g->d_rest = nullptr;
        g->rest_cap = 0;
        size_t cap = 4096;
        while (cap < ngroups)
            cap *= 2;
        HIPCHK(hipMalloc(&g->d_rest, cap));
        g->rest_cap = cap;
    }
    if (!g->d_any) {
        HIPCHK(hipMalloc(&g->d_any, 4));
        HIPCHK(hipMemsetAsync(g->d_any, 0, 4, st));
    }
    GcmWaveArgs W;
    W.A = A;
    W.rest = g->d_rest;
    W.any = g->d_any;
    W.seq = ++g->wave_seq;
    if (W.seq == 0)
        W.seq = ++g->wave_seq;
    const size_t wpb = GCMW_THREADS / 64;
    const size_t wgs = (ngroups + wpb - 1) / wpb;
    const size_t cap = (size_t)g->ncu;
    const dim3 grid((unsigned)(wgs < cap ? wgs : cap)), block(GCMW_THREADS);
    if (prot)
        hipLaunchKernelGGL((k_gcm_wave<NR, true>), grid, block, 0, st, W);
    else
        hipLaunchKernelGGL((k_gcm_wave<NR, false>), grid, block, 0, st, W);
    HIPCHK(hipGetLastError());
    A.rest = g->d_rest;
    A.any = g->d_any;
    A.any_seq = W.seq;
    return 1;
}

int launch_gcm_wave(srtp_gpu_t *g, GcmArgs &A, int nr, bool prot,
                    hipStream_t st)
{
    if (A.n < 64 || A.uni == 0xffffffffu || g->wave_off)
        return 0;
    if (nr == 10)
        return launch_gcm_wave_nr<10>(g, A, prot, st);
    if (nr == 14)
        return launch_gcm_wave_nr<14>(g, A, prot, st);
    return 0;
}
