// srtp_icm.hip -- k_icm_hmac: AES-ICM keystream + XOR + HMAC-SHA1 for SRTP
// protect / unprotect, one lane per packet, any mix of keys, lengths and
// header sizes; uniform-key batches take the lane-quad cooperative memory
// path in the steady state.
//
// Replaces, on the GPU, the per-packet crypto libsrtp's srtp_protect /
// srtp_unprotect run through the cipher/auth vtables:
//   AES-ICM   crypto/cipher/aes_icm.c:236-414  (+ aes.c:2102-2130)
//   HMAC-SHA1 crypto/hash/hmac.c:157-229, crypto/hash/sha1.c:91-463
// driven as in srtp/srtp.c:2493-2818 (protect), 2820-3172 (unprotect).
//
// Compiled once per AES round count (-DICM_NR=0 null cipher, 10, 12, 14)
// and key mode (-DICM_KM, IcmKeyMode in srtp_gpu_int.h).
#include "srtp_dev_common.h"
#include "srtp_gpu_int.h"
#include "srtp_fused.h"

#if !defined(ICM_NR) || !defined(ICM_KM)
#error "ICM_NR (0, 10, 12 or 14) and ICM_KM (IcmKeyMode) must be defined"
#endif

namespace {

// ---------------------------------------------------------------------------
// AES-ICM + HMAC-SHA1 protect / unprotect: one lane per packet.
#ifndef ICM_NB_N
#define ICM_NB_N 2
#endif
constexpr int ICM_NB = ICM_NB_N;   // AES blocks interleaved per round (steady state)
constexpr int ICM_PF = 1;   // chunks of packet data loaded ahead (per-lane path)

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
// words of the SHA-1 message tail (sha1.c srtp_sha1_final).  The keystream
// blocks that any payload byte uses come from the counter cache inside the
// first epoch (blocks 0..255), from full AES past it.
template <int NR, bool TAB4, bool AUTH, bool PROTECT, class KEY>
DEV void icm_chunk(uint32_t b, const IcmPkt &p, const CtrCache &C,
                   const KEY &rk, const AesLds &T, uint32_t ks_prev[4],
                   uint32_t hst[5], uint32_t tailq[4], u32x4 (&oq)[4])
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
                if (jf + ICM_NB - 1 < 0 || 16 * jf >= (int)p.P)
                    continue;
                auto &kg = *reinterpret_cast<uint32_t(*)[ICM_NB][4]>(&ks[g]);
                if (jf >= 0 && jf + ICM_NB - 1 < 256) {
                    uint32_t jb[ICM_NB];
#pragma unroll
                    for (int j = 0; j < ICM_NB; j++)
                        jb[j] = (uint32_t)(jf + j) << 8;
                    aes_ctr<ICM_NB, NR, TAB4>(kg, jb, C, rk, T);
                } else {
                    aes_blocks<ICM_NB, NR, TAB4>(kg, rk, T);
                }
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
    if constexpr (NR > 0) {
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
    if (AUTH)
        sha1_compress(hst, wv);
}

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


// keystream of chunk b (4 counter blocks of the cached epoch)
template <int NR, bool TAB4, class KEY>
DEV void coop_keystream(uint32_t b, const IcmPkt &p, const CtrCache &C,
                        const KEY &rk, const AesLds &T, uint32_t (&ks)[4][4])
{
    if constexpr (NR > 0) {
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
            nx[j] = *(gcptr)(cp.in[j] + 64 * (b + 1));
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
        *(gptr)(cp.seg[j] + 64 * b) = sg[j];
    if (NEXT)
        coop_keystream<NR, TAB4>(b + 1, p, C, rk, T, ks);
    if (AUTH)
        sha1_compress(hst, wv);
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

// per-packet constants from the packet's meta record and header
template <int NR, bool AUTH>
DEV IcmPkt make_pkt(const uint8_t *in, uint8_t *out, const srtp_dev_meta_t &m,
                    const srtp_dev_key_t *key)
{
    IcmPkt p;
    p.in = in;
    p.out = out;
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

    return p;
}

// kernel variant id of this instantiation (meta info [31:24])
template <int NR, bool AUTH>
constexpr uint32_t icm_vid()
{
    return (NR == 0 ? 0u : 8u + 2u * ((NR - 8) / 2)) + (AUTH ? 1u : 0u);
}

// one packet, front to back: header chunks, steady payload chunks, tail
// chunks, partial quad, outer hash, tag (srtp.c:2694-2818 protect,
// 2987-3093 unprotect: the tag is compared, the caller decides).  i indexes
// auth_ok[]; slot is the key of KM_UNI / KM_WAVE launches (KM_LANE: m.key).
template <int NR, bool TAB4, bool AUTH, bool PROTECT, int KM, class KEY>
DEV void icm_packet(const IcmArgs &A, const srtp_dev_meta_t &m,
                    uint64_t in_off, uint64_t out_off, uint32_t i,
                    uint32_t slot, const AesLds &T, KEY &rk)
{
    if (SRTP_META_STATUS(m.info) || SRTP_META_VARIANT(m.info) != icm_vid<NR, AUTH>())
        return;
    if constexpr (KM == KM_LANE)
        slot = m.key;
    const srtp_dev_key_t *key = A.keys + slot;
    if constexpr (KM == KM_LANE && NR > 0)
        rk.reload(A.keys, slot);

    IcmPkt p = make_pkt<NR, AUTH>(A.in + in_off, A.out + out_off, m, key);

    uint32_t hst[5];
#pragma unroll
    for (int k = 0; k < 5; k++)
        hst[k] = AUTH ? key->ipad[k] : 0;

    uint32_t ks_prev[4] = { 0, 0, 0, 0 };
    uint32_t tailq[4] = { 0, 0, 0, 0 };
    u32x4 prev[4];   // output quads of the last chunk done
    // rounds 1-2 of the packet's first counter epoch (every chunk uses it)
    CtrCache C{};
    if constexpr (NR > 0) {
        if (p.conf)
            C = ctr_cache<NR, TAB4>(p.cb, rk, T);
    }
    uint32_t b = 0;
    {
        for (; b < p.bclean && b < p.nb; b++)
            icm_chunk<NR, TAB4, AUTH, PROTECT>(b, p, C, rk, T, ks_prev, hst,
                                               tailq, prev);

        // steady chunks: full chunks whose blocks j = 4b+t-qoff stay in counter
        // epoch 0 (j <= 255, 4 KiB of payload)
        uint32_t se = p.L >> 6;
        se = se < ((256 + p.qoff) >> 2) ? se : ((256 + p.qoff) >> 2);
        if (b < se) {
            bool coop = false;
            if constexpr (KM != KM_LANE) {
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
            icm_chunk<NR, TAB4, AUTH, PROTECT>(b, p, C, rk, T, ks_prev, hst,
                                               tailq, prev);
        if (p.L & 15)
            store_words_partial(p.out + (p.L & ~15u), tailq, (int)(p.L & 15));
    }

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

    // the tag: the first tag_len bytes of the digest (big-endian words)
    uint32_t tw[5];
#pragma unroll
    for (int k = 0; k < 5; k++)
        tw[k] = bswap(oh[k]);
    if (PROTECT) {
        for (uint32_t u = 0; u < mki_size; u++)
            out[L + u] = key->mki[u];
        store_tag(out + L + mki_size, tw, tag_len);
    } else {
        A.auth_ok[i] = tag_diff(p.in + L + mki_size, tw, tag_len) == 0;
    }
}

// the fused classification (fz_classify / fzu_classify, FzLane, GlbSrc):
// srtp_fused.h

// one packet of a fused batch from the arena: classification, crypto, and
// (unprotect) the verdict
template <int NR, bool TAB4, bool AUTH, bool PROTECT, int KM, class KEY>
DEV void fz_one(const IcmArgs &A, uint32_t i, FzLane &z, uint64_t off,
                uint32_t len, uint32_t cap, const GlbSrc &S, const AesLds &T,
                KEY &rk)
{
    if constexpr (PROTECT) {
        const srtp_dev_meta_t m =
            fz_classify(A, i, z, icm_vid<NR, AUTH>(), off, len, cap, S);
        icm_packet<NR, TAB4, AUTH, PROTECT, KM>(A, m, off, off, i, A.uni, T,
                                                rk);
    } else {
        uint64_t e;
        uint32_t sid;
        const srtp_dev_meta_t m = fzu_classify(A, i, z, icm_vid<NR, AUTH>(),
                                               off, len, cap, S, e, sid);
        icm_packet<NR, TAB4, AUTH, PROTECT, KM>(A, m, off, off, i, A.uni, T,
                                                rk);
        if (sid != FZ_NOCHAIN)
            fzu_verdict(A, i, z, m, e, sid, A.auth_ok[i] != 0);
    }
}

// All four T-tables (128 KiB of LDS, one 512-lane workgroup per CU).  The
// AES schedule sits in SGPRs (KM_UNI / KM_WAVE) or VGPRs (KM_LANE).  With
// per-lane keys the kernel needs 230-256 VGPRs, so two waves per SIMD is
// all a CU holds whatever the table size: (T0, T1) + rotations (64 KiB)
// bought no occupancy and cost 8 VALU per round (configs[3] kernel 2.31 ->
// 2.24 ms with four tables, MI355X A/B).  Persistent: the grid is sized to
// the CUs and each workgroup walks the batch, so the tables are loaded once
// per CU.
#ifndef ICM_THREADS_UNI_N
#define ICM_THREADS_UNI_N 512
#endif
constexpr int ICM_THREADS_UNI = ICM_THREADS_UNI_N;
constexpr int ICM_THREADS_LANE = 512;
constexpr uint32_t ICM_SKIP = 0xffffffffu;

// FUSED: 0 = meta descriptors, 1 = the order-free classification in the
// kernel, 2 = that over the wave groups k_icm_stg listed (fz.glist)
template <int NR, bool AUTH, bool PROTECT, int KM, int FUSED = 0>
__global__ __launch_bounds__(KM == KM_LANE ? ICM_THREADS_LANE : ICM_THREADS_UNI)
void k_icm_hmac(IcmArgs A)
{
    constexpr bool TAB4 = true;
    constexpr int NRK = NR ? NR : 1;
    constexpr int LDSB = NR ? AES_TAB4_BYTES : 16;
    __shared__ u32x4 s_tab[LDSB / 16];
    __shared__ uint32_t s_t0[256];   // the S-box row during the table build
    if (A.abort && *A.abort)
        return;
    // after k_icm_stg: only the groups it listed (usually none)
    if (FUSED == 2 && *(volatile const uint32_t *)A.fz.glist == 0)
        return;
    if (NR)
        load_aes_tables<TAB4>(s_tab, s_t0);
    __syncthreads();
    const AesLds T = make_aes_lds(s_tab);

    typename std::conditional<KM == KM_LANE, LaneKey<NRK>, UniKey<NRK>>::type rk;
    if (KM == KM_UNI && NR)
        rk.load(A.keys + A.uni);
    // lane L of a wave takes packet 16 * (L & 3) + (L >> 2) of the wave's 64
    // (the cooperative path exchanges data inside lane quads)
    const uint32_t L = threadIdx.x & 63;
    const uint32_t lpos = 16 * (L & 3) + (L >> 2);
    if (!A.rec) {
        // packet order
        const uint32_t stride = gridDim.x * blockDim.x;
        const uint32_t first = blockIdx.x * blockDim.x + (threadIdx.x & ~63u) + lpos;
        if constexpr (FUSED) {
            FzLane z;
            z.ssrc = 0;
            z.sid = FZ_NOCHAIN;
            z.run_sid = FZ_NOCHAIN;
            z.run_cnt = 0;
            z.run_max = 0;
            z.run_min = ~0ull;
            z.run_cmax = 0;
            z.bw_idx = 0;
            z.bw_bits = 0;
            // wave groups of 64 consecutive packets: every group in turn,
            // or (glmode) the groups k_icm_stg listed
            const uint32_t nw = gridDim.x * (blockDim.x >> 6);
            // (glmode: this wave's own list, the groups k_icm_stg's wave of
            // the same id left, so each lane keeps its stream and key)
            constexpr bool GL = FUSED == 2;
            const uint32_t wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
            const uint32_t gcap = (((A.n + 63) >> 6) + nw - 1) / nw;
            const uint32_t *gl = A.fz.glist + 1 + FZ_GL_WAVES + wid * gcap;
            const uint32_t cnt = GL ? A.fz.glist[1 + wid] : 0u;
            for (uint32_t k = 0, w = wid;; k++, w += nw) {
                if (GL ? k >= cnt : 64ull * w >= A.n)
                    break;
                const uint32_t i = 64 * (GL ? gl[k] : w) + lpos;
                if (i >= A.n)
                    continue;
                // fused batches are in place (fused_ok): one offset
                const uint64_t off = A.in_off[i];
                const GlbSrc S{ A.in + off };
                fz_one<NR, TAB4, AUTH, PROTECT, KM>(
                    A, i, z, off, A.fz.in_len[i], A.fz.cap[i], S, T, rk);
            }
            fz_flush<PROTECT>(A.fz, z);
            return;
        }
        if constexpr (KM == KM_UNI && FUSED == 0) {
            if (A.ch.st) {
                // one stream in order: packet 0 fixes seq_0 and e_0
                const srtp_dev_stream_t S = *A.ch.st;
                uint32_t seq0;
                uint64_t e0;
                const bool e0ok = srtp_inorder_head(S, A.in + A.in_off[0],
                                                    !PROTECT, seq0, e0);
                for (uint32_t i = first; i < A.n; i += stride) {
                    const uint64_t off = A.in_off[i];
                    icm_packet<NR, TAB4, AUTH, PROTECT, KM>(
                        A, inorder_meta<!PROTECT>(A, i, off, S, seq0, e0, e0ok),
                        off, A.out_off[i], i, A.uni, T, rk);
                }
                return;
            }
        }
        for (uint32_t i = first; i < A.n; i += stride)
            icm_packet<NR, TAB4, AUTH, PROTECT, KM>(
                A, A.meta[i], A.in_off[i], A.out_off[i], i, A.uni, T, rk);
        return;
    }
    // key buckets: records [range[0], range[1])
    const uint32_t beg = A.range[0], end = A.range[1];
    if constexpr (KM == KM_WAVE) {
        // one key per aligned group of 64 records (a stream's bucket)
        const uint32_t wpb = blockDim.x >> 6;
        const uint32_t nw = gridDim.x * wpb;
        for (uint32_t g = blockIdx.x * wpb + (threadIdx.x >> 6);
             beg + 64 * g < end; g += nw) {
            const uint32_t g0 = beg + 64 * g;
            const uint32_t info0 =
                __builtin_amdgcn_readfirstlane(A.rec[g0].meta.info);
            if (SRTP_META_STATUS(info0) ||
                SRTP_META_VARIANT(info0) != icm_vid<NR, AUTH>())
                continue;   // an empty group, or another kernel's stream
            const uint32_t slot =
                __builtin_amdgcn_readfirstlane(A.rec[g0].meta.key);
            if (NR)
                rk.load(A.keys + slot);
            const uint32_t pos = g0 + lpos;
            if (pos < end) {
                const srtp_dev_rec_t r = A.rec[pos];
                icm_packet<NR, TAB4, AUTH, PROTECT, KM>(
                    A, r.meta, r.in_off, r.out_off,
                    PROTECT ? 0u : A.rec_idx[pos], slot, T, rk);
            }
        }
    } else {
        const uint32_t stride = gridDim.x * blockDim.x;
        for (uint32_t pos = beg + blockIdx.x * blockDim.x + (threadIdx.x & ~63u) + lpos;
             pos < end; pos += stride) {
            const srtp_dev_rec_t r = A.rec[pos];
            icm_packet<NR, TAB4, AUTH, PROTECT, KM>(
                A, r.meta, r.in_off, r.out_off,
                PROTECT ? 0u : A.rec_idx[pos], A.uni, T, rk);
        }
    }
}

// ---------------------------------------------------------------------------
// Staged fused kernel (k_icm_stg): per-lane keys, the order-free
// classification inside the kernel, small packets in contiguous slots --
// BASELINE configs[3]'s shape (8M x 172-byte packets in 192-byte slots).
//
// The per-lane form moves every packet through 16-byte per-lane accesses:
// each wave instruction touches 64 packets 192 B apart, and a 172-byte
// packet costs its lane ~28 loads and ~18 stores, most to lines no other
// lane of the wave touches, behind two dependent steps (offset -> header,
// offset -> data).  Measured: the waves wait on memory 41 % of their
// cycles, and the counted traffic is 1.67x the algorithmic bytes
// (profiles/r04_g711_protect.md).  Here a wave takes 64 CONSECUTIVE packets
// (a group) and, when their slots tile one span [off0, off0 + 64 D) with
// D <= 192, moves the span through LDS:
//   * in: 4D/64 (12 for D = 192) global_load_lds_dwordx4 sweeps, 1 KiB of
//     contiguous bytes per wave-instruction, no VGPRs;
//   * every lane classifies, encrypts / decrypts and authenticates its
//     packet out of the image and writes the result (output words, tag,
//     MKI) back into it;
//   * out: the span is stored back with the same 1-KiB sweeps.  Bytes of
//     a slot past the packet (its capacity: cap >= D) go back unchanged.
// Granule k (16 B) of the span sits at LDS granule stg_swz(k) = k ^ ((k /
// 48) & 3): for D = 192 (packet p's granule q is k = 12p + q) every
// ds_read_b128 lane group of 16 reads 16 distinct banks (lanes p, p' of a
// group with equal p mod 4 differ in (p >> 2) & 3, and the XOR of those
// bits separates them; p mod 4 separates the rest through bits 2-3 of k).
// The swizzle changes only bits 0-1 of k as a function of bits >= 4, so it
// is its own inverse and each quarter-wave of a sweep still covers one
// 256-byte block.
// Slots of 64, 128 or 192 bytes (D a multiple of 64: see StgImg).
// LDS: the image, 12 KiB per wave (96 KiB for 8 waves), leaves 64 KiB for
// the AES tables: (T0, T1) with T2 / T3 as rotations (TAB4 = false).
// A group outside the conditions runs the per-lane form from the arena.
constexpr uint32_t STG_GRAN = 768;   // granules per wave image (12 KiB)
constexpr uint32_t STG_WAVES = 8;    // 512 lanes per workgroup

DEV uint32_t stg_swz(uint32_t k) { return k ^ ((k / 48u) & 3u); }

// the wave's image, seen from one lane's packet (first granule k0)
// Slots of D = 64, 128 or 192 bytes put the packet's first granule k0 =
// L * D / 16 on a multiple of 4 and keep its granules inside one 48-granule
// block, so its swizzle is one per-lane constant f on bits 0-1: granule q
// of the packet sits at k0 + (q ^ f)
struct StgImg {
    u32x4 *pk;               // image + k0
    uint32_t f;              // (k0 / 48) & 3
    uint32_t D;              // slot bytes
    const uint8_t *p;        // the packet in the arena (reads past the slot)
    DEV u32x4 *gp(uint32_t x) const { return pk + ((x >> 4) ^ f); }
    DEV u32x4 ld(uint32_t q) const { return pk[q ^ f]; }
    DEV void st(uint32_t q, const u32x4 &v) const { pk[q ^ f] = v; }
    // 4-aligned word / byte at byte offset x of the packet
    DEV uint32_t ldw(uint32_t x) const
    {
        return ((const uint32_t *)gp(x))[(x >> 2) & 3];
    }
    DEV void stw(uint32_t x, uint32_t v) const
    {
        ((uint32_t *)gp(x))[(x >> 2) & 3] = v;
    }
    DEV uint32_t byte(uint32_t x) const
    {
        return ((const uint8_t *)gp(x))[x & 15];
    }
    DEV void stb(uint32_t x, uint32_t v) const
    {
        ((uint8_t *)gp(x))[x & 15] = (uint8_t)v;
    }
    // srtp_parse_rtp (srtp_rtp_hdr.h) over the image
    DEV srtp_dev_hdr_t hdr(uint64_t off, uint32_t len) const
    {
        srtp_dev_hdr_t h;
        h.len = len;
        h.ssrc = 0;
        h.seq_len = 0;
        uint32_t err = 0, es = 0;
        if ((off & 15) != 0 || len < 12) {
            err = 2;
        } else {
            const u32x4 q = ld(0);
            const uint32_t w0 = bswap(q.x);
            h.ssrc = bswap(q.z);
            h.seq_len = w0 & 0xffffu;
            es = 12 + 4 * ((w0 >> 24) & 0xfu);
            if (len < es) {
                err = 2;
            } else if ((w0 >> 28) & 1) {
                if (len < es + 4) {
                    err = 2;
                } else {
                    es += ((bswap(ldw(es)) & 0xffffu) + 1) * 4;
                    if (len < es)
                        err = 2;
                }
            }
        }
        h.enc_start = err ? (err << 24) : es;
        return h;
    }
    // the tn (<= 16) bytes at x, little-endian words (fz_tail_save); past
    // the slot (a trailer longer than the slot holds: the group then runs
    // from the arena) from the arena
    DEV void tail(uint32_t x, uint32_t tn, u32x4 &w4) const
    {
        if (x + tn > D) {
            fz_tail_save(p + x, tn, w4);
            return;
        }
        const uint32_t a = x & ~3u, r = x & 3;
        uint32_t W[5];
#pragma unroll
        for (int k = 0; k < 5; k++)
            W[k] = a + 4 * k < x + tn ? ldw(a + 4 * k) : 0;
#pragma unroll
        for (int k = 0; k < 4; k++)
            w4[k] = __builtin_amdgcn_alignbyte(W[k + 1], W[k], r);
    }
    // the first n bytes of the little-endian words w at byte offset x
    template <int NW>
    DEV void put(uint32_t x, const uint32_t (&w4)[NW], uint32_t n) const
    {
        const bool al = (x & 3) == 0;
#pragma unroll
        for (int j = 0; j < NW; j++) {
            const int r = (int)n - 4 * j;
            if (r <= 0)
                break;
            if (r >= 4 && al) {
                stw(x + 4 * j, w4[j]);
                continue;
            }
#pragma unroll
            for (int b = 0; b < 4; b++)
                if (b < r)
                    stb(x + 4 * j + b, w4[j] >> (8 * b));
        }
    }
    template <int NW>
    DEV uint32_t diff(uint32_t x, const uint32_t (&w4)[NW], uint32_t n) const
    {
        const bool al = (x & 3) == 0;
        uint32_t d = 0;
#pragma unroll
        for (int j = 0; j < NW; j++) {
            const int r = (int)n - 4 * j;
            if (r <= 0)
                break;
            if (r >= 4 && al) {
                d |= ldw(x + 4 * j) ^ w4[j];
                continue;
            }
#pragma unroll
            for (int b = 0; b < 4; b++)
                if (b < r)
                    d |= byte(x + 4 * j + b) ^ ((w4[j] >> (8 * b)) & 0xffu);
        }
        return d;
    }
};

// icm_chunk over the image: chunk b's quads read from and written back to
// the lane's granules; the partial last quad keeps the image's bytes past
// the data (what follows the packet in its slot, or the tag on unprotect)
template <int S, int NR, bool AUTH, bool PROTECT, class KEY>
DEV void stg_chunk(uint32_t b, const IcmPkt &p, const CtrCache &C,
                   const KEY &rk, const AesLds &T, uint32_t ks_prev[4],
                   uint32_t hst[5], const StgImg &I)
{
    constexpr bool TAB4 = false;
    const uint32_t q0 = 4 * b;
    u32x4 v[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        v[t] = u32x4{ 0, 0, 0, 0 };
        if (q0 + t < p.nq)
            v[t] = I.ld(q0 + t);
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
    if (p.conf) {
#pragma unroll
        for (int g = 0; g < 4; g += ICM_NB) {
            const int jf = (int)(q0 + g) - (int)p.qoff;
            if (jf + ICM_NB - 1 < 0 || 16 * jf >= (int)p.P)
                continue;
            auto &kg = *reinterpret_cast<uint32_t(*)[ICM_NB][4]>(&ks[g]);
            if (jf >= 0 && jf + ICM_NB - 1 < 256) {
                uint32_t jb[ICM_NB];
#pragma unroll
                for (int j = 0; j < ICM_NB; j++)
                    jb[j] = (uint32_t)(jf + j) << 8;
                aes_ctr<ICM_NB, NR, TAB4>(kg, jb, C, rk, T);
            } else {
                aes_blocks<ICM_NB, NR, TAB4>(kg, rk, T);
            }
        }
    } else {
#pragma unroll
        for (int t = 0; t < 4; t++)
            ks[t][0] = ks[t][1] = ks[t][2] = ks[t][3] = 0;
    }
    uint32_t wv[16];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const uint32_t q = q0 + t;
        // the keystream shifted by S = header words mod 4 (register renaming)
        uint32_t kk[4];
#pragma unroll
        for (int u = 0; u < 4; u++)
            kk[u] = u >= S ? ks[t][u - S]
                           : (t ? ks[t - 1][u - S + 4] : ks_prev[u - S + 4]);
        if (b < p.bclean) {
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (4 * q + u < p.hw)
                    kk[u] = 0;   // header words are never encrypted
        }
        u32x4 o;
#pragma unroll
        for (int u = 0; u < 4; u++)
            o[u] = v[t][u] ^ kk[u];
        if (16 * q + 16 <= p.L) {
            I.st(q, o);
        } else if (16 * q < p.L) {
            // bytes [L, 16q + 16) keep what the image holds
            const uint32_t n = p.L - 16 * q;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int r = (int)n - 4 * u;
                const uint32_t m = r >= 4 ? ~0u
                                          : (r <= 0 ? 0u : (1u << (8 * r)) - 1);
                o[u] = bsel(m, o[u], v[t][u]);
            }
            I.st(q, o);
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            wv[4 * t + u] = bswap(PROTECT ? o[u] : v[t][u]);
    }
#pragma unroll
    for (int u = 0; u < 4; u++)
        ks_prev[u] = ks[3][u];
    if (AUTH) {
        if (64 * b + 64 > p.L) {
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

template <int S, int NR, bool AUTH, bool PROTECT, class KEY>
DEV void stg_chunks(const IcmPkt &p, const CtrCache &C, const KEY &rk,
                    const AesLds &T, uint32_t hst[5], const StgImg &I)
{
    uint32_t ks_prev[4] = { 0, 0, 0, 0 };
    for (uint32_t b = 0; b < p.nb; b++)
        stg_chunk<S, NR, AUTH, PROTECT>(b, p, C, rk, T, ks_prev, hst, I);
}

// The per-packet words of a key record (srtp_dev_key_t): loaded for the
// lane's last stream before the group's image arrives (one wait for both),
// again after the classification only when the packet has another key
struct StgKey {
    uint32_t slot;
    uint32_t salt[4], ipad[5], opad[5];
    uint32_t tag_len, mki_size, conf;
    DEV void load(const srtp_dev_key_t *keys, uint32_t s)
    {
        const srtp_dev_key_t *k = keys + s;
        slot = s;
#pragma unroll
        for (int j = 0; j < 4; j++)
            salt[j] = k->salt[j];
#pragma unroll
        for (int j = 0; j < 5; j++) {
            ipad[j] = k->ipad[j];
            opad[j] = k->opad[j];
        }
        tag_len = k->tag_len;
        mki_size = k->mki_size;
        conf = k->conf;
    }
};

// one packet out of the image (icm_packet restated over it); returns the
// tag verdict (unprotect; true on protect)
template <int NR, bool AUTH, bool PROTECT>
DEV bool stg_packet(const IcmArgs &A, const srtp_dev_meta_t &m,
                    const StgKey &K, const StgImg &I, const AesLds &T,
                    LaneKey<NR> &rk)
{
    constexpr bool TAB4 = false;
    const uint32_t slot = m.key;
    const srtp_dev_key_t *key = A.keys + slot;
    rk.reload(A.keys, slot);

    IcmPkt p;
    p.in = nullptr;
    p.out = nullptr;
    const uint32_t enc_start = SRTP_META_ENC_START(m.info);
    p.L = m.len;
    p.hw = enc_start >> 2;
    p.s = p.hw & 3;
    p.qoff = p.hw >> 2;
    p.P = p.L - enc_start;
    p.roc = m.roc;
    p.conf = K.conf != 0;
    p.nq = (p.L + 15) >> 4;
    p.nb = AUTH ? ((p.L + 12) >> 6) + 1 : ((p.nq + 3) >> 2);
    p.bclean = (p.qoff + 4) >> 2;
    // counter block (aes_icm.c:236-258, srtp.c:2694-2707)
    const uint32_t seq = bswap(I.ldw(0)) & 0xffffu;
    p.cb[0] = K.salt[0];
    p.cb[1] = K.salt[1] ^ I.ldw(8);   // SSRC bytes
    p.cb[2] = K.salt[2] ^ bswap(m.roc);
    p.cb[3] = K.salt[3] ^ (seq >> 8) ^ ((seq & 0xffu) << 8);

    uint32_t hst[5];
#pragma unroll
    for (int k = 0; k < 5; k++)
        hst[k] = AUTH ? K.ipad[k] : 0;
    CtrCache C{};
    if (p.conf)
        C = ctr_cache<NR, TAB4>(p.cb, rk, T);
    switch (p.s) {
    case 0: stg_chunks<0, NR, AUTH, PROTECT>(p, C, rk, T, hst, I); break;
    case 1: stg_chunks<1, NR, AUTH, PROTECT>(p, C, rk, T, hst, I); break;
    case 2: stg_chunks<2, NR, AUTH, PROTECT>(p, C, rk, T, hst, I); break;
    default: stg_chunks<3, NR, AUTH, PROTECT>(p, C, rk, T, hst, I); break;
    }

    const uint32_t tag_len = K.tag_len;
    const uint32_t mki_size = K.mki_size;
    if (!AUTH) {
        if (PROTECT && mki_size) {
            for (uint32_t u = 0; u < mki_size; u++)
                I.stb(p.L + u, key->mki[u]);
        }
        return true;
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
        oh[k] = K.opad[k];
    sha1_compress(oh, ow);
    uint32_t tw[5];
#pragma unroll
    for (int k = 0; k < 5; k++)
        tw[k] = bswap(oh[k]);
    if (PROTECT) {
        for (uint32_t u = 0; u < mki_size; u++)
            I.stb(p.L + u, key->mki[u]);
        I.put(p.L + mki_size, tw, tag_len);
        return true;
    }
    return I.diff(p.L + mki_size, tw, tag_len) == 0;
}

template <int NR, bool AUTH, bool PROTECT>
__global__ __launch_bounds__(512) void k_icm_stg(IcmArgs A)
{
    constexpr bool TAB4 = false;
    // one LDS object: the tables at LDS address 0, so a lookup's address is
    // its v_perm result (the ds_read immediate offset takes the odd table);
    // the images after them (96 KiB past a second object's base would cost
    // a v_add per lookup: the immediate offset holds 16 bits)
    constexpr uint32_t TABQ = AES_TAB2_BYTES / 16;
    __shared__ u32x4 s_lds[TABQ + STG_WAVES * STG_GRAN];
    if (A.abort && *A.abort)
        return;
    // the S-box row of the table build sits in the image area
    load_aes_tables<TAB4>(s_lds, (uint32_t *)(s_lds + TABQ));
    __syncthreads();
    const AesLds T = make_aes_lds(s_lds);
    LaneKey<NR> rk;
    const IcmFused &F = A.fz;
    FzLane z;
    z.ssrc = 0;
    z.sid = FZ_NOCHAIN;
    z.run_sid = FZ_NOCHAIN;
    z.run_cnt = 0;
    z.run_max = 0;
    z.run_min = ~0ull;
    z.run_cmax = 0;
    z.bw_idx = 0;
    z.bw_bits = 0;
    const uint32_t L = threadIdx.x & 63, wv = threadIdx.x >> 6;
    u32x4 *img = s_lds + TABQ + wv * STG_GRAN;
    constexpr uint32_t vid = icm_vid<NR, AUTH>();
    const uint32_t nw = gridDim.x * STG_WAVES;
    const uint32_t wid = blockIdx.x * STG_WAVES + wv;
    const uint32_t gcap = (((A.n + 63) >> 6) + nw - 1) / nw;
    uint32_t *gl = F.glist + 1 + FZ_GL_WAVES + wid * gcap;
    uint32_t nl = 0;   // groups on this wave's list
    // the swizzle of image granule 64 j + L, j = 0..11, two bits each
    uint32_t fr = 0;
#pragma unroll
    for (uint32_t j = 0; j < STG_GRAN / 64; j++)
        fr |= (stg_swz(64 * j + L) ^ (64 * j + L)) << (2 * j);
    StgKey K;   // the per-packet words of the lane's last key
    K.slot = FZ_NOCHAIN;
    // the group's offset, length and capacity, loaded one group ahead
    uint64_t n_off = 0;
    uint32_t n_len = 0, n_cap = 0;
    if (64 * wid + L < A.n) {
        n_off = A.in_off[64 * wid + L];
        n_len = F.in_len[64 * wid + L];
        n_cap = F.cap[64 * wid + L];
    }
    for (uint32_t g = wid; 64ull * g < A.n; g += nw) {
        const uint32_t i = 64 * g + L;
        const bool live = i < A.n;
        const uint64_t off = n_off;
        const uint32_t len = n_len, cap = n_cap;
        {
            const uint64_t i2 = 64ull * (g + nw) + L;
            if (i2 < A.n) {
                n_off = A.in_off[i2];
                n_len = F.in_len[i2];
                n_cap = F.cap[i2];
            }
        }
        // the group's slots tile one span: off = off0 + L * D
        const uint32_t olo = (uint32_t)off, ohi = (uint32_t)(off >> 32);
        const uint64_t off0 =
            ((uint64_t)__builtin_amdgcn_readfirstlane(ohi) << 32) |
            (uint32_t)__builtin_amdgcn_readfirstlane(olo);
        const uint32_t D =
            (uint32_t)__builtin_amdgcn_readlane((int)olo, 1) - (uint32_t)off0;
        // (protect: with the largest trailer of the batch's streams, so no
        // tag written into the image leaves the packet's slot)
        const bool fit = live && (off0 & 15) == 0 && (D & 63) == 0 && D >= 64 &&
                         D <= 16 * STG_GRAN / 64 && off == off0 + (uint64_t)L * D &&
                         cap >= D && len + (PROTECT ? F.max_trailer : 0u) <= D;
        if (__builtin_amdgcn_ballot_w64(fit) != ~0ull) {
            // the per-lane form runs this group after the launch (its
            // registers, inlined here, would spill the staged form's): on
            // this wave's list, no atomic (one counter for every wave
            // would serialise them)
            if (L == 0)
                gl[nl] = g;
            nl++;
            continue;
        }
        // fill the image: sweep j, lane L -> image granule 64 j + L, span
        // granule stg_swz(64 j + L)
        const uint32_t G = 4 * D;   // granules of the span
        const uint8_t *span = A.in + off0;
#pragma unroll
        for (uint32_t j = 0; j < STG_GRAN / 64; j++) {
            if (64 * j < G)
                __builtin_amdgcn_global_load_lds(
                    (const void __attribute__((address_space(1))) *)(span + 16ull * ((64 * j + L) ^ ((fr >> (2 * j)) & 3))),
                    (void __attribute__((address_space(3))) *)(img + 64 * j), 16, 0, 0);
        }
        // the key words of the lane's last stream, under the same wait,
        // when the lane's previous group left another key's words
        {
            const uint32_t want = z.sid != FZ_NOCHAIN ? z.key : 0u;
            if (want != K.slot)
                K.load(A.keys, want);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t k0 = (L * D) >> 4;
        const StgImg I{ img + k0, (k0 / 48) & 3, D, A.in + off };
        srtp_dev_meta_t m;
        uint64_t e = 0;
        uint32_t sid = FZ_NOCHAIN;
        if constexpr (PROTECT)
            m = fz_classify(A, i, z, vid, off, len, cap, I);
        else
            m = fzu_classify(A, i, z, vid, off, len, cap, I, e, sid);
        // a packet runs only for an eligible stream of this variant, whose
        // trailer is at most max_trailer: tag and MKI stay in the slot
        const bool run = SRTP_META_STATUS(m.info) == 0 &&
                         SRTP_META_VARIANT(m.info) == vid;
        bool ok = false;
        if (run && m.key != K.slot)
            K.load(A.keys, m.key);
        if (run)
            ok = stg_packet<NR, AUTH, PROTECT>(A, m, K, I, T, rk);
        if (!PROTECT && run && A.auth_ok)
            A.auth_ok[i] = ok ? 1 : 0;
        if (!PROTECT && sid != FZ_NOCHAIN)
            fzu_verdict(A, i, z, m, e, sid, ok);
        // the image back to the span: the same sweeps
        uint8_t *ospan = A.out + off0;
#pragma unroll
        for (uint32_t j = 0; j < STG_GRAN / 64; j++) {
            if (64 * j < G)
                *(gptr)(ospan + 16ull * ((64 * j + L) ^ ((fr >> (2 * j)) & 3))) =
                    img[64 * j + L];
        }
    }
    if (L == 0) {
        F.glist[1 + wid] = nl;
        if (nl)
            F.glist[0] = 1;
    }
    fz_flush<PROTECT>(F, z);
}

}   // namespace

template <int NR, int KM, bool AU, bool PR>
static void icm_go(const IcmArgs &A, int ncu, hipStream_t st)
{
    // persistent grid: one workgroup per CU (128 KiB of tables)
    const size_t T = KM == KM_LANE ? ICM_THREADS_LANE : ICM_THREADS_UNI;
    size_t wgs = A.rec ? (size_t)-1 : (A.n + T - 1) / T;
    const size_t cap = (size_t)ncu;
    if (wgs > cap)
        wgs = cap;
    if constexpr (KM == KM_LANE && NR > 0) {
        if (A.fused && A.stg) {
            // the staged kernel, then the per-lane form over the groups it
            // left (a persistent grid that returns at once when none)
            hipLaunchKernelGGL((k_icm_stg<NR, AU, PR>), dim3((unsigned)wgs),
                               dim3(512), 0, st, A);
            hipLaunchKernelGGL((k_icm_hmac<NR, AU, PR, KM, 2>),
                               dim3((unsigned)wgs), dim3((unsigned)T), 0, st, A);
            return;
        }
        if (A.fused) {
            hipLaunchKernelGGL((k_icm_hmac<NR, AU, PR, KM, 1>),
                               dim3((unsigned)wgs), dim3((unsigned)T), 0, st, A);
            return;
        }
    }
    hipLaunchKernelGGL((k_icm_hmac<NR, AU, PR, KM>), dim3((unsigned)wgs),
                       dim3((unsigned)T), 0, st, A);
}

template <int NR, int KM>
static void icm_dir(const IcmArgs &A, bool auth, bool prot, int ncu,
                    hipStream_t st)
{
    if (auth && prot)
        icm_go<NR, KM, true, true>(A, ncu, st);
    else if (auth)
        icm_go<NR, KM, true, false>(A, ncu, st);
    else if (prot)
        icm_go<NR, KM, false, true>(A, ncu, st);
    else
        icm_go<NR, KM, false, false>(A, ncu, st);
}

// one object per (ICM_NR, ICM_KM): srtp_gpu.hip launch_icm picks the mode
template <int NR, int KM>
int launch_icm_km(const IcmArgs &A, bool auth, bool prot, int ncu,
                  hipStream_t st)
{
    icm_dir<NR, KM>(A, auth, prot, ncu, st);
    HIPCHK(hipGetLastError());
    return 0;
}

template int launch_icm_km<ICM_NR, ICM_KM>(const IcmArgs &, bool, bool, int,
                                           hipStream_t);
