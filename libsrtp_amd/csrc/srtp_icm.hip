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
// Compiled once per AES round count: -DICM_NR=0 (null cipher), 10, 12, 14.
#include "srtp_dev_common.h"
#include "srtp_gpu_int.h"

#ifndef ICM_NR
#error "ICM_NR (0, 10, 12 or 14) must be defined"
#endif

namespace {

// ---------------------------------------------------------------------------
// AES-ICM + HMAC-SHA1 protect / unprotect: one lane per packet.
#ifndef ICM_NB
#define ICM_NB 2   // AES blocks interleaved per round in the steady state
#endif
#ifndef ICM_COOP
#define ICM_COOP 1   // wave-cooperative coalesced loads / aligned stores
#endif
#ifndef ICM_SEQ
#define ICM_SEQ 0    // low-register cooperative loop (icm_seq_run)
#endif
#ifndef ICM_PIPE
#define ICM_PIPE 0   // icm_seq_run: keystream computed one chunk ahead
#endif
#ifndef ICM_LDSX
#define ICM_LDSX 0   // icm_seq_run: lane-quad exchange through LDS
#endif
// cooperative-path packet loads / segment stores: plain, or non-temporal
// (streaming: each byte is touched once)
#ifndef ICM_NT
#define ICM_NT 0
#endif
#if ICM_NT & 1
#define ICM_LD(P) __builtin_nontemporal_load(P)
#else
#define ICM_LD(P) (*(P))
#endif
#if ICM_NT & 2
#define ICM_ST(V, P) __builtin_nontemporal_store((V), (P))
#else
#define ICM_ST(V, P) (*(P) = (V))
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
            nx[j] = ICM_LD((gcptr)(cp.in[j] + 64 * (b + 1)));
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
        ICM_ST(sg[j], (gptr)(cp.seg[j] + 64 * b));
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
        nx[j] = ICM_LD((gcptr)(cp.in[j] + 64 * b));
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

// The cooperative steady chunks with a small live set, for 3-4 waves per
// SIMD (ICM_SEQ): per chunk the keystream, then the exchange and store,
// then SHA-1, one after the other, so at most one phase's temporaries are
// live; the other waves of the SIMD fill each phase's LDS / VALU latency.
// Loads and stores are addressed as 32-bit offsets from the (uniform)
// arena bases; only the next chunk's data is held ahead.
template <int S, int NR, bool TAB4, bool AUTH, bool PROTECT, class KEY>
DEV void icm_seq_run(uint32_t &b, uint32_t e, const IcmPkt &p,
                     const CtrCache &C, const KEY &rk, const AesLds &T,
                     uint32_t ks_prev[4], uint32_t hst[5], u32x4 (&prev)[4],
                     const uint8_t *ib, uint8_t *ob, const uint32_t (&io)[4],
                     const uint32_t (&so)[4], uint32_t r0)
{
#if ICM_PIPE
    // keystream one chunk ahead: chunk b+1's AES and chunk b's SHA-1 share
    // a basic block, so one wave mixes LDS-bound and VALU-bound work
    uint32_t ks[4][4];
    coop_keystream<NR, TAB4>(b, p, C, rk, T, ks);
#endif
    for (; b < e; b++) {
        // the chunk's data is in flight during its keystream
        u32x4 v[4];
#pragma unroll
        for (int j = 0; j < 4; j++)
            v[j] = *(gcptr)(ib + (io[j] + 64 * b));
#if !ICM_PIPE
        uint32_t ks[4][4];
        coop_keystream<NR, TAB4>(b, p, C, rk, T, ks);
#endif
        quad_transpose(v);
        uint32_t wv[16];
        if (!PROTECT) {
#pragma unroll
            for (int t = 0; t < 4; t++)
#pragma unroll
                for (int u = 0; u < 4; u++)
                    wv[4 * t + u] = bswap(v[t][u]);
        }
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int u = 0; u < 4; u++)
                v[t][u] ^= u >= S ? ks[t][u - S]
                                  : (t ? ks[t - 1][u - S + 4]
                                       : ks_prev[u - S + 4]);
#pragma unroll
        for (int u = 0; u < 4; u++)
            ks_prev[u] = ks[3][u];
        u32x4 sg[4];
        seg_funnel(prev, v, r0, sg);
#pragma unroll
        for (int t = 0; t < 4; t++)
            prev[t] = v[t];
        quad_transpose(sg);
#pragma unroll
        for (int j = 0; j < 4; j++)
            *(gptr)(ob + (so[j] + 64 * b)) = sg[j];
        if (AUTH && PROTECT) {
#pragma unroll
            for (int t = 0; t < 4; t++)
#pragma unroll
                for (int u = 0; u < 4; u++)
                    wv[4 * t + u] = bswap(prev[t][u]);
        }
#if ICM_PIPE
        if (b + 1 < e)
            coop_keystream<NR, TAB4>(b + 1, p, C, rk, T, ks);
#endif
        if (AUTH)
            sha1_compress(hst, wv);
    }
    // quads 4e - r0 .. 4e - 1 (the head of segment e) are not stored yet
#pragma unroll
    for (int t = 1; t < 4; t++)
        if (4 - (int)r0 <= t)
            *(u32x4 *)(p.out + 16 * (4 * e - 4 + t)) = prev[t];
}

#if ICM_LDSX
// The cooperative steady chunks with the lane-quad exchange done by the LDS
// instead of DPP transposes (64 DPP moves + 64 selects per chunk each way).
// Each wave owns 4 KiB of LDS (xb): one chunk of its 64 packets.
//   in:  4 global_load_lds_dwordx4 (LDS DMA, no VGPRs, no VALU): in
//        instruction j, lane 4m+q reads 16 bytes of the chunk of packet
//        16j+m and the DMA puts them at slot 64j+4m+q; then every lane reads
//        its own packet's four 16-byte pieces (4 ds_read_b128)
//   out: every lane writes its aligned segment's four pieces (4
//        ds_write_b128), lane 4m+q of instruction j reads piece q of the
//        segment of packet 16j+m back (ds_read_b128) and stores it: 64
//        contiguous aligned bytes per quad, as before
// Piece t of the packet of lane L = 4m+j sits in slot 64j + 4m + ((t+m+j)&3):
// the rotation by m + j keeps every ds_read_b128 lane group (16 lanes) and
// every ds_write_b128 group (8 lanes) on distinct banks, and the DMA lanes
// of a quad still read 64 contiguous bytes (in rotated order).
template <int S, int NR, bool TAB4, bool AUTH, bool PROTECT, class KEY>
DEV void icm_ldsx_run(uint32_t &b, uint32_t e, const IcmPkt &p,
                      const CtrCache &C, const KEY &rk, const AesLds &T,
                      uint32_t ks_prev[4], uint32_t hst[5], u32x4 (&prev)[4],
                      const uint8_t *ib, uint8_t *ob, const uint32_t (&ibq)[4],
                      const uint32_t (&so)[4], uint32_t r0, u32x4 *xb)
{
    const uint32_t L = threadIdx.x & 63, m = L >> 2, q = L & 3;
    uint32_t io[4], rs[4], ro[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        io[j] = ibq[j] + 16 * ((q - m - (uint32_t)j) & 3);   // DMA source
        rs[j] = 64 * q + 4 * m + ((j + m + q) & 3);          // own piece j
        ro[j] = 64 * j + 4 * m + ((q + m + (uint32_t)j) & 3);  // store read
    }
    // chunk b's DMA is issued once chunk b-1 has left the buffer, before
    // chunk b-1's SHA-1 and chunk b's AES: both cover its latency
    auto dma = [&](uint32_t c) {
        // the previous chunk's store reads are complete before the DMA
        // overwrites the buffer
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < 4; j++)
            __builtin_amdgcn_global_load_lds(
                (const void __attribute__((address_space(1))) *)(ib + (io[j] + 64 * c)),
                (void __attribute__((address_space(3))) *)(xb + 64 * j), 16, 0,
                0);
    };
    dma(b);
    for (; b < e; b++) {
        uint32_t ks[4][4];
        coop_keystream<NR, TAB4>(b, p, C, rk, T, ks);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        u32x4 v[4];
#pragma unroll
        for (int t = 0; t < 4; t++)
            v[t] = xb[rs[t]];
        uint32_t wv[16];
        if (!PROTECT) {
#pragma unroll
            for (int t = 0; t < 4; t++)
#pragma unroll
                for (int u = 0; u < 4; u++)
                    wv[4 * t + u] = bswap(v[t][u]);
        }
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int u = 0; u < 4; u++)
                v[t][u] ^= u >= S ? ks[t][u - S]
                                  : (t ? ks[t - 1][u - S + 4]
                                       : ks_prev[u - S + 4]);
#pragma unroll
        for (int u = 0; u < 4; u++)
            ks_prev[u] = ks[3][u];
        u32x4 sg[4];
        seg_funnel(prev, v, r0, sg);
#pragma unroll
        for (int t = 0; t < 4; t++) {
            prev[t] = v[t];
            xb[rs[t]] = sg[t];
        }
#pragma unroll
        for (int j = 0; j < 4; j++)
            *(gptr)(ob + (so[j] + 64 * b)) = xb[ro[j]];
        if (b + 1 < e)
            dma(b + 1);
        if (AUTH) {
            if (PROTECT) {
#pragma unroll
                for (int t = 0; t < 4; t++)
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        wv[4 * t + u] = bswap(prev[t][u]);
            }
            sha1_compress(hst, wv);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // quads 4e - r0 .. 4e - 1 (the head of segment e) are not stored yet
#pragma unroll
    for (int t = 1; t < 4; t++)
        if (4 - (int)r0 <= t)
            *(u32x4 *)(p.out + 16 * (4 * e - 4 + t)) = prev[t];
}
#endif

// all 64 lanes active and in the same steady state: the cooperative path
DEV bool wave_uniform(uint32_t x)
{
    return __builtin_amdgcn_ballot_w64(x == (uint32_t)__builtin_amdgcn_readfirstlane(x)) ==
           ~0ull;
}

// per-packet constants from the packet's meta record and header
template <int NR, bool AUTH>
DEV IcmPkt make_pkt(const IcmArgs &A, uint32_t i, const srtp_dev_meta_t &m,
                    const srtp_dev_key_t *key)
{
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

    return p;
}

// one packet, front to back: header chunks, steady payload chunks, tail
// chunks, partial quad, outer hash, tag (srtp.c:2694-2818 protect,
// 2987-3093 unprotect: the tag is compared, the caller decides)
template <int NR, bool TAB4, bool AUTH, bool PROTECT, bool UNIFORM, class KEY>
DEV void icm_packet(const IcmArgs &A, uint32_t i, const AesLds &T, KEY &rk,
                    u32x4 *xb)
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

    IcmPkt p = make_pkt<NR, AUTH>(A, i, m, key);

    uint32_t hst[5];
#pragma unroll
    for (int k = 0; k < 5; k++)
        hst[k] = AUTH ? key->ipad[k] : 0;

    uint32_t ks_prev[4] = { 0, 0, 0, 0 };
    uint32_t tailq[4] = { 0, 0, 0, 0 };
    u32x4 prev[4];   // output quads of the last chunk done
    uint32_t b = 0;
#ifdef ICM_EXP_NOHEAD   // timing experiment only: skip the header chunks
    b = p.bclean;
#endif
    for (; b < p.bclean && b < p.nb; b++)
        icm_chunk<NR, TAB4, AUTH, PROTECT>(b, p, rk, T, ks_prev, hst, tailq,
                                           prev);

    // steady chunks: full chunks whose blocks j = 4b+t-qoff stay in counter
    // epoch 0 (j <= 255, 4 KiB of payload)
    uint32_t se = p.L >> 6;
    se = se < ((256 + p.qoff) >> 2) ? se : ((256 + p.qoff) >> 2);
#ifdef ICM_EXP_NOSTEADY   // timing experiment only: skip the steady chunks
    b = se;
#endif
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
#if ICM_SEQ
        // 32-bit offsets from the arena bases must cover the steady chunks
        const uint8_t *ib = A.in;
        uint8_t *ob = (uint8_t *)((uintptr_t)A.out & ~(uintptr_t)63);
        const uint64_t ioff = (uint64_t)(p.in - ib);
        const uint64_t soff = (uint64_t)(((uintptr_t)p.out & ~(uintptr_t)63) -
                                         (uintptr_t)ob);
        if (coop && __builtin_amdgcn_ballot_w64(ioff + 64 * se < (1ull << 32) &&
                                                soff + 64 * se + 64 <
                                                    (1ull << 32)) == ~0ull) {
            const uint32_t lq = 16 * (threadIdx.x & 3);
            const uint32_t i32 = (uint32_t)ioff, s32 = (uint32_t)soff;
            const uint32_t r0 = (uint32_t)(((uintptr_t)p.out >> 4) & 3);
            const uint32_t io[4] = { qperm<0x00>(i32) + lq, qperm<0x55>(i32) + lq,
                                     qperm<0xAA>(i32) + lq, qperm<0xFF>(i32) + lq };
            const uint32_t so[4] = { qperm<0x00>(s32) + lq, qperm<0x55>(s32) + lq,
                                     qperm<0xAA>(s32) + lq, qperm<0xFF>(s32) + lq };
#if ICM_LDSX
            const uint32_t ibq[4] = { qperm<0x00>(i32), qperm<0x55>(i32),
                                      qperm<0xAA>(i32), qperm<0xFF>(i32) };
#define ICM_RUN(SS)                                                            \
    icm_ldsx_run<SS, NR, TAB4, AUTH, PROTECT>(b, se, p, C, rk, T, ks_prev,     \
                                             hst, prev, ib, ob, ibq, so, r0, xb)
#else
            (void)xb;
#define ICM_RUN(SS)                                                            \
    icm_seq_run<SS, NR, TAB4, AUTH, PROTECT>(b, se, p, C, rk, T, ks_prev, hst, \
                                            prev, ib, ob, io, so, r0)
#endif
            switch (p.s) {
            case 0:
                ICM_RUN(0);
                break;
            case 1:
                ICM_RUN(1);
                break;
            case 2:
                ICM_RUN(2);
                break;
            default:
                ICM_RUN(3);
                break;
            }
#undef ICM_RUN
        } else
#endif
        if (!ICM_SEQ && coop) {
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
#if ICM_SEQ
    // re-derived rather than held in registers across the steady loop
    p = make_pkt<NR, AUTH>(A, i, A.meta[i], key);
#endif
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
    // per-wave exchange buffers of the LDS cooperative path (4 KiB a wave);
    // their first KiB also holds the S-box during the table build
    constexpr int XB = (UNIFORM && NR && ICM_LDSX) ? ICM_THREADS_UNI / 64 * 256
                                                   : 64;
    __shared__ u32x4 s_x[XB];
    if (A.abort && *A.abort)
        return;
    if (NR)
        load_aes_tables<TAB4>(s_tab, (uint32_t *)s_x);
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
        icm_packet<NR, TAB4, AUTH, PROTECT, UNIFORM>(
            A, i, T, rk, s_x + (XB > 64 ? (threadIdx.x >> 6) * 256 : 0));
}

}   // namespace

template <int NR>
int launch_icm_nr(const IcmArgs &A, bool auth, bool prot, int ncu,
                  hipStream_t st)
{
    // persistent grid: one workgroup per CU (128 KiB of tables) for uniform
    // keys, two 512-lane workgroups per CU otherwise
    const bool uni = A.uni != 0xffffffffu;
    const size_t T = uni ? ICM_THREADS_UNI : ICM_THREADS_LANE;
    const size_t wgs = (A.n + T - 1) / T;
    const size_t cap = (size_t)ncu * (uni ? ICM_UNI_WGS_PER_CU : 2);
    const dim3 grid((unsigned)(wgs < cap ? wgs : cap)), block((unsigned)T);
#define ICM_GO(AU, PR)                                                         \
    do {                                                                       \
        if (uni)                                                               \
            hipLaunchKernelGGL((k_icm_hmac<NR, AU, PR, true>), grid, block, 0, \
                               st, A);                                         \
        else                                                                   \
            hipLaunchKernelGGL((k_icm_hmac<NR, AU, PR, false>), grid, block,   \
                               0, st, A);                                      \
    } while (0)
#ifdef ICM_EXP_ONLY   // experiment builds: the bench kernel only
    ICM_GO(true, true);
    (void)auth;
    (void)prot;
#else
    if (auth && prot)
        ICM_GO(true, true);
    else if (auth)
        ICM_GO(true, false);
    else if (prot)
        ICM_GO(false, true);
    else
        ICM_GO(false, false);
#endif
#undef ICM_GO
    HIPCHK(hipGetLastError());
    return 0;
}

template int launch_icm_nr<ICM_NR>(const IcmArgs &, bool, bool, int,
                                   hipStream_t);
