// srtp_icm_wave.hip -- k_icm_wave: the streaming AES-ICM + HMAC-SHA1 protect
// kernel for uniform-key batches (the headline path, BASELINE configs[1]).
//
// Reference semantics: srtp_protect (srtp/srtp.c:2493-2818) through
// srtp_aes_icm_encrypt (crypto/cipher/aes_icm.c:297-414, counter formation
// 236-258) and HMAC-SHA1 (crypto/hash/hmac.c:157-229, sha1.c:91-463), with
// the ROC appended to the authenticated bytes (srtp.c:2726, 2785-2807).
//
// One wave takes a GROUP of 64 consecutive packets.  The group qualifies
// when all 64 packets are to be processed by this kernel variant and agree
// in length and header size (which makes every branch of the chunk loop
// wave-uniform), their payload stays in the first counter epoch (<= 4 KiB),
// the key has no MKI and the packets are 16-byte aligned.  Groups that do
// not qualify are flagged for k_icm_hmac (srtp_icm.hip), which runs next.
//
// Design (DESIGN.md "k_icm_wave"):
//  * AES (T-table, LDS, bank-conflict-free replicas) is LDS-bound and SHA-1
//    is VALU-bound.  The chunk loop keeps the working set <= 128 VGPRs so a
//    1024-lane workgroup runs 4 waves per SIMD: while some waves wait on
//    table reads, others run SHA-1 rounds.
//  * Memory: lane quads move 64 contiguous bytes of one packet per load
//    instruction, stores are whole 64-byte aligned segments (the lane-quad
//    transpose and funnel of srtp_dev_common.h); base addresses are SGPR
//    pairs, per-lane offsets 32-bit.
//  * The packet tail (partial last quad + tag) is written once per packet
//    from a register window with the widest aligned stores.
#include "srtp_dev_common.h"
#include "srtp_gpu_int.h"

#ifndef WAVE_NB
#define WAVE_NB 2   // AES blocks advanced together per round
#endif
#ifndef WAVE_THREADS
#define WAVE_THREADS 768   // 12 waves: 3 per SIMD at <= 168 VGPRs
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

struct WaveArgs {
    IcmArgs A;
    uint8_t *rest;      // per group: 1 = left to k_icm_hmac
    uint32_t *any;      // set to `seq` when some group was left
    uint32_t seq;
    unsigned long long *cnt;   // [0] += groups taken, [1] += groups left
};

// per-lane constants of one packet in the chunk loop
struct WavePkt {
    uint32_t di;        // own packet: input offset from ibase
    uint32_t dob;       // own packet: output segment 0 offset from obase
    uint32_t r0;        // own packet: (out >> 4) & 3
    uint32_t r0s;       // r0 of packet (L & ~3) + j at bits 2j+1:2j
    uint32_t roc;
};

// coop offsets: for j = 0..3 packet (L & ~3) + j's value, + 16 * (L & 3).
// DPP reads another lane's register: call it where every lane of the quad
// is active (uniform control flow), never under a per-lane predicate (a
// masked source lane returns a stale register).
DEV void coop_offs(uint32_t own, uint32_t (&o)[4])
{
    const uint32_t lq16 = 16 * (threadIdx.x & 3);
    o[0] = qperm<0x00>(own) + lq16;
    o[1] = qperm<0x55>(own) + lq16;
    o[2] = qperm<0xAA>(own) + lq16;
    o[3] = qperm<0xFF>(own) + lq16;
}

// readfirstlane of an unsigned word (the builtin returns int: widening its
// result directly would sign-extend)
DEV uint32_t rfl(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}

// keystream of chunk b: counter blocks j = 4b + t - qoff of the cached epoch;
// blocks before the payload (header quads) are zero
template <int NR>
DEV void wave_keystream(uint32_t b, uint32_t qoff, const CtrCache &C,
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
    for (int g = 0; g < 4; g += WAVE_NB) {
        uint32_t jb[WAVE_NB];
#pragma unroll
        for (int j = 0; j < WAVE_NB; j++)
            jb[j] = ((uint32_t)(j0 + g + j) & 0xffu) << 8;
        aes_ctr<WAVE_NB, NR, true>(
            *reinterpret_cast<uint32_t(*)[WAVE_NB][4]>(&ks[g]), jb, C, rk, T);
    }
    if (j0 < 0) {
#pragma unroll
        for (int t = 0; t < 3; t++)
            if (j0 + t < 0)
                ks[t][0] = ks[t][1] = ks[t][2] = ks[t][3] = 0;
    }
}

// The chunk loop of one packet per lane (S = header words mod 4, the
// keystream word shift inside a quad, as a compile-time constant).
//   L   bytes authenticated (header + payload), uniform
//   nb  SHA-1 chunks (data chunks + the message tail), uniform
template <int S, int NR, bool PROTECT>
DEV void wave_chunks(const WavePkt &p, const uint8_t *ibase, uint8_t *obase,
                     uint32_t L, uint32_t qoff, uint32_t nb, const CtrCache &C,
                     const UniKey<NR> &rk, const AesLds &T, uint32_t hst[5],
                     uint32_t &tailw)
{
    const uint32_t nq = (L + 15) >> 4;   // quads holding data
    const uint32_t nfq = L >> 4;         // full data quads (stored in loop)
    const uint32_t lq = threadIdx.x & 3;
    const uint32_t d = L & 15;           // data bytes of the partial quad
    uint32_t ks_prev[4] = { 0, 0, 0, 0 };
    u32x4 prev[4];
#pragma unroll
    for (int t = 0; t < 4; t++)
        prev[t] = u32x4{ 0, 0, 0, 0 };
    u32x4 nx[4];
    {
        // quads past the data are not read: such lanes read the packet's
        // first quad instead (those words never reach an output)
        uint32_t io[4];
        coop_offs(p.di, io);
#pragma unroll
        for (int j = 0; j < 4; j++)
            nx[j] = gload16(ibase, lq < nq ? io[j] : io[j] - 16 * lq);
    }
    for (uint32_t b = 0; b < nb; b++) {
        uint32_t di = p.di, dob = p.dob;
        asm volatile("" : "+v"(di), "+v"(dob));
        uint32_t ks[4][4];
        if (64 * b < L) {
            wave_keystream<NR>(b, qoff, C, rk, T, ks);
        } else {
#pragma unroll
            for (int t = 0; t < 4; t++)
                ks[t][0] = ks[t][1] = ks[t][2] = ks[t][3] = 0;
        }
        u32x4 v[4];
#pragma unroll
        for (int j = 0; j < 4; j++)
            v[j] = nx[j];
        if (b + 1 < nb) {
            // quads past the data are not read (the address falls back to
            // the packet's first quad; those words never reach an output:
            // tail_word replaces them in the SHA-1 tail)
            uint32_t io[4];
            coop_offs(di, io);
            const uint32_t sk = 4 * (b + 1) + lq < nq ? 64 * (b + 1) : 0u;
#pragma unroll
            for (int j = 0; j < 4; j++)
                nx[j] = gload16(ibase, io[j] + sk);
        }
        quad_transpose(v);
        u32x4 o[4];
        uint32_t w[16];
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t k = u >= S ? ks[t][u - S]
                                          : (t ? ks[t - 1][u - S + 4]
                                               : ks_prev[u - S + 4]);
                o[t][u] = v[t][u] ^ k;
                w[4 * t + u] = bswap(PROTECT ? o[t][u] : v[t][u]);
            }
#pragma unroll
        for (int u = 0; u < 4; u++)
            ks_prev[u] = ks[3][u];
        // the partial last quad: its whole words now, the last partial
        // word with the tag after the loop
        if (b == (nfq >> 2) && d) {
            const uint32_t tt = nfq & 3;
            uint32_t pq[4];
#pragma unroll
            for (int u = 0; u < 4; u++)
                pq[u] = tt == 0 ? o[0][u]
                                : tt == 1 ? o[1][u]
                                          : tt == 2 ? o[2][u] : o[3][u];
            uint8_t *dst = obase + dob + 16 * (nfq + p.r0);
#pragma unroll
            for (int u = 0; u < 3; u++)
                if ((uint32_t)(4 * u + 4) <= d)
                    *(uint32_t *)(dst + 4 * u) = pq[u];
            tailw = (d >> 2) == 0 ? pq[0]
                                  : (d >> 2) == 1 ? pq[1]
                                                  : (d >> 2) == 2 ? pq[2] : pq[3];
        }
        // aligned segment b = quads [4b - r0, 4b + 4 - r0) of the packet
        u32x4 sg[4];
        seg_funnel(prev, o, p.r0, sg);
#pragma unroll
        for (int t = 0; t < 4; t++)
            prev[t] = o[t];
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
        if (64 * b + 64 > L) {
            // message tail: ROC, 0x80, zero padding, bit length
            // (sha1.c srtp_sha1_final; hmac.c:181-229)
#pragma unroll
            for (int g = 0; g < 16; g++)
                w[g] = tail_word(w[g], (int)L - (int)(64 * b + 4 * g), p.roc);
            if (b == nb - 1) {
                w[14] = 0;
                w[15] = (64 + L + 4) * 8;
            }
        }
        sha1_compress(hst, w);
    }
    // segment nb: its quads below 4 * nb (r0 of them) are the packet's last
    const uint32_t b = nb;
    u32x4 sg[4];
    const u32x4 z[4] = { { 0, 0, 0, 0 }, { 0, 0, 0, 0 }, { 0, 0, 0, 0 },
                         { 0, 0, 0, 0 } };
    seg_funnel(prev, z, p.r0, sg);
    quad_transpose(sg);
    uint32_t so[4];
    coop_offs(p.dob, so);
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

template <int NR, bool AUTH, bool PROTECT>
__global__ __launch_bounds__(WAVE_THREADS) void k_icm_wave(WaveArgs W)
{
    const IcmArgs &A = W.A;
    __shared__ u32x4 s_tab[AES_TAB4_BYTES / 16];
    if (A.abort && *A.abort)
        return;
    load_aes_tables<true>(s_tab);
    __syncthreads();
    const AesLds T = make_aes_lds(s_tab);
    const srtp_dev_key_t *key = A.keys + A.uni;
    UniKey<NR> rk;
    rk.load(key);
    const uint32_t tag_len = rfl(key->tag_len);
    const bool key_ok = rfl(key->conf) != 0 &&
                        rfl(key->mki_size) == 0 &&
                        tag_len <= 20;
    constexpr uint32_t VID = 8u + 2u * ((NR - 8) / 2) + (AUTH ? 1u : 0u);

    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lq = lane & 3;
    const uint32_t ngroups = (A.n + 63) >> 6;
    const uint32_t wpb = blockDim.x >> 6;
    uint32_t n_take = 0, n_left = 0;
    for (uint32_t g = blockIdx.x * wpb + (threadIdx.x >> 6); g < ngroups;
         g += gridDim.x * wpb) {
        // lane L takes packet 16 * (L & 3) + (L >> 2) of the group: lane
        // quad m holds packets m, 16 + m, 32 + m, 48 + m
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
        // the group's uniform quantities and the per-lane checks
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
                        SRTP_META_ENC_START(m.info) == es && ((ia | oa) & 15) == 0 &&
                        di < 0xffff0000ull && dob < 0xffff0000ull;
        const bool take = key_ok && es >= 12 && L >= es && L - es <= 4096 &&
                          __builtin_amdgcn_ballot_w64(ok) == ~0ull;
        if (lane == 0) {
            W.rest[g] = take ? 0 : 1;
            if (!take)
                *W.any = W.seq;
        }
        if (!take) {
            n_left++;
            continue;
        }
        n_take++;

        // key fields used once per packet: re-read here (an opaque copy of
        // the pointer keeps them out of the chunk loop's SGPR budget)
        const srtp_dev_key_t *kp = key;
        asm volatile("" : "+s"(kp));
        uint32_t salt[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
            salt[k] = rfl(kp->salt[k]);
        const uint8_t *ibase = (const uint8_t *)(uintptr_t)ib;
        uint8_t *obase = (uint8_t *)(uintptr_t)ob;
        WavePkt p;
        p.roc = m.roc;
        p.r0 = (uint32_t)(oa >> 4) & 3u;
        p.di = (uint32_t)di;
        p.dob = (uint32_t)dob;
        p.r0s = qperm<0x00>(p.r0) | (qperm<0x55>(p.r0) << 2) |
                (qperm<0xAA>(p.r0) << 4) | (qperm<0xFF>(p.r0) << 6);

        // counter block (little-endian words), block counter in bytes 14..15
        // (aes_icm.c:236-258 IV formation, srtp.c:2694-2707)
        const uint8_t *pin = (const uint8_t *)(uintptr_t)ia;
        const uint32_t w0 = *(const uint32_t *)pin;
        const uint32_t seq = bswap(w0) & 0xffffu;
        uint32_t cb[4];
        cb[0] = salt[0];
        cb[1] = salt[1] ^ *(const uint32_t *)(pin + 8);   // SSRC bytes
        cb[2] = salt[2] ^ bswap(m.roc);
        cb[3] = salt[3] ^ (seq >> 8) ^ ((seq & 0xffu) << 8);
        const CtrCache C = ctr_cache<NR, true>(cb, rk, T);

        uint32_t hst[5];
#pragma unroll
        for (int k = 0; k < 5; k++)
            hst[k] = rfl(kp->ipad[k]);
        uint32_t tailw = 0;
        const uint32_t hw = es >> 2, qoff = hw >> 2;
        const uint32_t nb = ((L + 12) >> 6) + 1;
        switch (hw & 3) {
        case 0:
            wave_chunks<0, NR, PROTECT>(p, ibase, obase, L, qoff, nb, C, rk, T,
                                        hst, tailw);
            break;
        case 1:
            wave_chunks<1, NR, PROTECT>(p, ibase, obase, L, qoff, nb, C, rk, T,
                                        hst, tailw);
            break;
        case 2:
            wave_chunks<2, NR, PROTECT>(p, ibase, obase, L, qoff, nb, C, rk, T,
                                        hst, tailw);
            break;
        default:
            wave_chunks<3, NR, PROTECT>(p, ibase, obase, L, qoff, nb, C, rk, T,
                                        hst, tailw);
            break;
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
        const srtp_dev_key_t *kq = key;
        asm volatile("" : "+s"(kq));
        uint32_t oh[5];
#pragma unroll
        for (int k = 0; k < 5; k++)
            oh[k] = rfl(kq->opad[k]);
        sha1_compress(oh, ow);

        // the tag at L (srtp.c:2809-2815), merged with the packet's last
        // partial data word: window words from byte 4 * (L / 4)
        const uint32_t e = L & 3;
        uint32_t tw[6];
#pragma unroll
        for (int k = 0; k < 5; k++)
            tw[k] = bswap(oh[k]);
        tw[5] = 0;
        uint32_t win[6];
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const uint32_t lo = k ? tw[k - 1] : 0u;
            win[k] = e ? (uint32_t)((((uint64_t)tw[k] << 32) | lo) >> (32 - 8 * e))
                       : tw[k];
        }
        if (e)
            win[0] |= tailw & (0xffffffffu >> (32 - 8 * e));
        store_stream<6>((uint8_t *)(uintptr_t)(oa + (L & ~3u)), win,
                        e + (AUTH ? tag_len : 0));
    }
    if (lane == 0 && (n_take | n_left)) {
        atomicAdd(&W.cnt[0], (unsigned long long)n_take);
        atomicAdd(&W.cnt[1], (unsigned long long)n_left);
    }
}

}   // namespace

int launch_icm_wave(srtp_gpu_t *g, IcmArgs &A, int nr, bool auth, bool prot,
                    hipStream_t st)
{
    if (!prot || !auth || nr != 10 || A.n < 64 || A.uni == 0xffffffffu ||
        g->wave_off)
        return 0;
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
    WaveArgs W;
    W.A = A;
    W.rest = g->d_rest;
    W.any = g->d_any;
    W.cnt = g->d_wave_cnt;
    W.seq = ++g->wave_seq;
    if (W.seq == 0)
        W.seq = ++g->wave_seq;
    const size_t wpb = WAVE_THREADS / 64;
    const size_t wgs = (ngroups + wpb - 1) / wpb;
    const size_t cap = (size_t)g->ncu;
    hipLaunchKernelGGL((k_icm_wave<10, true, true>),
                       dim3((unsigned)(wgs < cap ? wgs : cap)),
                       dim3(WAVE_THREADS), 0, st, W);
    HIPCHK(hipGetLastError());
    A.rest = g->d_rest;
    A.any = g->d_any;
    A.any_seq = W.seq;
    return 1;
}
