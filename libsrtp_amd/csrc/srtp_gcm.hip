// srtp_gcm.hip -- k_gcm: AES-GCM seal / open for SRTP AEAD protect and
// unprotect (srtp/srtp.c:2088-2267, 2276-2491) with the semantics of
// libsrtp's OpenSSL EVP backend (crypto/cipher/aes_gcm_ossl.c:214-389):
// IV = (00 00 || SSRC || ROC || SEQ) ^ salt12, AAD = the RTP header, CTR from
// inc32(J0), tag = E(J0) ^ GHASH, 8 or 16 bytes.  One lane per packet.
//
// Compiled once per AES round count: -DGCM_NR=10 or 14.
#include "srtp_dev_common.h"
#include "srtp_gpu_int.h"
#include "srtp_fused.h"

#ifndef GCM_NR
#error "GCM_NR (10 or 14) must be defined"
#endif

namespace {

#ifndef GCM_PF
#define GCM_PF 2   // 64-byte payload chunks loaded ahead of their use
#endif
// uniform-key batches: the four AES tables (128 KiB) with 8 per-position
// GHASH tables (32 KiB, GhPos8); per-lane keys: (T0, T1) and each key's
// 4-bit table in global memory (GhNib4)

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
template <int NR>
constexpr uint32_t gcm_vid()
{
    return 16u + 2u * ((NR - 8) / 2);
}

// m: the packet's descriptor; in_off / out_off its offsets.  UNIFORM: the
// key of slot uslot is in rk and G already (the batch's, or the wave's in
// the bucketed form); else the packet's key is loaded here
template <int NR, bool PROTECT, bool UNIFORM, bool TAB4, class GT, class KEY>
DEV void gcm_packet(const GcmArgs &A, const srtp_dev_meta_t &m,
                    uint64_t in_off, uint64_t out_off, uint32_t i,
                    const AesLds &T, GT &G, KEY &rk, uint32_t uslot)
{
    constexpr uint32_t VID = gcm_vid<NR>();
    if (SRTP_META_STATUS(m.info) || SRTP_META_VARIANT(m.info) != VID)
        return;
    const uint32_t slot = UNIFORM ? uslot : m.key;
    const srtp_dev_key_t *key = A.keys + slot;
    if constexpr (!UNIFORM) {
        rk.reload(A.keys, slot);
        G.load(A.ghash, key->ghash_slot);
    }

    const uint8_t *in = A.in + in_off;
    uint8_t *out = A.out + out_off;
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
        const CtrCache C = ctr_cache<NR, TAB4>(cc, rk, T);
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
                aes_ctr<2, NR, TAB4>(
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
        aes_block<NR, TAB4>(k0, k1, k2, k3, rk, T);
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
    aes_block<NR, TAB4>(e0, e1, e2, e3, rk, T);
    uint32_t tagw[4] = { bswap(x[0]) ^ e0, bswap(x[1]) ^ e1, bswap(x[2]) ^ e2,
                         bswap(x[3]) ^ e3 };   // little-endian words of tag
    if (PROTECT) {
        uint8_t *tp = pout + P;
        store_tag(tp, tagw, tag_len);
        for (uint32_t u = 0; u < mki_size; u++)
            tp[tag_len + u] = key->mki[u];
    } else {
        A.auth_ok[i] = tag_diff(pin + P, tagw, tag_len) == 0;
    }
}

// Uniform keys: four AES tables + per-position GHASH tables (160 KiB, one
// 512-lane workgroup per CU); per-lane keys: (T0, T1) (64 KiB) + each
// lane's 4-bit GHASH table (256 B, GhNib4L), 256 lanes: one workgroup of
// 128 KiB per CU.  Persistent grid.
#ifndef GCM_THREADS_N
#define GCM_THREADS_N 512
#endif
constexpr int GCM_THREADS = GCM_THREADS_N;
#ifndef GCM_LANE_THREADS_N
#define GCM_LANE_THREADS_N 256
#endif
constexpr int GCM_LANE_THREADS = GCM_LANE_THREADS_N;

// FUSED (in place): the order-free classification in the kernel
// (srtp_fused.h; srtp_prepass.hip pp_protect_fused / pp_unprotect_fused), as
// k_icm_hmac does it for AES-ICM -- with per-lane keys, or one key for every
// stream (a template session's clones) and its LDS tables
template <int NR, bool PROTECT, bool UNIFORM, bool FUSED = false>
__global__ __launch_bounds__(UNIFORM ? GCM_THREADS : GCM_LANE_THREADS)
void k_gcm(GcmArgs A)
{
    constexpr bool TAB4 = UNIFORM;
    constexpr int GH8 = 256 * 16 * 8;   // the per-position GHASH tables
    constexpr int GHL = GCM_LANE_THREADS * 256;   // the lanes' 4-bit tables
    __shared__ u32x4 s_tab[(TAB4 ? AES_TAB4_BYTES + GH8
                                 : AES_TAB2_BYTES + GHL) / 16];
    if (A.abort && *A.abort)
        return;
    if constexpr (TAB4) {
        // the S-box row of the table build sits where the GHASH table goes
        uint32_t *t0 = (uint32_t *)((char *)s_tab + AES_TAB4_BYTES);
        load_aes_tables<true>(s_tab, t0);
        __syncthreads();
        const u32x4 *src =
            (const u32x4 *)(A.ghash + 1024 * A.keys[A.uni].ghash_slot);
        u32x4 *dst = (u32x4 *)((char *)s_tab + AES_TAB4_BYTES);
        // per-position tables: entry b of table t = M[b] * x^(8t)
        for (int b = threadIdx.x; b < 256; b += blockDim.x) {
            u32x4 z = src[ghash_nswap(b)];
#pragma unroll
            for (int t = 0; t < 8; t++) {
                dst[b * 8 + t] = z;
                z = ghash_mulx8(z);
            }
        }
    } else {
        // the S-box row of the table build sits where the lane tables go
        load_aes_tables<false>(s_tab,
                               (uint32_t *)((char *)s_tab + AES_TAB2_BYTES));
    }
    __syncthreads();
    const char *lds = (const char *)s_tab;
    const AesLds T = make_aes_lds(s_tab);

    typename std::conditional<UNIFORM, UniKey<NR>, LaneKey<NR>>::type rk;
    if (UNIFORM)
        rk.load(A.keys + A.uni);
    const uint32_t stride = gridDim.x * blockDim.x;
    FzLane z;
    if constexpr (FUSED) {
        z.ssrc = 0;
        z.sid = FZ_NOCHAIN;
        z.run_sid = FZ_NOCHAIN;
        z.run_cnt = 0;
        z.run_max = 0;
        z.run_min = ~0ull;
        z.run_cmax = 0;
        z.bw_idx = 0;
        z.bw_bits = 0;
    }
    constexpr uint32_t vid = gcm_vid<NR>();
    // one fused packet: classified here, then sealed / opened
    auto fused_packet = [&](uint32_t i, auto &G) {
        // fused batches are in place: one offset
        const uint64_t off = A.in_off[i];
        const GlbSrc S{ A.in + off };
        const uint32_t len = A.fz.in_len[i], cap = A.fz.cap[i];
        if constexpr (PROTECT) {
            const srtp_dev_meta_t m =
                fz_classify(A, i, z, vid, off, len, cap, S);
            gcm_packet<NR, PROTECT, UNIFORM, TAB4>(A, m, off, off, i, T, G,
                                                   rk, A.uni);
        } else {
            uint64_t e;
            uint32_t sid;
            const srtp_dev_meta_t m =
                fzu_classify(A, i, z, vid, off, len, cap, S, e, sid);
            gcm_packet<NR, PROTECT, UNIFORM, TAB4>(A, m, off, off, i, T, G,
                                                   rk, A.uni);
            if (sid != FZ_NOCHAIN)
                fzu_verdict(A, i, z, m, e, sid, A.auth_ok[i] != 0);
        }
    };
    if constexpr (TAB4) {
        GhPos8 G;
        G.init(lds, (uint32_t)AES_TAB4_BYTES, threadIdx.x);
        if constexpr (FUSED) {
            for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < A.n;
                 i += stride)
                fused_packet(i, G);
            fz_flush<PROTECT>(A.fz, z);
            return;
        }
        if (A.ch.st) {
            // one stream in order (IcmChain, srtp_fused.h inorder_meta)
            const srtp_dev_stream_t S = *A.ch.st;
            uint32_t seq0;
            uint64_t e0;
            const bool e0ok = srtp_inorder_head(S, A.in + A.in_off[0],
                                                !PROTECT, seq0, e0);
            for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < A.n;
                 i += stride) {
                const uint64_t off = A.in_off[i];
                gcm_packet<NR, PROTECT, UNIFORM, true>(
                    A, inorder_meta<!PROTECT>(A, i, off, S, seq0, e0, e0ok),
                    off, A.out_off[i], i, T, G, rk, A.uni);
            }
            return;
        }
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < A.n;
             i += stride)
            gcm_packet<NR, PROTECT, UNIFORM, true>(A, A.meta[i], A.in_off[i],
                                                   A.out_off[i], i, T, G, rk, A.uni);
        return;
    }
    GhNib4L G;   // the lane's copy of its packet's key table
    G.t = (LdsQuad)((char *)s_tab + AES_TAB2_BYTES + 256 * threadIdx.x);
    G.rot = threadIdx.x & 15u;
    G.slot = 0xffffffffu;
    if constexpr (FUSED) {
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < A.n;
             i += stride)
            fused_packet(i, G);
        fz_flush<PROTECT>(A.fz, z);
        return;
    }
    if (A.rec) {   // key buckets: the records of streams with few packets
        const uint32_t end = A.range[1];
        for (uint32_t pos = A.range[0] + blockIdx.x * blockDim.x + threadIdx.x;
             pos < end; pos += stride) {
            const srtp_dev_rec_t r = A.rec[pos];
            gcm_packet<NR, PROTECT, UNIFORM, false>(
                A, r.meta, r.in_off, r.out_off, PROTECT ? 0u : A.rec_idx[pos],
                T, G, rk, A.uni);
        }
        return;
    }
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < A.n;
         i += stride)
        gcm_packet<NR, PROTECT, UNIFORM, false>(A, A.meta[i], A.in_off[i],
                                                A.out_off[i], i, T, G, rk, A.uni);
}

// Shoup's 8-bit table of one key in LDS (ghash_mul's TAB): the 16 lookups
// of a multiply depend only on X, so they go out together
typedef const u32x4 __attribute__((address_space(3))) *lds_u32x4;
struct GhLdsShoup {
    lds_u32x4 g;
    DEV u32x4 get(uint32_t w, int k) const   // byte k of BE word w
    {
        return g[(w >> (24 - 8 * k)) & 0xffu];
    }
};

// Key buckets (srtp_prepass.hip bucket_pass): the 64 records of a wave group
// belong to one stream, so one key -- its schedule in SGPRs (UniKey) and its
// Shoup table copied into the wave's 4 KiB of LDS, where the per-lane form
// reads every packet's table from global memory (each of 64k keys' tables
// evicted from L2 between a lane's multiplies).  The four AES tables as in
// the uniform form: 128 KiB + 8 waves x 4 KiB = the 160 KiB of a CU.
template <int NR, bool PROTECT>
__global__ __launch_bounds__(GCM_THREADS) void k_gcm_bk(GcmArgs A)
{
    constexpr uint32_t WAVES = GCM_THREADS / 64;
    __shared__ u32x4 s_tab[(AES_TAB4_BYTES + WAVES * 4096) / 16];
    if (A.abort && *A.abort)
        return;
    // the S-box row of the table build sits where the GHASH tables go
    load_aes_tables<true>(s_tab, (uint32_t *)((char *)s_tab + AES_TAB4_BYTES));
    __syncthreads();
    const AesLds T = make_aes_lds(s_tab);
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    u32x4 *gtab = (u32x4 *)((char *)s_tab + AES_TAB4_BYTES + 4096 * wv);
    GhLdsShoup G;
    G.g = (lds_u32x4)gtab;
    constexpr uint32_t vid = gcm_vid<NR>();
    const uint32_t end = A.range[1], nw = gridDim.x * WAVES;
    for (uint32_t g = blockIdx.x * WAVES + wv; A.range[0] + 64 * g < end;
         g += nw) {
        const uint32_t g0 = A.range[0] + 64 * g;
        const uint32_t info0 =
            __builtin_amdgcn_readfirstlane(A.rec[g0].meta.info);
        if (SRTP_META_STATUS(info0) || SRTP_META_VARIANT(info0) != vid)
            continue;   // an empty group, or another kernel's stream
        const uint32_t slot =
            __builtin_amdgcn_readfirstlane(A.rec[g0].meta.key);
        UniKey<NR> rk;
        rk.load(A.keys + slot);
        // arena entry q holds M[ghash_nswap(q)]; this wave's previous group
        // finished its reads first (a wave's LDS operations run in order)
        const u32x4 *src =
            (const u32x4 *)(A.ghash + 1024 * A.keys[slot].ghash_slot);
        for (uint32_t q = lane; q < 256; q += 64)
            gtab[ghash_nswap(q)] = src[q];
        __builtin_amdgcn_wave_barrier();
        const uint32_t pos = g0 + lane;
        if (pos < end) {
            const srtp_dev_rec_t r = A.rec[pos];
            gcm_packet<NR, PROTECT, true, true>(
                A, r.meta, r.in_off, r.out_off, PROTECT ? 0u : A.rec_idx[pos],
                T, G, rk, slot);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

}   // namespace

template <int NR>
int launch_gcm_nr(const GcmArgs &A, bool prot, int ncu, hipStream_t st)
{
    if (A.rec) {
        // key buckets: the wave-aligned groups with a key per wave, then
        // the streams with few packets with a key per lane (their range)
        GcmArgs L = A;
        L.range = A.range + 2;
        const dim3 grid((unsigned)ncu), block(GCM_THREADS),
            lblock(GCM_LANE_THREADS);
        if (prot) {
            hipLaunchKernelGGL((k_gcm_bk<NR, true>), grid, block, 0, st, A);
            hipLaunchKernelGGL((k_gcm<NR, true, false>), grid, lblock, 0, st,
                               L);
        } else {
            hipLaunchKernelGGL((k_gcm_bk<NR, false>), grid, block, 0, st, A);
            hipLaunchKernelGGL((k_gcm<NR, false, false>), grid, lblock, 0, st,
                               L);
        }
        HIPCHK(hipGetLastError());
        return 0;
    }
    // persistent grid: one workgroup per CU (160 KiB of tables for uniform
    // keys, 128 KiB with 256 lanes otherwise)
    const bool uni = A.uni != 0xffffffffu;
    const size_t bt = uni ? GCM_THREADS : GCM_LANE_THREADS;
    const size_t wgs = (A.n + bt - 1) / bt;
    const size_t cap = (size_t)ncu;
    const dim3 grid((unsigned)(wgs < cap ? wgs : cap)), block((unsigned)bt);
    if (A.fused && uni && prot)
        hipLaunchKernelGGL((k_gcm<NR, true, true, true>), grid, block, 0, st,
                           A);
    else if (A.fused && uni)
        hipLaunchKernelGGL((k_gcm<NR, false, true, true>), grid, block, 0, st,
                           A);
    else if (A.fused && prot)
        hipLaunchKernelGGL((k_gcm<NR, true, false, true>), grid, block, 0, st,
                           A);
    else if (A.fused)
        hipLaunchKernelGGL((k_gcm<NR, false, false, true>), grid, block, 0, st,
                           A);
    else if (uni && prot)
        hipLaunchKernelGGL((k_gcm<NR, true, true>), grid, block, 0, st, A);
    else if (uni)
        hipLaunchKernelGGL((k_gcm<NR, false, true>), grid, block, 0, st, A);
    else if (prot)
        hipLaunchKernelGGL((k_gcm<NR, true, false>), grid, block, 0, st, A);
    else
        hipLaunchKernelGGL((k_gcm<NR, false, false>), grid, block, 0, st, A);
    HIPCHK(hipGetLastError());
    return 0;
}

template int launch_gcm_nr<GCM_NR>(const GcmArgs &, bool, int, hipStream_t);
