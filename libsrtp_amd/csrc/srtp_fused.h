// srtp_fused.h -- the order-free pre-pass's per-packet classification done
// inside the crypto kernels (k_icm_hmac / k_icm_stg in srtp_icm.hip, k_gcm
// in srtp_gcm.hip): header parse, stream lookup with a per-lane cache, the
// checks of srtp_host.c pre_protect / un_static, the index guessed from the
// stored index, and the per-stream aggregates the pre-pass checks after the
// kernel (srtp_prepass.hip pp_protect_fused / pp_unprotect_fused).
// ARGS: IcmArgs or GcmArgs (members fz, keys).
#pragma once

#include "srtp_dev_common.h"
#include "srtp_gpu_int.h"

namespace {

// The order-free protect pre-pass's classification of packet i inside the
// crypto kernel (IcmFused; srtp_prepass.hip k_pp_classify restated): header
// parse (the packet's first line, which chunk 0 reads again from cache),
// stream lookup, the checks of srtp_host.c pre_protect (srtp.c:2515-2600),
// the index guessed from the stream's stored index (rdbx.c:112-145), the
// descriptor, and the stream's packet count and highest index -- a wave's
// lanes of one stream merged by ballots before their atomics.  In-place
// packets save the bytes their tag will overwrite.
constexpr uint32_t FZ_NOCHAIN = 0xffffffffu;
// srtp_prepass.hip AB_* bits
constexpr uint32_t FZ_AB_UNKNOWN = 1, FZ_AB_INELIGIBLE = 2, FZ_AB_ORDER = 8,
                   FZ_AB_STATIC = 16, FZ_AB_MKI = 32;

// What a lane keeps between its packets: the last stream it looked up
// (a lane's packets of a batch are often one stream's: the persistent grid's
// stride is a multiple of the stream count in round-robin batches), and the
// running counts / highest / lowest index of its current stream, flushed
// with one atomic triple when the stream changes and at the end.  The
// per-packet atomics stalled the crypto behind them (an atomic stays in
// vmcnt for ~3000 cycles under load, MI355X_MICROARCH.md); the one
// per-packet atomic left, the bitmap bit, returns nothing and is not waited
// on.
// Unprotect (the receive side's order-free form, pp_unprotect_fused): the
// run counts authenticated packets (low 32 bits) and candidates (high), the
// highest authenticated index (run_max), the lowest and highest candidate
// index (run_min, run_cmax); candidates set a bit in `bmap`, authenticated
// packets one in `bmap2`.
struct FzLane {
    uint32_t ssrc, sid;            // cached lookup (sid ~0: none)
    uint32_t key, variant, flags, trailer, dir;
    uint32_t boff, bmask;          // bitmap word offset, M - 1
    uint32_t mki;                  // unprotect: srtp_dev_stream_t.mki
    uint64_t index;
    uint32_t run_sid;              // current run (run_sid ~0: none)
    uint64_t run_cnt;              // protect: packets | chain packets << 32
    uint64_t run_max, run_min;
    uint64_t run_cmax;             // unprotect only
    uint32_t bw_idx, bw_bits;      // protect: pending bits of one bitmap word
};

template <bool PROTECT>
DEV void fz_flush(const IcmFused &F, FzLane &z)
{
    if (PROTECT && z.bw_bits) {
        atomicOr(&F.bmap[z.bw_idx], z.bw_bits);
        z.bw_bits = 0;
    }
    if (z.run_sid != FZ_NOCHAIN) {
        atomicAdd(&F.cnt[z.run_sid], (unsigned long long)z.run_cnt);
        if (PROTECT) {
            if (z.run_cnt >> 32) {
                atomicMax(&F.new_index[z.run_sid],
                          (unsigned long long)z.run_max);
                atomicMin(&F.emin[z.run_sid], (unsigned long long)z.run_min);
            }
        } else {
            if (z.run_cnt >> 32) {
                atomicMax(&F.hicand[z.run_sid], (unsigned long long)z.run_cmax);
                atomicMin(&F.emin[z.run_sid], (unsigned long long)z.run_min);
            }
            if ((uint32_t)z.run_cnt)
                atomicMax(&F.new_index[z.run_sid],
                          (unsigned long long)z.run_max);
        }
    }
    z.run_sid = FZ_NOCHAIN;
    z.run_cnt = 0;
    z.run_max = 0;
    z.run_min = ~0ull;
    z.run_cmax = 0;
}

// unprotect: candidate e of stream sid
DEV void fzu_cand(const IcmFused &F, FzLane &z, uint32_t sid, uint64_t e)
{
    if (sid != z.run_sid) {
        fz_flush<false>(F, z);
        z.run_sid = sid;
    }
    z.run_cnt += 1ull << 32;
    z.run_cmax = e > z.run_cmax ? e : z.run_cmax;
    z.run_min = e < z.run_min ? e : z.run_min;
    const uint32_t r = (uint32_t)e & z.bmask;
    atomicOr(&F.bmap[z.boff + (r >> 5)], 1u << (r & 31));
}

// ... which authenticated (same run: right after its fzu_cand)
DEV void fzu_auth(const IcmFused &F, FzLane &z, uint64_t e)
{
    z.run_cnt += 1;
    z.run_max = e > z.run_max ? e : z.run_max;
    const uint32_t r = (uint32_t)e & z.bmask;
    atomicOr(&F.bmap2[z.boff + (r >> 5)], 1u << (r & 31));
}

// a packet of stream sid; chain packets (index e) also set their bitmap bit
DEV void fz_count(const IcmFused &F, FzLane &z, uint32_t sid, bool chain,
                  uint64_t e)
{
    if (sid != z.run_sid) {
        fz_flush<true>(F, z);
        z.run_sid = sid;
    }
    z.run_cnt += chain ? 1ull | (1ull << 32) : 1ull;
    if (chain) {
        z.run_max = e > z.run_max ? e : z.run_max;
        z.run_min = e < z.run_min ? e : z.run_min;
        // a lane's packets of one stream are often a few indices apart:
        // their bits are merged per bitmap word before the atomic
        const uint32_t r = (uint32_t)e & z.bmask;
        const uint32_t w = z.boff + (r >> 5);
        if (w != z.bw_idx) {
            if (z.bw_bits)
                atomicOr(&F.bmap[z.bw_idx], z.bw_bits);
            z.bw_idx = w;
            z.bw_bits = 0;
        }
        z.bw_bits |= 1u << (r & 31);
    }
}

// w = the tn (<= 16) bytes at t, little-endian words; bytes past tn are
// whatever memory holds
DEV void fz_tail_save(const uint8_t *t, uint32_t tn, u32x4 &w)
{
    const uintptr_t a8 = (uintptr_t)t & ~(uintptr_t)7;
    const uint32_t o = (uint32_t)((uintptr_t)t & 7), end = o + tn;
    uint32_t W[6] = { 0, 0, 0, 0, 0, 0 };
    if (tn == 0) {
        w = u32x4{ 0, 0, 0, 0 };
        return;
    }
    if (end > 8) {
        const u32x4 v = *(const u32x4a4 *)a8;
        W[0] = v[0]; W[1] = v[1]; W[2] = v[2]; W[3] = v[3];
    } else {
        const uint2 v = *(const uint2 *)a8;
        W[0] = v.x; W[1] = v.y;
    }
    if (end > 16) {
        const uint2 v = *(const uint2 *)(a8 + 16);
        W[4] = v.x; W[5] = v.y;
    }
    const bool q = o >= 4;
    const uint32_t r = o & 3;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t lo = q ? W[k + 1] : W[k];
        const uint32_t hi = q ? W[k + 2] : W[k + 1];
        w[k] = __builtin_amdgcn_alignbyte(hi, lo, r);
    }
}

// the lane's stream for SSRC ssrc: its cached one, else a map lookup and
// the stream record's fields
DEV void fz_lookup(const IcmFused &F, FzLane &z, uint32_t ssrc)
{
    if (ssrc == z.ssrc && z.sid != FZ_NOCHAIN)
        return;
    z.ssrc = ssrc;
    z.sid = srtp_map_lookup(F.hkey, F.hval, F.hmask, ssrc);
    if (z.sid == FZ_NOCHAIN)
        return;
    const srtp_dev_stream_t S = F.st[z.sid];
    z.key = S.key;
    z.variant = S.variant;
    z.flags = S.flags;
    z.trailer = S.trailer;
    z.dir = S.dir;
    z.index = S.index;
    z.boff = 2 * S.win_off;
    z.mki = S.mki;
    z.bmask = (S.win_bits > 32 ? 2u << (31 - __clz(S.win_bits - 1)) : 32u) - 1;
}

// `vid`: the kernel variant this launch runs (every eligible stream's, by
// fused_ok); a packet of another variant (only an ineligible stream can
// have one) is not encrypted here, so it must not count as done: the
// batch is declined without it
// `S`: where the packet's bytes are read (GlbSrc: the arena, StgImg: the
// wave's staged image); off / len / cap: the packet's offset, length and
// capacity, loaded by the caller
template <class ARGS, class SRC>
DEV srtp_dev_meta_t fz_classify(const ARGS &A, uint32_t i, FzLane &z,
                                uint32_t vid, uint64_t off, uint32_t len,
                                uint32_t cap, const SRC &S)
{
    const IcmFused &F = A.fz;
    const srtp_dev_hdr_t h = S.hdr(off, len);
    uint32_t code = 0, key = FZ_NOCHAIN, ab = 0;
    uint64_t e = 0;
    srtp_dev_meta_t m;
    m.key = 0;
    m.roc = 0;
    m.len = 0;
    m.info = 0xff0000u;   // no crypto
    if (h.enc_start >> 24) {
        code = h.enc_start >> 24;   // header does not parse: no stream touched
    } else {
        fz_lookup(F, z, h.ssrc);
        const uint32_t sid = z.sid;
        if (sid == FZ_NOCHAIN) {
            ab |= FZ_AB_UNKNOWN;    // template clone: host
        } else if (z.variant != vid) {
            ab |= FZ_AB_INELIGIBLE;
        } else {
            // an ineligible stream of this variant (its trailer may exceed
            // the 16 saved bytes) is neither encrypted nor recorded as done:
            // the batch is declined, and its bytes stay as they were
            const bool inel =
                !(z.flags & SRTP_DS_ELIGIBLE) || (z.dir & SRTP_DIR_RX);
            if (inel)
                ab |= FZ_AB_INELIGIBLE;
            if (cap < len + z.trailer) {
                code = 28;           // srtp_err_status_buffer_small
                fz_count(F, z, sid, false, 0);
            } else if (h.enc_start > len) {
                code = 21;           // srtp_err_status_parse_err
                fz_count(F, z, sid, false, 0);
            } else {
                key = inel ? FZ_NOCHAIN : sid;
                // aes_icm.c:317-322: at most 0xffff keystream blocks
                if ((z.flags & SRTP_DS_ICM_CONF) &&
                    (len - h.enc_start + 15) / 16 > 0xffffu)
                    code = 8;        // srtp_err_status_cipher_fail
                const uint32_t seq = h.seq_len & 0xffffu;
                // rdbx.c:112-145 (srtp_rtp_hdr.h)
                const int64_t delta = srtp_guess_index(z.index, seq, &e);
                if (delta < 1)
                    ab |= FZ_AB_ORDER;   // the sorted path decides
                fz_count(F, z, sid, true, e);
                if (code == 0 && !inel) {
                    m.key = z.key;
                    m.roc = (uint32_t)(e >> 16);
                    m.info = h.enc_start | (z.variant << 24);
                    m.len = len;
                    // the bytes the tag overwrites (in place), for the undo:
                    // at most two loads of the 8-byte-aligned span around
                    // them (each 8-byte half read holds a byte of
                    // [len, len + trailer), so no read leaves the pages the
                    // packet's buffer is in), then a byte-aligned extract
                    u32x4 w;
                    S.tail(len, z.trailer < 16 ? z.trailer : 16, w);
                    *(u32x4 *)F.tsave[i] = w;
                }
            }
        }
    }
    // the descriptor is not stored: a declined batch rebuilds it for the
    // undo (srtp_prepass.hip k_fz_meta).  Status and protected length are
    // written now (the commit of an accepted batch); a declined batch gets
    // its capacities back from the record and its statuses from the path
    // that then runs it
    *(u32x4 *)&F.rec[i] =
        u32x4{ (uint32_t)e, (uint32_t)(e >> 32) | (code << 16), key, cap };
    F.status[i] = (int32_t)code;
    if (code == 0 && key != FZ_NOCHAIN)
        F.cap[i] = len + z.trailer;
    if (ab)
        atomicOr(F.abort, ab);
    return m;
}

// The receive side's order-free classification inside the crypto kernel
// (pp_unprotect_fused; srtp_prepass.hip k_pu_classify restated): header
// parse, stream lookup, receive eligibility, the length / capacity checks of
// srtp_host.c un_static (srtp.c:2905-2990; a failing packet sends the batch
// to the host: its status would depend on the replay check), the MKI of the
// device key, and the index guessed from the stored index (rdbx.c:112-145).
// A candidate is decrypted and verified by icm_packet; fzu_verdict then
// writes its status and length.  `e` / `sid` out: the candidate's index and
// stream (sid ~0: not a candidate).
template <class ARGS, class SRC>
DEV srtp_dev_meta_t fzu_classify(const ARGS &A, uint32_t i, FzLane &z,
                                 uint32_t vid, uint64_t off, uint32_t len,
                                 uint32_t cap, const SRC &S, uint64_t &e,
                                 uint32_t &sid)
{
    const IcmFused &F = A.fz;
    const srtp_dev_hdr_t h = S.hdr(off, len);
    uint32_t code = 0, ab = 0;
    e = 0;
    sid = FZ_NOCHAIN;
    srtp_dev_meta_t m;
    m.key = 0;
    m.roc = 0;
    m.len = 0;
    m.info = 0xff0000u;   // no crypto
    if (h.enc_start >> 24) {
        code = h.enc_start >> 24;   // header does not parse: no stream touched
    } else {
        fz_lookup(F, z, h.ssrc);
        if (z.sid == FZ_NOCHAIN) {
            ab |= FZ_AB_UNKNOWN;    // template clone: host
        } else if (z.variant != vid) {
            ab |= FZ_AB_INELIGIBLE;  // not decrypted here (fz_classify)
        } else {
            if (!(z.flags & SRTP_DS_RX_ELIGIBLE) || (z.dir & SRTP_DIR_TX))
                ab |= FZ_AB_INELIGIBLE;
            const uint32_t tag = z.trailer;   // tag + MKI
            const uint32_t es = h.enc_start;
            if (len < tag || es > len - tag ||
                ((z.flags & SRTP_DS_AEAD) && len - es < tag) ||
                cap < len - tag ||
                ((z.flags & SRTP_DS_ICM_CONF) &&
                 (len - tag - es + 15) / 16 > 0xffffu)) {
                ab |= FZ_AB_STATIC;
            } else {
                if (z.mki) {
                    // srtp_prepass.hip mki_is_device_key
                    const uint32_t sz = z.mki & 0xffffu;
                    const uint32_t x = len - (z.mki >> 16);
                    const uint8_t *mk = A.keys[z.key].mki;
                    uint32_t d = 0;
                    for (uint32_t b = 0; b < sz; b++)
                        d |= S.byte(x + b) ^ mk[b];
                    if (d)
                        ab |= FZ_AB_MKI;
                }
                const uint32_t seq = h.seq_len & 0xffffu;
                // rdbx.c:112-145 (srtp_rtp_hdr.h)
                const int64_t delta = srtp_guess_index(z.index, seq, &e);
                if (delta < 1)
                    ab |= FZ_AB_ORDER;   // the sorted path decides
                sid = z.sid;
                fzu_cand(F, z, sid, e);
                m.key = z.key;
                m.roc = (uint32_t)(e >> 16);
                m.info = es | (z.variant << 24);
                m.len = len - tag;
            }
        }
    }
    *(u32x4 *)&F.rec[i] =
        u32x4{ (uint32_t)e, (uint32_t)(e >> 32) | (code << 16), sid, cap };
    if (sid == FZ_NOCHAIN)
        F.status[i] = (int32_t)code;   // a header error's status (any other
                                       // non-candidate aborts the batch)
    if (ab)
        atomicOr(F.abort, ab);
    return m;
}

// ... after icm_packet: the candidate's verdict (status, length; an
// authenticated packet's index into the run and the second bitmap)
template <class ARGS>
DEV void fzu_verdict(const ARGS &A, uint32_t i, FzLane &z,
                     const srtp_dev_meta_t &m, uint64_t e, uint32_t sid,
                     bool ok)
{
    if (sid == FZ_NOCHAIN)
        return;
    const IcmFused &F = A.fz;
    if (ok) {
        F.status[i] = 0;
        F.cap[i] = m.len;
        fzu_auth(F, z, e);
    } else {
        F.status[i] = 7;   // srtp_err_status_auth_fail
        atomicAdd(F.nfail, 1u);
    }
}

// One stream's in-order batch (IcmChain): the descriptor of packet i from
// its header (srtp_rtp_hdr.h srtp_inorder_desc), else no crypto and the
// batch is declined (*abort).  Protect in place saves the trailer bytes the
// tag will overwrite, for the decline's restore (Q.tsave; null when
// k_io_check verified the batch first).  The output is at out_off.
template <bool RX, class ARGS>
DEV srtp_dev_meta_t inorder_meta(const ARGS &A, uint32_t i, uint64_t off,
                                 const srtp_dev_stream_t &S, uint32_t seq0,
                                 uint64_t e0, bool e0ok)
{
    const IcmChain &Q = A.ch;
    const uint32_t len = Q.in_len[i], cap = Q.cap[i];
    const srtp_dev_hdr_t h = srtp_parse_rtp(A.in + off, off, len);
    srtp_dev_meta_t m;
    if (!srtp_inorder_desc(S, h, i, len, cap, seq0, e0, e0ok, RX, m)) {
        atomicOr(Q.abort, 1u);
        return m;
    }
    if constexpr (!RX) {
        if (Q.tsave) {
            u32x4 w;
            fz_tail_save(A.out + off + len, S.trailer < 16 ? S.trailer : 16,
                         w);
            *(u32x4 *)Q.tsave[i] = w;
        }
    }
    return m;
}

// The packet's bytes read from the arena (the fused classification's
// header, trailer save and MKI; srtp_parse_rtp's 16-byte header load)
struct GlbSrc {
    const uint8_t *p;   // the packet (in place: input and output)
    DEV srtp_dev_hdr_t hdr(uint64_t off, uint32_t len) const
    {
        return srtp_parse_rtp(p, off, len);
    }
    DEV void tail(uint32_t x, uint32_t tn, u32x4 &w) const
    {
        fz_tail_save(p + x, tn, w);
    }
    DEV uint32_t byte(uint32_t x) const { return p[x]; }
};


}   // namespace
