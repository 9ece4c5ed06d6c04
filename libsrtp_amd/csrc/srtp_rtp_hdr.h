// srtp_rtp_hdr.h -- device-side RTP header parse shared by the parse kernel
// and the device pre-passes.  Follows srtp_get_rtp_hdr_len (srtp/srtp.c:
// 96-125: fixed header + CSRCs) and srtp_validate_rtp_header (srtp.c:
// 307-336: length checks, the one-word extension header and its length) as
// restated in oracle/srtp_oracle.c.
#ifndef SRTP_RTP_HDR_H
#define SRTP_RTP_HDR_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "srtp_dev.h"

__device__ __forceinline__ uint32_t srtp_bswap32(uint32_t x)
{
    return __builtin_amdgcn_perm(0u, x, 0x00010203u);
}

// summary of packet p (len bytes, arena offset off): enc_start holds the
// header length, or (status << 24) when the header does not parse
// (srtp_err_status_bad_param, as the reference's length checks return)
__device__ __forceinline__ srtp_dev_hdr_t srtp_parse_rtp(const uint8_t *p,
                                                         uint64_t off,
                                                         uint32_t len)
{
    srtp_dev_hdr_t h;
    h.len = len;
    h.ssrc = 0;
    h.seq_len = 0;
    uint32_t err = 0, es = 0;
    if ((off & 15) != 0) {
        err = 2;
    } else if (len < 12) {
        err = 2;
    } else {
        // one 16-byte load: the packet is 16-B aligned and readable to
        // roundup16(len) >= 16
        const uint4 q = *(const uint4 *)p;
        uint32_t w0 = srtp_bswap32(q.x);
        h.ssrc = srtp_bswap32(q.z);
        h.seq_len = w0 & 0xffffu;
        es = 12 + 4 * ((w0 >> 24) & 0xfu);
        if (len < es) {
            err = 2;
        } else if ((w0 >> 28) & 1) {
            if (len < es + 4) {
                err = 2;
            } else {
                uint32_t xw = srtp_bswap32(*(const uint32_t *)(p + es));
                es += ((xw & 0xffffu) + 1) * 4;
                if (len < es)
                    err = 2;
            }
        }
    }
    h.enc_start = err ? (err << 24) : es;
    return h;
}

// SSRC -> device stream id through the device copy of the host's
// open-addressing map (srtp_host.c map_hash / map_get: first inserted wins,
// as srtp_stream_list_get, srtp.c:5292-5305); ~0 when absent
__device__ __forceinline__ uint32_t srtp_map_lookup(const uint32_t *hkey,
                                                    const uint32_t *hval,
                                                    uint32_t hmask,
                                                    uint32_t ssrc)
{
    uint32_t h = ssrc * 0x9e3779b1u;
    h ^= h >> 15;
    uint32_t p = h & hmask;
    for (uint32_t probe = 0; probe <= hmask; probe++) {
        const uint32_t v = hval[p];
        if (v == 0xffffffffu)
            return 0xffffffffu;
        if (hkey[p] == ssrc)
            return v;
        p = (p + 1) & hmask;
    }
    return 0xffffffffu;
}

// CSRC count, X bit and extension profile of a header srtp_parse_rtp
// accepted: [15:0] profile, [19:16] CC, bit 20 X
__device__ __forceinline__ uint32_t srtp_rtp_xinfo(const uint8_t *p,
                                                   const srtp_dev_hdr_t &h)
{
    if (h.enc_start >> 24)
        return 0;
    const uint32_t w0 = srtp_bswap32(*(const uint32_t *)p);
    const uint32_t cc = (w0 >> 24) & 0xfu, x = (w0 >> 28) & 1u;
    uint32_t v = cc << 16 | x << 20;
    if (x)
        v |= srtp_bswap32(*(const uint32_t *)(p + 12 + 4 * cc)) >> 16;
    return v;
}

// index_guess against a stream's stored index (srtp_host.c estimate /
// index_guess = crypto/replay/rdbx.c:112-145, 280-299): the 48-bit index
// of sequence number seq and the signed distance from idx
__device__ __forceinline__ int64_t srtp_guess_index(uint64_t idx, uint32_t seq,
                                                    uint64_t *est)
{
    if (idx > 32768) {
        const uint32_t lroc = (uint32_t)(idx >> 16);
        const uint32_t lseq = (uint32_t)(idx & 0xffffu);
        uint32_t roc = lroc;
        int64_t diff = (int64_t)seq - (int64_t)lseq;
        if (lseq < 32768) {
            if ((int)seq - (int)lseq > 32768) {
                roc = lroc - 1;
                diff -= 65536;
            }
        } else if ((int)lseq - 32768 > (int)seq) {
            roc = lroc + 1;
            diff += 65536;
        }
        *est = ((uint64_t)roc << 16) | seq;
        return diff;
    }
    *est = seq;
    return (int64_t)seq - (int64_t)idx;
}

// One stream's in-order batch (srtp_prepass.hip pp_protect_inorder /
// pp_unprotect_inorder): packet i belongs to the run when its header parses
// with the stream's SSRC, its sequence number is seq_0 + i and the checks
// of the host pre-pass pass (protect: srtp_host.c pre_protect, srtp.c:
// 2515-2600; unprotect: un_static, srtp.c:2905-2990); its index is then
// e_0 + i.  Returns false (no descriptor) otherwise: the batch is declined.
__device__ __forceinline__ bool srtp_inorder_desc(
    const srtp_dev_stream_t &S, const srtp_dev_hdr_t &h, uint32_t i,
    uint32_t len, uint32_t cap, uint32_t seq0, uint64_t e0, bool e0ok,
    bool rx, srtp_dev_meta_t &m)
{
    m.key = 0;
    m.roc = 0;
    m.len = 0;
    m.info = 0xff0000u;   // no crypto
    if (!e0ok || (h.enc_start >> 24) != 0 || h.ssrc != S.ssrc ||
        (h.seq_len & 0xffffu) != ((seq0 + i) & 0xffffu))
        return false;
    const uint32_t es = h.enc_start, tag = S.trailer;
    uint32_t plen = len;   // the authenticated / encrypted region's end
    if (rx) {
        if (S.mki || len < tag || es > len - tag ||
            ((S.flags & SRTP_DS_AEAD) && len - es < tag) || cap < len - tag)
            return false;
        plen = len - tag;
    } else if (es > len || cap < len + tag) {
        return false;
    }
    if ((S.flags & SRTP_DS_ICM_CONF) && (plen - es + 15) / 16 > 0xffffu)
        return false;
    const uint64_t e = e0 + i;
    m.key = S.key;
    m.roc = (uint32_t)(e >> 16);
    m.info = es | (S.variant << 24);
    m.len = plen;
    return true;
}

// ... and its packet 0: seq_0, e_0 (the stored index's guess; the run must
// lie above it) and whether the stream may run this direction
__device__ __forceinline__ bool srtp_inorder_head(const srtp_dev_stream_t &S,
                                                  const uint8_t *pkt0, bool rx,
                                                  uint32_t &seq0,
                                                  uint64_t &e0)
{
    seq0 = srtp_bswap32(*(const uint32_t *)pkt0) & 0xffffu;
    e0 = 0;
    const bool dir = rx ? ((S.flags & SRTP_DS_RX_ELIGIBLE) &&
                           !(S.dir & SRTP_DIR_TX))
                        : ((S.flags & SRTP_DS_ELIGIBLE) &&
                           !(S.dir & SRTP_DIR_RX));
    return srtp_guess_index(S.index, seq0, &e0) >= 1 && dir;
}

#endif
