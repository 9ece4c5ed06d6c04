// srtp_prepass.hip -- the pre-passes of srtp_protect_device and
// srtp_unprotect_device on the GPU (unprotect: see k_pu_classify below).
//
// The host pre-pass (srtp_host.c pre_protect, following srtp/srtp.c:
// 2493-2712 and 2088-2233) walks the batch in order: stream lookup, key
// usage (crypto/kernel/key.c:74-90), index estimate and replay update
// (srtp.c:2038-2081, crypto/replay/rdbx.c:112-145, 227-270).  Per stream
// those steps form a chain: packet k's index is packet k-1's index plus the
// 16-bit sequence advance, as long as every advance is in [1, 2^15) -- the
// range where rdbx's index_guess returns exactly prev + d.  Under that
// condition the whole batch reduces to
//   classify (parse, SSRC hash lookup)  -> stable radix sort by stream
//   -> segmented inclusive scan of advances (first packet: the exact
//      estimate from the stream's stored index)  -> replay window update
//   -> commit (meta, status, out_len, stream state)
// and every packet's result equals the sequential reference's.
//
// Many streams (ns > 1, e.g. BASELINE configs[3]: 64k SSRCs) take an
// order-free form first: every chain packet's index is guessed from its
// stream's STORED index (index_guess).  When, per stream, every index of
// the batch is above the stored one and within one replay window of the
// batch's highest (hi - est < window bits <= 2^15), the reference's
// in-order walk accepts every packet at exactly that guess (each running
// top is the stored index or a batch index less than a window away, so
// each guess is the same, and no packet is ever "old"), whatever the
// packets' order -- unless two share an index, which the window bitmap
// catches (atomicOr sees the bit set).  Then the new state is index = hi,
// window = old window shifted by hi - stored plus one bit per packet, and
// the whole pre-pass is classify (with the per-stream max and packet
// count, wave-aggregated) -> window shift -> set bits -> commit: no sort.
// A batch outside that condition (AB_ORDER: a stream with more packets
// than its window, or an index at or below the stored one) is re-run
// through the sorted chain path.  Anything
// outside the condition (unknown SSRC needing a template clone, a stream
// with a pending ROC / receiver direction, a protect batch's duplicate
// index, an MKI other than the device key's on receive) raises the abort
// word: nothing is committed, the crypto kernels exit, and the host runs
// its exact path on the untouched state.  MKI streams run with the one
// master key the host's device table selected (srtp_host.c
// dev_mki_select).  One-stream receive batches in any arrival order:
// pp_unprotect_chain1 below.  The order-free protect form of in-place
// AES-ICM batches classifies inside the crypto kernel (pp_protect_fused,
// srtp_icm.hip fz_classify).  Key-limit
// events cannot occur on this path: the host only takes it while every key
// has more than SOFT_LIMIT uses left after the batch.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "srtp_dev.h"
#include "srtp_gpu_int.h"
#include "srtp_rtp_hdr.h"
#include "srtp_scan.h"

int srtp_gpu_fail(hipError_t e, const char *what);   // srtp_gpu.hip

namespace {

constexpr uint32_t SEQ_MEDIAN = 32768;
constexpr uint32_t ST_BAD_PARAM = 2, ST_CIPHER_FAIL = 8, ST_PARSE_ERR = 21,
                   ST_BUFFER_SMALL = 28;
constexpr uint32_t NOCHAIN = 0xffffffffu;

// abort reasons (bits of the abort word; any bit -> host path)
enum { AB_UNKNOWN_SSRC = 1, AB_INELIGIBLE = 2, AB_SEQUENCE = 4,
       AB_ORDER = 8, /* order-free form does not apply: sorted path */
       AB_STATIC = 16, /* unprotect: a packet with a length/capacity error */
       AB_MKI = 32, /* unprotect: a packet whose MKI is not the device key's */
       AB_PENDING = 512, /* unprotect: the first packet of a stream whose
                            pending ROC it resolved did not authenticate */
       AB_GAP = 2048 /* in-order unprotect: a packet 2^15 or more past the
                        last accepted index (its estimate would differ) */ };

struct PpState {
    // stream table
    srtp_dev_stream_t *st = nullptr;
    uint32_t ns = 0, ns_cap = 0;
    uint32_t *win = nullptr, *wnew = nullptr;
    uint32_t nwords = 0, nwords_cap = 0;
    uint32_t *hkey = nullptr, *hval = nullptr;
    uint32_t hcap = 0, hcap_cap = 0;
    uint32_t *bcount = nullptr;     // packets charged per stream (batch)
    uint32_t *seg_first = nullptr;  // sorted position of a stream's first
    uint64_t *new_index = nullptr;  // per stream, 0 = no chain packet
    // per-packet scratch
    size_t n_cap = 0;
    srtp_dev_hdr_t *hdr = nullptr;
    uint32_t *pstat = nullptr;      // status code of the packet
    uint32_t *skey = nullptr, *skey2 = nullptr, *perm = nullptr,
             *perm2 = nullptr;
    uint64_t *val = nullptr, *est = nullptr;
    srtp_dev_meta_t *meta = nullptr;
    uint8_t *auth = nullptr;        // unprotect: tag verdict per packet
    uint8_t *rxj = nullptr;         // unprotect, MKI streams: key index
    uint64_t *top = nullptr;        // unprotect chain: highest accepted before
    uint32_t *bcount2 = nullptr;    // unprotect: authenticated per stream
    uint64_t *new_index2 = nullptr; // unprotect: highest authenticated
    // scratch of the scans and the radix sort (srtp_scan.h)
    srtp_scan::Agg *agg = nullptr;
    uint32_t *hist = nullptr;
    uint32_t *abort = nullptr;      // device word
    uint32_t *h_abort = nullptr;    // pinned, host-coherent: the final abort
                                    // word, published by the commit kernel
    uint32_t *h_abort_dev = nullptr;   // its device address
    // key buckets (many-key order-free batches): per-stream record offset
    // and cursor, the records and their packet indices, the region bounds
    uint32_t *bk_off = nullptr, *bk_cur = nullptr;
    srtp_dev_rec_t *rec = nullptr;
    uint32_t *rec_idx = nullptr;
    uint32_t *bk_range = nullptr;
    // fused single-stream chain form (k_pp_chain1): per-tile look-back
    // words, {next tile, uses} counters, two abort words used in turn (the
    // commit kernel of one batch clears the next batch's), the turn
    uint64_t *ch_tile = nullptr;
    uint32_t *ch_ctl = nullptr;
    uint32_t *ch_abort = nullptr;
    uint32_t ch_par = 0;
    size_t ch_tiles_cap = 0;
    // one-stream unprotect (k_pu_chain1 .. k_pu_commit1): two control blocks
    // used in turn, the look-back words of its two scans, the generation-
    // tagged first-authenticated-position array and its generation
    struct PuCtl *pu_ctl = nullptr;
    uint32_t pu_par = 0;
    uint64_t *pu_tile = nullptr;   // 2 x (ch_tiles_cap + 1) words
    unsigned long long *pu_first = nullptr;
    uint64_t pu_first_cap = 0;
    uint32_t pu_gen = 0;
    // order-free protect classified in the crypto kernel: the trailer bytes
    // each in-place packet's tag overwrites (16 per packet)
    FzRec *fzrec = nullptr;   // fused classification records
    uint32_t (*tsave)[4] = nullptr;
    // per stream: counts, lowest chain index; index bitmaps (2 x nwords)
    unsigned long long *fz_cnt = nullptr, *fz_emin = nullptr;
    uint32_t *fz_bmap = nullptr;   // 4 x nwords + 4: candidates | authenticated
    uint32_t bmap_cap = 0;
    unsigned long long *fz_hicand = nullptr;   // unprotect: highest candidate
    uint32_t *fz_nfail = nullptr;              // unprotect: failed tag checks
    uint32_t *fz_glist = nullptr;              // k_icm_stg's per-lane groups
    // pending ROCs (srtp_gpu_pp_pend_*): per stream the first packet and the
    // lowest / highest pending index; the listed streams, their results;
    // the records and windows an apply replaced, its streams' first packets
    uint32_t *pd_first = nullptr;
    unsigned long long *pd_min = nullptr, *pd_max = nullptr;
    uint32_t pd_cap = 0, pd_cap2 = 0, pd_cap3 = 0;
    uint32_t *pd_sids = nullptr;
    srtp_pend_info_t *pd_info = nullptr;
    uint64_t *pd_efirst = nullptr;
    uint32_t pd_list_cap = 0, pd_list_cap2 = 0, pd_list_cap3 = 0;
    srtp_dev_stream_t *pd_bak = nullptr;
    uint32_t pd_bak_cap = 0;
    uint32_t *pd_bakwin = nullptr;
    uint32_t pd_bakwin_cap = 0;
    uint32_t *pd_pos = nullptr;                // applied: first packets
    uint32_t pd_pos_cap = 0;
    uint32_t pd_nres = 0;                      // applied streams (0: none)
    // template clones (srtp_gpu_pp_clone): the template's record, spare
    // records after the uploaded ns0, window words of one, the device's
    // count of created streams and its overflow / spin-limit flag
    srtp_dev_stream_t tmpl{};
    bool has_tmpl = false;
    uint32_t ns0 = 0, spare = 0, tw = 0;
    uint32_t *cl_ctl = nullptr;                // [0] created, [1] flags
    // MKI streams: the key slots of their master keys (srtp_dev_stream_t
    // kbase / nkeys), the protect packets charged to each, and the batch's
    // per-packet key indices (srtp_gpu_pp_batch_t mki)
    uint64_t *io_e0 = nullptr;   // pp_unprotect_inorder: the run's e_0
    uint32_t *mkslot = nullptr;
    unsigned long long *kuses = nullptr;
    uint32_t nmk = 0, nmk_cap = 0;
    uint8_t *mki8 = nullptr;
    size_t mki8_cap = 0;
};

// the host reads the published abort word after the stream synchronises
constexpr uint32_t ABORT_UNSET = 0xffffffffu;

// one launch instead of a memset per array: the abort word and the
// per-stream aggregates of a pre-pass round
__global__ void k_pp_reset(uint32_t *abort, uint32_t *bcount,
                           unsigned long long *new_index, uint32_t *bcount2,
                           unsigned long long *new_index2, uint32_t ns)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s == 0)
        *abort = 0;
    if (s >= ns)
        return;
    bcount[s] = 0;
    new_index[s] = 0;
    if (bcount2) {
        bcount2[s] = 0;
        new_index2[s] = 0;
    }
}

// the final abort word to host memory, from the last kernel that reads it
__device__ __forceinline__ void publish_abort(uint32_t *pub,
                                              const uint32_t *abort)
{
    if (pub && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(pub, *abort, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// ... and, for a receive batch, the count of failed tags beside it (pub[1]):
// the host reads both from pinned memory after its one synchronize, no copy
__device__ __forceinline__ void publish_nfail(uint32_t *pub, uint32_t nfail)
{
    if (pub)
        __hip_atomic_store(pub + 1, nfail, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint32_t map_hash(uint32_t k, uint32_t mask)
{
    // srtp_host.c map_hash
    uint32_t h = k * 0x9e3779b1u;
    h ^= h >> 15;
    return h & mask;
}

// the stream of an SSRC in the device hash (NOCHAIN: none)
__device__ __forceinline__ uint32_t lookup_sid(const uint32_t *hkey,
                                               const uint32_t *hval,
                                               uint32_t hmask, uint32_t ssrc)
{
    uint32_t p = map_hash(ssrc, hmask);
    for (uint32_t probe = 0; probe <= hmask; probe++) {
        const uint32_t v = hval[p];
        if (v == NOCHAIN)
            return NOCHAIN;
        if (hkey[p] == ssrc)
            return v;
        p = (p + 1) & hmask;
    }
    return NOCHAIN;
}

struct ClassifyArgs {
    const uint8_t *in;
    const uint64_t *in_off;
    const uint32_t *in_len;
    const uint32_t *cap;
    const srtp_dev_stream_t *st;
    const uint32_t *hkey, *hval;
    uint32_t hmask;
    uint32_t n;
    srtp_dev_hdr_t *hdr;
    uint32_t *pstat, *skey, *perm, *bcount, *abort;
    // order-free form only (null otherwise): per-packet index guessed from
    // the stored index, per-stream highest index; the packet's crypto
    // descriptor and protected length, written here (no header summary and
    // no permutation are kept: commit only copies status and length)
    uint64_t *est;
    unsigned long long *new_index;
    srtp_dev_meta_t *meta;
    uint32_t *olen;
    // unprotect: the key records and the slots of the MKI streams' master
    // keys (a packet's MKI selects its key, mki_match), and per packet the
    // key index found (rxj: MKI_NONE = bad_mki)
    const srtp_dev_key_t *keys;
    const uint32_t *mkslot;
    uint8_t *rxj;
};

// the master key an MKI stream's packet (length checks passed) selects: the
// first of the stream's keys whose MKI equals the packet's (srtp.c:1961-2016
// srtp_get_session_keys_for_packet, keys in list order), MKI_NONE for none
// (srtp_err_status_bad_mki, after the replay check: srtp.c:2884-2912)
constexpr uint32_t MKI_NONE = 0xffu, ST_BAD_MKI = 25;
__device__ __forceinline__ uint32_t mki_match(const srtp_dev_key_t *keys,
                                              const uint32_t *mkslot,
                                              const srtp_dev_stream_t &S,
                                              const uint8_t *pkt, uint32_t len)
{
    const uint32_t sz = S.mki & 0xffffu, back = S.mki >> 16;
    const uint8_t *p = pkt + len - back;
    for (uint32_t j = 0; j < S.nkeys; j++) {
        const uint8_t *m = keys[mkslot[S.kbase + j]].mki;
        uint32_t d = 0;
        for (uint32_t b = 0; b < sz; b++)
            d |= p[b] ^ m[b];
        if (d == 0)
            return j;
    }
    return MKI_NONE;
}

// the tag verdict byte of unprotect (auth[]): 1 authenticated (or no tag
// check), 0 the tag failed, AUTH_BAD_MKI no key matched the packet's MKI (no
// crypto ran)
constexpr uint8_t AUTH_BAD_MKI = 2;

// index_guess against a stream's stored index (srtp_host.c estimate /
// index_guess = rdbx.c:112-145, 280-299); returns delta
__device__ __forceinline__ int64_t guess_index(uint64_t idx, uint32_t seq,
                                               uint64_t *est)
{
    return srtp_guess_index(idx, seq, est);   // srtp_rtp_hdr.h
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m)
{
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}

// per-stream packet count and highest index (order-free form, unprotect
// verdicts).  Per wave, up to four streams are reduced across the lanes;
// the first of them is merged across the block's waves in LDS, so a batch
// of one stream costs one atomic pair per block instead of one per lane
// (same-address atomics serialise in L2: 32k of them took 0.2 ms).  The
// remaining lanes (many streams per wave) use their own atomics.  Called by
// every thread of the block.
__device__ void agg_stream(uint32_t key, uint64_t e, uint32_t *bcount,
                           unsigned long long *new_index)
{
    __shared__ uint32_t s_key[16], s_cnt[16];
    __shared__ unsigned long long s_max[16];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    bool done = key == NOCHAIN;
    uint32_t gkey = NOCHAIN, gcnt = 0;
    uint64_t gmax = 0;
    for (int it = 0; it < 4; it++) {
        const uint64_t am = __ballot(!done);
        if (!am)
            break;
        const uint32_t lead =
            (uint32_t)__shfl((int)key, __ffsll((unsigned long long)am) - 1);
        const bool mine = !done && key == lead;
        const uint64_t mm = __ballot(mine);
        uint64_t v = mine ? e : 0;
        for (int m = 1; m < 64; m <<= 1) {
            const uint64_t o = shfl_xor64(v, m);
            v = o > v ? o : v;
        }
        if (it == 0) {
            gkey = lead;
            gcnt = (uint32_t)__popcll((unsigned long long)mm);
            gmax = v;
        } else if (lane == (uint32_t)(__ffsll((unsigned long long)mm) - 1)) {
            atomicAdd(&bcount[lead], (uint32_t)__popcll((unsigned long long)mm));
            atomicMax(&new_index[lead], (unsigned long long)v);
        }
        done = done || mine;
        // a stream that only one lane of the wave holds: the packets of the
        // wave are spread over many streams (64k-stream batches), so the
        // rest go straight to their own atomics
        if (__popcll((unsigned long long)mm) == 1)
            break;
    }
    if (!done) {
        atomicAdd(&bcount[key], 1u);
        atomicMax(&new_index[key], (unsigned long long)e);
    }
    if (lane == 0) {
        s_key[wave] = gkey;
        s_cnt[wave] = gcnt;
        s_max[wave] = gmax;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t nw = (blockDim.x + 63) >> 6;
        for (uint32_t w = 0; w < nw; w++) {
            const uint32_t k = s_key[w];
            if (k == NOCHAIN)
                continue;
            uint32_t c = s_cnt[w];
            unsigned long long m = s_max[w];
            for (uint32_t w2 = w + 1; w2 < nw; w2++)
                if (s_key[w2] == k) {
                    c += s_cnt[w2];
                    m = s_max[w2] > m ? s_max[w2] : m;
                    s_key[w2] = NOCHAIN;
                }
            atomicAdd(&bcount[k], c);
            atomicMax(&new_index[k], m);
        }
    }
}

__device__ uint32_t classify_one(const ClassifyArgs &A, uint32_t i,
                                 srtp_dev_hdr_t &h);

// parse, stream lookup, the per-packet checks of pre_protect that do not
// depend on stream state (srtp_host.c pre_protect; srtp.c:2515-2600)
__global__ void k_pp_classify(ClassifyArgs A)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t key = NOCHAIN;
    uint64_t e = 0;
    if (i < A.n) {
        srtp_dev_hdr_t h;
        key = classify_one(A, i, h);
        if (A.est) {
            srtp_dev_meta_t m;
            m.key = 0;
            m.roc = 0;
            m.len = 0;
            m.info = 0xff0000u;   // no crypto
            if (key != NOCHAIN) {
                const srtp_dev_stream_t &S = A.st[key];
                const uint32_t seq = h.seq_len & 0xffffu;
                // at or below the stored index (a replay, or an advance the
                // guess from the stored index cannot see): the sorted path
                // decides
                if (guess_index(S.index, seq, &e) < 1)
                    atomicOr(A.abort, AB_ORDER);
                A.est[i] = e;
                if (A.pstat[i] == 0) {
                    m.key = S.key;
                    m.roc = (uint32_t)(e >> 16);
                    m.info = h.enc_start | (S.variant << 24);
                    m.len = h.len;
                    A.olen[i] = h.len + S.trailer;
                }
            }
            A.meta[i] = m;
        }
    }
    if (A.est)
        agg_stream(key, e, A.bcount, A.new_index);
}

// order-free form: the replay bit of every chain packet (window already
// shifted to the stream's highest index by k_pp_window)
__global__ void k_pp_usetbits(const uint32_t *skey, const uint64_t *est,
                              const srtp_dev_stream_t *st, uint32_t ns,
                              uint32_t n, const uint64_t *new_index,
                              uint32_t *wnew, uint32_t *abort)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t s = skey[i];
    if (s >= ns)
        return;
    const uint64_t hi = new_index[s], e = est[i];
    const uint32_t bits = st[s].win_bits;
    // every running top of the in-order walk is the stored index or one of
    // the batch's indices (all within bits <= 2^15 of each other), so each
    // guess equals the one from the stored index
    if (hi - e >= bits) {
        atomicOr(abort, AB_ORDER);
        return;
    }
    const uint32_t bit = bits - 1 - (uint32_t)(hi - e);
    const uint32_t m = 1u << (bit & 31);
    if (atomicOr(&wnew[st[s].win_off + (bit >> 5)], m) & m)
        atomicOr(abort, AB_SEQUENCE);   // two packets with one index: host
}

// one packet of k_pp_classify: header, stream, status code; returns the
// chain key (stream id) or NOCHAIN
__device__ uint32_t classify_one(const ClassifyArgs &A, uint32_t i,
                                 srtp_dev_hdr_t &h)
{
    const uint64_t off = A.in_off[i];
    const uint32_t len = A.in_len[i];
    h = srtp_parse_rtp(A.in + off, off, len);
    if (!A.est) {   // the sorted chain form reads them back
        A.hdr[i] = h;
        A.perm[i] = i;
    }
    uint32_t code = 0, key = NOCHAIN;
    if (h.enc_start >> 24) {
        code = h.enc_start >> 24;   // header does not parse: no stream touched
    } else {
        uint32_t sid = NOCHAIN;
        uint32_t p = map_hash(h.ssrc, A.hmask);
        for (uint32_t probe = 0; probe <= A.hmask; probe++) {
            const uint32_t v = A.hval[p];
            if (v == NOCHAIN)
                break;
            if (A.hkey[p] == h.ssrc) {
                sid = v;
                break;
            }
            p = (p + 1) & A.hmask;
        }
        if (sid == NOCHAIN) {
            atomicOr(A.abort, AB_UNKNOWN_SSRC);   // template clone: host
        } else {
            const srtp_dev_stream_t &S = A.st[sid];
            if (!(S.flags & SRTP_DS_ELIGIBLE) || (S.dir & SRTP_DIR_RX))
                atomicOr(A.abort, AB_INELIGIBLE);
            // key usage (key.c:74) of packets that leave the chain here;
            // chain packets are counted per stream from the sorted segment
            // bounds (k_pp_seg_end) -- one atomic per packet on a hot
            // stream's counter would serialise the whole batch in L2
            if (A.cap[i] < len + S.trailer) {
                code = ST_BUFFER_SMALL;
                atomicAdd(&A.bcount[sid], 1u);
            } else if (h.enc_start > len) {
                code = ST_PARSE_ERR;
                atomicAdd(&A.bcount[sid], 1u);
            } else {
                key = sid;
                // aes_icm.c:317-322: at most 0xffff keystream blocks
                if ((S.flags & SRTP_DS_ICM_CONF) &&
                    (len - h.enc_start + 15) / 16 > 0xffffu)
                    code = ST_CIPHER_FAIL;   // index still advances
            }
        }
    }
    A.pstat[i] = code;
    A.skey[i] = key;
    return key;
}

// One stream (the common case of a single-session sender): the stable sort
// by stream id is a stable partition into the chain packets (key 0) and the
// rest (NOCHAIN), placed by an exclusive scan of the chain flags -- a scan
// and a scatter instead of a full radix sort.
// scan traits (srtp_scan.h): the chain flags of one stream -> positions
struct ChainFlags {
    const uint32_t *skey;
    uint32_t *out;
    __device__ uint32_t key(uint32_t) const { return 0; }
    __device__ uint64_t val(uint32_t i) const { return skey[i] == 0u; }
    __device__ void store(uint32_t i, uint64_t v) const { out[i] = (uint32_t)v; }
};

// 64-bit values, segmented by keys (null: one segment)
struct Seg64 {
    const uint32_t *keys;
    const uint64_t *in;
    uint64_t *out;
    __device__ uint32_t key(uint32_t i) const { return keys ? keys[i] : 0u; }
    __device__ uint64_t val(uint32_t i) const { return in[i]; }
    __device__ void store(uint32_t i, uint64_t v) const { out[i] = v; }
};

__global__ void k_pp_partition1(const uint32_t *skey, const uint32_t *excl,
                                uint32_t n, uint32_t *skey2, uint32_t *perm2)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t total = excl[n - 1] + (skey[n - 1] == 0u ? 1u : 0u);
    const uint32_t k = skey[i];
    const uint32_t pos = k == 0u ? excl[i] : total + (i - excl[i]);
    skey2[pos] = k;
    perm2[pos] = i;
}

// sorted position k: the advance over the previous packet of the stream,
// or for a stream's first packet the exact estimate from its stored index
// (srtp_host.c estimate / index_guess = rdbx.c:112-145, 280-299)
__global__ void k_pp_delta(const uint32_t *skey2, const uint32_t *perm2,
                           const srtp_dev_hdr_t *hdr,
                           const srtp_dev_stream_t *st, uint32_t ns,
                           uint32_t n, uint64_t *val, uint32_t *seg_first,
                           uint32_t *abort)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n)
        return;
    const uint32_t s = skey2[k];
    if (s >= ns) {
        val[k] = 0;
        return;
    }
    const uint32_t seq = hdr[perm2[k]].seq_len & 0xffffu;
    if (k > 0 && skey2[k - 1] == s) {
        const uint32_t pseq = hdr[perm2[k - 1]].seq_len & 0xffffu;
        const uint32_t d = (seq - pseq) & 0xffffu;
        if (d == 0 || d >= SEQ_MEDIAN)
            atomicOr(abort, AB_SEQUENCE);
        val[k] = d;
        return;
    }
    seg_first[s] = k;
    const uint64_t idx = st[s].index;
    uint64_t est;
    int64_t delta;
    if (idx > SEQ_MEDIAN) {
        const uint32_t lroc = (uint32_t)(idx >> 16);
        const uint32_t lseq = (uint32_t)(idx & 0xffffu);
        uint32_t roc = lroc;
        int64_t diff = (int64_t)seq - (int64_t)lseq;
        if (lseq < SEQ_MEDIAN) {
            if ((int)seq - (int)lseq > (int)SEQ_MEDIAN) {
                roc = lroc - 1;
                diff -= 65536;
            }
        } else if ((int)lseq - (int)SEQ_MEDIAN > (int)seq) {
            roc = lroc + 1;
            diff += 65536;
        }
        est = ((uint64_t)roc << 16) | seq;
        delta = diff;
    } else {
        est = seq;
        delta = (int64_t)seq - (int64_t)idx;
    }
    if (delta < 1)
        atomicOr(abort, AB_SEQUENCE);   // replay check / repeat: host path
    val[k] = est;
}

__global__ void k_pp_seg_end(const uint32_t *skey2, const uint64_t *est,
                             uint32_t ns, uint32_t n,
                             const uint32_t *seg_first, uint32_t *bcount,
                             uint64_t *new_index)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n)
        return;
    const uint32_t s = skey2[k];
    if (s < ns && (k + 1 == n || skey2[k + 1] != s)) {
        new_index[s] = est[k];
        atomicAdd(&bcount[s], k - seg_first[s] + 1);
    }
}

// window of stream s shifted by its advance (rdbx_add's bitvector shift,
// crypto/math/datatypes.c bitvector_left_shift)
__global__ void k_pp_window(const srtp_dev_stream_t *st, uint32_t ns,
                            const uint64_t *new_index, const uint32_t *win,
                            uint32_t *wnew)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ns || new_index[s] == 0)
        return;
    const srtp_dev_stream_t S = st[s];
    const uint64_t adv = new_index[s] - S.index;
    const uint32_t words = S.win_bits >> 5;
    const uint32_t *w = win + S.win_off;
    uint32_t *o = wnew + S.win_off;
    if (adv >= S.win_bits) {
        for (uint32_t i = 0; i < words; i++)
            o[i] = 0;
        return;
    }
    const uint32_t base = (uint32_t)adv >> 5, bi = (uint32_t)adv & 31;
    for (uint32_t i = 0; i < words; i++) {
        const uint32_t a = i + base < words ? w[i + base] : 0u;
        const uint32_t b = i + base + 1 < words ? w[i + base + 1] : 0u;
        o[i] = bi ? (a >> bi) | (b << (32 - bi)) : a;
    }
}

// the replay bit of every chain packet still inside the window, then the
// per-packet commit (sorted order k -> packet perm2[k])
__global__ void k_pp_setbits(const uint32_t *skey2, const uint64_t *est,
                             const srtp_dev_stream_t *st, uint32_t ns,
                             uint32_t n, const uint64_t *new_index,
                             uint32_t *wnew)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n)
        return;
    const uint32_t s = skey2[k];
    if (s >= ns)
        return;
    const uint64_t dist = new_index[s] - est[k];
    const uint32_t bits = st[s].win_bits;
    if (dist < bits) {
        const uint32_t bit = bits - 1 - (uint32_t)dist;
        atomicOr(&wnew[st[s].win_off + (bit >> 5)], 1u << (bit & 31));
    }
}

struct CommitArgs {
    const uint32_t *skey2, *perm2, *pstat;
    const uint64_t *est;
    const srtp_dev_hdr_t *hdr;
    const srtp_dev_stream_t *st;
    uint32_t ns, n;
    const uint32_t *abort;
    srtp_dev_meta_t *meta;
    int32_t *status;
    uint32_t *out_len;
};

__global__ void k_pp_commit_pkt(CommitArgs A)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= A.n || *A.abort)
        return;
    const uint32_t i = A.perm2[k];
    const uint32_t s = A.skey2[k];
    const uint32_t code = A.pstat[i];
    srtp_dev_meta_t m;
    m.key = 0;
    m.roc = 0;
    m.len = 0;
    m.info = 0xff0000u;
    if (s < A.ns && code == 0) {
        const srtp_dev_stream_t &S = A.st[s];
        const srtp_dev_hdr_t h = A.hdr[i];
        m.key = S.key;
        m.roc = (uint32_t)(A.est[k] >> 16);
        m.info = h.enc_start | (S.variant << 24);
        m.len = h.len;
        A.out_len[i] = h.len + S.trailer;
    }
    A.meta[i] = m;
    A.status[i] = (int32_t)code;   // error packets keep out_len = capacity
}

// order-free form: classify wrote the descriptors; unless aborted, the
// caller's status and protected length
__global__ void k_pp_commit_of(const uint32_t *pstat, const uint32_t *olen,
                               uint32_t n, const uint32_t *abort,
                               int32_t *status, uint32_t *out_len)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || *abort)
        return;
    const uint32_t code = pstat[i];
    status[i] = (int32_t)code;
    if (code == 0)
        out_len[i] = olen[i];   // error packets keep out_len = capacity
}

__global__ void k_pp_commit_stream(srtp_dev_stream_t *st, uint32_t ns,
                                   const uint64_t *new_index,
                                   const uint32_t *bcount, const uint32_t *wnew,
                                   uint32_t *win, const uint32_t *abort,
                                   uint32_t *pub)
{
    publish_abort(pub, abort);
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ns || *abort)
        return;
    st[s].uses += bcount[s];
    if (bcount[s])
        st[s].dir |= SRTP_DIR_TX;
    const uint64_t ni = new_index[s];
    if (ni == 0)
        return;
    st[s].index = ni;
    const uint32_t off = st[s].win_off, words = st[s].win_bits >> 5;
    for (uint32_t w = 0; w < words; w++)
        win[off + w] = wnew[off + w];
}

// One stream's in-order batch (pp_protect_inorder; the crypto kernel
// classified every packet, srtp_icm.hip inorder_meta): unless declined,
// every packet's status 0 and protected length, and the stream moved by n
// indices -- index e_0 + n - 1, the window shifted by the advance with the
// bits of the last min(n, window) indices set (rdbx.c:253-270), n key uses
// (key.c:74-90) -- and the verdict published to the host.
__global__ void k_io_commit(const uint8_t *in, const uint64_t *in_off,
                            const uint32_t *in_len, uint32_t n,
                            srtp_dev_stream_t *st, uint32_t *win,
                            const uint32_t *abort, uint32_t *abort_next,
                            uint32_t *pub, int32_t *status, uint32_t *out_len)
{
    const uint32_t ab = *abort;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    srtp_dev_stream_t &S = st[0];
    if (i < n && !ab) {
        status[i] = 0;
        out_len[i] = in_len[i] + S.trailer;
    }
    if (blockIdx.x != 0)
        return;
    __shared__ uint32_t s_win[SEQ_MEDIAN / 32];
    const uint32_t words = S.win_bits >> 5;
    const uint64_t old = S.index;
    uint32_t seq0;
    uint64_t e0;
    srtp_inorder_head(S, in + in_off[0], false, seq0, e0);
    const uint64_t hi = e0 + n - 1;
    if (!ab) {
        const uint64_t adv = hi - old;
        const uint32_t *w = win + S.win_off;
        const uint32_t setb = n < S.win_bits ? n : S.win_bits;
        for (uint32_t x = threadIdx.x; x < words; x += blockDim.x) {
            uint32_t v = 0;
            if (adv < S.win_bits) {
                const uint32_t b0 = (uint32_t)adv >> 5, bi = (uint32_t)adv & 31;
                const uint32_t a = x + b0 < words ? w[x + b0] : 0u;
                const uint32_t b = x + b0 + 1 < words ? w[x + b0 + 1] : 0u;
                v = bi ? (a >> bi) | (b << (32 - bi)) : a;
            }
            // bits [win_bits - setb, win_bits): the batch's last indices
            const uint32_t lo = S.win_bits - setb, base = 32 * x;
            for (uint32_t k = 0; k < 32; k++)
                if (base + k >= lo)
                    v |= 1u << k;
            s_win[x] = v;
        }
        __syncthreads();
        for (uint32_t x = threadIdx.x; x < words; x += blockDim.x)
            win[S.win_off + x] = s_win[x];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (!ab) {
            S.uses += n;
            S.dir |= SRTP_DIR_TX;
            S.index = hi;
        }
        if (pub)
            __hip_atomic_store(pub, ab, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        *abort_next = 0;   // the next batch's word (ch_abort pair)
    }
}

// ... out of place or asynchronous: the in-order conditions checked for
// every packet BEFORE the crypto kernel (the same test as inorder_meta,
// srtp_inorder_desc), so that a declined batch has written nothing -- out of
// place there is no input copy of the output to restore, and an
// asynchronous caller returns on the verdict while the kernel runs
// It writes every packet's descriptor as it goes, so the crypto kernel then
// runs from descriptors (its in-order classification -- the header, length
// and capacity loads -- is not repeated).  One thread per packet, one
// atomic per wave.  (A last-block ticket in place of k_io_publish cost
// 0.5 ms: every block's agent-scope release fence writes back L2 on gfx950.)
__global__ __launch_bounds__(256) void k_io_check(
    const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
    const uint32_t *cap, uint32_t n, const srtp_dev_stream_t *st,
    uint32_t *abort, srtp_dev_meta_t *meta)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const srtp_dev_stream_t &S = st[0];
    uint32_t seq0;
    uint64_t e0;
    const bool e0ok = srtp_inorder_head(S, in + in_off[0], false, seq0, e0);
    bool bad = false;
    if (i < n) {
        const uint64_t off = in_off[i];
        const uint32_t len = in_len[i];
        const srtp_dev_hdr_t h = srtp_parse_rtp(in + off, off, len);
        srtp_dev_meta_t m;
        bad = !srtp_inorder_desc(S, h, i, len, cap[i], seq0, e0, e0ok, false,
                                 m);
        meta[i] = m;
    }
    if (__ballot(bad) && (threadIdx.x & 63) == 0)
        atomicOr(abort, 1u);
}

// the checked verdict to host memory (asynchronous callers wait on it)
__global__ void k_io_publish(const uint32_t *abort, uint32_t *pub)
{
    publish_abort(pub, abort);
}

// The receive side of it (pp_unprotect_inorder): the crypto kernel
// verified and decrypted every packet of the run (auth[]); a rejected
// packet (auth_fail) changes no other packet's index -- every estimate is
// the same from the highest ACCEPTED index before it, each advance being
// 1 or more (rdbx.c:112-145) -- so, unless declined: the verdicts, the
// stream at the last accepted index with the window shifted to it and the
// accepted packets' bits set (rdbx.c:253-270, after the tag: srtp.c:
// 3157-3167), key uses (AES-ICM / HMAC the accepted packets, AES-GCM every
// packet: srtp_unprotect_aead counts before the tag), the failures counted
// for the host (their decryption is undone), the verdict published.
// Two launches: k_io_rx_status (one thread per packet: verdict, length,
// each block's failure count and first / last accepted position -- no
// atomics, so a forged-heavy batch costs no same-address serialisation) and
// k_io_rx_commit (one block: the sums, the gap check, the key uses, the
// window, the index, the publication).
constexpr uint32_t IO_NONE = 0xffffffffu;   // a block with no accepted packet

__global__ __launch_bounds__(256) void k_io_rx_status(
    const uint32_t *in_len, const uint8_t *auth, uint32_t n, uint32_t nblk,
    const srtp_dev_stream_t *st, const uint32_t *abort, uint32_t *brec,
    int32_t *status, uint32_t *out_len)
{
    if (*abort)   // grid-uniform
        return;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool f = false, a = false;
    if (i < n) {
        if (auth[i]) {
            status[i] = 0;
            out_len[i] = in_len[i] - st[0].trailer;
            a = true;
        } else {
            status[i] = 7;   // srtp_err_status_auth_fail
            f = true;
        }
    }
    __shared__ uint32_t s_f[4], s_lo[4], s_hi[4];
    const uint64_t m = __ballot(f), am = __ballot(a);
    const uint32_t w = threadIdx.x >> 6,
                   wbase = blockIdx.x * blockDim.x + 64 * w;
    if ((threadIdx.x & 63) == 0) {
        s_f[w] = (uint32_t)__popcll(m);
        s_lo[w] = am ? wbase + (uint32_t)__ffsll((long long)am) - 1 : IO_NONE;
        s_hi[w] = am ? wbase + 63 - (uint32_t)__clzll((long long)am) : IO_NONE;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t lo = IO_NONE, hi = IO_NONE;
        for (int k = 0; k < 4; k++)
            if (s_lo[k] != IO_NONE) {
                if (lo == IO_NONE)
                    lo = s_lo[k];
                hi = s_hi[k];
            }
        brec[blockIdx.x] = s_f[0] + s_f[1] + s_f[2] + s_f[3];
        brec[nblk + blockIdx.x] = lo;
        brec[2 * nblk + blockIdx.x] = hi;
    }
}

// brec: nblk failure counts, then nblk first and nblk last accepted
// positions (IO_NONE: none).  Every packet's index is e_0 + i only while
// the packet lies less than 2^15 past the last accepted one (or past the
// stored index, position S.index - e_0 <= -1): beyond, index_guess
// (rdbx.c:112-145) from that top returns another ROC and the reference
// says replay_old or decrypts at another index.  So every gap between
// consecutive accepted positions, and the tail after the last, is checked;
// a batch with one of 2^15 or more is declined (AB_GAP) before anything is
// committed -- the chain form decides it packet by packet (k_pu_verdict1).
__global__ __launch_bounds__(1024) void k_io_rx_commit(
    const uint8_t *in, const uint64_t *in_off, const uint8_t *auth, uint32_t n,
    uint32_t nblk, srtp_dev_stream_t *st, uint32_t *win, uint32_t *abort,
    uint32_t *abort_next, const uint32_t *brec, uint32_t *nfail, uint32_t *pub,
    uint64_t *e0_run)
{
    const uint32_t t = threadIdx.x, T = blockDim.x;
    uint32_t ab = *abort;
    srtp_dev_stream_t &S = st[0];
    __shared__ uint32_t s_fail;
    __shared__ uint32_t s_win[SEQ_MEDIAN / 32];
    __shared__ int64_t s_scan[1024];
    if (t == 0)
        s_fail = 0;
    const uint32_t words = S.win_bits >> 5;
    const uint64_t old = S.index;
    uint32_t seq0;
    uint64_t e0;
    srtp_inorder_head(S, in + in_off[0], true, seq0, e0);
    // the stored index as a batch position: e_0 is its guess, >= old + 1
    const int64_t virt = (int64_t)old - (int64_t)e0;
    constexpr int64_t NO_POS = INT64_MIN;
    // this thread's run of block records, in batch order
    const uint32_t per = (nblk + T - 1) / T;
    const uint32_t r0 = t * per < nblk ? t * per : nblk;
    const uint32_t r1 = r0 + per < nblk ? r0 + per : nblk;
    uint32_t f = 0;
    int64_t cfirst = NO_POS, clast = NO_POS;
    bool gap = false;
    for (uint32_t b = r0; b < r1 && !ab; b++) {
        f += brec[b];
        const uint32_t lo = brec[nblk + b];
        if (lo == IO_NONE)
            continue;
        if (clast != NO_POS && (int64_t)lo - clast >= (int64_t)SEQ_MEDIAN)
            gap = true;
        if (cfirst == NO_POS)
            cfirst = lo;
        clast = brec[2 * nblk + b];
    }
    __syncthreads();   // s_fail zeroed
    if (f)
        atomicAdd(&s_fail, f);
    // inclusive max-scan of the runs' last accepted positions
    s_scan[t] = clast;
    __syncthreads();
    for (uint32_t d = 1; d < T; d <<= 1) {
        const int64_t v = t >= d ? s_scan[t - d] : NO_POS;
        __syncthreads();
        if (v > s_scan[t])
            s_scan[t] = v;
        __syncthreads();
    }
    int64_t before = t ? s_scan[t - 1] : NO_POS;
    if (before < virt)
        before = virt;
    if (cfirst != NO_POS && cfirst - before >= (int64_t)SEQ_MEDIAN)
        gap = true;
    int64_t lastpos = s_scan[T - 1];
    if (t == 0 && (int64_t)n - 1 - (lastpos < virt ? virt : lastpos) >=
                      (int64_t)SEQ_MEDIAN)
        gap = true;
    // every thread reads the same verdict, and no shared word is written
    // after it: a uniform decision
    if (__syncthreads_or(gap ? 1 : 0) && !ab)
        ab = AB_GAP;
    const uint32_t nf = s_fail;
    const int64_t last = lastpos;   // NO_POS: nothing accepted
    if (t == 0) {
        if (ab && !*abort)
            *abort = ab;   // declined: the host restores, the chain form runs
        *e0_run = e0;   // for the undo of the rejected packets
        if (!ab) {
            // key uses: AES-GCM every packet (srtp_unprotect_aead counts
            // before the tag), AES-ICM / HMAC the accepted ones
            S.uses += (S.flags & SRTP_DS_AEAD) ? n : n - nf;
            if (nf < n)
                S.dir |= SRTP_DIR_RX;
        }
    }
    if (!ab && last >= 0) {
        const uint64_t hi = e0 + (uint64_t)last;
        const uint64_t adv = hi - old;
        const uint32_t *w = win + S.win_off;
        for (uint32_t x = threadIdx.x; x < words; x += blockDim.x) {
            uint32_t v = 0;
            if (adv < S.win_bits) {
                const uint32_t b0 = (uint32_t)adv >> 5, bi = (uint32_t)adv & 31;
                const uint32_t a = x + b0 < words ? w[x + b0] : 0u;
                const uint32_t b = x + b0 + 1 < words ? w[x + b0 + 1] : 0u;
                v = bi ? (a >> bi) | (b << (32 - bi)) : a;
            }
            s_win[x] = v;
        }
        __syncthreads();
        // the accepted packets among the window's indices below hi
        const uint32_t span = (uint64_t)last + 1 < S.win_bits
                                  ? (uint32_t)last + 1 : S.win_bits;
        for (uint32_t k = threadIdx.x; k < span; k += blockDim.x) {
            const uint64_t j = (uint64_t)last - k;
            if (auth[j]) {
                const uint32_t bit = S.win_bits - 1 - k;
                atomicOr(&s_win[bit >> 5], 1u << (bit & 31));
            }
        }
        __syncthreads();
        for (uint32_t x = threadIdx.x; x < words; x += blockDim.x)
            win[S.win_off + x] = s_win[x];
        __syncthreads();
        if (threadIdx.x == 0)
            S.index = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        *nfail = nf;
        publish_nfail(pub, nf);
        if (pub)
            __hip_atomic_store(pub, ab, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        *abort_next = 0;   // the next batch's word (ch_abort pair)
    }
}

// ... declined: the descriptors of the packets the kernel encrypted (the
// same test as inorder_meta) for the keystream undo, and their trailer
// bytes back
__global__ void k_io_restore_meta(const uint8_t *in, const uint64_t *in_off,
                                  const uint32_t *in_len, const uint32_t *cap,
                                  uint32_t n, const srtp_dev_stream_t *st,
                                  const uint8_t *auth, srtp_dev_meta_t *meta,
                                  int rx, const uint64_t *e0_run)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const srtp_dev_stream_t S = st[0];
    uint32_t seq0;
    uint64_t e0;
    bool e0ok = srtp_inorder_head(S, in + in_off[0], rx != 0, seq0, e0);
    if (e0_run) {
        // a committed batch: the stream has moved on; e_0 as the kernel
        // had it
        e0 = *e0_run;
        e0ok = true;
    }
    const uint64_t off = in_off[i];
    const uint32_t len = in_len[i];
    const srtp_dev_hdr_t h = srtp_parse_rtp(in + off, off, len);
    srtp_dev_meta_t m;
    // (receive, accepted batch: only the packets whose tag failed)
    if (!srtp_inorder_desc(S, h, i, len, cap[i], seq0, e0, e0ok, rx != 0, m) ||
        (auth && auth[i]))
        m.info = 0xff0000u;
    meta[i] = m;
}

__global__ void k_io_restore_tail(uint8_t *arena, const uint64_t *off,
                                  const uint32_t *in_len,
                                  const srtp_dev_stream_t *st,
                                  const srtp_dev_meta_t *meta,
                                  const uint32_t (*tsave)[4], uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || SRTP_META_STATUS(meta[i].info))
        return;
    const uint32_t tn = st[0].trailer < 16 ? st[0].trailer : 16;
    uint8_t *p = arena + off[i] + in_len[i];
    for (uint32_t b = 0; b < tn; b++)
        p[b] = (uint8_t)(tsave[i][b >> 2] >> (8 * (b & 3)));
}

// MKI streams on protect (srtp.c:2536-2545, srtp_get_session_keys): every
// packet of an MKI stream runs on the master key its mki_index selects and
// is charged to that key (key.c:74-90).  After the pre-pass committed (the
// sorted / order-free / one-stream forms; not the fused ones), each packet
// whose stream the classification found -- the packets it charged to the
// stream -- moves its charge from `uses` to kuses[kbase + j], and a packet
// with a crypto descriptor takes key mkslot[kbase + j].  j is below every
// MKI stream's key count (the host checked).
__global__ void k_mki_keys(const uint8_t *in, const uint64_t *in_off,
                           const uint32_t *in_len, srtp_dev_stream_t *st,
                           const uint32_t *hkey, const uint32_t *hval,
                           uint32_t hmask, uint32_t n, const uint8_t *mki,
                           const uint32_t *mkslot, unsigned long long *kuses,
                           srtp_dev_meta_t *meta, const uint32_t *abort)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || *abort)
        return;
    const uint64_t off = in_off[i];
    const srtp_dev_hdr_t h = srtp_parse_rtp(in + off, off, in_len[i]);
    if (h.enc_start >> 24)
        return;   // no stream touched
    uint32_t sid = NOCHAIN;
    uint32_t p = map_hash(h.ssrc, hmask);
    for (uint32_t probe = 0; probe <= hmask; probe++) {
        const uint32_t v = hval[p];
        if (v == NOCHAIN)
            break;
        if (hkey[p] == h.ssrc) {
            sid = v;
            break;
        }
        p = (p + 1) & hmask;
    }
    if (sid == NOCHAIN || st[sid].nkeys == 0)
        return;
    const uint32_t k = st[sid].kbase + mki[i];
    atomicAdd(&kuses[k], 1ull);
    atomicAdd((unsigned long long *)&st[sid].uses, ~0ull);   // - 1
    if (SRTP_META_STATUS(meta[i].info) == 0)
        meta[i].key = mkslot[k];
}

// MKI streams on unprotect (srtp.c:1961-2016 per packet, 2908; key.c:74-90
// per master key): after the commit, every packet the commit charged to its
// stream's `uses` -- AES-ICM / HMAC the accepted ones, AES-GCM every
// candidate past the replay check (srtp_unprotect_aead counts before the
// tag) -- moves that charge to kuses[kbase + j], j the key its MKI selected;
// a bad_mki packet's charge (AES-GCM candidates) is dropped: the reference
// returns before it uses a key.  The final statuses say which: 0 accepted,
// 7 auth_fail, 25 bad_mki.  ab_a / ab_b: the batch's abort words (nothing
// was committed when one is set).
__global__ void k_mki_rx_charge(const uint8_t *in, const uint64_t *in_off,
                                const uint32_t *in_len, srtp_dev_stream_t *st,
                                const uint32_t *hkey, const uint32_t *hval,
                                uint32_t hmask, uint32_t n, const uint8_t *rxj,
                                unsigned long long *kuses,
                                const int32_t *status, const uint32_t *ab_a,
                                const uint32_t *ab_b)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || *ab_a || (ab_b && *ab_b))
        return;
    const int32_t v = status[i];
    if (v != 0 && v != 7 && v != (int32_t)ST_BAD_MKI)
        return;
    const uint64_t off = in_off[i];
    const srtp_dev_hdr_t h = srtp_parse_rtp(in + off, off, in_len[i]);
    if (h.enc_start >> 24)
        return;
    const uint32_t sid = lookup_sid(hkey, hval, hmask, h.ssrc);
    if (sid == NOCHAIN || !st[sid].mki)
        return;
    const bool aead = (st[sid].flags & SRTP_DS_AEAD) != 0;
    if (v != 0 && !aead)
        return;   // not charged
    atomicAdd((unsigned long long *)&st[sid].uses, ~0ull);   // - 1
    if (v != (int32_t)ST_BAD_MKI)
        atomicAdd(&kuses[st[sid].kbase + rxj[i]], 1ull);
}

// An in-place batch classified inside the crypto kernel that the pre-pass
// then declined: the bytes past every encrypted packet that its tag
// overwrote come back (its payload is restored by k_undo_wave)
__global__ void k_pp_tail_restore(uint8_t *arena, const uint64_t *off,
                                  const uint32_t *in_len,
                                  const srtp_dev_stream_t *st,
                                  const srtp_dev_meta_t *meta,
                                  const FzRec *rec,
                                  const uint32_t (*tsave)[4], uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || SRTP_META_STATUS(meta[i].info))
        return;
    const uint32_t len = in_len[i], tn = st[rec[i].skey].trailer;
    uint8_t *t = arena + off[i] + len;
    for (uint32_t b = 0; b < tn && b < 16; b++)
        t[b] = (uint8_t)(tsave[i][b >> 2] >> (8 * (b & 3)));
}

// ---------------------------------------------------------------------------
// Pending ROCs (srtp_dev.h srtp_gpu_pp_pend_*; srtp.c:2038-2081, 2674-2678,
// 3161-3167, 5137-5167)
__global__ void k_pend_reset(const uint32_t *sids, uint32_t np, uint32_t *first,
                             unsigned long long *emin, unsigned long long *emax)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= np)
        return;
    const uint32_t s = sids[k];
    first[s] = NOCHAIN;
    emin[s] = ~0ull;
    emax[s] = 0;
}

// every packet of a pending stream that reaches the index estimate: its
// position (the first in batch order wins) and pending_roc || seq.  Protect:
// the header parses, the capacity holds the trailer and the header the
// length (srtp_host.c pre_protect, srtp.c:2515-2600; fz_classify's order);
// unprotect: the header parses (a packet failing a length check sends the
// batch to the host in every device form)
__global__ void k_pend_scan(const uint8_t *in, const uint64_t *in_off,
                            const uint32_t *in_len, const uint32_t *cap,
                            const srtp_dev_stream_t *st, const uint32_t *hkey,
                            const uint32_t *hval, uint32_t hmask, uint32_t n,
                            int unprotect, uint32_t *first,
                            unsigned long long *emin, unsigned long long *emax)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint64_t off = in_off[i];
    const uint32_t len = in_len[i];
    const srtp_dev_hdr_t h = srtp_parse_rtp(in + off, off, len);
    if (h.enc_start >> 24)
        return;
    const uint32_t sid = srtp_map_lookup(hkey, hval, hmask, h.ssrc);
    if (sid == NOCHAIN)
        return;
    const srtp_dev_stream_t &S = st[sid];
    if (!(S.flags & SRTP_DS_PENDING))
        return;
    if (!unprotect && (cap[i] < len + S.trailer || h.enc_start > len))
        return;
    const uint64_t e = ((uint64_t)S.rsv << 16) | (h.seq_len & 0xffffu);
    atomicMin(&first[sid], i);
    atomicMin(&emin[sid], (unsigned long long)e);
    atomicMax(&emax[sid], (unsigned long long)e);
}

__global__ void k_pend_gather(const uint32_t *sids, uint32_t np,
                              const uint8_t *in, const uint64_t *in_off,
                              const srtp_dev_stream_t *st, const uint32_t *first,
                              const unsigned long long *emin,
                              const unsigned long long *emax,
                              srtp_pend_info_t *out)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= np)
        return;
    const uint32_t s = sids[k], f = first[s];
    srtp_pend_info_t r;
    r.first = f;
    r.rsv = 0;
    r.efirst = 0;
    r.emin = emin[s];
    r.emax = emax[s];
    r.index = st[s].index;
    if (f != NOCHAIN) {
        const uint32_t w0 = srtp_bswap32(*(const uint32_t *)(in + in_off[f]));
        r.efirst = ((uint64_t)st[s].rsv << 16) | (w0 & 0xffffu);
    }
    out[k] = r;
}

// the state after the first packet's reset, one packet earlier: index - 1,
// an empty window, no pending ROC; the replaced record and window kept
__global__ void k_pend_apply(const uint32_t *sids, const uint64_t *efirst,
                             uint32_t nr, srtp_dev_stream_t *st, uint32_t *win,
                             srtp_dev_stream_t *bak, uint32_t *bakwin)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nr)
        return;
    const uint32_t s = sids[k];
    srtp_dev_stream_t S = st[s];
    bak[k] = S;
    const uint32_t words = S.win_bits >> 5;
    for (uint32_t w = 0; w < words; w++) {
        bakwin[S.win_off + w] = win[S.win_off + w];
        win[S.win_off + w] = 0;
    }
    S.index = efirst[k] - 1;
    S.flags &= ~(uint32_t)SRTP_DS_PENDING;
    S.rsv = 0;
    st[s] = S;
}

__global__ void k_pend_restore(const uint32_t *sids, uint32_t nr,
                               srtp_dev_stream_t *st, uint32_t *win,
                               const srtp_dev_stream_t *bak,
                               const uint32_t *bakwin)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nr)
        return;
    const srtp_dev_stream_t S = bak[k];
    st[sids[k]] = S;
    const uint32_t words = S.win_bits >> 5;
    for (uint32_t w = 0; w < words; w++)
        win[S.win_off + w] = bakwin[S.win_off + w];
}

// unprotect: an applied stream's first packet must authenticate
__global__ void k_pend_authchk(const uint32_t *pos, uint32_t nr,
                               const uint8_t *auth, uint32_t *abort)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < nr && auth[pos[k]] != 1)
        atomicOr(abort, (uint32_t)AB_PENDING);
}

// ---------------------------------------------------------------------------
// Template clones (srtp_gpu_pp_clone; srtp_stream_clone, srtp.c:762-863).
// One thread per packet: a packet whose SSRC is in the hash is done; else
// the thread claims the empty slot its probe reaches (CAS of the value word
// to CL_CLAIMED), takes the next spare record, copies the template into it
// (fresh index and window), then publishes key and record id.  A thread
// that meets a claimed slot reads it again on its next pass, so threads of
// one wave never wait inside a branch for each other; every pass is bounded.
constexpr uint32_t CL_EMPTY = 0xffffffffu, CL_CLAIMED = 0xfffffffeu,
                   CL_OVERFLOW = 0xfffffffdu;

__global__ void k_clone_insert(const uint8_t *in, const uint64_t *in_off,
                               const uint32_t *in_len, uint32_t n,
                               uint32_t *hkey, uint32_t *hval, uint32_t hmask,
                               srtp_dev_stream_t *st, uint32_t *win,
                               srtp_dev_stream_t tmpl, uint32_t ns0,
                               uint32_t spare, uint32_t tw, uint32_t *ctl)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint64_t off = in_off[i];
    const srtp_dev_hdr_t h = srtp_parse_rtp(in + off, off, in_len[i]);
    if (h.enc_start >> 24)
        return;
    const uint32_t ssrc = h.ssrc;
    uint32_t p = map_hash(ssrc, hmask);
    for (uint32_t pass = 0, probe = 0; probe <= hmask; pass++) {
        if (pass > (1u << 22)) {
            atomicOr(&ctl[1], 2u);   // a claim never published: decline
            return;
        }
        const uint32_t v = __hip_atomic_load(&hval[p], __ATOMIC_ACQUIRE,
                                             __HIP_MEMORY_SCOPE_AGENT);
        if (v == CL_CLAIMED)
            continue;                // published on a later pass
        if (v != CL_EMPTY) {
            if (__hip_atomic_load(&hkey[p], __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT) == ssrc)
                return;              // known, or created by another thread
            p = (p + 1) & hmask;
            probe++;
            continue;
        }
        uint32_t exp = CL_EMPTY;
        if (!__hip_atomic_compare_exchange_strong(
                &hval[p], &exp, CL_CLAIMED, __ATOMIC_ACQ_REL,
                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            continue;                // another thread took the slot: again
        const uint32_t k = atomicAdd(&ctl[0], 1u);
        uint32_t id = CL_OVERFLOW;
        if (k < spare) {
            id = ns0 + k;
            srtp_dev_stream_t S = tmpl;
            S.ssrc = ssrc;
            S.win_off = tmpl.win_off + k * tw;
            S.index = 0;
            S.uses = 0;
            S.dir = 0;
            st[id] = S;
            for (uint32_t w = 0; w < tw; w++)
                win[S.win_off + w] = 0;
        } else {
            atomicOr(&ctl[1], 1u);   // out of spare records: decline
        }
        __hip_atomic_store(&hkey[p], ssrc, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&hval[p], id, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
}

// Fused order-free form (IcmFused): the per-stream aggregates start at
// zero / empty (the bitmaps are zero between batches)
__global__ void k_fz_reset(uint32_t *abort, unsigned long long *cnt,
                           unsigned long long *new_index,
                           unsigned long long *emin,
                           unsigned long long *hicand, uint32_t *nfail,
                           uint32_t *glist, uint32_t ns)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s == 0) {
        *abort = 0;
        if (nfail)
            *nfail = 0;
        glist[0] = 0;
    }
    if (s >= ns)
        return;
    cnt[s] = 0;
    new_index[s] = 0;
    emin[s] = ~0ull;
    if (hicand)
        hicand[s] = 0;
}

// ... per stream, after the crypto: the conditions of the order-free form
// (k_pp_usetbits restated over the aggregates: every chain index within one
// window of the highest -- else AB_ORDER, the sorted path decides -- and as
// many distinct indices as chain packets -- else AB_SEQUENCE, two packets
// share an index: host), the window shifted by the advance with the batch's
// bits (rdbx_add, rdbx.c:253-270), and the bitmap cleared for the next batch
__global__ void k_fz_stream(const srtp_dev_stream_t *st, uint32_t ns,
                            const unsigned long long *cnt,
                            const unsigned long long *new_index,
                            const unsigned long long *emin, uint32_t *bmap,
                            const uint32_t *win, uint32_t *wnew,
                            uint32_t *abort)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ns)
        return;
    const uint32_t chain = (uint32_t)(cnt[s] >> 32);
    if (!chain)
        return;
    const srtp_dev_stream_t S = st[s];
    const uint64_t hi = new_index[s], lo = emin[s];
    const uint32_t bits = S.win_bits, words = bits >> 5;
    const uint32_t M = bits > 32 ? 2u << (31 - __clz(bits - 1)) : 32u;
    const uint32_t mw = M >> 5;
    uint32_t *bm = bmap + 2 * S.win_off;
    const uint32_t *w = win + S.win_off;
    uint32_t *o = wnew + S.win_off;
    const uint64_t adv = hi - S.index;
    // window bit p <-> index hi - bits + 1 + p <-> bitmap residue of it
    const uint32_t base = (uint32_t)(hi - bits + 1);
    uint32_t seen = 0;
    for (uint32_t j = 0; j < words; j++) {
        uint32_t v = 0;
        if (adv < bits) {
            const uint32_t q = (uint32_t)adv >> 5, bi = (uint32_t)adv & 31;
            const uint32_t a = j + q < words ? w[j + q] : 0u;
            const uint32_t b = j + q + 1 < words ? w[j + q + 1] : 0u;
            v = bi ? (a >> bi) | (b << (32 - bi)) : a;
        }
        const uint32_t r0 = (base + 32 * j) & (M - 1), sh = r0 & 31;
        const uint32_t b0 = bm[r0 >> 5], b1 = bm[((r0 >> 5) + 1) & (mw - 1)];
        const uint32_t x = sh ? (b0 >> sh) | (b1 << (32 - sh)) : b0;
        seen += __popc(x);
        o[j] = v | x;
    }
    for (uint32_t j = 0; j < mw; j++)
        bm[j] = 0;
    if (hi - lo >= bits)
        atomicOr(abort, AB_ORDER);
    else if (seen != chain)
        atomicOr(abort, AB_SEQUENCE);   // two packets with one index: host
}

// ... then, unless the batch was declined, every touched stream's state
// (the packets' statuses and lengths came from the crypto kernel)
__global__ void k_fz_commit(srtp_dev_stream_t *st, uint32_t ns,
                            const unsigned long long *cnt,
                            const unsigned long long *new_index,
                            const uint32_t *wnew, uint32_t *win,
                            const uint32_t *abort, uint32_t *pub)
{
    publish_abort(pub, abort);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (*abort || i >= ns)
        return;
    const uint32_t c = (uint32_t)cnt[i];
    if (!c)
        return;
    st[i].uses += c;
    st[i].dir |= SRTP_DIR_TX;
    const uint64_t ni = new_index[i];
    if (ni == 0)
        return;
    st[i].index = ni;
    const uint32_t off = st[i].win_off, words = st[i].win_bits >> 5;
    for (uint32_t w = 0; w < words; w++)
        win[off + w] = wnew[off + w];
}

// Fused order-free unprotect (pp_unprotect_fused), per stream after the
// crypto: k_pp_usetbits' conditions over the candidates (every index above
// the stored one -- checked in the kernel -- and within one window of the
// highest candidate, else AB_ORDER; as many distinct indices as candidates,
// else AB_SEQUENCE: a duplicate, whose verdict depends on the order), then
// the window (rdbx_add after the tag check, srtp.c:3157-3167): the stored
// one shifted to the highest AUTHENTICATED index, one bit per authenticated
// packet; both bitmaps cleared
__global__ void k_fzu_stream(const srtp_dev_stream_t *st, uint32_t ns,
                             const unsigned long long *cnt,
                             const unsigned long long *new_index,
                             const unsigned long long *hicand,
                             const unsigned long long *emin, uint32_t *bmap,
                             uint32_t *bmap2, const uint32_t *win,
                             uint32_t *wnew, uint32_t *abort)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ns)
        return;
    const uint32_t cand = (uint32_t)(cnt[s] >> 32), acc = (uint32_t)cnt[s];
    if (!cand)
        return;
    const srtp_dev_stream_t S = st[s];
    const uint32_t bits = S.win_bits, words = bits >> 5;
    const uint32_t M = bits > 32 ? 2u << (31 - __clz(bits - 1)) : 32u;
    const uint32_t mw = M >> 5;
    uint32_t *bc = bmap + 2 * S.win_off, *ba = bmap2 + 2 * S.win_off;
    // candidates: distinct within one window of the highest
    const uint64_t hc = hicand[s];
    uint32_t seen = 0;
    {
        const uint32_t base = (uint32_t)(hc - bits + 1);
        for (uint32_t j = 0; j < words; j++) {
            const uint32_t r0 = (base + 32 * j) & (M - 1), sh = r0 & 31;
            const uint32_t b0 = bc[r0 >> 5], b1 = bc[((r0 >> 5) + 1) & (mw - 1)];
            seen += __popc(sh ? (b0 >> sh) | (b1 << (32 - sh)) : b0);
        }
    }
    if (hc - emin[s] >= bits)
        atomicOr(abort, AB_ORDER);
    else if (seen != cand)
        atomicOr(abort, AB_SEQUENCE);
    if (acc) {
        const uint64_t hi = new_index[s], adv = hi - S.index;
        const uint32_t base = (uint32_t)(hi - bits + 1);
        const uint32_t *w = win + S.win_off;
        uint32_t *o = wnew + S.win_off;
        for (uint32_t j = 0; j < words; j++) {
            uint32_t v = 0;
            if (adv < bits) {
                const uint32_t q = (uint32_t)adv >> 5, bi = (uint32_t)adv & 31;
                const uint32_t a = j + q < words ? w[j + q] : 0u;
                const uint32_t b = j + q + 1 < words ? w[j + q + 1] : 0u;
                v = bi ? (a >> bi) | (b << (32 - bi)) : a;
            }
            const uint32_t r0 = (base + 32 * j) & (M - 1), sh = r0 & 31;
            const uint32_t b0 = ba[r0 >> 5], b1 = ba[((r0 >> 5) + 1) & (mw - 1)];
            o[j] = v | (sh ? (b0 >> sh) | (b1 << (32 - sh)) : b0);
        }
    }
    for (uint32_t j = 0; j < mw; j++) {
        bc[j] = 0;
        ba[j] = 0;
    }
}

// ... and unless the batch was declined, the streams (k_pu_commit_stream:
// key uses -- AES-GCM every candidate, AES-ICM the authenticated ones --,
// index and window when something authenticated)
__global__ void k_fzu_commit(srtp_dev_stream_t *st, uint32_t ns,
                             const unsigned long long *cnt,
                             const unsigned long long *new_index,
                             const uint32_t *wnew, uint32_t *win,
                             const uint32_t *abort, uint32_t *pub,
                             const uint32_t *nfail)
{
    publish_abort(pub, abort);
    if (blockIdx.x == 0 && threadIdx.x == 0)
        publish_nfail(pub, *nfail);   // final: the crypto kernel has ended
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (*abort || s >= ns)
        return;
    const uint64_t c = cnt[s];
    if (!c)
        return;
    st[s].uses += (st[s].flags & SRTP_DS_AEAD) ? (uint32_t)(c >> 32)
                                               : (uint32_t)c;
    const uint64_t ni = new_index[s];
    if (ni == 0)
        return;
    st[s].dir |= SRTP_DIR_RX;
    st[s].index = ni;
    const uint32_t off = st[s].win_off, words = st[s].win_bits >> 5;
    for (uint32_t w = 0; w < words; w++)
        win[off + w] = wnew[off + w];
}

// ... and a declined batch's descriptors, as k_icm_hmac had them, for the
// undo (k_undo_wave re-applies the keystream); the capacities come back
__global__ void k_fz_meta(const uint8_t *in, const uint64_t *in_off,
                          const uint32_t *in_len, const FzRec *rec,
                          const srtp_dev_stream_t *st, uint32_t n,
                          srtp_dev_meta_t *meta, uint32_t *cap,
                          int unprotect, const int32_t *only_status)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    srtp_dev_meta_t m;
    m.key = 0;
    m.roc = 0;
    m.len = 0;
    m.info = 0xff0000u;
    const uint4 r = *(const uint4 *)&rec[i];
    const uint32_t s = r.z, code = r.y >> 16;
    // only_status: just the packets with that status (unprotect: the
    // candidates whose tag check failed, status 7), capacities untouched
    if (s != NOCHAIN && code == 0 &&
        (!only_status || only_status[i] == 7)) {
        const uint64_t off = in_off[i];
        const srtp_dev_hdr_t h = srtp_parse_rtp(in + off, off, in_len[i]);
        m.key = st[s].key;
        m.roc = (r.x >> 16) | ((r.y & 0xffffu) << 16);
        m.info = h.enc_start | (st[s].variant << 24);
        m.len = in_len[i] - (unprotect ? st[s].trailer : 0u);
        if (!only_status)
            cap[i] = r.w;
    }
    meta[i] = m;
}

// ---------------------------------------------------------------------------
// Unprotect (srtp_unprotect_device): the order-free form of the receive
// pre-pass (srtp.c:2820-3172, srtp_host.c pre_unprotect / post_unprotect).
// Candidates are packets whose stream is known and eligible, whose index
// (guessed from the stored index) is above it, and that pass every length
// check; a packet failing a length check aborts the batch to the host (its
// status would depend on the replay check, srtp.c:2905-2990).  After the
// crypto kernel has verified the tags, only authenticated packets move the
// replay window and index (rdbx_add after the tag check, srtp.c:3157-3167).


__global__ void k_pu_classify(ClassifyArgs A)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t key = NOCHAIN;
    uint64_t e = 0;
    if (i < A.n) {
        const uint64_t off = A.in_off[i];
        const uint32_t len = A.in_len[i];
        const srtp_dev_hdr_t h = srtp_parse_rtp(A.in + off, off, len);
        A.hdr[i] = h;
        if (!A.est)   // the sorted chain form sorts it; order-free: identity
            A.perm[i] = i;
        uint32_t code = 0;
        if (h.enc_start >> 24) {
            code = h.enc_start >> 24;   // header does not parse: no stream
        } else {
            const uint32_t sid = lookup_sid(A.hkey, A.hval, A.hmask, h.ssrc);
            if (sid == NOCHAIN) {
                atomicOr(A.abort, AB_UNKNOWN_SSRC);   // template clone: host
            } else {
                const srtp_dev_stream_t &S = A.st[sid];
                const uint32_t tag = S.trailer;       // tag + MKI
                if (!(S.flags & SRTP_DS_RX_ELIGIBLE) || (S.dir & SRTP_DIR_TX))
                    atomicOr(A.abort, AB_INELIGIBLE);
                // srtp_host.c un_static (srtp.c:2905-2990, 2298-2352)
                if (len < tag || h.enc_start > len - tag ||
                    ((S.flags & SRTP_DS_AEAD) && len - h.enc_start < tag) ||
                    A.cap[i] < len - tag ||
                    ((S.flags & SRTP_DS_ICM_CONF) &&
                     (len - tag - h.enc_start + 15) / 16 > 0xffffu)) {
                    atomicOr(A.abort, AB_STATIC);
                } else {
                    if (S.mki)   // the key of the packet's MKI (k_pu_meta)
                        A.rxj[i] = (uint8_t)mki_match(A.keys, A.mkslot, S,
                                                      A.in + off, len);
                    key = sid;
                    if (A.est) {   // order-free form
                        const uint32_t seq = h.seq_len & 0xffffu;
                        if (guess_index(S.index, seq, &e) < 1)
                            atomicOr(A.abort, AB_ORDER);
                        A.est[i] = e;
                    }
                }
            }
        }
        A.pstat[i] = code;
        A.skey[i] = key;
    }
    if (A.est)
        agg_stream(key, e, A.bcount, A.new_index);
}

// The kernels below walk position k of an order: the packet order itself
// for the order-free form (perm = identity, est per packet), or the stable
// stream-sorted order of the chain form (perm2, est per sorted position).

// meta of every candidate for the crypto kernel (all others skipped); on an
// abort every packet is skipped, so the undo pass after the crypto is a
// no-op too
__global__ void k_pu_meta(const uint32_t *skey, const uint32_t *perm,
                          const uint64_t *est, const srtp_dev_hdr_t *hdr,
                          const srtp_dev_stream_t *st, uint32_t ns, uint32_t n,
                          const uint32_t *abort, srtp_dev_meta_t *meta,
                          uint8_t *auth, const uint32_t *mkslot,
                          const uint8_t *rxj)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n)
        return;
    const uint32_t i = perm ? perm[k] : k;   // null: the identity
    srtp_dev_meta_t m;
    m.key = 0;
    m.roc = 0;
    m.len = 0;
    m.info = 0xff0000u;
    const uint32_t s = skey[k];
    uint8_t a = 1;   // kernels without a tag check leave it: accepted
    if (!*abort && s < ns) {
        const srtp_dev_stream_t &S = st[s];
        const srtp_dev_hdr_t h = hdr[i];
        const uint32_t j = S.mki ? rxj[i] : 0u;
        if (j == MKI_NONE) {
            a = AUTH_BAD_MKI;   // no key: no crypto, verdict bad_mki
        } else {
            m.key = S.mki ? mkslot[S.kbase + j] : S.key;
            m.roc = (uint32_t)(est[k] >> 16);
            m.info = h.enc_start | (S.variant << 24);
            m.len = h.len - S.trailer;
        }
    }
    meta[i] = m;
    auth[i] = a;
}

// chain form: the reference guesses each index from the highest ACCEPTED
// one before it (top), not from the previous packet.  top comes from an
// exclusive max-scan of the authenticated estimates; every packet's guess
// from its top must equal the chain's estimate (it does unless a run of
// rejected packets spans 2^15 indices, or a fresh stream's first accepted
// packet is preceded by rejected ones across a wrap); est > top always
// holds (the chain increases), so no packet is old.  A mismatch sends the
// batch to the host.
__global__ void k_pu_accepted_est(const uint32_t *skey2, const uint32_t *perm2,
                                  const uint64_t *est, const uint8_t *auth,
                                  uint32_t ns, uint32_t n, uint64_t *val)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n)
        return;
    val[k] = skey2[k] < ns && auth[perm2[k]] == 1 ? est[k] : 0;
}

__global__ void k_pu_top_check(const uint32_t *skey2, const uint32_t *perm2,
                               const srtp_dev_hdr_t *hdr, const uint64_t *est,
                               const uint64_t *top, const srtp_dev_stream_t *st,
                               uint32_t ns, uint32_t n, uint32_t *abort)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n)
        return;
    const uint32_t s = skey2[k];
    if (s >= ns)
        return;
    // top[k]: exclusive scan restarting (at 0) on each stream
    uint64_t t = top[k];
    if (t < st[s].index)
        t = st[s].index;
    uint64_t g;
    guess_index(t, hdr[perm2[k]].seq_len & 0xffffu, &g);
    if (g != est[k])
        atomicOr(abort, AB_ORDER);
}

// the verdicts: status / length per packet, the authenticated packets'
// per-stream count and highest index; the meta of authenticated packets
// is cleared so that the undo pass restores only the rejected ones (after
// an abort nothing is cleared: the undo restores every packet for the host)
__global__ __launch_bounds__(1024) void k_pu_accept(const uint32_t *skey, const uint32_t *perm,
                            const uint64_t *est, const uint32_t *pstat,
                            const srtp_dev_hdr_t *hdr,
                            const srtp_dev_stream_t *st, uint32_t ns,
                            uint32_t n, const uint32_t *abort,
                            const uint8_t *auth, srtp_dev_meta_t *meta,
                            int32_t *status, uint32_t *out_len,
                            uint32_t *bcount2,
                            unsigned long long *new_index2)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = k < n && !*abort;
    uint32_t key = NOCHAIN;
    uint64_t e = 0;
    if (live) {
        const uint32_t i = perm ? perm[k] : k;   // null: the identity
        const uint32_t s = skey[k];
        if (s >= ns) {
            status[i] = (int32_t)pstat[i];   // header errors; out_len kept
        } else if (auth[i] == 1) {
            key = s;
            e = est[k];
            status[i] = 0;
            out_len[i] = hdr[i].len - st[s].trailer;
            meta[i].info = 0xff0000u;        // keep: nothing to undo
        } else {
            // srtp_err_status_auth_fail, or bad_mki (no crypto ran)
            status[i] = auth[i] == AUTH_BAD_MKI ? (int32_t)ST_BAD_MKI : 7;
        }
    }
    agg_stream(key, e, bcount2, new_index2);
}

// the authenticated packets' replay bits still inside the window shifted
// to their highest index
__global__ void k_pu_setbits(const uint32_t *skey, const uint32_t *perm,
                             const uint64_t *est, const srtp_dev_stream_t *st,
                             uint32_t ns, uint32_t n, const uint32_t *abort,
                             const uint8_t *auth, const uint64_t *new_index2,
                             uint32_t *wnew)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n || *abort)
        return;
    const uint32_t s = skey[k];
    if (s >= ns || auth[perm ? perm[k] : k] != 1)
        return;
    const uint32_t bits = st[s].win_bits;
    const uint64_t dist = new_index2[s] - est[k];
    if (dist < bits) {
        const uint32_t bit = bits - 1 - (uint32_t)dist;
        atomicOr(&wnew[st[s].win_off + (bit >> 5)], 1u << (bit & 31));
    }
}

__global__ void k_pu_commit_stream(srtp_dev_stream_t *st, uint32_t ns,
                                   const uint64_t *new_index2,
                                   const uint32_t *bcount,
                                   const uint32_t *bcount2,
                                   const uint32_t *wnew, uint32_t *win,
                                   const uint32_t *abort, uint32_t *pub)
{
    publish_abort(pub, abort);
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ns || *abort)
        return;
    // key usage: AES-GCM counts every packet that reached the tag check
    // (srtp_unprotect_aead), AES-ICM / HMAC the authenticated ones
    st[s].uses += (st[s].flags & SRTP_DS_AEAD) ? bcount[s] : bcount2[s];
    const uint64_t ni = new_index2[s];
    if (ni == 0)
        return;
    st[s].dir |= SRTP_DIR_RX;
    st[s].index = ni;
    const uint32_t off = st[s].win_off, words = st[s].win_bits >> 5;
    for (uint32_t w = 0; w < words; w++)
        win[off + w] = wnew[off + w];
}

// ---------------------------------------------------------------------------
// The chain form of ONE stream in two launches (the sender's common case,
// BASELINE configs[1] / configs[2]).  k_pp_chain1 parses every header,
// classifies the packet (classify_one's checks), and computes every chain
// packet's 48-bit index as the stored index's guess for the batch's first
// chain packet plus the sum of the 16-bit advances before it (the reference's
// per-packet index_guess, rdbx.c:112-145, when every advance is in
// [1, 2^15)) -- a single-pass scan with decoupled look-back over tiles of
// 1024 packets taken in dispatch order.  k_pp_chain1_commit then writes the
// statuses and lengths, and its block 0 the stream: index, key uses, the
// window shifted by the advance with one bit per chain packet inside it
// (rdbx_add, crypto/replay/rdbx.c:253-270), the host's abort word, and the
// reset of the look-back state for the next batch.
// tiles of 4096 packets: 1024 threads x 4, all of a thread's offset loads,
// then all of its header loads in flight (256 tiles for 2^20 packets: one
// round of workgroups on the 256 CUs); the commit kernel uses 256-thread
// blocks
#ifndef CH_THREADS_N
#define CH_THREADS_N 1024
#endif
#ifndef CH_ITEMS_N
#define CH_ITEMS_N 4
#endif
constexpr int CH_THREADS = CH_THREADS_N;
constexpr int CH_ITEMS = CH_ITEMS_N;
constexpr int CH_TILE = CH_THREADS * CH_ITEMS;
constexpr int CH_COMMIT_THREADS = 256;
// look-back word: [63:62] 1 = tile aggregate, 2 = inclusive prefix; [61] a
// chain packet seen; aggregate: [60:45] first seq, [44:29] last seq, [28:0]
// sum of the advances inside; prefix: [47:0] index of the last chain packet
constexpr uint64_t CH_AGG = 1ull << 62, CH_PRE = 2ull << 62,
                   CH_HAS = 1ull << 61, CH_FLAGS = 3ull << 62;
// chain aggregate of a run of packets: has a chain packet, the first and
// last chain packets' sequence numbers, the sum of the advances between
// consecutive chain packets inside the run.  The sum is 64-bit: one tile's
// is below 2^27 (4095 advances < 2^15, the 29-bit field of a published
// aggregate), but the look-back combines any number of tiles, and a valid
// sender chain of large advances passes 2^32 after ~32 tiles.
struct ChAgg {
    uint32_t has, first, last;
    uint64_t internal;
};
static_assert(CH_TILE - 1 < (1 << 14), "a tile's advance sum fits 29 bits");
// k_pp_chain1's look-back words are allocated per srtp_scan::TILE packets
static_assert(CH_TILE >= srtp_scan::TILE, "ch_tile sized by srtp_scan::TILE");

__device__ __forceinline__ ChAgg ch_none() { return ChAgg{ 0, 0, 0, 0 }; }

// advance from the previous chain packet, flagged outside [1, 2^15)
__device__ __forceinline__ uint32_t ch_adv(uint32_t from, uint32_t to,
                                           uint32_t *bad)
{
    const uint32_t d = (to - from) & 0xffffu;
    if (d == 0 || d >= SEQ_MEDIAN)
        *bad = 1;
    return d;
}

__device__ __forceinline__ ChAgg ch_combine(const ChAgg &a, const ChAgg &b,
                                            uint32_t *bad)
{
    if (!a.has)
        return b;
    if (!b.has)
        return a;
    return ChAgg{ 1, a.first, b.last,
                  a.internal + ch_adv(a.last, b.first, bad) + b.internal };
}

// a prefix state (has, index of the last chain packet) followed by a run
__device__ __forceinline__ void ch_apply(uint32_t &has, uint64_t &idx,
                                         const ChAgg &a, uint64_t stored,
                                         uint32_t *bad)
{
    if (!a.has)
        return;
    if (has) {
        idx += ch_adv((uint32_t)idx & 0xffffu, a.first, bad) + a.internal;
    } else {
        uint64_t e;
        if (guess_index(stored, a.first, &e) < 1)
            *bad = 1;   // at or below the stored index: the host decides
        idx = e + a.internal;
        has = 1;
    }
}

struct Chain1Args {
    ClassifyArgs C;          // in, offsets, lengths, capacities, streams, map
    uint64_t *tile;          // look-back words, zero at entry
    uint32_t *ctl;           // [0] next tile, [1] key uses
    uint32_t *abort;         // this batch's abort word, zero at entry
    uint32_t ntiles;
};

__device__ __forceinline__ uint64_t ch_pack_agg(const ChAgg &a)
{
    return CH_AGG | (a.has ? CH_HAS : 0) | ((uint64_t)a.first << 45) |
           ((uint64_t)a.last << 29) | (a.internal & 0x1fffffffu);
}

__device__ __forceinline__ ChAgg ch_unpack_agg(uint64_t v)
{
    return ChAgg{ (v & CH_HAS) ? 1u : 0u, (uint32_t)(v >> 45) & 0xffffu,
                  (uint32_t)(v >> 29) & 0xffffu, v & 0x1fffffffull };
}

__device__ __forceinline__ ChAgg ch_shfl_down(const ChAgg &a, int d)
{
    return ChAgg{ (uint32_t)__shfl_down((int)a.has, d),
                  (uint32_t)__shfl_down((int)a.first, d),
                  (uint32_t)__shfl_down((int)a.last, d),
                  (uint64_t)__shfl_down((long long)a.internal, d) };
}

// wave 0 of a tile: the published state of the tiles before it, 64 at a
// time (lane l reads tile j0 - l): the aggregates after the nearest
// inclusive prefix are combined in tile order by a shuffle reduction.
// Returns (has, index of the last chain packet) before the tile.
__device__ void ch_lookback(const uint64_t *tile, uint32_t t, uint64_t stored,
                            uint32_t &has, uint64_t &idx, uint32_t *bad)
{
    const int lane = threadIdx.x & 63;
    ChAgg suf = ch_none();   // combined aggregates after the prefix found
    has = 0;
    idx = 0;
    for (int64_t j0 = (int64_t)t - 1; j0 >= 0; j0 -= 64) {
        const int64_t j = j0 - lane;
        uint64_t v = CH_PRE;   // before tile 0: the stored state
        if (j >= 0)
            while (!((v = __hip_atomic_load(&tile[j], __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT)) &
                     CH_FLAGS))
                __builtin_amdgcn_s_sleep(1);
        const uint64_t pm = __ballot((v & CH_FLAGS) == CH_PRE);
        const int fl = pm ? __ffsll((unsigned long long)pm) - 1 : 64;
        // lanes below fl: aggregates, lane fl - 1 the earliest tile
        ChAgg a = lane < fl ? ch_unpack_agg(v) : ch_none();
        for (int d = 1; d < 64; d <<= 1) {
            const ChAgg o = ch_shfl_down(a, d);   // an earlier tile
            if (lane + d < 64)
                a = ch_combine(o, a, bad);
        }
        // lane 0 holds the aggregates of lanes [0, fl) in tile order
        const ChAgg w{ (uint32_t)__shfl((int)a.has, 0),
                       (uint32_t)__shfl((int)a.first, 0),
                       (uint32_t)__shfl((int)a.last, 0),
                       (uint64_t)__shfl((long long)a.internal, 0) };
        suf = ch_combine(w, suf, bad);
        if (pm) {
            const uint64_t pv = (uint64_t)__shfl((long long)v, fl);
            has = (pv & CH_HAS) ? 1u : 0u;
            idx = pv & 0xffffffffffffull;
            break;
        }
    }
    ch_apply(has, idx, suf, stored, bad);
}

__device__ __forceinline__ ChAgg ch_shfl_up(const ChAgg &a, int d)
{
    return ChAgg{ (uint32_t)__shfl_up((int)a.has, d),
                  (uint32_t)__shfl_up((int)a.first, d),
                  (uint32_t)__shfl_up((int)a.last, d),
                  (uint64_t)__shfl_up((long long)a.internal, d) };
}

// inclusive scan over the wave's lanes in lane order
__device__ __forceinline__ ChAgg ch_wave_scan(ChAgg a, uint32_t *bad)
{
    const int lane = threadIdx.x & 63;
    for (int d = 1; d < 64; d <<= 1) {
        const ChAgg o = ch_shfl_up(a, d);   // an earlier lane
        if (lane >= d)
            a = ch_combine(o, a, bad);
    }
    return a;
}

__global__ __launch_bounds__(CH_THREADS) void k_pp_chain1(Chain1Args A)
{
    const ClassifyArgs &C = A.C;
    __shared__ uint32_t s_tile, s_has, s_uses, s_abort;
    __shared__ uint64_t s_idx;
    __shared__ ChAgg s_w[CH_THREADS / 64];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t == 0) {
        s_tile = atomicAdd(&A.ctl[0], 1u);   // dispatch order: look-back safe
        s_uses = 0;
        s_abort = 0;
    }
    __syncthreads();
    const uint32_t tile = s_tile;
    // one stream: its record and its one SSRC (the map's only entry)
    const srtp_dev_stream_t S = C.st[0];
    const uint64_t stored = S.index;
    const uint32_t base = tile * CH_TILE + t * CH_ITEMS;
    uint32_t bad = 0, uses = 0, abort = 0, chain = 0;
    uint64_t off[CH_ITEMS];
    uint32_t len[CH_ITEMS], cap[CH_ITEMS], code[CH_ITEMS], seq[CH_ITEMS];
    srtp_dev_hdr_t hh[CH_ITEMS];
#pragma unroll
    for (int k = 0; k < CH_ITEMS; k++) {
        const uint32_t i = base + k < C.n ? base + k : C.n - 1;
        off[k] = C.in_off[i];
        len[k] = C.in_len[i];
        cap[k] = C.cap[i];
    }
#pragma unroll
    for (int k = 0; k < CH_ITEMS; k++)
        hh[k] = srtp_parse_rtp(C.in + off[k], off[k], len[k]);
    ChAgg mine = ch_none();
#pragma unroll
    for (int k = 0; k < CH_ITEMS; k++) {
        code[k] = 0;
        seq[k] = 0;
        if (base + k >= C.n)
            continue;
        const srtp_dev_hdr_t &h = hh[k];
        // classify_one's checks (srtp_host.c pre_protect; srtp.c:2515-2600)
        if (h.enc_start >> 24) {
            code[k] = h.enc_start >> 24;   // header does not parse
        } else if (h.ssrc != S.ssrc) {
            abort |= AB_UNKNOWN_SSRC;      // template clone: host
        } else {
            if (!(S.flags & SRTP_DS_ELIGIBLE) || (S.dir & SRTP_DIR_RX))
                abort |= AB_INELIGIBLE;
            uses++;                        // key usage (key.c:74)
            if (cap[k] < len[k] + S.trailer) {
                code[k] = ST_BUFFER_SMALL;
            } else if (h.enc_start > len[k]) {
                code[k] = ST_PARSE_ERR;
            } else {
                chain |= 1u << k;
                seq[k] = h.seq_len & 0xffffu;
                // aes_icm.c:317-322: at most 0xffff keystream blocks
                if ((S.flags & SRTP_DS_ICM_CONF) &&
                    (len[k] - h.enc_start + 15) / 16 > 0xffffu)
                    code[k] = ST_CIPHER_FAIL;   // index still advances
                mine = ch_combine(mine, ChAgg{ 1, seq[k], seq[k], 0 }, &bad);
            }
        }
    }
    // the tile's aggregate and each thread's exclusive prefix in the tile:
    // lanes by shuffles, waves through LDS
    const ChAgg incl = ch_wave_scan(mine, &bad);
    ChAgg lex = ch_shfl_up(incl, 1);
    if (lane == 0)
        lex = ch_none();
    if (lane == 63)
        s_w[wv] = incl;
    __syncthreads();
    if (t < 64) {
        ChAgg a = t < CH_THREADS / 64 ? s_w[t] : ch_none();
        a = ch_wave_scan(a, &bad);
        if (t < CH_THREADS / 64)
            s_w[t] = a;   // inclusive over waves 0..t
    }
    __syncthreads();
    const ChAgg wex = wv ? s_w[wv - 1] : ch_none();
    const ChAgg excl = ch_combine(wex, lex, &bad);
    const ChAgg tot = s_w[CH_THREADS / 64 - 1];
    if (t == 0 && tile > 0)   // the aggregate first: nobody waits on it
        __hip_atomic_store(&A.tile[tile], ch_pack_agg(tot), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (t < 64) {
        // wave 0: the exclusive prefix, then the inclusive one published
        uint32_t has = 0;
        uint64_t idx = 0;
        if (tile > 0)
            ch_lookback(A.tile, tile, stored, has, idx, &bad);
        if (t == 0) {
            s_has = has;
            s_idx = idx;
            ch_apply(has, idx, tot, stored, &bad);
            __hip_atomic_store(&A.tile[tile],
                               CH_PRE | (has ? CH_HAS : 0) |
                                   (idx & 0xffffffffffffull),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    // this thread's packets: indices from the tile's exclusive prefix
    uint32_t has = s_has;
    uint64_t idx = s_idx;
    ch_apply(has, idx, excl, stored, &bad);
#pragma unroll
    for (int k = 0; k < CH_ITEMS; k++) {
        const uint32_t i = base + k;
        if (i >= C.n)
            break;
        uint64_t e = 0;
        if (chain >> k & 1) {
            ch_apply(has, idx, ChAgg{ 1, seq[k], seq[k], 0 }, stored, &bad);
            e = idx;
        }
        C.est[i] = e;
        C.pstat[i] = code[k];
        srtp_dev_meta_t m;
        m.key = 0;
        m.roc = 0;
        m.len = 0;
        m.info = 0xff0000u;   // no crypto
        if ((chain >> k & 1) && code[k] == 0) {
            m.key = S.key;
            m.roc = (uint32_t)(e >> 16);
            m.info = hh[k].enc_start | (S.variant << 24);
            m.len = hh[k].len;
            C.olen[i] = hh[k].len + S.trailer;
        }
        C.meta[i] = m;
    }
    if (bad)
        abort |= AB_SEQUENCE;
    if (abort)
        atomicOr(&s_abort, abort);
    if (uses)
        atomicAdd(&s_uses, uses);
    __syncthreads();
    if (t == 0) {
        if (s_abort)
            atomicOr(A.abort, s_abort);
        if (s_uses)
            atomicAdd(&A.ctl[1], s_uses);
    }
}

struct Chain1Commit {
    const uint32_t *pstat, *olen;
    const uint64_t *est;
    uint32_t n;
    srtp_dev_stream_t *st;
    uint32_t *win;
    uint64_t *tile;
    uint32_t *ctl;
    uint32_t ntiles;
    const uint32_t *abort;     // this batch's
    uint32_t *abort_next;      // the next batch's, cleared here
    uint32_t *pub;             // host-coherent copy of the verdict
    int32_t *status;
    uint32_t *out_len;
};

__global__ __launch_bounds__(CH_COMMIT_THREADS) void k_pp_chain1_commit(Chain1Commit A)
{
    const uint32_t ab = *A.abort;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < A.n && !ab) {
        const uint32_t code = A.pstat[i];
        A.status[i] = (int32_t)code;
        if (code == 0)
            A.out_len[i] = A.olen[i];   // error packets keep out_len = capacity
    }
    if (blockIdx.x != 0)
        return;
    __shared__ uint32_t s_win[SEQ_MEDIAN / 32];   // up to 2^15 window bits
    __shared__ uint32_t s_stop;
    srtp_dev_stream_t &S = A.st[0];
    const uint64_t last = A.tile[A.ntiles - 1];
    const bool has = (last & CH_HAS) != 0;
    const uint64_t hi = last & 0xffffffffffffull;
    const uint32_t uses = A.ctl[1];
    const uint32_t words = S.win_bits >> 5;
    const uint64_t old = S.index;
    if (!ab && has) {
        // rdbx_add's shift by the advance, then one bit per chain packet
        // within win_bits of the new index (crypto/math/datatypes.c
        // bitvector_left_shift)
        const uint64_t adv = hi - old;
        const uint32_t *w = A.win + S.win_off;
        for (uint32_t x = threadIdx.x; x < words; x += blockDim.x) {
            uint32_t v = 0;
            if (adv < S.win_bits) {
                const uint32_t b0 = (uint32_t)adv >> 5, bi = (uint32_t)adv & 31;
                const uint32_t a = x + b0 < words ? w[x + b0] : 0u;
                const uint32_t b = x + b0 + 1 < words ? w[x + b0 + 1] : 0u;
                v = bi ? (a >> bi) | (b << (32 - bi)) : a;
            }
            s_win[x] = v;
        }
        if (threadIdx.x == 0)
            s_stop = 0;
        __syncthreads();
        // chain indices increase along the batch: walk back from its end
        // until a chain packet falls out of the window
        for (int64_t c = (int64_t)A.n - 1; c >= 0; c -= blockDim.x) {
            const int64_t j = c - (int64_t)threadIdx.x;
            if (j >= 0) {
                const uint64_t e = A.est[j];
                if (e) {
                    if (hi - e < S.win_bits) {
                        const uint32_t bit = S.win_bits - 1 - (uint32_t)(hi - e);
                        atomicOr(&s_win[bit >> 5], 1u << (bit & 31));
                    } else {
                        s_stop = 1;
                    }
                }
            }
            __syncthreads();
            const uint32_t stop = s_stop;
            __syncthreads();
            if (stop)
                break;
        }
        for (uint32_t x = threadIdx.x; x < words; x += blockDim.x)
            A.win[S.win_off + x] = s_win[x];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (!ab) {
            S.uses += uses;
            if (uses)
                S.dir |= SRTP_DIR_TX;
            if (has)
                S.index = hi;
        }
        if (A.pub)
            __hip_atomic_store(A.pub, ab, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        A.ctl[0] = 0;
        A.ctl[1] = 0;
        *A.abort_next = 0;
    }
    for (uint32_t x = threadIdx.x; x < A.ntiles; x += blockDim.x)
        A.tile[x] = 0;
}

// ---------------------------------------------------------------------------
// Unprotect of ONE stream in order or not: the receiver's batch with network
// reordering, duplicates, late and forged packets stays on the device.  The
// reference walks the packets in order (srtp.c:2884-2903 estimate and
// replay check, 3157-3167 replay add after the tag check; rdbx.c:112-145,
// 227-270):
//   est_k  = index_guess(T_{k-1}, seq_k), T = highest ACCEPTED index so far
//            (the stored index before the batch)
//   replay = est_k <= T_{k-1} and (T_{k-1} - est_k >= window bits: old, or
//            est_k's bit set: an earlier accepted packet had that index)
// In batch form:
//   k_pu_chain1    parse, classify (k_pu_classify's checks), and u_k for
//                  every candidate: the stored index's guess for the first
//                  one plus the SIGNED 16-bit advances (-2^15, 2^15) between
//                  consecutive candidates -- k_pp_chain1's single-pass
//                  look-back scan with signed sums
//   crypto         every candidate's tag verdict, speculative decryption
//   k_pu_first     (only when some advance was <= 0) the first authenticated
//                  position of every index: duplicates
//   k_pu_verdict1  a second look-back scan, max over the AUTHENTICATED u,
//                  gives T_{k-1} (a replayed or old packet never raises it:
//                  its index is at most T); the reference's estimate
//                  index_guess(T_{k-1}, seq_k) must equal u_k -- else the
//                  host decides -- and the verdict follows: replay_old,
//                  replay_fail (stored window bit, or an earlier accepted
//                  duplicate), auth_fail, accepted
//   k_pu_commit1   statuses / lengths; block 0 the stream: index, window
//                  (the stored one shifted, one bit per accepted packet in
//                  it), key uses, direction; accepted packets leave the undo
//                  set (meta cleared), the look-back state is reset
//   undo           every other candidate's decryption is taken back
// The first authenticated position uses a generation-tagged array (no reset
// between batches): entry = (~gen << 32) | position, atomicMin keeps the
// current batch's smallest position.
constexpr uint32_t ST_AUTH_FAIL = 7, ST_REPLAY_FAIL = 9, ST_REPLAY_OLD = 10;

// per-batch counters, two used in turn: a batch's commit kernel resets the
// next batch's (every block of it still reads its own)
struct PuCtl {
    uint32_t t_chain, t_verdict;   // tile tickets (dispatch order)
    uint32_t nonmono;              // some candidate advance was <= 0
    uint32_t cand, replays, accepted;
    uint32_t abort1;               // abort bits raised before the crypto
    uint32_t abort2;               // ... and after it
    unsigned long long umin, umax; // candidate indices of the batch
};

__device__ __forceinline__ void pu_ctl_reset(PuCtl &c)
{
    c.t_chain = c.t_verdict = 0;
    c.nonmono = c.cand = c.replays = c.accepted = c.abort1 = c.abort2 = 0;
    c.umin = ~0ull;
    c.umax = 0;
}

// the signed advance between consecutive candidates, in [-2^15, 2^15)
__device__ __forceinline__ uint64_t cs_adv(uint32_t from, uint32_t to,
                                           uint32_t *nm)
{
    const int32_t d = (int32_t)((to - from + 32768u) & 0xffffu) - 32768;
    if (d <= 0)
        *nm = 1;
    return (uint64_t)(int64_t)d;
}

__device__ __forceinline__ ChAgg cs_combine(const ChAgg &a, const ChAgg &b,
                                            uint32_t *nm)
{
    if (!a.has)
        return b;
    if (!b.has)
        return a;
    return ChAgg{ 1, a.first, b.last,
                  a.internal + cs_adv(a.last, b.first, nm) + b.internal };
}

// a tile aggregate's signed sum: |sum| < 4095 * 2^15 < 2^28 (29-bit field)
__device__ __forceinline__ ChAgg cs_unpack_agg(uint64_t v)
{
    ChAgg a = ch_unpack_agg(v);
    a.internal = (uint64_t)(((int64_t)(v << 35)) >> 35);
    return a;
}

// prefix (has, u of the last candidate) followed by a run; u is kept in
// 48 bits (an index below zero or past 2^48 sends the batch to the host)
__device__ __forceinline__ void cs_apply(uint32_t &has, uint64_t &idx,
                                         const ChAgg &a, uint64_t stored,
                                         uint32_t *nm, uint32_t *bad)
{
    if (!a.has)
        return;
    if (has) {
        idx += cs_adv((uint32_t)idx & 0xffffu, a.first, nm) + a.internal;
    } else {
        uint64_t e;
        guess_index(stored, a.first, &e);
        idx = e + a.internal;
        has = 1;
    }
    if (idx >> 48)
        *bad = 1;
}

__device__ __forceinline__ ChAgg cs_wave_scan(ChAgg a, uint32_t *nm)
{
    const int lane = threadIdx.x & 63;
    for (int d = 1; d < 64; d <<= 1) {
        const ChAgg o = ch_shfl_up(a, d);
        if (lane >= d)
            a = cs_combine(o, a, nm);
    }
    return a;
}

__device__ void cs_lookback(const uint64_t *tile, uint32_t t, uint64_t stored,
                            uint32_t &has, uint64_t &idx, uint32_t *nm,
                            uint32_t *bad)
{
    const int lane = threadIdx.x & 63;
    ChAgg suf = ch_none();
    has = 0;
    idx = 0;
    for (int64_t j0 = (int64_t)t - 1; j0 >= 0; j0 -= 64) {
        const int64_t j = j0 - lane;
        uint64_t v = CH_PRE;
        if (j >= 0)
            while (!((v = __hip_atomic_load(&tile[j], __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT)) &
                     CH_FLAGS))
                __builtin_amdgcn_s_sleep(1);
        const uint64_t pm = __ballot((v & CH_FLAGS) == CH_PRE);
        const int fl = pm ? __ffsll((unsigned long long)pm) - 1 : 64;
        ChAgg a = lane < fl ? cs_unpack_agg(v) : ch_none();
        for (int d = 1; d < 64; d <<= 1) {
            const ChAgg o = ch_shfl_down(a, d);
            if (lane + d < 64)
                a = cs_combine(o, a, nm);
        }
        const ChAgg w{ (uint32_t)__shfl((int)a.has, 0),
                       (uint32_t)__shfl((int)a.first, 0),
                       (uint32_t)__shfl((int)a.last, 0),
                       (uint64_t)__shfl((long long)a.internal, 0) };
        suf = cs_combine(w, suf, nm);
        if (pm) {
            const uint64_t pv = (uint64_t)__shfl((long long)v, fl);
            has = (pv & CH_HAS) ? 1u : 0u;
            idx = pv & 0xffffffffffffull;
            break;
        }
    }
    cs_apply(has, idx, suf, stored, nm, bad);
}

struct PuChainArgs {
    ClassifyArgs C;       // in, offsets, lengths, capacities, stream 0, map
    uint8_t *auth;
    uint64_t *tile;       // look-back words, zero at entry
    PuCtl *ctl;           // this batch's, reset
};

__global__ __launch_bounds__(CH_THREADS) void k_pu_chain1(PuChainArgs A)
{
    const ClassifyArgs &C = A.C;
    __shared__ uint32_t s_tile, s_has, s_cand, s_abort, s_nm;
    __shared__ uint64_t s_idx, s_min, s_max;
    __shared__ ChAgg s_w[CH_THREADS / 64];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t == 0) {
        s_tile = atomicAdd(&A.ctl->t_chain, 1u);
        s_cand = 0;
        s_abort = 0;
        s_nm = 0;
        s_min = ~0ull;
        s_max = 0;
    }
    __syncthreads();
    const uint32_t tile = s_tile;
    const srtp_dev_stream_t S = C.st[0];
    const uint64_t stored = S.index;
    const uint32_t tag = S.trailer;   // tag + MKI
    const uint32_t base = tile * CH_TILE + t * CH_ITEMS;
    uint32_t bad = 0, nm = 0, abort = 0, chain = 0, cand = 0;
    uint64_t off[CH_ITEMS];
    uint32_t len[CH_ITEMS], cap[CH_ITEMS], code[CH_ITEMS], seq[CH_ITEMS];
    uint32_t kj[CH_ITEMS];   // MKI streams: the key index of the packet
    srtp_dev_hdr_t hh[CH_ITEMS];
#pragma unroll
    for (int k = 0; k < CH_ITEMS; k++) {
        const uint32_t i = base + k < C.n ? base + k : C.n - 1;
        off[k] = C.in_off[i];
        len[k] = C.in_len[i];
        cap[k] = C.cap[i];
        kj[k] = 0;
    }
#pragma unroll
    for (int k = 0; k < CH_ITEMS; k++)
        hh[k] = srtp_parse_rtp(C.in + off[k], off[k], len[k]);
    ChAgg mine = ch_none();
#pragma unroll
    for (int k = 0; k < CH_ITEMS; k++) {
        code[k] = 0;
        seq[k] = 0;
        if (base + k >= C.n)
            continue;
        const srtp_dev_hdr_t &h = hh[k];
        // k_pu_classify's checks (srtp_host.c un_static; srtp.c:2905-2990)
        if (h.enc_start >> 24) {
            code[k] = h.enc_start >> 24;
        } else if (h.ssrc != S.ssrc) {
            abort |= AB_UNKNOWN_SSRC;
        } else {
            if (!(S.flags & SRTP_DS_RX_ELIGIBLE) || (S.dir & SRTP_DIR_TX))
                abort |= AB_INELIGIBLE;
            const uint32_t L = len[k];
            if (L < tag || h.enc_start > L - tag ||
                ((S.flags & SRTP_DS_AEAD) && L - h.enc_start < tag) ||
                cap[k] < L - tag ||
                ((S.flags & SRTP_DS_ICM_CONF) &&
                 (L - tag - h.enc_start + 15) / 16 > 0xffffu)) {
                abort |= AB_STATIC;
            } else {
                if (S.mki)   // the packet's key (MKI_NONE: bad_mki)
                    kj[k] = mki_match(C.keys, C.mkslot, S, C.in + off[k], L);
                chain |= 1u << k;
                cand++;
                seq[k] = h.seq_len & 0xffffu;
                mine = cs_combine(mine, ChAgg{ 1, seq[k], seq[k], 0 }, &nm);
            }
        }
    }
    const ChAgg incl = cs_wave_scan(mine, &nm);
    ChAgg lex = ch_shfl_up(incl, 1);
    if (lane == 0)
        lex = ch_none();
    if (lane == 63)
        s_w[wv] = incl;
    __syncthreads();
    if (t < 64) {
        ChAgg a = t < CH_THREADS / 64 ? s_w[t] : ch_none();
        a = cs_wave_scan(a, &nm);
        if (t < CH_THREADS / 64)
            s_w[t] = a;
    }
    __syncthreads();
    const ChAgg wex = wv ? s_w[wv - 1] : ch_none();
    const ChAgg excl = cs_combine(wex, lex, &nm);
    const ChAgg tot = s_w[CH_THREADS / 64 - 1];
    if (t == 0 && tile > 0)
        __hip_atomic_store(&A.tile[tile], ch_pack_agg(tot), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (t < 64) {
        uint32_t has = 0;
        uint64_t idx = 0;
        if (tile > 0)
            cs_lookback(A.tile, tile, stored, has, idx, &nm, &bad);
        if (t == 0) {
            s_has = has;
            s_idx = idx;
            cs_apply(has, idx, tot, stored, &nm, &bad);
            __hip_atomic_store(&A.tile[tile],
                               CH_PRE | (has ? CH_HAS : 0) |
                                   (idx & 0xffffffffffffull),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    uint32_t has = s_has;
    uint64_t idx = s_idx;
    cs_apply(has, idx, excl, stored, &nm, &bad);
    uint64_t umin = ~0ull, umax = 0;
#pragma unroll
    for (int k = 0; k < CH_ITEMS; k++) {
        const uint32_t i = base + k;
        if (i >= C.n)
            break;
        srtp_dev_meta_t m;
        m.key = 0;
        m.roc = 0;
        m.len = 0;
        m.info = 0xff0000u;   // no crypto
        uint64_t e = 0;
        uint8_t au = 1;   // kernels without a tag check leave it: accepted
        if (chain >> k & 1) {
            cs_apply(has, idx, ChAgg{ 1, seq[k], seq[k], 0 }, stored, &nm, &bad);
            e = idx;
            umin = e < umin ? e : umin;
            umax = e > umax ? e : umax;
            if (kj[k] == MKI_NONE) {
                au = AUTH_BAD_MKI;   // a candidate without crypto: bad_mki
            } else {
                m.key = S.mki ? C.mkslot[S.kbase + kj[k]] : S.key;
                m.roc = (uint32_t)(e >> 16);
                m.info = hh[k].enc_start | (S.variant << 24);
                m.len = hh[k].len - tag;
            }
            if (S.mki)
                C.rxj[i] = (uint8_t)kj[k];
        }
        C.est[i] = e;
        C.skey[i] = (chain >> k & 1) ? 0u : NOCHAIN;
        C.pstat[i] = code[k];
        C.meta[i] = m;
        A.auth[i] = au;
    }
    if (bad)
        abort |= AB_SEQUENCE;
    if (abort)
        atomicOr(&s_abort, abort);
    if (nm)
        s_nm = 1;
    if (cand) {
        atomicAdd(&s_cand, cand);
        atomicMin((unsigned long long *)&s_min, (unsigned long long)umin);
        atomicMax((unsigned long long *)&s_max, (unsigned long long)umax);
    }
    __syncthreads();
    if (t == 0) {
        if (s_abort)
            atomicOr(&A.ctl->abort1, s_abort);
        if (s_nm)
            atomicOr(&A.ctl->nonmono, 1u);
        if (s_cand) {
            atomicAdd(&A.ctl->cand, s_cand);
            atomicMin(&A.ctl->umin, (unsigned long long)s_min);
            atomicMax(&A.ctl->umax, (unsigned long long)s_max);
        }
    }
}

// duplicates (non-monotone batches only): the first authenticated position
// of every candidate index, generation-tagged (no reset between batches)
__global__ void k_pu_first(const uint32_t *skey, const uint64_t *est,
                           const uint8_t *auth, uint32_t n, PuCtl *ctl,
                           unsigned long long *first, uint64_t cap,
                           uint32_t gen)
{
    if (!ctl->nonmono || ctl->abort1)
        return;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t lo = ctl->umin, span = ctl->umax - ctl->umin + 1;
    if (span > cap) {
        if (i == 0)
            atomicOr(&ctl->abort2, AB_ORDER);   // indices too spread: host
        return;
    }
    if (i >= n || skey[i] != 0u || auth[i] != 1)
        return;
    const unsigned long long tagv = ((unsigned long long)(~gen) << 32) | i;
    atomicMin(&first[est[i] - lo], tagv);
}

struct PuVerdictArgs {
    const uint32_t *skey;
    const uint64_t *est;
    const uint8_t *auth;
    const unsigned long long *first;
    const srtp_dev_stream_t *st;
    const uint32_t *win;
    uint32_t n;
    uint64_t *tile;       // look-back words, zero at entry
    PuCtl *ctl;
    uint32_t *pstat;      // out: the verdict code of every candidate
    uint64_t *top;        // out: T_k inclusive (highest authenticated)
    uint32_t gen;         // k_pu_first's generation of this batch
    uint64_t first_cap;   // entries of `first` (k_pu_first's span check)
};

__global__ __launch_bounds__(CH_THREADS) void k_pu_verdict1(PuVerdictArgs A)
{
    __shared__ uint32_t s_tile, s_rep, s_acc;
    __shared__ uint64_t s_w[CH_THREADS / 64], s_pre;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t == 0) {
        s_tile = atomicAdd(&A.ctl->t_verdict, 1u);
        s_rep = 0;
        s_acc = 0;
    }
    __syncthreads();
    const uint32_t tile = s_tile;
    const srtp_dev_stream_t S = A.st[0];
    const uint64_t stored = S.index;
    const uint32_t bits = S.win_bits;
    // the first-authenticated array exists only when k_pu_first ran: some
    // advance <= 0 and the candidates' index span fits it (else k_pu_first
    // raised AB_ORDER and nothing is read from it here)
    const uint64_t lo = A.ctl->umin;
    const bool nonmono = A.ctl->nonmono != 0 &&
                         A.ctl->umax - lo + 1 <= A.first_cap;
    const uint32_t gen = A.gen;
    const uint32_t base = tile * CH_TILE + t * CH_ITEMS;
    uint64_t u[CH_ITEMS];
    uint32_t cand = 0, au = 0, bm = 0;   // bm: bad_mki candidates
    // values are index + 1 so that 0 means "no authenticated packet"
    uint64_t mx = 0;
#pragma unroll
    for (int k = 0; k < CH_ITEMS; k++) {
        const uint32_t i = base + k;
        u[k] = 0;
        if (i < A.n && A.skey[i] == 0u) {
            cand |= 1u << k;
            u[k] = A.est[i];
            const uint8_t a = A.auth[i];
            if (a == 1) {
                au |= 1u << k;
                mx = u[k] + 1 > mx ? u[k] + 1 : mx;
            } else if (a == AUTH_BAD_MKI) {
                bm |= 1u << k;
            }
        }
    }
    // block max-scan: inclusive over lanes, waves through LDS
    uint64_t incl = mx;
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = (uint64_t)__shfl_up((long long)incl, d);
        if (lane >= d)
            incl = o > incl ? o : incl;
    }
    uint64_t lex = (uint64_t)__shfl_up((long long)incl, 1);
    if (lane == 0)
        lex = 0;
    if (lane == 63)
        s_w[wv] = incl;
    __syncthreads();
    uint64_t wex = 0, tot = 0;
    for (int w = 0; w < CH_THREADS / 64; w++) {
        if (w == wv)
            wex = tot;
        tot = s_w[w] > tot ? s_w[w] : tot;
    }
    // look-back words: [63:62] 1 aggregate / 2 inclusive prefix, [48:0]
    // max authenticated index + 1 (0: none)
    if (t == 0 && tile > 0)
        __hip_atomic_store(&A.tile[tile], CH_AGG | tot, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (t < 64) {
        uint64_t pre = 0;
        for (int64_t j0 = (int64_t)tile - 1; j0 >= 0; j0 -= 64) {
            const int64_t j = j0 - lane;
            uint64_t v = CH_PRE;
            if (j >= 0)
                while (!((v = __hip_atomic_load(&A.tile[j], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT)) &
                         CH_FLAGS))
                    __builtin_amdgcn_s_sleep(1);
            const uint64_t pm = __ballot((v & CH_FLAGS) == CH_PRE);
            const int fl = pm ? __ffsll((unsigned long long)pm) - 1 : 64;
            uint64_t a = lane <= fl ? (v & ~CH_FLAGS) : 0;
            for (int m = 1; m < 64; m <<= 1) {
                const uint64_t o = (uint64_t)__shfl_xor((long long)a, m);
                a = o > a ? o : a;
            }
            pre = a > pre ? a : pre;
            if (pm)
                break;
        }
        if (t == 0) {
            s_pre = pre;
            __hip_atomic_store(&A.tile[tile], CH_PRE | (pre > tot ? pre : tot),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    uint64_t run = s_pre > wex ? s_pre : wex;
    run = lex > run ? lex : run;
    uint32_t bad = 0, rep = 0, acc = 0;
#pragma unroll
    for (int k = 0; k < CH_ITEMS; k++) {
        const uint32_t i = base + k;
        if (!(cand >> k & 1))
            continue;
        // T_{k-1}: the stored index or the highest authenticated before
        const uint64_t T = run > stored + 1 ? run - 1 : stored;
        uint64_t g;
        guess_index(T, (uint32_t)u[k] & 0xffffu, &g);
        if (g != u[k])
            bad = 1;   // the reference estimates this packet differently
        // not authenticated: the tag failed, or (after the replay check, as
        // srtp.c:2905-2912 orders them) no key matched its MKI
        const uint32_t rej = (bm >> k & 1) ? ST_BAD_MKI : ST_AUTH_FAIL;
        uint32_t v;
        if (u[k] > T) {
            v = (au >> k & 1) ? 0u : rej;
        } else if (T - u[k] >= bits) {
            v = ST_REPLAY_OLD;
        } else {
            bool seen = false;
            if (u[k] <= stored) {
                // the stored window (rdbx.c:227-243): bit (bits-1) = stored
                const uint32_t bit = bits - 1 - (uint32_t)(stored - u[k]);
                seen = (A.win[S.win_off + (bit >> 5)] >> (bit & 31)) & 1u;
            }
            if (!seen && nonmono) {
                const unsigned long long f = A.first[u[k] - lo];
                seen = (uint32_t)(f >> 32) == ~gen && (uint32_t)f < i;
            }
            v = seen ? ST_REPLAY_FAIL : (au >> k & 1) ? 0u : rej;
        }
        if (v == ST_REPLAY_FAIL || v == ST_REPLAY_OLD)
            rep++;
        if (v == 0)
            acc++;
        if (au >> k & 1)
            run = u[k] + 1 > run ? u[k] + 1 : run;
        A.pstat[i] = v;
        A.top[i] = run > stored + 1 ? run - 1 : stored;
    }
    if (bad)
        atomicOr(&A.ctl->abort2, AB_ORDER);
    if (rep)
        atomicAdd(&s_rep, rep);
    if (acc)
        atomicAdd(&s_acc, acc);
    __syncthreads();
    if (t == 0) {
        if (s_rep)
            atomicAdd(&A.ctl->replays, s_rep);
        if (s_acc)
            atomicAdd(&A.ctl->accepted, s_acc);
    }
}

struct PuCommitArgs {
    const uint32_t *skey, *pstat, *in_len;
    const uint64_t *est, *top;
    uint32_t n;
    srtp_dev_stream_t *st;
    uint32_t *win;
    uint64_t *tile, *vtile;
    uint32_t ntiles;
    PuCtl *ctl, *ctl_next;
    uint32_t *pub;
    srtp_dev_meta_t *meta;
    int32_t *status;
    uint32_t *out_len;
};

__global__ __launch_bounds__(CH_COMMIT_THREADS) void k_pu_commit1(PuCommitArgs A)
{
    // ab1: before the crypto (it ran on nothing), ab2: after it (every
    // candidate's decryption is undone)
    const uint32_t ab1 = A.ctl->abort1, ab2 = A.ctl->abort2, ab = ab1 | ab2;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const srtp_dev_stream_t S0 = A.st[0];
    if (i < A.n && ab1)
        A.meta[i].info = 0xff0000u;   // nothing ran: nothing to undo
    if (i < A.n && !ab) {
        if (A.skey[i] != 0u) {
            A.status[i] = (int32_t)A.pstat[i];   // header errors: no stream
        } else {
            const uint32_t v = A.pstat[i];
            A.status[i] = (int32_t)v;
            if (v == 0) {
                A.out_len[i] = A.in_len[i] - S0.trailer;
                A.meta[i].info = 0xff0000u;      // accepted: nothing to undo
            }
        }
    }
    if (blockIdx.x != 0)
        return;
    __shared__ uint32_t s_win[SEQ_MEDIAN / 32];
    __shared__ uint32_t s_stop;
    srtp_dev_stream_t &S = A.st[0];
    const uint64_t old = S.index;
    const uint32_t words = S.win_bits >> 5;
    uint64_t hi = old;
    if (A.ntiles) {
        const uint64_t last = A.vtile[A.ntiles - 1] & ~CH_FLAGS;
        if (last && last - 1 > hi)
            hi = last - 1;
    }
    const uint32_t acc = A.ctl->accepted;
    if (!ab && acc) {
        // the stored window shifted to the new top (rdbx_add), then the
        // accepted packets' bits inside it; the highest authenticated index
        // T_k never decreases along the batch, so the walk back from the
        // end stops at the first packet with T_k below the window
        const uint64_t adv = hi - old;
        const uint32_t *w = A.win + S.win_off;
        for (uint32_t x = threadIdx.x; x < words; x += blockDim.x) {
            uint32_t v = 0;
            if (adv < S.win_bits) {
                const uint32_t b0 = (uint32_t)adv >> 5, bi = (uint32_t)adv & 31;
                const uint32_t a = x + b0 < words ? w[x + b0] : 0u;
                const uint32_t b = x + b0 + 1 < words ? w[x + b0 + 1] : 0u;
                v = bi ? (a >> bi) | (b << (32 - bi)) : a;
            }
            s_win[x] = v;
        }
        if (threadIdx.x == 0)
            s_stop = 0;
        __syncthreads();
        for (int64_t c = (int64_t)A.n - 1; c >= 0; c -= blockDim.x) {
            const int64_t j = c - (int64_t)threadIdx.x;
            if (j >= 0 && A.skey[j] == 0u) {
                if (hi - A.top[j] >= S.win_bits) {
                    s_stop = 1;
                } else if (A.pstat[j] == 0) {
                    const uint64_t e = A.est[j];
                    if (hi - e < S.win_bits) {
                        const uint32_t bit =
                            S.win_bits - 1 - (uint32_t)(hi - e);
                        atomicOr(&s_win[bit >> 5], 1u << (bit & 31));
                    }
                }
            }
            __syncthreads();
            const uint32_t stop = s_stop;
            __syncthreads();
            if (stop)
                break;
        }
        for (uint32_t x = threadIdx.x; x < words; x += blockDim.x)
            A.win[S.win_off + x] = s_win[x];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (!ab) {
            // key usage: AES-GCM every candidate that passed the replay
            // check (srtp_unprotect_aead counts before the tag), AES-ICM /
            // HMAC the accepted ones
            S.uses += (S.flags & SRTP_DS_AEAD)
                          ? A.ctl->cand - A.ctl->replays
                          : acc;
            if (acc) {
                S.dir |= SRTP_DIR_RX;
                S.index = hi;
            }
        }
        if (A.pub)
            __hip_atomic_store(A.pub, ab, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        pu_ctl_reset(*A.ctl_next);
    }
    for (uint32_t x = threadIdx.x; x < A.ntiles; x += blockDim.x) {
        A.tile[x] = 0;
        A.vtile[x] = 0;
    }
}

// ---------------------------------------------------------------------------
// Key buckets: a batch of many streams with distinct keys
// is laid out for the crypto kernel as one bucket of records per stream, so
// that a wave's 64 packets share one key (SGPR round keys, the four-table
// LDS layout) instead of gathering a key per lane.  A counting sort of the
// packets by stream, not of their bytes: a 32-byte record (offsets and
// descriptor) per packet.  Streams with at least BK_MIN packets get buckets
// padded to a multiple of 64 records, in region A = [0, a); the others are
// packed into region B = [a, a + b), where keys differ per lane.  Padding and
// unused slots are records with a nonzero status.  Order inside a bucket is
// irrelevant: on the order-free form every packet's index is already fixed.
constexpr uint32_t BK_MIN = 32;

__device__ __forceinline__ uint64_t bk_size(uint32_t c)
{
    return c >= BK_MIN ? (uint64_t)((c + 63) & ~63u) << 32 : (uint64_t)c;
}

// one workgroup: per-stream record offsets (exclusive scans of the bucket
// sizes of both regions, packed in one 64-bit word), cursors reset, the
// region bounds {0, a, a, a + b}.  The counts go through LDS in chunks of
// BK_CHUNK streams, loaded coalesced (a thread walking its own contiguous
// run of counts in global memory waited on every load: 148 us for 64k
// streams), each chunk scanned with the running total of those before it.
constexpr uint32_t BK_CHUNK = 16384;

__global__ __launch_bounds__(1024) void k_bk_offsets(const uint32_t *bcount,
                                                     uint32_t ns, uint32_t *off,
                                                     uint32_t *cur,
                                                     uint32_t *range)
{
    __shared__ uint64_t s_part[1024];
    __shared__ uint32_t s_cnt[BK_CHUNK];
    const uint32_t t = threadIdx.x, T = blockDim.x;
    // the region totals first (region B starts after all of region A)
    // (16 guarded loads at a time, then their sizes: one wait per 16)
    uint64_t all = 0;
    for (uint32_t s0 = 0; s0 < ns; s0 += 16 * T) {
        uint32_t v[16];
#pragma unroll
        for (uint32_t j = 0; j < 16; j++) {
            const uint32_t s = s0 + j * T + t;
            v[j] = s < ns ? bcount[s] : 0u;
        }
#pragma unroll
        for (uint32_t j = 0; j < 16; j++)
            all += bk_size(v[j]);
    }
    s_part[t] = all;
    __syncthreads();
    for (uint32_t d = T / 2; d > 0; d >>= 1) {
        if (t < d)
            s_part[t] += s_part[t + d];
        __syncthreads();
    }
    const uint64_t tot = s_part[0];
    const uint32_t atot = (uint32_t)(tot >> 32), btot = (uint32_t)tot;
    __syncthreads();
    uint64_t carry = 0;   // both regions' records before this chunk
    for (uint32_t c0 = 0; c0 < ns; c0 += BK_CHUNK) {
        const uint32_t cn = ns - c0 < BK_CHUNK ? ns - c0 : BK_CHUNK;
        {
            uint32_t v[BK_CHUNK / 1024];   // blockDim.x = 1024
#pragma unroll
            for (uint32_t j = 0; j < BK_CHUNK / 1024; j++) {
                const uint32_t k = j * T + t;
                v[j] = k < cn ? bcount[c0 + k] : 0u;
            }
#pragma unroll
            for (uint32_t j = 0; j < BK_CHUNK / 1024; j++)
                if (j * T + t < cn)
                    s_cnt[j * T + t] = v[j];
        }
        __syncthreads();
        const uint32_t per = (cn + T - 1) / T;
        const uint32_t k0 = t * per < cn ? t * per : cn;
        const uint32_t k1 = k0 + per < cn ? k0 + per : cn;
        uint64_t sum = 0;
        for (uint32_t k = k0; k < k1; k++)
            sum += bk_size(s_cnt[k]);
        s_part[t] = sum;
        __syncthreads();
        for (uint32_t d = 1; d < T; d <<= 1) {
            const uint64_t v = t >= d ? s_part[t - d] : 0;
            __syncthreads();
            s_part[t] += v;
            __syncthreads();
        }
        uint64_t run = carry + s_part[t] - sum;   // exclusive
        for (uint32_t k = k0; k < k1; k++) {   // offsets over the counts
            const uint32_t c = s_cnt[k];
            s_cnt[k] = c >= BK_MIN ? (uint32_t)(run >> 32)
                                   : atot + (uint32_t)run;
            run += bk_size(c);
        }
        carry += s_part[T - 1];
        __syncthreads();
        for (uint32_t k = t; k < cn; k += T) {   // coalesced stores
            off[c0 + k] = s_cnt[k];
            cur[c0 + k] = 0;
        }
        __syncthreads();   // s_cnt / s_part reused by the next chunk
    }
    if (t == 0) {
        range[0] = 0;
        range[1] = atot;
        range[2] = atot;
        range[3] = atot + btot;
    }
}

// a slot in stream s's bucket: one atomic per stream present in the wave
// (up to four), the rest (a wave spread over many streams) one per lane
__device__ __forceinline__ uint32_t bk_claim(uint32_t s, uint32_t *cur)
{
    const uint32_t lane = threadIdx.x & 63;
    bool done = s == NOCHAIN;
    uint32_t pos = 0;
    for (int it = 0; it < 4; it++) {
        const uint64_t am = __ballot(!done);
        if (!am)
            return pos;
        const int ll = __ffsll((unsigned long long)am) - 1;
        const uint32_t lead = (uint32_t)__shfl((int)s, ll);
        const bool mine = !done && s == lead;
        const uint64_t mm = __ballot(mine);
        uint32_t base = 0;
        if ((int)lane == ll)
            base = atomicAdd(&cur[lead], (uint32_t)__popcll((unsigned long long)mm));
        base = (uint32_t)__shfl((int)base, ll);
        if (mine) {
            pos = base + (uint32_t)__popcll((unsigned long long)(mm & ((1ull << lane) - 1)));
            done = true;
        }
        if (__popcll((unsigned long long)mm) == 1)
            break;
    }
    if (!done)
        pos = atomicAdd(&cur[s], 1u);
    return pos;
}

// every crypto packet (a stream, status 0) to its bucket
__global__ void k_bk_scatter(const uint32_t *skey, const uint32_t *pstat,
                             const srtp_dev_meta_t *meta,
                             const uint64_t *in_off, const uint64_t *out_off,
                             uint32_t n, uint32_t ns, const uint32_t *off,
                             uint32_t *cur, srtp_dev_rec_t *rec,
                             uint32_t *rec_idx)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t s = NOCHAIN;
    if (i < n) {
        s = skey[i];
        if (s >= ns || pstat[i])
            s = NOCHAIN;
    }
    const uint32_t pos = bk_claim(s, cur);
    if (s == NOCHAIN)
        return;
    const uint32_t at = off[s] + pos;
    srtp_dev_rec_t r;
    r.in_off = in_off[i];
    r.out_off = out_off[i];
    r.meta = meta[i];
    rec[at] = r;
    rec_idx[at] = i;
}

// the unused slots of every bucket (wave padding, packets that left the
// chain with an error) become gaps
__global__ void k_bk_pad(const uint32_t *bcount, uint32_t ns,
                         const uint32_t *off, const uint32_t *cur,
                         srtp_dev_rec_t *rec)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ns)
        return;
    const uint32_t c = bcount[s];
    const uint32_t end = c >= BK_MIN ? (c + 63) & ~63u : c;
    for (uint32_t p = cur[s]; p < end; p++)
        rec[off[s] + p].meta.info = 0xff0000u;
}

// recorded where srtp_gpu_last_error() reports it (the host logs it)
int pp_fail(hipError_t e, const char *what)
{
    char m[160];
    snprintf(m, sizeof m, "device pre-pass: %s", what);
    return srtp_gpu_fail(e, m);
}

#define PPCHK(x)                                                               \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess)                                                  \
            return pp_fail(e_, #x);                                            \
    } while (0)

// SRTP_PP_DEBUG=1: synchronise and check after every pre-pass step, naming
// the step that failed (debug aid; off by default)
bool pp_debug()
{
    static int on = -1;
    if (on < 0) {
        const char *e = getenv("SRTP_PP_DEBUG");
        on = e && *e == '1';
    }
    return on;
}

int pp_step(hipStream_t st, const char *what)
{
    if (!pp_debug())
        return 0;
    hipError_t e = hipStreamSynchronize(st);
    if (e == hipSuccess)
        e = hipGetLastError();
    fprintf(stderr, "srtp_pp: %-14s %s\n", what, hipGetErrorString(e));
    return e == hipSuccess ? 0 : pp_fail(e, what);
}

template <class T>
int regrow(T **p, uint32_t *cap, uint32_t need)
{
    if (need <= *cap && *p)
        return 0;
    uint32_t nc = *cap ? *cap : 64;
    while (nc < need)
        nc *= 2;
    if (*p)
        PPCHK(hipFree(*p));
    *p = nullptr;
    PPCHK(hipMalloc((void **)p, (size_t)nc * sizeof(T)));
    *cap = nc;
    return 0;
}

PpState *pp_of(srtp_gpu_t *g)
{
    void **slot = srtp_gpu_pp_slot(g);
    if (!*slot)
        *slot = new PpState();
    return (PpState *)*slot;
}

int reserve_packets(PpState *P, size_t n, hipStream_t stream)
{
    if (n <= P->n_cap)
        return 0;
    size_t c = P->n_cap ? P->n_cap : 4096;
    while (c < n)
        c *= 2;
    void *old[] = { P->hdr, P->pstat, P->skey, P->skey2, P->perm,
                    P->perm2, P->val, P->est, P->meta, P->agg, P->hist,
                    P->auth, P->top, P->rec, P->rec_idx, P->rxj };
    for (void *o : old)
        if (o)
            PPCHK(hipFree(o));
    PPCHK(hipMalloc((void **)&P->hdr, c * sizeof(srtp_dev_hdr_t)));
    PPCHK(hipMalloc((void **)&P->pstat, c * 4));
    PPCHK(hipMalloc((void **)&P->skey, c * 4));
    PPCHK(hipMalloc((void **)&P->skey2, c * 4));
    PPCHK(hipMalloc((void **)&P->perm, c * 4));
    PPCHK(hipMalloc((void **)&P->perm2, c * 4));
    PPCHK(hipMalloc((void **)&P->val, c * 8));
    PPCHK(hipMalloc((void **)&P->est, c * 8));
    PPCHK(hipMalloc((void **)&P->meta, c * sizeof(srtp_dev_meta_t)));
    PPCHK(hipMalloc((void **)&P->auth, c));
    PPCHK(hipMalloc((void **)&P->rxj, c));
    PPCHK(hipMalloc((void **)&P->top, c * 8));
    if (P->fzrec)
        PPCHK(hipFree(P->fzrec));
    PPCHK(hipMalloc((void **)&P->fzrec, c * sizeof(FzRec)));
    if (P->tsave)
        PPCHK(hipFree(P->tsave));
    PPCHK(hipMalloc((void **)&P->tsave, c * 16));
    if (P->fz_glist)
        PPCHK(hipFree(P->fz_glist));
    PPCHK(hipMalloc((void **)&P->fz_glist,
                    (c / 64 + 2 + 2 * FZ_GL_WAVES) * 4));
    // buckets: region A <= 2 x its packets (>= BK_MIN per stream, padded
    // to 64), region B <= its packets
    PPCHK(hipMalloc((void **)&P->rec, 2 * c * sizeof(srtp_dev_rec_t)));
    PPCHK(hipMalloc((void **)&P->rec_idx, 2 * c * 4));
    // scan / sort scratch: digit histograms of 256 bins per tile, one scan
    // aggregate per tile of the largest scan (the histograms)
    const size_t nt = (c + srtp_scan::TILE - 1) / srtp_scan::TILE;
    PPCHK(hipMalloc((void **)&P->hist, 256 * nt * 4));
    PPCHK(hipMalloc((void **)&P->agg, (nt + 2) * sizeof(srtp_scan::Agg)));
    // k_pp_chain1 look-back words: zero between batches
    if (P->ch_tile)
        PPCHK(hipFree(P->ch_tile));
    PPCHK(hipMalloc((void **)&P->ch_tile, (nt + 1) * 8));
    PPCHK(hipMemsetAsync(P->ch_tile, 0, (nt + 1) * 8, stream));
    if (P->pu_tile)
        PPCHK(hipFree(P->pu_tile));
    PPCHK(hipMalloc((void **)&P->pu_tile, 2 * (nt + 1) * 8));
    PPCHK(hipMemsetAsync(P->pu_tile, 0, 2 * (nt + 1) * 8, stream));
    PPCHK(hipStreamSynchronize(stream));
    P->ch_tiles_cap = nt;
    P->n_cap = c;
    return 0;
}

}   // namespace

extern "C" {

void srtp_gpu_pp_free(void *p)
{
    PpState *P = (PpState *)p;
    if (!P)
        return;
    void *bufs[] = { P->st, P->win, P->wnew, P->hkey, P->hval, P->bcount,
                     P->seg_first, P->bcount2, P->new_index2,
                     P->new_index, P->hdr, P->pstat, P->skey, P->skey2,
                     P->perm, P->perm2, P->val, P->est, P->meta, P->agg,
                     P->hist, P->auth, P->top, P->abort, P->bk_off, P->bk_cur,
                     P->rec, P->rec_idx, P->bk_range, P->ch_tile,
                     P->ch_ctl, P->ch_abort, P->pu_ctl, P->pu_tile,
                     P->pu_first, P->fzrec, P->tsave, P->fz_cnt,
                     P->fz_emin, P->fz_bmap, P->fz_hicand, P->fz_nfail,
                     P->fz_glist, P->pd_first, P->pd_min, P->pd_max,
                     P->pd_sids, P->pd_info, P->pd_efirst, P->pd_bak,
                     P->pd_bakwin, P->pd_pos, P->cl_ctl, P->mkslot,
                     P->kuses, P->mki8, P->io_e0, P->rxj };
    for (void *b : bufs)
        if (b)
            (void)hipFree(b);
    if (P->h_abort)
        (void)hipHostFree(P->h_abort);
    delete P;
}

int srtp_gpu_pp_upload(srtp_gpu_t *g, const srtp_dev_stream_t *streams,
                       uint32_t ns_up, const uint32_t *win, uint32_t nwords,
                       const uint32_t *hkey, const uint32_t *hval,
                       uint32_t hcap, const srtp_dev_stream_t *tmpl,
                       uint32_t spare, const uint32_t *mkslot, uint32_t nmk)
{
    PpState *P = pp_of(g);
    hipStream_t stream = (hipStream_t)srtp_gpu_stream_of(g);
    if (!tmpl)
        spare = 0;
    // every per-stream array holds the spare records too
    const uint32_t ns = ns_up + spare;
    uint32_t c1 = P->ns_cap, c2 = P->ns_cap, c5 = P->ns_cap,
             c6 = P->ns_cap, c7 = P->ns_cap, c8 = P->ns_cap, c9 = P->ns_cap,
             c10 = P->ns_cap, c11 = P->ns_cap, c13 = P->ns_cap,
             c3 = P->nwords_cap;
    if (regrow(&P->st, &P->ns_cap, ns + 1) ||
        regrow(&P->bcount, &c1, ns + 1) || regrow(&P->new_index, &c2, ns + 1) ||
        regrow(&P->seg_first, &c5, ns + 1) ||
        regrow(&P->bcount2, &c6, ns + 1) ||
        regrow(&P->new_index2, &c7, ns + 1) ||
        regrow(&P->bk_off, &c8, ns + 1) || regrow(&P->bk_cur, &c9, ns + 1) ||
        regrow(&P->fz_cnt, &c10, ns + 1) || regrow(&P->fz_emin, &c11, ns + 1) ||
        regrow(&P->win, &P->nwords_cap, nwords + 1) ||
        regrow(&P->wnew, &c3, nwords + 1) ||
        regrow(&P->fz_bmap, &P->bmap_cap, 4 * nwords + 4) ||
        regrow(&P->fz_hicand, &c13, ns + 1))
        return -1;
    if (!P->fz_nfail)
        PPCHK(hipMalloc((void **)&P->fz_nfail, 4));
    if (hcap > P->hcap_cap || !P->hkey) {
        uint32_t c4 = P->hcap_cap;
        if (regrow(&P->hkey, &P->hcap_cap, hcap) || regrow(&P->hval, &c4, hcap))
            return -1;
    }
    if (!P->abort) {
        PPCHK(hipMalloc((void **)&P->abort, 4));
        PPCHK(hipMalloc((void **)&P->bk_range, 16));
        PPCHK(hipMalloc((void **)&P->ch_ctl, 8));
        PPCHK(hipMalloc((void **)&P->ch_abort, 8));
        PPCHK(hipMemset(P->ch_ctl, 0, 8));
        PPCHK(hipMemset(P->ch_abort, 0, 8));
        PPCHK(hipMalloc((void **)&P->pu_ctl, 2 * sizeof(PuCtl)));
        PuCtl h[2];
        memset(h, 0, sizeof h);
        h[0].umin = h[1].umin = ~0ull;
        PPCHK(hipMemcpy(P->pu_ctl, h, sizeof h, hipMemcpyHostToDevice));
        PPCHK(hipHostMalloc((void **)&P->h_abort, 8,
                            hipHostMallocMapped | hipHostMallocCoherent));
        PPCHK(hipHostGetDevicePointer((void **)&P->h_abort_dev, P->h_abort,
                                      0));
    }
    if (nmk) {
        uint32_t c14 = P->nmk_cap;
        if (regrow(&P->mkslot, &P->nmk_cap, nmk) || regrow(&P->kuses, &c14, nmk))
            return -1;
        PPCHK(hipMemcpyAsync(P->mkslot, mkslot, nmk * 4ull,
                             hipMemcpyHostToDevice, stream));
        PPCHK(hipMemsetAsync(P->kuses, 0, nmk * 8ull, stream));
    }
    P->nmk = nmk;
    if (!P->cl_ctl)
        PPCHK(hipMalloc((void **)&P->cl_ctl, 8));
    PPCHK(hipMemsetAsync(P->cl_ctl, 0, 8, stream));
    P->ns = ns_up;
    P->ns0 = ns_up;
    P->spare = spare;
    P->has_tmpl = tmpl != nullptr;
    if (tmpl) {
        P->tmpl = *tmpl;
        P->tw = tmpl->win_bits >> 5;
    }
    P->nwords = nwords;
    P->hcap = hcap;
    PPCHK(hipMemsetAsync(P->fz_bmap, 0, (4ull * nwords + 4) * 4, stream));
    PPCHK(hipMemcpyAsync(P->st, streams, ns_up * sizeof *streams,
                         hipMemcpyHostToDevice, stream));
    if (nwords) {
        PPCHK(hipMemcpyAsync(P->win, win, nwords * 4ull, hipMemcpyHostToDevice,
                             stream));
        PPCHK(hipMemcpyAsync(P->wnew, win, nwords * 4ull,
                             hipMemcpyHostToDevice, stream));
    }
    PPCHK(hipMemcpyAsync(P->hkey, hkey, hcap * 4ull, hipMemcpyHostToDevice,
                         stream));
    PPCHK(hipMemcpyAsync(P->hval, hval, hcap * 4ull, hipMemcpyHostToDevice,
                         stream));
    PPCHK(hipStreamSynchronize(stream));
    return 0;
}

int srtp_gpu_pp_download(srtp_gpu_t *g, srtp_dev_stream_t *streams,
                         uint32_t *win, uint32_t *ns_now, uint64_t *kuses)
{
    PpState *P = pp_of(g);
    *ns_now = P->ns;
    hipStream_t stream = (hipStream_t)srtp_gpu_stream_of(g);
    PPCHK(hipMemcpyAsync(streams, P->st, P->ns * sizeof *streams,
                         hipMemcpyDeviceToHost, stream));
    if (P->nwords)
        PPCHK(hipMemcpyAsync(win, P->win, P->nwords * 4ull,
                             hipMemcpyDeviceToHost, stream));
    if (kuses && P->nmk)
        PPCHK(hipMemcpyAsync(kuses, P->kuses, P->nmk * 8ull,
                             hipMemcpyDeviceToHost, stream));
    PPCHK(hipStreamSynchronize(stream));
    return 0;
}

int srtp_gpu_pp_clone(srtp_gpu_t *g, const srtp_gpu_pp_batch_t *b,
                      uint32_t *added)
{
    PpState *P = pp_of(g);
    hipStream_t stream = (hipStream_t)b->stream;
    *added = 0;
    if (!P->has_tmpl || !b->n)
        return 0;
    const uint32_t N = (uint32_t)b->n;
    hipLaunchKernelGGL(k_clone_insert, dim3((N + 255) / 256), dim3(256), 0,
                       stream, b->in, b->in_off, b->in_len, N, P->hkey,
                       P->hval, P->hcap - 1, P->st, P->win, P->tmpl, P->ns0,
                       P->spare, P->tw, P->cl_ctl);
    PPCHK(hipGetLastError());
    uint32_t ctl[2];
    PPCHK(hipMemcpyAsync(ctl, P->cl_ctl, 8, hipMemcpyDeviceToHost, stream));
    PPCHK(hipStreamSynchronize(stream));
    const uint32_t total = ctl[0] < P->spare ? ctl[0] : P->spare;
    *added = P->ns0 + total - P->ns;
    P->ns = P->ns0 + total;
    // a clone's window starts empty in the shifted-window copy too
    if (*added)
        PPCHK(hipMemcpyAsync(P->wnew, P->win, P->nwords * 4ull,
                             hipMemcpyDeviceToDevice, stream));
    return ctl[1] ? 1 : 0;
}

int srtp_gpu_pp_pend_scan(srtp_gpu_t *g, const srtp_gpu_pp_batch_t *b,
                          int unprotect, const uint32_t *sids, uint32_t np,
                          srtp_pend_info_t *out)
{
    PpState *P = pp_of(g);
    hipStream_t stream = (hipStream_t)b->stream;
    if (!np || !P->st)
        return 0;
    if (regrow(&P->pd_first, &P->pd_cap, P->ns + 1) ||
        regrow(&P->pd_min, &P->pd_cap2, P->ns + 1) ||
        regrow(&P->pd_max, &P->pd_cap3, P->ns + 1) ||
        regrow(&P->pd_sids, &P->pd_list_cap, np) ||
        regrow(&P->pd_info, &P->pd_list_cap2, np))
        return -1;
    PPCHK(hipMemcpyAsync(P->pd_sids, sids, np * 4ull, hipMemcpyHostToDevice,
                         stream));
    const dim3 blk(256), gl((np + 255) / 256);
    hipLaunchKernelGGL(k_pend_reset, gl, blk, 0, stream, P->pd_sids, np,
                       P->pd_first, P->pd_min, P->pd_max);
    const uint32_t N = (uint32_t)b->n;
    if (N)
        hipLaunchKernelGGL(k_pend_scan, dim3((N + 255) / 256), blk, 0, stream,
                           b->in, b->in_off, b->in_len, b->out_len, P->st,
                           P->hkey, P->hval, P->hcap - 1, N, unprotect,
                           P->pd_first, P->pd_min, P->pd_max);
    hipLaunchKernelGGL(k_pend_gather, gl, blk, 0, stream, P->pd_sids, np, b->in,
                       b->in_off, P->st, P->pd_first, P->pd_min, P->pd_max,
                       P->pd_info);
    PPCHK(hipGetLastError());
    PPCHK(hipMemcpyAsync(out, P->pd_info, np * sizeof *out,
                         hipMemcpyDeviceToHost, stream));
    PPCHK(hipStreamSynchronize(stream));
    return 0;
}

int srtp_gpu_pp_pend_apply(srtp_gpu_t *g, const uint32_t *sids,
                           const uint64_t *efirst, const uint32_t *first,
                           uint32_t nr, void *stream_)
{
    PpState *P = pp_of(g);
    hipStream_t stream = (hipStream_t)stream_;
    P->pd_nres = 0;
    if (!nr)
        return 0;
    if (regrow(&P->pd_sids, &P->pd_list_cap, nr) ||
        regrow(&P->pd_efirst, &P->pd_list_cap3, nr) ||
        regrow(&P->pd_pos, &P->pd_pos_cap, nr) ||
        regrow(&P->pd_bak, &P->pd_bak_cap, nr) ||
        regrow(&P->pd_bakwin, &P->pd_bakwin_cap, P->nwords + 1))
        return -1;
    PPCHK(hipMemcpyAsync(P->pd_sids, sids, nr * 4ull, hipMemcpyHostToDevice,
                         stream));
    PPCHK(hipMemcpyAsync(P->pd_efirst, efirst, nr * 8ull,
                         hipMemcpyHostToDevice, stream));
    PPCHK(hipMemcpyAsync(P->pd_pos, first, nr * 4ull, hipMemcpyHostToDevice,
                         stream));
    hipLaunchKernelGGL(k_pend_apply, dim3((nr + 255) / 256), dim3(256), 0,
                       stream, P->pd_sids, P->pd_efirst, nr, P->st, P->win,
                       P->pd_bak, P->pd_bakwin);
    PPCHK(hipGetLastError());
    // the host arrays are the caller's stack: the copies complete first
    PPCHK(hipStreamSynchronize(stream));
    P->pd_nres = nr;
    return 0;
}

int srtp_gpu_pp_pend_restore(srtp_gpu_t *g, void *stream_)
{
    PpState *P = pp_of(g);
    hipStream_t stream = (hipStream_t)stream_;
    const uint32_t nr = P->pd_nres;
    P->pd_nres = 0;
    if (!nr)
        return 0;
    hipLaunchKernelGGL(k_pend_restore, dim3((nr + 255) / 256), dim3(256), 0,
                       stream, P->pd_sids, nr, P->st, P->win, P->pd_bak,
                       P->pd_bakwin);
    PPCHK(hipGetLastError());
    PPCHK(hipStreamSynchronize(stream));
    return 0;
}

void srtp_gpu_pp_pend_clear(srtp_gpu_t *g) { pp_of(g)->pd_nres = 0; }

// 48-bit index of every sorted position: the segmented sum of the advances
// by stream.  One stream: its chain packets come first and every other
// position has advance 0 and is never read back, so a plain prefix sum is
// the same and costs half the segmented one.
// Waits for the commit kernel's published abort word without waiting for
// the kernels queued after it.  Returns the word, or ABORT_UNSET when the
// stream drained without it (the caller then synchronises and reads the
// device word).
// A stream in an error state never publishes the word and never drains:
// any hipStreamQuery result but hipErrorNotReady ends the wait, with the
// error in *err (srtp_mi355x_debug_fail_async_wait injects one for tests).
static int g_fail_waits;

extern "C" void srtp_gpu_pp_debug_fail_waits(int n) { g_fail_waits = n; }

static uint32_t wait_published(PpState *P, hipStream_t stream, hipError_t *err)
{
    volatile uint32_t *w = (volatile uint32_t *)P->h_abort;
    *err = hipSuccess;
    if (g_fail_waits > 0) {
        g_fail_waits--;
        (void)hipStreamSynchronize(stream);   // leave nothing running
        *err = hipErrorLaunchFailure;
        return ABORT_UNSET;
    }
    for (uint32_t k = 1;; k++) {
        const uint32_t v = *w;
        if (v != ABORT_UNSET)
            return v;
        if ((k & 1023) == 0) {
            const hipError_t q = hipStreamQuery(stream);
            if (q == hipSuccess)
                return *w;
            if (q != hipErrorNotReady) {
                *err = q;
                return ABORT_UNSET;
            }
        }
        __builtin_ia32_pause();
    }
}

// the key buckets of an order-free batch with more than one key; the crypto
// batch then walks them (srtp_gpu_batch_t rec / rec_idx / rec_range)
static int bucket_pass(PpState *P, uint32_t N, const srtp_gpu_pp_batch_t *b,
                       srtp_gpu_batch_t *cb, hipStream_t stream)
{
    const uint32_t ns = P->ns;
    const dim3 blk(256), gp((N + 255) / 256), gs((ns + 255) / 256);
    hipLaunchKernelGGL(k_bk_offsets, dim3(1), dim3(1024), 0, stream,
                       P->bcount, ns, P->bk_off, P->bk_cur, P->bk_range);
    hipLaunchKernelGGL(k_bk_scatter, gp, blk, 0, stream, P->skey, P->pstat,
                       P->meta, b->in_off, b->out_off, N, ns, P->bk_off,
                       P->bk_cur, P->rec, P->rec_idx);
    hipLaunchKernelGGL(k_bk_pad, gs, blk, 0, stream, P->bcount, ns,
                       P->bk_off, P->bk_cur, P->rec);
    PPCHK(hipGetLastError());
    cb->rec = P->rec;
    cb->rec_idx = P->rec_idx;
    cb->rec_range = P->bk_range;
    return pp_step(stream, "buckets");
}

// Many-key batches through the key buckets: srtp_mi355x_set_key_buckets(1)
// or SRTP_PP_BUCKETS=1 always, (0) / =0 never, (-1, the default) for
// AES-GCM only.  AES-ICM: measured on configs[3] (64k streams x 128
// packets, round-robin) the bucketed kernel (one key per wave) took 2.51 ms
// against 2.53 ms with a key per lane, and the bucket pass 0.39 ms on top
// (DESIGN.md §4).  AES-GCM with a key per stream: the per-lane form reads
// each packet's GHASH table from global memory, and 64k keys' tables miss
// in L2 (9.8 ms for configs[3]'s shape); with a key per wave (k_gcm_bk, the
// key's table in LDS) 3.9 ms in all.  So by default a GCM batch with
// per-stream keys and at least BK_MIN packets a stream on average -- the
// streams that get wave buckets -- takes them.
static int g_buckets = -2;   // -2: not read from the environment yet

extern "C" void srtp_gpu_pp_set_buckets(int on)
{
    g_buckets = on < 0 ? -1 : on ? 1 : 0;
}

static int buckets_mode()
{
    if (g_buckets == -2) {
        const char *e = getenv("SRTP_PP_BUCKETS");
        g_buckets = e && *e == '1' ? 1 : e && *e == '0' ? 0 : -1;
    }
    return g_buckets;
}

// the key buckets for an order-free batch of N packets over ns streams
static bool buckets_for(const srtp_gpu_pp_batch_t *b, uint32_t N, uint32_t ns)
{
    if (b->uniform_key != 0xffffffffu)
        return false;
    const int m = buckets_mode();
    if (m >= 0)
        return m == 1;
    return b->mask && (b->mask & 0x440000u) == b->mask &&
           (uint64_t)N >= (uint64_t)BK_MIN * ns;
}

static hipError_t index_scan(PpState *P, uint32_t ns, uint32_t N,
                             hipStream_t stream)
{
    return srtp_scan::scan_run<srtp_scan::OP_SUM, false>(
        Seg64{ ns == 1 ? nullptr : P->skey2, P->val, P->est }, N, P->agg,
        stream);
}

// the stable order by stream: one stream, a partition of the chain packets
// (a scan and a scatter); several, a radix sort over the stream-id bits
static hipError_t stream_order(PpState *P, uint32_t ns, uint32_t N,
                               hipStream_t stream)
{
    if (ns == 1) {
        // perm (the sort's identity values) is free: it takes the scan
        hipError_t e = srtp_scan::scan_run<srtp_scan::OP_SUM, true>(
            ChainFlags{ P->skey, P->perm }, N, P->agg, stream);
        if (e != hipSuccess)
            return e;
        hipLaunchKernelGGL(k_pp_partition1, dim3((N + 255) / 256), dim3(256),
                           0, stream, P->skey, P->perm, N, P->skey2, P->perm2);
        return hipGetLastError();
    }
    // NOCHAIN keys truncate to all-ones > any stream id
    int end_bit = 1;
    while ((1u << end_bit) <= ns && end_bit < 32)
        end_bit++;
    return srtp_scan::radix_sort(P->skey, P->perm, P->skey2, P->perm2, N,
                                 end_bit, P->hist, P->agg, stream);
}

// SRTP_PP_FUSED=0: one-stream batches through the multi-launch chain form
// SRTP_PP_FUSED_OF=0: the order-free protect form classifies in its own
// kernel (k_pp_classify) again
static bool fused_of_on()
{
    static const bool on = [] {
        const char *e = getenv("SRTP_PP_FUSED_OF");
        return !(e && *e == '0');
    }();
    return on;
}

static bool fused_on()
{
    static const bool on = [] {
        const char *e = getenv("SRTP_PP_FUSED");
        return !(e && *e == '0');
    }();
    return on;
}

// SRTP_PP_INORDER=0: one-stream batches skip the in-order form (A/B runs)
static bool inorder_on()
{
    static const bool on = [] {
        const char *e = getenv("SRTP_PP_INORDER");
        return !(e && *e == '0');
    }();
    return on;
}

// After the synchronize that ends a receive batch's commit: the abort word
// and the failed-tag count its last kernel published to pinned memory, each
// copied from device memory instead if the mapped store was not seen.
static int pp_published(PpState *P, const uint32_t *abort, uint32_t *nfail)
{
    volatile uint32_t *h = (volatile uint32_t *)P->h_abort;
    if (h[0] == ABORT_UNSET)
        PPCHK(hipMemcpy(P->h_abort, abort, 4, hipMemcpyDeviceToHost));
    if (h[1] == ABORT_UNSET)
        PPCHK(hipMemcpy(nfail, P->fz_nfail, 4, hipMemcpyDeviceToHost));
    else
        *nfail = h[1];
    return 0;
}

// An error after k_pp_chain1 was queued: only k_pp_chain1_commit zeroes the
// look-back words, the tile ticket / key-use counters and the next batch's
// abort word, so they are zeroed here (else the next one-stream batch would
// start from stale prefixes and a nonzero ticket).
static int chain1_fail(PpState *P, hipStream_t stream)
{
    (void)hipMemsetAsync(P->ch_tile, 0, (P->ch_tiles_cap + 1) * 8, stream);
    (void)hipMemsetAsync(P->ch_ctl, 0, 8, stream);
    (void)hipMemsetAsync(P->ch_abort, 0, 8, stream);
    (void)hipStreamSynchronize(stream);
    return -1;
}

// the one-stream chain form in two launches (k_pp_chain1 + commit), then
// the crypto kernels; see k_pp_chain1
// One stream, in place, one uniform-key AES-ICM / GCM variant: the in-order form
// first -- no separate pre-pass kernel, the crypto kernel takes every
// packet's index from packet 0's (IcmChain) -- then k_io_commit.  A batch
// that is not a run of consecutive sequence numbers (or has a packet with
// a length / parse error) is restored and *declined: the chain form runs.
// The abort word is the chain form's pair (ch_abort[ch_par], zero at every
// batch's start: each batch's last kernel clears the other word, and
// chain1_fail both after an error), so no memset is queued per batch.
static int pp_protect_inorder_run(srtp_gpu_t *g, PpState *P,
                                  srtp_gpu_pp_batch_t *b, hipStream_t stream,
                                  int *fallback, bool *declined)
{
    const uint32_t N = (uint32_t)b->n;
    const dim3 blk(256), gp((N + 255) / 256);
    *declined = false;
    *(volatile uint32_t *)P->h_abort = ABORT_UNSET;
    uint32_t *ab = P->ch_abort + P->ch_par;
    uint32_t *ab_next = P->ch_abort + (P->ch_par ^ 1);
    P->ch_par ^= 1;
    // out of place or asynchronous: checked first (k_io_check), so the
    // crypto kernel runs only on a batch that commits
    const bool pre = b->in != b->out || b->in_off != b->out_off || b->async;
    if (pre) {
        hipLaunchKernelGGL(k_io_check, gp, blk, 0, stream, b->in, b->in_off,
                           b->in_len, b->out_len, N, P->st, ab, P->meta);
        if (b->async)
            hipLaunchKernelGGL(k_io_publish, dim3(1), dim3(64), 0, stream, ab,
                               P->h_abort_dev);
        PPCHK(hipGetLastError());
    }
    IcmChain Q;
    Q.in_len = b->in_len;
    Q.cap = b->out_len;
    Q.st = P->st;
    Q.abort = ab;
    Q.tsave = pre ? nullptr : P->tsave;
    srtp_gpu_batch_t cb = {};
    cb.n = b->n;
    cb.in = b->in;
    cb.in_off = b->in_off;
    cb.out = b->out;
    cb.out_off = b->out_off;
    cb.meta = P->meta;   // checked first: k_io_check's descriptors
    cb.auth_ok = nullptr;
    cb.uniform_key = b->uniform_key;
    cb.mask = b->mask;
    cb.stream = stream;
    // the kernel itself classifies (it always runs), unless checked first:
    // then it runs from the descriptors, or not at all when declined
    cb.abort = pre ? ab : nullptr;
    cb.inorder = pre ? nullptr : &Q;
    if (srtp_gpu_run(g, 0, &cb) || pp_step(stream, "in-order crypto"))
        return -1;
    // asynchronous: k_io_publish gave the verdict and the caller returns on
    // it, so the commit must not publish -- it may run after the NEXT call
    // has reset the word, and would hand that call this batch's verdict
    hipLaunchKernelGGL(k_io_commit, gp, blk, 0, stream, b->in, b->in_off,
                       b->in_len, N, P->st, P->win, ab, ab_next,
                       b->async ? nullptr : P->h_abort_dev, b->status,
                       b->out_len);
    PPCHK(hipGetLastError());
    if (pp_step(stream, "in-order commit"))
        return -1;
    if (b->async) {
        hipError_t we;
        const uint32_t v = wait_published(P, stream, &we);
        if (we != hipSuccess)
            return pp_fail(we, "waiting for the in-order verdict");
        if (v == 0) {
            // committed: the crypto kernel and the commit are queued
            b->sorted = 1;
            *fallback = 0;
            return 0;
        }
    }
    PPCHK(hipStreamSynchronize(stream));
    if (*(volatile uint32_t *)P->h_abort == ABORT_UNSET)
        PPCHK(hipMemcpy(P->h_abort, ab, 4, hipMemcpyDeviceToHost));
    if (*(volatile uint32_t *)P->h_abort == 0) {
        b->sorted = 1;
        *fallback = 0;
        return 0;
    }
    if (pre) {   // declined before the crypto ran: nothing was written
        *declined = true;
        return 0;
    }
    // declined: the input comes back exactly
    hipLaunchKernelGGL(k_io_restore_meta, gp, blk, 0, stream, b->in,
                       b->in_off, b->in_len, b->out_len, N, P->st,
                       (const uint8_t *)nullptr, P->meta, 0,
                       (const uint64_t *)nullptr);
    PPCHK(hipGetLastError());
    if (srtp_gpu_undo(g, b->n, b->out, b->out_off, P->meta, stream))
        return -1;
    hipLaunchKernelGGL(k_io_restore_tail, gp, blk, 0, stream, b->out,
                       b->out_off, b->in_len, P->st, P->meta, P->tsave, N);
    PPCHK(hipGetLastError());
    PPCHK(hipStreamSynchronize(stream));
    *declined = true;
    return 0;
}

static int pp_protect_inorder(srtp_gpu_t *g, PpState *P,
                              srtp_gpu_pp_batch_t *b, hipStream_t stream,
                              int *fallback, bool *declined)
{
    if (pp_protect_inorder_run(g, P, b, stream, fallback, declined))
        return chain1_fail(P, stream);
    return 0;
}

// The receive side: one stream, in place, one uniform-key AES-ICM / GCM
// variant, no MKI.  The crypto kernel verifies and decrypts every packet of
// the run (its index e_0 + i, srtp_fused.h inorder_meta), k_io_rx_commit
// takes the verdicts; the packets whose tag failed have their decryption
// undone.  A batch that is not one run (a reordered, repeated or missing-
// header packet, a length error) comes back exactly and *declined: the
// chain form (k_pu_chain1) runs it.
static int pp_unprotect_inorder_run(srtp_gpu_t *g, PpState *P,
                                    srtp_gpu_pp_batch_t *b, hipStream_t stream,
                                    int *fallback, bool *declined)
{
    const uint32_t N = (uint32_t)b->n;
    const dim3 blk(256), gp((N + 255) / 256);
    *declined = false;
    *(volatile uint32_t *)P->h_abort = ABORT_UNSET;
    ((volatile uint32_t *)P->h_abort)[1] = ABORT_UNSET;
    if (!P->io_e0)
        PPCHK(hipMalloc((void **)&P->io_e0, 8));
    uint32_t *abw = P->ch_abort + P->ch_par;   // as pp_protect_inorder
    uint32_t *ab_next = P->ch_abort + (P->ch_par ^ 1);
    P->ch_par ^= 1;
    IcmChain Q;
    Q.in_len = b->in_len;
    Q.cap = b->out_len;
    Q.st = P->st;
    Q.abort = abw;
    Q.tsave = nullptr;
    srtp_gpu_batch_t cb = {};
    cb.n = b->n;
    cb.in = b->in;
    cb.in_off = b->in_off;
    cb.out = b->out;
    cb.out_off = b->out_off;
    cb.meta = P->meta;   // not read
    cb.auth_ok = P->auth;
    cb.uniform_key = b->uniform_key;
    cb.mask = b->mask;
    cb.stream = stream;
    cb.abort = nullptr;
    cb.inorder = &Q;
    if (srtp_gpu_run(g, 1, &cb) || pp_step(stream, "in-order rx crypto"))
        return -1;
    // the per-block records (failure count, first / last accepted: 3 words
    // per 256-packet block) in the metadata area, which the in-order form
    // does not read (k_io_restore_meta writes it after the commit)
    uint32_t *brec = (uint32_t *)P->meta;
    hipLaunchKernelGGL(k_io_rx_status, gp, blk, 0, stream, b->in_len, P->auth,
                       N, gp.x, P->st, abw, brec, b->status, b->out_len);
    hipLaunchKernelGGL(k_io_rx_commit, dim3(1), dim3(1024), 0, stream, b->in,
                       b->in_off, P->auth, N, gp.x, P->st, P->win, abw,
                       ab_next, brec, P->fz_nfail, P->h_abort_dev, P->io_e0);
    PPCHK(hipGetLastError());
    if (pp_step(stream, "in-order rx commit"))
        return -1;
    PPCHK(hipStreamSynchronize(stream));
    uint32_t nfail = 0;
    if (pp_published(P, abw, &nfail))
        return -1;
    const bool ab = *(volatile uint32_t *)P->h_abort != 0;
    if (!ab && !nfail) {
        b->sorted = 1;
        *fallback = 0;
        return 0;
    }
    // the decryption of every packet that ran (declined) or of the ones
    // whose tag failed (accepted batch) is undone
    hipLaunchKernelGGL(k_io_restore_meta, gp, blk, 0, stream, b->in,
                       b->in_off, b->in_len, b->out_len, N, P->st,
                       ab ? (const uint8_t *)nullptr : (const uint8_t *)P->auth,
                       P->meta, 1, ab ? (const uint64_t *)nullptr : P->io_e0);
    PPCHK(hipGetLastError());
    if (srtp_gpu_undo(g, b->n, b->out, b->out_off, P->meta, stream))
        return -1;
    PPCHK(hipStreamSynchronize(stream));
    if (ab) {
        *declined = true;
        return 0;
    }
    b->sorted = 1;
    *fallback = 0;
    return 0;
}

static int pp_unprotect_inorder(srtp_gpu_t *g, PpState *P,
                                srtp_gpu_pp_batch_t *b, hipStream_t stream,
                                int *fallback, bool *declined)
{
    if (pp_unprotect_inorder_run(g, P, b, stream, fallback, declined))
        return chain1_fail(P, stream);
    return 0;
}

// MKI streams: the batch's per-packet key indices to the device (before
// any kernel of the batch; synchronous: the host array is the caller's)
static int mki_stage(PpState *P, const srtp_gpu_pp_batch_t *b,
                     hipStream_t stream)
{
    if (!b->mki)
        return 0;
    if (b->n > P->mki8_cap) {
        if (P->mki8)
            PPCHK(hipFree(P->mki8));
        P->mki8 = nullptr;
        PPCHK(hipMalloc((void **)&P->mki8, b->n));
        P->mki8_cap = b->n;
    }
    PPCHK(hipStreamSynchronize(stream));
    PPCHK(hipMemcpy(P->mki8, b->mki, b->n, hipMemcpyHostToDevice));
    return 0;
}

// ... and, after the commit, every MKI stream packet's key (k_mki_keys)
static void mki_keys(PpState *P, const srtp_gpu_pp_batch_t *b,
                     const uint32_t *abort, hipStream_t stream)
{
    if (!b->mki)
        return;
    const uint32_t N = (uint32_t)b->n;
    hipLaunchKernelGGL(k_mki_keys, dim3((N + 255) / 256), dim3(256), 0, stream,
                       b->in, b->in_off, b->in_len, P->st, P->hkey, P->hval,
                       P->hcap - 1, N, P->mki8, P->mkslot, P->kuses, P->meta,
                       abort);
}

static int pp_protect_chain1(srtp_gpu_t *g, PpState *P, srtp_gpu_pp_batch_t *b,
                             hipStream_t stream, int *fallback)
{
    const uint32_t N = (uint32_t)b->n;
    const uint32_t nt = (N + CH_TILE - 1) / CH_TILE;
    uint32_t *ab = P->ch_abort + P->ch_par;
    uint32_t *ab_next = P->ch_abort + (P->ch_par ^ 1);
    P->ch_par ^= 1;
    *(volatile uint32_t *)P->h_abort = ABORT_UNSET;
    Chain1Args A;
    A.C.in = b->in;
    A.C.in_off = b->in_off;
    A.C.in_len = b->in_len;
    A.C.cap = b->out_len;
    A.C.st = P->st;
    A.C.hkey = P->hkey;
    A.C.hval = P->hval;
    A.C.hmask = P->hcap - 1;
    A.C.n = N;
    A.C.hdr = P->hdr;
    A.C.pstat = P->pstat;
    A.C.skey = P->skey;
    A.C.perm = P->perm;
    A.C.bcount = P->bcount;
    A.C.abort = ab;
    A.C.est = P->est;
    A.C.new_index = nullptr;
    A.C.meta = P->meta;
    A.C.olen = P->skey2;   // protected lengths
    A.tile = P->ch_tile;
    A.ctl = P->ch_ctl;
    A.abort = ab;
    A.ntiles = nt;
    hipLaunchKernelGGL(k_pp_chain1, dim3(nt), dim3(CH_THREADS), 0, stream, A);
    if (const hipError_t le = hipGetLastError(); le != hipSuccess) {
        pp_fail(le, "k_pp_chain1");
        return chain1_fail(P, stream);
    }
    if (pp_step(stream, "chain1"))
        return chain1_fail(P, stream);
    Chain1Commit K;
    K.pstat = P->pstat;
    K.olen = P->skey2;
    K.est = P->est;
    K.n = N;
    K.st = P->st;
    K.win = P->win;
    K.tile = P->ch_tile;
    K.ctl = P->ch_ctl;
    K.ntiles = nt;
    K.abort = ab;
    K.abort_next = ab_next;
    K.pub = P->h_abort_dev;
    K.status = b->status;
    K.out_len = b->out_len;
    hipLaunchKernelGGL(k_pp_chain1_commit,
                       dim3((N + CH_COMMIT_THREADS - 1) / CH_COMMIT_THREADS),
                       dim3(CH_COMMIT_THREADS), 0, stream, K);
    if (const hipError_t le = hipGetLastError(); le != hipSuccess) {
        pp_fail(le, "k_pp_chain1_commit");
        return chain1_fail(P, stream);
    }
    if (pp_step(stream, "chain1_commit"))
        return chain1_fail(P, stream);
    mki_keys(P, b, ab, stream);
    srtp_gpu_batch_t cb = {};
    cb.n = b->n;
    cb.in = b->in;
    cb.in_off = b->in_off;
    cb.out = b->out;
    cb.out_off = b->out_off;
    cb.meta = P->meta;
    cb.auth_ok = nullptr;
    cb.uniform_key = b->uniform_key;
    cb.mask = b->mask;
    cb.stream = stream;
    cb.abort = ab;
    if (srtp_gpu_run(g, 0, &cb))
        return -1;
    if (pp_step(stream, "crypto"))
        return -1;
    b->sorted = 1;
    if (b->async) {
        hipError_t we;
        const uint32_t v = wait_published(P, stream, &we);
        if (we != hipSuccess)
            return pp_fail(we, "waiting for the pre-pass verdict");
        if (v == 0) {
            *fallback = 0;
            return 0;
        }
    }
    PPCHK(hipStreamSynchronize(stream));
    if (*(volatile uint32_t *)P->h_abort == ABORT_UNSET)
        PPCHK(hipMemcpy(P->h_abort, ab, 4, hipMemcpyDeviceToHost));
    *fallback = (int)*P->h_abort;
    return 0;
}

// The order-free form with its classification inside the crypto kernel
// (IcmFused, srtp_icm.hip fz_classify): no separate header pass -- every
// packet's first line is read once, by the kernel that encrypts it.  The
// conditions of the order-free form (k_pp_usetbits) are checked after the
// crypto; a batch outside them (or with an unknown / ineligible stream) is
// restored -- k_undo_wave re-applies the keystream, k_pp_tail_restore writes back
// the bytes the tags overwrote -- and, for AB_ORDER, *sorted set: the caller
// runs the sorted chain form, else the host decides (*fallback).  Only in
// place, one AES-ICM kernel variant, trailers <= 16 bytes (fused_ok).
static int pp_protect_fused(srtp_gpu_t *g, PpState *P, srtp_gpu_pp_batch_t *b,
                            hipStream_t stream, int *fallback, bool *sorted)
{
    const uint32_t N = (uint32_t)b->n, ns = P->ns;
    const dim3 blk(256), gp((N + 255) / 256), gs((ns + 255) / 256);
    *sorted = false;
    *(volatile uint32_t *)P->h_abort = ABORT_UNSET;
    ((volatile uint32_t *)P->h_abort)[1] = ABORT_UNSET;
    unsigned long long *hi = (unsigned long long *)P->new_index;
    hipLaunchKernelGGL(k_fz_reset, dim3(ns / 256 + 1), blk, 0, stream,
                       P->abort, P->fz_cnt, hi, P->fz_emin, nullptr, nullptr,
                       P->fz_glist, ns);
    IcmFused F;
    F.in_len = b->in_len;
    F.cap = b->out_len;
    F.status = b->status;
    F.st = P->st;
    F.hkey = P->hkey;
    F.hval = P->hval;
    F.hmask = P->hcap - 1;
    F.rec = P->fzrec;
    F.tsave = P->tsave;
    F.max_trailer = b->max_trailer;
    F.glist = P->fz_glist;
    F.cnt = P->fz_cnt;
    F.new_index = hi;
    F.emin = P->fz_emin;
    F.bmap = P->fz_bmap;
    F.abort = P->abort;
    srtp_gpu_batch_t cb = {};
    cb.n = b->n;
    cb.in = b->in;
    cb.in_off = b->in_off;
    cb.out = b->out;
    cb.out_off = b->out_off;
    cb.meta = P->meta;
    cb.auth_ok = nullptr;
    // one key for every stream: k_gcm's fused form with its LDS tables
    // (k_icm_hmac's fused form takes per-lane keys)
    cb.uniform_key = (b->mask & 0x440000u) ? b->uniform_key : 0xffffffffu;
    cb.mask = b->mask;
    cb.stream = stream;
    cb.abort = nullptr;   // the kernel itself classifies: it always runs
    cb.fused = &F;
    // a failed step may leave bitmap bits behind: clear them all
    auto fail = [&]() {
        (void)hipMemsetAsync(P->fz_bmap, 0, (4ull * P->nwords + 4) * 4, stream);
        return -1;
    };
    if (srtp_gpu_run(g, 0, &cb) || pp_step(stream, "fused crypto"))
        return fail();
    hipLaunchKernelGGL(k_fz_stream, gs, blk, 0, stream, P->st, ns, P->fz_cnt,
                       hi, P->fz_emin, P->fz_bmap, P->win, P->wnew, P->abort);
    hipLaunchKernelGGL(k_fz_commit, gs, blk, 0, stream, P->st, ns, P->fz_cnt,
                       hi, P->wnew, P->win, P->abort, P->h_abort_dev);
    if (hipGetLastError() != hipSuccess || pp_step(stream, "fused commit"))
        return fail();
    PPCHK(hipStreamSynchronize(stream));
    if (*(volatile uint32_t *)P->h_abort == ABORT_UNSET)
        PPCHK(hipMemcpy(P->h_abort, P->abort, 4, hipMemcpyDeviceToHost));
    const uint32_t ab = *(volatile uint32_t *)P->h_abort;
    *fallback = (int)ab;
    if (!ab)
        return 0;
    // declined: the input comes back exactly
    hipLaunchKernelGGL(k_fz_meta, gp, blk, 0, stream, b->in, b->in_off,
                       b->in_len, P->fzrec, P->st, N, P->meta, b->out_len, 0,
                       nullptr);
    PPCHK(hipGetLastError());
    if (srtp_gpu_undo(g, b->n, b->out, b->out_off, P->meta, stream))
        return -1;
    hipLaunchKernelGGL(k_pp_tail_restore, gp, blk, 0, stream, b->out,
                       b->out_off, b->in_len, P->st, P->meta, P->fzrec,
                       P->tsave, N);
    PPCHK(hipGetLastError());
    PPCHK(hipStreamSynchronize(stream));
    *sorted = ab == AB_ORDER;
    return 0;
}

int srtp_gpu_pp_protect(srtp_gpu_t *g, srtp_gpu_pp_batch_t *b,
                        int *fallback)
{
    *fallback = 1;
    b->sorted = 0;
    PpState *P = pp_of(g);
    const size_t n = b->n;
    if (!n) {
        *fallback = 0;
        return 0;
    }
    if (!P->st || n > 0x7fffffffu)
        return 0;
    if (!P->ns) {
        // a template and no stream yet: every packet's stream is a clone
        if (P->has_tmpl)
            *fallback = AB_UNKNOWN_SSRC;
        return 0;
    }
    hipStream_t stream = (hipStream_t)b->stream;   // NULL = the null stream
    if (reserve_packets(P, n, stream) || pp_step(stream, "reserve") ||
        mki_stage(P, b, stream))
        return -1;
    const uint32_t N = (uint32_t)n, ns = P->ns;
    const dim3 blk(256), gp((N + 255) / 256), gs((ns + 255) / 256);
    if (ns == 1 && fused_on()) {
        if (b->inorder_ok && inorder_on()) {
            bool declined = false;
            if (pp_protect_inorder(g, P, b, stream, fallback, &declined))
                return -1;
            b->inorder = declined ? 2 : 1;
            if (!declined)
                return 0;
        }
        return pp_protect_chain1(g, P, b, stream, fallback);
    }

    // many streams: the order-free form first (no sort); AB_ORDER -> again
    // through the sorted chain path.  SRTP_PP_SORTED=1 forces the latter.
    static const bool force_sorted = [] {
        const char *e = getenv("SRTP_PP_SORTED");
        return e && *e == '1';
    }();
    bool unordered = ns > 1 && !force_sorted;
    if (unordered && b->fused_ok && !b->mki && fused_of_on() &&
        !buckets_for(b, N, ns)) {
        bool sorted = false;
        if (pp_protect_fused(g, P, b, stream, fallback, &sorted))
            return -1;
        if (!sorted)
            return 0;
        unordered = false;   // restored, nothing committed: the chain form
        b->bucketed = 0;
    }
    for (;;) {
    *(volatile uint32_t *)P->h_abort = ABORT_UNSET;
    hipLaunchKernelGGL(k_pp_reset, dim3(ns / 256 + 1), blk, 0, stream, P->abort, P->bcount,
                       (unsigned long long *)P->new_index, nullptr, nullptr,
                       ns);

    ClassifyArgs C;
    C.in = b->in;
    C.in_off = b->in_off;
    C.in_len = b->in_len;
    C.cap = b->out_len;
    C.st = P->st;
    C.hkey = P->hkey;
    C.hval = P->hval;
    C.hmask = P->hcap - 1;
    C.n = N;
    C.hdr = P->hdr;
    C.pstat = P->pstat;
    C.skey = P->skey;
    C.perm = P->perm;
    C.bcount = P->bcount;
    C.abort = P->abort;
    C.est = unordered ? P->est : nullptr;
    C.new_index = unordered ? (unsigned long long *)P->new_index : nullptr;
    C.meta = P->meta;
    C.olen = P->skey2;   // protected lengths (skey2 is the sorted path's)
    hipLaunchKernelGGL(k_pp_classify, gp, blk, 0, stream, C);
    PPCHK(hipGetLastError());
    if (pp_step(stream, "classify"))
        return -1;

    CommitArgs K;
    if (unordered) {
        hipLaunchKernelGGL(k_pp_window, gs, blk, 0, stream, P->st, ns,
                           P->new_index, P->win, P->wnew);
        hipLaunchKernelGGL(k_pp_usetbits, gp, blk, 0, stream, P->skey, P->est,
                           P->st, ns, N, P->new_index, P->wnew, P->abort);
        PPCHK(hipGetLastError());
        if (pp_step(stream, "usetbits"))
            return -1;
        K.skey2 = P->skey;   // packet order: perm is the identity
        K.perm2 = P->perm;
    } else {
    PPCHK(stream_order(P, ns, N, stream));
    if (pp_step(stream, "sort"))
        return -1;
    hipLaunchKernelGGL(k_pp_delta, gp, blk, 0, stream, P->skey2, P->perm2,
                       P->hdr, P->st, ns, N, P->val, P->seg_first, P->abort);
    PPCHK(hipGetLastError());
    if (pp_step(stream, "delta"))
        return -1;
    PPCHK(index_scan(P, ns, N, stream));
    if (pp_step(stream, "scan"))
        return -1;
    hipLaunchKernelGGL(k_pp_seg_end, gp, blk, 0, stream, P->skey2, P->est, ns,
                       N, P->seg_first, P->bcount, P->new_index);
    if (pp_step(stream, "seg_end"))
        return -1;
    hipLaunchKernelGGL(k_pp_window, gs, blk, 0, stream, P->st, ns,
                       P->new_index, P->win, P->wnew);
    if (pp_step(stream, "window"))
        return -1;
    hipLaunchKernelGGL(k_pp_setbits, gp, blk, 0, stream, P->skey2, P->est,
                       P->st, ns, N, P->new_index, P->wnew);
    if (pp_step(stream, "setbits"))
        return -1;
        K.skey2 = P->skey2;
        K.perm2 = P->perm2;
    }
    K.pstat = P->pstat;
    K.est = P->est;
    K.hdr = P->hdr;
    K.st = P->st;
    K.ns = ns;
    K.n = N;
    K.abort = P->abort;
    K.meta = P->meta;
    K.status = b->status;
    K.out_len = b->out_len;
    if (unordered)
        hipLaunchKernelGGL(k_pp_commit_of, gp, blk, 0, stream, P->pstat,
                           P->skey2, N, P->abort, b->status, b->out_len);
    else
        hipLaunchKernelGGL(k_pp_commit_pkt, gp, blk, 0, stream, K);
    if (pp_step(stream, "commit_pkt"))
        return -1;
    hipLaunchKernelGGL(k_pp_commit_stream, gs, blk, 0, stream, P->st, ns,
                       P->new_index, P->bcount, P->wnew, P->win, P->abort,
                       P->h_abort_dev);
    PPCHK(hipGetLastError());
    if (pp_step(stream, "commit_stream"))
        return -1;
    mki_keys(P, b, P->abort, stream);

    srtp_gpu_batch_t cb = {};
    // (not with MKI streams: k_mki_keys gave their packets a key each, and
    // the bucketed kernel takes one key per 64-record group)
    if (unordered && buckets_for(b, N, ns) && !b->mki) {
        if (bucket_pass(P, N, b, &cb, stream))
            return -1;
        b->bucketed = 1;
    }
    cb.n = n;
    cb.in = b->in;
    cb.in_off = b->in_off;
    cb.out = b->out;
    cb.out_off = b->out_off;
    cb.meta = P->meta;
    cb.auth_ok = nullptr;
    cb.uniform_key = b->uniform_key;
    cb.mask = b->mask;
    cb.stream = stream;
    cb.abort = P->abort;
    if (srtp_gpu_run(g, 0, &cb))
        return -1;
    if (pp_step(stream, "crypto"))
        return -1;
    // the commit kernel published the final abort word to host memory
    if (b->async) {
        hipError_t we;
        const uint32_t v = wait_published(P, stream, &we);
        if (we != hipSuccess)
            return pp_fail(we, "waiting for the pre-pass verdict");
        if (v == 0) {
            // committed: the crypto kernel is queued behind it on the stream
            b->sorted = !unordered;
            *fallback = 0;
            return 0;
        }
    }
    PPCHK(hipStreamSynchronize(stream));
    if (*(volatile uint32_t *)P->h_abort == ABORT_UNSET)
        PPCHK(hipMemcpy(P->h_abort, P->abort, 4, hipMemcpyDeviceToHost));
    if (unordered && *P->h_abort == AB_ORDER) {
        unordered = false;   // nothing was committed: the sorted path
        b->bucketed = 0;
        continue;
    }
    b->sorted = !unordered;
    *fallback = (int)*P->h_abort;   // abort reason bits (AB_*), 0 = done
    return 0;
    }
}

// an error after k_pu_chain1 was queued: both control blocks and the
// look-back words back to their reset state (normally the commit's job)
static int pu1_fail(PpState *P, hipStream_t stream)
{
    PuCtl h[2];
    memset(h, 0, sizeof h);
    h[0].umin = h[1].umin = ~0ull;
    (void)hipMemcpyAsync(P->pu_ctl, h, sizeof h, hipMemcpyHostToDevice, stream);
    (void)hipMemsetAsync(P->pu_tile, 0, 2 * (P->ch_tiles_cap + 1) * 8, stream);
    (void)hipStreamSynchronize(stream);
    return -1;
}

#define PU1CHK(x, what)                                                        \
    do {                                                                       \
        const hipError_t e_ = (x);                                             \
        if (e_ != hipSuccess) {                                                \
            pp_fail(e_, what);                                                 \
            return pu1_fail(P, stream);                                        \
        }                                                                      \
    } while (0)

// one stream: k_pu_chain1 -> crypto -> k_pu_first -> k_pu_verdict1 ->
// k_pu_commit1 -> undo (see k_pu_chain1)
static int pp_unprotect_chain1(srtp_gpu_t *g, PpState *P,
                               srtp_gpu_pp_batch_t *b, hipStream_t stream,
                               int *fallback)
{
    const uint32_t N = (uint32_t)b->n;
    const uint32_t nt = (N + CH_TILE - 1) / CH_TILE;
    // duplicates' index range: up to 4 indices per packet plus a window
    const uint64_t fcap = 4ull * N + 65536;
    if (fcap > P->pu_first_cap) {
        if (P->pu_first)
            PPCHK(hipFree(P->pu_first));
        P->pu_first = nullptr;
        PPCHK(hipMalloc((void **)&P->pu_first, fcap * 8));
        PPCHK(hipMemsetAsync(P->pu_first, 0xff, fcap * 8, stream));
        P->pu_first_cap = fcap;
    }
    if (++P->pu_gen == 0) {   // generations wrapped: forget every entry
        PPCHK(hipMemsetAsync(P->pu_first, 0xff, P->pu_first_cap * 8, stream));
        P->pu_gen = 1;
    }
    PuCtl *ctl = P->pu_ctl + P->pu_par, *nxt = P->pu_ctl + (P->pu_par ^ 1);
    P->pu_par ^= 1;
    uint64_t *tile = P->pu_tile, *vtile = P->pu_tile + P->ch_tiles_cap + 1;
    *(volatile uint32_t *)P->h_abort = ABORT_UNSET;
    PuChainArgs A;
    A.C.in = b->in;
    A.C.in_off = b->in_off;
    A.C.in_len = b->in_len;
    A.C.cap = b->out_len;
    A.C.st = P->st;
    A.C.hkey = P->hkey;
    A.C.hval = P->hval;
    A.C.hmask = P->hcap - 1;
    A.C.n = N;
    A.C.hdr = P->hdr;
    A.C.pstat = P->pstat;
    A.C.skey = P->skey;
    A.C.perm = P->perm;
    A.C.bcount = P->bcount;
    A.C.abort = nullptr;
    A.C.est = P->est;
    A.C.new_index = nullptr;
    A.C.meta = P->meta;
    A.C.olen = nullptr;
    A.C.keys = g->d_keys;
    A.C.mkslot = P->mkslot;
    A.C.rxj = P->rxj;
    A.auth = P->auth;
    A.tile = tile;
    A.ctl = ctl;
    hipLaunchKernelGGL(k_pu_chain1, dim3(nt), dim3(CH_THREADS), 0, stream, A);
    PU1CHK(hipGetLastError(), "k_pu_chain1");
    if (pp_step(stream, "pu_chain1"))
        return pu1_fail(P, stream);
    srtp_gpu_batch_t cb = {};
    cb.n = b->n;
    cb.in = b->in;
    cb.in_off = b->in_off;
    cb.out = b->out;
    cb.out_off = b->out_off;
    cb.meta = P->meta;
    cb.auth_ok = P->auth;
    cb.uniform_key = b->uniform_key;
    cb.mask = b->mask;
    cb.stream = stream;
    cb.abort = &ctl->abort1;
    if (srtp_gpu_run(g, 1, &cb) || pp_step(stream, "pu_crypto"))
        return pu1_fail(P, stream);
    const dim3 blk(256), gp((N + 255) / 256);
    if (P->pd_nres)
        hipLaunchKernelGGL(k_pend_authchk, dim3((P->pd_nres + 255) / 256), blk,
                           0, stream, P->pd_pos, P->pd_nres, P->auth,
                           &ctl->abort2);
    hipLaunchKernelGGL(k_pu_first, gp, blk, 0, stream, P->skey, P->est,
                       P->auth, N, ctl, P->pu_first, P->pu_first_cap,
                       P->pu_gen);
    PuVerdictArgs V;
    V.skey = P->skey;
    V.est = P->est;
    V.auth = P->auth;
    V.first = P->pu_first;
    V.st = P->st;
    V.win = P->win;
    V.n = N;
    V.tile = vtile;
    V.ctl = ctl;
    V.pstat = P->pstat;
    V.top = P->top;
    V.gen = P->pu_gen;
    V.first_cap = P->pu_first_cap;
    hipLaunchKernelGGL(k_pu_verdict1, dim3(nt), dim3(CH_THREADS), 0, stream, V);
    PU1CHK(hipGetLastError(), "k_pu_verdict1");
    if (pp_step(stream, "pu_verdict1"))
        return pu1_fail(P, stream);
    PuCommitArgs K;
    K.skey = P->skey;
    K.pstat = P->pstat;
    K.in_len = b->in_len;
    K.est = P->est;
    K.top = P->top;
    K.n = N;
    K.st = P->st;
    K.win = P->win;
    K.tile = tile;
    K.vtile = vtile;
    K.ntiles = nt;
    K.ctl = ctl;
    K.ctl_next = nxt;
    K.pub = P->h_abort_dev;
    K.meta = P->meta;
    K.status = b->status;
    K.out_len = b->out_len;
    hipLaunchKernelGGL(k_pu_commit1,
                       dim3((N + CH_COMMIT_THREADS - 1) / CH_COMMIT_THREADS),
                       dim3(CH_COMMIT_THREADS), 0, stream, K);
    PU1CHK(hipGetLastError(), "k_pu_commit1");
    if (b->mki_rx)
        hipLaunchKernelGGL(k_mki_rx_charge, gp, blk, 0, stream, b->in,
                           b->in_off, b->in_len, P->st, P->hkey, P->hval,
                           P->hcap - 1, N, P->rxj, P->kuses, b->status,
                           &ctl->abort1, &ctl->abort2);
    if (pp_step(stream, "pu_commit1"))
        return pu1_fail(P, stream);
    // rejected packets (every candidate after a post-crypto abort): their
    // speculative decryption is undone
    if (srtp_gpu_undo(g, b->n, b->out, b->out_off, P->meta, stream))
        return -1;
    PPCHK(hipStreamSynchronize(stream));
    *fallback = (int)*(volatile uint32_t *)P->h_abort;
    b->sorted = 1;
    return 0;
}

// The order-free receive form with its classification inside the AES-ICM
// kernel (IcmFused, srtp_icm.hip fzu_classify / fzu_verdict): no separate
// header, meta, accept or set-bits passes.  The conditions are checked on
// per-stream aggregates afterwards (k_fzu_stream); a batch outside them
// comes back exactly (every candidate's decryption undone, capacities
// restored) and, for AB_ORDER, *sorted is set: the sorted chain form runs
// it, else the host does.  Only in place, per-lane keys, one AES-ICM kernel
// variant, several streams (fused_ok).
static int pp_unprotect_fused(srtp_gpu_t *g, PpState *P,
                              srtp_gpu_pp_batch_t *b, hipStream_t stream,
                              int *fallback, bool *sorted)
{
    const uint32_t N = (uint32_t)b->n, ns = P->ns;
    const dim3 blk(256), gp((N + 255) / 256), gs((ns + 255) / 256);
    *sorted = false;
    *(volatile uint32_t *)P->h_abort = ABORT_UNSET;
    ((volatile uint32_t *)P->h_abort)[1] = ABORT_UNSET;
    unsigned long long *hi = (unsigned long long *)P->new_index;
    hipLaunchKernelGGL(k_fz_reset, dim3(ns / 256 + 1), blk, 0, stream,
                       P->abort, P->fz_cnt, hi, P->fz_emin, P->fz_hicand,
                       P->fz_nfail, P->fz_glist, ns);
    IcmFused F;
    F.in_len = b->in_len;
    F.cap = b->out_len;
    F.status = b->status;
    F.st = P->st;
    F.hkey = P->hkey;
    F.hval = P->hval;
    F.hmask = P->hcap - 1;
    F.rec = P->fzrec;
    F.tsave = nullptr;
    F.max_trailer = 0;
    F.glist = P->fz_glist;
    F.cnt = P->fz_cnt;
    F.new_index = hi;
    F.emin = P->fz_emin;
    F.bmap = P->fz_bmap;
    F.abort = P->abort;
    F.hicand = P->fz_hicand;
    F.bmap2 = P->fz_bmap + 2 * P->nwords + 2;
    F.nfail = P->fz_nfail;
    srtp_gpu_batch_t cb = {};
    cb.n = b->n;
    cb.in = b->in;
    cb.in_off = b->in_off;
    cb.out = b->out;
    cb.out_off = b->out_off;
    cb.meta = P->meta;
    cb.auth_ok = P->auth;
    // one key for every stream: k_gcm's fused form with its LDS tables
    // (k_icm_hmac's fused form takes per-lane keys)
    cb.uniform_key = (b->mask & 0x440000u) ? b->uniform_key : 0xffffffffu;
    cb.mask = b->mask;
    cb.stream = stream;
    cb.abort = nullptr;   // the kernel itself classifies: it always runs
    cb.fused = &F;
    auto fail = [&]() {
        (void)hipMemsetAsync(P->fz_bmap, 0, (4ull * P->nwords + 4) * 4, stream);
        return -1;
    };
    if (srtp_gpu_run(g, 1, &cb) || pp_step(stream, "fused unprotect crypto"))
        return fail();
    if (P->pd_nres)
        hipLaunchKernelGGL(k_pend_authchk, dim3((P->pd_nres + 255) / 256), blk,
                           0, stream, P->pd_pos, P->pd_nres, P->auth, P->abort);
    hipLaunchKernelGGL(k_fzu_stream, gs, blk, 0, stream, P->st, ns, P->fz_cnt,
                       hi, P->fz_hicand, P->fz_emin, P->fz_bmap, F.bmap2,
                       P->win, P->wnew, P->abort);
    hipLaunchKernelGGL(k_fzu_commit, gs, blk, 0, stream, P->st, ns, P->fz_cnt,
                       hi, P->wnew, P->win, P->abort, P->h_abort_dev,
                       P->fz_nfail);
    if (hipGetLastError() != hipSuccess ||
        pp_step(stream, "fused unprotect commit"))
        return fail();
    PPCHK(hipStreamSynchronize(stream));
    uint32_t nfail = 0;
    if (pp_published(P, P->abort, &nfail))
        return -1;
    const uint32_t ab = *(volatile uint32_t *)P->h_abort;
    *fallback = (int)ab;
    if (!ab && !nfail)
        return 0;
    // declined: every candidate back to its ciphertext, the capacities
    // back; accepted: the candidates whose tag failed back to ciphertext
    hipLaunchKernelGGL(k_fz_meta, gp, blk, 0, stream, b->in, b->in_off,
                       b->in_len, P->fzrec, P->st, N, P->meta, b->out_len, 1,
                       ab ? nullptr : (const int32_t *)b->status);
    PPCHK(hipGetLastError());
    if (srtp_gpu_undo(g, b->n, b->out, b->out_off, P->meta, stream))
        return -1;
    PPCHK(hipStreamSynchronize(stream));
    *sorted = ab == AB_ORDER;
    return 0;
}

int srtp_gpu_pp_unprotect(srtp_gpu_t *g, srtp_gpu_pp_batch_t *b,
                          int *fallback)
{
    *fallback = 1;
    b->sorted = 0;
    PpState *P = pp_of(g);
    const size_t n = b->n;
    if (!n) {
        *fallback = 0;
        return 0;
    }
    if (!P->st || n > 0x7fffffffu)
        return 0;
    if (!P->ns) {
        if (P->has_tmpl)
            *fallback = AB_UNKNOWN_SSRC;
        return 0;
    }
    hipStream_t stream = (hipStream_t)b->stream;   // NULL = the null stream
    if (reserve_packets(P, n, stream) || pp_step(stream, "reserve"))
        return -1;
    const uint32_t N = (uint32_t)n, ns = P->ns;
    const dim3 blk(256), gp((N + 255) / 256), gs((ns + 255) / 256);
    static const bool force_sorted = [] {
        const char *e = getenv("SRTP_PP_SORTED");
        return e && *e == '1';
    }();
    // one stream: the fused chain form, in order or not (k_pu_chain1);
    // several: order-free first, then the sorted chain form
    if (ns == 1 && fused_on()) {
        // (a pending ROC applied to this batch needs k_pend_authchk: the
        // chain form)
        if (b->inorder_ok && inorder_on() && !P->pd_nres) {
            bool declined = false;
            if (pp_unprotect_inorder(g, P, b, stream, fallback, &declined))
                return -1;
            b->inorder = declined ? 2 : 1;
            if (!declined)
                return 0;
        }
        return pp_unprotect_chain1(g, P, b, stream, fallback);
    }
    bool unordered = ns > 1 && !force_sorted;
    if (unordered && b->fused_ok && fused_of_on() &&
        !buckets_for(b, N, ns)) {
        bool sorted = false;
        if (pp_unprotect_fused(g, P, b, stream, fallback, &sorted))
            return -1;
        if (!sorted) {
            b->sorted = 0;
            return 0;
        }
        unordered = false;   // restored, nothing committed: the chain form
        b->bucketed = 0;
    }
    for (;;) {
    *(volatile uint32_t *)P->h_abort = ABORT_UNSET;
    hipLaunchKernelGGL(k_pp_reset, dim3(ns / 256 + 1), blk, 0, stream, P->abort, P->bcount,
                       (unsigned long long *)P->new_index, P->bcount2,
                       (unsigned long long *)P->new_index2, ns);

    ClassifyArgs C;
    C.in = b->in;
    C.in_off = b->in_off;
    C.in_len = b->in_len;
    C.cap = b->out_len;
    C.st = P->st;
    C.hkey = P->hkey;
    C.hval = P->hval;
    C.hmask = P->hcap - 1;
    C.n = N;
    C.hdr = P->hdr;
    C.pstat = P->pstat;
    C.skey = P->skey;
    C.perm = P->perm;
    C.bcount = P->bcount;
    C.abort = P->abort;
    C.est = unordered ? P->est : nullptr;
    C.new_index = unordered ? (unsigned long long *)P->new_index : nullptr;
    C.keys = g->d_keys;
    C.mkslot = P->mkslot;
    C.rxj = P->rxj;
    hipLaunchKernelGGL(k_pu_classify, gp, blk, 0, stream, C);
    PPCHK(hipGetLastError());
    const uint32_t *ks, *kp;   // the order the kernels below walk
    if (unordered) {
        // order-free conditions and duplicates over every candidate
        hipLaunchKernelGGL(k_pp_window, gs, blk, 0, stream, P->st, ns,
                           P->new_index, P->win, P->wnew);
        hipLaunchKernelGGL(k_pp_usetbits, gp, blk, 0, stream, P->skey, P->est,
                           P->st, ns, N, P->new_index, P->wnew, P->abort);
        ks = P->skey;
        kp = nullptr;   // the packet order itself
    } else {
        // chain form: stable stream order, advances, segmented sum
        PPCHK(stream_order(P, ns, N, stream));
        hipLaunchKernelGGL(k_pp_delta, gp, blk, 0, stream, P->skey2, P->perm2,
                           P->hdr, P->st, ns, N, P->val, P->seg_first,
                           P->abort);
        PPCHK(index_scan(P, ns, N, stream));
        // candidates per stream (AES-GCM key usage)
        hipLaunchKernelGGL(k_pp_seg_end, gp, blk, 0, stream, P->skey2, P->est,
                           ns, N, P->seg_first, P->bcount, P->new_index);
        ks = P->skey2;
        kp = P->perm2;
    }
    hipLaunchKernelGGL(k_pu_meta, gp, blk, 0, stream, ks, kp, P->est, P->hdr,
                       P->st, ns, N, P->abort, P->meta, P->auth, P->mkslot,
                       P->rxj);
    PPCHK(hipGetLastError());
    if (pp_step(stream, "pu_prepass"))
        return -1;

    srtp_gpu_batch_t cb = {};
    // (not with MKI streams: their packets carry a key each, and the
    // bucketed kernel takes one key per 64-record group)
    if (unordered && buckets_for(b, N, ns) && !b->mki_rx) {
        if (bucket_pass(P, N, b, &cb, stream))
            return -1;
        b->bucketed = 1;
    }
    cb.n = n;
    cb.in = b->in;
    cb.in_off = b->in_off;
    cb.out = b->out;
    cb.out_off = b->out_off;
    cb.meta = P->meta;
    cb.auth_ok = P->auth;
    cb.uniform_key = b->uniform_key;
    cb.mask = b->mask;
    cb.stream = stream;
    cb.abort = P->abort;
    if (srtp_gpu_run(g, 1, &cb))
        return -1;
    if (pp_step(stream, "pu_crypto"))
        return -1;
    if (P->pd_nres)
        hipLaunchKernelGGL(k_pend_authchk, dim3((P->pd_nres + 255) / 256), blk,
                           0, stream, P->pd_pos, P->pd_nres, P->auth, P->abort);

    if (!unordered) {
        hipLaunchKernelGGL(k_pu_accepted_est, gp, blk, 0, stream, P->skey2,
                           P->perm2, P->est, P->auth, ns, N, P->val);
        PPCHK((srtp_scan::scan_run<srtp_scan::OP_MAX, true>(
            Seg64{ P->skey2, P->val, P->top }, N, P->agg, stream)));
        hipLaunchKernelGGL(k_pu_top_check, gp, blk, 0, stream, P->skey2,
                           P->perm2, P->hdr, P->est, P->top, P->st, ns, N,
                           P->abort);
    }
    // 1024-thread blocks: agg_stream merges a block's waves, so one stream's
    // batch costs one same-address atomic pair per 1024 packets
    hipLaunchKernelGGL(k_pu_accept, dim3((N + 1023) / 1024), dim3(1024), 0,
                       stream, ks, kp, P->est,
                       P->pstat, P->hdr, P->st, ns, N, P->abort, P->auth,
                       P->meta, b->status, b->out_len, P->bcount2,
                       (unsigned long long *)P->new_index2);
    // the window again, from the stored one, for the authenticated packets
    hipLaunchKernelGGL(k_pp_window, gs, blk, 0, stream, P->st, ns,
                       P->new_index2, P->win, P->wnew);
    hipLaunchKernelGGL(k_pu_setbits, gp, blk, 0, stream, ks, kp, P->est,
                       P->st, ns, N, P->abort, P->auth, P->new_index2,
                       P->wnew);
    hipLaunchKernelGGL(k_pu_commit_stream, gs, blk, 0, stream, P->st, ns,
                       P->new_index2, P->bcount, P->bcount2, P->wnew, P->win,
                       P->abort, P->h_abort_dev);
    if (b->mki_rx)
        hipLaunchKernelGGL(k_mki_rx_charge, gp, blk, 0, stream, b->in,
                           b->in_off, b->in_len, P->st, P->hkey, P->hval,
                           P->hcap - 1, N, P->rxj, P->kuses, b->status,
                           P->abort, (const uint32_t *)nullptr);
    PPCHK(hipGetLastError());
    if (pp_step(stream, "pu_commit"))
        return -1;
    // rejected packets (all of them after a post-crypto abort): their
    // speculative decryption is undone
    if (srtp_gpu_undo(g, n, b->out, b->out_off, P->meta, stream))
        return -1;
    // the commit kernel published the final abort word to host memory
    PPCHK(hipStreamSynchronize(stream));
    if (*(volatile uint32_t *)P->h_abort == ABORT_UNSET)
        PPCHK(hipMemcpy(P->h_abort, P->abort, 4, hipMemcpyDeviceToHost));
    if (unordered && *P->h_abort == AB_ORDER) {
        unordered = false;   // nothing ran or changed: the chain form
        b->bucketed = 0;
        continue;
    }
    b->sorted = !unordered;
    *fallback = (int)*P->h_abort;
    return 0;
    }
}

}   // extern "C"
