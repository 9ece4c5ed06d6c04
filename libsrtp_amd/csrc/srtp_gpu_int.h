// srtp_gpu_int.h -- plumbing between the HIP translation units of
// libsrtp_mi355x (not part of the C ABI).
//
//   srtp_gpu.hip        the thin extern "C" FFI of srtp_dev.h, small kernels
//                       (undo, SRTCP, header parse), kernel dispatch
//   srtp_icm.hip        k_icm_hmac, the general one-lane-per-packet AES-ICM +
//                       HMAC-SHA1 kernel; compiled once per AES round count
//   srtp_gcm.hip        k_gcm (AES-GCM), one lane per packet, any batch;
//                       compiled once per round count
//   srtp_prepass.hip    the device pre-pass of srtp_protect_device
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "srtp_dev.h"

struct srtp_gpu {
    hipStream_t stream;
    srtp_dev_key_t *d_keys;
    uint32_t key_cap;
    uint32_t *d_ghash;
    uint32_t ghash_cap;
    hipEvent_t ev0, ev1;
    int timing;
    int ms_pending;   // ev0 / ev1 recorded, last_ms not read yet
    float last_ms;
    void *pp;         // device pre-pass state (srtp_prepass.hip)
    int ncu;          // compute units (persistent grids)
    // single-buffer cipher / auth calls of the crypto-kernel API
    // (srtp_plugin.c -> srtp_gpu_raw): scratch grown on demand
    uint8_t *d_raw;
    size_t raw_cap;
    // srtp_gpu_undo: the compacted list of packets to undo (+ its count)
    uint32_t *d_undo;
    size_t undo_cap;
    hipEvent_t marks[SRTP_GPU_MARKS];   // srtp_gpu_mark / _mark_wait
    hipStream_t aux[2];                 // srtp_gpu_aux_stream: copy streams
    // srtp_gpu_one (srtp_one.hip): the pinned, mapped staging buffer of the
    // per-call path, host and device addresses
    uint8_t *one_h, *one_d;
};

// The order-free protect pre-pass's classification done by k_icm_hmac
// itself (srtp_prepass.hip pp_protect_fused): per packet the header parse,
// stream lookup, checks and index guess of k_pp_classify (status, stream id,
// index out; the descriptor it encrypts with stays in registers), and the
// per-stream count / highest index; the bytes past the packet that its tag
// overwrites are saved first (an in-place batch the pre-pass then declines
// is restored from them).
// one packet's classification, one 16-byte store (dense: a wave writes
// whole cache lines)
struct alignas(16) FzRec {
    uint64_t est;          // the index guessed from the stored one (48 bits)
                           // | status code << 48
    uint32_t skey;         // stream id, ~0 when the packet is not a chain one
    uint32_t cap;          // the caller's capacity (out_len before the kernel
                           // wrote the protected length), for a decline
};

struct IcmFused {
    const uint32_t *in_len;
    uint32_t *cap;         // capacities in, protected lengths out
    int32_t *status;
    const srtp_dev_stream_t *st;
    const uint32_t *hkey, *hval;
    uint32_t hmask;
    FzRec *rec;
    uint32_t (*tsave)[4];  // the trailer bytes [len, len + trailer) (<= 16)
    // per stream: packets touched (low 32 bits) and chain packets (high),
    // highest and lowest chain index, and a bitmap of the chain indices mod
    // M = the window size rounded up to a power of two (M / 32 words at
    // word 2 * win_off; zero between batches)
    unsigned long long *cnt;
    unsigned long long *new_index, *emin;
    uint32_t *bmap;
    uint32_t *abort;
    // unprotect (pp_unprotect_fused): highest candidate index per stream,
    // the authenticated indices' bitmaps (same layout as bmap), the count of
    // candidates that failed their tag check
    unsigned long long *hicand;
    uint32_t *bmap2;
    uint32_t *nfail;
    // k_icm_stg: the largest trailer a protected packet of the batch gets,
    // and the wave groups (64 consecutive packets) it leaves to the
    // per-lane form, per wave w of the grid: glist[0] != 0 when any,
    // glist[1 + w] = wave w's count, its group ids from
    // glist[1 + FZ_GL_WAVES + w * cap], cap = ceil(groups / waves)
    uint32_t max_trailer;
    uint32_t *glist;
};
constexpr uint32_t FZ_GL_WAVES = 4096;   // waves of a persistent grid, max

// One stream's in-order protect batch, classified inside the uniform-key
// AES-ICM kernel (srtp_prepass.hip pp_protect_inorder): packet i has
// sequence number seq_0 + i and index e_0 + i, e_0 the stored index's
// guess for packet 0 -- what the reference's walk gives a sender's
// consecutive packets (rdbx.c:112-145: every advance is 1).  A packet
// outside that (or with a length / parse error) is not encrypted and sets
// *abort; the pre-pass then restores the batch and runs the chain form.
// Out of place or asynchronous, k_io_check has checked every packet before
// the kernel runs (nothing to restore): tsave is null then.
struct IcmChain {
    const uint32_t *in_len;
    const uint32_t *cap;
    const srtp_dev_stream_t *st;   // the batch's one stream
    uint32_t *abort;
    uint32_t (*tsave)[4];          // the trailer bytes the tag overwrites
};

// AES-ICM (+ HMAC-SHA1) kernel arguments
struct IcmArgs {
    const uint8_t *in;
    const uint64_t *in_off;
    uint8_t *out;
    const uint64_t *out_off;
    const srtp_dev_meta_t *meta;
    const srtp_dev_key_t *keys;
    uint8_t *auth_ok;
    const uint32_t *abort;   // device pre-pass fell back: do nothing
    uint32_t n;
    uint32_t uni;            // uniform key slot, ~0 if keys differ
    // key buckets (srtp_gpu_batch_t rec / rec_idx / rec_range), or null:
    // this launch walks rec[range[0] .. range[1])
    const srtp_dev_rec_t *rec;
    const uint32_t *rec_idx;
    const uint32_t *range;
    // order-free protect classified in the kernel (per-lane keys only):
    // fz valid when fused, meta then written, not read
    bool fused;
    IcmFused fz;
    // fused batches through the LDS-staged kernel (k_icm_stg; default on,
    // SRTP_ICM_STG=0 selects the per-lane form for A/B runs)
    bool stg;
    // one stream's in-order batch (ch.st != null), classified here
    IcmChain ch;
};

// AES-GCM kernel arguments
struct GcmArgs {
    const uint8_t *in;
    const uint64_t *in_off;
    uint8_t *out;
    const uint64_t *out_off;
    const srtp_dev_meta_t *meta;
    const srtp_dev_key_t *keys;
    const uint32_t *ghash;   // 1024 words per GCM key
    uint8_t *auth_ok;
    const uint32_t *abort;   // device pre-pass fell back: do nothing
    uint32_t n;
    uint32_t uni;
    // key buckets (srtp_gpu_batch_t rec / rec_idx / rec_range), or null: the
    // bucketed launch walks rec[range[0] .. range[1]) one key per wave, the
    // per-lane one rec[range[0] .. range[1]) of its own range pointer
    const srtp_dev_rec_t *rec;
    const uint32_t *rec_idx;
    const uint32_t *range;
    // order-free form classified in the kernel (per-lane keys; in place):
    // fz valid when fused, meta then neither read nor written
    bool fused;
    IcmFused fz;
    // one stream's in-order batch (ch.st != null), classified here
    IcmChain ch;
};

// records a HIP error in the FFI's error string, returns -1
int srtp_gpu_fail(hipError_t e, const char *what);

#define HIPCHK(x)                                                              \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess)                                                  \
            return srtp_gpu_fail(e_, #x);                                      \
    } while (0)

// where a k_icm_hmac launch takes each packet's key from
enum IcmKeyMode {
    KM_UNI = 0,    // one key for the whole batch (A.uni): SGPR schedule
    KM_LANE = 1,   // per lane (meta.key): VGPR schedule
    KM_WAVE = 2    // per aligned 64-record group of a key bucket: SGPR
                   // schedule, reloaded for every group
};

// k_icm_hmac launchers (srtp_icm.hip, one object per NR in {0,10,12,14}
// and key mode)
template <int NR, int KM>
int launch_icm_km(const IcmArgs &A, bool auth, bool prot, int ncu,
                  hipStream_t st);

// k_gcm launchers (srtp_gcm.hip, one object per NR in {10,14})
template <int NR>
int launch_gcm_nr(const GcmArgs &A, bool prot, int ncu, hipStream_t st);
