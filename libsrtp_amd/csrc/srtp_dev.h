/*
 * srtp_dev.h -- layouts shared by the host protocol engine (C) and the HIP
 * kernels, plus the thin extern "C" FFI the C host calls.
 *
 * Data layout in HBM (see DESIGN.md "Data layout"):
 *   key table   : srtp_dev_key_t[nkeys]  one 512-byte slot per session key
 *                 (round keys, salt, HMAC midstates, MKI, GHASH table index)
 *   ghash table : 4 KiB per GCM key: M[b] = b(x)*H for every byte b
 *   packet arena: caller bytes; packet i at in_off[i] (16-byte aligned,
 *                 readable up to in_off + roundup16(len))
 *   meta        : srtp_dev_meta_t[n] written by the pre-pass
 */
#ifndef SRTP_DEV_H
#define SRTP_DEV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* cipher families as the kernels see them */
enum {
    SRTP_DEV_NULL = 0,
    SRTP_DEV_ICM = 1,
    SRTP_DEV_GCM = 2
};

/* srtp_dev_key_t.xflags: RFC 6904 header-extension encryption (the ICM key
 * in slot xslot, IDs in xids) and RFC 9335 cryptex (srtp.c:135-305) */
enum { SRTP_XF_XTN = 1, SRTP_XF_CRYPTEX = 2,
       SRTP_XF_CONF = 4 /* the stream's RTP services include confidentiality */ };

/* The words a packet reads come first: with an AES-128 schedule the whole
 * per-packet part of a record is its first 256 bytes (two 128-byte cache
 * lines), which per-lane-key batches gather once per packet. */
typedef struct srtp_dev_key {
    uint32_t salt[4];   /* ICM: 14-byte salt || 00 00; GCM: 12-byte salt   */
    uint32_t ipad[5];   /* SHA-1 state after (K ^ ipad)                      */
    uint32_t opad[5];   /* SHA-1 state after (K ^ opad)                      */
    uint32_t tag_len;   /* bytes of tag on the wire                          */
    uint32_t mki_size;  /* bytes of MKI on the wire (0 if not used)          */
    uint32_t conf;      /* 1 = payload encrypted (sec_serv_conf)             */
    uint32_t ghash_slot;/* index into the GHASH table arena (GCM only)       */
    uint32_t rounds;    /* 10 / 12 / 14, 0 for the null cipher              */
    uint32_t family;    /* SRTP_DEV_*                                        */
    uint32_t rk[60];    /* AES round keys, little-endian words of the bytes
                           (byte offset 80: 16-byte aligned)                 */
    uint32_t auth;      /* 1 = HMAC-SHA1 computed, 0 = none                  */
    uint32_t xslot;     /* slot of the header-extension ICM key (SRTP_XF_XTN) */
    uint32_t h[4];      /* GCM hash subkey E_K(0^128), big-endian words      */
    uint8_t mki[128];
    uint32_t xids[8];   /* bitmap of the extension IDs to encrypt (0..255)  */
    uint32_t xflags;    /* SRTP_XF_*                                         */
    uint32_t pad1;
} srtp_dev_key_t;
#ifdef __cplusplus
static_assert(sizeof(srtp_dev_key_t) == 512, "one 512-byte key slot");
static_assert(offsetof(srtp_dev_key_t, rk) == 80, "rk 16-byte aligned");
#else
_Static_assert(sizeof(srtp_dev_key_t) == 512, "one 512-byte key slot");
_Static_assert(offsetof(srtp_dev_key_t, rk) == 80, "rk 16-byte aligned");
#endif

/* per-packet work descriptor written by the pre-pass */
typedef struct srtp_dev_meta {
    uint32_t key;   /* key slot                                              */
    uint32_t roc;   /* rollover counter of the estimated index               */
    uint32_t info;  /* [15:0] enc_start, [23:16] status (0 = run crypto),
                       [31:24] kernel variant (SRTP_VARIANT)                 */
    uint32_t len;   /* bytes authenticated / encrypted region end            */
} srtp_dev_meta_t;

/* one packet of a key-bucketed crypto pass (device pre-pass, batches with
 * many keys): its descriptor and offsets, stored at its bucket position so
 * the crypto kernel reads them contiguously */
typedef struct srtp_dev_rec {
    uint64_t in_off, out_off;
    srtp_dev_meta_t meta;
} srtp_dev_rec_t;

#define SRTP_META_ENC_START(i) ((i) & 0xffffu)
#define SRTP_META_STATUS(i) (((i) >> 16) & 0xffu)
#define SRTP_META_VARIANT(i) (((i) >> 24) & 0xffu)
/* kernel variant id: family*8 + rounds_code*2 + auth, rounds_code 0 null,
 * 1 AES-128, 2 AES-192, 3 AES-256 */
#define SRTP_VARIANT(fam, rc, au) ((uint32_t)((fam) * 8 + (rc) * 2 + (au)))
/* streams with header-extension encryption or cryptex: every packet goes to
 * the byte-wise k_xrtp (any family / key size); meta.info bit 0 is then the
 * caller's in-place flag (rtp == srtp in srtp_protect's terms) and bit 1
 * (undo only) says the run being undone applied cryptex */
#define SRTP_VARIANT_X 24u
/* session keys whose cipher or auth type an application replaced
 * (srtp_replace_cipher_type / srtp_replace_auth_type): no kernel takes
 * them; the host runs their crypto through the registered vtables */
#define SRTP_VARIANT_V 25u
#define SRTP_XI_INPLACE 1u
#define SRTP_XI_CRYPTEX 2u
/* k_xrtp result byte (auth_ok[i]): bit 0 authenticated (unprotect) / done,
 * bit 1 output written, bit 2 cryptex applied, bit 3 parse error of the
 * header extension (srtp_process_header_encryption / srtp_cryptex_protect) */
enum { SRTP_XR_OK = 1, SRTP_XR_WROTE = 2, SRTP_XR_CRYPTEX = 4,
       SRTP_XR_PARSE = 8 };

/* compact header summary produced by the device parse kernel */
typedef struct srtp_dev_hdr {
    uint32_t ssrc;      /* big-endian numeric value                          */
    uint32_t seq_len;   /* [15:0] seq, [31:16] reserved                      */
    uint32_t enc_start; /* header length incl. extension, or error code<<24 */
    uint32_t len;       /* packet length                                     */
} srtp_dev_hdr_t;

/* session-key derivation job for k_kdf (srtp_gpu_kdf): the SRTP KDF
 * (srtp.c:1070-1142: AES-ICM PRF keyed by the master key, offset = master
 * salt, label in byte 7) for one session key, then the device key record
 * (AES schedule, salt, HMAC midstates, GCM H and GHASH table).  The host
 * fills every field of `key` but rk / salt / ipad / opad / h. */
enum {
    SRTP_KDF_HMAC = 1,      /* ipad / opad from the auth key               */
    SRTP_KDF_GCM_H = 2,     /* h = E_K(0^128)                              */
    SRTP_KDF_GHASH = 4,     /* Shoup table of h into ghash slot            */
    SRTP_KDF_SALT_TAIL = 8  /* salt bytes salt_len.. from salt_tail        */
};

typedef struct srtp_kdf_job {
    srtp_dev_key_t key;
    uint8_t kdf_key[32];    /* the PRF's AES key                            */
    uint8_t kdf_salt[16];   /* its 14-byte offset                           */
    uint8_t salt_tail[2];
    uint8_t lab_enc, lab_salt, lab_auth, pad[3];
    uint32_t kdf_len;       /* 16 / 24 / 32                                 */
    uint32_t enc_len;       /* 0 (no AES key) / 16 / 24 / 32                */
    uint32_t salt_len;      /* bytes of PRF salt output: 0 / 12 / 14        */
    uint32_t auth_len;      /* bytes of PRF auth-key output (0..20)         */
    uint32_t flags;         /* SRTP_KDF_*                                   */
    uint32_t slot;          /* destination key slot                         */
} srtp_kdf_job_t;

/* ---- thin FFI implemented in HIP (srtp_gpu.hip) ----------------------- */

typedef struct srtp_gpu srtp_gpu_t;

int srtp_gpu_open(srtp_gpu_t **g);
void srtp_gpu_close(srtp_gpu_t *g);
int srtp_gpu_available(void);
const char *srtp_gpu_last_error(void);

/* key table (device copy of srtp_dev_key_t, grown on demand) */
int srtp_gpu_set_key(srtp_gpu_t *g, uint32_t slot, const srtp_dev_key_t *k,
                     const uint32_t *ghash_tab /* 1024 words or NULL */);

/* the key table as a whole (session replication, srtp_mi355x_session_*):
 * get copies slots [0, n) to dst; put writes slots [0, n) from src and
 * builds the GHASH table of every slot i with ghash_flag[i] != 0 from its
 * record's H (k_ghash_build).  Synchronous. */
int srtp_gpu_get_keys(srtp_gpu_t *g, uint32_t n, srtp_dev_key_t *dst);
int srtp_gpu_put_keys(srtp_gpu_t *g, uint32_t n, const srtp_dev_key_t *src,
                      const uint8_t *ghash_flag);

/* derive n session keys on the GPU (k_kdf) straight into the key table;
 * synchronous */
int srtp_gpu_kdf(srtp_gpu_t *g, const srtp_kdf_job_t *jobs, size_t n);

/* One pass over a batch in device memory.  Packets whose meta status is
 * non-zero are skipped.  For unprotect, auth_ok[i] receives 1 when the tag
 * verified.  op: 0 protect, 1 unprotect.  Asynchronous on the g's stream
 * unless `stream` is non-NULL (a hipStream_t). */
typedef struct srtp_gpu_batch {
    size_t n;
    const uint8_t *in;      /* device arena */
    const uint64_t *in_off; /* device */
    uint8_t *out;           /* device arena (may equal in) */
    const uint64_t *out_off;/* device */
    const srtp_dev_meta_t *meta; /* device */
    uint8_t *auth_ok;       /* device, unprotect only */
    uint32_t uniform_key;   /* slot when every packet uses one key, else ~0 */
    uint32_t mask;          /* bitmask of kernel variants present (hint)   */
    void *stream;           /* hipStream_t or NULL for the context stream */
    const uint32_t *abort;  /* device word; non-zero -> kernels do nothing
                               (device pre-pass fell back), or NULL     */
    /* key buckets (or NULL): the AES-ICM kernels walk rec[] instead of the
     * packet order.  rec_range (device) = {0, a, a, a + b}: [0, a) holds
     * one stream per aligned group of 64 records (one key per wave),
     * [a, a + b) the streams with few packets (keys differ per lane);
     * records with a nonzero status are gaps.  rec_idx[pos] = the packet
     * index of rec[pos] (unprotect's auth_ok[]). */
    const srtp_dev_rec_t *rec;
    const uint32_t *rec_idx;
    const uint32_t *rec_range;
    /* or NULL: the order-free protect pre-pass classifies inside the AES-ICM
     * kernel (IcmFused, srtp_gpu_int.h; srtp_prepass.hip pp_protect_fused):
     * meta is written there, not read */
    const void *fused;
    /* or NULL: one stream's in-order batch, the index of every packet
     * computed inside the AES-ICM kernel (IcmChain, srtp_gpu_int.h;
     * srtp_prepass.hip pp_protect_inorder): meta is neither read nor
     * written */
    const void *inorder;
} srtp_gpu_batch_t;

int srtp_gpu_run(srtp_gpu_t *g, int op, const srtp_gpu_batch_t *b);

/* The per-call path (srtp_one.hip k_one): ONE packet by one workgroup,
 * straight from / to a pinned staging buffer.  srtp_gpu_one_buf returns the
 * buffer's host address (SRTP_ONE_MAX bytes; NULL on allocation failure);
 * the caller copies the packet there, srtp_gpu_one runs `op` (0 protect, 1
 * unprotect: verify, then decrypt only an authentic packet) with the host
 * pre-pass's descriptor and waits for the kernel's done flag; the result is
 * in the buffer (protect: packet + MKI + tag; unprotect, *ok: plaintext).
 * Packets up to SRTP_ONE_MAX bytes, trailer included. */
#define SRTP_ONE_MAX 4096u
#define SRTP_ONE_FLAG SRTP_ONE_MAX   /* offset of the verdict / done word */
#define SRTP_ONE_TRAILER 160u        /* room for tag + MKI past the packet */
uint8_t *srtp_gpu_one_buf(srtp_gpu_t *g);
int srtp_gpu_one(srtp_gpu_t *g, int op, uint32_t len, const srtp_dev_meta_t *m,
                 void *stream, int *ok);

/* re-apply the keystream of the given (speculative) meta to the packets at
 * arena+off: undoes an in-place speculative decryption before a re-run */
int srtp_gpu_undo(srtp_gpu_t *g, size_t n, uint8_t *arena,
                  const uint64_t *off, const srtp_dev_meta_t *meta,
                  void *stream);

/* SRTCP (k_rtcp), packets in place at arena+off.  meta: key = RTCP key
 * slot, roc = 31-bit SRTCP index, info bit 0 = E bit (confidentiality),
 * [23:16] status, len = protect: RTCP length / unprotect: authenticated
 * length (RTCP + trailer).  op 0: write trailer, encrypt, MKI, tag;
 * op 1: verify the tag (auth_ok[i]), then decrypt a verified packet. */
int srtp_gpu_rtcp(srtp_gpu_t *g, int op, size_t n, uint8_t *arena,
                  const uint64_t *off, const srtp_dev_meta_t *meta,
                  uint8_t *auth_ok, void *stream);

/* device header parse for the device-resident API; xinfo_out[i] (may be
 * NULL): [15:0] extension profile, [19:16] CC, bit 20 X (cryptex checks) */
int srtp_gpu_parse(srtp_gpu_t *g, size_t n, const uint8_t *in,
                   const uint64_t *in_off, const uint32_t *in_len,
                   srtp_dev_hdr_t *hdr_out, uint32_t *xinfo_out, void *stream);

/* ---- device pre-pass (DESIGN.md "Device pre-pass") --------------------
 * A device mirror of the session's streams lets srtp_protect_device and
 * srtp_unprotect_device run the in-order index / replay / key-usage
 * pre-pass on the GPU.  The host stays authoritative: it uploads the table,
 * the GPU advances it, and the host pulls it back before any host-side use
 * of stream state. */
enum {
    SRTP_DS_ELIGIBLE = 1,    /* protect: sender/unknown direction (MKI: the
                                devtab's key index) */
    SRTP_DS_ICM_CONF = 2,    /* AES-ICM encrypting: 2^16 keystream blocks */
    SRTP_DS_RX_ELIGIBLE = 4, /* unprotect: receiver/unknown direction (MKI:
                                packets carrying another key's MKI abort to
                                the host) */
    SRTP_DS_AEAD = 8,        /* AES-GCM: key usage counted before the tag
                                check (srtp.c:2390-2406) */
    SRTP_DS_PENDING = 16     /* a ROC set by srtp_stream_set_roc is pending
                                (its value in srtp_dev_stream_t.rsv): the host
                                resolves it per batch (srtp_gpu_pp_pend_*) */
};
/* srtp_dev_stream_t.dir: directions the device batches used the stream in */
enum { SRTP_DIR_TX = 1, SRTP_DIR_RX = 2 };

typedef struct srtp_dev_stream {
    uint32_t ssrc;
    uint32_t key;       /* key slot of the stream's (only) session key      */
    uint32_t variant;   /* SRTP_VARIANT of that key                          */
    uint32_t flags;     /* SRTP_DS_*                                         */
    uint32_t trailer;   /* tag + MKI bytes appended by protect               */
    uint32_t win_bits;  /* replay window bits (multiple of 32)               */
    uint32_t win_off;   /* word offset of the window in the window arena     */
    uint32_t dir;       /* SRTP_DIR_* bits set by device batches             */
    uint32_t mki;       /* MKI streams: MKI bytes | their distance from the
                           packet end << 16 (tag + MKI; AES-GCM: MKI only,
                           srtp.c:1961-2016); 0 without MKI.  `key` is the
                           slot of the key device batches use (the host's
                           devtab mki_j-th master key)                     */
    uint32_t rsv;       /* SRTP_DS_PENDING: the pending ROC                   */
    uint32_t kbase;     /* MKI streams: the slots of master keys 0..nkeys-1
                           are mkslot[kbase ..] (srtp_gpu_pp_upload); protect
                           batches pick one per packet (srtp_gpu_pp_batch_t
                           mki)                                              */
    uint32_t nkeys;     /* MKI streams: number of master keys; 0 without MKI */
    uint64_t index;     /* rdbx index (ROC << 16 | SEQ)                      */
    uint64_t uses;      /* packets charged to the key since the upload       */
} srtp_dev_stream_t;

/* the table: streams[ns], window arena (nwords), SSRC hash (hcap a power of
 * two, open addressing with the host's hash, hval ~0 = empty slot).
 * Template sessions (ssrc_any_*; srtp_stream_clone, srtp.c:762-863, called
 * from srtp.c:2540 protect and 3141 unprotect): `tmpl` is the template's
 * record (ssrc unused; win_off the first of `spare` windows of
 * tmpl->win_bits bits at the end of the arena, which `nwords` includes),
 * and up to `spare` streams may be created on the device (srtp_gpu_pp_clone)
 * as records ns, ns + 1, ...; tmpl NULL: none. */
int srtp_gpu_pp_upload(srtp_gpu_t *g, const srtp_dev_stream_t *streams,
                       uint32_t ns, const uint32_t *win, uint32_t nwords,
                       const uint32_t *hkey, const uint32_t *hval,
                       uint32_t hcap, const srtp_dev_stream_t *tmpl,
                       uint32_t spare, const uint32_t *mkslot, uint32_t nmk);
/* the table back: *ns_now records (the uploaded ones, then the streams
 * created on the device in creation order), the whole window arena and
 * (kuses, nmk entries; may be NULL) the protect packets charged to each
 * master key of the MKI streams, mkslot's order */
int srtp_gpu_pp_download(srtp_gpu_t *g, srtp_dev_stream_t *streams,
                         uint32_t *win, uint32_t *ns_now, uint64_t *kuses);

typedef struct srtp_gpu_pp_batch {
    size_t n;
    const uint8_t *in;
    const uint64_t *in_off;
    const uint32_t *in_len;
    uint8_t *out;
    const uint64_t *out_off;
    uint32_t *out_len;      /* in: capacity, out: protected length */
    int32_t *status;
    void *stream;
    uint32_t uniform_key;   /* as srtp_gpu_batch_t */
    uint32_t mask;
    int sorted;             /* out: the sorted chain path ran (not the
                               order-free form) */
    int async;              /* protect: return once the pre-pass verdict is
                               published, the crypto kernel still queued */
    int fused_ok;           /* protect: in place, one AES-ICM kernel variant,
                               trailers <= 16 bytes: the order-free form may
                               classify inside the crypto kernel */
    uint32_t max_trailer;   /* protect: the largest tag + MKI of the streams
                               the device may encrypt */
    int inorder_ok;         /* one uniform-key AES-ICM / GCM variant,
                               trailers <= 16 bytes: a one-stream batch may
                               try the in-order form (indices computed in the
                               crypto kernel; protect out of place or async:
                               checked first by k_io_check) */
    int mki_rx;             /* unprotect: the table has MKI streams -- each
                               packet's MKI selects its master key on the
                               device (srtp.c:1961-2016), charged per key;
                               no key buckets */
    int inorder;            /* out: 1 the in-order form committed the batch,
                               2 it declined it (the chain form ran), 0 not
                               tried */
    int bucketed;           /* out: the crypto ran from key buckets */
    const uint8_t *mki;     /* protect, HOST array: each packet's master key
                               index for the MKI streams (srtp.c:2536-2545;
                               below every MKI stream's key count: the host
                               checks), NULL without MKI streams.  The
                               packets of an MKI stream run on key
                               mkslot[kbase + mki[i]] and are charged to it */
} srtp_gpu_pp_batch_t;

/* pre-pass + crypto for protect.  *fallback != 0: nothing was written (no
 * packet, status or stream state) and the batch must take the host path;
 * the value is the abort reason: 1 unknown SSRC, 2 ineligible stream,
 * 4 sequence outside the chain domain (bits may combine). */
int srtp_gpu_pp_protect(srtp_gpu_t *g, srtp_gpu_pp_batch_t *b,
                        int *fallback);

/* Template clones: every packet of the batch whose SSRC has no stream gets
 * one -- a record copied from the template (fresh index and window, no
 * direction yet; the pre-pass that then runs sets SRTP_DIR_TX on protect
 * and SRTP_DIR_RX on unprotect only when a packet of it authenticates,
 * srtp.c:3117-3155) and an entry in the SSRC hash.  *added: streams created
 * by this call.  Returns 1 when the spare records ran out (the batch must
 * take the host path; the host rebuilds the table). */
int srtp_gpu_pp_clone(srtp_gpu_t *g, const srtp_gpu_pp_batch_t *b,
                      uint32_t *added);

/* Pending ROCs (srtp_stream_set_roc, srtp.c:5137-5167): while a stream's
 * ROC is pending, a packet's index is pending_roc || seq (srtp.c:2038-2081),
 * and the first packet more than 2^15 past the stored index sets the index
 * and window to it and clears the pending ROC (2674-2678 protect,
 * 3161-3167 unprotect, after the tag).  Per batch, for the pending streams
 * `sids` (device stream ids), srtp_gpu_pp_pend_scan finds in batch order
 * the first packet that reaches the index estimate (protect: header, length
 * and capacity checks passed) and the lowest / highest pending_roc || seq
 * of the stream's packets.  The host decides; for a stream whose first
 * packet advances, srtp_gpu_pp_pend_apply gives the device the state from
 * which the normal order-free / chain forms reproduce the reference: index
 * = that packet's index - 1, an empty window, no pending ROC (the packet
 * then advances by one and sets its bit, as srtp_rdbx_set_roc_seq +
 * srtp_rdbx_add_index(0) do).  srtp_gpu_pp_pend_restore takes the applied
 * records back (a declined batch); srtp_gpu_pp_pend_clear forgets them (a
 * committed batch).  On unprotect every applied stream's first packet must
 * authenticate (else the reference would keep the ROC pending): the
 * pre-pass aborts the batch to the host when one does not. */
typedef struct srtp_pend_info {
    uint32_t first;     /* batch position of the first packet, ~0 if none   */
    uint32_t rsv;
    uint64_t efirst;    /* its pending_roc || seq                            */
    uint64_t emin, emax;/* over the stream's packets                         */
    uint64_t index;     /* the device's stored index of the stream           */
} srtp_pend_info_t;
int srtp_gpu_pp_pend_scan(srtp_gpu_t *g, const srtp_gpu_pp_batch_t *b,
                          int unprotect, const uint32_t *sids, uint32_t np,
                          srtp_pend_info_t *out);
int srtp_gpu_pp_pend_apply(srtp_gpu_t *g, const uint32_t *sids,
                           const uint64_t *efirst, const uint32_t *first,
                           uint32_t nr, void *stream);
int srtp_gpu_pp_pend_restore(srtp_gpu_t *g, void *stream);
void srtp_gpu_pp_pend_clear(srtp_gpu_t *g);

/* pre-pass + crypto + commit for unprotect (the order-free form only: per
 * stream every index above the stored one and within one replay window of
 * the batch's highest, no duplicate, no MKI, no packet with a length /
 * capacity error).  Packets failing authentication get auth_fail, leave the
 * stream state alone and have their decryption undone.  *fallback != 0:
 * nothing was written and the host path must run the batch (bits: 1
 * unknown SSRC, 2 ineligible stream, 8 order / replay domain, 16 a packet
 * with a static error). */
int srtp_gpu_pp_unprotect(srtp_gpu_t *g, srtp_gpu_pp_batch_t *b,
                          int *fallback);

/* ---- single-buffer operations of the crypto-kernel API ---------------
 * (cipher.h / auth.h vtables of the reference, srtp_plugin.c): one GPU
 * launch per call, host buffers in and out (copied through device scratch).
 *   SRTP_RAW_ICM:  dst = src ^ (lead[0..nlead) || AES(ctr + j), j = 0..)
 *                  with ICM's 16-bit block counter in ctr bytes 14..15;
 *                  ks_last = the keystream of the last block generated
 *   SRTP_RAW_GCM_SEAL / _OPEN: AES-GCM with iv (12 B), aad; seal writes
 *                  ciphertext || tag (tag_len) to dst, open verifies the tag
 *                  after src[0, len) (ok = 1 / 0) and writes the plaintext
 *   SRTP_RAW_HMAC: dst[0..20) = HMAC-SHA1 from the key's ipad/opad
 *                  midstates over src[0, len) */
enum { SRTP_RAW_ICM = 0, SRTP_RAW_GCM_SEAL = 1, SRTP_RAW_GCM_OPEN = 2,
       SRTP_RAW_HMAC = 3 };
typedef struct srtp_gpu_raw {
    int op;
    const srtp_dev_key_t *key;   /* host: rk / rounds / h / ipad / opad */
    const uint8_t *src;
    uint8_t *dst;
    size_t len;
    uint8_t ctr[16];
    uint8_t lead[16];
    uint32_t nlead;
    uint8_t ks_last[16];         /* out */
    uint8_t iv[12];
    const uint8_t *aad;
    size_t aad_len;
    uint32_t tag_len;
    int ok;                      /* out (GCM open) */
} srtp_gpu_raw_t;
int srtp_gpu_raw(srtp_gpu_t *g, srtp_gpu_raw_t *r);

/* plumbing between the two HIP translation units */
void **srtp_gpu_pp_slot(srtp_gpu_t *g);
void *srtp_gpu_stream_of(srtp_gpu_t *g);
void srtp_gpu_pp_free(void *pp);

/* memory helpers */
void *srtp_gpu_malloc(size_t bytes);
void srtp_gpu_free(void *p);
void *srtp_gpu_host_alloc(size_t bytes); /* pinned */
void srtp_gpu_host_free(void *p);
int srtp_gpu_h2d(srtp_gpu_t *g, void *dst, const void *src, size_t n,
                 void *stream);
int srtp_gpu_d2h(srtp_gpu_t *g, void *dst, const void *src, size_t n,
                 void *stream);
int srtp_gpu_sync(srtp_gpu_t *g, void *stream);
/* n bytes at dst (device) set to v, stream-ordered */
int srtp_gpu_memset(void *dst, int v, size_t n, void *stream);
/* a marker on `stream` after the work queued so far (slot < SRTP_GPU_MARKS),
 * and a host wait for it */
#define SRTP_GPU_MARKS 16
int srtp_gpu_mark(srtp_gpu_t *g, int slot, void *stream);
int srtp_gpu_mark_wait(srtp_gpu_t *g, int slot);
/* `stream` waits for the marker (device side) */
int srtp_gpu_mark_stream_wait(srtp_gpu_t *g, void *stream, int slot);
/* copy streams of the host-batch pipeline (k = 0 in, 1 out), created on
 * first use; NULL on failure */
void *srtp_gpu_aux_stream(srtp_gpu_t *g, int k);

/* timing of the last srtp_gpu_run kernels (ms, from HIP events) */
double srtp_gpu_last_kernel_ms(srtp_gpu_t *g);
void srtp_gpu_set_timing(srtp_gpu_t *g, int on);

#ifdef __cplusplus
}
#endif
#endif
