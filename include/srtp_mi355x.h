/*
 * srtp_mi355x.h -- C ABI of libsrtp_mi355x, an MI355X (gfx950) SRTP engine.
 *
 * Drop-in surface: every declaration in the first half keeps the name,
 * signature, struct layout and enum values of cisco/libsrtp 3.0.0's public
 * header (include/srtp.h; symbol list srtp.def:1-69 incl. the crypto-kernel
 * plugin ABI of srtp.def:46-69, below), so C code written
 * against libsrtp compiles and links against this library unchanged.  Each
 * group cites the reference declaration it replaces.
 *
 * The second half adds the batch extension that the throughput path uses:
 * many packets per call, either from host buffers or already resident in
 * device memory (HBM).  Per-packet semantics -- status codes, replay and
 * index handling, key-usage limits, events, output layout -- are exactly
 * those of calling srtp_protect()/srtp_unprotect() once per packet in array
 * order.
 *
 * All packet cryptography (AES-ICM, HMAC-SHA1, AES-GCM) runs in HIP kernels
 * on the GPU; there is no CPU crypto fallback.  Calls fail with
 * srtp_err_status_init_fail when no GPU is present.
 */
#ifndef SRTP_MI355X_H
#define SRTP_MI355X_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- constants: include/srtp.h:62-116 ----------------------------------- */
#define SRTP_MASTER_KEY_LEN 30
#define SRTP_MAX_KEY_LEN 64
#define SRTP_MAX_TAG_LEN 16
#define SRTP_MAX_MKI_LEN 128
#define SRTP_MAX_TRAILER_LEN (SRTP_MAX_TAG_LEN + SRTP_MAX_MKI_LEN)
#define SRTP_SRCTP_INDEX_LEN 4
#define SRTP_MAX_SRTCP_TRAILER_LEN \
    (SRTP_SRCTP_INDEX_LEN + SRTP_MAX_TAG_LEN + SRTP_MAX_MKI_LEN)
#define SRTP_MAX_NUM_MASTER_KEYS 16
#define SRTP_SALT_LEN 14
#define SRTP_AEAD_SALT_LEN 12
#define SRTP_AES_128_KEY_LEN 16
#define SRTP_AES_192_KEY_LEN 24
#define SRTP_AES_256_KEY_LEN 32
#define SRTP_AES_ICM_128_KEY_LEN_WSALT (SRTP_SALT_LEN + SRTP_AES_128_KEY_LEN)
#define SRTP_AES_ICM_192_KEY_LEN_WSALT (SRTP_SALT_LEN + SRTP_AES_192_KEY_LEN)
#define SRTP_AES_ICM_256_KEY_LEN_WSALT (SRTP_SALT_LEN + SRTP_AES_256_KEY_LEN)
#define SRTP_AES_GCM_128_KEY_LEN_WSALT (SRTP_AEAD_SALT_LEN + SRTP_AES_128_KEY_LEN)
#define SRTP_AES_GCM_192_KEY_LEN_WSALT (SRTP_AEAD_SALT_LEN + SRTP_AES_192_KEY_LEN)
#define SRTP_AES_GCM_256_KEY_LEN_WSALT (SRTP_AEAD_SALT_LEN + SRTP_AES_256_KEY_LEN)

/* cipher / auth type ids: crypto/include/crypto_types.h:55-114 */
#define SRTP_NULL_CIPHER 0
#define SRTP_AES_ICM_128 1
#define SRTP_AES_ICM_192 4
#define SRTP_AES_ICM_256 5
#define SRTP_AES_GCM_128 6
#define SRTP_AES_GCM_256 7
#define SRTP_NULL_AUTH 0
#define SRTP_HMAC_SHA1 3

typedef uint32_t srtp_cipher_type_id_t;
typedef uint32_t srtp_auth_type_id_t;

/* ---- error codes: include/srtp.h:183-220 (values are ABI) --------------- */
typedef enum {
    srtp_err_status_ok = 0,
    srtp_err_status_fail = 1,
    srtp_err_status_bad_param = 2,
    srtp_err_status_alloc_fail = 3,
    srtp_err_status_dealloc_fail = 4,
    srtp_err_status_init_fail = 5,
    srtp_err_status_terminus = 6,
    srtp_err_status_auth_fail = 7,
    srtp_err_status_cipher_fail = 8,
    srtp_err_status_replay_fail = 9,
    srtp_err_status_replay_old = 10,
    srtp_err_status_algo_fail = 11,
    srtp_err_status_no_such_op = 12,
    srtp_err_status_no_ctx = 13,
    srtp_err_status_cant_check = 14,
    srtp_err_status_key_expired = 15,
    srtp_err_status_socket_err = 16,
    srtp_err_status_signal_err = 17,
    srtp_err_status_nonce_bad = 18,
    srtp_err_status_read_fail = 19,
    srtp_err_status_write_fail = 20,
    srtp_err_status_parse_err = 21,
    srtp_err_status_encode_err = 22,
    srtp_err_status_semaphore_err = 23,
    srtp_err_status_pfkey_err = 24,
    srtp_err_status_bad_mki = 25,
    srtp_err_status_pkt_idx_old = 26,
    srtp_err_status_pkt_idx_adv = 27,
    srtp_err_status_buffer_small = 28,
    srtp_err_status_cryptex_err = 29
} srtp_err_status_t;

/* ---- policy types: include/srtp.h:222-358 ------------------------------- */
typedef struct srtp_ctx_t_ srtp_ctx_t;
typedef srtp_ctx_t *srtp_t;

typedef enum {
    sec_serv_none = 0,
    sec_serv_conf = 1,
    sec_serv_auth = 2,
    sec_serv_conf_and_auth = 3
} srtp_sec_serv_t;

typedef struct srtp_crypto_policy_t {
    srtp_cipher_type_id_t cipher_type;
    size_t cipher_key_len;
    srtp_auth_type_id_t auth_type;
    size_t auth_key_len;
    size_t auth_tag_len;
    srtp_sec_serv_t sec_serv;
} srtp_crypto_policy_t;

typedef enum {
    ssrc_undefined = 0,
    ssrc_specific = 1,
    ssrc_any_inbound = 2,
    ssrc_any_outbound = 3
} srtp_ssrc_type_t;

typedef struct {
    srtp_ssrc_type_t type;
    uint32_t value;
} srtp_ssrc_t;

typedef struct srtp_master_key_t {
    uint8_t *key;
    uint8_t *mki_id;
} srtp_master_key_t;

typedef struct srtp_policy_t {
    srtp_ssrc_t ssrc;
    srtp_crypto_policy_t rtp;
    srtp_crypto_policy_t rtcp;
    uint8_t *key;
    srtp_master_key_t **keys;
    size_t num_master_keys;
    bool use_mki;
    size_t mki_size;
    size_t window_size;
    bool allow_repeat_tx;
    uint8_t *enc_xtn_hdr;
    size_t enc_xtn_hdr_count;
    bool use_cryptex;
    struct srtp_policy_t *next;
} srtp_policy_t;

/* SRTP profiles, include/srtp.h:1010-1040 */
typedef enum {
    srtp_profile_reserved = 0,
    srtp_profile_aes128_cm_sha1_80 = 1,
    srtp_profile_aes128_cm_sha1_32 = 2,
    srtp_profile_null_sha1_80 = 5,
    srtp_profile_null_sha1_32 = 6,
    srtp_profile_aead_aes_128_gcm = 7,
    srtp_profile_aead_aes_256_gcm = 8
} srtp_profile_t;

/* events, include/srtp.h:1290-1352 */
typedef enum {
    event_ssrc_collision,
    event_key_soft_limit,
    event_key_hard_limit,
    event_packet_index_limit
} srtp_event_t;

typedef struct srtp_stream_ctx_t_ srtp_stream_ctx_t;
typedef srtp_stream_ctx_t *srtp_stream_t;

typedef struct srtp_event_data_t {
    srtp_t session;
    uint32_t ssrc;
    srtp_event_t event;
} srtp_event_data_t;

typedef void(srtp_event_handler_func_t)(srtp_event_data_t *data);

typedef enum {
    srtp_log_level_error,
    srtp_log_level_warning,
    srtp_log_level_info,
    srtp_log_level_debug
} srtp_log_level_t;

typedef void(srtp_log_handler_func_t)(srtp_log_level_t level,
                                      const char *msg,
                                      void *data);

/* ---- lifecycle: include/srtp.h:380-387, 512-604, 1001 ------------------- */
srtp_err_status_t srtp_init(void);
srtp_err_status_t srtp_shutdown(void);
srtp_err_status_t srtp_create(srtp_t *session, const srtp_policy_t *policy);
srtp_err_status_t srtp_stream_add(srtp_t session, const srtp_policy_t *policy);
srtp_err_status_t srtp_stream_remove(srtp_t session, uint32_t ssrc);
srtp_err_status_t srtp_update(srtp_t session, const srtp_policy_t *policy);
srtp_err_status_t srtp_stream_update(srtp_t session,
                                     const srtp_policy_t *policy);
srtp_err_status_t srtp_dealloc(srtp_t s);
srtp_stream_ctx_t *srtp_get_stream(srtp_t srtp, uint32_t ssrc);

/* ---- per-packet hot path: include/srtp.h:433-438, 485-489 --------------- */
srtp_err_status_t srtp_protect(srtp_t ctx,
                               const uint8_t *rtp,
                               size_t rtp_len,
                               uint8_t *srtp,
                               size_t *srtp_len,
                               size_t mki_index);
srtp_err_status_t srtp_unprotect(srtp_t ctx,
                                 const uint8_t *srtp,
                                 size_t srtp_len,
                                 uint8_t *rtp,
                                 size_t *rtp_len);

/* ---- crypto policy setters: include/srtp.h:625-984 ---------------------- */
void srtp_crypto_policy_set_rtp_default(srtp_crypto_policy_t *p);
void srtp_crypto_policy_set_rtcp_default(srtp_crypto_policy_t *p);
/* include/srtp.h:661-662: an alias of the RTP default */
#define srtp_crypto_policy_set_aes_cm_128_hmac_sha1_80(p) \
    srtp_crypto_policy_set_rtp_default(p)
void srtp_crypto_policy_set_aes_cm_128_hmac_sha1_32(srtp_crypto_policy_t *p);
void srtp_crypto_policy_set_aes_cm_128_null_auth(srtp_crypto_policy_t *p);
void srtp_crypto_policy_set_null_cipher_hmac_sha1_80(srtp_crypto_policy_t *p);
void srtp_crypto_policy_set_null_cipher_hmac_null(srtp_crypto_policy_t *p);
void srtp_crypto_policy_set_aes_cm_256_hmac_sha1_80(srtp_crypto_policy_t *p);
void srtp_crypto_policy_set_aes_cm_256_hmac_sha1_32(srtp_crypto_policy_t *p);
void srtp_crypto_policy_set_aes_cm_256_null_auth(srtp_crypto_policy_t *p);
void srtp_crypto_policy_set_aes_cm_192_hmac_sha1_80(srtp_crypto_policy_t *p);
void srtp_crypto_policy_set_aes_cm_192_hmac_sha1_32(srtp_crypto_policy_t *p);
void srtp_crypto_policy_set_aes_cm_192_null_auth(srtp_crypto_policy_t *p);
void srtp_crypto_policy_set_aes_gcm_128_16_auth(srtp_crypto_policy_t *p);
void srtp_crypto_policy_set_aes_gcm_256_16_auth(srtp_crypto_policy_t *p);

/* ---- profiles / keys: include/srtp.h:1042-1100 -------------------------- */
srtp_err_status_t srtp_crypto_policy_set_from_profile_for_rtp(
    srtp_crypto_policy_t *policy, srtp_profile_t profile);
srtp_err_status_t srtp_crypto_policy_set_from_profile_for_rtcp(
    srtp_crypto_policy_t *policy, srtp_profile_t profile);
size_t srtp_profile_get_master_key_length(srtp_profile_t profile);
size_t srtp_profile_get_master_salt_length(srtp_profile_t profile);
void srtp_append_salt_to_key(uint8_t *key,
                             size_t bytes_in_key,
                             uint8_t *salt,
                             size_t bytes_in_salt);

/* ---- RTCP: include/srtp.h:1162-1216 (srtp/srtp.c:3894-4837).  AES-ICM
 *      128/192/256 or null cipher with HMAC-SHA1 or null auth, and AES-GCM
 *      128/256 (AEAD SRTCP), crypto on the GPU (k_rtcp). ------------------ */
srtp_err_status_t srtp_protect_rtcp(srtp_t ctx,
                                    const uint8_t *rtcp,
                                    size_t rtcp_len,
                                    uint8_t *srtcp,
                                    size_t *srtcp_len,
                                    size_t mki_index);
srtp_err_status_t srtp_unprotect_rtcp(srtp_t ctx,
                                      const uint8_t *srtcp,
                                      size_t srtcp_len,
                                      uint8_t *rtcp,
                                      size_t *rtcp_len);

/* Batch extension for SRTCP, same contract as srtp_protect_batch /
 * srtp_unprotect_batch: per-packet status, results identical to n sequential
 * srtp_protect_rtcp / srtp_unprotect_rtcp calls, one GPU launch per batch. */
srtp_err_status_t srtp_protect_rtcp_batch(srtp_t ctx,
                                          size_t n,
                                          const uint8_t *const *rtcp,
                                          const size_t *rtcp_len,
                                          uint8_t *const *srtcp,
                                          size_t *srtcp_len,
                                          const size_t *mki_index,
                                          srtp_err_status_t *status);
srtp_err_status_t srtp_unprotect_rtcp_batch(srtp_t ctx,
                                            size_t n,
                                            const uint8_t *const *srtcp,
                                            const size_t *srtcp_len,
                                            uint8_t *const *rtcp,
                                            size_t *rtcp_len,
                                            srtp_err_status_t *status);

/* ---- misc: include/srtp.h:1240-1480 ------------------------------------- */
void srtp_set_user_data(srtp_t ctx, void *data);
void *srtp_get_user_data(srtp_t ctx);
srtp_err_status_t srtp_install_event_handler(srtp_event_handler_func_t func);
const char *srtp_get_version_string(void);
unsigned int srtp_get_version(void);
srtp_err_status_t srtp_set_debug_module(const char *mod_name, bool v);
srtp_err_status_t srtp_list_debug_modules(void);
srtp_err_status_t srtp_install_log_handler(srtp_log_handler_func_t func,
                                           void *data);
srtp_err_status_t srtp_get_protect_trailer_length(srtp_t session,
                                                  size_t mki_index,
                                                  size_t *length);
srtp_err_status_t srtp_get_protect_rtcp_trailer_length(srtp_t session,
                                                       size_t mki_index,
                                                       size_t *length);
srtp_err_status_t srtp_stream_set_roc(srtp_t session,
                                      uint32_t ssrc,
                                      uint32_t roc);
srtp_err_status_t srtp_stream_get_roc(srtp_t session,
                                      uint32_t ssrc,
                                      uint32_t *roc);

/* ======================================================================
 * Batch extension (new).  Semantics == a loop of single-packet calls.
 * ====================================================================== */

/*
 * Host buffers.  Packet i is rtp[i] (rtp_len[i] bytes); its result goes to
 * srtp[i] whose capacity is srtp_len[i] on input and whose length is stored
 * there on success.  srtp[i] may equal rtp[i] (in place).  mki_index may be
 * NULL (all zero).  status[i] receives the per-packet result; the return
 * value is srtp_err_status_ok unless the batch itself could not run.
 */
srtp_err_status_t srtp_protect_batch(srtp_t ctx,
                                     size_t n,
                                     const uint8_t *const *rtp,
                                     const size_t *rtp_len,
                                     uint8_t *const *srtp,
                                     size_t *srtp_len,
                                     const size_t *mki_index,
                                     srtp_err_status_t *status);
srtp_err_status_t srtp_unprotect_batch(srtp_t ctx,
                                       size_t n,
                                       const uint8_t *const *srtp,
                                       const size_t *srtp_len,
                                       uint8_t *const *rtp,
                                       size_t *rtp_len,
                                       srtp_err_status_t *status);

/*
 * Device-resident batch: every pointer below except mki_index is a device
 * (HBM) pointer.  Packet i occupies in[in_off[i] .. +in_len[i]); in_off[i]
 * must be 16-byte aligned and the arena readable up to
 * in_off[i] + roundup16(in_len[i]).  Output goes to out + out_off[i] (may be
 * the same bytes as the input: in place) with capacity out_len[i]; on
 * success out_len[i] is overwritten with the output length.  status[i] is an
 * int32 srtp_err_status_t.  `stream` is a hipStream_t; NULL means the HIP
 * null stream (PyTorch's default stream handle is 0), so work queued there
 * before the call is ordered before it.  The call returns after the batch
 * has completed.
 */
typedef struct srtp_device_batch_t {
    size_t n;
    const uint8_t *in;
    const uint64_t *in_off;
    const uint32_t *in_len;
    uint8_t *out;
    const uint64_t *out_off;
    uint32_t *out_len;
    int32_t *status;
    const uint8_t *mki_index; /* HOST array, protect only; may be NULL */
    void *stream;
} srtp_device_batch_t;

srtp_err_status_t srtp_protect_device(srtp_t ctx, const srtp_device_batch_t *b);
/* As srtp_protect_device, but for a batch the GPU pre-pass takes the call
 * returns as soon as the pre-pass has committed it (stream state, status[]
 * and out_len[] written on the device, the protect kernel queued on
 * b->stream); the output bytes are complete when that stream gets past the
 * call.  Consecutive batches on one stream then keep the GPU busy while the
 * host submits the next one.  A batch the pre-pass declines runs to
 * completion before the call returns, as with srtp_protect_device.  No
 * counterpart for unprotect: its verdict needs the tags. */
srtp_err_status_t srtp_protect_device_async(srtp_t ctx,
                                            const srtp_device_batch_t *b);
srtp_err_status_t srtp_unprotect_device(srtp_t ctx,
                                        const srtp_device_batch_t *b);

/* ======================================================================
 * Session replication across GPUs (new; north_star "RCCL broadcast of
 * session keys over xGMI").  The reference has no
 * counterpart: its session is one process's srtp_create
 * (include/srtp.h:512, srtp/srtp.c:1233-1607 derives the session keys).
 * A replica is a session on another device (or process) with the same
 * streams, template, derived session keys (the device key records: AES
 * schedules, salts, HMAC midstates, GCM H; GHASH tables are rebuilt from H)
 * and per-stream state (index / ROC, replay windows, SRTCP index window,
 * key-usage counters).  Master keys are not part of it: they are not kept
 * after srtp_create.  Sessions whose streams use replaced crypto types
 * (srtp_replace_cipher_type / _auth_type) cannot be exported
 * (srtp_err_status_bad_param): their keys live in host vtable objects.
 * ====================================================================== */
/* Serialise `ctx` into buf (cap bytes).  *len receives the blob size; with
 * buf == NULL (or cap too small: srtp_err_status_bad_param) nothing is
 * written but *len.  The blob holds secret key material. */
srtp_err_status_t srtp_mi355x_session_export(srtp_t ctx, void *buf,
                                             size_t cap, size_t *len);
/* A new session on the calling thread's current HIP device from a blob of
 * srtp_mi355x_session_export (same library build and host byte order). */
srtp_err_status_t srtp_mi355x_session_import(srtp_t *session, const void *blob,
                                             size_t len);
/* Collective over a caller's RCCL communicator (ncclComm_t passed as
 * void *): on the communicator's rank `root`, *session is an existing
 * session whose blob is broadcast from device memory with ncclBroadcast
 * (RCCL over xGMI); on every other rank *session receives the imported
 * replica.  `stream` is the hipStream_t the broadcast is enqueued on (NULL:
 * the null stream); the call returns once the replica exists.  RCCL is
 * resolved at run time from the process (dlsym RTLD_DEFAULT, then
 * librccl.so.1): srtp_err_status_init_fail when it is absent. */
srtp_err_status_t srtp_mi355x_session_broadcast(srtp_t *session,
                                                void *nccl_comm, int root,
                                                void *stream);

/* Instrumentation for bench.py: device time (ms) of the crypto kernels of
 * the last batch, measured with HIP events on the stream they ran on.  The
 * events are read once the batch has completed: timing adds no wait inside
 * a batch (an asynchronous batch's time is read when it is asked for). */
void srtp_mi355x_set_timing(srtp_t ctx, int on);
double srtp_mi355x_last_kernel_ms(srtp_t ctx);
/* device-API batches completed by the GPU pre-pass / by the host pre-pass
 * (the latter: streams needing a template clone, a pending ROC, a stream
 * used in the other direction, duplicate indices on protect, a protect
 * batch mixing MKI keys or a receive batch carrying another key's MKI, or
 * keys near their usage limit -- DESIGN.md "Device pre-passes") */
void srtp_mi355x_prepass_stats(srtp_t ctx, uint64_t *device_batches,
                               uint64_t *host_batches);
/* device pre-pass batches of more than one stream that could not use the
 * order-free form (a stream with more packets in the batch than its replay
 * window, a gap of 2^15 or more) and ran the sorted chain path */
uint64_t srtp_mi355x_prepass_sorted_batches(srtp_t ctx);
/* one-stream device batches the in-order form (indices computed inside the
 * crypto kernel, DESIGN.md "In-order form") committed / declined (restored,
 * then the chain form ran) since the session was created */
void srtp_mi355x_inorder_stats(srtp_t ctx, uint64_t *runs, uint64_t *declines);
/* device batches whose crypto ran from key buckets (one key per wave;
 * srtp_mi355x_set_key_buckets) since the session was created */
uint64_t srtp_mi355x_bucket_batches(srtp_t ctx);
/* why the most recent srtp_protect_device fallback left the device
 * pre-pass (0: none so far): 1 unknown SSRC (template clone), 2 stream with MKI / pending ROC
 * / receiver direction, 4 sequence number not advancing by 1..2^15-1,
 * 64 empty session, 128 a key near its usage limit */
int srtp_mi355x_prepass_last_abort(srtp_t ctx);
/* of the most recent unprotect batch (host-buffer or device API): post-pass
 * rounds, crypto launches and restore (undo) launches.  Rounds stay small
 * under forged traffic: see srtp_host.c unprotect_core. */
void srtp_mi355x_unprotect_stats(srtp_t ctx, uint32_t *rounds,
                                 uint32_t *launches, uint32_t *undo_launches);
/* 1 when a HIP device is usable from this process */
int srtp_mi355x_gpu_available(void);
/* test hook: uses left on the first session key of stream `ssrc` (host
 * order), to reach the key-usage soft / hard limits in tests */
srtp_err_status_t srtp_mi355x_debug_set_key_limit(srtp_t ctx, uint32_t ssrc,
                                                  uint64_t num_left);
/* test hook: uses left on master key j of stream `ssrc` (key.c:74-90's
 * counter, after the device state came back) */
srtp_err_status_t srtp_mi355x_debug_key_left(srtp_t ctx, uint32_t ssrc,
                                             size_t j, uint64_t *num_left);

/* test hook: make the next `count` waits for the device pre-pass verdict
 * (srtp_protect_device_async) or drains of a queued async batch report a
 * GPU failure, as a stream in an error state would.  A failed drain leaves
 * the session refusing packet calls (srtp_err_status_fail). */
/* Device pre-pass tuning (process-wide): batches with many keys are laid
 * out in key buckets so that a wave's 64 packets share one key, instead of
 * one key per lane: 1 always, 0 never, -1 (the default) for AES-GCM batches
 * with a key per stream and at least 32 packets a stream on average (the
 * key's GHASH table then sits in LDS; DESIGN.md §4 -- AES-ICM gains nothing
 * on BASELINE configs[3]).  SRTP_PP_BUCKETS=1 / =0 in the environment sets
 * 1 / 0. */
void srtp_mi355x_set_key_buckets(int on);

#define SRTP_MI355X_FAIL_VERDICT_WAIT 1
#define SRTP_MI355X_FAIL_ASYNC_DRAIN 2
/* ... or that the next `count` srtp_mi355x_session_broadcast calls of this
 * process fail to allocate their blob buffers (every rank then returns
 * srtp_err_status_alloc_fail) */
#define SRTP_MI355X_FAIL_BCAST_ALLOC 3
void srtp_mi355x_debug_inject_failure(int what, int count);

/* ========================================================================
 * The crypto-kernel plugin ABI (srtp.def:46-69): libsrtp's cipher / auth
 * vtables (crypto/include/cipher.h:60-260, auth.h:55-200), the type
 * registry with srtp_replace_cipher_type / srtp_replace_auth_type
 * (crypto/kernel/crypto_kernel.c:270-440) and the utilities srtp.def
 * exports with them.  Layouts and semantics follow the reference.  The
 * built-in types are GPU-backed: every encrypt / decrypt / compute call of
 * AES-ICM-128/192/256, AES-GCM-128/256 and HMAC-SHA1 is one HIP launch
 * (srtp_plugin.c -> srtp_gpu_raw); the null cipher and null auth need no
 * device.  A replacement type must pass its own known answers and the
 * built-in type's (as in the reference), i.e. compute the same function, so
 * the packet path keeps the GPU kernels for that algorithm id.
 * ====================================================================== */
typedef enum {
    srtp_direction_encrypt,
    srtp_direction_decrypt,
    srtp_direction_any
} srtp_cipher_direction_t;

typedef struct srtp_cipher_t *srtp_cipher_pointer_t;
typedef srtp_err_status_t (*srtp_cipher_alloc_func_t)(srtp_cipher_pointer_t *cp,
                                                      size_t key_len,
                                                      size_t tag_len);
typedef srtp_err_status_t (*srtp_cipher_init_func_t)(void *state,
                                                     const uint8_t *key);
typedef srtp_err_status_t (*srtp_cipher_dealloc_func_t)(
    srtp_cipher_pointer_t cp);
typedef srtp_err_status_t (*srtp_cipher_set_aad_func_t)(void *state,
                                                        const uint8_t *aad,
                                                        size_t aad_len);
typedef srtp_err_status_t (*srtp_cipher_encrypt_func_t)(void *state,
                                                        const uint8_t *src,
                                                        size_t src_len,
                                                        uint8_t *dst,
                                                        size_t *dst_len);
typedef srtp_err_status_t (*srtp_cipher_decrypt_func_t)(void *state,
                                                        const uint8_t *src,
                                                        size_t src_len,
                                                        uint8_t *dst,
                                                        size_t *dst_len);
typedef srtp_err_status_t (*srtp_cipher_set_iv_func_t)(
    void *state, uint8_t *iv, srtp_cipher_direction_t direction);

typedef struct srtp_cipher_test_case_t {
    size_t key_length_octets;
    const uint8_t *key;
    uint8_t *idx;
    size_t plaintext_length_octets;
    const uint8_t *plaintext;
    size_t ciphertext_length_octets;
    const uint8_t *ciphertext;
    size_t aad_length_octets;
    const uint8_t *aad;
    size_t tag_length_octets;
    const struct srtp_cipher_test_case_t *next_test_case;
} srtp_cipher_test_case_t;

typedef struct srtp_cipher_type_t {
    srtp_cipher_alloc_func_t alloc;
    srtp_cipher_dealloc_func_t dealloc;
    srtp_cipher_init_func_t init;
    srtp_cipher_set_aad_func_t set_aad;
    srtp_cipher_encrypt_func_t encrypt;
    srtp_cipher_decrypt_func_t decrypt;
    srtp_cipher_set_iv_func_t set_iv;
    const char *description;
    const srtp_cipher_test_case_t *test_data;
    srtp_cipher_type_id_t id;
} srtp_cipher_type_t;

typedef struct srtp_cipher_t {
    const srtp_cipher_type_t *type;
    void *state;
    size_t key_len;
    srtp_cipher_type_id_t algorithm;
} srtp_cipher_t;

size_t srtp_cipher_get_key_length(const srtp_cipher_t *c);
srtp_err_status_t srtp_cipher_type_self_test(const srtp_cipher_type_t *ct);
srtp_err_status_t srtp_cipher_type_test(
    const srtp_cipher_type_t *ct, const srtp_cipher_test_case_t *test_data);
uint64_t srtp_cipher_bits_per_second(srtp_cipher_t *c, size_t octets_in_buffer,
                                     size_t num_trials);
srtp_err_status_t srtp_cipher_type_alloc(const srtp_cipher_type_t *ct,
                                         srtp_cipher_t **c, size_t key_len,
                                         size_t tlen);
srtp_err_status_t srtp_cipher_dealloc(srtp_cipher_t *c);
srtp_err_status_t srtp_cipher_init(srtp_cipher_t *c, const uint8_t *key);
srtp_err_status_t srtp_cipher_set_iv(srtp_cipher_t *c, uint8_t *iv,
                                     srtp_cipher_direction_t direction);
srtp_err_status_t srtp_cipher_output(srtp_cipher_t *c, uint8_t *buffer,
                                     size_t *num_octets_to_output);
srtp_err_status_t srtp_cipher_encrypt(srtp_cipher_t *c, const uint8_t *src,
                                      size_t src_len, uint8_t *dst,
                                      size_t *dst_len);
srtp_err_status_t srtp_cipher_decrypt(srtp_cipher_t *c, const uint8_t *src,
                                      size_t src_len, uint8_t *dst,
                                      size_t *dst_len);
srtp_err_status_t srtp_cipher_set_aad(srtp_cipher_t *c, const uint8_t *aad,
                                      size_t aad_len);
srtp_err_status_t srtp_replace_cipher_type(const srtp_cipher_type_t *ct,
                                           srtp_cipher_type_id_t id);

typedef const struct srtp_auth_type_t *srtp_auth_type_pointer;
typedef struct srtp_auth_t *srtp_auth_pointer_t;
typedef srtp_err_status_t (*srtp_auth_alloc_func)(srtp_auth_pointer_t *ap,
                                                  size_t key_len,
                                                  size_t out_len);
typedef srtp_err_status_t (*srtp_auth_init_func)(void *state,
                                                 const uint8_t *key,
                                                 size_t key_len);
typedef srtp_err_status_t (*srtp_auth_dealloc_func)(srtp_auth_pointer_t ap);
typedef srtp_err_status_t (*srtp_auth_compute_func)(void *state,
                                                    const uint8_t *buffer,
                                                    size_t octets_to_auth,
                                                    size_t tag_len,
                                                    uint8_t *tag);
typedef srtp_err_status_t (*srtp_auth_update_func)(void *state,
                                                   const uint8_t *buffer,
                                                   size_t octets_to_auth);
typedef srtp_err_status_t (*srtp_auth_start_func)(void *state);

/* the reference's auth.h macros */
#define srtp_auth_type_alloc(at, a, klen, outlen)                              \
    ((at)->alloc((a), (klen), (outlen)))
#define srtp_auth_init(a, key)                                                 \
    (((a)->type)->init((a)->state, (key), ((a)->key_len)))
#define srtp_auth_compute(a, buf, len, res)                                    \
    (((a)->type)->compute((a)->state, (buf), (len), (a)->out_len, (res)))
#define srtp_auth_update(a, buf, len)                                          \
    (((a)->type)->update((a)->state, (buf), (len)))
#define srtp_auth_start(a) (((a)->type)->start((a)->state))
#define srtp_auth_dealloc(c) (((c)->type)->dealloc(c))

typedef struct srtp_auth_test_case_t {
    size_t key_length_octets;
    const uint8_t *key;
    size_t data_length_octets;
    const uint8_t *data;
    size_t tag_length_octets;
    const uint8_t *tag;
    const struct srtp_auth_test_case_t *next_test_case;
} srtp_auth_test_case_t;

typedef struct srtp_auth_type_t {
    srtp_auth_alloc_func alloc;
    srtp_auth_dealloc_func dealloc;
    srtp_auth_init_func init;
    srtp_auth_compute_func compute;
    srtp_auth_update_func update;
    srtp_auth_start_func start;
    const char *description;
    const srtp_auth_test_case_t *test_data;
    srtp_auth_type_id_t id;
} srtp_auth_type_t;

typedef struct srtp_auth_t {
    const srtp_auth_type_t *type;
    void *state;
    size_t out_len;
    size_t key_len;
    size_t prefix_len;
} srtp_auth_t;

size_t srtp_auth_get_key_length(const struct srtp_auth_t *a);
size_t srtp_auth_get_tag_length(const struct srtp_auth_t *a);
size_t srtp_auth_get_prefix_length(const struct srtp_auth_t *a);
srtp_err_status_t srtp_auth_type_self_test(const srtp_auth_type_t *at);
srtp_err_status_t srtp_auth_type_test(const srtp_auth_type_t *at,
                                      const srtp_auth_test_case_t *test_data);
srtp_err_status_t srtp_replace_auth_type(const srtp_auth_type_t *ct,
                                         srtp_auth_type_id_t id);

/* crypto/include/err.h:83-124, crypto_kernel.h:166 */
typedef enum {
    srtp_err_level_error,
    srtp_err_level_warning,
    srtp_err_level_info,
    srtp_err_level_debug
} srtp_err_reporting_level_t;
typedef struct {
    bool on;
    const char *name;
} srtp_debug_module_t;
void srtp_err_report(srtp_err_reporting_level_t level, const char *format,
                     ...);
srtp_err_status_t srtp_crypto_kernel_load_debug_module(
    srtp_debug_module_t *new_dm);

/* crypto/include/datatypes.h:81, 158, 239-242; rdbx.h:78-87 */
char *srtp_octet_string_hex_string(const void *str, size_t length);
bool srtp_octet_string_equal(const uint8_t *a, const uint8_t *b, size_t len);
typedef struct {
    size_t length;
    uint32_t *word;
} bitvector_t;
typedef uint64_t srtp_xtd_seq_num_t;
typedef struct {
    srtp_xtd_seq_num_t index;
    bitvector_t bitmask;
} srtp_rdbx_t;
size_t srtp_rdbx_get_window_size(const srtp_rdbx_t *rdbx);

/* extension: the built-in (GPU-backed) type registered for an id -- the
 * reference's srtp_aes_icm_128, srtp_hmac, ... objects (NULL if none) --
 * and whatever type the registry now holds for it after a replacement */
const srtp_cipher_type_t *srtp_mi355x_builtin_cipher_type(
    srtp_cipher_type_id_t id);
const srtp_auth_type_t *srtp_mi355x_builtin_auth_type(srtp_auth_type_id_t id);
const srtp_cipher_type_t *srtp_mi355x_registered_cipher_type(
    srtp_cipher_type_id_t id);
const srtp_auth_type_t *srtp_mi355x_registered_auth_type(
    srtp_auth_type_id_t id);

#ifdef __cplusplus
}
#endif
#endif /* SRTP_MI355X_H */
