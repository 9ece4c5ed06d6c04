/*
 * srtp_host.c -- the host half of libsrtp_mi355x: the libsrtp C API
 * (include/srtp_mi355x.h) on top of the HIP kernels (srtp_kernels.hip).
 *
 * What lives here is the part of srtp/srtp.c that is inherently sequential
 * per stream and cheap: session/stream management and key derivation
 * (srtp.c:594-1716, 3250-3648), the SSRC -> stream map (replaces the linear
 * list of srtp.c:5169-5335 with an O(1) open-addressing map; first inserted
 * wins, like srtp_stream_list_get), packet-index estimation and the replay
 * window (crypto/replay/rdbx.c), key-usage limits (crypto/kernel/key.c) and
 * events.  For a batch it runs a PRE-PASS in packet order that fixes every
 * packet's index/ROC, key slot and early error exactly as srtp_protect /
 * srtp_unprotect would, then hands the whole batch to the GPU, which does
 * all AES / HMAC / GHASH work.
 *
 * Unprotect is speculative: the pre-pass assumes earlier packets of the
 * batch authenticate; a POST-PASS replays the reference's per-packet logic
 * in order with the real authentication results (srtp.c:2994-3167), and
 * re-runs ("redo") any packet whose index estimate changed because an
 * earlier packet failed.  Outputs and statuses are therefore identical to
 * calling the reference once per packet.  Redo rounds are bounded: results
 * are kept per (packet, index), forged packets stop being speculated as
 * accepted, and after UNP_SPEC_ROUNDS the residue runs in exact rounds
 * (one unresolved packet per SSRC per launch).  Packets that end with an
 * error have their speculative decryption undone, so the buffer of a
 * rejected packet holds its ciphertext, as with the reference (which
 * verifies before decrypting).
 */
#define _GNU_SOURCE /* dlsym RTLD_DEFAULT (session broadcast) */
#include "srtp_mi355x.h"

#include <dlfcn.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "host_crypto.h"
#include "srtp_dev.h"

int srtp_mi355x_debug_index(size_t window, int allow_repeat_tx,
                            uint32_t pending_roc, size_t n,
                            const uint16_t *seq, int32_t *status,
                            uint64_t *est_out);

#define SEQ_MEDIAN 32768
#define SEQ_MAX 65536
#define SOFT_LIMIT 0x10000

enum { DIR_UNKNOWN = 0, DIR_SENDER = 1, DIR_RECEIVER = 2 };

/* ------------------------------------------------------------------------
 * logging / events (srtp.c:1723-1773, 5085-5135)
 * ---------------------------------------------------------------------- */
static srtp_log_handler_func_t *g_log_handler;
static void *g_log_data;

static void log_msg(srtp_log_level_t lvl, const char *msg)
{
    if (g_log_handler)
        g_log_handler(lvl, msg, g_log_data);
    else
        fprintf(stderr, "%s", msg);
}

/* for srtp_plugin.c (srtp_err_report, debug-module listing) */
void srtp_mi355x_log(int level, const char *msg)
    __attribute__((visibility("hidden")));
void srtp_mi355x_log(int level, const char *msg)
{
    log_msg((srtp_log_level_t)level, msg);
}

static void default_event_reporter(srtp_event_data_t *d)
{
    static const char *what[] = { "SSRC collision",
                                  "key usage soft limit reached",
                                  "key usage hard limit reached",
                                  "packet index limit reached" };
    char buf[128];
    snprintf(buf, sizeof buf, "srtp: in stream 0x%x: %s\n",
             (unsigned)d->ssrc,
             (unsigned)d->event < 4 ? what[d->event] : "unknown event");
    log_msg(srtp_log_level_warning, buf);
}

static srtp_event_handler_func_t *g_event_handler = default_event_reporter;

/* ------------------------------------------------------------------------
 * session keys: one per master key of a stream, shared by template clones
 * ---------------------------------------------------------------------- */
typedef struct {
    uint32_t slot;          /* device key slot                               */
    uint32_t cipher_type;   /* SRTP_* cipher id                              */
    uint32_t family;        /* SRTP_DEV_*                                    */
    uint32_t rounds;
    uint32_t variant;       /* kernel variant id (srtp_dev.h)                */
    size_t tag_len;
    uint8_t mki[SRTP_MAX_MKI_LEN];
    uint64_t num_left;      /* key.c: srtp_key_limit_ctx_t                   */
    int limit_state;        /* 0 normal, 1 past soft limit, 2 expired        */
    /* SRTCP session key (srtp.c:1527-1600, KDF labels 3/4/5): own device
     * slot, ~0 when the RTCP policy is not supported (srtp_protect_rtcp then
     * reports no_such_op) */
    uint32_t rslot;
    size_t rtag_len;
    int rgcm;               /* the RTCP cipher is AES-GCM (MKI offset)      */
    /* RFC 6904 extension-header key (srtp.c:1385-1500): own device slot,
     * ~0 without header-extension encryption */
    uint32_t xslot;
    /* routed key (variant SRTP_VARIANT_V): the RTP cipher / auth objects of
     * the REGISTERED types, as the reference allocates them from its crypto
     * kernel (srtp.c:594-752, 1342-1525), the AEAD salt, the services */
    srtp_cipher_t *vc;
    srtp_auth_t *va;
    uint8_t vsalt[12];
    uint32_t vcid;      /* cipher type id */
    int vconf, vauth;   /* sec_serv_conf / auth in force */
    size_t vmki;        /* MKI bytes of the stream */
} hkey_t;

typedef struct {
    int refs;
    size_t n;
    int cryptex;   /* policy use_cryptex (RFC 9335)                          */
    hkey_t k[SRTP_MAX_NUM_MASTER_KEYS];
} keyset_t;

/* replay database (crypto/replay/rdbx.c) */
typedef struct {
    uint64_t index;
    size_t bits;      /* window length rounded up to 32 (datatypes.c:264) */
    uint32_t *w;
    uint32_t pending_roc;
} rdbx_t;

struct srtp_stream_ctx_t_ {
    uint32_t ssrc;    /* host-order numeric value */
    int direction;
    int rtp_services;
    int rtcp_services;
    bool allow_repeat_tx;
    bool use_mki;
    size_t mki_size;
    keyset_t *keys;
    rdbx_t rdbx;
    size_t window_size; /* as requested */
    /* per-batch speculative shadow (unprotect pre-pass) */
    uint64_t spec_epoch;
    rdbx_t spec;
    uint32_t dev_sid;   /* id in the device stream table (dev_build) */
    size_t lpos;        /* index in ctx->list */
    /* SRTCP replay database (crypto/replay/rdb.c): 31-bit index window */
    uint32_t rtcp_start;
    uint32_t rtcp_bm[4];
};

typedef struct {
    uint32_t *keys; /* ssrc */
    srtp_stream_ctx_t **vals;
    size_t cap;     /* power of two */
    size_t used;
} ssrc_map_t;

typedef struct {
    /* host-buffer batch staging (pinned) and its device mirror */
    uint8_t *h_arena, *d_arena;
    size_t arena_cap;
    uint64_t *h_off, *d_off;
    srtp_dev_meta_t *h_meta, *d_meta;
    uint8_t *h_auth, *d_auth;
    srtp_dev_hdr_t *h_hdr, *d_hdr;
    uint32_t *h_xinfo, *d_xinfo; /* CC / X / profile (k_parse) */
    /* host-buffer batches on the device pre-pass: lengths in, capacities
     * in / lengths out, statuses out */
    uint32_t *h_len, *d_len, *h_cap, *d_cap;
    int32_t *h_st, *d_st;
    size_t n_cap;
} stage_t;

/* device mirror of the stream table for the device pre-pass
 * (srtp_prepass.hip); see dev_build / dev_pull */
typedef struct {
    int valid;              /* device table mirrors the host streams       */
    int dirty;              /* device state is newer than the host's       */
    uint32_t ns;
    srtp_stream_ctx_t **sv; /* stream id -> stream                         */
    srtp_dev_stream_t *hs;  /* host image of the table                     */
    uint32_t *hwin;         /* host image of the window arena              */
    uint32_t nwords;
    uint64_t num_left_min;  /* over the keys of eligible streams           */
    uint64_t uses_bound;    /* packets run on the device since the upload  */
    uint32_t uniform, mask;       /* over the protect-eligible streams    */
    uint32_t max_trailer;         /* ... and their largest trailer        */
    uint32_t rx_uniform, rx_mask; /* over the unprotect-eligible streams  */
    uint64_t fast_batches, host_batches;
    uint64_t sorted_batches; /* fast batches that needed the sorted path  */
    uint64_t io_runs, io_declines; /* one-stream in-order form: batches it
                                      committed / declined (chain form ran) */
    uint64_t bk_batches;    /* batches whose crypto ran from key buckets */
    int last_abort;         /* reason of the most recent fallback         */
    int async_pending;      /* srtp_protect_device_async left its protect
                               kernel (and the tail of its commit) queued */
    void *async_stream;     /* ... on this stream                          */
    int async_err;          /* a queued batch failed on the GPU: sticky,
                               every later packet call returns _fail      */
    /* MKI streams (srtp.c:1961-2036): protect batches run each packet on
     * the master key its mki_index selects, receive batches on the key its
     * MKI bytes select (the slots of every stream's keys in mkslot, the
     * packets charged to each counted in kuses) */
    int has_mki;
    int rx_multi;           /* a receive-eligible MKI stream has > 1 key   */
    uint32_t *mkslot, nmk;  /* key slots of the MKI streams' keys          */
    uint64_t *kuses;        /* downloaded per-key protect charges          */
    uint32_t mki_nmin;      /* fewest master keys of a protect-eligible
                               MKI stream                                  */
    uint32_t tmpl_kbase;    /* the template's keys in mkslot               */
    /* streams with a pending ROC (srtp_stream_set_roc) the device may take:
     * resolved per batch (pend_resolve); the ones the running batch applied */
    uint32_t *pend, npend;
    uint32_t *res, nres;
    /* template sessions: the device creates streams from the template
     * (srtp_gpu_pp_clone); dev_pull takes them over */
    int tmpl_ok;
} devtab_t;

struct srtp_ctx_t_ {
    srtp_stream_ctx_t *templ;
    srtp_stream_ctx_t **list; /* insertion order, like the reference list */
    size_t n, cap;
    ssrc_map_t map;
    void *user_data;
    srtp_gpu_t *gpu;
    uint32_t next_slot;
    uint32_t *free_slots;
    size_t n_free, free_cap;
    uint32_t variant_mask;
    stage_t st;
    uint64_t epoch;
    struct {
        uint32_t rounds, launches, undo_launches;
    } ustat; /* of the most recent unprotect batch */
    int timing;
    double last_ms;
    devtab_t dt;
    /* queued GPU key derivations (kq_flush); SRTP_MI355X_HOST_KDF=1 derives
     * on the host instead */
    srtp_kdf_job_t *kq;
    size_t kq_n, kq_cap;
    uint32_t *rel;          /* slots released while jobs were queued */
    size_t n_rel, rel_cap;
    int host_kdf;
    /* routed keys by device slot (run_routed), per-packet results of the
     * last routed run: protect status codes, unprotect's decrypted
     * packets' original bytes (undo) */
    hkey_t **vkeys;
    size_t vkeys_cap;
    uint8_t *vres;
    uint8_t **vsave;
    size_t vres_cap;
};

static void dev_pull(srtp_t ctx);
static int async_drain(srtp_t ctx);

/* after a queued (async) batch failed on the GPU the device stream state is
 * unknown: no packet call may run on the session any more */
#define ASYNC_POISON_CHECK(ctx)                                                \
    do {                                                                       \
        if ((ctx) && (ctx)->dt.async_err)                                      \
            return srtp_err_status_fail;                                       \
    } while (0)
/* the same, after the queued batch (if any) has finished: for calls that
 * read or change the stream state from the host */
#define ASYNC_DRAIN_CHECK(ctx)                                                 \
    do {                                                                       \
        if ((ctx) && async_drain(ctx))                                         \
            return srtp_err_status_fail;                                       \
    } while (0)

/* the session's own stream: host-buffer batches run on it.  Device-API
 * batches run on the caller's stream, NULL meaning the HIP null stream
 * (PyTorch's default stream handle is 0). */
#define HS(ctx) srtp_gpu_stream_of((ctx)->gpu)

/* ------------------------------------------------------------------------
 * SSRC map
 * ---------------------------------------------------------------------- */
static size_t map_hash(uint32_t k, size_t cap)
{
    uint32_t h = k * 0x9e3779b1u;
    h ^= h >> 15;
    return h & (cap - 1);
}

static int map_rebuild(srtp_t ctx, size_t cap)
{
    ssrc_map_t m;
    m.cap = cap;
    m.used = 0;
    m.keys = (uint32_t *)calloc(cap, sizeof(uint32_t));
    m.vals = (srtp_stream_ctx_t **)calloc(cap, sizeof(void *));
    if (!m.keys || !m.vals) {
        free(m.keys);
        free(m.vals);
        return -1;
    }
    for (size_t i = 0; i < ctx->n; i++) {
        srtp_stream_ctx_t *s = ctx->list[i];
        size_t h = map_hash(s->ssrc, cap);
        int dup = 0;
        while (m.vals[h]) {
            if (m.keys[h] == s->ssrc) {
                dup = 1; /* first inserted wins (srtp.c:5292-5305) */
                break;
            }
            h = (h + 1) & (cap - 1);
        }
        if (!dup) {
            m.keys[h] = s->ssrc;
            m.vals[h] = s;
            m.used++;
        }
    }
    free(ctx->map.keys);
    free(ctx->map.vals);
    ctx->map = m;
    return 0;
}

static srtp_stream_ctx_t *map_get(const srtp_t ctx, uint32_t ssrc)
{
    if (!ctx->map.cap)
        return NULL;
    size_t h = map_hash(ssrc, ctx->map.cap);
    while (ctx->map.vals[h]) {
        if (ctx->map.keys[h] == ssrc)
            return ctx->map.vals[h];
        h = (h + 1) & (ctx->map.cap - 1);
    }
    return NULL;
}

static int list_insert(srtp_t ctx, srtp_stream_ctx_t *s)
{
    if (ctx->n == ctx->cap) {
        size_t nc = ctx->cap ? 2 * ctx->cap : 4;
        void *p = realloc(ctx->list, nc * sizeof(void *));
        if (!p)
            return -1;
        ctx->list = (srtp_stream_ctx_t **)p;
        ctx->cap = nc;
    }
    s->lpos = ctx->n;
    ctx->list[ctx->n++] = s;
    if (2 * (ctx->map.used + 1) > ctx->map.cap)
        return map_rebuild(ctx, ctx->map.cap ? 2 * ctx->map.cap : 64);
    /* plain insert unless an older stream already owns the SSRC */
    size_t h = map_hash(s->ssrc, ctx->map.cap);
    while (ctx->map.vals[h]) {
        if (ctx->map.keys[h] == s->ssrc)
            return 0;
        h = (h + 1) & (ctx->map.cap - 1);
    }
    ctx->map.keys[h] = s->ssrc;
    ctx->map.vals[h] = s;
    ctx->map.used++;
    return 0;
}

static void list_remove(srtp_t ctx, srtp_stream_ctx_t *s)
{
    size_t i = s->lpos;
    if (i < ctx->n && ctx->list[i] == s) {
        memmove(&ctx->list[i], &ctx->list[i + 1],
                (ctx->n - i - 1) * sizeof(void *));
        ctx->n--;
        for (; i < ctx->n; i++)
            ctx->list[i]->lpos = i;
    }
    map_rebuild(ctx, ctx->map.cap ? ctx->map.cap : 64);
}

/* the stream `ns` takes old's place in the list and the SSRC map */
static void list_replace(srtp_t ctx, srtp_stream_ctx_t *old,
                         srtp_stream_ctx_t *ns)
{
    ns->lpos = old->lpos;
    ctx->list[old->lpos] = ns;
    for (size_t h = map_hash(old->ssrc, ctx->map.cap); ctx->map.vals[h];
         h = (h + 1) & (ctx->map.cap - 1))
        if (ctx->map.vals[h] == old) {
            ctx->map.vals[h] = ns;
            break;
        }
}

/* ------------------------------------------------------------------------
 * rdbx: crypto/replay/rdbx.c, bitvector of crypto/math/datatypes.c
 * ---------------------------------------------------------------------- */
static int rdbx_init(rdbx_t *r, size_t ws)
{
    r->bits = (ws + 31) & ~(size_t)31;
    r->w = (uint32_t *)calloc(r->bits / 32 + 1, sizeof(uint32_t));
    r->index = 0;
    r->pending_roc = 0;
    return r->w ? 0 : -1;
}

static void rdbx_copy(rdbx_t *dst, const rdbx_t *src)
{
    if (dst->bits != src->bits) {
        free(dst->w);
        dst->w = (uint32_t *)calloc(src->bits / 32 + 1, sizeof(uint32_t));
        dst->bits = src->bits;
    }
    memcpy(dst->w, src->w, src->bits / 8);
    dst->index = src->index;
    dst->pending_roc = src->pending_roc;
}

static void win_zero(rdbx_t *r) { memset(r->w, 0, r->bits / 8); }

static void win_shift(rdbx_t *r, size_t shift)
{
    size_t words = r->bits >> 5;
    if (shift >= r->bits) {
        win_zero(r);
        return;
    }
    size_t base = shift >> 5, bi = shift & 31;
    if (bi == 0) {
        memmove(r->w, r->w + base, (words - base) * 4);
    } else {
        for (size_t i = 0; i + base + 1 < words; i++)
            r->w[i] = (r->w[i + base] >> bi) | (r->w[i + base + 1] << (32 - bi));
        r->w[words - base - 1] = r->w[words - 1] >> bi;
    }
    memset(r->w + (words - base), 0, base * 4);
}

static int64_t index_guess(uint64_t local, uint64_t *guess, uint16_t s)
{
    /* rdbx.c:112-145 */
    uint32_t local_roc = (uint32_t)(local >> 16);
    uint16_t local_seq = (uint16_t)local;
    uint32_t roc;
    int64_t diff;
    if (local_seq < SEQ_MEDIAN) {
        if ((int)s - (int)local_seq > SEQ_MEDIAN) {
            roc = local_roc - 1;
            diff = (int64_t)s - local_seq - SEQ_MAX;
        } else {
            roc = local_roc;
            diff = (int64_t)s - local_seq;
        }
    } else {
        if ((int)local_seq - SEQ_MEDIAN > (int)s) {
            roc = local_roc + 1;
            diff = (int64_t)s - local_seq + SEQ_MAX;
        } else {
            roc = local_roc;
            diff = (int64_t)s - local_seq;
        }
    }
    *guess = ((uint64_t)roc << 16) | s;
    return diff;
}

static srtp_err_status_t estimate(const rdbx_t *r, uint16_t seq, uint64_t *est,
                                  int64_t *delta)
{
    /* srtp_get_est_pkt_index + srtp_estimate_index, srtp.c:2038-2081;
     * srtp_rdbx_estimate_index, rdbx.c:280-299 */
    if (r->pending_roc) {
        *est = ((uint64_t)r->pending_roc << 16) | seq;
        *delta = (int64_t)(*est - r->index);
        if (*est > r->index) {
            if (*est - r->index > SEQ_MEDIAN) {
                *delta = 0;
                return srtp_err_status_pkt_idx_adv;
            }
        } else if (*est < r->index) {
            if (r->index - *est > SEQ_MEDIAN) {
                *delta = 0;
                return srtp_err_status_pkt_idx_old;
            }
        }
        return srtp_err_status_ok;
    }
    if (r->index > SEQ_MEDIAN) {
        *delta = index_guess(r->index, est, seq);
    } else {
        *est = seq;
        *delta = (int64_t)seq - (int64_t)r->index;
    }
    return srtp_err_status_ok;
}

static srtp_err_status_t rdbx_check(const rdbx_t *r, int64_t delta)
{
    /* rdbx.c:227-243 */
    if (delta > 0)
        return srtp_err_status_ok;
    if ((int64_t)(r->bits - 1) + delta < 0)
        return srtp_err_status_replay_old;
    size_t bit = (size_t)((int64_t)(r->bits - 1) + delta);
    if ((r->w[bit >> 5] >> (bit & 31)) & 1)
        return srtp_err_status_replay_fail;
    return srtp_err_status_ok;
}

static void rdbx_add(rdbx_t *r, int64_t delta)
{
    /* rdbx.c:253-270 */
    size_t bit;
    if (delta > 0) {
        r->index += (uint16_t)delta;
        win_shift(r, (size_t)delta);
        bit = r->bits - 1;
    } else {
        bit = (size_t)((int64_t)(r->bits - 1) + delta);
    }
    r->w[bit >> 5] |= 1u << (bit & 31);
}

static void rdbx_set_roc_seq(rdbx_t *r, uint32_t roc, uint16_t seq)
{
    /* rdbx.c:323-338 */
    if (roc < (r->index >> 16))
        return;
    r->index = ((uint64_t)roc << 16) | seq;
    win_zero(r);
}

/* the index/replay step shared by protect and unprotect-commit */
static void rdbx_accept(rdbx_t *r, uint64_t est, int64_t delta, int adv)
{
    if (adv) {
        rdbx_set_roc_seq(r, (uint32_t)(est >> 16), (uint16_t)est);
        r->pending_roc = 0;
        rdbx_add(r, 0);
    } else {
        rdbx_add(r, delta);
    }
}

/* key.c:74-90 -> 0 normal, 1 soft, 2 hard */
static int key_limit_update(hkey_t *k)
{
    k->num_left--;
    if (k->num_left >= SOFT_LIMIT)
        return 0;
    if (k->limit_state == 0)
        k->limit_state = 1;
    if (k->num_left < 1) {
        k->limit_state = 2;
        return 2;
    }
    return 1;
}

static void fire(srtp_t ctx, const srtp_stream_ctx_t *s, srtp_event_t ev)
{
    if (g_event_handler) {
        srtp_event_data_t d;
        d.session = ctx;
        d.ssrc = s->ssrc;
        d.event = ev;
        g_event_handler(&d);
    }
}

/* ------------------------------------------------------------------------
 * KDF and key setup (srtp.c:1070-1142, 1233-1607)
 * ---------------------------------------------------------------------- */
static size_t full_key_length(uint32_t id)
{
    switch (id) {
    case SRTP_AES_ICM_128: return SRTP_AES_ICM_128_KEY_LEN_WSALT;
    case SRTP_AES_ICM_192: return SRTP_AES_ICM_192_KEY_LEN_WSALT;
    case SRTP_AES_ICM_256: return SRTP_AES_ICM_256_KEY_LEN_WSALT;
    case SRTP_AES_GCM_128: return SRTP_AES_GCM_128_KEY_LEN_WSALT;
    case SRTP_AES_GCM_256: return SRTP_AES_GCM_256_KEY_LEN_WSALT;
    default: return 0;
    }
}

static size_t base_key_length(uint32_t id, size_t key_len)
{
    switch (id) {
    case SRTP_NULL_CIPHER: return 0;
    case SRTP_AES_ICM_128:
    case SRTP_AES_ICM_192:
    case SRTP_AES_ICM_256: return key_len - SRTP_SALT_LEN;
    case SRTP_AES_GCM_128:
    case SRTP_AES_GCM_256: return key_len - SRTP_AEAD_SALT_LEN;
    default: return key_len;
    }
}

static int cipher_supported(const srtp_crypto_policy_t *c)
{
    switch (c->cipher_type) {
    case SRTP_NULL_CIPHER:
        return 1;
    case SRTP_AES_ICM_128:
    case SRTP_AES_ICM_192:
    case SRTP_AES_ICM_256:
        /* aes_icm(_ossl).c: key_len 30 / 38 / 46 only */
        return c->cipher_key_len == full_key_length(c->cipher_type);
    case SRTP_AES_GCM_128:
    case SRTP_AES_GCM_256:
        /* aes_gcm_ossl.c:97-99: tag 8 or 16 */
        return c->cipher_key_len == full_key_length(c->cipher_type) &&
               (c->auth_tag_len == 8 || c->auth_tag_len == 16);
    default:
        return 0;
    }
}

static int auth_supported(const srtp_crypto_policy_t *c)
{
    if (c->auth_type == SRTP_HMAC_SHA1)
        return c->auth_key_len <= 20 && c->auth_tag_len <= 20; /* hmac.c:76 */
    if (c->auth_type == SRTP_NULL_AUTH) /* a tag: prefix_mode() */
        return c->auth_tag_len <= SRTP_MAX_TAG_LEN;
    return 0;
}

/* libsrtp's legacy keystream-prefix mode: a null auth with a non-zero tag
 * and the auth service on (null_auth.c:80 prefix_len = out_len); the tag is
 * the first tag_len keystream bytes of the packet and the payload takes the
 * keystream after them (srtp.c:2729-2741, 3006-3020).  Such RTP sessions run
 * through the routed path (run_routed), not the kernels. */
static int prefix_mode(const srtp_crypto_policy_t *c)
{
    return c->auth_type == SRTP_NULL_AUTH && c->auth_tag_len > 0 &&
           (c->sec_serv & sec_serv_auth) &&
           c->cipher_type != SRTP_AES_GCM_128 &&
           c->cipher_type != SRTP_AES_GCM_256;
}

static void kdf_gen(const hc_aes_t *kdf, const uint8_t salt14[14],
                    uint8_t label, uint8_t *out, size_t len)
{
    uint8_t nonce[16] = { 0 };
    nonce[7] = label; /* srtp.c:1112-1113 */
    hc_icm_keystream(kdf, salt14, nonce, out, len);
}

/* a cipher / auth type id the application replaced: the reference then
 * runs that id's crypto through the registered type (crypto_kernel.c:
 * 272-348, 421-425, 445-506) */
static int cipher_routed(srtp_cipher_type_id_t id)
{
    const srtp_cipher_type_t *r = srtp_mi355x_registered_cipher_type(id);
    return r && r != srtp_mi355x_builtin_cipher_type(id);
}

static int auth_routed(srtp_auth_type_id_t id)
{
    const srtp_auth_type_t *r = srtp_mi355x_registered_auth_type(id);
    return r && r != srtp_mi355x_builtin_auth_type(id);
}

/* the KDF's AES-ICM type by the KDF key length (srtp_kdf_init,
 * srtp.c:1070-1103) */
static srtp_cipher_type_id_t kdf_cipher_id(size_t kdf_keylen)
{
    return kdf_keylen == 46   ? SRTP_AES_ICM_256
           : kdf_keylen == 38 ? SRTP_AES_ICM_192
                              : SRTP_AES_ICM_128;
}

/* srtp_kdf_generate (srtp.c:1105-1131) through a registered AES-ICM type:
 * key = the PRF key followed by its 14-byte salt (contiguous) */
static int vt_kdf_gen(srtp_cipher_type_id_t id, const uint8_t *key_salt,
                      size_t kdf_keylen, uint8_t label, uint8_t *out,
                      size_t len)
{
    memset(out, 0, len);
    if (!len)
        return 0;
    srtp_cipher_t *c = NULL;
    if (srtp_cipher_type_alloc(srtp_mi355x_registered_cipher_type(id), &c,
                               kdf_keylen, 0) || !c)
        return -1;
    uint8_t nonce[16] = { 0 };
    nonce[7] = label;
    size_t olen = len;
    int bad = srtp_cipher_init(c, key_salt) ||
              srtp_cipher_set_iv(c, nonce, srtp_direction_encrypt) ||
              srtp_cipher_encrypt(c, out, len, out, &olen);
    srtp_cipher_dealloc(c);
    return bad ? -1 : 0;
}

static uint32_t alloc_slot(srtp_t ctx)
{
    if (ctx->n_free)
        return ctx->free_slots[--ctx->n_free];
    return ctx->next_slot++;
}

/* Pending session-key derivations for the GPU (k_kdf, srtp_gpu_kdf): a
 * stream's keys are queued by init_key and derived in one launch when the
 * public call that created them returns (srtp_create with 64k policies is
 * one launch, not 64k host derivations and uploads).  A slot is never
 * released, reused or read by a kernel with its job still queued. */
static void free_slot_now(srtp_t ctx, uint32_t slot)
{
    if (ctx->n_free == ctx->free_cap) {
        size_t nc = ctx->free_cap ? 2 * ctx->free_cap : 16;
        uint32_t *p = (uint32_t *)realloc(ctx->free_slots, nc * 4);
        if (!p)
            return;
        ctx->free_slots = p;
        ctx->free_cap = nc;
    }
    ctx->free_slots[ctx->n_free++] = slot;
}

static int kq_flush(srtp_t ctx)
{
    int rc = 0;
    if (ctx->kq_n) {
        rc = srtp_gpu_kdf(ctx->gpu, ctx->kq, ctx->kq_n);
        ctx->kq_n = 0;
        if (rc)
            log_msg(srtp_log_level_error, srtp_gpu_last_error());
    }
    /* slots released while jobs were queued become reusable now */
    for (size_t i = 0; i < ctx->n_rel; i++)
        free_slot_now(ctx, ctx->rel[i]);
    ctx->n_rel = 0;
    return rc;
}

static srtp_kdf_job_t *kq_push(srtp_t ctx)
{
    if (ctx->kq_n == ctx->kq_cap) {
        size_t nc = ctx->kq_cap ? 2 * ctx->kq_cap : 64;
        srtp_kdf_job_t *q =
            (srtp_kdf_job_t *)realloc(ctx->kq, nc * sizeof(srtp_kdf_job_t));
        if (!q)
            return NULL;
        ctx->kq = q;
        ctx->kq_cap = nc;
    }
    srtp_kdf_job_t *j = &ctx->kq[ctx->kq_n++];
    memset(j, 0, sizeof *j);
    return j;
}

static void release_slot(srtp_t ctx, uint32_t slot)
{
    if (!ctx->kq_n) {
        free_slot_now(ctx, slot);
        return;
    }
    /* a queued job may still write this slot: reuse it after the flush */
    if (ctx->n_rel == ctx->rel_cap) {
        size_t nc = ctx->rel_cap ? 2 * ctx->rel_cap : 16;
        uint32_t *p = (uint32_t *)realloc(ctx->rel, nc * 4);
        if (!p)
            return;
        ctx->rel = p;
        ctx->rel_cap = nc;
    }
    ctx->rel[ctx->n_rel++] = slot;
}

/* one device key record: on the host (SRTP_MI355X_HOST_KDF=1) or queued for
 * k_kdf.  `kk` / `ks`: the PRF's AES key (kdf_len bytes) and 14-byte offset;
 * labels and output lengths as srtp_stream_init_keys draws them. */
typedef struct {
    const uint8_t *kk, *ks;
    size_t kdf_len;
    uint8_t lab_enc, lab_salt, lab_auth;
    size_t enc_len, salt_len, auth_len;
    int hmac, gcm_h, ghash;
    int tail;                 /* salt bytes salt_len, salt_len + 1 from tail */
    uint8_t tail_b[2];
    /* routed KDF: the PRF runs through this registered AES-ICM type id
     * (kdf_keylen = kdf_len + 14), on the host */
    int vkdf;
    srtp_cipher_type_id_t vkdf_id;
    /* routed key: the derived bytes are returned here and the device
     * record holds no key material */
    uint8_t *raw_ek, *raw_sa, *raw_ak;
} kspec_t;

static int put_key(srtp_t ctx, uint32_t slot, srtp_dev_key_t *dk,
                   const kspec_t *q)
{
    if (!ctx->host_kdf && !q->vkdf && !q->raw_ek) {
        srtp_kdf_job_t *j = kq_push(ctx);
        if (!j)
            return -1;
        j->key = *dk;
        memcpy(j->kdf_key, q->kk, q->kdf_len);
        memcpy(j->kdf_salt, q->ks, 14);
        j->kdf_len = (uint32_t)q->kdf_len;
        j->lab_enc = q->lab_enc;
        j->lab_salt = q->lab_salt;
        j->lab_auth = q->lab_auth;
        j->enc_len = (uint32_t)q->enc_len;
        j->salt_len = (uint32_t)q->salt_len;
        j->auth_len = (uint32_t)q->auth_len;
        j->flags = (q->hmac ? SRTP_KDF_HMAC : 0) |
                   (q->gcm_h ? SRTP_KDF_GCM_H : 0) |
                   (q->ghash ? SRTP_KDF_GHASH : 0) |
                   (q->tail ? SRTP_KDF_SALT_TAIL : 0);
        j->salt_tail[0] = q->tail_b[0];
        j->salt_tail[1] = q->tail_b[1];
        j->slot = slot;
        return 0;
    }
    uint8_t ek[32], sa[16], ak[20];
    memset(sa, 0, sizeof sa);
    if (q->vkdf) {
        const size_t kl = q->kdf_len + 14;
        if (q->ks != q->kk + q->kdf_len ||
            vt_kdf_gen(q->vkdf_id, q->kk, kl, q->lab_enc, ek, q->enc_len) ||
            vt_kdf_gen(q->vkdf_id, q->kk, kl, q->lab_salt, sa, q->salt_len) ||
            vt_kdf_gen(q->vkdf_id, q->kk, kl, q->lab_auth, ak, q->auth_len))
            return -1;
    } else {
        hc_aes_t kdf;
        hc_aes_init(&kdf, q->kk, q->kdf_len);
        kdf_gen(&kdf, q->ks, q->lab_enc, ek, q->enc_len);
        kdf_gen(&kdf, q->ks, q->lab_salt, sa, q->salt_len);
        kdf_gen(&kdf, q->ks, q->lab_auth, ak, q->auth_len);
    }
    if (q->tail) {
        sa[q->salt_len] = q->tail_b[0];
        sa[q->salt_len + 1] = q->tail_b[1];
    }
    if (q->raw_ek) {
        /* routed: the registered types get the bytes; the device record
         * stays empty (family NULL, no schedule: k_undo passes it by) */
        memcpy(q->raw_ek, ek, q->enc_len);
        memcpy(q->raw_sa, sa, q->salt_len);
        memcpy(q->raw_ak, ak, q->auth_len);
        memset(ek, 0, sizeof ek);
        memset(ak, 0, sizeof ak);
        srtp_dev_key_t z;
        memset(&z, 0, sizeof z);
        z.family = SRTP_DEV_NULL;
        z.ghash_slot = slot;
        return srtp_gpu_set_key(ctx->gpu, slot, &z, NULL);
    }
    for (int i = 0; i < 4; i++)
        dk->salt[i] = (uint32_t)sa[4 * i] | (uint32_t)sa[4 * i + 1] << 8 |
                      (uint32_t)sa[4 * i + 2] << 16 | (uint32_t)sa[4 * i + 3] << 24;
    uint32_t gbuf[1024];
    uint32_t *gtab = NULL;
    if (q->enc_len) {
        hc_aes_t ca;
        hc_aes_init(&ca, ek, q->enc_len);
        memcpy(dk->rk, ca.rk, sizeof dk->rk);
        if (q->gcm_h || q->ghash) {
            uint8_t z[16] = { 0 }, h[16];
            hc_aes_block(&ca, z, h);
            for (int i = 0; i < 4; i++)
                dk->h[i] = (uint32_t)h[4 * i] << 24 | (uint32_t)h[4 * i + 1] << 16 |
                           (uint32_t)h[4 * i + 2] << 8 | h[4 * i + 3];
            if (q->ghash) {
                hc_ghash_table(h, gbuf);
                gtab = gbuf;
            }
        }
    }
    if (q->hmac) {
        uint8_t pad[64];
        for (int i = 0; i < 64; i++)
            pad[i] = (uint8_t)((i < (int)q->auth_len ? ak[i] : 0) ^ 0x36);
        hc_sha1_midstate(pad, dk->ipad);
        for (int i = 0; i < 64; i++)
            pad[i] = (uint8_t)((i < (int)q->auth_len ? ak[i] : 0) ^ 0x5c);
        hc_sha1_midstate(pad, dk->opad);
    }
    memset(ek, 0, sizeof ek);
    memset(ak, 0, sizeof ak);
    return srtp_gpu_set_key(ctx->gpu, slot, dk, gtab);
}

static int vkeys_set(srtp_t ctx, uint32_t slot, hkey_t *hk)
{
    if (slot >= ctx->vkeys_cap) {
        size_t nc = ctx->vkeys_cap ? ctx->vkeys_cap : 64;
        while (nc <= slot)
            nc *= 2;
        hkey_t **v = (hkey_t **)realloc(ctx->vkeys, nc * sizeof *v);
        if (!v)
            return -1;
        memset(v + ctx->vkeys_cap, 0, (nc - ctx->vkeys_cap) * sizeof *v);
        ctx->vkeys = v;
        ctx->vkeys_cap = nc;
    }
    ctx->vkeys[slot] = hk;
    return 0;
}

/* a routed RTP key: cipher and auth objects of the registered types,
 * allocated and keyed as srtp_stream_alloc / srtp_stream_init_keys do
 * (srtp.c:615-641, 1378-1384, 1512-1518) */
static int route_key(srtp_t ctx, hkey_t *hk, const srtp_crypto_policy_t *rtp,
                     size_t base, size_t salt_len, const uint8_t *ek,
                     const uint8_t *sa, const uint8_t *ak)
{
    uint8_t kb[64];
    memcpy(kb, ek, base);
    memcpy(kb + base, sa, salt_len);
    if (srtp_cipher_type_alloc(srtp_mi355x_registered_cipher_type(
                                   rtp->cipher_type),
                               &hk->vc, rtp->cipher_key_len,
                               rtp->auth_tag_len) ||
        !hk->vc || srtp_cipher_init(hk->vc, kb)) {
        memset(kb, 0, sizeof kb);
        return -1;
    }
    memset(kb, 0, sizeof kb);
    const srtp_auth_type_t *at = srtp_mi355x_registered_auth_type(rtp->auth_type);
    if (!at || srtp_auth_type_alloc(at, &hk->va, rtp->auth_key_len,
                                    rtp->auth_tag_len) ||
        !hk->va || srtp_auth_init(hk->va, ak))
        return -1;
    memcpy(hk->vsalt, sa, 12);
    hk->vcid = rtp->cipher_type;
    hk->vconf = (rtp->sec_serv & sec_serv_conf) != 0 ||
                hk->family == SRTP_DEV_GCM;
    hk->vauth = (rtp->sec_serv & sec_serv_auth) != 0 &&
                hk->family != SRTP_DEV_GCM;
    hk->variant = SRTP_VARIANT_V;
    return vkeys_set(ctx, hk->slot, hk);
}

/* srtp_stream_init_keys (srtp.c:1233-1607) for one master key: the host
 * settles every policy question and the record layout; the derivations run
 * in put_key */
static srtp_err_status_t init_key(srtp_t ctx, hkey_t *hk,
                                  const srtp_policy_t *p, const uint8_t *master,
                                  const uint8_t *mki_id, size_t mki_size)
{
    const srtp_crypto_policy_t *rtp = &p->rtp, *rtcp = &p->rtcp;
    size_t input_keylen = full_key_length(rtp->cipher_type), t;
    if (rtp->auth_type == SRTP_HMAC_SHA1 && 30 > input_keylen)
        input_keylen = 30;
    t = full_key_length(rtcp->cipher_type);
    if (t > input_keylen)
        input_keylen = t;
    if (rtcp->auth_type == SRTP_HMAC_SHA1 && 30 > input_keylen)
        input_keylen = 30;
    size_t rtp_keylen = rtp->cipher_key_len, rtcp_keylen = rtcp->cipher_key_len;
    size_t base = base_key_length(rtp->cipher_type, rtp_keylen);
    size_t salt_len = rtp_keylen - base;
    if (rtp_keylen < input_keylen && rtcp_keylen < input_keylen)
        return srtp_err_status_bad_param; /* srtp.c:1293-1295 */
    size_t kdf_keylen = 30;
    if (rtp_keylen > kdf_keylen)
        kdf_keylen = rtp_keylen;
    if (rtcp_keylen > kdf_keylen)
        kdf_keylen = rtcp_keylen;
    if (input_keylen > kdf_keylen)
        kdf_keylen = input_keylen;
    if (kdf_keylen == SRTP_AES_GCM_128_KEY_LEN_WSALT ||
        kdf_keylen == SRTP_AES_GCM_256_KEY_LEN_WSALT)
        kdf_keylen += 2; /* srtp.c:1309-1312 */
    if (kdf_keylen != 30 && kdf_keylen != 38 && kdf_keylen != 46)
        return srtp_err_status_init_fail;
    if (base != 0 && base != 16 && base != 24 && base != 32)
        return srtp_err_status_init_fail;
    /* replaced types (srtp_replace_cipher_type / _auth_type): the KDF's
     * AES-ICM and the RTP cipher / auth run through the registered vtables
     * on the host, as the reference allocates them from its crypto kernel */
    const int kdfr = cipher_routed(kdf_cipher_id(kdf_keylen));
    const int gcm_rtp = rtp->cipher_type == SRTP_AES_GCM_128 ||
                        rtp->cipher_type == SRTP_AES_GCM_256;
    const int rtpr = cipher_routed(rtp->cipher_type) ||
                     (!gcm_rtp && (rtp->sec_serv & sec_serv_auth) &&
                      auth_routed(rtp->auth_type)) ||
                     prefix_mode(rtp);
    if (rtpr && ((p->enc_xtn_hdr && p->enc_xtn_hdr_count > 0) ||
                 p->use_cryptex))
        return srtp_err_status_bad_param; /* not routed: refused, not faked */

    /* the PRF: AES keyed by the zero-padded master key, offset = the 14
     * bytes after it (srtp.c:1322-1340) */
    uint8_t tmp[256];
    memset(tmp, 0, sizeof tmp);
    memcpy(tmp, master, input_keylen);
    const size_t kdf_len = kdf_keylen - SRTP_SALT_LEN;
    const uint8_t *kdf_salt = tmp + kdf_len;

    srtp_dev_key_t dk;
    memset(&dk, 0, sizeof dk);
    hk->cipher_type = rtp->cipher_type;
    hk->tag_len = rtp->auth_tag_len;
    hk->num_left = 0xffffffffffffULL; /* srtp.c:1251 */
    hk->limit_state = 0;
    memset(hk->mki, 0, sizeof hk->mki);
    if (mki_size)
        memcpy(hk->mki, mki_id, mki_size);
    memcpy(dk.mki, hk->mki, sizeof dk.mki);
    dk.mki_size = (uint32_t)mki_size;
    dk.tag_len = (uint32_t)hk->tag_len;
    dk.conf = (rtp->sec_serv & sec_serv_conf) ? 1 : 0;

    int rc_code = 0;
    if (rtp->cipher_type == SRTP_NULL_CIPHER) {
        hk->family = SRTP_DEV_NULL;
        hk->rounds = 0;
        dk.conf = 0;
    } else {
        hk->rounds = (uint32_t)(base / 4 + 6);
        rc_code = ((int)hk->rounds - 8) / 2;
        if (rtp->cipher_type == SRTP_AES_GCM_128 ||
            rtp->cipher_type == SRTP_AES_GCM_256) {
            hk->family = SRTP_DEV_GCM;
            dk.conf = 1; /* AEAD always encrypts (srtp.c:2088-2098) */
        } else {
            hk->family = SRTP_DEV_ICM;
        }
    }
    dk.rounds = hk->rounds;
    dk.family = hk->family;
    int auth_on = rtp->auth_type == SRTP_HMAC_SHA1 &&
                  (rtp->sec_serv & sec_serv_auth) && hk->family != SRTP_DEV_GCM;
    dk.auth = (uint32_t)auth_on;
    hk->variant = hk->family == SRTP_DEV_GCM
                      ? SRTP_VARIANT(SRTP_DEV_GCM, rc_code, 0)
                      : SRTP_VARIANT(hk->family, hk->family ? rc_code : 0,
                                     auth_on);
    hk->slot = alloc_slot(ctx);
    dk.ghash_slot = hk->slot;

    /* RFC 6904 header-extension encryption and RFC 9335 cryptex
     * (srtp.c:694-749, 1385-1500): every packet of such a stream goes to
     * k_xrtp; the extension cipher is the RTP cipher's type, or AES-ICM of
     * the same size for AES-GCM */
    hk->xslot = 0xffffffffu;
    const int xtn = p->enc_xtn_hdr && p->enc_xtn_hdr_count > 0;
    if (xtn || p->use_cryptex) {
        hk->variant = SRTP_VARIANT_X;
        dk.xflags = (p->use_cryptex ? SRTP_XF_CRYPTEX : 0) |
                    ((rtp->sec_serv & sec_serv_conf) ? SRTP_XF_CONF : 0);
    }
    if (xtn) {
        for (size_t i = 0; i < p->enc_xtn_hdr_count; i++)
            dk.xids[p->enc_xtn_hdr[i] >> 5] |= 1u << (p->enc_xtn_hdr[i] & 31);
        dk.xflags |= SRTP_XF_XTN;
        hk->xslot = alloc_slot(ctx);
        dk.xslot = hk->xslot;
        srtp_dev_key_t xk;
        memset(&xk, 0, sizeof xk);
        xk.family = SRTP_DEV_NULL;
        xk.ghash_slot = hk->xslot;
        uint8_t tx[256];
        memset(tx, 0, sizeof tx);
        kspec_t q;
        memset(&q, 0, sizeof q);
        q.kk = tmp;
        q.ks = kdf_salt;
        q.kdf_len = kdf_len;
        q.vkdf = kdfr;
        q.vkdf_id = kdf_cipher_id(kdf_keylen);
        q.lab_enc = 0x06; /* label_rtp_header_encryption */
        q.lab_salt = 0x07; /* label_rtp_header_salt */
        if (hk->family != SRTP_DEV_NULL) {
            xk.family = SRTP_DEV_ICM;
            xk.rounds = hk->rounds;
            q.enc_len = base;
            q.salt_len = 14;
            if (hk->family == SRTP_DEV_GCM) {
                /* a PRF of its own over the master key and the 12-byte
                 * salt, zero padded (srtp.c:1393-1441); the ICM cipher then
                 * reads 14 salt bytes, the last two being what the key
                 * buffer holds there (srtp.c:1487) */
                memcpy(tx, master, base + salt_len);
                q.kk = tx;
                q.ks = tx + kdf_len;
                q.salt_len = salt_len;
                q.tail = 1;
                q.tail_b[0] = tmp[base + 12];
                q.tail_b[1] = tmp[base + 13];
            }
        }
        int bad = put_key(ctx, hk->xslot, &xk, &q);
        memset(tx, 0, sizeof tx);
        if (bad)
            return srtp_err_status_init_fail;
    }

    /* the RTP record: labels 0 (cipher key), 2 (salt), 1 (auth key) */
    {
        kspec_t q;
        memset(&q, 0, sizeof q);
        q.kk = tmp;
        q.ks = kdf_salt;
        q.kdf_len = kdf_len;
        q.vkdf = kdfr;
        q.vkdf_id = kdf_cipher_id(kdf_keylen);
        q.lab_enc = 0x00;
        q.lab_salt = 0x02;
        q.lab_auth = 0x01;
        q.enc_len = hk->family == SRTP_DEV_NULL ? 0 : base;
        /* the record keeps 14 salt bytes for ICM, 12 for GCM (the rest of
         * the PRF's salt output is not used) */
        q.salt_len = hk->family == SRTP_DEV_ICM ? 14
                     : hk->family == SRTP_DEV_GCM ? 12 : 0;
        q.hmac = rtp->auth_type == SRTP_HMAC_SHA1;
        q.auth_len = q.hmac ? rtp->auth_key_len : 0;
        q.ghash = hk->family == SRTP_DEV_GCM;
        q.gcm_h = q.ghash;
        uint8_t vek[32], vsa[16], vak[20];
        if (rtpr) {
            /* the salt the reference's cipher init reads: rtp_keylen - base
             * bytes (14 AES-ICM, 12 AES-GCM; srtp.c:1353-1370) */
            q.salt_len = salt_len < 14 ? salt_len : 14;
            q.raw_ek = vek;
            q.raw_sa = vsa;
            q.raw_ak = vak;
            memset(vsa, 0, sizeof vsa);
        }
        srtp_dev_key_t rk = dk;
        if (put_key(ctx, hk->slot, &rk, &q))
            return srtp_err_status_init_fail;
        if (rtpr) {
            hk->vmki = mki_size;
            int bad = route_key(ctx, hk, rtp, base, q.salt_len, vek, vsa, vak);
            memset(vek, 0, sizeof vek);
            memset(vak, 0, sizeof vak);
            if (bad)
                return srtp_err_status_init_fail;
        }
    }

    /* SRTCP key: srtp.c:1527-1600 (labels 3 encryption, 5 salt, 4 auth).
     * AEAD RTCP stays off the GPU path (srtp_protect_rtcp reports
     * no_such_op for it). */
    hk->rslot = 0xffffffffu;
    hk->rtag_len = rtcp->auth_tag_len;
    int rtcp_gcm = rtcp->cipher_type == SRTP_AES_GCM_128 ||
                   rtcp->cipher_type == SRTP_AES_GCM_256;
    hk->rgcm = rtcp_gcm;
    /* srtp.c:4380-4384 picks the AEAD path from the RTP cipher: the two
     * must agree here */
    /* replaced RTCP types are not routed: srtp_protect_rtcp then reports
     * no_such_op instead of running the built-in kernel */
    int rtcp_gpu = !cipher_routed(rtcp->cipher_type) &&
                   !auth_routed(rtcp->auth_type) && !prefix_mode(rtcp) &&
                   rtcp_gcm == (hk->family == SRTP_DEV_GCM) &&
                   cipher_supported(rtcp) &&
                   (rtcp->auth_type == SRTP_NULL_AUTH ||
                    rtcp->auth_type == SRTP_HMAC_SHA1) &&
                   auth_supported(rtcp);
    if (rtcp_gpu) {
        srtp_dev_key_t rk;
        memset(&rk, 0, sizeof rk);
        size_t rbase = base_key_length(rtcp->cipher_type, rtcp_keylen);
        memcpy(rk.mki, hk->mki, sizeof rk.mki);
        rk.mki_size = (uint32_t)mki_size;
        rk.tag_len = (uint32_t)rtcp->auth_tag_len;
        kspec_t q;
        memset(&q, 0, sizeof q);
        q.kk = tmp;
        q.ks = kdf_salt;
        q.kdf_len = kdf_len;
        q.vkdf = kdfr;
        q.vkdf_id = kdf_cipher_id(kdf_keylen);
        q.lab_enc = 0x03;
        q.lab_salt = 0x05;
        q.lab_auth = 0x04;
        if (rtcp->cipher_type == SRTP_NULL_CIPHER) {
            rk.family = SRTP_DEV_NULL;
        } else {
            if (rbase != 16 && rbase != 24 && rbase != 32)
                return srtp_err_status_init_fail;
            q.enc_len = rbase;
            q.salt_len = rtcp_keylen - rbase; /* 14 ICM, 12 GCM */
            if (q.salt_len > 14)
                q.salt_len = 14;
            rk.rounds = (uint32_t)(rbase / 4 + 6);
            rk.family = rtcp_gcm ? SRTP_DEV_GCM : SRTP_DEV_ICM;
            rk.conf = 1;
            q.gcm_h = rtcp_gcm;
        }
        if (rtcp->auth_type == SRTP_HMAC_SHA1 && !rtcp_gcm) {
            q.hmac = 1;
            q.auth_len = rtcp->auth_key_len;
            rk.auth = 1;
        }
        hk->rslot = alloc_slot(ctx);
        rk.ghash_slot = hk->rslot;
        if (put_key(ctx, hk->rslot, &rk, &q))
            return srtp_err_status_init_fail;
    }
    memset(tmp, 0, sizeof tmp);
    ctx->variant_mask |= 1u << hk->variant;
    return srtp_err_status_ok;
}

static void keyset_release(srtp_t ctx, keyset_t *ks)
{
    if (!ks || --ks->refs > 0)
        return;
    for (size_t i = 0; i < ks->n; i++) {
        if (ks->k[i].vc)
            srtp_cipher_dealloc(ks->k[i].vc);
        if (ks->k[i].va)
            srtp_auth_dealloc(ks->k[i].va);
        if (ks->k[i].variant == SRTP_VARIANT_V &&
            ks->k[i].slot < ctx->vkeys_cap)
            ctx->vkeys[ks->k[i].slot] = NULL;
        release_slot(ctx, ks->k[i].slot);
        if (ks->k[i].rslot != 0xffffffffu)
            release_slot(ctx, ks->k[i].rslot);
        if (ks->k[i].xslot != 0xffffffffu)
            release_slot(ctx, ks->k[i].xslot);
    }
    memset(ks, 0, sizeof *ks);
    free(ks);
}

static void stream_free(srtp_t ctx, srtp_stream_ctx_t *s)
{
    if (!s)
        return;
    keyset_release(ctx, s->keys);
    free(s->rdbx.w);
    free(s->spec.w);
    free(s);
}

/* srtp_valid_policy, srtp.c:554-592 + what this build supports */
static srtp_err_status_t valid_policy(const srtp_policy_t *p)
{
    if (!p)
        return srtp_err_status_bad_param;
    if (p->key == NULL) {
        if (p->num_master_keys <= 0 ||
            p->num_master_keys > SRTP_MAX_NUM_MASTER_KEYS)
            return srtp_err_status_bad_param;
        if (p->use_mki) {
            if (p->mki_size == 0 || p->mki_size > SRTP_MAX_MKI_LEN)
                return srtp_err_status_bad_param;
        } else if (p->mki_size != 0) {
            return srtp_err_status_bad_param;
        }
        for (size_t i = 0; i < p->num_master_keys; i++) {
            if (p->keys[i]->key == NULL)
                return srtp_err_status_bad_param;
            if (p->use_mki && p->keys[i]->mki_id == NULL)
                return srtp_err_status_bad_param;
        }
    } else if (p->use_mki || p->mki_size != 0) {
        return srtp_err_status_bad_param;
    }
    return srtp_err_status_ok;
}

static srtp_err_status_t stream_new(srtp_t ctx, const srtp_policy_t *p,
                                    srtp_stream_ctx_t **out)
{
    srtp_err_status_t st = valid_policy(p);
    if (st)
        return st;
    if (!cipher_supported(&p->rtp) || !auth_supported(&p->rtp))
        return srtp_err_status_bad_param;
    if (p->window_size != 0 &&
        (p->window_size < 64 || p->window_size >= 0x8000))
        return srtp_err_status_bad_param; /* srtp.c:1670-1672 */
    srtp_stream_ctx_t *s = (srtp_stream_ctx_t *)calloc(1, sizeof *s);
    if (!s)
        return srtp_err_status_alloc_fail;
    s->window_size = p->window_size ? p->window_size : 128;
    if (rdbx_init(&s->rdbx, s->window_size)) {
        free(s);
        return srtp_err_status_alloc_fail;
    }
    s->ssrc = p->ssrc.value;
    s->rtp_services = p->rtp.sec_serv;
    s->rtcp_services = p->rtcp.sec_serv;
    s->direction = DIR_UNKNOWN;
    s->allow_repeat_tx = p->allow_repeat_tx;
    keyset_t *ks = (keyset_t *)calloc(1, sizeof *ks);
    if (!ks) {
        stream_free(ctx, s);
        return srtp_err_status_alloc_fail;
    }
    ks->refs = 1;
    ks->cryptex = p->use_cryptex;
    for (size_t i = 0; i < SRTP_MAX_NUM_MASTER_KEYS; i++)
        ks->k[i].rslot = ks->k[i].xslot = 0xffffffffu;
    s->keys = ks;
    if (p->key) {
        s->use_mki = false;
        s->mki_size = 0;
        ks->n = 1;
        st = init_key(ctx, &ks->k[0], p, p->key, NULL, 0);
    } else {
        s->use_mki = p->use_mki;
        s->mki_size = p->use_mki ? p->mki_size : 0;
        ks->n = p->num_master_keys;
        for (size_t i = 0; i < ks->n && !st; i++)
            st = init_key(ctx, &ks->k[i], p, p->keys[i]->key,
                          p->keys[i]->mki_id, s->mki_size);
    }
    if (st) {
        stream_free(ctx, s);
        return st;
    }
    *out = s;
    return srtp_err_status_ok;
}

static srtp_stream_ctx_t *stream_clone(const srtp_stream_ctx_t *t, uint32_t ssrc)
{
    /* srtp_stream_clone, srtp.c:762-863 */
    srtp_stream_ctx_t *s = (srtp_stream_ctx_t *)calloc(1, sizeof *s);
    if (!s)
        return NULL;
    if (rdbx_init(&s->rdbx, t->rdbx.bits)) {
        free(s);
        return NULL;
    }
    s->ssrc = ssrc;
    s->direction = t->direction;
    s->rtp_services = t->rtp_services;
    s->rtcp_services = t->rtcp_services;
    s->allow_repeat_tx = t->allow_repeat_tx;
    s->use_mki = t->use_mki;
    s->mki_size = t->mki_size;
    s->window_size = t->window_size;
    s->keys = t->keys;
    s->keys->refs++;
    return s;
}

/* ------------------------------------------------------------------------
 * public API: lifecycle
 * ---------------------------------------------------------------------- */
static int g_inited;

srtp_err_status_t srtp_init(void)
{
    if (!srtp_gpu_available()) {
        log_msg(srtp_log_level_error,
                "libsrtp_mi355x: no HIP device available\n");
        return srtp_err_status_init_fail;
    }
    g_inited = 1;
    return srtp_err_status_ok;
}

srtp_err_status_t srtp_shutdown(void)
{
    g_inited = 0;
    return srtp_err_status_ok;
}

static srtp_err_status_t add_stream(srtp_t ctx, const srtp_policy_t *p)
{
    srtp_stream_ctx_t *s;
    srtp_err_status_t st = stream_new(ctx, p, &s);
    if (st)
        return st;
    switch (p->ssrc.type) {
    case ssrc_any_outbound:
    case ssrc_any_inbound:
        if (ctx->templ) {
            stream_free(ctx, s);
            return srtp_err_status_bad_param;
        }
        s->direction = p->ssrc.type == ssrc_any_outbound ? DIR_SENDER
                                                         : DIR_RECEIVER;
        ctx->templ = s;
        return srtp_err_status_ok;
    case ssrc_specific:
        if (list_insert(ctx, s)) {
            stream_free(ctx, s);
            return srtp_err_status_alloc_fail;
        }
        return srtp_err_status_ok;
    default:
        stream_free(ctx, s);
        return srtp_err_status_bad_param;
    }
}

static srtp_err_status_t stream_add_queued(srtp_t ctx, const srtp_policy_t *p)
{
    dev_pull(ctx);
    srtp_err_status_t st = valid_policy(p);
    if (st)
        return st;
    return add_stream(ctx, p);
}

srtp_err_status_t srtp_stream_add(srtp_t ctx, const srtp_policy_t *p)
{
    if (!ctx)
        return srtp_err_status_bad_param;
    srtp_err_status_t st = stream_add_queued(ctx, p);
    if (kq_flush(ctx) && !st)
        st = srtp_err_status_init_fail;
    return st;
}

srtp_err_status_t srtp_create(srtp_t *session, const srtp_policy_t *policy)
{
    if (!session)
        return srtp_err_status_bad_param;
    if (policy && valid_policy(policy))
        return srtp_err_status_bad_param;
    srtp_t ctx = (srtp_t)calloc(1, sizeof *ctx);
    if (!ctx)
        return srtp_err_status_alloc_fail;
    if (srtp_gpu_open(&ctx->gpu)) {
        log_msg(srtp_log_level_error, srtp_gpu_last_error());
        log_msg(srtp_log_level_error, "\n");
        free(ctx);
        *session = NULL;
        return srtp_err_status_init_fail;
    }
    map_rebuild(ctx, 64);
    {
        const char *e = getenv("SRTP_MI355X_HOST_KDF");
        ctx->host_kdf = e && e[0] == '1';
    }
    *session = ctx;
    /* every stream's session keys are derived in one k_kdf launch */
    for (const srtp_policy_t *p = policy; p; p = p->next) {
        srtp_err_status_t st = stream_add_queued(ctx, p);
        if (st) {
            srtp_dealloc(ctx);
            *session = NULL;
            return st;
        }
    }
    if (kq_flush(ctx)) {
        srtp_dealloc(ctx);
        *session = NULL;
        return srtp_err_status_init_fail;
    }
    return srtp_err_status_ok;
}

static void stage_free(stage_t *st)
{
    srtp_gpu_host_free(st->h_arena);
    srtp_gpu_free(st->d_arena);
    srtp_gpu_host_free(st->h_off);
    srtp_gpu_free(st->d_off);
    srtp_gpu_host_free(st->h_meta);
    srtp_gpu_free(st->d_meta);
    srtp_gpu_host_free(st->h_auth);
    srtp_gpu_free(st->d_auth);
    srtp_gpu_host_free(st->h_hdr);
    srtp_gpu_free(st->d_hdr);
    srtp_gpu_host_free(st->h_xinfo);
    srtp_gpu_free(st->d_xinfo);
    srtp_gpu_host_free(st->h_len);
    srtp_gpu_free(st->d_len);
    srtp_gpu_host_free(st->h_cap);
    srtp_gpu_free(st->d_cap);
    srtp_gpu_host_free(st->h_st);
    srtp_gpu_free(st->d_st);
    memset(st, 0, sizeof *st);
}

static void routed_reset(srtp_t ctx);

srtp_err_status_t srtp_dealloc(srtp_t ctx)
{
    if (!ctx)
        return srtp_err_status_bad_param;
    (void)async_drain(ctx);   /* an error is logged; freeing goes on */
    ctx->kq_n = 0; /* keys about to be freed need no derivation */
    for (size_t i = 0; i < ctx->n; i++)
        stream_free(ctx, ctx->list[i]);
    stream_free(ctx, ctx->templ);
    free(ctx->list);
    free(ctx->map.keys);
    free(ctx->map.vals);
    free(ctx->free_slots);
    stage_free(&ctx->st);
    free(ctx->dt.sv);
    free(ctx->dt.hs);
    free(ctx->dt.hwin);
    free(ctx->dt.pend);
    free(ctx->dt.res);
    free(ctx->kq);
    free(ctx->rel);
    routed_reset(ctx);
    free(ctx->vres);
    free(ctx->vsave);
    free(ctx->vkeys);
    srtp_gpu_close(ctx->gpu);
    free(ctx);
    return srtp_err_status_ok;
}

srtp_stream_ctx_t *srtp_get_stream(srtp_t ctx, uint32_t ssrc_net)
{
    uint32_t v = ((ssrc_net & 0xff) << 24) | ((ssrc_net & 0xff00) << 8) |
                 ((ssrc_net >> 8) & 0xff00) | (ssrc_net >> 24);
    if (!ctx)
        return NULL;
    dev_pull(ctx);
    return map_get(ctx, v);
}

srtp_err_status_t srtp_stream_remove(srtp_t ctx, uint32_t ssrc)
{
    if (!ctx)
        return srtp_err_status_bad_param;
    dev_pull(ctx);
    srtp_stream_ctx_t *s = map_get(ctx, ssrc);
    if (!s)
        return srtp_err_status_no_ctx;
    list_remove(ctx, s);
    stream_free(ctx, s);
    return srtp_err_status_ok;
}

static srtp_err_status_t update_specific(srtp_t ctx, const srtp_policy_t *p)
{
    /* stream_update, srtp.c:3568-3617 */
    srtp_stream_ctx_t *s = map_get(ctx, p->ssrc.value);
    if (!s)
        return srtp_err_status_bad_param;
    if (s->use_mki != p->use_mki || (s->use_mki && s->mki_size != p->mki_size))
        return srtp_err_status_bad_param;
    /* the extended sequence number and the SRTCP replay database survive
     * the update (srtp.c:3594-3614: old_index, old_rtcp_rdb) */
    /* the reference removes the stream and adds a new one; here the new
     * stream takes the old one's place (the list order is not observable),
     * so a rekey of n streams is O(n) and its keys derive in one launch */
    srtp_stream_ctx_t *ns;
    srtp_err_status_t st = stream_new(ctx, p, &ns);
    if (st)
        return st;
    ns->rdbx.index = s->rdbx.index;
    ns->rtcp_start = s->rtcp_start;
    memcpy(ns->rtcp_bm, s->rtcp_bm, sizeof ns->rtcp_bm);
    list_replace(ctx, s, ns);
    stream_free(ctx, s);
    return srtp_err_status_ok;
}

static srtp_err_status_t update_template(srtp_t ctx, const srtp_policy_t *p)
{
    /* update_template_streams, srtp.c:3430-3560 */
    if (!ctx->templ)
        return srtp_err_status_bad_param;
    if (ctx->templ->use_mki != p->use_mki ||
        (ctx->templ->use_mki && ctx->templ->mki_size != p->mki_size))
        return srtp_err_status_bad_param;
    srtp_stream_ctx_t *nt;
    srtp_err_status_t st = stream_new(ctx, p, &nt);
    if (st)
        return st;
    /* streams cloned from the old template are re-cloned, keeping their
     * extended sequence number; other streams are kept as they are */
    keyset_t *old = ctx->templ->keys;
    /* every clone is made before any stream is replaced: an allocation
     * failure leaves the session exactly as it was */
    srtp_stream_ctx_t **nc =
        (srtp_stream_ctx_t **)calloc(ctx->n ? ctx->n : 1, sizeof *nc);
    if (!nc) {
        stream_free(ctx, nt);
        return srtp_err_status_alloc_fail;
    }
    for (size_t i = 0; i < ctx->n; i++) {
        srtp_stream_ctx_t *s = ctx->list[i];
        if (s->keys != old)
            continue;
        nc[i] = stream_clone(nt, s->ssrc);
        if (!nc[i]) {
            for (size_t k = 0; k < i; k++)
                stream_free(ctx, nc[k]);
            free(nc);
            stream_free(ctx, nt);
            return srtp_err_status_alloc_fail;
        }
    }
    for (size_t i = 0; i < ctx->n; i++) {
        srtp_stream_ctx_t *s = ctx->list[i], *c = nc[i];
        if (!c)
            continue;
        /* srtp.c:3459-3483: extended sequence number and SRTCP replay
         * database carried over */
        c->rdbx.index = s->rdbx.index;
        c->rtcp_start = s->rtcp_start;
        memcpy(c->rtcp_bm, s->rtcp_bm, sizeof c->rtcp_bm);
        c->lpos = i;
        ctx->list[i] = c;
        stream_free(ctx, s);
    }
    free(nc);
    stream_free(ctx, ctx->templ);
    ctx->templ = nt; /* direction stays unknown, as srtp_stream_init leaves it */
    map_rebuild(ctx, ctx->map.cap ? ctx->map.cap : 64);
    return srtp_err_status_ok;
}

static srtp_err_status_t stream_update_queued(srtp_t ctx,
                                              const srtp_policy_t *p)
{
    dev_pull(ctx);
    srtp_err_status_t st = valid_policy(p);
    if (st)
        return st;
    switch (p->ssrc.type) {
    case ssrc_any_outbound:
    case ssrc_any_inbound:
        return update_template(ctx, p);
    case ssrc_specific:
        return update_specific(ctx, p);
    default:
        return srtp_err_status_bad_param;
    }
}

srtp_err_status_t srtp_stream_update(srtp_t ctx, const srtp_policy_t *p)
{
    if (!ctx)
        return srtp_err_status_bad_param;
    srtp_err_status_t st = stream_update_queued(ctx, p);
    if (kq_flush(ctx) && !st)
        st = srtp_err_status_init_fail;
    return st;
}

/* a rekey of every stream in the list: one k_kdf launch */
srtp_err_status_t srtp_update(srtp_t ctx, const srtp_policy_t *p)
{
    if (!ctx)
        return srtp_err_status_bad_param;
    srtp_err_status_t st = valid_policy(p);
    if (st)
        return st;
    for (; p && !st; p = p->next)
        st = stream_update_queued(ctx, p);
    if (kq_flush(ctx) && !st)
        st = srtp_err_status_init_fail;
    return st;
}

/* ------------------------------------------------------------------------
 * header summary (srtp_validate_rtp_header, srtp.c:307-336)
 * ---------------------------------------------------------------------- */
typedef struct {
    uint32_t ssrc;
    uint16_t seq;
    uint16_t err;
    uint32_t enc_start;
    uint32_t len;
    uint16_t profile;  /* extension profile (X set)                          */
    uint8_t cc, x;
    uint8_t inplace;   /* the caller's output buffer is its input buffer    */
} pkt_sum_t;

static void summarize(const uint8_t *p, size_t len, pkt_sum_t *s)
{
    s->len = (uint32_t)len;
    s->err = 0;
    s->ssrc = 0;
    s->seq = 0;
    s->enc_start = 0;
    s->profile = 0;
    s->cc = s->x = 0;
    s->inplace = 0;
    if (len < 12) {
        s->err = srtp_err_status_bad_param;
        return;
    }
    size_t h = 12 + 4 * (size_t)(p[0] & 0x0f);
    s->cc = p[0] & 0x0f;
    s->x = (p[0] >> 4) & 1;
    s->seq = (uint16_t)(p[2] << 8 | p[3]);
    s->ssrc = (uint32_t)p[8] << 24 | (uint32_t)p[9] << 16 |
              (uint32_t)p[10] << 8 | p[11];
    if (len < h) {
        s->err = srtp_err_status_bad_param;
        return;
    }
    if (p[0] & 0x10) {
        if (len < h + 4) {
            s->err = srtp_err_status_bad_param;
            return;
        }
        s->profile = (uint16_t)(p[h] << 8 | p[h + 1]);
        h += ((size_t)(p[h + 2] << 8 | p[h + 3]) + 1) * 4;
        if (len < h) {
            s->err = srtp_err_status_bad_param;
            return;
        }
    }
    s->enc_start = (uint32_t)h;
}

static void from_dev_hdr(const srtp_dev_hdr_t *d, uint32_t xinfo, pkt_sum_t *s)
{
    s->ssrc = d->ssrc;
    s->seq = (uint16_t)(d->seq_len & 0xffff);
    s->len = d->len;
    s->profile = (uint16_t)(xinfo & 0xffff);
    s->cc = (uint8_t)((xinfo >> 16) & 15);
    s->x = (uint8_t)((xinfo >> 20) & 1);
    s->inplace = 0;
    if (d->enc_start >> 24) {
        s->err = (uint16_t)(d->enc_start >> 24);
        s->enc_start = 0;
    } else {
        s->err = 0;
        s->enc_start = d->enc_start;
    }
}

/* ------------------------------------------------------------------------
 * protect pre-pass: srtp_protect / srtp_protect_aead up to the crypto
 * (srtp.c:2493-2712, 2088-2233).  Mutates stream state exactly as the
 * reference does; the GPU then performs the crypto of all OK packets.
 * ---------------------------------------------------------------------- */
static srtp_err_status_t pre_protect(srtp_t ctx, const pkt_sum_t *s,
                                     size_t cap, size_t mki_index,
                                     srtp_dev_meta_t *meta, size_t *out_len)
{
    if (s->err)
        return (srtp_err_status_t)s->err;
    srtp_stream_ctx_t *st = map_get(ctx, s->ssrc);
    if (!st) {
        if (!ctx->templ)
            return srtp_err_status_no_ctx;
        st = stream_clone(ctx->templ, s->ssrc);
        if (!st)
            return srtp_err_status_alloc_fail;
        if (list_insert(ctx, st)) {
            stream_free(ctx, st);
            return srtp_err_status_alloc_fail;
        }
        st->direction = DIR_SENDER;
    }
    if (st->direction != DIR_SENDER) {
        if (st->direction == DIR_UNKNOWN)
            st->direction = DIR_SENDER;
        else
            fire(ctx, st, event_ssrc_collision);
    }
    hkey_t *k;
    if (st->use_mki) {
        if (mki_index >= st->keys->n)
            return srtp_err_status_bad_mki;
        k = &st->keys->k[mki_index];
    } else {
        k = &st->keys->k[0];
    }
    int ev = key_limit_update(k);
    if (k->family == SRTP_DEV_GCM) {
        if (ev == 2) {
            fire(ctx, st, event_key_hard_limit);
            return srtp_err_status_key_expired;
        }
        if (ev == 1)
            fire(ctx, st, event_key_soft_limit);
    } else {
        if (ev == 1)
            fire(ctx, st, event_key_soft_limit);
        if (ev == 2) {
            fire(ctx, st, event_key_hard_limit);
            return srtp_err_status_key_expired;
        }
    }
    size_t tag_len = k->tag_len;
    if (cap < s->len + st->mki_size + tag_len)
        return srtp_err_status_buffer_small;
    uint32_t es = s->enc_start;
    const int xv = k->variant == SRTP_VARIANT_X;
    if (xv && st->keys->cryptex && (st->rtp_services & sec_serv_conf)) {
        /* srtp_cryptex_protect_init (srtp.c:163-193, 2151-2155) */
        if (s->cc && !s->x)
            return srtp_err_status_cryptex_err;
        if (s->x) {
            es = 12 + 4u * s->cc + 4 - (s->inplace ? 4u * s->cc : 0);
            if (k->family == SRTP_DEV_GCM && !s->inplace && s->cc)
                return srtp_err_status_cryptex_err;
        }
    }
    if (es > s->len)
        return srtp_err_status_parse_err;
    uint64_t est;
    int64_t delta;
    srtp_err_status_t rc = estimate(&st->rdbx, s->seq, &est, &delta);
    if (rc && rc != srtp_err_status_pkt_idx_adv)
        return rc;
    if (rc == srtp_err_status_pkt_idx_adv) {
        rdbx_accept(&st->rdbx, est, 0, 1);
    } else {
        rc = rdbx_check(&st->rdbx, delta);
        if (rc && (rc != srtp_err_status_replay_fail || !st->allow_repeat_tx))
            return rc;
        rdbx_add(&st->rdbx, delta);
    }
    if (k->family == SRTP_DEV_ICM && (st->rtp_services & sec_serv_conf)) {
        /* aes_icm.c:317-322: at most 0xffff keystream blocks */
        if ((s->len - es + 15) / 16 > 0xffff)
            return srtp_err_status_cipher_fail;
    }
    meta->key = k->slot;
    meta->roc = (uint32_t)(est >> 16);
    meta->info = (xv ? (s->inplace ? SRTP_XI_INPLACE : 0) : s->enc_start) |
                 (k->variant << 24);
    meta->len = s->len;
    *out_len = s->len + tag_len + st->mki_size;
    return srtp_err_status_ok;
}

/* ------------------------------------------------------------------------
 * unprotect pre-pass (speculative) and post-pass (exact, in order)
 * ---------------------------------------------------------------------- */
typedef struct {
    srtp_err_status_t sverdict; /* state-independent verdict (this round)  */
    uint64_t est;               /* index the crypto last ran at            */
    int gpu;                    /* the crypto has run (at est)             */
    int auth;                   /* ... and authenticated                   */
    int failed;                 /* authentication failed at some index     */
    int dirty;                  /* output = input ^ keystream of `dm`      */
    uint8_t xres;               /* k_xrtp result bits (SRTP_XR_*)          */
    hkey_t *key;                /* key of the last run                     */
    srtp_dev_meta_t dm;         /* meta of the last run                    */
} upkt_t;

/* how the pre-pass treats a packet whose crypto has not run at its
 * speculated index */
enum {
    UNP_OPTIMISTIC = 0, /* accepted, unless it already failed elsewhere */
    UNP_CAUTIOUS = 1,   /* not accepted                                  */
    UNP_EXACT = 2       /* runs alone: later packets of its SSRC wait     */
};
#define UNP_SPEC_ROUNDS 4

/* SSRC set with O(1) generation clear (redo / exact-round blocking) */
typedef struct {
    uint32_t *k, *gen_of;
    size_t cap;
    uint32_t gen;
} sset_t;

static int sset_init(sset_t *t, size_t n)
{
    t->cap = 16;
    while (t->cap < 2 * n)
        t->cap *= 2;
    t->k = (uint32_t *)malloc(t->cap * 4);
    t->gen_of = (uint32_t *)calloc(t->cap, 4);
    t->gen = 1;
    return t->k && t->gen_of ? 0 : -1;
}

static void sset_free(sset_t *t)
{
    free(t->k);
    free(t->gen_of);
}

static int sset_has(const sset_t *t, uint32_t x)
{
    for (size_t h = map_hash(x, t->cap); t->gen_of[h] == t->gen;
         h = (h + 1) & (t->cap - 1))
        if (t->k[h] == x)
            return 1;
    return 0;
}

static void sset_add(sset_t *t, uint32_t x)
{
    size_t h = map_hash(x, t->cap);
    for (; t->gen_of[h] == t->gen; h = (h + 1) & (t->cap - 1))
        if (t->k[h] == x)
            return;
    t->gen_of[h] = t->gen;
    t->k[h] = x;
}

/* per-batch provisional streams (unknown SSRC + template) */
typedef struct {
    uint32_t ssrc;
    rdbx_t r;
    int created; /* a speculative success created the stream */
} prov_t;

typedef struct {
    prov_t *v;
    size_t n, cap;
} provset_t;

static prov_t *prov_get(provset_t *ps, uint32_t ssrc, size_t win_bits)
{
    for (size_t i = 0; i < ps->n; i++)
        if (ps->v[i].ssrc == ssrc)
            return &ps->v[i];
    if (ps->n == ps->cap) {
        size_t nc = ps->cap ? 2 * ps->cap : 8;
        prov_t *p = (prov_t *)realloc(ps->v, nc * sizeof(prov_t));
        if (!p)
            return NULL;
        ps->v = p;
        ps->cap = nc;
    }
    prov_t *p = &ps->v[ps->n++];
    memset(p, 0, sizeof *p);
    p->ssrc = ssrc;
    rdbx_init(&p->r, win_bits);
    return p;
}

static void provset_free(provset_t *ps)
{
    for (size_t i = 0; i < ps->n; i++)
        free(ps->v[i].r.w);
    free(ps->v);
    memset(ps, 0, sizeof *ps);
}

static rdbx_t *spec_state(srtp_t ctx, srtp_stream_ctx_t *s)
{
    if (s->spec_epoch != ctx->epoch) {
        if (!s->spec.w)
            rdbx_init(&s->spec, s->rdbx.bits);
        rdbx_copy(&s->spec, &s->rdbx);
        s->spec_epoch = ctx->epoch;
    }
    return &s->spec;
}

/* MKI lookup by the packet trailer, srtp.c:1961-2016 */
static hkey_t *mki_lookup(const srtp_stream_ctx_t *st, const uint8_t *tail_mki)
{
    for (size_t i = 0; i < st->keys->n; i++)
        if (memcmp(tail_mki, st->keys->k[i].mki, st->mki_size) == 0)
            return &st->keys->k[i];
    return NULL;
}

/* state-independent checks after index estimation (srtp.c:2905-2990,
 * 2298-2352).  `mki` points at the packet's MKI bytes (or NULL). */
static srtp_err_status_t un_static(const srtp_stream_ctx_t *st,
                                   const pkt_sum_t *s, size_t cap,
                                   const uint8_t *mki_bytes, hkey_t **key,
                                   srtp_dev_meta_t *meta)
{
    hkey_t *k = &st->keys->k[0];
    if (st->use_mki) {
        size_t tl = k->family == SRTP_DEV_GCM ? 0 : k->tag_len;
        if (tl > s->len || st->mki_size > s->len - tl)
            return srtp_err_status_bad_mki;
        if (!mki_bytes)
            return srtp_err_status_bad_mki;
        k = mki_lookup(st, mki_bytes);
        if (!k)
            return srtp_err_status_bad_mki;
    }
    *key = k;
    size_t tag_len = k->tag_len;
    uint32_t es = s->enc_start;
    const int xv = k->variant == SRTP_VARIANT_X;
    if (xv && st->keys->cryptex && s->x &&
        (s->profile == 0xC0DE || s->profile == 0xC2DE)) {
        /* srtp_cryptex_unprotect_init (srtp.c:237-265, 2331-2335) */
        es = 12 + 4u * s->cc + 4 - (s->inplace ? 4u * s->cc : 0);
        if (k->family == SRTP_DEV_GCM && !s->inplace && s->cc)
            return srtp_err_status_cryptex_err;
    }
    if (s->len < tag_len + st->mki_size ||
        es > s->len - tag_len - st->mki_size)
        return srtp_err_status_parse_err;
    if (k->family == SRTP_DEV_GCM) {
        if (s->len - es - st->mki_size < tag_len)
            return srtp_err_status_cipher_fail;
    }
    if (cap < s->len - st->mki_size - tag_len)
        return srtp_err_status_buffer_small;
    meta->key = k->slot;
    meta->info = (xv ? (s->inplace ? SRTP_XI_INPLACE : 0) : s->enc_start) |
                 (k->variant << 24);
    meta->len = (uint32_t)(s->len - tag_len - st->mki_size);
    return srtp_err_status_ok;
}

/* speculative pre-pass for packet s; returns 1 if the GPU must run it.
 * `blk` holds the SSRCs an exact round has already given a packet to. */
static int pre_unprotect(srtp_t ctx, provset_t *ps, const pkt_sum_t *s,
                         size_t cap, const uint8_t *mki_bytes, upkt_t *u,
                         srtp_dev_meta_t *meta, int mode, sset_t *blk)
{
    if (s->err) {
        u->sverdict = (srtp_err_status_t)s->err;
        return 0;
    }
    /* (sverdict is state-independent: a value from an earlier round stays
     * valid; one never computed is 0 and makes the post-pass redo) */
    if (mode == UNP_EXACT && sset_has(blk, s->ssrc))
        return 0; /* waits for the earlier packet of its SSRC */
    srtp_stream_ctx_t *st = map_get(ctx, s->ssrc);
    rdbx_t *r = NULL;
    const srtp_stream_ctx_t *kst = st;
    uint64_t est;
    int64_t delta = 0;
    int adv = 0;
    prov_t *pv = NULL;
    if (!st) {
        if (!ctx->templ) {
            u->sverdict = srtp_err_status_no_ctx;
            return 0;
        }
        kst = ctx->templ;
        pv = prov_get(ps, s->ssrc, ctx->templ->rdbx.bits);
        if (!pv) {
            u->sverdict = srtp_err_status_alloc_fail;
            return 0;
        }
        if (pv->created) {
            r = &pv->r;
        } else {
            est = s->seq;
            delta = (int64_t)est;
        }
    } else {
        r = spec_state(ctx, st);
    }
    if (r) {
        srtp_err_status_t rc = estimate(r, s->seq, &est, &delta);
        if (rc && rc != srtp_err_status_pkt_idx_adv)
            return 0; /* speculatively old; the post-pass decides */
        adv = rc == srtp_err_status_pkt_idx_adv;
        if (!adv && rdbx_check(r, delta))
            return 0; /* speculatively a replay; the post-pass decides */
    }
    hkey_t *k = NULL;
    u->sverdict = un_static(kst, s, cap, mki_bytes, &k, meta);
    if (u->sverdict)
        return 0;
    meta->roc = (uint32_t)(est >> 16);
    const int known = u->gpu && u->est == est;
    int accept, run = 0;
    if (known) {
        /* result already in hand at this index */
        accept = u->auth && !(u->xres & SRTP_XR_PARSE);
    } else {
        run = 1;
        accept = mode == UNP_OPTIMISTIC && !u->failed;
        if (mode == UNP_EXACT)
            sset_add(blk, s->ssrc);
        u->est = est;
        u->key = k;
    }
    if (accept) {
        if (pv && !pv->created) {
            pv->created = 1;
            rdbx_add(&pv->r, delta);
        } else if (r) {
            rdbx_accept(r, est, delta, adv);
        }
    }
    return run;
}

/* exact post-pass for one packet, in batch order.  Returns the final status
 * or -1 when the packet must be re-run (its index changed). */
static int post_unprotect(srtp_t ctx, const pkt_sum_t *s, upkt_t *u,
                          size_t *out_len)
{
    const int auth_ok = u->auth;
    if (s->err)
        return s->err;
    srtp_stream_ctx_t *st = map_get(ctx, s->ssrc);
    uint64_t est;
    int64_t delta;
    int adv = 0;
    srtp_stream_ctx_t *kst = st;
    if (!st) {
        if (!ctx->templ)
            return srtp_err_status_no_ctx;
        kst = ctx->templ;
        est = s->seq;
        delta = (int64_t)est;
    } else {
        srtp_err_status_t rc = estimate(&st->rdbx, s->seq, &est, &delta);
        if (rc && rc != srtp_err_status_pkt_idx_adv)
            return rc;
        adv = rc == srtp_err_status_pkt_idx_adv;
        if (!adv) {
            rc = rdbx_check(&st->rdbx, delta);
            if (rc)
                return rc;
        }
    }
    if (u->sverdict)
        return u->sverdict;
    if (!u->gpu || u->est != est)
        return -1; /* speculation was wrong: run the crypto again */
    hkey_t *k = u->key;
    if (k->family == SRTP_DEV_GCM) {
        /* srtp_unprotect_aead: key limit before the tag check */
        int ev = key_limit_update(k);
        if (ev == 1)
            fire(ctx, kst, event_key_soft_limit);
        if (ev == 2) {
            fire(ctx, kst, event_key_hard_limit);
            return srtp_err_status_key_expired;
        }
        if (!auth_ok)
            return srtp_err_status_auth_fail;
    } else {
        if (!auth_ok)
            return srtp_err_status_auth_fail;
        int ev = key_limit_update(k);
        if (ev == 1)
            fire(ctx, kst, event_key_soft_limit);
        if (ev == 2) {
            fire(ctx, kst, event_key_hard_limit);
            return srtp_err_status_key_expired;
        }
    }
    /* header-extension walk failed after authentication (srtp.c:3073-3080,
     * 2409-2418): no index is added */
    if (u->xres & SRTP_XR_PARSE)
        return srtp_err_status_parse_err;
    if (kst->direction != DIR_RECEIVER) {
        if (kst->direction == DIR_UNKNOWN)
            kst->direction = DIR_RECEIVER;
        else
            fire(ctx, kst, event_ssrc_collision);
    }
    if (!st) {
        st = stream_clone(ctx->templ, s->ssrc);
        if (!st)
            return srtp_err_status_alloc_fail;
        if (list_insert(ctx, st)) {
            stream_free(ctx, st);
            return srtp_err_status_alloc_fail;
        }
    }
    rdbx_accept(&st->rdbx, est, delta, adv);
    *out_len = s->len - k->tag_len - st->mki_size;
    return srtp_err_status_ok;
}

/* ------------------------------------------------------------------------
 * staging (pinned host + device buffers, grown on demand)
 * ---------------------------------------------------------------------- */
static int stage_reserve(srtp_t ctx, size_t n, size_t arena)
{
    stage_t *st = &ctx->st;
    if (arena > st->arena_cap) {
        size_t c = st->arena_cap ? st->arena_cap : 1 << 16;
        while (c < arena)
            c *= 2;
        srtp_gpu_host_free(st->h_arena);
        srtp_gpu_free(st->d_arena);
        st->h_arena = (uint8_t *)srtp_gpu_host_alloc(c);
        st->d_arena = (uint8_t *)srtp_gpu_malloc(c);
        st->arena_cap = st->h_arena && st->d_arena ? c : 0;
        if (!st->arena_cap)
            return -1;
    }
    if (n > st->n_cap) {
        size_t c = st->n_cap ? st->n_cap : 256;
        while (c < n)
            c *= 2;
#define REALLOC_PAIR(h, d, T)                                                  \
    srtp_gpu_host_free(st->h);                                                 \
    srtp_gpu_free(st->d);                                                      \
    st->h = (T *)srtp_gpu_host_alloc(c * sizeof(T));                           \
    st->d = (T *)srtp_gpu_malloc(c * sizeof(T));                               \
    if (!st->h || !st->d)                                                      \
        return -1;
        REALLOC_PAIR(h_off, d_off, uint64_t)
        REALLOC_PAIR(h_meta, d_meta, srtp_dev_meta_t)
        REALLOC_PAIR(h_auth, d_auth, uint8_t)
        REALLOC_PAIR(h_hdr, d_hdr, srtp_dev_hdr_t)
        REALLOC_PAIR(h_xinfo, d_xinfo, uint32_t)
        REALLOC_PAIR(h_len, d_len, uint32_t)
        REALLOC_PAIR(h_cap, d_cap, uint32_t)
        REALLOC_PAIR(h_st, d_st, int32_t)
#undef REALLOC_PAIR
        st->n_cap = c;
    }
    return 0;
}

static uint32_t uniform_slot(const srtp_dev_meta_t *m, size_t n)
{
    uint32_t slot = 0xffffffffu;
    for (size_t i = 0; i < n; i++) {
        if (SRTP_META_STATUS(m[i].info))
            continue;
        if (slot == 0xffffffffu)
            slot = m[i].key;
        else if (slot != m[i].key)
            return 0xffffffffu;
    }
    return slot;
}

static uint32_t variants_of(const srtp_dev_meta_t *m, size_t n)
{
    uint32_t mask = 0;
    for (size_t i = 0; i < n; i++)
        if (!SRTP_META_STATUS(m[i].info))
            mask |= 1u << SRTP_META_VARIANT(m[i].info);
    return mask;
}

/* ------------------------------------------------------------------------
 * routed keys (SRTP_VARIANT_V): packet crypto through the registered
 * cipher / auth vtables, in the reference's call order
 * ---------------------------------------------------------------------- */
static void be32_put(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}

/* the IV of srtp.c:2694-2717 (AES-ICM: 0^4 || SSRC || be64(idx << 16);
 * any other non-AEAD cipher: 0^8 || be64(idx)) or srtp_calc_aead_iv
 * (srtp.c:1925-1959: (00 00 || SSRC || ROC || SEQ) ^ salt) */
static void vt_iv(const hkey_t *k, const uint8_t *pkt, uint32_t roc,
                  uint8_t iv[16])
{
    const uint32_t seq = (uint32_t)pkt[2] << 8 | pkt[3];
    const uint64_t idx = (uint64_t)roc << 16 | seq;
    memset(iv, 0, 16);
    if (k->family == SRTP_DEV_GCM) {
        memcpy(iv + 2, pkt + 8, 4);
        be32_put(iv + 6, roc);
        iv[10] = (uint8_t)(seq >> 8);
        iv[11] = (uint8_t)seq;
        for (int j = 0; j < 12; j++)
            iv[j] ^= k->vsalt[j];
        return;
    }
    const uint64_t w = (k->vcid == SRTP_AES_ICM_128 ||
                        k->vcid == SRTP_AES_ICM_192 ||
                        k->vcid == SRTP_AES_ICM_256)
                           ? idx << 16
                           : idx;
    if (k->vcid == SRTP_AES_ICM_128 || k->vcid == SRTP_AES_ICM_192 ||
        k->vcid == SRTP_AES_ICM_256)
        memcpy(iv + 4, pkt + 8, 4);
    for (int j = 0; j < 8; j++)
        iv[8 + j] = (uint8_t)(w >> (56 - 8 * j));
}

/* protect crypto of one packet in buf (L bytes in, room for the trailer):
 * srtp.c:2688-2818 (ICM / null) and 2188-2264 (AEAD); 0 or a status */
static srtp_err_status_t vt_protect(hkey_t *k, uint8_t *buf, size_t L,
                                    size_t es, uint32_t roc)
{
    uint8_t iv[16];
    vt_iv(k, buf, roc, iv);
    if (srtp_cipher_set_iv(k->vc, iv, srtp_direction_encrypt))
        return srtp_err_status_cipher_fail;
    if (k->family == SRTP_DEV_GCM) {
        size_t outlen = L - es + k->tag_len;
        if (srtp_cipher_set_aad(k->vc, buf, es) ||
            srtp_cipher_encrypt(k->vc, buf + es, L - es, buf + es, &outlen))
            return srtp_err_status_cipher_fail;
        memcpy(buf + es + outlen, k->mki, k->vmki);   /* MKI after the tag */
        return srtp_err_status_ok;
    }
    /* keystream prefix (srtp.c:2729-2741): into the tag, before the
     * payload's keystream */
    size_t pl = k->vauth ? srtp_auth_get_prefix_length(k->va) : 0;
    if (pl && srtp_cipher_output(k->vc, buf + L + k->vmki, &pl))
        return srtp_err_status_cipher_fail;
    if (k->vconf) {
        size_t len = L - es;
        if (srtp_cipher_encrypt(k->vc, buf + es, L - es, buf + es, &len))
            return srtp_err_status_cipher_fail;
    }
    memcpy(buf + L, k->mki, k->vmki);
    if (k->vauth) {
        uint8_t rb[4];
        be32_put(rb, roc);
        srtp_err_status_t st;
        if ((st = srtp_auth_start(k->va)) ||
            (st = srtp_auth_update(k->va, buf, L)) ||
            (st = srtp_auth_compute(k->va, rb, 4, buf + L + k->vmki)))
            return st;
    }
    return srtp_err_status_ok;
}

/* unprotect crypto of one packet (srtp_len bytes, L authenticated): the
 * tag check, then the decryption of an authenticated packet (srtp.c:
 * 2925-3101, 2352-2420); 1 when it authenticated */
static int vt_unprotect(hkey_t *k, uint8_t *buf, size_t srtp_len, size_t L,
                        size_t es, uint32_t roc)
{
    uint8_t iv[16];
    vt_iv(k, buf, roc, iv);
    if (srtp_cipher_set_iv(k->vc, iv, srtp_direction_decrypt))
        return 0;
    if (k->family == SRTP_DEV_GCM) {
        size_t enc = srtp_len - es - k->vmki;   /* ciphertext and tag */
        size_t outlen = enc;
        return !srtp_cipher_set_aad(k->vc, buf, es) &&
               !srtp_cipher_decrypt(k->vc, buf + es, enc, buf + es, &outlen);
    }
    if (k->vauth) {
        uint8_t rb[4], tag[SRTP_MAX_TAG_LEN];
        be32_put(rb, roc);
        /* keystream prefix (srtp.c:3006-3020): the expected tag */
        size_t pl = srtp_auth_get_prefix_length(k->va);
        if (pl && srtp_cipher_output(k->vc, tag, &pl))
            return 0;
        if (srtp_auth_start(k->va) || srtp_auth_update(k->va, buf, L) ||
            srtp_auth_compute(k->va, rb, 4, tag))
            return 0;
        /* constant time (datatypes.c:407 srtp_octet_string_equal) */
        uint8_t d = 0;
        for (size_t j = 0; j < k->tag_len; j++)
            d |= tag[j] ^ buf[srtp_len - k->tag_len + j];
        if (d)
            return 0;
    }
    if (k->vconf) {
        size_t len = L - es;
        if (srtp_cipher_decrypt(k->vc, buf + es, L - es, buf + es, &len))
            return 0;
    }
    return 1;
}

static void routed_reset(srtp_t ctx)
{
    for (size_t i = 0; i < ctx->vres_cap; i++) {
        free(ctx->vsave[i]);
        ctx->vsave[i] = NULL;
        ctx->vres[i] = 0;
    }
}

/* the routed packets of one crypto pass, their bytes copied from and back
 * to the device arenas.  Protect: ctx->vres[i] = the status of a packet
 * whose cipher / auth call failed (its output untouched).  Unprotect:
 * auth_ok[i] = the verdict; only an authenticated packet is decrypted, its
 * original bytes kept in ctx->vsave[i] for undo_runs.  The routed packets
 * move as one gather and one scatter (every copy queued, one synchronize
 * each way): the vtable calls themselves are the host's per-packet work. */
static int run_routed(srtp_t ctx, int op, size_t n, const uint8_t *in,
                      const uint64_t *in_off, uint8_t *out,
                      const uint64_t *out_off, const srtp_dev_meta_t *h_meta,
                      void *stream)
{
    /* no status of an earlier (possibly failed) pass may survive into this
     * one's routed_status */
    if (ctx->vres_cap)
        memset(ctx->vres, 0, n < ctx->vres_cap ? n : ctx->vres_cap);
    size_t nv = 0;
    for (size_t i = 0; i < n; i++)
        if (!SRTP_META_STATUS(h_meta[i].info) &&
            SRTP_META_VARIANT(h_meta[i].info) == SRTP_VARIANT_V)
            nv++;
    if (!nv)
        return 0;
    if (n > ctx->vres_cap) {
        routed_reset(ctx);
        free(ctx->vres);
        free(ctx->vsave);
        ctx->vres = (uint8_t *)calloc(n, 1);
        ctx->vsave = (uint8_t **)calloc(n, sizeof(uint8_t *));
        ctx->vres_cap = ctx->vres && ctx->vsave ? n : 0;
        if (!ctx->vres_cap)
            return -1;
    }
    uint64_t *io = (uint64_t *)malloc(n * 8), *oo = (uint64_t *)malloc(n * 8);
    size_t *list = (size_t *)malloc(nv * sizeof(size_t));
    size_t *pos = (size_t *)malloc(nv * sizeof(size_t));
    uint8_t *okv = (uint8_t *)calloc(nv, 1);
    uint8_t *buf = NULL;
    int rc = -1;
    if (!io || !oo || !list || !pos || !okv || srtp_gpu_sync(ctx->gpu, stream) ||
        srtp_gpu_d2h(ctx->gpu, io, in_off, n * 8, stream) ||
        srtp_gpu_d2h(ctx->gpu, oo, out_off, n * 8, stream) ||
        srtp_gpu_sync(ctx->gpu, stream))
        goto out;
    /* gather: each routed packet's bytes (protect: the RTP packet, unprotect:
     * packet + MKI + tag) into one host buffer with room for the trailer */
    size_t tot = 0, j = 0;
    for (size_t i = 0; i < n; i++) {
        const srtp_dev_meta_t m = h_meta[i];
        if (SRTP_META_STATUS(m.info) ||
            SRTP_META_VARIANT(m.info) != SRTP_VARIANT_V)
            continue;
        hkey_t *k = m.key < ctx->vkeys_cap ? ctx->vkeys[m.key] : NULL;
        if (!k || m.len > 65535)
            goto out;
        list[j] = i;
        pos[j++] = tot;
        tot += m.len + k->vmki + k->tag_len + SRTP_MAX_TRAILER_LEN;
    }
    buf = (uint8_t *)malloc(tot + 1);
    if (!buf)
        goto out;
    for (j = 0; j < nv; j++) {
        const size_t i = list[j];
        const hkey_t *k = ctx->vkeys[h_meta[i].key];
        const size_t L = h_meta[i].len;
        if (srtp_gpu_d2h(ctx->gpu, buf + pos[j], in + io[i],
                         op == 0 ? L : L + k->vmki + k->tag_len, stream))
            goto out;
    }
    if (srtp_gpu_sync(ctx->gpu, stream))
        goto out;
    /* the registered types' calls, then the scatter */
    for (j = 0; j < nv; j++) {
        const size_t i = list[j];
        const srtp_dev_meta_t m = h_meta[i];
        hkey_t *k = ctx->vkeys[m.key];
        uint8_t *b = buf + pos[j];
        const size_t L = m.len, es = SRTP_META_ENC_START(m.info);
        const size_t total = L + k->vmki + k->tag_len;
        if (op == 0) {
            srtp_err_status_t st = vt_protect(k, b, L, es, m.roc);
            ctx->vres[i] = (uint8_t)st;
            if (!st && srtp_gpu_h2d(ctx->gpu, out + oo[i], b, total, stream))
                goto out;
        } else {
            uint8_t *orig = (uint8_t *)malloc(L ? L : 1);
            if (!orig)
                goto out;
            memcpy(orig, b, L);
            okv[j] = (uint8_t)vt_unprotect(k, b, total, L, es, m.roc);
            if (srtp_gpu_h2d(ctx->gpu, ctx->st.d_auth + i, &okv[j], 1, stream) ||
                (okv[j] && srtp_gpu_h2d(ctx->gpu, out + oo[i], b, L, stream))) {
                free(orig);
                goto out;
            }
            free(ctx->vsave[i]);
            ctx->vsave[i] = okv[j] ? orig : NULL;
            if (!okv[j])
                free(orig);
        }
    }
    rc = 0;
out:
    /* the queued copies read buf / okv: both stay until the stream is past
     * them */
    if (srtp_gpu_sync(ctx->gpu, stream))
        rc = -1;
    free(io);
    free(oo);
    free(list);
    free(pos);
    free(okv);
    free(buf);
    return rc;
}

/* protect passes: statuses of routed packets whose crypto call failed */
static void routed_status(srtp_t ctx, size_t n, srtp_err_status_t *status)
{
    for (size_t i = 0; i < n && i < ctx->vres_cap; i++) {
        if (!status[i] && ctx->vres[i])
            status[i] = (srtp_err_status_t)ctx->vres[i];
        ctx->vres[i] = 0;
    }
}

static int run_gpu(srtp_t ctx, int op, size_t n, const uint8_t *in,
                   const uint64_t *in_off, uint8_t *out,
                   const uint64_t *out_off, const srtp_dev_meta_t *h_meta,
                   void *stream)
{
    srtp_gpu_batch_t b;
    memset(&b, 0, sizeof b);
    b.n = n;
    b.in = in;
    b.in_off = in_off;
    b.out = out;
    b.out_off = out_off;
    b.meta = ctx->st.d_meta;
    b.auth_ok = ctx->st.d_auth;
    b.uniform_key = uniform_slot(h_meta, n);
    b.mask = variants_of(h_meta, n) & ~(1u << SRTP_VARIANT_V);
    b.stream = stream;
    if (b.mask) {
        if (srtp_gpu_h2d(ctx->gpu, ctx->st.d_meta, h_meta,
                         n * sizeof *h_meta, stream))
            return -1;
        srtp_gpu_set_timing(ctx->gpu, ctx->timing);
        if (srtp_gpu_run(ctx->gpu, op, &b))
            return -1;
        if (ctx->timing)
            ctx->last_ms = srtp_gpu_last_kernel_ms(ctx->gpu);
    }
    return run_routed(ctx, op, n, in, in_off, out, out_off, h_meta, stream);
}

static size_t r16(size_t x) { return (x + 15) & ~(size_t)15; }


/* k_xrtp verdicts of a protect batch: a header-extension parse error
 * (srtp_process_header_encryption / srtp_cryptex_protect, srtp.c:2745-2762)
 * comes after the index was taken.  Syncs `stream`. */
static int xrtp_protect_results(srtp_t ctx, size_t n, srtp_err_status_t *status,
                                void *stream)
{
    stage_t *sg = &ctx->st;
    if (!(variants_of(sg->h_meta, n) & (1u << SRTP_VARIANT_X)))
        return 0;
    if (srtp_gpu_d2h(ctx->gpu, sg->h_auth, sg->d_auth, n, stream) ||
        srtp_gpu_sync(ctx->gpu, stream))
        return -1;
    for (size_t i = 0; i < n; i++)
        if (!status[i] &&
            SRTP_META_VARIANT(sg->h_meta[i].info) == SRTP_VARIANT_X &&
            (sg->h_auth[i] & SRTP_XR_PARSE))
            status[i] = srtp_err_status_parse_err;
    return 0;
}

/* ------------------------------------------------------------------------
 * batch API over host buffers
 * ---------------------------------------------------------------------- */
static int protect_device_fast(srtp_t ctx, const srtp_device_batch_t *b,
                               int async, const size_t *mki_wide);
static int unprotect_device_fast(srtp_t ctx, const srtp_device_batch_t *b);

/* a parallel for over [0, n) on up to 8 host threads: the gather into and
 * scatter out of the pinned staging arena of host-buffer batches */
typedef struct {
    void (*fn)(void *arg, size_t lo, size_t hi);
    void *arg;
    size_t lo, hi;
} par_job_t;

static void *par_run(void *p)
{
    par_job_t *j = (par_job_t *)p;
    j->fn(j->arg, j->lo, j->hi);
    return NULL;
}

static void par_for_range(size_t lo, size_t hi,
                          void (*fn)(void *, size_t, size_t), void *arg);
#define STAGE_CHUNKS 8   /* < SRTP_GPU_MARKS */

/* fn over [lo, hi) on up to PAR_THREADS host threads (the GPU box grants
 * 16 CPUs per GPU) */
#define PAR_THREADS 16
static void par_for_range(size_t lo0, size_t hi0,
                          void (*fn)(void *, size_t, size_t), void *arg)
{
    const size_t n = hi0 - lo0;
    size_t t = n / 16384;
    if (t > PAR_THREADS)
        t = PAR_THREADS;
    if (t < 2) {
        fn(arg, lo0, hi0);
        return;
    }
    pthread_t th[PAR_THREADS];
    par_job_t jobs[PAR_THREADS];
    size_t started = 0;
    for (size_t k = 0; k < t; k++) {
        jobs[k].fn = fn;
        jobs[k].arg = arg;
        jobs[k].lo = lo0 + n * k / t;
        jobs[k].hi = lo0 + n * (k + 1) / t;
        if (k > 0 && pthread_create(&th[k], NULL, par_run, &jobs[k]) == 0)
            started |= (size_t)1 << k;
        else if (k > 0)
            fn(arg, jobs[k].lo, jobs[k].hi);   /* no thread: inline */
    }
    fn(arg, jobs[0].lo, jobs[0].hi);
    for (size_t k = 1; k < t; k++)
        if (started & ((size_t)1 << k))
            pthread_join(th[k], NULL);
}

typedef struct {
    stage_t *sg;
    const uint8_t *const *in;
    const size_t *in_len;
    uint8_t *const *out;
    size_t *out_len;
    const srtp_err_status_t *status;
    size_t extra; /* slot room after the input: protect's trailer */
} gather_t;

static void gather_part(void *p, size_t lo, size_t hi)
{
    gather_t *g = (gather_t *)p;
    for (size_t i = lo; i < hi; i++)
        memcpy(g->sg->h_arena + g->sg->h_off[i], g->in[i], g->in_len[i]);
}

static void scatter_part(void *p, size_t lo, size_t hi)
{
    gather_t *g = (gather_t *)p;
    for (size_t i = lo; i < hi; i++)
        if (g->sg->h_st[i] == 0) {
            memcpy(g->out[i], g->sg->h_arena + g->sg->h_off[i],
                   g->sg->h_cap[i]);
            g->out_len[i] = g->sg->h_cap[i];
        }
}

/* Host-buffer batch on the device pre-pass: gather into the pinned arena,
 * one H2D, srtp_{un}protect_device's GPU pre-pass + kernels, one D2H,
 * scatter.  Returns 1 when done, 0 when the batch must take the host
 * pre-pass path (nothing was changed), -1 on a device error. */
static int batch_device_fast(srtp_t ctx, int unprotect, size_t n,
                             const uint8_t *const *in, const size_t *in_len,
                             uint8_t *const *out, size_t *out_len,
                             const size_t *mki_index,
                             srtp_err_status_t *status)
{
    if (n < 64 || n > 0x7fffffffu)
        return 0;   /* small batches: the host path has less overhead */
    const size_t extra = unprotect ? 0 : SRTP_MAX_TRAILER_LEN;
    size_t arena = 0;
    for (size_t i = 0; i < n; i++) {
        if (in_len[i] > 0xffff || out_len[i] > 0xffffffffu)
            return 0;
        arena += r16(in_len[i] + extra);
    }
    if (stage_reserve(ctx, n, arena))
        return -1;
    stage_t *sg = &ctx->st;
    size_t off = 0;
    for (size_t i = 0; i < n; i++) {
        sg->h_off[i] = off;
        sg->h_len[i] = (uint32_t)in_len[i];
        sg->h_cap[i] = (uint32_t)out_len[i];
        off += r16(in_len[i] + extra);
    }
    gather_t g = { sg, in, in_len, out, out_len, status, extra };
    void *hs = HS(ctx);
    /* the gather of chunk c+1 on the host threads overlaps the copy of
     * chunk c (the arena is pinned: the copies are asynchronous) */
    const size_t nck = n >= 65536 ? STAGE_CHUNKS : 1;
    if (srtp_gpu_h2d(ctx->gpu, sg->d_off, sg->h_off, n * 8, hs) ||
        srtp_gpu_h2d(ctx->gpu, sg->d_len, sg->h_len, n * 4, hs) ||
        srtp_gpu_h2d(ctx->gpu, sg->d_cap, sg->h_cap, n * 4, hs))
        return -1;
    for (size_t c = 0; c < nck; c++) {
        const size_t lo = n * c / nck, hi = n * (c + 1) / nck;
        const size_t b0 = sg->h_off[lo], b1 = hi < n ? sg->h_off[hi] : off;
        par_for_range(lo, hi, gather_part, &g);
        if (srtp_gpu_h2d(ctx->gpu, sg->d_arena + b0, sg->h_arena + b0,
                         b1 - b0, hs))
            return -1;
    }
    srtp_device_batch_t b;
    memset(&b, 0, sizeof b);
    b.n = n;
    b.in = sg->d_arena;
    b.in_off = sg->d_off;
    b.in_len = sg->d_len;
    b.out = sg->d_arena;
    b.out_off = sg->d_off;
    b.out_len = sg->d_cap;
    b.status = sg->d_st;
    b.stream = hs;
    if (async_drain(ctx))   /* staged on the library's own stream */
        return -1;
    int fast = unprotect ? unprotect_device_fast(ctx, &b)
                         : protect_device_fast(ctx, &b, 0, mki_index);
    if (fast <= 0)
        return fast;
    ctx->dt.fast_batches++;
    /* statuses and lengths first, then the arena chunk by chunk: the
     * scatter of chunk c overlaps the copy of chunk c+1 */
    if (srtp_gpu_d2h(ctx->gpu, sg->h_cap, sg->d_cap, n * 4, hs) ||
        srtp_gpu_d2h(ctx->gpu, sg->h_st, sg->d_st, n * 4, hs) ||
        srtp_gpu_mark(ctx->gpu, 0, hs))
        return -1;
    for (size_t c = 0; c < nck; c++) {
        const size_t lo = n * c / nck, hi = n * (c + 1) / nck;
        const size_t b0 = sg->h_off[lo], b1 = hi < n ? sg->h_off[hi] : off;
        if (srtp_gpu_d2h(ctx->gpu, sg->h_arena + b0, sg->d_arena + b0,
                         b1 - b0, hs) ||
            srtp_gpu_mark(ctx->gpu, (int)c + 1, hs))
            return -1;
    }
    if (srtp_gpu_mark_wait(ctx->gpu, 0))
        return -1;
    for (size_t c = 0; c < nck; c++) {
        const size_t lo = n * c / nck, hi = n * (c + 1) / nck;
        if (srtp_gpu_mark_wait(ctx->gpu, (int)c + 1))
            return -1;
        par_for_range(lo, hi, scatter_part, &g);
    }
    for (size_t i = 0; i < n; i++)
        status[i] = (srtp_err_status_t)sg->h_st[i];
    return 1;
}

/* Large host-buffer batches: STAGE_CHUNKS consecutive device batches (the
 * reference's sequential semantics: chunk c's pre-pass runs on the state
 * chunk c-1 committed) with the copies on two copy streams, so that the
 * host threads gather chunk c+1 and scatter chunk c-1 while chunk c+1
 * goes to HBM and chunk c comes back (PCIe both ways at once).  *done
 * receives the packets completed, a prefix of whole chunks; when a chunk
 * is declined by the device pre-pass the pipeline drains and the caller
 * runs the rest on the host path.  Returns 1 when all n are done, 0
 * otherwise (see *done), -1 on a device error. */
#define PIPE_MIN (1u << 17)
static int batch_device_pipelined(srtp_t ctx, int unprotect, size_t n,
                                  const uint8_t *const *in,
                                  const size_t *in_len, uint8_t *const *out,
                                  size_t *out_len, const size_t *mki_index,
                                  srtp_err_status_t *status, size_t *done)
{
    *done = 0;
    const size_t extra = unprotect ? 0 : SRTP_MAX_TRAILER_LEN;
    size_t arena = 0;
    for (size_t i = 0; i < n; i++) {
        if (in_len[i] > 0xffff || out_len[i] > 0xffffffffu)
            return 0;
        arena += r16(in_len[i] + extra);
    }
    void *cin = srtp_gpu_aux_stream(ctx->gpu, 0);
    void *cout = srtp_gpu_aux_stream(ctx->gpu, 1);
    if (!cin || !cout)
        return 0;
    if (async_drain(ctx) || stage_reserve(ctx, n, arena))
        goto fail;
    stage_t *sg = &ctx->st;
    size_t off = 0;
    for (size_t i = 0; i < n; i++) {
        sg->h_off[i] = off;
        sg->h_len[i] = (uint32_t)in_len[i];
        sg->h_cap[i] = (uint32_t)out_len[i];
        off += r16(in_len[i] + extra);
    }
    gather_t g = { sg, in, in_len, out, out_len, status, extra };
    void *hs = HS(ctx);
    const size_t nck = STAGE_CHUNKS;
    size_t lo[STAGE_CHUNKS + 1];
    for (size_t c = 0; c <= nck; c++)
        lo[c] = n * c / nck;
#define CK_B0(c) (sg->h_off[lo[c]])
#define CK_B1(c) (lo[(c) + 1] < n ? sg->h_off[lo[(c) + 1]] : off)
    /* marks: 0..7 chunk c in HBM, 8..15 chunk c back in host memory */
    if (srtp_gpu_h2d(ctx->gpu, sg->d_off, sg->h_off, n * 8, cin) ||
        srtp_gpu_h2d(ctx->gpu, sg->d_len, sg->h_len, n * 4, cin) ||
        srtp_gpu_h2d(ctx->gpu, sg->d_cap, sg->h_cap, n * 4, cin))
        goto fail;
    par_for_range(lo[0], lo[1], gather_part, &g);
    if (srtp_gpu_h2d(ctx->gpu, sg->d_arena + CK_B0(0), sg->h_arena + CK_B0(0),
                     CK_B1(0) - CK_B0(0), cin) ||
        srtp_gpu_mark(ctx->gpu, 0, cin))
        goto fail;
    int rc = 1;
    size_t c = 0;
    for (; c < nck; c++) {
        if (c + 1 < nck) {
            par_for_range(lo[c + 1], lo[c + 2], gather_part, &g);
            if (srtp_gpu_h2d(ctx->gpu, sg->d_arena + CK_B0(c + 1),
                             sg->h_arena + CK_B0(c + 1),
                             CK_B1(c + 1) - CK_B0(c + 1), cin) ||
                srtp_gpu_mark(ctx->gpu, (int)c + 1, cin))
                goto fail;
        }
        const size_t a = lo[c], k = lo[c + 1] - lo[c];
        srtp_device_batch_t b;
        memset(&b, 0, sizeof b);
        b.n = k;
        b.in = sg->d_arena;
        b.in_off = sg->d_off + a;
        b.in_len = sg->d_len + a;
        b.out = sg->d_arena;
        b.out_off = sg->d_off + a;
        b.out_len = sg->d_cap + a;
        b.status = sg->d_st + a;
        b.stream = hs;
        if (srtp_gpu_mark_stream_wait(ctx->gpu, hs, (int)c))
            goto fail;
        const int fast = unprotect
            ? unprotect_device_fast(ctx, &b)
            : protect_device_fast(ctx, &b, 0, mki_index ? mki_index + a : NULL);
        if (fast < 0)
            goto fail;
        if (!fast) {
            rc = 0;
            break;
        }
        ctx->dt.fast_batches++;
        /* chunk c is complete on the compute stream (the synchronous
         * pre-pass waited for it): back to host memory on the other copy
         * stream */
        if (srtp_gpu_d2h(ctx->gpu, sg->h_cap + a, sg->d_cap + a, k * 4, cout) ||
            srtp_gpu_d2h(ctx->gpu, sg->h_st + a, sg->d_st + a, k * 4, cout) ||
            srtp_gpu_d2h(ctx->gpu, sg->h_arena + CK_B0(c),
                         sg->d_arena + CK_B0(c), CK_B1(c) - CK_B0(c), cout) ||
            srtp_gpu_mark(ctx->gpu, 8 + (int)c, cout))
            goto fail;
        if (c > 0) {
            if (srtp_gpu_mark_wait(ctx->gpu, 8 + (int)c - 1))
                goto fail;
            par_for_range(lo[c - 1], lo[c], scatter_part, &g);
        }
    }
    /* the last chunk that went through (c - 1), and whatever copy is still
     * in flight before the staging buffers are used again */
    if (c > 0) {
        if (srtp_gpu_mark_wait(ctx->gpu, 8 + (int)c - 1))
            goto fail;
        par_for_range(lo[c - 1], lo[c], scatter_part, &g);
    }
    if (srtp_gpu_sync(ctx->gpu, cin) || srtp_gpu_sync(ctx->gpu, cout))
        goto fail;
    for (size_t i = 0; i < lo[c]; i++)
        status[i] = (srtp_err_status_t)sg->h_st[i];
    *done = lo[c];
#undef CK_B0
#undef CK_B1
    return rc;
fail:
    /* no copy on either copy stream, nor a kernel reading the staging
     * arena, may outlive the call: the next batch reuses the buffers */
    (void)srtp_gpu_sync(ctx->gpu, cin);
    (void)srtp_gpu_sync(ctx->gpu, cout);
    (void)srtp_gpu_sync(ctx->gpu, HS(ctx));
    return -1;
}

/* the device paths of a host-buffer batch: pipelined chunks for large ones */
static int batch_device_run(srtp_t ctx, int unprotect, size_t n,
                            const uint8_t *const *in, const size_t *in_len,
                            uint8_t *const *out, size_t *out_len,
                            const size_t *mki_index,
                            srtp_err_status_t *status, size_t *done)
{
    *done = 0;
    if (n >= PIPE_MIN && n <= 0x7fffffffu)
        return batch_device_pipelined(ctx, unprotect, n, in, in_len, out,
                                      out_len, mki_index, status, done);
    const int fast = batch_device_fast(ctx, unprotect, n, in, in_len, out,
                                       out_len, mki_index, status);
    if (fast > 0)
        *done = n;
    return fast;
}

/* ------------------------------------------------------------------------
 * the per-call path: ONE packet, the host pre-pass's descriptor, the crypto
 * by one workgroup straight from a pinned copy (srtp_one.hip k_one) -- an
 * unchanged libsrtp caller's srtp_protect / srtp_unprotect per packet
 * ---------------------------------------------------------------------- */
static int one_fits(const srtp_dev_meta_t *m, size_t len)
{
    return SRTP_META_VARIANT(m->info) < SRTP_VARIANT_X &&
           len + SRTP_ONE_TRAILER <= SRTP_ONE_MAX &&
           m->len + SRTP_ONE_TRAILER <= SRTP_ONE_MAX;
}

/* the tag's verdict (protect: 1), -1 on a device error.  Protect: the
 * protected packet (out_len bytes) to `out`; unprotect leaves the plaintext
 * in the staging buffer (srtp_gpu_one_buf) for the caller to take once the
 * post-pass accepted it -- a rejected packet's buffer is never written. */
static int one_run(srtp_t ctx, int op, const uint8_t *in, size_t len,
                   const srtp_dev_meta_t *m, uint8_t *out, size_t out_len)
{
    uint8_t *ob = srtp_gpu_one_buf(ctx->gpu);
    if (!ob)
        return -1;
    memcpy(ob, in, len);
    int ok = 0;
    srtp_gpu_set_timing(ctx->gpu, 0);
    if (srtp_gpu_one(ctx->gpu, op, (uint32_t)len, m, HS(ctx), &ok))
        return -1;
    if (op == 0)
        memcpy(out, ob, out_len);
    return ok;
}

/* srtp_unprotect of one packet (unprotect_core for n = 1: the speculative
 * pre-pass, the crypto, the exact post-pass); 1 done, 0 not this path (a
 * header-extension / routed stream, a packet too large), -1 device error */
static int one_unprotect(srtp_t ctx, const uint8_t *srtp, size_t srtp_len,
                         uint8_t *rtp, size_t *rtp_len,
                         srtp_err_status_t *status)
{
    if (srtp_len + SRTP_ONE_TRAILER > SRTP_ONE_MAX)
        return 0;
    pkt_sum_t s;
    summarize(srtp, srtp_len, &s);
    s.inplace = srtp == rtp;
    const srtp_stream_ctx_t *st = s.err ? NULL : map_get(ctx, s.ssrc);
    if (!st)
        st = ctx->templ;
    const uint8_t *mki = NULL;
    if (st) {
        if (st->keys->k[0].variant >= SRTP_VARIANT_X)
            return 0;
        const hkey_t *k0 = &st->keys->k[0];
        const size_t tl = k0->family == SRTP_DEV_GCM ? 0 : k0->tag_len;
        if (st->use_mki && tl <= srtp_len && st->mki_size <= srtp_len - tl)
            mki = srtp + srtp_len - tl - st->mki_size;
    }
    sset_t blk;
    if (sset_init(&blk, 1)) {
        sset_free(&blk);
        return -1;
    }
    provset_t ps;
    memset(&ps, 0, sizeof ps);
    upkt_t u;
    memset(&u, 0, sizeof u);
    srtp_dev_meta_t m;
    memset(&m, 0, sizeof m);
    memset(&ctx->ustat, 0, sizeof ctx->ustat);
    ctx->epoch++;
    blk.gen++;
    const int run = pre_unprotect(ctx, &ps, &s, *rtp_len, mki, &u, &m,
                                  UNP_OPTIMISTIC, &blk);
    provset_free(&ps);
    sset_free(&blk);
    ctx->ustat.rounds = 1;
    size_t olen = 0;
    if (run) {
        ctx->ustat.launches = 1;
        const int ok = one_run(ctx, 1, srtp, srtp_len, &m, NULL, 0);
        if (ok < 0)
            return -1;
        u.gpu = 1;
        u.auth = ok;
        u.failed = !ok;
        u.dirty = 0;   /* nothing reached rtp unless it authenticated */
        u.dm = m;
    }
    const int rc = post_unprotect(ctx, &s, &u, &olen);
    if (rc < 0)
        return 0;   /* (not for one packet) nothing committed: the batch path */
    if (rc == 0) {   /* accepted: the plaintext from the staging buffer */
        memcpy(rtp, srtp_gpu_one_buf(ctx->gpu), olen);
        *rtp_len = olen;
    }
    *status = (srtp_err_status_t)rc;
    return 1;
}

srtp_err_status_t srtp_protect_batch(srtp_t ctx, size_t n,
                                     const uint8_t *const *rtp,
                                     const size_t *rtp_len,
                                     uint8_t *const *srtp, size_t *srtp_len,
                                     const size_t *mki_index,
                                     srtp_err_status_t *status)
{
    if (!ctx)
        return srtp_err_status_bad_param;
    ASYNC_DRAIN_CHECK(ctx);
    if (!n)
        return srtp_err_status_ok;
    {
        /* MKI: each packet's mki_index picks its key on the device
         * (protect_device_fast, dev_mki_index) */
        size_t done = 0;
        int fast = batch_device_run(ctx, 0, n, rtp, rtp_len, srtp, srtp_len,
                                    mki_index, status, &done);
        if (fast < 0) {
            log_msg(srtp_log_level_error, srtp_gpu_last_error());
            return srtp_err_status_fail;
        }
        if (fast)
            return srtp_err_status_ok;
        /* a declined chunk: the rest on the host path */
        n -= done;
        rtp += done;
        rtp_len += done;
        srtp += done;
        srtp_len += done;
        status += done;
        if (mki_index)
            mki_index += done;
    }
    dev_pull(ctx);
    size_t arena = 0;
    for (size_t i = 0; i < n; i++)
        arena += r16(rtp_len[i] + SRTP_MAX_TRAILER_LEN);
    if (stage_reserve(ctx, n, arena))
        return srtp_err_status_alloc_fail;
    stage_t *sg = &ctx->st;
    size_t *olen = (size_t *)malloc(n * sizeof(size_t));
    if (!olen)
        return srtp_err_status_alloc_fail;
    size_t off = 0;
    for (size_t i = 0; i < n; i++) {
        pkt_sum_t s;
        summarize(rtp[i], rtp_len[i], &s);
        s.inplace = rtp[i] == srtp[i];
        srtp_dev_meta_t *m = &sg->h_meta[i];
        memset(m, 0, sizeof *m);
        sg->h_off[i] = off;
        olen[i] = 0;
        status[i] = pre_protect(ctx, &s, srtp_len[i],
                                mki_index ? mki_index[i] : 0, m, &olen[i]);
        if (status[i]) {
            m->info = (uint32_t)(status[i] & 0xff) << 16;
        } else {
            memcpy(sg->h_arena + off, rtp[i], rtp_len[i]);
        }
        off += r16(rtp_len[i] + SRTP_MAX_TRAILER_LEN);
    }
    srtp_err_status_t ret = srtp_err_status_ok;
    if (n == 1 && status[0]) {   /* one packet, rejected by the pre-pass */
        free(olen);
        return ret;
    }
    if (n == 1 && one_fits(&sg->h_meta[0], rtp_len[0])) {
        /* one packet (srtp_protect): the per-call kernel on a pinned copy */
        const int r = one_run(ctx, 0, rtp[0], rtp_len[0], &sg->h_meta[0],
                              srtp[0], olen[0]);
        if (r < 0) {
            log_msg(srtp_log_level_error, srtp_gpu_last_error());
            status[0] = srtp_err_status_cipher_fail;
            ret = srtp_err_status_fail;
        } else {
            srtp_len[0] = olen[0];
        }
        free(olen);
        return ret;
    }
    if (srtp_gpu_h2d(ctx->gpu, sg->d_arena, sg->h_arena, off, HS(ctx)) ||
        srtp_gpu_h2d(ctx->gpu, sg->d_off, sg->h_off, n * 8, HS(ctx)) ||
        run_gpu(ctx, 0, n, sg->d_arena, sg->d_off, sg->d_arena, sg->d_off,
                sg->h_meta, HS(ctx)) ||
        srtp_gpu_d2h(ctx->gpu, sg->h_arena, sg->d_arena, off, HS(ctx)) ||
        srtp_gpu_sync(ctx->gpu, HS(ctx)) ||
        xrtp_protect_results(ctx, n, status, HS(ctx))) {
        log_msg(srtp_log_level_error, srtp_gpu_last_error());
        ret = srtp_err_status_fail;
    } else {
        routed_status(ctx, n, status);
    }
    for (size_t i = 0; i < n; i++) {
        if (ret) {
            status[i] = srtp_err_status_cipher_fail;
            continue;
        }
        if (status[i])
            continue;
        memcpy(srtp[i], sg->h_arena + sg->h_off[i], olen[i]);
        srtp_len[i] = olen[i];
    }
    free(olen);
    return ret;
}

/* XORs the keystream of each flagged packet's last run back over its
 * output (CTR: that restores the ciphertext); routed packets get the bytes
 * run_routed() kept */
static int undo_runs(srtp_t ctx, size_t n, const size_t *list, size_t nl,
                     upkt_t *u, uint8_t *d_out, const uint64_t *d_out_off,
                     void *stream)
{
    stage_t *sg = &ctx->st;
    size_t k = 0;
    for (size_t i = 0; i < n; i++)
        sg->h_meta[i].info = 0xff0000u;
    for (size_t j = 0; j < nl; j++) {
        size_t i = list[j];
        u[i].dirty = 0;
        if (SRTP_META_VARIANT(u[i].dm.info) == SRTP_VARIANT_V) {
            uint64_t o;
            if (i < ctx->vres_cap && ctx->vsave[i] &&
                (srtp_gpu_d2h(ctx->gpu, &o, d_out_off + i, 8, stream) ||
                 srtp_gpu_sync(ctx->gpu, stream) ||
                 srtp_gpu_h2d(ctx->gpu, d_out + o, ctx->vsave[i], u[i].dm.len,
                              stream) ||
                 srtp_gpu_sync(ctx->gpu, stream)))
                return -1;
            if (i < ctx->vres_cap) {
                free(ctx->vsave[i]);
                ctx->vsave[i] = NULL;
            }
            continue;
        }
        sg->h_meta[i] = u[i].dm;
        k++;
    }
    if (!k)
        return 0;
    ctx->ustat.undo_launches++;
    return srtp_gpu_h2d(ctx->gpu, sg->d_meta, sg->h_meta,
                        n * sizeof *sg->h_meta, stream) ||
           srtp_gpu_undo(ctx->gpu, n, d_out, d_out_off, sg->d_meta, stream) ||
           srtp_gpu_sync(ctx->gpu, stream);
}

static srtp_err_status_t unprotect_core(srtp_t ctx, size_t n,
                                        const pkt_sum_t *sum, const size_t *cap,
                                        const uint8_t *const *mki_ptr,
                                        const uint8_t *d_in,
                                        const uint64_t *d_in_off,
                                        uint8_t *d_out,
                                        const uint64_t *d_out_off,
                                        srtp_err_status_t *status,
                                        size_t *olen, void *stream)
{
    stage_t *sg = &ctx->st;
    const int inplace = d_out == d_in;
    upkt_t *u = (upkt_t *)calloc(n, sizeof(upkt_t));
    size_t *pend = (size_t *)malloc(n * sizeof(size_t));
    size_t *aux = (size_t *)malloc(n * sizeof(size_t));
    sset_t blk, redo;
    memset(&blk, 0, sizeof blk);
    memset(&redo, 0, sizeof redo);
    if (!u || !pend || !aux || sset_init(&blk, n) || sset_init(&redo, n)) {
        free(u);
        free(pend);
        free(aux);
        sset_free(&blk);
        sset_free(&redo);
        return srtp_err_status_alloc_fail;
    }
    for (size_t i = 0; i < n; i++)
        pend[i] = i;
    size_t npend = n;
    srtp_err_status_t ret = srtp_err_status_ok;
    memset(&ctx->ustat, 0, sizeof ctx->ustat);
    routed_reset(ctx);
    for (int round = 0; npend; round++) {
        const int mode = round < 2                 ? UNP_OPTIMISTIC
                         : round < UNP_SPEC_ROUNDS ? UNP_CAUTIOUS
                                                   : UNP_EXACT;
        provset_t ps;
        memset(&ps, 0, sizeof ps);
        ctx->epoch++;
        blk.gen++;
        for (size_t i = 0; i < n; i++)
            sg->h_meta[i].info = 0xff0000u; /* skip */
        size_t nrun = 0, nre = 0;
        for (size_t j = 0; j < npend; j++) {
            size_t i = pend[j];
            srtp_dev_meta_t m;
            memset(&m, 0, sizeof m);
            if (pre_unprotect(ctx, &ps, &sum[i], cap[i],
                              mki_ptr ? mki_ptr[i] : NULL, &u[i], &m, mode,
                              &blk)) {
                sg->h_meta[i] = m;
                if (inplace && u[i].dirty)
                    aux[nre++] = i; /* restore before it runs again */
                nrun++;
            }
        }
        provset_free(&ps);
        if (nre) {
            /* undo_runs() rewrites h_meta: keep this round's metas aside */
            srtp_dev_meta_t *keep =
                (srtp_dev_meta_t *)malloc(n * sizeof *keep);
            if (!keep) {
                ret = srtp_err_status_alloc_fail;
                break;
            }
            memcpy(keep, sg->h_meta, n * sizeof *keep);
            int bad = undo_runs(ctx, n, aux, nre, u, d_out, d_out_off, stream);
            memcpy(sg->h_meta, keep, n * sizeof *keep);
            free(keep);
            if (bad) {
                ret = srtp_err_status_fail;
                break;
            }
        }
        if (nrun) {
            ctx->ustat.launches++;
            if (run_gpu(ctx, 1, n, d_in, d_in_off, d_out, d_out_off,
                        sg->h_meta, stream) ||
                srtp_gpu_d2h(ctx->gpu, sg->h_auth, sg->d_auth, n, stream) ||
                srtp_gpu_sync(ctx->gpu, stream)) {
                log_msg(srtp_log_level_error, srtp_gpu_last_error());
                ret = srtp_err_status_fail;
                break;
            }
            for (size_t j = 0; j < npend; j++) {
                size_t i = pend[j];
                if (SRTP_META_STATUS(sg->h_meta[i].info))
                    continue;
                u[i].gpu = 1;
                u[i].auth = (sg->h_auth[i] & 1) != 0;
                u[i].failed |= !u[i].auth;
                u[i].dirty = 1;
                u[i].dm = sg->h_meta[i];
                u[i].xres = 0;
                if (SRTP_META_VARIANT(sg->h_meta[i].info) == SRTP_VARIANT_V)
                    u[i].dirty = u[i].auth; /* run_routed decrypts only then */
                if (SRTP_META_VARIANT(sg->h_meta[i].info) == SRTP_VARIANT_X) {
                    /* k_xrtp writes only authenticated packets; an undo
                     * needs to know whether cryptex was applied */
                    u[i].xres = sg->h_auth[i];
                    u[i].dirty = (sg->h_auth[i] & SRTP_XR_WROTE) != 0;
                    if (sg->h_auth[i] & SRTP_XR_CRYPTEX)
                        u[i].dm.info |= SRTP_XI_CRYPTEX;
                }
            }
        }
        /* exact in-order post-pass; a packet whose estimate moved is re-run
         * together with every later packet of its SSRC */
        redo.gen++;
        size_t again = 0;
        for (size_t j = 0; j < npend; j++) {
            size_t i = pend[j];
            if (!sum[i].err && sset_has(&redo, sum[i].ssrc)) {
                pend[again++] = i;
                continue;
            }
            int rc = post_unprotect(ctx, &sum[i], &u[i], &olen[i]);
            if (rc < 0) {
                sset_add(&redo, sum[i].ssrc);
                pend[again++] = i;
                continue;
            }
            status[i] = (srtp_err_status_t)rc;
        }
        npend = again;
        ctx->ustat.rounds = (uint32_t)round + 1;
    }
    /* rejected packets whose speculative decryption reached the output */
    if (!ret) {
        size_t nb = 0;
        for (size_t i = 0; i < n; i++)
            if (u[i].dirty && status[i] != srtp_err_status_ok)
                aux[nb++] = i;
        if (undo_runs(ctx, n, aux, nb, u, d_out, d_out_off, stream))
            ret = srtp_err_status_fail;
    }
    routed_reset(ctx);
    free(u);
    free(pend);
    free(aux);
    sset_free(&blk);
    sset_free(&redo);
    return ret;
}

srtp_err_status_t srtp_unprotect_batch(srtp_t ctx, size_t n,
                                       const uint8_t *const *srtp,
                                       const size_t *srtp_len,
                                       uint8_t *const *rtp, size_t *rtp_len,
                                       srtp_err_status_t *status)
{
    if (!ctx)
        return srtp_err_status_bad_param;
    ASYNC_DRAIN_CHECK(ctx);
    if (!n)
        return srtp_err_status_ok;
    size_t done = 0;
    int fast = batch_device_run(ctx, 1, n, srtp, srtp_len, rtp, rtp_len, NULL,
                                status, &done);
    if (fast < 0) {
        log_msg(srtp_log_level_error, srtp_gpu_last_error());
        return srtp_err_status_fail;
    }
    if (fast)
        return srtp_err_status_ok;
    /* a declined chunk: the rest on the host path */
    n -= done;
    srtp += done;
    srtp_len += done;
    rtp += done;
    rtp_len += done;
    status += done;
    dev_pull(ctx);
    if (n == 1) {   /* srtp_unprotect: the per-call path */
        const int r = one_unprotect(ctx, srtp[0], srtp_len[0], rtp[0],
                                    &rtp_len[0], &status[0]);
        if (r < 0) {
            log_msg(srtp_log_level_error, srtp_gpu_last_error());
            status[0] = srtp_err_status_cipher_fail;
            return srtp_err_status_fail;
        }
        if (r)
            return srtp_err_status_ok;
    }
    size_t arena = 0;
    for (size_t i = 0; i < n; i++)
        arena += r16(srtp_len[i]);
    if (stage_reserve(ctx, n, arena))
        return srtp_err_status_alloc_fail;
    stage_t *sg = &ctx->st;
    pkt_sum_t *sum = (pkt_sum_t *)malloc(n * sizeof(pkt_sum_t));
    const uint8_t **mki = (const uint8_t **)malloc(n * sizeof(void *));
    size_t *olen = (size_t *)calloc(n, sizeof(size_t));
    if (!sum || !mki || !olen) {
        free(sum);
        free(mki);
        free(olen);
        return srtp_err_status_alloc_fail;
    }
    size_t off = 0;
    for (size_t i = 0; i < n; i++) {
        summarize(srtp[i], srtp_len[i], &sum[i]);
        sum[i].inplace = srtp[i] == rtp[i];
        /* MKI bytes: the stream decides its size; point at the packet and
         * let un_static() index from the end */
        mki[i] = NULL;
        sg->h_off[i] = off;
        memcpy(sg->h_arena + off, srtp[i], srtp_len[i]);
        off += r16(srtp_len[i]);
    }
    /* resolve MKI pointers now that streams are known */
    for (size_t i = 0; i < n; i++) {
        if (sum[i].err)
            continue;
        const srtp_stream_ctx_t *st = map_get(ctx, sum[i].ssrc);
        if (!st)
            st = ctx->templ;
        if (!st || !st->use_mki)
            continue;
        const hkey_t *k0 = &st->keys->k[0];
        size_t tl = k0->family == SRTP_DEV_GCM ? 0 : k0->tag_len;
        if (tl <= srtp_len[i] && st->mki_size <= srtp_len[i] - tl)
            mki[i] = srtp[i] + srtp_len[i] - tl - st->mki_size;
    }
    srtp_err_status_t ret = srtp_err_status_ok;
    if (srtp_gpu_h2d(ctx->gpu, sg->d_arena, sg->h_arena, off, HS(ctx)) ||
        srtp_gpu_h2d(ctx->gpu, sg->d_off, sg->h_off, n * 8, HS(ctx)))
        ret = srtp_err_status_fail;
    if (!ret)
        ret = unprotect_core(ctx, n, sum, rtp_len, mki, sg->d_arena, sg->d_off,
                             sg->d_arena, sg->d_off, status, olen, HS(ctx));
    if (!ret && (srtp_gpu_d2h(ctx->gpu, sg->h_arena, sg->d_arena, off, HS(ctx)) ||
                 srtp_gpu_sync(ctx->gpu, HS(ctx))))
        ret = srtp_err_status_fail;
    for (size_t i = 0; i < n; i++) {
        if (ret) {
            status[i] = srtp_err_status_cipher_fail;
            continue;
        }
        if (status[i])
            continue;
        memcpy(rtp[i], sg->h_arena + sg->h_off[i], olen[i]);
        rtp_len[i] = olen[i];
    }
    free(sum);
    free(mki);
    free(olen);
    return ret;
}

/* single packet == batch of one (there is no CPU crypto path) */
srtp_err_status_t srtp_protect(srtp_t ctx, const uint8_t *rtp, size_t rtp_len,
                               uint8_t *srtp, size_t *srtp_len,
                               size_t mki_index)
{
    srtp_err_status_t st;
    srtp_err_status_t rc = srtp_protect_batch(ctx, 1, &rtp, &rtp_len, &srtp,
                                              srtp_len, &mki_index, &st);
    return rc ? rc : st;
}

srtp_err_status_t srtp_unprotect(srtp_t ctx, const uint8_t *srtp,
                                 size_t srtp_len, uint8_t *rtp, size_t *rtp_len)
{
    srtp_err_status_t st;
    srtp_err_status_t rc =
        srtp_unprotect_batch(ctx, 1, &srtp, &srtp_len, &rtp, rtp_len, &st);
    return rc ? rc : st;
}

/* ------------------------------------------------------------------------
 * batch API over device-resident arenas
 * ---------------------------------------------------------------------- */
static srtp_err_status_t dev_headers(srtp_t ctx, const srtp_device_batch_t *b,
                                     pkt_sum_t *sum, size_t *cap)
{
    stage_t *sg = &ctx->st;
    if (stage_reserve(ctx, b->n, 0))
        return srtp_err_status_alloc_fail;
    if (srtp_gpu_parse(ctx->gpu, b->n, b->in, b->in_off, b->in_len, sg->d_hdr,
                       sg->d_xinfo, b->stream) ||
        srtp_gpu_d2h(ctx->gpu, sg->h_hdr, sg->d_hdr, b->n * sizeof *sg->h_hdr,
                     b->stream) ||
        srtp_gpu_d2h(ctx->gpu, sg->h_xinfo, sg->d_xinfo, b->n * 4, b->stream))
        return srtp_err_status_fail;
    /* capacities: the caller's out_len array */
    uint32_t *caps = (uint32_t *)sg->h_arena;
    if (stage_reserve(ctx, b->n, b->n * 4))
        return srtp_err_status_alloc_fail;
    caps = (uint32_t *)sg->h_arena;
    if (srtp_gpu_d2h(ctx->gpu, caps, b->out_len, b->n * 4, b->stream) ||
        srtp_gpu_sync(ctx->gpu, b->stream))
        return srtp_err_status_fail;
    for (size_t i = 0; i < b->n; i++) {
        from_dev_hdr(&sg->h_hdr[i], sg->h_xinfo[i], &sum[i]);
        /* same arena: in place (an overlapping, different offset is not a
         * supported layout) */
        sum[i].inplace = b->in == b->out;
        cap[i] = caps[i];
    }
    return srtp_err_status_ok;
}

static srtp_err_status_t dev_results(srtp_t ctx, const srtp_device_batch_t *b,
                                     const srtp_err_status_t *status,
                                     const size_t *olen, const size_t *cap)
{
    stage_t *sg = &ctx->st;
    /* reuse the pinned arena for the two result arrays */
    if (stage_reserve(ctx, b->n, b->n * 8))
        return srtp_err_status_alloc_fail;
    int32_t *hs = (int32_t *)sg->h_arena;
    uint32_t *hl = (uint32_t *)(sg->h_arena + b->n * 4);
    for (size_t i = 0; i < b->n; i++) {
        hs[i] = (int32_t)status[i];
        hl[i] = (uint32_t)(status[i] ? cap[i] : olen[i]);
    }
    if (srtp_gpu_h2d(ctx->gpu, b->status, hs, b->n * 4, b->stream) ||
        srtp_gpu_h2d(ctx->gpu, b->out_len, hl, b->n * 4, b->stream) ||
        srtp_gpu_sync(ctx->gpu, b->stream))
        return srtp_err_status_fail;
    return srtp_err_status_ok;
}

/* ------------------------------------------------------------------------
 * device stream table (DESIGN.md "Device pre-pass")
 * ---------------------------------------------------------------------- */
/* the device record of stream st (or of the template: a clone's record,
 * fresh, usable in both directions -- srtp.c:2540 makes a protect clone a
 * sender, 3141 an unprotect clone a receiver), and the table's aggregates */
static void dev_record(devtab_t *dt, srtp_stream_ctx_t *st, int templ,
                       srtp_dev_stream_t *d, int *first, int *rx_first)
{
    /* MKI streams: every packet picks its key from the stream's list in
     * mkslot -- by mki_index on protect, by its MKI bytes on receive; the
     * record's own key is master key 0 */
    const hkey_t *k = &st->keys->k[0];
    memset(d, 0, sizeof *d);
    d->ssrc = st->ssrc;
    d->key = k->slot;
    d->variant = k->variant;
    uint64_t left = k->num_left;   /* protect: the least of the stream's keys */
    if (st->use_mki) {
        dt->has_mki = 1;
        const uint32_t back = (uint32_t)st->mki_size +
            (k->family == SRTP_DEV_GCM ? 0u : (uint32_t)k->tag_len);
        d->mki = (uint32_t)st->mki_size | (back << 16);
        d->kbase = dt->nmk;
        d->nkeys = (uint32_t)st->keys->n;
        for (size_t j = 0; j < st->keys->n; j++) {
            dt->mkslot[dt->nmk++] = st->keys->k[j].slot;
            if (st->keys->k[j].num_left < left)
                left = st->keys->k[j].num_left;
        }
    }
    /* header-extension encryption / cryptex streams and routed keys: host
     * pre-pass.  A pending ROC is resolved per batch (pend_resolve), in
     * either direction (srtp.c:2069-2076) */
    const int xs = k->variant >= SRTP_VARIANT_X;
    if (!templ && st->rdbx.pending_roc && !xs) {
        d->flags |= SRTP_DS_PENDING;
        d->rsv = st->rdbx.pending_roc;
    }
    if (!xs && (templ || st->direction != DIR_RECEIVER)) {
        d->flags |= SRTP_DS_ELIGIBLE;
        if (st->use_mki && st->keys->n < dt->mki_nmin)
            dt->mki_nmin = (uint32_t)st->keys->n;
        if (left < dt->num_left_min)
            dt->num_left_min = left;
        if (*first)
            dt->uniform = k->slot;
        else if (dt->uniform != k->slot)
            dt->uniform = 0xffffffffu;
        *first = 0;
        dt->mask |= 1u << k->variant;
        const uint32_t tr =
            (uint32_t)(k->tag_len + (st->use_mki ? st->mki_size : 0));
        if (tr > dt->max_trailer)
            dt->max_trailer = tr;
    }
    if (!xs && (templ || st->direction != DIR_SENDER)) {
        d->flags |= SRTP_DS_RX_ELIGIBLE;
        if (left < dt->num_left_min)   /* every key of an MKI stream */
            dt->num_left_min = left;
        if (st->use_mki && st->keys->n > 1)
            dt->rx_multi = 1;
        if (*rx_first)
            dt->rx_uniform = k->slot;
        else if (dt->rx_uniform != k->slot)
            dt->rx_uniform = 0xffffffffu;
        *rx_first = 0;
        dt->rx_mask |= 1u << k->variant;
    }
    if (k->family == SRTP_DEV_ICM && (st->rtp_services & sec_serv_conf))
        d->flags |= SRTP_DS_ICM_CONF;
    if (k->family == SRTP_DEV_GCM)
        d->flags |= SRTP_DS_AEAD;
    d->trailer = (uint32_t)(k->tag_len + (st->use_mki ? st->mki_size : 0));
    d->win_bits = (uint32_t)st->rdbx.bits;
    d->index = templ ? 0 : st->rdbx.index;
}

/* records of the streams the device may create from the template per
 * upload (dev_pull takes them over) */
#define DEV_SPARE_MIN 65536u

static int dev_build(srtp_t ctx)
{
    if (async_drain(ctx))
        return -1;
    devtab_t *dt = &ctx->dt;
    uint32_t ns = (uint32_t)ctx->n;
    size_t nwords = 0;
    for (size_t i = 0; i < ctx->n; i++)
        nwords += ctx->list[i]->rdbx.bits / 32;
    /* template sessions: spare records for the streams a batch creates */
    srtp_stream_ctx_t *tp = ctx->templ;
    const int tmpl_ok = tp && tp->keys->k[0].variant < SRTP_VARIANT_X;
    const uint32_t spare = tmpl_ok ? (ns > DEV_SPARE_MIN ? ns : DEV_SPARE_MIN)
                                   : 0;
    const size_t tw = tmpl_ok ? tp->rdbx.bits / 32 : 0;
    free(dt->sv);
    free(dt->hs);
    free(dt->hwin);
    free(dt->pend);
    free(dt->res);
    free(dt->mkslot);
    free(dt->kuses);
    size_t nmk = 1;   /* the MKI streams' keys (and the template's) */
    for (size_t i = 0; i < ctx->n; i++)
        if (ctx->list[i]->use_mki)
            nmk += ctx->list[i]->keys->n;
    if (tp && tp->use_mki)
        nmk += tp->keys->n;
    dt->mkslot = (uint32_t *)malloc(nmk * sizeof(uint32_t));
    dt->kuses = (uint64_t *)calloc(nmk, sizeof(uint64_t));
    dt->nmk = 0;
    dt->mki_nmin = UINT32_MAX;
    dt->pend = (uint32_t *)malloc((ns + 1) * sizeof(uint32_t));
    dt->res = (uint32_t *)malloc((ns + 1) * sizeof(uint32_t));
    dt->npend = dt->nres = 0;
    dt->sv = (srtp_stream_ctx_t **)calloc(ns + 1, sizeof(void *));
    dt->hs = (srtp_dev_stream_t *)calloc(ns + spare + 1,
                                         sizeof(srtp_dev_stream_t));
    dt->hwin = (uint32_t *)calloc(nwords + spare * tw + 1, 4);
    /* the device hash holds the spare streams too: load <= 1/2 */
    size_t hcap = ctx->map.cap ? ctx->map.cap : 1;
    while (hcap < 2 * ((size_t)ns + spare))
        hcap *= 2;
    uint32_t *hk = (uint32_t *)calloc(hcap, 4);
    uint32_t *hv = (uint32_t *)malloc(hcap * 4);
    int rc = -1;
    if (!dt->sv || !dt->hs || !dt->hwin || !hk || !hv || !dt->pend ||
        !dt->res || !dt->mkslot || !dt->kuses)
        goto out;
    dt->num_left_min = UINT64_MAX;
    dt->uniform = dt->rx_uniform = 0xffffffffu;
    dt->mask = dt->rx_mask = 0;
    dt->max_trailer = 0;
    int first = 1, rx_first = 1;
    uint32_t woff = 0;
    dt->has_mki = 0;
    dt->rx_multi = 0;
    for (uint32_t sid = 0; sid < ns; sid++) {
        srtp_stream_ctx_t *st = ctx->list[sid];
        srtp_dev_stream_t *d = &dt->hs[sid];
        dt->sv[sid] = st;
        st->dev_sid = sid;
        dev_record(dt, st, 0, d, &first, &rx_first);
        if (d->flags & SRTP_DS_PENDING)
            dt->pend[dt->npend++] = sid;
        d->win_off = woff;
        memcpy(dt->hwin + woff, st->rdbx.w, st->rdbx.bits / 8);
        woff += (uint32_t)(st->rdbx.bits / 32);
    }
    srtp_dev_stream_t td;
    if (tmpl_ok) {
        dev_record(dt, tp, 1, &td, &first, &rx_first);
        td.win_off = woff;   /* the spare windows (zero) follow */
        dt->tmpl_kbase = td.kbase;
    }
    for (size_t h = 0; h < hcap; h++)
        hv[h] = 0xffffffffu;
    for (size_t h = 0; h < ctx->map.cap; h++) {
        if (!ctx->map.vals[h])
            continue;
        const uint32_t key = ctx->map.keys[h];
        size_t p = map_hash(key, hcap);
        while (hv[p] != 0xffffffffu)
            p = (p + 1) & (hcap - 1);
        hk[p] = key;
        hv[p] = ctx->map.vals[h]->dev_sid;
    }
    if (srtp_gpu_pp_upload(ctx->gpu, dt->hs, ns, dt->hwin,
                           woff + (uint32_t)(spare * tw), hk, hv,
                           (uint32_t)hcap, tmpl_ok ? &td : NULL, spare,
                           dt->mkslot, dt->nmk))
        goto out;
    dt->ns = ns;
    dt->nwords = woff;
    dt->tmpl_ok = tmpl_ok;
    dt->uses_bound = 0;
    dt->valid = 1;
    dt->dirty = 0;
    rc = 0;
out:
    free(hk);
    free(hv);
    return rc;
}

/* bring the device-advanced stream state back into the host streams and
 * drop the mirror (the caller is about to use or change host state) */
/* work srtp_protect_device_async left queued is finished before anything
 * reads or changes the device stream table, the keys or the staging arenas
 * from another stream */
static int g_fail_drains;   /* test hook: srtp_mi355x_debug_inject_failure */
static int g_fail_bcast_alloc;   /* ... and for srtp_mi355x_session_broadcast */

/* returns -1 (and poisons the session) when the queued batch failed */
static int async_drain(srtp_t ctx)
{
    if (ctx->dt.async_err)
        return -1;
    if (!ctx->dt.async_pending)
        return 0;
    ctx->dt.async_pending = 0;
    int bad = srtp_gpu_sync(ctx->gpu, ctx->dt.async_stream) != 0;
    if (g_fail_drains > 0) {
        g_fail_drains--;
        bad = 1;
    }
    if (bad) {
        ctx->dt.async_err = 1;
        log_msg(srtp_log_level_error,
                "a queued srtp_protect_device_async batch failed on the GPU; "
                "the session refuses further packets");
        return -1;
    }
    return 0;
}

static void dev_pull(srtp_t ctx);

/* MKI sessions: the master key each protect packet selects (mki_index,
 * srtp.c:2536-2545) runs on the device when it is below every MKI stream's
 * key count; otherwise (srtp_err_status_bad_mki for some packet) the batch
 * takes the host path.  *out: the indices as bytes for the device (NULL:
 * the caller passed none, every packet uses key 0).  Returns 1 for the
 * host path, -1 on allocation failure. */
static int dev_mki_index(srtp_t ctx, const uint8_t *m8, const size_t *m64,
                         size_t n, uint8_t **out)
{
    devtab_t *dt = &ctx->dt;
    uint8_t *o = (uint8_t *)calloc(n ? n : 1, 1);
    if (!o)
        return -1;
    for (size_t i = 0; (m8 || m64) && i < n; i++) {
        const size_t j = m64 ? m64[i] : m8[i];
        if (j >= dt->mki_nmin) {
            free(o);
            dt->last_abort = 256;
            return 1;
        }
        o[i] = (uint8_t)j;
    }
    *out = o;
    return 0;
}

static void dev_pull(srtp_t ctx)
{
    devtab_t *dt = &ctx->dt;
    if (async_drain(ctx)) {
        /* never take stream state from a table a failed batch left */
        dt->valid = 0;
        dt->dirty = 0;
        return;
    }
    if (!dt->valid)
        return;
    dt->valid = 0;
    if (!dt->dirty)
        return;
    dt->dirty = 0;
    uint32_t ns_now = 0;
    if (srtp_gpu_pp_download(ctx->gpu, dt->hs, dt->hwin, &ns_now,
                             dt->kuses)) {
        log_msg(srtp_log_level_error, "device stream table download failed");
        return;
    }
    for (uint32_t sid = 0; sid < dt->ns; sid++) {
        srtp_stream_ctx_t *st = dt->sv[sid];
        const srtp_dev_stream_t *d = &dt->hs[sid];
        st->rdbx.index = d->index;
        memcpy(st->rdbx.w, dt->hwin + d->win_off, st->rdbx.bits / 8);
        /* uses: the packets charged to the stream's key (an MKI stream's
         * charges all moved to kuses: srtp_prepass.hip k_mki_keys,
         * k_mki_rx_charge); kuses: per master key */
        st->keys->k[0].num_left -= d->uses;
        for (uint32_t j = 0; j < d->nkeys; j++)
            st->keys->k[j].num_left -= dt->kuses[d->kbase + j];
        /* a device batch never used a stream against its direction (the
         * eligibility flags), so no ssrc_collision event is due here */
        if (st->direction == DIR_UNKNOWN && (d->dir & SRTP_DIR_TX))
            st->direction = DIR_SENDER;
        if (st->direction == DIR_UNKNOWN && (d->dir & SRTP_DIR_RX))
            st->direction = DIR_RECEIVER;
    }
    /* streams the device created from the template (srtp_gpu_pp_clone), in
     * creation order: a protect clone is a sender (srtp.c:2540-2559); a
     * receive clone exists once one of its packets authenticated
     * (srtp.c:3117-3155) -- before that its packets ran on the template's
     * keys, whose usage they still count (the clones share its limit,
     * srtp_key_limit_clone) */
    srtp_stream_ctx_t *tp = ctx->templ;
    if (tp && dt->tmpl_ok && tp->use_mki)
        for (size_t j = 0; j < tp->keys->n; j++)
            tp->keys->k[j].num_left -= dt->kuses[dt->tmpl_kbase + j];
    for (uint32_t sid = dt->ns; tp && sid < ns_now; sid++) {
        const srtp_dev_stream_t *d = &dt->hs[sid];
        tp->keys->k[0].num_left -= d->uses;
        if (!(d->dir & (SRTP_DIR_TX | SRTP_DIR_RX)))
            continue;
        srtp_stream_ctx_t *st = stream_clone(tp, d->ssrc);
        if (!st || list_insert(ctx, st)) {
            if (st)
                stream_free(ctx, st);
            log_msg(srtp_log_level_error,
                    "device-created stream: allocation failed");
            continue;
        }
        st->direction = (d->dir & SRTP_DIR_TX) ? DIR_SENDER : DIR_RECEIVER;
        st->rdbx.index = d->index;
        memcpy(st->rdbx.w, dt->hwin + d->win_off, st->rdbx.bits / 8);
    }
}

/* Pending ROCs (srtp_stream_set_roc; srtp.c:2038-2081, 5137-5167) of the
 * streams the device may take, resolved for this batch from the first
 * packet of each (srtp_dev.h srtp_gpu_pp_pend_*), in the reference's
 * per-packet terms:
 *   * the first packet's index pending_roc || seq more than 2^15 past the
 *     stored index: it sets index and window and clears the pending ROC
 *     (srtp.c:2674-2678, 3161-3167) -- the device gets the state one packet
 *     earlier and runs the stream as any other; the host clears the pending
 *     ROC when the batch commits;
 *   * every packet's pending_roc || seq within 2^15 of the stored index and
 *     of each other: each is the index the normal estimate gives, none
 *     advances past or falls behind the window by 2^15 -- the device runs
 *     it unchanged and the ROC stays pending;
 *   * anything else (a first packet 2^15 behind: pkt_idx_old, and the
 *     ROC stays pending for the next packet): the host path.
 * Returns 0 (the device may run the batch), 1 (host path), -1 (error). */
static int pend_resolve(srtp_t ctx, const srtp_gpu_pp_batch_t *pb,
                        int unprotect)
{
    devtab_t *dt = &ctx->dt;
    dt->nres = 0;
    if (!dt->npend)
        return 0;
    srtp_pend_info_t *inf =
        (srtp_pend_info_t *)malloc(dt->npend * sizeof *inf);
    uint64_t *ef = (uint64_t *)malloc(dt->npend * sizeof *ef);
    uint32_t *fp = (uint32_t *)malloc(dt->npend * sizeof *fp);
    int rc = -1;
    if (!inf || !ef || !fp ||
        srtp_gpu_pp_pend_scan(ctx->gpu, pb, unprotect, dt->pend, dt->npend,
                              inf))
        goto out;
    rc = 0;
    for (uint32_t k = 0; k < dt->npend && !rc; k++) {
        const srtp_pend_info_t *r = &inf[k];
        if (r->first == 0xffffffffu)
            continue;   /* no packet of the stream: the ROC stays pending */
        const uint64_t I0 = r->index, e1 = r->efirst;
        if (e1 > I0 && e1 - I0 > SEQ_MEDIAN) {
            dt->res[dt->nres] = dt->pend[k];
            ef[dt->nres] = e1;
            fp[dt->nres] = r->first;
            dt->nres++;
        } else if (!(r->emax - r->emin < SEQ_MEDIAN &&
                     (r->emax <= I0 || r->emax - I0 < SEQ_MEDIAN) &&
                     (r->emin >= I0 || I0 - r->emin < SEQ_MEDIAN))) {
            rc = 1;
        }
    }
    if (!rc && dt->nres &&
        srtp_gpu_pp_pend_apply(ctx->gpu, dt->res, ef, fp, dt->nres,
                               pb->stream))
        rc = -1;
    if (rc)
        dt->nres = 0;
    if (rc == 1)
        dt->last_abort = 1024;
out:
    free(inf);
    free(ef);
    free(fp);
    return rc;
}

/* after the pre-pass: committed (the applied streams' ROCs are no longer
 * pending) or declined (their device records back) */
static int pend_settle(srtp_t ctx, int committed, void *stream)
{
    devtab_t *dt = &ctx->dt;
    if (!dt->nres)
        return 0;
    int rc = 0;
    if (committed) {
        srtp_gpu_pp_pend_clear(ctx->gpu);
        for (uint32_t k = 0; k < dt->nres; k++) {
            const uint32_t sid = dt->res[k];
            dt->sv[sid]->rdbx.pending_roc = 0;
            for (uint32_t j = 0; j < dt->npend; j++)
                if (dt->pend[j] == sid) {
                    dt->pend[j] = dt->pend[--dt->npend];
                    break;
                }
        }
    } else {
        rc = srtp_gpu_pp_pend_restore(ctx->gpu, stream);
    }
    dt->nres = 0;
    return rc;
}

/* the device pre-pass of a batch (srtp_gpu_pp_protect / _unprotect) with
 * the pending ROCs resolved around it, and -- when the first run stopped at
 * SSRCs without a stream and the session has a template -- those streams
 * created on the device (srtp_gpu_pp_clone) and the batch run again.
 * Returns -1 on a device error, else 0 with *fallback the abort reason
 * (0: committed on the device). */
static int pp_run(srtp_t ctx, srtp_gpu_pp_batch_t *pb, int unprotect,
                  int *fallback)
{
    devtab_t *dt = &ctx->dt;
    for (int round = 0;; round++) {
        const int pr = pend_resolve(ctx, pb, unprotect);
        if (pr < 0)
            return -1;
        if (pr) {
            *fallback = 1024;
            return 0;
        }
        int fb = 1;
        if (unprotect ? srtp_gpu_pp_unprotect(ctx->gpu, pb, &fb)
                      : srtp_gpu_pp_protect(ctx->gpu, pb, &fb))
            return -1;
        if (pend_settle(ctx, !fb, pb->stream))
            return -1;
        *fallback = fb;
        if (round == 0 && (fb & 1) && dt->tmpl_ok) {
            uint32_t added = 0;
            const int c = srtp_gpu_pp_clone(ctx->gpu, pb, &added);
            if (c < 0)
                return -1;
            if (c == 0 && added)
                continue;
        }
        return 0;
    }
}

/* the kernel variant (one bit of a variant mask) whose kernel classifies
 * order-free batches itself: AES-ICM (variant ids 10..15) and AES-GCM (ids
 * 18, 22: k_gcm's per-lane form), any key mode -- one key for every stream
 * (a template session's clones) runs the per-lane form too, its key the
 * same in every lane */
static int fused_variant(uint32_t mask, uint32_t uniform)
{
    (void)uniform;
    return (mask & 0xfc00u) == mask || (mask & 0x440000u) == mask;
}

/* which way the one-stream in-order form went (srtp_mi355x_inorder_stats) */
static void io_count(devtab_t *dt, const srtp_gpu_pp_batch_t *pb)
{
    if (pb->inorder == 1)
        dt->io_runs++;
    else if (pb->inorder == 2)
        dt->io_declines++;
}

/* the device pre-pass; returns 1 when the batch was completed on the GPU,
 * 0 when the host path must run it, -1 on a device error */
static int protect_device_fast(srtp_t ctx, const srtp_device_batch_t *b,
                               int async, const size_t *mki_wide)
{
    devtab_t *dt = &ctx->dt;
    if ((!ctx->n && !ctx->templ) || b->n > 0x7fffffffu) {
        dt->last_abort = 64;
        return 0;
    }
    if (!dt->valid && dev_build(ctx))
        return -1;
    /* no key can reach its soft limit inside this batch (key.c:74-90) */
    if (dt->num_left_min == UINT64_MAX ||
        dt->num_left_min < dt->uses_bound + b->n + SOFT_LIMIT) {
        dt->last_abort = 128;
        return 0;
    }
    uint8_t *mki8 = NULL;
    if (dt->has_mki) {
        const int r = dev_mki_index(ctx, b->mki_index, mki_wide, b->n, &mki8);
        if (r)
            return r < 0 ? -1 : 0;
    }
    srtp_gpu_pp_batch_t pb;
    memset(&pb, 0, sizeof pb);
    pb.mki = mki8;
    pb.n = b->n;
    pb.in = b->in;
    pb.in_off = b->in_off;
    pb.in_len = b->in_len;
    pb.out = b->out;
    pb.out_off = b->out_off;
    pb.out_len = b->out_len;
    pb.status = b->status;
    pb.stream = b->stream;
    /* MKI streams: a key per packet */
    pb.uniform_key = mki8 ? 0xffffffffu : dt->uniform;
    pb.mask = dt->mask;
    pb.async = async;
    /* the order-free form may classify inside the AES-ICM kernel: in place
     * (the declined case restores the input), one AES-ICM kernel variant
     * (variant ids 10..15: family ICM, AES-128/192/256), and trailers the
     * kernel saves whole.  One key for every stream (a template session's
     * clones) takes it too: the per-lane key is then loaded once per lane */
    pb.fused_ok = b->in == b->out && b->in_off == b->out_off && dt->mask &&
                  (dt->mask & (dt->mask - 1)) == 0 &&
                  fused_variant(dt->mask, dt->uniform) &&
                  dt->max_trailer <= 16 && !async && !mki8;
    pb.max_trailer = dt->max_trailer;
    /* one stream in order: indices in the crypto kernel (uniform key, one
     * AES-ICM or AES-GCM variant; srtp_prepass.hip pp_protect_inorder --
     * out of place or asynchronous with the batch checked first) */
    pb.inorder_ok = dt->mask && (dt->mask & (dt->mask - 1)) == 0 &&
                    ((dt->mask & 0xfc00u) == dt->mask ||
                     (dt->mask & 0x440000u) == dt->mask) &&
                    dt->uniform != 0xffffffffu && dt->max_trailer <= 16 &&
                    !mki8;
    int fallback = 1;
    srtp_gpu_set_timing(ctx->gpu, ctx->timing);
    const int rr = pp_run(ctx, &pb, 0, &fallback);
    free(mki8);
    if (rr)
        return -1;
    io_count(dt, &pb);
    if (fallback) {
        dt->last_abort = fallback;
        return 0;
    }
    dt->bk_batches += pb.bucketed != 0;
    if (ctx->timing)
        ctx->last_ms = srtp_gpu_last_kernel_ms(ctx->gpu);
    dt->sorted_batches += pb.sorted;
    dt->uses_bound += b->n;
    dt->dirty = 1;
    return 1;
}

static srtp_err_status_t protect_device(srtp_t ctx,
                                        const srtp_device_batch_t *b,
                                        int async);

srtp_err_status_t srtp_protect_device(srtp_t ctx, const srtp_device_batch_t *b)
{
    return protect_device(ctx, b, 0);
}

srtp_err_status_t srtp_protect_device_async(srtp_t ctx,
                                            const srtp_device_batch_t *b)
{
    return protect_device(ctx, b, 1);
}

static srtp_err_status_t protect_device(srtp_t ctx,
                                        const srtp_device_batch_t *b,
                                        int async)
{
    if (!ctx || !b)
        return srtp_err_status_bad_param;
    ASYNC_POISON_CHECK(ctx);
    if (!b->n)
        return srtp_err_status_ok;
    /* the same stream orders a queued batch before this one */
    if (ctx->dt.async_pending && ctx->dt.async_stream != b->stream &&
        async_drain(ctx))
        return srtp_err_status_fail;
    int fast = protect_device_fast(ctx, b, async, NULL);
    if (fast < 0) {
        log_msg(srtp_log_level_error, srtp_gpu_last_error());
        return srtp_err_status_fail;
    }
    if (fast) {
        ctx->dt.fast_batches++;
        ctx->dt.async_pending = async;   /* else the stream was synchronised */
        ctx->dt.async_stream = b->stream;
        return srtp_err_status_ok;
    }
    ctx->dt.host_batches++;
    dev_pull(ctx);
    size_t n = b->n;
    pkt_sum_t *sum = (pkt_sum_t *)malloc(n * sizeof *sum);
    size_t *cap = (size_t *)malloc(n * sizeof(size_t));
    size_t *olen = (size_t *)calloc(n, sizeof(size_t));
    srtp_err_status_t *status =
        (srtp_err_status_t *)malloc(n * sizeof(srtp_err_status_t));
    srtp_err_status_t ret = srtp_err_status_alloc_fail;
    if (!sum || !cap || !olen || !status)
        goto out;
    ret = dev_headers(ctx, b, sum, cap);
    if (ret)
        goto out;
    for (size_t i = 0; i < n; i++) {
        srtp_dev_meta_t *m = &ctx->st.h_meta[i];
        memset(m, 0, sizeof *m);
        status[i] = pre_protect(ctx, &sum[i], cap[i],
                                b->mki_index ? b->mki_index[i] : 0, m, &olen[i]);
        if (status[i])
            m->info = (uint32_t)(status[i] & 0xff) << 16;
    }
    if (run_gpu(ctx, 0, n, b->in, b->in_off, b->out, b->out_off,
                ctx->st.h_meta, b->stream) ||
        xrtp_protect_results(ctx, n, status, b->stream)) {
        ret = srtp_err_status_fail;
        goto out;
    }
    routed_status(ctx, n, status);
    ret = dev_results(ctx, b, status, olen, cap);
out:
    free(sum);
    free(cap);
    free(olen);
    free(status);
    return ret;
}

/* the device unprotect pre-pass (srtp_prepass.hip srtp_gpu_pp_unprotect);
 * 1 done on the GPU, 0 host path, -1 device error */
static int unprotect_device_fast(srtp_t ctx, const srtp_device_batch_t *b)
{
    devtab_t *dt = &ctx->dt;
    if ((!ctx->n && !ctx->templ) || b->n > 0x7fffffffu) {
        dt->last_abort = 64;
        return 0;
    }
    if (!dt->valid && dev_build(ctx))
        return -1;
    if (dt->num_left_min == UINT64_MAX ||
        dt->num_left_min < dt->uses_bound + b->n + SOFT_LIMIT) {
        dt->last_abort = 128;
        return 0;
    }
    srtp_gpu_pp_batch_t pb;
    memset(&pb, 0, sizeof pb);
    pb.n = b->n;
    pb.in = b->in;
    pb.in_off = b->in_off;
    pb.in_len = b->in_len;
    pb.out = b->out;
    pb.out_off = b->out_off;
    pb.out_len = b->out_len;
    pb.status = b->status;
    pb.stream = b->stream;
    /* an MKI stream with several keys: a key per packet */
    pb.uniform_key = dt->rx_multi ? 0xffffffffu : dt->rx_uniform;
    pb.mki_rx = dt->has_mki;
    pb.mask = dt->rx_mask;
    /* the order-free receive form may classify inside the AES-ICM kernel:
     * in place (a declined batch is restored), one AES-ICM kernel variant,
     * no MKI streams (their per-packet keys are k_pu_classify's) */
    pb.fused_ok = b->in == b->out && b->in_off == b->out_off && dt->rx_mask &&
                  (dt->rx_mask & (dt->rx_mask - 1)) == 0 &&
                  fused_variant(dt->rx_mask, dt->rx_uniform) && !dt->has_mki;
    /* one stream in order (srtp_prepass.hip pp_unprotect_inorder), in place
     * or not (a rejected packet's output is undone to its ciphertext) */
    pb.inorder_ok = dt->rx_mask && (dt->rx_mask & (dt->rx_mask - 1)) == 0 &&
                    ((dt->rx_mask & 0xfc00u) == dt->rx_mask ||
                     (dt->rx_mask & 0x440000u) == dt->rx_mask) &&
                    dt->rx_uniform != 0xffffffffu && !dt->has_mki;
    int fallback = 1;
    srtp_gpu_set_timing(ctx->gpu, ctx->timing);
    if (pp_run(ctx, &pb, 1, &fallback))
        return -1;
    io_count(dt, &pb);
    if (fallback) {
        dt->last_abort = fallback;
        return 0;
    }
    dt->bk_batches += pb.bucketed != 0;
    if (ctx->timing)
        ctx->last_ms = srtp_gpu_last_kernel_ms(ctx->gpu);
    dt->uses_bound += b->n;
    dt->dirty = 1;
    return 1;
}

srtp_err_status_t srtp_unprotect_device(srtp_t ctx,
                                        const srtp_device_batch_t *b)
{
    if (!ctx || !b)
        return srtp_err_status_bad_param;
    ASYNC_POISON_CHECK(ctx);
    if (!b->n)
        return srtp_err_status_ok;
    if (async_drain(ctx))
        return srtp_err_status_fail;
    int fast = unprotect_device_fast(ctx, b);
    if (fast < 0) {
        log_msg(srtp_log_level_error, srtp_gpu_last_error());
        return srtp_err_status_fail;
    }
    if (fast) {
        ctx->dt.fast_batches++;
        memset(&ctx->ustat, 0, sizeof ctx->ustat);
        ctx->ustat.rounds = ctx->ustat.launches = 1;
        return srtp_err_status_ok;
    }
    dev_pull(ctx);
    ctx->dt.host_batches++;
    size_t n = b->n;
    pkt_sum_t *sum = (pkt_sum_t *)malloc(n * sizeof *sum);
    size_t *cap = (size_t *)malloc(n * sizeof(size_t));
    size_t *olen = (size_t *)calloc(n, sizeof(size_t));
    srtp_err_status_t *status =
        (srtp_err_status_t *)calloc(n, sizeof(srtp_err_status_t));
    uint8_t *mkibuf = NULL;
    const uint8_t **mki = NULL;
    srtp_err_status_t ret = srtp_err_status_alloc_fail;
    if (!sum || !cap || !olen || !status)
        goto out;
    ret = dev_headers(ctx, b, sum, cap);
    if (ret)
        goto out;
    /* MKI streams: fetch each packet's MKI bytes (rare; small copies) */
    {
        int any_mki = ctx->templ && ctx->templ->use_mki;
        for (size_t i = 0; i < ctx->n && !any_mki; i++)
            any_mki = ctx->list[i]->use_mki;
        if (any_mki) {
            mki = (const uint8_t **)calloc(n, sizeof(void *));
            mkibuf = (uint8_t *)calloc(n, SRTP_MAX_MKI_LEN);
            uint64_t *offs = (uint64_t *)malloc(n * 8);
            ret = srtp_err_status_alloc_fail;
            if (!mki || !mkibuf || !offs) {
                free(offs);
                goto out;
            }
            ret = srtp_err_status_fail;
            if (srtp_gpu_d2h(ctx->gpu, offs, b->in_off, n * 8, b->stream) ||
                srtp_gpu_sync(ctx->gpu, b->stream)) {
                free(offs);
                goto out;
            }
            for (size_t i = 0; i < n; i++) {
                if (sum[i].err)
                    continue;
                const srtp_stream_ctx_t *st = map_get(ctx, sum[i].ssrc);
                if (!st)
                    st = ctx->templ;
                if (!st || !st->use_mki)
                    continue;
                const hkey_t *k0 = &st->keys->k[0];
                size_t tl = k0->family == SRTP_DEV_GCM ? 0 : k0->tag_len;
                if (tl > sum[i].len || st->mki_size > sum[i].len - tl)
                    continue;
                size_t at = sum[i].len - tl - st->mki_size;
                if (srtp_gpu_d2h(ctx->gpu, mkibuf + i * SRTP_MAX_MKI_LEN,
                                 b->in + offs[i] + at, st->mki_size,
                                 b->stream)) {
                    free(offs);
                    goto out;
                }
                mki[i] = mkibuf + i * SRTP_MAX_MKI_LEN;
            }
            free(offs);
            if (srtp_gpu_sync(ctx->gpu, b->stream))
                goto out;
        }
    }
    ret = unprotect_core(ctx, n, sum, cap, mki, b->in, b->in_off, b->out,
                         b->out_off, status, olen, b->stream);
    if (!ret)
        ret = dev_results(ctx, b, status, olen, cap);
out:
    free(sum);
    free(cap);
    free(olen);
    free(status);
    free(mkibuf);
    free((void *)mki);
    return ret;
}

/* ------------------------------------------------------------------------
 * SRTCP (RFC 3711 3.4) for AES-ICM / null cipher with HMAC-SHA1 / null auth,
 * and AEAD SRTCP with AES-GCM-128/256 (srtp.c:3894-4300).  Host: stream
 * lookup, E-bit / 31-bit index trailer, replay database
 * (crypto/replay/rdb.c).  GPU (k_rtcp): keystream, trailer + MKI placement,
 * HMAC-SHA1 or GCM tag, and tag verification.
 * ---------------------------------------------------------------------- */
#define SRTCP_HDR_LEN 8u          /* octets_in_rtcp_header             */
#define SRTCP_TRAILER_LEN 4u      /* sizeof(srtcp_trailer_t)           */
#define SRTCP_RDB_BITS 128u       /* rdb_bits_in_bitmask               */

static uint32_t be32_at(const uint8_t *p)
{
    return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 |
           p[3];
}

/* v128_left_shift, crypto/math/datatypes.c:231-262: bit (i + shift) -> i */
static void rdb_shift(uint32_t bm[4], uint32_t shift)
{
    uint32_t o[4] = { 0, 0, 0, 0 };
    if (shift < 128) {
        uint32_t base = shift >> 5, bit = shift & 31;
        for (uint32_t i = 0; i + base < 4; i++) {
            uint32_t lo = bm[i + base];
            uint32_t hi = i + base + 1 < 4 ? bm[i + base + 1] : 0;
            o[i] = bit ? (lo >> bit) | (hi << (32 - bit)) : lo;
        }
    }
    memcpy(bm, o, sizeof o);
}

/* srtp_rdb_check, rdb.c:74-96 */
static srtp_err_status_t rdb_check(const srtp_stream_ctx_t *s, uint32_t idx)
{
    if ((uint64_t)idx >= (uint64_t)s->rtcp_start + SRTCP_RDB_BITS)
        return srtp_err_status_ok;
    if (idx < s->rtcp_start)
        return srtp_err_status_replay_old;
    uint32_t d = idx - s->rtcp_start;
    if ((s->rtcp_bm[d >> 5] >> (d & 31)) & 1)
        return srtp_err_status_replay_fail;
    return srtp_err_status_ok;
}

/* srtp_rdb_add_index, rdb.c:103-127 */
static void rdb_add(srtp_stream_ctx_t *s, uint32_t idx)
{
    if (idx < s->rtcp_start)
        return;
    uint32_t d = idx - s->rtcp_start;
    if (d < SRTCP_RDB_BITS) {
        s->rtcp_bm[d >> 5] |= 1u << (d & 31);
    } else {
        d -= SRTCP_RDB_BITS - 1;
        rdb_shift(s->rtcp_bm, d);
        s->rtcp_bm[3] |= 1u << 31;
        s->rtcp_start += d;
    }
}

/* k_rtcp over a staged batch: packet i at h_arena + h_off[i] (in place);
 * meta with a non-zero status byte is skipped by the kernel */
static srtp_err_status_t rtcp_run(srtp_t ctx, int op, size_t n, size_t arena)
{
    stage_t *sg = &ctx->st;
    void *hs = HS(ctx);
    memset(sg->h_auth, 0, n);
    if (srtp_gpu_h2d(ctx->gpu, sg->d_arena, sg->h_arena, arena, hs) ||
        srtp_gpu_h2d(ctx->gpu, sg->d_off, sg->h_off, n * 8, hs) ||
        srtp_gpu_h2d(ctx->gpu, sg->d_meta, sg->h_meta, n * sizeof *sg->h_meta,
                     hs) ||
        srtp_gpu_h2d(ctx->gpu, sg->d_auth, sg->h_auth, n, hs) ||
        srtp_gpu_rtcp(ctx->gpu, op, n, sg->d_arena, sg->d_off, sg->d_meta,
                      sg->d_auth, hs) ||
        srtp_gpu_d2h(ctx->gpu, sg->h_arena, sg->d_arena, arena, hs) ||
        srtp_gpu_d2h(ctx->gpu, sg->h_auth, sg->d_auth, n, hs) ||
        srtp_gpu_sync(ctx->gpu, hs)) {
        log_msg(srtp_log_level_error, srtp_gpu_last_error());
        return srtp_err_status_fail;
    }
    return srtp_err_status_ok;
}

/* protect bookkeeping of one packet, in call order (srtp.c:4304-4420,
 * 3939-3990): stream / template clone, direction, key, buffer, index */
static srtp_err_status_t rtcp_pre_protect(srtp_t ctx, const uint8_t *rtcp,
                                          size_t rtcp_len, size_t cap,
                                          size_t mki_index,
                                          srtp_dev_meta_t *m, size_t *out_len)
{
    if (!rtcp || rtcp_len < SRTCP_HDR_LEN)
        return srtp_err_status_bad_param;
    uint32_t ssrc = be32_at(rtcp + 4);
    srtp_stream_ctx_t *st = map_get(ctx, ssrc);
    if (!st) {
        if (!ctx->templ)
            return srtp_err_status_no_ctx;
        st = stream_clone(ctx->templ, ssrc);
        if (!st)
            return srtp_err_status_alloc_fail;
        if (list_insert(ctx, st)) {
            stream_free(ctx, st);
            return srtp_err_status_alloc_fail;
        }
    }
    if (st->direction != DIR_SENDER) {
        if (st->direction == DIR_UNKNOWN)
            st->direction = DIR_SENDER;
        else
            fire(ctx, st, event_ssrc_collision);
    }
    hkey_t *k = &st->keys->k[0];
    if (st->use_mki) {
        if (mki_index >= st->keys->n)
            return srtp_err_status_bad_mki;
        k = &st->keys->k[mki_index];
    }
    if (k->rslot == 0xffffffffu)
        return srtp_err_status_no_such_op;
    /* same length arithmetic for srtp_protect_rtcp_aead (srtp.c:3939-4100),
     * where the tag precedes the trailer */
    *out_len = rtcp_len + SRTCP_TRAILER_LEN + st->mki_size + k->rtag_len;
    if (cap < *out_len)
        return srtp_err_status_buffer_small;
    /* srtp_rdb_increment, rdb.c:133-140; the index is the new window start */
    if (st->rtcp_start >= 0x7fffffffu)
        return srtp_err_status_key_expired;
    m->key = k->rslot;
    m->roc = ++st->rtcp_start;
    m->info = (st->rtcp_services & sec_serv_conf) ? 1u : 0u;
    m->len = (uint32_t)rtcp_len;
    return srtp_err_status_ok;
}

/* Batched srtp_protect_rtcp: results identical to n sequential calls */
srtp_err_status_t srtp_protect_rtcp_batch(srtp_t ctx, size_t n,
                                          const uint8_t *const *rtcp,
                                          const size_t *rtcp_len,
                                          uint8_t *const *srtcp,
                                          size_t *srtcp_len,
                                          const size_t *mki_index,
                                          srtp_err_status_t *status)
{
    if (!ctx)
        return srtp_err_status_bad_param;
    ASYNC_DRAIN_CHECK(ctx);
    dev_pull(ctx);
    if (!n)
        return srtp_err_status_ok;
    size_t arena = 0;
    for (size_t i = 0; i < n; i++)
        arena += r16(rtcp_len[i] + SRTCP_TRAILER_LEN + SRTP_MAX_TRAILER_LEN);
    if (stage_reserve(ctx, n, arena))
        return srtp_err_status_alloc_fail;
    stage_t *sg = &ctx->st;
    size_t *olen = (size_t *)calloc(n, sizeof(size_t));
    if (!olen)
        return srtp_err_status_alloc_fail;
    size_t off = 0;
    for (size_t i = 0; i < n; i++) {
        srtp_dev_meta_t *m = &sg->h_meta[i];
        memset(m, 0, sizeof *m);
        sg->h_off[i] = off;
        status[i] = rtcp_pre_protect(ctx, rtcp[i], rtcp_len[i], srtcp_len[i],
                                     mki_index ? mki_index[i] : 0, m,
                                     &olen[i]);
        if (status[i])
            m->info = (uint32_t)(status[i] & 0xff) << 16;
        else
            memcpy(sg->h_arena + off, rtcp[i], rtcp_len[i]);
        off += r16(rtcp_len[i] + SRTCP_TRAILER_LEN + SRTP_MAX_TRAILER_LEN);
    }
    srtp_err_status_t ret = rtcp_run(ctx, 0, n, off);
    for (size_t i = 0; i < n; i++) {
        if (ret) {
            status[i] = srtp_err_status_cipher_fail;
            continue;
        }
        if (status[i])
            continue;
        memcpy(srtcp[i], sg->h_arena + sg->h_off[i], olen[i]);
        srtcp_len[i] = olen[i];
    }
    free(olen);
    return ret;
}

/* state-independent unprotect checks (srtp.c:4546-4700, 4102-4170): stream
 * or template, MKI, lengths, E bit; fills the kernel descriptor.  Replay
 * state is consulted later, in order (rtcp_post_unprotect). */
typedef struct {
    uint32_t ssrc, idx;
    int gcm;
    size_t out_len;
} rtcp_u_t;

static srtp_err_status_t rtcp_pre_unprotect(srtp_t ctx, const uint8_t *srtcp,
                                            size_t srtcp_len,
                                            srtp_dev_meta_t *m, rtcp_u_t *u)
{
    if (!srtcp || srtcp_len < SRTCP_HDR_LEN + SRTCP_TRAILER_LEN)
        return srtp_err_status_bad_param;
    u->ssrc = be32_at(srtcp + 4);
    srtp_stream_ctx_t *st = map_get(ctx, u->ssrc);
    if (!st) {
        if (!ctx->templ)
            return srtp_err_status_no_ctx;
        st = ctx->templ; /* provisional; clones share its keys/services */
    }
    /* srtp_get_session_keys_for_rtcp_packet, srtp.c:2018-2035: the MKI
     * sits before a tag whose length follows key 0's RTCP cipher */
    hkey_t *k = &st->keys->k[0];
    if (st->use_mki) {
        size_t tl = k->rgcm ? 0 : k->rtag_len;
        if (tl > srtcp_len || st->mki_size > srtcp_len - tl)
            return srtp_err_status_bad_mki;
        k = mki_lookup(st, srtcp + srtcp_len - tl - st->mki_size);
        if (!k)
            return srtp_err_status_bad_mki;
    }
    if (k->rslot == 0xffffffffu)
        return srtp_err_status_no_such_op;
    size_t tag_len = k->rtag_len;
    if (srtcp_len < SRTCP_HDR_LEN + SRTCP_TRAILER_LEN + st->mki_size + tag_len)
        return srtp_err_status_bad_param;
    m->key = k->rslot;
    u->gcm = k->family == SRTP_DEV_GCM;
    if (u->gcm) {
        /* srtp_unprotect_rtcp_aead: trailer after the tag, E bit from the
         * packet */
        const uint8_t *tp = srtcp + srtcp_len - SRTCP_TRAILER_LEN - st->mki_size;
        u->idx = be32_at(tp) & 0x7fffffffu;
        u->out_len = srtcp_len - tag_len - SRTCP_TRAILER_LEN - st->mki_size;
        m->info = (tp[0] & 0x80) ? 1u : 0u;
        m->len = (uint32_t)u->out_len;
    } else {
        int conf = st->rtcp_services == sec_serv_conf ||
                   st->rtcp_services == sec_serv_conf_and_auth;
        const uint8_t *tp = srtcp + srtcp_len -
                            (tag_len + st->mki_size + SRTCP_TRAILER_LEN);
        if (((tp[0] & 0x80) != 0) != (conf != 0))
            return srtp_err_status_cant_check;
        u->idx = be32_at(tp) & 0x7fffffffu;
        u->out_len = srtcp_len - tag_len - st->mki_size - SRTCP_TRAILER_LEN;
        m->info = conf ? 1u : 0u;
        m->len = (uint32_t)(u->out_len + SRTCP_TRAILER_LEN);
    }
    m->roc = u->idx;
    return srtp_err_status_ok;
}

/* in-order part of unprotect: replay check, tag verdict, buffer, then the
 * reference's post-auth bookkeeping (srtp.c:4747-4837) */
static srtp_err_status_t rtcp_post_unprotect(srtp_t ctx, const rtcp_u_t *u,
                                             int auth_ok, size_t cap)
{
    srtp_stream_ctx_t *st = map_get(ctx, u->ssrc);
    if (!st)
        st = ctx->templ;
    srtp_err_status_t rc = rdb_check(st, u->idx);
    if (rc)
        return rc;
    if (u->gcm && cap < u->out_len)     /* AEAD checks the buffer first */
        return srtp_err_status_buffer_small;
    if (!auth_ok)
        return srtp_err_status_auth_fail;
    if (cap < u->out_len)
        return srtp_err_status_buffer_small;
    if (st->direction != DIR_RECEIVER) {
        if (st->direction == DIR_UNKNOWN)
            st->direction = DIR_RECEIVER;
        else
            fire(ctx, st, event_ssrc_collision);
    }
    if (st == ctx->templ) {
        srtp_stream_ctx_t *ns = stream_clone(ctx->templ, u->ssrc);
        if (!ns)
            return srtp_err_status_alloc_fail;
        if (list_insert(ctx, ns)) {
            stream_free(ctx, ns);
            return srtp_err_status_alloc_fail;
        }
        st = ns;
    }
    rdb_add(st, u->idx);
    return srtp_err_status_ok;
}

/* Batched srtp_unprotect_rtcp: the tag checks of the whole batch run in one
 * launch (they do not depend on replay state); the replay database is then
 * walked in packet order, so results equal n sequential calls */
srtp_err_status_t srtp_unprotect_rtcp_batch(srtp_t ctx, size_t n,
                                            const uint8_t *const *srtcp,
                                            const size_t *srtcp_len,
                                            uint8_t *const *rtcp,
                                            size_t *rtcp_len,
                                            srtp_err_status_t *status)
{
    if (!ctx)
        return srtp_err_status_bad_param;
    ASYNC_DRAIN_CHECK(ctx);
    dev_pull(ctx);
    if (!n)
        return srtp_err_status_ok;
    size_t arena = 0;
    for (size_t i = 0; i < n; i++)
        arena += r16(srtcp_len[i] + 16);
    if (stage_reserve(ctx, n, arena))
        return srtp_err_status_alloc_fail;
    stage_t *sg = &ctx->st;
    rtcp_u_t *u = (rtcp_u_t *)calloc(n, sizeof *u);
    if (!u)
        return srtp_err_status_alloc_fail;
    size_t off = 0;
    for (size_t i = 0; i < n; i++) {
        srtp_dev_meta_t *m = &sg->h_meta[i];
        memset(m, 0, sizeof *m);
        sg->h_off[i] = off;
        status[i] = rtcp_pre_unprotect(ctx, srtcp[i], srtcp_len[i], m, &u[i]);
        if (status[i])
            m->info = (uint32_t)(status[i] & 0xff) << 16;
        else
            memcpy(sg->h_arena + off, srtcp[i], srtcp_len[i]);
        off += r16(srtcp_len[i] + 16);
    }
    srtp_err_status_t ret = rtcp_run(ctx, 1, n, off);
    for (size_t i = 0; i < n; i++) {
        if (ret) {
            status[i] = srtp_err_status_cipher_fail;
            continue;
        }
        if (status[i])
            continue;
        status[i] = rtcp_post_unprotect(ctx, &u[i], sg->h_auth[i],
                                        rtcp_len[i]);
        if (status[i])
            continue;
        memcpy(rtcp[i], sg->h_arena + sg->h_off[i], u[i].out_len);
        rtcp_len[i] = u[i].out_len;
    }
    free(u);
    return ret;
}

/* srtp_protect_rtcp, srtp.c:4304-4544: a batch of one */
srtp_err_status_t srtp_protect_rtcp(srtp_t ctx, const uint8_t *rtcp,
                                    size_t rtcp_len, uint8_t *srtcp,
                                    size_t *srtcp_len, size_t mki_index)
{
    if (!ctx || !srtcp || !srtcp_len)
        return srtp_err_status_bad_param;
    srtp_err_status_t st;
    srtp_err_status_t rc = srtp_protect_rtcp_batch(
        ctx, 1, &rtcp, &rtcp_len, &srtcp, srtcp_len, &mki_index, &st);
    return rc ? rc : st;
}

/* srtp_unprotect_rtcp, srtp.c:4546-4837: a batch of one */
srtp_err_status_t srtp_unprotect_rtcp(srtp_t ctx, const uint8_t *srtcp,
                                      size_t srtcp_len, uint8_t *rtcp,
                                      size_t *rtcp_len)
{
    if (!ctx || !rtcp || !rtcp_len)
        return srtp_err_status_bad_param;
    srtp_err_status_t st;
    srtp_err_status_t rc = srtp_unprotect_rtcp_batch(
        ctx, 1, &srtcp, &srtcp_len, &rtcp, rtcp_len, &st);
    return rc ? rc : st;
}

/* ------------------------------------------------------------------------
 * policies and profiles (srtp.c:3665-3860, 4848-4970)
 * ---------------------------------------------------------------------- */
static void setp(srtp_crypto_policy_t *p, uint32_t c, size_t ckl, uint32_t a,
                 size_t akl, size_t tag, srtp_sec_serv_t sv)
{
    p->cipher_type = c;
    p->cipher_key_len = ckl;
    p->auth_type = a;
    p->auth_key_len = akl;
    p->auth_tag_len = tag;
    p->sec_serv = sv;
}

void srtp_crypto_policy_set_rtp_default(srtp_crypto_policy_t *p)
{
    setp(p, SRTP_AES_ICM_128, 30, SRTP_HMAC_SHA1, 20, 10, sec_serv_conf_and_auth);
}
void srtp_crypto_policy_set_rtcp_default(srtp_crypto_policy_t *p)
{
    setp(p, SRTP_AES_ICM_128, 30, SRTP_HMAC_SHA1, 20, 10, sec_serv_conf_and_auth);
}
void srtp_crypto_policy_set_aes_cm_128_hmac_sha1_32(srtp_crypto_policy_t *p)
{
    setp(p, SRTP_AES_ICM_128, 30, SRTP_HMAC_SHA1, 20, 4, sec_serv_conf_and_auth);
}
void srtp_crypto_policy_set_aes_cm_128_null_auth(srtp_crypto_policy_t *p)
{
    setp(p, SRTP_AES_ICM_128, 30, SRTP_NULL_AUTH, 0, 0, sec_serv_conf);
}
void srtp_crypto_policy_set_null_cipher_hmac_sha1_80(srtp_crypto_policy_t *p)
{
    setp(p, SRTP_NULL_CIPHER, 30, SRTP_HMAC_SHA1, 20, 10, sec_serv_auth);
}
void srtp_crypto_policy_set_null_cipher_hmac_null(srtp_crypto_policy_t *p)
{
    setp(p, SRTP_NULL_CIPHER, 0, SRTP_NULL_AUTH, 0, 0, sec_serv_none);
}
void srtp_crypto_policy_set_aes_cm_256_hmac_sha1_80(srtp_crypto_policy_t *p)
{
    setp(p, SRTP_AES_ICM_256, 46, SRTP_HMAC_SHA1, 20, 10, sec_serv_conf_and_auth);
}
void srtp_crypto_policy_set_aes_cm_256_hmac_sha1_32(srtp_crypto_policy_t *p)
{
    setp(p, SRTP_AES_ICM_256, 46, SRTP_HMAC_SHA1, 20, 4, sec_serv_conf_and_auth);
}
void srtp_crypto_policy_set_aes_cm_256_null_auth(srtp_crypto_policy_t *p)
{
    setp(p, SRTP_AES_ICM_256, 46, SRTP_NULL_AUTH, 0, 0, sec_serv_conf);
}
void srtp_crypto_policy_set_aes_cm_192_hmac_sha1_80(srtp_crypto_policy_t *p)
{
    setp(p, SRTP_AES_ICM_192, 38, SRTP_HMAC_SHA1, 20, 10, sec_serv_conf_and_auth);
}
void srtp_crypto_policy_set_aes_cm_192_hmac_sha1_32(srtp_crypto_policy_t *p)
{
    setp(p, SRTP_AES_ICM_192, 38, SRTP_HMAC_SHA1, 20, 4, sec_serv_conf_and_auth);
}
void srtp_crypto_policy_set_aes_cm_192_null_auth(srtp_crypto_policy_t *p)
{
    setp(p, SRTP_AES_ICM_192, 38, SRTP_NULL_AUTH, 0, 0, sec_serv_conf);
}
void srtp_crypto_policy_set_aes_gcm_128_16_auth(srtp_crypto_policy_t *p)
{
    setp(p, SRTP_AES_GCM_128, 28, SRTP_NULL_AUTH, 0, 16, sec_serv_conf_and_auth);
}
void srtp_crypto_policy_set_aes_gcm_256_16_auth(srtp_crypto_policy_t *p)
{
    setp(p, SRTP_AES_GCM_256, 44, SRTP_NULL_AUTH, 0, 16, sec_serv_conf_and_auth);
}

srtp_err_status_t srtp_crypto_policy_set_from_profile_for_rtp(
    srtp_crypto_policy_t *policy, srtp_profile_t profile)
{
    switch (profile) {
    case srtp_profile_aes128_cm_sha1_80:
        srtp_crypto_policy_set_rtp_default(policy);
        break;
    case srtp_profile_aes128_cm_sha1_32:
        srtp_crypto_policy_set_aes_cm_128_hmac_sha1_32(policy);
        break;
    case srtp_profile_null_sha1_80:
        srtp_crypto_policy_set_null_cipher_hmac_sha1_80(policy);
        break;
    case srtp_profile_aead_aes_128_gcm:
        srtp_crypto_policy_set_aes_gcm_128_16_auth(policy);
        break;
    case srtp_profile_aead_aes_256_gcm:
        srtp_crypto_policy_set_aes_gcm_256_16_auth(policy);
        break;
    default:
        return srtp_err_status_bad_param;
    }
    return srtp_err_status_ok;
}

srtp_err_status_t srtp_crypto_policy_set_from_profile_for_rtcp(
    srtp_crypto_policy_t *policy, srtp_profile_t profile)
{
    switch (profile) {
    case srtp_profile_aes128_cm_sha1_80:
    case srtp_profile_aes128_cm_sha1_32: /* 32-bit RTCP tags not honoured */
        srtp_crypto_policy_set_rtp_default(policy);
        break;
    case srtp_profile_null_sha1_80:
        srtp_crypto_policy_set_null_cipher_hmac_sha1_80(policy);
        break;
    case srtp_profile_aead_aes_128_gcm:
        srtp_crypto_policy_set_aes_gcm_128_16_auth(policy);
        break;
    case srtp_profile_aead_aes_256_gcm:
        srtp_crypto_policy_set_aes_gcm_256_16_auth(policy);
        break;
    default:
        return srtp_err_status_bad_param;
    }
    return srtp_err_status_ok;
}

void srtp_append_salt_to_key(uint8_t *key, size_t bytes_in_key, uint8_t *salt,
                             size_t bytes_in_salt)
{
    memcpy(key + bytes_in_key, salt, bytes_in_salt);
}

size_t srtp_profile_get_master_key_length(srtp_profile_t profile)
{
    switch (profile) {
    case srtp_profile_aes128_cm_sha1_80:
    case srtp_profile_aes128_cm_sha1_32:
    case srtp_profile_null_sha1_80:
    case srtp_profile_aead_aes_128_gcm:
        return SRTP_AES_128_KEY_LEN;
    case srtp_profile_aead_aes_256_gcm:
        return SRTP_AES_256_KEY_LEN;
    default:
        return 0;
    }
}

size_t srtp_profile_get_master_salt_length(srtp_profile_t profile)
{
    switch (profile) {
    case srtp_profile_aes128_cm_sha1_80:
    case srtp_profile_aes128_cm_sha1_32:
    case srtp_profile_null_sha1_80:
        return SRTP_SALT_LEN;
    case srtp_profile_aead_aes_128_gcm:
    case srtp_profile_aead_aes_256_gcm:
        return SRTP_AEAD_SALT_LEN;
    default:
        return 0;
    }
}

/* ------------------------------------------------------------------------
 * misc
 * ---------------------------------------------------------------------- */
void srtp_set_user_data(srtp_t ctx, void *data) { ctx->user_data = data; }
void *srtp_get_user_data(srtp_t ctx) { return ctx->user_data; }

srtp_err_status_t srtp_install_event_handler(srtp_event_handler_func_t func)
{
    g_event_handler = func; /* NULL allowed, srtp.c:1762-1772 */
    return srtp_err_status_ok;
}

srtp_err_status_t srtp_install_log_handler(srtp_log_handler_func_t func,
                                           void *data)
{
    g_log_handler = func;
    g_log_data = data;
    return srtp_err_status_ok;
}

const char *srtp_get_version_string(void)
{
    return "libsrtp3 3.0.0 (libsrtp_mi355x)";
}

unsigned int srtp_get_version(void) { return (3u << 24) | (0u << 16) | 0u; }

/* the debug-module registry lives with the crypto-kernel registry
 * (srtp_plugin.c; crypto_kernel.c:210-260) */
srtp_err_status_t srtp_mi355x_set_debug_module(const char *name, bool v)
    __attribute__((visibility("hidden")));
void srtp_mi355x_list_debug_modules(void) __attribute__((visibility("hidden")));

srtp_err_status_t srtp_set_debug_module(const char *mod_name, bool v)
{
    return srtp_mi355x_set_debug_module(mod_name, v);
}

srtp_err_status_t srtp_list_debug_modules(void)
{
    srtp_mi355x_list_debug_modules();
    return srtp_err_status_ok;
}

static srtp_err_status_t trailer_of(const srtp_stream_ctx_t *s, int is_rtp,
                                    size_t mki_index, size_t *len)
{
    /* stream_get_protect_trailer_length, srtp.c:4972-5000 */
    const hkey_t *k;
    *len = 0;
    if (s->use_mki) {
        if (mki_index >= s->keys->n)
            return srtp_err_status_bad_mki;
        k = &s->keys->k[mki_index];
        *len += s->mki_size;
    } else {
        k = &s->keys->k[0];
    }
    *len += is_rtp ? k->tag_len : k->rtag_len; /* rtp_auth / rtcp_auth */
    if (!is_rtp)
        *len += 4; /* srtcp_trailer_t */
    return srtp_err_status_ok;
}

static srtp_err_status_t trailer_len(srtp_t ctx, int is_rtp, size_t mki_index,
                                     size_t *length)
{
    if (!ctx)
        return srtp_err_status_bad_param;
    int found = 0;
    size_t best = 0, t;
    if (ctx->templ) {
        found = 1;
        trailer_of(ctx->templ, is_rtp, mki_index, &best);
    }
    for (size_t i = 0; i < ctx->n; i++)
        if (trailer_of(ctx->list[i], is_rtp, mki_index, &t) ==
            srtp_err_status_ok) {
            found = 1;
            if (t > best)
                best = t;
        }
    if (!found)
        return srtp_err_status_bad_param;
    *length = best;
    return srtp_err_status_ok;
}

srtp_err_status_t srtp_get_protect_trailer_length(srtp_t session,
                                                  size_t mki_index,
                                                  size_t *length)
{
    return trailer_len(session, 1, mki_index, length);
}

srtp_err_status_t srtp_get_protect_rtcp_trailer_length(srtp_t session,
                                                       size_t mki_index,
                                                       size_t *length)
{
    return trailer_len(session, 0, mki_index, length);
}

srtp_err_status_t srtp_stream_set_roc(srtp_t session, uint32_t ssrc,
                                      uint32_t roc)
{
    ASYNC_DRAIN_CHECK(session);
    if (session)
        dev_pull(session);
    srtp_stream_ctx_t *s = session ? map_get(session, ssrc) : NULL;
    if (!s)
        return srtp_err_status_bad_param;
    s->rdbx.pending_roc = roc;
    return srtp_err_status_ok;
}

srtp_err_status_t srtp_stream_get_roc(srtp_t session, uint32_t ssrc,
                                      uint32_t *roc)
{
    ASYNC_DRAIN_CHECK(session);
    if (session)
        dev_pull(session);
    srtp_stream_ctx_t *s = session ? map_get(session, ssrc) : NULL;
    if (!s)
        return srtp_err_status_bad_param;
    *roc = (uint32_t)(s->rdbx.index >> 16);
    return srtp_err_status_ok;
}

void srtp_mi355x_set_timing(srtp_t ctx, int on)
{
    if (ctx)
        ctx->timing = on;
}

double srtp_mi355x_last_kernel_ms(srtp_t ctx) { return ctx ? ctx->last_ms : 0; }

int srtp_mi355x_gpu_available(void) { return srtp_gpu_available(); }

void srtp_mi355x_unprotect_stats(srtp_t ctx, uint32_t *rounds,
                                 uint32_t *launches, uint32_t *undo_launches)
{
    if (!ctx)
        return;
    if (rounds)
        *rounds = ctx->ustat.rounds;
    if (launches)
        *launches = ctx->ustat.launches;
    if (undo_launches)
        *undo_launches = ctx->ustat.undo_launches;
}

/* Test hook: the number of uses left on the first session key of stream
 * `ssrc` (host order) -- what a test of the reference writes into the
 * stream's srtp_key_limit_ctx_t to reach the soft / hard limits (key.c:74-90)
 * without 2^48 packets. */
void srtp_gpu_pp_debug_fail_waits(int n);
void srtp_gpu_pp_set_buckets(int on);

void srtp_mi355x_set_key_buckets(int on) { srtp_gpu_pp_set_buckets(on); }

void srtp_mi355x_debug_inject_failure(int what, int count)
{
    if (what == SRTP_MI355X_FAIL_BCAST_ALLOC)
        g_fail_bcast_alloc = count;
    else if (what == SRTP_MI355X_FAIL_VERDICT_WAIT)
        srtp_gpu_pp_debug_fail_waits(count);
    else if (what == SRTP_MI355X_FAIL_ASYNC_DRAIN)
        g_fail_drains = count;
}

srtp_err_status_t srtp_mi355x_debug_set_key_limit(srtp_t ctx, uint32_t ssrc,
                                                  uint64_t num_left)
{
    if (!ctx)
        return srtp_err_status_bad_param;
    dev_pull(ctx);
    srtp_stream_ctx_t *st = map_get(ctx, ssrc);
    if (!st)
        return srtp_err_status_no_ctx;
    st->keys->k[0].num_left = num_left;
    ctx->dt.valid = 0;   /* the device table's key bound is stale */
    return srtp_err_status_ok;
}

srtp_err_status_t srtp_mi355x_debug_key_left(srtp_t ctx, uint32_t ssrc,
                                             size_t j, uint64_t *num_left)
{
    if (!ctx || !num_left)
        return srtp_err_status_bad_param;
    dev_pull(ctx);
    srtp_stream_ctx_t *st = map_get(ctx, ssrc);
    if (!st)
        return srtp_err_status_no_ctx;
    if (j >= st->keys->n)
        return srtp_err_status_bad_param;
    *num_left = st->keys->k[j].num_left;
    return srtp_err_status_ok;
}

uint64_t srtp_mi355x_prepass_sorted_batches(srtp_t ctx)
{
    return ctx ? ctx->dt.sorted_batches : 0;
}

uint64_t srtp_mi355x_bucket_batches(srtp_t ctx)
{
    return ctx ? ctx->dt.bk_batches : 0;
}

void srtp_mi355x_inorder_stats(srtp_t ctx, uint64_t *runs, uint64_t *declines)
{
    if (runs)
        *runs = ctx ? ctx->dt.io_runs : 0;
    if (declines)
        *declines = ctx ? ctx->dt.io_declines : 0;
}

int srtp_mi355x_prepass_last_abort(srtp_t ctx)
{
    return ctx ? ctx->dt.last_abort : 0;
}

void srtp_mi355x_prepass_stats(srtp_t ctx, uint64_t *device_batches,
                               uint64_t *host_batches)
{
    if (device_batches)
        *device_batches = ctx ? ctx->dt.fast_batches : 0;
    if (host_batches)
        *host_batches = ctx ? ctx->dt.host_batches : 0;
}

/* Test hook (no GPU): drives the protect pre-pass index / replay logic of a
 * fresh stream over a sequence of sequence numbers, as srtp_protect would
 * (srtp.c:2662-2690).  pending_roc != 0 emulates srtp_stream_set_roc()
 * before the first packet.  Returns per packet the status and the estimated
 * 48-bit index (0 on error). */
int srtp_mi355x_debug_index(size_t window, int allow_repeat_tx,
                            uint32_t pending_roc, size_t n,
                            const uint16_t *seq, int32_t *status,
                            uint64_t *est_out)
{
    rdbx_t r;
    if (rdbx_init(&r, window ? window : 128))
        return -1;
    r.pending_roc = pending_roc;
    for (size_t i = 0; i < n; i++) {
        uint64_t est = 0;
        int64_t delta = 0;
        srtp_err_status_t rc = estimate(&r, seq[i], &est, &delta);
        est_out[i] = 0;
        if (rc && rc != srtp_err_status_pkt_idx_adv) {
            status[i] = rc;
            continue;
        }
        if (rc == srtp_err_status_pkt_idx_adv) {
            rdbx_accept(&r, est, 0, 1);
        } else {
            rc = rdbx_check(&r, delta);
            if (rc && (rc != srtp_err_status_replay_fail || !allow_repeat_tx)) {
                status[i] = rc;
                continue;
            }
            rdbx_add(&r, delta);
        }
        status[i] = 0;
        est_out[i] = est;
    }
    free(r.w);
    return 0;
}

/* ------------------------------------------------------------------------
 * Session replication (srtp_mi355x_session_export / _import / _broadcast):
 * the multi-GPU sender of SURVEY.md §8(e) keeps one session per GPU; rank
 * root derives the session keys once (srtp_create, srtp.c:1233-1607 on the
 * GPU), every other rank receives them -- the device key records, not the
 * master keys -- with the stream table over RCCL.
 *
 * Blob: header, key sets (the hkey_t fields that are not pointers), streams
 * (policy fields, rdbx index + window words, SRTCP window), then the key
 * records of slots [0, nslots).  Fixed-width little-endian host layout: a
 * blob is read by the same build on the same kind of host.
 * ---------------------------------------------------------------------- */
#define REP_MAGIC "SRTPREP1"

typedef struct {
    char magic[8];
    uint32_t nslots, nkeysets, nstreams, has_templ;
    uint64_t total;
} rep_hdr_t;

typedef struct {
    uint32_t slot, cipher_type, family, rounds, variant, tag_len;
    uint32_t rslot, rtag_len, rgcm, xslot, limit_state, pad;
    uint64_t num_left;
    uint8_t mki[SRTP_MAX_MKI_LEN];
} rep_key_t;

typedef struct {
    uint32_t ssrc, keyset, direction, rtp_services, rtcp_services;
    uint32_t allow_repeat_tx, use_mki, mki_size, window_size, bits;
    uint32_t pending_roc, rtcp_start, rtcp_bm[4];
    uint64_t index;
} rep_stream_t;

typedef struct {
    const keyset_t *ks;
    uint32_t idx;
} rep_kref_t;

static int rep_kref_cmp(const void *a, const void *b)
{
    const uintptr_t x = (uintptr_t)((const rep_kref_t *)a)->ks,
                    y = (uintptr_t)((const rep_kref_t *)b)->ks;
    return x < y ? -1 : x > y;
}

/* by key set, then by the first stream using it */
static int rep_kref_cmp2(const void *a, const void *b)
{
    const int c = rep_kref_cmp(a, b);
    if (c)
        return c;
    const uint32_t x = ((const rep_kref_t *)a)->idx,
                   y = ((const rep_kref_t *)b)->idx;
    return x < y ? -1 : x > y;
}

static int rep_kref_cmp_idx(const void *a, const void *b)
{
    const uint32_t x = ((const rep_kref_t *)a)->idx,
                   y = ((const rep_kref_t *)b)->idx;
    return x < y ? -1 : x > y;
}

/* the streams in blob order: the list (insertion order), then the template */
static srtp_stream_ctx_t *rep_stream_at(srtp_t ctx, size_t i)
{
    return i < ctx->n ? ctx->list[i] : ctx->templ;
}

srtp_err_status_t srtp_mi355x_session_export(srtp_t ctx, void *buf, size_t cap,
                                             size_t *len)
{
    if (!ctx || !len)
        return srtp_err_status_bad_param;
    ASYNC_DRAIN_CHECK(ctx);
    dev_pull(ctx);
    if (kq_flush(ctx))
        return srtp_err_status_fail;
    const size_t ns = ctx->n + (ctx->templ ? 1 : 0);
    /* key sets, each once (template clones share theirs), in the order of
     * the first stream that uses each: the blob does not depend on where
     * the heap put them, so a replica exports the same bytes */
    rep_kref_t *ref = (rep_kref_t *)malloc((ns + 1) * sizeof *ref);
    rep_kref_t *ord = (rep_kref_t *)malloc((ns + 1) * sizeof *ord);
    if (!ref || !ord) {
        free(ref);
        free(ord);
        return srtp_err_status_alloc_fail;
    }
    for (size_t i = 0; i < ns; i++) {
        ref[i].ks = rep_stream_at(ctx, i)->keys;
        ref[i].idx = (uint32_t)i;
    }
    qsort(ref, ns, sizeof *ref, rep_kref_cmp2);
    size_t nk = 0;
    for (size_t i = 0; i < ns; i++)
        if (!nk || ref[nk - 1].ks != ref[i].ks)
            ref[nk++] = ref[i];
    memcpy(ord, ref, nk * sizeof *ord);
    qsort(ord, nk, sizeof *ord, rep_kref_cmp_idx);
    for (size_t k = 0; k < nk; k++) {
        rep_kref_t *e = (rep_kref_t *)bsearch(&ord[k], ref, nk, sizeof *ref,
                                              rep_kref_cmp);
        e->idx = (uint32_t)k;
    }
    size_t total = sizeof(rep_hdr_t), nkeys = 0;
    srtp_err_status_t rc = srtp_err_status_ok;
    for (size_t k = 0; k < nk; k++) {
        const keyset_t *ks = ord[k].ks;
        for (size_t j = 0; j < ks->n; j++)
            if (ks->k[j].variant == SRTP_VARIANT_V)
                rc = srtp_err_status_bad_param; /* keys in host vtables */
        nkeys += ks->n;
    }
    total += nk * 2 * sizeof(uint32_t) + nkeys * sizeof(rep_key_t);
    for (size_t i = 0; i < ns; i++)
        total += sizeof(rep_stream_t) + rep_stream_at(ctx, i)->rdbx.bits / 8;
    const uint32_t nslots = ctx->next_slot;
    total += (size_t)nslots * sizeof(srtp_dev_key_t);
    *len = total;
    if (rc || !buf || cap < total) {
        free(ref);
        free(ord);
        return rc ? rc : (buf ? srtp_err_status_bad_param : srtp_err_status_ok);
    }
    uint8_t *p = (uint8_t *)buf;
    rep_hdr_t h;
    memset(&h, 0, sizeof h);
    memcpy(h.magic, REP_MAGIC, 8);
    h.nslots = nslots;
    h.nkeysets = (uint32_t)nk;
    h.nstreams = (uint32_t)ns;
    h.has_templ = ctx->templ != NULL;
    h.total = total;
    memcpy(p, &h, sizeof h);
    p += sizeof h;
    for (size_t k = 0; k < nk; k++) {
        const keyset_t *ks = ord[k].ks;
        uint32_t w[2] = { (uint32_t)ks->n, (uint32_t)ks->cryptex };
        memcpy(p, w, sizeof w);
        p += sizeof w;
        for (size_t j = 0; j < ks->n; j++) {
            const hkey_t *hk = &ks->k[j];
            rep_key_t r;
            memset(&r, 0, sizeof r);
            r.slot = hk->slot;
            r.cipher_type = hk->cipher_type;
            r.family = hk->family;
            r.rounds = hk->rounds;
            r.variant = hk->variant;
            r.tag_len = (uint32_t)hk->tag_len;
            r.rslot = hk->rslot;
            r.rtag_len = (uint32_t)hk->rtag_len;
            r.rgcm = (uint32_t)hk->rgcm;
            r.xslot = hk->xslot;
            r.limit_state = (uint32_t)hk->limit_state;
            r.num_left = hk->num_left;
            memcpy(r.mki, hk->mki, sizeof r.mki);
            memcpy(p, &r, sizeof r);
            p += sizeof r;
        }
    }
    for (size_t i = 0; i < ns; i++) {
        const srtp_stream_ctx_t *s = rep_stream_at(ctx, i);
        rep_kref_t key = { s->keys, 0 };
        const rep_kref_t *f =
            (const rep_kref_t *)bsearch(&key, ref, nk, sizeof *ref, rep_kref_cmp);
        rep_stream_t r;
        memset(&r, 0, sizeof r);
        r.ssrc = s->ssrc;
        r.keyset = f->idx;
        r.direction = (uint32_t)s->direction;
        r.rtp_services = (uint32_t)s->rtp_services;
        r.rtcp_services = (uint32_t)s->rtcp_services;
        r.allow_repeat_tx = s->allow_repeat_tx;
        r.use_mki = s->use_mki;
        r.mki_size = (uint32_t)s->mki_size;
        r.window_size = (uint32_t)s->window_size;
        r.bits = (uint32_t)s->rdbx.bits;
        r.pending_roc = s->rdbx.pending_roc;
        r.rtcp_start = s->rtcp_start;
        memcpy(r.rtcp_bm, s->rtcp_bm, sizeof r.rtcp_bm);
        r.index = s->rdbx.index;
        memcpy(p, &r, sizeof r);
        p += sizeof r;
        memcpy(p, s->rdbx.w, s->rdbx.bits / 8);
        p += s->rdbx.bits / 8;
    }
    free(ref);
    free(ord);
    if (srtp_gpu_get_keys(ctx->gpu, nslots, (srtp_dev_key_t *)p)) {
        log_msg(srtp_log_level_error, srtp_gpu_last_error());
        return srtp_err_status_fail;
    }
    return srtp_err_status_ok;
}

/* bounds-checked reader over the blob */
typedef struct {
    const uint8_t *p, *end;
} rep_rd_t;

static int rep_take(rep_rd_t *r, void *dst, size_t n)
{
    if ((size_t)(r->end - r->p) < n)
        return -1;
    memcpy(dst, r->p, n);
    r->p += n;
    return 0;
}

static srtp_err_status_t rep_fill(srtp_t ctx, rep_rd_t *rd)
{
    rep_hdr_t h;
    if (rep_take(rd, &h, sizeof h) || memcmp(h.magic, REP_MAGIC, 8) ||
        h.total != (uint64_t)(rd->end - rd->p) + sizeof h ||
        h.nstreams < (h.has_templ ? 1u : 0u))
        return srtp_err_status_bad_param;
    keyset_t **ks = (keyset_t **)calloc(h.nkeysets + 1, sizeof *ks);
    uint8_t *used = (uint8_t *)calloc(h.nslots + 1, 1);
    uint8_t *gh = (uint8_t *)calloc(h.nslots + 1, 1);
    srtp_dev_key_t *recs = NULL;
    srtp_err_status_t rc = srtp_err_status_bad_param;
    if (!ks || !used || !gh)
        goto out_alloc;
    for (uint32_t k = 0; k < h.nkeysets; k++) {
        uint32_t w[2];
        if (rep_take(rd, w, sizeof w) || w[0] == 0 ||
            w[0] > SRTP_MAX_NUM_MASTER_KEYS)
            goto out;
        ks[k] = (keyset_t *)calloc(1, sizeof(keyset_t));
        if (!ks[k])
            goto out_alloc;
        ks[k]->n = w[0];
        ks[k]->cryptex = (int)w[1];
        for (uint32_t j = 0; j < w[0]; j++) {
            rep_key_t r;
            if (rep_take(rd, &r, sizeof r) || r.slot >= h.nslots ||
                (r.rslot != 0xffffffffu && r.rslot >= h.nslots) ||
                (r.xslot != 0xffffffffu && r.xslot >= h.nslots) ||
                r.variant >= SRTP_VARIANT_V)
                goto out;
            hkey_t *hk = &ks[k]->k[j];
            hk->slot = r.slot;
            hk->cipher_type = r.cipher_type;
            hk->family = r.family;
            hk->rounds = r.rounds;
            hk->variant = r.variant;
            hk->tag_len = r.tag_len;
            hk->rslot = r.rslot;
            hk->rtag_len = r.rtag_len;
            hk->rgcm = (int)r.rgcm;
            hk->xslot = r.xslot;
            hk->limit_state = (int)r.limit_state;
            hk->num_left = r.num_left;
            memcpy(hk->mki, r.mki, sizeof hk->mki);
            used[r.slot] = 1;
            gh[r.slot] = r.family == SRTP_DEV_GCM;
            if (r.rslot != 0xffffffffu)
                used[r.rslot] = 1;
            if (r.xslot != 0xffffffffu)
                used[r.xslot] = 1;
            ctx->variant_mask |= 1u << r.variant;
        }
    }
    /* the key records keep their slot numbers: the session's next_slot is
     * the exporter's, the slots no key set uses are free */
    ctx->next_slot = h.nslots;
    for (uint32_t s = 0; s < h.nslots; s++)
        if (!used[s])
            free_slot_now(ctx, s);
    for (uint32_t i = 0; i < h.nstreams; i++) {
        rep_stream_t r;
        if (rep_take(rd, &r, sizeof r) || r.keyset >= h.nkeysets ||
            r.bits == 0 || (r.bits & 31) || r.bits > 0x8000 ||
            r.mki_size > SRTP_MAX_MKI_LEN)
            goto out;
        srtp_stream_ctx_t *s = (srtp_stream_ctx_t *)calloc(1, sizeof *s);
        if (!s || rdbx_init(&s->rdbx, r.bits)) {
            free(s);
            rc = srtp_err_status_alloc_fail;
            goto out;
        }
        s->ssrc = r.ssrc;
        s->direction = (int)r.direction;
        s->rtp_services = (int)r.rtp_services;
        s->rtcp_services = (int)r.rtcp_services;
        s->allow_repeat_tx = r.allow_repeat_tx != 0;
        s->use_mki = r.use_mki != 0;
        s->mki_size = r.mki_size;
        s->window_size = r.window_size;
        s->rdbx.index = r.index;
        s->rdbx.pending_roc = r.pending_roc;
        s->rtcp_start = r.rtcp_start;
        memcpy(s->rtcp_bm, r.rtcp_bm, sizeof s->rtcp_bm);
        s->keys = ks[r.keyset];
        s->keys->refs++;
        if (rep_take(rd, s->rdbx.w, r.bits / 8)) {
            stream_free(ctx, s);
            goto out;
        }
        if (h.has_templ && i + 1 == h.nstreams) {
            ctx->templ = s;
        } else if (list_insert(ctx, s)) {
            stream_free(ctx, s);
            rc = srtp_err_status_alloc_fail;
            goto out;
        }
    }
    /* key sets no stream references would leak: a blob never holds one */
    for (uint32_t k = 0; k < h.nkeysets; k++)
        if (ks[k]->refs == 0)
            goto out;
    recs = (srtp_dev_key_t *)malloc((size_t)h.nslots * sizeof *recs + 1);
    if (!recs) {
        rc = srtp_err_status_alloc_fail;
        goto out;
    }
    if (rep_take(rd, recs, (size_t)h.nslots * sizeof *recs) || rd->p != rd->end)
        goto out;
    for (uint32_t s = 0; s < h.nslots; s++)
        if (gh[s] && recs[s].ghash_slot != s)
            goto out;
    if (srtp_gpu_put_keys(ctx->gpu, h.nslots, recs, gh)) {
        log_msg(srtp_log_level_error, srtp_gpu_last_error());
        rc = srtp_err_status_init_fail;
        goto out;
    }
    rc = srtp_err_status_ok;
    goto done;
out:
out_alloc:
    if (rc == srtp_err_status_ok)
        rc = srtp_err_status_alloc_fail;
    /* key sets without a stream are freed here, the rest with the streams */
    for (uint32_t k = 0; ks && k < h.nkeysets; k++)
        if (ks[k] && ks[k]->refs == 0)
            free(ks[k]);
done:
    free(recs);
    free(ks);
    free(used);
    free(gh);
    return rc;
}

srtp_err_status_t srtp_mi355x_session_import(srtp_t *session, const void *blob,
                                             size_t len)
{
    if (!session || !blob)
        return srtp_err_status_bad_param;
    *session = NULL;
    srtp_t ctx;
    srtp_err_status_t st = srtp_create(&ctx, NULL);
    if (st)
        return st;
    rep_rd_t rd = { (const uint8_t *)blob, (const uint8_t *)blob + len };
    st = rep_fill(ctx, &rd);
    if (st) {
        srtp_dealloc(ctx);
        return st;
    }
    *session = ctx;
    return srtp_err_status_ok;
}

/* RCCL, resolved at run time from a copy the process has ALREADY loaded --
 * the one the caller's communicator comes from (PyTorch's bundled
 * librccl.so, soname librccl.so.1, is loaded privately, so RTLD_DEFAULT does
 * not see it; RTLD_NOLOAD finds it by soname).  A fresh dlopen would be a
 * second library instance, possibly another version, handed a communicator
 * it did not create: no such load is made, the call fails instead. */

typedef int (*rccl_bcast_fn)(const void *, void *, size_t, int, int, void *,
                             void *);
typedef int (*rccl_allred_fn)(const void *, void *, size_t, int, int, void *,
                              void *);
typedef int (*rccl_rank_fn)(void *, int *);
typedef const char *(*rccl_err_fn)(int);

static void *rccl_sym(const char *name)
{
    void *f = dlsym(RTLD_DEFAULT, name);
    if (f)
        return f;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h)
        h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h)
        return NULL;
    f = dlsym(h, name);
    dlclose(h);   /* drops the reference NOLOAD took; the library stays */
    return f;
}

/* Every step below is collective: each rank makes the same sequence of
 * calls whatever happens locally, so no rank is left waiting in RCCL.
 *   1. the root exports; the blob length is broadcast (0: export failed,
 *      every rank returns srtp_err_status_fail);
 *   2. every rank allocates; a max-reduction of the failure flags makes
 *      every rank return srtp_err_status_alloc_fail if any failed;
 *   3. the blob is broadcast, the other ranks import it.
 * Secrets (derived keys, HMAC midstates, salts) are wiped from the host
 * and device copies of the blob on every exit path. */
srtp_err_status_t srtp_mi355x_session_broadcast(srtp_t *session,
                                                void *nccl_comm, int root,
                                                void *stream)
{
    /* rccl.h: ncclUint8 = 1, ncclUint64 = 5, ncclMax = 2 */
    enum { NCCL_UINT8 = 1, NCCL_UINT64 = 5, NCCL_MAX = 2 };
    if (!session || !nccl_comm)
        return srtp_err_status_bad_param;
    rccl_bcast_fn bcast = (rccl_bcast_fn)rccl_sym("ncclBroadcast");
    rccl_allred_fn allred = (rccl_allred_fn)rccl_sym("ncclAllReduce");
    rccl_rank_fn urank = (rccl_rank_fn)rccl_sym("ncclCommUserRank");
    rccl_err_fn estr = (rccl_err_fn)rccl_sym("ncclGetErrorString");
    if (!bcast || !allred || !urank) {
        log_msg(srtp_log_level_error,
                "session broadcast: no RCCL loaded in this process\n");
        return srtp_err_status_init_fail;
    }
    int rank = -1;
    if (urank(nccl_comm, &rank))
        return srtp_err_status_bad_param;
    const int is_root = rank == root;
    srtp_err_status_t st = srtp_err_status_ok;
    uint64_t hlen = 0, flag;
    size_t blen = 0;   /* bytes of blob to wipe */
    uint8_t *blob = NULL, *dblob = NULL;
    uint64_t *dlen = (uint64_t *)srtp_gpu_malloc(sizeof(uint64_t));
    if (!dlen)
        return srtp_err_status_alloc_fail;   /* before any collective: the
                                              * same as RCCL's own allocation
                                              * failures, fatal for the comm */
    if (is_root) {
        size_t n = 0;
        st = *session ? srtp_mi355x_session_export(*session, NULL, 0, &n)
                      : srtp_err_status_bad_param;
        blob = st ? NULL : (uint8_t *)malloc(n);
        blen = blob ? n : 0;
        if (!st && !blob)
            st = srtp_err_status_alloc_fail;
        if (!st)
            st = srtp_mi355x_session_export(*session, blob, n, &n);
        /* a failed export still broadcasts (length 0) so that no rank is
         * left waiting in the collective */
        hlen = st ? 0 : n;
    }
    int nr = 0;
    if (srtp_gpu_h2d(NULL, dlen, &hlen, sizeof hlen, stream) ||
        (nr = bcast(dlen, dlen, sizeof hlen, NCCL_UINT8, root, nccl_comm,
                    stream)) ||
        srtp_gpu_d2h(NULL, &hlen, dlen, sizeof hlen, stream) ||
        srtp_gpu_sync(NULL, stream)) {
        st = srtp_err_status_fail;
        goto out;
    }
    if (!hlen) {
        if (!st)
            st = srtp_err_status_fail;   /* the root's export failed */
        goto out;
    }
    dblob = (uint8_t *)srtp_gpu_malloc(hlen);
    if (!is_root) {
        blob = (uint8_t *)malloc(hlen);
        blen = blob ? hlen : 0;
    }
    flag = (!dblob || !blob) ? 1 : 0;
    if (g_fail_bcast_alloc > 0) {
        g_fail_bcast_alloc--;
        flag = 1;
    }
    if (srtp_gpu_h2d(NULL, dlen, &flag, sizeof flag, stream) ||
        (nr = allred(dlen, dlen, 1, NCCL_UINT64, NCCL_MAX, nccl_comm,
                     stream)) ||
        srtp_gpu_d2h(NULL, &flag, dlen, sizeof flag, stream) ||
        srtp_gpu_sync(NULL, stream)) {
        st = srtp_err_status_fail;
        goto out;
    }
    if (flag) {
        st = srtp_err_status_alloc_fail;   /* on some rank: all return */
        goto out;
    }
    if ((is_root && srtp_gpu_h2d(NULL, dblob, blob, hlen, stream)) ||
        (nr = bcast(dblob, dblob, hlen, NCCL_UINT8, root, nccl_comm, stream)) ||
        (!is_root && srtp_gpu_d2h(NULL, blob, dblob, hlen, stream)) ||
        srtp_gpu_sync(NULL, stream)) {
        st = srtp_err_status_fail;
        goto out;
    }
    if (!is_root)
        st = srtp_mi355x_session_import(session, blob, hlen);
out:
    if (nr && estr) {
        char m[160];
        snprintf(m, sizeof m, "session broadcast: RCCL: %s\n", estr(nr));
        log_msg(srtp_log_level_error, m);
    }
    if (blob) {
        memset(blob, 0, blen);
        free(blob);
    }
    if (dblob) {
        /* the device copy holds the same secrets: cleared before the free
         * (stream-ordered behind any copy still reading it) */
        (void)srtp_gpu_memset(dblob, 0, hlen, stream);
    }
    /* whatever failed above, nothing queued on the caller's stream (the
     * broadcast, a copy, the clear) may still read the buffers freed below */
    if ((dblob || dlen) && srtp_gpu_sync(NULL, stream))
        (void)srtp_gpu_sync(NULL, NULL);
    srtp_gpu_free(dblob);
    srtp_gpu_free(dlen);
    return st;
}
