/*
 * srtp_plugin.c -- libsrtp's crypto-kernel plugin ABI (srtp.def:46-69) on
 * the MI355X engine.
 *
 * The reference lets an application allocate and drive ciphers and auth
 * functions through vtables (crypto/include/cipher.h:60-260,
 * crypto/include/auth.h:55-200, wrappers crypto/cipher/cipher.c:63-140,
 * crypto/hash/auth.c:50-66), self-test them against known answers
 * (cipher.c:150-520, auth.c:68-170) and replace the implementation of an
 * algorithm id (crypto/kernel/crypto_kernel.c:270-440).  Here the built-in
 * types are GPU-backed: each encrypt / decrypt / compute of AES-ICM, AES-GCM
 * and HMAC-SHA1 is one launch of k_raw (srtp_gpu.hip, srtp_gpu_raw) -- the
 * host keeps only the per-object bookkeeping the reference keeps (counter,
 * keystream carry-over, AAD, buffered HMAC input) and the setup-time key
 * schedule / HMAC midstates / GHASH subkey, like srtp_create's KDF.
 *
 * Replacement: srtp_replace_cipher_type / srtp_replace_auth_type run the
 * new type's own self-test and the registered type's known answers, exactly
 * as the reference does, and then hold it in the registry
 * (srtp_mi355x_registered_*_type).  A type that passes the built-in known
 * answers computes the same function, so the packet path keeps its GPU
 * kernels for that algorithm id.
 *
 * Built-in known answers (published vectors, checked against the pinned
 * oracle): AES-ICM-128 RFC 3711 B.2; AES-ICM-192/256 RFC 6188 7.1; AES-GCM
 * "The Galois/Counter Mode of Operation" test cases 4 (128) and 16 (256),
 * tags 16 and 8; HMAC-SHA1 RFC 2202 test case 1.
 */
#include "srtp_mi355x.h"

#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "host_crypto.h"
#include "srtp_dev.h"

/* srtp_host.c: the installed log handler */
void srtp_mi355x_log(int level, const char *msg)
    __attribute__((visibility("hidden")));

#define SALT_ICM 14
#define SALT_GCM 12

/* ------------------------------------------------------------------------
 * the device context of single-buffer calls (one per process)
 * ---------------------------------------------------------------------- */
static pthread_mutex_t g_raw_mu = PTHREAD_MUTEX_INITIALIZER;
static srtp_gpu_t *g_raw;

static srtp_err_status_t raw_call(srtp_gpu_raw_t *r)
{
    pthread_mutex_lock(&g_raw_mu);
    if (!g_raw && srtp_gpu_open(&g_raw)) {
        pthread_mutex_unlock(&g_raw_mu);
        srtp_mi355x_log(0, srtp_gpu_last_error());
        return srtp_err_status_init_fail;
    }
    int rc = srtp_gpu_raw(g_raw, r);
    pthread_mutex_unlock(&g_raw_mu);
    if (rc) {
        srtp_mi355x_log(0, srtp_gpu_last_error());
        return srtp_err_status_cipher_fail;
    }
    return srtp_err_status_ok;
}

/* ------------------------------------------------------------------------
 * AES-ICM (crypto/cipher/aes_icm.c:80-414): key = AES key || 14-byte salt
 * ---------------------------------------------------------------------- */
typedef struct {
    size_t key_size;          /* 30 / 38 / 46 */
    srtp_dev_key_t key;       /* device image: rk, rounds */
    uint8_t offset[16];       /* salt || 00 00 */
    uint8_t counter[16];
    uint8_t ks[16];           /* keystream of the last block */
    size_t bytes_in_buffer;   /* its unused tail */
} icm_state_t;

extern const srtp_cipher_type_t srtp_mi355x_aes_icm_128, srtp_mi355x_aes_icm_192,
    srtp_mi355x_aes_icm_256;

static srtp_err_status_t icm_alloc(srtp_cipher_t **c, size_t key_len,
                                   size_t tlen)
{
    (void)tlen;
    const srtp_cipher_type_t *t;
    if (key_len == 30)
        t = &srtp_mi355x_aes_icm_128;
    else if (key_len == 38)
        t = &srtp_mi355x_aes_icm_192;
    else if (key_len == 46)
        t = &srtp_mi355x_aes_icm_256;
    else
        return srtp_err_status_bad_param;
    *c = (srtp_cipher_t *)calloc(1, sizeof(srtp_cipher_t));
    icm_state_t *s = (icm_state_t *)calloc(1, sizeof(icm_state_t));
    if (!*c || !s) {
        free(*c);
        free(s);
        *c = NULL;
        return srtp_err_status_alloc_fail;
    }
    s->key_size = key_len;
    (*c)->type = t;
    (*c)->state = s;
    (*c)->key_len = key_len;
    (*c)->algorithm = t->id;
    return srtp_err_status_ok;
}

static srtp_err_status_t icm_dealloc(srtp_cipher_t *c)
{
    if (c->state) {
        memset(c->state, 0, sizeof(icm_state_t));
        free(c->state);
    }
    memset(c, 0, sizeof *c);
    free(c);
    return srtp_err_status_ok;
}

static srtp_err_status_t icm_init(void *sv, const uint8_t *key)
{
    icm_state_t *s = (icm_state_t *)sv;
    const size_t base = s->key_size - SALT_ICM;
    hc_aes_t a;
    if (hc_aes_init(&a, key, base))
        return srtp_err_status_bad_param;
    memset(&s->key, 0, sizeof s->key);
    memcpy(s->key.rk, a.rk, sizeof a.rk);
    s->key.rounds = (uint32_t)a.rounds;
    memset(s->offset, 0, 16);
    memcpy(s->offset, key + base, SALT_ICM);
    memcpy(s->counter, s->offset, 16);
    s->bytes_in_buffer = 0;
    return srtp_err_status_ok;
}

static srtp_err_status_t icm_set_iv(void *sv, uint8_t *iv,
                                    srtp_cipher_direction_t dir)
{
    (void)dir;
    icm_state_t *s = (icm_state_t *)sv;
    for (int i = 0; i < 16; i++)
        s->counter[i] = s->offset[i] ^ iv[i];
    s->bytes_in_buffer = 0;
    return srtp_err_status_ok;
}

static srtp_err_status_t icm_encrypt(void *sv, const uint8_t *src,
                                     size_t src_len, uint8_t *dst,
                                     size_t *dst_len)
{
    icm_state_t *s = (icm_state_t *)sv;
    if (*dst_len < src_len)
        return srtp_err_status_buffer_small;
    *dst_len = src_len;
    const size_t lead = src_len < s->bytes_in_buffer ? src_len
                                                     : s->bytes_in_buffer;
    const size_t body = src_len - lead;
    const size_t nb = (body + 15) / 16;
    const uint32_t c16 = (uint32_t)s->counter[14] << 8 | s->counter[15];
    /* at most 0xffff keystream blocks per IV (aes_icm.c:317-322) */
    if (nb + c16 > 0xffff)
        return srtp_err_status_terminus;
    if (!src_len)
        return srtp_err_status_ok;
    srtp_gpu_raw_t r;
    memset(&r, 0, sizeof r);
    r.op = SRTP_RAW_ICM;
    r.key = &s->key;
    r.src = src;
    r.dst = dst;
    r.len = src_len;
    memcpy(r.ctr, s->counter, 16);
    memcpy(r.lead, s->ks + (16 - s->bytes_in_buffer), lead);
    r.nlead = (uint32_t)lead;
    srtp_err_status_t st = raw_call(&r);
    if (st)
        return st;
    s->bytes_in_buffer -= lead;
    if (nb) {
        const uint32_t c = c16 + (uint32_t)nb;
        s->counter[14] = (uint8_t)(c >> 8);
        s->counter[15] = (uint8_t)c;
        memcpy(s->ks, r.ks_last, 16);
        s->bytes_in_buffer = (body & 15) ? 16 - (body & 15) : 0;
    }
    return srtp_err_status_ok;
}

/* ------------------------------------------------------------------------
 * AES-GCM (crypto/cipher/aes_gcm_ossl.c:80-389): key = AES key || 12-byte
 * salt (the salt is SRTP's, not the cipher's); encrypt appends the tag,
 * decrypt verifies it
 * ---------------------------------------------------------------------- */
typedef struct {
    size_t key_size;          /* 16 / 32 */
    uint32_t tag_len;
    srtp_dev_key_t key;       /* rk, rounds, h */
    uint8_t iv[12];
    srtp_cipher_direction_t dir;
    uint8_t *aad;
    size_t aad_len, aad_cap;
} gcm_state_t;

extern const srtp_cipher_type_t srtp_mi355x_aes_gcm_128, srtp_mi355x_aes_gcm_256;

static srtp_err_status_t gcm_alloc(srtp_cipher_t **c, size_t key_len,
                                   size_t tlen)
{
    const srtp_cipher_type_t *t;
    if (key_len == 16 + SALT_GCM)
        t = &srtp_mi355x_aes_gcm_128;
    else if (key_len == 32 + SALT_GCM)
        t = &srtp_mi355x_aes_gcm_256;
    else
        return srtp_err_status_bad_param;
    if (tlen != 16 && tlen != 8)
        return srtp_err_status_bad_param;
    *c = (srtp_cipher_t *)calloc(1, sizeof(srtp_cipher_t));
    gcm_state_t *s = (gcm_state_t *)calloc(1, sizeof(gcm_state_t));
    if (!*c || !s) {
        free(*c);
        free(s);
        *c = NULL;
        return srtp_err_status_alloc_fail;
    }
    s->key_size = key_len - SALT_GCM;
    s->tag_len = (uint32_t)tlen;
    s->dir = srtp_direction_any;
    (*c)->type = t;
    (*c)->state = s;
    (*c)->key_len = key_len;
    (*c)->algorithm = t->id;
    return srtp_err_status_ok;
}

static srtp_err_status_t gcm_dealloc(srtp_cipher_t *c)
{
    gcm_state_t *s = (gcm_state_t *)c->state;
    if (s) {
        free(s->aad);
        memset(s, 0, sizeof *s);
        free(s);
    }
    memset(c, 0, sizeof *c);
    free(c);
    return srtp_err_status_ok;
}

static srtp_err_status_t gcm_init(void *sv, const uint8_t *key)
{
    gcm_state_t *s = (gcm_state_t *)sv;
    hc_aes_t a;
    if (hc_aes_init(&a, key, s->key_size))
        return srtp_err_status_bad_param;
    memset(&s->key, 0, sizeof s->key);
    memcpy(s->key.rk, a.rk, sizeof a.rk);
    s->key.rounds = (uint32_t)a.rounds;
    /* the hash subkey E_K(0^128), a setup-time block like the KDF's */
    uint8_t zero[16] = { 0 }, h[16];
    hc_aes_block(&a, zero, h);
    for (int w = 0; w < 4; w++)
        s->key.h[w] = (uint32_t)h[4 * w] << 24 | (uint32_t)h[4 * w + 1] << 16 |
                      (uint32_t)h[4 * w + 2] << 8 | h[4 * w + 3];
    s->dir = srtp_direction_any;
    s->aad_len = 0;
    return srtp_err_status_ok;
}

static srtp_err_status_t gcm_set_iv(void *sv, uint8_t *iv,
                                    srtp_cipher_direction_t dir)
{
    gcm_state_t *s = (gcm_state_t *)sv;
    if (dir != srtp_direction_encrypt && dir != srtp_direction_decrypt)
        return srtp_err_status_bad_param;
    s->dir = dir;
    memcpy(s->iv, iv, 12);
    s->aad_len = 0;   /* a new IV starts a new message */
    return srtp_err_status_ok;
}

static srtp_err_status_t gcm_set_aad(void *sv, const uint8_t *aad,
                                     size_t aad_len)
{
    gcm_state_t *s = (gcm_state_t *)sv;
    if (s->aad_len + aad_len > s->aad_cap) {
        size_t nc = s->aad_cap ? 2 * s->aad_cap : 64;
        while (nc < s->aad_len + aad_len)
            nc *= 2;
        uint8_t *p = (uint8_t *)realloc(s->aad, nc);
        if (!p)
            return srtp_err_status_alloc_fail;
        s->aad = p;
        s->aad_cap = nc;
    }
    if (aad_len)
        memcpy(s->aad + s->aad_len, aad, aad_len);
    s->aad_len += aad_len;
    return srtp_err_status_ok;
}

static srtp_err_status_t gcm_run(gcm_state_t *s, int op, const uint8_t *src,
                                 size_t len, uint8_t *dst, int *ok)
{
    srtp_gpu_raw_t r;
    memset(&r, 0, sizeof r);
    r.op = op;
    r.key = &s->key;
    r.src = src;
    r.dst = dst;
    r.len = len;
    memcpy(r.iv, s->iv, 12);
    r.aad = s->aad;
    r.aad_len = s->aad_len;
    r.tag_len = s->tag_len;
    srtp_err_status_t st = raw_call(&r);
    s->aad_len = 0;
    if (ok)
        *ok = r.ok;
    return st;
}

static srtp_err_status_t gcm_encrypt(void *sv, const uint8_t *src,
                                     size_t src_len, uint8_t *dst,
                                     size_t *dst_len)
{
    gcm_state_t *s = (gcm_state_t *)sv;
    if (s->dir != srtp_direction_encrypt)
        return srtp_err_status_bad_param;
    if (*dst_len < src_len + s->tag_len)
        return srtp_err_status_buffer_small;
    srtp_err_status_t st = gcm_run(s, SRTP_RAW_GCM_SEAL, src, src_len, dst,
                                   NULL);
    if (st)
        return srtp_err_status_algo_fail;
    *dst_len = src_len + s->tag_len;
    return srtp_err_status_ok;
}

static srtp_err_status_t gcm_decrypt(void *sv, const uint8_t *src,
                                     size_t src_len, uint8_t *dst,
                                     size_t *dst_len)
{
    gcm_state_t *s = (gcm_state_t *)sv;
    if (s->dir != srtp_direction_decrypt)
        return srtp_err_status_bad_param;
    if (src_len < s->tag_len)
        return srtp_err_status_bad_param;
    if (*dst_len < src_len - s->tag_len)
        return srtp_err_status_buffer_small;
    int ok = 0;
    srtp_err_status_t st = gcm_run(s, SRTP_RAW_GCM_OPEN, src,
                                   src_len - s->tag_len, dst, &ok);
    if (st)
        return srtp_err_status_algo_fail;
    *dst_len = src_len - s->tag_len;
    return ok ? srtp_err_status_ok : srtp_err_status_auth_fail;
}

/* ------------------------------------------------------------------------
 * null cipher (crypto/cipher/null_cipher.c:55-120)
 * ---------------------------------------------------------------------- */
extern const srtp_cipher_type_t srtp_mi355x_null_cipher;

static srtp_err_status_t null_alloc(srtp_cipher_t **c, size_t key_len,
                                    size_t tlen)
{
    (void)tlen;
    *c = (srtp_cipher_t *)calloc(1, sizeof(srtp_cipher_t));
    if (!*c)
        return srtp_err_status_alloc_fail;
    (*c)->algorithm = SRTP_NULL_CIPHER;
    (*c)->type = &srtp_mi355x_null_cipher;
    (*c)->state = (void *)0x1; /* stateless, like the reference */
    (*c)->key_len = key_len;
    return srtp_err_status_ok;
}

static srtp_err_status_t null_dealloc(srtp_cipher_t *c)
{
    memset(c, 0, sizeof *c);
    free(c);
    return srtp_err_status_ok;
}

static srtp_err_status_t null_init(void *sv, const uint8_t *key)
{
    (void)sv;
    (void)key;
    return srtp_err_status_ok;
}

static srtp_err_status_t null_set_iv(void *sv, uint8_t *iv,
                                     srtp_cipher_direction_t dir)
{
    (void)sv;
    (void)iv;
    (void)dir;
    return srtp_err_status_ok;
}

static srtp_err_status_t null_encrypt(void *sv, const uint8_t *src,
                                      size_t src_len, uint8_t *dst,
                                      size_t *dst_len)
{
    (void)sv;
    if (src != dst) {
        if (*dst_len < src_len)
            return srtp_err_status_buffer_small;
        memcpy(dst, src, src_len);
    }
    *dst_len = src_len;
    return srtp_err_status_ok;
}

/* ------------------------------------------------------------------------
 * HMAC-SHA1 (crypto/hash/hmac.c:60-229): the input is buffered on the host
 * between start / update and hashed on the GPU by compute
 * ---------------------------------------------------------------------- */
typedef struct {
    srtp_dev_key_t key;       /* ipad / opad midstates */
    uint8_t *buf;
    size_t len, cap;
} hmac_state_t;

extern const srtp_auth_type_t srtp_mi355x_hmac, srtp_mi355x_null_auth;

static srtp_err_status_t hmac_alloc(srtp_auth_t **a, size_t key_len,
                                    size_t out_len)
{
    if (key_len > 20 || out_len > 20)
        return srtp_err_status_bad_param;
    *a = (srtp_auth_t *)calloc(1, sizeof(srtp_auth_t));
    hmac_state_t *s = (hmac_state_t *)calloc(1, sizeof(hmac_state_t));
    if (!*a || !s) {
        free(*a);
        free(s);
        *a = NULL;
        return srtp_err_status_alloc_fail;
    }
    (*a)->type = &srtp_mi355x_hmac;
    (*a)->state = s;
    (*a)->out_len = out_len;
    (*a)->key_len = key_len;
    (*a)->prefix_len = 0;
    return srtp_err_status_ok;
}

static srtp_err_status_t hmac_dealloc(srtp_auth_t *a)
{
    hmac_state_t *s = (hmac_state_t *)a->state;
    if (s) {
        free(s->buf);
        memset(s, 0, sizeof *s);
        free(s);
    }
    memset(a, 0, sizeof *a);
    free(a);
    return srtp_err_status_ok;
}

static srtp_err_status_t hmac_init(void *sv, const uint8_t *key,
                                   size_t key_len)
{
    hmac_state_t *s = (hmac_state_t *)sv;
    if (key_len > 20)
        return srtp_err_status_bad_param;
    uint8_t ip[64], op[64];
    for (int i = 0; i < 64; i++) {
        const uint8_t k = i < (int)key_len ? key[i] : 0;
        ip[i] = k ^ 0x36;
        op[i] = k ^ 0x5c;
    }
    memset(&s->key, 0, sizeof s->key);
    hc_sha1_midstate(ip, s->key.ipad);
    hc_sha1_midstate(op, s->key.opad);
    s->len = 0;
    return srtp_err_status_ok;
}

static srtp_err_status_t hmac_start(void *sv)
{
    ((hmac_state_t *)sv)->len = 0;
    return srtp_err_status_ok;
}

static srtp_err_status_t hmac_update(void *sv, const uint8_t *buf, size_t n)
{
    hmac_state_t *s = (hmac_state_t *)sv;
    if (s->len + n > s->cap) {
        size_t nc = s->cap ? 2 * s->cap : 256;
        while (nc < s->len + n)
            nc *= 2;
        uint8_t *p = (uint8_t *)realloc(s->buf, nc);
        if (!p)
            return srtp_err_status_alloc_fail;
        s->buf = p;
        s->cap = nc;
    }
    if (n)
        memcpy(s->buf + s->len, buf, n);
    s->len += n;
    return srtp_err_status_ok;
}

static srtp_err_status_t hmac_compute(void *sv, const uint8_t *buf, size_t n,
                                      size_t tag_len, uint8_t *tag)
{
    hmac_state_t *s = (hmac_state_t *)sv;
    if (tag_len > 20)
        return srtp_err_status_bad_param;
    srtp_err_status_t st = hmac_update(sv, buf, n);
    if (st)
        return st;
    uint8_t mac[20];
    srtp_gpu_raw_t r;
    memset(&r, 0, sizeof r);
    r.op = SRTP_RAW_HMAC;
    r.key = &s->key;
    r.src = s->buf;
    r.dst = mac;
    r.len = s->len;
    st = raw_call(&r);
    s->len = 0;
    if (st)
        return srtp_err_status_auth_fail;
    memcpy(tag, mac, tag_len);
    return srtp_err_status_ok;
}

/* null auth (crypto/hash/null_auth.c) */
static srtp_err_status_t nauth_alloc(srtp_auth_t **a, size_t key_len,
                                     size_t out_len)
{
    *a = (srtp_auth_t *)calloc(1, sizeof(srtp_auth_t));
    if (!*a)
        return srtp_err_status_alloc_fail;
    (*a)->type = &srtp_mi355x_null_auth;
    (*a)->state = (void *)0x1;
    (*a)->out_len = out_len;
    (*a)->key_len = key_len;
    (*a)->prefix_len = out_len;
    return srtp_err_status_ok;
}

static srtp_err_status_t nauth_dealloc(srtp_auth_t *a)
{
    memset(a, 0, sizeof *a);
    free(a);
    return srtp_err_status_ok;
}

static srtp_err_status_t nauth_init(void *sv, const uint8_t *key, size_t n)
{
    (void)sv;
    (void)key;
    (void)n;
    return srtp_err_status_ok;
}

static srtp_err_status_t nauth_compute(void *sv, const uint8_t *buf, size_t n,
                                       size_t tag_len, uint8_t *tag)
{
    (void)sv;
    (void)buf;
    (void)n;
    (void)tag_len;
    (void)tag;
    return srtp_err_status_ok;
}

static srtp_err_status_t nauth_update(void *sv, const uint8_t *buf, size_t n)
{
    (void)sv;
    (void)buf;
    (void)n;
    return srtp_err_status_ok;
}

static srtp_err_status_t nauth_start(void *sv)
{
    (void)sv;
    return srtp_err_status_ok;
}

/* ------------------------------------------------------------------------
 * built-in known answers
 * ---------------------------------------------------------------------- */
static const uint8_t kat_icm_salt[14] = { 0xf0, 0xf1, 0xf2, 0xf3, 0xf4,
                                          0xf5, 0xf6, 0xf7, 0xf8, 0xf9,
                                          0xfa, 0xfb, 0xfc, 0xfd };
static uint8_t kat_zero16[16];
static const uint8_t kat_zero32[32];

/* RFC 3711 B.2 */
static const uint8_t kat_icm128_key[30] = {
    0x2b, 0x7e, 0x15, 0x16, 0x28, 0xae, 0xd2, 0xa6, 0xab, 0xf7, 0x15, 0x88,
    0x09, 0xcf, 0x4f, 0x3c, 0xf0, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7,
    0xf8, 0xf9, 0xfa, 0xfb, 0xfc, 0xfd
};
static const uint8_t kat_icm128_ks[32] = {
    0xe0, 0x3e, 0xad, 0x09, 0x35, 0xc9, 0x5e, 0x80, 0xe1, 0x66, 0xb1,
    0x6d, 0xd9, 0x2b, 0x4e, 0xb4, 0xd2, 0x35, 0x13, 0x16, 0x2b, 0x02,
    0xd0, 0xf7, 0x2a, 0x43, 0xa2, 0xfe, 0x4a, 0x5f, 0x97, 0xab
};
/* RFC 6188 7.1 (AES-192 / AES-256 counter mode) */
static uint8_t kat_icm192_key[38];
static const uint8_t kat_icm192_aes[24] = {
    0xea, 0xb2, 0x34, 0x76, 0x4e, 0x51, 0x7b, 0x2d, 0x3d, 0x16, 0x0d, 0x58,
    0x7d, 0x8c, 0x86, 0x21, 0x97, 0x40, 0xf6, 0x5f, 0x99, 0xb6, 0xbc, 0xf7
};
static const uint8_t kat_icm192_ks[32] = {
    0x35, 0x09, 0x6c, 0xba, 0x46, 0x10, 0x02, 0x8d, 0xc1, 0xb5, 0x75,
    0x03, 0x80, 0x4c, 0xe3, 0x7c, 0x5d, 0xe9, 0x86, 0x29, 0x1d, 0xcc,
    0xe1, 0x61, 0xd5, 0x16, 0x5e, 0xc4, 0x56, 0x8f, 0x5c, 0x9a
};
static uint8_t kat_icm256_key[46];
static const uint8_t kat_icm256_aes[32] = {
    0x57, 0xf8, 0x2f, 0xe3, 0x61, 0x3f, 0xd1, 0x70, 0xa8, 0x5e, 0xc9,
    0x3c, 0x40, 0xb1, 0xf0, 0x92, 0x2e, 0xc4, 0xcb, 0x0d, 0xc0, 0x25,
    0xb5, 0x82, 0x72, 0x14, 0x7c, 0xc4, 0x38, 0x94, 0x4a, 0x98
};
static const uint8_t kat_icm256_ks[32] = {
    0x92, 0xbd, 0xd2, 0x8a, 0x93, 0xc3, 0xf5, 0x25, 0x11, 0xc6, 0x77,
    0xd0, 0x8b, 0x55, 0x15, 0xa4, 0x9d, 0xa7, 0x1b, 0x23, 0x78, 0xa8,
    0x54, 0xf6, 0x70, 0x50, 0x75, 0x6d, 0xed, 0x16, 0x5b, 0xac
};

/* GCM test cases 4 and 16: key (|| 12 zero salt bytes), IV, AAD, P, C||T */
static uint8_t kat_gcm128_key[28], kat_gcm256_key[44];
static const uint8_t kat_gcm_k16[16] = { 0xfe, 0xff, 0xe9, 0x92, 0x86, 0x65,
                                         0x73, 0x1c, 0x6d, 0x6a, 0x8f, 0x94,
                                         0x67, 0x30, 0x83, 0x08 };
static uint8_t kat_gcm_iv[12] = { 0xca, 0xfe, 0xba, 0xbe, 0xfa, 0xce,
                                  0xdb, 0xad, 0xde, 0xca, 0xf8, 0x88 };
static const uint8_t kat_gcm_aad[20] = { 0xfe, 0xed, 0xfa, 0xce, 0xde,
                                         0xad, 0xbe, 0xef, 0xfe, 0xed,
                                         0xfa, 0xce, 0xde, 0xad, 0xbe,
                                         0xef, 0xab, 0xad, 0xda, 0xd2 };
static const uint8_t kat_gcm_pt[60] = {
    0xd9, 0x31, 0x32, 0x25, 0xf8, 0x84, 0x06, 0xe5, 0xa5, 0x59, 0x09, 0xc5,
    0xaf, 0xf5, 0x26, 0x9a, 0x86, 0xa7, 0xa9, 0x53, 0x15, 0x34, 0xf7, 0xda,
    0x2e, 0x4c, 0x30, 0x3d, 0x8a, 0x31, 0x8a, 0x72, 0x1c, 0x3c, 0x0c, 0x95,
    0x95, 0x68, 0x09, 0x53, 0x2f, 0xcf, 0x0e, 0x24, 0x49, 0xa6, 0xb5, 0x25,
    0xb1, 0x6a, 0xed, 0xf5, 0xaa, 0x0d, 0xe6, 0x57, 0xba, 0x63, 0x7b, 0x39
};
static const uint8_t kat_gcm128_ct[76] = {
    0x42, 0x83, 0x1e, 0xc2, 0x21, 0x77, 0x74, 0x24, 0x4b, 0x72, 0x21, 0xb7,
    0x84, 0xd0, 0xd4, 0x9c, 0xe3, 0xaa, 0x21, 0x2f, 0x2c, 0x02, 0xa4, 0xe0,
    0x35, 0xc1, 0x7e, 0x23, 0x29, 0xac, 0xa1, 0x2e, 0x21, 0xd5, 0x14, 0xb2,
    0x54, 0x66, 0x93, 0x1c, 0x7d, 0x8f, 0x6a, 0x5a, 0xac, 0x84, 0xaa, 0x05,
    0x1b, 0xa3, 0x0b, 0x39, 0x6a, 0x0a, 0xac, 0x97, 0x3d, 0x58, 0xe0, 0x91,
    0x5b, 0xc9, 0x4f, 0xbc, 0x32, 0x21, 0xa5, 0xdb, 0x94, 0xfa, 0xe9, 0x5a,
    0xe7, 0x12, 0x1a, 0x47
};
static const uint8_t kat_gcm256_ct[76] = {
    0x52, 0x2d, 0xc1, 0xf0, 0x99, 0x56, 0x7d, 0x07, 0xf4, 0x7f, 0x37, 0xa3,
    0x2a, 0x84, 0x42, 0x7d, 0x64, 0x3a, 0x8c, 0xdc, 0xbf, 0xe5, 0xc0, 0xc9,
    0x75, 0x98, 0xa2, 0xbd, 0x25, 0x55, 0xd1, 0xaa, 0x8c, 0xb0, 0x8e, 0x48,
    0x59, 0x0d, 0xbb, 0x3d, 0xa7, 0xb0, 0x8b, 0x10, 0x56, 0x82, 0x88, 0x38,
    0xc5, 0xf6, 0x1e, 0x63, 0x93, 0xba, 0x7a, 0x0a, 0xbc, 0xc9, 0xf6, 0x62,
    0x76, 0xfc, 0x6e, 0xce, 0x0f, 0x4e, 0x17, 0x68, 0xcd, 0xdf, 0x88, 0x53,
    0xbb, 0x2d, 0x55, 0x1b
};
/* the same with an 8-byte tag: 60 bytes of ciphertext, then 8 of the tag */
static uint8_t kat_gcm128_ct8[68], kat_gcm256_ct8[68];

/* RFC 2202 test case 1 */
static const uint8_t kat_hmac_key[20] = { 0x0b, 0x0b, 0x0b, 0x0b, 0x0b,
                                          0x0b, 0x0b, 0x0b, 0x0b, 0x0b,
                                          0x0b, 0x0b, 0x0b, 0x0b, 0x0b,
                                          0x0b, 0x0b, 0x0b, 0x0b, 0x0b };
static const uint8_t kat_hmac_data[8] = { 'H', 'i', ' ', 'T', 'h', 'e', 'r',
                                          'e' };
static const uint8_t kat_hmac_tag[20] = { 0xb6, 0x17, 0x31, 0x86, 0x55,
                                          0x05, 0x72, 0x64, 0xe2, 0x8b,
                                          0xc0, 0xb6, 0xfb, 0x37, 0x8c,
                                          0x8e, 0xf1, 0x46, 0xbe, 0x00 };

static srtp_cipher_test_case_t tc_icm128 = { 30, kat_icm128_key, kat_zero16,
                                             32, kat_zero32, 32, kat_icm128_ks,
                                             0, NULL, 0, NULL };
static srtp_cipher_test_case_t tc_icm192 = { 38, kat_icm192_key, kat_zero16,
                                             32, kat_zero32, 32, kat_icm192_ks,
                                             0, NULL, 0, NULL };
static srtp_cipher_test_case_t tc_icm256 = { 46, kat_icm256_key, kat_zero16,
                                             32, kat_zero32, 32, kat_icm256_ks,
                                             0, NULL, 0, NULL };
static srtp_cipher_test_case_t tc_gcm128_8 = {
    28, kat_gcm128_key, kat_gcm_iv, 60, kat_gcm_pt, 68, kat_gcm128_ct8,
    20, kat_gcm_aad, 8, NULL
};
static srtp_cipher_test_case_t tc_gcm128 = {
    28, kat_gcm128_key, kat_gcm_iv, 60, kat_gcm_pt, 76, kat_gcm128_ct,
    20, kat_gcm_aad, 16, &tc_gcm128_8
};
static srtp_cipher_test_case_t tc_gcm256_8 = {
    44, kat_gcm256_key, kat_gcm_iv, 60, kat_gcm_pt, 68, kat_gcm256_ct8,
    20, kat_gcm_aad, 8, NULL
};
static srtp_cipher_test_case_t tc_gcm256 = {
    44, kat_gcm256_key, kat_gcm_iv, 60, kat_gcm_pt, 76, kat_gcm256_ct,
    20, kat_gcm_aad, 16, &tc_gcm256_8
};
static const srtp_cipher_test_case_t tc_null = { 0, NULL, NULL, 0, NULL, 0,
                                                 NULL, 0, NULL, 0, NULL };
static const srtp_auth_test_case_t tc_hmac = { 20, kat_hmac_key, 8,
                                               kat_hmac_data, 20, kat_hmac_tag,
                                               NULL };
static const srtp_auth_test_case_t tc_nauth = { 0, NULL, 0, NULL, 0, NULL,
                                                NULL };

static void kat_setup(void)
{
    memcpy(kat_icm192_key, kat_icm192_aes, 24);
    memcpy(kat_icm192_key + 24, kat_icm_salt, 14);
    memcpy(kat_icm256_key, kat_icm256_aes, 32);
    memcpy(kat_icm256_key + 32, kat_icm_salt, 14);
    memcpy(kat_gcm128_key, kat_gcm_k16, 16);
    memcpy(kat_gcm256_key, kat_gcm_k16, 16);
    memcpy(kat_gcm256_key + 16, kat_gcm_k16, 16);
    memcpy(kat_gcm128_ct8, kat_gcm128_ct, 68);
    memcpy(kat_gcm256_ct8, kat_gcm256_ct, 68);
}

const srtp_cipher_type_t srtp_mi355x_aes_icm_128 = {
    icm_alloc, icm_dealloc, icm_init, NULL, icm_encrypt, icm_encrypt,
    icm_set_iv, "AES-128 integer counter mode (MI355X)", &tc_icm128,
    SRTP_AES_ICM_128
};
const srtp_cipher_type_t srtp_mi355x_aes_icm_192 = {
    icm_alloc, icm_dealloc, icm_init, NULL, icm_encrypt, icm_encrypt,
    icm_set_iv, "AES-192 integer counter mode (MI355X)", &tc_icm192,
    SRTP_AES_ICM_192
};
const srtp_cipher_type_t srtp_mi355x_aes_icm_256 = {
    icm_alloc, icm_dealloc, icm_init, NULL, icm_encrypt, icm_encrypt,
    icm_set_iv, "AES-256 integer counter mode (MI355X)", &tc_icm256,
    SRTP_AES_ICM_256
};
const srtp_cipher_type_t srtp_mi355x_aes_gcm_128 = {
    gcm_alloc, gcm_dealloc, gcm_init, gcm_set_aad, gcm_encrypt, gcm_decrypt,
    gcm_set_iv, "AES-128 GCM (MI355X)", &tc_gcm128, SRTP_AES_GCM_128
};
const srtp_cipher_type_t srtp_mi355x_aes_gcm_256 = {
    gcm_alloc, gcm_dealloc, gcm_init, gcm_set_aad, gcm_encrypt, gcm_decrypt,
    gcm_set_iv, "AES-256 GCM (MI355X)", &tc_gcm256, SRTP_AES_GCM_256
};
const srtp_cipher_type_t srtp_mi355x_null_cipher = {
    null_alloc, null_dealloc, null_init, NULL, null_encrypt, null_encrypt,
    null_set_iv, "null cipher", &tc_null, SRTP_NULL_CIPHER
};
const srtp_auth_type_t srtp_mi355x_hmac = {
    hmac_alloc, hmac_dealloc, hmac_init, hmac_compute, hmac_update,
    hmac_start, "hmac sha-1 authentication function (MI355X)", &tc_hmac,
    SRTP_HMAC_SHA1
};
const srtp_auth_type_t srtp_mi355x_null_auth = {
    nauth_alloc, nauth_dealloc, nauth_init, nauth_compute, nauth_update,
    nauth_start, "null authentication function", &tc_nauth, SRTP_NULL_AUTH
};

/* ------------------------------------------------------------------------
 * the registry (crypto_kernel.c:270-440)
 * ---------------------------------------------------------------------- */
typedef struct ctype_node {
    const srtp_cipher_type_t *t;
    srtp_cipher_type_id_t id;
    struct ctype_node *next;
} ctype_node_t;
typedef struct atype_node {
    const srtp_auth_type_t *t;
    srtp_auth_type_id_t id;
    struct atype_node *next;
} atype_node_t;
typedef struct dmod_node {
    srtp_debug_module_t *m;
    struct dmod_node *next;
} dmod_node_t;

static pthread_mutex_t g_reg_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_once_t g_reg_once = PTHREAD_ONCE_INIT;
static ctype_node_t *g_ctypes;
static atype_node_t *g_atypes;
static dmod_node_t *g_dmods;

static const srtp_cipher_type_t *const k_builtin_ciphers[] = {
    &srtp_mi355x_null_cipher, &srtp_mi355x_aes_icm_128,
    &srtp_mi355x_aes_icm_192, &srtp_mi355x_aes_icm_256,
    &srtp_mi355x_aes_gcm_128, &srtp_mi355x_aes_gcm_256
};
static const srtp_auth_type_t *const k_builtin_auths[] = {
    &srtp_mi355x_null_auth, &srtp_mi355x_hmac
};

/* the debug modules of the reference's kernel (crypto_kernel.c:93-160) */
static srtp_debug_module_t g_mod_names[] = {
    { false, "crypto kernel" }, { false, "auth func" }, { false, "cipher" },
    { false, "alloc" },         { false, "aes icm" },   { false, "aes gcm" },
    { false, "hmac sha-1" },    { false, "srtp" }
};

static void reg_init(void)
{
    kat_setup();
    /* the built-ins are loaded without running their tests: those launch
     * GPU work, and registration happens on first use of the registry
     * (srtp_cipher_type_self_test runs them on demand) */
    for (size_t i = 0; i < sizeof k_builtin_ciphers / sizeof *k_builtin_ciphers;
         i++) {
        ctype_node_t *n = (ctype_node_t *)calloc(1, sizeof *n);
        if (!n)
            return;
        n->t = k_builtin_ciphers[i];
        n->id = n->t->id;
        n->next = g_ctypes;
        g_ctypes = n;
    }
    for (size_t i = 0; i < sizeof k_builtin_auths / sizeof *k_builtin_auths;
         i++) {
        atype_node_t *n = (atype_node_t *)calloc(1, sizeof *n);
        if (!n)
            return;
        n->t = k_builtin_auths[i];
        n->id = n->t->id;
        n->next = g_atypes;
        g_atypes = n;
    }
    for (size_t i = 0; i < sizeof g_mod_names / sizeof *g_mod_names; i++) {
        dmod_node_t *n = (dmod_node_t *)calloc(1, sizeof *n);
        if (!n)
            return;
        n->m = &g_mod_names[i];
        n->next = g_dmods;
        g_dmods = n;
    }
}

static void reg_ready(void) { pthread_once(&g_reg_once, reg_init); }

const srtp_cipher_type_t *srtp_mi355x_builtin_cipher_type(
    srtp_cipher_type_id_t id)
{
    reg_ready();
    for (size_t i = 0; i < sizeof k_builtin_ciphers / sizeof *k_builtin_ciphers;
         i++)
        if (k_builtin_ciphers[i]->id == id)
            return k_builtin_ciphers[i];
    return NULL;
}

const srtp_auth_type_t *srtp_mi355x_builtin_auth_type(srtp_auth_type_id_t id)
{
    reg_ready();
    for (size_t i = 0; i < sizeof k_builtin_auths / sizeof *k_builtin_auths;
         i++)
        if (k_builtin_auths[i]->id == id)
            return k_builtin_auths[i];
    return NULL;
}

const srtp_cipher_type_t *srtp_mi355x_registered_cipher_type(
    srtp_cipher_type_id_t id)
{
    reg_ready();
    pthread_mutex_lock(&g_reg_mu);
    const srtp_cipher_type_t *t = NULL;
    for (ctype_node_t *n = g_ctypes; n; n = n->next)
        if (n->id == id) {
            t = n->t;
            break;
        }
    pthread_mutex_unlock(&g_reg_mu);
    return t;
}

const srtp_auth_type_t *srtp_mi355x_registered_auth_type(srtp_auth_type_id_t id)
{
    reg_ready();
    pthread_mutex_lock(&g_reg_mu);
    const srtp_auth_type_t *t = NULL;
    for (atype_node_t *n = g_atypes; n; n = n->next)
        if (n->id == id) {
            t = n->t;
            break;
        }
    pthread_mutex_unlock(&g_reg_mu);
    return t;
}

srtp_err_status_t srtp_replace_cipher_type(const srtp_cipher_type_t *ct,
                                           srtp_cipher_type_id_t id)
{
    reg_ready();
    if (!ct || ct->id != id)
        return srtp_err_status_bad_param;
    srtp_err_status_t st = srtp_cipher_type_self_test(ct);
    if (st)
        return st;
    pthread_mutex_lock(&g_reg_mu);
    ctype_node_t *hit = NULL;
    for (ctype_node_t *n = g_ctypes; n; n = n->next) {
        if (n->id == id) {
            hit = n;
            break;
        }
        if (n->t == ct) {
            pthread_mutex_unlock(&g_reg_mu);
            return srtp_err_status_bad_param;
        }
    }
    const srtp_cipher_test_case_t *old = hit ? hit->t->test_data : NULL;
    pthread_mutex_unlock(&g_reg_mu);
    if (hit) {
        st = srtp_cipher_type_test(ct, old);
        if (st)
            return st;
    }
    pthread_mutex_lock(&g_reg_mu);
    if (!hit) {
        hit = (ctype_node_t *)calloc(1, sizeof *hit);
        if (!hit) {
            pthread_mutex_unlock(&g_reg_mu);
            return srtp_err_status_alloc_fail;
        }
        hit->next = g_ctypes;
        g_ctypes = hit;
    }
    hit->t = ct;
    hit->id = id;
    pthread_mutex_unlock(&g_reg_mu);
    return srtp_err_status_ok;
}

srtp_err_status_t srtp_replace_auth_type(const srtp_auth_type_t *at,
                                         srtp_auth_type_id_t id)
{
    reg_ready();
    if (!at || at->id != id)
        return srtp_err_status_bad_param;
    srtp_err_status_t st = srtp_auth_type_self_test(at);
    if (st)
        return st;
    pthread_mutex_lock(&g_reg_mu);
    atype_node_t *hit = NULL;
    for (atype_node_t *n = g_atypes; n; n = n->next) {
        if (n->id == id) {
            hit = n;
            break;
        }
        if (n->t == at) {
            pthread_mutex_unlock(&g_reg_mu);
            return srtp_err_status_bad_param;
        }
    }
    const srtp_auth_test_case_t *old = hit ? hit->t->test_data : NULL;
    pthread_mutex_unlock(&g_reg_mu);
    if (hit) {
        st = srtp_auth_type_test(at, old);
        if (st)
            return st;
    }
    pthread_mutex_lock(&g_reg_mu);
    if (!hit) {
        hit = (atype_node_t *)calloc(1, sizeof *hit);
        if (!hit) {
            pthread_mutex_unlock(&g_reg_mu);
            return srtp_err_status_alloc_fail;
        }
        hit->next = g_atypes;
        g_atypes = hit;
    }
    hit->t = at;
    hit->id = id;
    pthread_mutex_unlock(&g_reg_mu);
    return srtp_err_status_ok;
}

srtp_err_status_t srtp_crypto_kernel_load_debug_module(
    srtp_debug_module_t *new_dm)
{
    reg_ready();
    if (!new_dm || !new_dm->name)
        return srtp_err_status_bad_param;
    pthread_mutex_lock(&g_reg_mu);
    for (dmod_node_t *n = g_dmods; n; n = n->next)
        if (n->m == new_dm || strncmp(new_dm->name, n->m->name, 64) == 0) {
            pthread_mutex_unlock(&g_reg_mu);
            return srtp_err_status_bad_param;
        }
    dmod_node_t *n = (dmod_node_t *)calloc(1, sizeof *n);
    if (!n) {
        pthread_mutex_unlock(&g_reg_mu);
        return srtp_err_status_alloc_fail;
    }
    n->m = new_dm;
    n->next = g_dmods;
    g_dmods = n;
    pthread_mutex_unlock(&g_reg_mu);
    return srtp_err_status_ok;
}

/* srtp_set_debug_module / srtp_list_debug_modules (srtp.c:4903-4921 over
 * crypto_kernel.c:210-260) */
srtp_err_status_t srtp_mi355x_set_debug_module(const char *name, bool v)
    __attribute__((visibility("hidden")));
srtp_err_status_t srtp_mi355x_set_debug_module(const char *name, bool v)
{
    reg_ready();
    if (!name)
        return srtp_err_status_bad_param;
    srtp_err_status_t st = srtp_err_status_fail;
    pthread_mutex_lock(&g_reg_mu);
    for (dmod_node_t *n = g_dmods; n; n = n->next)
        if (strncmp(name, n->m->name, 64) == 0) {
            n->m->on = v;
            st = srtp_err_status_ok;
            break;
        }
    pthread_mutex_unlock(&g_reg_mu);
    return st;
}

void srtp_mi355x_list_debug_modules(void) __attribute__((visibility("hidden")));
void srtp_mi355x_list_debug_modules(void)
{
    reg_ready();
    char line[128];
    pthread_mutex_lock(&g_reg_mu);
    for (dmod_node_t *n = g_dmods; n; n = n->next) {
        snprintf(line, sizeof line, "  %s %s", n->m->name,
                 n->m->on ? "(on)" : "(off)");
        srtp_mi355x_log(3, line);
    }
    pthread_mutex_unlock(&g_reg_mu);
}

/* ------------------------------------------------------------------------
 * the cipher / auth wrappers (cipher.c:63-140, auth.c:50-66)
 * ---------------------------------------------------------------------- */
srtp_err_status_t srtp_cipher_type_alloc(const srtp_cipher_type_t *ct,
                                         srtp_cipher_t **c, size_t key_len,
                                         size_t tlen)
{
    if (!ct || !ct->alloc)
        return srtp_err_status_bad_param;
    return ct->alloc(c, key_len, tlen);
}

srtp_err_status_t srtp_cipher_dealloc(srtp_cipher_t *c)
{
    if (!c || !c->type)
        return srtp_err_status_bad_param;
    return c->type->dealloc(c);
}

srtp_err_status_t srtp_cipher_init(srtp_cipher_t *c, const uint8_t *key)
{
    if (!c || !c->type || !c->state)
        return srtp_err_status_bad_param;
    return c->type->init(c->state, key);
}

srtp_err_status_t srtp_cipher_set_iv(srtp_cipher_t *c, uint8_t *iv,
                                     srtp_cipher_direction_t direction)
{
    if (!c || !c->type || !c->state)
        return srtp_err_status_bad_param;
    return c->type->set_iv(c->state, iv, direction);
}

srtp_err_status_t srtp_cipher_output(srtp_cipher_t *c, uint8_t *buffer,
                                     size_t *num_octets_to_output)
{
    memset(buffer, 0, *num_octets_to_output);
    return c->type->encrypt(c->state, buffer, *num_octets_to_output, buffer,
                            num_octets_to_output);
}

srtp_err_status_t srtp_cipher_encrypt(srtp_cipher_t *c, const uint8_t *src,
                                      size_t src_len, uint8_t *dst,
                                      size_t *dst_len)
{
    if (!c || !c->type || !c->state)
        return srtp_err_status_bad_param;
    return c->type->encrypt(c->state, src, src_len, dst, dst_len);
}

srtp_err_status_t srtp_cipher_decrypt(srtp_cipher_t *c, const uint8_t *src,
                                      size_t src_len, uint8_t *dst,
                                      size_t *dst_len)
{
    if (!c || !c->type || !c->state)
        return srtp_err_status_bad_param;
    return c->type->decrypt(c->state, src, src_len, dst, dst_len);
}

srtp_err_status_t srtp_cipher_set_aad(srtp_cipher_t *c, const uint8_t *aad,
                                      size_t aad_len)
{
    if (!c || !c->type || !c->state)
        return srtp_err_status_bad_param;
    if (!c->type->set_aad)
        return srtp_err_status_no_such_op;
    return c->type->set_aad(c->state, aad, aad_len);
}

size_t srtp_cipher_get_key_length(const srtp_cipher_t *c)
{
    return c->key_len;
}

size_t srtp_auth_get_key_length(const srtp_auth_t *a) { return a->key_len; }
size_t srtp_auth_get_tag_length(const srtp_auth_t *a) { return a->out_len; }
size_t srtp_auth_get_prefix_length(const srtp_auth_t *a)
{
    return a->prefix_len;
}

/* ------------------------------------------------------------------------
 * known-answer and invertibility tests (cipher.c:150-520, auth.c:68-170)
 * ---------------------------------------------------------------------- */
#define SELF_TEST_BUF_OCTETS 128
#define NUM_RAND_TESTS 128
#define MAX_KEY_LEN 64

static int is_gcm(const srtp_cipher_t *c)
{
    return c->algorithm == SRTP_AES_GCM_128 || c->algorithm == SRTP_AES_GCM_256;
}

/* one direction of a known answer: init, IV, AAD, run, compare */
static srtp_err_status_t kat_run(srtp_cipher_t *c,
                                 const srtp_cipher_test_case_t *tc,
                                 srtp_cipher_direction_t dir)
{
    uint8_t buf[SELF_TEST_BUF_OCTETS];
    const size_t in_len = dir == srtp_direction_encrypt
                              ? tc->plaintext_length_octets
                              : tc->ciphertext_length_octets;
    const uint8_t *in = dir == srtp_direction_encrypt ? tc->plaintext
                                                      : tc->ciphertext;
    const size_t want_len = dir == srtp_direction_encrypt
                                ? tc->ciphertext_length_octets
                                : tc->plaintext_length_octets;
    const uint8_t *want = dir == srtp_direction_encrypt ? tc->ciphertext
                                                        : tc->plaintext;
    srtp_err_status_t st = srtp_cipher_init(c, tc->key);
    if (st)
        return st;
    if (tc->ciphertext_length_octets > SELF_TEST_BUF_OCTETS)
        return srtp_err_status_bad_param;
    if (in_len)
        memcpy(buf, in, in_len);
    st = srtp_cipher_set_iv(c, tc->idx, dir);
    if (st)
        return st;
    if (is_gcm(c)) {
        st = srtp_cipher_set_aad(c, tc->aad, tc->aad_length_octets);
        if (st)
            return st;
    }
    size_t len = sizeof buf;
    st = dir == srtp_direction_encrypt
             ? srtp_cipher_encrypt(c, buf, in_len, buf, &len)
             : srtp_cipher_decrypt(c, buf, in_len, buf, &len);
    if (st)
        return st;
    if (len != want_len)
        return srtp_err_status_algo_fail;
    for (size_t k = 0; k < want_len; k++)
        if (buf[k] != want[k])
            return srtp_err_status_algo_fail;
    return srtp_err_status_ok;
}

static void rand_bytes(uint8_t *p, size_t n)
{
    /* the reference's srtp_cipher_rand_for_tests (cipher.c:165-181) */
    while (n--)
        *p++ = (uint8_t)(rand() & 0xff);
}

srtp_err_status_t srtp_cipher_type_test(
    const srtp_cipher_type_t *ct, const srtp_cipher_test_case_t *test_data)
{
    reg_ready();
    const srtp_cipher_test_case_t *tc = test_data;
    srtp_cipher_t *c;
    srtp_err_status_t st;
    if (!ct || !tc)
        return srtp_err_status_cant_check;
    for (; tc; tc = tc->next_test_case) {
        st = srtp_cipher_type_alloc(ct, &c, tc->key_length_octets,
                                    tc->tag_length_octets);
        if (st)
            return st;
        st = kat_run(c, tc, srtp_direction_encrypt);
        if (!st)
            st = kat_run(c, tc, srtp_direction_decrypt);
        srtp_err_status_t st2 = srtp_cipher_dealloc(c);
        if (st)
            return st;
        if (st2)
            return st2;
    }
    /* random invertibility tests with the first case's parameters */
    tc = test_data;
    st = srtp_cipher_type_alloc(ct, &c, tc->key_length_octets,
                                tc->tag_length_octets);
    if (st)
        return st;
    for (size_t j = 0; j < NUM_RAND_TESTS; j++) {
        uint8_t buf[SELF_TEST_BUF_OCTETS], buf2[SELF_TEST_BUF_OCTETS];
        uint8_t key[MAX_KEY_LEN];
        uint32_t r;
        rand_bytes((uint8_t *)&r, sizeof r);
        const size_t pt_len = r % (SELF_TEST_BUF_OCTETS - 64);
        rand_bytes(buf, pt_len);
        memcpy(buf2, buf, pt_len);
        if (tc->key_length_octets > MAX_KEY_LEN) {
            srtp_cipher_dealloc(c);
            return srtp_err_status_cant_check;
        }
        rand_bytes(key, tc->key_length_octets);
        size_t enc_len = sizeof buf, dec_len = sizeof buf;
        st = srtp_cipher_init(c, key);
        if (!st)
            st = srtp_cipher_set_iv(c, tc->idx, srtp_direction_encrypt);
        if (!st && is_gcm(c))
            st = srtp_cipher_set_aad(c, tc->aad, tc->aad_length_octets);
        if (!st)
            st = srtp_cipher_encrypt(c, buf, pt_len, buf, &enc_len);
        if (!st)
            st = srtp_cipher_init(c, key);
        if (!st)
            st = srtp_cipher_set_iv(c, tc->idx, srtp_direction_decrypt);
        if (!st && is_gcm(c))
            st = srtp_cipher_set_aad(c, tc->aad, tc->aad_length_octets);
        if (!st)
            st = srtp_cipher_decrypt(c, buf, enc_len, buf, &dec_len);
        if (!st && (dec_len != pt_len || memcmp(buf, buf2, pt_len)))
            st = srtp_err_status_algo_fail;
        if (st) {
            srtp_cipher_dealloc(c);
            return st;
        }
    }
    return srtp_cipher_dealloc(c);
}

srtp_err_status_t srtp_cipher_type_self_test(const srtp_cipher_type_t *ct)
{
    if (!ct)
        return srtp_err_status_bad_param;
    return srtp_cipher_type_test(ct, ct->test_data);
}

srtp_err_status_t srtp_auth_type_test(const srtp_auth_type_t *at,
                                      const srtp_auth_test_case_t *test_data)
{
    reg_ready();
    if (!at || !test_data)
        return srtp_err_status_cant_check;
    for (const srtp_auth_test_case_t *tc = test_data; tc;
         tc = tc->next_test_case) {
        uint8_t tag[32];
        srtp_auth_t *a;
        if (tc->tag_length_octets > sizeof tag)
            return srtp_err_status_bad_param;
        srtp_err_status_t st = srtp_auth_type_alloc(at, &a,
                                                    tc->key_length_octets,
                                                    tc->tag_length_octets);
        if (st)
            return st;
        st = srtp_auth_init(a, tc->key);
        if (!st)
            st = srtp_auth_start(a);
        memset(tag, 0, tc->tag_length_octets);
        if (!st)
            st = srtp_auth_compute(a, tc->data, tc->data_length_octets, tag);
        if (!st)
            for (size_t i = 0; i < tc->tag_length_octets; i++)
                if (tag[i] != tc->tag[i])
                    st = srtp_err_status_algo_fail;
        srtp_err_status_t st2 = srtp_auth_dealloc(a);
        if (st)
            return st;
        if (st2)
            return st2;
    }
    return srtp_err_status_ok;
}

srtp_err_status_t srtp_auth_type_self_test(const srtp_auth_type_t *at)
{
    if (!at)
        return srtp_err_status_bad_param;
    return srtp_auth_type_test(at, at->test_data);
}

/* cipher.c:550-600: encryptions of a buffer per second, in bits */
uint64_t srtp_cipher_bits_per_second(srtp_cipher_t *c, size_t octets_in_buffer,
                                     size_t num_trials)
{
    uint8_t *buf = (uint8_t *)calloc(1, octets_in_buffer + 64);
    if (!buf)
        return 0;
    uint8_t nonce[16];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (size_t i = 0; i < num_trials; i++) {
        memset(nonce, 0, sizeof nonce);
        memcpy(nonce + 8, &i, sizeof i < 8 ? sizeof i : 8);
        if (srtp_cipher_set_iv(c, nonce, srtp_direction_encrypt)) {
            free(buf);
            return 0;
        }
        if (is_gcm(c) && srtp_cipher_set_aad(c, buf, 0)) {
            free(buf);
            return 0;
        }
        size_t len = octets_in_buffer + 64;
        if (srtp_cipher_encrypt(c, buf, octets_in_buffer, buf, &len)) {
            free(buf);
            return 0;
        }
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(buf);
    const double s = (double)(t1.tv_sec - t0.tv_sec) +
                     1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    if (s <= 0)
        return 0;
    return (uint64_t)((double)num_trials * (double)octets_in_buffer * 8.0 / s);
}

/* ------------------------------------------------------------------------
 * utilities exported with the plugin ABI
 * ---------------------------------------------------------------------- */
/* datatypes.c:89-107: hex of up to 511 octets in a static buffer */
char *srtp_octet_string_hex_string(const void *s, size_t length)
{
    static char buf[1024];
    static const char hx[] = "0123456789abcdef";
    const uint8_t *p = (const uint8_t *)s;
    size_t n = length * 2 < sizeof buf - 1 ? length : (sizeof buf - 1) / 2;
    for (size_t i = 0; i < n; i++) {
        buf[2 * i] = hx[p[i] >> 4];
        buf[2 * i + 1] = hx[p[i] & 15];
    }
    buf[2 * n] = 0;
    return buf;
}

/* datatypes.c:321-333: the running time depends only on len */
bool srtp_octet_string_equal(const uint8_t *a, const uint8_t *b, size_t len)
{
    uint8_t acc = 0;
    for (size_t i = 0; i < len; i++)
        acc |= a[i] ^ b[i];
    return acc == 0;
}

/* rdbx.c:207-210 */
size_t srtp_rdbx_get_window_size(const srtp_rdbx_t *rdbx)
{
    return rdbx->bitmask.length;
}

/* err.c:79-110 */
void srtp_err_report(srtp_err_reporting_level_t level, const char *format, ...)
{
    char msg[512];
    va_list args;
    va_start(args, format);
    vsnprintf(msg, sizeof msg, format, args);
    va_end(args);
    srtp_mi355x_log((int)level, msg);
}
