/*
 * gen_golden.c -- emits tests/golden/*.json by driving the REFERENCE
 * (cisco/libsrtp built from /root/reference sources into oracle/_ref/ by
 * Makefile.ref).  Test infrastructure: run in the build container only
 * (`make -f oracle/Makefile.golden`); its outputs are committed as data
 * fixtures so the GPU box never needs /root/reference.
 *
 * Built twice: without REF_OSSL against libsrtp_ref_int.so (internal crypto
 * kernel: AES-ICM-128/256, HMAC-SHA1, SHA-1, AES block) and with REF_OSSL
 * against libsrtp_ref_ossl.so (adds AES-GCM-128/256 and AES-ICM-192).
 *
 * All inputs are generated from splitmix64 with fixed seeds; nothing here is
 * transcribed from the reference except the srtp_driver.c test keys and the
 * published packet KATs of test/srtp_driver.c (srtp_validate*, empty
 * payload: see k_kats), which anchor the fixture to the reference's own
 * known answers -- the generator exits 1 unless the build reproduces them.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

#include "srtp.h"
#include "srtp_priv.h"
#include "cipher.h"
#include "auth.h"
#include "crypto_kernel.h"
#ifndef REF_OSSL
#include "aes.h"
#include "sha1.h"
#endif

static uint64_t g_rng = 0x5352545030303031ULL; /* "SRTP0001" */
static uint64_t rng(void)
{
    uint64_t z = (g_rng += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
static void rfill(uint8_t *p, size_t n)
{
    for (size_t i = 0; i < n; i++)
        p[i] = (uint8_t)rng();
}

static FILE *g_out;
static int g_first_item;

static void hex(const uint8_t *p, size_t n)
{
    fputc('"', g_out);
    for (size_t i = 0; i < n; i++)
        fprintf(g_out, "%02x", p[i]);
    fputc('"', g_out);
}

static void item_begin(void)
{
    fputs(g_first_item ? "\n    {" : ",\n    {", g_out);
    g_first_item = 0;
}

/* ---------------------------------------------------------------------- */
#ifndef REF_OSSL
static void gen_aes(void)
{
    static const size_t klens[] = { 16, 32 };
    fputs("  \"aes\": [", g_out);
    g_first_item = 1;
    for (int k = 0; k < 2; k++)
        for (int t = 0; t < 8; t++) {
            uint8_t key[32];
            v128_t blk;
            srtp_aes_expanded_key_t ek;
            rfill(key, klens[k]);
            rfill(blk.v8, 16);
            uint8_t in[16];
            memcpy(in, blk.v8, 16);
            srtp_aes_expand_encryption_key(key, klens[k], &ek);
            srtp_aes_encrypt(&blk, &ek);
            item_begin();
            fputs("\"key\": ", g_out);
            hex(key, klens[k]);
            fputs(", \"in\": ", g_out);
            hex(in, 16);
            fputs(", \"out\": ", g_out);
            hex(blk.v8, 16);
            fputs("}", g_out);
        }
    fputs("\n  ],\n", g_out);
}

static void gen_sha1(void)
{
    static const size_t lens[] = { 0,  1,  3,   55,  56,  57,  60,   63,
                                   64, 65, 100, 119, 120, 127, 128, 200,
                                   1000, 1416 };
    fputs("  \"sha1\": [", g_out);
    g_first_item = 1;
    for (size_t i = 0; i < sizeof(lens) / sizeof(lens[0]); i++) {
        uint8_t msg[1500];
        uint32_t h[5];
        uint8_t d[20];
        srtp_sha1_ctx_t ctx;
        rfill(msg, lens[i]);
        srtp_sha1_init(&ctx);
        srtp_sha1_update(&ctx, msg, lens[i]);
        srtp_sha1_final(&ctx, h);
        memcpy(d, h, 20); /* srtp_sha1_final writes big-endian words */
        item_begin();
        fputs("\"msg\": ", g_out);
        hex(msg, lens[i]);
        fputs(", \"digest\": ", g_out);
        hex(d, 20);
        fputs("}", g_out);
    }
    fputs("\n  ],\n", g_out);
}

static void gen_hmac(void)
{
    static const size_t lens[] = { 0, 4, 28, 64, 172, 1416 };
    fputs("  \"hmac\": [", g_out);
    g_first_item = 1;
    for (size_t i = 0; i < sizeof(lens) / sizeof(lens[0]); i++) {
        srtp_auth_t *a;
        uint8_t key[20], msg[1500], tag[20];
        size_t klen = i == 0 ? 16 : 20;
        rfill(key, klen);
        rfill(msg, lens[i]);
        srtp_crypto_kernel_alloc_auth(SRTP_HMAC_SHA1, &a, klen, 20);
        srtp_auth_init(a, key);
        srtp_auth_start(a);
        srtp_auth_compute(a, msg, lens[i], tag);
        srtp_auth_dealloc(a);
        item_begin();
        fputs("\"key\": ", g_out);
        hex(key, klen);
        fputs(", \"msg\": ", g_out);
        hex(msg, lens[i]);
        fputs(", \"tag\": ", g_out);
        hex(tag, 20);
        fputs("}", g_out);
    }
    fputs("\n  ],\n", g_out);
}
#endif

/* AES-ICM through the cipher vtable (aes_icm.c or aes_icm_ossl.c). */
static void gen_icm(const char *name, srtp_cipher_type_id_t id, size_t klen)
{
    static const size_t lens[] = { 0, 1, 15, 16, 17, 100, 1400 };
    fprintf(g_out, "  \"%s\": [", name);
    g_first_item = 1;
    for (size_t i = 0; i < sizeof(lens) / sizeof(lens[0]); i++) {
        srtp_cipher_t *c;
        uint8_t key[46], iv[16], buf[1500], in[1500];
        size_t n = lens[i];
        rfill(key, klen);
        rfill(iv, 16);
        iv[14] = 0;
        iv[15] = (uint8_t)(i == 6 ? 0xf0 : 0); /* exercise the byte carry */
        rfill(in, n);
        memcpy(buf, in, n);
        srtp_crypto_kernel_alloc_cipher(id, &c, klen, 0);
        srtp_cipher_init(c, key);
        srtp_cipher_set_iv(c, iv, srtp_direction_encrypt);
        size_t out_len = n;
        srtp_cipher_encrypt(c, buf, n, buf, &out_len);
        srtp_cipher_dealloc(c);
        item_begin();
        fputs("\"key\": ", g_out);
        hex(key, klen);
        fputs(", \"iv\": ", g_out);
        hex(iv, 16);
        fputs(", \"in\": ", g_out);
        hex(in, n);
        fputs(", \"out\": ", g_out);
        hex(buf, n);
        fputs("}", g_out);
    }
    fputs("\n  ],\n", g_out);
}

#ifdef REF_OSSL
static void gen_gcm(const char *name, srtp_cipher_type_id_t id, size_t klen,
                    size_t tag_len)
{
    static const size_t lens[] = { 0, 1, 16, 17, 160, 1400 };
    static const size_t aads[] = { 12, 12, 16, 20, 0, 12 };
    fprintf(g_out, "  \"%s\": [", name);
    g_first_item = 1;
    for (size_t i = 0; i < sizeof(lens) / sizeof(lens[0]); i++) {
        srtp_cipher_t *c;
        uint8_t key[32 + 12], iv[16] = { 0 }, aad[32], pt[1500],
                                   out[1500 + 16];
        size_t n = lens[i], kb = klen - 12;
        rfill(key, klen);
        rfill(iv, 12);
        rfill(aad, aads[i]);
        rfill(pt, n);
        srtp_crypto_kernel_alloc_cipher(id, &c, klen, tag_len);
        srtp_cipher_init(c, key);
        srtp_cipher_set_iv(c, iv, srtp_direction_encrypt);
        srtp_cipher_set_aad(c, aad, aads[i]);
        size_t out_len = sizeof out;
        srtp_cipher_encrypt(c, pt, n, out, &out_len);
        srtp_cipher_dealloc(c);
        item_begin();
        fputs("\"key\": ", g_out);
        hex(key, kb);
        fputs(", \"iv\": ", g_out);
        hex(iv, 12);
        fputs(", \"aad\": ", g_out);
        hex(aad, aads[i]);
        fputs(", \"in\": ", g_out);
        hex(pt, n);
        fprintf(g_out, ", \"tag_len\": %zu, \"out\": ", tag_len);
        hex(out, out_len);
        fputs("}", g_out);
    }
    fputs("\n  ],\n", g_out);
}
#endif

/* ---------------------------------------------------------------------- */
/* Packet-level cases: sequences of srtp_protect / srtp_unprotect calls.   */

typedef struct {
    const char *name;
    void (*set)(srtp_crypto_policy_t *);
    size_t tag_override; /* 0 = keep */
    size_t nkeys;
    size_t mki_size;
    size_t window;
    int allow_repeat_tx;
    srtp_ssrc_type_t snd_type, rcv_type;
    const uint8_t *fixed_key; /* srtp_driver.c key, or NULL for random */
    size_t fixed_key_len;
} policy_desc_t;

/* master keys of test/srtp_driver.c:5844-5867 and 6139-6146 */
static const uint8_t k_test_key[46] = {
    0xe1, 0xf9, 0x7a, 0x0d, 0x3e, 0x01, 0x8b, 0xe0, 0xd6, 0x4f, 0xa3, 0x2c,
    0x06, 0xde, 0x41, 0x39, 0x0e, 0xc6, 0x75, 0xad, 0x49, 0x8a, 0xfe, 0xeb,
    0xb6, 0x96, 0x0b, 0x3a, 0xab, 0xe6, 0xc1, 0x73, 0xc3, 0x17, 0xf2, 0xda,
    0xbe, 0x35, 0x77, 0x93, 0xb6, 0x96, 0x0b, 0x3a, 0xab, 0xe6
};
static const uint8_t k_test_256_key[46] = {
    0xf0, 0xf0, 0x49, 0x14, 0xb5, 0x13, 0xf2, 0x76, 0x3a, 0x1b, 0x1f, 0xa1,
    0x30, 0xf1, 0x0e, 0x29, 0x98, 0xf6, 0xf6, 0xe4, 0x3e, 0x43, 0x09, 0xd1,
    0xe6, 0x22, 0xa0, 0xe3, 0x32, 0xb9, 0xf1, 0xb6, 0x3b, 0x04, 0x80, 0x3d,
    0xe5, 0x1e, 0xe7, 0xc9, 0x64, 0x23, 0xab, 0x5b, 0x78, 0xd2
};
static const uint8_t k_test_key_gcm[28] = {
    0x00, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07, 0x08, 0x09,
    0x0a, 0x0b, 0x0c, 0x0d, 0x0e, 0x0f, 0xa0, 0xa1, 0xa2, 0xa3,
    0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xab
};
/* expected ciphertext of srtp_validate(), test/srtp_driver.c:2356-2362 */
static const uint8_t k_validate_ct[38] = {
    0x80, 0x0f, 0x12, 0x34, 0xde, 0xca, 0xfb, 0xad, 0xca, 0xfe,
    0xba, 0xbe, 0x4e, 0x55, 0xdc, 0x4c, 0xe7, 0x99, 0x78, 0xd8,
    0x8c, 0xa4, 0xd2, 0x15, 0x94, 0x9d, 0x24, 0x02, 0xb7, 0x8d,
    0x6a, 0xcc, 0x99, 0xea, 0x17, 0x9b, 0x8d, 0xbb
};

static void emit_policy(const srtp_policy_t *p, uint8_t keys[][64],
                        uint8_t mkis[][16], size_t nkeys)
{
    fprintf(g_out,
            "{\"ssrc_type\": %d, \"ssrc\": %u, \"cipher_type\": %u, "
            "\"cipher_key_len\": %zu, \"auth_type\": %u, \"auth_key_len\": "
            "%zu, \"auth_tag_len\": %zu, \"sec_serv\": %d, "
            "\"rtcp_cipher_type\": %u, \"rtcp_cipher_key_len\": %zu, "
            "\"rtcp_auth_type\": %u, \"rtcp_auth_key_len\": %zu, "
            "\"rtcp_auth_tag_len\": %zu, \"rtcp_sec_serv\": %d, "
            "\"use_mki\": %d, \"mki_size\": %zu, \"window_size\": %zu, "
            "\"allow_repeat_tx\": %d, \"keys\": [",
            (int)p->ssrc.type, p->ssrc.value, p->rtp.cipher_type,
            p->rtp.cipher_key_len, p->rtp.auth_type, p->rtp.auth_key_len,
            p->rtp.auth_tag_len, (int)p->rtp.sec_serv, p->rtcp.cipher_type,
            p->rtcp.cipher_key_len, p->rtcp.auth_type, p->rtcp.auth_key_len,
            p->rtcp.auth_tag_len, (int)p->rtcp.sec_serv, (int)p->use_mki,
            p->mki_size, p->window_size, (int)p->allow_repeat_tx);
    for (size_t i = 0; i < nkeys; i++) {
        if (i)
            fputs(", ", g_out);
        hex(keys[i], 46);
    }
    fputs("], \"mki_ids\": [", g_out);
    for (size_t i = 0; p->use_mki && i < nkeys; i++) {
        if (i)
            fputs(", ", g_out);
        hex(mkis[i], p->mki_size);
    }
    fputs("]}", g_out);
}

static size_t build_rtp(uint8_t *pkt, uint32_t ssrc, uint16_t seq,
                        uint32_t ts, int cc, int xwords, size_t payload)
{
    size_t h = 12;
    pkt[0] = (uint8_t)(0x80 | (xwords >= 0 ? 0x10 : 0) | (cc & 0xf));
    pkt[1] = 96;
    pkt[2] = (uint8_t)(seq >> 8);
    pkt[3] = (uint8_t)seq;
    pkt[4] = (uint8_t)(ts >> 24);
    pkt[5] = (uint8_t)(ts >> 16);
    pkt[6] = (uint8_t)(ts >> 8);
    pkt[7] = (uint8_t)ts;
    pkt[8] = (uint8_t)(ssrc >> 24);
    pkt[9] = (uint8_t)(ssrc >> 16);
    pkt[10] = (uint8_t)(ssrc >> 8);
    pkt[11] = (uint8_t)ssrc;
    rfill(pkt + h, 4 * (size_t)cc);
    h += 4 * (size_t)cc;
    if (xwords >= 0) {
        pkt[h] = 0xbe;
        pkt[h + 1] = 0xde;
        pkt[h + 2] = (uint8_t)(xwords >> 8);
        pkt[h + 3] = (uint8_t)xwords;
        rfill(pkt + h + 4, 4 * (size_t)xwords);
        h += 4 + 4 * (size_t)xwords;
    }
    rfill(pkt + h, payload);
    return h + payload;
}

static void emit_op(const char *sess, const char *op, const uint8_t *in,
                    size_t in_len, size_t cap, size_t mki_index, int status,
                    const uint8_t *out, size_t out_len)
{
    item_begin();
    fprintf(g_out, "\"sess\": \"%s\", \"op\": \"%s\", \"in\": ", sess, op);
    hex(in, in_len);
    fprintf(g_out, ", \"cap\": %zu, \"mki_index\": %zu, \"status\": %d, "
                   "\"out\": ",
            cap, mki_index, status);
    if (status == 0)
        hex(out, out_len);
    else
        fputs("null", g_out);
    fputs("}", g_out);
}

/* one packet through protect on snd, then (optionally) unprotect on rcv */
typedef struct {
    srtp_t snd, rcv;
    uint8_t last_srtp[2200];
    size_t last_len;
} pair_t;

static int do_protect(pair_t *pp, const uint8_t *rtp, size_t len, size_t cap,
                      size_t mki_index)
{
    uint8_t out[2200];
    size_t olen = cap;
    memset(out, 0, sizeof out);
    srtp_err_status_t st = srtp_protect(pp->snd, rtp, len, out, &olen,
                                        mki_index);
    emit_op("snd", "protect", rtp, len, cap, mki_index, (int)st, out, olen);
    if (st == 0) {
        memcpy(pp->last_srtp, out, olen);
        pp->last_len = olen;
    }
    return (int)st;
}

static int do_unprotect(pair_t *pp, const uint8_t *srtp, size_t len,
                        size_t cap)
{
    uint8_t out[2200];
    size_t olen = cap;
    memset(out, 0, sizeof out);
    srtp_err_status_t st = srtp_unprotect(pp->rcv, srtp, len, out, &olen);
    emit_op("rcv", "unprotect", srtp, len, cap, 0, (int)st, out, olen);
    return (int)st;
}

static void gen_case(const policy_desc_t *d, int first_case)
{
    srtp_policy_t ps, pr;
    uint8_t keys[16][64], mkis[16][16];
    srtp_master_key_t mk[16], *mkp[16];
    const uint32_t ssrc = 0xcafebabe;

    memset(&ps, 0, sizeof ps);
    d->set(&ps.rtp);
    d->set(&ps.rtcp);
    if (d->tag_override)
        ps.rtp.auth_tag_len = ps.rtcp.auth_tag_len = d->tag_override;
    for (size_t i = 0; i < d->nkeys; i++) {
        rfill(keys[i], 64);
        rfill(mkis[i], 16);
        if (i == 0 && d->fixed_key) {
            memset(keys[0], 0, 64);
            memcpy(keys[0], d->fixed_key, d->fixed_key_len);
        }
        mk[i].key = keys[i];
        mk[i].mki_id = mkis[i];
        mkp[i] = &mk[i];
    }
    if (d->mki_size) {
        ps.keys = mkp;
        ps.num_master_keys = d->nkeys;
        ps.use_mki = true;
        ps.mki_size = d->mki_size;
    } else {
        ps.key = keys[0];
    }
    ps.window_size = d->window;
    ps.allow_repeat_tx = d->allow_repeat_tx;
    pr = ps;
    ps.ssrc.type = d->snd_type;
    ps.ssrc.value = ssrc;
    pr.ssrc.type = d->rcv_type;
    pr.ssrc.value = ssrc;

    pair_t pp;
    if (srtp_create(&pp.snd, &ps) || srtp_create(&pp.rcv, &pr)) {
        fprintf(stderr, "srtp_create failed for %s\n", d->name);
        exit(1);
    }
    fprintf(g_out, "%s    {\"name\": \"%s\", \"snd\": ", first_case ? "" : ",\n",
            d->name);
    emit_policy(&ps, keys, mkis, d->nkeys);
    fputs(", \"rcv\": ", g_out);
    emit_policy(&pr, keys, mkis, d->nkeys);
    fputs(", \"ops\": [", g_out);
    g_first_item = 1;

    static const size_t payloads[] = { 0,   1,    15,   16,   17,  160,
                                       172, 1388, 1400, 1452, 33,  64 };
    uint8_t rtp[2100], saved[40][2200];
    size_t saved_len[40], nsaved = 0;
    uint16_t seq = 0x1234;
    uint32_t ts = 0xdecafbad;
    size_t trailer = 16 + d->mki_size + 4;
    size_t nk = d->mki_size ? d->nkeys : 1;

    /* the srtp_validate() packet first (test/srtp_driver.c:2344-2354) */
    {
        uint8_t p[28] = { 0x80, 0x0f, 0x12, 0x34, 0xde, 0xca, 0xfb, 0xad,
                          0xca, 0xfe, 0xba, 0xbe };
        memset(p + 12, 0xab, 16);
        if (do_protect(&pp, p, 28, 28 + trailer, 0) == 0) {
            if (d->fixed_key == k_test_key && !d->mki_size &&
                (pp.last_len != 38 ||
                 memcmp(pp.last_srtp, k_validate_ct, 38))) {
                fprintf(stderr, "reference build fails srtp_validate KAT\n");
                exit(1);
            }
            memcpy(saved[nsaved], pp.last_srtp, pp.last_len);
            saved_len[nsaved++] = pp.last_len;
        }
        seq = 0x1235;
    }
    for (size_t i = 0; i < sizeof(payloads) / sizeof(payloads[0]); i++) {
        int cc = (i == 4) ? 2 : (i == 6 ? 1 : 0);
        int xw = (i == 5) ? 2 : (i == 10 ? 0 : -1);
        size_t len = build_rtp(rtp, ssrc, seq++, ts, cc, xw, payloads[i]);
        ts += 3000;
        if (do_protect(&pp, rtp, len, len + trailer, i % nk) == 0 &&
            nsaved < 40) {
            memcpy(saved[nsaved], pp.last_srtp, pp.last_len);
            saved_len[nsaved++] = pp.last_len;
        }
    }
    /* error rows on the sender: buffer too small, replayed seq, bad mki */
    {
        size_t len = build_rtp(rtp, ssrc, seq, ts, 0, -1, 40);
        do_protect(&pp, rtp, len, len + 1, 0);             /* buffer_small */
        build_rtp(rtp, ssrc, (uint16_t)(seq - 3), ts, 0, -1, 40);
        do_protect(&pp, rtp, len, len + trailer, 0);       /* replay */
        if (d->mki_size) {
            build_rtp(rtp, ssrc, seq++, ts, 0, -1, 40);
            do_protect(&pp, rtp, len, len + trailer, d->nkeys); /* bad mki */
        }
        build_rtp(rtp, ssrc, seq, ts, 0, -1, 3);
        do_protect(&pp, rtp, 9, 40, 0);                    /* short header */
    }
    /* two fresh packets kept back for the tamper rows */
    uint8_t fresh[2][2200];
    size_t fresh_len[2] = { 0, 0 };
    for (int i = 0; i < 2; i++) {
        size_t len = build_rtp(rtp, ssrc, seq++, ts, i, -1, 100 + 300 * i);
        if (do_protect(&pp, rtp, len, len + trailer, 0) == 0) {
            memcpy(fresh[i], pp.last_srtp, pp.last_len);
            fresh_len[i] = pp.last_len;
        }
    }
    /* receiver: every saved packet, then tamper / replay rows */
    for (size_t i = 0; i < nsaved; i++)
        do_unprotect(&pp, saved[i], saved_len[i], saved_len[i]);
    if (nsaved > 3)
        do_unprotect(&pp, saved[1], saved_len[1], saved_len[1]); /* replay */
    for (int i = 0; i < 2; i++) {
        uint8_t bad[2200];
        if (!fresh_len[i])
            continue;
        memcpy(bad, fresh[i], fresh_len[i]);
        if (i == 0)
            bad[fresh_len[i] - 1] ^= 0x01; /* tag (or mki) byte */
        else
            bad[20] ^= 0x80; /* ciphertext byte */
        do_unprotect(&pp, bad, fresh_len[i], fresh_len[i]);
        /* the genuine packet still passes: failed auth adds no index */
        do_unprotect(&pp, fresh[i], fresh_len[i], fresh_len[i]);
    }
    do_unprotect(&pp, saved[0], saved_len[0] > 4 ? 3 : 0, 64); /* short */
    /* a run across a sequence-number wrap: ROC 0 -> 1 */
    seq = 0xfffa;
    for (int i = 0; i < 10; i++) {
        size_t len = build_rtp(rtp, ssrc, seq++, ts, 0, -1, 20 + i);
        ts += 160;
        if (do_protect(&pp, rtp, len, len + trailer, 0) == 0)
            do_unprotect(&pp, pp.last_srtp, pp.last_len, pp.last_len);
    }
    /* reordered arrivals within the window */
    {
        uint8_t held[3][2200];
        size_t held_len[3] = { 0, 0, 0 };
        for (int i = 0; i < 3; i++) {
            size_t len = build_rtp(rtp, ssrc, seq++, ts, 0, -1, 48);
            if (do_protect(&pp, rtp, len, len + trailer, 0) == 0) {
                memcpy(held[i], pp.last_srtp, pp.last_len);
                held_len[i] = pp.last_len;
            }
        }
        for (int i = 2; i >= 0; i--)
            if (held_len[i])
                do_unprotect(&pp, held[i], held_len[i], held_len[i]);
    }
    fputs("\n    ]}", g_out);
    srtp_dealloc(pp.snd);
    srtp_dealloc(pp.rcv);
}

/* multi-SSRC template sessions (ssrc_any_outbound / ssrc_any_inbound) */
static void gen_template_case(int first_case, void (*set)(srtp_crypto_policy_t *),
                              const char *name)
{
    srtp_policy_t ps, pr;
    uint8_t keys[1][64], mkis[1][16];
    memset(&ps, 0, sizeof ps);
    set(&ps.rtp);
    set(&ps.rtcp);
    rfill(keys[0], 64);
    ps.key = keys[0];
    pr = ps;
    ps.ssrc.type = ssrc_any_outbound;
    pr.ssrc.type = ssrc_any_inbound;
    pair_t pp;
    srtp_create(&pp.snd, &ps);
    srtp_create(&pp.rcv, &pr);
    fprintf(g_out, "%s    {\"name\": \"%s\", \"snd\": ", first_case ? "" : ",\n",
            name);
    emit_policy(&ps, keys, mkis, 1);
    fputs(", \"rcv\": ", g_out);
    emit_policy(&pr, keys, mkis, 1);
    fputs(", \"ops\": [", g_out);
    g_first_item = 1;
    uint8_t rtp[400];
    uint16_t seqs[5] = { 7, 40000, 65535, 1, 0 };
    for (int r = 0; r < 6; r++)
        for (int s = 0; s < 5; s++) {
            uint32_t ssrc = 0x10000000u + 0x01010101u * (uint32_t)s;
            size_t len = build_rtp(rtp, ssrc, (uint16_t)(seqs[s] + r),
                                   (uint32_t)r * 160, 0, -1, 160);
            if (do_protect(&pp, rtp, len, len + 40, 0) == 0) {
                if (r == 2 && s == 1) {
                    uint8_t bad[400];
                    memcpy(bad, pp.last_srtp, pp.last_len);
                    bad[20] ^= 1;
                    do_unprotect(&pp, bad, pp.last_len, pp.last_len);
                }
                do_unprotect(&pp, pp.last_srtp, pp.last_len, pp.last_len);
            }
        }
    fputs("\n    ]}", g_out);
    srtp_dealloc(pp.snd);
    srtp_dealloc(pp.rcv);
}

static void set_gcm_256_8(srtp_crypto_policy_t *p)
{
    srtp_crypto_policy_set_aes_gcm_256_16_auth(p);
    p->auth_tag_len = 8;
}

/* the legacy keystream-prefix mode (srtp.c:2729-2741, 3006-3020): null
 * auth with a non-zero tag and the auth service on; the "tag" is the first
 * tag_len bytes of the packet's keystream, the payload takes the rest */
static void set_icm128_prefix(srtp_crypto_policy_t *p)
{
    srtp_crypto_policy_set_aes_cm_128_null_auth(p);
    p->sec_serv = sec_serv_conf_and_auth;
}

static void set_icm256_prefix(srtp_crypto_policy_t *p)
{
    srtp_crypto_policy_set_aes_cm_256_null_auth(p);
    p->sec_serv = sec_serv_conf_and_auth;
}

static void set_null_prefix(srtp_crypto_policy_t *p)
{
    srtp_crypto_policy_set_null_cipher_hmac_null(p);
    p->sec_serv = sec_serv_auth;
}


/* ---------------------------------------------------------------------- */
/* Published packet KATs of test/srtp_driver.c.  The reference build must
 * reproduce every published byte (the generator exits 1 otherwise); the
 * rows are then emitted under "kats" so the oracle and the GPU path are
 * checked against the same published vectors.                            */

typedef struct {
    const char *name, *cite;
    void (*set)(srtp_crypto_policy_t *);
    const uint8_t *key; /* NULL: no key material (null cipher, null auth) */
    size_t key_len;
    int mki;            /* two master keys with the driver's 4-byte MKI ids */
    uint32_t ssrc;
    const char *rtp, *srtp; /* srtp NULL: only the length is published */
    size_t srtp_len;
    const char *rtcp, *srtcp;
    size_t srtcp_len;
} kat_t;

/* test/srtp_driver.c:5853-5875 */
static const uint8_t k_test_key_2[46] = {
    0xf0, 0xf0, 0x49, 0x14, 0xb5, 0x13, 0xf2, 0x76, 0x3a, 0x1b, 0x1f, 0xa1,
    0x30, 0xf1, 0x0e, 0x29, 0x98, 0xf6, 0xf6, 0xe4, 0x3e, 0x43, 0x09, 0xd1,
    0xe6, 0x22, 0xa0, 0xe3, 0x32, 0xb9, 0xf1, 0xb6, 0xc3, 0x17, 0xf2, 0xda,
    0xbe, 0x35, 0x77, 0x93, 0xb6, 0x96, 0x0b, 0x3a, 0xab, 0xe6
};
static const uint8_t k_test_mki_1[4] = { 0xe1, 0xf9, 0x7a, 0x0d };
static const uint8_t k_test_mki_2[4] = { 0xf3, 0xa1, 0x46, 0x71 };
#ifdef REF_OSSL
/* test/srtp_driver.c:4114-4121 */
static const uint8_t k_test_192_key[38] = {
    0x73, 0xed, 0xc6, 0x6c, 0x4f, 0xa1, 0x57, 0x76, 0xfb, 0x57, 0xf9, 0x50,
    0x5c, 0x17, 0x13, 0x65, 0x50, 0xff, 0xda, 0x71, 0xf3, 0xe8, 0xe5, 0xf1,
    0xc8, 0x52, 0x2f, 0x3a, 0xcd, 0x4c, 0xe8, 0x6d, 0x5a, 0xdd, 0x78, 0xed,
    0xbb, 0x11
};
#endif

#define AB16 "abababababababababababababababab"
#define RTP28 "800f1234decafbadcafebabe" AB16
#define RTCP24 "81c8000bcafebabe" AB16

static const kat_t k_kats[] = {
#ifndef REF_OSSL
    { "srtp_validate", "test/srtp_driver.c:2342-2498",
      srtp_crypto_policy_set_rtp_default, k_test_key, 46, 0, 0xcafebabe,
      RTP28, "800f1234decafbadcafebabe4e55dc4ce79978d88ca4d215949d2402"
             "b78d6acc99ea179b8dbb", 38,
      RTCP24, "81c8000bcafebabe7128035be487b9bdbef89041f977a5a8"
              "80000001993e08cd54d6c1230798", 38 },
    { "srtp_validate_mki", "test/srtp_driver.c:2500-2668",
      srtp_crypto_policy_set_rtp_default, k_test_key, 46, 1, 0xcafebabe,
      RTP28, "800f1234decafbadcafebabe4e55dc4ce79978d88ca4d215949d2402"
             "e1f97a0db78d6acc99ea179b8dbb", 42,
      RTCP24, "81c8000bcafebabe7128035be487b9bdbef89041f977a5a8"
              "80000001e1f97a0d993e08cd54d6c1230798", 42 },
    { "srtp_validate_null_sha1_80", "test/srtp_driver.c:2677-2827",
      srtp_crypto_policy_set_null_cipher_hmac_sha1_80, k_test_key, 46, 0,
      0xcafebabe, RTP28, RTP28 "aba136270b679134ce9b", 38,
      RTCP24, RTCP24 "00000001fe88c7fdfd37ebce615d", 38 },
    { "srtp_validate_null_null", "test/srtp_driver.c:2836-2997",
      srtp_crypto_policy_set_null_cipher_hmac_null, NULL, 0, 0, 0xcafebabe,
      RTP28, RTP28, 28, RTCP24, RTCP24 "00000001", 28 },
    { "srtp_validate_aes_256", "test/srtp_driver.c:4206-4315",
      srtp_crypto_policy_set_aes_cm_256_hmac_sha1_80, k_test_256_key, 46, 0,
      0xcafebabe, RTP28,
      "800f1234decafbadcafebabef1d9de17ff251ff1aa007774b0b4b40d"
      "a08d9d9a5b3a55d8873b", 38, NULL, NULL, 0 },
    { "srtp_test_empty_payload", "test/srtp_driver.c:4364-4437",
      srtp_crypto_policy_set_rtp_default, k_test_key, 46, 0, 0xcafebabe,
      "800f000100000001cafebabe", NULL, 22, NULL, NULL, 0 },
#else
    { "srtp_validate_gcm", "test/srtp_driver.c:3386-3547",
      srtp_crypto_policy_set_aes_gcm_128_16_auth, k_test_key_gcm, 28, 0,
      0xcafebabe, RTP28,
      "800f1234decafbadcafebabec5002ede04cfdd2eb91159e0880aa06e"
      "d2976826f796b201df3131a127e8a392", 44,
      RTCP24, "81c8000bcafebabec98b8b5df0392a55852b6c21ac8e7025"
              "c52c6fbea2b3b446ea31123ba88ce61e80000001", 44 },
    { "srtp_validate_aes_192", "test/srtp_driver.c:4111-4197",
      srtp_crypto_policy_set_aes_cm_192_hmac_sha1_80, k_test_192_key, 38, 0,
      0x00000000, "800f0000decafbad00000000" AB16,
      "800f0000decafbad00000000d98865552f2762c3ef37f837acfdb712"
      "2d6bc4dc84c76f74aea5", 38, NULL, NULL, 0 },
    { "srtp_test_empty_payload_gcm", "test/srtp_driver.c:4440-4513",
      srtp_crypto_policy_set_aes_gcm_128_16_auth, k_test_key, 46, 0,
      0xcafebabe, "800f000100000001cafebabe", NULL, 28, NULL, NULL, 0 },
#endif
};

static size_t unhex(const char *h, uint8_t *out)
{
    size_t n = strlen(h) / 2;
    for (size_t i = 0; i < n; i++) {
        unsigned v;
        sscanf(h + 2 * i, "%2x", &v);
        out[i] = (uint8_t)v;
    }
    return n;
}

/* ---------------------------------------------------------------------- */
/* Key-usage limit and SSRC-collision events (srtp.c:1723-1773, key.c:74-90)
 * with the reference's own bookkeeping: the key limit is lowered by
 * writing the stream's srtp_key_limit_ctx_t (srtp_priv.h) -- reaching 2^48
 * packets is not practical -- and every event srtp_handle_event raises
 * during an op is recorded with it.                                        */
static int g_nev;
static uint32_t g_ev[16][2];

static void ev_handler(srtp_event_data_t *d)
{
    if (g_nev < 16) {
        g_ev[g_nev][0] = (uint32_t)d->event;
        g_ev[g_nev][1] = d->ssrc;
        g_nev++;
    }
}

static void ev_emit_tail(void)
{
    fputs(", \"events\": [", g_out);
    for (int i = 0; i < g_nev; i++)
        fprintf(g_out, "%s[%u, %u]", i ? ", " : "", g_ev[i][0], g_ev[i][1]);
    fputs("]}", g_out);
    g_nev = 0;
}

/* emit_op without its closing brace, then the events */
static void ev_op(pair_t *pp, const char *sess, const char *op,
                  const uint8_t *in, size_t len, size_t cap)
{
    uint8_t out[2200];
    size_t olen = cap;
    memset(out, 0, sizeof out);
    g_nev = 0;
    srtp_t s = sess[0] == 's' ? pp->snd : pp->rcv;
    srtp_err_status_t st = op[0] == 'p'
                               ? srtp_protect(s, in, len, out, &olen, 0)
                               : srtp_unprotect(s, in, len, out, &olen);
    item_begin();
    fprintf(g_out, "\"sess\": \"%s\", \"op\": \"%s\", \"in\": ", sess, op);
    hex(in, len);
    fprintf(g_out, ", \"cap\": %zu, \"mki_index\": 0, \"status\": %d, "
                   "\"out\": ", cap, (int)st);
    if (st == 0)
        hex(out, olen);
    else
        fputs("null", g_out);
    ev_emit_tail();
    if (st == 0 && op[0] == 'p') {
        memcpy(pp->last_srtp, out, olen);
        pp->last_len = olen;
    }
}

static void ev_set_limit(pair_t *pp, const char *sess, uint32_t ssrc,
                         uint64_t num_left)
{
    srtp_t s = sess[0] == 's' ? pp->snd : pp->rcv;
    srtp_stream_t st = srtp_get_stream(s, htonl(ssrc));
    if (!st) {
        fprintf(stderr, "gen_events: no stream %08x\n", ssrc);
        exit(1);
    }
    st->session_keys[0].limit->num_left = num_left;
    item_begin();
    fprintf(g_out, "\"sess\": \"%s\", \"op\": \"set_limit\", "
                   "\"ssrc\": %u, \"num_left\": %llu, \"events\": []}",
            sess, ssrc, (unsigned long long)num_left);
}

static void gen_events_case(const char *name, void (*set)(srtp_crypto_policy_t *),
                            int first)
{
    const uint32_t X = 0x5eedf00d;
    srtp_policy_t ps, pr;
    uint8_t keys[1][64], mkis[1][16];
    memset(&ps, 0, sizeof ps);
    set(&ps.rtp);
    set(&ps.rtcp);
    rfill(keys[0], 64);
    ps.key = keys[0];
    ps.ssrc.type = ssrc_specific;
    ps.ssrc.value = X;
    ps.window_size = 128;
    pr = ps;
    pair_t pp;
    if (srtp_create(&pp.snd, &ps) || srtp_create(&pp.rcv, &pr))
        exit(1);
    fprintf(g_out, "%s    {\"name\": \"%s\", \"snd\": ", first ? "" : ",\n",
            name);
    emit_policy(&ps, keys, mkis, 1);
    fputs(", \"rcv\": ", g_out);
    emit_policy(&pr, keys, mkis, 1);
    fputs(", \"ops\": [", g_out);
    g_first_item = 1;
    uint8_t rtp[300], sent[12][300];
    size_t sent_len[12];
    uint16_t seq = 0x2000;
    /* sender: across the soft limit, then the hard limit (and past it) */
    ev_set_limit(&pp, "snd", X, 0x10000 + 2);
    for (int i = 0; i < 5; i++) {
        size_t len = build_rtp(rtp, X, seq++, 0, 0, -1, 40 + i);
        ev_op(&pp, "snd", "protect", rtp, len, len + 32);
        memcpy(sent[i], pp.last_srtp, pp.last_len);
        sent_len[i] = pp.last_len;
    }
    ev_set_limit(&pp, "snd", X, 2);
    for (int i = 5; i < 9; i++) {
        size_t len = build_rtp(rtp, X, seq++, 0, 0, -1, 40 + i);
        ev_op(&pp, "snd", "protect", rtp, len, len + 32);
        memcpy(sent[i], pp.last_srtp, pp.last_len);
        sent_len[i] = pp.last_len;
    }
    /* receiver: a lowered limit, a tampered packet (AES-GCM counts it, the
     * HMAC path does not), then the soft limit */
    ev_op(&pp, "rcv", "unprotect", sent[0], sent_len[0], sent_len[0]);
    ev_set_limit(&pp, "rcv", X, 0x10000 + 1);
    {
        uint8_t bad[300];
        memcpy(bad, sent[1], sent_len[1]);
        bad[sent_len[1] - 1] ^= 1;
        ev_op(&pp, "rcv", "unprotect", bad, sent_len[1], sent_len[1]);
    }
    for (int i = 1; i < 5; i++)
        ev_op(&pp, "rcv", "unprotect", sent[i], sent_len[i], sent_len[i]);
    ev_set_limit(&pp, "rcv", X, 1);
    ev_op(&pp, "rcv", "unprotect", sent[5], sent_len[5], sent_len[5]);
    /* SSRC collision: the receiver's stream used to send, the sender's to
     * receive (srtp.c:2607-2623, 3104-3121) */
    {
        size_t len = build_rtp(rtp, X, 0x3000, 0, 0, -1, 20);
        ev_op(&pp, "rcv", "protect", rtp, len, len + 32);
        ev_op(&pp, "snd", "unprotect", pp.last_srtp, pp.last_len,
              pp.last_len);
    }
    fputs("\n    ]}", g_out);
    srtp_dealloc(pp.snd);
    srtp_dealloc(pp.rcv);
}

static void gen_events(void)
{
    srtp_install_event_handler(ev_handler);
    fputs(",\n  \"events\": [\n", g_out);
#ifndef REF_OSSL
    gen_events_case("events_icm128_hmac80", srtp_crypto_policy_set_rtp_default,
                    1);
    gen_events_case("events_icm256_hmac32",
                    srtp_crypto_policy_set_aes_cm_256_hmac_sha1_32, 0);
#else
    gen_events_case("events_gcm128_16",
                    srtp_crypto_policy_set_aes_gcm_128_16_auth, 1);
    gen_events_case("events_gcm256_8", set_gcm_256_8, 0);
#endif
    fputs("\n  ]", g_out);
    srtp_install_event_handler(NULL);
}

static void kat_fail(const kat_t *k, const char *what)
{
    fprintf(stderr, "reference build fails %s (%s): %s\n", k->name, k->cite,
            what);
    exit(1);
}

static void gen_kats(void)
{
    fputs(",\n  \"kats\": [\n", g_out);
    for (size_t ki = 0; ki < sizeof(k_kats) / sizeof(k_kats[0]); ki++) {
        const kat_t *k = &k_kats[ki];
        srtp_policy_t pol;
        uint8_t keys[2][64], mkis[2][16];
        srtp_master_key_t mk[2], *mkp[2];
        memset(&pol, 0, sizeof pol);
        memset(keys, 0, sizeof keys);
        memset(mkis, 0, sizeof mkis);
        k->set(&pol.rtp);
        k->set(&pol.rtcp);
        pol.ssrc.type = ssrc_specific;
        pol.ssrc.value = k->ssrc;
        if (k->key)
            memcpy(keys[0], k->key, k->key_len);
        if (k->mki) {
            memcpy(keys[1], k_test_key_2, 46);
            memcpy(mkis[0], k_test_mki_1, 4);
            memcpy(mkis[1], k_test_mki_2, 4);
            for (int i = 0; i < 2; i++) {
                mk[i].key = keys[i];
                mk[i].mki_id = mkis[i];
                mkp[i] = &mk[i];
            }
            pol.keys = mkp;
            pol.num_master_keys = 2;
            pol.use_mki = true;
            pol.mki_size = 4;
        } else {
            pol.key = keys[0];
        }
        pol.window_size = 128;
        srtp_t snd, rcv;
        if (srtp_create(&snd, &pol) || srtp_create(&rcv, &pol))
            kat_fail(k, "srtp_create");
        fprintf(g_out, "%s    {\"name\": \"%s\", \"cite\": \"%s\", \"snd\": ",
                ki ? ",\n" : "", k->name, k->cite);
        emit_policy(&pol, keys, mkis, k->mki ? 2 : 1);
        fputs(", \"rcv\": ", g_out);
        emit_policy(&pol, keys, mkis, k->mki ? 2 : 1);
        fputs(", \"ops\": [", g_out);
        g_first_item = 1;

        uint8_t in[128], exp[128], out[128];
        size_t in_len, exp_len = 0, olen;
        srtp_err_status_t st;
        /* RTP: protect the plaintext, then unprotect the published packet
         * (or, with only a length published, the reference's own output) */
        in_len = unhex(k->rtp, in);
        olen = sizeof out;
        st = srtp_protect(snd, in, in_len, out, &olen, 0);
        emit_op("snd", "protect", in, in_len, in_len + 64, 0, (int)st, out,
                olen);
        if (st || olen != k->srtp_len)
            kat_fail(k, "srtp_protect length");
        if (k->srtp) {
            exp_len = unhex(k->srtp, exp);
            if (exp_len != olen || memcmp(exp, out, olen))
                kat_fail(k, "srtp_protect bytes");
        } else {
            memcpy(exp, out, olen);
            exp_len = olen;
        }
        olen = sizeof out;
        st = srtp_unprotect(rcv, exp, exp_len, out, &olen);
        emit_op("rcv", "unprotect", exp, exp_len, exp_len, 0, (int)st, out,
                olen);
        if (st || olen != in_len || memcmp(out, in, in_len))
            kat_fail(k, "srtp_unprotect");
        if (k->rtcp) {
            in_len = unhex(k->rtcp, in);
            olen = sizeof out;
            st = srtp_protect_rtcp(snd, in, in_len, out, &olen, 0);
            emit_op("snd", "protect_rtcp", in, in_len, in_len + 64, 0,
                    (int)st, out, olen);
            exp_len = unhex(k->srtcp, exp);
            if (st || olen != k->srtcp_len || exp_len != olen ||
                memcmp(exp, out, olen))
                kat_fail(k, "srtp_protect_rtcp");
            olen = sizeof out;
            st = srtp_unprotect_rtcp(rcv, exp, exp_len, out, &olen);
            emit_op("rcv", "unprotect_rtcp", exp, exp_len, exp_len, 0,
                    (int)st, out, olen);
            if (st || olen != in_len || memcmp(out, in, in_len))
                kat_fail(k, "srtp_unprotect_rtcp");
        }
        fputs("\n    ]}", g_out);
        srtp_dealloc(snd);
        srtp_dealloc(rcv);
    }
    fputs("\n  ]", g_out);
}

int main(int argc, char **argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s out.json\n", argv[0]);
        return 2;
    }
    if (srtp_init()) {
        fprintf(stderr, "srtp_init failed\n");
        return 1;
    }
    g_out = fopen(argv[1], "w");
    fputs("{\n", g_out);
#ifdef PREFIX_CASES
    /* tests/golden/ref_prefix.json: keystream-prefix sessions only */
    {
        static const policy_desc_t pcases[] = {
            { "prefix_icm128_tag4", set_icm128_prefix, 4, 1, 0, 128, 0,
              ssrc_specific, ssrc_specific },
            { "prefix_icm128_tag10", set_icm128_prefix, 10, 1, 0, 128, 0,
              ssrc_specific, ssrc_specific },
            { "prefix_icm256_tag7_mki", set_icm256_prefix, 7, 2, 4, 128, 0,
              ssrc_specific, ssrc_specific },
            { "prefix_null_tag4", set_null_prefix, 4, 1, 0, 64, 0,
              ssrc_specific, ssrc_specific },
        };
        fputs("  \"backend\": \"internal\",\n  \"cases\": [\n", g_out);
        for (size_t i = 0; i < sizeof pcases / sizeof pcases[0]; i++)
            gen_case(&pcases[i], i == 0);
        fputs("\n  ]\n}\n", g_out);
        fclose(g_out);
        return 0;
    }
#endif
#ifndef REF_OSSL
    fputs("  \"backend\": \"internal\",\n", g_out);
    gen_aes();
    gen_sha1();
    gen_hmac();
    gen_icm("icm128", SRTP_AES_ICM_128, 30);
    gen_icm("icm256", SRTP_AES_ICM_256, 46);
    static const policy_desc_t cases[] = {
        { "kat_srtp_validate", srtp_crypto_policy_set_rtp_default, 0, 1, 0,
          128, 0, ssrc_specific, ssrc_specific, k_test_key, 46 },
        { "kat_validate_aes_256", srtp_crypto_policy_set_aes_cm_256_hmac_sha1_80,
          0, 1, 0, 128, 0, ssrc_specific, ssrc_specific, k_test_256_key, 46 },
        { "icm128_hmac80", srtp_crypto_policy_set_rtp_default, 0, 1, 0, 128,
          0, ssrc_specific, ssrc_specific },
        { "icm128_hmac32", srtp_crypto_policy_set_aes_cm_128_hmac_sha1_32, 0,
          1, 0, 128, 0, ssrc_specific, ssrc_specific },
        { "icm128_nullauth", srtp_crypto_policy_set_aes_cm_128_null_auth, 0,
          1, 0, 64, 0, ssrc_specific, ssrc_specific },
        { "null_hmac80", srtp_crypto_policy_set_null_cipher_hmac_sha1_80, 0,
          1, 0, 128, 0, ssrc_specific, ssrc_specific },
        { "icm256_hmac80", srtp_crypto_policy_set_aes_cm_256_hmac_sha1_80, 0,
          1, 0, 1024, 0, ssrc_specific, ssrc_specific },
        { "icm256_hmac32", srtp_crypto_policy_set_aes_cm_256_hmac_sha1_32, 0,
          1, 0, 128, 1, ssrc_specific, ssrc_specific },
        { "icm128_hmac80_mki", srtp_crypto_policy_set_rtp_default, 0, 3, 4,
          128, 0, ssrc_specific, ssrc_specific },
    };
#else
    fputs("  \"backend\": \"openssl\",\n", g_out);
    gen_icm("icm192", SRTP_AES_ICM_192, 38);
    gen_gcm("gcm128_16", SRTP_AES_GCM_128, 28, 16);
    gen_gcm("gcm256_16", SRTP_AES_GCM_256, 44, 16);
    gen_gcm("gcm128_8", SRTP_AES_GCM_128, 28, 8);
    gen_gcm("gcm256_8", SRTP_AES_GCM_256, 44, 8);
    static const policy_desc_t cases[] = {
        { "kat_validate_gcm", srtp_crypto_policy_set_aes_gcm_128_16_auth, 0,
          1, 0, 128, 0, ssrc_specific, ssrc_specific, k_test_key_gcm, 28 },
        { "kat_bench_gcm256", srtp_crypto_policy_set_aes_gcm_256_16_auth, 0,
          1, 0, 128, 0, ssrc_specific, ssrc_specific, k_test_256_key, 44 },
        { "gcm128_16", srtp_crypto_policy_set_aes_gcm_128_16_auth, 0, 1, 0,
          128, 0, ssrc_specific, ssrc_specific },
        { "gcm256_16", srtp_crypto_policy_set_aes_gcm_256_16_auth, 0, 1, 0,
          128, 0, ssrc_specific, ssrc_specific },
        { "gcm256_8", set_gcm_256_8, 0, 1, 0, 128, 0, ssrc_specific,
          ssrc_specific },
        { "gcm256_16_mki", srtp_crypto_policy_set_aes_gcm_256_16_auth, 0, 2,
          8, 128, 0, ssrc_specific, ssrc_specific },
        { "icm192_hmac80", srtp_crypto_policy_set_aes_cm_192_hmac_sha1_80, 0,
          1, 0, 128, 0, ssrc_specific, ssrc_specific },
        { "icm128_hmac80_ossl", srtp_crypto_policy_set_rtp_default, 0, 1, 0,
          128, 0, ssrc_specific, ssrc_specific },
    };
#endif
    fputs("  \"cases\": [\n", g_out);
    for (size_t i = 0; i < sizeof(cases) / sizeof(cases[0]); i++)
        gen_case(&cases[i], i == 0);
#ifndef REF_OSSL
    gen_template_case(0, srtp_crypto_policy_set_rtp_default,
                      "template_icm128_hmac80");
#else
    gen_template_case(0, srtp_crypto_policy_set_aes_gcm_256_16_auth,
                      "template_gcm256_16");
#endif
    fputs("\n  ]", g_out);
    gen_kats();
    gen_events();
    fputs("\n}\n", g_out);
    fclose(g_out);
    srtp_shutdown();
    return 0;
}
