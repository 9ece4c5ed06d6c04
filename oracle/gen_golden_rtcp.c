/*
 * gen_golden_rtcp.c -- emits tests/golden/ref_rtcp.json by driving the
 * REFERENCE's srtp_protect_rtcp / srtp_unprotect_rtcp (srtp/srtp.c:4304-4837;
 * cisco/libsrtp built from /root/reference sources into oracle/_ref/ by
 * Makefile.ref, internal crypto kernel).  Test infrastructure: build
 * container only (`make -f oracle/Makefile.golden rtcp`); the JSON is
 * committed as a data fixture.
 *
 * Cases are sender/receiver session pairs; every op records the input, the
 * capacity, the reference's status and (on success) its output.  Inputs come
 * from splitmix64 seeded with "SRTCP001".
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

#include "srtp.h"

static uint64_t g_rng = 0x5352544350303031ULL; /* "SRTCP001" */
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
static int g_first;

static void hex(const uint8_t *p, size_t n)
{
    fputc('"', g_out);
    for (size_t i = 0; i < n; i++)
        fprintf(g_out, "%02x", p[i]);
    fputc('"', g_out);
}

static void policy_json(const srtp_policy_t *p, uint8_t keys[][64],
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
        fputs(i ? ", " : "", g_out);
        hex(keys[i], 46);
    }
    fputs("], \"mki_ids\": [", g_out);
    for (size_t i = 0; p->use_mki && i < nkeys; i++) {
        fputs(i ? ", " : "", g_out);
        hex(mkis[i], p->mki_size);
    }
    fputs("]}", g_out);
}

typedef struct {
    srtp_t snd, rcv;
    uint8_t last[2200];
    size_t last_len;
} pair_t;

static void emit(const char *sess, const char *op, const uint8_t *in,
                 size_t len, size_t cap, size_t mki_index, int st,
                 const uint8_t *out, size_t out_len)
{
    fprintf(g_out, "%s\n      {", g_first ? "" : ",");
    g_first = 0;
    fprintf(g_out, "\"sess\": \"%s\", \"op\": \"%s\", \"in\": ", sess, op);
    hex(in, len);
    fprintf(g_out, ", \"cap\": %zu, \"mki_index\": %zu, \"status\": %d, "
                   "\"out\": ", cap, mki_index, st);
    if (st == 0)
        hex(out, out_len);
    else
        fputs("null", g_out);
    fputc('}', g_out);
}

static int prot(pair_t *pp, const uint8_t *in, size_t len, size_t cap,
                size_t mki_index)
{
    uint8_t out[2200];
    size_t olen = cap;
    memset(out, 0, sizeof out);
    int st = (int)srtp_protect_rtcp(pp->snd, in, len, out, &olen, mki_index);
    emit("snd", "protect_rtcp", in, len, cap, mki_index, st, out, olen);
    if (st == 0) {
        memcpy(pp->last, out, olen);
        pp->last_len = olen;
    }
    return st;
}

static int unprot(pair_t *pp, const uint8_t *in, size_t len, size_t cap)
{
    uint8_t out[2200];
    size_t olen = cap;
    memset(out, 0, sizeof out);
    int st = (int)srtp_unprotect_rtcp(pp->rcv, in, len, out, &olen);
    emit("rcv", "unprotect_rtcp", in, len, cap, 0, st, out, olen);
    return st;
}

/* compound RTCP: SR header (V=2, PT=200) with the SSRC at bytes 4..7 */
static size_t build_rtcp(uint8_t *p, uint32_t ssrc, size_t len)
{
    rfill(p, len);
    p[0] = 0x80;
    p[1] = 200;
    p[2] = (uint8_t)(((len / 4) - 1) >> 8);
    p[3] = (uint8_t)((len / 4) - 1);
    p[4] = (uint8_t)(ssrc >> 24);
    p[5] = (uint8_t)(ssrc >> 16);
    p[6] = (uint8_t)(ssrc >> 8);
    p[7] = (uint8_t)ssrc;
    return len;
}

typedef struct {
    const char *name;
    void (*rtp)(srtp_crypto_policy_t *);
    void (*rtcp)(srtp_crypto_policy_t *);
    int rtcp_serv;           /* -1: setter's */
    size_t nkeys, mki_size;
    int snd_type, rcv_type;
} desc_t;

static void gen(const desc_t *d, int first)
{
    srtp_policy_t ps, pr;
    uint8_t keys[4][64], mkis[4][16];
    srtp_master_key_t mk[4], *mkp[4];
    const uint32_t ssrc = 0x5eed1234;
    memset(&ps, 0, sizeof ps);
    d->rtp(&ps.rtp);
    d->rtcp(&ps.rtcp);
    if (d->rtcp_serv >= 0)
        ps.rtcp.sec_serv = (srtp_sec_serv_t)d->rtcp_serv;
    for (size_t i = 0; i < d->nkeys; i++) {
        rfill(keys[i], 64);
        rfill(mkis[i], 16);
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
    ps.window_size = 128;
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
    fprintf(g_out, "%s    {\"name\": \"%s\", \"snd\": ", first ? "" : ",\n",
            d->name);
    policy_json(&ps, keys, mkis, d->nkeys);
    fputs(", \"rcv\": ", g_out);
    policy_json(&pr, keys, mkis, d->nkeys);
    fputs(", \"ops\": [", g_out);
    g_first = 1;

    static const size_t sizes[] = { 8, 12, 28, 52, 64, 100, 160, 500, 1200 };
    uint8_t pkt[1300], saved[16][1400], bad[1400];
    size_t saved_len[16], ns = 0;
    size_t nk = d->mki_size ? d->nkeys : 1;
    size_t tr = 4 + d->mki_size + 20;
    for (size_t i = 0; i < sizeof sizes / sizeof sizes[0]; i++) {
        size_t len = build_rtcp(pkt, ssrc, sizes[i]);
        if (prot(&pp, pkt, len, len + tr, i % nk) == 0) {
            memcpy(saved[ns], pp.last, pp.last_len);
            saved_len[ns++] = pp.last_len;
            if (i == 3) {           /* tampered tag / body / E bit */
                memcpy(bad, pp.last, pp.last_len);
                bad[pp.last_len - 1] ^= 0x40;
                unprot(&pp, bad, pp.last_len, pp.last_len);
                memcpy(bad, pp.last, pp.last_len);
                bad[9] ^= 1;
                unprot(&pp, bad, pp.last_len, pp.last_len);
                memcpy(bad, pp.last, pp.last_len);
                bad[len] ^= 0x80;
                unprot(&pp, bad, pp.last_len, pp.last_len);
            }
            if (i != 5)             /* index 6 arrives late, below */
                unprot(&pp, pp.last, pp.last_len, pp.last_len);
        }
    }
    /* late arrival, then replay of an accepted packet, small out buffer */
    if (ns > 5) {
        unprot(&pp, saved[5], saved_len[5], saved_len[5]);
        unprot(&pp, saved[2], saved_len[2], saved_len[2]);
        size_t len = build_rtcp(pkt, ssrc, 40);
        if (prot(&pp, pkt, len, len + tr, 0) == 0)
            unprot(&pp, pp.last, pp.last_len, 10);
    }
    /* error rows: short packet, small buffer, bad MKI index */
    build_rtcp(pkt, ssrc, 8);
    prot(&pp, pkt, 7, 64, 0);
    build_rtcp(pkt, ssrc, 32);
    prot(&pp, pkt, 32, 33, 0);
    if (d->mki_size)
        prot(&pp, pkt, 32, 80, d->nkeys);
    unprot(&pp, pkt, 11, 64);
    /* window: 140 packets, the receiver takes the last 130 only, then the
     * first ones are too old */
    uint8_t win[140][200];
    size_t wl[140];
    for (int i = 0; i < 140; i++) {
        size_t len = build_rtcp(pkt, ssrc, 28);
        size_t ol = sizeof win[i];
        if (srtp_protect_rtcp(pp.snd, pkt, len, win[i], &ol, 0))
            exit(3);
        wl[i] = ol;
    }
    for (int i = 10; i < 140; i += 13)
        unprot(&pp, win[i], wl[i], wl[i]);
    unprot(&pp, win[139], wl[139], wl[139]);
    unprot(&pp, win[2], wl[2], wl[2]);
    unprot(&pp, win[20], wl[20], wl[20]);
    /* other SSRCs: templates clone, specific sessions report no_ctx */
    for (uint32_t s = 1; s <= 3; s++) {
        size_t len = build_rtcp(pkt, 0x01000000u * s + s, 24 + 8 * s);
        if (prot(&pp, pkt, len, len + tr, 0) == 0)
            unprot(&pp, pp.last, pp.last_len, pp.last_len);
    }
    fputs("\n    ]}", g_out);
    srtp_dealloc(pp.snd);
    srtp_dealloc(pp.rcv);
}

int main(int argc, char **argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s out.json\n", argv[0]);
        return 2;
    }
    if (srtp_init())
        return 1;
    g_out = fopen(argv[1], "w");
    if (!g_out)
        return 1;
#ifdef REF_OSSL
    static const desc_t d[] = {
        { "rtcp_gcm128_16", srtp_crypto_policy_set_aes_gcm_128_16_auth,
          srtp_crypto_policy_set_aes_gcm_128_16_auth, -1, 1, 0, ssrc_specific,
          ssrc_specific },
        { "rtcp_gcm256_16", srtp_crypto_policy_set_aes_gcm_256_16_auth,
          srtp_crypto_policy_set_aes_gcm_256_16_auth, -1, 1, 0, ssrc_specific,
          ssrc_specific },
        { "rtcp_gcm256_auth_only", srtp_crypto_policy_set_aes_gcm_256_16_auth,
          srtp_crypto_policy_set_aes_gcm_256_16_auth, sec_serv_auth, 1, 0,
          ssrc_specific, ssrc_specific },
        { "rtcp_gcm128_mki2", srtp_crypto_policy_set_aes_gcm_128_16_auth,
          srtp_crypto_policy_set_aes_gcm_128_16_auth, -1, 2, 3, ssrc_specific,
          ssrc_specific },
        { "rtcp_gcm256_template", srtp_crypto_policy_set_aes_gcm_256_16_auth,
          srtp_crypto_policy_set_aes_gcm_256_16_auth, -1, 1, 0,
          ssrc_any_outbound, ssrc_any_inbound },
        { "rtcp_icm192_sha1_80", srtp_crypto_policy_set_aes_cm_192_hmac_sha1_80,
          srtp_crypto_policy_set_aes_cm_192_hmac_sha1_80, -1, 1, 0,
          ssrc_specific, ssrc_specific },
    };
#else
    static const desc_t d[] = {
        { "rtcp_default", srtp_crypto_policy_set_rtp_default,
          srtp_crypto_policy_set_rtcp_default, -1, 1, 0, ssrc_specific,
          ssrc_specific },
        { "rtcp_icm256_sha1_80", srtp_crypto_policy_set_aes_cm_256_hmac_sha1_80,
          srtp_crypto_policy_set_aes_cm_256_hmac_sha1_80, -1, 1, 0,
          ssrc_specific, ssrc_specific },
        { "rtcp_icm128_sha1_32", srtp_crypto_policy_set_aes_cm_128_hmac_sha1_32,
          srtp_crypto_policy_set_aes_cm_128_hmac_sha1_32, -1, 1, 0,
          ssrc_specific, ssrc_specific },
        { "rtcp_auth_only", srtp_crypto_policy_set_rtp_default,
          srtp_crypto_policy_set_rtcp_default, sec_serv_auth, 1, 0,
          ssrc_specific, ssrc_specific },
        { "rtcp_null_cipher_sha1_80", srtp_crypto_policy_set_rtp_default,
          srtp_crypto_policy_set_null_cipher_hmac_sha1_80, -1, 1, 0,
          ssrc_specific, ssrc_specific },
        { "rtcp_null_null", srtp_crypto_policy_set_rtp_default,
          srtp_crypto_policy_set_null_cipher_hmac_null, -1, 1, 0,
          ssrc_specific, ssrc_specific },
        { "rtcp_icm128_null_auth", srtp_crypto_policy_set_rtp_default,
          srtp_crypto_policy_set_aes_cm_128_null_auth, -1, 1, 0,
          ssrc_specific, ssrc_specific },
        { "rtcp_mki3", srtp_crypto_policy_set_rtp_default,
          srtp_crypto_policy_set_rtcp_default, -1, 3, 4, ssrc_specific,
          ssrc_specific },
        { "rtcp_template", srtp_crypto_policy_set_aes_cm_256_hmac_sha1_32,
          srtp_crypto_policy_set_aes_cm_256_hmac_sha1_80, -1, 1, 0,
          ssrc_any_outbound, ssrc_any_inbound },
    };
#endif
#ifdef REF_OSSL
    fputs("{\n  \"generator\": \"oracle/gen_golden_rtcp.c against "
          "oracle/_ref/libsrtp_ref_ossl.so (cisco/libsrtp 3.0.0, OpenSSL)\",\n"
          "  \"cases\": [\n", g_out);
#else
    fputs("{\n  \"generator\": \"oracle/gen_golden_rtcp.c against "
          "oracle/_ref/libsrtp_ref_int.so (cisco/libsrtp 3.0.0)\",\n"
          "  \"cases\": [\n", g_out);
#endif
    for (size_t i = 0; i < sizeof d / sizeof d[0]; i++)
        gen(&d[i], i == 0);
    fputs("\n  ]\n}\n", g_out);
    fclose(g_out);
    srtp_shutdown();
    return 0;
}
