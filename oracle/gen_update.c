/*
 * gen_update.c -- srtp_update / srtp_stream_update fixtures
 * (tests/golden/ref_update*.json) from the REFERENCE built by Makefile.ref.
 * Test infrastructure, build container only; outputs are committed data.
 *
 * What srtp.c:3430-3617 keeps across an update: the RTP extended sequence
 * number (rdbx index) and the SRTCP replay database (rtcp_rdb: the sender's
 * next SRTCP index and the receiver's replay window), for a specific-SSRC
 * stream and for streams cloned from a template.  Rows: RTP and SRTCP
 * protect / unprotect around updates with the same key (indices continue;
 * old SRTCP packets are replays, old RTP packets are accepted again because
 * the RTP replay bitmap starts empty) and with a new key (old-key packets
 * fail authentication), for AES-ICM + HMAC-SHA1 and AES-GCM.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

#include "srtp.h"

static uint64_t g_rng = 0x5550444154453031ULL; /* "UPDATE01" */
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
static int g_first_item, g_first_case = 1;

static void hex(const uint8_t *p, size_t n)
{
    fputc('"', g_out);
    for (size_t i = 0; i < n; i++)
        fprintf(g_out, "%02x", p[i]);
    fputc('"', g_out);
}

static void emit_policy(const srtp_policy_t *p)
{
    fprintf(g_out,
            "{\"ssrc_type\": %d, \"ssrc\": %u, \"cipher_type\": %u, "
            "\"cipher_key_len\": %zu, \"auth_type\": %u, \"auth_key_len\": "
            "%zu, \"auth_tag_len\": %zu, \"sec_serv\": %d, "
            "\"rtcp_cipher_type\": %u, \"rtcp_cipher_key_len\": %zu, "
            "\"rtcp_auth_type\": %u, \"rtcp_auth_key_len\": %zu, "
            "\"rtcp_auth_tag_len\": %zu, \"rtcp_sec_serv\": %d, "
            "\"use_mki\": 0, \"mki_size\": 0, \"window_size\": %zu, "
            "\"allow_repeat_tx\": %d, \"keys\": [",
            (int)p->ssrc.type, p->ssrc.value, p->rtp.cipher_type,
            p->rtp.cipher_key_len, p->rtp.auth_type, p->rtp.auth_key_len,
            p->rtp.auth_tag_len, (int)p->rtp.sec_serv, p->rtcp.cipher_type,
            p->rtcp.cipher_key_len, p->rtcp.auth_type, p->rtcp.auth_key_len,
            p->rtcp.auth_tag_len, (int)p->rtcp.sec_serv, p->window_size,
            (int)p->allow_repeat_tx);
    hex(p->key, 64);
    fputs("], \"mki_ids\": []}", g_out);
}

static void item(void)
{
    fputs(g_first_item ? "\n    {" : ",\n    {", g_out);
    g_first_item = 0;
}

/* one protect / unprotect (RTP or SRTCP); out receives the result */
static int op(srtp_t s, const char *sess, const char *name, const uint8_t *in,
              size_t len, uint8_t *out, size_t *olen)
{
    size_t cap = name[0] == 'p' ? len + 64 : len;
    srtp_err_status_t st;
    *olen = cap;
    if (!strcmp(name, "protect"))
        st = srtp_protect(s, in, len, out, olen, 0);
    else if (!strcmp(name, "unprotect"))
        st = srtp_unprotect(s, in, len, out, olen);
    else if (!strcmp(name, "protect_rtcp"))
        st = srtp_protect_rtcp(s, in, len, out, olen, 0);
    else
        st = srtp_unprotect_rtcp(s, in, len, out, olen);
    item();
    fprintf(g_out, "\"sess\": \"%s\", \"op\": \"%s\", \"in\": ", sess, name);
    hex(in, len);
    fprintf(g_out, ", \"cap\": %zu, \"status\": %d, \"out\": ", cap, (int)st);
    if (st == 0)
        hex(out, *olen);
    else
        fputs("null", g_out);
    fputs("}", g_out);
    return (int)st;
}

static void update(srtp_t s, const char *sess, const srtp_policy_t *p)
{
    srtp_err_status_t st = srtp_update(s, p);
    item();
    fprintf(g_out, "\"sess\": \"%s\", \"op\": \"update\", \"status\": %d, "
                   "\"policy\": ", sess, (int)st);
    emit_policy(p);
    fputs("}", g_out);
}

static size_t rtp(uint8_t *p, uint32_t ssrc, uint16_t seq, size_t pay)
{
    p[0] = 0x80;
    p[1] = 96;
    p[2] = (uint8_t)(seq >> 8);
    p[3] = (uint8_t)seq;
    rfill(p + 4, 4);
    p[8] = (uint8_t)(ssrc >> 24);
    p[9] = (uint8_t)(ssrc >> 16);
    p[10] = (uint8_t)(ssrc >> 8);
    p[11] = (uint8_t)ssrc;
    rfill(p + 12, pay);
    return 12 + pay;
}

static size_t rtcp(uint8_t *p, uint32_t ssrc, size_t body)
{
    p[0] = 0x81;
    p[1] = 0xc8;
    p[2] = 0;
    p[3] = (uint8_t)((body + 8) / 4 - 1);
    p[4] = (uint8_t)(ssrc >> 24);
    p[5] = (uint8_t)(ssrc >> 16);
    p[6] = (uint8_t)(ssrc >> 8);
    p[7] = (uint8_t)ssrc;
    rfill(p + 8, body);
    return 8 + body;
}

typedef struct {
    uint8_t b[400];
    size_t n;
} pkt_t;

static void gen(const char *name, void (*set)(srtp_crypto_policy_t *),
                int templ)
{
    uint8_t k1[64], k2[64];
    rfill(k1, 64);
    rfill(k2, 64);
    const uint32_t X = 0x0badcafe, Y = 0x0badbeef;
    srtp_policy_t ps, pr;
    memset(&ps, 0, sizeof ps);
    set(&ps.rtp);
    set(&ps.rtcp);
    ps.key = k1;
    ps.window_size = 128;
    ps.ssrc.type = templ ? ssrc_any_outbound : ssrc_specific;
    ps.ssrc.value = X;
    pr = ps;
    pr.ssrc.type = templ ? ssrc_any_inbound : ssrc_specific;
    srtp_t snd, rcv;
    if (srtp_create(&snd, &ps) || srtp_create(&rcv, &pr)) {
        fprintf(stderr, "srtp_create failed (%s)\n", name);
        exit(1);
    }
    fprintf(g_out, "%s    {\"name\": \"%s\", \"snd\": ", g_first_case ? "" : ",\n",
            name);
    g_first_case = 0;
    emit_policy(&ps);
    fputs(", \"rcv\": ", g_out);
    emit_policy(&pr);
    fputs(", \"ops\": [", g_out);
    g_first_item = 1;

    pkt_t sent[64];
    int ns = 0;
    uint8_t in[400], out[500];
    size_t ol;
    const uint32_t ssrcs[2] = { X, Y };
    int nss = templ ? 2 : 1;
    uint16_t seq[2] = { 0xfffd, 100 }; /* the first stream wraps its ROC */
    /* phase 1: RTP and SRTCP under key 1 */
    for (int r = 0; r < 3; r++)
        for (int k = 0; k < nss; k++) {
            size_t n = rtp(in, ssrcs[k], seq[k]++, 40 + r);
            if (!op(snd, "snd", "protect", in, n, out, &ol)) {
                memcpy(sent[ns].b, out, ol);
                sent[ns++].n = ol;
            }
            n = rtcp(in, ssrcs[k], 24);
            if (!op(snd, "snd", "protect_rtcp", in, n, out, &ol)) {
                memcpy(sent[ns].b, out, ol);
                sent[ns++].n = ol | 0x10000; /* flag: SRTCP */
            }
        }
    /* the receiver takes phase 1 */
    for (int i = 0; i < ns; i++)
        op(rcv, "rcv", (sent[i].n & 0x10000) ? "unprotect_rtcp" : "unprotect",
           sent[i].b, sent[i].n & 0xffff, out, &ol);
    /* same-key update on both sides: indices continue; every phase-1
     * packet again (SRTCP: replay_fail; RTP: the window was cleared) */
    update(snd, "snd", &ps);
    update(rcv, "rcv", &pr);
    for (int k = 0; k < nss; k++) {
        size_t n = rtp(in, ssrcs[k], seq[k]++, 33);
        if (!op(snd, "snd", "protect", in, n, out, &ol))
            op(rcv, "rcv", "unprotect", out, ol, in, &ol);
        n = rtcp(in, ssrcs[k], 16);
        if (!op(snd, "snd", "protect_rtcp", in, n, out, &ol))
            op(rcv, "rcv", "unprotect_rtcp", out, ol, in, &ol);
    }
    for (int i = 0; i < ns; i++)
        op(rcv, "rcv", (sent[i].n & 0x10000) ? "unprotect_rtcp" : "unprotect",
           sent[i].b, sent[i].n & 0xffff, out, &ol);
    /* new key at the sender only: the receiver's old key rejects it; then
     * the receiver too */
    ps.key = k2;
    pr.key = k2;
    update(snd, "snd", &ps);
    pkt_t late[8];
    int nl = 0;
    for (int k = 0; k < nss; k++) {
        size_t n = rtp(in, ssrcs[k], seq[k]++, 50);
        if (!op(snd, "snd", "protect", in, n, out, &ol)) {
            memcpy(late[nl].b, out, ol);
            late[nl++].n = ol;
            op(rcv, "rcv", "unprotect", out, ol, in, &ol);
        }
        n = rtcp(in, ssrcs[k], 20);
        if (!op(snd, "snd", "protect_rtcp", in, n, out, &ol)) {
            memcpy(late[nl].b, out, ol);
            late[nl++].n = ol | 0x10000;
            op(rcv, "rcv", "unprotect_rtcp", out, ol, in, &ol);
        }
    }
    update(rcv, "rcv", &pr);
    for (int i = 0; i < nl; i++)
        op(rcv, "rcv", (late[i].n & 0x10000) ? "unprotect_rtcp" : "unprotect",
           late[i].b, late[i].n & 0xffff, out, &ol);
    fputs("\n    ]}", g_out);
    srtp_dealloc(snd);
    srtp_dealloc(rcv);
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
#ifndef REF_OSSL
    fputs("{\n  \"backend\": \"internal\",\n  \"cases\": [\n", g_out);
    gen("update_icm128_hmac80", srtp_crypto_policy_set_rtp_default, 0);
    gen("update_template_icm128_hmac80", srtp_crypto_policy_set_rtp_default,
        1);
    gen("update_icm256_hmac32", srtp_crypto_policy_set_aes_cm_256_hmac_sha1_32,
        0);
#else
    fputs("{\n  \"backend\": \"openssl\",\n  \"cases\": [\n", g_out);
    gen("update_gcm128_16", srtp_crypto_policy_set_aes_gcm_128_16_auth, 0);
    gen("update_template_gcm256_16",
        srtp_crypto_policy_set_aes_gcm_256_16_auth, 1);
#endif
    fputs("\n  ]\n}\n", g_out);
    fclose(g_out);
    srtp_shutdown();
    return 0;
}
