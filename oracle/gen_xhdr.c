/*
 * gen_xhdr.c -- RFC 6904 header-extension encryption and RFC 9335 cryptex
 * fixtures (tests/golden/ref_xhdr*.json), produced by driving the REFERENCE
 * (cisco/libsrtp built from /root/reference by Makefile.ref into
 * oracle/_ref/).  Test infrastructure, build container only; the outputs are
 * committed as data so the GPU box never needs /root/reference.
 *
 * The oracle (srtp_oracle.c) does not restate these two features: the GPU
 * path is pinned directly against the reference's outputs here.
 *
 * Built without REF_OSSL (internal crypto: AES-ICM-128/256, HMAC-SHA1) and
 * with REF_OSSL (AES-GCM-128/256, AES-ICM-192).  Published vectors of
 * test/srtp_driver.c (srtp_validate_cryptex :3004, srtp_validate_gcm_cryptex
 * :3553, srtp_validate_encrypted_extensions_headers :3848 and _gcm :3976,
 * srtp_test_cryptex_csrc_but_no_extension_header :3266) must be reproduced
 * byte for byte or the generator exits 1; the rest are splitmix64-seeded
 * packets with one- and two-byte extensions, CSRCs, padding, ID 15,
 * malformed elements and unknown profiles, protected and unprotected in
 * place and not in place.
 *
 * Not-in-place calls are made the way test/srtp_driver.c:228-267 makes
 * them: the output buffer starts as a copy of the input.  The reference
 * depends on that -- srtp_cryptex_unprotect_init reads the profile from the
 * output buffer before anything was copied there (srtp.c:246-249 via
 * 2968), and protect walks the extension in the output before its data was
 * copied (srtp.c:2643-2645, 2745-2754).
 *
 * One reference behaviour is kept out of the random rows: AES-GCM unprotect
 * in place with cryptex, CSRCs and header-extension encryption reads the
 * last CSRC as the extension header (srtp.c:2384 moved it, 2413 does not
 * move it back); such rows are kept only when that CSRC does not look like
 * an extension profile (then both return parse_err).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

#include "srtp.h"

static uint64_t g_rng = 0x5852545030303036ULL;
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

static void emit_policy(const srtp_policy_t *p, const uint8_t *key)
{
    fprintf(g_out,
            "{\"ssrc_type\": %d, \"ssrc\": %u, \"cipher_type\": %u, "
            "\"cipher_key_len\": %zu, \"auth_type\": %u, \"auth_key_len\": "
            "%zu, \"auth_tag_len\": %zu, \"sec_serv\": %d, "
            "\"rtcp_cipher_type\": %u, \"rtcp_cipher_key_len\": %zu, "
            "\"rtcp_auth_type\": %u, \"rtcp_auth_key_len\": %zu, "
            "\"rtcp_auth_tag_len\": %zu, \"rtcp_sec_serv\": %d, "
            "\"use_mki\": 0, \"mki_size\": 0, \"window_size\": %zu, "
            "\"allow_repeat_tx\": %d, \"use_cryptex\": %d, \"enc_xtn_hdr\": [",
            (int)p->ssrc.type, p->ssrc.value, p->rtp.cipher_type,
            p->rtp.cipher_key_len, p->rtp.auth_type, p->rtp.auth_key_len,
            p->rtp.auth_tag_len, (int)p->rtp.sec_serv, p->rtcp.cipher_type,
            p->rtcp.cipher_key_len, p->rtcp.auth_type, p->rtcp.auth_key_len,
            p->rtcp.auth_tag_len, (int)p->rtcp.sec_serv, p->window_size,
            (int)p->allow_repeat_tx, (int)p->use_cryptex);
    for (size_t i = 0; i < p->enc_xtn_hdr_count; i++)
        fprintf(g_out, "%s%u", i ? ", " : "", p->enc_xtn_hdr[i]);
    fputs("], \"keys\": [", g_out);
    hex(key, 64);
    fputs("], \"mki_ids\": []}", g_out);
}

typedef struct {
    srtp_t snd, rcv;
    srtp_policy_t ps, pr;
    uint8_t key[64];
} pair_t;

static void case_begin(pair_t *pp, const char *name, const char *cite)
{
    if (srtp_create(&pp->snd, &pp->ps) || srtp_create(&pp->rcv, &pp->pr)) {
        fprintf(stderr, "srtp_create failed for %s\n", name);
        exit(1);
    }
    fprintf(g_out, "%s    {\"name\": \"%s\", \"cite\": \"%s\", \"snd\": ",
            g_first_case ? "" : ",\n", name, cite);
    g_first_case = 0;
    emit_policy(&pp->ps, pp->key);
    fputs(", \"rcv\": ", g_out);
    emit_policy(&pp->pr, pp->key);
    fputs(", \"ops\": [", g_out);
    g_first_item = 1;
}

static void case_end(pair_t *pp)
{
    fputs("\n    ]}", g_out);
    srtp_dealloc(pp->snd);
    srtp_dealloc(pp->rcv);
}

/* one op; returns the status, the output in out/olen */
static int op(pair_t *pp, int rcv, int protect, const uint8_t *in,
              size_t len, int inplace, uint8_t *out, size_t *olen)
{
    uint8_t buf[2400];
    size_t cap = protect ? len + 64 : len;
    srtp_t s = rcv ? pp->rcv : pp->snd;
    srtp_err_status_t st;
    memset(buf, 0, sizeof buf);
    memcpy(buf, in, len); /* see the header comment */
    *olen = cap;
    if (protect)
        st = srtp_protect(s, inplace ? buf : in, len, buf, olen, 0);
    else
        st = srtp_unprotect(s, inplace ? buf : in, len, buf, olen);
    fputs(g_first_item ? "\n    {" : ",\n    {", g_out);
    g_first_item = 0;
    fprintf(g_out, "\"sess\": \"%s\", \"op\": \"%s\", \"inplace\": %d, "
                   "\"in\": ",
            rcv ? "rcv" : "snd", protect ? "protect" : "unprotect", inplace);
    hex(in, len);
    fprintf(g_out, ", \"cap\": %zu, \"status\": %d, \"out\": ", cap, (int)st);
    if (st == 0)
        hex(buf, *olen);
    else
        fputs("null", g_out);
    fputs("}", g_out);
    if (st == 0)
        memcpy(out, buf, *olen);
    return (int)st;
}

static void pair_init(pair_t *pp, void (*set)(srtp_crypto_policy_t *),
                      const uint8_t *key, size_t klen, uint32_t ssrc)
{
    memset(pp, 0, sizeof *pp);
    set(&pp->ps.rtp);
    set(&pp->ps.rtcp);
    memcpy(pp->key, key, klen);
    pp->ps.key = pp->key;
    pp->ps.ssrc.type = ssrc_specific;
    pp->ps.ssrc.value = ssrc;
    pp->ps.window_size = 128;
    pp->pr = pp->ps;
}

/* ---- published vectors ------------------------------------------------ */
static const uint8_t k_test_key[30] = {
    0xe1, 0xf9, 0x7a, 0x0d, 0x3e, 0x01, 0x8b, 0xe0, 0xd6, 0x4f,
    0xa3, 0x2c, 0x06, 0xde, 0x41, 0x39, 0x0e, 0xc6, 0x75, 0xad,
    0x49, 0x8a, 0xfe, 0xeb, 0xb6, 0x96, 0x0b, 0x3a, 0xab, 0xe6
};
#ifdef REF_OSSL
static const uint8_t k_test_key_gcm[28] = {
    0x00, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07, 0x08, 0x09,
    0x0a, 0x0b, 0x0c, 0x0d, 0x0e, 0x0f, 0xa0, 0xa1, 0xa2, 0xa3,
    0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xab
};
#endif

#define AB16 "abababababababababababababababab"
static const char *k_cryptex_pt[6] = {
    "900f1235decafbadcafebabebede000151000200" AB16,
    "900f1236decafbadcafebabe1000000105020002" AB16,
    "920f1238decafbadcafebabe0001e2400000b26ebede000151000200" AB16,
    "920f1239decafbadcafebabe0001e2400000b26e1000000105020002" AB16,
    "920f123adecafbadcafebabe0001e2400000b26ebede0000" AB16,
    "920f123bdecafbadcafebabe0001e2400000b26e10000000" AB16,
};
#ifndef REF_OSSL
/* test/srtp_driver.c:3019-3175, AES-CM-128/HMAC-SHA1-80 */
static const char *k_cryptex_ct[6] = {
    "900f1235decafbadcafebabec0de0001eb92365251c3e036f8de27e9c27ee3e0"
    "b4651d9fbc4218a70244522f34a5",
    "900f1236decafbadcafebabec2de00014ed9cc4e6a712b3096c5ca77339d4204"
    "ce0d77396cab69585fbce38194a5",
    "920f1238decafbadcafebabe8bb6e12b5cff16ddc0de000192838c8c09e58393"
    "e1de3a9a74734d6745671338c3acf11da2df8423bee0",
    "920f1239decafbadcafebabef70e513eb90b9b25c2de0001bbed4848faa64466"
    "5f3d7f34125914e9f4d0ae923c6f479b95a0f7b53133",
    "920f123adecafbadcafebabe7130b6abfe2ab0e3c0de0000e3d9f64b25c9e74c"
    "b4cf8e43fb92e3781c2c0ceab6b3a499a14c",
    "920f123bdecafbadcafebabecbf24c124330e1c8c2de0000599dd45bc9d687b6"
    "03e8b59d771fd38e88b170e0cd31e125eabe",
};
#else
/* test/srtp_driver.c:3575-3738, AES-GCM-128 (16-byte tag) */
static const char *k_cryptex_ct[6] = {
    "900f1235decafbadcafebabec0de000139972dc9572c4d99e8fc355de743fb2e"
    "94f9d8ff54e72f4193bbc5c74ffab0fa9fa0fbeb",
    "900f1236decafbadcafebabec2de0001bb75a4c545cd1f413bdb7daa2b1e3263"
    "de313667c963249081b35a65f5cb6c88b394235f",
    "920f1238decafbadcafebabe63bbccc4a7f695c4c0de00018ad7c71fac70a80c"
    "92866b4c6ba98546ef913586e95ffaaffe956885bb0647a8bc094ac8",
    "920f1239decafbadcafebabe3680524f8d312b00c2de0001c78d120038422bc1"
    "11a7187a18246f980c059cc6bc9df8b626394eca344e4b05d80fea83",
    "920f123adecafbadcafebabe15b6bb4337906fffc0de0000b7b964537a2b03ab"
    "7ba5389ce93317126b5d974df30c6884dcb651c5e120c1da",
    "920f123bdecafbadcafebabedcb38c9e48bf95f4c2de000061ee432cf9203170"
    "76613258d3ce4236c06ac429681ad08413512dc98b5207d8",
};
#endif

static void fail(const char *what)
{
    fprintf(stderr, "reference build fails %s\n", what);
    exit(1);
}

static void gen_cryptex_kats(void)
{
    for (int v = 0; v < 6; v++)
        for (int inplace = 1; inplace >= 0; inplace--) {
            pair_t pp;
            char name[64];
            uint8_t pt[128], ct[128], out[256];
            size_t ptl = unhex(k_cryptex_pt[v], pt);
            size_t ctl = unhex(k_cryptex_ct[v], ct), ol;
#ifndef REF_OSSL
            pair_init(&pp, srtp_crypto_policy_set_rtp_default, k_test_key, 30,
                      0xcafebabe);
            snprintf(name, sizeof name, "kat_cryptex_%d_%s", v,
                     inplace ? "inplace" : "io");
            const char *cite = "test/srtp_driver.c:3004-3264";
#else
            pair_init(&pp, srtp_crypto_policy_set_aes_gcm_128_16_auth,
                      k_test_key_gcm, 28, 0xcafebabe);
            snprintf(name, sizeof name, "kat_gcm_cryptex_%d_%s", v,
                     inplace ? "inplace" : "io");
            const char *cite = "test/srtp_driver.c:3553-3841";
#endif
            pp.ps.use_cryptex = pp.pr.use_cryptex = true;
            case_begin(&pp, name, cite);
            int st = op(&pp, 0, 1, pt, ptl, inplace, out, &ol);
#ifdef REF_OSSL
            if (!inplace && (pt[0] & 0x0f)) {
                /* cryptex + CSRCs + AEAD not in place (srtp_driver.c:3803) */
                if (st != srtp_err_status_cryptex_err)
                    fail("gcm cryptex not-in-place CSRC status");
                case_end(&pp);
                continue;
            }
#endif
            if (st || ol != ctl || memcmp(out, ct, ctl))
                fail("cryptex protect vector");
            st = op(&pp, 1, 0, ct, ctl, inplace, out, &ol);
            if (st || ol != ptl || memcmp(out, pt, ptl))
fail("cryptex unprotect vector");
            case_end(&pp);
        }
    /* srtp_test_cryptex_csrc_but_no_extension_header (srtp_driver.c:3266) */
    {
        pair_t pp;
        uint8_t pt[128], out[256];
        size_t ol;
        size_t ptl = unhex("820f1238decafbadcafebabe0001e2400000b26e" AB16, pt);
#ifndef REF_OSSL
        pair_init(&pp, srtp_crypto_policy_set_rtp_default, k_test_key, 30,
                  0xcafebabe);
#else
        pair_init(&pp, srtp_crypto_policy_set_aes_gcm_128_16_auth,
                  k_test_key_gcm, 28, 0xcafebabe);
#endif
        pp.ps.use_cryptex = pp.pr.use_cryptex = true;
        case_begin(&pp, "kat_cryptex_csrc_no_xtn",
                   "test/srtp_driver.c:3266-3311");
        for (int inplace = 1; inplace >= 0; inplace--)
            if (op(&pp, 0, 1, pt, ptl, inplace, out, &ol) !=
                srtp_err_status_cryptex_err)
                fail("cryptex csrc without extension");
        case_end(&pp);
    }
}

/* RFC 6904 Appendix A (srtp_driver.c:3848-3970, _gcm 3976-4098) */
static void gen_xtn_kat(void)
{
    static const uint8_t ids[3] = { 1, 3, 4 };
    const char *pt_hex = "900f1234decafbadcafebabebede000617414273a4752627"
                         "48220000c8308e4655996386b395fb00" AB16;
    for (int inplace = 1; inplace >= 0; inplace--) {
        pair_t pp;
        uint8_t pt[128], out[256], back[256];
        size_t ptl = unhex(pt_hex, pt), ol, bl;
#ifndef REF_OSSL
        static const uint8_t exp[66] = {
            0x90, 0x0f, 0x12, 0x34, 0xde, 0xca, 0xfb, 0xad, 0xca, 0xfe, 0xba,
            0xbe, 0xBE, 0xDE, 0x00, 0x06, 0x17, 0x58, 0x8A, 0x92, 0x70, 0xF4,
            0xE1, 0x5E, 0x1C, 0x22, 0x00, 0x00, 0xC8, 0x30, 0x95, 0x46, 0xA9,
            0x94, 0xF0, 0xBC, 0x54, 0x78, 0x97, 0x00, 0x4e, 0x55, 0xdc, 0x4c,
            0xe7, 0x99, 0x78, 0xd8, 0x8c, 0xa4, 0xd2, 0x15, 0x94, 0x9d, 0x24,
            0x02, 0x5a, 0x46, 0xb3, 0xca, 0x35, 0xc5, 0x35, 0xa8, 0x91, 0xc7
        };
        pair_init(&pp, srtp_crypto_policy_set_rtp_default, k_test_key, 30,
                  0xcafebabe);
        const char *cite = "test/srtp_driver.c:3848-3970";
        const char *name = inplace ? "kat_xtn_rfc6904_inplace"
                                   : "kat_xtn_rfc6904_io";
#else
        static const uint8_t exp[72] = {
            0x90, 0x0f, 0x12, 0x34, 0xde, 0xca, 0xfb, 0xad, 0xca, 0xfe, 0xba,
            0xbe, 0xBE, 0xDE, 0x00, 0x06, 0x17, 0x12, 0xe0, 0x20, 0x5b, 0xfa,
            0x94, 0x9b, 0x1C, 0x22, 0x00, 0x00, 0xC8, 0x30, 0xbb, 0x46, 0x73,
            0x27, 0x78, 0xd9, 0x92, 0x9a, 0xab, 0x00, 0x0e, 0xca, 0x0c, 0xf9,
            0x5e, 0xe9, 0x55, 0xb2, 0x6c, 0xd3, 0xd2, 0x88, 0xb4, 0x9f, 0x6c,
            0xa9, 0xf4, 0xb1, 0xb7, 0x59, 0x71, 0x9e, 0xb5, 0xbc, 0x11, 0x3b,
            0x9f, 0xf1, 0xd4, 0x0c, 0xd2, 0x5a
        };
        /* the driver keys AES-GCM-128 with its 30-byte test key */
        pair_init(&pp, srtp_crypto_policy_set_aes_gcm_128_16_auth, k_test_key,
                  30, 0xcafebabe);
        const char *cite = "test/srtp_driver.c:3976-4098";
        const char *name = inplace ? "kat_xtn_rfc6904_gcm_inplace"
                                   : "kat_xtn_rfc6904_gcm_io";
#endif
        pp.ps.enc_xtn_hdr = pp.pr.enc_xtn_hdr = (uint8_t *)ids;
        pp.ps.enc_xtn_hdr_count = pp.pr.enc_xtn_hdr_count = 3;
        case_begin(&pp, name, cite);
        if (op(&pp, 0, 1, pt, ptl, inplace, out, &ol) || ol != sizeof exp ||
            memcmp(out, exp, sizeof exp))
            fail("RFC 6904 protect vector");
        if (op(&pp, 1, 0, exp, sizeof exp, inplace, back, &bl) || bl != ptl ||
            memcmp(back, pt, ptl))
            fail("RFC 6904 unprotect vector");
        case_end(&pp);
    }
}

/* ---- random rows ---------------------------------------------------- */
/* an RTP packet: `prof` 0 = no extension; elements from the rng (one-byte
 * or two-byte by the profile), `mode` 1 adds an ID 15 element, 2 makes the
 * last element overrun the extension */
static size_t build(uint8_t *p, uint32_t ssrc, uint16_t seq, int cc,
                    uint16_t prof, int mode, size_t payload)
{
    size_t h = 12;
    p[0] = (uint8_t)(0x80 | (prof ? 0x10 : 0) | cc);
    p[1] = 96;
    p[2] = (uint8_t)(seq >> 8);
    p[3] = (uint8_t)seq;
    rfill(p + 4, 4);
    p[8] = (uint8_t)(ssrc >> 24);
    p[9] = (uint8_t)(ssrc >> 16);
    p[10] = (uint8_t)(ssrc >> 8);
    p[11] = (uint8_t)ssrc;
    rfill(p + h, 4 * (size_t)cc);
    h += 4 * (size_t)cc;
    if (prof) {
        uint8_t x[256];
        size_t n = 0;
        int two = (prof & 0xfff0) == 0x1000;
        int ne = 1 + (int)(rng() % 5);
        for (int e = 0; e < ne && n < 200; e++) {
            if (rng() % 4 == 0)
                x[n++] = 0; /* padding */
            if (two) {
                static const uint8_t tid[6] = { 1, 3, 4, 7, 200, 0 };
                uint8_t len = (uint8_t)(rng() % 9);
                x[n++] = tid[rng() % 6];
                x[n++] = len;
                rfill(x + n, len);
                n += len;
            } else {
                uint8_t id = (uint8_t)(1 + rng() % 14);
                uint8_t len = (uint8_t)(1 + rng() % 8);
                x[n++] = (uint8_t)(id << 4 | (len - 1));
                rfill(x + n, len);
                n += len;
            }
        }
        if (mode == 2) {
            /* an element whose length runs past the end */
            if (two) {
                x[n++] = 3;
                x[n++] = 40;
            } else {
                x[n++] = 0x2f;
            }
            x[n++] = 0x55;
        }
        if (mode == 1 && !two) {
            x[n++] = 0xf3; /* ID 15: the walk stops here */
            rfill(x + n, 6);
            n += 6;
        }
        while (n % 4)
            x[n++] = 0;
        p[h] = (uint8_t)(prof >> 8);
        p[h + 1] = (uint8_t)prof;
        p[h + 2] = (uint8_t)((n / 4) >> 8);
        p[h + 3] = (uint8_t)(n / 4);
        memcpy(p + h + 4, x, n);
        h += 4 + n;
    }
    rfill(p + h, payload);
    return h + payload;
}

typedef struct {
    const char *name;
    void (*set)(srtp_crypto_policy_t *);
    size_t key_len;
    int xtn, cryptex, gcm, auth_only;
} xdesc_t;

static void aes_cm_128_auth_only(srtp_crypto_policy_t *p)
{
    srtp_crypto_policy_set_rtp_default(p);
    p->sec_serv = sec_serv_auth;
}

static void gen_random(const xdesc_t *d)
{
    static const uint8_t ids[5] = { 1, 3, 4, 7, 200 };
    pair_t pp;
    uint8_t key[64];
    rfill(key, sizeof key);
    pair_init(&pp, d->set, key, 64, 0x5eed0000u + (uint32_t)(rng() & 0xffff));
    if (d->xtn) {
        pp.ps.enc_xtn_hdr = pp.pr.enc_xtn_hdr = (uint8_t *)ids;
        pp.ps.enc_xtn_hdr_count = pp.pr.enc_xtn_hdr_count = 5;
    }
    pp.ps.use_cryptex = pp.pr.use_cryptex = d->cryptex;
    case_begin(&pp, d->name, "srtp/srtp.c:135-305, 1802-1894");
    static const uint16_t profs[4] = { 0, 0xbede, 0x1000, 0x1003 };
    static const size_t pays[5] = { 0, 1, 17, 160, 1000 };
    uint8_t rtp[2200], srtp[2400], back[2400];
    uint16_t seq = (uint16_t)rng();
    uint32_t ssrc = pp.ps.ssrc.value;
    for (int i = 0; i < 48; i++) {
        int cc = (int)(rng() % 3) * ((rng() & 1) ? 1 : 2); /* 0..4 */
        uint16_t prof = profs[rng() % 4];
        int mode = (int)(rng() % 8);
        mode = mode == 1 ? 1 : (mode == 2 && d->xtn ? 2 : 0);
        if (i % 16 == 15)
            prof = 0x1234; /* not an RFC 8285 profile */
        int pin = (int)(rng() & 1), uin = (int)(rng() & 1);
        if (d->cryptex && !prof && cc && (rng() & 3))
            cc = 0; /* cryptex_err rows: a few */
        size_t len = build(rtp, ssrc, seq++, cc, prof, mode, pays[rng() % 5]);
        size_t sl, bl;
        if (op(&pp, 0, 1, rtp, len, pin, srtp, &sl))
            continue;
        if (d->gcm && uin && d->cryptex && d->xtn && cc) {
            /* see the header comment: the last CSRC must not read as an
             * extension profile */
            uint16_t v = (uint16_t)(rtp[12 + 4 * cc - 4] << 8 |
                                    rtp[12 + 4 * cc - 3]);
            if (v == 0xbede || (v & 0xfff0) == 0x1000)
                uin = 0;
        }
        if (i % 12 == 5) {
            uint8_t bad[2400];
            memcpy(bad, srtp, sl);
            bad[sl - 1] ^= 0x10;
            op(&pp, 1, 0, bad, sl, uin, back, &bl);
        }
        op(&pp, 1, 0, srtp, sl, uin, back, &bl);
        if (i % 12 == 7)
            op(&pp, 1, 0, srtp, sl, !uin, back, &bl); /* replay */
    }
    case_end(&pp);
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
#ifndef REF_OSSL
    fputs("{\n  \"backend\": \"internal\",\n  \"cases\": [\n", g_out);
#else
    fputs("{\n  \"backend\": \"openssl\",\n  \"cases\": [\n", g_out);
#endif
    gen_cryptex_kats();
    gen_xtn_kat();
    /* the sender without cryptex, the receiver with it: cryptex is detected
     * by the profile on the wire (srtp_driver.c:3313-3379) */
    {
        pair_t pp;
        uint8_t key[64], rtp[256], srtp[320], back[320];
        size_t sl, bl;
        rfill(key, sizeof key);
#ifndef REF_OSSL
        pair_init(&pp, srtp_crypto_policy_set_rtp_default, key, 64, 0xcafebabe);
#else
        pair_init(&pp, srtp_crypto_policy_set_aes_gcm_256_16_auth, key, 64,
                  0xcafebabe);
#endif
        pp.pr.use_cryptex = true;
        case_begin(&pp, "cryptex_receiver_only", "test/srtp_driver.c:3313-3379");
        for (int i = 0; i < 6; i++) {
            size_t len = build(rtp, 0xcafebabe, (uint16_t)(100 + i), i % 3,
                               i % 2 ? 0xbede : 0x1000, 0, 40);
            if (!op(&pp, 0, 1, rtp, len, i & 1, srtp, &sl))
                op(&pp, 1, 0, srtp, sl, (i >> 1) & 1, back, &bl);
        }
        case_end(&pp);
    }
#ifndef REF_OSSL
    static const xdesc_t xs[] = {
        { "icm128_xtn", srtp_crypto_policy_set_rtp_default, 30, 1, 0, 0, 0 },
        { "icm128_cryptex", srtp_crypto_policy_set_rtp_default, 30, 0, 1, 0, 0 },
        { "icm128_xtn_cryptex", srtp_crypto_policy_set_rtp_default, 30, 1, 1, 0,
          0 },
        { "icm256_hmac32_xtn_cryptex",
          srtp_crypto_policy_set_aes_cm_256_hmac_sha1_32, 46, 1, 1, 0, 0 },
        { "icm128_nullauth_xtn_cryptex",
          srtp_crypto_policy_set_aes_cm_128_null_auth, 30, 1, 1, 0, 0 },
        { "null_hmac80_xtn_cryptex",
          srtp_crypto_policy_set_null_cipher_hmac_sha1_80, 30, 1, 1, 0, 0 },
        { "icm128_authonly_xtn_cryptex", aes_cm_128_auth_only, 30, 1, 1, 0, 1 },
    };
#else
    static const xdesc_t xs[] = {
        { "gcm128_xtn", srtp_crypto_policy_set_aes_gcm_128_16_auth, 28, 1, 0, 1,
          0 },
        { "gcm128_cryptex", srtp_crypto_policy_set_aes_gcm_128_16_auth, 28, 0,
          1, 1, 0 },
        { "gcm256_xtn_cryptex", srtp_crypto_policy_set_aes_gcm_256_16_auth, 44,
          1, 1, 1, 0 },
        { "icm192_xtn_cryptex", srtp_crypto_policy_set_aes_cm_192_hmac_sha1_80,
          38, 1, 1, 0, 0 },
    };
#endif
    for (size_t i = 0; i < sizeof xs / sizeof xs[0]; i++)
        gen_random(&xs[i]);
    fputs("\n  ]\n}\n", g_out);
    fclose(g_out);
    srtp_shutdown();
    return 0;
}
