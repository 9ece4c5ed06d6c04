/*
 * plugin_test.c -- the crypto-kernel plugin ABI (srtp.def:46-69) of
 * libsrtp_mi355x, driven the way the reference's own callers drive it
 * (test/cipher_driver.c, test/kernel_driver.c, crypto_kernel.c:270-440).
 *
 *   plugin_test [path/to/reference/libsrtp_ref_ossl.so]
 *
 * With the reference build given (oracle/_ref, test infrastructure), every
 * GPU-backed built-in type is also run against the REFERENCE's own known
 * answers: the test_data of its srtp_aes_icm_128 / _192 / _256,
 * srtp_aes_gcm_128 / _256 and srtp_hmac objects -- exactly what
 * srtp_replace_cipher_type checks (crypto_kernel.c:300-306).  Only data is
 * read from that library.  Exit status 0 = all checks passed.
 *
 * Routing (section 7): once a user type is registered for an id, sessions
 * using that id run their packet crypto through the registered vtable, as
 * the reference's do (srtp.c:594-752 allocates the stream's cipher / auth
 * from the crypto kernel).  The wrappers count their calls; batches
 * protected before and after the replacement must be bit-identical, and
 * unprotect must round-trip, refuse a tampered packet without touching it,
 * and refuse a replay.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "srtp_mi355x.h"

static int g_fail;

#define CHECK(cond, ...)                                                       \
    do {                                                                       \
        if (!(cond)) {                                                         \
            printf("FAIL %s:%d: ", __FILE__, __LINE__);                        \
            printf(__VA_ARGS__);                                               \
            printf("\n");                                                      \
            g_fail++;                                                          \
        }                                                                      \
    } while (0)

static const uint8_t *hx(const char *h, uint8_t *out)
{
    size_t n = strlen(h) / 2;
    for (size_t i = 0; i < n; i++) {
        unsigned v;
        sscanf(h + 2 * i, "%2x", &v);
        out[i] = (uint8_t)v;
    }
    return out;
}

/* ---- a user cipher type: forwards to the built-in AES-ICM-128, as a
 * hardware-offload plugin would wrap its engine; `broken` flips a bit ---- */
static const srtp_cipher_type_t *g_icm;
static int g_broken;
static srtp_cipher_type_t user_icm;

static srtp_err_status_t u_alloc(srtp_cipher_t **c, size_t kl, size_t tl)
{
    srtp_err_status_t st = g_icm->alloc(c, kl, tl);
    if (!st)
        (*c)->type = &user_icm;
    return st;
}
static srtp_err_status_t u_dealloc(srtp_cipher_t *c) { return g_icm->dealloc(c); }
static srtp_err_status_t u_init(void *s, const uint8_t *k)
{
    return g_icm->init(s, k);
}
static srtp_err_status_t u_set_iv(void *s, uint8_t *iv,
                                  srtp_cipher_direction_t d)
{
    return g_icm->set_iv(s, iv, d);
}
static long g_cipher_calls, g_auth_calls;
static srtp_err_status_t u_crypt(void *s, const uint8_t *src, size_t n,
                                 uint8_t *dst, size_t *dn)
{
    g_cipher_calls++;
    srtp_err_status_t st = g_icm->encrypt(s, src, n, dst, dn);
    if (!st && g_broken && n)
        dst[0] ^= 1;
    return st;
}

/* ---- a user auth type wrapping the built-in HMAC-SHA1 ---- */
static const srtp_auth_type_t *g_hmac;
static srtp_auth_type_t user_hmac;
static srtp_err_status_t ua_alloc(srtp_auth_t **a, size_t kl, size_t ol)
{
    srtp_err_status_t st = g_hmac->alloc(a, kl, ol);
    if (!st)
        (*a)->type = &user_hmac;
    return st;
}
static srtp_err_status_t ua_compute(void *s, const uint8_t *m, size_t n,
                                    size_t tl, uint8_t *res)
{
    g_auth_calls++;
    return g_hmac->compute(s, m, n, tl, res);
}

/* ---- a user AES-GCM-256 type (AEAD: seal / open counted) ---- */
static const srtp_cipher_type_t *g_gcm;
static srtp_cipher_type_t user_gcm;
static long g_gcm_calls;
static srtp_err_status_t ug_alloc(srtp_cipher_t **c, size_t kl, size_t tl)
{
    srtp_err_status_t st = g_gcm->alloc(c, kl, tl);
    if (!st)
        (*c)->type = &user_gcm;
    return st;
}
static srtp_err_status_t ug_enc(void *s, const uint8_t *src, size_t n,
                                uint8_t *dst, size_t *dn)
{
    g_gcm_calls++;
    return g_gcm->encrypt(s, src, n, dst, dn);
}
static srtp_err_status_t ug_dec(void *s, const uint8_t *src, size_t n,
                                uint8_t *dst, size_t *dn)
{
    g_gcm_calls++;
    return g_gcm->decrypt(s, src, n, dst, dn);
}

/* ---- one session pass: a batch protected, then unprotected in place ---- */
enum { NB = 96, PK = 320 };
static uint8_t g_in[NB][PK];
static size_t g_in_len[NB];

static void make_packets(void)
{
    uint64_t x = 0x726f757465643031ULL;
    for (size_t i = 0; i < NB; i++) {
        g_in_len[i] = 12 + 1 + (i * 37) % 200;
        for (size_t j = 0; j < g_in_len[i]; j++) {
            x ^= x << 13;
            x ^= x >> 7;
            x ^= x << 17;
            g_in[i][j] = (uint8_t)x;
        }
        const uint16_t seq = (uint16_t)(0xffd0 + i); /* crosses the ROC */
        g_in[i][0] = 0x80;
        g_in[i][1] = 96;
        g_in[i][2] = (uint8_t)(seq >> 8);
        g_in[i][3] = (uint8_t)seq;
        g_in[i][8] = 0xca;
        g_in[i][9] = 0xfe;
        g_in[i][10] = 0xba;
        g_in[i][11] = 0xbe;
    }
}

/* gcm: AES-GCM-256 else AES-CM-128 + HMAC-SHA1-80; mki: two master keys
 * with 4-byte MKIs, packets alternating between them.  out / olen = the
 * protected batch. */
static void session_pass(int gcm, int mki, uint8_t out[][PK], size_t *olen)
{
    static uint8_t key[2][46], id[2][4];
    for (int k = 0; k < 2; k++)
        for (int j = 0; j < 46; j++)
            key[k][j] = (uint8_t)(0x31 * j + 7 * k + 1);
    memcpy(id[0], "\x01\x02\x03\x04", 4);
    memcpy(id[1], "\xa0\xb0\xc0\xd0", 4);
    srtp_master_key_t mk[2] = { { key[0], id[0] }, { key[1], id[1] } };
    srtp_master_key_t *mkp[2] = { &mk[0], &mk[1] };
    srtp_policy_t p;
    memset(&p, 0, sizeof p);
    if (gcm) {
        srtp_crypto_policy_set_aes_gcm_256_16_auth(&p.rtp);
        srtp_crypto_policy_set_aes_gcm_256_16_auth(&p.rtcp);
    } else {
        srtp_crypto_policy_set_rtp_default(&p.rtp);
        srtp_crypto_policy_set_rtcp_default(&p.rtcp);
    }
    p.ssrc.type = ssrc_specific;
    p.ssrc.value = 0xcafebabe;
    if (mki) {
        p.keys = mkp;
        p.num_master_keys = 2;
        p.use_mki = true;
        p.mki_size = 4;
    } else {
        p.key = key[0];
    }
    p.window_size = 128;
    srtp_t tx, rx;
    CHECK(srtp_create(&tx, &p) == 0 && srtp_create(&rx, &p) == 0,
          "create gcm=%d mki=%d", gcm, mki);
    const uint8_t *in[NB];
    uint8_t *op[NB];
    size_t mi[NB];
    srtp_err_status_t st[NB];
    for (size_t i = 0; i < NB; i++) {
        in[i] = g_in[i];
        op[i] = out[i];
        olen[i] = PK;
        mi[i] = mki ? i & 1 : 0;
    }
    CHECK(srtp_protect_batch(tx, NB, in, g_in_len, op, olen, mi, st) == 0,
          "protect batch");
    int bad = 0;
    for (size_t i = 0; i < NB; i++)
        bad += st[i] != 0 || olen[i] != g_in_len[i] + (mki ? 4 : 0) +
                                               (gcm ? 16 : 10);
    CHECK(!bad, "protect statuses / lengths gcm=%d mki=%d: %d bad", gcm, mki,
          bad);
    /* receive in place; packet 5 tampered */
    static uint8_t rxb[NB][PK];
    uint8_t *rp[NB];
    size_t rl[NB];
    for (size_t i = 0; i < NB; i++) {
        memcpy(rxb[i], out[i], olen[i]);
        rp[i] = rxb[i];
        rl[i] = olen[i];
    }
    rxb[5][20] ^= 1;
    uint8_t tampered[PK];
    memcpy(tampered, rxb[5], olen[5]);
    CHECK(srtp_unprotect_batch(rx, NB, (const uint8_t *const *)rp, rl, rp, rl,
                               st) == 0,
          "unprotect batch");
    bad = 0;
    for (size_t i = 0; i < NB; i++) {
        if (i == 5)
            continue;
        bad += st[i] != 0 || rl[i] != g_in_len[i] ||
               memcmp(rxb[i], g_in[i], g_in_len[i]) != 0;
    }
    CHECK(!bad, "round trip gcm=%d mki=%d: %d bad", gcm, mki, bad);
    CHECK(st[5] == srtp_err_status_auth_fail &&
              memcmp(rxb[5], tampered, olen[5]) == 0,
          "tampered packet refused untouched (status %d)", st[5]);
    uint8_t again[PK];
    size_t al = olen[7];
    memcpy(again, out[7], olen[7]);
    CHECK(srtp_unprotect(rx, again, al, again, &al) ==
              srtp_err_status_replay_fail,
          "replay refused");
    srtp_dealloc(tx);
    srtp_dealloc(rx);
}

static void log_cb(srtp_log_level_t level, const char *msg, void *data)
{
    (void)level;
    snprintf((char *)data, 256, "%s", msg);
}

int main(int argc, char **argv)
{
    uint8_t b1[256], b2[256], b3[256];
    CHECK(srtp_init() == srtp_err_status_ok, "srtp_init");

    /* 1. the built-in (GPU-backed) types pass their own known answers */
    static const srtp_cipher_type_id_t cids[] = {
        SRTP_NULL_CIPHER, SRTP_AES_ICM_128, SRTP_AES_ICM_192,
        SRTP_AES_ICM_256, SRTP_AES_GCM_128, SRTP_AES_GCM_256
    };
    for (size_t i = 0; i < sizeof cids / sizeof *cids; i++) {
        const srtp_cipher_type_t *t = srtp_mi355x_builtin_cipher_type(cids[i]);
        CHECK(t && t->id == cids[i], "builtin cipher %u", cids[i]);
        if (t)
            CHECK(srtp_cipher_type_self_test(t) == srtp_err_status_ok,
                  "self test %s", t->description);
    }
    g_hmac = srtp_mi355x_builtin_auth_type(SRTP_HMAC_SHA1);
    CHECK(g_hmac && srtp_auth_type_self_test(g_hmac) == srtp_err_status_ok,
          "hmac self test");
    CHECK(srtp_auth_type_self_test(srtp_mi355x_builtin_auth_type(
              SRTP_NULL_AUTH)) == srtp_err_status_ok,
          "null auth self test");

    /* 2. ... and the reference's own known answers */
    if (argc > 1) {
        void *ref = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
        CHECK(ref != NULL, "dlopen %s: %s", argv[1], dlerror());
        static const struct {
            const char *sym;
            srtp_cipher_type_id_t id;
        } rc[] = { { "srtp_aes_icm_128", SRTP_AES_ICM_128 },
                   { "srtp_aes_icm_192", SRTP_AES_ICM_192 },
                   { "srtp_aes_icm_256", SRTP_AES_ICM_256 },
                   { "srtp_aes_gcm_128", SRTP_AES_GCM_128 },
                   { "srtp_aes_gcm_256", SRTP_AES_GCM_256 },
                   { "srtp_null_cipher", SRTP_NULL_CIPHER } };
        for (size_t i = 0; ref && i < sizeof rc / sizeof *rc; i++) {
            const srtp_cipher_type_t *rt =
                (const srtp_cipher_type_t *)dlsym(ref, rc[i].sym);
            CHECK(rt != NULL, "dlsym %s", rc[i].sym);
            if (!rt)
                continue;
            srtp_err_status_t st = srtp_cipher_type_test(
                srtp_mi355x_builtin_cipher_type(rc[i].id), rt->test_data);
            CHECK(st == srtp_err_status_ok, "reference KATs of %s: %d",
                  rc[i].sym, st);
            printf("reference KATs of %-18s through the GPU type: %s\n",
                   rc[i].sym, st ? "FAIL" : "ok");
        }
        const srtp_auth_type_t *rh =
            ref ? (const srtp_auth_type_t *)dlsym(ref, "srtp_hmac") : NULL;
        if (rh) {
            srtp_err_status_t st = srtp_auth_type_test(g_hmac, rh->test_data);
            CHECK(st == srtp_err_status_ok, "reference KATs of srtp_hmac");
            printf("reference KATs of %-18s through the GPU type: %s\n",
                   "srtp_hmac", st ? "FAIL" : "ok");
        }
    }

    /* 3. AES-ICM through the cipher API: RFC 3711 B.2 keystream, produced
     * in pieces (the keystream carry-over between calls), and output() */
    g_icm = srtp_mi355x_builtin_cipher_type(SRTP_AES_ICM_128);
    srtp_cipher_t *c;
    CHECK(srtp_cipher_type_alloc(g_icm, &c, 30, 0) == srtp_err_status_ok,
          "alloc icm");
    srtp_cipher_t *bad;
    CHECK(srtp_cipher_type_alloc(g_icm, &bad, 31, 0) ==
              srtp_err_status_bad_param,
          "icm key length 31 rejected");
    hx("2b7e151628aed2a6abf7158809cf4f3cf0f1f2f3f4f5f6f7f8f9fafbfcfd", b1);
    CHECK(srtp_cipher_init(c, b1) == 0, "icm init");
    CHECK(srtp_cipher_get_key_length(c) == 30, "key length");
    uint8_t iv[16] = { 0 };
    CHECK(srtp_cipher_set_iv(c, iv, srtp_direction_encrypt) == 0, "iv");
    memset(b2, 0, sizeof b2);
    size_t pieces[] = { 5, 20, 0, 1, 6 }, off = 0;
    for (size_t i = 0; i < 5; i++) {
        size_t n = pieces[i];
        CHECK(srtp_cipher_encrypt(c, b2 + off, n, b2 + off, &n) == 0 &&
                  n == pieces[i],
              "encrypt piece %zu", i);
        off += pieces[i];
    }
    hx("e03ead0935c95e80e166b16dd92b4eb4d23513162b02d0f72a43a2fe4a5f97ab", b3);
    CHECK(memcmp(b2, b3, 32) == 0, "icm keystream in pieces: %s",
          srtp_octet_string_hex_string(b2, 32));
    CHECK(srtp_cipher_set_iv(c, iv, srtp_direction_encrypt) == 0, "iv");
    size_t n = 32;
    memset(b2, 0xaa, sizeof b2);
    CHECK(srtp_cipher_output(c, b2, &n) == 0 && n == 32 &&
              memcmp(b2, b3, 32) == 0,
          "srtp_cipher_output");
    n = 4;
    CHECK(srtp_cipher_encrypt(c, b2, 8, b2, &n) ==
              srtp_err_status_buffer_small,
          "buffer_small");
    CHECK(srtp_cipher_set_aad(c, b1, 4) == srtp_err_status_no_such_op,
          "icm has no aad");
    CHECK(srtp_cipher_bits_per_second(c, 1024, 16) > 0, "bits per second");
    CHECK(srtp_cipher_dealloc(c) == 0, "dealloc");

    /* 4. AES-GCM: AAD in two calls, seal, open, tamper */
    const srtp_cipher_type_t *gcm = srtp_mi355x_builtin_cipher_type(
        SRTP_AES_GCM_128);
    CHECK(srtp_cipher_type_alloc(gcm, &c, 28, 16) == 0, "alloc gcm");
    CHECK(srtp_cipher_type_alloc(gcm, &bad, 28, 12) ==
              srtp_err_status_bad_param,
          "gcm tag 12 rejected");
    hx("feffe9928665731c6d6a8f9467308308000000000000000000000000", b1);
    uint8_t giv[12], aad[20], pt[60], want[76];
    hx("cafebabefacedbaddecaf888", giv);
    hx("feedfacedeadbeeffeedfacedeadbeefabaddad2", aad);
    hx("d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a721c3c0c"
       "95956809532fcf0e2449a6b525b16aedf5aa0de657ba637b39",
       pt);
    hx("42831ec2217774244b7221b784d0d49ce3aa212f2c02a4e035c17e2329aca12e21d514"
       "b25466931c7d8f6a5aac84aa051ba30b396a0aac973d58e0915bc94fbc3221a5db94fa"
       "e95ae7121a47",
       want);
    CHECK(srtp_cipher_init(c, b1) == 0, "gcm init");
    CHECK(srtp_cipher_set_iv(c, giv, srtp_direction_encrypt) == 0, "gcm iv");
    CHECK(srtp_cipher_set_aad(c, aad, 7) == 0 &&
              srtp_cipher_set_aad(c, aad + 7, 13) == 0,
          "gcm aad");
    n = sizeof b2;
    CHECK(srtp_cipher_encrypt(c, pt, 60, b2, &n) == 0 && n == 76 &&
              memcmp(b2, want, 76) == 0,
          "gcm seal: %s", srtp_octet_string_hex_string(b2, n));
    CHECK(srtp_cipher_set_iv(c, giv, srtp_direction_decrypt) == 0, "iv");
    CHECK(srtp_cipher_set_aad(c, aad, 20) == 0, "aad");
    n = sizeof b3;
    CHECK(srtp_cipher_decrypt(c, want, 76, b3, &n) == 0 && n == 60 &&
              memcmp(b3, pt, 60) == 0,
          "gcm open");
    want[70] ^= 1;
    CHECK(srtp_cipher_set_iv(c, giv, srtp_direction_decrypt) == 0 &&
              srtp_cipher_set_aad(c, aad, 20) == 0,
          "iv");
    n = sizeof b3;
    CHECK(srtp_cipher_decrypt(c, want, 76, b3, &n) ==
              srtp_err_status_auth_fail,
          "gcm tampered tag");
    CHECK(srtp_cipher_set_iv(c, giv, srtp_direction_any) ==
              srtp_err_status_bad_param,
          "gcm direction any");
    CHECK(srtp_cipher_dealloc(c) == 0, "dealloc");

    /* 5. HMAC-SHA1: start / update / compute, truncated tag */
    srtp_auth_t *a;
    CHECK(srtp_auth_type_alloc(g_hmac, &a, 20, 10) == 0, "alloc hmac");
    CHECK(srtp_auth_get_key_length(a) == 20 && srtp_auth_get_tag_length(a) ==
                                                   10 &&
              srtp_auth_get_prefix_length(a) == 0,
          "hmac lengths");
    memset(b1, 0x0b, 20);
    CHECK(srtp_auth_init(a, b1) == 0 && srtp_auth_start(a) == 0, "hmac init");
    CHECK(srtp_auth_update(a, (const uint8_t *)"Hi ", 3) == 0, "update");
    uint8_t tag[20];
    CHECK(srtp_auth_compute(a, (const uint8_t *)"There", 5, tag) == 0,
          "compute");
    hx("b617318655057264e28bc0b6fb378c8ef146be00", b3);
    CHECK(memcmp(tag, b3, 10) == 0, "hmac tag: %s",
          srtp_octet_string_hex_string(tag, 10));
    CHECK(srtp_auth_dealloc(a) == 0, "dealloc");
    CHECK(srtp_auth_type_alloc(g_hmac, &a, 21, 10) ==
              srtp_err_status_bad_param,
          "hmac key 21 rejected");

    /* 6a. batches through the built-in types, before any replacement */
    static uint8_t gold[3][NB][PK], got[NB][PK];
    size_t gold_len[3][NB], got_len[NB];
    make_packets();
    session_pass(0, 0, gold[0], gold_len[0]);
    session_pass(0, 1, gold[1], gold_len[1]);
    session_pass(1, 1, gold[2], gold_len[2]);

    /* 6. replacement: a conforming user type is accepted and registered,
     * a broken one and a mismatched id are refused (crypto_kernel.c:270-330) */
    user_icm = *g_icm;
    user_icm.alloc = u_alloc;
    user_icm.dealloc = u_dealloc;
    user_icm.init = u_init;
    user_icm.set_iv = u_set_iv;
    user_icm.encrypt = u_crypt;
    user_icm.decrypt = u_crypt;
    user_icm.description = "user AES-128 ICM";
    g_broken = 1;
    CHECK(srtp_replace_cipher_type(&user_icm, SRTP_AES_ICM_128) ==
              srtp_err_status_algo_fail,
          "broken replacement refused");
    CHECK(srtp_mi355x_registered_cipher_type(SRTP_AES_ICM_128) == g_icm,
          "registry unchanged");
    g_broken = 0;
    CHECK(srtp_replace_cipher_type(&user_icm, SRTP_AES_ICM_256) ==
              srtp_err_status_bad_param,
          "id mismatch refused");
    CHECK(srtp_replace_cipher_type(NULL, SRTP_AES_ICM_128) ==
              srtp_err_status_bad_param,
          "NULL refused");
    CHECK(srtp_replace_cipher_type(&user_icm, SRTP_AES_ICM_128) ==
              srtp_err_status_ok,
          "conforming replacement accepted");
    CHECK(srtp_mi355x_registered_cipher_type(SRTP_AES_ICM_128) == &user_icm,
          "registered");
    user_hmac = *g_hmac;
    user_hmac.alloc = ua_alloc;
    user_hmac.compute = ua_compute;
    user_hmac.description = "user HMAC-SHA1";
    CHECK(srtp_replace_auth_type(&user_hmac, SRTP_HMAC_SHA1) ==
              srtp_err_status_ok,
          "auth replacement accepted");
    CHECK(srtp_mi355x_registered_auth_type(SRTP_HMAC_SHA1) == &user_hmac,
          "auth registered");
    g_gcm = srtp_mi355x_builtin_cipher_type(SRTP_AES_GCM_256);
    user_gcm = *g_gcm;
    user_gcm.alloc = ug_alloc;
    user_gcm.encrypt = ug_enc;
    user_gcm.decrypt = ug_dec;
    user_gcm.description = "user AES-256 GCM";
    CHECK(srtp_replace_cipher_type(&user_gcm, SRTP_AES_GCM_256) ==
              srtp_err_status_ok,
          "gcm replacement accepted");

    /* 7. the packet path after replacement: srtp_validate's published
     * packet (test/srtp_driver.c:2342-2426) */
    {
        srtp_policy_t p;
        srtp_t s;
        memset(&p, 0, sizeof p);
        srtp_crypto_policy_set_rtp_default(&p.rtp);
        srtp_crypto_policy_set_rtcp_default(&p.rtcp);
        p.ssrc.type = ssrc_specific;
        p.ssrc.value = 0xcafebabe;
        hx("e1f97a0d3e018be0d64fa32c06de41390ec675ad498afeebb6960b3aabe6", b1);
        p.key = b1;
        p.window_size = 128;
        CHECK(srtp_create(&s, &p) == 0, "srtp_create");
        hx("800f1234decafbadcafebabeabababababababababababababababab", b2);
        size_t len = sizeof b3;
        CHECK(srtp_protect(s, b2, 28, b3, &len, 0) == 0 && len == 38, "protect");
        hx("800f1234decafbadcafebabe4e55dc4ce79978d88ca4d215949d2402b78d6acc99ea"
           "179b8dbb",
           b1);
        CHECK(srtp_octet_string_equal(b3, b1, 38), "srtp_validate KAT: %s",
              srtp_octet_string_hex_string(b3, 38));
        srtp_dealloc(s);
    }

    /* 7b. routing: the registered types do the packet crypto, and the
     * batches come out bit-identical to the built-in ones */
    for (int v = 0; v < 3; v++) {
        const long c0 = g_cipher_calls, a0 = g_auth_calls, g0 = g_gcm_calls;
        session_pass(v == 2, v > 0, got, got_len);
        int bad = 0;
        for (size_t i = 0; i < NB; i++)
            bad += got_len[i] != gold_len[v][i] ||
                   memcmp(got[i], gold[v][i], got_len[i]) != 0;
        CHECK(!bad, "routed batch %d: %d packets differ from the built-in "
                    "types'", v, bad);
        const long dc = g_cipher_calls - c0, da = g_auth_calls - a0,
                   dg = g_gcm_calls - g0;
        /* protect NB + unprotect NB - 1 authenticated + 1 tampered (auth
         * only) + the replay (refused before any crypto) */
        if (v < 2)
            CHECK(dc >= 2 * NB - 1 && da >= 2 * NB && dg == 0,
                  "routed calls %d: cipher %ld auth %ld gcm %ld", v, dc, da,
                  dg);
        else
            CHECK(dg >= 2 * NB && dc == 0 && da == 0,
                  "routed calls %d: cipher %ld auth %ld gcm %ld", v, dc, da,
                  dg);
        printf("routed session %d (%s): bit-exact %s, calls cipher %ld "
               "auth %ld gcm %ld\n",
               v, v == 2 ? "AES-GCM-256, MKI" : v ? "AES-CM-128, MKI"
                                                 : "AES-CM-128",
               bad ? "NO" : "yes", dc, da, dg);
    }

    /* 8. the utilities */
    CHECK(!srtp_octet_string_equal((const uint8_t *)"abcd",
                                   (const uint8_t *)"abce", 4),
          "octet_string_equal");
    CHECK(strcmp(srtp_octet_string_hex_string("\x01\xab", 2), "01ab") == 0,
          "hex string");
    uint32_t words[4];
    srtp_rdbx_t r = { 5, { 128, words } };
    CHECK(srtp_rdbx_get_window_size(&r) == 128, "rdbx window size");
    static srtp_debug_module_t mod = { false, "plugin test" };
    CHECK(srtp_crypto_kernel_load_debug_module(&mod) == 0, "load module");
    CHECK(srtp_crypto_kernel_load_debug_module(&mod) ==
              srtp_err_status_bad_param,
          "module twice");
    CHECK(srtp_set_debug_module("plugin test", true) == 0 && mod.on,
          "set module");
    CHECK(srtp_set_debug_module("no such module", true) ==
              srtp_err_status_fail,
          "unknown module");
    char logged[256] = "";
    srtp_install_log_handler(log_cb, logged);
    srtp_err_report(srtp_err_level_error, "value %d", 42);
    CHECK(strcmp(logged, "value 42") == 0, "err_report -> log handler: %s",
          logged);
    srtp_install_log_handler(NULL, NULL);

    printf("%s (%d failures)\n", g_fail ? "FAILED" : "PASSED", g_fail);
    return g_fail ? 1 : 0;
}
