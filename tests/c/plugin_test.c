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
static srtp_err_status_t u_crypt(void *s, const uint8_t *src, size_t n,
                                 uint8_t *dst, size_t *dn)
{
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
    user_hmac.description = "user HMAC-SHA1";
    CHECK(srtp_replace_auth_type(&user_hmac, SRTP_HMAC_SHA1) ==
              srtp_err_status_ok,
          "auth replacement accepted");
    CHECK(srtp_mi355x_registered_auth_type(SRTP_HMAC_SHA1) == &user_hmac,
          "auth registered");

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
