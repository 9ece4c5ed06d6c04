/*
 * percall_bench.c -- the drop-in per-call path: an unchanged libsrtp caller
 * makes one srtp_protect() / srtp_unprotect() per packet, and through this
 * library each call is a GPU batch of one (DESIGN.md §6 "Per-call path").
 * The loop is srtp_bits_per_second's (reference test/srtp_driver.c:
 * 1202-1268): one reused 1412-byte RTP packet (1400-byte payload), its
 * sequence number advanced after every protect, `calls` calls timed with a
 * monotonic clock.  Unprotect: a sender session protects the same number of
 * packets first (untimed, stored), then each is unprotected in order, one
 * call per packet.  Cipher: AES-128-ICM + HMAC-SHA1-80 (the reference's
 * default policy) or AES-256-GCM-16.
 *
 *   usage: percall_bench [calls] [icm|gcm]
 *   prints one JSON line: per-call microseconds and calls/s, both ops.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "srtp_mi355x.h"

#define PAYLOAD 1400
#define RTP_LEN (12 + PAYLOAD)
#define SLOT (RTP_LEN + 64)

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

#define CHECK(x)                                                               \
    do {                                                                       \
        srtp_err_status_t s_ = (x);                                            \
        if (s_ != srtp_err_status_ok) {                                        \
            fprintf(stderr, "%s:%d: %s -> %d\n", __FILE__, __LINE__, #x,       \
                    (int)s_);                                                  \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

static srtp_t make_session(int gcm, uint8_t *key)
{
    srtp_policy_t p;
    memset(&p, 0, sizeof p);
    if (gcm) {
        srtp_crypto_policy_set_aes_gcm_256_16_auth(&p.rtp);
        srtp_crypto_policy_set_aes_gcm_256_16_auth(&p.rtcp);
    } else {
        srtp_crypto_policy_set_rtp_default(&p.rtp);
        srtp_crypto_policy_set_rtp_default(&p.rtcp);
    }
    p.ssrc.type = ssrc_specific;
    p.ssrc.value = 0xdeadbeef;
    p.key = key;
    p.window_size = 128;
    srtp_t s;
    CHECK(srtp_create(&s, &p));
    return s;
}

/* create_rtp_test_packet's shape: version 2, PT 1, the SSRC, seq 1, a
 * payload pattern */
static void make_packet(uint8_t *p, uint16_t seq)
{
    memset(p, 0, SLOT);
    p[0] = 0x80;
    p[1] = 1;
    p[2] = (uint8_t)(seq >> 8);
    p[3] = (uint8_t)seq;
    p[8] = 0xde;
    p[9] = 0xad;
    p[10] = 0xbe;
    p[11] = 0xef;
    for (int i = 0; i < PAYLOAD; i++)
        p[12 + i] = (uint8_t)(0xab ^ i);
}

int main(int argc, char **argv)
{
    const long calls = argc > 1 ? atol(argv[1]) : 100000;
    const int gcm = argc > 2 && strcmp(argv[2], "gcm") == 0;
    uint8_t key[46];
    for (int i = 0; i < 46; i++)
        key[i] = (uint8_t)(0x11 * i + 3);
    CHECK(srtp_init());
    if (!srtp_mi355x_gpu_available()) {
        fprintf(stderr, "no HIP device\n");
        return 1;
    }

    /* protect: srtp_bits_per_second's loop */
    srtp_t snd = make_session(gcm, key);
    uint8_t *msg = malloc(SLOT);
    make_packet(msg, 1);
    for (int w = 0; w < 200; w++) {   /* warm-up: first launches, caches */
        uint8_t tmp[SLOT];
        memcpy(tmp, msg, SLOT);
        size_t len = SLOT;
        CHECK(srtp_protect(snd, tmp, RTP_LEN, tmp, &len, 0));
        uint16_t s = (uint16_t)((msg[2] << 8 | msg[3]) + 1);
        msg[2] = (uint8_t)(s >> 8);
        msg[3] = (uint8_t)s;
    }
    double t0 = now();
    for (long i = 0; i < calls; i++) {
        size_t len = SLOT;   /* capacity in, protected length out */
        /* in place, as call_srtp_protect does with its one buffer */
        CHECK(srtp_protect(snd, msg, RTP_LEN, msg, &len, 0));
        /* the next packet: the same bytes, the sequence number advanced */
        uint16_t s = (uint16_t)((msg[2] << 8 | msg[3]) + 1);
        msg[2] = (uint8_t)(s >> 8);
        msg[3] = (uint8_t)s;
    }
    const double tp = now() - t0;

    /* unprotect: a second sender makes `calls` packets (untimed), a receiver
     * takes them one call each, in order */
    srtp_t snd2 = make_session(gcm, key), rcv = make_session(gcm, key);
    uint8_t *arena = malloc((size_t)(calls + 200) * SLOT);
    size_t *lens = malloc((size_t)(calls + 200) * sizeof(size_t));
    for (long i = 0; i < calls + 200; i++) {
        uint8_t *p = arena + (size_t)i * SLOT;
        make_packet(p, (uint16_t)(1 + i));
        lens[i] = SLOT;
        CHECK(srtp_protect(snd2, p, RTP_LEN, p, &lens[i], 0));
    }
    for (long i = 0; i < 200; i++) {
        size_t len = lens[i];
        uint8_t *p = arena + (size_t)i * SLOT;
        CHECK(srtp_unprotect(rcv, p, lens[i], p, &len));
    }
    t0 = now();
    for (long i = 200; i < calls + 200; i++) {
        size_t len = lens[i];
        uint8_t *p = arena + (size_t)i * SLOT;
        CHECK(srtp_unprotect(rcv, p, lens[i], p, &len));
    }
    const double tu = now() - t0;

    printf("{\"cipher\": \"%s\", \"calls\": %ld, \"payload\": %d, "
           "\"protect_us_per_call\": %.3f, \"protect_calls_per_s\": %.1f, "
           "\"unprotect_us_per_call\": %.3f, \"unprotect_calls_per_s\": %.1f}\n",
           gcm ? "AES-256-GCM-16" : "AES-128-ICM + HMAC-SHA1-80", calls,
           PAYLOAD, tp / calls * 1e6, calls / tp, tu / calls * 1e6,
           calls / tu);
    srtp_dealloc(snd);
    srtp_dealloc(snd2);
    srtp_dealloc(rcv);
    free(msg);
    free(arena);
    free(lens);
    return 0;
}
