/*
 * rtcp_bench.c -- C-level SRTCP rate through srtp_protect_rtcp_batch /
 * srtp_unprotect_rtcp_batch (host buffers: staging, PCIe and k_rtcp
 * included).  usage: rtcp_bench [packets] [bytes] [iters]; one JSON line per
 * policy.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "srtp_mi355x.h"

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char **argv)
{
    size_t n = argc > 1 ? strtoull(argv[1], 0, 0) : 262144;
    size_t sz = argc > 2 ? strtoull(argv[2], 0, 0) : 100;
    int iters = argc > 3 ? atoi(argv[3]) : 5;
    if (sz < 8 || sz > 1500 || !n || iters < 1)
        return 2;
    if (srtp_init())
        return 1;
    const size_t cap = sz + 64;
    uint8_t *in = malloc(n * cap), *enc = malloc(n * cap), *out = malloc(n * cap);
    const uint8_t **ip = malloc(n * sizeof *ip), **ep = malloc(n * sizeof *ep);
    uint8_t **eo = malloc(n * sizeof *eo), **oo = malloc(n * sizeof *oo);
    size_t *il = malloc(n * 8), *el = malloc(n * 8), *ol = malloc(n * 8);
    srtp_err_status_t *st = malloc(n * sizeof *st);
    if (!in || !enc || !out || !ip || !ep || !eo || !oo || !il || !el || !ol ||
        !st)
        return 3;
    for (size_t i = 0; i < n; i++) {
        uint8_t *p = in + i * cap;
        for (size_t j = 0; j < sz; j++)
            p[j] = (uint8_t)(i * 131 + j * 7);
        p[0] = 0x80;
        p[1] = 200;
        p[4] = 0x12, p[5] = 0x34, p[6] = 0x56, p[7] = 0x78;
        ip[i] = p;
        il[i] = sz;
        eo[i] = enc + i * cap;
        ep[i] = eo[i];
        oo[i] = out + i * cap;
    }
    uint8_t key[46];
    for (int i = 0; i < 46; i++)
        key[i] = (uint8_t)(i * 29 + 3);
    const char *names[2] = { "icm128_sha1_80", "gcm256_16" };
    for (int pi = 0; pi < 2; pi++) {
        srtp_policy_t pol;
        memset(&pol, 0, sizeof pol);
        if (pi == 0) {
            srtp_crypto_policy_set_rtp_default(&pol.rtp);
            srtp_crypto_policy_set_rtcp_default(&pol.rtcp);
        } else {
            srtp_crypto_policy_set_aes_gcm_256_16_auth(&pol.rtp);
            srtp_crypto_policy_set_aes_gcm_256_16_auth(&pol.rtcp);
        }
        pol.key = key;
        pol.ssrc.type = ssrc_specific;
        pol.ssrc.value = 0x12345678;
        pol.window_size = 128;
        srtp_t snd, rcv;
        if (srtp_create(&snd, &pol) || srtp_create(&rcv, &pol))
            return 4;
        double tp = 0, tu = 0;
        for (int it = 0; it <= iters; it++) { /* iteration 0 warms up */
            for (size_t i = 0; i < n; i++)
                el[i] = cap, ol[i] = cap;
            double t0 = now();
            if (srtp_protect_rtcp_batch(snd, n, ip, il, eo, el, NULL, st))
                return 5;
            double t1 = now();
            for (size_t i = 0; i < n; i++)
                if (st[i])
                    return 6;
            if (srtp_unprotect_rtcp_batch(rcv, n, ep, el, oo, ol, st))
                return 7;
            double t2 = now();
            for (size_t i = 0; i < n; i++)
                if (st[i] || ol[i] != sz || memcmp(oo[i], ip[i], sz))
                    return 8;
            if (it) {
                tp += t1 - t0;
                tu += t2 - t1;
            }
        }
        printf("{\"tool\": \"rtcp_bench\", \"policy\": \"%s\", \"packets\": %zu, "
               "\"bytes\": %zu, \"iters\": %d, \"protect_pkt_per_s\": %.0f, "
               "\"unprotect_pkt_per_s\": %.0f, \"verified\": true}\n",
               names[pi], n, sz, iters, n * iters / tp, n * iters / tu);
        srtp_dealloc(snd);
        srtp_dealloc(rcv);
    }
    return 0;
}
