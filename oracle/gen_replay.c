/*
 * gen_replay.c -- emits tests/golden/ref_replay.json: replay-window and
 * index-estimation runs of the REFERENCE (cisco/libsrtp built from
 * /root/reference sources into oracle/_ref/ by Makefile.ref), driven by the
 * reference's own unreliable-connection simulator test/ut_sim.c (compiled
 * from its source where it lies; see Makefile.golden), as its
 * test/rdbx_driver.c (test_replay_dbx: sequential, ut_sim non-sequential,
 * large-gap insertion) and test/roc_driver.c do -- but at the packet level,
 * through srtp_protect / srtp_unprotect, so the same rows can be replayed
 * through every entry point of the GPU library (host pre-pass, batches,
 * device pre-pass).
 *
 * Windows 64, 128, 1024 and 32767 (the range srtp.c:1670-1678 accepts).
 * Per window, three runs:
 *   "rx_ut"   sender protects in order; receiver gets ut_sim order plus
 *             re-deliveries at chosen distances behind the newest packet;
 *   "rx_gaps" sender indices advance by 1 << (rand % 12) (rdbx_driver.c's
 *             large-gap insertion, crossing many ROC values); receiver gets
 *             them in order plus re-deliveries;
 *   "tx_ut"   the SENDER protects in ut_sim order (its own replay check and
 *             index estimate under reordering); receiver gets its output.
 * Packet j of a run: index idx_j (48-bit), seq = idx_j & 0xffff, ts = j,
 * SSRC 0x5eed0001, 4-byte payload = BE32(idx_j * 2654435761).  Sequences
 * start at seq 64836 so every run crosses ROC 0 -> 1.
 *
 * Test infrastructure: build container only; output committed as data.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

#include "srtp.h"
#include "ut_sim.h"

#define NPKT 2000
#define BASE 64836u

static FILE *g_out;

static uint64_t fnv(uint64_t h, const uint8_t *p, size_t n)
{
    for (size_t i = 0; i < n; i++)
        h = (h ^ p[i]) * 0x100000001b3ULL;
    return h;
}

static size_t build(uint8_t *pkt, uint64_t idx, uint32_t ts)
{
    const uint32_t pay = (uint32_t)(idx * 2654435761u);
    const uint16_t seq = (uint16_t)idx;
    const uint8_t h[16] = { 0x80,
                            0x60,
                            (uint8_t)(seq >> 8),
                            (uint8_t)seq,
                            (uint8_t)(ts >> 24),
                            (uint8_t)(ts >> 16),
                            (uint8_t)(ts >> 8),
                            (uint8_t)ts,
                            0x5e,
                            0xed,
                            0x00,
                            0x01,
                            (uint8_t)(pay >> 24),
                            (uint8_t)(pay >> 16),
                            (uint8_t)(pay >> 8),
                            (uint8_t)pay };
    memcpy(pkt, h, 16);
    return 16;
}

static void ints(const char *key, const int64_t *v, size_t n)
{
    fprintf(g_out, ", \"%s\": [", key);
    for (size_t i = 0; i < n; i++)
        fprintf(g_out, "%s%lld", i ? "," : "", (long long)v[i]);
    fputc(']', g_out);
}

/* re-delivery distances behind the newest delivered index, cycled */
static int64_t redeliver_delta(size_t k, size_t w)
{
    const int64_t d[8] = { 0, 1, 17, (int64_t)w - 1, (int64_t)w,
                           (int64_t)w + 1, 100, 3 };
    return d[k % 8];
}

static void run(size_t w, const char *pattern, int first)
{
    static int64_t tx_idx[NPKT + 200], tx_st[NPKT + 200];
    static int64_t rx_src[2 * NPKT], rx_st[2 * NPKT];
    static uint8_t tx_out[NPKT + 200][64];
    static size_t tx_len[NPKT + 200];
    uint8_t key[30];
    srand(1);
    for (int i = 0; i < 30; i++)
        key[i] = (uint8_t)(rand() >> 3);

    srtp_policy_t pol;
    memset(&pol, 0, sizeof pol);
    srtp_crypto_policy_set_rtp_default(&pol.rtp);
    srtp_crypto_policy_set_rtp_default(&pol.rtcp);
    pol.ssrc.type = ssrc_specific;
    pol.ssrc.value = 0x5eed0001;
    pol.key = key;
    pol.window_size = w;
    srtp_t snd, rcv;
    if (srtp_create(&snd, &pol) || srtp_create(&rcv, &pol)) {
        fprintf(stderr, "srtp_create failed (window %zu)\n", w);
        exit(1);
    }

    const int gaps = !strcmp(pattern, "rx_gaps");
    const int tx_reorder = !strcmp(pattern, "tx_ut");
    const size_t ntx = gaps ? NPKT : NPKT + 160;
    ut_connection utc;
    ut_init(&utc);
    /* sender */
    uint64_t idx = BASE;
    for (size_t j = 0; j < ntx; j++) {
        if (tx_reorder)
            tx_idx[j] = BASE + ut_next_index(&utc);
        else {
            tx_idx[j] = (int64_t)idx;
            idx += gaps ? (1u << (rand() % 12)) : 1u;
        }
        uint8_t pkt[64];
        size_t len = build(pkt, (uint64_t)tx_idx[j], (uint32_t)j);
        tx_len[j] = sizeof tx_out[j];
        tx_st[j] = srtp_protect(snd, pkt, len, tx_out[j], &tx_len[j], 0);
        if (tx_st[j])
            tx_len[j] = 0;
    }
    /* receiver: delivery order (positions into the sender's outputs) */
    size_t nrx = 0, nre = 0;
    int64_t newest = -1;
    if (!strcmp(pattern, "rx_ut"))
        ut_init(&utc);
    for (size_t k = 0; k < NPKT; k++) {
        size_t src = !strcmp(pattern, "rx_ut") ? ut_next_index(&utc) : k;
        rx_src[nrx++] = (int64_t)src;
        if ((int64_t)src > newest)
            newest = (int64_t)src;
        if (k % 37 == 36) {
            int64_t back = newest - redeliver_delta(nre++, w);
            if (back >= 0)
                rx_src[nrx++] = back;
        }
    }
    uint64_t rx_h = 0xcbf29ce484222325ULL, tx_h = 0xcbf29ce484222325ULL;
    for (size_t j = 0; j < ntx; j++)
        tx_h = fnv(tx_h, tx_out[j], tx_len[j]);
    for (size_t k = 0; k < nrx; k++) {
        size_t s = (size_t)rx_src[k];
        uint8_t pt[64];
        size_t plen = sizeof pt;
        if (!tx_len[s]) {
            rx_st[k] = -1; /* nothing was sent */
            continue;
        }
        rx_st[k] = srtp_unprotect(rcv, tx_out[s], tx_len[s], pt, &plen);
        if (rx_st[k] == 0)
            rx_h = fnv(rx_h, pt, plen);
    }
    uint32_t roc_tx = 0, roc_rx = 0;
    srtp_stream_get_roc(snd, 0x5eed0001, &roc_tx);
    srtp_stream_get_roc(rcv, 0x5eed0001, &roc_rx);

    fprintf(g_out, "%s    {\"window\": %zu, \"pattern\": \"%s\", \"key\": \"",
            first ? "" : ",\n", w, pattern);
    for (int i = 0; i < 30; i++)
        fprintf(g_out, "%02x", key[i]);
    fputc('"', g_out);
    ints("tx_idx", tx_idx, ntx);
    ints("tx_status", tx_st, ntx);
    fprintf(g_out, ", \"tx_fnv\": \"%016llx\"", (unsigned long long)tx_h);
    ints("rx_src", rx_src, nrx);
    ints("rx_status", rx_st, nrx);
    fprintf(g_out, ", \"rx_fnv\": \"%016llx\", \"roc_tx\": %u, "
                   "\"roc_rx\": %u}",
            (unsigned long long)rx_h, roc_tx, roc_rx);
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
    fputs("{\n  \"npkt\": 2000, \"base\": 64836, \"ssrc\": 1592590337,\n"
          "  \"runs\": [\n",
          g_out);
    static const size_t windows[] = { 64, 128, 1024, 32767 };
    static const char *patterns[] = { "rx_ut", "rx_gaps", "tx_ut" };
    int first = 1;
    for (int wi = 0; wi < 4; wi++)
        for (int pi = 0; pi < 3; pi++) {
            run(windows[wi], patterns[pi], first);
            first = 0;
        }
    fputs("\n  ]\n}\n", g_out);
    fclose(g_out);
    srtp_shutdown();
    return 0;
}
