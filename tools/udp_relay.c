/*
 * udp_relay.c -- the socket-side batching caller: the
 * replacement for libsrtp's one-packet rtp_sendto / rtp_recvfrom loop
 * (test/rtp.c:61-149) in front of the batch API.
 *
 *   source --UDP--> relay: recvmmsg() into a packet arena until a batch is
 *                   full -> srtp_protect_batch() (one GPU pass) ->
 *                   sendmmsg() --UDP--> sink: recvmmsg() ->
 *                   srtp_unprotect_batch() -> byte-compare with the source
 *
 * All sockets are on 127.0.0.1 (no network).  The source and the relay move
 * packets in chunks of `chunk` datagrams so the kernel socket buffers never
 * overflow; a batch is many chunks.  Prints one JSON line with the relay's
 * rate (recv + protect + send, wall clock) and the number of packets that
 * came back bit-identical.
 *
 *   usage: udp_relay [packets] [payload] [batch] [chunk]
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <netinet/in.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "srtp_mi355x.h"

#define MAXPKT 2048

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static uint64_t rs = 0x55445052454c4159ull; /* "UDPRELAY" */
static uint64_t rnd(void)
{
    uint64_t z = (rs += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static int udp_bound(struct sockaddr_in *a)
{
    int fd = socket(AF_INET, SOCK_DGRAM, 0);
    if (fd < 0)
        return -1;
    memset(a, 0, sizeof *a);
    a->sin_family = AF_INET;
    a->sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    socklen_t l = sizeof *a;
    if (bind(fd, (struct sockaddr *)a, sizeof *a) ||
        getsockname(fd, (struct sockaddr *)a, &l))
        return -1;
    int sz = 8 << 20;
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof sz);
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof sz);
    return fd;
}

/* send n datagrams (pointers/lengths) to dst with sendmmsg */
static int send_n(int fd, const struct sockaddr_in *dst, uint8_t *const *p,
                  const size_t *len, size_t n)
{
    struct mmsghdr m[256];
    struct iovec v[256];
    size_t done = 0;
    while (done < n) {
        size_t k = n - done < 256 ? n - done : 256;
        for (size_t i = 0; i < k; i++) {
            v[i].iov_base = p[done + i];
            v[i].iov_len = len[done + i];
            memset(&m[i], 0, sizeof m[i]);
            m[i].msg_hdr.msg_name = (void *)dst;
            m[i].msg_hdr.msg_namelen = sizeof *dst;
            m[i].msg_hdr.msg_iov = &v[i];
            m[i].msg_hdr.msg_iovlen = 1;
        }
        int r = sendmmsg(fd, m, (unsigned)k, 0);
        if (r <= 0)
            return -1;
        done += (size_t)r;
    }
    return 0;
}

/* receive exactly n datagrams into p[i] (capacity MAXPKT) with recvmmsg */
static int recv_n(int fd, uint8_t *const *p, size_t *len, size_t n)
{
    struct mmsghdr m[256];
    struct iovec v[256];
    size_t done = 0;
    while (done < n) {
        size_t k = n - done < 256 ? n - done : 256;
        for (size_t i = 0; i < k; i++) {
            v[i].iov_base = p[done + i];
            v[i].iov_len = MAXPKT;
            memset(&m[i], 0, sizeof m[i]);
            m[i].msg_hdr.msg_iov = &v[i];
            m[i].msg_hdr.msg_iovlen = 1;
        }
        struct timespec to = { 5, 0 };
        int r = recvmmsg(fd, m, (unsigned)k, MSG_WAITFORONE, &to);
        if (r <= 0)
            return -1;
        for (int i = 0; i < r; i++)
            len[done + (size_t)i] = m[i].msg_len;
        done += (size_t)r;
    }
    return 0;
}

static uint8_t **arena(size_t n)
{
    uint8_t **p = (uint8_t **)malloc(n * sizeof *p);
    uint8_t *a = (uint8_t *)malloc(n * MAXPKT);
    if (!p || !a)
        exit(3);
    for (size_t i = 0; i < n; i++)
        p[i] = a + i * MAXPKT;
    return p;
}

int main(int argc, char **argv)
{
    size_t total = argc > 1 ? strtoull(argv[1], 0, 0) : 65536;
    size_t payload = argc > 2 ? strtoull(argv[2], 0, 0) : 1400;
    size_t batch = argc > 3 ? strtoull(argv[3], 0, 0) : 8192;
    size_t chunk = argc > 4 ? strtoull(argv[4], 0, 0) : 64;
    /* optional: a dump of the master key and of every (RTP sent, SRTP the
     * sink received) pair, for an independent check of the wire bytes
     * (tests/test_gpu_udp_relay.py compares them with the oracle) */
    FILE *dump = argc > 5 ? fopen(argv[5], "wb") : NULL;
    if (argc > 5 && !dump) {
        perror(argv[5]);
        return 2;
    }
    if (payload + 12 + 64 > MAXPKT || !batch || !chunk) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    if (srtp_init()) {
        fprintf(stderr, "srtp_init failed (no GPU?)\n");
        return 1;
    }
    uint8_t key[30];
    for (int i = 0; i < 30; i++)
        key[i] = (uint8_t)rnd();
    srtp_policy_t pol;
    memset(&pol, 0, sizeof pol);
    srtp_crypto_policy_set_rtp_default(&pol.rtp);
    srtp_crypto_policy_set_rtcp_default(&pol.rtcp);
    pol.key = key;
    pol.window_size = 1024;
    srtp_t snd, rcv;
    pol.ssrc.type = ssrc_any_outbound;
    if (srtp_create(&snd, &pol))
        return 1;
    pol.ssrc.type = ssrc_any_inbound;
    if (srtp_create(&rcv, &pol))
        return 1;
    if (dump)
        fwrite(key, 1, sizeof key, dump);

    struct sockaddr_in a_src, a_relay, a_sink;
    int f_src = udp_bound(&a_src), f_relay = udp_bound(&a_relay),
        f_sink = udp_bound(&a_sink);
    if (f_src < 0 || f_relay < 0 || f_sink < 0) {
        perror("socket");
        return 1;
    }
    uint8_t **plain = arena(batch), **rx = arena(batch), **enc = arena(batch),
            **back = arena(batch), **got = arena(batch);
    size_t *plen = malloc(batch * 8), *rxlen = malloc(batch * 8),
           *elen = malloc(batch * 8), *glen = malloc(batch * 8),
           *blen = malloc(batch * 8);
    srtp_err_status_t *st = malloc(batch * sizeof *st);
    if (!plen || !rxlen || !elen || !glen || !blen || !st)
        return 3;

    double t_relay = 0;
    size_t verified = 0, failed = 0;
    uint16_t seq = 0;
    for (size_t base = 0; base < total; base += batch) {
        size_t n = total - base < batch ? total - base : batch;
        for (size_t i = 0; i < n; i++) {
            uint8_t *p = plain[i];
            uint32_t ssrc = 0x51000000u + (uint32_t)((base + i) % 16);
            uint16_t s = (uint16_t)(seq + (base + i) / 16);
            p[0] = 0x80;
            p[1] = 96;
            p[2] = (uint8_t)(s >> 8);
            p[3] = (uint8_t)s;
            memset(p + 4, 0, 4);
            p[8] = (uint8_t)(ssrc >> 24);
            p[9] = (uint8_t)(ssrc >> 16);
            p[10] = (uint8_t)(ssrc >> 8);
            p[11] = (uint8_t)ssrc;
            for (size_t j = 0; j < payload; j++)
                p[12 + j] = (uint8_t)rnd();
            plen[i] = 12 + payload;
        }
        /* relay: receive the batch chunk by chunk as the source sends it */
        double t0 = now();
        double src_time = 0;
        for (size_t c = 0; c < n; c += chunk) {
            size_t k = n - c < chunk ? n - c : chunk;
            double s0 = now();
            if (send_n(f_src, &a_relay, plain + c, plen + c, k))
                return 4;
            src_time += now() - s0;
            if (recv_n(f_relay, rx + c, rxlen + c, k))
                return 5;
        }
        for (size_t i = 0; i < n; i++)
            elen[i] = MAXPKT;
        if (srtp_protect_batch(snd, n, (const uint8_t *const *)rx, rxlen, enc,
                               elen, NULL, st))
            return 6;
        /* sink: receive what the relay sends, chunk by chunk */
        double sink_time = 0;
        for (size_t c = 0; c < n; c += chunk) {
            size_t k = n - c < chunk ? n - c : chunk;
            for (size_t i = c; i < c + k; i++)
                if (st[i])
                    elen[i] = 0; /* never happens; keeps counts aligned */
            if (send_n(f_relay, &a_sink, enc + c, elen + c, k))
                return 7;
            double s0 = now();
            if (recv_n(f_sink, got + c, glen + c, k))
                return 8;
            sink_time += now() - s0;
        }
        t_relay += now() - t0 - src_time - sink_time;
        for (size_t i = 0; i < n; i++)
            blen[i] = MAXPKT;
        if (srtp_unprotect_batch(rcv, n, (const uint8_t *const *)got, glen,
                                 back, blen, st))
            return 9;
        for (size_t i = 0; dump && i < n; i++) {
            const uint16_t a = (uint16_t)plen[i], b = (uint16_t)glen[i];
            fwrite(&a, 2, 1, dump);
            fwrite(plain[i], 1, a, dump);
            fwrite(&b, 2, 1, dump);
            fwrite(got[i], 1, b, dump);
        }
        for (size_t i = 0; i < n; i++) {
            if (st[i] == 0 && blen[i] == plen[i] &&
                memcmp(back[i], plain[i], plen[i]) == 0)
                verified++;
            else
                failed++;
        }
    }
    printf("{\"tool\": \"udp_relay\", \"packets\": %zu, \"payload\": %zu, "
           "\"batch\": %zu, \"chunk\": %zu, \"relay_pkt_per_s\": %.1f, "
           "\"relay_s\": %.4f, \"verified\": %zu, \"failed\": %zu}\n",
           total, payload, batch, chunk, t_relay > 0 ? total / t_relay : 0.0,
           t_relay, verified, failed);
    if (dump)
        fclose(dump);
    srtp_dealloc(snd);
    srtp_dealloc(rcv);
    close(f_src);
    close(f_relay);
    close(f_sink);
    return failed ? 10 : 0;
}
