/*
 * e2e_bench.c -- host-memory (PCIe-inclusive) rates of the protect and
 * unprotect paths, for DESIGN.md "End-to-end rate".  The packets start and
 * end in host memory, as they do behind a socket:
 *
 *   batch   srtp_protect_batch() / srtp_unprotect_batch() over per-packet
 *           host pointers (the libsrtp call shape: the library gathers into
 *           pinned memory, copies H2D, runs the device pre-pass and the
 *           kernels, copies D2H and scatters)
 *   pinned  the application keeps a pinned packet arena: hipMemcpyAsync H2D,
 *           srtp_{un}protect_device() (GPU pre-pass + kernels),
 *           hipMemcpyAsync D2H
 *   pipelined  the same arena in `chunks` pieces over three HIP streams:
 *           H2D(k+1) on a copy stream || {un}protect(k) on the compute
 *           stream || D2H(k-1) on a second copy stream (PCIe is full duplex)
 *
 * For unprotect every timed batch is first protected (untimed) by a sender
 * session on the device and copied to host memory.
 *
 *   usage: e2e_bench [packets] [payload] [iters] [chunks] [protect|unprotect]
 *   prints one JSON line.
 */
#include <hip/hip_runtime_api.h>
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

static uint64_t sm_state = 0x5352545030303031ull; /* splitmix64 "SRTP0001" */
static uint64_t splitmix64(void)
{
    uint64_t z = (sm_state += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

#define CHECK(x)                                                               \
    do {                                                                       \
        if ((x) != 0) {                                                        \
            fprintf(stderr, "%s:%d: %s failed\n", __FILE__, __LINE__, #x);     \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

static srtp_t make_session(uint8_t *key)
{
    srtp_policy_t p;
    memset(&p, 0, sizeof p);
    srtp_crypto_policy_set_rtp_default(&p.rtp);
    srtp_crypto_policy_set_rtp_default(&p.rtcp);
    p.ssrc.type = ssrc_specific;
    p.ssrc.value = 0xcafebabe;
    p.key = key;
    p.window_size = 128;
    srtp_t s;
    CHECK(srtp_create(&s, &p));
    return s;
}

static void fill(uint8_t *pk, size_t slot, size_t n, size_t len, uint32_t seq0)
{
    for (size_t i = 0; i < n; i++) {
        uint8_t *p = pk + i * slot;
        uint32_t seq = (seq0 + (uint32_t)i) & 0xffff;
        p[0] = 0x80;
        p[1] = 96;
        p[2] = (uint8_t)(seq >> 8);
        p[3] = (uint8_t)seq;
        memset(p + 4, 0, 4);
        p[8] = 0xca;
        p[9] = 0xfe;
        p[10] = 0xba;
        p[11] = 0xbe;
    }
    (void)len;
}

/* the sender side of the unprotect runs: n packets from seq0 protected on
 * the device by `snd` (untimed), then copied to h_dst */
typedef struct {
    srtp_t snd;
    uint8_t *d_arena;
    uint64_t *d_off;
    uint32_t *d_len, *d_cap;
    int32_t *d_st;
    hipStream_t st;
} sender_t;

static void produce(sender_t *S, uint8_t *h_dst, size_t n, size_t slot,
                    size_t len, uint32_t seq0, const uint32_t *h_cap)
{
    fill(h_dst, slot, n, len, seq0);
    CHECK(hipMemcpyAsync(S->d_arena, h_dst, n * slot, hipMemcpyHostToDevice,
                         S->st));
    CHECK(hipMemcpyAsync(S->d_cap, h_cap, n * 4, hipMemcpyHostToDevice, S->st));
    srtp_device_batch_t b;
    memset(&b, 0, sizeof b);
    b.n = n;
    b.in = S->d_arena;
    b.in_off = S->d_off;
    b.in_len = S->d_len;
    b.out = S->d_arena;
    b.out_off = S->d_off;
    b.out_len = S->d_cap;
    b.status = S->d_st;
    b.stream = S->st;
    CHECK(srtp_protect_device(S->snd, &b));
    CHECK(hipMemcpyAsync(h_dst, S->d_arena, n * slot, hipMemcpyDeviceToHost,
                         S->st));
    CHECK(hipStreamSynchronize(S->st));
}

int main(int argc, char **argv)
{
    size_t n = argc > 1 ? strtoul(argv[1], 0, 0) : (1u << 20);
    size_t payload = argc > 2 ? strtoul(argv[2], 0, 0) : 1400;
    int iters = argc > 3 ? atoi(argv[3]) : 5;
    size_t chunks = argc > 4 ? strtoul(argv[4], 0, 0) : 16;
    const int un = argc > 5 && strcmp(argv[5], "unprotect") == 0;
    size_t len = 12 + payload, slen = len + 10,
           slot = (slen + 15) & ~(size_t)15;
    /* what goes in and what comes out of the measured call */
    const size_t in_l = un ? slen : len, out_l = un ? len : slen;
    uint8_t key[30];
    for (int i = 0; i < 30; i++)
        key[i] = (uint8_t)splitmix64();
    CHECK(srtp_init());

    /* ---- pinned arena + device API ----------------------------------- */
    uint8_t *h_arena, *d_arena;
    uint64_t *h_off, *d_off;
    uint32_t *h_len, *h_cap, *d_len, *d_olen, *h_plen;
    int32_t *d_st;
    CHECK(hipHostMalloc((void **)&h_arena, n * slot, 0));
    CHECK(hipHostMalloc((void **)&h_off, n * 8, 0));
    CHECK(hipHostMalloc((void **)&h_len, n * 4, 0));
    CHECK(hipHostMalloc((void **)&h_plen, n * 4, 0));
    CHECK(hipHostMalloc((void **)&h_cap, n * 4, 0));
    CHECK(hipMalloc((void **)&d_arena, n * slot));
    CHECK(hipMalloc((void **)&d_off, n * 8));
    CHECK(hipMalloc((void **)&d_len, n * 4));
    CHECK(hipMalloc((void **)&d_olen, n * 4));
    CHECK(hipMalloc((void **)&d_st, n * 4));
    for (size_t i = 0; i < n * slot; i += 8) {
        uint64_t r = splitmix64();
        memcpy(h_arena + i, &r, n * slot - i < 8 ? n * slot - i : 8);
    }
    for (size_t i = 0; i < n; i++) {
        h_off[i] = i * slot;
        h_len[i] = (uint32_t)in_l;
        h_plen[i] = (uint32_t)len;
        h_cap[i] = (uint32_t)slot;
    }
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    CHECK(hipMemcpy(d_off, h_off, n * 8, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_len, h_len, n * 4, hipMemcpyHostToDevice));
    sender_t S;
    memset(&S, 0, sizeof S);
    if (un) {
        CHECK(hipMalloc((void **)&S.d_arena, n * slot));
        CHECK(hipMalloc((void **)&S.d_len, n * 4));
        CHECK(hipMalloc((void **)&S.d_cap, n * 4));
        CHECK(hipMalloc((void **)&S.d_st, n * 4));
        CHECK(hipMemcpy(S.d_len, h_plen, n * 4, hipMemcpyHostToDevice));
        S.d_off = d_off;
        S.st = st;
    }
    srtp_err_status_t (*dev_op)(srtp_t, const srtp_device_batch_t *) =
        un ? srtp_unprotect_device : srtp_protect_device;
    srtp_t s1 = make_session(key);
    if (un)
        S.snd = make_session(key);
    srtp_device_batch_t b;
    memset(&b, 0, sizeof b);
    b.n = n;
    b.in = d_arena;
    b.in_off = d_off;
    b.in_len = d_len;
    b.out = d_arena;
    b.out_off = d_off;
    b.out_len = d_olen;
    b.status = d_st;
    b.stream = st;
    uint32_t seq0 = 0x1234;
    double t_pinned = 0;
    for (int it = -1; it < iters; it++) {
        if (un)
            produce(&S, h_arena, n, slot, len, seq0, h_cap);
        else
            fill(h_arena, slot, n, len, seq0);
        seq0 += (uint32_t)n;
        double t0 = now();
        CHECK(hipMemcpyAsync(d_arena, h_arena, n * slot, hipMemcpyHostToDevice,
                             st));
        CHECK(hipMemcpyAsync(d_olen, h_cap, n * 4, hipMemcpyHostToDevice, st));
        CHECK(dev_op(s1, &b));
        CHECK(hipMemcpyAsync(h_arena, d_arena, n * slot, hipMemcpyDeviceToHost,
                             st));
        CHECK(hipStreamSynchronize(st));
        if (it >= 0)
            t_pinned += now() - t0;
    }
    t_pinned /= iters;
    /* verify lengths came back */
    CHECK(hipMemcpy(h_len, d_olen, n * 4, hipMemcpyDeviceToHost));
    if (h_len[0] != out_l) {
        fprintf(stderr, "unexpected out_len %u\n", h_len[0]);
        return 1;
    }
    uint64_t dev_b = 0, host_b = 0;
    srtp_mi355x_prepass_stats(s1, &dev_b, &host_b);

    /* ---- pipelined: chunks over three streams ------------------------- */
    if (chunks < 1 || n % chunks) {
        fprintf(stderr, "packets must be a multiple of chunks\n");
        return 2;
    }
    const size_t cn = n / chunks;
    hipStream_t s_h2d, s_d2h;
    CHECK(hipStreamCreateWithFlags(&s_h2d, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s_d2h, hipStreamNonBlocking));
    hipEvent_t *ev_in = (hipEvent_t *)malloc(chunks * sizeof(hipEvent_t));
    hipEvent_t *ev_done = (hipEvent_t *)malloc(chunks * sizeof(hipEvent_t));
    for (size_t k = 0; k < chunks; k++) {
        CHECK(hipEventCreateWithFlags(&ev_in[k], hipEventDisableTiming));
        CHECK(hipEventCreateWithFlags(&ev_done[k], hipEventDisableTiming));
    }
    srtp_t s3 = make_session(key);
    if (un) {
        srtp_dealloc(S.snd);
        S.snd = make_session(key);
    }
    seq0 = 0x1234;
    double t_pipe = 0;
    size_t pipe_bad = 0;
    for (int it = -1; it < iters; it++) {
        if (un)
            produce(&S, h_arena, n, slot, len, seq0, h_cap);
        else
            fill(h_arena, slot, n, len, seq0);
        seq0 += (uint32_t)n;
        double t0 = now();
        for (size_t k = 0; k <= chunks; k++) {
            if (k < chunks) {   /* stage chunk k in */
                CHECK(hipMemcpyAsync(d_arena + k * cn * slot,
                                     h_arena + k * cn * slot, cn * slot,
                                     hipMemcpyHostToDevice, s_h2d));
                CHECK(hipMemcpyAsync(d_olen + k * cn, h_cap + k * cn, cn * 4,
                                     hipMemcpyHostToDevice, s_h2d));
                CHECK(hipEventRecord(ev_in[k], s_h2d));
            }
            if (k == 0)
                continue;
            /* {un}protect chunk k-1 while chunk k is in flight */
            const size_t j = k - 1;
            CHECK(hipStreamWaitEvent(st, ev_in[j], 0));
            srtp_device_batch_t c = b;
            c.n = cn;
            c.in_off = d_off + j * cn;
            c.in_len = d_len + j * cn;
            c.out_off = d_off + j * cn;
            c.out_len = d_olen + j * cn;
            c.status = d_st + j * cn;
            CHECK(dev_op(s3, &c));
            CHECK(hipEventRecord(ev_done[j], st));
            CHECK(hipStreamWaitEvent(s_d2h, ev_done[j], 0));
            CHECK(hipMemcpyAsync(h_arena + j * cn * slot,
                                 d_arena + j * cn * slot, cn * slot,
                                 hipMemcpyDeviceToHost, s_d2h));
        }
        CHECK(hipStreamSynchronize(s_d2h));
        if (it >= 0)
            t_pipe += now() - t0;
    }
    t_pipe /= iters;
    CHECK(hipMemcpy(h_len, d_olen, n * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; i++)
        pipe_bad += h_len[i] != out_l;
    uint64_t dev_p = 0, host_p = 0;
    srtp_mi355x_prepass_stats(s3, &dev_p, &host_p);

    /* ---- libsrtp-shaped batch over host pointers --------------------- */
    srtp_t s2 = make_session(key);
    if (un) {
        srtp_dealloc(S.snd);
        S.snd = make_session(key);
    }
    uint8_t *pk = (uint8_t *)malloc(n * slot);
    const uint8_t **in = (const uint8_t **)malloc(n * sizeof(void *));
    uint8_t **out = (uint8_t **)malloc(n * sizeof(void *));
    size_t *il = (size_t *)malloc(n * sizeof(size_t));
    size_t *ol = (size_t *)malloc(n * sizeof(size_t));
    srtp_err_status_t *sts = (srtp_err_status_t *)malloc(n * sizeof(*sts));
    memcpy(pk, h_arena, n * slot);
    for (size_t i = 0; i < n; i++) {
        in[i] = pk + i * slot;
        out[i] = pk + i * slot;
        il[i] = in_l;
    }
    seq0 = 0x1234;
    double t_batch = 0;
    uint64_t dev_h0 = 0, host_h0 = 0, dev_h = 0, host_h = 0;
    for (int it = -1; it < iters; it++) {
        if (un) {
            produce(&S, h_arena, n, slot, len, seq0, h_cap);
            memcpy(pk, h_arena, n * slot);
        } else {
            fill(pk, slot, n, len, seq0);
        }
        seq0 += (uint32_t)n;
        for (size_t i = 0; i < n; i++)
            ol[i] = slot;
        if (it == 0)
            srtp_mi355x_prepass_stats(s2, &dev_h0, &host_h0);
        double t0 = now();
        if (un)
            CHECK(srtp_unprotect_batch(s2, n, in, il, out, ol, sts));
        else
            CHECK(srtp_protect_batch(s2, n, in, il, out, ol, NULL, sts));
        if (it >= 0)
            t_batch += now() - t0;
        if (sts[0] || ol[0] != out_l) {
            fprintf(stderr, "batch status %d len %zu\n", sts[0], ol[0]);
            return 1;
        }
    }
    t_batch /= iters;
    srtp_mi355x_prepass_stats(s2, &dev_h, &host_h);
    double bytes = (double)n * (2.0 * len + 10);
    printf("{\"op\": \"%s\", \"packets\": %zu, \"payload\": %zu, \"iters\": %d, "
           "\"pinned_device_api\": {\"pkt_per_s\": %.1f, \"ms\": %.3f, "
           "\"algorithmic_GBps\": %.2f, \"pcie_bytes\": %.0f, "
           "\"device_prepass_batches\": %llu, \"host_prepass_batches\": %llu}, "
           "\"pipelined_device_api\": {\"chunks\": %zu, \"pkt_per_s\": %.1f, "
           "\"ms\": %.3f, \"pcie_GBps_each_way\": %.2f, "
           "\"device_prepass_batches\": %llu, \"host_prepass_batches\": %llu, "
           "\"bad_lengths\": %zu}, "
           "\"host_batch_api\": {\"pkt_per_s\": %.1f, \"ms\": %.3f, "
           "\"algorithmic_GBps\": %.2f, \"device_prepass_batches\": %llu, "
           "\"host_prepass_batches\": %llu}}\n",
           un ? "unprotect" : "protect", n, payload, iters, n / t_pinned,
           t_pinned * 1e3, bytes / t_pinned / 1e9, 2.0 * n * slot + 8.0 * n,
           (unsigned long long)dev_b, (unsigned long long)host_b, chunks,
           n / t_pipe, t_pipe * 1e3, n * (double)slot / t_pipe / 1e9,
           (unsigned long long)dev_p, (unsigned long long)host_p, pipe_bad,
           n / t_batch, t_batch * 1e3, bytes / t_batch / 1e9,
           (unsigned long long)(dev_h - dev_h0),
           (unsigned long long)(host_h - host_h0));
    srtp_dealloc(s1);
    srtp_dealloc(s2);
    srtp_dealloc(s3);
    if (un)
        srtp_dealloc(S.snd);
    return pipe_bad ? 1 : 0;
}
