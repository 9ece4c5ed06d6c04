/*
 * bench_ref.c -- CPU baseline driver (test infrastructure): times the
 * REFERENCE (oracle/_ref/libsrtp_ref_*.so, cisco/libsrtp built from its own
 * sources) calling srtp_protect() once per packet, T threads with one
 * srtp_t each, like BASELINE.md's probe.  Each thread cycles over a pool of
 * distinct packet buffers, protecting in place with seq += 1.
 *
 * int ref_bench(int threads, long pkts_per_thread, int payload,
 *               int gcm, double *seconds)  -> packets protected
 *
 * Receive side: ref_bench_unprotect() -- each thread protects its pool
 * (untimed) with a sender srtp_t, then srtp_unprotect()s it in place on a
 * receiver srtp_t (timed), pool after pool; *seconds is the slowest
 * thread's unprotect time.
 *
 * Many streams (BASELINE configs[3]): ref_bench_streams() -- each thread's
 * srtp_t holds nstreams specific-SSRC streams with distinct master keys
 * (srtp_create over a policy list; untimed) and protects packets
 * round-robin over them, so every srtp_protect() goes through the
 * reference's stream-list lookup (srtp/srtp.c:5292-5305, a linear scan).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "srtp.h"

typedef struct {
    long n;
    int payload, gcm, pool, unprotect;
    long done;
    double secs; /* unprotect: time spent in srtp_unprotect */
} job_t;

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static const uint8_t key46[46] = {
    0xe1, 0xf9, 0x7a, 0x0d, 0x3e, 0x01, 0x8b, 0xe0, 0xd6, 0x4f, 0xa3, 0x2c,
    0x06, 0xde, 0x41, 0x39, 0x0e, 0xc6, 0x75, 0xad, 0x49, 0x8a, 0xfe, 0xeb,
    0xb6, 0x96, 0x0b, 0x3a, 0xab, 0xe6, 0xc1, 0x73, 0xc3, 0x17, 0xf2, 0xda,
    0xbe, 0x35, 0x77, 0x93, 0xb6, 0x96, 0x0b, 0x3a, 0xab, 0xe6 };

static void *run(void *arg)
{
    job_t *j = (job_t *)arg;
    srtp_policy_t p;
    srtp_t s;
    memset(&p, 0, sizeof p);
    if (j->gcm) {
        srtp_crypto_policy_set_aes_gcm_256_16_auth(&p.rtp);
        srtp_crypto_policy_set_aes_gcm_256_16_auth(&p.rtcp);
    } else {
        srtp_crypto_policy_set_rtp_default(&p.rtp);
        srtp_crypto_policy_set_rtcp_default(&p.rtcp);
    }
    p.ssrc.type = ssrc_any_outbound;
    p.key = (uint8_t *)key46;
    p.window_size = 128;
    if (srtp_create(&s, &p))
        return NULL;
    srtp_t r = NULL;
    if (j->unprotect) {
        p.ssrc.type = ssrc_any_inbound;
        if (srtp_create(&r, &p))
            return NULL;
    }
    size_t slot = (size_t)(12 + j->payload + 64 + 63) & ~(size_t)63;
    uint8_t *buf = (uint8_t *)aligned_alloc(64, slot * (size_t)j->pool);
    uint64_t x = 0x5352545030303031ULL ^ (uint64_t)(uintptr_t)j;
    for (size_t i = 0; i < slot * (size_t)j->pool; i++) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        buf[i] = (uint8_t)x;
    }
    uint16_t seq = 0x1234;
    size_t *plen = (size_t *)malloc(sizeof(size_t) * (size_t)j->pool);
    for (long i = 0; i < j->n;) {
        long m = j->unprotect ? j->pool : 1;
        if (m > j->n - i)
            m = j->n - i;
        for (long q = 0; q < m; q++) {
            uint8_t *pk = buf + slot * (size_t)((i + q) % j->pool);
            pk[0] = 0x80;
            pk[1] = 96;
            pk[2] = (uint8_t)(seq >> 8);
            pk[3] = (uint8_t)seq;
            pk[8] = 0xca; pk[9] = 0xfe; pk[10] = 0xba; pk[11] = 0xbe;
            size_t len = slot;
            plen[q] = 0;
            if (srtp_protect(s, pk, 12 + (size_t)j->payload, pk, &len, 0) == 0) {
                if (!j->unprotect)
                    j->done++;
                plen[q] = len;
            }
            seq++;
        }
        if (j->unprotect) {
            double t0 = now();
            for (long q = 0; q < m; q++) {
                uint8_t *pk = buf + slot * (size_t)((i + q) % j->pool);
                size_t len = slot;
                if (plen[q] && srtp_unprotect(r, pk, plen[q], pk, &len) == 0)
                    j->done++;
            }
            j->secs += now() - t0;
        }
        i += m;
    }
    free(plen);
    free(buf);
    srtp_dealloc(s);
    if (r)
        srtp_dealloc(r);
    return NULL;
}

/* srtp_init() once per process, whichever driver runs first */
static int ref_init(void)
{
    static int inited;
    if (!inited) {
        if (srtp_init())
            return -1;
        inited = 1;
    }
    return 0;
}

static int bench(int threads, long pkts_per_thread, int payload, int gcm,
                 int unprotect, double *seconds)
{
    if (ref_init())
        return -1;
    pthread_t th[256];
    job_t jobs[256];
    if (threads > 256)
        threads = 256;
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int t = 0; t < threads; t++) {
        jobs[t].n = pkts_per_thread;
        jobs[t].payload = payload;
        jobs[t].gcm = gcm;
        jobs[t].pool = 4096;
        jobs[t].unprotect = unprotect;
        jobs[t].done = 0;
        jobs[t].secs = 0;
        pthread_create(&th[t], NULL, run, &jobs[t]);
    }
    long done = 0;
    double slowest = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        done += jobs[t].done;
        if (jobs[t].secs > slowest)
            slowest = jobs[t].secs;
    }
    clock_gettime(CLOCK_MONOTONIC, &b);
    *seconds = unprotect ? slowest
                         : (double)(b.tv_sec - a.tv_sec) +
                               1e-9 * (double)(b.tv_nsec - a.tv_nsec);
    return (int)done;
}

typedef struct {
    long n;
    int payload, nstreams;
    int rx;      /* run_template: time a receiver's template path instead */
    int gcm;     /* run_template: AES-256-GCM-16 instead of the default */
    long done;
    double secs; /* protect (or unprotect) time, setup excluded */
} sjob_t;

static void *run_streams(void *arg)
{
    sjob_t *j = (sjob_t *)arg;
    const int ns = j->nstreams;
    srtp_policy_t *p = (srtp_policy_t *)calloc((size_t)ns, sizeof *p);
    uint8_t *keys = (uint8_t *)malloc((size_t)ns * 46);
    uint64_t x = 0x5352545030303031ULL ^ (uint64_t)(uintptr_t)j;
    for (size_t i = 0; i < (size_t)ns * 46; i++) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        keys[i] = (uint8_t)x;
    }
    for (int k = 0; k < ns; k++) {
        srtp_crypto_policy_set_rtp_default(&p[k].rtp);
        srtp_crypto_policy_set_rtcp_default(&p[k].rtcp);
        p[k].ssrc.type = ssrc_specific;
        p[k].ssrc.value = 0x10000000u + (uint32_t)k;
        p[k].key = keys + 46 * (size_t)k;
        p[k].window_size = 128;
        p[k].next = k + 1 < ns ? &p[k + 1] : NULL;
    }
    srtp_t s;
    if (srtp_create(&s, p)) {
        free(keys);
        free(p);
        return NULL;
    }
    const size_t slot = (size_t)(12 + j->payload + 64 + 63) & ~(size_t)63;
    const int pool = 4096;
    uint8_t *buf = (uint8_t *)aligned_alloc(64, slot * (size_t)pool);
    for (size_t i = 0; i < slot * (size_t)pool; i++) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        buf[i] = (uint8_t)x;
    }
    const double t0 = now();
    for (long i = 0; i < j->n; i++) {
        uint8_t *pk = buf + slot * (size_t)(i % pool);
        const uint32_t ssrc = 0x10000000u + (uint32_t)(i % ns);
        const uint16_t seq = (uint16_t)(0x1234 + i / ns);
        pk[0] = 0x80;
        pk[1] = 96;
        pk[2] = (uint8_t)(seq >> 8);
        pk[3] = (uint8_t)seq;
        pk[8] = (uint8_t)(ssrc >> 24);
        pk[9] = (uint8_t)(ssrc >> 16);
        pk[10] = (uint8_t)(ssrc >> 8);
        pk[11] = (uint8_t)ssrc;
        size_t len = slot;
        if (srtp_protect(s, pk, 12 + (size_t)j->payload, pk, &len, 0) == 0)
            j->done++;
    }
    j->secs = now() - t0;
    free(buf);
    srtp_dealloc(s);
    free(keys);
    free(p);
    return NULL;
}

/* configs[3]'s template variant: ONE ssrc_any_outbound policy per srtp_t;
 * packets round-robin over nstreams SSRCs, so the first pass creates every
 * stream by srtp_stream_clone (srtp.c:2540-2559, 762-863) and every later
 * srtp_protect() scans the cloned list (srtp.c:5292-5305).  With j->rx the
 * receiver's side is timed instead: a sender (untimed, its own template)
 * protects each pool of packets, then ONE ssrc_any_inbound srtp_t
 * unprotects them (timed): its first pass clones a stream per SSRC once the
 * packet authenticates (srtp.c:3117-3155) */
static void *run_template(void *arg)
{
    sjob_t *j = (sjob_t *)arg;
    const int ns = j->nstreams;
    srtp_policy_t p;
    memset(&p, 0, sizeof p);
    if (j->gcm) {
        srtp_crypto_policy_set_aes_gcm_256_16_auth(&p.rtp);
        srtp_crypto_policy_set_aes_gcm_256_16_auth(&p.rtcp);
    } else {
        srtp_crypto_policy_set_rtp_default(&p.rtp);
        srtp_crypto_policy_set_rtcp_default(&p.rtcp);
    }
    p.ssrc.type = ssrc_any_outbound;
    p.key = (uint8_t *)key46;
    p.window_size = 128;
    srtp_t s, r = NULL;
    if (srtp_create(&s, &p))
        return NULL;
    if (j->rx) {
        p.ssrc.type = ssrc_any_inbound;
        if (srtp_create(&r, &p)) {
            srtp_dealloc(s);
            return NULL;
        }
    }
    const size_t slot = (size_t)(12 + j->payload + 64 + 63) & ~(size_t)63;
    const int pool = 4096;
    uint8_t *buf = (uint8_t *)aligned_alloc(64, slot * (size_t)pool);
    size_t *plen = (size_t *)malloc(sizeof(size_t) * (size_t)pool);
    uint64_t x = 0x5352545030303031ULL ^ (uint64_t)(uintptr_t)j;
    for (size_t i = 0; i < slot * (size_t)pool; i++) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        buf[i] = (uint8_t)x;
    }
    for (long i0 = 0; i0 < j->n; i0 += pool) {
        const long m = j->n - i0 < pool ? j->n - i0 : pool;
        const double t0 = now();
        for (long q = 0; q < m; q++) {
            const long i = i0 + q;
            uint8_t *pk = buf + slot * (size_t)q;
            const uint32_t ssrc = 0x10000000u + (uint32_t)(i % ns);
            const uint16_t seq = (uint16_t)(0x1234 + i / ns);
            pk[0] = 0x80;
            pk[1] = 96;
            pk[2] = (uint8_t)(seq >> 8);
            pk[3] = (uint8_t)seq;
            pk[8] = (uint8_t)(ssrc >> 24);
            pk[9] = (uint8_t)(ssrc >> 16);
            pk[10] = (uint8_t)(ssrc >> 8);
            pk[11] = (uint8_t)ssrc;
            size_t len = slot;
            plen[q] = 0;
            if (srtp_protect(s, pk, 12 + (size_t)j->payload, pk, &len, 0) == 0) {
                plen[q] = len;
                if (!r)
                    j->done++;
            }
        }
        if (!r) {
            j->secs += now() - t0;
            continue;
        }
        const double t1 = now();
        for (long q = 0; q < m; q++) {
            uint8_t *pk = buf + slot * (size_t)q;
            size_t len = slot;
            if (plen[q] && srtp_unprotect(r, pk, plen[q], pk, &len) == 0)
                j->done++;
        }
        j->secs += now() - t1;
    }
    free(plen);
    free(buf);
    srtp_dealloc(s);
    if (r)
        srtp_dealloc(r);
    return NULL;
}

static int bench_sjobs(void *(*fn)(void *), int threads, long pkts_per_thread,
                       int payload, int nstreams, int rx, double *seconds);

int ref_bench_template(int threads, long pkts_per_thread, int payload,
                       int nstreams, double *seconds)
{
    return bench_sjobs(run_template, threads, pkts_per_thread, payload,
                       nstreams, 0, seconds);
}

int ref_bench_template_unprotect(int threads, long pkts_per_thread,
                                 int payload, int nstreams, double *seconds)
{
    return bench_sjobs(run_template, threads, pkts_per_thread, payload,
                       nstreams, 1, seconds);
}

/* either direction (rx), either policy (gcm: AES-256-GCM-16) */
int ref_bench_template_policy(int threads, long pkts_per_thread, int payload,
                              int nstreams, int rx, int gcm, double *seconds)
{
    return bench_sjobs(run_template, threads, pkts_per_thread, payload,
                       nstreams, (rx ? 1 : 0) | (gcm ? 2 : 0), seconds);
}

int ref_bench_streams(int threads, long pkts_per_thread, int payload,
                      int nstreams, double *seconds)
{
    return bench_sjobs(run_streams, threads, pkts_per_thread, payload,
                       nstreams, 0, seconds);
}

static int bench_sjobs(void *(*fn)(void *), int threads, long pkts_per_thread,
                       int payload, int nstreams, int rx, double *seconds)
{
    *seconds = 0;
    if (ref_init())
        return -1;
    pthread_t th[256];
    sjob_t jobs[256];
    if (threads > 256)
        threads = 256;
    for (int t = 0; t < threads; t++) {
        memset(&jobs[t], 0, sizeof jobs[t]);
        jobs[t].n = pkts_per_thread;
        jobs[t].payload = payload;
        jobs[t].nstreams = nstreams;
        jobs[t].rx = rx & 1;
        jobs[t].gcm = rx >> 1 & 1;
        pthread_create(&th[t], NULL, fn, &jobs[t]);
    }
    long done = 0;
    double slowest = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        done += jobs[t].done;
        if (jobs[t].secs > slowest)
            slowest = jobs[t].secs;
    }
    *seconds = slowest;
    return (int)done;
}

int ref_bench(int threads, long pkts_per_thread, int payload, int gcm,
              double *seconds)
{
    return bench(threads, pkts_per_thread, payload, gcm, 0, seconds);
}

int ref_bench_unprotect(int threads, long pkts_per_thread, int payload,
                        int gcm, double *seconds)
{
    return bench(threads, pkts_per_thread, payload, gcm, 1, seconds);
}
