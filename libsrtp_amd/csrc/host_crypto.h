/*
 * host_crypto.h -- session-setup crypto on the host (never per packet):
 * AES key schedules and the few AES blocks the SRTP KDF needs
 * (srtp/srtp.c:1070-1142), SHA-1 midstates for HMAC (hmac.c:115-155) and
 * the GHASH byte table of a GCM key.  All per-packet work is on the GPU.
 */
#ifndef HOST_CRYPTO_H
#define HOST_CRYPTO_H
#include <stddef.h>
#include <stdint.h>

typedef struct {
    int rounds;           /* 10 / 12 / 14 */
    uint32_t rk[60];      /* little-endian words of the round key bytes */
} hc_aes_t;

int hc_aes_init(hc_aes_t *a, const uint8_t *key, size_t key_len);
void hc_aes_block(const hc_aes_t *a, const uint8_t in[16], uint8_t out[16]);
/* AES-ICM keystream over zeros (the KDF PRF): counter = salt14||0 ^ iv16 */
void hc_icm_keystream(const hc_aes_t *a, const uint8_t salt14[14],
                      const uint8_t iv16[16], uint8_t *out, size_t len);
/* SHA-1 state after compressing one 64-byte block from the standard IV */
void hc_sha1_midstate(const uint8_t block[64], uint32_t h[5]);
/* GHASH byte table: tab[4*b .. 4*b+3] = b(x) * H, big-endian words */
void hc_ghash_table(const uint8_t h[16], uint32_t tab[1024]);
#endif
