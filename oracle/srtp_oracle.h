/*
 * srtp_oracle.h -- CPU restatement of the libsrtp RTP protect/unprotect path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under libsrtp_amd/ includes, links or
 * loads this code; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, as the checker.  Parity of this restatement is
 * pinned against (a) the reference built from its own sources into
 * oracle/_ref/ (see Makefile.ref) and (b) the committed fixtures in
 * tests/golden/ generated from that build (oracle/gen_golden.c).
 *
 * Every function cites the reference file:line whose behaviour it restates
 * (paths relative to the cisco/libsrtp tree, libsrtp3 3.0.0).
 */
#ifndef SRTP_ORACLE_H
#define SRTP_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- primitives -------------------------------------------------------- */

/* AES key schedule + single block (FIPS-197); crypto/cipher/aes.c:1404-1515,
 * srtp_aes_encrypt aes.c:2102-2130.  key_len in {16, 24, 32}. */
int orc_aes_encrypt(const uint8_t *key, size_t key_len, const uint8_t in[16],
                    uint8_t out[16]);

/* SHA-1 (FIPS 180); crypto/hash/sha1.c:91-463. */
void orc_sha1(const uint8_t *msg, size_t len, uint8_t out[20]);

/* HMAC-SHA1 with key <= 20 bytes; crypto/hash/hmac.c:115-229. */
int orc_hmac_sha1(const uint8_t *key, size_t key_len, const uint8_t *msg,
                  size_t len, uint8_t out[20]);

/* AES-ICM keystream XOR exactly as srtp_aes_icm_set_iv/encrypt
 * (crypto/cipher/aes_icm.c:236-414): counter = (salt14 || 00 00) ^ iv16,
 * 16-bit block counter in bytes 14..15. key_len = 16/24/32 AES key bytes. */
int orc_icm_xor(const uint8_t *key, size_t key_len, const uint8_t salt14[14],
                const uint8_t iv16[16], const uint8_t *in, size_t len,
                uint8_t *out);

/* AES-GCM seal/open with 12-byte IV (NIST SP 800-38D), as driven by
 * crypto/cipher/aes_gcm_ossl.c:214-389.  tag_len in {8, 16}. open returns 0
 * on success, 7 (auth_fail) on tag mismatch. */
int orc_gcm_seal(const uint8_t *key, size_t key_len, const uint8_t iv[12],
                 const uint8_t *aad, size_t aad_len, const uint8_t *pt,
                 size_t len, uint8_t *ct, uint8_t *tag, size_t tag_len);
int orc_gcm_open(const uint8_t *key, size_t key_len, const uint8_t iv[12],
                 const uint8_t *aad, size_t aad_len, const uint8_t *ct,
                 size_t len, const uint8_t *tag, size_t tag_len, uint8_t *pt);

/* ---- SRTP session model (RTP only) ------------------------------------- */

/* cipher / auth ids as crypto/include/crypto_types.h:55-114 */
enum {
    ORC_NULL_CIPHER = 0,
    ORC_AES_ICM_128 = 1,
    ORC_AES_ICM_192 = 4,
    ORC_AES_ICM_256 = 5,
    ORC_AES_GCM_128 = 6,
    ORC_AES_GCM_256 = 7,
    ORC_NULL_AUTH = 0,
    ORC_HMAC_SHA1 = 3
};

/* One stream policy; mirrors the fields of srtp_policy_t (include/srtp.h
 * :330-358) that the RTP path reads.  ssrc_type: 1 specific, 2 any inbound,
 * 3 any outbound. */
typedef struct {
    int ssrc_type;
    uint32_t ssrc;
    uint32_t cipher_type;
    size_t cipher_key_len;
    uint32_t auth_type;
    size_t auth_key_len;
    size_t auth_tag_len;
    int sec_serv; /* 1 conf, 2 auth, 3 both */
    size_t num_master_keys;
    const uint8_t *keys[16];
    const uint8_t *mki_ids[16];
    int use_mki;
    size_t mki_size;
    size_t window_size;
    int allow_repeat_tx;
} orc_policy_t;

typedef struct orc_session orc_session_t;

int orc_session_create(orc_session_t **s);
int orc_session_add(orc_session_t *s, const orc_policy_t *p);
void orc_session_free(orc_session_t *s);
int orc_protect(orc_session_t *s, const uint8_t *rtp, size_t rtp_len,
                uint8_t *srtp, size_t *srtp_len, size_t mki_index);
int orc_unprotect(orc_session_t *s, const uint8_t *srtp, size_t srtp_len,
                  uint8_t *rtp, size_t *rtp_len);
int orc_get_roc(orc_session_t *s, uint32_t ssrc, uint32_t *roc);
int orc_set_roc(orc_session_t *s, uint32_t ssrc, uint32_t roc);
int orc_key_left(orc_session_t *s, uint32_t ssrc, size_t j, uint64_t *left);

/* Derived session keys for a master key (KDF, srtp/srtp.c:1070-1142,
 * 1233-1607): enc key, salt (14 or 12 bytes), auth key (20). */
int orc_derive(uint32_t cipher_type, size_t cipher_key_len,
               const uint8_t *master, uint8_t *enc_key, uint8_t *salt,
               uint8_t *auth_key, size_t auth_key_len);

/* Batch driver for the CPU baseline: protect n packets laid out at in_off[i]
 * (len in_len[i]) into out at out_off[i]; returns number of failures. */
size_t orc_protect_many(orc_session_t *s, size_t n, const uint8_t *in,
                        const uint64_t *in_off, const uint32_t *in_len,
                        uint8_t *out, const uint64_t *out_off,
                        uint32_t *out_len, uint32_t out_cap);
void orc_unprotect_many(orc_session_t *s, size_t n, const uint8_t *in,
                        const uint64_t *in_off, const uint32_t *in_len,
                        uint8_t *out, const uint64_t *out_off,
                        uint32_t *out_len, uint32_t out_cap, int32_t *status);

#ifdef __cplusplus
}
#endif
#endif
