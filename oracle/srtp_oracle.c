/*
 * srtp_oracle.c -- plain-C restatement of the libsrtp RTP hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see srtp_oracle.h).  This is the checker the
 * HIP path is compared against; it is never linked into libsrtp_amd.  It is
 * written for clarity, not speed: byte-oriented AES straight from FIPS-197,
 * bit-serial GHASH straight from SP 800-38D, a textbook SHA-1.
 *
 * Parity pin: tests/test_oracle_golden.py checks every function here against
 * fixtures produced by the reference itself (oracle/gen_golden.c linked to
 * oracle/_ref/libsrtp_ref_{int,ossl}.so built from /root/reference sources).
 */
#include "srtp_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ======================================================================
 * AES (FIPS-197).  Restates crypto/cipher/aes.c: key expansion
 * (aes.c:1404-1515) and block encryption (srtp_aes_encrypt, 2102-2130).
 * The S-box is derived from the GF(2^8) inverse + affine map rather than
 * transcribed.
 * ====================================================================== */

static uint8_t g_sbox[256];
static int g_sbox_ready = 0;

static uint8_t gf_mul(uint8_t a, uint8_t b)
{
    uint8_t r = 0;
    while (b) {
        if (b & 1)
            r ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return r;
}

static void build_sbox(void)
{
    if (g_sbox_ready)
        return;
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        if (x) {
            for (int y = 1; y < 256; y++) {
                if (gf_mul((uint8_t)x, (uint8_t)y) == 1) {
                    inv = (uint8_t)y;
                    break;
                }
            }
        }
        uint8_t s = inv, r = inv;
        for (int i = 0; i < 4; i++) {
            r = (uint8_t)((r << 1) | (r >> 7));
            s ^= r;
        }
        g_sbox[x] = s ^ 0x63;
    }
    g_sbox_ready = 1;
}

typedef struct {
    int rounds;
    uint8_t rk[15][16];
} aes_ks_t;

static int aes_expand(aes_ks_t *ks, const uint8_t *key, size_t key_len)
{
    build_sbox();
    size_t nk = key_len / 4;
    if (key_len != 16 && key_len != 24 && key_len != 32)
        return 2;
    ks->rounds = (int)nk + 6;
    size_t total = 4 * (size_t)(ks->rounds + 1);
    uint8_t w[60][4];
    uint8_t rcon = 1;
    for (size_t i = 0; i < nk; i++)
        memcpy(w[i], key + 4 * i, 4);
    for (size_t i = nk; i < total; i++) {
        uint8_t t[4];
        memcpy(t, w[i - 1], 4);
        if (i % nk == 0) {
            uint8_t t0 = t[0];
            t[0] = (uint8_t)(g_sbox[t[1]] ^ rcon);
            t[1] = g_sbox[t[2]];
            t[2] = g_sbox[t[3]];
            t[3] = g_sbox[t0];
            rcon = gf_mul(rcon, 2);
        } else if (nk > 6 && i % nk == 4) {
            for (int j = 0; j < 4; j++)
                t[j] = g_sbox[t[j]];
        }
        for (int j = 0; j < 4; j++)
            w[i][j] = w[i - nk][j] ^ t[j];
    }
    for (int r = 0; r <= ks->rounds; r++)
        for (int c = 0; c < 4; c++)
            memcpy(&ks->rk[r][4 * c], w[4 * r + c], 4);
    return 0;
}

static void aes_block(const aes_ks_t *ks, const uint8_t in[16], uint8_t out[16])
{
    uint8_t s[16], t[16];
    for (int i = 0; i < 16; i++)
        s[i] = in[i] ^ ks->rk[0][i];
    for (int r = 1; r <= ks->rounds; r++) {
        /* SubBytes + ShiftRows: state byte (row i, col c) is s[4c+i] */
        for (int c = 0; c < 4; c++)
            for (int i = 0; i < 4; i++)
                t[4 * c + i] = g_sbox[s[4 * ((c + i) & 3) + i]];
        if (r != ks->rounds) {
            for (int c = 0; c < 4; c++) {
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2],
                        a3 = t[4 * c + 3];
                s[4 * c + 0] = gf_mul(a0, 2) ^ gf_mul(a1, 3) ^ a2 ^ a3;
                s[4 * c + 1] = a0 ^ gf_mul(a1, 2) ^ gf_mul(a2, 3) ^ a3;
                s[4 * c + 2] = a0 ^ a1 ^ gf_mul(a2, 2) ^ gf_mul(a3, 3);
                s[4 * c + 3] = gf_mul(a0, 3) ^ a1 ^ a2 ^ gf_mul(a3, 2);
            }
        } else {
            memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; i++)
            s[i] ^= ks->rk[r][i];
    }
    memcpy(out, s, 16);
}

int orc_aes_encrypt(const uint8_t *key, size_t key_len, const uint8_t in[16],
                    uint8_t out[16])
{
    aes_ks_t ks;
    int st = aes_expand(&ks, key, key_len);
    if (st)
        return st;
    aes_block(&ks, in, out);
    return 0;
}

/* ======================================================================
 * SHA-1 (crypto/hash/sha1.c:91-463).  The reference keeps a 32-bit bit
 * count (sha1.c:326-330); packets are far below 2^29 bytes so the 64-bit
 * length word's high half is always zero, as here.
 * ====================================================================== */

typedef struct {
    uint32_t h[5];
    uint8_t buf[64];
    size_t nbuf;
    uint64_t total;
} sha1_t;

#define ROL(x, n) (((x) << (n)) | ((x) >> (32 - (n))))

static void sha1_compress(uint32_t h[5], const uint8_t blk[64])
{
    uint32_t w[80];
    for (int t = 0; t < 16; t++)
        w[t] = (uint32_t)blk[4 * t] << 24 | (uint32_t)blk[4 * t + 1] << 16 |
               (uint32_t)blk[4 * t + 2] << 8 | blk[4 * t + 3];
    for (int t = 16; t < 80; t++)
        w[t] = ROL(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    for (int t = 0; t < 80; t++) {
        uint32_t f, k;
        if (t < 20) {
            f = (b & c) | (~b & d);
            k = 0x5a827999;
        } else if (t < 40) {
            f = b ^ c ^ d;
            k = 0x6ed9eba1;
        } else if (t < 60) {
            f = (b & c) | (b & d) | (c & d);
            k = 0x8f1bbcdc;
        } else {
            f = b ^ c ^ d;
            k = 0xca62c1d6;
        }
        uint32_t tmp = ROL(a, 5) + f + e + k + w[t];
        e = d;
        d = c;
        c = ROL(b, 30);
        b = a;
        a = tmp;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
}

static void sha1_init(sha1_t *s)
{
    s->h[0] = 0x67452301;
    s->h[1] = 0xefcdab89;
    s->h[2] = 0x98badcfe;
    s->h[3] = 0x10325476;
    s->h[4] = 0xc3d2e1f0;
    s->nbuf = 0;
    s->total = 0;
}

static void sha1_update(sha1_t *s, const uint8_t *m, size_t n)
{
    s->total += n;
    while (n) {
        size_t take = 64 - s->nbuf;
        if (take > n)
            take = n;
        memcpy(s->buf + s->nbuf, m, take);
        s->nbuf += take;
        m += take;
        n -= take;
        if (s->nbuf == 64) {
            sha1_compress(s->h, s->buf);
            s->nbuf = 0;
        }
    }
}

static void sha1_final(sha1_t *s, uint8_t out[20])
{
    uint64_t bits = s->total * 8;
    uint8_t pad = 0x80, z = 0, len[8];
    sha1_update(s, &pad, 1);
    while (s->nbuf != 56)
        sha1_update(s, &z, 1);
    for (int i = 0; i < 8; i++)
        len[i] = (uint8_t)(bits >> (56 - 8 * i));
    sha1_update(s, len, 8);
    for (int i = 0; i < 5; i++) {
        out[4 * i] = (uint8_t)(s->h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(s->h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(s->h[i] >> 8);
        out[4 * i + 3] = (uint8_t)s->h[i];
    }
}

void orc_sha1(const uint8_t *msg, size_t len, uint8_t out[20])
{
    sha1_t s;
    sha1_init(&s);
    sha1_update(&s, msg, len);
    sha1_final(&s, out);
}

/* HMAC-SHA1, crypto/hash/hmac.c:115-229 (key zero-padded to 64 bytes). */
typedef struct {
    sha1_t inner;
    uint8_t opad[64];
} hmac_t;

static int hmac_init(hmac_t *h, const uint8_t *key, size_t key_len)
{
    uint8_t ipad[64];
    if (key_len > 20)
        return 2;
    for (size_t i = 0; i < 64; i++) {
        uint8_t k = i < key_len ? key[i] : 0;
        ipad[i] = k ^ 0x36;
        h->opad[i] = k ^ 0x5c;
    }
    sha1_init(&h->inner);
    sha1_update(&h->inner, ipad, 64);
    return 0;
}

static void hmac_two_part(const hmac_t *h, const uint8_t *m1, size_t n1,
                          const uint8_t *m2, size_t n2, uint8_t out[20])
{
    sha1_t in = h->inner, outer;
    uint8_t ih[20];
    sha1_update(&in, m1, n1);
    sha1_update(&in, m2, n2);
    sha1_final(&in, ih);
    sha1_init(&outer);
    sha1_update(&outer, h->opad, 64);
    sha1_update(&outer, ih, 20);
    sha1_final(&outer, out);
}

int orc_hmac_sha1(const uint8_t *key, size_t key_len, const uint8_t *msg,
                  size_t len, uint8_t out[20])
{
    hmac_t h;
    if (hmac_init(&h, key, key_len))
        return 2;
    hmac_two_part(&h, msg, len, NULL, 0, out);
    return 0;
}

/* ======================================================================
 * AES-ICM (crypto/cipher/aes_icm.c:182-414).
 * ====================================================================== */

static int icm_run(const aes_ks_t *ks, const uint8_t salt14[14],
                   const uint8_t iv16[16], const uint8_t *in, size_t len,
                   uint8_t *out)
{
    uint8_t ctr[16], kb[16];
    for (int i = 0; i < 16; i++)
        ctr[i] = (uint8_t)((i < 14 ? salt14[i] : 0) ^ iv16[i]);
    /* terminus check, aes_icm.c:317-322 */
    size_t blocks = (len + 15) / 16;
    unsigned start = (unsigned)ctr[14] << 8 | ctr[15];
    if (blocks + start > 0xffff)
        return 6; /* srtp_err_status_terminus */
    for (size_t off = 0; off < len; off += 16) {
        aes_block(ks, ctr, kb);
        size_t n = len - off < 16 ? len - off : 16;
        for (size_t j = 0; j < n; j++)
            out[off + j] = in[off + j] ^ kb[j];
        /* 16-bit counter: carry from byte 15 into byte 14 only,
         * aes_icm.c:279-281 */
        if (++ctr[15] == 0)
            ++ctr[14];
    }
    return 0;
}

int orc_icm_xor(const uint8_t *key, size_t key_len, const uint8_t salt14[14],
                const uint8_t iv16[16], const uint8_t *in, size_t len,
                uint8_t *out)
{
    aes_ks_t ks;
    if (aes_expand(&ks, key, key_len))
        return 2;
    return icm_run(&ks, salt14, iv16, in, len, out);
}

/* ======================================================================
 * AES-GCM (SP 800-38D), behaviour of crypto/cipher/aes_gcm_ossl.c.
 * GHASH by the bit-serial algorithm 1 of SP 800-38D.
 * ====================================================================== */

typedef struct {
    uint64_t hi, lo;
} u128;

static u128 load128(const uint8_t *b)
{
    u128 r = { 0, 0 };
    for (int i = 0; i < 8; i++) {
        r.hi = r.hi << 8 | b[i];
        r.lo = r.lo << 8 | b[8 + i];
    }
    return r;
}

static void store128(u128 v, uint8_t *b)
{
    for (int i = 0; i < 8; i++) {
        b[i] = (uint8_t)(v.hi >> (56 - 8 * i));
        b[8 + i] = (uint8_t)(v.lo >> (56 - 8 * i));
    }
}

static u128 gf128_mul(u128 x, u128 y)
{
    u128 z = { 0, 0 }, v = y;
    for (int i = 0; i < 128; i++) {
        uint64_t bit = i < 64 ? (x.hi >> (63 - i)) & 1 : (x.lo >> (127 - i)) & 1;
        if (bit) {
            z.hi ^= v.hi;
            z.lo ^= v.lo;
        }
        uint64_t lsb = v.lo & 1;
        v.lo = (v.lo >> 1) | (v.hi << 63);
        v.hi >>= 1;
        if (lsb)
            v.hi ^= 0xe100000000000000ULL;
    }
    return z;
}

static void ghash_blocks(u128 *acc, u128 h, const uint8_t *d, size_t n)
{
    uint8_t blk[16];
    for (size_t off = 0; off < n; off += 16) {
        size_t k = n - off < 16 ? n - off : 16;
        memset(blk, 0, 16);
        memcpy(blk, d + off, k);
        u128 x = load128(blk);
        acc->hi ^= x.hi;
        acc->lo ^= x.lo;
        *acc = gf128_mul(*acc, h);
    }
}

static void gcm_core(const aes_ks_t *ks, const uint8_t iv[12],
                     const uint8_t *aad, size_t aad_len, const uint8_t *in,
                     size_t len, uint8_t *out, int encrypt, uint8_t tag[16])
{
    uint8_t zero[16] = { 0 }, hb[16], j0[16], ctr[16], kb[16];
    aes_block(ks, zero, hb);
    u128 h = load128(hb);
    memcpy(j0, iv, 12);
    j0[12] = j0[13] = j0[14] = 0;
    j0[15] = 1;
    memcpy(ctr, j0, 16);
    u128 acc = { 0, 0 };
    ghash_blocks(&acc, h, aad, aad_len);
    const uint8_t *ct = encrypt ? out : in;
    for (size_t off = 0; off < len; off += 16) {
        /* inc32 */
        for (int i = 15; i >= 12; i--)
            if (++ctr[i])
                break;
        aes_block(ks, ctr, kb);
        size_t n = len - off < 16 ? len - off : 16;
        for (size_t j = 0; j < n; j++)
            out[off + j] = in[off + j] ^ kb[j];
    }
    ghash_blocks(&acc, h, ct, len);
    uint8_t lb[16];
    uint64_t abits = (uint64_t)aad_len * 8, cbits = (uint64_t)len * 8;
    for (int i = 0; i < 8; i++) {
        lb[i] = (uint8_t)(abits >> (56 - 8 * i));
        lb[8 + i] = (uint8_t)(cbits >> (56 - 8 * i));
    }
    ghash_blocks(&acc, h, lb, 16);
    uint8_t s[16];
    store128(acc, s);
    aes_block(ks, j0, kb);
    for (int i = 0; i < 16; i++)
        tag[i] = s[i] ^ kb[i];
}

int orc_gcm_seal(const uint8_t *key, size_t key_len, const uint8_t iv[12],
                 const uint8_t *aad, size_t aad_len, const uint8_t *pt,
                 size_t len, uint8_t *ct, uint8_t *tag, size_t tag_len)
{
    aes_ks_t ks;
    uint8_t t[16];
    if (aes_expand(&ks, key, key_len) || (tag_len != 8 && tag_len != 16))
        return 2;
    gcm_core(&ks, iv, aad, aad_len, pt, len, ct, 1, t);
    memcpy(tag, t, tag_len);
    return 0;
}

int orc_gcm_open(const uint8_t *key, size_t key_len, const uint8_t iv[12],
                 const uint8_t *aad, size_t aad_len, const uint8_t *ct,
                 size_t len, const uint8_t *tag, size_t tag_len, uint8_t *pt)
{
    aes_ks_t ks;
    uint8_t t[16];
    if (aes_expand(&ks, key, key_len) || (tag_len != 8 && tag_len != 16))
        return 2;
    gcm_core(&ks, iv, aad, aad_len, ct, len, pt, 0, t);
    uint8_t diff = 0;
    for (size_t i = 0; i < tag_len; i++)
        diff |= (uint8_t)(t[i] ^ tag[i]);
    return diff ? 7 : 0;
}

/* ======================================================================
 * SRTP session model -- RTP path of srtp/srtp.c.
 * ====================================================================== */

enum {
    ST_OK = 0,
    ST_FAIL = 1,
    ST_BAD_PARAM = 2,
    ST_ALLOC = 3,
    ST_INIT_FAIL = 5,
    ST_AUTH_FAIL = 7,
    ST_CIPHER_FAIL = 8,
    ST_REPLAY_FAIL = 9,
    ST_REPLAY_OLD = 10,
    ST_NO_CTX = 13,
    ST_KEY_EXPIRED = 15,
    ST_PARSE_ERR = 21,
    ST_BAD_MKI = 25,
    ST_PKT_IDX_OLD = 26,
    ST_PKT_IDX_ADV = 27,
    ST_BUFFER_SMALL = 28
};

enum { DIR_UNKNOWN = 0, DIR_SENDER = 1, DIR_RECEIVER = 2 };

typedef struct {
    uint64_t num_left;
    int state; /* 0 normal, 1 past soft, 2 expired */
} key_limit_t;

typedef struct {
    uint32_t cipher_type;
    size_t cipher_key_len; /* total incl. salt, as in policy */
    size_t enc_key_len;
    aes_ks_t aes;
    uint8_t salt[14]; /* 14 (ICM) or 12 (GCM) meaningful bytes */
    uint32_t auth_type;
    size_t auth_key_len;
    size_t tag_len;
    hmac_t hmac;
    uint8_t mki[128];
    key_limit_t *limit; /* shared with clones, key.c:64-72 */
} session_keys_t;

typedef struct stream {
    uint32_t ssrc_net; /* as in header */
    int is_template;
    int direction;
    int sec_serv;
    int allow_repeat_tx;
    int use_mki;
    size_t mki_size;
    size_t num_keys;
    session_keys_t *keys; /* shared with clones */
    int owns_keys;
    /* rdbx (crypto/replay/rdbx.c) */
    uint64_t index;
    size_t win_bits; /* rounded up to 32, datatypes.c:264-268 */
    uint32_t *win;
    uint32_t pending_roc;
} stream_t;

struct orc_session {
    stream_t *templ;
    stream_t **list;
    size_t n, cap;
};

static uint32_t be32(const uint8_t *p)
{
    return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 |
           p[3];
}

static uint32_t ssrc_net_of(uint32_t host_ssrc)
{
    /* the reference stores SSRC as it appears in memory (network order);
     * we keep the big-endian numeric value instead and compare the same. */
    return host_ssrc;
}

/* ---- KDF: srtp/srtp.c:1066-1142 (AES-CM PRF, kdr 0) -------------------- */

static size_t full_key_length(uint32_t id)
{
    switch (id) {
    case ORC_AES_ICM_128: return 30;
    case ORC_AES_ICM_192: return 38;
    case ORC_AES_ICM_256: return 46;
    case ORC_AES_GCM_128: return 28;
    case ORC_AES_GCM_256: return 44;
    default: return 0;
    }
}

static size_t base_key_length(uint32_t id, size_t key_len)
{
    switch (id) {
    case ORC_NULL_CIPHER: return 0;
    case ORC_AES_ICM_128:
    case ORC_AES_ICM_192:
    case ORC_AES_ICM_256: return key_len - 14;
    case ORC_AES_GCM_128:
    case ORC_AES_GCM_256: return key_len - 12;
    default: return key_len;
    }
}

static void kdf_gen(const aes_ks_t *kdf, const uint8_t salt14[14],
                    uint8_t label, uint8_t *out, size_t len)
{
    uint8_t nonce[16] = { 0 }, zeros[256] = { 0 };
    nonce[7] = label; /* srtp.c:1112-1113 */
    icm_run(kdf, salt14, nonce, zeros, len, out);
}

/* Restates srtp_stream_init_keys (srtp.c:1233-1607) for the RTP keys,
 * taking the RTCP cipher into account only where it changes the KDF key
 * length (srtp.c:1266-1312); here RTCP is assumed to use the RTP policy. */
static int derive_keys(session_keys_t *sk, const uint8_t *master,
                       uint32_t cipher_type, size_t cipher_key_len,
                       uint32_t auth_type, size_t auth_key_len)
{
    size_t input_keylen = full_key_length(cipher_type);
    size_t a = auth_type == ORC_HMAC_SHA1 ? 30 : 0;
    if (a > input_keylen)
        input_keylen = a;
    size_t rtp_keylen = cipher_key_len;
    size_t base = base_key_length(cipher_type, rtp_keylen);
    size_t salt_len = rtp_keylen - base;
    if (rtp_keylen < input_keylen)
        return ST_BAD_PARAM; /* srtp.c:1293-1295 (rtcp == rtp here) */
    size_t kdf_keylen = 30;
    if (rtp_keylen > kdf_keylen)
        kdf_keylen = rtp_keylen;
    if (input_keylen > kdf_keylen)
        kdf_keylen = input_keylen;
    if (kdf_keylen == 28 || kdf_keylen == 44)
        kdf_keylen += 2; /* srtp.c:1309-1312 */
    if (kdf_keylen != 30 && kdf_keylen != 38 && kdf_keylen != 46)
        return ST_INIT_FAIL;
    uint8_t tmp[256];
    memset(tmp, 0, sizeof tmp);
    memcpy(tmp, master, input_keylen);
    aes_ks_t kdf;
    aes_expand(&kdf, tmp, kdf_keylen - 14);
    uint8_t kdf_salt[14];
    memcpy(kdf_salt, tmp + kdf_keylen - 14, 14);

    uint8_t ek[32], salt[32] = { 0 }, ak[20];
    kdf_gen(&kdf, kdf_salt, 0x00, ek, base);
    if (salt_len > 0)
        kdf_gen(&kdf, kdf_salt, 0x02, salt, salt_len);
    sk->cipher_type = cipher_type;
    sk->cipher_key_len = cipher_key_len;
    sk->enc_key_len = base;
    memset(sk->salt, 0, sizeof sk->salt);
    memcpy(sk->salt, salt, salt_len < 14 ? salt_len : 14);
    if (base)
        aes_expand(&sk->aes, ek, base);
    kdf_gen(&kdf, kdf_salt, 0x01, ak, auth_key_len);
    sk->auth_type = auth_type;
    sk->auth_key_len = auth_key_len;
    if (auth_type == ORC_HMAC_SHA1)
        hmac_init(&sk->hmac, ak, auth_key_len);
    return ST_OK;
}

int orc_derive(uint32_t cipher_type, size_t cipher_key_len,
               const uint8_t *master, uint8_t *enc_key, uint8_t *salt,
               uint8_t *auth_key, size_t auth_key_len)
{
    session_keys_t sk;
    memset(&sk, 0, sizeof sk);
    /* same derivation as a stream with HMAC-SHA1 auth; expose raw outputs */
    size_t input_keylen = full_key_length(cipher_type);
    if (input_keylen < 30)
        input_keylen = 30;
    size_t base = base_key_length(cipher_type, cipher_key_len);
    size_t salt_len = cipher_key_len - base;
    size_t kdf_keylen = 30;
    if (cipher_key_len > kdf_keylen)
        kdf_keylen = cipher_key_len;
    if (input_keylen > kdf_keylen)
        kdf_keylen = input_keylen;
    if (kdf_keylen == 28 || kdf_keylen == 44)
        kdf_keylen += 2;
    uint8_t tmp[256] = { 0 };
    memcpy(tmp, master, input_keylen);
    aes_ks_t kdf;
    aes_expand(&kdf, tmp, kdf_keylen - 14);
    uint8_t kdf_salt[14];
    memcpy(kdf_salt, tmp + kdf_keylen - 14, 14);
    kdf_gen(&kdf, kdf_salt, 0x00, enc_key, base);
    if (salt_len)
        kdf_gen(&kdf, kdf_salt, 0x02, salt, salt_len);
    kdf_gen(&kdf, kdf_salt, 0x01, auth_key, auth_key_len);
    return 0;
}

/* ---- rdbx: crypto/replay/rdbx.c + bitvector (crypto/math/datatypes.c) -- */

#define SEQ_MEDIAN 32768
#define SEQ_MAX 65536

static int64_t index_guess(uint64_t local, uint64_t *guess, uint16_t s)
{
    /* rdbx.c:112-145 */
    uint32_t local_roc = (uint32_t)(local >> 16);
    uint16_t local_seq = (uint16_t)local;
    uint32_t guess_roc;
    int64_t diff;
    if (local_seq < SEQ_MEDIAN) {
        if ((int)s - (int)local_seq > SEQ_MEDIAN) {
            guess_roc = local_roc - 1;
            diff = (int64_t)s - local_seq - SEQ_MAX;
        } else {
            guess_roc = local_roc;
            diff = (int64_t)s - local_seq;
        }
    } else {
        if ((int)local_seq - SEQ_MEDIAN > (int)s) {
            guess_roc = local_roc + 1;
            diff = (int64_t)s - local_seq + SEQ_MAX;
        } else {
            guess_roc = local_roc;
            diff = (int64_t)s - local_seq;
        }
    }
    *guess = ((uint64_t)guess_roc << 16) | s;
    return diff;
}

static int64_t rdbx_estimate(const stream_t *st, uint64_t *guess, uint16_t s)
{
    /* rdbx.c:280-299 */
    if (st->index > SEQ_MEDIAN)
        return index_guess(st->index, guess, s);
    *guess = s;
    return (int64_t)s - (int64_t)st->index;
}

static int win_get(const stream_t *st, size_t bit)
{
    return (st->win[bit >> 5] >> (bit & 31)) & 1;
}

static void win_set(stream_t *st, size_t bit)
{
    st->win[bit >> 5] |= 1u << (bit & 31);
}

static void win_zero(stream_t *st)
{
    memset(st->win, 0, st->win_bits / 8);
}

static void win_shift(stream_t *st, size_t shift)
{
    /* bitvector_left_shift: moves bits toward index 0, datatypes.c:375-406 */
    size_t words = st->win_bits >> 5;
    if (shift >= st->win_bits) {
        win_zero(st);
        return;
    }
    size_t base = shift >> 5, bi = shift & 31;
    if (bi == 0) {
        for (size_t i = 0; i < words - base; i++)
            st->win[i] = st->win[i + base];
    } else {
        for (size_t i = 0; i < words - base - 1; i++)
            st->win[i] = (st->win[i + base] >> bi) ^
                         (st->win[i + base + 1] << (32 - bi));
        st->win[words - base - 1] = st->win[words - 1] >> bi;
    }
    for (size_t i = words - base; i < words; i++)
        st->win[i] = 0;
}

static int rdbx_check(const stream_t *st, int64_t delta)
{
    /* rdbx.c:227-243 */
    if (delta > 0)
        return ST_OK;
    if ((int64_t)(st->win_bits - 1) + delta < 0)
        return ST_REPLAY_OLD;
    if (win_get(st, (size_t)((int64_t)(st->win_bits - 1) + delta)))
        return ST_REPLAY_FAIL;
    return ST_OK;
}

static void rdbx_add(stream_t *st, int64_t delta)
{
    /* rdbx.c:253-270 */
    if (delta > 0) {
        st->index += (uint16_t)delta; /* srtp_index_advance takes a seq */
        win_shift(st, (size_t)delta);
        win_set(st, st->win_bits - 1);
    } else {
        win_set(st, (size_t)((int64_t)(st->win_bits - 1) + delta));
    }
}

static void rdbx_set_roc_seq(stream_t *st, uint32_t roc, uint16_t seq)
{
    /* rdbx.c:323-338 (return value unused by the callers in srtp.c) */
    if (roc < (st->index >> 16))
        return;
    st->index = ((uint64_t)roc << 16) | seq;
    win_zero(st);
}

static int estimate_pkt_index(stream_t *st, uint16_t seq, uint64_t *est,
                              int64_t *delta)
{
    /* srtp_get_est_pkt_index / srtp_estimate_index, srtp.c:2038-2081 */
    if (st->pending_roc) {
        *est = ((uint64_t)st->pending_roc << 16) | seq;
        *delta = (int64_t)(*est - st->index);
        if (*est > st->index) {
            if (*est - st->index > SEQ_MEDIAN) {
                *delta = 0;
                return ST_PKT_IDX_ADV;
            }
        } else if (*est < st->index) {
            if (st->index - *est > SEQ_MEDIAN) {
                *delta = 0;
                return ST_PKT_IDX_OLD;
            }
        }
        return ST_OK;
    }
    *delta = rdbx_estimate(st, est, seq);
    return ST_OK;
}

static int key_limit_update(key_limit_t *k)
{
    /* crypto/kernel/key.c:74-90; 0 normal, 1 soft, 2 hard */
    k->num_left--;
    if (k->num_left >= 0x10000)
        return 0;
    if (k->state == 0)
        k->state = 1;
    if (k->num_left < 1) {
        k->state = 2;
        return 2;
    }
    return 1;
}

/* ---- sessions --------------------------------------------------------- */

int orc_session_create(orc_session_t **s)
{
    *s = (orc_session_t *)calloc(1, sizeof(orc_session_t));
    return *s ? ST_OK : ST_ALLOC;
}

static stream_t *stream_new(size_t win_bits)
{
    stream_t *st = (stream_t *)calloc(1, sizeof(stream_t));
    st->win_bits = (win_bits + 31) & ~(size_t)31;
    st->win = (uint32_t *)calloc(st->win_bits / 32 + 4, 4);
    return st;
}

static void stream_free(stream_t *st)
{
    if (st->owns_keys) {
        for (size_t i = 0; i < st->num_keys; i++)
            free(st->keys[i].limit);
        free(st->keys);
    }
    free(st->win);
    free(st);
}

static void list_insert(orc_session_t *s, stream_t *st)
{
    if (s->n == s->cap) {
        s->cap = s->cap ? 2 * s->cap : 4;
        s->list = (stream_t **)realloc(s->list, s->cap * sizeof(stream_t *));
    }
    s->list[s->n++] = st;
}

static stream_t *list_get(orc_session_t *s, uint32_t ssrc)
{
    for (size_t i = 0; i < s->n; i++) /* first match, srtp.c:5292-5305 */
        if (s->list[i]->ssrc_net == ssrc)
            return s->list[i];
    return NULL;
}

int orc_session_add(orc_session_t *s, const orc_policy_t *p)
{
    if (p->window_size != 0 &&
        (p->window_size < 64 || p->window_size >= 0x8000))
        return ST_BAD_PARAM; /* srtp.c:1670-1672 */
    if (p->num_master_keys < 1 || p->num_master_keys > 16)
        return ST_BAD_PARAM;
    stream_t *st = stream_new(p->window_size ? p->window_size : 128);
    st->ssrc_net = ssrc_net_of(p->ssrc);
    st->sec_serv = p->sec_serv;
    st->allow_repeat_tx = p->allow_repeat_tx;
    st->use_mki = p->use_mki;
    st->mki_size = p->use_mki ? p->mki_size : 0;
    st->num_keys = p->num_master_keys;
    st->keys = (session_keys_t *)calloc(st->num_keys, sizeof(session_keys_t));
    st->owns_keys = 1;
    for (size_t i = 0; i < st->num_keys; i++) {
        session_keys_t *k = &st->keys[i];
        k->limit = (key_limit_t *)calloc(1, sizeof(key_limit_t));
        k->limit->num_left = 0xffffffffffffULL; /* srtp.c:1251 */
        int rc = derive_keys(k, p->keys[i], p->cipher_type, p->cipher_key_len,
                             p->auth_type, p->auth_key_len);
        if (rc) {
            stream_free(st);
            return rc;
        }
        k->tag_len = p->auth_tag_len;
        if (st->use_mki)
            memcpy(k->mki, p->mki_ids[i], st->mki_size);
    }
    switch (p->ssrc_type) {
    case 3: /* any outbound, srtp.c:3275-3283 */
    case 2:
        if (s->templ) {
            stream_free(st);
            return ST_BAD_PARAM;
        }
        st->is_template = 1;
        st->direction = p->ssrc_type == 3 ? DIR_SENDER : DIR_RECEIVER;
        s->templ = st;
        break;
    case 1:
        list_insert(s, st);
        break;
    default:
        stream_free(st);
        return ST_BAD_PARAM;
    }
    return ST_OK;
}

void orc_session_free(orc_session_t *s)
{
    if (!s)
        return;
    for (size_t i = 0; i < s->n; i++)
        stream_free(s->list[i]);
    if (s->templ)
        stream_free(s->templ);
    free(s->list);
    free(s);
}

static stream_t *stream_clone(const stream_t *t, uint32_t ssrc)
{
    /* srtp_stream_clone, srtp.c:762-863: shares keys + key limit */
    stream_t *st = stream_new(t->win_bits);
    st->ssrc_net = ssrc;
    st->direction = t->direction;
    st->sec_serv = t->sec_serv;
    st->allow_repeat_tx = t->allow_repeat_tx;
    st->use_mki = t->use_mki;
    st->mki_size = t->mki_size;
    st->num_keys = t->num_keys;
    st->keys = t->keys;
    st->owns_keys = 0;
    return st;
}

static size_t rtp_hdr_len(const uint8_t *p)
{
    return 12 + 4 * (size_t)(p[0] & 0x0f);
}

static int validate_header(const uint8_t *p, size_t len)
{
    /* srtp_validate_rtp_header, srtp.c:307-336 */
    if (len < 12)
        return ST_BAD_PARAM;
    size_t h = rtp_hdr_len(p);
    if (len < h)
        return ST_BAD_PARAM;
    if (p[0] & 0x10) {
        if (len < h + 4)
            return ST_BAD_PARAM;
        h += ((size_t)(p[h + 2] << 8 | p[h + 3]) + 1) * 4;
        if (len < h)
            return ST_BAD_PARAM;
    }
    return ST_OK;
}

static size_t enc_start_of(const uint8_t *p)
{
    size_t h = rtp_hdr_len(p);
    if (p[0] & 0x10)
        h += ((size_t)(p[h + 2] << 8 | p[h + 3]) + 1) * 4;
    return h;
}

static int is_gcm(uint32_t c)
{
    return c == ORC_AES_GCM_128 || c == ORC_AES_GCM_256;
}

static void gcm_iv(const session_keys_t *k, uint32_t ssrc, uint64_t est,
                   uint8_t iv[12])
{
    /* srtp_calc_aead_iv, srtp.c:1925-1959 */
    uint32_t roc = (uint32_t)(est >> 16);
    uint16_t seq = (uint16_t)est;
    uint8_t in[12] = { 0, 0,
                       (uint8_t)(ssrc >> 24), (uint8_t)(ssrc >> 16),
                       (uint8_t)(ssrc >> 8), (uint8_t)ssrc,
                       (uint8_t)(roc >> 24), (uint8_t)(roc >> 16),
                       (uint8_t)(roc >> 8), (uint8_t)roc,
                       (uint8_t)(seq >> 8), (uint8_t)seq };
    for (int i = 0; i < 12; i++)
        iv[i] = in[i] ^ k->salt[i];
}

static void icm_iv(uint32_t ssrc, uint64_t est, uint8_t iv[16])
{
    /* srtp.c:2694-2707: v32[0]=0, v32[1]=ssrc, v64[1]=be64(est<<16) */
    memset(iv, 0, 16);
    iv[4] = (uint8_t)(ssrc >> 24);
    iv[5] = (uint8_t)(ssrc >> 16);
    iv[6] = (uint8_t)(ssrc >> 8);
    iv[7] = (uint8_t)ssrc;
    uint64_t v = est << 16;
    for (int i = 0; i < 8; i++)
        iv[8 + i] = (uint8_t)(v >> (56 - 8 * i));
}

static int protect_aead(stream_t *st, session_keys_t *k, const uint8_t *rtp,
                        size_t rtp_len, uint8_t *srtp, size_t *srtp_len)
{
    /* srtp_protect_aead, srtp.c:2088-2267 */
    int ev = key_limit_update(k->limit);
    if (ev == 2)
        return ST_KEY_EXPIRED;
    size_t tag_len = k->tag_len;
    if (*srtp_len < rtp_len + tag_len + st->mki_size)
        return ST_BUFFER_SMALL;
    size_t enc_start = enc_start_of(rtp);
    if (enc_start > rtp_len)
        return ST_PARSE_ERR;
    size_t enc_len = rtp_len - enc_start;
    uint16_t seq = (uint16_t)(rtp[2] << 8 | rtp[3]);
    uint64_t est;
    int64_t delta;
    int rc = estimate_pkt_index(st, seq, &est, &delta);
    if (rc && rc != ST_PKT_IDX_ADV)
        return rc;
    if (rc == ST_PKT_IDX_ADV) {
        rdbx_set_roc_seq(st, (uint32_t)(est >> 16), (uint16_t)est);
        st->pending_roc = 0;
        rdbx_add(st, 0);
    } else {
        rc = rdbx_check(st, delta);
        if (rc && (rc != ST_REPLAY_FAIL || !st->allow_repeat_tx))
            return rc;
        rdbx_add(st, delta);
    }
    uint8_t iv[12], tag[16];
    gcm_iv(k, be32(rtp + 8), est, iv);
    if (rtp != srtp)
        memmove(srtp, rtp, enc_start);
    uint8_t *tmp = (uint8_t *)malloc(enc_len + 1);
    gcm_core(&k->aes, iv, srtp, enc_start, rtp + enc_start, enc_len, tmp, 1,
             tag);
    memcpy(srtp + enc_start, tmp, enc_len);
    free(tmp);
    memcpy(srtp + enc_start + enc_len, tag, tag_len);
    if (st->use_mki)
        memcpy(srtp + enc_start + enc_len + tag_len, k->mki, st->mki_size);
    *srtp_len = enc_start + enc_len + tag_len + st->mki_size;
    return ST_OK;
}

int orc_protect(orc_session_t *s, const uint8_t *rtp, size_t rtp_len,
                uint8_t *srtp, size_t *srtp_len, size_t mki_index)
{
    /* srtp_protect, srtp.c:2493-2818 */
    int rc = validate_header(rtp, rtp_len);
    if (rc)
        return rc;
    uint32_t ssrc = be32(rtp + 8);
    stream_t *st = list_get(s, ssrc);
    if (!st) {
        if (!s->templ)
            return ST_NO_CTX;
        st = stream_clone(s->templ, ssrc);
        list_insert(s, st);
        st->direction = DIR_SENDER;
    }
    if (st->direction != DIR_SENDER) {
        if (st->direction == DIR_UNKNOWN)
            st->direction = DIR_SENDER;
        /* else: ssrc collision event, no status change */
    }
    session_keys_t *k;
    if (st->use_mki) {
        if (mki_index >= st->num_keys)
            return ST_BAD_MKI;
        k = &st->keys[mki_index];
    } else {
        k = &st->keys[0];
    }
    if (is_gcm(k->cipher_type))
        return protect_aead(st, k, rtp, rtp_len, srtp, srtp_len);
    if (key_limit_update(k->limit) == 2)
        return ST_KEY_EXPIRED;
    size_t tag_len = k->tag_len; /* srtp_auth_get_tag_length, srtp.c:2612 */
    if (*srtp_len < rtp_len + st->mki_size + tag_len)
        return ST_BUFFER_SMALL;
    size_t enc_start = enc_start_of(rtp);
    if (enc_start > rtp_len)
        return ST_PARSE_ERR;
    size_t enc_len = rtp_len - enc_start;
    if (rtp != srtp)
        memmove(srtp, rtp, enc_start);
    if (st->use_mki)
        memcpy(srtp + rtp_len, k->mki, st->mki_size);
    uint16_t seq = (uint16_t)(rtp[2] << 8 | rtp[3]);
    uint64_t est;
    int64_t delta;
    rc = estimate_pkt_index(st, seq, &est, &delta);
    if (rc && rc != ST_PKT_IDX_ADV)
        return rc;
    if (rc == ST_PKT_IDX_ADV) {
        rdbx_set_roc_seq(st, (uint32_t)(est >> 16), (uint16_t)est);
        st->pending_roc = 0;
        rdbx_add(st, 0);
    } else {
        rc = rdbx_check(st, delta);
        if (rc && (rc != ST_REPLAY_FAIL || !st->allow_repeat_tx))
            return rc;
        rdbx_add(st, delta);
    }
    if (st->sec_serv & 1) {
        if (k->cipher_type != ORC_NULL_CIPHER) {
            uint8_t iv[16];
            icm_iv(ssrc, est, iv);
            rc = icm_run(&k->aes, k->salt, iv, rtp + enc_start, enc_len,
                         srtp + enc_start);
            if (rc)
                return ST_CIPHER_FAIL;
        } else if (rtp != srtp) {
            memmove(srtp + enc_start, rtp + enc_start, enc_len);
        }
    } else if (rtp != srtp) {
        memmove(srtp + enc_start, rtp + enc_start, enc_len);
    }
    if ((st->sec_serv & 2) && k->auth_type == ORC_HMAC_SHA1) {
        uint8_t roc[4], full[20];
        uint32_t r = (uint32_t)(est >> 16);
        roc[0] = (uint8_t)(r >> 24);
        roc[1] = (uint8_t)(r >> 16);
        roc[2] = (uint8_t)(r >> 8);
        roc[3] = (uint8_t)r;
        hmac_two_part(&k->hmac, srtp, rtp_len, roc, 4, full);
        memcpy(srtp + rtp_len + st->mki_size, full, tag_len);
    }
    *srtp_len = enc_start + enc_len + tag_len + st->mki_size;
    return ST_OK;
}

static int unprotect_aead(orc_session_t *s, stream_t *st, session_keys_t *k,
                          int64_t delta, uint64_t est, const uint8_t *srtp,
                          size_t srtp_len, uint8_t *rtp, size_t *rtp_len,
                          int advance)
{
    /* srtp_unprotect_aead, srtp.c:2276-2491 */
    size_t tag_len = k->tag_len;
    size_t enc_start = enc_start_of(srtp);
    if (enc_start > srtp_len - tag_len - st->mki_size)
        return ST_PARSE_ERR;
    size_t enc_len = srtp_len - enc_start - st->mki_size;
    if (enc_len < tag_len)
        return ST_CIPHER_FAIL;
    if (*rtp_len < srtp_len - st->mki_size - tag_len)
        return ST_BUFFER_SMALL;
    if (key_limit_update(k->limit) == 2)
        return ST_KEY_EXPIRED;
    uint8_t iv[12], tag[16];
    gcm_iv(k, be32(srtp + 8), est, iv);
    size_t ct_len = enc_len - tag_len;
    uint8_t *tmp = (uint8_t *)malloc(ct_len + 1);
    gcm_core(&k->aes, iv, srtp, enc_start, srtp + enc_start, ct_len, tmp, 0,
             tag);
    uint8_t diff = 0;
    for (size_t i = 0; i < tag_len; i++)
        diff |= (uint8_t)(tag[i] ^ srtp[enc_start + ct_len + i]);
    if (diff) {
        free(tmp);
        return ST_AUTH_FAIL;
    }
    if (srtp != rtp)
        memmove(rtp, srtp, enc_start);
    memcpy(rtp + enc_start, tmp, ct_len);
    free(tmp);
    if (st->direction != DIR_RECEIVER && st->direction == DIR_UNKNOWN)
        st->direction = DIR_RECEIVER;
    if (st == s->templ) {
        stream_t *ns = stream_clone(s->templ, be32(srtp + 8));
        list_insert(s, ns);
        st = ns;
    }
    if (advance) {
        rdbx_set_roc_seq(st, (uint32_t)(est >> 16), (uint16_t)est);
        st->pending_roc = 0;
        rdbx_add(st, 0);
    } else {
        rdbx_add(st, delta);
    }
    *rtp_len = enc_start + ct_len;
    return ST_OK;
}

int orc_unprotect(orc_session_t *s, const uint8_t *srtp, size_t srtp_len,
                  uint8_t *rtp, size_t *rtp_len)
{
    /* srtp_unprotect, srtp.c:2820-3172 */
    int rc = validate_header(srtp, srtp_len);
    if (rc)
        return rc;
    uint32_t ssrc = be32(srtp + 8);
    uint16_t seq = (uint16_t)(srtp[2] << 8 | srtp[3]);
    stream_t *st = list_get(s, ssrc);
    uint64_t est;
    int64_t delta;
    int advance = 0;
    if (!st) {
        if (!s->templ)
            return ST_NO_CTX;
        st = s->templ;
        est = seq;
        delta = (int64_t)est;
    } else {
        rc = estimate_pkt_index(st, seq, &est, &delta);
        if (rc && rc != ST_PKT_IDX_ADV)
            return rc;
        if (rc == ST_PKT_IDX_ADV)
            advance = 1;
        if (!advance) {
            rc = rdbx_check(st, delta);
            if (rc)
                return rc;
        }
    }
    /* session keys by MKI, srtp.c:1961-2036 (tag_len 0 for GCM) */
    session_keys_t *k = &st->keys[0];
    if (st->use_mki) {
        size_t tl = is_gcm(st->keys[0].cipher_type) ? 0 : st->keys[0].tag_len;
        if (tl > srtp_len)
            return ST_BAD_MKI;
        size_t loc = srtp_len - tl;
        if (st->mki_size > loc)
            return ST_BAD_MKI;
        loc -= st->mki_size;
        k = NULL;
        for (size_t i = 0; i < st->num_keys; i++)
            if (memcmp(srtp + loc, st->keys[i].mki, st->mki_size) == 0) {
                k = &st->keys[i];
                break;
            }
        if (!k)
            return ST_BAD_MKI;
    }
    if (is_gcm(k->cipher_type))
        return unprotect_aead(s, st, k, delta, est, srtp, srtp_len, rtp,
                              rtp_len, advance);
    size_t tag_len = k->tag_len;
    size_t enc_start = enc_start_of(srtp);
    if (enc_start > srtp_len - tag_len - st->mki_size)
        return ST_PARSE_ERR;
    size_t enc_len = srtp_len - enc_start - st->mki_size - tag_len;
    if (*rtp_len < srtp_len - st->mki_size - tag_len)
        return ST_BUFFER_SMALL;
    if ((st->sec_serv & 2) && k->auth_type == ORC_HMAC_SHA1) {
        uint8_t roc[4], full[20];
        uint32_t r = (uint32_t)(est >> 16);
        roc[0] = (uint8_t)(r >> 24);
        roc[1] = (uint8_t)(r >> 16);
        roc[2] = (uint8_t)(r >> 8);
        roc[3] = (uint8_t)r;
        hmac_two_part(&k->hmac, srtp, srtp_len - tag_len - st->mki_size, roc,
                      4, full);
        uint8_t diff = 0;
        for (size_t i = 0; i < tag_len; i++)
            diff |= (uint8_t)(full[i] ^ srtp[srtp_len - tag_len + i]);
        if (diff)
            return ST_AUTH_FAIL;
    }
    if (key_limit_update(k->limit) == 2)
        return ST_KEY_EXPIRED;
    if (srtp != rtp)
        memmove(rtp, srtp, enc_start);
    if ((st->sec_serv & 1) && k->cipher_type != ORC_NULL_CIPHER) {
        uint8_t iv[16];
        icm_iv(ssrc, est, iv);
        rc = icm_run(&k->aes, k->salt, iv, srtp + enc_start, enc_len,
                     rtp + enc_start);
        if (rc)
            return ST_CIPHER_FAIL;
    } else if (srtp != rtp) {
        memmove(rtp + enc_start, srtp + enc_start, enc_len);
    }
    if (st->direction != DIR_RECEIVER && st->direction == DIR_UNKNOWN)
        st->direction = DIR_RECEIVER;
    if (st == s->templ) {
        stream_t *ns = stream_clone(s->templ, ssrc);
        list_insert(s, ns);
        st = ns;
    }
    if (advance) {
        rdbx_set_roc_seq(st, (uint32_t)(est >> 16), (uint16_t)est);
        st->pending_roc = 0;
        rdbx_add(st, 0);
    } else {
        rdbx_add(st, delta);
    }
    *rtp_len = enc_start + enc_len;
    return ST_OK;
}

int orc_get_roc(orc_session_t *s, uint32_t ssrc, uint32_t *roc)
{
    stream_t *st = list_get(s, ssrc);
    if (!st)
        return ST_BAD_PARAM;
    *roc = (uint32_t)(st->index >> 16);
    return ST_OK;
}

/* the uses left of master key j of stream ssrc (key.c:74-90's counter) */
int orc_key_left(orc_session_t *s, uint32_t ssrc, size_t j, uint64_t *left)
{
    stream_t *st = list_get(s, ssrc);
    if (!st || j >= st->num_keys)
        return ST_BAD_PARAM;
    *left = st->keys[j].limit->num_left;
    return ST_OK;
}

int orc_set_roc(orc_session_t *s, uint32_t ssrc, uint32_t roc)
{
    stream_t *st = list_get(s, ssrc);
    if (!st)
        return ST_BAD_PARAM;
    st->pending_roc = roc;
    return ST_OK;
}

size_t orc_protect_many(orc_session_t *s, size_t n, const uint8_t *in,
                        const uint64_t *in_off, const uint32_t *in_len,
                        uint8_t *out, const uint64_t *out_off,
                        uint32_t *out_len, uint32_t out_cap)
{
    size_t bad = 0;
    for (size_t i = 0; i < n; i++) {
        size_t len = out_cap;
        int rc = orc_protect(s, in + in_off[i], in_len[i], out + out_off[i],
                             &len, 0);
        out_len[i] = rc ? 0 : (uint32_t)len;
        bad += rc != 0;
    }
    return bad;
}

/* orc_unprotect over n packets in order (test infrastructure: the reference
 * receive loop of test/rtp.c:104-149, one srtp_unprotect per packet):
 * status[i] per packet, out_len[i] the plaintext length (0 on error) */
void orc_unprotect_many(orc_session_t *s, size_t n, const uint8_t *in,
                        const uint64_t *in_off, const uint32_t *in_len,
                        uint8_t *out, const uint64_t *out_off,
                        uint32_t *out_len, uint32_t out_cap, int32_t *status)
{
    for (size_t i = 0; i < n; i++) {
        size_t len = out_cap;
        int rc = orc_unprotect(s, in + in_off[i], in_len[i], out + out_off[i],
                               &len);
        status[i] = rc;
        out_len[i] = rc ? 0 : (uint32_t)len;
    }
}
