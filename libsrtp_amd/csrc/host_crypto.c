/*
 * host_crypto.c -- see host_crypto.h.  Word-oriented AES with tables built
 * at first use; plain SHA-1 compression; GHASH table by doubling.
 */
#include "host_crypto.h"

#include <string.h>

static uint32_t te[256]; /* MixColumns(S[x]) column, little-endian */
static uint8_t sb[256];
static int ready;

static uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a >> 7) * 0x1b)); }

static void tables(void)
{
    if (ready)
        return;
    /* walk the multiplicative group with generator 3 to get inverses */
    uint8_t pw[256], lg[256];
    uint8_t x = 1;
    for (int i = 0; i < 255; i++) {
        pw[i] = x;
        lg[x] = (uint8_t)i;
        x = (uint8_t)(x ^ xt(x)); /* x * 3 */
    }
    for (int v = 0; v < 256; v++) {
        uint8_t inv = v ? pw[(255 - lg[v]) % 255] : 0;
        uint8_t s = inv;
        for (int k = 1; k <= 4; k++)
            s ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
        sb[v] = s ^ 0x63;
    }
    for (int v = 0; v < 256; v++) {
        uint8_t s = sb[v], s2 = xt(s), s3 = (uint8_t)(s2 ^ s);
        te[v] = (uint32_t)s2 | (uint32_t)s << 8 | (uint32_t)s << 16 |
                (uint32_t)s3 << 24;
    }
    ready = 1;
}

static uint32_t rol8(uint32_t w, int n) { return (w << n) | (w >> (32 - n)); }

int hc_aes_init(hc_aes_t *a, const uint8_t *key, size_t key_len)
{
    tables();
    if (key_len != 16 && key_len != 24 && key_len != 32)
        return -1;
    int nk = (int)key_len / 4;
    a->rounds = nk + 6;
    int total = 4 * (a->rounds + 1);
    uint32_t rc = 1;
    for (int i = 0; i < nk; i++)
        a->rk[i] = (uint32_t)key[4 * i] | (uint32_t)key[4 * i + 1] << 8 |
                   (uint32_t)key[4 * i + 2] << 16 |
                   (uint32_t)key[4 * i + 3] << 24;
    for (int i = nk; i < total; i++) {
        uint32_t t = a->rk[i - 1];
        if (i % nk == 0) {
            t = (t >> 8) | (t << 24); /* RotWord on little-endian bytes */
            t = (uint32_t)sb[t & 0xff] | (uint32_t)sb[(t >> 8) & 0xff] << 8 |
                (uint32_t)sb[(t >> 16) & 0xff] << 16 |
                (uint32_t)sb[t >> 24] << 24;
            t ^= rc;
            rc = xt((uint8_t)rc);
        } else if (nk > 6 && i % nk == 4) {
            t = (uint32_t)sb[t & 0xff] | (uint32_t)sb[(t >> 8) & 0xff] << 8 |
                (uint32_t)sb[(t >> 16) & 0xff] << 16 |
                (uint32_t)sb[t >> 24] << 24;
        }
        a->rk[i] = a->rk[i - nk] ^ t;
    }
    for (int i = total; i < 60; i++)
        a->rk[i] = 0;
    return 0;
}

void hc_aes_block(const hc_aes_t *a, const uint8_t in[16], uint8_t out[16])
{
    uint32_t s[4], t[4];
    for (int c = 0; c < 4; c++)
        s[c] = ((uint32_t)in[4 * c] | (uint32_t)in[4 * c + 1] << 8 |
                (uint32_t)in[4 * c + 2] << 16 | (uint32_t)in[4 * c + 3] << 24) ^
               a->rk[c];
    for (int r = 1; r < a->rounds; r++) {
        for (int c = 0; c < 4; c++)
            t[c] = te[s[c] & 0xff] ^ rol8(te[(s[(c + 1) & 3] >> 8) & 0xff], 8) ^
                   rol8(te[(s[(c + 2) & 3] >> 16) & 0xff], 16) ^
                   rol8(te[s[(c + 3) & 3] >> 24], 24) ^ a->rk[4 * r + c];
        memcpy(s, t, sizeof s);
    }
    for (int c = 0; c < 4; c++)
        t[c] = ((uint32_t)sb[s[c] & 0xff] |
                (uint32_t)sb[(s[(c + 1) & 3] >> 8) & 0xff] << 8 |
                (uint32_t)sb[(s[(c + 2) & 3] >> 16) & 0xff] << 16 |
                (uint32_t)sb[s[(c + 3) & 3] >> 24] << 24) ^
               a->rk[4 * a->rounds + c];
    for (int c = 0; c < 4; c++)
        for (int b = 0; b < 4; b++)
            out[4 * c + b] = (uint8_t)(t[c] >> (8 * b));
}

void hc_icm_keystream(const hc_aes_t *a, const uint8_t salt14[14],
                      const uint8_t iv16[16], uint8_t *out, size_t len)
{
    uint8_t ctr[16], ks[16];
    for (int i = 0; i < 16; i++)
        ctr[i] = (uint8_t)((i < 14 ? salt14[i] : 0) ^ iv16[i]);
    for (size_t off = 0; off < len; off += 16) {
        hc_aes_block(a, ctr, ks);
        size_t n = len - off < 16 ? len - off : 16;
        memcpy(out + off, ks, n);
        if (++ctr[15] == 0)
            ++ctr[14];
    }
}

static uint32_t rl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

void hc_sha1_midstate(const uint8_t block[64], uint32_t h[5])
{
    static const uint32_t iv[5] = { 0x67452301u, 0xefcdab89u, 0x98badcfeu,
                                    0x10325476u, 0xc3d2e1f0u };
    uint32_t w[80], a = iv[0], b = iv[1], c = iv[2], d = iv[3], e = iv[4];
    for (int t = 0; t < 16; t++)
        w[t] = (uint32_t)block[4 * t] << 24 | (uint32_t)block[4 * t + 1] << 16 |
               (uint32_t)block[4 * t + 2] << 8 | block[4 * t + 3];
    for (int t = 16; t < 80; t++)
        w[t] = rl(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);
    for (int t = 0; t < 80; t++) {
        uint32_t f, k;
        if (t < 20) {
            f = d ^ (b & (c ^ d));
            k = 0x5a827999u;
        } else if (t < 40) {
            f = b ^ c ^ d;
            k = 0x6ed9eba1u;
        } else if (t < 60) {
            f = (b & c) ^ (d & (b ^ c));
            k = 0x8f1bbcdcu;
        } else {
            f = b ^ c ^ d;
            k = 0xca62c1d6u;
        }
        uint32_t tmp = rl(a, 5) + f + e + k + w[t];
        e = d;
        d = c;
        c = rl(b, 30);
        b = a;
        a = tmp;
    }
    h[0] = iv[0] + a;
    h[1] = iv[1] + b;
    h[2] = iv[2] + c;
    h[3] = iv[3] + d;
    h[4] = iv[4] + e;
}

void hc_ghash_table(const uint8_t hb[16], uint32_t tab[1024])
{
    /* element v as 4 big-endian words; v * x = v >> 1 (^ 0xe1 || 0^120) */
    uint32_t v[4];
    for (int i = 0; i < 4; i++)
        v[i] = (uint32_t)hb[4 * i] << 24 | (uint32_t)hb[4 * i + 1] << 16 |
               (uint32_t)hb[4 * i + 2] << 8 | hb[4 * i + 3];
    memset(tab, 0, 1024 * sizeof(uint32_t));
    for (int bit = 0x80; bit; bit >>= 1) {
        memcpy(tab + 4 * bit, v, sizeof v);
        uint32_t lsb = v[3] & 1;
        v[3] = (v[3] >> 1) | (v[2] << 31);
        v[2] = (v[2] >> 1) | (v[1] << 31);
        v[1] = (v[1] >> 1) | (v[0] << 31);
        v[0] >>= 1;
        if (lsb)
            v[0] ^= 0xe1000000u;
    }
    for (int b = 1; b < 256; b++) {
        int low = b & -b;
        if (b == low)
            continue;
        for (int i = 0; i < 4; i++)
            tab[4 * b + i] = tab[4 * low + i] ^ tab[4 * (b ^ low) + i];
    }
}
