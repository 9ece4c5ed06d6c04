// bsaes.hip -- prototype: AES-128 counter-mode keystream for SRTP ICM with
// a BITSLICED AES on the VALU (no LDS) against the T-table form the
// shipped kernels use (4 tables x 32 copies in LDS, one v_perm per
// lookup).  Timing and a bit-exact check of both against a plain host AES.
// Not part of the library; the measurement behind DESIGN.md's next-round
// note on the headline kernel.
//
// One lane = one packet's keystream: counter block j = IV ^ (0...0 || j16)
// (crypto/cipher/aes_icm.c:199-210, 279-281; IV bytes 14-15 are zero in
// SRTP), NBLK blocks.  Bitsliced: 32 blocks per lane at a time, state
// R[p][b] (byte position p, bit b): bit k of R[p][b] = bit b of byte p of
// block k.  ShiftRows is a renaming, MixColumns XORs across registers,
// SubBytes the 113-gate Boyar-Peralta circuit (checked exhaustively on the
// host), AddRoundKey one XOR with a 0 / ~0 mask from a uniform table.
// Output: a 32 x 32 bit transpose per column gives block k's column words.
//
//   hipcc -O3 --offload-arch=gfx950 tools/bsaes.hip -o tools/bsaes
//   ./bsaes            (host check only when no GPU)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define HD __host__ __device__ __forceinline__

// ---- host AES (FIPS-197), S-box from the GF(2^8) inverse ----------------
static uint8_t h_sbox[256];
static uint8_t gmul(uint8_t a, uint8_t b)
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
static void make_sbox()
{
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        for (int y = 1; y < 256 && x; y++)
            if (gmul((uint8_t)x, (uint8_t)y) == 1)
                inv = (uint8_t)y;
        uint8_t s = 0x63;
        for (int i = 0; i < 8; i++) {
            int bit = ((inv >> i) ^ (inv >> ((i + 4) & 7)) ^ (inv >> ((i + 5) & 7)) ^
                       (inv >> ((i + 6) & 7)) ^ (inv >> ((i + 7) & 7))) & 1;
            s ^= (uint8_t)(bit << i);
        }
        h_sbox[x] = s;
    }
}
static void expand(const uint8_t key[16], uint8_t rk[11][16])
{
    memcpy(rk[0], key, 16);
    uint8_t rc = 1;
    for (int r = 1; r <= 10; r++) {
        uint8_t t[4] = { h_sbox[rk[r - 1][13]], h_sbox[rk[r - 1][14]],
                         h_sbox[rk[r - 1][15]], h_sbox[rk[r - 1][12]] };
        t[0] ^= rc;
        rc = gmul(rc, 2);
        for (int i = 0; i < 16; i++) {
            rk[r][i] = rk[r - 1][i] ^ t[i & 3];
            if ((i & 3) == 3)
                memcpy(t, &rk[r][i - 3], 4);
        }
    }
}
static void h_aes(const uint8_t rk[11][16], const uint8_t in[16], uint8_t out[16])
{
    uint8_t s[16];
    for (int i = 0; i < 16; i++)
        s[i] = in[i] ^ rk[0][i];
    for (int r = 1; r <= 10; r++) {
        uint8_t t[16];
        for (int i = 0; i < 16; i++)
            t[i] = h_sbox[s[i]];
        for (int c = 0; c < 4; c++)
            for (int row = 0; row < 4; row++)
                s[row + 4 * c] = t[row + 4 * ((c + row) & 3)];
        if (r < 10)
            for (int c = 0; c < 4; c++) {
                uint8_t a[4] = { s[4 * c], s[4 * c + 1], s[4 * c + 2], s[4 * c + 3] };
                for (int i = 0; i < 4; i++)
                    s[4 * c + i] = gmul(a[i], 2) ^ gmul(a[(i + 1) & 3], 3) ^
                                   a[(i + 2) & 3] ^ a[(i + 3) & 3];
            }
        for (int i = 0; i < 16; i++)
            s[i] ^= rk[r][i];
    }
    memcpy(out, s, 16);
}

// ---- bitsliced AES ---------------------------------------------------------
// Boyar-Peralta S-box; U0 = bit 7 (MSB) ... U7 = bit 0; in place on x[8]
// where x[b] = bit b
HD void bs_sbox(uint32_t *x)
{
    const uint32_t U0 = x[7], U1 = x[6], U2 = x[5], U3 = x[4], U4 = x[3],
                   U5 = x[2], U6 = x[1], U7 = x[0];
    const uint32_t T1 = U0 ^ U3, T2 = U0 ^ U5, T3 = U0 ^ U6, T4 = U3 ^ U5,
                   T5 = U4 ^ U6, T6 = T1 ^ T5, T7 = U1 ^ U2, T8 = U7 ^ T6,
                   T9 = U7 ^ T7, T10 = T6 ^ T7, T11 = U1 ^ U5, T12 = U2 ^ U5,
                   T13 = T3 ^ T4, T14 = T6 ^ T11, T15 = T5 ^ T11,
                   T16 = T5 ^ T12, T17 = T9 ^ T16, T18 = U3 ^ U7,
                   T19 = T7 ^ T18, T20 = T1 ^ T19, T21 = U6 ^ U7,
                   T22 = T7 ^ T21, T23 = T2 ^ T22, T24 = T2 ^ T10,
                   T25 = T20 ^ T17, T26 = T3 ^ T16, T27 = T1 ^ T12;
    const uint32_t M1 = T13 & T6, M2 = T23 & T8, M3 = T14 ^ M1, M4 = T19 & U7,
                   M5 = M4 ^ M1, M6 = T3 & T16, M7 = T22 & T9, M8 = T26 ^ M6,
                   M9 = T20 & T17, M10 = M9 ^ M6, M11 = T1 & T15,
                   M12 = T4 & T27, M13 = M12 ^ M11, M14 = T2 & T10,
                   M15 = M14 ^ M11, M16 = M3 ^ M2, M17 = M5 ^ T24,
                   M18 = M8 ^ M7, M19 = M10 ^ M15, M20 = M16 ^ M13,
                   M21 = M17 ^ M15, M22 = M18 ^ M13, M23 = M19 ^ T25,
                   M24 = M22 ^ M23, M25 = M22 & M20, M26 = M21 ^ M25,
                   M27 = M20 ^ M21, M28 = M23 ^ M25, M29 = M28 & M27,
                   M30 = M26 & M24, M31 = M20 & M23, M32 = M27 & M31,
                   M33 = M27 ^ M25, M34 = M21 & M22, M35 = M24 & M34,
                   M36 = M24 ^ M25, M37 = M21 ^ M29, M38 = M32 ^ M33,
                   M39 = M23 ^ M30, M40 = M35 ^ M36, M41 = M38 ^ M40,
                   M42 = M37 ^ M39, M43 = M37 ^ M38, M44 = M39 ^ M40,
                   M45 = M42 ^ M41, M46 = M44 & T6, M47 = M40 & T8,
                   M48 = M39 & U7, M49 = M43 & T16, M50 = M38 & T9,
                   M51 = M37 & T17, M52 = M42 & T15, M53 = M45 & T27,
                   M54 = M41 & T10, M55 = M44 & T13, M56 = M40 & T23,
                   M57 = M39 & T19, M58 = M43 & T3, M59 = M38 & T22,
                   M60 = M37 & T20, M61 = M42 & T1, M62 = M45 & T4,
                   M63 = M41 & T2;
    const uint32_t L0 = M61 ^ M62, L1 = M50 ^ M56, L2 = M46 ^ M48,
                   L3 = M47 ^ M55, L4 = M54 ^ M58, L5 = M49 ^ M61,
                   L6 = M62 ^ L5, L7 = M46 ^ L3, L8 = M51 ^ M59,
                   L9 = M52 ^ M53, L10 = M53 ^ L4, L11 = M60 ^ L2,
                   L12 = M48 ^ M51, L13 = M50 ^ L0, L14 = M52 ^ M61,
                   L15 = M55 ^ L1, L16 = M56 ^ L0, L17 = M57 ^ L1,
                   L18 = M58 ^ L8, L19 = M63 ^ L4, L20 = L0 ^ L1,
                   L21 = L1 ^ L7, L22 = L3 ^ L12, L23 = L18 ^ L2,
                   L24 = L15 ^ L9, L25 = L6 ^ L10, L26 = L7 ^ L9,
                   L27 = L8 ^ L10, L28 = L11 ^ L14, L29 = L11 ^ L17;
    x[7] = L6 ^ L24;
    x[6] = ~(L16 ^ L26);
    x[5] = ~(L19 ^ L28);
    x[4] = L6 ^ L21;
    x[3] = L20 ^ L22;
    x[2] = L25 ^ L29;
    x[1] = ~(L13 ^ L27);
    x[0] = ~(L6 ^ L23);
}

// state R[p * 8 + b]; mask table km[r * 128 + p * 8 + b] = 0 or ~0
template <bool LAST>
HD void bs_round(uint32_t *R, const uint32_t *km)
{
#pragma unroll
    for (int p = 0; p < 16; p++)
        bs_sbox(R + 8 * p);
    uint32_t S[128];
    // ShiftRows: new[row + 4c] = old[row + 4((c + row) & 3)]
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int row = 0; row < 4; row++)
#pragma unroll
            for (int b = 0; b < 8; b++)
                S[8 * (row + 4 * c) + b] = R[8 * (row + 4 * ((c + row) & 3)) + b];
    if (!LAST) {
        // MixColumns: out_i = a_i ^ all ^ xtime(a_i ^ a_(i+1))
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t *a = S + 32 * c;
            uint32_t t[4][8], all[8];
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int b = 0; b < 8; b++)
                    t[i][b] = a[8 * i + b] ^ a[8 * ((i + 1) & 3) + b];
#pragma unroll
            for (int b = 0; b < 8; b++)
                all[b] = t[0][b] ^ t[2][b];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t *u = t[i];
                const uint32_t xt[8] = { u[7], u[0] ^ u[7], u[1], u[2] ^ u[7],
                                         u[3] ^ u[7], u[4], u[5], u[6] };
#pragma unroll
                for (int b = 0; b < 8; b++)
                    R[32 * c + 8 * i + b] = a[8 * i + b] ^ all[b] ^ xt[b] ^ km[32 * c + 8 * i + b];
            }
        }
    } else {
#pragma unroll
        for (int q = 0; q < 128; q++)
            R[q] = S[q] ^ km[q];
    }
}

// 32 x 32 bit transpose: A[q] bit k  ->  A[k] bit q
HD void transpose32(uint32_t *A)
{
    uint32_t m = 0x0000ffffu;
#pragma unroll
    for (int j = 16; j != 0; j >>= 1, m ^= (m << j)) {
#pragma unroll
        for (int k = 0; k < 32; k = (k + j + 1) & ~j) {
            const uint32_t t = ((A[k] >> j) ^ A[k + j]) & m;
            A[k] ^= t << j;
            A[k + j] ^= t;
        }
    }
}

// 32 keystream blocks m*32 .. m*32+31 of one lane; iv = 14 bytes as
// 4 LE words (bytes 14, 15 zero), out: ks[k][4] (LE words of block k)
HD void bs_ctr32(const uint32_t iv[4], uint32_t m, const uint32_t *km,
                 uint32_t *ks, uint32_t &acc, bool store)
{
    uint32_t R[128];
#pragma unroll
    for (int p = 0; p < 16; p++) {
        const uint32_t byte = (iv[p >> 2] >> (8 * (p & 3))) & 0xffu;
#pragma unroll
        for (int b = 0; b < 8; b++)
            R[8 * p + b] = ((byte >> b) & 1) ? ~0u : 0u;
    }
    // byte 15 = 32 m + k (m < 8), byte 14 = 0
    const uint32_t kpat[5] = { 0xaaaaaaaau, 0xccccccccu, 0xf0f0f0f0u,
                               0xff00ff00u, 0xffff0000u };
#pragma unroll
    for (int b = 0; b < 8; b++)
        R[120 + b] = b < 5 ? kpat[b < 5 ? b : 0] : (((m >> (b - 5)) & 1) ? ~0u : 0u);
#pragma unroll
    for (int q = 0; q < 128; q++)
        R[q] ^= km[q];
#if BS_ROLLED   // the round loop rolled (code size) or unrolled (no moves)
#pragma unroll 1
#else
#pragma unroll
#endif
    for (int r = 1; r < 10; r++)
        bs_round<false>(R, km + 128 * r);
    bs_round<true>(R, km + 1280);
    // column c: R[32c .. 32c+31] = bits (row, b) -> word bit 8 row + b
#pragma unroll
    for (int c = 0; c < 4; c++) {
        transpose32(R + 32 * c);
#pragma unroll
        for (int k = 0; k < 32; k++) {
            if (store)
                ks[4 * k + c] = R[32 * c + k];
            acc ^= R[32 * c + k];
        }
    }
}

// ---- kernels ---------------------------------------------------------------
#ifndef NBATCH
#define NBATCH 3   // 96 blocks per lane (a 1400-byte payload needs 88)
#endif

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_bs(const uint32_t *__restrict__ iv, const uint32_t *__restrict__ km,
                                             uint32_t *__restrict__ ks, uint32_t *__restrict__ acc_out,
                                             uint32_t n, int store)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    uint32_t v[4] = { iv[4 * i], iv[4 * i + 1], iv[4 * i + 2], iv[4 * i + 3] };
    uint32_t acc = 0;
    for (uint32_t m = 0; m < NBATCH; m++)
        bs_ctr32(v, m, km, ks + ((size_t)i * 32 * NBATCH + 32 * m) * 4, acc,
                 store != 0);
    acc_out[i] = acc;
}

// T-table form: T0..T3 (Te tables, LE words), 32 copies, lane reads copy
// lane & 31; one v_perm per lookup address
__global__ __launch_bounds__(512) void k_tt(const uint32_t *iv, const uint32_t *rkw,
                                             const uint32_t *te, uint32_t *ks,
                                             uint32_t *acc_out, uint32_t n, int store)
{
    __shared__ uint32_t s_t[4 * 256 * 32];
    for (int q = threadIdx.x; q < 4 * 256 * 32; q += blockDim.x)
        s_t[q] = te[q >> 5];   // entry (t, b) copy c at (t*256 + b)*32 + c
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t c4 = (threadIdx.x & 31) * 4;
    const char *lds = (const char *)s_t;
#define TL(t, w, sh) (*(const uint32_t *)(lds + (t) * 32768 + (((w) >> (sh)) & 0xff) * 128 + c4))
    uint32_t acc = 0;
    for (uint32_t j = 0; j < 32 * NBATCH; j++) {
        uint32_t s0 = iv[4 * i] ^ rkw[0], s1 = iv[4 * i + 1] ^ rkw[1],
                 s2 = iv[4 * i + 2] ^ rkw[2],
                 s3 = (iv[4 * i + 3] | (j << 24)) ^ rkw[3];
        for (int r = 1; r < 10; r++) {
            const uint32_t *k = rkw + 4 * r;
            const uint32_t t0 = TL(0, s0, 0) ^ TL(1, s1, 8) ^ TL(2, s2, 16) ^ TL(3, s3, 24) ^ k[0];
            const uint32_t t1 = TL(0, s1, 0) ^ TL(1, s2, 8) ^ TL(2, s3, 16) ^ TL(3, s0, 24) ^ k[1];
            const uint32_t t2 = TL(0, s2, 0) ^ TL(1, s3, 8) ^ TL(2, s0, 16) ^ TL(3, s1, 24) ^ k[2];
            const uint32_t t3 = TL(0, s3, 0) ^ TL(1, s0, 8) ^ TL(2, s1, 16) ^ TL(3, s2, 24) ^ k[3];
            s0 = t0; s1 = t1; s2 = t2; s3 = t3;
        }
        // last round: S-box bytes from T-table entries (T2 holds S at byte 0..)
        const uint32_t *k = rkw + 40;
#define SB(w, sh, byte) ((TL(((byte) + 2) & 3, w, sh) >> (8 * (byte))) & 0xff)
        const uint32_t o0 = (SB(s0, 0, 0) | SB(s1, 8, 1) << 8 | SB(s2, 16, 2) << 16 | SB(s3, 24, 3) << 24) ^ k[0];
        const uint32_t o1 = (SB(s1, 0, 0) | SB(s2, 8, 1) << 8 | SB(s3, 16, 2) << 16 | SB(s0, 24, 3) << 24) ^ k[1];
        const uint32_t o2 = (SB(s2, 0, 0) | SB(s3, 8, 1) << 8 | SB(s0, 16, 2) << 16 | SB(s1, 24, 3) << 24) ^ k[2];
        const uint32_t o3 = (SB(s3, 0, 0) | SB(s0, 8, 1) << 8 | SB(s1, 16, 2) << 16 | SB(s2, 24, 3) << 24) ^ k[3];
        if (store) {
            uint32_t *o = ks + ((size_t)i * 32 * NBATCH + j) * 4;
            o[0] = o0; o[1] = o1; o[2] = o2; o[3] = o3;
        }
        acc ^= o0 ^ o1 ^ o2 ^ o3;
    }
    acc_out[i] = acc;
}

// ---- host ---------------------------------------------------------------
int main(int argc, char **argv)
{
    make_sbox();
    uint8_t key[16], rk[11][16];
    for (int i = 0; i < 16; i++)
        key[i] = (uint8_t)(i * 37 + 11);
    expand(key, rk);
    // FIPS-197 C.1 sanity: AES-128(000102..0f, 00112233..ff)
    {
        uint8_t k2[16], r2[11][16], pt[16], ct[16];
        for (int i = 0; i < 16; i++) {
            k2[i] = (uint8_t)i;
            pt[i] = (uint8_t)(0x11 * i);
        }
        expand(k2, r2);
        h_aes(r2, pt, ct);
        const uint8_t want[16] = { 0x69, 0xc4, 0xe0, 0xd8, 0x6a, 0x7b, 0x04, 0x30,
                                   0xd8, 0xcd, 0xb7, 0x80, 0x70, 0xb4, 0xc5, 0x5a };
        if (memcmp(ct, want, 16)) {
            printf("host AES wrong\n");
            return 1;
        }
    }
    // masks
    static uint32_t km[11 * 128];
    for (int r = 0; r < 11; r++)
        for (int p = 0; p < 16; p++)
            for (int b = 0; b < 8; b++)
                km[r * 128 + p * 8 + b] = ((rk[r][p] >> b) & 1) ? ~0u : 0u;
    // Te tables, LE words: Te0[b] bytes (2S, S, S, 3S), Te_t = rotl(Te0, 8t)
    static uint32_t te[4 * 256];
    for (int b = 0; b < 256; b++) {
        const uint8_t s = h_sbox[b];
        const uint32_t w = (uint32_t)gmul(s, 2) | (uint32_t)s << 8 |
                           (uint32_t)s << 16 | (uint32_t)gmul(s, 3) << 24;
        for (int t = 0; t < 4; t++)
            te[t * 256 + b] = t ? (w << (8 * t)) | (w >> (32 - 8 * t)) : w;
    }
    static uint32_t rkw[44];
    memcpy(rkw, rk, sizeof rk);
    // host check of the bitsliced form on 3 lanes
    const int NB = 32 * NBATCH;
    for (int lane = 0; lane < 3; lane++) {
        uint32_t iv[4] = { 0x01020304u * (lane + 1), 0xdeadbeefu ^ lane,
                           0x55aa55aau + lane, 0x0000c0deu + lane };
        static uint32_t ks[32][4];
        uint32_t acc = 0;
        for (uint32_t m = 0; m < NBATCH; m++) {
            bs_ctr32(iv, m, km, &ks[0][0], acc, true);
            for (int k = 0; k < 32; k++) {
                uint8_t in[16], want[16];
                memcpy(in, iv, 16);
                in[14] = 0;
                in[15] = (uint8_t)(32 * m + k);
                h_aes(rk, in, want);
                if (memcmp(want, ks[k], 16)) {
                    printf("bitsliced mismatch lane %d block %u\n", lane, 32 * m + k);
                    return 1;
                }
            }
        }
    }
    printf("host: bitsliced AES-128 CTR matches FIPS-197 AES (3 lanes x %d blocks)\n", NB);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return 0;

    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
    uint32_t *d_iv, *d_km, *d_te, *d_rk, *d_ks, *d_acc;
    const uint32_t nchk = 4096;
    if (hipMalloc(&d_iv, (size_t)n * 16) || hipMalloc(&d_km, sizeof km) ||
        hipMalloc(&d_te, sizeof te) || hipMalloc(&d_rk, sizeof rkw) ||
        hipMalloc(&d_ks, (size_t)nchk * NB * 16) || hipMalloc(&d_acc, (size_t)n * 4))
        return 1;
    uint32_t *h_iv = (uint32_t *)malloc((size_t)n * 16);
    for (uint32_t i = 0; i < n; i++) {
        h_iv[4 * i] = i * 2654435761u;
        h_iv[4 * i + 1] = i ^ 0x9e3779b9u;
        h_iv[4 * i + 2] = 0x12345678u + i;
        h_iv[4 * i + 3] = (i * 7) & 0xffffu;   // bytes 14, 15 zero
    }
    (void)hipMemcpy(d_iv, h_iv, (size_t)n * 16, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_km, km, sizeof km, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_te, te, sizeof te, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_rk, rkw, sizeof rkw, hipMemcpyHostToDevice);
    // device check: both kernels on nchk lanes, every block vs host AES
    uint32_t *h_ks = (uint32_t *)malloc((size_t)nchk * NB * 16);
    for (int kern = 0; kern < 2; kern++) {
        if (kern == 0)
            hipLaunchKernelGGL(k_bs, dim3(nchk / 256), dim3(256), 0, 0, d_iv, d_km, d_ks, d_acc, nchk, 1);
        else
            hipLaunchKernelGGL(k_tt, dim3(nchk / 512), dim3(512), 0, 0, d_iv, d_rk, d_te, d_ks, d_acc, nchk, 1);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("kernel %d failed\n", kern);
            return 1;
        }
        (void)hipMemcpy(h_ks, d_ks, (size_t)nchk * NB * 16, hipMemcpyDeviceToHost);
        for (uint32_t i = 0; i < nchk; i += 97)
            for (int j = 0; j < NB; j++) {
                uint8_t in[16], want[16];
                memcpy(in, h_iv + 4 * i, 16);
                in[14] = 0;
                in[15] = (uint8_t)j;
                h_aes(rk, in, want);
                if (memcmp(want, h_ks + ((size_t)i * NB + j) * 4, 16)) {
                    printf("%s mismatch lane %u block %d\n", kern ? "k_tt" : "k_bs", i, j);
                    return 1;
                }
            }
        printf("device: %s bit-exact (sampled lanes x %d blocks)\n", kern ? "k_tt" : "k_bs", NB);
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int kern = 0; kern < 2; kern++) {
        float best = 1e30f;
        for (int rep = 0; rep < 4; rep++) {
            (void)hipEventRecord(e0);
            if (kern == 0)
                hipLaunchKernelGGL(k_bs, dim3(n / 256), dim3(256), 0, 0, d_iv, d_km, d_ks, d_acc, n, 0);
            else
                hipLaunchKernelGGL(k_tt, dim3(n / 512), dim3(512), 0, 0, d_iv, d_rk, d_te, d_ks, d_acc, n, 0);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep && ms < best)
                best = ms;
        }
        printf("%s: %u lanes x %d blocks: %.3f ms, %.3f ns per block-lane per CU "
               "(%.1f Gblock/s)\n", kern ? "k_tt (T-tables, LDS)" : "k_bs (bitsliced, VALU)",
               n, NB, best, best * 1e6 * 256 / ((double)n * NB), (double)n * NB / best / 1e6);
    }
    return 0;
}
