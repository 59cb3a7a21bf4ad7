/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, called by or shipped
 * with the product path (prysm_amd/).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load liboracle.so, and only as the
 * checker / the timed CPU baseline.
 *
 * CPU restatement of the reference digest:
 *   shared/hashutil/hash.go:11-25  Hash(data) = sha3.NewLegacyKeccak256()
 *     .Write(data).Sum()   (golang.org/x/crypto/sha3 @ b8fe1690c613,
 *     WORKSPACE:542-546; not vendored in the reference).
 * Legacy Keccak-256 = Keccak[c=512] with the ORIGINAL (pre-FIPS) padding:
 *   rate 136 bytes, pad byte 0x01 after the message, 0x80 OR-ed into the
 *   last byte of the final block, 24 rounds of Keccak-f[1600] (FIPS 202 §3),
 *   output = first 32 bytes of the state, lanes little-endian.
 * Parity pins: shared/hashutil/hash_test.go:13-31 (three KATs), checked by
 * tests/test_oracle.py; with pad 0x06 the same permutation reproduces
 * Python's hashlib.sha3_256 (FIPS 202), which pins the permutation itself.
 */
#include <stdint.h>
#include <string.h>
#include "oracle.h"

static const uint64_t RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL,
    0x8000000080008000ULL, 0x000000000000808BULL, 0x0000000080000001ULL,
    0x8000000080008081ULL, 0x8000000000008009ULL, 0x000000000000008AULL,
    0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL,
    0x8000000000008003ULL, 0x8000000000008002ULL, 0x8000000000000080ULL,
    0x000000000000800AULL, 0x800000008000000AULL, 0x8000000080008081ULL,
    0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

/* rho offsets r[x][y], lane index x + 5y (FIPS 202 Table 2) */
static const int RHO[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                            25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};

static inline uint64_t rotl(uint64_t v, int n) {
    return n ? (v << n) | (v >> (64 - n)) : v;
}

void or_keccak_f1600(uint64_t A[25]) {
    for (int round = 0; round < 24; ++round) {
        uint64_t C[5], D[5], B[25];
        for (int x = 0; x < 5; ++x)
            C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
        for (int x = 0; x < 5; ++x)
            D[x] = C[(x + 4) % 5] ^ rotl(C[(x + 1) % 5], 1);
        for (int i = 0; i < 25; ++i) A[i] ^= D[i % 5];
        /* rho + pi: B[y][2x+3y] = rot(A[x][y], r[x][y]) */
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y)
                B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl(A[x + 5 * y], RHO[x + 5 * y]);
        /* chi */
        for (int y = 0; y < 5; ++y)
            for (int x = 0; x < 5; ++x)
                A[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
        /* iota */
        A[0] ^= RC[round];
    }
}

static inline uint64_t load_le64(const uint8_t* p) {
#if defined(__BYTE_ORDER__) && __BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__
    uint64_t v;
    memcpy(&v, p, 8);
#else
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
#endif
    return v;
}

/* The permutation every sponge below runs: the loop form above (default) or
 * the unrolled x/crypto-shaped one (keccak_fast.c) for the CPU baselines.
 * Process-wide; set it before starting a computation, not during one. */
static void (*g_perm)(uint64_t A[25]) = or_keccak_f1600;

int or_set_fast_permutation(int on) {
    int was = g_perm == or_keccak_f1600_unrolled;
    g_perm = on ? or_keccak_f1600_unrolled : or_keccak_f1600;
    return was;
}

/* Sponge over a message with a selectable domain pad byte (0x01 legacy
 * Keccak, 0x06 FIPS SHA3).  rate in bytes, out_len <= rate. */
void or_sponge(const uint8_t* in, uint64_t len, uint8_t pad, uint32_t rate,
               uint8_t* out, uint32_t out_len) {
    uint64_t A[25];
    memset(A, 0, sizeof A);
    uint8_t block[200];
    while (len >= rate) {
        for (uint32_t i = 0; i < rate / 8; ++i) A[i] ^= load_le64(in + 8 * i);
        g_perm(A);
        in += rate;
        len -= rate;
    }
    memset(block, 0, rate);
    memcpy(block, in, len);
    block[len] ^= pad;
    block[rate - 1] ^= 0x80;
    for (uint32_t i = 0; i < rate / 8; ++i) A[i] ^= load_le64(block + 8 * i);
    g_perm(A);
    for (uint32_t i = 0; i < out_len; ++i) out[i] = (uint8_t)(A[i / 8] >> (8 * (i % 8)));
}

/* hashutil.Hash (shared/hashutil/hash.go:11-25) */
void or_keccak256(const uint8_t* in, uint64_t len, uint8_t out[32]) {
    or_sponge(in, len, 0x01, 136, out, 32);
}

/* FIPS SHA3-256, used only to pin the permutation against hashlib. */
void or_sha3_256(const uint8_t* in, uint64_t len, uint8_t out[32]) {
    or_sponge(in, len, 0x06, 136, out, 32);
}

/* n messages of msg_len bytes each, contiguous; out n*32.  nthreads<=1 is the
 * single-goroutine reference shape; >1 splits the batch with OpenMP. */
void or_keccak256_batch(const uint8_t* in, uint64_t n, uint32_t msg_len, uint8_t* out,
                        int nthreads) {
    if (nthreads <= 1) {
        for (uint64_t i = 0; i < n; ++i) or_keccak256(in + i * msg_len, msg_len, out + 32 * i);
        return;
    }
#pragma omp parallel for num_threads(nthreads) schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i)
        or_keccak256(in + (uint64_t)i * msg_len, msg_len, out + 32 * (uint64_t)i);
}

/* n variable-length messages: message i = in[offs[i] .. offs[i+1]). */
void or_keccak256_var(const uint8_t* in, const uint64_t* offs, uint64_t n, uint8_t* out) {
    for (uint64_t i = 0; i < n; ++i) or_keccak256(in + offs[i], offs[i + 1] - offs[i], out + 32 * i);
}
