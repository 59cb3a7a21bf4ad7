/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, called by or shipped
 * with the product path (prysm_amd/).  Only tests/ and bench.py's
 * cpu_baseline leg select it (or_set_fast_permutation).
 *
 * The same Keccak-f[1600] as or_keccak_f1600 (keccak_ref.c), written in the
 * shape of the permutation the reference actually runs: golang.org/x/crypto/
 * sha3 @ b8fe1690c613 (WORKSPACE:542-546; shared/hashutil/hash.go:14 calls
 * sha3.NewLegacyKeccak256), whose keccakF1600 keeps the 25 lanes in locals
 * and unrolls the rounds (keccakf.go; keccakf_amd64.s is the same dataflow
 * with lane complementing, which only saves NOTs where the ISA has no
 * and-not — this file is compiled for x86-64-v3, whose ANDN does ~b & c in
 * one instruction).  Two rounds per loop iteration ping-pong between the a*
 * and e* locals, so pi is pure renaming and no lane is copied.
 *
 * Used as the CPU baseline's permutation (bench.py, tools/bench_configs.py);
 * pinned against or_keccak_f1600 and hashlib.sha3_256 by tests/test_oracle.py.
 */
#include <stdint.h>
#include "oracle.h"

#define ROL(v, n) (((v) << (n)) | ((v) >> (64 - (n))))

static const uint64_t RCF[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL,
    0x8000000080008000ULL, 0x000000000000808BULL, 0x0000000080000001ULL,
    0x8000000080008081ULL, 0x8000000000008009ULL, 0x000000000000008AULL,
    0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL,
    0x8000000000008003ULL, 0x8000000000008002ULL, 0x8000000000000080ULL,
    0x000000000000800AULL, 0x800000008000000AULL, 0x8000000080008081ULL,
    0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

/* One round a -> e (lane index x + 5y): theta, rho + pi (B row y of the
 * output takes lane (x', y') with y = 2x' + 3y' mod 5), chi, iota. */
#define KF_ROUND(a, e, rc) do { \
    C0 = a##0 ^ a##5 ^ a##10 ^ a##15 ^ a##20; \
    C1 = a##1 ^ a##6 ^ a##11 ^ a##16 ^ a##21; \
    C2 = a##2 ^ a##7 ^ a##12 ^ a##17 ^ a##22; \
    C3 = a##3 ^ a##8 ^ a##13 ^ a##18 ^ a##23; \
    C4 = a##4 ^ a##9 ^ a##14 ^ a##19 ^ a##24; \
    D0 = C4 ^ ROL(C1, 1); \
    D1 = C0 ^ ROL(C2, 1); \
    D2 = C1 ^ ROL(C3, 1); \
    D3 = C2 ^ ROL(C4, 1); \
    D4 = C3 ^ ROL(C0, 1); \
    B0 = a##0 ^ D0; B1 = ROL(a##6 ^ D1, 44); B2 = ROL(a##12 ^ D2, 43); B3 = ROL(a##18 ^ D3, 21); \
    B4 = ROL(a##24 ^ D4, 14); \
    e##0 = B0 ^ (~B1 & B2); e##1 = B1 ^ (~B2 & B3); e##2 = B2 ^ (~B3 & B4); e##3 = B3 ^ (~B4 & B0); \
    e##4 = B4 ^ (~B0 & B1); \
    B0 = ROL(a##3 ^ D3, 28); B1 = ROL(a##9 ^ D4, 20); B2 = ROL(a##10 ^ D0, 3); B3 = ROL(a##16 ^ D1, 45); \
    B4 = ROL(a##22 ^ D2, 61); \
    e##5 = B0 ^ (~B1 & B2); e##6 = B1 ^ (~B2 & B3); e##7 = B2 ^ (~B3 & B4); e##8 = B3 ^ (~B4 & B0); \
    e##9 = B4 ^ (~B0 & B1); \
    B0 = ROL(a##1 ^ D1, 1); B1 = ROL(a##7 ^ D2, 6); B2 = ROL(a##13 ^ D3, 25); B3 = ROL(a##19 ^ D4, 8); \
    B4 = ROL(a##20 ^ D0, 18); \
    e##10 = B0 ^ (~B1 & B2); e##11 = B1 ^ (~B2 & B3); e##12 = B2 ^ (~B3 & B4); e##13 = B3 ^ (~B4 & B0); \
    e##14 = B4 ^ (~B0 & B1); \
    B0 = ROL(a##4 ^ D4, 27); B1 = ROL(a##5 ^ D0, 36); B2 = ROL(a##11 ^ D1, 10); B3 = ROL(a##17 ^ D2, 15); \
    B4 = ROL(a##23 ^ D3, 56); \
    e##15 = B0 ^ (~B1 & B2); e##16 = B1 ^ (~B2 & B3); e##17 = B2 ^ (~B3 & B4); e##18 = B3 ^ (~B4 & B0); \
    e##19 = B4 ^ (~B0 & B1); \
    B0 = ROL(a##2 ^ D2, 62); B1 = ROL(a##8 ^ D3, 55); B2 = ROL(a##14 ^ D4, 39); B3 = ROL(a##15 ^ D0, 41); \
    B4 = ROL(a##21 ^ D1, 2); \
    e##20 = B0 ^ (~B1 & B2); e##21 = B1 ^ (~B2 & B3); e##22 = B2 ^ (~B3 & B4); e##23 = B3 ^ (~B4 & B0); \
    e##24 = B4 ^ (~B0 & B1); \
    e##0 ^= (rc); \
} while (0)

#define LANES(p) p##0, p##1, p##2, p##3, p##4, p##5, p##6, p##7, p##8, p##9, p##10, p##11, p##12, \
                 p##13, p##14, p##15, p##16, p##17, p##18, p##19, p##20, p##21, p##22, p##23, p##24

void or_keccak_f1600_unrolled(uint64_t A[25]) {
    uint64_t LANES(a), LANES(e);
    uint64_t C0, C1, C2, C3, C4, D0, D1, D2, D3, D4, B0, B1, B2, B3, B4;
    a0 = A[0]; a1 = A[1]; a2 = A[2]; a3 = A[3]; a4 = A[4];
    a5 = A[5]; a6 = A[6]; a7 = A[7]; a8 = A[8]; a9 = A[9];
    a10 = A[10]; a11 = A[11]; a12 = A[12]; a13 = A[13]; a14 = A[14];
    a15 = A[15]; a16 = A[16]; a17 = A[17]; a18 = A[18]; a19 = A[19];
    a20 = A[20]; a21 = A[21]; a22 = A[22]; a23 = A[23]; a24 = A[24];
    for (int r = 0; r < 24; r += 4) {
        KF_ROUND(a, e, RCF[r]);
        KF_ROUND(e, a, RCF[r + 1]);
        KF_ROUND(a, e, RCF[r + 2]);
        KF_ROUND(e, a, RCF[r + 3]);
    }
    A[0] = a0; A[1] = a1; A[2] = a2; A[3] = a3; A[4] = a4;
    A[5] = a5; A[6] = a6; A[7] = a7; A[8] = a8; A[9] = a9;
    A[10] = a10; A[11] = a11; A[12] = a12; A[13] = a13; A[14] = a14;
    A[15] = a15; A[16] = a16; A[17] = a17; A[18] = a18; A[19] = a19;
    A[20] = a20; A[21] = a21; A[22] = a22; A[23] = a23; A[24] = a24;
}
