/*
 * C-ABI harness: consumes include/prysm_merkle.h the way the cgo package
 * gpu/merkle would (C99, no C++ or torch), links libprysm_merkle.so and calls
 * the host-buffer entry points from NTHREADS pthreads at once.  Every thread
 * checks its results against the committed fixture values passed on the
 * command line (tests/golden/c_abi_fixture.json, made by
 * tests/golden/make_c_abi_fixture.py with the CPU oracle), and checks that
 * failures come back through the failing call's own mk_call context.
 *
 *   harness <threads> <rounds> <merkle_hex x8> <batch_hex x8> <trie_root_hex> <branch_hex> <many_hex x3>
 *   MK_INJECT_EHIP=1 harness inject
 *   harness cgo <m0> <m1> <m2> <m5> <m10x16> <m10x32> <t0> <tz4> <t1x6>
 *
 * `cgo` replays the call sequences of INTEGRATION.md's Go wrappers exactly,
 * including the pointers cgo passes for empty slices (ptr(b) == NULL when
 * len(b) == 0) and every early-return branch of the Go code, against the
 * reference's own vectors (shared/ssz/hash_test.go:80-90,151-178) and oracle
 * fixtures (tests/golden/c_abi_fixture.json "cgo").
 *
 * `inject` runs with the library's failure-injection hook on: every compute
 * call must come back with MK_EHIP and the detail in its own mk_call (the
 * cgo package maps it to an error; only MK_ENODEV may select a CPU path).
 *
 * Inputs are SplitMix64 streams, identical to oracle/merkle_ref.c.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "prysm_merkle.h"

#define NT_MAX 8
#define SEED_BASE 0x5EED000000000700ull

static uint64_t splitmix(uint64_t seed, uint64_t k) {
    uint64_t z = seed + k * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* bytes [8*word0, 8*word0 + n) of the stream */
static void fill(uint8_t* dst, size_t n, uint64_t seed, uint64_t word0) {
    for (size_t i = 0; i < n; ++i) dst[i] = (uint8_t)(splitmix(seed, word0 + i / 8) >> (8 * (i % 8)));
}

static void hex(const uint8_t* b, char* out) {
    for (int i = 0; i < 32; ++i) sprintf(out + 2 * i, "%02x", b[i]);
}

static const char* g_merkle[NT_MAX];
static const char* g_batch[NT_MAX];
static const char* g_trie_root;
static const char* g_branch;
static const char* g_many[3];
static int g_rounds = 1;

struct result {
    int failures;
    char msg[512];
};

#define CHECK(cond, ...)                                                     \
    do {                                                                     \
        if (!(cond)) {                                                       \
            r->failures++;                                                   \
            snprintf(r->msg, sizeof r->msg, __VA_ARGS__);                    \
            return;                                                          \
        }                                                                    \
    } while (0)

static int same(const uint8_t* got, const char* want) {
    char h[65];
    hex(got, h);
    return strcmp(h, want) == 0;
}

static void run_once(int t, struct result* r) {
    mk_call call;
    uint8_t out[32];
    call.device = -1;

    /* ssz.merkleHash of 100003 + t items of 32 B */
    const uint64_t n = 100003 + (uint64_t)t;
    uint8_t* items = malloc(n * 32);
    fill(items, n * 32, SEED_BASE + (uint64_t)t, 0);
    int rc = mk_ssz_merkle_hash(&call, items, n, 32, out);
    free(items);
    CHECK(rc == MK_OK && call.code == MK_OK && call.err[0] == 0, "merkle rc %d: %s", rc, call.err);
    CHECK(same(out, g_merkle[t]), "thread %d: merkle root mismatch", t);

    /* hashutil.Hash batch of 1000 x 64 B, then Hash of the 32000 digest bytes */
    uint8_t* msgs = malloc(1000 * 64);
    uint8_t* dig = malloc(1000 * 32);
    fill(msgs, 1000 * 64, SEED_BASE + 0x100 + (uint64_t)t, 0);
    rc = mk_hash_batch(&call, msgs, 1000, 64, dig);
    if (rc == MK_OK) rc = mk_hash(&call, dig, 1000 * 32, out);
    free(msgs);
    free(dig);
    CHECK(rc == MK_OK, "hash rc %d: %s", rc, call.err);
    CHECK(same(out, g_batch[t]), "thread %d: hash batch mismatch", t);

    /* deposit trie handle: Root() before every UpdateDepositTrie (powchain saveInTrie) */
    mk_trie* trie = NULL;
    rc = mk_deposit_trie_new(&call, 32, 0, &trie);
    CHECK(rc == MK_OK && trie, "trie_new rc %d: %s", rc, call.err);
    uint8_t dep[280];
    uint64_t offs[2] = {0, 280};
    uint8_t* before = malloc(300 * 32); /* Root() read before each deposit */
    uint8_t* all = malloc(300 * 280);
    uint64_t* alloffs = malloc(301 * sizeof(uint64_t));
    for (int i = 0; i < 300 && rc == MK_OK; ++i) {
        rc = mk_deposit_trie_root(&call, trie, before + 32 * i);
        fill(dep, 280, SEED_BASE + 0x200, 35 * (uint64_t)i);
        memcpy(all + 280 * i, dep, 280);
        alloffs[i] = 280 * (uint64_t)i;
        if (rc == MK_OK) rc = mk_deposit_trie_append(&call, trie, dep, offs, 1);
    }
    alloffs[300] = 300 * 280;
    uint8_t branch[32 * 32];
    if (rc == MK_OK) rc = mk_deposit_trie_root(&call, trie, out);
    int root_ok = rc == MK_OK && same(out, g_trie_root);
    if (rc == MK_OK) rc = mk_deposit_trie_branch(&call, trie, 7, branch);
    if (rc == MK_OK) rc = mk_hash(&call, branch, sizeof branch, out);
    CHECK(mk_deposit_trie_count(trie) == 300, "trie count %llu", (unsigned long long)mk_deposit_trie_count(trie));
    mk_deposit_trie_free(trie);

    /* the same 300 logs through the batched per-log check, log 150 carrying a
     * wrong root: the reference skips it, and every later log then fails its
     * check too (their roots assume deposit 150) */
    mk_trie* t2 = NULL;
    int rc2 = mk_deposit_trie_new(&call, 32, 0, &t2);
    uint8_t acc[300];
    uint8_t root2[32];
    memset(before + 32 * 150, 0xAB, 32);
    if (rc2 == MK_OK) rc2 = mk_deposit_trie_save_logs(&call, t2, all, alloffs, 300, before, acc);
    if (rc2 == MK_OK) rc2 = mk_deposit_trie_root(&call, t2, root2);
    CHECK(rc2 == MK_OK, "save_logs rc %d: %s", rc2, call.err);
    int acc_ok = 1;
    for (int i = 0; i < 300; ++i) acc_ok &= acc[i] == (i < 150 ? 1 : 0);
    CHECK(acc_ok, "thread %d: save_logs accept flags", t);
    CHECK(mk_deposit_trie_count(t2) == 150, "thread %d: save_logs count %llu", t,
          (unsigned long long)mk_deposit_trie_count(t2));
    {
        /* Root() after the 150 accepted deposits = the root read before deposit 150 in the first loop */
        mk_trie* t3 = NULL;
        uint8_t r3[32];
        int rc3 = mk_deposit_trie_new(&call, 32, 0, &t3);
        if (rc3 == MK_OK) rc3 = mk_deposit_trie_append(&call, t3, all, alloffs, 150);
        if (rc3 == MK_OK) rc3 = mk_deposit_trie_root(&call, t3, r3);
        CHECK(rc3 == MK_OK && memcmp(r3, root2, 32) == 0, "thread %d: save_logs root", t);
        mk_deposit_trie_free(t3);
    }
    mk_deposit_trie_free(t2);
    free(before);
    free(all);
    free(alloffs);
    CHECK(rc == MK_OK, "trie rc %d: %s", rc, call.err);
    CHECK(root_ok, "thread %d: trie root mismatch", t);
    CHECK(same(out, g_branch), "thread %d: branch mismatch", t);

    /* many lists in one call: 5 x 32 B, 1000 x 8 B, empty */
    uint8_t* buf = malloc(160 + 8000);
    fill(buf, 160 + 8000, SEED_BASE + 0x300, 0);
    uint64_t moffs[3] = {0, 160, 0};
    uint64_t mn[3] = {5, 1000, 0};
    uint32_t mil[3] = {32, 8, 32};
    uint8_t roots[3 * 32];
    rc = mk_ssz_merkle_many(&call, buf, moffs, mn, mil, 3, roots);
    free(buf);
    CHECK(rc == MK_OK, "many rc %d: %s", rc, call.err);
    for (int i = 0; i < 3; ++i) CHECK(same(roots + 32 * i, g_many[i]), "thread %d: many root %d mismatch", t, i);

    /* failures travel with the call: item_len 0 (the reference's divide by zero) */
    uint8_t one[64];
    memset(one, 0, sizeof one);
    rc = mk_ssz_merkle_hash(&call, one, 5, 0, out);
    CHECK(rc == MK_EINVAL && call.code == MK_EINVAL && strstr(call.err, "divide by zero"),
          "thread %d: item_len 0 gave rc %d '%s'", t, rc, call.err);
    call.device = 1000 + t; /* a device that does not exist */
    rc = mk_hash_batch(&call, one, 1, 64, out);
    char want[64];
    snprintf(want, sizeof want, "device %d out of range", 1000 + t);
    CHECK(rc == MK_ENODEV && call.code == MK_ENODEV && strstr(call.err, want),
          "thread %d: bad device gave rc %d '%s'", t, rc, call.err);
    call.device = -1;
    rc = mk_hash_batch(&call, one, 1, 64, out);
    CHECK(rc == MK_OK && call.err[0] == 0, "thread %d: error detail leaked into the next call: '%s'", t, call.err);
}

struct arg {
    int t;
    struct result r;
};

static void* worker(void* p) {
    struct arg* a = (struct arg*)p;
    for (int k = 0; k < g_rounds && a->r.failures == 0; ++k) run_once(a->t, &a->r);
    return NULL;
}

/* With MK_INJECT_EHIP=1: a failed HIP launch inside the library surfaces as
 * MK_EHIP with its detail in the failing call's context, for every family. */
static int inject_check(void) {
    mk_call call;
    uint8_t out[32];
    uint8_t* items = calloc(100003, 32);
    int bad = 0;
    struct {
        const char* name;
        int rc;
    } r[3];
    call.device = -1;
    r[0].name = "mk_ssz_merkle_hash";
    r[0].rc = mk_ssz_merkle_hash(&call, items, 100003, 32, out);
    bad |= r[0].rc != MK_EHIP || call.code != MK_EHIP || !strstr(call.err, "injected");
    r[1].name = "mk_hash_batch";
    r[1].rc = mk_hash_batch(&call, items, 1000, 64, items + 64000);
    bad |= r[1].rc != MK_EHIP || call.code != MK_EHIP || !strstr(call.err, "injected");
    r[2].name = "mk_ssz_tree_hash_bytes_list";
    r[2].rc = mk_ssz_tree_hash_bytes_list(&call, items, 100003, 32, out);
    bad |= r[2].rc != MK_EHIP || call.code != MK_EHIP || !strstr(call.err, "injected");
    free(items);
    for (int i = 0; i < 3; ++i) printf("%s -> %d (%s)\n", r[i].name, r[i].rc, mk_strerror(r[i].rc));
    printf(bad ? "FAIL: injected failure not surfaced\n" : "ok: injected failures surfaced as MK_EHIP\n");
    return bad;
}

/* ---- cgo replay (gpu/merkle) --------------------------- */
/* ptr(b): cgo passes NULL for an empty Go slice */
static const uint8_t* gptr(const uint8_t* b, size_t len) { return len ? b : NULL; }

static int g_bad = 0;
static void expect_root(const char* what, int rc, const mk_call* call, const uint8_t* out, const char* want) {
    char h[65];
    hex(out, h);
    int ok = rc == MK_OK && call->code == MK_OK && strcmp(h, want) == 0;
    printf("%-58s rc=%d %s\n", what, rc, ok ? "ok" : "MISMATCH");
    if (!ok) {
        printf("   got %s\n  want %s  (%s)\n", h, want, call->err);
        g_bad = 1;
    }
}
static void expect_rc(const char* what, int rc, const mk_call* call, int want_rc, const char* want_err) {
    int ok = rc == want_rc && call->code == want_rc && (!want_err || strstr(call->err, want_err));
    printf("%-58s rc=%d %s\n", what, rc, ok ? "ok" : "MISMATCH");
    if (!ok) {
        printf("   want rc %d '%s', err '%s'\n", want_rc, want_err ? want_err : "", call->err);
        g_bad = 1;
    }
}

/* merkle.MerkleHashFlat(items, n, itemLen): one mk_ssz_merkle_hash, ptr(items) */
static int go_merkle_hash_flat(mk_call* call, const uint8_t* flat, size_t flat_len, uint64_t n, uint32_t item_len,
                               uint8_t out[32]) {
    call->device = -1;
    return mk_ssz_merkle_hash(call, gptr(flat, flat_len), n, item_len, out);
}

static int cgo_replay(char** want) {
    mk_call call;
    uint8_t out[32];
    memset(&call, 0, sizeof call);
    /* ssz.merkleHash(list) -> MerkleHashFlat(flatten(list), len(list), len(list[0])) */
    expect_root("merkleHash n=0 (flat=nil, itemLen 32)", go_merkle_hash_flat(&call, NULL, 0, 0, 32, out), &call,
                out, want[0]);
    const uint8_t one[2] = {1, 0}; /* []uint16{1}: le16 items */
    expect_root("merkleHash n=1 (2-B item)", go_merkle_hash_flat(&call, one, 2, 1, 2, out), &call, out, want[1]);
    const uint8_t two[4] = {1, 2, 3, 4};
    expect_root("merkleHash n=2 ([0102 0304])", go_merkle_hash_flat(&call, two, 4, 2, 2, out), &call, out, want[2]);
    uint8_t five[5 * 32];
    fill(five, sizeof five, SEED_BASE + 0x400, 0);
    expect_root("merkleHash n=5 (32-B items)", go_merkle_hash_flat(&call, five, sizeof five, 5, 32, out), &call, out,
                want[3]);
    uint8_t ten16[10 * 16], ten32[10 * 32];
    for (int i = 0; i < 10; ++i) {
        memset(ten16 + 16 * i, i + 1, 16);
        memset(ten32 + 32 * i, i + 1, 32);
    }
    expect_root("merkleHash n=10 (16-B items)", go_merkle_hash_flat(&call, ten16, sizeof ten16, 10, 16, out), &call,
                out, want[4]);
    expect_root("merkleHash n=10 (32-B items)", go_merkle_hash_flat(&call, ten32, sizeof ten32, 10, 32, out), &call,
                out, want[5]);
    /* len(list[0]) == 0: every item empty, flat == nil, itemLen 0 (the
     * reference divides by zero; the wrapper gets MK_EINVAL with that text) */
    expect_rc("merkleHash len(list[0])==0 (flat=nil, n=3)", go_merkle_hash_flat(&call, NULL, 0, 3, 0, out), &call,
              MK_EINVAL, "divide by zero");
    /* merkle.TreeHashBytesList(flat, n, elemLen) */
    call.device = -1;
    expect_root("TreeHashBytesList n=0 (elems=nil)", mk_ssz_tree_hash_bytes_list(&call, NULL, 0, 32, out), &call, out,
                want[6]);
    expect_root("TreeHashBytesList elemLen=0 (elems=nil, n=4)", mk_ssz_tree_hash_bytes_list(&call, NULL, 4, 0, out),
                &call, out, want[7]);
    const uint8_t six[6] = {1, 2, 3, 4, 5, 6};
    expect_root("TreeHashBytesList n=1 elemLen=6", mk_ssz_tree_hash_bytes_list(&call, six, 1, 6, out), &call, out,
                want[8]);
    /* merkle.MerkleHashMany with k == 0 returns before the call; the call
     * itself must also be a no-op (no list, nil slices) */
    int rc = mk_ssz_merkle_many(&call, NULL, NULL, NULL, NULL, 0, NULL);
    expect_rc("MerkleHashMany k=0 (nil slices)", rc, &call, MK_OK, NULL);
    /* merkle.HashBatch with n == 0 returns before the call; likewise a no-op */
    rc = mk_hash_batch(&call, NULL, 0, 64, NULL);
    expect_rc("HashBatch n=0 (nil slices)", rc, &call, MK_OK, NULL);
    /* Trie.Append / SaveLogs of zero deposits: flat == nil, offs == [0] */
    mk_trie* t = NULL;
    rc = mk_deposit_trie_new(&call, 32, 0, &t);
    expect_rc("NewTrie(32)", rc, &call, MK_OK, NULL);
    if (rc == MK_OK) {
        uint64_t offs0[1] = {0};
        uint8_t r0[32], r1[32];
        rc = mk_deposit_trie_root(&call, t, r0);
        expect_rc("Trie.Root() empty", rc, &call, MK_OK, NULL);
        rc = mk_deposit_trie_append(&call, t, NULL, offs0, 0);
        expect_rc("Trie.Append(no deposits)", rc, &call, MK_OK, NULL);
        rc = mk_deposit_trie_save_logs(&call, t, NULL, offs0, 0, NULL, NULL);
        expect_rc("Trie.SaveLogs(no logs)", rc, &call, MK_OK, NULL);
        rc = mk_deposit_trie_root(&call, t, r1);
        int same_root = rc == MK_OK && memcmp(r0, r1, 32) == 0 && mk_deposit_trie_count(t) == 0;
        printf("%-58s %s\n", "Trie root/count unchanged", same_root ? "ok" : "MISMATCH");
        g_bad |= !same_root;
        mk_deposit_trie_free(t);
    }
    printf(g_bad ? "FAIL: cgo replay\n" : "ok: cgo replay\n");
    return g_bad;
}

int main(int argc, char** argv) {
    if (argc == 2 && strcmp(argv[1], "inject") == 0) return inject_check();
    if (argc == 11 && strcmp(argv[1], "cgo") == 0) return cgo_replay(argv + 2);
    if (argc != 3 + NT_MAX + NT_MAX + 2 + 3) {
        fprintf(stderr, "usage: %s threads rounds merkle x8 batch x8 trie_root branch many x3\n", argv[0]);
        return 2;
    }
    int nt = atoi(argv[1]);
    g_rounds = atoi(argv[2]);
    if (nt < 1 || nt > NT_MAX) return 2;
    for (int i = 0; i < NT_MAX; ++i) g_merkle[i] = argv[3 + i];
    for (int i = 0; i < NT_MAX; ++i) g_batch[i] = argv[3 + NT_MAX + i];
    g_trie_root = argv[3 + 2 * NT_MAX];
    g_branch = argv[4 + 2 * NT_MAX];
    for (int i = 0; i < 3; ++i) g_many[i] = argv[5 + 2 * NT_MAX + i];
    printf("%s, %d visible gfx950 device(s)\n", mk_version(), mk_device_count());
    pthread_t th[NT_MAX];
    struct arg args[NT_MAX];
    for (int t = 0; t < nt; ++t) {
        args[t].t = t;
        args[t].r.failures = 0;
        args[t].r.msg[0] = 0;
        if (pthread_create(&th[t], NULL, worker, &args[t]) != 0) return 3;
    }
    int bad = 0;
    for (int t = 0; t < nt; ++t) {
        pthread_join(th[t], NULL);
        if (args[t].r.failures) {
            fprintf(stderr, "thread %d FAILED: %s\n", t, args[t].r.msg);
            bad = 1;
        }
    }
    printf(bad ? "FAIL\n" : "ok: %d threads x %d rounds\n", nt, g_rounds);
    return bad;
}
