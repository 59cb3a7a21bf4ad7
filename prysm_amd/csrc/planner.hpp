// Host-side planning of the Merkleization engine: the error sink of the C
// ABI, the merkleHash pass planner (shared/ssz/hash.go:194-239 as a sequence
// of fused kernel passes), the subtree shard plan, the
// deposit-trie level layout (deposit_trie.go:29-63) and the many-lists plan.
// No HIP here: tests/c_abi/planner_fuzz.cpp builds this file with
// -fsanitize=address,undefined on the CPU.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "plan_types.hpp"
#include "prysm_merkle.h"

namespace mk {

// ---- error sink ----------------------------------------------------------
// fail() records the detail for the calling thread (mk_last_error) and, when
// a call context is active on this thread, in call->err / call->code.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
const char* last_error();
void clear_error();
mk_call* current_call();
mk_call* swap_call(mk_call* c);  // returns the previous context

// ---- arithmetic ------------------------------------------------------------
inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
inline uint64_t chunk_bytes(uint32_t item_len) {
    return item_len < 128 ? (uint64_t)(128 / item_len) * item_len : item_len;
}
inline uint64_t perms_for_len(uint64_t len) { return len / 136 + 1; }
uint32_t ilog2(uint64_t v);
uint32_t levels_to_one(uint64_t count);  // hashing levels from `count` nodes to one

// ---- merkleHash pass plan --------------------------------------------------
// Plans made while a WideWaves is alive on this thread give every latency
// (k_wave3) pass full 1024-thread workgroups: the finishers that run beside a
// CU-filling phase-locked launch then only land on the CUs its grid leaves
// free, instead of squeezing one-wave workgroups in beside its locked waves
// (starved ~10x there).
struct WideWaves {
    WideWaves();
    ~WideWaves();
    bool prev;
};

struct Pass {
    bool leaf;
    bool wave;  // latency pass (k_wave*) instead of the throughput pass (k_reduce)
    uint64_t nwg, nfast;
    bool w3;      // k_wave3 (bit-interleaved latency form)
    bool sp;      // k_spread_leaf (one state per wave, 16 windows per workgroup)
    uint32_t nt;  // threads per workgroup
    uint32_t ni;  // k_reduce: window pairs per thread (span 512 * ni)
    uint64_t nlock;  // leaf: k_leaf_lock_sc workgroups (4 spans each) before the k_reduce ones (levels == 3);
                     // node: k_node_lock groups (kNodeLockSpans spans each, levels == 5)
    ReduceArgs a;
    int in_ws;   // -1 = user input, else ping-pong slot
    int out_ws;  // -1 = user output, else ping-pong slot
    double perms;
    double hashes;  // digests produced (each ends in one digest-only permutation)
};

struct Plan {
    bool small = false;  // <= 1 chunk: one final hash of the raw bytes
    std::vector<Pass> passes;
    uint64_t slot_nodes[2] = {0, 0};
    uint64_t total = 0, n = 0;
    uint64_t out_nodes = 1;  // nodes written to the output (frontier mode: > 1)
};

// subtree=false: full merkleHash with the length mix-in; subtree=true: exactly
// `height` levels above the chunks, one output node (pad_at_one keeps the odd
// rule alive at count 1).  node_input: n 32-B nodes reduced pairwise
// (MerkleRoot heap bands, a gathered frontier level); without subtree mode the
// final pass mixes in `mixin_n`.  frontier (subtree mode): stop `frontier`
// levels below the subtree root and write that level.  leaf_ni1: the leaf
// pass's throughput workgroups take one window pair per thread (k_reduce_elem).
int make_plan(uint64_t n, uint32_t item_len, bool subtree, uint32_t height, bool pad_at_one, bool aligned16, Plan& p,
              bool node_input = false, uint32_t frontier = 0, uint64_t mixin_n = 0, bool leaf_ni1 = false);
uint64_t plan_ws_bytes(const Plan& p);

int shard_plan(uint64_t n, uint32_t item_len, uint32_t nshards, uint32_t* height, uint32_t* nonempty,
               uint64_t* begin);
// nodes of a shard `k` levels below its root (>= 1 with pad_at_one)
uint64_t frontier_nodes(uint64_t shard_n, uint32_t item_len, uint32_t height, uint32_t k);

// ---- deposit trie layout ------------------------------------------------------
// level d starts at node trie_level_off(cap, d) = sum_{i<d} ceil(cap / 2^i)
uint64_t trie_level_off(uint64_t cap, uint32_t d);
uint64_t trie_levels_nodes(uint64_t cap, uint32_t depth);
inline uint64_t trie_count(uint64_t count, uint32_t d) { return d >= 64 ? (count ? 1 : 0) : ceil_div(count, 1ull << d); }

// ---- many lists (segmented merkleHash) -------------------------------------------
// Lists of more than kManyBigChunks chunks run their own fused plan; smaller
// lists with >= 2 chunks share one leaf launch and one launch per level
// (ManyList, act tables); lists of <= 1 chunk only get the final hash.
constexpr uint64_t kManyBigChunks = 1ull << 15;

struct ManyPlan {
    std::vector<ManyList> lists;         // every list (big: c1 = 0, levels = UINT32_MAX)
    std::vector<uint32_t> big;           // indices of the big lists
    std::vector<Plan> big_plans;         // their plans (final, with mix-in)
    uint32_t nlevels = 0;                // node levels of the segmented part (level 1 = windows)
    // act table of level l+1 (l = 0: windows) = act[lvl_begin[l], lvl_begin[l+1]):
    // the lists with nodes there, out_first = exclusive prefix sum of their
    // node counts; level l+1 is written to buffer l % 2, and a list's top
    // node (its last level) also to tops[list] (the buffers are reused)
    std::vector<ManyAct> act;
    std::vector<uint64_t> lvl_begin;     // nlevels + 1
    std::vector<uint64_t> lvl_nodes;     // nodes computed at each level
    uint64_t buf_nodes[2] = {0, 0};      // capacity of the two level buffers
    uint64_t big_ws = 0;                 // max plan_ws_bytes of the big lists
    // workspace layout (bytes from the workspace start, 256-aligned)
    uint64_t off_lists = 0, off_act = 0, off_tops = 0, off_buf0 = 0, off_buf1 = 0, off_big = 0;
    uint64_t ws_bytes = 0;
    double perms = 0;                    // algorithmic permutations of the whole call
};
int make_many_plan(const uint64_t* offs, const uint64_t* n, const uint32_t* item_len, uint32_t nlists,
                   uint64_t items_bytes, bool base_aligned16, ManyPlan& mp);

}  // namespace mk
