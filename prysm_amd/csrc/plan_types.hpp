// Types and shape constants shared by the HIP kernels and the host planner.
// Plain C++ (no HIP headers), so the planner also builds host-only with
// gcc -fsanitize=address,undefined (tests/c_abi/planner_fuzz.cpp).
#pragma once
#include <stdint.h>

namespace mk {

constexpr uint32_t kReduceThreads = 256;             // 4 waves
constexpr uint64_t kReduceSpan1 = 4 * kReduceThreads;  // first-level nodes per workgroup
constexpr uint64_t kReduceSpan2 = kReduceSpan1 / 2;    // level-2 nodes per workgroup (LDS)
constexpr uint32_t kMaxPassLevels = 5;               // levels per non-final pass (1024 -> 64)
constexpr uint32_t kWaveThreads = 64;                // smallest k_wave3 workgroup: one wave
constexpr uint32_t kWave2Span = kWaveThreads / 2;    // lane pairs per wave: 32 nodes (dev_finish takes <= 64 roots)
constexpr uint32_t kMidThreads = 1024;               // largest k_wave3: 16 waves, 512 lane pairs, 10 levels
// Wide leaf passes of full windows run the phase-locked k_leaf_lock_sc
// (merkle_kernels.hip, planner.cpp) instead of k_reduce's fused form.
#define MK_LEAF_LOCK 1
// Wide node passes of whole trees run the phase-locked k_node_lock: 16 node
// pairs per thread folded 5 levels in registers (1024-thread workgroups of
// 16 k_reduce spans each, the same output order).
constexpr uint32_t kNodeLockPairs = 16;
constexpr uint32_t kNodeLockLevels = 5;
constexpr uint64_t kNodeLockSpans = 16;  // k_reduce node spans (2 * 2 * kReduceThreads pairs) per group
static_assert(kNodeLockSpans * 4 * kReduceThreads == 1024ull * kNodeLockPairs, "a group = 16 spans");
#ifndef MK_LOCK_BARS
#define MK_LOCK_BARS 2  // s_barriers per locked Keccak round (keccak_dev.hpp round_asm)
#endif

struct ReduceArgs {
    const uint8_t* items;  // LEAF: item bytes; NODE: 32-B input nodes
    uint64_t total;        // LEAF: item bytes in the tree (shard)
    uint64_t cb;           // LEAF: chunk bytes
    uint64_t nchunks;      // LEAF: chunks in the tree (shard)
    uint64_t cin;          // NODE: input node count
    uint64_t c1;           // first-level node count (windows / input pairs)
    uint64_t c1_full;      // first-level nodes eligible for the fast path
    uint8_t* out;          // output nodes (or the 32-B digest when finalize)
    uint64_t n_items;      // length mix-in value (finalize)
    uint32_t levels;       // hashing levels this pass performs
    uint32_t finalize;     // reduce to the root and mix in the length
    uint32_t pad_at_one;   // subtree mode: keep hashing (x || 0^128) at count 1
    uint64_t wg_base;      // workgroup index offset of this launch
    uint32_t in_ilv;       // k_wave3: input nodes are bit-interleaved lane pairs
    uint32_t out_ilv;      // k_wave3: write bit-interleaved output nodes
    uint32_t elem_len;     // LEAF, k_reduce_elem: `items` are n elements of elem_len bytes and the
                           // tree's 32-B items are their digests K(le32(elem_len) || element)
    uint8_t* pair_block;   // finalize (k_wave3), nullable: a two-field struct root -- the list root goes to
                           // pair_block[32 pair_slot..), and the second of the two finishers of epoch
                           // pair_epoch to complete writes K(pair_block[0..64)) to pair_block[64..96)
                           // (arrival word at [96..100))
    uint32_t pair_slot;
    uint32_t pair_epoch;
};

// One list of a segmented (many-lists) merkleHash level: k_many_leaf /
// k_many_level map a global thread index to (list, node) by binary search
// over `first` (exclusive prefix sum of this level's node counts).
struct ManyList {
    uint64_t items_off;  // byte offset of the list's items in the input buffer
    uint64_t total;      // item bytes
    uint64_t cb;         // chunk bytes
    uint64_t nchunks;    // chunks
    uint64_t n;          // items (length mix-in)
    uint64_t c1;         // level-1 node count (0: the list has <= 1 chunk)
    uint32_t levels;     // hashing levels above the chunks (0 for <= 1 chunk)
    uint32_t fast;       // 256-B contiguous windows (item_len | 128, 16-B aligned)
};

// Entry of a level's act table: list `list` writes its nodes of this level at
// [out_first, out_first + count) and reads the level below at in_first.
struct ManyAct {
    uint32_t list;
    uint32_t level;     // 1 = windows (input: the list's item bytes)
    uint64_t out_first;
    uint64_t in_first;
};

}  // namespace mk
