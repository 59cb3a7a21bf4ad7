// Shared declarations between the HIP kernels and the host planner / C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "plan_types.hpp"

namespace mk {

constexpr uint32_t kMaxStructFields = 32;
#define MK_STRUCT_THREADS 256
constexpr uint32_t kStructThreads = MK_STRUCT_THREADS;  // k_struct_fused: one record per thread
constexpr uint32_t kStructFusedMaxMsg = 160;          // LDS: kStructThreads * msg_len bytes
constexpr uint32_t kStructFusedMaxField = 64;         // bytes fields held in 16 registers
struct StructSpec {                 // flat fixed-layout record (hash.go:141-159)
    uint32_t kind[kMaxStructFields];   // 1 = bytes (hashed with le32 prefix), 2 = raw scalar
    uint32_t off[kMaxStructFields];    // byte offset inside the record
    uint32_t len[kMaxStructFields];    // field length in bytes
    uint32_t out_off[kMaxStructFields];  // byte offset inside the struct message
    uint32_t nfields, rec_len, msg_len;
};

template <bool LEAF, bool FAST, int NI>
__global__ void k_reduce(ReduceArgs a);
// Phase-locked leaf pass (merkle_kernels.hip): 4096 full windows per
// workgroup -> 1024 nodes three levels above the chunks.
constexpr uint32_t kLockThreads = 1024;
constexpr uint64_t kLockWindows = 4 * kLockThreads;
__global__ void k_leaf_lock_sc(ReduceArgs a, uint64_t ngroups);  // coalesced LDS-DMA staging, persistent grid
#define MK_LOCK_DMA_ROUND 14  // k_leaf_lock_sc: round of a window's second permutation after which the last part of the next block 1 is fetched
#define MK_LOCK_GRID 256
template <bool FAST>
__global__ void k_reduce_elem(ReduceArgs a);
// phase-locked element windows: nwin window digests (level-1 nodes) of 8 x 32-B elements each
__global__ void k_elem_lock(const uint4* elems, uint64_t nwin, uint4* out);
template <bool FAST32>
__global__ void k_elem_digests(const uint8_t* elems, uint64_t n, uint32_t elem_len, uint4* out);
template <bool FAST>
__global__ void k_struct_fields(const uint8_t* rec, uint64_t n, StructSpec sp, uint8_t* msg);
__global__ void k_struct_fused(const uint8_t* rec, uint64_t n, StructSpec sp, uint32_t vec16, uint4* roots);
template <int NB, int NRAW>
__global__ void k_struct_reg(const uint8_t* rec, uint64_t n, StructSpec sp, uint32_t vec16, uint4* roots);
// validator layout (kValOff/kValLen in merkle_kernels.hip), any n (a partial last group);
// gpw > 0: contiguous groups per workgroup plus the level-1 windows of the roots' merkleHash
// (and of a second list of vbytes bytes at vals, when vals != nullptr)
// PREV (a stream of states, gpw == 4): the same launch also builds levels
// 2..10 of the PREVIOUS state's registry tree over its level-1 windows and
// levels 2..4 of its second list's, one extra lock-step permutation per wave
// (see the kernel); workgroup b < nfull takes the complete 512-window
// registry subtree [512 b, 512 b + 512), b < nvfull the 128-window one.
struct StructPrev {
    const uint4* l1;   // the previous state's level-1 windows (complete)
    uint4* lv[9];      // its levels 2..10: level k node j of subtree b at lv[k - 2][(512 >> (k - 1)) b + j]
    const uint4* v1;   // the previous state's second-list level-1 windows (128 per workgroup)
    uint4* vlv[3];     // its levels 2..4: level k node j of subtree b at vlv[k - 2][(128 >> (k - 1)) b + j]
    uint32_t nfull;    // registry subtrees (workgroups) with all 512 windows
    uint32_t nvfull;   // second-list subtrees with all 128 windows
    uint32_t live;     // 0: no previous state (the slots hash zeros, store nothing)
};
template <bool PREV>
__global__ void k_struct_lock(const uint8_t* rec, uint64_t n, uint4* roots, uint32_t gpw, uint4* wins,
                              const uint8_t* vals, uint64_t vbytes, uint4* vwins, StructPrev prev);
#define MK_STRUCT_LOCK 1
template <int NB, int NRAW>
__global__ void k_struct_split(const uint8_t* rec, uint64_t n, StructSpec sp, uint32_t vec16, uint4* roots);
#define MK_STRUCT_SPLIT_MAX_N 32768
constexpr uint64_t kStructSplitMaxN = MK_STRUCT_SPLIT_MAX_N;  // k_struct_split at or below (0: never)
template <uint32_t NT, bool LEAF>
__global__ void k_wave3(ReduceArgs a);
#define MK_WAVE3_SPREAD 1  // k_wave3's last levels one state per wave (the pair finalize needs it)
__global__ void k_final_small(const uint8_t* items, uint64_t total, uint64_t n, uint8_t* out);
__global__ void k_keccak64(const uint4* in, uint64_t n, uint4* out);
__global__ void k_keccak64_lock(const uint4* in, uint64_t n, uint4* out);  // any n (a partial last group)
// phase-locked node pass: ngroups whole groups of 1024 x kNodeLockPairs complete node pairs, persistent grid
__global__ void k_node_lock(ReduceArgs a, uint64_t ngroups);
#define MK_K64_LOCK 1
__global__ void k_keccak_fixed(const uint8_t* in, uint64_t n, uint32_t msg_len, uint4* out);
__global__ void k_keccak_var(const uint8_t* in, const uint64_t* offs, uint64_t n, uint4* out);
__global__ void k_trie_level(const uint4* in, uint64_t cin, uint4* out);
__global__ void k_keccak_words(const uint2* in, uint64_t n, uint32_t nwords, uint4* out);
template <int NW>
__global__ void k_keccak_rec(const uint2* in, uint64_t n, uint4* out);
// Phase-locked deposit-trie front: leaves + levels 1..log2(DPT) of a trie of
// 280-B deposits, ngroups * NT * DPT deposits (the host runs the rest).
// PIPE: the same launch also builds levels 3..7 of the PREVIOUS trie of a
// stream (one wave-wide permutation per wave, in the lock-step slots, see
// the kernel); one group per workgroup.
struct TriePrev {
    const uint4* l2;  // the previous trie's level 2 (complete)
    uint4* l[5];      // its levels 3..7 (written)
    uint32_t live;    // 0: no previous trie (the slots hash zeros, store nothing)
};
template <uint32_t NT, int DPT, bool PIPE>
__global__ void k_trie_rec_lock(const uint2* in, uint64_t ngroups, uint4* L0, uint4* L1, uint4* L2, uint4* L3,
                                TriePrev prev);
template <uint32_t NT>
__global__ void k_trie_rec_lock_sm(const uint2* in, uint64_t ngroups, uint4* L0, uint4* L1, uint4* L2);
#define MK_TRIE_LOCK 1
#define MK_TRIE_LOCK_GRID 256  // persistent grid cap
#define MK_TRIE_LOCK_MIN (1u << 18)  // deposits: at least one group per CU

#define MK_REC_THREADS 256
constexpr uint32_t kRecThreads = MK_REC_THREADS;  // k_keccak_rec workgroup size
#define MK_REC_GRID 4096
constexpr uint32_t kRecGridMax = MK_REC_GRID;  // k_keccak_rec grid cap (A/B at 2^20: 512..4096 WGs, 4096 best)
template <uint32_t NT>
__global__ void k_trie_top3(const uint32_t* in, uint64_t cin, uint32_t* lv_out, uint32_t levels, uint64_t capn);
__global__ void k_verify_branches(const uint4* leaves, const uint4* branches, const uint64_t* indices,
                                  uint32_t depth, uint32_t tree_depth, const uint4* roots, uint64_t n,
                                  uint8_t* ok);
template <uint32_t NT>
__global__ void k_trie_append(uint32_t* levels, uint64_t cap, uint32_t d0, uint64_t lo, uint64_t c, uint32_t d_end,
                              uint32_t depth, uint32_t* root_out);
#define MK_TRIE_SPREAD 1
#define MK_SPREAD_WAVES_MAX 16
constexpr uint32_t kSpreadWavesMax = MK_SPREAD_WAVES_MAX;  // k_trie_spread: one state per wave (<= 4 per SIMD)
template <uint32_t SPAN>
__global__ void k_spread_leaf(ReduceArgs a, uint32_t w8);
template <int NB, int NRAW>
__global__ void k_struct_list_fused(const uint8_t* rec, uint64_t n, StructSpec sp, uint32_t vec16, uint4* roots,
                                    ReduceArgs a, uint32_t* sub, uint32_t* out, uint32_t slot);
// new deposits k_trie_spread hashes into level 0 first (k == 0: none)
struct SpreadLeaves {
    const uint8_t* data;
    const uint64_t* offs;  // device, k+1 entries relative to data; NULL: fixed_len records
    uint32_t fixed_len;
    uint32_t k;
    uint32_t aligned8;     // data, offsets / fixed_len multiples of 8
};
template <uint32_t NW>
__global__ void k_trie_spread(uint32_t* levels, uint64_t cap, uint32_t d0, uint64_t lo, uint64_t c, uint32_t d_end,
                              uint32_t depth, uint32_t* root_out, SpreadLeaves lv);
// fused tree tops: arrival counter slots (one per fused launch in flight)
constexpr uint32_t kArriveSlots = 4096;
// k_trie_top_fused: the last of each kTopGroup workgroups reduces the group's
// nodes before the last group finishes the top
// nodes before the next stage / the last group finishes the top (0: the last
// workgroup alone reduces all the grid's nodes)
#define MK_TOP_GROUP_LOG2 4
constexpr uint32_t kTopGroupLog2 = MK_TOP_GROUP_LOG2, kTopGroup = 1u << kTopGroupLog2;
constexpr uint32_t kTopGroupSlots = kTopGroupLog2 ? 1 + 2 * 1024 / kTopGroup : 1;  // arrival slots of one launch
template <uint32_t NT>
__global__ void k_trie_top_fused(uint32_t* levels, uint64_t cap, uint64_t c0, uint32_t d0, uint32_t depth,
                                 uint32_t* root_out, uint32_t slot);
// k_merkle_top_fused: one list's part of the launch
struct MerkleTopList {
    const uint4* nodes;  // a complete level of the list's tree (plain 32-B nodes)
    uint64_t c;          // its node count
    uint64_t n_items;    // the length mix-in (hash.go:237-238)
    uint32_t* sub;       // workspace: one published node per workgroup (32 B each)
    uint32_t* out;       // the list root (32 B; with a pair: its slot of the pair block)
    uint32_t wg0, nwg;   // this list's workgroups
    uint32_t span_log2;  // level nodes per workgroup
    uint32_t slot;       // first of its arrival counters (g_arrive; capi.cpp top_arrive_slots)
};
struct MerkleTopArgs {
    MerkleTopList l[2];
    uint32_t nlists;
    uint32_t* pair;      // two lists: the pair block (roots at [0, 64), the struct root at [64, 96)), else NULL
    uint32_t pair_slot;  // two lists: the arrival counter of the two finishers
};
template <uint32_t NT>
__global__ void k_merkle_top_fused(MerkleTopArgs a);
__global__ void k_trie_append1(uint32_t* levels, uint64_t cap, uint64_t count, uint32_t depth, uint32_t* root_out,
                               SpreadLeaves lv);
template <uint32_t NW>
__global__ void k_trie_prefix_roots(const uint4* levels, uint64_t cap, uint64_t count0, uint64_t m, uint32_t depth,
                                    uint4* roots);
__global__ void k_trie_branch(const uint4* levels, uint64_t cap, uint64_t count, uint32_t depth, uint64_t index,
                              uint4* branch);
template <bool LEAF>
__global__ void k_many_level(const uint8_t* items, const ManyList* lists, const ManyAct* act, uint32_t nact,
                             uint64_t nodes, const uint4* in, uint4* out, uint4* tops);
__global__ void k_many_final(const uint8_t* items, const ManyList* lists, uint32_t nlists, const uint4* tops,
                             uint4* roots);
__global__ void k_synth(uint64_t* dst, uint64_t nwords, uint64_t seed, uint64_t word0);

}  // namespace mk
