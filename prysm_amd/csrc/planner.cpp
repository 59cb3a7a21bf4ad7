// Host-side planning (see planner.hpp).  No HIP calls in this file.
#include "planner.hpp"

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>

namespace mk {

// ---- error sink ------------------------------------------------------------------
namespace {
thread_local std::string t_err;
thread_local mk_call* t_call = nullptr;
}  // namespace

int fail(int code, const char* fmt, ...) {
    char buf[MK_ERR_LEN];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_err = buf;
    if (t_call) {
        t_call->code = code;
        std::memcpy(t_call->err, buf, sizeof buf);  // vsnprintf NUL-terminates within MK_ERR_LEN
    }
    return code;
}
const char* last_error() { return t_err.c_str(); }
void clear_error() { t_err.clear(); }
mk_call* current_call() { return t_call; }
mk_call* swap_call(mk_call* c) {
    mk_call* prev = t_call;
    t_call = c;
    return prev;
}

// ---- configuration (compile-time knobs; A/B variants via the Makefile) ----------
// latency passes: k_wave3 (bit-interleaved lane pairs, one state per wave at
// the top; round 4 removed the lo/hi-halves k_wave2 it replaced in round 1)
#define MK_NODE_WAVE_MAX_LOG2 17
// node passes switch to the latency form at or below this width: the first
// level is throughput-bound either way, but the throughput kernel spends ~9
// serial permutations on its 5 levels where the wave pass spends 6
constexpr uint64_t kNodeWaveMaxC1 = 1ull << MK_NODE_WAVE_MAX_LOG2;
#define MK_NODE_WAVE_WGS 256
constexpr uint64_t kNodeWaveWgs = MK_NODE_WAVE_WGS;
#define MK_LEAF_WAVE_MAX_LOG2 17
constexpr uint64_t kLeafWaveMaxC1 = 1ull << MK_LEAF_WAVE_MAX_LOG2;  // leaf passes at or below: latency form
#define MK_REDUCE_NI2_MIN_LOG2 18
constexpr uint64_t kReduceNi2MinC1 = 1ull << MK_REDUCE_NI2_MIN_LOG2;  // leaf passes narrower than this use NI = 1
// Largest k_wave3 workgroup the planner picks (64..1024 threads).
#define MK_W3_MAX_NT 1024
constexpr uint32_t kW3MaxNt = MK_W3_MAX_NT < kMidThreads ? MK_W3_MAX_NT : kMidThreads;
// leaf passes of at most this many windows: k_spread_leaf (0: never)
#define MK_SPREAD_LEAF_MAX_LOG2 12
constexpr uint64_t kSpreadLeafMaxC1 = MK_SPREAD_LEAF_MAX_LOG2 < 0 ? 0 : 1ull << MK_SPREAD_LEAF_MAX_LOG2;
constexpr uint64_t kSpreadSpan = 16;  // windows per k_spread_leaf workgroup
// Phase-locked leaf pass (k_leaf_lock_sc, merkle_kernels.hip): wide leaf passes
// of full 256-B windows fold 3 levels (windows -> node pairs -> one node per
// 4 windows) in 1024-thread workgroups whose Keccak rounds hold an s_barrier;
// the next (node) pass takes the levels the leaf pass used to fuse in LDS.
constexpr bool kLeafLock = MK_LEAF_LOCK != 0;  // plan_types.hpp
// tests/test_planner_fuzz.py overrides it (-D) to reach the locked plan at fuzz sizes
#ifndef MK_LEAF_LOCK_MIN_LOG2
#define MK_LEAF_LOCK_MIN_LOG2 20
#endif
constexpr uint64_t kLeafLockMinC1 = 1ull << MK_LEAF_LOCK_MIN_LOG2;  // windows (first-level nodes)
constexpr uint32_t kLockLevels = 3;
constexpr uint64_t kLockSpans = 4;  // k_reduce spans (1024 windows) per k_leaf_lock_sc workgroup
// Phase-locked node pass (k_node_lock): a wide node pass of complete pairs
// runs whole multiples of kNodeLockGroupMul groups of 16 k_reduce spans
// (16,384 pairs) each, one group per CU at a time; a pass with fewer groups
// than CUs keeps k_reduce, which spreads over every CU.  One-process A/B at
// 2^28 (profiles/r05/node_lock/): whole tree 9.004 -> 8.871 ms (the node pass
// 0.836 -> 0.689 ms by rocprof), 9 interleaved rounds.
constexpr uint64_t kNodeLockGroupMul = 256;
#define MK_NODE_LOCK 1

uint32_t ilog2(uint64_t v) {
    uint32_t l = 0;
    while (v > 1) {
        v >>= 1;
        ++l;
    }
    return l;
}

uint32_t levels_to_one(uint64_t count) {
    uint32_t l = 0;
    while (count > 1) {
        count = (count + 1) / 2;
        ++l;
    }
    return l;
}

// ---- merkleHash pass plan ---------------------------------------------------------
thread_local bool t_wide_waves = false;
WideWaves::WideWaves() : prev(t_wide_waves) { t_wide_waves = true; }
WideWaves::~WideWaves() { t_wide_waves = prev; }

int make_plan(uint64_t n, uint32_t item_len, bool subtree, uint32_t height, bool pad_at_one, bool aligned16, Plan& p,
              bool node_input, uint32_t frontier, uint64_t mixin_n, bool leaf_ni1) {
    p = Plan();
    p.n = n;
    if (n > 0 && item_len == 0) return fail(MK_EINVAL, "item_len == 0 (reference: integer divide by zero)");
    if (node_input && item_len != 32) return fail(MK_EINVAL, "planner: node input is 32-B nodes");
    if (node_input && !subtree && n < 2) return fail(MK_EINVAL, "planner: node finisher needs >= 2 nodes");
    if (frontier && (!subtree || frontier >= height)) return fail(MK_EINVAL, "planner: bad frontier %u", frontier);
    if (subtree && height >= 64) return fail(MK_EINVAL, "subtree: height %u >= 64", height);
    if (!node_input && n > (UINT64_MAX / 2) / (item_len ? item_len : 1)) return fail(MK_EINVAL, "n * item_len overflows");
    const uint64_t total = n * (uint64_t)item_len;
    const uint64_t cb = node_input ? 32 : n ? chunk_bytes(item_len) : 128;
    const uint64_t nchunks = node_input ? n : n ? ceil_div(total, cb) : 0;
    p.total = total;
    if (!subtree && nchunks <= 1) {
        p.small = true;
        return MK_OK;
    }
    if (subtree && (height == 0 || nchunks == 0 || nchunks > (1ull << height)))
        return fail(MK_EINVAL, "subtree: bad height %u for %llu chunks", height, (unsigned long long)nchunks);

    uint32_t remaining = subtree ? height - frontier : levels_to_one(nchunks);
    if (frontier) {  // nodes at the frontier level (the odd rule keeps >= 1 with pad_at_one)
        const uint64_t span = 1ull << (height - frontier);
        p.out_nodes = std::max<uint64_t>(1, ceil_div(nchunks, span));
    }
    bool leaf = !node_input;
    uint64_t cin = nchunks;  // leaf: chunks; node: input nodes
    int slot = 0;
    int in_slot = -1;
    while (true) {
        Pass ps{};
        ps.leaf = leaf;
        ReduceArgs& a = ps.a;
        const uint64_t c1 = (cin > 1 || pad_at_one) ? ceil_div(cin, 2) : 1;
        a.c1 = c1;
        a.pad_at_one = pad_at_one ? 1 : 0;
        a.n_items = (node_input && !subtree) ? mixin_n : n;
        if (leaf) {
            a.total = total;
            a.cb = cb;
            a.nchunks = nchunks;
            a.c1_full = (cb == 128 && aligned16) ? total / 256 : 0;
        } else {
            a.cin = cin;
            a.c1_full = cin / 2;
        }
        // algorithmic permutations of this pass (first level + fused levels)
        double perms = 0, hashes = 0;
        if (leaf) {
            const uint64_t full = total / (2 * cb);
            perms += (double)std::min<uint64_t>(full, c1) * perms_for_len(2 * cb);
            for (uint64_t j = full; j < c1; ++j) {  // at most one ragged window
                const uint64_t lo = j * 2 * cb;
                const uint64_t len = (2 * j + 1 < nchunks) ? std::min(total, lo + 2 * cb) - lo : total - lo + 128;
                perms += (double)perms_for_len(len);
            }
            hashes += (double)c1;
        } else if (cin > 1 || pad_at_one) {
            perms += (double)(cin / 2) + (cin % 2 ? 2.0 : 0.0);
            hashes += (double)ceil_div(cin, 2);
        }
        uint64_t c = c1;
        const bool sp = leaf && c1 <= kSpreadLeafMaxC1;
        const bool wave = sp || c1 <= (leaf ? kLeafWaveMaxC1 : kNodeWaveMaxC1);
        const bool w3 = !sp && wave;
        // k_wave3: the smallest workgroup (64..1024 threads, 2 per pair) that
        // keeps the pass within ~256 workgroups, one per CU
        uint32_t nt = w3 ? kWaveThreads : kReduceThreads;
        if (w3) {
            while (nt < kW3MaxNt && ceil_div(c1, nt / 2) > kNodeWaveWgs) nt *= 2;
            // the last <= 512 pairs in one workgroup of the full 1024 threads
            // even when fewer pairs need them: k_wave3 switches to one state
            // per wave once a level has at most NT/64 parents, so 16 waves run
            // the last 4 levels and the mix-in in the spread form (one launch
            // to the root)
            if (c1 <= kW3MaxNt / 2 || t_wide_waves) nt = kW3MaxNt;
        }
        // throughput pass: 2 window pairs per thread on wide passes, 1 on mid-size
        // leaf passes so they still spread over the CUs
        const uint32_t ni = (!wave && leaf && (c1 < kReduceNi2MinC1 || leaf_ni1)) ? 1 : 2;
        if (sp) nt = 1024;
        const uint64_t span = sp ? kSpreadSpan
                            : w3 ? nt / 2 : (uint64_t)2 * ni * kReduceThreads;
        const bool final_pass = c1 <= span;
        const uint32_t max_lv = sp ? 1 + ilog2(kSpreadSpan)
                              : w3 ? 1 + ilog2(nt / 2) : kMaxPassLevels;
        uint32_t lv = final_pass ? remaining : std::min<uint32_t>(max_lv, remaining);
        const bool lock = kLeafLock && leaf && !wave && !final_pass && !leaf_ni1 && ni == 2 &&
                          a.c1_full >= kLeafLockMinC1 && remaining > kLockLevels &&
                          a.c1_full / span >= kLockSpans;
        if (lock) lv = kLockLevels;
        const uint64_t nodelock = (MK_NODE_LOCK && !leaf && !wave && !final_pass && ni == 2 && remaining > kNodeLockLevels &&
                                   (in_slot >= 0 || aligned16))
                                      ? (a.c1_full / span) / kNodeLockSpans / kNodeLockGroupMul * kNodeLockGroupMul
                                      : 0;
        if (nodelock) lv = kNodeLockLevels;
        for (uint32_t l = 1; l < lv; ++l) {  // fused levels above the first
            if (c <= 1 && !pad_at_one) break;
            perms += (double)(c / 2) + (c % 2 ? 2.0 : 0.0);
            hashes += (double)ceil_div(c, 2);
            c = ceil_div(c, 2);
        }
        ps.perms = perms;
        ps.hashes = hashes;
        ps.wave = wave;
        ps.nt = nt;
        a.in_ilv = (w3 && !leaf && !p.passes.empty() && p.passes.back().w3) ? 1 : 0;
        ps.w3 = w3;
        ps.sp = sp;
        a.out_ilv = w3 ? 1 : 0;  // cleared below for the final pass
        a.levels = lv;
        ps.nwg = ceil_div(c1, span);
        ps.nfast = wave ? 0 : std::min<uint64_t>(ps.nwg, a.c1_full / span);
        ps.ni = ni;
        ps.nlock = lock ? ps.nfast / kLockSpans : nodelock;
        ps.in_ws = in_slot;
        if (final_pass) {
            if (!subtree) {
                a.finalize = 1;
                a.levels = 64;
                perms += 1;  // the length mix-in K(root || lenc)
                hashes += 1;
            } else if (!wave && c1 > span / 2 && lv < 2) {
                return fail(MK_EINVAL, "planner: unsupported single-level pass");
            }
            ps.perms = perms;
            ps.hashes = hashes;
            ps.out_ws = -1;
            ps.a.out_ilv = 0;
            p.passes.push_back(ps);
            break;
        }
        if (!wave && lv < 2)  // k_reduce always folds the pair level (a frontier one level above the chunks)
            return fail(MK_EINVAL, "planner: unsupported single-level pass (frontier %u of height %u)", frontier,
                        height);
        if (frontier && remaining == lv) {  // the frontier level: plain nodes to the output
            ps.out_ws = -1;
            ps.a.out_ilv = 0;
            p.passes.push_back(ps);
            break;
        }
        ps.out_ws = slot;
        p.slot_nodes[slot] = std::max<uint64_t>(p.slot_nodes[slot], c);
        p.passes.push_back(ps);
        remaining -= lv;
        in_slot = slot;
        slot ^= 1;
        leaf = false;
        cin = c;
        if (remaining == 0) return fail(MK_EINVAL, "planner: ran out of levels");
    }
    return MK_OK;
}

uint64_t plan_ws_bytes(const Plan& p) { return 32 * (p.slot_nodes[0] + p.slot_nodes[1]) + 256; }

int shard_plan(uint64_t n, uint32_t item_len, uint32_t nshards, uint32_t* height, uint32_t* nonempty,
               uint64_t* begin) {
    if (nshards == 0) return fail(MK_EINVAL, "nshards == 0");
    if (n > 0 && item_len == 0) return fail(MK_EINVAL, "item_len == 0");
    if (n > (UINT64_MAX / 2) / (item_len ? item_len : 1)) return fail(MK_EINVAL, "n * item_len overflows");
    const uint64_t total = n * (uint64_t)item_len;
    const uint64_t cb = n ? chunk_bytes(item_len) : 128;
    const uint64_t per_chunk_items = item_len < 128 ? 128 / item_len : 1;
    const uint64_t nchunks = n ? ceil_div(total, cb) : 0;
    uint32_t h = 0;
    while ((1ull << h) * nshards < nchunks) ++h;
    const uint64_t ne = nchunks ? ceil_div(nchunks, 1ull << h) : 0;
    if (h == 0 || ne <= 1) {  // too small to shard: everything on shard 0
        *height = h;
        *nonempty = 1;
        for (uint32_t s = 0; s <= nshards; ++s) begin[s] = s == 0 ? 0 : n;
        return MK_OK;
    }
    *height = h;
    *nonempty = (uint32_t)ne;
    for (uint32_t s = 0; s <= nshards; ++s) {
        const uint64_t item = (uint64_t)s * (1ull << h) * per_chunk_items;
        begin[s] = item < n ? item : n;
    }
    return MK_OK;
}

uint64_t frontier_nodes(uint64_t shard_n, uint32_t item_len, uint32_t height, uint32_t k) {
    const uint64_t cb = chunk_bytes(item_len);
    const uint64_t chunks = ceil_div(shard_n * (uint64_t)item_len, cb);
    return std::max<uint64_t>(1, ceil_div(chunks, 1ull << (height - k)));
}

// ---- deposit trie layout ---------------------------------------------------------------
uint64_t trie_level_off(uint64_t cap, uint32_t d) {
    uint64_t off = 0;
    for (uint32_t i = 0; i < d; ++i) off += trie_count(cap, i);
    return off;
}
uint64_t trie_levels_nodes(uint64_t cap, uint32_t depth) { return trie_level_off(cap, depth + 1); }

// ---- many lists ----------------------------------------------------------------------------
static uint64_t align256(uint64_t x) { return (x + 255) & ~255ull; }

int make_many_plan(const uint64_t* offs, const uint64_t* n, const uint32_t* item_len, uint32_t nlists,
                   uint64_t items_bytes, bool base_aligned16, ManyPlan& mp) {
    mp = ManyPlan();
    if (nlists && (!n || !item_len)) return fail(MK_EINVAL, "many: null n/item_len");
    mp.lists.resize(nlists);
    uint32_t maxlv = 0;
    for (uint32_t i = 0; i < nlists; ++i) {
        ManyList& L = mp.lists[i];
        if (n[i] > 0 && item_len[i] == 0)
            return fail(MK_EINVAL, "list %u: item_len == 0 (reference: integer divide by zero)", i);
        if (n[i] > (UINT64_MAX / 4) / (item_len[i] ? item_len[i] : 1)) return fail(MK_EINVAL, "list %u too long", i);
        L.items_off = offs ? offs[i] : 0;
        L.total = n[i] * (uint64_t)item_len[i];
        if (L.total && (!offs || L.items_off > items_bytes || L.total > items_bytes - L.items_off))
            return fail(MK_EINVAL, "list %u: bytes [%llu, +%llu) outside the input", i,
                        (unsigned long long)L.items_off, (unsigned long long)L.total);
        L.cb = n[i] ? chunk_bytes(item_len[i]) : 128;
        L.nchunks = n[i] ? ceil_div(L.total, L.cb) : 0;
        L.n = n[i];
        L.fast = (L.cb == 128 && base_aligned16 && L.items_off % 16 == 0) ? 1 : 0;
        if (L.nchunks <= 1) {  // one final hash of the raw bytes
            L.c1 = 0;
            L.levels = 0;
        } else if (L.nchunks > kManyBigChunks) {
            L.c1 = 0;
            L.levels = UINT32_MAX;
            mp.big.push_back(i);
            mp.big_plans.emplace_back();
            int rc = make_plan(n[i], item_len[i], false, 0, false, L.fast != 0, mp.big_plans.back());
            if (rc != MK_OK) return rc;
            mp.big_ws = std::max(mp.big_ws, plan_ws_bytes(mp.big_plans.back()));
            for (const Pass& ps : mp.big_plans.back().passes) mp.perms += ps.perms;
        } else {
            L.c1 = ceil_div(L.nchunks, 2);
            L.levels = levels_to_one(L.nchunks);
            maxlv = std::max(maxlv, L.levels);
            const uint64_t full = L.total / (2 * L.cb);
            mp.perms += (double)std::min(full, L.c1) * perms_for_len(2 * L.cb);
            for (uint64_t j = full; j < L.c1; ++j) {
                const uint64_t lo = j * 2 * L.cb;
                const uint64_t len =
                    (2 * j + 1 < L.nchunks) ? std::min(L.total, lo + 2 * L.cb) - lo : L.total - lo + 128;
                mp.perms += (double)perms_for_len(len);
            }
            for (uint64_t c = L.c1; c > 1; c = ceil_div(c, 2)) mp.perms += (double)(c / 2) + (c % 2 ? 2.0 : 0.0);
        }
        if (L.levels != UINT32_MAX)  // the length mix-in (or the whole small list)
            mp.perms += (double)perms_for_len(L.nchunks <= 1 ? L.total + (n[i] ? 0 : 128) + 32 : 64);
    }
    mp.nlevels = maxlv;
    mp.lvl_begin.assign(1, 0);
    // level l (1 = windows): ceil(nchunks / 2^l) nodes of every list with >= l
    // levels, written to buffer (l - 1) % 2 at the exclusive prefix sum
    std::vector<uint64_t> prev_first(nlists, 0);
    for (uint32_t l = 1; l <= maxlv; ++l) {
        uint64_t first = 0;
        for (uint32_t i = 0; i < nlists; ++i) {
            ManyList& L = mp.lists[i];
            if (L.levels == UINT32_MAX || L.levels == 0 || L.levels < l) continue;
            mp.act.push_back(ManyAct{i, l, first, prev_first[i]});
            prev_first[i] = first;
            first += ceil_div(L.c1, 1ull << (l - 1));
        }
        mp.lvl_begin.push_back(mp.act.size());
        mp.lvl_nodes.push_back(first);
        mp.buf_nodes[(l - 1) % 2] = std::max(mp.buf_nodes[(l - 1) % 2], first);
    }
    uint64_t off = 0;
    mp.off_lists = off;
    off += align256(sizeof(ManyList) * std::max<uint64_t>(1, nlists));
    mp.off_act = off;
    off += align256(sizeof(ManyAct) * std::max<size_t>(1, mp.act.size()));
    mp.off_tops = off;
    off += align256(32 * std::max<uint64_t>(1, nlists));
    mp.off_buf0 = off;
    off += align256(32 * std::max<uint64_t>(1, mp.buf_nodes[0]));
    mp.off_buf1 = off;
    off += align256(32 * std::max<uint64_t>(1, mp.buf_nodes[1]));
    mp.off_big = off;
    off += align256(std::max<uint64_t>(256, mp.big_ws));
    mp.ws_bytes = off;
    return MK_OK;
}

}  // namespace mk
