// Host-only fuzz of the pass planner (prysm_amd/csrc/planner.cpp), built with
// g++ -fsanitize=address,undefined by tests/test_planner_fuzz.py.  For random
// (n, item_len, height, frontier, pad_at_one) it builds merkleHash, subtree,
// frontier and node-input plans, the shard plan, the many-lists plan and the
// deposit-trie layout, checks their internal invariants (abort on violation)
// and prints one line per case for the Python restatements
// (tests/test_distributed.py::_plan_cpu, parallel.frontier_count):
//   S n item_len world h nonempty b0 .. bworld
//   F n item_len height k out_nodes
//   M nlists seg_levels ws_bytes
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "planner.hpp"

using namespace mk;

#define REQUIRE(c)                                                                   \
    do {                                                                             \
        if (!(c)) {                                                                  \
            std::fprintf(stderr, "invariant failed at line %d: %s\n", __LINE__, #c); \
            std::abort();                                                            \
        }                                                                            \
    } while (0)

// Replays a plan's node counts: pass p turns cin into c1 = ceil(cin/2)
// (1 when cin == 1 and no pad_at_one), then `levels - 1` more halvings.
static uint64_t g_lock_passes = 0;
static uint64_t g_node_lock_passes = 0;

static uint64_t replay(const Plan& p, uint64_t nchunks, bool pad) {
    uint64_t c = nchunks;
    for (size_t i = 0; i < p.passes.size(); ++i) {
        const Pass& ps = p.passes[i];
        const uint64_t c1 = (c > 1 || pad) ? ceil_div(c, 2) : 1;
        REQUIRE(ps.a.c1 == c1);
        if (!ps.leaf) REQUIRE(ps.a.cin == c);
        REQUIRE(ps.in_ws == (i == 0 ? -1 : p.passes[i - 1].out_ws));
        c = c1;
        const uint32_t lv = ps.a.finalize ? 64u : ps.a.levels;
        for (uint32_t l = 1; l < lv; ++l) {
            if (c <= 1 && !pad) break;
            c = ceil_div(c, 2);
        }
        if (ps.out_ws >= 0) REQUIRE(p.slot_nodes[ps.out_ws] >= c);
        if (ps.nlock && ps.leaf) {  // k_leaf_lock: whole groups of 4 full spans, exactly 3 levels, never the final pass
            ++g_lock_passes;
            REQUIRE(!ps.wave && !ps.sp && ps.ni == 2 && !ps.a.finalize && ps.a.levels == 3);
            REQUIRE(4 * ps.nlock <= ps.nfast && ps.nfast * 2 * ps.ni * kReduceThreads <= ps.a.c1_full);
        }
        if (ps.nlock && !ps.leaf) {  // k_node_lock: whole multiples of 256 groups of 16 full spans, exactly 5 levels
            ++g_node_lock_passes;
            REQUIRE(!ps.wave && !ps.sp && ps.ni == 2 && !ps.a.finalize && ps.a.levels == kNodeLockLevels);
            REQUIRE(ps.nlock % 256 == 0 && kNodeLockSpans * ps.nlock <= ps.nfast);
            REQUIRE(ps.nlock * 1024 * kNodeLockPairs <= ps.a.c1_full && ps.a.c1_full == ps.a.cin / 2);
        }
        REQUIRE(ps.nfast <= ps.nwg);
        REQUIRE(ps.nwg >= 1);
    }
    return c;
}

int main(int argc, char** argv) {
    const uint64_t seed = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1;
    const int cases = argc > 2 ? std::atoi(argv[2]) : 2000;
    std::mt19937_64 rng(seed);
    auto pick = [&](uint64_t lo, uint64_t hi) { return lo + rng() % (hi - lo + 1); };
    for (int t = 0; t < cases; ++t) {
        const uint64_t n = rng() % 4 == 0 ? pick(0, 64) : pick(0, 1ull << 22);
        const uint32_t il = rng() % 3 == 0 ? 32 : (uint32_t)pick(1, 300);
        const uint64_t cb = n ? chunk_bytes(il) : 128;
        const uint64_t nchunks = n ? ceil_div(n * (uint64_t)il, cb) : 0;
        // full merkleHash plan
        Plan p;
        int rc = make_plan(n, il, false, 0, false, rng() & 1, p);
        REQUIRE(rc == MK_OK);
        if (nchunks <= 1) {
            REQUIRE(p.small);
        } else {
            REQUIRE(!p.small && !p.passes.empty() && p.passes.back().a.finalize);
            REQUIRE(replay(p, nchunks, false) == 1);
            REQUIRE(plan_ws_bytes(p) >= 32 * (p.slot_nodes[0] + p.slot_nodes[1]));
        }
        // the element-digest tree's plan (k_reduce_elem: one window pair per
        // thread in throughput leaf passes): same tree, NI = 1 leaf workgroups
        if (n > 4) {
            Plan ep;
            REQUIRE(make_plan(n, 32, false, 0, false, true, ep, false, 0, 0, true) == MK_OK);
            REQUIRE(!ep.small && replay(ep, ceil_div(n, 4), false) == 1);
            const Pass& lp = ep.passes[0];
            if (!lp.wave && !lp.sp) REQUIRE(lp.ni == 1 && lp.nwg == ceil_div(lp.a.c1, 2 * kReduceThreads));
        }
        // shard plan + per-shard frontier plans
        const uint32_t world = (uint32_t)pick(1, 16);
        uint32_t h = 0, ne = 0;
        std::vector<uint64_t> begin(world + 1);
        REQUIRE(shard_plan(n, il, world, &h, &ne, begin.data()) == MK_OK);
        REQUIRE(begin[0] == 0 && begin[world] == n);
        std::printf("S %llu %u %u %u %u", (unsigned long long)n, il, world, h, ne);
        for (uint32_t s = 0; s <= world; ++s) {
            std::printf(" %llu", (unsigned long long)begin[s]);
            if (s) REQUIRE(begin[s] >= begin[s - 1]);
        }
        std::printf("\n");
        if (ne > 1) {
            for (uint32_t s = 0; s < ne; ++s) {
                const uint64_t sn = begin[s + 1] - begin[s];
                const uint64_t sch = ceil_div(sn * (uint64_t)il, cb);
                REQUIRE(sch >= 1 && sch <= (1ull << h));
                Plan sp;
                REQUIRE(make_plan(sn, il, true, h, true, true, sp) == MK_OK);
                REQUIRE(replay(sp, sch, true) == 1);
                const uint32_t k = h > 1 ? (uint32_t)pick(1, h - 1) : 0;
                if (!k) continue;
                Plan fp;
                rc = make_plan(sn, il, true, h, true, true, fp, false, k);
                if (rc != MK_OK) {  // the planner refuses a single-level throughput pass; say so
                    REQUIRE(h - k == 1);
                    continue;
                }
                REQUIRE(fp.out_nodes == frontier_nodes(sn, il, h, k));
                REQUIRE(replay(fp, sch, true) == fp.out_nodes);
                std::printf("F %llu %u %u %u %llu\n", (unsigned long long)sn, il, h, k,
                            (unsigned long long)fp.out_nodes);
            }
        }
        // node-input finisher plan over a gathered level
        const uint64_t cnt = pick(2, 1ull << 16);
        Plan np;
        REQUIRE(make_plan(cnt, 32, false, 0, false, true, np, true, 0, n) == MK_OK);
        REQUIRE(replay(np, cnt, false) == 1);
        // many lists
        const uint32_t nl = (uint32_t)pick(0, 40);
        std::vector<uint64_t> ns(nl), offs(nl);
        std::vector<uint32_t> ils(nl);
        uint64_t pos = 0;
        for (uint32_t i = 0; i < nl; ++i) {
            ns[i] = rng() % 5 == 0 ? pick(0, 3) : pick(0, rng() % 7 == 0 ? 200000 : 3000);
            ils[i] = rng() % 2 ? 32 : (uint32_t)pick(1, 200);
            offs[i] = pos;
            pos += ns[i] * ils[i] + pick(0, 20);
        }
        ManyPlan mp;
        REQUIRE(make_many_plan(offs.data(), ns.data(), ils.data(), nl, pos, true, mp) == MK_OK);
        REQUIRE(mp.lvl_begin.size() == mp.nlevels + 1 && mp.lvl_nodes.size() == mp.nlevels);
        for (uint32_t l = 0; l < mp.nlevels; ++l) {
            uint64_t expect = 0;
            for (uint64_t e = mp.lvl_begin[l]; e < mp.lvl_begin[l + 1]; ++e) {
                const ManyAct& A = mp.act[e];
                const ManyList& L = mp.lists[A.list];
                REQUIRE(A.level == l + 1 && A.out_first == expect);
                expect += ceil_div(L.c1, 1ull << l);
            }
            REQUIRE(expect == mp.lvl_nodes[l] && expect <= mp.buf_nodes[l % 2]);
        }
        REQUIRE(mp.off_tops + 32 * nl <= mp.off_buf0);
        REQUIRE(mp.off_big + 256 <= mp.ws_bytes);
        std::printf("M %u %u %llu\n", nl, mp.nlevels, (unsigned long long)mp.ws_bytes);
        // deposit-trie layout: levels are disjoint and in order
        const uint64_t cap = pick(1, 1ull << 20);
        for (uint32_t d = 0; d < 33; ++d) REQUIRE(trie_level_off(cap, d + 1) == trie_level_off(cap, d) + trie_count(cap, d));
    }
    // wide node passes (k_node_lock): whole trees of 2^27..2^29 32-B items and
    // node-input plans of >= 2^23 nodes, ragged and aligned; planning only
    const uint64_t wide[] = {1ull << 27, (1ull << 28) - 1, 1ull << 28, (1ull << 28) + 5, 3ull << 27, 1ull << 29};
    for (uint64_t n : wide) {
        Plan wp;
        REQUIRE(make_plan(n, 32, false, 0, false, true, wp) == MK_OK);
        REQUIRE(replay(wp, ceil_div(n, 4), false) == 1);
        const uint64_t cnt = n / 32 + (n & 7);
        Plan np;
        REQUIRE(make_plan(cnt, 32, false, 0, false, true, np, true, 0, n) == MK_OK);
        REQUIRE(replay(np, cnt, false) == 1);
        REQUIRE(make_plan(cnt, 32, false, 0, false, false, np, true, 0, n) == MK_OK);  // unaligned: no lock
        REQUIRE(np.passes[0].nlock == 0 && replay(np, cnt, false) == 1);
    }
    {
        Plan wp;  // the 2^28 headline: leaf lock, then one node-lock pass of 256 groups
        REQUIRE(make_plan(1ull << 28, 32, false, 0, false, true, wp) == MK_OK);
        REQUIRE(wp.passes.size() >= 2 && wp.passes[1].nlock == 256 && wp.passes[1].nfast == 16 * 256);
    }
    // invalid inputs are rejected, not crashed on
    Plan p;
    REQUIRE(make_plan(5, 0, false, 0, false, true, p) == MK_EINVAL);
    REQUIRE(make_plan(1ull << 40, 32, true, 10, true, true, p) == MK_EINVAL);
    REQUIRE(make_plan(100, 32, true, 64, true, true, p) == MK_EINVAL);
    REQUIRE(make_plan(UINT64_MAX, 300, false, 0, false, true, p) == MK_EINVAL);
    uint32_t h, ne;
    uint64_t b[2];
    REQUIRE(shard_plan(5, 32, 0, &h, &ne, b) == MK_EINVAL);
    std::fprintf(stderr, "planner fuzz: %d cases clean (%llu phase-locked leaf passes, %llu node passes)\n", cases,
                 (unsigned long long)g_lock_passes, (unsigned long long)g_node_lock_passes);
    return 0;
}
