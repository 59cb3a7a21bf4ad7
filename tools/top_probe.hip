// Diagnostic probe: per-level timeline of the fused trie top
// (k_trie_top_fused) from in-kernel s_memtime stamps (-DMK_TOP_STAMPS=1, a
// build of the kernel source of its own, never the shipped library).  A
// depth-32 trie's level-2 nodes (2^18 random, the C5 shape) reduced to the
// root `iters` times; prints, per stamp, the median over workgroups of the
// cycles since the workgroup's first stamp, and the last workgroup's stamps.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DMK_TOP_STAMPS=1
//        -I../prysm_amd/csrc -I../include top_probe.hip -o top_probe
#include "../prysm_amd/csrc/merkle_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

static void print_wgs(const std::vector<uint64_t>& st, uint32_t b0, uint32_t b1, const char* name) {
    // the workgroup of [b0, b1) with the most stamps (the last arriver), cycles between its stamps
    uint32_t lb = b0, best = 0;
    for (uint32_t b = b0; b < b1; ++b) {
        uint32_t k = 0;
        while (k < 64 && st[b * 64 + k]) ++k;
        if (k > best) best = k, lb = b;
    }
    printf("\"%s\": {\"wg\": %u, \"level_cycles\": [", name, lb);
    for (uint32_t k = 1; k < best; ++k)
        printf("%s%llu", k > 1 ? ", " : "", (unsigned long long)(st[lb * 64 + k] - st[lb * 64 + k - 1]));
    printf("], \"total\": %llu}", (unsigned long long)(st[lb * 64 + best - 1] - st[lb * 64]));
}

// C3's fused list top (k_merkle_top_fused): 125,000 registry + 31,250
// balances level-1 nodes, spans 1024 / 256 (capi.cpp top_plan)
static int merkle_probe(int iters) {
    const uint64_t c0 = 125000, c1 = 31250;
    uint32_t *n0, *n1, *ws, *pair;
    (void)hipMalloc(&n0, c0 * 32);
    (void)hipMalloc(&n1, c1 * 32);
    (void)hipMalloc(&ws, 1 << 16);
    (void)hipMalloc(&pair, 128);
    (void)hipMemset(n0, 0x5A, c0 * 32);
    (void)hipMemset(n1, 0xA5, c1 * 32);
    (void)hipMemset(pair, 0, 128);
    mk::MerkleTopArgs a{};
    a.nlists = 2;
    a.pair = pair;
    const uint32_t sl[2] = {10, 8};
    const uint64_t c[2] = {c0, c1};
    uint32_t* nodes[2] = {n0, n1};
    uint32_t wg = 0;
    for (int l = 0; l < 2; ++l) {
        a.l[l].nodes = (const uint4*)nodes[l];
        a.l[l].c = c[l];
        a.l[l].n_items = 1000000;
        a.l[l].sub = ws + 8 * wg;
        a.l[l].out = pair + 8 * l;
        a.l[l].wg0 = wg;
        a.l[l].nwg = (uint32_t)((c[l] + (1u << sl[l]) - 1) >> sl[l]);
        a.l[l].span_log2 = sl[l];
        wg += a.l[l].nwg;
    }
    std::vector<uint64_t> zero(1024 * 64, 0), st(1024 * 64);
    for (int it = 0; it < iters; ++it) {
        a.pair_slot = 4000 + it % 30;
        a.l[0].slot = (2 * (it % 10)) * mk::kTopGroupSlots;
        a.l[1].slot = (2 * (it % 10) + 1) * mk::kTopGroupSlots;
        if (it + 1 == iters) (void)hipMemcpyToSymbol(HIP_SYMBOL(mk::g_top_stamps), zero.data(), zero.size() * 8);
        hipLaunchKernelGGL(mk::k_merkle_top_fused<1024>, dim3(wg), dim3(1024), 0, 0, a);
        (void)hipDeviceSynchronize();
    }
    (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(mk::g_top_stamps), st.size() * 8);
    printf("{\"merkle_top\": {");
    print_wgs(st, 0, a.l[0].nwg, "registry");
    printf(", ");
    print_wgs(st, a.l[1].wg0, wg, "balances");
    printf("}}\n");
    return 0;
}

// The whole-trie front (k_trie_rec_lock_sm) over 2^20 random 280-B
// deposits, `iters` times: per workgroup its start and end on the 100-MHz
// s_memrealtime clock (g_front_stamps), to see how far apart the workgroups
// finish -- the time a top fused into the front could start early.
static int front_probe(int iters) {
    const uint64_t n = 1u << 20;
    uint2* in;
    uint4 *l0, *l1, *l2;
    (void)hipMalloc(&in, n * 280);
    (void)hipMalloc(&l0, n * 32);
    (void)hipMalloc(&l1, n * 16);
    (void)hipMalloc(&l2, n * 8);
    (void)hipMemset(in, 0x3C, n * 280);
    const uint64_t ngroups = n / 4096;
    std::vector<uint64_t> st(2 * 1024);
    for (int it = 0; it < iters; ++it) {
        hipLaunchKernelGGL(mk::k_trie_rec_lock_sm<1024>, dim3((uint32_t)ngroups), dim3(1024), 0, 0, in, ngroups, l0,
                           l1, l2);
        (void)hipDeviceSynchronize();
    }
    (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(mk::g_front_stamps), st.size() * 8);
    std::vector<uint64_t> s0, s1, dur;
    for (uint64_t b = 0; b < ngroups; ++b) {
        s0.push_back(st[2 * b]);
        s1.push_back(st[2 * b + 1]);
        dur.push_back(st[2 * b + 1] - st[2 * b]);
    }
    const uint64_t t0 = *std::min_element(s0.begin(), s0.end());
    std::sort(s0.begin(), s0.end());
    std::sort(s1.begin(), s1.end());
    std::sort(dur.begin(), dur.end());
    auto us = [](uint64_t t) { return t / 100.0; };  // 100-MHz ticks -> us
    printf("{\"front_wgs\": %llu, \"start_us\": [%.2f, %.2f, %.2f], \"end_us\": [%.2f, %.2f, %.2f, %.2f], "
           "\"dur_us\": [%.2f, %.2f, %.2f]}\n",
           (unsigned long long)ngroups, us(s0.front() - t0), us(s0[s0.size() / 2] - t0), us(s0.back() - t0),
           us(s1.front() - t0), us(s1[s1.size() / 10] - t0), us(s1[s1.size() / 2] - t0), us(s1.back() - t0),
           us(dur.front()), us(dur[dur.size() / 2]), us(dur.back()));
    // mean end (us after the first start) per XCD (workgroup b on XCD b mod 8)
    printf("{\"end_us_by_xcd\": [");
    for (int x = 0; x < 8; ++x) {
        double sum = 0;
        int k = 0;
        for (uint64_t b = x; b < ngroups; b += 8, ++k) sum += us(st[2 * b + 1] - t0);
        printf("%s%.2f", x ? ", " : "", sum / k);
    }
    printf("], \"slowest_wgs\": [");
    std::vector<std::pair<uint64_t, uint64_t>> e;
    for (uint64_t b = 0; b < ngroups; ++b) e.push_back({st[2 * b + 1], b});
    std::sort(e.begin(), e.end());
    for (int k = 0; k < 16; ++k) printf("%s%llu", k ? ", " : "", (unsigned long long)e[e.size() - 1 - k].second);
    printf("]}\n");
    return 0;
}

// The C4 leaf pass (k_leaf_lock_sc) over 2^28 32-B items, one workgroup per
// CU (256, 32 groups of 4,096 windows each, statically strided): per
// workgroup its end on the 100-MHz clock, per XCD the mean, to see whether a
// slow XCD leaves a tail behind a static group assignment.
static int leaf_probe(int iters) {
    const uint64_t n = 1ull << 28, windows = n * 32 / 256, ngroups = windows / 4096;
    uint8_t* items;
    uint8_t* out;
    if (hipMalloc(&items, n * 32) != hipSuccess || hipMalloc(&out, ngroups * 1024 * 32) != hipSuccess) return 1;
    (void)hipMemset(items, 0x5A, n * 32);
    mk::ReduceArgs a{};
    a.items = items;
    a.out = out;
    const uint32_t grid = 256;
    std::vector<uint64_t> st(2 * 1024);
    for (int it = 0; it < iters; ++it) {
        hipLaunchKernelGGL(mk::k_leaf_lock_sc, dim3(grid), dim3(1024), 0, 0, a, ngroups);
        (void)hipDeviceSynchronize();
        (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(mk::g_leaf_stamps), st.size() * 8);
        uint64_t t0 = ~0ull, e0 = ~0ull, e1 = 0;
        for (uint32_t b = 0; b < grid; ++b) {
            t0 = std::min(t0, st[2 * b]);
            e0 = std::min(e0, st[2 * b + 1]);
            e1 = std::max(e1, st[2 * b + 1]);
        }
        printf("{\"leaf_wgs\": %u, \"groups\": %llu, \"first_end_us\": %.1f, \"last_end_us\": %.1f, \"end_us_by_xcd\": [",
               grid, (unsigned long long)ngroups, (e0 - t0) / 100.0, (e1 - t0) / 100.0);
        for (int x = 0; x < 8; ++x) {
            double sum = 0, mx = 0;
            int k = 0;
            for (uint32_t b = x; b < grid; b += 8, ++k) {
                sum += (st[2 * b + 1] - t0) / 100.0;
                mx = std::max(mx, (st[2 * b + 1] - t0) / 100.0);
            }
            printf("%s[%.1f, %.1f]", x ? ", " : "", sum / k, mx);
        }
        printf("]}\n");
        fflush(stdout);
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 2 && argv[2][0] == 'l') return leaf_probe(atoi(argv[1]));
    if (argc > 2 && argv[2][0] == 'f') return front_probe(atoi(argv[1]));
    if (argc > 2) return merkle_probe(atoi(argv[1]));
    const uint64_t n = 1u << 20, cap = n;
    const uint32_t depth = 32, d0 = 2;
    const int iters = argc > 1 ? atoi(argv[1]) : 5;
    uint64_t total = 0, c = cap;
    for (uint32_t d = 0; d <= depth; ++d) {
        total += c;
        c = (c + 1) / 2;
    }
    uint32_t *lv, *root;
    (void)hipMalloc(&lv, total * 32);
    (void)hipMalloc(&root, 32);
    std::vector<uint32_t> h(total * 8);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto& v : h) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        v = (uint32_t)x;
    }
    (void)hipMemcpy(lv, h.data(), total * 32, hipMemcpyHostToDevice);
    const uint64_t c0 = n >> d0;
    const uint32_t grid = (uint32_t)((c0 + 1023) / 1024);
    std::vector<uint64_t> zero(1024 * 64, 0);
    for (int it = 0; it < iters; ++it) {
        if (it + 1 == iters) (void)hipMemcpyToSymbol(HIP_SYMBOL(mk::g_top_stamps), zero.data(), zero.size() * 8);
        hipLaunchKernelGGL(mk::k_trie_top_fused<1024>, dim3(grid), dim3(1024), 0, 0, lv, cap, c0, d0, depth, root,
                           (uint32_t)(it % 30) * mk::kTopGroupSlots);
        (void)hipDeviceSynchronize();
    }
    std::vector<uint64_t> st(1024 * 64);
    (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(mk::g_top_stamps), st.size() * 8);
    // per stamp index: median over workgroups of (stamp - stamp 0) where set
    uint64_t t0min = ~0ull;
    for (uint32_t b = 0; b < grid; ++b) t0min = std::min(t0min, st[b * 64]);
    printf("{\"grid\": %u, \"stamps_median_cycles\": [", grid);
    for (int k = 0; k < 13; ++k) {
        std::vector<uint64_t> v;
        for (uint32_t b = 0; b < grid; ++b)
            if (st[b * 64 + k]) v.push_back(st[b * 64 + k] - t0min);
        std::sort(v.begin(), v.end());
        printf("%s%llu", k ? ", " : "", v.empty() ? 0ull : (unsigned long long)v[v.size() / 2]);
    }
    // the last workgroup: the one with the most stamps
    uint32_t lb = 0, best = 0;
    for (uint32_t b = 0; b < grid; ++b) {
        uint32_t k = 0;
        while (k < 64 && st[b * 64 + k]) ++k;
        if (k > best) best = k, lb = b;
    }
    printf("], \"last_wg\": %u, \"last_wg_cycles\": [", lb);
    for (uint32_t k = 0; k < best; ++k) printf("%s%llu", k ? ", " : "", (unsigned long long)(st[lb * 64 + k] - t0min));
    printf("]}\n");
    return 0;
}
