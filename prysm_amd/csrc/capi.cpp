// C-ABI of the MI355X Merkleization engine: device management, the
// merkleHash pass planner, and the host/device entry points declared in
// include/prysm_merkle.h.  Compiled with hipcc into libprysm_merkle.so.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "merkle_kernels.hpp"
#include "prysm_merkle.h"

namespace {

using mk::ReduceArgs;
using mk::kReduceThreads;

#ifndef MK_SIDE_PRIO
#define MK_SIDE_PRIO 1
#endif
constexpr bool kSidePrio = MK_SIDE_PRIO != 0;  // library side/copy streams at high priority
#ifndef MK_WAVE2
#define MK_WAVE2 1
#endif
constexpr bool kWave2 = MK_WAVE2 != 0;  // two-lanes-per-state latency pass
#ifndef MK_WAVE3
#define MK_WAVE3 1
#endif
constexpr bool kWave3 = kWave2 && MK_WAVE3 != 0;  // node latency passes bit-interleaved (k_wave3)
#ifndef MK_NODE_WAVE_MAX_LOG2
#define MK_NODE_WAVE_MAX_LOG2 17
#endif
// node passes switch to the latency form at or below this width: the first
// level is throughput-bound either way, but the throughput kernel spends ~9
// serial permutations on its 5 levels where the wave pass spends 6
constexpr uint64_t kNodeWaveMaxC1 = 1ull << MK_NODE_WAVE_MAX_LOG2;
#ifndef MK_NODE_WAVE_WGS
#define MK_NODE_WAVE_WGS 256
#endif
constexpr uint64_t kNodeWaveWgs = MK_NODE_WAVE_WGS;
#ifndef MK_LEAF_WAVE3
#define MK_LEAF_WAVE3 1
#endif
constexpr bool kLeafWave3 = MK_LEAF_WAVE3 != 0;  // narrow leaf passes bit-interleaved too
#ifndef MK_LEAF_WAVE_MAX_LOG2
#define MK_LEAF_WAVE_MAX_LOG2 17
#endif
constexpr uint64_t kLeafWaveMaxC1 = 1ull << MK_LEAF_WAVE_MAX_LOG2;  // leaf passes at or below: latency form
#ifndef MK_REDUCE_NI2_MIN_LOG2
#define MK_REDUCE_NI2_MIN_LOG2 18
#endif
constexpr uint64_t kReduceNi2MinC1 = 1ull << MK_REDUCE_NI2_MIN_LOG2;  // leaf passes narrower than this use NI = 1
#ifndef MK_TOP_ONE_WG
#define MK_TOP_ONE_WG 1
#endif
constexpr bool kTopOneWg = MK_TOP_ONE_WG != 0;
#ifndef MK_REC_KERNEL
#define MK_REC_KERNEL 1
#endif
constexpr bool kRecKernel = MK_REC_KERNEL != 0;  // k_keccak_rec<35> for 280-B deposit leaves
#ifndef MK_STRUCT_FUSED
#define MK_STRUCT_FUSED 1
#endif
constexpr bool kStructFused = MK_STRUCT_FUSED != 0;  // k_struct_fused instead of fields + message kernels
uint32_t ilog2(uint64_t v) {
    uint32_t l = 0;
    while (v > 1) {
        v >>= 1;
        ++l;
    }
    return l;
}

thread_local std::string t_err;
thread_local int t_dev = -1;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_err = buf;
    return code;
}

#define HIPCHK(x)                                                                            \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) return fail(MK_EHIP, "%s: %s", #x, hipGetErrorString(e_));     \
    } while (0)

// ---- devices ---------------------------------------------------------------
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

struct DevCtx {
    std::mutex mu;
    hipStream_t stream = nullptr;
    DevBuf in, out, ws, aux, aux2;
    // side stream + events: the ragged last workgroup of a pass runs
    // concurrently with the pass's full workgroups (fork/join on events)
    std::mutex side_mu;
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    // host-buffer entries: records copied in chunks on `copy` while the
    // compute stream hashes the previous chunk (guarded by `mu`)
    hipStream_t copy = nullptr;
    hipEvent_t h2d = nullptr;
};

std::mutex g_mu;
int g_ndev = -1;
std::vector<DevCtx*> g_ctx;

int probe_devices() {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ndev >= 0) return g_ndev;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    int good = 0;
    for (int d = 0; d < n; ++d) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) != hipSuccess) break;
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) break;  // gfx950 only
        ++good;
    }
    g_ndev = good;
    g_ctx.resize(good, nullptr);
    return g_ndev;
}

int bind(int dev) {
    if (probe_devices() <= 0) return fail(MK_ENODEV, "no gfx950 device visible");
    if (dev < 0) dev = t_dev >= 0 ? t_dev : 0;
    if (dev >= g_ndev) return fail(MK_ENODEV, "device %d out of range (%d visible)", dev, g_ndev);
    HIPCHK(hipSetDevice(dev));
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!g_ctx[dev]) {
            auto* c = new DevCtx();
            // side/copy streams at the highest priority: a default-priority
            // stream can share the caller's hardware queue (GPU_MAX_HW_QUEUES=4)
            // and then runs after, not beside, the work it should overlap
            int lo = 0, hi = 0;
            if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess || !kSidePrio) hi = lo = 0;
            if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
                hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, hi) != hipSuccess ||
                hipEventCreateWithFlags(&c->fork, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&c->join, hipEventDisableTiming) != hipSuccess ||
                hipStreamCreateWithPriority(&c->copy, hipStreamNonBlocking, hi) != hipSuccess ||
                hipEventCreateWithFlags(&c->h2d, hipEventDisableTiming) != hipSuccess) {
                delete c;
                return fail(MK_EHIP, "stream/event creation failed on device %d", dev);
            }
            g_ctx[dev] = c;
        }
    }
    t_dev = dev;
    return MK_OK;
}

int grow(DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return MK_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    if (hipMalloc(&b.p, bytes) != hipSuccess) return fail(MK_ENOMEM, "hipMalloc(%zu) failed", bytes);
    b.cap = bytes;
    return MK_OK;
}

#define TRY(x)                      \
    do {                            \
        int rc_ = (x);              \
        if (rc_ != MK_OK) return rc_; \
    } while (0)

// ---- measurement -------------------------------------------------------------
struct ProfRec {
    hipEvent_t a, b;
    double perms, hashes;
};
std::mutex g_prof_mu;
bool g_prof_on = false;
std::vector<ProfRec> g_prof;

// ---- merkleHash planner ---------------------------------------------------------
uint64_t chunk_bytes(uint32_t item_len) {
    return item_len < 128 ? (uint64_t)(128 / item_len) * item_len : item_len;
}
uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
uint64_t perms_for_len(uint64_t len) { return len / 136 + 1; }

struct Pass {
    bool leaf;
    bool wave;  // latency pass (k_wave) instead of the throughput pass (k_reduce)
    uint64_t nwg, nfast;
    bool w3;      // k_wave3 (bit-interleaved latency form)
    uint32_t nt;  // threads per workgroup
    uint32_t ni;  // k_reduce: window pairs per thread (span 512 * ni)
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

// Hashing levels from `count` nodes down to one (reference loop length).
uint32_t levels_to_one(uint64_t count) {
    uint32_t l = 0;
    while (count > 1) {
        count = (count + 1) / 2;
        ++l;
    }
    return l;
}

// Builds the pass sequence.  subtree=false: full merkleHash with the length
// mix-in; subtree=true: exactly `height` levels above the chunks, output one
// node (pad_at_one keeps the odd rule alive at count 1).
// node_input: the input is n 32-B nodes reduced pairwise (a plain binary
// tree, no chunking; hashutil.MerkleRoot's heap bands, or a gathered tree
// level for the multi-GPU finisher).  Without subtree mode the final pass
// mixes in `mixin_n` (the item count of the whole tree), n must be >= 2.
// frontier (subtree mode): stop `frontier` levels below the subtree root and
// write the level there (2^frontier nodes, fewer for a ragged shard).
int make_plan(uint64_t n, uint32_t item_len, bool subtree, uint32_t height, bool pad_at_one,
              bool aligned16, Plan& p, bool node_input = false, uint32_t frontier = 0, uint64_t mixin_n = 0) {
    p = Plan();
    p.n = n;
    if (n > 0 && item_len == 0) return fail(MK_EINVAL, "item_len == 0 (reference: integer divide by zero)");
    if (node_input && item_len != 32) return fail(MK_EINVAL, "planner: node input is 32-B nodes");
    if (node_input && !subtree && n < 2) return fail(MK_EINVAL, "planner: node finisher needs >= 2 nodes");
    if (frontier && (!subtree || frontier >= height)) return fail(MK_EINVAL, "planner: bad frontier %u", frontier);
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
        const bool wave = c1 <= (leaf || !kWave3 ? kLeafWaveMaxC1 : kNodeWaveMaxC1);
        const bool w3 = kWave3 && wave && (!leaf || kLeafWave3);
        // k_wave3: the smallest workgroup (64..1024 threads, 2 per pair) that
        // keeps the pass within ~256 workgroups, one per CU
        uint32_t nt = w3 ? mk::kWaveThreads : (wave ? mk::kWaveThreads : kReduceThreads);
        if (w3) {
            while (nt < mk::kMidThreads && ceil_div(c1, nt / 2) > kNodeWaveWgs) nt *= 2;
            if (kTopOneWg)  // the last <= 512 pairs in one workgroup: one launch to the root
                while (nt < mk::kMidThreads && c1 <= mk::kMidThreads / 2 && c1 > nt / 2) nt *= 2;
        }
        // throughput pass: 2 window pairs per thread on wide passes, 1 on mid-size
        // leaf passes so they still spread over the CUs
        const uint32_t ni = (!wave && leaf && c1 < kReduceNi2MinC1) ? 1 : 2;
        const uint64_t span = w3 ? nt / 2 : wave ? (kWave2 ? mk::kWave2Span : mk::kWaveThreads)
                                                 : (uint64_t)2 * ni * kReduceThreads;
        const bool final_pass = c1 <= span;
        const uint32_t max_lv = w3 ? 1 + ilog2(nt / 2)
                              : wave ? (kWave2 ? mk::kWave2Levels : mk::kWaveLevels) : mk::kMaxPassLevels;
        uint32_t lv = final_pass ? remaining : std::min<uint32_t>(max_lv, remaining);
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
        a.out_ilv = w3 ? 1 : 0;  // cleared below for the final pass
        a.levels = lv;
        ps.nwg = ceil_div(c1, span);
        ps.nfast = wave ? 0 : std::min<uint64_t>(ps.nwg, a.c1_full / span);
        ps.ni = ni;
        ps.in_ws = in_slot;
        if (final_pass) {
            if (!subtree) {
                a.finalize = 1;
                a.levels = 64;
            } else if (!wave && c1 > span / 2 && lv < 2) {
                return fail(MK_EINVAL, "planner: unsupported single-level pass");
            }
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

template <bool LEAF>
void launch_wave3(uint32_t nt, uint64_t nwg, const ReduceArgs& a, hipStream_t st) {
    switch (nt) {
        case 64: hipLaunchKernelGGL((mk::k_wave3<64, LEAF>), dim3(nwg), dim3(64), 0, st, a); break;
        case 128: hipLaunchKernelGGL((mk::k_wave3<128, LEAF>), dim3(nwg), dim3(128), 0, st, a); break;
        case 256: hipLaunchKernelGGL((mk::k_wave3<256, LEAF>), dim3(nwg), dim3(256), 0, st, a); break;
        case 512: hipLaunchKernelGGL((mk::k_wave3<512, LEAF>), dim3(nwg), dim3(512), 0, st, a); break;
        default: hipLaunchKernelGGL((mk::k_wave3<1024, LEAF>), dim3(nwg), dim3(1024), 0, st, a); break;
    }
}

uint64_t plan_ws_bytes(const Plan& p) { return 32 * (p.slot_nodes[0] + p.slot_nodes[1]) + 256; }

int launch_plan(const Plan& p, const uint8_t* d_items, uint8_t* d_out32, uint8_t* d_ws, uint64_t ws_bytes,
                hipStream_t st) {
    if (p.small) {
        hipLaunchKernelGGL(mk::k_final_small, dim3(1), dim3(64), 0, st, d_items, p.total, p.n, d_out32);
        HIPCHK(hipGetLastError());
        return MK_OK;
    }
    if (ws_bytes < plan_ws_bytes(p)) return fail(MK_ENOMEM, "workspace too small: %llu < %llu",
                                                 (unsigned long long)ws_bytes, (unsigned long long)plan_ws_bytes(p));
    uint8_t* slots[2] = {d_ws, d_ws + 32 * p.slot_nodes[0]};
    bool prof;
    {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        prof = g_prof_on;
    }
    for (const Pass& ps : p.passes) {
        ReduceArgs a = ps.a;
        a.items = ps.in_ws < 0 ? d_items : slots[ps.in_ws];
        a.out = ps.out_ws < 0 ? d_out32 : slots[ps.out_ws];
        ProfRec rec{};
        const bool rec_this = prof && ps.leaf;
        if (rec_this) {
            HIPCHK(hipEventCreate(&rec.a));
            HIPCHK(hipEventCreate(&rec.b));
            HIPCHK(hipEventRecord(rec.a, st));
        }
        if (ps.wave) {
            a.wg_base = 0;
            if (ps.w3) {
                if (ps.leaf)
                    launch_wave3<true>(ps.nt, ps.nwg, a, st);
                else
                    launch_wave3<false>(ps.nt, ps.nwg, a, st);
            } else if (kWave2) {
                if (ps.leaf)
                    hipLaunchKernelGGL((mk::k_wave2<true>), dim3(ps.nwg), dim3(mk::kWaveThreads), 0, st, a);
                else
                    hipLaunchKernelGGL((mk::k_wave2<false>), dim3(ps.nwg), dim3(mk::kWaveThreads), 0, st, a);
            } else {
                if (ps.leaf)
                    hipLaunchKernelGGL((mk::k_wave<true>), dim3(ps.nwg), dim3(mk::kWaveThreads), 0, st, a);
                else
                    hipLaunchKernelGGL((mk::k_wave<false>), dim3(ps.nwg), dim3(mk::kWaveThreads), 0, st, a);
            }
            HIPCHK(hipGetLastError());
        } else {
            // The ragged workgroup(s) of a pass are latency-bound; when the pass
            // also has full workgroups they go first, on the side stream, so
            // they overlap the full ones (fork/join through events on `st`).
            const bool ragged = ps.nwg > ps.nfast;
            DevCtx* c = (ragged && ps.nfast) ? g_ctx[t_dev] : nullptr;
            std::unique_lock<std::mutex> lk;
            if (ragged) {
                hipStream_t gs = st;
                if (c) {
                    lk = std::unique_lock<std::mutex>(c->side_mu);
                    HIPCHK(hipEventRecord(c->fork, st));
                    HIPCHK(hipStreamWaitEvent(c->side, c->fork, 0));
                    gs = c->side;
                }
                ReduceArgs g = a;
                g.wg_base = ps.nfast;
                if (ps.leaf && ps.ni == 1)
                    hipLaunchKernelGGL((mk::k_reduce<true, false, 1>), dim3(ps.nwg - ps.nfast), dim3(kReduceThreads),
                                       0, gs, g);
                else if (ps.leaf)
                    hipLaunchKernelGGL((mk::k_reduce<true, false, 2>), dim3(ps.nwg - ps.nfast), dim3(kReduceThreads),
                                       0, gs, g);
                else
                    hipLaunchKernelGGL((mk::k_reduce<false, false, 2>), dim3(ps.nwg - ps.nfast), dim3(kReduceThreads),
                                       0, gs, g);
                HIPCHK(hipGetLastError());
                if (c) HIPCHK(hipEventRecord(c->join, c->side));
            }
            if (ps.nfast) {
                a.wg_base = 0;
                if (ps.leaf && ps.ni == 1)
                    hipLaunchKernelGGL((mk::k_reduce<true, true, 1>), dim3(ps.nfast), dim3(kReduceThreads), 0, st, a);
                else if (ps.leaf)
                    hipLaunchKernelGGL((mk::k_reduce<true, true, 2>), dim3(ps.nfast), dim3(kReduceThreads), 0, st, a);
                else
                    hipLaunchKernelGGL((mk::k_reduce<false, true, 2>), dim3(ps.nfast), dim3(kReduceThreads), 0, st, a);
                HIPCHK(hipGetLastError());
            }
            if (c) HIPCHK(hipStreamWaitEvent(st, c->join, 0));
        }
        if (rec_this) {
            HIPCHK(hipEventRecord(rec.b, st));
            rec.perms = ps.perms;
            rec.hashes = ps.hashes;
            std::lock_guard<std::mutex> lk(g_prof_mu);
            g_prof.push_back(rec);
        }
    }
    return MK_OK;
}

struct Locked {
    DevCtx* c;
    std::unique_lock<std::mutex> lk;
};

int lock_current(Locked& L) {
    TRY(bind(-1));
    L.c = g_ctx[t_dev];
    L.lk = std::unique_lock<std::mutex>(L.c->mu);
    return MK_OK;
}

int shard_plan(uint64_t n, uint32_t item_len, uint32_t nshards, uint32_t* height, uint32_t* nonempty,
               uint64_t* begin) {
    if (nshards == 0) return fail(MK_EINVAL, "nshards == 0");
    if (n > 0 && item_len == 0) return fail(MK_EINVAL, "item_len == 0");
    const uint64_t total = n * (uint64_t)item_len;
    const uint64_t cb = n ? chunk_bytes(item_len) : 128;
    const uint64_t per_chunk_items = item_len < 128 ? 128 / item_len : 1;
    const uint64_t nchunks = n ? ceil_div(total, cb) : 0;
    uint32_t h = 0;
    while ((1ull << h) * nshards < nchunks) ++h;
    uint64_t ne = nchunks ? ceil_div(nchunks, 1ull << h) : 0;
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

}  // namespace

// =============================================================================
extern "C" {

const char* mk_version(void) { return "prysm_merkle 0.1 (gfx950)"; }

const char* mk_strerror(int code) {
    switch (code) {
        case MK_OK: return "ok";
        case MK_EINVAL: return "invalid argument";
        case MK_ENODEV: return "no usable gfx950 device";
        case MK_ENOMEM: return "out of memory";
        case MK_EHIP: return "HIP runtime error";
        case MK_ECOMM: return "RCCL error";
        default: return "unknown error";
    }
}

const char* mk_last_error(void) { return t_err.c_str(); }

int mk_device_count(void) { return probe_devices(); }

int mk_init(int device) { return bind(device < 0 ? 0 : device); }

// ---- hashing ------------------------------------------------------------------
int mk_dev_hash_batch(const void* d_in, uint64_t n, uint32_t msg_len, void* d_out, void* stream) {
    TRY(bind(-1));
    if (n == 0) return MK_OK;
    if (!d_in || !d_out) return fail(MK_EINVAL, "null pointer");
    hipStream_t st = (hipStream_t)stream;
    const uint64_t grid = ceil_div(n, 256);
    if (msg_len == 64 && ((uintptr_t)d_in % 16) == 0 && ((uintptr_t)d_out % 16) == 0)
        hipLaunchKernelGGL(mk::k_keccak64, dim3(grid), dim3(256), 0, st, (const uint4*)d_in, n, (uint4*)d_out);
    else if (kRecKernel && msg_len == 280 && ((uintptr_t)d_in % 8) == 0 && ((uintptr_t)d_out % 16) == 0)
        hipLaunchKernelGGL((mk::k_keccak_rec<35>),
                           dim3(std::min<uint64_t>(ceil_div(n, mk::kRecThreads), mk::kRecGridMax)),
                           dim3(mk::kRecThreads), 0, st, (const uint2*)d_in, n, (uint4*)d_out);
    else if (msg_len % 8 == 0 && msg_len > 0 && ((uintptr_t)d_in % 8) == 0 && ((uintptr_t)d_out % 16) == 0)
        hipLaunchKernelGGL(mk::k_keccak_words, dim3(grid), dim3(256), 0, st, (const uint2*)d_in, n, msg_len / 8,
                           (uint4*)d_out);
    else
        hipLaunchKernelGGL(mk::k_keccak_fixed, dim3(grid), dim3(256), 0, st, (const uint8_t*)d_in, n, msg_len,
                           (uint4*)d_out);
    HIPCHK(hipGetLastError());
    return MK_OK;
}

int mk_dev_hash_batch_var(const void* d_in, const uint64_t* d_offs, uint64_t n, void* d_out, void* stream) {
    TRY(bind(-1));
    if (n == 0) return MK_OK;
    hipLaunchKernelGGL(mk::k_keccak_var, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const uint8_t*)d_in, d_offs, n, (uint4*)d_out);
    HIPCHK(hipGetLastError());
    return MK_OK;
}

int mk_hash_batch(const uint8_t* in, uint64_t n, uint32_t msg_len, uint8_t* out) {
    if (n && (!in && msg_len) ) return fail(MK_EINVAL, "null input");
    if (n && !out) return fail(MK_EINVAL, "null output");
    Locked L;
    TRY(lock_current(L));
    if (n == 0) return MK_OK;
    const size_t inb = n * (size_t)msg_len;
    TRY(grow(L.c->in, inb));
    TRY(grow(L.c->out, 32 * n));
    hipStream_t st = L.c->stream;
    if (inb) HIPCHK(hipMemcpyAsync(L.c->in.p, in, inb, hipMemcpyHostToDevice, st));
    TRY(mk_dev_hash_batch(L.c->in.p, n, msg_len, L.c->out.p, st));
    HIPCHK(hipMemcpyAsync(out, L.c->out.p, 32 * n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

int mk_hash(const uint8_t* data, uint64_t len, uint8_t out[32]) {
    if (len > UINT32_MAX) {
        uint64_t offs[2] = {0, len};
        return mk_hash_batch_var(data, offs, 1, out);
    }
    static const uint8_t empty = 0;
    return mk_hash_batch(len ? data : &empty, 1, (uint32_t)len, out);
}

int mk_hash_batch_var(const uint8_t* in, const uint64_t* offs, uint64_t n, uint8_t* out) {
    if (n && (!offs || !out)) return fail(MK_EINVAL, "null pointer");
    Locked L;
    TRY(lock_current(L));
    if (n == 0) return MK_OK;
    const size_t inb = offs[n];
    TRY(grow(L.c->in, inb));
    TRY(grow(L.c->aux, 8 * (n + 1)));
    TRY(grow(L.c->out, 32 * n));
    hipStream_t st = L.c->stream;
    if (inb) HIPCHK(hipMemcpyAsync(L.c->in.p, in, inb, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(L.c->aux.p, offs, 8 * (n + 1), hipMemcpyHostToDevice, st));
    TRY(mk_dev_hash_batch_var(L.c->in.p, (const uint64_t*)L.c->aux.p, n, L.c->out.p, st));
    HIPCHK(hipMemcpyAsync(out, L.c->out.p, 32 * n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

// ---- merkleHash ---------------------------------------------------------------
uint64_t mk_ssz_merkle_workspace_bytes(uint64_t n, uint32_t item_len) {
    Plan p;
    if (make_plan(n, item_len, false, 0, false, true, p) != MK_OK) return 0;
    return p.small ? 256 : plan_ws_bytes(p);
}

int mk_dev_ssz_merkle_hash(const void* d_items, uint64_t n, uint32_t item_len, void* d_out32, void* d_ws,
                           uint64_t ws_bytes, void* stream) {
    TRY(bind(-1));
    if (!d_out32 || (n && !d_items)) return fail(MK_EINVAL, "null pointer");
    Plan p;
    TRY(make_plan(n, item_len, false, 0, false, ((uintptr_t)d_items % 16) == 0, p));
    return launch_plan(p, (const uint8_t*)d_items, (uint8_t*)d_out32, (uint8_t*)d_ws, ws_bytes,
                       (hipStream_t)stream);
}

int mk_ssz_merkle_hash(const uint8_t* items, uint64_t n, uint32_t item_len, uint8_t out[32]) {
    if (!out || (n && item_len && !items)) return fail(MK_EINVAL, "null pointer");
    Locked L;
    TRY(lock_current(L));
    Plan p;
    TRY(make_plan(n, item_len, false, 0, false, true, p));
    const size_t inb = n * (size_t)item_len;
    TRY(grow(L.c->in, inb));
    TRY(grow(L.c->out, 32));
    TRY(grow(L.c->ws, p.small ? 256 : plan_ws_bytes(p)));
    hipStream_t st = L.c->stream;
    if (inb) HIPCHK(hipMemcpyAsync(L.c->in.p, items, inb, hipMemcpyHostToDevice, st));
    TRY(launch_plan(p, (const uint8_t*)L.c->in.p, (uint8_t*)L.c->out.p, (uint8_t*)L.c->ws.p, L.c->ws.cap, st));
    HIPCHK(hipMemcpyAsync(out, L.c->out.p, 32, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

// ---- sharding -------------------------------------------------------------------
int mk_ssz_merkle_shard_plan(uint64_t n, uint32_t item_len, uint32_t nshards, uint32_t* height,
                             uint32_t* nonempty, uint64_t* item_begin) {
    if (!height || !nonempty || !item_begin) return fail(MK_EINVAL, "null pointer");
    return shard_plan(n, item_len, nshards, height, nonempty, item_begin);
}

int mk_dev_ssz_merkle_subtree(const void* d_shard_items, uint64_t shard_n, uint32_t item_len, uint32_t height,
                              int pad_at_one, void* d_out32, void* d_ws, uint64_t ws_bytes, void* stream) {
    TRY(bind(-1));
    Plan p;
    TRY(make_plan(shard_n, item_len, true, height, pad_at_one != 0, ((uintptr_t)d_shard_items % 16) == 0, p));
    return launch_plan(p, (const uint8_t*)d_shard_items, (uint8_t*)d_out32, (uint8_t*)d_ws, ws_bytes,
                       (hipStream_t)stream);
}

int mk_dev_ssz_merkle_subtree_frontier(const void* d_shard_items, uint64_t shard_n, uint32_t item_len,
                                       uint32_t height, uint32_t frontier_log2, int pad_at_one, void* d_out,
                                       uint64_t* nodes_out, void* d_ws, uint64_t ws_bytes, void* stream) {
    TRY(bind(-1));
    if (!d_out || (shard_n && !d_shard_items)) return fail(MK_EINVAL, "null pointer");
    Plan p;
    TRY(make_plan(shard_n, item_len, true, height, pad_at_one != 0, ((uintptr_t)d_shard_items % 16) == 0, p, false,
                  frontier_log2));
    if (nodes_out) *nodes_out = p.out_nodes;
    return launch_plan(p, (const uint8_t*)d_shard_items, (uint8_t*)d_out, (uint8_t*)d_ws, ws_bytes,
                       (hipStream_t)stream);
}

uint64_t mk_ssz_merkle_node_frontier_workspace_bytes(uint64_t count, uint32_t height, uint32_t frontier_log2) {
    Plan p;
    if (make_plan(count, 32, true, height, true, true, p, true, frontier_log2) != MK_OK) return 0;
    return std::max<uint64_t>(256, plan_ws_bytes(p));
}

int mk_dev_ssz_merkle_node_frontier(const void* d_nodes, uint64_t count, uint32_t height, uint32_t frontier_log2,
                                    int pad_at_one, void* d_out, uint64_t* nodes_out, void* d_ws, uint64_t ws_bytes,
                                    void* stream) {
    TRY(bind(-1));
    if (!d_out || !d_nodes || count == 0) return fail(MK_EINVAL, "null pointer or empty level");
    Plan p;
    TRY(make_plan(count, 32, true, height, pad_at_one != 0, ((uintptr_t)d_nodes % 16) == 0, p, true,
                  frontier_log2));
    if (nodes_out) *nodes_out = frontier_log2 ? p.out_nodes : 1;
    return launch_plan(p, (const uint8_t*)d_nodes, (uint8_t*)d_out, (uint8_t*)d_ws, ws_bytes, (hipStream_t)stream);
}

uint64_t mk_ssz_merkle_finish_workspace_bytes(uint64_t count) {
    Plan p;
    if (count <= 2 * mk::kWave2Span) return 256;
    if (make_plan(count, 32, false, 0, false, true, p, true, 0, 1) != MK_OK) return 0;
    return plan_ws_bytes(p);
}

int mk_dev_ssz_merkle_finish_nodes(const void* d_nodes, uint64_t count, uint64_t n_total, void* d_out32,
                                   void* d_ws, uint64_t ws_bytes, void* stream) {
    if (count <= 2 * mk::kWave2Span) return mk_dev_ssz_merkle_finish(d_nodes, count, n_total, d_out32, stream);
    TRY(bind(-1));
    if (!d_nodes || !d_out32) return fail(MK_EINVAL, "null pointer");
    Plan p;
    TRY(make_plan(count, 32, false, 0, false, ((uintptr_t)d_nodes % 16) == 0, p, true, 0, n_total));
    return launch_plan(p, (const uint8_t*)d_nodes, (uint8_t*)d_out32, (uint8_t*)d_ws, ws_bytes, (hipStream_t)stream);
}

int mk_dev_ssz_merkle_finish(const void* d_roots, uint64_t nroots, uint64_t n_total, void* d_out32, void* stream) {
    TRY(bind(-1));
    if (nroots == 0 || nroots > 2 * mk::kWave2Span)
        return fail(MK_EINVAL, "nroots %llu out of range (1..%u)", (unsigned long long)nroots, 2 * mk::kWave2Span);
    // the reference level loop over the shard roots (odd -> 0^128) plus the
    // length mix-in is one finalizing node pass of the two-lane latency kernel
    // (plain 32-B roots in, plain digest out)
    ReduceArgs a{};
    a.items = (const uint8_t*)d_roots;
    a.cin = nroots;
    a.c1 = nroots > 1 ? (nroots + 1) / 2 : 1;
    a.c1_full = nroots / 2;
    a.out = (uint8_t*)d_out32;
    a.n_items = n_total;
    a.levels = 64;
    a.finalize = 1;
    launch_wave3<false>(mk::kWaveThreads, 1, a, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return MK_OK;
}

int mk_ssz_merkle_hash_multi(const uint8_t* items, uint64_t n, uint32_t item_len, int ndev, uint8_t out[32]) {
    if (ndev <= 1) return mk_ssz_merkle_hash(items, n, item_len, out);
    if (probe_devices() < ndev) return fail(MK_ENODEV, "%d devices requested, %d visible", ndev, g_ndev);
    uint32_t h = 0, ne = 0;
    std::vector<uint64_t> begin(ndev + 1);
    TRY(shard_plan(n, item_len, (uint32_t)ndev, &h, &ne, begin.data()));
    if (ne <= 1) return mk_ssz_merkle_hash(items, n, item_len, out);

    static std::mutex comm_mu;
    static std::vector<ncclComm_t> comms;
    std::lock_guard<std::mutex> clk(comm_mu);
    if ((int)comms.size() != ndev) {
        for (auto c : comms) ncclCommDestroy(c);
        comms.assign(ndev, nullptr);
        std::vector<int> devs(ndev);
        for (int d = 0; d < ndev; ++d) devs[d] = d;
        if (ncclCommInitAll(comms.data(), ndev, devs.data()) != ncclSuccess) {
            comms.clear();
            return fail(MK_ECOMM, "ncclCommInitAll(%d) failed", ndev);
        }
    }
    std::vector<std::unique_lock<std::mutex>> locks;
    std::vector<DevCtx*> ctx(ndev);
    for (int d = 0; d < ndev; ++d) {
        TRY(bind(d));
        ctx[d] = g_ctx[d];
        locks.emplace_back(ctx[d]->mu);
    }
    // per device: shard upload + reduce to the shard's frontier level (2^k
    // nodes, k levels below the shard root) into block `d` of the level buffer
    const uint32_t k = h > 5 ? std::min<uint32_t>(10, h - 5) : 0;
    const size_t block = (size_t)32 << k;
    uint64_t last_nodes = 1;
    for (int d = 0; d < ndev; ++d) {
        TRY(bind(d));
        DevCtx* c = ctx[d];
        const uint64_t sn = begin[d + 1] - begin[d];
        const size_t inb = sn * (size_t)item_len;
        TRY(grow(c->in, inb));
        TRY(grow(c->out, block * ndev + 32));
        uint8_t* lvl = (uint8_t*)c->out.p;
        if (sn) {
            Plan p;
            TRY(make_plan(sn, item_len, true, h, true, true, p, false, k));
            if (d == (int)ne - 1) last_nodes = p.out_nodes;
            TRY(grow(c->ws, plan_ws_bytes(p)));
            HIPCHK(hipMemcpyAsync(c->in.p, items + begin[d] * item_len, inb, hipMemcpyHostToDevice, c->stream));
            TRY(launch_plan(p, (const uint8_t*)c->in.p, lvl + block * d, (uint8_t*)c->ws.p, c->ws.cap, c->stream));
        } else {
            HIPCHK(hipMemsetAsync(lvl + block * d, 0, block, c->stream));
        }
    }
    // gather the frontier blocks over RCCL (in place: block d of every device)
    if (ncclGroupStart() != ncclSuccess) return fail(MK_ECOMM, "ncclGroupStart");
    for (int d = 0; d < ndev; ++d) {
        uint8_t* lvl = (uint8_t*)ctx[d]->out.p;
        if (ncclAllGather(lvl + block * d, lvl, block, ncclUint8, comms[d], ctx[d]->stream) != ncclSuccess) {
            ncclGroupEnd();
            return fail(MK_ECOMM, "ncclAllGather on device %d", d);
        }
    }
    if (ncclGroupEnd() != ncclSuccess) return fail(MK_ECOMM, "ncclGroupEnd");
    TRY(bind(0));
    uint8_t* lvl0 = (uint8_t*)ctx[0]->out.p;
    const uint64_t count = ((uint64_t)(ne - 1) << k) + last_nodes;
    if (k) {
        TRY(grow(ctx[0]->ws, mk_ssz_merkle_finish_workspace_bytes(count)));
        TRY(mk_dev_ssz_merkle_finish_nodes(lvl0, count, n, lvl0 + block * ndev, ctx[0]->ws.p, ctx[0]->ws.cap,
                                           ctx[0]->stream));
    } else {
        TRY(mk_dev_ssz_merkle_finish(lvl0, ne, n, lvl0 + block * ndev, ctx[0]->stream));
    }
    HIPCHK(hipMemcpyAsync(out, lvl0 + block * ndev, 32, hipMemcpyDeviceToHost, ctx[0]->stream));
    for (int d = 0; d < ndev; ++d) {
        TRY(bind(d));
        HIPCHK(hipStreamSynchronize(ctx[d]->stream));
    }
    TRY(bind(0));
    return MK_OK;
}

// ---- struct hashing ---------------------------------------------------------------
static int make_spec(const mk_field* fields, uint32_t nfields, uint32_t record_len, mk::StructSpec& sp) {
    if (!fields || nfields == 0 || nfields > mk::kMaxStructFields)
        return fail(MK_EINVAL, "nfields %u out of range (1..%u)", nfields, mk::kMaxStructFields);
    std::memset(&sp, 0, sizeof sp);
    uint32_t out = 0;
    for (uint32_t f = 0; f < nfields; ++f) {
        const mk_field& fd = fields[f];
        if (fd.kind == MK_FIELD_BYTES) {
            if (fd.offset % 4) return fail(MK_EINVAL, "bytes field %u: offset not 4-byte aligned", f);
        } else if (fd.kind == MK_FIELD_RAW) {
            if (fd.len != 1 && fd.len != 2 && fd.len != 4 && fd.len != 8)
                return fail(MK_EINVAL, "raw field %u: len %u not in {1,2,4,8}", f, fd.len);
        } else {
            return fail(MK_EINVAL, "field %u: unknown kind %u", f, fd.kind);
        }
        if (record_len && (uint64_t)fd.offset + fd.len > record_len)
            return fail(MK_EINVAL, "field %u exceeds the record", f);
        sp.kind[f] = fd.kind;
        sp.off[f] = fd.offset;
        sp.len[f] = fd.len;
        sp.out_off[f] = out;
        out += fd.kind == MK_FIELD_BYTES ? 32 : fd.len;
    }
    if (record_len % 4) return fail(MK_EINVAL, "record_len %u not a multiple of 4", record_len);
    sp.nfields = nfields;
    sp.rec_len = record_len;
    sp.msg_len = out;
    return MK_OK;
}

// roots of n records into d_roots (n x 32); d_msg holds n x msg_len bytes
static int launch_struct_roots(const void* d_rec, uint64_t n, const mk::StructSpec& sp, void* d_msg, void* d_roots,
                               hipStream_t st) {
    if (n == 0) return MK_OK;
    // fused path: dword-granular single-block fields, dword-aligned message
    bool fused = kStructFused && sp.msg_len % 4 == 0 && sp.msg_len <= mk::kStructFusedMaxMsg &&
                 ((uintptr_t)d_rec % 4) == 0;
    bool vec16 = ((uintptr_t)d_rec % 16) == 0 && sp.rec_len % 16 == 0;
    for (uint32_t f = 0; f < sp.nfields; ++f) {
        if (sp.out_off[f] % 4) fused = false;
        if (sp.kind[f] == MK_FIELD_BYTES) {
            if ((sp.len[f] % 4) != 0 || sp.len[f] > mk::kStructFusedMaxField) fused = false;
            if (sp.off[f] % 16 || sp.off[f] + ((sp.len[f] + 15) & ~15u) > sp.rec_len) vec16 = false;
        } else if (sp.len[f] % 4 || sp.off[f] % 4) {
            fused = false;
        }
    }
    if (fused) {
        hipLaunchKernelGGL(mk::k_struct_fused, dim3(ceil_div(n, mk::kStructThreads)), dim3(mk::kStructThreads),
                           mk::kStructThreads * sp.msg_len, st, (const uint8_t*)d_rec, n, sp, vec16 ? 1u : 0u,
                           (uint4*)d_roots);
        HIPCHK(hipGetLastError());
        return MK_OK;
    }
    bool fast = true;  // every bytes field hashes as one dword-granular block
    for (uint32_t f = 0; f < sp.nfields; ++f)
        if (sp.kind[f] == MK_FIELD_BYTES && ((sp.len[f] % 4) != 0 || sp.len[f] + 4 >= 136)) fast = false;
    if (fast)
        hipLaunchKernelGGL((mk::k_struct_fields<true>), dim3(ceil_div(n * sp.nfields, 256)), dim3(256), 0, st,
                           (const uint8_t*)d_rec, n, sp, (uint8_t*)d_msg);
    else
        hipLaunchKernelGGL((mk::k_struct_fields<false>), dim3(ceil_div(n * sp.nfields, 256)), dim3(256), 0, st,
                           (const uint8_t*)d_rec, n, sp, (uint8_t*)d_msg);
    HIPCHK(hipGetLastError());
    if (sp.msg_len % 8 == 0)
        hipLaunchKernelGGL(mk::k_keccak_words, dim3(ceil_div(n, 256)), dim3(256), 0, st, (const uint2*)d_msg, n,
                           sp.msg_len / 8, (uint4*)d_roots);
    else
        hipLaunchKernelGGL(mk::k_keccak_fixed, dim3(ceil_div(n, 256)), dim3(256), 0, st, (const uint8_t*)d_msg, n,
                           sp.msg_len, (uint4*)d_roots);
    HIPCHK(hipGetLastError());
    return MK_OK;
}

extern "C" uint64_t mk_ssz_struct_msg_len(const mk_field* fields, uint32_t nfields) {
    mk::StructSpec sp;
    if (make_spec(fields, nfields, 0, sp) != MK_OK) return 0;
    return sp.msg_len;
}

static uint64_t align256(uint64_t x) { return (x + 255) & ~255ull; }
// host-buffer entries: H2D in up to kH2dChunks pieces of at least kH2dMinChunk records
#ifndef MK_H2D_CHUNKS
#define MK_H2D_CHUNKS 8
#endif
#ifndef MK_H2D_MIN_CHUNK
#define MK_H2D_MIN_CHUNK 65536
#endif
constexpr uint64_t kH2dChunks = MK_H2D_CHUNKS;
constexpr uint64_t kH2dMinChunk = MK_H2D_MIN_CHUNK;

extern "C" uint64_t mk_ssz_struct_list_workspace_bytes(uint64_t n, const mk_field* fields, uint32_t nfields) {
    mk::StructSpec sp;
    if (make_spec(fields, nfields, 0, sp) != MK_OK) return 0;
    return align256(n * sp.msg_len) + align256(32 * n) + mk_ssz_merkle_workspace_bytes(n, 32);
}

extern "C" int mk_dev_ssz_struct_list_root(const void* d_records, uint64_t n, uint32_t record_len,
                                           const mk_field* fields, uint32_t nfields, void* d_out32, void* d_ws,
                                           uint64_t ws_bytes, void* stream) {
    TRY(bind(-1));
    mk::StructSpec sp;
    TRY(make_spec(fields, nfields, record_len, sp));
    if (ws_bytes < mk_ssz_struct_list_workspace_bytes(n, fields, nfields)) return fail(MK_ENOMEM, "workspace too small");
    uint8_t* ws = (uint8_t*)d_ws;
    uint8_t* msg = ws;
    uint8_t* roots = ws + align256(n * sp.msg_len);
    uint8_t* mws = roots + align256(32 * n);
    hipStream_t st = (hipStream_t)stream;
    TRY(launch_struct_roots(d_records, n, sp, msg, roots, st));
    return mk_dev_ssz_merkle_hash(roots, n, 32, d_out32, mws, ws_bytes - (uint64_t)(mws - ws), stream);
}

extern "C" int mk_dev_ssz_struct_roots(const void* d_records, uint64_t n, uint32_t record_len,
                                       const mk_field* fields, uint32_t nfields, void* d_roots, void* d_ws,
                                       uint64_t ws_bytes, void* stream) {
    TRY(bind(-1));
    mk::StructSpec sp;
    TRY(make_spec(fields, nfields, record_len, sp));
    if (n && (!d_records || !d_roots)) return fail(MK_EINVAL, "null pointer");
    if (ws_bytes < n * (uint64_t)sp.msg_len) return fail(MK_ENOMEM, "workspace too small");
    TRY(launch_struct_roots(d_records, n, sp, d_ws, d_roots, (hipStream_t)stream));
    return MK_OK;
}

extern "C" int mk_ssz_struct_roots(const uint8_t* records, uint64_t n, uint32_t record_len, const mk_field* fields,
                                   uint32_t nfields, uint8_t* roots) {
    mk::StructSpec sp;
    TRY(make_spec(fields, nfields, record_len, sp));
    if (n && (!records || !roots)) return fail(MK_EINVAL, "null pointer");
    Locked L;
    TRY(lock_current(L));
    if (n == 0) return MK_OK;
    hipStream_t st = L.c->stream;
    TRY(grow(L.c->in, n * (size_t)record_len));
    TRY(grow(L.c->ws, align256(n * sp.msg_len)));
    TRY(grow(L.c->out, 32 * n));
    HIPCHK(hipMemcpyAsync(L.c->in.p, records, n * (size_t)record_len, hipMemcpyHostToDevice, st));
    TRY(launch_struct_roots(L.c->in.p, n, sp, L.c->ws.p, L.c->out.p, st));
    HIPCHK(hipMemcpyAsync(roots, L.c->out.p, 32 * n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

extern "C" int mk_ssz_struct_list_root(const uint8_t* records, uint64_t n, uint32_t record_len,
                                       const mk_field* fields, uint32_t nfields, uint8_t out[32]) {
    mk::StructSpec sp;
    TRY(make_spec(fields, nfields, record_len, sp));
    if (!out || (n && !records)) return fail(MK_EINVAL, "null pointer");
    Locked L;
    TRY(lock_current(L));
    hipStream_t st = L.c->stream;
    const uint64_t wsb = mk_ssz_struct_list_workspace_bytes(n, fields, nfields);
    TRY(grow(L.c->in, n * (size_t)record_len));
    TRY(grow(L.c->ws, wsb));
    TRY(grow(L.c->out, 32));
    // Same layout as mk_dev_ssz_struct_list_root.  The records cross PCIe in
    // chunks on the copy stream; the struct-roots kernel of chunk i runs on
    // the compute stream while chunk i+1 is in flight, so only the last
    // chunk's roots and the list merkleHash follow the copy.
    uint8_t* ws = (uint8_t*)L.c->ws.p;
    uint8_t* msg = ws;
    uint8_t* roots = ws + align256(n * sp.msg_len);
    uint8_t* mws = roots + align256(32 * n);
    const uint8_t* din = (const uint8_t*)L.c->in.p;
    uint64_t chunk = std::max<uint64_t>(kH2dMinChunk, ceil_div(n, kH2dChunks));
    chunk = (chunk + 15) & ~15ull;  // chunk starts keep the records' 16-B alignment
    for (uint64_t off = 0; off < n; off += chunk) {
        const uint64_t cnt = std::min(chunk, n - off);
        HIPCHK(hipMemcpyAsync((uint8_t*)L.c->in.p + off * record_len, records + off * record_len,
                              cnt * (size_t)record_len, hipMemcpyHostToDevice, L.c->copy));
        HIPCHK(hipEventRecord(L.c->h2d, L.c->copy));
        HIPCHK(hipStreamWaitEvent(st, L.c->h2d, 0));
        TRY(launch_struct_roots(din + off * record_len, cnt, sp, msg + off * sp.msg_len, roots + 32 * off, st));
    }
    TRY(mk_dev_ssz_merkle_hash(roots, n, 32, L.c->out.p, mws, wsb - (uint64_t)(mws - ws), st));
    HIPCHK(hipMemcpyAsync(out, L.c->out.p, 32, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

// ---- hashutil.MerkleRoot (merkleRoot.go:12-30) ------------------------------------
// Heap o[1..2n): leaves o[n+i] = Hash(values[i]); o[i] = Hash(o[2i] || o[2i+1])
// for i = n-1 .. 1; the result is o[1].  The children of a heap band
// [2^k, 2^(k+1)) are the contiguous range [2^(k+1), 2^(k+2)), so with
// P = 2^floor(log2 n): when n > P the partial band [P, n) is one pairwise
// level over o[2P, 2n), and everything above is a power-of-two binary tree
// over o[P, 2P) -- a node-input merkle plan.  (The reference's spurious
// newSet[0] = Hash(nil || o[1]) is computed and discarded; it is skipped.)
static uint64_t pow2_floor(uint64_t n) {
    uint64_t p = 1;
    while (p * 2 <= n) p *= 2;
    return p;
}

extern "C" uint64_t mk_merkle_root_workspace_bytes(uint64_t n) {
    if (n == 0) return 0;
    const uint64_t P = pow2_floor(n);
    Plan p;
    uint64_t ws = 0;
    if (P > 1 && make_plan(P, 32, true, ilog2(P), false, true, p, true) == MK_OK) ws = plan_ws_bytes(p);
    return 64 * n + align256(ws) + 256;
}

extern "C" int mk_dev_merkle_root(const void* d_data, const uint64_t* d_offs, uint64_t n, uint32_t fixed_len,
                                  void* d_heap, uint64_t heap_bytes, void* d_leaves32, void* d_out32, void* stream) {
    TRY(bind(-1));
    if (n == 0) return fail(MK_EINVAL, "MerkleRoot of an empty list (reference: index out of range)");
    if (!d_heap || !d_out32 || (!d_offs && !d_data && fixed_len)) return fail(MK_EINVAL, "null pointer");
    if (heap_bytes < mk_merkle_root_workspace_bytes(n)) return fail(MK_ENOMEM, "heap workspace too small");
    hipStream_t st = (hipStream_t)stream;
    uint8_t* heap = (uint8_t*)d_heap;  // node i at heap + 32 i (node 0 unused)
    uint4* leaves = (uint4*)(heap + 32 * n);
    if (d_offs) {
        hipLaunchKernelGGL(mk::k_keccak_var, dim3(ceil_div(n, 256)), dim3(256), 0, st, (const uint8_t*)d_data, d_offs,
                           n, leaves);
    } else if (fixed_len == 64 && ((uintptr_t)d_data % 16) == 0) {
        hipLaunchKernelGGL(mk::k_keccak64, dim3(ceil_div(n, 256)), dim3(256), 0, st, (const uint4*)d_data, n, leaves);
    } else if (fixed_len % 8 == 0 && ((uintptr_t)d_data % 8) == 0) {
        hipLaunchKernelGGL(mk::k_keccak_words, dim3(ceil_div(n, 256)), dim3(256), 0, st, (const uint2*)d_data, n,
                           fixed_len / 8, leaves);
    } else {
        hipLaunchKernelGGL(mk::k_keccak_fixed, dim3(ceil_div(n, 256)), dim3(256), 0, st, (const uint8_t*)d_data, n,
                           fixed_len, leaves);
    }
    HIPCHK(hipGetLastError());
    if (d_leaves32 && d_leaves32 != (void*)leaves)
        HIPCHK(hipMemcpyAsync(d_leaves32, leaves, 32 * n, hipMemcpyDeviceToDevice, st));
    if (n == 1) {  // the loop body never runs: o[1] is the hashed value
        HIPCHK(hipMemcpyAsync(d_out32, leaves, 32, hipMemcpyDeviceToDevice, st));
        return MK_OK;
    }
    const uint64_t P = pow2_floor(n);
    if (P < n)  // partial band [P, n): o[i] = Hash(o[2i] || o[2i+1]) over o[2P, 2n)
        hipLaunchKernelGGL(mk::k_trie_level, dim3(ceil_div(n - P, 256)), dim3(256), 0, st,
                           (const uint4*)(heap + 64 * P), 2 * (n - P), (uint4*)(heap + 32 * P));
    HIPCHK(hipGetLastError());
    Plan p;
    TRY(make_plan(P, 32, true, ilog2(P), false, true, p, true));
    uint8_t* ws = heap + 64 * n;
    return launch_plan(p, heap + 32 * P, (uint8_t*)d_out32, ws, heap_bytes - 64 * n, st);
}

extern "C" int mk_merkle_root(const uint8_t* data, const uint64_t* offs, uint64_t n, uint8_t* leaves_out,
                              uint8_t out[32]) {
    if (!out || (n && !offs)) return fail(MK_EINVAL, "null pointer");
    if (n == 0) return fail(MK_EINVAL, "MerkleRoot of an empty list (reference: index out of range)");
    Locked L;
    TRY(lock_current(L));
    hipStream_t st = L.c->stream;
    const size_t inb = offs[n] - offs[0];
    bool uniform = true;
    const uint64_t len0 = offs[1] - offs[0];
    for (uint64_t i = 1; uniform && i < n; ++i) uniform = (offs[i + 1] - offs[i]) == len0;
    uniform = uniform && len0 <= UINT32_MAX;
    const uint64_t wsb = mk_merkle_root_workspace_bytes(n);
    TRY(grow(L.c->in, inb + 16));
    TRY(grow(L.c->aux, 8 * (n + 1)));
    TRY(grow(L.c->ws, wsb));
    TRY(grow(L.c->out, 32));
    if (inb) HIPCHK(hipMemcpyAsync(L.c->in.p, data + offs[0], inb, hipMemcpyHostToDevice, st));
    if (!uniform) {
        std::vector<uint64_t> rel(offs, offs + n + 1);
        for (auto& o : rel) o -= offs[0];
        HIPCHK(hipMemcpyAsync(L.c->aux.p, rel.data(), 8 * (n + 1), hipMemcpyHostToDevice, st));
        TRY(mk_dev_merkle_root(L.c->in.p, (const uint64_t*)L.c->aux.p, n, 0, L.c->ws.p, wsb, nullptr, L.c->out.p,
                               st));
        HIPCHK(hipStreamSynchronize(st));  // rel is a stack vector
    } else {
        TRY(mk_dev_merkle_root(L.c->in.p, nullptr, n, (uint32_t)len0, L.c->ws.p, wsb, nullptr, L.c->out.p, st));
    }
    HIPCHK(hipMemcpyAsync(out, L.c->out.p, 32, hipMemcpyDeviceToHost, st));
    if (leaves_out) HIPCHK(hipMemcpyAsync(leaves_out, (uint8_t*)L.c->ws.p + 32 * n, 32 * n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

// ---- deposit trie -------------------------------------------------------------------
uint64_t mk_deposit_trie_levels_bytes(uint64_t n, uint32_t depth) {
    if (n == 0) return 0;
    uint64_t nodes = 0, c = n;
    for (uint32_t d = 0; d <= depth; ++d) {
        nodes += c;
        c = (c + 1) / 2;
    }
    return 32 * nodes;
}

int mk_dev_deposit_trie_build(const void* d_data, const uint64_t* d_offs, uint64_t n, uint32_t fixed_len,
                              uint32_t depth, void* d_levels, void* d_root32, void* stream) {
    TRY(bind(-1));
    if (!d_root32 || (n && !d_levels) || (n && !d_offs && !d_data && fixed_len)) return fail(MK_EINVAL, "null pointer");
    if (depth > 63) return fail(MK_EINVAL, "depth %u > 63", depth);
    hipStream_t st = (hipStream_t)stream;
    if (n == 0) {
        HIPCHK(hipMemsetAsync(d_root32, 0, 32, st));
        return MK_OK;
    }
    uint4* lv = (uint4*)d_levels;
    if (d_offs) {
        hipLaunchKernelGGL(mk::k_keccak_var, dim3(ceil_div(n, 256)), dim3(256), 0, st, (const uint8_t*)d_data, d_offs,
                           n, lv);
    } else if (kRecKernel && fixed_len == 280 && ((uintptr_t)d_data % 8) == 0) {  // deposit leaves
        hipLaunchKernelGGL((mk::k_keccak_rec<35>),
                           dim3(std::min<uint64_t>(ceil_div(n, mk::kRecThreads), mk::kRecGridMax)),
                           dim3(mk::kRecThreads), 0, st, (const uint2*)d_data, n, lv);
    } else if (fixed_len % 8 == 0 && ((uintptr_t)d_data % 8) == 0) {
        hipLaunchKernelGGL(mk::k_keccak_words, dim3(ceil_div(n, 256)), dim3(256), 0, st, (const uint2*)d_data, n,
                           fixed_len / 8, lv);
    } else {
        hipLaunchKernelGGL(mk::k_keccak_fixed, dim3(ceil_div(n, 256)), dim3(256), 0, st, (const uint8_t*)d_data, n,
                           fixed_len, lv);
    }
    HIPCHK(hipGetLastError());
    // level d lives at lv + 2 * sum_{i<d} count_i (uint4 units).  Wide levels:
    // one launch per level (every lane busy); the narrow top (<= 2^17 nodes)
    // plus the zero-sibling tail: k_trie_top3 (bit-interleaved lane pairs),
    // log2(NT) levels per workgroup of NT inputs, the last launch to the top.
    uint64_t c = n;
    uint4* cur = lv;
    uint32_t d = 0;
    const uint64_t top_max = kWave3 ? kNodeWaveMaxC1 : (1ull << 15);
    while (d < depth && c > top_max) {
        uint4* nxt = cur + 2 * c;
        const uint64_t cn = (c + 1) / 2;
        hipLaunchKernelGGL(mk::k_trie_level, dim3(ceil_div(cn, 256)), dim3(256), 0, st, cur, c, nxt);
        HIPCHK(hipGetLastError());
        cur = nxt;
        c = cn;
        ++d;
    }
    while (d < depth) {
        uint32_t k = 0, nt = 0;
        uint64_t nwg = 0;
        if (kWave3) {
            nt = mk::kWaveThreads;
            while (nt < mk::kMidThreads && ceil_div(c, nt) > kNodeWaveWgs) nt *= 2;
            if (kTopOneWg)  // the last <= 1024 nodes in one workgroup
                while (nt < mk::kMidThreads && c <= mk::kMidThreads && c > nt) nt *= 2;
            nwg = ceil_div(c, nt);
            k = nwg == 1 ? depth - d : std::min<uint32_t>(ilog2(nt), depth - d);
        } else {
            nwg = ceil_div(c, 2 * mk::kWave2Span);
            uint64_t cc = c;
            if (nwg == 1) {
                k = depth - d;
            } else {
                while (k < mk::kWave2Levels && cc > 1) {
                    cc = (cc + 1) / 2;
                    ++k;
                }
            }
        }
        const uint32_t* src = (const uint32_t*)cur;
        uint32_t* dst = (uint32_t*)(cur + 2 * c);
        switch (nt) {
            case 0: hipLaunchKernelGGL(mk::k_trie_top2, dim3(nwg), dim3(mk::kWaveThreads), 0, st, src, c, dst, k); break;
            case 64: hipLaunchKernelGGL(mk::k_trie_top3<64>, dim3(nwg), dim3(64), 0, st, src, c, dst, k); break;
            case 128: hipLaunchKernelGGL(mk::k_trie_top3<128>, dim3(nwg), dim3(128), 0, st, src, c, dst, k); break;
            case 256: hipLaunchKernelGGL(mk::k_trie_top3<256>, dim3(nwg), dim3(256), 0, st, src, c, dst, k); break;
            case 512: hipLaunchKernelGGL(mk::k_trie_top3<512>, dim3(nwg), dim3(512), 0, st, src, c, dst, k); break;
            default: hipLaunchKernelGGL(mk::k_trie_top3<1024>, dim3(nwg), dim3(1024), 0, st, src, c, dst, k); break;
        }
        HIPCHK(hipGetLastError());
        for (uint32_t i = 0; i < k; ++i) {
            cur += 2 * c;
            c = (c + 1) / 2;
        }
        d += k;
    }
    uint4* root_node = cur;
    HIPCHK(hipMemcpyAsync(d_root32, root_node, 32, hipMemcpyDeviceToDevice, st));
    return MK_OK;
}

int mk_deposit_trie_build(const uint8_t* data, const uint64_t* offs, uint64_t n, uint32_t depth,
                          uint8_t* levels_out, uint8_t root[32]) {
    if (!root || (n && !offs)) return fail(MK_EINVAL, "null pointer");
    if (depth > 63) return fail(MK_EINVAL, "depth %u > 63", depth);
    Locked L;
    TRY(lock_current(L));
    if (n == 0) {
        std::memset(root, 0, 32);
        return MK_OK;
    }
    hipStream_t st = L.c->stream;
    const size_t inb = offs[n];
    const uint64_t lv_bytes = mk_deposit_trie_levels_bytes(n, depth);
    TRY(grow(L.c->in, inb));
    TRY(grow(L.c->aux, 8 * (n + 1)));
    TRY(grow(L.c->ws, lv_bytes));
    TRY(grow(L.c->out, 32));
    bool uniform = offs[0] == 0;
    const uint64_t len0 = offs[1] - offs[0];
    for (uint64_t i = 1; uniform && i < n; ++i) uniform = (offs[i + 1] - offs[i]) == len0;
    uniform = uniform && len0 <= UINT32_MAX;
    if (inb) HIPCHK(hipMemcpyAsync(L.c->in.p, data, inb, hipMemcpyHostToDevice, st));
    if (!uniform) HIPCHK(hipMemcpyAsync(L.c->aux.p, offs, 8 * (n + 1), hipMemcpyHostToDevice, st));
    TRY(mk_dev_deposit_trie_build(L.c->in.p, uniform ? nullptr : (const uint64_t*)L.c->aux.p, n,
                                  uniform ? (uint32_t)len0 : 0, depth, L.c->ws.p, L.c->out.p, st));
    HIPCHK(hipMemcpyAsync(root, L.c->out.p, 32, hipMemcpyDeviceToHost, st));
    if (levels_out) HIPCHK(hipMemcpyAsync(levels_out, L.c->ws.p, lv_bytes, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

int mk_verify_merkle_branches(const uint8_t* leaves, const uint8_t* branches, const uint64_t* indices, uint64_t n,
                              uint32_t depth, uint32_t tree_depth, const uint8_t* roots, uint8_t* ok) {
    if (n && (!leaves || !indices || !roots || !ok || (depth && !branches))) return fail(MK_EINVAL, "null pointer");
    Locked L;
    TRY(lock_current(L));
    if (n == 0) return MK_OK;
    hipStream_t st = L.c->stream;
    const size_t bb = 32 * (size_t)depth * n;
    TRY(grow(L.c->in, bb + 64 * n + 16));
    TRY(grow(L.c->aux, 8 * n));
    TRY(grow(L.c->out, n));
    uint8_t* base = (uint8_t*)L.c->in.p;
    uint8_t* d_leaves = base;
    uint8_t* d_roots = base + 32 * n;
    uint8_t* d_br = base + 64 * n;
    HIPCHK(hipMemcpyAsync(d_leaves, leaves, 32 * n, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_roots, roots, 32 * n, hipMemcpyHostToDevice, st));
    if (bb) HIPCHK(hipMemcpyAsync(d_br, branches, bb, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(L.c->aux.p, indices, 8 * n, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(mk::k_verify_branches, dim3(ceil_div(n, 256)), dim3(256), 0, st, (const uint4*)d_leaves,
                       (const uint4*)d_br, (const uint64_t*)L.c->aux.p, depth, tree_depth, (const uint4*)d_roots, n,
                       (uint8_t*)L.c->out.p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(ok, L.c->out.p, n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

// ---- synthetic inputs -------------------------------------------------------------
int mk_dev_synth_fill(void* d_dst, uint64_t nbytes, uint64_t seed, uint64_t word0, void* stream) {
    TRY(bind(-1));
    if (nbytes % 8) return fail(MK_EINVAL, "nbytes %% 8 != 0");
    if ((uintptr_t)d_dst % 8) return fail(MK_EINVAL, "destination not 8-byte aligned");
    const uint64_t nwords = nbytes / 8;
    if (!nwords) return MK_OK;
    const uint64_t grid = std::min<uint64_t>(ceil_div(nwords, 256), 256 * 64);
    hipLaunchKernelGGL(mk::k_synth, dim3(grid), dim3(256), 0, (hipStream_t)stream, (uint64_t*)d_dst, nwords, seed,
                       word0);
    HIPCHK(hipGetLastError());
    return MK_OK;
}

// ---- measurement ----------------------------------------------------------------------
int mk_prof_enable(int on) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_on = on != 0;
    return MK_OK;
}

int mk_prof_read(double* leaf_ms, uint64_t* leaf_launches, double* leaf_perms, double* leaf_hashes) {
    std::vector<ProfRec> recs;
    {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        recs.swap(g_prof);
    }
    double ms = 0, perms = 0, hashes = 0;
    for (auto& r : recs) {
        HIPCHK(hipEventSynchronize(r.b));
        float t = 0;
        HIPCHK(hipEventElapsedTime(&t, r.a, r.b));
        ms += t;
        perms += r.perms;
        hashes += r.hashes;
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
    }
    if (leaf_ms) *leaf_ms = ms;
    if (leaf_launches) *leaf_launches = recs.size();
    if (leaf_perms) *leaf_perms = perms;
    if (leaf_hashes) *leaf_hashes = hashes;
    return MK_OK;
}

}  // extern "C"
