// C-ABI of the MI355X Merkleization engine: devices, streams and buffers,
// the launch side of the pass planner (planner.cpp), and the host/device
// entry points declared in include/prysm_merkle.h.  Built with hipcc into
// libprysm_merkle.so.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

#include "merkle_kernels.hpp"
#include "planner.hpp"
#include "prysm_merkle.h"

using mk::ceil_div;
using mk::fail;
using mk::ilog2;
using mk::Plan;
using mk::Pass;
using mk::ReduceArgs;
using mk::kReduceThreads;

namespace {

#define MK_SIDE_PRIO 1
constexpr bool kSidePrio = MK_SIDE_PRIO != 0;  // library side/copy streams at high priority
// a whole trie's top (every level from the first of <= 2^20 nodes) in one
// launch, k_trie_top_fused (0: the k_trie_level / k_trie_top3 / k_trie_spread chain)
#define MK_TRIE_TOP_FUSED 1
#define MK_TRIE_TOP_MAX_LOG2 17
constexpr uint64_t kTrieTopMax = 1ull << MK_TRIE_TOP_MAX_LOG2;  // trie levels at or below: k_trie_top3
constexpr uint64_t kTrieTopWgs = 256;
constexpr uint64_t kAppendMaxRange = 1020;  // k_trie_append<1024>: one parent per lane pair
#define MK_STAGE_BYTES (32ull << 20)
constexpr size_t kStageBytes = MK_STAGE_BYTES;  // H2D chunk of the multi-device upload

#define HIPCHK(x)                                                                            \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) return fail(MK_EHIP, "%s: %s", #x, hipGetErrorString(e_));     \
    } while (0)

#define TRY(x)                        \
    do {                              \
        int rc_ = (x);                \
        if (rc_ != MK_OK) return rc_; \
    } while (0)

// ---- devices ---------------------------------------------------------------
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

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

// small pinned upload ring: descriptor tables for dev entry points (the
// source must outlive the async copy; a slot is reused after its event)
struct SmallStage {
    std::mutex mu;
    static constexpr int kSlots = 4;
    void* host[kSlots] = {};
    size_t cap[kSlots] = {};
    hipEvent_t ev[kSlots] = {};
    bool used[kSlots] = {};
    int next = 0;
};

struct DevCtx {
    std::mutex mu;  // host-buffer entry points: in/out/ws/aux and the big staging
    hipStream_t stream = nullptr;
    DevBuf in, out, ws, aux, dig;  // dig: element digests of the multi-shard TreeHash path
    // side stream + events: the ragged last workgroup of a pass runs
    // concurrently with the pass's full workgroups (fork/join on events)
    std::mutex side_mu;
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;

    // host-buffer uploads on `copy` overlapping compute on `stream`
    hipStream_t copy = nullptr;
    hipEvent_t h2d = nullptr;
    hipEvent_t region_ev[2] = {nullptr, nullptr};  // multi: compute of a shard region done
    bool region_used[2] = {false, false};
    SmallStage small;
    // mk_dev_ssz_merkle_hash_multi's own frontier blocks / workspaces: that
    // path enqueues on the caller's streams without this device's `mu`, so it
    // must never share in/out/ws/aux with the host-buffer entry points
    DevBuf mout, mws, maux;
};

std::mutex g_mu;
int g_ndev = -1;
std::vector<DevCtx*> g_ctx;
thread_local int t_bound = -1;  // device bound by the current call

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

// Makes `dev` the thread's current device and creates its context once.
int bind_dev(int dev) {
    if (probe_devices() <= 0) return fail(MK_ENODEV, "no gfx950 device visible");
    if (dev < 0 || dev >= g_ndev) return fail(MK_ENODEV, "device %d out of range (%d visible)", dev, g_ndev);
    HIPCHK(hipSetDevice(dev));
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_ctx[dev]) {
        auto* c = new DevCtx();
        // side/copy streams at the highest priority: a default-priority
        // stream can share the caller's hardware queue (GPU_MAX_HW_QUEUES=4)
        // and then runs after, not beside, the work it should overlap
        int lo = 0, hi = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess || !kSidePrio) hi = lo = 0;
        bool ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
                  hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, hi) == hipSuccess &&
                  hipEventCreateWithFlags(&c->fork, hipEventDisableTiming) == hipSuccess &&
                  hipEventCreateWithFlags(&c->join, hipEventDisableTiming) == hipSuccess &&
                  hipStreamCreateWithPriority(&c->copy, hipStreamNonBlocking, hi) == hipSuccess &&
                  hipEventCreateWithFlags(&c->h2d, hipEventDisableTiming) == hipSuccess;
        for (int i = 0; ok && i < 2; ++i)
            ok = hipEventCreateWithFlags(&c->region_ev[i], hipEventDisableTiming) == hipSuccess;
        for (int i = 0; ok && i < SmallStage::kSlots; ++i)
            ok = hipEventCreateWithFlags(&c->small.ev[i], hipEventDisableTiming) == hipSuccess;
        if (!ok) {
            delete c;
            return fail(MK_EHIP, "stream/event creation failed on device %d", dev);
        }
        g_ctx[dev] = c;
    }
    t_bound = dev;
    return MK_OK;
}

DevCtx* ctx() { return g_ctx[t_bound]; }

// The device a call runs on: call->device, else the thread's current device.
int bind_call() {
    const mk_call* c = mk::current_call();
    int dev = c ? c->device : -1;
    if (dev < 0) {
        if (probe_devices() <= 0) return fail(MK_ENODEV, "no gfx950 device visible");
        if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    }
    return bind_dev(dev);
}

// dev entry points: the device of `stream` (call->device must agree), else as bind_call
int bind_stream(hipStream_t st) {
    if (!st) return bind_call();
    if (probe_devices() <= 0) return fail(MK_ENODEV, "no gfx950 device visible");
    hipDevice_t d = -1;
    HIPCHK(hipStreamGetDevice(st, &d));
    const mk_call* c = mk::current_call();
    if (c && c->device >= 0 && c->device != (int)d)
        return fail(MK_EINVAL, "stream belongs to device %d, call->device is %d", (int)d, c->device);
    return bind_dev((int)d);
}

// Per-call scope of an extern "C" entry point: installs the call context,
// restores the thread's current device on exit.
struct Scope {
    mk_call* prev;
    int saved = -1;
    bool restore = false;
    explicit Scope(mk_call* c, bool gpu = true) {
        prev = mk::swap_call(c);
        if (c) {
            c->code = MK_OK;
            c->err[0] = 0;
        }
        if (gpu && probe_devices() > 0) restore = hipGetDevice(&saved) == hipSuccess;
    }
    int done(int rc) {
        if (mk::current_call()) mk::current_call()->code = rc;
        return rc;
    }
    ~Scope() {
        int cur = -1;
        if (restore && hipGetDevice(&cur) == hipSuccess && cur != saved) (void)hipSetDevice(saved);
        t_bound = -1;
        mk::swap_call(prev);
    }
};

// Uploads `bytes` of host data to device memory on `st` through the
// context's small pinned ring (the caller's buffer may die on return).
int upload_small(DevCtx* c, void* d_dst, const void* src, size_t bytes, hipStream_t st) {
    if (!bytes) return MK_OK;
    SmallStage& S = c->small;
    std::lock_guard<std::mutex> lk(S.mu);
    const int i = S.next;
    S.next = (S.next + 1) % SmallStage::kSlots;
    if (S.used[i]) HIPCHK(hipEventSynchronize(S.ev[i]));
    if (S.cap[i] < bytes) {
        if (S.host[i]) (void)hipHostFree(S.host[i]);
        S.host[i] = nullptr;
        S.cap[i] = 0;
        const size_t cap = std::max<size_t>(bytes, 64 << 10);
        if (hipHostMalloc(&S.host[i], cap, hipHostMallocDefault) != hipSuccess)
            return fail(MK_ENOMEM, "hipHostMalloc(%zu) failed", cap);
        S.cap[i] = cap;
    }
    std::memcpy(S.host[i], src, bytes);
    HIPCHK(hipMemcpyAsync(d_dst, S.host[i], bytes, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(S.ev[i], st));
    S.used[i] = true;
    return MK_OK;
}

// ---- measurement -------------------------------------------------------------
struct ProfRec {
    hipEvent_t a, b;
    double perms, hashes;
};
std::mutex g_prof_mu;
bool g_prof_on = false;
std::vector<ProfRec> g_prof;

bool prof_on() {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    return g_prof_on;
}

// ---- merkleHash plan launch --------------------------------------------------------
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

// Test hook (MK_INJECT_EHIP=1 in the environment when the library is
// loaded): every merkle plan launch and Hash batch fails the way a failed HIP
// launch does (MK_EHIP with its detail in the call's context), so a binding
// can prove a GPU failure reaches its caller as an error and is never
// answered by a CPU fallback (tests/c_abi/harness.c `inject`).
bool inject_ehip() {
    static const bool on = [] {
        const char* e = std::getenv("MK_INJECT_EHIP");
        return e && e[0] == '1';
    }();
    return on;
}

// Workgroups of a persistent phase-locked launch on `st`: one per CU the
// stream may use (its CU mask, hipExtStreamCreateWithCUMask), at most
// MK_LOCK_GRID.  A persistent 1024-thread workgroup needs a whole CU, so a
// grid larger than the stream's CUs would run a second, straggling round.
uint64_t lock_grid_cap(hipStream_t st) {
    // no stream query inside a graph capture (the default grid is recorded)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) {
        (void)hipGetLastError();
        return MK_LOCK_GRID;
    }
    uint32_t m[16] = {0};  // up to 512 CUs
    if (hipExtStreamGetCUMask(st, 16, m) != hipSuccess) {
        (void)hipGetLastError();
        return MK_LOCK_GRID;
    }
    uint64_t c = 0;
    for (uint32_t w : m) c += (uint64_t)__builtin_popcount(w);
    return c ? std::min<uint64_t>(c, MK_LOCK_GRID) : MK_LOCK_GRID;
}

int launch_plan(const Plan& p, const uint8_t* d_items, uint8_t* d_out32, uint8_t* d_ws, uint64_t ws_bytes,
                hipStream_t st, uint8_t* pair_block = nullptr, uint32_t pair_slot = 0, uint32_t pair_epoch = 0) {
    if (inject_ehip()) return fail(MK_EHIP, "hipLaunchKernelGGL: injected failure (MK_INJECT_EHIP)");
    if (p.small && pair_block) return fail(MK_EINVAL, "internal: pair finalize needs a k_wave3 plan");
    if (p.small) {
        hipLaunchKernelGGL(mk::k_final_small, dim3(1), dim3(64), 0, st, d_items, p.total, p.n, d_out32);
        HIPCHK(hipGetLastError());
        return MK_OK;
    }
    if (ws_bytes < mk::plan_ws_bytes(p))
        return fail(MK_ENOMEM, "workspace too small: %llu < %llu", (unsigned long long)ws_bytes,
                    (unsigned long long)mk::plan_ws_bytes(p));
    if (pair_block)  // checked before any pass is launched
        for (const Pass& ps : p.passes)
            if (ps.a.finalize && (!MK_WAVE3_SPREAD || !ps.wave || !ps.w3))
                return fail(MK_EINVAL, "internal: pair finalize needs the spread-form k_wave3 final pass");
    uint8_t* slots[2] = {d_ws, d_ws + 32 * p.slot_nodes[0]};
    const bool prof = prof_on();
    for (const Pass& ps : p.passes) {
        ReduceArgs a = ps.a;
        a.items = ps.in_ws < 0 ? d_items : slots[ps.in_ws];
        a.out = ps.out_ws < 0 ? d_out32 : slots[ps.out_ws];
        if (a.finalize && pair_block) {  // a two-field struct root (wave3_spread_final)
            a.pair_block = pair_block;
            a.pair_slot = pair_slot;
            a.pair_epoch = pair_epoch;
            a.out = pair_block + 32 * pair_slot;
        }
        ProfRec rec{};
        const bool rec_this = prof && ps.leaf;
        if (rec_this) {
            HIPCHK(hipEventCreate(&rec.a));
            HIPCHK(hipEventCreate(&rec.b));
            HIPCHK(hipEventRecord(rec.a, st));
        }
        if (ps.sp) {
            a.wg_base = 0;
            const uint32_t w8 = (((uintptr_t)a.items % 8) == 0 && a.cb % 8 == 0) ? 1u : 0u;
            hipLaunchKernelGGL(mk::k_spread_leaf<16>, dim3(ps.nwg), dim3(1024), 0, st, a, w8);
            HIPCHK(hipGetLastError());
        } else if (ps.wave) {
            a.wg_base = 0;
            if (ps.leaf)
                launch_wave3<true>(ps.nt, ps.nwg, a, st);
            else
                launch_wave3<false>(ps.nt, ps.nwg, a, st);
            HIPCHK(hipGetLastError());
        } else {
            // The ragged workgroup(s) of a pass are latency-bound; when the pass
            // also has full workgroups they go first, on the side stream, so
            // they overlap the full ones (fork/join through events on `st`).
            const bool ragged = ps.nwg > ps.nfast;
            DevCtx* c = (ragged && ps.nfast) ? ctx() : nullptr;
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
                if (ps.leaf && a.elem_len)  // planned with NI = 1
                    hipLaunchKernelGGL((mk::k_reduce_elem<false>), dim3(ps.nwg - ps.nfast), dim3(kReduceThreads), 0,
                                       gs, g);
                else if (ps.leaf && ps.ni == 1)
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
            uint64_t fast_base = 0;
            if (ps.nlock && ps.leaf && !a.elem_len) {  // phase-locked leaf workgroups first: 4 spans each, levels == 3
                a.wg_base = 0;
                // persistent grid (one 1024-thread workgroup per CU), whole trees and subtree shards
                // alike: a shard's pipelined step beside its side-stream passes measured 1.2-3.7 %
                // faster than one group per workgroup (profiles/r05/shard_persist/)
                hipLaunchKernelGGL(mk::k_leaf_lock_sc, dim3(std::min<uint64_t>(ps.nlock, lock_grid_cap(st))),
                                   dim3(mk::kLockThreads), 0, st, a, ps.nlock);
                HIPCHK(hipGetLastError());
                fast_base = ps.nlock * 4;
            } else if (ps.nlock && !ps.leaf) {  // phase-locked node groups first: 16 spans each, levels == 5
                a.wg_base = 0;
                hipLaunchKernelGGL(mk::k_node_lock, dim3(std::min<uint64_t>(ps.nlock, lock_grid_cap(st))),
                                   dim3(mk::kLockThreads), 0, st, a, ps.nlock);
                HIPCHK(hipGetLastError());
                fast_base = ps.nlock * mk::kNodeLockSpans;
            }
            if (ps.nfast > fast_base) {
                a.wg_base = fast_base;
                const uint64_t nfast = ps.nfast - fast_base;
                if (ps.leaf && a.elem_len)
                    hipLaunchKernelGGL((mk::k_reduce_elem<true>), dim3(nfast), dim3(kReduceThreads), 0, st, a);
                else if (ps.leaf && ps.ni == 1)
                    hipLaunchKernelGGL((mk::k_reduce<true, true, 1>), dim3(nfast), dim3(kReduceThreads), 0, st, a);
                else if (ps.leaf)
                    hipLaunchKernelGGL((mk::k_reduce<true, true, 2>), dim3(nfast), dim3(kReduceThreads), 0, st, a);
                else
                    hipLaunchKernelGGL((mk::k_reduce<false, true, 2>), dim3(nfast), dim3(kReduceThreads), 0, st, a);
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

// ---- hashing ----------------------------------------------------------------------
int dev_hash_batch(const void* d_in, uint64_t n, uint32_t msg_len, void* d_out, hipStream_t st) {
    if (n == 0) return MK_OK;
    if (inject_ehip()) return fail(MK_EHIP, "hipLaunchKernelGGL: injected failure (MK_INJECT_EHIP)");
    if (!d_out || (!d_in && msg_len)) return fail(MK_EINVAL, "null pointer");
    const uint64_t grid = ceil_div(n, 256);
    if (msg_len == 64 && ((uintptr_t)d_in % 16) == 0 && ((uintptr_t)d_out % 16) == 0) {
        if (MK_K64_LOCK && n >= (1u << 18))  // phase-locked (a partial last group included)
            hipLaunchKernelGGL(mk::k_keccak64_lock,
                               dim3(std::min<uint64_t>(ceil_div(n, mk::kLockThreads), lock_grid_cap(st))),
                               dim3(mk::kLockThreads), 0, st, (const uint4*)d_in, n, (uint4*)d_out);
        else
            hipLaunchKernelGGL(mk::k_keccak64, dim3(grid), dim3(256), 0, st, (const uint4*)d_in, n, (uint4*)d_out);
    } else if (msg_len == 280 && ((uintptr_t)d_in % 8) == 0 && ((uintptr_t)d_out % 16) == 0) {
        hipLaunchKernelGGL((mk::k_keccak_rec<35>), dim3(std::min<uint64_t>(ceil_div(n, mk::kRecThreads), mk::kRecGridMax)),
                           dim3(mk::kRecThreads), 0, st, (const uint2*)d_in, n, (uint4*)d_out);
    } else if (msg_len % 8 == 0 && msg_len > 0 && ((uintptr_t)d_in % 8) == 0 && ((uintptr_t)d_out % 16) == 0) {
        hipLaunchKernelGGL(mk::k_keccak_words, dim3(grid), dim3(256), 0, st, (const uint2*)d_in, n, msg_len / 8,
                           (uint4*)d_out);
    } else {
        hipLaunchKernelGGL(mk::k_keccak_fixed, dim3(grid), dim3(256), 0, st, (const uint8_t*)d_in, n, msg_len,
                           (uint4*)d_out);
    }
    HIPCHK(hipGetLastError());
    return MK_OK;
}

int dev_hash_var(const void* d_in, const uint64_t* d_offs, uint64_t n, void* d_out, hipStream_t st) {
    if (n == 0) return MK_OK;
    if (!d_offs || !d_out) return fail(MK_EINVAL, "null pointer");
    hipLaunchKernelGGL(mk::k_keccak_var, dim3(ceil_div(n, 256)), dim3(256), 0, st, (const uint8_t*)d_in, d_offs, n,
                       (uint4*)d_out);
    HIPCHK(hipGetLastError());
    return MK_OK;
}

// Leaf hashes of deposits/values: offsets (device) or fixed-length records.
int dev_leaf_hashes(const void* d_data, const uint64_t* d_offs, uint64_t n, uint32_t fixed_len, uint4* out,
                    hipStream_t st) {
    if (n == 0) return MK_OK;
    if (d_offs) return dev_hash_var(d_data, d_offs, n, out, st);
    return dev_hash_batch(d_data, n, fixed_len, out, st);
}

// Uniform message length of offs[0..n] (relative), or -1.
int64_t uniform_len(const uint64_t* offs, uint64_t n) {
    const uint64_t len0 = offs[1] - offs[0];
    for (uint64_t i = 1; i < n; ++i)
        if (offs[i + 1] - offs[i] != len0) return -1;
    return len0 <= UINT32_MAX ? (int64_t)len0 : -1;
}

// ---- merkleHash entry bodies -------------------------------------------------------
// The latency form of a small list's tree (round 6): merkleHash of n items
// whose first level has 16 < windows <= 2^12 (C1's 16,384 ValidatorRecord
// roots: 2,048 windows).  k_spread_leaf<8> hashes the windows one per wave, 8
// per workgroup (two waves per SIMD, where the general plan's 16 put four on
// each: 2 x ~9.8 k cycles against 2 x ~17.8 k -- a lone wave is issue-bound,
// DESIGN §4.5), and folds each workgroup's 8 to one node 3 levels up;
// k_merkle_top_fused takes those nodes 16 per workgroup (4 levels in the
// spread form), groups of 16 workgroups, and the last to the root and the
// length mix-in -- where the general plan ran one 1024-thread k_wave3 over
// the last <= 256 nodes, whose widest levels run as lane pairs at ~14 k
// cycles each.  C1 0.095 -> 0.085 ms (profiles/r06/c1/).
uint64_t align256(uint64_t x) { return (x + 255) & ~255ull; }
static uint64_t list_tree_windows(uint64_t n, uint32_t item_len) {
    if (n == 0 || item_len == 0 || n > (UINT64_MAX / 4) / item_len) return 0;
    return ceil_div(ceil_div(n * (uint64_t)item_len, mk::chunk_bytes(item_len)), 2);
}
static bool list_tree_ok(uint64_t n, uint32_t item_len) {
    const uint64_t c1 = list_tree_windows(n, item_len);
    return c1 > 16 && c1 <= 4096;
}
static uint64_t list_tree_ws(uint64_t n, uint32_t item_len) {
    if (!list_tree_ok(n, item_len)) return 0;
    const uint64_t c4 = ceil_div(list_tree_windows(n, item_len), 8);
    return align256(32 * c4) + align256(32 * ceil_div(c4, 16));
}
static int launch_top_span(const void* d_nodes, uint64_t c, uint64_t n_items, uint32_t span_log2, void* d_out32,
                           uint8_t* d_ws, hipStream_t st);
static int dev_list_tree(const void* d_items, uint64_t n, uint32_t item_len, void* d_out32, uint8_t* ws,
                         hipStream_t st) {
    if (inject_ehip()) return fail(MK_EHIP, "hipLaunchKernelGGL: injected failure (MK_INJECT_EHIP)");
    mk::ReduceArgs a{};
    a.cb = mk::chunk_bytes(item_len);
    a.total = n * (uint64_t)item_len;
    a.nchunks = ceil_div(a.total, a.cb);
    a.c1 = ceil_div(a.nchunks, 2);
    a.items = (const uint8_t*)d_items;
    a.out = ws;
    a.n_items = n;
    a.levels = 4;  // the windows + 3 levels: one node per workgroup
    const uint32_t w8 = (((uintptr_t)d_items % 8) == 0 && a.cb % 8 == 0) ? 1u : 0u;
    hipLaunchKernelGGL(mk::k_spread_leaf<8>, dim3(ceil_div(a.c1, 8)), dim3(1024), 0, st, a, w8);
    HIPCHK(hipGetLastError());
    const uint64_t c4 = ceil_div(a.c1, 8);
    return launch_top_span(ws, c4, n, 4, d_out32, ws + align256(32 * c4), st);
}

int dev_merkle_hash(const void* d_items, uint64_t n, uint32_t item_len, void* d_out32, void* d_ws, uint64_t ws_bytes,
                    hipStream_t st) {
    if (!d_out32 || (n && item_len && !d_items)) return fail(MK_EINVAL, "null pointer");
    if (list_tree_ok(n, item_len) && ws_bytes >= list_tree_ws(n, item_len) && (uintptr_t)d_ws % 16 == 0)
        return dev_list_tree(d_items, n, item_len, d_out32, (uint8_t*)d_ws, st);
    Plan p;
    TRY(mk::make_plan(n, item_len, false, 0, false, ((uintptr_t)d_items % 16) == 0, p));
    return launch_plan(p, (const uint8_t*)d_items, (uint8_t*)d_out32, (uint8_t*)d_ws, ws_bytes, st);
}

int dev_finish(const void* d_roots, uint64_t nroots, uint64_t n_total, void* d_out32, hipStream_t st,
               void* d_pair_block = nullptr, uint32_t pair_slot = 0, uint32_t pair_epoch = 0) {
    if (nroots == 0 || nroots > 2 * mk::kWave2Span)
        return fail(MK_EINVAL, "nroots %llu out of range (1..%u)", (unsigned long long)nroots, 2 * mk::kWave2Span);
    if (!d_roots || (!d_out32 && !d_pair_block)) return fail(MK_EINVAL, "null pointer");
    // the reference level loop over the shard roots (odd -> 0^128) plus the
    // length mix-in is one finalizing node pass of the two-lane latency kernel
    ReduceArgs a{};
    a.items = (const uint8_t*)d_roots;
    a.cin = nroots;
    a.c1 = nroots > 1 ? (nroots + 1) / 2 : 1;
    a.c1_full = nroots / 2;
    a.out = (uint8_t*)d_out32;
    a.n_items = n_total;
    a.levels = 64;
    a.finalize = 1;
    if (d_pair_block) {
        a.pair_block = (uint8_t*)d_pair_block;
        a.pair_slot = pair_slot;
        a.pair_epoch = pair_epoch;
        a.out = (uint8_t*)d_pair_block + 32 * pair_slot;
    }
    launch_wave3<false>(mk::kWaveThreads, 1, a, st);
    HIPCHK(hipGetLastError());
    return MK_OK;
}

uint64_t finish_ws_bytes(uint64_t count) {
    Plan p;
    if (count <= 2 * mk::kWave2Span) return 256;
    if (mk::make_plan(count, 32, false, 0, false, true, p, true, 0, 1) != MK_OK) return 0;
    return mk::plan_ws_bytes(p);
}

int dev_finish_nodes(const void* d_nodes, uint64_t count, uint64_t n_total, void* d_out32, void* d_ws,
                     uint64_t ws_bytes, hipStream_t st, void* d_pair_block = nullptr, uint32_t pair_slot = 0,
                     uint32_t pair_epoch = 0) {
    if (count <= 2 * mk::kWave2Span)
        return dev_finish(d_nodes, count, n_total, d_out32, st, d_pair_block, pair_slot, pair_epoch);
    if (!d_nodes || (!d_out32 && !d_pair_block)) return fail(MK_EINVAL, "null pointer");
    Plan p;
    TRY(mk::make_plan(count, 32, false, 0, false, ((uintptr_t)d_nodes % 16) == 0, p, true, 0, n_total));
    return launch_plan(p, (const uint8_t*)d_nodes, (uint8_t*)d_out32, (uint8_t*)d_ws, ws_bytes, st,
                       (uint8_t*)d_pair_block, pair_slot, pair_epoch);
}

// ---- TreeHash of a list of byte strings (makeSliceHasher + hashedEncoding) ---------------
// The tree's items are the n element digests K(le32(elem_len) || element)
// (hash.go:100-107, 118-139).  Fused (k_reduce_elem, no digest array) when
// the elements are 32 B, 16-B aligned and the leaf pass is a throughput
// pass; otherwise the digests go to the workspace first (k_elem_digests) and
// the ordinary plan runs over them.
struct ElemPlan {
    Plan p;
    bool fused = false;
    uint64_t dig_bytes = 0;  // two-phase: digest array at the start of the workspace
    uint64_t ws_bytes = 0;
    bool locked = false;  // k_elem_lock writes the window digests, `p` reduces them (node input, mix-in n)
    uint64_t nwin = 0;
};

#define MK_ELEM_LOCK 1
#define MK_ELEM_LOCK_MIN_LOG2 23  // elements (2^20 windows: 1024 groups)

int make_elem_plan(uint64_t n, uint32_t elem_len, bool aligned16, ElemPlan& e) {
    e = ElemPlan();
    if (n > (UINT64_MAX / 4) / 32) return fail(MK_EINVAL, "n too large");
    const bool fast32 = elem_len == 32 && aligned16;
    if (MK_ELEM_LOCK && fast32 && n % 8 == 0 && n >= (1ull << MK_ELEM_LOCK_MIN_LOG2)) {
        // phase-locked element windows (every window full: 8 elements = 2
        // chunks), then the tree above them from its level-1 nodes
        e.locked = true;
        e.nwin = n / 8;
        TRY(mk::make_plan(e.nwin, 32, false, 0, false, true, e.p, /*node_input=*/true, 0, /*mixin_n=*/n));
        e.dig_bytes = (32 * e.nwin + 255) & ~255ull;
        e.ws_bytes = e.dig_bytes + mk::plan_ws_bytes(e.p);
        return MK_OK;
    }
    TRY(mk::make_plan(n, 32, false, 0, false, fast32, e.p, false, 0, 0, /*leaf_ni1=*/fast32));
    e.fused = fast32 && !e.p.small && !e.p.passes.empty() && !e.p.passes[0].wave && !e.p.passes[0].sp;
    if (!e.fused && fast32) TRY(mk::make_plan(n, 32, false, 0, false, true, e.p));  // the ordinary plan over digests
    if (e.fused) {
        Pass& ps = e.p.passes[0];
        ps.a.elem_len = 32;
        ps.perms += (double)n;  // one permutation per 36-B element message
        ps.hashes += (double)n;
        e.ws_bytes = mk::plan_ws_bytes(e.p);
    } else {
        e.dig_bytes = (32 * n + 255) & ~255ull;
        e.ws_bytes = e.dig_bytes + (e.p.small ? 256 : mk::plan_ws_bytes(e.p));
    }
    return MK_OK;
}

int launch_elem_digests(const void* d_elems, uint64_t n, uint32_t elem_len, void* d_dig, hipStream_t st) {
    if (n == 0) return MK_OK;
    if (elem_len == 32 && ((uintptr_t)d_elems % 16) == 0)
        hipLaunchKernelGGL(mk::k_elem_digests<true>, dim3(ceil_div(n, 256)), dim3(256), 0, st,
                           (const uint8_t*)d_elems, n, elem_len, (uint4*)d_dig);
    else
        hipLaunchKernelGGL(mk::k_elem_digests<false>, dim3(ceil_div(n, 256)), dim3(256), 0, st,
                           (const uint8_t*)d_elems, n, elem_len, (uint4*)d_dig);
    HIPCHK(hipGetLastError());
    return MK_OK;
}

int dev_tree_hash_elems(const void* d_elems, uint64_t n, uint32_t elem_len, void* d_out32, void* d_ws,
                        uint64_t ws_bytes, hipStream_t st) {
    if (!d_out32 || (n && elem_len && !d_elems)) return fail(MK_EINVAL, "null pointer");
    ElemPlan e;
    TRY(make_elem_plan(n, elem_len, ((uintptr_t)d_elems % 16) == 0, e));
    if (ws_bytes < e.ws_bytes)
        return fail(MK_ENOMEM, "workspace too small: %llu < %llu", (unsigned long long)ws_bytes,
                    (unsigned long long)e.ws_bytes);
    if (n && !d_ws) return fail(MK_EINVAL, "null workspace");
    if (e.fused) return launch_plan(e.p, (const uint8_t*)d_elems, (uint8_t*)d_out32, (uint8_t*)d_ws, ws_bytes, st);
    uint8_t* dig = (uint8_t*)d_ws;
    if (e.locked) {
        ProfRec rec{};
        const bool prof = prof_on();
        if (prof) {
            HIPCHK(hipEventCreate(&rec.a));
            HIPCHK(hipEventCreate(&rec.b));
            HIPCHK(hipEventRecord(rec.a, st));
        }
        hipLaunchKernelGGL(mk::k_elem_lock, dim3(std::min<uint64_t>(ceil_div(e.nwin, mk::kLockThreads), lock_grid_cap(st))),
                           dim3(mk::kLockThreads), 0, st, (const uint4*)d_elems, e.nwin, (uint4*)dig);
        HIPCHK(hipGetLastError());
        if (prof) {
            HIPCHK(hipEventRecord(rec.b, st));
            rec.perms = 10.0 * (double)e.nwin;  // 8 element digests + the 2-block window
            rec.hashes = 9.0 * (double)e.nwin;
            std::lock_guard<std::mutex> lk(g_prof_mu);
            g_prof.push_back(rec);
        }
        return launch_plan(e.p, dig, (uint8_t*)d_out32, dig + e.dig_bytes, ws_bytes - e.dig_bytes, st);
    }
    if (n) {
        ProfRec rec{};
        const bool prof = prof_on();
        if (prof) {
            HIPCHK(hipEventCreate(&rec.a));
            HIPCHK(hipEventCreate(&rec.b));
            HIPCHK(hipEventRecord(rec.a, st));
        }
        TRY(launch_elem_digests(d_elems, n, elem_len, dig, st));
        if (prof) {
            HIPCHK(hipEventRecord(rec.b, st));
            rec.perms = (double)n * (double)mk::perms_for_len((uint64_t)elem_len + 4);
            rec.hashes = (double)n;
            std::lock_guard<std::mutex> lk(g_prof_mu);
            g_prof.push_back(rec);
        }
    }
    return launch_plan(e.p, dig, (uint8_t*)d_out32, dig + e.dig_bytes, ws_bytes - e.dig_bytes, st);
}

int host_tree_hash_elems_plain(const uint8_t* elems, uint64_t n, uint32_t elem_len, uint8_t* out) {
    if (!out || (n && elem_len && !elems)) return fail(MK_EINVAL, "null pointer");
    if (elem_len && n > (UINT64_MAX / 4) / elem_len) return fail(MK_EINVAL, "n * elem_len overflows");
    TRY(bind_call());
    DevCtx* c = ctx();
    std::lock_guard<std::mutex> lk(c->mu);
    ElemPlan e;
    TRY(make_elem_plan(n, elem_len, true, e));
    const size_t inb = n * (size_t)elem_len;
    TRY(grow(c->in, inb));
    TRY(grow(c->out, 32));
    TRY(grow(c->ws, e.ws_bytes));
    hipStream_t st = c->stream;
    if (inb) HIPCHK(hipMemcpyAsync(c->in.p, elems, inb, hipMemcpyHostToDevice, st));
    TRY(dev_tree_hash_elems(c->in.p, n, elem_len, c->out.p, c->ws.p, c->ws.cap, st));
    HIPCHK(hipMemcpyAsync(out, c->out.p, 32, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

int host_merkle_hash_plain(const uint8_t* items, uint64_t n, uint32_t item_len, uint8_t* out) {
    if (!out || (n && item_len && !items)) return fail(MK_EINVAL, "null pointer");
    TRY(bind_call());
    DevCtx* c = ctx();
    std::lock_guard<std::mutex> lk(c->mu);
    Plan p;
    TRY(mk::make_plan(n, item_len, false, 0, false, true, p));
    const size_t inb = n * (size_t)item_len;
    TRY(grow(c->in, inb));
    TRY(grow(c->out, 32));
    TRY(grow(c->ws, std::max<uint64_t>(p.small ? 256 : mk::plan_ws_bytes(p), list_tree_ws(n, item_len))));
    hipStream_t st = c->stream;
    if (inb) HIPCHK(hipMemcpyAsync(c->in.p, items, inb, hipMemcpyHostToDevice, st));
    if (list_tree_ok(n, item_len))
        TRY(dev_list_tree(c->in.p, n, item_len, c->out.p, (uint8_t*)c->ws.p, st));
    else
        TRY(launch_plan(p, (const uint8_t*)c->in.p, (uint8_t*)c->out.p, (uint8_t*)c->ws.p, c->ws.cap, st));
    HIPCHK(hipMemcpyAsync(out, c->out.p, 32, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

int host_merkle_multi(const uint8_t* items, uint64_t n, uint32_t item_len, int nshards, const int* devs_in,
                      uint8_t* out, uint32_t elem_len = 0);
int host_tree_hash_elems_plain(const uint8_t* elems, uint64_t n, uint32_t elem_len, uint8_t* out);

// merkleHash of a host buffer (the cgo TreeHash path).  A large buffer goes
// through the sharded path with its shards on this one device: shard i+1
// crosses PCIe while shard i's passes run, so the compute hides under the
// copy (8 GiB: copy then compute 162-164 ms) and the device holds
// two shard regions instead of the whole input.
#define MK_HOST_OVERLAP_MIN_LOG2 28  // bytes; 64 = never
int host_merkle_hash(const uint8_t* items, uint64_t n, uint32_t item_len, uint8_t* out) {
    if (!out || (n && item_len && !items)) return fail(MK_EINVAL, "null pointer");
    const uint64_t inb = n * (uint64_t)item_len;
    if (MK_HOST_OVERLAP_MIN_LOG2 < 64 && item_len && n <= (UINT64_MAX / 2) / item_len &&
        inb >= (1ull << (MK_HOST_OVERLAP_MIN_LOG2 & 63))) {
        TRY(bind_call());
        const int d = t_bound;
        const int ns = (int)std::min<uint64_t>(8, std::max<uint64_t>(2, inb >> 26));  // >= 64 MB per shard
        std::vector<int> devs(ns, d);
        return host_merkle_multi(items, n, item_len, ns, devs.data(), out);
    }
    return host_merkle_hash_plain(items, n, item_len, out);
}

// TreeHash of a host list of byte strings (the cgo path): like
// host_merkle_hash, a buffer of at least 2^MK_HOST_OVERLAP_MIN_LOG2 bytes goes
// through the sharded path on its one device, so shard i+1's elements cross
// PCIe while shard i is hashed (element digests, then the digest subtree).
int host_tree_hash_elems(const uint8_t* elems, uint64_t n, uint32_t elem_len, uint8_t* out) {
    if (!out || (n && elem_len && !elems)) return fail(MK_EINVAL, "null pointer");
    if (elem_len && n > (UINT64_MAX / 4) / elem_len) return fail(MK_EINVAL, "n * elem_len overflows");
    const uint64_t inb = n * (uint64_t)elem_len;
    if (MK_HOST_OVERLAP_MIN_LOG2 < 64 && elem_len && inb >= (1ull << (MK_HOST_OVERLAP_MIN_LOG2 & 63))) {
        TRY(bind_call());
        const int d = t_bound;
        const int ns = (int)std::min<uint64_t>(8, std::max<uint64_t>(2, inb >> 26));  // >= 64 MB per shard
        std::vector<int> devs(ns, d);
        return host_merkle_multi(elems, n, 32, ns, devs.data(), out, elem_len);
    }
    return host_tree_hash_elems_plain(elems, n, elem_len, out);
}

// ---- many lists ------------------------------------------------------------------------
int dev_merkle_many(const void* d_items, const mk::ManyPlan& mp, uint32_t nlists, void* d_roots, void* d_ws,
                    uint64_t ws_bytes, hipStream_t st) {
    if (ws_bytes < mp.ws_bytes)
        return fail(MK_ENOMEM, "workspace too small: %llu < %llu", (unsigned long long)ws_bytes,
                    (unsigned long long)mp.ws_bytes);
    if (nlists == 0) return MK_OK;
    if (!d_roots || !d_ws) return fail(MK_EINVAL, "null pointer");
    // the per-list descriptors are planned on the host and uploaded through
    // the pinned ring: a captured copy node would replay whatever a later
    // call left in that slot, so this entry point refuses stream capture
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIPCHK(hipStreamIsCapturing(st, &cap));
    if (cap != hipStreamCaptureStatusNone)
        return fail(MK_EINVAL, "mk_dev_ssz_merkle_many cannot be captured into a graph (host-planned descriptors)");
    uint8_t* ws = (uint8_t*)d_ws;
    auto* lists = (mk::ManyList*)(ws + mp.off_lists);
    auto* act = (mk::ManyAct*)(ws + mp.off_act);
    uint4* buf[2] = {(uint4*)(ws + mp.off_buf0), (uint4*)(ws + mp.off_buf1)};
    uint4* tops = (uint4*)(ws + mp.off_tops);
    DevCtx* c = ctx();
    TRY(upload_small(c, lists, mp.lists.data(), sizeof(mk::ManyList) * nlists, st));
    TRY(upload_small(c, act, mp.act.data(), sizeof(mk::ManyAct) * mp.act.size(), st));
    const uint8_t* items = (const uint8_t*)d_items;
    for (uint32_t l = 0; l < mp.nlevels; ++l) {  // level l+1 into buffer l % 2
        const uint64_t nodes = mp.lvl_nodes[l];
        const uint32_t nact = (uint32_t)(mp.lvl_begin[l + 1] - mp.lvl_begin[l]);
        if (!nodes) continue;
        const mk::ManyAct* a = act + mp.lvl_begin[l];
        if (l == 0)
            hipLaunchKernelGGL((mk::k_many_level<true>), dim3(ceil_div(nodes, 256)), dim3(256), 0, st, items, lists, a,
                               nact, nodes, (const uint4*)nullptr, buf[0], tops);
        else
            hipLaunchKernelGGL((mk::k_many_level<false>), dim3(ceil_div(nodes, 256)), dim3(256), 0, st, items, lists,
                               a, nact, nodes, (const uint4*)buf[(l - 1) % 2], buf[l % 2], tops);
        HIPCHK(hipGetLastError());
    }
    hipLaunchKernelGGL(mk::k_many_final, dim3(ceil_div(nlists, 256)), dim3(256), 0, st, items, lists, nlists,
                       (const uint4*)tops, (uint4*)d_roots);
    HIPCHK(hipGetLastError());
    for (size_t b = 0; b < mp.big.size(); ++b) {  // big lists: their own fused plans, one shared workspace
        const mk::ManyList& L = mp.lists[mp.big[b]];
        TRY(launch_plan(mp.big_plans[b], items + L.items_off, (uint8_t*)d_roots + 32 * (uint64_t)mp.big[b],
                        ws + mp.off_big, ws_bytes - mp.off_big, st));
    }
    return MK_OK;
}

// ---- struct hashing ---------------------------------------------------------------
int make_spec(const mk_field* fields, uint32_t nfields, uint32_t record_len, mk::StructSpec& sp) {
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

// k_struct_lock's compile-time layout: the SURVEY §8d ValidatorRecord
// (3 bytes fields, 6 uint64, 160-B records)
bool validator_layout(const mk::StructSpec& sp) {
    static const uint32_t off[9] = {0, 48, 80, 112, 120, 128, 136, 144, 152};
    static const uint32_t len[9] = {48, 32, 32, 8, 8, 8, 8, 8, 8};
    if (sp.nfields != 9 || sp.rec_len != 160 || sp.msg_len != 144) return false;
    for (uint32_t f = 0; f < 9; ++f) {
        const bool bytes = f < 3;
        if (sp.kind[f] != (bytes ? MK_FIELD_BYTES : MK_FIELD_RAW) || sp.off[f] != off[f] || sp.len[f] != len[f] ||
            sp.out_off[f] != (bytes ? 32 * f : 96 + 8 * (f - 3)))
            return false;
    }
    return true;
}

// The struct kernels' selectors for n records of layout sp at d_rec
struct StructForm {
    bool fused, vec16, layout, split;
    uint32_t nb, nraw;
};
static StructForm struct_form(const void* d_rec, uint64_t n, const mk::StructSpec& sp) {
    StructForm f{};
    // fused path: dword-granular single-block fields, dword-aligned message
    f.fused = sp.msg_len % 4 == 0 && sp.msg_len <= mk::kStructFusedMaxMsg && ((uintptr_t)d_rec % 4) == 0;
    f.vec16 = ((uintptr_t)d_rec % 16) == 0 && sp.rec_len % 16 == 0;
    for (uint32_t k = 0; k < sp.nfields; ++k) {
        if (sp.out_off[k] % 4) f.fused = false;
        if (sp.kind[k] == MK_FIELD_BYTES) {
            if ((sp.len[k] % 4) != 0 || sp.len[k] > mk::kStructFusedMaxField) f.fused = false;
            if (sp.off[k] % 16 || sp.off[k] + ((sp.len[k] + 15) & ~15u) > sp.rec_len) f.vec16 = false;
        } else if (sp.len[k] % 4 || sp.off[k] % 4) {
            f.fused = false;
        }
    }
    // compile-time message layout: NB dword-granular bytes fields (<= 64 B)
    // first, then NRAW 8-byte scalars, at 4-byte aligned record offsets
    while (f.nb < sp.nfields && sp.kind[f.nb] == MK_FIELD_BYTES) ++f.nb;
    f.layout = f.fused && f.nb > 0;
    for (uint32_t k = f.nb; k < sp.nfields; ++k)
        if (sp.kind[k] != MK_FIELD_RAW || sp.len[k] != 8) f.layout = false;
    f.nraw = sp.nfields - f.nb;
    f.split = n <= mk::kStructSplitMaxN;  // latency-bound: 4 lanes per record
    return f;
}

// roots of n records into d_roots (n x 32); d_msg holds n x msg_len bytes
int launch_struct_roots(const void* d_rec, uint64_t n, const mk::StructSpec& sp, void* d_msg, void* d_roots,
                        hipStream_t st) {
    if (n == 0) return MK_OK;
    const StructForm sf = struct_form(d_rec, n, sp);
    const bool fused = sf.fused, vec16 = sf.vec16, layout = sf.layout, split = sf.split;
    const uint32_t nb = sf.nb, nraw = sf.nraw;
    if (layout && split && nb == 3 && nraw == 6) {
        hipLaunchKernelGGL((mk::k_struct_split<3, 6>), dim3(ceil_div(n, 64)), dim3(256), 0, st, (const uint8_t*)d_rec,
                           n, sp, vec16 ? 1u : 0u, (uint4*)d_roots);
        HIPCHK(hipGetLastError());
        return MK_OK;
    }
    if (layout && split && nb == 2 && nraw == 0) {
        hipLaunchKernelGGL((mk::k_struct_split<2, 0>), dim3(ceil_div(n, 64)), dim3(256), 0, st, (const uint8_t*)d_rec,
                           n, sp, vec16 ? 1u : 0u, (uint4*)d_roots);
        HIPCHK(hipGetLastError());
        return MK_OK;
    }
    if (layout && nb == 3 && nraw == 6) {
        if (MK_STRUCT_LOCK && vec16 && validator_layout(sp) && n >= (1u << 18))  // phase-locked, partial last group
            hipLaunchKernelGGL(mk::k_struct_lock<false>,
                               dim3(std::min<uint64_t>(ceil_div(n, mk::kLockThreads), lock_grid_cap(st))),
                               dim3(mk::kLockThreads), 0, st, (const uint8_t*)d_rec, n, (uint4*)d_roots, 0u,
                               (uint4*)nullptr, (const uint8_t*)nullptr, (uint64_t)0, (uint4*)nullptr,
                               mk::StructPrev{});
        else
            hipLaunchKernelGGL((mk::k_struct_reg<3, 6>), dim3(ceil_div(n, mk::kStructThreads)),
                               dim3(mk::kStructThreads), 0, st, (const uint8_t*)d_rec, n, sp, vec16 ? 1u : 0u,
                               (uint4*)d_roots);
        HIPCHK(hipGetLastError());
        return MK_OK;
    }
    if (layout && nb == 2 && nraw == 0) {
        hipLaunchKernelGGL((mk::k_struct_reg<2, 0>), dim3(ceil_div(n, mk::kStructThreads)), dim3(mk::kStructThreads),
                           0, st, (const uint8_t*)d_rec, n, sp, vec16 ? 1u : 0u, (uint4*)d_roots);
        HIPCHK(hipGetLastError());
        return MK_OK;
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

// host-buffer entries: H2D in up to kH2dChunks pieces of at least kH2dMinChunk records
#define MK_H2D_CHUNKS 8
// (smaller floors measured slower: C1's 16,384 records 0.212 ms in one piece,
// 0.280 / 0.421 ms in 4 / 8 pieces; the per-piece copy + event cost outweighs
// the overlap, profiles/r05/h2d_chunk_ab.txt)
#define MK_H2D_MIN_CHUNK 65536
constexpr uint64_t kH2dChunks = MK_H2D_CHUNKS;
constexpr uint64_t kH2dMinChunk = MK_H2D_MIN_CHUNK;

// The registry list root with the merkleHash leaf pass fused into the
// phase-locked struct kernel (k_struct_lock gpw > 0): whole ValidatorRecord
// registries of >= 2^18 records at a 16-B aligned address.  The kernel writes
// the roots and the level-1 windows; the node passes and the length mix-in
// finish from the windows (dev_finish_nodes: the same odd rule at every
// level, hash.go:225-237).  false: not this layout / size (caller takes the
// two-launch path).
#define MK_STRUCT_WIN 1
bool struct_win_ok(const void* d_rec, uint64_t n, const mk::StructSpec& sp) {
    if (!MK_STRUCT_WIN || !MK_STRUCT_LOCK || n < (1u << 18)) return false;
    if (((uintptr_t)d_rec % 16) != 0 || sp.rec_len % 16 != 0 || !validator_layout(sp)) return false;
    for (uint32_t f = 0; f < sp.nfields; ++f)
        if (sp.kind[f] == MK_FIELD_BYTES && (sp.off[f] % 16 || sp.off[f] + ((sp.len[f] + 15) & ~15u) > sp.rec_len))
            return false;
    return true;
}

// d_vals (nullable): a second list of vbytes bytes whose level-1 windows the
// kernel hashes on its leftover lanes (item length dividing 128, 16-B aligned)
uint32_t struct_gpw(uint64_t n, hipStream_t st) {  // contiguous groups per workgroup
    return (uint32_t)ceil_div(ceil_div(n, mk::kLockThreads), lock_grid_cap(st));
}
int dev_struct_level1(const void* d_rec, uint64_t n, void* d_roots, void* d_wins, hipStream_t st,
                      const void* d_vals = nullptr, uint64_t vbytes = 0, void* d_vwins = nullptr,
                      const mk::StructPrev* prev = nullptr) {
    if (inject_ehip()) return fail(MK_EHIP, "hipLaunchKernelGGL: injected failure (MK_INJECT_EHIP)");
    const uint64_t ngroups = ceil_div(n, mk::kLockThreads);
    const uint32_t gpw = struct_gpw(n, st);
    if (prev)
        hipLaunchKernelGGL(mk::k_struct_lock<true>, dim3(ceil_div(ngroups, gpw)), dim3(mk::kLockThreads), 0, st,
                           (const uint8_t*)d_rec, n, (uint4*)d_roots, gpw, (uint4*)d_wins,
                           (const uint8_t*)(vbytes ? d_vals : nullptr), vbytes, (uint4*)d_vwins, *prev);
    else
        hipLaunchKernelGGL(mk::k_struct_lock<false>, dim3(ceil_div(ngroups, gpw)), dim3(mk::kLockThreads), 0, st,
                           (const uint8_t*)d_rec, n, (uint4*)d_roots, gpw, (uint4*)d_wins,
                           (const uint8_t*)(vbytes ? d_vals : nullptr), vbytes, (uint4*)d_vwins, mk::StructPrev{});
    HIPCHK(hipGetLastError());
    return MK_OK;
}

int dev_struct_list_root_win(const void* d_rec, uint64_t n, void* d_roots, void* d_wins, void* d_out32,
                             void* d_ws, uint64_t ws_bytes, hipStream_t st) {
    TRY(dev_struct_level1(d_rec, n, d_roots, d_wins, st));
    const uint64_t c1 = ceil_div(n, 8);  // windows: ceil(ceil(n / 4) / 2) chunk pairs
    if (ws_bytes < finish_ws_bytes(c1)) return fail(MK_ENOMEM, "workspace too small for the registry top");
    return dev_finish_nodes(d_wins, c1, n, d_out32, d_ws, ws_bytes, st);
}

// A small list of ValidatorRecord-shaped structs (3 bytes fields, 6 8-byte
// scalars: C1) in ONE launch, k_struct_list_fused<3, 6>: the k_struct_split
// records, the latency list tree's windows and levels, and the fused top's
// groups and mix-in, where they were three launches (round 6)
uint32_t next_arrive_slots(uint32_t k);
uint32_t top_arrive_slots(uint64_t parts);
static bool struct_list_fused_ok(const void* d_rec, uint64_t n, const mk::StructSpec& sp) {
    const StructForm f = struct_form(d_rec, n, sp);
    return n && f.layout && f.split && f.nb == 3 && f.nraw == 6 && list_tree_ok(n, 32);
}
static int launch_struct_list_fused(const void* d_rec, uint64_t n, const mk::StructSpec& sp, uint8_t* d_roots,
                                    uint8_t* d_sub, void* d_out32, hipStream_t st) {
    if (inject_ehip()) return fail(MK_EHIP, "hipLaunchKernelGGL: injected failure (MK_INJECT_EHIP)");
    const StructForm f = struct_form(d_rec, n, sp);
    mk::ReduceArgs a{};  // the window pass over the roots, as dev_list_tree's
    a.cb = 128;
    a.total = 32 * n;
    a.nchunks = ceil_div(a.total, a.cb);
    a.c1 = ceil_div(a.nchunks, 2);
    a.items = d_roots;
    a.n_items = n;
    a.levels = 4;
    const uint64_t nwg = ceil_div(n, 64);  // = the level-4 nodes, ceil(c1 / 8)
    hipLaunchKernelGGL((mk::k_struct_list_fused<3, 6>), dim3((uint32_t)nwg), dim3(1024), 0, st, (const uint8_t*)d_rec,
                       n, sp, f.vec16 ? 1u : 0u, (uint4*)d_roots, a, (uint32_t*)d_sub, (uint32_t*)d_out32,
                       next_arrive_slots(top_arrive_slots(nwg)));
    HIPCHK(hipGetLastError());
    return MK_OK;
}

uint64_t struct_list_ws(uint64_t n, const mk::StructSpec& sp) {
    Plan p;
    uint64_t mws = 256;
    if (mk::make_plan(n, 32, false, 0, false, true, p) == MK_OK && !p.small) mws = mk::plan_ws_bytes(p);
    mws = std::max(mws, list_tree_ws(n, 32));
    return align256(n * sp.msg_len) + align256(32 * n) + mws;
}

// ---- hashutil.MerkleRoot (merkleRoot.go:12-30) ------------------------------------
// Heap o[1..2n): leaves o[n+i] = Hash(values[i]); o[i] = Hash(o[2i] || o[2i+1])
// for i = n-1 .. 1; the result is o[1].  The children of a heap band
// [2^k, 2^(k+1)) are the contiguous range [2^(k+1), 2^(k+2)), so with
// P = 2^floor(log2 n): when n > P the partial band [P, n) is one pairwise
// level over o[2P, 2n), and everything above is a power-of-two binary tree
// over o[P, 2P) -- a node-input merkle plan.  (The reference's spurious
// newSet[0] = Hash(nil || o[1]) is computed and discarded; it is skipped.)
uint64_t pow2_floor(uint64_t n) {
    uint64_t p = 1;
    while (p * 2 <= n) p *= 2;
    return p;
}

uint64_t merkle_root_ws(uint64_t n) {
    if (n == 0) return 0;
    const uint64_t P = pow2_floor(n);
    Plan p;
    uint64_t ws = 0;
    if (P > 1 && mk::make_plan(P, 32, true, ilog2(P), false, true, p, true) == MK_OK) ws = mk::plan_ws_bytes(p);
    return 64 * n + align256(ws) + 256;
}

int dev_merkle_root(const void* d_data, const uint64_t* d_offs, uint64_t n, uint32_t fixed_len, void* d_heap,
                    uint64_t heap_bytes, void* d_leaves32, void* d_out32, hipStream_t st) {
    if (n == 0) return fail(MK_EINVAL, "MerkleRoot of an empty list (reference: index out of range)");
    if (!d_heap || !d_out32 || (!d_offs && !d_data && fixed_len)) return fail(MK_EINVAL, "null pointer");
    if (heap_bytes < merkle_root_ws(n)) return fail(MK_ENOMEM, "heap workspace too small");
    uint8_t* heap = (uint8_t*)d_heap;  // node i at heap + 32 i (node 0 unused)
    uint4* leaves = (uint4*)(heap + 32 * n);
    TRY(dev_leaf_hashes(d_data, d_offs, n, fixed_len, leaves, st));
    if (d_leaves32 && d_leaves32 != (void*)leaves)
        HIPCHK(hipMemcpyAsync(d_leaves32, leaves, 32 * n, hipMemcpyDeviceToDevice, st));
    if (n == 1) {  // the loop body never runs: o[1] is the hashed value
        HIPCHK(hipMemcpyAsync(d_out32, leaves, 32, hipMemcpyDeviceToDevice, st));
        return MK_OK;
    }
    const uint64_t P = pow2_floor(n);
    if (P < n) {  // partial band [P, n): o[i] = Hash(o[2i] || o[2i+1]) over o[2P, 2n)
        hipLaunchKernelGGL(mk::k_trie_level, dim3(ceil_div(n - P, 256)), dim3(256), 0, st,
                           (const uint4*)(heap + 64 * P), 2 * (n - P), (uint4*)(heap + 32 * P));
        HIPCHK(hipGetLastError());
    }
    Plan p;
    TRY(mk::make_plan(P, 32, true, ilog2(P), false, true, p, true));
    uint8_t* ws = heap + 64 * n;
    return launch_plan(p, heap + 32 * P, (uint8_t*)d_out32, ws, heap_bytes - 64 * n, st);
}

// ---- deposit trie -------------------------------------------------------------------
uint4* trie_level(void* d_levels, uint64_t cap, uint32_t d) {
    return (uint4*)d_levels + 2 * mk::trie_level_off(cap, d);
}

int check_trie(uint64_t cap, uint64_t count, uint64_t k, uint32_t depth) {
    if (depth == 0 || depth > 63) return fail(MK_EINVAL, "depth %u out of range (1..63)", depth);
    if (count + k > cap) return fail(MK_EINVAL, "trie capacity %llu < %llu deposits", (unsigned long long)cap,
                                     (unsigned long long)(count + k));
    if (count + k > (1ull << depth))
        return fail(MK_EINVAL, "%llu deposits do not fit a depth-%u trie", (unsigned long long)(count + k), depth);
    return MK_OK;
}

// Most parents any level d .. d_end-1 has when the nodes [lo, c) of level d
// changed (the right edge of an append; lo = 0 for a batch top).
uint64_t edge_max_parents(uint64_t lo, uint64_t c, uint32_t d, uint32_t d_end) {
    uint64_t m = 0;
    for (; d < d_end; ++d) {
        const uint64_t plo = lo >> 1, cp = (c + 1) >> 1;
        m = std::max(m, cp - plo);
        lo = plo;
        c = cp;
    }
    return m;
}

// k_trie_spread over levels d .. d_end-1 (one wave per parent, <= 16 parents;
// with leaves.k > 0 it first hashes the new deposits into level 0 [lo, c))
int launch_trie_spread(void* d_levels, uint64_t cap, uint32_t d, uint64_t lo, uint64_t c, uint32_t d_end,
                       uint32_t depth, void* d_root32, hipStream_t st, mk::SpreadLeaves leaves = {}) {
    const uint64_t m = std::max<uint64_t>(edge_max_parents(lo, c, d, d_end), leaves.k);
    uint32_t* lv = (uint32_t*)d_levels;
    uint32_t* root = (uint32_t*)d_root32;
    if (m <= 1)
        hipLaunchKernelGGL(mk::k_trie_spread<1>, dim3(1), dim3(64), 0, st, lv, cap, d, lo, c, d_end, depth, root,
                           leaves);
    else if (m <= 2)
        hipLaunchKernelGGL(mk::k_trie_spread<2>, dim3(1), dim3(128), 0, st, lv, cap, d, lo, c, d_end, depth, root,
                           leaves);
    else if (m <= 4)
        hipLaunchKernelGGL(mk::k_trie_spread<4>, dim3(1), dim3(256), 0, st, lv, cap, d, lo, c, d_end, depth, root,
                           leaves);
    else if (m <= 16 && m <= mk::kSpreadWavesMax)
        hipLaunchKernelGGL(mk::k_trie_spread<16>, dim3(1), dim3(1024), 0, st, lv, cap, d, lo, c, d_end, depth, root,
                           leaves);
    else
        return fail(MK_EINVAL, "internal: trie edge of %llu parents for the spread kernel", (unsigned long long)m);
    HIPCHK(hipGetLastError());
    return MK_OK;
}

// First of `k` consecutive arrival-counter slots for the next fused-top
// launch (mk::g_arrive, round robin, never running past the last slot; each
// counter's last arriving workgroup resets it).
uint32_t next_arrive_slots(uint32_t k) {
    static std::atomic<uint64_t> next{0};
    uint64_t cur = next.load(std::memory_order_relaxed), start;
    do {
        const uint64_t base = cur % mk::kArriveSlots;
        start = base + k > mk::kArriveSlots ? cur + (mk::kArriveSlots - base) : cur;
    } while (!next.compare_exchange_weak(cur, start + k, std::memory_order_relaxed));
    return (uint32_t)(start % mk::kArriveSlots);
}
uint32_t next_arrive_slot() { return next_arrive_slots(1); }
// Arrival slots one fused top of `parts` workgroups uses (k_trie_top_fused,
// k_merkle_top_fused): the final counter plus one per group of each grouping
// stage.  Reserving only those, not kTopGroupSlots, keeps ~1,300 small fused
// tops (C1's list tree: 16 workgroups, one slot) in flight on a device
// before a slot comes round again, where a fixed 129 allowed 31.
uint32_t top_arrive_slots(uint64_t parts) {
    uint32_t k = 1;
    while (mk::kTopGroupLog2 > 0 && parts > mk::kTopGroup) {
        parts = ceil_div(parts, (uint64_t)mk::kTopGroup);
        k += (uint32_t)parts;
    }
    return k;
}

// Levels d_from+1 .. d_to of the batch build over `n` deposits, level d_from
// complete; the root (level depth node 0) to d_root32 when d_to == depth.
// nt_max / spread_max: the largest k_trie_top3 workgroup and k_trie_spread
// wave count (256 / 4: at most one wave per SIMD, which fits beside a
// resident k_trie_rec_lock<1024, 4, true> workgroup of 104 VGPRs).
int trie_levels_range(void* d_levels, uint64_t cap, uint64_t n, uint32_t d_from, uint32_t d_to, uint32_t depth,
                      void* d_root32, hipStream_t st, uint32_t nt_max = mk::kMidThreads,
                      uint32_t spread_max = mk::kSpreadWavesMax, bool fused = false) {
    // Wide levels: one launch per level (every lane busy); the narrow top
    // (<= 2^17 nodes) plus the zero-sibling tail: k_trie_top3 (bit-interleaved
    // lane pairs), log2(NT) levels per workgroup of NT inputs, the last
    // launch to the top.  `fused` (a whole trie alone on the stream): every
    // level from the first of <= 2^20 nodes to the root in one launch
    // (k_trie_top_fused).
    uint64_t c = mk::trie_count(n, d_from);
    uint32_t d = d_from;
    if (fused && MK_TRIE_TOP_FUSED && d_to == depth && d_root32) {
        constexpr uint64_t NT = 1024;
        while (d < d_to && c > NT * NT) {
            const uint64_t cn = (c + 1) / 2;
            hipLaunchKernelGGL(mk::k_trie_level, dim3(ceil_div(cn, 256)), dim3(256), 0, st,
                               (const uint4*)trie_level(d_levels, cap, d), c, trie_level(d_levels, cap, d + 1));
            HIPCHK(hipGetLastError());
            c = cn;
            ++d;
        }
        hipLaunchKernelGGL(mk::k_trie_top_fused<NT>, dim3(ceil_div(c, NT)), dim3(NT), 0, st, (uint32_t*)d_levels, cap,
                           c, d, depth, (uint32_t*)d_root32, next_arrive_slots(top_arrive_slots(ceil_div(c, NT))));
        HIPCHK(hipGetLastError());
        return MK_OK;
    }
    while (d < d_to && c > kTrieTopMax) {
        const uint64_t cn = (c + 1) / 2;
        hipLaunchKernelGGL(mk::k_trie_level, dim3(ceil_div(cn, 256)), dim3(256), 0, st,
                           (const uint4*)trie_level(d_levels, cap, d), c, trie_level(d_levels, cap, d + 1));
        HIPCHK(hipGetLastError());
        c = cn;
        ++d;
    }
    bool root_done = false;
    while (d < d_to) {
        if (MK_TRIE_SPREAD && c <= 2 * spread_max) {  // the last <= 5 levels + zero-sibling tail
            void* root = d_to == depth ? d_root32 : nullptr;
            TRY(launch_trie_spread(d_levels, cap, d, 0, c, d_to, depth, root, st));
            root_done = root != nullptr;
            d = d_to;
            break;
        }
        uint32_t nt = mk::kWaveThreads;
        while (nt < nt_max && ceil_div(c, nt) > kTrieTopWgs) nt *= 2;
        while (nt < nt_max && c <= nt_max && c > nt) nt *= 2;  // the last <= nt_max nodes in one WG
        const uint64_t nwg = ceil_div(c, nt);
        uint32_t k = nwg == 1 ? d_to - d : std::min<uint32_t>(ilog2(nt), d_to - d);
        if (MK_TRIE_SPREAD && nwg == 1) {  // stop where k_trie_spread takes over
            uint64_t cc = c;
            uint32_t kk = 0;
            while (kk < k && cc > 2 * spread_max) {
                cc = (cc + 1) / 2;
                ++kk;
            }
            k = kk;
        }
        const uint32_t* src = (const uint32_t*)trie_level(d_levels, cap, d);
        uint32_t* dst = (uint32_t*)trie_level(d_levels, cap, d + 1);
        const uint64_t capn = mk::trie_count(cap, d + 1);
        switch (nt) {
            case 64: hipLaunchKernelGGL(mk::k_trie_top3<64>, dim3(nwg), dim3(64), 0, st, src, c, dst, k, capn); break;
            case 128: hipLaunchKernelGGL(mk::k_trie_top3<128>, dim3(nwg), dim3(128), 0, st, src, c, dst, k, capn); break;
            case 256: hipLaunchKernelGGL(mk::k_trie_top3<256>, dim3(nwg), dim3(256), 0, st, src, c, dst, k, capn); break;
            case 512: hipLaunchKernelGGL(mk::k_trie_top3<512>, dim3(nwg), dim3(512), 0, st, src, c, dst, k, capn); break;
            default: hipLaunchKernelGGL(mk::k_trie_top3<1024>, dim3(nwg), dim3(1024), 0, st, src, c, dst, k, capn); break;
        }
        HIPCHK(hipGetLastError());
        for (uint32_t i = 0; i < k; ++i) c = (c + 1) / 2;
        d += k;
    }
    if (d_to == depth && d_root32 && !root_done)
        HIPCHK(hipMemcpyAsync(d_root32, trie_level(d_levels, cap, depth), 32, hipMemcpyDeviceToDevice, st));
    return MK_OK;
}

// Levels 1..nlv of the batch build for the leaves [done, n) (level 0 holds
// them; the levels of [0, done) are already built): the suffix of each level,
// one k_trie_level launch per level.
int trie_suffix_levels(void* d_levels, uint64_t cap, uint64_t n, uint64_t done, uint32_t nlv, hipStream_t st) {
    for (uint32_t d = 0; d < nlv; ++d) {
        const uint64_t c = mk::trie_count(n, d), plo = done >> (d + 1);
        if (c <= 2 * plo) continue;  // nothing left at this level
        hipLaunchKernelGGL(mk::k_trie_level, dim3(ceil_div(((c + 1) >> 1) - plo, 256)), dim3(256), 0, st,
                           (const uint4*)(trie_level(d_levels, cap, d) + 2 * (2 * plo)), c - 2 * plo,
                           trie_level(d_levels, cap, d + 1) + 2 * plo);
        HIPCHK(hipGetLastError());
    }
    return MK_OK;
}

// Batch build front over an empty trie: leaf hashes into level 0, then
// levels 1 .. d_to.  A whole trie in one call (d_to == depth) of 280-B
// deposits at a 16-B aligned address: whole groups of the phase-locked
// k_trie_rec_lock_sm (leaves + levels 1-2 in one launch), the rest (a
// partial group) k_keccak_rec + k_trie_level.  A front whose top the caller
// runs elsewhere (d_to < depth: pipeline.TriePipeline overlaps trie i's top
// with trie i+1's front) keeps the free-running kernels: a locked workgroup
// fills its CU, so the top could not co-run (one process, same box,
// profiles/r04c-r04d: one trie 0.596 -> 0.582 ms locked, the stream of
// tries 0.514 -> 0.604 ms/step).
int trie_front(void* d_levels, uint64_t cap, const void* d_data, const uint64_t* d_offs, uint64_t n,
               uint32_t fixed_len, uint32_t d_to, uint32_t depth, void* d_root32, hipStream_t st) {
    constexpr uint32_t NT = 1024, DPT = 4, nlv = 2;  // k_trie_rec_lock_sm: 4 slots per thread, levels 0-2
    const uint64_t ng = (MK_TRIE_LOCK && !d_offs && fixed_len == 280 && ((uintptr_t)d_data % 16) == 0 &&
                         n >= MK_TRIE_LOCK_MIN && d_to == depth && depth >= nlv)
                            ? n / (NT * DPT)
                            : 0;
    if (!ng) {
        TRY(dev_leaf_hashes(d_data, d_offs, n, fixed_len, trie_level(d_levels, cap, 0), st));
        return trie_levels_range(d_levels, cap, n, 0, d_to, depth, d_root32, st, mk::kMidThreads,
                                 mk::kSpreadWavesMax, d_to == depth);
    }
    if (inject_ehip()) return fail(MK_EHIP, "hipLaunchKernelGGL: injected failure (MK_INJECT_EHIP)");
    uint4* L[3];
    for (uint32_t d = 0; d <= nlv; ++d) L[d] = trie_level(d_levels, cap, d);
    // persistent: every workgroup runs the same number of groups where possible
    const uint64_t cap_wg = std::min<uint64_t>(MK_TRIE_LOCK_GRID, lock_grid_cap(st));
    const uint64_t grid = ceil_div(ng, ceil_div(ng, cap_wg));
    // slot-major (lane m, slot i: deposit 64 i + m), not the row form of the
    // stream's k_trie_rec_lock<1024, 4, true> (deposits 4m .. 4m + 3 per
    // lane): one trie 0.4908-0.4913 -> 0.4781-0.4798 ms, fetch 561 -> 535 MB
    // (profiles/r06/c5_slot_major/, interleaved on one box)
    hipLaunchKernelGGL(mk::k_trie_rec_lock_sm<NT>, dim3(grid), dim3(NT), 0, st, (const uint2*)d_data, ng, L[0], L[1],
                       L[2]);
    HIPCHK(hipGetLastError());
    const uint64_t done = ng * NT * DPT;
    if (done < n) {
        TRY(dev_hash_batch((const uint8_t*)d_data + done * 280, n - done, 280, L[0] + 2 * done, st));
        TRY(trie_suffix_levels(d_levels, cap, n, done, nlv, st));
    }
    return trie_levels_range(d_levels, cap, n, nlv, d_to, depth, d_root32, st, mk::kMidThreads, mk::kSpreadWavesMax,
                             true);
}

// A stream of tries with the previous trie's wide top in the front's
// lock-step slots (k_trie_rec_lock<1024, 4, true>): 280-B deposits at a 16-B
// aligned address, n a whole number of 4096-deposit groups, one group per
// workgroup (n / 4096 <= the stream's CUs), depth >= 7.
bool trie_pipe_ok(const void* d_data, uint64_t n, uint32_t fixed_len, uint32_t depth, hipStream_t st) {
    constexpr uint64_t G = 1024 * 4;
    return MK_TRIE_LOCK && fixed_len == 280 && ((uintptr_t)d_data % 16) == 0 && n >= G && n % G == 0 &&
           n / G <= std::min<uint64_t>(MK_TRIE_LOCK_GRID, lock_grid_cap(st)) && depth >= 7;
}

// Levels 0..2 of the trie in d_levels and levels 3..7 of the previous one in
// d_prev (NULL: none), one launch.
int trie_front_pipe(void* d_levels, void* d_prev, uint64_t cap, const void* d_data, uint64_t n, uint32_t depth,
                    hipStream_t st) {
    if (inject_ehip()) return fail(MK_EHIP, "hipLaunchKernelGGL: injected failure (MK_INJECT_EHIP)");
    uint4* L[4];
    for (uint32_t d = 0; d < 4; ++d) L[d] = trie_level(d_levels, cap, d);
    mk::TriePrev prev{};
    if (d_prev) {
        prev.l2 = trie_level(d_prev, cap, 2);
        for (uint32_t k = 0; k < 5; ++k) prev.l[k] = trie_level(d_prev, cap, 3 + k);
        prev.live = 1;
    }
    const uint64_t ng = n / (1024 * 4);
    hipLaunchKernelGGL((mk::k_trie_rec_lock<1024, 4, true>), dim3(ng), dim3(1024), 0, st, (const uint2*)d_data, ng,
                       L[0], L[1], L[2], L[3], prev);
    HIPCHK(hipGetLastError());
    return MK_OK;
}

int dev_trie_append(void* d_levels, uint64_t cap, uint64_t count, const void* d_data, const uint64_t* d_offs,
                    uint64_t k, uint32_t fixed_len, uint32_t depth, void* d_root32, hipStream_t st) {
    TRY(check_trie(cap, count, k, depth));
    if (!d_root32 || (cap && !d_levels)) return fail(MK_EINVAL, "null pointer");
    if (k && !d_offs && !d_data && fixed_len) return fail(MK_EINVAL, "null deposits");
    if (count + k == 0) {
        HIPCHK(hipMemsetAsync(d_root32, 0, 32, st));
        return MK_OK;
    }
    if (MK_TRIE_SPREAD && k <= mk::kSpreadWavesMax && edge_max_parents(count, count + k, 0, depth) <=
                                                          mk::kSpreadWavesMax) {
        // a few deposits (powchain's one log at a time): the leaf hashes and
        // the whole right edge in one single-workgroup launch
        const bool w8 = !d_offs && fixed_len % 8 == 0 && ((uintptr_t)d_data % 8) == 0;
        mk::SpreadLeaves lv{(const uint8_t*)d_data, d_offs, fixed_len, (uint32_t)k, (uint32_t)w8};
        // one deposit: a register chain with the siblings prefetched
        // (k_trie_append1: 100.5 against 102.6 us per append + Root() through
        // k_trie_spread<1>, 2^16-deposit trie, profiles/r06/append/)
        if (k == 1 && depth <= 64) {
            hipLaunchKernelGGL(mk::k_trie_append1, dim3(1), dim3(64), 0, st, (uint32_t*)d_levels, cap, count, depth,
                               (uint32_t*)d_root32, lv);
            HIPCHK(hipGetLastError());
            return MK_OK;
        }
        return launch_trie_spread(d_levels, cap, 0, count, count + k, depth, depth, d_root32, st, lv);
    }
    if (count == 0) return trie_front(d_levels, cap, d_data, d_offs, k, fixed_len, depth, depth, d_root32, st);
    // leaf hashes of the new deposits: Hash(depositData) (deposit_trie.go:32)
    TRY(dev_leaf_hashes(d_data, d_offs, k, fixed_len, trie_level(d_levels, cap, 0) + 2 * count, st));
    // right edge only: level d changes on [lo, c)
    uint64_t lo = count, c = count + k;
    uint32_t d = 0;
    while (d < depth && c - lo > kAppendMaxRange) {
        const uint64_t plo = lo >> 1;
        hipLaunchKernelGGL(mk::k_trie_level, dim3(ceil_div(((c + 1) >> 1) - plo, 256)), dim3(256), 0, st,
                           (const uint4*)(trie_level(d_levels, cap, d) + 2 * (2 * plo)), c - 2 * plo,
                           trie_level(d_levels, cap, d + 1) + 2 * plo);
        HIPCHK(hipGetLastError());
        lo = plo;
        c = (c + 1) >> 1;
        ++d;
    }
    if (d == depth) {
        HIPCHK(hipMemcpyAsync(d_root32, trie_level(d_levels, cap, depth), 32, hipMemcpyDeviceToDevice, st));
        return MK_OK;
    }
    // lane pairs (k_trie_append) while a level has more than kSpreadWavesMax
    // changed parents, then one state per wave (k_trie_spread) to the root
    uint32_t d_stop = d;
    uint64_t slo = lo, sc = c;
    while (d_stop < depth && (!MK_TRIE_SPREAD || edge_max_parents(slo, sc, d_stop, depth) > mk::kSpreadWavesMax)) {
        slo >>= 1;
        sc = (sc + 1) >> 1;
        ++d_stop;
    }
    const uint64_t r = c - lo;
    uint32_t* lv = (uint32_t*)d_levels;
    uint32_t* root = (uint32_t*)d_root32;
    if (d_stop > d) {
        if (r <= 60)
            hipLaunchKernelGGL(mk::k_trie_append<64>, dim3(1), dim3(64), 0, st, lv, cap, d, lo, c, d_stop, depth, root);
        else if (r <= 252)
            hipLaunchKernelGGL(mk::k_trie_append<256>, dim3(1), dim3(256), 0, st, lv, cap, d, lo, c, d_stop, depth,
                               root);
        else
            hipLaunchKernelGGL(mk::k_trie_append<1024>, dim3(1), dim3(1024), 0, st, lv, cap, d, lo, c, d_stop, depth,
                               root);
        HIPCHK(hipGetLastError());
    }
    if (d_stop < depth) TRY(launch_trie_spread(d_levels, cap, d_stop, slo, sc, depth, depth, d_root32, st));
    return MK_OK;
}

int dev_trie_branch(const void* d_levels, uint64_t cap, uint64_t count, uint32_t depth, uint64_t index,
                    void* d_branch, hipStream_t st) {
    if (depth == 0 || depth > 63) return fail(MK_EINVAL, "depth %u out of range (1..63)", depth);
    if (!d_branch || (count && !d_levels)) return fail(MK_EINVAL, "null pointer");
    if (count > cap) return fail(MK_EINVAL, "count > capacity");
    hipLaunchKernelGGL(mk::k_trie_branch, dim3(1), dim3(64), 0, st, (const uint4*)d_levels, cap, count, depth, index,
                       (uint4*)d_branch);
    HIPCHK(hipGetLastError());
    return MK_OK;
}

// ---- multi-device ------------------------------------------------------------------------
std::mutex g_multi_mu;  // one multi-device call at a time (device locks are taken per device)
std::map<std::vector<int>, std::vector<ncclComm_t>> g_comms;

int comms_for(const std::vector<int>& devs, std::vector<ncclComm_t>*& out) {
    auto it = g_comms.find(devs);
    if (it == g_comms.end()) {
        std::vector<ncclComm_t> comms(devs.size(), nullptr);
        if (ncclCommInitAll(comms.data(), (int)devs.size(), devs.data()) != ncclSuccess)
            return fail(MK_ECOMM, "ncclCommInitAll(%zu) failed", devs.size());
        it = g_comms.emplace(devs, std::move(comms)).first;
    }
    out = &it->second;
    return MK_OK;
}

// Shard s of the frontier sharding reduced on the bound device: nodes of
// level (h - k) into d_block (k = 0: the 32-B shard root).
int launch_shard(const uint8_t* d_items, uint64_t sn, uint32_t item_len, uint32_t h, uint32_t k, uint8_t* d_block,
                 const DevBuf& ws, hipStream_t st) {
    if (sn == 0) {
        HIPCHK(hipMemsetAsync(d_block, 0, (size_t)32 << k, st));
        return MK_OK;
    }
    Plan p;
    TRY(mk::make_plan(sn, item_len, true, h, true, ((uintptr_t)d_items % 16) == 0, p, false, k));
    return launch_plan(p, d_items, d_block, (uint8_t*)ws.p, ws.cap, st);
}

uint32_t multi_frontier(uint32_t h) { return h > 5 ? std::min<uint32_t>(10, h - 5) : 0; }

// Test hook (MK_FORCE_COLLECTIVE=1 in the environment when the library is
// loaded): a one-device multi call takes the sharded path with one shard —
// frontier pass, ncclCommInitAll + in-place ncclAllGather over one rank,
// finisher — instead of the plain one-device merkleHash, so the library's
// RCCL code runs on a one-GPU box (RCCL refuses two ranks on one device).
bool force_collective() {
    static const bool on = [] {
        const char* e = std::getenv("MK_FORCE_COLLECTIVE");
        return e && e[0] == '1';
    }();
    return on;
}

// Uploads items[0, bytes) into d_dst on `copy`: chunked hipMemcpyAsync
// straight from the caller's pageable buffer, i.e. the runtime's own staged
// DMA (52-55 GB/s on one MI355X link).  The first multi-device form copied
// through two pinned slots with a host memcpy per chunk; one host thread's
// memcpy capped that at 22-35 GB/s (profiles/r02d/multi_host_probe.log).
int staged_upload(DevCtx* c, uint8_t* d_dst, const uint8_t* src, size_t bytes) {
    for (size_t off = 0; off < bytes; off += kStageBytes)
        HIPCHK(hipMemcpyAsync(d_dst + off, src + off, std::min(kStageBytes, bytes - off), hipMemcpyHostToDevice,
                              c->copy));
    return MK_OK;
}

struct MultiJob {
    int dev;
    std::vector<uint32_t> shards;  // shard indices on this device, in order
};

// Worker of mk_ssz_merkle_hash_multi for one device: its shards are uploaded
// into two alternating regions on the copy stream; each shard's passes run on
// the compute stream once its upload landed, while the next shard uploads.
// elem_len > 0 (the TreeHash-of-byte-strings path): `items` are elements of
// elem_len bytes and the tree's 32-B items are their digests
// K(le32(elem_len) || element); a shard's elements are uploaded, hashed into
// the matching digest region (k_elem_digests) and reduced from there.
int multi_device_worker(const MultiJob& job, const uint8_t* items, const std::vector<uint64_t>& begin,
                        uint32_t item_len, uint32_t h, uint32_t k, size_t block, uint32_t elem_len = 0) {
    TRY(bind_dev(job.dev));
    DevCtx* c = ctx();
    const size_t tree_region = (size_t)((1ull << h) * mk::chunk_bytes(item_len));  // tree items of a shard
    const size_t per_shard_items = tree_region / item_len;
    const size_t region = elem_len ? per_shard_items * elem_len : tree_region;     // uploaded bytes of a shard
    const int nreg = job.shards.size() > 1 ? 2 : 1;
    TRY(grow(c->in, std::max<size_t>(region, 16) * nreg));
    if (elem_len) TRY(grow(c->dig, tree_region * nreg));
    TRY(grow(c->out, block * (begin.size() - 1) + 32));
    Plan p;
    uint64_t wsb = 256;
    for (uint32_t s : job.shards) {
        const uint64_t sn = begin[s + 1] - begin[s];
        if (sn && mk::make_plan(sn, item_len, true, h, true, true, p, false, k) == MK_OK)
            wsb = std::max(wsb, mk::plan_ws_bytes(p));
    }
    TRY(grow(c->ws, wsb));
    c->region_used[0] = c->region_used[1] = false;
    for (size_t i = 0; i < job.shards.size(); ++i) {
        const uint32_t s = job.shards[i];
        const int r = (int)(i % 2);
        uint8_t* dreg = (uint8_t*)c->in.p + region * r;
        const uint64_t sn = begin[s + 1] - begin[s];
        const uint32_t up_len = elem_len ? elem_len : item_len;
        if (c->region_used[r]) HIPCHK(hipStreamWaitEvent(c->copy, c->region_ev[r], 0));  // its last shard is done
        TRY(staged_upload(c, dreg, items + begin[s] * up_len, sn * (size_t)up_len));
        HIPCHK(hipEventRecord(c->h2d, c->copy));
        HIPCHK(hipStreamWaitEvent(c->stream, c->h2d, 0));
        const uint8_t* tree_items = dreg;
        if (elem_len) {
            uint8_t* dg = (uint8_t*)c->dig.p + tree_region * r;
            TRY(launch_elem_digests(dreg, sn, elem_len, dg, c->stream));
            tree_items = dg;
        }
        TRY(launch_shard(tree_items, sn, item_len, h, k, (uint8_t*)c->out.p + block * s, c->ws, c->stream));
        HIPCHK(hipEventRecord(c->region_ev[r], c->stream));
        c->region_used[r] = true;
    }
    return MK_OK;
}

int host_merkle_multi(const uint8_t* items, uint64_t n, uint32_t item_len, int nshards, const int* devs_in,
                      uint8_t* out, uint32_t elem_len) {
    if (nshards <= 0) return fail(MK_EINVAL, "nshards %d <= 0", nshards);
    if (elem_len && item_len != 32) return fail(MK_EINVAL, "element digests are 32-B tree items");
    if (!out || (n && item_len && !items)) return fail(MK_EINVAL, "null pointer");
    const int nvis = probe_devices();
    if (nvis <= 0) return fail(MK_ENODEV, "no gfx950 device visible");
    std::vector<int> devs(nshards);
    for (int s = 0; s < nshards; ++s) {
        devs[s] = devs_in ? devs_in[s] : s;
        if (devs[s] < 0 || devs[s] >= nvis)
            return fail(MK_ENODEV, "shard %d: device %d out of range (%d visible)", s, devs[s], nvis);
    }
    uint32_t h = 0, ne = 0;
    std::vector<uint64_t> begin(nshards + 1);
    TRY(mk::shard_plan(n, item_len, (uint32_t)nshards, &h, &ne, begin.data()));
    if (ne <= 1 && !(nshards == 1 && h > 5 && force_collective())) {  // too small to shard: one device
        mk_call local{};
        local.device = devs[0];
        mk_call* prev = mk::swap_call(&local);
        const int rc = elem_len ? host_tree_hash_elems_plain(items, n, elem_len, out)
                                : host_merkle_hash_plain(items, n, item_len, out);
        mk::swap_call(prev);
        return rc ? fail(rc, "%s", local.err) : MK_OK;
    }
    std::vector<int> uniq;
    for (int d : devs)
        if (std::find(uniq.begin(), uniq.end(), d) == uniq.end()) uniq.push_back(d);
    const bool one_each = (int)uniq.size() == nshards;
    // several devices or RCCL: one multi-device call at a time (device lock
    // order, the communicator cache); shards on one device need only that
    // device's lock, so one-device calls on different devices stay concurrent
    std::unique_lock<std::mutex> mlk(g_multi_mu, std::defer_lock);
    if (uniq.size() > 1 || one_each) mlk.lock();
    const uint32_t k = multi_frontier(h);
    const size_t block = (size_t)32 << k;
    std::vector<MultiJob> jobs;
    for (int d : uniq) {
        MultiJob j{d, {}};
        for (int s = 0; s < nshards; ++s)
            if (devs[s] == d && begin[s + 1] > begin[s]) j.shards.push_back((uint32_t)s);
        jobs.push_back(j);
    }
    std::vector<std::unique_lock<std::mutex>> locks;
    for (int d : uniq) {
        TRY(bind_dev(d));
        locks.emplace_back(g_ctx[d]->mu);
    }
    // one host thread per device: uploads through pinned staging + the shard passes
    std::vector<int> rcs(jobs.size(), MK_OK);
    std::vector<std::string> errs(jobs.size());
    std::vector<std::thread> th;
    mk_call* parent = mk::current_call();
    for (size_t j = 0; j < jobs.size(); ++j)
        th.emplace_back([&, j]() {
            mk_call local{};
            local.device = jobs[j].dev;
            mk::swap_call(&local);
            rcs[j] = multi_device_worker(jobs[j], items, begin, item_len, h, k, block, elem_len);
            if (rcs[j] == MK_OK && !one_each && hipStreamSynchronize(g_ctx[jobs[j].dev]->stream) != hipSuccess)
                rcs[j] = fail(MK_EHIP, "hipStreamSynchronize failed on device %d", jobs[j].dev);
            errs[j] = local.err;
            mk::swap_call(nullptr);
        });
    for (auto& t : th) t.join();
    for (size_t j = 0; j < jobs.size(); ++j)
        if (rcs[j] != MK_OK) {
            mk::swap_call(parent);
            return fail(rcs[j], "device %d: %s", jobs[j].dev, errs[j].c_str());
        }
    DevCtx* c0 = g_ctx[devs[0]];
    uint8_t* lvl0 = (uint8_t*)c0->out.p;
    if (one_each) {  // gather the frontier blocks over RCCL (in place: block s of every device)
        std::vector<ncclComm_t>* comms = nullptr;
        TRY(comms_for(devs, comms));
        // (blocks of empty shards are never read: they follow the non-empty ones)
        if (ncclGroupStart() != ncclSuccess) return fail(MK_ECOMM, "ncclGroupStart");
        for (int s = 0; s < nshards; ++s) {
            uint8_t* lvl = (uint8_t*)g_ctx[devs[s]]->out.p;
            if (ncclAllGather(lvl + block * s, lvl, block, ncclUint8, (*comms)[s], g_ctx[devs[s]]->stream) !=
                ncclSuccess) {
                ncclGroupEnd();
                return fail(MK_ECOMM, "ncclAllGather on device %d", devs[s]);
            }
        }
        if (ncclGroupEnd() != ncclSuccess) return fail(MK_ECOMM, "ncclGroupEnd");
    } else {  // several shards per device: copy the other devices' blocks to devs[0]
        TRY(bind_dev(devs[0]));
        for (uint32_t s = 0; s < ne; ++s)  // (blocks of the trailing empty shards are never read)
            if (devs[s] != devs[0])
                HIPCHK(hipMemcpyPeerAsync(lvl0 + block * s, devs[0], (uint8_t*)g_ctx[devs[s]]->out.p + block * s,
                                          devs[s], block, c0->stream));
    }
    TRY(bind_dev(devs[0]));
    const uint64_t last_nodes = k ? mk::frontier_nodes(begin[ne] - begin[ne - 1], item_len, h, k) : 1;
    const uint64_t count = ((uint64_t)(ne - 1) << k) + last_nodes;
    uint8_t* root = lvl0 + block * nshards;
    if (k) {
        TRY(grow(c0->aux, finish_ws_bytes(count)));
        TRY(dev_finish_nodes(lvl0, count, n, root, c0->aux.p, c0->aux.cap, c0->stream));
    } else {
        TRY(dev_finish(lvl0, ne, n, root, c0->stream));
    }
    HIPCHK(hipMemcpyAsync(out, root, 32, hipMemcpyDeviceToHost, c0->stream));
    for (int d : uniq) {
        TRY(bind_dev(d));
        HIPCHK(hipStreamSynchronize(g_ctx[d]->stream));
    }
    return MK_OK;
}

int dev_merkle_multi(const void* const* d_shards, uint64_t n, uint32_t item_len, int ndev, void* d_out32,
                     void* const* streams) {
    if (ndev <= 0 || !d_shards || !d_out32) return fail(MK_EINVAL, "bad arguments");
    if (probe_devices() < ndev) return fail(MK_ENODEV, "%d devices requested, %d visible", ndev, g_ndev);
    uint32_t h = 0, ne = 0;
    std::vector<uint64_t> begin(ndev + 1);
    TRY(mk::shard_plan(n, item_len, (uint32_t)ndev, &h, &ne, begin.data()));
    auto stream_of = [&](int d) { return streams && streams[d] ? (hipStream_t)streams[d] : g_ctx[d]->stream; };
    // one multi call at a time: the mout/mws/maux buffers and the communicator cache
    std::lock_guard<std::mutex> mlk(g_multi_mu);
    if (ne <= 1 && !(ndev == 1 && h > 5 && force_collective())) {
        TRY(bind_dev(0));
        DevCtx* c = ctx();
        Plan p;
        TRY(mk::make_plan(n, item_len, false, 0, false, ((uintptr_t)d_shards[0] % 16) == 0, p));
        TRY(grow(c->mws, p.small ? 256 : mk::plan_ws_bytes(p)));
        return launch_plan(p, (const uint8_t*)d_shards[0], (uint8_t*)d_out32, (uint8_t*)c->mws.p, c->mws.cap,
                           stream_of(0));
    }
    const uint32_t k = multi_frontier(h);
    const size_t block = (size_t)32 << k;
    const uint64_t last_nodes = k ? mk::frontier_nodes(begin[ne] - begin[ne - 1], item_len, h, k) : 1;
    const uint64_t count = ((uint64_t)(ne - 1) << k) + last_nodes;
    std::vector<int> devs(ndev);
    for (int d = 0; d < ndev; ++d) devs[d] = d;
    // size every buffer (and the communicators) before the first launch, so
    // no call frees or allocates between its own enqueues
    for (int d = 0; d < ndev; ++d) {
        TRY(bind_dev(d));
        DevCtx* c = ctx();
        TRY(grow(c->mout, block * ndev + 32));
        const uint64_t sn = begin[d + 1] - begin[d];
        Plan p;
        if (sn) {
            TRY(mk::make_plan(sn, item_len, true, h, true, ((uintptr_t)d_shards[d] % 16) == 0, p, false, k));
            TRY(grow(c->mws, mk::plan_ws_bytes(p)));
        }
        if (d == 0 && k) TRY(grow(c->maux, finish_ws_bytes(count)));
    }
    std::vector<ncclComm_t>* comms = nullptr;
    TRY(comms_for(devs, comms));
    for (int d = 0; d < ndev; ++d) {  // every device: its shard to the frontier level, block d
        TRY(bind_dev(d));
        DevCtx* c = ctx();
        TRY(launch_shard((const uint8_t*)d_shards[d], begin[d + 1] - begin[d], item_len, h, k,
                         (uint8_t*)c->mout.p + block * d, c->mws, stream_of(d)));
    }
    if (ncclGroupStart() != ncclSuccess) return fail(MK_ECOMM, "ncclGroupStart");
    for (int d = 0; d < ndev; ++d) {
        uint8_t* lvl = (uint8_t*)g_ctx[d]->mout.p;
        if (ncclAllGather(lvl + block * d, lvl, block, ncclUint8, (*comms)[d], stream_of(d)) != ncclSuccess) {
            ncclGroupEnd();
            return fail(MK_ECOMM, "ncclAllGather on device %d", d);
        }
    }
    if (ncclGroupEnd() != ncclSuccess) return fail(MK_ECOMM, "ncclGroupEnd");
    TRY(bind_dev(0));
    DevCtx* c0 = ctx();
    if (k) return dev_finish_nodes(c0->mout.p, count, n, d_out32, c0->maux.p, c0->maux.cap, stream_of(0));
    return dev_finish(c0->mout.p, ne, n, d_out32, stream_of(0));
}

}  // namespace

// ---- deposit trie handle -----------------------------------------------------------------
struct mk_trie {
    std::mutex mu;
    int dev = 0;
    uint32_t depth = 32;
    uint64_t cap = 0, count = 0;
    DevBuf levels, root, in, offs, branch;
};

// =============================================================================
extern "C" {

#define MK_STR2(x) #x
#define MK_STR(x) MK_STR2(x)
// MK_BUILD_FLAGS: the -D knobs of a variant build (Makefile `variant`), "default"
// for the shipped library; __graft_entry__.build() refuses any other value
#ifndef MK_BUILD_FLAGS
#define MK_BUILD_FLAGS "default"
#endif
const char* mk_version(void) {
    return "prysm_merkle 0.4 (gfx950; leaf_lock=" MK_STR(MK_LEAF_LOCK) " lock_bars=" MK_STR(MK_LOCK_BARS)
           " elem_lock=" MK_STR(MK_ELEM_LOCK) " trie_lock=" MK_STR(MK_TRIE_LOCK) " flags=" MK_BUILD_FLAGS ")";
}

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

const char* mk_last_error(void) { return mk::last_error(); }

int mk_device_count(void) { return probe_devices(); }

int mk_init(int device) {
    Scope S(nullptr);
    return S.done(bind_dev(device < 0 ? 0 : device));
}

// ---- hashing ------------------------------------------------------------------
int mk_dev_hash_batch(mk_call* call, const void* d_in, uint64_t n, uint32_t msg_len, void* d_out, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    return S.done(rc ? rc : dev_hash_batch(d_in, n, msg_len, d_out, (hipStream_t)stream));
}

int mk_dev_hash_batch_var(mk_call* call, const void* d_in, const uint64_t* d_offs, uint64_t n, void* d_out,
                          void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    return S.done(rc ? rc : dev_hash_var(d_in, d_offs, n, d_out, (hipStream_t)stream));
}

static int host_hash_batch(const uint8_t* in, uint64_t n, uint32_t msg_len, uint8_t* out) {
    if (n && !in && msg_len) return fail(MK_EINVAL, "null input");
    if (n && !out) return fail(MK_EINVAL, "null output");
    TRY(bind_call());
    if (n == 0) return MK_OK;
    DevCtx* c = ctx();
    std::lock_guard<std::mutex> lk(c->mu);
    const size_t inb = n * (size_t)msg_len;
    TRY(grow(c->in, inb));
    TRY(grow(c->out, 32 * n));
    hipStream_t st = c->stream;
    if (inb) HIPCHK(hipMemcpyAsync(c->in.p, in, inb, hipMemcpyHostToDevice, st));
    TRY(dev_hash_batch(c->in.p, n, msg_len, c->out.p, st));
    HIPCHK(hipMemcpyAsync(out, c->out.p, 32 * n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

static int host_hash_var(const uint8_t* in, const uint64_t* offs, uint64_t n, uint8_t* out) {
    if (n && (!offs || !out)) return fail(MK_EINVAL, "null pointer");
    TRY(bind_call());
    if (n == 0) return MK_OK;
    DevCtx* c = ctx();
    std::lock_guard<std::mutex> lk(c->mu);
    const size_t inb = offs[n] - offs[0];
    TRY(grow(c->in, inb));
    TRY(grow(c->aux, 8 * (n + 1)));
    TRY(grow(c->out, 32 * n));
    hipStream_t st = c->stream;
    std::vector<uint64_t> rel(offs, offs + n + 1);
    for (auto& o : rel) o -= offs[0];
    if (inb) HIPCHK(hipMemcpyAsync(c->in.p, in + offs[0], inb, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(c->aux.p, rel.data(), 8 * (n + 1), hipMemcpyHostToDevice, st));
    TRY(dev_hash_var(c->in.p, (const uint64_t*)c->aux.p, n, c->out.p, st));
    HIPCHK(hipMemcpyAsync(out, c->out.p, 32 * n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

int mk_hash_batch(mk_call* call, const uint8_t* in, uint64_t n, uint32_t msg_len, uint8_t* out) {
    Scope S(call);
    return S.done(host_hash_batch(in, n, msg_len, out));
}

int mk_hash_batch_var(mk_call* call, const uint8_t* in, const uint64_t* offs, uint64_t n, uint8_t* out) {
    Scope S(call);
    return S.done(host_hash_var(in, offs, n, out));
}

int mk_hash(mk_call* call, const uint8_t* data, uint64_t len, uint8_t out[32]) {
    Scope S(call);
    if (len && !data) return S.done(fail(MK_EINVAL, "null input"));
    if (len > UINT32_MAX) {
        uint64_t offs[2] = {0, len};
        return S.done(host_hash_var(data, offs, 1, out));
    }
    static const uint8_t empty = 0;
    return S.done(host_hash_batch(len ? data : &empty, 1, (uint32_t)len, out));
}

// ---- merkleHash ---------------------------------------------------------------
uint64_t mk_ssz_merkle_workspace_bytes(uint64_t n, uint32_t item_len) {
    Scope S(nullptr, false);
    Plan p;
    if (mk::make_plan(n, item_len, false, 0, false, true, p) != MK_OK) return 0;
    return std::max<uint64_t>(p.small ? 256 : mk::plan_ws_bytes(p), list_tree_ws(n, item_len));
}

int mk_dev_ssz_merkle_hash(mk_call* call, const void* d_items, uint64_t n, uint32_t item_len, void* d_out32,
                           void* d_ws, uint64_t ws_bytes, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    return S.done(rc ? rc : dev_merkle_hash(d_items, n, item_len, d_out32, d_ws, ws_bytes, (hipStream_t)stream));
}

int mk_ssz_merkle_hash(mk_call* call, const uint8_t* items, uint64_t n, uint32_t item_len, uint8_t out[32]) {
    Scope S(call);
    return S.done(host_merkle_hash(items, n, item_len, out));
}

uint64_t mk_ssz_tree_hash_bytes_list_workspace_bytes(uint64_t n, uint32_t elem_len) {
    ElemPlan e;
    if (make_elem_plan(n, elem_len, true, e) != MK_OK) return 0;
    return e.ws_bytes;
}

int mk_dev_ssz_tree_hash_bytes_list(mk_call* call, const void* d_elems, uint64_t n, uint32_t elem_len,
                                    void* d_out32, void* d_ws, uint64_t ws_bytes, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    return S.done(rc ? rc : dev_tree_hash_elems(d_elems, n, elem_len, d_out32, d_ws, ws_bytes, (hipStream_t)stream));
}

int mk_ssz_tree_hash_bytes_list(mk_call* call, const uint8_t* elems, uint64_t n, uint32_t elem_len, uint8_t out[32]) {
    Scope S(call);
    return S.done(host_tree_hash_elems(elems, n, elem_len, out));
}

uint64_t mk_ssz_merkle_many_workspace_bytes(const uint64_t* n, const uint32_t* item_len, uint32_t nlists) {
    Scope S(nullptr, false);
    mk::ManyPlan mp;
    std::vector<uint64_t> offs(nlists, 0);  // the layout does not depend on the offsets
    if (mk::make_many_plan(offs.data(), n, item_len, nlists, UINT64_MAX, true, mp) != MK_OK) return 0;
    return mp.ws_bytes;
}

int mk_dev_ssz_merkle_many(mk_call* call, const void* d_items, const uint64_t* offs, const uint64_t* n,
                           const uint32_t* item_len, uint32_t nlists, void* d_roots, void* d_ws, uint64_t ws_bytes,
                           void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    if (nlists && !offs) return S.done(fail(MK_EINVAL, "null offsets"));
    mk::ManyPlan mp;
    rc = mk::make_many_plan(offs, n, item_len, nlists, UINT64_MAX, ((uintptr_t)d_items % 16) == 0, mp);
    if (rc) return S.done(rc);
    return S.done(dev_merkle_many(d_items, mp, nlists, d_roots, d_ws, ws_bytes, (hipStream_t)stream));
}

static int host_merkle_many(const uint8_t* items, const uint64_t* offs, const uint64_t* n, const uint32_t* item_len,
                            uint32_t nlists, uint8_t* roots) {
    if (nlists == 0) return MK_OK;
    if (!offs || !n || !item_len || !roots) return fail(MK_EINVAL, "null pointer");
    uint64_t lo = UINT64_MAX, hi = 0;
    for (uint32_t i = 0; i < nlists; ++i) {
        const uint64_t b = n[i] * (uint64_t)item_len[i];
        if (b) {
            lo = std::min(lo, offs[i]);
            hi = std::max(hi, offs[i] + b);
        }
    }
    if (lo == UINT64_MAX) lo = hi = 0;
    if (hi > lo && !items) return fail(MK_EINVAL, "null items");
    // upload [lo, hi) of the caller's buffer; offsets shift by lo (rounded down to 16 keeps alignment)
    lo &= ~15ull;
    std::vector<uint64_t> rel(offs, offs + nlists);
    for (uint32_t i = 0; i < nlists; ++i) rel[i] = n[i] * (uint64_t)item_len[i] ? offs[i] - lo : 0;
    mk::ManyPlan mp;
    // the device copy starts 256-B aligned: a list is 16-B aligned there iff its offset is
    TRY(mk::make_many_plan(rel.data(), n, item_len, nlists, hi - lo, true, mp));
    TRY(bind_call());
    DevCtx* c = ctx();
    std::lock_guard<std::mutex> lk(c->mu);
    hipStream_t st = c->stream;
    TRY(grow(c->in, hi - lo));
    TRY(grow(c->ws, mp.ws_bytes));
    TRY(grow(c->out, 32 * (size_t)nlists));
    if (hi > lo) HIPCHK(hipMemcpyAsync(c->in.p, items + lo, hi - lo, hipMemcpyHostToDevice, st));
    TRY(dev_merkle_many(c->in.p, mp, nlists, c->out.p, c->ws.p, c->ws.cap, st));
    HIPCHK(hipMemcpyAsync(roots, c->out.p, 32 * (size_t)nlists, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

int mk_ssz_merkle_many(mk_call* call, const uint8_t* items, const uint64_t* offs, const uint64_t* n,
                       const uint32_t* item_len, uint32_t nlists, uint8_t* roots) {
    Scope S(call);
    return S.done(host_merkle_many(items, offs, n, item_len, nlists, roots));
}

// ---- sharding -------------------------------------------------------------------
int mk_ssz_merkle_shard_plan(mk_call* call, uint64_t n, uint32_t item_len, uint32_t nshards, uint32_t* height,
                             uint32_t* nonempty, uint64_t* item_begin) {
    Scope S(call, false);
    if (!height || !nonempty || !item_begin) return S.done(fail(MK_EINVAL, "null pointer"));
    return S.done(mk::shard_plan(n, item_len, nshards, height, nonempty, item_begin));
}

int mk_dev_ssz_merkle_subtree(mk_call* call, const void* d_shard_items, uint64_t shard_n, uint32_t item_len,
                              uint32_t height, int pad_at_one, void* d_out32, void* d_ws, uint64_t ws_bytes,
                              void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    if (!d_out32 || (shard_n && !d_shard_items)) return S.done(fail(MK_EINVAL, "null pointer"));
    Plan p;
    rc = mk::make_plan(shard_n, item_len, true, height, pad_at_one != 0, ((uintptr_t)d_shard_items % 16) == 0, p);
    if (rc) return S.done(rc);
    return S.done(launch_plan(p, (const uint8_t*)d_shard_items, (uint8_t*)d_out32, (uint8_t*)d_ws, ws_bytes,
                              (hipStream_t)stream));
}

int mk_dev_ssz_merkle_subtree_frontier(mk_call* call, const void* d_shard_items, uint64_t shard_n,
                                       uint32_t item_len, uint32_t height, uint32_t frontier_log2, int pad_at_one,
                                       void* d_out, uint64_t* nodes_out, void* d_ws, uint64_t ws_bytes,
                                       void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    if (!d_out || (shard_n && !d_shard_items)) return S.done(fail(MK_EINVAL, "null pointer"));
    Plan p;
    rc = mk::make_plan(shard_n, item_len, true, height, pad_at_one != 0, ((uintptr_t)d_shard_items % 16) == 0, p,
                       false, frontier_log2);
    if (rc) return S.done(rc);
    if (nodes_out) *nodes_out = p.out_nodes;
    return S.done(launch_plan(p, (const uint8_t*)d_shard_items, (uint8_t*)d_out, (uint8_t*)d_ws, ws_bytes,
                              (hipStream_t)stream));
}

uint64_t mk_ssz_merkle_node_frontier_workspace_bytes(uint64_t count, uint32_t height, uint32_t frontier_log2) {
    Scope S(nullptr, false);
    Plan p;
    if (mk::make_plan(count, 32, true, height, true, true, p, true, frontier_log2) != MK_OK) return 0;
    return std::max<uint64_t>(256, mk::plan_ws_bytes(p));
}

int mk_dev_ssz_merkle_node_frontier(mk_call* call, const void* d_nodes, uint64_t count, uint32_t height,
                                    uint32_t frontier_log2, int pad_at_one, void* d_out, uint64_t* nodes_out,
                                    void* d_ws, uint64_t ws_bytes, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    if (!d_out || !d_nodes || count == 0) return S.done(fail(MK_EINVAL, "null pointer or empty level"));
    Plan p;
    rc = mk::make_plan(count, 32, true, height, pad_at_one != 0, ((uintptr_t)d_nodes % 16) == 0, p, true,
                       frontier_log2);
    if (rc) return S.done(rc);
    if (nodes_out) *nodes_out = frontier_log2 ? p.out_nodes : 1;
    return S.done(launch_plan(p, (const uint8_t*)d_nodes, (uint8_t*)d_out, (uint8_t*)d_ws, ws_bytes,
                              (hipStream_t)stream));
}

uint64_t mk_ssz_merkle_finish_workspace_bytes(uint64_t count) {
    Scope S(nullptr, false);
    return finish_ws_bytes(count);
}

int mk_dev_ssz_merkle_finish_nodes(mk_call* call, const void* d_nodes, uint64_t count, uint64_t n_total,
                                   void* d_out32, void* d_ws, uint64_t ws_bytes, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    return S.done(rc ? rc : dev_finish_nodes(d_nodes, count, n_total, d_out32, d_ws, ws_bytes, (hipStream_t)stream));
}

// ---- fused list tops (k_merkle_top_fused) -------------------------------------------
// Workgroups of NT = 1024 threads (one per CU).  Per list: nodes per
// workgroup = the power of two that gives the list about 256 / nlists
// workgroups, so the throughput-bound lower levels spread over the chip (two
// lists side by side in one grid), 64..1024; a list of <= 1024 nodes runs in
// one workgroup (no hand-off).  C3 (125,000 + 31,250 nodes): 123 + 123
// workgroups.  (512-thread workgroups, two per CU, 245 + 245 of them:
// C3 one state 0.5748 / 0.5819 against 0.5712 / 0.5719 ms, rejected.)
struct TopPlan {
    static constexpr uint32_t nt = 1024;
    uint32_t span_log2[2] = {0, 0}, nwg[2] = {0, 0};
    uint64_t ws = 0;
};
static int top_plan(const uint64_t* c, uint32_t nl, TopPlan& p) {
    p = TopPlan();
    for (uint32_t l = 0; l < nl; ++l) {
        if (c[l] == 0) return fail(MK_EINVAL, "empty level");
        if (c[l] > (1ull << 20)) return fail(MK_EINVAL, "fused top: %llu nodes > 2^20", (unsigned long long)c[l]);
    }
    const uint32_t lmax = 10;
    const uint64_t target = 256 / nl;
    for (uint32_t l = 0; l < nl; ++l) {
        uint32_t sl = lmax;
        if (c[l] > p.nt) {
            sl = 6;
            while (sl < lmax && (c[l] >> sl) >= target) ++sl;
        }
        p.span_log2[l] = sl;
        p.nwg[l] = (uint32_t)ceil_div(c[l], 1ull << sl);
        p.ws += 32 * (uint64_t)p.nwg[l];
    }
    p.ws = (p.ws + 255) & ~255ull;
    return MK_OK;
}

static int launch_top_fused(const TopPlan& p, uint32_t nl, const void* const* nodes, const uint64_t* c,
                            const uint64_t* nit, void* d_out, uint32_t epoch, void* d_ws, hipStream_t st);

uint64_t mk_ssz_merkle_top_fused_workspace_bytes(uint64_t count0, uint64_t count1) {
    const uint64_t c[2] = {count0, count1};
    TopPlan p;
    return top_plan(c, count1 ? 2 : 1, p) == MK_OK ? p.ws : 0;
}

int mk_dev_ssz_merkle_top_fused(mk_call* call, const void* d_nodes0, uint64_t count0, uint64_t n0,
                                const void* d_nodes1, uint64_t count1, uint64_t n1, void* d_out, uint32_t epoch,
                                void* d_ws, uint64_t ws_bytes, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    const uint32_t nl = count1 ? 2 : 1;
    const uint64_t c[2] = {count0, count1};
    const void* nodes[2] = {d_nodes0, d_nodes1};
    const uint64_t nit[2] = {n0, n1};
    TopPlan p;
    rc = top_plan(c, nl, p);
    if (rc) return S.done(rc);
    if (!d_out || !d_ws || !d_nodes0 || (nl == 2 && !d_nodes1)) return S.done(fail(MK_EINVAL, "null pointer"));
    if (ws_bytes < p.ws) return S.done(fail(MK_ENOMEM, "workspace too small: %llu < %llu", (unsigned long long)ws_bytes,
                                            (unsigned long long)p.ws));
    if ((uintptr_t)d_nodes0 % 8 || (uintptr_t)d_nodes1 % 8 || (uintptr_t)d_ws % 16)
        return S.done(fail(MK_EINVAL, "nodes not 8-B aligned or workspace not 16-B aligned"));
    if (nl == 2) {
        if (epoch == 0 || epoch >= (1u << 30))
            return S.done(fail(MK_EINVAL, "pair epoch %u out of range (1..2^30-1)", epoch));
        if ((uintptr_t)d_out % 16) return S.done(fail(MK_EINVAL, "pair block not 16-B aligned"));
    }
    return S.done(launch_top_fused(p, nl, nodes, c, nit, d_out, epoch, d_ws, (hipStream_t)stream));
}

static int launch_top_fused(const TopPlan& p, uint32_t nl, const void* const* nodes, const uint64_t* c,
                            const uint64_t* nit, void* d_out, uint32_t epoch, void* d_ws, hipStream_t st) {
    if (inject_ehip()) return fail(MK_EHIP, "hipLaunchKernelGGL: injected failure (MK_INJECT_EHIP)");
    mk::MerkleTopArgs a{};
    a.nlists = nl;
    a.pair = nl == 2 ? (uint32_t*)d_out : nullptr;
    a.pair_slot = nl == 2 ? next_arrive_slot() : 0;
    (void)epoch;  // both finishers are in this launch: an arrival counter, not the epoch word
    uint32_t wg = 0;
    uint32_t* sub = (uint32_t*)d_ws;
    for (uint32_t l = 0; l < nl; ++l) {
        mk::MerkleTopList& t = a.l[l];
        t.nodes = (const uint4*)nodes[l];
        t.c = c[l];
        t.n_items = nit[l];
        t.sub = sub;
        t.out = nl == 2 ? (uint32_t*)d_out + 8 * l : (uint32_t*)d_out;
        t.wg0 = wg;
        t.nwg = p.nwg[l];
        t.span_log2 = p.span_log2[l];
        t.slot = next_arrive_slots(top_arrive_slots(t.nwg));
        wg += t.nwg;
        sub += 8 * t.nwg;
    }
    hipLaunchKernelGGL(mk::k_merkle_top_fused<1024>, dim3(wg), dim3(1024), 0, st, a);
    HIPCHK(hipGetLastError());
    return MK_OK;
}

// k_merkle_top_fused over one list's complete level of c nodes in spans of
// 2^span_log2 nodes per workgroup, to the root with the length mix-in
// (dev_list_tree, declared in the anonymous namespace above)
namespace {
static int launch_top_span(const void* d_nodes, uint64_t c, uint64_t n_items, uint32_t span_log2, void* d_out32,
                           uint8_t* d_ws, hipStream_t st) {
    TopPlan p;
    p.span_log2[0] = span_log2;
    p.nwg[0] = (uint32_t)ceil_div(c, 1ull << span_log2);
    p.ws = align256(32 * (uint64_t)p.nwg[0]);
    const void* nodes[1] = {d_nodes};
    const uint64_t cc[1] = {c}, nit[1] = {n_items};
    return launch_top_fused(p, 1, nodes, cc, nit, d_out32, 0, d_ws, st);
}
}  // namespace

int mk_dev_ssz_merkle_finish_nodes_pair(mk_call* call, const void* d_nodes, uint64_t count, uint64_t n_total,
                                        void* d_pair_block, uint32_t slot, uint32_t epoch, void* d_ws,
                                        uint64_t ws_bytes, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    if (!d_pair_block) return S.done(fail(MK_EINVAL, "null pointer"));
    if (slot > 1) return S.done(fail(MK_EINVAL, "pair slot %u out of range (0..1)", slot));
    if (epoch == 0 || epoch >= (1u << 30)) return S.done(fail(MK_EINVAL, "pair epoch %u out of range (1..2^30-1)", epoch));
    if ((uintptr_t)d_pair_block % 16) return S.done(fail(MK_EINVAL, "pair block not 16-B aligned"));
    return S.done(dev_finish_nodes(d_nodes, count, n_total, nullptr, d_ws, ws_bytes, (hipStream_t)stream,
                                   d_pair_block, slot, epoch));
}

int mk_dev_ssz_merkle_finish(mk_call* call, const void* d_roots, uint64_t nroots, uint64_t n_total, void* d_out32,
                             void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    return S.done(rc ? rc : dev_finish(d_roots, nroots, n_total, d_out32, (hipStream_t)stream));
}

int mk_ssz_merkle_hash_multi(mk_call* call, const uint8_t* items, uint64_t n, uint32_t item_len, int nshards,
                             const int* devs, uint8_t out[32]) {
    Scope S(call);
    return S.done(host_merkle_multi(items, n, item_len, nshards, devs, out));
}

int mk_dev_ssz_merkle_hash_multi(mk_call* call, const void* const* d_shards, uint64_t n, uint32_t item_len,
                                 int ndev, void* d_out32, void* const* streams) {
    Scope S(call);
    return S.done(dev_merkle_multi(d_shards, n, item_len, ndev, d_out32, streams));
}

// ---- struct hashing ---------------------------------------------------------------
uint64_t mk_ssz_struct_msg_len(const mk_field* fields, uint32_t nfields) {
    Scope S(nullptr, false);
    mk::StructSpec sp;
    if (make_spec(fields, nfields, 0, sp) != MK_OK) return 0;
    return sp.msg_len;
}

uint64_t mk_ssz_struct_list_workspace_bytes(uint64_t n, const mk_field* fields, uint32_t nfields) {
    Scope S(nullptr, false);
    mk::StructSpec sp;
    if (make_spec(fields, nfields, 0, sp) != MK_OK) return 0;
    return struct_list_ws(n, sp);
}

int mk_dev_ssz_struct_list_root(mk_call* call, const void* d_records, uint64_t n, uint32_t record_len,
                                const mk_field* fields, uint32_t nfields, void* d_out32, void* d_ws,
                                uint64_t ws_bytes, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    mk::StructSpec sp;
    rc = make_spec(fields, nfields, record_len, sp);
    if (rc) return S.done(rc);
    if (ws_bytes < struct_list_ws(n, sp)) return S.done(fail(MK_ENOMEM, "workspace too small"));
    if (n && !d_records) return S.done(fail(MK_EINVAL, "null pointer"));
    uint8_t* ws = (uint8_t*)d_ws;
    uint8_t* msg = ws;
    uint8_t* roots = ws + align256(n * sp.msg_len);
    uint8_t* mws = roots + align256(32 * n);
    hipStream_t st = (hipStream_t)stream;
    if (struct_win_ok(d_records, n, sp))  // the windows go where the two-launch path keeps its messages
        return S.done(dev_struct_list_root_win(d_records, n, roots, msg, d_out32, mws,
                                               ws_bytes - (uint64_t)(mws - ws), st));
    if (struct_list_fused_ok(d_records, n, sp) && ws_bytes - (uint64_t)(mws - ws) >= list_tree_ws(n, 32))
        return S.done(launch_struct_list_fused(d_records, n, sp, roots, mws, d_out32, st));
    rc = launch_struct_roots(d_records, n, sp, msg, roots, st);
    if (rc) return S.done(rc);
    return S.done(dev_merkle_hash(roots, n, 32, d_out32, mws, ws_bytes - (uint64_t)(mws - ws), st));
}

int mk_ssz_struct_list_level1_ok(const void* d_records, uint64_t n, uint32_t record_len, const mk_field* fields,
                                 uint32_t nfields) {
    Scope S(nullptr, false);
    mk::StructSpec sp;
    if (make_spec(fields, nfields, record_len, sp) != MK_OK) return 0;
    return struct_win_ok(d_records, n, sp) ? 1 : 0;
}

int mk_dev_ssz_struct_list_level1(mk_call* call, const void* d_records, uint64_t n, uint32_t record_len,
                                  const mk_field* fields, uint32_t nfields, void* d_roots, void* d_nodes,
                                  const void* d_values, uint64_t nvalues, uint32_t value_len, void* d_value_nodes,
                                  void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    mk::StructSpec sp;
    rc = make_spec(fields, nfields, record_len, sp);
    if (rc) return S.done(rc);
    if (!d_records || !d_roots || !d_nodes) return S.done(fail(MK_EINVAL, "null pointer"));
    if (!struct_win_ok(d_records, n, sp))
        return S.done(fail(MK_EINVAL, "level-1 front needs >= 2^18 ValidatorRecords at a 16-B aligned address"));
    if (nvalues) {
        if (!d_values || !d_value_nodes) return S.done(fail(MK_EINVAL, "null pointer"));
        if (value_len % 8 || value_len == 0 || 128 % value_len || ((uintptr_t)d_values % 16))
            return S.done(fail(MK_EINVAL, "second list: items of 8, 16, 32, 64 or 128 B at a 16-B aligned address"));
        if (nvalues * value_len <= 128)
            return S.done(fail(MK_EINVAL, "second list of one chunk has no level-1 window"));
    }
    return S.done(dev_struct_level1(d_records, n, d_roots, d_nodes, (hipStream_t)stream, d_values,
                                    nvalues * (uint64_t)value_len, d_value_nodes));
}

// ---- a stream of states (registry.StatePipeline) ----------------------------
// Workgroup b of the pipelined launch writes the level-1 nodes [sub b, sub b +
// sub) of each tree -- sub = 512 for the registry (4 groups x 1024 records /
// 8), 128 for the second list (the balances) -- a complete subtree whose
// levels 2..K the NEXT launch builds in its slots (k_struct_lock<true>): K =
// 10 for the registry (1 node per subtree), 4 for the second list (16).  A
// levels buffer holds level k (2..K) of subtree b at node offset
// level_off(k) + (sub >> (k - 1)) b, the levels back to back, level K last
// with room after the nfull complete subtrees' nodes for the ragged last
// subtree's (its level-1 nodes reduced on the finisher's stream).
struct PipeTree {
    uint64_t sub;   // level-1 nodes per subtree
    uint32_t K;     // the highest level the slots build
    uint64_t c1;    // level-1 nodes of the whole tree
    uint64_t nfull() const { return c1 / sub; }
    uint64_t per_top() const { return sub >> (K - 1); }
    uint64_t level_off(uint32_t k) const {  // nodes before level k
        uint64_t off = 0;
        for (uint32_t j = 2; j < k; ++j) off += (sub >> (j - 1)) * nfull();
        return off;
    }
    uint64_t levels_bytes() const { return 32 * (level_off(K + 1) + per_top()); }
};
PipeTree pipe_reg(uint64_t n) { return {512, 10, ceil_div(n, 8)}; }
PipeTree pipe_val(uint64_t nvalues, uint32_t value_len) { return {128, 4, ceil_div(nvalues * value_len, 256)}; }
bool struct_pipe_ok(const void* d_rec, uint64_t n, const mk::StructSpec& sp, hipStream_t st) {
    return struct_win_ok(d_rec, n, sp) && struct_gpw(n, st) == 4 && pipe_reg(n).nfull() >= 1;
}

int mk_ssz_struct_pipe_ok(const void* d_records, uint64_t n, uint32_t record_len, const mk_field* fields,
                          uint32_t nfields, void* stream) {
    Scope S(nullptr);
    mk::StructSpec sp;
    if (make_spec(fields, nfields, record_len, sp) != MK_OK || bind_stream((hipStream_t)stream)) return S.done(0);
    return S.done(struct_pipe_ok(d_records, n, sp, (hipStream_t)stream) ? 1 : 0);
}

uint64_t mk_ssz_struct_pipe_levels_bytes(uint64_t n, uint64_t nvalues, uint32_t value_len, uint32_t which) {
    if (which > 1 || (which == 1 && (value_len == 0 || nvalues == 0))) return 0;
    return which ? pipe_val(nvalues, value_len).levels_bytes() : pipe_reg(n).levels_bytes();
}

static uint64_t pipe_top_ws(const PipeTree& t) {
    mk::WideWaves wide;  // the plans mk_dev_ssz_struct_pipe_top makes
    const uint64_t rag = t.c1 - t.sub * t.nfull();
    uint64_t ws = std::max<uint64_t>(256, finish_ws_bytes(t.nfull() * t.per_top() + t.per_top()));
    Plan p;
    if (rag && mk::make_plan(rag, 32, true, 63 - __builtin_clzll(t.sub), true, true, p, true,
                             63 - __builtin_clzll(t.per_top())) == MK_OK)
        ws = std::max<uint64_t>(ws, mk::plan_ws_bytes(p));
    return ws;
}

uint64_t mk_ssz_struct_pipe_top_workspace_bytes(uint64_t n, uint64_t nvalues, uint32_t value_len, uint32_t which) {
    Scope S(nullptr, false);
    if (which > 1 || (which == 1 && (value_len == 0 || nvalues == 0))) return 0;
    return pipe_top_ws(which ? pipe_val(nvalues, value_len) : pipe_reg(n));
}

int mk_dev_ssz_struct_list_level1_pipe(mk_call* call, const void* d_records, uint64_t n, uint32_t record_len,
                                       const mk_field* fields, uint32_t nfields, void* d_roots, void* d_nodes,
                                       const void* d_values, uint64_t nvalues, uint32_t value_len,
                                       void* d_value_nodes, const void* d_prev_nodes, void* d_prev_levels,
                                       const void* d_prev_value_nodes, void* d_prev_value_levels, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    mk::StructSpec sp;
    rc = make_spec(fields, nfields, record_len, sp);
    if (rc) return S.done(rc);
    if (!d_records || !d_roots || !d_nodes || (d_prev_nodes && !d_prev_levels) ||
        (d_prev_value_nodes && !d_prev_value_levels))
        return S.done(fail(MK_EINVAL, "null pointer"));
    if (!struct_pipe_ok(d_records, n, sp, (hipStream_t)stream))
        return S.done(fail(MK_EINVAL, "pipelined struct launch needs ValidatorRecords at a 16-B aligned address, "
                                      "4 groups of 1024 per workgroup (n = %llu)", (unsigned long long)n));
    if (d_prev_nodes && d_prev_nodes == d_nodes)
        return S.done(fail(MK_EINVAL, "the previous state's nodes alias this state's"));
    const uint64_t grid = ceil_div(ceil_div(n, mk::kLockThreads), 4);
    if (nvalues) {
        if (!d_values || !d_value_nodes) return S.done(fail(MK_EINVAL, "null pointer"));
        if (value_len % 8 || value_len == 0 || 128 % value_len || ((uintptr_t)d_values % 16))
            return S.done(fail(MK_EINVAL, "second list: items of 8, 16, 32, 64 or 128 B at a 16-B aligned address"));
        if (nvalues * value_len <= 128)
            return S.done(fail(MK_EINVAL, "second list of one chunk has no level-1 window"));
        if (pipe_val(nvalues, value_len).c1 > 128 * grid)
            return S.done(fail(MK_EINVAL, "second list longer than 128 windows per workgroup"));
        if (d_prev_value_nodes && d_prev_value_nodes == d_value_nodes)
            return S.done(fail(MK_EINVAL, "the previous state's second-list nodes alias this state's"));
    } else if (d_prev_value_nodes) {
        return S.done(fail(MK_EINVAL, "previous second list without this state's"));
    }
    const PipeTree reg = pipe_reg(n), val = pipe_val(nvalues, value_len);
    mk::StructPrev prev{};
    prev.nfull = (uint32_t)reg.nfull();
    prev.live = d_prev_nodes ? 1u : 0u;
    prev.l1 = (const uint4*)d_prev_nodes;
    for (uint32_t k = 2; k <= 10; ++k)
        prev.lv[k - 2] = d_prev_levels ? (uint4*)d_prev_levels + 2 * reg.level_off(k) : nullptr;
    // the second list's slots (waves 13-15) only with a previous second list
    prev.nvfull = d_prev_value_nodes ? (uint32_t)val.nfull() : 0u;
    prev.v1 = (const uint4*)d_prev_value_nodes;
    for (uint32_t k = 2; k <= 4; ++k)
        prev.vlv[k - 2] = d_prev_value_levels ? (uint4*)d_prev_value_levels + 2 * val.level_off(k) : nullptr;
    return S.done(dev_struct_level1(d_records, n, d_roots, d_nodes, (hipStream_t)stream, d_values,
                                    nvalues * (uint64_t)value_len, d_value_nodes, &prev));
}

int mk_dev_ssz_struct_pipe_top(mk_call* call, const void* d_nodes, uint64_t n, uint64_t nvalues,
                               uint32_t value_len, uint32_t which, void* d_levels, void* d_pair_block, uint32_t slot,
                               uint32_t epoch, void* d_ws, uint64_t ws_bytes, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    if (!d_nodes || !d_levels || !d_pair_block) return S.done(fail(MK_EINVAL, "null pointer"));
    if (which > 1 || (which == 1 && (value_len == 0 || nvalues == 0)))
        return S.done(fail(MK_EINVAL, "tree %u: 0 = the registry, 1 = a non-empty second list", which));
    if (slot > 1) return S.done(fail(MK_EINVAL, "pair slot %u out of range (0..1)", slot));
    if (epoch == 0 || epoch >= (1u << 30)) return S.done(fail(MK_EINVAL, "pair epoch %u out of range (1..2^30-1)", epoch));
    if ((uintptr_t)d_pair_block % 16) return S.done(fail(MK_EINVAL, "pair block not 16-B aligned"));
    const PipeTree t = which ? pipe_val(nvalues, value_len) : pipe_reg(n);
    const uint64_t nfull = t.nfull(), rag = t.c1 - t.sub * nfull;
    if (nfull == 0) return S.done(fail(MK_EINVAL, "no complete subtree"));
    mk::WideWaves wide;  // beside the next pipelined launch: whole-CU workgroups only
    if (ws_bytes < pipe_top_ws(t)) return S.done(fail(MK_ENOMEM, "workspace too small"));
    uint8_t* top = (uint8_t*)d_levels + 32 * t.level_off(t.K);  // level K: per_top nodes per subtree
    uint64_t count = nfull * t.per_top();
    if (rag) {  // the ragged last subtree from level 1 to level K, the odd rule at every level (pad_at_one)
        Plan p;
        const uint32_t h = 63 - __builtin_clzll(t.sub), f = 63 - __builtin_clzll(t.per_top());
        rc = mk::make_plan(rag, 32, true, h, true, ((uintptr_t)d_nodes % 16) == 0, p, true, f);
        if (rc) return S.done(rc);
        rc = launch_plan(p, (const uint8_t*)d_nodes + 32 * t.sub * nfull, top + 32 * count, (uint8_t*)d_ws,
                         ws_bytes, (hipStream_t)stream);
        if (rc) return S.done(rc);
        count += f ? p.out_nodes : 1;
    }
    return S.done(dev_finish_nodes(top, count, which ? nvalues : n, nullptr, d_ws, ws_bytes, (hipStream_t)stream,
                                   d_pair_block, slot, epoch));
}

int mk_dev_ssz_struct_roots(mk_call* call, const void* d_records, uint64_t n, uint32_t record_len,
                            const mk_field* fields, uint32_t nfields, void* d_roots, void* d_ws, uint64_t ws_bytes,
                            void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    mk::StructSpec sp;
    rc = make_spec(fields, nfields, record_len, sp);
    if (rc) return S.done(rc);
    if (n && (!d_records || !d_roots)) return S.done(fail(MK_EINVAL, "null pointer"));
    if (ws_bytes < n * (uint64_t)sp.msg_len) return S.done(fail(MK_ENOMEM, "workspace too small"));
    return S.done(launch_struct_roots(d_records, n, sp, d_ws, d_roots, (hipStream_t)stream));
}

static int host_struct_roots(const uint8_t* records, uint64_t n, uint32_t record_len, const mk_field* fields,
                             uint32_t nfields, uint8_t* roots) {
    mk::StructSpec sp;
    TRY(make_spec(fields, nfields, record_len, sp));
    if (n && (!records || !roots)) return fail(MK_EINVAL, "null pointer");
    TRY(bind_call());
    if (n == 0) return MK_OK;
    DevCtx* c = ctx();
    std::lock_guard<std::mutex> lk(c->mu);
    hipStream_t st = c->stream;
    TRY(grow(c->in, n * (size_t)record_len));
    TRY(grow(c->ws, align256(n * sp.msg_len)));
    TRY(grow(c->out, 32 * n));
    HIPCHK(hipMemcpyAsync(c->in.p, records, n * (size_t)record_len, hipMemcpyHostToDevice, st));
    TRY(launch_struct_roots(c->in.p, n, sp, c->ws.p, c->out.p, st));
    HIPCHK(hipMemcpyAsync(roots, c->out.p, 32 * n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

int mk_ssz_struct_roots(mk_call* call, const uint8_t* records, uint64_t n, uint32_t record_len,
                        const mk_field* fields, uint32_t nfields, uint8_t* roots) {
    Scope S(call);
    return S.done(host_struct_roots(records, n, record_len, fields, nfields, roots));
}

static int host_struct_list_root(const uint8_t* records, uint64_t n, uint32_t record_len, const mk_field* fields,
                                 uint32_t nfields, uint8_t* out) {
    mk::StructSpec sp;
    TRY(make_spec(fields, nfields, record_len, sp));
    if (!out || (n && !records)) return fail(MK_EINVAL, "null pointer");
    TRY(bind_call());
    DevCtx* c = ctx();
    std::lock_guard<std::mutex> lk(c->mu);
    hipStream_t st = c->stream;
    const uint64_t wsb = struct_list_ws(n, sp);
    TRY(grow(c->in, n * (size_t)record_len));
    TRY(grow(c->ws, wsb));
    TRY(grow(c->out, 32));
    // The records cross PCIe in chunks on the copy stream; the struct-roots
    // kernel of chunk i runs on the compute stream while chunk i+1 is in
    // flight, so only the last chunk's roots and the list merkleHash follow
    // the copy.
    uint8_t* ws = (uint8_t*)c->ws.p;
    uint8_t* msg = ws;
    uint8_t* roots = ws + align256(n * sp.msg_len);
    uint8_t* mws = roots + align256(32 * n);
    const uint8_t* din = (const uint8_t*)c->in.p;
    uint64_t chunk = std::max<uint64_t>(kH2dMinChunk, ceil_div(n, kH2dChunks));
    chunk = (chunk + 15) & ~15ull;  // chunk starts keep the records' 16-B alignment
    if (n <= chunk && struct_list_fused_ok(din, n, sp) && wsb - (uint64_t)(mws - ws) >= list_tree_ws(n, 32)) {
        // one piece: the records cross PCIe, then the whole list in one launch
        HIPCHK(hipMemcpyAsync((uint8_t*)c->in.p, records, n * (size_t)record_len, hipMemcpyHostToDevice, c->copy));
        HIPCHK(hipEventRecord(c->h2d, c->copy));
        HIPCHK(hipStreamWaitEvent(st, c->h2d, 0));
        TRY(launch_struct_list_fused(din, n, sp, roots, mws, c->out.p, st));
        HIPCHK(hipMemcpyAsync(out, c->out.p, 32, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        return MK_OK;
    }
    for (uint64_t off = 0; off < n; off += chunk) {
        const uint64_t cnt = std::min(chunk, n - off);
        HIPCHK(hipMemcpyAsync((uint8_t*)c->in.p + off * record_len, records + off * record_len,
                              cnt * (size_t)record_len, hipMemcpyHostToDevice, c->copy));
        HIPCHK(hipEventRecord(c->h2d, c->copy));
        HIPCHK(hipStreamWaitEvent(st, c->h2d, 0));
        TRY(launch_struct_roots(din + off * record_len, cnt, sp, msg + off * sp.msg_len, roots + 32 * off, st));
    }
    TRY(dev_merkle_hash(roots, n, 32, c->out.p, mws, wsb - (uint64_t)(mws - ws), st));
    HIPCHK(hipMemcpyAsync(out, c->out.p, 32, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

int mk_ssz_struct_list_root(mk_call* call, const uint8_t* records, uint64_t n, uint32_t record_len,
                            const mk_field* fields, uint32_t nfields, uint8_t out[32]) {
    Scope S(call);
    return S.done(host_struct_list_root(records, n, record_len, fields, nfields, out));
}

// ---- hashutil.MerkleRoot -----------------------------------------------------------
uint64_t mk_merkle_root_workspace_bytes(uint64_t n) {
    Scope S(nullptr, false);
    return merkle_root_ws(n);
}

int mk_dev_merkle_root(mk_call* call, const void* d_data, const uint64_t* d_offs, uint64_t n, uint32_t fixed_len,
                       void* d_heap, uint64_t heap_bytes, void* d_leaves32, void* d_out32, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    return S.done(rc ? rc
                     : dev_merkle_root(d_data, d_offs, n, fixed_len, d_heap, heap_bytes, d_leaves32, d_out32,
                                       (hipStream_t)stream));
}

static int host_merkle_root(const uint8_t* data, const uint64_t* offs, uint64_t n, uint8_t* leaves_out,
                            uint8_t* out) {
    if (!out || (n && !offs)) return fail(MK_EINVAL, "null pointer");
    if (n == 0) return fail(MK_EINVAL, "MerkleRoot of an empty list (reference: index out of range)");
    TRY(bind_call());
    DevCtx* c = ctx();
    std::lock_guard<std::mutex> lk(c->mu);
    hipStream_t st = c->stream;
    const size_t inb = offs[n] - offs[0];
    const int64_t ulen = uniform_len(offs, n);
    const uint64_t wsb = merkle_root_ws(n);
    TRY(grow(c->in, inb + 16));
    TRY(grow(c->aux, 8 * (n + 1)));
    TRY(grow(c->ws, wsb));
    TRY(grow(c->out, 32));
    if (inb) HIPCHK(hipMemcpyAsync(c->in.p, data + offs[0], inb, hipMemcpyHostToDevice, st));
    std::vector<uint64_t> rel;
    if (ulen < 0) {
        rel.assign(offs, offs + n + 1);
        for (auto& o : rel) o -= offs[0];
        HIPCHK(hipMemcpyAsync(c->aux.p, rel.data(), 8 * (n + 1), hipMemcpyHostToDevice, st));
    }
    TRY(dev_merkle_root(c->in.p, ulen < 0 ? (const uint64_t*)c->aux.p : nullptr, n, ulen < 0 ? 0 : (uint32_t)ulen,
                        c->ws.p, wsb, nullptr, c->out.p, st));
    HIPCHK(hipMemcpyAsync(out, c->out.p, 32, hipMemcpyDeviceToHost, st));
    if (leaves_out) HIPCHK(hipMemcpyAsync(leaves_out, (uint8_t*)c->ws.p + 32 * n, 32 * n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));  // `rel` and the caller's buffers are released after this
    return MK_OK;
}

int mk_merkle_root(mk_call* call, const uint8_t* data, const uint64_t* offs, uint64_t n, uint8_t* leaves_out,
                   uint8_t out[32]) {
    Scope S(call);
    return S.done(host_merkle_root(data, offs, n, leaves_out, out));
}

// ---- deposit trie -------------------------------------------------------------------
uint64_t mk_deposit_trie_levels_bytes(uint64_t capacity, uint32_t depth) {
    if (capacity == 0) return 0;
    return 32 * mk::trie_levels_nodes(capacity, depth);
}

int mk_dev_deposit_trie_append(mk_call* call, void* d_levels, uint64_t capacity, uint64_t count, const void* d_data,
                               const uint64_t* d_offs, uint64_t k, uint32_t fixed_len, uint32_t depth,
                               void* d_root32, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    return S.done(rc ? rc
                     : dev_trie_append(d_levels, capacity, count, d_data, d_offs, k, fixed_len, depth, d_root32,
                                       (hipStream_t)stream));
}

int mk_dev_deposit_trie_build(mk_call* call, void* d_levels, uint64_t capacity, const void* d_data,
                              const uint64_t* d_offs, uint64_t n, uint32_t fixed_len, uint32_t d_to, uint32_t depth,
                              void* d_root32, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    rc = check_trie(capacity, 0, n, depth);
    if (rc) return S.done(rc);
    if (d_to > depth) return S.done(fail(MK_EINVAL, "level %u out of range (0..%u)", d_to, depth));
    if (n == 0) return S.done(fail(MK_EINVAL, "empty trie"));
    if (!d_levels || (d_to == depth && !d_root32) || (!d_offs && !d_data && fixed_len))
        return S.done(fail(MK_EINVAL, "null pointer"));
    return S.done(trie_front(d_levels, capacity, d_data, d_offs, n, fixed_len, d_to, depth,
                             d_to == depth ? d_root32 : nullptr, (hipStream_t)stream));
}

int mk_deposit_trie_pipe_ok(const void* d_data, uint64_t n, uint32_t deposit_len, uint32_t depth, void* stream) {
    // the same check mk_dev_deposit_trie_build_pipe makes, on the caller's
    // stream (its CU mask bounds the persistent grid), on its device
    Scope S(nullptr);
    if (bind_stream((hipStream_t)stream)) return S.done(0);
    return S.done(trie_pipe_ok(d_data, n, deposit_len, depth, (hipStream_t)stream) ? 1 : 0);
}

int mk_dev_deposit_trie_build_pipe(mk_call* call, void* d_levels, void* d_prev_levels, uint64_t capacity,
                                   const void* d_data, uint64_t n, uint32_t deposit_len, uint32_t depth,
                                   void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    rc = check_trie(capacity, 0, n, depth);
    if (rc) return S.done(rc);
    if (!d_levels || !d_data) return S.done(fail(MK_EINVAL, "null pointer"));
    if (d_prev_levels == d_levels) return S.done(fail(MK_EINVAL, "the previous trie's levels alias this trie's"));
    if (!trie_pipe_ok(d_data, n, deposit_len, depth, (hipStream_t)stream))
        return S.done(fail(MK_EINVAL, "pipelined front needs 280-B deposits, 16-B aligned, n a multiple of 4096 "
                                      "with one group per CU, depth >= 7 (n = %llu)", (unsigned long long)n));
    return S.done(trie_front_pipe(d_levels, d_prev_levels, capacity, d_data, n, depth, (hipStream_t)stream));
}

int mk_dev_deposit_trie_pipe_top(mk_call* call, void* d_levels, uint64_t capacity, uint64_t count, uint32_t depth,
                                 void* d_root32, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    rc = check_trie(capacity, count, 0, depth);
    if (rc) return S.done(rc);
    if (!d_levels || !d_root32 || count == 0) return S.done(fail(MK_EINVAL, "null pointer or empty trie"));
    if (depth < 7) return S.done(fail(MK_EINVAL, "depth %u < 7", depth));
    return S.done(trie_levels_range(d_levels, capacity, count, 7, depth, depth, d_root32, (hipStream_t)stream, 256, 4));
}

int mk_dev_deposit_trie_levels(mk_call* call, void* d_levels, uint64_t capacity, uint64_t count, uint32_t d_from,
                               uint32_t d_to, uint32_t depth, void* d_root32, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    rc = check_trie(capacity, count, 0, depth);
    if (rc) return S.done(rc);
    if (d_from > d_to || d_to > depth) return S.done(fail(MK_EINVAL, "levels %u..%u out of range", d_from, d_to));
    if (!d_levels || count == 0 || (d_to == depth && !d_root32))
        return S.done(fail(MK_EINVAL, "null pointer or empty trie"));
    return S.done(trie_levels_range(d_levels, capacity, count, d_from, d_to, depth, d_root32, (hipStream_t)stream));
}

int mk_dev_deposit_trie_branch(mk_call* call, const void* d_levels, uint64_t capacity, uint64_t count,
                               uint32_t depth, uint64_t index, void* d_branch, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    return S.done(rc ? rc : dev_trie_branch(d_levels, capacity, count, depth, index, d_branch, (hipStream_t)stream));
}

// Uploads host deposits (data, offs[k+1]) for an append; fixed_len > 0 when uniform.
static int upload_deposits(DevCtx* c, DevBuf& in, DevBuf& offs_buf, const uint8_t* data, const uint64_t* offs,
                           uint64_t k, const uint64_t** d_offs, uint32_t* fixed_len, std::vector<uint64_t>& rel) {
    const size_t inb = offs[k] - offs[0];
    const int64_t ulen = uniform_len(offs, k);
    TRY(grow(in, inb + 16));
    if (inb) HIPCHK(hipMemcpyAsync(in.p, data + offs[0], inb, hipMemcpyHostToDevice, c->stream));
    if (ulen >= 0) {
        *d_offs = nullptr;
        *fixed_len = (uint32_t)ulen;
        return MK_OK;
    }
    rel.assign(offs, offs + k + 1);
    for (auto& o : rel) o -= offs[0];
    TRY(grow(offs_buf, 8 * (k + 1)));
    HIPCHK(hipMemcpyAsync(offs_buf.p, rel.data(), 8 * (k + 1), hipMemcpyHostToDevice, c->stream));
    *d_offs = (const uint64_t*)offs_buf.p;
    *fixed_len = 0;
    return MK_OK;
}

static int host_trie_build(const uint8_t* data, const uint64_t* offs, uint64_t n, uint32_t depth,
                           uint8_t* levels_out, uint8_t* root) {
    if (!root || (n && !offs)) return fail(MK_EINVAL, "null pointer");
    TRY(check_trie(n, 0, n, depth));
    if (n == 0) {
        std::memset(root, 0, 32);
        return MK_OK;
    }
    TRY(bind_call());
    DevCtx* c = ctx();
    std::lock_guard<std::mutex> lk(c->mu);
    hipStream_t st = c->stream;
    const uint64_t lv_bytes = mk_deposit_trie_levels_bytes(n, depth);
    TRY(grow(c->ws, lv_bytes));
    TRY(grow(c->out, 32));
    const uint64_t* d_offs = nullptr;
    uint32_t fixed = 0;
    std::vector<uint64_t> rel;
    TRY(upload_deposits(c, c->in, c->aux, data, offs, n, &d_offs, &fixed, rel));
    TRY(dev_trie_append(c->ws.p, n, 0, c->in.p, d_offs, n, fixed, depth, c->out.p, st));
    HIPCHK(hipMemcpyAsync(root, c->out.p, 32, hipMemcpyDeviceToHost, st));
    if (levels_out) HIPCHK(hipMemcpyAsync(levels_out, c->ws.p, lv_bytes, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

int mk_deposit_trie_build(mk_call* call, const uint8_t* data, const uint64_t* offs, uint64_t n, uint32_t depth,
                          uint8_t* levels_out, uint8_t root[32]) {
    Scope S(call);
    return S.done(host_trie_build(data, offs, n, depth, levels_out, root));
}

int mk_deposit_trie_new(mk_call* call, uint32_t depth, uint64_t capacity, mk_trie** out) {
    Scope S(call);
    if (!out) return S.done(fail(MK_EINVAL, "null pointer"));
    *out = nullptr;
    if (depth == 0 || depth > 63) return S.done(fail(MK_EINVAL, "depth %u out of range (1..63)", depth));
    int rc = bind_call();
    if (rc) return S.done(rc);
    auto* t = new (std::nothrow) mk_trie();
    if (!t) return S.done(fail(MK_ENOMEM, "trie allocation failed"));
    t->dev = t_bound;
    t->depth = depth;
    t->cap = std::max<uint64_t>(capacity, 1024);
    if (depth < 63) t->cap = std::min<uint64_t>(t->cap, 1ull << depth);
    rc = grow(t->levels, mk_deposit_trie_levels_bytes(t->cap, depth));
    if (!rc) rc = grow(t->root, 32);
    if (!rc) rc = grow(t->branch, 32 * (size_t)depth);
    if (rc) {
        mk_deposit_trie_free(t);
        return S.done(rc);
    }
    *out = t;
    return S.done(MK_OK);
}

void mk_deposit_trie_free(mk_trie* t) {
    if (!t) return;
    int saved = -1;
    const bool restore = hipGetDevice(&saved) == hipSuccess;
    (void)hipSetDevice(t->dev);
    for (DevBuf* b : {&t->levels, &t->root, &t->in, &t->offs, &t->branch})
        if (b->p) (void)hipFree(b->p);
    if (restore) (void)hipSetDevice(saved);
    delete t;
}

uint64_t mk_deposit_trie_count(const mk_trie* t) { return t ? t->count : 0; }

// keep == nullptr: synchronous (the caller's buffers may die on return);
// otherwise the relative offsets live in *keep and the caller synchronizes.
static int trie_append_locked(mk_trie* t, const uint8_t* data, const uint64_t* offs, uint64_t k,
                              std::vector<uint64_t>* keep = nullptr) {
    if (k == 0) return MK_OK;
    TRY(check_trie(UINT64_MAX, t->count, k, t->depth));
    TRY(bind_dev(t->dev));
    DevCtx* c = ctx();
    hipStream_t st = c->stream;
    if (t->count + k > t->cap) {  // double the capacity, moving every level to its new slot
        uint64_t ncap = std::max(2 * t->cap, t->count + k);
        if (t->depth < 63) ncap = std::min<uint64_t>(ncap, 1ull << t->depth);
        DevBuf nl;
        TRY(grow(nl, mk_deposit_trie_levels_bytes(ncap, t->depth)));
        for (uint32_t d = 0; d <= t->depth && t->count; ++d)
            HIPCHK(hipMemcpyAsync(trie_level(nl.p, ncap, d), trie_level(t->levels.p, t->cap, d),
                                  32 * mk::trie_count(t->count, d), hipMemcpyDeviceToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
        (void)hipFree(t->levels.p);
        t->levels = nl;
        t->cap = ncap;
    }
    const uint64_t* d_offs = nullptr;
    uint32_t fixed = 0;
    std::vector<uint64_t> own;
    std::vector<uint64_t>& rel = keep ? *keep : own;
    TRY(upload_deposits(c, t->in, t->offs, data, offs, k, &d_offs, &fixed, rel));
    TRY(dev_trie_append(t->levels.p, t->cap, t->count, t->in.p, d_offs, k, fixed, t->depth, t->root.p, st));
    if (!keep) HIPCHK(hipStreamSynchronize(st));  // the caller's buffers and `rel` are released after this
    t->count += k;
    return MK_OK;
}

static int trie_append(mk_trie* t, const uint8_t* data, const uint64_t* offs, uint64_t k) {
    if (!t || (k && !offs)) return fail(MK_EINVAL, "null pointer");
    std::lock_guard<std::mutex> tl(t->mu);
    return trie_append_locked(t, data, offs, k);
}

int mk_deposit_trie_append(mk_call* call, mk_trie* t, const uint8_t* data, const uint64_t* offs, uint64_t k) {
    Scope S(call);
    return S.done(trie_append(t, data, offs, k));
}

static int trie_root_locked(mk_trie* t, uint8_t* root) {
    if (t->count == 0) {
        std::memset(root, 0, 32);
        return MK_OK;
    }
    TRY(bind_dev(t->dev));
    HIPCHK(hipMemcpyAsync(root, t->root.p, 32, hipMemcpyDeviceToHost, ctx()->stream));
    HIPCHK(hipStreamSynchronize(ctx()->stream));
    return MK_OK;
}

static int trie_root(mk_trie* t, uint8_t* root) {
    if (!t || !root) return fail(MK_EINVAL, "null pointer");
    std::lock_guard<std::mutex> tl(t->mu);
    return trie_root_locked(t, root);
}

int mk_deposit_trie_root(mk_call* call, mk_trie* t, uint8_t root[32]) {
    Scope S(call);
    return S.done(trie_root(t, root));
}

// saveInTrie over a batch of logs (service.go:379-386 called per log by
// ProcessDepositLog :248-258, which skips a log whose check fails): in log
// order, deposit j is appended iff Root() before it equals log_roots[j].
// A round appends every remaining deposit at once, computes the root after
// each (k_trie_prefix_roots) and compares on the host; at the first
// mismatch the trie is cut back to the deposits before it (the right edge
// of the new last leaf recomputed) and the next round starts after the
// skipped log.
static int trie_save_logs(mk_trie* t, const uint8_t* data, const uint64_t* offs, uint64_t k,
                          const uint8_t* log_roots, uint8_t* accepted) {
    if (!t || (k && (!offs || !log_roots || !accepted))) return fail(MK_EINVAL, "null pointer");
    std::lock_guard<std::mutex> tl(t->mu);
    uint64_t pos = 0;
    while (pos < k) {
        const uint64_t m = k - pos;
        const uint64_t count0 = t->count;
        TRY(bind_dev(t->dev));
        hipStream_t st = ctx()->stream;
        // d_roots[f] = Root() before log pos + f: [0] the current root, [1..m]
        // the root after each appended deposit (the last one is the append's)
        TRY(grow(t->branch, std::max<size_t>(32 * (size_t)t->depth, 32 * (m + 1))));
        uint8_t* d_roots = (uint8_t*)t->branch.p;
        if (count0)
            HIPCHK(hipMemcpyAsync(d_roots, t->root.p, 32, hipMemcpyDeviceToDevice, st));
        else
            HIPCHK(hipMemsetAsync(d_roots, 0, 32, st));
        std::vector<uint64_t> rel;
        TRY(trie_append_locked(t, data, offs + pos, m, &rel));
        if (m > 1) {  // one wave per prefix, one wave per SIMD
            hipLaunchKernelGGL((mk::k_trie_prefix_roots<4>), dim3(ceil_div(m - 1, 4)), dim3(256), 0, st,
                               (const uint4*)t->levels.p, t->cap, count0, m - 1, t->depth, (uint4*)(d_roots + 32));
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipMemcpyAsync(d_roots + 32 * m, t->root.p, 32, hipMemcpyDeviceToDevice, st));
        std::vector<uint8_t> roots(32 * (m + 1));
        HIPCHK(hipMemcpyAsync(roots.data(), d_roots, 32 * (m + 1), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        uint64_t f = 0;
        while (f < m && std::memcmp(roots.data() + 32 * f, log_roots + 32 * (pos + f), 32) == 0) {
            accepted[pos + f] = 1;
            ++f;
        }
        if (f == m) break;
        accepted[pos + f] = 0;  // skipped; the deposits after it were appended tentatively
        t->count = count0 + f;
        if (t->count) {  // recompute the last leaf's path without the cut deposits
            TRY(launch_trie_spread(t->levels.p, t->cap, 0, t->count - 1, t->count, t->depth, t->depth, t->root.p,
                                   st));
            HIPCHK(hipStreamSynchronize(st));
        }
        pos += f + 1;
    }
    return MK_OK;
}

int mk_deposit_trie_save_logs(mk_call* call, mk_trie* t, const uint8_t* data, const uint64_t* offs, uint64_t k,
                              const uint8_t* log_roots, uint8_t* accepted) {
    Scope S(call);
    return S.done(trie_save_logs(t, data, offs, k, log_roots, accepted));
}

static int trie_branch(mk_trie* t, uint64_t index, uint8_t* branch) {
    if (!t || !branch) return fail(MK_EINVAL, "null pointer");
    std::lock_guard<std::mutex> tl(t->mu);
    if (t->count == 0) {
        std::memset(branch, 0, 32 * (size_t)t->depth);
        return MK_OK;
    }
    TRY(bind_dev(t->dev));
    hipStream_t st = ctx()->stream;
    TRY(dev_trie_branch(t->levels.p, t->cap, t->count, t->depth, index, t->branch.p, st));
    HIPCHK(hipMemcpyAsync(branch, t->branch.p, 32 * (size_t)t->depth, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

int mk_deposit_trie_branch(mk_call* call, mk_trie* t, uint64_t index, uint8_t* branch) {
    Scope S(call);
    return S.done(trie_branch(t, index, branch));
}

static int trie_leaves(mk_trie* t, uint64_t first, uint64_t cnt, uint8_t* out) {
    if (!t || (cnt && !out)) return fail(MK_EINVAL, "null pointer");
    std::lock_guard<std::mutex> tl(t->mu);
    if (first > t->count || cnt > t->count - first)
        return fail(MK_EINVAL, "leaves [%llu, +%llu) beyond %llu deposits", (unsigned long long)first,
                    (unsigned long long)cnt, (unsigned long long)t->count);
    if (!cnt) return MK_OK;
    TRY(bind_dev(t->dev));
    hipStream_t st = ctx()->stream;
    HIPCHK(hipMemcpyAsync(out, trie_level(t->levels.p, t->cap, 0) + 2 * first, 32 * cnt, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

int mk_deposit_trie_leaves(mk_call* call, mk_trie* t, uint64_t first, uint64_t cnt, uint8_t* out) {
    Scope S(call);
    return S.done(trie_leaves(t, first, cnt, out));
}

static int host_verify(const uint8_t* leaves, const uint8_t* branches, const uint64_t* indices, uint64_t n,
                       uint32_t depth, uint32_t tree_depth, const uint8_t* roots, uint8_t* ok) {
    if (n && (!leaves || !indices || !roots || !ok || (depth && !branches))) return fail(MK_EINVAL, "null pointer");
    TRY(bind_call());
    if (n == 0) return MK_OK;
    DevCtx* c = ctx();
    std::lock_guard<std::mutex> lk(c->mu);
    hipStream_t st = c->stream;
    const size_t bb = 32 * (size_t)depth * n;
    TRY(grow(c->in, bb + 64 * n + 16));
    TRY(grow(c->aux, 8 * n));
    TRY(grow(c->out, n));
    uint8_t* base = (uint8_t*)c->in.p;
    uint8_t* d_leaves = base;
    uint8_t* d_roots = base + 32 * n;
    uint8_t* d_br = base + 64 * n;
    HIPCHK(hipMemcpyAsync(d_leaves, leaves, 32 * n, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_roots, roots, 32 * n, hipMemcpyHostToDevice, st));
    if (bb) HIPCHK(hipMemcpyAsync(d_br, branches, bb, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(c->aux.p, indices, 8 * n, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(mk::k_verify_branches, dim3(ceil_div(n, 256)), dim3(256), 0, st, (const uint4*)d_leaves,
                       (const uint4*)d_br, (const uint64_t*)c->aux.p, depth, tree_depth, (const uint4*)d_roots, n,
                       (uint8_t*)c->out.p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(ok, c->out.p, n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MK_OK;
}

int mk_verify_merkle_branches(mk_call* call, const uint8_t* leaves, const uint8_t* branches,
                              const uint64_t* indices, uint64_t n, uint32_t depth, uint32_t tree_depth,
                              const uint8_t* roots, uint8_t* ok) {
    Scope S(call);
    return S.done(host_verify(leaves, branches, indices, n, depth, tree_depth, roots, ok));
}

// ---- synthetic inputs -------------------------------------------------------------
int mk_dev_synth_fill(mk_call* call, void* d_dst, uint64_t nbytes, uint64_t seed, uint64_t word0, void* stream) {
    Scope S(call);
    int rc = bind_stream((hipStream_t)stream);
    if (rc) return S.done(rc);
    if (nbytes % 8) return S.done(fail(MK_EINVAL, "nbytes %% 8 != 0"));
    if ((uintptr_t)d_dst % 8) return S.done(fail(MK_EINVAL, "destination not 8-byte aligned"));
    const uint64_t nwords = nbytes / 8;
    if (!nwords) return S.done(MK_OK);
    const uint64_t grid = std::min<uint64_t>(ceil_div(nwords, 256), 256 * 64);
    hipLaunchKernelGGL(mk::k_synth, dim3(grid), dim3(256), 0, (hipStream_t)stream, (uint64_t*)d_dst, nwords, seed,
                       word0);
    hipError_t e = hipGetLastError();
    return S.done(e == hipSuccess ? MK_OK : fail(MK_EHIP, "k_synth: %s", hipGetErrorString(e)));
}

// ---- measurement ----------------------------------------------------------------------
int mk_prof_enable(int on) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_on = on != 0;
    return MK_OK;
}

static int prof_read(double* leaf_ms, uint64_t* leaf_launches, double* leaf_perms, double* leaf_hashes) {
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

int mk_prof_read(mk_call* call, double* leaf_ms, uint64_t* leaf_launches, double* leaf_perms, double* leaf_hashes) {
    Scope S(call);
    return S.done(prof_read(leaf_ms, leaf_launches, leaf_perms, leaf_hashes));
}

}  // extern "C"
