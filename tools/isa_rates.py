"""Generate and build tools/isa_rates.hip: per-instruction issue costs on gfx950
for the integer VALU instructions a Keccak round can be built from.

Each test is an inline-asm block on FIXED registers (v40..v63), 8 independent
chains, so the operand VGPR banks (reg % 4) are under control — plain HIP
leaves register choice to the allocator.  Two modes:
  * throughput: 1024 workgroups x 256 threads (4 waves per SIMD);
  * lone wave:  1 workgroup of 64 threads (what one wave alone sustains —
    the cost that sets a permutation's latency at the narrow top of a tree).
Output: one JSON line per (test, mode) with cycles per wave-instruction per SIMD.

  python tools/isa_rates.py          # writes + builds tools/isa_rates
  ./tools/isa_rates                  # on the GPU box
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

# name -> (template, kind); {d} destination of chain c (v40+c), {a}/{b} sources.
# kind "same": sources in the destination's bank; "diff": three distinct banks.
B3 = "v_bitop3_b32 {d}, {d}, {a}, {b} bitop3:0x96"
CH = "v_bitop3_b32 {d}, {d}, {b}, {a} bitop3:0xd2"
AL = "v_alignbit_b32 {d}, {d}, {a}, 7"
XO = "v_xor_b32 {d}, {a}, {d}"
# name -> (instruction sequence, kind); instruction k of the block works on
# chain k % 8 (destination v40+c, sources in other banks unless "same").
TESTS = {
    "xor": ([XO], "diff"),
    "bitop3": ([B3], "diff"),
    "alignbit": ([AL], "diff"),
    "alignbit_s0": (["v_alignbit_b32 {d}, {d}, {a}, 0"], "diff"),
    "lshlrev32_nc": (["v_lshlrev_b32 {d}, 7, {a}"], "diff"),
    "lshrrev32_nc": (["v_lshrrev_b32 {d}, 7, {a}"], "diff"),
    "lshlrev32_v": (["v_lshlrev_b32 {d}, {b}, {a}"], "diff"),
    "lshl_or_nc": (["v_lshl_or_b32 {d}, {a}, 7, {b}"], "diff"),
    "add": (["v_add_u32 {d}, {a}, {d}"], "diff"),
    "and": (["v_and_b32 {d}, {a}, {d}"], "diff"),
    "or": (["v_or_b32 {d}, {a}, {d}"], "diff"),
    "not": (["v_not_b32 {d}, {a}"], "diff"),
    "bfe": (["v_bfe_u32 {d}, {a}, 3, 7"], "diff"),
    "or3": (["v_or3_b32 {d}, {d}, {a}, {b}"], "diff"),
    "add3": (["v_add3_u32 {d}, {d}, {a}, {b}"], "diff"),
    "xad": (["v_xad_u32 {d}, {d}, {a}, {b}"], "diff"),
    "and_or": (["v_and_or_b32 {d}, {d}, {a}, {b}"], "diff"),
    "xor_e64": (["v_xor_b32_e64 {d}, {a}, {d}"], "diff"),
    "mul_u24": (["v_mul_u32_u24 {d}, {a}, {d}"], "diff"),
    "pk_add_u16": (["v_pk_add_u16 {d}, {a}, {d}"], "diff"),
    "lshrrev64": (["v_lshrrev_b64 {D}, 7, {D}"], "pair"),
    "B_X": ([B3, XO], "diff"),
    "B_L": ([B3, "v_lshrrev_b32 {d}, 7, {a}"], "diff"),
    "B_A": ([B3, AL], "diff"),
    "B8_A8": ([B3] * 8 + [AL] * 8, "diff"),
    "B32_A32": ([B3] * 32 + [AL] * 32, "diff"),
    "B3_A1_x16": ([B3, CH, B3] * 16 + [AL] * 16, "diff"),
    "X_D": ([XO, "v_mov_b32_dpp {d}, {a} quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"], "diff"),
    "lshl_add_u64": (["v_lshl_add_u64 {D}, {D}, 7, {A}"], "pair"),
    "lshlrev64": (["v_lshlrev_b64 {D}, 7, {D}"], "pair"),
    "mad_u64_u32": (["v_mad_u64_u32 {D}, vcc, {d0}, v60, {D}"], "pair"),
    "mov_b64": (["v_mov_b64 {D}, {A}"], "pair"),
    "lshl_add_u32": (["v_lshl_add_u32 {d}, {d}, 7, {a}"], "diff"),
    "add_lshl": (["v_add_lshl_u32 {d}, {d}, {a}, 7"], "diff"),
    "rot64_shr_lshladd": (["v_lshrrev_b64 {D}, 57, {A}", "v_lshl_add_u64 {D}, {A}, 7, {D}"], "pair"),
}
# wave-specialised: even workgroups run SPLIT[0], odd ones SPLIT[1]
SPLIT = {"split_B_A": ([B3], [AL]), "split_B_B": ([B3], [CH])}
# phase-aligned: 1024-thread workgroups (4 waves per SIMD, all of one
# workgroup) so an s_barrier lines up every wave of a SIMD on the same
# instruction class.  name -> segments; "|" between segments = s_barrier,
# a trailing barrier closes every iteration when bar_end is set.
# (segments, bar_end)
SYNC = {
    "s_B": ([[B3] * 64], True),
    "s_A": ([[AL] * 64], True),
    "s_B32A32_nobar": ([[B3] * 32 + [AL] * 32], False),
    "s_B32A32_bar1": ([[B3] * 32 + [AL] * 32], True),
    "s_B32|A32": ([[B3] * 32, [AL] * 32], True),
    "s_B64|A64": ([[B3] * 64, [AL] * 64], True),
    "s_B128|A128": ([[B3] * 128, [AL] * 128], True),
    # Keccak-round shaped: F72 H10 F50 H48 (122 full + 58 half)
    "s_round_nobar": ([[B3] * 72 + [AL] * 10 + [B3] * 50 + [AL] * 48], False),
    "s_round_bar1": ([[B3] * 72 + [AL] * 10 + [B3] * 50 + [AL] * 48], True),
    "s_round_bar4": ([[B3] * 72, [AL] * 10, [B3] * 50, [AL] * 48], True),
    "s_round_bar2": ([[B3] * 72 + [AL] * 10 + [B3] * 50, [AL] * 48], True),
}

def regs(c, kind):
    if kind == "pair":  # 64-bit chains v[40+2c : 41+2c] (4 chains reused twice)
        c4 = c % 4
        return {"D": f"v[{40 + 2 * c4}:{41 + 2 * c4}]", "A": f"v[{56 + 2 * (c4 % 2)}:{57 + 2 * (c4 % 2)}]",
                "d0": f"v{40 + 2 * c4}"}
    d = 40 + c
    if kind == "same":
        a, b = 48 + c, 56 + c  # same bank as d (mod 4)
    else:
        a, b = 48 + (c + 1) % 8, 56 + (c + 2) % 8
    return {"d": f"v{d}", "a": f"v{a}", "b": f"v{b}"}


def asm_body(seq, kind):
    lines = []
    k = 0
    n = max(64, len(seq))
    while len(lines) < n or len(lines) % len(seq):
        lines.append(seq[k % len(seq)].format(**regs(k % 8, kind)))
        k += 1
    return lines


def gen():
    out = ["// GENERATED by tools/isa_rates.py -- do not edit",
           "#include <hip/hip_runtime.h>", "#include <cstdio>", "#include <cstdlib>", "",
           "#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, \"%s\\n\", hipGetErrorString(e)); exit(1);} } while (0)",
           ""]
    clob = ", ".join(f'"v{r}"' for r in range(40, 64)) + ', "vcc"'
    names = []
    def emit(name, bodies):
        out.append(f"__global__ __launch_bounds__(256) void k_{name}(unsigned* out, int iters, unsigned long long* clk) {{")
        out.append("    unsigned seed = threadIdx.x * 2654435761u + blockIdx.x;")
        out.append("    asm volatile(")
        out.append("        \"v_mov_b32 v40, %0\\n v_add_u32 v41, 1, v40\\n v_add_u32 v42, 2, v40\\n v_add_u32 v43, 3, v40\\n\"")
        out.append("        \"v_add_u32 v44, 4, v40\\n v_add_u32 v45, 5, v40\\n v_add_u32 v46, 6, v40\\n v_add_u32 v47, 7, v40\\n\"")
        for r in range(48, 64):
            out.append(f"        \"v_add_u32 v{r}, {r}, v40\\n\"")
        out.append("        \"s_mov_b32 vcc_lo, 0x55555555\\n s_mov_b32 vcc_hi, 0x55555555\\n\"")
        out.append(f"        :: \"v\"(seed) : {clob});")
        out.append("    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();")
        for bi, body in enumerate(bodies):
            if len(bodies) > 1:
                out.append(f"    if ((blockIdx.x & 1) == {bi}) {{")
            asm_lines = "\n".join(f'        "{l}\\n"' for l in body)
            out.append("#pragma unroll 1")
            out.append("    for (int it = 0; it < iters; ++it) {")
            out.append("        asm volatile(")
            out.append(asm_lines)
            out.append(f"        ::: {clob});")
            out.append("    }")
            if len(bodies) > 1:
                out.append("    }")
        out.append("    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();")
        out.append("    unsigned x;")
        out.append("    asm volatile(\"v_xor_b32 %0, v40, v41\\n v_xor_b32 %0, v42, %0\\n\" : \"=v\"(x) :: " + clob + ");")
        out.append("    out[blockIdx.x * blockDim.x + threadIdx.x] = x;")
        out.append("    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }")
        out.append("}")
        out.append("")

    for name, (seq, kind) in TESTS.items():
        body = asm_body(seq, kind)
        names.append((name, len(body)))
        emit(name, [body])
    for name, (s0, s1) in SPLIT.items():
        b0, b1 = asm_body(s0, "diff"), asm_body(s1, "diff")
        assert len(b0) == len(b1)
        names.append((name, len(b0)))
        emit(name, [b0, b1])
    def emit_sync(name, segs, bar_end):
        out.append(f"__global__ __launch_bounds__(1024) void k_{name.replace('|', '_')}(unsigned* out, int iters, unsigned long long* clk) {{")
        out.append("    unsigned seed = threadIdx.x * 2654435761u + blockIdx.x;")
        out.append("    asm volatile(\"v_mov_b32 v40, %0\\n\"")
        for r in list(range(41, 48)) + list(range(48, 64)):
            out.append(f"        \"v_add_u32 v{r}, {r}, v40\\n\"")
        out.append(f"        :: \"v\"(seed) : {clob});")
        out.append("    __syncthreads();")
        out.append("    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();")
        out.append("#pragma unroll 1")
        out.append("    for (int it = 0; it < iters; ++it) {")
        lines = []
        for si, seg in enumerate(segs):
            lines += [seg[k].format(**regs(k % 8, "diff")) for k in range(len(seg))]
            if si + 1 < len(segs) or bar_end:
                lines.append("s_barrier")
        out.append("        asm volatile(")
        out.append("\n".join(f'        "{l}\\n"' for l in lines))
        out.append(f"        ::: {clob});")
        out.append("    }")
        out.append("    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();")
        out.append("    unsigned x;")
        out.append("    asm volatile(\"v_xor_b32 %0, v40, v41\\n v_xor_b32 %0, v42, %0\\n\" : \"=v\"(x) :: " + clob + ");")
        out.append("    out[blockIdx.x * blockDim.x + threadIdx.x] = x;")
        out.append("    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }")
        out.append("}")
        out.append("")

    if ONLY != "sync":
        pass
    else:
        del names[:]
        out[:] = out[:7]
    sync_names = []
    for name, (segs, bar_end) in SYNC.items():
        emit_sync(name, segs, bar_end)
        sync_names.append((name, sum(len(x) for x in segs)))
    out.append("""
typedef void (*kfn)(unsigned*, int, unsigned long long*);
static void run(const char* name, kfn k, int ninstr, int blocks, int threads, int iters) {
    unsigned* out; unsigned long long* clk;
    CHECK(hipMalloc(&out, (size_t)blocks * threads * 4));
    CHECK(hipMalloc(&clk, 16));
    hipLaunchKernelGGL(k, blocks, threads, 0, 0, out, iters, clk);
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(k, blocks, threads, 0, 0, out, iters, clk);
    CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
    float ms = 0; CHECK(hipEventElapsedTime(&ms, a, b));
    unsigned long long h[2]; CHECK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
    const double ghz = h[1] ? (double)h[0] / (double)h[1] * 0.1 : 0;
    const double wave_instr = (double)ninstr * iters;            // per wave
    const double cyc_in_kernel = (double)h[0];                   // shader clocks, wave 0
    const double waves = (double)blocks * threads / 64;
    const double waves_per_simd = waves / 1024.0;
    // cycles per wave-instruction per SIMD (throughput: all waves of a SIMD share it)
    const double cpi_simd = blocks == 1 ? cyc_in_kernel / wave_instr
                                        : (ms / 1e3) * ghz * 1e9 / (wave_instr * waves_per_simd);
    char mode[16];
    if (blocks == 1) snprintf(mode, sizeof mode, "lone");
    else snprintf(mode, sizeof mode, "%s%g", threads == 1024 ? "sync_w" : "w", waves_per_simd);
    printf("{\\"test\\": \\"%s\\", \\"mode\\": \\"%s\\", \\"cycles_per_instr\\": %.3f, \\"Tops\\": %.2f, \\"ms\\": %.3f, \\"clock_GHz\\": %.3f}\\n",
           name, mode, cpi_simd,
           blocks == 1 ? 0.0 : wave_instr * waves * 64 / (ms / 1e3) / 1e12, ms, ghz);
    CHECK(hipFree(out)); CHECK(hipFree(clk));
}

int main() {
""")
    for name, n in names:
        it = max(100, 256000 // n)
        for w in (2, 4, 8):
            out.append(f"    run(\"{name}\", k_{name}, {n}, {256 * w}, 256, {it});")
        out.append(f"    run(\"{name}\", k_{name}, {n}, 1, 64, {it // 4});")
    for name, n in sync_names:
        it = max(100, 256000 // n)
        for w in (4, 8):
            out.append(f"    run(\"{name}\", k_{name.replace('|', '_')}, {n}, {256 * w // 4}, 1024, {it});")
    out.append("    return 0;\n}")
    return "\n".join(out) + "\n"


ONLY = ""


def main():
    global ONLY
    if len(sys.argv) > 1 and sys.argv[1] == "--only-sync":
        ONLY = "sync"
    src = os.path.join(HERE, "isa_rates.hip")
    with open(src, "w") as f:
        f.write(gen())
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", src, "-o", os.path.join(HERE, "isa_rates")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.stderr.write(r.stderr[-4000:])
        sys.exit(r.returncode)
    print("built tools/isa_rates")


if __name__ == "__main__":
    main()
