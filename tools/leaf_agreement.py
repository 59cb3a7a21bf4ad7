"""Does the rocprofv3 kernel trace agree with bench.py's own hipEvent timing
of the leaf kernel?  Reads <prof dir>/stats/run_kernel_trace.csv and the
bench JSON line in <prof dir>/stats.log (the same command), and prints the
per-launch trace durations, their average over the timed launches (the last
`steps`), and bench.py's avg_launch_ms.

  python tools/leaf_agreement.py gpurun_out/prof_<tag> [kernel-prefix]
"""
import csv
import json
import os
import sys


def main():
    d = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else "void mk::k_reduce<true, true, 2>"
    bench = None
    for line in open(os.path.join(d, "stats.log")):
        if line.startswith("{"):
            bench = json.loads(line)
    rows = [r for r in csv.DictReader(open(os.path.join(d, "stats", "run_kernel_trace.csv")))
            if r["Kernel_Name"].startswith(kern)]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    steps = bench["steps"]
    timed = ms[-steps:]
    out = {"kernel": kern, "trace_launch_ms": [round(x, 4) for x in ms],
           "trace_avg_timed_ms": sum(timed) / len(timed), "trace_avg_all_ms": sum(ms) / len(ms),
           "bench_hipevent_avg_launch_ms": bench["roofline"]["avg_launch_ms"],
           "note": f"the last {steps} trace launches are the bench's timed steps; the earlier ones are the "
                   "pipelined-root check and the warmup (clock ramp)"}
    out["ratio_trace_over_hipevent"] = out["trace_avg_timed_ms"] / out["bench_hipevent_avg_launch_ms"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
