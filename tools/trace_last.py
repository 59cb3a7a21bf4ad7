"""Kernels around the last launch of a named kernel in a rocprofv3 kernel
trace: name, queue, workgroups x size, start (us, mod 1 s), duration, gap
to the previous kernel's end.

  python tools/trace_last.py TRACE.csv SUBSTR [BEFORE AFTER]"""
import csv
import sys


def short(n):
    return n.split("(")[0].replace("void ", "")[:46]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    b, a = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (3, 8)
    idx = [i for i, r in enumerate(rows) if sys.argv[2] in r["Kernel_Name"]]
    i = idx[-1]
    prev = None
    for r in rows[max(0, i - b):i + a]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        print(f"{short(r['Kernel_Name']):46s} q={r['Queue_Id']} wg={wg:6d}x{r['Workgroup_Size_X']:>4s} "
              f"s={s % 10**9 / 1e3:10.1f} dur={(e - s) / 1e3:7.1f} gap={gap:6.1f}")
        prev = e


if __name__ == "__main__":
    main()
