"""Per-kernel timeline of the last merkleHash step from a rocprofv3 kernel
trace (run_kernel_trace.csv): name, workgroups, duration, gap before it."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
nlast = int(sys.argv[2]) if len(sys.argv) > 2 else 12
prev = None
for r in rows[-nlast:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
    print(f"{r['Kernel_Name'][:44]:44s} wg={wg:6d}x{r['Workgroup_Size_X']:>4s} dur={(e - s) / 1e3:8.1f}us gap={gap:6.1f}us")
    prev = e
