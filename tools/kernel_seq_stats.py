"""Consecutive same-kernel runs of a rocprofv3 kernel-trace CSV, in launch order: for each run
of identical (kernel, grid) launches, the count and mean duration — so a script that sweeps
tuning hooks shows each setting's kernels in sequence.
    python3 tools/kernel_seq_stats.py DIR/.../kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
runs = []
for r in rows:
    key = (r["Kernel_Name"][:56], r.get("Grid_Size_X") or r.get("Grid_Size", ""))
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if runs and runs[-1][0] == key:
        runs[-1][1].append(d)
    else:
        runs.append((key, [d]))
for (name, grid), v in runs:
    print(f"{name:56s} grid {grid:>9s} n={len(v):3d} mean {sum(v) / len(v):9.2f} us")
