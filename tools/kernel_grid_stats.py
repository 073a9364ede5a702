"""Per (kernel, grid size) mean duration of a rocprofv3 kernel-trace CSV.
    python3 tools/kernel_grid_stats.py DIR/.../kernel_trace.csv"""
import collections
import csv
import sys

acc = collections.defaultdict(list)
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    key = (r["Kernel_Name"][:60], r.get("Grid_Size_X") or r.get("Grid_Size", ""))
    acc[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (name, grid), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    print(f"{name:60s} grid {grid:>9s}  n={len(v):4d}  mean {sum(v) / len(v):9.2f} us  "
          f"min {min(v):9.2f} us")
