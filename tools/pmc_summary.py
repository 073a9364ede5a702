"""Summarise rocprofv3 --pmc CSV passes for one kernel into a JSON (profiles/).

usage: python tools/pmc_summary.py OUT.json KERNEL_SUBSTR DIR [DIR ...]
Each DIR holds one pass's *counter_collection.csv.  Values are averaged per dispatch of the
kernel, separately for each grid size (the one-launch UnN step's grid carries the next
repartition on extra blocks; a plain count launch does not).  HBM bytes = (FETCH_SIZE + WRITE_SIZE) * 1024 (rocprofv3 reports KB); on gfx950
FETCH_SIZE under-reports 16-B/lane streaming reads by 2x (MI355X_MICROARCH.md §HBM) — the
count kernel reads x with 8-B/lane loads and z through the scalar cache, widths the guide
lists as uncalibrated, so the raw value is reported beside the algorithmic bytes."""
import csv
import glob
import json
import sys
from collections import defaultdict

out, kname, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
# counter -> grid size -> dispatch -> value: launches of one kernel with different grids (the
# one-launch UnN step carries extra blocks) are summarised separately
per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
for d in dirs:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if kname not in row.get("Kernel_Name", ""):
                continue
            per[row["Counter_Name"]][row.get("Grid_Size", "?")][row["Dispatch_Id"]] += \
                float(row["Counter_Value"])
res = {"kernel": kname, "passes": dirs, "by_grid": {}}
for c, grids in per.items():
    for g, disp in grids.items():
        vals = list(disp.values())
        e = res["by_grid"].setdefault(g, {})
        e[c] = sum(vals) / len(vals)
        e[c + "_dispatches"] = len(vals)
for g, e in res["by_grid"].items():
    if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
        e["hbm_bytes_per_launch"] = (e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024.0
# the largest grid is the timed one-launch step (count blocks + the next repartition's spare
# blocks); the next largest is a plain count launch of the same shards (other, smaller grids
# come from the bench's other lines, e.g. the C1/C2 launches)
grids = sorted((g for g in res["by_grid"] if g.isdigit()), key=int, reverse=True)
main = grids[0] if grids else next(iter(res["by_grid"]))
res["timed_grid"] = main
res["plain_grid"] = grids[1] if len(grids) > 1 else None
res["hbm_bytes_per_launch"] = res["by_grid"][main].get("hbm_bytes_per_launch")
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
