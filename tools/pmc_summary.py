"""Summarise rocprofv3 --pmc CSV passes for one kernel into a JSON (profiles/).

usage: python tools/pmc_summary.py OUT.json KERNEL_SUBSTR DIR [DIR ...]
Each DIR holds one pass's *counter_collection.csv.  Values are averaged per dispatch of the
kernel.  HBM bytes = (FETCH_SIZE + WRITE_SIZE) * 1024 (rocprofv3 reports KB); on gfx950
FETCH_SIZE under-reports 16-B/lane streaming reads by 2x (MI355X_MICROARCH.md §HBM) — the
count kernel reads x with 8-B/lane loads and z through the scalar cache, widths the guide
lists as uncalibrated, so the raw value is reported beside the algorithmic bytes."""
import csv
import glob
import json
import sys
from collections import defaultdict

out, kname, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
per = defaultdict(lambda: defaultdict(float))
for d in dirs:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if kname not in row.get("Kernel_Name", ""):
                continue
            per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
res = {"kernel": kname, "passes": dirs}
for c, disp in per.items():
    vals = list(disp.values())
    res[c] = sum(vals) / len(vals)
    res[c + "_dispatches"] = len(vals)
if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
    res["hbm_bytes_per_launch"] = (res["FETCH_SIZE"] + res["WRITE_SIZE"]) * 1024.0
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
