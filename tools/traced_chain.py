"""The headline count kernel's TRACED duration (the traced figure beside
bench.py's live `roofline.frac`): from a rocprofv3 --kernel-trace CSV of `bench.py --steps K`,
the strict k_count_chain launches of the largest grid and at least half the longest one's
duration (the K-step chunks of the headline's UnN_many calls; the strong_C3 and half-ties lines
launch shorter calls or the HALF kernel),
their mean and minimum duration, and the lane-op fraction they imply; in time order the first
is the bench's untimed warm-up call (a cold chip: its clock is still rising), the SECOND the
timed call whose HIP-event duration gives the live `frac` — `timed_ms` / `frac_timed` is that
same launch as the tracer saw it — and (round 5, late) a third the `first_call_ranking` line's
call of the same steps.
    python3 tools/traced_chain.py TRACE.csv K OUT.json"""
import csv
import json
import sys

PAIRS_PER_STEP = 64 * 15625 * 15625  # n = 1e6/class, N = 64 shards
PEAK = 256 * 64 * 2.4e9  # lane-op/s

path, K, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rows = [r for r in csv.DictReader(open(path))
        if "k_count_chain<" in r["Kernel_Name"] and ", false>" in r["Kernel_Name"]]
grid = lambda r: int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
g = max(grid(r) for r in rows)
big = sorted((r for r in rows if grid(r) == g), key=lambda r: int(r["Start_Timestamp"]))
ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in big]
# (round 5, late: the z chunks are sized for a fixed count of work items, so calls of other
# step counts — the bench's 5-step settle calls — launch the same grid; the K-step launches
# are the long ones)
ds = [d for d in ds if d >= 0.5 * max(ds)]
mean, lo = sum(ds) / len(ds), min(ds)
res = {"kernel": rows[0]["Kernel_Name"].split("(")[0], "grid": g, "launches": len(ds),
       "steps_per_launch": K, "mean_ms": mean, "min_ms": lo,
       "frac_mean": K * PAIRS_PER_STEP / (mean * 1e-3) / PEAK,
       "frac_min": K * PAIRS_PER_STEP / (lo * 1e-3) / PEAK, "launch_ms_in_order": ds,
       "timed_ms": ds[min(1, len(ds) - 1)],
       "frac_timed": K * PAIRS_PER_STEP / (ds[min(1, len(ds) - 1)] * 1e-3) / PEAK,
       "source": path}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
