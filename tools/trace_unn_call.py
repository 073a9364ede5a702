"""UnN_many calls of K = 20 steps (or argv[1]) at the bench shape (1e6/class, 64 shards), for a rocprofv3
--kernel-trace run; with a CSV argument instead, prints the last call's kernel timeline (start
offsets, durations, idle gaps) to see the per-call overhead beside the K count launches.
    rocprofv3 --kernel-trace --output-format csv -d DIR -- python3 tools/trace_unn_call.py
    python3 tools/trace_unn_call.py DIR/.../kernel_trace.csv"""
import csv
import pathlib
import sys
import time

if len(sys.argv) > 1 and sys.argv[1].endswith(".csv"):
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70])
                for r in rows)
    # the last call: after the last idle gap of > 200 us
    cut = 0
    for k in range(1, len(ev)):
        if ev[k][0] - ev[k - 1][1] > 200_000:
            cut = k
    t0 = ev[cut][0]
    prev = t0
    for s, e, n in ev[cut:]:
        print(f"{(s - t0) / 1e3:9.1f} us  +gap {(s - prev) / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f}  {n}")
        prev = e
    sys.exit(0)

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import tuplewise  # noqa: E402,F401
from tuplewise.device import ShardedSample  # noqa: E402

torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(1)
X = torch.randn(1_000_000, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(1_000_000, dtype=torch.float64, device="cuda", generator=g)
S = ShardedSample(X, Z, 64, algo="pairs")
K = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 20
for c in range(6):
    torch.cuda.synchronize()
    time.sleep(0.01)  # a gap the summary cuts on
    t0 = time.perf_counter()
    S.UnN_many(range(100 * c, 100 * c + K))
    torch.cuda.synchronize()
    print(f"call {c}: {(time.perf_counter() - t0) * 1e3:.3f} ms", flush=True)
