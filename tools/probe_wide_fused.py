"""C5 B = 100 (bench.py's C5_scaled_d512 line) with the fused wide step (learning.WIDE_FUSED:
one tw_sgd_step_wide launch per step, the previous update spread over its blocks behind a grid
barrier) and without (gradient + update launches), alternating, then both settings' kernel
means in one torch.profiler session (in-process).
    python tools/probe_wide_fused.py"""
import json
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch

import bench
import tuplewise.learning as lr
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent))
from probe_learn_ranks import kernel_means  # noqa: E402

data = bench.sgd_data(bench.C5_N, bench.C5_N, 512)
res = {}
for rep in range(2):
    for fused in (True, False):
        lr.WIDE_FUSED = fused
        r = bench.sgd_steps_per_s(bench.C5_N, bench.C5_N, 512, 256, 100, 25, 500, 2, data=data)
        res.setdefault(str(fused), []).append(round(r["ms_per_step"] * 1e3, 2))
print(json.dumps({"us_per_step (fused, unfused; two rounds)": res}), flush=True)


def both():  # one profiler session (a second one in the same process crashed the tracer)
    for fused in (True, False):
        lr.WIDE_FUSED = fused
        bench.sgd_steps_per_s(bench.C5_N, bench.C5_N, 512, 256, 100, 25, 200, 1, data=data)


print(json.dumps({"kernels (both settings, 200 steps each)": kernel_means(both)}, indent=1),
      flush=True)
