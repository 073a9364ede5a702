"""The C4 replay line's first-run penalty: bench.py's sequence — one
50-step warm learning_process call, then 2000-step calls — with the one-time costs inside each
call timed: pinned-ring / table-stack (re)allocations and replay-graph captures.
    python tools/replay_first_run.py [runs]"""
import logging
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np
import torch

import bench
import tuplewise.learning as lr

logging.disable(logging.CRITICAL)
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
cost = {}


def timed(cls, name):
    f = getattr(cls, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            c = cost.setdefault(name, [0, 0.0])
            c[0] += 1
            c[1] += time.perf_counter() - t0
    setattr(cls, name, g)


for n in ("_rows_buffers", "_seg_buffers", "native_pipe"):
    timed(lr._ReplayDraws, n)
timed(lr.SGDEngine, "table_stacks")
timed(lr.SGDEngine, "run_replay_segment")
X, Z, w0 = bench.c4_problem()
p = {"n_it": 2000, "margin": 1, "N": 100, "B": 100, "reshuffle_mod": 25, "reg": 0.05,
     "learning_rate": 0.01, "eval_mod": 10 ** 9, "w_init": w0, "test_X": X[:10],
     "test_Z": Z[:10], "train_mon_pairs": [(0, 0)], "train_X": X, "train_Z": Z}
np.random.seed(0)
for i in range(runs + 1):
    cost.clear()
    pp = dict(p, n_it=50) if i == 0 else p
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lr.learning_process(X, Z, pp)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    eng = lr._ENGINE["eng"]
    ng = len(getattr(eng, "_replay_graphs", {}) or {})
    print(f"{'warm' if i == 0 else 'run'} {pp['n_it']} steps: {dt * 1e3:.2f} ms "
          f"({pp['n_it'] / dt:.0f} steps/s), graphs cached {ng}; "
          + ", ".join(f"{k} {c[0]}x {c[1] * 1e3:.2f} ms" for k, c in cost.items()),
          flush=True)
