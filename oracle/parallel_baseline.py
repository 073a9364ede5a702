"""ORACLE — test/benchmark infrastructure only (bench.py's cpu_baseline leg).

All-cores CPU figure for the north-star workload ("plus an all-cores figure,
with shards spread over worker processes — a restatement, because the reference itself is
serial"): one est.UnN (estimation-experiment/main.py:72-74) — the in-place shuffles, then the
N prop-SWOR blocks' est.Un (main.py:29-31, oracle.est_Un) spread over `workers` processes.
Run as a fresh process that never touches the GPU:
    python -m oracle.parallel_baseline N_PER_CLASS N_SHARDS WORKERS
prints one JSON object."""
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np


def _block(args):
    x, z = args
    return int((x[:, None] > z[None, :]).sum())  # est.Un's compare (main.py:29-31), counted


def main(n: int, N: int, workers: int) -> dict:
    rng = np.random.RandomState(0)
    X, Z = rng.normal(0.5, 1, n), rng.normal(0, 1, n)
    k = n // N
    rows = max(1, -(-workers // N))  # row chunks per block, so that every worker has blocks
    step = -(-k // rows)
    with ProcessPoolExecutor(max_workers=workers) as ex:
        list(ex.map(_block, [(X[:64], Z[:64])] * workers))  # start the workers
        t0 = time.perf_counter()
        np.random.shuffle(X)
        np.random.shuffle(Z)
        tasks = [(X[s * k + a:s * k + min(k, a + step)], Z[s * k:(s + 1) * k])
                 for s in range(N) for a in range(0, k, step)]
        cnt = list(ex.map(_block, tasks))
        per = [sum(cnt[s * rows:(s + 1) * rows]) / (k * k) for s in range(N)]
        float(np.mean(per))
        dt = time.perf_counter() - t0
    return {"value": N * k * k / dt, "unit": "pairs/s", "cores": workers, "kind": "port",
            "sample": f"est.UnN (in-place shuffle + {N} prop-SWOR blocks of {k}x{k}, each "
                      f"cut into {rows} row chunks) over {workers} processes, n={n}/class, "
                      f"{dt:.2f} s"}


if __name__ == "__main__":
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    print(json.dumps(main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]))))
