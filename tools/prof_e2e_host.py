"""Host-side profile of the C4 learning_process with an evaluation every 25 steps (bench's
learning_end_to_end, device RNG or replay): where the Python time of one eval-to-eval cycle
goes.  GPU box:  python tools/prof_e2e_host.py [device|replay]"""
import cProfile
import pathlib
import pstats
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import logging

import numpy as np
import torch

import tuplewise.learning as lr

mode = sys.argv[1] if len(sys.argv) > 1 else "device"
rng = np.random.RandomState(4)
X = np.hstack([rng.normal(size=(9117, 9)), np.ones((9117, 1))])
Z = np.hstack([rng.normal(0.5, 1, size=(702, 9)), np.ones((702, 1))])
Xe = np.hstack([rng.normal(size=(2279, 9)), np.ones((2279, 1))])
Ze = np.hstack([rng.normal(0.5, 1, size=(175, 9)), np.ones((175, 1))])
mon = list(zip(rng.randint(0, 9117, 450000), rng.randint(0, 702, 450000)))
steps = 20000
p = {"n_it": steps, "margin": 1, "N": 100, "B": 100, "reshuffle_mod": 25, "reg": 0.05,
     "learning_rate": 0.01, "eval_mod": 25, "w_init": rng.normal(size=(10, 1)),
     "test_X": Xe, "test_Z": Ze, "train_mon_pairs": mon, "train_X": X, "train_Z": Z}
logging.disable(logging.CRITICAL)
np.random.seed(0)
lr.learning_process(X, Z, dict(p, n_it=50), rng_mode=mode)  # warm
for _ in range(2):
    p["iter"] = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lr.learning_process(X, Z, p, rng_mode=mode)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{mode}: {steps / dt:.0f} steps/s, {dt / (steps / 25) * 1e6:.1f} us per "
          f"eval-to-eval cycle of 25 steps", flush=True)
p["iter"] = []
pr = cProfile.Profile()
torch.cuda.synchronize()
pr.enable()
lr.learning_process(X, Z, p, rng_mode=mode)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(35)
st.sort_stats("cumulative").print_stats(45)
