"""Host timeline of the bit-exact drop-in est.UnNT(X, Z, 64, 4, "prop-SWOR") at n = 1e6/class
(VERDICT r04 item 5): the marks _blocks._run_un_repeated_device leaves (its DROPIN_MARKS hook),
per call, in ms from the call's start; round 5: each setting of the pipelining switches
(_blocks.EARLY_COUNTS, STREAM_LAST_SHUFFLE, THREADED_LAUNCHES) in turn, median call time per setting.
    python tools/time_dropin_parts.py [calls]"""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np
import torch

import tuplewise.estimation as est
from tuplewise import _blocks as Bk

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 6
rng = np.random.RandomState(0)
X, Z = rng.normal(0.5, 1, 1_000_000), rng.normal(0, 1, 1_000_000)
np.random.seed(1)
est.UnNT(X, Z, 64, 4, "prop-SWOR")  # warm
torch.cuda.synchronize()
for early, pieces, thr in ((False, 0, False), (False, 4, False), (False, 0, True),
                          (False, 4, True), (True, 4, True), (True, 8, True), (True, 0, True)):
    Bk.EARLY_COUNTS, Bk.STREAM_LAST_SHUFFLE, Bk.THREADED_LAUNCHES = early, pieces, thr
    est.UnNT(X, Z, 64, 4, "prop-SWOR")  # warm this setting
    ts = []
    for c in range(calls):
        Bk.DROPIN_MARKS = []
        t0 = time.perf_counter()
        est.UnNT(X, Z, 64, 4, "prop-SWOR")
        t1 = time.perf_counter()
        marks = Bk.DROPIN_MARKS
        Bk.DROPIN_MARKS = None
        ts.append((t1 - t0) * 1e3)
        if c < 2:
            print(f"  early={early} pieces={pieces} threaded={thr} call {c}: {ts[-1]:.2f} ms | "
                  + ", ".join(f"{lab} {(tm - t0) * 1e3:.2f}" for lab, tm in marks), flush=True)
    print(f"early={early} pieces={pieces} threaded={thr}: median {np.median(ts):.2f} ms/call, min "
          f"{min(ts):.2f} over {calls} calls", flush=True)
