"""The paper's estimation experiment (estimation-experiment/main.py:82-116) on the device.

For each epsilon: n_tries draws of Un, UnN, UnNT with the Bernoulli generators of
main.py:97-101 (n=5000, m=50, N=10, T=4, prop-SWOR), via estimation.replicate (bit-identical
to the reference loop).  Prints wall time and the variance ratios the paper plots; with
--cpu-tries also times the oracle's restatement of the same loop for a few tries.  Round 6: also
the HOST FLOOR of the same loop — the NumPy work the drop-in must do on the host to stay
bit-identical (the generators' binomial draws, and for UnN / UnNT the in-place
np.random.shuffle of X and Z per repartition, main.py:46-47) with no estimator at all — which
bounds what any device can save on this experiment.  Round 6, late: the floor again with the
drop-in's own native shuffles, and estimation.replicate's fixed-layout path (Un / prop-SWOR:
snapshot rows, broadcast offsets, row means instead of per-block Python).
"""
import argparse
import pathlib
import sys
import time

import numpy as np

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))

ap = argparse.ArgumentParser()
ap.add_argument("--tries", type=int, default=5000)
ap.add_argument("--cpu-tries", type=int, default=0)
a = ap.parse_args()
n, m, N, T = 5000, 50, 10, 4
eps = [0.00016, 0.0008, 0.004, 0.02, 0.1, 0.5]

if a.cpu_tries:
    from oracle import oracle as O
    e = eps[3]
    gx = lambda: 2 * np.random.binomial(1, 1 - e, n)
    gz = lambda: 2 * np.random.binomial(1, e, m) - 1
    np.random.seed(0)
    t0 = time.perf_counter()
    [O.est_Un(gx(), gz()) for _ in range(a.cpu_tries)]
    [O.est_UnN(gx(), gz(), N, "prop-SWOR") for _ in range(a.cpu_tries)]
    [O.est_UnNT(gx(), gz(), N, T, "prop-SWOR") for _ in range(a.cpu_tries)]
    dt = time.perf_counter() - t0
    print(f"cpu (reference loop restated): {dt / a.cpu_tries * 1e3:.3f} ms per try-triple, "
          f"extrapolated full experiment {dt / a.cpu_tries * 5000 * 6:.1f} s")

import tuplewise.estimation as est
np.random.seed(0)
t0 = time.perf_counter()
for e in eps:
    gx = lambda: 2 * np.random.binomial(1, 1 - e, n)
    gz = lambda: 2 * np.random.binomial(1, e, m) - 1
    v1 = est.replicate(est.Un, gx, gz, a.tries)
    v2 = est.replicate(est.UnN, gx, gz, a.tries, N, "prop-SWOR")
    v3 = est.replicate(est.UnNT, gx, gz, a.tries, N, T, "prop-SWOR")
    V = est.Var_Un(e, n, m)
    print(f"eps={e:<8} var/Var_Un: Un {np.var(v1) / V:.3f}  UnN {np.var(v2) / V:.3f}  "
          f"UnNT {np.var(v3) / V:.3f}", flush=True)
dt = time.perf_counter() - t0
print(f"device: full experiment ({len(eps)} eps x {a.tries} tries x 3 estimators) {dt:.2f} s")

# the host floor: the same RNG consumption with no estimator (generators; shuffles per UN call)
np.random.seed(0)
t0 = time.perf_counter()
for e in eps:
    gx = lambda: 2 * np.random.binomial(1, 1 - e, n)
    gz = lambda: 2 * np.random.binomial(1, e, m) - 1
    for shuffles in (0, 1, T):  # Un, UnN, UnNT
        for _ in range(a.tries):
            x, z = gx(), gz()
            for _ in range(shuffles):
                np.random.shuffle(x)
                np.random.shuffle(z)
fl = time.perf_counter() - t0
print(f"host floor (generators + the reference's in-place shuffles, no estimator): {fl:.2f} s "
      f"= {fl / dt:.2f} of the device run")
# the same with the drop-in's own in-place shuffles (numpy_rng.shuffle_pair: NumPy's legacy
# draws and swaps in native code, bit-identical): the floor the drop-in itself runs against
from tuplewise._blocks import shuffle_pair  # noqa: E402
np.random.seed(0)
t0 = time.perf_counter()
for e in eps:
    gx = lambda: 2 * np.random.binomial(1, 1 - e, n)
    gz = lambda: 2 * np.random.binomial(1, e, m) - 1
    for shuffles in (0, 1, T):
        for _ in range(a.tries):
            x, z = gx(), gz()
            for _ in range(shuffles):
                shuffle_pair(x, z)
fn = time.perf_counter() - t0
print(f"host floor with the drop-in's native shuffles: {fn:.2f} s = {fn / dt:.2f} of the device "
      f"run; the rest {dt - fn:.2f} s ({(dt - fn) / (len(eps) * a.tries * 3) * 1e6:.1f} us per "
      f"estimator call: snapshots, one batched count per ~16M scores, block values)")
