"""Host speed of the replay draws (numpy_rng: one C4 step = 2 x 100 randint calls of 100 draws,
kx = 91, kz = 7) per SIMD level, in fresh processes (TW_NP_RNG_ISA / TW_NP_RNG_SCALAR are read
once per process).  Run on the GPU box: its host CPU is what the replay loop runs on."""
import os
import subprocess
import sys

CODE = r'''
import sys, time; sys.path.insert(0, ".")
import numpy as np
from tuplewise.numpy_rng import Session
np.random.seed(0)
s = Session()
out = np.empty((25, 2, 100, 100), np.int64)
best = 1e9
for _ in range(30):
    t0 = time.perf_counter(); s.pairs_steps(25, 100, 91, 7, 100, out); best = min(best, time.perf_counter() - t0)
print("%.2f us/step" % (best / 25 * 1e6))
o16 = np.empty((25, 2, 100, 100), np.uint16)
best = 1e9
for _ in range(30):
    t0 = time.perf_counter(); s.pairs_steps_u16(25, 100, 91, 7, 100, o16); best = min(best, time.perf_counter() - t0)
print("uint16 %.2f us/step" % (best / 25 * 1e6))
o8 = np.empty((25, 2, 100, 100), np.uint8)
best = 1e9
for _ in range(30):
    t0 = time.perf_counter(); s.pairs_steps_u8(25, 100, 91, 7, 100, o8); best = min(best, time.perf_counter() - t0)
print("uint8 %.2f us/step" % (best / 25 * 1e6))
# one reshuffle's SWR_divide rows at C4 (100 calls of 91 on [0, 9117), 100 of 7 on [0, 702))
lo = np.zeros(200, np.int64); hi = np.array([9117] * 100 + [702] * 100, np.int64)
cnt = np.array([91] * 100 + [7] * 100, np.int64); rows = np.empty(9800, np.int64)
best = 1e9
for _ in range(300):
    t0 = time.perf_counter(); s.randint_flat(lo, hi, cnt, out=rows); best = min(best, time.perf_counter() - t0)
print("SWR rows %.2f us/reshuffle (incl. the Python call)" % (best * 1e6))
from tuplewise import _lib as L
r16 = np.empty(9800, np.uint16); f = L.lib().tw_np_randint_batch_u16
best = 1e9
for _ in range(300):
    t0 = time.perf_counter(); f(s._key, s._pos, 200, lo.ctypes.data, hi.ctypes.data, cnt.ctypes.data, r16.ctypes.data); best = min(best, time.perf_counter() - t0)
print("SWR rows uint16 %.2f us/reshuffle (incl. the ctypes call)" % (best * 1e6))
'''
for label, env in (("widest", {}), ("avx2", {"TW_NP_RNG_ISA": "avx2"}),
                   ("portable", {"TW_NP_RNG_SCALAR": "1"})):
    r = subprocess.run([sys.executable, "-c", CODE], env=dict(os.environ, **env),
                       capture_output=True, text=True, timeout=120)
    print(label, r.stdout.strip() or r.stderr[-300:], flush=True)
