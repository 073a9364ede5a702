"""Where a replay-mode learning_process call's time goes at the C4 shape (bench
sgd_replay_steps_per_s: N = 100, B = 100, reshuffle every 25 steps, no evaluation), GPU box:
  full      : the call as the bench times it (median of 5)
  short     : the same call with n_it = 25 (one segment: the per-call fixed cost)
  no_draws  : the draw worker's native calls replaced by no-ops (buffers keep earlier draws):
              the main thread + device bound
  draws     : the native draws alone for the same segments, one thread
  device    : the segment graphs alone, replayed back to back on one resident buffer
"""
import logging
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import tuplewise.learning as lr  # noqa: E402
from tuplewise.numpy_rng import Session  # noqa: E402

rng = np.random.RandomState(3)
X = np.hstack([rng.normal(size=(9117, 9)), np.ones((9117, 1))])
Z = np.hstack([rng.normal(0.5, 1, size=(702, 9)), np.ones((702, 1))])
STEPS = 2000
p = {"n_it": STEPS, "margin": 1, "N": 100, "B": 100, "reshuffle_mod": 25, "reg": 0.05,
     "learning_rate": 0.01, "eval_mod": 10 ** 9, "w_init": rng.normal(size=(10, 1)),
     "test_X": X[:10], "test_Z": Z[:10], "train_mon_pairs": [(0, 0)], "train_X": X,
     "train_Z": Z}
logging.disable(logging.CRITICAL)


def timed(fn, reps=5):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts


np.random.seed(0)
lr.learning_process(X, Z, dict(p, n_it=50))
full, ts = timed(lambda: lr.learning_process(X, Z, p))
print(f"full      {STEPS / full:9.0f} steps/s  {full * 1e3:7.2f} ms  runs "
      + " ".join(f"{STEPS / t:.0f}" for t in ts), flush=True)
lr.PIPE_STATS = []
lr.learning_process(X, Z, p)
w = np.array(lr.PIPE_STATS) * 1e6
lr.PIPE_STATS = None
print(f"waits     main thread waited for the draws: {w.sum() / 1e3:.2f} ms over {len(w)} segments "
      f"(median {np.median(w):.1f} us, max {w.max():.1f} us)", flush=True)
eg, ts = timed(lambda: lr.learning_process(X, Z, p, graphs=False))
print(f"eager     {STEPS / eg:9.0f} steps/s  {eg * 1e3:7.2f} ms  runs "
      + " ".join(f"{STEPS / t:.0f}" for t in ts) + "  (graphs=False: the segment kernels "
      "launched eagerly)", flush=True)
lr.FUSED_SHIP = False
fs, ts = timed(lambda: lr.learning_process(X, Z, p))
print(f"unfused   {STEPS / fs:9.0f} steps/s  {fs * 1e3:7.2f} ms  runs "
      + " ".join(f"{STEPS / t:.0f}" for t in ts) + "  (FUSED_SHIP off: widen + 2 row copies, "
      "eager before the graph)", flush=True)
lr.FUSED_SHIP = True
lr.NATIVE_DRAWS = False
nd, ts = timed(lambda: lr.learning_process(X, Z, p))
print(f"pyworker  {STEPS / nd:9.0f} steps/s  {nd * 1e3:7.2f} ms  runs "
      + " ".join(f"{STEPS / t:.0f}" for t in ts) + "  (NATIVE_DRAWS off: Python worker thread)",
      flush=True)
lr.NATIVE_DRAWS = True
lr.NARROW_DRAWS_U8 = False
u16, ts = timed(lambda: lr.learning_process(X, Z, p))
print(f"u16       {STEPS / u16:9.0f} steps/s  {u16 * 1e3:7.2f} ms  runs "
      + " ".join(f"{STEPS / t:.0f}" for t in ts) + "  (NARROW_DRAWS_U8 off)", flush=True)
lr.NARROW_DRAWS_U8 = True
lr.ENGINE_CACHE = False
off, ts = timed(lambda: lr.learning_process(X, Z, p))
print(f"fresh     {STEPS / off:9.0f} steps/s  {off * 1e3:7.2f} ms  runs "
      + " ".join(f"{STEPS / t:.0f}" for t in ts) + "  (ENGINE_CACHE off: a new engine per call)",
      flush=True)
one, _ = timed(lambda: lr.learning_process(X, Z, dict(p, n_it=1)))
print(f"fresh one n_it=1:  {one * 1e3:7.3f} ms per call", flush=True)
lr.ENGINE_CACHE = True
lr.learning_process(X, Z, p)
short, _ = timed(lambda: lr.learning_process(X, Z, dict(p, n_it=25)))
print(f"short     n_it=25: {short * 1e3:7.3f} ms per call", flush=True)
one, _ = timed(lambda: lr.learning_process(X, Z, dict(p, n_it=1)))
print(f"one       n_it=1:  {one * 1e3:7.3f} ms per call", flush=True)

# main thread + device: the worker's native draws become no-ops after a first fill
orig_fill, orig_swr = lr._ReplayDraws.fill_segment, lr._ReplayDraws.swr_rows_staged


def fill_noop(self, k, S):
    self._seg_buffers(3)
    if not getattr(self, "_filled", None):
        self._filled = set()
    if k not in self._filled:
        self._filled.add(k)
        return orig_fill(self, k, S)
    return k


lr._ReplayDraws.fill_segment = fill_noop
nod, ts = timed(lambda: lr.learning_process(X, Z, p))
lr._ReplayDraws.fill_segment = orig_fill
print(f"no_draws  {STEPS / nod:9.0f} steps/s  {nod * 1e3:7.2f} ms  runs "
      + " ".join(f"{STEPS / t:.0f}" for t in ts), flush=True)

# the draws alone: SWR rows + 25-step pair segments, as the worker makes them
s = Session()
N, kx, kz, B = 100, 91, 7, 100
o16 = np.empty((25, 2, N, B), np.uint16)
d = lr._ReplayDraws(N, kx, kz, B)
args = d._swr_setup(9117, 702)
rows = np.empty(N * kx + N * kz, np.int64)
t0 = time.perf_counter()
for _ in range(STEPS // 25):
    s.randint_flat(*args, out=rows)
    s.pairs_steps_u16(25, N, kx, kz, B, o16)
dr = time.perf_counter() - t0
print(f"draws     {STEPS / dr:9.0f} steps/s  {dr / STEPS * 1e6:6.2f} us/step (one thread)",
      flush=True)

# device only: one engine, segment graphs replayed back to back on one buffer
eng = lr.SGDEngine(X, Z, p["w_init"], N, B, 1, 0.05, 0.01, "momentum")
dd = lr._ReplayDraws(N, eng.kx, eng.kz, B)
rx, rz = dd.swr_rows(9117, 702)
eng.set_shards(rx, rz)
k = dd.fill_segment(0, 25)
buf = dd.ship_segment(k, 25)
for _ in range(3):
    eng.run_replay_segment(buf, 25, True, k)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(STEPS // 25):
    eng.run_replay_segment(buf, 25, True, k)
torch.cuda.synchronize()
dv = time.perf_counter() - t0
print(f"device    {STEPS / dv:9.0f} steps/s  {dv / STEPS * 1e6:6.2f} us/step (graphs only)",
      flush=True)
t0 = time.perf_counter()
for _ in range(STEPS // 25):
    eng.set_shards(rx, rz)
    eng.run_replay_segment(buf, 25, True, k)
torch.cuda.synchronize()
dv2 = time.perf_counter() - t0
print(f"dev+rows  {STEPS / dv2:9.0f} steps/s  {dv2 / STEPS * 1e6:6.2f} us/step "
      "(set_shards each segment)", flush=True)
