"""Time evaluation_step (make_exps.py:143-190) at shuttle-like shapes (C4)."""
import sys, pathlib, time, logging
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np, torch
import tuplewise.learning as lr
rng = np.random.RandomState(0)
Xt = np.hstack([rng.normal(size=(9117, 9)), np.ones((9117, 1))])
Zt = np.hstack([rng.normal(0.5, 1, size=(702, 9)), np.ones((702, 1))])
Xe = np.hstack([rng.normal(size=(2279, 9)), np.ones((2279, 1))])
Ze = np.hstack([rng.normal(0.5, 1, size=(175, 9)), np.ones((175, 1))])
mon = list(zip(list(rng.randint(0, 9117, 450000)), list(rng.randint(0, 702, 450000))))
p = {"margin": 1, "reg": 0.05, "train_X": Xt, "train_Z": Zt, "test_X": Xe, "test_Z": Ze,
     "train_mon_pairs": mon}
w = rng.normal(size=(10, 1))
logging.disable(logging.CRITICAL)
lr.evaluation_step(0, None, None, w, p)  # warm: caches device copies + the pair array
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(20):
    lr.evaluation_step(i, None, None, w, p)
torch.cuda.synchronize()
print(f"evaluation_step: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms per call "
      f"(reference: 158 ms, SURVEY.md §3)")
wd = torch.from_numpy(w.reshape(-1)).cuda()
lr.evaluation_step(0, None, None, w, p, _w_dev=wd)  # warm: captures the evaluation graph
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(20):
    lr.evaluation_step(i, None, None, w, p, _w_dev=wd)
torch.cuda.synchronize()
print(f"evaluation_step with w resident (the learning loop's call): "
      f"{(time.perf_counter() - t0) / 20 * 1e3:.3f} ms per call")
