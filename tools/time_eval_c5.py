"""evaluation_step (make_exps.py:143-190) at a C5-like scale on the device (GPU box): d = 512,
train 1e6 + 1e6 rows with 450k monitor pairs, test 1e6 + 1e6 rows (the complete test surrogate
and AUC are 1e12 pairs each).  Prints ms per call and the share of each device statistic."""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import tuplewise  # noqa: E402,F401
import tuplewise.learning as lr  # noqa: E402
from tuplewise import _engine as E, _lib as L  # noqa: E402

n_tr = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
n_te = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
d = 512
g = torch.Generator(device="cuda").manual_seed(9)
trX = torch.randn((n_tr, d), dtype=torch.float64, device="cuda", generator=g) + 0.02
trZ = torch.randn((n_tr, d), dtype=torch.float64, device="cuda", generator=g)
teX = torch.randn((n_te, d), dtype=torch.float64, device="cuda", generator=g) + 0.02
teZ = torch.randn((n_te, d), dtype=torch.float64, device="cuda", generator=g)
rs = np.random.RandomState(1)
mon = list(zip(rs.randint(0, n_tr, 450_000), rs.randint(0, n_tr, 450_000)))
w = np.random.RandomState(2).normal(0, 0.05, (d, 1))
wd = torch.from_numpy(w.reshape(-1)).cuda()
p = {"margin": 1.0, "reg": 0.01, "train_X": trX, "train_Z": trZ, "train_mon_pairs": mon,
     "test_X": teX, "test_Z": teZ}
lr.evaluation_step(0, None, None, w, p, _w_dev=wd)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(3):
    lr.evaluation_step(i, None, None, w, p, _w_dev=wd)
torch.cuda.synchronize()
print(f"evaluation_step: {(time.perf_counter() - t0) / 3 * 1e3:.2f} ms/call "
      f"(tc {p['tc_AUC'][-1]:.6f}, tr {p['tr_AUC'][-1]:.6f})", flush=True)
# the parts
sxt, szt = lr._scores(teX, wd), lr._scores(teZ, wd)
xo, zo, xod, zod = lr._offsets(n_te, n_te)
sh = E.Shards(sxt, xo, szt, zo, L.TW_F64)
sh._x_off_dev, sh._z_off_dev = xod, zod
for name, fn in (("test GEMVs", lambda: (lr._scores(teX, wd), lr._scores(teZ, wd))),
                 ("test hinge (all pairs)", lambda: E.pair_sum_complete_dev(sh, 2, 1.0, "pairs")),
                 ("test hinge (sorted)", lambda: E.pair_sum_complete_dev(sh, 2, 1.0, "sorted")),
                 ("test AUC count", lambda: E.count_launch(
                     sxt, xod, szt, zod, 1, n_te, n_te, L.TW_F64, L.TW_PRED_GT,
                     E.pick_algo("auto", n_te, n_te, "gt")))):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    val = f" = {r[0].item():.17g}" if "hinge" in name else ""
    print(f"  {name}: {dt * 1e3:.2f} ms{val}", flush=True)
