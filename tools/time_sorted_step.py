"""UnN_many with the exact sorted count (algo='sorted', bench `sorted_count` shape: 1e6 scores
per class, 64 prop-SWOR shards), three ways: the K steps in one call with the partition kept as
destination-bucketed records between steps (tw_count_pairs_sorted_steps, the default), one
launch per step with the next repartition's gathers in the count threads
(tw_count_pairs_sorted_step), and the count and the permute kernel in turn.  Estimates and
final arrays must match.  GPU box."""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
import tuplewise  # noqa: E402,F401
from tuplewise.device import HipOps, ShardedSample  # noqa: E402


def _no_attr(self):
    raise AttributeError


class PerStep(HipOps):  # no records entry: one launch per step
    count_sorted_steps = property(_no_attr)


class TwoKernels(PerStep):  # neither: repartition, then count
    count_sorted_step = property(_no_attr)


torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(1)
n, N, K = 1_000_000, 64, 100
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
res = None
for rep in range(2):
    for name, ops in (("two kernels", TwoKernels), ("one launch per step", PerStep),
                      ("records", HipOps)):
        S = ShardedSample(X.clone(), Z.clone(), N, algo="sorted", ops=ops())
        S.UnN_many(range(30_000, 30_010))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        est = S.UnN_many(range(K))
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K
        res = res or (est, S.X.clone())
        same = res[0] == est and torch.equal(res[1], S.X)
        print(f"{name}: {dt * 1e3:.4f} ms/step, {N * (n // N) ** 2 / dt:.3e} logical pairs/s, "
              f"same estimates and arrays {same}", flush=True)
