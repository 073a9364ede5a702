"""Time the one-launch UnN step (tw_count_pairs_step) against the plain count launch, for
several placements of the spare blocks that carry the next repartition (bench workload:
1e6 scores per class, 64 prop-SWOR shards).  Run on the GPU box."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch
import tuplewise  # noqa: F401
from tuplewise import _lib as L
from tuplewise.device import ShardedSample

torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(1)
n, N = 1_000_000, 64
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
S = ShardedSample(X, Z, N, algo="pairs")
ops = S.ops


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


out = torch.zeros(N, dtype=torch.int64, device="cuda")
out_n = torch.zeros(N, dtype=torch.int64, device="cuda")
Xn, Zn = torch.empty_like(X), torch.empty_like(Z)
args = (S.X, S.x_off_dev, S.Z, S.z_off_dev, N, S.max_nx, S.max_nz, S.dtype, S.pred)
print(f"count only (tw_count_pairs incl. memset): {timeit(lambda: ops.count(*args)):.4f} ms")
print(f"count_step without next: "
      f"{timeit(lambda: ops.count_step(*args, out, None, 0, None, 0, None)):.4f} ms")
print(f"permute_pair alone: {timeit(lambda: ops.permute_pair(S.X, 3, S.Z, 4)):.4f} ms")
plans = [(0, 0, 0), (0, 0, 1), (256, 0, 1), (512, 0, 1), (768, 0, 1), (1024, 0, 1),
         (1536, 0, 1), (2048, 0, 1), (4096, 0, 1)]
if len(sys.argv) > 1:
    plans = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]]
for blocks, every, tail in plans:
    L.call("tw_count_step_set_plan", blocks, every, tail)
    t = timeit(lambda: ops.count_step(*args, out, Xn, 3, Zn, 4, out_n))
    print(f"step blocks={blocks:5d} every={every:4d} tail={tail}: {t:.4f} ms")
L.call("tw_count_step_set_plan", 0, 0, 0)
