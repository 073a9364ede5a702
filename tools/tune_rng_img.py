"""Time the device-RNG image count (k_count_rng_img, bench `incomplete`) per Philox unroll
(tw_count_rng_img_set_unroll 1/2/4) on the bench workload: 1e6 scores per class, 64 prop-SWOR
shards, B = 1e6 drawn pairs per shard; counts must not depend on the unroll.  GPU box."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
import tuplewise  # noqa: E402,F401
from tuplewise import _lib as L  # noqa: E402
from tuplewise.device import ShardedSample  # noqa: E402

torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(1)
n, N, B = 1_000_000, 64, 1_000_000
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
S = ShardedSample(X, Z, N, algo="pairs")
ref = None
for qu in [int(a) for a in sys.argv[1:]] or [1, 2, 4]:
    L.call("tw_count_rng_img_set_unroll", qu)
    for _ in range(3):
        c = S._count_rng(B, 7).clone()
    torch.cuda.synchronize()
    if ref is None:
        ref = c
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(20):
        S._count_rng(B, i)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"unroll {qu}: {ms:.4f} ms/launch, {N * B / ms / 1e-3:.3e} pairs/s, "
          f"same counts {bool(torch.equal(c, ref))}", flush=True)
