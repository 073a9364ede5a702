"""Time the bench count launch (n=1e6/class, N=64 shards) for each libtuplewise variant built
by tools/build_count_variants.sh (GPU box).  Usage: count_variants.py tag [tag ...]"""
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
if len(sys.argv) > 2 and sys.argv[1] != "--one":
    for tag in sys.argv[1:]:  # one child process per variant (each loads its own library)
        subprocess.run([sys.executable, __file__, "--one", tag], check=True)
    sys.exit(0)
tag = sys.argv[-1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402
from tuplewise import _lib as L  # noqa: E402

if tag != "base":
    L.LIB_PATH = ROOT / "tools" / "variants" / f"libtuplewise_{tag}.so"
from tuplewise.device import ShardedSample  # noqa: E402

N = 64
for per in (15625, 16384):
    n = N * per
    g = torch.Generator(device="cuda").manual_seed(1)
    X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
    Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
    S = ShardedSample(X, Z, N, algo="pairs")
    S.repartition(1)
    pairs = N * per * per
    for R in (4, 8):
        L.call("tw_count_set_plan", R, 0)
        for _ in range(3):
            S.local_counts()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            c = S.local_counts()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(f"{tag:10s} shard {per} R={R}  {ms:.4f} ms  frac={pairs / ms / 1e-3 / 3.93216e13:.3f}"
              f"  sum={int(c.sum())}", flush=True)
