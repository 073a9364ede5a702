"""Time the device-RNG incomplete count (bench shape: n=1e6/class, N=64, B=1e6 per shard) for
each libtuplewise variant (tools/build_count_variants.sh), ranked and plain.  GPU box."""
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
if len(sys.argv) > 2 and sys.argv[1] != "--one":
    for tag in sys.argv[1:]:
        subprocess.run([sys.executable, __file__, "--one", tag], check=True)
    sys.exit(0)
tag = sys.argv[-1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402
from tuplewise import _lib as L  # noqa: E402

if tag != "base":
    L.LIB_PATH = ROOT / "tools" / "variants" / f"libtuplewise_{tag}.so"
from tuplewise.device import ShardedSample  # noqa: E402

n, N, B = 1_000_000, 64, 1_000_000
g = torch.Generator(device="cuda").manual_seed(1)
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
S = ShardedSample(X, Z, N, algo="pairs")
S.repartition(1)
import os  # noqa: E402

caps = [int(c) for c in os.environ.get("CAPS", "4096").split(",")]
# (ranked, chunk cap, codes by bucket)
for ranked, cap, bucket in ([(True, c, 0) for c in caps] + [(True, 4096, 1)] +
                            [(False, 4096, 1)]):
    L.call("tw_count_sorted_set_chunk", cap)
    L.call("tw_count_rng_set_codes", bucket)
    kw = dict(max_nx=S.max_nx, max_nz=S.max_nz) if ranked else {}
    f = lambda i: S.ops.count_rng(S.X, S.x_off_dev, S.Z, S.z_off_dev, N, B, i, 0, S.dtype,
                                  S.pred, **kw)
    for i in range(3):
        f(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(20):
        c = f(i)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"{tag:10s} {'ranked' if ranked else 'plain ':6s} cap={cap:5d} bucket={bucket} "
          f"{ms:.4f} ms  "
          f"{N * B / ms / 1e-3:.3e} pairs/s  sum={int(c.sum())}", flush=True)
L.call("tw_count_sorted_set_chunk", 4096)
