"""Clock warm-up probe for bench.py's settle phase (GPU box): times the one-launch UnN step
(count_step, HIP events) over successive K-step runs from a cold start, showing the first ~10 ms
of load run ~3 % slower."""
import sys, time, pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch, numpy as np
import tuplewise  # noqa: F401
from tuplewise.device import ShardedSample


def main():
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda").manual_seed(1)
    n, N = 1_000_000, 64
    X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
    Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
    S = ShardedSample(X, Z, N, algo="pairs")
    ops = S.ops
    orig = ops.count_step
    ev = []
    def timed(*a, **k):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); o = orig(*a, **k); e1.record(); ev.append((e0, e1)); return o
    def run(K, label):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        S.UnN_many(range(100, 100 + K)); torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        km = np.mean([a.elapsed_time(b) for a, b in ev]) if ev else float('nan')
        print(f"{label}: {dt/K*1e3:.4f} ms/step, kernel {km:.4f} ms", flush=True)
        ev.clear()
    run(20, "cold, no events")
    ops.count_step = timed
    run(20, "events")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        S.UnN_many(range(5)); torch.cuda.synchronize()
    ev.clear()
    run(20, "after settle, events")
    ops.count_step = orig
    run(20, "after settle, no events")
    ops.count_step = timed
    run(100, "after settle, events, K=100")


if __name__ == "__main__":
    main()
