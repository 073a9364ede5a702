"""The C5 learning step loop (d = 512, n = 1e7 rows, N = 256, B = 100, device RNG, replicated X;
bench.sgd_steps_per_s) for a rocprofv3 --kernel-trace run: per-kernel durations and the device
idle gap before each kernel (tools/trace_gaps.py) — where a step's time goes beyond the
gradient kernel."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
r = bench.sgd_steps_per_s(bench.C5_N, bench.C5_N, 512, 256, 100, 25, 300, 1)
print(f"C5 B=100: {r['steps_per_s']:.0f} steps/s, {r['ms_per_step'] * 1e3:.1f} us/step", flush=True)
