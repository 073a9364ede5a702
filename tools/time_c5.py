"""C5 SGD steps/s (bench.sgd_steps_per_s at d=512, n=1e7, N=256, B=100 and 4096) on their own
(GPU box)."""
import json
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402

torch.cuda.set_device(0)
for _ in range(2):
    a = bench.sgd_steps_per_s(bench.C5_N, bench.C5_N, 512, 256, 100, 25, 500, 2)
    b = bench.sgd_steps_per_s(bench.C5_N, bench.C5_N, 512, 256, 4096, 25, 100, 1)
    print(json.dumps({"C5_B100_steps_per_s": a["steps_per_s"],
                      "C5_B4096_steps_per_s": b["steps_per_s"]}), flush=True)

# A/B of the wide kernels (tw_hinge_set_variant: 0 streaming, 2 burst-pipelined)
from tuplewise import _lib as L  # noqa: E402
for v in (0, 2, 0, 2):
    L.call("tw_hinge_set_variant", v)
    a = bench.sgd_steps_per_s(bench.C5_N, bench.C5_N, 512, 256, 100, 25, 500, 2)
    b = bench.sgd_steps_per_s(bench.C5_N, bench.C5_N, 512, 256, 4096, 25, 100, 1)
    print(json.dumps({"variant": v, "C5_B100_steps_per_s": a["steps_per_s"],
                      "C5_B4096_steps_per_s": b["steps_per_s"]}), flush=True)
L.call("tw_hinge_set_variant", 0)
