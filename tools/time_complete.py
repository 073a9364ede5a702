"""C5 complete-block gradient steps/s (bench.sgd_complete_steps_per_s), hinge and logistic
(GPU box).  Usage: time_complete.py [steps] [losses]"""
import json
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402

torch.cuda.set_device(0)
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
for loss in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["hinge"]):
    r = bench.sgd_complete_steps_per_s(bench.C5_N, bench.C5_N, 512, 256, steps, loss=loss)
    print(json.dumps(r), flush=True)
