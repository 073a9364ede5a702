"""C4 SGD steps/s (bench.sgd_steps_per_s, sgd_replay_steps_per_s) on their own (GPU box),
with the persistent narrow segment kernel (learning.NARROW_SEGMENT) and without it."""
import json
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402

import tuplewise.learning as lr  # noqa: E402

torch.cuda.set_device(0)
for seg in (True, False, True):
    lr.NARROW_SEGMENT = seg
    a = bench.sgd_steps_per_s(9117, 702, 10, 100, 100, 25, 4000, 2)
    b = bench.sgd_replay_steps_per_s(2000)
    print(json.dumps({"narrow_segment": seg, "device_steps_per_s": a["steps_per_s"],
                      "replay_steps_per_s": b["steps_per_s"]}), flush=True)
lr.NARROW_SEGMENT = True
