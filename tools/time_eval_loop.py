"""learning_process at the C4 shape WITH evaluations every 25 steps (bench.learning_end_to_end),
device RNG and replay, with the evaluations deferred (learning.DEFER_EVALS: device part
enqueued, host part once the statistics are back) and synchronous, alternating (GPU box)."""
import json
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
import tuplewise.learning as lr  # noqa: E402

torch.cuda.set_device(0)
for rep in range(2):
    for defer in (False, True):
        lr.DEFER_EVALS = defer
        a = bench.learning_end_to_end(2000, "device")["runs_steps_per_s"]
        b = bench.learning_end_to_end(2000, "replay")["runs_steps_per_s"]
        print(json.dumps({"defer": defer, "device": [round(v) for v in a],
                          "replay": [round(v) for v in b]}), flush=True)
lr.DEFER_EVALS = True
