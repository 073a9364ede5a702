"""Run one SGD configuration of bench.py (for rocprofv3 kernel traces)."""
import sys, pathlib, json
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch
import bench
cfg = {"c4": (9117, 702, 10, 100, 100, 25, 2000, 1),
       "c5": (1_000_000, 1_000_000, 512, 256, 100, 25, 300, 1),
       "c5b": (1_000_000, 1_000_000, 512, 256, 4096, 25, 50, 1),
       "c5full": (5_000_000, 5_000_000, 512, 256, 100, 25, 500, 1)}[sys.argv[1]]
torch.cuda.set_device(0)
if "perstep" in sys.argv[2:]:  # per-step launches instead of the persistent segment kernel
    import tuplewise.learning as lr
    lr.SEGMENT_KERNEL = False
print(json.dumps(bench.sgd_steps_per_s(*cfg)))
