"""bench.learning_end_to_end (C4 learning_process with an evaluation every 25 steps) for a
rocprofv3 --kernel-trace run; argument: "replay" or "device" (default device)."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import bench  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "device"
print(bench.learning_end_to_end(2000, mode)["steps_per_s"], flush=True)
