"""C4 replay (bit-exact NumPy draws) steps/s across the reference's reshuffle_mod sweep, with
replay segments running through their reshuffles (learning.REPLAY_THROUGH) and cut at each
reshuffle, interleaved in one process.  Also the host side alone: the
native draw worker's time per segment (learning.PIPE_STATS: the main thread's waits)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    import tuplewise.learning as lr
    mods = [int(m) for m in (sys.argv[1].split(",") if len(sys.argv) > 1
                             else "1,5,25,125,10000".split(","))]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    out = {"steps": steps, "mods": mods, "through": {}, "cut": {}, "wait_ms_per_step": {}}
    for mod in mods:
        for through in (True, False, True, False):
            lr.REPLAY_THROUGH = through
            r = bench.sgd_replay_steps_per_s(steps, mod, runs=3, audit=False)
            out["through" if through else "cut"].setdefault(str(mod), []).append(
                r["steps_per_s"])
        lr.REPLAY_THROUGH = True
        lr.PIPE_STATS = []
        t0 = time.perf_counter()
        bench.sgd_replay_steps_per_s(steps, mod, runs=1, audit=False)
        out["wait_ms_per_step"][str(mod)] = sum(lr.PIPE_STATS) / (steps + 50) * 1e3
        lr.PIPE_STATS = None
        print(f"mod {mod}: through {out['through'][str(mod)]} cut {out['cut'][str(mod)]} "
              f"({time.perf_counter() - t0:.1f} s)", flush=True)
    best = {m: max(v) for m, v in out["through"].items()}
    out["through_best"] = best
    out["through_spread"] = max(best.values()) / min(best.values())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
