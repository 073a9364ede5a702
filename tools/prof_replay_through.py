"""One C4 replay learning_process run (2000 steps, no evaluation) at a given reshuffle_mod with
replay segments running through reshuffles (learning.REPLAY_THROUGH) or cut at each one —
the program rocprofv3 --kernel-trace --stats profiles to split the loop's device time by kernel
(VERDICT r03 item 3).  Usage: prof_replay_through.py MOD THROUGH(0|1) [STEPS]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import tuplewise.learning as lr
    mod, through = int(sys.argv[1]), bool(int(sys.argv[2]))
    lr.REPLAY_THROUGH = through
    t0 = time.perf_counter()
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
    r = bench.sgd_replay_steps_per_s(steps, mod, runs=1, audit=False)
    print(f"mod {mod} through {through}: {r['steps_per_s']:.0f} steps/s "
          f"({time.perf_counter() - t0:.2f} s with warm-up)", flush=True)


if __name__ == "__main__":
    main()
