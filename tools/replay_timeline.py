"""Timeline of the LAST learning_process call in a rocprofv3 kernel-trace CSV of
tools/prof_replay_through.py: per replay segment, the device idle gap before its upload, the
upload, the segment kernel and the small launches after it — where a run's wall time goes
beyond kernel time.
    python3 tools/replay_timeline.py DIR/run_kernel_trace.csv [SEGMENTS]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
seg_idx = [i for i, e in enumerate(ev) if "k_sgd_segment_narrow" in e[2]]
# the last call: its segments follow the largest device gap before a ship in the trace's tail
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 12
first = seg_idx[-n_last]
# the call's first kernel: walk back to the upload before the first segment
start = first
while start > 0 and "k_ship" not in ev[start][2]:
    start -= 1
tot_gap = tot_busy = 0
prev_end = ev[start][0]
print(f"{'kernel':34s} {'gap_us':>8s} {'dur_us':>9s}")
for s, e, n in ev[start:]:
    name = n.split("(")[0].replace("void ", "").replace("tw::", "")[:34]
    gap = max(0, s - prev_end)
    tot_gap += gap
    tot_busy += e - s
    print(f"{name:34s} {gap / 1e3:8.2f} {(e - s) / 1e3:9.2f}")
    prev_end = max(prev_end, e)
print(f"busy {tot_busy / 1e3:.1f} us, idle {tot_gap / 1e3:.1f} us, "
      f"span {(prev_end - ev[start][0]) / 1e3:.1f} us")
