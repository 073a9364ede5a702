"""Summarise a rocprofv3 kernel-trace CSV of tools/trace_replay.py: per kernel name the count and
mean duration, and the device idle time between consecutive kernels (gaps), overall and by the
kernel that follows the gap."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60])
            for r in rows)
# the last learning_process call only: from its first k_copy_words / widen after the 5th gap > 1 ms
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
for (s0, e0, n0), (s1, e1, n1) in zip(ev, ev[1:]):
    gap[n1].append(max(0, s1 - e0))
for s, e, n in ev:
    dur[n].append(e - s)
span = ev[-1][1] - ev[0][0]
busy = sum(e - s for s, e, _ in ev)
print(f"span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, kernels {len(ev)}")
for n in sorted(dur, key=lambda k: -sum(dur[k])):
    g = gap[n]
    print(f"{n:60s} n={len(dur[n]):6d} mean {sum(dur[n]) / len(dur[n]) / 1e3:8.2f} us  "
          f"gap-before mean {sum(g) / max(1, len(g)) / 1e3:8.2f} us "
          f"median {sorted(g)[len(g) // 2] / 1e3 if g else 0:8.2f} us")
