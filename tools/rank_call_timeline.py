"""Kernel timeline of the chain probe's rank calls (tools/chain_probe.py under rocprofv3
--kernel-trace): the trace cut into calls at each ranking or, carried, at each k_chain_zero_heads (the
first kernel of an over-ranks emission), each call's kernels with their start offsets and durations, and per
kernel the median duration over the calls without a ranking (the carried calls) — what the
probe's HIP-event parts time beside what the device spent inside each kernel; the difference is
launch and hand-off latency.
Run on the GPU box, e.g. (only G = 8, K = 4):
    TW_PROBE_G=8 rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- \
        python3 tools/chain_probe.py 4
    python3 tools/rank_call_timeline.py TRACE.csv [OUT.log]"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
short = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "").replace("tw::", "")
calls, cur = [], None
for r in rows:
    name = short(r)
    # a call starts at its ranking (k_rank_sample_*) or, carried, at its zero_heads
    if "k_rank_sample" in name or ("k_chain_zero_heads" in name and (
            cur is None or any("k_chain_zero_heads" in n for n, _, _ in cur))):
        cur = []
        calls.append(cur)
    if cur is not None:
        cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
out = []
per = {}
calls = [c for c in calls if any("k_chain_zero_heads" in n for n, _, _ in c)]  # over ranks
for i, c in enumerate(calls):
    t0 = c[0][1]
    ranked = any("rank" in n for n, _, _ in c)
    span = (max(e for _, _, e in c) - t0) / 1e3
    out.append(f"call {i}: {'first' if ranked else 'carried'} span {span:.1f} us: " + ", ".join(
        f"{n[:28]}@{(s - t0) / 1e3:.1f}+{(e - s) / 1e3:.1f}" for n, s, e in c))
    if not ranked:
        for n, s, e in c:
            per.setdefault(n, []).append((e - s) / 1e3)
out.append("carried calls, median device time per kernel (us): " + ", ".join(
    f"{n} {statistics.median(v):.1f} (x{len(v)})" for n, v in per.items()))
text = "\n".join(out)
print(text)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(text + "\n")
