"""A/B of the persistent segments' grid barrier (csrc/sgdseg.hip TW_SEG_BARRIER; VERDICT r03
item 6): C4 device-RNG steps/s (bench.sgd_steps_per_s, reshuffle_mod 25, 4000 steps) with the
default library (release arrival, relaxed spin + one acquire fence) and the A/B builds
(`make -C <pkg>/csrc ab-barrier`: 0 = relaxed, the round-3 barrier; 1 = acquire loads in the
spin), each in a fresh process, alternated."""
import json
import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
CODE = r'''
import json, sys
sys.path.insert(0, sys.argv[1])
import bench
r = bench.sgd_steps_per_s(9117, 702, 10, 100, 100, 25, 4000, 2)
print(json.dumps(r["steps_per_s"]))
'''
libs = {"default (release + fence)": None,
        "relaxed (round 3)": ROOT / "tools/variants/libtuplewise_seg0.so",
        "acquire in spin": ROOT / "tools/variants/libtuplewise_seg1.so"}
out = {k: [] for k in libs}
for rep in range(3):
    for k, lib in libs.items():
        env = dict(os.environ)
        if lib is not None:
            env["TW_LIB_PATH"] = str(lib)
        r = subprocess.run([sys.executable, "-c", CODE, str(ROOT)], env=env, capture_output=True,
                           text=True, timeout=300)
        if r.returncode != 0:
            print(k, "failed:", r.stderr[-1500:], flush=True)
            sys.exit(1)
        out[k].append(json.loads(r.stdout.strip().splitlines()[-1]))
        print(f"{k:28s} {out[k][-1]:10.0f} steps/s", flush=True)
print(json.dumps({k: sorted(v)[len(v) // 2] for k, v in out.items()}))
