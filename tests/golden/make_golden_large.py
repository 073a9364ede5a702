"""Large-n goldens: the REFERENCE run at the BASELINE sizes (SURVEY.md §8(c) "Large-n goldens").

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_large.py   (~3-4 min, ~12 GB RAM)

Runs /root/reference/estimation-experiment/main.py and learning-experiment/compute_stats.py
read-only (importlib, as make_golden.py does) on inputs regenerated from a committed seed:
`np.random.RandomState(seed).normal(loc, 1, n)` — so no multi-MB arrays are committed, only
the seed, the reference's value, the global-RNG probe drawn right after the call and the
SHA-256 of the arrays the call shuffled in place.  Output: golden_large.json (data only).

Cases (BASELINE.json configs):
  C2  est.Un(X, Z) at n = m = 1e5, one shard (main.py:29-31; a 10 GB bool temporary here),
      on Gaussian scores and on scores rounded to 2 decimals (ties: strict > counts them 0);
  C3  est.UnNT(X, Z, 64, 4, "prop-SWOR") at 1e6/class (main.py:76-79, 33-69),
      est.UnN(X, Z, 64, "SWOR") at 1e6/class (the binomial block sizes, main.py:50-52),
      cs.UnNBT(X, Z, 64, 1e6, 2, "prop-SWOR", kernel="AUC") at 1e6/class
      (compute_stats.py:119-123, 104-110, 37-42).
The GPU box never runs this script (the reference is absent there); tests/test_gpu_large_golden.py
regenerates the inputs and checks the drop-in against these numbers bit-for-bit.
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import pathlib
import sys
import time

import numpy as np

REF = pathlib.Path(os.environ.get("TW_REFERENCE", "/root/reference"))
OUT = pathlib.Path(__file__).resolve().parent


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


sys.path.insert(0, str(OUT))
from shapes import large_inputs as inputs  # noqa: E402  (the generator the GPU test uses too)

CASES = [
    {"name": "C2_est_Un_gauss", "call": "est.Un", "n": 100_000, "m": 100_000,
     "data_seed": 61, "loc_x": 0.5},
    {"name": "C2_est_Un_ties", "call": "est.Un", "n": 100_000, "m": 100_000,
     "data_seed": 62, "loc_x": 0.5, "round": 2},
    {"name": "C3_est_UnNT_propSWOR", "call": "est.UnNT", "n": 1_000_000, "m": 1_000_000,
     "data_seed": 63, "loc_x": 0.5, "N": 64, "T": 4, "sampling": "prop-SWOR", "rng_seed": 2063},
    {"name": "C3_est_UnN_SWOR", "call": "est.UnN", "n": 1_000_000, "m": 1_000_000,
     "data_seed": 64, "loc_x": 0.5, "N": 64, "sampling": "SWOR", "rng_seed": 2064},
    {"name": "C3_cs_UnNBT_AUC", "call": "cs.UnNBT", "n": 1_000_000, "m": 1_000_000,
     "data_seed": 65, "loc_x": 0.5, "N": 64, "B": 1_000_000, "T": 2, "sampling": "prop-SWOR",
     "rng_seed": 2065},
]


def main():
    sys.dont_write_bytecode = True
    est = _load("ref_est_main", REF / "estimation-experiment" / "main.py")
    cs = _load("ref_compute_stats", REF / "learning-experiment" / "compute_stats.py")
    out = []
    for spec in CASES:
        X, Z = inputs(spec)
        rec = dict(spec)
        rec["sha_X_in"], rec["sha_Z_in"] = sha(X), sha(Z)
        t0 = time.time()
        if spec["call"] == "est.Un":
            val = est.Un(X, Z)
        else:
            np.random.seed(spec["rng_seed"])
            if spec["call"] == "est.UnNT":
                val = est.UnNT(X, Z, spec["N"], spec["T"], spec["sampling"])
            elif spec["call"] == "est.UnN":
                val = est.UnN(X, Z, spec["N"], spec["sampling"])
            else:
                val = cs.UnNBT(X, Z, spec["N"], spec["B"], spec["T"], spec["sampling"],
                               kernel="AUC")
            rec["probe"] = int(np.random.randint(0, 2 ** 31 - 1))
            rec["sha_X_after"], rec["sha_Z_after"] = sha(X), sha(Z)
        rec["value"] = float(val)
        rec["value_hex"] = float(val).hex()
        rec["ref_seconds"] = round(time.time() - t0, 2)
        print(rec["name"], rec["value_hex"], rec["ref_seconds"], "s", flush=True)
        out.append(rec)
    meta = {"generator": "np.random.RandomState(data_seed).normal(loc_x, 1, n) then "
                         ".normal(0, 1, m); rounded to `round` decimals when given",
            "numpy": np.__version__, "cases": out}
    (OUT / "golden_large.json").write_text(json.dumps(meta, indent=1))
    print("wrote", OUT / "golden_large.json")


if __name__ == "__main__":
    main()
