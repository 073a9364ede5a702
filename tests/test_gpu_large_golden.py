"""The drop-in against REFERENCE runs at the BASELINE sizes (SURVEY.md §8(c) "Large-n goldens").

tests/golden/golden_large.json holds what /root/reference computed here on seeded inputs
(tests/golden/make_golden_large.py): est.Un at n = m = 1e5 (configs[1]), est.UnNT(X, Z, 64, 4,
"prop-SWOR") and est.UnN(X, Z, 64, "SWOR") at 1e6/class and cs.UnNBT(X, Z, 64, 1e6, 2,
"prop-SWOR", kernel="AUC") (configs[2]).  Each test regenerates the inputs from the committed
seed, runs the package's drop-in on host arrays exactly as main.py / compute_stats.py callers
do, and compares bit-for-bit: the estimate, the global-RNG probe drawn after the call and the
SHA-256 of the arrays the call shuffles in place.
"""
import hashlib
import json
import pathlib
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = pathlib.Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(HERE))
from shapes import large_inputs  # noqa: E402

CASES = {c["name"]: c for c in json.loads((HERE / "golden_large.json").read_text())["cases"]}


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", sorted(CASES))
def test_drop_in_matches_reference_run(gpu, name):
    import tuplewise.compute_stats as cs
    import tuplewise.estimation as est
    spec = CASES[name]
    X, Z = large_inputs(spec)
    assert _sha(X) == spec["sha_X_in"] and _sha(Z) == spec["sha_Z_in"], "input generator drifted"
    if spec["call"] == "est.Un":
        got = est.Un(X, Z)
    else:
        np.random.seed(spec["rng_seed"])
        if spec["call"] == "est.UnNT":
            got = est.UnNT(X, Z, spec["N"], spec["T"], spec["sampling"])
        elif spec["call"] == "est.UnN":
            got = est.UnN(X, Z, spec["N"], spec["sampling"])
        else:
            got = cs.UnNBT(X, Z, spec["N"], spec["B"], spec["T"], spec["sampling"],
                           kernel="AUC")
        assert int(np.random.randint(0, 2 ** 31 - 1)) == spec["probe"], "RNG consumption"
        assert _sha(X) == spec["sha_X_after"] and _sha(Z) == spec["sha_Z_after"], "shuffles"
    assert float(got).hex() == spec["value_hex"], (name, float(got), spec["value"])
