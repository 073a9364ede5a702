"""Drop-in replacement for the estimator functions of estimation-experiment/main.py.

Un, UN, UnN, UnNT keep the reference's names, signatures, in-place shuffling and RNG order
(estimation-experiment/main.py:29-79); the pair counts run in libtuplewise.so.  The closed-form
moments of the Bernoulli experiment (main.py:10-27, :103-104) are pure formulas and are kept
here verbatim in meaning, since the statistical tests use them as known answers.

Extension (BASELINE.json): ``Un(X, Z, tie_mode="half")`` scores ties 1/2.  The default
"strict" is the reference semantics (ties score 0).
"""
from __future__ import annotations

import numpy as np

from . import _blocks as Bk


def p(e):
    return e


def q(e):
    return 1 - e


def sigma_1(e):
    return (p(e) ** 2) * q(e) * (1 - q(e))


def sigma_2(e):
    return ((1 - q(e)) ** 2) * p(e) * (1 - p(e))


def sigma_0(e):
    return p(e) * q(e) * (1 - p(e)) * (1 - q(e))


def Mean_Un(e):
    return q(e) + (1 - q(e)) * (1 - p(e))


def Var_Un(e, n, m):
    """main.py:103-104 (a closure over n, m there)."""
    return sigma_1(e) / n + sigma_2(e) / m + sigma_0(e) / (n * m)


def _un_block(tie_mode):
    spec = Bk.CompleteCount(literal_sub=False, tie_mode=tie_mode)

    def Un_block(X, Z):
        X = np.asarray(X)
        Z = np.asarray(Z)
        return spec.evaluate(X, Z, [Bk.whole(X, Z)])[0]

    Un_block._tw_block = spec
    return Un_block


_UN_STRICT = _un_block("strict")
_UN_HALF = _un_block("half")


def Un(X, Z, tie_mode="strict"):
    """Computes Un, full two-sample U-statistic.  (main.py:29-31)"""
    return (_UN_HALF if tie_mode == "half" else _UN_STRICT)(X, Z)


# UN(..., f_block=Un) must dispatch in one launch: expose the tagged block function's spec.
Un._tw_block = _UN_STRICT._tw_block


def UN(X, Z, N, f_block, sampling_type="SWOR"):
    """Computes complete or incomplete (depending on f_block) two-sample U-statistic on each
    worker and averages them.  Cuts the dataset X,Z in N splits.  sampling_type can be SWOR,
    prop-SWOR or prop-SWR.  (main.py:33-69)"""
    return Bk.run_un(X, Z, N, f_block, sampling_type, variant="est")


def UnN(X, Z, N, sampling_type, tie_mode="strict"):
    """Computes block-wise complete U-statistic.  (main.py:72-74)"""
    return UN(X, Z, N, _UN_HALF if tie_mode == "half" else Un, sampling_type=sampling_type)


def UnNT(X, Z, N, T, sampling_type, tie_mode="strict"):
    """Computes reshuffled block-wise complete U-statistic.  (main.py:76-79)"""
    return np.mean([UnN(X, Z, N, sampling_type=sampling_type, tie_mode=tie_mode)
                    for _ in range(T)])
