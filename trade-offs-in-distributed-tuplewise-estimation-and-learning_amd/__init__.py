"""tuplewise — MI355X-native tuplewise hot path of "Trade-offs in Large Scale Distributed
Tuplewise Estimation and Learning" (reference: RobinVogel/Trade-offs-in-Distributed-Tuplewise-
Estimation-and-Learning).

Drop-in modules (same names/signatures as the reference):
  tuplewise.estimation     <- estimation-experiment/main.py   (Un, UN, UnN, UnNT, moments)
  tuplewise.compute_stats  <- learning-experiment/compute_stats.py
  tuplewise.learning       <- learning-experiment/make_exps.py (learning_process, evaluation_step)
Device-resident / multi-GPU path:
  tuplewise.device         ShardedSample: repartition + count on the GPU(s), RCCL exchange
Native library: libtuplewise.so (csrc/*.hip, C ABI in include/tuplewise.h), loaded by _lib.
"""
from . import _lib  # noqa: F401
from . import compute_stats, estimation, device  # noqa: F401

__all__ = ["compute_stats", "estimation", "device", "learning"]


def __getattr__(name):
    if name == "learning":  # imports logging config helpers lazily
        # importlib, not "from . import": that form probes hasattr(package, "learning") first,
        # which would re-enter this function
        import importlib
        return importlib.import_module(__name__ + ".learning")
    raise AttributeError(name)
