#!/usr/bin/env python3
"""Benchmark: pair comparisons/s of the sharded AUC U-statistic (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[2]): n = 1e6 X-scores and 1e6 Z-scores (float64, synthetic
N(0.5,1) / N(0,1)) resident in HBM, cut into N = 64 prop-SWOR shards of 15625 x 15625 pairs —
in total over the G ranks (strong scaling, the default: n/G scores per class and 64/G shards
per rank), or per rank with --scaling weak (the nested `weak_C3` line at G > 1).  One step = one
block-wise complete U-statistic UnN (estimation-experiment/main.py:72-74): a fresh device
repartition of BOTH samples (one global keyed permutation; at G > 1 one RCCL all-to-all moves
every element to its new owner) and the exact pair count of all shards.  The K steps run as
est.UnNT's loop (ShardedSample.UnN_many): one ranking of X u Z in a sample's first call (rank
images, csrc/rankimage.hip; later calls carry the images of their final arrays — the timed call
is such a call, `first_call_ranking` times the same steps with the ranking), then per step one launch that counts on packed f32 images and carries the
next repartition (one GPU) or the count beside the exchange on a side stream (several), the
per-shard counts of all K steps combined by one all-reduce and the host's np.mean at the end.

value = pairs compared by all ranks / max-over-ranks wall time of the K timed steps.
roofline: the count kernel (k_count_rank, the one-launch step that also carries the next
repartition), VALU-bound: 1 compared pair = 1 lane-op against the f64 vector lane-op peak
3.93e13/s (256 CU x 64 lanes x 2.4 GHz); its duration is measured live with
HIP events on the stream it runs on.
cpu_baseline: the CPU port of the reference (oracle/oracle.py, identical NumPy operations to
est.UnN) timed on rank 0 at N=1 on one full UnN of the same configuration.
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

N_PER_CLASS = 1_000_000
C5_N = 5_000_000  # n=1e7 rows (5e6/5e6), d=512 fp64 = 41 GB
N_SHARDS = 64
PEAK_LANE_OPS = 256 * 64 * 2.4e9  # 3.93e13 f64 vector lane-ops/s (MI355X_MICROARCH chip table)
HBM_PEAK_GBS = 8000.0
INC_LANE_OPS = 53  # algorithmic lane-ops per device-RNG incomplete pair
# 32-bit integer VOP2 ops (v_xor/v_and/v_lshrrev_b32) issue at 1.60-1.63 wave-instructions/
# cycle/CU (profiles/r01_microbench_valu_issue2.log): 6.3e13 lane-op/s measured at 2.4 GHz
INT_LANE_OPS_MEASURED = 6.29e13


class EventPool:
    """Pre-created timing events; wrap(fn) records a pair around every `stride`-th call (until
    the pool runs out); used() lists the pairs recorded since the last clear(stride).  Timing
    every launch is not needed for the mean, so a timed region samples about 20 launches
    spread over it (the events are made before any timed region)."""

    def __init__(self, torch, n):
        self._ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    for _ in range(n)]
        self._w = [1] * n
        self._i = 0
        self._calls = 0
        self._stride = 1

    def clear(self, stride=1):
        self._i = 0
        self._calls = 0
        self._stride = max(1, int(stride))

    def used(self):
        return self._ev[:self._i]

    def ms_per_unit(self):
        """Mean milliseconds per unit of work over the recorded calls (weight = units per call,
        e.g. the steps one chain count launch carries)."""
        ms = [a.elapsed_time(b) for a, b in self.used()]
        return sum(ms) / max(1, sum(self._w[:self._i])) if ms else float("nan")

    def wrap(self, fn, weight=None):
        def timed(*a, **kw):
            c = self._calls
            self._calls += 1
            if self._i >= len(self._ev) or c % self._stride:
                return fn(*a, **kw)
            e0, e1 = self._ev[self._i]
            self._w[self._i] = weight(*a, **kw) if weight else 1
            self._i += 1
            e0.record()
            out = fn(*a, **kw)
            e1.record()
            return out
        timed.__wrapped__ = fn
        return timed


class Span:
    """Max-over-ranks wall time of a region: barrier + synchronize on both sides (the driver's
    timing contract), the slowest rank's seconds all-reduced."""

    def __init__(self, torch, dist, group, barrier):
        self.torch, self.dist, self.group, self.barrier = torch, dist, group, barrier

    def __call__(self, fn):
        t = self.torch
        t.cuda.synchronize()
        self.barrier()
        t.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        t.cuda.synchronize()
        self.barrier()
        t.cuda.synchronize()
        dt = time.perf_counter() - t0
        if self.group is not None:
            tt = t.tensor([dt], dtype=t.float64, device="cuda")
            self.dist.all_reduce(tt, op=self.dist.ReduceOp.MAX, group=self.group)
            dt = float(tt.item())
        return dt, out


_T_START = time.perf_counter()


def progress(msg):
    """One line per bench section on stderr (rank 0), so a long multi-GPU run shows it is alive;
    stdout carries only the JSON line."""
    if os.environ.get("RANK", "0") == "0":
        print(f"[bench {time.perf_counter() - _T_START:7.1f} s] {msg}", file=sys.stderr,
              flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of the run; without WORLD_SIZE in the environment, N > 1 "
                         "spawns N ranks of this script (no torchrun needed); with WORLD_SIZE "
                         "it must agree")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=N_PER_CLASS)
    ap.add_argument("--shards", type=int, default=N_SHARDS)
    ap.add_argument("--settle-ms", type=float, default=200.0,
                    help="untimed steps before the warmup, until the GPU clock is steady")
    ap.add_argument("--incomplete-B", type=int, default=1_000_000,
                    help="pairs per shard of the incomplete-statistic line")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sgd", action="store_true", help="skip the SGD steps/s secondary")
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the strong-scaling C3 line (n = 1e6/class, 64 shards in total)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="headline at N > 1 GPUs: strong = BASELINE configs[2]'s fixed problem "
                         "(--n per class and --shards in total over the ranks), weak = --n per "
                         "class and --shards per rank")
    ap.add_argument("--no-c5", action="store_true",
                    help="skip the C5 learning lines (41 GB of rows per rank; for gloo "
                         "rehearsals, where every exchange is staged through host memory)")
    ap.add_argument("--no-tradeoff", action="store_true",
                    help="skip the reshuffle_mod trade-off curve of the learning lines")
    ap.add_argument("--strong-T", type=int, default=4,
                    help="repartitions per estimate of the strong-scaling C3 line (UnNT's T)")
    ap.add_argument("--cpu-inc-shards", type=int, default=16,
                    help="shards of the incomplete CPU-baseline sample")
    ap.add_argument("--cpu-shards", type=int, default=N_SHARDS,
                    help="shards of the CPU-baseline sample (64 = one full UnN)")
    return ap.parse_args()


def cpu_baseline(n, N, shards):
    """The reference's UnN restated with its own NumPy operations (oracle.est_Un per block),
    single-threaded, on `shards` of the N prop-SWOR blocks of one shuffled sample."""
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    from oracle import oracle as O
    rng = np.random.RandomState(0)
    X, Z = rng.normal(0.5, 1, n), rng.normal(0, 1, n)
    k = n // N
    t0 = time.perf_counter()
    np.random.shuffle(X)
    np.random.shuffle(Z)
    vals = [O.est_Un(X[s * k:(s + 1) * k], Z[s * k:(s + 1) * k]) for s in range(shards)]
    float(np.mean(vals))
    dt = time.perf_counter() - t0
    pairs = shards * k * k
    return {"value": pairs / dt, "unit": "pairs/s", "cores": 1, "kind": "port",
            "host_cores": {"os_cpu_count": os.cpu_count(),
                           "affinity": len(os.sched_getaffinity(0))},
            "sample": f"est.UnN body (in-place shuffle + {shards} of {N} prop-SWOR blocks of "
                      f"{k}x{k}, NumPy broadcast compare), n={n}/class, {dt:.2f} s"}


def cpu_baseline_all_cores(n, N, workers):
    """The same est.UnN with its blocks spread over `workers` CPU processes (SURVEY.md §8(d)
    all-cores figure), run by a fresh Python process that never touches the GPU."""
    import subprocess
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-m", "oracle.parallel_baseline", str(n), str(N),
                        str(workers)], cwd=str(ROOT), env=env, capture_output=True, text=True,
                       timeout=600)
    if r.returncode != 0:
        return {"error": r.stderr.strip()[-300:]}
    return json.loads(r.stdout.strip().splitlines()[-1])


def sgd_complete_steps_per_s(n_X, n_Z, d, N, steps, loss="hinge"):
    """SGD steps with the complete-block gradient (extension; north_star item (2)): every step
    takes ALL pairs of every shard through per-point pair coefficients + X^T c
    (tw_pair_grad_complete), device-RNG shards, one reshuffle before the timed steps."""
    import torch
    from tuplewise.learning import SGDEngine
    g = torch.Generator(device="cuda").manual_seed(9)
    X = torch.randn((n_X, d), dtype=torch.float64, device="cuda", generator=g)
    Z = torch.randn((n_Z, d), dtype=torch.float64, device="cuda", generator=g) + 0.3
    w0 = torch.randn((d, 1), dtype=torch.float64, device="cuda", generator=g) / d ** 0.5
    eng = SGDEngine(X, Z, w0, N, 1, margin=1, reg=0.05, learning_rate=0.01,
                    optim_type="momentum", loss=loss, gradient="complete")
    eng.enable_device_rng(99)
    eng.run_segment(1, True, graphs=False)  # reshuffle + one warm step
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run_segment(steps, False, graphs=False)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    pairs = N * eng.kx * eng.kz
    rows_bytes = 2 * N * (eng.kx + eng.kz) * d * 8  # scores pass + weighted column sums
    # step floor = the two row passes at the HBM peak + the coefficient work at the f64 lane-op
    # peak (hinge: binary searches, ~log2(k) lane-ops per point, negligible; logistic: 7.5 VALU
    # per sigma, PMC-counted) -- serial phases, so the floors add
    lane_ops = 7.5 * pairs if loss == "logistic" else 2 * N * (eng.kx + eng.kz) * 15
    floor_s = rows_bytes / (HBM_PEAK_GBS * 1e9) + lane_ops / PEAK_LANE_OPS
    t_step = dt / steps
    return {"steps_per_s": steps / dt, "ms_per_step": dt / steps * 1e3,
            "pairs_per_step": pairs, "pairs_per_s": pairs * steps / dt,
            "row_GBps": rows_bytes * steps / dt / 1e9,
            "roofline": {"bound": "valu" if loss == "logistic" else "hbm",
                         "floor_ms": floor_s * 1e3, "frac": floor_s / t_step,
                         "hbm_bytes_per_step": rows_bytes, "lane_ops_per_step": lane_ops,
                         "note": "frac = (row bytes / HBM peak + coefficient lane-ops / f64 "
                                 "lane-op peak) / measured step; logistic counts 7.5 VALU per "
                                 "sigma (PMC), hinge ~15 per point (binary searches)"},
            "config": {"n_X": n_X, "n_Z": n_Z, "d": d, "N": N, "loss": loss,
                       "gradient": "complete (per-point pair coefficients + X^T c)",
                       "steps": steps}}


def plumbing_C1(with_cpu, reps=200):
    """est.UnNT(X, Z, N=10, T=4, "prop-SWOR") at n = 1000/class (BASELINE configs[0]) through
    the drop-in API on host arrays: latency per call, and the CPU restatement beside it."""
    import tuplewise.estimation as est
    rng = np.random.RandomState(0)
    X, Z = rng.normal(0.5, 1, 1000), rng.normal(0, 1, 1000)
    np.random.seed(1)
    for _ in range(5):
        est.UnNT(X, Z, 10, 4, "prop-SWOR")
    t0 = time.perf_counter()
    for _ in range(reps):
        v = est.UnNT(X, Z, 10, 4, "prop-SWOR")
    dt = (time.perf_counter() - t0) / reps
    out = {"note": "BASELINE configs[0]: est.UnNT on host arrays (drop-in), n=1000/class, "
                   "N=10, T=4, prop-SWOR; host shuffles (reference RNG order) + one device launch "
                   "for the T repetitions",
           "ms_per_call": dt * 1e3, "pairs_per_call": 4 * 10 * 100 * 100, "last_value": v}
    if with_cpu:
        sys.path.insert(0, str(ROOT))
        from oracle import oracle as O
        t0 = time.perf_counter()
        for _ in range(reps):
            O.est_UnNT(X, Z, 10, 4, "prop-SWOR")
        out["cpu_ms_per_call"] = (time.perf_counter() - t0) / reps * 1e3
        out["cpu_kind"] = "port (oracle est_UnNT, NumPy, 1 core)"
    return out


def drop_in_C3(reps=10, T=4, N=64, n=N_PER_CLASS):
    """The user-visible drop-in at BASELINE configs[2]'s size: est.UnNT(X, Z, 64, 4, "prop-SWOR")
    (estimation-experiment/main.py:76-79) on HOST arrays of n = 1e6 per class, exactly as a
    reference script calls it.  Default path: the host makes every draw in the reference's RNG
    order (the T shuffles' index draws by the native restatement, numpy_rng.shuffle_draws32),
    X and Z go up once, the device applies the T shuffles' swaps keeping every state
    (csrc/devshuffle.hip; launches made by a launcher thread while the host draws, the last
    shuffle streamed in window groups), each step's blocks are counted while the next step is
    drawn, and the caller's arrays receive the last state.  ms_per_call: the median of `reps`
    calls (mean beside it).  The host-swap path (shuffle_pair + T snapshots uploaded) is timed
    beside it, and the parts of the default path alone on the same shapes."""
    import torch
    import tuplewise.estimation as est
    from tuplewise import _blocks as Bk, _engine as E, _lib as L
    from tuplewise.numpy_rng import shuffle_draws32
    rng = np.random.RandomState(0)
    X, Z = rng.normal(0.5, 1, n), rng.normal(0, 1, n)

    def timed(min_items):
        old = Bk.DEVICE_SHUFFLE_MIN
        Bk.DEVICE_SHUFFLE_MIN = min_items
        try:
            Xc, Zc = X.copy(), Z.copy()  # both paths from the same arrays and RNG state
            np.random.seed(1)
            for _ in range(3):  # warm (a reference script calls it in a loop: steady state;
                # after one warm call the first series still ran ~0.3 ms/call slower than a later
                # one on the same path, profiles/r05s19_bench.json / r05s38_bench.json)
                est.UnNT(Xc, Zc, N, T, "prop-SWOR")
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                v = est.UnNT(Xc, Zc, N, T, "prop-SWOR")
                ts.append(time.perf_counter() - t0)
            timed.mean = float(np.mean(ts))
            return float(np.median(ts)), v
        finally:
            Bk.DEVICE_SHUFFLE_MIN = old

    dt, v = timed(Bk.DEVICE_SHUFFLE_MIN)
    dt_mean = timed.mean
    dt_host, v_host = timed(1 << 62)
    # the same call with two device slots visible (a multi-GPU node's default device list;
    # slots [0, 0] on one GPU): the blocks' sorted count stays below the spreading threshold,
    # so the device-shuffle path is kept
    from tuplewise import _multi as M
    M.set_devices([0, 0])
    try:
        dt_slots, v_slots = timed(Bk.DEVICE_SHUFFLE_MIN)
    finally:
        M.set_devices(None)
    # the parts of the default path, timed alone on the same shapes
    t0 = time.perf_counter()
    jx, jz = [], []
    for _ in range(T):
        jx.append(shuffle_draws32(n))
        jz.append(shuffle_draws32(n))
    draws = time.perf_counter() - t0
    t0 = time.perf_counter()
    for _ in range(T):
        np.random.shuffle(X)
        np.random.shuffle(Z)
    np_shuffles = time.perf_counter() - t0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    xd0, zd0 = L.to_device(X), L.to_device(Z)
    torch.cuda.synchronize()
    h2d = time.perf_counter() - t0
    E.shuffle_snapshots_device(xd0, zd0, jx, jz)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    xs, zs = E.shuffle_snapshots_device(xd0, zd0, jx, jz)
    torch.cuda.synchronize()
    dev_shuffle = time.perf_counter() - t0
    t0 = time.perf_counter()
    X[...] = xs[T - 1].cpu().numpy()
    Z[...] = zs[T - 1].cpu().numpy()
    d2h = time.perf_counter() - t0
    k = n // N
    off = np.arange(T * N + 1, dtype=np.int64) * k
    offd = L.to_device(off)
    algo = E.pick_algo("auto", k, k, "gt")
    xf, zf = xs.reshape(-1), zs.reshape(-1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    E.count_launch(xf, offd, zf, offd, T * N, k, k, L.TW_F64, L.TW_PRED_GT, algo)
    e0.record()
    E.count_launch(xf, offd, zf, offd, T * N, k, k, L.TW_F64, L.TW_PRED_GT, algo)
    e1.record()
    torch.cuda.synchronize()
    pairs = T * N * k * k
    return {"note": "est.UnNT(X, Z, 64, 4, 'prop-SWOR') on host arrays, n=1e6/class (the drop-in "
                    "as a reference script calls it): host draws in the reference's order, the "
                    "shuffles' swaps on the device (csrc/devshuffle.hip), the caller's arrays "
                    "written back; parts timed alone on the same shapes",
            "ms_per_call": dt * 1e3, "ms_per_call_mean": dt_mean * 1e3, "calls": reps,
            "value": pairs / dt,
            # the sorted count decides every pair without comparing it: logical pairs
            "unit": "logical pairs/s" if algo == "sorted" else "pairs/s",
            "host_swap_path_ms_per_call": dt_host * 1e3,
            "same_value_both_paths": bool(v == v_host),
            "slots_0_0_ms_per_call": dt_slots * 1e3,
            "slots_0_0_same_value": bool(v_slots == v),
            "host_draws_ms": draws * 1e3, "numpy_shuffles_ms": np_shuffles * 1e3,
            "h2d_ms": h2d * 1e3, "device_shuffles_ms": dev_shuffle * 1e3,
            "d2h_ms": d2h * 1e3, "count_algo": algo,
            "kernel_ms": e0.elapsed_time(e1), "last_value": float(v)}


def cpu_baseline_incomplete(n, N, B, shards):
    """The reference's UnNB(kernel="AUC") restated (oracle.UB per block: two randint draws and
    a fancy-indexed compare, compute_stats.py:37-42), single-threaded, on `shards` of the N
    prop-SWOR blocks of one shuffled sample."""
    from oracle import oracle as O
    rng = np.random.RandomState(1)
    X, Z = rng.normal(0.5, 1, n), rng.normal(0, 1, n)
    k = n // N
    t0 = time.perf_counter()
    np.random.shuffle(X)
    np.random.shuffle(Z)
    vals = [O.UB(X[s * k:(s + 1) * k], Z[s * k:(s + 1) * k], B, kernel="AUC")
            for s in range(shards)]
    float(np.mean(vals))
    dt = time.perf_counter() - t0
    return {"value": shards * B / dt, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": f"cs.UnNB body (in-place shuffle + {shards} of {N} prop-SWOR blocks, "
                      f"B={B} randint pairs each), n={n}/class, {dt:.2f} s"}


def sgd_data(n_X, n_Z, d):
    """Synthetic learning rows generated on the device (the same on every rank: one seed)."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(7)
    X = torch.randn((n_X, d), dtype=torch.float64, device="cuda", generator=g)
    Z = torch.randn((n_Z, d), dtype=torch.float64, device="cuda", generator=g) + 0.3
    w0 = torch.randn((d, 1), dtype=torch.float64, device="cuda", generator=g)
    return X, Z, w0


def sgd_steps_per_s(n_X, n_Z, d, N, B, reshuffle_mod, steps, warmup, layout="replicated",
                    group=None, span=None, data=None, check_prefix=0, loss="hinge"):
    """Pairwise-hinge SGD steps/s (BASELINE metric, second half): learning_process's loop
    (make_exps.py:122-141) without evaluation, device-RNG mode, hipGraph-replayed segments.
    Synthetic data of the given shape generated on the device.  layout="partitioned" also
    times one reshuffle's row exchange (row tables + route + pack of the remote rows + the
    all_to_all; at one GPU every row is owned: the tables only).  group: the ranks of the run (each
    owns N/G shards; one all-gather of the shard gradients per step); check_prefix > 0: the
    first steps' w is compared with a one-rank engine's on rank 0 (bit for bit)."""
    import torch
    from tuplewise.learning import SGDEngine
    X, Z, w0 = data if data is not None else sgd_data(n_X, n_Z, d)
    eng = SGDEngine(X, Z, w0, N, B, margin=1, reg=0.05, learning_rate=0.01,
                    optim_type="momentum", x_layout=layout, group=group, loss=loss)
    eng.enable_device_rng(12345)

    import tuplewise.learning as lr
    swr = lr.SWR_IN_KERNEL and eng.swr_segments_ok()

    def run(e, k):
        if swr and k > 1:
            # the persistent narrow segment draws every reshuffle's rows itself: segments are
            # not cut at reshuffles (learning_process cuts them at evaluations only)
            i = 0
            while i < k:
                n = min(k - i, 4096)
                if k - i - n == 1:
                    n -= 1  # never leave a one-step tail
                e.run_segment(n, False, graphs=True, swr_mod=reshuffle_mod)
                i += n
            return
        i = 0
        while i < k:
            nxt = min(k, (i // reshuffle_mod + 1) * reshuffle_mod)
            e.run_segment(nxt - i, i % reshuffle_mod == 0, graphs=True)
            i = nxt

    # warm: the timed schedule itself once (the same segment lengths, so every hipGraph the
    # timed run replays is captured here), then `warmup` more reshuffle periods
    run(eng, steps)
    run(eng, warmup * min(reshuffle_mod, steps))
    if span is None:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(eng, steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    else:
        dt, _ = span(lambda: run(eng, steps))
    eng.check()  # a persistent segment that gave up at a barrier invalidates the run
    same_1rank = None
    if check_prefix and group is not None:
        # the trajectory does not depend on G: a fresh engine over the ranks and a one-rank
        # engine on rank 0, same seed, the same first steps, w compared bit for bit
        e_g = SGDEngine(X, Z, w0, N, B, margin=1, reg=0.05, learning_rate=0.01,
                        optim_type="momentum", x_layout=layout, group=group, loss=loss)
        e_g.enable_device_rng(777)
        run(e_g, check_prefix)
        w_g = e_g.w_host()
        if torch.distributed.get_rank(group) == 0:
            e_1 = SGDEngine(X, Z, w0, N, B, margin=1, reg=0.05, learning_rate=0.01,
                            optim_type="momentum", loss=loss)
            e_1.enable_device_rng(777)
            run(e_1, check_prefix)
            same_1rank = bool(np.array_equal(w_g, e_1.w_host()))
            del e_1
        del e_g
    launches = ("one persistent launch per segment over the ranks, shard gradients exchanged "
                "GPU to GPU through IPC-mapped peer buffers (csrc/peer.hip)"
                + (", reshuffles drawn in the kernel" if swr else "")
                if getattr(eng, "peer_seg", False) else
                "gradient launch + one publish-wait-update launch per step (csrc/peer.hip)"
                if getattr(eng, "peer", None) is not None else
                "one persistent launch per run of <= 4096 steps, reshuffles drawn in the "
                "kernel" if swr and eng.narrow_seg else
                "gradient + update launch per step (hipGraph-replayed segments), each "
                "reshuffle's rows drawn in the gradient kernel" if swr else
                "one persistent launch per segment" if eng.narrow_seg else
                "one launch per step" if eng.fused else "gradient + update per step")
    G = 1 if group is None else torch.distributed.get_world_size(group)
    out = {"steps_per_s": steps / dt, "ms_per_step": dt / steps * 1e3,
           "pairs_per_step": N * B, "gathered_bytes_per_step": N * B * 16 * d,
           "gather_GBps": N * B * 16 * d * steps / dt / 1e9,
           "config": {"n_X": n_X, "n_Z": n_Z, "d": d, "N": N, "B": B, "loss": loss,
                      "reshuffle_mod": reshuffle_mod, "optim": "momentum",
                      "rng": "device (Philox)", "graphs": True, "steps": steps,
                      "x_layout": layout, "launches": launches, "ranks": G}}
    if same_1rank is not None:
        out["trajectory_equal_1rank"] = {"steps": check_prefix, "equal": same_1rank}
    if layout == "partitioned":
        reps = 3

        def resh():
            for _ in range(reps):
                eng.reshuffle_device()
        if span is None:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            resh()
            torch.cuda.synchronize()
            rs = (time.perf_counter() - t0) / reps
        else:
            rs = span(resh)[0] / reps
        rows = eng.N_loc * (eng.kx + eng.kz)  # this rank's drawn positions
        remote = rows * (G - 1) // G  # expected rows owned elsewhere (the only ones that move)
        # table write per position; a remote row: read in the partition, written with its
        # position into the send bucket (the receive side writes it in place: RCCL's bytes)
        moved = rows * 8 + remote * 8 * (2 * d + 1)
        out["reshuffle_exchange"] = {"ms": rs * 1e3, "rows": rows, "remote_rows": remote,
                                     "bytes": moved, "GBps": moved / rs / 1e9,
                                     "note": "owned rows are read in place in the partition; "
                                             "only remote rows travel (none at G = 1)"}
    return out


def c4_problem():
    rng = np.random.RandomState(3)
    X = np.hstack([rng.normal(size=(9117, 9)), np.ones((9117, 1))])
    Z = np.hstack([rng.normal(0.5, 1, size=(702, 9)), np.ones((702, 1))])
    return X, Z, rng.normal(size=(10, 1))


def sgd_replay_steps_per_s(steps, mod=25, group=None, span=None, runs=3, audit=True):
    """learning_process in replay mode (NumPy's own draws, bit-identical to the reference)
    at the C4 shape, no evaluation: host RNG (one native MT19937 batch per segment) + index
    upload + the persistent segment kernel.  group: every rank makes the full draw sequence
    and uses its shards (make_exps.py:122-141 over the ranks)."""
    import logging
    import torch
    import tuplewise.learning as lr
    X, Z, w0 = c4_problem()
    p = {"n_it": steps, "margin": 1, "N": 100, "B": 100, "reshuffle_mod": mod, "reg": 0.05,
         "learning_rate": 0.01, "eval_mod": 10 ** 9, "w_init": w0,
         "test_X": X[:10], "test_Z": Z[:10], "train_mon_pairs": [(0, 0)], "train_X": X,
         "train_Z": Z}
    logging.disable(logging.CRITICAL)
    np.random.seed(0)
    lr.learning_process(X, Z, dict(p, n_it=50), group=group)  # warm
    # host-bound (NumPy-exact draws on the box's shared host cores): the median of the runs
    ts = []
    for _ in range(runs):
        if span is None:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            lr.learning_process(X, Z, p, group=group)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        else:
            ts.append(span(lambda: lr.learning_process(X, Z, p, group=group))[0])
    dt = float(np.median(ts))
    out = {"steps_per_s": steps / dt, "ms_per_step": dt / steps * 1e3,
           "runs_steps_per_s": [steps / r for r in ts],
           "config": {"n_X": 9117, "n_Z": 702, "d": 10, "N": 100, "B": 100,
                      "reshuffle_mod": mod, "rng": "replay (NumPy legacy MT19937, bit-exact)",
                      "steps": steps,
                      "ranks": 1 if group is None else torch.distributed.get_world_size(group)}}
    if audit and group is None:
        # hinge-filter sign audit, untimed: the device's S against NumPy/BLAS's
        # on every pair of 300 replay steps of the same run
        aud = []
        np.random.seed(0)
        lr.learning_process(X, Z, dict(p, n_it=300), sign_audit=aud)
        out["sign_audit"] = {"steps": len(aud), "pairs": sum(a["pairs"] for a in aud),
                             "near_zero_S": sum(a["near_zero"] for a in aud),
                             "filter_flips": sum(a["flips"] for a in aud),
                             "note": "pairs whose |S| is within the dot product's rounding "
                                     "bound, and pairs whose hinge filter differs from NumPy's"}
    return out


def cpu_port_c4(mod, steps=150):
    """The reference loop restated with its own NumPy operations (oracle.learning_trajectory:
    SWR_divide every reshuffle_mod steps, grad_inc_block per shard, momentum update;
    make_exps.py:122-141 without evaluation), single-threaded, at the C4 shape."""
    from oracle import oracle as O
    X, Z, w0 = c4_problem()
    p = {"n_it": steps, "margin": 1, "N": 100, "B": 100, "reshuffle_mod": mod, "reg": 0.05,
         "learning_rate": 0.01, "w_init": w0}
    np.random.seed(0)
    t0 = time.perf_counter()
    O.learning_trajectory(X, Z, p, capture_every=10 ** 9)
    return steps / (time.perf_counter() - t0)


def learning_end_to_end(steps, rng_mode, group=None, span=None):
    """learning_process at the C4 shape WITH its evaluation every 25 steps (make_exps.py:
    122-141, 143-190): shuttle-shaped synthetic train/test sets, 450k fixed monitor pairs
    (make_exps.py:216-224).  The reference spends ~2.6 ms per step and 158 ms per evaluation
    here, i.e. ~110 steps/s."""
    import logging
    import torch
    import tuplewise.learning as lr
    rng = np.random.RandomState(4)
    X = np.hstack([rng.normal(size=(9117, 9)), np.ones((9117, 1))])
    Z = np.hstack([rng.normal(0.5, 1, size=(702, 9)), np.ones((702, 1))])
    Xe = np.hstack([rng.normal(size=(2279, 9)), np.ones((2279, 1))])
    Ze = np.hstack([rng.normal(0.5, 1, size=(175, 9)), np.ones((175, 1))])
    mon = list(zip(rng.randint(0, 9117, 450000), rng.randint(0, 702, 450000)))
    p = {"n_it": steps, "margin": 1, "N": 100, "B": 100, "reshuffle_mod": 25, "reg": 0.05,
         "learning_rate": 0.01, "eval_mod": 25, "w_init": rng.normal(size=(10, 1)),
         "test_X": Xe, "test_Z": Ze, "train_mon_pairs": mon, "train_X": X, "train_Z": Z}
    logging.disable(logging.CRITICAL)
    np.random.seed(0)
    lr.learning_process(X, Z, dict(p, n_it=50), rng_mode=rng_mode, group=group)  # warm
    runs = []
    for _ in range(3):  # the median of 3 runs (the replay draws run on shared host cores)
        p["iter"] = []
        if span is None:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            lr.learning_process(X, Z, p, rng_mode=rng_mode)
            torch.cuda.synchronize()
            runs.append(time.perf_counter() - t0)
        else:
            runs.append(span(lambda: lr.learning_process(X, Z, p, rng_mode=rng_mode,
                                                         group=group))[0])
    dt = float(np.median(runs))
    return {"steps_per_s": steps / dt, "ms_per_step": dt / steps * 1e3,
            "runs_steps_per_s": [steps / r for r in runs],
            "evaluations": len(p["iter"]),
            "config": {"n_X": 9117, "n_Z": 702, "d": 10, "N": 100, "B": 100,
                       "reshuffle_mod": 25, "eval_mod": 25, "monitor_pairs": 450000,
                       "test": "2279 x 175", "rng": rng_mode, "steps": steps,
                       "ranks": 1 if group is None else torch.distributed.get_world_size(group)}}


def pmc_traffic(kernel="k_count_complete"):
    """HBM bytes per launch of the count kernel from the committed rocprofv3 --pmc summary of
    this workload (profiles/*count_pmc*.json, FETCH_SIZE + WRITE_SIZE): the timed one-launch
    step (count + next repartition) and, when present, a plain count launch."""
    import re
    # newest round/session first: natural order of the numbers in the name (r01s27 > r01s5)
    cands = sorted(ROOT.glob("profiles/*count_pmc*.json"),
                   key=lambda p: [int(v) for v in re.findall(r"\d+", p.name)])
    d = None
    for c in reversed(cands):  # the newest summary OF THIS KERNEL (other kernels' files match)
        try:
            e = json.loads(c.read_text())
        except Exception:
            continue
        if str(e.get("kernel", "")).startswith(kernel):
            d = e
            break
    if d is None:
        return None, None
    plain = d.get("by_grid", {}).get(d.get("plain_grid") or "", {}).get("hbm_bytes_per_launch")
    per = d.get("hbm_bytes_per_launch")
    k = d.get("steps_per_launch")  # a k_count_chain launch counts every step of a chunk
    if k and per is not None:
        return per / k, None
    return per, plain


def traced_count_chain(steps):
    """The committed rocprofv3 kernel-trace summary of the headline count launch at this K
    (profiles/*count_chain_traced*.json, tools/traced_chain.py): mean / min duration of the
    K-step k_count_chain launches and the lane-op fractions they imply — the traced figure
    printed beside the live frac."""
    cands = sorted(ROOT.glob("profiles/*count_chain_traced*.json"),
                   key=lambda p: p.stat().st_mtime, reverse=True)
    for c in cands:
        try:
            d = json.loads(c.read_text())
        except Exception:
            continue
        if int(d.get("steps_per_launch", -1)) == int(steps):
            return {k: d[k] for k in ("mean_ms", "min_ms", "frac_mean", "frac_min", "launches",
                                      "timed_ms", "frac_timed", "launch_ms_in_order")
                    if k in d} | {"source": str(c.relative_to(ROOT))}
    return None


def pmc_emit_traffic():
    """HBM bytes per step of the step chains' emission (k_chain_emit) in the bench's timed
    K-step call, from the committed per-dispatch --pmc summary (profiles/*chain_emit_pmc.json)."""
    import re
    cands = sorted(ROOT.glob("profiles/*chain_emit_pmc*.json"),
                   key=lambda p: [int(v) for v in re.findall(r"\d+", p.name)])
    if not cands:
        return None
    try:
        t = json.loads(cands[-1].read_text())["timed_call"]
        # (the guide's gfx950 correction of FETCH_SIZE, doubled, where the summary has it)
        return (t["write_MB"] + t.get("fetch_MB_doubled", t["fetch_MB"])) * 1e6 / t["steps"]
    except Exception:
        return None


def pmc_replay_traffic():
    """HBM bytes per launch of k_count_idx_img from the committed rocprofv3 --pmc summary
    (profiles/*replay_img_pmc*.json): FETCH_SIZE doubled — the index streams are 16-B/lane
    coalesced reads, which gfx950's FETCH_SIZE reports at exactly half (MI355X_MICROARCH.md
    §HBM) — plus WRITE_SIZE; the raw sum beside it."""
    import re
    cands = sorted(ROOT.glob("profiles/*replay_img_pmc*.json"),
                   key=lambda p: [int(v) for v in re.findall(r"\d+", p.name)])
    if not cands:
        return None, None
    try:
        d = json.loads(cands[-1].read_text())
        g = d["by_grid"][d.get("timed_grid") or next(iter(d["by_grid"]))]
        return (2 * g["FETCH_SIZE"] + g["WRITE_SIZE"]) * 1024, \
            (g["FETCH_SIZE"] + g["WRITE_SIZE"]) * 1024
    except Exception:
        return None, None


def incomplete_replay(X, Z, shards, B, reps=20):
    """UnNB in replay mode (compute_stats.py:37-42 via UB): B explicit index pairs per shard,
    as NumPy's randint hands them over after the drop-in's bound check narrows them to int32
    (8 B per pair), already resident in HBM, counted by tw_count_pairs_idx32_ws:
    k_count_idx_img stages each shard's float32 score images in LDS and streams the index pairs
    (pairs with equal images are decided on the scores).  HBM-bound on the index streams.  Indices are
    drawn on the device here (uniform within each shard's contiguous range); the kernel sees the
    same layout as the drop-in UB/UnNB path.  The plain gather kernel (tw_count_pairs_idx32,
    the fallback for shard pairs too large for LDS) and the int64-index call are timed beside
    it."""
    import torch
    from tuplewise import _engine, _lib as L
    n = X.numel()
    k = n // shards
    g = torch.Generator(device="cuda").manual_seed(4321)
    base = (torch.arange(shards, device="cuda", dtype=torch.int64) * k).repeat_interleave(B)
    ix64 = base + torch.randint(0, k, (shards * B,), device="cuda", generator=g)
    iz64 = base + torch.randint(0, k, (shards * B,), device="cuda", generator=g)
    ix, iz = ix64.to(torch.int32), iz64.to(torch.int32)
    del base
    pair_off = np.arange(shards + 1, dtype=np.int64) * B
    pod = L.to_device(pair_off)

    off = L.to_device(np.arange(shards + 1, dtype=np.int64) * k)
    work = L.empty((int(L.lib().tw_count_pairs_rng_work_bytes(shards, k, k, L.TW_F64,
                                                              L.TW_PRED_GT)),), torch.uint8)

    def plain():
        return _engine.count_indexed_dev(X, Z, L.TW_F64, ix, iz, pair_off, L.TW_PRED_GT, pod)

    def ranked():
        return _engine.count_indexed_ranked_dev(X, off, Z, off, k, k, L.TW_F64, ix, iz,
                                                pair_off, L.TW_PRED_GT, pod, work)

    def ranked64():
        return _engine.count_indexed_ranked_dev(X, off, Z, off, k, k, L.TW_F64, ix64, iz64,
                                                pair_off, L.TW_PRED_GT, pod, work)

    def timed(launch):
        for _ in range(3):
            launch()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(reps)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for e0, e1 in ev:
            e0.record()
            out = launch()
            e1.record()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        return out, dt, float(np.mean([a.elapsed_time(b) for a, b in ev]))

    out_p, dt_p, kms_p = timed(plain)
    out64, dt64, kms64 = timed(ranked64)
    out, dt, kms = timed(ranked)
    # every shard against a torch gather-compare of its pairs (exact integers)
    want = (X[ix64] > Z[iz64]).view(shards, B).sum(1)
    pairs = shards * B
    bpp = 8  # algorithmic bytes per pair: two int32 indices
    traffic, traffic_raw = pmc_replay_traffic()
    return {"note": "UnNB replay mode: B explicit int32 index pairs per shard resident in HBM "
                    "(NumPy-drawn and narrowed after the bound check in the drop-in path; "
                    "device-drawn here); tw_count_pairs_idx32_ws: k_count_idx_img compares "
                    "float32 score images held in LDS (equal images decided on the scores)",
            "B_per_shard": B, "value": pairs * reps / dt, "unit": "pairs/s",
            "ms_per_call": dt / reps * 1e3,
            "counts_identical_to_plain": bool(torch.equal(out, out_p)),
            "counts_identical_to_int64": bool(torch.equal(out, out64)),
            "all_shards_match_torch": bool(torch.equal(out, want)),
            "plain_k_count_idx_int32": {"value": pairs * reps / dt_p,
                                        "ms_per_call": dt_p / reps * 1e3, "kernel_ms": kms_p,
                                        "GBps_indices": bpp * pairs / (kms_p * 1e-3) / 1e9},
            "ranked_int64_indices": {"value": pairs * reps / dt64, "kernel_ms": kms64,
                                     "GBps_indices": 16 * pairs / (kms64 * 1e-3) / 1e9},
            "roofline": {"bound": "hbm", "kernel": "k_count_idx_img",
                         "achieved": bpp * pairs / (kms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": bpp * pairs / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "kernel_ms": kms, "traffic": traffic, "traffic_raw": traffic_raw,
                         "algorithmic_bytes": bpp * pairs,
                         "note": "8 algorithmic bytes per pair (two int32 indices, SURVEY.md "
                                 "§8(d)); kernel_ms = the whole call: one kernel that stages "
                                 "each shard's float32 score images in LDS and streams the "
                                 "index pairs (csrc/imagecount.hip); traffic = HBM bytes per "
                                 "launch from the committed rocprofv3 --pmc summary "
                                 "(profiles/r02_replay_img_pmc.json): FETCH_SIZE x2 (16-B/lane "
                                 "streaming reads, MI355X_MICROARCH.md §HBM) + WRITE_SIZE; "
                                 "traffic_raw uncorrected"}}


def spawn_ranks(n: int, script: str | None = None, argv: list | None = None) -> int:
    """`python bench.py --gpus N` without a launcher: start N ranks of this script as child
    processes (one per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set as torch.distributed.run
    would, rendezvous on 127.0.0.1) before this process touches any GPU; rank 0 prints the JSON
    line.  Returns the exit code (non-zero if any rank failed; the others are then stopped)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        cmd = [sys.executable, script or os.path.abspath(__file__)]
        cmd += sys.argv[1:] if argv is None else argv
        procs.append(subprocess.Popen(cmd, env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    while procs:
        for pr in list(procs):
            code = pr.poll()
            if code is None:
                continue
            procs.remove(pr)
            if code != 0 and rc == 0:
                rc = code
                for other in procs:  # one rank failed: the collectives would hang
                    other.terminate()
        time.sleep(0.05)
    return rc


def resolve_world(args) -> int:
    """World size from WORLD_SIZE (launcher) or --gpus (self-spawn); a disagreement is an
    error, not a silent one-rank run."""
    env = os.environ.get("WORLD_SIZE")
    if env is None:
        return args.gpus if args.gpus is not None else 1
    world = int(env)
    if args.gpus is not None and args.gpus != world:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}\n")
        sys.exit(2)
    return world


def strong_c3(args, group, rank, world, barrier, torch, dist):
    """BASELINE configs[2] as strong scaling: n = 1e6/class and N = 64 shards IN TOTAL, so each
    of G ranks holds n/G scores per class and 64/G shards (8 per GPU at G = 8, the survey's
    '8 GPUs x 8 shards'); est.UnNT / cs.UnNBT steps with T repartitions per estimate.  The
    global permutation, hence every shard's count and every estimate, does not depend on G."""
    from tuplewise.device import ShardedSample
    n_tot, N_tot = N_PER_CLASS, N_SHARDS
    if N_tot % world or n_tot % world:
        return {"skipped": f"n={n_tot}, N={N_tot} do not divide over {world} ranks"}
    n_loc, N_loc = n_tot // world, N_tot // world
    gen = torch.Generator(device="cuda").manual_seed(5000 + rank)
    X = torch.randn(n_loc, dtype=torch.float64, device="cuda", generator=gen) + 0.5
    Z = torch.randn(n_loc, dtype=torch.float64, device="cuda", generator=gen)
    S = ShardedSample(X, Z, N_loc, group=group, algo="pairs")
    k = n_tot // N_tot
    T = max(1, args.strong_T)
    reps = max(1, args.steps // T)

    def timed(fn):
        for w in range(3):  # warm: same shapes, other keys (a sample's first calls rank and
            # allocate; the reference calls est.UnNT in a loop, main.py:110-111 — on fresh
            # samples there: the first-call cost is `first_call_ranking` beside the headline)
            fn(90_000 + 1000 * w)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ests = [fn(r * T) for r in range(reps)]
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if group is not None:
            tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=group)
            dt = float(tt.item())
        return dt, ests[-1]

    dt_c, est_c = timed(lambda k0: S.UnNT(T, k0))
    B = args.incomplete_B
    dt_i, est_i = timed(lambda k0: float(np.mean(S.UnNB_many(B, 777 + k0, range(k0, k0 + T)))))
    pairs_c = N_tot * k * k * T * reps
    pairs_i = N_tot * B * T * reps
    return {"note": "BASELINE configs[2] strong scaling: n=1e6/class and N=64 prop-SWOR shards in "
                    "total (64/G shards and 1e6/G scores per class per rank), T repartitions per "
                    "estimate (UnNT complete, UnNBT incomplete with device-drawn pairs); value = "
                    "pairs of all ranks / max-over-ranks wall time",
            "scaling": "strong", "n_per_class_total": n_tot, "shards_total": N_tot,
            "shards_per_rank": N_loc, "T": T, "estimates": reps,
            "complete": {"value": pairs_c / dt_c, "unit": "pairs/s",
                         "ms_per_estimate": dt_c / reps * 1e3, "estimate_last": float(est_c)},
            "incomplete": {"B_per_shard": B, "value": pairs_i / dt_i, "unit": "pairs/s",
                           "ms_per_estimate": dt_i / reps * 1e3, "estimate_last": float(est_i)}}


RESHUFFLE_MODS = (1, 5, 25, 125, 10000)  # learning-experiment/main.py:20


def tradeoff_curve(args, group, span, with_cpu):
    """The paper's trade-off axis: SGD steps/s for every reshuffle_mod of the reference's sweep
    (learning-experiment/main.py:20; a reshuffle = a new SWR draw of every shard, make_exps.py:
    123-125).  C4 (shuttle shape) with device and replay draws; C5 (d = 512, n = 1e7, N = 256,
    B = 100) with X replicated (a reshuffle is new row tables, no data moves) and row-partitioned
    (a reshuffle moves every drawn row to its shard's rank: the communication side of the
    trade-off); the reference loop restated on one CPU core beside the C4 points."""
    import torch
    out = {"note": "steps/s per reshuffle_mod (learning-experiment/main.py:20); device = "
                   "Philox draws + hipGraph segments, replay = NumPy's own MT19937 draws "
                   "(bit-exact); C5 partitioned: every reshuffle exchanges the drawn rows "
                   "owned by other ranks (at G = 1: none, only new row tables)",
           "reshuffle_mod": list(RESHUFFLE_MODS)}
    c4d, c4r, cpu = {}, {}, {}
    for mod in RESHUFFLE_MODS:
        progress(f"trade-off curve C4, reshuffle_mod {mod}")
        c4d[mod] = sgd_steps_per_s(9117, 702, 10, 100, 100, mod, 2000, 1, group=group,
                                   span=span)["steps_per_s"]
        # replay is bound by the host's NumPy-exact draws: the median of three 1000-step runs
        # (one run swung 70-88k at mod 1 on the same box)
        c4r[mod] = sgd_replay_steps_per_s(1000, mod, group=group, span=span, runs=3,
                                          audit=False)["steps_per_s"]
        if with_cpu:
            cpu[mod] = cpu_port_c4(mod)
    out["C4_device"], out["C4_replay"] = c4d, c4r
    if cpu:
        out["C4_cpu_port_1core"] = cpu
    if args.no_c5:
        return out
    data = sgd_data(C5_N, C5_N, 512)
    c5r, c5p = {}, {}
    for mod in RESHUFFLE_MODS:
        progress(f"trade-off curve C5, reshuffle_mod {mod}")
        c5r[mod] = sgd_steps_per_s(C5_N, C5_N, 512, 256, 100, mod, 200, 1, group=group,
                                   span=span, data=data)["steps_per_s"]
        # a partitioned reshuffle moves the ~n (G-1)/G remote rows: fewer steps at mod 1, G > 1
        G = 1 if group is None else torch.distributed.get_world_size(group)
        steps_p = 200 if G == 1 else 10 if mod == 1 else 50 if mod == 5 else 100
        c5p[mod] = sgd_steps_per_s(C5_N, C5_N, 512, 256, 100, mod, steps_p, 1,
                                   layout="partitioned", group=group, span=span,
                                   data=data)["steps_per_s"]
    del data
    torch.cuda.empty_cache()
    out["C5_B100_replicated"], out["C5_B100_partitioned"] = c5r, c5p
    return out


def half_ties_line(args, group, span, torch, X, Z, shards, pairs_per_step_rank, world):
    """The north star's "+0.5 on ties" mode (tie_mode="half": 2 #{x > z} + #{x == z} half
    units) on the headline's UnN steps: step chains whose x images are {g(x), h(x)} pairs, one
    clamped packed add giving [x > z] and [x >= z] for a z — 2 lane-ops of the contract per
    pair."""
    from tuplewise.device import ShardedSample
    S = ShardedSample(X.clone(), Z.clone(), shards, group=group, tie_mode="half", algo="pairs")
    pool = EventPool(torch, 64)
    S.ops.count_chain = pool.wrap(S.ops.count_chain, weight=lambda *a, **kw: a[5])
    S.UnN_many(range(90_000, 90_000 + args.steps))
    S.UnN_many(range(args.warmup))
    pool.clear()
    dt, ests = span(lambda: S.UnN_many(range(args.warmup, args.warmup + args.steps)))
    kms = pool.ms_per_unit()
    lane_ops = 2 * pairs_per_step_rank
    return {"note": "tie_mode='half' UnN steps (same shape, same keys as the headline): "
                    "estimates in half units 2#{x>z} + #{x==z} over 2 #pairs; step chains on "
                    "{g, h} image pairs (csrc/chain.hip); frac counts 2 lane-ops per pair",
            "value": pairs_per_step_rank * world * args.steps / dt, "unit": "pairs/s",
            "ms_per_step": dt / args.steps * 1e3, "estimate_last_step": float(ests[-1]),
            "chain_path": S._chain_ok(),
            "roofline": {"bound": "valu", "kernel": "k_count_chain<8, half>",
                         "count_kernel_ms": kms,
                         "achieved": lane_ops / (kms * 1e-3) / 1e12,
                         "peak": PEAK_LANE_OPS / 1e12, "unit": "Tlane-op/s",
                         "frac": lane_ops / (kms * 1e-3) / PEAK_LANE_OPS}}


def weak_c3(args, group, rank, world, span, torch):
    """The weak-scaling form of the headline: n = 1e6/class and N = 64 shards PER GPU (the
    per-GPU work of the one-GPU run), K UnN steps over all ranks."""
    from tuplewise.device import ShardedSample
    gen = torch.Generator(device="cuda").manual_seed(3000 + rank)
    X = torch.randn(N_PER_CLASS, dtype=torch.float64, device="cuda", generator=gen) + 0.5
    Z = torch.randn(N_PER_CLASS, dtype=torch.float64, device="cuda", generator=gen)
    S = ShardedSample(X, Z, N_SHARDS, group=group, algo="pairs")
    S.UnN_many(range(70_000, 70_000 + args.warmup + 1))
    dt, ests = span(lambda: S.UnN_many(range(args.warmup, args.warmup + args.steps)))
    k = N_PER_CLASS // N_SHARDS
    pairs = world * N_SHARDS * k * k * args.steps
    return {"note": "weak scaling: n=1e6/class and N=64 prop-SWOR shards PER GPU (8e6/class and "
                    "512 shards at 8 GPUs), one global repartition per step",
            "scaling": "weak", "value": pairs / dt, "unit": "pairs/s",
            "ms_per_step": dt / args.steps * 1e3, "n_per_class_per_gpu": N_PER_CLASS,
            "shards_per_gpu": N_SHARDS, "estimate_last_step": float(ests[-1])}


def main():
    args = parse()
    world = resolve_world(args)
    if args.scaling == "strong" and (args.n % world or args.shards % world):
        sys.stderr.write(f"bench.py: n={args.n}, N={args.shards} do not split over {world} ranks "
                         "(strong scaling; --scaling weak runs them per rank)\n")
        sys.exit(2)
    if world > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(world))
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    group = None
    # TW_BENCH_RCCL_WORLD1=1: a world-size-1 RCCL group with every multi-rank branch forced
    # (TW_FORCE_COLLECTIVES), so each collective of the G > 1 path runs on the one GPU
    rccl1 = world == 1 and os.environ.get("TW_BENCH_RCCL_WORLD1", "") == "1"
    if rccl1:
        os.environ["TW_FORCE_COLLECTIVES"] = "1"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if world > 1 or rccl1:
        # RCCL over xGMI; TW_BENCH_BACKEND=gloo only to rehearse several ranks on one GPU
        backend = os.environ.get("TW_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            # RCCL kernels on a high-priority stream: the repartition's all-to-all runs beside
            # the VALU-bound count kernel of the previous step (ShardedSample.UnN_many)
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                    pg_options=opts)
        else:
            dist.init_process_group(backend)
        group = dist.group.WORLD
    import tuplewise  # noqa: F401
    from tuplewise.device import ShardedSample

    # the headline's problem: strong (default) = BASELINE configs[2]'s fixed n per class and
    # N shards IN TOTAL over the ranks; weak = n and N per rank
    if args.scaling == "strong":
        n, shards = args.n // world, args.shards // world
    else:
        n, shards = args.n, args.shards
    gen = torch.Generator(device="cuda").manual_seed(1000 + rank)
    X = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) + 0.5
    Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen)
    S = ShardedSample(X, Z, shards, group=group, algo="pairs")
    k = n // shards
    pairs_per_step_rank = shards * k * k

    # live kernel timing: HIP events on the stream the C ABI launches on (torch's current
    # stream), created before the timed regions (creating them inside the loop stalled the
    # launch queue: 0.75 ms/step at K = 100 against 0.67 with a pre-made pool)
    kernel_ms = EventPool(torch, 64)
    sample = max(1, args.steps // 20)  # launches per timed event pair
    ops = S.ops
    ops.count = kernel_ms.wrap(ops.count)
    ops.count_step = kernel_ms.wrap(ops.count_step)  # count + next repartition on spare blocks
    ops.count_rank_step = kernel_ms.wrap(ops.count_rank_step)  # the same on rank images
    # the step chains (csrc/chain.hip): one count launch per chunk of steps (weight: its steps)
    # and the chunk's emission
    chain_ms = EventPool(torch, 64)
    ops.count_chain = chain_ms.wrap(ops.count_chain, weight=lambda *a, **kw: a[5])
    # (over ranks the chunk's unpack and count run as one native call: timed together)
    ops.chain_unpack_count = chain_ms.wrap(ops.chain_unpack_count, weight=lambda *a, **kw: a[2])
    emit_ms = EventPool(torch, 64)
    ops.chain_emit = emit_ms.wrap(ops.chain_emit, weight=lambda *a, **kw: len(a[8]))
    chain_path = S._chain_ok()
    rank_ms = EventPool(torch, 8)  # the once-per-call ranking of X u Z (tw_rank_images)
    ops.rank_images = rank_ms.wrap(ops.rank_images)
    ops.rank_images_query = rank_ms.wrap(ops.rank_images_query)
    rank_path = S._rank_path_ok()
    ops.count_sorted_step = kernel_ms.wrap(ops.count_sorted_step)  # sorted count + next
    ops.count_sorted_steps = kernel_ms.wrap(ops.count_sorted_steps)  # all K sorted steps
    # algo="sorted" on the step chains: the exact bucket count of a chunk's bags (weight: steps)
    ops.count_chain_bucket = kernel_ms.wrap(ops.count_chain_bucket, weight=lambda *a, **kw: a[5])

    def barrier():
        if group is not None:
            if dist.get_backend(group) == "nccl":
                dist.barrier(device_ids=[local])
            else:
                dist.barrier()

    span = Span(torch, dist, group, barrier)

    progress(f"headline: {args.steps} UnN steps on {world} rank(s)")
    # settle: untimed steps for >= settle_ms so the timed steps run at the steady-state clock
    # (the chip raises its clock over the first ~10 ms of load; measured 3 % on this step)
    # one untimed run at the timed run's length first: the first K-step UnN_many of a process
    # ran ~7 % slower than the later ones at K = 100 (tools/bench_bisect.py)
    S.UnN_many(range(40_000, 40_000 + args.steps))
    # the process's objects so far (torch's import, the sample, the pools) into the cyclic
    # collector's permanent generation: its passes inside a timed call then scan only the
    # call's own young objects (a 2e6-object heap cost a K = 20 call ~0.15 ms of host time,
    # tools/headline_call_probe.py, profiles/r05s55_headline_call.log).  Before the settle
    # steps: a collection right before the timed call idled the GPU long enough for its clock
    # to drop (the count launch ran at 0.78 of peak instead of 0.95, profiles/r05s57_*)
    import gc
    gc.collect()
    gc.freeze()
    t_s = time.perf_counter()
    while True:
        S.UnN_many(range(20_000, 20_005))
        go = time.perf_counter() - t_s < args.settle_ms * 1e-3
        if group is not None:  # rank 0 decides, so every rank runs the same collectives
            flag = torch.tensor([int(go)], dtype=torch.int64, device="cuda")
            dist.broadcast(flag, 0, group=group)
            go = bool(flag.item())
        if not go:
            break
    S.UnN_many(range(args.warmup))
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    X_start, Z_start = S.X.clone(), S.Z.clone()  # the score-kernel line replays the same steps
    kernel_ms.clear(sample)
    rank_ms.clear()
    chain_ms.clear()
    emit_ms.clear()
    t0 = time.perf_counter()
    # K UnN steps (est.UnNT's loop): repartition i+1 overlaps the counts of step i
    ests = S.UnN_many(range(args.warmup, args.warmup + args.steps))
    est = ests[-1]
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if group is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    kms = float(np.mean([a.elapsed_time(b) for a, b in kernel_ms.used()] or [float("nan")]))
    chain_launch_ms = float(np.mean([a.elapsed_time(b) for a, b in chain_ms.used()]
                                    or [float("nan")]))
    if chain_path:  # per-step device time of the chain count launches
        kms = chain_ms.ms_per_unit()
    emit_step_ms = emit_ms.ms_per_unit() if chain_path else None
    rank_call_ms = float(np.mean([a.elapsed_time(b) for a, b in rank_ms.used()] or [0.0]))

    # the same K steps as a sample's FIRST call: the ranking inside the call (the timed call
    # above carries the images of the previous call's final arrays, device.CARRY_IMAGES —
    # the repartitions never change the multiset the images rank against)
    fresh_line = None
    if chain_path:
        from tuplewise import device as Dv0
        Dv0.CARRY_IMAGES = False
        try:
            S.X, S.Z = X_start.clone(), Z_start.clone()
            rank_ms.clear()
            torch.cuda.synchronize()
            barrier()
            t6 = time.perf_counter()
            ests_fresh = S.UnN_many(range(args.warmup, args.warmup + args.steps))
            torch.cuda.synchronize()
            barrier()
            dt_fresh = time.perf_counter() - t6
            if group is not None:
                tt = torch.tensor([dt_fresh], dtype=torch.float64, device="cuda")
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                dt_fresh = float(tt.item())
            fresh_rank_ms = float(np.mean([a.elapsed_time(b) for a, b in rank_ms.used()]
                                          or [0.0]))
        finally:
            Dv0.CARRY_IMAGES = True
        fresh_line = {
            "note": "the headline's K steps (same keys) as a sample's first UnN_many call: the "
                    "ranking of X u Z inside the timed call (device.CARRY_IMAGES off); the "
                    "headline call carries the images of the previous call's final arrays",
            "value": pairs_per_step_rank * world * args.steps / dt_fresh, "unit": "pairs/s",
            "ms_per_step": dt_fresh / args.steps * 1e3, "ranking_ms_per_call": fresh_rank_ms,
            "same_estimates": bool(ests_fresh == ests)}

    # the same steps with the score-compare kernel (csrc/count.hip: v_cmp_f64 + VALU/SALU
    # counting), for comparison: identical estimates
    score_line = None
    if rank_path:
        from tuplewise import device as Dv
        Dv.RANK_IMAGES = False
        try:
            S.UnN_many(range(60_000, 60_000 + args.warmup))
            S.X, S.Z = X_start, Z_start
            torch.cuda.synchronize()
            barrier()
            kernel_ms.clear(sample)
            t5 = time.perf_counter()
            ests_score = S.UnN_many(range(args.warmup, args.warmup + args.steps))
            torch.cuda.synchronize()
            barrier()
            dt_score = time.perf_counter() - t5
            kms_score = float(np.mean([a.elapsed_time(b) for a, b in kernel_ms.used()]))
        finally:
            Dv.RANK_IMAGES = True
        score_line = {
            "note": "the same K steps (same keys, same estimates) with the score-compare kernel "
                    "k_count_complete (csrc/count.hip): one v_cmp_f64 per 64 pairs, counted "
                    "half on the VALU (carry-add) and half on the scalar unit (s_bcnt1)",
            "value": pairs_per_step_rank * world * args.steps / dt_score, "unit": "pairs/s",
            "ms_per_step": dt_score / args.steps * 1e3, "kernel_ms": kms_score,
            "frac": pairs_per_step_rank / (kms_score * 1e-3) / PEAK_LANE_OPS,
            "same_estimates": bool(ests_score == ests)}

    progress("half ties")
    half_line = half_ties_line(args, group, span, torch, X_start, Z_start, shards,
                               pairs_per_step_rank, world)

    # same workload, exact sort + binary-search count (csrc/rankcount.hip): logical pairs/s
    same_counts = bool(torch.equal(S.local_counts(), (setattr(S, "algo", "sorted"),
                                                      S.local_counts())[1]))
    S.algo = "sorted"
    from tuplewise import device as _D
    sorted_chain = (S._chain_ok() and S.max_nz <= _D.CHAIN_BUCKET_MAX
                    and hasattr(S.ops, "count_chain_bucket"))
    S.UnN_many(range(10_000, 10_000 + args.warmup))
    torch.cuda.synchronize()
    barrier()
    kernel_ms.clear(sample if not sorted_chain else 1)
    emit_ms.clear()
    rank_ms.clear()
    t1 = time.perf_counter()
    # same keys as the timed all-pairs steps
    est_sorted = S.UnN_many(range(args.warmup, args.warmup + args.steps))[-1]
    torch.cuda.synchronize()
    barrier()
    dt_sorted = time.perf_counter() - t1
    if group is not None:
        tt = torch.tensor([dt_sorted], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt_sorted = float(tt.item())
    if sorted_chain:  # per step: the bags' bucket count + the emission (+ the call's ranking)
        sorted_parts = {"bucket_count_ms_per_step": kernel_ms.ms_per_unit(),
                        "emission_ms_per_step": emit_ms.ms_per_unit(),
                        "ranking_ms_per_call": (float(np.mean([a.elapsed_time(b)
                                                               for a, b in rank_ms.used()]))
                                                if rank_ms.used() else None)}
        kms_sorted = (sorted_parts["bucket_count_ms_per_step"]
                      + sorted_parts["emission_ms_per_step"])
    else:  # one tw_count_pairs_sorted_steps call carries all K steps: per-step device time
        sorted_parts = None
        kms_sorted = float(np.mean([a.elapsed_time(b) for a, b in kernel_ms.used()])) / args.steps
    S.algo = "pairs"

    # incomplete U-statistic (BASELINE config C3: B pairs per shard + a repartition per step;
    # cs.UnNBT's loop, device-RNG draws): pairs/s and the k_count_rng roofline
    ops.count_rng = kernel_ms.wrap(ops.count_rng)
    ops.count_rng_step = kernel_ms.wrap(ops.count_rng_step)  # count + next repartition
    # over ranks (round 6) UnNB_many walks the step chains: one tw_count_pairs_chain_rng launch
    # counts every step of a chunk (weight = its steps, so kernel_ms stays per step)
    inc_chain = bool(S.coll and S._chain_rng_ok())
    ops.count_chain_rng = kernel_ms.wrap(ops.count_chain_rng, weight=lambda *a, **k: a[5])
    B_inc = args.incomplete_B
    S.UnNB_many(B_inc, 5, range(30_000, 30_000 + args.warmup))
    torch.cuda.synchronize()
    barrier()
    kernel_ms.clear(sample)
    t2 = time.perf_counter()
    est_inc = S.UnNB_many(B_inc, 1234, range(args.warmup, args.warmup + args.steps))[-1]
    torch.cuda.synchronize()
    barrier()
    dt_inc = time.perf_counter() - t2
    if group is not None:
        tt = torch.tensor([dt_inc], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt_inc = float(tt.item())
    kms_inc = kernel_ms.ms_per_unit()
    ops.count_rng = ops.count_rng.__wrapped__
    ops.count_rng_step = ops.count_rng_step.__wrapped__
    ops.count_chain_rng = ops.count_chain_rng.__wrapped__
    inc_pairs_rank = shards * B_inc
    progress("incomplete replay")
    inc_replay = incomplete_replay(X, Z, shards, B_inc)
    progress("strong C3")
    strong = None if args.no_strong else strong_c3(args, group, rank, world, barrier, torch, dist)

    # BASELINE.json configs[1] (C2): complete AUC U-statistic, n = 1e5/class, ONE shard (est.Un,
    # estimation-experiment/main.py:29-31), 1e10 pairs per call; no repartition.  One-shot
    # counts of this size rank X u Z and count packed f32 images (ShardedSample.local_counts):
    # the call = the ranking + one count launch, both timed
    n1 = 100_000
    g1 = torch.Generator(device="cuda").manual_seed(7 + rank)
    X1 = torch.randn(n1, dtype=torch.float64, device="cuda", generator=g1) + 0.5
    Z1 = torch.randn(n1, dtype=torch.float64, device="cuda", generator=g1)
    S1 = ShardedSample(X1, Z1, 1, algo="pairs")
    c2_rank = S1._oneshot_rank_ok()
    c2_count = EventPool(torch, 64)
    c2_rankms = EventPool(torch, 64)
    S1.ops.count = c2_count.wrap(S1.ops.count)
    S1.ops.count_chain = c2_count.wrap(S1.ops.count_chain)
    S1.ops.rank_images_query = c2_rankms.wrap(S1.ops.rank_images_query)
    for _ in range(20):  # ~7 ms of warm calls: the clock settles after the previous lines
        S1.local_counts()
    torch.cuda.synchronize()
    c2_count.clear()
    c2_rankms.clear()
    reps1 = 20
    t3 = time.perf_counter()
    for _ in range(reps1):
        c1 = S1.local_counts()
    torch.cuda.synchronize()
    dt1 = time.perf_counter() - t3
    kms1 = float(np.mean([a.elapsed_time(b) for a, b in c2_count.used()]))
    rms1 = float(np.mean([a.elapsed_time(b) for a, b in c2_rankms.used()] or [0.0]))
    c1 = int(c1.sum())
    call_ms = dt1 / reps1 * 1e3
    single = {"note": "BASELINE configs[1]: est.Un complete AUC, n=1e5/class, one shard "
                      "(1e10 pairs per call), inputs resident, per-rank; "
                      + ("one-shot count on rank images: the ranking of X u Z "
                         "(tw_rank_images_query, compact) + one k_count_chain launch, both "
                         "inside the timed call" if c2_rank else
                         "the double-compare kernel k_count_complete"),
              "value": n1 * n1 * reps1 / dt1, "unit": "pairs/s", "ms_per_call": call_ms,
              "count": c1, "estimate": c1 / (n1 * n1),
              "roofline": {"bound": "valu",
                           "kernel": "k_count_chain" if c2_rank else "k_count_complete",
                           "achieved": n1 * n1 / (kms1 * 1e-3) / 1e12,
                           "peak": PEAK_LANE_OPS / 1e12, "unit": "Tlane-op/s",
                           "frac": n1 * n1 / (kms1 * 1e-3) / PEAK_LANE_OPS, "kernel_ms": kms1,
                           "ranking_ms": rms1 if c2_rank else None,
                           "frac_with_ranking": n1 * n1 / ((kms1 + rms1) * 1e-3) / PEAK_LANE_OPS,
                           "frac_wall": n1 * n1 / (call_ms * 1e-3) / PEAK_LANE_OPS}}
    del S1, X1, Z1

    # BASELINE.json configs[0] (C1, plumbing): estimation-experiment/main.py's UnNT on host
    # arrays through the drop-in API (host shuffles as the reference, one device launch for
    # the T repetitions), n = 1000/class, N = 10, T = 4; the reference restated on the CPU
    progress("plumbing C1")
    c1 = plumbing_C1(rank == 0 and world == 1 and not args.no_cpu_baseline)

    count_kernel = ("k_count_chain" if chain_path else "k_count_rank" if rank_path
                    else "k_count_complete")
    traffic, traffic_plain = pmc_traffic(count_kernel)
    total_pairs = pairs_per_step_rank * world * args.steps
    value = total_pairs / dt
    achieved = pairs_per_step_rank / (kms * 1e-3)  # lane-ops/s, 1 compare per pair (strict)
    out = {
        "metric": "pair comparisons/sec (node) for sharded AUC U-stat at n=1e6/class (UnN, "
                  "N=64 prop-SWOR shards, device repartition each step)",
        "value": value,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle_ms": args.settle_ms,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: X~N(0.5,1), Z~N(0,1) float64 scores generated on the device",
        "config": {"workload": "UnN sharded complete AUC U-statistic (estimation-experiment/"
                               "main.py:72-74) + device repartition per step, K steps as "
                               "est.UnNT's loop (BASELINE configs[2])",
                   "repartition": ("device keyed Feistel permutation per step (a device-RNG "
                                   "stand-in for np.random.shuffle, pinned against the oracle's "
                                   "restatement and validated statistically, DESIGN.md §4.5); "
                                   "the NumPy-order drop-in path is the drop_in_C3 line"),
                   "n_per_class_total": n * world if args.scaling == "weak" else args.n,
                   "shards_total": shards * world,
                   "n_per_class_per_gpu": n, "shards_per_gpu": shards,
                   "pairs_per_step_per_gpu": pairs_per_step_rank,
                   "parallelism": (f"dp{world}: shards over ranks, "
                                   + ("RCCL" if os.environ.get("TW_BENCH_BACKEND", "nccl")
                                      == "nccl" else "gloo (rehearsal)")
                                   + (" step chains: all-gather of the sample once per call, "
                                      "each rank walks its own elements' repartitions, one "
                                      "all-to-all of {image, position} records per chunk of "
                                      "<= 32 steps, every step of a chunk counted in one launch"
                                      if S._chain_ok() else " all-to-all repartition")
                                   + " + all-reduce of counts"
                                   if world > 1 else
                                   ("dp1: one GPU; step chains: every element walks the K "
                                    "repartitions (k_chain_emit, one launch per chunk of <= 32 "
                                    "steps) and one k_count_chain launch counts every shard of "
                                    "the chunk's steps"
                                    + (" — RCCL world-size-1 rehearsal: every multi-rank "
                                       "collective forced" if S.coll else "")))},
        "roofline": {"bound": "valu", "kernel": count_kernel,
                     "achieved": achieved / 1e12, "peak": PEAK_LANE_OPS / 1e12,
                     "unit": "Tlane-op/s", "frac": achieved / PEAK_LANE_OPS,
                     # the same launches under rocprofv3 --kernel-trace (committed summary)
                     "frac_traced": traced_count_chain(args.steps) if chain_path else None,
                     "count_kernel_ms": kms, "traffic": traffic,
                     "traffic_count_only": traffic_plain,
                     "traffic_unit": ("HBM bytes per step: the chunk's k_count_chain launch / its "
                                      "steps" if chain_path else "HBM bytes per launch"),
                     "traffic_emit_per_step": pmc_emit_traffic() if chain_path else None,
                     # the count reads each step's 4-B images of its n + n scores once
                     "algorithmic_bytes_per_step": (4 * 2 * n if chain_path
                                                    else None),
                     "traffic_source": ("rocprofv3 --pmc FETCH_SIZE+WRITE_SIZE of this kernel "
                                        "at the one-GPU shape (profiles/*count_pmc*.json), "
                                        "not measured at this run's per-rank shape"
                                        if world > 1 else
                                        "rocprofv3 --pmc FETCH_SIZE+WRITE_SIZE of this kernel "
                                        "at this shape (profiles/*count_pmc*.json)"),
                     "ranking_ms_per_call": rank_call_ms if rank_path or chain_path else None,
                     "chain_count_launch_ms": chain_launch_ms if chain_path else None,
                     "chain_emit_ms_per_step": emit_step_ms,
                     "note": ("1 compared pair = 1 lane-op of the contract (f64 vector "
                              "lane-op peak); the count compares packed f32 rank images of "
                              "the scores (two pairs per lane per instruction: a clamped "
                              "v_pk_add_f32 and an accumulating one), exact by construction; "
                              "the ranking of X u Z runs in a sample's first UnN_many call; "
                              "later calls carry the images of the final arrays "
                              "(device.CARRY_IMAGES: the timed call, ranking_ms_per_call = 0; "
                              "first_call_ranking times the same steps with the ranking) "
                              if rank_path or chain_path else "1 v_cmp_f64 lane-op per pair; ")
                             + ("step chains (csrc/chain.hip): every element walks the call's "
                                "repartitions once (k_chain_emit, chain_emit_ms_per_step) and "
                                "ONE k_count_chain launch counts all steps of a chunk "
                                "(chain_count_launch_ms); count_kernel_ms = that launch per "
                                "step; traffic = HBM bytes per step of the count launch "
                                "(FETCH_SIZE+WRITE_SIZE) from the committed rocprofv3 --pmc "
                                "summary" if chain_path else
                                "the timed launch also carries the next repartition on its tail "
                                "blocks; traffic = HBM bytes/launch (FETCH_SIZE+WRITE_SIZE) from "
                                "the committed rocprofv3 --pmc summary of this kernel: the timed "
                                "launch, and a launch without the repartition")},
        "first_call_ranking": fresh_line,
        "score_compare_kernel": score_line,
        "half_ties": half_line,
        "estimate_last_step": float(est),
        "plumbing_C1": c1,
        "single_shard_C2": single,
        "sorted_count": ({
            "note": "same UnN steps with the exact O(n+m) count (algo='sorted' on the step "
                    "chains: the call's ranking, the chains' (step, shard) image bags, each bag "
                    "counted by a counting sort of its integer z images in LDS, "
                    "tw_count_pairs_chain_bucket; bit-identical estimates and arrays); "
                    "count_kernels_ms = bucket count + emission per step (the ranking once per "
                    "call beside it); pairs are logical, not compared one by one",
            "value": total_pairs / dt_sorted, "unit": "logical pairs/s",
            "ms_per_step": dt_sorted / args.steps * 1e3, "count_kernels_ms": kms_sorted,
            "parts": sorted_parts,
            "estimate_last_step": float(est_sorted),
            "counts_identical_to_all_pairs": same_counts,
            # algorithmic bytes per element and step: its 4-B image appended to a bag and read
            # back by the count (positions and records stay in registers across a chunk)
            "roofline": {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                         "bytes_per_element": 8,
                         "achieved": 8 * 2 * n / (kms_sorted * 1e-3) / 1e9,
                         "frac": 8 * 2 * n / (kms_sorted * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "note": "count_kernels_ms per step against 8 B per element; both "
                                 "kernels are issue-bound (the emission's Feistel walk and LDS "
                                 "histogram, the bucket count's LDS counting sort), not "
                                 "bandwidth-bound"}}
            if sorted_chain else {
            "note": "same UnN steps with the exact O((n+m) log m)-class count (algo='sorted':"
                    " value buckets of z in LDS for shards of <= 16384, else sort + binary "
                    "search; bit-identical estimates; the K steps in one call with the "
                    "partition kept as destination-bucketed records between steps, so each "
                    "repartition streams; count_kernels_ms = that call's device time / K); "
                    "pairs are logical, not compared one by one",
            "value": total_pairs / dt_sorted, "unit": "logical pairs/s",
            "ms_per_step": dt_sorted / args.steps * 1e3, "count_kernels_ms": kms_sorted,
            "estimate_last_step": float(est_sorted),
            "counts_identical_to_all_pairs": same_counts,
            # algorithmic bytes per step: every record {8-B value, 4-B position} of both samples
            # read once and written once to its next bucket (csrc/records.h)
            # (one GPU: the K steps are one records launch; over ranks the count is per step)
            "roofline": None if world > 1 else {
                         "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                         "bytes_per_element": 24,
                         "achieved": 24 * 2 * n / (kms_sorted * 1e-3) / 1e9,
                         "frac": 24 * 2 * n / (kms_sorted * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "note": "count_kernels_ms per step against 24 B per element; the step "
                                 "is latency-bound (Feistel + load/atomic/store chain, DESIGN "
                                 "4.6), not bandwidth-bound"}}),
        "incomplete": {
            "note": "UnNBT loop (compute_stats.py:104-123): a device repartition + B device-"
                    "drawn pairs per shard (Philox4x32-10, two pairs per block, Lemire maps) "
                    + ("counted on the step chains' exact-position rank-image bags, one "
                       "exchange and one count launch per chunk (tw_count_pairs_chain_rng)"
                       if inc_chain else
                       "counted per step on float32 score images in LDS; one launch per step "
                       "(the next repartition rides in the count threads)"),
            "B_per_shard": B_inc, "value": inc_pairs_rank * world * args.steps / dt_inc,
            "unit": "pairs/s", "ms_per_step": dt_inc / args.steps * 1e3,
            "estimate_last_step": float(est_inc),
            "roofline": {"bound": "valu",
                         "kernel": "k_count_rng_chain" if inc_chain else "k_count_rng_img",
                         "frac_vs_int32_op_peak": INC_LANE_OPS * inc_pairs_rank / (kms_inc * 1e-3)
                         / INT_LANE_OPS_MEASURED,
                         "int32_op_peak": INT_LANE_OPS_MEASURED / 1e12,
                         "achieved": INC_LANE_OPS * inc_pairs_rank / (kms_inc * 1e-3) / 1e12,
                         "peak": PEAK_LANE_OPS / 1e12, "unit": "Tlane-op/s",
                         "frac": INC_LANE_OPS * inc_pairs_rank / (kms_inc * 1e-3)
                         / PEAK_LANE_OPS,
                         "kernel_ms": kms_inc,
                         "note": f"{INC_LANE_OPS} lane-ops per pair (SURVEY.md §8(d) contract "
                                 "constant: 2 Philox4x32-10 words + 2 range maps + 1 compare); "
                                 "kernel_ms = per step: over ranks the chunk's "
                                 "tw_count_pairs_chain_rng launch / its steps; in one process "
                                 "the whole tw_count_pairs_rng_step call (one "
                                 "kernel: float32 score images in LDS, Philox draws, compares, "
                                 "and the next repartition's gathers in the same threads); "
                                 "frac is against the f64 lane-op "
                                 "peak of the contract, frac_vs_int32_op_peak against the "
                                 "measured 32-bit integer VOP2 issue rate (the Philox work is "
                                 "32-bit integer)"}},
        "incomplete_replay": inc_replay,
        "strong_C3": strong,
    }
    # Every section after the headline runs guarded: an exception there is recorded in the line
    # ({"error": ...}) and ends the remaining sections, on every rank alike (over ranks the
    # ranks agree through one small all-reduce per section), so the headline is still printed
    broken = []

    def guarded(name, fn, collective=True, independent=False):
        # collective=False: a section only rank 0 runs (no agreement round); independent: it
        # runs even after a failed section (no collectives, nothing it needs from the others)
        if broken and not independent:
            return {"error": f"skipped: an earlier section failed ({broken[0]})"}
        err = None
        try:
            if os.environ.get("TW_BENCH_FAIL_SECTION") == name:  # the guard's own test hook
                raise RuntimeError(f"forced failure of section {name} (TW_BENCH_FAIL_SECTION)")
            res = fn()
        except Exception as e:  # noqa: BLE001 — recorded in the line, the run goes on
            res, err = None, f"{type(e).__name__}: {e}"
            sys.stderr.write(f"bench.py: section {name} failed: {err}\n")
        if group is not None and collective:
            flag = torch.tensor([0 if err is None else 1], dtype=torch.int32, device="cuda")
            if dist.get_backend(group) != "nccl":
                flag = flag.cpu()
            dist.all_reduce(flag, group=group)
            if int(flag.item()) and err is None:
                err = "failed on another rank"
        if err is not None:
            broken.append(name)
            return {"error": err}
        return res

    if world > 1:
        # the weak-scaling form of the headline (per-GPU work of the one-GPU run)
        progress("weak C3")
        out["weak_C3"] = guarded("weak_C3", lambda: weak_c3(args, group, rank, world, span,
                                                            torch))

    sec = {"metric": "SGD steps/sec (pairwise hinge, linear scorer; no evaluation)"}

    def sgd_section():  # fills `sec` line by line (a failure keeps the lines before it)
        # reference CPU numbers (BASELINE.md, 1 core): 262-413 steps/s at C4, 3.3-9.4 at C5';
        # at G > 1 every line runs over the ranks (shards split, one all-gather of the shard
        # gradients per step; SGDEngine(group=)), C4/C5 checked against a one-rank run
        chk = 20 if world > 1 else 0
        g = group
        progress("C4 device RNG")
        sec["C4_shuttle_shape"] = sgd_steps_per_s(9117, 702, 10, 100, 100, 25, 4000, 2, group=g,
                                                  span=span, check_prefix=chk)
        # BASELINE configs[3] names pairwise-LOGISTIC SGD: the same loop with loss="logistic"
        # (the weight sigma(S) per drawn pair instead of the hinge filter)
        progress("C4 logistic")
        sec["C4_shuttle_shape_logistic"] = sgd_steps_per_s(9117, 702, 10, 100, 100, 25, 4000, 2,
                                                           group=g, span=span,
                                                           check_prefix=chk, loss="logistic")
        progress("C4 partitioned")
        sec["C4_shuttle_shape_partitioned"] = sgd_steps_per_s(
            9117, 702, 10, 100, 100, 25, 2000, 2, layout="partitioned", group=g, span=span,
            check_prefix=chk)
        progress("C4 replay")
        sec["C4_shuttle_shape_replay"] = sgd_replay_steps_per_s(2000, group=g, span=span)
        progress("C4 end to end (replay, device)")
        sec["C4_end_to_end_with_evaluation_replay"] = learning_end_to_end(2000, "replay", g, span)
        sec["C4_end_to_end_with_evaluation_device"] = learning_end_to_end(2000, "device", g, span)
        c5 = None if args.no_c5 else sgd_data(C5_N, C5_N, 512)
        if c5 is not None:
            progress("C5 B = 100, 4096, partitioned")
            sec["C5_scaled_d512"] = sgd_steps_per_s(C5_N, C5_N, 512, 256, 100, 25, 500, 2,
                                                    group=g, span=span, data=c5,
                                                    check_prefix=chk)
            sec["C5_scaled_d512_B4096"] = sgd_steps_per_s(C5_N, C5_N, 512, 256, 4096, 25, 100,
                                                          1, group=g, span=span, data=c5)
            sec["C5_scaled_d512_partitioned"] = sgd_steps_per_s(
                C5_N, C5_N, 512, 256, 100, 25, 100, 1, layout="partitioned", group=g,
                span=span, data=c5, check_prefix=chk)
            del c5
            torch.cuda.empty_cache()
        if world == 1 and not args.no_c5:
            # one-GPU extensions (north_star item (2)): the complete-block gradient
            progress("C5 complete-block gradients")
            sec["C5_scaled_d512_complete_gradient"] = sgd_complete_steps_per_s(
                C5_N, C5_N, 512, 256, 3)
            sec["C5_scaled_d512_complete_gradient_logistic"] = sgd_complete_steps_per_s(
                C5_N, C5_N, 512, 256, 2, loss="logistic")
        return sec

    if not args.no_sgd:
        res = guarded("secondary", sgd_section)
        out["secondary"] = sec if res is sec else {**sec, **res}
        if not args.no_tradeoff:
            out["tradeoff_reshuffle_mod"] = guarded(
                "tradeoff_reshuffle_mod", lambda: tradeoff_curve(
                    args, group, span, rank == 0 and world == 1 and not args.no_cpu_baseline))
    if rank == 0 and not args.no_cpu_baseline:
        # at every G (the GPU work of every rank is done; the others wait at the final barrier):
        # the reference's est.UnN restated on 1 core, and the same blocks spread over the host
        # cores of this run's CPU share: on a whole 8-GPU node every core of the affinity mask
        # (the node-wide figure); on the pool's smaller boxes 16 per GPU (os.cpu_count() and the
        # affinity mask show the whole machine, which those boxes share out per GPU).  Host
        # work only: run even after a failed GPU section, its own failure recorded
        progress("CPU baselines")
        try:
            out["cpu_baseline"] = cpu_baseline(args.n, args.shards, args.cpu_shards)
            aff = len(os.sched_getaffinity(0))
            node = world >= 8
            share = aff if node else min(16 * world, aff)
            allc = cpu_baseline_all_cores(args.n, args.shards, share)
            allc["label"] = ((f"{share} host cores = the whole affinity mask of the {world}-GPU "
                              "node" if node else
                              f"{share} host cores = 16 per GPU x {world} GPU(s), the pool's "
                              "CPU share") + f" (affinity mask {aff}, os.cpu_count() "
                             f"{os.cpu_count()})")
            out["cpu_baseline"]["all_cores"] = allc
            out["incomplete"]["cpu_baseline"] = cpu_baseline_incomplete(
                args.n, args.shards, B_inc, args.cpu_inc_shards)
        except Exception as e:  # noqa: BLE001
            sys.stderr.write(f"bench.py: CPU baselines failed: {type(e).__name__}: {e}\n")
            out.setdefault("cpu_baseline", {})["error"] = f"{type(e).__name__}: {e}"
    if rank == 0 and world == 1:
        progress("drop-in C3")

        def drop_in():
            d3 = drop_in_C3()
            if "value" in out.get("cpu_baseline", {}):  # the reference restated: T x est.UnN
                unn_s = out["cpu_baseline"]["value"]
                d3["cpu_port_ms_per_call"] = 4 * N_SHARDS * (n // N_SHARDS) ** 2 / unn_s * 1e3
                d3["cpu_port_note"] = ("4 x the cpu_baseline est.UnN time (same blocks, NumPy "
                                       "broadcast compare, 1 core); not rerun here (~23 s)")
            return d3
        out["drop_in_C3"] = guarded("drop_in_C3", drop_in, collective=False, independent=True)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if group is not None:
        barrier()  # rank 0's CPU baselines run after every rank's GPU work
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
