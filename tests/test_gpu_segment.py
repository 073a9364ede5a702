"""The persistent SGD segment kernel (tw_sgd_segment, csrc/sgdseg.hip) against per-step
launches (k_hinge_grad_stream + k_sgd_update): identical bits for every step of every segment.

Wide rows (32 < d <= 512) on one GPU take the segment path in SGDEngine.run_segment /
run_replay_segment; the per-step launches are themselves checked against the reference's
trajectory (tests/test_gpu_learning.py) and the gradient restatement (tests/test_gpu_parity.py).
Cases: d = 512 (the C5 width, the FULL kernel) and d = 40 (masked columns); device and replay
draws; hinge and logistic; momentum and SGD; B above one index phase (1024 pairs); a grid of 3
blocks so that blocks loop over several shards and update several column groups each; the
next step's first chunks prefetched as rows (default) and as indices only.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(X, Z, w0, N, B, optim, loss, mode, segment, graphs, segs):
    import torch
    import tuplewise.learning as lr
    old = lr.SEGMENT_KERNEL
    lr.SEGMENT_KERNEL = True
    try:
        eng = lr.SGDEngine(X, Z, w0, N, B, 1.0, 0.05, 0.01, optim, loss=loss)
    finally:
        lr.SEGMENT_KERNEL = old
    assert not eng.fused
    if not segment:
        eng.segment = False
    else:
        assert eng.segment
    kx, kz = X.shape[0] // N, Z.shape[0] // N
    ws = []
    if mode == "device":
        eng.enable_device_rng(2024)
        for n, resh in segs:
            eng.run_segment(n, resh, graphs)
            ws.append(eng.w_host())
    else:
        rr = np.random.RandomState(9)
        eng.set_shards([rr.randint(0, X.shape[0], kx) for _ in range(N)],
                       [rr.randint(0, Z.shape[0], kz) for _ in range(N)])
        for tag, (n, _) in enumerate(segs):
            d = np.stack([np.stack([rr.randint(0, kx, (N, B)), rr.randint(0, kz, (N, B))])
                          for _ in range(n)]).astype(np.int64)
            eng.run_replay_segment(torch.from_numpy(d).cuda(), n, graphs, tag)
            ws.append(eng.w_host())
    torch.cuda.synchronize()
    eng.check()
    return np.stack(ws), eng.dw.cpu().numpy(), eng.grads.cpu().numpy()


@pytest.mark.parametrize("d,N,B,grid", [(512, 16, 100, 0), (40, 7, 37, 0), (512, 8, 1500, 0),
                                        (40, 10, 30, 3), (512, 9, 50, 3)])
@pytest.mark.parametrize("mode", ["device", "replay"])
def test_segment_equals_per_step_launches(gpu, d, N, B, grid, mode):
    from tuplewise import _lib as L
    rng = np.random.RandomState(d + N + B)
    X = rng.normal(0.2, 1.0, size=(N * 40, d))
    Z = rng.normal(0.0, 1.0, size=(N * 30, d))
    w0 = rng.normal(0, 0.1, size=(d, 1))
    segs = ((1, True), (2, False), (7, True), (5, False))
    cases = [("momentum", "hinge"), ("SGD", "logistic")] if grid == 0 else [("momentum", "hinge")]
    for optim, loss in cases:
        ref = _run(X, Z, w0, N, B, optim, loss, mode, False, False, segs)
        assert np.all(np.isfinite(ref[0])) and np.abs(ref[0][-1] - w0).max() > 0
        L.call("tw_sgd_segment_set_grid", grid)
        try:
            for graphs, rows in ((False, 1), (True, 1), (False, 0)):
                L.call("tw_sgd_segment_set_prefetch", rows)
                got = _run(X, Z, w0, N, B, optim, loss, mode, True, graphs, segs)
                for a, b, what in zip(got, ref, ("w", "dw", "grads")):
                    assert np.array_equal(a, b), (what, optim, loss, graphs, rows)
        finally:
            L.call("tw_sgd_segment_set_grid", 0)
            L.call("tw_sgd_segment_set_prefetch", 1)


def test_segment_learning_process_matches_per_step(gpu, monkeypatch):
    """learning_process with the device RNG at a wide shape: the same norm_w / AUC history with
    the segment kernel as with per-step launches."""
    import tuplewise.learning as lr
    rng = np.random.RandomState(4)
    n, d = 4000, 64
    X = rng.normal(0.3, 1.0, size=(n, d))
    Z = rng.normal(0.0, 1.0, size=(n, d))
    hist = []
    for seg in (False, True):
        monkeypatch.setattr(lr, "SEGMENT_KERNEL", seg)
        mon = np.random.RandomState(1)
        p = {"N": 8, "B": 64, "margin": 1.0, "reg": 0.01, "learning_rate": 0.05,
             "n_it": 60, "reshuffle_mod": 10, "eval_mod": 20, "w_init": np.full((d, 1), 0.01),
             "test_X": X[:500], "test_Z": Z[:500], "train_X": X, "train_Z": Z,
             "train_mon_pairs": list(zip(mon.randint(0, n, 300), mon.randint(0, n, 300)))}
        np.random.seed(7)
        lr.learning_process(X, Z, p, rng_mode="device")
        hist.append((p["norm_w"], p["tr_AUC"]))
    assert hist[0] == hist[1]


@pytest.mark.parametrize("mod", [1, 3, 10])
def test_wide_swr_in_kernel_equals_row_tables(gpu, mod, monkeypatch):
    """learning.SWR_IN_KERNEL for wide rows (d = 64: per-step gradient launches,
    tw_pair_grad_rng_swr drawing each reshuffle's rows in the kernel, segments cut at
    evaluations only) against the row-table path: the same statistics bit for bit."""
    import tuplewise.learning as lr
    rng = np.random.RandomState(5)
    n, d = 3000, 64
    X = rng.normal(0.3, 1.0, size=(n, d))
    Z = rng.normal(0.0, 1.0, size=(n, d))
    hist = {}
    for swr in (True, False):
        monkeypatch.setattr(lr, "SWR_IN_KERNEL", swr)
        mon = np.random.RandomState(2)
        p = {"N": 8, "B": 64, "margin": 1.0, "reg": 0.01, "learning_rate": 0.05,
             "n_it": 47, "reshuffle_mod": mod, "eval_mod": 20, "w_init": np.full((d, 1), 0.01),
             "test_X": X[:400], "test_Z": Z[:400], "train_X": X, "train_Z": Z,
             "train_mon_pairs": list(zip(mon.randint(0, n, 300), mon.randint(0, n, 300)))}
        np.random.seed(9)
        lr.learning_process(X, Z, p, rng_mode="device")
        hist[swr] = p
    for k in ("norm_w", "bc_AUC", "br_AUC", "tc_AUC", "tr_AUC"):
        assert hist[True][k] == hist[False][k], k
