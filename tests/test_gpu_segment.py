"""Wide rows (32 < d <= 512: per-step gradient launches) with the device RNG drawing each
reshuffle's SWR rows in the gradient kernel (learning.SWR_IN_KERNEL) against the row-table
path: the same statistics bit for bit.  (The wide persistent segment kernel these tests once
covered, tw_sgd_segment, measured slower than the per-step launches at C5 and was removed in
round 5.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


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


@pytest.mark.parametrize("d,N,B,loss", [(64, 8, 64, "hinge"), (512, 256, 100, "hinge"),
                                        (100, 37, 300, "logistic"), (40, 200, 16, "hinge"),
                                        (512, 3, 2000, "hinge")])
@pytest.mark.parametrize("swr", [True, False])
def test_wide_fused_step_equals_two_launches(gpu, d, N, B, loss, swr, monkeypatch):
    """learning.WIDE_FUSED (tw_sgd_step_wide: the previous step's update spread over the
    gradient launch's blocks behind a grid barrier) against the gradient + update launches:
    w after segments of 1, 2, 7 and 40 steps through reshuffles (mod 5), bit for bit, SWR rows
    drawn in the kernel or read from the row tables; N = 200 with d = 40 puts one column per
    block on the first 40 blocks and none on the rest."""
    import torch
    import tuplewise.learning as lr
    rng = np.random.RandomState(d + N)
    n = 4000
    X = torch.from_numpy(rng.normal(0.3, 1.0, size=(n, d))).cuda()
    Z = torch.from_numpy(rng.normal(0.0, 1.0, size=(n, d))).cuda()
    w0 = torch.from_numpy(rng.normal(size=(d, 1))).cuda()
    monkeypatch.setattr(lr, "SWR_IN_KERNEL", swr)
    out = {}
    for fused in (True, False):
        monkeypatch.setattr(lr, "WIDE_FUSED", fused)
        e = lr.SGDEngine(X, Z, w0, N, B, margin=1, reg=0.05, learning_rate=0.01,
                         optim_type="momentum", loss=loss)
        assert e.wide_fused == fused
        e.enable_device_rng(4242)
        traj, done = [], 0
        for seg in (1, 2, 7, 40):
            use_swr = lr.SWR_IN_KERNEL and e.swr_segments_ok()
            if use_swr:
                e.run_segment(seg, False, graphs=True, swr_mod=5)
            else:
                i = done
                while i < done + seg:
                    nxt = min(done + seg, (i // 5 + 1) * 5)
                    e.run_segment(nxt - i, i % 5 == 0, graphs=True)
                    i = nxt
            done += seg
            traj.append(e.w_host().copy())
        e.check()
        out[fused] = traj
    for a, b in zip(out[True], out[False]):
        assert np.array_equal(a, b)
