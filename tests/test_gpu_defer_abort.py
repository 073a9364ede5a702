"""Deferred evaluations (learning._DeferredEvals) check the SGD engine's abort word from the
copy taken with each evaluation (no device-wide wait per evaluation): an evaluation enqueued
after a persistent segment gave up at its grid barrier raises before its statistics reach
p_learn; the evaluations before it are written."""
import pytest


@pytest.mark.gpu
def test_deferred_eval_abort_word_raises_before_history(gpu):
    import torch
    from tuplewise import learning as lr
    w = torch.zeros((10, 1), dtype=torch.float64, device="cuda")
    ctl = torch.zeros((2,), dtype=torch.int32, device="cuda")
    res = torch.arange(4, dtype=torch.float64, device="cuda")
    seen = []
    d = lr._DeferredEvals(w, (10, 1), slots=4, ctl=ctl[1:2])
    d.push(0, res, w, lambda i, h, wv: seen.append(i))
    torch.cuda._sleep(1000)  # the later evaluation is still in flight when the abort lands
    ctl[1] = 1  # a segment between the two evaluations timed out at its barrier
    d.push(25, res, w, lambda i, h, wv: seen.append(i))
    with pytest.raises(RuntimeError, match="grid barrier timed out"):
        d.drain()
    assert seen == [0]
