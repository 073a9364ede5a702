"""Host time of the drop-in's per-step count enqueue (_blocks.CompleteCount.enqueue_device on
a side stream) and of its parts, at the C3 shape (64 prop-SWOR blocks of 15625 + 15625 in a
1e6 + 1e6 sample): the offsets' pinned upload, the stream waits, the count launch.
    python tools/time_enqueue.py"""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np
import torch

from tuplewise import _blocks as Bk, _engine as E, _lib as L


def host_us(fn, reps=200):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    dt = (time.perf_counter() - t0) / reps * 1e6
    torch.cuda.synchronize()
    return dt


n, N = 1_000_000, 64
k = n // N
xd = torch.randn(n, dtype=torch.float64, device="cuda")
zd = torch.randn(n, dtype=torch.float64, device="cuda")
blocks = [Bk.Block((i * k, (i + 1) * k), (i * k, (i + 1) * k), None) for i in range(N)]
spec = Bk.CompleteCount(False)
cs, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
xo = Bk._slice_offsets(blocks, "x")
zo = Bk._slice_offsets(blocks, "z")
res = {
    "slice_offsets": host_us(lambda: (Bk._slice_offsets(blocks, "x"),
                                      Bk._slice_offsets(blocks, "z"))),
    "to_device_many pageable": host_us(lambda: L.to_device_many([xo, zo])),
    "to_device_many pinned": host_us(lambda: L.to_device_many([xo, zo], pinned=True)),
    "3 wait_stream": host_us(lambda: (cs.wait_stream(torch.cuda.current_stream()),
                                      cs.wait_stream(s2), cs.wait_stream(s3))),
    "4 record_stream": host_us(lambda: [a.record_stream(cs) for a in (xd, zd, xd, zd)]),
}
xod, zod = L.to_device_many([xo, zo])
for algo in ("sorted", "pairs"):
    res[f"count_launch {algo}"] = host_us(
        lambda: E.count_launch(xd, xod, zd, zod, N, k, k, L.TW_F64, L.TW_PRED_GT, algo), 50)
res["enqueue_device (side stream)"] = host_us(
    lambda: spec.enqueue_device(xd, zd, blocks, stream=cs, after=(s2, s3)), 50)
res["enqueue_device + done"] = host_us(
    lambda: spec.enqueue_device(xd, zd, blocks, stream=cs, after=(s2, s3))(), 20)
for key, v in res.items():
    print(f"{key}: {v:.1f} us host", flush=True)
