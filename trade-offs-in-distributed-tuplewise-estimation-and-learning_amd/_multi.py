"""Single-process multi-device execution of the drop-in estimators.

The reference's "N workers" are a serial loop inside one Python process
(learning-experiment/compute_stats.py:71-91, estimation-experiment/main.py:48-68), so a
reference script calling est.UnNT / cs.UnNBT / est.replicate makes ONE process's calls.  This
module lets those unchanged calls use every GPU of the node: the blocks of a call are cut into
contiguous groups of about equal work, each group is uploaded to and counted on its own device
(one HIP stream per slot, all groups enqueued before any result is read), and the per-block
integers or sums are combined in block order — by an RCCL all-gather over xGMI when the slots
are distinct devices (tw_allgather_u64 / _f64, csrc/comm.hip), else by host copies.  Results
are identical to one device: every block is computed by the same kernel on the same data.

Devices: set_devices([...]) or TW_DEVICES="0,1,..." (a device may repeat: two slots on one GPU
get two streams — how the path is tested on a one-GPU box); default: all visible devices, or
only the current one inside a multi-process launch (LOCAL_WORLD_SIZE / WORLD_SIZE > 1).
Calls whose work is below MIN_WORK (pair compares) stay on the current device.
"""
from __future__ import annotations

import ctypes
import os
import warnings

import numpy as np

from . import _lib as L

# work (all-pairs compare equivalents, BlockSpec.work) below which a call stays on one device:
# 2^33 is ~0.25 ms of one MI355X's count kernel, about what spreading costs (per-device
# uploads, launches, the gather)
MIN_WORK = 1 << 33
_DEVICES = None
_STREAMS = {}
_COMMS = {}


def set_devices(devs=None, min_work: int | None = None):
    """Devices the drop-in calls spread their blocks over (None: TW_DEVICES or all visible);
    min_work: the work threshold (pair compares) below which a call stays on one device."""
    global _DEVICES, MIN_WORK
    _DEVICES = None if devs is None else [int(d) for d in devs]
    if min_work is not None:
        MIN_WORK = int(min_work)


def devices() -> list:
    if _DEVICES is not None:
        return list(_DEVICES)
    env = os.environ.get("TW_DEVICES")
    if env:
        return [int(v) for v in env.split(",") if v.strip()]
    if int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1"))) > 1:
        # one process per GPU (torchrun): the other GPUs belong to the other ranks
        return [L.torch().cuda.current_device()]
    n = L.torch().cuda.device_count()
    return list(range(n)) if n > 0 else [0]


def split(weights, parts: int) -> list:
    """Contiguous ranges [a, b) of len(weights) items, one per part, of about equal total
    weight (greedy on the cumulative sum; empty ranges when there are fewer items)."""
    w = np.asarray(weights, dtype=np.float64)
    n = len(w)
    if n == 0:
        return [(0, 0)] * parts
    cum = np.concatenate([[0.0], np.cumsum(w)])
    tot = cum[-1]
    cuts = [0]
    for p in range(1, parts):
        c = int(np.searchsorted(cum, tot * p / parts, side="left"))
        cuts.append(min(max(c, cuts[-1]), n))
    cuts.append(n)
    return [(cuts[i], cuts[i + 1]) for i in range(parts)]


def slots_for(total_work: float, n_items: int):
    """The device slots a call of this size is spread over, or None (stay on one device)."""
    devs = devices()
    if len(devs) < 2 or n_items < 2 or total_work < MIN_WORK:
        return None
    return devs


class _Slot:
    """Device + dedicated stream of slot k (torch's current device/stream inside)."""

    def __init__(self, dev: int, k: int):
        t = L.torch()
        self.dev, self.k = dev, k
        key = (dev, k)
        if key not in _STREAMS:
            _STREAMS[key] = t.cuda.Stream(device=dev)
        self.stream = _STREAMS[key]
        self._ctx = None

    def __enter__(self):
        t = L.torch()
        self._dctx = t.cuda.device(self.dev)
        self._dctx.__enter__()
        self._sctx = t.cuda.stream(self.stream)
        self._sctx.__enter__()
        return self

    def __exit__(self, *exc):
        self._sctx.__exit__(*exc)
        self._dctx.__exit__(*exc)
        return False


def spread(items, weight, enqueue):
    """Enqueue every group of items on its slot: enqueue(sub_items) -> a device tensor of one
    value per item (int64 or float64), left in flight.  Returns [(slot, tensor, n_items)]."""
    devs = devices()
    groups = split([weight(b) for b in items], len(devs))
    out = []
    for k, (dev, (a, b)) in enumerate(zip(devs, groups)):
        if a == b:
            continue
        slot = _Slot(dev, k)
        with slot:
            out.append((slot, enqueue(items[a:b]), b - a))
    return out


def _comm(devs: tuple):
    """RCCL communicator over distinct devices (cached), or None when RCCL is unavailable."""
    if devs not in _COMMS:
        c = ctypes.c_int32(-1)
        arr = (ctypes.c_int32 * len(devs))(*devs)
        rc = L.lib().tw_comm_init(len(devs), arr, ctypes.byref(c))
        _COMMS[devs] = int(c.value) if rc == L.TW_OK else None
    return _COMMS[devs]


def gather(parts) -> np.ndarray:
    """The values of spread()'s groups, in item order, on the host (int64 or float64)."""
    t = L.torch()
    if not parts:
        return np.zeros(0)
    dt = parts[0][1].dtype
    devs = tuple(s.dev for s, _, _ in parts)
    comm = _comm(devs) if len(set(devs)) == len(devs) and len(devs) > 1 else None
    if comm is None:  # host copies, each on its slot's stream
        vals = []
        for slot, v, _ in parts:
            with slot:
                vals.append(v.cpu().numpy())
        return np.concatenate(vals)
    # all-gather over RCCL: every slot contributes its values padded to the longest group
    M = max(n for _, _, n in parts)
    send, recv, streams = [], [], []
    for slot, v, n in parts:
        with slot:
            pad = t.zeros((M,), dtype=dt, device=v.device)
            pad[:n].copy_(v)
            send.append(pad)
            recv.append(t.empty((len(parts) * M,), dtype=dt, device=v.device))
            streams.append(slot.stream.cuda_stream)
    P = ctypes.c_void_p * len(parts)
    fn = "tw_allgather_f64" if dt == t.float64 else "tw_allgather_u64"
    try:
        L.call(fn, comm, P(*[a.data_ptr() for a in send]), P(*[a.data_ptr() for a in recv]), M,
               P(*streams))
        # bounded wait: an RCCL failure (a peer that never answers) aborts the communicator
        # and raises here instead of hanging the copy below (tw_comm_wait)
        L.call("tw_comm_wait", comm, P(*streams), 0)
    except (L.TuplewiseError, ValueError) as err:
        _COMMS[devs] = None  # this device set gathers on the host from now on
        warnings.warn(f"RCCL all-gather failed ({err}); gathering on the host", RuntimeWarning)
        vals = []
        for slot, v, n in parts:
            with slot:
                vals.append(v[:n].cpu().numpy())
        return np.concatenate(vals)
    with parts[0][0]:
        allv = recv[0].cpu().numpy().reshape(len(parts), M)
    return np.concatenate([allv[k, :n] for k, (_, _, n) in enumerate(parts)])
