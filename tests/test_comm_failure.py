"""RCCL failure detection of the single-process communicator (csrc/comm.hip) on
CPU: a stub library (tests/native/rccl_stub.cpp, bound through TW_RCCL_LIB) reports a failed
peer or a collective that never completes; tw_comm_wait must return an error instead of
hanging, abort every device's communicator, and leave the handle dead for later calls.  Each
case runs in a fresh process (the library binds RCCL once per process)."""
import ctypes
import json
import os
import pathlib
import subprocess
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]

_CHILD = r"""
import ctypes, json, sys
sys.path.insert(0, sys.argv[1])
from tuplewise import _lib as L
lib = L.lib()
stub = ctypes.CDLL(sys.argv[2])
comm = ctypes.c_int32(-1)
devs = (ctypes.c_int32 * 2)(0, 1)
out = {"init": lib.tw_comm_init(2, devs, ctypes.byref(comm))}
P = ctypes.c_void_p * 2
streams = P(None, None)
bufs = P(None, None)
out["gather"] = lib.tw_allgather_u64(comm.value, bufs, bufs, 4, streams)
out["wait"] = lib.tw_comm_wait(comm.value, streams, 2000)
out["msg"] = lib.tw_last_error().decode()
out["aborts"] = stub.stub_aborts()
out["again"] = lib.tw_allgather_u64(comm.value, bufs, bufs, 4, streams)
out["again_msg"] = lib.tw_last_error().decode()
out["gathers"] = stub.stub_gathers()
print(json.dumps(out))
"""


@pytest.fixture(scope="module")
def stub(tmp_path_factory):
    so = tmp_path_factory.mktemp("rccl") / "librccl_stub.so"
    subprocess.run(["g++", "-O1", "-shared", "-fPIC", "-o", str(so),
                    str(ROOT / "tests" / "native" / "rccl_stub.cpp")], check=True)
    return so


@pytest.mark.parametrize("mode", ["error", "inprogress"])
def test_comm_wait_fails_instead_of_hanging(stub, mode):
    env = dict(os.environ, TW_RCCL_LIB=str(stub), STUB_MODE=mode, HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-c", _CHILD, str(ROOT), str(stub)], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["init"] == 0 and out["gather"] == 0 and out["gathers"] == 2
    assert out["wait"] == 2  # TW_ERR_HIP, returned (no hang)
    if mode == "error":
        assert "asynchronous error" in out["msg"] and "stub: system error" in out["msg"]
    else:  # the collective never reports completion: the stream query or the deadline ends it
        assert "aborted" in out["msg"]
    assert out["aborts"] == 2  # both devices' communicators
    assert out["again"] == 2 and "aborted after an RCCL failure" in out["again_msg"]


_SLOW = r"""
import ctypes, json, sys
sys.path.insert(0, sys.argv[1])
import torch
from tuplewise import _lib as L
lib = L.lib()
stub = ctypes.CDLL(sys.argv[2])
comm = ctypes.c_int32(-1)
devs = (ctypes.c_int32 * 1)(0)
out = {"init": lib.tw_comm_init(1, devs, ctypes.byref(comm))}
a = torch.randn(4096, 4096, device="cuda")
torch.cuda.synchronize()
for _ in range(200):  # ~0.1-0.3 s of queued work before the collective
    a = a @ a
    a = a / a.norm()
P = ctypes.c_void_p * 1
streams = P(L.stream_handle().value)
bufs = P(a.data_ptr())
out["busy_at_gather"] = not torch.cuda.current_stream().query()
out["gather"] = lib.tw_allgather_u64(comm.value, bufs, bufs, 4, streams)
out["wait"] = lib.tw_comm_wait(comm.value, streams, 20)  # a 20 ms deadline
out["msg"] = lib.tw_last_error().decode()
out["aborts"] = stub.stub_aborts()
print(json.dumps(out))
"""


@pytest.mark.gpu
def test_comm_wait_deadline_starts_after_prior_work(stub):
    """tw_comm_wait's deadline covers the collective, not the work queued before it
    on the same stream — a long queue ahead of the all-gather (here ~0.2 s against a 20 ms
    deadline) must not be taken for an RCCL failure (no abort)."""
    env = dict(os.environ, TW_RCCL_LIB=str(stub), STUB_MODE="ok")
    r = subprocess.run([sys.executable, "-c", _SLOW, str(ROOT), str(stub)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["init"] == 0 and out["gather"] == 0 and out["busy_at_gather"]
    assert out["wait"] == 0, out["msg"]
    assert out["aborts"] == 0


_WEDGED = r"""
import ctypes, json, sys
sys.path.insert(0, sys.argv[1])
import torch
from tuplewise import _lib as L
lib = L.lib()
stub = ctypes.CDLL(sys.argv[2])
comm = ctypes.c_int32(-1)
devs = (ctypes.c_int32 * 1)(0)
out = {"init": lib.tw_comm_init(1, devs, ctypes.byref(comm))}
out["set"] = lib.tw_comm_set_prior_timeout(ctypes.c_int64(30))  # 30 ms for the prior work
a = torch.randn(4096, 4096, device="cuda")
torch.cuda.synchronize()
for _ in range(400):  # ~0.2-0.6 s queued ahead of the collective: "wedged" against 30 ms
    a = a @ a
    a = a / a.norm()
P = ctypes.c_void_p * 1
streams = P(L.stream_handle().value)
bufs = P(a.data_ptr())
out["gather"] = lib.tw_allgather_u64(comm.value, bufs, bufs, 4, streams)
out["wait"] = lib.tw_comm_wait(comm.value, streams, 60000)
out["msg"] = lib.tw_last_error().decode()
out["aborts"] = stub.stub_aborts()
torch.cuda.synchronize()  # the queued work drains before the process ends
print(json.dumps(out))
"""


@pytest.mark.gpu
def test_comm_wait_prior_work_has_its_own_deadline(stub):
    """the work queued before a collective is waited for under its own deadline
    (tw_comm_set_prior_timeout), so a stream that never drains ends in an error and an aborted
    communicator instead of an unbounded wait."""
    env = dict(os.environ, TW_RCCL_LIB=str(stub), STUB_MODE="ok")
    r = subprocess.run([sys.executable, "-c", _WEDGED, str(ROOT), str(stub)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["init"] == 0 and out["set"] == 0 and out["gather"] == 0
    assert out["wait"] == 2 and "prior deadline" in out["msg"], out
    assert out["aborts"] == 1
