"""Phase breakdown of k_rank_codes_bucket at the bench shape (64 shards of 15625 + 15625
doubles): builds tools/_dbg/libtw_phase.so from csrc/{capi,count,rankcount}.hip with
-DTW_PHASE_TIMING (thread 0 of every block stamps clock64() at each phase boundary), runs one
tw_count_pairs_idx32_ws call per rank-code mode and prints the median cycles per phase.
Phases: 0 start, 1 loads + range, 2 coarse histogram + prefix, 3 fine map + histogram, 4
scatter, 5 codes.  (The instrumented build is for this study only.)"""
import ctypes
import pathlib
import subprocess
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "trade-offs-in-distributed-tuplewise-estimation-and-learning_amd" / "csrc"
OUT = ROOT / "tools" / "_dbg" / "libtw_phase.so"

if len(sys.argv) > 1 and sys.argv[1] == "build":
    # extra -D flags: python tools/phase_codes.py build [-DTW_IDX_STREAM_ONLY ...] [name]
    flags = [a for a in sys.argv[2:] if a.startswith("-D")]
    names = [a for a in sys.argv[2:] if not a.startswith("-D")]
    if names:
        OUT = OUT.with_name(f"libtw_{names[0]}.so")
    OUT.parent.mkdir(exist_ok=True)
    objs = []
    for src in ("capi.hip", "count.hip", "rankcount.hip"):
        o = OUT.parent / (OUT.stem + "_" + src + ".o")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC",
                        "-std=c++17", "-ffp-contract=off", "-DTW_PHASE_TIMING"] + flags +
                       ["-c", str(CSRC / src), "-o", str(o)], check=True)
        objs.append(str(o))
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    str(OUT)] + objs, check=True)
    sys.exit(0)

import torch  # noqa: E402  (before the dlopen: one HIP runtime)

if len(sys.argv) > 1 and sys.argv[1] != "build":
    OUT = OUT.with_name(f"libtw_{sys.argv[1]}.so")
lib = ctypes.CDLL(str(OUT))
vp = ctypes.c_void_p
k, N, B = 15625, 64, 1_000_000
g = torch.Generator(device="cuda").manual_seed(1000)
X = torch.randn(N * k, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(N * k, dtype=torch.float64, device="cuda", generator=g)
base = (torch.arange(N, device="cuda", dtype=torch.int64) * k).repeat_interleave(B)
ix = (base + torch.randint(0, k, (N * B,), device="cuda", generator=g)).to(torch.int32)
iz = (base + torch.randint(0, k, (N * B,), device="cuda", generator=g)).to(torch.int32)
off = torch.arange(N + 1, dtype=torch.int64, device="cuda") * k
po = torch.arange(N + 1, dtype=torch.int64, device="cuda") * B
lib.tw_count_pairs_rng_work_bytes.restype = ctypes.c_int64
lib.tw_count_pairs_rng_work_bytes.argtypes = [ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
                                              ctypes.c_int32, ctypes.c_int32]
wb = lib.tw_count_pairs_rng_work_bytes(N, k, k, 0, 0)
work = torch.empty(wb, dtype=torch.uint8, device="cuda")
out = torch.empty(N, dtype=torch.int64, device="cuda")
fn = lib.tw_count_pairs_idx32_ws
fn.argtypes = [vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, vp, vp, vp,
               ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, vp, ctypes.c_int64, vp, vp]
lib.tw_count_rng_set_codes.argtypes = [ctypes.c_int32]
buf = (ctypes.c_ulonglong * 65536)()
for mode in (1, 2):
    lib.tw_count_rng_set_codes(mode)
    for _ in range(3):
        rc = fn(X.data_ptr(), off.data_ptr(), Z.data_ptr(), off.data_ptr(), N, k, k,
                ix.data_ptr(), iz.data_ptr(), po.data_ptr(), B, 0, 0, work.data_ptr(), wb,
                out.data_ptr(), None)
        assert rc == 0
    torch.cuda.synchronize()
    assert lib.tw_debug_phases(buf, 65536) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8)[:256].astype(np.int64)
    d = np.diff(a[:, :6], axis=1)
    tot = a[:, 5] - a[:, 0]
    print(f"mode {mode}: median cycles per phase {np.median(d, axis=0).tolist()} "
          f"total median {np.median(tot):.0f} max {tot.max()}  block start spread "
          f"{a[:, 0].max() - a[:, 0].min()} (clock64 ticks; per-CU counters)", flush=True)

# whole-call time of the int32 replay count with this build (HIP events), per load variant
lib.tw_count_rng_set_codes(1)
lib.tw_count_idx_set_variant.argtypes = [ctypes.c_int32]
for var in range(6):
    lib.tw_count_idx_set_variant(var)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(20)]
    for e0, e1 in ev:
        e0.record()
        fn(X.data_ptr(), off.data_ptr(), Z.data_ptr(), off.data_ptr(), N, k, k, ix.data_ptr(),
           iz.data_ptr(), po.data_ptr(), B, 0, 0, work.data_ptr(), wb, out.data_ptr(), None)
        e1.record()
    torch.cuda.synchronize()
    ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
    print(f"{OUT.name} variant {var}: whole call {ms * 1e3:.1f} us = "
          f"{8 * N * B / (ms * 1e-3) / 1e12:.2f} TB/s of int32 indices", flush=True)
lib.tw_count_idx_set_variant(0)
