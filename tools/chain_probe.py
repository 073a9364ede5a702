"""Probe the step chains (csrc/chain.hip) on ONE GPU: (1) one UnN_many call of K steps at the
bench shape (n = 1e6/class, N = 64) through the chains against the one-launch-per-step path, and
(2) what rank r of G does in one strong-scaling call (1e6/class and 64 shards in total, 64/G
shards per rank), the ranking included: the Z structure of the whole Z and the images of the
rank's own 1/G of the elements (tw_rank_images_query), the chain emission into G send buckets,
a device copy of the send buffer standing in for the all-to-all (the same bytes; RCCL's xGMI
transfer is not simulated), the unpack, (round 5) a device copy standing in for the Z
all-gather and the local part of the counts' reduction, one count launch of K x 64/G bags and the inverse-chain
gather of the rank's final arrays.  Reports ms per call and the efficiency against the one-GPU
call / G.  Round 5: the efficiency takes both ranks' UNinstrumented times (the per-part event
markers of the parts run cost a G = 8 rank's K = 4 call ~0.07 ms, which the round-4 figure
charged to rank G - 1); and every G is timed twice — a sample's FIRST call (the ranking, the Z
all-gather it waits for) and its later calls with the images carried (device.CARRY_IMAGES: no
ranking; the all-gathers of both samples and of both record arrays, as device copies, and the
inverse-chain gathers of scores and records on a side stream beside the counts), each against
the one-GPU call of the same kind / G.  The sub-chunk schedules of the round-5 study are in
profiles/r05s36_chain_probe.log.  Run on the GPU box:
    python tools/chain_probe.py [K ...]      (TW_PROBE_G=8: only those G)"""
import os
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np
import torch

import tuplewise  # noqa: F401
from tuplewise import _lib as L
from tuplewise import device as D
from tuplewise.device import HipOps, ShardedSample, prop_swor_layout

torch.cuda.set_device(0)
gen = torch.Generator(device="cuda").manual_seed(1)
n, N = 1_000_000, 64
Ks = [int(a) for a in sys.argv[1:]] or [20, 4, 100]
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen)
M64 = 2 ** 64 - 1


def ev_time(fn, reps, warm=3):
    # (warm: a sample's first calls allocate; one warm call left the one-GPU product call
    # ~0.1 ms above its steady 1.89 ms at K = 4, profiles/r05s43_sync_probe.log)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0.record()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, (time.perf_counter() - t0) / reps * 1e3


def one_gpu_call(K, chain, carry):
    D.CHAIN_STEPS = chain
    D.CARRY_IMAGES = carry
    S = ShardedSample(X.clone(), Z.clone(), N, algo="pairs")
    base = [1000]

    def call():
        base[0] += K
        S.UnN_many(range(base[0], base[0] + K))
    try:
        return ev_time(call, 10)
    finally:
        D.CHAIN_STEPS = True
        D.CARRY_IMAGES = True


# every element's records (one ranking of the whole sample): the carried records all ranks hold
XR, ZR = HipOps().rank_images_query(Z, X, Z, L.TW_F64)


def rank_call(G, r, K, parts=False, carried=False):
    """Rank r's device work in one call of the strong problem split over G ranks, the
    product's schedule (device.CHAIN_SUB = 0: one exchange, unpack and count per chunk).
    carried: a later call of the sample (device.CARRY_IMAGES): no Z all-gather to wait for and
    no ranking; the all-gathers (device copies) and the final gathers of scores and records on
    a side stream."""
    ops = HipOps()
    nl, Nl = n // G, N // G
    x_off, z_off, _ = prop_swor_layout(nl, nl, Nl)
    xo, zo = torch.from_numpy(x_off).cuda(), torch.from_numpy(z_off).cuda()
    kx = int(nl / Nl)
    kz = int(2 * nl / Nl) - kx
    xq, zq = X[r * nl:(r + 1) * nl], Z[r * nl:(r + 1) * nl]
    C = min(K, D.CHAIN_MAX)
    tot = 2 * nl
    cap = max(1, tot // G + tot // (8 * G) + 1024)
    send = torch.empty(G * C * (cap + 1), dtype=torch.int64, device="cuda")
    recv = torch.empty_like(send)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    x_bag = torch.empty((C, nl), dtype=torch.float32, device="cuda")
    z_bag = torch.empty((C, nl), dtype=torch.float32, device="cuda")
    xpos = torch.empty(nl, dtype=torch.int32, device="cuda")
    zpos = torch.empty(nl, dtype=torch.int32, device="cuda")
    counts = torch.empty((K, Nl), dtype=torch.int64, device="cuda")
    cur = torch.empty(C * 2 * (Nl + 1), dtype=torch.int32, device="cuda")
    keys = list(range(500, 500 + K))
    kxs = [(2 * k) & M64 for k in keys]
    kzs = [(2 * k + 1) & M64 for k in keys]
    t = {}

    def mark(name, fn):
        if not parts:
            return fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn()
        e1.record()
        t.setdefault(name, []).append((e0, e1))
        return out

    # the all-gathered arrays (device copies of the same bytes)
    Xg, Zg, RXg, RZg = (torch.empty_like(a) for a in (X, Z, XR, ZR))
    full = torch.zeros(K * N + 1, dtype=torch.int64, device="cuda")
    fs = torch.cuda.Stream()
    xr_c, zr_c = XR[r * nl:(r + 1) * nl], ZR[r * nl:(r + 1) * nl]

    # round 6 (device.FINAL_EXCHANGE): the final arrays and carried records by one exchange of
    # the walked elements, forked on the side stream once the last emission has run
    # (device.FINAL_EARLY, the fork at the call's start on tw_chain_walk positions, measured
    # slower: profiles/r06s22_*)
    tot = 2 * nl
    fcap = max(1, tot // G + tot // (8 * G) + 1024)
    fsend = torch.empty(G * (fcap + 1) * 3, dtype=torch.int64, device="cuda")
    frecv = torch.empty_like(fsend)
    fcur = torch.zeros(G, dtype=torch.int64, device="cuda")
    Xf, Zf = torch.empty_like(xq), torch.empty_like(zq)
    RXf, RZf = torch.empty(nl, dtype=torch.int64, device="cuda"), torch.empty(
        nl, dtype=torch.int64, device="cuda")

    def final_exchange(xr, zr):
        ops.chain_final_pack(xq, xr, xpos, zq, zr, zpos, G, fcap, fcur, fsend, flag)
        frecv.copy_(fsend)  # the all-to-all (device copy)
        ops.chain_final_scatter(frecv, G, fcap, nl, nl, Xf, RXf, Zf, RZf, flag)

    def side_work(xr, zr, ev=None):
        # (ev: the last emission's event — the fork is enqueued after the count launch)
        if ev is not None:
            fs.wait_event(ev)
        else:
            fs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(fs):
            final_exchange(xr, zr)

    def call():
        main = torch.cuda.current_stream()
        if carried:
            xr, zr = xr_c, zr_c
        else:
            if G > 1:  # the Z all-gather the ranking waits for
                mark("all-gather Z (device copy)", lambda: Zg.copy_(Z))
            xr, zr = mark("ranking", lambda: ops.rank_images_query(Z, xq, zq, L.TW_F64))
        if G > 1 and carried:  # every rank's async Z all-gather (device copy)
            fs.wait_stream(main)
            with torch.cuda.stream(fs):
                Zg.copy_(Z)
        for i0 in range(0, K, C):
            c = min(C, K - i0)
            first = i0 == 0
            if G == 1:  # one process: straight into the bags
                mark("emit", lambda: ops.chain_emit(xr, zr, False, xpos, zpos, first, 0, 1,
                                                    kxs[i0:i0 + c], kzs[i0:i0 + c], kx, kz, Nl,
                                                    x_bag=x_bag, z_bag=z_bag, cursors=cur))
                mark("count", lambda: ops.count_chain(x_bag, xo, z_bag, zo, Nl, c, nl, nl, kx,
                                                      kz, False, counts[i0:i0 + c]))
            else:
                mark("emit", lambda: ops.chain_emit(xr, zr, False, xpos, zpos, first, r, G,
                                                    kxs[i0:i0 + c], kzs[i0:i0 + c], kx, kz, Nl,
                                                    send=send, cap=cap, flag=flag))
                ev = torch.cuda.Event()
                ev.record()
                sz = G * c * (cap + 1)
                mark("exchange (device copy)", lambda: recv[:sz].copy_(send[:sz]))
                # (round 6: the product's receive side in one native call)
                mark("unpack + count", lambda: ops.chain_unpack_count(
                    recv, G, c, cap, False, nl, nl, x_bag, z_bag, flag, kx, kz, Nl, xo, zo, kx,
                    kz, counts[i0:i0 + c]))
            if G > 1 and i0 + c >= K:  # the final exchange beside the last chunk's count
                if parts:
                    mark("final exchange (side stream in the product)",
                         lambda: final_exchange(xr, zr))
                else:
                    side_work(xr, zr, ev)
        if G == 1:
            mark("final scatter (scores, records)",
                 lambda: (ops.chain_scatter(X, xpos, Z, zpos),
                          ops.chain_scatter(xr, xpos, zr, zpos)))
        else:
            main.wait_stream(fs)
            # the counts' all-reduce (with the overflow flag) stands in as its local fill
            mark("counts reduce (local part)",
                 lambda: full[:-1].view(K, N)[:, r * Nl:(r + 1) * Nl].copy_(counts))
    ms, host = ev_time(call, 5)
    if parts:
        t = {k: sum(a.elapsed_time(b) for a, b in v) / 8 for k, v in t.items()}
    return ms, host, t


for K in Ks:
    one_gpu_call(K, True, True)  # warm: the process's first calls run before the clock has risen
    ch, ch_host = one_gpu_call(K, True, True)
    chf, _ = one_gpu_call(K, True, False)
    st, st_host = one_gpu_call(K, False, True)
    print(f"K={K}: one GPU, step chains {ch:.3f} ms/call with carried images ({ch / K:.4f} "
          f"ms/step; host {ch_host:.3f}), {chf:.3f} ranking every call; one launch per step "
          f"{st:.3f} ms/call ({st / K:.4f} ms/step)", flush=True)
    for G in [int(g) for g in os.environ.get("TW_PROBE_G", "1,2,4,8").split(",")]:
        for carried, ideal, label in ((False, chf, "first call (ranking)"),
                                      (True, ch, "later calls (carried images)")):
            ms = [rank_call(G, r, K, carried=carried)[0] for r in sorted({0, G - 1})]
            _, _, parts = rank_call(G, G - 1, K, parts=True, carried=carried)
            print(f"  G={G} {label}: ranks 0/{G - 1} " + "/".join(f"{v:.3f}" for v in ms)
                  + f" ms/call, efficiency {ideal / G / max(ms):.3f} (ideal: the one-GPU call "
                  f"/ G = {ideal / G:.3f}); parts (instrumented rank {G - 1}) "
                  + ", ".join(f"{k} {v:.3f}" for k, v in parts.items()), flush=True)
