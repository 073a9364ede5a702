"""Probe configs[2]'s INCOMPLETE leg over ranks on ONE GPU: what rank r of
G does in one UnNB_many call of the strong problem (n = 1e6 per class, N = 64 shards in all,
64/G per rank, B pairs per shard, T steps), in two designs:

  per-step   the round-5 path (device.py _run_steps over ranks): per step the fixed-capacity
             pack of the rank's scores into G buckets (tw_exchange_pack_fixed), the exchange, the
             scatter into place (tw_scatter_buckets) and the device-RNG count of the rank's
             shards (tw_count_pairs_rng_ws);
  chains     device.CHAIN_RNG (round 6): per chunk of <= 32 steps ONE emission of the rank's
             rank images into (destination, step) buckets (tw_chain_emit), ONE exchange, the
             exact-position unpack (tw_chain_unpack_exact) and ONE count launch of all the
             chunk's (step, shard) bags (tw_count_pairs_chain_rng); the final arrays by the
             inverse chains on a side stream; a sample's first call also ranks (Z all-gather +
             tw_rank_images_query), later calls carry the images.

The exchange is a device copy of the send buffer (the same bytes; RCCL's xGMI transfer and its
latency are not simulated), the counts' all-reduce its local fill.  Efficiency = (the one-GPU
product call / G) / the slower of ranks 0 and G-1.  Run on the GPU box:
    python tools/chain_rng_probe.py [T ...]"""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch

import tuplewise  # noqa: F401
from tuplewise import _lib as L
from tuplewise import device as D
from tuplewise.device import HipOps, ShardedSample, prop_swor_layout

torch.cuda.set_device(0)
gen = torch.Generator(device="cuda").manual_seed(1)
n, N, B = 1_000_000, 64, 1_000_000
Ts = [int(a) for a in sys.argv[1:]] or [4, 20]
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen)
M64 = 2 ** 64 - 1
XR, ZR = HipOps().rank_images_query(Z, X, Z, L.TW_F64)


def ev_time(fn, reps, warm=3):
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


def one_gpu_call(T):
    S = ShardedSample(X.clone(), Z.clone(), N, algo="pairs")
    base = [1000]

    def call():
        base[0] += T
        S.UnNB_many(B, base[0], range(base[0], base[0] + T))
    return ev_time(call, 10)[0]


def rank_setup(G, r):
    nl, Nl = n // G, N // G
    x_off, z_off, _ = prop_swor_layout(nl, nl, Nl)
    return nl, Nl, torch.from_numpy(x_off).cuda(), torch.from_numpy(z_off).cuda(), x_off, z_off


def per_step_call(G, r, T):
    ops = HipOps()
    nl, Nl, xo, zo, x_off, z_off = rank_setup(G, r)
    kx = int(x_off[1] - x_off[0])
    tot = 2 * nl
    cap = max(1, min(tot, tot // G + tot // (8 * G) + 1024))
    cursor = torch.zeros(G, dtype=torch.int64, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    send = torch.empty((G * (cap + 1), 2), dtype=torch.int64, device="cuda")
    recv = torch.empty_like(send)
    st = {"X": X[r * nl:(r + 1) * nl].clone(), "Z": Z[r * nl:(r + 1) * nl].clone()}
    full = torch.zeros(T * N + 1, dtype=torch.int64, device="cuda")

    def call():
        outs = []
        for t in range(T):
            key = 700 + t
            ops.exchange_pack_fixed(st["X"], st["Z"], r, G, (2 * key) & M64,
                                    (2 * key + 1) & M64, cap, cursor, send, flag)
            recv.copy_(send)  # the exchange (device copy)
            XZ = torch.empty(2 * nl, dtype=torch.float64, device="cuda")
            ops.scatter_buckets(recv, G, cap, XZ, flag)
            st["X"], st["Z"] = XZ[:nl], XZ[nl:]
            outs.append(ops.count_rng(st["X"], xo, st["Z"], zo, Nl, B, 5 + t, r * Nl, L.TW_F64,
                                      L.TW_PRED_GT, max_nx=kx, max_nz=kx))
        full[:-1].view(T, N)[:, r * Nl:(r + 1) * Nl].copy_(torch.stack(outs))
    return ev_time(call, 5)[0]


def chain_call(G, r, T, carried, parts=False):
    ops = HipOps()
    nl, Nl, xo, zo, x_off, z_off = rank_setup(G, r)
    kx = int(x_off[1] - x_off[0])
    kz = int(2 * nl / Nl) - kx
    C = min(T, D.CHAIN_MAX)
    tot = 2 * nl
    cap = max(1, tot // G + tot // (8 * G) + 1024)
    send = torch.empty(G * C * (cap + 1), dtype=torch.int64, device="cuda")
    recv = torch.empty_like(send)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    x_bag = torch.empty((C, nl), dtype=torch.float32, device="cuda")
    z_bag = torch.empty((C, nl), dtype=torch.float32, device="cuda")
    xpos = torch.empty(nl, dtype=torch.int32, device="cuda")
    zpos = torch.empty(nl, dtype=torch.int32, device="cuda")
    counts = torch.empty((T, Nl), dtype=torch.int64, device="cuda")
    keys = list(range(500, 500 + T))
    kxs = [(2 * k) & M64 for k in keys]
    kzs = [(2 * k + 1) & M64 for k in keys]
    xq, zq = X[r * nl:(r + 1) * nl], Z[r * nl:(r + 1) * nl]
    xr_c, zr_c = XR[r * nl:(r + 1) * nl], ZR[r * nl:(r + 1) * nl]
    Xg, Zg, RXg, RZg = (torch.empty_like(a) for a in (X, Z, XR, ZR))
    full = torch.zeros(T * N + 1, dtype=torch.int64, device="cuda")
    fs = torch.cuda.Stream()
    t = {}

    def mark(name, fn):  # parts: events around each launch (the side stream's work serial)
        if not parts:
            return fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn()
        e1.record()
        t.setdefault(name, []).append((e0, e1))
        return out

    # round 6 (device.FINAL_EXCHANGE): the final arrays and carried records by one exchange
    # of the walked elements, forked on the side stream once the last emission has run
    # (device.FINAL_EARLY, the fork at the call's start on tw_chain_walk positions, measured
    # slower: profiles/r06s22_*)
    fcap = max(1, tot // G + tot // (8 * G) + 1024)
    fsend = torch.empty(G * (fcap + 1) * 3, dtype=torch.int64, device="cuda")
    frecv = torch.empty_like(fsend)
    fcur = torch.zeros(G, dtype=torch.int64, device="cuda")
    Xf, Zf = torch.empty_like(xq), torch.empty_like(zq)
    RXf = torch.empty(nl, dtype=torch.int64, device="cuda")
    RZf = torch.empty(nl, dtype=torch.int64, device="cuda")

    def final(xr, zr):
        ops.chain_final_pack(xq, xr, xpos, zq, zr, zpos, G, fcap, fcur, fsend, flag)
        frecv.copy_(fsend)  # the all-to-all (device copy)
        ops.chain_final_scatter(frecv, G, fcap, nl, nl, Xf, RXf, Zf, RZf, flag)

    def call():
        main = torch.cuda.current_stream()
        if carried:
            xr, zr = xr_c, zr_c
        else:
            Zg.copy_(Z)
            xr, zr = mark("ranking", lambda: ops.rank_images_query(Zg, xq, zq, L.TW_F64))
        if carried:  # every rank's async Z all-gather (device copy)
            fs.wait_stream(main)
            with torch.cuda.stream(fs):
                Zg.copy_(Z)
        for i0 in range(0, T, C):
            c = min(C, T - i0)
            mark("emit", lambda: ops.chain_emit(xr, zr, False, xpos, zpos, i0 == 0, r, G,
                                                kxs[i0:i0 + c], kzs[i0:i0 + c], kx, kz, Nl,
                                                send=send, cap=cap, flag=flag))
            ev = torch.cuda.Event()  # (the fork below waits for the emission only)
            ev.record()
            sz = G * c * (cap + 1)
            mark("exchange (device copy)", lambda: recv[:sz].copy_(send[:sz]))
            mark("unpack exact", lambda: ops.chain_unpack_exact(recv, G, c, cap, nl, nl, x_bag,
                                                                z_bag, flag))
            mark("count", lambda: ops.count_chain_rng(x_bag, xo, z_bag, zo, Nl, c, nl, nl, kx,
                                                      kz, B, 5 + i0, r * Nl,
                                                      counts[i0:i0 + c]))
            if i0 + c >= T:  # the final exchange beside the last chunk's count
                if parts:
                    mark("final exchange (side stream in the product)", lambda: final(xr, zr))
                else:
                    fs.wait_event(ev)
                    with torch.cuda.stream(fs):
                        final(xr, zr)
        if not parts:
            main.wait_stream(fs)
        mark("counts reduce (local part)",
             lambda: full[:-1].view(T, N)[:, r * Nl:(r + 1) * Nl].copy_(counts))
    ms = ev_time(call, 5)[0]
    if parts:
        return {k: sum(a.elapsed_time(b) for a, b in v) / 8 for k, v in t.items()}
    return ms


for T in Ts:
    one_gpu_call(T)  # warm (clock)
    ideal = one_gpu_call(T)
    print(f"T={T}: one GPU UnNB_many {ideal:.3f} ms/call ({ideal / T:.4f} ms/step)", flush=True)
    for G in (2, 4, 8):
        ranks = sorted({0, G - 1})
        ps = max(per_step_call(G, r, T) for r in ranks)
        cf = max(chain_call(G, r, T, False) for r in ranks)
        cc = max(chain_call(G, r, T, True) for r in ranks)
        pp = chain_call(G, G - 1, T, True, parts=True)
        print(f"  G={G}: ideal {ideal / G:.3f} ms; per-step exchange {ps:.3f} ms "
              f"(eff {ideal / G / ps:.3f}); chains first call {cf:.3f} ms (eff "
              f"{ideal / G / cf:.3f}), carried {cc:.3f} ms (eff {ideal / G / cc:.3f}); "
              "carried parts (ms/call, serialised) "
              + ", ".join(f"{k} {v:.4f}" for k, v in pp.items()), flush=True)
