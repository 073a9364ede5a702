"""Multi-rank repartition + reduction of tuplewise.device.ShardedSample on CPU (gloo).

The product runs one process per GPU over RCCL; here the same orchestration (global keyed
permutation, send counts from the forward and receive counts from the inverse permutation,
one all-to-all of {value, position} records for X and Z together, scatter, zero-padded
all-reduce of per-shard counts, host np.mean) runs at world size 2 and 4 with
gloo, with the device operations replaced by their oracle restatements (test-only).  Checks:
the permuted global arrays equal the single-process permutation, and the estimate is
bit-identical to the G = 1 result — the G-invariance the design promises.  Three exchange
protocols: step-by-step primitives, the counted fused exchange, and the fixed-capacity one
(equal-split all-to-all, the default).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O


class OracleOps:
    """CPU stand-ins for tuplewise.device.HipOps (test infrastructure)."""

    def perm_index(self, n, base, n_total, key):
        return torch.from_numpy(O.feistel_perm(np.arange(base, base + n), n_total, key))

    def permute(self, vals, key):
        return torch.from_numpy(O.permute_scatter(vals.numpy(), key))

    def permute_pair(self, X, kx, Z, kz):
        return self.permute(X, kx), self.permute(Z, kz)

    def rank_histogram(self, perm, n_loc, G):
        return torch.from_numpy(np.bincount(perm.numpy() // n_loc, minlength=G).astype(np.int64))

    def source_histogram(self, n, base, n_total, key, n_loc, G):
        src = O.feistel_perm_inv(np.arange(base, base + n), n_total, key)
        return torch.from_numpy(np.bincount(src // n_loc, minlength=G).astype(np.int64))

    def bucket_scatter(self, perm, vals, n_loc, G, start, send, pos_base):
        p = perm.numpy()
        dst = p // n_loc
        order = np.argsort(dst, kind="stable")
        k = np.arange(len(p)) - np.searchsorted(dst[order], dst[order])  # slot in its bucket
        rows = start.numpy()[dst[order]] + k
        rec = send.numpy()
        rec[rows, 0] = vals.numpy().view(np.int64)[order]
        rec[rows, 1] = (p - dst * n_loc)[order] + pos_base
        return send

    def scatter_records(self, rec, out):
        o = out.numpy().view(np.int64)
        r = rec.numpy()
        o[r[:, 1]] = r[:, 0]
        return out

    def count(self, x, x_off_dev, z, z_off_dev, n_shards, max_nx, max_nz, dtype, pred,
              algo="pairs"):
        xo, zo = x_off_dev.numpy(), z_off_dev.numpy()
        xs, zs = x.numpy(), z.numpy()
        f = O.un_count if pred == 0 else O.count_half_sorted
        return torch.tensor([f(xs[xo[s]:xo[s + 1]], zs[zo[s]:zo[s + 1]])
                             for s in range(n_shards)], dtype=torch.int64)

    def count_rng(self, x, x_off_dev, z, z_off_dev, n_shards, B, seed, shard_base, dtype, pred,
                  max_nx=None, max_nz=None):
        xo, zo = x_off_dev.numpy(), z_off_dev.numpy()
        out = []
        for s in range(n_shards):
            xs, zs = x.numpy()[xo[s]:xo[s + 1]], z.numpy()[zo[s]:zo[s + 1]]
            i, j = O.rng_pairs(len(xs), len(zs), B, seed, shard_base + s)
            out.append(int((xs[i] > zs[j]).sum()))
        return torch.tensor(out, dtype=torch.int64)

    def to_dev(self, arr):
        return torch.from_numpy(np.ascontiguousarray(arr))


class OracleOpsFused(OracleOps):
    """Adds the fused exchange (tw_exchange_counts / tw_exchange_pack) restated."""

    def exchange_counts(self, n_loc, m_loc, rank, G, key_x, key_z):
        out = []
        for n, key in ((n_loc, key_x), (m_loc, key_z)):
            g = np.arange(rank * n, (rank + 1) * n)
            out.append(np.bincount(O.feistel_perm(g, G * n, key) // n, minlength=G))
            out.append(np.bincount(O.feistel_perm_inv(g, G * n, key) // n, minlength=G))
        return torch.from_numpy(np.concatenate(out).astype(np.int64)), None

    def exchange_pack(self, X, Z, rank, G, key_x, key_z, counts, cursor):
        n_loc, m_loc = X.numel(), Z.numel()
        recs = []
        for side, (A, n, key, base) in enumerate(((X, n_loc, key_x, 0), (Z, m_loc, key_z, n_loc))):
            p = O.feistel_perm(np.arange(rank * n, (rank + 1) * n), G * n, key)
            dst = p // n
            recs.append((dst, np.full(n, side), A.numpy().view(np.int64), p - dst * n + base))
        dst, side, val, pos = (np.concatenate(c) for c in zip(*recs))
        order = np.lexsort((side, dst))  # bucket g = [X records | Z records]
        return torch.from_numpy(np.stack([val[order], pos[order]], axis=1))


class OracleOpsFixed(OracleOps):
    """Adds the fixed-capacity exchange (tw_exchange_pack_fixed / tw_scatter_buckets, the
    default of ShardedSample) restated: equal buckets of 1 + cap records, a count header each,
    an equal-split all-to-all, overflow flagged."""

    def exchange_pack_fixed(self, X, Z, rank, G, key_x, key_z, cap, cursor, send, flag):
        n_loc, m_loc = X.numel(), Z.numel()
        dst, val, pos = [], [], []
        for A, n, key, base in ((X, n_loc, key_x, 0), (Z, m_loc, key_z, n_loc)):
            p = O.feistel_perm(np.arange(rank * n, (rank + 1) * n), G * n, key)
            dst.append(p // n)
            val.append(A.numpy().view(np.int64))
            pos.append(p - (p // n) * n + base)
        dst, val, pos = np.concatenate(dst), np.concatenate(val), np.concatenate(pos)
        b = send.numpy().reshape(G, cap + 1, 2)
        for g in range(G):
            sel = np.flatnonzero(dst == g)
            b[g, 0] = (len(sel), 0)
            if len(sel) > cap:
                flag.numpy()[0] = 1
                sel = sel[:cap]
            b[g, 1:1 + len(sel), 0] = val[sel]
            b[g, 1:1 + len(sel), 1] = pos[sel]
        return send

    def scatter_buckets(self, recv, G, cap, out, flag):
        o = out.numpy().view(np.int64)
        b = recv.numpy().reshape(G, cap + 1, 2)
        for g in range(G):
            c = int(b[g, 0, 0])
            if c > cap:
                flag.numpy()[0] = 1
            r = b[g, 1:1 + min(c, cap)]
            o[r[:, 1]] = r[:, 0]
        return out


class OracleOpsRank(OracleOpsFixed):
    """Adds the rank-image step chain (tw_rank_images / tw_count_pairs_rank_step /
    tw_gather_records) restated, so UnN_many takes the replicated rank path on host tensors."""

    def rank_images(self, X, Z, dtype):
        xr, zr = O.rank_records(X.numpy(), Z.numpy())
        return torch.from_numpy(xr), torch.from_numpy(zr)

    def count_rank_step(self, xr, x_off_dev, zr, z_off_dev, n_shards, max_nx, max_nz, out,
                        x_next, key_x, z_next, key_z, out_next):
        img = lambda r: (r.numpy() & 0xFFFFFFFF).astype(np.uint32).view(np.float32)
        gx, nz = img(xr), img(zr)  # z images stored negated: x > z <=> gx + nz >= 1
        xo, zo = x_off_dev.numpy(), z_off_dev.numpy()
        for s in range(n_shards):
            a, b = gx[xo[s]:xo[s + 1]], nz[zo[s]:zo[s + 1]]
            out[s] += int((a[:, None] + b[None, :] >= 1).sum())
        if x_next is not None:
            x_next.copy_(torch.from_numpy(O.permute_scatter(xr.numpy(), key_x)))
            z_next.copy_(torch.from_numpy(O.permute_scatter(zr.numpy(), key_z)))
        if out_next is not None:
            out_next.zero_()
        return out

    def gather_records(self, vals, rec):
        return vals[rec >> 32]


class OracleOpsChain(OracleOpsRank):
    """Adds the step chains (tw_rank_images_query / tw_chain_emit / tw_chain_unpack /
    tw_count_pairs_chain / tw_chain_scatter / tw_chain_gather, csrc/chain.hip) restated, so
    UnN_many takes the chain path on host tensors (bags written at exact positions, one valid
    arrangement of the device's shard multisets)."""

    def rank_images_query(self, Z_all, X, Z, dtype, half=False):
        xr, zr = O.rank_records(X.numpy(), Z.numpy(), half=half, Z_all=Z_all.numpy())
        return torch.from_numpy(xr), torch.from_numpy(zr)

    def chain_emit(self, xr, zr, half, xpos, zpos, first, rank, world, keys_x, keys_z, kx, kz,
                   n_shards, x_bag=None, z_bag=None, cursors=None, send=None, cap=0, flag=None):
        n, m = xr.numel(), zr.numel()
        W = 2 if half else 1
        steps = len(keys_x)
        buckets = {}
        for side, (rec, pos, keys, nl) in enumerate(((xr, xpos, keys_x, n), (zr, zpos, keys_z, m))):
            r = rec.numpy().view(np.uint64)
            val = r if (half and side == 0) else r & np.uint64(0xFFFFFFFF)
            p = (np.arange(rank * nl, (rank + 1) * nl) if first
                 else pos.numpy().view(np.uint32).astype(np.int64))
            for c, key in enumerate(keys):
                p = O.feistel_perm(p, world * nl, int(key))
                if send is None:  # one process: the bags (a send buffer: the exchange)
                    bag = (x_bag if side == 0 else z_bag)[c].numpy()
                    bag.view(np.uint64 if (half and side == 0) else np.uint32)[p] = val
                else:
                    dst = p // nl
                    loc = p - dst * nl + (n if side else 0)
                    for g in range(world):
                        sel = dst == g
                        buckets.setdefault((g, c), []).append((val[sel], loc[sel]))
            pos.numpy()[:] = p.astype(np.uint32).view(np.int32)
        if send is not None:
            buf = send.numpy().view(np.uint64)
            for g in range(world):
                for c in range(steps):
                    v = np.concatenate([a for a, _ in buckets[(g, c)]])
                    q = np.concatenate([b for _, b in buckets[(g, c)]]).astype(np.uint64)
                    b0 = (g * steps + c) * (cap + 1) * W
                    buf[b0] = len(v)
                    if len(v) > cap:
                        flag.numpy()[0] = 1
                        v, q = v[:cap], q[:cap]
                    recs = buf[b0 + W:b0 + W * (1 + len(v))].reshape(-1, W)
                    if W == 1:
                        recs[:, 0] = v | (q << np.uint64(32))
                    else:
                        recs[:, 0], recs[:, 1] = v, q

    def chain_unpack(self, recv, world, steps, cap, half, n, m, x_bag, z_bag, flag, kx=0, kz=0,
                     n_shards=0):
        # (positions kept: the device appends each shard's records in runs, in any order)
        W = 2 if half else 1
        buf = recv.numpy().view(np.uint64)
        for b in range(world * steps):
            c = b % steps
            b0 = b * (cap + 1) * W
            cnt = int(buf[b0] & np.uint64(0xFFFFFFFF))
            if cnt > cap:
                flag.numpy()[0] = 1
            recs = buf[b0 + W:b0 + W * (1 + min(cnt, cap))].reshape(-1, W)
            v = recs[:, 0] if W == 2 else recs[:, 0] & np.uint64(0xFFFFFFFF)
            p = (recs[:, 1] if W == 2 else recs[:, 0] >> np.uint64(32)).astype(np.int64)
            isx = p < n
            x_bag[c].numpy().view(np.uint64 if half else np.uint32)[p[isx]] = v[isx]
            z_bag[c].numpy().view(np.uint32)[p[~isx] - n] = v[~isx]

    def chain_unpack_count(self, recv, world, steps, cap, half, n, m, x_bag, z_bag, flag, kx,
                           kz, n_shards, x_off_dev, z_off_dev, max_nx, max_nz, out):
        """tw_chain_unpack_count restated: the unpack, then the count of the filled bags."""
        self.chain_unpack(recv, world, steps, cap, half, n, m, x_bag, z_bag, flag, kx, kz,
                          n_shards)
        return self.count_chain(x_bag, x_off_dev, z_bag, z_off_dev, n_shards, steps, n, m,
                                max_nx, max_nz, half, out)

    def count_chain(self, x_bag, x_off_dev, z_bag, z_off_dev, n_shards, steps, x_stride,
                    z_stride, max_nx, max_nz, half, out):
        xo, zo = x_off_dev.numpy(), z_off_dev.numpy()
        for c in range(steps):
            xb = x_bag[c].numpy().view(np.float32)
            nz = z_bag[c].numpy().view(np.float32)
            for s in range(n_shards):
                b = nz[zo[s]:zo[s + 1]]
                if half:  # {g, h} pairs: [x > z] + [x >= z]
                    a = xb.reshape(-1, 2)[xo[s]:xo[s + 1]]
                    cnt = (a[:, 0, None] + b >= 1).sum() + (a[:, 1, None] + b >= 1).sum()
                else:
                    cnt = (xb[xo[s]:xo[s + 1], None] + b >= 1).sum()
                out[c, s] = int(cnt)
        return out

    def chain_scatter(self, X, xpos, Z, zpos):
        Xo, Zo = torch.empty_like(X), torch.empty_like(Z)
        Xo.numpy()[xpos.numpy().view(np.uint32)] = X.numpy()
        Zo.numpy()[zpos.numpy().view(np.uint32)] = Z.numpy()
        return Xo, Zo

    def chain_walk(self, x_base, n, NX, z_base, m, NZ, keys_x, keys_z, xpos, zpos):
        """tw_chain_walk restated: the rank's positions through every step, no emission."""
        for base, cnt, N_, keys, out in ((x_base, n, NX, keys_x, xpos),
                                         (z_base, m, NZ, keys_z, zpos)):
            p = np.arange(base, base + cnt)
            for key in keys:
                p = O.feistel_perm(p, N_, int(key))
            out.numpy()[:] = p.astype(np.uint32).view(np.int32)

    def chain_final_pack(self, X, xr, xpos, Z, zr, zpos, world, cap, cursor, send, flag):
        """tw_chain_final_pack restated: {score, record, local position} records of the walked
        elements into the buckets of the ranks holding their final positions (a header record
        with the count first; order inside a bucket is free)."""
        n, m = X.numel(), Z.numel()
        buf = send.numpy().view(np.uint64).reshape(world, cap + 1, 3)
        buf[:, 0, :] = 0
        recs = []
        for A, R, P, nl, off in ((X, xr, xpos, n, 0), (Z, zr, zpos, m, n)):
            p = P.numpy().view(np.uint32).astype(np.int64)
            recs.append((p // nl, A.numpy().view(np.uint64), R.numpy().view(np.uint64),
                         (p % nl + off).astype(np.uint64)))
        dst, val, rec, pos = (np.concatenate(c) for c in zip(*recs))
        for g in range(world):
            sel = np.flatnonzero(dst == g)
            buf[g, 0, 0] = len(sel)
            if len(sel) > cap:
                flag.numpy()[0] = 1
                sel = sel[:cap]
            buf[g, 1:1 + len(sel), 0] = val[sel]
            buf[g, 1:1 + len(sel), 1] = rec[sel]
            buf[g, 1:1 + len(sel), 2] = pos[sel]

    def chain_final_scatter(self, recv, world, cap, n, m, Xo, XRo, Zo, ZRo, flag):
        """tw_chain_final_scatter restated."""
        buf = recv.numpy().view(np.uint64).reshape(world, cap + 1, 3)
        for g in range(world):
            c = int(buf[g, 0, 0])
            if c > cap:
                flag.numpy()[0] = 1
            r = buf[g, 1:1 + min(c, cap)]
            p = r[:, 2].astype(np.int64)
            isx = p < n
            Xo.numpy().view(np.uint64)[p[isx]] = r[isx, 0]
            XRo.numpy().view(np.uint64)[p[isx]] = r[isx, 1]
            Zo.numpy().view(np.uint64)[p[~isx] - n] = r[~isx, 0]
            ZRo.numpy().view(np.uint64)[p[~isx] - n] = r[~isx, 1]

    def chain_unpack_exact(self, recv, world, steps, cap, n, m, x_bag, z_bag, flag):
        """tw_chain_unpack_exact restated: every record at its exact position of its bag."""
        buf = recv.numpy().view(np.uint64)
        for b in range(world * steps):
            c = b % steps
            b0 = b * (cap + 1)
            cnt = int(buf[b0] & np.uint64(0xFFFFFFFF))
            if cnt > cap:
                flag.numpy()[0] = 1
            recs = buf[b0 + 1:b0 + 1 + min(cnt, cap)]
            v = (recs & np.uint64(0xFFFFFFFF)).astype(np.uint32)
            p = (recs >> np.uint64(32)).astype(np.int64)
            isx = p < n
            x_bag[c].numpy().view(np.uint32)[p[isx]] = v[isx]
            z_bag[c].numpy().view(np.uint32)[p[~isx] - n] = v[~isx]

    def count_chain_rng(self, x_bag, x_off_dev, z_bag, z_off_dev, n_shards, steps, x_stride,
                        z_stride, max_nx, max_nz, B, seed, shard_base, out):
        """tw_count_pairs_chain_rng restated: the oracle's device draws (count_rng's) of each
        (step, shard) bag, compared on the images (x > z <=> g(x) - g(z) >= 1)."""
        xo, zo = x_off_dev.numpy(), z_off_dev.numpy()
        for c in range(steps):
            xb = x_bag[c].numpy().view(np.float32)
            zb = z_bag[c].numpy().view(np.float32)
            for s in range(n_shards):
                a, b = xb[xo[s]:xo[s + 1]], zb[zo[s]:zo[s + 1]]
                i, j = O.rng_pairs(len(a), len(b), B, (seed + c) % 2 ** 64, shard_base + s)
                out[c, s] = int((a[i] + b[j] >= 1).sum())
        return out

    def words_checksum(self, A, B, acc, expect=None, verdict=None, good=1, bad=0):
        """tw_words_checksum (csrc/guard.hip) restated: sum of splitmix64-finalised words
        xored with position * golden, wrapping."""
        w = np.concatenate([A.numpy().reshape(-1).view(np.uint64),
                            B.numpy().reshape(-1).view(np.uint64)])
        with np.errstate(over="ignore"):
            z = w ^ (np.arange(w.size, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
            acc.numpy().view(np.uint64)[0] = z.sum(dtype=np.uint64)
        if verdict is not None:
            verdict[0] = good if int(acc[0]) == int(expect[0]) else bad
        return acc

    def chain_gather(self, X_all, Z_all, x_base, n, z_base, m, keys_x, keys_z, X2=None,
                     Z2=None):
        out, src = [], []
        for A, base, cnt, keys in ((X_all, x_base, n, keys_x), (Z_all, z_base, m, keys_z)):
            p = np.arange(base, base + cnt)
            for key in reversed(keys):
                p = O.feistel_perm_inv(p, A.numel(), int(key))
            out.append(torch.from_numpy(A.numpy()[p].copy()))
            src.append(p)
        if X2 is not None:  # tw_chain_gather2: the second pair from the same walk
            out += [torch.from_numpy(X2.numpy()[src[0]].copy()),
                    torch.from_numpy(Z2.numpy()[src[1]].copy())]
        return tuple(out)


_OPS = {"plain": OracleOps, "fused": OracleOpsFused, "fixed": OracleOpsFixed,
        "rank": OracleOpsRank, "chain": OracleOpsChain}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _global_data(G, n_loc, m_loc):
    rng = np.random.RandomState(42)
    return rng.normal(0.4, 1, G * n_loc), rng.normal(0, 1, G * m_loc)


def _worker(rank, G, port, n_loc, m_loc, N, keys, B, q, fused):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=G)
    from tuplewise.device import ShardedSample
    X, Z = _global_data(G, n_loc, m_loc)
    S = ShardedSample(torch.from_numpy(X[rank * n_loc:(rank + 1) * n_loc].copy()),
                      torch.from_numpy(Z[rank * m_loc:(rank + 1) * m_loc].copy()), N,
                      group=dist.group.WORLD, ops=_OPS[fused]())
    vals = [float(S.UnN(k)) for k in keys]
    inc = float(S.UnNB(B, seed=77))
    Xg = [torch.empty_like(S.X) for _ in range(G)]
    Zg = [torch.empty_like(S.Z) for _ in range(G)]
    dist.all_gather(Xg, S.X)
    dist.all_gather(Zg, S.Z)
    if rank == 0:
        q.put((vals, inc, torch.cat(Xg).numpy(), torch.cat(Zg).numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("G,fused", [(G, f) for G in (2, 4) for f in ("plain", "fused", "fixed")]
                         + [(8, "fixed")])  # 8 = the driver's scaling run, default protocol
def test_multirank_repartition_is_G_invariant(G, fused):
    import tuplewise  # noqa: F401  (package import only; no device work in this test)
    from tuplewise.device import ShardedSample
    n_loc, m_loc, N, keys, B = 600, 450, 3, [5, 6], 200
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, G, port, n_loc, m_loc, N, keys, B, q, fused))
             for r in range(G)]
    for p in procs:
        p.start()
    vals, inc, Xg, Zg = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    # single-process reference of the same global problem (G*N shards of the same layout)
    X, Z = _global_data(G, n_loc, m_loc)
    S1 = ShardedSample(torch.from_numpy(X.copy()), torch.from_numpy(Z.copy()), G * N,
                       ops=OracleOps())
    # the global permutation after both repartitions equals the G=1 permutation
    Xp, Zp = X.copy(), Z.copy()
    for k in keys:
        Xp = O.permute_scatter(Xp, 2 * k)
        Zp = O.permute_scatter(Zp, 2 * k + 1)
    assert np.array_equal(Xg, Xp) and np.array_equal(Zg, Zp)
    # per-rank shards are the rank-local prop-SWOR blocks; with n_loc divisible by N they
    # coincide with the global layout, so the estimates are bit-identical to G = 1
    want = [float(S1.UnN(k)) for k in keys]
    assert vals == want
    assert inc == float(S1.UnNB(B, seed=77))


def _rank_worker(rank, G, port, n_loc, m_loc, N, keys, q, tie_mode="strict", sub=0,
                 final="exchange"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=G)
    from tuplewise import device as D
    from tuplewise.device import ShardedSample
    D.CHAIN_SUB = sub
    # the final arrays: one exchange after the last emission (default), one exchange forked at
    # the call's start on walked positions (tw_chain_walk), or the inverse-chain gathers
    D.FINAL_EXCHANGE = final != "gather"
    D.FINAL_EARLY = final == "early"
    X, Z = _global_data(G, n_loc, m_loc)
    S = ShardedSample(torch.from_numpy(X[rank * n_loc:(rank + 1) * n_loc].copy()),
                      torch.from_numpy(Z[rank * m_loc:(rank + 1) * m_loc].copy()), N,
                      group=dist.group.WORLD, ops=OracleOpsChain(), tie_mode=tie_mode,
                      algo="pairs")
    assert S.algo == "pairs" and S._chain_ok()
    vals = [float(v) for v in S.UnN_many(keys)]
    Xg = [torch.empty_like(S.X) for _ in range(G)]
    Zg = [torch.empty_like(S.Z) for _ in range(G)]
    dist.all_gather(Xg, S.X)
    dist.all_gather(Zg, S.Z)
    if rank == 0:
        q.put((vals, torch.cat(Xg).numpy(), torch.cat(Zg).numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("G,tie_mode,sub,final", [
    (2, "strict", 0, "exchange"), (4, "strict", 0, "exchange"), (8, "strict", 0, "exchange"),
    (2, "half", 0, "exchange"), (4, "strict", 5, "exchange"), (3, "half", 0, "early"),
    (2, "strict", 5, "early"), (3, "strict", 0, "gather")])
def test_chain_steps_are_G_invariant(G, tie_mode, sub, final):
    """UnN_many's step chains over G ranks (csrc/chain.hip, restated): every rank images its
    own elements against the all-gathered Z, walks their chains into per-(rank, step) buckets,
    one all-to-all per chunk (sub > 0: per sub-chunk of <= sub steps, async), counts its bags;
    one all-reduce of the counts per call.  The estimates equal the one-process score path's (est.UnNT's loop, key by key) and the ranks'
    final arrays, concatenated, equal the global permutation chain."""
    import tuplewise  # noqa: F401
    from tuplewise import device as D
    assert D.CHAIN_STEPS
    from tuplewise.device import ShardedSample
    # 12 steps: with sub = 5, sub-chunks of (5, 5, 2) steps, each its own async all-to-all,
    # unpacked and counted in order
    n_loc, m_loc, N = 600, 450, 3
    keys = [5, 6, 9, 11, 2, 7, 8, 13, 21, 3, 4, 17] if G != 8 else [5, 6, 9, 11, 2, 7, 8]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker,
                         args=(r, G, port, n_loc, m_loc, N, keys, q, tie_mode, sub, final))
             for r in range(G)]
    for p in procs:
        p.start()
    vals, Xg, Zg = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    X, Z = _global_data(G, n_loc, m_loc)
    S1 = ShardedSample(torch.from_numpy(X.copy()), torch.from_numpy(Z.copy()), G * N,
                       ops=OracleOps(), tie_mode=tie_mode, algo="pairs")
    assert vals == [float(S1.UnN(k)) for k in keys]  # the score path, key by key
    assert np.array_equal(Xg, S1.X.numpy()) and np.array_equal(Zg, S1.Z.numpy())
    S1c = ShardedSample(torch.from_numpy(X.copy()), torch.from_numpy(Z.copy()), G * N,
                        ops=OracleOpsChain(), tie_mode=tie_mode, algo="pairs")
    assert [float(v) for v in S1c.UnN_many(keys)] == vals  # the one-process chain
    assert np.array_equal(S1c.X.numpy(), Xg)


def _rng_chain_worker(rank, G, port, n_loc, m_loc, N, B, seed, calls, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=G)
    from tuplewise.device import ShardedSample
    X, Z = _global_data(G, n_loc, m_loc)
    S = ShardedSample(torch.from_numpy(X[rank * n_loc:(rank + 1) * n_loc].copy()),
                      torch.from_numpy(Z[rank * m_loc:(rank + 1) * m_loc].copy()), N,
                      group=dist.group.WORLD, ops=OracleOpsChain(), algo="pairs")
    assert S._chain_rng_ok()
    vals, carried = [], []
    for i, keys in enumerate(calls):  # later calls carry the images (device.CARRY_IMAGES)
        carried.append(S._carried(False) is not None)
        vals.append([float(v) for v in S.UnNB_many(B, seed + 100 * i, keys)])
    Xg = [torch.empty_like(S.X) for _ in range(G)]
    Zg = [torch.empty_like(S.Z) for _ in range(G)]
    dist.all_gather(Xg, S.X)
    dist.all_gather(Zg, S.Z)
    if rank == 0:
        q.put((vals, carried, torch.cat(Xg).numpy(), torch.cat(Zg).numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("G", [2, 3, 8])
def test_incomplete_chain_steps_are_G_invariant(G):
    """UnNB_many over ranks on the step chains (cs.UnNBT's loop,
    compute_stats.py:119-123): one exchange per chunk, records unpacked at their EXACT
    positions (tw_chain_unpack_exact, restated), B device-drawn pairs per (step, shard) bag
    counted on the rank images (tw_count_pairs_chain_rng, restated).  Estimates equal the
    one-process score path's UnNB(B, seed + t, key_t), key by key, including a second call that
    carries the images; the ranks' final arrays equal the global permutation chain."""
    import tuplewise  # noqa: F401
    from tuplewise.device import ShardedSample
    n_loc, m_loc, N, B, seed = 600, 450, 3, 700, 0xC3C3_0042
    calls = [[5, 6, 9, 11], [2, 7]] if G != 8 else [[5, 6, 9], [2]]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rng_chain_worker,
                         args=(r, G, port, n_loc, m_loc, N, B, seed, calls, q))
             for r in range(G)]
    for p in procs:
        p.start()
    vals, carried, Xg, Zg = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert carried == [False, True]
    X, Z = _global_data(G, n_loc, m_loc)
    S1 = ShardedSample(torch.from_numpy(X.copy()), torch.from_numpy(Z.copy()), G * N,
                       ops=OracleOps(), algo="pairs")
    want = [[float(S1.UnNB(B, seed + 100 * i + t, k)) for t, k in enumerate(keys)]
            for i, keys in enumerate(calls)]
    assert vals == want
    assert np.array_equal(Xg, S1.X.numpy()) and np.array_equal(Zg, S1.Z.numpy())


def _overflow_worker(rank, G, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=G)
    from tuplewise.device import ShardedSample
    X, Z = _global_data(G, 600, 450)
    S = ShardedSample(torch.from_numpy(X[rank * 600:(rank + 1) * 600].copy()),
                      torch.from_numpy(Z[rank * 450:(rank + 1) * 450].copy()), 3,
                      group=dist.group.WORLD, ops=OracleOpsFixed())
    cap = 10  # far below the ~525 records of a bucket: every bucket overflows
    S._xf = {"cap": cap, "cursor": torch.zeros((G,), dtype=torch.int64),
             "flag": torch.zeros((1,), dtype=torch.int32),
             "send": torch.empty((G * (cap + 1), 2), dtype=torch.int64),
             "recv": torch.empty((G * (cap + 1), 2), dtype=torch.int64)}
    raised = []
    for _ in range(2):  # the flag is sticky: a later repartition raises too
        try:
            S.repartition(5)
            raised.append(False)
        except RuntimeError:
            raised.append(True)
    S.repartition(6, check=False)  # the pipelined estimators' form: no check here...
    try:
        S.values(S.global_counts(S.local_counts()))  # ...but values() refuses the arrays
        raised.append(False)
    except RuntimeError:
        raised.append(True)
    q.put((rank, raised))
    dist.barrier()
    dist.destroy_process_group()


def test_exchange_overflow_raises_at_repartition():
    """a fixed-capacity exchange that overflows must not leave X/Z silently
    corrupt — repartition() raises on every rank (and keeps raising: the flag is sticky)."""
    import tuplewise  # noqa: F401
    G = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overflow_worker, args=(r, G, port, q)) for r in range(G)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(G))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(got[r] == [True, True, True] for r in range(G)), got


def _flag_worker(rank, G, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=G)
    from tuplewise.device import ShardedSample
    X, Z = _global_data(G, 600, 450)
    S = ShardedSample(torch.from_numpy(X[rank * 600:(rank + 1) * 600].copy()),
                      torch.from_numpy(Z[rank * 450:(rank + 1) * 450].copy()), 3,
                      group=dist.group.WORLD, ops=OracleOpsChain(), algo="pairs")
    if rank == 0:  # an overflow seen by rank 0 only (a sending rank and its receiver)
        S._chain_flag = torch.ones((1,), dtype=torch.int32)
    try:
        S.UnN_many([5, 6])
        raised = False
    except RuntimeError:
        raised = True
    q.put((rank, raised))
    dist.barrier()
    dist.destroy_process_group()


def test_chain_overflow_raises_on_every_rank():
    """a step-chain bucket overflow flags only the sending and the receiving rank;
    the flag rides in the counts' all-reduce, so EVERY rank raises in values() — none returns
    estimates built from the corrupted counts, and the ranks agree."""
    import tuplewise  # noqa: F401
    G = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_flag_worker, args=(r, G, port, q)) for r in range(G)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(G))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(got[r] for r in range(G)), got


def _forced_worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    from tuplewise.device import ShardedSample
    X, Z = _global_data(1, 1800, 1350)
    out = {}
    for tie in ("strict", "half"):
        S = ShardedSample(torch.from_numpy(X.copy()), torch.from_numpy(Z.copy()), 9,
                          group=dist.group.WORLD, ops=OracleOpsChain(), tie_mode=tie,
                          algo="pairs", collectives=True)
        assert S.coll and S._multi()
        vals = [float(v) for v in S.UnN_many([5, 6, 9, 11, 2, 7, 8])]
        vals.append(float(S.UnN(3)))  # the fixed exchange + one all-reduce
        out[tie] = (vals, S.X.numpy().copy(), S.Z.numpy().copy())
    q.put(out)
    dist.destroy_process_group()


def test_forced_collectives_at_world_size_one_equal_one_process():
    """VERDICT r04 item 1 on CPU: ShardedSample(collectives=True) on a world-size-1 group runs
    the multi-rank branches (all-gathers, chain emission into send buckets, the all-to-all,
    unpack, chain_gather, the counts' all-reduce, the fixed exchange) and must equal the
    one-process path bit for bit; tests/test_gpu_rccl.py runs the same on RCCL."""
    import tuplewise  # noqa: F401
    from tuplewise.device import ShardedSample
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_forced_worker, args=(_free_port(), q))
    p.start()
    got = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    X, Z = _global_data(1, 1800, 1350)
    for tie in ("strict", "half"):
        S = ShardedSample(torch.from_numpy(X.copy()), torch.from_numpy(Z.copy()), 9,
                          ops=OracleOpsChain(), tie_mode=tie, algo="pairs")
        want = [float(v) for v in S.UnN_many([5, 6, 9, 11, 2, 7, 8])]
        want.append(float(S.UnN(3)))
        vals, Xf, Zf = got[tie]
        assert vals == want
        assert np.array_equal(Xf, S.X.numpy()) and np.array_equal(Zf, S.Z.numpy())


def _carry_worker(rank, G, port, q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=G)
    from tuplewise.device import ShardedSample
    n_loc, m_loc, N = 600, 450, 3  # shards that tile the global layout rank by rank
    X, Z = _global_data(G, n_loc, m_loc)
    S = ShardedSample(torch.from_numpy(X[rank * n_loc:(rank + 1) * n_loc].copy()),
                      torch.from_numpy(Z[rank * m_loc:(rank + 1) * m_loc].copy()), N,
                      group=dist.group.WORLD, ops=OracleOpsChain(), algo="pairs")
    out = {"vals": [], "carried": []}
    try:
        for keys in ([3, 4, 5], [6, 7], [8, 9, 10, 11]):
            if mode == "inplace" and keys[0] == 8:
                S.Z.mul_(1)  # an in-place change on every rank: the images are recomputed
            if mode == "one_rank" and keys[0] == 8 and rank == 0:
                S.Z.mul_(1)  # on rank 0 alone: the ranks disagree, every rank recounts
            if mode.startswith("hidden") and keys[0] == 8 and (rank == 0 or mode == "hidden"):
                # two scores exchanged behind the version counter (.data has its own): the
                # images still look carried, the checksum verdict makes every rank recount
                S.X.data[[0, 1]] = S.X.data[[1, 0]].clone()
            out["carried"].append(S._carried(False) is not None)
            out["vals"] += [float(v) for v in S.UnN_many(keys)]
        out["recounts"] = getattr(S, "stale_recounts", 0)
        Xg = [torch.empty_like(S.X) for _ in range(G)]
        Zg = [torch.empty_like(S.Z) for _ in range(G)]
        dist.all_gather(Xg, S.X)
        dist.all_gather(Zg, S.Z)
        out["X"], out["Z"] = torch.cat(Xg).numpy(), torch.cat(Zg).numpy()
    except RuntimeError as e:
        out["raised"] = str(e)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("G,mode", [(2, "carry"), (3, "carry"), (2, "inplace"), (3, "one_rank"),
                                    (2, "hidden"), (3, "hidden_one")])
def test_carried_images_over_ranks(G, mode):
    """device.CARRY_IMAGES over ranks: the second and later UnN_many calls carry every rank's
    records through the inverse chains (all-gathered records, chain_gather) instead of ranking
    again; estimates and final arrays equal the one-process score path call after call.  An
    in-place change of the sample on every rank drops the carried images; on one rank alone the
    ranks disagree and every rank recounts the call from a fresh ranking.  A write behind the
    version counter (.data) on every rank or on one is caught by the arrays' checksum
    (tw_words_checksum): every rank recounts, estimates stay exact."""
    import tuplewise  # noqa: F401
    from tuplewise.device import ShardedSample
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_carry_worker, args=(r, G, port, q, mode)) for r in range(G)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(G))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all("raised" not in got[r] for r in range(G)), got
    out = got[0]
    hidden = mode.startswith("hidden")
    assert out["carried"] == [False, True, mode == "carry" or hidden]  # (rank 0's view)
    assert all(got[r]["recounts"] == (1 if mode == "one_rank" or hidden else 0)
               for r in range(G)), got
    X, Z = _global_data(G, 600, 450)
    S1 = ShardedSample(torch.from_numpy(X.copy()), torch.from_numpy(Z.copy()), G * 3,
                       ops=OracleOps(), algo="pairs")
    want = []
    for k in [3, 4, 5, 6, 7, 8, 9, 10, 11]:
        if k == 8 and hidden:  # the same exchange in the one-process reference
            Xh = S1.X.clone()
            for r in (range(G) if mode == "hidden" else [0]):
                Xh[[r * 600, r * 600 + 1]] = Xh[[r * 600 + 1, r * 600]].clone()
            S1.X = Xh
        want.append(float(S1.UnN(k)))
    assert out["vals"] == want
    assert np.array_equal(out["X"], S1.X.numpy()) and np.array_equal(out["Z"], S1.Z.numpy())


def test_one_process_carried_images_checksum_verdict():
    """The one-process branch of the carried images' guard (device.py _chain_call): the hash
    verdict lands in a host word read after the counts; a write through `.data` between calls
    (no version bump) makes the call recount from a fresh ranking — estimates and arrays equal
    a fresh sample's on the written arrays; an untouched sample keeps carrying, no recount."""
    import tuplewise  # noqa: F401
    from tuplewise.device import ShardedSample
    X, Z = _global_data(1, 1800, 1350)
    for write in (False, True):
        S = ShardedSample(torch.from_numpy(X.copy()), torch.from_numpy(Z.copy()), 9,
                          ops=OracleOpsChain(), algo="pairs")
        S.UnN_many([5, 6, 9])
        assert S._carried(False) is not None
        if write:
            S.X.data[[0, 7]] = S.X.data[[7, 0]].clone()
            S.Z.data[:40] += 0.25
        Xw, Zw = S.X.clone(), S.Z.clone()
        got = [float(v) for v in S.UnN_many([2, 7, 8])]
        assert getattr(S, "stale_recounts", 0) == (1 if write else 0)
        F = ShardedSample(Xw, Zw, 9, ops=OracleOps(), algo="pairs")
        assert got == [float(F.UnN(k)) for k in (2, 7, 8)]
        assert np.array_equal(S.X.numpy(), F.X.numpy()) and np.array_equal(S.Z.numpy(),
                                                                            F.Z.numpy())
