"""Drop-in replacement for the learning loop of learning-experiment/make_exps.py.

learning_process(X, Z, p_learn, optim_type="momentum")  make_exps.py:96-141
evaluation_step(i, X_s, Z_s, w, p_learn)                 make_exps.py:143-190

Same logging lines, same p_learn side effects (iter, norm_w, bc_AUC, br_AUC, tr_AUC, tc_AUC
lists), same NumPy global-RNG draws in the same order (the initial redundant SWR_divide, the
per-reshuffle SWR_divide draws, and per shard the two randint calls of grad_inc_block).  The
state lives on the GPU: X, Z, the shard row indices, w and the momentum buffer; each step is
one tw_hinge_grad launch (all shards) + one tw_sgd_update launch.  w is copied to the host
only when evaluation_step needs it.  Evaluation runs on the device too: score GEMVs, the
fixed-pair hinge and AUC, the complete test hinge and AUC.

Keyword-only extra: ``trajectory`` (a list) receives a copy of w before every gradient step,
the value the reference passes to grad_inc_block at make_exps.py:130.
"""
from __future__ import annotations

import ctypes
import logging

import numpy as np

from . import _engine as E
from . import _lib as L
from . import _learn
from . import compute_stats as cs
from .numpy_rng import Session

SEED_SHUFFLE = 42
# narrow rows (C4): a segment of fused steps in ONE persistent launch (tw_sgd_segment_narrow:
# one grid barrier per step, the update recomputed in every block); off: one launch per step
NARROW_SEGMENT = True
# replay loop: the host's NumPy-exact draws made two segments ahead by a worker thread
# (_replay_pipelined); False keeps the sequential loop (A/B, tests)
DRAW_AHEAD = True
# evaluations of the learning loop: device part enqueued, host part once the results are back
# (no device wait per evaluation); off: evaluation_step waits for its results
DEFER_EVALS = True
# pipelined replay loop: draws shipped as uint8 when every index is < 256 (C4: kx = 91, kz = 7),
# else uint16; the device widens them (the H2D bytes are read over PCIe by the widen kernel)
NARROW_DRAWS_U8 = True
# learning_process keeps its engine (device buffers, captured segment graphs, replay draw
# buffers) for the next call of the same shapes and hyper-parameters on host arrays — the
# reference's make_exps calls learning_process once per configuration and repetition — so that
# call loads its X, Z and w into the same buffers and replays the graphs already captured
# instead of capturing new ones.  Problems up to ENGINE_CACHE_MAX_BYTES of rows only.
ENGINE_CACHE = True
ENGINE_CACHE_MAX_BYTES = 256 << 20
_ENGINE = {"key": None, "eng": None}
# pipelined replay loop: each segment's narrowed draws and a reshuffle's row tables go up in ONE
# launch (tw_ship_draws) instead of a widen and two row copies
FUSED_SHIP = True
# device-RNG loop: persistent narrow segments run through their reshuffles, the kernel drawing
# each reshuffle's SWR rows (tw_sgd_segment_narrow_swr) instead of a row-table launch and a new
# segment per reshuffle
SWR_IN_KERNEL = True
# evaluation_step (FIXED_PAIRS) on small problems: scores, monitor and test statistics in two
# launches (tw_eval_small) instead of a dozen, same values
EVAL_FUSED = True
# pipelined replay loop: the draws made ahead by a native thread (csrc/drawpipe.hip) rather
# than a Python worker thread
NATIVE_DRAWS = True
# replay segments run through reshuffles (one process, replicated X, narrow segments): the
# reshuffles' SWR tables ride in the segment's upload, the kernel switches tables by step
REPLAY_THROUGH = True
PIPE_STATS = None  # a list: the pipelined replay loop appends its wait for each segment's draws
# learning over ranks: the shard gradients exchanged by the GPUs through IPC-mapped peer buffers
# (csrc/peer.hip: the persistent narrow segment, or per step one publish-wait-update launch)
# instead of a host-enqueued RCCL all-gather per step; False keeps the all-gather (A/B)
PEER_EXCHANGE = True
# the per-step peer exchange by column owners (tw_peer_step_cols: each partial column goes to
# its owner only, the owner updates its columns and publishes them) rather than every rank
# receiving every partial and updating all d columns (tw_peer_step); same bits.  None = from 8
# ranks on: it moves (G-1)/G of the bytes less but adds a second cross-rank hand-off per step,
# and co-resident rehearsals (ranks sharing one GPU's HBM, where bytes are cheap) measured it
# slower at 2 and 4 ranks (C5 B = 100: 61.0 vs 57.2 us, 170 vs 161 us; profiles/r06_learn*)
PEER_COLUMNS = None
PEER_COLUMNS_MIN_RANKS = 8
TYPE_TRAIN_MONITOR = "FIXED_PAIRS"  # or "SAME_AS_BATCH" (make_exps.py:31-33)
SEED_TRAIN_MONITOR = 54
SIZE_TRAIN_MONITOR = 450000
PROP_TEST = 0.2
DEFAULT_ITE_NUMBER = 5000


class SGDEngine:
    """Device-resident pairwise-hinge SGD state for one learning_process run.

    Multi-GPU (group = a torch.distributed process group, one process per GPU): X and Z are
    replicated (n x d fp64 fits every MI355X's 288 GB up to n*d ~ 3e10), rank r owns shards
    [r*N/G, (r+1)*N/G); each step computes its shards' gradients, all-gathers the (N/G, d)
    partials in shard order (one RCCL all-gather) and applies the same shard-ordered update
    on every rank — so w, and the whole trajectory, is identical for any G.

    x_layout="partitioned" is the other side of the memory/communication trade-off (SURVEY.md
    §8(e)): rank r keeps only rows [r*n/G, (r+1)*n/G) of X and of Z, and every reshuffle moves
    the drawn rows to the ranks whose shards drew them (tw_row_pack -> one all_to_all ->
    tw_row_unpack into a shard-local matrix).  The gradient kernels then read the local matrix
    through an identity row table, so the arithmetic — and the trajectory — is unchanged."""

    def __init__(self, X, Z, w_init, N, B, margin, reg, learning_rate, optim_type, group=None,
                 x_layout="replicated", loss="hinge", gradient="incomplete", vgroup=None,
                 collectives=None):
        """X, Z, w_init: NumPy arrays (copied to the device) or device tensors (used as is).
        vgroup=(G, r): slot r of G on ONE process (MultiDeviceSGD): shards as rank r, but the
        shard gradients are gathered and the update applied by the driver (_apply_update).
        collectives: None = the over-ranks step (eager launches, one all-gather per step, the
        partitioned exchange) exactly when the group has several ranks; True forces it on a
        world-size-1 group (every RCCL call of the path runs on one GPU, same trajectory)."""
        t = L.torch()
        self.t = t
        self.group = group
        self.vgroup = vgroup
        if vgroup is not None:
            if group is not None:
                raise ValueError("vgroup and group are exclusive")
            self.dist = None
            self.G, self.rank = int(vgroup[0]), int(vgroup[1])
        elif group is not None:
            import torch.distributed as dist
            self.dist = dist
            self.G, self.rank = dist.get_world_size(group), dist.get_rank(group)
        else:
            self.dist, self.G, self.rank = None, 1, 0
        self.coll = (self.dist is not None
                     and (L.collectives_default(group, self.G) if collectives is None
                          else bool(collectives)))
        if collectives and self.dist is None:
            raise ValueError("collectives=True needs a process group")
        # one process, one device, no collective: the fused / persistent / graph paths apply
        self.solo = self.G == 1 and not self.coll
        if vgroup is not None and int(N) % self.G:
            raise ValueError(f"N={N} shards do not split evenly over {self.G} slots")
        if int(N) < self.G:
            raise ValueError(f"N={N} shards cannot give each of {self.G} ranks one")
        # rank r owns shards [r N / G, (r + 1) N / G): balanced and uneven where G does not
        # divide N (the reference's N = 100 shuttle shards over 8 GPUs: 12 or 13 per rank);
        # N_pad = the most any rank owns (padded per-rank layouts of the exchanges)
        G_ = self.G
        self.shard_bounds = [g * int(N) // G_ for g in range(G_ + 1)]
        self.shard_base = self.shard_bounds[self.rank]
        self.N_loc = self.shard_bounds[self.rank + 1] - self.shard_base
        self.N_pad = -(-int(N) // G_)
        self.even = int(N) % G_ == 0
        if x_layout not in ("replicated", "partitioned"):
            raise ValueError(f"x_layout must be 'replicated' or 'partitioned', not {x_layout!r}")
        self.layout = x_layout
        self.n_X, self.d = int(X.shape[0]), int(X.shape[1])
        self.n_Z = int(Z.shape[0])
        self.N, self.B = int(N), int(B)
        self.kx, self.kz = int(self.n_X / N), int(self.n_Z / N)
        if x_layout == "replicated":
            self.X = _dev_f64(X)
            self.Z = _dev_f64(Z)
        else:
            G, r = self.G, self.rank
            self.x_own = (r * self.n_X // G, (r + 1) * self.n_X // G)
            self.z_own = (r * self.n_Z // G, (r + 1) * self.n_Z // G)
            # each side's matrix is [this rank's partition | receive area]: owned draws are read
            # in the partition, remote ones where the exchange lands them (csrc/exchange.hip);
            # the row tables (partition_tables) point into it
            self.X = self._side_matrix(X[self.x_own[0]:self.x_own[1]], self.kx)
            self.Z = self._side_matrix(Z[self.z_own[0]:self.z_own[1]], self.kz)
            self.X_part = self.X[:self.x_own[1] - self.x_own[0]]
            self.Z_part = self.Z[:self.z_own[1] - self.z_own[0]]
            dev = self.X.device
            self.tab_x = t.zeros((self.N_loc, self.kx), dtype=t.int64, device=dev)
            self.tab_z = t.zeros((self.N_loc, self.kz), dtype=t.int64, device=dev)
        self.margin, self.reg, self.lr = float(margin), float(reg), float(learning_rate)
        self.loss = cs._loss_codes(loss)[1]
        if gradient not in ("incomplete", "complete"):
            raise ValueError(f"gradient must be 'incomplete' or 'complete', not {gradient!r}")
        self.complete = gradient == "complete"
        self._cwork = None
        self.momentum = 0.9 if optim_type == "momentum" else -1.0
        self.w_shape = tuple(w_init.shape)
        self.w = _dev_f64(w_init).reshape(-1).clone()
        self.dw = t.zeros_like(self.w)
        self.grads = L.empty((self.N, self.d), t.float64)  # all shards, global order
        # over ranks: this rank's partials (N_pad rows: the padded all-gather of uneven splits)
        self.grads_loc = self.grads if self.solo else L.empty((self.N_pad, self.d), t.float64)
        self.rows_x = self.rows_z = None
        self.step_ctr = None
        # one launch per step (tw_sgd_step: the previous step's update fused into the gradient
        # launch) for narrow rows on one GPU; fused=False keeps grad + update launches
        self.fused = (self.solo and not self.complete
                      and bool(L.lib().tw_sgd_step_fusable(self.d, self.N_loc)))
        self._slot1 = None
        self.narrow_seg = (NARROW_SEGMENT and self.fused
                           and bool(L.lib().tw_sgd_segment_narrow_ok(self.d, self.N_loc, self.B)))
        # over ranks: the device-resident gradient exchange (csrc/peer.hip), when every rank
        # could map every other rank's peer buffer (else the per-step RCCL all-gather)
        self.peer = _PeerBuffers.create(self) if self.coll and PEER_EXCHANGE else None
        self.peer_seg = (self.peer is not None and not self.complete
                         and bool(L.lib().tw_sgd_segment_narrow_ok(self.d, self.N, self.B)))
        self._ctl = (t.zeros((2,), dtype=t.int32, device=self.w.device)
                     if self.narrow_seg or self.peer is not None else None)

    def reload(self, X, Z, w_init):
        """A new run on this engine (learning_process's engine cache): X, Z (host arrays of
        this engine's shapes) and w_init into the existing buffers, momentum and the abort word
        zeroed; captured graphs stay valid (same addresses, same scalars)."""
        t = self.t
        for dst, src in ((self.X, X), (self.Z, Z)):
            dst.copy_(t.from_numpy(np.ascontiguousarray(src, dtype=np.float64)).reshape(
                dst.shape))
        self.w_shape = tuple(w_init.shape)
        self.w.copy_(t.from_numpy(np.ascontiguousarray(w_init, dtype=np.float64)).reshape(-1))
        self.dw.zero_()
        if self._ctl is not None:
            self._ctl.zero_()

    def check(self):
        """Raise if a persistent segment launch gave up waiting at a grid barrier, or a peer
        wait of the exchange over ranks expired (its bounded spin: blocks not co-resident, or
        a rank that stopped stepping); the state is then invalid."""
        if self._ctl is not None and int(self._ctl[1].item()) != 0:
            raise RuntimeError("SGD segment: a grid barrier or peer wait timed out (blocks not "
                               "co-resident, or a rank stopped); the SGD state is invalid")

    def table_stacks(self, ntab: int):
        """Replay segments through reshuffles (tw_sgd_segment_narrow_tables): the row tables
        become slot 0 of stacks of 1 + ntab tables (N, kx) / (N, kz), the segment's reshuffles
        shipped into slots 1.. (0.. when it starts at one).  Growing them moves rows_x /
        rows_z: captured replay graphs hold the old addresses and are dropped."""
        st = getattr(self, "_stacks", None)
        if st is None or st[0].shape[0] < ntab + 1:
            t = self.t
            sx = L.empty((ntab + 1, self.N_loc, self.kx), t.int64)
            sz = L.empty((ntab + 1, self.N_loc, self.kz), t.int64)
            if self.rows_x is not None:
                sx[0].copy_(self.rows_x)
                sz[0].copy_(self.rows_z)
            self._stacks = st = (sx, sz)
            self.rows_x, self.rows_z = sx[0], sz[0]
            self._replay_graphs = {}
        return st

    def _fused_steps(self, nsteps: int, draws_dev=None, swr_mod=0, tables=None):
        """nsteps steps as nsteps tw_sgd_step launches + one tw_sgd_update_to (ping-pong
        slots for w/dw/grads; slot 0 = self.w/self.dw/self.grads holds the state before and
        after).  Same bits as step()/step_device() + _update() per step."""
        t = self.t
        if self._slot1 is None:
            self._slot1 = (t.empty_like(self.w), t.empty_like(self.dw), t.empty_like(self.grads))
        W, DW, Gs = zip((self.w, self.dw, self.grads), self._slot1)
        s = L.stream_handle()
        seed = getattr(self, "seed", 0) if draws_dev is None else 0
        if self.narrow_seg and nsteps > 1:
            # the whole segment in one persistent launch; then the last step's update, as below
            ix = iz = None
            stride = 0
            if draws_dev is not None:
                ix, iz = draws_dev[0, 0], draws_dev[0, 1]
                stride = int(draws_dev.stride(0))
            if tables is not None:  # replay through reshuffles: the stacks' tables by step
                sx, sz = self._stacks
                phase, mod = tables
                L.call("tw_sgd_segment_narrow_tables", L.ptr(self.X), L.ptr(self.Z), self.d,
                       L.ptr(sx), self.kx, L.ptr(sz), self.kz, int(sx.stride(0)),
                       int(sz.stride(0)), int(phase), int(mod), L.ptr(ix), L.ptr(iz), stride,
                       self.N_loc, self.B, self.margin, self.loss, seed, L.ptr(self.step_ctr),
                       self.shard_base, nsteps, L.ptr(W[0]), L.ptr(DW[0]), self.reg, self.lr,
                       self.momentum, L.ptr(Gs[0]), L.ptr(Gs[1]), L.ptr(W[1]), L.ptr(DW[1]),
                       L.ptr(self._ctl), s)
                # the last reshuffle's tables become slot 0 (evaluations, later segments)
                last_tab = (int(phase) + nsteps - 1) // int(mod)
                if last_tab > 0:
                    L.call("tw_copy_words", L.ptr(sx[last_tab]), sx[0].numel(), L.ptr(sx[0]), s)
                    L.call("tw_copy_words", L.ptr(sz[last_tab]), sz[0].numel(), L.ptr(sz[0]), s)
            elif swr_mod:  # device RNG: the segment draws its reshuffles' rows itself
                L.call("tw_sgd_segment_narrow_swr", L.ptr(self.X), L.ptr(self.Z), self.d,
                       self.n_X, self.n_Z, self.kx, self.kz, self.N_loc, self.B, self.margin,
                       self.loss, seed, L.ptr(self.step_ctr), self.shard_base, nsteps,
                       int(swr_mod), 0, L.ptr(W[0]), L.ptr(DW[0]), self.reg, self.lr,
                       self.momentum, L.ptr(Gs[0]), L.ptr(Gs[1]), L.ptr(W[1]), L.ptr(DW[1]),
                       L.ptr(self._ctl), s)
            else:
                L.call("tw_sgd_segment_narrow", L.ptr(self.X), L.ptr(self.Z), self.d,
                       L.ptr(self.rows_x), self.kx, L.ptr(self.rows_z), self.kz, L.ptr(ix),
                       L.ptr(iz), stride, self.N_loc, self.B, self.margin, self.loss, seed,
                       L.ptr(self.step_ctr), self.shard_base, nsteps, L.ptr(W[0]),
                       L.ptr(DW[0]), self.reg, self.lr, self.momentum, L.ptr(Gs[0]),
                       L.ptr(Gs[1]), L.ptr(W[1]), L.ptr(DW[1]), L.ptr(self._ctl), s)
            last = (nsteps - 1) & 1
            L.call("tw_sgd_update_to", L.ptr(W[1]), L.ptr(DW[1]), L.ptr(W[0]), L.ptr(DW[0]),
                   L.ptr(Gs[last]), self.N, self.d, self.reg, self.lr, self.momentum,
                   L.ptr(self.step_ctr), nsteps, s)
            return
        for k in range(nsteps):
            a, b = (k - 1) & 1, k & 1
            ix = iz = None
            if draws_dev is not None:
                ix, iz = draws_dev[k, 0], draws_dev[k, 1]
            pend = k > 0
            L.call("tw_sgd_step", L.ptr(self.X), L.ptr(self.Z), self.d, L.ptr(self.rows_x),
                   self.kx, L.ptr(self.rows_z), self.kz, L.ptr(ix), L.ptr(iz), self.N_loc,
                   self.B, self.margin, self.loss, seed, L.ptr(self.step_ctr), k,
                   self.shard_base, L.ptr(W[a] if pend else W[0]),
                   L.ptr(DW[a] if pend else None), L.ptr(Gs[a] if pend else None), self.reg,
                   self.lr, self.momentum, L.ptr(W[b] if pend else None),
                   L.ptr(DW[b] if pend else None), L.ptr(Gs[b]), s)
        last = (nsteps - 1) & 1
        L.call("tw_sgd_update_to", L.ptr(W[last]), L.ptr(DW[last]), L.ptr(W[0]), L.ptr(DW[0]),
               L.ptr(Gs[last]), self.N, self.d, self.reg, self.lr, self.momentum,
               L.ptr(self.step_ctr), nsteps, s)

    def _local(self, a):
        return a[self.shard_base:self.shard_base + self.N_loc]

    def set_shards(self, rows_x, rows_z):
        """Replay mode: the full SWR draw (all N shards; identical on every rank)."""
        if self.layout == "partitioned":
            self._exchange(L.to_device(np.stack(rows_x).astype(np.int64).reshape(-1)), 0)
            self._exchange(L.to_device(np.stack(rows_z).astype(np.int64).reshape(-1)), 1)
            self.rows_x, self.rows_z = self.tab_x, self.tab_z
            return
        # copied into persistent tables (captured replay graphs keep valid pointers) through a
        # pinned staging buffer, asynchronously: the host does not wait for queued steps
        t = self.t
        rx, rz = np.asarray(self._local(rows_x)), np.asarray(self._local(rows_z))
        if self.rows_x is None or tuple(self.rows_x.shape) != rx.shape:
            self.rows_x = L.empty(rx.shape, t.int64)
            self.rows_z = L.empty(rz.shape, t.int64)
            self._rows_pinned = (t.empty(rx.shape, dtype=t.int64, pin_memory=True),
                                 t.empty(rz.shape, dtype=t.int64, pin_memory=True))
            self._rows_done = None
        if self._rows_done is not None:
            self._rows_done.synchronize()  # the previous upload has left the staging buffer
        hx, hz = self._rows_pinned
        hx.numpy()[...] = rx
        hz.numpy()[...] = rz
        self.rows_x.copy_(hx, non_blocking=True)
        self.rows_z.copy_(hz, non_blocking=True)
        self._rows_done = t.cuda.Event()
        self._rows_done.record()

    def set_shards_staged(self, staged):
        """set_shards from rows already in pinned host tensors (the pipelined replay loop's
        staging ring, flat (N*kx + N*kz,)): two asynchronous copies of this engine's shards
        into the persistent tables; the caller keeps the staging buffer until they have run.
        False where the layout needs the host path (set_shards)."""
        if self.layout == "partitioned" or self.rows_x is None:
            return False
        flat, hdev = staged
        nx = self.N * self.kx
        a = self.shard_base
        if hdev is not None:  # the copy kernel reads the pinned buffer in place
            st = L.stream_handle()
            L.call("tw_copy_words", ctypes.c_void_p(hdev + 8 * a * self.kx),
                   self.N_loc * self.kx, L.ptr(self.rows_x), st)
            L.call("tw_copy_words", ctypes.c_void_p(hdev + 8 * (nx + a * self.kz)),
                   self.N_loc * self.kz, L.ptr(self.rows_z), st)
            return True
        self.rows_x.view(-1).copy_(flat[a * self.kx:(a + self.N_loc) * self.kx],
                                   non_blocking=True)
        self.rows_z.view(-1).copy_(flat[nx + a * self.kz:nx + (a + self.N_loc) * self.kz],
                                   non_blocking=True)
        return True

    def replay_through_ok(self) -> bool:
        """Replay segments may run through reshuffles (tw_sgd_segment_narrow_tables): one
        process, replicated X, the persistent narrow segment kernel."""
        return (self.narrow_seg and self.solo and self.layout == "replicated"
                and not self.complete and self.N_loc == self.N and self.rows_x is not None)

    def rows_ship_args(self, staged):
        """tw_ship_draws' row-table arguments for a reshuffle whose rows sit in a mapped pinned
        staging buffer (the pipelined replay loop; one process, replicated layout): (source
        device address, nx, rows_x, nz, rows_z), or None where set_shards_staged / set_shards
        must do it."""
        if self.layout == "partitioned" or self.rows_x is None or self.N_loc != self.N:
            return None
        flat, hdev = staged
        if hdev is None:
            return None
        return (hdev, self.N * self.kx, L.ptr(self.rows_x), self.N * self.kz,
                L.ptr(self.rows_z))

    def _side_matrix(self, part, k, remote=None):
        """One side's device matrix of the partitioned layout: the partition's rows, then room
        for `remote` received rows (default: the expected count with headroom, none at G = 1)
        — a remote row takes its d doubles, each sender's positions ceil(c / d) rows more."""
        t = self.t
        n_own = int(part.shape[0])
        if remote is None:
            M_q = self.N_loc * k
            remote = (0 if self.G == 1 else
                      M_q * (self.G - 1) // self.G + M_q // 16 + M_q // self.d + 2 * self.G)
        m = L.empty((n_own + remote, self.d), t.float64)
        if isinstance(part, t.Tensor):
            m[:n_own].copy_(part)
        else:
            m[:n_own].copy_(t.from_numpy(np.ascontiguousarray(part, dtype=np.float64)).reshape(
                n_own, self.d))
        return m

    def _records(self, name, words):
        """Persistent flat float64 send buffer for the row exchange, kept across reshuffles and
        grown with headroom only when a draw needs more (a fresh allocation per reshuffle made
        the caching allocator flush and re-map: a 1 s stall at C5)."""
        bufs = self.__dict__.setdefault("_xbufs", {})
        b = bufs.get(name)
        if b is None or b.shape[0] < words:
            bufs[name] = None  # release the old block first
            b = bufs[name] = L.empty((max(words + words // 16, 1),), self.t.float64)
        return b

    def _exchange(self, rows, side):
        """Partitioned layout, at a reshuffle: this rank's row table for `side` (0 = X, 1 = Z)
        from the global draws `rows` (all N*k global row indices, shard-major).  Owned rows are
        read in place in the partition; only rows owned by other ranks travel (one all_to_all
        of [rows | positions] buckets) and stay where they land in the receive area — no unpack
        pass, and at G = 1 nothing moves (compute_stats.py:48-54's copies become tables)."""
        t, G, d = self.t, self.G, self.d
        s = L.stream_handle()
        k = self.kx if side == 0 else self.kz
        lo, hi = self.x_own if side == 0 else self.z_own
        table = self.tab_x if side == 0 else self.tab_z
        n_own = hi - lo
        if not self.even:
            # uneven splits: every rank's positions padded to N_pad shards (row -1: owned by
            # no rank, so never counted, packed or received), the kernels' equal layout
            b, kp = self.shard_bounds, self.N_pad * k
            pad = t.full((G * kp,), -1, dtype=t.int64, device=rows.device)
            for g in range(G):
                pad[g * kp:g * kp + (b[g + 1] - b[g]) * k].copy_(rows[b[g] * k:b[g + 1] * k])
            rows = pad
        M, M_q = G * self.N_pad * k, self.N_pad * k
        mine = rows[self.rank * M_q:self.rank * M_q + self.N_loc * k]
        L.call("tw_row_table_local", L.ptr(mine), self.N_loc * k, lo, hi, L.ptr(table), s)
        if not self.coll:
            return
        part = self.X_part if side == 0 else self.Z_part
        counts = L.empty((G,), t.int64)
        L.call("tw_row_route_remote_counts", L.ptr(rows), M, M_q, lo, hi, G, self.rank,
               L.ptr(counts), s)
        rcounts = t.empty_like(counts)
        self.dist.all_to_all_single(rcounts, counts, group=self.group)
        both = t.stack([counts, rcounts]).cpu().tolist()
        sc, rc = both

        def layout(cs):  # per bucket: c rows of d words, then c positions padded to rows
            words = [c * d + -(-c // d) * d for c in cs]
            start = np.concatenate([[0], np.cumsum(words)[:-1]]).astype(np.int64)
            return words, start

        swords, sstart = layout(sc)
        rwords, rstart = layout(rc)
        send = self._records("send", int(sum(swords)))
        cursor = L.empty((G,), t.int64)
        # the device copies go to call() as tensors, held until the launch is enqueued: a
        # bare ptr() of a temporary freed it inside the argument list and handed its block to
        # the next temporary (round 4: the table call read its bucket starts from the prefix
        # array — masked at G = 2, where both begin 0, 0; found at G = 3).  ptr() now refuses
        # such a temporary (_lib.py).
        L.call("tw_row_pack_remote", L.ptr(rows), M, M_q, lo, hi, G, self.rank, L.ptr(part), d,
               L.to_device(sstart), L.ptr(counts), L.ptr(cursor), L.ptr(send), s)
        mat = self.X if side == 0 else self.Z
        need = n_own + int(sum(rwords)) // d
        if need > mat.shape[0]:  # more remote rows than the receive area holds: grow it
            mat = self._side_matrix(part, k, remote=need - n_own + need // 16)
            if side == 0:
                self.X, self.X_part = mat, mat[:n_own]
            else:
                self.Z, self.Z_part = mat, mat[:n_own]
            self._graphs, self._replay_graphs = {}, {}  # they hold the old matrix's address
        recv = mat.view(-1)[n_own * d:n_own * d + int(sum(rwords))]
        self.dist.all_to_all_single(recv, send[:int(sum(swords))], output_split_sizes=rwords,
                                    input_split_sizes=swords, group=self.group)
        rprefix = np.concatenate([[0], np.cumsum(rc)]).astype(np.int64)
        bad = t.zeros((1,), dtype=t.int64, device=table.device)
        L.call("tw_row_table_remote", L.ptr(recv), G, L.to_device(rstart), L.ptr(rcounts),
               L.to_device(rprefix), int(rprefix[-1]), d, n_own, L.ptr(table), table.numel(),
               recv.numel(), L.ptr(bad), s)
        b = int(bad.item())  # (the exchange already synchronised on its split sizes)
        if b:
            raise RuntimeError(f"partitioned row exchange: a received position ({b - 1}) lies "
                               f"outside this rank's {table.numel()}-entry row table "
                               f"(side {side}, G={G}, rank {self.rank}, sc={sc}, rc={rc})")

    def _update(self):
        if self.vgroup is not None:  # MultiDeviceSGD gathers the slots' gradients, then updates
            return
        if self.peer is not None:
            # one launch: this rank's partials into every rank's slot, wait for all, update
            par = self.peer.pstep & 1
            self.peer.pstep += 1
            cols = (self.G >= PEER_COLUMNS_MIN_RANKS if PEER_COLUMNS is None
                    else bool(PEER_COLUMNS)) and self.G > 1
            L.call("tw_peer_step_cols" if cols else "tw_peer_step",
                   L.ptr(self.grads_loc), self.N_loc * self.d,
                   self.shard_base * self.d, self.peer.bases, self.G, self.rank, self.N, self.d,
                   par, L.ptr(self.w), L.ptr(self.dw), self.reg, self.lr, self.momentum,
                   L.ptr(self.step_ctr), L.ptr(self._ctl[1:]), L.stream_handle())
            return
        if self.coll:
            if self.even:
                self.dist.all_gather_into_tensor(self.grads, self.grads_loc, group=self.group)
            else:  # padded per-rank blocks, then the N valid rows in shard order
                if getattr(self, "_gpad", None) is None:
                    t, b = self.t, self.shard_bounds
                    self._gpad = L.empty((self.G * self.N_pad, self.d), t.float64)
                    self._gidx = L.to_device(np.concatenate(
                        [np.arange(b[g + 1] - b[g]) + g * self.N_pad
                         for g in range(self.G)]).astype(np.int64))
                self.dist.all_gather_into_tensor(self._gpad, self.grads_loc, group=self.group)
                self.t.index_select(self._gpad, 0, self._gidx, out=self.grads)
        self._apply_update()

    def _peer_segment(self, nsteps: int, draws_dev=None, swr_mod: int = 0):
        """nsteps steps over ranks as ONE persistent launch (tw_sgd_segment_narrow_peer): this
        rank's shards, their gradients pushed into every rank's peer buffer in the launch, the
        update (the last one included) applied from the rank's own — the one-GPU trajectory.
        draws_dev: the replay draws (S, 2, N, B) of all shards, or None (device RNG)."""
        ix = iz = None
        stride = 0
        if draws_dev is not None:
            ix = draws_dev[0, 0, self.shard_base:]
            iz = draws_dev[0, 1, self.shard_base:]
            stride = int(draws_dev.stride(0))
        seed = getattr(self, "seed", 0) if draws_dev is None else 0
        L.call("tw_sgd_segment_narrow_peer", L.ptr(self.X), L.ptr(self.Z), self.d,
               L.ptr(self.rows_x), self.kx, L.ptr(self.rows_z), self.kz, L.ptr(ix), L.ptr(iz),
               stride, self.N_loc, self.B, self.margin, self.loss, seed, L.ptr(self.step_ctr),
               self.shard_base, nsteps, self.n_X, self.n_Z, int(swr_mod), L.ptr(self.w),
               L.ptr(self.dw), self.reg, self.lr, self.momentum, L.ptr(self._ctl),
               self.peer.bases, self.G, self.rank, self.N, L.stream_handle())

    def _apply_update(self):
        L.call("tw_sgd_update", L.ptr(self.w), L.ptr(self.dw), L.ptr(self.grads), self.N,
               self.d, self.reg, self.lr, self.momentum, L.ptr(self.step_ctr),
               L.stream_handle())

    def step_complete(self):
        """One step with the complete-block gradient (all kx*kz pairs of every local shard,
        tw_pair_grad_complete) — no pair draws."""
        t = self.t
        if self._cwork is None:
            nb = int(L.lib().tw_pair_grad_complete_work_bytes(self.N_loc, self.kx, self.kz,
                                                              self.d))
            self._cwork = L.empty((max(nb, 1),), t.uint8)
        L.call("tw_pair_grad_complete", L.ptr(self.X), L.ptr(self.Z), self.d,
               L.ptr(self.rows_x), self.kx, L.ptr(self.rows_z), self.kz, self.N_loc,
               L.ptr(self.w), self.margin, self.loss, L.ptr(self._cwork),
               L.ptr(self.grads_loc), L.stream_handle())
        self._update()

    def step(self, ix, iz, scores=None, local=False):
        """Replay mode: ix, iz are the (N, B) NumPy draws of every shard (host arrays or
        device tensors; local=True: already this engine's (N_loc, B) rows, on its device).
        scores: an (N_loc, B) float64 device tensor that receives every pair's
        S = diff . w + margin as the kernel computed it (tw_pair_grad_audit)."""
        t = self.t
        if local:
            ixd, izd = ix, iz
        else:
            ixd = self._local(ix) if isinstance(ix, t.Tensor) else L.to_device(self._local(ix))
            izd = self._local(iz) if isinstance(iz, t.Tensor) else L.to_device(self._local(iz))
        if scores is not None:
            L.call("tw_pair_grad_audit", L.ptr(self.X), L.ptr(self.Z), self.d,
                   L.ptr(self.rows_x), self.kx, L.ptr(self.rows_z), self.kz, L.ptr(ixd),
                   L.ptr(izd), self.N_loc, self.B, L.ptr(self.w), self.margin, self.loss,
                   L.ptr(self.grads_loc), L.ptr(scores), L.stream_handle())
        else:
            L.call("tw_pair_grad", L.ptr(self.X), L.ptr(self.Z), self.d, L.ptr(self.rows_x),
                   self.kx, L.ptr(self.rows_z), self.kz, L.ptr(ixd), L.ptr(izd), self.N_loc,
                   self.B, L.ptr(self.w), self.margin, self.loss, L.ptr(self.grads_loc),
                   L.stream_handle())
        self._update()

    def run_replay_segment(self, draws_dev, nsteps: int, graphs: bool = True, tag=0,
                           upload=None, tables=None):
        """nsteps replay steps whose NumPy draws sit in draws_dev[s] ((2, N, B) int64 on the
        device): one gradient + one update launch per step, replayed from a hipGraph captured
        per (tag, nsteps) — tag names the draw buffer, whose address the graph holds — or
        launched eagerly (graphs=False, or a collective in the step).  upload: (key, fn) — fn
        enqueues the segment's upload (tw_ship_draws), captured in the same graph (one graph
        launch per segment); key names its arguments.  tables: (phase, mod) — a narrow segment
        running through reshuffles whose row tables sit in table_stacks (replay_through)."""
        def one(st):
            if self.complete:
                self.step_complete()
            else:
                self.step(draws_dev[st, 0], draws_dev[st, 1])

        def steps():
            if self.peer_seg:
                self._peer_segment(nsteps, draws_dev)
            elif self.fused:
                self._fused_steps(nsteps, draws_dev, tables=tables)
            else:
                for st in range(nsteps):
                    one(st)

        # a persistent narrow segment is two launches (plus the upload): eager launches cost
        # ~1.5 us per boundary on the stream, a graph launch ~12 (kernel traces r03s31/s32)
        if not graphs or not self.solo or (self.narrow_seg and nsteps > 1 and not self.complete):
            if upload is not None:
                upload[1]()
            steps()
            return
        t = self.t
        if not hasattr(self, "_replay_graphs"):
            self._replay_graphs = {}
        # tables (phase, mod) in the key: a captured graph holds its table-stack phase, so a
        # graph captured for one phase is never replayed at another
        key = (tag, nsteps, draws_dev.data_ptr() if draws_dev is not None else 0,
               None if upload is None else upload[0], tables)
        g = self._replay_graphs.get(key)
        if g is None:
            if self.complete and self._cwork is None:  # allocated outside the capture
                nb = int(L.lib().tw_pair_grad_complete_work_bytes(self.N_loc, self.kx,
                                                                  self.kz, self.d))
                self._cwork = L.empty((max(nb, 1),), t.uint8)
            if self.fused and self._slot1 is None:  # allocated outside the capture
                self._slot1 = (t.empty_like(self.w), t.empty_like(self.dw),
                               t.empty_like(self.grads))
            g = t.cuda.CUDAGraph()
            with L.capture(g):
                if upload is not None:
                    upload[1]()
                steps()
            self._replay_graphs[key] = g
        g.replay()

    def batch_view(self):
        """The current shards as evaluation_step's SAME_AS_BATCH reads them: (X, Z, row tables
        or None, N, kx, kz) on the device (one process only; None with several ranks)."""
        if not self.solo or self.rows_x is None:
            return None
        return (self.X, self.Z, self.rows_x, self.rows_z, self.N, self.kx, self.kz)

    def w_host(self) -> np.ndarray:
        self.check()
        return self.w.cpu().numpy().reshape(self.w_shape)

    def w_host_async(self):
        """Start copying w to pinned host memory; returns a callable that waits and gives
        the array (the host can draw the next segment meanwhile)."""
        t = self.t
        if getattr(self, "_w_pinned", None) is None:
            self._w_pinned = t.empty(self.w.shape, dtype=t.float64, pin_memory=True)
            self._w_event = t.cuda.Event()
        self._w_pinned.copy_(self.w, non_blocking=True)
        self._w_event.record()

        def wait():
            self._w_event.synchronize()
            self.check()
            return self._w_pinned.numpy().reshape(self.w_shape).copy()
        return wait

    # ------------------------------------------------------------ device-RNG mode
    def enable_device_rng(self, seed: int):
        """Draw SWR rows and pair indices on the device (Philox keyed by `seed`, counter =
        the step number kept in device memory).  Steps then need no host work at all and can
        be captured in hipGraphs."""
        t = self.t
        self.seed = int(seed) & (2 ** 64 - 1)
        self.step_ctr = t.zeros((1,), dtype=t.int64, device=self.w.device)
        if self.layout == "partitioned":  # owners need every shard's draws
            self.rows_all_x = t.empty((self.N, self.kx), dtype=t.int64, device=self.w.device)
            self.rows_all_z = t.empty((self.N, self.kz), dtype=t.int64, device=self.w.device)
            self.rows_x, self.rows_z = self.tab_x, self.tab_z
        else:
            self.rows_x = t.empty((self.N_loc, self.kx), dtype=t.int64, device=self.w.device)
            self.rows_z = t.empty((self.N_loc, self.kz), dtype=t.int64, device=self.w.device)
        self._graphs = {}

    def swr_segments_ok(self, nsteps: int = 2) -> bool:
        """run_segment(nsteps, swr_mod=) applies: device RNG, one process, replicated rows,
        the incomplete gradient, and a kernel that draws the rows — the persistent narrow
        segment (nsteps > 1) or the per-step gradient launches of wide rows."""
        # (partitioned at G = 1: the partition is all of X and the tables are the draws)
        if self.peer_seg and getattr(self, "seed", None) is not None:
            # over ranks: the peer segment draws the rows itself (global rows: replicated X)
            return self.layout == "replicated" or self.G == 1
        if getattr(self, "seed", None) is None or not self.solo or self.complete:
            return False
        if self.narrow_seg:
            return nsteps > 1
        return not self.fused

    def reshuffle_device(self, counter=None):
        """New SWR row tables from the device RNG at the current step counter, or at `counter`
        (the step of an earlier reshuffle: the tables a swr segment left stale)."""
        s = L.stream_handle()
        if counter is not None:
            t = self.t
            if getattr(self, "_swr_ctr", None) is None:
                self._swr_ctr = t.zeros((1,), dtype=t.int64, device=self.w.device)
            self._swr_ctr.copy_(t.tensor([int(counter)], dtype=t.int64))
            for side, rows, k, n in ((0, self.rows_x, self.kx, self.n_X),
                                     (1, self.rows_z, self.kz, self.n_Z)):
                L.call("tw_swr_rows_rng", L.ptr(rows), self.N_loc, k, n, self.seed,
                       L.ptr(self._swr_ctr), side, self.shard_base, s)
            return
        if self.layout == "partitioned":
            L.call("tw_swr_rows_rng", L.ptr(self.rows_all_x), self.N, self.kx, self.n_X,
                   self.seed, L.ptr(self.step_ctr), 0, 0, s)
            L.call("tw_swr_rows_rng", L.ptr(self.rows_all_z), self.N, self.kz, self.n_Z,
                   self.seed, L.ptr(self.step_ctr), 1, 0, s)
            self._exchange(self.rows_all_x.view(-1), 0)
            self._exchange(self.rows_all_z.view(-1), 1)
            return
        L.call("tw_swr_rows_rng", L.ptr(self.rows_x), self.N_loc, self.kx, self.n_X, self.seed,
               L.ptr(self.step_ctr), 0, self.shard_base, s)
        L.call("tw_swr_rows_rng", L.ptr(self.rows_z), self.N_loc, self.kz, self.n_Z, self.seed,
               L.ptr(self.step_ctr), 1, self.shard_base, s)

    def step_device(self, swr_mod: int = 0):
        if self.complete:
            return self.step_complete()
        if swr_mod:  # the rows of the step's last reshuffle, drawn in the kernel
            L.call("tw_pair_grad_rng_swr", L.ptr(self.X), L.ptr(self.Z), self.d, self.n_X,
                   self.n_Z, self.kx, self.kz, self.N_loc, self.B, L.ptr(self.w), self.margin,
                   self.loss, self.seed, L.ptr(self.step_ctr), self.shard_base, int(swr_mod), 0,
                   L.ptr(self.grads_loc), L.stream_handle())
            self._update()
            return
        L.call("tw_pair_grad_rng", L.ptr(self.X), L.ptr(self.Z), self.d, L.ptr(self.rows_x),
               self.kx, L.ptr(self.rows_z), self.kz, self.N_loc, self.B, L.ptr(self.w),
               self.margin, self.loss, self.seed, L.ptr(self.step_ctr), self.shard_base,
               L.ptr(self.grads_loc), L.stream_handle())
        self._update()

    def run_segment(self, nsteps: int, reshuffle_first: bool, graphs: bool = True,
                    swr_mod: int = 0):
        """nsteps device-RNG steps (reshuffling first if asked), replayed from a captured
        hipGraph per distinct segment shape (eager when the step holds a collective).
        swr_mod: the kernels draw the SWR rows of every reshuffle (one every swr_mod steps from
        step counter 0) themselves (tw_sgd_segment_narrow_swr, tw_pair_grad_rng_swr) — the
        device row tables are then NOT updated (swr_segments_ok says when this applies)."""
        t = self.t
        if swr_mod:
            assert self.swr_segments_ok(nsteps) and not reshuffle_first
            if self.peer_seg:
                self._peer_segment(nsteps, swr_mod=swr_mod)
                return
            if self.fused and self._slot1 is None:
                self._slot1 = (t.empty_like(self.w), t.empty_like(self.dw),
                               t.empty_like(self.grads))
            if self.narrow_seg and nsteps > 1:  # one persistent launch, eager (§4.4e)
                self._fused_steps(nsteps, swr_mod=swr_mod)
                return
        if reshuffle_first and self.layout == "partitioned":
            self.reshuffle_device()  # the exchange sizes its buffers on the host: not captured
            reshuffle_first = False

        def steps(n):
            if swr_mod:
                for _ in range(n):
                    self.step_device(swr_mod=swr_mod)
            elif self.peer_seg:
                self._peer_segment(n)
            elif self.fused:
                self._fused_steps(n)
            else:
                for _ in range(n):
                    self.step_device()

        if not graphs or not self.solo:
            if reshuffle_first:
                self.reshuffle_device()
            steps(nsteps)
            return
        if self.fused and self._slot1 is None:  # allocated outside any capture
            self._slot1 = (t.empty_like(self.w), t.empty_like(self.dw), t.empty_like(self.grads))
        while nsteps > 0:
            n = min(nsteps, 256)
            key = (n, reshuffle_first, swr_mod)
            g = self._graphs.get(key)
            if g is None:
                g = t.cuda.CUDAGraph()
                side = t.cuda.Stream()
                side.wait_stream(t.cuda.current_stream())
                with t.cuda.stream(side):  # warm the launch path outside capture
                    pass
                t.cuda.current_stream().wait_stream(side)
                with L.capture(g):
                    if reshuffle_first:
                        self.reshuffle_device()
                    steps(n)
                self._graphs[key] = g
            g.replay()
            nsteps -= n
            reshuffle_first = False


_PEERS = {}  # (process group, G, rank, N, d) -> _PeerBuffers: one set per shape, kept


class _PeerBuffers:
    """This rank's peer buffer (csrc/peer.hip, tw_peer_alloc: counters and gradient slots of
    the device-resident exchange) and every other rank's, mapped through IPC handles exchanged
    once over the process group.  create() is collective: every rank learns whether all ranks
    allocated and mapped their buffers, and all fall back to the RCCL all-gather together if
    one could not (a warning names the reason).  The buffers of a (group, N, d) shape are kept
    for the process and handed to every later engine of that shape: freeing one while a peer
    still maps it, and mapping its successor at the same address, made the next open fail (a
    C5 engine after a C4 one).  The persistent segments' epoch lives in the buffer and the
    per-step exchange's parity (pstep) lives here, so a later engine continues both."""

    def __init__(self, mine, uncached, opened, bases):
        self.mine = ctypes.c_void_p(mine)
        self.uncached = uncached
        self.opened = opened
        self.bases = bases
        self.pstep = 0  # steps of the per-step exchange through these buffers (its parity)

    @staticmethod
    def create(eng):
        import warnings
        dist, group, G, r = eng.dist, eng.group, eng.G, eng.rank
        key = (id(group), G, r, eng.N, eng.d)
        have = _PEERS.get(key)
        flags = [None] * G
        dist.all_gather_object(flags, have is not None, group=group)
        if all(flags):
            return have
        lib = L.lib()
        mine, unc, handle, why = None, 0, None, None
        try:
            nb = int(lib.tw_peer_buffer_bytes(eng.N, eng.d))
            p, u = ctypes.c_void_p(), ctypes.c_int32(0)
            if G <= 16 and nb > 0:
                L.call("tw_peer_alloc", nb, ctypes.byref(p), ctypes.byref(u))
                mine, unc = p.value, int(u.value)
                h = (ctypes.c_uint8 * 64)()
                if G > 1:
                    L.call("tw_peer_handle", ctypes.c_void_p(mine), h)
                handle = bytes(h)
            else:
                why = f"{G} ranks (at most 16)"
        except Exception as e:  # this rank cannot take part: every rank falls back
            handle, why = None, f"allocation / handle: {e}"
        handles = [None] * G
        dist.all_gather_object(handles, handle, group=group)
        opened, bases, ok = [], [], all(hb is not None for hb in handles)
        if ok:
            try:
                for q, hb in enumerate(handles):
                    if q == r:
                        bases.append(mine)
                        continue
                    v = ctypes.c_void_p()
                    L.call("tw_peer_open", (ctypes.c_uint8 * 64).from_buffer_copy(hb),
                           ctypes.byref(v))
                    opened.append(v.value)
                    bases.append(v.value)
            except Exception as e:
                ok, why = False, f"opening a peer's handle: {e}"
        # the handshake: every rank's GPU stores a token into every rank's buffer through the
        # mappings; each checks its own after a barrier (a mapping that opened but does not
        # carry stores is found here, before any step relies on it)
        token = 0x7E5E_0000_0000 + 1 + int(np.random.default_rng().integers(1 << 30))
        tokens = [None] * G
        dist.all_gather_object(tokens, token if ok else None, group=group)
        ok = ok and all(tk is not None for tk in tokens)
        token = tokens[0] if ok else 0
        if ok:
            try:
                bases_arr = (ctypes.c_void_p * G)(*bases)
                L.call("tw_peer_hello", bases_arr, G, r, token, L.stream_handle())
            except Exception as e:
                ok, why = False, f"handshake stores: {e}"
        dist.all_gather_object([None] * G, ok, group=group)  # the barrier: every hello landed
        if ok:
            good = ctypes.c_int32(0)
            try:
                L.call("tw_peer_check", ctypes.c_void_p(mine), G, token, ctypes.byref(good))
                ok = bool(good.value)
                if not ok:
                    why = "handshake: a peer's token did not arrive"
            except Exception as e:
                ok, why = False, f"handshake check: {e}"
        oks = [None] * G
        dist.all_gather_object(oks, (ok, why), group=group)
        if not all(o for o, _ in oks):
            for v in opened:
                lib.tw_peer_close(ctypes.c_void_p(v))
            if mine is not None:
                lib.tw_peer_free(ctypes.c_void_p(mine))
            reasons = "; ".join(f"rank {q}: {w}" for q, (o, w) in enumerate(oks) if not o)
            warnings.warn("learning over ranks: the device-resident gradient exchange is "
                          f"unavailable ({reasons}); using the RCCL all-gather per step")
            return None
        pb = _PeerBuffers(mine, unc, opened, (ctypes.c_void_p * G)(*bases))
        _PEERS[key] = pb
        return pb


class MultiDeviceSGD:
    """learning_process's engine over several devices of ONE process (the
    reference's N workers are a serial in-process loop, make_exps.py:126-141 calling UN_split,
    compute_stats.py:44-46).  Slot r (one SGDEngine per device, its own stream) owns shards
    [r*N/G, (r+1)*N/G) with replicated X and Z; every step each slot computes its shards'
    gradients, the (N/G, d) blocks are all-gathered in shard order — RCCL (tw_allgather_f64)
    when the devices are distinct, stream-ordered device copies otherwise — and every slot
    applies the same shard-ordered update, so w (hence the trajectory) is identical to one
    device bit for bit.  Eager launches (no graphs); replicated layout, incomplete gradient.
    Device lists may repeat a device (tests run [0, 0] on a one-GPU box)."""

    def __init__(self, X, Z, w_init, N, B, margin, reg, learning_rate, optim_type, devices,
                 loss="hinge"):
        from . import _multi as M
        t = L.torch()
        self.t, self.M = t, M
        devs = [int(v) for v in devices]
        self.G = len(devs)
        if self.G < 2 or int(N) % self.G:
            raise ValueError(f"N={N} shards do not split over {self.G} devices")
        self.slots = [M._Slot(dev, k) for k, dev in enumerate(devs)]
        self.subs = []
        for r, slot in enumerate(self.slots):
            with slot:
                self.subs.append(SGDEngine(X, Z, w_init, N, B, margin, reg, learning_rate,
                                           optim_type, loss=loss, vgroup=(self.G, r)))
        e0 = self.subs[0]
        self.N, self.B, self.d, self.kx, self.kz = e0.N, e0.B, e0.d, e0.kx, e0.kz
        self.N_loc, self.complete, self.layout, self.fused = e0.N_loc, False, "replicated", False
        self.comm = M._comm(tuple(devs)) if len(set(devs)) == len(devs) else None
        self.rows_x = None

    # ---------------------------------------------------------------- per step
    def _gather_update(self):
        """All slots' (N_loc, d) gradients -> every slot's (N, d) buffer, then the update."""
        t, subs, slots = self.t, self.subs, self.slots
        if self.comm is not None:
            P = ctypes.c_void_p * self.G
            L.call("tw_allgather_f64", self.comm, P(*[e.grads_loc.data_ptr() for e in subs]),
                   P(*[e.grads.data_ptr() for e in subs]), self.N_loc * self.d,
                   P(*[sl.stream.cuda_stream for sl in slots]))
        else:
            evs = []
            for sl in slots:
                with sl:
                    ev = t.cuda.Event()
                    ev.record()
                    evs.append(ev)
            for sl, e in zip(slots, subs):
                with sl:
                    for ev in evs:
                        t.cuda.current_stream().wait_event(ev)
                    for r, o in enumerate(subs):
                        e.grads[r * self.N_loc:(r + 1) * self.N_loc].copy_(o.grads_loc)
        for sl, e in zip(slots, subs):
            with sl:
                e._apply_update()
        # a slot's next gradients overwrite grads_loc, which the others' copies read
        if self.comm is None:
            evs = []
            for sl in slots:
                with sl:
                    ev = t.cuda.Event()
                    ev.record()
                    evs.append(ev)
            for sl in slots:
                with sl:
                    for ev in evs:
                        t.cuda.current_stream().wait_event(ev)

    def step(self, ix, iz, scores=None):
        if scores is not None:
            raise ValueError("sign_audit runs on one device")
        t = self.t
        if not isinstance(ix, t.Tensor):  # host draws: each slot uploads its own rows
            for sl, e in zip(self.slots, self.subs):
                with sl:
                    e.step(ix, iz)
            self._gather_update()
            return
        # device draws live on the caller's device, written on the caller's stream (a
        # non-blocking upload): each slot orders its stream after it, takes a copy of its rows
        # on its own device, and the caller's stream waits for those copies before the draw
        # buffer can be refilled (as run_replay_segment does)
        caller = t.cuda.current_stream()
        loc = []
        for sl, e in zip(self.slots, self.subs):
            with sl:
                t.cuda.current_stream().wait_stream(caller)
                a = e.shard_base
                # copy=True: on a repeated device .to() would return a view of the buffer
                loc.append((ix[a:a + e.N_loc].to(L.device(), non_blocking=True, copy=True),
                            iz[a:a + e.N_loc].to(L.device(), non_blocking=True, copy=True)))
        for sl in self.slots:
            caller.wait_stream(sl.stream)
        for sl, e, (lx, lz) in zip(self.slots, self.subs, loc):
            with sl:
                e.step(lx, lz, local=True)
        self._gather_update()

    def set_shards(self, rows_x, rows_z):
        for sl, e in zip(self.slots, self.subs):
            with sl:
                e.set_shards(rows_x, rows_z)
        self.rows_x = True

    def run_replay_segment(self, draws_dev, nsteps: int, graphs: bool = True, tag=0):
        """nsteps replay steps, eagerly: each slot gets its shards' draws on its device."""
        t = self.t
        caller = t.cuda.current_stream()  # the draws were uploaded on it
        loc = []
        for sl, e in zip(self.slots, self.subs):
            with sl:
                t.cuda.current_stream().wait_stream(caller)
                a = e.shard_base
                loc.append(draws_dev[:nsteps, :, a:a + e.N_loc].to(L.device(), non_blocking=True)
                           .contiguous())
        for sl in self.slots:  # the draw buffer is refilled on the caller's stream later
            caller.wait_stream(sl.stream)
        for st in range(nsteps):
            for sl, e, dl in zip(self.slots, self.subs, loc):
                with sl:
                    e.step(dl[st, 0], dl[st, 1], local=True)
            self._gather_update()

    # ---------------------------------------------------------------- device RNG
    def enable_device_rng(self, seed: int):
        for sl, e in zip(self.slots, self.subs):
            with sl:
                e.enable_device_rng(seed)
        self.rows_x = True

    def reshuffle_device(self):
        for sl, e in zip(self.slots, self.subs):
            with sl:
                e.reshuffle_device()

    def step_device(self):
        for sl, e in zip(self.slots, self.subs):
            with sl:
                e.step_device()
        self._gather_update()

    def run_segment(self, nsteps: int, reshuffle_first: bool, graphs: bool = True):
        if reshuffle_first:
            self.reshuffle_device()
        for _ in range(nsteps):
            self.step_device()

    # ---------------------------------------------------------------- w
    @property
    def w(self):
        """Slot 0's w, ordered after slot 0's queued steps on the caller's current stream."""
        self.t.cuda.current_stream().wait_stream(self.slots[0].stream)
        return self.subs[0].w

    def w_host(self) -> np.ndarray:
        with self.slots[0]:
            return self.subs[0].w_host()

    def w_host_async(self):
        with self.slots[0]:
            return self.subs[0].w_host_async()

    def batch_view(self):
        return None

    def check(self):
        pass


MULTI_DEVICE_MIN_BYTES = 1 << 30  # gathered row bytes per step below which one device is used


def _engine_for(X, Z, w, N, B, margin, reg, learning_rate, optim_type, group, x_layout, loss,
                gradient, rng_mode, plain, collectives=None):
    """learning_process's one-device engine: the cached one when this call matches it (replay
    mode on host arrays, same shapes and hyper-parameters; ENGINE_CACHE), else a new one
    (cached in turn when the call qualifies).  Device-RNG runs are not cached: their graphs
    hold the run's seed."""
    cacheable = (ENGINE_CACHE and plain and rng_mode == "replay" and group is None
                 and not collectives
                 and x_layout == "replicated"
                 and isinstance(X, np.ndarray) and isinstance(Z, np.ndarray)
                 and X.ndim == 2 and Z.ndim == 2
                 and 8 * (X.shape[0] + Z.shape[0]) * X.shape[1] <= ENGINE_CACHE_MAX_BYTES)
    key = None
    if cacheable:
        key = (X.shape, Z.shape, int(np.asarray(w).size), int(N), int(B), float(margin),
               float(reg), float(learning_rate), optim_type, loss, gradient,
               L.torch().cuda.current_device(), NARROW_SEGMENT)
        eng = _ENGINE["eng"]
        if _ENGINE["key"] == key:
            eng.reload(X, Z, np.asarray(w, dtype=np.float64))
            return eng
    eng = SGDEngine(X, Z, w, N, B, margin, reg, learning_rate, optim_type, group=group,
                    x_layout=x_layout, loss=loss, gradient=gradient, collectives=collectives)
    if cacheable:
        _ENGINE["key"], _ENGINE["eng"] = None, None  # release the previous engine first
        _ENGINE["key"], _ENGINE["eng"] = key, eng
    return eng


def _engine_devices(devices, N, B, d, group, x_layout, gradient):
    """The device list learning_process spreads over, or None (one device): explicit
    `devices`, else TW_DEVICES / every visible device once a step gathers >= 1 GiB of rows."""
    from . import _multi as M
    if group is not None or x_layout != "replicated" or gradient != "incomplete":
        if devices is not None and len(devices) > 1:
            raise ValueError("devices= needs group=None, x_layout='replicated' and the "
                             "incomplete gradient")
        return None
    if devices is None:
        devs = M.devices()
        if len(devs) < 2 or 16 * N * B * d < MULTI_DEVICE_MIN_BYTES:
            return None
        devices = devs
    devices = list(devices)
    if len(devices) < 2:
        return None
    G = len(devices)
    while G > 1 and N % G:
        G -= 1
    return devices[:G] if G > 1 else None


def _dev_f64(a):
    t = L.torch()
    if isinstance(a, t.Tensor):
        return a.to(device=L.device(), dtype=t.float64).contiguous()
    return L.to_device(np.asarray(a, dtype=np.float64))


class _ReplayDraws:
    """NumPy's own draws for the replay loop, made natively (tuplewise.numpy_rng.Session):
    SWR_divide's rows (compute_stats.py:52-53) and grad_inc_block's pairs (:155-156).  Pair
    draws go into one of two pinned host buffers and ship with one asynchronous H2D copy, so
    the host draws step i+1 while the device runs step i."""

    def __init__(self, N, kx, kz, B):
        t = L.torch()
        self.N, self.kx, self.kz, self.B = N, kx, kz, B
        self.host = [t.empty((2, N, B), dtype=t.int64, pin_memory=True) for _ in range(2)]
        self.hnp = [h.numpy() for h in self.host]
        self.dev = [L.empty((2, N, B), t.int64) for _ in range(2)]
        self.done = [None, None]  # event: the copy out of host[k] has finished
        self.k = 0
        self.rng = Session()

    def _swr_setup(self, n_X, n_Z):
        """SWR_divide's randint arguments: N calls on [0, n_X) of kx draws, then N on [0, n_Z)."""
        N, kx, kz = self.N, int(n_X / self.N), int(n_Z / self.N)
        if getattr(self, "_swr_args", (None,))[0] != (N, n_X, n_Z, kx, kz):
            self._swr_args = ((N, n_X, n_Z, kx, kz), np.zeros(2 * N, np.int64),
                              np.array([n_X] * N + [n_Z] * N, np.int64),
                              np.array([kx] * N + [kz] * N, np.int64))
        return self._swr_args[1:]

    def swr_rows(self, n_X, n_Z):
        N, kx, kz = self.N, int(n_X / self.N), int(n_Z / self.N)
        flat = self.rng.randint_flat(*self._swr_setup(n_X, n_Z))
        # (N, kx) and (N, kz) arrays: row s is shard s's draw (indexable like the list of
        # arrays SWR_divide returns)
        return flat[:N * kx].reshape(N, kx), flat[N * kx:].reshape(N, kz)

    def swr_rows_staged(self, k, n_X, n_Z):
        """swr_rows drawn straight into pinned row buffer k of the pipelined loop (ring of 3,
        reused once the upload out of it has finished): (rows_x, rows_z) host views and the
        pinned tensors."""
        N, kx, kz = self._rows_buffers(n_X, n_Z)
        buf, ev = self.rows3[k]
        if self.rows3_used[k]:
            ev.synchronize()
        flat = buf.numpy()[:N * kx + N * kz]
        self.rng.randint_flat(*self._swr_setup(n_X, n_Z), out=flat)
        return (flat[:N * kx].reshape(N, kx), flat[N * kx:].reshape(N, kz)), (buf,
                                                                             self.rows3_hdev[k])

    def _rows_buffers(self, n_X, n_Z, ntab=1):
        """The ring of three pinned SWR row buffers (flat N*kx + N*kz int64 per table, ntab
        tables; mapped)."""
        t = L.torch()
        N, kx, kz = self.N, int(n_X / self.N), int(n_Z / self.N)
        per = N * kx + N * kz
        if (getattr(self, "rows3", None) is None or self.rows3_per != per
                or self.rows3[0][0].shape[0] < per * ntab):
            self.rows3 = None  # release the old ring first
            self.rows3_per = per
            self.rows3 = [(t.empty((per * ntab,), dtype=t.int64, pin_memory=True),
                           t.cuda.Event()) for _ in range(3)]
            self.rows3_used = [False] * 3
            self.rows3_hdev = [L.host_device_pointer(b) for b, _ in self.rows3]
        return N, kx, kz

    def native_pipe(self, segs, n_X, n_Z, mod, row_width=8, through=False):
        """The loop's draws made ahead by a native thread (tw_draw_pipe_*, csrc/drawpipe.hip)
        into the ring of pinned segment and row buffers: segs = [(i, nxt, ntab)] — ntab row
        tables in segment [i, nxt) (its reshuffles: the steps i + k with (i + k) % mod == 0;
        a segment cut at reshuffles has ntab 1 when it starts at one, else 0).  row_width 2:
        the tables drawn as uint16 (n_X, n_Z <= 65536; ship_tables widens them)."""
        t = L.torch()
        self._seg_buffers(3)
        ntab = max([1] + [int(r) for _, _, r in segs])
        if ntab > 1 or through:
            # through reshuffles: room for a full segment's tables (see table_stacks) — also on
            # a run whose own segments hold one table at most (a short first call), so a later
            # longer run does not re-allocate the pinned ring inside its loop (the first-run
            # penalty of VERDICT r04 weak 6: ~60 MB of pinned memory at C4)
            ntab = max(ntab, min(self.segment_capacity(), self.table_capacity(n_X, n_Z)))
        N, kx, kz = self._rows_buffers(n_X, n_Z, ntab)
        t.cuda.current_stream().synchronize()  # earlier uploads out of the ring have run
        steps = np.array([b - a for a, b, _ in segs], dtype=np.int32)
        phase = np.array([a % mod for a, _, _ in segs], dtype=np.int32)
        P = ctypes.c_void_p * 3
        segp = P(*[h.data_ptr() for h in self.seg3_host])
        rowp = P(*[b.data_ptr() for b, _ in self.rows3])
        h = ctypes.c_void_p()
        L.call("tw_draw_pipe_start", self.rng._key, self.rng._pos, len(segs),
               steps.ctypes.data, phase.ctypes.data, int(mod), N, self.kx, self.kz, self.B,
               int(n_X), int(n_Z), self.seg3_w, 3, segp, rowp, ntab, int(row_width),
               ctypes.byref(h))
        self.rows3_rw = int(row_width)
        return _NativeDraws(self, h, segs, N, kx, kz, (steps, phase, segp, rowp))

    def ship_tables(self, k, S, ntab, slot, eng):
        """Main side, replay through reshuffles: buffer k's S steps of draws widened on the
        device and its ntab row tables into eng's table stacks from `slot` on, in one launch
        (tw_ship_draws_tables); returns the int64 device draws."""
        sx, sz = eng._stacks
        n = int(S) * 2 * self.N * self.B
        L.call("tw_ship_draws_tables", ctypes.c_void_p(self.seg3_hdev[k]), self.seg3_w, n,
               L.ptr(self.seg3_dev[k]), ctypes.c_void_p(self.rows3_hdev[k]), self.rows3_rw,
               int(ntab),
               sx[0].numel(), L.ptr(sx[slot]), sz[0].numel(), L.ptr(sz[slot]),
               L.stream_handle())
        return self.seg3_dev[k]

    def table_capacity(self, n_X, n_Z) -> int:
        """Row tables per segment when replaying through reshuffles: <= 32 MiB of int64 rows
        per ring buffer."""
        per = 8 * (self.N * int(n_X / self.N) + self.N * int(n_Z / self.N))
        return int(max(1, (32 << 20) // per))

    def rows_uploaded(self, k):
        """Main side: the upload out of pinned row buffer k has been enqueued."""
        self.rows3[k][1].record()
        self.rows3_used[k] = True

    def segment_capacity(self) -> int:
        """Steps per drawn segment: <= 256, and <= 64 MiB of int64 draws per buffer."""
        per = 2 * self.N * self.B * 8
        return int(max(1, min(256, (64 << 20) // per)))

    def pairs_segment(self, S):
        """Draws of the next S steps (NumPy's order) into one of two pinned buffers, shipped
        with one asynchronous H2D copy; returns (device buffer (S_cap, 2, N, B), tag)."""
        t = L.torch()
        if not hasattr(self, "seg_host"):
            cap = self.segment_capacity()
            shape = (cap, 2, self.N, self.B)
            self.seg_host = [t.empty(shape, dtype=t.int64, pin_memory=True) for _ in range(2)]
            self.seg_np = [h.numpy() for h in self.seg_host]
            self.seg_dev = [L.empty(shape, t.int64) for _ in range(2)]
            self.seg_done = [None, None]
            self.seg_k = 0
        k = self.seg_k
        self.seg_k ^= 1
        if self.seg_done[k] is not None:
            self.seg_done[k].synchronize()  # the copy out of seg_host[k] two segments back
        self.rng.pairs_steps(S, self.N, self.kx, self.kz, self.B, self.seg_np[k])
        # stream-ordered: the graph that read seg_dev[k] two segments back precedes this copy
        self.seg_dev[k][:S].copy_(self.seg_host[k][:S], non_blocking=True)
        if self.seg_done[k] is None:
            self.seg_done[k] = t.cuda.Event()
        self.seg_done[k].record()
        return self.seg_dev[k], k

    def _seg_buffers(self, nbuf):
        """Pinned draw buffers of the pipelined loop, narrowed when every index fits — uint8
        (kx, kz <= 256; NARROW_DRAWS_U8) or uint16 (<= 65536): an eighth / a quarter of the
        int64 bytes (a 25-step C4 segment is 4 MB as int64) — and widened on the device into
        the int64 buffers the segment graphs read."""
        t = L.torch()
        if getattr(self, "seg3_host", None) is None:
            cap = self.segment_capacity()
            shape = (cap, 2, self.N, self.B)
            self.seg3_w = (1 if NARROW_DRAWS_U8 and self.kx <= 256 and self.kz <= 256
                           else 2 if self.kx <= 65536 and self.kz <= 65536 else 8)
            # torch storage of the narrow bits (viewed unsigned on the host)
            hdt, npv = {1: (t.uint8, np.uint8), 2: (t.int16, np.uint16),
                        8: (t.int64, np.int64)}[self.seg3_w]
            self.seg3_host = [t.empty(shape, dtype=hdt, pin_memory=True) for _ in range(nbuf)]
            self.seg3_np = [h.numpy().view(npv) for h in self.seg3_host]
            self.seg3_stage = ([L.empty(shape, hdt) for _ in range(nbuf)]
                               if self.seg3_w < 8 else None)
            self.seg3_dev = [L.empty(shape, t.int64) for _ in range(nbuf)]
            self.seg3_done = [t.cuda.Event() for _ in range(nbuf)]
            self.seg3_used = [False] * nbuf
            # the widening kernel reads the pinned buffers in place (mapped host memory): one
            # launch per segment instead of a copy call and a launch
            self.seg3_hdev = [L.host_device_pointer(h) if self.seg3_w < 8 else None
                              for h in self.seg3_host]

    def fill_segment(self, k, S):
        """Worker side of the pipelined replay loop: the next S steps' draws into pinned
        buffer k, once the copy out of it (three segments back) has finished."""
        self._seg_buffers(3)
        if self.seg3_used[k]:
            self.seg3_done[k].synchronize()
        fill = {1: self.rng.pairs_steps_u8, 2: self.rng.pairs_steps_u16,
                8: self.rng.pairs_steps}[self.seg3_w]
        fill(S, self.N, self.kx, self.kz, self.B, self.seg3_np[k])
        return k

    def ship_segment(self, k, S, rows=None, record=True):
        """Main side: the asynchronous H2D copy of buffer k (stream-ordered after the graph
        that read its device copy three segments back), widened on the device when narrowed;
        returns the int64 device buffer.  rows: SGDEngine.rows_ship_args of a reshuffle — its
        row tables go up in the same launch (tw_ship_draws; narrowed, mapped draws only)."""
        n = int(S) * 2 * self.N * self.B
        widen = "tw_widen_u8" if self.seg3_w == 1 else "tw_widen_u16"
        if rows is not None or (FUSED_SHIP and self.seg3_w < 8
                                and self.seg3_hdev[k] is not None):
            assert self.seg3_w < 8 and self.seg3_hdev[k] is not None
            src, nx, dx, nz, dz = rows if rows is not None else (None, 0, None, 0, None)
            L.call("tw_ship_draws", ctypes.c_void_p(self.seg3_hdev[k]), self.seg3_w, n,
                   L.ptr(self.seg3_dev[k]), ctypes.c_void_p(src), nx, dx, nz, dz,
                   L.stream_handle())
        elif self.seg3_w < 8 and self.seg3_hdev[k] is not None:
            L.call(widen, ctypes.c_void_p(self.seg3_hdev[k]), n, L.ptr(self.seg3_dev[k]),
                   L.stream_handle())
        elif self.seg3_w < 8:
            st = self.seg3_stage[k]
            st[:S].copy_(self.seg3_host[k][:S], non_blocking=True)
            L.call(widen, L.ptr(st), n, L.ptr(self.seg3_dev[k]), L.stream_handle())
        else:
            self.seg3_dev[k][:S].copy_(self.seg3_host[k][:S], non_blocking=True)
        if record:  # (record=False inside a graph capture: the caller records after the replay)
            self.shipped_out(k)
        return self.seg3_dev[k]

    def shipped_out(self, k):
        """The upload out of pinned buffer k is enqueued (on the current stream)."""
        self.seg3_done[k].record()
        self.seg3_used[k] = True

    def pairs(self):
        t = L.torch()
        k = self.k
        self.k ^= 1
        if self.done[k] is not None:
            self.done[k].synchronize()
        h = self.hnp[k]
        self.rng.pairs(self.N, self.kx, self.kz, self.B, h[0], h[1])
        self.last = h  # the host draws of this step (valid until the buffer's reuse)
        # stream-ordered: dev[k]'s previous reader (two steps back) precedes this copy
        self.dev[k].copy_(self.host[k], non_blocking=True)
        if self.done[k] is None:
            self.done[k] = t.cuda.Event()
        self.done[k].record()
        return self.dev[k][0], self.dev[k][1]


class _NativeDraws:
    """Handle of a running tw_draw_pipe (the pipelined replay loop's native draw worker)."""

    def __init__(self, draws, h, segs, N, kx, kz, keep):
        self.draws, self.h, self.segs = draws, h, segs
        self.N, self.kx, self.kz = N, kx, kz
        self._keep = keep  # the arrays the native side reads

    def wait(self, j, rows=True):
        """Block (interpreter lock released) until segment j is drawn: (rows, k) as the
        Python worker returns them — rows = ((rows_x, rows_z) views, (pinned, device
        address)) for a reshuffle, else None (always None with rows=False); k = the ring
        slot."""
        L.call("tw_draw_pipe_wait", self.h, j)
        k = j % 3
        if not rows or not self.segs[j][2]:
            return None, k
        buf = self.draws.rows3[k][0]
        flat = buf.numpy()
        N, kx = self.N, self.kx
        return ((flat[:N * kx].reshape(N, kx),
                 flat[N * kx:N * kx + N * self.kz].reshape(N, self.kz)),
                (buf, self.draws.rows3_hdev[k])), k

    def shipped(self, j):
        L.call("tw_draw_pipe_shipped", self.h, j, L.stream_handle())

    def stop(self):
        if self.h is not None:
            L.call("tw_draw_pipe_stop", self.h)
            self.h = None


def sign_audit_step(X, Z, rows_x, rows_z, ix, iz, w, margin, scores) -> dict:
    """One replay step's hinge-filter audit: the reference filters on
    S = diff.dot(w) + margin with BLAS's summation order (compute_stats.py:157-159), the device
    on its own order.  near_zero: pairs whose |S| is within the dot product's rounding bound
    d * eps * (sum |diff_j w_j| + |margin|), where the two orders may disagree; flips: pairs
    whose filter actually differs."""
    near = flips = 0
    w = np.asarray(w, dtype=np.float64).reshape(-1, 1)
    d = w.shape[0]
    for s in range(len(rows_x)):
        diff = Z[rows_z[s][iz[s]]] - X[rows_x[s][ix[s]]]
        S = (diff.dot(w) + margin).ravel()
        bound = d * np.finfo(np.float64).eps * (np.abs(diff * w.ravel()).sum(axis=1)
                                                + abs(margin))
        near += int(np.sum(np.abs(S) <= bound))
        flips += int(np.sum((S > 0) != (scores[s] > 0)))
    return {"pairs": int(len(rows_x) * ix.shape[1]), "near_zero": near, "flips": flips}


def learning_process(X, Z, p_learn, optim_type="momentum", *, trajectory=None,
                     rng_mode="replay", graphs=True, group=None, x_layout="replicated",
                     loss="hinge", gradient="incomplete", sign_audit=None, devices=None,
                     collectives=None):
    """Learning process for our experiments.  (make_exps.py:96-141)

    rng_mode="replay" (default): NumPy's own draws, bit-compatible with the reference; the
    steps between two reshuffles/evaluations are drawn in one native call and, with
    graphs=True, replayed as one hipGraph.
    rng_mode="device": SWR rows and pairs drawn on the device from a seed taken from the
    global RNG (one randint); statistically equivalent, and with graphs=True each run of
    steps between evaluations/reshuffles is one hipGraph replay.
    group: a torch.distributed group (one process per GPU); shards are spread over its ranks
    and the trajectory is identical to the single-GPU one.  Every rank must call with the
    same inputs and the same NumPy global RNG state.
    x_layout: "replicated" (X, Z whole on every GPU; a reshuffle moves no data) or
    "partitioned" (1/G of the rows per GPU; a reshuffle exchanges the drawn rows).
    loss: "hinge" (the reference) or "logistic" (SURVEY.md §8 row L3 extension: pairwise
    logistic loss softplus(diff . w + margin); evaluation reports its surrogate too).
    gradient: "incomplete" (the reference: B sampled pairs per shard) or "complete" (extension:
    all pairs of every shard via per-point pair coefficients + X^T c; draws no pairs).
    sign_audit: a list (replay mode, one process, replicated X) that receives, per step,
    sign_audit_step's counts of near-zero scores and of hinge-filter disagreements between the
    device's S and NumPy/BLAS's S; the steps then run one at a time.
    devices: a list of devices for ONE process to spread the shards over (MultiDeviceSGD:
    bit-identical trajectory); default None = TW_DEVICES / every visible device when a step
    gathers >= 1 GiB of rows (C5 at large B), else one device.
    collectives: with group, True runs the over-ranks step even on a world-size-1 group (the
    RCCL calls of the multi-GPU path on one GPU; same trajectory); None = only with G > 1."""
    n_X, n_Z = X.shape[0], Z.shape[0]
    N = p_learn["N"]
    B = p_learn["B"]
    learning_rate = p_learn["learning_rate"]
    margin = p_learn["margin"]
    w = p_learn["w_init"]

    to_log = ["{} : {}".format(k, v) for k, v in p_learn.items()
              if not k.startswith(("train_", "test_", "w"))]
    i = 0
    while i < len(to_log) / 4:
        logging.info("%s", " / ".join(to_log[(i * 4):(i * 4 + 4)]))
        i += 1
    logging.info("#X: %d / #Z: %d ", n_X, n_Z)
    logging.info("#X/N: %d / #Z/N: %d ", n_X / N, n_Z / N)
    logging.info("pairs_per_clust: %d ", (n_X / N) * (n_Z / N))
    logging.info("#eval_pairs_before_reshuffle: %d ", B * p_learn["reshuffle_mod"])

    devs = None if sign_audit is not None else _engine_devices(
        devices, N, B, int(np.asarray(w).size), group, x_layout, gradient)
    if devs is not None:
        eng = MultiDeviceSGD(X, Z, w, N, B, margin, p_learn["reg"], learning_rate,
                             optim_type, devs, loss=loss)
    else:
        eng = _engine_for(X, Z, w, N, B, margin, p_learn["reg"], learning_rate, optim_type,
                          group, x_layout, loss, gradient, rng_mode, sign_audit is None,
                          collectives)
    if rng_mode == "device":
        assert optim_type in ["SGD", "momentum"]
        return _learning_device(eng, X, Z, p_learn, trajectory, graphs, loss)
    if rng_mode != "replay":
        raise ValueError(f"rng_mode must be 'replay' or 'device', not {rng_mode!r}")
    draws = getattr(eng, "_draws", None)
    if draws is None or sign_audit is not None:
        draws = _ReplayDraws(N, eng.kx, eng.kz, B)
        if _ENGINE["eng"] is eng:
            eng._draws = draws  # kept with the engine: its buffers' addresses are in the graphs
    else:
        draws.rng.acquire()  # NumPy's global state as it is now
    audit_scores = None
    if sign_audit is not None:
        if eng.complete or not eng.solo or eng.layout != "replicated":
            raise ValueError("sign_audit needs the incomplete gradient on one process with "
                             "replicated X")
        audit_scores = L.empty((eng.N_loc, B), eng.t.float64)
        if trajectory is None:
            trajectory = []  # the audit runs the steps one at a time
        Xh, Zh = np.asarray(X, dtype=np.float64), np.asarray(Z, dtype=np.float64)
    defer = _deferred_evals(eng, graphs, trajectory)
    with draws.rng:  # the global RNG state lives natively until the loop ends
        rows_x, rows_z = draws.swr_rows(n_X, n_Z)  # the reference's redundant draw (:119)
        eng.set_shards(rows_x, rows_z)
        n_it, mod, eval_mod = p_learn["n_it"], p_learn["reshuffle_mod"], p_learn["eval_mod"]
        assert optim_type in ["SGD", "momentum"]
        if trajectory is None and not eng.complete and DRAW_AHEAD:
            _replay_pipelined(eng, draws, X, Z, p_learn, loss, graphs, defer, rows_x, rows_z)
            n_it = 0  # done
        i = 0
        while i < n_it:
            if i % mod == 0:
                rows_x, rows_z = draws.swr_rows(n_X, n_Z)
                eng.set_shards(rows_x, rows_z)
            assert optim_type in ["SGD", "momentum"]
            if trajectory is not None:  # one step at a time, recording w
                if i % eval_mod == 0:
                    _evaluate(i, eng, eng.w_host(), rows_x, rows_z, X, Z, p_learn, loss, graphs)
                trajectory.append(eng.w_host())
                if eng.complete:
                    eng.step_complete()
                else:
                    ix, iz = draws.pairs()
                    eng.step(ix, iz, scores=audit_scores)
                    if audit_scores is not None:
                        hx, hz = draws.last[0].copy(), draws.last[1].copy()
                        rec = sign_audit_step(Xh, Zh, rows_x, rows_z, hx, hz, trajectory[-1],
                                              margin, audit_scores.cpu().numpy())
                        rec["step"] = i
                        sign_audit.append(rec)
                i += 1
                continue
            # The steps up to the next reshuffle / evaluation draw nothing else from the RNG
            # (evaluation_step draws nothing either): draw them all at once, in the same
            # order, while the device still runs the previous segment, and replay them as one
            # graph.  At an evaluation, w leaves the device asynchronously before the draws.
            nxt = min(n_it, (i // eval_mod + 1) * eval_mod, (i // mod + 1) * mod,
                      i + draws.segment_capacity())
            w_pending = None
            if i % eval_mod == 0:
                if defer is not None:  # device part enqueued now, host part later
                    _evaluate(i, eng, None, rows_x, rows_z, X, Z, p_learn, loss, graphs, defer)
                else:
                    w_pending = eng.w_host_async()
            buf, tag = (None, 0) if eng.complete else draws.pairs_segment(nxt - i)
            if w_pending is not None:
                _evaluate(i, eng, w_pending(), rows_x, rows_z, X, Z, p_learn, loss, graphs)
            eng.run_replay_segment(buf, nxt - i, graphs, tag)
            i = nxt
    eng.check()  # before the deferred evaluations write their history
    if defer is not None:
        defer.drain()
    return None


def _replay_pipelined(eng, draws, X, Z, p_learn, loss, graphs, defer, rows_x, rows_z):
    """The replay loop's segments (runs of steps up to the next reshuffle / evaluation, at most
    segment_capacity() steps) with the host's NumPy-exact draws made AHEAD by a worker: the
    draws of later segments (their SWR rows, make_exps.py:123-125, then their steps' pairs,
    compute_stats.py:155-156 — the reference's order, one MT19937 stream) run while this thread
    uploads the row tables, evaluates and launches segment j.  NATIVE_DRAWS: a native thread
    (tw_draw_pipe, csrc/drawpipe.hip) filling a ring of three pinned buffers, each refilled once
    the upload out of it has run; else a Python worker thread two segments ahead (ctypes
    releases the GIL during the draws).  Same draws, same trajectory as the sequential loop
    (tests/test_gpu_learning*.py)."""
    n_X, n_Z = X.shape[0], Z.shape[0]
    n_it, mod, eval_mod = p_learn["n_it"], p_learn["reshuffle_mod"], p_learn["eval_mod"]
    draws._seg_buffers(3)
    through = (REPLAY_THROUGH and NATIVE_DRAWS and isinstance(eng, SGDEngine)
               and eng.replay_through_ok() and draws.seg3_w < 8
               and draws.seg3_hdev[0] is not None)
    segs, i = [], 0
    while i < n_it:
        # capacity, a growing head and a halving tail: the device starts only once the first
        # segment is drawn, and runs the last one after the host's last draw, unoverlapped —
        # 256-step segments there cost ~10 % of a 2000-step run at C4 (profiles/r04s3_*).  The
        # head grows by 1.25x a segment: the host draws a step in ~0.75 of the device's time
        # (C4, mod 25), so doubling left the device idle while the next segment was drawn
        # (profiles/r04s6_replay_timeline.log)
        cap = min(draws.segment_capacity(), int(16 * 1.25 ** min(len(segs), 24)),
                  max(8, -(-(n_it - i) // 2)))
        if through:
            # segments end at evaluations and at capacity only: the reshuffles inside one go
            # up with its draws and the kernel switches tables at their steps
            nxt = min(n_it, (i // eval_mod + 1) * eval_mod, i + cap)
            first = (mod - i % mod) % mod  # the segment's first reshuffle, from its start
            nxt = min(nxt, i + first + draws.table_capacity(n_X, n_Z) * mod)
            segs.append((i, nxt, (nxt - 1) // mod - (i - 1) // mod))
        else:
            nxt = min(n_it, (i // eval_mod + 1) * eval_mod, (i // mod + 1) * mod, i + cap)
            segs.append((i, nxt, int(i % mod == 0)))
        i = nxt

    def run(wait, shipped):
        _replay_segments(eng, draws, segs, wait, shipped, X, Z, p_learn, loss, graphs, defer,
                         rows_x, rows_z)

    if through:
        # the stacks and the pinned ring sized for the most tables a segment can hold, not this
        # run's: a later call at another reshuffle_mod must not re-allocate (pinned allocations
        # cost milliseconds inside the caller's loop)
        cap_tabs = min(draws.segment_capacity(), draws.table_capacity(n_X, n_Z))
        eng.table_stacks(max([cap_tabs] + [r for _, _, r in segs]))
        # the tables as uint16 where every row index fits: a quarter of the host stores and
        # of the upload, and the 64-word compaction of the draws (csrc/numpy_rng.cpp)
        rw = 2 if n_X <= 65536 and n_Z <= 65536 else 8
        pipe = draws.native_pipe(segs, n_X, n_Z, mod, row_width=rw, through=True)
        try:
            _replay_through(eng, draws, segs, pipe, mod, p_learn, loss, graphs, defer, X, Z)
        finally:
            pipe.stop()
        return
    if NATIVE_DRAWS:
        pipe = draws.native_pipe(segs, n_X, n_Z, mod)
        try:
            run(pipe.wait, pipe.shipped)
        finally:
            pipe.stop()
        return
    from concurrent.futures import ThreadPoolExecutor
    staged = isinstance(eng, SGDEngine) and eng.layout == "replicated"

    def work(idx):
        a, b, resh = segs[idx]
        rows = None
        if resh:
            rows = (draws.swr_rows_staged(idx % 3, n_X, n_Z) if staged
                    else (draws.swr_rows(n_X, n_Z), None))
        return rows, draws.fill_segment(idx % 3, b - a)

    ahead = 2
    draws._seg_buffers(3)  # on this thread: its current device and stream
    with ThreadPoolExecutor(max_workers=1) as pool:
        futs = [pool.submit(work, j) for j in range(min(ahead, len(segs)))]

        def wait(idx):
            r = futs[idx].result()
            if idx + ahead < len(segs):
                futs.append(pool.submit(work, idx + ahead))
            return r

        run(wait, None)


def _replay_segments(eng, draws, segs, wait, shipped, X, Z, p_learn, loss, graphs, defer,
                     rows_x, rows_z):
    """The main thread's side of _replay_pipelined: per segment, its draws (wait(j) -> (rows,
    ring slot)), a reshuffle's row tables, the upload, the evaluation, the steps."""
    eval_mod = p_learn["eval_mod"]
    for idx, (i, nxt, resh) in enumerate(segs):
        if PIPE_STATS is not None:  # study hook (tools/time_replay_parts.py)
            import time
            t0 = time.perf_counter()
            rows, k = wait(idx)
            PIPE_STATS.append(time.perf_counter() - t0)
        else:
            rows, k = wait(idx)
        rargs = None
        if rows is not None:
            (rows_x, rows_z), pinned = rows
            if TYPE_TRAIN_MONITOR == "SAME_AS_BATCH":
                # a host-formula evaluation (several ranks or devices: no batch_view) reads
                # these rows at this or a later segment, after shipped(idx) may have let the
                # draw worker refill their ring slot with a later reshuffle: own copies
                rows_x, rows_z = np.array(rows_x), np.array(rows_z)
            staged = pinned is not None and isinstance(eng, SGDEngine)
            if staged and FUSED_SHIP:
                rargs = eng.rows_ship_args(pinned)
            if rargs is not None:
                pass  # the row tables go up with the segment's draws, in one launch
            elif staged and eng.set_shards_staged(pinned):
                if shipped is None:
                    draws.rows_uploaded(k)
            else:
                eng.set_shards(rows_x, rows_z)
        evaluating = i % eval_mod == 0
        # the upload rides in the segment's graph when nothing enqueued between them reads
        # the new rows: no evaluation here, or FIXED_PAIRS monitoring (its statistics read w
        # and the fixed pairs only); otherwise it goes first — the reference reshuffles, then
        # evaluates (make_exps.py:123-128)
        upload = None
        if (graphs and FUSED_SHIP and isinstance(eng, SGDEngine) and eng.solo
                and (rows is None or rargs is not None)
                and draws.seg3_w < 8 and draws.seg3_hdev[k] is not None
                and (not evaluating or TYPE_TRAIN_MONITOR == "FIXED_PAIRS")):
            buf = draws.seg3_dev[k]
            upload = ((k, nxt - i, rargs is not None),
                      lambda k=k, S=nxt - i, r=rargs: draws.ship_segment(k, S, r, record=False))
        else:
            # (the native worker keeps its own event per ring slot: no torch event records)
            buf = draws.ship_segment(k, nxt - i, rargs, record=shipped is None)
            if shipped is None and rargs is not None:
                draws.rows_uploaded(k)
            if shipped is not None:
                shipped(idx)
        w_pending = None
        if evaluating:
            if defer is not None:  # device part enqueued now, host part later
                _evaluate(i, eng, None, rows_x, rows_z, X, Z, p_learn, loss, graphs, defer)
            else:
                w_pending = eng.w_host_async()
        if w_pending is not None:
            _evaluate(i, eng, w_pending(), rows_x, rows_z, X, Z, p_learn, loss, graphs)
        if upload is None:
            eng.run_replay_segment(buf, nxt - i, graphs, k)
        else:
            eng.run_replay_segment(buf, nxt - i, graphs, k, upload=upload)
            if shipped is None:
                draws.shipped_out(k)
                if rargs is not None:
                    draws.rows_uploaded(k)
            else:
                shipped(idx)


def _replay_through(eng, draws, segs, pipe, mod, p_learn, loss, graphs, defer, X, Z):
    """_replay_segments for segments running through their reshuffles (REPLAY_THROUGH; one
    process, replicated X, the persistent narrow segment): per segment, its draws and the row
    tables of every reshuffle inside it (drawn ahead in the reference's order by the native
    worker) go up in one launch into the engine's table stacks — slot 0 when the segment starts
    at a reshuffle, which the reference makes before it evaluates (make_exps.py:123-128), else
    slots 1.. — then the evaluation (SAME_AS_BATCH reads slot 0), then one persistent launch
    that switches tables at the reshuffle steps and leaves the last one in slot 0."""
    eval_mod = p_learn["eval_mod"]
    for idx, (i, nxt, ntab) in enumerate(segs):
        if PIPE_STATS is not None:  # study hook (tools/time_replay_parts.py)
            import time
            t0 = time.perf_counter()
            pipe.wait(idx, rows=False)
            PIPE_STATS.append(time.perf_counter() - t0)
        else:
            pipe.wait(idx, rows=False)
        # the table slots (0 at a segment that starts at a reshuffle, else 1..) and the copy of
        # the last table into slot 0 hold only while evaluations sit at segment starts, which
        # the segmentation guarantees: no evaluation step inside (i, nxt)
        assert (nxt - 1) // eval_mod == i // eval_mod, (i, nxt, eval_mod)
        k, phase = idx % 3, i % mod
        buf = draws.ship_tables(k, nxt - i, ntab, 0 if phase == 0 else 1, eng)
        pipe.shipped(idx)  # the only reader of the pinned buffers has been enqueued
        if i % eval_mod == 0:
            if defer is not None:  # device part enqueued now, host part later
                _evaluate(i, eng, None, None, None, X, Z, p_learn, loss, graphs, defer)
            else:
                _evaluate(i, eng, eng.w_host(), None, None, X, Z, p_learn, loss, graphs)
        eng.run_replay_segment(buf, nxt - i, graphs, k, tables=(phase, mod))


def _evaluate(i, eng, w, rows_x, rows_z, X, Z, p_learn, loss, graphs, defer=None):
    """evaluation_step at step i of the replay loop (make_exps.py:127-128); with defer, w is
    None (copied from the device with the statistics)."""
    X_s = Z_s = batch = None  # FIXED_PAIRS evaluation does not read the shards
    if TYPE_TRAIN_MONITOR == "SAME_AS_BATCH":
        batch = eng.batch_view()
        if batch is None:  # several ranks: the host formula on the global shards
            X_s = [X[r] for r in rows_x]
            Z_s = [Z[r] for r in rows_z]
    evaluation_step(i, X_s, Z_s, w, p_learn, loss=loss, _w_dev=eng.w, _graph=graphs,
                    _batch=batch, _defer=defer)


def _learning_device(eng, X, Z, p_learn, trajectory, graphs, loss="hinge"):
    if TYPE_TRAIN_MONITOR == "SAME_AS_BATCH" and (isinstance(eng, MultiDeviceSGD)
                                                   or getattr(eng, "G", 1) > 1):
        # the device-drawn shards exist only as per-slot / per-rank row tables
        raise ValueError("TYPE_TRAIN_MONITOR='SAME_AS_BATCH' with rng_mode='device' runs on "
                         "one device and one rank; use rng_mode='replay' (the host formula "
                         "over the global shards) for several")
    eng.enable_device_rng(int(np.random.randint(0, 2 ** 63 - 1, dtype=np.int64)))
    n_it, mod, eval_mod = p_learn["n_it"], p_learn["reshuffle_mod"], p_learn["eval_mod"]
    if trajectory is not None:
        graphs = False
    defer = _deferred_evals(eng, graphs, trajectory)
    # segments through their reshuffles (the kernel draws the rows) where nothing reads the
    # device row tables: FIXED_PAIRS monitoring, no per-step trajectory
    swr = (SWR_IN_KERNEL and trajectory is None and TYPE_TRAIN_MONITOR == "FIXED_PAIRS"
           and isinstance(eng, SGDEngine) and eng.swr_segments_ok())
    stale = False  # the device tables lag behind a swr segment's reshuffles
    i = 0
    while i < n_it:
        resh = i % mod == 0
        if swr:
            if i % eval_mod == 0:
                evaluation_step(i, None, None, None if defer is not None else eng.w_host(),
                                p_learn, loss=loss, _w_dev=eng.w, _graph=graphs, _defer=defer)
            nxt = min(n_it, (i // eval_mod + 1) * eval_mod)
            if eng.swr_segments_ok(nxt - i):
                eng.run_segment(nxt - i, False, graphs, swr_mod=mod)
                stale = True
            else:  # one step: the row tables, drawn at this step's last reshuffle
                if resh or stale:
                    eng.reshuffle_device(counter=None if resh else i - i % mod)
                    stale = False
                eng.run_segment(1, False, graphs)
            i = nxt
            continue
        if i % eval_mod == 0:
            batch = None
            if TYPE_TRAIN_MONITOR == "SAME_AS_BATCH":
                # the reference reshuffles before it evaluates (make_exps.py:123-128)
                if resh:
                    eng.reshuffle_device()
                    resh = False
                batch = eng.batch_view()
            evaluation_step(i, None, None, None if defer is not None else eng.w_host(),
                            p_learn, loss=loss, _w_dev=eng.w, _graph=graphs, _batch=batch,
                            _defer=defer)
        if trajectory is not None:  # one step at a time, recording w
            if resh:
                eng.reshuffle_device()
            trajectory.append(eng.w_host())
            eng.step_device()
            i += 1
            continue
        nxt = min(n_it, (i // eval_mod + 1) * eval_mod, (i // mod + 1) * mod)
        eng.run_segment(nxt - i, resh, graphs)
        i = nxt
    eng.check()  # before the deferred evaluations write their history
    if defer is not None:
        defer.drain()
    return None


class _DeferredEvals:
    """Evaluations of the learning loop whose device part (one graph replay) is enqueued in
    stream order and whose host part — the statistics' formulas, the log line, p_learn's lists
    (make_exps.py:162-190) — runs once their results have reached pinned host memory, in order
    (and all of them before learning_process returns).  The loop no longer waits for the device
    at every evaluation; the values are the same bits."""

    def __init__(self, w_dev, w_shape, slots=64, check=None, ctl=None):
        t = L.torch()
        self.t = t
        self.w_shape = w_shape
        # the engine's abort word (ctl, a 1-element device tensor), copied beside each
        # evaluation's results and checked before its history is written; without it, the
        # engine's blocking check() runs instead
        self.check = check
        self.ctl = ctl
        # slot k: [4 statistics | w | abort word], written by ONE tw_stage_eval launch
        self.nw = int(w_dev.numel())
        self.host = t.zeros((slots, 4 + self.nw + 1), dtype=t.float64, pin_memory=True)
        self.host_dev = L.host_device_pointer(self.host)  # the kernel's address of slot 0
        if self.host_dev is None:
            raise RuntimeError("deferred evaluations: pinned host slots are not device-mapped")
        self.events = [t.cuda.Event() for _ in range(slots)]
        self.free = list(range(slots))[::-1]
        self.pending = []

    def push(self, i, res_dev, w_dev, finish):
        if not self.free:
            self._pop()
        k = self.free.pop()
        res = res_dev.reshape(-1)
        assert res.dtype == self.t.float64 and res.numel() == 4 and res.is_contiguous()
        assert w_dev.dtype == self.t.float64 and w_dev.numel() == self.nw and w_dev.is_contiguous()
        L.call("tw_stage_eval", L.ptr(res), 4, L.ptr(w_dev), self.nw,
               L.ptr(self.ctl),
               ctypes.c_void_p(self.host_dev + k * 8 * (4 + self.nw + 1)), L.stream_handle())
        self.events[k].record()
        self.pending.append((i, k, finish))
        while len(self.pending) > 1 and self.events[self.pending[0][1]].query():
            self._pop()

    def _pop(self):
        i, k, finish = self.pending.pop(0)
        self.events[k].synchronize()
        # a persistent segment that gave up at its grid barrier left w invalid: raise before
        # its statistics reach p_learn or the log (the word is sticky, so the copy taken with
        # this evaluation covers every segment before it, without a device-wide wait here)
        if self.ctl is not None:
            if int(self.host[k, 4 + self.nw:].numpy().view(np.int64)[0]) != 0:
                raise RuntimeError("tw_sgd_segment_narrow: a grid barrier timed out (blocks not "
                                   "co-resident); the SGD state is invalid")
        elif self.check is not None:
            self.check()
        h = self.host[k].numpy()
        finish(i, h[:4].copy(), h[4:4 + self.nw].copy().reshape(self.w_shape))
        self.free.append(k)

    def drain(self):
        while self.pending:
            self._pop()


def _deferred_evals(eng, graphs, trajectory):
    """A _DeferredEvals for the loop when its evaluations can be deferred: hipGraphs on, FIXED_PAIRS
    monitoring (SAME_AS_BATCH reduces on the host), one process, no trajectory recording."""
    if (not DEFER_EVALS or not graphs or trajectory is not None
            or TYPE_TRAIN_MONITOR != "FIXED_PAIRS" or getattr(eng, "G", 1) != 1):
        return None
    ctl = getattr(eng, "_ctl", None)
    return _DeferredEvals(eng.w, eng.w_shape, check=eng.check,
                          ctl=ctl[1:2] if ctl is not None else None)


class _EvalCache:
    """Device copies of p_learn's evaluation matrices and monitor pairs, reused across calls
    while p_learn holds the same objects."""

    def __init__(self):
        self.src = {}
        self.dev = {}

    def get(self, key, obj, make):
        if self.src.get(key) is not obj:
            self.src[key] = obj
            self.dev[key] = make(obj)
        return self.dev[key]


_CACHE = _EvalCache()


def _pairs_dev(pairs):
    """The monitor pairs as device index columns: int32 when they fit (8 B per pair), which
    lets evaluation read them once for both statistics (tw_pair_sum_idx32_f64 with a count)."""
    a = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
    off = np.array([0, a.shape[0]], dtype=np.int64)
    fits = a.size == 0 or (int(a.min()) >= -2 ** 31 and int(a.max()) < 2 ** 31)
    dt = np.int32 if fits else np.int64
    return (L.to_device(np.ascontiguousarray(a[:, 0]), dt),
            L.to_device(np.ascontiguousarray(a[:, 1]), dt), off, L.to_device(off))


def _pairs_range(pairs):
    """(min x, max x, min z, max z) of the monitor pairs ((0, -1, 0, -1) when empty)."""
    a = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
    if a.size == 0:
        return 0, -1, 0, -1
    return int(a[:, 0].min()), int(a[:, 0].max()), int(a[:, 1].min()), int(a[:, 1].max())


def _scores(A_dev, wd):
    """A @ w on the device (tw_gemv_f64); wd: w as a (d,) float64 device tensor."""
    t = L.torch()
    out = L.empty((A_dev.shape[0],), t.float64)
    L.call("tw_gemv_f64", L.ptr(A_dev), A_dev.shape[0], A_dev.shape[1], L.ptr(wd), L.ptr(out),
           L.stream_handle())
    return out


def _eval_sources(p_learn, fixed):
    """The p_learn objects the device evaluation reads (a cached graph is valid while
    p_learn still holds these very objects)."""
    keys = ("test_X", "test_Z") + (("train_X", "train_Z", "train_mon_pairs") if fixed else ())
    return tuple(p_learn[k] for k in keys)


_OFFSETS = {}


def _offsets(n, m):
    """Host and device offsets of one (n, m) shard, uploaded once."""
    if (n, m) not in _OFFSETS:
        xo, zo = np.array([0, n], np.int64), np.array([0, m], np.int64)
        _OFFSETS[(n, m)] = (xo, zo, L.to_device(xo), L.to_device(zo))
    return _OFFSETS[(n, m)]


def _eval_device(wd, p_learn, loss, margin, fixed):
    """Every device statistic of evaluation_step, enqueued only (graph-capturable: no host
    copies, no syncs).  Returns (float64 device tensor [monitor surrogate sum, monitor count
    bits, test surrogate sum, test count bits], #monitor pairs, #test pairs)."""
    t = L.torch()
    kern = cs._loss_codes(loss)[0]
    if fixed:  # the monitor pairs index the training scores (make_exps.py:162-168)
        lo_x, hi_x, lo_z, hi_z = _CACHE.get("pairs_range", p_learn["train_mon_pairs"],
                                            _pairs_range)
        nx, nz = len(p_learn["train_X"]), len(p_learn["train_Z"])
        if lo_x < 0 or lo_z < 0 or hi_x >= nx or hi_z >= nz:
            raise IndexError(f"train_mon_pairs index out of range for {nx} x {nz} rows "
                             f"(x in [{lo_x}, {hi_x}], z in [{lo_z}, {hi_z}])")
    small = _eval_small(wd, p_learn, kern, margin) if fixed and EVAL_FUSED else None
    if small is not None:
        return small
    parts = []
    n_pairs = 0
    if fixed:
        tX = _CACHE.get("train_X", p_learn["train_X"], _dev_f64)  # NumPy or device arrays
        tZ = _CACHE.get("train_Z", p_learn["train_Z"], _dev_f64)
        # the monitor pairs live on the device for as long as p_learn holds the same list
        ixd, izd, off, offd = _CACHE.get("pairs", p_learn["train_mon_pairs"], _pairs_dev)
        n_pairs = int(off[1])
        sx, sz = _scores(tX, wd), _scores(tZ, wd)
        if ixd.dtype == t.int32:  # one pass over the pairs: hinge sum and AUC count
            cnt = L.empty((1,), t.int64)
            parts += [E.pair_sum_indexed_dev(sx, sz, ixd, izd, off, kern, float(margin),
                                             pair_off_dev=offd, count_out=cnt),
                      cnt.view(t.float64)]
        else:
            parts += [E.pair_sum_indexed_dev(sx, sz, ixd, izd, off, kern, float(margin),
                                             pair_off_dev=offd),
                      E.count_indexed_dev(sx, sz, L.TW_F64, ixd, izd, off, L.TW_PRED_GT,
                                          pair_off_dev=offd).view(t.float64)]
    else:
        parts.append(t.zeros((2,), dtype=t.float64, device=wd.device))
    eX = _CACHE.get("test_X", p_learn["test_X"], _dev_f64)
    eZ = _CACHE.get("test_Z", p_learn["test_Z"], _dev_f64)
    sxt, szt = _scores(eX, wd), _scores(eZ, wd)
    n, m = sxt.shape[0], szt.shape[0]
    xo, zo, xod, zod = _offsets(n, m)
    sh = E.Shards(sxt, xo, szt, zo, L.TW_F64)
    sh._x_off_dev, sh._z_off_dev = xod, zod
    parts += [E.pair_sum_complete_dev(sh, kern, margin),
              E.count_launch(sxt, xod, szt, zod, 1, n, m, L.TW_F64, L.TW_PRED_GT,
                             E.pick_algo("auto", n, m, "gt")).view(t.float64)]
    return t.cat([v.reshape(-1) for v in parts]), n_pairs, n * m


def _eval_small(wd, p_learn, kern, margin):
    """_eval_device's FIXED_PAIRS statistics in two launches (tw_eval_small) when the problem
    is small enough for the all-pairs test statistics (the paths _eval_device would take
    anyway) and the monitor pairs are int32: the same values, or None."""
    t = L.torch()
    if kern not in (L.TW_KERN_HINGE, L.TW_KERN_LOGISTIC):
        return None
    tX = _CACHE.get("train_X", p_learn["train_X"], _dev_f64)
    tZ = _CACHE.get("train_Z", p_learn["train_Z"], _dev_f64)
    eX = _CACHE.get("test_X", p_learn["test_X"], _dev_f64)
    eZ = _CACHE.get("test_Z", p_learn["test_Z"], _dev_f64)
    ixd, izd, off, offd = _CACHE.get("pairs", p_learn["train_mon_pairs"], _pairs_dev)
    mats = (tX, tZ, eX, eZ)
    if any(a.dim() != 2 or a.shape[1] != wd.numel() or a.shape[0] == 0 for a in mats):
        return None
    n, m, n_pairs = eX.shape[0], eZ.shape[0], int(off[1])
    if (ixd.dtype != t.int32 or wd.numel() > 32 or n_pairs == 0 or len(off) != 2
            or n * m >= E.HINGE_SORTED_MIN_PAIRS
            or E.pick_algo("auto", n, m, "gt") != "pairs"):
        return None
    key = ("eval_small",) + tuple(a.shape[0] for a in mats) + (n_pairs, wd.numel())
    bufs = _CACHE.dev.get(key)
    if bufs is None:  # made outside any capture (evaluation_step warms before capturing)
        nw = int(L.lib().tw_eval_small_work(n_pairs, n, m))
        rows = sum(a.shape[0] for a in mats)
        bufs = (L.empty((rows,), t.float64), L.empty((nw,), t.float64),
                L.empty((nw,), t.int64), t.zeros((1,), dtype=t.int32, device=wd.device),
                L.to_device(np.array([0, n_pairs, 0, n, 0, m], dtype=np.int64)))
        _CACHE.dev[key] = bufs
    scores, work, cwork, ticket, offs = bufs
    out = L.empty((4,), t.float64)
    L.call("tw_eval_small", L.ptr(tX), tX.shape[0], L.ptr(tZ), tZ.shape[0], L.ptr(eX), n,
           L.ptr(eZ), m, wd.numel(), L.ptr(wd), L.ptr(ixd), L.ptr(izd), n_pairs, L.ptr(offs),
           kern, float(margin), L.ptr(scores), L.ptr(work), L.ptr(cwork), L.ptr(ticket),
           L.ptr(out), L.stream_handle())
    _eval_small.last = out.data_ptr()  # evaluation_step: this output came from the fused path
    return out, n_pairs, n * m


def _same_as_batch_device(batch, wd, margin, loss):
    """evaluation_step's SAME_AS_BATCH statistics (make_exps.py:154-160) on the device: the
    scores of the current shards (one GEMV per sample over the resident rows, gathered through
    the shard row tables), every shard's complete surrogate sum and AUC count in one launch
    each, and the reference's UN_split averages (np.mean over shards of the per-shard means)
    on the host.  batch = (X, Z, rows_x | None, rows_z | None, N, kx, kz) on the device."""
    t = L.torch()
    Xd, Zd, rx, rz, N, kx, kz = batch
    sx, sz = _scores(Xd, wd), _scores(Zd, wd)
    if rx is not None:
        sx = sx.index_select(0, rx.reshape(-1))
        sz = sz.index_select(0, rz.reshape(-1))
    xo, zo, xod, zod = _shard_offsets(N, kx, kz)
    sh = E.Shards(sx, xo, sz, zo, L.TW_F64)
    sh._x_off_dev, sh._z_off_dev = xod, zod
    kern = cs._loss_codes(loss)[0]
    sums = E.pair_sum_complete_dev(sh, kern, float(margin))
    cnt = E.count_launch(sx, xod, sz, zod, N, kx, kz, L.TW_F64, L.TW_PRED_GT,
                         E.pick_algo("auto", kx, kz, "gt"))
    res = t.cat([sums, cnt.view(t.float64)]).cpu().numpy()
    pairs = kx * kz
    bc = np.mean([np.float64(v / np.float64(pairs)) for v in res[:N]], axis=0)
    br = np.mean([E.ratio(c, pairs) for c in res[N:].view(np.uint64)], axis=0)
    return bc, br


def _shard_offsets(N, kx, kz):
    key = ("shards", N, kx, kz)
    if key not in _OFFSETS:
        xo = np.arange(N + 1, dtype=np.int64) * kx
        zo = np.arange(N + 1, dtype=np.int64) * kz
        _OFFSETS[key] = (xo, zo, L.to_device(xo), L.to_device(zo))
    return _OFFSETS[key]


def evaluation_step(i, X_s, Z_s, w, p_learn, *, loss="hinge", _w_dev=None, _graph=True,
                    _batch=None, _defer=None):
    """
        Modify the value of p_learn to add to the evaluation.  (make_exps.py:143-190)
        Monitored values, added in p_learn:
        * br_AUC: block real AUC, on the training data,
        * bc_AUC: block convexified AUC, on the training data,
        * tr_AUC: real AUC, on the testing data,
        * tc_AUC: convexified AUC, on the testing data,
    """
    margin = p_learn["margin"]
    logging.debug("Step %d: Begin evaluation", i)
    fixed = TYPE_TRAIN_MONITOR == "FIXED_PAIRS"
    deferred = _defer is not None and fixed and _w_dev is not None and _graph
    t = L.torch()
    bc = br_AUC = None  # SAME_AS_BATCH: the shards' surrogate (without the reg term) and AUC
    if TYPE_TRAIN_MONITOR == "SAME_AS_BATCH":
        if _batch is not None:  # the learning loop's shards, resident on the device
            wd = _w_dev if _w_dev is not None else L.to_device(
                np.asarray(w, np.float64).reshape(-1))
            bc, br_AUC = _same_as_batch_device(_batch, wd, margin, loss)
        else:
            sc_X = [x.dot(w) for x in X_s]
            sc_Z = [z.dot(w) for z in Z_s]
            bc = cs.UN_split(sc_X, sc_Z, cs.conv_AUC(margin, loss=loss))
            br_AUC = cs.UN_split(sc_X, sc_Z, lambda x, z: cs.Un(x, z, kernel="AUC"))
    if _w_dev is not None and _graph:  # the learning loop: w resident, device work one graph
        # one cached graph: valid while p_learn holds the same objects; w reaches it through
        # a persistent buffer, so later runs (new engines, new w) replay it too
        key = (fixed, loss, float(margin), int(_w_dev.numel()))
        srcs = _eval_sources(p_learn, fixed)
        ent = _CACHE.dev.get("eval_graph")
        if (ent is None or ent[0] != key or len(ent[1]) != len(srcs)
                or any(a is not b for a, b in zip(ent[1], srcs))):
            _CACHE.dev["eval_graph"] = None  # release the previous graph's pool first
            g = t.cuda.CUDAGraph()
            wbuf = t.empty_like(_w_dev)
            wbuf.copy_(_w_dev)
            _eval_device(wbuf, p_learn, loss, margin, fixed)  # warm: caches, allocations
            t.cuda.synchronize()
            _eval_small.last = None
            with L.capture(g):
                out = _eval_device(wbuf, p_learn, loss, margin, fixed)
            # only the fused small evaluation (two short launches) runs beside a persistent
            # segment: a larger one could hold CUs long enough for the segment's co-resident
            # grid barrier to give up
            small = out[0].data_ptr() == getattr(_eval_small, "last", None)
            # the entry keeps the device copies the graph reads alive, even if a later call
            # with other p_learn objects replaces them in _CACHE
            held = tuple(_CACHE.dev[k] for k in ("test_X", "test_Z") +
                         (("train_X", "train_Z", "pairs") if fixed else ()))
            ent = (key, srcs, g, out, held, wbuf, small)
            _CACHE.dev["eval_graph"] = ent
        res_dev, n_pairs, n_test = ent[3]
        if deferred and not ent[6]:  # serialised with the steps on the loop's stream
            side = _CACHE.dev.get("eval_side")
            if side is not None:
                t.cuda.current_stream().wait_stream(side)
            ent[5].copy_(_w_dev)
            ent[2].replay()
            _defer.push(i, res_dev, ent[5], lambda it, res, wh: _eval_host(
                it, res, wh, n_pairs, n_test, p_learn, fixed, None, None))
            return
        if deferred:
            # the evaluation runs on a side stream BESIDE the next segment of steps: w is
            # snapshotted into the graph's buffer on the loop's stream (after the previous
            # evaluation has read it), the graph and the staging of its results follow on the
            # side stream; the persistent segment holds N CUs, the evaluation's blocks take the
            # others.  The statistics and the snapshot leave the device as before (same bits).
            main = t.cuda.current_stream()
            side = _CACHE.dev.get("eval_side")
            if side is None:
                side = _CACHE.dev["eval_side"] = t.cuda.Stream()
            main.wait_stream(side)
            wbuf = ent[5]
            if (_w_dev.dtype == t.float64 and _w_dev.is_contiguous()
                    and wbuf.is_contiguous()):
                L.call("tw_copy_words", L.ptr(_w_dev), int(_w_dev.numel()), L.ptr(wbuf),
                       L.stream_handle())
            else:
                wbuf.copy_(_w_dev)
            side.wait_stream(main)
            with t.cuda.stream(side):
                ent[2].replay()
                _defer.push(i, res_dev, wbuf, lambda it, res, wh: _eval_host(
                    it, res, wh, n_pairs, n_test, p_learn, fixed, None, None))
            return
        side = _CACHE.dev.get("eval_side")
        if side is not None:  # a deferred evaluation may still read the graph's buffers
            t.cuda.current_stream().wait_stream(side)
        ent[5].copy_(_w_dev)
        ent[2].replay()
    else:
        wd = _w_dev if _w_dev is not None else L.to_device(np.asarray(w, np.float64).reshape(-1))
        res_dev, n_pairs, n_test = _eval_device(wd, p_learn, loss, margin, fixed)
    res = res_dev.cpu().numpy()  # the ONE copy back: [hinge sum, count] x (pairs, test)
    _eval_host(i, res, w, n_pairs, n_test, p_learn, fixed, bc, br_AUC)


def _eval_host(i, res, w, n_pairs, n_test, p_learn, fixed, bc, br_AUC):
    """evaluation_step's host part from the copied statistics res = [monitor surrogate sum,
    monitor count bits, test surrogate sum, test count bits] (make_exps.py:162-190); bc, br_AUC:
    the SAME_AS_BATCH monitor statistics (None with FIXED_PAIRS)."""
    reg_term = p_learn["reg"] * (np.linalg.norm(w) ** 2) / 2
    if fixed:
        bc_AUC = np.float64(res[0] / np.float64(n_pairs)) + reg_term
        br_AUC = E.ratio(int(res[1:2].view(np.uint64)[0]), n_pairs)
    else:
        bc_AUC = bc + reg_term
    tc_AUC = np.float64(res[2] / np.float64(n_test)) + reg_term
    tr_AUC = E.ratio(int(res[3:4].view(np.uint64)[0]), n_test)

    s_log = ("it %5d: bc_AUC = %.4f | br_AUC = %.4f "
             + "| tc_AUC = %5.4f | tr_AUC = %5.4f")
    logging.info(s_log, i, bc_AUC, br_AUC, tc_AUC, tr_AUC)

    elems = [("iter", i), ("norm_w", np.linalg.norm(w)),
             ("bc_AUC", bc_AUC), ("br_AUC", br_AUC),
             ("tr_AUC", tr_AUC), ("tc_AUC", tc_AUC)]
    for k, v in elems:
        if k in p_learn:
            p_learn[k].append(v)
        else:
            p_learn[k] = [v]
    logging.debug("Step %d: End evaluation", i)


# convenience re-export for drivers that import SWR_divide / UN_split from here
SWR_divide = cs.SWR_divide
ShardList = _learn.ShardList


# ------------------------------------------------------------------ driver I/O (make_exps.py)
def load_preprocess_data(data=None):
    """Loads and preprocesses the data.  (make_exps.py:51-93)

    data: a dict with "X" (n, d) and "y" (n,) in {-1, +1} (the shuttle pickle's content);
    None reads "shuttle.pickle" from the working directory like the reference (the user's own
    file, produced by convert_data_to_pickle).  Reproduces the reference exactly, including
    its train split `X_tot[~ind_X_test]`: `~` on an int index array is -(i+1), so "train" is
    a same-size sample taken from the other end, not the complement of the test indices."""
    if data is None:
        import pickle
        with open("shuttle.pickle", "rb") as fh:
            data = pickle.load(fh)
    X = data["X"]
    y = data["y"]
    # label +1 (the rare class) is the Z sample, -1 the X sample
    Z_tot, X_tot = X[y == +1], X[y == -1]

    np.random.seed(SEED_SHUFFLE)
    ind_X_test = np.random.choice(X_tot.shape[0], size=int(PROP_TEST * X_tot.shape[0]),
                                  replace=False)
    ind_Z_test = np.random.choice(Z_tot.shape[0], size=int(PROP_TEST * Z_tot.shape[0]),
                                  replace=False)
    np.random.seed()
    Z_train, X_train = Z_tot[~ind_Z_test], X_tot[~ind_X_test]
    Z_test, X_test = Z_tot[ind_Z_test], X_tot[ind_X_test]
    train_tot = np.vstack([X_train, Z_train])

    train_mean = train_tot.mean(axis=0)
    train_std = train_tot.std(axis=0)
    if np.min(train_std) == 0:
        raise ValueError("One of the columns in the data has constant var.")

    X_train = (X_train - train_mean) / train_std
    Z_train = (Z_train - train_mean) / train_std
    X_test = (X_test - train_mean) / train_std
    Z_test = (Z_test - train_mean) / train_std

    def add_constant(a):
        return np.hstack([a, np.ones((a.shape[0], 1))])

    return (add_constant(Z_train), add_constant(X_train), add_constant(Z_test),
            add_constant(X_test))


def make_exps(reshuffle_mod, out_folder="exps/test", p_learn=None, data=None,
              rng_mode="replay"):
    """Make the experiments for the desired parameters.  (make_exps.py:192-243, without the
    plots): writes <out_folder>/learning_process.log and <out_folder>/dynamics.json with the
    reference's schema (scalar parameters + the iter/norm_w/bc_AUC/br_AUC/tr_AUC/tc_AUC
    lists).  Returns p_learn."""
    import json
    import os
    import shutil
    if not os.path.exists(out_folder):
        os.makedirs(out_folder)
        shutil.copy(__file__, "{}/executed_script.py".format(out_folder))

    Z_train, X_train, Z_test, X_test = load_preprocess_data(data)
    n_feats = Z_train.shape[1]

    logging.basicConfig(filename='{}/learning_process.log'.format(out_folder),
                        format='%(asctime)s - %(message)s',
                        level=logging.INFO, datefmt='%m/%d/%y %I:%M:%S %p', filemode="w")

    if p_learn is None:
        p_learn = {"n_it": DEFAULT_ITE_NUMBER, "margin": 1, "N": 100,
                   "B": 100, "reshuffle_mod": reshuffle_mod, "reg": 0.05,
                   "learning_rate": 0.01, "eval_mod": 25,
                   "w_init": np.random.normal(0, 1, (n_feats, 1)),
                   "test_X": X_test, "test_Z": Z_test}

    if TYPE_TRAIN_MONITOR == "FIXED_PAIRS":
        np.random.seed(SEED_TRAIN_MONITOR)
        p_learn["train_mon_pairs"] = list(zip(
            list(np.random.randint(0, X_train.shape[0], SIZE_TRAIN_MONITOR)),
            list(np.random.randint(0, Z_train.shape[0], SIZE_TRAIN_MONITOR))))
        p_learn["train_X"] = X_train
        p_learn["train_Z"] = Z_train
        np.random.seed()

    print("Started optimization")
    learning_process(X_train, Z_train, p_learn, rng_mode=rng_mode)
    print("Finished optimization")

    for x in [k for k in p_learn if k.startswith(("train_", "test_", "w_"))]:
        p_learn.pop(x)
    with open("{}/dynamics.json".format(out_folder), "wt") as fh:
        json.dump(p_learn, fh)
    return p_learn
