"""Fused MNIST MLP trainer -- the bundled reference workload, built MI355X-first.

Model = the reference's demo job (`mnist_with_summaries`: 784-500-10, ReLU, dropout keep 0.9,
softmax cross-entropy, Adam lr 1e-3, batch 100; `docs/userguide/1-tfjob-standalone.md:178-186`),
and `dist-mnist`'s 784-100-10 variant via ``hidden=100``.

Execution design:
  * ALL parameters live in ONE flat fp32 buffer (Adam m/v and the gradient bucket mirror it), so
    the data-parallel gradient all-reduce is a single RCCL call on a contiguous buffer and Adam is a
    single launch -- no flatten/unflatten copies, no per-tensor launches.
  * The training set lives in HBM as uint8; the batch gather (permutation + device step counter)
    and the /255 dequantisation are fused into the first GEMM and the loss head.
  * One step = 2 launches on one GPU: mlp_fwd_logits (hidden layer + per-tile partial logits,
    atomically accumulated) -> wgrad_grouped (every workgroup recomputes the 100x10 softmax-xent,
    derives dz in LDS, computes both layers' dW and applies Adam in its epilogue). No kernel
    waits on another workgroup. With data parallelism: fwd -> wgrad (grad bucket) -> all_reduce
    -> adam_flat.
  * Every per-step scalar (data cursor, Adam t, dropout step, metric slot) is a device counter, so
    ``steps_per_graph`` consecutive steps are captured into ONE hipGraph and replayed.
Step-counter protocol (no intra-kernel races): A = completed steps, B = current Adam t.
  mlp_fwd_logits reads A and writes B=A+1; wgrad reads B (cursor = B-1);
  the last kernel of the step (wgrad with fused Adam, or adam_flat) writes A=B.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

from .. import ops
from ..runtime import heartbeat


@dataclass
class MLPConfig:
    in_dim: int = 784
    hidden: int = 500
    classes: int = 10
    keep_prob: float = 0.9
    batch: int = 100            # per-rank batch
    lr: float = 1e-3
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    tf_adam: bool = False       # TF AdamOptimizer epsilon placement
    seed: int = 0
    init: str = "tf"            # "tf": truncated normal(0.1), bias 0.1 (mnist_with_summaries)
    hist_len: int = 4096


def _pad4(n: int) -> int:
    return (n + 3) // 4 * 4


@dataclass
class FlatLayout:
    shapes: dict
    offsets: dict = field(default_factory=dict)
    total: int = 0

    def __post_init__(self):
        off = 0
        for name, shp in self.shapes.items():
            self.offsets[name] = off
            off += _pad4(math.prod(shp))
        self.total = off

    def view(self, flat: torch.Tensor, name: str) -> torch.Tensor:
        shp = self.shapes[name]
        o = self.offsets[name]
        return flat[o:o + math.prod(shp)].view(shp)


class FusedMLPTrainer:
    """Single-hidden-layer MLP trained entirely by the native HIP kernels (or the CPU reference)."""

    def __init__(self, cfg: MLPConfig, train_x: torch.Tensor, train_y: torch.Tensor,
                 device: torch.device | str = "cuda", process_group=None,
                 rank: int = 0, world: int = 1, external_update: bool = False,
                 comm: str = "auto"):
        """``external_update``: steps only produce the flat gradient ``G`` (the optimizer runs
        elsewhere -- the parameter server in PS mode); the step counter still advances.
        ``comm`` (data parallel on GPUs): "xgmi" = fused reduce-scatter/Adam/all-gather kernel over
        xGMI peer memory, "rccl" = graph-captured RCCL all_reduce + flat Adam, "auto" = xgmi when
        its self-test passes on every rank of a single-node job, else rccl."""
        self.cfg = cfg
        self.external_update = external_update
        self.device = torch.device(device)
        self.pg = process_group
        self.rank, self.world = rank, world
        self.distributed = world > 1
        dev = self.device
        D, H, C = cfg.in_dim, cfg.hidden, cfg.classes
        if D % 4 or H % 4:
            raise ValueError("in_dim and hidden must be multiples of 4 (vectorised MFMA operands)")
        self.layout = FlatLayout({"W1": (H, D), "b1": (H,), "W2": (C, H), "b2": (C,)})  # [out, in]
        n = self.layout.total
        self.P = torch.zeros(n, device=dev)
        self.M = torch.zeros(n, device=dev)
        self.V = torch.zeros(n, device=dev)
        self.G = torch.zeros(n, device=dev) if (self.distributed or external_update) else None
        self._init_params()
        import os as _os
        self._x_from_dataset = _os.environ.get("ARENA_WGRAD_X", "published") == "dataset"
        # forward row gather: "counter" (cursor -> permutation in the forward) or "rows" (the
        # backward precomputes the next step's rows); measured equal-or-slower, so off by default
        self._rows_ahead = _os.environ.get("ARENA_FWD_ROWS", "counter") == "rows"
        self.xgmi = None
        if self.distributed:
            import torch.distributed as dist
            if dev.type == "cuda" and comm in ("auto", "xgmi"):
                self._setup_xgmi(n, required=(comm == "xgmi"))
            if self.xgmi is not None:
                # rank 0's initial parameters, pulled over xGMI straight into every rank's
                # registered parameter buffer
                self.xgmi.broadcast_(self.P, 0)
            else:
                dist.broadcast(self.P, src=0, group=self.pg)
        self.comm = "xgmi" if self.xgmi is not None else ("rccl" if self.distributed else "none")
        L = self.layout
        self.W1, self.b1 = L.view(self.P, "W1"), L.view(self.P, "b1")
        self.W2, self.b2 = L.view(self.P, "W2"), L.view(self.P, "b2")
        self.mW1, self.mb1 = L.view(self.M, "W1"), L.view(self.M, "b1")
        self.mW2, self.mb2 = L.view(self.M, "W2"), L.view(self.M, "b2")
        self.vW1, self.vb1 = L.view(self.V, "W1"), L.view(self.V, "b1")
        self.vW2, self.vb2 = L.view(self.V, "W2"), L.view(self.V, "b2")
        if self.G is not None:
            self.gW1, self.gb1 = L.view(self.G, "W1"), L.view(self.G, "b1")
            self.gW2, self.gb2 = L.view(self.G, "W2"), L.view(self.G, "b2")
        B = cfg.batch
        self.Hbuf = torch.empty(B, H, device=dev)
        self.dlogits = torch.empty(B, C, device=dev)
        self.W2snap = torch.empty(C, H, device=dev)
        self.logits2 = torch.zeros(2, B, C, device=dev)  # step-parity double buffer
        self.xb = torch.zeros(B, D, dtype=torch.uint8, device=dev)  # this step's gathered batch
        self.yb = torch.zeros(B, dtype=torch.int32, device=dev)
        self.ctrA = torch.zeros(1, dtype=torch.int64, device=dev)
        self.ctrB = torch.zeros(1, dtype=torch.int64, device=dev)
        self.loss_hist = torch.zeros(cfg.hist_len, device=dev)
        self.corr_hist = torch.zeros(cfg.hist_len, dtype=torch.int32, device=dev)
        self.lr_t = torch.full((1,), cfg.lr, device=dev)
        # data: resident in HBM, rank-sharded (Horovod-style DP), reshuffled per epoch
        self.train_x = train_x.to(dev).contiguous()
        self.train_y = train_y.to(dev).contiguous()
        n_all = self.train_x.shape[0]
        self.shard = torch.arange(rank, n_all, world, dtype=torch.int64)
        if self.shard.numel() < B:
            raise ValueError("dataset shard smaller than one batch")
        if int(self.shard.max()) >= n_all:
            raise ValueError("shard index out of range")
        self.shard = self.shard.to(dev)
        self._gen = torch.Generator(device=dev).manual_seed(cfg.seed * 7919 + rank)
        self.perm = torch.empty(self.shard.numel(), dtype=torch.int32, device=dev)
        # this step's dataset rows: written one step ahead by the backward kernel, so the forward
        # reads them directly (host refreshes them when the permutation changes)
        self.rows = torch.empty(B, dtype=torch.int32, device=dev)
        self.steps_done = 0
        self._reshuffle()
        self._graphs: dict[int, torch.cuda.CUDAGraph] = {}
        self.graph_mode = None
        self.graph_steps = self.eager_steps = 0   # how train_steps executed (bench reports it)
        self._graph_parity0 = 0

    def _setup_xgmi(self, n: int, required: bool) -> None:
        """Move P and G into hipIpc-registered memory shared with the other ranks."""
        from ..parallel import xgmi
        if not xgmi.usable(self.pg):
            if required:
                raise xgmi.XgmiUnavailable("xGMI collective not usable for this process group")
            return
        try:
            comm = xgmi.XgmiComm(self.pg, staging_elems=n, param_elems=n)
        except xgmi.XgmiUnavailable as e:
            if required:
                raise
            import logging
            logging.getLogger("arena.mlp").warning("xGMI collective unavailable, using RCCL: %s", e)
            return
        P = comm.params()[:n]
        P.copy_(self.P)
        G = comm.buffer()[:n]
        G.zero_()
        self.P, self.G, self.xgmi = P, G, comm
        self.shard_lo, self.shard_hi = comm.shard(n)

    # ------------------------------------------------------------------------------------------
    def _init_params(self):
        g = torch.Generator().manual_seed(self.cfg.seed)
        L = self.layout
        for name, shp in L.shapes.items():
            if name.startswith("W"):
                if self.cfg.init == "tf":
                    w = torch.randn(shp, generator=g) * 0.1
                    bad = w.abs() > 0.2
                    while bad.any():  # truncated normal: redraw beyond 2 sigma
                        w[bad] = torch.randn(int(bad.sum()), generator=g) * 0.1
                        bad = w.abs() > 0.2
                else:
                    bound = 1.0 / math.sqrt(shp[1])
                    w = (torch.rand(shp, generator=g) * 2 - 1) * bound
                L.view(self.P, name).copy_(w)
            else:
                L.view(self.P, name).fill_(0.1 if self.cfg.init == "tf" else 0.0)

    def _reshuffle(self):
        """New epoch order, generated on the device (no host sync). Indices are a permutation of
        this rank's shard, which was range-checked against the dataset at construction."""
        rp = torch.randperm(self.shard.numel(), generator=self._gen, device=self.device)
        self.perm.copy_(self.shard[rp].to(torch.int32))
        self._sync_rows()

    def set_permutation(self, perm: torch.Tensor) -> None:
        """Replace this epoch's sample order (e.g. to replay another trainer's order)."""
        self.perm.copy_(perm.to(self.perm.device, torch.int32))
        self._sync_rows()

    def _sync_rows(self):
        """rows = perm[(step * B + r) % len] for the next step (host-known step count)."""
        B, L = self.cfg.batch, self.perm.numel()
        pos = (self.steps_done * B + torch.arange(B, device=self.device)) % L
        self.rows.copy_(self.perm[pos])

    def pick_steps_per_graph(self, cap: int = 64, runs=()) -> int:
        """Largest divisor of the epoch length <= cap, so graphs never straddle a reshuffle.
        ``runs``: step counts that will be requested from ``train_steps`` in sequence (e.g. the
        bench's warmup and timed steps); the graph length then divides each of them too, so every
        one of those steps is a graph replay (no eager remainder, no misaligned start)."""
        g = self.steps_per_epoch
        for r in runs:
            if r > 0:
                g = math.gcd(g, int(r))
        return max(d for d in range(1, min(cap, g) + 1) if g % d == 0)

    @property
    def steps_per_epoch(self) -> int:
        return self.perm.numel() // self.cfg.batch

    # ------------------------------------------------------------------------------------------
    def _launch_step(self, parity: int = -1):
        """Enqueue one training step (no host sync, graph-capturable). ``parity`` = this step's
        index & 1 when known at launch (lets the backward issue its logits loads without waiting
        for the step counter); -1 = read it from the counter in-kernel."""
        if self.distributed:
            for part in range(3):
                self._launch_step_part(part, parity)
            return
        if self.external_update:
            self._launch_fwd_head()
            self._launch_wgrad(adam=False, commit=True, parity=parity)
            return
        self._launch_fwd_head()
        self._launch_wgrad(adam=True, parity=parity)

    def _launch_fwd_head(self):
        """Hidden layer + logits accumulation (one launch); writes B = A + 1."""
        cfg, B, A, Bc = self.cfg, self.cfg.batch, self.ctrA, self.ctrB
        ops.mlp_fwd_logits(self.train_x, self.W1, self.b1, self.Hbuf, self.W2, self.logits2,
                           W2_copy=self.W2snap, xb=self.xb, labels=self.train_y, yb=self.yb,
                           x_scale=1.0 / 255.0, idx=self.perm, cursor=A,
                           batch=B, keep_prob=cfg.keep_prob,
                           seed=cfg.seed * 2654435761 + self.rank, step=A, ctr_dst=Bc,
                           ctr_src=A, ctr_add=1, rows=self.rows if self._rows_ahead else None)

    def _launch_wgrad(self, adam: bool, commit: bool = False, parity: int = -1):
        """Softmax-xent recomputed per workgroup from the logits; dW1 (dz via the W2 snapshot and
        the H mask) and dW2 in one launch. With ``adam`` the update is the epilogue (and A = B is
        committed), else the grads go to the flat all-reduce bucket."""
        cfg, B, A, Bc = self.cfg, self.cfg.batch, self.ctrA, self.ctrB
        # the batch rows/labels published by the forward: no gather chain in the backward
        common = dict(x_scales=[1.0 / 255.0, 1.0], gather=[False, False], head_modes=[2, 1],
                      head_w2=[self.W2snap, None], head_h=[self.Hbuf, None],
                      head_keep_prob=cfg.keep_prob, head_logits2=self.logits2, head_step=Bc,
                      head_step_off=-1, head_b2=self.b2, head_labels=self.yb,
                      head_loss_scale=1.0 / B, head_loss_acc=self.loss_hist,
                      head_correct_acc=self.corr_hist,
                      next_rows=self.rows if self._rows_ahead else None,
                      next_rows_perm=self.perm if self._rows_ahead else None,
                      head_parity=parity)
        xs, dzs = [self.xb, self.Hbuf], [None, None]
        if self._x_from_dataset:
            # gather the batch rows from the (never written) dataset instead of the forward's
            # freshly published copy: the rows sit in this XCD's L2 from the forward's own reads
            xs = [self.train_x, self.Hbuf]
            # labels follow the layer-input gather: dataset labels, same rows
            common.update(gather=[True, False], idx=self.perm, cursor=Bc, cursor_off=-1, batch=B,
                          head_labels=self.train_y)
        if adam:
            ops.wgrad_grouped(xs, dzs, [self.W1, self.W2], [self.b1, self.b2], mode=1,
                              mW=[self.mW1, self.mW2], vW=[self.vW1, self.vW2],
                              mB=[self.mb1, self.mb2], vB=[self.vb1, self.vb2],
                              lr=cfg.lr, lr_t=self.lr_t, betas=cfg.betas, eps=cfg.eps,
                              t_step=Bc, tf_style=cfg.tf_adam, ctr_dst=A, ctr_src=Bc, ctr_add=0,
                              **common)
        else:
            ctr = dict(ctr_dst=A, ctr_src=Bc, ctr_add=0) if commit else {}
            ops.wgrad_grouped(xs, dzs, [self.gW1, self.gW2], [self.gb1, self.gb2], mode=0,
                              grad_scale=1.0, **ctr, **common)

    def _capture(self, nsteps: int) -> torch.cuda.CUDAGraph:
        # an even-length graph replayed from steps of one parity sees the same parity sequence
        # every time, so the parity is baked into the launches (train_steps only replays it from
        # steps whose parity is ``_graph_parity0``)
        self._graph_static = nsteps % 2 == 0
        p0 = self._graph_parity0
        # thread_local: the RCCL process group's watchdog thread polls the events of earlier
        # collectives (the xGMI handle exchange, barriers); under the default global capture mode
        # such a poll landing inside the capture is an error that aborts the rank
        # (tests/test_xgmi_gpu.py::test_rccl_allreduce_is_graph_capturable hit it on a GPU run)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            for i in range(nsteps):
                self._launch_step(parity=((p0 + i) & 1) if self._graph_static else -1)
        return g

    def enable_graphs(self, steps_per_graph: int = 50, start_parity: int = 0) -> bool:
        """Capture ``steps_per_graph`` steps per hipGraph. Returns False if capture failed
        (e.g. a collective backend that refuses capture) -- steps then run eagerly.
        ``start_parity``: parity (step & 1) of the steps the replays will start from, e.g. 1 when
        an odd number of warmup steps precedes the timed ones."""
        if self.device.type != "cuda":
            return False
        self.steps_per_graph = steps_per_graph
        self._graph_parity0 = start_parity & 1
        # warm up on a side stream (allocator / collective communicators initialised outside
        # capture), then restore the state so warm-up steps do not count as training.
        state = (self.P, self.M, self.V, self.ctrA, self.ctrB, self.logits2, self.rows,
                 self.loss_hist, self.corr_hist)
        snap = [t.clone() for t in state]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for k in range(2):
                self._launch_step(parity=(self.steps_done + k) & 1)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        for t, v in zip(state, snap):
            t.copy_(v)
        try:
            g = self._capture(steps_per_graph)
            # one replay now, undone: the first launch of an instantiated graph uploads it to
            # the device, which would otherwise land in the first timed replay (the baked step
            # parity may not match step 0 here; every buffer it touches is restored anyway)
            g.replay()
            torch.cuda.synchronize()
            for t, v in zip(state, snap):
                t.copy_(v)
            self._graphs[steps_per_graph] = g
            self.graph_mode = "full"
        except Exception as e:  # noqa: BLE001
            self._graph_error = repr(e)
            self._graphs.clear()
            self.graph_mode = None
            torch.cuda.synchronize()
            if self.distributed:
                return self._enable_split_graphs()
            return False
        torch.cuda.synchronize()
        return True

    def _enable_split_graphs(self) -> bool:
        """Collective refused capture: graph the compute before/after an eager all_reduce."""
        try:
            pre, post = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            self._split = True
            with torch.cuda.graph(pre, capture_error_mode="thread_local"):
                self._launch_step_part(0)
            with torch.cuda.graph(post, capture_error_mode="thread_local"):
                self._launch_step_part(2)
            self._split_graphs = (pre, post)
            self.graph_mode = "split"
            torch.cuda.synchronize()
            return True
        except Exception as e:  # noqa: BLE001
            self._graph_error += " | split: " + repr(e)
            self._split_graphs = None
            self.graph_mode = None
            torch.cuda.synchronize()
            return False

    def _launch_step_part(self, part: int, parity: int = -1):
        """DP step in three parts: 0 = compute up to the grad bucket, 1 = all_reduce, 2 = Adam."""
        cfg, A, Bc = self.cfg, self.ctrA, self.ctrB
        if part == 0:
            self._launch_fwd_head()
            self._launch_wgrad(adam=False, parity=parity)
        elif part == 1:
            if self.xgmi is not None:
                return  # the reduction is fused into part 2
            import torch.distributed as dist
            dist.all_reduce(self.G, group=self.pg)
        elif self.xgmi is not None:
            # reduce-scatter G over xGMI + Adam on the owned shard + all-gather P, one kernel
            self.xgmi.adam_(self.M, self.V, self.layout.total, lr=cfg.lr, lr_t=self.lr_t,
                            betas=cfg.betas, eps=cfg.eps, t_step=Bc,
                            grad_scale=1.0 / self.world, tf_style=cfg.tf_adam, ctr_dst=A,
                            ctr_src=Bc, ctr_add=0)
        else:
            ops.adam_flat(self.P, self.M, self.V, self.G, grad_scale=1.0 / self.world,
                          ctr_dst=A, ctr_src=Bc, ctr_add=0, lr=cfg.lr, lr_t=self.lr_t,
                          betas=cfg.betas, eps=cfg.eps, t_step=Bc, tf_style=cfg.tf_adam)

    def train_steps(self, n: int):
        """Run n steps (graph replays where possible). Reshuffles at epoch boundaries."""
        spe = self.steps_per_epoch
        while n > 0:
            to_epoch_end = spe - (self.steps_done % spe)
            chunk = min(n, to_epoch_end)
            k = getattr(self, "steps_per_graph", 0)
            while chunk > 0:
                aligned = (not getattr(self, "_graph_static", False)
                           or self.steps_done % 2 == self._graph_parity0)
                if self._graphs and chunk >= k and aligned:
                    self._graphs[k].replay()
                    done = k
                    self.graph_steps += k
                elif self.graph_mode == "split":
                    pre, post = self._split_graphs
                    pre.replay()
                    self._launch_step_part(1)
                    post.replay()
                    done = 1
                    self.graph_steps += 1
                else:
                    self._launch_step(parity=self.steps_done & 1)
                    done = 1
                    self.eager_steps += 1
                chunk -= done
                n -= done
                self.steps_done += done
            if self.steps_done % spe == 0:
                self._reshuffle()
        heartbeat.beat(self.steps_done)  # progress for the runtime's hang detection

    # ------------------------------------------------------------------------------------------
    def recent_metrics(self, last: int = 100):
        """(mean loss, train accuracy) over the last ``last`` completed steps (host sync)."""
        done = int(self.ctrA.item())
        L = self.cfg.hist_len
        last = min(last, done, L - 1)
        if last <= 0:
            return float("nan"), float("nan")
        idx = torch.tensor([(done - 1 - i) % L for i in range(last)], device=self.device)
        loss = float(self.loss_hist[idx].mean().item())
        acc = float(self.corr_hist[idx].float().mean().item()) / self.cfg.batch
        return loss, acc

    @torch.no_grad()
    def evaluate(self, test_x: torch.Tensor, test_y: torch.Tensor, chunk: int = 10000):
        """Test-set (loss, accuracy) with dropout off, on the same kernels."""
        dev = self.device
        n = test_x.shape[0]
        loss_acc = torch.zeros(1, device=dev)
        corr = torch.zeros(1, dtype=torch.int32, device=dev)
        tx = test_x.to(dev).contiguous()
        ty = test_y.to(dev).contiguous()
        for s in range(0, n, chunk):
            xs = tx[s:s + chunk]
            ys = ty[s:s + chunk]
            h = torch.empty(xs.shape[0], self.cfg.hidden, device=dev)
            ops.linear_fwd(xs, self.W1, h, self.b1, x_scale=1.0 / 255.0, act=1, keep_prob=1.0)
            ops.xent_head(h, self.W2, self.b2, ys, loss_acc=loss_acc, correct_acc=corr,
                          loss_scale=1.0 / n)
        return float(loss_acc.item()), float(corr.item()) / n

    def state_dict(self):
        M, V = self.M, self.V
        if self.xgmi is not None:
            # optimizer state is sharded (each rank updates its chunk; the rest stays zero), so a
            # sum over ranks reassembles it
            M, V = M.clone(), V.clone()
            self.xgmi.all_reduce_(M)
            self.xgmi.all_reduce_(V)
        # the epoch order and the shuffle generator too, so a resumed run replays exactly the
        # batches (and dropout masks: keyed by the step counter) the uninterrupted run would see
        return {"P": self.P.detach().cpu(), "M": M.detach().cpu(), "V": V.detach().cpu(),
                "step": int(self.ctrA.item()), "layout": dict(self.layout.shapes),
                "perm": self.perm.detach().cpu(), "rng": self._gen.get_state(),
                "rank": self.rank, "world": self.world}

    def load_state_dict(self, sd):
        self.P.copy_(sd["P"])
        self.M.copy_(sd["M"])
        self.V.copy_(sd["V"])
        if self.xgmi is not None:  # keep only this rank's optimizer shard
            for t in (self.M, self.V):
                t[:self.shard_lo].zero_()
                t[self.shard_hi:].zero_()
        self.ctrA.fill_(int(sd["step"]))
        self.ctrB.fill_(int(sd["step"]))
        self.steps_done = int(sd["step"])
        if (sd.get("perm") is not None and sd.get("world", self.world) == self.world
                and sd.get("rank", self.rank) == self.rank
                and sd["perm"].numel() == self.perm.numel()):
            self.perm.copy_(sd["perm"])
            self._gen.set_state(sd["rng"])
        self._sync_rows()
