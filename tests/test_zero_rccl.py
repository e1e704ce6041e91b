"""ShardedMasterSGD's RCCL backend and its bucket layout, on CPU over gloo.

Ranks that cannot map each other's GPUs (multi-pod, multi-node) keep the bf16-weight sharded
design: reduce_scatter_tensor of each bucket's sub-range -> shard_sgd on the owned equal-size
shard -> all_gather_into_tensor. Here worlds 2 and 4 on gloo with CPU tensors (the shard update
runs its PyTorch reference; the HIP kernel is checked against it in tests/test_optim.py) against
fp32 ``torch.optim.SGD`` on the averaged gradient, for bf16 weights (fp32 masters) and fp32
weights, mixed buckets, several steps, an lr change and unused parameters.
"""
from __future__ import annotations

import os
import socket
import traceback

import pytest
import torch
import torch.multiprocessing as mp


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


SHAPES = [((16, 8, 3, 3), "bf16"), ((16,), "fp32"), ((16,), "fp32"), ((32, 16), "bf16"),
          ((7,), "fp32"), ((64, 32, 1, 1), "bf16"), ((33,), "fp32"), ((10, 64), "bf16"),
          ((10,), "fp32")]


def _params():
    g = torch.Generator().manual_seed(42)
    ps = []
    for shp, kind in SHAPES:
        t = torch.randn(shp, generator=g)
        if len(shp) == 4:
            t = t.contiguous(memory_format=torch.channels_last)
        ps.append((torch.nn.Parameter(t.to(torch.bfloat16) if kind == "bf16" else t), kind))
    return ps


def _grads(step, rank, params):
    g = torch.Generator().manual_seed(1000 * step + rank)
    out = []
    for p, _ in params:
        t = (torch.randn(p.shape, generator=g) * 0.1).to(p.dtype)
        if p.dim() == 4:
            t = t.contiguous(memory_format=torch.channels_last)
        out.append(t)
    return out


def _worker(rank, world, port, reduce_fp32, q, backend="rccl", local_size=None,
            skew_order=False):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world))
        import torch.distributed as dist
        dist.init_process_group("gloo")
        from arena_amd.parallel.zero import ShardedMasterSGD
        lr, mu, wd = 0.05, 0.9, 1e-3
        params = _params()
        order = [p for p, _ in params]
        ref = [torch.nn.Parameter(p.detach().float().clone()) for p, _ in params]
        ropt = torch.optim.SGD([{"params": [r for r, (_, k) in zip(ref, params) if k == "bf16"],
                                 "weight_decay": wd},
                                {"params": [r for r, (_, k) in zip(ref, params) if k == "fp32"],
                                 "weight_decay": 0.0}], lr=lr, momentum=mu)
        opt = ShardedMasterSGD([{"params": [p for p, k in params if k == "bf16"],
                                 "weight_decay": wd},
                                {"params": [p for p, k in params if k == "fp32"],
                                 "weight_decay": 0.0, "weights": "fp32"}],
                               lr=lr, momentum=mu, bucket_mb=0.004, last_bucket_mb=0.001,
                               backend=backend, order=order, rccl_reduce_fp32=reduce_fp32,
                               local_size=local_size)
        res = {"backend": opt.backend, "nbuckets": len(opt.buckets),
               "shards": {str(dt): [opt.shard_ranges(r, dt) for r in range(world)]
                          for dt in (torch.bfloat16, torch.float32)},
               "mixed": sum(1 for b in opt.buckets if len(b.ranges) == 2)}
        # layout: each sub-range splits into equal 16-byte-aligned shards
        res["padded"] = all((r.end - r.start) % (world * (8 if r.dtype == torch.bfloat16 else 4))
                            == 0 for b in opt.buckets for r in b.ranges)
        res["last_bucket_params"] = [tuple(p.shape) for p in opt.buckets[-1].params]
        for step in range(4):
            if step == 3:
                for grp in list(opt.param_groups) + list(ropt.param_groups):
                    grp["lr"] = lr * 2
            grads = [_grads(step, r, params) for r in range(world)]
            unused = 4 if step == 1 else -1          # parameter 4 gets no gradient in step 1
            for i, ((p, _), g) in enumerate(zip(params, grads[rank])):
                p.grad = None if i == unused else g.clone()
            if skew_order:
                # gradients become ready in a rank-dependent order (data-dependent control flow):
                # rank 0 output side first, the others input side first
                idx = list(range(len(params)))
                for i in (idx[::-1] if rank == 0 else idx):
                    if i != unused:
                        opt._on_grad(params[i][0])
            opt.step()
            opt.zero_grad()
            for i, r in enumerate(ref):
                if i == unused:
                    r.grad = torch.zeros_like(r)
                    continue
                acc = grads[0][i].float()
                for gr in grads[1:]:
                    acc = acc + gr[i].float()
                r.grad = acc / world
            ropt.step()
            ropt.zero_grad()
        sd = opt.state_dict()
        pos = {id(p): i for i, p in enumerate(opt.params)}
        worst_master, worst_w = 0.0, 0.0
        for (p, kind), r in zip(params, ref):
            m = sd["master"][pos[id(p)]]
            scale = float(r.detach().abs().max()) + 1e-12
            worst_master = max(worst_master, float((m - r.detach()).abs().max()) / scale)
            if kind == "bf16":
                # weights = the rounded masters, bit for bit
                worst_w = max(worst_w, float((p.detach().float() - m.to(torch.bfloat16).float())
                                             .abs().max()))
        res["master_rel"] = worst_master
        res["w_vs_master"] = worst_w
        flat = torch.cat([p.detach().float().reshape(-1) for p, _ in params])
        res["digest"] = float(flat.double().sum())
        opt.close()
        dist.destroy_process_group()
        q.put((rank, res, None))
    except Exception:  # noqa: BLE001
        q.put((rank, None, traceback.format_exc()))


def _run(world, reduce_fp32, backend="rccl", local_size=None, skew_order=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, reduce_fp32, q, backend,
                                                local_size, skew_order))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, res, err = q.get(timeout=180)
            assert err is None, f"rank {r} failed:\n{err}"
            out[r] = res
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    return out


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("reduce_fp32", [True, False])
def test_rccl_sharded_sgd_matches_torch_sgd(world, reduce_fp32):
    out = _run(world, reduce_fp32)
    for r, res in out.items():
        assert res["backend"] == "rccl" and res["padded"], res
        assert res["nbuckets"] >= 3 and res["mixed"] >= 1, res
        # the input-side bucket (last ready) is the small one: the first layer's params only
        assert res["last_bucket_params"][-1] == (16, 8, 3, 3), res
        # fp32 sums in gloo's order vs the reference's: a few fp32 ulps; bf16 sums round per add
        tol = 1e-5 if reduce_fp32 else 2e-2
        assert res["master_rel"] < tol, (r, res)
        assert res["w_vs_master"] == 0.0, (r, res)
    assert len({res["digest"] for res in out.values()}) == 1, out     # replicas identical


def _check_shards_partition(res, world):
    """Every sub-range's W shards are disjoint, equal and cover it exactly."""
    for dt, per_rank in res["shards"].items():
        for j in range(len(per_rank[0])):
            spans = sorted(per_rank[r][j] for r in range(world))
            for (a, b), (c, _) in zip(spans, spans[1:]):
                assert b == c, (dt, j, spans)
            assert len({b - a for a, b in spans}) == 1, (dt, j, spans)


@pytest.mark.parametrize("world,local_size", [(4, 2), (6, 2), (8, 4)])
@pytest.mark.parametrize("reduce_fp32", [True, False])
def test_hier_sharded_sgd_matches_torch_sgd(world, local_size, reduce_fp32):
    """Hierarchical backend (Horovod's hierarchical allreduce, sharded): node-level
    reduce-scatter, then between nodes on the 1/L chunk; shard update; all-gathers in reverse.
    Here 2 and 3 'nodes' of 2 ranks each on gloo."""
    out = _run(world, reduce_fp32, backend="hier", local_size=local_size)
    for r, res in out.items():
        assert res["backend"] == "hier" and res["padded"], res
        _check_shards_partition(res, world)
        tol = 1e-5 if reduce_fp32 else 2e-2
        assert res["master_rel"] < tol, (r, res)
        assert res["w_vs_master"] == 0.0, (r, res)
    assert len({res["digest"] for res in out.values()}) == 1, out
    # the hierarchical slice order differs from the flat one: local rank l, node k owns
    # slice l * nodes + k
    nodes = world // local_size
    sh = out[0]["shards"][str(torch.bfloat16)]
    base = sh[0][0][0]
    sl = sh[0][0][1] - base
    for r in range(world):
        assert sh[r][0][0] == base + ((r % local_size) * nodes + r // local_size) * sl


def test_auto_picks_hier_across_nodes():
    """auto -> hier when the job spans several nodes of more than one rank each (ranks that
    cannot map each other); an explicit rccl stays flat; one node -> flat rccl."""
    assert all(res["backend"] == "hier" for res in _run(4, False, "auto", 2).values())
    assert all(res["backend"] == "rccl" for res in _run(4, False, "rccl", 2).values())
    assert all(res["backend"] == "rccl" for res in _run(2, False, "auto", 2).values())


def test_hier_rejects_bad_local_size():
    """local_size must divide the world and leave more than one node of more than one rank."""
    import torch.distributed as dist
    from arena_amd.parallel.zero import ShardedMasterSGD
    store = dist.HashStore()
    dist.init_process_group("gloo", store=store, rank=0, world_size=1)
    try:
        p = torch.nn.Parameter(torch.randn(8, 8).to(torch.bfloat16))
        with pytest.raises(ValueError, match="1 < local_size < world"):
            ShardedMasterSGD([p], lr=0.1, backend="hier", local_size=1)
        with pytest.raises(ValueError, match="must divide"):
            ShardedMasterSGD([p], lr=0.1, backend="hier", local_size=3)
        # flat RCCL never uses local_size: a non-dividing value is not an error there
        ShardedMasterSGD([torch.nn.Parameter(torch.randn(8, 8).to(torch.bfloat16))], lr=0.1,
                         backend="rccl", local_size=3).close()
        with pytest.raises(ValueError, match="backend must be"):
            ShardedMasterSGD([p], lr=0.1, backend="ring")
        opt = ShardedMasterSGD([p], lr=0.1, backend="auto")   # one rank: flat, no level groups
        assert opt.backend == "rccl" and opt._intra is None
        opt.close()
    finally:
        dist.destroy_process_group()


def test_bucket_launch_order_independent_of_gradient_order():
    """ADVICE r5 (zero.py:458): with overlap, a bucket used to launch as soon as its gradients
    were ready on THAT rank, so ranks whose gradients arrive in different orders issued their
    collectives in different orders (hang, or one bucket reduced against another). Buckets now
    launch strictly in index order; the result must still match torch SGD on every rank."""
    out = _run(2, True, skew_order=True)
    for r, res in out.items():
        assert res["master_rel"] < 1e-5 and res["w_vs_master"] == 0.0, (r, res)
    assert len({res["digest"] for res in out.values()}) == 1, out


def test_uneven_local_world_size_falls_back_to_flat(monkeypatch):
    """ADVICE r5 (zero.py:593): a LOCAL_WORLD_SIZE that does not divide the world only rules
    the hierarchical backend out; it no longer fails flat RCCL."""
    from arena_amd.parallel.zero import ShardedMasterSGD
    o = ShardedMasterSGD.__new__(ShardedMasterSGD)
    o.world = 6
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    assert o._local_size(None, strict=False) == 6
    o.local_size = 6
    assert o._flat_or_hier() == "rccl"
    with pytest.raises(ValueError):
        o._local_size(None, strict=True)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    o.local_size = o._local_size(None, strict=False)
    assert o._flat_or_hier() == "hier"
