"""Parallel layer on CPU: Horovod-style API over gloo (world 2) and the native parameter server."""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from arena_amd import _build
from arena_amd.parallel import ps as psmod


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _hvd_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from torch import nn
    from arena_amd.parallel import hvd
    hvd.init("gloo")
    try:
        assert hvd.rank() == rank and hvd.size() == world
        # allreduce average / sum, allgather with ragged first dims, broadcast
        t = torch.tensor([float(rank + 1)] * 3)
        avg = hvd.allreduce(t)
        tot = hvd.allreduce(t, average=False)
        ag = hvd.allgather(torch.full((rank + 1, 2), float(rank)))
        b = torch.tensor([float(rank * 10)])
        hvd.broadcast_(b, root_rank=1)
        # model: different init per rank -> broadcast_parameters makes them equal
        torch.manual_seed(100 + rank)
        model = nn.Sequential(nn.Linear(12, 16), nn.ReLU(), nn.Linear(16, 4))
        hvd.broadcast_parameters(model.state_dict(), root_rank=0)
        opt = hvd.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1),
                                       named_parameters=model.named_parameters(), bucket_mb=0.0002)
        g = torch.Generator().manual_seed(7)
        data = [(torch.randn(8, 12, generator=g), torch.randint(0, 4, (8,), generator=g))
                for _ in range(2 * world)]
        # each rank takes its half of every global batch
        for step in range(3):
            x, y = data[step % len(data)]
            xs, ys = x[rank::world], y[rank::world]
            loss = nn.functional.cross_entropy(model(xs), ys, reduction="sum") / x.shape[0] * world
            opt.zero_grad()
            loss.backward()
            opt.step()
        flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
        q.put((rank, avg.tolist(), tot.tolist(), ag.tolist(), b.item(), flat.numpy(),
               len(opt.buckets)))
    finally:
        hvd.shutdown()


@pytest.mark.timeout(180)
def test_hvd_api_world2_matches_single_process():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_hvd_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=150) for _ in range(world))
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    (_, avg0, tot0, ag0, b0, flat0, nb0), (_, avg1, tot1, ag1, b1, flat1, nb1) = res
    assert avg0 == avg1 == [1.5] * 3 and tot0 == [3.0] * 3
    assert ag0 == [[0.0, 0.0], [1.0, 1.0], [1.0, 1.0]] == ag1
    assert b0 == b1 == 10.0
    assert nb0 > 1  # tiny bucket cap -> several buckets, reduced as grads become ready
    np.testing.assert_array_equal(flat0, flat1)  # replicas stay identical
    # == single-process SGD on the full batch from rank 0's initial weights
    from torch import nn
    torch.manual_seed(100)
    model = nn.Sequential(nn.Linear(12, 16), nn.ReLU(), nn.Linear(16, 4))
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(7)
    data = [(torch.randn(8, 12, generator=g), torch.randint(0, 4, (8,), generator=g))
            for _ in range(2 * world)]
    for step in range(3):
        x, y = data[step % len(data)]
        loss = nn.functional.cross_entropy(model(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).numpy()
    np.testing.assert_allclose(flat0, ref, rtol=1e-5, atol=1e-6)


def _hvd_optstate_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from torch import nn
    from arena_amd.ops.optim import OptimizerGroup
    from arena_amd.parallel import hvd
    hvd.init("gloo")
    try:
        torch.manual_seed(3)
        m = nn.Linear(3, 5)
        o = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
        m(torch.ones(2, 3) * (rank + 1)).sum().backward()   # momentum differs per rank
        o.step()

        class Stateless:       # e.g. ShardedMasterSGD: masters derive from the weights
            param_groups: list = []
            state: dict = {}

        hvd.broadcast_optimizer_state(OptimizerGroup(o, Stateless()), root_rank=1)
        bufs = torch.cat([o.state[p]["momentum_buffer"].reshape(-1) for p in m.parameters()])
        q.put((rank, bufs.numpy()))
    finally:
        hvd.shutdown()


@pytest.mark.timeout(120)
def test_hvd_broadcast_optimizer_state_recurses_groups():
    """broadcast_optimizer_state walks OptimizerGroup members and skips state-less optimizers:
    every rank ends with the root's momentum buffers."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_hvd_optstate_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    np.testing.assert_array_equal(res[0], res[1])
    # root (rank 1) weight gradient: input 2 per sample x 2 samples -> 4 (rank 0 had 2)
    assert res[0][0] == 4.0


def _hvd_root_only_state_worker(rank, world, port, q, device="cpu", fused=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    from torch import nn
    from arena_amd.parallel import hvd
    if device == "cuda":
        torch.cuda.set_device(0)
    hvd.init("gloo")
    try:
        torch.manual_seed(3)
        m = nn.Linear(3, 5).to(device)
        o = torch.optim.Adam(m.parameters(), lr=0.1, fused=fused or None)
        if rank == 0:       # "checkpoint loaded on the root only": only rank 0 has state
            m(torch.ones(2, 3, device=device)).sum().backward()
            o.step()
            o.step()
        hvd.broadcast_optimizer_state(o, root_rank=0)
        st = [o.state[p] for p in m.parameters()]
        q.put((rank, {"m": torch.cat([s["exp_avg"].reshape(-1) for s in st]).cpu().numpy(),
                      "v": torch.cat([s["exp_avg_sq"].reshape(-1) for s in st]).cpu().numpy(),
                      "step": [float(s["step"]) for s in st],
                      "step_dev": [s["step"].device.type for s in st]}))
        # the optimizer keeps working on every rank afterwards
        m(torch.ones(2, 3, device=device)).sum().backward()
        o.step()
    finally:
        hvd.shutdown()


@pytest.mark.gpu
@pytest.mark.timeout(180)
def test_hvd_broadcast_optimizer_state_root_only_fused_adam():
    """ADVICE r5 (hvd.py:328): with Adam(fused=True) the root's "step" lives on the GPU; rank 1
    (no state) must create it there too, or the (dtype, device)-grouped broadcast sizes differ."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_hvd_root_only_state_worker, args=(r, world, port, q, "cuda", True))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=150) for _ in range(world))
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    np.testing.assert_array_equal(res[0]["m"], res[1]["m"])
    assert res[1]["step"] == [2.0, 2.0] and res[1]["step_dev"] == ["cuda", "cuda"], res


@pytest.mark.timeout(120)
def test_hvd_broadcast_optimizer_state_root_only_state():
    """ADVICE r4 (hvd.py:211): the Horovod pattern of restoring a checkpoint on rank 0 and
    broadcasting the optimizer state. Rank 1 has NO state; it must not skip the collectives
    (that hung the job): the root's state layout is broadcast first and rank 1 creates it."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_hvd_root_only_state_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    np.testing.assert_array_equal(res[0]["m"], res[1]["m"])
    np.testing.assert_array_equal(res[0]["v"], res[1]["v"])
    assert res[1]["step"] == [2.0, 2.0] and np.abs(res[1]["m"]).sum() > 0


def test_cluster_spec_parsing():
    env = {"TF_CONFIG": '{"cluster":{"ps":["h:1"],"worker":["a:2","b:3"]},'
                        '"task":{"type":"worker","index":1}}'}
    s = psmod.ClusterSpec.from_env(env)
    assert s.ps == ["h:1"] and s.worker == ["a:2", "b:3"] and s.task_index == 1 and not s.is_chief
    env = {"MX_CLUSTER_SPEC": '{"cluster":{"ps":["h:1"],"chief":["c:9"],"worker":["a:2"]},'
                              '"task":{"type":"worker","index":0}}'}
    s = psmod.ClusterSpec.from_env(env)
    assert s.worker == ["c:9", "a:2"] and s.task_index == 1
    assert psmod.shard_ranges(10, 3) == [(0, 4), (4, 8), (8, 10)]
    assert psmod.shard_ranges(5, 1) == [(0, 5)]


@pytest.fixture(scope="module")
def ps_tool():
    _build.build_native_tools()


def _torch_adam(p0, grads, lr):
    p = torch.tensor(p0.copy(), requires_grad=True)
    opt = torch.optim.Adam([p], lr=lr)
    for g in grads:
        p.grad = torch.tensor(g)
        opt.step()
    return p.detach().numpy()


def test_native_ps_async_adam_matches_torch(ps_tool):
    n, lr = 1003, 1e-2
    ports = [_free_port(), _free_port()]
    servers = [psmod.spawn_server(p, 1, lr=lr) for p in ports]
    try:
        cl = psmod.PSClient([f"127.0.0.1:{p}" for p in ports], n, timeout_s=10)
        rng = np.random.default_rng(0)
        p0 = rng.standard_normal(n).astype(np.float32)
        cl.init(p0)
        cl.init(p0 + 1)  # second INIT ignored (only the chief's takes effect)
        out = np.empty(n, np.float32)
        assert cl.pull(out) == 0
        np.testing.assert_array_equal(out, p0)
        grads = [rng.standard_normal(n).astype(np.float32) for _ in range(5)]
        for i, g in enumerate(grads):
            assert cl.push_pull(g, out) == i + 1
        np.testing.assert_allclose(out, _torch_adam(p0, grads, lr), rtol=2e-5, atol=2e-6)
        st = cl.stats()
        assert [s[0] for s in st] == [5, 5] and sum(s[1] for s in st) == n
        cl.done()
        for s in servers:
            assert s.wait(10) == 0  # all (1) workers done -> servers exit cleanly
    finally:
        for s in servers:
            if s.poll() is None:
                s.kill()


def test_native_ps_sync_averages_one_grad_per_worker(ps_tool):
    import threading
    n, lr = 64, 0.5
    port = _free_port()
    srv = psmod.spawn_server(port, 2, lr=lr, optimizer="sgd", sync=True)
    try:
        p0 = np.zeros(n, np.float32)
        clients = [psmod.PSClient([f"127.0.0.1:{port}"], n, timeout_s=10) for _ in range(2)]
        clients[0].init(p0)
        outs = [np.empty(n, np.float32) for _ in range(2)]
        steps = [None, None]

        def go(i):
            g = np.full(n, float(i + 1), np.float32)     # 1 and 2 -> mean 1.5
            steps[i] = clients[i].push_pull(g, outs[i])
        ts = [threading.Thread(target=go, args=(i,)) for i in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(10)
        assert steps == [1, 1]
        np.testing.assert_allclose(outs[0], -lr * 1.5)
        np.testing.assert_array_equal(outs[0], outs[1])
        for c in clients:
            c.done()
        assert srv.wait(10) == 0
    finally:
        if srv.poll() is None:
            srv.kill()


def test_trainer_external_update_produces_grads_only():
    from arena_amd.models.mlp import FusedMLPTrainer, MLPConfig
    torch.manual_seed(0)
    x = torch.randint(0, 256, (400, 784), dtype=torch.uint8)
    y = torch.randint(0, 10, (400,), dtype=torch.uint8)
    cfg = MLPConfig(batch=100)
    tr = FusedMLPTrainer(cfg, x, y, device="cpu", external_update=True)
    p_before = tr.P.clone()
    tr.train_steps(2)
    assert torch.equal(tr.P, p_before)              # no local optimizer
    assert tr.G.abs().sum() > 0 and int(tr.ctrA.item()) == 2


def _hvd_nhwc_worker(rank, world, port, q):
    """Channels_last conv weights: their gradients are NHWC-strided, not contiguous."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from torch import nn
    from arena_amd.parallel import hvd
    hvd.init("gloo")
    try:
        torch.manual_seed(3)
        model = nn.Sequential(nn.Conv2d(3, 8, 3), nn.ReLU(), nn.Conv2d(8, 4, 1),
                              nn.Flatten(), nn.LazyLinear(5))
        model(torch.zeros(1, 3, 6, 6))
        model = model.to(memory_format=torch.channels_last)
        opt = hvd.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1),
                                       named_parameters=model.named_parameters(), bucket_mb=0.001)
        g = torch.Generator().manual_seed(100 + rank)
        x = torch.randn(4, 3, 6, 6, generator=g).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 5, (4,), generator=g)
        loss = nn.functional.cross_entropy(model(x), y)
        opt.zero_grad()
        loss.backward()
        strided = any(not p.grad.is_contiguous() for p in model.parameters())
        opt.step()
        flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
        q.put((rank, flat.numpy(), strided))
    finally:
        hvd.shutdown()


@pytest.mark.timeout(180)
def test_hvd_channels_last_gradients_average_correctly():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_hvd_nhwc_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=150) for _ in range(world)), key=lambda t: t[0])
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    (_, f0, strided), (_, f1, _) = res
    assert strided                                   # the case under test actually occurred
    np.testing.assert_array_equal(f0, f1)
    # reference: mean of the two ranks' gradients, one SGD step, in one process
    from torch import nn
    torch.manual_seed(3)
    model = nn.Sequential(nn.Conv2d(3, 8, 3), nn.ReLU(), nn.Conv2d(8, 4, 1), nn.Flatten(),
                          nn.LazyLinear(5))
    model(torch.zeros(1, 3, 6, 6))
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    opt.zero_grad()
    for r in range(world):
        g = torch.Generator().manual_seed(100 + r)
        x = torch.randn(4, 3, 6, 6, generator=g)
        y = torch.randint(0, 5, (4,), generator=g)
        (nn.functional.cross_entropy(model(x), y) / world).backward()
    opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).numpy()
    np.testing.assert_allclose(f0, ref, rtol=1e-5, atol=1e-6)


def test_identities_share_node_rules():
    from arena_amd.parallel.xgmi import identities_share_node as share
    a = {"host": "n1", "boot": "b", "own": "g0", "visible": ["g0", "g1"]}
    b = {"host": "n1", "boot": "b", "own": "g1", "visible": ["g0", "g1"]}
    assert share([a, b])
    assert not share([a, {**b, "host": "n2"}])                  # another host
    assert not share([a, {**b, "boot": "other"}])               # same name, another machine boot
    # K8s pods: each process sees only its own device-plugin GPU
    assert not share([{**a, "visible": ["g0"]}, {**b, "visible": ["g1"]}])
    # ranks time-sharing one GPU (the same-GPU test setup) are mappable
    assert share([{**a, "visible": ["g0"]}, {**a, "visible": ["g0"]}])
    # unknown GPU identities: the host check decides
    assert share([{**a, "own": "", "visible": []}, {**b, "own": "", "visible": []}])
    assert not share([])


def _guard_worker(rank, world, port, q, hosts):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from arena_amd.parallel import xgmi
    socket.gethostname = lambda: hosts[rank]        # what each rank reports as its host
    dist.init_process_group("gloo")
    try:
        q.put((rank, xgmi.same_node(), xgmi.usable()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("hosts,want", [(("a", "a"), True), (("a", "b"), False)])
def test_xgmi_same_host_guard_gloo(hosts, want, monkeypatch):
    """The collective guard on real gloo ranks: mixed hostnames refuse xGMI on every rank (and
    without a GPU, usable() is False everywhere, decided collectively)."""
    monkeypatch.delenv("LOCAL_WORLD_SIZE", raising=False)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_guard_worker, args=(r, 2, port, q, hosts)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r, (s, u)) for r, s, u in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(30)
    assert got[0] == got[1] == (want, False)


def _verify_worker(rank, world, port, q, perturb):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from arena_amd.parallel.verify import ReplicaCheck, ReplicaMismatch, param_checksum
    dist.init_process_group("gloo")
    try:
        ps = [torch.arange(12, dtype=torch.float32).view(3, 4), torch.ones(5, dtype=torch.bfloat16)]
        chk = ReplicaCheck(2, lambda: ps)
        out = []
        for step in range(1, 5):
            if perturb and step == 3 and rank == 1:
                ps[0][1, 2] += 1e-3            # one element off on one rank
            try:
                chk.maybe(step)
                out.append("ok")
            except ReplicaMismatch as e:
                out.append(str(e))
        # a swap of two elements keeps the plain sum but not the checksum
        a = torch.tensor([1.0, 2.0, 3.0])
        swapped = not torch.equal(param_checksum([a]), param_checksum([a.flip(0)]))
        q.put((rank, out, chk.checks, swapped))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("perturb", [False, True])
def test_replica_check_gloo(perturb):
    """--verify-every: replicas compared every K steps; one perturbed element on one rank makes
    EVERY rank raise at the next check (no rank left waiting in a collective)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_verify_worker, args=(r, 2, port, q, perturb)) for r in range(2)]
    for p in procs:
        p.start()
    got = {r: (o, n, s) for r, o, n, s in (q.get(timeout=120) for _ in range(2))}
    for p in procs:
        p.join(30)
    for r in (0, 1):
        out, n, swapped = got[r]
        assert swapped and n == 2
        assert out[0] == out[2] == "ok"                 # steps 1, 3: no check
        assert out[1] == "ok"                           # step 2: agree
        if perturb:
            assert "diverged at step 4" in out[3]
        else:
            assert out[3] == "ok"
