#!/usr/bin/env python3
"""Does a captured ResNet training step use memory the caching allocator considers free?

Capture one step, replay it, then allocate NaN-filled junk tensors outside the graph (the
ordinary pool) and free them, and replay again. A graph that only touches its own private pool
and live tensors is unaffected; one that kept a pointer to freed memory now reads NaN.
Feature switches bisect which component holds such a pointer.

    python tools/graph_mem_check.py --mode auto [--no_master] [--bn_ref] [--no_join]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="auto")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--no_master", action="store_true", help="torch SGD, fp32 weights")
    ap.add_argument("--bn_ref", action="store_true", help="BatchNorm on the PyTorch path")
    ap.add_argument("--no_join", action="store_true", help="no residual-gradient join")
    ap.add_argument("--junk_gb", type=float, default=8.0)
    ap.add_argument("--empty_cache", action="store_true", help="torch.cuda.empty_cache() first")
    ap.add_argument("--second_model", default="",
                    help="conv mode of a second model trained EAGERLY (4 steps) between replays")
    ap.add_argument("--second_bn_ref", action="store_true", help="second model: PyTorch BN")
    ap.add_argument("--fin_p", type=int, default=0, help="BN finalize blocks per channel group")
    ap.add_argument("--eager_kernel", default="",
                    help="between replays, launch N eager kernels of this kind on junk tensors: "
                         "conv_fwd | conv_wgrad | flip | bn | sgd | foreach | torch_small")
    ap.add_argument("--eager_n", type=int, default=200)
    ap.add_argument("--deterministic", action="store_true", help="cudnn.deterministic (MIOpen)")
    ap.add_argument("--diag_model", action="store_true",
                    help="ResNet-50 blocks with every stride 1 and no stem, on a 64-channel "
                         "input: no convolution that only MIOpen can run (stem, stride-2 dgrad)")
    ap.add_argument("--second_graph", action="store_true",
                    help="capture a second (junk-writing) graph before the junk allocations")
    a = ap.parse_args()
    from arena_amd.examples import cnn_bench
    from arena_amd.models import resnet as R
    from arena_amd.ops import batchnorm, conv
    from arena_amd.parallel import hvd
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    hvd.init("gloo")
    conv.set_mode(a.mode)
    torch.backends.cudnn.deterministic = a.deterministic
    if a.fin_p:
        from arena_amd.ops import _ext
        _ext.load().bn_set_fin_max_blocks(a.fin_p)
    if a.bn_ref:
        batchnorm.kernel_ok = lambda *args, **kw: False
    if a.no_join:
        class NoJoin(conv.GradJoin):
            def register(self):
                return self
        R.GradJoin = NoJoin
    argv = ["--model", "resnet50", "--batch_size", str(a.batch)]
    if a.no_master:
        argv += ["--master_weights", "off"]
    args = cnn_bench.parse(argv)
    if a.diag_model:
        from torch import nn

        class Diag(nn.Module):
            def __init__(self):
                super().__init__()
                blocks, cin = [], 64
                for i, n in enumerate([3, 4, 6, 3]):
                    mid = 64 * 2 ** i
                    for _ in range(n):
                        blocks.append(R.Bottleneck(cin, mid, 1))
                        cin = mid * 4
                self.layers = nn.ModuleList(blocks)
                self.fc = nn.Linear(cin, 1000)
                self.stem = nn.ModuleList([nn.Identity(), blocks[0].bn1])  # finite() probes

            def forward(self, t):
                link = None
                for b in self.layers:
                    out_link = conv.BNGradLink()
                    t = b(t, link=link, link_out=out_link)
                    link = out_link
                return self.fc(torch.flatten(nn.functional.adaptive_avg_pool2d(t, 1), 1))

        from arena_amd.ops.optim import MasterSGD, OptimizerGroup
        torch.manual_seed(1234)
        model = Diag().to(dev).to(memory_format=torch.channels_last)
        decay = [p for p in model.parameters() if p.ndim > 1]
        nodecay = [p for p in model.parameters() if p.ndim <= 1]
        opt = OptimizerGroup(MasterSGD(decay, lr=0.1, momentum=0.9, weight_decay=4e-5),
                             torch.optim.SGD(nodecay, lr=0.1, momentum=0.9, foreach=True))
        gg = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(a.batch, 64, 28, 28, device=dev, generator=gg).contiguous(
            memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (a.batch,), device=dev, generator=gg)
    else:
        model, opt, x, y = cnn_bench.build(args, dev, 1)
    for _ in range(4):
        cnn_bench.train_step(model, opt, x, y, torch.bfloat16)
    torch.cuda.synchronize()
    g, loss = cnn_bench.capture_step(model, opt, x, y, torch.bfloat16)

    def finite():
        bad = [n for n, p in model.named_parameters()
               if not bool(torch.isfinite(p.detach().float()).all())]
        return len(bad), bad[:3]

    g.replay()
    torch.cuda.synchronize()
    print(f"replay 0: loss {float(loss):.4f} nonfinite {finite()}", flush=True)
    if a.empty_cache:
        torch.cuda.empty_cache()
    def live_state():
        t = {"x": x, "y": y}
        for n, p in model.named_parameters():
            t["p:" + n] = p.detach()
            if p.grad is not None:
                t["g:" + n] = p.grad
        for n, b in model.named_buffers():
            t["b:" + n] = b
        for k, o in enumerate(getattr(opt, "opts", [opt])):
            for attr in ("master", "mom", "wbf"):
                if hasattr(o, attr):
                    t[f"opt{k}.{attr}"] = getattr(o, attr)
            for j, st in enumerate(getattr(o, "state", {}).values()):
                for kk, v in st.items():
                    if torch.is_tensor(v) and v.is_cuda:
                        t[f"opt{k}.state{j}.{kk}"] = v
        return t

    before = {k: v.clone() for k, v in live_state().items()}
    if a.eager_kernel:
        from arena_amd.ops import _ext, fused
        ext = _ext.load()
        xj = torch.randn(16, 64, 28, 28, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        wj = torch.randn(64, 64, 3, 3, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        for _ in range(a.eager_n):
            if a.eager_kernel == "conv_fwd":
                conv.conv2d_fwd(xj, wj, 1, 1, 3, with_stats=True)
            elif a.eager_kernel == "conv_wgrad":
                conv.conv2d_wgrad(xj, xj, (3, 3), 1, 1, 3, 0)
            elif a.eager_kernel == "flip":
                conv.flip_weight(wj)
            elif a.eager_kernel == "bn":
                from arena_amd.ops.batchnorm import BatchNormAct2d
                bnm = BatchNormAct2d(64).to(dev)
                bnm(xj)
            elif a.eager_kernel == "foreach":   # torch multi-tensor kernels: ~4 KB of kernargs
                ts = [torch.randn(4096, device=dev) for _ in range(60)]
                torch._foreach_add_(ts, 1.0)
                torch._foreach_mul_(ts, 0.5)
            elif a.eager_kernel == "torch_small":   # plain elementwise kernels, small args
                t = torch.randn(1 << 20, device=dev)
                for _ in range(3):
                    t = t * 1.0001 + 0.5
            elif a.eager_kernel == "sgd":
                ps = [torch.randn(64 * 64, device=dev).to(torch.bfloat16) for _ in range(60)]
                m = torch.zeros(60 * 64 * 64, device=dev)
                fused.mt_sgd_master(ps, [i * 4096 for i in range(60)], m, m.clone(),
                                    torch.zeros(60 * 4096, device=dev, dtype=torch.bfloat16),
                                    lr=0.1, momentum=0.9, weight_decay=0.0)
        torch.cuda.synchronize()
        print(f"{a.eager_n} eager {a.eager_kernel} launches done", flush=True)
    if a.second_model:
        conv.set_mode(a.second_model)
        saved_ok = batchnorm.kernel_ok
        if a.second_bn_ref:
            batchnorm.kernel_ok = lambda *args, **kw: False
        m2, o2, x2, y2 = cnn_bench.build(args, dev, 1)
        for _ in range(4):
            cnn_bench.train_step(m2, o2, x2, y2, torch.bfloat16)
        torch.cuda.synchronize()
        batchnorm.kernel_ok = saved_ok
        print(f"second model trained eagerly ({a.second_model}); model 1 nonfinite {finite()}",
              flush=True)
        changed = [k for k, v in live_state().items() if not torch.equal(v, before[k])]
        print(f"model 1 live tensors changed by the second model: {changed[:10]} "
              f"({len(changed)} of {len(before)})", flush=True)
    keep = None
    if a.second_graph:
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2):
            t = [torch.full((1 << k,), float("nan"), device=dev) for k in range(10, 28)]
            t2 = [u * 2 for u in t]
        g2.replay()
        torch.cuda.synchronize()
        keep = (g2, t2)
    n = int(a.junk_gb * (1 << 30) / 4)
    chunks = []
    for _ in range(4):   # several sizes, so freed blocks of many size classes get overwritten
        chunks.append(torch.full((n // 4,), float("nan"), device=dev))
    small = [torch.full((1 << k,), float("nan"), device=dev) for k in range(10, 26)]
    torch.cuda.synchronize()
    del chunks, small
    for k in range(1, 4):
        g.replay()
        torch.cuda.synchronize()
        print(f"replay {k}: loss {float(loss):.4f} nonfinite {finite()}", flush=True)
    del keep
    hvd.shutdown()


if __name__ == "__main__":
    main()
