#!/usr/bin/env python3
"""Per-kernel steady-state cost: each op is captured REPS times into one hipGraph and replayed;
time per launch = graph time / REPS (includes the dependent-kernel boundary, like the real step).
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from arena_amd import ops  # noqa: E402
from arena_amd.data.mnist import render_synthetic  # noqa: E402
from arena_amd.models.mlp import FusedMLPTrainer, MLPConfig  # noqa: E402

REPS = 200


def bench(fn, reps=REPS, iters=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(iters):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


def main():
    x, y = render_synthetic(6000, 1)
    tr = FusedMLPTrainer(MLPConfig(), x, y, device="cuda")
    tiny = torch.zeros(1, device="cuda")
    res = {}
    res["torch_fill_1elem"] = bench(lambda: tiny.fill_(1.0))
    A, Bc, cfg, B = tr.ctrA, tr.ctrB, tr.cfg, tr.cfg.batch

    def fwd():
        ops.linear_fwd(tr.train_x, tr.W1, tr.Hbuf, tr.b1, x_scale=1 / 255.0, idx=tr.perm,
                       cursor=A, batch=B, act=1, keep_prob=cfg.keep_prob, seed=1, step=A)

    dZ = torch.empty_like(tr.Hbuf)

    def head():
        ops.xent_head(tr.Hbuf, tr.W2, tr.b2, tr.train_y, loss_acc=tr.loss_hist,
                      correct_acc=tr.corr_hist, idx=tr.perm, cursor=A, batch=B,
                      dlogits=tr.dlogits, dZ=dZ, keep_prob=cfg.keep_prob, relu_mask=True,
                      loss_scale=1.0 / B, hist_step=A, ctr_dst=Bc, ctr_src=A, ctr_add=0)

    def head_nograd():
        ops.xent_head(tr.Hbuf, tr.W2, tr.b2, tr.train_y, loss_acc=tr.loss_hist,
                      correct_acc=tr.corr_hist, idx=tr.perm, cursor=A, batch=B,
                      keep_prob=cfg.keep_prob, relu_mask=True, loss_scale=1.0 / B, hist_step=A)

    def wgrad_adam():
        ops.wgrad_grouped([tr.train_x, tr.Hbuf], [dZ, tr.dlogits], [tr.W1, tr.W2],
                          [tr.b1, tr.b2], mode=1, mW=[tr.mW1, tr.mW2], vW=[tr.vW1, tr.vW2],
                          mB=[tr.mb1, tr.mb2], vB=[tr.vb1, tr.vb2], x_scales=[1 / 255.0, 1.0],
                          gather=[True, False], idx=tr.perm, cursor=Bc, cursor_off=-1, batch=B,
                          lr=1e-9, t_step=Bc)

    G = torch.zeros_like(tr.P)
    L = tr.layout
    gW1, gb1, gW2, gb2 = (L.view(G, n) for n in ("W1", "b1", "W2", "b2"))

    def wgrad_grad():
        ops.wgrad_grouped([tr.train_x, tr.Hbuf], [dZ, tr.dlogits], [gW1, gW2], [gb1, gb2],
                          mode=0, x_scales=[1 / 255.0, 1.0], gather=[True, False], idx=tr.perm,
                          cursor=Bc, cursor_off=-1, batch=B)

    def wgrad_l1_only():
        ops.wgrad_grouped([tr.train_x], [dZ], [gW1], [gb1], mode=0, x_scales=[1 / 255.0],
                          gather=[True], idx=tr.perm, cursor=Bc, cursor_off=-1, batch=B)

    def adam():
        ops.adam_flat(tr.P, tr.M, tr.V, G, lr=1e-9, t_step=Bc)

    xf = (tr.train_x[:B].float() / 255.0).contiguous()
    xu = tr.train_x[:B].contiguous()
    yb = tr.train_y[:B].contiguous()

    def fwd_f32_nogather():
        ops.linear_fwd(xf, tr.W1, tr.Hbuf, tr.b1, act=1, keep_prob=cfg.keep_prob, seed=1, step=A)

    def fwd_u8_nogather_nodrop():
        ops.linear_fwd(xu, tr.W1, tr.Hbuf, tr.b1, x_scale=1 / 255.0, act=1)

    def head_nogather():
        ops.xent_head(tr.Hbuf, tr.W2, tr.b2, yb, loss_acc=tr.loss_hist, correct_acc=tr.corr_hist,
                      dlogits=tr.dlogits, dZ=dZ, keep_prob=cfg.keep_prob, relu_mask=True,
                      loss_scale=1.0 / B)

    def wgrad_l1_nogather():
        ops.wgrad_grouped([xu], [dZ], [gW1], [gb1], mode=0, x_scales=[1 / 255.0],
                          gather=[False])

    def wgrad_l2_only():
        ops.wgrad_grouped([tr.Hbuf], [tr.dlogits], [gW2], [gb2], mode=0, x_scales=[1.0],
                          gather=[False])

    Bc.fill_(1)
    for name, fn in [("fwd_f32_nogather", fwd_f32_nogather),
                     ("fwd_u8_nogather_nodrop", fwd_u8_nogather_nodrop),
                     ("head_nogather", head_nogather), ("wgrad_l1_nogather", wgrad_l1_nogather),
                     ("wgrad_l2_only", wgrad_l2_only),("linear_fwd", fwd), ("xent_head", head), ("xent_head_nograd", head_nograd),
                     ("wgrad_adam", wgrad_adam), ("wgrad_grad", wgrad_grad),
                     ("wgrad_l1_grad", wgrad_l1_only), ("adam_flat", adam)]:
        res[name] = bench(fn)
    def fused_fwd_head():
        tr._launch_fwd_head()

    def fused_wgrad_adam():
        tr._launch_wgrad(adam=True)

    res["fused_fwd_head"] = bench(fused_fwd_head)
    res["fused_wgrad_adam"] = bench(fused_wgrad_adam)
    tr.enable_graphs(60)
    res["full_step"] = bench(lambda: tr._launch_step(), reps=60)
    for k, v in res.items():
        print(f"{k:22s} {v:8.2f} us")
    print(json.dumps({k: round(v, 3) for k, v in res.items()}))


if __name__ == "__main__":
    main()
