#!/usr/bin/env python3
"""Parameter gradients of the tiny ResNet with the fused cross-entropy vs F.cross_entropy (debug)."""
import os
import sys
import types

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from arena_amd.examples import cnn_bench  # noqa: E402
from arena_amd.ops import conv  # noqa: E402
from arena_amd.ops.pool import cross_entropy  # noqa: E402

conv.set_mode("ours")
args = types.SimpleNamespace(model="resnet_tiny", data_format="NHWC", batch_size=8, image_size=32,
                             num_classes=10, width=64, learning_rate=0.05, momentum=0.9,
                             weight_decay=1e-3, bucket_mb=0.05, comm="xgmi", master_weights="auto",
                             dtype="bf16")
dev = torch.device("cuda", 0)
model, opt, x, y = cnn_bench.build(args, dev, 1)
params = list(model.parameters())
out = {}
for name in ("torch", "fused", "torch2"):
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        logits = model(x)
        if name != "fused":
            loss = torch.nn.functional.cross_entropy(logits, y)
    if name == "fused":
        loss = cross_entropy(logits, y)
    print(name, float(loss), logits.dtype, logits.shape, logits.is_contiguous())
    out[name] = [g.float() for g in torch.autograd.grad(loss, params)]
for other in ("fused", "torch2"):
    worst = max((float((a - b).abs().max() / (b.abs().max() + 1e-12)), i, tuple(params[i].shape))
                for i, (a, b) in enumerate(zip(out[other], out["torch"])))
    print(other, "vs torch worst rel", worst)
