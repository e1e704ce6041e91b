"""MNIST-shaped datasets for the bundled reference workloads.

The reference's demo jobs train TF MNIST models on data pulled from the network or a PVC
(`docs/userguide/1-tfjob-standalone.md:178-186`, `4-tfjob-distributed-data.md:6-40`). There is no
network here, so two sources are supported:

* real MNIST IDX files (``train-images-idx3-ubyte[.gz]`` ...) from a mounted ``--data`` dir;
* a deterministic **synthetic MNIST**: 28x28 uint8 digit glyphs rendered from stroke skeletons
  under random affine warps, stroke jitter, thickness, distractor strokes and pixel noise. It has
  MNIST's shapes, dtypes and sizes (60k/10k) and is hard enough that a 784-500-10 MLP lands in the
  same ~97-98 % band as on real MNIST (so accuracy parity with BASELINE.md is meaningful).
"""
from __future__ import annotations

import gzip
import math
import os
import struct
from dataclasses import dataclass

import numpy as np
import torch

IMG = 28

# Stroke skeletons in a unit box (x right, y down); each digit is a list of polylines.
def _circle(cx, cy, rx, ry, n=14, a0=0.0, a1=2 * math.pi):
    return [(cx + rx * math.cos(a0 + (a1 - a0) * i / n), cy + ry * math.sin(a0 + (a1 - a0) * i / n))
            for i in range(n + 1)]


_GLYPHS = {
    0: [_circle(0.5, 0.5, 0.22, 0.33)],
    1: [[(0.38, 0.27), (0.52, 0.15), (0.52, 0.85)], [(0.4, 0.85), (0.64, 0.85)]],
    2: [[(0.27, 0.3), (0.36, 0.18), (0.55, 0.15), (0.7, 0.26), (0.69, 0.42), (0.27, 0.85),
         (0.76, 0.85)]],
    3: [[(0.27, 0.2), (0.58, 0.14), (0.7, 0.29), (0.46, 0.48), (0.71, 0.62), (0.64, 0.81),
         (0.27, 0.85)]],
    4: [[(0.62, 0.85), (0.62, 0.14), (0.25, 0.62), (0.77, 0.62)]],
    5: [[(0.71, 0.15), (0.31, 0.15), (0.28, 0.46), (0.56, 0.42), (0.71, 0.6), (0.61, 0.82),
         (0.27, 0.82)]],
    6: [[(0.66, 0.15), (0.38, 0.38), (0.28, 0.64), (0.44, 0.85), (0.66, 0.76), (0.67, 0.56),
         (0.46, 0.49), (0.3, 0.62)]],
    7: [[(0.25, 0.16), (0.76, 0.16), (0.44, 0.86)], [(0.42, 0.5), (0.66, 0.5)]],
    8: [_circle(0.5, 0.31, 0.17, 0.16), _circle(0.5, 0.67, 0.2, 0.19)],
    9: [_circle(0.49, 0.34, 0.18, 0.18), [(0.67, 0.34), (0.62, 0.86)]],
}


def _segments():
    segs = []
    for d in range(10):
        s = []
        for line in _GLYPHS[d]:
            s += [(line[i], line[i + 1]) for i in range(len(line) - 1)]
        segs.append(s)
    smax = max(len(s) for s in segs)
    A = np.full((10, smax, 2), 50.0, np.float32)
    B = np.full((10, smax, 2), 50.0, np.float32)
    for d, s in enumerate(segs):
        for j, (a, b) in enumerate(s):
            A[d, j] = a
            B[d, j] = b
    return torch.from_numpy(A), torch.from_numpy(B)


def render_synthetic(n: int, seed: int, device="cpu", chunk: int = 2000):
    """Render ``n`` synthetic digits. Returns (images uint8 [n, 784], labels uint8 [n])."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    A0, B0 = _segments()
    labels = torch.randint(0, 10, (n,), generator=g)
    ys, xs = torch.meshgrid(torch.arange(IMG), torch.arange(IMG), indexing="ij")
    pix = torch.stack([(xs.reshape(-1) + 0.5) / IMG, (ys.reshape(-1) + 0.5) / IMG], -1)  # [784,2]
    out = torch.empty(n, IMG * IMG, dtype=torch.uint8)
    for s0 in range(0, n, chunk):
        lab = labels[s0:s0 + chunk]
        b = lab.numel()
        A = A0[lab].clone()
        B = B0[lab].clone()
        S = A.shape[1]
        # per-sample affine: rotation, anisotropic scale, shear, translation (about the centre)
        th = (torch.rand(b, generator=g) - 0.5) * math.radians(26)
        sx = 0.82 + 0.3 * torch.rand(b, generator=g)
        sy = 0.82 + 0.3 * torch.rand(b, generator=g)
        sh = (torch.rand(b, generator=g) - 0.5) * 0.4
        tx = (torch.rand(b, generator=g) - 0.5) * 0.18
        ty = (torch.rand(b, generator=g) - 0.5) * 0.18
        c, s_ = torch.cos(th), torch.sin(th)
        m00, m01 = c * sx, (c * sh - s_) * sy
        m10, m11 = s_ * sx, (s_ * sh + c) * sy

        def warp(P):
            x = P[..., 0] - 0.5
            y = P[..., 1] - 0.5
            jit = 0.028 * torch.randn(P.shape[:-1] + (2,), generator=g)
            nx = m00[:, None] * x + m01[:, None] * y + 0.5 + tx[:, None] + jit[..., 0]
            ny = m10[:, None] * x + m11[:, None] * y + 0.5 + ty[:, None] + jit[..., 1]
            return torch.stack([nx, ny], -1)

        far = A[..., 0] > 10
        A = torch.where(far[..., None], A, warp(A))
        B = torch.where(far[..., None], B, warp(B))
        # distractor stroke on ~35 % of samples
        dA = torch.rand(b, 1, 2, generator=g)
        dB = dA + (torch.rand(b, 1, 2, generator=g) - 0.5) * 0.45
        use = (torch.rand(b, 1, 1, generator=g) < 0.35)
        dA = torch.where(use, dA, torch.full_like(dA, 50.0))
        dB = torch.where(use, dB, torch.full_like(dB, 50.0))
        A = torch.cat([A, dA], 1)
        B = torch.cat([B, dB], 1)
        thick = (0.04 + 0.05 * torch.rand(b, 1, generator=g))
        P = pix.to(device)[None, None]                       # [1,1,784,2]
        Ad, Bd = A.to(device)[:, :, None], B.to(device)[:, :, None]  # [b,S+1,1,2]
        AB = Bd - Ad
        t = (((P - Ad) * AB).sum(-1) / (AB * AB).sum(-1).clamp_min(1e-8)).clamp(0, 1)
        d = ((Ad + t[..., None] * AB) - P).norm(dim=-1).min(dim=1).values  # [b,784]
        gain = 0.75 + 0.25 * torch.rand(b, 1, generator=g)
        inten = (1.0 - ((d - thick.to(device)) / 0.035).clamp_min(0)).clamp(0, 1) * gain.to(device)
        inten = inten + 0.06 * torch.randn(b, IMG * IMG, generator=g).to(device)
        out[s0:s0 + b] = (inten.clamp(0, 1) * 255.0).round().to(torch.uint8).cpu()
        del S
    return out, labels.to(torch.uint8)


# ----------------------------------------------------------------------------------------------
# IDX reader (real MNIST from a mounted dataset directory)
# ----------------------------------------------------------------------------------------------
def _open(path):
    return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")


def read_idx(path: str) -> np.ndarray:
    with _open(path) as f:
        zero, dtype_code, ndim = struct.unpack(">HBB", f.read(4))
        if zero != 0 or dtype_code != 0x08:
            raise ValueError(f"{path}: not a uint8 IDX file")
        dims = struct.unpack(">" + "I" * ndim, f.read(4 * ndim))
        data = np.frombuffer(f.read(), dtype=np.uint8)
    return data.reshape(dims)


def _find(data_dir: str, stem: str):
    for name in (stem, stem + ".gz", stem.replace("-idx", ".idx"), stem.replace("-idx", ".idx") + ".gz"):
        p = os.path.join(data_dir, name)
        if os.path.exists(p):
            return p
    return None


@dataclass
class MNIST:
    train_images: torch.Tensor  # uint8 [60000, 784]
    train_labels: torch.Tensor  # uint8 [60000]
    test_images: torch.Tensor   # uint8 [10000, 784]
    test_labels: torch.Tensor   # uint8 [10000]
    source: str

    def to(self, device) -> "MNIST":
        return MNIST(self.train_images.to(device), self.train_labels.to(device),
                     self.test_images.to(device), self.test_labels.to(device), self.source)


def load_mnist(data_dir: str | None = None, n_train: int = 60000, n_test: int = 10000,
               seed: int = 1234, cache_dir: str | None = None) -> MNIST:
    """Real MNIST from ``data_dir`` when the IDX files are there, else synthetic MNIST."""
    if data_dir:
        ti = _find(data_dir, "train-images-idx3-ubyte")
        tl = _find(data_dir, "train-labels-idx1-ubyte")
        vi = _find(data_dir, "t10k-images-idx3-ubyte")
        vl = _find(data_dir, "t10k-labels-idx1-ubyte")
        if ti and tl and vi and vl:
            return MNIST(torch.from_numpy(read_idx(ti).reshape(-1, 784).copy())[:n_train],
                         torch.from_numpy(read_idx(tl).copy())[:n_train],
                         torch.from_numpy(read_idx(vi).reshape(-1, 784).copy())[:n_test],
                         torch.from_numpy(read_idx(vl).copy())[:n_test], "mnist-idx:" + data_dir)
    cache_dir = cache_dir or os.environ.get("ARENA_DATA_CACHE",
                                            os.path.join(os.path.expanduser("~"), ".cache", "arena_amd"))
    path = os.path.join(cache_dir, f"synthetic_mnist_{n_train}_{n_test}_{seed}.npz")
    if os.path.exists(path):
        z = np.load(path)  # arrays only (allow_pickle=False default)
        return MNIST(torch.from_numpy(z["xi"]), torch.from_numpy(z["yi"]),
                     torch.from_numpy(z["xt"]), torch.from_numpy(z["yt"]), "synthetic")
    xi, yi = render_synthetic(n_train, seed)
    xt, yt = render_synthetic(n_test, seed + 1)
    try:
        os.makedirs(cache_dir, exist_ok=True)
        tmp = path + f".tmp{os.getpid()}.npz"
        np.savez(tmp, xi=xi.numpy(), yi=yi.numpy(), xt=xt.numpy(), yt=yt.numpy())
        os.replace(tmp, path)
    except OSError:
        pass
    return MNIST(xi, yi, xt, yt, "synthetic")
