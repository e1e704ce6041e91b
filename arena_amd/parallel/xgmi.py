"""Intra-node xGMI collectives (hipIpc peer memory) with an automatic RCCL fallback.

The Horovod-equivalent gradient path of SURVEY §2.10/§2.12 ("xGMI one-/two-shot allreduce with
RCCL fallback"). Kernels live in csrc/ccl/xgmi_ccl.hip; this module owns the registered memory:

* every rank allocates a staging buffer (and optionally a parameter buffer) with hipMalloc and a
  flag buffer in uncached memory, exports hipIpc handles, and exchanges them over the process
  group (gloo or RCCL) with ``all_gather_object``;
* ``all_reduce_`` = one kernel. Two-shot above 64 KB: copy-in, barrier, reduce own chunk from all
  W ranks (W-1 xGMI links read in parallel), write it to all ranks, barrier, copy-out. One-shot up
  to 64 KB: stage into a double-buffered tail, barrier, read the whole vector from all ranks and
  reduce locally (one barrier instead of two: latency-bound sizes);
* ``adam_`` = reduce-scatter of the gradient + Adam on the owned chunk + all-gather of the
  updated parameters, in one kernel (ZeRO-1-style sharded optimizer state);
* ``broadcast_`` / ``all_gather`` = one copy kernel each (direct pull or scatter + all-gather for
  broadcast; every rank pulls every shard for all-gather), any dtype (moved as raw 4-byte words);
* construction runs a self-test on every rank and agrees on the outcome over the process group,
  so either ALL ranks use xGMI or all fall back to RCCL (never a split decision). Barrier waits are
  bounded in-kernel; a timeout sets an error flag that ``check()`` raises on.

Only meaningful on a single node (all ranks' GPUs in one xGMI hive, mapped into every rank's
process). ``usable()`` establishes that collectively: every rank reports its host (name + boot
id), its own GPU and the GPUs it can see, and xGMI is used only if all ranks share the host and
each rank's GPU is visible to every other rank -- true for the local backend's ranks, false for
K8s pods (one device-plugin allocation per pod) or multi-node jobs, which then use RCCL.
"""
from __future__ import annotations

import os
import socket
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import _ext
from ..utils.logs import get_logger

log = get_logger("xgmi")


class XgmiUnavailable(RuntimeError):
    pass


def _sig_bytes(ext) -> int:
    return getattr(ext, "ccl_phases", 2) * ext.ccl_max_blocks * ext.ccl_max_ranks * 4


def _device_id(i: int) -> str:
    p = torch.cuda.get_device_properties(i)
    uuid = getattr(p, "uuid", None)
    if uuid is not None and str(uuid).strip("0-"):
        return str(uuid)
    bus = getattr(p, "pci_bus_id", None)
    return f"pci:{getattr(p, 'pci_domain_id', 0)}:{bus}" if bus is not None else ""


def host_identity() -> dict:
    """What decides whether two ranks can map each other's GPU memory (see module doc)."""
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        boot = ""
    ident = {"host": socket.gethostname(), "boot": boot, "own": "", "visible": []}
    if torch.cuda.is_available():
        try:
            ident["visible"] = [_device_id(i) for i in range(torch.cuda.device_count())]
            ident["own"] = ident["visible"][torch.cuda.current_device()]
        except Exception:  # noqa: BLE001 - no identity: the visibility check is skipped
            ident["own"], ident["visible"] = "", []
    return ident


def identities_share_node(infos: List[dict]) -> bool:
    """True iff every rank runs on one host (same name and boot) and, where GPU identities are
    known, each rank's own GPU is visible in every rank's process."""
    if not infos or len({(i.get("host"), i.get("boot")) for i in infos}) != 1:
        return False
    owns = [i.get("own") for i in infos]
    if all(owns):
        if len(set(owns)) != len(owns) and len(set(owns)) != 1:
            return False          # some ranks share a GPU and others do not: not a layout we map
        for i in infos:
            vis = set(i.get("visible") or [])
            if not all(o in vis for o in owns):
                return False
    return True


def same_node(group=None) -> bool:
    """Collective: gather every rank's :func:`host_identity` and check
    :func:`identities_share_node` (identical answer on all ranks)."""
    w = dist.get_world_size(group)
    infos: List[Optional[dict]] = [None] * w
    dist.all_gather_object(infos, host_identity(), group=group)
    return identities_share_node(infos)


def usable(group=None) -> bool:
    """Same-node world of 2..8 GPU ranks with the native extension present on every rank.
    Collective over ``group`` (all ranks must call it) once the cheap env checks pass."""
    if os.environ.get("ARENA_XGMI", "1") == "0":
        return False
    if not dist.is_initialized():
        return False
    w = dist.get_world_size(group)
    if not 2 <= w <= 8:
        return False
    local = os.environ.get("LOCAL_WORLD_SIZE")
    if local is not None and int(local) != int(os.environ.get("WORLD_SIZE", w)):
        return False  # multi-node job: inter-node traffic belongs to RCCL
    ok = bool(torch.cuda.is_available() and _ext.available())
    infos: List[Optional[dict]] = [None] * w
    dist.all_gather_object(infos, {"ok": ok, **host_identity()}, group=group)
    return all(i["ok"] for i in infos) and identities_share_node(infos)


def _words(t: torch.Tensor) -> Optional[torch.Tensor]:
    """1-D float32 view of a dense tensor's bytes (any dtype), or None when its size or address
    is not a multiple of 16 bytes (the kernels move float4 words)."""
    if not t.is_contiguous() or t.numel() == 0:
        return None
    nbytes = t.numel() * t.element_size()
    if nbytes % 16 or t.data_ptr() % 16:
        return None
    return t.reshape(-1).view(torch.uint8).view(torch.float32)


def _round4(n: int) -> int:
    return (n + 3) // 4 * 4


class XgmiComm:
    def __init__(self, group=None, staging_elems: int = 8 << 20, param_elems: int = 0,
                 timeout_s: float = 20.0, selftest: bool = True):
        if not dist.is_initialized():
            raise XgmiUnavailable("torch.distributed is not initialised")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if not 2 <= self.world <= 8:
            raise XgmiUnavailable(f"world size {self.world} outside 2..8")
        ext = _ext.load()
        self.ext = ext
        self.device = torch.cuda.current_device()
        # ranks sharing one GPU (same-device rehearsals): their launches must fit on it together,
        # so each collective launch gets at most 128 / W blocks (csrc/ccl/xgmi_ccl.hip
        # g_max_blocks; the same cap on every rank, so the block geometries still match)
        devs: List[Optional[str]] = [None] * self.world
        dist.all_gather_object(devs, _device_id(self.device), group=group)
        self.shared_gpu = len(set(devs)) < self.world and all(devs)
        if hasattr(ext, "ccl_set_max_blocks"):
            ext.ccl_set_max_blocks(max(4, 128 // self.world) if self.shared_gpu
                                   else ext.ccl_max_blocks)
        self.staging_elems = _round4(staging_elems)
        self.param_elems = _round4(param_elems) if param_elems else 0
        self._own, self._opened = [], []
        ok = 1
        err_msg = ""
        handles = {}
        try:
            # staging floats + the one-shot kernel's double-buffered tail right behind them
            buf_bytes = (self.staging_elems + 2 * ext.ccl_oneshot_elems) * 4
            buf = ext.ccl_malloc(buf_bytes, False)
            self._own.append(buf)
            sig = ext.ccl_malloc(_sig_bytes(ext), True)
            self._own.append(sig)
            ext.ccl_memset(sig, 0, _sig_bytes(ext))
            ext.ccl_memset(buf, 0, buf_bytes)
            handles = {"buf": ext.ccl_ipc_get(buf), "sig": ext.ccl_ipc_get(sig)}
            local = {"buf": buf, "sig": sig}
            if self.param_elems:
                b2 = ext.ccl_malloc(self.param_elems * 4, False)
                self._own.append(b2)
                ext.ccl_memset(b2, 0, self.param_elems * 4)
                handles["buf2"] = ext.ccl_ipc_get(b2)
                local["buf2"] = b2
        except Exception as e:  # noqa: BLE001
            ok, err_msg = 0, repr(e)
        allh = [None] * self.world
        dist.all_gather_object(allh, (ok, handles), group=group)
        if not all(h[0] for h in allh):
            self._free()
            raise XgmiUnavailable(f"allocation failed on some rank ({err_msg})")
        ptrs = {k: [0] * self.world for k in handles}
        try:
            for r in range(self.world):
                for k in handles:
                    if r == self.rank:
                        ptrs[k][r] = local[k]
                    else:
                        p = ext.ccl_ipc_open(allh[r][1][k])
                        self._opened.append(p)
                        ptrs[k][r] = p
        except Exception as e:  # noqa: BLE001
            ok, err_msg = 0, repr(e)
        self._epoch = torch.zeros(ext.ccl_max_blocks, dtype=torch.int32, device="cuda")
        self._err = torch.zeros(1, dtype=torch.int32, device="cuda")
        self._ptrs = ptrs
        self.selftest_result: dict = {}
        self.form = "pull"
        if ok:
            self.peers = ext.XgmiPeers(ptrs["buf"], ptrs.get("buf2", []), ptrs["sig"], self._epoch,
                                       self._err, self.staging_elems, self.param_elems, self.rank,
                                       float(timeout_s))
            self._buf = ext.ccl_tensor(local["buf"], self.staging_elems, self.device)
            self._buf2 = (ext.ccl_tensor(local["buf2"], self.param_elems, self.device)
                          if self.param_elems else None)
        torch.cuda.synchronize()
        self._agree(ok, f"hipIpc mapping failed: {err_msg}")
        if selftest:
            self._selftest_all()

    # --------------------------------------------------------------------------------- setup
    def _agree(self, ok: int, why: str) -> None:
        """All ranks learn whether every rank succeeded (so they fall back together)."""
        flags = [None] * self.world
        dist.all_gather_object(flags, int(ok), group=self.group)
        if not all(flags):
            self.close()
            raise XgmiUnavailable(why if not ok else "a peer rank failed")

    def _selftest_all(self) -> None:
        """Run every kernel kind this communicator will serve on known data and agree on the
        outcome collectively. The pull form (the default: no kernel stores into a peer's buffer) is
        tested unless ``ARENA_XGMI_PUSH=1`` asks for the push form, which is kept only if ITS test
        passes on every rank (otherwise the pull form is tested and used). Any pull failure raises
        :class:`XgmiUnavailable` on every rank, so callers fall back to RCCL at construction
        instead of meeting a bad kernel mid-run. Result: ``selftest_result`` {kernel: "ok" or the
        failure}, ``form`` ("pull" / "push")."""
        forms = ["push", "pull"] if os.environ.get("ARENA_XGMI_PUSH", "0") == "1" else ["pull"]
        for form in forms:
            self.peers.push = form == "push"
            res = self._selftest()
            everyone = [None] * self.world
            dist.all_gather_object(everyone, res, group=self.group)
            merged = {}
            for r, d in enumerate(everyone):
                for k, v in d.items():
                    if v != "ok" and k not in merged:
                        merged[k] = f"rank {r}: {v}"
                    merged.setdefault(k, "ok")
            self.selftest_result = merged
            bad = [k for k, v in merged.items() if v != "ok"]
            if not bad:
                self.form = form
                log.info("xGMI self-test passed (%s form): %s", form, ", ".join(merged))
                return
            log.warning("xGMI self-test of the %s form failed: %s", form,
                        "; ".join(f"{k}: {merged[k]}" for k in bad))
            if "timeout" in bad:
                break       # a barrier timed out: the flag protocol itself is broken
        self.peers.push = False
        self.close()
        raise XgmiUnavailable("xGMI self-test failed: " + "; ".join(
            f"{k}: {v}" for k, v in self.selftest_result.items() if v != "ok"))

    def _peer_view(self, key: str, r: int, n: int) -> torch.Tensor:
        return self.ext.ccl_tensor(self._ptrs[key][r], n, self.device)

    def _gate(self) -> None:
        """Every rank's inputs are ready and every rank is here: launch the next self-test
        kernel together. Without it a rank spins in a kernel's barrier while a peer is still
        loading code objects for its first torch ops -- with several ranks sharing one GPU, long
        enough to hit the barrier timeout."""
        torch.cuda.synchronize()
        dist.barrier(group=self.group)

    def _prewarm(self) -> None:
        """Read every rank's registered buffers through this rank's mappings, so any line that
        could go stale (a peer's data cached in this GPU's L2, or this rank's own lines) is
        resident before the kernel under test runs."""
        acc = torch.zeros((), device="cuda")
        for key, n in (("buf", self.staging_elems), ("buf2", self.param_elems)):
            if key in self._ptrs and n:
                for r in range(self.world):
                    acc += self._peer_view(key, r, n).sum()
        torch.cuda.synchronize()

    def _selftest(self) -> dict:
        """One pass over every kernel kind; returns {kernel: "ok" | reason}. Inputs are small
        integers (sums exact in fp32 whatever the order) and the optimizer steps use
        power-of-two coefficients, so the expected results are bit-exact."""
        res = {}
        W, rk = self.world, self.rank
        tot = W * (W + 1) // 2

        def run(name, fn):
            try:
                self._prewarm()
                ok = fn()
                torch.cuda.synchronize()
                res[name] = "ok" if ok else "mismatch"
                if int(self._err.item()):   # attribute a barrier timeout to its kernel
                    res[name] = "barrier timeout"
                    self._err.zero_()
            except Exception as e:  # noqa: BLE001
                res[name] = repr(e)[:200]

        cap = self.staging_elems
        big = min(cap, 300004) // 4 * 4
        oneshot_max = self.ext.ccl_get_oneshot_max()

        def allreduce(n):
            base = torch.arange(n, device="cuda", dtype=torch.float32) % 977
            for it in range(2):                      # second call reads lines the first cached
                out = torch.empty(n, device="cuda")
                inp = base * (rk + 1 + it)
                self._gate()
                self.all_reduce_(inp, out=out)
                if not torch.equal(out, base * (tot + W * it)):
                    return False
            stage = self._buf[:n]                    # zero-copy, in place on the staging buffer
            stage.copy_(base * (rk + 1))
            self._gate()
            self.all_reduce_(stage)
            return bool(torch.equal(stage, base * tot))

        run("allreduce_oneshot", lambda: allreduce(min(1000, cap) // 4 * 4 or 4))
        if big > oneshot_max:
            run("allreduce_twoshot", lambda: allreduce(big))

        def bcast(n):
            for root in (0, W - 1):
                t = (torch.arange(n, device="cuda", dtype=torch.float32) % 101) * (root + 3)
                x = t.clone() if rk == root else torch.full((n,), -1.0, device="cuda")
                self._gate()
                self.broadcast_(x, root=root)
                if not torch.equal(x, t):
                    return False
            return True

        run("broadcast_direct", lambda: bcast(min(1000, cap) // 4 * 4 or 4))
        if W > 2 and big > (128 << 10):
            run("broadcast_twoshot", lambda: bcast(big))

        def allgather():
            m = min(4096, cap)
            x = torch.arange(m, device="cuda", dtype=torch.float32) + 10000 * rk
            self._gate()
            got = self.all_gather(x)
            want = torch.stack([torch.arange(m, device="cuda", dtype=torch.float32) + 10000 * q
                                for q in range(W)])
            return bool(torch.equal(got, want))

        run("allgather", allgather)
        if self.param_elems:
            run("adam", self._selftest_adam)
            run("sgd_bf16", self._selftest_sgd_bf16)
            run("sgd_f32", self._selftest_sgd_f32)
        if int(self._err.item()):
            res["timeout"] = "a barrier wait timed out during the self-test"
            self._err.zero_()
        # leave the registered buffers as construction made them
        self._buf.zero_()
        if self._buf2 is not None:
            self._buf2.zero_()
        torch.cuda.synchronize()
        return res

    def _grad_rows(self, n: int, step: int, scale: float = 1.0):
        """Every rank's gradient for ``step`` (deterministic, identical on all ranks)."""
        i = torch.arange(n, device="cuda", dtype=torch.float32)
        return [((i * (q + 3) + 7 * step) % 17 - 8) * scale for q in range(self.world)]

    def _selftest_adam(self) -> bool:
        from ..ops import fused
        n = min(self.staging_elems, self.param_elems, 1 << 16) // 4 * 4
        P0 = (torch.arange(n, device="cuda", dtype=torch.float32) % 31) + 100.0
        Pref, Mref, Vref = P0.clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
        M, V = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
        self._buf2[:n].copy_(P0)
        for step in range(1, 3):
            g = self._grad_rows(n, step)
            gsum = g[0].clone()
            for x in g[1:]:
                gsum += x
            t = torch.full((1,), step, dtype=torch.int64, device="cuda")
            self._buf[:n].copy_(g[self.rank])
            self._prewarm()
            self._gate()
            self.adam_(M, V, n, lr=0.25, t_step=t)
            fused.adam_flat(Pref, Mref, Vref, gsum, lr=0.25, t_step=t)
            torch.cuda.synchronize()
            if not torch.allclose(self._buf2[:n], Pref, rtol=1e-6, atol=0):
                return False
        return True

    def _selftest_sgd_bf16(self) -> bool:
        bf = torch.bfloat16
        words = min(self.staging_elems, self.param_elems)
        off = 8 * 3                                      # a bucket that does not start at 0
        n = (min(2 * words - off, 1 << 17) // 8) * 8
        if n <= 0:
            return True
        wbf = self._buf2.view(bf)
        stage = self._buf.view(bf)
        w0 = ((torch.arange(n, device="cuda", dtype=torch.float32) % 64) - 32) * 0.125
        master = torch.zeros(off + n, device="cuda")
        mom = torch.zeros(off + n, device="cuda")
        master[off:] = w0
        wbf[off:off + n].copy_(w0.to(bf))
        ref_w, ref_m = w0.clone(), torch.zeros(n, device="cuda")
        lr, mu, wd = 2.0 ** -4, 0.5, 2.0 ** -10
        for step in range(2):
            g = self._grad_rows(n, step, 0.25)
            stage[off:off + n].copy_(g[self.rank].to(bf))
            gsum = g[0].clone()
            for x in g[1:]:
                gsum += x
            ref_m = mu * ref_m + (gsum + wd * ref_w)
            ref_w = ref_w - lr * ref_m
            self._prewarm()
            self._gate()
            self.peers.sgd_bf16(master, mom, off, n, lr, mu, wd, 1.0)
            torch.cuda.synchronize()
            if not torch.equal(wbf[off:off + n], ref_w.to(bf)):
                return False
        lo, hi = self.ext.ccl_sgd_shard(off, n, self.world, self.rank)
        return bool(torch.equal(master[lo:hi], ref_w[lo - off:hi - off]))

    def _selftest_sgd_f32(self) -> bool:
        words = min(self.staging_elems, self.param_elems)
        off = 4 * 5
        n = (min(words - off, 1 << 16) // 4) * 4
        if n <= 0:
            return True
        w0 = ((torch.arange(n, device="cuda", dtype=torch.float32) % 64) - 32) * 0.125
        self._buf2[off:off + n].copy_(w0)
        mom = torch.zeros(n, device="cuda")
        ref_w, ref_m = w0.clone(), torch.zeros(n, device="cuda")
        lr, mu, wd = 2.0 ** -4, 0.5, 2.0 ** -10
        for step in range(2):
            g = self._grad_rows(n, step, 0.25)
            self._buf[off:off + n].copy_(g[self.rank])
            gsum = g[0].clone()
            for x in g[1:]:
                gsum += x
            ref_m = mu * ref_m + (gsum + wd * ref_w)
            ref_w = ref_w - lr * ref_m
            self._prewarm()
            self._gate()
            self.peers.sgd_f32(mom, off, n, lr, mu, wd, 1.0)
            torch.cuda.synchronize()
            if not torch.equal(self._buf2[off:off + n], ref_w):
                return False
        return True

    def _free(self):
        for p in self._own:
            try:
                self.ext.ccl_free(p)
            except Exception:  # noqa: BLE001
                pass
        self._own = []

    def close(self, collective: bool = True) -> None:
        """Unmap the peers' buffers, then free this rank's. Collective by default: every rank
        unmaps before any rank frees, so no buffer is freed while a peer still maps it. (Freed
        under a live peer mapping, the next allocation could land on the same addresses, and
        exporting it then failed with ``hipIpcGetMemHandle: invalid argument`` -- seen with 8
        ranks on one GPU, where a temporary broadcast communicator is closed right before the
        optimizer's is created.)"""
        torch.cuda.synchronize()
        for p in self._opened:
            try:
                self.ext.ccl_ipc_close(p)
            except Exception:  # noqa: BLE001
                pass
        self._opened = []
        self.peers = None
        if collective and dist.is_initialized():
            dist.barrier(group=self.group)
        self._free()

    # ------------------------------------------------------------------------------- buffers
    def buffer(self) -> torch.Tensor:
        """This rank's registered staging buffer (zero-copy input for ``all_reduce_``)."""
        return self._buf

    def params(self) -> torch.Tensor:
        if self._buf2 is None:
            raise XgmiUnavailable("communicator was created without a parameter buffer")
        return self._buf2

    def shard(self, n: int):
        """[lo, hi) of the flat vector whose optimizer state this rank owns under ``adam_``."""
        lo, hi = self.ext.ccl_shard(n, self.world, self.rank)
        return lo, hi

    # ----------------------------------------------------------------------------- collectives
    def all_reduce_(self, t: torch.Tensor, scale: float = 1.0, out: Optional[torch.Tensor] = None):
        """Sum (times ``scale``) of ``t`` over ranks into ``out`` (default: in place)."""
        if t.dtype != torch.float32 or not t.is_cuda:
            raise TypeError("xGMI allreduce takes float32 GPU tensors")
        out = t if out is None else out
        src, dst = t.reshape(-1), out.reshape(-1)
        n = src.numel()
        cap = self.staging_elems
        buf = self._buf
        if (n % 4 == 0 and n <= cap and src.is_contiguous() and dst.is_contiguous()):
            self.peers.allreduce(src, dst, float(scale))
            return out
        # ragged or larger than the staging buffer: go through it in zero-padded pieces
        for s in range(0, n, cap):
            m = min(cap, n - s)
            m4 = _round4(m)
            view = buf[:m4]
            view[:m].copy_(src[s:s + m])
            if m4 != m:
                view[m:].zero_()
            self.peers.allreduce(view, view, float(scale))
            dst[s:s + m].copy_(view[:m])
        return out

    def adam_(self, M: torch.Tensor, V: torch.Tensor, n: int, *, lr: float = 1e-3,
              lr_t: Optional[torch.Tensor] = None, betas=(0.9, 0.999), eps: float = 1e-8,
              weight_decay: float = 0.0, t_step: Optional[torch.Tensor] = None,
              grad_scale: float = 1.0, tf_style: bool = False,
              ctr_dst: Optional[torch.Tensor] = None, ctr_src: Optional[torch.Tensor] = None,
              ctr_add: int = 0) -> None:
        """Gradient in ``buffer()[:n]`` -> Adam on the owned shard -> parameters in every rank's
        ``params()[:n]``."""
        self.peers.adam(M, V, int(n), float(lr), lr_t, float(betas[0]), float(betas[1]),
                        float(eps), float(weight_decay), t_step, float(grad_scale), bool(tf_style),
                        ctr_dst, ctr_src, int(ctr_add))

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        """In-place broadcast of ``t`` (any dtype) from ``root`` -- bit-exact copy."""
        if not t.is_cuda:
            raise TypeError("xGMI broadcast takes GPU tensors")
        w = _words(t)
        if w is not None and w.numel() <= self.staging_elems:
            self.peers.broadcast(w, w, int(root))
            return t
        src = t if t.is_contiguous() else t.contiguous()
        raw = src.reshape(-1).view(torch.uint8)
        stage = self._buf.view(torch.uint8)
        piece = self.staging_elems * 4
        for s0 in range(0, raw.numel(), piece):
            m = min(piece, raw.numel() - s0)
            m16 = (m + 15) // 16 * 16
            if self.rank == root:
                stage[:m].copy_(raw[s0:s0 + m])
            view = self._buf[:m16 // 4]
            self.peers.broadcast(view, view, int(root))
            if self.rank != root:
                raw[s0:s0 + m].copy_(stage[:m])
        if src is not t:
            t.copy_(src)
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """``torch.cat`` over ranks of equally shaped ``t`` along a new leading dim: returns
        [world, *t.shape] (bit-exact copies)."""
        if not t.is_cuda:
            raise TypeError("xGMI all-gather takes GPU tensors")
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        wi, wo = _words(t), _words(out)
        if wi is not None and wo is not None and wi.numel() <= self.staging_elems:
            self.peers.allgather(wi, wo)
            return out
        raw = t.contiguous().reshape(-1).view(torch.uint8)
        dst = out.view(self.world, -1).view(torch.uint8)
        stage = self._buf.view(torch.uint8)
        piece = self.staging_elems * 4
        for s0 in range(0, raw.numel(), piece):
            m = min(piece, raw.numel() - s0)
            m16 = (m + 15) // 16 * 16
            stage[:m].copy_(raw[s0:s0 + m])
            tmp = torch.empty(self.world * m16, dtype=torch.uint8, device=t.device)
            self.peers.allgather(self._buf[:m16 // 4], tmp.view(torch.float32))
            dst[:, s0:s0 + m].copy_(tmp.view(self.world, m16)[:, :m])
        return out

    def check(self) -> None:
        """Raise if any barrier wait timed out since construction (host sync)."""
        if int(self._err.item()):
            raise RuntimeError("xGMI collective: a barrier wait timed out (a peer rank stalled "
                               "or died); results since then are invalid")
