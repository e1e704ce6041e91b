"""Host-code sanitizers for the native runtime (SURVEY §5 "race detection / sanitizers").

The reference has no race detector or sanitizer build at all (Makefile:55-62, no tests). Here
every native runtime tool is built twice more -- ASan+UBSan and TSan (arena_amd/_build.py) --
and driven through its real protocol:

* arena-ps (multi-threaded TCP PS): sync rounds from two concurrent workers under TSan, async
  Adam over two shards under ASan/UBSan;
* arena-supervisor: a standalone job (success + retry after failure) and an allreduce gang
  under ASan/UBSan via the LocalBackend, with ARENA_NATIVE_SANITIZE selecting the build;
* arena-probe: a fake sysfs topology under ASan/UBSan.

A sanitizer report makes the tool exit 66 (see SANITIZER_ENV), which the tests assert against.
"""
from __future__ import annotations

import io
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

from arena_amd import _build

REPORT_MARKERS = ("ERROR: AddressSanitizer", "ERROR: LeakSanitizer", "WARNING: ThreadSanitizer",
                  "runtime error:", "SUMMARY: UndefinedBehaviorSanitizer")


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _san_env(variant: str) -> dict:
    env = dict(os.environ)
    env.update(_build.sanitizer_env(variant))
    # the runtime library must not insist on coming first in the link order when the host
    # process environment already preloads something
    for k in ("ASAN_OPTIONS", "TSAN_OPTIONS"):
        if k in env:
            env[k] += ":verify_asan_link_order=0" if k == "ASAN_OPTIONS" else ""
    env["ARENA_NATIVE_SANITIZE"] = variant
    return env


@pytest.fixture(scope="module")
def san_tools():
    try:
        _build.build_native_tools(sanitize="asan")
        _build.build_native_tools(sanitize="tsan")
    except (subprocess.CalledProcessError, OSError) as e:  # toolchain without sanitizer runtimes
        pytest.skip(f"sanitizer build unavailable: {e}")
    return True


def _start_ps(variant, port, workers, sync=False, optimizer="adam", lr=1e-3):
    argv = [_build.tool_path("arena-ps", variant), "--port", str(port), "--host", "127.0.0.1",
            "--workers", str(workers), "--optimizer", optimizer, "--lr", repr(lr)]
    if sync:
        argv.append("--sync")
    p = subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                         env=_san_env(variant))
    line = p.stdout.readline()
    if "serving" not in line:
        p.kill()
        raise AssertionError(f"sanitized arena-ps failed to start: {line}{p.stdout.read()}")
    out = []
    t = threading.Thread(target=lambda: out.extend(p.stdout), daemon=True)
    t.start()
    return p, out, t


def _finish(p, out, t, timeout=60):
    rc = p.wait(timeout=timeout)
    t.join(timeout=5)
    text = "".join(out)
    assert not any(m in text for m in REPORT_MARKERS), text
    assert rc == 0, f"rc={rc}\n{text}"


def test_ps_sync_rounds_under_tsan(san_tools):
    from arena_amd.parallel import ps as psmod
    n, rounds, lr = 4096, 25, 0.5
    port = _free_port()
    p, out, t = _start_ps("tsan", port, 2, sync=True, optimizer="sgd", lr=lr)
    try:
        clients = [psmod.PSClient([f"127.0.0.1:{port}"], n, timeout_s=30) for _ in range(2)]
        p0 = np.zeros(n, np.float32)
        clients[0].init(p0)
        clients[1].init(np.full(n, 9.0, np.float32))       # ignored: first INIT wins
        outs = [np.empty(n, np.float32) for _ in range(2)]
        errs = []

        def worker(i):
            try:
                for r in range(rounds):
                    clients[i].push_pull(np.full(n, float(i + 1), np.float32), outs[i])
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        th = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=60)
        assert not errs, errs
        # every round averages one grad per worker: mean(1, 2) = 1.5 -> p -= lr * 1.5
        np.testing.assert_allclose(outs[0], -lr * 1.5 * rounds, rtol=1e-5)
        np.testing.assert_array_equal(outs[0], outs[1])
        for c in clients:
            c.done()
    finally:
        if p.poll() is None:
            time.sleep(0.5)
    _finish(p, out, t)


def test_ps_async_adam_two_shards_under_asan(san_tools):
    from arena_amd.parallel import ps as psmod
    n = 10_007
    ports = [_free_port(), _free_port()]
    procs = [_start_ps("asan", pt, 1) for pt in ports]
    cl = psmod.PSClient([f"127.0.0.1:{pt}" for pt in ports], n, timeout_s=30)
    rng = np.random.default_rng(0)
    w = rng.standard_normal(n).astype(np.float32)
    cl.init(w)
    got = np.empty(n, np.float32)
    for _ in range(5):
        cl.push_pull(rng.standard_normal(n).astype(np.float32), got)
    assert np.isfinite(got).all() and not np.array_equal(got, w)
    stats = cl.stats()
    assert [s[0] for s in stats] == [5, 5] and sum(s[1] for s in stats) == n
    cl.done()
    for p, out, t in procs:
        _finish(p, out, t)


def test_supervisor_and_probe_under_asan(san_tools, tmp_path, monkeypatch):
    from arena_amd.cli.commands import run
    from arena_amd.cluster.local import LocalBackend
    for k, v in _san_env("asan").items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("ARENA_LOCAL_GPUS", "2")
    monkeypatch.setenv("ARENA_NODE_IP", "10.0.0.7")
    assert _build.ensure_tool("arena-supervisor").endswith("/asan/arena-supervisor")
    b = LocalBackend(str(tmp_path / "home"), node_name="san-0")

    def cli(*argv):
        o = io.StringIO()
        rc = run(list(argv), backend=b, out=o)
        return rc, o.getvalue()

    py = sys.executable
    marker = tmp_path / "attempt"
    # fails on the first attempt, succeeds on the retry (backoffLimit = --retry 1)
    script = (f"import os,sys; p={str(marker)!r}; "
              f"first=not os.path.exists(p); open(p,'a').write('x'); "
              f"print('attempt', 'one' if first else 'two'); sys.exit(3 if first else 0)")
    rc, out = cli("submit", "sj", "--name", "san-sj", "--image", "i", "--retry", "1",
                  py, "-c", f'"{script}"')
    assert rc == 0, out
    rc, out = cli("submit", "mpi", "--name", "san-mpi", "--image", "i", "--workers", "2",
                  py, "-c", '"print(42)"')
    assert rc == 0, out
    deadline = time.time() + 90
    phases = {}
    while time.time() < deadline:
        phases = {n: b._state(n).get("phase") for n in ("san-sj", "san-mpi")}
        if all(v in ("Succeeded", "Failed") for v in phases.values()):
            break
        time.sleep(0.1)
    assert phases == {"san-sj": "Succeeded", "san-mpi": "Succeeded"}, phases
    assert marker.read_text() == "xx"                  # failed once, retried once
    # no sanitizer report from either supervisor (checked before delete removes the job dir)
    for name in ("san-sj", "san-mpi"):
        text = open(os.path.join(b.job_dir(name), "supervisor.log"), errors="replace").read()
        assert not any(m in text for m in REPORT_MARKERS), text
    for name in ("san-sj", "san-mpi"):
        cli("delete", name)

    # native probe over a fake sysfs topology
    root = tmp_path / "sys"
    node = root / "sys/class/kfd/kfd/topology/nodes/1"
    node.mkdir(parents=True)
    (node / "properties").write_text("simd_count 1024\ngfx_target_version 90500\n"
                                     "drm_render_minor 128\nlocation_id 256\n")
    r = subprocess.run([_build.tool_path("arena-probe", "asan"), "--root", str(root)],
                       capture_output=True, text=True, timeout=60, env=_san_env("asan"))
    assert not any(m in r.stderr for m in REPORT_MARKERS), r.stderr
    assert r.returncode == 0, r.stderr
