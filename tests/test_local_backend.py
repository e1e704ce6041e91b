"""LocalBackend end-to-end on CPU: real processes under the native supervisor.

Covers SURVEY §7.3 step 4: job store, GPU allocator, rank launcher (standalone / allreduce /
PS-worker), per-rank logs with timestamps and --follow, delete, retry (backoffLimit), jobmon
reaping on success and failure, fault injection, and the native topology probe.
"""
from __future__ import annotations

import io
import json
import os
import sys
import time

import pytest

from arena_amd import _build
from arena_amd.cli.commands import run
from arena_amd.cluster.local import LocalBackend, pick_gpus

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = sys.executable


@pytest.fixture(scope="module", autouse=True)
def _tools():
    _build.build_native_tools()


@pytest.fixture
def env(tmp_path, monkeypatch):
    monkeypatch.setenv("ARENA_LOCAL_GPUS", "2")
    monkeypatch.setenv("ARENA_NODE_IP", "10.0.0.7")
    monkeypatch.setenv("ARENA_DATA_CACHE", str(tmp_path / "cache"))
    b = LocalBackend(str(tmp_path / "home"), node_name="mi355x-0")
    yield b
    for name in b._release_names():
        try:
            b.delete_release(name)
        except Exception:  # noqa: BLE001
            pass


def cli(backend, *argv) -> str:
    out = io.StringIO()
    rc = run(list(argv), backend=backend, out=out)
    return out.getvalue() if rc == 0 else f"rc={rc}\n" + out.getvalue()


def wait_phase(b: LocalBackend, name: str, phases=("Succeeded", "Failed"), timeout=60.0) -> dict:
    deadline = time.time() + timeout
    while time.time() < deadline:
        st = b._state(name)
        if st.get("phase") in phases and (st.get("finished") or st.get("phase") != "Running"):
            return st
        time.sleep(0.05)
    raise AssertionError(f"{name} did not reach {phases}: {b._state(name)}")


def test_standalone_job_lifecycle(env):
    out = cli(env, "submit", "sj", "--name", "hello", "--gpus", "1",
              "echo hello from $HOSTNAME gpus=$HIP_VISIBLE_DEVICES; echo second line")
    assert "hello-training" in out
    st = wait_phase(env, "hello")
    assert st["phase"] == "Succeeded" and st["attempts"] == 1
    lst = cli(env, "list")
    assert lst.splitlines()[1].split()[:3] == ["hello", "SUCCEEDED", "STANDALONEJOB"]
    logs = cli(env, "logs", "hello")
    assert logs.startswith("hello from hello-training-") and "gpus=0" in logs
    assert logs.splitlines()[1] == "second line"
    ts = cli(env, "logs", "--timestamps", "--tail", "1", "hello")
    assert ts.split(" ", 1)[0].endswith("Z") and ts.rstrip().endswith("second line")
    got = cli(env, "get", "hello")
    assert "standalonejob" in got and "hello-training-" in got
    assert "deleted" in cli(env, "delete", "hello")
    assert not os.path.exists(env.job_dir("hello"))
    assert "doesn't exist" in cli(env, "get", "hello")


def test_retry_is_backoff_limit(env):
    cli(env, "submit", "sj", "--name", "flaky", "--retry", "2", "echo try; exit 3")
    st = wait_phase(env, "flaky")
    assert st["phase"] == "Failed" and st["attempts"] == 3
    pod = next(iter(st["pods"].values()))
    assert pod["exit_code"] == 3 and pod["restarts"] == 2
    logs = cli(env, "logs", "flaky")
    assert logs.count("try") == 3 and "restarting (attempt 3)" in logs
    assert cli(env, "list").splitlines()[1].split()[1] == "FAILED"


def test_gpu_allocation_and_exhaustion(env):
    cli(env, "submit", "sj", "--name", "a", "--gpus", "1", "sleep 30")
    cli(env, "submit", "sj", "--name", "b", "--gpus", "1", "sleep 30")
    ra = json.load(open(os.path.join(env.job_dir("a"), "release.json")))
    rb = json.load(open(os.path.join(env.job_dir("b"), "release.json")))
    assert sorted(list(ra["gpus"].values())[0] + list(rb["gpus"].values())[0]) == [0, 1]
    out = cli(env, "submit", "sj", "--name", "c", "--gpus", "1", "sleep 1")
    assert "insufficient GPUs" in out
    top = cli(env, "top", "node")
    assert "2           2" in top.replace("\t", " ") or "2/2" in top
    env.delete_release("a")
    # a's GPU is free again
    cli(env, "submit", "sj", "--name", "c", "--gpus", "1", "sleep 1")
    rc = json.load(open(os.path.join(env.job_dir("c"), "release.json")))
    assert list(rc["gpus"].values())[0] == list(ra["gpus"].values())[0]


def test_pick_gpus_prefers_one_hive():
    inv = {"count": 4, "gpus": [{"index": 0, "hive_id": "A"}, {"index": 1, "hive_id": "B"},
                                {"index": 2, "hive_id": "B"}, {"index": 3, "hive_id": "A"}]}
    assert pick_gpus(inv, set(), 2) == [0, 3] or pick_gpus(inv, set(), 2) == [1, 2]
    assert pick_gpus(inv, {0}, 2) == [1, 2]
    assert pick_gpus(inv, {0, 1}, 2) == [2, 3]   # no hive has 2 free: span hives


def test_delete_kills_running_processes(env):
    cli(env, "submit", "sj", "--name", "sleeper", "sleep 60")
    deadline = time.time() + 10
    pid = -1
    while time.time() < deadline and pid <= 0:
        st = env._state("sleeper")
        pid = next(iter(st.get("pods", {}).values()), {}).get("pid", -1)
        time.sleep(0.05)
    assert pid > 0 and os.path.exists(f"/proc/{pid}")
    assert cli(env, "list").splitlines()[1].split()[1] == "RUNNING"
    env.delete_release("sleeper")
    time.sleep(0.2)
    gone = not os.path.exists(f"/proc/{pid}") or open(f"/proc/{pid}/stat").read().split()[2] == "Z"
    assert gone


ALLREDUCE = (
    "import os, torch, torch.distributed as d; d.init_process_group('gloo'); "
    "t = torch.tensor([float(d.get_rank() + 1)]); d.all_reduce(t); "
    "print('rank', d.get_rank(), 'of', d.get_world_size(), 'sum', t.item(), "
    "'addr', os.environ['MASTER_ADDR']); d.destroy_process_group()")


def test_allreduce_job_ranks_rendezvous_and_reap(env):
    cli(env, "submit", "mpi", "--name", "ar", "--workers", "3", f'{PY} -c "{ALLREDUCE}"')
    st = wait_phase(env, "ar", timeout=120)
    assert st["phase"] == "Succeeded", st
    logs = "".join(open(os.path.join(env.job_dir("ar"), "logs", f)).read()
                   for f in os.listdir(os.path.join(env.job_dir("ar"), "logs")))
    for r in range(3):
        assert f"rank {r} of 3 sum 6.0 addr 127.0.0.1" in logs
    # jobmon semantics: worker StatefulSet pods are gone, the launcher Job shows SUCCEEDED
    pods = env.list_pods("default", {"release": "ar"})
    assert not [p for p in pods if p.meta.labels.get("role") == "mpiworker"]
    assert cli(env, "list").splitlines()[1].split()[:3] == ["ar", "SUCCEEDED", "MPIJOB"]


RANKS = (
    "import os, torch, torch.distributed as d; d.init_process_group('gloo'); "
    "t = torch.tensor([float(d.get_rank() + 1)]); d.all_reduce(t); "
    "e = os.environ; print('rank', d.get_rank(), 'of', d.get_world_size(), 'sum', t.item(), "
    "'local', e['LOCAL_RANK'], 'lws', e['LOCAL_WORLD_SIZE'], 'group', e['GROUP_RANK'], "
    "'vis', e.get('HIP_VISIBLE_DEVICES')); d.destroy_process_group()")


def test_allreduce_several_ranks_per_pod(env, monkeypatch):
    """`--workers 2 --gpus 4` on an 8-GPU node: 2 pods x 4 ranks (one per GPU), rendezvous of all
    8 over gloo; every rank sees the job's 8 GPUs and picks its own with a node-wide LOCAL_RANK
    (so one-node jobs keep the xGMI collectives)."""
    monkeypatch.setenv("ARENA_LOCAL_GPUS", "8")
    cli(env, "submit", "mpi", "--name", "rpp", "--workers", "2", "--gpus", "4",
        f'{PY} -c "{RANKS}"')
    plan = json.load(open(os.path.join(env.job_dir("rpp"), "plan.json")))
    assert len(plan["pods"]) == 2 and all("podlaunch" in " ".join(p["argv"]) for p in plan["pods"])
    st = wait_phase(env, "rpp", timeout=180)
    assert st["phase"] == "Succeeded", st
    logs = "".join(open(os.path.join(env.job_dir("rpp"), "logs", f)).read()
                   for f in os.listdir(os.path.join(env.job_dir("rpp"), "logs")))
    seen = {}
    for line in logs.splitlines():
        w = line.split()
        if "rank" in w and "sum" in w:
            i = w.index("rank")
            seen[int(w[i + 1])] = dict(zip(w[i + 2::2], w[i + 3::2]))
    assert sorted(seen) == list(range(8)), logs
    for r, kv in seen.items():
        assert kv["of"] == "8" and kv["sum"] == "36.0" and kv["lws"] == "8"
        assert kv["group"] == str(r // 4) and kv["vis"] == "0,1,2,3,4,5,6,7"
    assert sorted(int(kv["local"]) for kv in seen.values()) == list(range(8))


def test_podlaunch_failing_rank_takes_the_gang_down(tmp_path):
    """The in-pod launcher: one rank exits 7 -> its siblings (blocked, as in a collective) are
    terminated and the pod exits 7 quickly instead of hanging."""
    import subprocess
    env = dict(os.environ, ARENA_RANKS_PER_POD="3", ARENA_PODS="1", ARENA_POD_INDEX="0",
               ARENA_RANK_GRACE_S="2", PYTHONPATH=REPO,
               ARENA_RANK_COMMAND='if [ "$RANK" = 1 ]; then exit 7; fi; sleep 60')
    t0 = time.time()
    r = subprocess.run([PY, "-m", "arena_amd.runtime.podlaunch"], env=env, timeout=60)
    assert r.returncode == 7 and time.time() - t0 < 20
    from arena_amd.runtime import podlaunch
    envs = podlaunch.rank_envs({"ARENA_RANKS_PER_POD": "4", "ARENA_PODS": "3",
                                "POD_NAME": "job-tf-horovod-1"})
    assert [e["RANK"] for e in envs] == ["8", "9", "10", "11"]
    assert {e["WORLD_SIZE"] for e in envs} == {"12"} and envs[0]["GROUP_RANK"] == "2"


def _pid_alive(pid: int) -> bool:
    try:
        with open(f"/proc/{pid}/status") as f:
            return "\nState:\tZ" not in f.read()      # a zombie has exited
    except OSError:
        return False


def test_podlaunch_takes_down_grandchildren_of_compound_commands(tmp_path):
    """A compound rank command (``cd dir && python ...`` inside a subshell) runs the real rank as
    a grandchild of the launcher; when a peer rank fails, the whole rank's process group must be
    signalled, not just its shell (podlaunch.py:116)."""
    import subprocess
    prog = ("import os, time; open(os.path.join(%r, 'pid' + os.environ['RANK']), 'w')"
            ".write(str(os.getpid())); time.sleep(120)") % str(tmp_path)
    cmd = (f'if [ "$RANK" = 1 ]; then sleep 2; exit 5; fi; cd {tmp_path} && '
           f'( {PY} -c "{prog}" ); true')
    env = dict(os.environ, ARENA_RANKS_PER_POD="3", ARENA_PODS="1", ARENA_POD_INDEX="0",
               ARENA_RANK_GRACE_S="2", PYTHONPATH=REPO, ARENA_RANK_COMMAND=cmd)
    r = subprocess.run([PY, "-m", "arena_amd.runtime.podlaunch"], env=env, timeout=60)
    assert r.returncode == 5
    pids = [int((tmp_path / f"pid{k}").read_text()) for k in (0, 2)]
    deadline = time.time() + 10
    while time.time() < deadline and any(_pid_alive(p) for p in pids):
        time.sleep(0.1)
    assert not any(_pid_alive(p) for p in pids), pids


def test_local_world_envs_for_self_launching_bench():
    """bench.py --gpus N without torchrun: the environments it gives its N ranks."""
    from arena_amd.runtime import podlaunch
    envs = podlaunch.local_world_envs(4, {"PATH": "/bin", "ARENA_RANK_LOCAL_IDS": "5,6"},
                                      master_port=29123)
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    for e in envs:
        assert e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29123"
        assert e["GROUP_RANK"] == "0" and e["GROUP_WORLD_SIZE"] == "1" and e["PATH"] == "/bin"
        assert "ARENA_RANK_LOCAL_IDS" not in e and "ARENA_PODS" not in e


def test_allreduce_worker_fault_fails_job_and_reaps(env, monkeypatch):
    monkeypatch.setenv("ARENA_FAULT_POD", "fi-tf-horovod-0")
    monkeypatch.setenv("ARENA_FAULT_AFTER_MS", "300")
    cli(env, "submit", "mpi", "--name", "fi", "--workers", "2", "sleep 30")
    st = wait_phase(env, "fi", timeout=60)
    assert st["phase"] == "Failed"
    assert "fault injected" in st["message"] or st["pods"]["fi-tf-horovod-0"]["exit_code"] == 137
    assert all(p["pid"] == -1 for p in st["pods"].values())  # everything reaped (Q11)
    assert cli(env, "list").splitlines()[1].split()[1] == "FAILED"


def test_allreduce_retry_restarts_gang(env, monkeypatch):
    # the first attempt's worker dies; the retry runs the whole gang again and succeeds
    cmd = ("if [ \"$RANK\" = 1 ] && [ ! -f $ARENA_JOB_DIR/once ]; then touch $ARENA_JOB_DIR/once;"
           " exit 9; fi; sleep 0.5; echo ok $RANK")
    cli(env, "submit", "mpi", "--name", "rt", "--workers", "2", "--retry", "1", cmd)
    st = wait_phase(env, "rt", timeout=60)
    assert st["phase"] == "Succeeded" and st["attempts"] == 2, st


def test_tfjob_ps_workers_train_mnist(env):
    cmd = (f"{PY} -m arena_amd.examples.mnist_ps --max_steps 40 --n_train 1000 --device cpu "
           "--eval_every 20")
    out = cli(env, "submit", "tf", "--name", "dist", "--ps", "1", "--workers", "2", cmd)
    assert "dist-tfjob" in out or "TFJob" in out
    plan = json.load(open(os.path.join(env.job_dir("dist"), "plan.json")))
    tfc = [json.loads(p["env"]["TF_CONFIG"]) for p in plan["pods"] if "TF_CONFIG" in p["env"]]
    assert {t["task"]["type"] for t in tfc} == {"ps", "worker"}
    assert len(tfc[0]["cluster"]["worker"]) == 2 and len(tfc[0]["cluster"]["ps"]) == 1
    st = wait_phase(env, "dist", timeout=180)
    assert st["phase"] == "Succeeded", st
    (w0pod,) = [p.name for p in env.list_pods("default", {"release": "dist"})
                if p.name.rsplit("-", 1)[0] == "dist-tfjob-worker-0"]
    w0 = cli(env, "logs", "dist", "-i", w0pod)
    assert "Accuracy at step" in w0 and "test accuracy" in w0
    assert "TFJOB" in cli(env, "list")
    scal = os.path.join(env.job_dir("dist"), "tb", "test")
    assert os.listdir(scal)


def test_logs_follow_streams_until_exit(env):
    cli(env, "submit", "sj", "--name", "fol", "for i in 1 2 3; do echo line $i; sleep 0.3; done")
    time.sleep(0.2)
    lines = list(env.pod_logs("default", env.list_pods("default", {"release": "fol"})[0].name,
                              follow=True))
    assert [x.strip() for x in lines] == ["line 1", "line 2", "line 3"]


def test_data_mounts_and_env(env, tmp_path):
    host = tmp_path / "hostdata"
    host.mkdir()
    (host / "f.txt").write_text("payload")
    cli(env, "submit", "sj", "--name", "dm", "--dataDir", f"{host}:/data",
        "cat $ARENA_MOUNT_ROOT/data/f.txt; echo; echo $ARENA_DATADIR_TRAINING_DATA_0")
    wait_phase(env, "dm")
    logs = cli(env, "logs", "dm")
    assert "payload" in logs and str(host) in logs


def test_code_sync_copy(env, tmp_path):
    src = tmp_path / "proj"
    src.mkdir()
    (src / "train.py").write_text("print('synced code ran')\n")
    cli(env, "submit", "sj", "--name", "cs", "--syncMode", "rsync", "--syncSource", str(src),
        f"{PY} code/proj/train.py")
    st = wait_phase(env, "cs")
    assert st["phase"] == "Succeeded", cli(env, "logs", "cs")
    assert "synced code ran" in cli(env, "logs", "cs")


def test_probe_reads_fake_sysfs(tmp_path):
    import subprocess
    topo = tmp_path / "sys/class/kfd/kfd/topology/nodes"
    (topo / "0").mkdir(parents=True)
    (topo / "0/properties").write_text("simd_count 0\n")
    for n, other in ((1, 2), (2, 1)):
        d = topo / str(n)
        (d / "io_links/0").mkdir(parents=True)
        (d / "io_links/1").mkdir(parents=True)
        (d / "properties").write_text(
            f"simd_count 1024\ngfx_target_version 90500\nhive_id 77\nnum_xcc 8\n"
            f"drm_render_minor {127 + n}\nunique_id {n}\nlocation_id {n * 256}\n")
        (d / "io_links/0/properties").write_text("type 2\nnode_to 0\nweight 20\n")
        (d / "io_links/1/properties").write_text(f"type 11\nnode_to {other}\nweight 15\n")
        dev = tmp_path / f"sys/class/drm/renderD{127 + n}/device"
        (dev / "hwmon/hwmon0").mkdir(parents=True)
        (dev / "gpu_busy_percent").write_text("37\n")
        (dev / "mem_info_vram_total").write_text(str(288 * 2**30) + "\n")
        (dev / "mem_info_vram_used").write_text(str(2**30) + "\n")
        (dev / "hwmon/hwmon0/power1_average").write_text("750000000\n")
    out = subprocess.run([_build.ensure_tool("arena-probe"), "--root", str(tmp_path)],
                         capture_output=True, text=True, check=True).stdout
    inv = json.loads(out)
    assert inv["count"] == 2
    g0 = inv["gpus"][0]
    assert g0["gfx"] == "gfx950" and g0["hive_id"] == "77" and g0["num_xcc"] == 8
    assert g0["links"] == [{"to": 1, "type": "xgmi", "weight": 15}]
    assert g0["busy_percent"] == 37 and g0["vram_total"] == 288 * 2**30
    assert g0["power_uw"] == 750000000


def test_logviewer_serves_dashboard_urls(env):
    import signal
    import urllib.request
    cli(env, "submit", "sj", "--name", "lvw", "echo viewer line")
    wait_phase(env, "lvw")
    out = cli(env, "logviewer", "lvw")
    info = json.load(open(os.path.join(env.home, "logviewer.json")))
    try:
        assert f"10.0.0.7:{info['port']}/#!/log/default/lvw-training-" in out
        base = f"http://127.0.0.1:{info['port']}"
        jobs = json.load(urllib.request.urlopen(base + "/api/jobs", timeout=10))
        pod = jobs[0]["pods"][0]["name"]
        assert jobs[0]["name"] == "lvw" and jobs[0]["status"] == "SUCCEEDED"   # as `arena list`
        text = urllib.request.urlopen(f"{base}/api/log/default/{pod}", timeout=10).read().decode()
        assert text == "viewer line\n"
        assert b"arena log viewer" in urllib.request.urlopen(base + "/tfjobs/ui/", timeout=10).read()
    finally:
        os.kill(info["pid"], signal.SIGTERM)


def test_profile_gpu_runs_ranks_under_rocprofv3(env, tmp_path, monkeypatch):
    """--profile-gpu: each rank is exec'd by rocprofv3 (no shell hop) with traces in the job dir,
    and keeps its RANK although the chart's `export RANK=...` shell prefix is dropped."""
    bindir = tmp_path / "fakebin"
    bindir.mkdir()
    fake = bindir / "rocprofv3"
    fake.write_text("#!/bin/sh\n"
                    "while [ \"$1\" != \"--\" ]; do\n"
                    "  if [ \"$1\" = \"-d\" ]; then shift; mkdir -p \"$1\"; "
                    "echo traced > \"$1/run_kernel_stats.csv\"; fi\n"
                    "  shift\ndone\nshift\nexec \"$@\"\n")
    fake.chmod(0o755)
    monkeypatch.setenv("PATH", f"{bindir}{os.pathsep}{os.environ['PATH']}")
    script = tmp_path / "ar.py"
    script.write_text(ALLREDUCE.replace("; ", "\n"))
    cli(env, "submit", "mpi", "--name", "pg", "--workers", "2", "--profile-gpu",
        f"{PY} {script}")
    st = wait_phase(env, "pg", timeout=120)
    assert st["phase"] == "Succeeded", st
    jd = env.job_dir("pg")
    logs = "".join(open(os.path.join(jd, "logs", f)).read() for f in os.listdir(os.path.join(jd, "logs")))
    for r in range(2):
        assert f"rank {r} of 2 sum 3.0" in logs
    traced = sorted(os.listdir(os.path.join(jd, "traces")))
    assert len(traced) == 2 and all(
        os.path.exists(os.path.join(jd, "traces", t, "run_kernel_stats.csv")) for t in traced)


HANG_ONCE = """
import os, sys, time
from arena_amd.runtime import heartbeat
heartbeat.configure(os.environ["ARENA_HEARTBEAT_FILE"], min_interval=0.05)
marker = os.path.join(os.environ["ARENA_JOB_DIR"], "hung-once")
# the launcher (rank 0) hangs on the first attempt: a hung worker would just be reaped once the
# launcher succeeds (jobmon semantics), which is not what this test is about
first = os.environ.get("RANK", "0") == "0" and not os.path.exists(marker)
if first:
    open(marker, "a").close()
for step in range(10):
    heartbeat.beat(step)
    time.sleep(0.05)
if first:
    print("stuck in a collective", flush=True)
    time.sleep(120)          # no more beats: the supervisor must kill this rank
print("done", flush=True)
"""


def test_heartbeat_timeout_kills_hung_rank_and_retry_recovers(env, tmp_path):
    script = tmp_path / "hang_once.py"
    script.write_text(HANG_ONCE)
    cli(env, "submit", "mpi", "--name", "hb", "--workers", "2", "--retry", "1",
        "--heartbeatTimeout", "1.0", f"{PY} {script}")
    st = wait_phase(env, "hb", timeout=90)
    assert st["phase"] == "Succeeded" and st["attempts"] == 2, st
    logs = "".join(open(os.path.join(env.job_dir("hb"), "logs", f)).read()
                   for f in os.listdir(os.path.join(env.job_dir("hb"), "logs")))
    assert "heartbeat timeout" in logs and logs.count("done") >= 2


def test_heartbeat_timeout_without_retry_fails_job(env, tmp_path):
    script = tmp_path / "hang.py"
    script.write_text(HANG_ONCE)
    cli(env, "submit", "sj", "--name", "hb2", "--heartbeatTimeout", "1.0", f"{PY} {script}")
    st = wait_phase(env, "hb2", timeout=60)
    assert st["phase"] == "Failed", st
    pod = next(iter(st["pods"].values()))
    assert pod["exit_code"] == 137
