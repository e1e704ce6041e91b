"""CLI on the in-memory FakeBackend: golden outputs for every table, trainer
discovery/status rules and the submit pipeline."""
import io

import pytest

from arena_amd.cli.commands import run
from arena_amd.cluster.fake import FakeBackend, make_node


class Clock:
    def __init__(self, t=1_000_000.0):
        self.t = t

    def __call__(self):
        return self.t


@pytest.fixture
def env(monkeypatch):
    clock = Clock()
    nodes = [make_node("master-0", "192.168.1.116", 0, master=True),
             make_node("node-a", "192.168.1.119", 8),
             make_node("node-b", "192.168.1.120", 8)]
    fake = FakeBackend(nodes, clock=clock)
    monkeypatch.setattr("time.time", clock)

    def arena(*argv):
        out = io.StringIO()
        rc = run(list(argv), backend=fake, out=out)
        return rc, out.getvalue()

    return fake, clock, arena


def _task_pod(fake, task):
    """The pod of a PS/worker task Job ``<release>-tfjob-<type>-<i>`` (Job pods get a suffix)."""
    (p,) = [p for p in fake.list_pods() if p.name.rsplit("-", 1)[0] == task]
    return p


def test_submit_tf_and_list_get_top(env):
    fake, clock, arena = env
    rc, out = arena("submit", "tf", "--name", "tf-git", "--gpus", "1", "--image", "img",
                    "--syncMode", "git", "--syncSource", "https://x/tensorflow-sample-code.git",
                    "python", "main.py", "--max_steps", "1000")
    assert rc == 0, out
    # operator-free: one batch Job + headless Service per task (no TFJob CRD needed)
    assert "==> batch/v1/Job" in out and "==> v1/Service" in out
    assert "tf-git-tfjob-worker-0" in out and "TFJob" not in out
    rel = fake.get_release("tf-git")
    assert rel.values["syncGitProjectName"] == "tensorflow-sample-code"
    assert rel.values["command"] == "python main.py --max_steps 1000"
    assert rel.values["envs"] == {"workers": "1", "gpus": "1"}
    # pending until scheduled
    rc, out = arena("list")
    assert out == ("NAME    STATUS   TRAINER  AGE  NODE\n"
                   "tf-git  PENDING  TFJOB    0s   N/A\n")
    fake.schedule()
    clock.t += 17
    rc, out = arena("top", "job")
    assert out == ("NAME    STATUS   TRAINER  AGE  NODE           GPU(Requests)  GPU(Allocated)\n"
                   "tf-git  RUNNING  TFJOB    17s  192.168.1.119  1              1\n"
                   "\n\nTotal Allocated GPUs of Training Job:\n1   \n\n"
                   "Total Requested GPUs of Training Job:\n1   \n")
    rc, out = arena("top", "node")
    assert out == ("NAME      IPADDRESS      ROLE    GPU(Total)  GPU(Allocated)\n"
                   "master-0  192.168.1.116  master  0           0\n"
                   "node-a    192.168.1.119  worker  8           1\n"
                   "node-b    192.168.1.120  worker  8           0\n"
                   + "-" * 89 + "\n"
                   "Allocated/Total GPUs In Cluster:\n1/16 (6%)  \n")
    rc, out = arena("get", "tf-git")
    chief = _task_pod(fake, "tf-git-tfjob-worker-0").name
    assert out == ("NAME    STATUS   TRAINER  AGE  INSTANCE                     NODE\n"
                   f"tf-git  RUNNING  tfjob    17s  {chief}  192.168.1.119\n")
    rc, out = arena("get", "tf-git", "-o", "name")
    assert out == "tf-git\n"
    rc, out = arena("get", "nope")
    assert rc == 1 and "doesn't exist" in out


def test_tf_status_precedence(env):
    fake, clock, arena = env
    arena("submit", "tf", "--name", "dist", "--gpus", "1", "--image", "i", "--workers", "2",
          "--ps", "1", "python", "dist.py")
    tasks = sorted(p.name.rsplit("-", 1)[0] for p in fake.list_pods("default"))
    assert tasks == ["dist-tfjob-ps-0", "dist-tfjob-worker-0", "dist-tfjob-worker-1"]
    w0 = _task_pod(fake, "dist-tfjob-worker-0")
    assert w0.meta.labels["group_name"] == "kubeflow.org"
    assert w0.meta.labels["tf-replica-index"] == "0"
    assert arena("list")[1].splitlines()[1].split()[1] == "PENDING"
    fake.schedule()
    assert arena("list")[1].splitlines()[1].split()[1] == "RUNNING"
    for t in ("dist-tfjob-worker-0", "dist-tfjob-worker-1"):
        fake.set_phase("default", _task_pod(fake, t).name, "Succeeded")
    assert arena("list")[1].splitlines()[1].split()[1] == "SUCCEEDED"
    # PS has no GPU; two workers x 1 GPU, completed -> requested 2, allocated 1 (ps not GPU)
    out = arena("top", "job")[1]
    assert out.splitlines()[1].split()[-2:] == ["2", "0"]


def test_mpi_job_chief_is_newest_job_pod_and_workers_listed(env):
    fake, clock, arena = env
    rc, out = arena("submit", "mpi", "--name", "hvd", "--gpus", "2", "--workers", "3",
                    "--image", "img", "python", "train.py")
    assert rc == 0, out
    rel = fake.get_release("hvd")
    assert rel.values["workers"] == 2 and rel.values["envs"]["workers"] == "3"
    names = sorted(p.name for p in fake.list_pods())
    assert "hvd-tf-horovod-0" in names and "hvd-tf-horovod-1" in names
    job_pods = [p for p in fake.list_pods() if "Job" in p.meta.owner_kinds
                and p.meta.labels.get("role") == "mpimaster"]
    assert len(job_pods) == 1
    # the jobmon job lives in arena-system with the reap contract env
    assert fake.get_job("arena-system", "hvd-tf-horovod-jobmon") is not None
    jm_pod = [p for p in fake.list_pods("arena-system")][0]
    assert jm_pod.containers[0].env == {"NAMESPACE": "default", "JOBNAME": "hvd-tf-horovod-job",
                                        "STATEFULSETNAME": "hvd-tf-horovod",
                                        "ARENA_BACKEND": "k8s", "ARENA_JOBMON_TIMEOUT": "168h"}
    fake.schedule()
    rc, out = arena("get", "hvd")
    lines = out.splitlines()
    assert lines[-1].split()[4].startswith("hvd-tf-horovod-job-")  # chief listed last
    master_env = job_pods[0].containers[0].env
    assert master_env["MASTER_ADDR"] == "hvd-tf-horovod-master"
    assert master_env["WORLD_SIZE"] == "6"        # 3 pods x 2 GPUs: one rank per GPU
    assert master_env["ARENA_RANKS_PER_POD"] == "2"
    out = arena("top", "job")[1]
    assert out.splitlines()[1].split()[-2:] == ["6", "6"]


def test_standalone_and_delete_many(env):
    fake, clock, arena = env
    for n in ("a1", "a2", "a3"):
        rc, out = arena("submit", "sj", "--name", n, "--image", "i", "--gpus", "1", "python", "x.py")
        assert rc == 0, out   # Q1: no spurious "already exist" error
    rc, out = arena("submit", "sj", "--name", "a1", "--image", "i", "python", "x.py")
    assert rc == 1 and "already exist" in out
    rc, out = arena("delete", "a1", "a2", "zz")
    assert rc == 1                                    # one failed
    assert fake.deleted == ["a1", "a2"]               # Q2: all names processed
    assert sorted(fake.list_releases()) == ["a3"]


def test_list_orders_newest_first(env):
    fake, clock, arena = env
    arena("submit", "sj", "--name", "old", "--image", "i", "python", "x.py")
    fake.schedule()
    clock.t += 100
    arena("submit", "sj", "--name", "new", "--image", "i", "python", "x.py")
    fake.schedule()
    clock.t += 10
    names = [l.split()[0] for l in arena("list")[1].splitlines()[1:]]
    assert names == ["new", "old"]


def test_validation_errors(env):
    fake, clock, arena = env
    rc, out = arena("submit", "tf", "--name", "Bad_Name", "--image", "i", "python", "x")
    assert rc == 1 and "lower case" in out
    rc, out = arena("submit", "tf", "--name", "x", "python", "x")
    assert rc == 1 and "--image or --workerImage must be set" in out
    rc, out = arena("submit", "tf", "--name", "x", "--image", "i", "--cleanTaskPolicy", "All",
                    "python")
    assert rc == 1 and "Unsupported cleanTaskPolicy" in out
    rc, out = arena("submit", "tf", "--name", "x", "--image", "i", "--dataDir", "rel", "python")
    assert rc == 1 and "must be absolute" in out   # Q3: transform errors propagate
    rc, out = arena("submit", "tf", "--name", "x", "--image", "i", "--syncMode", "hdfs",
                    "python")
    assert rc == 1 and "Unknown sync mode" in out


def test_env_data_tensorboard_values(env):
    fake, clock, arena = env
    rc, out = arena("submit", "tf", "--name", "tb", "--image", "i", "--gpus", "1",
                    "-e", "A=1", "-e", "B=x=y", "-d", "mnist-pvc:/data", "--dataDir",
                    "/host/logs:/logs", "--tensorboard", "python", "m.py")
    assert rc == 0, out
    v = fake.get_release("tb").values
    assert v["envs"] == {"A": "1", "B": "x=y", "workers": "1", "gpus": "1"}
    assert v["dataset"] == {"mnist-pvc": "/data"}
    assert v["dataDirs"] == [{"name": "training-data-0", "hostPath": "/host/logs",
                              "containerPath": "/logs"}]
    assert v["hostLogPath"].startswith("/arena_logs/training") and len(v["hostLogPath"]) == 29
    assert v["gpuResource"] == "amd.com/gpu"
    fake.schedule()
    rc, out = arena("get", "tb")
    assert "Your tensorboard will be available on:" in out
    assert "http://192.168.1.116:30000" in out
    w0 = _task_pod(fake, "tb-tfjob-worker-0")
    assert w0.containers[0].limits == {"amd.com/gpu": 1}


def test_logs_tail_since_timestamps(env):
    fake, clock, arena = env
    arena("submit", "sj", "--name", "lg", "--image", "i", "python", "x.py")
    fake.schedule()
    pod = fake.list_pods(selector={"release": "lg"})[0].name
    for i in range(10):
        fake.add_log("default", pod, f"Accuracy at step {i * 10}: 0.9", t=clock.t - 100 + i * 10)
    rc, out = arena("logs", "lg", "--tail", "2")
    assert out == "Accuracy at step 80: 0.9\nAccuracy at step 90: 0.9\n"
    rc, out = arena("logs", "lg", "--since", "25s")
    assert out.count("\n") == 2
    rc, out = arena("logs", "lg", "--tail", "1", "--timestamps")
    assert out.startswith("1970-01-12T") and out.endswith("Accuracy at step 90: 0.9\n")
    rc, out = arena("logs", "lg", "-i", "nope")
    assert rc == 1


def test_logviewer(env):
    fake, clock, arena = env
    arena("submit", "tf", "--name", "lv", "--image", "i", "python", "x.py")
    rc, out = arena("logviewer", "lv")
    assert rc == 1 and "No LOGVIEWER Installed." in out
    fake.add_endpoints("arena-system", "tf-job-dashboard", "192.168.1.120", 8080)
    rc, out = arena("logviewer", "lv")
    assert out == ("Your LogViewer will be available on:\n"
                   "192.168.1.120:8080/tfjobs/ui/#/default/lv-tfjob\n")


def test_top_node_details(env):
    fake, clock, arena = env
    arena("submit", "sj", "--name", "d1", "--image", "i", "--gpus", "2", "python", "x.py")
    fake.schedule()
    rc, out = arena("top", "node", "-d")
    assert "NAME:       node-a" in out
    assert "Total GPUs In Node node-a:      8" in out
    assert "Allocated GPUs In Node node-a:  2 (25%)" in out
    assert out.rstrip().endswith("Allocated/Total GPUs In Cluster:  2/16 (12%)")


def test_top_node_summary_with_live_telemetry():
    """Local backend: `top node` adds the probe's live busy %, VRAM and power columns."""
    from arena_amd.cli import display
    from arena_amd.jobs.nodes import NodeInfo
    node = make_node("mi355x-0", "10.0.0.7", 8)
    out = io.StringIO()
    display.top_node_summary(out, [NodeInfo(node, [])],
                             telemetry={"mi355x-0": {"busy": "37%", "vram": "12/2304",
                                                     "power": "5600"}})
    lines = out.getvalue().splitlines()
    assert lines[0].split() == ["NAME", "IPADDRESS", "ROLE", "GPU(Total)", "GPU(Allocated)",
                                "GPU(Busy%)", "VRAM(Used/Total", "GiB)", "Power(W)"]
    assert lines[1].split() == ["mi355x-0", "10.0.0.7", "worker", "8", "0", "37%", "12/2304",
                                "5600"]


def test_version_and_completion(env):
    fake, clock, arena = env
    rc, out = arena("version")
    assert rc == 0 and out.startswith("Version: v")
    rc, out = arena("version", "--short")
    assert out.startswith("v")
    rc, out = arena("completion", "bash")
    assert "complete -F _arena arena" in out and "submit" in out
    rc, out = arena("completion", "zsh")
    assert "compdef _arena arena" in out


def test_global_flags_after_subcommand(env):
    """cobra persistent flags (root.go:39-44) work before or after the subcommand."""
    fake, clock, arena = env
    rc, out = arena("submit", "sj", "--name", "ns1", "--image", "i", "--namespace", "team-a",
                    "python", "x.py")
    assert rc == 0, out
    fake.schedule()
    rc, out = arena("list", "--namespace", "team-a")
    assert rc == 0 and "ns1" in out
    rc, out = arena("--namespace", "team-a", "get", "ns1")
    assert rc == 0 and "ns1" in out
    with pytest.raises(SystemExit) as ei:          # util/logs.go:20-21: fatal
        arena("top", "job", "--loglevel", "bogus")
    assert ei.value.code == 1


def test_pprof_writes_cpu_profile(tmp_path, monkeypatch, capsys):
    """B1: --pprof anywhere on the command line dumps a CPU profile (cmd/arena/main.go:14-39)."""
    import pstats
    from arena_amd.cli.main import _pprof_enabled, main
    prof = tmp_path / "cpu_profile"
    monkeypatch.setenv("ARENA_PPROF_PATH", str(prof))
    monkeypatch.setenv("ARENA_HOME", str(tmp_path / "home"))
    assert main(["version", "--short", "--pprof"]) == 0
    assert capsys.readouterr().out.startswith("v")
    st = pstats.Stats(str(prof))
    assert any("cmd_version" in fn for (_, _, fn) in st.stats)
    assert not _pprof_enabled(["--pprof=false", "list"]) and _pprof_enabled(["list", "--pprof"])
