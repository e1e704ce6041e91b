// arena-supervisor: native gang supervisor for the local backend.
//
// Replaces, on one machine, what the reference delegates to Kubernetes controllers and mpirun
// (SURVEY §2.7-§2.10, §5): batch Job backoffLimit retries, TFJob restart/clean-pod policies,
// the MPI launcher + worker StatefulSet lifecycle, and jobmon's "reap the workers when the
// launcher finishes" (on success AND failure -- quirk Q11 fixed).
//
//   arena-supervisor <job_dir>
//
// Reads <job_dir>/plan.json, starts one process group per pod (sh -c semantics come from the
// pod's argv), captures stdout+stderr through a pipe into <job_dir>/logs/<pod>.log with an
// RFC3339Nano timestamp per line (so `arena logs --since/--timestamps` work like the kubelet's),
// applies the job policy, and publishes <job_dir>/state.json atomically (write + rename) on every
// change and as a 1 s heartbeat. Control: a file <job_dir>/control/kill-<pod> terminates and
// deletes that pod (jobmon's StatefulSet delete); control/stop (or SIGTERM) stops everything.
// Never touches the GPU.
#include <dirent.h>
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "json.h"

using arena::Json;

namespace {

volatile sig_atomic_t g_stop = 0;
void on_signal(int) { g_stop = 1; }

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

std::string rfc3339nano() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  tm t;
  gmtime_r(&ts.tv_sec, &t);
  char buf[64];
  std::snprintf(buf, sizeof buf, "%04d-%02d-%02dT%02d:%02d:%02d.%09ldZ", t.tm_year + 1900,
                t.tm_mon + 1, t.tm_mday, t.tm_hour, t.tm_min, t.tm_sec, ts.tv_nsec);
  return buf;
}

std::string read_file(const std::string& p) {
  std::ifstream f(p);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

bool write_atomic(const std::string& path, const std::string& data) {
  const std::string tmp = path + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "w");
  if (!f) return false;
  std::fwrite(data.data(), 1, data.size(), f);
  std::fflush(f);
  fsync(fileno(f));
  std::fclose(f);
  return std::rename(tmp.c_str(), path.c_str()) == 0;
}

struct Pod {
  // spec
  std::string name, role;
  std::vector<std::string> argv;
  std::vector<std::pair<std::string, std::string>> env;
  std::string cwd, log_path;
  bool long_running = false;  // services (TensorBoard): not part of job completion
  // state
  pid_t pid = -1;
  int out_fd = -1;
  FILE* log = nullptr;
  std::string partial;
  std::string phase = "Pending";
  double start = 0, end = 0;
  int exit_code = -1;
  int restarts = 0;
  bool deleted = false;
  bool fault_done = false;
  std::string heartbeat;  // progress file the pod touches (empty: no hang detection)
};

struct Plan {
  std::string kind = "standalone";  // standalone | tfjob | allreduce
  int retry = 0;
  std::string launcher;             // allreduce: pod whose exit ends the job
  std::string clean_pod_policy = "Running";
  std::string restart_policy = "Never";  // Never | OnFailure | ExitCode (tfjob)
  double grace_s = 5.0;
  double heartbeat_timeout_s = 0;   // 0: off; else a pod silent this long after a beat is hung
  std::vector<Pod> pods;
};

class Supervisor {
 public:
  explicit Supervisor(std::string dir) : dir_(std::move(dir)) {}

  int run() {
    load_plan();
    mkdir((dir_ + "/logs").c_str(), 0755);
    mkdir((dir_ + "/control").c_str(), 0755);
    const char* fp = std::getenv("ARENA_FAULT_POD");
    if (fp) fault_pod_ = fp;
    if (const char* fa = std::getenv("ARENA_FAULT_AFTER_MS")) fault_after_ = std::atof(fa) / 1e3;
    if (const char* fs = std::getenv("ARENA_FAULT_SIGNAL")) fault_sig_ = std::atoi(fs);
    job_phase_ = "Running";
    for (auto& p : plan_.pods) start_pod(p);
    publish(true);
    double last_pub = now_s();
    while (true) {
      pump_io(200);
      reap();
      control();
      inject_fault();
      watchdog();
      policy();
      if (g_stop) stop_all("Stopped");
      const double t = now_s();
      if (dirty_ || t - last_pub > 1.0) {
        publish(false);
        last_pub = t;
      }
      if (!any_alive()) break;
    }
    pump_io(0);
    if (job_phase_ == "Running") job_phase_ = g_stop ? "Stopped" : "Failed";
    finished_ = true;
    publish(true);
    return job_phase_ == "Succeeded" ? 0 : 1;
  }

 private:
  std::string dir_;
  Plan plan_;
  std::string job_phase_ = "Pending";
  int attempts_ = 1;
  bool dirty_ = true;
  bool finished_ = false;
  std::string fault_pod_;
  double fault_after_ = 0;
  int fault_sig_ = SIGKILL;
  std::string message_;

  void load_plan() {
    Json j = Json::parse(read_file(dir_ + "/plan.json"));
    plan_.kind = j["kind"].as_str().empty() ? "standalone" : j["kind"].as_str();
    plan_.retry = (int)j["retry"].as_int(0);
    plan_.launcher = j["launcher"].as_str();
    if (!j["clean_pod_policy"].as_str().empty()) plan_.clean_pod_policy = j["clean_pod_policy"].as_str();
    if (!j["restart_policy"].as_str().empty()) plan_.restart_policy = j["restart_policy"].as_str();
    plan_.grace_s = j["grace_s"].as_num(5.0);
    plan_.heartbeat_timeout_s = j["heartbeat_timeout_s"].as_num(0.0);
    for (const auto& pj : j["pods"].elems()) {
      Pod p;
      p.name = pj["name"].as_str();
      p.role = pj["role"].as_str();
      for (const auto& a : pj["argv"].elems()) p.argv.push_back(a.as_str());
      for (const auto& kv : pj["env"].items()) p.env.emplace_back(kv.first, kv.second.as_str());
      p.cwd = pj["cwd"].as_str();
      p.log_path = pj["log"].as_str().empty() ? dir_ + "/logs/" + p.name + ".log" : pj["log"].as_str();
      p.long_running = pj["long_running"].as_bool(false);
      p.heartbeat = pj["heartbeat"].as_str();
      plan_.pods.push_back(std::move(p));
    }
  }

  Pod* find(const std::string& name) {
    for (auto& p : plan_.pods)
      if (p.name == name) return &p;
    return nullptr;
  }

  void log_line(Pod& p, const std::string& line) {
    if (!p.log) return;
    std::fprintf(p.log, "%s %s\n", rfc3339nano().c_str(), line.c_str());
    std::fflush(p.log);
  }

  void start_pod(Pod& p) {
    int fds[2];
    if (pipe(fds) != 0) {
      p.phase = "Failed";
      p.exit_code = 127;
      return;
    }
    if (!p.log) p.log = std::fopen(p.log_path.c_str(), "a");
    if (!p.heartbeat.empty()) unlink(p.heartbeat.c_str());  // a restart starts unbeaten
    pid_t pid = fork();
    if (pid == 0) {
      // child: own process group (so the whole tree can be signalled), output into the pipe
      setpgid(0, 0);
      dup2(fds[1], 1);
      dup2(fds[1], 2);
      close(fds[0]);
      close(fds[1]);
      int devnull = open("/dev/null", O_RDONLY);
      if (devnull >= 0) dup2(devnull, 0);
      for (auto& kv : p.env) setenv(kv.first.c_str(), kv.second.c_str(), 1);
      if (!p.cwd.empty() && chdir(p.cwd.c_str()) != 0) {
        std::fprintf(stderr, "arena-supervisor: chdir %s: %s\n", p.cwd.c_str(), std::strerror(errno));
        _exit(126);
      }
      std::vector<char*> av;
      for (auto& a : p.argv) av.push_back(const_cast<char*>(a.c_str()));
      av.push_back(nullptr);
      execvp(av[0], av.data());
      std::fprintf(stderr, "arena-supervisor: exec %s: %s\n", av[0], std::strerror(errno));
      _exit(127);
    }
    close(fds[1]);
    if (pid < 0) {
      close(fds[0]);
      p.phase = "Failed";
      p.exit_code = 127;
      return;
    }
    setpgid(pid, pid);
    fcntl(fds[0], F_SETFL, fcntl(fds[0], F_GETFL) | O_NONBLOCK);
    p.pid = pid;
    p.out_fd = fds[0];
    p.partial.clear();
    p.phase = "Running";
    p.start = now_s();
    p.end = 0;
    p.exit_code = -1;
    dirty_ = true;
  }

  void drain(Pod& p) {
    if (p.out_fd < 0) return;
    char buf[65536];
    while (true) {
      ssize_t n = read(p.out_fd, buf, sizeof buf);
      if (n > 0) {
        p.partial.append(buf, (size_t)n);
        size_t pos;
        while ((pos = p.partial.find('\n')) != std::string::npos) {
          log_line(p, p.partial.substr(0, pos));
          p.partial.erase(0, pos + 1);
        }
        continue;
      }
      if (n == 0) {  // EOF: every writer closed the pipe
        if (!p.partial.empty()) log_line(p, p.partial);
        p.partial.clear();
        close(p.out_fd);
        p.out_fd = -1;
      }
      break;
    }
  }

  void pump_io(int timeout_ms) {
    std::vector<pollfd> fds;
    std::vector<Pod*> who;
    for (auto& p : plan_.pods) {
      if (p.out_fd >= 0) {
        fds.push_back({p.out_fd, POLLIN, 0});
        who.push_back(&p);
      }
    }
    if (fds.empty()) {
      if (timeout_ms > 0) usleep(timeout_ms * 1000);
      return;
    }
    int r = poll(fds.data(), fds.size(), timeout_ms);
    if (r <= 0) return;
    for (size_t i = 0; i < fds.size(); ++i)
      if (fds[i].revents) drain(*who[i]);
  }

  void reap() {
    while (true) {
      int status = 0;
      pid_t pid = waitpid(-1, &status, WNOHANG);
      if (pid <= 0) break;
      for (auto& p : plan_.pods) {
        if (p.pid != pid) continue;
        drain(p);
        p.pid = -1;
        p.end = now_s();
        if (WIFEXITED(status)) p.exit_code = WEXITSTATUS(status);
        else if (WIFSIGNALED(status)) p.exit_code = 128 + WTERMSIG(status);
        if (!p.deleted) p.phase = p.exit_code == 0 ? "Succeeded" : "Failed";
        // a surviving child of the pod may still hold the pipe: keep the group signalled
        dirty_ = true;
      }
    }
  }

  void terminate(Pod& p, bool hard = false) {
    if (p.pid > 0) kill(-p.pid, hard ? SIGKILL : SIGTERM);
  }

  void terminate_all(std::vector<Pod*> pods) {
    for (auto* p : pods) terminate(*p);
    const double deadline = now_s() + plan_.grace_s;
    while (now_s() < deadline) {
      pump_io(50);
      reap();
      bool alive = false;
      for (auto* p : pods) alive |= p->pid > 0;
      if (!alive) return;
    }
    for (auto* p : pods) terminate(*p, true);
    for (int i = 0; i < 50; ++i) {
      pump_io(20);
      reap();
      bool alive = false;
      for (auto* p : pods) alive |= p->pid > 0;
      if (!alive) return;
    }
  }

  void stop_all(const char* why) {
    std::vector<Pod*> all;
    for (auto& p : plan_.pods) all.push_back(&p);
    terminate_all(all);
    if (job_phase_ == "Running") job_phase_ = why;
    g_stop = 0;
    stopped_ = true;
    dirty_ = true;
  }
  bool stopped_ = false;

  bool any_alive() const {
    for (const auto& p : plan_.pods)
      if (p.pid > 0 || p.out_fd >= 0) return true;
    return false;
  }

  void control() {
    const std::string cdir = dir_ + "/control";
    DIR* d = opendir(cdir.c_str());
    if (!d) return;
    std::vector<std::string> names;
    while (dirent* e = readdir(d)) {
      if (e->d_name[0] != '.') names.push_back(e->d_name);
    }
    closedir(d);
    for (const auto& n : names) {
      const std::string path = cdir + "/" + n;
      unlink(path.c_str());
      if (n == "stop") {
        g_stop = 1;
      } else if (n.rfind("kill-", 0) == 0) {
        Pod* p = find(n.substr(5));
        if (p) {
          p->deleted = true;  // jobmon deleted its StatefulSet: the pod disappears
          terminate_all({p});
          message_ = "deleted " + p->name;
          dirty_ = true;
        }
      }
    }
  }

  void inject_fault() {
    if (fault_pod_.empty()) return;
    Pod* p = find(fault_pod_);
    if (!p || p->fault_done || p->pid <= 0) return;
    if (now_s() - p->start >= fault_after_) {
      p->fault_done = true;
      kill(-p->pid, fault_sig_);
      message_ = "fault injected into " + p->name;
    }
  }

  // Hang detection: a running pod that has beaten at least once (its heartbeat file exists) and
  // has been silent for heartbeat_timeout_s is killed; the exit (137) then goes through the
  // normal retry / gang-restart policy. Pods that never beat are not judged (no opt-in).
  void watchdog() {
    if (plan_.heartbeat_timeout_s <= 0) return;
    const double t = now_s();
    for (auto& p : plan_.pods) {
      if (p.pid <= 0 || p.heartbeat.empty() || p.deleted) continue;
      struct stat st;
      if (stat(p.heartbeat.c_str(), &st) != 0) continue;
      const double mt = st.st_mtim.tv_sec + st.st_mtim.tv_nsec * 1e-9;
      const double silent = t - std::max(mt, p.start);
      if (silent > plan_.heartbeat_timeout_s) {
        char buf[160];
        std::snprintf(buf, sizeof buf, "heartbeat timeout: %s made no progress for %.1f s",
                      p.name.c_str(), silent);
        message_ = buf;
        log_line(p, std::string("arena-supervisor: ") + buf + "; killing it");
        kill(-p.pid, SIGKILL);
        unlink(p.heartbeat.c_str());
        dirty_ = true;
      }
    }
  }

  std::vector<Pod*> job_pods() {
    std::vector<Pod*> out;
    for (auto& p : plan_.pods)
      if (!p.long_running && !p.deleted) out.push_back(&p);
    return out;
  }

  void restart_gang(const std::vector<Pod*>& pods) {
    terminate_all(pods);
    ++attempts_;
    for (auto* p : pods) {
      p->restarts += 1;
      log_line(*p, "arena-supervisor: restarting (attempt " + std::to_string(attempts_) + ")");
      start_pod(*p);
    }
  }

  void finish(const std::string& phase) {
    job_phase_ = phase;
    dirty_ = true;
  }

  void policy() {
    if (job_phase_ != "Running" || stopped_) return;
    auto pods = job_pods();
    if (plan_.kind == "allreduce") {
      Pod* launcher = find(plan_.launcher);
      if (!launcher) return;
      std::vector<Pod*> workers;
      for (auto* p : pods)
        if (p != launcher) workers.push_back(p);
      bool worker_failed = false;
      for (auto* w : workers) worker_failed |= w->phase == "Failed";
      if (launcher->phase == "Succeeded") {
        // jobmon: the launcher Job succeeded -> delete the worker StatefulSet
        for (auto* w : workers) w->deleted = true;
        terminate_all(workers);
        finish("Succeeded");
      } else if (launcher->phase == "Failed" || worker_failed) {
        if (attempts_ <= plan_.retry) {
          restart_gang(pods);
        } else {
          for (auto* w : workers) w->deleted = true;  // Q11: reap on failure too
          std::vector<Pod*> live = workers;
          if (launcher->pid > 0) live.push_back(launcher);
          terminate_all(live);
          if (launcher->phase == "Running") launcher->phase = "Failed";
          finish("Failed");
        }
      }
    } else if (plan_.kind == "tfjob") {
      std::vector<Pod*> workers, others;
      for (auto* p : pods) (p->role == "worker" ? workers : others).push_back(p);
      bool all_workers_ok = !workers.empty();
      for (auto* w : workers) all_workers_ok &= w->phase == "Succeeded";
      Pod* failed = nullptr;
      for (auto* p : pods)
        if (p->phase == "Failed") { failed = p; break; }
      if (failed) {
        const int code = failed->exit_code;
        const bool retryable = plan_.restart_policy == "OnFailure" ||
                               (plan_.restart_policy == "ExitCode" && code >= 128 && code <= 255);
        if (retryable && failed->restarts < std::max(plan_.retry, 1) * 8) {
          failed->restarts += 1;
          log_line(*failed, "arena-supervisor: restarting after exit code " + std::to_string(code));
          start_pod(*failed);
          return;
        }
        clean_running(pods);
        finish("Failed");
      } else if (all_workers_ok) {
        clean_running(pods);
        finish("Succeeded");
      }
    } else {  // standalone: batch Job with backoffLimit = retry
      Pod* main = pods.empty() ? nullptr : pods.front();
      if (!main) return;
      if (main->phase == "Succeeded") {
        finish("Succeeded");
      } else if (main->phase == "Failed") {
        if (attempts_ <= plan_.retry) restart_gang({main});
        else finish("Failed");
      }
    }
  }

  void clean_running(const std::vector<Pod*>& pods) {
    if (plan_.clean_pod_policy != "Running") return;
    std::vector<Pod*> live;
    for (auto* p : pods)
      if (p->pid > 0) {
        p->deleted = true;
        live.push_back(p);
      }
    terminate_all(live);
  }

  // Written on every change and, unchanged, at least once a second: the mtime/"heartbeat" field
  // is how the CLI tells a live supervisor from a dead one.
  void publish(bool /*force*/) {
    Json st = Json::object();
    st.set("supervisor_pid", (long long)getpid());
    st.set("heartbeat", now_s());
    st.set("phase", job_phase_);
    st.set("attempts", attempts_);
    st.set("finished", finished_);
    st.set("message", message_);
    Json pods = Json::object();
    for (const auto& p : plan_.pods) {
      Json pj = Json::object();
      pj.set("phase", p.phase);
      pj.set("pid", (long long)p.pid);
      pj.set("start", p.start);
      pj.set("end", p.end);
      pj.set("exit_code", p.exit_code);
      pj.set("restarts", p.restarts);
      pj.set("deleted", p.deleted);
      pods.set(p.name, pj);
    }
    st.set("pods", pods);
    write_atomic(dir_ + "/state.json", st.dump());
    dirty_ = false;
  }
};

}  // namespace

int main(int argc, char** argv) {
  if (argc != 2) {
    std::fprintf(stderr, "usage: %s <job_dir>\n", argv[0]);
    return 2;
  }
  struct sigaction sa;
  std::memset(&sa, 0, sizeof sa);
  sa.sa_handler = on_signal;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  signal(SIGPIPE, SIG_IGN);
  try {
    Supervisor s(argv[1]);
    return s.run();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "arena-supervisor: %s\n", e.what());
    return 3;
  }
}
