// arena-ps: native parameter-server task for PS/worker ("tfjob") jobs.
//
// The reference's PS mode is TensorFlow's gRPC parameter server inside the user image
// (SURVEY §2.9, §2.12 "TF PS push/pull ... every step"; ports psPort 22223 / workerPort 22222,
// submit_tfjob.go:64-65). Here the PS is a small C++ server owning one contiguous shard of the
// model's flat fp32 parameter vector; workers (arena_amd/parallel/ps.py) split their flat
// gradient across the PS tasks listed in TF_CONFIG / MX_CLUSTER_SPEC and talk to all shards in
// parallel. The optimizer update runs here (TF applies gradients on the PS device), vectorised
// over the shard, so a push is one memcpy-sized message and one pass over the shard.
//
//   arena-ps --port P [--host 0.0.0.0] [--workers W] [--sync] [--optimizer adam|sgd]
//            [--lr 1e-3] [--beta1 0.9] [--beta2 0.999] [--eps 1e-8] [--tf-adam]
//
// Wire format (little-endian): request  = u32 magic 'APS1', u32 op, u64 nbytes, payload
//                              response = u32 magic, u32 status (0 ok), u64 nbytes, payload
//   INIT(1)     payload = f32[n]   first INIT defines the shard; later INITs are ignored
//                                  (non-chief workers); reply = u64 step
//   PULL(2)     reply = u64 step, f32[n]
//   PUSH(3)     payload = f32[n] gradient; async: applied at once; sync (--sync): averaged over
//               W pushes of the same round, applied once, every pusher released after the
//               apply (SyncReplicasOptimizer semantics); reply = u64 step
//   PUSHPULL(4) PUSH then PULL in one round trip; reply = u64 step, f32[n]
//   DONE(5)     a worker finished; after W DONEs the server exits 0
//   STAT(6)     reply = u64 step, u64 n, u64 pushes
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr uint32_t kMagic = 0x31535041;  // "APS1"
enum Op : uint32_t { INIT = 1, PULL = 2, PUSH = 3, PUSHPULL = 4, DONE = 5, STAT = 6 };

struct Config {
  std::string host = "0.0.0.0";
  int port = 22223;
  int workers = 1;
  bool sync = false;
  bool adam = true;
  bool tf_adam = false;
  float lr = 1e-3f, beta1 = 0.9f, beta2 = 0.999f, eps = 1e-8f;
};

struct Shard {
  std::mutex mu;
  std::condition_variable cv;
  bool ready = false;
  std::vector<float> p, m, v, acc;
  uint64_t step = 0;       // applied updates (Adam t)
  uint64_t pushes = 0;
  int round_count = 0;     // sync: pushes received in the current round
  uint64_t round_id = 0;
  int done = 0;
};

Config g_cfg;
Shard g_shard;
std::atomic<bool> g_exit{false};

bool read_full(int fd, void* buf, size_t n) {
  auto* p = static_cast<char*>(buf);
  while (n) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      return false;
    }
    p += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

bool write_full(int fd, const void* buf, size_t n) {
  auto* p = static_cast<const char*>(buf);
  while (n) {
    ssize_t r = ::send(fd, p, n, MSG_NOSIGNAL);
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      return false;
    }
    p += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

bool reply(int fd, uint32_t status, const void* a, size_t na, const void* b = nullptr,
           size_t nb = 0) {
  struct {
    uint32_t magic, status;
    uint64_t n;
  } h{kMagic, status, na + nb};
  return write_full(fd, &h, sizeof h) && (na == 0 || write_full(fd, a, na)) &&
         (nb == 0 || write_full(fd, b, nb));
}

// One optimizer step over the shard with gradient g (already averaged). Caller holds mu.
void apply(const float* g) {
  Shard& s = g_shard;
  const size_t n = s.p.size();
  s.step += 1;
  float* __restrict p = s.p.data();
  if (!g_cfg.adam) {
    const float lr = g_cfg.lr;
    for (size_t i = 0; i < n; ++i) p[i] -= lr * g[i];
    return;
  }
  float* __restrict m = s.m.data();
  float* __restrict v = s.v.data();
  const float b1 = g_cfg.beta1, b2 = g_cfg.beta2, eps = g_cfg.eps;
  const double t = static_cast<double>(s.step);
  const float bc1 = static_cast<float>(1.0 - std::pow(static_cast<double>(b1), t));
  const float bc2 = static_cast<float>(1.0 - std::pow(static_cast<double>(b2), t));
  if (g_cfg.tf_adam) {
    // TF AdamOptimizer: lr_t = lr * sqrt(1-b2^t)/(1-b1^t); p -= lr_t * m / (sqrt(v) + eps)
    const float lr_t = g_cfg.lr * std::sqrt(bc2) / bc1;
    for (size_t i = 0; i < n; ++i) {
      const float gi = g[i];
      const float mi = b1 * m[i] + (1.f - b1) * gi;
      const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
      m[i] = mi;
      v[i] = vi;
      p[i] -= lr_t * mi / (std::sqrt(vi) + eps);
    }
  } else {
    // torch.optim.Adam: p -= lr * (m/bc1) / (sqrt(v/bc2) + eps)
    const float step_size = g_cfg.lr / bc1;
    const float inv_sqrt_bc2 = 1.f / std::sqrt(bc2);
    for (size_t i = 0; i < n; ++i) {
      const float gi = g[i];
      const float mi = b1 * m[i] + (1.f - b1) * gi;
      const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
      m[i] = mi;
      v[i] = vi;
      p[i] -= step_size * mi / (std::sqrt(vi) * inv_sqrt_bc2 + eps);
    }
  }
}

// Returns the step after this worker's gradient is applied.
uint64_t push(const std::vector<float>& g) {
  Shard& s = g_shard;
  std::unique_lock<std::mutex> lk(s.mu);
  s.pushes += 1;
  if (!g_cfg.sync || g_cfg.workers <= 1) {
    apply(g.data());
    return s.step;
  }
  const size_t n = s.p.size();
  if (s.round_count == 0) std::fill(s.acc.begin(), s.acc.end(), 0.f);
  for (size_t i = 0; i < n; ++i) s.acc[i] += g[i];
  const uint64_t my_round = s.round_id;
  if (++s.round_count == g_cfg.workers) {
    const float inv = 1.f / static_cast<float>(g_cfg.workers);
    for (size_t i = 0; i < n; ++i) s.acc[i] *= inv;
    apply(s.acc.data());
    s.round_count = 0;
    s.round_id += 1;
    s.cv.notify_all();
  } else {
    s.cv.wait(lk, [&] { return s.round_id != my_round || g_exit.load(); });
  }
  return s.step;
}

void serve(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  std::vector<float> buf;
  std::vector<float> snap;
  for (;;) {
    struct {
      uint32_t magic, op;
      uint64_t n;
    } h;
    if (!read_full(fd, &h, sizeof h) || h.magic != kMagic) break;
    if (h.n % 4 || h.n > (uint64_t(1) << 36)) break;
    buf.resize(h.n / 4);
    if (h.n && !read_full(fd, buf.data(), h.n)) break;
    Shard& s = g_shard;
    bool ok = true;
    switch (h.op) {
      case INIT: {
        uint64_t step;
        {
          std::lock_guard<std::mutex> lk(s.mu);
          if (!s.ready) {
            s.p = buf;
            s.m.assign(buf.size(), 0.f);
            s.v.assign(buf.size(), 0.f);
            s.acc.assign(buf.size(), 0.f);
            s.ready = true;
            s.cv.notify_all();
          }
          step = s.step;
        }
        ok = reply(fd, 0, &step, 8);
        break;
      }
      case PULL: {
        uint64_t step;
        {
          std::unique_lock<std::mutex> lk(s.mu);
          s.cv.wait(lk, [&] { return s.ready || g_exit.load(); });
          snap = s.p;
          step = s.step;
        }
        ok = reply(fd, 0, &step, 8, snap.data(), snap.size() * 4);
        break;
      }
      case PUSH:
      case PUSHPULL: {
        if (!s.ready || buf.size() != s.p.size()) {
          ok = reply(fd, 1, nullptr, 0);
          break;
        }
        uint64_t step = push(buf);
        if (h.op == PUSH) {
          ok = reply(fd, 0, &step, 8);
        } else {
          {
            std::lock_guard<std::mutex> lk(s.mu);
            snap = s.p;
            step = s.step;
          }
          ok = reply(fd, 0, &step, 8, snap.data(), snap.size() * 4);
        }
        break;
      }
      case DONE: {
        int d;
        {
          std::lock_guard<std::mutex> lk(s.mu);
          d = ++s.done;
        }
        ok = reply(fd, 0, nullptr, 0);
        if (d >= g_cfg.workers) {
          std::printf("arena-ps: all %d workers done after %llu updates\n", g_cfg.workers,
                      static_cast<unsigned long long>(s.step));
          std::fflush(stdout);
          std::_Exit(0);
        }
        break;
      }
      case STAT: {
        uint64_t st[3];
        {
          std::lock_guard<std::mutex> lk(s.mu);
          st[0] = s.step;
          st[1] = s.p.size();
          st[2] = s.pushes;
        }
        ok = reply(fd, 0, st, sizeof st);
        break;
      }
      default:
        ok = reply(fd, 2, nullptr, 0);
    }
    if (!ok) break;
  }
  ::close(fd);
}

void usage() {
  std::fprintf(stderr,
               "usage: arena-ps --port P [--host H] [--workers W] [--sync] "
               "[--optimizer adam|sgd] [--lr X] [--beta1 X] [--beta2 X] [--eps X] [--tf-adam]\n");
}

}  // namespace

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&](const char* name) -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "arena-ps: %s needs a value\n", name);
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--port") g_cfg.port = std::atoi(next("--port"));
    else if (a == "--host") g_cfg.host = next("--host");
    else if (a == "--workers") g_cfg.workers = std::atoi(next("--workers"));
    else if (a == "--sync") g_cfg.sync = true;
    else if (a == "--optimizer") g_cfg.adam = std::string(next("--optimizer")) != "sgd";
    else if (a == "--lr") g_cfg.lr = std::strtof(next("--lr"), nullptr);
    else if (a == "--beta1") g_cfg.beta1 = std::strtof(next("--beta1"), nullptr);
    else if (a == "--beta2") g_cfg.beta2 = std::strtof(next("--beta2"), nullptr);
    else if (a == "--eps") g_cfg.eps = std::strtof(next("--eps"), nullptr);
    else if (a == "--tf-adam") g_cfg.tf_adam = true;
    else if (a == "-h" || a == "--help") {
      usage();
      return 0;
    } else {
      usage();
      return 2;
    }
  }
  if (g_cfg.workers < 1) g_cfg.workers = 1;
  signal(SIGPIPE, SIG_IGN);
  int ls = ::socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(g_cfg.port));
  if (inet_pton(AF_INET, g_cfg.host.c_str(), &addr.sin_addr) != 1) {
    std::fprintf(stderr, "arena-ps: bad host %s\n", g_cfg.host.c_str());
    return 2;
  }
  if (::bind(ls, reinterpret_cast<sockaddr*>(&addr), sizeof addr) != 0 || ::listen(ls, 64) != 0) {
    std::perror("arena-ps: bind/listen");
    return 1;
  }
  std::printf("arena-ps: serving on %s:%d workers=%d mode=%s optimizer=%s lr=%g\n",
              g_cfg.host.c_str(), g_cfg.port, g_cfg.workers, g_cfg.sync ? "sync" : "async",
              g_cfg.adam ? (g_cfg.tf_adam ? "adam(tf)" : "adam") : "sgd", g_cfg.lr);
  std::fflush(stdout);
  for (;;) {
    int fd = ::accept(ls, nullptr, nullptr);
    if (fd < 0) {
      if (errno == EINTR) continue;
      std::perror("arena-ps: accept");
      return 1;
    }
    std::thread(serve, fd).detach();
  }
}
