// arena-probe: GPU inventory, xGMI topology and live telemetry for the local backend
// (`arena top node`, the xGMI-hive-aware GPU allocator). Reads only sysfs -- never opens the GPU,
// so it is safe to run from the CLI and from the supervisor.
//
//   /sys/class/kfd/kfd/topology/nodes/<n>/properties   simd_count, gfx_target_version, hive_id,
//                                                       drm_render_minor, unique_id, location_id
//   /sys/class/kfd/kfd/topology/nodes/<n>/io_links/*/properties   type, node_to, weight
//   /sys/class/drm/renderD<minor>/device/               gpu_busy_percent, mem_info_vram_{total,used},
//                                                       hwmon/hwmon*/{power1_average,temp1_input}
//
// Output: one JSON document on stdout. `--root DIR` reads a fake sysfs tree (tests).
#include <dirent.h>

#include <algorithm>
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

std::string g_root;

std::string read_file(const std::string& path) {
  std::ifstream f(g_root + path);
  if (!f) return "";
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

std::map<std::string, std::string> read_props(const std::string& path) {
  std::map<std::string, std::string> out;
  std::istringstream in(read_file(path));
  std::string k, v;
  while (in >> k >> v) out[k] = v;
  return out;
}

std::vector<std::string> list_dir(const std::string& path) {
  std::vector<std::string> out;
  DIR* d = opendir((g_root + path).c_str());
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] != '.') out.push_back(e->d_name);
  }
  closedir(d);
  std::sort(out.begin(), out.end(), [](const std::string& a, const std::string& b) {
    char* ea = nullptr;
    char* eb = nullptr;
    long ia = std::strtol(a.c_str(), &ea, 10), ib = std::strtol(b.c_str(), &eb, 10);
    if (*ea == 0 && *eb == 0) return ia < ib;
    return a < b;
  });
  return out;
}

long long to_ll(const std::string& s, long long dflt = -1) {
  if (s.empty()) return dflt;
  char* end = nullptr;
  long long v = std::strtoll(s.c_str(), &end, 0);
  return end == s.c_str() ? dflt : v;
}

std::string trim(std::string s) {
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ')) s.pop_back();
  return s;
}

// KFD io_link type values (kfd_crat.h): 2 = PCIe (IOLINK_TYPE_PCIEXPRESS), 11 = xGMI
const char* link_name(long long t) {
  switch (t) {
    case 2: return "pcie";
    case 11: return "xgmi";
    default: return "other";
  }
}

}  // namespace

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--root") && i + 1 < argc) g_root = argv[++i];
  }
  const std::string topo = "/sys/class/kfd/kfd/topology/nodes";
  Json gpus = Json::array();
  std::map<long long, int> kfd_to_gpu;
  int idx = 0;
  std::vector<std::string> nodes = list_dir(topo);
  // first pass: GPU nodes in KFD order (the order HIP enumerates devices)
  for (const auto& n : nodes) {
    auto p = read_props(topo + "/" + n + "/properties");
    if (to_ll(p["simd_count"], 0) <= 0) continue;  // CPU node
    kfd_to_gpu[to_ll(n)] = idx++;
  }
  for (const auto& n : nodes) {
    auto p = read_props(topo + "/" + n + "/properties");
    if (to_ll(p["simd_count"], 0) <= 0) continue;
    Json g = Json::object();
    const long long kfd = to_ll(n);
    g.set("index", kfd_to_gpu[kfd]);
    g.set("kfd_node", kfd);
    const long long gfx = to_ll(p["gfx_target_version"], 0);
    char gfxs[32];
    std::snprintf(gfxs, sizeof gfxs, "gfx%lld%lld%llx", gfx / 10000, (gfx / 100) % 100, gfx % 100);
    g.set("gfx", std::string(gfxs));
    g.set("simd_count", to_ll(p["simd_count"], 0));
    g.set("num_xcc", to_ll(p["num_xcc"], 1));
    g.set("hive_id", std::to_string((unsigned long long)to_ll(p["hive_id"], 0)));
    g.set("unique_id", p["unique_id"]);
    g.set("location_id", to_ll(p["location_id"], 0));
    const long long minor = to_ll(p["drm_render_minor"], -1);
    g.set("render_minor", minor);
    Json links = Json::array();
    const std::string ld = topo + "/" + n + "/io_links";
    for (const auto& l : list_dir(ld)) {
      auto lp = read_props(ld + "/" + l + "/properties");
      const long long to = to_ll(lp["node_to"], -1);
      if (!kfd_to_gpu.count(to)) continue;  // link to a CPU node
      Json lj = Json::object();
      lj.set("to", kfd_to_gpu[to]);
      lj.set("type", link_name(to_ll(lp["type"], 0)));
      lj.set("weight", to_ll(lp["weight"], 0));
      links.push(lj);
    }
    g.set("links", links);
    if (minor >= 0) {
      const std::string dev = "/sys/class/drm/renderD" + std::to_string(minor) + "/device";
      g.set("busy_percent", to_ll(trim(read_file(dev + "/gpu_busy_percent")), -1));
      g.set("vram_total", to_ll(trim(read_file(dev + "/mem_info_vram_total")), -1));
      g.set("vram_used", to_ll(trim(read_file(dev + "/mem_info_vram_used")), -1));
      long long power = -1, temp = -1;
      for (const auto& h : list_dir(dev + "/hwmon")) {
        const std::string hp = dev + "/hwmon/" + h;
        if (power < 0) power = to_ll(trim(read_file(hp + "/power1_average")), -1);
        if (power < 0) power = to_ll(trim(read_file(hp + "/power1_input")), -1);
        if (temp < 0) temp = to_ll(trim(read_file(hp + "/temp1_input")), -1);
      }
      g.set("power_uw", power);
      g.set("temp_mc", temp);
    }
    gpus.push(g);
  }
  Json out = Json::object();
  out.set("gpus", gpus);
  out.set("count", (int)gpus.size());
  std::printf("%s\n", out.dump().c_str());
  return 0;
}
