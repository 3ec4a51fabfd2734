#include "affinity.h"

#include <pthread.h>
#include <sched.h>

#include <cstdlib>
#include <fstream>
#include <sstream>

namespace ksa {

bool pin_current_thread(const CpuList& cpus) {
  if (cpus.empty()) return true;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus)
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
  return pthread_setaffinity_np(pthread_self(), sizeof set, &set) == 0;
}

namespace {

constexpr int64_t kUs = 1000;

bool parse_i64(const std::string& s, int64_t* out) {
  const char* b = s.c_str();
  while (*b == ' ' || *b == '\t') ++b;
  char* end = nullptr;
  const long long v = std::strtoll(b, &end, 10);
  if (end == b) return false;
  while (*end == ' ' || *end == '\t' || *end == '\n') ++end;
  if (*end != '\0') return false;
  *out = v;
  return true;
}

bool read_file(const std::string& path, std::string* out) {
  std::ifstream f(path);
  if (!f) return false;
  std::ostringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

}  // namespace

CpuQuota parse_cpu_max(const std::string& text) {
  CpuQuota q;
  std::istringstream in(text);
  std::string quota, period;
  if (!(in >> quota >> period) || quota == "max") return q;
  int64_t qu = 0, pe = 0;
  if (!parse_i64(quota, &qu) || !parse_i64(period, &pe) || qu <= 0 || pe <= 0) return q;
  q.quota_ns = qu * kUs;
  q.period_ns = pe * kUs;
  return q;
}

CpuQuota parse_cfs_quota(const std::string& quota_us, const std::string& period_us) {
  CpuQuota q;
  int64_t qu = 0, pe = 0;
  if (!parse_i64(quota_us, &qu) || !parse_i64(period_us, &pe) || qu <= 0 || pe <= 0) return q;
  q.quota_ns = qu * kUs;
  q.period_ns = pe * kUs;
  return q;
}

CpuQuota read_cpu_quota(const std::string& root) {
  std::string v2_path, v1_path, cg;
  if (read_file("/proc/self/cgroup", &cg)) {
    std::istringstream lines(cg);
    std::string line;
    while (std::getline(lines, line)) {  // "<id>:<controllers>:<path>"
      const size_t a = line.find(':'), b = a == std::string::npos ? a : line.find(':', a + 1);
      if (b == std::string::npos) continue;
      const std::string ctl = line.substr(a + 1, b - a - 1), path = line.substr(b + 1);
      if (ctl.empty()) v2_path = path;
      std::istringstream names(ctl);
      std::string name;
      while (std::getline(names, name, ','))
        if (name == "cpu") v1_path = path;
    }
  }
  std::string text, quota, period;
  for (const std::string& dir : {root + v2_path, root}) {
    if (read_file(dir + "/cpu.max", &text)) return parse_cpu_max(text);
  }
  for (const std::string& ctl : {std::string("/cpu"), std::string("/cpu,cpuacct"), std::string("/cpuacct,cpu")}) {
    for (const std::string& dir : {root + ctl + v1_path, root + ctl}) {
      if (read_file(dir + "/cpu.cfs_quota_us", &quota) && read_file(dir + "/cpu.cfs_period_us", &period))
        return parse_cfs_quota(quota, period);
    }
  }
  return CpuQuota();
}

}  // namespace ksa
