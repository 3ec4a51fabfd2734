// Loopback round-trip probe: N clients, each with its own echo server process, as N threads of
// one process or as N processes -- the same placement either way. Separates what the kernel
// does differently for threads of one process (shared mm, files, signal struct) from anything in
// the autoscaler's own code. Used to attribute the multi-queue latency rise (profiles/README.md).
//
//   loopback_probe <threads|threads-unshare|procs> <n> <iterations> <cpu-spec>
// threads-unshare: each client thread first takes a private file table (unshare(CLONE_FILES)),
// to test whether the shared fd table is what threads pay for.
// cpu-spec: "client0:server0,client1:server1,..." (CPU numbers; "-" = unpinned)
// Prints one JSON line per client: {"client":i,"p50_ns":...,"p90_ns":...}.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <sched.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

void pin(int cpu) {
  if (cpu < 0) return;
  cpu_set_t s;
  CPU_ZERO(&s);
  CPU_SET(cpu, &s);
  sched_setaffinity(0, sizeof s, &s);
}

// Blocking echo server on an ephemeral port; writes the port to `port_fd` and serves one client.
void echo_server(int cpu, int port_fd) {
  pin(cpu);
  int ls = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  bind(ls, reinterpret_cast<sockaddr*>(&a), sizeof a);
  listen(ls, 1);
  socklen_t len = sizeof a;
  getsockname(ls, reinterpret_cast<sockaddr*>(&a), &len);
  int port = ntohs(a.sin_port);
  if (write(port_fd, &port, sizeof port) != sizeof port) _exit(1);
  close(port_fd);
  int c = accept(ls, nullptr, nullptr);
  int one = 1;
  setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  char buf[4096];
  while (true) {
    ssize_t r = recv(c, buf, sizeof buf, 0);
    if (r <= 0) break;
    if (send(c, buf, static_cast<size_t>(r), MSG_NOSIGNAL) != r) break;
  }
  _exit(0);
}

// One client: connect, then `iters` 64-byte request/response round trips with a busy-polled
// receive (the autoscaler's --busy-poll path); returns sorted RTTs.
std::vector<int64_t> client(int cpu, int port, int iters, bool unshare_files = false) {
  pin(cpu);
  if (unshare_files && ::unshare(CLONE_FILES) != 0) return {};
  int s = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (connect(s, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) return {};
  int one = 1;
  setsockopt(s, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  char req[64];
  std::memset(req, 'x', sizeof req);
  char buf[4096];
  std::vector<int64_t> rtt;
  rtt.reserve(static_cast<size_t>(iters));
  for (int i = 0; i < iters + 1000; ++i) {
    const int64_t t0 = now_ns();
    send(s, req, sizeof req, MSG_NOSIGNAL);
    size_t got = 0;
    while (got < sizeof req) {
      ssize_t r = recv(s, buf, sizeof buf, MSG_DONTWAIT);
      if (r > 0) got += static_cast<size_t>(r);
      else if (r == 0 || (errno != EAGAIN && errno != EWOULDBLOCK)) return rtt;
    }
    if (i >= 1000) rtt.push_back(now_ns() - t0);  // first 1000: warm-up
  }
  close(s);
  std::sort(rtt.begin(), rtt.end());
  return rtt;
}

void report(int i, const std::vector<int64_t>& v) {
  if (v.empty()) {
    std::printf("{\"client\":%d,\"error\":true}\n", i);
  } else {
    std::printf("{\"client\":%d,\"p50_ns\":%lld,\"p90_ns\":%lld}\n", i, static_cast<long long>(v[v.size() / 2]),
                static_cast<long long>(v[v.size() * 9 / 10]));
  }
  std::fflush(stdout);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s threads|procs n iterations cpu-spec\n", argv[0]);
    return 2;
  }
  const bool unshare_files = std::strcmp(argv[1], "threads-unshare") == 0;
  const bool threads = std::strcmp(argv[1], "threads") == 0 || unshare_files;
  const int n = std::atoi(argv[2]);
  const int iters = std::atoi(argv[3]);
  std::vector<int> ccpu(static_cast<size_t>(n), -1), scpu(static_cast<size_t>(n), -1);
  {
    std::string spec = argv[4];
    size_t pos = 0;
    for (int i = 0; i < n && pos <= spec.size(); ++i) {
      size_t e = spec.find(',', pos);
      std::string item = spec.substr(pos, e == std::string::npos ? std::string::npos : e - pos);
      size_t colon = item.find(':');
      if (colon != std::string::npos) {
        if (item[0] != '-') ccpu[static_cast<size_t>(i)] = std::atoi(item.c_str());
        if (item[colon + 1] != '-') scpu[static_cast<size_t>(i)] = std::atoi(item.c_str() + colon + 1);
      }
      if (e == std::string::npos) break;
      pos = e + 1;
    }
  }
  std::vector<int> ports(static_cast<size_t>(n));
  std::vector<pid_t> servers;
  for (int i = 0; i < n; ++i) {
    int p[2];
    if (pipe(p) != 0) return 1;
    pid_t pid = fork();
    if (pid == 0) {
      close(p[0]);
      echo_server(scpu[static_cast<size_t>(i)], p[1]);
    }
    close(p[1]);
    if (read(p[0], &ports[static_cast<size_t>(i)], sizeof(int)) != sizeof(int)) return 1;
    close(p[0]);
    servers.push_back(pid);
  }
  if (threads) {
    std::vector<std::vector<int64_t>> res(static_cast<size_t>(n));
    std::vector<std::thread> ts;
    for (int i = 0; i < n; ++i)
      ts.emplace_back([&, i] {
        res[static_cast<size_t>(i)] =
            client(ccpu[static_cast<size_t>(i)], ports[static_cast<size_t>(i)], iters, unshare_files);
      });
    for (auto& t : ts) t.join();
    for (int i = 0; i < n; ++i) report(i, res[static_cast<size_t>(i)]);
  } else {
    std::vector<pid_t> kids;
    for (int i = 0; i < n; ++i) {
      pid_t pid = fork();
      if (pid == 0) {
        auto v = client(ccpu[static_cast<size_t>(i)], ports[static_cast<size_t>(i)], iters);
        report(i, v);
        _exit(0);
      }
      kids.push_back(pid);
    }
    for (pid_t k : kids) waitpid(k, nullptr, 0);
  }
  for (pid_t s : servers) waitpid(s, nullptr, 0);
  return 0;
}
