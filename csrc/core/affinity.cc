#include "affinity.h"

#include <pthread.h>
#include <sched.h>

namespace ksa {

bool pin_current_thread(const CpuList& cpus) {
  if (cpus.empty()) return true;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus)
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
  return pthread_setaffinity_np(pthread_self(), sizeof set, &set) == 0;
}

}  // namespace ksa
