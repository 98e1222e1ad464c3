// Host worker threads this process may use: TWTML_HOST_THREADS if set (the
// launchers set it to the CPUs of the rank's NUMA node divided by the ranks
// sharing that node, parallel/affinity.py share_host_threads), else the CPUs
// of the process's affinity mask -- never std::thread::hardware_concurrency(),
// which counts the whole machine: 8 ranks bound 4 to a NUMA node would each
// start a thread per CPU of the machine.
#pragma once

#include <sched.h>

#include <algorithm>
#include <cstdlib>
#include <thread>

namespace twtml {

inline int host_threads() {
  if (const char* e = std::getenv("TWTML_HOST_THREADS")) {
    const int v = std::atoi(e);
    if (v > 0) return v;
  }
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0) return std::max(1, CPU_COUNT(&set));
  return int(std::max(1u, std::thread::hardware_concurrency()));
}

}  // namespace twtml
