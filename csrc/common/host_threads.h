// Host worker threads this process may use: TWTML_HOST_THREADS if set (the
// launchers set it to the CPUs of the rank's NUMA node divided by the ranks
// sharing that node, parallel/affinity.py share_host_threads), else the CPUs
// of the process's affinity mask capped by its cgroup CPU quota -- never
// std::thread::hardware_concurrency(), which counts the whole machine: 8
// ranks bound 4 to a NUMA node would each start a thread per CPU of the
// machine.  The quota matters as much as the mask: a container may see 256
// CPUs and be allowed 16, and threads past the quota get the whole cgroup
// throttled for the rest of a 100 ms CFS period (measured on the MI355X
// boxes: tools/diag/plot_stall.py, cgroup cpu.stat).
#pragma once

#include <sched.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <thread>

namespace twtml {

// CPUs allowed by the cgroup (v2 cpu.max, else v1 cfs quota), rounded up; 0 = no limit
inline int cgroup_cpu_limit() {
  long long quota = -1, period = 0;
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    if (std::fscanf(f, "%31s %lld", q, &period) == 2 && q[0] != 'm') quota = std::atoll(q);
    std::fclose(f);
  } else if (FILE* f1 = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
    if (std::fscanf(f1, "%lld", &quota) != 1) quota = -1;
    std::fclose(f1);
    if (FILE* f2 = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
      if (std::fscanf(f2, "%lld", &period) != 1) period = 0;
      std::fclose(f2);
    }
  }
  if (quota <= 0 || period <= 0) return 0;
  return int(std::max<long long>(1, (quota + period - 1) / period));
}

inline int host_threads() {
  if (const char* e = std::getenv("TWTML_HOST_THREADS")) {
    const int v = std::atoi(e);
    if (v > 0) return v;
  }
  int n = int(std::max(1u, std::thread::hardware_concurrency()));
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = std::max(1, CPU_COUNT(&set));
  const int lim = cgroup_cpu_limit();
  return lim > 0 ? std::min(n, lim) : n;
}

}  // namespace twtml
