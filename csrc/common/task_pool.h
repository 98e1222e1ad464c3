// Persistent host worker pool for the per-batch staging loops (row words,
// scalar ranges, bit packing).  Spawning fresh std::threads per call cost
// tens of microseconds per thread on every batch -- visible once the device
// work per batch is small (the 2-feature k-means stages a 1M-tweet batch in
// under a millisecond).  Workers are created once, sized to the CPUs this
// process may use (host_threads.h: its share of the GPU's NUMA node), capped
// at kMaxWorkers.  run() blocks until every task is done; the
// caller takes tasks too.  Each run is its own Job (task counter, done
// count), so a worker waking late for a finished run cannot take a task of
// the next one.
#pragma once

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "host_threads.h"

namespace twtml {

class TaskPool {
 public:
  static constexpr int kMaxWorkers = 16;

  static TaskPool& get() {
    static TaskPool pool;
    return pool;
  }

  // Threads that run() uses (workers + the caller).
  int width() const { return int(workers_.size()) + 1; }

  // fn(i) for i in [0, ntasks), spread over the workers and the caller.
  void run(int ntasks, const std::function<void(int)>& fn) {
    if (ntasks <= 0) return;
    if (ntasks == 1 || workers_.empty()) {
      for (int i = 0; i < ntasks; ++i) fn(i);
      return;
    }
    auto job = std::make_shared<Job>(fn, ntasks);
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = job;
      ++gen_;
    }
    cv_.notify_all();
    job->drain();
    std::unique_lock<std::mutex> lk(job->mu);
    job->cv.wait(lk, [&] { return job->done == job->ntasks; });
  }

  ~TaskPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  struct Job {
    Job(const std::function<void(int)>& f, int n) : fn(f), ntasks(n) {}
    const std::function<void(int)>& fn;   // outlives the job's tasks: run() waits for all of them
    const int ntasks;
    std::atomic<int> next{0};
    std::mutex mu;
    std::condition_variable cv;
    int done = 0;
    void drain() {
      int k = 0;
      for (int i = next.fetch_add(1); i < ntasks; i = next.fetch_add(1)) {
        fn(i);
        ++k;
      }
      if (k) {
        std::lock_guard<std::mutex> lk(mu);
        done += k;
        if (done == ntasks) cv.notify_all();
      }
    }
  };

  TaskPool() {
    const int cpus = host_threads();
    const int n = std::max(0, std::min(kMaxWorkers, cpus) - 1);
    for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }

  void loop() {
    uint64_t seen = 0;
    for (;;) {
      std::shared_ptr<Job> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        job = job_;
      }
      if (job) job->drain();
    }
  }

  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::shared_ptr<Job> job_;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace twtml
