// Host-runtime self test for sanitizer builds (SURVEY §5 "Race detection /
// sanitizers"): the multi-threaded synthetic generator, the multi-threaded
// wire packer and its inverse, the special-row pre-lowering and the CPU
// featurizer, run end to end on a batch with Unicode / special rows, and the
// staging task pool (back-to-back and concurrent runs).
// tests/test_host_sanitizers.py compiles it with -fsanitize=address,undefined
// and with -fsanitize=thread (the GPU code is never built with sanitizers
// on this pool).  Exit status 0 = every check passed.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <atomic>
#include <thread>

#include "common/task_pool.h"
#include "host/featurize_cpu.h"
#include "host/synth.h"
#include "host/unicode_lower.h"
#include "host/wire.h"

using namespace twtml;

static int fails = 0;
#define CHECK(cond)                                                          \
  do {                                                                       \
    if (!(cond)) {                                                           \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++fails;                                                               \
    }                                                                        \
  } while (0)

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? size_t(std::atol(argv[1])) : 20000;
  const int threads = argc > 2 ? std::atoi(argv[2]) : 4;
  SynthParams p;
  p.seed = 77;
  p.unicode_fraction = 0.3;
  p.special_fraction = 0.05;
  const size_t cap = synth_max_units(p, n);
  std::vector<uint16_t> text(cap);
  std::vector<int64_t> off(n + 1), sc(5 * n);
  std::vector<uint8_t> rt(n);
  const int64_t units = synth_generate(p, 0, n, text.data(), cap, off.data(), rt.data(), sc.data(), threads);
  CHECK(units > 0 && off[n] == units);

  // determinism across thread counts (rows are a pure function of (seed, index))
  {
    std::vector<uint16_t> t1(cap);
    std::vector<int64_t> o1(n + 1), s1(5 * n);
    std::vector<uint8_t> r1(n);
    const int64_t u1 = synth_generate(p, 0, n, t1.data(), cap, o1.data(), r1.data(), s1.data(), 1);
    CHECK(u1 == units);
    CHECK(std::memcmp(t1.data(), text.data(), sizeof(uint16_t) * size_t(units)) == 0);
    CHECK(o1 == off && s1 == sc && r1 == rt);
  }

  // special rows: full lowering on the host
  std::vector<uint16_t> lt;
  std::vector<int64_t> lo;
  const size_t special = prelower_special_rows(text.data(), off.data(), n, lt, lo);
  CHECK(special == count_special_rows(text.data(), off.data(), n));
  CHECK(lo.size() == n + 1);

  // wire format round trip (multi-threaded pack)
  std::vector<uint8_t> wire(static_cast<size_t>(wire_bound(lo[n], int64_t(n))));
  std::vector<int64_t> woff(n + 1);
  std::vector<uint8_t> flags(n);
  const int64_t bytes = wire_pack(lt.data(), lo.data(), rt.data(), int64_t(n), wire.data(), int64_t(wire.size()),
                                  woff.data(), flags.data(), threads);
  CHECK(bytes > 0 && bytes <= int64_t(wire.size()) && woff[n] == bytes);
  CHECK(wire_units(wire.data(), woff.data(), flags.data(), int64_t(n)) == lo[n]);
  std::vector<uint16_t> back(static_cast<size_t>(lo[n]));
  std::vector<int64_t> boff(n + 1);
  std::vector<uint8_t> brt(n);
  wire_unpack(wire.data(), woff.data(), flags.data(), int64_t(n), back.data(), boff.data(), brt.data());
  CHECK(boff == lo && brt == rt);
  CHECK(std::memcmp(back.data(), lt.data(), sizeof(uint16_t) * size_t(lo[n])) == 0);

  // CPU featurizer: same indices single- and multi-threaded, all in range
  std::vector<int64_t> rows(n);
  for (size_t i = 0; i < n; ++i) rows[i] = int64_t(i);
  for (int hk = 0; hk < 2; ++hk) {
    const int64_t F = hk ? 100000000 : 1000000;
    std::vector<int64_t> ip1, ix1, ip4, ix4;
    featurize_rows_cpu(lt.data(), lo.data(), rows.data(), n, F, hk, ip1, ix1, 1);
    featurize_rows_cpu(lt.data(), lo.data(), rows.data(), n, F, hk, ip4, ix4, threads);
    CHECK(ip1 == ip4 && ix1 == ix4);
    CHECK(ip1.size() == n + 1);
    bool in_range = true;
    for (int64_t v : ix1) in_range &= v >= 0 && v < F;
    CHECK(in_range);
  }
  // per-unit lowering over the whole BMP
  for (uint32_t c = 0; c < 0x10000; ++c) {
    const uint16_t u = uint16_t(c), l = lower_unit(u);
    if (c >= 'A' && c <= 'Z') CHECK(l == c + 32);
  }
  const uint8_t abc[3] = {'a', 'b', 'c'};
  CHECK(murmur3_spark(abc, 3, 42) == murmur3_spark(abc, 3, 42));

  // staging task pool: every task exactly once, runs back to back (a worker
  // waking late for a finished run must not take the next run's tasks) and
  // from two callers at once
  {
    TaskPool& pool = TaskPool::get();
    bool once = true;
    for (int r = 0; r < 2000; ++r) {
      const int nt = 1 + r % 37;
      std::vector<std::atomic<int>> hits(static_cast<size_t>(nt));
      for (auto& h : hits) h.store(0);
      pool.run(nt, [&](int i) { hits[size_t(i)].fetch_add(1); });
      for (auto& h : hits) once &= h.load() == 1;
    }
    CHECK(once);
    std::atomic<long> sum{0};
    auto caller = [&](int base) {
      for (int r = 0; r < 300; ++r) pool.run(16, [&](int i) { sum.fetch_add(base + i); });
    };
    std::thread a(caller, 0), b(caller, 1000);
    a.join();
    b.join();
    CHECK(sum.load() == 300L * (120 + 16 * 1000 + 120));
  }

  if (fails) {
    std::fprintf(stderr, "%d check(s) failed\n", fails);
    return 1;
  }
  std::printf("host selftest ok: rows=%zu units=%lld wire=%lld special=%zu\n", n, (long long)units,
              (long long)bytes, special);
  return 0;
}
