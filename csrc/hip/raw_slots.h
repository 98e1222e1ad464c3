// Multi-buffered device copies of raw wire-format batches (csrc/host/wire.h).
//
// submit() enqueues the H2D of a pinned HostBatch on the copy stream into one
// of the engine's raw slots; the compute stream waits on that slot's h2d event and
// records `consumed` once its kernels no longer read the raw bytes, so the
// next H2D into the slot overlaps the rest of the batch's compute.  With three
// slots the host can keep two batches queued ahead of the one being trained,
// so the PCIe copy engine never idles while the host waits for a batch's
// results (double buffering only starts batch t+1's copy once batch t-1 has
// returned to the host).  More slots let the copy engine run further ahead
// while young-model batches (many GD iterations) keep the GPU busier than
// the link: the slack is spent when the model converges and batches run at
// GPU speed (kDefaultRawSlots; LRConfig / KMConfig raw_slots).
#pragma once
#include <hip/hip_runtime.h>

#include <array>
#include <atomic>
#include <mutex>
#include <cstdint>
#include <vector>

#include "kernels.h"

namespace twtml {

struct HostBatch;

// 6: the knee of the headline bench's depth sweep (profiles/r6/raw_slots_sweep.txt:
// 4 -> 237 M tweets/s at p50 10.0 ms, 5 -> 248 M / 12.7 ms, 6 -> 260 M / 14.9 ms,
// 8 -> 261 M / 21.1 ms); the streaming drivers size their own (apps/, scheduler
// prefetch depth + 2)
constexpr int kDefaultRawSlots = 6;
constexpr int kMaxRawSlots = 32;

class RawSlots {
 public:
  RawSlots() = default;
  RawSlots(const RawSlots&) = delete;
  RawSlots& operator=(const RawSlots&) = delete;
  ~RawSlots() { release(); }

  void init(int n_slots, int64_t max_rows, int64_t max_bytes);
  int count() const { return int(slots_.size()); }
  void release();
  // H2D of rows [0, n) / `bytes` text bytes of hb into `slot` on `copy`.
  // scalar_cols: leading scalar columns to copy (the rest stay stale); the
  // batch's scalars must have been encoded with hb.pack_scalars(n)
  // ext_text: the batch's text bytes live outside hb (a registered host
  // buffer, e.g. the receiver's UTF-16 batch): DMA'd from there.
  void submit(const HostBatch& hb, int64_t n, int64_t bytes, int slot, hipStream_t copy,
              int scalar_cols = 5, const uint8_t* ext_text = nullptr);
  // Make `compute` wait for the slot's H2D; returns the device view.
  DevRawBatch acquire(int slot, hipStream_t compute);
  // Rows lowered (special full case mapping) / narrowed by the last acquire
  // of `slot` (device counters, valid once the compute stream passed acquire).
  const int64_t* norm_stats(int slot) const { return slots_[check(slot)].nstats; }
  // Host wait for the slot's last H2D (its staging buffer may be rewritten).
  void wait_h2d(int slot) const;
  // The compute stream is done reading the slot's raw bytes.
  void release_slot(int slot, hipStream_t compute);
  int64_t rows(int slot) const { return slots_[check(slot)].n; }
  int64_t max_rows() const { return max_rows_; }
  // device text bytes per slot: the wire bytes, then room for cesu rows
  // expanded to UTF-16 / narrowed UTF-16 rows (<= 2 bytes per wire byte),
  // then for lowered special rows (<= 2 bytes per wire byte, rows.hip)
  int64_t max_bytes() const { return max_bytes_; }
  // bytes enqueued host-to-device by submit() so far (every copy of a batch)
  int64_t h2d_bytes() const { return h2d_bytes_.load(std::memory_order_relaxed); }
  // TWTML_H2D_TIMING=1 (diagnostics): timing events around every submit's
  // copies; h2d_timeline() synchronises them and returns, per submit in
  // order, (queued, start, end, bytes) with times in ms from the first
  // submit's queued mark.  queued is recorded before the wait for the slot's
  // previous batch (so start - queued is slot back-pressure, and a queued
  // mark after the previous copy's end is the host submitting late).
  std::vector<std::array<double, 4>> h2d_timeline();
  // Timing event on `copy` (diagnostics: the bench marks its timed window's
  // ends with it); h2d_window() returns them in the timeline's time base.
  void h2d_window_mark(hipStream_t copy);
  std::vector<double> h2d_window();

 private:
  int check(int slot) const;
  bool timing_on();   // TWTML_H2D_TIMING, read once
  struct Slot {
    uint8_t* text_base = nullptr;     // [row words prefix | text] (one H2D copy)
    uint8_t* text = nullptr;
    int64_t* offsets = nullptr;
    uint8_t* flags = nullptr;
    int64_t* scalars = nullptr;       // wire-encoded scalar columns (bytes)
    uint16_t* rowpack = nullptr;      // packed row words (when the batch shipped them)
    int64_t* tsum = nullptr;          // unpack scan scratch (per 8192-row tile)
    int64_t* rstart = nullptr;        // cesu batches: row start / end after expansion
    int64_t* rend = nullptr;
    int64_t cesu_rows = 0, wide_rows = 0;
    int64_t* nstats = nullptr;        // [4] rows lowered / narrowed by row_normalize, special-list length
    int32_t* special = nullptr;       // UTF-8 batches: the decoder's kRowSpecial rows
    bool packed = false, utf16 = false, utf8 = false;
    int64_t soff[kScalarCols] = {};
    int64_t sbase[kScalarCols] = {};
    uint8_t sw[kScalarCols] = {};
    int64_t n = 0, bytes = 0;
    hipEvent_t h2d_done = nullptr, consumed = nullptr;
    bool used = false;
  };
  std::vector<Slot> slots_;
  int64_t max_rows_ = 0, max_bytes_ = 0;
  std::atomic<int64_t> h2d_bytes_{0};
  struct H2DMark {
    hipEvent_t q = nullptr, a = nullptr, b = nullptr;
    int64_t bytes = 0;
  };
  std::mutex tl_mu_;
  std::vector<H2DMark> tl_;
  std::vector<hipEvent_t> win_;
  int tl_on_ = -1;   // TWTML_H2D_TIMING, read once
  DevCaseTables case_{};
};

}  // namespace twtml
