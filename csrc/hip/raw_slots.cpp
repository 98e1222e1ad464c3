#include "raw_slots.h"
#include "alloc.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>

#include "engine.h"

namespace twtml {

template <typename T>
static T* slot_alloc(size_t n) {
  return static_cast<T*>(dev_alloc(n * sizeof(T)));
}

int RawSlots::check(int slot) const {
  if (slot < 0 || slot >= int(slots_.size())) throw std::invalid_argument("slot must be in [0, raw slots)");
  return slot;
}

void RawSlots::init(int n_slots, int64_t max_rows, int64_t max_bytes) {
  if (max_rows < 0 || max_bytes < 0) throw std::invalid_argument("RawSlots: negative capacity");
  if (n_slots < 2 || n_slots > kMaxRawSlots) throw std::invalid_argument("RawSlots: 2 .. 32 slots");
  release();
  slots_.assign(size_t(n_slots), Slot{});
  max_rows_ = max_rows;
  max_bytes_ = max_bytes;
  for (auto& s : slots_) {
    // wire bytes + cesu rows expanded behind them (UTF-16: at most twice the
    // wire bytes of those rows); slack: featurize over-reads <= 80 B
    const size_t pre = (rowpack_prefix(max_rows) + 255) & ~size_t(255);
    s.text_base = slot_alloc<uint8_t>(pre + 5 * size_t(max_bytes) + 256);
    s.nstats = slot_alloc<int64_t>(4);
    s.special = slot_alloc<int32_t>(size_t(max_rows) + 1);
    s.text = s.text_base + pre;
    s.offsets = slot_alloc<int64_t>(size_t(max_rows) + 1);
    s.flags = slot_alloc<uint8_t>(size_t(max_rows));
    s.scalars = slot_alloc<int64_t>(5 * size_t(max_rows));
    s.tsum = slot_alloc<int64_t>(size_t(max_rows) / 8192 + 2);
    s.rstart = slot_alloc<int64_t>(size_t(max_rows) + 1);
    s.rend = slot_alloc<int64_t>(size_t(max_rows) + 1);
    TWTML_HIP_CHECK(hipEventCreateWithFlags(&s.h2d_done, hipEventDisableTiming));
    TWTML_HIP_CHECK(hipEventCreateWithFlags(&s.consumed, hipEventDisableTiming));
  }
  upload_case_tables(&case_);
}

std::vector<std::array<double, 4>> RawSlots::h2d_timeline() {
  std::lock_guard<std::mutex> lk(tl_mu_);
  std::vector<std::array<double, 4>> out;
  if (tl_.empty()) return out;
  TWTML_HIP_CHECK(hipEventSynchronize(tl_.back().b));
  for (const H2DMark& m : tl_) {
    float q = 0.f, a = 0.f, b = 0.f;
    TWTML_HIP_CHECK(hipEventElapsedTime(&q, tl_.front().q, m.q));
    TWTML_HIP_CHECK(hipEventElapsedTime(&a, tl_.front().q, m.a));
    TWTML_HIP_CHECK(hipEventElapsedTime(&b, tl_.front().q, m.b));
    out.push_back({double(q), double(a), double(b), double(m.bytes)});
  }
  return out;
}

bool RawSlots::timing_on() {
  if (tl_on_ < 0) {
    const char* e = std::getenv("TWTML_H2D_TIMING");
    tl_on_ = e && e[0] == '1' ? 1 : 0;
  }
  return tl_on_ == 1;
}

void RawSlots::h2d_window_mark(hipStream_t copy) {
  if (!timing_on()) return;
  hipEvent_t e = nullptr;
  TWTML_HIP_CHECK(hipEventCreate(&e));
  TWTML_HIP_CHECK(hipEventRecord(e, copy));
  std::lock_guard<std::mutex> lk(tl_mu_);
  win_.push_back(e);
}

std::vector<double> RawSlots::h2d_window() {
  std::lock_guard<std::mutex> lk(tl_mu_);
  std::vector<double> out;
  if (tl_.empty()) return out;
  for (hipEvent_t e : win_) {
    TWTML_HIP_CHECK(hipEventSynchronize(e));
    float t = 0.f;
    TWTML_HIP_CHECK(hipEventElapsedTime(&t, tl_.front().q, e));
    out.push_back(double(t));
  }
  return out;
}

void RawSlots::release() {
  for (hipEvent_t e : win_) (void)hipEventDestroy(e);
  win_.clear();
  for (H2DMark& m : tl_) {
    if (m.q) (void)hipEventDestroy(m.q);
    if (m.a) (void)hipEventDestroy(m.a);
    if (m.b) (void)hipEventDestroy(m.b);
  }
  tl_.clear();
  for (auto& s : slots_) {
    if (s.text_base) (void)hipFree(s.text_base);
    if (s.offsets) (void)hipFree(s.offsets);
    if (s.flags) (void)hipFree(s.flags);
    if (s.scalars) (void)hipFree(s.scalars);
    if (s.tsum) (void)hipFree(s.tsum);
    if (s.rstart) (void)hipFree(s.rstart);
    if (s.rend) (void)hipFree(s.rend);
    if (s.nstats) (void)hipFree(s.nstats);
    if (s.special) (void)hipFree(s.special);
    if (s.h2d_done) (void)hipEventDestroy(s.h2d_done);
    if (s.consumed) (void)hipEventDestroy(s.consumed);
    s = Slot{};
  }
  slots_.clear();
  free_case_tables(&case_);
}

void RawSlots::submit(const HostBatch& hb, int64_t n, int64_t bytes, int slot, hipStream_t copy,
                      int scalar_cols, const uint8_t* ext_text) {
  Slot& s = slots_[check(slot)];
  if (scalar_cols < 1 || scalar_cols > 5) throw std::invalid_argument("scalar_cols must be in [1, 5]");
  if (n < 0 || n > max_rows_ || n > hb.max_rows) throw std::invalid_argument("rows exceed capacity");
  if (bytes < 0 || bytes > max_bytes_ || (!ext_text && bytes > hb.max_bytes))
    throw std::invalid_argument("text bytes exceed capacity");
  if (hb.offsets[0] != 0 || hb.offsets[n] != bytes) throw std::invalid_argument("offsets[n] != bytes");
  if (n > 0 && hb.spacked_n != n) throw std::logic_error("HostBatch scalars not packed for this row count");
  if (n > 0 && hb.spacked_cols < scalar_cols)
    throw std::logic_error("HostBatch packed fewer scalar columns than this engine reads");
  if (n > 0 && hb.rows_scanned_n != n) throw std::logic_error("HostBatch rows not packed (pack_rows) for this row count");
  const bool timed = timing_on();
  H2DMark mark;
  if (timed) {   // queued: before the slot wait
    TWTML_HIP_CHECK(hipEventCreate(&mark.q));
    TWTML_HIP_CHECK(hipEventCreate(&mark.a));
    TWTML_HIP_CHECK(hipEventCreate(&mark.b));
    TWTML_HIP_CHECK(hipEventRecord(mark.q, copy));
  }
  // wait until the compute stream has finished reading this slot
  if (s.used) TWTML_HIP_CHECK(hipStreamWaitEvent(copy, s.consumed, 0));
  // after the slot wait: a..b times the copies themselves
  if (timed) TWTML_HIP_CHECK(hipEventRecord(mark.a, copy));
  // offsets + flags: one u16 per row when the batch was packed (the compute
  // stream rebuilds both in acquire), else as they are.  Packed row words sit
  // right before the text on both sides and travel with it (below).
  const bool packed = n > 0 && hb.rowpacked_n == n;
  const size_t pre = packed ? rowpack_prefix(n) : 0;
  if (packed && reinterpret_cast<const uint8_t*>(hb.rowpack) + pre != hb.text)
    throw std::logic_error("HostBatch row words not adjacent to the text");
  s.rowpack = reinterpret_cast<uint16_t*>(s.text - pre);
  if (!packed) {
    TWTML_HIP_CHECK(hipMemcpyAsync(s.offsets, hb.offsets, sizeof(int64_t) * size_t(n + 1),
                                   hipMemcpyHostToDevice, copy));
  }
  if (n > 0) {
    if (!packed)
      TWTML_HIP_CHECK(hipMemcpyAsync(s.flags, hb.flags, size_t(n), hipMemcpyHostToDevice, copy));
    // wire-encoded columns are consecutive, so the leading scalar_cols of
    // them are one contiguous copy; it must fit both the host block's spack
    // region (its tail) and the slot's 5 x 8 B per row
    const int64_t sbytes = hb.soff[scalar_cols];
    const uint8_t* hend = static_cast<const uint8_t*>(hb.base) + hb.bytes;
    if (sbytes < 0 || sbytes > 5 * int64_t(sizeof(int64_t)) * n || hb.spack + sbytes > hend)
      throw std::logic_error("RawSlots::submit: packed scalar bytes out of range (" + std::to_string(sbytes) +
                             " for " + std::to_string(n) + " rows)");
    TWTML_HIP_CHECK(hipMemcpyAsync(s.scalars, hb.spack, size_t(sbytes), hipMemcpyHostToDevice, copy));
    TWTML_DEBUG_POINT("raw slot H2D: row flags + packed scalars", copy);
  }
  // row words + text last: the small copy goes first, so the gap the copy
  // engine leaves after a long transfer falls between batches, not inside one
  if (ext_text) {   // row words from the staging buffer, text from the caller's buffer
    if (pre > 0)
      TWTML_HIP_CHECK(hipMemcpyAsync(s.text - pre, hb.text - pre, pre, hipMemcpyHostToDevice, copy));
    if (bytes > 0)
      TWTML_HIP_CHECK(hipMemcpyAsync(s.text, ext_text, size_t(bytes), hipMemcpyHostToDevice, copy));
  } else if (bytes > 0 || pre > 0) {
    TWTML_HIP_CHECK(hipMemcpyAsync(s.text - pre, hb.text - pre, pre + size_t(bytes),
                                   hipMemcpyHostToDevice, copy));
  }
  TWTML_DEBUG_POINT(ext_text ? "raw slot H2D: row words + text (external buffer)" : "raw slot H2D: row words + text",
                    copy);
  TWTML_HIP_CHECK(hipEventRecord(s.h2d_done, copy));
  int64_t moved = int64_t(pre) + bytes;
  if (!packed) moved += int64_t(sizeof(int64_t)) * (n + 1) + (n > 0 ? n : 0);
  if (n > 0) moved += hb.soff[scalar_cols];
  h2d_bytes_.fetch_add(moved, std::memory_order_relaxed);
  if (timed) {
    TWTML_HIP_CHECK(hipEventRecord(mark.b, copy));
    mark.bytes = moved;
    std::lock_guard<std::mutex> lk(tl_mu_);
    tl_.push_back(mark);
  }
  for (int c = 0; c < kScalarCols; ++c) {
    s.soff[c] = hb.soff[c];
    s.sbase[c] = hb.sbase[c];
    s.sw[c] = hb.sw[c];
  }
  s.packed = packed;
  s.cesu_rows = n > 0 ? hb.cesu_rows : 0;
  s.wide_rows = n > 0 ? hb.wide_rows : 0;
  s.utf16 = n > 0 && hb.utf16;
  s.utf8 = n > 0 && hb.utf8;
  s.n = n;
  s.bytes = bytes;
  s.used = true;
}

DevRawBatch RawSlots::acquire(int slot, hipStream_t compute) {
  Slot& s = slots_[check(slot)];
  if (!s.used) throw std::logic_error("process() on a slot that was never submitted");
  TWTML_HIP_CHECK(hipStreamWaitEvent(compute, s.h2d_done, 0));
  if (s.packed) launch_unpack_rows(s.rowpack, s.n, s.offsets, s.flags, s.tsum, compute);
  DevRawBatch b{};
  b.text = s.text;
  b.offsets = s.offsets;
  b.oend = s.offsets + 1;
  b.flags = s.flags;
  const int64_t tail = (s.bytes + 15) / 16 * 16;
  TWTML_HIP_CHECK(hipMemsetAsync(s.nstats, 0, 4 * sizeof(int64_t), compute));
  // UTF-8 batches: the decoder flags the candidate special rows (and narrows
  // the Latin-1 ones itself) and lists them; only those are walked, one wave
  // per row (launch_row_special).  TWTML_NORMALIZE_ALL=1 scans every wide
  // row instead (A/B); TWTML_NORMALIZE_LIST=0 walks the flagged rows by
  // 64-row group (the round-5 pass, A/B).
  static const bool scan_all = [] {
    const char* e = std::getenv("TWTML_NORMALIZE_ALL");
    return e && e[0] == '1';
  }();
  static const bool by_list = [] {
    const char* e = std::getenv("TWTML_NORMALIZE_LIST");
    return !(e && e[0] == '0');
  }();
  const bool flagged_only = s.utf8 && !s.utf16 && s.cesu_rows > 0 && !scan_all;
  const bool listed = flagged_only && by_list;
  if (s.cesu_rows > 0) {   // expand cesu / UTF-8 rows behind the wire bytes (16-byte aligned)
    launch_cesu_expand(s.text, s.offsets, s.flags, s.n, tail, s.rstart, s.rend, s.nstats, compute,
                       listed ? s.special : nullptr);
    b.offsets = s.rstart;
    b.oend = s.rend;
  }
  const int64_t lower_base = tail + 2 * ((s.bytes + 15) / 16 * 16);
  if (listed) {
    launch_row_special(s.text, s.offsets, s.rstart, s.rend, s.flags, s.special, s.n, tail, lower_base, case_,
                       s.nstats, compute);
  } else if (s.utf16 || s.cesu_rows > 0 || s.wide_rows > 0) {
    // special rows -> fully lower-cased UTF-16; UTF-16 / UTF-8 batches: Latin-1
    // rows narrowed (a decoded UTF-8 row in place: byte i <- unit i, forward)
    launch_row_normalize(s.text, s.offsets, b.offsets, b.oend, s.flags, s.rstart, s.rend, s.n, tail,
                         lower_base, s.utf16 || s.utf8, case_, s.nstats, compute, flagged_only);
    b.offsets = s.rstart;
    b.oend = s.rend;
  }
  const uint8_t* sc = reinterpret_cast<const uint8_t*>(s.scalars);
  for (int c = 0; c < kScalarCols; ++c) {
    b.scol[c] = sc + s.soff[c];
    b.sbase[c] = s.sbase[c];
    b.sw[c] = s.sw[c];
  }
  b.n = s.n;
  b.bytes = s.bytes;
  return b;
}

void RawSlots::wait_h2d(int slot) const {
  const Slot& s = slots_[check(slot)];
  if (s.used) TWTML_HIP_CHECK(hipEventSynchronize(s.h2d_done));
}

void RawSlots::release_slot(int slot, hipStream_t compute) {
  TWTML_HIP_CHECK(hipEventRecord(slots_[check(slot)].consumed, compute));
}

}  // namespace twtml
