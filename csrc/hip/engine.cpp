// LREngine implementation; see engine.h.
#include "engine.h"
#include "../common/task_pool.h"
#include "alloc.h"
#include "trace.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace twtml {

void launch_batch_init(const DevSgd& d, double m_global, int n_loss, hipStream_t s);
void launch_plot_sample(const float* pred, const float* real, int64_t n, int64_t P, float* out, hipStream_t s);

HostBatch::HostBatch(int64_t rows, int64_t text_bytes) : max_rows(rows), max_bytes(text_bytes) {
  if (rows < 0 || text_bytes < 0) throw std::invalid_argument("HostBatch: negative capacity");
  auto up = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t t = up(size_t(text_bytes));
  const size_t o = up(sizeof(int64_t) * size_t(rows + 1));
  const size_t r = up(size_t(rows));
  const size_t sc = up(sizeof(int64_t) * 5 * size_t(rows));
  const size_t rp = up(sizeof(uint16_t) * size_t(rows) + 16);
  bytes = rp + t + o + r + 2 * sc;
  TWTML_HIP_CHECK(hipHostMalloc(&base, bytes, hipHostMallocDefault));
  // [row words | text | offsets | flags | scalars | spack]: the row words of
  // n rows end right before the text (pack_rows), so both cross PCIe as one copy
  char* p = static_cast<char*>(base);
  text = reinterpret_cast<uint8_t*>(p + rp);
  rowpack = reinterpret_cast<uint16_t*>(p);
  p += rp;
  offsets = reinterpret_cast<int64_t*>(p + t);
  flags = reinterpret_cast<uint8_t*>(p + t + o);
  scalars = reinterpret_cast<int64_t*>(p + t + o + r);
  spack = reinterpret_cast<uint8_t*>(p + t + o + r + sc);
  offsets[0] = 0;
}

void HostBatch::pack_scalars(int64_t n, const int64_t* src, const int64_t* range) {
  if (n < 0 || n > max_rows) throw std::invalid_argument("pack_scalars: bad row count");
  if (!src) src = scalars;
  int64_t lo[kScalarCols], hi[kScalarCols];
  const int ncols = std::max(1, std::min(scalar_cols, kScalarCols));
  TaskPool& pool = TaskPool::get();
  // chunks of whole 32-row words: a column's chunks own disjoint words of its stream
  const int per_col = int(std::max<int64_t>(1, std::min<int64_t>((pool.width() + ncols - 1) / ncols,
                                                                   (n + 65535) / 65536)));
  const int64_t part = std::max<int64_t>(32, (n / per_col + 31) / 32 * 32);
  const int nparts = int(std::max<int64_t>(1, (n + part - 1) / part));
  std::vector<int64_t> plo(size_t(ncols) * nparts), phi(size_t(ncols) * nparts);
  if (range && n > 0) {   // the receiver's bounds: one pass (checked while packing)
    for (int c = 0; c < ncols; ++c) {
      plo[size_t(c) * nparts] = range[c];
      phi[size_t(c) * nparts] = range[kScalarCols + c];
      for (int k = 1; k < nparts; ++k) {
        plo[size_t(c) * nparts + k] = range[c];
        phi[size_t(c) * nparts + k] = range[kScalarCols + c];
      }
    }
  } else pool.run(ncols * nparts, [&](int task) {
    const int c = task / nparts;
    const int64_t i0 = int64_t(task % nparts) * part, i1 = std::min(n, i0 + part);
    const int64_t* v = src + int64_t(c) * n;
    int64_t a = i0 < i1 ? v[i0] : INT64_MAX, b = i0 < i1 ? v[i0] : INT64_MIN;
    for (int64_t i = i0 + 1; i < i1; ++i) { a = std::min(a, v[i]); b = std::max(b, v[i]); }
    plo[size_t(task)] = a;
    phi[size_t(task)] = b;
  });
  for (int c = 0; c < ncols; ++c) {
    lo[c] = hi[c] = 0;
    if (n == 0) continue;
    lo[c] = INT64_MAX;
    hi[c] = INT64_MIN;
    for (int k = 0; k < nparts; ++k) {
      lo[c] = std::min(lo[c], plo[size_t(c) * nparts + k]);
      hi[c] = std::max(hi[c], phi[size_t(c) * nparts + k]);
    }
  }
  for (int c = ncols; c < kScalarCols; ++c) lo[c] = hi[c] = 0;   // not shipped
  soff[0] = 0;
  for (int c = 0; c < kScalarCols; ++c) {
    // range in unsigned arithmetic (hi - lo may overflow int64); a column
    // ships as a bit stream of `bits`-bit offsets from its base, or raw int64
    const uint64_t span = uint64_t(hi[c]) - uint64_t(lo[c]);
    const int bits = span > uint64_t(UINT32_MAX) ? 64 : span == 0 ? 1 : 64 - __builtin_clzll(span);
    sw[c] = uint8_t(bits);
    sbase[c] = bits == 64 ? 0 : lo[c];
    // + one u32 of slack: the device reads two consecutive words per value
    const int64_t cb = c >= ncols ? 0 : bits == 64 ? 8 * n : ((n * bits + 31) / 32 + 1) * 4;
    soff[c + 1] = soff[c] + ((cb + 7) & ~int64_t(7));   // columns 8-B aligned
  }
  // rows [i0, i1) of column c; chunk boundaries are multiples of 32 rows, so
  // chunks own whole 32-bit words of the stream.  Returns false if a value
  // lies outside the column's encoding (a range hint that does not hold).
  auto put = [&](int c, int64_t i0, int64_t i1) -> bool {
    const int64_t* v = src + int64_t(c) * n;
    uint8_t* o = spack + soff[c];
    const int bits = sw[c];
    if (bits == 64) {
      std::memcpy(o + 8 * i0, v + i0, sizeof(int64_t) * size_t(i1 - i0));
      return true;
    }
    // word-at-a-time writer: the chunk starts on a word boundary
    uint32_t* out = reinterpret_cast<uint32_t*>(o) + ((i0 * bits) >> 5);
    const uint64_t b = uint64_t(sbase[c]);
    uint64_t acc = 0, over = 0;
    int nb = 0;
    for (int64_t i = i0; i < i1; ++i) {
      const uint64_t x = uint64_t(v[i]) - b;
      over |= x >> bits;   // bits < 64 here
      acc |= x << nb;
      nb += bits;
      if (nb >= 32) {
        *out++ = uint32_t(acc);
        acc >>= 32;
        nb -= 32;
      }
    }
    if (nb > 0) *out++ = uint32_t(acc);
    if (i1 == n)   // the column's slack words
      for (uint32_t* end = reinterpret_cast<uint32_t*>(o + (soff[c + 1] - soff[c])); out < end;) *out++ = 0u;
    return over == 0;
  };
  std::vector<uint8_t> fits(size_t(ncols) * nparts, 1);
  pool.run(ncols * nparts, [&](int task) {
    const int c = task / nparts;
    const int64_t i0 = int64_t(task % nparts) * part;
    fits[size_t(task)] = put(c, i0, std::min(n, i0 + part)) ? 1 : 0;
  });
  if (range && n > 0) {
    bool ok = true;
    for (auto f : fits) ok = ok && f;
    if (!ok) {   // the hint did not hold: the exact two-pass encoding
      ++range_misses;
      pack_scalars(n, src, nullptr);
      return;
    }
    ++range_hits;
  }
  spacked_n = n;
  spacked_cols = ncols;
}

bool HostBatch::pack_rows(int64_t n) {
  if (n < 0 || n > max_rows) throw std::invalid_argument("pack_rows: bad row count");
  rowpacked_n = -1;
  rowpack = reinterpret_cast<uint16_t*>(text - rowpack_prefix(n));
  int64_t cesu = 0, wide = 0;
  bool fits = true;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t len = offsets[i + 1] - offsets[i];
    cesu += (flags[i] & kRowCesu) ? 1 : 0;
    wide += (flags[i] & kRowWide) ? 1 : 0;
    if (len < 0 || len >= (int64_t(1) << kRowLenBits)) fits = false;
    else rowpack[i] = uint16_t(len | (int64_t(flags[i] & 7) << kRowLenBits));
  }
  cesu_rows = cesu;
  wide_rows = wide;
  utf16 = false;
  utf8 = false;
  rows_scanned_n = n;
  if (fits) rowpacked_n = n;
  return fits;
}

// Raw staging shared by the UTF-16 and UTF-8 ingest modes: row words
// (byte length | flags), offsets, packed scalars, and optionally the text.
// `scale` is the bytes per offset unit (2: UTF-16 units, 1: UTF-8 bytes),
// `row_flags` the wire flags every row carries besides the retweet bit.
void HostBatch::load_raw(const uint8_t* t, const int64_t* uoff, int64_t scale, uint8_t row_flags,
                         const uint8_t* is_rt, const int64_t* sc, int64_t n, bool copy_text, int threads,
                         const int64_t* range) {
  if (n < 0 || n > max_rows) throw std::invalid_argument("load: bad row count");
  const int64_t bytes = n > 0 ? scale * (uoff[n] - uoff[0]) : 0;
  if (copy_text && bytes > max_bytes) throw std::invalid_argument("load: text exceeds staging capacity");
  if (n > 0 && uoff[0] != 0) throw std::invalid_argument("load: offsets must start at 0");
  rowpacked_n = -1;
  rowpack = reinterpret_cast<uint16_t*>(text - rowpack_prefix(n));
  TaskPool& pool = TaskPool::get();
  if (threads <= 0) threads = pool.width();
  const int T = int(std::max<int64_t>(1, std::min<int64_t>(threads, (n + 65535) / 65536)));
  std::vector<uint8_t> fit(size_t(T), 1);
  // offsets / flags: the device rebuilds both from the row words of a packed
  // batch, so the DMA path (text not copied) writes them only when a row does
  // not fit a row word; a copied batch keeps them for as_raw()
  auto host_rows = [&](int64_t r0, int64_t r1) {
    for (int64_t i = r0; i < r1; ++i) {
      offsets[i + 1] = scale * uoff[i + 1];
      flags[i] = uint8_t((is_rt[i] ? kRowRetweet : 0) | row_flags);
    }
  };
  auto rows = [&](int c) {
    const int64_t r0 = n * c / T, r1 = n * (c + 1) / T;
    bool ok = true;
    for (int64_t i = r0; i < r1; ++i) {
      const int64_t len = scale * (uoff[i + 1] - uoff[i]);
      const uint32_t f = (is_rt[i] ? kRowRetweet : 0) | row_flags;
      if (len < 0 || len >= (int64_t(1) << kRowLenBits)) ok = false;
      else rowpack[i] = uint16_t(len | (int64_t(f) << kRowLenBits));
    }
    fit[size_t(c)] = ok ? 1 : 0;
    if (copy_text) {   // this thread's share of the text bytes
      host_rows(r0, r1);
      const int64_t b0 = scale * uoff[r0], b1 = scale * uoff[r1];
      if (b1 > b0) std::memcpy(text + b0, t + b0, size_t(b1 - b0));
    }
  };
  pool.run(T, rows);
  bool all = true;
  for (auto f : fit) all = all && f;
  if (!copy_text && !all) pool.run(T, [&](int c) { host_rows(n * c / T, n * (c + 1) / T); });
  offsets[0] = 0;
  offsets[n] = scale * uoff[n];
  pack_scalars(n, sc, range);
  rows_scanned_n = n;
  if (all) rowpacked_n = n;
}

void HostBatch::load_utf16(const uint16_t* t, const int64_t* uoff, const uint8_t* is_rt, const int64_t* sc,
                           int64_t n, bool copy_text, int threads, const int64_t* range) {
  load_raw(reinterpret_cast<const uint8_t*>(t), uoff, 2, kRowWide, is_rt, sc, n, copy_text, threads, range);
  cesu_rows = 0;
  wide_rows = n;
  utf16 = true;
  utf8 = false;
}

// UTF-8 as the network delivers tweet text: every row is flagged cesu (the
// device decoder handles UTF-8, incl. 4-byte sequences); the device keeps
// ASCII rows as they are and narrows decoded Latin-1 rows.
void HostBatch::load_utf8(const uint8_t* t, const int64_t* boff, const uint8_t* is_rt, const int64_t* sc,
                          int64_t n, bool copy_text, int threads, const int64_t* range) {
  load_raw(t, boff, 1, kRowCesu, is_rt, sc, n, copy_text, threads, range);
  cesu_rows = n;
  wide_rows = 0;
  utf16 = false;
  utf8 = true;
}

HostBatch::~HostBatch() {
  if (base) (void)hipHostFree(base);
}

template <typename T>
static T* dmalloc(size_t n) {
  return static_cast<T*>(dev_alloc(n * sizeof(T)));
}

LREngine::LREngine(int device, const LRConfig& cfg, std::shared_ptr<Comm> comm)
    : device_(device), cfg_(cfg), comm_(std::move(comm)) {
  if (cfg_.num_text_features <= 0) throw std::invalid_argument("numTextFeatures must be > 0");
  if (cfg_.max_rows <= 0 || cfg_.max_units < 0) throw std::invalid_argument("bad capacity");
  if (cfg_.max_rows >= (int64_t(1) << 31)) throw std::invalid_argument("max_rows must be < 2^31");
  if (cfg_.fraction <= 0.0 || cfg_.fraction > 1.0 + 1e-12)
    throw std::invalid_argument("miniBatchFraction must be in (0, 1]");
  if (const char* v = std::getenv("TWTML_FORCE_TIERED")) force_tiered_ = v[0] == '1';   // tests
  world_ = comm_ ? comm_->world() : 1;
  // forced DP (tests / bench --force-dp): a world-1 communicator carries every
  // DP collective (packet all-gather, packed int64 all-reduce, stats)
  const char* fdp = std::getenv("TWTML_FORCE_DP");
  dp_ = world_ > 1 || (comm_ && (cfg_.force_dp != 0 || (fdp && fdp[0] == '1')));
  comm_timing_ = dp_ && cfg_.comm_timing != 0;
  if (const char* e = std::getenv("TWTML_RCCL_STANDIN"); e && dp_) standin_wgs_ = std::max(0, std::atoi(e));
  // Prepare-ahead of batch t+1 while t trains: all of it on one GPU; on DP
  // ranks the local part, then (after the training thread all-gathered the
  // ranks' packets between two of t's GD iterations) the rest.
  overlap_ = cfg_.overlap != 0;
  if (const char* v = std::getenv("TWTML_OVERLAP")) overlap_ = overlap_ && v[0] != '0';
  TWTML_HIP_CHECK(hipSetDevice(device_));
  hipDeviceProp_t prop;
  TWTML_HIP_CHECK(hipGetDeviceProperties(&prop, device_));
  num_cu_ = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  // the GD loop outranks the prepare-ahead of the next batch for free CUs
  int lo = 0, hi = 0;
  TWTML_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  TWTML_HIP_CHECK(hipStreamCreateWithPriority(&compute_, hipStreamNonBlocking, hi));
  // TWTML_PREP_CU=k:n[:s] (tuning, off by default): the prep stream may only
  // use CUs i with (i / s) % n < k (measured: no gain, profiles/README.md)
  if (const char* v = std::getenv("TWTML_PREP_CU")) {
    int k = 0, n = 0, st = 1;
    if (std::sscanf(v, "%d:%d:%d", &k, &n, &st) >= 2 && n > 0 && k > 0 && k < n && st > 0) {
      std::vector<uint32_t> mask(size_t((num_cu_ + 31) / 32), 0u);
      for (int i = 0; i < num_cu_; ++i)
        if ((i / st) % n < k) mask[size_t(i / 32)] |= 1u << (i % 32);
      TWTML_HIP_CHECK(hipExtStreamCreateWithCUMask(&pstream_, uint32_t(mask.size()), mask.data()));
    }
  }
  if (!pstream_) TWTML_HIP_CHECK(hipStreamCreateWithPriority(&pstream_, hipStreamNonBlocking, lo));
  TWTML_HIP_CHECK(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking));
  raw_.init(cfg_.raw_slots, cfg_.max_rows, text_bytes_for_units(cfg_.max_units));
  for (auto& e : ev_) TWTML_HIP_CHECK(hipEventCreate(&e));
  upload_lower_tables(compute_, &lower_page_, &lower_blocks_);
  near_cap_ = tier_near_cap();
  if (const char* v = std::getenv("TWTML_NEAR_CAP"))   // tests / tuning: a smaller LDS tier
    near_cap_ = std::max<int64_t>(64, std::min<int64_t>(near_cap_, std::atoll(v)));
  for (int k = 0; k < (overlap_ ? 2 : 1); ++k) alloc_prepared(pb_[k]);
  const int64_t nw = num_weights();
  sgd_.F = cfg_.num_text_features;
  sgd_.w64 = dmalloc<double>(size_t(nw));
  TWTML_HIP_CHECK(hipMemset(sgd_.w64, 0, sizeof(double) * size_t(nw)));  // Vectors.zeros
  sgd_.touched = dmalloc<uint8_t>(size_t(nw));
  TWTML_HIP_CHECK(hipMemset(sgd_.touched, 0, size_t(nw)));
  sgd_.stats = dmalloc<double>(8);
  sgd_.stat_i = dmalloc<int64_t>(16);
  sgd_.stat_part = dmalloc<int64_t>(size_t(kStatBlocks) * 16);
  sgd_.state = dmalloc<double>(kStateLen);
  sgd_.loss_hist = dmalloc<double>(size_t(std::max(1, cfg_.num_iterations)) + 2);
  sgd_.itrec = dmalloc<double>((size_t(std::max(1, cfg_.num_iterations)) + 2) * kRecStride);
  sgd_.pred_out = dmalloc<float>(size_t(cfg_.max_rows));
  sgd_.real_out = dmalloc<float>(size_t(cfg_.max_rows));
  sgd_.nrm = dmalloc<double>(2 * kNormParts);
  sgd_.wnorm_next = dmalloc<double>(1);
  sgd_.world = world_;
  sgd_.rank = comm_ ? comm_->rank() : 0;
  sgd_.tail_len = sgd_tail_len(world_);
  // Compact weights / packed gradients sized for the largest active set the
  // configuration allows (ids the hash can produce, at most one per unit of
  // a full batch; capped at 16M slots = 448 MB): growing them later means a
  // stream sync + hipFree (a device-wide wait) on the training thread in the
  // middle of the stream.  Larger active sets still grow on demand.
  ensure_compact((kNumNumeric + active_set_hint() + kPadSlots + 63) / 64 * 64);
  // the batch's results: written by k_batch_out into mapped host memory
  TWTML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&host_stat_), 16 * sizeof(int64_t),
                                hipHostMallocMapped | hipHostMallocCoherent));
  TWTML_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&host_stat_dev_), host_stat_, 0));
  TWTML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&host_out_),
                                (32 + size_t(std::max(1, cfg_.num_iterations))) * sizeof(double),
                                hipHostMallocMapped | hipHostMallocCoherent));
  TWTML_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&host_out_dev_), host_out_, 0));
  // the plot sample: written by k_plot_sample straight into mapped host
  // memory (no copy engine: an 80 KB D2H on the compute stream was measured
  // waiting 25 ms behind other transfers once per process)
  TWTML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&plot_host_), 2 * sizeof(float) * size_t(cfg_.max_rows),
                                hipHostMallocMapped | hipHostMallocCoherent));
  TWTML_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&plot_dev_), plot_host_, 0));
  TWTML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&host_flags_),
                                (2 + size_t(std::max(1, cfg_.num_iterations))) * sizeof(double),
                                hipHostMallocMapped | hipHostMallocCoherent));
  TWTML_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&sgd_.host_flags), host_flags_, 0));
  if (dp_) {
    TWTML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&ready_host_), 64, hipHostMallocMapped | hipHostMallocCoherent));
    *ready_host_ = 0;
    int64_t* dev_ready = nullptr;
    TWTML_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev_ready), ready_host_, 0));
    sgd_.ready_word = dev_ready;
    dnu_ = dmalloc<int64_t>(size_t(world_));
    TWTML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&hnu_), sizeof(int64_t) * size_t(world_),
                                  hipHostMallocDefault));
  }
  TWTML_HIP_CHECK(hipDeviceSynchronize());
  if (overlap_) worker_ = std::thread([this] { prep_worker(); });
}

void LREngine::alloc_prepared(PrepBuf& b) {
  DevPrepared& p = b.dp;
  const int64_t R = cfg_.max_rows;
  const int64_t C = (R + kRowsPerChunk - 1) / kRowsPerChunk;
  const int64_t R16 = C * kRowsPerChunk;
  int64_t E = 2 * cfg_.max_units + 2 * C * kChunkStride + 65536;
  E = (E + kChunkStride - 1) / kChunkStride * kChunkStride;
  p.cap_rows = R;
  p.cap_rows16 = R16;
  p.cap_chunks = C;
  p.cap_entries = E;
  p.kept = dmalloc<int64_t>(size_t(R));
  p.nnz = dmalloc<int32_t>(size_t(R));
  p.sorted = dmalloc<int32_t>(size_t(R));
  p.blk = dmalloc<int64_t>(size_t(R / kBlock + 2));
  p.hist = dmalloc<int64_t>(kLenBuckets + 1);
  p.clen8 = dmalloc<int32_t>(size_t(C) + 1);
  p.cfast = dmalloc<uint8_t>(size_t(C) + 1);
  p.clen8d = dmalloc<int32_t>(size_t(C) + 1);
  p.cnt = dmalloc<uint16_t>(size_t(E));
  p.cslot = dmalloc<uint16_t>(size_t(E));
  p.hot_dense = dmalloc<uint32_t>(size_t(C) * kWave * 4);
  p.clen8c = dmalloc<int32_t>(size_t(C) + 1);
  p.hot_slot = dmalloc<int32_t>(kHot);
  p.hot_of = dmalloc<uint8_t>(kMaxHybridSlots);
  p.slot_hist = dmalloc<uint32_t>(kMaxHybridSlots);
  b.slot_hist_cap = kMaxHybridSlots;
  p.code = dmalloc<uint16_t>(8192);
  p.cbase = dmalloc<int64_t>(size_t(C) + 1);
  p.idx = dmalloc<int32_t>(size_t(E));
  p.slot = dmalloc<uint32_t>(size_t(E));
  p.y = dmalloc<float>(size_t(R16));
  p.num = dmalloc<float>(4 * size_t(R16));
  p.perm = dmalloc<int32_t>(size_t(R16));
  p.rtext = dmalloc<int64_t>(size_t(R16));
  p.scan_tmp = dmalloc<int64_t>(size_t(C) / 2048 + 2);   // multi-block scan tiles of 2048
  // active-feature flags: Java-hash bigrams are < 2^21 whatever F is
  const int64_t F = cfg_.num_text_features;
  int64_t fl = cfg_.hash_kind == 0 ? std::min<int64_t>(F, int64_t(1) << 21) : F;
  fl = (fl + 4095) / 4096 * 4096;
  p.flag_len = fl;
  p.flags = dmalloc<uint8_t>(size_t(fl));
  TWTML_HIP_CHECK(hipMemset(p.flags, 0, size_t(fl)));
  p.uniq = dmalloc<int32_t>(size_t(fl));
  p.slot_of = dmalloc<int32_t>(size_t(fl));
  p.ublk = dmalloc<int64_t>(size_t(fl / 4096) + 2);
  p.counters = dmalloc<int64_t>(8);
  b.n_global = dmalloc<int64_t>(2 * size_t(world_) + 2);
  b.bounds = dmalloc<double>(kBoundsLen);
  TWTML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&b.host_counters),
                                (8 + 2 * size_t(world_)) * sizeof(int64_t), hipHostMallocDefault));
  TWTML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&b.host_norm), 2 * sizeof(int64_t), hipHostMallocDefault));
  TWTML_HIP_CHECK(hipEventCreate(&b.ev_start));
  TWTML_HIP_CHECK(hipEventCreate(&b.ev_done));
  if (dp_) {
    TWTML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&b.host_hdr),
                                  sizeof(int64_t) * size_t(world_) * (kC1HeaderWords / 2), hipHostMallocDefault));
    TWTML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&b.host_bounds), sizeof(double) * kBoundsLen,
                                  hipHostMallocDefault));
    TWTML_HIP_CHECK(hipEventCreateWithFlags(&b.ev_c1, hipEventDisableTiming));
  }
}

void LREngine::free_prepared(PrepBuf& b) {
  DevPrepared& p = b.dp;
  void* bufs[] = {p.kept, p.nnz, p.sorted, p.blk, p.hist, p.clen8, p.cfast, p.clen8d, p.cnt, p.cslot,
                  p.hot_dense, p.clen8c, p.hot_slot, p.hot_of, p.slot_hist, p.code, p.cbase, p.idx, p.slot,
                  p.y, p.num, p.perm, p.rtext, p.scan_tmp, p.flags, p.uniq, p.slot_of, p.ublk, p.counters,
                  p.fslot, p.fcount, p.fhist, p.fcur, p.fcsc, p.newslot, p.slot_fid, p.tscan,
                  p.tscan_blk, p.hist_near, p.tparam, b.n_global, b.ugather, b.bounds, b.packet, b.gathered};
  for (void* x : bufs) if (x) (void)hipFree(x);
  if (b.host_counters) (void)hipHostFree(b.host_counters);
  if (b.host_norm) (void)hipHostFree(b.host_norm);
  if (b.host_hdr) (void)hipHostFree(b.host_hdr);
  if (b.host_bounds) (void)hipHostFree(b.host_bounds);
  if (b.ev_c1) (void)hipEventDestroy(b.ev_c1);
  if (b.ev_start) (void)hipEventDestroy(b.ev_start);
  if (b.ev_done) (void)hipEventDestroy(b.ev_done);
  b = PrepBuf{};
}

// Host side of the early stop: spin (with back-off) on the zero-copy verdict
// of update j, which iteration j+1's gradient kernel publishes in its
// prologue.  Bounded: the stream is synchronised as a fallback so a kernel
// fault surfaces as a HIP error instead of a hang.
double LREngine::wait_flag(int j) {
  volatile double* f = host_flags_ + j;
  for (int spin = 0; spin < (1 << 22); ++spin) {
    const double v = *f;
    if (v >= 0.0) {
      if (std::getenv("TWTML_DEBUG_EARLY")) std::fprintf(stderr, "early-stop check j=%d flag=%g\n", j, v);
      return v;
    }
    if (spin > 4096) std::this_thread::yield();
  }
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
  const double v = *f;
  if (v < 0.0) throw std::runtime_error("GD early-stop verdict never published");
  return v;
}

// Tiered-layout buffers of a prepared batch: arrays of the nU compact slots
// (grown on demand) and, at its first tiered batch, the entry-sized far
// lists / CSC.  The residual buffer of the far backward is the trainer's.
void LREngine::ensure_tier(PrepBuf& b, int64_t n_unique, hipStream_t s) {
  DevPrepared& p = b.dp;
  if (!p.fslot) {
    const size_t E = size_t(p.cap_entries);
    p.fslot = dmalloc<uint32_t>(E);
    p.fcsc = dmalloc<uint2>(E);
    p.fcount = dmalloc<int32_t>(size_t(p.cap_chunks) + 1);
    p.hist_near = dmalloc<uint32_t>(kMaxHybridSlots);
    p.tparam = dmalloc<int64_t>(4);
  }
  if (n_unique <= p.cap_tier) return;
  // first sized for the configuration's largest active set (see the
  // constructor): a regrowth syncs and frees on the prep thread, and hipFree
  // waits for the whole device -- the batch training meanwhile stalls
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  void* old[] = {p.newslot, p.slot_fid, p.tscan, p.tscan_blk, p.fhist, p.fcur};
  for (void* x : old) if (x) (void)hipFree(x);
  const int64_t cap = std::max({n_unique, p.cap_tier * 2, p.cap_tier == 0 ? active_set_hint() : int64_t(0)});
  p.cap_tier = cap;
  p.newslot = dmalloc<int32_t>(size_t(cap));
  p.slot_fid = dmalloc<int32_t>(size_t(cap) + kNumNumeric + 2 * kPadSlots);
  p.tscan = dmalloc<int64_t>(size_t(cap) + 1 + 2048);   // + 4096 u32 count buckets
  p.tscan_blk = dmalloc<int64_t>(size_t(cap) / 2048 + 4);   // multi-block scan tiles of 2048
  p.fhist = dmalloc<uint64_t>(size_t(cap) + 1);
  p.fcur = dmalloc<uint64_t>(size_t(cap) + 1);
  if (cap + kNumNumeric + 64 > b.slot_hist_cap) {
    (void)hipFree(p.slot_hist);
    b.slot_hist_cap = cap + kNumNumeric + 64;
    p.slot_hist = dmalloc<uint32_t>(size_t(b.slot_hist_cap));
    // stream-ordered: the null stream does not order against the engine's
    // non-blocking streams, so a plain hipMemset could land after the
    // histogram pass that follows on `s`
    TWTML_HIP_CHECK(hipMemsetAsync(p.slot_hist, 0, sizeof(uint32_t) * size_t(b.slot_hist_cap), s));
  }
}

// Upper bound of a batch's active set (text slots) under the configuration:
// the ids the hash can produce (Java-hash bigrams < 2^21), at most one per
// text unit of a full batch, capped at 16M.
int64_t LREngine::active_set_hint() const {
  const int64_t F = cfg_.num_text_features;
  const int64_t ids = cfg_.hash_kind == 0 ? std::min<int64_t>(F, int64_t(1) << 21) : F;
  return std::max<int64_t>(1, std::min({ids, cfg_.max_units + 64, int64_t(1) << 24}));
}

void LREngine::ensure_part(int64_t n) {
  if (n <= part_cap_) return;
  if (sgd_.part) {
    TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
    (void)hipFree(sgd_.part);
  }
  part_cap_ = std::max<int64_t>(n, part_cap_ * 2);
  sgd_.part = dmalloc<int64_t>(size_t(part_cap_));
}

void LREngine::ensure_compact(int64_t ns) {
  if (ns <= ns_cap_) return;
  int64_t cap = std::max<int64_t>(ns, ns_cap_ * 2);
  if (sgd_.wc64) {
    TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
    (void)hipFree(sgd_.wc64);
    (void)hipFree(sgd_.wc32);
    (void)hipFree(sgd_.gacc);
  }
  sgd_.wc64 = dmalloc<double>(size_t(cap));
  sgd_.wc32 = dmalloc<float>(size_t(cap));
  // packed int64 buffer: near columns (<= cap) | tail | far slots (<= cap)
  const size_t gl = 2 * size_t(cap) + size_t(sgd_tail_len(world_)) + 64;
  sgd_.gacc = dmalloc<int64_t>(gl);
  // zeroed on the compute stream, ahead of the kernels that accumulate into
  // it (a null-stream hipMemset is unordered against the non-blocking
  // compute stream and could wipe an iteration's far gradients)
  TWTML_HIP_CHECK(hipMemsetAsync(sgd_.gacc, 0, sizeof(int64_t) * gl, compute_));
  ns_cap_ = cap;
}

LREngine::~LREngine() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (worker_.joinable()) worker_.join();
  (void)hipSetDevice(device_);
  // a fault of this engine's last work surfaces here: report it (and keep it
  // for teardown_errors()) instead of leaving it to the next engine's first call
  report_teardown_error("LREngine", device_, hipDeviceSynchronize());
  raw_.release();
  for (auto& e : ev_) (void)hipEventDestroy(e);
  for (auto& b : pb_) free_prepared(b);
  if (snap_stream_) {
    (void)hipStreamSynchronize(snap_stream_);
    (void)hipStreamDestroy(snap_stream_);
  }
  if (snap_ev_) (void)hipEventDestroy(snap_ev_);
  if (snap_src_ev_) (void)hipEventDestroy(snap_src_ev_);
  for (void* b : {static_cast<void*>(snap_cnt_), static_cast<void*>(snap_off_), static_cast<void*>(snap_idx_),
                  static_cast<void*>(snap_val_), static_cast<void*>(snap_tidx_), static_cast<void*>(snap_tval_)})
    if (b) (void)hipFree(b);
  if (snap_total_) (void)hipHostFree(snap_total_);
  if (snap_stage_) (void)hipHostFree(snap_stage_);
  void* bufs[] = {sgd_.gacc, sgd_.rbuf, sgd_.pbuf, sgd_.stat_i, sgd_.stat_part, sgd_.w64, sgd_.touched, sgd_.wc64,
                  sgd_.wc32,
                  sgd_.stats, sgd_.state,
                  sgd_.loss_hist, sgd_.pred_out, sgd_.real_out, sgd_.nrm, sgd_.wnorm_next, sgd_.part, sgd_.itrec, iter_tdbg_, iter_kdbg_,
                  lower_page_, lower_blocks_};
  for (void* b : bufs) if (b) (void)hipFree(b);
  if (host_out_) (void)hipHostFree(host_out_);
  if (host_stat_) (void)hipHostFree(host_stat_);
  if (plot_host_) (void)hipHostFree(plot_host_);
  if (host_flags_) (void)hipHostFree(host_flags_);
  if (ready_host_) (void)hipHostFree(ready_host_);
  if (hnu_) (void)hipHostFree(hnu_);
  if (dnu_) (void)hipFree(dnu_);
  if (standin_buf_) (void)hipFree(standin_buf_);
  for (auto e : iter_events_) (void)hipEventDestroy(e);
  for (auto e : comm_ev_) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(compute_);
  (void)hipStreamDestroy(pstream_);
  (void)hipStreamDestroy(copy_);
}

void LREngine::submit(const HostBatch& hb, int64_t n, int64_t bytes, int slot, const uint8_t* ext_text,
                      int64_t now_ms) {
  TraceRange tr("twtml.lr.submit_h2d");
  TWTML_HIP_CHECK(hipSetDevice(device_));
  std::lock_guard<std::mutex> lk(mu_);
  raw_.submit(hb, n, bytes, slot, copy_, kScalarCols, ext_text);
  submitted_.push_back({slot, now_ms});
  cv_.notify_all();
}

// ---------------------------------------------------------------------------
// prepare: filter .. layout of one raw slot into a PrepBuf, on stream `s`
// (the prep stream; host syncs for the batch's counts stay on this thread).
// One GPU: prepare_local + prepare_global.  DP: prepare_local (ends with the
// rank's packet), the all-gather by the training thread (issue_c1), then
// prepare_global_dp.
// ---------------------------------------------------------------------------

// Local part (no collectives): decode / lower rows, filter, sort, chunk
// layout, featurize, this rank's active set; ends with its counts on the
// host.  DP: + the sampled counts of the local active ids and the packet.
void LREngine::prepare_local(PrepBuf& pb, int slot, int64_t now_ms, hipStream_t s) {
  TraceRange tr_prep("twtml.lr.prep");   // filter .. remap
  TWTML_HIP_CHECK(hipSetDevice(device_));
  const int world = world_;
  DevPrepared& prep = pb.dp;
  BatchResult& res = pb.res;
  res = BatchResult{};
  const DevRawBatch b = raw_.acquire(slot, s);
  res.n_raw = b.n;
  TWTML_HIP_CHECK(hipEventRecord(pb.ev_start, s));
  // fault injection (tests): TWTML_INJECT_PREP_FAIL=<rank>:<n> fails this
  // rank's n-th local prep (1-based)
  if (const char* f = std::getenv("TWTML_INJECT_PREP_FAIL")) {
    int fr = -1, fn = 1;
    if (std::sscanf(f, "%d:%d", &fr, &fn) >= 1 && comm_ && fr == comm_->rank() && ++prep_calls_ == fn)
      throw std::runtime_error("injected prep failure");
  }

  FeaturizeParams fp{cfg_.num_text_features, cfg_.hash_kind, cfg_.require_retweet,
                     cfg_.range_filter, cfg_.begin, cfg_.end, now_ms};
  launch_prep_init(prep, pb.n_global, 2 * world + 2, s, pb.bounds, kBoundsLen);
  launch_filter_sort(b, prep, fp, s);
  launch_chunk_layout(b, prep, s);
  // lazy ids: only the histogram's sample chunks keep their hashed ids; the
  // hybrid remap re-reads the (still resident) raw text for the rest
  static const int lazy_env = [] {   // TWTML_LAZY_IDX=0/1 forces (A/B)
    const char* e = std::getenv("TWTML_LAZY_IDX");
    return e ? std::atoi(e) : -1;
  }();
  const bool lazy = (lazy_env >= 0 ? lazy_env != 0 : cfg_.lazy_idx != 0) && cfg_.hybrid && !cfg_.dedup;
  fp.idx_mode = lazy ? 1 : 0;
  launch_featurize(b, prep, fp, lower_page_, lower_blocks_, s);
  launch_batch_bounds(prep, pb.bounds, s, true);   // fixed-point scale bounds of this rank's rows
  if (!lazy) raw_.release_slot(slot, s);  // raw slot may be overwritten now
  launch_compact_active(prep, s);        // this rank's active ids (clears the flags)
  TWTML_HIP_CHECK(hipMemcpyAsync(pb.host_counters, prep.counters, 4 * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  TWTML_HIP_CHECK(hipMemcpyAsync(pb.host_norm, raw_.norm_stats(slot), 2 * sizeof(int64_t),
                                 hipMemcpyDeviceToHost, s));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  if (pb.host_counters[3] != 0) throw std::runtime_error("feature buffer capacity exceeded");
  if (dp_) {
    // the packet: sampled counts of the local active ids (the same sampled
    // chunks as the tiered near-tier choice), then header + (id, count) pairs
    const int64_t nU = pb.host_counters[1];
    ensure_tier(pb, nU, s);
    if (nU > 0) {
      TWTML_HIP_CHECK(hipMemsetAsync(prep.slot_hist + kNumNumeric, 0, sizeof(uint32_t) * size_t(nU), s));
      launch_tier_hist(prep, nU, num_cu_, s);
    }
    if (nU > pb.pkt_cap || !pb.packet) {
      if (pb.packet) (void)hipFree(pb.packet);
      pb.pkt_cap = std::max<int64_t>(std::max<int64_t>(2 * nU, 4096), pb.pkt_cap);
      pb.packet = dmalloc<int32_t>(size_t(c1_packet_words(pb.pkt_cap)));
    }
    launch_pack_c1(prep, pb.bounds, pb.packet, nU, s);
    // back to zero for the hybrid remap's own histogram (k_prep_init zeroed the rest)
    TWTML_HIP_CHECK(hipMemsetAsync(prep.slot_hist, 0,
                                   sizeof(uint32_t) * size_t(std::min<int64_t>(kNumNumeric + nU, pb.slot_hist_cap)), s));
    TWTML_HIP_CHECK(hipStreamSynchronize(s));
    pb.nu_local = nU;
  }
  pb.raw = b;
  pb.fp = fp;
  pb.lazy = lazy;
  pb.slot = slot;
  pb.stage = 1;
}

// One GPU: counts from the device, then the layout.
void LREngine::prepare_global(PrepBuf& pb, hipStream_t s) {
  TraceRange tr_prep("twtml.lr.prep_global");
  TWTML_HIP_CHECK(hipSetDevice(device_));
  const int64_t* hc = pb.host_counters;
  BatchResult& res = pb.res;
  res.n_kept = hc[0];
  res.n_kept_global = hc[0];
  res.rows_lowered = pb.host_norm[0];
  res.rows_narrowed = pb.host_norm[1];
  res.n_unique = hc[1];
  res.entries = hc[2] * kChunkStride;
  pb.row_offset = 0;
  finish_layout(pb, s, false);
}

// DP: the all-gather of the ranks' packets, on the compute stream, between
// two GD iterations of the previous batch (or in line, issue_c1_inline).
// Every rank issues it at the same point of its collective sequence.
void LREngine::issue_c1(PrepBuf& pb, int64_t max_u) {
  TraceRange tr("twtml.lr.prep_allgather");
  hipStream_t s = compute_;
  const int64_t pw = c1_packet_words(max_u);
  if (max_u > pb.pkt_cap) {   // another rank's active set is larger than this packet holds (rare)
    int32_t* np = dmalloc<int32_t>(size_t(pw));
    TWTML_HIP_CHECK(hipMemcpyAsync(np, pb.packet, sizeof(int32_t) * size_t(c1_packet_words(pb.nu_local)),
                                   hipMemcpyDeviceToDevice, s));
    TWTML_HIP_CHECK(hipStreamSynchronize(s));
    (void)hipFree(pb.packet);
    pb.packet = np;
    pb.pkt_cap = max_u;
  }
  if (max_u > pb.gath_cap || !pb.gathered) {
    if (pb.gathered) {
      TWTML_HIP_CHECK(hipStreamSynchronize(s));
      (void)hipFree(pb.gathered);
    }
    pb.gath_cap = std::max<int64_t>(max_u + max_u / 4 + 1024, pb.gath_cap);
    pb.gathered = dmalloc<int32_t>(size_t(world_) * size_t(c1_packet_words(pb.gath_cap)));
  }
  if (max_u > pb.nu_local)   // pad this rank's pairs to the largest rank's: id -1
    TWTML_HIP_CHECK(hipMemsetAsync(pb.packet + c1_packet_words(pb.nu_local), 0xFF,
                                   sizeof(int32_t) * 2 * size_t(max_u - pb.nu_local), s));
  comm_->allgather(pb.packet, pb.gathered, size_t(pw), ncclInt32, s);
  TWTML_HIP_CHECK(hipEventRecord(pb.ev_c1, s));
  std::lock_guard<std::mutex> lk(mu_);
  pb.c1_maxu = max_u;
  pb.c1 = 2;
  __atomic_store_n(ready_host_, int64_t(0), __ATOMIC_RELEASE);
  cv_.notify_all();
}

// DP, the packets were not gathered during the previous batch (first batch,
// or the ranks' local parts finished after its GD loop): size the all-gather
// with an all-reduce of one active-set size per rank, then gather.
bool LREngine::issue_c1_inline(PrepBuf* pb) {
  hipStream_t s = compute_;
  const int rank = comm_->rank();
  // a rank whose local prep failed contributes -1: every rank then skips the
  // all-gather and raises, instead of the others blocking in it
  for (int r = 0; r < world_; ++r) hnu_[r] = r == rank ? (pb ? pb->nu_local : int64_t(-1)) : 0;
  TWTML_HIP_CHECK(hipMemcpyAsync(dnu_, hnu_, sizeof(int64_t) * size_t(world_), hipMemcpyHostToDevice, s));
  comm_->allreduce(dnu_, size_t(world_), ncclInt64, ncclSum, s);
  TWTML_HIP_CHECK(hipMemcpyAsync(hnu_, dnu_, sizeof(int64_t) * size_t(world_), hipMemcpyDeviceToHost, s));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  int64_t mx = 0;
  bool ok = true;
  for (int r = 0; r < world_; ++r) {
    mx = std::max(mx, hnu_[r]);
    ok = ok && hnu_[r] >= 0;
  }
  if (ok && pb) issue_c1(*pb, mx);
  return ok;
}

// DP global part, no collectives: per-rank kept rows (global m, sampling
// offsets) and bounds from the gathered headers, the active-id union
// (flags + compaction: every rank numbers the same slots), the union's
// summed sampled counts (tiered near tier), then the layout.
void LREngine::prepare_global_dp(PrepBuf& pb, hipStream_t s) {
  TraceRange tr_prep("twtml.lr.prep_global");
  TWTML_HIP_CHECK(hipSetDevice(device_));
  // A failure here (after the packet all-gather) raises on this rank only:
  // its peers go on into the batch's first gradient all-reduce and wait
  // there, and the batch watchdog (--batchTimeout; bench.py --timeout) or
  // the launcher tearing the group down after this rank's exit ends them.
  // TWTML_INJECT_GLOBAL_PREP_FAIL=<rank>:<n> (tests) fails this rank's n-th
  // global prep.
  if (const char* f = std::getenv("TWTML_INJECT_GLOBAL_PREP_FAIL")) {
    int fr = -1, fn = 1;
    if (std::sscanf(f, "%d:%d", &fr, &fn) >= 1 && fr == comm_->rank() && ++gprep_calls_ == fn)
      throw std::runtime_error("injected global prep failure");
  }
  const int world = world_, rank = comm_->rank();
  DevPrepared& prep = pb.dp;
  BatchResult& res = pb.res;
  const int64_t max_u = pb.c1_maxu;
  const int64_t pw = c1_packet_words(max_u);
  constexpr int kH = kC1HeaderWords / 2;   // int64 header words per rank
  TWTML_HIP_CHECK(hipStreamWaitEvent(s, pb.ev_c1, 0));
  for (int r = 0; r < world; ++r)
    TWTML_HIP_CHECK(hipMemcpyAsync(pb.host_hdr + r * kH, pb.gathered + int64_t(r) * pw, sizeof(int64_t) * kH,
                                   hipMemcpyDeviceToHost, s));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  int64_t row_offset = 0, n_glob = 0;
  for (int k = 0; k < kBoundsLen; ++k) pb.host_bounds[k] = 0.0;
  for (int r = 0; r < world; ++r) {
    const int64_t* h = pb.host_hdr + r * kH;
    if (r < rank) row_offset += h[0];
    n_glob += h[0];
    for (int k = 0; k < kBoundsLen; ++k)
      pb.host_bounds[k] = std::max(pb.host_bounds[k], __builtin_bit_cast(double, h[2 + k]));
  }
  TWTML_HIP_CHECK(hipMemcpyAsync(pb.bounds, pb.host_bounds, sizeof(double) * kBoundsLen, hipMemcpyHostToDevice, s));
  launch_union_flag(pb.gathered, world, max_u, prep, s);
  launch_compact_active(prep, s);
  int64_t* hc = pb.host_counters;
  TWTML_HIP_CHECK(hipMemcpyAsync(hc + 1, prep.counters + 1, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  res.n_kept = hc[0];
  res.n_kept_global = n_glob;
  res.rows_lowered = pb.host_norm[0];
  res.rows_narrowed = pb.host_norm[1];
  res.n_unique = hc[1];
  res.entries = hc[2] * kChunkStride;
  pb.row_offset = row_offset;
  finish_layout(pb, s, true);
}

// Compact space of the (global) active set and the hybrid / tiered layout.
// dp_hist: slot counts for the tiered near tier from the gathered packets
// (every rank numbers the slots from the same counts), else sampled here.
void LREngine::finish_layout(PrepBuf& pb, hipStream_t s, bool dp_hist) {
  DevPrepared& prep = pb.dp;
  BatchResult& res = pb.res;
  const DevRawBatch& b = pb.raw;
  const FeaturizeParams& fp = pb.fp;
  const bool lazy = pb.lazy;
  const int64_t nU = res.n_unique;
  int64_t ns = kNumNumeric + nU + kPadSlots;
  ns = (ns + 63) / 64 * 64;
  // Active sets beyond LDS take the tiered layout (hot_split.hip / k_far_grad):
  // decided from the global active set, so every DP rank takes the same path.
  const bool tiered = !(ns <= 65536 && sgd_hybrid_fits(ns)) || force_tiered_;
  const bool u16 = ns <= 65536 || tiered;   // tiered: the near streams are u16
  const bool dedup = cfg_.dedup && !tiered && dedup_supported(ns);
  prep.tiered = tiered ? 1 : 0;
  prep.hybrid = (tiered || (!dedup && cfg_.hybrid && res.n_kept > 0)) ? 1 : 0;
  pb.ns = ns;
  pb.nl = ns;
  pb.n_near = nU;
  pb.far_base = kNumNumeric + nU;
  pb.u16 = u16;
  if (tiered) {
    const int64_t n_near = std::min(nU, near_cap_);
    const int64_t nl = (kNumNumeric + n_near + kPadSlots + 63) / 64 * 64;
    ensure_tier(pb, nU, s);
    prep.near_end = kNumNumeric + n_near;
    TWTML_HIP_CHECK(hipMemsetAsync(prep.slot_hist + kNumNumeric, 0, sizeof(uint32_t) * size_t(nU), s));
    if (dp_hist) launch_union_hist(pb.gathered, world_, pb.c1_maxu, prep, s);
    else launch_tier_hist(prep, nU, num_cu_, s);
    launch_tier_layout(prep, res.entries, nU, n_near, ns, nl, num_cu_, b, fp, lazy, s);
    pb.nl = nl;
    pb.n_near = n_near;
    pb.far_base = kNumNumeric + n_near;
    res.tiered = true;
  } else {
    if (lazy && !prep.hybrid) launch_featurize_fast_ids(b, prep, fp, s);   // every id after all
    if (prep.hybrid) launch_remap_hybrid(prep, res.entries, ns, kNumNumeric + nU, num_cu_, b, fp, lazy, s);
    else launch_remap(prep, res.entries, nU, u16, s);
  }
  if (lazy) raw_.release_slot(pb.slot, s);
  prep.dedup = dedup ? 1 : 0;
  if (prep.dedup) launch_dedup(prep, ns, kNumNumeric + nU, res.n_kept, s);
  res.n_near = pb.n_near;
  TWTML_HIP_CHECK(hipEventRecord(pb.ev_done, s));
  pb.stage = 2;
}

// ---------------------------------------------------------------------------
// train: GD on a prepared batch, on the compute stream (after its prep).
// ---------------------------------------------------------------------------
BatchResult LREngine::train(PrepBuf& pb, bool want_pred, int64_t plot_points) {
  TWTML_HIP_CHECK(hipSetDevice(device_));
  hipStream_t s = compute_;
  const int world = world_;
  DevPrepared& prep = pb.dp;
  BatchResult res = pb.res;
  using Clk = std::chrono::steady_clock;
  Clk::time_point th[5];
  th[0] = Clk::now();
  TWTML_HIP_CHECK(hipStreamWaitEvent(s, pb.ev_done, 0));
  TWTML_HIP_CHECK(hipEventRecord(ev_[0], s));
  const int64_t nU = res.n_unique;
  const int64_t n_glob = res.n_kept_global;
  const bool tiered = res.tiered;
  const bool u16 = pb.u16;
  ensure_compact(pb.ns);
  sgd_.ns = pb.ns;
  sgd_.n_unique = nU;
  sgd_.nl = pb.nl;
  sgd_.n_near = pb.n_near;
  sgd_.far_base = pb.far_base;
  sgd_.slot_fid = tiered ? prep.slot_fid : nullptr;
  sgd_.bounds = pb.bounds;
  sgd_.far_off = pb.nl + sgd_.tail_len;
  if (tiered) {
    if (!sgd_.rbuf) sgd_.rbuf = dmalloc<float>(size_t(prep.cap_rows16));
    sgd_.fcsc = prep.fcsc;
    sgd_.far_n = prep.tparam + 2;
  }
  if (!sgd_.pbuf) sgd_.pbuf = dmalloc<float>(size_t(prep.cap_rows16));
  launch_batch_init(sgd_, double(n_glob), cfg_.num_iterations + 2, s);  // state[5] = m (global kept rows)
  if (norm_age_ < 0 || norm_age_ >= kNormRefresh) {
    launch_norm2(sgd_.w64, num_weights(), &sgd_.state[4], sgd_, s);
    norm_age_ = 0;
  } else {
    launch_norm_carry(sgd_, s);
  }
  ++norm_age_;
  launch_gather_w(sgd_, prep, s);
  TWTML_HIP_CHECK(hipEventRecord(ev_[1], s));
  th[1] = Clk::now();
  TraceRange tr_train("twtml.lr.train");   // GD iterations (host enqueue + early-stop polling)

  const int64_t nl = sgd_.nl;
  int grid = cfg_.sgd_grid > 0 ? cfg_.sgd_grid : sgd_iter_grid(nl, res.n_kept, num_cu_, prep.hybrid != 0);
  sgd_.pstride = sgd_part_stride(nl);
  sgd_.nparts = sgd_partials(nl, u16, grid);
  ensure_part(int64_t(sgd_.nparts) * sgd_.pstride);
  SgdParams sp{};
  sp.step_size = cfg_.step_size;
  sp.fraction = cfg_.fraction;
  sp.tol = cfg_.tol;
  sp.num_iterations = cfg_.num_iterations;
  sp.row_offset = pb.row_offset;
  sp.want_pred = want_pred ? 1 : 0;
  sp.sample = cfg_.fraction < 1.0 ? 1 : 0;
  sp.ablate = cfg_.ablate;
  sp.dp = dp_ ? 1 : 0;
  sp.rank0 = (comm_ ? comm_->rank() : 0) == 0 ? 1 : 0;
  const int64_t n_far = kNumNumeric + nU - sgd_.far_base;
  res.diverged = diverged_;
  int comm_iters = 0;   // DP: gradient all-reduces issued for this batch
  if (n_glob > 0 && !diverged_) {
    // Host-side early stop: the convergence test of update j runs in the
    // prologue of iteration j+1's gradient kernel, which copies its verdict
    // to pinned memory (zero copy); the host keeps at most `depth`
    // iterations queued and stops enqueueing once an earlier verdict is
    // set.  Verdicts derive from all-reduced values in a fixed summation
    // order, so every rank stops at the same iteration and the collectives
    // match.
    const int depth = std::max(2, cfg_.early_exit_depth);
    const int iters = cfg_.num_iterations;
    std::fill(host_flags_, host_flags_ + iters + 2, -1.0);   // -1: verdict not published yet
    // single GPU with partial rows: the update kernel reduces them itself
    const bool fused = !dp_ && sgd_.nparts > 0;
    const bool itime = std::getenv("TWTML_ITER_TIMING") != nullptr;
    if (itime && !iter_tdbg_) iter_tdbg_ = dmalloc<uint64_t>(4096 + size_t(iters + 2) * 32);
    const size_t kd_words = size_t(iters + 2) * kKdbgKinds * kKdbgWgs * 2;
    if (itime && !iter_kdbg_) iter_kdbg_ = dmalloc<uint64_t>(kd_words);
    sgd_.tdbg = itime ? iter_tdbg_ : nullptr;
    sgd_.kdbg = itime ? iter_kdbg_ : nullptr;
    if (itime) TWTML_HIP_CHECK(hipMemsetAsync(iter_tdbg_, 0, sizeof(uint64_t) * (4096 + size_t(iters + 2) * 32), s));
    if (itime) TWTML_HIP_CHECK(hipMemsetAsync(iter_kdbg_, 0, sizeof(uint64_t) * kd_words, s));
    if (comm_timing_ && comm_ev_.size() < size_t(2 * iters)) {
      for (size_t q = comm_ev_.size(); q < size_t(2 * iters); ++q) {
        hipEvent_t e;
        TWTML_HIP_CHECK(hipEventCreate(&e));
        comm_ev_.push_back(e);
      }
    }
    for (int i = 1; i <= iters; ++i) {
      if (i > depth) {
        const int j = i - depth;                       // verdict after update j
        const int64_t v = int64_t(wait_flag(j));       // bit 0 stop; DP: bit 1 every rank's next
                                                       // packet ready, >> 2 the largest one
        if (dp_ && (v & 2)) {
          // the next batch's packets are ready on every rank: all-gather them
          // here, between iterations j + depth - 1 and j + depth -- every rank
          // sees the same all-reduced flag at the same point
          PrepBuf* nb = nullptr;
          {
            std::lock_guard<std::mutex> lk(mu_);
            for (auto& b : pb_)
              if (&b != &pb && b.c1 == 1) nb = &b;
          }
          if (nb) issue_c1(*nb, v >> 2);
        }
        if (v & 1) break;
      }
      sp.iteration = i;
      // every rank launches the gradient kernel (an empty shard writes zero
      // partials) so every rank runs the convergence prologue
      launch_sgd_iter(sgd_, prep, sp, pb.host_counters[2], u16, grid, s);
      if (i == 1) launch_batch_stats(sgd_, prep, s);   // exact moments of the prequential pass
      if (tiered) launch_far_grad(sgd_, sp, num_cu_, s);
      if (dp_) {
        // ONE collective per iteration: the packed int64 buffer (near
        // columns, loss, sampled m, verdict, ready words, far slots); integer
        // sums are exact in any order, so every rank gets the same bits
        launch_sgd_reduce(sgd_, sp, s);
        if (comm_timing_) TWTML_HIP_CHECK(hipEventRecord(comm_ev_[size_t(2 * (i - 1))], s));
        comm_->allreduce(sgd_.gacc, size_t(sgd_.far_off + n_far), ncclInt64, ncclSum, s);
        res.comm_bytes += int64_t(sizeof(int64_t)) * (sgd_.far_off + n_far);
        if (standin_wgs_ > 0) {   // DP cost model: the CU footprint of a multi-rank all-reduce
          const int64_t nw = sgd_.far_off + n_far;
          if (nw > standin_cap_) {
            if (standin_buf_) {
              TWTML_HIP_CHECK(hipStreamSynchronize(s));
              (void)hipFree(standin_buf_);
            }
            standin_cap_ = nw + nw / 4;
            standin_buf_ = dmalloc<int64_t>(size_t(standin_cap_));
          }
          launch_rccl_standin(sgd_.gacc, standin_buf_, nw, standin_wgs_, sgd_.kdbg, i, s);
        }
        if (comm_timing_) TWTML_HIP_CHECK(hipEventRecord(comm_ev_[size_t(2 * (i - 1) + 1)], s));
        ++comm_iters;
      }
      launch_sgd_update(sgd_, sp, fused ? sgd_.nparts : 0, s);
    }
    launch_sgd_finish(sgd_, sp, s);
    if (snap_guard_) {   // a checkpoint snapshot still reading the master weights
      TWTML_HIP_CHECK(hipStreamWaitEvent(s, snap_ev_, 0));
      snap_guard_ = false;
    }
    launch_scatter_w(sgd_, prep, s);
    launch_norm_next(sgd_, true, s);
    if (itime) print_iter_timing(iters);
  }
  if (n_glob <= 0 || diverged_) launch_norm_next(sgd_, false, s);   // weights unchanged: carry |w|^2 as is
  TWTML_HIP_CHECK(hipEventRecord(ev_[2], s));
  th[2] = Clk::now();
  if (dp_) {
    // the exact int64 moments (any summation order gives the same bits), then
    // the fp64 sums of spill rows (zero unless a prediction left +-2^31)
    comm_->allreduce(sgd_.stat_i, size_t(kStatI), ncclInt64, ncclSum, s);
    comm_->allreduce(sgd_.stats, 6, ncclFloat64, ncclSum, s);
  }
  launch_batch_out(sgd_, host_out_dev_, host_stat_dev_, cfg_.num_iterations + 1, s);
  TWTML_HIP_CHECK(hipEventRecord(ev_[4], s));
  // the plot's (pred, real) pairs of this rank's kept rows: all of them, or
  // plot_points evenly spaced ones sampled on the device, written by the
  // kernel into mapped host memory
  size_t P = 0;
  if (want_pred && res.n_kept > 0) {
    P = size_t(plot_points > 0 ? std::min<int64_t>(plot_points, res.n_kept) : res.n_kept);
    launch_plot_sample(sgd_.pred_out, sgd_.real_out, res.n_kept, int64_t(P), plot_dev_, s);
  }
  TWTML_HIP_CHECK(hipEventRecord(ev_[3], s));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  th[3] = Clk::now();
  if (comm_) comm_->check_async();
  if (P > 0) {
    res.pred.resize(P);
    res.real.resize(P);
    for (size_t i = 0; i < P; ++i) {
      res.pred[i] = plot_host_[2 * i];
      res.real[i] = plot_host_[2 * i + 1];
    }
  }
  {
    // exact moments (int64; squares from two 32-bit limbs, as 128-bit) plus
    // the fp64 spill sums (0.0 unless a prediction left +-2^31: then exact)
    const int64_t* si = host_stat_;
    auto limbs = [](int64_t hi, int64_t lo) { return double((__int128)hi * 4294967296LL + lo); };
    const double ex[6] = {double(si[0]), double(si[1]), limbs(si[3], si[4]), double(si[2]), limbs(si[5], si[6]),
                          limbs(si[7], si[8])};
    for (int k = 0; k < 6; ++k) res.stats[k] = ex[k] + host_out_[k];
    res.stats_spill = si[9];
  }
  const double* st = host_out_ + 8;
  res.converged = st[1] != 0.0;
  res.diverged = diverged_ || st[7] == 1.0;
  diverged_ = res.diverged;
  res.iterations = int32_t(st[3]);
  for (int i = 1; i <= res.iterations; ++i) res.loss_history.push_back(host_out_[16 + i]);
  // prep_ms: the batch's prep on its own stream (overlapped with the previous
  // batch's training when prepared ahead); train_ms: compute stream
  TWTML_HIP_CHECK(hipEventElapsedTime(&res.prep_ms, pb.ev_start, pb.ev_done));
  TWTML_HIP_CHECK(hipEventElapsedTime(&res.train_ms, ev_[1], ev_[2]));
  th[4] = Clk::now();
  for (int q = 0; q < 4; ++q) res.phases[q] = std::chrono::duration<float, std::milli>(th[q + 1] - th[q]).count();
  TWTML_HIP_CHECK(hipEventElapsedTime(&res.phases[4], ev_[0], ev_[1]));
  TWTML_HIP_CHECK(hipEventElapsedTime(&res.phases[5], ev_[2], ev_[3]));
  TWTML_HIP_CHECK(hipEventElapsedTime(&res.phases[6], ev_[2], ev_[4]));
  res.comm_iters = comm_iters;
  if (comm_timing_) {   // the per-iteration gradient all-reduces on the compute stream
    for (int q = 0; q < comm_iters; ++q) {
      float ms = 0.f;
      TWTML_HIP_CHECK(hipEventElapsedTime(&ms, comm_ev_[size_t(2 * q)], comm_ev_[size_t(2 * q + 1)]));
      res.comm_ms += ms;
    }
  }
  return res;
}

void LREngine::print_iter_timing(int iters) {
  // iteration-kernel phases (us): stop-check, lds init, chunks, hot reduce, scalars, slots
  hipStream_t s = compute_;
  std::vector<uint64_t> tb(4096 + size_t(iters + 2) * 32);
  TWTML_HIP_CHECK(hipMemcpyAsync(tb.data(), iter_tdbg_, tb.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  for (int which = 0; which < 2; ++which) {
    double acc[6] = {0, 0, 0, 0, 0, 0};
    int n = 0;
    for (int i = 2; i <= iters; ++i) {
      const uint64_t* t = tb.data() + (size_t(i) * 2 + size_t(which)) * 8;
      if (t[6] == 0) continue;
      for (int k = 0; k < 6; ++k) acc[k] += double(t[k + 1] - t[k]) * 0.01;
      ++n;
    }
    if (n) std::fprintf(stderr, "iter timing wg %s (us, %d iters): stop %.2f init %.2f chunks %.2f hotred %.2f scalars %.2f slots %.2f\n",
                        which ? "last" : "0", n, acc[0] / n, acc[1] / n, acc[2] / n, acc[3] / n, acc[4] / n, acc[5] / n);
  }
  const int i = std::min(10, iters);   // wave end spread inside WG 0, iteration 10
  const uint64_t* t0 = tb.data() + (size_t(i) * 2) * 8;
  const uint64_t* we = tb.data() + 4096 + size_t(i) * 32;
  std::fprintf(stderr, "wave ends (us after kernel start) / chunks, WG 0 it %d:", i);
  for (int w = 0; w < 16; ++w) std::fprintf(stderr, " %.1f/%d", double(we[2 * w] - t0[0]) * 0.01, int(we[2 * w + 1]));
  std::fprintf(stderr, "\n");
  // per-kernel workgroup stamps: dispatch ramp (last start - first start),
  // span (last end - first start), median / max workgroup time, and the gap
  // from the previous kernel's last end to this one's first start
  const size_t kd_words = size_t(iters + 2) * kKdbgKinds * kKdbgWgs * 2;
  std::vector<uint64_t> kd(kd_words);
  TWTML_HIP_CHECK(hipMemcpyAsync(kd.data(), iter_kdbg_, kd_words * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  const char* names[kKdbgKinds] = {"iteration", "far backward", "update", "rccl stand-in"};
  double acc[kKdbgKinds][5] = {};
  int cnt[kKdbgKinds] = {0, 0, 0, 0};
  // launch order within an iteration: iteration, far backward, [stand-in], update
  const int order[kKdbgKinds] = {0, 1, 3, 2};
  for (int it = 2; it <= iters; ++it) {
    uint64_t prev_end = 0;
    for (int ko = 0; ko < kKdbgKinds; ++ko) {
      const int k = order[ko];
      const uint64_t* b = kd.data() + (size_t(it) * kKdbgKinds + size_t(k)) * kKdbgWgs * 2;
      uint64_t s0 = UINT64_MAX, s1 = 0, e1 = 0;
      std::vector<double> dur;
      for (int g = 0; g < kKdbgWgs; ++g) {
        if (b[2 * g] == 0 || b[2 * g + 1] == 0) continue;
        s0 = std::min(s0, b[2 * g]);
        s1 = std::max(s1, b[2 * g]);
        e1 = std::max(e1, b[2 * g + 1]);
        dur.push_back(double(b[2 * g + 1] - b[2 * g]) * 0.01);
      }
      if (dur.empty()) continue;
      std::sort(dur.begin(), dur.end());
      acc[k][0] += double(s1 - s0) * 0.01;
      acc[k][1] += double(e1 - s0) * 0.01;
      acc[k][2] += dur[dur.size() / 2];
      acc[k][3] += dur.back();
      acc[k][4] += prev_end ? double(int64_t(s0) - int64_t(prev_end)) * 0.01 : 0.0;
      prev_end = e1;
      ++cnt[k];
    }
  }
  for (int k = 0; k < kKdbgKinds; ++k)
    if (cnt[k])
      std::fprintf(stderr, "kernel %-13s (us, %d iters): ramp %.2f span %.2f wg p50 %.2f wg max %.2f gap before %.2f\n",
                   names[k], cnt[k], acc[k][0] / cnt[k], acc[k][1] / cnt[k], acc[k][2] / cnt[k], acc[k][3] / cnt[k],
                   acc[k][4] / cnt[k]);
}

// ---------------------------------------------------------------------------
// Prepare-ahead: the prep thread prepares the oldest submitted slot that is
// not prepared yet into a free PrepBuf while the caller trains.
// ---------------------------------------------------------------------------
void LREngine::prep_worker() {
  (void)hipSetDevice(device_);
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    cv_.wait(lk, [&] { return stop_ || job_ >= 0; });
    if (stop_) return;
    PrepBuf& b = pb_[job_];
    const int slot = b.slot;
    const int64_t now_ms = b.now_ms;
    lk.unlock();
    std::exception_ptr err;
    try {
      prepare_local(b, slot, now_ms, pstream_);
      if (dp_) {
        // packet ready: announce it (the ready word travels in the gradient
        // all-reduce) and wait for the training thread's all-gather
        lk.lock();
        b.c1 = 1;
        __atomic_store_n(ready_host_, b.nu_local + 1, __ATOMIC_RELEASE);
        cv_.notify_all();
        cv_.wait(lk, [&] { return stop_ || b.c1 == 2 || b.c1 == -2; });
        if (stop_) return;
        if (b.c1 == -2) throw std::runtime_error("DP: a peer rank failed to prepare this batch");
        lk.unlock();
        prepare_global_dp(b, pstream_);
      } else {
        prepare_global(b, pstream_);
      }
    } catch (...) {
      err = std::current_exception();
    }
    if (!lk.owns_lock()) lk.lock();
    b.error = err;
    if (err && b.c1 == 1) b.c1 = -1;
    b.state = 2;
    job_ = -1;
    cv_.notify_all();
  }
}

// Caller holds mu_: start preparing the next submitted slot if a buffer and
// the prep thread are free.
void LREngine::schedule_ahead_locked() {
  if (!overlap_ || job_ >= 0 || submitted_.empty()) return;
  int free_buf = -1;
  for (int k = 0; k < 2; ++k)
    if (pb_[k].state == 0) free_buf = k;
  if (free_buf < 0) return;
  const auto next = submitted_.front();
  for (auto& b : pb_)
    if (b.state != 0 && b.slot == next.first) return;   // already there
  submitted_.pop_front();
  PrepBuf& b = pb_[free_buf];
  b.state = 1;
  b.slot = next.first;
  b.now_ms = next.second;
  job_ = free_buf;
  cv_.notify_all();
}

// A submitted batch that will never be processed (the host pipeline matched
// no take() to its prefetch): drop it from the prepare-ahead queue, release a
// prepared buffer that holds it (after its preparation finished), and order
// every read of the slot's raw bytes before the next H2D into the slot.
// Without this an orphan is prepared ahead, evicted and prepared again on
// every later batch, and a reused slot races its own stale preparation.
void LREngine::discard(int slot) {
  TWTML_HIP_CHECK(hipSetDevice(device_));
  std::unique_lock<std::mutex> lk(mu_);
  if (dp_)   // every rank must issue the same collectives: no rank may skip a batch
    throw std::logic_error("DP: every submitted batch must be processed, in submission order");
  for (auto it = submitted_.begin(); it != submitted_.end();)
    it = it->first == slot ? submitted_.erase(it) : std::next(it);
  for (auto& b : pb_) {
    if (b.state == 0 || b.slot != slot) continue;
    cv_.wait(lk, [&] { return b.state == 2; });
    b.state = 0;
    b.c1 = 0;
    b.error = nullptr;
  }
  raw_.release_slot(slot, pstream_);
  schedule_ahead_locked();
  lk.unlock();           // (the copy stream does not depend on the prep thread)
  raw_.wait_h2d(slot);   // the host staging buffer of the slot may be rewritten on return
}

BatchResult LREngine::process(int slot, int64_t now_ms, bool want_pred, int64_t plot_points) {
  TraceRange tr_batch("twtml.lr.batch");
  TWTML_HIP_CHECK(hipSetDevice(device_));
  const auto t_in = std::chrono::steady_clock::now();
  int k = -1;
  bool ahead = false;
  {
    std::unique_lock<std::mutex> lk(mu_);
    for (int i = 0; i < 2; ++i)
      if (pb_[i].state != 0 && pb_[i].slot == slot) k = i;
    ahead = k >= 0;
    if (k >= 0 && dp_) {
      // DP: the packets were all-gathered during the previous batch, or are
      // now, in line -- the same choice on every rank (it follows the
      // all-reduced ready words); then the prep thread finishes the layout
      cv_.wait(lk, [&] { return pb_[k].c1 != 0 || pb_[k].state == 2; });
      if (pb_[k].c1 == 1) {
        lk.unlock();
        const bool ok = issue_c1_inline(&pb_[k]);
        lk.lock();
        if (!ok) {   // a peer's prep failed: release the prep thread, raise on every rank
          pb_[k].c1 = -2;
          cv_.notify_all();
        }
      } else if (pb_[k].c1 == 0 && pb_[k].state == 2 && pb_[k].error) {
        // this rank's local prep failed before its packet: tell the peers
        lk.unlock();
        (void)issue_c1_inline(nullptr);
        lk.lock();
      }
      cv_.wait(lk, [&] { return pb_[k].state == 2; });
      if (pb_[k].error) {
        std::exception_ptr err = pb_[k].error;
        pb_[k].error = nullptr;
        pb_[k].state = 0;
        pb_[k].c1 = 0;
        std::rethrow_exception(err);
      }
    } else if (k >= 0) {
      cv_.wait(lk, [&] { return pb_[k].state == 2; });
      // prepared ahead with the batch time given at submit; a different time
      // here is re-prepared
      if (pb_[k].error || pb_[k].now_ms != now_ms) {   // failed ahead / other time
        std::exception_ptr err = pb_[k].error;
        pb_[k].error = nullptr;
        if (err && pb_[k].now_ms == now_ms) {
          pb_[k].state = 0;
          std::rethrow_exception(err);
        }
        pb_[k].state = 1;
        lk.unlock();
        prepare_local(pb_[k], slot, now_ms, pstream_);
        prepare_global(pb_[k], pstream_);
        lk.lock();
        pb_[k].state = 2;
      }
    } else {
      // not prepared ahead: drop it from the submission queue, prepare in line
      for (auto it = submitted_.begin(); it != submitted_.end(); ++it)
        if (it->first == slot) { submitted_.erase(it); break; }
      if (dp_) {
        // every rank must issue the same collectives in the same order: a
        // batch prepared (and possibly all-gathered) ahead may not be skipped
        for (int i = 0; i < 2; ++i)
          if (pb_[i].state != 0)
            throw std::logic_error("DP: batches must be processed in submission order");
      }
      for (int i = 0; i < (overlap_ ? 2 : 1); ++i)
        if (pb_[i].state == 0) k = i;
      if (k < 0) {
        // one GPU: every buffer holds a batch prepared ahead that is not this
        // one (submitted but processed out of order): evict one -- its slot
        // goes back to the front of the queue and is prepared again when due
        cv_.wait(lk, [&] { return job_ < 0; });
        for (int i = 0; i < 2 && k < 0; ++i)
          if (pb_[i].state == 2) {
            submitted_.push_front({pb_[i].slot, pb_[i].now_ms});
            pb_[i].state = 0;
            pb_[i].error = nullptr;
            k = i;
          }
        if (k < 0) throw std::logic_error("no free prepared-batch buffer");
      }
      pb_[k].state = 1;
      pb_[k].slot = slot;
      pb_[k].now_ms = now_ms;
      lk.unlock();
      try {
        bool local_ok = false;
        try {
          prepare_local(pb_[k], slot, now_ms, pstream_);
          local_ok = true;
        } catch (...) {
          if (dp_) (void)issue_c1_inline(nullptr);   // the peers raise too instead of waiting
          throw;
        }
        if (dp_) {
          if (local_ok && !issue_c1_inline(&pb_[k]))
            throw std::runtime_error("DP: a peer rank failed to prepare this batch");
          prepare_global_dp(pb_[k], pstream_);
        } else {
          prepare_global(pb_[k], pstream_);
        }
      } catch (...) {
        lk.lock();
        pb_[k].state = 0;
        pb_[k].c1 = 0;
        throw;
      }
      lk.lock();
      pb_[k].state = 2;
    }
    last_buf_ = k;
    schedule_ahead_locked();   // batch t+1's prep overlaps batch t's training
  }
  BatchResult res;
  const auto t_train = std::chrono::steady_clock::now();
  try {
    res = train(pb_[k], want_pred, plot_points);
    res.prepared_ahead = ahead;
    res.wait_ms = std::chrono::duration<float, std::milli>(t_train - t_in).count();
    res.train_wall_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t_train).count();
  } catch (...) {
    std::lock_guard<std::mutex> lk(mu_);
    pb_[k].state = 0;
    pb_[k].c1 = 0;
    throw;
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    pb_[k].state = 0;
    pb_[k].c1 = 0;
    schedule_ahead_locked();
  }
  return res;
}

void LREngine::set_weights(const double* w, int64_t n) {
  if (n != num_weights()) throw std::invalid_argument("weights size mismatch");
  TWTML_HIP_CHECK(hipSetDevice(device_));
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
  if (snap_guard_) {
    TWTML_HIP_CHECK(hipEventSynchronize(snap_ev_));
    snap_guard_ = false;
  }
  // stream-ordered, complete on return (a pageable hipMemcpy may return
  // before its DMA lands, unordered against the non-blocking compute stream)
  TWTML_HIP_CHECK(hipMemcpyAsync(sgd_.w64, w, sizeof(double) * size_t(n), hipMemcpyHostToDevice, compute_));
  launch_mark_nonzero(sgd_.w64, sgd_.touched, n, compute_);
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
  norm_age_ = -1;   // the carried |w|^2 no longer holds
  diverged_ = false;
}

void LREngine::get_weights(double* w, int64_t n) const {
  if (n != num_weights()) throw std::invalid_argument("weights size mismatch");
  TWTML_HIP_CHECK(hipSetDevice(device_));
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
  TWTML_HIP_CHECK(hipMemcpy(w, sgd_.w64, sizeof(double) * size_t(n), hipMemcpyDeviceToHost));
}

void LREngine::snapshot_begin() {
  TWTML_HIP_CHECK(hipSetDevice(device_));
  std::lock_guard<std::mutex> lk(snap_mu_);
  if (snap_pending_) throw std::runtime_error("snapshot_begin: the previous snapshot was not copied yet");
  const int64_t n = num_weights();
  if (n >= (int64_t(1) << 31)) throw std::runtime_error("snapshot: more than 2^31 weights");
  if (!snap_idx_) {   // once: F+4 pairs worst case (1.2 GB at F = 1e8, of 288 GB)
    const int64_t nb = snapshot_chunks(n);
    snap_cnt_ = static_cast<uint32_t*>(dev_alloc(sizeof(uint32_t) * size_t(nb)));
    snap_off_ = static_cast<int64_t*>(dev_alloc(sizeof(int64_t) * size_t(nb + 1)));
    snap_idx_ = static_cast<int32_t*>(dev_alloc(sizeof(int32_t) * size_t(n)));
    snap_val_ = static_cast<double*>(dev_alloc(sizeof(double) * size_t(n)));
    snap_tidx_ = static_cast<int32_t*>(dev_alloc(sizeof(int32_t) * size_t(n)));
    snap_tval_ = static_cast<double*>(dev_alloc(sizeof(double) * size_t(n)));
    TWTML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&snap_total_), sizeof(int64_t), hipHostMallocMapped));
    TWTML_HIP_CHECK(hipHostMalloc(&snap_stage_, size_t(kSnapStage), hipHostMallocDefault));
    int lo = 0, hi = 0;
    TWTML_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    TWTML_HIP_CHECK(hipStreamCreateWithPriority(&snap_stream_, hipStreamNonBlocking, lo));
    TWTML_HIP_CHECK(hipEventCreateWithFlags(&snap_ev_, hipEventDisableTiming));
    TWTML_HIP_CHECK(hipEventCreateWithFlags(&snap_src_ev_, hipEventDisableTiming));
  }
  *snap_total_ = -1;
  int64_t* dtot = nullptr;
  TWTML_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dtot), snap_total_, 0));
  // The master weights change only in k_scatter_w at the end of a batch, so
  // the compaction runs on its own low-priority stream behind the last
  // batch and overlaps the next batch's prep and GD loop; that batch's
  // scatter waits for it (train: snap_guard_).
  TWTML_HIP_CHECK(hipEventRecord(snap_src_ev_, compute_));
  TWTML_HIP_CHECK(hipStreamWaitEvent(snap_stream_, snap_src_ev_, 0));
  launch_snapshot(sgd_.w64, sgd_.touched, n, snap_cnt_, snap_off_, snap_tidx_, snap_tval_, snap_idx_, snap_val_,
                  dtot, snap_stream_);
  TWTML_HIP_CHECK(hipGetLastError());
  TWTML_HIP_CHECK(hipEventRecord(snap_ev_, snap_stream_));
  snap_guard_ = true;
  snap_pending_ = true;
}

void LREngine::snapshot_host(int64_t nnz, int32_t** idx, double** val) {
  if (int64_t(snap_hidx_.size()) < nnz) {   // value-initialised: every page is touched now
    const size_t cap = size_t(std::max<int64_t>(nnz + nnz / 4, int64_t(1) << 16));
    snap_hidx_.assign(cap, 0);
    snap_hval_.assign(cap, 0.0);
  }
  *idx = snap_hidx_.data();
  *val = snap_hval_.data();
}

int64_t LREngine::snapshot_wait() {
  TWTML_HIP_CHECK(hipSetDevice(device_));
  {
    std::lock_guard<std::mutex> lk(snap_mu_);
    if (!snap_pending_) throw std::runtime_error("snapshot_wait: no snapshot was begun");
  }
  TWTML_HIP_CHECK(hipEventSynchronize(snap_ev_));
  const int64_t nnz = __atomic_load_n(snap_total_, __ATOMIC_ACQUIRE);
  if (nnz < 0 || nnz > num_weights()) throw std::runtime_error("snapshot: bad non-zero count");
  return nnz;
}

void LREngine::snapshot_copy(int32_t* idx, double* val) {
  const int64_t nnz = snapshot_wait();
  // Chunks through the page-locked stage (the DMA never waits on pageable
  // memory), paced to a byte rate of duty x 50 GB/s (2.5 GB/s at the default
  // 0.05): a batch's H2D that meets a chunk on the DMA engine waits for at
  // most that chunk.  A checkpoint is not latency critical: 36 MB of pairs
  // (F = 1e8 after 60 wide batches) take ~15 ms, against ~25 ms of parquet
  // write.  Pacing by the pairs' bytes (not by each chunk's measured time)
  // keeps the copy's duration independent of the chunk size, so the chunks
  // can be small (256 KB).  The checkpoint p99 gate (500K-tweet wide
  // batches at F = 1e8, a checkpoint due every batch) moves with how many
  // snapshots a run takes, not with the chunk size or the rate:
  // profiles/r6/ckpt_d2h_chunks.txt.
  static const double duty = [] {
    const char* e = std::getenv("TWTML_SNAP_DUTY");
    const double d = e ? std::atof(e) : 0.05;
    return d > 0.0 && d <= 1.0 ? d : 0.05;
  }();
  static const int64_t chunk = [] {   // TWTML_SNAP_CHUNK_KB (A/B)
    const char* e = std::getenv("TWTML_SNAP_CHUNK_KB");
    const int64_t kb = e ? std::atoll(e) : 256;
    return std::min<int64_t>(kSnapStage, std::max<int64_t>(64, kb) << 10);
  }();
  const double rate = duty * 50e9;   // bytes per second
  const auto start = std::chrono::steady_clock::now();
  int64_t done = 0;
  for (int part = 0; part < 2; ++part) {
    const int64_t esz = part == 0 ? int64_t(sizeof(int32_t)) : int64_t(sizeof(double));
    const int64_t per = chunk / esz;
    const char* src = part == 0 ? reinterpret_cast<const char*>(snap_idx_) : reinterpret_cast<const char*>(snap_val_);
    char* dst = part == 0 ? reinterpret_cast<char*>(idx) : reinterpret_cast<char*>(val);
    for (int64_t o = 0; o < nnz; o += per) {
      const int64_t c = std::min(per, nnz - o);
      TWTML_HIP_CHECK(hipMemcpyAsync(snap_stage_, src + o * esz, size_t(c * esz), hipMemcpyDeviceToHost,
                                     snap_stream_));
      TWTML_HIP_CHECK(hipStreamSynchronize(snap_stream_));
      std::memcpy(dst + o * esz, snap_stage_, size_t(c * esz));
      done += c * esz;
      if (duty < 1.0)
        std::this_thread::sleep_until(start + std::chrono::duration_cast<std::chrono::steady_clock::duration>(
                                                  std::chrono::duration<double>(double(done) / rate)));
    }
  }
  std::lock_guard<std::mutex> lk(snap_mu_);
  snap_pending_ = false;
}

void LREngine::set_step(double step, int iters, double fraction) {
  if (iters > cfg_.num_iterations) throw std::invalid_argument("cannot raise numIterations after init");
  cfg_.step_size = step;
  cfg_.num_iterations = iters;
  cfg_.fraction = fraction;
}

void LREngine::synchronize() {
  TWTML_HIP_CHECK(hipSetDevice(device_));
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
  TWTML_HIP_CHECK(hipStreamSynchronize(pstream_));
  TWTML_HIP_CHECK(hipStreamSynchronize(copy_));
}

void LREngine::debug_merged(std::vector<int32_t>& slot, std::vector<int32_t>& cnt,
                            std::vector<int32_t>& clen8d) const {
  TWTML_HIP_CHECK(hipSetDevice(device_));
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
  TWTML_HIP_CHECK(hipStreamSynchronize(pstream_));
  const DevPrepared& lp = pb_[last_buf_ < 0 ? 0 : last_buf_].dp;
  slot.clear(); cnt.clear(); clen8d.clear();
  if (!lp.dedup) return;
  int64_t counters[4];
  TWTML_HIP_CHECK(hipMemcpy(counters, lp.counters, sizeof(counters), hipMemcpyDeviceToHost));
  const int64_t C = (counters[0] + kRowsPerChunk - 1) / kRowsPerChunk;
  const int64_t E = counters[2] * kChunkStride;
  std::vector<uint16_t> s16(static_cast<size_t>(E)), c16(static_cast<size_t>(E));
  clen8d.resize(size_t(C));
  if (E) {
    TWTML_HIP_CHECK(hipMemcpy(s16.data(), lp.slot, sizeof(uint16_t) * size_t(E), hipMemcpyDeviceToHost));
    TWTML_HIP_CHECK(hipMemcpy(c16.data(), lp.cnt, sizeof(uint16_t) * size_t(E), hipMemcpyDeviceToHost));
  }
  if (C) TWTML_HIP_CHECK(hipMemcpy(clen8d.data(), lp.clen8d, sizeof(int32_t) * size_t(C), hipMemcpyDeviceToHost));
  slot.assign(s16.begin(), s16.end());
  cnt.assign(c16.begin(), c16.end());
}

void LREngine::debug_hybrid(std::vector<int32_t>& hot_slot, std::vector<uint32_t>& hot_dense,
                            std::vector<int32_t>& clen8c, std::vector<int32_t>& cslot) const {
  TWTML_HIP_CHECK(hipSetDevice(device_));
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
  TWTML_HIP_CHECK(hipStreamSynchronize(pstream_));
  const DevPrepared& lp = pb_[last_buf_ < 0 ? 0 : last_buf_].dp;
  hot_slot.clear(); hot_dense.clear(); clen8c.clear(); cslot.clear();
  if (!lp.hybrid) return;
  int64_t counters[4];
  TWTML_HIP_CHECK(hipMemcpy(counters, lp.counters, sizeof(counters), hipMemcpyDeviceToHost));
  const int64_t C = (counters[0] + kRowsPerChunk - 1) / kRowsPerChunk;
  const int64_t E = counters[2] * kChunkStride;
  hot_slot.resize(kHot);
  hot_dense.resize(size_t(C) * kWave * 4);
  clen8c.resize(size_t(C));
  std::vector<uint16_t> c16(static_cast<size_t>(E));
  TWTML_HIP_CHECK(hipMemcpy(hot_slot.data(), lp.hot_slot, sizeof(int32_t) * kHot, hipMemcpyDeviceToHost));
  if (C) {
    TWTML_HIP_CHECK(hipMemcpy(hot_dense.data(), lp.hot_dense, sizeof(uint32_t) * hot_dense.size(),
                              hipMemcpyDeviceToHost));
    TWTML_HIP_CHECK(hipMemcpy(clen8c.data(), lp.clen8c, sizeof(int32_t) * size_t(C), hipMemcpyDeviceToHost));
  }
  if (E) TWTML_HIP_CHECK(hipMemcpy(c16.data(), lp.cslot, sizeof(uint16_t) * size_t(E), hipMemcpyDeviceToHost));
  cslot.assign(c16.begin(), c16.end());
}

void LREngine::debug_prepared(std::vector<int64_t>& counters, std::vector<int32_t>& clen8,
                              std::vector<int64_t>& cbase, std::vector<int32_t>& idx,
                              std::vector<int32_t>& perm, std::vector<float>& y,
                              std::vector<float>& num, std::vector<int32_t>& uniq) {
  TWTML_HIP_CHECK(hipSetDevice(device_));
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
  TWTML_HIP_CHECK(hipStreamSynchronize(pstream_));
  const DevPrepared& lp = pb_[last_buf_ < 0 ? 0 : last_buf_].dp;
  counters.resize(4);
  TWTML_HIP_CHECK(hipMemcpy(counters.data(), lp.counters, 4 * sizeof(int64_t), hipMemcpyDeviceToHost));
  const int64_t nk = counters[0], nu = counters[1], groups = counters[2];
  const int64_t C = (nk + kRowsPerChunk - 1) / kRowsPerChunk;
  const int64_t R = C * kRowsPerChunk;
  clen8.resize(size_t(C));
  cbase.resize(size_t(C));
  idx.resize(size_t(groups * kChunkStride));
  perm.resize(size_t(R));
  y.resize(size_t(R));
  num.resize(size_t(4 * R));
  uniq.resize(size_t(nu));
  if (C) {
    TWTML_HIP_CHECK(hipMemcpy(clen8.data(), lp.clen8, sizeof(int32_t) * size_t(C), hipMemcpyDeviceToHost));
    TWTML_HIP_CHECK(hipMemcpy(cbase.data(), lp.cbase, sizeof(int64_t) * size_t(C), hipMemcpyDeviceToHost));
    TWTML_HIP_CHECK(hipMemcpy(perm.data(), lp.perm, sizeof(int32_t) * size_t(R), hipMemcpyDeviceToHost));
    TWTML_HIP_CHECK(hipMemcpy(y.data(), lp.y, sizeof(float) * size_t(R), hipMemcpyDeviceToHost));
    for (int k = 0; k < 4; ++k)
      TWTML_HIP_CHECK(hipMemcpy(num.data() + k * R, lp.num + k * lp.cap_rows16,
                                sizeof(float) * size_t(R), hipMemcpyDeviceToHost));
  }
  if (groups)
    TWTML_HIP_CHECK(hipMemcpy(idx.data(), lp.idx, sizeof(int32_t) * idx.size(), hipMemcpyDeviceToHost));
  if (nu)
    TWTML_HIP_CHECK(hipMemcpy(uniq.data(), lp.uniq, sizeof(int32_t) * size_t(nu), hipMemcpyDeviceToHost));
}

}  // namespace twtml
