// MI355X micro-batch engine for StreamingLinearRegressionWithSGD.
//
// One engine per process/GPU.  A micro-batch flows:
//   pinned host RawBatch --(copy stream, async H2D)--> device slot (x4)
//   prep stream: decode / lower rows -> filter -> length sort -> featurize
//   -> compact -> layout (hybrid / tiered) -- for batch t+1 while batch t
//   trains (prep thread).  DP: the local part ends in one packet per rank
//   (kept rows, active ids + sampled counts, bounds) that the training
//   thread all-gathers between two of batch t's GD iterations (the ONE prep
//   collective); the prep thread finishes t+1 from it on the prep stream.
//   compute stream: gather w -> numIterations x ( fused predict/gradient
//   kernel -> [RCCL all-reduce of the packed gradient] -> fp64 update +
//   convergence ) -> scatter w
// Four device slots let the H2D of the next batches overlap batch t's
// training (SURVEY §2.4 "Ingest || compute pipelining").  Output op #1 (prequential stats)
// is fused into iteration 1, so it sees the weights before training on the
// batch (LinearRegression.scala:53-86 ordering).
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <deque>
#include <exception>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "comm.h"
#include "common.h"
#include "kernels.h"
#include "raw_slots.h"

namespace twtml {

struct LRConfig {
  int64_t num_text_features = 1000;
  int32_t hash_kind = 0;
  double step_size = 0.005;
  int32_t num_iterations = 50;
  double fraction = 1.0;
  double tol = 1e-3;
  int64_t begin = 100, end = 1000;
  int32_t require_retweet = 1, range_filter = 1;
  int64_t max_rows = 1 << 16;
  int64_t max_units = (1 << 16) * 281;
  int32_t sgd_grid = 0;       // 0 = auto
  int32_t early_exit_depth = 3;  // host run-ahead (iterations) for early stop
  int32_t ablate = 0;            // perf diagnostics only (see SgdParams)
  int32_t dedup = 0;             // merge repeated bigrams of a row into counts
  int32_t hybrid = 1;            // dense 4-bit counts for the batch's hottest slots (hot_split.hip)
  int32_t lazy_idx = 1;          // hybrid: fast chunks' ids re-derived from text by the remap
  int32_t overlap = 1;           // prepare batch t+1 (prep stream, prep thread) while t trains
  int32_t force_dp = 0;          // take the DP path (packet all-gather, packed all-reduce, stats
                                 // all-reduce) even with a world-1 communicator (also TWTML_FORCE_DP=1)
  int32_t comm_timing = 0;       // DP: time the per-iteration gradient all-reduce (events)
  int32_t raw_slots = kDefaultRawSlots;   // device raw-batch slots (H2D run-ahead depth + 1)
};

// Pinned staging buffer of one raw batch in the wire format
// (csrc/host/wire.h): narrow/wide rows in `text`, byte offsets, per-row
// flags (bit0 isRetweet, bit1 wide), scalars [5][n] int64 (the record
// values), and their wire encoding (`spack`, see DevRawBatch in kernels.h).
// Bytes of row words (u16 per row) placed right before a batch's text, on
// the host and in a device raw slot, so the two are one H2D copy.
inline size_t rowpack_prefix(int64_t n) { return (sizeof(uint16_t) * size_t(n) + 15) & ~size_t(15); }

struct HostBatch {
  void* base = nullptr;
  size_t bytes = 0;
  uint8_t* text = nullptr;
  int64_t* offsets = nullptr;
  uint8_t* flags = nullptr;
  int64_t* scalars = nullptr;
  uint8_t* spack = nullptr;            // packed columns, column c at soff[c]
  int64_t soff[kScalarCols + 1] = {};  // byte offsets of the columns (8-B aligned)
  int64_t sbase[kScalarCols] = {};
  uint8_t sw[kScalarCols] = {};        // wire bits per value (DevRawBatch::sw)
  int64_t spacked_n = -1;              // rows of the last pack_scalars (-1: none)
  int scalar_cols = kScalarCols;       // leading columns pack_scalars encodes (k-means reads 2)
  int spacked_cols = 0;                // ... and the last call did
  uint16_t* rowpack = nullptr;         // per row: byte length | wire flags << kRowLenBits;
                                       // ends rowpack_prefix(n) bytes before `text`
  int64_t rowpacked_n = -1;            // rows of the last successful pack_rows (-1: none)
  int64_t cesu_rows = 0;               // cesu rows of the last pack_rows (device expands them)
  int64_t wide_rows = 0;               // wide rows of the last pack_rows (device checks them for
                                       // special lower-casing, rows.hip)
  bool utf16 = false;                  // text is plain UTF-16LE (load_utf16): the device narrows
                                       // Latin-1 rows itself
  bool utf8 = false;                   // text is UTF-8 (load_utf8): the device decodes non-ASCII
                                       // rows and narrows the Latin-1 ones
  int64_t rows_scanned_n = -1;         // rows of the last pack_rows call (fit or not)
  int64_t range_hits = 0, range_misses = 0;   // pack_scalars with a range hint: one pass / fell back
  int64_t max_rows = 0, max_bytes = 0;
  HostBatch(int64_t rows, int64_t text_bytes);
  ~HostBatch();
  // Encode scalars[:, :n] (or src [5][n]) into spack (one thread per column).
  // range: optional [lo 0..4 | hi 0..4] column bounds the receiver recorded
  // while sealing the batch: the encoding is chosen from them and the packing
  // pass checks every value against them (one pass over the scalars instead
  // of a min/max pass plus a packing pass); a value outside falls back to
  // the two-pass encoding, so a wrong hint costs time, never correctness.
  void pack_scalars(int64_t n, const int64_t* src = nullptr, const int64_t* range = nullptr);
  // Raw UTF-16 ingest: row words / offsets / flags for `n` rows of UTF-16
  // text with unit offsets uoff [n+1], scalars from sc [5][n]; the text is
  // copied into `text` only if copy_text (else it is DMA'd from the caller's
  // registered buffer by submit).  No per-unit host work besides the copy:
  // the device narrows Latin-1 rows and lowers special rows (rows.hip).
  void load_utf16(const uint16_t* t, const int64_t* uoff, const uint8_t* is_rt, const int64_t* sc,
                  int64_t n, bool copy_text, int threads, const int64_t* range = nullptr);
  // Raw UTF-8 ingest (the bytes the network delivers): same contract with
  // byte offsets boff [n+1].  ~1.1 B per unit of tweet text on PCIe and no
  // per-byte host work: the device decodes (k_cesu_decode) and narrows.
  void load_utf8(const uint8_t* t, const int64_t* boff, const uint8_t* is_rt, const int64_t* sc,
                 int64_t n, bool copy_text, int threads, const int64_t* range = nullptr);
  // Offsets + flags of rows [0, n) as one u16 per row (the device rebuilds
  // both with a scan): 9 -> 2 bytes per row on PCIe.  False (and the batch
  // ships offsets + flags as before) if a row has >= 8192 wire bytes.
  // Also counts the cesu rows (either way).
  bool pack_rows(int64_t n);

 private:
  void load_raw(const uint8_t* t, const int64_t* off, int64_t scale, uint8_t row_flags, const uint8_t* is_rt,
                const int64_t* sc, int64_t n, bool copy_text, int threads, const int64_t* range);
};

// bytes of device text buffer for `units` UTF-16 units: all rows wide (2 B
// per unit) or UTF-8 (<= 3 B per unit: a BMP unit >= U+0800; an astral pair
// is 4 B for 2 units)
inline int64_t text_bytes_for_units(int64_t units) { return 3 * units + 64; }

struct BatchResult {
  int64_t n_raw = 0, n_kept = 0, n_kept_global = 0, n_unique = 0, entries = 0;
  int32_t iterations = 0;
  bool converged = false;
  bool diverged = false;  // the model left any usable range (|r| bound >= 1e30 or non-finite
                          // weights): training stopped at that iteration (sgd.hip sgd_scales)
  int64_t rows_lowered = 0, rows_narrowed = 0;   // device row normalisation (rows.hip)
  bool tiered = false;    // active set beyond LDS: tiered layout (near slots in LDS, far via CSC)
  int64_t n_near = 0;     // text slots in the LDS tier
  double stats[6] = {0, 0, 0, 0, 0, 0};  // n, sum y, sum y^2, sum p, sum p^2, sum (y-p)^2
  int64_t stats_spill = 0;   // kept rows whose |y| or |prediction| >= 2^31 (fp64 moments, not order-exact)
  std::vector<double> loss_history;
  std::vector<float> pred;   // want_pred: rounded predictions of this rank's kept rows (or a sample)
  std::vector<float> real;   // ... and their labels
  float prep_ms = 0.f, train_ms = 0.f;
  int32_t comm_iters = 0;   // DP: gradient all-reduces issued (one per GD iteration)
  float comm_ms = 0.f;      // DP + comm_timing: their summed time on the compute stream
  int64_t comm_bytes = 0;   // DP: bytes of those gradient all-reduces (packed int64 buffer)
  // host side of process(): waiting for / doing this batch's preparation, and
  // train() end to end (enqueue, early-exit polling, the result copies)
  float wait_ms = 0.f, train_wall_ms = 0.f;
  bool prepared_ahead = false;   // the batch was prepared on the prep thread ahead of process()
  // train() on the host: up to the first GD kernel's enqueue, the GD loop
  // (enqueue + verdict polling), the final stream sync, the result copies;
  // on the device: batch init .. weight gather, and the tail after the GD
  // loop (stats / plot sample copies)
  float phases[7] = {0, 0, 0, 0, 0, 0, 0};   // [6]: the tail's result copies alone
};

// One prepared micro-batch: filtered, featurized, compacted and laid out for
// the GD kernels.  Two of them, so batch t+1 is prepared on the prep stream
// (by the engine's prep thread) while batch t trains on the compute stream.
struct PrepBuf {
  DevPrepared dp{};
  int64_t slot_hist_cap = 0;
  int64_t* n_global = nullptr;        // device [2 world + 2]: per-rank kept rows | active-set sizes
  int32_t* ugather = nullptr;         // DP active-set union: all-gathered id lists
  int64_t ugather_cap = 0;
  int64_t* host_counters = nullptr;   // pinned [8 + 2 world]: counters | per-rank kept | per-rank active
  // DP prep packet (dp_prep.hip) and the all-gathered packets of every rank
  int32_t* packet = nullptr;          // device [c1_packet_words(pkt_cap)]
  int64_t pkt_cap = 0;
  int32_t* gathered = nullptr;        // device [world * c1_packet_words(gath_cap)]
  int64_t gath_cap = 0;
  int64_t* host_hdr = nullptr;        // pinned [world * kC1HeaderWords / 2] gathered headers
  double* host_bounds = nullptr;      // pinned [kBoundsLen]
  hipEvent_t ev_c1 = nullptr;         // compute stream, after the all-gather
  int64_t nu_local = 0;               // this rank's active ids (packet pairs)
  int64_t c1_maxu = 0;                // pairs per rank in the all-gather
  int c1 = 0;                         // guarded by mu_: 0 -, 1 packet ready, 2 all-gather issued, -1 failed,
                                      // -2 a peer failed (no all-gather)
  int64_t* host_norm = nullptr;       // pinned [2] rows lowered / narrowed on the device
  double* bounds = nullptr;           // device [kBoundsLen] batch bounds of the fixed-point scales
                                      // (DP: the max over ranks)
  hipEvent_t ev_start = nullptr, ev_done = nullptr;
  // guarded by LREngine::mu_
  int state = 0;                      // 0 free, 1 being prepared, 2 prepared
  int slot = -1;
  int64_t now_ms = 0;
  std::exception_ptr error;
  // prepare() outputs
  int stage = 0;                      // 1: local part done (prepare_local), 2: ready to train
  DevRawBatch raw{};                  // the raw slot's device view (global part, lazy remap)
  FeaturizeParams fp{};
  bool lazy = false;
  BatchResult res;                    // n_raw .. n_near, rows lowered / narrowed
  int64_t row_offset = 0;             // global index of this rank's first kept row
  bool u16 = true;
  int64_t ns = 0, nl = 0, n_near = 0, far_base = 0;
};

class LREngine {
 public:
  // comm: the DP communicator (one per rank; null on one GPU).  Per GD
  // iteration one int64 all-reduce; per batch one all-gather of the prep
  // packets (issued between two GD iterations of the previous batch) and one
  // all-reduce of the 6 batch statistics.  DP batches must be processed in
  // submission order (every rank trains the same sequence).
  LREngine(int device, const LRConfig& cfg, std::shared_ptr<Comm> comm);
  ~LREngine();

  // Async H2D of rows [0, n) of a pinned host batch into device slot `slot`.
  // now_ms: the batch's time (featurizeNumbers), used if it is prepared ahead.
  void submit(const HostBatch& hb, int64_t n, int64_t bytes, int slot, const uint8_t* ext_text = nullptr,
              int64_t now_ms = 0);
  // Train on the batch in `slot` (blocks until done); stats use w before
  // training.  The next submitted slot is then prepared ahead (prep thread,
  // prep stream) while this one trains.
  // plot_points > 0: pred / real hold that many evenly spaced kept rows
  // (sampled on the device), else all of them.
  BatchResult process(int slot, int64_t now_ms, bool want_pred, int64_t plot_points = 0);
  // Forget a submitted batch that will not be processed (one GPU only): the
  // slot may be submitted again afterwards (ops/ingest.py SlotPipeline).
  void discard(int slot);

  void set_weights(const double* w, int64_t n);
  void get_weights(double* w, int64_t n) const;
  int64_t num_weights() const { return cfg_.num_text_features + kNumNumeric; }
  // Device bytes allocated on demand: by the first tiered batch (per prepared
  // buffer: the entry-sized far lists and CSC, the slot-sized tier arrays; the trainer's residual row
  // buffer) and by the first checkpoint snapshot ((index, value) pairs for
  // every weight): ops/sizing.py adds them to the construction footprint.
  int64_t h2d_bytes() const { return raw_.h2d_bytes(); }   // host-to-device bytes submitted so far
  std::vector<std::array<double, 4>> h2d_timeline() { return raw_.h2d_timeline(); }   // TWTML_H2D_TIMING
  void h2d_window_mark() { raw_.h2d_window_mark(copy_); }
  std::vector<double> h2d_window() { return raw_.h2d_window(); }
  int raw_slots() const { return raw_.count(); }
  int64_t lazy_bytes() const {
    const int nbuf = overlap_ ? 2 : 1;
    // + the slot-sized tier arrays (newslot, slot_fid, tscan, fhist, fcur,
    // slot_hist: 36 B per slot of active_set_hint())
    return int64_t(nbuf) * 3 * int64_t(sizeof(uint32_t)) * pb_[0].dp.cap_entries +
           (pb_[0].dp.cap_tier ? 0 : int64_t(nbuf) * 36 * active_set_hint()) +
           int64_t(sizeof(float)) * pb_[0].dp.cap_rows16 +
           (snap_idx_ ? 0 : 2 * num_weights() * int64_t(sizeof(int32_t) + sizeof(double)));
  }
  // Non-blocking checkpoints: snapshot_begin() (training thread, between
  // batches) compacts the non-zero master weights on the device behind the
  // last batch; snapshot_wait() (any thread) returns their count once the
  // compaction is done and snapshot_copy() copies the (index, value) pairs to
  // host memory on the snapshot stream in page-locked chunks, then releases
  // the snapshot.  One snapshot at a time (begin throws if one is pending).
  void snapshot_begin();
  int64_t snapshot_wait();
  void snapshot_copy(int32_t* idx, double* val);
  // Host buffers that outlive a snapshot (grown, never shrunk, faulted in
  // once): the checkpoint writer's copy lands in memory that is already
  // mapped instead of ~36 MB of fresh pages per checkpoint.  Valid until the
  // next call.
  void snapshot_host(int64_t nnz, int32_t** idx, double** val);
  const LRConfig& config() const { return cfg_; }
  bool dp() const { return dp_; }
  void set_step(double step, int iters, double fraction);
  void synchronize();
  int device() const { return device_; }
  // Debug/test access to the last batch's prepared features (host copies).
  void debug_prepared(std::vector<int64_t>& counters, std::vector<int32_t>& clen8,
                      std::vector<int64_t>& cbase, std::vector<int32_t>& idx,
                      std::vector<int32_t>& perm, std::vector<float>& y,
                      std::vector<float>& num, std::vector<int32_t>& uniq);
  // Merged (slot, count) layout the iteration kernels read (empty if not merged).
  void debug_merged(std::vector<int32_t>& slot, std::vector<int32_t>& cnt,
                    std::vector<int32_t>& clen8d) const;
  // Hybrid dense-hot layout of the last batch (empty if not used).
  void debug_hybrid(std::vector<int32_t>& hot_slot, std::vector<uint32_t>& hot_dense,
                    std::vector<int32_t>& clen8c, std::vector<int32_t>& cslot) const;

 private:
  void alloc_prepared(PrepBuf& b);
  void free_prepared(PrepBuf& b);
  void ensure_compact(int64_t ns);
  void ensure_part(int64_t n);
  int64_t active_set_hint() const;
  void ensure_tier(PrepBuf& b, int64_t n_unique, hipStream_t s);
  void prepare_local(PrepBuf& b, int slot, int64_t now_ms, hipStream_t s);
  void prepare_global(PrepBuf& b, hipStream_t s);
  // DP: the all-gather of b's packet, on the compute stream (max_u pairs per rank)
  void issue_c1(PrepBuf& b, int64_t max_u);
  // DP, not issued during the previous batch: size it with an all-reduce
  // first, which also carries every rank's prep status (b == null: this
  // rank's prep failed).  False (no all-gather issued) if any rank failed.
  bool issue_c1_inline(PrepBuf* b);
  // DP: union, global counts / bounds and layout from the gathered packets
  void prepare_global_dp(PrepBuf& b, hipStream_t s);
  // shared tail of prepare_global / prepare_global_dp: compact space + layout
  void finish_layout(PrepBuf& b, hipStream_t s, bool dp_hist);
  BatchResult train(PrepBuf& b, bool want_pred, int64_t plot_points);
  void prep_worker();
  void schedule_ahead_locked();
  void print_iter_timing(int iters);
  double wait_flag(int j);

  int device_;
  LRConfig cfg_;
  std::shared_ptr<Comm> comm_;
  int world_ = 1;
  bool dp_ = false;                 // DP path: world > 1, or forced with a world-1 communicator
  bool comm_timing_ = false;
  std::vector<hipEvent_t> comm_ev_; // comm_timing: [2 iters] around each gradient all-reduce
  hipStream_t compute_ = nullptr, pstream_ = nullptr, copy_ = nullptr;
  RawSlots raw_;
  PrepBuf pb_[2];
  int last_buf_ = -1;               // buffer of the last trained batch (debug_*)
  bool overlap_ = true;
  int64_t* ready_host_ = nullptr;   // DP: pinned mapped ready word (next packet's pairs + 1; 0: none)
  int64_t* dnu_ = nullptr;          // DP: device [world] active-set sizes (in-line all-gather sizing)
  int64_t* hnu_ = nullptr;          // pinned [world]
  // prepare-ahead: submitted slots in order, the prep thread's job (a pb_ index)
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::pair<int, int64_t>> submitted_;
  int job_ = -1;
  bool stop_ = false;
  std::thread worker_;
  DevSgd sgd_{};
  int64_t ns_cap_ = 0;
  // |w|^2 is carried from batch to batch (|w_rest|^2 + trained active part)
  // instead of a pass over all F+4 weights (800 MB at F = 1e8); recomputed
  // after set_weights and every kNormRefresh batches
  static constexpr int kNormRefresh = 256;
  int norm_age_ = -1;   // batches since the last full pass (-1: carried value invalid)
  int64_t part_cap_ = 0;
  // The model diverged (a batch stopped on invalid fixed-point scales):
  // later batches are not trained -- like MLlib's NaN weights, which never
  // recover -- until set_weights() installs a new model.  Identical on every
  // DP rank (decided from all-reduced values), so no collective is skipped
  // on one rank only.
  bool diverged_ = false;
  int64_t near_cap_ = 0;          // tiered layout: LDS-resident text slots (tier_near_cap)
  bool force_tiered_ = false;     // TWTML_FORCE_TIERED=1: tiered layout for any active set (tests)
  int prep_calls_ = 0;            // local preps so far (TWTML_INJECT_PREP_FAIL, tests)
  int gprep_calls_ = 0;           // DP global preps so far (TWTML_INJECT_GLOBAL_PREP_FAIL, tests)
  uint64_t* iter_tdbg_ = nullptr;
  uint8_t* lower_page_ = nullptr;
  uint16_t* lower_blocks_ = nullptr;
  double* host_out_ = nullptr;        // mapped pinned [16 + iters]: stats, state, loss history
  int64_t* host_stat_ = nullptr;      // mapped pinned [16]: exact batch moments (stat_i)
  double* host_out_dev_ = nullptr;    // device view of host_out_ (k_batch_out)
  int64_t* host_stat_dev_ = nullptr;  // device view of host_stat_
  uint64_t* iter_kdbg_ = nullptr;     // TWTML_ITER_TIMING: per-workgroup GD kernel stamps
  int standin_wgs_ = 0;               // DP: TWTML_RCCL_STANDIN workgroups after each gradient all-reduce
  int64_t* standin_buf_ = nullptr;    // ... their destination buffer
  int64_t standin_cap_ = 0;
  float* plot_host_ = nullptr;        // mapped pinned [2 max_rows]: sampled (pred, real) pairs
  float* plot_dev_ = nullptr;         // ... its device address (k_plot_sample writes it)
  double* host_flags_ = nullptr;      // pinned [iters + 1] convergence flag per iteration
  std::vector<hipEvent_t> iter_events_;
  hipEvent_t ev_[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  int num_cu_ = 256;
  // weight snapshot (snapshot.hip); allocated on the first snapshot_begin
  std::mutex snap_mu_;
  bool snap_pending_ = false;
  uint32_t* snap_cnt_ = nullptr;
  int64_t* snap_off_ = nullptr;
  int32_t* snap_idx_ = nullptr;
  double* snap_val_ = nullptr;
  int32_t* snap_tidx_ = nullptr;      // scratch pairs of the one-pass compaction (snapshot.hip)
  double* snap_tval_ = nullptr;
  int64_t* snap_total_ = nullptr;     // pinned mapped
  void* snap_stage_ = nullptr;        // pinned staging, kSnapStage bytes
  std::vector<int32_t> snap_hidx_;    // snapshot_host
  std::vector<double> snap_hval_;
  hipStream_t snap_stream_ = nullptr;
  hipEvent_t snap_ev_ = nullptr;      // snapshot kernels done (snap_stream_)
  hipEvent_t snap_src_ev_ = nullptr;  // the batch the snapshot is taken after (compute_)
  bool snap_guard_ = false;           // the next scatter into w64 must wait for snap_ev_
  static constexpr int64_t kSnapStage = 32ll << 20;
};

}  // namespace twtml
