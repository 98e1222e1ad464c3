// Host-callable launchers of the engine's HIP kernels.
//
// Kernel map:
//   K3  filter + stream compaction          launch_filter
//       length counting-sort (SELL-64 prep)  launch_sort_rows / launch_chunk_layout
//   K1+K2 bigram hash + numeric features     launch_featurize
//       active-set union / slot compaction   launch_compact_active / launch_remap
//   K4+K5 predict + LSQ gradient (fused)     launch_sgd_iter
//   K6  SimpleUpdater + convergence          launch_sgd_update
//   K7  batch stats (fused into K4 at i=1)
//   K8-K11 k-means / scaler                  kmeans.hip
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

namespace twtml {

// ---------------------------------------------------------------------------
// Raw batch on the device (one ingest slot).
// Raw batch in the wire format (csrc/host/wire.h).
//
// Scalar columns (retweetCount, followers, favourites, friends, createdAt) are
// int64 in the record; on the wire column c is a bit stream of offsets from a
// per-batch base in the fewest bits that hold the batch's range (1..32), or
// the raw int64 if the range needs more than 32 bits (HostBatch::pack_scalars).
// Counts are small and createdAt spans far less than 49 days within a batch,
// so a tweet's five scalars take ~12 B instead of 40 (14 B with whole-byte
// widths).  Exact either way.
constexpr int kScalarCols = 5;

struct DevRawBatch {
  const uint8_t* text;      // [bytes] narrow (1 B/unit) or wide (UTF-16LE) rows
  const int64_t* offsets;   // [n] byte offset where row r starts
  const int64_t* oend;      // [n] byte offset where it ends (offsets + 1 unless rows were relocated)
  const uint8_t* flags;     // [n] bit0 isRetweet, bit1 wide (cesu rows are expanded to wide)
  const uint8_t* scol[kScalarCols];   // column c: n values of sw[c] bits (+ sbase[c]), 8-B aligned
  int64_t sbase[kScalarCols];
  uint8_t sw[kScalarCols];  // bits per value: 1..32 (offset from sbase, bit stream) or 64 (raw int64)
  int64_t n;                // rows in this batch (host-known)
  int64_t bytes;
};

// Scalar column c of raw row r (the width test is wave-uniform).
__device__ __forceinline__ int64_t raw_scalar(const DevRawBatch& b, int c, int64_t r) {
  const int bits = b.sw[c];
  if (bits == 64) return reinterpret_cast<const int64_t*>(b.scol[c])[r];
  // bit stream: value r at bit r * bits, read from two aligned words
  const uint32_t* p = reinterpret_cast<const uint32_t*>(b.scol[c]);
  const uint64_t off = uint64_t(r) * uint64_t(bits);
  const uint64_t w = uint64_t(p[off >> 5]) | (uint64_t(p[(off >> 5) + 1]) << 32);
  return b.sbase[c] + int64_t((w >> (off & 31)) & ((uint64_t(1) << bits) - 1u));
}

constexpr uint8_t kRowRetweet = 1;
constexpr uint8_t kRowWide = 2;
constexpr uint8_t kRowCesu = 4;   // wire only (csrc/host/wire.h); expanded by launch_cesu_expand
// device only: a row launch_cesu_expand decoded holds a unit whose lower-casing
// is not one unit per unit (candidate for k_row_normalize's full case mapping)
constexpr uint8_t kRowSpecial = 8;
// Packed row words on the wire (HostBatch::pack_rows): byte length in the
// low kRowLenBits bits, the three flag bits above.
constexpr int kRowLenBits = 13;
// cesu / UTF-8 rows -> rows behind the wire bytes (row with wire bytes
// [o, e) -> from byte tail + 2 * o): UTF-16LE (flag wide), or narrow bytes
// for Latin-1 rows; ASCII rows stay in place.  Writes every row's start /
// end offset; stats[1] (nullable) counts the rows decoded to narrow bytes.
// text needs tail + 2 * bytes + 64.
// special (nullable): the rows flagged kRowSpecial are appended to it, their
// count in stats[2] (the list k_row_special walks, one wave per row).
void launch_cesu_expand(uint8_t* text, const int64_t* offsets, uint8_t* flags, int64_t n, int64_t tail,
                        int64_t* rstart, int64_t* rend, int64_t* stats, hipStream_t s,
                        int32_t* special = nullptr);
// Rebuild offsets [n+1] (exclusive scan of the lengths) and flags [n] from
// packed row words on `s`; tsum: scratch of ceil(n / 8192) int64.
void launch_unpack_rows(const uint16_t* rowpack, int64_t n, int64_t* offsets, uint8_t* flags, int64_t* tsum,
                        hipStream_t s);

// Unicode case tables for the special-row full case mapping (rows.hip).
struct DevCaseTables {
  const uint32_t* supp_lower = nullptr;    // [n_supp][2] astral code point -> lower case
  const uint32_t* case_ranges = nullptr;   // [n_ranges][3] lo, hi, class (1 ignorable, 2 cased)
  const uint32_t* bmp_class = nullptr;     // [4096] the class of every BMP code point, 2 bits each
  int32_t n_supp = 0, n_ranges = 0;
};
void upload_case_tables(DevCaseTables* ct);
void free_case_tables(DevCaseTables* ct);
// Special-row full case mapping (+ narrowing of Latin-1 rows of UTF-16
// batches when `narrow`), see rows.hip.  Reads rows at [cur_s, cur_e),
// writes every row's extents to out_s / out_e (may alias cur_*) and clears
// the wide flag of narrowed rows.  text needs lower_base + 2 * wire bytes.
// flagged_only (UTF-8 batches: every wide row came out of the decoder, which
// flags kRowSpecial candidates and narrows Latin-1 rows itself): only flagged
// rows are scanned.
void launch_row_normalize(uint8_t* text, const int64_t* wire_off, const int64_t* cur_s, const int64_t* cur_e,
                          uint8_t* flags, int64_t* out_s, int64_t* out_e, int64_t n, int64_t tail,
                          int64_t lower_base, bool narrow, const DevCaseTables& ct, int64_t* stats,
                          hipStream_t s, bool flagged_only = false);
// UTF-8 batches: the same for the decoder's list of kRowSpecial rows only
// (stats[2] of them), one wave per row, every listed row at once.  The other
// rows keep the extents and flags the decoder wrote (out_* alias cur_*).
void launch_row_special(uint8_t* text, const int64_t* wire_off, int64_t* cur_s, int64_t* cur_e,
                        uint8_t* flags, const int32_t* special, int64_t n, int64_t tail, int64_t lower_base,
                        const DevCaseTables& ct, int64_t* stats, hipStream_t s);

// Row r: byte offset, wide flag and length in UTF-16 units.
struct RowText {
  int64_t o, len;
  int wide;
};

__device__ __forceinline__ RowText row_text(const DevRawBatch& b, int64_t r) {
  const int64_t o = b.offsets[r];
  const int wide = (b.flags[r] & kRowWide) ? 1 : 0;
  return RowText{o, (b.oend[r] - o) >> wide, wide};
}

// UTF-16 unit j of a row (wide rows may be unaligned: assembled from bytes)
__device__ __forceinline__ uint32_t row_unit(const DevRawBatch& b, const RowText& t, int64_t j) {
  if (!t.wide) return b.text[t.o + j];
  const uint8_t* p = b.text + t.o + 2 * j;
  return uint32_t(p[0]) | (uint32_t(p[1]) << 8);
}

// Per-batch prepared (SELL-64, length-sorted) sparse features.
struct DevPrepared {
  // filter/sort
  int64_t* kept;            // [R]   raw row id of kept row k
  int32_t* nnz;             // [R]   entries of kept row k
  int32_t* sorted;          // [R]   kept index at sorted position p
  int64_t* blk;             // [R/256+2] scratch (block counts / offsets)
  int64_t* hist;            // [kLenBuckets+1]
  // chunk layout
  int32_t* clen8;           // [C]   groups of 8 entries per lane in chunk c
  uint8_t* cfast;           // [C]   1: all rows narrow and short (k_featurize_narrow)
  int64_t* cbase;           // [C+1] first group of chunk c (entries = groups*512)
  int32_t* idx;             // [E]   hashed feature index per entry (-1 = pad)
  void* slot;               // [E]   compact slot per entry (u16 or u32)
  float* y;                 // [R16] label at sorted position p
  float* num;               // [4][R16] numeric features (SoA by sorted position)
  int32_t* perm;            // [R16] kept index at sorted position p, -1 if none
  int64_t* rtext;           // [R16] fast chunks: text byte offset * 512 + length of the row at p
  int64_t* scan_tmp;        // [C/2048+2] tile sums of the multi-block chunk-base scan
  // active set
  uint8_t* flags;           // [Fh]
  int32_t* uniq;            // [Fh]  sorted touched feature ids
  int32_t* slot_of;         // [Fh]  feature id -> slot (valid for touched ids)
  int64_t* ublk;            // [Fh/4096+2]
  // per-row duplicate merging (HashingTF term counts): slots rewritten in
  // place as (slot, count) with the count in `cnt`, chunk lengths in clen8d
  uint16_t* cnt;            // [E]   term count per entry (0 = pad); valid if dedup
  int32_t* clen8d;          // [C]   groups per lane after merging
  int32_t dedup;            // 1: iteration kernels use cnt / clen8d
  // hybrid dense-hot layout (hot_split.hip): the kHot most frequent slots of
  // the batch become 4-bit counts per row, the rest a cold SELL stream
  uint32_t* hot_dense;      // [C][64] uint4: lane (row r, quarter t) = 32 nibbles, hot ids 32t..32t+31
  uint16_t* cslot;          // [E]   cold slots (+ count overflow), same chunk bases as slot, kColdGroup groups
  int32_t* clen8c;          // [C]   cold kColdGroup-entry groups per lane; -1 = chunk left in the plain layout
  int32_t* hot_slot;        // [kHot] slot of hot id h (a zero-weight pad slot when unused)
  uint8_t* hot_of;          // [kMaxHybridSlots] hot id of a slot (0xFF = cold)
  uint16_t* code;           // [8192] remap code of small hashed ids (hot_split.hip)
  uint32_t* slot_hist;      // [max(kMaxHybridSlots, cap_tier + 64)] sampled slot frequencies
  int32_t hybrid;           // 1: iteration kernels use the hybrid layout
  // Tiered layout (active sets beyond LDS, tiered.hip): the near_end - 4
  // most frequent text slots [4, near_end) keep the hybrid layout (hot
  // counts + LDS cold stream); far slots [near_end, 4 + nU) are per-chunk
  // lists of (row << 28 | slot) entries for the forward pass plus a
  // slot-sorted CSC of the same entries for the backward segmented sum.
  int32_t tiered;
  int64_t near_end;
  uint32_t* fslot;          // [E] far entries of chunk c from cbase[c] * 512 on
  int32_t* fcount;          // [C] far entries per chunk
  uint64_t* fhist;          // [cap_tier + 1] entries per far slot, scanned in place into CSC offsets
  uint64_t* fcur;           // [cap_tier] CSC scatter cursors
  uint2* fcsc;              // [E] CSC: (sorted position of the entry's row, far slot) -- one 8-B scattered store
  int32_t* newslot;         // [cap_tier] compact index u -> slot
  int32_t* slot_fid;        // [cap_tier + 64] slot -> feature id
  int64_t* tscan;           // [cap_tier + 1] scan scratch
  int64_t* tscan_blk;       // [cap_tier / 2048 + 4]
  uint32_t* hist_near;      // [kMaxHybridSlots] sampled counts of the near slots (new numbering)
  int64_t* tparam;          // [4] near threshold T, ties to take, far entries, -
  int64_t cap_tier;
  // counters (device): [0]=n_kept [1]=n_unique [2]=groups [3]=error
  int64_t* counters;
  int64_t cap_rows, cap_rows16, cap_entries, cap_chunks, flag_len;
};

struct FeaturizeParams {
  int64_t num_text_features;  // F
  int32_t hash_kind;          // 0 = Java String.hashCode, 1 = Spark-2 murmur3
  int32_t require_retweet;    // filter: isRetweet
  int32_t range_filter;       // filter: begin <= rtCount <= end
  int64_t begin, end;
  int64_t now_ms;
  int32_t idx_mode = 0;       // narrow featurizer ids: 0 all, 1 lazy (sampled chunks), 2 all, no flags
  // chunk slice [c_lo, c_hi) of one launch (prep kernels split into slices,
  // see prep_slices())
  int64_t c_lo = 0, c_hi = INT64_MAX;
};

void upload_lower_tables(hipStream_t s, uint8_t** d_page, uint16_t** d_blocks);

// zero counters, length histogram, n_global[0..ng) and the hybrid slot
// histogram (before launch_filter_sort)
void launch_prep_init(const DevPrepared& p, int64_t* n_global, int ng, hipStream_t s, double* bounds = nullptr,
                      int nb = 0);
void launch_filter_sort(const DevRawBatch& b, const DevPrepared& p, const FeaturizeParams& fp,
                        hipStream_t s);
void launch_chunk_layout(const DevRawBatch& b, const DevPrepared& p, hipStream_t s);
void launch_featurize(const DevRawBatch& b, const DevPrepared& p, const FeaturizeParams& fp,
                      const uint8_t* lower_page, const uint16_t* lower_blocks, hipStream_t s);
// after a lazy (idx_mode 1) featurize: the ids of every fast chunk (idx_mode 2)
void launch_featurize_fast_ids(const DevRawBatch& b, const DevPrepared& p, FeaturizeParams fp, hipStream_t s);
void launch_compact_active(const DevPrepared& p, hipStream_t s);
// DP: flag the ids of all-gathered active lists (< 0: padding) for a second compaction
void launch_flag_ids(const int32_t* ids, int64_t n, const DevPrepared& p, hipStream_t s);
void launch_remap(const DevPrepared& p, int64_t entries, int64_t n_unique, bool u16, hipStream_t s);
// per-row duplicate merging for u16 slot spaces up to 8192 slots
bool dedup_supported(int64_t ns);
void launch_dedup(const DevPrepared& p, int64_t ns, int64_t pad_base, int64_t n_kept, hipStream_t s);

// Hybrid dense-hot layout (u16 slot spaces up to kMaxHybridSlots), in place
// of launch_remap: sampled slot histogram -> top-kHot selection -> per chunk
// 4-bit hot counts + each lane's cold entries (hot_split.hip).
constexpr int kHot = 128;
// Cold stream of the hybrid layout: kColdGroup u16 slots per lane and group
// (one 8-byte load), kColdStride entries per (chunk, group).
constexpr int kColdGroup = 4;
constexpr int kColdStride = 64 * kColdGroup;
constexpr int kMaxHybridSlots = 16384;
// from_text: fast chunks were featurized lazily (idx_mode 1); their ids are
// re-derived from the raw batch b (which must still be resident)
void launch_remap_hybrid(const DevPrepared& p, int64_t entries, int64_t ns, int64_t pad_base, int num_cu,
                         const DevRawBatch& b, const FeaturizeParams& fp, bool from_text, hipStream_t s);

// Exclusive int64 scan (in place safe); tsum: ceil(n / 2048) + 2 scratch.
void launch_scan_excl(const int64_t* in, int64_t* out, int64_t n, int64_t* total, int64_t* tsum, hipStream_t s,
                      int64_t* out2 = nullptr);

// ---------------------------------------------------------------------------
// Tiered layout (tiered.hip), in place of launch_remap_hybrid when the active
// set does not fit LDS.  Step 1 (before the DP sum of the histogram):
// sampled counts of the nU compact slots into slot_hist[4 + u].
void launch_tier_hist(const DevPrepared& p, int64_t n_unique, int num_cu, hipStream_t s);
// Step 2: near tier = the n_near most frequent slots (ties by index, so
// every DP rank numbers slots alike), renumbering, hot ids among the near
// slots, id codes, then the remap (hybrid streams + far lists) and the far
// CSC.  ns: 4 + nU + pads; nl: LDS slot space (4 + n_near + pads).
void launch_tier_layout(const DevPrepared& p, int64_t entries, int64_t n_unique, int64_t n_near, int64_t ns,
                        int64_t nl, int num_cu, const DevRawBatch& b, const FeaturizeParams& fp, bool from_text,
                        hipStream_t s);
// Largest n_near whose LDS slot space 4 + n_near + pads fits the hybrid kernel.
int64_t tier_near_cap();

// ---------------------------------------------------------------------------
// SGD on the compact active set.
//
// Exact, partition-independent GD arithmetic (sgd.hip): every weight enters
// the forward dot as an int32 fixed-point value (scale 2^K from max |w|),
// every row residual enters the gradient as q = rint(r * 2^S) (S from a
// rigorous bound on |r|), and every gradient / loss / numeric-feature sum is
// an int64 fixed-point sum.  Integer sums do not depend on the order rows are
// added in, so a row's contribution is the same whichever layout (hot dense,
// LDS cold stream, far tier), workgroup or DP rank it goes through: DP over
// any sharding is bit-identical to one GPU on the concatenated batch.
struct DevSgd {
  double* w64;          // [F+4] master weights (fp64)
  uint8_t* touched;     // [F+4] 1: the weight was ever written (k_scatter_w / set_weights), for the snapshot
  double* wc64;         // [NS]  compact master weights
  float* wc32;          // [NS]  compact fp32 copy read by the gradient kernel
  // Packed int64 gradient buffer (one all-reduce per GD iteration in DP):
  //   [0, nl)              numeric (2^N_k) and near text (2^S) columns, pads
  //   [nl, nl + tail_len)  loss (2^L), sampled m, DP verdict, per-rank ready words
  //   [far_off, +n_far)    far text slots (2^S), slot - far_base (tiered)
  int64_t* gacc;
  int64_t far_off;      // = nl + tail_len
  int32_t tail_len;
  double* stats;        // [8] fp64 moments of the spill rows (k_batch_stats): n, sum_y, sum_y2, sum_p, sum_p2, sum_e2
  int64_t* stat_i;      // [kStatI] exact int64 batch moments (k_batch_stats)
  int64_t* stat_part;   // [kStatBlocks][16] block partials of k_batch_stats
  float* pbuf;          // [R16] rounded prediction per sorted position (iteration 1)
  double* state;        // [kStateLen] see below
  double* loss_hist;    // [max_iters+1]
  float* pred_out;      // [R] rounded predictions in kept order (optional)
  float* real_out;      // [R] labels in kept order, written with pred_out (the plot's real series)
  double* host_flags;   // [max_iters+1] pinned host memory: done flag after each update
  int64_t* part;        // [nparts][pstride] per-workgroup int64 partial rows
  double* itrec;        // [max_iters+2][kRecStride] per-iteration scale / update records
  uint64_t* tdbg;       // optional phase stamps (TWTML_ITER_TIMING): [iter][wg 0 / last][8]
  uint64_t* kdbg;       // optional per-workgroup start / end stamps (TWTML_ITER_TIMING):
                        // [iter][iteration, far backward, update, rccl stand-in][kKdbgWgs][2]
  const double* bounds; // [8] batch bounds: max row bigram count, max |y|, max |n_k| (k = 0..3)
  const volatile int64_t* ready_word;   // DP: host-mapped, this rank's next-batch ready word
  int32_t rank, world;
  // LDS / partial-row slot space: nl slots (= ns unless tiered), text slots
  // [4, 4 + n_near) in LDS; tiered: far slots [far_base, 4 + n_unique)
  int64_t nl;
  int64_t n_near;
  int64_t far_base;
  float* rbuf;          // [R16] residual per sorted position (tiered backward)
  const int32_t* slot_fid;   // slot -> feature id (tiered); null: uniq[slot - 4]
  const uint2* fcsc;
  const int64_t* far_n;      // device: far entries (CSC length)
  int64_t F;
  int64_t ns;           // 4 + n_unique + pads (rounded)
  int64_t n_unique;
  int64_t pstride;      // nl + 64: slots, then loss, m, 6 batch stats (see sgd_part_stride)
  int32_t nparts;       // partial rows written by the last iteration launch
  double* nrm;          // [2 kNormParts] per-block partial squared norms | max |w| (fixed-order)
  double* wnorm_next;   // [1] |w|^2 after the last batch (state[4] of the next batch)
};

constexpr int kNormParts = 1024;   // grid cap of the norm / gather / scatter kernels
constexpr int kKdbgWgs = 1024;     // workgroups stamped per kernel (TWTML_ITER_TIMING)
// kernels stamped per GD iteration: iteration, far backward, update, and the
// DP RCCL-footprint stand-in (TWTML_RCCL_STANDIN)
constexpr int kKdbgKinds = 4;


// Iteration record i: [0] updates so far, [1] m, [2] update workgroups,
// [3] K, [4] S, [5] L, [6..9] N_0..N_3 (fixed-point exponents of iteration
// i, written by its gradient kernel), [10] |r| bound B, [11] scales invalid
// (diverged); [kRecHead + c kMaxUpdGrid + w] the ||dw||^2 (c = 0), ||w||^2
// (c = 1) and max |w_text| (c = 2) partials of update workgroup w.
constexpr int kMaxUpdGrid = 1024;   // update workgroups: near column tiles + far slot ranges
constexpr int kRecHead = 16;
constexpr int kRecStride = kRecHead + 3 * kMaxUpdGrid;
constexpr int kRecK = 3, kRecS = 4, kRecL = 5, kRecN = 6, kRecB = 10, kRecBad = 11;

// Packed-buffer tail (DevSgd::gacc + nl): loss, sampled m, DP verdict, then
// one ready word per rank (next batch's local prep done: its active-set size + 1).
constexpr int kTailLoss = 0, kTailM = 1, kTailVerdict = 2, kTailReady = 3;
inline int32_t sgd_tail_len(int world) { return (kTailReady + world + 7) / 8 * 8; }

// Exact int64 batch moments (stat_i): n, sum y, sum p, sum y^2 hi/lo,
// sum p^2 hi/lo, sum (y-p)^2 hi/lo (32-bit limbs), spill rows.
constexpr int kStatI = 10;
constexpr int kStatBlocks = 256;   // k_batch_stats grid: stat_part holds kStatBlocks x 16 words
// After iteration 1: the batch moments from pbuf and the labels (exact
// int64; DP: all-reduced as ncclInt64 after the GD loop).
void launch_batch_out(const DevSgd& d, double* out, int64_t* stat, int n_loss, hipStream_t s);
void launch_batch_stats(const DevSgd& d, const DevPrepared& p, hipStream_t s);

// Partial-row stride for a compact space of ns slots (multiple of 64).
constexpr int64_t sgd_part_stride(int64_t ns) { return ns + 64; }

// DevSgd::state: [0] done, [1] converged, [2] updates applied, [3] last
// iteration, [4] |w|^2, [5] rows m, [6] |w_active|^2, [7] diverged (the
// |r| bound or the weights left the fixed-point range: training stopped),
// [8] DP: iteration whose gradient pass this rank skipped, [9] max |w_text|
// at gather (iteration 1's weight scale)
constexpr int kStateLen = 12;
// bounds: [0] max bigram count of a row, [1] max |y|, [2..5] max |n_k|
constexpr int kBoundsLen = 8;

struct SgdParams {
  double step_size;
  double fraction;
  double tol;
  int32_t iteration;    // 1-based
  int32_t num_iterations;
  int64_t row_offset;   // global row id of this rank's kept row 0 (sampling)
  int32_t want_pred;
  int32_t sample;       // fraction < 1
  int32_t ablate;       // perf diagnostics (hybrid): 7 = no chunks (fixed cost), 8 = no far forward
  int32_t dp;           // world > 1: convergence verdicts travel in the gradient all-reduce
  int32_t rank0;        // this rank's verdict is the one that counts (DP)
};

void launch_gather_w(const DevSgd& d, const DevPrepared& p, hipStream_t s);
void launch_norm2(const double* v, int64_t n, double* out, const DevSgd& d, hipStream_t s);
void launch_sgd_iter(const DevSgd& d, const DevPrepared& p, const SgdParams& sp, int64_t groups,
                     bool u16, int grid, hipStream_t s);
// Partial rows an iteration launch of `grid` workgroups writes.
int sgd_partials(int64_t ns, bool u16, int grid);
// DP: gacc[0, nl + 2) = sums of the d.nparts partial rows (+ stats), verdict and ready words
void launch_sgd_reduce(const DevSgd& d, const SgdParams& sp, hipStream_t s);
// nparts > 0: sums the partial rows itself (single GPU, no separate reduce)
void launch_sgd_update(const DevSgd& d, const SgdParams& sp, int nparts, hipStream_t s);
// Far backward of one iteration: gacc[far_off + slot - far_base] += sum of the
// fixed-point residuals of the slot's entries (CSC segmented sums).
void launch_far_grad(const DevSgd& d, const SgdParams& sp, int num_cu, hipStream_t s);
// after the GD loop: convergence of the last update -> state
void launch_sgd_finish(const DevSgd& d, const SgdParams& sp, hipStream_t s);
// DP cost model: a kernel with the CU footprint of an RCCL all-reduce of n
// int64 (wgs workgroups of 256 threads reading n and writing n words), with
// TWTML_ITER_TIMING stamps as kind 3 of iteration `it`
void launch_rccl_standin(const int64_t* src, int64_t* dst, int64_t n, int wgs, uint64_t* kdbg, int it,
                         hipStream_t s);
void launch_scatter_w(const DevSgd& d, const DevPrepared& p, hipStream_t s);
// |w|^2 for the next batch: |w_rest|^2 + |w_active after training|^2, from
// the scatter's block partials (trained) or state[4] unchanged (no rows)
void launch_norm_next(const DevSgd& d, bool trained, hipStream_t s);
// state[4] = wnorm_next (instead of a full |w|^2 pass over all F+4 weights)
void launch_norm_carry(const DevSgd& d, hipStream_t s);
// batch bounds of the scale choice (max row bigram count, max |y|, max |n_k|)
// of this rank's kept rows -> out[kBoundsLen] (zeroed here)
void launch_batch_bounds(const DevPrepared& p, double* out, hipStream_t s, bool zeroed = false);
int sgd_lds_rep(int64_t ns);
// the hybrid iteration kernel's LDS (gradient replicas + hot partials) fits
bool sgd_hybrid_fits(int64_t ns);
int sgd_iter_grid(int64_t ns, int64_t n_kept, int num_cu, bool hybrid);

// ---------------------------------------------------------------------------
// DP batch preparation (dp_prep.hip): one packet per rank, all-gathered once.
// Packet (int32 words): header kC1HeaderWords (16 int64: kept rows, active
// ids, kBoundsLen fp64 bounds, 0) then max_u (id, sampled count) pairs.
constexpr int kC1HeaderWords = 32;
__host__ __device__ constexpr int64_t c1_packet_words(int64_t max_u) { return kC1HeaderWords + 2 * max_u; }
// this rank's packet from its local active set (slot_hist[4 + u] = sampled counts)
void launch_pack_c1(const DevPrepared& p, const double* bounds, int32_t* packet, int64_t n_unique, hipStream_t s);
// flag the ids of all gathered packets (the next compaction numbers the union)
void launch_union_flag(const int32_t* gathered, int world, int64_t max_u, const DevPrepared& p, hipStream_t s);
// slot_hist[4 + slot_of[id]] += gathered sampled counts (union slots numbered)
void launch_union_hist(const int32_t* gathered, int world, int64_t max_u, const DevPrepared& p, hipStream_t s);

// ---- sparse weight snapshot (snapshot.hip): non-zero (index, value) pairs
// of the master weights, in index order, for non-blocking checkpoints --------
constexpr int64_t kSnapChunk = 16384;   // weights per counting / writing workgroup
int64_t snapshot_chunks(int64_t n);
// tidx / tval: scratch pairs of n entries (each chunk's pairs packed at its base);
// touched (nullable): only weights marked there can be non-zero, the others
// are not read
void launch_snapshot(const double* w, const uint8_t* touched, int64_t n, uint32_t* cnt, int64_t* off,
                     int32_t* tidx, double* tval, int32_t* idx, double* val, volatile int64_t* host_total,
                     hipStream_t s);
// touched[i] = w[i] != 0 for every weight (after set_weights)
void launch_mark_nonzero(const double* w, uint8_t* touched, int64_t n, hipStream_t s);

// (k-means launchers: kmeans_kernels.h)

// Grid-cap multiplier of the grid-stride prep kernels (TWTML_PREP_WG_MULT,
// default 1): prep workgroups that live for the whole kernel hold their CUs
// against the GD loop's next launch on the compute stream.
// Launches per long prep kernel (TWTML_PREP_SLICES, default 1): the chunk
// range is split so a launch on the prep stream ends before the GD loop's
// next kernel has waited long behind it.
inline int prep_slices() {
  static const int m = [] {
    const char* e = std::getenv("TWTML_PREP_SLICES");
    const int v = e ? std::atoi(e) : 1;
    return v >= 1 && v <= 64 ? v : 1;
  }();
  return m;
}

// def: the default when the variable is unset (4 for the tiered layout's
// remap / far CSC: +0.5-1 % on wide and 1e8 murmur3; 1 for featurize, where
// 4x the grid costs the toy bench ~0.5 %).
inline int prep_grid_mult(int def = 1) {
  static const int m = [] {
    const char* e = std::getenv("TWTML_PREP_WG_MULT");
    const int v = e ? std::atoi(e) : 0;
    return v >= 1 && v <= 64 ? v : 0;
  }();
  return m ? m : def;
}

}  // namespace twtml
