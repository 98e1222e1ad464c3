// Streaming k-means engine (K8-K11) on one GPU, RCCL data parallel.
#pragma once
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <memory>
#include <vector>

#include "comm.h"
#include "common.h"
#include "engine.h"
#include "kernels.h"

namespace twtml {

struct KMConfig {
  int32_t k = 3;
  int32_t text_dims = 0;       // hashed bigram dims appended to [retweetCount, followers]
  double decay = 0.8705505632961241;  // setHalfLife(5, "batches")
  int32_t points_unit = 0;     // timeUnit "points"
  int32_t scale = 1;           // StandardScaler(false, true) per batch
  // matrix-core assignment: 1 = bf16x3 split MFMA where 16 <= dp <= 128 and
  // k <= 4096 (fp32 MFMA otherwise), 2 = fp32 MFMA only, 0 = scalar fp32
  int32_t mfma = 1;
  int64_t max_rows = 1 << 16;
  int64_t max_units = (1 << 16) * 281;
  int32_t force_dp = 0;        // DP collectives even with a world-1 communicator (also TWTML_FORCE_DP=1)
  int32_t raw_slots = kDefaultRawSlots;   // device raw-batch slots (H2D run-ahead depth + 1)
};

struct KMResult {
  int64_t n_raw = 0, n_local = 0, n_global = 0;
  std::vector<double> std;     // scaler std per column
  std::vector<int32_t> labels; // labels of this rank's points (new model) if requested
  float ms = 0.f;
};

class KMEngine {
 public:
  KMEngine(int device, const KMConfig& cfg, std::shared_ptr<Comm> comm);
  ~KMEngine();
  void submit(const HostBatch& hb, int64_t n, int64_t bytes, int slot, const uint8_t* ext_text = nullptr);
  KMResult process(int slot, bool want_labels);
  // Forget a submitted batch that will not be processed: waits for its H2D
  // (the staging buffer may then be rewritten); the copy stream keeps the
  // slot's next H2D in order behind it.
  void discard(int slot) { raw_.wait_h2d(slot); }
  void set_state(const double* centers, const double* weights);
  void get_state(double* centers, double* weights) const;
  // Debug/test: the labels left by the last process() (the update's
  // assignment with the old centres when want_labels was false).
  std::vector<int32_t> debug_labels() const;
  // Debug/test: the unscaled fp32 feature rows [n_local][dp] of the last batch.
  std::vector<float> debug_features() const;
  int k() const { return cfg_.k; }
  int d() const { return d_; }
  int dp() const { return dp_; }
  int64_t h2d_bytes() const { return raw_.h2d_bytes(); }
  int raw_slots() const { return raw_.count(); }
  void synchronize();

 private:
  int device_;
  KMConfig cfg_;
  int d_, dp_;
  bool dist_ = false;   // DP collectives: world > 1, or forced with a world-1 communicator
  std::shared_ptr<Comm> comm_;
  hipStream_t compute_ = nullptr, copy_ = nullptr;
  RawSlots raw_;
  DevPrepared prep_{};
  float* X_ = nullptr;
  double *centers_ = nullptr, *weights_ = nullptr, *sums_ = nullptr;
  int64_t* sums_i_ = nullptr;          // [k d + k] per-cluster integer sums of q, counts (all-reduced)
  int64_t* qmom_ = nullptr;            // [d] column max | n | [d][4] integer moments (all-reduced)
  int64_t* host_q_ = nullptr;          // pinned copy of qmom_
  void* host_fac_ = nullptr;           // pinned [dp] fp64 + [dp] fp32 factors (H2D staging)
  float *c32_ = nullptr, *cnorm_ = nullptr, *fac32_ = nullptr;
  double *fac64_ = nullptr, *blend_ = nullptr;
  int32_t *labels_ = nullptr, *order_ = nullptr, *refine_ = nullptr;
  uint16_t* frag_ = nullptr;           // bf16x3 centre fragments
  float* cnp_ = nullptr;               // |c|^2 padded to 32-centre tiles
  int64_t* lhist_ = nullptr;
  uint8_t* lower_page_ = nullptr;
  uint16_t* lower_blocks_ = nullptr;
  double* host_out_ = nullptr;
  hipEvent_t ev0_ = nullptr, ev1_ = nullptr;
};

void bind_kmeans(pybind11::module_& m);

}  // namespace twtml
