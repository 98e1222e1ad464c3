// KMEngine: the streaming k-means micro-batch pipeline (see kmeans.hip).
#include "kmeans_engine.h"
#include "alloc.h"
#include "trace.h"

#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "kmeans_kernels.h"

namespace py = pybind11;

namespace twtml {

template <typename T>
static T* km_alloc(size_t n) {
  return static_cast<T*>(dev_alloc(n * sizeof(T)));
}

static int pad_dim(int d) {
  for (int p : {2, 4, 8, 16, 32, 64, 128})
    if (d <= p) return p;
  return d;
}

KMEngine::KMEngine(int device, const KMConfig& cfg, std::shared_ptr<Comm> comm)
    : device_(device), cfg_(cfg), comm_(std::move(comm)) {
  if (cfg_.k < 1) throw std::invalid_argument("k must be >= 1");
  // the feature kernel keeps a per-wave bigram histogram in LDS (4 waves x 4 B)
  if (cfg_.text_dims < 0 || cfg_.text_dims > 4000)
    throw std::invalid_argument("text_dims must be in [0, 4000]");
  if (cfg_.max_rows <= 0 || cfg_.max_rows >= (int64_t(1) << 31)) throw std::invalid_argument("bad max_rows");
  d_ = 2 + cfg_.text_dims;
  const char* fdp = std::getenv("TWTML_FORCE_DP");
  dist_ = comm_ && (comm_->world() > 1 || cfg_.force_dp != 0 || (fdp && fdp[0] == '1'));
  dp_ = pad_dim(d_);
  TWTML_HIP_CHECK(hipSetDevice(device_));
  TWTML_HIP_CHECK(hipStreamCreateWithFlags(&compute_, hipStreamNonBlocking));
  TWTML_HIP_CHECK(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking));
  raw_.init(cfg_.raw_slots, cfg_.max_rows, text_bytes_for_units(cfg_.max_units));
  const int64_t R = cfg_.max_rows;
  prep_.cap_rows = R;
  prep_.kept = km_alloc<int64_t>(size_t(R));
  prep_.nnz = km_alloc<int32_t>(size_t(R));
  prep_.blk = km_alloc<int64_t>(size_t(R / kBlock + 2));
  prep_.hist = km_alloc<int64_t>(kLenBuckets + 1);
  prep_.counters = km_alloc<int64_t>(8);
  X_ = km_alloc<float>(size_t(R) * size_t(dp_));
  const size_t k = size_t(cfg_.k), d = size_t(d_);
  centers_ = km_alloc<double>(k * d);
  weights_ = km_alloc<double>(k);
  sums_ = km_alloc<double>(k * d + k);
  sums_i_ = km_alloc<int64_t>(k * d + k);
  qmom_ = km_alloc<int64_t>(d + 1 + 4 * d);   // [d] column max | n | [d][4] sums of q and limbs
  fac64_ = km_alloc<double>(size_t(dp_));
  fac32_ = km_alloc<float>(size_t(dp_));
  blend_ = km_alloc<double>(2 * k);
  c32_ = km_alloc<float>(k * size_t(dp_));
  cnorm_ = km_alloc<float>(k);
  labels_ = km_alloc<int32_t>(size_t(R));
  order_ = km_alloc<int32_t>(size_t(R));
  refine_ = km_alloc<int32_t>(6 * size_t(R));
  frag_ = km_alloc<uint16_t>(km_frag_elems(cfg_.k, dp_));
  cnp_ = km_alloc<float>(size_t((cfg_.k + 31) / 32) * 32);
  lhist_ = km_alloc<int64_t>(k + 1);
  // on the compute stream: the null stream does not order against it
  TWTML_HIP_CHECK(hipMemsetAsync(centers_, 0, sizeof(double) * k * d, compute_));
  TWTML_HIP_CHECK(hipMemsetAsync(weights_, 0, sizeof(double) * k, compute_));
  upload_lower_tables(compute_, &lower_page_, &lower_blocks_);
  TWTML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&host_out_), sizeof(double) * (4 + d),
                                hipHostMallocDefault));
  TWTML_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&host_q_), sizeof(int64_t) * (d + 1 + 4 * d),
                                hipHostMallocDefault));
  TWTML_HIP_CHECK(hipHostMalloc(&host_fac_, sizeof(double) * size_t(dp_) + sizeof(float) * size_t(dp_),
                                hipHostMallocDefault));
  TWTML_HIP_CHECK(hipEventCreate(&ev0_));
  TWTML_HIP_CHECK(hipEventCreate(&ev1_));
  launch_km_centers32(centers_, cfg_.k, d_, dp_, c32_, cnorm_, compute_);
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
}

KMEngine::~KMEngine() {
  (void)hipSetDevice(device_);
  // a fault of this engine's last work surfaces here: report it (and keep it
  // for teardown_errors()) instead of leaving it to the next engine's first call
  report_teardown_error("KMEngine", device_, hipDeviceSynchronize());
  raw_.release();
  void* bufs[] = {prep_.kept, prep_.nnz, prep_.blk, prep_.hist, prep_.counters, X_, centers_,
                  weights_, sums_, sums_i_, qmom_, c32_, cnorm_, labels_, order_, refine_, frag_, cnp_, lhist_, fac64_, fac32_, blend_,
                  lower_page_, lower_blocks_};
  for (void* b : bufs) if (b) (void)hipFree(b);
  if (host_out_) (void)hipHostFree(host_out_);
  if (host_q_) (void)hipHostFree(host_q_);
  if (host_fac_) (void)hipHostFree(host_fac_);
  (void)hipEventDestroy(ev0_);
  (void)hipEventDestroy(ev1_);
  (void)hipStreamDestroy(compute_);
  (void)hipStreamDestroy(copy_);
}

void KMEngine::submit(const HostBatch& hb, int64_t n, int64_t bytes, int slot, const uint8_t* ext_text) {
  TraceRange tr("twtml.km.submit_h2d");
  TWTML_HIP_CHECK(hipSetDevice(device_));
  // features read only retweetCount and followersCount (scalar rows 0, 1)
  raw_.submit(hb, n, bytes, slot, copy_, 2, ext_text);
}

KMResult KMEngine::process(int slot, bool want_labels) {
  TraceRange tr("twtml.km.batch");
  TWTML_HIP_CHECK(hipSetDevice(device_));
  hipStream_t s = compute_;
  const int k = cfg_.k, d = d_;
  KMResult res;
  const DevRawBatch b = raw_.acquire(slot, s);
  res.n_raw = b.n;
  TWTML_HIP_CHECK(hipEventRecord(ev0_, s));
  FeaturizeParams fp{1, 0, 1, 0, 0, 0, 0};   // filter: isRetweet only (KMeans.scala:77-80)
  TWTML_HIP_CHECK(hipMemsetAsync(prep_.counters, 0, 8 * sizeof(int64_t), s));
  launch_filter_only(b, prep_, fp, s);
  launch_km_features(b, prep_.kept, prep_.counters, X_, dp_, cfg_.text_dims, lower_page_,
                     lower_blocks_, cfg_.max_rows, s);
  raw_.release_slot(slot, s);
  // K11 scaler, exact: the column max (all-reduced MAX) fixes every column's
  // quantization shift, then n and the integer column sums (all-reduced SUM);
  // both are the same bits on every rank and in any summation order
  int64_t* mx = qmom_;
  int64_t* mq = qmom_ + d;
  TWTML_HIP_CHECK(hipMemsetAsync(qmom_, 0, sizeof(int64_t) * size_t(d + 1 + 4 * d), s));
  launch_km_colmax(X_, prep_.counters, d, dp_, mx, cfg_.max_rows, s);
  if (dist_) comm_->allreduce(mx, size_t(d), ncclInt64, ncclMax, s);
  launch_km_moments_q(X_, prep_.counters, d, dp_, mx, mq, cfg_.max_rows, s);
  if (dist_) comm_->allreduce(mq, size_t(1 + 4 * d), ncclInt64, ncclSum, s);
  TWTML_HIP_CHECK(hipMemcpyAsync(host_q_, qmom_, sizeof(int64_t) * size_t(d + 1 + 4 * d), hipMemcpyDeviceToHost, s));
  TWTML_HIP_CHECK(hipMemcpyAsync(host_out_ + 1, prep_.counters, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  res.n_global = host_q_[d];
  int64_t nl;
  std::memcpy(&nl, host_out_ + 1, sizeof(int64_t));
  res.n_local = nl;
  if (res.n_global == 0) {                  // if (rdd.count > 0) { ... }
    TWTML_HIP_CHECK(hipEventRecord(ev1_, s));
    TWTML_HIP_CHECK(hipStreamSynchronize(s));
    return res;
  }
  // std_j = sqrt(M2_j / (n - 1)) (n < 2 -> 0); factor_j = std_j != 0 ? 1 / std_j : 0
  // (StandardScalerModel.transform), M2 = (n sum q^2 - (sum q)^2) / n in
  // 128-bit integers; scale == 0 -> factor 1
  double* f64 = static_cast<double*>(host_fac_);
  float* f32 = reinterpret_cast<float*>(f64 + dp_);
  if (cfg_.scale) res.std.assign(size_t(d), 0.0);
  for (int j = 0; j < dp_; ++j) {
    double f = 0.0;
    if (j < d) {
      if (cfg_.scale) {
        const int64_t n = res.n_global;
        const int64_t* m = host_q_ + d + 1 + 4 * j;
        const __int128 s2 = (__int128(m[1]) << 32) + (__int128(m[2]) << 16) + __int128(m[3]);
        const __int128 num = __int128(n) * s2 - __int128(m[0]) * __int128(m[0]);
        double sd = 0.0;
        if (n > 1 && num > 0) {
          const long double var = std::ldexp(static_cast<long double>(num), 2 * km_quant_shift(host_q_[j])) /
                                  (static_cast<long double>(n) * static_cast<long double>(n - 1));
          sd = std::sqrt(static_cast<double>(var));
        }
        res.std[size_t(j)] = sd;
        f = sd != 0.0 ? 1.0 / sd : 0.0;
      } else {
        f = 1.0;
      }
    }
    f64[j] = f;
    f32[j] = float(f);
  }
  TWTML_HIP_CHECK(hipMemcpyAsync(fac64_, f64, sizeof(double) * size_t(dp_), hipMemcpyHostToDevice, s));
  TWTML_HIP_CHECK(hipMemcpyAsync(fac32_, f32, sizeof(float) * size_t(dp_), hipMemcpyHostToDevice, s));
  // K8 assignment with the current centres, K9 sums, K10 update.  The
  // near-tie lists in refine_, their counts in counters[5..6].
  auto* refine_cnt = reinterpret_cast<unsigned long long*>(prep_.counters + 5);
  launch_km_assign(X_, fac32_, fac64_, prep_.counters, c32_, cnorm_, centers_, k, d, dp_, labels_,
                   refine_, refine_cnt, frag_, cnp_, cfg_.max_rows, cfg_.mfma != 0, cfg_.mfma == 1, s);
  // TWTML_DEBUG_KM=1: per-assignment near-tie counts (synchronises the stream)
  static const bool debug = std::getenv("TWTML_DEBUG_KM") != nullptr;
  auto debug_refine = [&](const char* what) {
    if (!debug) return;
    unsigned long long c[2];
    TWTML_HIP_CHECK(hipMemcpyAsync(c, refine_cnt, sizeof(c), hipMemcpyDeviceToHost, s));
    TWTML_HIP_CHECK(hipStreamSynchronize(s));
    std::fprintf(stderr, "[km] %s: n=%lld refine full=%llu candidates=%llu\n", what,
                 static_cast<long long>(res.n_local), c[0], c[1]);
  };
  debug_refine("update");
  TWTML_HIP_CHECK(hipMemsetAsync(sums_i_, 0, sizeof(int64_t) * (size_t(k) * d + k), s));
  launch_km_cluster_sums(X_, mx, labels_, prep_.counters, k, d, dp_, lhist_, order_, sums_i_, cfg_.max_rows, s,
                         &scan_excl_launch);
  if (dist_) comm_->allreduce(sums_i_, size_t(k) * d + k, ncclInt64, ncclSum, s);
  launch_km_sums_f64(sums_i_, mx, fac64_, k, d, sums_, sums_ + size_t(k) * d, s);
  launch_km_update(centers_, weights_, sums_, sums_ + size_t(k) * d, k, d, cfg_.decay,
                   cfg_.points_unit != 0, blend_, c32_, cnorm_, dp_, s);
  if (want_labels)   // KMeans.scala:113 predicts with the updated model
    launch_km_assign(X_, fac32_, fac64_, prep_.counters, c32_, cnorm_, centers_, k, d, dp_, labels_,
                     refine_, refine_cnt, frag_, cnp_, cfg_.max_rows, cfg_.mfma != 0, cfg_.mfma == 1, s);
  if (want_labels) debug_refine("predict");
  TWTML_HIP_CHECK(hipEventRecord(ev1_, s));
  if (want_labels && res.n_local > 0) {
    res.labels.resize(size_t(res.n_local));
    TWTML_HIP_CHECK(hipMemcpyAsync(res.labels.data(), labels_, sizeof(int32_t) * size_t(res.n_local),
                                   hipMemcpyDeviceToHost, s));
  }
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
  if (comm_) comm_->check_async();
  TWTML_HIP_CHECK(hipEventElapsedTime(&res.ms, ev0_, ev1_));
  return res;
}

void KMEngine::set_state(const double* centers, const double* weights) {
  TWTML_HIP_CHECK(hipSetDevice(device_));
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
  // stream-ordered and complete on return (a pageable hipMemcpy may return
  // before its DMA lands, unordered against the non-blocking compute stream)
  TWTML_HIP_CHECK(hipMemcpyAsync(centers_, centers, sizeof(double) * size_t(cfg_.k) * d_, hipMemcpyHostToDevice,
                                 compute_));
  TWTML_HIP_CHECK(hipMemcpyAsync(weights_, weights, sizeof(double) * size_t(cfg_.k), hipMemcpyHostToDevice,
                                 compute_));
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
  launch_km_centers32(centers_, cfg_.k, d_, dp_, c32_, cnorm_, compute_);
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
}

std::vector<int32_t> KMEngine::debug_labels() const {
  TWTML_HIP_CHECK(hipSetDevice(device_));
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
  int64_t n = 0;
  TWTML_HIP_CHECK(hipMemcpy(&n, prep_.counters, sizeof(int64_t), hipMemcpyDeviceToHost));
  std::vector<int32_t> out(size_t(std::max<int64_t>(n, 0)));
  if (n > 0) TWTML_HIP_CHECK(hipMemcpy(out.data(), labels_, sizeof(int32_t) * size_t(n), hipMemcpyDeviceToHost));
  return out;
}

std::vector<float> KMEngine::debug_features() const {
  TWTML_HIP_CHECK(hipSetDevice(device_));
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
  int64_t n = 0;
  TWTML_HIP_CHECK(hipMemcpy(&n, prep_.counters, sizeof(int64_t), hipMemcpyDeviceToHost));
  std::vector<float> out(size_t(std::max<int64_t>(n, 0)) * size_t(dp_));
  if (n > 0) TWTML_HIP_CHECK(hipMemcpy(out.data(), X_, sizeof(float) * out.size(), hipMemcpyDeviceToHost));
  return out;
}

void KMEngine::get_state(double* centers, double* weights) const {
  TWTML_HIP_CHECK(hipSetDevice(device_));
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
  TWTML_HIP_CHECK(hipMemcpy(centers, centers_, sizeof(double) * size_t(cfg_.k) * d_, hipMemcpyDeviceToHost));
  TWTML_HIP_CHECK(hipMemcpy(weights, weights_, sizeof(double) * size_t(cfg_.k), hipMemcpyDeviceToHost));
}

void KMEngine::synchronize() {
  TWTML_HIP_CHECK(hipSetDevice(device_));
  TWTML_HIP_CHECK(hipStreamSynchronize(compute_));
  TWTML_HIP_CHECK(hipStreamSynchronize(copy_));
}

// ---------------------------------------------------------------------------
void bind_kmeans(py::module_& m) {
  py::class_<KMEngine, std::shared_ptr<KMEngine>>(m, "KMEngine")
      .def(py::init([](int device, const py::dict& d, std::shared_ptr<Comm> comm) {
             KMConfig c;
#define GET(name, type) if (d.contains(#name)) c.name = d[#name].cast<type>();
             GET(k, int32_t) GET(text_dims, int32_t) GET(decay, double) GET(points_unit, int32_t)
             GET(scale, int32_t) GET(mfma, int32_t) GET(max_rows, int64_t) GET(max_units, int64_t)
             GET(force_dp, int32_t) GET(raw_slots, int32_t)
#undef GET
             py::gil_scoped_release nogil;
             return std::make_shared<KMEngine>(device, c, comm);
           }),
           py::arg("device"), py::arg("config"), py::arg("comm") = nullptr)
      .def("submit", [](KMEngine& e, const HostBatch& hb, int64_t n, int64_t bytes, int slot, uintptr_t ext_text) {
        py::gil_scoped_release nogil;
        e.submit(hb, n, bytes, slot, reinterpret_cast<const uint8_t*>(ext_text));
      }, py::arg("host_batch"), py::arg("n"), py::arg("bytes"), py::arg("slot"), py::arg("ext_text") = 0)
      .def("discard", [](KMEngine& e, int slot) {
        py::gil_scoped_release nogil;
        e.discard(slot);
      }, py::arg("slot"), "forget a submitted batch that will not be processed")
      .def_property_readonly("h2d_bytes", &KMEngine::h2d_bytes, "host-to-device bytes submitted so far")
      .def_property_readonly("raw_slots", &KMEngine::raw_slots, "device raw-batch slots")
      .def("process", [](KMEngine& e, int slot, bool want_labels) {
        KMResult r;
        {
          py::gil_scoped_release nogil;
          r = e.process(slot, want_labels);
        }
        py::dict out;
        out["n_raw"] = r.n_raw;
        out["n_local"] = r.n_local;
        out["n"] = r.n_global;
        out["std"] = r.std;
        out["ms"] = r.ms;
        if (!r.labels.empty())
          out["pred"] = py::array_t<int32_t>(py::ssize_t(r.labels.size()), r.labels.data());
        else
          out["pred"] = py::none();
        return out;
      }, py::arg("slot"), py::arg("want_labels") = false)
      .def("set_state", [](KMEngine& e, py::array_t<double, py::array::c_style | py::array::forcecast> c,
                           py::array_t<double, py::array::c_style | py::array::forcecast> w) {
        if (c.size() != py::ssize_t(e.k()) * e.d() || w.size() != e.k())
          throw std::invalid_argument("state shape mismatch");
        e.set_state(c.data(), w.data());
      })
      .def("get_state", [](const KMEngine& e) {
        py::array_t<double> c({py::ssize_t(e.k()), py::ssize_t(e.d())});
        py::array_t<double> w(py::ssize_t(e.k()));
        e.get_state(c.mutable_data(), w.mutable_data());
        return py::make_tuple(c, w);
      })
      .def("synchronize", &KMEngine::synchronize)
      .def("debug_labels", [](const KMEngine& e) {
        std::vector<int32_t> v;
        {
          py::gil_scoped_release nogil;
          v = e.debug_labels();
        }
        return py::array_t<int32_t>(py::ssize_t(v.size()), v.data());
      })
      .def("debug_features", [](const KMEngine& e) {
        std::vector<float> v;
        {
          py::gil_scoped_release nogil;
          v = e.debug_features();
        }
        const py::ssize_t dp = py::ssize_t(e.dp());
        py::array_t<float> a({py::ssize_t(v.size()) / dp, dp});
        std::copy(v.begin(), v.end(), a.mutable_data());
        return a;
      })
      .def_property_readonly("k", &KMEngine::k)
      .def_property_readonly("d", &KMEngine::d);
}

}  // namespace twtml
