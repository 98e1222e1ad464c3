// pybind11 bindings of the MI355X engine (_twtml_hip).
#include <ctime>
#include <hip/hip_runtime.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <memory>

#include "alloc.h"
#include "comm.h"
#include "common.h"
#include "engine.h"
#include "kmeans_engine.h"

namespace py = pybind11;
using namespace twtml;

template <typename T>
static py::array_t<T> view(T* ptr, std::vector<py::ssize_t> shape, py::handle owner) {
  std::vector<py::ssize_t> strides(shape.size());
  py::ssize_t st = sizeof(T);
  for (int i = int(shape.size()) - 1; i >= 0; --i) {
    strides[size_t(i)] = st;
    st *= shape[size_t(i)];
  }
  return py::array_t<T>(shape, strides, ptr, owner);
}

static LRConfig lr_config(const py::dict& d) {
  LRConfig c;
#define GET(name, type) if (d.contains(#name)) c.name = d[#name].cast<type>();
  GET(num_text_features, int64_t) GET(hash_kind, int32_t) GET(step_size, double)
  GET(num_iterations, int32_t) GET(fraction, double) GET(tol, double) GET(begin, int64_t)
  GET(end, int64_t) GET(require_retweet, int32_t) GET(range_filter, int32_t)
  GET(max_rows, int64_t) GET(max_units, int64_t) GET(sgd_grid, int32_t)
  GET(early_exit_depth, int32_t) GET(ablate, int32_t) GET(dedup, int32_t) GET(hybrid, int32_t) GET(lazy_idx, int32_t)
  GET(overlap, int32_t) GET(force_dp, int32_t) GET(comm_timing, int32_t) GET(raw_slots, int32_t)
#undef GET
  return c;
}

static py::dict result_dict(BatchResult& r) {
  py::dict d;
  d["n_raw"] = r.n_raw;
  d["n_kept"] = r.n_kept;
  d["n_kept_global"] = r.n_kept_global;
  d["n_unique"] = r.n_unique;
  d["entries"] = r.entries;
  d["iterations"] = r.iterations;
  d["converged"] = r.converged;
  d["diverged"] = r.diverged;
  d["stats"] = std::vector<double>(r.stats, r.stats + 6);
  d["loss_history"] = r.loss_history;
  d["prep_ms"] = r.prep_ms;
  d["rows_lowered"] = r.rows_lowered;
  d["rows_narrowed"] = r.rows_narrowed;
  d["tiered"] = r.tiered;
  d["n_near"] = r.n_near;
  d["train_ms"] = r.train_ms;
  d["comm_iters"] = r.comm_iters;
  d["comm_ms"] = r.comm_ms;
  d["comm_bytes"] = r.comm_bytes;
  d["stats_spill"] = r.stats_spill;
  d["wait_ms"] = r.wait_ms;
  d["train_wall_ms"] = r.train_wall_ms;
  d["prepared_ahead"] = r.prepared_ahead;
  d["phases"] = std::vector<float>(r.phases, r.phases + 7);
  if (!r.real.empty()) {
    auto* v = new std::vector<float>(std::move(r.real));
    py::capsule own(v, [](void* p) { delete static_cast<std::vector<float>*>(p); });
    d["real"] = py::array_t<float>({py::ssize_t(v->size())}, {py::ssize_t(sizeof(float))}, v->data(), own);
  } else {
    d["real"] = py::none();
  }
  if (!r.pred.empty()) {
    auto* v = new std::vector<float>(std::move(r.pred));
    py::capsule own(v, [](void* p) { delete static_cast<std::vector<float>*>(p); });
    d["pred"] = py::array_t<float>({py::ssize_t(v->size())}, {py::ssize_t(sizeof(float))}, v->data(), own);
  } else {
    d["pred"] = py::none();
  }
  return d;
}

PYBIND11_MODULE(_twtml_hip, m) {
  m.doc() = "twtml MI355X engine: HIP/CDNA4 kernels, micro-batch engines, RCCL";
  m.attr("RAW_SLOTS") = kDefaultRawSlots;   // default device raw-batch slots per engine (submit/process)

  m.def("pci_bus_id", [](int device) {
    char buf[64] = {0};
    TWTML_HIP_CHECK(hipDeviceGetPCIBusId(buf, int(sizeof(buf)), device));
    return std::string(buf);
  }, py::arg("device"));
  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  m.def("device_name", [](int dev) {
    hipDeviceProp_t p;
    TWTML_HIP_CHECK(hipGetDeviceProperties(&p, dev));
    return std::string(p.name) + " (" + p.gcnArchName + ", " + std::to_string(p.multiProcessorCount) + " CUs)";
  });
  m.def("rccl_unique_id", []() { return py::bytes(rccl_unique_id()); });
  m.def("tier_near_cap", &tier_near_cap, "LDS-resident text slots of the tiered layout");
  m.def("sgd_hybrid_fits", &sgd_hybrid_fits, py::arg("ns"));
  // Page-lock a host buffer (e.g. a receiver's batch) so submit(ext_text=...)
  // DMAs straight from it; it MUST be unregistered before the buffer is freed
  // (ops/lr_engine.py register_host ties that to the array's lifetime).  A
  // registration the runtime still holds for memory that was freed stays in
  // its host-pointer map: a later buffer mapped at an overlapping address is
  // then resolved to the stale registration (wrong size: hipMemcpyAsync
  // "invalid argument"; wrong GPU mapping: an illegal memory access in a DMA).
  // The registry below refuses such an overlap instead (round-5 faults,
  // profiles/README.md "Round 6").
  m.def("host_register", [](uintptr_t ptr, size_t bytes) {
    host_registry_add(ptr, bytes);
    const hipError_t e = hipHostRegister(reinterpret_cast<void*>(ptr), bytes, hipHostRegisterDefault);
    if (e != hipSuccess) {
      host_registry_remove(ptr);
      TWTML_HIP_CHECK(e);
    }
  }, py::arg("ptr"), py::arg("bytes"));
  m.def("host_unregister", [](uintptr_t ptr) {
    py::gil_scoped_release nogil;
    // no DMA may still read the range once it is unpinned (and then freed)
    TWTML_HIP_CHECK(hipDeviceSynchronize());
    host_registry_remove(ptr);
    TWTML_HIP_CHECK(hipHostUnregister(reinterpret_cast<void*>(ptr)));
  }, py::arg("ptr"));
  m.def("host_registrations", [] {
    std::vector<std::pair<uintptr_t, size_t>> v = host_registry_snapshot();
    return v;
  }, "live host_register ranges (ptr, bytes)");
  m.def("teardown_errors", &take_teardown_errors,
        "device errors engine destructors found since the last call (and clears them)");
  m.attr("DEBUG_SYNC") = debug_sync_enabled();
  m.def("rccl_version", &rccl_version);
  // device bytes allocated by the engines so far (monotonic; HBM batch sizing)
  m.def("device_bytes_allocated", [] { return uint64_t(dev_alloc_bytes().load()); });

  py::class_<Comm, std::shared_ptr<Comm>>(m, "CommBase")
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("world", &Comm::world)
      .def_property_readonly("kind", &Comm::kind)
      .def("abort", &Comm::abort)
      .def("check", &Comm::check_async)
      .def("counters", [](const Comm& c) {
        const auto v = c.counters();
        py::dict d;
        d["allreduce_calls"] = v[0];
        d["allreduce_bytes"] = v[1];
        d["allgather_calls"] = v[2];
        d["allgather_bytes"] = v[3];
        d["broadcast_calls"] = v[4];
        d["broadcast_bytes"] = v[5];
        return d;
      })
      // In-place fp64 sum over a device buffer on a private stream, then
      // synchronise: exercises the communicator outside an engine (tests,
      // link checks).  The engines issue their collectives on their own streams.
      .def("allreduce_f64", [](Comm& c, uintptr_t dev_ptr, size_t count) {
        py::gil_scoped_release nogil;
        hipStream_t s;
        TWTML_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        c.allreduce(reinterpret_cast<void*>(dev_ptr), count, ncclFloat64, ncclSum, s);
        TWTML_HIP_CHECK(hipStreamSynchronize(s));
        TWTML_HIP_CHECK(hipStreamDestroy(s));
        c.check_async();
      }, py::arg("dev_ptr"), py::arg("count"));
  // RCCL communicator (one process per GPU)
  m.def("Comm", [](py::bytes uid, int rank, int world, int device) {
        std::string s = uid;
        py::gil_scoped_release nogil;
        return std::shared_ptr<Comm>(std::make_shared<RcclComm>(s, rank, world, device));
      },
      py::arg("unique_id"), py::arg("rank"), py::arg("world"), py::arg("device"));
  // Host-staged communicator over a Python callback (torch.distributed gloo):
  // fn(array, op, root) runs the collective in place on a numpy view of the
  // pinned staging buffer (op 0 sum, 1 max, 2 min, -1 broadcast, -2 all-gather)
  m.def("HostComm", [](int rank, int world, py::function fn) {
        // the callable is released with the GIL held, whichever thread drops the comm
        std::shared_ptr<py::function> f(new py::function(std::move(fn)), [](py::function* p) {
          py::gil_scoped_acquire g;
          delete p;
        });
        auto cb = [f, world](void* host, size_t count, ncclDataType_t dt, int op, int root) {
          py::gil_scoped_acquire g;
          std::string fmt;
          switch (dt) {
            case ncclUint8: fmt = "u1"; break;
            case ncclInt32: fmt = "i4"; break;
            case ncclUint32: fmt = "u4"; break;
            case ncclInt64: fmt = "i8"; break;
            case ncclUint64: fmt = "u8"; break;
            case ncclFloat32: fmt = "f4"; break;
            case ncclFloat64: fmt = "f8"; break;
            default: throw std::invalid_argument("HostComm: unsupported dtype");
          }
          const size_t n = op == -2 ? count * size_t(world) : count;
          py::capsule view(host, [](void*) {});   // a view: the callback must not keep it
          py::array arr(py::dtype(fmt), {py::ssize_t(n)}, {py::ssize_t(comm_dtype_size(dt))}, host, view);
          (*f)(arr, op, root);
        };
        return std::shared_ptr<Comm>(std::make_shared<HostComm>(rank, world, cb));
      },
      py::arg("rank"), py::arg("world"), py::arg("fn"));
  // In-process loopback group: N engines on threads of one process (tests)
  py::class_<LoopbackHub, std::shared_ptr<LoopbackHub>>(m, "LoopbackGroup")
      .def(py::init<int>(), py::arg("world"))
      .def("comm", [](std::shared_ptr<LoopbackHub> hub, int rank) {
        if (rank < 0 || rank >= hub->world()) throw std::invalid_argument("rank out of range");
        return std::shared_ptr<Comm>(std::make_shared<LoopbackComm>(hub, rank));
      });

  py::class_<HostBatch, std::shared_ptr<HostBatch>>(m, "HostBatch")
      .def(py::init<int64_t, int64_t>(), py::arg("max_rows"), py::arg("max_bytes"))
      .def_readonly("max_rows", &HostBatch::max_rows)
      .def_readonly("max_bytes", &HostBatch::max_bytes)
      .def_readonly("bytes", &HostBatch::bytes)   // page-locked bytes of the staging buffer
      .def_property_readonly("text", [](py::object self) {
        auto& h = self.cast<HostBatch&>();
        return view<uint8_t>(h.text, {py::ssize_t(h.max_bytes)}, self);
      })
      .def_property_readonly("offsets", [](py::object self) {
        auto& h = self.cast<HostBatch&>();
        return view<int64_t>(h.offsets, {py::ssize_t(h.max_rows + 1)}, self);
      })
      .def_property_readonly("flags", [](py::object self) {
        auto& h = self.cast<HostBatch&>();
        return view<uint8_t>(h.flags, {py::ssize_t(h.max_rows)}, self);
      })
      .def_property_readonly("scalars_flat", [](py::object self) {
        auto& h = self.cast<HostBatch&>();
        return view<int64_t>(h.scalars, {py::ssize_t(5 * h.max_rows)}, self);
      })
      .def_property_readonly("spack_bytes", [](py::object self) {   // the packed scalar columns (tests)
        auto& h = self.cast<HostBatch&>();
        const size_t cap = static_cast<const uint8_t*>(h.base) + h.bytes - h.spack;
        return view<uint8_t>(h.spack, {py::ssize_t(cap)}, self);
      })
      .def("pack_rows", [](HostBatch& h, int64_t n) {
        py::gil_scoped_release nogil;
        return h.pack_rows(n);
      }, py::arg("n"))
      .def_readwrite("scalar_cols", &HostBatch::scalar_cols)
      .def("pack_scalars", [](HostBatch& h, int64_t n) {
        py::gil_scoped_release nogil;
        h.pack_scalars(n);
      }, py::arg("n"))
      .def("load_utf16",
           [](HostBatch& h, py::array_t<uint16_t, py::array::c_style> text,
              py::array_t<int64_t, py::array::c_style> offsets, py::array_t<uint8_t, py::array::c_style> is_rt,
              py::array_t<int64_t, py::array::c_style> scalars, bool copy_text, int threads,
              py::object range) {
             const int64_t n = int64_t(offsets.size()) - 1;
             if (n < 0 || is_rt.size() < n || scalars.size() < 5 * n)
               throw std::invalid_argument("load_utf16: offsets / is_rt / scalars mismatch");
             if (n > 0 && offsets.data()[n] > text.size()) throw std::invalid_argument("offsets exceed text");
             std::vector<int64_t> rng;   // optional [lo 0..4 | hi 0..4] from the receiver
             if (!range.is_none()) {
               auto r = range.cast<py::array_t<int64_t, py::array::c_style | py::array::forcecast>>();
               if (r.size() != 2 * kScalarCols) throw std::invalid_argument("range: 10 int64 (lo[5], hi[5])");
               rng.assign(r.data(), r.data() + 2 * kScalarCols);
             }
             py::gil_scoped_release nogil;
             h.load_utf16(text.data(), offsets.data(), is_rt.data(), scalars.data(), n, copy_text, threads,
                         rng.empty() ? nullptr : rng.data());
             return n > 0 ? 2 * offsets.data()[n] : int64_t(0);
           },
           py::arg("text"), py::arg("offsets"), py::arg("is_rt"), py::arg("scalars"),
           py::arg("copy_text") = true, py::arg("threads") = 0, py::arg("range") = py::none(),
           "Stage a raw UTF-16 batch (row words, offsets, packed scalars; text copied only if "
           "copy_text); returns the text bytes.")
      .def("load_utf8",
           [](HostBatch& h, py::array_t<uint8_t, py::array::c_style> text,
              py::array_t<int64_t, py::array::c_style> offsets, py::array_t<uint8_t, py::array::c_style> is_rt,
              py::array_t<int64_t, py::array::c_style> scalars, bool copy_text, int threads,
              py::object range) {
             const int64_t n = int64_t(offsets.size()) - 1;
             if (n < 0 || is_rt.size() < n || scalars.size() < 5 * n)
               throw std::invalid_argument("load_utf8: offsets / is_rt / scalars mismatch");
             if (n > 0 && offsets.data()[n] > text.size()) throw std::invalid_argument("offsets exceed text");
             std::vector<int64_t> rng;   // optional [lo 0..4 | hi 0..4] from the receiver
             if (!range.is_none()) {
               auto r = range.cast<py::array_t<int64_t, py::array::c_style | py::array::forcecast>>();
               if (r.size() != 2 * kScalarCols) throw std::invalid_argument("range: 10 int64 (lo[5], hi[5])");
               rng.assign(r.data(), r.data() + 2 * kScalarCols);
             }
             py::gil_scoped_release nogil;
             h.load_utf8(text.data(), offsets.data(), is_rt.data(), scalars.data(), n, copy_text, threads,
                         rng.empty() ? nullptr : rng.data());
             return n > 0 ? offsets.data()[n] : int64_t(0);
           },
           py::arg("text"), py::arg("offsets"), py::arg("is_rt"), py::arg("scalars"),
           py::arg("copy_text") = true, py::arg("threads") = 0, py::arg("range") = py::none(),
           "Stage a raw UTF-8 batch (row words, offsets, packed scalars; text copied only if "
           "copy_text); returns the text bytes.")
      .def_readonly("utf16", &HostBatch::utf16)
      .def_readonly("utf8", &HostBatch::utf8)
      .def_readonly("rowpacked_n", &HostBatch::rowpacked_n)
      .def_readonly("range_hits", &HostBatch::range_hits)
      .def_readonly("range_misses", &HostBatch::range_misses)
      .def_readonly("wide_rows", &HostBatch::wide_rows)
      .def_property_readonly("scalar_wire", [](const HostBatch& h) {
        py::dict d;   // wire encoding of the last pack_scalars (tests / diagnostics)
        std::vector<int64_t> off(h.soff, h.soff + kScalarCols + 1), base(h.sbase, h.sbase + kScalarCols);
        d["offsets"] = off;
        d["base"] = base;
        std::vector<int> w(h.sw, h.sw + kScalarCols);
        d["widths"] = w;
        int mask = 0;
        for (int c = 0; c < kScalarCols; ++c) mask |= (h.sw[c] == 64 ? 1 : 0) << c;
        d["wide_mask"] = mask;
        d["rows"] = h.spacked_n;
        return d;
      });

  py::class_<LREngine, std::shared_ptr<LREngine>>(m, "LREngine")
      .def(py::init([](int device, const py::dict& cfg, std::shared_ptr<Comm> comm) {
             LRConfig c = lr_config(cfg);
             py::gil_scoped_release nogil;
             // The destructor stops and joins the prep thread and drains the
             // device: never do that holding the GIL (a training-thread
             // collective on a host communicator takes it in a callback).
             return std::shared_ptr<LREngine>(new LREngine(device, c, comm), [](LREngine* e) {
               if (PyGILState_Check()) {
                 py::gil_scoped_release nogil2;
                 delete e;
               } else {
                 delete e;
               }
             });
           }),
           py::arg("device"), py::arg("config"), py::arg("comm") = nullptr)
      .def("submit",
           [](LREngine& e, const HostBatch& hb, int64_t n, int64_t bytes, int slot, uintptr_t ext_text,
              int64_t now_ms) {
             py::gil_scoped_release nogil;
             e.submit(hb, n, bytes, slot, reinterpret_cast<const uint8_t*>(ext_text), now_ms);
           },
           py::arg("host_batch"), py::arg("n"), py::arg("bytes"), py::arg("slot"), py::arg("ext_text") = 0,
           py::arg("now_ms") = 0)
      .def("process",
           [](LREngine& e, int slot, int64_t now_ms, bool want_pred, int64_t plot_points) {
             BatchResult r;
             int64_t done_ns = 0;
             {
               py::gil_scoped_release nogil;
               r = e.process(slot, now_ms, want_pred, plot_points);
               timespec ts;
               clock_gettime(CLOCK_MONOTONIC, &ts);
               done_ns = int64_t(ts.tv_sec) * 1000000000 + ts.tv_nsec;
             }
             // done_ns (time.monotonic_ns clock): the engine's return, before
             // this thread took the GIL back -- the GIL wait is the difference
             auto d = result_dict(r);
             d["done_ns"] = done_ns;
             return d;
           },
           py::arg("slot"), py::arg("now_ms"), py::arg("want_pred") = false, py::arg("plot_points") = 0)
      .def("discard",
           [](LREngine& e, int slot) {
             py::gil_scoped_release nogil;
             e.discard(slot);
           },
           py::arg("slot"), "forget a submitted batch that will not be processed (one GPU)")
      .def_property_readonly("h2d_bytes", &LREngine::h2d_bytes, "host-to-device bytes submitted so far")
      .def("h2d_timeline", [](LREngine& e) {
             py::gil_scoped_release nogil;
             return e.h2d_timeline();
           },
           "TWTML_H2D_TIMING=1: per submitted batch (queued ms, start ms, end ms, bytes) of its copies")
      .def("h2d_window_mark", &LREngine::h2d_window_mark,
           "TWTML_H2D_TIMING=1: a timing event on the copy stream (the bench's window ends)")
      .def("h2d_window", [](LREngine& e) {
             py::gil_scoped_release nogil;
             return e.h2d_window();
           },
           "the h2d_window_mark events, ms in the h2d_timeline time base")
      .def_property_readonly("raw_slots", &LREngine::raw_slots, "device raw-batch slots")
      .def_property_readonly("lazy_bytes", &LREngine::lazy_bytes,
                             "device bytes the engine allocates on its first tiered batch (sizing)")
      .def("get_weights", [](const LREngine& e) {
        py::array_t<double> out(e.num_weights());
        e.get_weights(out.mutable_data(), e.num_weights());
        return out;
      })
      .def("set_weights", [](LREngine& e, py::array_t<double, py::array::c_style | py::array::forcecast> w) {
        e.set_weights(w.data(), w.size());
      })
      .def("debug_prepared", [](LREngine& e) {
        std::vector<int64_t> counters, cbase;
        std::vector<int32_t> clen8, idx, perm, uniq;
        std::vector<float> y, num;
        e.debug_prepared(counters, clen8, cbase, idx, perm, y, num, uniq);
        py::dict d;
        d["counters"] = py::array_t<int64_t>(py::ssize_t(counters.size()), counters.data());
        d["clen8"] = py::array_t<int32_t>(py::ssize_t(clen8.size()), clen8.data());
        d["cbase"] = py::array_t<int64_t>(py::ssize_t(cbase.size()), cbase.data());
        d["idx"] = py::array_t<int32_t>(py::ssize_t(idx.size()), idx.data());
        d["perm"] = py::array_t<int32_t>(py::ssize_t(perm.size()), perm.data());
        d["y"] = py::array_t<float>(py::ssize_t(y.size()), y.data());
        d["num"] = py::array_t<float>(py::ssize_t(num.size()), num.data());
        d["uniq"] = py::array_t<int32_t>(py::ssize_t(uniq.size()), uniq.data());
        return d;
      })
      .def("debug_merged", [](const LREngine& e) {
        std::vector<int32_t> slot, cnt, clen8d;
        e.debug_merged(slot, cnt, clen8d);
        py::dict d;
        d["slot"] = py::array_t<int32_t>(py::ssize_t(slot.size()), slot.data());
        d["cnt"] = py::array_t<int32_t>(py::ssize_t(cnt.size()), cnt.data());
        d["clen8d"] = py::array_t<int32_t>(py::ssize_t(clen8d.size()), clen8d.data());
        return d;
      })
      .def("debug_hybrid", [](const LREngine& e) {
        std::vector<int32_t> hot_slot, clen8c, cslot;
        std::vector<uint32_t> hot_dense;
        e.debug_hybrid(hot_slot, hot_dense, clen8c, cslot);
        py::dict d;
        d["hot_slot"] = py::array_t<int32_t>(py::ssize_t(hot_slot.size()), hot_slot.data());
        d["hot_dense"] = py::array_t<uint32_t>(py::ssize_t(hot_dense.size()), hot_dense.data());
        d["clen8c"] = py::array_t<int32_t>(py::ssize_t(clen8c.size()), clen8c.data());
        d["cslot"] = py::array_t<int32_t>(py::ssize_t(cslot.size()), cslot.data());
        return d;
      })
      .def("set_step", &LREngine::set_step)
      .def("synchronize", &LREngine::synchronize)
      .def_property_readonly("num_weights", &LREngine::num_weights)
      .def("snapshot_begin",
           [](LREngine& e) {
             py::gil_scoped_release nogil;
             e.snapshot_begin();
           },
           "compact the non-zero weights on the device behind the last batch (non-blocking)")
      .def("snapshot_fetch",
           [](py::object self, bool reuse) {
             LREngine& e = self.cast<LREngine&>();
             int64_t nnz;
             {
               py::gil_scoped_release nogil;
               nnz = e.snapshot_wait();
             }
             if (reuse) {   // views of the engine's host buffers, valid until the next fetch
               int32_t* pi = nullptr;
               double* pv = nullptr;
               {
                 py::gil_scoped_release nogil;
                 e.snapshot_host(nnz, &pi, &pv);
                 e.snapshot_copy(pi, pv);
               }
               py::array_t<int32_t> idx({nnz}, {int64_t(sizeof(int32_t))}, pi, self);
               py::array_t<double> val({nnz}, {int64_t(sizeof(double))}, pv, self);
               return py::make_tuple(idx, val);
             }
             py::array_t<int32_t> idx(nnz);
             py::array_t<double> val(nnz);
             int32_t* pi = idx.mutable_data();
             double* pv = val.mutable_data();
             {
               py::gil_scoped_release nogil;
               e.snapshot_copy(pi, pv);
             }
             return py::make_tuple(idx, val);
           },
           py::arg("reuse") = false,
           "(indices int32, values fp64) of the begun snapshot's non-zero weights, in index order; "
           "reuse=True: views of buffers the engine keeps (valid until the next fetch)")
      .def_property_readonly("device", &LREngine::device);

  bind_kmeans(m);
}
