// pybind11 bindings of the host-side native runtime (_twtml_host).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <charconv>
#include <cmath>
#include <stdexcept>
#include <string>
#include <vector>

#include "featurize_cpu.h"
#include "http_post.h"
#include "synth.h"
#include "unicode_lower.h"
#include "wire.h"

namespace py = pybind11;
using namespace twtml;

template <typename T>
using Arr = py::array_t<T, py::array::c_style | py::array::forcecast>;

template <typename T>
static T* mut_ptr(py::array& a, size_t need, const char* what) {
  if (!(a.flags() & py::array::c_style)) throw std::invalid_argument(std::string(what) + " not contiguous");
  if (a.itemsize() != sizeof(T)) throw std::invalid_argument(std::string(what) + ": wrong dtype");
  if (size_t(a.size()) < need) throw std::invalid_argument(std::string(what) + ": too small");
  if (!a.writeable()) throw std::invalid_argument(std::string(what) + ": read-only");
  return static_cast<T*>(a.mutable_data());
}

static SynthParams params_from(const py::dict& d) {
  SynthParams p;
#define GET(name, type) if (d.contains(#name)) p.name = d[#name].cast<type>();
  GET(seed, uint64_t) GET(retweet_fraction, double) GET(rt_lo, int64_t) GET(rt_hi, int64_t)
  GET(rt_base, double) GET(rt_slope, double) GET(rt_noise, double) GET(rt_tail, double)
  GET(min_len, int32_t) GET(max_len, int32_t) GET(unicode_fraction, double)
  GET(special_fraction, double) GET(now_ms, int64_t) GET(max_age_ms, int64_t)
  GET(vocab, int32_t) GET(vocab_size, int32_t)
#undef GET
  return p;
}

template <typename T>
static py::array_t<T> to_numpy(std::vector<T>&& v) {
  auto* heap = new std::vector<T>(std::move(v));
  py::capsule owner(heap, [](void* p) { delete static_cast<std::vector<T>*>(p); });
  return py::array_t<T>({heap->size()}, {sizeof(T)}, heap->data(), owner);
}

PYBIND11_MODULE(_twtml_host, m) {
  m.doc() = "twtml host runtime: synthetic tweet source, unicode lowering, CPU featurizer";

  m.def("synth_max_units", [](const py::dict& d, size_t n) { return synth_max_units(params_from(d), n); });

  m.def("synth_generate_into",
        [](const py::dict& d, uint64_t start, size_t n, py::array text, py::array offsets,
           py::array is_rt, py::array scalars, int nthreads) {
          SynthParams p = params_from(d);
          uint16_t* t = mut_ptr<uint16_t>(text, 0, "text");
          int64_t* o = mut_ptr<int64_t>(offsets, n + 1, "offsets");
          uint8_t* r = mut_ptr<uint8_t>(is_rt, n, "is_rt");
          int64_t* s = mut_ptr<int64_t>(scalars, 5 * n, "scalars");
          int64_t res;
          {
            py::gil_scoped_release nogil;
            res = synth_generate(p, start, n, t, size_t(text.size()), o, r, s, nthreads);
          }
          return res;
        },
        py::arg("params"), py::arg("start"), py::arg("n"), py::arg("text"), py::arg("offsets"),
        py::arg("is_rt"), py::arg("scalars"), py::arg("nthreads") = 0,
        "Generate rows [start, start+n) into caller buffers; returns units written or -needed.");

  m.def("count_special_rows", [](Arr<uint16_t> text, Arr<int64_t> offsets) {
    const size_t n = size_t(offsets.size()) - 1;
    return count_special_rows(text.data(), offsets.data(), n);
  });

  m.def("prelower_special_rows", [](Arr<uint16_t> text, Arr<int64_t> offsets) {
    const size_t n = size_t(offsets.size()) - 1;
    std::vector<uint16_t> ot;
    std::vector<int64_t> oo;
    size_t changed;
    {
      py::gil_scoped_release nogil;
      changed = prelower_special_rows(text.data(), offsets.data(), n, ot, oo);
    }
    return py::make_tuple(to_numpy(std::move(ot)), to_numpy(std::move(oo)), changed);
  });

  m.def("lower_row", [](Arr<uint16_t> units) {
    std::vector<uint16_t> out;
    lower_full(units.data(), size_t(units.size()), out);
    return to_numpy(std::move(out));
  });

  m.def("row_needs_special", [](Arr<uint16_t> units) {
    return row_needs_special(units.data(), size_t(units.size()));
  });

  m.def("featurize_rows",
        [](Arr<uint16_t> text, Arr<int64_t> offsets, Arr<int64_t> rows, int64_t F,
           const std::string& hash, int nthreads) {
          const int kind = hash == "java" ? 0 : hash == "murmur3" ? 1 : -1;
          if (kind < 0) throw std::invalid_argument("hash must be 'java' or 'murmur3'");
          if (F <= 0) throw std::invalid_argument("F must be positive");
          const int64_t nr = offsets.size() - 1;
          if (nr < 0) throw std::invalid_argument("offsets must have n + 1 entries");
          // every row's units must lie in the text (a batch whose UTF-16 copy
          // was dropped for its UTF-8 bytes has an empty text: RawBatch.ensure_text)
          if (nr > 0 && (offsets.data()[0] < 0 || offsets.data()[nr] > int64_t(text.size())))
            throw std::invalid_argument("featurize_rows: offsets exceed the text (" +
                                        std::to_string(offsets.data()[nr]) + " > " +
                                        std::to_string(text.size()) + " units)");
          for (int64_t i = 0; i < nr; ++i)
            if (offsets.data()[i + 1] < offsets.data()[i]) throw std::invalid_argument("offsets not ascending");
          for (py::ssize_t i = 0; i < rows.size(); ++i)
            if (rows.data()[i] < 0 || rows.data()[i] >= nr) throw std::out_of_range("row id");
          std::vector<int64_t> indptr, indices;
          {
            py::gil_scoped_release nogil;
            featurize_rows_cpu(text.data(), offsets.data(), rows.data(), size_t(rows.size()), F,
                               kind, indptr, indices, nthreads);
          }
          return py::make_tuple(to_numpy(std::move(indptr)), to_numpy(std::move(indices)));
        },
        py::arg("text"), py::arg("offsets"), py::arg("rows"), py::arg("F"),
        py::arg("hash") = "java", py::arg("nthreads") = 0);

  m.def("term_index", [](Arr<uint16_t> units, int64_t F, const std::string& hash) {
    return term_index(units.data(), int(units.size()), F, hash == "java" ? 0 : 1);
  });

  m.def("wire_bound", &wire_bound, py::arg("units"), py::arg("rows"));
  m.def("utf8_bound", &utf8_bound, py::arg("units"));
  // JSON array text of a float64 vector (shortest round-trip digits, like
  // Python's repr; non-finite values as null), built with the GIL released:
  // the Lightning plot's series are tens of thousands of numbers per append,
  // and json.dumps holds the GIL for milliseconds (report/lightning.py).
  // report/http.py: a whole POST with the GIL released (http_post.cpp)
  py::register_exception<HttpError>(m, "HttpError", PyExc_ConnectionError);
  m.def("http_post", [](const std::string& host, int port, const std::string& path, const py::bytes& body,
                        const std::string& headers, double timeout_s) {
    std::string b = body;
    HttpResponse r;
    {
      py::gil_scoped_release nogil;
      r = http_post(host, port, path, b, headers, timeout_s);
    }
    return py::make_tuple(r.status, py::bytes(r.body));
  }, py::arg("host"), py::arg("port"), py::arg("path"), py::arg("body"), py::arg("headers") = "",
     py::arg("timeout") = 5.0);
  m.def("json_floats", [](Arr<double> v) {
    std::string out;
    {
      py::gil_scoped_release nogil;
      const double* x = v.data();
      const size_t n = size_t(v.size());
      out.reserve(n * 12 + 2);
      out.push_back('[');
      char buf[32];
      for (size_t i = 0; i < n; ++i) {
        if (i) out.push_back(',');
        if (!std::isfinite(x[i])) {
          out += "null";
          continue;
        }
        const auto r = std::to_chars(buf, buf + sizeof(buf), x[i]);
        out.append(buf, r.ptr);
      }
      out.push_back(']');
    }
    return py::bytes(out);
  }, py::arg("values"));
  m.def("utf8_encode",
        [](Arr<uint16_t> text, Arr<int64_t> offsets, int threads) {
          const int64_t n = int64_t(offsets.size()) - 1;
          if (n < 0) throw std::invalid_argument("offsets must have n + 1 entries");
          if (n > 0 && offsets.data()[n] > int64_t(text.size())) throw std::invalid_argument("offsets exceed text");
          const int64_t units = n > 0 ? offsets.data()[n] : 0;
          py::array_t<uint8_t> out(py::ssize_t(utf8_bound(units)));
          py::array_t<int64_t> oo(py::ssize_t(n + 1));
          int64_t total;
          {
            py::gil_scoped_release nogil;
            total = utf8_encode(text.data(), offsets.data(), n, out.mutable_data(), int64_t(out.size()),
                                oo.mutable_data(), threads);
          }
          return py::make_tuple(out[py::slice(0, total, 1)], oo);
        },
        py::arg("text"), py::arg("offsets"), py::arg("threads") = 0,
        "UTF-16 rows -> (UTF-8 bytes, byte offsets [n+1]); astral pairs as 4 bytes, lone surrogates as 3.");
  m.def("wire_pack",
        [](Arr<uint16_t> text, Arr<int64_t> offsets, Arr<uint8_t> is_rt, py::array out,
           py::array out_offsets, py::array flags, int nthreads) {
          const int64_t n = int64_t(offsets.size()) - 1;
          if (n < 0 || is_rt.size() < n) throw std::invalid_argument("offsets / is_rt mismatch");
          if (n > 0 && offsets.data()[n] > text.size()) throw std::invalid_argument("offsets exceed text");
          uint8_t* o = mut_ptr<uint8_t>(out, 0, "out");
          int64_t* oo = mut_ptr<int64_t>(out_offsets, size_t(n) + 1, "out_offsets");
          uint8_t* f = mut_ptr<uint8_t>(flags, size_t(n), "flags");
          py::gil_scoped_release nogil;
          return wire_pack(text.data(), offsets.data(), is_rt.data(), n, o, int64_t(out.size()), oo, f,
                           nthreads);
        },
        py::arg("text"), py::arg("offsets"), py::arg("is_rt"), py::arg("out"), py::arg("out_offsets"),
        py::arg("flags"), py::arg("nthreads") = 0,
        "Pack a UTF-16 batch into the narrow/cesu/wide wire format; returns bytes written.");
  m.def("wire_unpack", [](Arr<uint8_t> wire, Arr<int64_t> woff, Arr<uint8_t> flags) {
    const int64_t n = int64_t(woff.size()) - 1;
    if (n < 0 || flags.size() < n) throw std::invalid_argument("woff / flags mismatch");
    const int64_t units = wire_units(wire.data(), woff.data(), flags.data(), n);
    py::array_t<uint16_t> text(units);
    py::array_t<int64_t> offsets(n + 1);
    py::array_t<uint8_t> is_rt(n);
    wire_unpack(wire.data(), woff.data(), flags.data(), n, text.mutable_data(), offsets.mutable_data(),
                is_rt.mutable_data());
    return py::make_tuple(text, offsets, is_rt);
  });
}
