// Streaming k-means engine (K8-K11) -- bindings entry point.
#pragma once
#include <pybind11/pybind11.h>

namespace twtml {
void bind_kmeans(pybind11::module_& m);
}  // namespace twtml
