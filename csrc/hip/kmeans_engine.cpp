#include "kmeans_engine.h"

namespace twtml {
void bind_kmeans(pybind11::module_& m) { (void)m; }
}  // namespace twtml
