// Native host runtime of mpi_pytorch_amd: data prefetch ring + profiler markers.
#pragma once
#include <torch/extension.h>

namespace mpa_runtime {
void register_bindings(pybind11::module_& m);
}
