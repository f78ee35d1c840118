// pybind11 registration of the host-side C++ runtime (tokenizers, safetensors IO, datasets,
// host offload tier, power monitor).  The runtime sources under csrc/runtime/ are plain C++17
// (no torch, no python) so they can also be used from a standalone binary.
#include <torch/extension.h>

namespace py = pybind11;

void register_runtime(py::module_& m) {
  auto rt = m.def_submodule("runtime", "host C++ runtime");
  (void)rt;
}
