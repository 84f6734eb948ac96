// Torch bindings for the MobileNet-SSD inference kernels (vision.hip). Filled in as the
// kernels land; registering an empty set keeps the module layout stable.
#include <torch/extension.h>

void vcx_register_vision(pybind11::module& m) { (void)m; }
