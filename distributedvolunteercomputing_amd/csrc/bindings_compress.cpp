// Torch bindings for the gradient-compression kernels (compress.hip).
#include <torch/extension.h>

void vcx_register_compress(pybind11::module& m) { (void)m; }
