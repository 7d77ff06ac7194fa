// pybind11 bindings for the rocfm HIP kernels (module rocfm._rocfm_hip).
//
// The module deliberately does not include torch headers: every op takes raw device pointers
// (tensor.data_ptr()) and the HIP stream handle (torch.cuda.current_stream().cuda_stream) so
// that (a) it builds in seconds with hipcc, (b) kernels launch on PyTorch's current stream and
// are captured by torch.cuda.CUDAGraph, and (c) shape/dtype checks live in one place, the
// Python wrappers in rocfm/ops/.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <hip/hip_runtime.h>
#include "ops.h"
#include "kernels/wgrad_body.h"  // wgrad_prepare (the wgrad_plan binding)

namespace py = pybind11;
using namespace rocfm;

static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
template <typename T>
static T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}

PYBIND11_MODULE(_rocfm_hip, m) {
  m.doc() = "rocfm HIP kernels for MI355X (gfx950)";
  m.def("arch", []() {
    int dev = 0;
    ROCFM_HIP_CHECK(hipGetDevice(&dev));
    hipDeviceProp_t prop;
    ROCFM_HIP_CHECK(hipGetDeviceProperties(&prop, dev));
    return py::make_tuple(std::string(prop.gcnArchName), prop.multiProcessorCount,
                          (long long)prop.totalGlobalMem);
  });
#include "bindings.inc"
}
