// Toolchain probe: verifies that gfx950 code objects built by this image's hipcc load under
// the HIP runtime that PyTorch ships, and reports the device's architecture/CU count.
#include "../common.h"

namespace rocfm {

__global__ void probe_kernel(float* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    // wave64 sanity: lane id and wave size.
    out[i] = (float)(__lane_id() + 64 * (int)(warpSize == 64));
  }
}

void launch_probe(float* out, int n, hipStream_t stream) {
  hipLaunchKernelGGL(probe_kernel, dim3(cdiv(n, 256)), dim3(256), 0, stream, out, n);
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
