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

namespace rocfm {

// Weight-fragment load probe: each of 8 waves loads NF bf16x8 fragments (16 B per lane) of a
// [rows][K] bf16 matrix, either in the MFMA B-operand pattern (lane → row l&15, k-offset 8·(l>>4);
// 16 rows × 64 B per instruction) or from a pre-swizzled copy (1 KiB contiguous per instruction),
// then consumes them (xor-reduce) so the loads cannot be dropped.  Stamps: start / all landed.
template <int NF>
__global__ __launch_bounds__(512) void frag_probe_kernel(const uint16_t* W, int K, int swz, unsigned long long* st,
                                                         uint32_t* sink) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t == 0) st[blockIdx.x * 2] = __builtin_amdgcn_s_memrealtime();
  bf16x8 f[NF];
  if (swz) {
    const bf16x8* base = reinterpret_cast<const bf16x8*>(W) + (size_t)wave * NF * 64 + lane;
#pragma unroll
    for (int u = 0; u < NF; ++u) f[u] = base[u * 64];
  } else {
    // NF fragments: tile j = u / (K/32), k-step = u % (K/32); rows 16·(8j + wave) + (lane & 15)
    const int ks = K / 32;
#pragma unroll
    for (int u = 0; u < NF; ++u) {
      const int j = u / ks, kk = u - j * ks;
      const uint16_t* bp = W + (size_t)((8 * j + wave) * 16 + (lane & 15)) * K + 32 * kk + 8 * (lane >> 4);
      f[u] = *reinterpret_cast<const bf16x8*>(bp);
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int u = 0; u < NF; ++u) x ^= (uint32_t)f[u][0] ^ ((uint32_t)f[u][7] << 16);
  __syncthreads();
  if (t == 0) st[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_memrealtime();
  if (x == 0x12345678u) sink[t] = x;
}

void launch_frag_probe(const uint16_t* W, int K, int swz, int nblocks, unsigned long long* st, uint32_t* sink,
                       hipStream_t stream) {
  hipLaunchKernelGGL(frag_probe_kernel<16>, dim3(nblocks), dim3(512), 0, stream, W, K, swz, st, sink);
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
