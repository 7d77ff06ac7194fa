// MLP weight gradients (+ fused optimizer) and dense-parameter maintenance kernels.
//
// dW_l = h_lᵀ · dz_{l+1} reduces over the batch, the one cross-example reduction of the MLP.
// The row kernel (deepfm_rows.hip) leaves h and dz transposed ([feature][batch], bf16) in the
// fragment-swizzled order of common.h act_swz, so every operand load of a wave is one contiguous
// 1 KiB block:
//   A[i][b] = actT[i][b], B[b][o] = dzT[o][b]  →  v_mfma_f32_32x32x16_bf16, f32 accumulate.
// One workgroup owns one 32×32 tile of one layer's dW (no atomics, no split-K seam): its 4 waves
// take a quarter of the batch each and combine through LDS; the tile's epilogue then applies the
// optimizer to the f32 master weights and re-emits both bf16 copies (Wᵀ for the forward, W for
// the backward) — single-GPU steps need no separate optimizer launch.  In data-parallel mode the
// epilogue writes the gradient instead, RCCL all-reduces it, and dense_apply_kernel finishes.
// Bias and output-layer gradients (Σ_b dz, hᵀ·g, Σ g) run in extra workgroups of the same grid.
#include "wgrad_body.h"

namespace rocfm {

template <bool PUSH>
__global__ __launch_bounds__(kWgThreads) void mlp_wgrad_kernel(const WgradParams p) {
  wgrad_body<PUSH>(p, blockIdx.x);
}

void launch_mlp_wgrad(WgradParams p, hipStream_t stream) {
  const int grid = wgrad_prepare(p);
  if (p.push.W > 0 && !p.fuse_opt) {  // fused DP push: gradients straight into the receive slots
    ROCFM_REQUIRE(p.push.W <= kPushMaxW, "mlp_wgrad: push world > 8");
    hipLaunchKernelGGL(mlp_wgrad_kernel<true>, dim3(grid), dim3(kWgThreads), 0, stream, p);
  } else {
    hipLaunchKernelGGL(mlp_wgrad_kernel<false>, dim3(grid), dim3(kWgThreads), 0, stream, p);
  }
  ROCFM_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// dense_apply_kernel: elementwise optimizer over the flat dense buffer (after the DP all-reduce),
// or (apply == 0) just refresh the bf16 weight copies from the f32 masters (init / restore).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dense_apply_kernel(const DenseApplyParams p) {
  dense_apply_body(p, blockIdx.x, gridDim.x);
}

void launch_dense_apply(DenseApplyParams p, hipStream_t stream) {
  const int grid = std::min(cdiv(p.n, 256), 2048);
  if (grid <= 0) return;
  hipLaunchKernelGGL(dense_apply_kernel, dim3(grid), dim3(256), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
