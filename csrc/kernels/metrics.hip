// Streaming-AUC histogram: for every prediction p, k = #{thresholds < p} (binary search over the
// thresholds staged in LDS, float32 compares exactly as TF's `predictions > thresholds`); the
// (label, k) counts go to an LDS histogram, then one 64-bit global add per non-empty bucket.
// TP(thr_i) = #positives with k > i, FP likewise (suffix sums on the host), so accumulating the
// histogram over batches (and all-reducing it over ranks) reproduces tf.metrics.auc's counts.
#include "metrics.h"

#include <algorithm>

namespace rocfm {
namespace {

constexpr int kAucThreads = 256;
constexpr int kMaxThr = 1024;

__global__ __launch_bounds__(kAucThreads) void auc_hist_kernel(AucHistParams p) {
  __shared__ float s_thr[kMaxThr];
  __shared__ unsigned int s_hist[2 * (kMaxThr + 1)];
  __shared__ float s_loss[kAucThreads / kWave];
  const int t = threadIdx.x;
  const int nb = 2 * (p.nt + 1);
  for (int i = t; i < p.nt; i += kAucThreads) s_thr[i] = p.thr[i];
  for (int i = t; i < nb; i += kAucThreads) s_hist[i] = 0u;
  __syncthreads();
  float lsum = 0.f;
  for (int i = blockIdx.x * kAucThreads + t; i < p.n; i += gridDim.x * kAucThreads) {
    const float x = p.prob[i];
    int lo = 0, hi = p.nt;  // first index with thr >= x  ==  #thresholds strictly below x
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s_thr[mid] < x) lo = mid + 1; else hi = mid;
    }
    const int pos = p.labels[i] > 0.5f ? 1 : 0;
    atomicAdd(&s_hist[pos * (p.nt + 1) + lo], 1u);
    if (p.loss) lsum += p.loss[i];
  }
  if (p.loss_sum) {
    lsum = wave_sum(lsum);
    if ((t & 63) == 0) s_loss[t >> 6] = lsum;
  }
  __syncthreads();
  for (int i = t; i < nb; i += kAucThreads)
    if (s_hist[i]) atomicAdd(&p.hist[i], (unsigned long long)s_hist[i]);
  if (p.loss_sum && t == 0) {
    float s = 0.f;
    for (int w = 0; w < kAucThreads / kWave; ++w) s += s_loss[w];
    atomicAdd(&p.loss_sum[0], (double)s);
    if (blockIdx.x == 0) atomicAdd(&p.loss_sum[1], (double)p.n);  // example count, once per batch
  }
}

}  // namespace

void launch_auc_hist(const AucHistParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.nt >= 2 && p.nt <= kMaxThr, "auc_hist: 2 <= num_thresholds <= 1024");
  if (p.n <= 0) return;
  const int blocks = std::min(cdiv(p.n, kAucThreads), 1024);
  hipLaunchKernelGGL(auc_hist_kernel, dim3(blocks), dim3(kAucThreads), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
