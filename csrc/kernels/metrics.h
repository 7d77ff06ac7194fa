// Evaluation-metric kernels (metrics.hip): the reference's tf.metrics.auc (PS:282, HVD:271 —
// 200 thresholds, confusion counts accumulated over eval batches) as one histogram pass per batch.
#pragma once
#include "../common.h"

namespace rocfm {

struct AucHistParams {
  const float* prob;    // [n] predictions
  const float* labels;  // [n] 0/1 labels (> 0.5 = positive)
  const float* loss;    // [n] per-example loss (nullable) — summed into loss_sum
  int n;
  const float* thr;     // [nt] ascending thresholds (TF: -1e-7, i/(nt-1) for i=1..nt-2, 1+1e-7), float32
  int nt;               // <= 1024
  unsigned long long* hist;  // [2][nt+1]: count of (label, k) with k = #thresholds strictly below the prediction
  double* loss_sum;     // [2]: Σ loss, count (nullable)
};

void launch_auc_hist(const AucHistParams& p, hipStream_t stream);

}  // namespace rocfm
