// Parameter block of the batch-fetch kernel (batch.hip).
#pragma once
#include "../common.h"
#include "optim.h"

namespace rocfm {

struct FetchParams {
  const int32_t* ids_pool;
  const float* vals_pool;
  const float* labels_pool;
  long long pool_batches;
  int B, F;
  const int64_t* cur_src;
  int64_t* cur_dst;  // nullable
  int advance;
  const int64_t* step_src;
  int64_t* step_dst;  // nullable
  int step_advance;
  int32_t* ids;
  float* vals;
  float* labels;
  float* lrt_dst;  // nullable: lr_t for the step published in step_dst (Adam bias correction)
  float lr, beta1, beta2;
  int opt_type;
};

void launch_fetch_batch(const FetchParams& p, hipStream_t stream);

}  // namespace rocfm
