// Parameter block of the batch-fetch kernel (batch.hip).
#pragma once
#include "../common.h"

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
};

void launch_fetch_batch(const FetchParams& p, hipStream_t stream);

}  // namespace rocfm
