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
  // device-side id guard (ROCFM_CHECK_IDS): ids outside [0, max_id) set *bad_ids and are fetched
  // as row 0, so no kernel indexes outside the table; the host raises at its next check()
  int32_t* bad_ids;  // nullable (guard off)
  uint32_t max_id;
};

void launch_fetch_batch(const FetchParams& p, hipStream_t stream);

// Batch preparation for a multi-step graph (S steps per replay): copies the next graph's S batches
// into static slots in one launch, writes each lookup's composite sort key (slot << id_bits | id),
// and the per-step global_step / Adam lr_t arrays.  Counters are double-buffered by graph parity:
// batches start at *cur_src + advance (advance = the size of the graph running concurrently);
// *cur_dst / *step_dst receive that start for the next preparation.
struct FetchMultiParams {
  const int32_t* ids_pool;
  const float* vals_pool;
  const float* labels_pool;
  long long pool_batches;
  int B, F, Bp;
  int S;        // batches to prepare
  int advance;  // steps of the graph this preparation runs beside
  const int64_t* cur_src;
  int64_t* cur_dst;
  const int64_t* step_src;
  int64_t* step_dst;
  int32_t* ids;     // [S][Bp][F]
  float* vals;      // [S][Bp][F]
  float* labels;    // [S][Bp]
  uint32_t* keys;   // [S][B*F] composite sort keys (nullable): step k's keys are k << id_bits | id
  int id_bits;
  unsigned long long* keys64;  // [S][B*F] (nullable; instead of keys): k << id_bits | id as 64-bit
                               // keys — vocabularies too wide for S << id_bits to fit 32 bits
  int shard_W;      // > 0: keys are owner-major row-shard keys (id % W)·Vs + id / W (shard.hip)
  uint32_t shard_Vs;
  const uint32_t* shard_hot;  // replicated ids (ascending; shard_key in shard.h), nullable
  int shard_nhot;
  int64_t* steps;   // [S] global_step of each prepared step
  float* lrt;       // [S] lr_t of each prepared step
  float lr, beta1, beta2;
  int opt_type;
  int32_t* bad_ids;  // nullable: device-side id guard, as in FetchParams
  uint32_t max_id;
};

void launch_fetch_multi(const FetchMultiParams& p, hipStream_t stream);

// After the multi-batch sort: each lookup's position in its batch's sorted order (the row kernel
// writes its gradient row there, so the embedding update reads rows contiguously) and, per
// batch and `chunk`-entry workgroup chunk, the end of the run holding the chunk's last entry.
struct SortAuxParams {
  const uint32_t* skeys;  // [S·n] sorted (batch << id_bits | id)
  const uint32_t* svals;  // [S·n] global lookup index (batch · n + lookup)
  int n, S, chunk;
  int32_t* pos;           // [S·n] pos[batch · n + lookup] = sorted position within the batch
  int32_t* chunk_end;     // [S][ceil(n / chunk)] (nullable)
  // 64-bit key sorts: skeys64 are the sorted keys; their ids (low id_bits) are written to
  // skeys_out as plain 32-bit per-batch keys for the consumers (skeys is then unused)
  const unsigned long long* skeys64;
  uint32_t* skeys_out;
  int id_bits;
  // nullable: [S][ceil(n / chunk)] run heads per chunk (the sorted DP export's output bases,
  // EmbUpdateParams::chunk_heads); chunk must be a multiple of 64 and at most 1024
  int32_t* chunk_heads;
};
void launch_sort_aux(const SortAuxParams& p, hipStream_t stream);

}  // namespace rocfm
