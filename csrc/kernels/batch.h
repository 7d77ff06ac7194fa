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
                               // keys — vocabularies too wide for S << id_bits to fit 32 bits, sorted
                               // by rocPRIM (ROCFM_SORT_LIB=rocprim A/B only)
  int plain_keys;   // 1: keys holds the plain id keys of each batch (no k << id_bits): the segmented
                    // sort (seg_sort.hip) orders every batch on its own id bits, so the 100M-1B-row
                    // vocabularies need no 64-bit composite keys
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
  const int32_t* halt;  // nullable: the input pipeline's sticky error word (decode.hip); non-zero →
                        // every prepared step carries kHaltStepBit (optim.h: its updates are skipped)
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

// Per-tile dedup of the sorted lookups (the row kernel pre-reduces duplicate ids inside each of its
// workgroups' row tiles).  In a batch's sorted order the lookups of one id are ascending in position,
// so those of one (id, row tile) pair — a "group" — are contiguous.  Every lookup gets its group's
// index in the compacted (one entry per group) sorted list: pos[lookup] = c for the group's first
// lookup, ~c for the others, and nxt[lookup] = the next lookup of its group (in-batch index, -1 at
// the end); the compacted keys, their count and the embedding update's per-chunk run ends / run
// heads are rebuilt over the compacted list.  Deterministic (no atomics).
struct DedupParams {
  const uint32_t* skeys;  // [S·n] sorted keys (per-batch segments; equal key ⇔ equal id in a segment)
  const uint32_t* svals;  // [S·n] lookup index: batch_base + b·F + f, batch_base = k·n (val_base_step = n)
  int n, S, F, rt;        // lookups per batch, batches, fields, examples per row-kernel workgroup
  int val_base_step;      // n for multi-batch sorts (global indices), 0 for one batch's local indices
  int32_t* pos;           // [S·n] by lookup index
  int32_t* nxt;           // [S·n] by lookup index
  uint32_t* ckeys;        // [S·n] compacted keys (segment k at k·n)
  int32_t* count;         // [S] compacted entries per batch
  int32_t* bcount;        // scratch [S][ceil(n / 1024)]
  int chunk;              // entries per embedding-update workgroup
  int32_t* chunk_end;     // [S][ceil(n / chunk)] (nullable) end of each chunk's last run (compacted)
  int32_t* chunk_heads;   // [S][ceil(n / chunk)] (nullable) run heads per compacted chunk
};
void launch_dedup(const DedupParams& p, hipStream_t stream);
int dedup_scratch_ints(int n, int S);

}  // namespace rocfm
