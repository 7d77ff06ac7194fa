// Multi-source row-gradient merge (merge.hip): direct addressing, or an open-addressing hash for
// vocabularies whose W × V position maps would not fit a memory budget.
//
// W source lists (one per rank) each hold UNIQUE keys with one gradient row per key — the DP
// all-gather of every rank's (id, Σ grad) export, or an owner's per-source requests in row-shard
// mode.  Instead of radix-sorting the W·cap gathered keys, two kernels use HBM-resident position
// maps (W × Vmap int32, 32 MB for a 1M vocabulary at W=8; kept at −1 between steps):
//   merge_scatter : pos[r][key] = j ; rep[key] = min r holding key
//   merge_apply   : the representative entry (r == rep[key]) sums the rows of key over r..W−1 in
//                   rank order (deterministic, no float atomics), applies lazy L2 + the row
//                   optimizer (or writes a dense gradient row), and restores pos/rep.
// merge_search_apply with maps bound (pos / rep, or the hash table) applies through the maps a
// merge_scatter launch filled instead of searching — measured faster from W = 4 on
// (tools/bench_merge.py: W=8, 60k entries: search 20.6 µs, scatter + apply 13.7 µs; W=1: 3.9 vs 8.9).
// Search mode (merge_search_apply; every source list ascending within its count, pads last — the
// row-shard request lists and the sorted DP export): ONE launch and no maps at all.  Each entry
// binary-searches its key in the other W−1 lists (all searches advance together, one round of
// L2-resident loads per halving); an entry found in a lower rank's list is not the representative,
// the representative sums the rows it found in rank order and applies the optimizer as above.  At
// W = 1 no search is made.  The MLP optimizer (dense_apply over the gathered rank segments) rides
// as extra workgroups of the same launch.
// Hash mode (hash_slots > 0; O(W·cap) memory whatever the vocabulary — the 1B-row tables): a
// linear-probing table of hash_slots ≥ 2·W·cap slots replaces the maps.  Every word carries the
// step's tag T = global_step + 1 in its high half, so slots of earlier steps read as empty and
// nothing is ever cleared (clearing while other threads still probe through a slot would break
// their chains):
//   hkeys[slot] = T<<32 | row                      (claimed by 64-bit CAS)
//   hrep[slot]  = T<<32 | (0xFFFFFFFF − r)         (atomicMax → the lowest rank holding row)
//   hpos[slot·W + r] = T<<32 | j
#pragma once
#include "../common.h"
#include "optim.h"
#include "push.h"

namespace rocfm {

struct MergeParams {
  // source r: keys at keys + r*key_stride, rows at rows + r*row_stride ([cap][Kp] f32),
  // count at counts[r*count_stride] (nullable: lists are padded with key 0xFFFFFFFF instead)
  const uint32_t* keys;
  long long key_stride;
  const float* rows;
  long long row_stride;
  const int32_t* counts;
  long long count_stride;
  int W, cap, Kp, K1;
  uint32_t key_div;   // table row = key / key_div (1: DP; W: row-shard owner, global id → local row)
  uint32_t Vmap;      // rows of the table / maps
  int32_t* pos;       // [W][Vmap], -1 = empty
  int32_t* rep;       // [Vmap], W = none
  // apply
  float* emb;  // [Vmap][Kp]
  float* s0;
  float* s1;
  float l2;
  float grad_scale;
  OptParams opt;
  const int64_t* step;
  int mode;           // 0: lazy L2 + optimizer on the rows; 1: dense_grad[row] = Σ · grad_scale
  float* dense_grad;  // mode 1
  int32_t* overflow;  // nullable: sticky flag, set when a source's count exceeds cap
  uint32_t* touched;  // mode 1 (nullable): touched[row] = step + 1 (EmbDenseParams::touched)
  // hash mode (hash_slots > 0, a power of two ≥ 2·W·cap; pos/rep/Vmap maps unused)
  int hash_slots;
  unsigned long long* hkeys;  // [hash_slots], zero-initialised once
  unsigned long long* hrep;   // [hash_slots]
  unsigned long long* hpos;   // [hash_slots][W]
  int tbl_bf16;               // 1: emb holds bf16 rows (stochastic-rounded updates, common.h)
  int use_maps;               // merge_search_apply: 1 = apply through the maps a merge_scatter filled
  // range mode (merge_range_apply): every source list ascending with a bucket directory —
  // dirs + r·dir_stride holds nb + 1 offsets, dir[b] = first position of source r whose key is
  // ≥ b·bucket_div (the sorted DP export writes it beside its keys)
  const int32_t* dirs;
  long long dir_stride;
  int nb;
  uint32_t bucket_div;
  // owner-sharded DP (emb_shard replicate_table, mode 0): every updated row is also appended to a
  // broadcast list — slot = atomicAdd(bc_count) — as (global id = row · bc_mul + bc_add, f32 row);
  // the X5 all-gather carries the lists to every rank's full table replica (row_scatter)
  int32_t* bc_count;  // nullable: no broadcast
  uint32_t* bc_keys;
  float* bc_rows;     // [bc_cap][Kp]
  int bc_cap;
  uint32_t bc_mul, bc_add;
  PushTarget bc_push;  // W > 0: the lists go straight into every rank's X5 slot (keys at +4, rows at
                       // +4 + bc_cap floats); the X5 launch then carries only bc_count + the hand-off
};

// Every rank's full table replica takes the rows the owners broadcast (X5): source r's list at
// recv + r·slot_stride = [count int32 | pad 3 | keys cap | rows cap·Kp].
struct RowScatterParams {
  const float* recv;
  long long slot_stride;  // floats
  int W, cap, Kp;
  float* table;           // [V][Kp] f32
  uint32_t rows;          // V (keys ≥ V are skipped)
};
void launch_row_scatter(const RowScatterParams& p, hipStream_t stream);

void launch_merge_scatter(const MergeParams& p, hipStream_t stream);
void launch_merge_apply(const MergeParams& p, hipStream_t stream);
void launch_merge_init(const MergeParams& p, hipStream_t stream);  // pos = −1, rep = W
struct DenseApplyParams;
void launch_merge_scatter_dense(const MergeParams& p, const DenseApplyParams& d, hipStream_t stream);
// Row-shard hot-row replication: every rank applies the same update to its replica of the
// replicated rows from the X4 bucket's hot part (per rank: [H·Kp gradient sums | H touched flags]).
struct HotApplyParams {
  float* rows;            // [H][Kp] replica (the received-rows buffer behind the W owner segments)
  float* s0;              // [H][Kp] optimizer slots (nullable)
  float* s1;
  const float* grads;     // segment r at grads + r·seg_stride: [H·Kp | H]
  int nseg;               // 1: already summed (all-reduce); W: rank segments summed in rank order
  long long seg_stride;   // floats
  float* zero;            // nullable: this rank's bucket part, cleared after it is read
  int H, Kp, K1;
  float l2, grad_scale;
  OptParams opt;
  const int64_t* step;
  int dense;              // 1 (exact): every replicated row is updated (g = λ·θ when untouched)
};

// Range mode: one workgroup per key bucket stages the W sources' entries of its bucket (keys and
// gradient rows, located through the directories: one round trip) in LDS, matches equal keys
// there (LDS binary searches instead of the search mode's global ones), and the representative
// (lowest rank holding the key) sums the rows in rank order and applies the optimizer — the same
// arithmetic as the search / maps merges.  Buckets larger than the LDS stage fall back to global
// binary searches inside their bucket.  d (nullable): the MLP optimizer as extra workgroups.
void launch_merge_range_apply(const MergeParams& p, const DenseApplyParams* d, hipStream_t stream);
int merge_range_lds_entries(int Kp);

// ---- plan-ahead merge (merge_plan.hip) ------------------------------------------------------------
// Side chain, per graph of S steps: this rank's unique ids per step (uniq_keys), then — after the
// exchange of every rank's lists — the union of the W lists of each step with every id's position in
// every rank's list (plan_build).  Main chain, per step: merge_plan_apply.
struct PlanParams {
  int S, W, cap;
  // uniq_keys: this rank's sorted lookup keys [S][n] with their per-chunk run-head counts [S][nch]
  const uint32_t* skeys;
  const int32_t* chunk_heads;
  int n, chunk, nch;
  int id_shift;             // > 0: the sorted keys are composite (k << id_shift | id): ids = key − (k << id_shift)
  uint32_t* ukeys;          // step k's unique ids at ukeys + k·ukey_stride (ascending, ≤ cap)
  long long ukey_stride;
  int32_t* ucount;          // step k's count at ucount[k·ucount_stride]
  long long ucount_stride;
  int32_t* overflow;        // nullable sticky flag: more than cap unique ids
  // plan_build: rank r's list of step k at gkeys + r·gk_stride + k·gkey_step, its count at
  // gcounts + r·gc_stride + k·gcount_step (the gathered send buffers: gk_stride == gc_stride)
  const uint32_t* gkeys;
  const int32_t* gcounts;
  long long gk_stride, gc_stride, gkey_step, gcount_step;
  uint32_t pad_key;         // > every id (the vocabulary size): pads sort last
  uint32_t* pkeys;          // [S][W·cap] sort input
  uint32_t* skeys_sorted;   // [S][W·cap]
  uint32_t* svals_sorted;   // [S][W·cap] global index k·W·cap + r·cap + j
  int32_t* tile_counts;     // [S][⌈W·cap / 1024⌉]
  uint32_t* plan_rows;      // [S][W·cap] union ids (ascending)
  int32_t* plan_pos;        // [S][W·cap][W] position of the id in rank r's list, −1 if absent
  int32_t* plan_count;      // [S] union sizes
};
struct PlanStep {            // one step's plan (the slices of PlanParams' outputs for step k)
  const uint32_t* rows;
  const int32_t* pos;
  const int32_t* count;
};
void launch_uniq_keys(const PlanParams& p, hipStream_t stream);
size_t plan_sort_temp_bytes(int S, int W, int cap, int bits);
int plan_tile_ints(int S, int W, int cap);
void launch_plan_build(const PlanParams& p, void* temp, size_t temp_bytes, int bits, hipStream_t stream);
// the step's merge from its plan (the gathered rows: MergeParams rows / row_stride / Kp / W / cap;
// the optimizer / dense-gradient outputs as in the other merges); d: the MLP optimizer as extra
// workgroups (nullable)
void launch_merge_plan_apply(const MergeParams& p, const PlanStep& ps, const DenseApplyParams* d, hipStream_t stream);

// search mode; d (nullable): the MLP optimizer launched as extra workgroups; sv (nullable): a
// row-shard serve (shard.h) as further workgroups; hot (nullable): the replicated rows' update
struct ShardServeParams;
void launch_merge_search_apply(const MergeParams& p, const DenseApplyParams* d, const ShardServeParams* sv,
                               const HotApplyParams* hot, hipStream_t stream);

}  // namespace rocfm
