// Parameter blocks of the embedding-update kernels (emb_update.hip).
#pragma once
#include "../common.h"
#include "optim.h"
#include "push.h"

namespace rocfm {

struct EmbUpdateParams {
  const uint32_t* skeys;  // [n] sorted ids
  const uint32_t* svals;  // [n] lookup index into contrib
  int n;
  const float* contrib;  // [*][Kp]
  int K1;                // real columns: K + 1 (fm_v row + fm_w)
  int Kp;                // row stride (multiple of 4, <= 64)
  float* emb;            // [V][Kp]
  float* s0;
  float* s1;
  float l2;
  float grad_scale;
  OptParams opt;
  const int64_t* step;
  int mode;
  float* dense_grad;   // mode 1: [V][Kp]
  uint32_t* out_keys;  // mode 2
  float* out_rows;     // mode 2: [cap][Kp]
  int* out_count;      // mode 2
  uint32_t id_offset;  // subtracted from keys before indexing emb (multi-batch sort segment prefix)
  int id_stride;       // keys are mapped to local rows by (key - id_offset) / id_stride
  uint32_t max_key;    // runs with key >= max_key are skipped (padding sentinels); 0 = no limit
  int contrib_seg;     // if > 0: lookup j lives at contrib + (j/seg)*seg_stride + (j%seg)*Kp
  long long contrib_seg_stride;  // floats between segments (per-rank blocks of a gathered buffer)
  int out_cap;         // mode 2: capacity of out_keys/out_rows (rows past it are dropped, count kept)
  unsigned long long* stamps;  // diagnostic (nullable)
  uint32_t val_base;   // subtracted from svals (a batch's segment of a multi-batch sort)
  int sorted_contrib;  // 1: contrib rows are already in sorted order (row i ↔ sorted entry i; svals unused)
  const int32_t* chunk_end;  // nullable: per workgroup chunk, end of the run holding its last entry
  uint32_t* touched;   // mode 1 (nullable): touched[row] = step + 1 for every row whose gradient it wrote
  // mode 2 (nullable): run heads per workgroup chunk (sort_aux, side chain).  The export then
  // places chunk c's rows at Σ heads of chunks < c — the list comes out in sorted key order and is
  // deterministic — and workgroup 0 stores the total count (no atomics; out_count need not be zeroed)
  const int32_t* chunk_heads;
  int nch;  // chunks of this batch (entries of chunk_heads)
  // mode 1 (nullable): rows >= hot_base are replicated rows (row-shard hot replication); their sums
  // go to hot_out[(row − hot_base)·Kp] and a 1 to hot_out[n_hot·Kp + row − hot_base] (the X4 bucket)
  float* hot_out;
  uint32_t hot_base;
  int n_hot;
  int tbl_bf16;  // 1: emb holds bf16 rows (stochastic-rounded updates, common.h)
  // mode 2 with push.W > 0: keys / rows are stored into the W receive slots (push.h) at these
  // float offsets instead of out_keys / out_rows; the count still goes to out_count (local).
  // mode 1 with push.W > 0 and push_seg > 0 (row-shard X3): gradient row rr goes to destination
  // rr / push_seg, row rr % push_seg of its slot, instead of dense_grad[rr]
  PushTarget push;
  int push_off_keys, push_off_rows;
  int push_seg;
  // with push: also store each result locally — row-shard X3: every row gradient (dense_grad[rr]);
  // DP export (mode 2): keys / rows / directory (out_keys, out_rows, out_dir).  The shadow
  // exchange (rocfm.parallel.validate) sends that local copy through RCCL and compares it bitwise
  // with what the producers pushed into the peers' slots
  int push_mirror;
  // nullable: the entry count is this device word (per-tile dedup: the compacted list's length,
  // written by the side chain); n is then the maximum and sizes the grid
  const int32_t* n_dev;
  // mode 2 sorted export (chunk_heads): bucket directory of the exported keys (merge range mode):
  // dir[b] = first output slot whose row id is ≥ b·dir_div, b = 0..dir_nb (dir[dir_nb] = count);
  // out_dir (local) or, with push, every receive slot at push_off_dir
  int32_t* out_dir;
  int dir_nb;
  uint32_t dir_div;
  int push_off_dir;
  // apply mode, planned step tail (emb_plan.hip; nullable): this batch's work plan from the side
  // chain — plan_nw items {es, ee, lead slot, tail slot} (one per embedding workgroup) and the
  // split-run slots {key, first non-head window, last window, pieces}.  The shared combine state:
  // plan_win [n/64 + 1][Kp] window pieces, plan_head [plan_nw][Kp] head-item folds, plan_ctr
  // [plan_nw] arrival counters (zero between launches: the last arrival resets its slot)
  const int4* plan_items;
  const int4* plan_slots;
  // nullable: per item [kPlanSlab] words — [0] its run-head count, [1 ..] the heads' keys in order —
  // so the table / Adam-slot rows of its complete runs are loaded at entry, under the scan
  const uint32_t* plan_hslab;
  int plan_nw;
  float* plan_win;
  float* plan_head;
  uint32_t* plan_ctr;
};

// The step tail's embedding work plan (emb_plan.hip), built on the side chain for every batch of
// the next multi-step graph.  The sorted lookups are cut into plan_nw contiguous items of equal cost
// (an entry costs 1, a run head `beta` more: its table / Adam-slot round trip), at run heads or —
// inside runs longer than `lsplit` — at 64-entry window boundaries.  A run cut that way is "split":
// every item holding a part of it publishes its window pieces (the head item its fold of them) and
// the last item to arrive sums them in window order and applies the optimizer, so the result is the
// same left-to-right fold of window pieces that the unplanned update computes (emb_body.h).
struct EmbPlanParams {
  const uint32_t* skeys;  // [S][n] sorted keys, one segment per batch
  int n, S, nw;           // lookups per batch, batches, items per batch (= tail embedding workgroups)
  int beta, lsplit;       // cost of a run head (in entries); shortest run that may be split
  int32_t* runs;          // scratch [S][n + 1]
  int4* items;            // [S][nw]
  int4* slots;            // [S][nw]
  uint32_t* hslab;        // nullable: [S][nw][kPlanSlab] run-head count and keys per item
};
void launch_emb_plan(const EmbPlanParams& p, hipStream_t stream);
// the planned tail's bounds (emb_plan_body.h): run heads and window pieces per item
constexpr int kPlanHcap = 264;
constexpr int kPlanPcap = kPlanHcap + 64;
constexpr int kPlanSlab = 272;     // words per item of the head-key slab (≥ kPlanHcap + 1)
constexpr int kPlanMaxNw = 1024;   // items per batch the plan kernel's LDS head ranges hold

struct EmbDenseParams {
  float* emb;
  float* s0;
  float* s1;
  float* dense_grad;
  long long n4;  // number of float4 in the table
  int Kp, K1;
  float l2;
  float grad_scale;
  OptParams opt;
  const int64_t* step;
  // nullable: touched[row] == step + 1 marks the rows whose dense_grad holds this step's gradient
  // (written by the mode-1 scatter / merge).  Other rows read no gradient row (g = λ·θ only) and
  // their dense_grad stays zero — the update never reads or clears the whole gradient table.
  const uint32_t* touched;
  int tbl_bf16;  // 1: emb holds bf16 rows
};

void launch_emb_rows_update(EmbUpdateParams p, hipStream_t stream);
void launch_emb_dense_update(EmbDenseParams p, hipStream_t stream);
void launch_emb_sumsq(const float* emb, long long n4, int Kp, int K1, float* partial, int nblocks, hipStream_t stream,
                      int tbl_bf16 = 0);

}  // namespace rocfm
