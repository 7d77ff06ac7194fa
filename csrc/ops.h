// Host-side launch entry points of the rocfm HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "kernels/deepfm_rows.h"
#include "kernels/batch.h"
#include "kernels/emb_update.h"
#include "kernels/optim.h"
#include "kernels/shard.h"
#include "kernels/merge.h"
#include "kernels/metrics.h"
#include "kernels/p2p.h"
#include "kernels/decode.h"

namespace rocfm {

// deepfm_rows.hip
RowsLds rows_lds_layout(const int* dims, int nl, int F, int K, int bn = 0, int dedup_kp = 0, int rt = 16,
                        bool gr_alias = false, bool fp8 = false);
RowsLds rows_lds_layout_for(const RowsParams& p);  // the layout the launcher uses
void launch_deepfm_rows(RowsParams p, hipStream_t stream);
int deepfm_rows_tile(const RowsParams& p);
int deepfm_rows_split(const RowsParams& p);  // workgroups per row tile the launcher will use (1 or 2)
bool deepfm_rows_static(const RowsParams& p);  // a compile-time-shape instantiation will run

// mlp_wgrad.hip
void launch_mlp_wgrad(WgradParams p, hipStream_t stream);
void launch_dense_apply(DenseApplyParams p, hipStream_t stream);

// emb_update.hip (declared in kernels/emb_update.h)

// step_tail.hip: mlp_wgrad + emb_rows_update as workgroup roles of one launch
void launch_step_tail(WgradParams w, EmbUpdateParams e, hipStream_t stream);
int tail_chunk_entries();  // sorted entries per embedding workgroup of the fused tail
int tail_plan_workgroups(WgradParams w, int n);  // embedding workgroups of the planned tail (emb_plan.hip)

// sort.hip
size_t sort_pairs_temp_bytes(int n, int end_bit);
void sort_pairs_iota(void* temp, size_t temp_bytes, const uint32_t* keys_in, uint32_t* keys_out, uint32_t* vals_out,
                     int n, int end_bit, hipStream_t stream, uint32_t first_val = 0);
// seg_sort.hip: stable LSD radix sort of (key, first_val + index) over nseg segments of seg_len
// keys each, by key bits [0, bits) (every segment sorted on its own; keys keep their other bits)
size_t seg_sort_temp_bytes(int nseg, int seg_len, int bits);
void seg_sort_iota(void* temp, size_t temp_bytes, const uint32_t* keys_in, uint32_t* keys_out, uint32_t* vals_out,
                   int nseg, int seg_len, int bits, hipStream_t stream, uint32_t first_val = 0);
size_t sort_pairs64_temp_bytes(int n, int end_bit);
void sort_pairs64_iota(void* temp, size_t temp_bytes, const uint64_t* keys_in, uint64_t* keys_out, uint32_t* vals_out,
                       int n, int end_bit, hipStream_t stream);
size_t sort_pairs_vals_temp_bytes(int n, int end_bit);
void sort_pairs_vals(void* temp, size_t temp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                     const uint32_t* vals_in, uint32_t* vals_out, int n, int end_bit, hipStream_t stream);

}  // namespace rocfm
