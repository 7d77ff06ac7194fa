// The tail of a training step in ONE launch (step_tail.hip): kernel templates and the per-row-width
// launchers.  The instantiations are spread over three translation units by float4 columns per row
// (step_tail_k{a,b,c}.hip: KP4 1-4, 5-8, 9-12) so they compile in parallel.
#pragma once
#include "../ops.h"
#include "emb_body.h"
#include "emb_plan_body.h"
#include "wgrad_body.h"

namespace rocfm {

constexpr int kTailThreads = 512;
constexpr int kTailEntries = 256;  // sorted entries per unplanned embedding workgroup (2 threads each)
static_assert(kTailThreads == kWgThreads, "wgrad role uses 512-thread workgroups");

template <int KP4, bool BT, bool PUSH>
__global__ __launch_bounds__(kTailThreads) void step_tail_kernel(const WgradParams w, const EmbUpdateParams e,
                                                                 const int n_emb) {
  const int bid = blockIdx.x;
  unsigned long long* stp = bid < n_emb ? e.stamps : w.stamps;  // (diagnostics: entry / exit stamps 15 / 14)
  ROCFM_STAMP(stp, 15);
  if (bid < n_emb)
    emb_rows_body<KP4, kTailThreads, BT, PUSH, kTailEntries>(e, bid);  // the longer role first: dispatched first
  else
    wgrad_body<PUSH>(w, bid - n_emb);
  ROCFM_STAMP(stp, 14);
}

// planned embedding role (emb_plan_body.h): plan item bid of the side chain's work plan
template <int KP4, bool BT>
__global__ __launch_bounds__(kTailThreads) void step_tail_plan_kernel(const WgradParams w, const EmbUpdateParams e,
                                                                      const int n_emb) {
  const int bid = blockIdx.x;
  unsigned long long* stp = bid < n_emb ? e.stamps : w.stamps;  // (diagnostics: entry / exit stamps 15 / 14)
  ROCFM_STAMP(stp, 15);
  ROCFM_STAMP_HWID(stp, 13);
  if (bid < n_emb)
    emb_plan_body<KP4, BT>(e, bid);
  else
    wgrad_body<false>(w, bid - n_emb);
  ROCFM_STAMP(stp, 14);
}

struct TailLaunch {
  dim3 grid, block;
  int n_emb;
  bool plan, push;
};

template <int KP4>
void launch_tail_kp4(const WgradParams& w, const EmbUpdateParams& e, const TailLaunch& l, hipStream_t s) {
  if (l.plan) {
    if (e.tbl_bf16)
      hipLaunchKernelGGL((step_tail_plan_kernel<KP4, true>), l.grid, l.block, 0, s, w, e, l.n_emb);
    else
      hipLaunchKernelGGL((step_tail_plan_kernel<KP4, false>), l.grid, l.block, 0, s, w, e, l.n_emb);
  } else if (l.push) {
    if (e.tbl_bf16)
      hipLaunchKernelGGL((step_tail_kernel<KP4, true, true>), l.grid, l.block, 0, s, w, e, l.n_emb);
    else
      hipLaunchKernelGGL((step_tail_kernel<KP4, false, true>), l.grid, l.block, 0, s, w, e, l.n_emb);
  } else {
    if (e.tbl_bf16)
      hipLaunchKernelGGL((step_tail_kernel<KP4, true, false>), l.grid, l.block, 0, s, w, e, l.n_emb);
    else
      hipLaunchKernelGGL((step_tail_kernel<KP4, false, false>), l.grid, l.block, 0, s, w, e, l.n_emb);
  }
}

// one per translation unit: KP4 in [lo, lo + 4)
void launch_tail_group_a(int kp4, const WgradParams& w, const EmbUpdateParams& e, const TailLaunch& l, hipStream_t s);
void launch_tail_group_b(int kp4, const WgradParams& w, const EmbUpdateParams& e, const TailLaunch& l, hipStream_t s);
void launch_tail_group_c(int kp4, const WgradParams& w, const EmbUpdateParams& e, const TailLaunch& l, hipStream_t s);

}  // namespace rocfm
