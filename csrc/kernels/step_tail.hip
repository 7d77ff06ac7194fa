// The tail of a training step in ONE launch: the MLP weight gradients + fused optimizer
// (wgrad_body, mlp_wgrad.hip) and the embedding-row update (emb_rows_body, emb_update.hip; or the
// planned emb_plan_body, emb_plan.hip) are independent — one reads the transposed activations /
// output gradients, the other the per-lookup gradient rows and the sorted keys — so they run as
// disjoint workgroup roles of one grid (≈60-90 wgrad + the embedding workgroups, all co-resident on
// 256 CUs).  This replaces two serial launches (≈10 + 15 µs) or a second stream (whose fork/join
// inside a HIP graph costs more than it overlaps) with ≈max of the two.  Kernels: step_tail_kern.h.
#include "step_tail_kern.h"

#include <cstdlib>
#include <cstring>

namespace rocfm {

// Sorted entries per unplanned embedding workgroup of the tail.  The side chain's per-chunk run
// ends / run-head counts are cut at the same size (tail_chunk binding).
int tail_chunk_entries() { return kTailEntries; }

// compute units of the current device (the step tail sizes its roles to one dispatch round)
static int tail_cus() {
  static const int n = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus > 0 ? cus : 256;
  }();
  return n;
}
constexpr int kTailMaxKp = 48;  // K <= 47 (notebook shape K = 32 → Kp = 36)

static int tail_wgrad_workgroups(WgradParams& w, int n) {
  // widened weight-gradient tiles when the two roles exceed one dispatch round (wgrad_prepare;
  // ROCFM_WGRAD_TW=1 keeps plain 32 × 32 tiles), laid out for the unplanned chunk count
  const char* tw = std::getenv("ROCFM_WGRAD_TW");
  const bool widen = !(tw && std::strcmp(tw, "1") == 0);
  return wgrad_prepare(w, widen ? (n > 0 ? cdiv(n, kTailEntries) : 0) : -1, tail_cus());
}

// the planned tail's embedding workgroups: at least the unplanned chunk count, and the CUs the
// weight-gradient role leaves free less ROCFM_EMB_PLAN_RESERVE (default 16) for the side chain's
// kernels, which run beside the main graph (with every CU taken, one tail workgroup waited 3.8 µs
// for a CU: profiles/r6_planned_tail.md)
int tail_plan_workgroups(WgradParams w, int n) {
  const int n_wg = tail_wgrad_workgroups(w, n);
  const char* r = std::getenv("ROCFM_EMB_PLAN_RESERVE");
  const int reserve = r ? std::max(0, std::atoi(r)) : 16;
  return std::max(cdiv(n, kTailEntries), tail_cus() - n_wg - reserve);
}

void launch_step_tail(WgradParams w, EmbUpdateParams e, hipStream_t stream) {
  ROCFM_REQUIRE(e.Kp % 4 == 0 && e.Kp <= kTailMaxKp && e.K1 <= e.Kp,
                "step_tail: Kp must be a multiple of 4 and <= 48");
  if (e.id_stride <= 0) e.id_stride = 1;
  TailLaunch l{};
  l.plan = e.plan_items != nullptr && e.mode == 0 && e.n > 0;
  ROCFM_REQUIRE(!l.plan || (e.sorted_contrib && e.n_dev == nullptr && e.max_key == 0 && e.push.W == 0 &&
                            (w.push.W == 0 || w.fuse_opt) && e.plan_nw >= cdiv(e.n, kTailEntries) && e.plan_slots &&
                            e.plan_win && e.plan_head && e.plan_ctr),
                "step_tail: the planned embedding role needs sorted gradient rows, no dedup / sentinels / push, "
                "and its plan buffers");
  l.n_emb = l.plan ? e.plan_nw : (e.n > 0 ? cdiv(e.n, kTailEntries) : 0);
  const int n_wg = tail_wgrad_workgroups(w, e.n);
  l.grid = dim3(l.n_emb + n_wg);
  l.block = dim3(kTailThreads);
  // fused DP push: the export role (mode 2) and the gradient-emitting wgrad role write the slots
  l.push = (e.push.W > 0 && (e.mode == 2 || (e.mode == 1 && e.push_seg > 0))) || (w.push.W > 0 && !w.fuse_opt);
  ROCFM_REQUIRE(!l.push || (e.push.W <= kPushMaxW && w.push.W <= kPushMaxW), "step_tail: push world > 8");
  const int kp4 = e.Kp / 4;
  // (beyond Kp = 48 the 256-entry row staging of the unplanned role + the wgrad reduction tiles
  // exceed 160 KiB of LDS: mlp_wgrad + emb_rows_update run as two launches)
  if (kp4 <= 4)
    launch_tail_group_a(kp4, w, e, l, stream);
  else if (kp4 <= 8)
    launch_tail_group_b(kp4, w, e, l, stream);
  else
    launch_tail_group_c(kp4, w, e, l, stream);
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
