// The tail of a training step in ONE launch: the MLP weight gradients + fused optimizer
// (wgrad_body, mlp_wgrad.hip) and the embedding-row update (emb_rows_body, emb_update.hip) are
// independent — one reads the transposed activations / output gradients, the other the per-lookup
// gradient rows and the sorted keys — so they run as disjoint workgroup roles of one grid
// (≈70 wgrad + ⌈B·F/512⌉ embedding workgroups, all co-resident on 256 CUs).  This replaces two
// serial launches (≈10 + 15 µs) or a second stream (whose fork/join inside a HIP graph costs more
// than it overlaps) with ≈max of the two.
#include "../ops.h"
#include "emb_body.h"
#include "wgrad_body.h"

#include <cstdlib>
#include <cstring>

namespace rocfm {

constexpr int kTailThreads = 512;

// Sorted entries per embedding workgroup of the tail (ROCFM_TAIL_CHUNK = 256 | 512).  The side
// chain's per-chunk run ends / run-head counts are cut at the same size (tail_chunk binding).
int tail_chunk_entries() {
  static const int n = [] {
    const char* v = std::getenv("ROCFM_TAIL_CHUNK");
    const int x = v ? std::atoi(v) : kTailChunkDefault;
    return (x == 256 || x == 512) ? x : kTailChunkDefault;
  }();
  return n;
}
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
static_assert(kTailThreads == kWgThreads, "wgrad role uses 512-thread workgroups");

template <int KP4, bool BT, bool PUSH, int kE, bool PRE = false>
__global__ __launch_bounds__(kTailThreads) void step_tail_kernel(const WgradParams w, const EmbUpdateParams e,
                                                                 const int n_emb) {
  const int bid = blockIdx.x;
  if (bid < n_emb)
    emb_rows_body<KP4, kTailThreads, BT, PUSH, kE, PRE>(e, bid);  // the longer role first: its workgroups dispatch first
  else
    wgrad_body<PUSH>(w, bid - n_emb);
}

// the embedding role's table-load prologue (emb_body.h PRE): apply mode with the side chain's
// run-head keys, sorted gradient rows, and both optimizer slots or an f32 table (the missing
// slots' loads then read the table as a stand-in)
static bool tail_pre(const EmbUpdateParams& e) {
  return e.mode == 0 && e.hkeys != nullptr && e.rows > 0 && e.sorted_contrib && e.n_dev == nullptr &&
         (!e.tbl_bf16 || (e.s0 && e.s1));
}

template <int KP4, bool PUSH, int kE>
static void launch_tail_e(const WgradParams& w, const EmbUpdateParams& e, int n_emb, dim3 grid, dim3 block,
                          hipStream_t stream) {
  if constexpr (!PUSH) {
    if (tail_pre(e)) {
      if (e.tbl_bf16)
        hipLaunchKernelGGL((step_tail_kernel<KP4, true, false, kE, true>), grid, block, 0, stream, w, e, n_emb);
      else
        hipLaunchKernelGGL((step_tail_kernel<KP4, false, false, kE, true>), grid, block, 0, stream, w, e, n_emb);
      return;
    }
  }
  if (e.tbl_bf16)
    hipLaunchKernelGGL((step_tail_kernel<KP4, true, PUSH, kE>), grid, block, 0, stream, w, e, n_emb);
  else
    hipLaunchKernelGGL((step_tail_kernel<KP4, false, PUSH, kE>), grid, block, 0, stream, w, e, n_emb);
}

template <int KP4, bool PUSH>
static void launch_tail_t(const WgradParams& w, const EmbUpdateParams& e, int n_emb, dim3 grid, dim3 block,
                          hipStream_t stream) {
  if (tail_chunk_entries() == 256)
    launch_tail_e<KP4, PUSH, 256>(w, e, n_emb, grid, block, stream);
  else
    launch_tail_e<KP4, PUSH, 512>(w, e, n_emb, grid, block, stream);
}

void launch_step_tail(WgradParams w, EmbUpdateParams e, hipStream_t stream) {
  ROCFM_REQUIRE(e.Kp % 4 == 0 && e.Kp <= kTailMaxKp && e.K1 <= e.Kp,
                "step_tail: Kp must be a multiple of 4 and <= 48");
  if (e.id_stride <= 0) e.id_stride = 1;
  const int n_emb = e.n > 0 ? cdiv(e.n, tail_chunk_entries()) : 0;
  // widened weight-gradient tiles when the two roles exceed one dispatch round (wgrad_prepare;
  // ROCFM_WGRAD_TW=1 keeps plain 32 × 32 tiles)
  const char* tw = std::getenv("ROCFM_WGRAD_TW");
  const bool widen = !(tw && std::strcmp(tw, "1") == 0);
  const int n_wg = wgrad_prepare(w, widen ? n_emb : -1, tail_cus());
  const dim3 grid(n_emb + n_wg), block(kTailThreads);
  // fused DP push: the export role (mode 2) and the gradient-emitting wgrad role write the slots
  const bool push = (e.push.W > 0 && (e.mode == 2 || (e.mode == 1 && e.push_seg > 0))) || (w.push.W > 0 && !w.fuse_opt);
  ROCFM_REQUIRE(!push || (e.push.W <= kPushMaxW && w.push.W <= kPushMaxW), "step_tail: push world > 8");
  switch (e.Kp / 4) {
#define ROCFM_KP4(N)                                                   \
  case N:                                                              \
    if (push)                                                          \
      launch_tail_t<N, true>(w, e, n_emb, grid, block, stream);        \
    else                                                               \
      launch_tail_t<N, false>(w, e, n_emb, grid, block, stream);       \
    break;
    ROCFM_KP4(1) ROCFM_KP4(2) ROCFM_KP4(3) ROCFM_KP4(4) ROCFM_KP4(5) ROCFM_KP4(6) ROCFM_KP4(7) ROCFM_KP4(8)
    ROCFM_KP4(9) ROCFM_KP4(10) ROCFM_KP4(11) ROCFM_KP4(12)
#undef ROCFM_KP4
    default:  // the 512-entry row staging of larger rows (8 KiB per float4 column) + the wgrad
              // reduction tiles exceed 160 KiB of LDS beyond Kp = 48
      throw std::invalid_argument("step_tail: Kp > 48 unsupported (use mlp_wgrad + emb_rows_update)");
  }
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
