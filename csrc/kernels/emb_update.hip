// Embedding-table gradient aggregation + optimizer (the reference's UnsortedSegmentSum + ApplyAdam
// on fm_w / fm_v).
//
// Input: the B·F lookups sorted by row id (sort.hip: radix sort of (id, lookup index)), and the
// per-lookup gradient rows written by deepfm_rows.hip ([x·de | g·x], Kp floats each).
// Each workgroup takes 256 consecutive sorted entries and owns every run (= unique id) whose
// FIRST entry falls in its chunk; runs that continue past the chunk are followed to their end.
// Short runs go to 16-lane groups (one lane per column, 64-B coalesced row reads); long runs —
// the hot rows: at B=1024 on the bundled data 65 ids take 68 % of all lookups, max multiplicity
// 1026 — are summed by the whole workgroup and combined through LDS.  No float atomics: every sum
// runs in sorted (id, lookup) order, so results are bitwise reproducible.
//
// mode 0 (sparse): optimizer on the touched rows with lazy L2 (g += λ·θ for touched rows only)
// mode 1 (exact) : write Σ grads into a dense grad table; emb_dense_update_kernel then applies
//                  λ·θ + optimizer to EVERY row, as TF does for the dense gradient (Q1)
// mode 2 (export): emit (id, Σ grad row) compacted, for cross-rank exchange (DP / row-shard)
#include "emb_body.h"

namespace rocfm {

template <int KP4, bool BT, bool PUSH>
__global__ __launch_bounds__(kEmbChunk) void emb_rows_update_kernel(const EmbUpdateParams p) {
  emb_rows_body<KP4, kEmbChunk, BT, PUSH>(p, blockIdx.x);
}

template <int KP4>
static void launch_rows_update_t(const EmbUpdateParams& p, hipStream_t stream) {
  const dim3 grid(cdiv(p.n, kEmbChunk)), block(kEmbChunk);
  if (p.push.W > 0 && (p.mode == 2 || (p.mode == 1 && p.push_seg > 0))) {  // producer push (push.h)
    ROCFM_REQUIRE(p.push.W <= kPushMaxW, "emb_update: push world > 8");
    if (p.tbl_bf16)
      hipLaunchKernelGGL((emb_rows_update_kernel<KP4, true, true>), grid, block, 0, stream, p);
    else
      hipLaunchKernelGGL((emb_rows_update_kernel<KP4, false, true>), grid, block, 0, stream, p);
  } else if (p.tbl_bf16) {
    hipLaunchKernelGGL((emb_rows_update_kernel<KP4, true, false>), grid, block, 0, stream, p);
  } else {
    hipLaunchKernelGGL((emb_rows_update_kernel<KP4, false, false>), grid, block, 0, stream, p);
  }
}

void launch_emb_rows_update(EmbUpdateParams p, hipStream_t stream) {
  ROCFM_REQUIRE(p.Kp % 4 == 0 && p.Kp <= 64 && p.K1 <= p.Kp, "emb_update: Kp must be a multiple of 4 and <= 64");
  if (p.id_stride <= 0) p.id_stride = 1;
  if (p.n <= 0) return;
  // the side chain's precomputed run ends are cut at the FUSED tail's chunk (step_tail.hip); this
  // launch's workgroups take kEmbChunk entries and find their last run's end themselves
  p.chunk_end = nullptr;
  switch (p.Kp / 4) {
#define ROCFM_KP4(N) \
  case N:            \
    launch_rows_update_t<N>(p, stream); \
    break;
    ROCFM_KP4(1) ROCFM_KP4(2) ROCFM_KP4(3) ROCFM_KP4(4) ROCFM_KP4(5) ROCFM_KP4(6) ROCFM_KP4(7) ROCFM_KP4(8)
    ROCFM_KP4(9) ROCFM_KP4(10) ROCFM_KP4(11) ROCFM_KP4(12) ROCFM_KP4(13) ROCFM_KP4(14) ROCFM_KP4(15) ROCFM_KP4(16)
#undef ROCFM_KP4
    default:
      throw std::invalid_argument("emb_update: unsupported Kp");
  }
  ROCFM_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// Exact mode: dense update of EVERY row: g = G + λ·θ (full-table l2_loss gradient, PS:277-278),
// optimizer, and G reset to 0 for the next step.  float4-vectorised; pad columns are skipped.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void emb_dense_update_kernel(const EmbDenseParams p) {
  const OptStep st = opt_step(p.opt, p.step ? *p.step : 0);
  const bool bf = p.tbl_bf16 != 0;
  const uint32_t stp = p.step ? (uint32_t)*p.step : 0u;
  float4* G = reinterpret_cast<float4*>(p.dense_grad);
  float4* A = reinterpret_cast<float4*>(p.s0);
  float4* Bv = reinterpret_cast<float4*>(p.s1);
  const int kp4 = p.Kp >> 2;
  const uint32_t tag = (uint32_t)(p.step ? *p.step : 0) + 1u;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < p.n4; i += (long long)gridDim.x * 256) {
    const int c0 = (int)(i % kp4) * 4;
    const bool has_g = p.touched == nullptr || p.touched[i / kp4] == tag;
    float4 w = tbl_load4_rt(p.emb, i, bf), g = make_float4(0, 0, 0, 0);
    if (has_g) g = G[i];
    float4 a = A ? A[i] : make_float4(0, 0, 0, 0), b = Bv ? Bv[i] : make_float4(0, 0, 0, 0);
    float* wp = &w.x;
    float* gp = &g.x;
    float* ap = &a.x;
    float* bp = &b.x;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (c0 + u < p.K1) opt_apply(p.opt, st, wp[u], l2_grad(gp[u] * p.grad_scale, p.l2, wp[u]), ap[u], bp[u]);
    tbl_store4_rt(p.emb, i, w, stp, bf);
    if (has_g) G[i] = make_float4(0, 0, 0, 0);
    if (A) A[i] = a;
    if (Bv) Bv[i] = b;
  }
}

void launch_emb_dense_update(EmbDenseParams p, hipStream_t stream) {
  const int grid = (int)std::min<long long>((p.n4 + 255) / 256, 4096);
  if (grid <= 0) return;
  hipLaunchKernelGGL(emb_dense_update_kernel, dim3(grid), dim3(256), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// Σ θ² over the real columns of the table (the l2_loss terms, only evaluated when logged).
// Writes one partial per workgroup; the host sums the partials (deterministic).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void emb_sumsq_kernel(const float* emb, long long n4, int Kp, int K1,
                                                        float* partial, int bf) {
  __shared__ float s[4];
  const int kp4 = Kp >> 2;
  float acc = 0.f;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const int c0 = (int)(i % kp4) * 4;
    const float4 w = tbl_load4_rt(emb, i, bf != 0);
    acc += (c0 + 0 < K1 ? w.x * w.x : 0.f) + (c0 + 1 < K1 ? w.y * w.y : 0.f) + (c0 + 2 < K1 ? w.z * w.z : 0.f) +
           (c0 + 3 < K1 ? w.w * w.w : 0.f);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

void launch_emb_sumsq(const float* emb, long long n4, int Kp, int K1, float* partial, int nblocks,
                      hipStream_t stream, int tbl_bf16) {
  hipLaunchKernelGGL(emb_sumsq_kernel, dim3(nblocks), dim3(256), 0, stream, emb, n4, Kp, K1, partial, tbl_bf16);
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
