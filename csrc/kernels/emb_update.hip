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
#include "emb_update.h"

namespace rocfm {

namespace {

constexpr int kChunk = 256;
constexpr int kLongRun = 48;

__device__ __forceinline__ void finish_row(const EmbUpdateParams& p, const OptStep& st, uint32_t key, int col,
                                           float g, int out_slot) {
  if (col >= p.K1) return;
  g *= p.grad_scale;
  if (p.mode == 2) {
    p.out_rows[(size_t)out_slot * p.Kp + col] = g;
    return;
  }
  const size_t row = (size_t)((key - (uint32_t)p.id_offset) / (uint32_t)p.id_stride);
  const size_t idx = row * p.Kp + col;
  if (p.mode == 1) {
    p.dense_grad[idx] = g;
    return;
  }
  float w = p.emb[idx];
  float a = p.s0 ? p.s0[idx] : 0.f, b = p.s1 ? p.s1[idx] : 0.f;
  opt_apply(p.opt, st, w, g + p.l2 * w, a, b);
  p.emb[idx] = w;
  if (p.s0) p.s0[idx] = a;
  if (p.s1) p.s1[idx] = b;
}

}  // namespace

__global__ __launch_bounds__(kChunk) void emb_rows_update_kernel(const EmbUpdateParams p) {
  __shared__ int s_head[kChunk + 1];
  __shared__ int s_wcnt[4];
  __shared__ int s_nh, s_last_end, s_out_base;
  __shared__ float s_part[16][64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c0 = blockIdx.x * kChunk;
  const int i = c0 + t;
  const OptStep st = opt_step(p.opt, p.step ? *p.step : 0);

  // 1. run heads inside the chunk, compacted in order
  uint32_t key = 0;
  bool head = false;
  if (i < p.n) {
    key = p.skeys[i];
    head = (i == 0) || (p.skeys[i - 1] != key);
  }
  const unsigned long long m = __ballot(head);
  const int before = __popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) s_wcnt[wave] = __popcll(m);
  __syncthreads();
  int base = 0;
  for (int w = 0; w < wave; ++w) base += s_wcnt[w];
  if (head) s_head[base + before] = i;
  if (t == 0) s_nh = s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
  __syncthreads();
  const int nh = s_nh;
  if (nh == 0) return;

  // 2. end of the last run (may extend beyond the chunk): wave 0 scans forward
  if (wave == 0) {
    const int last = s_head[nh - 1];
    const uint32_t lk = p.skeys[last];
    int pos = min(c0 + kChunk, p.n);
    int end = p.n;
    while (pos < p.n) {
      const int j = pos + lane;
      const bool diff = (j < p.n) && (p.skeys[j] != lk);
      const unsigned long long dm = __ballot(diff || j >= p.n);
      if (dm) {
        end = pos + __ffsll((long long)dm) - 1;
        if (end > p.n) end = p.n;
        break;
      }
      pos += 64;
    }
    if (lane == 0) {
      s_last_end = end;
      if (p.mode == 2) s_out_base = atomicAdd(p.out_count, nh);
    }
  }
  __syncthreads();
  s_head[nh] = s_last_end;
  __syncthreads();

  // 3. short runs: one 16-lane group each, lane = column (Kp <= 64 → 4 columns per lane)
  const int grp = t >> 4, q = t & 15;
  for (int r = grp; r < nh; r += 16) {
    const int s = s_head[r], e = s_head[r + 1];
    if (e - s > kLongRun) continue;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (int k = s; k < e; ++k) {
      const float* src = p.contrib + (size_t)p.svals[k] * p.Kp;
      a0 += (q < p.Kp) ? src[q] : 0.f;
      a1 += (q + 16 < p.Kp) ? src[q + 16] : 0.f;
      a2 += (q + 32 < p.Kp) ? src[q + 32] : 0.f;
      a3 += (q + 48 < p.Kp) ? src[q + 48] : 0.f;
    }
    const uint32_t kk = p.skeys[s];
    const int slot = (p.mode == 2) ? s_out_base + r : 0;
    if (p.mode == 2 && q == 0) p.out_keys[slot] = kk;
    finish_row(p, st, kk, q, a0, slot);
    finish_row(p, st, kk, q + 16, a1, slot);
    finish_row(p, st, kk, q + 32, a2, slot);
    finish_row(p, st, kk, q + 48, a3, slot);
  }

  // 4. long runs: the whole workgroup, 16 groups stride the run, combine through LDS
  for (int r = 0; r < nh; ++r) {
    const int s = s_head[r], e = s_head[r + 1];
    if (e - s <= kLongRun) continue;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (int k = s + grp; k < e; k += 16) {
      const float* src = p.contrib + (size_t)p.svals[k] * p.Kp;
      a0 += (q < p.Kp) ? src[q] : 0.f;
      a1 += (q + 16 < p.Kp) ? src[q + 16] : 0.f;
      a2 += (q + 32 < p.Kp) ? src[q + 32] : 0.f;
      a3 += (q + 48 < p.Kp) ? src[q + 48] : 0.f;
    }
    __syncthreads();
    s_part[grp][q] = a0;
    s_part[grp][q + 16] = a1;
    s_part[grp][q + 32] = a2;
    s_part[grp][q + 48] = a3;
    __syncthreads();
    if (t < 64) {
      float tot = 0.f;
      for (int g2 = 0; g2 < 16; ++g2) tot += s_part[g2][t];
      const uint32_t kk = p.skeys[s];
      const int slot = (p.mode == 2) ? s_out_base + r : 0;
      if (p.mode == 2 && t == 0) p.out_keys[slot] = kk;
      finish_row(p, st, kk, t, tot, slot);
    }
  }
}

void launch_emb_rows_update(EmbUpdateParams p, hipStream_t stream) {
  ROCFM_REQUIRE(p.Kp % 4 == 0 && p.Kp <= 64 && p.K1 <= p.Kp, "emb_update: Kp must be a multiple of 4 and <= 64");
  if (p.id_stride <= 0) p.id_stride = 1;
  if (p.n <= 0) return;
  hipLaunchKernelGGL(emb_rows_update_kernel, dim3(cdiv(p.n, kChunk)), dim3(kChunk), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// Exact mode: dense update of EVERY row: g = G + λ·θ (full-table l2_loss gradient, PS:277-278),
// optimizer, and G reset to 0 for the next step.  float4-vectorised; pad columns are skipped.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void emb_dense_update_kernel(const EmbDenseParams p) {
  const OptStep st = opt_step(p.opt, p.step ? *p.step : 0);
  float4* E = reinterpret_cast<float4*>(p.emb);
  float4* G = reinterpret_cast<float4*>(p.dense_grad);
  float4* A = reinterpret_cast<float4*>(p.s0);
  float4* Bv = reinterpret_cast<float4*>(p.s1);
  const int kp4 = p.Kp >> 2;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < p.n4; i += (long long)gridDim.x * 256) {
    const int c0 = (int)(i % kp4) * 4;
    float4 w = E[i], g = G[i];
    float4 a = A ? A[i] : make_float4(0, 0, 0, 0), b = Bv ? Bv[i] : make_float4(0, 0, 0, 0);
    float* wp = &w.x;
    float* gp = &g.x;
    float* ap = &a.x;
    float* bp = &b.x;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (c0 + u < p.K1) opt_apply(p.opt, st, wp[u], gp[u] + p.l2 * wp[u], ap[u], bp[u]);
    E[i] = w;
    G[i] = make_float4(0, 0, 0, 0);
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
                                                        float* partial) {
  __shared__ float s[4];
  const float4* E = reinterpret_cast<const float4*>(emb);
  const int kp4 = Kp >> 2;
  float acc = 0.f;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const int c0 = (int)(i % kp4) * 4;
    const float4 w = E[i];
    acc += (c0 + 0 < K1 ? w.x * w.x : 0.f) + (c0 + 1 < K1 ? w.y * w.y : 0.f) + (c0 + 2 < K1 ? w.z * w.z : 0.f) +
           (c0 + 3 < K1 ? w.w * w.w : 0.f);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

void launch_emb_sumsq(const float* emb, long long n4, int Kp, int K1, float* partial, int nblocks,
                      hipStream_t stream) {
  hipLaunchKernelGGL(emb_sumsq_kernel, dim3(nblocks), dim3(256), 0, stream, emb, n4, Kp, K1, partial);
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
