// Plan-ahead DP row merge: the union of every rank's exported ids, and each id's position in every
// rank's export, built on the SIDE chain for the next graph's steps — so the step's critical path
// keeps only a plan-driven gather-sum of the gathered rows (the reference's Horovod all-reduce of
// the embedding gradient, …vectorized-map.py:296, is the step's cross-rank hand-off it replaces).
//
// Every rank's export of step t is its batch's UNIQUE ids in ascending order (the sorted export of
// the step tail, emb_body.h mode 2): the side chain knows them a graph ahead (it sorts the next
// graph's batches).  Per graph, on the side stream:
//   uniq_keys     this rank's unique ids of each of the S batches (the sorted keys' run heads, at
//                 the same positions the export will use: the per-chunk head counts of sort_aux)
//   (exchange)    every rank's lists to every rank (p2p push or RCCL all-gather, dp.py)
//   plan_input    S segments of the W ranks' lists, rank-major, pads → key V (sorts last)
//   seg_sort      each segment on its id bits (stable: equal ids stay in rank order)
//   plan_count / plan_write   runs of equal ids → union entry u: plan_rows[u] = id and
//                 plan_pos[u][r] = the id's position in rank r's export, or −1
// On the main chain, after the step's all-gather of the exported rows, merge_plan_apply sums the
// W rows of each union entry in rank order (the same order as the search / maps merges: bitwise
// the same result) and applies lazy L2 + the row optimizer; the MLP optimizer rides as extra
// workgroups of the launch.
#include "../ops.h"
#include "merge.h"
#include "wgrad_body.h"

#include <algorithm>

namespace rocfm {
namespace {

constexpr int kPlanThreads = 256;
constexpr int kPlanTile = 1024;   // sorted entries per plan_count / plan_write workgroup
constexpr int kPlanApplyThreads = 64;

// ---- uniq_keys: one workgroup per (chunk, step) -------------------------------------------------
__global__ __launch_bounds__(1024) void uniq_keys_kernel(const PlanParams p) {
  __shared__ int s_w[16];
  __shared__ int s_base;
  const int c = blockIdx.x, k = blockIdx.y, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint32_t* kb = p.skeys + (size_t)k * p.n;
  const int32_t* ch = p.chunk_heads + (size_t)k * p.nch;
  if (t < 64) {  // heads in the chunks before this one (fixed order)
    int b = 0;
    for (int q = lane; q < c; q += 64) b += ch[q];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) b += __shfl_xor(b, o, 64);
    if (t == 0) s_base = b;
  }
  const int i = c * p.chunk + t;
  const bool in = t < p.chunk && i < p.n;
  const uint32_t key = in ? kb[i] : 0u;
  const bool head = in && (i == 0 || kb[i - 1] != key);
  const unsigned long long m = __ballot(head);
  if (lane == 0) s_w[wave] = __popcll(m);
  __syncthreads();
  int before = s_base;
  for (int w = 0; w < wave; ++w) before += s_w[w];
  before += __popcll(m & ((1ull << lane) - 1ull));
  uint32_t* out = p.ukeys + (size_t)k * p.ukey_stride;
  if (head && before < p.cap) out[before] = p.id_shift > 0 ? key - ((uint32_t)k << p.id_shift) : key;
  if (c == p.nch - 1 && t == 0) {
    int tot = s_base;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += s_w[w];
    p.ucount[(size_t)k * p.ucount_stride] = tot;
    if (tot > p.cap && p.overflow) *p.overflow = 1;
  }
}

// ---- plan_input: S segments of W·cap keys (rank r's list at r·cap), pads = V ----------------------
__global__ __launch_bounds__(kPlanThreads) void plan_input_kernel(const PlanParams p) {
  const long long i = (long long)blockIdx.x * kPlanThreads + threadIdx.x;
  const long long seg = (long long)p.W * p.cap;
  if (i >= (long long)p.S * seg) return;
  const int k = (int)(i / seg), rj = (int)(i - (long long)k * seg), r = rj / p.cap, j = rj - r * p.cap;
  const int32_t cnt = p.gcounts[(size_t)r * p.gc_stride + (size_t)k * p.gcount_step];
  const uint32_t key = j < min(cnt, p.cap) ? p.gkeys[(size_t)r * p.gk_stride + (size_t)k * p.gkey_step + j] : p.pad_key;
  p.pkeys[i] = key;
}

// ---- plan_count / plan_write: runs of equal ids in each sorted segment --------------------------
__device__ __forceinline__ bool plan_head(const PlanParams& p, const uint32_t* sk, int i) {
  const uint32_t key = sk[i];
  return key != p.pad_key && (i == 0 || sk[i - 1] != key);
}

__global__ __launch_bounds__(kPlanTile) void plan_count_kernel(const PlanParams p, int ntile) {
  __shared__ int s_w[kPlanTile / 64];
  const int k = blockIdx.y, tile = blockIdx.x, t = threadIdx.x;
  const int seg = p.W * p.cap;
  const uint32_t* sk = p.skeys_sorted + (size_t)k * seg;
  const int i = tile * kPlanTile + t;
  const bool h = i < seg && plan_head(p, sk, i);
  const unsigned long long m = __ballot(h);
  if ((t & 63) == 0) s_w[t >> 6] = __popcll(m);
  __syncthreads();
  if (t == 0) {
    int c = 0;
    for (int w = 0; w < kPlanTile / 64; ++w) c += s_w[w];
    p.tile_counts[(size_t)k * ntile + tile] = c;
  }
}

// A head writes its union entry whole: its id and the positions of the ≤ W equal ids that follow
// it (rank order, one per rank: every rank's list is unique) — no other thread writes the entry.
__global__ __launch_bounds__(kPlanTile) void plan_write_kernel(const PlanParams p, int ntile) {
  __shared__ int s_w[kPlanTile / 64];
  __shared__ int s_base;
  const int k = blockIdx.y, tile = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int seg = p.W * p.cap;
  const uint32_t* sk = p.skeys_sorted + (size_t)k * seg;
  const uint32_t* sv = p.svals_sorted + (size_t)k * seg;
  if (t < 64) {
    int b = 0;
    for (int q = lane; q < tile; q += 64) b += p.tile_counts[(size_t)k * ntile + q];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) b += __shfl_xor(b, o, 64);
    if (t == 0) s_base = b;
  }
  const int i = tile * kPlanTile + t;
  const bool h = i < seg && plan_head(p, sk, i);
  const unsigned long long m = __ballot(h);
  if (lane == 0) s_w[wave] = __popcll(m);
  __syncthreads();
  int u = s_base;
  for (int w = 0; w < wave; ++w) u += s_w[w];
  u += __popcll(m & ((1ull << lane) - 1ull));
  if (h) {
    const uint32_t key = sk[i];
    int32_t* pp = p.plan_pos + ((size_t)k * seg + u) * p.W;
    for (int q = 0; q < p.W; ++q) pp[q] = -1;
    for (int e = i; e < seg && e < i + p.W && sk[e] == key; ++e) {
      const uint32_t g = sv[e] - (uint32_t)((size_t)k * seg);  // r·cap + j
      const int r = (int)(g / (uint32_t)p.cap);
      pp[r] = (int)(g - (uint32_t)r * (uint32_t)p.cap);
    }
    p.plan_rows[(size_t)k * seg + u] = key;
  }
  if (tile == ntile - 1 && t == 0) {
    int tot = s_base;
    for (int w = 0; w < kPlanTile / 64; ++w) tot += s_w[w];
    p.plan_count[k] = tot;
  }
}

// ---- merge_plan_apply: one thread per union entry ----------------------------------------------
template <int KP4, int WMAX>
__device__ __forceinline__ void plan_apply_body(const MergeParams& p, const PlanStep& ps, const int u) {
  if (u >= *ps.count) return;
  const uint32_t row = ps.rows[u] / p.key_div;
  if (row >= p.Vmap) {  // (never: every plan id is a table row) a bad plan writes nothing past the table and
    if (p.overflow) atomicOr(p.overflow, 2);  // raises at check(): its gradients were not applied
    return;
  }
  const int32_t* pp = ps.pos + (size_t)u * p.W;
  const int W = p.W;
  const size_t base = (size_t)row * KP4;
  // the table row and its slots depend only on the id: issued with the positions
  float4 w[KP4], a[KP4], b[KP4];
  const float4* a4r = reinterpret_cast<const float4*>(p.s0 ? p.s0 : p.emb) + base;
  const float4* b4r = reinterpret_cast<const float4*>(p.s1 ? p.s1 : p.emb) + base;
#pragma unroll
  for (int c = 0; c < KP4; ++c) {
    w[c] = tbl_load4_rt(p.emb, base + c, p.tbl_bf16 != 0);
    a[c] = a4r[c];
    b[c] = b4r[c];
  }
  if (!p.s0)
#pragma unroll
    for (int c = 0; c < KP4; ++c) a[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (!p.s1)
#pragma unroll
    for (int c = 0; c < KP4; ++c) b[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 acc[KP4];
#pragma unroll
  for (int c = 0; c < KP4; ++c) acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (WMAX <= 8 && KP4 <= 4) {
    int pj[WMAX];
#pragma unroll
    for (int q = 0; q < WMAX; ++q) pj[q] = q < W ? pp[q] : -1;
    float4 v[WMAX][KP4];
#pragma unroll
    for (int q = 0; q < WMAX; ++q) {
      if (q >= W) break;
      const float4* src = reinterpret_cast<const float4*>(
          p.rows + (pj[q] >= 0 ? (size_t)q * p.row_stride + (size_t)pj[q] * p.Kp : 0));
#pragma unroll
      for (int c = 0; c < KP4; ++c) v[q][c] = src[c];
    }
#pragma unroll
    for (int q = 0; q < WMAX; ++q) {  // rank order: the search / maps merges' sum, bit for bit
      if (q >= W) break;
      if (pj[q] < 0) continue;
#pragma unroll
      for (int c = 0; c < KP4; ++c) {
        acc[c].x += v[q][c].x;
        acc[c].y += v[q][c].y;
        acc[c].z += v[q][c].z;
        acc[c].w += v[q][c].w;
      }
    }
  } else {
    for (int q = 0; q < W; ++q) {
      const int pq = pp[q];
      if (pq < 0) continue;
      const float4* src = reinterpret_cast<const float4*>(p.rows + (size_t)q * p.row_stride + (size_t)pq * p.Kp);
#pragma unroll
      for (int c = 0; c < KP4; ++c) {
        const float4 x = src[c];
        acc[c].x += x.x;
        acc[c].y += x.y;
        acc[c].z += x.z;
        acc[c].w += x.w;
      }
    }
  }
  if (p.mode == 1) {
    float4* dg = reinterpret_cast<float4*>(p.dense_grad) + base;
#pragma unroll
    for (int c = 0; c < KP4; ++c)
      dg[c] = make_float4(acc[c].x * p.grad_scale, acc[c].y * p.grad_scale, acc[c].z * p.grad_scale,
                          acc[c].w * p.grad_scale);
    if (p.touched) p.touched[row] = (uint32_t)*p.step + 1u;
    return;
  }
  const OptStep st = opt_step(p.opt, *p.step);
  float4* a4 = p.s0 ? reinterpret_cast<float4*>(p.s0) + base : nullptr;
  float4* b4 = p.s1 ? reinterpret_cast<float4*>(p.s1) + base : nullptr;
#pragma unroll
  for (int c = 0; c < KP4; ++c) {
    float* wc = &w[c].x;
    float* ac = &a[c].x;
    float* bc = &b[c].x;
    const float* gc = &acc[c].x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (c * 4 + e >= p.K1) continue;
      opt_apply(p.opt, st, wc[e], l2_grad(gc[e] * p.grad_scale, p.l2, wc[e]), ac[e], bc[e]);
    }
    tbl_store4_rt(p.emb, base + c, w[c], (uint32_t)*p.step, p.tbl_bf16 != 0);
    if (a4) a4[c] = a[c];
    if (b4) b4[c] = b[c];
  }
}

template <int KP4, int WMAX>
__global__ __launch_bounds__(kPlanApplyThreads) void merge_plan_apply_kernel(MergeParams p, PlanStep ps,
                                                                               DenseApplyParams d, int n_apply,
                                                                               int n_dense) {
  if ((int)blockIdx.x < n_apply) {
    plan_apply_body<KP4, WMAX>(p, ps, blockIdx.x * kPlanApplyThreads + threadIdx.x);
  } else if (n_dense > 0) {
    dense_apply_body<kPlanApplyThreads>(d, blockIdx.x - n_apply, n_dense);
  }
}

}  // namespace

size_t plan_sort_temp_bytes(int S, int W, int cap, int bits) { return seg_sort_temp_bytes(S, W * cap, bits); }

void launch_plan_build(const PlanParams& p, void* temp, size_t temp_bytes, int bits, hipStream_t stream) {
  ROCFM_REQUIRE(p.S > 0 && p.W >= 1 && p.W <= 64 && p.cap > 0, "plan_build: bad shape");
  ROCFM_REQUIRE(p.gkeys && p.gcounts && p.pkeys && p.skeys_sorted && p.svals_sorted && p.plan_rows && p.plan_pos &&
                    p.plan_count && p.tile_counts,
                "plan_build: null buffer");
  ROCFM_REQUIRE((long long)p.S * p.W * p.cap < (1ll << 31), "plan_build: more than 2^31 entries");
  const long long tot = (long long)p.S * p.W * p.cap;
  hipLaunchKernelGGL(plan_input_kernel, dim3((unsigned)((tot + kPlanThreads - 1) / kPlanThreads)), dim3(kPlanThreads),
                     0, stream, p);
  seg_sort_iota(temp, temp_bytes, p.pkeys, p.skeys_sorted, p.svals_sorted, p.S, p.W * p.cap, bits, stream, 0u);
  const int ntile = cdiv(p.W * p.cap, kPlanTile);
  hipLaunchKernelGGL(plan_count_kernel, dim3(ntile, p.S), dim3(kPlanTile), 0, stream, p, ntile);
  hipLaunchKernelGGL(plan_write_kernel, dim3(ntile, p.S), dim3(kPlanTile), 0, stream, p, ntile);
  ROCFM_HIP_CHECK(hipGetLastError());
}

int plan_tile_ints(int S, int W, int cap) { return S * cdiv(W * cap, kPlanTile); }

void launch_uniq_keys(const PlanParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.skeys && p.chunk_heads && p.ukeys && p.ucount && p.n > 0 && p.S > 0, "uniq_keys: bad params");
  ROCFM_REQUIRE(p.chunk % 64 == 0 && p.chunk <= 1024 && p.nch == cdiv(p.n, p.chunk), "uniq_keys: chunk");
  hipLaunchKernelGGL(uniq_keys_kernel, dim3(p.nch, p.S), dim3(p.chunk), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

void launch_merge_plan_apply(const MergeParams& p, const PlanStep& ps, const DenseApplyParams* d, hipStream_t stream) {
  ROCFM_REQUIRE(p.W >= 1 && p.W <= 64 && p.cap > 0 && ps.rows && ps.pos && ps.count && p.step,
                "merge_plan_apply: bad params");
  const int n_apply = cdiv(p.W * p.cap, kPlanApplyThreads);
  const int n_dense = d ? std::max(1, std::min(cdiv(d->n, kPlanApplyThreads), 1024)) : 0;
  const DenseApplyParams dd = d ? *d : DenseApplyParams{};
  const dim3 grid(n_apply + n_dense), block(kPlanApplyThreads);
  switch (p.Kp / 4) {
#define ROCFM_PLAN_KP4(N)                                                                                   \
  case N:                                                                                                   \
    if (p.W <= 8)                                                                                           \
      hipLaunchKernelGGL((merge_plan_apply_kernel<N, 8>), grid, block, 0, stream, p, ps, dd, n_apply, n_dense); \
    else                                                                                                    \
      hipLaunchKernelGGL((merge_plan_apply_kernel<N, 64>), grid, block, 0, stream, p, ps, dd, n_apply, n_dense); \
    break;
    ROCFM_PLAN_KP4(1) ROCFM_PLAN_KP4(2) ROCFM_PLAN_KP4(3) ROCFM_PLAN_KP4(4) ROCFM_PLAN_KP4(5) ROCFM_PLAN_KP4(6)
    ROCFM_PLAN_KP4(7) ROCFM_PLAN_KP4(8) ROCFM_PLAN_KP4(9) ROCFM_PLAN_KP4(10) ROCFM_PLAN_KP4(11) ROCFM_PLAN_KP4(12)
    ROCFM_PLAN_KP4(13) ROCFM_PLAN_KP4(14) ROCFM_PLAN_KP4(15) ROCFM_PLAN_KP4(16)
#undef ROCFM_PLAN_KP4
    default:
      throw std::invalid_argument("merge_plan_apply: unsupported Kp");
  }
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
