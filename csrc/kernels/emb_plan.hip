// The step tail's embedding work plan (EmbPlanParams, emb_update.h), one workgroup per batch, run on
// the side chain for every batch of the next multi-step graph (fused.py _prepare_multi).
//
// Why: the unplanned tail gives every workgroup 256 consecutive sorted lookups.  A chunk's cost is
// its gradient rows plus one table / Adam-slot round trip per run head, and heads per chunk range
// 0-176 at the bench shapes (the Zipf tail is all heads, the hot ids are runs of up to 1,024), so the
// slowest chunks set the role's span (profiles/r5_phases_*: span 8.3 / 14.2 µs against a per-chunk
// mean of 6.3 / 11.3 at k = 10 / 32).  The plan cuts the lookups into `nw` items of EQUAL cost —
// entries + beta · heads — one per embedding workgroup, so the role spreads over every CU the
// weight-gradient role leaves free.
//
// Cuts: item k holds the cut positions c with floor((c + beta · runs before c) / Q) = k,
// Q = ceil((n + beta · U) / nw).  Allowed cuts are run heads, and inside runs longer than `lsplit`
// the 64-entry window boundaries.  A run cut inside is split: its head item (tail slot) publishes the
// fold of its window pieces, every later item (lead slot) its window pieces, and the last arrival
// combines them (emb_plan_body.h).  Items hold ≤ Q/(1+beta)+1 heads and ≤ Q+lsplit+63 entries.
// Deterministic: a pure function of the sorted keys.
#include "emb_update.h"

namespace rocfm {

constexpr int kPlanThreads = 1024;

// exclusive prefix sum over the workgroup (16 waves); total to every thread; s_w[17] scratch
__device__ __forceinline__ int plan_scan(int v, int* s_w, int& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[wave] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int a = 0;
    for (int w = 0; w < kPlanThreads / 64; ++w) {
      const int c = s_w[w];
      s_w[w] = a;
      a += c;
    }
    s_w[kPlanThreads / 64] = a;
  }
  __syncthreads();
  const int r = s_w[wave] + x - v;
  total = s_w[kPlanThreads / 64];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(kPlanThreads) void emb_plan_kernel(const EmbPlanParams p) {
  __shared__ int s_w[kPlanThreads / 64 + 1];
  const int k = blockIdx.x, t = threadIdx.x, n = p.n;
  const uint32_t* kb = p.skeys + (size_t)k * n;
  int32_t* runs = p.runs + (size_t)k * (n + 1);
  int* it = reinterpret_cast<int*>(p.items + (size_t)k * p.nw);  // {es, ee, lead, tail} per item
  int4* slots = p.slots + (size_t)k * p.nw;
  for (int j = t; j < p.nw; j += kPlanThreads) p.items[(size_t)k * p.nw + j] = make_int4(0, 0, -1, -1);
  // 1. run starts, compacted in order
  const int m = (n + kPlanThreads - 1) / kPlanThreads;
  const int i0 = min(n, t * m), i1 = min(n, i0 + m);
  int h = 0;
  {
    uint32_t prev = i0 > 0 ? kb[i0 - 1] : 0u;
    for (int i = i0; i < i1; ++i) {
      const uint32_t key = kb[i];
      h += (i == 0 || key != prev) ? 1 : 0;
      prev = key;
    }
  }
  int U = 0;
  int base = plan_scan(h, s_w, U);
  {
    uint32_t prev = i0 > 0 ? kb[i0 - 1] : 0u;
    for (int i = i0; i < i1; ++i) {
      const uint32_t key = kb[i];
      if (i == 0 || key != prev) runs[base++] = i;
      prev = key;
    }
  }
  if (t == 0) runs[U] = n;
  __syncthreads();  // (the item initialisation above and the run list: read by other threads below)
  // 2. cuts → items; split runs → slots
  const long long beta = p.beta, Q = max(1ll, ((long long)n + beta * U + p.nw - 1) / p.nw);
  const int ls = p.lsplit;
  auto item_of = [&](int c, int r) { return (int)(((long long)c + beta * r) / Q); };
  auto last_cut = [&](int r) {  // the last allowed cut inside run r (its head if it is not split-able)
    const int s = runs[r], e = runs[r + 1];
    if (e - s > ls) {
      const int c = (e - 1) & ~63;
      return c > s ? c : s;
    }
    return s;
  };
  const int ru = (U + kPlanThreads - 1) / kPlanThreads;
  const int r0 = min(U, t * ru), r1 = min(U, r0 + ru);
  int nsplit = 0;
  for (int r = r0; r < r1; ++r) {
    const int s = runs[r], e = runs[r + 1];
    if (e - s > ls && item_of(last_cut(r), r) != item_of(s, r)) ++nsplit;
  }
  int NS = 0;
  int slot = plan_scan(nsplit, s_w, NS);
  for (int r = r0; r < r1; ++r) {
    const int s = runs[r], e = runs[r + 1];
    const int ih = item_of(s, r);
    const int ip = r > 0 ? item_of(last_cut(r - 1), r - 1) : -1;
    if (ih != ip) {  // a new item starts at this head
      it[4 * ih + 0] = s;
      if (ip >= 0) it[4 * ip + 1] = s;
    }
    int cur = ih, pieces = 1, sl = -1, wh = 0;
    if (e - s > ls) {
      for (int c = (s & ~63) + 64; c < e; c += 64) {
        const int ic = item_of(c, r);
        if (ic == cur) continue;
        if (sl < 0) {
          sl = slot++;
          wh = c >> 6;
          it[4 * ih + 3] = sl;  // the head item folds its pieces into plan_head[sl]
        }
        it[4 * ic + 0] = c;
        it[4 * cur + 1] = c;
        it[4 * ic + 2] = sl;  // a later item: its window pieces of this run
        cur = ic;
        ++pieces;
      }
    }
    if (sl >= 0) slots[sl] = make_int4((int)kb[s], wh, (e - 1) >> 6, pieces);
    if (r == U - 1) it[4 * cur + 1] = n;
  }
}

void launch_emb_plan(const EmbPlanParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.n > 0 && p.S > 0 && p.nw > 0 && p.beta >= 0 && p.lsplit >= 64, "emb_plan: bad sizes");
  ROCFM_REQUIRE(p.skeys && p.runs && p.items && p.slots, "emb_plan: buffers missing");
  // item bounds the planned tail relies on (emb_plan_body.h): heads ≤ Q/(1+beta) + 1 ≤ kPlanHcap
  const long long qmax = ((long long)p.n * (1 + p.beta) + p.nw - 1) / p.nw;
  ROCFM_REQUIRE(qmax / (1 + p.beta) + 2 <= kPlanHcap, "emb_plan: too few items for the batch (raise nw)");
  ROCFM_REQUIRE((qmax + p.lsplit + 64) / 64 + 2 <= kPlanPcap - kPlanHcap, "emb_plan: items too long (raise nw)");
  hipLaunchKernelGGL(emb_plan_kernel, dim3(p.S), dim3(kPlanThreads), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
