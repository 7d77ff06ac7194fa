// The step tail's embedding work plan (EmbPlanParams, emb_update.h), one workgroup per batch, run on
// the side chain for every batch of the next multi-step graph (fused.py _prepare_multi).
// 256 threads (48 VGPRs: one wave per SIMD): a plan workgroup fits on a CU beside a k = 32 row-tile
// workgroup (the split ones included), so the 256-workgroup row kernels no longer wait for CUs the
// plan holds (1,024 threads: up to 4 row tiles entered 14 µs late; profiles/r6_side_overlap.md)
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

constexpr int kPlanThreads = 256;

constexpr int kPlanWaves = kPlanThreads / 64;

// exclusive prefix over the 16 waves of one value per wave (lane 0's), to every lane; one barrier
// pair.  s_w[kPlanWaves + 1] scratch; the total in s_w[kPlanWaves].
__device__ __forceinline__ int plan_wave_base(int v, int* s_w) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) s_w[wave] = v;
  __syncthreads();
  int b = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kPlanWaves; ++w) {
    const int c = s_w[w];
    b += w < wave ? c : 0;
    tot += c;
  }
  __syncthreads();
  if (threadIdx.x == 0) s_w[kPlanWaves] = tot;
  __syncthreads();
  return b;
}

// Each wave walks its own contiguous segment of the batch's entries (then of its runs) 64 at a time
// — coalesced loads, eight groups in flight, ranks by ballot — so the launch needs four barriers in
// all (a workgroup-wide rank per 1024-entry tile cost two barriers each: 45 µs per launch).
__global__ __launch_bounds__(kPlanThreads) void emb_plan_kernel(const EmbPlanParams p) {
  __shared__ int s_w[kPlanWaves + 1];
  __shared__ int s_r0[kPlanMaxNw], s_r1[kPlanMaxNw];  // per item: first / last run whose head it holds
  const int k = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6, n = p.n;
  const uint32_t* kb = p.skeys + (size_t)k * n;
  int32_t* runs = p.runs + (size_t)k * (n + 1);
  int* it = reinterpret_cast<int*>(p.items + (size_t)k * p.nw);  // {es, ee, lead, tail} per item
  int4* slots = p.slots + (size_t)k * p.nw;
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int j = t; j < p.nw; j += kPlanThreads) {
    p.items[(size_t)k * p.nw + j] = make_int4(0, 0, -1, -1);
    s_r0[j] = 0x7fffffff;
    s_r1[j] = -1;
  }
  // 1. run starts, compacted in order: count per wave segment, prefix over waves, write
  constexpr int kG = 8;  // 64-entry groups loaded before any is ranked
  const int seg = ((n + kPlanWaves - 1) / kPlanWaves + 63) & ~63;
  const int e0 = min(n, wave * seg), e1 = min(n, e0 + seg);
  auto heads = [&](int g0, unsigned long long (&hm)[kG]) {  // head ballots of groups g0 .. g0+kG-1
    uint32_t key[kG], prev[kG];
#pragma unroll
    for (int q = 0; q < kG; ++q) {
      const int i = g0 + 64 * q + lane;
      key[q] = i < e1 ? kb[i] : 0u;
      prev[q] = (i > 0 && i < e1) ? kb[i - 1] : 0u;
    }
#pragma unroll
    for (int q = 0; q < kG; ++q) {
      const int i = g0 + 64 * q + lane;
      hm[q] = __ballot(i < e1 && (i == 0 || key[q] != prev[q]));
    }
  };
  int cnt = 0;
  for (int g0 = e0; g0 < e1; g0 += 64 * kG) {
    unsigned long long hm[kG];
    heads(g0, hm);
#pragma unroll
    for (int q = 0; q < kG; ++q) cnt += __popcll(hm[q]);
  }
  int base = plan_wave_base(cnt, s_w);
  const int U = s_w[kPlanWaves];
  for (int g0 = e0; g0 < e1; g0 += 64 * kG) {
    unsigned long long hm[kG];
    heads(g0, hm);
#pragma unroll
    for (int q = 0; q < kG; ++q) {
      if ((hm[q] >> lane) & 1ull) runs[base + __popcll(hm[q] & lt)] = g0 + 64 * q + lane;
      base += __popcll(hm[q]);
    }
  }
  if (t == 0) runs[U] = n;
  __syncthreads();  // (the item initialisation above and the run list: read by other threads below)
  // 2. cuts → items; split runs → slots, numbered in run order
  // (32-bit cost positions: n · (1 + beta) < 2^31, checked by the launcher; a 64-bit division is a
  // long software sequence per cut)
  const uint32_t beta = (uint32_t)p.beta, Q = max(1u, ((uint32_t)n + beta * (uint32_t)U + p.nw - 1) / (uint32_t)p.nw);
  const int ls = p.lsplit;
  auto item_of = [&](int c, int r) { return (int)(((uint32_t)c + beta * (uint32_t)r) / Q); };
  auto last_cut = [&](int s, int e) {  // the last allowed cut inside run [s, e) (its head if not split-able)
    if (e - s > ls) {
      const int c = (e - 1) & ~63;
      return c > s ? c : s;
    }
    return s;
  };
  const int rseg = ((U + kPlanWaves - 1) / kPlanWaves + 63) & ~63;
  const int q0 = min(U, wave * rseg), q1 = min(U, q0 + rseg);
  constexpr int kR = 4;  // 64-run groups loaded before any is used
  auto split_of = [&](int s, int e, int r) { return e - s > ls && item_of(last_cut(s, e), r) != item_of(s, r); };
  int nsp = 0;
  for (int g0 = q0; g0 < q1; g0 += 64 * kR) {
    int rs[kR], re[kR];
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      const int r = g0 + 64 * q + lane;
      rs[q] = r < q1 ? runs[r] : 0;
      re[q] = r < q1 ? runs[r + 1] : 0;
    }
#pragma unroll
    for (int q = 0; q < kR; ++q) nsp += __popcll(__ballot(g0 + 64 * q + lane < q1 && split_of(rs[q], re[q], g0 + 64 * q + lane)));
  }
  int slot = plan_wave_base(nsp, s_w);
  for (int g0 = q0; g0 < q1; g0 += 64 * kR) {
    int rs[kR], re[kR], rp[kR];
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      const int r = g0 + 64 * q + lane;
      rs[q] = r < q1 ? runs[r] : 0;
      re[q] = r < q1 ? runs[r + 1] : 0;
      rp[q] = (r > 0 && r < q1) ? runs[r - 1] : 0;
    }
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      const int r = g0 + 64 * q + lane;
      const bool live = r < q1;
      const int s = rs[q], e = re[q], sp = rp[q];
      const bool split = live && split_of(s, e, r);
      const unsigned long long sm = __ballot(split);
      const int sl = slot + __popcll(sm & lt);
      slot += __popcll(sm);
      if (!live) continue;
      const int ih = item_of(s, r);
      atomicMin(&s_r0[ih], r);
      atomicMax(&s_r1[ih], r);
      const int ip = r > 0 ? item_of(last_cut(sp, s), r - 1) : -1;
      if (ih != ip) {  // a new item starts at this head
        it[4 * ih + 0] = s;
        if (ip >= 0) it[4 * ip + 1] = s;
      }
      int cur = ih, pieces = 1, wh = 0;
      if (split) {
        for (int c = (s & ~63) + 64; c < e; c += 64) {
          const int ic = item_of(c, r);
          if (ic == cur) continue;
          if (pieces == 1) {
            wh = c >> 6;
            it[4 * ih + 3] = sl;  // the head item folds its pieces into plan_head[sl]
          }
          it[4 * ic + 0] = c;
          it[4 * cur + 1] = c;
          it[4 * ic + 2] = sl;  // a later item: its window pieces of this run
          cur = ic;
          ++pieces;
        }
        slots[sl] = make_int4((int)kb[s], wh, (e - 1) >> 6, pieces);
      }
      if (r == U - 1) it[4 * cur + 1] = n;
    }
  }
  if (!p.hslab) return;
  // 3. each item's run-head keys in order, behind its head count (the tail prefetches their rows)
  __syncthreads();
  uint32_t* slab = p.hslab + (size_t)k * p.nw * kPlanSlab;
  for (int j = t; j < p.nw; j += kPlanThreads) slab[(size_t)j * kPlanSlab] = s_r1[j] >= 0 ? (uint32_t)(s_r1[j] - s_r0[j] + 1) : 0u;
  for (int g0 = q0; g0 < q1; g0 += 64 * kR) {
    int rs[kR];
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      const int r = g0 + 64 * q + lane;
      rs[q] = r < q1 ? runs[r] : 0;
    }
    uint32_t key[kR];
#pragma unroll
    for (int q = 0; q < kR; ++q) key[q] = kb[rs[q]];
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      const int r = g0 + 64 * q + lane;
      if (r >= q1) continue;
      const int ih = item_of(rs[q], r), j = r - s_r0[ih];
      if (j < kPlanSlab - 1) slab[(size_t)ih * kPlanSlab + 1 + j] = key[q];
    }
  }
}

void launch_emb_plan(const EmbPlanParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.n > 0 && p.S > 0 && p.nw > 0 && p.beta >= 0 && p.lsplit >= 64, "emb_plan: bad sizes");
  ROCFM_REQUIRE((long long)p.n * (1 + p.beta) + p.nw < (1ll << 31), "emb_plan: cost positions exceed 32 bits");
  ROCFM_REQUIRE(p.skeys && p.runs && p.items && p.slots, "emb_plan: buffers missing");
  ROCFM_REQUIRE(p.nw <= kPlanMaxNw, "emb_plan: more items than the kernel's head ranges hold");
  // item bounds the planned tail relies on (emb_plan_body.h): heads ≤ Q/(1+beta) + 1 ≤ kPlanHcap
  const long long qmax = ((long long)p.n * (1 + p.beta) + p.nw - 1) / p.nw;
  ROCFM_REQUIRE(qmax / (1 + p.beta) + 2 <= kPlanHcap, "emb_plan: too few items for the batch (raise nw)");
  ROCFM_REQUIRE((qmax + p.lsplit + 64) / 64 + 2 <= kPlanPcap - kPlanHcap, "emb_plan: items too long (raise nw)");
  hipLaunchKernelGGL(emb_plan_kernel, dim3(p.S), dim3(kPlanThreads), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
