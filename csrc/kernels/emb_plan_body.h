// Planned embedding-row update: the step tail's embedding role driven by the side chain's work plan
// (emb_plan.hip).  Apply mode (sparse update on one GPU), gradient rows in sorted order.
//
// Workgroup bid takes plan item {es, ee, lead, tail}: the sorted entries [es, ee), whole runs
// except where the plan split a long run at a 64-entry window boundary.
//   1. rounds of 512 entries (one per thread, windows aligned to the sorted list; the next round's
//      loads issued before this one is scanned): keys, gradient rows, the segmented DPP scan
//      (emb_body.h), and every "piece" — a run's part of one window, the scan value at its last
//      entry — stored in LDS in order, with each run head's first piece;
//   2. a LEAD item (it holds the continuation of a run whose head lies in an earlier item) publishes
//      those window pieces to plan_win with write-through stores, drains them, and adds one to the
//      run's counter (agent scope, no return value: nothing waits on it);
//   3. the optimizer on every complete run (fold of its pieces, as emb_body.h step 6);
//   4. the TAIL item of a split run (its head item) waits until the counter shows every lead item
//      arrived (bounded polling: all items of a step are co-resident, the grid is one dispatch round),
//      folds its own pieces and then the published window pieces in window order, applies the
//      optimizer to that row and resets the counter.
// Every run's gradient is the left-to-right fold of its window pieces — the same bits as the
// unplanned body (emb_body.h step 5) that the per-step path runs.  The hand-off follows the
// row-tile split's exchange (deepfm_rows.hip): write-through payload, drained, one agent-scope
// atomic per arrival, write-through (sc1) loads after the wait.  A wait that runs out sets the
// plan's sticky error word (plan_ctr[plan_nw] bit 1) and skips that row; check() raises.
#pragma once
#include "emb_body.h"

namespace rocfm {

typedef __attribute__((address_space(1))) unsigned long long pg_u64;
typedef __attribute__((address_space(1))) unsigned int pg_u32;
constexpr uint64_t kPlanSpinTicks = 100000000ull;  // 1 s of s_memrealtime (100 MHz): a lead item never arrived

__device__ __forceinline__ void wt_store4(float* dst, float4 v) {
  const unsigned long long lo = (unsigned long long)__float_as_uint(v.x) | ((unsigned long long)__float_as_uint(v.y) << 32);
  const unsigned long long hi = (unsigned long long)__float_as_uint(v.z) | ((unsigned long long)__float_as_uint(v.w) << 32);
  __hip_atomic_store((pg_u64*)dst, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store((pg_u64*)dst + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float4 wt_load4(const float* src) {
  const unsigned long long lo = __hip_atomic_load((pg_u64*)src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long hi = __hip_atomic_load((pg_u64*)src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_float4(__uint_as_float((uint32_t)lo), __uint_as_float((uint32_t)(lo >> 32)),
                     __uint_as_float((uint32_t)hi), __uint_as_float((uint32_t)(hi >> 32)));
}

// optimizer on float4 column u4 (index idx) of a table row, loaded as w / a / b, with gradient
// sum acc (emb_body.h step 6, apply mode)
template <bool BT>
__device__ __forceinline__ void plan_apply4_rows(const EmbUpdateParams& p, const OptStep& st, size_t idx, float4 w,
                                                 float4 a, float4 b, int u4, float4 acc, uint32_t stp) {
#pragma clang fp contract(off)
  const float4 g = make_float4(acc.x * p.grad_scale, acc.y * p.grad_scale, acc.z * p.grad_scale, acc.w * p.grad_scale);
  float* wc = &w.x;
  float* ac = &a.x;
  float* bc = &b.x;
  const float* gc = &g.x;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (u4 * 4 + c >= p.K1) continue;
    opt_apply(p.opt, st, wc[c], l2_grad(gc[c], p.l2, wc[c]), ac[c], bc[c]);
  }
  tbl_store4<BT>(p.emb, idx, w, stp);
  if (p.s0) reinterpret_cast<float4*>(p.s0)[idx] = a;
  if (p.s1) reinterpret_cast<float4*>(p.s1)[idx] = b;
}

template <int KP4, bool BT>
__device__ __forceinline__ void emb_plan_body(const EmbUpdateParams& p, const int bid) {
  constexpr int kT = 512, kW = kT / 64;
  __shared__ float4 s_piece[kPlanPcap * KP4];
  __shared__ uint32_t s_hkey[kPlanHcap];
  __shared__ int s_hp[kPlanHcap + 1];  // first piece of each run; [nh] = the piece count
  __shared__ int s_wp[kW], s_wh[kW];
  __shared__ int s_last[1];
  const int4 item = p.plan_items[bid];
  const int es = item.x, ee = item.y, lead = item.z, tail = item.w;
  if (es >= ee) return;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const OptStep st = opt_step(p.opt, p.step ? *p.step : 0);
  const uint32_t stp = p.step ? (uint32_t)*p.step : 0u;
  int4 sl_tail = make_int4(0, 0, 0, 0);
  if (tail >= 0) sl_tail = p.plan_slots[tail];
  // the tail split run's table row (wave 1, one float4 column per lane), loaded now: only its head
  // item (this workgroup) updates that row in this launch
  const int grp = t >> 6;
  const bool cmb = grp == 1 && lane < KP4 && tail >= 0;
  float4 cw = make_float4(0.f, 0.f, 0.f, 0.f), ca = cw, cb = cw;
  size_t cidx = 0;
  if (cmb) {
    const int4 sl = sl_tail;
    cidx = (size_t)(((uint32_t)sl.x - (uint32_t)p.id_offset) / (uint32_t)p.id_stride) * KP4 + lane;
    cw = tbl_load4<BT>(p.emb, cidx);
    if (p.s0) ca = reinterpret_cast<const float4*>(p.s0)[cidx];
    if (p.s1) cb = reinterpret_cast<const float4*>(p.s1)[cidx];
  }
  // 0. the table / Adam-slot rows of the item's complete runs (first 4·512 (run, float4 column)
  //    items), loaded now from the plan's head-key slab so they arrive under phase 1's scan; the
  //    count and the keys are independent loads (one memory latency, then the rows)
  float4 w[4], a[4], b[4];
  size_t idx4[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    w[u] = a[u] = b[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    idx4[u] = 0;
  }
  int pf_heads = -1;  // the slab's head count (-1: no slab; phase 2 loads the rows itself)
  if (p.plan_hslab) {
    const uint32_t* slab = p.plan_hslab + (size_t)bid * kPlanSlab;
    uint32_t hk[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) hk[u] = slab[1 + min((u * kT + t) / KP4, kPlanSlab - 2)];
    pf_heads = (int)slab[0];
    const int pf_items = (pf_heads - (tail >= 0 ? 1 : 0)) * KP4;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int itm = u * kT + t;
      idx4[u] = (size_t)((hk[u] - (uint32_t)p.id_offset) / (uint32_t)p.id_stride) * KP4 + (itm % KP4);
      if (itm < pf_items) {
        w[u] = tbl_load4<BT>(p.emb, idx4[u]);
        if (p.s0) a[u] = reinterpret_cast<const float4*>(p.s0)[idx4[u]];
        if (p.s1) b[u] = reinterpret_cast<const float4*>(p.s1)[idx4[u]];
      }
    }
  }
  ROCFM_STAMP(p.stamps, 0);
  // 1. pieces; the next round's keys and gradient rows are loaded before this round is scanned
  int np = 0, nh = 0;
  const unsigned long long lt = (1ull << lane) - 1ull;
  uint32_t key = 0u, prevk = 0u;
  float4 v[KP4];
  auto load_round = [&](int r0, uint32_t& k, uint32_t& pk, float4 (&x)[KP4]) {
    const int i = r0 + t;
    const bool live = i >= es && i < ee;
    k = live ? p.skeys[i] : 0u;
    pk = (live && i > 0) ? p.skeys[i - 1] : 0u;
    const float4* src = reinterpret_cast<const float4*>(p.contrib + (size_t)(live ? i : 0) * p.Kp);
#pragma unroll
    for (int u = 0; u < KP4; ++u) x[u] = live ? src[u] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  load_round(es & ~63, key, prevk, v);
  for (int r0 = es & ~63; r0 < ee; r0 += kT) {
    const int i = r0 + t;
    const bool live = i >= es && i < ee;
    const bool head = live && (i == 0 || prevk != key);
    uint32_t nkey = 0u, nprev = 0u;
    float4 nv[KP4];
    if (r0 + kT < ee) load_round(r0 + kT, nkey, nprev, nv);  // (uniform)
    const unsigned long long hm = __ballot(head || lane == 0 || !live);
    const unsigned long long below = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
    seg_scan_dpp(v, lane, 63 - __clzll(hm & below));
    const unsigned long long hb = __ballot(head);
    const bool nexthead = lane < 63 && ((hb >> (lane + 1)) & 1ull);
    const bool pend = live && (lane == 63 || i + 1 == ee || nexthead);
    const unsigned long long pm = __ballot(pend);
    if (lane == 0) {
      s_wp[wave] = __popcll(pm);
      s_wh[wave] = __popcll(hb);
    }
    __syncthreads();
    int bp = np, bh = nh, tp = 0, th = 0;
#pragma unroll
    for (int w = 0; w < kW; ++w) {
      bp += w < wave ? s_wp[w] : 0;
      bh += w < wave ? s_wh[w] : 0;
      tp += s_wp[w];
      th += s_wh[w];
    }
    const int pslot = bp + __popcll(pm & lt);
    if (pend && pslot < kPlanPcap) {
#pragma unroll
      for (int u = 0; u < KP4; ++u) s_piece[pslot * KP4 + u] = v[u];
    }
    if (head) {
      const int hs = bh + __popcll(hb & lt);
      if (hs < kPlanHcap) {
        s_hkey[hs] = key;
        s_hp[hs] = pslot;  // the piece this head's run starts in
      }
    }
    np += tp;
    nh += th;
    __syncthreads();
    key = nkey;
    prevk = nprev;
#pragma unroll
    for (int u = 0; u < KP4; ++u) v[u] = nv[u];
  }
  if (np > kPlanPcap || nh >= kPlanHcap) {  // outside the plan's bounds (emb_plan.hip): never trains wrong
    if (t == 0) atomicOr(reinterpret_cast<int*>(p.plan_ctr) + p.plan_nw, 1);
    return;
  }
  if (t == 0) s_hp[nh] = np;
  __syncthreads();
  ROCFM_STAMP(p.stamps, 1);
  // 2. lead items: publish the continuation's window pieces (write-through stores)
  const int nlead = lead >= 0 ? (nh > 0 ? s_hp[0] : np) : 0;
  if (lead >= 0) {
    for (int q = t; q < nlead * KP4; q += kT) {
      const int j = q / KP4, u = q - j * KP4;
      wt_store4(p.plan_win + ((size_t)(es >> 6) + j) * p.Kp + 4 * u, s_piece[q]);
    }
  }
  // 3. complete runs: (run, float4 column) items over all threads; each round's table / slot loads
  //    first (emb_body.h step 6) — the first round's are issued before the lead arrival below, so
  //    the drain of the publish stores runs under them
  const int nfull = nh - (tail >= 0 ? 1 : 0);
  const int nitems = nfull * KP4;
  if (pf_heads >= 0 && pf_heads != nh && t == 0)  // the slab disagrees with the item's keys: a plan bug
    atomicOr(reinterpret_cast<int*>(p.plan_ctr) + p.plan_nw, 4);
  auto load_items = [&](int base) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int itm = min(base + u * kT + t, nitems - 1);
      const int r = itm / KP4, u4 = itm - r * KP4;
      const size_t row = (size_t)((s_hkey[r] - (uint32_t)p.id_offset) / (uint32_t)p.id_stride);
      idx4[u] = row * KP4 + u4;
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      w[u] = tbl_load4<BT>(p.emb, idx4[u]);
      a[u] = p.s0 ? reinterpret_cast<const float4*>(p.s0)[idx4[u]] : z;
      b[u] = p.s1 ? reinterpret_cast<const float4*>(p.s1)[idx4[u]] : z;
    }
  };
  if (nitems > 0 && pf_heads != nh) load_items(0);  // (prefetched at entry when the slab is there)
  if (lead >= 0) {  // arrival: the pieces drained first, then one counter increment
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) __hip_atomic_fetch_add((pg_u32*)(p.plan_ctr + lead), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int base = 0; base < nitems; base += kT * 4) {
#pragma clang fp contract(off)
    if (base > 0) load_items(base);
    float4 g[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int itm = min(base + u * kT + t, nitems - 1);
      const int r = itm / KP4, u4 = itm - r * KP4;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int j = s_hp[r]; j < s_hp[r + 1]; ++j) acc = f4add(acc, s_piece[j * KP4 + u4]);
      g[u] = make_float4(acc.x * p.grad_scale, acc.y * p.grad_scale, acc.z * p.grad_scale, acc.w * p.grad_scale);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int itm = base + u * kT + t;
      if (itm >= nitems) continue;
      const int u4 = itm % KP4;
      float* wc = &w[u].x;
      float* ac = &a[u].x;
      float* bc = &b[u].x;
      const float* gc = &g[u].x;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (u4 * 4 + c >= p.K1) continue;
        opt_apply(p.opt, st, wc[c], l2_grad(gc[c], p.l2, wc[c]), ac[c], bc[c]);
      }
      tbl_store4<BT>(p.emb, idx4[u], w[u], stp);
      if (p.s0) reinterpret_cast<float4*>(p.s0)[idx4[u]] = a[u];
      if (p.s1) reinterpret_cast<float4*>(p.s1)[idx4[u]] = b[u];
    }
  }
  ROCFM_STAMP(p.stamps, 2);
  // 4. the head item of a split run: wait for its lead items, fold, optimizer, reset
  if (tail >= 0) {
    if (t == 0) {
      const unsigned want = (unsigned)sl_tail.w - 1u;
      pg_u32* ctr = (pg_u32*)(p.plan_ctr + tail);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      int ok = 1;
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > kPlanSpinTicks) {
          atomicOr(reinterpret_cast<int*>(p.plan_ctr) + p.plan_nw, 2);
          ok = 0;
          break;
        }
      }
      s_last[0] = ok;
    }
    __syncthreads();
    if (grp == 1 && lane < KP4 && s_last[0]) {  // (cmb: the tail row's w / a / b were loaded at the start)
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int j = s_hp[nh - 1]; j < np; ++j) acc = f4add(acc, s_piece[j * KP4 + lane]);
      constexpr int kB = 16;  // every piece's write-through load issued before the fold uses any
      for (int w0 = sl_tail.y; w0 <= sl_tail.z; w0 += kB) {
        float4 x[kB];
#pragma unroll
        for (int q = 0; q < kB; ++q)
          x[q] = wt_load4(p.plan_win + (size_t)min(w0 + q, sl_tail.z) * p.Kp + 4 * lane);
#pragma unroll
        for (int q = 0; q < kB; ++q)
          if (w0 + q <= sl_tail.z) acc = f4add(acc, x[q]);
      }
      plan_apply4_rows<BT>(p, st, cidx, cw, ca, cb, lane, acc, stp);
      if (lane == 0) __hip_atomic_store((pg_u32*)(p.plan_ctr + tail), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  ROCFM_STAMP(p.stamps, 3);
}

}  // namespace rocfm
