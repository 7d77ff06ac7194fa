// Multi-source row-gradient merge by direct addressing — see merge.h.
#include "merge.h"
#include "wgrad_body.h"
#include "shard_body.h"

#include <algorithm>

namespace rocfm {
namespace {

constexpr uint32_t kPadKey = 0xFFFFFFFFu;
constexpr int kMergeThreads = 256;
// merge_apply: ≈cap·W threads, each a chain of dependent loads: one wave per workgroup spreads the
// few waves over as many CUs (and their L1 / address units) as possible instead of 4 per CU
constexpr int kApplyThreads = 64;
constexpr int kMaxW = 64;

__device__ __forceinline__ float4 f4add_m(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

__device__ __forceinline__ bool entry_valid(const MergeParams& p, int r, int j, uint32_t key) {
  if (key == kPadKey) return false;
  if (p.counts && j >= p.counts[(size_t)r * p.count_stride]) return false;
  return key / p.key_div < p.Vmap;
}

// ---- hash mode ------------------------------------------------------------------------------
typedef unsigned long long u64;
__device__ __forceinline__ uint32_t hash_row(uint32_t x) {  // murmur3 finaliser
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t merge_tag(const MergeParams& p) { return (uint32_t)*p.step + 1u; }

// Insert (or find) row in this step's table; returns its slot (the table has ≥ 2× the entries)
__device__ __forceinline__ int hash_claim(const MergeParams& p, uint32_t row, uint32_t T) {
  const uint32_t mask = (uint32_t)p.hash_slots - 1u;
  const u64 mine = ((u64)T << 32) | row;
  uint32_t slot = hash_row(row) & mask;
  for (int probe = 0; probe < p.hash_slots; ++probe) {
    u64 cur = __hip_atomic_load(p.hkeys + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while ((uint32_t)(cur >> 32) != T) {  // stale (earlier step) or never used: claim it
      const u64 prev = atomicCAS(p.hkeys + slot, cur, mine);
      if (prev == cur) return (int)slot;
      cur = prev;
    }
    if ((uint32_t)cur == row) return (int)slot;
    slot = (slot + 1u) & mask;
  }
  return -1;  // unreachable with hash_slots ≥ 2·W·cap
}

__device__ __forceinline__ int hash_find(const MergeParams& p, uint32_t row, uint32_t T) {
  const uint32_t mask = (uint32_t)p.hash_slots - 1u;
  const u64 mine = ((u64)T << 32) | row;
  uint32_t slot = hash_row(row) & mask;
  for (int probe = 0; probe < p.hash_slots; ++probe) {
    const u64 cur = p.hkeys[slot];
    if (cur == mine) return (int)slot;
    if ((uint32_t)(cur >> 32) != T) return -1;  // an empty slot ends the chain
    slot = (slot + 1u) & mask;
  }
  return -1;
}

__global__ __launch_bounds__(kMergeThreads) void merge_init_kernel(MergeParams p) {
  const long long i = (long long)blockIdx.x * kMergeThreads + threadIdx.x;
  const long long n = (long long)p.W * p.Vmap;
  if (i < n) p.pos[i] = -1;
  if (i < p.Vmap) p.rep[i] = p.W;
}

__device__ __forceinline__ void merge_scatter_body(const MergeParams& p, const int bid) {
  const int i = bid * kMergeThreads + threadIdx.x;
  if (i >= p.W * p.cap) return;
  const int r = i / p.cap, j = i - r * p.cap;
  if (j == 0 && p.overflow && p.counts && p.counts[(size_t)r * p.count_stride] > p.cap) *p.overflow = 1;
  const uint32_t key = p.keys[(size_t)r * p.key_stride + j];
  if (!entry_valid(p, r, j, key)) return;
  const uint32_t row = key / p.key_div;
  if (p.hash_slots > 0) {
    const uint32_t T = merge_tag(p);
    const int slot = hash_claim(p, row, T);
    if (slot < 0) {
      if (p.overflow) *p.overflow = 1;
      return;
    }
    p.hpos[(size_t)slot * p.W + r] = ((u64)T << 32) | (uint32_t)j;
    atomicMax(p.hrep + slot, ((u64)T << 32) | (0xFFFFFFFFu - (uint32_t)r));
    return;
  }
  p.pos[(size_t)r * p.Vmap + row] = j;
  atomicMin(&p.rep[row], r);
}

__global__ __launch_bounds__(kMergeThreads) void merge_scatter_kernel(MergeParams p) {
  merge_scatter_body(p, blockIdx.x);
}

// Owner-sharded DP: append the updated row to the broadcast list (MergeParams::bc_*).
// With bc_push the peers' "entered" flags (raised by their row kernels) are read at the start of the
// merge body (bc_seen) and compared before the first store into their slots.
__device__ __forceinline__ PushSeen bc_seen(const MergeParams& p) {
  return (p.bc_count != nullptr && p.bc_push.W > 0) ? push_ready_load(p.bc_push) : PushSeen{};
}

template <int KP4>
__device__ __forceinline__ void bcast_row(const MergeParams& p, uint32_t row, const float4 (&w)[KP4],
                                          const PushSeen& seen) {
  if (p.bc_count == nullptr) return;
  const int s = atomicAdd(p.bc_count, 1);
  if (s >= p.bc_cap) return;  // (cannot happen: bc_cap = W·cap ≥ every source's entries)
  const uint32_t gid = row * p.bc_mul + p.bc_add;
  if (p.bc_push.W > 0) {
    push_wait_ready(p.bc_push, seen);
    for (int d = 0; d < p.bc_push.W; ++d) {
      float* b = p.bc_push.slot[d];
      reinterpret_cast<uint32_t*>(b + 4)[s] = gid;
      float4* o = reinterpret_cast<float4*>(b + 4 + p.bc_cap) + (size_t)s * KP4;
#pragma unroll
      for (int c = 0; c < KP4; ++c) o[c] = w[c];
    }
    push_drain();
    return;
  }
  p.bc_keys[s] = gid;
  float4* o = reinterpret_cast<float4*>(p.bc_rows) + (size_t)s * KP4;
#pragma unroll
  for (int c = 0; c < KP4; ++c) o[c] = w[c];
}

// One thread per source entry; only representatives (lowest rank holding the key) do work.
// WMAX = 8 (one node): every later source's position and row are loaded before any is summed.
template <int KP4, int WMAX>
__device__ __forceinline__ void merge_maps_body(const MergeParams& p, const int i) {
  if (i >= p.W * p.cap) return;
  const int r = i / p.cap, j = i - r * p.cap;
  const uint32_t key = p.keys[(size_t)r * p.key_stride + j];
  if (!entry_valid(p, r, j, key)) return;
  const uint32_t row = key / p.key_div;
  const bool hashed = p.hash_slots > 0;
  const uint32_t T = hashed ? merge_tag(p) : 0u;
  int slot = -1;
  if (hashed) {
    slot = hash_find(p, row, T);
    if (slot < 0) return;
    const u64 rv = p.hrep[slot];
    if ((uint32_t)(rv >> 32) != T || 0xFFFFFFFFu - (uint32_t)rv != (uint32_t)r) return;
  } else if (p.rep[row] != r) {
    return;
  }
  // position of `row` in source q's list this step, or −1
  auto pos_of = [&](int q) -> int {
    if (hashed) {
      const u64 v = p.hpos[(size_t)slot * p.W + q];
      return (uint32_t)(v >> 32) == T ? (int)(uint32_t)v : -1;
    }
    return p.pos[(size_t)q * p.Vmap + row];
  };
  const int W = p.W;
  const size_t base = (size_t)row * KP4;
  const PushSeen seen = bc_seen(p);
  // the table row and its optimizer slots depend only on the row: issued now, in the same round
  // trip as the other sources' positions (one dependent global round trip less per row)
  // (mode 1 does not need them; the loads are harmless there: emb / slots are always valid)
  // Absent slots read the table instead and are zeroed after the load: a `ptr ? load : 0` here
  // became a select between a global and a private address (flat access + scratch).
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
    for (int q = 0; q < WMAX; ++q)
      pj[q] = (q < W && q > r) ? pos_of(q) : (q == r ? j : -1);
    float4 v[WMAX][KP4];
#pragma unroll
    for (int q = 0; q < WMAX; ++q) {
      if (q >= W) break;  // wave-uniform: no loads for ranks that do not exist
      const float4* src = reinterpret_cast<const float4*>(
          p.rows + (pj[q] >= 0 ? (size_t)q * p.row_stride + (size_t)pj[q] * p.Kp : 0));
#pragma unroll
      for (int c = 0; c < KP4; ++c) v[q][c] = src[c];
    }
#pragma unroll
    for (int q = 0; q < WMAX; ++q) {  // rank order: deterministic sum
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
    for (int q = r; q < W; ++q) {  // rank order: deterministic sum
      const int pq = q == r ? j : pos_of(q);
      if (pq < 0) continue;
      const float4* src = reinterpret_cast<const float4*>(p.rows + (size_t)q * p.row_stride + (size_t)pq * p.Kp);
#pragma unroll
      for (int c = 0; c < KP4; ++c) {
        const float4 v = src[c];
        acc[c].x += v.x;
        acc[c].y += v.y;
        acc[c].z += v.z;
        acc[c].w += v.w;
      }
    }
  }
  // restore the maps for the next step (no other thread reads them for this key any more); the
  // hash table needs no restore (its words are tagged with the step)
  if (!hashed) {
    for (int q = r; q < W; ++q) p.pos[(size_t)q * p.Vmap + row] = -1;
    p.rep[row] = W;
  }

  if (p.mode == 1) {
    float4* dg = reinterpret_cast<float4*>(p.dense_grad) + base;
#pragma unroll
    for (int c = 0; c < KP4; ++c) {
      float4 g = acc[c];
      g.x *= p.grad_scale;
      g.y *= p.grad_scale;
      g.z *= p.grad_scale;
      g.w *= p.grad_scale;
      dg[c] = g;
    }
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
    for (int u = 0; u < 4; ++u) {
      if (c * 4 + u >= p.K1) continue;
      opt_apply(p.opt, st, wc[u], l2_grad(gc[u] * p.grad_scale, p.l2, wc[u]), ac[u], bc[u]);
    }
    tbl_store4_rt(p.emb, base + c, w[c], (uint32_t)*p.step, p.tbl_bf16 != 0);
    if (a4) a4[c] = a[c];
    if (b4) b4[c] = b[c];
  }
  bcast_row<KP4>(p, row, w, seen);
}

template <int KP4, int WMAX>
__global__ __launch_bounds__(kApplyThreads) void merge_apply_kernel(MergeParams p) {
  merge_maps_body<KP4, WMAX>(p, blockIdx.x * kApplyThreads + threadIdx.x);
}

// merge_scatter with the DP MLP optimizer (dense_apply over the gathered rank segments) as extra
// workgroups of the same launch: the two are independent, the merge_apply that follows needs both.
__global__ __launch_bounds__(kMergeThreads) void merge_scatter_dense_kernel(MergeParams p, DenseApplyParams d,
                                                                            int n_scatter, int n_dense) {
  if ((int)blockIdx.x < n_scatter) {
    merge_scatter_body(p, blockIdx.x);
  } else {
    dense_apply_body(d, blockIdx.x - n_scatter, n_dense);
  }
}

// ---- search mode ----------------------------------------------------------------------------
// Source q's list and its valid length (counts, else the cap: pads sort last)
__device__ __forceinline__ const uint32_t* list_of(const MergeParams& p, int q) { return p.keys + (size_t)q * p.key_stride; }
__device__ __forceinline__ int len_of(const MergeParams& p, int q) {
  return p.counts ? min(max(p.counts[(size_t)q * p.count_stride], 0), p.cap) : p.cap;
}

// Optimizer (mode 0) or dense-gradient row (mode 1) of one merged row: shared by the search apply
template <int KP4>
__device__ __forceinline__ void merged_row_out(const MergeParams& p, uint32_t row, float4 (&w)[KP4], float4 (&a)[KP4],
                                               float4 (&b)[KP4], const float4 (&acc)[KP4],
                                               const PushSeen& seen = PushSeen{}) {
  const size_t base = (size_t)row * KP4;
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
    for (int u = 0; u < 4; ++u) {
      if (c * 4 + u >= p.K1) continue;
      opt_apply(p.opt, st, wc[u], l2_grad(gc[u] * p.grad_scale, p.l2, wc[u]), ac[u], bc[u]);
    }
    tbl_store4_rt(p.emb, base + c, w[c], (uint32_t)*p.step, p.tbl_bf16 != 0);
    if (a4) a4[c] = a[c];
    if (b4) b4[c] = b[c];
  }
  bcast_row<KP4>(p, row, w, seen);
}

// WMAX = 8: the W−1 searches advance together (≈log2(cap) rounds of up to 7 independent loads);
// larger worlds search the lists one after another.
template <int KP4, int WMAX>
__device__ __forceinline__ void merge_search_body(const MergeParams& p, const int i) {
  if (i >= p.W * p.cap) return;
  const int r = i / p.cap, j = i - r * p.cap;
  if (j == 0 && p.overflow && p.counts && p.counts[(size_t)r * p.count_stride] > p.cap) *p.overflow = 1;
  const uint32_t key = p.keys[(size_t)r * p.key_stride + j];
  if (!entry_valid(p, r, j, key)) return;
  const uint32_t row = key / p.key_div;
  const int W = p.W;
  const size_t base = (size_t)row * KP4;
  const PushSeen seen = bc_seen(p);
  // the row's parameters and slots: issued before the searches (same as merge_apply)
  float4 w[KP4], a[KP4], b[KP4];
  const float4* a4r = reinterpret_cast<const float4*>(p.s0 ? p.s0 : p.emb) + base;
  const float4* b4r = reinterpret_cast<const float4*>(p.s1 ? p.s1 : p.emb) + base;
  if (p.mode == 0) {
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
  }
  float4 acc[KP4];
  const float4* own = reinterpret_cast<const float4*>(p.rows + (size_t)r * p.row_stride + (size_t)j * p.Kp);
#pragma unroll
  for (int c = 0; c < KP4; ++c) acc[c] = own[c];
  if (W > 1) {
    if constexpr (WMAX <= 8) {
      int lo[WMAX], len[WMAX], at[WMAX];
      // bucket directories (the sorted export's dir[b] = first position whose key ≥ b·bucket_div):
      // each search starts inside the key's bucket — one round of directory loads, then
      // ≈log2(bucket) instead of ≈log2(cap) dependent halvings
      const bool use_dir = p.dirs != nullptr && p.nb > 0;
      const int bk = use_dir ? (int)min(key / p.bucket_div, (uint32_t)p.nb - 1u) : 0;
#pragma unroll
      for (int q = 0; q < WMAX; ++q) {
        lo[q] = 0;
        at[q] = -1;
        len[q] = (q < W && q != r) ? len_of(p, q) : 0;
        if (use_dir && len[q] > 0) {
          const int32_t* d = p.dirs + (size_t)q * p.dir_stride;
          const int b0 = min(max(d[bk], 0), len[q]), b1 = min(max(d[bk + 1], 0), len[q]);
          lo[q] = b0;
          len[q] = max(b1 - b0, 0);
        }
      }
      for (;;) {
        bool any = false;
#pragma unroll
        for (int q = 0; q < WMAX; ++q) {
          if (len[q] <= 0) continue;
          any = true;
          const int half = len[q] >> 1;
          const uint32_t v = list_of(p, q)[lo[q] + half];
          if (v == key) {
            at[q] = lo[q] + half;
            len[q] = 0;
          } else if (v < key) {
            lo[q] += half + 1;
            len[q] -= half + 1;
          } else {
            len[q] = half;
          }
        }
        if (!any) break;
      }
#pragma unroll
      for (int q = 0; q < WMAX; ++q)
        if (q < r && at[q] >= 0) return;  // a lower rank holds the key: not the representative
      // rank order, this entry's own row first (it is the lowest rank holding the key)
      float4 v[WMAX][KP4];
#pragma unroll
      for (int q = 0; q < WMAX; ++q) {
        const float4* src = reinterpret_cast<const float4*>(
            p.rows + (at[q] >= 0 ? (size_t)q * p.row_stride + (size_t)at[q] * p.Kp : 0));
#pragma unroll
        for (int c = 0; c < KP4; ++c) v[q][c] = (q < W && q > r && at[q] >= 0) ? src[c] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int q = 0; q < WMAX; ++q) {
        if (q >= W || q <= r || at[q] < 0) continue;
#pragma unroll
        for (int c = 0; c < KP4; ++c) acc[c] = f4add_m(acc[c], v[q][c]);
      }
    } else {
      auto find = [&](int q) -> int {
        const uint32_t* L = list_of(p, q);
        int lo = 0, len = len_of(p, q);
        while (len > 0) {
          const int half = len >> 1;
          const uint32_t v = L[lo + half];
          if (v == key) return lo + half;
          if (v < key) {
            lo += half + 1;
            len -= half + 1;
          } else {
            len = half;
          }
        }
        return -1;
      };
      for (int q = 0; q < r; ++q)
        if (find(q) >= 0) return;
      for (int q = r + 1; q < W; ++q) {
        const int at = find(q);
        if (at < 0) continue;
        const float4* src = reinterpret_cast<const float4*>(p.rows + (size_t)q * p.row_stride + (size_t)at * p.Kp);
#pragma unroll
        for (int c = 0; c < KP4; ++c) acc[c] = f4add_m(acc[c], src[c]);
      }
    }
  }
  merged_row_out<KP4>(p, row, w, a, b, acc, seen);
}

// One thread per replicated row (all KP4 float4 columns): Σ of the rank segments in rank order
// (the owner merge's order, so replicated and owned rows take bit-identical updates), then the
// row optimizer on the replica; the bucket part is cleared for the next step.
// The row's touched-count word is read AND cleared by this one thread.  With the bucket reduced
// in place (h.zero == h.grads: world 1 / RCCL all-reduce) a per-column thread layout had the
// c == 0 thread clear the word while sibling columns — in a later wave or workgroup when KP4
// does not divide 64 — had yet to read it: those columns then skipped (sparse) or took an
// L2-only update (exact), which made exact + hot rows non-reproducible under CU contention.
template <int KP4>
__device__ __forceinline__ void hot_apply_body(const HotApplyParams& h, const int r) {
  if (r >= h.H) return;
  float4 acc[KP4];
#pragma unroll
  for (int c = 0; c < KP4; ++c) acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  float cnt = 0.f;
  for (int q = 0; q < h.nseg; ++q) {
    const float* seg = h.grads + (size_t)q * h.seg_stride;
    const float4* s4 = reinterpret_cast<const float4*>(seg) + (size_t)r * KP4;
#pragma unroll
    for (int c = 0; c < KP4; ++c) acc[c] = f4add_m(acc[c], s4[c]);
    cnt += seg[(size_t)h.H * KP4 * 4 + r];
  }
  if (h.zero) {
    float4* z4 = reinterpret_cast<float4*>(h.zero) + (size_t)r * KP4;
#pragma unroll
    for (int c = 0; c < KP4; ++c) z4[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    h.zero[(size_t)h.H * KP4 * 4 + r] = 0.f;
  }
  const bool has = cnt > 0.f;
  if (!has && !h.dense) return;
  const OptStep st = opt_step(h.opt, *h.step);
#pragma unroll
  for (int c = 0; c < KP4; ++c) {
    const size_t at = (size_t)r * KP4 + c;
    float4 w = reinterpret_cast<const float4*>(h.rows)[at];
    float4 a = h.s0 ? reinterpret_cast<const float4*>(h.s0)[at] : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 b = h.s1 ? reinterpret_cast<const float4*>(h.s1)[at] : make_float4(0.f, 0.f, 0.f, 0.f);
    float* wc = &w.x;
    float* ac = &a.x;
    float* bc = &b.x;
    const float* gc = &acc[c].x;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (c * 4 + u >= h.K1) continue;
      const float g = has ? gc[u] * h.grad_scale : 0.f;
      opt_apply(h.opt, st, wc[u], l2_grad(g, h.l2, wc[u]), ac[u], bc[u]);
    }
    reinterpret_cast<float4*>(h.rows)[at] = w;
    if (h.s0) reinterpret_cast<float4*>(h.s0)[at] = a;
    if (h.s1) reinterpret_cast<float4*>(h.s1)[at] = b;
  }
}

// Roles by workgroup: [merge apply | MLP optimizer | serve of the NEXT step's requests (bounded-
// staleness row-shard mode: it reads rows this launch may be updating, Hogwild-style like the
// reference's asynchronous parameter server) | replicated-row update]
template <int KP4, int WMAX>
__global__ __launch_bounds__(kApplyThreads) void merge_search_apply_kernel(MergeParams p, DenseApplyParams d,
                                                                           ShardServeParams sv, HotApplyParams hot,
                                                                           int n_apply, int n_dense, int n_serve) {
  const int b = blockIdx.x;
  if (b < n_apply) {
    if (p.use_maps)  // maps filled by a merge_scatter launch (larger worlds)
      merge_maps_body<KP4, WMAX>(p, b * kApplyThreads + threadIdx.x);
    else
      merge_search_body<KP4, WMAX>(p, b * kApplyThreads + threadIdx.x);
  } else if (b < n_apply + n_dense) {
    dense_apply_body<kApplyThreads>(d, b - n_apply, n_dense);
  } else if (b < n_apply + n_dense + n_serve) {
    shard_serve_body(sv, (long long)(b - n_apply - n_dense) * kApplyThreads + threadIdx.x);
  } else {
    hot_apply_body<KP4>(hot, (b - n_apply - n_dense - n_serve) * kApplyThreads + threadIdx.x);
  }
}

// ---- range mode ------------------------------------------------------------------------------
constexpr int kRangeThreads = 256;
// LDS stage per workgroup: small enough for several workgroups per CU (W = 8 launches ≈ 316 of them
// on 256 CUs); larger buckets take the global-search fallback
constexpr int kRangeLdsBytes = 36 * 1024;

// Position of key in the ascending run [lo, hi) of an LDS key array, or -1
__device__ __forceinline__ int lds_find(const uint32_t* k, int lo, int hi, uint32_t key) {
  int len = hi - lo;
  while (len > 0) {
    const int half = len >> 1;
    const uint32_t v = k[lo + half];
    if (v == key) return lo + half;
    if (v < key) {
      lo += half + 1;
      len -= half + 1;
    } else {
      len = half;
    }
  }
  return -1;
}

// ... of a source list in global memory: positions [lo, hi) of source q
__device__ __forceinline__ int glob_find(const MergeParams& p, int q, int lo, int hi, uint32_t key) {
  const uint32_t* L = list_of(p, q);
  int len = hi - lo;
  while (len > 0) {
    const int half = len >> 1;
    const uint32_t v = L[lo + half];
    if (v == key) return lo + half;
    if (v < key) {
      lo += half + 1;
      len -= half + 1;
    } else {
      len = half;
    }
  }
  return -1;
}

// The row's parameters / slots (mode 0), then the optimizer or the dense-gradient row
template <int KP4>
__device__ __forceinline__ void range_row_out(const MergeParams& p, uint32_t row, const float4 (&acc)[KP4]) {
  const size_t base = (size_t)row * KP4;
  float4 w[KP4], a[KP4], b[KP4];
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  if (p.mode == 0) {
    const float4* a4r = reinterpret_cast<const float4*>(p.s0 ? p.s0 : p.emb) + base;
    const float4* b4r = reinterpret_cast<const float4*>(p.s1 ? p.s1 : p.emb) + base;
#pragma unroll
    for (int c = 0; c < KP4; ++c) {
      w[c] = tbl_load4_rt(p.emb, base + c, p.tbl_bf16 != 0);
      a[c] = p.s0 ? a4r[c] : z;
      b[c] = p.s1 ? b4r[c] : z;
    }
  }
  merged_row_out<KP4>(p, row, w, a, b, acc);
}

template <int KP4>
__device__ __forceinline__ void merge_range_body(const MergeParams& p, const int bkt, const int cap_lds) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float4* s_row = reinterpret_cast<float4*>(smem);                                 // [cap_lds][KP4]
  uint32_t* s_key = reinterpret_cast<uint32_t*>(smem + (size_t)cap_lds * KP4 * 16);  // [cap_lds]
  __shared__ int s_lo[kMaxW], s_off[kMaxW + 1];
  const int W = p.W, t = threadIdx.x;
  if (t < W) {  // this bucket's range of source t: one round trip for all sources
    const int len = len_of(p, t);
    const int32_t* d = p.dirs + (size_t)t * p.dir_stride;
    const int lo = min(max(d[bkt], 0), len), hi = min(max(d[bkt + 1], 0), len);
    s_lo[t] = lo;
    s_off[t + 1] = max(hi - lo, 0);
  }
  __syncthreads();
  if (t == 0) {
    s_off[0] = 0;
    for (int q = 0; q < W; ++q) s_off[q + 1] += s_off[q];
  }
  __syncthreads();
  const int m = s_off[W];
  if (m == 0) return;
  if (m <= cap_lds) {
    // 1. stage every source's keys + gradient rows of the bucket (independent loads)
    for (int e = t; e < m; e += kRangeThreads) {
      int r = 0;
      while (r + 1 < W && e >= s_off[r + 1]) ++r;
      const int j = s_lo[r] + e - s_off[r];
      s_key[e] = list_of(p, r)[j];
      const float4* src = reinterpret_cast<const float4*>(p.rows + (size_t)r * p.row_stride + (size_t)j * p.Kp);
#pragma unroll
      for (int c = 0; c < KP4; ++c) s_row[(size_t)e * KP4 + c] = src[c];
    }
    __syncthreads();
    // 2. representatives (no lower rank holds the key) sum the rows in rank order
    for (int e = t; e < m; e += kRangeThreads) {
      int r = 0;
      while (r + 1 < W && e >= s_off[r + 1]) ++r;
      const uint32_t key = s_key[e];
      if (key == kPadKey || key / p.key_div >= p.Vmap) continue;
      bool rep = true;
      for (int q = 0; q < r && rep; ++q) rep = lds_find(s_key, s_off[q], s_off[q + 1], key) < 0;
      if (!rep) continue;
      float4 acc[KP4];
#pragma unroll
      for (int c = 0; c < KP4; ++c) acc[c] = s_row[(size_t)e * KP4 + c];
      for (int q = r + 1; q < W; ++q) {
        const int f = lds_find(s_key, s_off[q], s_off[q + 1], key);
        if (f < 0) continue;
#pragma unroll
        for (int c = 0; c < KP4; ++c) acc[c] = f4add_m(acc[c], s_row[(size_t)f * KP4 + c]);
      }
      range_row_out<KP4>(p, key / p.key_div, acc);
    }
  } else {  // a bucket larger than the stage: global binary searches inside the bucket's ranges
    for (int e = t; e < m; e += kRangeThreads) {
      int r = 0;
      while (r + 1 < W && e >= s_off[r + 1]) ++r;
      const int j = s_lo[r] + e - s_off[r];
      const uint32_t key = list_of(p, r)[j];
      if (key == kPadKey || key / p.key_div >= p.Vmap) continue;
      bool rep = true;
      for (int q = 0; q < r && rep; ++q) rep = glob_find(p, q, s_lo[q], s_lo[q] + s_off[q + 1] - s_off[q], key) < 0;
      if (!rep) continue;
      float4 acc[KP4];
      const float4* own = reinterpret_cast<const float4*>(p.rows + (size_t)r * p.row_stride + (size_t)j * p.Kp);
#pragma unroll
      for (int c = 0; c < KP4; ++c) acc[c] = own[c];
      for (int q = r + 1; q < W; ++q) {
        const int f = glob_find(p, q, s_lo[q], s_lo[q] + s_off[q + 1] - s_off[q], key);
        if (f < 0) continue;
        const float4* src = reinterpret_cast<const float4*>(p.rows + (size_t)q * p.row_stride + (size_t)f * p.Kp);
#pragma unroll
        for (int c = 0; c < KP4; ++c) acc[c] = f4add_m(acc[c], src[c]);
      }
      range_row_out<KP4>(p, key / p.key_div, acc);
    }
  }
}

template <int KP4>
__global__ __launch_bounds__(kRangeThreads) void merge_range_apply_kernel(MergeParams p, DenseApplyParams d,
                                                                          int n_range, int n_dense, int cap_lds) {
  if ((int)blockIdx.x < n_range)
    merge_range_body<KP4>(p, blockIdx.x, cap_lds);
  else
    dense_apply_body<kRangeThreads>(d, blockIdx.x - n_range, n_dense);
}

template <int KP4>
void launch_range_t(const MergeParams& p, const DenseApplyParams* d, hipStream_t stream) {
  const int cap_lds = merge_range_lds_entries(p.Kp);
  const int lds = cap_lds * (KP4 * 16 + 4);
  auto kern = merge_range_apply_kernel<KP4>;
  static bool attr = false;
  if (!attr) {
    ROCFM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kRangeLdsBytes));
    attr = true;
  }
  const int n_dense = d ? std::max(1, std::min(cdiv(d->n, kRangeThreads), 256)) : 0;
  DenseApplyParams dd{};
  if (d) dd = *d;
  hipLaunchKernelGGL(kern, dim3(p.nb + n_dense), dim3(kRangeThreads), lds, stream, p, dd, p.nb, n_dense, cap_lds);
}

template <int KP4>
void launch_search_t(const MergeParams& p, const DenseApplyParams* d, const ShardServeParams* sv,
                     const HotApplyParams* hot, hipStream_t stream) {
  const int n_apply = p.cap > 0 ? cdiv(p.W * p.cap, kApplyThreads) : 0;
  const int n_dense = d ? std::max(1, std::min(cdiv(d->n, kApplyThreads), 1024)) : 0;
  const long long n_sv = sv ? (long long)sv->m * (sv->Kp / 4) : 0;
  const int n_serve = (int)((n_sv + kApplyThreads - 1) / kApplyThreads);
  DenseApplyParams dd{};
  if (d) dd = *d;
  ShardServeParams ss{};
  if (sv) ss = *sv;
  HotApplyParams hh{};
  if (hot) hh = *hot;
  const int n_hot = hot ? cdiv(hot->H, kApplyThreads) : 0;  // one thread per replicated row
  if (n_apply + n_dense + n_serve + n_hot == 0) return;
  const dim3 grid(n_apply + n_dense + n_serve + n_hot), block(kApplyThreads);
  if (p.W <= 8)
    hipLaunchKernelGGL((merge_search_apply_kernel<KP4, 8>), grid, block, 0, stream, p, dd, ss, hh, n_apply, n_dense,
                       n_serve);
  else
    hipLaunchKernelGGL((merge_search_apply_kernel<KP4, kMaxW>), grid, block, 0, stream, p, dd, ss, hh, n_apply,
                       n_dense, n_serve);
}

template <int KP4>
void launch_apply_t(const MergeParams& p, hipStream_t stream) {
  const dim3 grid(cdiv(p.W * p.cap, kApplyThreads)), block(kApplyThreads);
  if (p.W <= 8)
    hipLaunchKernelGGL((merge_apply_kernel<KP4, 8>), grid, block, 0, stream, p);
  else
    hipLaunchKernelGGL((merge_apply_kernel<KP4, kMaxW>), grid, block, 0, stream, p);
}

void check(const MergeParams& p) {
  ROCFM_REQUIRE(p.W >= 1 && p.W <= kMaxW, "merge: 1 <= W <= 64");
  ROCFM_REQUIRE(p.Kp % 4 == 0 && p.Kp >= 4 && p.Kp <= 64 && p.K1 <= p.Kp, "merge: bad Kp");
  ROCFM_REQUIRE((long long)p.W * p.cap < (1ll << 31), "merge: W*cap overflows int32");
  ROCFM_REQUIRE(p.key_div >= 1, "merge: key_div");
  if (p.hash_slots > 0) {
    ROCFM_REQUIRE((p.hash_slots & (p.hash_slots - 1)) == 0 && (long long)p.hash_slots >= 2ll * p.W * p.cap,
                  "merge: hash_slots must be a power of two >= 2*W*cap");
    ROCFM_REQUIRE(p.hkeys && p.hrep && p.hpos && p.step, "merge: hash buffers / step missing");
  } else {
    ROCFM_REQUIRE(p.pos && p.rep, "merge: maps missing");
  }
}

}  // namespace

template <int KP4>
__global__ __launch_bounds__(kMergeThreads) void row_scatter_kernel(RowScatterParams p) {
  const long long per = (long long)p.cap * KP4;
  const long long n = (long long)p.W * per;
  for (long long it = (long long)blockIdx.x * kMergeThreads + threadIdx.x; it < n;
       it += (long long)gridDim.x * kMergeThreads) {
    const int r = (int)(it / per);
    const long long e = it - r * per;
    const int i = (int)(e / KP4), c = (int)(e - (long long)i * KP4);
    const float* slot = p.recv + (size_t)r * p.slot_stride;
    if (i >= reinterpret_cast<const int32_t*>(slot)[0]) continue;
    const uint32_t key = reinterpret_cast<const uint32_t*>(slot + 4)[i];
    if (key >= p.rows) continue;
    const float4 v = reinterpret_cast<const float4*>(slot + 4 + p.cap)[(size_t)i * KP4 + c];
    reinterpret_cast<float4*>(p.table)[(size_t)key * KP4 + c] = v;
  }
}

void launch_row_scatter(const RowScatterParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.recv && p.table && p.W >= 1 && p.cap >= 0 && p.cap % 4 == 0 && p.Kp % 4 == 0 && p.Kp <= 64,
                "row_scatter: bad parameters");
  ROCFM_REQUIRE(p.slot_stride >= 4 + (long long)p.cap * (1 + p.Kp), "row_scatter: slot too small");
  const long long n = (long long)p.W * p.cap * (p.Kp / 4);
  if (n == 0) return;
  const unsigned grid = (unsigned)std::min<long long>((n + kMergeThreads - 1) / kMergeThreads, 2048);
  switch (p.Kp / 4) {
#define ROCFM_KP4(N)                                                                        \
  case N:                                                                                   \
    hipLaunchKernelGGL(row_scatter_kernel<N>, dim3(grid), dim3(kMergeThreads), 0, stream, p); \
    break;
    ROCFM_KP4(1) ROCFM_KP4(2) ROCFM_KP4(3) ROCFM_KP4(4) ROCFM_KP4(5) ROCFM_KP4(6) ROCFM_KP4(7) ROCFM_KP4(8)
    ROCFM_KP4(9) ROCFM_KP4(10) ROCFM_KP4(11) ROCFM_KP4(12) ROCFM_KP4(13) ROCFM_KP4(14) ROCFM_KP4(15) ROCFM_KP4(16)
#undef ROCFM_KP4
    default:
      throw std::invalid_argument("row_scatter: unsupported Kp");
  }
  ROCFM_HIP_CHECK(hipGetLastError());
}

void launch_merge_init(const MergeParams& p, hipStream_t stream) {
  check(p);
  if (p.hash_slots > 0) return;  // the tagged hash table starts zeroed and is never reset
  const long long n = (long long)p.W * p.Vmap;
  hipLaunchKernelGGL(merge_init_kernel, dim3((unsigned)((n + kMergeThreads - 1) / kMergeThreads)),
                     dim3(kMergeThreads), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

void launch_merge_scatter(const MergeParams& p, hipStream_t stream) {
  check(p);
  if (p.cap <= 0) return;
  hipLaunchKernelGGL(merge_scatter_kernel, dim3(cdiv(p.W * p.cap, kMergeThreads)), dim3(kMergeThreads), 0, stream,
                     p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

void launch_merge_scatter_dense(const MergeParams& p, const DenseApplyParams& d, hipStream_t stream) {
  check(p);
  const int n_scatter = p.cap > 0 ? cdiv(p.W * p.cap, kMergeThreads) : 0;
  const int n_dense = std::max(1, std::min(cdiv(d.n, 256), 256));
  hipLaunchKernelGGL(merge_scatter_dense_kernel, dim3(n_scatter + n_dense), dim3(kMergeThreads), 0, stream, p, d,
                     n_scatter, n_dense);
  ROCFM_HIP_CHECK(hipGetLastError());
}

void launch_merge_search_apply(const MergeParams& p, const DenseApplyParams* d, const ShardServeParams* sv,
                               const HotApplyParams* hot, hipStream_t stream) {
  ROCFM_REQUIRE(p.W >= 1 && p.W <= kMaxW, "merge: 1 <= W <= 64");
  ROCFM_REQUIRE(p.Kp % 4 == 0 && p.Kp >= 4 && p.Kp <= 64 && p.K1 <= p.Kp, "merge: bad Kp");
  ROCFM_REQUIRE((long long)p.W * p.cap < (1ll << 31), "merge: W*cap overflows int32");
  ROCFM_REQUIRE(p.key_div >= 1 && p.keys && p.rows && p.step, "merge: keys / rows / step missing");
  if (p.use_maps) check(p);  // maps mode: validated as merge_apply
  ROCFM_REQUIRE(p.mode == 1 ? p.dense_grad != nullptr : p.emb != nullptr, "merge_search_apply: missing outputs");
  ROCFM_REQUIRE(sv == nullptr || (sv->Kp % 4 == 0 && sv->Kp > 0 && sv->ids && sv->table),
                "merge_search_apply: bad serve params");
  ROCFM_REQUIRE(hot == nullptr || (hot->Kp == p.Kp && hot->H > 0 && hot->rows && hot->grads && hot->step &&
                                   hot->nseg >= 1 && hot->K1 <= hot->Kp),
                "merge_search_apply: bad hot-row params");
  switch (p.Kp / 4) {
#define ROCFM_KP4(N)                    \
  case N:                               \
    launch_search_t<N>(p, d, sv, hot, stream); \
    break;
    ROCFM_KP4(1) ROCFM_KP4(2) ROCFM_KP4(3) ROCFM_KP4(4) ROCFM_KP4(5) ROCFM_KP4(6) ROCFM_KP4(7) ROCFM_KP4(8)
    ROCFM_KP4(9) ROCFM_KP4(10) ROCFM_KP4(11) ROCFM_KP4(12) ROCFM_KP4(13) ROCFM_KP4(14) ROCFM_KP4(15) ROCFM_KP4(16)
#undef ROCFM_KP4
    default:
      throw std::invalid_argument("merge: unsupported Kp");
  }
  ROCFM_HIP_CHECK(hipGetLastError());
}

int merge_range_lds_entries(int Kp) {
  const int per = Kp * 4 + 4;  // gradient row + key
  return std::min(512, kRangeLdsBytes / per / 64 * 64);
}

void launch_merge_range_apply(const MergeParams& p, const DenseApplyParams* d, hipStream_t stream) {
  ROCFM_REQUIRE(p.W >= 1 && p.W <= kMaxW, "merge_range: 1 <= W <= 64");
  ROCFM_REQUIRE(p.Kp % 4 == 0 && p.Kp >= 4 && p.Kp <= 64 && p.K1 <= p.Kp, "merge_range: bad Kp");
  ROCFM_REQUIRE(p.key_div >= 1 && p.keys && p.rows && p.step && p.dirs && p.nb >= 1 && p.bucket_div >= 1,
                "merge_range: keys / rows / step / directories missing");
  ROCFM_REQUIRE(p.mode == 1 ? p.dense_grad != nullptr : p.emb != nullptr, "merge_range: missing outputs");
  switch (p.Kp / 4) {
#define ROCFM_KP4(N)                 \
  case N:                            \
    launch_range_t<N>(p, d, stream); \
    break;
    ROCFM_KP4(1) ROCFM_KP4(2) ROCFM_KP4(3) ROCFM_KP4(4) ROCFM_KP4(5) ROCFM_KP4(6) ROCFM_KP4(7) ROCFM_KP4(8)
    ROCFM_KP4(9) ROCFM_KP4(10) ROCFM_KP4(11) ROCFM_KP4(12) ROCFM_KP4(13) ROCFM_KP4(14) ROCFM_KP4(15) ROCFM_KP4(16)
#undef ROCFM_KP4
    default:
      throw std::invalid_argument("merge_range: unsupported Kp");
  }
  ROCFM_HIP_CHECK(hipGetLastError());
}

void launch_merge_apply(const MergeParams& p, hipStream_t stream) {
  check(p);
  if (p.cap <= 0) return;
  ROCFM_REQUIRE(p.mode == 1 ? p.dense_grad != nullptr : (p.emb != nullptr && p.step != nullptr),
                "merge_apply: missing outputs");
  switch (p.Kp / 4) {
#define ROCFM_KP4(N)               \
  case N:                          \
    launch_apply_t<N>(p, stream);  \
    break;
    ROCFM_KP4(1) ROCFM_KP4(2) ROCFM_KP4(3) ROCFM_KP4(4) ROCFM_KP4(5) ROCFM_KP4(6) ROCFM_KP4(7) ROCFM_KP4(8)
    ROCFM_KP4(9) ROCFM_KP4(10) ROCFM_KP4(11) ROCFM_KP4(12) ROCFM_KP4(13) ROCFM_KP4(14) ROCFM_KP4(15) ROCFM_KP4(16)
#undef ROCFM_KP4
    default:
      throw std::invalid_argument("merge: unsupported Kp");
  }
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
