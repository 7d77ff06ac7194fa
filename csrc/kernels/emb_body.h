// Device body of the embedding-row update (emb_update.hip; also fused into step_tail.hip).
// See emb_update.hip for the algorithm.  kE ≤ kChunk sorted entries per workgroup of kChunk threads.
#pragma once
#include "emb_update.h"

namespace rocfm {

namespace {

constexpr int kEmbChunk = 256;

__device__ __forceinline__ const float4* contrib_row4(const EmbUpdateParams& p, uint32_t j) {
  const float* r = (p.contrib_seg > 0) ? p.contrib + (size_t)(j / (uint32_t)p.contrib_seg) * p.contrib_seg_stride +
                                             (size_t)(j % (uint32_t)p.contrib_seg) * p.Kp
                                       : p.contrib + (size_t)j * p.Kp;
  return reinterpret_cast<const float4*>(r);
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 f4shfl_up(float4 v, int d) {
  return make_float4(__shfl_up(v.x, d, 64), __shfl_up(v.y, d, 64), __shfl_up(v.z, d, 64), __shfl_up(v.w, d, 64));
}
__device__ __forceinline__ float4 f4shfl_xor(float4 v, int d) {
  return make_float4(__shfl_xor(v.x, d, 64), __shfl_xor(v.y, d, 64), __shfl_xor(v.z, d, 64), __shfl_xor(v.w, d, 64));
}

// DPP lane moves (VALU, no LDS traffic; __shfl_* compile to ds_bpermute, which shares the LDS
// pipe with the chunk's row staging).
// v += take · dpp(v) as ONE v_fmac_f32_dpp per float (m = take ? 1 : 0): the same bits as
// v + (take ? x : 0) for finite x (x·1 = x exactly, x·0 = ±0 and v ± 0 = v; only a −0 run sum can
// come out +0 instead).  Written out because the compiler keeps a separate v_mov_b32_dpp and packs
// the fmas into v_pk_fma_f32 (no DPP form); the leading s_nop 1 is the two wait states a DPP read
// needs after a VALU write of its source (the hazard recognizer does not see into inline asm).
// Rows outside ROW_MASK are not written (v unchanged); bound_ctrl zero-fills sources outside the row.
#define ROCFM_FMAC_DPP4(v, m, MOD)                                                                 \
  asm volatile("s_nop 1\n\t"                                                                      \
               "v_fmac_f32_dpp %0, %0, %4 " MOD "\n\t"                                            \
               "v_fmac_f32_dpp %1, %1, %4 " MOD "\n\t"                                            \
               "v_fmac_f32_dpp %2, %2, %4 " MOD "\n\t"                                            \
               "v_fmac_f32_dpp %3, %3, %4 " MOD                                                    \
               : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)                                         \
               : "v"(m))

// Inclusive segmented scan over the 64 lanes: v[lane] = Σ v[seg .. lane] (seg = the first lane of
// this lane's segment, ≤ lane).  Rows of 16 lanes first (row_shr 1, 2, 4, 8), then row 0's last
// lane into row 1 and row 2's into row 3 (row_bcast:15), then lane 31 into rows 2-3
// (row_bcast:31) — each step only where the segment reaches back that far.  seg = 0 everywhere:
// lane 63 holds the wave's total.
template <int N>
__device__ __forceinline__ void seg_scan_dpp(float4 (&v)[N], int lane, int seg) {
  const int rl = lane & 15, row = lane >> 4;
  const bool t1 = rl >= 1 && lane - 1 >= seg, t2 = rl >= 2 && lane - 2 >= seg;
  const bool t4 = rl >= 4 && lane - 4 >= seg, t8 = rl >= 8 && lane - 8 >= seg;
  const bool t15 = (row & 1) && seg < (lane & ~15), t31 = row >= 2 && seg <= 31;
  const float m1 = t1 ? 1.f : 0.f, m2 = t2 ? 1.f : 0.f, m4 = t4 ? 1.f : 0.f, m8 = t8 ? 1.f : 0.f;
  const float m15 = t15 ? 1.f : 0.f, m31 = t31 ? 1.f : 0.f;
#pragma unroll
  for (int u = 0; u < N; ++u) ROCFM_FMAC_DPP4(v[u], m1, "row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1");
#pragma unroll
  for (int u = 0; u < N; ++u) ROCFM_FMAC_DPP4(v[u], m2, "row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1");
#pragma unroll
  for (int u = 0; u < N; ++u) ROCFM_FMAC_DPP4(v[u], m4, "row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1");
#pragma unroll
  for (int u = 0; u < N; ++u) ROCFM_FMAC_DPP4(v[u], m8, "row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1");
#pragma unroll
  for (int u = 0; u < N; ++u) ROCFM_FMAC_DPP4(v[u], m15, "row_bcast:15 row_mask:0xa bank_mask:0xf");
#pragma unroll
  for (int u = 0; u < N; ++u) ROCFM_FMAC_DPP4(v[u], m31, "row_bcast:31 row_mask:0xc bank_mask:0xf");
}

}  // namespace

// One workgroup per 256 consecutive sorted entries.  Every thread loads ONE entry's gradient row
// (Kp floats, float4 loads) into LDS, so the chunk's rows arrive in one memory latency; run pieces
// are summed by a wave-level segmented scan (shfl_up, fixed order); each run owned by the chunk
// (its first entry lies here) adds its ≤4 wave pieces and, for the chunk's last run, the
// continuation chunks; then one 16-lane group per run applies the optimizer to the table row.
// PUSH: the fused DP push variant (mode 2 with p.push set); a compile-time switch so the other
// launches keep their memory-op stream (and waitcnt placement) free of the push's branches.
// kE < kChunk (the fused tail: 256 entries on 512 threads): twice the workgroups for the same
// entries, so a chunk's run heads — its optimizer items, the scattered table / slot round trip
// that bounds the slowest chunks — are spread over twice the CUs; the threads past kE load no
// entry but take part in the end search, the continuation rounds and the optimizer items.
template <int KP4, int kChunk, bool BT = false, bool PUSH = false, int kE = kChunk>
__device__ __forceinline__ void emb_rows_body(const EmbUpdateParams& p, const int bid) {
  constexpr int kWaves = kChunk / 64;
  __shared__ float4 s_rows[kE * KP4];  // the chunk's entries only (threads past kE hold none): with the
                                       // fused tail's kE = 256 two 512-thread workgroups fit a CU at Kp = 36
  __shared__ float4 s_cont[2 * kWaves * KP4];  // continuation: one round's window pieces, then the fold
  __shared__ int s_head[kChunk + 1];
  __shared__ uint32_t s_hkey[kChunk + 1];
  __shared__ uint32_t s_hprev[kChunk + 1];  // sorted export directory: key of the entry before each head
  __shared__ int s_total;
  __shared__ int s_wcnt[kWaves];
  __shared__ int s_nh, s_last_end, s_out_base;
  __shared__ int s_hb[2 * kWaves];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  static_assert(kE <= kChunk && kE % 64 == 0, "entries per chunk");
  const int n = p.n_dev ? *p.n_dev : p.n;  // (dedup: the compacted list's length, ≤ p.n)
  const int c0 = bid * kE;
  if (c0 >= n) return;  // grid sized for p.n
  const int cend = min(c0 + kE, n);
  // kSplit (the fused tail: 256 entries on 512 threads): both halves of the workgroup hold the
  // chunk's 256 entries, each the float4 columns of its half of the row — half the row loads and
  // half the segmented scan per thread (k = 32: 5 + 4 of 9 float4); heads are compacted by half 0
  constexpr bool kSplit = 2 * kE == kChunk && KP4 >= 2;
  constexpr int KH = kSplit ? (KP4 + 1) / 2 : KP4;  // float4 columns per thread in steps 1-2
  const int te = kSplit ? t % kE : t, half = kSplit ? t / kE : 0;
  const int i = c0 + te;
  const bool live_e = te < kE && i < n;     // this thread's slot holds one of the chunk's entries
  const bool live = live_e && half == 0;    // … and this thread represents it in the compaction
  const OptStep st = opt_step(p.opt, p.step ? *p.step : 0);
  const int ce_pre = (p.chunk_end != nullptr && t == 0) ? p.chunk_end[bid] : 0;  // issued with the keys
  // fused DP push (mode 2): the peers' "entered" flags, read with the keys, checked before the stores
  const bool push = PUSH && p.push.W > 0 && (p.mode == 2 || (p.mode == 1 && p.push_seg > 0));
  PushSeen push_seen{};
  if (PUSH && p.push.W > 0) push_seen = push_ready_load(p.push);  // (the tail's other role may be the pusher)
  // sorted export (mode 2 + chunk_heads): this chunk's output base and the batch's total, from the
  // side chain's per-chunk head counts (loaded with the keys; reduced below with the head compaction)
  int hb_before = 0, hb_total = 0;
  if (p.mode == 2 && p.chunk_heads != nullptr) {
    for (int c = t; c < p.nch; c += kChunk) {
      const int h = p.chunk_heads[c];
      hb_total += h;
      hb_before += c < bid ? h : 0;
    }
  }
  ROCFM_STAMP(p.stamps, 0);

  // 1. keys, run heads, and every entry's gradient row (one latency for the whole chunk)
  uint32_t key = 0xffffffffu, prevk = 0xffffffffu;
  bool head = false;
  float4 v[KH];
  if (live_e) {
    key = p.skeys[i];
    if (i > 0) prevk = p.skeys[i - 1];
    head = (i == 0) || (prevk != key);
    const bool skip = p.max_key && key >= p.max_key;
    const float4* src = p.sorted_contrib ? reinterpret_cast<const float4*>(p.contrib + (size_t)i * p.Kp)
                                         : contrib_row4(p, p.svals[i] - p.val_base);
#pragma unroll
    for (int u = 0; u < KH; ++u) {
      const int c = half * KH + u;
      const float4 x = src[min(c, KP4 - 1)];
      v[u] = (skip || c >= KP4) ? make_float4(0.f, 0.f, 0.f, 0.f) : x;
    }
  } else {
#pragma unroll
    for (int u = 0; u < KH; ++u) v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // 2. wave-level segmented inclusive scan (segments: runs, cut at wave boundaries)
  {
    const unsigned long long hm = __ballot(head || lane == 0 || !live_e);
    const unsigned long long below = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
    const int seg = 63 - __clzll(hm & below);
    seg_scan_dpp(v, lane, seg);
    if (te < kE) {  // (wave-uniform: kE is a multiple of 64)
#pragma unroll
      for (int u = 0; u < KH; ++u) {
        const int c = half * KH + u;
        if (c < KP4) s_rows[te * KP4 + c] = v[u];
      }
    }
  }
  // 3. compact the heads in order (one representative thread per entry: half 0)
  if (!live) head = false;
  const unsigned long long m = __ballot(head);
  const int before = __popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) s_wcnt[wave] = __popcll(m);
  const bool sorted_out = p.mode == 2 && p.chunk_heads != nullptr;
  if (sorted_out) {
    hb_before = wave_sum_i(hb_before);
    hb_total = wave_sum_i(hb_total);
    if (lane == 0) {
      s_hb[wave] = hb_before;
      s_hb[kWaves + wave] = hb_total;
    }
  }
  __syncthreads();
  if (sorted_out && t == 0) {
    int b = 0, tot = 0;
    for (int w = 0; w < kWaves; ++w) {
      b += s_hb[w];
      tot += s_hb[kWaves + w];
    }
    s_out_base = b;
    s_total = tot;
    if (bid == 0) *p.out_count = tot;
  }
  {
    int base = 0;
    for (int w = 0; w < wave; ++w) base += s_wcnt[w];
    if (head) {
      s_head[base + before] = i;
      s_hkey[base + before] = key;
      s_hprev[base + before] = i > 0 ? prevk : 0xffffffffu;
    }
  }
  if (t == 0) {
    int tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) tot += s_wcnt[w];
    s_nh = tot;
  }
  __syncthreads();
  ROCFM_STAMP(p.stamps, 1);
  const int nh = s_nh;
  if (nh == 0) return;
  // 4. end of the last run (all 256 threads probe 256 entries per round); mode 2 reserves slots
  {
    const uint32_t lk = s_hkey[nh - 1];
    const bool sentinel = p.max_key && lk >= p.max_key;  // sentinel padding sorts last: runs to n
    int pos = sentinel ? n : cend;
    if (t == 0) s_last_end = n;
    if (p.chunk_end != nullptr && !sentinel) {  // precomputed by the side chain (sort_aux)
      pos = n;
      if (t == 0) s_last_end = ce_pre;
    }
    __syncthreads();
    while (pos < n) {
      const int j = pos + t;
      const bool diff = (j >= n) || (p.skeys[j] != lk);
      const unsigned long long dm = __ballot(diff);
      if (lane == 0) s_wcnt[wave] = dm ? (__ffsll((long long)dm) - 1) : 64;
      __syncthreads();
      int found = -1;
      for (int w = 0; w < kWaves; ++w)
        if (s_wcnt[w] < 64) {
          found = pos + 64 * w + s_wcnt[w];
          break;
        }
      __syncthreads();
      if (found >= 0) {
        if (t == 0) s_last_end = min(found, n);
        break;
      }
      pos += kChunk;
    }
    if (t == 0 && p.mode == 2 && !sorted_out) s_out_base = atomicAdd(p.out_count, nh);
  }
  __syncthreads();
  ROCFM_STAMP(p.stamps, 2);
  if (t == 0) s_head[nh] = min(s_last_end, cend);
  // 5. continuation of the last run past the chunk.  A run's sum is, everywhere, the left-to-right
  //    fold from 0 of its window pieces — the segmented scan of each 64-entry window of the sorted
  //    list (aligned to the list) at the run's last entry in that window — so the planned tail
  //    (emb_plan_body.h), which cuts the list elsewhere and combines split runs across workgroups,
  //    gets the same bits.  Threads t < KP4 hold the fold: first the run's in-chunk pieces, then
  //    every following window's piece in order (each wave scans 2 windows per round).
  const int last_end = s_last_end;
  const bool cont = last_end > cend && !(p.max_key && s_hkey[nh - 1] >= p.max_key);
  if (cont) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t < KP4) {
      const int s = s_head[nh - 1], e = s_head[nh];
      for (int ww = (s - c0) >> 6; ww <= (e - 1 - c0) >> 6; ++ww)
        acc = f4add(acc, s_rows[(min(e, c0 + 64 * (ww + 1)) - 1 - c0) * KP4 + t]);
    }
    constexpr int kNW = 2;  // windows per wave per round
    for (int w0 = cend; w0 < last_end; w0 += kNW * kChunk) {
      float4 x[kNW][KP4];
#pragma unroll
      for (int h = 0; h < kNW; ++h) {
        const int j = w0 + (h * kWaves + wave) * 64 + lane;
        if (j < last_end) {
          const float4* src = p.sorted_contrib ? reinterpret_cast<const float4*>(p.contrib + (size_t)j * p.Kp)
                                               : contrib_row4(p, p.svals[j] - p.val_base);
#pragma unroll
          for (int u = 0; u < KP4; ++u) x[h][u] = src[u];
        } else {
#pragma unroll
          for (int u = 0; u < KP4; ++u) x[h][u] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int h = 0; h < kNW; ++h) {
        seg_scan_dpp(x[h], lane, 0);
        const int ws = w0 + (h * kWaves + wave) * 64;  // this window's piece ends at the run's last entry in it
        if (ws < last_end && lane == min(63, last_end - 1 - ws)) {
#pragma unroll
          for (int u = 0; u < KP4; ++u) s_cont[(h * kWaves + wave) * KP4 + u] = x[h][u];
        }
      }
      __syncthreads();
      if (t < KP4) {
        for (int q = 0; q < kNW * kWaves && w0 + q * 64 < last_end; ++q) acc = f4add(acc, s_cont[q * KP4 + t]);
      }
      __syncthreads();
    }
    if (t < KP4) s_cont[t] = acc;  // the run's whole fold
  }
  __syncthreads();
  ROCFM_STAMP(p.stamps, 3);
  // 6. (run, float4 column group) items over all threads: add the run's wave pieces (+ the
  //    continuation), then the optimizer on a float4 of the table row; every thread issues its
  //    table/slot loads for up to 4 items before using any.
  const int nitems = nh * KP4;
  if (push) push_wait_ready(p.push, push_seen);
  for (int base = 0; base < nitems; base += kChunk * 4) {
#pragma clang fp contract(off)  // (the gradient scale and L2 terms: the same bits in every instantiation)
    float4 w[4], a[4], b[4], g[4];
    uint32_t kk[4];
    size_t idx4[4];
    // the table / slot loads of all 4 items depend only on the run's key: issued first (one LDS
    // read each), the run's gradient pieces are summed out of LDS while they are in flight
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int it = min(base + u * kChunk + t, nitems - 1);
      const int r = it / KP4, u4 = it - r * KP4;
      kk[u] = s_hkey[r];
      const bool skip = p.max_key && kk[u] >= p.max_key;
      const size_t row = skip ? 0 : (size_t)((kk[u] - (uint32_t)p.id_offset) / (uint32_t)p.id_stride);
      idx4[u] = row * KP4 + u4;
      if (p.mode == 0) {  // issue the row's parameter + slot loads now
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        w[u] = tbl_load4<BT>(p.emb, idx4[u]);
        a[u] = p.s0 ? reinterpret_cast<const float4*>(p.s0)[idx4[u]] : z;
        b[u] = p.s1 ? reinterpret_cast<const float4*>(p.s1)[idx4[u]] : z;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int it = min(base + u * kChunk + t, nitems - 1);
      const int r = it / KP4, u4 = it - r * KP4;
      const int s = s_head[r], e = s_head[r + 1];  // piece inside this chunk: [s, e)
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      if (cont && r == nh - 1) {
        acc = s_cont[u4];  // the fold of step 5
      } else {
        const int w0 = (s - c0) >> 6, w1 = (e - 1 - c0) >> 6;
        for (int ww = w0; ww <= w1; ++ww) {
          const int lastw = min(e, c0 + 64 * (ww + 1)) - 1 - c0;
          acc = f4add(acc, s_rows[lastw * KP4 + u4]);
        }
      }
      g[u] = make_float4(acc.x * p.grad_scale, acc.y * p.grad_scale, acc.z * p.grad_scale, acc.w * p.grad_scale);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int it = base + u * kChunk + t;
      if (it >= nitems) continue;
      const int r = it / KP4, u4 = it - r * KP4;
      if (p.max_key && kk[u] >= p.max_key) continue;
      if (p.mode == 2) {
        const int slot = s_out_base + r;
        if (sorted_out && p.dir_nb > 0 && u4 == 0) {  // this head opens the buckets (prev, own]
          const uint32_t row_id = (kk[u] - p.id_offset) / (uint32_t)p.id_stride;
          const int bc = (int)min(row_id / p.dir_div, (uint32_t)p.dir_nb - 1u);
          const uint32_t pk = s_hprev[r];
          const int bp = pk == 0xffffffffu ? -1
                                           : (int)min(((pk - p.id_offset) / (uint32_t)p.id_stride) / p.dir_div,
                                                      (uint32_t)p.dir_nb - 1u);
          const int b_end = (slot == s_total - 1) ? p.dir_nb : bc;  // the last head closes the directory
          for (int bb = bp + 1; bb <= b_end; ++bb) {
            const int v = bb <= bc ? slot : s_total;
            if (push) {
              for (int d = 0; d < p.push.W; ++d) reinterpret_cast<int32_t*>(p.push.slot[d] + p.push_off_dir)[bb] = v;
              if (p.push_mirror && p.out_dir) p.out_dir[bb] = v;
            } else {
              p.out_dir[bb] = v;
            }
          }
        }
        if (slot < p.out_cap) {
          const uint32_t row_id = (kk[u] - p.id_offset) / (uint32_t)p.id_stride;  // the table row id
          if (push) {  // this rank's slot in every receive buffer (xGMI stores under the tail)
            for (int d = 0; d < p.push.W; ++d) {
              float* b = p.push.slot[d];
              reinterpret_cast<float4*>(b + p.push_off_rows)[(size_t)slot * KP4 + u4] = g[u];
              if (u4 == 0) reinterpret_cast<uint32_t*>(b + p.push_off_keys)[slot] = row_id;
            }
            if (p.push_mirror) {  // the shadow exchange's local reference (DP export)
              reinterpret_cast<float4*>(p.out_rows)[(size_t)slot * KP4 + u4] = g[u];
              if (u4 == 0) p.out_keys[slot] = row_id;
            }
          } else {
            reinterpret_cast<float4*>(p.out_rows)[(size_t)slot * KP4 + u4] = g[u];  // pad columns are 0
            if (u4 == 0) p.out_keys[slot] = row_id;
          }
        }
      } else if (p.mode == 1) {
        const uint32_t rr = (uint32_t)(idx4[u] / KP4);
        if (p.hot_out != nullptr && rr >= p.hot_base) {  // replicated row → the X4 bucket
          reinterpret_cast<float4*>(p.hot_out)[(size_t)(rr - p.hot_base) * KP4 + u4] = g[u];
          if (u4 == 0) p.hot_out[(size_t)p.n_hot * KP4 * 4 + (rr - p.hot_base)] = 1.f;
          continue;
        }
        if (push) {  // row-shard X3: straight into the owner's receive slot
          const uint32_t d = rr / (uint32_t)p.push_seg, j = rr - d * (uint32_t)p.push_seg;
          reinterpret_cast<float4*>(p.push.slot[d])[(size_t)j * KP4 + u4] = g[u];
          if (p.push_mirror) reinterpret_cast<float4*>(p.dense_grad)[idx4[u]] = g[u];
          continue;
        }
        reinterpret_cast<float4*>(p.dense_grad)[idx4[u]] = g[u];
        if (p.touched && u4 == 0) p.touched[idx4[u] / KP4] = (uint32_t)*p.step + 1u;
      } else {
        float* wc = &w[u].x;
        float* ac = &a[u].x;
        float* bc = &b[u].x;
        const float* gc = &g[u].x;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (u4 * 4 + c >= p.K1) continue;  // padding columns keep their (zero) values
          opt_apply(p.opt, st, wc[c], l2_grad(gc[c], p.l2, wc[c]), ac[c], bc[c]);
        }
        tbl_store4<BT>(p.emb, idx4[u], w[u], p.step ? (uint32_t)*p.step : 0u);
        if (p.s0) reinterpret_cast<float4*>(p.s0)[idx4[u]] = a[u];
        if (p.s1) reinterpret_cast<float4*>(p.s1)[idx4[u]] = b[u];
      }
    }
  }
  if (push) push_drain();
  __syncthreads();
  ROCFM_STAMP(p.stamps, 4);
}


}  // namespace rocfm
