// Device body of the MLP weight-gradient kernel (mlp_wgrad.hip; also fused into step_tail.hip).
#pragma once
#include "deepfm_rows.h"

#include <cstdlib>
#include <cstring>

namespace rocfm {

namespace {

// A gradient of the flat dense buffer: the local grads buffer, or (fused DP push) this rank's slot
// in every receive buffer — the MLP gradients lead each slot, as they lead the send buffer.
template <bool PUSH>
__device__ __forceinline__ void put_grad(const WgradParams& p, int idx, float g) {
  if (PUSH && p.push.W > 0) {
    for (int d = 0; d < p.push.W; ++d) p.push.slot[d][idx] = g;
    if (p.push_mirror) p.grads[idx] = g;
  } else {
    p.grads[idx] = g;
  }
}

template <bool PUSH>
__device__ __forceinline__ void emit(const WgradParams& p, const OptStep& st, int idx, float g) {
  if (p.fuse_opt) {
    float w = p.params[idx], a = p.s0 ? p.s0[idx] : 0.f, b = p.s1 ? p.s1[idx] : 0.f;
    opt_apply(p.opt, st, w, g, a, b);
    p.params[idx] = w;
    if (p.s0) p.s0[idx] = a;
    if (p.s1) p.s1[idx] = b;
  } else {
    put_grad<PUSH>(p, idx, g);
  }
}

__device__ __forceinline__ float sum_bf16x8(uint4 v) {
  return bf2f(v.x & 0xffff) + bf2f(v.x >> 16) + bf2f(v.y & 0xffff) + bf2f(v.y >> 16) + bf2f(v.z & 0xffff) +
         bf2f(v.z >> 16) + bf2f(v.w & 0xffff) + bf2f(v.w >> 16);
}
__device__ __forceinline__ float dot_bf16x8_f32(uint4 v, const float* g) {
  return bf2f(v.x & 0xffff) * g[0] + bf2f(v.x >> 16) * g[1] + bf2f(v.y & 0xffff) * g[2] + bf2f(v.y >> 16) * g[3] +
         bf2f(v.z & 0xffff) * g[4] + bf2f(v.z >> 16) * g[5] + bf2f(v.w & 0xffff) * g[6] + bf2f(v.w >> 16) * g[7];
}

// one f32 → fp8-e4m3 byte (saturating: a delayed scale can be exceeded by the new weights)
__device__ __forceinline__ uint8_t fp8_e4m3(float x) {
  x = fminf(fmaxf(x, -kFp8Max), kFp8Max);
  return (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(x, 0.f, 0, false) & 0xff);
}

// The fp8 input-layer refresh (deepfm_rows.h Fp8W0) of this thread's weights: quantise with the
// delayed scale and publish the de-scale; returns the wave's max |w| of the new weights (the caller
// reduces it over the workgroup and adds it with ONE atomic max — hundreds of waves' atomics on one
// address serialise in L2: +2.8 µs on the step tail; max is order-independent, so the result is
// deterministic).  `N` weights (i, o, w) per thread; every lane of the wave must call it (shuffles).
template <int N>
__device__ __forceinline__ float fp8_refresh(const Fp8W0& q8, int64_t step, int Din, int Dout, const int* ii,
                                             const int* oo, const float* w, const bool* valid, bool publish) {
  const float src = fmaxf(q8.amax[step & 1], 1e-30f);
  const float qs = kFp8Max / src;
  float m = 0.f;
#pragma unroll
  for (int e = 0; e < N; ++e) {
    if (!valid[e]) continue;
    const uint8_t v = fp8_e4m3(w[e] * qs);
    q8.f[frag_swz(oo[e], ii[e], Din)] = v;
    q8.b[frag_swz(ii[e], oo[e], Dout)] = v;
    m = fmaxf(m, fabsf(w[e]));
  }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) m = fmaxf(m, __shfl_xor(m, d, 64));
  if (publish) *q8.inv_scale = src / kFp8Max;
  return m;
}

}  // namespace

constexpr int kWgThreads = 512;  // 8 waves

// One weight-gradient tile of layer li: 32 input rows × TW·32 output columns, dW = actᵀ·dz over the
// batch.  TW subtiles of 32×32; the 8 waves split the batch 8/TW ways per subtile (wave w → subtile
// w % TW, batch part w / TW), reduce through LDS, then the fused optimizer / gradient store.
// TW > 1 (wide tiles, WgradParams::tw) cuts the workgroup count TW-fold for wide layers, so the
// step tail's wgrad + embedding roles stay within one dispatch round on 256 CUs (the reference's
// flag defaults, 1248 → 256: 312 32×32 tiles).
template <bool PUSH, int TW>
__device__ __forceinline__ void wgrad_tile(const WgradParams& p, const OptStep& st, const int bid, const int li,
                                           const bool push, const PushSeen& push_seen, float* s_red, float* s_m8) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int Bp = p.Bp;
  const int Din = p.dims[li], Dout = p.dims[li + 1];
  const int local = bid - p.tile_start[li];
  const int nto = Dout / (32 * TW);
  const int ti = local / nto, to = local % nto;
  const int sub = wave % TW, part = wave / TW;
  const int oc = (to * TW + sub) * 32;  // this wave's 32 output columns
  // fragment-swizzled operands (common.h act_swz): the k-step at batch b is the contiguous 1 KiB
  // block (tile, b / 16), lane l's 8 elements at 8·l — one coalesced read per wave
  const uint16_t* A = p.actT[li] + act_swz(ti * 32, 0, Bp) + 8 * lane;
  const uint16_t* Bm = p.dzT[li + 1] + act_swz(oc, 0, Bp) + 8 * lane;
  const int q = Bp * TW / 8;  // batch share per wave (Bp % 128 == 0 → a multiple of 16)
  f32x16 acc = {};
  const int bs = part * q, be = bs + q;
  const bf16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int b0 = bs; b0 < be; b0 += 16 * 8) {  // 8 k-steps of loads in flight per batch
    bf16x8 fa[8], fb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int b = max(bs, min(b0 + 16 * u, be - 16));
      fa[u] = *reinterpret_cast<const bf16x8*>(A + (size_t)b * 32);  // block b / 16 = 512 elements
      fb[u] = *reinterpret_cast<const bf16x8*>(Bm + (size_t)b * 32);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (b0 + 16 * u >= be) fa[u] = zero;
      acc = mfma32x32x16(fa[u], fb[u], acc);
    }
  }
  // every wave parks its partial tile in LDS; then all 512 threads own 2·TW tile elements each
#pragma unroll
  for (int r = 0; r < 16; ++r) s_red[(wave * 16 + r) * 64 + lane] = acc[r];
  __syncthreads();
  ROCFM_STAMP(p.stamps, 1);
  constexpr int NE = 2 * TW;
  float g[NE], w[NE], a[NE], b[NE];
  int idx[NE], ii[NE], oo[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const int el = t + kWgThreads * e, s = el >> 10, r = (el >> 6) & 15, ln = el & 63;
    float v = 0.f;
#pragma unroll
    for (int h = 0; h < 8 / TW; ++h) v += s_red[((h * TW + s) * 16 + r) * 64 + ln];  // fixed order
    g[e] = v * p.grad_scale;
    ii[e] = ti * 32 + (r & 3) + 8 * (r >> 2) + 4 * (ln >> 5);
    oo[e] = (to * TW + s) * 32 + (ln & 31);
    idx[e] = p.offW[li] + ii[e] * Dout + oo[e];
  }
  if (!p.fuse_opt) {
    if (push) push_wait_ready(p.push, push_seen);
#pragma unroll
    for (int e = 0; e < NE; ++e) put_grad<PUSH>(p, idx[e], g[e]);
    if (push) push_drain();
    return;
  }
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    w[e] = p.params[idx[e]];
    a[e] = p.s0 ? p.s0[idx[e]] : 0.f;
    b[e] = p.s1 ? p.s1[idx[e]] : 0.f;
  }
  __syncthreads();  // s_red is reused below as the transposed bf16 tiles [TW][32][34]
  uint16_t* s_T = reinterpret_cast<uint16_t*>(s_red);
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    opt_apply(p.opt, st, w[e], g[e], a[e], b[e]);
    p.params[idx[e]] = w[e];
    if (p.s0) p.s0[idx[e]] = a[e];
    if (p.s1) p.s1[idx[e]] = b[e];
    const int el = t + kWgThreads * e;
    s_T[(el >> 10) * (32 * 34) + (oo[e] & 31) * 34 + (ii[e] & 31)] = f2bf(w[e]);
  }
  const bool q8 = li == 0 && p.w8.f;
  if (q8) {
    bool ok[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) ok[e] = true;
    const float m = fp8_refresh<NE>(p.w8, p.step ? *p.step : 0, Din, Dout, ii, oo, w, ok, bid == 0 && t == 0);
    if (lane == 0) s_m8[wave] = m;
  }
  __syncthreads();
  if (q8 && p.w8.track && t == 0) {  // one atomic per workgroup
    float m = 0.f;
#pragma unroll
    for (int ww = 0; ww < kWgThreads / 64; ++ww) m = fmaxf(m, s_m8[ww]);
    atomicMax(reinterpret_cast<unsigned*>(p.w8.amax + (((p.step ? *p.step : 0) + 1) & 1)), __float_as_uint(m));
  }
  // the bf16 weight copies of the refreshed tile, from the LDS tile T[o][i] (stride 34): every store
  // is a coalesced 4-B (row-major copies, 64-B runs) or 16-B (swizzled copies: a 32×32 tile is two
  // contiguous 1 KiB fragment blocks in each) piece — per-element 2-B stores cost an epilogue ∝ TW
#pragma unroll
  for (int s = 0; s < TW; ++s) {
    const uint16_t* T = s_T + s * (32 * 34);
    const int o0 = (to * TW + s) * 32, i0 = ti * 32;
    {  // Wᵀ rows (o-major) and W rows (i-major), 4 B per thread
      const int r = t >> 4, cp = (t & 15) * 2;
      const uint32_t wt = (uint32_t)T[r * 34 + cp] | ((uint32_t)T[r * 34 + cp + 1] << 16);
      *reinterpret_cast<uint32_t*>(p.WT[li] + (size_t)(o0 + r) * Din + i0 + cp) = wt;
      const uint32_t wb = (uint32_t)T[cp * 34 + r] | ((uint32_t)T[(cp + 1) * 34 + r] << 16);
      *reinterpret_cast<uint32_t*>(p.Wb[li] + (size_t)(i0 + r) * Dout + o0 + cp) = wb;
    }
    if (p.WTs[li] && t < 256) {  // frag_swz copies: 2 blocks × 64 lanes × 8 elements each
      const int ln = t & 63, blk = (t >> 6) & 1, which = t >> 7;  // which 0: WTs, 1: Wbs
      const int r16 = ln & 15, c8 = 8 * (ln >> 4);
      uint32_t q[4];
      if (which == 0) {  // WTs [Dout][Din]: row o = o0 + 16·blk + r16, columns i0 + c8 .. +7
        const uint16_t* src = T + (16 * blk + r16) * 34 + c8;
#pragma unroll
        for (int j = 0; j < 4; ++j) q[j] = (uint32_t)src[2 * j] | ((uint32_t)src[2 * j + 1] << 16);
        *reinterpret_cast<uint4*>(p.WTs[li] + frag_swz(o0 + 16 * blk + r16, i0 + c8, Din)) =
            make_uint4(q[0], q[1], q[2], q[3]);
      } else {  // Wbs [Din][Dout]: row i = i0 + 16·blk + r16, columns o0 + c8 .. +7
        const int ir = 16 * blk + r16;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          q[j] = (uint32_t)T[(c8 + 2 * j) * 34 + ir] | ((uint32_t)T[(c8 + 2 * j + 1) * 34 + ir] << 16);
        *reinterpret_cast<uint4*>(p.Wbs[li] + frag_swz(i0 + ir, o0 + c8, Dout)) = make_uint4(q[0], q[1], q[2], q[3]);
      }
    }
  }
  ROCFM_STAMP(p.stamps, 2);
}

// PUSH: the fused DP push variant (gradients into the W receive slots, fuse_opt == 0); a
// compile-time switch so single-GPU tails keep their code unchanged.
template <bool PUSH = false>
__device__ __forceinline__ void wgrad_body(const WgradParams& p, const int bid) {
  __shared__ __attribute__((aligned(16))) float s_red[(kWgThreads / 64) * 16 * 64];
  __shared__ float s_m8[kWgThreads / 64];  // fp8 refresh: per-wave max |w|
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int n_tiles = p.tile_start[p.nl], n_bias = p.bias_start[p.nl];
  const OptStep st = opt_step(p.opt, p.step ? *p.step : 0);
  const int Bp = p.Bp;
  // fused DP push: the peers' "entered" flags are read now, long before the stores that need them
  const bool push = PUSH && !p.fuse_opt && p.push.W > 0;
  PushSeen push_seen{};
  if (PUSH && p.push.W > 0) push_seen = push_ready_load(p.push);  // (the tail's other role may be the pusher)
  ROCFM_STAMP(p.stamps, 0);

  if (bid < n_tiles) {
    int li = 0;
    while (bid >= p.tile_start[li + 1]) ++li;
    if (p.tw[li] == 4)
      wgrad_tile<PUSH, 4>(p, st, bid, li, push, push_seen, s_red, s_m8);
    else if (p.tw[li] == 2)
      wgrad_tile<PUSH, 2>(p, st, bid, li, push, push_seen, s_red, s_m8);
    else
      wgrad_tile<PUSH, 1>(p, st, bid, li, push, push_seen, s_red, s_m8);
    return;
  }
  // column reductions over the batch: 16 threads per column, 8 chunks (64 rows) in flight each
  const int sub = t & 15;
  if (bid < n_tiles + n_bias) {  // bias gradients: Σ_b dz[o][b] for 32 columns
    const int lb = bid - n_tiles;
    int li = 0;
    while (lb >= p.bias_start[li + 1]) ++li;
    const int cb = lb - p.bias_start[li];
    const int o = cb * 32 + (t >> 4);
    const uint16_t* dz = p.dzT[li + 1];
    float s = 0.f;
    for (int b0 = sub * 8; b0 < Bp; b0 += 128 * 8) {
      uint4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const uint4*>(dz + act_swz(o, min(b0 + 128 * u, Bp - 8), Bp));
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (b0 + 128 * u < Bp) s += sum_bf16x8(v[u]);
    }
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) s += __shfl_xor(s, d, 64);
    if (push) push_wait_ready(p.push, push_seen);
    if (sub == 0) emit<PUSH>(p, st, p.offb[li] + o, s * p.grad_scale);
    if (push) push_drain();
    return;
  }
  // output layer: dW_out[c] = Σ_b h[c][b]·g[b]; d b_out = d fm_bias = Σ_b g[b]
  {
    const int Dn = p.dims[p.nl];
    const uint16_t* H = p.actT[p.nl];
    if (push) push_wait_ready(p.push, push_seen);
    for (int c0 = 0; c0 < Dn; c0 += 32) {
      const int c = min(c0 + (t >> 4), Dn - 1);
      float s = 0.f;
      for (int b0 = sub * 8; b0 < Bp; b0 += 128 * 8) {
        uint4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const uint4*>(H + act_swz(c, min(b0 + 128 * u, Bp - 8), Bp));
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (b0 + 128 * u < Bp) s += dot_bf16x8_f32(v[u], p.g + b0 + 128 * u);
      }
#pragma unroll
      for (int d = 1; d < 16; d <<= 1) s += __shfl_xor(s, d, 64);
      if (sub == 0 && c0 + (t >> 4) < Dn) emit<PUSH>(p, st, p.off_wout + c, s * p.grad_scale);
    }
    float s = 0.f;
    for (int b = t; b < Bp; b += kWgThreads) s += p.g[b];
    s = wave_sum(s);
    if (lane == 0) s_red[wave] = s;
    __syncthreads();
    if (t == 0) {
      float tot = 0.f;
      for (int w = 0; w < kWgThreads / 64; ++w) tot += s_red[w];
      tot *= p.grad_scale;
      emit<PUSH>(p, st, p.off_bout, tot);
      emit<PUSH>(p, st, p.off_fmb, tot);
    }
    if (p.bn) {  // batch_norm γ / β: column sums already reduced over the batch by deepfm_rows
      for (int l = 0; l < p.nl; ++l)
        for (int c = t; c < p.dims[l + 1]; c += kWgThreads) {
          emit<PUSH>(p, st, p.off_gamma[l] + c, p.bn_grad[(size_t)(2 * l) * p.bn_dmax + c] * p.grad_scale);
          emit<PUSH>(p, st, p.off_beta[l] + c, p.bn_grad[(size_t)(2 * l + 1) * p.bn_dmax + c] * p.grad_scale);
        }
    }
    if (push) push_drain();
  }
}


// Elementwise optimizer over the flat dense buffer (+ bf16 / swizzled weight refresh), block `bid`
// of `nblocks` 256-thread blocks (grid-strided).
template <int TPB = 256>
__device__ __forceinline__ void dense_apply_body(const DenseApplyParams& p, const int bid, const int nblocks) {
  const OptStep st = opt_step(p.opt, p.step ? *p.step : 0);
  const bool q8 = p.w8.f != nullptr && p.nl > 0;
  const int64_t s8 = p.step ? *p.step : 0;
  const float q8s = q8 ? kFp8Max / fmaxf(p.w8.amax[s8 & 1], 1e-30f) : 0.f;
  float q8m = 0.f;  // max |w| of the layer-0 weights this thread refreshed
  for (int idx = bid * TPB + (int)threadIdx.x; idx < p.n; idx += nblocks * TPB) {
    float w = p.params[idx];
    if (p.apply) {
      float a = p.s0 ? p.s0[idx] : 0.f, b = p.s1 ? p.s1[idx] : 0.f;
      float g = p.grads[idx];
      for (int r = 1; r < p.nseg; ++r) g += p.grads[(size_t)r * p.seg_stride + idx];  // rank order
      opt_apply(p.opt, st, w, g * p.grad_scale, a, b);
      p.params[idx] = w;
      if (p.s0) p.s0[idx] = a;
      if (p.s1) p.s1[idx] = b;
    }
    for (int l = 0; l < p.nl; ++l) {
      const int sz = p.dims[l] * p.dims[l + 1];
      if (idx >= p.offW[l] && idx < p.offW[l] + sz) {
        const int k = idx - p.offW[l];
        const int i = k / p.dims[l + 1], o = k % p.dims[l + 1];
        const uint16_t h = f2bf(w);
        p.WT[l][(size_t)o * p.dims[l] + i] = h;
        p.Wb[l][(size_t)i * p.dims[l + 1] + o] = h;
        if (p.WTs[l]) {
          p.WTs[l][frag_swz(o, i, p.dims[l])] = h;
          p.Wbs[l][frag_swz(i, o, p.dims[l + 1])] = h;
        }
        if (l == 0 && q8) {
          const uint8_t v = fp8_e4m3(w * q8s);
          p.w8.f[frag_swz(o, i, p.dims[0])] = v;
          p.w8.b[frag_swz(i, o, p.dims[1])] = v;
          q8m = fmaxf(q8m, fabsf(w));
          if (k == 0) *p.w8.inv_scale = 1.f / q8s;
        }
      }
    }
  }
  if (q8 && p.w8.track) {  // (every thread of the block reaches this point) one atomic per block
    __shared__ float s_q8[TPB / 64];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) q8m = fmaxf(q8m, __shfl_xor(q8m, d, 64));
    if ((threadIdx.x & 63) == 0) s_q8[threadIdx.x >> 6] = q8m;
    __syncthreads();
    if (threadIdx.x == 0) {
      float m = 0.f;
#pragma unroll
      for (int w = 0; w < TPB / 64; ++w) m = fmaxf(m, s_q8[w]);
      if (m > 0.f) atomicMax(reinterpret_cast<unsigned*>(p.w8.amax + ((s8 + 1) & 1)), __float_as_uint(m));
    }
  }
}


// Fills the per-layer tile / bias workgroup offsets; returns the grid size.
// ``co_resident`` ≥ 0 (step tail, ROCFM_WGRAD_TW=auto): workgroups of the launch's other role; the
// tile widths are widened (WgradParams::tw, largest layers first, up to 4 subtiles) until tiles +
// bias blocks + 1 + the other role fit ``max_wg`` (one dispatch round).  Measured no faster at the
// reference's k = 32 shapes (profiles/r4_k32_tail_ab.md), so the step tail keeps 32×32 tiles
// unless asked; ROCFM_WGRAD_TW=2|4 forces a width.  < 0: plain 32×32 tiles.
inline int wgrad_prepare(WgradParams& p, int co_resident = -1, int max_wg = 256) {
  ROCFM_REQUIRE(p.Bp % 128 == 0, "mlp_wgrad: Bp must be a multiple of 128");
  for (int l = 0; l < kMaxHidden; ++l) p.tw[l] = 1;
  auto fill = [&p] {
    p.tile_start[0] = 0;
    p.bias_start[0] = 0;
    for (int l = 0; l < p.nl; ++l) {
      ROCFM_REQUIRE(p.dims[l] % 32 == 0 && p.dims[l + 1] % 32 == 0, "mlp_wgrad: dims must be padded to 32");
      p.tile_start[l + 1] = p.tile_start[l] + (p.dims[l] / 32) * (p.dims[l + 1] / (32 * p.tw[l]));
      p.bias_start[l + 1] = p.bias_start[l] + p.dims[l + 1] / 32;
    }
    for (int l = p.nl + 1; l <= kMaxHidden; ++l) {
      p.tile_start[l] = p.tile_start[p.nl];
      p.bias_start[l] = p.bias_start[p.nl];
    }
    return p.tile_start[p.nl] + p.bias_start[p.nl] + 1;
  };
  int n = fill();
  if (co_resident < 0) return n;
  // ROCFM_WGRAD_TW: unset = widen automatically up to 32 × 64 tiles (the default: the reference's
  // k = 32 shapes measured 57.4 → 55.0 µs and 44.1 → 43.3 µs per step with it, the 32 × 128 tiles
  // of `auto` lost, profiles/r5_wgrad_swizzle.md); auto = up to 32 × 128; 2 | 4 = that width on
  // every layer it divides
  const char* env = getenv("ROCFM_WGRAD_TW");
  const int forced = env ? atoi(env) : 0;
  if (forced == 2 || forced == 4) {
    for (int l = 0; l < p.nl; ++l)
      if (p.dims[l + 1] % (32 * forced) == 0) p.tw[l] = forced;
    return fill();
  }
  const int tw_max = (env && std::strcmp(env, "auto") == 0) ? 4 : 2;
  while (n + co_resident > max_wg) {  // widen the layer with the most tiles that can still widen
    int best = -1, bt = 0;
    for (int l = 0; l < p.nl; ++l) {
      const int nt = p.tile_start[l + 1] - p.tile_start[l];
      if (p.tw[l] < tw_max && p.dims[l + 1] % (64 * p.tw[l]) == 0 && nt > bt) {
        best = l;
        bt = nt;
      }
    }
    if (best < 0) break;
    p.tw[best] *= 2;
    n = fill();
  }
  return n;
}

}  // namespace rocfm
