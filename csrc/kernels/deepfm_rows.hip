// DeepFM fused row-tile kernel: the whole per-example part of a training step in ONE launch.
//
// One 256-thread workgroup owns 16 consecutive examples (one MFMA M-tile) and runs, entirely
// out of LDS:
//   A  gather fm_v/fm_w rows (f32, 16-B vector loads) → e = V[id]·x, h0 = bf16(e)  (PS:207-213)
//   B  S = Σ_f e, y_v = ½Σ_k(S² − Σ_f e²), y_w = Σ_f w·x, y_lin = b + y_w + y_v    (PS:214-217)
//   C  hidden layers: h_{l+1} = dropout(relu(h_l·W_l + c_l)) on v_mfma_f32_16x16x32_bf16
//      (Philox keep-mask, keep = `dropout` flag value)                             (PS:234-246)
//   D  y_d = h_L·w_out + c_out, y = y_lin + y_d, p = σ(y), loss, g = dL/dy          (PS:248-276)
//   E  backward data path through the MLP (dz_l = 1[h_l>0]/keep · dh_l, dh = dz·Wᵀ)
//   F  FM backward: de = g·(S − e) + dh0, per-lookup gradient row [x·de | g·x]
// It writes bf16 activations/dz transposed ([feature][batch]) for the weight-gradient kernel
// (mlp_wgrad.hip) and the per-lookup gradient rows for the sort-based embedding update
// (emb_update.hip).  Nothing here reduces across examples, so no atomics and no inter-workgroup
// communication are needed.  Weights are read from L2 as MFMA B fragments (16 B per lane).
#include "deepfm_rows.h"

namespace rocfm {

namespace {

__device__ __forceinline__ bf16x8 ld_frag(const uint16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

__device__ __forceinline__ uint32_t pick4(const Philox4& b, int i) {
  return i == 0 ? b.x : i == 1 ? b.y : i == 2 ? b.z : b.w;
}

// acc[j] = A(16 × Kd, LDS bf16, row stride lda) · B(Kd × 16) for the n-tiles nt = nt0 + 4j (j < NTW)
// owned by this wave.  B fragments come from global/L2: tile nt, k-step ks at
// Bt + (nt*16 + (lane&15))*ldb + ks + 8*(lane>>4).  Latency-oriented: every batch issues KU k-steps
// × NTW tiles of 16-B loads before the first MFMA; out-of-range k-steps load a clamped (valid)
// address and are zeroed on the VALUE (no per-load predication — cdna guide §5 trap (c)).
template <int NTW, int KU>
__device__ __forceinline__ void rowtile_gemm(const uint16_t* A, int lda, const uint16_t* Bt, int ldb, int ntiles,
                                             int nt0, int Kd, int lane, f32x4 (&acc)[NTW]) {
#pragma unroll
  for (int j = 0; j < NTW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint16_t* ap = A + (lane & 15) * lda + 8 * (lane >> 4);
  const uint16_t* bp[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = min(nt0 + 4 * j, ntiles - 1);
    bp[j] = Bt + (size_t)(nt * 16 + (lane & 15)) * ldb + 8 * (lane >> 4);
  }
  const bf16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int k0 = 0; k0 < Kd; k0 += 32 * KU) {
    bf16x8 a[KU], b[NTW][KU];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int ks = min(k0 + 32 * u, Kd - 32);
#pragma unroll
      for (int j = 0; j < NTW; ++j) b[j][u] = ld_frag(bp[j] + ks);
    }
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int ks = min(k0 + 32 * u, Kd - 32);
      a[u] = (k0 + 32 * u < Kd) ? ld_frag(ap + ks) : zero;
    }
#pragma unroll
    for (int u = 0; u < KU; ++u)
#pragma unroll
      for (int j = 0; j < NTW; ++j)
        if (nt0 + 4 * j < ntiles) acc[j] = mfma16x16x32(a[u], b[j][u], acc[j]);
  }
}

}  // namespace

__global__ __launch_bounds__(kRowThreads) void deepfm_rows_kernel(const RowsParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const RowsLds& L = p.lds;
  int32_t* s_ids = reinterpret_cast<int32_t*>(smem + L.ids);
  float* s_vals = reinterpret_cast<float*>(smem + L.vals);
  float* s_wx = reinterpret_cast<float*>(smem + L.wx);
  float* s_S = reinterpret_cast<float*>(smem + L.S);
  float* s_ylin = reinterpret_cast<float*>(smem + L.ylin);
  float* s_g = reinterpret_cast<float*>(smem + L.g);
  float* s_f32 = reinterpret_cast<float*>(smem + L.f32);  // e (forward) / dh0 (backward), stride dims[0]

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int row0 = blockIdx.x * kRowTile;
  const int F = p.F, K = p.K, Kp = p.Kp, D0 = F * K, D0p = p.dims[0];
  const int Bp = p.Bp;
  const uint32_t step = p.step ? (uint32_t)(*p.step) : 0u;

  // ---- phase 0: stage ids / values ------------------------------------------------------------
  for (int i = t; i < kRowTile * F; i += kRowThreads) {
    const int r = i / F, gr = row0 + r;
    const bool valid = gr < p.B;
    s_ids[i] = valid ? p.ids[(size_t)row0 * F + i] : 0;
    s_vals[i] = valid ? p.vals[(size_t)row0 * F + i] : 0.f;
  }
  __syncthreads();

  // ---- phase A: gather rows, e = V·x (f32 scratch), h0 = bf16(e), w·x ---------------------------
  // Work items (row, field, float4-column) are flattened so each thread issues up to 8 independent
  // 16-B row loads before consuming any (one HBM/MALL latency for the whole tile's gather).
  {
    uint16_t* h0 = reinterpret_cast<uint16_t*>(smem + L.act[0]);
    const int lda = L.lda[0];
    const int KP4 = Kp >> 2;
    const int nitems = kRowTile * F * KP4;
    const float4* emb4 = reinterpret_cast<const float4*>(p.emb);
    for (int base = 0; base < nitems; base += kRowThreads * 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int idx = min(base + u * kRowThreads + t, nitems - 1);
        const int rf = idx / KP4, c4 = idx - rf * KP4;
        v[u] = emb4[(size_t)s_ids[rf] * KP4 + c4];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int idx = base + u * kRowThreads + t;
        if (idx < nitems) {
          const int rf = idx / KP4, c4 = idx - rf * KP4;
          const int r = rf / F, f = rf - r * F;
          const float x = s_vals[rf];
          const float vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int k = c4 * 4 + c;
            const float e = vv[c] * x;
            if (k < K) {
              s_f32[r * D0p + f * K + k] = e;
              h0[r * lda + f * K + k] = f2bf(e);
            } else if (k == K) {
              s_wx[rf] = e;
            }
          }
        }
      }
    }
    const int r = t >> 4, q = t & 15;
    for (int c = D0 + q; c < D0p; c += 16) h0[r * lda + c] = 0;
  }
  __syncthreads();

  // ---- phase B: FM second order + first order -------------------------------------------------
  {
    const int r = t >> 4, q = t & 15;
    float cterm = 0.f, yw = 0.f;
    for (int k = q; k < K; k += 16) {
      float S = 0.f, Q = 0.f;
      for (int f = 0; f < F; ++f) {
        const float e = s_f32[r * D0p + f * K + k];
        S += e;
        Q += e * e;
      }
      s_S[r * K + k] = S;
      cterm += S * S - Q;
    }
    for (int f = q; f < F; f += 16) yw += s_wx[r * F + f];
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      cterm += __shfl_xor(cterm, o, 64);
      yw += __shfl_xor(yw, o, 64);
    }
    if (q == 0) s_ylin[r] = *p.fm_bias + yw + 0.5f * cterm;
  }
  if (p.train) {  // h0ᵀ for dW_0: 8 rows × 1 column per item → one 16-B store
    const uint16_t* h0 = reinterpret_cast<const uint16_t*>(smem + L.act[0]);
    const int lda = L.lda[0];
    for (int it = t; it < D0p * 2; it += kRowThreads) {
      const int c = it >> 1, h = it & 1;
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        w[j] = (uint32_t)h0[(h * 8 + 2 * j) * lda + c] | ((uint32_t)h0[(h * 8 + 2 * j + 1) * lda + c] << 16);
      *reinterpret_cast<uint4*>(p.actT[0] + (size_t)c * Bp + row0 + h * 8) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }

  // ---- phase C: hidden layers on MFMA --------------------------------------------------------
  for (int l = 0; l < p.nl; ++l) {
    const int Din = p.dims[l], Dout = p.dims[l + 1];
    const uint16_t* A = reinterpret_cast<const uint16_t*>(smem + L.act[l]);
    uint16_t* O = reinterpret_cast<uint16_t*>(smem + L.act[l + 1]);
    const int lda = L.lda[l], ldo = L.lda[l + 1];
    const uint16_t* W = p.WT[l];
    const float keep = p.keep[l];
    const bool drop = p.train && keep < 1.f;
    const float inv_keep = 1.f / keep;
    __syncthreads();  // previous layer's tile (and phase A/B) complete
    const int ntiles = Dout >> 4;
    for (int nt0 = wave; nt0 < ntiles; nt0 += 8) {
      f32x4 accs[2];
      rowtile_gemm<2, 8>(A, lda, W, Din, ntiles, nt0, Din, lane, accs);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int nt = nt0 + 4 * j;
        if (nt >= ntiles) continue;
        const f32x4 acc = accs[j];
        const int c = nt * 16 + (lane & 15), rb = (lane >> 4) * 4;
        const float bc = p.bias[l][c];
        Philox4 bits{0u, 0u, 0u, 0u};
        if (drop) bits = dropout_bits(p.seed, (uint32_t)l, step, (uint32_t)(row0 + rb) >> 2, (uint32_t)c);
        float hv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float a = fmaxf(acc[i] + bc, 0.f);
          if (drop) a = keep_from_bits(pick4(bits, i), keep) ? a * inv_keep : 0.f;
          if (row0 + rb + i >= p.B) a = 0.f;
          hv[i] = a;
          O[(rb + i) * ldo + c] = f2bf(a);
        }
        if (p.train)
          *reinterpret_cast<uint2*>(p.actT[l + 1] + (size_t)c * Bp + row0 + rb) =
              make_uint2(pack_bf2(hv[0], hv[1]), pack_bf2(hv[2], hv[3]));
      }
    }
  }
  __syncthreads();

  // ---- phase D: output layer + loss head (wave 0) ----------------------------------------------
  if (wave == 0) {
    const int Dn = p.dims[p.nl];
    const uint16_t* H = reinterpret_cast<const uint16_t*>(smem + L.act[p.nl]);
    const int ldh = L.lda[p.nl];
    const int r = lane >> 2, q = lane & 3;
    float s = 0.f;
    for (int c = q; c < Dn; c += 4) s += bf2f(H[r * ldh + c]) * p.w_out[c];
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (q == 0) {
      const int gr = row0 + r;
      const bool valid = gr < p.B;
      const float y = s_ylin[r] + s + *p.b_out;
      const float tl = valid ? p.labels[gr] : 0.f;
      const float pr = 1.f / (1.f + __expf(-y));
      float loss, g;
      if (p.loss_type == 0) {
        loss = fmaxf(y, 0.f) - y * tl + log1pf(__expf(-fabsf(y)));
        g = pr - tl;
      } else {
        const float d = pr - tl;
        loss = d * d;
        g = 2.f * d * pr * (1.f - pr);
      }
      g = valid ? g * p.inv_scale : 0.f;
      s_g[r] = g;
      if (valid) {
        p.prob[gr] = pr;
        if (p.loss_rows) p.loss_rows[gr] = loss;
      }
      if (p.train) p.g_out[gr] = g;
    }
  }
  if (!p.train) return;
  __syncthreads();

  // ---- phase E: backward through the MLP ------------------------------------------------------
  uint16_t* dz_cur = reinterpret_cast<uint16_t*>(smem + L.dzA);
  uint16_t* dz_nxt = reinterpret_cast<uint16_t*>(smem + L.dzB);
  const int ldz = L.ldz;
  {
    const int a = p.nl, Dn = p.dims[a];
    const uint16_t* H = reinterpret_cast<const uint16_t*>(smem + L.act[a]);
    const int ldh = L.lda[a];
    const float inv_keep = 1.f / p.keep[a - 1];
    for (int it = t; it < Dn * 4; it += kRowThreads) {
      const int c = it % Dn, rg = it / Dn;
      const float wc = p.w_out[c];
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = rg * 4 + i;
        const float h = bf2f(H[r * ldh + c]);
        v[i] = h > 0.f ? s_g[r] * wc * inv_keep : 0.f;
        dz_cur[r * ldz + c] = f2bf(v[i]);
      }
      *reinterpret_cast<uint2*>(p.dzT[a] + (size_t)c * Bp + row0 + rg * 4) =
          make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
    }
  }
  for (int a = p.nl; a >= 1; --a) {
    __syncthreads();
    const int li = a - 1, Dout = p.dims[a], Din = p.dims[li];
    const uint16_t* W = p.Wb[li];  // [Din][Dout]
    const int ntiles = Din >> 4;
    for (int nt0 = wave; nt0 < ntiles; nt0 += 16) {
      f32x4 accs[4];
      rowtile_gemm<4, 4>(dz_cur, ldz, W, Dout, ntiles, nt0, Dout, lane, accs);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int nt = nt0 + 4 * j;
        if (nt >= ntiles) continue;
        const f32x4 acc = accs[j];
        const int c = nt * 16 + (lane & 15), rb = (lane >> 4) * 4;
        if (li >= 1) {
          const uint16_t* H = reinterpret_cast<const uint16_t*>(smem + L.act[li]);
          const int ldh = L.lda[li];
          const float inv_keep = 1.f / p.keep[li - 1];
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float h = bf2f(H[(rb + i) * ldh + c]);
            v[i] = h > 0.f ? acc[i] * inv_keep : 0.f;
            dz_nxt[(rb + i) * ldz + c] = f2bf(v[i]);
          }
          *reinterpret_cast<uint2*>(p.dzT[li] + (size_t)c * Bp + row0 + rb) =
              make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) s_f32[(rb + i) * D0p + c] = acc[i];
        }
      }
    }
    uint16_t* tmp = dz_cur;
    dz_cur = dz_nxt;
    dz_nxt = tmp;
  }
  __syncthreads();

  // ---- phase F: FM backward → per-lookup gradient rows -----------------------------------------
  {
    const int KP4 = Kp >> 2;
    const int nitems = kRowTile * F * KP4;
    const float4* emb4 = reinterpret_cast<const float4*>(p.emb);
    for (int base = 0; base < nitems; base += kRowThreads * 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int idx = min(base + u * kRowThreads + t, nitems - 1);
        const int rf = idx / KP4, c4 = idx - rf * KP4;
        v[u] = emb4[(size_t)s_ids[rf] * KP4 + c4];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int idx = base + u * kRowThreads + t;
        if (idx >= nitems) continue;
        const int rf = idx / KP4, c4 = idx - rf * KP4;
        const int r = rf / F, f = rf - r * F;
        if (row0 + r >= p.B) continue;
        const float g = s_g[r], x = s_vals[rf];
        const float* S = s_S + r * K;
        const float* dh = s_f32 + r * D0p + f * K;
        const float vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
        float o[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int k = c4 * 4 + c;
          o[c] = (k < K) ? x * (g * (S[k] - vv[c] * x) + dh[k]) : ((k == K) ? g * x : 0.f);
        }
        reinterpret_cast<float4*>(p.contrib + ((size_t)(row0 + r) * F + f) * Kp)[c4] = make_float4(o[0], o[1], o[2], o[3]);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
static int align16(int x) { return (x + 15) & ~15; }

RowsLds rows_lds_layout(const int* dims, int nl, int F, int K) {
  RowsLds L{};
  int off = 0;
  auto take = [&](int bytes) {
    int o = off;
    off += align16(bytes);
    return o;
  };
  L.ids = take(kRowTile * F * 4);
  L.vals = take(kRowTile * F * 4);
  L.wx = take(kRowTile * F * 4);
  L.S = take(kRowTile * K * 4);
  L.ylin = take(kRowTile * 4);
  L.g = take(kRowTile * 4);
  int maxh = 0;
  for (int a = 0; a <= nl; ++a) {
    L.lda[a] = dims[a] + 8;  // +16 B per row breaks the power-of-two row stride
    L.act[a] = take(kRowTile * L.lda[a] * 2);
    if (a > 0 && dims[a] > maxh) maxh = dims[a];
  }
  L.ldz = maxh + 8;
  L.dzA = take(kRowTile * L.ldz * 2);
  L.dzB = take(kRowTile * L.ldz * 2);
  L.f32 = take(kRowTile * dims[0] * 4);
  L.total = off;
  return L;
}

void launch_deepfm_rows(RowsParams p, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {  // allow > 64 KiB of dynamic LDS (160 KiB per CU on gfx950)
    ROCFM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(deepfm_rows_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  ROCFM_REQUIRE(p.nl >= 1 && p.nl <= kMaxHidden, "deepfm_rows: 1..6 hidden layers supported");
  ROCFM_REQUIRE(p.Kp % 4 == 0 && p.Kp >= p.K + 1, "deepfm_rows: Kp must be a multiple of 4 and > K");
  ROCFM_REQUIRE(p.dims[0] % 32 == 0 && p.dims[0] >= p.F * p.K, "deepfm_rows: dims[0] = round_up(F*K, 32)");
  for (int a = 1; a <= p.nl; ++a) ROCFM_REQUIRE(p.dims[a] % 32 == 0, "deepfm_rows: hidden dims padded to 32");
  ROCFM_REQUIRE(p.Bp % kRowTile == 0 && p.Bp >= p.B, "deepfm_rows: Bp must be a multiple of 16 and >= B");
  ROCFM_REQUIRE((p.Bp % 64) == 0 || !p.train, "deepfm_rows: training needs Bp % 64 == 0");
  p.lds = rows_lds_layout(p.dims, p.nl, p.F, p.K);
  ROCFM_REQUIRE(p.lds.total <= 160 * 1024, "deepfm_rows: LDS budget exceeded (F*K too large)");
  const int grid = p.Bp / kRowTile;
  if (grid == 0) return;
  hipLaunchKernelGGL(deepfm_rows_kernel, dim3(grid), dim3(kRowThreads), p.lds.total, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
