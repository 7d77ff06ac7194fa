// DeepFM fused row-tile kernel: the whole per-example part of a training step in ONE launch.
//
// One 512-thread workgroup (8 waves) owns RT consecutive examples (row_tile: 8 by default — 128
// workgroups at B = 1024; 16 = one full MFMA M-tile, 4 for small batches; profiles/r3_row_tile.md)
// and runs, entirely out of LDS:
//   A  gather fm_v/fm_w rows (f32, 16-B vector loads) → e = V[id]·x, h0 = bf16(e)  (PS:207-213)
//   B  S = Σ_f e, y_v = ½Σ_k(S² − Σ_f e²), y_w = Σ_f w·x, y_lin = b + y_w + y_v    (PS:214-217)
//   C  hidden layers: h_{l+1} = dropout(relu(h_l·W_l + c_l)) on v_mfma_f32_16x16x32_bf16
//      (Philox keep-mask, keep = `dropout` flag value)                             (PS:234-246)
//   D  y_d = h_L·w_out + c_out, y = y_lin + y_d, p = σ(y), loss, g = dL/dy          (PS:248-276)
//   E  backward data path through the MLP (dz_l = 1[h_l>0]/keep · dh_l, dh = dz·Wᵀ)
//   F  FM backward: de = g·(S − e) + dh0, per-lookup gradient row [x·de | g·x]
// It writes bf16 activations/dz transposed ([feature][batch], fragment-swizzled: common.h act_swz) for the weight-gradient kernel
// (mlp_wgrad.hip) and the per-lookup gradient rows for the embedding update (emb_update.hip).
// Nothing reduces across examples, so there are no atomics and no inter-workgroup hand-offs.
//
// At the reference's 1024-row batches the kernel is LATENCY-bound (128 workgroups for 256 CUs,
// one wave per SIMD):
// its time is the chain of dependent memory round trips plus each wave's serial instruction
// stream.  So:
//  * every phase issues all of its global loads before consuming any (flattened gather items);
//  * barriers wait for LDS only (lds_barrier): global stores stay in flight across phases;
//  * small parameters (biases, deep_out, labels) are staged into LDS in phase 0;
//  * the shape is a template parameter.  For the common model shapes (CtShape instantiations)
//    every loop unrolls, all index arithmetic folds, and EVERY layer's MFMA weight fragments are
//    prefetched into registers one or more phases before they are needed (forward layer 0 at
//    kernel entry, under the id/value staging + gather; the backward fragments during the
//    forward), so no GEMM phase waits on memory.  Other shapes run the same code with a runtime
//    shape (RtShape) and per-GEMM batched fragment loads.
#include "deepfm_rows.h"

namespace rocfm {

namespace {

__device__ __forceinline__ bf16x8 ld_frag(const uint16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }
// Input-layer weight fragments: bf16x8 from the swizzled bf16 copy, or (FP8) the 8 pre-quantised
// e4m3 bytes at the same element offset of the fp8 copy (deepfm_rows.h Fp8W0) — one MFMA operand.
template <bool FP8>
struct W0Frag {
  using type = bf16x8;
};
template <>
struct W0Frag<true> {
  using type = long;
};
template <bool FP8>
__device__ __forceinline__ typename W0Frag<FP8>::type ld_w0(const uint16_t* bf, const uint8_t* f8, size_t off) {
  if constexpr (FP8)
    return *reinterpret_cast<const long*>(f8 + off);
  else
    return ld_frag(bf + off);
}

// fp8 (OCP e4m3fn, gfx950) quantisation of 8 bf16 values scaled by s into one MFMA operand
// (byte j = element j; round-to-nearest-even conversion).
__device__ __forceinline__ long quant_fp8x8(bf16x8 v, float s) {
  int lo = 0, hi = 0;
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f((uint16_t)v[0]) * s, bf2f((uint16_t)v[1]) * s, lo, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f((uint16_t)v[2]) * s, bf2f((uint16_t)v[3]) * s, lo, true);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f((uint16_t)v[4]) * s, bf2f((uint16_t)v[5]) * s, hi, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f((uint16_t)v[6]) * s, bf2f((uint16_t)v[7]) * s, hi, true);
  return (long)(uint32_t)lo | ((long)(uint32_t)hi << 32);
}

__device__ __forceinline__ uint32_t pick4(const Philox4& b, int i) {
  return i == 0 ? b.x : i == 1 ? b.y : i == 2 ? b.z : b.w;
}

// lane exchange within DPP rows: v of lane quad_perm / mirror partner (full waves only)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// sum over each 32-lane half of a wave, to every lane of the half: lanes ^1 and ^2 (quad_perm),
// then the 8- and 16-lane mirrors (after the quad steps every lane of a quad holds its sum, so the
// mirror partner is a partner of the other quad / half-row), on DPP; then the other 16-lane row by
// one ds_bpermute — four of the five butterfly levels without an LDS-pipe round trip
__device__ __forceinline__ float half_wave_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]: lane ^ 2
  v += dpp_f<0x141>(v);  // row_half_mirror: lane i <-> 7 - i within 8
  v += dpp_f<0x140>(v);  // row_mirror: lane i <-> 15 - i within 16
  return v + __shfl_xor(v, 16, 64);
}

// x / F for x < 4096, F <= 64 (host-checked): magic = floor(2^32 / F) + 1
__device__ __forceinline__ int fdiv(int x, uint32_t magic) { return (int)__umulhi((uint32_t)x, magic); }

constexpr int kWaves = kRowThreads / 64;

// acc[j] = A(16 × Kd, LDS bf16, row stride lda) · B(Kd × 16) for the n-tiles nt = nt0 + step*j
// (j < NTW).  B fragments come from global/L2: tile nt, k-step ks at
// Bt + (nt*16 + (lane&15))*ldb + ks + 8*(lane>>4).  Every batch issues KU k-steps × NTW tiles of
// 16-B loads before the first MFMA; out-of-range k-steps load a clamped (valid) address and are
// zeroed on the VALUE (no per-load predication — cdna guide §5 trap (c)).
// Bs (nullable): the same matrix in the frag_swz layout — every B fragment is then one 1 KiB
// contiguous read instead of 16 strided row pieces (the runtime-shape kernel's weight traffic).
template <int NTW, int KU>
__device__ __forceinline__ void rowtile_gemm(const uint16_t* A, int lda, const uint16_t* Bt, int ldb, int ntiles,
                                             int nt0, int step, int Kd, int lane, f32x4 (&acc)[NTW],
                                             const uint16_t* Bs = nullptr) {
#pragma unroll
  for (int j = 0; j < NTW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint16_t* ap = A + (lane & 15) * lda + 8 * (lane >> 4);
  const uint16_t* bp[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = min(nt0 + step * j, ntiles - 1);
    bp[j] = Bs ? Bs + frag_at(nt, 0, ldb, lane) : Bt + (size_t)(nt * 16 + (lane & 15)) * ldb + 8 * (lane >> 4);
  }
  // consecutive k-steps of one swizzled tile are 512 elements apart; of the row-major matrix, 32
  const int kstride = Bs ? 512 / 32 : 1;
  const bf16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int k0 = 0; k0 < Kd; k0 += 32 * KU) {
    bf16x8 a[KU], b[NTW][KU];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int ks = min(k0 + 32 * u, Kd - 32);
#pragma unroll
      for (int j = 0; j < NTW; ++j) b[j][u] = ld_frag(bp[j] + (size_t)ks * kstride);
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
        if (nt0 + step * j < ntiles) acc[j] = mfma16x16x32(a[u], b[j][u], acc[j]);
  }
}

// ---- batch normalisation (batch_norm=True) -----------------------------------------------------
// Batch moments couple every row of the batch, so the BN layers split the launch with grid-wide
// barriers (2 per hidden layer: forward moments, backward column sums).  The launcher checks that
// the whole grid is resident; every spin is bounded (1 s) and flags bn_error instead of hanging.
constexpr uint64_t kBnSpinTicks = 100000000ull;  // s_memrealtime runs at 100 MHz
typedef __attribute__((address_space(1))) unsigned bn_gu32;
typedef __attribute__((address_space(1))) unsigned long long xg_u64;

// Grid barrier k (0-based, in execution order) of this launch on one monotonic arrival counter:
// every wave drains its stores, one lane per workgroup releases at agent scope (writes back this
// XCD's L2), arrives, polls relaxed with s_sleep, then acquires (drops this CU's stale L1 lines),
// so the partial moments other workgroups stored before the barrier are read fresh after it.
__device__ __forceinline__ void bn_grid_sync(const RowsParams& p, unsigned k) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    bn_gu32* c = (bn_gu32*)(p.bn_sync);
    const unsigned target = (k + 1u) * gridDim.x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kBnSpinTicks) {
        atomicOr(p.bn_error, 1);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// After the last barrier: the last workgroup out zeroes both counters for the next launch.
__device__ __forceinline__ void bn_grid_exit(const RowsParams& p) {
  __syncthreads();
  if (threadIdx.x == 0) {
    bn_gu32* c = (bn_gu32*)(p.bn_sync);
    if (__hip_atomic_fetch_add(c + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u) {
      __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(c + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Rows of workgroup w that are real batch rows (the padded tail contributes nothing).
__device__ __forceinline__ int bn_rows(int B, int w) { return max(0, min(kRowTile, B - w * kRowTile)); }

// ---- shapes ----------------------------------------------------------------------------------
// Runtime shape: any F/K/MLP the host validated.
struct RtShape {
  static constexpr bool kStatic = false;
  static constexpr int KSF0 = 1, KSF1 = 1, KSF2 = 1, NJB0 = 1, KSB0 = 1, KSB1 = 1, KSB2 = 1;
  static constexpr int GU = 4;                 // gathered rows per thread per batch (phases A, F)
  static constexpr int KSF0E = 1, NJB0H = 1, NTF0 = 1, NTB1 = 1;
  static constexpr bool kLateBw0 = false, kWide = false;
  static constexpr int G = 1, T0F = 0, FG = 0, T0B = 0;
  int F, K, nl, d[kMaxHidden + 1];
  __device__ explicit RtShape(const RowsParams& p) : F(p.F), K(p.K), nl(p.nl) {
#pragma unroll
    for (int i = 0; i <= kMaxHidden; ++i) d[i] = p.dims[i];
  }
  __device__ int dim(int l) const { return d[l]; }
};

// Compile-time shape: F fields, K embedding dims, hidden widths D1 ≥ … (0 = absent), ≤ 3 layers of
// ≤ 128 units, F·K ≤ 1280 (host-checked).  Fragment-prefetch counts per wave:
//   forward layer l : one 16-column tile (wave w owns tile w), dims[l]/32 k-steps   → KSF_l
//   backward li     : tiles w, w+8, … of dims[li]/16 (NJB_li of them), dims[li+1]/32 k-steps → KSB_li
// GU: gathered table rows per thread (phases A and F issue all of a tile's loads at once).
// kLateBw0: the layer-0 forward and backward fragments together exceed the register budget (wide
// input layers, e.g. the notebook's 39×32 = 1248): the backward ones are then prefetched at the
// last hidden layer's forward GEMM (under it, the head and the upper backward layers) instead of
// before layer 0, and phase F re-gathers its rows after the layer-0 backward GEMM.
// G_ > 1: the row-tile split — G_ workgroups share one row tile (profiles/r5_layer0_split.md).
// Member m computes layer 0's forward tiles [m·T0F, (m+1)·T0F) and hands them to the others
// through an in-launch exchange (RowsParams::xbuf / xctr), the layer-0 dgrad tiles of its fields
// [m·FG, (m+1)·FG) and those fields' per-lookup gradient rows; everything else runs on every
// member (its global stores on member 0 only), so each CU streams 1/G_ of W0 twice per step.
template <int F_, int K_, int D1, int D2, int D3, int G_ = 1>
struct CtShape {
  static constexpr bool kStatic = true;
  static constexpr int F = F_, K = K_;
  static constexpr int nl = D3 ? 3 : (D2 ? 2 : 1);
  static constexpr int D0 = (F_ * K_ + 31) / 32 * 32;
  __device__ static constexpr int dim(int l) { return l == 0 ? D0 : l == 1 ? D1 : l == 2 ? D2 : D3; }
  static constexpr int G = G_;
  static constexpr int T0F = D1 / 16 / G_;                    // layer-0 forward tiles per member
  static constexpr int FG = (F_ + G_ - 1) / G_;               // fields per member (the last: fewer)
  static constexpr int T0B = G_ > 1 ? FG * K_ / 16 : D0 / 16;  // layer-0 dgrad tiles per member (≤)
  static_assert(G_ == 1 || (K_ % 16 == 0 && (D1 / 16) % G_ == 0), "row split: K and D1/16 multiples");
  static constexpr int KSF0 = D0 / 32, KSF1 = D1 / 32 > 0 ? D1 / 32 : 1, KSF2 = D2 / 32 > 0 ? D2 / 32 : 1;
  static constexpr int NJB0 = (T0B + kWaves - 1) / kWaves;
  static constexpr int KSB0 = D1 / 32, KSB1 = D2 / 32 > 0 ? D2 / 32 : 1, KSB2 = D3 / 32 > 0 ? D3 / 32 : 1;
  static constexpr int KP4 = (K_ + 1 + 3) / 4;
  static constexpr int GU = (kRowTile * F_ * KP4 + kRowThreads - 1) / kRowThreads;
  static constexpr bool kLateBw0 = (KSF0 + NJB0 * KSB0) * 4 > 128;
  // layer-0 forward fragments prefetched at kernel entry; kLateBw0 shapes load the rest after the
  // gather (phase A holds GU gathered rows + their scaled copies in registers)
  static constexpr int KSF0E = kLateBw0 ? 8 : KSF0;
  // Wide first hidden layer (D1 = 256, the reference's default 256-128-64): each wave owns NTF0 = 2
  // forward tiles of layer 0 and NTB1 = 2 backward tiles of layer 1.  Layer 0's forward fragments
  // then stream through the KSF0 registers of one tile — slot u is refilled with the next tile's
  // k-step u right after its MFMA has been issued — so the second tile's loads fly under the first
  // tile's MFMAs and epilogue (the per-CU fragment bandwidth, not registers, bounds the layer).
  static constexpr int NTF0 = (T0F + kWaves - 1) / kWaves;
  static constexpr int NTB1 = (D1 / 16 + kWaves - 1) / kWaves;
  static constexpr bool kWide = NTF0 > 1;
  // registers for layer-0 backward fragments: all NJB0 tiles, or (kLateBw0) a ring of NJB0H tiles —
  // slot j % NJB0H is refilled with tile j + NJB0H right after tile j's MFMAs have been issued (wide
  // shapes: 4 slots of 8 k-steps, the rest of the register file holds the upper layers)
  static constexpr int NJB0H = kLateBw0 ? (kWide ? 4 : (NJB0 + 1) / 2) : NJB0;
  __device__ explicit CtShape(const RowsParams&) {}
  static_assert(D0 <= 1280 && D1 <= 256 && D2 <= 128 && D3 <= 128, "CtShape limits");
  static_assert(!kWide || (kLateBw0 && NTF0 == 2), "CtShape: a 256-wide first layer needs the streamed layer 0");
  static_assert(D1 % 32 == 0 && D2 % 32 == 0 && D3 % 32 == 0, "hidden dims padded to 32");
  static_assert(GU <= 12, "CtShape: at most 12 gathered rows per thread");
  static_assert(G_ == 1 || kLateBw0, "row split: wide input layers only");
};

template <class SH, int RT, int KP4>
__device__ constexpr int gather_units();
// phase F's per-lookup items of one member: its FG fields (all F without the split)
template <class SH, int RT, int KP4>
__device__ constexpr int gather_units_f() {
  if constexpr (SH::kStatic && SH::G > 1)
    return (RT * SH::FG * KP4 + kRowThreads - 1) / kRowThreads;
  else
    return gather_units<SH, RT, KP4>();
}

template <class SH, int RT, int KP4>
__device__ constexpr int gather_units() {
  if constexpr (SH::kStatic)
    return (RT * SH::F * KP4 + kRowThreads - 1) / kRowThreads;
  else
    return SH::GU;
}

}  // namespace

// Diagnostic phase stamps kept in LDS and written out once at the end, so that recording them
// adds no global store (and no vmcnt wait) inside the measured phases.
#define ROWS_STAMP(i)                                                                             \
  do {                                                                                            \
    if (DIAG && p.stamps != nullptr && threadIdx.x == 0) s_stamp[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// FP8 is a template parameter (not a runtime branch on p.fp8): the fp8 input-layer path kept in the
// bf16 kernel raised its register demand past the 256 VGPRs of a 2-wave/SIMD workgroup and spilled.
// MODE (kInfer / kTrain / kDynamic = read p.train) and DIAG (phase stamps + ablations) are template
// parameters as well: in the compile-time-shape kernels a runtime `if (train)` around the backward
// weight prefetch, or an ablation test around a phase, splits the memory-op stream into branches,
// and the waitcnt insertion then merges them pessimistically — it waited for EVERY outstanding
// load and activation store (vmcnt(0..5)) at each hidden layer instead of only that layer's
// prefetched fragments.  Branch-free static kernels wait only for what they consume.
constexpr int kInfer = 0, kTrain = 1, kDynamic = 2;

// RT: examples per workgroup (16, or 8 for twice the workgroups on a 256-CU chip).  The LDS tiles
// and MFMA M tiles stay 16 rows; with RT = 8 rows 8..15 are zero padding whose outputs are
// discarded (no global store touches them), so the arithmetic of every valid row is unchanged.
// BN: a compile-time-shape kernel with batch_norm layers (16-row workgroups, grid barriers); the
// runtime-shape kernel reads p.bn, the other compile-time-shape kernels have no batch-norm code.
template <int KP4, class SH, bool FP8, int MODE, bool DIAG, bool BT, int RT, bool BN = false>
__global__ __launch_bounds__(kRowThreads) void deepfm_rows_kernel(const RowsParams p) {
  static_assert(RT == 16 || RT == 8 || RT == 4, "rows per workgroup: 16, 8 or 4");
  static_assert(!BN || (SH::kStatic && RT == kRowTile && !FP8), "batch_norm kernels: 16-row tiles, bf16");
  static_assert(RT != 4 || SH::kStatic, "4-row workgroups: compile-time shapes only");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ unsigned long long s_stamp[16];
  const SH sh(p);
  const RowsLds& L = p.lds;
  int32_t* s_ids = reinterpret_cast<int32_t*>(smem + L.ids);
  float* s_vals = reinterpret_cast<float*>(smem + L.vals);
  int32_t* s_pos = reinterpret_cast<int32_t*>(smem + L.pos);
  int32_t* s_nxt = reinterpret_cast<int32_t*>(smem + L.nxt);  // (dedup only)
  float* s_wx = reinterpret_cast<float*>(smem + L.wx);
  float* s_S = reinterpret_cast<float*>(smem + L.S);
  float* s_ylin = reinterpret_cast<float*>(smem + L.ylin);
  float* s_g = reinterpret_cast<float*>(smem + L.g);
  float* s_amax = reinterpret_cast<float*>(smem + L.amax);  // fp8: per-row max |h0|
  float* s_f32 = reinterpret_cast<float*>(smem + L.f32);  // e (forward) / dh0 (backward), stride dims[0]
  float* s_prm = reinterpret_cast<float*>(smem + L.prm);

  constexpr int Kp = KP4 * 4;
  // gathered table rows per thread (phases A, F): the whole tile's rows in one batch (static shapes)
  constexpr int kGU = gather_units<SH, RT, KP4>();
  const bool train = MODE == kDynamic ? (p.train != 0) : (MODE == kTrain);
  const int ablate = DIAG ? p.ablate : 0;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  // row-tile split: the G members of row tile rt are blocks (rt / 8)·8G + m·8 + rt % 8 — equal
  // blockIdx % 8, one XCD under round-robin dispatch (a speed matter only), consecutive in dispatch
  // order (the exchange's waiters never wait on a block queued behind them)
  constexpr int G = SH::G;
  const int mbr = G > 1 ? (int)((blockIdx.x >> 3) % G) : 0;
  const int rtile = G > 1 ? (int)((blockIdx.x / (8 * G)) * 8 + (blockIdx.x & 7)) : (int)blockIdx.x;
  const bool lead = mbr == 0;  // the member that stores the row tile's shared outputs
  const int row0 = rtile * RT;
  // write-through store targets (RowsParams::wt): buffer descriptors over contrib / h0ᵀ
  const __amdgpu_buffer_rsrc_t wt_contrib = __builtin_amdgcn_make_buffer_rsrc(p.contrib, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t wt_h0 = __builtin_amdgcn_make_buffer_rsrc(p.actT[0], (short)0, 0x7fffffff, 0x00020000);
  // layer-0 dgrad tiles of this member: its fields' columns (all of dims[0] without the split)
  const int tb0 = G > 1 ? mbr * SH::T0B : 0;
  const int tb1 = G > 1 ? min(tb0 + SH::T0B, sh.dim(0) / 16) : sh.dim(0) / 16;
  const int F = sh.F, K = sh.K, NL = sh.nl;
  const int D0 = F * K, D0p = sh.dim(0);
  const uint32_t magicF = p.magicF;
  const int Bp = p.Bp;
  const void* emb4 = p.emb;  // f32 or (BT) bf16 rows: tbl_load4
  const bf16x8 zero8 = {0, 0, 0, 0, 0, 0, 0, 0};
  ROWS_STAMP(0);
  if (p.zero_word != nullptr && blockIdx.x == 0 && t == 0) *p.zero_word = 0;
  // fp8: de-scale of the pre-quantised input-layer weights; training zeroes the slot this step's
  // weight refresh accumulates the new max into (deepfm_rows.h Fp8W0)
  const float w8inv = FP8 ? *p.w8.inv_scale : 0.f;
  if (FP8 && train && blockIdx.x == 0 && t == 0) p.w8.amax[((p.step ? *p.step : 0) + 1) & 1] = 0.f;

  // ---- phase 0: stage ids / values and every small parameter the later phases read -----------
  // The ids are the head of the kernel's latency chain (ids → gathered rows): their loads are
  // issued first; the layer-0 weight prefetch is issued behind them and lands during phase A.
  typename W0Frag<FP8>::type fw0[SH::KSF0];
  if constexpr (SH::kStatic) {
    // every load unconditional (clamped index, value selected afterwards): no exec branches in
    // the memory-op stream (see MODE above); the kernarg pointers are read up front
    constexpr int kItems = (RT * SH::F + kRowThreads - 1) / kRowThreads;
    const int32_t* ids_g = p.ids;
    const float* vals_g = p.vals;
    const int32_t* pos_g = p.contrib_pos ? p.contrib_pos : p.ids;  // any valid [B][F] int32 buffer
    const bool has_pos = p.contrib_pos != nullptr;
    const bool dedup = p.dedup != 0;
    const int32_t* nxt_g = dedup ? p.contrib_nxt : p.ids;
    const int nvalid = max(0, min(RT, p.B - row0)) * F;  // valid lookups of this tile
    const int last = max(p.B * F - 1, 0);                        // clamp target: a valid lookup
    int32_t idr[kItems];
    float vlr[kItems];
    int32_t psr[kItems], nxr[kItems];
#pragma unroll
    for (int u = 0; u < kItems; ++u) {
      const int i = t + u * kRowThreads;
      const size_t gi = (size_t)min(row0 * F + i, last);
      idr[u] = ids_g[gi];
      vlr[u] = vals_g[gi];
      psr[u] = pos_g[gi];
      nxr[u] = nxt_g[gi];
    }
    float br[SH::nl];
#pragma unroll
    for (int l = 0; l < SH::nl; ++l) br[l] = p.bias[l][min(t, sh.dim(l + 1) - 1)];
    const float wo = p.w_out[min(t, sh.dim(SH::nl) - 1)];
    const float lab = p.labels[min(row0 + (t & (RT - 1)), max(p.B - 1, 0))];
    const float bo = *p.b_out, fb = *p.fm_bias;
    const int nt = G > 1 ? mbr * SH::T0F + min(wave, SH::T0F - 1) : min(wave, sh.dim(1) / 16 - 1);
#pragma unroll
    for (int u = 0; u < SH::KSF0E; ++u) fw0[u] = ld_w0<FP8>(p.WTs[0], p.w8.f, frag_at(nt, u, sh.dim(0), lane));
#pragma unroll
    for (int u = 0; u < kItems; ++u) {
      const int i = t + u * kRowThreads;
      if (i < RT * F) {
        const bool valid = i < nvalid;
        s_ids[i] = valid ? idr[u] : 0;
        s_vals[i] = valid ? vlr[u] : 0.f;
        s_pos[i] = (valid && has_pos) ? psr[u] : (int32_t)((size_t)row0 * F + i);
        if (dedup) s_nxt[i] = (valid && nxr[u] >= 0) ? nxr[u] - row0 * F : -1;  // tile-local (same tile)
      }
    }
#pragma unroll
    for (int l = 0; l < SH::nl; ++l)
      if (t < sh.dim(l + 1)) s_prm[L.prm_bias[l] + t] = br[l];
    if (t < sh.dim(SH::nl)) s_prm[L.prm_wout + t] = wo;
    if (t == 0) {
      s_prm[L.prm_bout] = bo;
      s_prm[L.prm_fmb] = fb;
    }
    if (t < kRowTile) s_prm[L.prm_lab + t] = (t < RT && row0 + t < p.B) ? lab : 0.f;
  } else {
    for (int i = t; i < RT * F; i += kRowThreads) {
      const bool valid = row0 + fdiv(i, magicF) < p.B;
      s_ids[i] = valid ? p.ids[(size_t)row0 * F + i] : 0;
      s_vals[i] = valid ? p.vals[(size_t)row0 * F + i] : 0.f;
      s_pos[i] = (valid && p.contrib_pos) ? p.contrib_pos[(size_t)row0 * F + i] : (int32_t)((size_t)row0 * F + i);
      if (p.dedup) {
        const int nx = valid ? p.contrib_nxt[(size_t)row0 * F + i] : -1;
        s_nxt[i] = nx >= 0 ? nx - row0 * F : -1;
      }
    }
#pragma unroll
    for (int l = 0; l < NL; ++l)
      for (int c = t; c < sh.dim(l + 1); c += kRowThreads) s_prm[L.prm_bias[l] + c] = p.bias[l][c];
    for (int c = t; c < sh.dim(NL); c += kRowThreads) s_prm[L.prm_wout + c] = p.w_out[c];
    if (t == 0) {
      s_prm[L.prm_bout] = *p.b_out;
      s_prm[L.prm_fmb] = *p.fm_bias;
    }
    if (t < kRowTile) s_prm[L.prm_lab + t] = (t < RT && row0 + t < p.B) ? p.labels[row0 + t] : 0.f;
  }
  const uint32_t step = p.step ? (uint32_t)(*p.step) : 0u;
  lds_barrier();
  ROWS_STAMP(1);

  // ---- phase A: gather rows, e = V·x (f32 scratch), h0 = bf16(e), w·x ---------------------------
  {
    uint16_t* h0 = reinterpret_cast<uint16_t*>(smem + L.act[0]);
    const int lda = L.lda[0];
    const int nitems = RT * F * KP4;
    constexpr int U = kGU;  // static shapes: the whole tile's rows in one batch
    for (int base = 0; base < nitems; base += kRowThreads * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = min(base + u * kRowThreads + t, nitems - 1);
        const int rf = idx / KP4, c4 = idx - rf * KP4;
        v[u] = tbl_load4<BT>(emb4, (size_t)s_ids[rf] * KP4 + c4);
      }
      // every gathered row is consumed (scaled) in straight-line code before any branch, so the
      // four loads are waited for once; the branches below hold LDS stores only
      float ev[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = min(base + u * kRowThreads + t, nitems - 1);
        const float x = s_vals[idx / KP4];
        ev[u][0] = v[u].x * x;
        ev[u][1] = v[u].y * x;
        ev[u][2] = v[u].z * x;
        ev[u][3] = v[u].w * x;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = base + u * kRowThreads + t;
        if (idx < nitems) {
          const int rf = idx / KP4, c4 = idx - rf * KP4;
          const int r = fdiv(rf, magicF), f = rf - r * F;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int k = c4 * 4 + c;
            const float e = ev[u][c];
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
    for (int i = t; i < RT * (D0p - D0); i += kRowThreads) {
      const int r = i / (D0p - D0), c = D0 + i - r * (D0p - D0);
      h0[r * lda + c] = 0;
    }
    if constexpr (RT < kRowTile) {  // padding rows of the MFMA tile: zero (finite) operands
      for (int i = t; i < (kRowTile - RT) * (lda / 8); i += kRowThreads) {
        const int r = RT + i / (lda / 8), c8 = i - (r - RT) * (lda / 8);
        *reinterpret_cast<uint4*>(h0 + r * lda + 8 * c8) = make_uint4(0u, 0u, 0u, 0u);
      }
      if constexpr (FP8 && SH::kStatic) {
        uint8_t* q8 = reinterpret_cast<uint8_t*>(smem + L.q8);
        for (int i = t; i < (kRowTile - RT) * (SH::D0 / 8); i += kRowThreads) {
          const int r = RT + i / (SH::D0 / 8), c8 = i - (r - RT) * (SH::D0 / 8);
          *reinterpret_cast<long*>(q8 + r * L.ldq + 8 * c8) = 0;
        }
      }
    }
  }
  lds_barrier();
  ROWS_STAMP(2);

  if constexpr (SH::kStatic && SH::KSF0E < SH::KSF0) {  // the rest of layer 0's forward fragments
    const int nt = G > 1 ? mbr * SH::T0F + min(wave, SH::T0F - 1) : min(wave, sh.dim(1) / 16 - 1);
#pragma unroll
    for (int u = SH::KSF0E; u < SH::KSF0; ++u) fw0[u] = ld_w0<FP8>(p.WTs[0], p.w8.f, frag_at(nt, u, sh.dim(0), lane));
  }

  // ---- phase B: FM second order + first order (32 lanes per row) ------------------------------
  if (!(ablate & 2) && (t >> 5) < RT) {  // (wave-uniform: two rows per wave)
    const int r = t >> 5, q = t & 31;
    float cterm = 0.f, yw = 0.f, amx = 0.f;
    // G = ⌊32/K⌋ lanes per embedding column split the F fields (field f → group f mod G); the
    // group partials are combined in group order through shuffles (deterministic)
    const int G = K <= 32 ? 32 / K : 1;
    if (G > 1) {
      const int k = q % K, gq = q / K;
      float S = 0.f, Q = 0.f;
      if (gq < G) {
#pragma unroll 4
        for (int f = gq; f < F; f += G) {
          const float e = s_f32[r * D0p + f * K + k];
          S += e;
          Q += e * e;
          amx = fmaxf(amx, fabsf(e));
        }
      }
      float St = 0.f, Qt = 0.f;
      for (int j = 0; j < G; ++j) {  // uniform loop: every lane takes part in each shuffle
        const int src = (lane & 32) + k + j * K;
        St += __shfl(S, src, 64);
        Qt += __shfl(Q, src, 64);
      }
      if (gq == 0) {
        s_S[r * K + k] = St;
        cterm = St * St - Qt;
      }
    } else {
      for (int k = q; k < K; k += 32) {
        float S = 0.f, Q = 0.f;
#pragma unroll 4
        for (int f = 0; f < F; ++f) {
          const float e = s_f32[r * D0p + f * K + k];
          S += e;
          Q += e * e;
          amx = fmaxf(amx, fabsf(e));
        }
        s_S[r * K + k] = S;
        cterm += S * S - Q;
      }
    }
    if constexpr (FP8) {  // row max |bf16(e)| = bf16(max |e|) (rounding is monotonic)
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) amx = fmaxf(amx, __shfl_xor(amx, o, 64));
      amx = bf2f(f2bf(amx));
      if (q == 0) s_amax[r] = amx;
      if constexpr (SH::kStatic) {  // this row's h0 → e4m3 (the layer-0 A operand), by its own lanes
        const uint16_t* h0 = reinterpret_cast<const uint16_t*>(smem + L.act[0]);
        uint8_t* q8 = reinterpret_cast<uint8_t*>(smem + L.q8);
        const float sa = kFp8Max / fmaxf(amx, 1e-30f);
        for (int c8 = q; c8 < SH::D0 / 8; c8 += 32)
          *reinterpret_cast<long*>(q8 + r * L.ldq + 8 * c8) = quant_fp8x8(ld_frag(h0 + r * L.lda[0] + 8 * c8), sa);
      }
    }
    for (int f = q; f < F; f += 32) yw += s_wx[r * F + f];
    cterm = half_wave_sum(cterm);  // (each row: one 32-lane half of the wave)
    yw = half_wave_sum(yw);
    if (q == 0) s_ylin[r] = s_prm[L.prm_fmb] + yw + 0.5f * cterm;
  }
  if (train && !(ablate & 1)) {  // h0ᵀ for dW_0: 8 rows × 1 column per item → one 16-B store
    const uint16_t* h0 = reinterpret_cast<const uint16_t*>(smem + L.act[0]);
    const int lda = L.lda[0];
    // (split: the member's own fields' columns; the last member also the padding columns)
    const int cb = G > 1 ? mbr * SH::FG * K : 0;
    const int ce = (G > 1 && mbr < G - 1) ? cb + SH::FG * K : D0p;
    if constexpr (RT >= 8) {
      for (int it = t; it < (ce - cb) * (RT / 8); it += kRowThreads) {
        const int c = cb + (RT == 8 ? it : it >> 1), h = RT == 8 ? 0 : it & 1;
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          w[j] = (uint32_t)h0[(h * 8 + 2 * j) * lda + c] | ((uint32_t)h0[(h * 8 + 2 * j + 1) * lda + c] << 16);
        if (p.wt & 2) {  // write-through (sc1): nothing of it left dirty in L2 at the kernel's end
          const u32x4 v = {w[0], w[1], w[2], w[3]};
          __builtin_amdgcn_raw_buffer_store_b128(v, wt_h0, (int)(act_swz(c, row0 + h * 8, Bp) * 2), 0, 16);
        } else {
          *reinterpret_cast<uint4*>(p.actT[0] + act_swz(c, row0 + h * 8, Bp)) = make_uint4(w[0], w[1], w[2], w[3]);
        }
      }
    } else {  // 4 rows × 1 column per item → one 8-B store
      for (int c = cb + t; c < ce; c += kRowThreads) {
        const uint32_t w0 = (uint32_t)h0[c] | ((uint32_t)h0[lda + c] << 16);
        const uint32_t w1 = (uint32_t)h0[2 * lda + c] | ((uint32_t)h0[3 * lda + c] << 16);
        *reinterpret_cast<uint2*>(p.actT[0] + act_swz(c, row0, Bp)) = make_uint2(w0, w1);
      }
    }
  }

  // ---- prefetch (static shapes): forward layers 1..2 and every backward fragment ----------------
  bf16x8 fw1[SH::KSF1], fw2[SH::KSF2];
  typename W0Frag<FP8>::type bw0[SH::NJB0H][SH::KSB0];
  bf16x8 bw1[SH::NTB1][SH::KSB1], bw2[SH::KSB2];
  // forward layers 1..2 and the upper backward layers' fragments (a few KiB per wave)
  auto prefetch_upper = [&]() {
    if constexpr (SH::kStatic) {
    if constexpr (SH::nl >= 2) {
      const int nt = min(wave, sh.dim(2) / 16 - 1);
#pragma unroll
      for (int u = 0; u < SH::KSF1; ++u) fw1[u] = ld_frag(p.WTs[1] + frag_at(nt, u, sh.dim(1), lane));
    }
    if constexpr (SH::nl >= 3) {
      const int nt = min(wave, sh.dim(3) / 16 - 1);
#pragma unroll
      for (int u = 0; u < SH::KSF2; ++u) fw2[u] = ld_frag(p.WTs[2] + frag_at(nt, u, sh.dim(2), lane));
    }
    if (train) {
      if constexpr (SH::nl >= 2) {
#pragma unroll
        for (int j = 0; j < SH::NTB1; ++j) {
          const int nt = min(wave + kWaves * j, sh.dim(1) / 16 - 1);
#pragma unroll
          for (int u = 0; u < SH::KSB1; ++u) bw1[j][u] = ld_frag(p.Wbs[1] + frag_at(nt, u, sh.dim(2), lane));
        }
      }
      if constexpr (SH::nl >= 3) {
        const int nt = min(wave, sh.dim(2) / 16 - 1);
#pragma unroll
        for (int u = 0; u < SH::KSB2; ++u) bw2[u] = ld_frag(p.Wbs[2] + frag_at(nt, u, sh.dim(3), lane));
      }
    }
    }
  };
  if constexpr (SH::kStatic) if (!(ablate & 4)) {
    if constexpr (!SH::kLateBw0) {  // wide input layers: issued once layer 0's forward fragments are dead
      prefetch_upper();
      if (train) {
        // backward of layer 0: dh0 tiles w + 8j of dims[0]/16, k = dims[1]
#pragma unroll
        for (int j = 0; j < SH::NJB0; ++j) {
          const int nt = min(wave + kWaves * j, sh.dim(0) / 16 - 1);
#pragma unroll
          for (int u = 0; u < SH::KSB0; ++u) bw0[j][u] = ld_w0<FP8>(p.Wbs[0], p.w8.b, frag_at(nt, u, sh.dim(1), lane));
        }
      }
    }
  }

  // ---- phase C: hidden layers on MFMA -----------------------------------------------------------
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const int Din = sh.dim(l), Dout = sh.dim(l + 1);
    const uint16_t* A = reinterpret_cast<const uint16_t*>(smem + L.act[l]);
    uint16_t* O = reinterpret_cast<uint16_t*>(smem + L.act[l + 1]);
    const int lda = L.lda[l], ldo = L.lda[l + 1];
    const float keep = p.keep[l];
    const bool drop = train && keep < 1.f;
    const float inv_keep = 1.f / keep;
    lds_barrier();  // previous layer's tile (and phase A/B) complete
    ROWS_STAMP(3 + l);

    if constexpr (SH::kStatic && SH::kLateBw0) {
      if (l == 1 && !(ablate & 4)) prefetch_upper();
      // from the last hidden layer on, only its own forward fragments are live: the layer-0 backward
      // ones now (hidden under that layer, the head and the upper backward layers)
      if (l == SH::nl - 1 && train && !(ablate & 4)) {
#pragma unroll
        for (int j = 0; j < SH::NJB0H; ++j) {
          const int nt = min(tb0 + wave + kWaves * j, tb1 - 1);
#pragma unroll
          for (int u = 0; u < SH::KSB0; ++u) bw0[j][u] = ld_w0<FP8>(p.Wbs[0], p.w8.b, frag_at(nt, u, sh.dim(1), lane));
        }
      }
    }
    const int ntiles = Dout >> 4;
    // split: layer 0's forward tiles of this member only
    const int ltb = (G > 1 && l == 0) ? mbr * SH::T0F : 0;
    const int lte = (G > 1 && l == 0) ? ltb + SH::T0F : ntiles;
    // compile-time shapes: tile j of this wave is wave + 8j (layer 0 of a wide shape has 2, every
    // other layer 1 — the outer loop then runs once); runtime shapes: one tile per iteration
    constexpr int kNT = SH::kStatic ? SH::NTF0 : 1;
    for (int nt0 = ltb + wave; nt0 < lte; nt0 += kNT * kWaves) {
#pragma unroll
     for (int j = 0; j < kNT; ++j) {
      const int nt = nt0 + kWaves * j;
      if (j > 0 && (l > 0 || nt >= lte)) break;
      // diagnostics (ablate bits 4 / 5): only 1/2 or 1/4 of layer 0's forward tiles — what a
      // workgroup of a row-group split over 2 / 4 workgroups would stream (profiles/r5_layer0_split.md)
      if (DIAG && l == 0 && (ablate & 48)) {
        if (j > 0 && SH::kWide) break;
        const int wcut = SH::kWide ? ((ablate & 32) ? 4 : 8) : ((ablate & 32) ? 2 : 4);
        if (wave >= wcut) break;
      }
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if constexpr (SH::kStatic) {
        const uint16_t* ap = A + (lane & 15) * lda + 8 * (lane >> 4);
        if (l == 0 && SH::kWide && !FP8) {
          // streamed layer 0: slot u is refilled with the next tile's k-step u right behind its MFMA
          const int nxt = min(nt + kWaves, ntiles - 1);
#pragma unroll
          for (int u = 0; u < SH::KSF0; ++u) {
            acc = mfma16x16x32(ld_frag(ap + 32 * u), fw0[u], acc);
            if (j + 1 < kNT && !(DIAG && (ablate & 48))) fw0[u] = ld_w0<FP8>(p.WTs[0], p.w8.f, frag_at(nxt, u, sh.dim(0), lane));
          }
        } else if (l == 0) {
          if constexpr (FP8) {
            // fp8-e4m3 MFMA: the weights come pre-quantised (one scale per tensor, w8inv), the
            // activations are quantised per row here; the product is de-scaled in the epilogue
            const uint8_t* aq = reinterpret_cast<const uint8_t*>(smem + L.q8) + (lane & 15) * L.ldq + 8 * (lane >> 4);
#pragma unroll
            for (int u = 0; u < SH::KSF0; ++u)
              acc = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(*reinterpret_cast<const long*>(aq + 32 * u), fw0[u],
                                                              acc, 0, 0, 0);
            const int rbq = (lane >> 4) * 4;
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i] *= (fmaxf(rbq + i < RT ? s_amax[rbq + i] : 0.f, 1e-30f) / kFp8Max) * w8inv;
          } else {
#pragma unroll
            for (int u = 0; u < SH::KSF0; ++u) acc = mfma16x16x32(ld_frag(ap + 32 * u), fw0[u], acc);
          }
        } else if (l == 1) {
#pragma unroll
          for (int u = 0; u < SH::KSF1; ++u) acc = mfma16x16x32(ld_frag(ap + 32 * u), fw1[u], acc);
        } else {
#pragma unroll
          for (int u = 0; u < SH::KSF2; ++u) acc = mfma16x16x32(ld_frag(ap + 32 * u), fw2[u], acc);
        }
      } else {
        f32x4 accs[1];
        rowtile_gemm<1, 16>(A, lda, p.WT[l], Din, ntiles, nt, kWaves, Din, lane, accs, p.WTs[l]);
        acc = accs[0];
      }
      const int c = nt * 16 + (lane & 15), rb = (lane >> 4) * 4;
      const float bc = s_prm[L.prm_bias[l] + c];
      if constexpr (!SH::kStatic || BN) {
        if (p.bn) {  // training: keep r = relu(z) for the batch moments; inference: moving moments
          float* R = reinterpret_cast<float*>(smem + L.bnr[l]);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float a = fmaxf(acc[i] + bc, 0.f);
            if (!train)
              a = (a - p.bn_mean[l][c]) * rsqrtf(p.bn_var[l][c] + p.bn_eps) * p.bn_gamma[l][c] + p.bn_beta[l][c];
            if (row0 + rb + i >= p.B) a = 0.f;
            if (train)
              R[(rb + i) * Dout + c] = a;
            else
              O[(rb + i) * ldo + c] = f2bf(a);
          }
          continue;
        }
      }
      Philox4 bits{0u, 0u, 0u, 0u};
      if (drop) bits = dropout_bits(p.seed, (uint32_t)l, step, (uint32_t)(row0 + rb) >> 2, (uint32_t)c);
      float hv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float a = fmaxf(acc[i] + bc, 0.f);
        if (drop) a = keep_from_bits(pick4(bits, i), keep) ? a * inv_keep : 0.f;
        if (rb + i >= RT || row0 + rb + i >= p.B) a = 0.f;
        hv[i] = a;
        O[(rb + i) * ldo + c] = f2bf(a);
      }
      if (train && rb < RT && (G == 1 || l == 0 || lead))
        *reinterpret_cast<uint2*>(p.actT[l + 1] + act_swz(c, row0 + rb, Bp)) =
            make_uint2(pack_bf2(hv[0], hv[1]), pack_bf2(hv[2], hv[3]));
      if (G > 1 && l == 0 && rb < RT) {  // the exchange: 4 rows of column c, one 8-B write-through store
        const size_t xo = (((size_t)rtile * G + mbr) * (SH::T0F * 16) + (c - ltb * 16)) * 16 + rb;
        const unsigned long long v8 = (unsigned long long)pack_bf2(hv[0], hv[1]) |
                                      ((unsigned long long)pack_bf2(hv[2], hv[3]) << 32);
        __hip_atomic_store((xg_u64*)(p.xbuf + xo), v8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
     }
    }
    if constexpr (G > 1) {
      if (l == 0) {
        // hand-off (MI355X_MICROARCH.md § visibility, Valid forms row 1): every wave drains its
        // write-through stores, ONE lane adds to the row tile's arrival counter (agent scope); the
        // last arrival learns it from the returned value, the others poll it (sc1 loads, s_sleep,
        // bounded); every load of a peer's columns is an sc1 load.  The counter rises by G per
        // launch and is never reset (arrival parity = old mod G).
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) {
          bn_gu32* ctr = (bn_gu32*)(p.xctr) + rtile;
          const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const unsigned gen0 = old - old % (unsigned)G;
          if (old - gen0 != (unsigned)G - 1u) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - gen0 < (unsigned)G) {
              __builtin_amdgcn_s_sleep(1);
              if (__builtin_amdgcn_s_memrealtime() - t0 > kBnSpinTicks) {
                atomicOr(p.xerr, 1);
                break;
              }
            }
          }
        }
        __syncthreads();
        constexpr int kCols = SH::T0F * 16, kPc = RT / 4;  // a member's columns; 4-row pieces per column
        for (int it = t; it < (G - 1) * kCols * kPc; it += kRowThreads) {
          const int pi = it / (kCols * kPc), rem = it - pi * (kCols * kPc);
          const int q = pi < mbr ? pi : pi + 1;  // the peer member
          const int cc = rem / kPc, r4 = (rem - cc * kPc) * 4;
          const unsigned long long v8 = __hip_atomic_load(
              (xg_u64*)(p.xbuf + (((size_t)rtile * G + q) * kCols + cc) * 16 + r4), __ATOMIC_RELAXED,
              __HIP_MEMORY_SCOPE_AGENT);
          const int c = q * kCols + cc;
#pragma unroll
          for (int i = 0; i < 4; ++i) O[(r4 + i) * ldo + c] = (uint16_t)(v8 >> (16 * i));
        }
        if constexpr (RT < kRowTile) {  // padding rows of the peers' columns: zero MFMA operands
          for (int it = t; it < (kRowTile - RT) * (G - 1) * kCols; it += kRowThreads) {
            const int r = RT + it / ((G - 1) * kCols), k = it - (r - RT) * ((G - 1) * kCols);
            const int q = k / kCols < mbr ? k / kCols : k / kCols + 1;
            O[r * ldo + q * kCols + (k % kCols)] = 0;
          }
        }
      }
    }
    if constexpr (!SH::kStatic || BN) {
      if (p.bn && train) {
        // batch moments of r over all B rows: this workgroup's (mean, M2) per column → grid
        // barrier → Chan's combination in workgroup order (deterministic) → normalise, dropout
        lds_barrier();
        const float* R = reinterpret_cast<const float*>(smem + L.bnr[l]);
        float* ST = reinterpret_cast<float*>(smem + L.bnst[l]);
        const int nv = bn_rows(p.B, blockIdx.x);
        float2* part = reinterpret_cast<float2*>(p.bn_part) + (size_t)l * gridDim.x * p.bn_dmax;
        for (int c = t; c < Dout; c += kRowThreads) {
          float sm = 0.f;
          for (int r = 0; r < nv; ++r) sm += R[r * Dout + c];
          const float m = nv ? sm / (float)nv : 0.f;
          float q = 0.f;
          for (int r = 0; r < nv; ++r) {
            const float d = R[r * Dout + c] - m;
            q += d * d;
          }
          part[(size_t)blockIdx.x * p.bn_dmax + c] = make_float2(m, q);
        }
        bn_grid_sync(p, (unsigned)l);
        for (int c = t; c < Dout; c += kRowThreads) {
          float sm = 0.f;
          for (int w = 0; w < (int)gridDim.x; ++w) sm += (float)bn_rows(p.B, w) * part[(size_t)w * p.bn_dmax + c].x;
          const float mean = sm / (float)p.B;
          float m2 = 0.f;
          for (int w = 0; w < (int)gridDim.x; ++w) {
            const float2 v = part[(size_t)w * p.bn_dmax + c];
            const float d = v.x - mean;
            m2 += v.y + (float)bn_rows(p.B, w) * d * d;
          }
          ST[c] = mean;
          ST[Dout + c] = rsqrtf(m2 / (float)p.B + p.bn_eps);
          if (blockIdx.x == 0 && !(p.step && (*p.step & kHaltStepBit))) {  // moving averages (not in a
            // halted step, optim.h); the variance one is unbiased (TF fused BN)
            p.bn_mean[l][c] = p.bn_mean[l][c] * p.bn_decay + mean * (1.f - p.bn_decay);
            p.bn_var[l][c] = p.bn_var[l][c] * p.bn_decay + (m2 / (float)max(p.B - 1, 1)) * (1.f - p.bn_decay);
          }
        }
        lds_barrier();
        for (int it = t; it < (kRowTile / 4) * Dout; it += kRowThreads) {
          const int rg = it / Dout, c = it - rg * Dout;
          Philox4 bits{0u, 0u, 0u, 0u};
          if (drop) bits = dropout_bits(p.seed, (uint32_t)l, step, (uint32_t)(row0 + 4 * rg) >> 2, (uint32_t)c);
          const float mean = ST[c], rstd = ST[Dout + c], ga = p.bn_gamma[l][c], be = p.bn_beta[l][c];
          float hv[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 4 * rg + i;
            float a = (R[r * Dout + c] - mean) * rstd * ga + be;
            if (drop) a = keep_from_bits(pick4(bits, i), keep) ? a * inv_keep : 0.f;
            if (row0 + r >= p.B) a = 0.f;
            hv[i] = a;
            O[r * ldo + c] = f2bf(a);
          }
          *reinterpret_cast<uint2*>(p.actT[l + 1] + act_swz(c, row0 + 4 * rg, Bp)) =
              make_uint2(pack_bf2(hv[0], hv[1]), pack_bf2(hv[2], hv[3]));
        }
      }
    }
  }
  lds_barrier();

  ROWS_STAMP(9);
  // ---- phase D: output layer + loss head (wave 0) ----------------------------------------------
  if (wave == 0) {
    const int Dn = sh.dim(NL);
    const uint16_t* H = reinterpret_cast<const uint16_t*>(smem + L.act[NL]);
    const int ldh = L.lda[NL];
    const int r = lane >> 2, q = lane & 3;
    float s = 0.f;
    for (int c = q; c < Dn; c += 4) s += bf2f(H[r * ldh + c]) * s_prm[L.prm_wout + c];
    s += dpp_f<0xB1>(s);  // lane ^ 1 (quad_perm; the same sums as the xor shuffles)
    s += dpp_f<0x4E>(s);  // lane ^ 2
    if (q == 0) {
      const int gr = row0 + r;
      const bool valid = r < RT && gr < p.B;
      const float y = s_ylin[r] + s + s_prm[L.prm_bout];
      const float tl = s_prm[L.prm_lab + r];
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
      if (valid && lead) {
        p.prob[gr] = pr;
        if (p.loss_rows) p.loss_rows[gr] = loss;
      }
      if (train && r < RT && lead) p.g_out[gr] = g;
    }
  }
  if (!train) return;
  // fp8: s_amax now collects the per-row max |dz| of the input layer's output gradient (the A
  // operand of the fp8 dgrad GEMM below); forward layer 0, its last reader, is done
  if (FP8 && t < kRowTile) s_amax[t] = 0.f;

  // phase F's embedding rows are re-read here, long before they are needed (hidden by phase E);
  // kLateBw0 shapes re-read them after the layer-0 backward GEMM (register budget)
  // phase F's items: (row, field, float4 column); split: only this member's FG fields — item
  // (r, fl, c4) is field mbr·FG + fl, past F on the last member (no item)
  constexpr int FI = (G > 1) ? SH::FG : 0;  // fields per member (0: all F)
  const int nitemsF = RT * (G > 1 ? FI : F) * KP4;
  constexpr int UF = gather_units_f<SH, RT, KP4>();
  auto item_rf = [&](int idx) {  // lookup (r·F + f) of item idx
    if constexpr (G > 1) {
      const int rfl = idx / KP4, r = rfl / FI, f = min(mbr * FI + (rfl - r * FI), F - 1);
      return r * F + f;
    } else {
      return idx / KP4;
    }
  };
  float4 rowsF[UF];
  if constexpr (!SH::kLateBw0) {
#pragma unroll
    for (int u = 0; u < UF; ++u) {
      const int idx = min(u * kRowThreads + t, nitemsF - 1);
      const int rf = item_rf(idx), c4 = idx % KP4;
      rowsF[u] = tbl_load4<BT>(emb4, (size_t)s_ids[rf] * KP4 + c4);
    }
  }
  lds_barrier();

  // ---- phase E: backward through the MLP ------------------------------------------------------
  uint16_t* dz_cur = reinterpret_cast<uint16_t*>(smem + L.dzA);
  uint16_t* dz_nxt = reinterpret_cast<uint16_t*>(smem + L.dzB);
  const int ldz = L.ldz;
  // batch-norm backward of hidden layer l from dy (LDS, gradient w.r.t. the BN output before
  // dropout): column sums Σdy, Σdy·x̂ over the batch (grid barrier), then
  // dz = 1[r > 0]·γ·rstd·(dy − mean(dy) − x̂·mean(dy·x̂)) → bf16 tile `dst` + dzT[l+1]
  auto bn_backward = [&](int l, uint16_t* dst) {
    lds_barrier();
    const int D = sh.dim(l + 1);
    const float* R = reinterpret_cast<const float*>(smem + L.bnr[l]);
    const float* ST = reinterpret_cast<const float*>(smem + L.bnst[l]);
    const float* DY = reinterpret_cast<const float*>(smem + L.bndy);
    float* TOT = reinterpret_cast<float*>(smem + L.bntot);
    const int nv = bn_rows(p.B, blockIdx.x);
    const int kb = NL + (NL - 1 - l);
    float2* part = reinterpret_cast<float2*>(p.bn_part) + (size_t)kb * gridDim.x * p.bn_dmax;
    for (int c = t; c < D; c += kRowThreads) {
      float s1 = 0.f, s2 = 0.f;
      for (int r = 0; r < nv; ++r) {
        const float dy = DY[r * D + c];
        s1 += dy;
        s2 += dy * (R[r * D + c] - ST[c]) * ST[D + c];
      }
      part[(size_t)blockIdx.x * p.bn_dmax + c] = make_float2(s1, s2);
    }
    bn_grid_sync(p, (unsigned)kb);
    for (int c = t; c < D; c += kRowThreads) {
      float s1 = 0.f, s2 = 0.f;
      for (int w = 0; w < (int)gridDim.x; ++w) {
        const float2 v = part[(size_t)w * p.bn_dmax + c];
        s1 += v.x;
        s2 += v.y;
      }
      TOT[c] = s1 / (float)p.B;
      TOT[D + c] = s2 / (float)p.B;
      if (blockIdx.x == 0) {
        p.bn_grad[(size_t)(2 * l) * p.bn_dmax + c] = s2;      // d γ
        p.bn_grad[(size_t)(2 * l + 1) * p.bn_dmax + c] = s1;  // d β
      }
    }
    lds_barrier();
    for (int it = t; it < (kRowTile / 4) * D; it += kRowThreads) {
      const int rg = it / D, c = it - rg * D;
      const float mean = ST[c], rstd = ST[D + c], gs = p.bn_gamma[l][c] * rstd;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * rg + i;
        const float rv = R[r * D + c];
        const float xh = (rv - mean) * rstd;
        const float dz = gs * (DY[r * D + c] - TOT[c] - xh * TOT[D + c]);
        v[i] = (rv > 0.f && row0 + r < p.B) ? dz : 0.f;
        dst[r * ldz + c] = f2bf(v[i]);
      }
      *reinterpret_cast<uint2*>(p.dzT[l + 1] + act_swz(c, row0 + 4 * rg, Bp)) =
          make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
    }
  };
  bool bn_head = false;
  if constexpr (!SH::kStatic || BN) {
    if (p.bn) {  // dy of the last hidden layer's BN output: g·w_out through its dropout mask
      const int l = NL - 1, Dn = sh.dim(NL);
      float* DY = reinterpret_cast<float*>(smem + L.bndy);
      const float keep = p.keep[l], inv_keep = 1.f / keep;
      const bool drop = keep < 1.f;
      for (int it = t; it < (kRowTile / 4) * Dn; it += kRowThreads) {
        const int rg = it / Dn, c = it - rg * Dn;
        Philox4 bits{0u, 0u, 0u, 0u};
        if (drop) bits = dropout_bits(p.seed, (uint32_t)l, step, (uint32_t)(row0 + 4 * rg) >> 2, (uint32_t)c);
        const float wc = s_prm[L.prm_wout + c];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * rg + i;
          const bool kept = !drop || keep_from_bits(pick4(bits, i), keep);
          DY[r * Dn + c] = kept ? s_g[r] * wc * inv_keep : 0.f;
        }
      }
      bn_backward(l, dz_cur);
      bn_head = true;
    }
  }
  if (!bn_head) {
    const int a = NL, Dn = sh.dim(a);
    const uint16_t* H = reinterpret_cast<const uint16_t*>(smem + L.act[a]);
    const int ldh = L.lda[a];
    const float inv_keep = 1.f / p.keep[a - 1];
    for (int it = t; it < Dn * 4; it += kRowThreads) {
      const int rg = it / Dn, c = it - rg * Dn;
      const float wc = s_prm[L.prm_wout + c];
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = rg * 4 + i;
        const float h = bf2f(H[r * ldh + c]);
        v[i] = h > 0.f ? s_g[r] * wc * inv_keep : 0.f;
        dz_cur[r * ldz + c] = f2bf(v[i]);
        if (FP8 && a == 1) atomicMax(reinterpret_cast<unsigned*>(s_amax) + r, __float_as_uint(fabsf(bf2f(f2bf(v[i])))));
      }
      if (rg * 4 < RT && lead)
        *reinterpret_cast<uint2*>(p.dzT[a] + act_swz(c, row0 + rg * 4, Bp)) =
            make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
    }
  }
#pragma unroll
  for (int a = NL; a >= 1; --a) {
    lds_barrier();
    if (a == NL) ROWS_STAMP(10);
    const int li = a - 1, Dout = sh.dim(a), Din = sh.dim(li);

    // (split: the layer-0 dgrad tiles of this member's fields)
    const int ntb = li == 0 ? tb0 : 0;
    const int ntiles = li == 0 ? tb1 : (Din >> 4);
    constexpr int NJ = SH::kStatic ? (SH::NJB0 > 1 ? SH::NJB0 : 1) : 4;
    for (int nt0 = ntb + wave; nt0 < ntiles; nt0 += NJ * kWaves) {
      f32x4 accs[NJ];
      if constexpr (SH::kStatic) {
        const uint16_t* ap = dz_cur + (lane & 15) * ldz + 8 * (lane >> 4);
#pragma unroll
        for (int j = 0; j < NJ; ++j) accs[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (li == 0 && SH::kLateBw0) {
          if constexpr (SH::kLateBw0 && !FP8) {  // (the launcher keeps fp8 off these shapes)
          // tile-major, software-pipelined over the NJB0H fragment slots (see CtShape::NJB0H)
          bf16x8 av[SH::KSB0];
#pragma unroll
          for (int u = 0; u < SH::KSB0; ++u) av[u] = ld_frag(ap + 32 * u);
          // (diagnostics, ablate bits 4 / 5: only the first 1/2 or 1/4 of the tiles, as above)
          const int jcut = (DIAG && (ablate & 48)) ? ((ablate & 32) ? (NJ + 3) / 4 : (NJ + 1) / 2) : NJ;
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int slot = j % SH::NJB0H;
            if (nt0 + kWaves * j < ntiles && j < jcut) {
#pragma unroll
              for (int u = 0; u < SH::KSB0; ++u) accs[j] = mfma16x16x32(av[u], bw0[slot][u], accs[j]);
            }
            if (j + SH::NJB0H < SH::NJB0 && j + SH::NJB0H < jcut) {
              const int nt = min(tb0 + wave + kWaves * (j + SH::NJB0H), tb1 - 1);
#pragma unroll
              for (int u = 0; u < SH::KSB0; ++u) bw0[slot][u] = ld_w0<FP8>(p.Wbs[0], p.w8.b, frag_at(nt, u, sh.dim(1), lane));
            }
          }
          }
        } else if (li == 0) {
          if constexpr (FP8) {
            // fp8-e4m3 dgrad dh0 = dz·W0ᵀ: dz quantised per row (s_amax), W0ᵀ pre-quantised (one
            // scale per tensor, w8inv); de-scaled after
            // (dz's 4 k-steps are quantised per wave: a shared LDS copy would cost a barrier)
            const float sa = kFp8Max / fmaxf(s_amax[lane & 15], 1e-30f);
#pragma unroll
            for (int u = 0; u < SH::KSB0; ++u) {
              const long av = quant_fp8x8(ld_frag(ap + 32 * u), sa);
#pragma unroll
              for (int j = 0; j < NJ; ++j)
                if (j < SH::NJB0H && nt0 + kWaves * j < ntiles)
                  accs[j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(av, bw0[j][u], accs[j], 0, 0, 0);
            }
            const int rbq = (lane >> 4) * 4;
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
              for (int i = 0; i < 4; ++i) accs[j][i] *= (fmaxf(s_amax[rbq + i], 1e-30f) / kFp8Max) * w8inv;
          } else {
#pragma unroll
            for (int u = 0; u < SH::KSB0; ++u) {
              const bf16x8 av = ld_frag(ap + 32 * u);
#pragma unroll
              for (int j = 0; j < NJ; ++j)
                if (j < SH::NJB0H && nt0 + kWaves * j < ntiles) accs[j] = mfma16x16x32(av, bw0[j][u], accs[j]);
            }
          }
        } else if (li == 1) {
#pragma unroll
          for (int u = 0; u < SH::KSB1; ++u) {
            const bf16x8 av = ld_frag(ap + 32 * u);
#pragma unroll
            for (int j = 0; j < SH::NTB1; ++j) accs[j] = mfma16x16x32(av, bw1[j][u], accs[j]);
          }
        } else {
#pragma unroll
          for (int u = 0; u < SH::KSB2; ++u) accs[0] = mfma16x16x32(ld_frag(ap + 32 * u), bw2[u], accs[0]);
        }
        (void)zero8;
      } else {
        rowtile_gemm<NJ, 4>(dz_cur, ldz, p.Wb[li], Dout, ntiles, nt0, kWaves, Dout, lane, accs, p.Wbs[li]);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int nt = nt0 + kWaves * j;
        if (nt >= ntiles) continue;
        if (SH::kStatic && li > 0 && j >= (li == 1 ? SH::NTB1 : 1)) continue;
        const f32x4 acc = accs[j];
        const int c = nt * 16 + (lane & 15), rb = (lane >> 4) * 4;
        if (li >= 1) {
          if constexpr (!SH::kStatic || BN) {
            if (p.bn) {  // gradient w.r.t. layer li-1's BN output, through its dropout mask
              float* DY = reinterpret_cast<float*>(smem + L.bndy);
              const float keep = p.keep[li - 1], inv_keep = 1.f / keep;
              const bool drop = keep < 1.f;
              Philox4 bits{0u, 0u, 0u, 0u};
              if (drop) bits = dropout_bits(p.seed, (uint32_t)(li - 1), step, (uint32_t)(row0 + rb) >> 2, (uint32_t)c);
#pragma unroll
              for (int i = 0; i < 4; ++i)
                DY[(rb + i) * Din + c] = (!drop || keep_from_bits(pick4(bits, i), keep)) ? acc[i] * inv_keep : 0.f;
              continue;
            }
          }
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
          if (FP8 && li == 1) {  // per-row max |bf16 dz| over this tile's 16 columns → s_amax
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              float m = fabsf(bf2f(f2bf(v[i])));
#pragma unroll
              for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
              if ((lane & 15) == 0) atomicMax(reinterpret_cast<unsigned*>(s_amax) + rb + i, __float_as_uint(m));
            }
          }
          if (rb < RT && lead)
            *reinterpret_cast<uint2*>(p.dzT[li] + act_swz(c, row0 + rb, Bp)) =
                make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) s_f32[(rb + i) * D0p + c] = acc[i];
        }
      }
    }
    if constexpr (!SH::kStatic || BN) {
      if (p.bn && li >= 1) bn_backward(li - 1, dz_nxt);
    }
    uint16_t* tmp = dz_cur;
    dz_cur = dz_nxt;
    dz_nxt = tmp;
  }
  lds_barrier();
  ROWS_STAMP(11);

  // ---- phase F: FM backward → per-lookup gradient rows -----------------------------------------
  for (int base = 0; base < nitemsF; base += kRowThreads * UF) {
    if (base > 0 || SH::kLateBw0) {  // more rows than one batch (large F·Kp), or not prefetched
#pragma unroll
      for (int u = 0; u < UF; ++u) {
        const int idx = min(base + u * kRowThreads + t, nitemsF - 1);
        const int rf = item_rf(idx), c4 = idx % KP4;
        rowsF[u] = tbl_load4<BT>(emb4, (size_t)s_ids[rf] * KP4 + c4);
      }
    }
    // all four items' gradient rows are computed in straight-line code (clamped items, LDS reads
    // and the prefetched rows) before the first store: one wait for rowsF, and no store of an
    // earlier item is waited for by a later one
    float o[UF][4];
    int dst[UF];
    bool ok[UF];
#pragma unroll
    for (int u = 0; u < UF; ++u) {
      const int idx0 = base + u * kRowThreads + t;
      const int idx = min(idx0, nitemsF - 1);
      const int rf = item_rf(idx), c4 = idx % KP4;
      const int r = fdiv(rf, magicF), f = rf - r * F;
      ok[u] = idx0 < nitemsF && row0 + r < p.B;
      if constexpr (G > 1) ok[u] = ok[u] && mbr * FI + (idx / KP4) % FI < F;
      const float g = s_g[r], x = s_vals[rf];
      const float* S = s_S + r * K;
      const float* dh = s_f32 + r * D0p + f * K;
      const float vv[4] = {rowsF[u].x, rowsF[u].y, rowsF[u].z, rowsF[u].w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int k = c4 * 4 + c;
        o[u][c] = (k < K) ? x * (g * (S[min(k, K - 1)] - vv[c] * x) + dh[min(k, K - 1)]) : ((k == K) ? g * x : 0.f);
      }
      dst[u] = s_pos[rf] * KP4 + c4;
    }
    if (G == 1 && p.dedup) {  // the tile's rows stay in LDS: summed per group below (no split)
      if (L.gr == L.f32) lds_barrier();  // (over dh0: every thread's reads of it are done)
      float4* s_gr = reinterpret_cast<float4*>(smem + L.gr);
#pragma unroll
      for (int u = 0; u < UF; ++u) {
        const int idx0 = base + u * kRowThreads + t;
        if (ok[u]) s_gr[idx0] = make_float4(o[u][0], o[u][1], o[u][2], o[u][3]);
      }
    } else {
#pragma unroll
      for (int u = 0; u < UF; ++u)
        if (ok[u]) {
          if (p.wt & 1) {  // write-through (sc1)
            const f32x4 v = {o[u][0], o[u][1], o[u][2], o[u][3]};
            __builtin_amdgcn_raw_buffer_store_b128(v, wt_contrib, dst[u] * 16, 0, 16);
          } else {
            reinterpret_cast<float4*>(p.contrib)[dst[u]] = make_float4(o[u][0], o[u][1], o[u][2], o[u][3]);
          }
        }
    }
  }
  if (G == 1 && p.dedup) {
    // per-tile dedup: each group (equal id within this row tile) sums its lookups' rows in lookup
    // order — head first, then along the nxt chain — and stores ONE row at its compacted index
    lds_barrier();
    const float4* s_gr = reinterpret_cast<const float4*>(smem + L.gr);
    for (int idx = t; idx < nitemsF; idx += kRowThreads) {
      const int rf = idx / KP4, c4 = idx - rf * KP4;
      const int c = s_pos[rf];
      if (c < 0 || row0 + fdiv(rf, magicF) >= p.B) continue;  // not a group head / padding row
      float4 acc = s_gr[idx];
      for (int j = s_nxt[rf]; j >= 0; j = s_nxt[j]) {
        const float4 v = s_gr[j * KP4 + c4];
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
      }
      reinterpret_cast<float4*>(p.contrib)[(size_t)c * KP4 + c4] = acc;
    }
  }
  lds_barrier();
  ROWS_STAMP(12);
  // DP fused push: the previous merge (last reader of this rank's receive slots) is done.  Raised
  // by the last instructions of workgroup 0 (the exchange-counter load it needs would otherwise
  // hold wave 0 for a memory round trip in front of the id loads); the peers' producers that
  // read it store only at the end of their step tail.
  if (blockIdx.x == 0 && t == 0) {
    if (p.push.W > 0) push_signal_ready(p.push);
    if (p.push2.W > 0) push_signal_ready(p.push2);
    if (p.push3.W > 0) push_signal_ready(p.push3);
  }
  if constexpr (!SH::kStatic || BN) {
    if (p.bn) bn_grid_exit(p);
  }
  // diagnostics (ablate bit 3): one grid-wide barrier after the step's row work, as a persistent
  // rows → tail kernel would need — its in-launch price against the kernel boundary it would replace
  // (profiles/r5_persistent_step.md; p.bn_sync / bn_error set by tools/diag_phases.py)
  if (DIAG && (ablate & 8) && p.bn_sync != nullptr) {
    ROWS_STAMP(13);
    bn_grid_sync(p, 0);
    ROWS_STAMP(14);
    bn_grid_exit(p);
  }
  if (DIAG && p.stamps != nullptr) {
    lds_barrier();
    if (t < 15) p.stamps[blockIdx.x * 16 + t] = s_stamp[t];
  }
}

// ------------------------------------------------------------------------------------------------
static int align16(int x) { return (x + 15) & ~15; }

RowsLds rows_lds_layout(const int* dims, int nl, int F, int K, int bn, int dedup_kp, int rt, bool gr_alias,
                        bool fp8) {
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
  L.pos = take(kRowTile * F * 4);
  L.S = take(kRowTile * K * 4);
  L.ylin = take(kRowTile * 4);
  L.amax = take(kRowTile * 4);
  L.g = take(kRowTile * 4);
  int maxh = 0;
  for (int a = 0; a <= nl; ++a) {
    L.lda[a] = dims[a] + 8;  // +16 B per row breaks the power-of-two row stride
    L.act[a] = take(kRowTile * L.lda[a] * 2);
    if (a > 0 && dims[a] > maxh) maxh = dims[a];
  }
  L.ldz = maxh + 8;
  if (2 * L.ldz <= L.lda[0]) {  // h0's tile is dead after the first layer: the dz tiles reuse it
    L.dzA = L.act[0];
    L.dzB = L.act[0] + kRowTile * L.ldz * 2;
  } else {
    L.dzA = take(kRowTile * L.ldz * 2);
    L.dzB = take(kRowTile * L.ldz * 2);
  }
  L.f32 = take(kRowTile * dims[0] * 4);
  if (fp8) {
    L.ldq = dims[0] + 16;
    L.q8 = take(kRowTile * L.ldq);
  }
  if (dedup_kp > 0) {
    L.nxt = take(kRowTile * F * 4);
    // the tile's gradient rows: over the f32 scratch (dh0, dead once phase F has read it — the
    // compile-time-shape kernels read all of it before the first row is stored), else their own
    const int gb = rt * F * dedup_kp * 4;
    L.gr = (gr_alias && gb <= kRowTile * dims[0] * 4) ? L.f32 : take(gb);
  }
  if (bn) {
    for (int l = 0; l < nl; ++l) {
      L.bnr[l] = take(kRowTile * dims[l + 1] * 4);
      L.bnst[l] = take(2 * dims[l + 1] * 4);
    }
    L.bndy = take(kRowTile * maxh * 4);
    L.bntot = take(2 * maxh * 4);
  }
  int n = 0;
  for (int l = 0; l < nl; ++l) {
    L.prm_bias[l] = n;
    n += dims[l + 1];
  }
  L.prm_wout = n;
  n += dims[nl];
  L.prm_bout = n++;
  L.prm_fmb = n++;
  L.prm_lab = n;
  n += kRowTile;
  L.prm_n = n;
  L.prm = take(n * 4);
  L.total = off;
  return L;
}

template <int KP4, class SH, bool FP8, int MODE, bool DIAG, bool BT, int RT = kRowTile, bool BN = false>
static void launch_rows_impl(const RowsParams& p, hipStream_t stream) {
  auto kern = deepfm_rows_kernel<KP4, SH, FP8, MODE, DIAG, BT, RT, BN>;
  static bool attr_set = false;
  static int max_dyn = 0;
  if (!attr_set) {  // allow > 64 KiB of dynamic LDS (160 KiB per CU on gfx950, minus the static part)
    hipFuncAttributes fa{};
    ROCFM_HIP_CHECK(hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(kern)));
    max_dyn = 160 * 1024 - (int)fa.sharedSizeBytes;
    ROCFM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, max_dyn));
    attr_set = true;
  }
  ROCFM_REQUIRE(p.lds.total <= max_dyn, "deepfm_rows: LDS layout exceeds the 160 KiB per workgroup");
  if (p.bn && p.train) {  // grid barriers: every workgroup must be resident at once
    int per_cu = 0, dev = 0, cus = 0;
    ROCFM_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern),
                                                                 kRowThreads, p.lds.total));
    ROCFM_HIP_CHECK(hipGetDevice(&dev));
    ROCFM_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    // the occupancy query can over-report by one block per CU: trust one fewer when it says > 1
    const int limit = cus * (per_cu > 1 ? per_cu - 1 : per_cu);
    ROCFM_REQUIRE(p.Bp / kRowTile <= limit, "deepfm_rows: batch_norm needs every workgroup of the batch resident "
                                            "at once (batch too large for one launch; use engine=torch)");
  }
  hipLaunchKernelGGL(kern, dim3(p.Bp / RT * SH::G), dim3(kRowThreads), p.lds.total, stream, p);
}

// Static shapes: branch-free train / inference kernels; the diagnostic (stamps, ablations)
// instantiation only for the benchmark shape's training kernel.
template <int KP4, class SH, bool BT, int RT>
static void launch_rows_t(const RowsParams& p, hipStream_t stream) {
  if constexpr (SH::kStatic) {
    if (p.bn) {  // batch_norm: 16-row tiles, f32 table, bf16 (static_ok)
      if constexpr (!BT && RT == kRowTile) {
        if (p.train)
          launch_rows_impl<KP4, SH, false, kTrain, false, false, kRowTile, true>(p, stream);
        else
          launch_rows_impl<KP4, SH, false, kInfer, false, false, kRowTile, true>(p, stream);
        return;
      } else {
        throw std::logic_error("deepfm_rows: batch_norm kernels are built for 16-row tiles and f32 tables");
      }
    }
    const bool diag = p.stamps != nullptr || p.ablate != 0;
    if (diag) {
      if constexpr (SH::F == 39 && (SH::K == 10 || SH::K == 32) && SH::nl == 3 && !BT) {
        ROCFM_REQUIRE(!p.fp8 && p.train, "deepfm_rows: diagnostics are built for the bf16 training kernel only");
        launch_rows_impl<KP4, SH, false, kTrain, true, false, RT>(p, stream);
        return;
      } else {
        throw std::invalid_argument("deepfm_rows: diagnostics (stamps/ablate) need a 39-field k=10 or k=32 "
                                    "3-layer shape and an f32 table");
      }
    }
    if (p.fp8) {
      if constexpr (SH::kLateBw0) {  // the fp8 quantisation of a wide input layer's fragments spills
        throw std::invalid_argument("deepfm_rows: compute_dtype=fp8 supports input layers up to 512 wide");
      } else {
        if (p.train)
          launch_rows_impl<KP4, SH, true, kTrain, false, BT, RT>(p, stream);
        else
          launch_rows_impl<KP4, SH, true, kInfer, false, BT, RT>(p, stream);
        return;
      }
    }
    if (p.train)
      launch_rows_impl<KP4, SH, false, kTrain, false, BT, RT>(p, stream);
    else
      launch_rows_impl<KP4, SH, false, kInfer, false, BT, RT>(p, stream);
  } else {
    launch_rows_impl<KP4, SH, false, kDynamic, true, BT, RT>(p, stream);
  }
}

// rows per workgroup (RowsParams::row_tile, 0 = kDefaultRowTile): 8 doubles the workgroups of a
// batch (128 instead of 64 at B = 1024 on 256 CUs) at the same per-workgroup weight-fragment
// traffic — measured 35.9 → 33.3 µs per step in 20-step windows, 33.4 → 32.2 over 200 steps
// (profiles/r3_row_tile.md).  The runtime-shape kernel takes 16 or 8 (4 asks for 8 there), and 16
// with batch norm (its statistics partials are per 16-row workgroup).
constexpr int kDefaultRowTile = 8;
// wide input layers (F·K ≥ 1024: the reference's k = 32 shapes, whose row phases are bound by
// streaming the layer-0 weights through each CU): 4 examples per workgroup — 256 workgroups halve
// the gather / FM / FM-backward work per CU at the same weight stream (k = 32: 57.4 → 56.3 and
// 44.1 → 43.5 µs per step; k = 10 unchanged, profiles/r5_wgrad_swizzle.md)
static bool split_ok(const RowsParams& p);
static int row_tile_for(const RowsParams& p, bool is_static_shape) {
  if (is_static_shape && split_ok(p)) return 8;  // the row-tile split: 8-row tiles (2 × 128 workgroups)
  const int rt = p.row_tile ? p.row_tile : (is_static_shape && p.dims[0] >= 1024 ? 4 : kDefaultRowTile);
  if (p.bn) return kRowTile;  // batch-norm statistics partials are per 16-row workgroup
  if (is_static_shape) return rt;
  return rt == 4 ? 8 : rt;
}
template <int KP4, class SH>
static void launch_rows_tb(const RowsParams& p, hipStream_t stream) {
  const int rt = row_tile_for(p, SH::kStatic);
  if (p.tbl_bf16) {
    if constexpr (SH::kStatic)
      if (rt == 4) return launch_rows_t<KP4, SH, true, 4>(p, stream);
    if (rt == 8)
      launch_rows_t<KP4, SH, true, 8>(p, stream);
    else
      launch_rows_t<KP4, SH, true, 16>(p, stream);
  } else {
    if constexpr (SH::kStatic)
      if (rt == 4) return launch_rows_t<KP4, SH, false, 4>(p, stream);
    if (rt == 8)
      launch_rows_t<KP4, SH, false, 8>(p, stream);
    else
      launch_rows_t<KP4, SH, false, 16>(p, stream);
  }
}

// Compile-time-shape instantiations (the benchmark / notebook-style models, and the reference's
// flag defaults k=32, 256-128-64 — PS:52,62).  Anything else runs the runtime-shape kernel.
template <int F, int K, int D1, int D2, int D3>
static bool static_match(const RowsParams& p) {
  const int nl = D3 ? 3 : (D2 ? 2 : 1);
  if (p.F != F || p.K != K || p.nl != nl || p.dims[1] != D1 || (nl >= 2 && p.dims[2] != D2) ||
      (nl >= 3 && p.dims[3] != D3))
    return false;
  for (int l = 0; l < nl; ++l)
    if (!p.WTs[l] || !p.Wbs[l]) return false;  // the static kernels load the frag_swz weight copies
  return true;
}

template <int F, int K, int D1, int D2, int D3>
static bool try_static(const RowsParams& p, hipStream_t stream) {
  if (!static_match<F, K, D1, D2, D3>(p)) return false;
  constexpr int KP4 = (K + 1 + 3) / 4;
  launch_rows_tb<KP4, CtShape<F, K, D1, D2, D3>>(p, stream);
  return true;
}

// The row-tile split (2 workgroups per 8-row tile) for the training kernel of the reference's flag
// defaults (39 × 32 → 256-128-64: W0 is 624 KiB; profiles/r5_layer0_split.md), bf16 MFMA, no
// per-tile dedup, no batch norm.  ROCFM_ROW_SPLIT / RowsParams::split = 2 asks for it.
static bool split_ok(const RowsParams& p) {
  return p.split == 2 && p.train && !p.fp8 && !p.bn && !p.dedup && !p.force_generic && p.xbuf && p.xctr &&
         p.xerr && static_match<39, 32, 256, 128, 64>(p) && (p.row_tile == 0 || p.row_tile == 8) &&
         (p.Bp / 8) % 8 == 0;
}
static bool try_split(const RowsParams& p, hipStream_t stream) {
  if (!split_ok(p)) return false;
  using SH = CtShape<39, 32, 256, 128, 64, 2>;
  constexpr int KP4 = 9;
  const bool diag = p.stamps != nullptr || p.ablate != 0;
  if (p.tbl_bf16) {
    if (diag) throw std::invalid_argument("deepfm_rows: split diagnostics need an f32 table");
    launch_rows_impl<KP4, SH, false, kTrain, false, true, 8>(p, stream);
  } else if (diag) {
    launch_rows_impl<KP4, SH, false, kTrain, true, false, 8>(p, stream);
  } else {
    launch_rows_impl<KP4, SH, false, kTrain, false, false, 8>(p, stream);
  }
  return true;
}

// batch_norm runs the compile-time-shape kernels too, with an f32 table and bf16 MFMA
static bool static_ok(const RowsParams& p) { return !p.force_generic && !(p.bn && (p.tbl_bf16 || p.fp8)); }

static bool is_static(const RowsParams& p) {
  return static_ok(p) &&
         (static_match<39, 10, 128, 64, 32>(p) || static_match<39, 8, 128, 64, 32>(p) ||
          static_match<39, 12, 128, 64, 32>(p) || static_match<39, 10, 64, 32, 0>(p) ||
          static_match<39, 32, 128, 64, 32>(p) || static_match<39, 32, 256, 128, 64>(p));
}

// Examples per workgroup the launcher will use for these parameters (the per-tile dedup of the side
// chain must cut the same tiles).
int deepfm_rows_split(const RowsParams& p) { return static_ok(p) && split_ok(p) ? 2 : 1; }

int deepfm_rows_tile(const RowsParams& p) {
  return row_tile_for(p, is_static(p));
}

bool deepfm_rows_static(const RowsParams& p) { return is_static(p); }

RowsLds rows_lds_layout_for(const RowsParams& p) {
  return rows_lds_layout(p.dims, p.nl, p.F, p.K, p.bn, p.dedup ? p.Kp : 0, deepfm_rows_tile(p), is_static(p),
                         p.fp8 != 0 && is_static(p));
}

void launch_deepfm_rows(RowsParams p, hipStream_t stream) {
  ROCFM_REQUIRE(p.nl >= 1 && p.nl <= kMaxHidden, "deepfm_rows: 1..6 hidden layers supported");
  ROCFM_REQUIRE(p.Kp % 4 == 0 && p.Kp >= p.K + 1 && p.Kp <= 64, "deepfm_rows: Kp must be a multiple of 4, > K, <= 64");
  ROCFM_REQUIRE(p.F >= 1 && p.F <= 64, "deepfm_rows: field_size must be in [1, 64]");
  ROCFM_REQUIRE(p.dims[0] % 32 == 0 && p.dims[0] >= p.F * p.K, "deepfm_rows: dims[0] = round_up(F*K, 32)");
  for (int a = 1; a <= p.nl; ++a) ROCFM_REQUIRE(p.dims[a] % 32 == 0, "deepfm_rows: hidden dims padded to 32");
  ROCFM_REQUIRE(p.Bp % kRowTile == 0 && p.Bp >= p.B, "deepfm_rows: Bp must be a multiple of 16 and >= B");
  ROCFM_REQUIRE((p.Bp % 64) == 0 || !p.train, "deepfm_rows: training needs Bp % 64 == 0");
  p.magicF = (uint32_t)((1ull << 32) / (uint64_t)p.F + 1ull);
  ROCFM_REQUIRE(p.row_tile == 0 || p.row_tile == 4 || p.row_tile == 8 || p.row_tile == 16,
                "deepfm_rows: row_tile must be 0, 4, 8 or 16");
  ROCFM_REQUIRE(!p.dedup || (p.contrib_pos && p.contrib_nxt && !p.bn), "deepfm_rows: dedup needs contrib_pos / _nxt");
  ROCFM_REQUIRE(!p.fp8 || (p.w8.f && p.w8.b && p.w8.amax && p.w8.inv_scale),
                "deepfm_rows: compute_dtype=fp8 needs the pre-quantised input-layer copies (set_w8)");
  p.lds = rows_lds_layout_for(p);
  ROCFM_REQUIRE(p.lds.total <= 160 * 1024, "deepfm_rows: LDS budget exceeded (F*K too large)");
  if (p.Bp / kRowTile == 0) return;
  if (p.bn && p.train) {
    ROCFM_REQUIRE(p.bn_part && p.bn_grad && p.bn_sync && p.bn_error, "deepfm_rows: batch_norm buffers missing");
    for (int a = 1; a <= p.nl; ++a) ROCFM_REQUIRE(p.dims[a] <= p.bn_dmax, "deepfm_rows: bn_dmax < hidden dim");
  }
  if (static_ok(p)) {
    if (try_split(p, stream) || try_static<39, 10, 128, 64, 32>(p, stream) || try_static<39, 8, 128, 64, 32>(p, stream) ||
        try_static<39, 12, 128, 64, 32>(p, stream) || try_static<39, 10, 64, 32, 0>(p, stream) ||
        try_static<39, 32, 128, 64, 32>(p, stream) || try_static<39, 32, 256, 128, 64>(p, stream)) {
      ROCFM_HIP_CHECK(hipGetLastError());
      return;
    }
  }
  ROCFM_REQUIRE(!p.fp8, "deepfm_rows: compute_dtype=fp8 needs a compile-time-shape instantiation (39 fields, "
                        "k in {8,10,12,32}, MLP 128-64-32 or 64-32) or compute_dtype=bf16");
  switch (p.Kp / 4) {
#define ROCFM_KP4(N)                          \
  case N:                                     \
    launch_rows_tb<N, RtShape>(p, stream);    \
    break;
    ROCFM_KP4(1) ROCFM_KP4(2) ROCFM_KP4(3) ROCFM_KP4(4) ROCFM_KP4(5) ROCFM_KP4(6) ROCFM_KP4(7) ROCFM_KP4(8)
    ROCFM_KP4(9) ROCFM_KP4(10) ROCFM_KP4(11) ROCFM_KP4(12) ROCFM_KP4(13) ROCFM_KP4(14) ROCFM_KP4(15) ROCFM_KP4(16)
#undef ROCFM_KP4
    default:
      throw std::invalid_argument("deepfm_rows: unsupported Kp");
  }
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
