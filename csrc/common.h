// rocfm — common device/host helpers for the gfx950 (CDNA4) kernels.
//
// Every kernel in csrc/kernels is written for MI355X only: wave64, MFMA bf16 tiles,
// 160 KiB LDS per CU.  Launch wrappers take raw device pointers plus a hipStream_t so
// they can be captured into HIP graphs by the Python engine (rocfm/models/fused.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdexcept>
#include <string>

#define ROCFM_HIP_CHECK(expr)                                                        \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess)                                                           \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + \
                               " at " __FILE__ ":" + std::to_string(__LINE__));     \
  } while (0)

#define ROCFM_REQUIRE(cond, msg)                                   \
  do {                                                            \
    if (!(cond)) throw std::invalid_argument(std::string(msg));   \
  } while (0)

// Diagnostic phase stamps (cdna guide §7 "In-kernel stamps"): when a kernel's `stamps` pointer is
// non-null, thread 0 of each workgroup records the 100 MHz real-time counter at phase boundaries
// into stamps[blockIdx.x * 16 + i].  Null in production launches (one uniform branch per phase).
#define ROCFM_STAMP(ptr, i)                                                               \
  do {                                                                                    \
    if ((ptr) != nullptr && threadIdx.x == 0)                                             \
      (ptr)[blockIdx.x * 16 + (i)] = (unsigned long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)

// (diagnostics) where the workgroup runs: XCC id << 32 | HW_ID (CU id bits 8-11, SH bit 12, SE bits 13-15)
#define ROCFM_STAMP_HWID(ptr, i)                                                                   \
  do {                                                                                             \
    if ((ptr) != nullptr && threadIdx.x == 0)                                                      \
      (ptr)[blockIdx.x * 16 + (i)] = ((unsigned long long)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32) | \
                                     (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);         \
  } while (0)

namespace rocfm {

constexpr int kWave = 64;

typedef __attribute__((ext_vector_type(8))) short bf16x8;   // MFMA A/B fragment (4 VGPR), raw bits
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4;    // 16x16 MFMA accumulator
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;  // 16-B buffer-store payload
typedef __attribute__((ext_vector_type(16))) float f32x16;  // 32x32 MFMA accumulator

// D = A(16x32) · B(32x16) + C.  Lane l holds A[l&15][8(l>>4)+j] and B[8(l>>4)+j][l&15];
// C/D element i of lane l is (row (l>>4)*4+i, col l&15).
__device__ __forceinline__ f32x4 mfma16x16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                 c, 0, 0, 0);
}
// D = A(32x16) · B(16x32) + C.  Lane l holds A[l&31][8(l>>5)+j] and B[8(l>>5)+j][l&31];
// C/D register r of lane l is (row (r&3)+8(r>>2)+4(l>>5), col l&31).
__device__ __forceinline__ f32x16 mfma32x32x16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                 c, 0, 0, 0);
}

// f32 -> bf16, round-to-nearest-even.  NaN stays NaN (cdna guide: avoid the integer trick for NaN).
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

__host__ __device__ __forceinline__ int cdiv(int a, int b) { return (a + b - 1) / b; }

// ---- embedding-table storage: f32 or bf16 rows ([V][Kp], one float4 column group = 16 B or 8 B) ----
// bf16 tables are updated with stochastic rounding (unbiased: updates far below one bf16 ulp still
// move the weight in expectation); the random bits hash the element index and the step, so the
// result is reproducible.  Optimizer slots stay f32.
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint16_t f2bf_sr(float f, uint32_t r16) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return f2bf(f);  // inf / NaN
  u += r16 & 0xffffu;
  return (uint16_t)(u >> 16);
}
template <bool BT>
__device__ __forceinline__ float4 tbl_load4(const void* t, size_t i) {
  if constexpr (BT) {
    const uint2 h = reinterpret_cast<const uint2*>(t)[i];
    return make_float4(__uint_as_float(h.x << 16), __uint_as_float(h.x & 0xffff0000u), __uint_as_float(h.y << 16),
                       __uint_as_float(h.y & 0xffff0000u));
  } else {
    return reinterpret_cast<const float4*>(t)[i];
  }
}
template <bool BT>
__device__ __forceinline__ void tbl_store4(void* t, size_t i, float4 v, uint32_t step) {
  if constexpr (BT) {
    const uint32_t r0 = mix32((uint32_t)i * 2u ^ (step * 0x9e3779b9u)), r1 = mix32((uint32_t)i * 2u + 1u ^ (step * 0x9e3779b9u));
    uint2 h;
    h.x = (uint32_t)f2bf_sr(v.x, r0) | ((uint32_t)f2bf_sr(v.y, r0 >> 16) << 16);
    h.y = (uint32_t)f2bf_sr(v.z, r1) | ((uint32_t)f2bf_sr(v.w, r1 >> 16) << 16);
    reinterpret_cast<uint2*>(t)[i] = h;
  } else {
    reinterpret_cast<float4*>(t)[i] = v;
  }
}
__device__ __forceinline__ float4 tbl_load4_rt(const void* t, size_t i, bool bf) {
  return bf ? tbl_load4<true>(t, i) : tbl_load4<false>(t, i);
}
__device__ __forceinline__ void tbl_store4_rt(void* t, size_t i, float4 v, uint32_t step, bool bf) {
  if (bf)
    tbl_store4<true>(t, i, v, step);
  else
    tbl_store4<false>(t, i, v, step);
}

// MFMA B-fragment swizzle of a row-major bf16 matrix [R][C] (R % 16 == 0, C % 32 == 0): the
// 16-row × 32-column block (nt, u) is stored as 64 lanes × 8 contiguous elements in the order the
// 16x16x32 B operand wants them (lane l: row 16·nt + (l & 15), columns 32·u + 8·(l >> 4) .. +7),
// so one fragment load is a 1 KiB contiguous read (3.1× faster per workgroup than the strided
// row-major pattern, tools/frag_probe.py).
__host__ __device__ __forceinline__ size_t frag_swz(int r, int c, int C) {
  const int nt = r >> 4, rl = r & 15, u = c >> 5, cc = c & 31;
  return ((size_t)(nt * (C >> 5) + u) * 64 + rl + 16 * (cc >> 3)) * 8 + (cc & 7);
}
// Offset (elements) of fragment (nt, u) for this lane in a frag_swz matrix with C columns.
__device__ __forceinline__ size_t frag_at(int nt, int u, int C, int lane) {
  return ((size_t)(nt * (C >> 5) + u) * 64 + lane) * 8;
}
__host__ __device__ __forceinline__ int round_up(int a, int b) { return cdiv(a, b) * b; }

// MFMA-fragment-swizzled layout of the transposed activations / output gradients actT, dzT
// ([feature c][batch b], features padded to 32, Bp % 16 == 0) that the weight-gradient tiles read
// as 32x32x16 operands: the block (c / 32, b / 16) is 32 features × 16 batch rows = 512 elements
// stored as 64 lanes × 8 in the order the operand wants them (lane l: feature 32·(c/32) + (l & 31),
// batch rows 16·(b/16) + 8·(l >> 5) .. +7), so every fragment load of a wave is ONE contiguous 1 KiB
// read (the row-major [c][b] layout cost 32 strided 32-B pieces per load).  Any 8 batch rows b..b+7
// with b % 8 == 0 of one feature stay contiguous (the row kernel's 8-B / 16-B stores).
__host__ __device__ __forceinline__ size_t act_swz(int c, int b, int Bp) {
  return ((size_t)(c >> 5) * (size_t)(Bp >> 4) + (size_t)(b >> 4)) * 512 +
         (size_t)(((c & 31) + 32 * ((b >> 3) & 1)) * 8 + (b & 7));
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS operations (lgkmcnt(0)) and
// leaves its global stores in flight (no vmcnt(0)), unlike __syncthreads().  Valid where no wave
// reads, within the kernel, global memory another wave of the workgroup wrote (the fused kernels
// exchange data between waves only through LDS).  Global-load results are still waited for by the
// compiler at their first use.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Wave-wide reductions (64 lanes).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG (dropout masks).  Keyed by (seed, step); counter by
// (row, column-group).  The same (seed, step, row, col) always yields the same mask, so the
// backward pass and the eager oracle (rocfm/ops/reference.py) can regenerate it exactly.
// ---------------------------------------------------------------------------------------
struct Philox4 {
  uint32_t x, y, z, w;
};
__host__ __device__ __forceinline__ uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t* hi) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}
__host__ __device__ __forceinline__ Philox4 philox4x32_10(Philox4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0, hi1;
    uint32_t lo0 = mulhilo(0xD2511F53u, c.x, &hi0);
    uint32_t lo1 = mulhilo(0xCD9E8D57u, c.z, &hi1);
    Philox4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
// Dropout keep decisions for the 4 rows 4*rg .. 4*rg+3 of column `col` of hidden layer `layer`.
// u = (philox lane >> 8) / 2^24; keep iff u < keep.  rocfm/ops/reference.py replicates this.
__host__ __device__ __forceinline__ Philox4 dropout_bits(uint64_t seed, uint32_t layer, uint32_t step,
                                                         uint32_t rg, uint32_t col) {
  Philox4 c{rg, col, layer, step};
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}
__host__ __device__ __forceinline__ bool keep_from_bits(uint32_t v, float keep) {
  return (float)(v >> 8) * (1.0f / 16777216.0f) < keep;
}

}  // namespace rocfm
