// Device-side tf.train.Example parser (see decode.h) — the reference's tf.parse_example over a
// batch of serialized Examples (PS:117-126, HVD:109-118), for the fixed DeepFM schema
// {label: float[1], ids: int64[F], values: float[F]} with configurable feature names.
//
// One wave per workgroup takes up to 64 consecutive records of one batch:
//   1. the records' payload span (contiguous in the raw buffer) is staged into LDS with 16-byte
//      coalesced loads (≈19 KiB for 64 Criteo records);
//   2. every lane walks ITS record's protobuf wire format out of LDS.  A varint is decoded from one
//      8-byte window (three aligned ds_read_b32 + v_alignbyte): the terminating byte is the first
//      with bit 7 clear (ctz of ~w & 0x80…80) and the 7-bit groups are compacted with shifts, so
//      a field costs one LDS round trip instead of one per byte.  Lanes follow the same structure
//      (three map entries, 39 ids, 39 floats) and stay converged;
//   3. ids / values / label go to an LDS tile [64][F] that is then written to the batch ring with
//      coalesced stores.
// The walk mirrors the host decoder (csrc/io/tfrecord.cpp decode_example) case for case: packed
// and unpacked lists, unknown fields and features skipped, int64 labels accepted, the last
// occurrence of a feature wins, a list longer than F counted but not stored.  A record that fails
// sets the sticky error word (first failure wins) and is written as zeros, so a training step
// can never index out of the table with it; the host raises on the error word.
// Spans that do not fit the LDS stage (records > 512 B on average) are parsed from global memory
// by the same code.
#include "decode.h"

#include <algorithm>

namespace rocfm {
namespace {

constexpr int kDecRecs = 64;                 // records (lanes) per workgroup
constexpr int kStageBytes = kDecRecs * 512;  // LDS stage: 32 KiB
constexpr int kStageWords = kStageBytes / 4 + 8;

enum : int { kOk = 0, kBadProto = 1, kMissing = 2, kWrongLen = 3, kIdRange = 4, kBadOffsets = 5 };

extern __shared__ uint32_t dec_lds[];

// word source: the LDS stage (ds_read) or the batch row in global memory
template <bool L>
struct Src {
  const uint32_t* g;
  __device__ __forceinline__ uint32_t w(int i) const {
    if constexpr (L)
      return dec_lds[i];
    else
      return g[i];
  }
  __device__ __forceinline__ uint32_t byte(int p) const { return (w(p >> 2) >> ((p & 3) * 8)) & 0xffu; }
  __device__ __forceinline__ uint32_t ld32(int p) const {
    const int i = p >> 2;
    return __builtin_amdgcn_alignbyte(w(i + 1), w(i), (uint32_t)(p & 3));
  }
  __device__ __forceinline__ uint64_t win8(int p) const {
    const int i = p >> 2;
    const uint32_t a = w(i), b = w(i + 1), c = w(i + 2), s = (uint32_t)(p & 3);
    return ((uint64_t)__builtin_amdgcn_alignbyte(c, b, s) << 32) | __builtin_amdgcn_alignbyte(b, a, s);
  }
};

__device__ __forceinline__ uint64_t compact7(uint64_t x) {
  return (x & 0x7full) | ((x >> 1) & (0x7full << 7)) | ((x >> 2) & (0x7full << 14)) | ((x >> 3) & (0x7full << 21)) |
         ((x >> 4) & (0x7full << 28)) | ((x >> 5) & (0x7full << 35)) | ((x >> 6) & (0x7full << 42)) |
         ((x >> 7) & (0x7full << 49));
}

// protobuf varint at p (< end); advances p.  Same acceptance as the host read_varint: at most 10
// bytes, bits beyond 64 dropped, a 10th byte with its continuation bit set is malformed.
template <bool L>
__device__ __forceinline__ bool varint(const Src<L>& m, int& p, int end, uint64_t& v) {
  const int avail = end - p;
  if (avail <= 0) return false;
  {  // ≤ 4-byte varints (every tag and length, ids < 2^28): one 32-bit window, 32-bit arithmetic
    uint32_t x = m.ld32(p);
    uint32_t t = ~x & 0x80808080u;
    if (avail < 4) t &= (1u << (8 * avail)) - 1u;
    if (t) {
      const int nb = (__builtin_ctz(t) >> 3) + 1;
      if (nb < 4) x &= (1u << (8 * nb)) - 1u;
      v = (x & 0x7fu) | ((x >> 1) & (0x7fu << 7)) | ((x >> 2) & (0x7fu << 14)) | ((x >> 3) & (0x7fu << 21));
      p += nb;
      return true;
    }
  }
  uint64_t x = m.win8(p);
  uint64_t t = ~x & 0x8080808080808080ull;
  if (avail < 8) t &= (1ull << (8 * avail)) - 1;
  if (t) {
    const int nb = (__builtin_ctzll(t) >> 3) + 1;
    if (nb < 8) x &= (1ull << (8 * nb)) - 1;
    v = compact7(x);
    p += nb;
    return true;
  }
  if (avail < 9) return false;
  v = compact7(x);
  const uint32_t b8 = m.byte(p + 8);
  v |= (uint64_t)(b8 & 0x7f) << 56;
  if (!(b8 & 0x80)) {
    p += 9;
    return true;
  }
  if (avail < 10) return false;
  const uint32_t b9 = m.byte(p + 9);
  v |= (uint64_t)(b9 & 0x7f) << 63;
  if (b9 & 0x80) return false;
  p += 10;
  return true;
}

template <bool L>
__device__ __forceinline__ bool skip_field(const Src<L>& m, int& p, int end, uint32_t wire) {
  uint64_t v;
  switch (wire) {
    case 0:
      return varint(m, p, end, v);
    case 1:
      if (end - p < 8) return false;
      p += 8;
      return true;
    case 2:
      if (!varint(m, p, end, v) || (uint64_t)(end - p) < v) return false;
      p += (int)v;
      return true;
    case 5:
      if (end - p < 4) return false;
      p += 4;
      return true;
    default:
      return false;
  }
}

// FloatList body [p, end) → dst[0..cap); returns the value count or -1 (host parse_float_list)
template <bool L>
__device__ __forceinline__ int float_list(const Src<L>& m, int p, int end, float* dst, int cap) {
  int cnt = 0;
  while (p < end) {
    uint64_t tag;
    if (!varint(m, p, end, tag)) return -1;
    const uint32_t fno = (uint32_t)(tag >> 3), wire = (uint32_t)(tag & 7);
    if (fno == 1 && wire == 2) {
      uint64_t len;
      if (!varint(m, p, end, len) || (uint64_t)(end - p) < len || (len & 3)) return -1;
      const int k = (int)(len >> 2);
      if (cnt + k <= cap)
        for (int i = 0; i < k; ++i) dst[cnt + i] = __uint_as_float(m.ld32(p + 4 * i));
      cnt += k;
      p += (int)len;
    } else if (fno == 1 && wire == 5) {
      if (end - p < 4) return -1;
      if (cnt < cap) dst[cnt] = __uint_as_float(m.ld32(p));
      ++cnt;
      p += 4;
    } else if (!skip_field(m, p, end, wire)) {
      return -1;
    }
  }
  return cnt;
}

// Int64List body → int32 dst[0..cap); flags ids out of [0, max_id) (host parse_int64_list)
template <bool L>
__device__ __forceinline__ int int64_list(const Src<L>& m, int p, int end, int32_t* dst, int cap, long long max_id,
                                          bool* oob) {
  int cnt = 0;
  while (p < end) {
    uint64_t tag;
    if (!varint(m, p, end, tag)) return -1;
    const uint32_t fno = (uint32_t)(tag >> 3), wire = (uint32_t)(tag & 7);
    if (fno == 1 && wire == 2) {
      uint64_t len;
      if (!varint(m, p, end, len) || (uint64_t)(end - p) < len) return -1;
      const int e2 = p + (int)len;
      const uint64_t lim = (max_id > 0 && max_id < 0x80000000LL) ? (uint64_t)max_id : 0x80000000ull;
      bool bad = false;
      while (p < e2) {
        uint64_t v;
        if (!varint(m, p, e2, v)) return -1;
        bad |= v >= lim;
        if (cnt < cap) dst[cnt] = (int32_t)v;
        ++cnt;
      }
      if (bad) *oob = true;
    } else if (fno == 1 && wire == 0) {
      uint64_t v;
      if (!varint(m, p, end, v)) return -1;
      const long long sv = (long long)v;
      if (sv < 0 || (max_id > 0 && sv >= max_id) || sv > 0x7fffffffLL) *oob = true;
      if (cnt < cap) dst[cnt] = (int32_t)sv;
      ++cnt;
    } else if (!skip_field(m, p, end, wire)) {
      return -1;
    }
  }
  return cnt;
}

// feature name [kp, kp+kl) == key w?
template <bool L>
__device__ __forceinline__ bool key_is(const Src<L>& m, int kp, int kl, const DecodeParams& P, int w) {
  if (kl != P.klen[w]) return false;
  uint64_t a = 0, b = 0;
  const uint64_t ka = P.keyw[w][0], kb = P.keyw[w][1];
  if (kl > 0) a = m.win8(kp);
  if (kl > 8) b = m.win8(kp + 8);
  const uint64_t ma = kl >= 8 ? ~0ull : ((1ull << (8 * kl)) - 1);
  const int k2 = kl - 8;
  const uint64_t mb = k2 <= 0 ? 0ull : (k2 >= 8 ? ~0ull : ((1ull << (8 * k2)) - 1));
  return ((a ^ ka) & ma) == 0 && ((b ^ kb) & mb) == 0;
}

// One Example [p, end) → ids/vals (LDS rows of F), label; returns a ParseStatus.
template <bool L>
__device__ __forceinline__ int parse_example(const Src<L>& m, int p, const int end, const DecodeParams& P, int32_t* ids, float* vals,
                             float* label, int32_t* itmp) {
  const int F = P.F;
  int nl = -1, ni = -1, nv = -1;
  bool oob = false;
  while (p < end) {  // Example
    uint64_t tag;
    if (!varint(m, p, end, tag)) return kBadProto;
    if ((tag >> 3) != 1 || (tag & 7) != 2) {
      if (!skip_field(m, p, end, (uint32_t)(tag & 7))) return kBadProto;
      continue;
    }
    uint64_t flen;
    if (!varint(m, p, end, flen) || (uint64_t)(end - p) < flen) return kBadProto;
    const int fend = p + (int)flen;
    while (p < fend) {  // Features: map entries (field 1)
      uint64_t t2;
      if (!varint(m, p, fend, t2)) return kBadProto;
      if ((t2 >> 3) != 1 || (t2 & 7) != 2) {
        if (!skip_field(m, p, fend, (uint32_t)(t2 & 7))) return kBadProto;
        continue;
      }
      uint64_t elen;
      if (!varint(m, p, fend, elen) || (uint64_t)(fend - p) < elen) return kBadProto;
      const int eend = p + (int)elen;
      int kp = -1, kl = 0, vp = -1, vl = 0;
      while (p < eend) {  // {1: key, 2: Feature}
        uint64_t t3;
        if (!varint(m, p, eend, t3)) return kBadProto;
        const uint32_t fno = (uint32_t)(t3 >> 3), wire = (uint32_t)(t3 & 7);
        if ((fno == 1 || fno == 2) && wire == 2) {
          uint64_t l;
          if (!varint(m, p, eend, l) || (uint64_t)(eend - p) < l) return kBadProto;
          if (fno == 1) {
            kp = p;
            kl = (int)l;
          } else {
            vp = p;
            vl = (int)l;
          }
          p += (int)l;
        } else if (!skip_field(m, p, eend, wire)) {
          return kBadProto;
        }
      }
      p = eend;
      if (kp < 0 || vp < 0) continue;
      const int w = key_is(m, kp, kl, P, 0) ? 0 : key_is(m, kp, kl, P, 1) ? 1 : key_is(m, kp, kl, P, 2) ? 2 : -1;
      if (w < 0) continue;
      int q = vp;
      const int qend = vp + vl;
      while (q < qend) {  // Feature {1: bytes_list, 2: float_list, 3: int64_list}
        uint64_t t4;
        if (!varint(m, q, qend, t4)) return kBadProto;
        const uint32_t fno = (uint32_t)(t4 >> 3), wire = (uint32_t)(t4 & 7);
        if (wire != 2) {
          if (!skip_field(m, q, qend, wire)) return kBadProto;
          continue;
        }
        uint64_t l;
        if (!varint(m, q, qend, l) || (uint64_t)(qend - q) < l) return kBadProto;
        const int le = q + (int)l;
        if (w == 0 && fno == 2) {
          const int c = float_list(m, q, le, label, 1);
          if (c < 0) return kBadProto;
          nl = c;
        } else if (w == 2 && fno == 2) {
          nv = float_list(m, q, le, vals, F);
          if (nv < 0) return kBadProto;
        } else if (w == 1 && fno == 3) {
          ni = int64_list(m, q, le, ids, F, P.max_id, &oob);
          if (ni < 0) return kBadProto;
        } else if (w == 0 && fno == 3) {  // tolerate int64 labels
          bool o2 = false;
          const int c = int64_list(m, q, le, itmp, 1, 0, &o2);
          if (c < 0) return kBadProto;
          if (c >= 1) *label = (float)itmp[0];
          nl = c;
        }
        q = le;
      }
    }
    p = fend;
  }
  if (nl < 0 || ni < 0 || nv < 0) return kMissing;
  if (nl != 1 || ni != F || nv != F) return kWrongLen;
  if (oob) return kIdRange;
  return kOk;
}

__global__ __launch_bounds__(kDecRecs) void decode_examples_kernel(DecodeParams P) {
  const int nblk = cdiv(P.B, kDecRecs);
  const int b = blockIdx.x / nblk, r0 = (blockIdx.x % nblk) * kDecRecs;
  const int nr = min(kDecRecs, P.B - r0), lane = threadIdx.x, F = P.F;
  const int32_t* offs = P.offs + (size_t)b * (P.B + 1);
  const uint8_t* row = P.bytes + (size_t)b * P.cap;
  // LDS: stage words | ids [64][F] | vals [64][F] | labels [64] | int scratch [64]
  int32_t* s_ids = reinterpret_cast<int32_t*>(dec_lds + kStageWords);
  float* s_vals = reinterpret_cast<float*>(s_ids + kDecRecs * F);
  float* s_lab = s_vals + kDecRecs * F;
  int32_t* s_tmp = reinterpret_cast<int32_t*>(s_lab + kDecRecs);
  const int s0 = offs[r0], s1 = offs[r0 + nr];
  const bool span_ok = 0 <= s0 && s0 <= s1 && (long long)s1 <= P.cap;
  const int a0 = s0 & ~15;
  const bool staged = span_ok && (s1 - a0) + 32 <= kStageBytes;
  if (staged) {
    const int nvec = (s1 - a0 + 15) >> 4;
    const uint4* g4 = reinterpret_cast<const uint4*>(row + a0);
    uint4* l4 = reinterpret_cast<uint4*>(dec_lds);
    for (int i = lane; i < nvec + 2; i += kDecRecs) l4[i] = i < nvec ? g4[i] : make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  int st = kOk;
  float lab = 0.f;
  if (lane < nr) {
    const int rs = offs[r0 + lane], re = offs[r0 + lane + 1];
    s_lab[lane] = 0.f;
    if (!span_ok || rs < s0 || re < rs || re > s1) {
      st = kBadOffsets;
    } else if (staged) {
      Src<true> m{nullptr};
      st = parse_example(m, rs - a0, re - a0, P, s_ids + lane * F, s_vals + lane * F, s_lab + lane, s_tmp + lane);
    } else {
      Src<false> m{reinterpret_cast<const uint32_t*>(row)};
      st = parse_example(m, rs, re, P, s_ids + lane * F, s_vals + lane * F, s_lab + lane, s_tmp + lane);
    }
    if (st != kOk) {
      for (int f = 0; f < F; ++f) {
        s_ids[lane * F + f] = 0;
        s_vals[lane * F + f] = 0.f;
      }
      s_lab[lane] = 0.f;
      if (atomicCAS(&P.err[0], 0, st) == 0) {
        P.err[1] = P.batch0 + b;
        P.err[2] = r0 + lane;
      }
    }
    lab = s_lab[lane];
  }
  __syncthreads();
  const int slot = (P.slot0 + b) % P.R;
  int32_t* gi = P.ids + ((size_t)slot * P.B + r0) * F;
  float* gv = P.vals + ((size_t)slot * P.B + r0) * F;
  for (int i = lane; i < nr * F; i += kDecRecs) {
    gi[i] = s_ids[i];
    gv[i] = s_vals[i];
  }
  if (lane < nr) P.labels[(size_t)slot * P.B + r0 + lane] = lab;
}

}  // namespace

size_t decode_lds_bytes(int F) { return (size_t)kStageWords * 4 + (size_t)kDecRecs * F * 8 + kDecRecs * 8; }

bool decode_fits(int F) {
  static int max_lds = -1;
  if (max_lds < 0) {
    int dev = 0, v = 0;
    ROCFM_HIP_CHECK(hipGetDevice(&dev));
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess || v <= 0)
      ROCFM_HIP_CHECK(hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
    max_lds = v;
  }
  return F >= 1 && F <= 192 && decode_lds_bytes(F) <= (size_t)max_lds;
}

void launch_decode_examples(const DecodeParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.B > 0 && p.F > 0 && p.F <= 192 && p.nb >= 0 && p.R > 0 && p.cap % 16 == 0,
                "decode_examples: bad shape");
  ROCFM_REQUIRE(p.bytes && p.offs && p.ids && p.vals && p.labels && p.err, "decode_examples: null pointer");
  for (int w = 0; w < 3; ++w) ROCFM_REQUIRE(p.klen[w] >= 0 && p.klen[w] <= kDecodeKeyMax, "decode: key too long");
  if (p.nb == 0) return;
  const size_t lds = decode_lds_bytes(p.F);
  const int blocks = p.nb * cdiv(p.B, kDecRecs);
  // the device's opt-in LDS limit (160 KiB per workgroup on gfx950): a wider schema is refused here,
  // before any launch, and the Estimator parses on the host instead (decode_fits)
  ROCFM_REQUIRE(decode_fits(p.F), "decode_examples: field_size " + std::to_string(p.F) + " needs " +
                                      std::to_string(lds) + " B of LDS, more than this device allows");
  if (lds > 65536) {  // beyond the default dynamic-LDS limit (160 KiB per CU on gfx950)
    ROCFM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(decode_examples_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  }
  hipLaunchKernelGGL(decode_examples_kernel, dim3(blocks), dim3(kDecRecs), lds, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
