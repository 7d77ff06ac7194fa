// Stable LSD radix sort of (key, index) pairs over equal-length segments — the sort of the
// embedding-gradient aggregation (the reference's tf.unique_with_counts / segment sums behind
// the sparse embedding update, …vectorized-map.py:296 / multiInstance.py:307), written for the
// engine's shapes instead of a general library sort.
//
// The multi-step side chain sorts S batches of n = B·F lookups at once (fused.py _prepare_multi).
// rocPRIM sorts the S·n composite keys (step << id_bits | id) on its merge-sort path below 1M
// items (≈160 µs per 16 steps) and on its onesweep path above (3 passes + 9 memsets, ≈140 µs per
// 32 steps; profiles/r4_radix_ab.md).  Here every batch is its own segment and only the id bits are
// sorted — the same permutation as the composite sort, with no inter-workgroup hand-off:
//
//   per 8-bit digit pass:  hist    one workgroup per 1,024-key tile: digit counts in LDS →
//                                  cnt[segment][tile][256]
//                          scatter one workgroup per tile: the tile's first slot per digit from
//                                  the segment's counts (column sums + an LDS scan over the
//                                  digits; a separate scan launch was measured 7.8 µs of serial
//                                  latency per pass), then the stable rank of every key among the
//                                  tile's equal digits (64-lane match by 8 ballots + per-wave
//                                  counts in LDS, 4 rounds in index order) → out[first + rank]
//
// Everything is plain loads / stores and LDS; the counts are exact and the ranks follow the input
// order, so the result is deterministic and equals a stable sort (tests/test_sort_gpu.py checks it
// against torch.sort(stable=True) and against the rocPRIM path).
#include "../ops.h"

namespace rocfm {
namespace {

constexpr int kSortThreads = 256;
constexpr int kSortItems = 4;
constexpr int kTile = kSortThreads * kSortItems;
constexpr int kRadixBits = 8;
constexpr int kRadix = 1 << kRadixBits;
constexpr int kSortWaves = kSortThreads / 64;
static_assert(kRadix == kSortThreads, "one digit per thread in the count / scan steps");

struct Layout {
  size_t keys[2], vals[2], cnt, total;
};

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

Layout layout(int nseg, int seg_len) {
  const size_t N = (size_t)nseg * seg_len;
  const size_t T = (size_t)cdiv(seg_len, kTile);
  const size_t nc = (size_t)nseg * T * kRadix;
  Layout L{};
  size_t o = 0;
  for (int b = 0; b < 2; ++b) {
    L.keys[b] = o;
    o = align256(o + N * 4);
    L.vals[b] = o;
    o = align256(o + N * 4);
  }
  L.cnt = o;
  o = align256(o + nc * 4);
  L.total = o;
  return L;
}

__global__ __launch_bounds__(kSortThreads) void seg_hist_kernel(const uint32_t* __restrict__ keys, int seg_len, int T,
                                                                int shift, uint32_t dmask, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t h[kRadix];
  const int t = threadIdx.x, seg = blockIdx.x / T, tile = blockIdx.x - seg * T;
  h[t] = 0;
  __syncthreads();
  const uint32_t* k = keys + (size_t)seg * seg_len;
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    const int idx = tile * kTile + i * kSortThreads + t;
    if (idx < seg_len) atomicAdd(&h[(k[idx] >> shift) & dmask], 1u);  // LDS counts: order-free
  }
  __syncthreads();
  cnt[((size_t)seg * T + tile) * kRadix + t] = h[t];
}

// vals_in == nullptr: the values are first_val + the key's global index (the first pass)
__global__ __launch_bounds__(kSortThreads) void seg_scatter_kernel(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, uint32_t* __restrict__ keys_out,
    uint32_t* __restrict__ vals_out, const uint32_t* __restrict__ cnt, int seg_len, int T, int shift, uint32_t dmask,
    int nbits, uint32_t first_val) {
  __shared__ uint32_t s_off[kRadix];
  __shared__ uint32_t s_wc[kSortWaves][kRadix];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int seg = blockIdx.x / T, tile = blockIdx.x - seg * T;
  const size_t sbase = (size_t)seg * seg_len;
  uint32_t key[kSortItems], val[kSortItems];
  bool ok[kSortItems];
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {  // every load of the tile before the first use
    const int idx = tile * kTile + i * kSortThreads + t;
    ok[i] = idx < seg_len;
    key[i] = ok[i] ? keys_in[sbase + idx] : 0u;
    val[i] = vals_in == nullptr ? first_val + (uint32_t)(sbase + idx) : (ok[i] ? vals_in[sbase + idx] : 0u);
  }
  // this tile's first slot for digit t: the digits below t over the whole segment + digit t in the
  // tiles before this one (thread t walks the segment's counts column t; coalesced rows of 256)
  {
    const uint32_t* c = cnt + (size_t)seg * T * kRadix + t;
    uint32_t tot = 0, before = 0;
#pragma unroll 8
    for (int j = 0; j < T; ++j) {
      const uint32_t v = c[(size_t)j * kRadix];
      tot += v;
      before += j < tile ? v : 0u;
    }
    s_wc[0][t] = tot;
    __syncthreads();
    for (int o = 1; o < kRadix; o <<= 1) {  // inclusive scan of the digit totals
      const uint32_t v = t >= o ? s_wc[0][t - o] : 0u;
      __syncthreads();
      s_wc[0][t] += v;
      __syncthreads();
    }
    s_off[t] = s_wc[0][t] - tot + before;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < kSortWaves; ++w) s_wc[w][t] = 0;
    __syncthreads();
  }
  const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {  // rounds in index order: item i·256 + t
    const uint32_t d = (key[i] >> shift) & dmask;
    unsigned long long m = __ballot(ok[i]);
    for (int b = 0; b < nbits; ++b) {  // lanes of this wave with the same digit
      const bool bit = (d >> b) & 1u;
      const unsigned long long bb = __ballot(ok[i] && bit);
      m &= bit ? bb : ~bb;
    }
    const int r = __popcll(m & lt);
    if (ok[i] && r == 0) s_wc[wave][d] = (uint32_t)__popcll(m);
    __syncthreads();
    if (ok[i]) {
      uint32_t pos = s_off[d] + (uint32_t)r;
      for (int w = 0; w < wave; ++w) pos += s_wc[w][d];
      if (pos < (uint32_t)seg_len) {
        keys_out[sbase + pos] = key[i];
        vals_out[sbase + pos] = val[i];
      }
    }
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (int w = 0; w < kSortWaves; ++w) {
      add += s_wc[w][t];
      s_wc[w][t] = 0;
    }
    s_off[t] += add;
    __syncthreads();
  }
}

}  // namespace

size_t seg_sort_temp_bytes(int nseg, int seg_len, int bits) {
  ROCFM_REQUIRE(nseg >= 1 && seg_len >= 0 && bits >= 0 && bits <= 32, "seg_sort: bad shape");
  (void)bits;
  return layout(nseg, seg_len).total;
}

void seg_sort_iota(void* temp, size_t temp_bytes, const uint32_t* keys_in, uint32_t* keys_out, uint32_t* vals_out,
                   int nseg, int seg_len, int bits, hipStream_t stream, uint32_t first_val) {
  ROCFM_REQUIRE(nseg >= 1 && seg_len >= 0 && bits >= 0 && bits <= 32, "seg_sort: bad shape");
  ROCFM_REQUIRE((long long)nseg * seg_len < (1LL << 31), "seg_sort: more than 2^31 keys");
  if (seg_len == 0) return;
  const Layout L = layout(nseg, seg_len);
  ROCFM_REQUIRE(temp != nullptr && temp_bytes >= L.total, "seg_sort: temporary storage too small");
  ROCFM_REQUIRE(keys_in && keys_out && vals_out, "seg_sort: null pointer");
  ROCFM_REQUIRE(keys_in != keys_out, "seg_sort: keys_out must not alias keys_in (the last pass scatters into it)");
  uint8_t* tb = static_cast<uint8_t*>(temp);
  uint32_t* K[2] = {reinterpret_cast<uint32_t*>(tb + L.keys[0]), reinterpret_cast<uint32_t*>(tb + L.keys[1])};
  uint32_t* V[2] = {reinterpret_cast<uint32_t*>(tb + L.vals[0]), reinterpret_cast<uint32_t*>(tb + L.vals[1])};
  uint32_t* cnt = reinterpret_cast<uint32_t*>(tb + L.cnt);
  const int T = cdiv(seg_len, kTile);
  const int np = bits > 0 ? cdiv(bits, kRadixBits) : 1;
  const dim3 tiles(nseg * T), block(kSortThreads);
  for (int p = 0; p < np; ++p) {
    const int shift = p * kRadixBits;
    const int nb = bits > 0 ? min(kRadixBits, bits - shift) : 0;
    const uint32_t dmask = nb > 0 ? ((1u << nb) - 1u) : 0u;
    const uint32_t* kin = p == 0 ? keys_in : K[(p - 1) & 1];
    const uint32_t* vin = p == 0 ? nullptr : V[(p - 1) & 1];
    uint32_t* kout = p == np - 1 ? keys_out : K[p & 1];
    uint32_t* vout = p == np - 1 ? vals_out : V[p & 1];
    hipLaunchKernelGGL(seg_hist_kernel, tiles, block, 0, stream, kin, seg_len, T, shift, dmask, cnt);
    hipLaunchKernelGGL(seg_scatter_kernel, tiles, block, 0, stream, kin, vin, kout, vout, cnt, seg_len, T, shift,
                       dmask, nb, first_val);
  }
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
