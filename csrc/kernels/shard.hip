// Row-shard routing kernels: the Parameter-Server placement of the reference (PS:521-531 — the
// embedding variables live on the PS tasks, every worker pulls the rows its batch needs and pushes
// their gradients back) re-designed as an owner-sharded table exchanged with RCCL all-to-all.
//
// Per step and rank (rocfm/parallel/emb_shard.py):
//   shard_keys   ids → owner-major keys, so the batch's radix sort groups lookups by owner
//   shard_route  sorted keys → unique ids per owner (send buffer), the received-row index of every
//                lookup (the fused row kernel then gathers from the received rows as its table),
//                and the same indices in sorted order (input of the local gradient reduction)
//   shard_serve  owner: requested ids → table rows (forward) and local row keys (update)
#include "shard.h"
#include "shard_body.h"

#include <algorithm>

namespace rocfm {
namespace {

constexpr int kRT = 256;                 // route threads per workgroup
constexpr int kRI = 4;                   // sorted entries per thread
constexpr int kRTile = kRT * kRI;        // entries per workgroup
constexpr int kRWaves = kRT / kWave;
constexpr int kMaxOwners = 1024;
constexpr uint32_t kPad = 0xFFFFFFFFu;

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  return v;
}

// Exclusive scan over the kRT threads of the workgroup; `total` receives the sum.
__device__ __forceinline__ int block_excl_scan(int v, int* s_w, int& total) {
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int inc = wave_incl_scan(v);
  if (lane == 63) s_w[wave] = inc;
  __syncthreads();
  int before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kRWaves; ++w) {
    const int x = s_w[w];
    before += w < wave ? x : 0;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return before + inc - v;
}

__global__ __launch_bounds__(256) void shard_keys_kernel(ShardKeysParams p) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= p.n) return;
  p.keys[i] = shard_key((uint32_t)p.ids[i], (uint32_t)p.W, p.Vs, p.hot_ids, p.n_hot);
}

// Multi-workgroup routing of the sorted (key', lookup) pairs (tile = 1024 entries per workgroup).
//   count  : per tile, the run heads (unique ids) it contains; per owner, its unique ids (atomics,
//            one per owner change per thread)
//   assign : every tile derives its first unique rank (Σ earlier tiles) and every owner's first
//            unique rank (scan of the owner counts), then j = rank − first[owner] per entry;
//            heads publish their global id to the owner's request list; pads the lists.
__device__ __forceinline__ void load_tile(const ShardRouteParams& p, int i0, uint32_t (&k)[kRI], uint32_t& prev) {
#pragma unroll
  for (int u = 0; u < kRI; ++u) k[u] = (i0 + u < p.n) ? p.skeys[i0 + u] - p.key_base : kPad;
  prev = (i0 > 0 && i0 <= p.n) ? p.skeys[i0 - 1] - p.key_base : kPad;
}

// Owner counts are reduced per workgroup in LDS first (one global atomic per owner present in the
// tile): with every thread adding straight to p.counts[owner], the few owners of a small world
// took ~10k same-address global atomics per step (34 µs at world 1; MI355X guide §atomics).
__global__ __launch_bounds__(kRT) void shard_route_count_kernel(ShardRouteParams p) {
  __shared__ int s_w[kRWaves];
  __shared__ int s_cnt[kMaxOwners];
  const int t = threadIdx.x;
  for (int o = t; o < p.W; o += kRT) s_cnt[o] = 0;
  __syncthreads();
  const int i0 = blockIdx.x * kRTile + t * kRI;
  uint32_t k[kRI], prev;
  load_tile(p, i0, k, prev);
  int heads = 0, cur_o = -1, cur_c = 0;
#pragma unroll
  for (int u = 0; u < kRI; ++u) {
    if (i0 + u < p.n && k[u] != prev) {
      ++heads;
      const int o = min((int)(k[u] / p.Vs), p.W);  // W: replicated rows (not counted)
      if (o != cur_o) {
        if (cur_c && cur_o < p.W) atomicAdd(&s_cnt[cur_o], cur_c);
        cur_o = o;
        cur_c = 0;
      }
      ++cur_c;
    }
    if (i0 + u < p.n) prev = k[u];
  }
  if (cur_c && cur_o < p.W) atomicAdd(&s_cnt[cur_o], cur_c);
  int total;
  block_excl_scan(heads, s_w, total);  // (its barriers also order the LDS count adds)
  if (t == 0) p.scratch[blockIdx.x] = total;
  for (int o = t; o < p.W; o += kRT)
    if (s_cnt[o]) atomicAdd(&p.counts[o], s_cnt[o]);
}

__global__ __launch_bounds__(kRT) void shard_route_assign_kernel(ShardRouteParams p) {
  __shared__ int s_w[kRWaves];
  __shared__ int s_first[kMaxOwners];
  __shared__ int s_cnt[kMaxOwners];
  const int t = threadIdx.x, W = p.W;
  // first unique rank of this tile: Σ heads of the tiles before it
  int acc = 0;
  for (int g = t; g < (int)blockIdx.x; g += kRT) acc += p.scratch[g];
  int tile_base;
  block_excl_scan(acc, s_w, tile_base);
  // first unique rank of every owner: exclusive scan of the owner counts
  int carry = 0;
  for (int o0 = 0; o0 < W; o0 += kRT) {
    const int o = o0 + t;
    const int c = o < W ? p.counts[o] : 0;
    int tot;
    const int f = block_excl_scan(c, s_w, tot);
    if (o < W) {
      s_first[o] = carry + f;
      s_cnt[o] = c;
      if (blockIdx.x == 0 && c > p.cap) *p.overflow = 1;
    }
    carry += tot;
  }
  const int i0 = blockIdx.x * kRTile + t * kRI;
  uint32_t k[kRI], v[kRI], prev;
  load_tile(p, i0, k, prev);
#pragma unroll
  for (int u = 0; u < kRI; ++u) v[u] = (i0 + u < p.n) ? p.svals[i0 + u] - p.val_base : 0u;
  int heads = 0;
  {
    uint32_t pv = prev;
#pragma unroll
    for (int u = 0; u < kRI; ++u) {
      if (i0 + u < p.n && k[u] != pv) ++heads;
      if (i0 + u < p.n) pv = k[u];
    }
  }
  int tot;
  const int before = block_excl_scan(heads, s_w, tot);  // also orders s_first/s_cnt writes
  int urun = tile_base + before - 1;
#pragma unroll
  for (int u = 0; u < kRI; ++u) {
    if (i0 + u >= p.n) continue;
    const bool head = k[u] != prev;
    prev = k[u];
    urun += head ? 1 : 0;
    const int o = (int)(k[u] / p.Vs);
    if (o >= W) {  // replicated row: the local replica behind the W owner segments
      const uint32_t lk = (uint32_t)W * (uint32_t)p.cap + (k[u] - (uint32_t)W * p.Vs);
      p.skeys_local[i0 + u] = lk;
      p.local_idx[v[u]] = (int32_t)lk;
      continue;
    }
    const int j = urun - s_first[o];
    const uint32_t lk = (uint32_t)o * (uint32_t)p.cap + (uint32_t)min(j, p.cap - 1);
    p.skeys_local[i0 + u] = lk;
    p.local_idx[v[u]] = (int32_t)lk;
    if (head && j < p.cap) p.send_ids[(size_t)o * p.cap + j] = (k[u] - (uint32_t)o * p.Vs) * (uint32_t)W + o;
  }
  // pad every owner's request list past its count (grid-strided over all slots)
  const int tot_slots = W * p.cap;
  for (int s = blockIdx.x * kRT + t; s < tot_slots; s += gridDim.x * kRT) {
    const int o = s / p.cap, j = s - o * p.cap;
    if (j >= s_cnt[o]) p.send_ids[s] = kPad;
  }
}

__global__ __launch_bounds__(256) void shard_serve_kernel(ShardServeParams p) {
  shard_serve_body(p, (long long)blockIdx.x * 256 + threadIdx.x);
}

}  // namespace

void launch_shard_keys(const ShardKeysParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.W >= 1 && (unsigned long long)(p.W + (p.n_hot > 0)) * p.Vs < 0xFFFFFFFFull,
                "shard_keys: (W + hot) * Vs must fit in 32 bits");
  ROCFM_REQUIRE(p.n_hot == 0 || (p.hot_ids != nullptr && (uint32_t)p.n_hot <= p.Vs), "shard_keys: hot ids");
  if (p.n <= 0) return;
  hipLaunchKernelGGL(shard_keys_kernel, dim3(cdiv(p.n, 256)), dim3(256), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

void launch_shard_route(const ShardRouteParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.W >= 1 && p.W < kMaxOwners, "shard_route: 1 <= world < 1024");
  ROCFM_REQUIRE(p.cap >= 1, "shard_route: capacity must be positive");
  ROCFM_REQUIRE((unsigned long long)p.W * p.cap < (1ull << 31), "shard_route: W*cap overflows int32");
  ROCFM_REQUIRE(p.scratch != nullptr, "shard_route: scratch (>= route_scratch_ints(n)) required");
  ROCFM_HIP_CHECK(hipMemsetAsync(p.counts, 0, sizeof(int32_t) * p.W, stream));
  const int tiles = std::max(1, cdiv(p.n, kRTile));
  if (p.n > 0) hipLaunchKernelGGL(shard_route_count_kernel, dim3(tiles), dim3(kRT), 0, stream, p);
  hipLaunchKernelGGL(shard_route_assign_kernel, dim3(tiles), dim3(kRT), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

int route_scratch_ints(int n) { return std::max(1, cdiv(n, kRTile)); }

void launch_shard_serve(const ShardServeParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.Kp % 4 == 0 && p.Kp > 0, "shard_serve: Kp must be a positive multiple of 4");
  if (p.m <= 0) return;
  const long long n = (long long)p.m * (p.Kp / 4);
  hipLaunchKernelGGL(shard_serve_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
