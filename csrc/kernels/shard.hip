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

namespace rocfm {
namespace {

constexpr int kRouteThreads = 1024;
constexpr int kRouteWaves = kRouteThreads / kWave;
constexpr int kMaxOwners = 1024;
constexpr uint32_t kPad = 0xFFFFFFFFu;
constexpr int kUnroll = 8;

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  return v;
}

// Exclusive scan over the 1024 threads of the workgroup; `total` receives the sum.
__device__ __forceinline__ int block_excl_scan(int v, int* s_w, int& total) {
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int inc = wave_incl_scan(v);
  if (lane == 63) s_w[wave] = inc;
  __syncthreads();
  if (t < 64) {
    const int x = t < kRouteWaves ? s_w[t] : 0;
    const int xi = wave_incl_scan(x);
    if (t < kRouteWaves) s_w[kRouteWaves + t] = xi - x;
    if (t == kRouteWaves - 1) s_w[2 * kRouteWaves] = xi;
  }
  __syncthreads();
  total = s_w[2 * kRouteWaves];
  const int r = s_w[kRouteWaves + wave] + inc - v;
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void shard_keys_kernel(ShardKeysParams p) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= p.n) return;
  const uint32_t id = (uint32_t)p.ids[i];
  p.keys[i] = (id % (uint32_t)p.W) * p.Vs + id / (uint32_t)p.W;
}

// One workgroup: each thread owns a contiguous chunk of the sorted keys.  Pass 1 counts run heads
// (unique ids) and, per owner, the unique ids it holds; two block scans give every chunk its first
// unique rank and every owner its first unique rank; pass 2 assigns j = rank − first[owner].
__global__ __launch_bounds__(kRouteThreads) void shard_route_kernel(ShardRouteParams p) {
  __shared__ int s_cnt[kMaxOwners];
  __shared__ int s_first[kMaxOwners];
  __shared__ int s_w[2 * kRouteWaves + 1];
  const int t = threadIdx.x;
  const int W = p.W;
  for (int o = t; o < W; o += kRouteThreads) s_cnt[o] = 0;
  __syncthreads();
  const int per = (p.n + kRouteThreads - 1) / kRouteThreads;
  const int b = min(t * per, p.n), e = min(b + per, p.n);

  // pass 1: heads in this chunk + per-owner unique counts (one LDS atomic per owner change)
  int heads = 0;
  {
    uint32_t prev = b > 0 ? p.skeys[b - 1] : kPad;
    int cur_o = -1, cur_c = 0;
    for (int i0 = b; i0 < e; i0 += kUnroll) {
      uint32_t k[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) k[u] = (i0 + u < e) ? p.skeys[i0 + u] : kPad;
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        if (i0 + u < e && k[u] != prev) {
          ++heads;
          const int o = (int)(k[u] / p.Vs);
          if (o != cur_o) {
            if (cur_c) atomicAdd(&s_cnt[cur_o], cur_c);
            cur_o = o;
            cur_c = 0;
          }
          ++cur_c;
        }
        prev = (i0 + u < e) ? k[u] : prev;
      }
    }
    if (cur_c) atomicAdd(&s_cnt[cur_o], cur_c);
  }
  int total;
  const int base = block_excl_scan(heads, s_w, total);
  for (int o0 = 0; o0 < W; o0 += kRouteThreads) {  // W <= kMaxOwners == kRouteThreads: one round
    const int o = o0 + t;
    const int c = o < W ? s_cnt[o] : 0;
    int tot2;
    const int f = block_excl_scan(c, s_w, tot2);
    if (o < W) {
      s_first[o] = f;
      p.counts[o] = c;
      if (c > p.cap) *p.overflow = 1;
    }
  }
  __syncthreads();

  // pass 2: row index of every lookup; run heads publish their id to the owner's request list
  {
    int urun = base - 1;
    uint32_t prev = b > 0 ? p.skeys[b - 1] : kPad;
    for (int i0 = b; i0 < e; i0 += kUnroll) {
      uint32_t k[kUnroll], v[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const bool in = i0 + u < e;
        k[u] = in ? p.skeys[i0 + u] : kPad;
        v[u] = in ? p.svals[i0 + u] : 0u;
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        if (i0 + u >= e) continue;
        const bool head = k[u] != prev;
        prev = k[u];
        urun += head ? 1 : 0;
        const int o = (int)(k[u] / p.Vs);
        const int j = urun - s_first[o];
        const uint32_t lk = (uint32_t)o * (uint32_t)p.cap + (uint32_t)min(j, p.cap - 1);
        p.skeys_local[i0 + u] = lk;
        p.local_idx[v[u]] = (int32_t)lk;
        if (head && j < p.cap) p.send_ids[(size_t)o * p.cap + j] = (k[u] - (uint32_t)o * p.Vs) * (uint32_t)W + o;
      }
    }
  }
  // pass 3: pad every owner's request list past its count
  const int tot_slots = W * p.cap;
  for (int s = t; s < tot_slots; s += kRouteThreads) {
    const int o = s / p.cap, j = s - o * p.cap;
    if (j >= s_cnt[o]) p.send_ids[s] = kPad;
  }
}

__global__ __launch_bounds__(256) void shard_serve_kernel(ShardServeParams p) {
  const int KP4 = p.Kp >> 2;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)p.m * KP4) return;
  const int r = (int)(i / KP4), c = (int)(i - (long long)r * KP4);
  const uint32_t id = p.ids[r];
  const bool pad = id == kPad;
  const uint32_t lr = id / (uint32_t)p.W;
  const bool ok = !pad && (int)(id % (uint32_t)p.W) == p.rank && lr < p.Vs;
  if (!pad && !ok && p.bad) *p.bad = 1;
  if (p.rows_out) {
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    reinterpret_cast<float4*>(p.rows_out)[(size_t)r * KP4 + c] =
        ok ? reinterpret_cast<const float4*>(p.table)[(size_t)lr * KP4 + c] : z;
  }
  if (c == 0 && p.lkeys) p.lkeys[r] = ok ? lr : p.Vs;
}

}  // namespace

void launch_shard_keys(const ShardKeysParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.W >= 1 && (unsigned long long)p.W * p.Vs < 0xFFFFFFFFull, "shard_keys: W*Vs must fit in 32 bits");
  if (p.n <= 0) return;
  hipLaunchKernelGGL(shard_keys_kernel, dim3(cdiv(p.n, 256)), dim3(256), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

void launch_shard_route(const ShardRouteParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.W >= 1 && p.W <= kMaxOwners, "shard_route: 1 <= world <= 1024");
  ROCFM_REQUIRE(p.cap >= 1, "shard_route: capacity must be positive");
  ROCFM_REQUIRE((unsigned long long)p.W * p.cap < (1ull << 31), "shard_route: W*cap overflows int32");
  hipLaunchKernelGGL(shard_route_kernel, dim3(1), dim3(kRouteThreads), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

void launch_shard_serve(const ShardServeParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.Kp % 4 == 0 && p.Kp > 0, "shard_serve: Kp must be a positive multiple of 4");
  if (p.m <= 0) return;
  const long long n = (long long)p.m * (p.Kp / 4);
  hipLaunchKernelGGL(shard_serve_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
