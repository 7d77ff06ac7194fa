// Batch fetch for graph-replayed steps: copy batch (cursor + advance) of a device-resident pool
// ([NB][B][F] ids/values, [NB][B] labels — an HBM-resident dataset or the loader's staging ring)
// into a static input slot, and publish the next step's cursor / global_step.
//
// The engine double-buffers everything a step reads (input slot, sorted keys, cursor, step) by
// step parity, so this kernel runs on a side stream one step AHEAD of the compute (it fetches and
// the sort orders batch i+1 while step i trains) and never writes a word the concurrent step
// reads: it reads cursor[p]/step[p] and writes cursor[1-p]/step[1-p].
#include "batch.h"
#include "shard.h"

namespace rocfm {

// ROCFM_CHECK_IDS guard: an id outside [0, max_id) is flagged (sticky, vector atomic) and replaced
// by row 0 before any kernel can index the table with it
__device__ __forceinline__ int32_t guard_id(int32_t id, int32_t* bad, uint32_t max_id) {
  if (bad != nullptr && (uint32_t)id >= max_id) {
    atomicOr(bad, 1);
    return 0;
  }
  return id;
}

__global__ __launch_bounds__(256) void fetch_batch_kernel(const FetchParams p) {
  const long long nb = p.pool_batches;
  long long b = (*p.cur_src + p.advance) % nb;
  if (b < 0) b += nb;
  const long long n = (long long)p.B * p.F;
  const int4* si = reinterpret_cast<const int4*>(p.ids_pool + b * n);
  const int4* sv = reinterpret_cast<const int4*>(p.vals_pool + b * n);
  int4* di = reinterpret_cast<int4*>(p.ids);
  int4* dv = reinterpret_cast<int4*>(p.vals);
  const long long n4 = (n & 3) ? 0 : (n >> 2);  // vector path only when every batch is 16-B aligned
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    int4 v = si[i];
    if (p.bad_ids != nullptr) {
      v.x = guard_id(v.x, p.bad_ids, p.max_id);
      v.y = guard_id(v.y, p.bad_ids, p.max_id);
      v.z = guard_id(v.z, p.bad_ids, p.max_id);
      v.w = guard_id(v.w, p.bad_ids, p.max_id);
    }
    di[i] = v;
    dv[i] = sv[i];
  }
  for (long long i = (n4 << 2) + blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    p.ids[i] = guard_id(p.ids_pool[b * n + i], p.bad_ids, p.max_id);
    p.vals[i] = p.vals_pool[b * n + i];
  }
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < p.B; i += (long long)gridDim.x * 256)
    p.labels[i] = p.labels_pool[b * p.B + i];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (p.cur_dst) *p.cur_dst = *p.cur_src + p.advance;
    const int64_t st = *p.step_src + p.step_advance;
    if (p.step_dst) *p.step_dst = st;
    if (p.lrt_dst) *p.lrt_dst = p.opt_type == kAdam ? adam_lr_t(p.lr, p.beta1, p.beta2, st) : p.lr;
  }
}

void launch_fetch_batch(const FetchParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.pool_batches > 0, "fetch_batch: empty pool");
  ROCFM_REQUIRE(p.cur_dst != p.cur_src && (p.step_dst == nullptr || p.step_dst != p.step_src),
                "fetch_batch: source and destination counters must differ");
  const long long n4 = (long long)p.B * p.F / 4;
  const int grid = (int)std::max<long long>(1, std::min<long long>((n4 + 255) / 256, 256));
  hipLaunchKernelGGL(fetch_batch_kernel, dim3(grid), dim3(256), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

// grid: (blocks per batch, S)
__global__ __launch_bounds__(256) void fetch_multi_kernel(const FetchMultiParams p) {
  const int k = blockIdx.y;
  const long long nb = p.pool_batches;
  const long long start = *p.cur_src + p.advance;
  long long b = (start + k) % nb;
  if (b < 0) b += nb;
  const long long n = (long long)p.B * p.F;
  const int32_t* si = p.ids_pool + b * n;
  const float* sv = p.vals_pool + b * n;
  int32_t* di = p.ids + (long long)k * p.Bp * p.F;
  float* dv = p.vals + (long long)k * p.Bp * p.F;
  uint32_t* dk = p.keys ? p.keys + (long long)k * n : nullptr;
  const uint32_t kb = (p.keys64 || p.plain_keys) ? 0u : (uint32_t)k << p.id_bits;
  unsigned long long* dk64 = p.keys64 ? p.keys64 + (long long)k * n : nullptr;
  const unsigned long long kb64 = (unsigned long long)k << p.id_bits;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int32_t id = guard_id(si[i], p.bad_ids, p.max_id);
    di[i] = id;
    dv[i] = sv[i];
    if (dk || dk64) {
      const uint32_t u = (uint32_t)id;
      const uint32_t key =
          p.shard_W > 0 ? shard_key(u, (uint32_t)p.shard_W, p.shard_Vs, p.shard_hot, p.shard_nhot) : u;
      if (dk64)
        dk64[i] = kb64 | key;
      else
        dk[i] = kb | key;
    }
  }
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < p.B; i += (long long)gridDim.x * 256)
    p.labels[(long long)k * p.Bp + i] = p.labels_pool[b * p.B + i];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t st = *p.step_src + p.advance + k;
    p.steps[k] = (p.halt != nullptr && *p.halt != 0) ? (st | kHaltStepBit) : st;
    p.lrt[k] = p.opt_type == kAdam ? adam_lr_t(p.lr, p.beta1, p.beta2, st) : p.lr;
    if (k == 0) {
      *p.cur_dst = start;
      *p.step_dst = *p.step_src + p.advance;
    }
  }
}

__global__ __launch_bounds__(256) void sort_aux_kernel(const SortAuxParams p) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long total = (long long)p.S * p.n;
  if (i < total) {
    const int k = (int)(i / p.n);
    p.pos[p.svals[i]] = (int32_t)(i - (long long)k * p.n);
    if (p.skeys64) p.skeys_out[i] = (uint32_t)(p.skeys64[i] & ((1ull << p.id_bits) - 1ull));
  }
  if (p.chunk_end) {
    const int nch = (p.n + p.chunk - 1) / p.chunk;
    if (i < (long long)p.S * nch) {
      const int k = (int)(i / nch), c = (int)(i - (long long)k * nch);
      const int last = min((c + 1) * p.chunk, p.n) - 1;
      int lo = last + 1, hi = p.n;  // first position after `last` whose key differs (sorted)
      if (p.skeys64) {  // (the 32-bit copies are being written by this same launch)
        const unsigned long long* kb = p.skeys64 + (size_t)k * p.n;
        const unsigned long long key = kb[last];
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (kb[mid] == key) lo = mid + 1; else hi = mid;
        }
      } else {
        const uint32_t* kb = p.skeys + (size_t)k * p.n;
        const uint32_t key = kb[last];
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (kb[mid] == key) lo = mid + 1; else hi = mid;
        }
      }
      p.chunk_end[i] = lo;
    }
  }
}

// One workgroup of `chunk` threads per (batch, chunk): run heads of the chunk (ballot counts).
__global__ __launch_bounds__(1024) void chunk_heads_kernel(const SortAuxParams p, int nch) {
  __shared__ int s_w[16];
  const int k = blockIdx.y, c = blockIdx.x, t = threadIdx.x;
  const uint32_t* kb = (p.skeys64 ? p.skeys_out : p.skeys) + (size_t)k * p.n;
  const int i = c * p.chunk + t;
  const uint32_t key = i < p.n ? kb[i] : 0u;
  const bool head = i < p.n && (i == 0 || key != kb[i - 1]);
  const unsigned long long m = __ballot(head);
  if ((t & 63) == 0) s_w[t >> 6] = __popcll(m);
  __syncthreads();
  if (p.chunk_heads != nullptr && t == 0) {
    int h = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) h += s_w[w];
    p.chunk_heads[(size_t)k * nch + c] = h;
  }
}

void launch_sort_aux(const SortAuxParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.n > 0 && p.S > 0 && p.chunk > 0, "sort_aux: bad sizes");
  ROCFM_REQUIRE(p.skeys64 == nullptr || (p.skeys_out != nullptr && p.id_bits >= 1 && p.id_bits <= 32),
                "sort_aux: 64-bit keys need skeys_out and id_bits");
  const long long total = std::max<long long>((long long)p.S * p.n, (long long)p.S * ((p.n + p.chunk - 1) / p.chunk));
  hipLaunchKernelGGL(sort_aux_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
  if (p.chunk_heads) {  // after sort_aux: the 64-bit path reads the plain ids it wrote
    ROCFM_REQUIRE(p.chunk % 64 == 0 && p.chunk <= 1024, "sort_aux: chunk_heads needs chunk % 64 == 0, <= 1024");
    const int nch = (p.n + p.chunk - 1) / p.chunk;
    hipLaunchKernelGGL(chunk_heads_kernel, dim3(nch, p.S), dim3(p.chunk), 0, stream, p, nch);
    ROCFM_HIP_CHECK(hipGetLastError());
  }
}

// ---- per-tile dedup (DedupParams) ----------------------------------------------------------------
constexpr int kDedupBlock = 1024;

// Group head: first entry of its batch segment, or its id or row tile differs from the previous
// entry's.  (Entries of one id are ascending in lookup index, so tiles are non-decreasing.)
__device__ __forceinline__ bool dedup_head(const DedupParams& p, int k, int j) {
  if (j == 0) return true;
  const size_t o = (size_t)k * p.n;
  if (p.skeys[o + j] != p.skeys[o + j - 1]) return true;
  const int vb = k * p.val_base_step;
  const int ta = ((int)p.svals[o + j] - vb) / p.F / p.rt, tb = ((int)p.svals[o + j - 1] - vb) / p.F / p.rt;
  return ta != tb;
}

__global__ __launch_bounds__(kDedupBlock) void dedup_count_kernel(const DedupParams p, int nblk) {
  __shared__ int s_w[kDedupBlock / 64];
  const int k = blockIdx.y, blk = blockIdx.x, t = threadIdx.x;
  const int j = blk * kDedupBlock + t;
  const bool h = j < p.n && dedup_head(p, k, j);
  const unsigned long long m = __ballot(h);
  if ((t & 63) == 0) s_w[t >> 6] = __popcll(m);
  __syncthreads();
  if (t == 0) {
    int c = 0;
    for (int w = 0; w < kDedupBlock / 64; ++w) c += s_w[w];
    p.bcount[(size_t)k * nblk + blk] = c;
  }
}

__global__ __launch_bounds__(kDedupBlock) void dedup_write_kernel(const DedupParams p, int nblk) {
  __shared__ int s_w[kDedupBlock / 64];
  __shared__ int s_base;
  const int k = blockIdx.y, blk = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t < 64) {  // heads before this block: Σ of the earlier blocks' counts (fixed order)
    int b = 0;
    for (int q = lane; q < blk; q += 64) b += p.bcount[(size_t)k * nblk + q];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) b += __shfl_xor(b, o, 64);
    if (t == 0) s_base = b;
  }
  const int j = blk * kDedupBlock + t;
  const bool in = j < p.n;
  const bool h = in && dedup_head(p, k, j);
  const unsigned long long m = __ballot(h);
  if (lane == 0) s_w[wave] = __popcll(m);
  __syncthreads();
  int before = s_base;
  for (int w = 0; w < wave; ++w) before += s_w[w];
  before += __popcll(m & ((1ull << lane) - 1ull));
  if (!in) return;
  const int c = before + (h ? 0 : -1);  // this lookup's group in the compacted list
  const size_t o = (size_t)k * p.n;
  const int vb = k * p.val_base_step;
  const int lk = (int)p.svals[o + j] - vb;  // in-batch lookup index
  p.pos[o + lk] = h ? c : ~c;
  const bool more = j + 1 < p.n && !dedup_head(p, k, j + 1);
  p.nxt[o + lk] = more ? (int)p.svals[o + j + 1] - vb : -1;
  if (h) p.ckeys[o + c] = p.skeys[o + j];
  if (j == p.n - 1) p.count[k] = c + 1;
}

// One workgroup of `chunk` threads per (batch, compacted chunk): the end of the chunk's last run
// (binary search) and its run heads.
__global__ __launch_bounds__(512) void dedup_chunks_kernel(const DedupParams p, int nch) {
  __shared__ int s_w[8];
  const int k = blockIdx.y, c = blockIdx.x, t = threadIdx.x;
  const int cnt = p.count[k];
  const uint32_t* kb = p.ckeys + (size_t)k * p.n;
  const int i0 = c * p.chunk;
  if (p.chunk_heads) {
    int h = 0;
    for (int i = i0 + t; i < min(i0 + p.chunk, cnt); i += blockDim.x) h += (i == 0 || kb[i] != kb[i - 1]) ? 1 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o, 64);
    if ((t & 63) == 0) s_w[t >> 6] = h;
    __syncthreads();
    if (t == 0) {
      int tot = 0;
      for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += s_w[w];
      p.chunk_heads[(size_t)k * nch + c] = tot;
    }
  }
  if (p.chunk_end && t == 0) {
    int end = cnt;
    if (i0 < cnt) {
      const int last = min(i0 + p.chunk, cnt) - 1;
      const uint32_t key = kb[last];
      int lo = last + 1, hi = cnt;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (kb[mid] == key) lo = mid + 1; else hi = mid;
      }
      end = lo;
    }
    p.chunk_end[(size_t)k * nch + c] = end;
  }
}

int dedup_scratch_ints(int n, int S) { return S * ((n + kDedupBlock - 1) / kDedupBlock); }

void launch_dedup(const DedupParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.n > 0 && p.S > 0 && p.F > 0 && (p.rt == 4 || p.rt == 8 || p.rt == 16), "dedup: bad sizes");
  ROCFM_REQUIRE(p.skeys && p.svals && p.pos && p.nxt && p.ckeys && p.count && p.bcount, "dedup: buffers missing");
  ROCFM_REQUIRE(p.chunk > 0 && p.chunk <= 512 && (p.chunk_end || p.chunk_heads || true), "dedup: chunk");
  const int nblk = (p.n + kDedupBlock - 1) / kDedupBlock;
  hipLaunchKernelGGL(dedup_count_kernel, dim3(nblk, p.S), dim3(kDedupBlock), 0, stream, p, nblk);
  hipLaunchKernelGGL(dedup_write_kernel, dim3(nblk, p.S), dim3(kDedupBlock), 0, stream, p, nblk);
  if (p.chunk_end || p.chunk_heads) {
    const int nch = (p.n + p.chunk - 1) / p.chunk;
    hipLaunchKernelGGL(dedup_chunks_kernel, dim3(nch, p.S), dim3(std::min(512, (p.chunk + 63) / 64 * 64)), 0, stream,
                       p, nch);
  }
  ROCFM_HIP_CHECK(hipGetLastError());
}

void launch_fetch_multi(const FetchMultiParams& p, hipStream_t stream) {
  ROCFM_REQUIRE(p.pool_batches > 0 && p.S > 0, "fetch_multi: empty pool / S");
  ROCFM_REQUIRE(p.cur_dst != p.cur_src && p.step_dst != p.step_src, "fetch_multi: counters must differ");
  ROCFM_REQUIRE(p.keys == nullptr || p.plain_keys || ((unsigned long long)p.S << p.id_bits) <= (1ull << 32),
                "fetch_multi: S << id_bits must fit in 32 bits (use plain per-batch keys)");
  ROCFM_REQUIRE(!p.plain_keys || (p.keys != nullptr && p.keys64 == nullptr), "fetch_multi: plain_keys needs keys");
  ROCFM_REQUIRE(p.keys64 == nullptr || p.id_bits <= 32, "fetch_multi: ids wider than 32 bits");
  const long long n = (long long)p.B * p.F;
  const int gx = (int)std::max<long long>(1, std::min<long long>((n + 255) / 256, 64));
  hipLaunchKernelGGL(fetch_multi_kernel, dim3(gx, p.S), dim3(256), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

}  // namespace rocfm
