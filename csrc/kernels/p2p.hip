// One-shot xGMI push exchange — see p2p.h for the protocol.
#include "p2p.h"

#include <cstring>

namespace rocfm {
namespace {

constexpr int kP2PThreads = 256;

__device__ __forceinline__ uint32_t ld_acquire_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_release_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Bounded wait for *p >= n (wrap-safe).  Returns false on timeout.
__device__ bool wait_geq(const uint32_t* p, uint32_t n, long long limit) {
  for (long long i = 0; i < limit; ++i) {
    if ((int32_t)(ld_acquire_sys(p) - n) >= 0) return true;
    __builtin_amdgcn_s_sleep(2);
  }
  return false;
}

// One exchange's share of a push launch: workgroup bid of its nblocks = W * chunks.
__device__ __forceinline__ void p2p_push_body(const P2PParams& p, const int bid, const int nblocks) {
  const int W = p.W, me = p.rank;
  const int d = bid / p.chunks, c = bid - d * p.chunks;
  __shared__ uint32_t s_n;
  if (threadIdx.x == 0) {
    const uint32_t n = __hip_atomic_load(p.ctrl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    s_n = n;
    if (bid == 0)  // this rank has entered exchange n: peers may overwrite its slots
      for (int r = 0; r < W; ++r)
        if (r != me) st_release_sys(p.sig[r] + me, n);
    if (d != me && !wait_geq(p.sig[me] + d, n, p.spin_limit)) atomicOr(p.error, 1);
  }
  __syncthreads();
  const uint32_t n = s_n;

  const long long per = (p.n4 + p.chunks - 1) / p.chunks;
  const long long lo = (long long)c * per;
  const long long hi = lo + per < p.n4 ? lo + per : p.n4;
  const float4* __restrict__ s = p.src + (long long)d * p.src_stride4;
  float4* __restrict__ o = p.recv[d] + (long long)me * p.slot4;
  constexpr int U = 4;
  long long i = lo + threadIdx.x;
  for (; i + (U - 1) * kP2PThreads < hi; i += U * kP2PThreads) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = s[i + u * kP2PThreads];
#pragma unroll
    for (int u = 0; u < U; ++u) o[i + u * kP2PThreads] = v[u];
  }
  for (; i < hi; i += kP2PThreads) o[i] = s[i];
  // Publish (counter form, system scope): every wave waits for its own payload stores → barrier →
  // lane 0 release fence → an explicit wait (the compiler may drop the fence's own) → the ticket.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // "" = system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t prev = __hip_atomic_fetch_add(p.ctrl + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (uint32_t)nblocks - 1u) {  // last workgroup: every payload store of this rank is done
      __hip_atomic_store(p.ctrl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      for (int r = 0; r < W; ++r)
        if (r != me) st_release_sys(p.sig[r] + W + me, n);
      bool ok = true;
      for (int r = 0; r < W; ++r)
        if (r != me) ok = wait_geq(p.sig[me] + W + r, n, p.spin_limit) && ok;
      if (!ok) atomicOr(p.error, 1);
      __hip_atomic_store(p.ctrl, n, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ __launch_bounds__(kP2PThreads) void p2p_push_kernel(P2PParams p) {
  p2p_push_body(p, blockIdx.x, gridDim.x);
}

// Several independent exchanges handed off by ONE launch (row-shard X3 + X4 + the next step's X1):
// each exchange keeps its own flags and counters, so their peer waits overlap instead of running
// as consecutive launches.  Workgroups [start[i], start[i+1]) serve exchange i.
__global__ __launch_bounds__(kP2PThreads) void p2p_push_multi_kernel(P2PMulti m) {
  int i = 0;
#pragma unroll
  for (int j = 1; j < kP2PMultiMax; ++j)
    if (j < m.n && (int)blockIdx.x >= m.start[j]) i = j;
  p2p_push_body(m.x[i], blockIdx.x - m.start[i], m.start[i + 1] - m.start[i]);
}

}  // namespace

static void check_push(const P2PParams& p) {
  ROCFM_REQUIRE(p.W >= 1 && p.W <= kP2PMaxW && p.rank >= 0 && p.rank < p.W, "p2p: bad W/rank");
  ROCFM_REQUIRE(p.chunks >= 1 && (long long)p.W * p.chunks < (1ll << 24), "p2p: bad chunks");
  ROCFM_REQUIRE(p.src && p.ctrl && p.error && p.n4 >= 0 && p.slot4 >= p.n4, "p2p: bad buffers");
  for (int r = 0; r < p.W; ++r) ROCFM_REQUIRE(p.recv[r] && p.sig[r], "p2p: peer buffer not mapped");
}

void launch_p2p_push(const P2PParams& p, hipStream_t stream) {
  check_push(p);
  hipLaunchKernelGGL(p2p_push_kernel, dim3(p.W * p.chunks), dim3(kP2PThreads), 0, stream, p);
  ROCFM_HIP_CHECK(hipGetLastError());
}

void launch_p2p_push_multi(const std::vector<P2PParams>& ps, hipStream_t stream) {
  ROCFM_REQUIRE(!ps.empty() && (int)ps.size() <= kP2PMultiMax, "p2p: 1..4 exchanges per multi push");
  P2PMulti m{};
  m.n = (int)ps.size();
  int tot = 0;
  for (int i = 0; i < m.n; ++i) {
    check_push(ps[i]);
    for (int j = 0; j < i; ++j)  // each exchange's counters are its own (one launch per exchange at a time)
      ROCFM_REQUIRE(ps[j].ctrl != ps[i].ctrl, "p2p: one exchange twice in a multi push");
    m.x[i] = ps[i];
    m.start[i] = tot;
    tot += ps[i].W * ps[i].chunks;
  }
  m.start[m.n] = tot;
  hipLaunchKernelGGL(p2p_push_multi_kernel, dim3(tot), dim3(kP2PThreads), 0, stream, m);
  ROCFM_HIP_CHECK(hipGetLastError());
}

uintptr_t p2p_malloc(size_t bytes, int kind) {
  void* ptr = nullptr;
  if (kind == 0)
    ROCFM_HIP_CHECK(hipExtMallocWithFlags(&ptr, bytes, hipDeviceMallocUncached));
  else if (kind == 1)
    ROCFM_HIP_CHECK(hipExtMallocWithFlags(&ptr, bytes, hipDeviceMallocFinegrained));
  else
    ROCFM_HIP_CHECK(hipMalloc(&ptr, bytes));
  ROCFM_HIP_CHECK(hipMemset(ptr, 0, bytes));
  ROCFM_HIP_CHECK(hipDeviceSynchronize());
  return reinterpret_cast<uintptr_t>(ptr);
}

void p2p_free(uintptr_t ptr) { ROCFM_HIP_CHECK(hipFree(reinterpret_cast<void*>(ptr))); }

void p2p_ipc_handle(uintptr_t ptr, char* out64) {
  hipIpcMemHandle_t h;
  static_assert(sizeof(h) == 64, "hipIpcMemHandle_t is 64 bytes");
  ROCFM_HIP_CHECK(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(ptr)));
  std::memcpy(out64, &h, sizeof(h));
}

uintptr_t p2p_ipc_open(const char* handle64) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle64, sizeof(h));
  void* ptr = nullptr;
  ROCFM_HIP_CHECK(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess));
  return reinterpret_cast<uintptr_t>(ptr);
}

void p2p_ipc_close(uintptr_t ptr) { ROCFM_HIP_CHECK(hipIpcCloseMemHandle(reinterpret_cast<void*>(ptr))); }

}  // namespace rocfm
