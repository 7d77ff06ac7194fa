// Producer-side push of the DP exchange (see p2p.h for the flag protocol).
//
// With the plain p2p exchange a step runs  tail (MLP wgrad ‖ row export into a local send
// buffer) → push kernel (copy the buffer into every peer's receive slot) → merge.  With a
// PushTarget the producers write their results straight into the W receive slots instead — the
// wgrad workgroups their MLP gradients, the export workgroups their (id, Σ grad row) pairs — so
// the xGMI transfer runs under the tail's own compute, the way Horovod overlaps its fusion-buffer
// all-reduce with the backward (HVD:296).  The push launch that follows carries only the row
// count (16 B) and the data hand-off.
//
// Readiness: rank d may be written into for exchange n once it has entered n, i.e. once its
// merge of exchange n−1 (the last reader of its receive buffer) is done.  The row kernel of step
// n runs after that merge in stream order, so its workgroup 0 raises "entered n" at every peer
// (push_signal_ready); producers check the flags before their first store into a peer's slot
// (issued early with push_ready_load, polled again only if a peer is behind).  n is the local
// exchange counter + 1 (the push launch advances the counter at the end of every exchange).
#pragma once
#include "../common.h"

namespace rocfm {

constexpr int kPushMaxW = 8;  // one node

struct PushTarget {
  int W;                           // 0: no fused push (producers write their local buffers)
  int rank;
  float* slot[kPushMaxW];          // this rank's slot in rank d's receive buffer (d == rank: local)
  uint32_t* peer_sig[kPushMaxW];   // rank d's flag block [ready W][data W] (IPC-mapped)
  const uint32_t* ctrl;            // local exchange counter (p2p.hip)
  int32_t* error;                  // local sticky flag: a peer never became ready
  long long spin_limit;
};

__device__ __forceinline__ uint32_t push_exchange_no(const PushTarget& t) {
  return __hip_atomic_load(t.ctrl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
}

// One thread of the row kernel: this rank has entered exchange n.  The flag publishes no data of
// this rank (its reads of the slots ended with an earlier kernel), so the store is relaxed: a
// release here would write back this XCD's whole L2 ahead of the row kernel's first loads.
__device__ __forceinline__ void push_signal_ready(const PushTarget& t) {
  const uint32_t n = push_exchange_no(t);
  for (int r = 0; r < t.W; ++r)
    if (r != t.rank) __hip_atomic_store(t.peer_sig[r] + t.rank, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// What a producer reads at its start (ctrl and every peer's "entered" flag) without waiting on any
// of it: the values are only compared at its first store (push_wait_ready), so the loads fly under
// the producer's own first round trip instead of holding the wave in front of it.
struct PushSeen {
  uint32_t done;               // exchanges completed (ctrl): this exchange is done + 1
  uint32_t ready[kPushMaxW];   // ready[d]: last exchange rank d entered
};

__device__ __forceinline__ PushSeen push_ready_load(const PushTarget& t) {
  PushSeen s;
  s.done = __hip_atomic_load(t.ctrl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t* mine = t.peer_sig[t.rank];
#pragma unroll
  for (int d = 0; d < kPushMaxW; ++d)
    s.ready[d] = (d < t.W && d != t.rank) ? __hip_atomic_load(mine + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                          : 0u;
  return s;
}

// Before the first store into a peer's slot: every peer has entered exchange n (bounded wait).
// Only a load → store order is needed (the peer's reads of the slot finished before it signalled):
// the stores are issued after the flag values have returned and been compared, so the polls are
// relaxed — an acquire fence here would invalidate this XCD's L2 under the tail's own loads.
__device__ __forceinline__ void push_wait_ready(const PushTarget& t, const PushSeen& s) {
  const uint32_t n = s.done + 1u;
  const uint32_t* mine = t.peer_sig[t.rank];
#pragma unroll
  for (int d = 0; d < kPushMaxW; ++d) {
    if (d >= t.W || d == t.rank || (int32_t)(s.ready[d] - n) >= 0) continue;
    long long i = 0;
    while ((int32_t)(__hip_atomic_load(mine + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - n) < 0) {
      if (++i >= t.spin_limit) {
        atomicOr(t.error, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
}

// End of a producer's pushes: wait until this wave's stores into the slots are acknowledged.  The
// push launch that follows signals the data to the peers; stores still in flight when a wave
// ends are not covered by that launch's release fence (measured: the last stores of the tail
// arrived after the hand-off without this wait).
__device__ __forceinline__ void push_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace rocfm
