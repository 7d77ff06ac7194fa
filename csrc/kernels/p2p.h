// One-shot xGMI push exchange over IPC-mapped peer buffers (p2p.hip).
//
// RCCL's all-gather of the ~1 MB DP bucket is latency-bound on a
// fully connected xGMI node (8 ranks → 7 ring hops).  Here every rank PUSHES its buffer straight
// into every peer's receive buffer — 7 peer links carry 7 copies at once, one hop each — and a
// flag hand-off replaces the collective's protocol:
//
//   ready[s] at rank d  : d has entered exchange n (its readers of the previous exchange are done,
//                         by stream order), so s may overwrite d's slot s.
//   data[s]  at rank d  : s's payload of exchange n is in d's slot s (written after every
//                         workgroup of s fenced its stores at system scope).
//
// Flags carry the exchange number (a device counter that the kernel advances itself, so the
// launch is graph-capturable and replays correctly) and are only ever compared with ">=", so
// they never need resetting.  Receive buffers and flags are allocated uncached
// (hipDeviceMallocUncached) so peer writes are visible to later kernels without L2 maintenance.
// Every wait is bounded: a peer that never arrives sets a sticky error flag instead of hanging
// the GPU; the host checks it.
#pragma once
#include "../common.h"

#include <vector>

namespace rocfm {

constexpr int kP2PMaxW = 16;

struct P2PParams {
  const float4* src;      // local payload; destination d reads src + d * src_stride4
  long long n4;           // float4s per destination
  long long src_stride4;  // 0: all-gather (same payload to every rank); >0: equal-split all-to-all
  long long slot4;        // receive-slot stride: rank s's payload lands at recv[d] + s * slot4
  float4* recv[kP2PMaxW];   // recv[r]: rank r's receive buffer (IPC-mapped; recv[rank] is local)
  uint32_t* sig[kP2PMaxW];  // sig[r]: rank r's flags, [ready W][data W] u32 (IPC-mapped)
  uint32_t* ctrl;         // local [epoch, arrive]: exchanges done, workgroup arrivals of this launch
  int32_t* error;         // local sticky flag: 1 = a peer wait timed out
  int W, rank, chunks;    // grid = W * chunks workgroups: (destination, chunk)
  long long spin_limit;   // polls (≈60 ns each) before a wait gives up
};

void launch_p2p_push(const P2PParams& p, hipStream_t stream);

// Up to kP2PMultiMax distinct exchanges handed off by one launch (their peer waits overlap).
constexpr int kP2PMultiMax = 4;
struct P2PMulti {
  P2PParams x[kP2PMultiMax];
  int start[kP2PMultiMax + 1];  // first workgroup of each exchange; start[n] = grid size
  int n;
};
void launch_p2p_push_multi(const std::vector<P2PParams>& ps, hipStream_t stream);

// Memory for peer-visible buffers.  kind: 0 uncached, 1 fine-grained, 2 plain hipMalloc.
uintptr_t p2p_malloc(size_t bytes, int kind);
void p2p_free(uintptr_t ptr);
void p2p_ipc_handle(uintptr_t ptr, char* out64);          // hipIpcGetMemHandle (64 bytes)
uintptr_t p2p_ipc_open(const char* handle64);            // hipIpcOpenMemHandle (lazy peer access)
void p2p_ipc_close(uintptr_t ptr);

}  // namespace rocfm
