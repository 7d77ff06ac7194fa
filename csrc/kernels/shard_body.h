// Device body of the owner's row serve (shard.hip; also a workgroup role of merge.hip's
// search-mode apply in the bounded-staleness row-shard mode).
#pragma once
#include "shard.h"

namespace rocfm {

// Thread i serves float4 column (i mod Kp/4) of request (i div Kp/4).
__device__ __forceinline__ void shard_serve_body(const ShardServeParams& p, const long long i) {
  const int KP4 = p.Kp >> 2;
  if (i >= (long long)p.m * KP4) return;
  const int r = (int)(i / KP4), c = (int)(i - (long long)r * KP4);
  const uint32_t id = p.ids[r];
  const bool pad = id == 0xFFFFFFFFu;
  const uint32_t lr = id / (uint32_t)p.W;
  const bool ok = !pad && (int)(id % (uint32_t)p.W) == p.rank && lr < p.Vs;
  if (!pad && !ok && p.bad) *p.bad = 1;
  if (p.rows_out) {
    // load row 0 for requests this owner does not serve and zero the value: `ok ? load : 0`
    // compiled to a select between a global and a private address (flat access + scratch)
    float4 v = tbl_load4_rt(p.table, (size_t)(ok ? lr : 0u) * KP4 + c, p.tbl_bf16 != 0);
    if (!ok) v = make_float4(0.f, 0.f, 0.f, 0.f);
    reinterpret_cast<float4*>(p.rows_out)[(size_t)r * KP4 + c] = v;
  }
  if (c == 0 && p.lkeys) p.lkeys[r] = ok ? lr : p.Vs;
}

}  // namespace rocfm
