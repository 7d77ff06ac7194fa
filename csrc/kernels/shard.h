// Parameter blocks of the row-shard routing kernels (shard.hip) — the Parameter-Server mode of the
// reference (PS:521-531, every fm_w/fm_v row lives on exactly one server) as a row-sharded table:
// id i is owned by rank i % W and stored there at local row i / W.
#pragma once
#include "../common.h"

namespace rocfm {

// key' = (id % W) * Vs + id / W : owner-major order, so one radix sort groups a batch's lookups by
// owner and, inside an owner, by local row.
struct ShardKeysParams {
  const int32_t* ids;  // [n] global ids
  int n;
  int W;
  uint32_t Vs;         // rows per shard (ceil(V / W))
  uint32_t* keys;      // [n] owner-major keys
  const uint32_t* hot_ids;  // [n_hot] ascending replicated ("hot") ids (nullable)
  int n_hot;
};

// Hot-row replication: the n_hot replicated ids form a virtual owner W (key W·Vs + slot) — sorted
// after every real owner, never requested from anyone; their lookups read the local replica.
__device__ __forceinline__ uint32_t shard_key(uint32_t id, uint32_t W, uint32_t Vs, const uint32_t* hot, int nhot) {
  if (nhot > 0) {
    int lo = 0, len = nhot;
    while (len > 0) {
      const int h = len >> 1;
      if (hot[lo + h] < id) {
        lo += h + 1;
        len -= h + 1;
      } else {
        len = h;
      }
    }
    if (lo < nhot && hot[lo] == id) return W * Vs + (uint32_t)lo;
  }
  return (id % W) * Vs + id / W;
}

// From the sorted (key', lookup) pairs of one batch: the unique ids each owner must serve, and for
// every lookup the row of the received-rows buffer ([W][cap][Kp]) that will hold its embedding.
struct ShardRouteParams {
  const uint32_t* skeys;  // [n] sorted owner-major keys
  const uint32_t* svals;  // [n] lookup index (row * F + field)
  int n;
  int W;
  uint32_t Vs;
  int cap;                // per-owner capacity of the exchange buffers
  uint32_t* send_ids;     // [W][cap] global ids requested from each owner; 0xFFFFFFFF = padding
  int32_t* local_idx;     // [>= n] lookup order: row (o * cap + j) of the received-rows buffer
                          //   (hot ids, virtual owner W: row W·cap + slot, the local replica)
  uint32_t* skeys_local;  // [n] sorted order: the same rows (input of the local gradient reduction)
  int32_t* counts;        // [W] unique ids per owner this batch (> cap means overflow)
  int32_t* overflow;      // sticky flag: set to 1 when any owner needs more than cap rows
  int32_t* scratch;       // [route_scratch_ints(n)] per-tile run-head counts
  uint32_t key_base;      // subtracted from skeys (a batch's segment of a multi-batch sort)
  uint32_t val_base;      // subtracted from svals (ditto)
};

// Owner side: serve the requested rows and emit the local row keys of the requests.
struct ShardServeParams {
  const uint32_t* ids;  // [m] requested global ids (0xFFFFFFFF = padding)
  int m;
  int W, rank;
  uint32_t Vs;
  const float* table;   // [Vs][Kp] this rank's shard
  int Kp;
  float* rows_out;      // [m][Kp] (nullable: keys only)
  uint32_t* lkeys;      // [m] local row, Vs for padding (nullable: rows only)
  int32_t* bad;         // nullable: set to 1 if a request is not owned by this rank
  int tbl_bf16;         // 1: table holds bf16 rows (rows_out stays f32)
};

void launch_shard_keys(const ShardKeysParams& p, hipStream_t stream);
void launch_shard_route(const ShardRouteParams& p, hipStream_t stream);
int route_scratch_ints(int n);
void launch_shard_serve(const ShardServeParams& p, hipStream_t stream);

}  // namespace rocfm
