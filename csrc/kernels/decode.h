// Device-side tf.train.Example parsing (decode.hip): the reference's vectorized
// tf.parse_example (PS:117-126, HVD:109-118) moved off the host.  The host loader (raw mode,
// csrc/io/loader.h) only resolves frames, checks CRCs and copies the payload bytes of each batch
// into pinned memory; after the H2D copy this kernel parses every record into the engine's batch
// ring (ids int32 [B,F], values f32 [B,F], label f32 [B]) on the copy stream.
#pragma once
#include "../common.h"

namespace rocfm {

constexpr int kDecodeKeyMax = 16;  // feature-name bytes compared on the device

struct DecodeParams {
  const uint8_t* bytes;   // [nb][cap] payloads of batch b back to back from bytes + b·cap
  const int32_t* offs;    // [nb][B+1] record r of batch b = bytes[b·cap + offs[r] .. offs[r+1])
  long long cap;          // bytes per batch row (multiple of 16)
  int nb, B, F;
  int32_t* ids;           // ring [R][B][F]
  float* vals;            // ring [R][B][F]
  float* labels;          // ring [R][B]
  int slot0, R;           // batch b → ring slot (slot0 + b) % R
  long long max_id;       // ids must be < max_id (0: < 2^31)
  int batch0;             // sequence number of batch 0 (error reports)
  int32_t* err;           // [4] sticky: status (tfrecord.h ParseStatus), batch, record, 0
  unsigned long long keyw[3][2];  // label, ids, values feature names: ≤ 16 bytes each, little-endian
  int klen[3];                     //   words (zero-padded), compared 8 bytes at a time
};

void launch_decode_examples(const DecodeParams& p, hipStream_t stream);
size_t decode_lds_bytes(int F);  // dynamic LDS of one decode workgroup
bool decode_fits(int F);         // F ≤ 192 and that LDS fits the current device (opt-in limit)

}  // namespace rocfm
