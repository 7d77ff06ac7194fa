// rocfm host runtime: TFRecord framing, CRC32C, fixed-schema tf.train.Example codec.
//
// Replaces the native pieces the reference gets from TensorFlow:
//   * tf.data.TFRecordDataset framing + masked CRC32C       (PS:147, HVD:128)
//   * tf.parse_example with three FixedLenFeatures           (PS:117-126, HVD:109-118)
//   * tf.python_io.TFRecordWriter + Example serialisation    (tools/libsvm_to_tfrecord.py:29-57)
// The decoder is a hand-rolled protobuf wire-format walker specialised to the DeepFM schema
// {label: float[1], ids: int64[F], values: float[F]} (feature names configurable).  It accepts
// packed and unpacked repeated fields, ignores unknown features and decodes straight into the
// caller's batch buffers (ids narrowed to int32 — feature_size < 2^31).
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string>
#include <vector>

namespace rocfm {
namespace io {

uint32_t crc32c(const uint8_t* data, size_t n, uint32_t crc = 0);
// CRC32C of three buffers at once (interleaved instruction streams).
void crc32c_x3(const uint8_t* const p[3], const size_t n[3], uint32_t out[3]);
inline uint32_t mask_crc(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }
inline uint32_t unmask_crc(uint32_t m) {
  uint32_t r = m - 0xa282ead8u;
  return (r >> 17) | (r << 15);
}

struct Schema {
  std::string label_key = "label";
  std::string ids_key = "ids";
  std::string vals_key = "values";
  int field_size = 0;
};

enum ParseStatus : int {
  kOk = 0,
  kBadProto = 1,
  kMissingFeature = 2,
  kWrongLength = 3,
  kIdOutOfRange = 4,
};

// Decode one serialised Example into label/ids/vals (each field_size long).  Returns ParseStatus.
int decode_example(const uint8_t* p, size_t n, const Schema& s, float* label, int32_t* ids, float* vals,
                   int64_t max_id);

// Serialise one Example with the schema (int64 ids, packed).  Appends to out.
void encode_example(const Schema& s, float label, const int64_t* ids, const float* vals, int n,
                    std::string* out);

// Append one TFRecord frame around payload.
void frame_record(const uint8_t* payload, size_t n, std::string* out);

// Walk a TFRecord buffer; returns record (offset,len) pairs of payloads.  On a framing or CRC
// failure: if skip_bad, stops at the first framing error and skips CRC-bad records; otherwise
// throws std::runtime_error.
struct RecordRef {
  const uint8_t* data;
  uint32_t len;
};
// verify_data = false checks the framing only (length CRCs); the caller then owns the data CRCs.
size_t scan_records(const uint8_t* buf, size_t n, bool verify_crc, bool skip_bad, std::vector<RecordRef>* out,
                    size_t* bad_records, bool verify_data = true);

}  // namespace io
}  // namespace rocfm
