// rocfm host runtime: persistent per-file TFRecord offset index ("<file>.rfidx").
//
// The reference's record sharding (`dataset.shard(hvd.size(), hvd.rank())`, HVD:132-133; PS:153-156)
// keeps every P-th record, so each of P ranks would otherwise walk the length chain of EVERY record
// of every file to find its own (one dependent memory access per record, ≈70-90 ns) and the
// aggregate decode rate of one host stopped scaling with the rank count
// (profiles/r3_loader_aggregate.md: 18.7 M ex/s at 8 processes).  With the index a rank jumps to
// its own records: offsets[r], offsets[r + P], … and never touches the others.
//
// Layout (little endian):  IdxHeader (48 bytes) | uint64 frame_offset[n]
// The index is tied to the data file by (size, mtime_ns) and checked on load against the file's
// framing (first frame at 0, last frame ends exactly at EOF); any mismatch = stale = rebuilt.
// Written atomically (temporary file + rename) next to the data file, or under $ROCFM_INDEX_DIR
// when set (read-only data directories); a write failure is not an error (the index then lives
// in memory for this process only).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

#include "tfrecord.h"

namespace rocfm {
namespace io {

struct IdxHeader {
  char magic[8];        // "RFIDX\0v1"
  uint64_t file_size;   // data file size in bytes
  int64_t mtime_ns;     // data file modification time
  uint64_t n;           // records
  uint32_t max_len;     // longest payload (bytes)
  uint32_t flags;       // bit 0: every data CRC was verified when the index was built
  uint64_t reserved;
};
static_assert(sizeof(IdxHeader) == 48, "IdxHeader layout");

struct RecordIndex {
  const uint64_t* off = nullptr;  // frame start offsets [n]
  size_t n = 0;
  uint32_t max_len = 0;
  bool loaded = false;                // came from a sidecar (vs built by a walk)
  std::vector<uint64_t> own;          // storage when built in memory
  std::shared_ptr<void> map;          // mmap of the sidecar when loaded
};

// Sidecar path of a data file ($ROCFM_INDEX_DIR/<hash>-<basename>.rfidx or <path>.rfidx).
std::string index_path(const std::string& data_path);

// Load a valid sidecar for the mapped data file (buf, size); false when missing or stale.
bool load_index(const std::string& data_path, const uint8_t* buf, size_t size, RecordIndex* out);

// Index from walked payload references (the loader's framing walk): frame offset = payload - 12.
void index_from_refs(const uint8_t* buf, const std::vector<RecordRef>& refs, RecordIndex* out);

// Write the sidecar (atomic).  Returns false (and leaves no partial file) on any failure.
bool save_index(const std::string& data_path, const RecordIndex& ix, bool crc_verified);

// Walk + write in one call (converters / writers); returns the record count or throws on a
// framing error.  Verifies every CRC when verify_crc.
size_t build_index_file(const std::string& data_path, bool verify_crc);

}  // namespace io
}  // namespace rocfm
