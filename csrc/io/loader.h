// rocfm host runtime: multi-threaded TFRecord batch loader (replaces the tf.data C++ runtime the
// reference's input_fn drives: PS:112-169, HVD:104-161).
//
// Pipeline (per epoch, like the reference's shard → batch(drop_remainder) → parse → repeat):
//   reader thread : mmap file (or read a FIFO/stdin in pipe mode) → record offsets from the file's
//                   persistent index (record_index.h; built by one framing walk and saved the
//                   first time) → keep every shard_count-th record starting at shard_index
//                   (record index runs over the concatenated file list, = Dataset.shard) without
//                   touching the others → optional shuffle buffer → cut batches of batch_size
//                   (tail dropped per epoch when drop_remainder; its records' CRCs are still
//                   checked) → job queue
//   N workers     : resolve a job's frames (length + length CRC), check the data CRCs (three
//                   records interleaved) and either decode the records straight into output slot
//                   (seq % num_slots) — host decode — or copy the raw Example payloads into the
//                   slot's byte buffer with their offsets (raw mode: the GPU parses them,
//                   csrc/kernels/decode.hip, so the host only moves bytes)
// skip_bad (on_bad_record=skip) keeps the legacy full walk: dropping a corrupt record there shifts
// the record index every rank shards by, so it must happen before sharding.
//   consumer      : next() returns slots strictly in sequence order; release() recycles them.
// Output slots are caller-provided host buffers (Python passes pinned torch tensors so the H2D copy
// is a true async DMA on a side HIP stream).
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "tfrecord.h"

namespace rocfm {
namespace io {

struct LoaderOptions {
  std::vector<std::string> files;
  Schema schema;
  int64_t max_id = 0;  // ids must be < max_id (0 = unchecked)
  int batch_size = 1024;
  bool drop_remainder = true;
  int num_epochs = 1;  // < 0 → forever
  int shard_count = 1;
  int shard_index = 0;
  int num_threads = 4;
  int num_slots = 4;
  bool verify_crc = true;
  bool skip_bad = false;
  int shuffle_buffer = 0;  // records; 0 = no record shuffle (reference default, Q6)
  uint64_t seed = 0;
  bool stream_mode = false;  // pipe mode: files are FIFOs / "-" for stdin, read sequentially
  int64_t skip_batches = 0;  // drop the first N batches undecoded (resume after a restart)
  int64_t max_batches_per_epoch = 0;  // > 0: stop each epoch after this many batches (ranks agree
                                      // on a common per-epoch count; the surplus is dropped)
  bool use_index = true;     // persistent per-file offset index (file mode without skip_bad)
  bool raw = false;          // raw mode: slots receive Example payload bytes + offsets
  int64_t raw_cap = 0;       // raw mode: byte capacity of one slot's payload buffer
};

struct Slot {
  int32_t* ids = nullptr;
  float* vals = nullptr;
  float* labels = nullptr;
  uint8_t* bytes = nullptr;  // raw mode: payloads of the batch, back to back
  int32_t* offs = nullptr;   // raw mode: [batch_size + 1] payload offsets into bytes
};

class BatchLoader {
 public:
  explicit BatchLoader(const LoaderOptions& opt);
  ~BatchLoader();
  void set_slot(int i, int32_t* ids, float* vals, float* labels);
  void set_raw_slot(int i, uint8_t* bytes, int32_t* offs);
  void start();
  // Blocks until the next batch is decoded.  Returns slot index and fills nrows/epoch; returns -1
  // at end of data.  Throws on decode/framing errors.
  int next(int* nrows, int* epoch);
  void release(int slot);
  // Up to max_n consecutive batches in consecutive slots (a group never wraps the slot ring):
  // blocks until all of them are decoded.  Returns the first slot and fills n (0 at end of data),
  // the row count of the group's last batch and its epoch.
  int next_group(int max_n, int* n, int* last_rows, int* epoch);
  void release_group(int first, int n);
  void stop();
  size_t bad_records() const { return bad_.load(); }
  size_t records_seen() const { return seen_.load(); }
  size_t index_fallbacks() const { return fallbacks_.load(); }  // files indexed by the sequential walk
  size_t index_loads() const { return index_loads_.load(); }    // files whose saved index was used
  size_t index_builds() const { return index_builds_.load(); }  // files indexed by a walk (and saved)

  struct Chunk;  // owns the bytes (mmap or arena)

 private:
  struct Job {
    int64_t seq;
    int epoch;
    std::vector<RecordRef> recs;  // framed: frame start + bytes left in the file (workers resolve)
    std::vector<std::shared_ptr<Chunk>> keep;
    bool framed = false;
  };
  void reader_main();
  void worker_main();
  void push_job(Job&& j);
  void fail(const std::string& msg);
  // framed refs → payload refs with every CRC checked (workers, and the reader for the dropped
  // remainder); returns an error message or ""
  std::string resolve(std::vector<RecordRef>* recs, int64_t seq) const;

  LoaderOptions opt_;
  std::vector<Slot> slots_;
  std::vector<int> slot_state_;    // 0 free, 1 filling, 2 ready
  std::vector<int64_t> slot_seq_;  // seq the slot currently holds / will hold
  std::vector<int> slot_rows_, slot_epoch_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job> jobs_;
  int64_t next_consume_ = 0;
  int64_t jobs_total_ = -1;  // set when reader finishes
  bool stop_ = false;
  std::string error_;
  std::thread reader_;
  std::vector<std::thread> workers_;
  std::atomic<size_t> bad_{0}, seen_{0}, fallbacks_{0}, index_loads_{0}, index_builds_{0};
  bool started_ = false;
};

// Decode an entire TFRecord file (small files: validation sets, tests).
size_t decode_file(const std::string& path, const Schema& s, int64_t max_id, bool verify_crc, bool skip_bad,
                   std::vector<float>* labels, std::vector<int32_t>* ids, std::vector<float>* vals);

// libsvm ("label id:val id:val ...") → TFRecord, multi-threaded, output order = input order.
// Mirrors tools/libsvm_to_tfrecord.py:22-61 (one Example per line, every pair kept).
// Returns number of records written.
// libsvm lines "label id:val id:val …" → tf.train.Example records (TOOL:22-61), written to
// out_paths.size() shards of contiguous records (input order kept).  Returns the record count.
size_t convert_libsvm(const std::string& in_path, const std::vector<std::string>& out_paths, const Schema& s,
                      int num_threads);

}  // namespace io
}  // namespace rocfm
