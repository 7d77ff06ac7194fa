// rocfm host runtime: multi-threaded TFRecord batch loader (see loader.h).
#include "loader.h"

#include "record_index.h"

#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <fstream>
#include <future>
#include <random>
#include <sstream>
#include <stdexcept>

namespace rocfm {
namespace io {

struct BatchLoader::Chunk {
  const uint8_t* data = nullptr;
  size_t size = 0;
  void* map = nullptr;
  std::string arena;  // stream mode
  ~Chunk() {
    if (map && map != MAP_FAILED) munmap(map, size);
  }
};

namespace {
std::shared_ptr<BatchLoader::Chunk> map_file(const std::string& path, bool populate = false);
}

BatchLoader::BatchLoader(const LoaderOptions& opt) : opt_(opt) {
  if (opt_.batch_size <= 0) throw std::invalid_argument("batch_size must be > 0");
  if (opt_.shard_count <= 0 || opt_.shard_index < 0 || opt_.shard_index >= opt_.shard_count)
    throw std::invalid_argument("bad shard spec");
  if (opt_.num_slots < 2) opt_.num_slots = 2;
  if (opt_.num_threads < 1) opt_.num_threads = 1;
  if (opt_.raw && opt_.raw_cap <= 0) throw std::invalid_argument("raw mode needs raw_cap > 0");
  if (opt_.raw && opt_.skip_bad)
    throw std::invalid_argument("raw mode cannot skip bad records (a malformed Example is found on the GPU)");
  slots_.resize(opt_.num_slots);
  slot_state_.assign(opt_.num_slots, 0);
  slot_seq_.resize(opt_.num_slots);
  for (int i = 0; i < opt_.num_slots; ++i) slot_seq_[i] = i;
  slot_rows_.assign(opt_.num_slots, 0);
  slot_epoch_.assign(opt_.num_slots, 0);
}

BatchLoader::~BatchLoader() { stop(); }

void BatchLoader::set_slot(int i, int32_t* ids, float* vals, float* labels) {
  if (i < 0 || i >= (int)slots_.size()) throw std::out_of_range("slot");
  slots_[i] = Slot{ids, vals, labels};
}

void BatchLoader::set_raw_slot(int i, uint8_t* bytes, int32_t* offs) {
  if (i < 0 || i >= (int)slots_.size()) throw std::out_of_range("slot");
  slots_[i].bytes = bytes;
  slots_[i].offs = offs;
}

void BatchLoader::start() {
  if (started_) return;
  for (auto& s : slots_)
    if (opt_.raw ? (!s.bytes || !s.offs) : (!s.ids || !s.vals || !s.labels))
      throw std::runtime_error("all slots must be set before start()");
  started_ = true;
  reader_ = std::thread(&BatchLoader::reader_main, this);
  for (int i = 0; i < opt_.num_threads; ++i) workers_.emplace_back(&BatchLoader::worker_main, this);
}

void BatchLoader::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (reader_.joinable()) reader_.join();
  for (auto& t : workers_)
    if (t.joinable()) t.join();
  workers_.clear();
}

void BatchLoader::fail(const std::string& msg) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (error_.empty()) error_ = msg;
    stop_ = true;
  }
  cv_.notify_all();
}

void BatchLoader::push_job(Job&& j) {
  std::unique_lock<std::mutex> lk(mu_);
  // bound the queue: at most 2 × slots outstanding jobs
  cv_.wait(lk, [&] { return stop_ || (int)jobs_.size() < 2 * opt_.num_slots; });
  if (stop_) return;
  jobs_.push_back(std::move(j));
  lk.unlock();
  cv_.notify_all();
}

namespace {

// populate: map the page-cache pages up front (MAP_POPULATE) for files up to 1 GiB, so the decode
// workers never take minor faults (they serialise on the mm lock) — index mode reads records
// without a walk that would otherwise touch the pages first
std::shared_ptr<BatchLoader::Chunk> map_file(const std::string& path, bool populate) {
  auto c = std::make_shared<BatchLoader::Chunk>();
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("cannot open " + path + ": " + strerror(errno));
  struct stat st;
  if (fstat(fd, &st) != 0) {
    ::close(fd);
    throw std::runtime_error("cannot stat " + path);
  }
  c->size = (size_t)st.st_size;
  if (c->size) {
    const bool pop = populate && c->size <= ((size_t)1 << 30) && !getenv("ROCFM_NO_POPULATE");
    c->map = mmap(nullptr, c->size, PROT_READ, MAP_PRIVATE | (pop ? MAP_POPULATE : 0), fd, 0);
    if (c->map == MAP_FAILED) {
      ::close(fd);
      throw std::runtime_error("mmap failed for " + path);
    }
    madvise(c->map, c->size, MADV_SEQUENTIAL | MADV_WILLNEED);
    c->data = static_cast<const uint8_t*>(c->map);
  }
  ::close(fd);
  return c;
}

// Read TFRecord frames from a stream (FIFO / stdin) into an arena of ≈arena_bytes.
bool read_stream_chunk(FILE* f, size_t arena_bytes, bool verify, bool skip_bad, BatchLoader::Chunk* c,
                       std::vector<RecordRef>* recs, size_t* bad) {
  std::string& a = c->arena;
  a.clear();
  std::vector<std::pair<size_t, uint32_t>> offs;
  while (a.size() < arena_bytes) {
    uint8_t hdr[12];
    size_t got = fread(hdr, 1, 12, f);
    if (got == 0) break;
    if (got != 12) throw std::runtime_error("TFRecord stream: truncated header");
    uint64_t len;
    memcpy(&len, hdr, 8);
    uint32_t lcrc;
    memcpy(&lcrc, hdr + 8, 4);
    if (verify && mask_crc(crc32c(hdr, 8)) != lcrc) throw std::runtime_error("TFRecord stream: corrupt length CRC");
    size_t off = a.size();
    a.resize(off + len + 4);
    if (fread(&a[off], 1, len + 4, f) != len + 4) throw std::runtime_error("TFRecord stream: truncated record");
    bool ok = true;
    if (verify) {
      uint32_t dcrc;
      memcpy(&dcrc, &a[off + len], 4);
      ok = mask_crc(crc32c(reinterpret_cast<const uint8_t*>(&a[off]), len)) == dcrc;
      if (!ok && !skip_bad) throw std::runtime_error("TFRecord stream: corrupt data CRC");
    }
    if (ok)
      offs.emplace_back(off, (uint32_t)len);
    else
      ++*bad;
  }
  c->data = reinterpret_cast<const uint8_t*>(a.data());
  c->size = a.size();
  for (auto& o : offs) recs->push_back(RecordRef{c->data + o.first, o.second});
  return !offs.empty();
}

// First valid frame header at or after `from` (length CRC matches, frame fits), or n.  Searches at
// most `limit` bytes.
size_t resync(const uint8_t* buf, size_t n, size_t from, size_t limit) {
  const size_t stop = std::min(n, from + limit);
  for (size_t p = from; p + 16 <= stop; ++p) {
    uint64_t len;
    memcpy(&len, buf + p, 8);
    if (len > n - p - 16) continue;
    uint32_t lcrc;
    memcpy(&lcrc, buf + p + 8, 4);
    if (mask_crc(crc32c(buf + p, 8)) == lcrc) return p;
  }
  return n;
}

// Parallel framing walk of a mapped file.  The file is cut into `parts` byte ranges; each thread
// resynchronises to the first frame header in its range (length CRC match) and walks the frames
// whose header starts inside it, verifying CRCs when asked (so the CRC work is parallel too).
// The walk is exact: range k's chain must end precisely where range k+1's starts (range 0 starts
// at offset 0), which a false header match or any framing error breaks — then the caller falls
// back to the sequential scan_records, which also produces the reference error semantics.
// TFRecord framing is a length chain; a single thread walking it is bound by one memory latency
// per record (≈70-90 ns), i.e. it cannot feed more than ≈12 M records/s.
bool index_parallel(const uint8_t* buf, size_t n, bool verify, bool verify_data, bool skip_bad, int parts,
                    std::vector<RecordRef>* out, size_t* bad) {
  struct Part {
    size_t first = 0, end = 0, bad = 0;
    bool error = false;
    std::vector<RecordRef> recs;
  };
  volatile uint8_t sink = 0;  // page touches (non-verifying walk) must not be optimised away
  std::vector<Part> P(parts);
  auto run = [&](int k) {
    Part& pt = P[k];
    const size_t s = n * k / parts, e = n * (k + 1) / parts;
    size_t p = (k == 0) ? 0 : resync(buf, n, s, (size_t)16 << 20);
    pt.first = p;
    pt.recs.reserve((e - s) / 256 + 16);
    while (p < e && p + 12 <= n) {
      uint64_t len;
      memcpy(&len, buf + p, 8);
      uint32_t lcrc;
      memcpy(&lcrc, buf + p + 8, 4);
      if ((verify && mask_crc(crc32c(buf + p, 8)) != lcrc) || len > n - p - 16) {
        pt.error = true;
        return;
      }
      const uint8_t* payload = buf + p + 12;
      bool ok = true;
      if (verify && verify_data) {
        uint32_t dcrc;
        memcpy(&dcrc, payload + len, 4);
        ok = mask_crc(crc32c(payload, len)) == dcrc;
        if (!ok && !skip_bad) {
          pt.error = true;
          return;
        }
      } else {
        // touch the payload's pages here (the CRC pass does it when verifying): the mapping is
        // faulted in by these parallel index threads one file ahead, not by the decoders, whose
        // minor faults serialise on the mm lock (4 decoders ran 3x slower than 1)
        for (size_t q = ((size_t)(payload - buf) + 4095) & ~(size_t)4095; q < (size_t)(payload - buf) + len; q += 4096)
          sink += buf[q];
      }
      if (ok)
        pt.recs.push_back(RecordRef{payload, (uint32_t)len});
      else
        ++pt.bad;
      p += 12 + len + 4;
    }
    pt.end = p;
  };
  std::vector<std::thread> th;
  for (int k = 1; k < parts; ++k) th.emplace_back(run, k);
  run(0);
  for (auto& t : th) t.join();
  for (int k = 0; k < parts; ++k) {
    if (P[k].error) return false;
    const size_t next = (k + 1 < parts) ? P[k + 1].first : n;
    if (P[k].end != next) return false;
  }
  size_t tot = 0;
  for (auto& pt : P) tot += pt.recs.size();
  out->reserve(out->size() + tot);
  for (auto& pt : P) {
    out->insert(out->end(), pt.recs.begin(), pt.recs.end());
    *bad += pt.bad;
  }
  return true;
}

}  // namespace

void BatchLoader::reader_main() {
  try {
    int64_t seq = 0, skipped = 0;
    std::mt19937_64 rng(opt_.seed);
    const int B = opt_.batch_size;
    // index mode (file mode without skip_bad): every file's record offsets come from its saved
    // index, or from one parallel framing walk that then saves it; files are indexed one file
    // ahead of the emission.  Legacy mode (skip_bad): the walk checks every CRC and drops bad
    // records before sharding.
    const bool index_mode = opt_.use_index && !opt_.skip_bad;
    struct Indexed {
      std::shared_ptr<Chunk> chunk;
      std::vector<RecordRef> recs;  // legacy mode: payload refs
      RecordIndex ix;               // index mode
      size_t bad = 0;
    };
    const int parts = std::max(1, opt_.num_threads);
    auto walk = [this, parts](Indexed& ix, bool vdata) {
      const size_t n = ix.chunk->size;
      const int np = (int)std::min<size_t>((size_t)parts, std::max<size_t>(1, n >> 22));
      if (np < 2 ||
          !index_parallel(ix.chunk->data, n, opt_.verify_crc, vdata, opt_.skip_bad, np, &ix.recs, &ix.bad)) {
        if (np >= 2) ++fallbacks_;
        ix.recs.clear();
        ix.bad = 0;
        scan_records(ix.chunk->data, n, opt_.verify_crc, opt_.skip_bad, &ix.recs, &ix.bad, vdata);
      }
    };
    auto index = [this, walk, index_mode](const std::string& path) {
      Indexed ix;
      ix.chunk = map_file(path, index_mode);
      if (!index_mode) {
        walk(ix, true);
        return ix;
      }
      if (load_index(path, ix.chunk->data, ix.chunk->size, &ix.ix)) {
        ++index_loads_;
        return ix;
      }
      // framing + length CRCs only: every record's data CRC is checked by whoever resolves it
      walk(ix, false);
      index_from_refs(ix.chunk->data, ix.recs, &ix.ix);
      ix.recs.clear();
      ix.recs.shrink_to_fit();
      save_index(path, ix.ix, false);
      ++index_builds_;
      return ix;
    };
    std::future<Indexed> pending;
    if (!opt_.stream_mode && !opt_.files.empty()) pending = std::async(std::launch::async, index, opt_.files[0]);
    for (int epoch = 0; opt_.num_epochs < 0 || epoch < opt_.num_epochs; ++epoch) {
      Job cur;
      cur.epoch = epoch;
      cur.framed = index_mode && !opt_.stream_mode;
      std::vector<RecordRef> shuf;  // shuffle buffer
      std::vector<std::shared_ptr<Chunk>> shuf_keep;
      int64_t ridx = 0;  // record index across the concatenated file list (Dataset.shard)
      int64_t ep_batches = 0;
      const int64_t maxb = opt_.max_batches_per_epoch;
      auto full = [&] { return maxb > 0 && ep_batches >= maxb; };
      cur.recs.reserve(B);
      auto emit = [&](const RecordRef& r, const std::shared_ptr<Chunk>& keep) {
        if (full()) return;
        if (cur.keep.empty() || cur.keep.back() != keep) cur.keep.push_back(keep);
        cur.recs.push_back(r);
        if ((int)cur.recs.size() == B) {
          ++ep_batches;
          if (skipped < opt_.skip_batches) {  // resume: drop whole batches without decoding them
            ++skipped;
            cur.recs.clear();
            cur.keep.clear();
            return;
          }
          cur.seq = seq++;
          const bool framed = cur.framed;
          push_job(std::move(cur));
          cur = Job();
          cur.epoch = epoch;
          cur.framed = framed;
          cur.recs.reserve(B);
        }
      };
      auto take_own = [&](const RecordRef& r, const std::shared_ptr<Chunk>& keep) {
        if (opt_.shuffle_buffer > 0) {
          shuf.push_back(r);
          shuf_keep.push_back(keep);
          if ((int)shuf.size() >= opt_.shuffle_buffer) {
            size_t k = rng() % shuf.size();
            emit(shuf[k], shuf_keep[k]);
            shuf[k] = shuf.back();
            shuf_keep[k] = shuf_keep.back();
            shuf.pop_back();
            shuf_keep.pop_back();
          }
        } else {
          emit(r, keep);
        }
      };
      auto take = [&](const RecordRef& r, const std::shared_ptr<Chunk>& keep) {
        ++seen_;
        if ((ridx++ % opt_.shard_count) != opt_.shard_index) return;
        take_own(r, keep);
      };
      size_t fi = 0;
      for (const auto& path : opt_.files) {
        {
          std::lock_guard<std::mutex> g(mu_);
          if (stop_) return;
        }
        if (full() && opt_.shuffle_buffer <= 0 && !opt_.stream_mode) {
          // this epoch's agreed batches are out: the rest of the files is not read (their
          // indexes are still taken in order, one file ahead)
          Indexed skip = pending.get();
          if (fi + 1 < opt_.files.size() || epoch + 1 < opt_.num_epochs || opt_.num_epochs < 0)
            pending = std::async(std::launch::async, index, opt_.files[(fi + 1) % opt_.files.size()]);
          ++fi;
          continue;
        }
        if (opt_.stream_mode) {
          FILE* f = (path == "-") ? stdin : fopen(path.c_str(), "rb");
          if (!f) throw std::runtime_error("cannot open stream " + path);
          while (true) {
            auto c = std::make_shared<Chunk>();
            std::vector<RecordRef> recs;
            size_t bad = 0;
            bool any = read_stream_chunk(f, (size_t)8 << 20, opt_.verify_crc, opt_.skip_bad, c.get(), &recs, &bad);
            bad_ += bad;
            for (auto& r : recs) take(r, c);
            if (!any) break;
            std::lock_guard<std::mutex> g(mu_);
            if (stop_) break;
          }
          if (f != stdin) fclose(f);
        } else {
          Indexed ix = pending.get();  // this file's index (started one file ahead)
          if (fi + 1 < opt_.files.size() || epoch + 1 < opt_.num_epochs || opt_.num_epochs < 0)
            pending = std::async(std::launch::async, index, opt_.files[(fi + 1) % opt_.files.size()]);
          bad_ += ix.bad;
          if (index_mode) {
            // only this shard's records: j ≡ shard_index − ridx (mod shard_count)
            const int64_t P = opt_.shard_count, n = (int64_t)ix.ix.n;
            const int64_t j0 = ((opt_.shard_index - ridx) % P + P) % P;
            const uint8_t* base = ix.chunk->data;
            const uint64_t size = ix.chunk->size;
            for (int64_t j = j0; j < n && !full(); j += P) {
              const uint64_t o = ix.ix.off[j];
              if (o >= size) throw std::runtime_error("TFRecord index: offset beyond the end of " + path);
              take_own(RecordRef{base + o, (uint32_t)std::min<uint64_t>(size - o, UINT32_MAX)}, ix.chunk);
            }
            ridx += n;
            seen_ += (size_t)n;
          } else {
            for (auto& r : ix.recs) take(r, ix.chunk);
          }
        }
        ++fi;
      }
      // drain the shuffle buffer
      while (!shuf.empty()) {
        size_t k = rng() % shuf.size();
        emit(shuf[k], shuf_keep[k]);
        shuf[k] = shuf.back();
        shuf_keep[k] = shuf_keep.back();
        shuf.pop_back();
        shuf_keep.pop_back();
      }
      if (!cur.recs.empty() && !opt_.drop_remainder) {
        cur.seq = seq++;
        push_job(std::move(cur));
      } else if (!cur.recs.empty() && cur.framed && opt_.verify_crc) {
        // the dropped remainder is never decoded, but its records are still checked (tf.data
        // reads and checks every record before batch(drop_remainder) drops the tail)
        std::string err = resolve(&cur.recs, -1);
        if (!err.empty()) throw std::runtime_error(err);
      }
      if (opt_.stream_mode && opt_.num_epochs < 0) break;  // a pipe cannot be rewound
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      jobs_total_ = seq;
    }
    cv_.notify_all();
  } catch (const std::exception& e) {
    fail(e.what());
  }
}

std::string BatchLoader::resolve(std::vector<RecordRef>* recs, int64_t seq) const {
  const size_t n = recs->size();
  auto where = [seq](size_t r) {
    return (seq >= 0 ? " in batch " + std::to_string(seq) : std::string(" in the dropped remainder")) +
           " record " + std::to_string(r);
  };
  for (size_t r = 0; r < n; ++r) {
    RecordRef& x = (*recs)[r];
    const uint64_t left = x.len;  // bytes from the frame start to the end of the file
    if (left < 16) return "TFRecord: truncated record" + where(r);
    uint64_t len;
    memcpy(&len, x.data, 8);
    if (len > left - 16 || len > UINT32_MAX) return "TFRecord: truncated record" + where(r);
    // the length CRC is checked even with verify_crc off (8 bytes per record): a frame offset taken
    // from a sidecar index (record_index.h) is trusted only through (size, mtime, both ends), so a
    // file rewritten in place with the same size and a coarse mtime would otherwise decode garbage
    uint32_t lcrc;
    memcpy(&lcrc, x.data + 8, 4);
    if (mask_crc(crc32c(x.data, 8)) != lcrc)
      return std::string("TFRecord: corrupt length CRC") + (opt_.verify_crc ? "" : " (stale record index?)") + where(r);
    x.data += 12;
    x.len = (uint32_t)len;
  }
  if (opt_.verify_crc) {
    size_t r = 0;
    for (; r + 3 <= n; r += 3) {
      const uint8_t* p[3] = {(*recs)[r].data, (*recs)[r + 1].data, (*recs)[r + 2].data};
      const size_t l[3] = {(*recs)[r].len, (*recs)[r + 1].len, (*recs)[r + 2].len};
      uint32_t c[3];
      crc32c_x3(p, l, c);
      for (int k = 0; k < 3; ++k) {
        uint32_t d;
        memcpy(&d, p[k] + l[k], 4);
        if (mask_crc(c[k]) != d) return "TFRecord: corrupt data CRC" + where(r + k);
      }
    }
    for (; r < n; ++r) {
      uint32_t d;
      memcpy(&d, (*recs)[r].data + (*recs)[r].len, 4);
      if (mask_crc(crc32c((*recs)[r].data, (*recs)[r].len)) != d) return "TFRecord: corrupt data CRC" + where(r);
    }
  }
  return "";
}

void BatchLoader::worker_main() {
  const int F = opt_.schema.field_size;
  while (true) {
    Job job;
    int slot;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !jobs_.empty(); });
      if (stop_) return;
      job = std::move(jobs_.front());
      jobs_.pop_front();
      cv_.notify_all();
      slot = (int)(job.seq % opt_.num_slots);
      cv_.wait(lk, [&] { return stop_ || (slot_state_[slot] == 0 && slot_seq_[slot] == job.seq); });
      if (stop_) return;
      slot_state_[slot] = 1;
    }
    Slot& s = slots_[slot];
    int n = (int)job.recs.size();
    std::string err;
    if (job.framed) err = resolve(&job.recs, job.seq);
    if (err.empty() && opt_.raw) {
      // raw mode: payloads back to back + offsets; the device decoder parses them
      int64_t cursor = 0;
      for (int r = 0; r < n; ++r) {
        const RecordRef& x = job.recs[r];
        if (cursor + (int64_t)x.len > opt_.raw_cap) {
          err = "raw batch capacity exceeded in batch " + std::to_string(job.seq) + " (" +
                std::to_string(opt_.raw_cap) + " bytes; records up to " + std::to_string(x.len) +
                " bytes): use a larger raw_record_bytes or host decoding";
          break;
        }
        s.offs[r] = (int32_t)cursor;
        memcpy(s.bytes + cursor, x.data, x.len);
        cursor += x.len;
      }
      s.offs[n] = (int32_t)cursor;
    } else if (err.empty()) {
      for (int r = 0; r < n; ++r) {
        int st = decode_example(job.recs[r].data, job.recs[r].len, opt_.schema, s.labels + r,
                                s.ids + (size_t)r * F, s.vals + (size_t)r * F, opt_.max_id);
        if (st != kOk) {
          static const char* names[] = {"ok", "malformed Example protobuf", "missing feature",
                                        "wrong feature length (FixedLenFeature expects field_size values)",
                                        "id out of range [0, feature_size)"};
          err = std::string("decode error in batch ") + std::to_string(job.seq) + " record " + std::to_string(r) +
                ": " + names[st];
          break;
        }
      }
    }
    if (!err.empty()) {
      fail(err);
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      slot_rows_[slot] = n;
      slot_epoch_[slot] = job.epoch;
      slot_state_[slot] = 2;
    }
    cv_.notify_all();
  }
}

int BatchLoader::next(int* nrows, int* epoch) {
  std::unique_lock<std::mutex> lk(mu_);
  int slot = (int)(next_consume_ % opt_.num_slots);
  cv_.wait(lk, [&] {
    return !error_.empty() || (slot_state_[slot] == 2 && slot_seq_[slot] == next_consume_) ||
           (jobs_total_ >= 0 && next_consume_ >= jobs_total_) || (stop_ && error_.empty());
  });
  if (!error_.empty()) throw std::runtime_error(error_);
  if (slot_state_[slot] == 2 && slot_seq_[slot] == next_consume_) {
    *nrows = slot_rows_[slot];
    *epoch = slot_epoch_[slot];
    ++next_consume_;
    return slot;
  }
  return -1;
}

int BatchLoader::next_group(int max_n, int* n, int* last_rows, int* epoch) {
  std::unique_lock<std::mutex> lk(mu_);
  const int S = opt_.num_slots;
  const int first = (int)(next_consume_ % S);
  int want = 0;
  cv_.wait(lk, [&] {
    if (!error_.empty() || (stop_ && error_.empty())) return true;
    want = std::min(max_n, S - first);
    if (jobs_total_ >= 0) want = (int)std::min<int64_t>(want, std::max<int64_t>(0, jobs_total_ - next_consume_));
    for (int k = 0; k < want; ++k) {
      const int s = first + k;
      if (slot_state_[s] != 2 || slot_seq_[s] != next_consume_ + k) return false;
    }
    return want == 0 ? jobs_total_ >= 0 : true;
  });
  if (!error_.empty()) throw std::runtime_error(error_);
  if (stop_ || want == 0) {
    *n = 0;
    return -1;
  }
  *n = want;
  *last_rows = slot_rows_[first + want - 1];
  *epoch = slot_epoch_[first + want - 1];
  next_consume_ += want;
  return first;
}

void BatchLoader::release_group(int first, int n) {
  {
    std::lock_guard<std::mutex> g(mu_);
    for (int k = 0; k < n; ++k) {
      const int slot = first + k;
      if (slot < 0 || slot >= opt_.num_slots || slot_state_[slot] != 2) continue;
      slot_state_[slot] = 0;
      slot_seq_[slot] += opt_.num_slots;
    }
  }
  cv_.notify_all();
}

void BatchLoader::release(int slot) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (slot < 0 || slot >= opt_.num_slots || slot_state_[slot] != 2) return;
    slot_state_[slot] = 0;
    slot_seq_[slot] += opt_.num_slots;
  }
  cv_.notify_all();
}

size_t decode_file(const std::string& path, const Schema& s, int64_t max_id, bool verify_crc, bool skip_bad,
                   std::vector<float>* labels, std::vector<int32_t>* ids, std::vector<float>* vals) {
  auto c = map_file(path);
  std::vector<RecordRef> recs;
  size_t bad = 0;
  scan_records(c->data, c->size, verify_crc, skip_bad, &recs, &bad);
  const int F = s.field_size;
  labels->resize(recs.size());
  ids->resize(recs.size() * (size_t)F);
  vals->resize(recs.size() * (size_t)F);
  size_t out = 0;
  for (size_t r = 0; r < recs.size(); ++r) {
    int st = decode_example(recs[r].data, recs[r].len, s, labels->data() + out, ids->data() + out * F,
                            vals->data() + out * F, max_id);
    if (st != kOk) {
      if (skip_bad) continue;
      throw std::runtime_error("decode error in " + path + " record " + std::to_string(r) + " (status " +
                               std::to_string(st) + ")");
    }
    ++out;
  }
  labels->resize(out);
  ids->resize(out * (size_t)F);
  vals->resize(out * (size_t)F);
  return out;
}

// ------------------------------------------------------------------------------------------------
// libsvm → TFRecord
// ------------------------------------------------------------------------------------------------
namespace {
bool parse_libsvm_line(const char* p, const char* end, float* label, std::vector<int64_t>* ids,
                       std::vector<float>* vals) {
  ids->clear();
  vals->clear();
  while (p < end && (*p == ' ' || *p == '\t')) ++p;
  if (p >= end) return false;
  char* q;
  *label = strtof(p, &q);
  if (q == p) return false;
  p = q;
  while (p < end) {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\r')) ++p;
    if (p >= end) break;
    long long id = strtoll(p, &q, 10);
    if (q == p || q >= end || *q != ':') return false;
    p = q + 1;
    float v = strtof(p, &q);
    if (q == p) return false;
    p = q;
    ids->push_back(id);
    vals->push_back(v);
  }
  return true;
}
}  // namespace

size_t convert_libsvm(const std::string& in_path, const std::vector<std::string>& out_paths, const Schema& s,
                      int num_threads) {
  if (out_paths.empty()) throw std::invalid_argument("convert_libsvm: no output path");
  auto c = map_file(in_path);
  const char* base = reinterpret_cast<const char*>(c->data);
  size_t n = c->size;
  if (num_threads < 1) num_threads = 1;
  // split on line boundaries
  std::vector<size_t> cuts{0};
  for (int t = 1; t < num_threads; ++t) {
    size_t pos = n * t / num_threads;
    while (pos < n && base[pos] != '\n') ++pos;
    if (pos < n) ++pos;
    if (pos > cuts.back()) cuts.push_back(pos);
  }
  cuts.push_back(n);
  int parts = (int)cuts.size() - 1;
  std::vector<std::string> outs(parts);
  std::vector<std::vector<size_t>> ends(parts);  // end offset of every framed record in outs[t]
  std::vector<std::string> errs(parts);
  std::vector<std::thread> th;
  for (int t = 0; t < parts; ++t) {
    th.emplace_back([&, t] {
      std::vector<int64_t> ids;
      std::vector<float> vals;
      std::string ex;
      const char* p = base + cuts[t];
      const char* end = base + cuts[t + 1];
      while (p < end) {
        const char* nl = (const char*)memchr(p, '\n', end - p);
        const char* le = nl ? nl : end;
        float label;
        if (parse_libsvm_line(p, le, &label, &ids, &vals)) {
          ex.clear();
          encode_example(s, label, ids.data(), vals.data(), (int)ids.size(), &ex);
          frame_record(reinterpret_cast<const uint8_t*>(ex.data()), ex.size(), &outs[t]);
          ends[t].push_back(outs[t].size());
        } else {
          const char* q = p;
          while (q < le && (*q == ' ' || *q == '\t' || *q == '\r')) ++q;
          if (q < le && errs[t].empty()) errs[t] = std::string("cannot parse libsvm line: ") + std::string(p, le);
        }
        p = le + 1;
      }
    });
  }
  for (auto& x : th) x.join();
  for (auto& e : errs)
    if (!e.empty()) throw std::runtime_error(e);
  size_t total = 0;
  for (int t = 0; t < parts; ++t) total += ends[t].size();
  // shard k holds the contiguous records [k·N/S, (k+1)·N/S) in input order
  const size_t S = out_paths.size();
  int t = 0;
  size_t r_in_t = 0;  // next record of part t
  for (size_t k = 0; k < S; ++k) {
    const size_t hi = total * (k + 1) / S, lo = total * k / S;
    FILE* f = fopen(out_paths[k].c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + out_paths[k]);
    size_t left = hi - lo;
    while (left > 0) {
      while (r_in_t >= ends[t].size()) {
        ++t;
        r_in_t = 0;
      }
      const size_t take = std::min(left, ends[t].size() - r_in_t);
      const size_t b0 = r_in_t ? ends[t][r_in_t - 1] : 0, b1 = ends[t][r_in_t + take - 1];
      if (fwrite(outs[t].data() + b0, 1, b1 - b0, f) != b1 - b0) {
        fclose(f);
        throw std::runtime_error("short write to " + out_paths[k]);
      }
      r_in_t += take;
      left -= take;
    }
    fclose(f);
  }
  return total;
}

}  // namespace io
}  // namespace rocfm
