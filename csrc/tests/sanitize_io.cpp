// Host-sanitizer harness for the C++ IO runtime (race detection / sanitizers).
//
// Not part of the Python module (build.py compiles csrc/io only): tests/test_io_sanitizers.py compiles it with
// tfrecord.cpp and loader.cpp under -fsanitize=address,undefined and -fsanitize=thread and runs it.
// It exercises every entry point on valid data (round trips checked value by value) and on
// corrupted data (truncations, bit flips, forged lengths): the runtime must reject or skip bad input
// with an exception or a status — never read out of bounds, overflow, or race.
//
//   ./harness <tmpdir> [fuzz_iters]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <fstream>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include <fcntl.h>
#include <sys/stat.h>
#include "../io/loader.h"
#include "../io/record_index.h"
#include "../io/tfrecord.h"

using namespace rocfm::io;

namespace {

int g_fail = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                    \
    }                                                              \
  } while (0)

constexpr int kF = 39;

std::string make_records(int n, std::mt19937& rng, std::vector<int64_t>* all_ids, std::vector<float>* labels) {
  Schema s;
  s.field_size = kF;
  std::string out;
  std::uniform_int_distribution<int64_t> id(0, 99999);
  std::uniform_real_distribution<float> v(0.f, 1.f);
  for (int r = 0; r < n; ++r) {
    int64_t ids[kF];
    float vals[kF];
    for (int f = 0; f < kF; ++f) {
      ids[f] = id(rng);
      vals[f] = v(rng);
      all_ids->push_back(ids[f]);
    }
    const float lab = (float)(r & 1);
    labels->push_back(lab);
    std::string ex;
    encode_example(s, lab, ids, vals, kF, &ex);
    frame_record(reinterpret_cast<const uint8_t*>(ex.data()), ex.size(), &out);
  }
  return out;
}

void write_file(const std::string& path, const std::string& bytes) {
  std::ofstream f(path, std::ios::binary);
  f.write(bytes.data(), (std::streamsize)bytes.size());
}

// Every record of a (possibly corrupted) buffer through the framing walk and the decoder.
void walk_and_decode(const std::string& buf, bool verify, bool skip_bad) {
  Schema s;
  s.field_size = kF;
  std::vector<RecordRef> recs;
  size_t bad = 0;
  try {
    scan_records(reinterpret_cast<const uint8_t*>(buf.data()), buf.size(), verify, skip_bad, &recs, &bad);
  } catch (const std::exception&) {
    return;  // rejected: fine
  }
  float label;
  int32_t ids[kF];
  float vals[kF];
  for (const RecordRef& r : recs) {
    CHECK(r.data >= reinterpret_cast<const uint8_t*>(buf.data()));
    CHECK(r.data + r.len <= reinterpret_cast<const uint8_t*>(buf.data()) + buf.size());
    (void)decode_example(r.data, r.len, s, &label, ids, vals, 100000);
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <tmpdir> [fuzz_iters]\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const int iters = argc > 2 ? atoi(argv[2]) : 300;
  std::mt19937 rng(12345);
  std::vector<int64_t> all_ids;
  std::vector<float> labels;
  const int n = 1000;
  const std::string buf = make_records(n, rng, &all_ids, &labels);
  const std::string path = dir + "/h.tfrecords";
  write_file(path, buf);

  // 1. whole-file decode, value by value
  {
    Schema s;
    s.field_size = kF;
    std::vector<float> lab, vals;
    std::vector<int32_t> ids;
    const size_t got = decode_file(path, s, 100000, true, false, &lab, &ids, &vals);
    CHECK(got == (size_t)n);
    for (int i = 0; i < n * kF && i < (int)ids.size(); ++i) CHECK(ids[i] == (int32_t)all_ids[i]);
    for (int r = 0; r < n && r < (int)lab.size(); ++r) CHECK(lab[r] == labels[r]);
  }

  // 2. the threaded batch loader (2 files, shards, several epochs, worker pool): every row once
  {
    write_file(dir + "/h2.tfrecords", buf);
    for (int shard = 0; shard < 2; ++shard) {
      LoaderOptions o;
      o.files = {path, dir + "/h2.tfrecords"};
      o.schema.field_size = kF;
      o.max_id = 100000;
      o.batch_size = 64;
      o.num_epochs = 2;
      o.shard_count = 2;
      o.shard_index = shard;
      o.num_threads = 4;
      o.num_slots = 6;
      BatchLoader L(o);
      std::vector<std::vector<int32_t>> sid(o.num_slots, std::vector<int32_t>(64 * kF));
      std::vector<std::vector<float>> sv(o.num_slots, std::vector<float>(64 * kF)), sl(o.num_slots, std::vector<float>(64));
      for (int i = 0; i < o.num_slots; ++i) L.set_slot(i, sid[i].data(), sv[i].data(), sl[i].data());
      L.start();
      long rows = 0;
      int nrows = 0, epoch = 0, slot;
      while ((slot = L.next(&nrows, &epoch)) >= 0) {
        for (int j = 0; j < nrows * kF; ++j) CHECK(sid[slot][j] >= 0 && sid[slot][j] < 100000);
        rows += nrows;
        L.release(slot);
      }
      L.stop();
      CHECK(rows == 2L * (n / 64) * 64);  // 2 epochs × (2 files × n / 2 shards), whole batches
    }
  }

  // 2b. raw mode (payload bytes + offsets) through the saved record index, every row once; the
  //     payloads decode to the same ids as the host path
  {
    for (int shard = 0; shard < 2; ++shard) {
      LoaderOptions o;
      o.files = {path, dir + "/h2.tfrecords"};
      o.schema.field_size = kF;
      o.batch_size = 64;
      o.num_epochs = 2;
      o.shard_count = 2;
      o.shard_index = shard;
      o.num_threads = 3;
      o.num_slots = 6;
      o.raw = true;
      o.raw_cap = 64 * 512;
      o.max_batches_per_epoch = 5;
      BatchLoader L(o);
      std::vector<std::vector<uint8_t>> sb(o.num_slots, std::vector<uint8_t>(o.raw_cap));
      std::vector<std::vector<int32_t>> so(o.num_slots, std::vector<int32_t>(65));
      for (int i = 0; i < o.num_slots; ++i) L.set_raw_slot(i, sb[i].data(), so[i].data());
      L.start();
      long rows = 0;
      int nrows = 0, epoch = 0, slot;
      Schema s;
      s.field_size = kF;
      while ((slot = L.next(&nrows, &epoch)) >= 0) {
        for (int r = 0; r < nrows; ++r) {
          CHECK(so[slot][r] <= so[slot][r + 1] && so[slot][r + 1] <= o.raw_cap);
          float lab;
          int32_t ids[kF];
          float vals[kF];
          CHECK(decode_example(sb[slot].data() + so[slot][r], so[slot][r + 1] - so[slot][r], s, &lab, ids, vals,
                               100000) == kOk);
        }
        rows += nrows;
        L.release(slot);
      }
      L.stop();
      CHECK(rows == 2L * 5 * 64);  // capped at 5 batches per epoch
    }
  }

  // 3. corrupted inputs: truncations, bit flips, forged lengths — rejected or skipped, never a
  //    wild read (ASan) or UB (UBSan)
  std::uniform_int_distribution<size_t> pos(0, buf.size() - 1);
  for (int it = 0; it < iters; ++it) {
    std::string b = buf;
    switch (it % 4) {
      case 0:
        b.resize(pos(rng));
        break;
      case 1:
        for (int k = 0; k < 8; ++k) b[pos(rng)] ^= (char)(1u << (rng() & 7));
        break;
      case 2: {  // forge a huge or wrapping record length at a frame boundary-ish offset
        const size_t p = pos(rng) & ~size_t(7);
        const uint64_t len = (it & 8) ? ~0ull - (rng() & 31) : (uint64_t)rng() << 20;
        if (p + 8 <= b.size()) memcpy(&b[p], &len, 8);
        break;
      }
      default:
        for (int k = 0; k < 64; ++k) b[pos(rng)] = (char)rng();
    }
    walk_and_decode(b, false, false);
    walk_and_decode(b, true, true);
    walk_and_decode(b, false, true);
    if (it % 25 == 0) {  // and through the loader's index mode, the index taken from the intact
      //                      file and forced to look current (same size and mtime): the workers'
      //                      frame checks must reject whatever the corruption did
      const std::string bad = dir + "/badix.tfrecords";
      write_file(bad, buf);
      build_index_file(bad, true);
      struct stat st0;
      stat(bad.c_str(), &st0);
      std::string c = b;
      c.resize(buf.size(), '\0');  // same size (truncations zero-filled)
      write_file(bad, c);
      struct timespec ts[2] = {st0.st_atim, st0.st_mtim};
      utimensat(AT_FDCWD, bad.c_str(), ts, 0);
      for (int raw = 0; raw < 2; ++raw) {
        LoaderOptions o;
        o.files = {bad};
        o.schema.field_size = kF;
        o.max_id = 100000;
        o.batch_size = 32;
        o.num_threads = 2;
        o.num_slots = 4;
        o.raw = raw;
        o.raw_cap = 32 * 1024;
        BatchLoader L(o);
        std::vector<std::vector<uint8_t>> sb(4, std::vector<uint8_t>(o.raw_cap));
        std::vector<std::vector<int32_t>> so(4, std::vector<int32_t>(33)), sid(4, std::vector<int32_t>(32 * kF));
        std::vector<std::vector<float>> sv(4, std::vector<float>(32 * kF)), sl(4, std::vector<float>(32));
        for (int i = 0; i < 4; ++i) {
          L.set_slot(i, sid[i].data(), sv[i].data(), sl[i].data());
          L.set_raw_slot(i, sb[i].data(), so[i].data());
        }
        try {
          L.start();
          int nrows = 0, epoch = 0, slot;
          while ((slot = L.next(&nrows, &epoch)) >= 0) L.release(slot);
        } catch (const std::exception&) {
        }
        L.stop();
      }
    }
    if (it % 50 == 0) {  // and through the file reader
      const std::string bad = dir + "/bad.tfrecords";
      write_file(bad, b);
      Schema s;
      s.field_size = kF;
      std::vector<float> lab, vals;
      std::vector<int32_t> ids;
      try {
        decode_file(bad, s, 100000, true, true, &lab, &ids, &vals);
      } catch (const std::exception&) {
      }
    }
  }

  // 4. libsvm → TFRecord conversion (threaded, sharded) and back
  {
    const std::string svm = dir + "/in.libsvm";
    std::ofstream f(svm);
    for (int r = 0; r < 300; ++r) {
      f << (r & 1);
      for (int k = 0; k < kF; ++k) f << ' ' << (r * kF + k) % 5000 << ':' << 0.5f;
      f << '\n';
    }
    f.close();
    Schema s;
    s.field_size = kF;
    const size_t w = convert_libsvm(svm, {dir + "/c0.tfrecords", dir + "/c1.tfrecords", dir + "/c2.tfrecords"}, s, 4);
    CHECK(w == 300);
    size_t back = 0;
    for (int i = 0; i < 3; ++i) {
      std::vector<float> lab, vals;
      std::vector<int32_t> ids;
      back += decode_file(dir + "/c" + std::to_string(i) + ".tfrecords", s, 5000, true, false, &lab, &ids, &vals);
    }
    CHECK(back == 300);
  }

  if (g_fail) {
    fprintf(stderr, "%d checks failed\n", g_fail);
    return 1;
  }
  printf("sanitize harness ok\n");
  return 0;
}
