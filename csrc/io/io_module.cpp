// pybind11 bindings for the host runtime (module rocfm._rocfm_io).  Host-only: builds and runs on
// CPU-only machines (tests) and feeds pinned buffers on the GPU box.
#include <pybind11/numpy.h>
#include <cstring>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "loader.h"
#include "record_index.h"
#include "tfrecord.h"

namespace py = pybind11;
using namespace rocfm::io;

static Schema make_schema(int field_size, const std::string& label_key, const std::string& ids_key,
                          const std::string& vals_key) {
  Schema s;
  s.field_size = field_size;
  s.label_key = label_key;
  s.ids_key = ids_key;
  s.vals_key = vals_key;
  return s;
}

PYBIND11_MODULE(_rocfm_io, m) {
  m.doc() = "rocfm host runtime: TFRecord/Example codec, CRC32C, batch loader, libsvm converter";

  m.def("crc32c", [](py::bytes b) {
    std::string s = b;
    return crc32c(reinterpret_cast<const uint8_t*>(s.data()), s.size());
  });
  m.def("masked_crc32c", [](py::bytes b) {
    std::string s = b;
    return mask_crc(crc32c(reinterpret_cast<const uint8_t*>(s.data()), s.size()));
  });

  m.def(
      "encode_example",
      [](float label, py::array_t<int64_t, py::array::c_style | py::array::forcecast> ids,
         py::array_t<float, py::array::c_style | py::array::forcecast> vals, const std::string& label_key,
         const std::string& ids_key, const std::string& vals_key) {
        if (ids.size() != vals.size()) throw std::invalid_argument("ids/vals length mismatch");
        Schema s = make_schema((int)ids.size(), label_key, ids_key, vals_key);
        std::string out;
        encode_example(s, label, ids.data(), vals.data(), (int)ids.size(), &out);
        return py::bytes(out);
      },
      py::arg("label"), py::arg("ids"), py::arg("vals"), py::arg("label_key") = "label", py::arg("ids_key") = "ids",
      py::arg("vals_key") = "values");

  m.def(
      "decode_example",
      [](py::bytes payload, int field_size, int64_t max_id, const std::string& label_key, const std::string& ids_key,
         const std::string& vals_key) {
        std::string p = payload;
        Schema s = make_schema(field_size, label_key, ids_key, vals_key);
        float label = 0;
        py::array_t<int32_t> ids(field_size);
        py::array_t<float> vals(field_size);
        int st = decode_example(reinterpret_cast<const uint8_t*>(p.data()), p.size(), s, &label,
                                ids.mutable_data(), vals.mutable_data(), max_id);
        return py::make_tuple(st, label, ids, vals);
      },
      py::arg("payload"), py::arg("field_size"), py::arg("max_id") = 0, py::arg("label_key") = "label",
      py::arg("ids_key") = "ids", py::arg("vals_key") = "values");

  // Write a whole batch of Examples as a TFRecord file (synthetic data generation, tests).
  m.def(
      "write_tfrecord",
      [](const std::string& path, py::array_t<float, py::array::c_style | py::array::forcecast> labels,
         py::array_t<int64_t, py::array::c_style | py::array::forcecast> ids,
         py::array_t<float, py::array::c_style | py::array::forcecast> vals, bool append) {
        if (ids.ndim() != 2 || vals.ndim() != 2 || ids.shape(0) != labels.size() || vals.shape(0) != labels.size() ||
            ids.shape(1) != vals.shape(1))
          throw std::invalid_argument("write_tfrecord: expects labels[N], ids[N,F], vals[N,F]");
        const int64_t N = labels.size();
        const int F = (int)ids.shape(1);
        Schema s = make_schema(F, "label", "ids", "values");
        std::string out, ex;
        out.reserve((size_t)N * (16 + 12 * F + 64));
        {
          py::gil_scoped_release nogil;
          for (int64_t i = 0; i < N; ++i) {
            ex.clear();
            encode_example(s, labels.data()[i], ids.data() + i * F, vals.data() + i * F, F, &ex);
            frame_record(reinterpret_cast<const uint8_t*>(ex.data()), ex.size(), &out);
          }
        }
        FILE* f = fopen(path.c_str(), append ? "ab" : "wb");
        if (!f) throw std::runtime_error("cannot open " + path);
        size_t w = fwrite(out.data(), 1, out.size(), f);
        fclose(f);
        if (w != out.size()) throw std::runtime_error("short write " + path);
        return N;
      },
      py::arg("path"), py::arg("labels"), py::arg("ids"), py::arg("vals"), py::arg("append") = false);

  m.def(
      "decode_file",
      [](const std::string& path, int field_size, int64_t max_id, bool verify_crc, bool skip_bad) {
        Schema s = make_schema(field_size, "label", "ids", "values");
        std::vector<float> labels, vals;
        std::vector<int32_t> ids;
        size_t n;
        {
          py::gil_scoped_release nogil;
          n = decode_file(path, s, max_id, verify_crc, skip_bad, &labels, &ids, &vals);
        }
        py::array_t<float> L((py::ssize_t)n);
        py::array_t<int32_t> I({(py::ssize_t)n, (py::ssize_t)field_size});
        py::array_t<float> V({(py::ssize_t)n, (py::ssize_t)field_size});
        std::copy(labels.begin(), labels.end(), L.mutable_data());
        std::copy(ids.begin(), ids.end(), I.mutable_data());
        std::copy(vals.begin(), vals.end(), V.mutable_data());
        return py::make_tuple(L, I, V);
      },
      py::arg("path"), py::arg("field_size"), py::arg("max_id") = 0, py::arg("verify_crc") = true,
      py::arg("skip_bad") = false);

  m.def(
      "scan_file",
      [](const std::string& path, bool verify_crc, bool skip_bad) {
        // returns (num_records, bad_records, list of payload lengths)
        FILE* f = fopen(path.c_str(), "rb");
        if (!f) throw std::runtime_error("cannot open " + path);
        std::string buf;
        char tmp[1 << 16];
        size_t g;
        while ((g = fread(tmp, 1, sizeof(tmp), f)) > 0) buf.append(tmp, g);
        fclose(f);
        std::vector<RecordRef> recs;
        size_t bad = 0;
        scan_records(reinterpret_cast<const uint8_t*>(buf.data()), buf.size(), verify_crc, skip_bad, &recs, &bad);
        std::vector<uint32_t> lens;
        for (auto& r : recs) lens.push_back(r.len);
        return py::make_tuple(recs.size(), bad, lens);
      },
      py::arg("path"), py::arg("verify_crc") = true, py::arg("skip_bad") = false);

  m.def(
      "count_records",
      [](const std::string& path) {
        // framing walk only (u64 length, u32 crc, payload, u32 crc) over a read-only mapping: no
        // payload read, no CRC check (a stdio seek per record costs a syscall each)
        py::gil_scoped_release nogil;
        int fd = ::open(path.c_str(), O_RDONLY);
        if (fd < 0) throw std::runtime_error("cannot open " + path);
        struct stat st;
        if (fstat(fd, &st) != 0) {
          ::close(fd);
          throw std::runtime_error("cannot stat " + path);
        }
        const size_t size = (size_t)st.st_size;
        int64_t n = 0;
        if (size >= 12) {
          void* m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
          if (m == MAP_FAILED) {
            ::close(fd);
            throw std::runtime_error("mmap failed for " + path);
          }
          const uint8_t* b = static_cast<const uint8_t*>(m);
          for (size_t off = 0; off + 12 <= size; ++n) {
            uint64_t len;
            std::memcpy(&len, b + off, 8);
            if (len > size - off - 12) break;
            off += 12 + len + 4;
          }
          munmap(m, size);
        }
        ::close(fd);
        return n;
      },
      py::arg("path"));

  m.def(
      "convert_libsvm",
      [](const std::string& in_path, const std::string& out_path, int num_threads) {
        Schema s = make_schema(0, "label", "ids", "values");
        py::gil_scoped_release nogil;
        return convert_libsvm(in_path, std::vector<std::string>{out_path}, s, num_threads);
      },
      py::arg("in_path"), py::arg("out_path"), py::arg("num_threads") = 4);
  m.def(
      "convert_libsvm_sharded",
      [](const std::string& in_path, const std::vector<std::string>& out_paths, int num_threads) {
        Schema s = make_schema(0, "label", "ids", "values");
        py::gil_scoped_release nogil;
        return convert_libsvm(in_path, out_paths, s, num_threads);
      },
      py::arg("in_path"), py::arg("out_paths"), py::arg("num_threads") = 4);

  py::class_<BatchLoader>(m, "BatchLoader")
      .def(py::init([](std::vector<std::string> files, int field_size, int64_t max_id, int batch_size,
                       bool drop_remainder, int num_epochs, int shard_count, int shard_index, int num_threads,
                       int num_slots, bool verify_crc, bool skip_bad, int shuffle_buffer, uint64_t seed,
                       bool stream_mode, int64_t skip_batches, bool use_index, bool raw, int64_t raw_cap,
                       int64_t max_batches_per_epoch) {
             LoaderOptions o;
             o.files = std::move(files);
             o.schema.field_size = field_size;
             o.max_id = max_id;
             o.batch_size = batch_size;
             o.drop_remainder = drop_remainder;
             o.num_epochs = num_epochs;
             o.shard_count = shard_count;
             o.shard_index = shard_index;
             o.num_threads = num_threads;
             o.num_slots = num_slots;
             o.verify_crc = verify_crc;
             o.skip_bad = skip_bad;
             o.shuffle_buffer = shuffle_buffer;
             o.seed = seed;
             o.stream_mode = stream_mode;
             o.skip_batches = skip_batches;
             o.use_index = use_index;
             o.raw = raw;
             o.raw_cap = raw_cap;
             o.max_batches_per_epoch = max_batches_per_epoch;
             return new BatchLoader(o);
           }),
           py::arg("files"), py::arg("field_size"), py::arg("max_id") = 0, py::arg("batch_size") = 1024,
           py::arg("drop_remainder") = true, py::arg("num_epochs") = 1, py::arg("shard_count") = 1,
           py::arg("shard_index") = 0, py::arg("num_threads") = 4, py::arg("num_slots") = 4,
           py::arg("verify_crc") = true, py::arg("skip_bad") = false, py::arg("shuffle_buffer") = 0,
           py::arg("seed") = 0, py::arg("stream_mode") = false, py::arg("skip_batches") = 0,
           py::arg("use_index") = true, py::arg("raw") = false, py::arg("raw_cap") = 0,
           py::arg("max_batches_per_epoch") = 0)
      .def("set_slot",
           [](BatchLoader& L, int i, uintptr_t ids, uintptr_t vals, uintptr_t labels) {
             L.set_slot(i, reinterpret_cast<int32_t*>(ids), reinterpret_cast<float*>(vals),
                        reinterpret_cast<float*>(labels));
           })
      .def("set_raw_slot",
           [](BatchLoader& L, int i, uintptr_t bytes, uintptr_t offs) {
             L.set_raw_slot(i, reinterpret_cast<uint8_t*>(bytes), reinterpret_cast<int32_t*>(offs));
           })
      .def("start", &BatchLoader::start)
      .def("next",
           [](BatchLoader& L) {
             int rows = 0, epoch = 0, slot;
             {
               py::gil_scoped_release nogil;
               slot = L.next(&rows, &epoch);
             }
             return py::make_tuple(slot, rows, epoch);
           })
      .def("release", &BatchLoader::release)
      .def("next_group",
           [](BatchLoader& L, int max_n) {
             int n = 0, rows = 0, epoch = 0, first;
             {
               py::gil_scoped_release nogil;
               first = L.next_group(max_n, &n, &rows, &epoch);
             }
             return py::make_tuple(first, n, rows, epoch);
           })
      .def("release_group", &BatchLoader::release_group)
      .def("stop", &BatchLoader::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("bad_records", &BatchLoader::bad_records)
      .def_property_readonly("records_seen", &BatchLoader::records_seen)
      .def_property_readonly("index_fallbacks", &BatchLoader::index_fallbacks)
      .def_property_readonly("index_loads", &BatchLoader::index_loads)
      .def_property_readonly("index_builds", &BatchLoader::index_builds);

  // persistent record index (record_index.h)
  m.def(
      "build_index",
      [](const std::string& path, bool verify_crc) {
        py::gil_scoped_release nogil;
        return build_index_file(path, verify_crc);
      },
      py::arg("path"), py::arg("verify_crc") = true);
  m.def("index_path", &index_path, py::arg("path"));
  m.def(
      "index_info",
      [](const std::string& path) -> py::object {
        // (records, max payload bytes) from a valid saved index, or None
        int fd = ::open(path.c_str(), O_RDONLY);
        if (fd < 0) return py::none();
        struct stat st;
        if (fstat(fd, &st) != 0) {
          ::close(fd);
          return py::none();
        }
        const size_t size = (size_t)st.st_size;
        void* m = size ? mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0) : nullptr;
        ::close(fd);
        if (size && m == MAP_FAILED) return py::none();
        RecordIndex ix;
        const bool ok = load_index(path, static_cast<const uint8_t*>(m), size, &ix);
        py::object out = ok ? py::object(py::make_tuple(ix.n, ix.max_len)) : py::object(py::none());
        ix = RecordIndex();
        if (m) munmap(m, size);
        return out;
      },
      py::arg("path"));
}
