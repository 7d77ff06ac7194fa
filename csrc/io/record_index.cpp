// rocfm host runtime: persistent TFRecord offset index (see record_index.h).
#include "record_index.h"

#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <stdexcept>

namespace rocfm {
namespace io {
namespace {

constexpr char kMagic[8] = {'R', 'F', 'I', 'D', 'X', 0, 'v', '1'};

bool stat_file(const std::string& path, uint64_t* size, int64_t* mtime_ns) {
  struct stat st;
  if (::stat(path.c_str(), &st) != 0) return false;
  *size = (uint64_t)st.st_size;
  *mtime_ns = (int64_t)st.st_mtim.tv_sec * 1000000000LL + st.st_mtim.tv_nsec;
  return true;
}

// 64-bit FNV-1a of the absolute path (sidecar names under $ROCFM_INDEX_DIR)
uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

struct Unmap {
  size_t n;
  void operator()(void* p) const {
    if (p && p != MAP_FAILED) munmap(p, n);
  }
};

}  // namespace

std::string index_path(const std::string& data_path) {
  const char* dir = getenv("ROCFM_INDEX_DIR");
  if (!dir || !*dir) return data_path + ".rfidx";
  char* abs = realpath(data_path.c_str(), nullptr);
  std::string a = abs ? std::string(abs) : data_path;
  free(abs);
  const size_t slash = a.find_last_of('/');
  const std::string base = slash == std::string::npos ? a : a.substr(slash + 1);
  char hex[17];
  snprintf(hex, sizeof(hex), "%016llx", (unsigned long long)fnv1a(a));
  return std::string(dir) + "/" + hex + "-" + base + ".rfidx";
}

bool load_index(const std::string& data_path, const uint8_t* buf, size_t size, RecordIndex* out) {
  uint64_t fsize;
  int64_t mtime;
  if (!stat_file(data_path, &fsize, &mtime) || fsize != size) return false;
  const std::string ip = index_path(data_path);
  int fd = ::open(ip.c_str(), O_RDONLY);
  if (fd < 0) return false;
  struct stat st;
  if (fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(IdxHeader)) {
    ::close(fd);
    return false;
  }
  const size_t isz = (size_t)st.st_size;
  void* m = mmap(nullptr, isz, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
  ::close(fd);
  if (m == MAP_FAILED) return false;
  std::shared_ptr<void> keep(m, Unmap{isz});
  IdxHeader h;
  memcpy(&h, m, sizeof(h));
  if (memcmp(h.magic, kMagic, 8) != 0 || h.file_size != fsize || h.mtime_ns != mtime ||
      isz != sizeof(IdxHeader) + 8 * h.n)
    return false;
  const uint64_t* off = reinterpret_cast<const uint64_t*>(static_cast<const uint8_t*>(m) + sizeof(IdxHeader));
  // the framing must agree at both ends: first frame at 0, the last frame ends exactly at EOF
  if (h.n == 0) {
    if (size != 0) return false;
  } else {
    if (off[0] != 0 || off[h.n - 1] + 16 > size) return false;
    uint64_t len;
    memcpy(&len, buf + off[h.n - 1], 8);
    if (len > size || off[h.n - 1] + 16 + len != size) return false;
  }
  out->off = off;
  out->n = (size_t)h.n;
  out->max_len = h.max_len;
  out->loaded = true;
  out->own.clear();
  out->map = std::move(keep);
  return true;
}

void index_from_refs(const uint8_t* buf, const std::vector<RecordRef>& refs, RecordIndex* out) {
  out->own.resize(refs.size());
  uint32_t mx = 0;
  for (size_t i = 0; i < refs.size(); ++i) {
    out->own[i] = (uint64_t)(refs[i].data - buf) - 12;
    mx = std::max(mx, refs[i].len);
  }
  out->off = out->own.data();
  out->n = refs.size();
  out->max_len = mx;
  out->loaded = false;
  out->map.reset();
}

bool save_index(const std::string& data_path, const RecordIndex& ix, bool crc_verified) {
  if (getenv("ROCFM_NO_INDEX_WRITE")) return false;
  IdxHeader h;
  memcpy(h.magic, kMagic, 8);
  if (!stat_file(data_path, &h.file_size, &h.mtime_ns)) return false;
  h.n = ix.n;
  h.max_len = ix.max_len;
  h.flags = crc_verified ? 1u : 0u;
  h.reserved = 0;
  const std::string ip = index_path(data_path);
  // unique temporary name: several ranks may build the same index at once; the renames are
  // atomic and their contents identical, so the last one simply wins
  char suffix[64];
  snprintf(suffix, sizeof(suffix), ".tmp.%d.%llx", (int)getpid(), (unsigned long long)(uintptr_t)&ix);
  const std::string tmp = ip + suffix;
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) return false;
  bool ok = fwrite(&h, sizeof(h), 1, f) == 1 && (ix.n == 0 || fwrite(ix.off, 8, ix.n, f) == ix.n);
  ok = (fclose(f) == 0) && ok;
  if (ok) ok = rename(tmp.c_str(), ip.c_str()) == 0;
  if (!ok) unlink(tmp.c_str());
  return ok;
}

size_t build_index_file(const std::string& data_path, bool verify_crc) {
  int fd = ::open(data_path.c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("cannot open " + data_path);
  struct stat st;
  if (fstat(fd, &st) != 0) {
    ::close(fd);
    throw std::runtime_error("cannot stat " + data_path);
  }
  const size_t n = (size_t)st.st_size;
  std::shared_ptr<void> keep;
  const uint8_t* buf = nullptr;
  if (n) {
    void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) {
      ::close(fd);
      throw std::runtime_error("mmap failed for " + data_path);
    }
    madvise(m, n, MADV_SEQUENTIAL);
    keep = std::shared_ptr<void>(m, Unmap{n});
    buf = static_cast<const uint8_t*>(m);
  }
  ::close(fd);
  std::vector<RecordRef> refs;
  size_t bad = 0;
  scan_records(buf, n, verify_crc, false, &refs, &bad);
  RecordIndex ix;
  index_from_refs(buf, refs, &ix);
  save_index(data_path, ix, verify_crc);
  return ix.n;
}

}  // namespace io
}  // namespace rocfm
