// rocfm host runtime: TFRecord framing + CRC32C + fixed-schema Example codec (see tfrecord.h).
#include "tfrecord.h"

#include <nmmintrin.h>
#include <string.h>

#include <algorithm>
#include <stdexcept>

namespace rocfm {
namespace io {

// ---------------------------------------------------------------------------------------------
// CRC32C (Castagnoli).  SSE4.2 crc32 instruction, 8 bytes per step, three independent streams
// interleaved for large buffers is not needed here (records are ~300 B).
// ---------------------------------------------------------------------------------------------
uint32_t crc32c(const uint8_t* p, size_t n, uint32_t crc) {
  uint64_t c = ~crc;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    c = _mm_crc32_u8((uint32_t)c, *p++);
    --n;
  }
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  while (n--) c = _mm_crc32_u8((uint32_t)c, *p++);
  return ~(uint32_t)c;
}

// Three independent CRC32C streams interleaved: the crc32 instruction has a 3-cycle latency and a
// 1-cycle issue rate, so three records checked together cost about as much as one alone.
void crc32c_x3(const uint8_t* const p[3], const size_t n[3], uint32_t out[3]) {
  uint64_t c0 = 0xffffffffu, c1 = 0xffffffffu, c2 = 0xffffffffu;
  const size_t m = std::min(n[0], std::min(n[1], n[2])) & ~(size_t)7;
  const uint8_t *a = p[0], *b = p[1], *c = p[2];
  for (size_t i = 0; i < m; i += 8) {
    uint64_t va, vb, vc;
    memcpy(&va, a + i, 8);
    memcpy(&vb, b + i, 8);
    memcpy(&vc, c + i, 8);
    c0 = _mm_crc32_u64(c0, va);
    c1 = _mm_crc32_u64(c1, vb);
    c2 = _mm_crc32_u64(c2, vc);
  }
  // tails continue from the raw states (crc32c() complements its argument on entry)
  out[0] = crc32c(a + m, n[0] - m, ~(uint32_t)c0);
  out[1] = crc32c(b + m, n[1] - m, ~(uint32_t)c1);
  out[2] = crc32c(c + m, n[2] - m, ~(uint32_t)c2);
}

// ---------------------------------------------------------------------------------------------
// protobuf wire-format helpers
// ---------------------------------------------------------------------------------------------
namespace {

inline bool read_varint(const uint8_t*& p, const uint8_t* end, uint64_t* out) {
  uint64_t v = 0;
  int shift = 0;
  while (p < end && shift < 64) {
    uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) {
      *out = v;
      return true;
    }
    shift += 7;
  }
  return false;
}

inline bool skip_field(const uint8_t*& p, const uint8_t* end, uint32_t wire) {
  uint64_t v;
  switch (wire) {
    case 0:
      return read_varint(p, end, &v);
    case 1:
      if (end - p < 8) return false;
      p += 8;
      return true;
    case 2:
      if (!read_varint(p, end, &v) || (uint64_t)(end - p) < v) return false;
      p += v;
      return true;
    case 5:
      if (end - p < 4) return false;
      p += 4;
      return true;
    default:
      return false;
  }
}

enum Which { kNone = 0, kLabel, kIds, kVals };

// Parse a FloatList message body into dst (capacity cap); returns count or -1.
inline int parse_float_list(const uint8_t* p, const uint8_t* end, float* dst, int cap) {
  int cnt = 0;
  while (p < end) {
    uint64_t tag;
    if (!read_varint(p, end, &tag)) return -1;
    uint32_t fno = (uint32_t)(tag >> 3), wire = (uint32_t)(tag & 7);
    if (fno == 1 && wire == 2) {  // packed
      uint64_t len;
      if (!read_varint(p, end, &len) || (uint64_t)(end - p) < len || (len & 3)) return -1;
      int k = (int)(len / 4);
      if (cnt + k <= cap) memcpy(dst + cnt, p, len);
      cnt += k;
      p += len;
    } else if (fno == 1 && wire == 5) {
      if (end - p < 4) return -1;
      if (cnt < cap) memcpy(dst + cnt, p, 4);
      ++cnt;
      p += 4;
    } else if (!skip_field(p, end, wire)) {
      return -1;
    }
  }
  return cnt;
}

inline int parse_int64_list(const uint8_t* p, const uint8_t* end, int32_t* dst, int cap, int64_t max_id,
                            bool* oob) {
  int cnt = 0;
  while (p < end) {
    uint64_t tag;
    if (!read_varint(p, end, &tag)) return -1;
    uint32_t fno = (uint32_t)(tag >> 3), wire = (uint32_t)(tag & 7);
    if (fno == 1 && wire == 2) {
      uint64_t len;
      if (!read_varint(p, end, &len) || (uint64_t)(end - p) < len) return -1;
      const uint8_t* e2 = p + len;
      // ids < 2^21 (any realistic vocabulary) are 1-3 byte varints: decoded without the loop;
      // negative int64 ids read as huge unsigned values and fail the single range compare
      const uint64_t lim = (max_id > 0 && max_id < 0x80000000LL) ? (uint64_t)max_id : 0x80000000ull;
      bool bad = false;
      while (p < e2) {
        uint64_t v;
        const uint32_t b0 = p[0];
        if (b0 < 0x80) {
          v = b0;
          p += 1;
        } else if (e2 - p >= 2 && p[1] < 0x80) {
          v = (b0 & 0x7f) | ((uint64_t)p[1] << 7);
          p += 2;
        } else if (e2 - p >= 3 && p[1] >= 0x80 && p[2] < 0x80) {
          v = (b0 & 0x7f) | ((uint64_t)(p[1] & 0x7f) << 7) | ((uint64_t)p[2] << 14);
          p += 3;
        } else if (!read_varint(p, e2, &v)) {
          return -1;
        }
        bad |= v >= lim;
        if (cnt < cap) dst[cnt] = (int32_t)v;
        ++cnt;
      }
      if (bad) *oob = true;
    } else if (fno == 1 && wire == 0) {
      uint64_t v;
      if (!read_varint(p, end, &v)) return -1;
      int64_t sv = (int64_t)v;
      if (sv < 0 || (max_id > 0 && sv >= max_id) || sv > 0x7fffffffLL) *oob = true;
      if (cnt < cap) dst[cnt] = (int32_t)sv;
      ++cnt;
    } else if (!skip_field(p, end, wire)) {
      return -1;
    }
  }
  return cnt;
}

inline bool key_eq(const uint8_t* k, uint64_t kl, const std::string& s) {
  return kl == s.size() && memcmp(k, s.data(), kl) == 0;
}

}  // namespace

int decode_example(const uint8_t* p, size_t n, const Schema& s, float* label, int32_t* ids, float* vals,
                   int64_t max_id) {
  const uint8_t* end = p + n;
  int nl = -1, ni = -1, nv = -1;
  bool oob = false;
  const int F = s.field_size;
  while (p < end) {  // Example
    uint64_t tag;
    if (!read_varint(p, end, &tag)) return kBadProto;
    if ((tag >> 3) != 1 || (tag & 7) != 2) {
      if (!skip_field(p, end, (uint32_t)(tag & 7))) return kBadProto;
      continue;
    }
    uint64_t flen;
    if (!read_varint(p, end, &flen) || (uint64_t)(end - p) < flen) return kBadProto;
    const uint8_t* fend = p + flen;
    while (p < fend) {  // Features: repeated map entries (field 1)
      uint64_t t2;
      if (!read_varint(p, fend, &t2)) return kBadProto;
      if ((t2 >> 3) != 1 || (t2 & 7) != 2) {
        if (!skip_field(p, fend, (uint32_t)(t2 & 7))) return kBadProto;
        continue;
      }
      uint64_t elen;
      if (!read_varint(p, fend, &elen) || (uint64_t)(fend - p) < elen) return kBadProto;
      const uint8_t* eend = p + elen;
      const uint8_t* key = nullptr;
      uint64_t klen = 0;
      const uint8_t* val = nullptr;
      uint64_t vlen = 0;
      while (p < eend) {  // map entry {1: key, 2: Feature}
        uint64_t t3;
        if (!read_varint(p, eend, &t3)) return kBadProto;
        uint32_t fno = (uint32_t)(t3 >> 3), wire = (uint32_t)(t3 & 7);
        if ((fno == 1 || fno == 2) && wire == 2) {
          uint64_t l;
          if (!read_varint(p, eend, &l) || (uint64_t)(eend - p) < l) return kBadProto;
          if (fno == 1) {
            key = p;
            klen = l;
          } else {
            val = p;
            vlen = l;
          }
          p += l;
        } else if (!skip_field(p, eend, wire)) {
          return kBadProto;
        }
      }
      p = eend;
      if (!key || !val) continue;
      Which w = key_eq(key, klen, s.label_key) ? kLabel
                : key_eq(key, klen, s.ids_key) ? kIds
                : key_eq(key, klen, s.vals_key) ? kVals
                                                : kNone;
      if (w == kNone) continue;
      // Feature { 1: bytes_list, 2: float_list, 3: int64_list }
      const uint8_t* q = val;
      const uint8_t* qend = val + vlen;
      while (q < qend) {
        uint64_t t4;
        if (!read_varint(q, qend, &t4)) return kBadProto;
        uint32_t fno = (uint32_t)(t4 >> 3), wire = (uint32_t)(t4 & 7);
        if (wire != 2) {
          if (!skip_field(q, qend, wire)) return kBadProto;
          continue;
        }
        uint64_t l;
        if (!read_varint(q, qend, &l) || (uint64_t)(qend - q) < l) return kBadProto;
        if (w == kLabel && fno == 2) {
          float tmp[1];
          int c = parse_float_list(q, q + l, tmp, 1);
          if (c < 0) return kBadProto;
          if (c >= 1) *label = tmp[0];
          nl = c;
        } else if (w == kVals && fno == 2) {
          nv = parse_float_list(q, q + l, vals, F);
          if (nv < 0) return kBadProto;
        } else if (w == kIds && fno == 3) {
          ni = parse_int64_list(q, q + l, ids, F, max_id, &oob);
          if (ni < 0) return kBadProto;
        } else if (w == kLabel && fno == 3) {  // tolerate int64 labels
          int32_t tmp[1];
          bool o2 = false;
          int c = parse_int64_list(q, q + l, tmp, 1, 0, &o2);
          if (c < 0) return kBadProto;
          if (c >= 1) *label = (float)tmp[0];
          nl = c;
        }
        q += l;
      }
    }
    p = fend;
  }
  if (nl < 0 || ni < 0 || nv < 0) return kMissingFeature;
  if (nl != 1 || ni != F || nv != F) return kWrongLength;
  if (oob) return kIdOutOfRange;
  return kOk;
}

// ---------------------------------------------------------------------------------------------
// encoder
// ---------------------------------------------------------------------------------------------
namespace {
inline void put_varint(std::string* o, uint64_t v) {
  while (v >= 0x80) {
    o->push_back((char)(v | 0x80));
    v >>= 7;
  }
  o->push_back((char)v);
}
inline size_t varint_size(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}
inline void put_len(std::string* o, uint32_t fno, const std::string& body) {
  put_varint(o, (fno << 3) | 2);
  put_varint(o, body.size());
  o->append(body);
}
std::string feature_entry(const std::string& key, const std::string& feature) {
  std::string e;
  put_len(&e, 1, key);
  put_len(&e, 2, feature);
  return e;
}
}  // namespace

void encode_example(const Schema& s, float label, const int64_t* ids, const float* vals, int n,
                    std::string* out) {
  // label: Feature{float_list{value: [label]}}
  std::string fl, lab, idsf, il, valf, vl, features, ex;
  {
    std::string packed(reinterpret_cast<const char*>(&label), 4);
    put_len(&fl, 1, packed);
    put_len(&lab, 2, fl);
  }
  {
    std::string packed;
    for (int i = 0; i < n; ++i) put_varint(&packed, (uint64_t)ids[i]);
    put_len(&il, 1, packed);
    put_len(&idsf, 3, il);
  }
  {
    std::string packed(reinterpret_cast<const char*>(vals), 4 * (size_t)n);
    put_len(&vl, 1, packed);
    put_len(&valf, 2, vl);
  }
  // map entries are written in key order like protobuf's deterministic map serialisation
  put_len(&features, 1, feature_entry(s.ids_key, idsf));
  put_len(&features, 1, feature_entry(s.label_key, lab));
  put_len(&features, 1, feature_entry(s.vals_key, valf));
  put_len(&ex, 1, features);
  out->append(ex);
}

void frame_record(const uint8_t* payload, size_t n, std::string* out) {
  uint64_t len = n;
  uint8_t hdr[12];
  memcpy(hdr, &len, 8);
  uint32_t c1 = mask_crc(crc32c(hdr, 8));
  memcpy(hdr + 8, &c1, 4);
  out->append(reinterpret_cast<char*>(hdr), 12);
  out->append(reinterpret_cast<const char*>(payload), n);
  uint32_t c2 = mask_crc(crc32c(payload, n));
  out->append(reinterpret_cast<char*>(&c2), 4);
}

size_t scan_records(const uint8_t* buf, size_t n, bool verify_crc, bool skip_bad, std::vector<RecordRef>* out,
                    size_t* bad_records, bool verify_data) {
  size_t off = 0, cnt = 0;
  while (off + 12 <= n) {
    uint64_t len;
    memcpy(&len, buf + off, 8);
    uint32_t lcrc;
    memcpy(&lcrc, buf + off + 8, 4);
    if (verify_crc && mask_crc(crc32c(buf + off, 8)) != lcrc) {
      if (skip_bad) {
        ++*bad_records;
        break;  // framing is unrecoverable after a corrupt length
      }
      throw std::runtime_error("TFRecord: corrupt length CRC at offset " + std::to_string(off));
    }
    // no wraparound: a corrupt or hostile 64-bit length must not pass the bounds check
    // (RecordRef stores 32-bit lengths, so anything wider is rejected as well)
    if (len > n - off - 12 || n - off - 12 - len < 4 || len > UINT32_MAX) {
      if (skip_bad) {
        ++*bad_records;
        break;
      }
      throw std::runtime_error("TFRecord: truncated record at offset " + std::to_string(off));
    }
    const uint8_t* payload = buf + off + 12;
    bool ok = true;
    if (verify_crc && verify_data) {
      uint32_t dcrc;
      memcpy(&dcrc, payload + len, 4);
      ok = mask_crc(crc32c(payload, len)) == dcrc;
      if (!ok && !skip_bad) throw std::runtime_error("TFRecord: corrupt data CRC at offset " + std::to_string(off));
    }
    if (ok) {
      out->push_back(RecordRef{payload, (uint32_t)len});
      ++cnt;
    } else {
      ++*bad_records;
    }
    off += 12 + len + 4;
  }
  if (off != n && !skip_bad && off + 12 > n && off < n)
    throw std::runtime_error("TFRecord: trailing garbage at offset " + std::to_string(off));
  return cnt;
}

}  // namespace io
}  // namespace rocfm
