// Host-side native runtime core (no Python): CRC-32C, TFRecord framing,
// minimal tf.Example decoding, leveldb-format SSTable (tensor-bundle .index).
// Shared by the `_host` pybind module (runtime.cpp) and the sanitizer self-test
// (tests/native/runtime_selftest.cpp, built with -fsanitize=address,undefined).
//
// Replaces the TF 1.x C++ runtime pieces the reference leans on:
//   N15  TFRecordReader + ParseSingleExample   -> split_records / decode_example
//   N20  tensor-bundle Saver (.index SSTable)  -> sstable_build / sstable_parse
//   N21  events.out.tfevents framing           -> frame
// Formats are byte-compatible with TensorFlow:
//   * TFRecord: u64 length | u32 masked_crc(length) | data | u32 masked_crc(data)
//   * SSTable (leveldb table format as used by tensorflow/core/lib/io/table):
//     prefix-compressed data blocks (restart interval 16), no compression, block
//     trailer = type byte + masked crc32c, metaindex + index blocks, 48-byte footer
//     with magic 0xdb4775248b80fb57.
// Every parser bounds-checks against its buffer end and throws std::runtime_error
// on malformed input (fuzzed under ASan/UBSan by the self-test).
#pragma once
#include <cpuid.h>
#include <nmmintrin.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <fstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace mnistx_host {

// ------------------------------------------------------------------ crc32c
inline uint32_t kTable[8][256];
inline bool g_hw = false;

struct CrcInit {
  CrcInit() {
    const uint32_t poly = 0x82F63B78u;
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : c >> 1;
      kTable[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int t = 1; t < 8; ++t) kTable[t][i] = (kTable[t - 1][i] >> 8) ^ kTable[0][kTable[t - 1][i] & 0xff];
    unsigned a, b, c, d;
    if (__get_cpuid(1, &a, &b, &c, &d)) g_hw = (c & bit_SSE4_2) != 0;
  }
};
inline CrcInit g_crc_init;

__attribute__((target("sse4.2"))) inline uint32_t crc_hw(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = crc;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32;
}

inline uint32_t crc_sw(uint32_t crc, const uint8_t* p, size_t n) {
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= crc;
    crc = kTable[7][lo & 0xff] ^ kTable[6][(lo >> 8) & 0xff] ^ kTable[5][(lo >> 16) & 0xff] ^ kTable[4][lo >> 24] ^
          kTable[3][hi & 0xff] ^ kTable[2][(hi >> 8) & 0xff] ^ kTable[1][(hi >> 16) & 0xff] ^ kTable[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) crc = (crc >> 8) ^ kTable[0][(crc ^ *p++) & 0xff];
  return crc;
}

inline uint32_t crc32c_extend(uint32_t init, const uint8_t* p, size_t n) {
  uint32_t c = ~init;
  c = g_hw ? crc_hw(c, p, n) : crc_sw(c, p, n);
  return ~c;
}

inline uint32_t crc32c(const uint8_t* p, size_t n) { return crc32c_extend(0, p, n); }

constexpr uint32_t kMaskDelta = 0xa282ead8u;
inline uint32_t mask_crc(uint32_t c) { return ((c >> 15) | (c << 17)) + kMaskDelta; }
inline uint32_t unmask_crc(uint32_t m) {
  uint32_t r = m - kMaskDelta;
  return (r >> 17) | (r << 15);
}

// ------------------------------------------------------------------ helpers
inline std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  f.seekg(0, std::ios::end);
  std::string s((size_t)f.tellg(), '\0');
  f.seekg(0);
  f.read(&s[0], (std::streamsize)s.size());
  return s;
}

inline void put_u32(std::string& s, uint32_t v) { s.append((const char*)&v, 4); }
inline void put_u64(std::string& s, uint64_t v) { s.append((const char*)&v, 8); }
inline uint32_t get_u32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
inline uint64_t get_u64(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}

inline void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)(v | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}

inline bool get_varint(const uint8_t*& p, const uint8_t* end, uint64_t& v) {
  v = 0;
  for (int shift = 0; shift <= 63 && p < end; shift += 7) {
    uint64_t b = *p++;
    v |= (b & 0x7f) << shift;
    if (!(b & 0x80)) return true;
  }
  return false;
}

// ------------------------------------------------------------------ TFRecord
inline std::string frame(const std::string& rec) {
  std::string out;
  out.reserve(rec.size() + 16);
  const uint64_t len = rec.size();
  put_u64(out, len);
  put_u32(out, mask_crc(crc32c((const uint8_t*)&len, 8)));
  out += rec;
  put_u32(out, mask_crc(crc32c((const uint8_t*)rec.data(), rec.size())));
  return out;
}

inline std::vector<std::pair<size_t, size_t>> split_records(const std::string& buf, bool verify) {
  std::vector<std::pair<size_t, size_t>> recs;
  const uint8_t* base = (const uint8_t*)buf.data();
  size_t off = 0;
  while (off < buf.size()) {
    if (off + 12 > buf.size()) throw std::runtime_error("truncated TFRecord header");
    const uint64_t len = get_u64(base + off);
    if (verify && unmask_crc(get_u32(base + off + 8)) != crc32c(base + off, 8))
      throw std::runtime_error("TFRecord length crc mismatch at offset " + std::to_string(off));
    const size_t data = off + 12;
    if (len > buf.size() || data + len + 4 > buf.size()) throw std::runtime_error("truncated TFRecord payload");
    if (verify && unmask_crc(get_u32(base + data + len)) != crc32c(base + data, len))
      throw std::runtime_error("TFRecord data crc mismatch at offset " + std::to_string(off));
    recs.emplace_back(data, (size_t)len);
    off = data + len + 4;
  }
  return recs;
}

inline void tfrecord_write(const std::string& path, const std::vector<std::string>& records, bool append) {
  std::ofstream f(path, std::ios::binary | (append ? std::ios::app : std::ios::trunc));
  if (!f) throw std::runtime_error("cannot open " + path);
  for (auto& r : records) {
    const std::string fr = frame(r);
    f.write(fr.data(), (std::streamsize)fr.size());
  }
  f.flush();
}

// ------------------------------------------------------------------ tf.Example (minimal decoder)
// Example{features=1: Features{feature=1: map<string,Feature>}}; Feature{bytes_list=1, float_list=2,
// int64_list=3}; BytesList{value=1 (bytes)}; Int64List{value=1 (packed or not)}.
struct Field {
  const uint8_t* p = nullptr;
  uint64_t n = 0;
};

inline bool next_field(const uint8_t*& p, const uint8_t* end, uint32_t& num, uint32_t& wt, Field& f, uint64_t& ival) {
  if (p >= end) return false;
  uint64_t key;
  if (!get_varint(p, end, key)) throw std::runtime_error("bad proto key");
  num = (uint32_t)(key >> 3);
  wt = (uint32_t)(key & 7);
  switch (wt) {
    case 0:
      if (!get_varint(p, end, ival)) throw std::runtime_error("bad varint");
      break;
    case 1:
      if (end - p < 8) throw std::runtime_error("truncated fixed64");
      p += 8;
      break;
    case 2: {
      uint64_t n;
      if (!get_varint(p, end, n) || n > (uint64_t)(end - p)) throw std::runtime_error("bad length-delimited field");
      f.p = p;
      f.n = n;
      p += n;
      break;
    }
    case 5:
      if (end - p < 4) throw std::runtime_error("truncated fixed32");
      p += 4;
      break;
    default:
      throw std::runtime_error("unsupported wire type");
  }
  return true;
}

struct Decoded {
  std::string image;
  int64_t label = -1;
  bool has_image = false, has_label = false;
};

inline Decoded decode_example(const uint8_t* p, const uint8_t* end, const std::string& ikey, const std::string& lkey) {
  Decoded d;
  uint32_t num, wt;
  Field f;
  uint64_t iv;
  while (next_field(p, end, num, wt, f, iv)) {
    if (num != 1 || wt != 2) continue;  // Example.features
    const uint8_t* q = f.p;
    const uint8_t* qe = f.p + f.n;
    Field e;
    while (next_field(q, qe, num, wt, e, iv)) {
      if (num != 1 || wt != 2) continue;  // Features.feature (map entry)
      const uint8_t* r = e.p;
      const uint8_t* re = e.p + e.n;
      std::string key;
      Field val;
      Field g;
      while (next_field(r, re, num, wt, g, iv)) {
        if (num == 1 && wt == 2) key.assign((const char*)g.p, g.n);
        if (num == 2 && wt == 2) val = g;
      }
      if (!val.p) continue;
      const uint8_t* s = val.p;
      const uint8_t* se = val.p + val.n;
      Field h;
      while (next_field(s, se, num, wt, h, iv)) {
        if (wt != 2) continue;
        const uint8_t* t = h.p;
        const uint8_t* te = h.p + h.n;
        if (num == 1 && key == ikey) {  // BytesList
          Field b;
          while (next_field(t, te, num, wt, b, iv))
            if (num == 1 && wt == 2) {
              d.image.assign((const char*)b.p, b.n);
              d.has_image = true;
            }
        } else if (num == 3 && key == lkey) {  // Int64List
          Field b;
          uint64_t v;
          while (t < te) {
            uint64_t k2;
            if (!get_varint(t, te, k2)) break;
            if ((k2 & 7) == 0) {
              if (!get_varint(t, te, v)) throw std::runtime_error("bad int64 value");
              d.label = (int64_t)v;
              d.has_label = true;
            } else if ((k2 & 7) == 2) {  // packed
              uint64_t n2;
              if (!get_varint(t, te, n2) || n2 > (uint64_t)(te - t)) throw std::runtime_error("bad packed int64");
              const uint8_t* pe = t + n2;
              while (t < pe) {
                if (!get_varint(t, pe, v)) throw std::runtime_error("bad packed int64 value");
                d.label = (int64_t)v;
                d.has_label = true;
              }
            } else {
              break;
            }
          }
        }
      }
    }
  }
  return d;
}

// Decode the (image_raw, label) pair of every record in a set of TFRecord files:
// concatenated image bytes, labels, bytes per image.  Multi-threaded.
struct DecodedFiles {
  std::string images;
  std::vector<int64_t> labels;
  size_t per = 0;
};

inline DecodedFiles decode_mnist_files(const std::vector<std::string>& paths, const std::string& ikey,
                                       const std::string& lkey, bool verify, int threads) {
  std::vector<std::string> bufs(paths.size());
  std::vector<std::vector<std::pair<size_t, size_t>>> recs(paths.size());
  size_t total = 0;
  for (size_t i = 0; i < paths.size(); ++i) {
    bufs[i] = read_file(paths[i]);
    recs[i] = split_records(bufs[i], verify);
    total += recs[i].size();
  }
  std::vector<const uint8_t*> ptr;
  std::vector<size_t> len;
  ptr.reserve(total);
  len.reserve(total);
  for (size_t i = 0; i < paths.size(); ++i)
    for (auto& r : recs[i]) {
      ptr.push_back((const uint8_t*)bufs[i].data() + r.first);
      len.push_back(r.second);
    }
  std::vector<Decoded> dec(total);
  if (threads < 1) threads = 1;
  std::vector<std::thread> pool;
  std::vector<std::string> errs(threads);
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      try {
        for (size_t i = t; i < total; i += threads) dec[i] = decode_example(ptr[i], ptr[i] + len[i], ikey, lkey);
      } catch (const std::exception& e) {
        errs[t] = e.what();
      }
    });
  for (auto& th : pool) th.join();
  for (auto& e : errs)
    if (!e.empty()) throw std::runtime_error("tf.Example decode: " + e);
  size_t per = total ? dec[0].image.size() : 0;
  std::string images;
  images.reserve(per * total);
  std::vector<int64_t> labels(total);
  for (size_t i = 0; i < total; ++i) {
    if (!dec[i].has_image || !dec[i].has_label)
      throw std::runtime_error("record " + std::to_string(i) + " lacks '" + ikey + "' or '" + lkey + "'");
    if (dec[i].image.size() != per) throw std::runtime_error("records have different image sizes");
    images += dec[i].image;
    labels[i] = dec[i].label;
  }
  DecodedFiles r;
  r.images = std::move(images);
  r.labels = std::move(labels);
  r.per = per;
  return r;
}

// ------------------------------------------------------------------ SSTable (leveldb table format)
constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;
constexpr int kRestartInterval = 16;
constexpr size_t kBlockSize = 262144;  // tensorflow table::Options default

struct BlockBuilder {
  std::string buf;
  std::vector<uint32_t> restarts{0};
  std::string last;
  int counter = 0;
  size_t entries = 0;
  void add(const std::string& k, const std::string& v) {
    size_t shared = 0;
    if (counter < kRestartInterval) {
      const size_t mn = std::min(last.size(), k.size());
      while (shared < mn && last[shared] == k[shared]) ++shared;
    } else {
      restarts.push_back((uint32_t)buf.size());
      counter = 0;
    }
    put_varint(buf, shared);
    put_varint(buf, k.size() - shared);
    put_varint(buf, v.size());
    buf.append(k, shared, std::string::npos);
    buf += v;
    last = k;
    ++counter;
    ++entries;
  }
  std::string finish() {
    std::string out = buf;
    for (uint32_t r : restarts) put_u32(out, r);
    put_u32(out, (uint32_t)restarts.size());
    return out;
  }
  size_t size_estimate() const { return buf.size() + restarts.size() * 4 + 4; }
};

inline std::string write_block(std::string& file, const std::string& contents) {
  // returns the encoded BlockHandle
  std::string handle;
  put_varint(handle, file.size());
  put_varint(handle, contents.size());
  file += contents;
  const char type = 0;  // kNoCompression
  file.push_back(type);
  uint32_t c = crc32c((const uint8_t*)contents.data(), contents.size());
  c = crc32c_extend(c, (const uint8_t*)&type, 1);
  put_u32(file, mask_crc(c));
  return handle;
}

// entries must be sorted by key (bytewise) and unique.
inline std::string sstable_build(const std::vector<std::pair<std::string, std::string>>& entries) {
  for (size_t i = 1; i < entries.size(); ++i)
    if (!(entries[i - 1].first < entries[i].first)) throw std::runtime_error("sstable keys must be sorted and unique");
  std::string file;
  BlockBuilder data, index;
  for (auto& kv : entries) {
    data.add(kv.first, kv.second);
    if (data.size_estimate() >= kBlockSize) {
      const std::string h = write_block(file, data.finish());
      index.add(data.last, h);
      data = BlockBuilder();
    }
  }
  if (data.entries > 0) {
    const std::string h = write_block(file, data.finish());
    index.add(data.last, h);
  }
  BlockBuilder meta;
  const std::string meta_h = write_block(file, meta.finish());
  const std::string index_h = write_block(file, index.finish());
  std::string footer = meta_h + index_h;
  footer.resize(40, '\0');
  put_u64(footer, kTableMagic);
  file += footer;
  return file;
}

inline std::string read_block(const std::string& file, uint64_t off, uint64_t size, bool verify) {
  if (off > file.size() || size > file.size() || off + size + 5 > file.size())
    throw std::runtime_error("sstable block out of range");
  const uint8_t* p = (const uint8_t*)file.data() + off;
  const uint8_t type = p[size];
  if (type != 0) throw std::runtime_error("compressed sstable blocks are not supported");
  if (verify) {
    uint32_t c = crc32c(p, size);
    c = crc32c_extend(c, p + size, 1);
    if (mask_crc(c) != get_u32(p + size + 1)) throw std::runtime_error("sstable block crc mismatch");
  }
  return file.substr(off, size);
}

inline std::vector<std::pair<std::string, std::string>> parse_block(const std::string& b) {
  std::vector<std::pair<std::string, std::string>> out;
  if (b.size() < 4) throw std::runtime_error("bad block");
  const uint8_t* p = (const uint8_t*)b.data();
  const uint32_t nrest = get_u32(p + b.size() - 4);
  if ((uint64_t)nrest * 4 + 4 > b.size()) throw std::runtime_error("bad restart array");
  const uint8_t* end = p + b.size() - 4 - 4 * nrest;
  std::string key;
  while (p < end) {
    uint64_t shared, nons, vlen;
    if (!get_varint(p, end, shared) || !get_varint(p, end, nons) || !get_varint(p, end, vlen))
      throw std::runtime_error("bad block entry");
    if (shared > key.size() || nons > (uint64_t)(end - p) || vlen > (uint64_t)(end - p) - nons)
      throw std::runtime_error("corrupt block entry");
    key.resize(shared);
    key.append((const char*)p, nons);
    p += nons;
    out.emplace_back(key, std::string((const char*)p, vlen));
    p += vlen;
  }
  return out;
}

inline std::vector<std::pair<std::string, std::string>> sstable_parse(const std::string& file, bool verify) {
  if (file.size() < 48) throw std::runtime_error("file too small for an sstable");
  const uint8_t* f = (const uint8_t*)file.data() + file.size() - 48;
  if (get_u64(f + 40) != kTableMagic) throw std::runtime_error("bad sstable magic");
  const uint8_t* p = f;
  uint64_t mo, ms, io, is;
  if (!get_varint(p, f + 40, mo) || !get_varint(p, f + 40, ms) || !get_varint(p, f + 40, io) ||
      !get_varint(p, f + 40, is))
    throw std::runtime_error("bad footer");
  std::vector<std::pair<std::string, std::string>> out;
  for (auto& ie : parse_block(read_block(file, io, is, verify))) {
    const uint8_t* h = (const uint8_t*)ie.second.data();
    const uint8_t* he = h + ie.second.size();
    uint64_t bo, bs;
    if (!get_varint(h, he, bo) || !get_varint(h, he, bs)) throw std::runtime_error("bad block handle");
    for (auto& kv : parse_block(read_block(file, bo, bs, verify))) out.emplace_back(kv.first, kv.second);
  }
  return out;
}

}  // namespace mnistx_host
