// Sanitizer self-test of the host runtime core (csrc/host/runtime_core.h).
//
// Built twice by tests/test_native_sanitizers.py:
//   * -fsanitize=address,undefined : round trips + mutation fuzzing of every parser
//     (malformed input must throw std::runtime_error, never read out of bounds)
//   * -fsanitize=thread            : the multi-threaded tf.Example decoder (race detector)
// Prints "ALL OK" and exits 0 on success; any sanitizer report aborts non-zero.
#include <cstdio>
#include <cstdlib>
#include <random>

#include "runtime_core.h"

using namespace mnistx_host;

#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                 \
    }                                                               \
  } while (0)

static std::string key_field(uint32_t num, const std::string& payload) {
  std::string s;
  put_varint(s, (uint64_t)num << 3 | 2);
  put_varint(s, payload.size());
  return s + payload;
}

// tf.Example{features{feature{key: "image_raw", bytes_list{value}}, feature{key: "label", int64_list{value}}}}
static std::string make_example(const std::string& img, int64_t label, bool packed) {
  std::string bl = key_field(1, img);                      // BytesList.value
  std::string il;
  if (packed) {
    std::string v;
    put_varint(v, (uint64_t)label);
    il = key_field(1, v);
  } else {
    put_varint(il, 1 << 3 | 0);
    put_varint(il, (uint64_t)label);
  }
  const std::string fimg = key_field(1, bl), flab = key_field(3, il);          // Feature
  const std::string e1 = key_field(1, "image_raw") + key_field(2, fimg);       // map entry
  const std::string e2 = key_field(1, "label") + key_field(2, flab);
  const std::string feats = key_field(1, e1) + key_field(1, e2);               // Features
  return key_field(1, feats);                                                  // Example
}

template <class F>
static int fuzz(const std::string& good, F&& parse, std::mt19937& rng, int iters) {
  int rejected = 0;
  for (int it = 0; it < iters; ++it) {
    std::string b = good;
    const int kind = it % 3;
    if (kind == 0 && !b.empty()) {                      // flip random bytes
      const int n = 1 + rng() % 4;
      for (int k = 0; k < n; ++k) b[rng() % b.size()] ^= (char)(1 + rng() % 255);
    } else if (kind == 1) {                             // truncate
      b.resize(rng() % (b.size() + 1));
    } else {                                            // garbage tail / random buffer
      b = b.substr(0, rng() % (b.size() + 1));
      const int n = rng() % 64;
      for (int k = 0; k < n; ++k) b.push_back((char)rng());
    }
    try {
      parse(b);
    } catch (const std::runtime_error&) {
      ++rejected;
    }
  }
  return rejected;
}

int main() {
  std::mt19937 rng(1234);
  // ---- crc32c: standard check value, hardware == software path
  const char* nine = "123456789";
  CHECK(crc32c((const uint8_t*)nine, 9) == 0xE3069283u);
  CHECK(crc32c((const uint8_t*)"", 0) == 0u);
  for (int it = 0; it < 200; ++it) {
    std::string s(rng() % 1000, '\0');
    for (auto& c : s) c = (char)rng();
    const uint32_t sw = ~crc_sw(~0u, (const uint8_t*)s.data(), s.size());
    CHECK(sw == crc32c((const uint8_t*)s.data(), s.size()));
    if (g_hw) CHECK(sw == ~crc_hw(~0u, (const uint8_t*)s.data(), s.size()));
    CHECK(unmask_crc(mask_crc(sw)) == sw);
  }
  // ---- TFRecord framing round trip + corruption detection + fuzz
  std::vector<std::string> recs;
  std::string file;
  for (int i = 0; i < 50; ++i) {
    std::string r(rng() % 300, '\0');
    for (auto& c : r) c = (char)rng();
    recs.push_back(r);
    file += frame(r);
  }
  auto spans = split_records(file, true);
  CHECK(spans.size() == recs.size());
  for (size_t i = 0; i < recs.size(); ++i) CHECK(file.substr(spans[i].first, spans[i].second) == recs[i]);
  {
    std::string bad = file;
    bad[spans[3].first] ^= 1;
    bool threw = false;
    try {
      split_records(bad, true);
    } catch (const std::runtime_error&) {
      threw = true;
    }
    CHECK(threw);
  }
  fuzz(file, [](const std::string& b) { split_records(b, true); }, rng, 3000);
  fuzz(file, [](const std::string& b) { split_records(b, false); }, rng, 3000);
  // ---- tf.Example decode round trip + fuzz
  std::string img(784, '\0');
  for (auto& c : img) c = (char)rng();
  for (bool packed : {false, true}) {
    const std::string ex = make_example(img, 7, packed);
    Decoded d = decode_example((const uint8_t*)ex.data(), (const uint8_t*)ex.data() + ex.size(), "image_raw", "label");
    CHECK(d.has_image && d.has_label && d.label == 7 && d.image == img);
    fuzz(ex, [](const std::string& b) {
      decode_example((const uint8_t*)b.data(), (const uint8_t*)b.data() + b.size(), "image_raw", "label");
    }, rng, 5000);
  }
  // ---- multi-threaded file decode (the TSan build checks this for races)
  {
    const char* dir = std::getenv("SELFTEST_TMP");
    const std::string base = std::string(dir ? dir : "/tmp") + "/selftest_";
    std::vector<std::string> paths;
    int64_t want = 0;
    for (int f = 0; f < 3; ++f) {
      std::vector<std::string> rs;
      for (int i = 0; i < 40; ++i) {
        rs.push_back(make_example(img, (f * 40 + i) % 10, i % 2));
        want += (f * 40 + i) % 10;
      }
      paths.push_back(base + std::to_string(f) + ".tfrecord");
      tfrecord_write(paths.back(), rs, false);
    }
    DecodedFiles d = decode_mnist_files(paths, "image_raw", "label", true, 4);
    CHECK(d.per == 784 && d.labels.size() == 120 && d.images.size() == 120 * 784);
    int64_t got = 0;
    for (auto v : d.labels) got += v;
    CHECK(got == want);
    for (auto& p : paths) std::remove(p.c_str());
  }
  // ---- SSTable round trip (several 256 KiB data blocks) + fuzz
  std::vector<std::pair<std::string, std::string>> kv;
  for (int i = 0; i < 400; ++i) {
    char k[32];
    std::snprintf(k, sizeof k, "layer%03d/weights", i);
    std::string v(rng() % 4000, '\0');
    for (auto& c : v) c = (char)rng();
    kv.emplace_back(k, v);
  }
  const std::string table = sstable_build(kv);
  const auto back = sstable_parse(table, true);
  CHECK(back == kv);
  // small table for a dense fuzz
  std::vector<std::pair<std::string, std::string>> small(kv.begin(), kv.begin() + 20);
  for (auto& e : small) e.second.resize(e.second.size() % 64);
  const std::string st = sstable_build(small);
  fuzz(st, [](const std::string& b) { sstable_parse(b, true); }, rng, 4000);
  fuzz(st, [](const std::string& b) { sstable_parse(b, false); }, rng, 4000);
  std::printf("ALL OK (crc32c hw=%d)\n", (int)g_hw);
  return 0;
}
