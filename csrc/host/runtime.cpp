// Python bindings of the host runtime (module `_host`); the logic lives in
// runtime_core.h (shared with the sanitizer self-test).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime_core.h"

namespace py = pybind11;
using namespace mnistx_host;

namespace {

py::list tfrecord_read(const std::string& path, bool verify) {
  const std::string buf = read_file(path);
  py::list out;
  for (auto& r : split_records(buf, verify)) out.append(py::bytes(buf.data() + r.first, r.second));
  return out;
}

py::tuple decode_files(const std::vector<std::string>& paths, const std::string& ikey, const std::string& lkey,
                       bool verify, int threads) {
  DecodedFiles d;
  {
    py::gil_scoped_release nogil;
    d = decode_mnist_files(paths, ikey, lkey, verify, threads);
  }
  return py::make_tuple(py::bytes(d.images), d.labels, d.per);
}

std::vector<std::pair<py::bytes, py::bytes>> parse_table(const std::string& file, bool verify) {
  std::vector<std::pair<py::bytes, py::bytes>> out;
  for (auto& kv : sstable_parse(file, verify)) out.emplace_back(py::bytes(kv.first), py::bytes(kv.second));
  return out;
}

}  // namespace

PYBIND11_MODULE(_host, m) {
  m.doc() = "Host-side native runtime: crc32c, TFRecord, tf.Example, SSTable (tensor bundle)";
  m.def("crc32c", [](py::bytes b) {
    std::string s = b;
    return crc32c((const uint8_t*)s.data(), s.size());
  });
  m.def("masked_crc32c", [](py::bytes b) {
    std::string s = b;
    return mask_crc(crc32c((const uint8_t*)s.data(), s.size()));
  });
  m.def("crc32c_hw", []() { return g_hw; });
  m.def("tfrecord_read", &tfrecord_read, py::arg("path"), py::arg("verify") = true);
  m.def("tfrecord_write", &tfrecord_write, py::arg("path"), py::arg("records"), py::arg("append") = false);
  m.def("tfrecord_frame", [](py::bytes b) { return py::bytes(frame(std::string(b))); });
  m.def("decode_mnist_files", &decode_files, py::arg("paths"), py::arg("image_key") = "image_raw",
        py::arg("label_key") = "label", py::arg("verify") = true, py::arg("threads") = 4);
  m.def("sstable_build", [](const std::vector<std::pair<std::string, std::string>>& e) {
    return py::bytes(sstable_build(e));
  });
  m.def("sstable_parse", [](py::bytes b, bool verify) { return parse_table(std::string(b), verify); },
        py::arg("data"), py::arg("verify") = true);
}
