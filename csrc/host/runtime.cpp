// Python bindings of the host runtime (module `_host`); the logic lives in
// runtime_core.h (shared with the sanitizer self-test).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "ps_shm.h"
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

// parallel/ps.py ShmTransport: one ps_serve call (GIL released).  Pointers are raw
// addresses (the segment mapping, and the contiguous CPU tensors / numpy arrays the PS owns).
py::tuple ps_shm_serve(uintptr_t base, std::vector<int64_t> lay, uintptr_t params, uintptr_t mom, uintptr_t ema,
                       uintptr_t wd, std::vector<double> opt, std::vector<int64_t> st, uintptr_t per_worker,
                       uintptr_t last_seq, uintptr_t arrivals, int64_t arrivals_cap, uintptr_t mark_steps,
                       uintptr_t mark_times, int nmarks, uintptr_t phase, double idle_timeout) {
  if (lay.size() != 7 || opt.size() != 7 || st.size() != 7) throw std::invalid_argument("ps_shm_serve: bad tuple");
  PsLayout L{lay[0], lay[1], lay[2], lay[3], lay[4], lay[5], lay[6]};
  PsOpt o{opt[0], opt[1], (int64_t)opt[2], opt[3], (int)opt[4], (int)opt[5], opt[6]};
  PsState S{};
  S.gstep = st[0];
  S.max_steps = st[1];
  S.applied = st[2];
  S.rejected = st[3];
  S.kill_step = st[4];
  S.narr = st[5];
  S.last = (int)st[6];
  S.per_worker = (int64_t*)per_worker;
  S.last_seq = (int64_t*)last_seq;
  S.arrivals = (int32_t*)arrivals;
  S.arrivals_cap = arrivals_cap;
  S.mark_steps = (const int64_t*)mark_steps;
  S.mark_times = (double*)mark_times;
  S.nmarks = nmarks;
  double* ph = (double*)phase;
  for (int i = 0; i < 3; ++i) S.phase[i] = ph[i];
  S.idle_timeout = idle_timeout;
  int who = -1, rc;
  {
    py::gil_scoped_release nogil;
    rc = ps_serve((uint8_t*)base, L, (float*)params, (float*)mom, (float*)ema, (const float*)wd, o, S, &who);
  }
  for (int i = 0; i < 3; ++i) ph[i] = S.phase[i];
  return py::make_tuple(rc, who, S.gstep, S.applied, S.rejected, S.narr, S.last);
}

// the same update alone (tests: bitwise runtime/torchnet.torch_update)
void ps_apply_once(uintptr_t params, uintptr_t grads, uintptr_t mom, uintptr_t ema, uintptr_t wd, int64_t n,
                   std::vector<double> opt, int64_t step) {
  if (opt.size() != 7) throw std::invalid_argument("ps_apply_once: bad opt tuple");
  PsOpt o{opt[0], opt[1], (int64_t)opt[2], opt[3], (int)opt[4], (int)opt[5], opt[6]};
  py::gil_scoped_release nogil;
  ps_apply((float*)params, (const float*)grads, (float*)mom, (float*)ema, (const float*)wd, n, o, step);
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
  m.def("ps_shm_serve", &ps_shm_serve);
  m.def("ps_apply_once", &ps_apply_once);
  m.def("sstable_parse", [](py::bytes b, bool verify) { return parse_table(std::string(b), verify); },
        py::arg("data"), py::arg("verify") = true);
}
