// pybind11 module `_native`: host runtime of the volunteer-computing framework.
// All blocking calls release the GIL (without_gil: never re-entering a finalizing interpreter).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <unistd.h>

#include <algorithm>

#include "colour.h"
#include "scheduler.h"
#include "transport.h"

namespace py = pybind11;
using namespace vcxrt;

namespace {

// A received frame whose payload is exposed through the buffer protocol without a copy
// (numpy.frombuffer(frame, dtype) views the bytes the transport thread filled).
struct PyFrame {
  Frame f;
};

// C-contiguous check for raw uint8 buffers handed to the colour loops (which index them linearly)
void require_c_contiguous(const py::buffer_info& b, const char* what) {
  py::ssize_t expect = b.itemsize;
  for (int d = (int)b.ndim - 1; d >= 0; --d) {
    if (b.shape[d] > 1 && b.strides[d] != expect) throw std::invalid_argument(std::string(what) + ": not C-contiguous");
    expect *= b.shape[d];
  }
}

// Blocking calls run without the GIL. A daemon Python thread still inside one when the
// interpreter finalizes is pthread_exit()ed the moment it re-takes the GIL; from inside
// gil_scoped_release's (noexcept) destructor that forced unwind is a std::terminate — "terminate
// called without an active exception", exit status 134 after an otherwise clean run. Such a
// thread parks instead of re-entering the interpreter; process exit reclaims it.
[[noreturn]] void park_forever() {
  for (;;) ::pause();
}

template <class F>
auto without_gil(F&& f) {
  PyThreadState* ts = PyEval_SaveThread();
  auto r = f();
  if (_Py_IsFinalizing()) park_forever();
  PyEval_RestoreThread(ts);
  return r;
}

// Hub::recv in slices of <= 100 ms, so a finalizing interpreter is noticed promptly
bool recv_sliced(Hub& h, Frame* f, double timeout) {
  for (;;) {
    const double slice = timeout < 0 ? 0.1 : std::min(timeout, 0.1);
    if (h.recv(f, slice)) return true;
    if (_Py_IsFinalizing()) park_forever();
    if (timeout >= 0) {
      timeout -= slice;
      if (timeout <= 0) return false;
    }
    if (h.closed()) return false;
  }
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "C++ runtime: framed TCP transport, chunk scheduler, reorder index";

  py::class_<PyFrame>(m, "Frame", py::buffer_protocol())
      .def_property_readonly("header", [](const PyFrame& p) { return py::str(p.f.header); })
      .def_property_readonly("peer", [](const PyFrame& p) { return p.f.peer; })
      .def_property_readonly("nbytes", [](const PyFrame& p) { return p.f.payload.size(); })
      .def_buffer([](PyFrame& p) -> py::buffer_info {
        return py::buffer_info(p.f.payload.data(), 1, py::format_descriptor<uint8_t>::format(), 1,
                               {(py::ssize_t)p.f.payload.size()}, {(py::ssize_t)1});
      });

  py::class_<Hub>(m, "Hub")
      .def(py::init<const std::string&, int, size_t, bool, uint64_t, uint32_t>(), py::arg("bind_host") = "",
           py::arg("port") = 0, py::arg("capacity") = 64, py::arg("ack") = true,
           py::arg("max_payload") = Hub::kDefaultMaxPayload, py::arg("max_header") = Hub::kDefaultMaxHeader)
      .def_property_readonly("port", &Hub::port)
      .def(
          "recv",
          [](Hub& h, double timeout) -> py::object {
            auto pf = std::make_unique<PyFrame>();
            const bool ok = without_gil([&] { return recv_sliced(h, &pf->f, timeout); });
            if (!ok) return py::none();
            return py::cast(pf.release(), py::return_value_policy::take_ownership);
          },
          py::arg("timeout") = -1.0)
      .def("pending", &Hub::pending)
      .def("close", [](Hub& h) { without_gil([&] { h.close(); return 0; }); })
      .def_property_readonly("frames_received", &Hub::frames_received)
      .def_property_readonly("bytes_received", &Hub::bytes_received)
      .def_property_readonly("frames_rejected", &Hub::frames_rejected);

  py::class_<Sender>(m, "Sender")
      .def(py::init([](const std::string& host, int port, bool ack, double connect_timeout) {
             return without_gil([&] { return new Sender(host, port, ack, connect_timeout); });
           }),
           py::arg("host"), py::arg("port"), py::arg("ack") = true, py::arg("connect_timeout") = 10.0)
      .def(
          "send",
          [](Sender& s, const std::string& header, py::buffer payload, double timeout) {
            py::buffer_info bi = payload.request();
            size_t n = (size_t)bi.size * (size_t)bi.itemsize;
            // require C-contiguous bytes; the python layer makes arrays contiguous first
            if (bi.ndim > 0) {
              py::ssize_t expect = bi.itemsize;
              for (int d = (int)bi.ndim - 1; d >= 0; --d) {
                if (bi.shape[d] > 1 && bi.strides[d] != expect)
                  throw std::invalid_argument("Sender.send: payload must be C-contiguous");
                expect *= bi.shape[d];
              }
            }
            const uint8_t* ptr = (const uint8_t*)bi.ptr;
            return without_gil([&] { return s.send(header, ptr, n, timeout); });
          },
          py::arg("header"), py::arg("payload"), py::arg("timeout") = 60.0)
      .def("close", &Sender::close)
      .def_property_readonly("connected", &Sender::connected)
      .def_property_readonly("bytes_sent", &Sender::bytes_sent);

  py::class_<Assignment>(m, "Assignment")
      .def_readonly("chunk", &Assignment::chunk)
      .def_readonly("worker", &Assignment::worker)
      .def_readonly("requester", &Assignment::requester)
      .def("valid", &Assignment::valid);

  py::class_<ChunkScheduler> cs(m, "ChunkScheduler");
  py::enum_<ChunkScheduler::Policy>(cs, "Policy")
      .value("ROUND_ROBIN", ChunkScheduler::ROUND_ROBIN)
      .value("LEAST_LOADED", ChunkScheduler::LEAST_LOADED);
  cs.def(py::init<int, int>(), py::arg("policy") = 0, py::arg("credits") = 2)
      .def("add_worker", &ChunkScheduler::add_worker)
      .def("remove_worker", &ChunkScheduler::remove_worker)
      .def("set_available", &ChunkScheduler::set_available)
      .def("has_worker", &ChunkScheduler::has_worker)
      .def("workers", &ChunkScheduler::workers)
      .def("available_workers", &ChunkScheduler::available_workers)
      .def("heartbeat", &ChunkScheduler::heartbeat)
      .def("expire", &ChunkScheduler::expire)
      .def("submit", &ChunkScheduler::submit)
      .def("requeue_front", &ChunkScheduler::requeue_front)
      .def_property_readonly("requeued", &ChunkScheduler::requeued)
      .def("next", &ChunkScheduler::next)
      .def("complete", &ChunkScheduler::complete)
      .def("fail", &ChunkScheduler::fail)
      .def("cancel_requester", &ChunkScheduler::cancel_requester)
      .def("queued", &ChunkScheduler::queued)
      .def("inflight", &ChunkScheduler::inflight)
      .def("inflight_of", &ChunkScheduler::inflight_of)
      .def_property_readonly("dispatched", &ChunkScheduler::dispatched);

  // colour conversion for the video I/O path (GIL released); buffers are C-contiguous uint8
  m.def(
      "bgr_to_yuv444",
      [](py::buffer src, py::buffer dst, int64_t w, int64_t h) {
        py::buffer_info a = src.request(), b = dst.request(true);
        require_c_contiguous(a, "bgr_to_yuv444 src");
        require_c_contiguous(b, "bgr_to_yuv444 dst");
        if (a.size * a.itemsize < 3 * w * h || b.size * b.itemsize < 3 * w * h)
          throw std::invalid_argument("bgr_to_yuv444: buffers smaller than 3 * w * h bytes");
        without_gil([&] {
          bgr_to_yuv444((const uint8_t*)a.ptr, (uint8_t*)b.ptr, w, h);
          return 0;
        });
      },
      py::arg("src"), py::arg("dst"), py::arg("w"), py::arg("h"));
  m.def(
      "bgr_to_yuv444_frames",
      [](py::buffer src, py::buffer dst, int64_t k, int64_t w, int64_t h) {
        py::buffer_info a = src.request(), b = dst.request(true);
        require_c_contiguous(a, "bgr_to_yuv444_frames src");
        require_c_contiguous(b, "bgr_to_yuv444_frames dst");
        if (k < 0 || a.size * a.itemsize < 3 * k * w * h || b.size * b.itemsize < 3 * k * w * h)
          throw std::invalid_argument("bgr_to_yuv444_frames: buffers smaller than 3 * k * w * h bytes");
        without_gil([&] {
          bgr_to_yuv444_frames((const uint8_t*)a.ptr, (uint8_t*)b.ptr, k, w, h);
          return 0;
        });
      },
      py::arg("src"), py::arg("dst"), py::arg("k"), py::arg("w"), py::arg("h"));
  m.def(
      "write_bytes",
      [](int fd, int64_t off, py::buffer src) {
        py::buffer_info a = src.request();
        require_c_contiguous(a, "write_bytes src");
        if (off < 0) throw std::invalid_argument("write_bytes: negative offset");
        const int64_t n = a.size * a.itemsize;
        return without_gil([&] { return write_bytes(fd, off, (const uint8_t*)a.ptr, n); });
      },
      py::arg("fd"), py::arg("off"), py::arg("src"));
  m.def(
      "write_frames",
      [](int fd, int64_t off, py::buffer src, int64_t k, int64_t w, int64_t h, bool y4m) {
        py::buffer_info a = src.request();
        require_c_contiguous(a, "write_frames src");
        if (k < 0 || w <= 0 || h <= 0 || off < 0 || a.size * a.itemsize < 3 * k * w * h)
          throw std::invalid_argument("write_frames: buffer smaller than 3 * k * w * h bytes");
        return without_gil([&] { return write_frames(fd, off, (const uint8_t*)a.ptr, k, w, h, y4m); });
      },
      py::arg("fd"), py::arg("off"), py::arg("src"), py::arg("k"), py::arg("w"), py::arg("h"), py::arg("y4m"));
  m.def(
      "yuv_to_bgr",
      [](py::buffer y, py::buffer u, py::buffer v, py::buffer dst, int64_t w, int64_t h, int64_t cw) {
        py::buffer_info Y = y.request(), U = u.request(), V = v.request(), D = dst.request(true);
        for (auto* b : {&Y, &U, &V, &D}) require_c_contiguous(*b, "yuv_to_bgr");
        const int64_t ch = cw == w ? h : (h + 1) / 2;
        if ((cw != w && cw != (w + 1) / 2) || Y.size < w * h || U.size < cw * ch || V.size < cw * ch ||
            D.size < 3 * w * h)
          throw std::invalid_argument("yuv_to_bgr: plane sizes do not match w, h, cw");
        without_gil([&] {
          yuv_to_bgr((const uint8_t*)Y.ptr, (const uint8_t*)U.ptr, (const uint8_t*)V.ptr, (uint8_t*)D.ptr, w, h, cw);
          return 0;
        });
      },
      py::arg("y"), py::arg("u"), py::arg("v"), py::arg("dst"), py::arg("w"), py::arg("h"), py::arg("cw"));

  py::class_<ReorderIndex>(m, "ReorderIndex")
      .def(py::init<int64_t>(), py::arg("first") = 1)
      .def("push", &ReorderIndex::push)
      .def("reset", &ReorderIndex::reset)
      .def_property_readonly("next_expected", &ReorderIndex::next_expected)
      .def_property_readonly("stashed", &ReorderIndex::stashed);
}
