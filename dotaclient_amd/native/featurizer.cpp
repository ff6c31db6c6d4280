// Native actor-side runtime: protobuf wire decoder + featurizer, shared-memory experience ring, crc32c.
//
// * featurize_batch: CMsgBotWorldState wire bytes → (env (N,3), units (N,U,10), handles (N,U)) for a batch of
//   (observation, player) pairs, multithreaded, GIL released. Hand-rolled proto2 wire decoding of exactly the fields
//   the featurizer reads; field numbers mirror dotaclient_amd/protos/schema.py (checked by tests). Semantics are the
//   reference's agent.py:456-637 (unit_separation, unit_matrix, env features, handle validity rules) and are tested
//   against the python featurizer.
// * ShmRing: multi-producer / multi-consumer byte-message ring in POSIX shared memory with a process-shared robust
//   mutex and condition variables — the node-local replacement for the RabbitMQ experience queue (bounded, blocking
//   with timeouts).
// * crc32c: SSE4.2 (hardware) CRC32-C for TensorBoard event records.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "core.h"

namespace py = pybind11;

namespace {

using namespace dca_native;

py::tuple featurize_batch(const std::vector<py::bytes>& states, const std::vector<int>& player_ids,
                          const std::vector<int>& team_ids, const std::vector<int>& counts, int threads) {
  const size_t N = states.size();
  if (player_ids.size() != N || team_ids.size() != N) throw std::invalid_argument("length mismatch");
  if (counts.size() != 6) throw std::invalid_argument("counts must have 6 entries");
  int U = 0;
  for (int c : counts) U += c;
  py::array_t<float> env({(py::ssize_t)N, (py::ssize_t)3});
  py::array_t<float> units({(py::ssize_t)N, (py::ssize_t)U, (py::ssize_t)10});
  py::array_t<int64_t> handles({(py::ssize_t)N, (py::ssize_t)U});
  py::array_t<int32_t> n_creep({(py::ssize_t)N});
  std::vector<std::string_view> views(N);
  for (size_t i = 0; i < N; ++i) {
    char* buf;
    py::ssize_t len;
    PYBIND11_BYTES_AS_STRING_AND_SIZE(states[i].ptr(), &buf, &len);
    views[i] = std::string_view(buf, (size_t)len);
  }
  float* envp = env.mutable_data();
  float* up = units.mutable_data();
  int64_t* hp = handles.mutable_data();
  int32_t* cp = n_creep.mutable_data();
  std::vector<std::string> errors(N);
  {
    py::gil_scoped_release rel;
    const int T = std::max(1, std::min<int>(threads, (int)N));
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (size_t i; (i = next.fetch_add(1)) < N;) {
        try {
          World w;
          parse_world((const uint8_t*)views[i].data(), views[i].size(), w);
          cp[i] = featurize_one(w, player_ids[i], team_ids[i], counts.data(), U, envp + 3 * i, up + (size_t)i * U * 10,
                                hp + (size_t)i * U);
        } catch (const std::exception& e) {
          errors[i] = e.what();
        }
      }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < T; ++t) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
  }
  for (size_t i = 0; i < N; ++i)
    if (!errors[i].empty()) throw std::runtime_error("observation " + std::to_string(i) + ": " + errors[i]);
  return py::make_tuple(env, units, handles, n_creep);
}

// pybind face of the ring: the GIL is released around every blocking call
class ShmRing {
 public:
  ShmRing(const std::string& name, uint64_t capacity, bool create) : r_(name, capacity, create) {}
  bool push(py::bytes msg, double timeout, bool drop_oldest) {
    char* buf;
    py::ssize_t len;
    PYBIND11_BYTES_AS_STRING_AND_SIZE(msg.ptr(), &buf, &len);
    py::gil_scoped_release rel;
    return r_.push(buf, (size_t)len, timeout, drop_oldest);
  }
  py::object pop(double timeout) {
    std::string out;
    bool got;
    {
      py::gil_scoped_release rel;
      got = r_.pop(&out, timeout);
    }
    if (!got) return py::none();
    return py::bytes(out);
  }
  uint64_t size() { return r_.size(); }
  uint64_t dropped() { return r_.dropped(); }
  static void unlink(const std::string& name) { RingCore::unlink(name); }

 private:
  RingCore r_;
};

uint32_t crc32c(py::bytes b) {
  char* buf;
  py::ssize_t len;
  PYBIND11_BYTES_AS_STRING_AND_SIZE(b.ptr(), &buf, &len);
  return crc32c_raw((const uint8_t*)buf, (size_t)len);
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "dotaclient_amd native actor runtime (protobuf featurizer, shm ring, crc32c)";
  m.def("featurize_batch", &featurize_batch, py::arg("states"), py::arg("player_ids"), py::arg("team_ids"),
        py::arg("counts"), py::arg("threads") = 4,
        "Decode CMsgBotWorldState bytes and featurize for (player, team): returns env, units, handles, n_allied_creep");
  m.def("crc32c", &crc32c);
  py::class_<ShmRing>(m, "ShmRing")
      .def(py::init<const std::string&, uint64_t, bool>(), py::arg("name"), py::arg("capacity") = 1 << 26,
           py::arg("create") = true)
      .def("push", &ShmRing::push, py::arg("msg"), py::arg("timeout") = -1.0, py::arg("drop_oldest") = false)
      .def("pop", &ShmRing::pop, py::arg("timeout") = -1.0)
      .def("size", &ShmRing::size)
      .def("dropped", &ShmRing::dropped)
      .def_static("unlink", &ShmRing::unlink);
}
