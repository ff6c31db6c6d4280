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

#include <malloc.h>

#include <cstdlib>
#include <map>

#include "core.h"
#include "vecenv.h"

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

// raw form (GPU featurization, ops/csrc/featurize.hip): → (env (N,3), hero (N,4), raw (N,U,8) int32, handles (N,U),
// n_allied_creep)
py::tuple featurize_batch_raw(const std::vector<py::bytes>& states, const std::vector<int>& player_ids,
                              const std::vector<int>& team_ids, const std::vector<int>& counts, int threads) {
  const size_t N = states.size();
  if (player_ids.size() != N || team_ids.size() != N) throw std::invalid_argument("length mismatch");
  if (counts.size() != 6) throw std::invalid_argument("counts must have 6 entries");
  int U = 0;
  for (int c : counts) U += c;
  py::array_t<float> env({(py::ssize_t)N, (py::ssize_t)3});
  py::array_t<float> hero({(py::ssize_t)N, (py::ssize_t)4});
  py::array_t<int32_t> raw({(py::ssize_t)N, (py::ssize_t)U, (py::ssize_t)kRawWords});
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
  float* herop = hero.mutable_data();
  int32_t* rp = raw.mutable_data();
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
          cp[i] = featurize_one_raw(w, player_ids[i], team_ids[i], counts.data(), envp + 3 * i, herop + 4 * i,
                                    rp + i * (size_t)U * kRawWords, hp + (size_t)i * U);
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
  return py::make_tuple(env, hero, raw, handles, n_creep);
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
  // the message as a uint8 numpy array that owns the popped buffer: one copy out of the ring (GIL released) and no
  // second one into a bytes object under the GIL (≈1.2 MB per whole-game rollout on the learner's decode thread)
  py::object pop_view(double timeout) {
    auto* out = new std::string();
    bool got;
    {
      py::gil_scoped_release rel;
      got = r_.pop(out, timeout);
    }
    if (!got) {
      delete out;
      return py::none();
    }
    py::capsule owner(out, [](void* p) { delete static_cast<std::string*>(p); });
    return py::array_t<uint8_t>({(py::ssize_t)out->size()}, {(py::ssize_t)1},
                                reinterpret_cast<const uint8_t*>(out->data()), owner);
  }
  // pop_view + the DCX2 trailer check in the same pass: the payload is copied out in 64 KB blocks and each block's
  // CRC-32C is taken while it is still in cache (combined per block), instead of a second full read of the message
  // by the decoder. Returns (array, ok): ok = True (DCX2, CRC matches), False (DCX2, mismatch — corrupted), None
  // (another format: the decoder checks it).
  py::object pop_checked(double timeout) {
    uint8_t* buf = nullptr;
    uint64_t n = 0;
    int ok = -1;
    bool got;
    {
      py::gil_scoped_release rel;
      got = r_.pop_with([&](const uint8_t* src, uint64_t len) {
        buf = static_cast<uint8_t*>(std::malloc(len ? len : 1));
        n = len;
        const bool dcx2 = len >= 12 && std::memcmp(src, "DCX2", 4) == 0;
        const uint64_t body = dcx2 ? len - 4 : len;
        uint32_t crc = 0;
        constexpr uint64_t kBlk = 64 << 10;
        for (uint64_t o = 0; o < len; o += kBlk) {
          const uint64_t b = std::min(kBlk, len - o);
          std::memcpy(buf + o, src + o, b);
          if (dcx2 && o < body) {
            const uint64_t c = std::min(b, body - o);
            crc = o == 0 ? crc32c_raw(buf, c) : crc32c_combine(crc, crc32c_raw(buf + o, c), c);
          }
        }
        if (dcx2) {
          uint32_t want;
          std::memcpy(&want, buf + body, 4);
          ok = crc == want ? 1 : 0;
        }
      }, timeout);
    }
    if (!got) return py::none();
    py::capsule owner(buf, [](void* p) { std::free(p); });
    py::array_t<uint8_t> arr({(py::ssize_t)n}, {(py::ssize_t)1}, buf, owner);
    return py::make_tuple(arr, ok < 0 ? py::object(py::none()) : py::object(py::bool_(ok == 1)));
  }
  // zero-copy: (uint8 array viewing the message IN the shared ring, token) — the region stays reserved until
  // release(token); the array must not be read after that. The array keeps this ring object alive.
  py::object claim(py::object self, double timeout) {
    uint64_t pos, len, token;
    bool got;
    {
      py::gil_scoped_release rel;
      got = r_.claim(&pos, &len, timeout, &token);
    }
    if (!got) return py::none();
    py::array_t<uint8_t> arr({(py::ssize_t)len}, {(py::ssize_t)1}, r_.payload(pos), self);
    return py::make_tuple(arr, token);
  }
  void set_claim_abandon(double seconds) { r_.set_claim_abandon(seconds); }
  bool claim_valid(uint64_t token) {
    py::gil_scoped_release rel;
    return r_.claim_valid(token);
  }
  void release(uint64_t token) {
    py::gil_scoped_release rel;
    r_.release(token);
  }
  void release_many(std::vector<uint64_t> tokens) {
    py::gil_scoped_release rel;
    r_.release_many(tokens.data(), tokens.size());
  }
  RingCore* core() { return &r_; }
  uint64_t size() { return r_.size(); }
  uint64_t dropped() { return r_.dropped(); }
  static void unlink(const std::string& name) { RingCore::unlink(name); }

 private:
  RingCore r_;
};

// ---- vectorised self-play runtime (vecenv.h) -----------------------------------------------------------------
template <typename T>
T* checked(py::array a, std::vector<py::ssize_t> shape, const char* what, bool writeable) {
  if (!a.dtype().is(py::dtype::of<T>())) throw std::invalid_argument(std::string(what) + ": wrong dtype");
  if (!(a.flags() & py::array::c_style)) throw std::invalid_argument(std::string(what) + ": must be C-contiguous");
  if (a.ndim() != (py::ssize_t)shape.size()) throw std::invalid_argument(std::string(what) + ": wrong rank");
  for (size_t i = 0; i < shape.size(); ++i)
    if (shape[i] >= 0 && a.shape(i) != shape[i]) throw std::invalid_argument(std::string(what) + ": wrong shape");
  if (writeable && !a.writeable()) throw std::invalid_argument(std::string(what) + ": must be writeable");
  return static_cast<T*>(a.mutable_data());
}

class PyVecEnv {
 public:
  PyVecEnv(int n_games, int mode, uint64_t seed, double max_dota_time, long rollout_size, int hidden_stride,
           int hidden_size, std::vector<int> counts, int threads, double latest_weights_prob, bool validation,
           bool fog, double start_time, std::string tag, bool stagger, bool wire, bool raw)
      : env_(make(n_games, mode, seed, max_dota_time, rollout_size, hidden_stride, hidden_size, counts, threads,
                  latest_weights_prob, validation, fog, start_time, tag, stagger, wire, raw)) {
    S_ = env_.slots();
    U_ = env_.units();
    H_ = hidden_size;
  }
  py::array_t<int32_t> begin_step() {
    std::vector<int> r;
    {
      py::gil_scoped_release rel;
      r = env_.begin_step();
    }
    return py::array_t<int32_t>((py::ssize_t)r.size(), r.data());
  }
  py::array_t<int32_t> observe_raw(py::array env, py::array hero, py::array raw, py::array handles,
                                   py::array active) {
    if (!env_.raw()) throw std::invalid_argument("observe_raw: the VecEnv was not created with raw=True");
    float* e = checked<float>(env, {S_, 3}, "env", true);
    float* hr = checked<float>(hero, {S_, 4}, "hero", true);
    int32_t* r = checked<int32_t>(raw, {S_, U_, kRawWords}, "raw", true);
    int64_t* h = checked<int64_t>(handles, {S_, U_}, "handles", true);
    uint8_t* a = checked<uint8_t>(active, {S_}, "active", true);
    std::vector<int> need;
    {
      py::gil_scoped_release rel;
      need = env_.observe_raw(e, hr, r, h, a);
    }
    return py::array_t<int32_t>((py::ssize_t)need.size(), need.data());
  }
  py::array_t<int32_t> observe_raw16(py::array env, py::array hero, py::array raw16, py::array handles,
                                     py::array active) {
    if (!env_.raw()) throw std::invalid_argument("observe_raw16: the VecEnv was not created with raw=True");
    float* e = checked<float>(env, {S_, 3}, "env", true);
    float* hr = checked<float>(hero, {S_, 4}, "hero", true);
    int32_t* r = checked<int32_t>(raw16, {S_, U_, kRaw16Words}, "raw16", true);
    int64_t* h = checked<int64_t>(handles, {S_, U_}, "handles", true);
    uint8_t* a = checked<uint8_t>(active, {S_}, "active", true);
    std::vector<int> need;
    {
      py::gil_scoped_release rel;
      need = env_.observe_raw16(e, hr, r, h, a);
    }
    return py::array_t<int32_t>((py::ssize_t)need.size(), need.data());
  }
  py::array_t<int32_t> observe(py::array env, py::array units, py::array handles, py::array active) {
    if (env_.raw()) throw std::invalid_argument("observe: the VecEnv was created with raw=True (use observe_raw)");
    float* e = checked<float>(env, {S_, 3}, "env", true);
    float* u = checked<float>(units, {S_, U_, 10}, "units", true);
    int64_t* h = checked<int64_t>(handles, {S_, U_}, "handles", true);
    uint8_t* a = checked<uint8_t>(active, {S_}, "active", true);
    std::vector<int> need;
    {
      py::gil_scoped_release rel;
      need = env_.observe(e, u, h, a);
    }
    return py::array_t<int32_t>((py::ssize_t)need.size(), need.data());
  }
  void act(py::array idx, py::array act, py::array msk, py::array logp, py::array value, py::object hidden,
           py::object hidden_slots, py::array handles, long weight_version) {
    const int A = 21 + U_;
    const int32_t* ix = checked<int32_t>(idx, {S_, 4}, "idx", false);
    const uint8_t* ac = checked<uint8_t>(act, {S_, A}, "act", false);
    const uint8_t* mk = checked<uint8_t>(msk, {S_, A}, "msk", false);
    const float* lp = checked<float>(logp, {S_}, "logp", false);
    const float* vl = checked<float>(value, {S_}, "value", false);
    const int64_t* hd = checked<int64_t>(handles, {S_, U_}, "handles", false);
    const float* hid = nullptr;
    const int* hs = nullptr;
    int nh = 0;
    if (!hidden.is_none()) {
      py::array ha = hidden.cast<py::array>(), sa = hidden_slots.cast<py::array>();
      nh = (int)sa.shape(0);
      hid = checked<float>(ha, {nh, 2, H_}, "hidden", false);
      hs = checked<int32_t>(sa, {nh}, "hidden_slots", false);
      for (int i = 0; i < nh; ++i)
        if (hs[i] < 0 || hs[i] >= S_) throw std::invalid_argument("hidden_slots out of range");
    }
    for (py::ssize_t i = 0; i < (py::ssize_t)S_ * 4; ++i)
      if ((i % 4 == 0 && (ix[i] < 0 || ix[i] > 2)) || ((i % 4 == 1 || i % 4 == 2) && (ix[i] < 0 || ix[i] > 8)))
        throw std::invalid_argument("idx: action index out of range");
    py::gil_scoped_release rel;
    env_.act(ix, ac, mk, lp, vl, hid, hs, nh, hd, weight_version);
  }
  py::list pop_rollouts() {
    std::vector<std::string> r = env_.pop_rollouts();
    py::list out;
    for (auto& b : r) out.append(py::bytes(b));
    return out;
  }
  py::list pop_results() {
    py::list out;
    for (auto& r : env_.pop_results()) out.append(py::make_tuple(r[0], r[1], r[2]));
    return out;
  }
  py::array_t<int32_t> opponent_slots() {
    std::vector<int> s = env_.opponent_slots();
    return py::array_t<int32_t>((py::ssize_t)s.size(), s.data());
  }
  int slots() const { return S_; }
  bool raw() const { return env_.raw(); }
  int players_per_game() const { return env_.players_per_game(); }
  long games_finished() const { return env_.games_finished(); }
  long steps_taken() const { return env_.steps_taken(); }
  long rollouts_sent() const { return env_.rollouts_sent(); }
  long sink_lost() const { return env_.sink_lost(); }
  // finished rollouts go straight into this ring (encoded in place by the worker threads); the ring object is kept
  // alive by this env
  void set_ring_sink(py::object ring, double timeout, bool drop_oldest) {
    ring_ref_ = ring;
    env_.set_sink(ring.cast<ShmRing&>().core(), timeout, drop_oldest);
  }
  long wire_bytes() const { return env_.wire_bytes(); }
  double dota_time(int g) const { return env_.dota_time(g); }
  int status(int g) const { return env_.status(g); }

 private:
  static VecConfig make(int n_games, int mode, uint64_t seed, double max_dota_time, long rollout_size,
                        int hidden_stride, int hidden_size, const std::vector<int>& counts, int threads,
                        double latest_weights_prob, bool validation, bool fog, double start_time,
                        const std::string& tag, bool stagger, bool wire, bool raw) {
    if (n_games < 1 || mode < 0 || mode > 3 || counts.size() != 6 || rollout_size < 1 || hidden_size < 0)
      throw std::invalid_argument("VecEnv: bad configuration");
    VecConfig c;
    c.n_games = n_games;
    c.mode = mode;
    c.seed = seed;
    c.max_dota_time = max_dota_time;
    c.rollout_size = rollout_size;
    c.hidden_stride = hidden_stride;
    c.hidden_size = hidden_size;
    for (int i = 0; i < 6; ++i) c.counts[i] = counts[i];
    c.threads = threads;
    c.latest_weights_prob = latest_weights_prob;
    c.validation = validation;
    c.fog = fog;
    c.start_time = start_time;
    c.tag = tag;
    c.stagger = stagger;
    c.wire = wire;
    c.raw = raw;
    return c;
  }
  py::object ring_ref_;     // (declared before env_: destroyed after it)
  VecEnv env_;
  int S_ = 0, U_ = 0, H_ = 0;
};

// one SimGame driven step by step with explicit orders (parity tests against env/synthetic.py)
class PySimGame {
 public:
  PySimGame(std::vector<std::tuple<int, int, int>> picks, uint64_t seed, double start_time, bool fog, double dt) {
    std::vector<Pick> p;
    for (auto& t : picks) p.push_back(Pick{std::get<0>(t), std::get<1>(t), std::get<2>(t)});
    g_.init(p, seed, start_time, fog, dt);
  }
  // orders: (player, type 0/1/2, mx, my, target handle)
  void step(std::vector<std::tuple<int, int, double, double, int64_t>> orders) {
    std::vector<SimGame::Order> o;
    for (auto& t : orders) {
      SimGame::Order x;
      x.player = std::get<0>(t);
      x.type = std::get<1>(t);
      x.mx = std::get<2>(t);
      x.my = std::get<3>(t);
      x.target = std::get<4>(t);
      o.push_back(x);
    }
    g_.step(o);
  }
  py::bytes world_bytes(int team) {
    std::string b;
    g_.world_bytes(team, b);
    return py::bytes(b);
  }
  py::tuple featurize(int team, int player_id, std::vector<int> counts) {
    World w;
    g_.world(team, w);
    int U = 0;
    for (int c : counts) U += c;
    py::array_t<float> env({(py::ssize_t)3});
    py::array_t<float> units({(py::ssize_t)U, (py::ssize_t)10});
    py::array_t<int64_t> handles({(py::ssize_t)U});
    featurize_one(w, player_id, team, counts.data(), U, env.mutable_data(), units.mutable_data(),
                  handles.mutable_data());
    return py::make_tuple(env, units, handles);
  }
  py::tuple featurize_raw(int team, int player_id, std::vector<int> counts) {
    World w;
    g_.world(team, w);
    int U = 0;
    for (int c : counts) U += c;
    py::array_t<float> env({(py::ssize_t)3});
    py::array_t<float> hero({(py::ssize_t)4});
    py::array_t<int32_t> raw({(py::ssize_t)U, (py::ssize_t)kRawWords});
    py::array_t<int64_t> handles({(py::ssize_t)U});
    featurize_one_raw(w, player_id, team, counts.data(), env.mutable_data(), hero.mutable_data(), raw.mutable_data(),
                      handles.mutable_data());
    return py::make_tuple(env, hero, raw, handles);
  }
  py::array_t<double> reward(int player_id, int team) {   // reward vs the previous call's view
    RewardView cur = reward_view(g_, player_id, team);
    py::array_t<double> r((py::ssize_t)9);
    auto it = prev_.find(player_id);
    if (it == prev_.end()) {
      std::fill(r.mutable_data(), r.mutable_data() + 9, 0.0);
    } else {
      shaped_reward(it->second, cur, r.mutable_data());
    }
    prev_[player_id] = cur;
    return r;
  }
  // (handle, unit_type, team, x, y, hp, alive, target) per unit, python dict order
  std::vector<std::tuple<int, int, int, double, double, double, bool, int>> units() const {
    std::vector<std::tuple<int, int, int, double, double, double, bool, int>> o;
    for (const SUnit& u : g_.units) o.emplace_back(u.handle, u.unit_type, u.team, u.x, u.y, u.hp, u.alive, u.target);
    return o;
  }
  double dota_time() const { return g_.dota_time; }
  int status() const { return g_.status; }

 private:
  SimGame g_;
  std::map<int, RewardView> prev_;
};

uint32_t crc32c(py::bytes b) {
  char* buf;
  py::ssize_t len;
  PYBIND11_BYTES_AS_STRING_AND_SIZE(b.ptr(), &buf, &len);
  return crc32c_raw((const uint8_t*)buf, (size_t)len);
}

// CRC-32C of the first n bytes (n < 0: all) of any contiguous buffer (bytes, memoryview, numpy), GIL released —
// the DCX2 experience-message check on the learner's stager thread runs beside the training thread
uint32_t crc32c_buf(py::buffer b, py::ssize_t n) {
  py::buffer_info info = b.request();
  const py::ssize_t total = info.size * info.itemsize;
  if (n < 0 || n > total) n = total;
  const uint8_t* p = static_cast<const uint8_t*>(info.ptr);
  py::gil_scoped_release nogil;
  return crc32c_raw(p, (size_t)n);
}

// Parallel memcpy of a job list (n, 3) int64 = (dst address, src address, bytes), GIL released: the learner's ingest
// stager packs an iteration's rollout fields (≈40 MB for 16 sequences of 1400 steps) into its pinned upload slot with
// `threads` threads instead of one numpy copy after another. Jobs are split into ≤ 1 MB pieces and dealt round-robin.
void copy_jobs(py::array_t<int64_t, py::array::c_style> jobs, int threads) {
  if (jobs.ndim() != 2 || jobs.shape(1) != 3) throw std::invalid_argument("jobs must be (n, 3) int64");
  const int64_t* j = jobs.data();
  const py::ssize_t n = jobs.shape(0);
  struct Piece { uint8_t* d; const uint8_t* s; size_t b; };
  std::vector<Piece> pcs;
  constexpr size_t kPiece = 1 << 20;
  for (py::ssize_t i = 0; i < n; ++i) {
    if (j[3 * i + 2] < 0) throw std::invalid_argument("negative byte count");
    uint8_t* d = reinterpret_cast<uint8_t*>(j[3 * i]);
    const uint8_t* s = reinterpret_cast<const uint8_t*>(j[3 * i + 1]);
    const size_t b = (size_t)j[3 * i + 2];
    for (size_t o = 0; o < b; o += kPiece) pcs.push_back({d + o, s + o, std::min(kPiece, b - o)});
  }
  py::gil_scoped_release rel;
  const int T = std::max(1, std::min<int>(threads, (int)pcs.size()));
  auto work = [&](int t) {
    for (size_t k = t; k < pcs.size(); k += T) std::memcpy(pcs[k].d, pcs[k].s, pcs[k].b);
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < T; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
}

// The stager's whole field packing in one call: for every field (dst (Lv, ...) contiguous, [src_i or None]) the
// rollouts' rows go to dst[pos[i]:pos[i+1]] — same-dtype memcpy, f64 → f32 conversion (rewards) or zero fill
// (missing field) — split into ≤ 1 MB pieces over `threads` threads with the GIL released. Replaces a Python loop
// over rollouts × fields (≈8 ms per 16 × 1400-step iteration on the node's busy CPU, most of it waiting for the GIL
// the decode, writer and main threads also need).
void pack_rows(py::list fields, py::array_t<int64_t, py::array::c_style> pos, int threads) {
  const int64_t* p = pos.data();
  const py::ssize_t n = pos.size() - 1;
  if (n < 0) throw std::invalid_argument("pos must hold n + 1 offsets");
  struct Piece { uint8_t* d; const uint8_t* s; size_t count; int kind; };   // kind 0 memcpy, 1 f64→f32, 2 zero
  std::vector<Piece> pcs;
  constexpr size_t kPiece = 1 << 20;
  for (py::handle fh : fields) {
    py::tuple f = py::reinterpret_borrow<py::tuple>(fh);
    if (f.size() != 2) throw std::invalid_argument("fields are (dst, [src...]) pairs");
    py::array dst = py::reinterpret_borrow<py::array>(f[0]);
    py::list srcs = py::reinterpret_borrow<py::list>(f[1]);
    if (!(dst.flags() & py::array::c_style) || !dst.writeable()) throw std::invalid_argument("dst must be contiguous");
    if ((py::ssize_t)srcs.size() != n) throw std::invalid_argument("one source per rollout");
    const py::ssize_t rows = dst.ndim() ? dst.shape(0) : 0;
    if (rows < p[n]) throw std::invalid_argument("dst has fewer rows than the rollouts");
    const size_t row_bytes = rows ? (size_t)dst.nbytes() / (size_t)rows : 0;
    const size_t isz = (size_t)dst.itemsize();
    uint8_t* dbase = static_cast<uint8_t*>(dst.mutable_data());
    const char dk = dst.dtype().kind();
    for (py::ssize_t i = 0; i < n; ++i) {
      const int64_t r0 = p[i], r1 = p[i + 1];
      if (r1 < r0 || r0 < 0) throw std::invalid_argument("pos must be non-decreasing");
      uint8_t* d = dbase + (size_t)r0 * row_bytes;
      const size_t bytes = (size_t)(r1 - r0) * row_bytes;
      py::handle sh = srcs[i];
      if (sh.is_none()) {
        for (size_t o = 0; o < bytes; o += kPiece) pcs.push_back({d + o, nullptr, std::min(kPiece, bytes - o), 2});
        continue;
      }
      py::array s = py::reinterpret_borrow<py::array>(sh);
      if (!(s.flags() & py::array::c_style)) throw std::invalid_argument("source arrays must be C-contiguous");
      if (s.ndim() == 0 || s.shape(0) != r1 - r0) throw std::invalid_argument("source rows != pos range");
      const char sk = s.dtype().kind();
      const size_t ssz = (size_t)s.itemsize();
      const uint8_t* sp = static_cast<const uint8_t*>(s.data());
      if (sk == dk && ssz == isz && (size_t)s.nbytes() == bytes) {
        for (size_t o = 0; o < bytes; o += kPiece) pcs.push_back({d + o, sp + o, std::min(kPiece, bytes - o), 0});
      } else if (dk == 'f' && isz == 4 && sk == 'f' && ssz == 8 && (size_t)s.nbytes() == 2 * bytes) {
        const size_t elems = bytes / 4, step = kPiece / 8;
        for (size_t e = 0; e < elems; e += step)
          pcs.push_back({d + 4 * e, sp + 8 * e, std::min(step, elems - e), 1});
      } else {
        throw std::invalid_argument("source dtype / size does not match its destination field");
      }
    }
  }
  py::gil_scoped_release rel;
  const int T = std::max(1, std::min<int>(threads, (int)pcs.size()));
  auto work = [&](int t) {
    for (size_t k = t; k < pcs.size(); k += T) {
      const Piece& q = pcs[k];
      if (q.kind == 0) {
        std::memcpy(q.d, q.s, q.count);
      } else if (q.kind == 2) {
        std::memset(q.d, 0, q.count);
      } else {
        const double* s = reinterpret_cast<const double*>(q.s);
        float* d = reinterpret_cast<float*>(q.d);
        for (size_t e = 0; e < q.count; ++e) d[e] = (float)s[e];
      }
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < T; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
}

}  // namespace

// glibc malloc for the actor runtime's allocation pattern: every step appends to per-player trajectories (≈2 MB
// per whole-game player) and every finished game encodes multi-MB rollouts that Python frees right after the
// publish. With the default (dynamic mmap threshold, 128 KB trim) those blocks cycle through mmap / munmap, and the
// page faults of 12 worker threads serialise on the process's address-space lock: measured on the synthetic engine
// (6 threads, 1024 games) observe + act 4.5 → 2.3 µs per player-step with a fixed 32 MB mmap threshold and a 1 GB
// trim threshold (freed memory stays in the arenas and is reused without faults). DCA_MALLOC_TUNE=0 keeps the
// defaults.
static bool tune_malloc() {
  const char* e = std::getenv("DCA_MALLOC_TUNE");
  if (e && e[0] == '0') return false;
  return mallopt(M_MMAP_THRESHOLD, 32 << 20) == 1 && mallopt(M_TRIM_THRESHOLD, 1 << 30) == 1;
}

PYBIND11_MODULE(_native, m) {
  m.doc() = "dotaclient_amd native actor runtime (protobuf featurizer, shm ring, crc32c)";
  m.attr("MALLOC_TUNED") = tune_malloc();
  m.def("featurize_batch", &featurize_batch, py::arg("states"), py::arg("player_ids"), py::arg("team_ids"),
        py::arg("counts"), py::arg("threads") = 4,
        "Decode CMsgBotWorldState bytes and featurize for (player, team): returns env, units, handles, n_allied_creep");
  m.def("featurize_batch_raw", &featurize_batch_raw, py::arg("states"), py::arg("player_ids"), py::arg("team_ids"),
        py::arg("counts"), py::arg("threads") = 4,
        "featurize_batch's raw form for GPU featurization: returns env, hero, raw (N,U,8) int32, handles, "
        "n_allied_creep");
  m.attr("RAW_WORDS") = kRawWords;
  m.def("pack_raw16", [](py::array_t<int32_t, py::array::c_style> raw) {
    if (raw.ndim() < 1 || raw.shape(raw.ndim() - 1) != kRawWords) throw std::invalid_argument("pack_raw16: (..., 8)");
    std::vector<py::ssize_t> shape(raw.shape(), raw.shape() + raw.ndim());
    shape.back() = kRaw16Words;
    py::array_t<int32_t> out(shape);
    const py::ssize_t n = raw.size() / kRawWords;
    raw_to_raw16(raw.data(), (int)n, out.mutable_data());
    return out;
  }, py::arg("raw"), "the 16-byte (binary16) form of raw unit records (fp8 policy step staging)");
  m.def("crc32c", &crc32c);
  m.def("copy_jobs", &copy_jobs, py::arg("jobs"), py::arg("threads") = 4,
        "memcpy a (n, 3) int64 job list of (dst address, src address, bytes) on `threads` threads (GIL released)");
  m.def("pack_rows", &pack_rows, py::arg("fields"), py::arg("pos"), py::arg("threads") = 4,
        "pack per-rollout rows of every (dst, [src or None]) field into dst[pos[i]:pos[i+1]] (memcpy, f64->f32, "
        "zero fill) on `threads` threads, GIL released");
  m.def("crc32c_buf", &crc32c_buf, py::arg("buf"), py::arg("n") = -1,
        "CRC-32C of the first n bytes of a contiguous buffer (GIL released)");
  py::class_<PyVecEnv>(m, "VecEnv")
      .def(py::init<int, int, uint64_t, double, long, int, int, std::vector<int>, int, double, bool, bool, double,
                    std::string, bool, bool, bool>(),
           py::arg("n_games"), py::arg("mode") = 0, py::arg("seed") = 0, py::arg("max_dota_time") = 600.0,
           py::arg("rollout_size") = (long)1 << 40, py::arg("hidden_stride") = 0, py::arg("hidden_size") = 0,
           py::arg("counts") = std::vector<int>{1, 5, 16, 16, 1, 1}, py::arg("threads") = 8,
           py::arg("latest_weights_prob") = 1.0, py::arg("validation") = false, py::arg("fog") = true,
           py::arg("start_time") = -10.0, py::arg("tag") = std::string("vec"), py::arg("stagger") = false,
           py::arg("wire") = false, py::arg("raw") = false)
      .def("begin_step", &PyVecEnv::begin_step)
      .def("observe", &PyVecEnv::observe, py::arg("env"), py::arg("units"), py::arg("handles"), py::arg("active"))
      .def("observe_raw", &PyVecEnv::observe_raw, py::arg("env"), py::arg("hero"), py::arg("raw"), py::arg("handles"),
           py::arg("active"))
      .def("observe_raw16", &PyVecEnv::observe_raw16, py::arg("env"), py::arg("hero"), py::arg("raw16"),
           py::arg("handles"), py::arg("active"))
      .def_property_readonly("raw", [](const PyVecEnv& e) { return e.raw(); })
      .def("act", &PyVecEnv::act, py::arg("idx"), py::arg("act"), py::arg("msk"), py::arg("logp"), py::arg("value"),
           py::arg("hidden"), py::arg("hidden_slots"), py::arg("handles"), py::arg("weight_version"))
      .def("pop_rollouts", &PyVecEnv::pop_rollouts)
      .def("pop_results", &PyVecEnv::pop_results)
      .def("opponent_slots", &PyVecEnv::opponent_slots)
      .def_property_readonly("slots", &PyVecEnv::slots)
      .def_property_readonly("players_per_game", &PyVecEnv::players_per_game)
      .def_property_readonly("games_finished", &PyVecEnv::games_finished)
      .def_property_readonly("steps_taken", &PyVecEnv::steps_taken)
      .def_property_readonly("rollouts_sent", &PyVecEnv::rollouts_sent)
      .def_property_readonly("sink_lost", &PyVecEnv::sink_lost)
      .def("set_ring_sink", &PyVecEnv::set_ring_sink, py::arg("ring"), py::arg("timeout") = -1.0,
           py::arg("drop_oldest") = true)
      .def_property_readonly("wire_bytes", &PyVecEnv::wire_bytes)
      .def("dota_time", &PyVecEnv::dota_time)
      .def("status", &PyVecEnv::status);
  py::class_<PySimGame>(m, "SimGame")
      .def(py::init<std::vector<std::tuple<int, int, int>>, uint64_t, double, bool, double>(), py::arg("picks"),
           py::arg("seed"), py::arg("start_time") = -10.0, py::arg("fog") = true, py::arg("dt") = 0.5)
      .def("step", &PySimGame::step)
      .def("featurize", &PySimGame::featurize)
      .def("featurize_raw", &PySimGame::featurize_raw)
      .def("world_bytes", &PySimGame::world_bytes)
      .def("reward", &PySimGame::reward)
      .def("units", &PySimGame::units)
      .def_property_readonly("dota_time", &PySimGame::dota_time)
      .def_property_readonly("status", &PySimGame::status);
  py::class_<ShmRing>(m, "ShmRing")
      .def(py::init<const std::string&, uint64_t, bool>(), py::arg("name"), py::arg("capacity") = 1 << 26,
           py::arg("create") = true)
      .def("push", &ShmRing::push, py::arg("msg"), py::arg("timeout") = -1.0, py::arg("drop_oldest") = false)
      .def("pop", &ShmRing::pop, py::arg("timeout") = -1.0)
      .def("pop_view", &ShmRing::pop_view, py::arg("timeout") = -1.0)
      .def("pop_checked", &ShmRing::pop_checked, py::arg("timeout") = -1.0)
      .def("claim", [](py::object self, double timeout) { return self.cast<ShmRing&>().claim(self, timeout); },
           py::arg("timeout") = -1.0)
      .def("release", &ShmRing::release, py::arg("token"))
      .def("release_many", &ShmRing::release_many, py::arg("tokens"))
      .def("set_claim_abandon", &ShmRing::set_claim_abandon, py::arg("seconds"))
      .def("claim_valid", &ShmRing::claim_valid, py::arg("token"),
           "whether a zero-copy claim still owns its region (False once abandoned and reclaimed)")
      .def("size", &ShmRing::size)
      .def("dropped", &ShmRing::dropped)
      .def_static("unlink", &ShmRing::unlink);
}
