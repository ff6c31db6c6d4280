// Native actor-side runtime core (no Python): proto2 wire decoder + featurizer, shared-memory MPMC ring, crc32c.
// Included by the pybind11 module (featurizer.cpp) and by the sanitizer driver (sanitize_main.cpp), which runs it
// under AddressSanitizer / UndefinedBehaviorSanitizer / ThreadSanitizer: decoder fuzzing on malformed bytes, the
// ring under concurrent producers and consumers. See featurizer.cpp for the reference semantics.
#pragma once
#include <errno.h>
#include <fcntl.h>
#include <nmmintrin.h>
#include <pthread.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

namespace dca_native {


// ============================================================================================================
// proto2 wire decoding
// ============================================================================================================
struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  bool ok() const { return p < e; }
  uint64_t varint() {
    uint64_t v = 0;
    int s = 0;
    while (p < e) {
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return v;
      s += 7;
      if (s > 63) break;
    }
    throw std::runtime_error("malformed varint");
  }
  float f32() {
    if (e - p < 4) throw std::runtime_error("truncated fixed32");
    float f;
    std::memcpy(&f, p, 4);
    p += 4;
    return f;
  }
  std::string_view bytes() {
    const uint64_t n = varint();
    if ((uint64_t)(e - p) < n) throw std::runtime_error("truncated length-delimited field");
    std::string_view s((const char*)p, n);
    p += n;
    return s;
  }
  void skip(int wt) {
    switch (wt) {
      case 0: varint(); break;
      case 1: p += 8; break;
      case 2: bytes(); break;
      case 5: p += 4; break;
      default: throw std::runtime_error("unsupported wire type");
    }
    if (p > e) throw std::runtime_error("truncated field");
  }
};

// proto2 wire encoding (the synthetic engine's CMsgBotWorldState on the wire, vecenv.h SimGame::world_bytes):
// fields are appended in field-number order, so the bytes equal python protobuf's SerializeToString of the same
// message with the same fields set
struct Writer {
  std::string* o;
  void varint(uint64_t v) {
    while (v >= 0x80) { o->push_back((char)(uint8_t)(v | 0x80)); v >>= 7; }
    o->push_back((char)(uint8_t)v);
  }
  void tag(int f, int wt) { varint(((uint64_t)f << 3) | (uint64_t)wt); }
  void u64(int f, uint64_t v) { tag(f, 0); varint(v); }
  void i32(int f, int32_t v) { tag(f, 0); varint((uint64_t)(int64_t)v); }   // negative: 10-byte sign extension
  void boolean(int f, bool v) { tag(f, 0); o->push_back(v ? 1 : 0); }
  void f32(int f, float v) { tag(f, 5); char b[4]; std::memcpy(b, &v, 4); o->append(b, 4); }
  void bytes(int f, std::string_view s) { tag(f, 2); varint(s.size()); o->append(s.data(), s.size()); }
};

enum UnitTypeE { HERO = 1, CREEP_HERO = 2, LANE_CREEP = 3, TOWER = 6 };

struct Unit {
  uint32_t handle = 0;
  int unit_type = 0;
  std::string_view name;
  uint32_t team_id = 0;
  float x = 0, y = 0, z = 0;
  bool is_alive = false;
  int32_t player_id = 0;
  float facing = 0;
  int32_t health = 0, health_max = 0;
  int32_t attack_range = 0;
  uint32_t attack_target = 0;
  int32_t anim = 0;
  bool invuln = false, attack_immune = false;
  std::vector<uint32_t> attack_casters;   // incoming tracking projectiles with is_attack
};

struct World {
  float dota_time = 0;
  std::vector<Unit> units;
};

void parse_vector(std::string_view s, Unit& u) {
  Reader r{(const uint8_t*)s.data(), (const uint8_t*)s.data() + s.size()};
  while (r.ok()) {
    const uint64_t k = r.varint();
    const int f = (int)(k >> 3), wt = (int)(k & 7);
    if (wt == 5 && f == 1) u.x = r.f32();
    else if (wt == 5 && f == 2) u.y = r.f32();
    else if (wt == 5 && f == 3) u.z = r.f32();
    else r.skip(wt);
  }
}

void parse_projectile(std::string_view s, Unit& u) {
  Reader r{(const uint8_t*)s.data(), (const uint8_t*)s.data() + s.size()};
  uint32_t caster = 0;
  bool is_attack = false;
  while (r.ok()) {
    const uint64_t k = r.varint();
    const int f = (int)(k >> 3), wt = (int)(k & 7);
    if (wt == 0 && f == 1) caster = (uint32_t)r.varint();
    else if (wt == 0 && f == 4) is_attack = r.varint() != 0;
    else r.skip(wt);
  }
  if (is_attack) u.attack_casters.push_back(caster);
}

void parse_unit(std::string_view s, Unit& u) {
  Reader r{(const uint8_t*)s.data(), (const uint8_t*)s.data() + s.size()};
  while (r.ok()) {
    const uint64_t k = r.varint();
    const int f = (int)(k >> 3), wt = (int)(k & 7);
    if (wt == 0) {
      const uint64_t v = r.varint();
      switch (f) {
        case 1: u.handle = (uint32_t)v; break;
        case 2: u.unit_type = (int)v; break;
        case 4: u.team_id = (uint32_t)v; break;
        case 7: u.is_alive = v != 0; break;
        case 8: u.player_id = (int32_t)v; break;
        case 20: u.health = (int32_t)v; break;
        case 21: u.health_max = (int32_t)v; break;
        case 30: u.attack_range = (int32_t)v; break;
        case 35: u.attack_target = (uint32_t)v; break;
        case 40: u.anim = (int32_t)v; break;
        case 50: u.invuln = v != 0; break;
        case 51: u.attack_immune = v != 0; break;
        default: break;
      }
    } else if (wt == 5) {
      const float v = r.f32();
      if (f == 11) u.facing = v;
    } else if (wt == 2) {
      const std::string_view b = r.bytes();
      if (f == 3) u.name = b;
      else if (f == 6) parse_vector(b, u);
      else if (f == 70) parse_projectile(b, u);
    } else {
      r.skip(wt);
    }
  }
}

void parse_world(const uint8_t* data, size_t n, World& w) {
  Reader r{data, data + n};
  while (r.ok()) {
    const uint64_t k = r.varint();
    const int f = (int)(k >> 3), wt = (int)(k & 7);
    if (wt == 5 && f == 3) {
      w.dota_time = r.f32();
    } else if (wt == 2 && f == 11) {
      w.units.emplace_back();
      parse_unit(r.bytes(), w.units.back());
    } else {
      r.skip(wt);
    }
  }
}

// ============================================================================================================
// featurizer (reference agent.py:496-637)
// ============================================================================================================
constexpr double kMapHalf = 7000.0;

bool ends_with(std::string_view s, std::string_view suf) {
  return s.size() >= suf.size() && s.substr(s.size() - suf.size()) == suf;
}

float attacking(const Unit& a, const Unit& t) {
  if (a.attack_target == t.handle) return 1.f;
  for (uint32_t c : t.attack_casters)
    if (c == a.handle) return 1.f;
  return 0.f;
}

void unit_rows(const std::vector<const Unit*>& list, const Unit& hero, bool only_self, int max_units, float* m,
               int64_t* handles) {
  for (int i = 0; i < max_units; ++i) {
    handles[i] = -1;
    for (int k = 0; k < 10; ++k) m[i * 10 + k] = 0.f;
  }
  int i = 0;
  const uint32_t opp = hero.team_id == 2 ? 3 : (hero.team_id == 3 ? 2 : 0);
  for (const Unit* up : list) {
    const Unit& u = *up;
    if (!u.is_alive) continue;
    if (only_self && u.handle != hero.handle) continue;
    if (i >= max_units) break;
    // every feature in double, cast once (the python featurizer's arithmetic, agent.py:521-532), so the native
    // path is bit-identical to featurizer.py rather than merely close
    const double hp = u.health_max ? (double)u.health / (double)u.health_max : 0.0;
    const double dx = (double)hero.x - (double)u.x, dy = (double)hero.y - (double)u.y;
    const double dist = std::sqrt(dx * dx + dy * dy);
    const double tau = 2.0 * 3.14159265358979323846;
    float* r = m + i * 10;
    r[0] = (float)(1.0 - hp);
    r[1] = (float)((double)u.x / kMapHalf);
    r[2] = (float)((double)u.y / kMapHalf);
    r[3] = (float)((double)u.z / 512.0 - 0.5);
    r[4] = (float)(dist / kMapHalf - 0.5);
    double sf, cf;
    sincos((double)u.facing * tau / 360.0, &sf, &cf);      // one argument reduction for both (same values)
    r[5] = (float)sf;
    r[6] = (float)cf;
    r[7] = (dist <= (double)hero.attack_range ? 1.f : 0.f) - 0.5f;
    r[8] = attacking(u, hero) - 0.5f;
    r[9] = attacking(hero, u) - 0.5f;
    int64_t h = (int64_t)u.handle;
    if (u.invuln || u.attack_immune) h = -1;
    else if (u.team_id == opp && u.unit_type == TOWER && u.anim == 1500) h = -1;
    else if (u.team_id == hero.team_id && u.unit_type == TOWER) h = -1;
    else if (u.team_id == hero.team_id && hp > 0.5) h = -1;
    handles[i] = h;
    ++i;
  }
}

// the observing hero and its six unit blocks in slot order (agent.py:456-493, 575-611); returns the number of allied
// lane creeps (for the creep-spawn sanity check), or -1 when the hero is missing. The lists are per-thread scratch.
int separate(const World& w, int player_id, const int* counts, const Unit*& hero,
             const std::vector<const Unit*>* (&lists)[6]) {
  hero = nullptr;
  for (const Unit& u : w.units)
    if (u.unit_type == HERO && u.player_id == player_id) { hero = &u; break; }
  if (!hero) return -1;
  // per-thread scratch lists (capacity reused across calls: no allocation per observation)
  thread_local std::vector<const Unit*> ah, eh, anhc, enhc, ac, ec, at, et, s5;
  ah.clear(); eh.clear(); anhc.clear(); enhc.clear(); ac.clear(); ec.clear(); at.clear(); et.clear();
  for (const Unit& u : w.units) {
    const bool ally = u.team_id == hero->team_id;
    switch (u.unit_type) {
      case HERO: (ally ? ah : eh).push_back(&u); break;
      case CREEP_HERO: (ally ? anhc : enhc).push_back(&u); break;   // non-hero creeps first, lane creeps after
      case LANE_CREEP: (ally ? ac : ec).push_back(&u); break;
      case TOWER:
        if (ends_with(u.name, "1_mid")) (ally ? at : et).push_back(&u);
        break;
      default: break;
    }
  }
  anhc.insert(anhc.end(), ac.begin(), ac.end());
  enhc.insert(enhc.end(), ec.begin(), ec.end());
  if (counts[0] > 1) {   // 5v5: self first, then teammates
    s5.clear();
    s5.push_back(hero);
    for (const Unit* u : ah)
      if (u->player_id != player_id) s5.push_back(u);
    ah.swap(s5);
  }
  lists[0] = &ah; lists[1] = &eh; lists[2] = &anhc; lists[3] = &enhc; lists[4] = &at; lists[5] = &et;
  return (int)ac.size();
}

void env_row(const World& w, int team_id, float* env) {
  env[0] = (float)((double)w.dota_time / 1200.0);
  env[1] = (float)std::sin((double)w.dota_time * (2.0 * 3.14159265358979323846) / 60.0);
  env[2] = team_id == 3 ? -0.2f : 0.2f;
}

// returns number of allied lane creeps (for the creep-spawn sanity check), or -1 when the hero is missing
int featurize_one(const World& w, int player_id, int team_id, const int* counts, int U, float* env, float* units,
                  int64_t* handles) {
  const Unit* hero;
  const std::vector<const Unit*>* lists[6];
  const int nc = separate(w, player_id, counts, hero, lists);
  if (nc < 0) return -1;
  env_row(w, team_id, env);
  int off = 0;
  for (int t = 0; t < 6; ++t) {
    unit_rows(*lists[t], *hero, t == 0 && counts[0] == 1, counts[t], units + off * 10, handles + off);
    off += counts[t];
  }
  (void)U;
  return nc;
}

// ---- raw unit records for GPU featurization (ops/csrc/featurize.hip, features/raw.py): 8 words per slot —
// x, y, z, facing (f32) | 1 − health / health_max (f32, double then rounded once), handle (−1: not targetable), flags
// (bit 0 present, 1 attacks the hero, 2 the hero attacks it), 0 — and a hero record (x, y, attack range, 0). The
// slot selection, validity rules and attack cross-references are unit_rows'; the distance / sincos / range arithmetic
// is left to the device. (Handles are stored as int32: the engines' handles are far below 2^31.)
constexpr int kRawWords = 8;

void unit_rows_raw(const std::vector<const Unit*>& list, const Unit& hero, bool only_self, int max_units, int32_t* r,
                   int64_t* handles) {
  std::memset(r, 0, sizeof(int32_t) * kRawWords * (size_t)max_units);
  for (int i = 0; i < max_units; ++i) handles[i] = -1;
  int i = 0;
  const uint32_t opp = hero.team_id == 2 ? 3 : (hero.team_id == 3 ? 2 : 0);
  for (const Unit* up : list) {
    const Unit& u = *up;
    if (!u.is_alive) continue;
    if (only_self && u.handle != hero.handle) continue;
    if (i >= max_units) break;
    const double hp = u.health_max ? (double)u.health / (double)u.health_max : 0.0;
    int32_t* w = r + i * kRawWords;
    const float rel = (float)(1.0 - hp);
    std::memcpy(w + 0, &u.x, 4);
    std::memcpy(w + 1, &u.y, 4);
    std::memcpy(w + 2, &u.z, 4);
    std::memcpy(w + 3, &u.facing, 4);
    std::memcpy(w + 4, &rel, 4);
    int64_t h = (int64_t)u.handle;
    if (u.invuln || u.attack_immune) h = -1;
    else if (u.team_id == opp && u.unit_type == TOWER && u.anim == 1500) h = -1;
    else if (u.team_id == hero.team_id && u.unit_type == TOWER) h = -1;
    else if (u.team_id == hero.team_id && hp > 0.5) h = -1;
    w[5] = (int32_t)h;
    w[6] = 1 | (attacking(u, hero) != 0.f ? 2 : 0) | (attacking(hero, u) != 0.f ? 4 : 0);
    handles[i] = h;
    ++i;
  }
}

// IEEE binary16 of a float, round to nearest even (the F16C / numpy astype(float16) result; no F16C dependency)
inline uint16_t f32_to_f16(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const uint32_t ax = x & 0x7fffffffu;
  if (ax >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (ax > 0x7f800000u ? 0x200u : 0u));   // inf / nan
  if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);                                       // overflow → inf
  if (ax < 0x38800000u) {                                                                          // subnormal / 0
    if (ax < 0x33000000u) return (uint16_t)sign;
    const uint32_t m = (ax & 0x7fffffu) | 0x800000u;
    const int e = (int)(ax >> 23);
    const int shift = 126 - e;                      // 14..24
    uint32_t h = m >> (shift);
    const uint32_t rem = m & ((1u << shift) - 1u), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (h & 1u))) ++h;
    return (uint16_t)(sign | h);
  }
  uint32_t h = ((ax - 0x38000000u) >> 13);
  const uint32_t rem = ax & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
  return (uint16_t)(sign | h);
}

// 16-byte form of a raw record for the fp8 policy step (its features are fp16 anyway): x | y, z | facing, 1 − hp |
// flags as binary16 pairs, then the handle (ops/csrc/featurize.hip featurize_raw16_kernel, features/raw.py pack_raw16)
constexpr int kRaw16Words = 4;
inline void raw_to_raw16(const int32_t* r, int U, int32_t* o) {
  for (int u = 0; u < U; ++u, r += kRawWords, o += kRaw16Words) {
    float f[5];
    std::memcpy(f, r, sizeof(f));
    o[0] = (int32_t)((uint32_t)f32_to_f16(f[0]) | ((uint32_t)f32_to_f16(f[1]) << 16));
    o[1] = (int32_t)((uint32_t)f32_to_f16(f[2]) | ((uint32_t)f32_to_f16(f[3]) << 16));
    o[2] = (int32_t)((uint32_t)f32_to_f16(f[4]) | ((uint32_t)(r[6] & 0xffff) << 16));
    o[3] = r[5];
  }
}

// raw form of featurize_one: env (3), hero (4), raw (U, 8) and the host's handles (U) (the action decoder's targets)
int featurize_one_raw(const World& w, int player_id, int team_id, const int* counts, float* env, float* hero4,
                      int32_t* raw, int64_t* handles) {
  const Unit* hero;
  const std::vector<const Unit*>* lists[6];
  const int nc = separate(w, player_id, counts, hero, lists);
  if (nc < 0) return -1;
  env_row(w, team_id, env);
  hero4[0] = hero->x;
  hero4[1] = hero->y;
  hero4[2] = (float)hero->attack_range;
  hero4[3] = 0.f;
  int off = 0;
  for (int t = 0; t < 6; ++t) {
    unit_rows_raw(*lists[t], *hero, t == 0 && counts[0] == 1, counts[t], raw + (size_t)off * kRawWords,
                  handles + off);
    off += counts[t];
  }
  return nc;
}

// ============================================================================================================
// Shared-memory MPMC ring
//
// Payload copies run OUTSIDE the process-shared mutex: a producer reserves its region under the lock, copies, and
// commits; a consumer claims the oldest committed message under the lock, copies it out, and releases its region.
// (Copying under the lock serialised every push against every pop: with ≈1.35 MB whole-game rollouts at ≈1 750 per
// second each way the lock was held most of the time, and two dedicated threads moved 2 850 messages/s.) Each message
// is a u64 word + the payload padded to 8 bytes; the word holds the state in its top byte and the length below
// (~0 marks "wrap to the start"). Regions are reclaimed oldest-first once their consumer is done (free_off), so
// the producers' space limit is free_off, not head; drop_oldest drops only what it can reclaim.
// ============================================================================================================
struct RingHeader {
  uint64_t magic;
  uint64_t capacity;   // bytes of the data area
  uint64_t head;       // next message to claim (monotonic offset)
  uint64_t tail;       // next write offset (monotonic)
  uint64_t count;      // messages between head and tail (being written or ready)
  uint64_t dropped;
  uint64_t free_off;   // oldest byte still in use; [free_off, head) holds messages being read or done
  uint64_t stuck_off;  // a claimed region seen blocking the reclaim at free_off, and since when (CLOCK_MONOTONIC ns)
  uint64_t stuck_ns;
  uint64_t wstuck_off; // the message at head seen still being written, and since when (CLOCK_MONOTONIC ns): shared by
  uint64_t wstuck_ns;  // every consumer call, so short polling claims add up to the writer-abandonment time
  pthread_mutex_t mu;
  pthread_cond_t not_empty;
  pthread_cond_t not_full;
};
constexpr uint64_t kMagic = 0x444341524e473034ull;   // "DCARNG04"

void deadline_in(double seconds, timespec& ts) {
  clock_gettime(CLOCK_REALTIME, &ts);
  const double s = std::max(0.0, seconds);
  const long sec = (long)s;
  long nsec = ts.tv_nsec + (long)((s - sec) * 1e9);
  ts.tv_sec += sec + nsec / 1000000000L;
  ts.tv_nsec = nsec % 1000000000L;
}

class RingCore {
 public:
  // message states (top byte of the word)
  static constexpr uint64_t kWriting = 1, kReady = 2, kReading = 3, kDone = 4;
  static constexpr uint64_t kLenMask = (1ull << 56) - 1;
  static constexpr uint64_t kWrap = ~0ull;
  // a producer that reserved a region and never committed it (it died mid-copy) is skipped after this long
  // (set_writer_abandon: tests)
  double writer_abandon_s_ = 30.0;
  void set_writer_abandon(double s) { writer_abandon_s_ = s; }
  // a claimed region that blocks the reclaim (its consumer died, or holds it) is given up after this long when a
  // producer needs the space (set_claim_abandon: tests); its late release is then ignored (claim tokens are
  // monotonic offsets, below free_off once reclaimed)
  double claim_abandon_s_ = 60.0;
  void set_claim_abandon(double s) { claim_abandon_s_ = s; }

  RingCore(const std::string& name, uint64_t capacity, bool create) : name_(name) {
    const int flags = create ? (O_CREAT | O_RDWR) : O_RDWR;
    fd_ = shm_open(name.c_str(), flags, 0600);
    if (fd_ < 0) throw std::runtime_error("shm_open failed: " + std::string(strerror(errno)));
    size_ = sizeof(RingHeader) + capacity;
    if (create && ftruncate(fd_, (off_t)size_) != 0) throw std::runtime_error("ftruncate failed");
    if (!create) {
      struct stat st;
      fstat(fd_, &st);
      size_ = (size_t)st.st_size;
    }
    base_ = (uint8_t*)mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
    if (base_ == MAP_FAILED) throw std::runtime_error("mmap failed");
    hdr_ = (RingHeader*)base_;
    data_ = base_ + sizeof(RingHeader);
    if (create) {
      std::memset(hdr_, 0, sizeof(RingHeader));
      hdr_->capacity = capacity;
      pthread_mutexattr_t ma;
      pthread_mutexattr_init(&ma);
      pthread_mutexattr_setpshared(&ma, PTHREAD_PROCESS_SHARED);
      pthread_mutexattr_setrobust(&ma, PTHREAD_MUTEX_ROBUST);
      pthread_mutex_init(&hdr_->mu, &ma);
      pthread_condattr_t ca;
      pthread_condattr_init(&ca);
      pthread_condattr_setpshared(&ca, PTHREAD_PROCESS_SHARED);
      pthread_cond_init(&hdr_->not_empty, &ca);
      pthread_cond_init(&hdr_->not_full, &ca);
      hdr_->magic = kMagic;
    } else if (hdr_->magic != kMagic) {
      throw std::runtime_error("not a dotaclient_amd shm ring (or one of another version)");
    }
  }
  ~RingCore() {
    if (base_ && base_ != MAP_FAILED) munmap(base_, size_);
    if (fd_ >= 0) close(fd_);
  }

  void lock() {
    const int r = pthread_mutex_lock(&hdr_->mu);
    if (r == EOWNERDEAD) pthread_mutex_consistent(&hdr_->mu);   // a process died holding the lock
  }
  void unlock() { pthread_mutex_unlock(&hdr_->mu); }

  bool push(const char* msg_data, size_t msg_size, double timeout, bool drop_oldest) {
    uint64_t pos, tok;
    if (!reserve(msg_size, timeout, drop_oldest, &pos, &tok)) return false;
    std::memcpy(data_ + pos + 8, msg_data, msg_size);     // outside the lock
    return commit(pos, msg_size, tok);
  }

  // producer side in two steps: reserve a region for msg_size bytes (writable at wpayload(pos) without the lock),
  // then commit it with the reservation's token (the message's monotonic offset). False from reserve: no space
  // within the timeout; false from commit: the region was given up as abandoned (writer_abandon_s_) and the message
  // is lost.
  uint8_t* wpayload(uint64_t pos) { return data_ + pos + 8; }
  // true when msg_size bytes can never fit (reserve would throw): callers on worker threads count such a message as
  // lost instead of letting the exception escape the thread
  bool too_large(size_t msg_size) const { return padded(msg_size) + 8 > hdr_->capacity || msg_size > kLenMask; }
  bool reserve(size_t msg_size, double timeout, bool drop_oldest, uint64_t* pos_out, uint64_t* token_out) {
    const uint64_t need = padded(msg_size);
    if (need + 8 > hdr_->capacity || msg_size > kLenMask) throw std::invalid_argument("message larger than ring");
    timespec ts;
    if (timeout > 0) deadline_in(timeout, ts);
    lock();
    while (true) {
      const uint64_t cap = hdr_->capacity;
      const uint64_t used = hdr_->tail - hdr_->free_off;
      const uint64_t pos = hdr_->tail % cap;
      const uint64_t to_end = cap - pos;
      const uint64_t want = (to_end < need) ? to_end + need : need;
      if (used + want <= cap) {
        if (to_end < need) {
          if (to_end >= 8) set_word(pos, kWrap);
          hdr_->tail += to_end;
        }
        const uint64_t p = hdr_->tail % cap;
        set_word(p, (kWriting << 56) | (uint64_t)msg_size);
        *token_out = hdr_->tail;
        hdr_->tail += need;
        hdr_->count += 1;
        unlock();
        *pos_out = p;
        return true;
      }
      if (drop_oldest && drop_head_locked()) continue;
      if (abandon_stuck_claim_locked()) continue;
      if (timeout == 0.0) { unlock(); return false; }
      // bounded waits (≤ 1 s) so a claim abandoned meanwhile is noticed without a wake-up
      timespec wt;
      deadline_in(1.0, wt);
      if (timeout > 0 && (ts.tv_sec < wt.tv_sec || (ts.tv_sec == wt.tv_sec && ts.tv_nsec < wt.tv_nsec))) wt = ts;
      if (pthread_cond_timedwait(&hdr_->not_full, &hdr_->mu, &wt) == ETIMEDOUT && timeout > 0) {
        timespec now;
        clock_gettime(CLOCK_REALTIME, &now);
        if (now.tv_sec > ts.tv_sec || (now.tv_sec == ts.tv_sec && now.tv_nsec >= ts.tv_nsec)) {
          unlock();
          return false;
        }
      }
    }
  }
  // The token, not the ring position, identifies the message: a writer skipped as abandoned (writer_abandon_s_) has
  // its region reclaimed, and a NEW producer may reserve the same position with the same size — the old writer's late
  // commit must not mark that half-written region ready. A skipped message lies below head (consumers moved past
  // it); a live one never does.
  bool commit(uint64_t pos, size_t msg_size, uint64_t token) {
    lock();
    const bool ok = token >= hdr_->head && token % hdr_->capacity == pos &&
                    word_at(pos) == ((kWriting << 56) | (uint64_t)msg_size);   // (else given up as abandoned)
    if (ok) set_word(pos, (kReady << 56) | (uint64_t)msg_size);
    pthread_cond_broadcast(&hdr_->not_empty);
    pthread_cond_broadcast(&hdr_->not_full);   // a drop_oldest producer may be waiting for this commit
    unlock();
    return ok;
  }

  bool pop(std::string* out, double timeout) {
    return pop_with([out](const uint8_t* src, uint64_t len) { if (out) out->assign((const char*)src, len); }, timeout);
  }

  // pop the oldest committed message, handing (payload, length) to fn OUTSIDE the lock (fn copies it out)
  template <class F>
  bool pop_with(F&& fn, double timeout) {
    uint64_t pos, len, tok;
    if (!claim(&pos, &len, timeout, &tok)) return false;
    fn(data_ + pos + 8, len);
    release(tok);
    return true;
  }

  // zero-copy consumption: claim the oldest committed message (its region stays reserved, readable at
  // payload(pos), until release(token)); releases may come in any order, space is reclaimed oldest-first. The token
  // is the message's monotonic offset: a release that arrives after its region was abandoned and reclaimed
  // (token < free_off) is ignored instead of touching whatever message occupies that position now.
  const uint8_t* payload(uint64_t pos) const { return data_ + pos + 8; }
  // whether the claim `token` still owns its region: false once it was abandoned (claim_abandon_s_) and reclaimed —
  // a producer may then have overwritten the bytes. A zero-copy consumer checks this AFTER copying a claimed message
  // out (the CRC was checked at claim time) and drops what it copied when the claim is gone.
  bool claim_valid(uint64_t token) {
    lock();
    bool ok = token >= hdr_->free_off && token < hdr_->head;
    if (ok) {
      uint64_t off = token;
      const uint64_t pos = resolve(off);
      ok = off == token && (word_at(pos) >> 56) == kReading;
    }
    unlock();
    return ok;
  }
  void release(uint64_t token) { release_many(&token, 1); }
  // several claimed regions given back under ONE lock acquisition and one wake-up of the producers
  void release_many(const uint64_t* tokens, size_t n) {
    lock();
    bool any = false;
    for (size_t i = 0; i < n; ++i) {
      uint64_t off = tokens[i];
      if (off < hdr_->free_off || off >= hdr_->head) continue;     // reclaimed (abandoned) or never claimed
      const uint64_t pos = resolve(off);
      const uint64_t w = word_at(pos);
      if ((w >> 56) == kReading) {
        set_word(pos, (kDone << 56) | (w & kLenMask));
        any = true;
      }
    }
    if (any) {
      reclaim_locked();
      pthread_cond_broadcast(&hdr_->not_full);
    }
    unlock();
  }
  bool claim(uint64_t* pos_out, uint64_t* len_out, double timeout, uint64_t* token_out = nullptr) {
    timespec ts;
    if (timeout > 0) deadline_in(timeout, ts);
    lock();
    while (true) {
      if (hdr_->count > 0) {
        uint64_t off = hdr_->head;
        const uint64_t pos = resolve(off);
        hdr_->head = off;               // (past a wrap: the message after it exists, count > 0)
        const uint64_t w = word_at(pos), st = w >> 56, len = w & kLenMask;
        if (st == kReady) {
          set_word(pos, (kReading << 56) | len);
          hdr_->head = off + padded(len);
          hdr_->count -= 1;
          unlock();
          *pos_out = pos;
          *len_out = len;
          if (token_out) *token_out = off;
          return true;
        }
        // the oldest message is still being written: wait for its commit; a producer that never commits (it died
        // mid-copy) is skipped after writer_abandon_s_ — measured across calls (the header's wstuck clock), since
        // consumers poll in short claims — and its late commit then fails (commit checks the token against head)
        if (writer_stuck_locked(off)) {
          set_word(pos, (kDone << 56) | len);
          hdr_->head = off + padded(len);
          hdr_->count -= 1;
          hdr_->dropped += 1;
          hdr_->wstuck_ns = 0;
          reclaim_locked();
          pthread_cond_broadcast(&hdr_->not_full);
          continue;
        }
      }
      if (timeout == 0.0) break;
      // bounded waits while a writer is mid-copy, so the abandonment clock above is re-checked
      timespec wt;
      if (hdr_->count > 0) {
        deadline_in(std::min(1.0, std::max(0.01, writer_abandon_s_)), wt);
        if (timeout > 0 && (ts.tv_sec < wt.tv_sec || (ts.tv_sec == wt.tv_sec && ts.tv_nsec < wt.tv_nsec))) wt = ts;
      } else if (timeout > 0) {
        wt = ts;
      }
      int r;
      if (hdr_->count == 0 && timeout < 0) r = pthread_cond_wait(&hdr_->not_empty, &hdr_->mu);
      else r = pthread_cond_timedwait(&hdr_->not_empty, &hdr_->mu, &wt);
      if (r == ETIMEDOUT && timeout > 0) {
        timespec now;
        clock_gettime(CLOCK_REALTIME, &now);
        if (now.tv_sec > ts.tv_sec || (now.tv_sec == ts.tv_sec && now.tv_nsec >= ts.tv_nsec)) {
          // one last look (a commit may have landed with the timeout, or the writer's time ran out)
          if (hdr_->count > 0) {
            uint64_t off = hdr_->head;
            const uint64_t pos = resolve(off);
            const uint64_t st = word_at(pos) >> 56;
            if (st == kReady || (st == kWriting && writer_stuck_locked(off, false))) continue;
          }
          break;
        }
      }
    }
    unlock();
    return false;
  }

  uint64_t size() { lock(); const uint64_t c = hdr_->count; unlock(); return c; }
  uint64_t dropped() { return hdr_->dropped; }
  static void unlink(const std::string& name) { shm_unlink(name.c_str()); }

 private:
  static uint64_t padded(uint64_t len) { return 8 + ((len + 7) & ~7ull); }
  uint64_t word_at(uint64_t pos) const { uint64_t w; std::memcpy(&w, data_ + pos, 8); return w; }
  void set_word(uint64_t pos, uint64_t w) { std::memcpy(data_ + pos, &w, 8); }
  // data position of the message at monotonic offset `off`, moving `off` past a wrap (marker or < 8 bytes left)
  uint64_t resolve(uint64_t& off) const {
    const uint64_t cap = hdr_->capacity, pos = off % cap;
    if (cap - pos < 8 || word_at(pos) == kWrap) {
      off += cap - pos;
      return 0;
    }
    return pos;
  }
  // whether the message being written at monotonic offset `off` (the head) has been for writer_abandon_s_; starts
  // its clock on first sight (`arm`)
  bool writer_stuck_locked(uint64_t off, bool arm = true) {
    timespec now;
    clock_gettime(CLOCK_MONOTONIC, &now);
    const uint64_t ns = (uint64_t)now.tv_sec * 1000000000ull + (uint64_t)now.tv_nsec;
    if (hdr_->wstuck_off != off || hdr_->wstuck_ns == 0) {
      if (arm) {
        hdr_->wstuck_off = off;
        hdr_->wstuck_ns = ns;
      }
      return false;
    }
    return (double)(ns - hdr_->wstuck_ns) * 1e-9 > writer_abandon_s_;
  }
  // a claimed region at free_off that has blocked the reclaim for claim_abandon_s_ (the same region, seen by the
  // producers waiting for space): given up — marked done and counted as dropped — so a consumer that died holding
  // claims cannot stop the node's actors for good
  bool abandon_stuck_claim_locked() {
    if (hdr_->free_off >= hdr_->head) return false;
    uint64_t off = hdr_->free_off;
    const uint64_t pos = resolve(off);
    const uint64_t w = word_at(pos);
    if ((w >> 56) != kReading) return false;
    timespec now;
    clock_gettime(CLOCK_MONOTONIC, &now);
    const uint64_t ns = (uint64_t)now.tv_sec * 1000000000ull + (uint64_t)now.tv_nsec;
    if (hdr_->stuck_off != off || hdr_->stuck_ns == 0) {
      hdr_->stuck_off = off;
      hdr_->stuck_ns = ns;
      return false;
    }
    if ((double)(ns - hdr_->stuck_ns) * 1e-9 < claim_abandon_s_) return false;
    set_word(pos, (kDone << 56) | (w & kLenMask));
    hdr_->dropped += 1;
    hdr_->stuck_ns = 0;
    reclaim_locked();
    return true;
  }
  // reclaim the finished regions at the old end: [free_off, head) holds messages being read or done
  void reclaim_locked() {
    const uint64_t cap = hdr_->capacity;
    while (hdr_->free_off < hdr_->head) {
      const uint64_t pos = hdr_->free_off % cap;
      if (cap - pos < 8) { hdr_->free_off += cap - pos; continue; }
      const uint64_t w = word_at(pos);
      if (w == kWrap) { hdr_->free_off += cap - pos; continue; }
      if ((w >> 56) != kDone) break;
      hdr_->free_off += padded(w & kLenMask);
    }
  }
  // drop_oldest: discard the oldest committed message (not one still being written) — only when that frees space:
  // with an older message still claimed (zero-copy consumers hold regions for a whole staging pass) the dropped
  // region could not be reclaimed, and a full ring would drop every new message while the consumer, short of one
  // more rollout to finish its batch, waits forever. The producer then waits for the release instead.
  bool drop_head_locked() {
    if (hdr_->count == 0) return false;
    reclaim_locked();
    if (hdr_->free_off != hdr_->head) return false;
    uint64_t off = hdr_->head;
    const uint64_t pos = resolve(off);
    const uint64_t w = word_at(pos);
    if ((w >> 56) != kReady) return false;
    hdr_->head = off;
    set_word(pos, (kDone << 56) | (w & kLenMask));
    hdr_->head = off + padded(w & kLenMask);
    hdr_->count -= 1;
    hdr_->dropped += 1;
    reclaim_locked();
    return true;
  }

  std::string name_;
  int fd_ = -1;
  size_t size_ = 0;
  uint8_t* base_ = nullptr;
  RingHeader* hdr_ = nullptr;
  uint8_t* data_ = nullptr;
};

// ============================================================================================================
inline uint32_t crc32c_serial(const uint8_t* p, size_t n) {
  uint64_t crc = 0xFFFFFFFFu;
  while (n >= 8) { uint64_t v; std::memcpy(&v, p, 8); crc = _mm_crc32_u64(crc, v); p += 8; n -= 8; }
  while (n--) crc = _mm_crc32_u8((uint32_t)crc, *p++);
  return (uint32_t)crc ^ 0xFFFFFFFFu;
}

// crc(A ‖ B) from crc(A), crc(B) and |B|: crc(A) times x^(8·|B|) mod P, with x^(8·|B|) from a table of x^(2^k)
// by square-and-multiply (zlib ≥ 1.2.12's multmodp / x2nmodp; Castagnoli polynomial, reflected 0x82F63B78, bit 31
// = x^0). The earlier GF(2)-matrix form (32×32 operator squared log₂|B| times) cost ≈47 µs per combine — two per
// rollout message on both the actor (encode) and the learner (check): most of a 700 KB message's CRC time.
inline uint32_t crc32c_multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ 0x82F63B78u : b >> 1;
  }
  return p;
}
struct Crc32cX2n {
  uint32_t t[32];
  Crc32cX2n() {
    uint32_t p = 1u << 30;                 // x^1
    t[0] = p;
    for (int n = 1; n < 32; ++n) t[n] = p = crc32c_multmodp(p, p);
  }
};
inline uint32_t crc32c_x2nmodp(size_t n, unsigned k) {   // x^(n·2^k) mod P
  static const Crc32cX2n tab;
  uint32_t p = 1u << 31;                   // x^0
  while (n) {
    if (n & 1) p = crc32c_multmodp(tab.t[k & 31], p);
    n >>= 1;
    ++k;
  }
  return p;
}
inline uint32_t crc32c_combine(uint32_t crc1, uint32_t crc2, size_t len2) {
  if (len2 == 0) return crc1;
  return crc32c_multmodp(crc32c_x2nmodp(len2, 3), crc1) ^ crc2;
}

// CRC-32C: three independent crc32 chains over thirds of the buffer (the instruction's 3-cycle latency otherwise
// caps one chain at a third of its throughput), joined by crc32c_combine
inline uint32_t crc32c_raw(const uint8_t* p, size_t n) {
  if (n < (size_t)3 << 16) return crc32c_serial(p, n);
  const size_t third = (n / 3) & ~(size_t)7;
  const uint8_t *a = p, *b = p + third, *c = p + 2 * third;
  uint64_t ca = 0xFFFFFFFFu, cb = 0xFFFFFFFFu, cc = 0xFFFFFFFFu;
  for (size_t i = 0; i < third; i += 8) {
    uint64_t va, vb, vc;
    std::memcpy(&va, a + i, 8);
    std::memcpy(&vb, b + i, 8);
    std::memcpy(&vc, c + i, 8);
    ca = _mm_crc32_u64(ca, va);
    cb = _mm_crc32_u64(cb, vb);
    cc = _mm_crc32_u64(cc, vc);
  }
  const size_t rest = n - 3 * third;     // tail of the last part
  const uint8_t* t = c + third;
  for (size_t i = 0; i + 8 <= rest; i += 8) { uint64_t v; std::memcpy(&v, t + i, 8); cc = _mm_crc32_u64(cc, v); }
  for (size_t i = rest & ~(size_t)7; i < rest; ++i) cc = _mm_crc32_u8((uint32_t)cc, t[i]);
  const uint32_t fa = (uint32_t)ca ^ 0xFFFFFFFFu, fb = (uint32_t)cb ^ 0xFFFFFFFFu, fc = (uint32_t)cc ^ 0xFFFFFFFFu;
  return crc32c_combine(crc32c_combine(fa, fb, third), fc, third + rest);
}

}  // namespace dca_native
