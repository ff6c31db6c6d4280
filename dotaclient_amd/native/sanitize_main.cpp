// Sanitizer driver for the native actor runtime core (core.h) — SURVEY §5 "race detection / sanitizers": the host
// code runs under AddressSanitizer + UndefinedBehaviorSanitizer (build kind "asan") or ThreadSanitizer ("tsan").
//
//   sanitize <seed_file> [iterations]
//
// 1. decoder: every seed message (length-prefixed CMsgBotWorldState wire bytes written by the test from the synthetic
//    environment) must parse and featurize; then `iterations` random mutations (bit flips, byte overwrites,
//    truncations, splices, random insertions) must either parse or throw std::runtime_error — never read or write out
//    of bounds (ASan) or hit undefined behaviour (UBSan).
// 2. ring: 4 producer and 4 consumer threads move 40 000 checksummed messages of random sizes through a small
//    (wrapping) shared-memory ring, plus a drop-oldest phase; every message must arrive exactly once and intact
//    (TSan checks the locking).
// 3. crc32c known-answer test ("123456789" → 0xE3069283).
// Exit status 0 = all checks passed.
#include <cstdio>
#include <fstream>
#include <iterator>
#include <random>
#include <set>

#include "core.h"

using namespace dca_native;

static int fail(const char* what) {
  std::fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

static std::vector<std::string> read_seeds(const char* path) {
  std::ifstream f(path, std::ios::binary);
  std::string all((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  std::vector<std::string> out;
  size_t p = 0;
  while (p + 4 <= all.size()) {
    uint32_t n;
    std::memcpy(&n, all.data() + p, 4);
    p += 4;
    if (p + n > all.size()) break;
    out.emplace_back(all.data() + p, n);
    p += n;
  }
  return out;
}

static int check_decoder(const std::vector<std::string>& seeds, int iters) {
  const int counts[6] = {1, 5, 16, 16, 1, 1};
  const int U = 40;
  std::vector<float> env(3), units(U * 10);
  std::vector<int64_t> handles(U);
  for (const std::string& s : seeds) {
    World w;
    parse_world((const uint8_t*)s.data(), s.size(), w);
    if (w.units.empty()) return fail("seed without units");
    int pid = -1, team = 2;
    for (const Unit& u : w.units)
      if (u.unit_type == HERO) { pid = u.player_id; team = (int)u.team_id; break; }
    if (featurize_one(w, pid, team, counts, U, env.data(), units.data(), handles.data()) < 0)
      return fail("seed: hero not found");
  }
  std::mt19937_64 rng(1234);
  size_t parsed = 0, rejected = 0;
  for (int it = 0; it < iters; ++it) {
    std::string m = seeds[rng() % seeds.size()];
    const int edits = 1 + (int)(rng() % 4);
    for (int e = 0; e < edits && !m.empty(); ++e) {
      switch (rng() % 5) {
        case 0: m[rng() % m.size()] ^= (char)(1u << (rng() % 8)); break;               // bit flip
        case 1: m[rng() % m.size()] = (char)(rng() & 0xff); break;                     // byte overwrite
        case 2: m.resize(rng() % m.size()); break;                                     // truncation
        case 3: {                                                                      // splice of another seed
          const std::string& o = seeds[rng() % seeds.size()];
          const size_t a = rng() % m.size(), b = rng() % o.size();
          m = m.substr(0, a) + o.substr(b);
          break;
        }
        default: {                                                                     // random insertion
          std::string r(1 + rng() % 16, '\0');
          for (char& c : r) c = (char)(rng() & 0xff);
          m.insert(rng() % (m.size() + 1), r);
        }
      }
    }
    // copy into an exactly-sized heap buffer so ASan sees any read past the end
    std::vector<uint8_t> buf(m.begin(), m.end());
    try {
      World w;
      parse_world(buf.data(), buf.size(), w);
      int pid = 0, team = 2;
      for (const Unit& u : w.units)
        if (u.unit_type == HERO) { pid = u.player_id; team = (int)u.team_id; break; }
      featurize_one(w, pid, team, counts, U, env.data(), units.data(), handles.data());
      ++parsed;
    } catch (const std::runtime_error&) {
      ++rejected;
    }
  }
  std::printf("decoder: %zu seeds ok, %d mutations (%zu parsed, %zu rejected)\n", seeds.size(), iters, parsed,
              rejected);
  return 0;
}

static uint64_t fnv(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}

static int check_ring() {
  const std::string name = "/dca_sanitize_" + std::to_string((long)getpid());
  RingCore::unlink(name);
  constexpr int P = 4, C = 4, PER = 10000;
  std::atomic<int> bad{0};
  std::vector<std::vector<uint64_t>> got(C);
  {
    RingCore ring(name, 1 << 16, true);                 // 64 KB: wraps constantly
    std::vector<std::thread> th;
    for (int p = 0; p < P; ++p)
      th.emplace_back([&, p] {
        std::mt19937 rng(p);
        for (int i = 0; i < PER; ++i) {
          std::string m(8 + rng() % 600, '\0');
          const uint64_t id = ((uint64_t)p << 32) | (uint64_t)i;
          std::memcpy(&m[0], &id, 8);
          for (size_t k = 8; k < m.size(); ++k) m[k] = (char)((id * 31 + k) & 0xff);
          if (!ring.push(m.data(), m.size(), 5.0, false)) bad.fetch_add(1);
        }
      });
    std::atomic<int> remaining{P * PER};
    for (int c = 0; c < C; ++c)
      th.emplace_back([&, c] {
        std::string m;
        while (remaining.load() > 0) {
          if (!ring.pop(&m, 0.05)) continue;
          remaining.fetch_sub(1);
          uint64_t id;
          if (m.size() < 8) { bad.fetch_add(1); continue; }
          std::memcpy(&id, m.data(), 8);
          for (size_t k = 8; k < m.size(); ++k)
            if ((unsigned char)m[k] != (unsigned char)((id * 31 + k) & 0xff)) { bad.fetch_add(1); break; }
          got[c].push_back(id);
        }
      });
    for (auto& t : th) t.join();
    if (ring.size() != 0) return fail("ring not drained");
    // drop-oldest: a full ring keeps accepting, the oldest messages go
    const std::string big(1000, 'x');
    for (int i = 0; i < 200; ++i)
      if (!ring.push(big.data(), big.size(), 0.0, true)) return fail("drop-oldest push refused");
    if (ring.dropped() == 0) return fail("drop-oldest never dropped");
  }
  RingCore::unlink(name);
  std::set<uint64_t> seen;
  size_t total = 0;
  for (auto& v : got) {
    total += v.size();
    seen.insert(v.begin(), v.end());
  }
  if (bad.load() != 0) return fail("corrupted / refused ring messages");
  if (total != (size_t)P * PER || seen.size() != (size_t)P * PER) return fail("ring lost or duplicated messages");
  std::printf("ring: %d messages through %d producers / %d consumers intact\n", P * PER, P, C);
  return 0;
}

// A writer skipped as abandoned must not be able to commit into the region a NEW producer reserved at the same ring
// position with the same size (commit checks the reservation's monotonic token, not the position + size word).
static int check_stale_commit() {
  const std::string name = "/dca_sanitize_sc_" + std::to_string((long)getpid());
  RingCore::unlink(name);
  {
    RingCore ring(name, 224, true);       // two 112-byte slots (8-byte word + 104-byte padded payload of 100 bytes)
    ring.set_writer_abandon(0.05);
    const std::string a(100, 'a'), b(100, 'b'), c(100, 'c');
    uint64_t pa, ta, pos, len, tok;
    if (!ring.reserve(100, 1.0, false, &pa, &ta)) return fail("stale-commit: reserve A");
    // writer A stalls; the consumer skips its region after the abandonment time (nothing else to claim)
    if (ring.claim(&pos, &len, 0.3, &tok)) return fail("stale-commit: claimed an uncommitted message");
    // B1 fills the second slot and is consumed; B2 wraps to A's position with A's size
    if (!ring.push(b.data(), b.size(), 1.0, false)) return fail("stale-commit: push B1");
    std::string m;
    if (!ring.pop(&m, 1.0) || m != b) return fail("stale-commit: pop B1");
    uint64_t p2, t2;
    if (!ring.reserve(100, 1.0, false, &p2, &t2)) return fail("stale-commit: reserve B2");
    if (p2 != pa || t2 == ta) return fail("stale-commit: B2 did not reuse A's position");
    std::memcpy(ring.wpayload(pa), a.data(), a.size());   // A's late copy ...
    if (ring.commit(pa, 100, ta)) return fail("stale-commit: A's late commit was accepted");
    if (ring.claim(&pos, &len, 0.0, &tok)) return fail("stale-commit: B2's half-written region became ready");
    std::memcpy(ring.wpayload(p2), c.data(), c.size());
    if (!ring.commit(p2, 100, t2)) return fail("stale-commit: B2's commit refused");
    if (!ring.pop(&m, 1.0) || m != c) return fail("stale-commit: B2's message");
  }
  RingCore::unlink(name);
  std::printf("ring: stale commit of a skipped writer refused\n");
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) return fail("usage: sanitize <seed_file> [iterations]");
  const int iters = argc > 2 ? std::atoi(argv[2]) : 20000;
  const std::vector<std::string> seeds = read_seeds(argv[1]);
  if (seeds.empty()) return fail("no seeds");
  if (check_decoder(seeds, iters)) return 1;
  if (check_ring()) return 1;
  if (check_stale_commit()) return 1;
  const char* kat = "123456789";
  if (crc32c_raw((const uint8_t*)kat, 9) != 0xE3069283u) return fail("crc32c known answer");
  std::printf("crc32c ok\nall sanitizer checks passed\n");
  return 0;
}
