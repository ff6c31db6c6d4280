// Native vectorised self-play runtime: N synthetic 1v1-mid / 5v5 games stepped in lockstep on host threads, with
// the actor's per-step work fused in — observation → World → featurize (featurize_one), shaped reward, trajectory
// canvas, trajectory recording, action decoding, the simulator step, rollout triggers and DCX1 encoding.
//
// Reference behaviour reproduced (agent.py:744-852): per observation each team observes, every
// controlled player gets its shaped reward (agent.py:118-158) and featurized input (agent.py:496-637), acts
// (agent.py:665-709), the game advances after both teams acted; zero-sum ``enemy`` term (829-833); rollouts every
// ``rollout_size`` steps and at game end (835-847), end-state win/loss/−0.25 (325-337); only players on the latest
// weights roll out (445-448).
//
// The simulator is a bit-for-bit port of dotaclient_amd/env/synthetic.py (the oracle, tested step by step):
// CPython's MT19937 (init_by_array seeding, 53-bit random(), uniform = a + (b-a)·random()), dict-ordered units,
// double arithmetic in the same order (compiled with -ffp-contract=off), protobuf field conversions (float32 positions
// and facing, int32 health) where the python path goes through a CMsgBotWorldState.
//
// Both teams are observed at once: the reference's observe(D) happens before the engine advances, so it does not
// depend on R's action — one batched policy step serves both teams of every game.
#pragma once
#include <array>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "core.h"

namespace dca_native {

// ============================================================================================================
// CPython's random.Random (MT19937, random_seed for non-negative ints, random(), uniform())
// ============================================================================================================
struct PyRandom {
  uint32_t mt[624];
  int mti = 625;

  void init_genrand(uint32_t s) {
    mt[0] = s;
    for (mti = 1; mti < 624; mti++) mt[mti] = 1812433253U * (mt[mti - 1] ^ (mt[mti - 1] >> 30)) + (uint32_t)mti;
  }
  void init_by_array(const uint32_t* key, size_t klen) {
    init_genrand(19650218U);
    size_t i = 1, j = 0;
    for (size_t k = 624 > klen ? 624 : klen; k; k--) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525U)) + key[j] + (uint32_t)j;
      i++;
      j++;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
      if (j >= klen) j = 0;
    }
    for (size_t k = 623; k; k--) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941U)) - (uint32_t)i;
      i++;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
    }
    mt[0] = 0x80000000U;
    mti = 624;
  }
  void seed(uint64_t n) {   // random.Random(n), n >= 0: little-endian 32-bit words of n (one word for 0)
    uint32_t key[2] = {(uint32_t)n, (uint32_t)(n >> 32)};
    init_by_array(key, key[1] ? 2 : 1);
  }
  uint32_t genrand() {
    static const uint32_t mag01[2] = {0x0U, 0x9908b0dfU};
    uint32_t y;
    if (mti >= 624) {
      int kk;
      for (kk = 0; kk < 624 - 397; kk++) {
        y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
        mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 0x1U];
      }
      for (; kk < 623; kk++) {
        y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
        mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 0x1U];
      }
      y = (mt[623] & 0x80000000U) | (mt[0] & 0x7fffffffU);
      mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 0x1U];
      mti = 0;
    }
    y = mt[mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
  }
  double random() {
    const uint32_t a = genrand() >> 5, b = genrand() >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
  }
  double uniform(double a, double b) { return a + (b - a) * random(); }
};

// ============================================================================================================
// constants (dotaclient_amd/constants.py, env/synthetic.py)
// ============================================================================================================
enum { TEAM_R = 2, TEAM_D = 3 };
enum { ST_OK = 0, ST_RADIANT_WIN = 1, ST_DIRE_WIN = 2 };
enum { CTRL_IDLE = 0, CTRL_DEFAULT = 1, CTRL_CONTROLLED = 2 };
enum { HERO_SNIPER = 35, HERO_NEVERMORE = 11 };
enum Kind { K_HERO, K_TOWER1, K_TOWER2, K_MELEE, K_RANGED };

constexpr double kVision = 1800.0, kXpRadius = 1300.0;
constexpr int kXpToReach[26] = {0,     0,     230,   600,   1080,  1680,  2300,  2940,  3600,
                                4280,  5080,  5900,  6740,  7640,  8865,  10115, 11390, 12690,
                                14015, 15415, 16905, 18405, 20155, 22155, 24405, 26905};

inline void fountain(int t, double& x, double& y) { x = t == TEAM_R ? -6700.0 : 6600.0; y = t == TEAM_R ? -6200.0 : 6000.0; }
inline void creep_spawn(int t, double& x, double& y) { x = t == TEAM_R ? -4700.0 : 4000.0; y = t == TEAM_R ? -4300.0 : 3600.0; }
inline void t1_mid(int t, double& x, double& y) { x = t == TEAM_R ? -1544.0 : 524.0; y = t == TEAM_R ? -1408.0 : 652.0; }
inline void ancient(int t, double& x, double& y) { x = t == TEAM_R ? -5400.0 : 5200.0; y = t == TEAM_R ? -5000.0 : 4700.0; }
inline int opp(int t) { return t == TEAM_R ? TEAM_D : TEAM_R; }

// level_from_total_xp (constants.py)
inline void level_from_total_xp(double total_xp, int& level, int& need) {
  level = 1;
  for (int l = 1; l < 26; ++l)
    if (total_xp >= kXpToReach[l]) level = l;
  if (level >= 25) { level = 25; need = 0; return; }
  need = (int)(kXpToReach[level + 1] - total_xp);   // python int(): truncation
}
inline int total_xp_from(int level, int need) {   // get_total_xp (agent.py:110-115)
  if (level >= 25) return kXpToReach[25];
  return kXpToReach[level] + ((kXpToReach[level + 1] - kXpToReach[level]) - need);
}
// python float % for a positive divisor
inline double pymod(double a, double b) {
  double m = std::fmod(a, b);
  if (m != 0.0) {
    if ((b < 0) != (m < 0)) m += b;
  } else {
    m = std::copysign(0.0, b);
  }
  return m;
}
inline double hyp(double dx, double dy) { return std::sqrt(dx * dx + dy * dy); }
inline double facing_to(double dy, double dx) { return pymod(std::atan2(dy, dx) * (180.0 / 3.141592653589793) + 360.0, 360.0); }

// ============================================================================================================
// simulator (env/synthetic.py SyntheticGame)
// ============================================================================================================
struct SUnit {
  int handle = 0, unit_type = 0, kind = 0, team = 0;
  double x = 0, y = 0, hp = 0, hp_max = 0, damage = 0, attack_range = 0, attack_period = 0, speed = 0;
  int player_id = -1;
  double mana = 0, mana_max = 0;
  int level = 1;
  double total_xp = 0, facing = 0;
  bool alive = true;
  double cooldown = 0;
  int target = 0, last_hits = 0, denies = 0;
  double respawn_at = 0;
  bool has_move = false;
  double mx = 0, my = 0;
  int control = CTRL_IDLE;
  std::vector<int> projectiles;   // caster handles of incoming attack projectiles (this observation)
  bool invulnerable = false;
  int last_attacker_player = -1;
};

struct PStats {
  int player_id, team_id, hero_id, kills = 0, deaths = 0;
};

struct Pick {
  int team, hero_id, control;
};

class SimGame {
 public:
  std::vector<SUnit> units;       // python dict insertion order
  std::vector<SUnit> keep_;       // step() scratch (reused capacity)
  std::vector<PStats> players;    // dict keyed by player_id, insertion order
  PyRandom rng;
  double dt = 0.5, dota_time = -10.0;
  bool fog = true;
  int next_handle = 100, status = ST_OK, n_steps = 0;
  bool has_wave = false;
  long last_wave = 0;

  void init(const std::vector<Pick>& picks, uint64_t seed, double start_time, bool fog_of_war, double dt_) {
    units.clear();
    players.clear();
    rng.seed(seed);
    dt = dt_;
    dota_time = start_time;
    fog = fog_of_war;
    next_handle = 100;
    status = ST_OK;
    n_steps = 0;
    has_wave = false;
    int pid[4] = {0, 0, 0, 5};
    for (const Pick& p : picks) {
      const int team = p.team;
      const int id = pid[team]++;
      const bool controlled = p.control != CTRL_IDLE;
      double fx, fy;
      fountain(team, fx, fy);
      if (controlled) {
        double tx, ty;
        t1_mid(team, tx, ty);
        const double d = team == TEAM_R ? 400.0 : -400.0;
        fx = tx - d + rng.uniform(-100, 100);
        fy = ty - d + rng.uniform(-100, 100);
      }
      SUnit u;
      u.handle = ++next_handle;
      u.unit_type = HERO;
      u.kind = K_HERO;
      u.team = team;
      u.x = fx; u.y = fy; u.hp = 600.0; u.hp_max = 600.0; u.damage = 55.0; u.attack_range = 500.0;
      u.attack_period = 1.6; u.speed = 315.0; u.player_id = id; u.mana = 290.0; u.mana_max = 290.0;
      u.facing = team == TEAM_R ? 45.0 : 225.0;
      u.control = p.control;
      units.push_back(u);
      players.push_back(PStats{id, team, p.hero_id});
    }
    for (int team : {TEAM_R, TEAM_D}) {
      double tx, ty;
      t1_mid(team, tx, ty);
      SUnit t;
      t.handle = ++next_handle; t.unit_type = TOWER; t.kind = K_TOWER1; t.team = team;
      t.x = tx; t.y = ty; t.hp = 1800.0; t.hp_max = 1800.0; t.damage = 100.0; t.attack_range = 700.0;
      t.attack_period = 1.0; t.speed = 0.0;
      units.push_back(t);
      SUnit t2 = t;
      t2.handle = ++next_handle; t2.kind = K_TOWER2; t2.x = tx * 2.2; t2.y = ty * 2.2; t2.invulnerable = true;
      units.push_back(t2);
    }
  }

  SUnit* find(int handle) {
    for (SUnit& u : units)
      if (u.handle == handle) return &u;
    return nullptr;
  }
  PStats* player(int pid) {
    for (PStats& p : players)
      if (p.player_id == pid) return &p;
    return nullptr;
  }
  SUnit* hero_of(int pid) {
    for (SUnit& u : units)
      if (u.unit_type == HERO && u.player_id == pid) return &u;
    return nullptr;
  }

  void spawn_wave() {
    for (int team : {TEAM_R, TEAM_D}) {
      double sx, sy;
      creep_spawn(team, sx, sy);
      for (int k = 0; k < 4; ++k) {
        const bool ranged = k == 3;
        SUnit c;
        c.handle = ++next_handle; c.unit_type = LANE_CREEP; c.kind = ranged ? K_RANGED : K_MELEE; c.team = team;
        c.x = sx + rng.uniform(-80, 80);
        c.y = sy + rng.uniform(-80, 80);
        c.hp = ranged ? 300.0 : 550.0; c.hp_max = c.hp;
        c.damage = ranged ? 24.0 : 21.0; c.attack_range = ranged ? 500.0 : 100.0; c.attack_period = 1.0;
        c.speed = 325.0; c.facing = team == TEAM_R ? 45.0 : 225.0;
        units.push_back(c);
      }
    }
  }

  static double dist(const SUnit& a, const SUnit& b) { return hyp(a.x - b.x, a.y - b.y); }

  void move_towards(SUnit& u, double tx, double ty) {
    const double dx = tx - u.x, dy = ty - u.y;
    const double d = hyp(dx, dy);
    if (d < 1e-3) return;
    const double step = std::min(d, u.speed * dt);
    u.x += dx / d * step;
    u.y += dy / d * step;
    u.facing = facing_to(dy, dx);
    u.x = std::max(-8000.0, std::min(8000.0, u.x));
    u.y = std::max(-8000.0, std::min(8000.0, u.y));
  }

  // nearest alive non-invulnerable enemy of `team` within max_range (python: last candidate wins ties)
  // (the squared-distance pre-test only skips units whose correctly rounded sqrt must exceed bd — the kept
  // comparison is the python one, so the choice is bit-identical; it saves the sqrt of every far unit)
  SUnit* nearest(const SUnit& u, int team, double max_range, bool non_hero_only) {
    SUnit* best = nullptr;
    double bd = max_range;
    for (SUnit& v : units) {
      if (!v.alive || v.team == team || v.invulnerable) continue;
      if (non_hero_only && v.unit_type == HERO) continue;
      const double dx = u.x - v.x, dy = u.y - v.y, d2 = dx * dx + dy * dy;
      if (d2 > bd * bd * (1.0 + 1e-14)) continue;
      const double d = std::sqrt(d2);
      if (d <= bd) { best = &v; bd = d; }
    }
    return best;
  }

  void share_xp(const SUnit& dead, double xp) {
    std::vector<SUnit*> hs;
    for (SUnit& h : units)
      if (h.unit_type == HERO && h.alive && h.team != dead.team && dist(h, dead) <= kXpRadius) hs.push_back(&h);
    for (SUnit* h : hs) {
      h->total_xp += xp / (double)hs.size();
      int lvl, need;
      level_from_total_xp(h->total_xp, lvl, need);
      if (lvl > h->level) {
        h->hp_max += 20.0 * (lvl - h->level);
        h->damage += 3.0 * (lvl - h->level);
        h->level = lvl;
      }
    }
  }

  void kill(SUnit& target, const SUnit& killer) {
    target.alive = false;
    target.hp = 0.0;
    target.target = 0;
    if (target.unit_type == HERO) {
      player(target.player_id)->deaths += 1;
      target.respawn_at = dota_time + 6.0 + 2.0 * target.level;
      const int kp = killer.unit_type == HERO ? killer.player_id : target.last_attacker_player;
      if (kp >= 0 && player(kp)->team_id != target.team) player(kp)->kills += 1;
      share_xp(target, (double)(100 + 20 * target.level));
    } else if (target.unit_type == LANE_CREEP) {
      if (killer.unit_type == HERO) {
        if (killer.team != target.team) {
          const_cast<SUnit&>(killer).last_hits += 1;
        } else {
          const_cast<SUnit&>(killer).denies += 1;
        }
      }
      if (killer.team != target.team) share_xp(target, target.kind == K_RANGED ? 69.0 : 57.0);
    } else if (target.unit_type == TOWER && target.kind == K_TOWER1) {
      status = target.team == TEAM_R ? ST_DIRE_WIN : ST_RADIANT_WIN;
    }
  }

  void attack(SUnit& a, SUnit& t) {
    a.target = t.handle;
    a.facing = facing_to(t.y - a.y, t.x - a.x);
    if (a.cooldown > 0) return;
    a.cooldown = a.attack_period;
    if (a.attack_range > 150) t.projectiles.push_back(a.handle);
    const double dmg = a.damage * rng.uniform(0.9, 1.1);
    t.hp -= dmg;
    if (a.unit_type == HERO) t.last_attacker_player = a.player_id;
    if (t.hp <= 0) kill(t, a);
  }

  void default_bot(SUnit& h) {
    if (h.hp < 0.3 * h.hp_max) {
      t1_mid(h.team, h.mx, h.my);
      h.has_move = true;
      h.target = 0;
      return;
    }
    SUnit* lowest = nullptr;
    std::vector<SUnit*> enemies;
    // python: min(enemies + allies, key=hp) over creeps within 900 — enemies first, then low-hp allies
    for (SUnit& v : units)
      if (v.alive && v.unit_type == LANE_CREEP && dist(h, v) <= 900.0 && v.team != h.team) enemies.push_back(&v);
    std::vector<SUnit*> cand(enemies);
    for (SUnit& v : units)
      if (v.alive && v.unit_type == LANE_CREEP && dist(h, v) <= 900.0 && v.team == h.team && v.hp < 0.5 * v.hp_max)
        cand.push_back(&v);
    for (SUnit* v : cand)
      if (!lowest || v->hp < lowest->hp) lowest = v;
    if (lowest && lowest->hp <= h.damage * 1.3) {
      h.target = lowest->handle;
      h.has_move = false;
    } else if (!enemies.empty()) {
      double ex = 0, ey = 0;
      for (SUnit* v : enemies) ex += v->x;
      for (SUnit* v : enemies) ey += v->y;
      ex = ex / (double)enemies.size();
      ey = ey / (double)enemies.size();
      const double d = h.team == TEAM_R ? 450.0 : -450.0;
      h.has_move = true; h.mx = ex - d; h.my = ey - d; h.target = 0;
    } else {
      double tx, ty;
      t1_mid(h.team, tx, ty);
      h.has_move = true; h.mx = tx * 0.3; h.my = ty * 0.3; h.target = 0;
    }
  }

  // decoded order for one controlled hero (features/actions.py action_to_pb → SyntheticGame._apply_action)
  struct Order {
    int player = -1, type = 0;   // 0 none, 1 move, 2 attack
    double mx = 0, my = 0;
    int64_t target = -1;
  };

  void apply(SUnit& h, const Order& o) {
    if (o.type == 1) {
      h.has_move = true; h.mx = o.mx; h.my = o.my; h.target = 0;
    } else if (o.type == 2) {
      SUnit* t = (o.target >= 0 && o.target <= 0x7fffffff) ? find((int)o.target) : nullptr;
      h.has_move = false;
      h.target = (t && t->alive) ? t->handle : 0;
    } else {
      h.has_move = false;
      h.target = 0;
    }
  }

  bool is_1v1() const {
    int n = 0;
    for (const SUnit& u : units)
      if (u.unit_type == HERO && u.control != CTRL_IDLE) ++n;
    return n <= 2;
  }

  // SyntheticGame.step with the radiant orders applied before the dire ones (act order of the service)
  void step(const std::vector<Order>& orders) {
    if (status != ST_OK) return;
    for (SUnit& u : units) u.projectiles.clear();
    for (int team : {TEAM_R, TEAM_D})
      for (const Order& o : orders) {
        SUnit* h = hero_of(o.player);
        if (h && h->alive && h->team == team) apply(*h, o);
      }
    if (dota_time >= 0) {
      const long wave = (long)std::floor(dota_time / 30.0);
      if (!has_wave || wave != last_wave) {
        has_wave = true;
        last_wave = wave;
        spawn_wave();
      }
    }
    const size_t n0 = units.size();   // python iterates a snapshot list of the values
    for (size_t i = 0; i < n0; ++i) {
      SUnit& u = units[i];
      u.cooldown = std::max(0.0, u.cooldown - dt);
      if (!u.alive) {
        if (u.unit_type == HERO && dota_time >= u.respawn_at) {
          u.alive = true;
          u.hp = u.hp_max;
          fountain(u.team, u.x, u.y);
          u.has_move = false;
          u.target = 0;
        }
        continue;
      }
      if (u.unit_type == HERO) {
        if (u.control == CTRL_IDLE) continue;
        if (u.control == CTRL_DEFAULT) default_bot(u);
        u.hp = std::min(u.hp_max, u.hp + 1.5 * dt);
        if (u.target) {
          SUnit* t = find(u.target);
          if (!t || !t->alive || t->invulnerable) u.target = 0;
          else if (dist(u, *t) <= u.attack_range) attack(u, *t);
          else move_towards(u, t->x, t->y);
        } else if (u.has_move) {
          move_towards(u, u.mx, u.my);
        }
      } else if (u.unit_type == LANE_CREEP) {
        SUnit* t = nearest(u, u.team, 500.0, true);
        if (!t) t = nearest(u, u.team, 500.0, false);
        if (t) {
          if (dist(u, *t) <= u.attack_range + 40.0) {
            attack(u, *t);
          } else {
            u.target = 0;
            move_towards(u, t->x, t->y);
          }
        } else {
          u.target = 0;
          double ex, ey;
          ancient(opp(u.team), ex, ey);
          move_towards(u, ex, ey);
        }
      } else if (u.unit_type == TOWER && !u.invulnerable) {
        SUnit* t = nearest(u, u.team, u.attack_range, true);
        if (!t) t = nearest(u, u.team, u.attack_range, false);
        if (t) attack(u, *t);
        else u.target = 0;
      }
    }
    // creeps that died before this step are removed; the ones that died in it linger one observation
    keep_.clear();
    keep_.reserve(units.size());
    for (SUnit& u : units)
      if (!(!u.alive && u.unit_type == LANE_CREEP && u.respawn_at == -1.0)) keep_.push_back(std::move(u));
    units.swap(keep_);
    for (SUnit& u : units)
      if (!u.alive && u.unit_type == LANE_CREEP) u.respawn_at = -1.0;
    for (const PStats& p : players)
      if (p.kills >= 2 && is_1v1()) status = p.team_id == TEAM_R ? ST_RADIANT_WIN : ST_DIRE_WIN;
    dota_time += dt;
    n_steps += 1;
  }

  bool visible(const SUnit& u, int team) const {
    if (!fog || u.team == team || u.unit_type == TOWER) return true;
    for (const SUnit& a : units) {
      if (a.team != team || !a.alive) continue;
      const double dx = a.x - u.x, dy = a.y - u.y, d2 = dx * dx + dy * dy;
      if (d2 > kVision * kVision * (1.0 + 1e-14)) continue;       // sqrt(d2) > kVision for sure
      if (std::sqrt(d2) <= kVision) return true;
    }
    return false;
  }

  // CMsgBotWorldState(team) serialised on the wire, field for field what env/synthetic.py world_state() sets (so
  // the bytes equal its SerializeToString): the protobuf observation the reference's actor receives from
  // DotaService.observe (agent.py:805-810) and featurizes from (agent.py:564-637).
  void world_bytes(int team, std::string& out) const {
    out.clear();
    Writer w{&out};
    w.u64(1, (uint64_t)team);
    w.f32(2, (float)(dota_time + 90.0));
    w.f32(3, (float)dota_time);
    thread_local std::string sub, unit;
    for (const PStats& p : players) {
      sub.clear();
      Writer s{&sub};
      s.i32(1, p.player_id);
      s.u64(2, (uint64_t)p.hero_id);
      s.u64(5, (uint64_t)p.kills);
      s.u64(6, (uint64_t)p.deaths);
      s.u64(8, (uint64_t)p.team_id);
      w.bytes(10, sub);
    }
    for (const SUnit& u : units) {
      if (!visible(u, team)) continue;
      unit.clear();
      Writer s{&unit};
      s.u64(1, (uint64_t)(uint32_t)u.handle);
      s.u64(2, (uint64_t)u.unit_type);
      s.bytes(3, unit_name(u));
      s.u64(4, (uint64_t)u.team);
      s.u64(5, (uint64_t)(uint32_t)u.level);
      sub.clear();
      Writer l{&sub};
      l.f32(1, (float)u.x);
      l.f32(2, (float)u.y);
      l.f32(3, 128.0f);
      s.bytes(6, sub);
      s.boolean(7, u.alive);
      s.i32(8, u.player_id);
      s.f32(11, (float)u.facing);
      s.i32(20, (int32_t)std::max(0.0, u.hp));
      s.i32(21, (int32_t)u.hp_max);
      s.f32(23, (float)u.mana);
      s.f32(24, (float)u.mana_max);
      s.i32(30, (int32_t)u.attack_range);
      s.i32(31, (int32_t)u.damage);
      s.u64(35, (uint64_t)(uint32_t)u.target);
      if (u.unit_type == TOWER) s.i32(40, u.target ? 1503 : 1500);
      s.boolean(50, u.invulnerable);
      if (u.unit_type == HERO) {
        int lvl, need;
        level_from_total_xp(u.total_xp, lvl, need);
        s.u64(60, (uint64_t)(uint32_t)need);
      }
      s.u64(61, (uint64_t)(uint32_t)u.last_hits);
      s.u64(62, (uint64_t)(uint32_t)u.denies);
      for (int c : u.projectiles) {
        sub.clear();
        Writer q{&sub};
        q.u64(1, (uint64_t)(uint32_t)c);
        q.boolean(4, true);
        s.bytes(70, sub);
      }
      w.bytes(11, unit);
    }
  }

  std::string_view unit_name(const SUnit& u) const {
    const bool r = u.team == TEAM_R;
    switch (u.kind) {
      case K_HERO:
        for (const PStats& p : players)
          if (p.player_id == u.player_id)
            return p.hero_id == HERO_NEVERMORE ? "npc_dota_hero_nevermore" : "npc_dota_hero_sniper";
        return "npc_dota_hero_sniper";
      case K_TOWER1: return r ? "npc_dota_goodguys_tower1_mid" : "npc_dota_badguys_tower1_mid";
      case K_TOWER2: return r ? "npc_dota_goodguys_tower2_mid" : "npc_dota_badguys_tower2_mid";
      case K_MELEE: return r ? "npc_dota_creep_goodguys_melee" : "npc_dota_creep_badguys_melee";
      default: return r ? "npc_dota_creep_goodguys_ranged" : "npc_dota_creep_badguys_ranged";
    }
  }

  // CMsgBotWorldState(team) as the featurizer sees it after the protobuf round trip
  void world(int team, World& w) const {
    w.dota_time = (float)dota_time;
    // the team's living units' positions, compacted once (the fog test below scans them per enemy unit)
    thread_local std::vector<double> ax, ay;
    if (fog) {
      ax.clear();
      ay.clear();
      for (const SUnit& a : units)
        if (a.team == team && a.alive) {
          ax.push_back(a.x);
          ay.push_back(a.y);
        }
    }
    size_t k = 0;                   // overwrite w's units in place: their attack_casters keep their capacity
    for (const SUnit& u : units) {
      if (fog && u.team != team && u.unit_type != TOWER) {
        bool seen = false;
        for (size_t j = 0; j < ax.size(); ++j) {
          const double dx = ax[j] - u.x, dy = ay[j] - u.y, d2 = dx * dx + dy * dy;
          if (d2 > kVision * kVision * (1.0 + 1e-14)) continue;       // sqrt(d2) > kVision for sure
          if (std::sqrt(d2) <= kVision) { seen = true; break; }
        }
        if (!seen) continue;
      }
      if (k == w.units.size()) w.units.emplace_back();
      Unit& m = w.units[k++];
      m.handle = (uint32_t)u.handle;
      m.unit_type = u.unit_type;
      m.name = u.kind == K_TOWER1 ? std::string_view("tower1_mid") : (u.kind == K_TOWER2 ? std::string_view("tower2_mid")
                                                                                         : std::string_view());
      m.team_id = (uint32_t)u.team;
      m.x = (float)u.x;
      m.y = (float)u.y;
      m.z = 128.0f;
      m.is_alive = u.alive;
      m.player_id = u.player_id;
      m.facing = (float)u.facing;
      m.health = (int32_t)std::max(0.0, u.hp);
      m.health_max = (int32_t)u.hp_max;
      m.attack_range = (int32_t)u.attack_range;
      m.attack_target = (uint32_t)u.target;
      m.anim = u.unit_type == TOWER ? (u.target ? 1503 : 1500) : 0;
      m.invuln = u.invulnerable;
      m.attack_immune = false;
      m.attack_casters.clear();
      for (int c : u.projectiles) m.attack_casters.push_back((uint32_t)c);
    }
    w.units.resize(k);
  }
};

// the fields of one observation that the shaped reward reads (agent.py:118-158): own hero, own player, own T1 tower
struct RewardView {
  int level = 1, xp_needed = 0, health = 0, health_max = 1, last_hits = 0, denies = 0, kills = 0, deaths = 0;
  bool alive = true;
  int tower_health = 0;
  float hx = 0, hy = 0;   // hero location (float32, as observed): canvas + move orders
};

inline RewardView reward_view(SimGame& g, int pid, int team) {
  RewardView v;
  const SUnit* h = g.hero_of(pid);
  int lvl, need;
  level_from_total_xp(h->total_xp, lvl, need);
  v.level = h->level;
  v.xp_needed = need;
  v.health = (int32_t)std::max(0.0, h->hp);
  v.health_max = (int32_t)h->hp_max;
  v.alive = h->alive;
  v.last_hits = h->last_hits;
  v.denies = h->denies;
  const PStats* p = g.player(pid);
  v.kills = p->kills;
  v.deaths = p->deaths;
  for (const SUnit& u : g.units)
    if (u.unit_type == TOWER && u.team == team && u.kind == K_TOWER1) { v.tower_health = (int32_t)std::max(0.0, u.hp); break; }
  v.hx = (float)h->x;
  v.hy = (float)h->y;
  return v;
}

// the nine sub-rewards in REWARD_KEYS order [enemy, win, xp, hp, kills, death, lh, denies, tower_hp]
inline void shaped_reward(const RewardView& a, const RewardView& b, double* r) {
  for (int k = 0; k < 9; ++k) r[k] = 0.0;
  const int xa = total_xp_from(a.level, a.xp_needed), xb = total_xp_from(b.level, b.xp_needed);
  r[2] = (double)(xb - xa) * 0.001;
  if (a.alive && b.alive) {
    const double ra = (double)a.health / (double)a.health_max, rb = (double)b.health / (double)b.health_max;
    const double low = 1. + (1 - rb) * (1 - rb);
    r[3] = (rb - ra) * low * 0.2;
  }
  r[4] = (double)(b.kills - a.kills) * 0.4;
  r[5] = (double)(b.deaths - a.deaths) * -0.4;
  r[6] = (double)(b.last_hits - a.last_hits) * 0.1;
  r[7] = (double)(b.denies - a.denies) * 0.05;
  r[8] = (double)(b.tower_health - a.tower_health) / 1900.;
}

// ============================================================================================================
// DCX2 encoding (transport/codec.py encode): JSON header + raw little-endian arrays + CRC-32C trailer (SSE4.2; the
// DCX1 form carried zlib's CRC-32, a table walk at ≈0.85 GB/s that dominated the learner's decode — DCX1 is still
// accepted by the decoder). crc32_zlib stays for that check.
// ============================================================================================================
// slice-by-8 (8 bytes per step through 8 derived tables, ≈4× the byte-wise loop): a whole-game rollout is ≈2 MB
inline uint32_t crc32_zlib(const uint8_t* p, size_t n, uint32_t crc = 0) {
  static uint32_t T[8][256];
  static std::once_flag once;
  std::call_once(once, [] {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320U ^ (c >> 1) : c >> 1;
      T[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int t = 1; t < 8; ++t) T[t][i] = (T[t - 1][i] >> 8) ^ T[0][T[t - 1][i] & 0xff];
  });
  crc = ~crc;
  while (n >= 8) {
    uint32_t lo, hi;
    std::memcpy(&lo, p, 4);
    std::memcpy(&hi, p + 4, 4);
    lo ^= crc;
    crc = T[7][lo & 0xff] ^ T[6][(lo >> 8) & 0xff] ^ T[5][(lo >> 16) & 0xff] ^ T[4][lo >> 24] ^
          T[3][hi & 0xff] ^ T[2][(hi >> 8) & 0xff] ^ T[1][(hi >> 16) & 0xff] ^ T[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) crc = T[0][(crc ^ *p++) & 0xff] ^ (crc >> 8);
  return ~crc;
}

struct ArrayRef {
  const char* name;
  const char* dtype;   // numpy dtype.str
  std::vector<int64_t> shape;
  const void* data;
  size_t bytes;
};

inline std::string json_escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') o.push_back('\\');
    o.push_back(c);
  }
  return o;
}

// DCX2 header JSON of a message (transport/codec.py encode); *arrays_bytes = Σ array payload bytes
inline std::string dcx2_header(const std::string& game_id, int team_id, int player_id, long weight_version,
                               double bootstrap, bool done, int hidden_stride, const int* layout,
                               const std::vector<ArrayRef>& arrays, size_t* arrays_bytes) {
  std::string h = "{\"game_id\":\"" + json_escape(game_id) + "\",\"team_id\":" + std::to_string(team_id) +
                  ",\"player_id\":" + std::to_string(player_id) + ",\"weight_version\":" +
                  std::to_string(weight_version) + ",\"bootstrap_value\":";
  char num[64];
  std::snprintf(num, sizeof num, "%.17g", bootstrap);
  h += num;
  h += std::string(",\"done\":") + (done ? "true" : "false") + ",\"hidden_stride\":" + std::to_string(hidden_stride) +
       ",\"layout\":[";
  for (int i = 0; i < 6; ++i) h += (i ? "," : "") + std::to_string(layout[i]);
  h += "],\"arrays\":[";
  size_t off = 0;
  for (size_t i = 0; i < arrays.size(); ++i) {
    const ArrayRef& a = arrays[i];
    h += (i ? ",[\"" : "[\"") + std::string(a.name) + "\",\"" + a.dtype + "\",[";
    for (size_t d = 0; d < a.shape.size(); ++d) h += (d ? "," : "") + std::to_string(a.shape[d]);
    h += "]," + std::to_string(off) + "," + std::to_string(a.bytes) + "]";
    off += a.bytes;
  }
  h += "]}";
  *arrays_bytes = off;
  return h;
}
inline size_t dcx2_size(const std::string& h, size_t arrays_bytes) { return 8 + h.size() + arrays_bytes + 4; }

// write a DCX2 message (dcx2_size bytes) into dst: magic, header length, header, arrays, CRC-32C trailer. Each piece
// is copied in 64 KB blocks and CRC'd right after, while the block is in cache (per-block CRCs combined), instead of a
// second full pass over the message.
inline void dcx2_write(uint8_t* dst, const std::string& h, const std::vector<ArrayRef>& arrays) {
  uint32_t crc = 0;
  size_t at = 0;
  auto put = [&](const void* src, size_t n) {
    constexpr size_t kBlk = 64 << 10;
    for (size_t o = 0; o < n; o += kBlk) {
      const size_t b = std::min(kBlk, n - o);
      std::memcpy(dst + at, static_cast<const uint8_t*>(src) + o, b);
      const uint32_t c = crc32c_raw(dst + at, b);
      crc = at == 0 ? c : crc32c_combine(crc, c, b);
      at += b;
    }
  };
  const uint32_t hl = (uint32_t)h.size();
  put("DCX2", 4);
  put(&hl, 4);
  put(h.data(), h.size());
  for (const ArrayRef& a : arrays) put(a.data, a.bytes);
  std::memcpy(dst + at, &crc, 4);
}

inline std::string encode_dcx1(const std::string& game_id, int team_id, int player_id, long weight_version,
                               double bootstrap, bool done, int hidden_stride, const int* layout,
                               const std::vector<ArrayRef>& arrays) {
  size_t ab;
  const std::string h = dcx2_header(game_id, team_id, player_id, weight_version, bootstrap, done, hidden_stride,
                                    layout, arrays, &ab);
  std::string out(dcx2_size(h, ab), '\0');
  dcx2_write(reinterpret_cast<uint8_t*>(&out[0]), h, arrays);
  return out;
}

// ============================================================================================================
// persistent worker pool: parallel_for over games
// ============================================================================================================
class Pool {
 public:
  explicit Pool(int n) : n_(std::max(1, n)) {
    for (int i = 1; i < n_; ++i) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void run(int count, const std::function<void(int)>& fn) {
    if (n_ == 1 || count <= 1) {
      for (int i = 0; i < count; ++i) fn(i);
      return;
    }
    {
      std::lock_guard<std::mutex> g(m_);
      fn_ = &fn;
      count_ = count;
      next_.store(0);
      active_ = (int)th_.size();
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> l(m_);
    done_cv_.wait(l, [this] { return active_ == 0; });
    fn_ = nullptr;
  }

 private:
  void work() {
    for (int i; (i = next_.fetch_add(1)) < count_;) (*fn_)(i);
  }
  void loop() {
    uint64_t seen = 0;
    while (true) {
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      work();
      std::lock_guard<std::mutex> g(m_);
      if (--active_ == 0) done_cv_.notify_all();
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  std::atomic<int> next_{0};
  int count_ = 0, active_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// ============================================================================================================
// the vectorised actor runtime
// ============================================================================================================
struct VecConfig {
  int n_games = 1;
  int mode = 0;                  // 0 1v1 self-play, 1 5v5 self-play, 2 1v1 controlled vs the default bot, 3 5v5 vs it
  uint64_t seed = 0;
  double start_time = -10.0, max_dota_time = 600.0, dt = 0.5;
  bool fog = true;
  long rollout_size = 1L << 40;
  int hidden_stride = 0, hidden_size = 0;
  double latest_weights_prob = 1.0;
  int counts[6] = {1, 5, 16, 16, 1, 1};
  int threads = 8;
  bool validation = false;
  // staggered resets: the FIRST game of slot gi ends at start + (max - start)·(gi+1)/n_games instead of max, so
  // lockstep games do not all finish (and publish whole-game rollouts) on the same step
  bool stagger = false;
  std::string tag = "vec";
  // observations as serialised CMsgBotWorldState protobufs decoded by the wire featurizer (the reference actor's
  // observe → featurize path) instead of straight from the engine's state
  bool wire = false;
  // observations as compact raw unit records (native/core.h featurize_one_raw) for GPU featurization
  // (ops/csrc/featurize.hip): observe_raw() fills the staging buffers, the trajectories keep the records and the
  // rollouts carry them ('units_raw' (T, U, 8) int32 + 'hero' (T, 4) fp32) instead of 'units' (T, U, 10)
  bool raw = false;
};

struct Traj {
  std::vector<float> env, units, logp, values, hiddens;   // (raw mode: units holds the raw records' 32-bit words)
  std::vector<float> hero;                                  // raw mode: the observing hero record, 4 per step
  std::vector<uint8_t> actions, masks;
  std::vector<double> rewards;
  std::vector<uint8_t> canvas;   // snapshot taken when a truncated rollout is cut (published one step later)
  long n = 0;
  void clear() {
    env.clear(); units.clear(); hero.clear(); logp.clear(); values.clear(); hiddens.clear(); actions.clear(); masks.clear();
    rewards.clear(); canvas.clear();
    n = 0;
  }
};

struct VPlayer {
  int player_id = 0, team = 0, slot = 0;
  bool latest = true;
  RewardView prev;
  bool rewarded = false, stepped = false;
  Traj traj;
  bool has_pending = false;
  Traj pending;
  long total_steps = 0;
  double last_reward_sum = 0;
};

struct VGame {
  SimGame sim;
  std::vector<VPlayer> players;
  std::vector<uint8_t> canvas;   // (256, 256, 3)
  std::string game_id;
  bool running = false, done = false, fresh = false;
  int end_state = -1;            // Status, -1 = none (time limit)
  float obs_time = 0;
  double limit = 0;              // dota time at which this game ends (max_dota_time, or staggered)
  int opponent_team = 0;         // 0: both latest; else the team playing the opponent (old) weights
  uint64_t serial = 0;
  std::vector<SimGame::Order> orders;
  double last_reward_sum[2] = {0, 0};   // per-team Σ of this step's shaped rewards (zero-sum ``enemy`` term)
  World world_buf[2];
  std::string wire_buf[2];       // wire mode: this step's serialised observations (World names point into them)
};

class VecEnv {
 public:
  explicit VecEnv(const VecConfig& c) : cfg_(c), pool_(c.threads) {
    U_ = 0;
    for (int i = 0; i < 6; ++i) U_ += cfg_.counts[i];
    A_ = 21 + U_;
    per_game_ = cfg_.mode == 1 ? 10 : (cfg_.mode == 2 ? 1 : (cfg_.mode == 3 ? 5 : 2));
    games_.resize(cfg_.n_games);
    rng_.seed(cfg_.seed ^ 0x9e3779b97f4a7c15ULL);
  }
  int slots() const { return cfg_.n_games * per_game_; }
  int players_per_game() const { return per_game_; }
  int units() const { return U_; }

  // start games that are not running; returns the slots whose recurrent state must be zeroed
  std::vector<int> begin_step() {
    std::vector<int> reset;
    for (int gi = 0; gi < cfg_.n_games; ++gi) {
      VGame& g = games_[gi];
      if (g.running) continue;
      start(gi);
      for (const VPlayer& p : g.players) reset.push_back(p.slot);
    }
    return reset;
  }

  // observe every running game (both teams): shaped rewards, canvas, features into env/units/handles (slot rows);
  // returns the slots whose trajectory records an LSTM state this step (hidden_stride)
  std::vector<int> observe(float* env, float* units, int64_t* handles, uint8_t* active) {
    std::vector<std::vector<int>> need(cfg_.n_games);
    pool_.run(cfg_.n_games,
              [&](int gi) { observe_game(gi, env, units, nullptr, nullptr, nullptr, handles, active, need[gi]); });
    std::vector<int> out;
    for (auto& v : need) out.insert(out.end(), v.begin(), v.end());
    return out;
  }
  // raw mode: env (slots, 3), hero (slots, 4), raw (slots, U, 8) and the host's handles (slots, U) (action targets)
  std::vector<int> observe_raw(float* env, float* hero, int32_t* raw, int64_t* handles, uint8_t* active) {
    std::vector<std::vector<int>> need(cfg_.n_games);
    pool_.run(cfg_.n_games,
              [&](int gi) { observe_game(gi, env, nullptr, hero, raw, nullptr, handles, active, need[gi]); });
    std::vector<int> out;
    for (auto& v : need) out.insert(out.end(), v.begin(), v.end());
    return out;
  }
  // raw mode, fp8 policy step: the staged records in their 16-byte form (raw16 (slots, U, 4)); the trajectories keep
  // the full records (the learner's exact features)
  std::vector<int> observe_raw16(float* env, float* hero, int32_t* raw16, int64_t* handles, uint8_t* active) {
    std::vector<std::vector<int>> need(cfg_.n_games);
    pool_.run(cfg_.n_games,
              [&](int gi) { observe_game(gi, env, nullptr, hero, nullptr, raw16, handles, active, need[gi]); });
    std::vector<int> out;
    for (auto& v : need) out.insert(out.end(), v.begin(), v.end());
    return out;
  }
  bool raw() const { return cfg_.raw; }

  // record the policy outputs, decode orders, advance the engines, rollout bookkeeping
  // (handles: the (slots, U) unit handles of the observe() these outputs answer — attack targets)
  void act(const int32_t* idx, const uint8_t* act, const uint8_t* msk, const float* logp, const float* value,
           const float* hidden, const int* hidden_slots, int n_hidden, const int64_t* handles, long weight_version) {
    std::vector<int> hrow(slots(), -1);
    for (int i = 0; i < n_hidden; ++i) hrow[hidden_slots[i]] = i;
    pool_.run(cfg_.n_games, [&](int gi) {
      act_game(gi, idx, act, msk, logp, value, hidden, hrow.data(), handles, weight_version);
    });
    for (VGame& g : games_) {
      if (!g.running && g.serial) {
        games_finished_ += 1;
        g.serial = 0;
      }
    }
  }

  std::vector<std::string> pop_rollouts() {
    std::lock_guard<std::mutex> l(out_m_);
    std::vector<std::string> o;
    o.swap(out_);
    return o;
  }
  // slots played with the opponent (old) weights in running games
  std::vector<int> opponent_slots() const {
    std::vector<int> s;
    for (const VGame& g : games_)
      if (g.running && g.opponent_team)
        for (const VPlayer& p : g.players)
          if (p.team == g.opponent_team) s.push_back(p.slot);
    return s;
  }
  long games_finished() const { return games_finished_; }
  long steps_taken() const { return steps_taken_.load(); }
  long rollouts_sent() const { return rollouts_sent_.load(); }
  long sink_lost() const { return sink_lost_.load(); }
  // publish finished rollouts straight into a shared-memory ring (the caller keeps it alive) instead of out_
  void set_sink(RingCore* ring, double timeout, bool drop_oldest) {
    sink_ = ring;
    sink_timeout_ = timeout;
    sink_drop_ = drop_oldest;
  }
  long wire_bytes() const { return wire_bytes_.load(); }
  double dota_time(int gi) const { return games_[gi].sim.dota_time; }
  int status(int gi) const { return games_[gi].sim.status; }
  const std::vector<uint8_t>& canvas(int gi) const { return games_[gi].canvas; }
  // per-game results of finished games since the last call:
  // (game index, team of the latest-weights side or 0 when both sides played the latest weights, end_state)
  std::vector<std::array<int, 3>> pop_results() {
    std::lock_guard<std::mutex> l(out_m_);
    std::vector<std::array<int, 3>> r;
    r.swap(results_);
    return r;
  }

 private:
  std::vector<Pick> picks(uint64_t s) const {
    std::vector<Pick> p;
    auto team = [&](int t, int first_mode, int n_ctrl) {
      for (int i = 0; i < 5; ++i)
        p.push_back(i < n_ctrl ? Pick{t, HERO_NEVERMORE, first_mode} : Pick{t, HERO_SNIPER, CTRL_IDLE});
    };
    if (cfg_.mode == 1) {
      team(TEAM_R, CTRL_CONTROLLED, 5);
      team(TEAM_D, CTRL_CONTROLLED, 5);
    } else if (cfg_.mode == 2 || cfg_.mode == 3) {   // controlled vs the default bot (1v1 / 5v5), sides alternate
      const bool r_ctrl = (s & 1) == 0;             // with the game serial
      const int nh = cfg_.mode == 3 ? 5 : 1;
      team(TEAM_R, r_ctrl ? CTRL_CONTROLLED : CTRL_DEFAULT, nh);
      team(TEAM_D, r_ctrl ? CTRL_DEFAULT : CTRL_CONTROLLED, nh);
    } else {
      team(TEAM_R, CTRL_CONTROLLED, 1);
      team(TEAM_D, CTRL_CONTROLLED, 1);
    }
    return p;
  }

  void start(int gi) {
    VGame& g = games_[gi];
    const uint64_t serial = ++started_;
    const uint64_t seed = cfg_.seed * 1000003ULL + serial;
    const std::vector<Pick> pk = picks(serial);
    g.sim.init(pk, seed, cfg_.start_time, cfg_.fog, cfg_.dt);
    g.game_id = cfg_.tag + "_" + std::to_string(serial);
    g.serial = serial;
    g.limit = cfg_.max_dota_time;
    if (cfg_.stagger && serial <= (uint64_t)cfg_.n_games)
      g.limit = cfg_.start_time + (cfg_.max_dota_time - cfg_.start_time) * (double)(gi + 1) / (double)cfg_.n_games;
    g.running = true;
    g.done = false;
    g.fresh = true;
    g.end_state = -1;
    g.canvas.assign(256 * 256 * 3, 255);
    g.opponent_team = 0;
    if (!cfg_.validation && rng_.random() > cfg_.latest_weights_prob)
      g.opponent_team = rng_.random() < 0.5 ? TEAM_R : TEAM_D;
    g.players.clear();
    int k = 0;
    for (const PStats& ps : g.sim.players) {
      const SUnit* h = g.sim.hero_of(ps.player_id);
      if (h->control != CTRL_CONTROLLED) continue;
      VPlayer p;
      p.player_id = ps.player_id;
      p.team = ps.team_id;
      p.slot = gi * per_game_ + k++;
      p.latest = g.opponent_team != p.team;
      p.prev = reward_view(g.sim, p.player_id, p.team);   // reset's world_state_<team>
      g.players.push_back(std::move(p));
    }
  }

  void observe_game(int gi, float* env, float* units, float* hero, int32_t* raw, int32_t* raw16, int64_t* handles,
                    uint8_t* active, std::vector<int>& need) {
    VGame& g = games_[gi];
    for (VPlayer& p : g.players) {
      active[p.slot] = 0;
      p.rewarded = false;
      p.stepped = false;
    }
    if (!g.running) return;
    if (g.sim.status != ST_OK) {   // observe() returns a final status: the game ends without this step
      g.done = true;
      g.end_state = g.sim.status;
      return;
    }
    g.obs_time = (float)g.sim.dota_time;
    World* w = g.world_buf;        // per-game scratch: the unit vectors keep their capacity across steps
    if (cfg_.wire) {
      // the reference actor's path: serialised CMsgBotWorldState per team → wire decode → featurize
      for (int ti = 0; ti < 2; ++ti) {
        g.sim.world_bytes(ti == 0 ? TEAM_R : TEAM_D, g.wire_buf[ti]);
        w[ti].units.clear();
        parse_world((const uint8_t*)g.wire_buf[ti].data(), g.wire_buf[ti].size(), w[ti]);
        wire_bytes_ += (long)g.wire_buf[ti].size();
      }
    } else {
      g.sim.world(TEAM_R, w[0]);
      g.sim.world(TEAM_D, w[1]);
    }
    double reward_sum[2] = {0, 0};
    for (VPlayer& p : g.players) {
      const int ti = p.team == TEAM_R ? 0 : 1;
      const RewardView cur = reward_view(g.sim, p.player_id, p.team);
      // trajectory canvas (actor/drawing.py): hero pixel in the team colour
      {
        const double ratio = 128.0 / 8000.0;
        int x = (int)(((double)cur.hx * ratio) + 128.0), y = (int)(256.0 - ((double)cur.hy * ratio) - 128.0);
        x = std::min(std::max(x, 0), 255);
        y = std::min(std::max(y, 0), 255);
        uint8_t* px = &g.canvas[((size_t)y * 256 + x) * 3];
        px[0] = p.team == TEAM_D ? 255 : 0;
        px[1] = p.team == TEAM_R ? 255 : 0;
        px[2] = 0;
      }
      double r[9];
      shaped_reward(p.prev, cur, r);
      double s = 0;
      for (int k = 0; k < 9; ++k) s += r[k];
      reward_sum[ti] += s;
      p.traj.rewards.insert(p.traj.rewards.end(), r, r + 9);
      p.prev = cur;
      p.rewarded = true;
      const int slot = p.slot;
      if (cfg_.raw) {
        thread_local std::vector<int32_t> scratch;
        int32_t* rr;
        if (raw16) {
          scratch.resize((size_t)U_ * kRawWords);
          rr = scratch.data();
        } else {
          rr = raw + (size_t)slot * U_ * kRawWords;
        }
        featurize_one_raw(w[ti], p.player_id, p.team, cfg_.counts, env + 3 * (size_t)slot, hero + 4 * (size_t)slot,
                          rr, handles + (size_t)slot * U_);
        if (raw16) raw_to_raw16(rr, U_, raw16 + (size_t)slot * U_ * kRaw16Words);
        // keep the raw records for the trajectory (their 32-bit words; the learner featurizes them on the GPU)
        const float* rf = reinterpret_cast<const float*>(rr);
        p.traj.units.insert(p.traj.units.end(), rf, rf + (size_t)U_ * kRawWords);
        p.traj.hero.insert(p.traj.hero.end(), hero + 4 * (size_t)slot, hero + 4 * (size_t)slot + 4);
      } else {
        featurize_one(w[ti], p.player_id, p.team, cfg_.counts, U_, env + 3 * (size_t)slot,
                      units + (size_t)slot * U_ * 10, handles + (size_t)slot * U_);
        // keep the features for the trajectory
        p.traj.units.insert(p.traj.units.end(), units + (size_t)slot * U_ * 10, units + (size_t)(slot + 1) * U_ * 10);
      }
      active[slot] = 1;
      p.stepped = true;
      if (cfg_.hidden_size && cfg_.hidden_stride && p.traj.n % cfg_.hidden_stride == 0) need.push_back(slot);
      p.traj.env.insert(p.traj.env.end(), env + 3 * (size_t)slot, env + 3 * (size_t)slot + 3);
    }
    g.last_reward_sum[0] = reward_sum[0];
    g.last_reward_sum[1] = reward_sum[1];
    g.fresh = false;
  }

  void emit(VGame& g, VPlayer& p, Traj& t, bool done, double bootstrap, long version) {
    if (cfg_.validation || !p.latest || t.n == 0) return;
    const long T = t.n;
    std::vector<ArrayRef> arr;
    arr.push_back({"env", "<f4", {T, 3}, t.env.data(), t.env.size() * 4});
    if (cfg_.raw) {
      arr.push_back({"units_raw", "<i4", {T, U_, kRawWords}, t.units.data(), t.units.size() * 4});
      arr.push_back({"hero", "<f4", {T, 4}, t.hero.data(), t.hero.size() * 4});
    } else {
      arr.push_back({"units", "<f4", {T, U_, 10}, t.units.data(), t.units.size() * 4});
    }
    arr.push_back({"actions", "|u1", {T, A_}, t.actions.data(), t.actions.size()});
    arr.push_back({"masks", "|u1", {T, A_}, t.masks.data(), t.masks.size()});
    arr.push_back({"rewards", "<f8", {T, 9}, t.rewards.data(), t.rewards.size() * 8});
    const std::vector<uint8_t>& cv = t.canvas.empty() ? g.canvas : t.canvas;
    arr.push_back({"canvas", "|u1", {256, 256, 3}, cv.data(), cv.size()});
    arr.push_back({"logp", "<f4", {T}, t.logp.data(), t.logp.size() * 4});
    arr.push_back({"values", "<f4", {T}, t.values.data(), t.values.size() * 4});
    if (!t.hiddens.empty()) {
      const long K = (long)(t.hiddens.size() / (2 * (size_t)cfg_.hidden_size));
      arr.push_back({"hiddens", "<f4", {K, 2, cfg_.hidden_size}, t.hiddens.data(), t.hiddens.size() * 4});
    }
    if (sink_ != nullptr) {
      // encoded straight into a reserved region of the node's experience ring (no intermediate string, no Python
      // bytes object, no second copy by a publish call) from this worker thread
      size_t ab;
      const std::string h = dcx2_header(g.game_id, p.team, p.player_id, version, bootstrap, done,
                                        t.hiddens.empty() ? 0 : cfg_.hidden_stride, cfg_.counts, arr, &ab);
      const size_t n = dcx2_size(h, ab);
      uint64_t pos, tok;
      // (a rollout larger than the whole ring is lost, not thrown: this runs on a Pool worker thread)
      if (sink_->too_large(n) || !sink_->reserve(n, sink_timeout_, sink_drop_, &pos, &tok)) {
        sink_lost_ += 1;
        return;
      }
      dcx2_write(sink_->wpayload(pos), h, arr);
      if (!sink_->commit(pos, n, tok)) {
        sink_lost_ += 1;
        return;
      }
      rollouts_sent_ += 1;
      return;
    }
    std::string b = encode_dcx1(g.game_id, p.team, p.player_id, version, bootstrap, done,
                                t.hiddens.empty() ? 0 : cfg_.hidden_stride, cfg_.counts, arr);
    {
      std::lock_guard<std::mutex> l(out_m_);
      out_.push_back(std::move(b));
    }
    rollouts_sent_ += 1;
  }

  void act_game(int gi, const int32_t* idx, const uint8_t* act, const uint8_t* msk, const float* logp,
                const float* value, const float* hidden, const int* hrow, const int64_t* handles, long version) {
    VGame& g = games_[gi];
    if (!g.running) return;
    const int H = cfg_.hidden_size;
    long stepped = 0;
    g.orders.clear();
    if (!g.done) {
      for (VPlayer& p : g.players) {
        if (!p.stepped) continue;
        const int s = p.slot;
        Traj& t = p.traj;
        if (p.has_pending) {   // truncated rollout waiting for this step's value (bootstrap)
          emit(g, p, p.pending, false, (double)value[s], version);
          p.has_pending = false;
          p.pending.clear();
        }
        if (H && cfg_.hidden_stride && t.n % cfg_.hidden_stride == 0) {
          const int r = hrow[s];
          if (r >= 0) t.hiddens.insert(t.hiddens.end(), hidden + (size_t)r * 2 * H, hidden + (size_t)(r + 1) * 2 * H);
          else t.hiddens.insert(t.hiddens.end(), (size_t)2 * H, 0.f);
        }
        t.actions.insert(t.actions.end(), act + (size_t)s * A_, act + (size_t)(s + 1) * A_);
        t.masks.insert(t.masks.end(), msk + (size_t)s * A_, msk + (size_t)(s + 1) * A_);
        t.logp.push_back(logp[s]);
        t.values.push_back(value[s]);
        t.n += 1;
        p.total_steps += 1;
        stepped += 1;
        // decode the sampled heads into an order (features/actions.py action_to_pb)
        SimGame::Order o;
        o.player = p.player_id;
        const int e = idx[(size_t)s * 4 + 0];
        if (e == 1) {
          static const float kMove[9] = {-275.f, -206.25f, -137.5f, -68.75f, 0.f, 68.75f, 137.5f, 206.25f, 275.f};
          o.type = 1;
          o.mx = (double)(float)((double)p.prev.hx + (double)kMove[idx[(size_t)s * 4 + 1]]);
          o.my = (double)(float)((double)p.prev.hy + (double)kMove[idx[(size_t)s * 4 + 2]]);
        } else if (e == 2) {
          o.type = 2;
          const int ti = idx[(size_t)s * 4 + 3];
          o.target = (ti >= 0 && ti < U_) ? handles[(size_t)s * U_ + ti] : -1;
        }
        g.orders.push_back(o);
      }
      if (cfg_.wire) wire_orders(g);
      g.sim.step(g.orders);
      // zero-sum shaping: subtract the opponent team's summed step reward (agent.py:829-833)
      if (!cfg_.validation)
        for (VPlayer& p : g.players)
          if (p.rewarded) p.traj.rewards[(size_t)(p.traj.n - 1) * 9 + 0] = -g.last_reward_sum[p.team == TEAM_R ? 1 : 0];
      for (VPlayer& p : g.players)
        if (p.stepped && p.traj.n > 0 && p.traj.n % cfg_.rollout_size == 0 && !cfg_.validation) {
          p.pending.clear();
          std::swap(p.pending, p.traj);
          p.pending.canvas = g.canvas;
          p.has_pending = true;
        }
    }
    steps_taken_ += stepped;
    if (g.done || (double)g.obs_time >= g.limit) finish(g, version);
  }

  // wire mode: each team's orders travel as the reference's Actions protobuf (CMsgBotWorldState.Actions{dota_time,
  // actions[]}, features/actions.py action_to_pb ↔ agent.py:665-695, 822-825) and are decoded back into the engine's
  // orders — the act() half of the DotaService round trip
  void wire_orders(VGame& g) {
    std::string& buf = g.wire_buf[0];          // observations of this step are featurized already
    std::vector<SimGame::Order> decoded;
    for (int team : {TEAM_R, TEAM_D}) {
      buf.clear();
      Writer w{&buf};
      w.f32(1, (float)g.obs_time);
      thread_local std::string a, sub, loc;
      for (const SimGame::Order& o : g.orders) {
        if (team_of(g, o.player) != team) continue;
        a.clear();
        Writer x{&a};
        x.u64(1, o.type == 1 ? 37u : (o.type == 2 ? 4u : 0u));   // MOVE_DIRECTLY / ATTACK_TARGET / NONE
        x.i32(2, o.player);
        x.i32(3, 0);                                             // actionDelay
        if (o.type == 1) {
          loc.clear();
          Writer l{&loc};
          l.f32(1, (float)o.mx);
          l.f32(2, (float)o.my);
          l.f32(3, 0.f);
          sub.clear();
          Writer m{&sub};
          m.bytes(2, loc);
          x.bytes(10, sub);
        } else if (o.type == 2) {
          sub.clear();
          Writer m{&sub};
          m.i32(2, (int32_t)o.target);
          m.boolean(3, true);
          x.bytes(12, sub);
        }
        w.bytes(2, a);
      }
      wire_bytes_ += (long)buf.size();
      parse_actions((const uint8_t*)buf.data(), buf.size(), decoded);
    }
    g.orders.swap(decoded);
  }

  static int team_of(const VGame& g, int player) {
    for (const VPlayer& p : g.players)
      if (p.player_id == player) return p.team;
    return 0;
  }

  static void parse_actions(const uint8_t* data, size_t n, std::vector<SimGame::Order>& out) {
    Reader r{data, data + n};
    while (r.ok()) {
      const uint64_t k = r.varint();
      const int f = (int)(k >> 3), wt = (int)(k & 7);
      if (!(wt == 2 && f == 2)) { r.skip(wt); continue; }
      const std::string_view a = r.bytes();
      Reader ar{(const uint8_t*)a.data(), (const uint8_t*)a.data() + a.size()};
      SimGame::Order o;
      uint64_t type = 0;
      while (ar.ok()) {
        const uint64_t ak = ar.varint();
        const int af = (int)(ak >> 3), awt = (int)(ak & 7);
        if (awt == 0 && af == 1) type = ar.varint();
        else if (awt == 0 && af == 2) o.player = (int)(int32_t)ar.varint();
        else if (awt == 2 && (af == 10 || af == 12)) {
          const std::string_view m = ar.bytes();
          Reader mr{(const uint8_t*)m.data(), (const uint8_t*)m.data() + m.size()};
          while (mr.ok()) {
            const uint64_t mk = mr.varint();
            const int mf = (int)(mk >> 3), mwt = (int)(mk & 7);
            if (af == 10 && mwt == 2 && mf == 2) {
              Unit tmp;
              parse_vector(mr.bytes(), tmp);
              o.mx = (double)tmp.x;
              o.my = (double)tmp.y;
            } else if (af == 12 && mwt == 0 && mf == 2) {
              o.target = (int64_t)(int32_t)mr.varint();
            } else {
              mr.skip(mwt);
            }
          }
        } else {
          ar.skip(awt);
        }
      }
      o.type = type == 37 ? 1 : (type == 4 ? 2 : 0);
      out.push_back(o);
    }
  }

  void finish(VGame& g, long version) {
    int latest_team = 0;
    for (VPlayer& p : g.players) {
      // end-state reward on the last step (agent.py:325-337)
      if (p.traj.n > 0) {
        double w = -0.25;
        if (g.end_state == ST_RADIANT_WIN) w = p.team == TEAM_R ? 1.0 : -1.0;
        else if (g.end_state == ST_DIRE_WIN) w = p.team == TEAM_D ? 1.0 : -1.0;
        p.traj.rewards[(size_t)(p.traj.n - 1) * 9 + 1] = w;
      }
      if (p.has_pending) {
        emit(g, p, p.pending, false, 0.0, version);
        p.has_pending = false;
        p.pending.clear();
      }
      emit(g, p, p.traj, true, 0.0, version);
      p.traj.clear();
      if (p.latest) latest_team = p.team;
    }
    {
      std::lock_guard<std::mutex> l(out_m_);
      results_.push_back({(int)(&g - games_.data()), g.opponent_team ? latest_team : 0, g.end_state});
    }
    g.running = false;
  }

 private:
  VecConfig cfg_;
  Pool pool_;
  int U_ = 40, A_ = 61, per_game_ = 2;
  std::vector<VGame> games_;
  PyRandom rng_;
  uint64_t started_ = 0;
  long games_finished_ = 0;
  std::atomic<long> steps_taken_{0}, rollouts_sent_{0}, wire_bytes_{0}, sink_lost_{0};
  RingCore* sink_ = nullptr;
  double sink_timeout_ = -1.0;
  bool sink_drop_ = true;
  std::mutex out_m_;
  std::vector<std::string> out_;
  std::vector<std::array<int, 3>> results_;
};

}  // namespace dca_native
