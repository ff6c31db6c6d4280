// XCD-team persistent LSTM recurrence (forward / backward) for gfx950 — the default learner recurrence.
//
// Same math as lstm.hip (reference north star: policy.py:67-68, 143-145 sketch an LSTM; BASELINE.json names the
// LSTM policy), different machine mapping. A recurrence step is latency-bound: its critical path is one
// all-to-all hand-off of the step's state between the workgroups that own slices of W_hh. lstm.hip spreads 64
// workgroups over all 8 XCDs, so every hand-off crosses the Infinity Fabric (write-through + L2-bypassing polls,
// ≈2.5-3 µs per all-gather under load). Here a TEAM of 32 workgroups — one per CU of a single XCD — runs a whole
// sequence chain and exchanges through that XCD's shared L2: plain stores keep the lines in L2 and sc1 polls (L1
// bypass, L2-served) see them ≈0.2 µs later (scripts/ubench/xcd_pingpong.hip: 451 ns round trip same-XCD vs
// 768 ns cross-XCD, idle). Up to 8 teams (one per XCD) run independent chains of ≤ 32 sequences concurrently.
//
// Team formation is placement-robust: every workgroup reads HW_REG_XCC_ID and takes a ticket on its XCC's
// counter; the first 32 of an XCC form its team, a leader commits the team only when all 32 arrived (bounded
// wait), and committed teams pull chains from a shared queue — so any dispatch that lands ≥ 32 workgroups on at
// least one XCD finishes every chain. An XCD whose team cannot form is not an error by itself (the other teams
// drain the queue); only chains left UNPROCESSED are: the last workgroup to exit checks the queue and sets
// *err = 3. Error codes (1 forward hand-off timeout, 2 backward timeout, 3 unprocessed chains) are sticky; the
// learner reduces the flag across DP ranks with the has-grad counts and the fused Adam skips the update when it
// is set (learner/engine.py), so a failed recurrence never reaches the weights; FusedPolicy.check_error raises at
// the iteration boundary (before checkpoint / publish). DCA_TEAM_FAIL=1 makes every workgroup refuse to form a
// team (fault-injection tests).
//
// Layouts (unit-major gates "(H,4)" so a hidden unit's 4 gates are one 16-byte vector):
//   xp4    (B, S, H, 4) f32  x·W_ihᵀ + b_ih + b_hh with W_ih rows permuted to (unit, gate) order
//   whh    (4H, H)      bf16 PyTorch layout (gate-major rows i,f,g,o)
//   gates4 (B, S, H, 4) f32  activated i, f, g, o          dgates4 (B, S, H, 4) f32 ∂L/∂pre-activations
//   hs (B,S,H) bf16, hsf (B,S,H) f32 (optional), cs (B,S,H) f32, h0/c0/hn/cn/dh0/dc0 (B,H) f32
// Each workgroup (member m of 32) owns U = H/32 hidden units J_m = [mU, mU+U) and their 4U gate rows.
//
// Forward step t:  gather h_{t-1} (B×H bf16, tagged granules, all 256 threads) → LDS → barrier → waves w < U/4
//   each own one 16-column MFMA tile = 4 units × 4 gates over the full K = H, W slice in VGPRs → 4×4 lane
//   transpose puts (i,f,g,o) of one (row, unit) in one lane → cell update (c in registers) → publish h_t granules.
// Backward step t (reduce-scatter, partials in bf16): gather Σ_producers partial dh for own units (xor-shuffle
//   reduction over the 32 producers) → barrier → gate gradients per (row, unit) → dG (bf16) to LDS → barrier →
//   partial dh_{t-1} (B×H) = dG_own (B×4U) · W_own (4U×H) on MFMA, W slice in VGPRs → LDS transpose → full-wave
//   16-byte chunk stores {2×bf16, tag, 2×bf16, tag} to each consumer's block.
//
// Tried and measured slower (kept out): a role-separated forward whose 5th "IO" wave owns every HBM access of a step
// (x·W_ih prefetch 1-2 steps ahead into an LDS ring, h/c/gate outputs from an LDS staging ring) so the MFMA waves'
// in-order vmcnt waits see only polls and publishes: 2.17-2.22 vs 1.92 µs per forward step at B=8, H=512. Also
// slower: storing a step's outputs after the NEXT step's gather barrier instead of right after the publish (2.08 vs
// 1.96 µs forward, 2.33 vs 2.28 backward — stores queued ahead of the publish delay it), although skipping the
// output stores altogether (knob) saves 0.14 µs per forward step; the x·W_ih load's placement does not matter.
// Two ways of getting those stores out of the pollers' vmcnt queue that measured no better: (1) a "ring" forward that
// publishes every step into its own slot (the slots then ARE the h output; gates recomputed by one GEMM, c kept):
// 1.99 vs 1.98 µs — a fresh slot misses the XCD L2 where the reused parity buffers hit; (2) polling waves 0,1
// staging their outputs in LDS for the non-polling waves 2,3 to store: 2.05-2.12 vs 1.94 µs. Not the residency of the
// written lines: outputs redirected into an 8-step L2-resident window ran 1.93-1.95 µs (no change), non-temporal
// stores 1.891 vs 1.895 — the cost follows the NUMBER of store instructions ahead of the next poll. Backward: its gate-gradient store costs 0.05-0.07 µs per step (2.27-2.30 vs 2.23 µs without it), but
// taking wave 0 (whose lanes store) off the poll, with waves 1-3 gathering 3 chunks per thread, was slower: 2.34-2.36.
// Round 2, fp32 V1 path (B=8, H=512): a double-buffered poll (second unpredicated round issued 0-4 sleeps after the
// first, so a late granule is seen up to half a round trip sooner) ran 1.435 vs 1.287 µs per forward step — the
// extra L2 reads slow the publishers more than the finer granularity gains; the poll back-off sleep (reset per step
// or removed, knob bits 12/13) measured within ±0.01 µs; a backward whose activation prefetch always hits L2 (step
// S-1 every step) ran 1.379 vs 1.385 µs — the saved-activation loads are not on the critical path either.
// Forward store COUNT matters more than bytes: one packed 16-B record {bf16 gates, f32 c, bf16 h} per (row, unit)
// instead of the three stores ran 1.84 vs 1.895 µs — left out (bf16 saved gates for the backward, and an h unpack
// pass would eat half the gain).
#include "common.h"
#include <cstdlib>

namespace {

using dca::bf16x8;
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int kT = 32;                  // workgroups per team (CUs per XCD); VAR bit 4: half teams (16, see below)
constexpr int kMaxTeams = 8;
constexpr int kThreads = 256;
constexpr int kSc1 = 16;                // buffer cache policy: sc1 (bypass the CU's L1, served by the XCD L2)
constexpr int kPlain = 0;               // plain store: write-through L1, line stays in the XCD L2
constexpr unsigned kSpinLimit = 1u << 22;

// Persistent control block (one per stream, zero-initialised once, caller-owned). It is SELF-CLEANING: the last
// workgroup of a launch to exit resets every field and bumps ``epoch``, so a launch never depends on a memset —
// which also makes the kernels safe to replay from a hipGraph. ``epoch`` is folded into every hand-off tag, so
// exchange buffers need no zeroing either: data left by an earlier launch can never match.
struct TeamCtl {
  unsigned xcnt[16];                     // tickets per XCC
  unsigned state[kMaxTeams];             // 0 pending, 1 committed, 2 aborted
  unsigned chain[kMaxTeams];             // (announce iter << 16) | chain id
  unsigned done[kMaxTeams];              // members that finished their current chain
  unsigned next_chain;
  unsigned abort;
  unsigned exits;                        // workgroups that have left the launch
  unsigned epoch;                        // launches completed on this control block
};
static_assert(sizeof(TeamCtl) <= 256, "TeamCtl must fit the 256-byte control tensor");

__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xf; }
__device__ __forceinline__ unsigned ld_acq(const unsigned* p) {
  return __hip_atomic_load((__attribute__((address_space(1))) unsigned*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rel(unsigned* p, unsigned v) {
  __hip_atomic_store((__attribute__((address_space(1))) unsigned*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned add_agent(unsigned* p, unsigned v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// explicit global (not flat) stores for the per-lane-address merged stores: a flat store would also count in lgkmcnt,
// which the LDS barriers wait on
template <typename T>
__device__ __forceinline__ void gstore(T* p, T v) { *(__attribute__((address_space(1))) T*)p = v; }
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// 8 consecutive fp32 values → hi / lo bf16 fragments (x = hi + lo up to ≈2⁻¹⁷ relative)
__device__ __forceinline__ void split_frag(const float* __restrict__ p, bf16x8& hi, bf16x8& lo) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hi[j] = dca::f2bf(v[j]);
    lo[j] = dca::f2bf(v[j] - dca::bf2f(hi[j]));
  }
}

// ---- V1 (exact fp32 VALU) dot products. Lane (r = lane/16, s = lane%16) of a wave owns FOUR outputs (the 4 gates
// of one unit forward, 4 units backward) over ONE K slice of KSL = K/16 elements: the slice's operand is read from LDS
// once (KSL/4 ds_read_b128, shared by the 4 rows through the LDS broadcast) and feeds 4 outputs, then a DPP row
// reduction sums the 16 slices. The step is bound by LDS return bandwidth and VALU issue, not by the FMAs: the first
// layout (lane = one output over a K quarter) read 4× the bytes — 32 × 1 KB per wave per step, 0.64 µs of compute
// phase at H = 512 — and a register/DPP-broadcast operand (one v_mov_dpp per FMA) was slower still (0.84 µs). FMAs
// issue as packed fp32 (v_pk_fma_f32, two outputs per instruction), two chains (even / odd k) per output pair.
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <int KSL>
__device__ __forceinline__ void pk_dot4(const float* wq, const float* x, float& o0, float& o1, float& o2, float& o3) {
  f32x2 a01e = {0.f, 0.f}, a01o = {0.f, 0.f}, a23e = {0.f, 0.f}, a23o = {0.f, 0.f};
#pragma unroll
  for (int j = 0; j < KSL; j += 4) {
    const float4 v = *reinterpret_cast<const float4*>(x + j);
    a01e = __builtin_elementwise_fma(f32x2{wq[j], wq[KSL + j]}, f32x2{v.x, v.x}, a01e);
    a23e = __builtin_elementwise_fma(f32x2{wq[2 * KSL + j], wq[3 * KSL + j]}, f32x2{v.x, v.x}, a23e);
    a01o = __builtin_elementwise_fma(f32x2{wq[j + 1], wq[KSL + j + 1]}, f32x2{v.y, v.y}, a01o);
    a23o = __builtin_elementwise_fma(f32x2{wq[2 * KSL + j + 1], wq[3 * KSL + j + 1]}, f32x2{v.y, v.y}, a23o);
    a01e = __builtin_elementwise_fma(f32x2{wq[j + 2], wq[KSL + j + 2]}, f32x2{v.z, v.z}, a01e);
    a23e = __builtin_elementwise_fma(f32x2{wq[2 * KSL + j + 2], wq[3 * KSL + j + 2]}, f32x2{v.z, v.z}, a23e);
    a01o = __builtin_elementwise_fma(f32x2{wq[j + 3], wq[KSL + j + 3]}, f32x2{v.w, v.w}, a01o);
    a23o = __builtin_elementwise_fma(f32x2{wq[2 * KSL + j + 3], wq[3 * KSL + j + 3]}, f32x2{v.w, v.w}, a23o);
  }
  const f32x2 a01 = a01e + a01o, a23 = a23e + a23o;
  o0 = a01.x; o1 = a01.y; o2 = a23.x; o3 = a23.y;
}
// Σ over the 16 lanes of this lane's DPP row, result in every lane: xor 1, xor 2 (quad_perm), half-row and row mirrors
__device__ __forceinline__ float row_sum16(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));
  return v;
}

// activations: the fast forms (v_exp_f32 + v_rcp_f32, ≈1e-7 relative) or, in the fp32-exact learner, libm expf /
// tanhf with IEEE division
template <bool PREC>
__device__ __forceinline__ float sigm(float x) { return PREC ? 1.f / (1.f + expf(-x)) : dca::sigmoidf_(x); }
template <bool PREC>
__device__ __forceinline__ float tanh_(float x) { return PREC ? tanhf(x) : dca::tanhf_(x); }

// Σ over the 32 lanes of this lane's half-wave (two DPP rows), result in every lane: row sum, then xor 16 by
// ds_swizzle (bit mode, and 0x1f / xor 0x10 inside each 32-lane group)
__device__ __forceinline__ float row_sum32(float v) {
  v = row_sum16(v);
  return v + __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401F));
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, int bytes) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// Bounded spin bookkeeping; true when this wave must give up (timeout or another workgroup raised an error). The
// limit is WALL-CLOCK per wait (s_memrealtime, 100 MHz): ≈2 s without one hand-off arriving (DCA_TEAM_PATIENT: ≈60 s,
// for runs that share the GPU with another process's kernels). It used to count polls over the whole launch, so a
// recurrence slowed by co-resident kernels (the node loop's actor graph replays) could trip it with no hand-off ever
// lost — the cumulative count grows with every step's extra polls (the config-5 loop's one backward timeout, code 2).
// `spins` restarts at every step (the back-off sleep after 32 polls: within ±0.01 µs of never sleeping).
__device__ __forceinline__ bool spin_fail(unsigned& spins, unsigned long long& since, TeamCtl* ctl, unsigned* err,
                                          unsigned code, int knobs) {
  asm volatile("" ::: "memory");        // compiler barrier: re-issue the poll loads every round
  if (spins++ == 0) since = __builtin_amdgcn_s_memrealtime();
  if ((spins & 255u) == 0) {
    if (ld_acq(&ctl->abort) != 0) return true;
    const unsigned long long limit = ((knobs >> 15) & 1) ? 6000000000ull : 200000000ull;
    if (__builtin_amdgcn_s_memrealtime() - since > limit) {
      st_rel(err, code);
      st_rel(&ctl->abort, 1u);
      return true;
    }
  }
  if (spins > 32 && !((knobs >> 13) & 1)) __builtin_amdgcn_s_sleep(1);
  return false;
}

// Team formation + chain queue. Returns the team id (≥ 0) or -1 if this workgroup must exit. Called by all
// threads; thread 0 does the global traffic, the result is broadcast through LDS.
__device__ int join_team(TeamCtl* ctl, unsigned* err, int* sh, unsigned* sh_epoch, int ts, bool refuse = false) {
  if (threadIdx.x == 0) {
    *sh_epoch = ld_acq(&ctl->epoch);
    int res = -1;
    const unsigned x = xcc_id();
    if (x < kMaxTeams && !refuse) {
      const unsigned r = add_agent(&ctl->xcnt[x], 1u);
      if (r < (unsigned)ts) {
        res = (int)x * 64 + (int)r;        // team x, member r
        unsigned spins = 0;
        if (r == 0) {
          bool ok = false;
          while (true) {
            if (ld_acq(&ctl->xcnt[x]) >= (unsigned)ts) { ok = true; break; }
            if (++spins > (1u << 16)) break;
            __builtin_amdgcn_s_sleep(2);
          }
          st_rel(&ctl->state[x], ok ? 1u : 2u);
          if (!ok) res = -1;                 // no team on this XCD (placement/residency); others may drain the queue
        } else {
          unsigned s;
          while ((s = ld_acq(&ctl->state[x])) == 0) {
            if (++spins > (1u << 18)) break;
            __builtin_amdgcn_s_sleep(2);
          }
          if (s != 1) res = -1;
        }
      }
    }
    *sh = res;
  }
  __syncthreads();
  return *sh;
}

// Next chain for this team (all members agree). Returns chain id or -1 when the queue is drained / aborted.
__device__ int next_chain(TeamCtl* ctl, int team, int member, unsigned iter, int nch, int* sh, int ts) {
  if (threadIdx.x == 0) {
    int res = -1;
    unsigned spins = 0;
    if (member == 0) {
      // every member finished the previous chain (its exchange buffers are free again)
      while (ld_acq(&ctl->done[team]) < (unsigned)ts * iter) {
        if (ld_acq(&ctl->abort) || ++spins > (1u << 24)) { spins = ~0u; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      unsigned c = spins == ~0u ? 0xffffu : add_agent(&ctl->next_chain, 1u);
      if (c > 0xffffu) c = 0xffffu;
      st_rel(&ctl->chain[team], ((iter + 1) << 16) | c);
      res = (c < (unsigned)nch) ? (int)c : -1;
    } else {
      unsigned v;
      while (((v = ld_acq(&ctl->chain[team])) >> 16) != iter + 1) {
        if (ld_acq(&ctl->abort) || ++spins > (1u << 24)) { v = 0xffffu; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      const unsigned c = v & 0xffffu;
      res = (c < (unsigned)nch) ? (int)c : -1;
    }
    *sh = res;
  }
  __syncthreads();
  return *sh;
}

// Every workgroup calls this last (all threads). The last one to leave flags chains that no team processed
// (*err = 3), then resets the control block for the next launch on the same stream and advances the epoch.
__device__ void team_exit(TeamCtl* ctl, unsigned* err, int nch) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned e = add_agent(&ctl->exits, 1u);
    if (e == gridDim.x - 1) {
      if (ld_acq(&ctl->next_chain) < (unsigned)nch) st_rel(err, 3u);
      for (int i = 0; i < 16; ++i) st_rel(&ctl->xcnt[i], 0u);
      for (int i = 0; i < kMaxTeams; ++i) {
        st_rel(&ctl->state[i], 0u);
        st_rel(&ctl->chain[i], 0u);
        st_rel(&ctl->done[i], 0u);
      }
      st_rel(&ctl->next_chain, 0u);
      st_rel(&ctl->abort, 0u);
      st_rel(&ctl->exits, 0u);
      st_rel(&ctl->epoch, ld_acq(&ctl->epoch) + 1u);
    }
  }
}

__device__ __forceinline__ unsigned make_tagbase(unsigned epoch, unsigned iter) {
  return ((epoch & 0x7ffu) << 21) | (((iter + 1u) & 0x1fu) << 16);   // | (t + 1): 16 bits
}

// =============================================================================================================
// Forward. MT = 16-row batch tiles per chain (Bc ≤ 16·MT), KS = H/128.
// xg (per team): [2 parity][Bc][H/2] u64 granules {lo: 2×bf16 h, hi: tag}
// =============================================================================================================
// V1 (F32 only, one sequence row per chain — every launch of B ≤ 8 sequences): the recurrent product runs as exact
// fp32 VALU dot products instead of MFMA tiles whose 16 rows would be 15/16 padding. Lane (col, kg) of a wave keeps
// W_hh[row(col)][kg·H/4 … kg·H/4 + H/4) as fp32 VGPRs (128 at H = 512), reads h_{t-1} (fp32, LDS) with broadcast
// 16-B loads, and the four k-quarters are summed with two cross-lane adds; a quad broadcast then hands each lane
// of the (row 0, unit) quad all four gates — the lane mapping of the MFMA path after its 4×4 transpose.
// VAR: 0 = MFMA tiles, 1 = V1 (exact fp32 VALU, 4 waves: lane = (unit, one of 16 K slices)), 2 = V2 (V1 on 8
// waves — two per SIMD — at H = 512: lane = (unit, one of 32 K slices of 16), so a SIMD interleaves two waves' FMA
// streams instead of issuing one wave's every other cycle; each wave owns 2 units, a lane half the K slice)
template <int MT, int KS, bool F32, int VAR>
__device__ __forceinline__ void lstm_team_fwd_body(
    const float* __restrict__ xp4, const void* __restrict__ whh_, const float* __restrict__ h0,
    const float* __restrict__ c0, short* __restrict__ hs, float* __restrict__ hsf, float* __restrict__ cs,
    float* __restrict__ gates4, float* __restrict__ hn, float* __restrict__ cn, unsigned long long* xg_all,
    TeamCtl* ctl, unsigned* err, int Btot, int Bc, int nch, int S, int sb, int st, unsigned long long* trace,
    int knobs, const float* __restrict__ bias4, const unsigned char* __restrict__ rst) {
  constexpr int H = 128 * KS;
  constexpr int TS = (VAR & 16) ? 16 : kT;   // workgroups per team
  constexpr int U = H / TS;             // units per workgroup (4·KS; half teams 8·KS)
  constexpr int NTILE = U / 4;          // 16-column MFMA tiles per workgroup (= KS)
  constexpr int KSTEP = H / 32;         // k-steps of the full K
  constexpr int HP = H + 8;             // LDS row pitch (bf16)
  constexpr int RB = MT * 16;
  constexpr int VV = VAR & 3;                     // variant; VAR & 4: precise (libm-class) activations
  constexpr bool PREC = (VAR & 4) != 0;
  constexpr bool V1 = VV >= 1;
  constexpr int NT = (VV == 2 || TS == 16) ? 512 : kThreads;    // threads per workgroup (half teams: 8 waves)
  constexpr int LPU = VV == 2 ? 32 : 16;          // V1/V2: lanes (K slices) per unit
  constexpr int UPW = 64 / LPU;                   // V1/V2: units per wave
  constexpr int KSL = H / LPU;                    // V1/V2: K slice per lane
  constexpr int R = V1 ? (1 << ((VAR >> 5) & 3)) : 1;   // V1: rows per chain (VAR bits 5-6: 1, 2, 4)
  constexpr int NR = V1 ? R : MT;                 // per-lane row registers (V1: every row; MFMA: one per tile)
  static_assert(!V1 || (F32 && MT == 1), "V1 is the fp32 exact VALU variant");
  static_assert(VV != 2 || H == 512, "V2 maps 8 waves x 2 units onto the 16 units of H = 512");
  static_assert(TS == kT || (VV == 1 && H == 512), "half teams: the V1 form at H = 512 (8 waves x 4 units)");
  __shared__ short hl[V1 ? 1 : 2][V1 ? 1 : RB][V1 ? 1 : HP];
  __shared__ short hlo[F32 && !V1 ? 2 : 1][F32 && !V1 ? RB : 1][F32 && !V1 ? HP : 1];   // F32: lo bf16 half of h
  // V1: h_{t-1} of each row as 16 K slices, each padded by 4 floats (the 16 lanes of a row read 16 different slices
  // with one ds_read_b128: unpadded 128-B strides would put pairs of lanes on the same banks)
  constexpr int SP = KSL + 4;
  constexpr int ROWF = LPU * SP;                  // V1: floats per row image
  __shared__ __attribute__((aligned(16))) float hf[V1 ? 2 : 1][V1 ? R * ROWF : 4];
  __shared__ int sh_int;
  __shared__ unsigned sh_epoch;

  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int me = join_team(ctl, err, &sh_int, &sh_epoch, TS, (knobs >> 11) & 1);
  const unsigned epoch = sh_epoch;
  if (me < 0) return;
  const int team = me >> 6, m = me & 63;
  const int j0 = m * U;
#define TSTAMP(ev)                                                                                        \
  if (trace && lane == 0 && wv < 4 && chain == 0 && t < 64)                                                \
    trace[(((size_t)m * 4 + wv) * 64 + t) * 8 + (ev)] = __builtin_amdgcn_s_memrealtime()
  // granules per row: bf16 h → H/2 (2 units each), F32 h → H (one unit each)
  constexpr int GPR = F32 ? H : H / 2;
  unsigned long long* xg = xg_all + (size_t)team * 2 * Bc * GPR;

  // zero the padding rows of both h buffers once
  if constexpr (!V1)
    for (int i = tid; i < 2 * RB * HP; i += NT) (&hl[0][0][0])[i] = 0;
  if constexpr (F32 && !V1)
    for (int i = tid; i < 2 * RB * HP; i += NT) (&hlo[0][0][0])[i] = 0;

  // W_hh slice for this wave's tile: columns c = 4·ul + q ↔ gate row q·H + j0 + 4·wv + ul, full K, in VGPRs
  // (F32: fp32 W_hh split into hi/lo bf16 fragments once, here)
  const bool mfma_wave = VV == 2 || wv < NTILE;
  const int col = lane & 15, kg = lane >> 4;
  bf16x8 wf[V1 ? 1 : KSTEP];
  bf16x8 wfl[F32 && !V1 ? KSTEP : 1];
  float wq[V1 ? 4 * KSL : 1];
  if (mfma_wave) {
    const int row = (col & 3) * H + j0 + 4 * wv + (col >> 2);
    if constexpr (V1) {
      // lane (u = lane/LPU, slice = lane%LPU): W_hh rows of the 4 gates of unit j0 + UPW·wv + u over the slice
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float* wr = static_cast<const float*>(whh_) + (size_t)(g * H + j0 + UPW * wv + lane / LPU) * H +
                          (lane % LPU) * KSL;
#pragma unroll
        for (int j = 0; j < KSL; j += 4) {
          const float4 v = *reinterpret_cast<const float4*>(wr + j);
          wq[g * KSL + j] = v.x; wq[g * KSL + j + 1] = v.y; wq[g * KSL + j + 2] = v.z; wq[g * KSL + j + 3] = v.w;
        }
      }
    } else if constexpr (F32) {
      const float* whh = static_cast<const float*>(whh_);
#pragma unroll
      for (int ks = 0; ks < KSTEP; ++ks) split_frag(whh + (size_t)row * H + ks * 32 + 8 * kg, wf[ks], wfl[ks]);
    } else {
      const short* whh = static_cast<const short*>(whh_);
#pragma unroll
      for (int ks = 0; ks < KSTEP; ++ks)
        wf[ks] = *reinterpret_cast<const bf16x8*>(whh + (size_t)row * H + ks * 32 + 8 * kg);
    }
  }
  // elementwise mapping after the 4×4 transpose: lane → (row 4·kg + (col&3) [+16·mt], unit j0 + 4·wv + col/4)
  // (V1: lane (u, slice) → row = slice — only slice 0 is a live row —, unit j0 + 4·wv + u)
  const int erow = V1 ? (lane % LPU) : 4 * kg + (col & 3);
  const int eunit = j0 + (V1 ? UPW * wv + lane / LPU : 4 * wv + (col >> 2));
  // folded LSTM bias (b_ih + b_hh, unit-major): xp4 may then be the bare input projection
  const dca::f32x4 bv = (bias4 && mfma_wave) ? *reinterpret_cast<const dca::f32x4*>(bias4 + eunit * 4)
                                             : dca::f32x4{0.f, 0.f, 0.f, 0.f};

  // V1/V2 merged outputs: every lane of a unit's LPU-lane group carries every row's state (the dot products are
  // summed into all of them anyway), so c and h leave in ONE store instruction — slice-2r lanes write row r's c,
  // slice-(2r+1) lanes its h — and a step queues two output stores (c|h, gates) behind its publish instead of three
  // (cs, hsf, gates): the stores ahead of the next poll are what the step pays for (see the notes at the top).
  // Measured (scripts/team_store_ab.py, bench A/B on one box): 1.420 vs 1.447 µs per standalone forward step,
  // 4.874 vs 4.945 ms per learner step.
  const int slice = V1 ? lane % LPU : 0;
  unsigned spins = 0;
  unsigned long long since = 0;
  for (unsigned iter = 0;; ++iter) {
    const int chain = next_chain(ctl, team, m, iter, nch, &sh_int, TS);
    if (chain < 0) break;
    const int b0 = chain * Bc;
    const int B = min(Bc, Btot - b0);
    const unsigned tagbase = make_tagbase(epoch, iter);
    float creg[NR], hreg[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int b = V1 ? i : i * 16 + erow;
      creg[i] = (mfma_wave && b < B) ? c0[(size_t)(b0 + b) * H + eunit] : 0.f;
      hreg[i] = 0.f;
    }
    bool dead = false;
    for (int t = 0; t < S; ++t) {
      const int par = t & 1;
      spins = 0;
      TSTAMP(0);
      // ---- prefetch this step's input projection (one 16-B vector per owned (row, unit)). Loading it one step
      // ahead instead measured slower (2.11 vs 1.94 µs per step at B=8, H=512).
      dca::f32x4 xv[NR];
      // sequence packing: an episode starts at step t (h, c := 0). The flag byte is kept raw and compared only at its
      // use, after the gather: a compare here (the old `rst[..] != 0` bool) waited out the load before the gather
      // started — measured +0.29 ms per B=8, S=1400 call for passing any reset tensor, zeros included.
      int rzb[NR];
      if (mfma_wave) {
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int b = V1 ? i : i * 16 + erow;         // (V1: the group's lanes load the same 16 B, one request)
          const size_t tx = ((knobs >> 10) & 1) ? 0 : (size_t)t;   // knob: every step reads step 0 (L2-resident)
          xv[i] = (b < B) ? *reinterpret_cast<const dca::f32x4*>(xp4 + (((size_t)(b0 + b) * sb + tx * st) * H + eunit) * 4)
                          : dca::f32x4{0.f, 0.f, 0.f, 0.f};
          rzb[i] = 0;
          if (rst != nullptr)                           // (uniform; rows >= B read row 0's flag and are never stored)
            rzb[i] = rst[(size_t)(b0 + (b < B ? b : 0)) * sb + (size_t)t * st];
        }
      }
      // ---- gather h_{t-1} into hl[par]
      if (t == 0) {
        for (int i = tid; i < B * H; i += NT) {
          const int b = i / H, k = i % H;
          const float v = h0[(size_t)(b0 + b) * H + k];
          if constexpr (V1) {
            hf[par][b * ROWF + (k / KSL) * SP + k % KSL] = v;
          } else {
            hl[par][b][k] = dca::f2bf(v);
            if constexpr (F32) hlo[par][b][k] = dca::f2bf(v - dca::bf2f(dca::f2bf(v)));
          }
        }
      } else {
        const unsigned tag = tagbase | (unsigned)t;          // h_{t-1} carries tag t
        const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(xg + (size_t)((t - 1) & 1) * Bc * GPR, Bc * GPR * 8);
        constexpr int CPR = F32 ? H / 2 : H / 4;              // 16-B chunks (2 f32 / 4 bf16 h values) per row
        constexpr int NL = ((V1 ? R : RB) * CPR + NT - 1) / NT;   // (V1: R rows)
        // every chunk is re-polled only until it has arrived, so later rounds move only the missing bytes
        i32x4 g[NL];
        bool okc[NL];
#pragma unroll
        for (int i = 0; i < NL; ++i) okc[i] = tid + NT * i >= B * CPR;
        for (int i = 0; i < (knobs & 0xff); ++i) __builtin_amdgcn_s_sleep(1);
        if ((knobs >> 9) & 1) {
          while (!okc[0]) {
            g[0] = __builtin_amdgcn_raw_buffer_load_b128(rs, tid * 16, 0, kSc1);
            okc[0] = ((unsigned)g[0].y == tag) & ((unsigned)g[0].w == tag);
            if (__all(okc[0])) break;
            if (spin_fail(spins, since, ctl, err, 1u, knobs)) { dead = true; break; }
          }
        }
        while (!dead) {
#pragma unroll
          for (int i = 0; i < NL; ++i)
            if (!okc[i]) g[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (tid + NT * i) * 16, 0, kSc1);
          bool ok = true;
#pragma unroll
          for (int i = 0; i < NL; ++i) {
            okc[i] = okc[i] || (((unsigned)g[i].y == tag) & ((unsigned)g[i].w == tag));
            ok &= okc[i];
          }
          if (__all(ok)) break;
          if (spin_fail(spins, since, ctl, err, 1u, knobs)) { dead = true; break; }
        }
#pragma unroll
        for (int i = 0; i < NL; ++i) {
          const int ci = tid + NT * i;
          if (ci < B * CPR) {
            if constexpr (V1) {
              const int b = ci / CPR, k = 2 * (ci % CPR);
              *reinterpret_cast<float2*>(&hf[par][b * ROWF + (k / KSL) * SP + k % KSL]) =
                  make_float2(__int_as_float(g[i].x), __int_as_float(g[i].z));
            } else if constexpr (F32) {
              const int b = ci / CPR, k = (ci % CPR) * 2;
              const float x = __int_as_float(g[i].x), z = __int_as_float(g[i].z);
              const short xh = dca::f2bf(x), zh = dca::f2bf(z);
              *reinterpret_cast<unsigned*>(&hl[par][b][k]) = (unsigned)(unsigned short)xh | ((unsigned)(unsigned short)zh << 16);
              *reinterpret_cast<unsigned*>(&hlo[par][b][k]) =
                  (unsigned)(unsigned short)dca::f2bf(x - dca::bf2f(xh)) |
                  ((unsigned)(unsigned short)dca::f2bf(z - dca::bf2f(zh)) << 16);
            } else {
              const int b = ci / CPR, k = (ci % CPR) * 4;
              *reinterpret_cast<u32x2*>(&hl[par][b][k]) = u32x2{(unsigned)g[i].x, (unsigned)g[i].z};
            }
          }
        }
      }
      TSTAMP(1);
      if (dead) sh_int = -2;
      lds_barrier();
      if (sh_int == -2) break;
      TSTAMP(2);
      if constexpr (V1) {
       // (only the waves that own units: at H < 512 a workgroup's U = H/32 units take U/4 of its 4 waves — the
       // others have no W_hh slice and would publish / store other workgroups' units)
       if (mfma_wave) {
        // ---- exact fp32 VALU, R rows: the 4 gates of this lane's unit over its K slice for every row (W_hh slice in
        // VGPRs reused across the rows), summed over the unit's LPU slices — every lane of the group holds every row
        float g[R][4];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (r < B) {                                        // (B is uniform)
            pk_dot4<KSL>(wq, &hf[par][r * ROWF + slice * SP], g[r][0], g[r][1], g[r][2], g[r][3]);
            // (Tried, one row: a reduce-SCATTER over the 16 slices — xor 1 / xor 2 quad swaps then row_ror 4 / 8, 4
            // DPP moves instead of 16 — with one activation per lane and a quad broadcast of the four gates: 1.500 vs
            // 1.481 µs per standalone step, no gain in the learner step; the plain row sums stay.)
#pragma unroll
            for (int q = 0; q < 4; ++q) g[r][q] = LPU == 32 ? row_sum32(g[r][q]) : row_sum16(g[r][q]);
          }
        }
        float act[R][4], cr[R], hr[R], hpub = 0.f;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          cr[r] = hr[r] = 0.f;
          act[r][0] = act[r][1] = act[r][2] = act[r][3] = 0.f;
          if (r < B) {
            if (rzb[r]) { g[r][0] = 0.f; g[r][1] = 0.f; g[r][2] = 0.f; g[r][3] = 0.f; }   // episode start
            const float pi = g[r][0] + (xv[r][0] + bv[0]), pf = g[r][1] + (xv[r][1] + bv[1]),
                        pg = g[r][2] + (xv[r][2] + bv[2]), po = g[r][3] + (xv[r][3] + bv[3]);
            const float ig = sigm<PREC>(pi), fg = sigm<PREC>(pf), gg = tanh_<PREC>(pg), og = sigm<PREC>(po);
            const float c = fg * (rzb[r] ? 0.f : creg[r]) + ig * gg;
            const float hv = og * tanh_<PREC>(c);
            creg[r] = c; hreg[r] = hv; cr[r] = c; hr[r] = hv;
            act[r][0] = ig; act[r][1] = fg; act[r][2] = gg; act[r][3] = og;
            if (slice == r) hpub = hv;
          }
        }
        TSTAMP(3);
        // ---- publish h_t: the slice-r lane of every unit group publishes row r's granule {f32 h(u), tag}
        if (slice < B) {
          const u32x2 gv = {(unsigned)__float_as_int(hpub), tagbase | (unsigned)(t + 1)};
          const __amdgpu_buffer_rsrc_t ws = uniform_rsrc(xg + (size_t)par * Bc * GPR, Bc * GPR * 8);
          __builtin_amdgcn_raw_buffer_store_b64(gv, ws, (slice * H + eunit) * 8, 0, kPlain);
        }
        TSTAMP(4);
        // ---- outputs, one store instruction per lane: slice 2r → row r's c (+ its gates), slice 2r+1 → row r's h
        // (one b32 store for everything — slices 0-3 the gates, 4 c, 5 h — measured slower: 1.476 vs 1.410 µs)
        const int orow = slice >> 1;
        if (orow < B && orow < R && !((knobs >> 8) & 1)) {
          float cv = 0.f, hv = 0.f;
          dca::f32x4 av = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int r = 0; r < R; ++r)
            if (orow == r) { cv = cr[r]; hv = hr[r]; av = dca::f32x4{act[r][0], act[r][1], act[r][2], act[r][3]}; }
          const size_t o = ((size_t)(b0 + orow) * sb + (size_t)t * st) * H + eunit;
          gstore((slice & 1) ? hsf + o : cs + o, (slice & 1) ? hv : cv);
          if (!(slice & 1)) *reinterpret_cast<dca::f32x4*>(gates4 + o * 4) = av;
        }
        TSTAMP(5);
       }
      } else if (mfma_wave) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          if (mt * 16 >= B) break;                            // wave-uniform
          float gq0 = 0.f, gq1 = 0.f, gq2 = 0.f, gq3 = 0.f;
          {
          // ---- gates pre-activation tile: rows = batch, columns = (unit, gate)
          dca::f32x4 acc = {0.f, 0.f, 0.f, 0.f};
          if constexpr (F32) {
            // three independent accumulation chains (hi·hi, lo·hi, hi·lo) keep the MFMA pipe full
            dca::f32x4 a1 = {0.f, 0.f, 0.f, 0.f}, a2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < KSTEP; ++ks) {
              const bf16x8 a = *reinterpret_cast<const bf16x8*>(&hl[par][mt * 16 + col][ks * 32 + 8 * kg]);
              const bf16x8 al = *reinterpret_cast<const bf16x8*>(&hlo[par][mt * 16 + col][ks * 32 + 8 * kg]);
              acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[ks], acc, 0, 0, 0);
              a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, wf[ks], a1, 0, 0, 0);
              a2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wfl[ks], a2, 0, 0, 0);
            }
            acc += a1 + a2;
          } else {
#pragma unroll
            for (int ks = 0; ks < KSTEP; ++ks) {
              const bf16x8 a = *reinterpret_cast<const bf16x8*>(&hl[par][mt * 16 + col][ks * 32 + 8 * kg]);
              acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[ks], acc, 0, 0, 0);
            }
          }
          // ---- 4×4 transpose inside each group of 4 lanes: lane (q' = col&3) gets gate q of row 4kg+q'. Round j:
          // lane a sends its value for row (a-j)&3 and receives from lane (a+j)&3 of its quad — a DPP quad_perm
          // (register-to-register, a few cycles) instead of an LDS-routed ds_bpermute
          const int q0 = col & 3;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int sel = (q0 - j) & 3;                       // what this lane sends in round j
            const float send = sel == 0 ? acc[0] : sel == 1 ? acc[1] : sel == 2 ? acc[2] : acc[3];
            const int qs = (q0 + j) & 3;                        // gate carried by the received value
            // quad_perm [(0+j)&3, (1+j)&3, (2+j)&3, (3+j)&3]: 0xE4 (identity), 0x39, 0x4E, 0x93
            float got = send;
            if (j == 1) got = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(send), 0x39, 0xF, 0xF, false));
            if (j == 2) got = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(send), 0x4E, 0xF, 0xF, false));
            if (j == 3) got = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(send), 0x93, 0xF, 0xF, false));
            gq0 = qs == 0 ? got : gq0;
            gq1 = qs == 1 ? got : gq1;
            gq2 = qs == 2 ? got : gq2;
            gq3 = qs == 3 ? got : gq3;
          }
          }
          const int b = mt * 16 + erow;
          if (rzb[mt]) { gq0 = 0.f; gq1 = 0.f; gq2 = 0.f; gq3 = 0.f; }   // episode start: no recurrent term
          // (bias added here, at the use: an add right after the prefetch would wait out the load before the gather)
          const float pi = gq0 + (xv[mt][0] + bv[0]), pf = gq1 + (xv[mt][1] + bv[1]), pg = gq2 + (xv[mt][2] + bv[2]),
                      po = gq3 + (xv[mt][3] + bv[3]);
          const float ig = sigm<PREC>(pi), fg = sigm<PREC>(pf), gg = tanh_<PREC>(pg), og = sigm<PREC>(po);
          const float c = fg * (rzb[mt] ? 0.f : creg[mt]) + ig * gg;
          const float hv = og * tanh_<PREC>(c);
          if (b < B) { creg[mt] = c; hreg[mt] = hv; }
          TSTAMP(3);
          if constexpr (F32) {
            // ---- publish h_t: granule {f32 h(u), tag} by every lane of a live row
            if (b < B) {
              const u32x2 gv = {(unsigned)__float_as_int(hv), tagbase | (unsigned)(t + 1)};
              const __amdgpu_buffer_rsrc_t ws = uniform_rsrc(xg + (size_t)par * Bc * GPR, Bc * GPR * 8);
              __builtin_amdgcn_raw_buffer_store_b64(gv, ws, (b * H + eunit) * 8, 0, kPlain);
            }
          } else {
            // ---- publish h_t: granule {h(u), h(u+1)} by the even-unit lane (partner unit is 4 lanes up)
            // partner unit's h from 4 lanes up, same 16-lane row: DPP row_shl:4 (register-to-register)
            const float hnb = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(hv), 0x104, 0xF, 0xF, false));
            if (b < B && ((col >> 2) & 1) == 0) {
              const unsigned pl = (unsigned)(unsigned short)dca::f2bf(hv) | ((unsigned)(unsigned short)dca::f2bf(hnb) << 16);
              const u32x2 gv = {pl, tagbase | (unsigned)(t + 1)};
              const __amdgpu_buffer_rsrc_t ws = uniform_rsrc(xg + (size_t)par * Bc * GPR, Bc * GPR * 8);
              __builtin_amdgcn_raw_buffer_store_b64(gv, ws, (b * (H / 2) + (eunit >> 1)) * 8, 0, kPlain);
            }
          }
          TSTAMP(4);
          // ---- outputs
          if (b < B && !((knobs >> 8) & 1)) {
            const size_t bt = (size_t)(b0 + b) * sb + (size_t)t * st;
            if (hs) hs[bt * H + eunit] = dca::f2bf(hv);
            if (hsf) hsf[bt * H + eunit] = hv;
            cs[bt * H + eunit] = c;
            *reinterpret_cast<dca::f32x4*>(gates4 + (bt * H + eunit) * 4) = dca::f32x4{ig, fg, gg, og};
          }
          TSTAMP(5);
        }
      }
    }
#undef TSTAMP
    if (sh_int == -2) return;
    if (mfma_wave) {
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        const int b = V1 ? i : i * 16 + erow;
        if (b < B && (!V1 || slice == i)) {
          hn[(size_t)(b0 + b) * H + eunit] = hreg[i];
          cn[(size_t)(b0 + b) * H + eunit] = creg[i];
        }
      }
    }
    __syncthreads();
    if (tid == 0) add_agent(&ctl->done[team], 1u);
  }
}

// =============================================================================================================
// Backward (all-gather of dG). Measured: what limits an in-XCD hand-off is the bytes WRITTEN per step (they also
// leave the XCD), not the bytes read from L2 — a reduce-scatter of B×H partials per workgroup (512 KB per step per
// team at B=8, H=512) took 2.7 µs per hand-off, so the backward gathers the B×4H gate gradients instead (32 KB
// written per step) and every workgroup computes its own units' recurrent gradient over the full K = 4H:
//   dh_{t}[b, J_m] = Σ_gc dG_{t+1}[b, gc] · W_hh[row(gc), J_m]      (gc = 4·j + q unit-major, row = q·H + j)
// xg (per team): [2 parity][Bc][H] 16-B chunks {bf16 d_i,d_f | tag | bf16 d_g,d_o | tag} (one per (row, unit)).
// Waves split K = 4H in quarters (W_hhᵀ slice of the owned units in VGPRs); partial tiles are summed via LDS.
// =============================================================================================================
// V1 (F32, one row per chain): the partial recurrent gradient as exact fp32 VALU dot products — lane (u, kg) keeps
// W_hhᵀ[gc][j0 + u] for its wave's K quarter and k-group as fp32 VGPRs, dG_{t+1} of row 0 sits in LDS in fp32.
// VAR 2 (V2, H = 512): 8 waves, each over one eighth of K = 4H (lane = (4 units, one of 16 slices of 16 gate columns))
template <int MT, int KS, bool F32, int VAR>
__device__ __forceinline__ void lstm_team_bwd_body(
    const float* __restrict__ dhs, const float* __restrict__ gates4, const float* __restrict__ cs,
    const float* __restrict__ c0, const float* __restrict__ dhn, const float* __restrict__ dcn,
    const void* __restrict__ whh_, float* __restrict__ dgates4, float* __restrict__ dh0, float* __restrict__ dc0,
    i32x4* xg_all, TeamCtl* ctl, unsigned* err, int Btot, int Bc, int nch, int S, int sb, int st,
    unsigned long long* trace, short* __restrict__ dg16, float* __restrict__ dbpart, int knobs,
    const unsigned char* __restrict__ rst) {
  constexpr int H = 128 * KS;
  constexpr int TS = (VAR & 16) ? 16 : kT;   // workgroups per team
  constexpr int U = H / TS;             // 4·KS units per workgroup (MFMA N, zero-padded to 16; half teams 8·KS)
  constexpr int VV = VAR & 3;
  constexpr bool PREC = (VAR & 4) != 0;
  constexpr bool V1 = VV >= 1;
  constexpr int NWK = VV == 2 ? 8 : 4;  // K parts (waves per 16-unit group)
  constexpr int UH = V1 && U > 16 ? U / 16 : 1;   // V1 16-unit groups (half teams: 2)
  constexpr int NW = NWK * UH;          // waves
  constexpr int NT = 64 * NW;
  constexpr int KW = 4 * H / NWK;       // K (= 4H gate columns) per wave
  constexpr int KSTEP = KW / 32;
  constexpr int RB = MT * 16;
  constexpr int GP = 4 * H + 8;         // LDS pitch (bf16) of the gathered dG rows
  constexpr int KSL = KW / 16;          // V1: K slice per lane of a wave's K part
  constexpr int R = V1 ? (1 << ((VAR >> 5) & 3)) : 1;   // V1: rows per chain (VAR bits 5-6: 1, 2, 4)
  constexpr int NPAIR = ((V1 ? R : RB) * U + NT - 1) / NT;
  static_assert(!V1 || (F32 && MT == 1), "V1 is the fp32 exact VALU variant");
  static_assert(VV != 2 || H == 512, "V2 is the H = 512 variant");
  static_assert(TS == kT || (VV == 1 && H == 512), "half teams: the V1 form at H = 512 (2 unit groups x 4 K parts)");
  // (Measured and removed in round 5: ∂W_hh accumulated inside this recurrence — 128 accumulators per lane on every
  // step's critical path, 3755 vs 2091 µs for the backward, 7.03 vs 5.59 ms per learner step.)
  __shared__ short dgl[V1 ? 1 : RB][V1 ? 1 : GP];
  __shared__ short dglo[F32 && !V1 ? RB : 1][F32 && !V1 ? GP : 1];   // F32: lo bf16 half of the gathered dG
  // V1: dG_{t+1} of row 0, fp32, as 64 K slices each padded by 4 floats (bank spread, as forward)
  constexpr int SP = KSL + 4;
  constexpr int DROW = (4 * H / KSL) * SP;   // V1: floats per row image of dG_{t+1}
  __shared__ __attribute__((aligned(16))) float dgf[V1 ? R * DROW : 4];
  __shared__ float red[NWK][RB][(U > 16 ? U : 16) + 1];
  __shared__ float dbs[RB * U * 4];     // per-(row, unit, gate) bias-gradient sums of a chain
  __shared__ int sh_int;
  __shared__ unsigned sh_epoch;
  // packing: the chain's episode-start flags as a bit image (row b, step t → bit t of rbits[b·wpr + t/32]), built
  // once per chain. Byte loads of the flags at every step — two per owned pair, compared where they were issued —
  // measured +0.32 ms per B = 8, S = 1400 backward call on some boxes (1921 → 2244 µs, scripts/reset_probe.py);
  // chains with more than kRstWords·32 (row, step) flags read them from global memory as before (so do the half-team
  // variants, whose LDS is full).
  constexpr int kRstWords = (VAR & 16) ? 1 : 2048;
  __shared__ unsigned rbits[kRstWords];

  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int me = join_team(ctl, err, &sh_int, &sh_epoch, TS);
  const unsigned epoch = sh_epoch;
  if (me < 0) return;
  const int team = me >> 6, m = me & 63;
  const int j0 = m * U;
  const int wpr = (S + 31) >> 5;        // flag words per row
  // 16-B chunks per (row, unit): bf16 {d_i,d_f | tag | d_g,d_o | tag}; F32 {d_i, tag, d_f, tag} {d_g, tag, d_o, tag}
  constexpr int CPU_ = F32 ? 2 : 1;
  i32x4* xg = xg_all + (size_t)team * 2 * Bc * H * CPU_;
#define TSTAMPB(ev)                                                                                       \
  if (trace && lane == 0 && wv < 4 && chain == 0 && k < 64)                                               \
    trace[(((size_t)m * 4 + wv) * 64 + k) * 8 + (ev)] = __builtin_amdgcn_s_memrealtime()

  if constexpr (!V1)
    for (int i = tid; i < RB * GP; i += NT) (&dgl[0][0])[i] = 0;
  if constexpr (F32 && !V1)
    for (int i = tid; i < RB * GP; i += NT) (&dglo[0][0])[i] = 0;

  // B operand: lane holds Wᵀ[gc][u] for gc = wv·H + ks·32 + 8·kg + j, u = lane & 15 (zero for u ≥ U)
  const int col = lane & 15, kg = lane >> 4;
  bf16x8 wf[V1 ? 1 : KSTEP];
  bf16x8 wfl[F32 && !V1 ? KSTEP : 1];
  float wq[V1 ? 4 * KSL : 1];
  if constexpr (V1) {
    // lane (ug = lane/16, slice = lane%16): W_hhᵀ of units j0 + 4·ug + uu (uu < 4) over the slice's gate columns
#pragma unroll
    for (int uu = 0; uu < 4; ++uu) {
      const int unit = 16 * (wv / NWK) + 4 * (lane >> 4) + uu;
#pragma unroll
      for (int j = 0; j < KSL; ++j) {
        const int gc = (wv % NWK) * KW + (lane & 15) * KSL + j;
        wq[uu * KSL + j] =
            (unit < U) ? static_cast<const float*>(whh_)[(size_t)((gc & 3) * H + (gc >> 2)) * H + j0 + unit] : 0.f;
      }
    }
  }
#pragma unroll
  for (int ks = 0; ks < (V1 ? 0 : KSTEP); ++ks) {
    bf16x8 v, vl;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int gc = wv * KW + ks * 32 + 8 * kg + j;
      const size_t wi = (size_t)((gc & 3) * H + (gc >> 2)) * H + j0 + col;
      if constexpr (F32) {
        const float w = (col < U) ? static_cast<const float*>(whh_)[wi] : 0.f;
        v[j] = dca::f2bf(w);
        vl[j] = dca::f2bf(w - dca::bf2f(v[j]));
      } else {
        v[j] = (col < U) ? static_cast<const short*>(whh_)[wi] : (short)0;
      }
    }
    wf[ks] = v;
    if constexpr (F32 && !V1) wfl[ks] = vl;
  }

  // (Tried: one 16-B store instruction for the two hand-off chunks and the ∂gates record — lanes 16·r + u of wave 0
  // computing unit u redundantly, role r picking the record — the forward's merged-store idea applied here: 1.578 vs
  // 1.535 µs per step, slower; the three stores of the 16 unit lanes stay.)
  unsigned spins = 0;
  unsigned long long since = 0;
  for (unsigned iter = 0;; ++iter) {
    const int chain = next_chain(ctl, team, m, iter, nch, &sh_int, TS);
    if (chain < 0) break;
    const int b0 = chain * Bc;
    const int B = min(Bc, Btot - b0);
    const unsigned tagbase = make_tagbase(epoch, iter);
    const bool rl = rst != nullptr && B * wpr <= kRstWords;    // flags from the LDS bit image
    if (rl) {
      for (int w = tid; w < B * wpr; w += NT) {
        const int b = w / wpr, tb = (w - b * wpr) * 32;
        const unsigned char* fr = rst + (size_t)(b0 + b) * sb;
        unsigned v = 0;
#pragma unroll
        for (int j = 0; j < 32; ++j)
          if (tb + j < S) v |= (fr[(size_t)(tb + j) * st] != 0 ? 1u : 0u) << j;
        rbits[w] = v;
      }
      lds_barrier();
    }
    float dcarry[NPAIR];
    dca::f32x4 dsum[NPAIR];               // Σ_t ∂gates of the owned pairs (bias gradient)
#pragma unroll
    for (int i = 0; i < NPAIR; ++i) dsum[i] = dca::f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < NPAIR; ++i) {
      const int pi = tid + NT * i;
      dcarry[i] = (pi < B * U && dcn) ? dcn[(size_t)(b0 + pi / U) * H + j0 + pi % U] : 0.f;
    }
    bool dead = false;
    for (int k = 0; k <= S; ++k) {
      const int t = S - 1 - k;          // step whose gate gradients are produced this iteration (-1: final)
      spins = 0;
      TSTAMPB(0);
      // ---- prefetch the saved activations of step t for the owned pairs
      dca::f32x4 gv[NPAIR];
      float cv[NPAIR], cpv[NPAIR], dv[NPAIR];
      bool rcur[NPAIR], rnext[NPAIR];     // packing: episode starts at t (c_{t-1} unused) / at t+1 (h_t unused by t+1)
      if (t >= 0) {
#pragma unroll
        for (int i = 0; i < NPAIR; ++i) {
          const int pi = tid + NT * i;
          rcur[i] = rnext[i] = false;
          if (pi < B * U) {
            const int b = pi / U, u = pi % U;
            const size_t bt = (size_t)(b0 + b) * sb + (size_t)t * st;
            gv[i] = *reinterpret_cast<const dca::f32x4*>(gates4 + (bt * H + j0 + u) * 4);
            cv[i] = cs[bt * H + j0 + u];
            cpv[i] = t > 0 ? cs[(bt - st) * H + j0 + u] : c0[(size_t)(b0 + b) * H + j0 + u];
            dv[i] = dhs[bt * H + j0 + u];
            if (rl) {
              const unsigned* rw = rbits + b * wpr;
              rcur[i] = (rw[t >> 5] >> (t & 31)) & 1u;
              rnext[i] = t + 1 < S && ((rw[(t + 1) >> 5] >> ((t + 1) & 31)) & 1u);
            } else if (rst != nullptr) {
              rcur[i] = rst[bt] != 0;
              rnext[i] = t + 1 < S && rst[bt + st] != 0;
            }
          }
        }
      }
      // ---- gather dG_{t+1} (B × 4H bf16) into LDS, all loads of a group of 8 rows in flight
      if (k > 0) {
        const unsigned tag = tagbase | (unsigned)(t + 2);
        const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(xg + (size_t)((t + 1) & 1) * Bc * H * CPU_, Bc * H * CPU_ * 16);
        constexpr int RG = V1 ? R : (F32 ? 4 : 8);         // rows per gather group
        constexpr int NL = RG * H * CPU_ / NT;             // chunks per thread per group
        for (int g0 = 0; g0 < B && !dead; g0 += RG) {
          const int nck = min(RG, B - g0) * H * CPU_;
          i32x4 g[NL];
          bool okc[NL];
#pragma unroll
          for (int i = 0; i < NL; ++i) okc[i] = tid + NT * i >= nck;
          while (true) {
#pragma unroll
            for (int i = 0; i < NL; ++i)
              if (!okc[i]) g[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (g0 * H * CPU_ + tid + NT * i) * 16, 0, kSc1);
            bool ok = true;
#pragma unroll
            for (int i = 0; i < NL; ++i) {
              okc[i] = okc[i] || (((unsigned)g[i].y == tag) & ((unsigned)g[i].w == tag));
              ok &= okc[i];
            }
            if (__all(ok)) break;
            if (spin_fail(spins, since, ctl, err, 2u, knobs)) { dead = true; break; }
          }
#pragma unroll
          for (int i = 0; i < NL; ++i) {
            const int ci = tid + NT * i;
            if (ci < nck) {
              if constexpr (V1) {
                const int b = ci / (H * CPU_), r = ci % (H * CPU_), gc = 4 * (r >> 1) + 2 * (r & 1);
                *reinterpret_cast<float2*>(&dgf[b * DROW + (gc / KSL) * SP + gc % KSL]) =
                    make_float2(__int_as_float(g[i].x), __int_as_float(g[i].z));
              } else if constexpr (F32) {
                const int b = g0 + ci / (2 * H), r = ci % (2 * H), gc = 4 * (r >> 1) + 2 * (r & 1);
                const float x = __int_as_float(g[i].x), z = __int_as_float(g[i].z);
                const short xh = dca::f2bf(x), zh = dca::f2bf(z);
                *reinterpret_cast<unsigned*>(&dgl[b][gc]) = (unsigned)(unsigned short)xh | ((unsigned)(unsigned short)zh << 16);
                *reinterpret_cast<unsigned*>(&dglo[b][gc]) =
                    (unsigned)(unsigned short)dca::f2bf(x - dca::bf2f(xh)) |
                    ((unsigned)(unsigned short)dca::f2bf(z - dca::bf2f(zh)) << 16);
              } else {
                const int b = g0 + ci / H, j = ci % H;
                *reinterpret_cast<u32x2*>(&dgl[b][4 * j]) = u32x2{(unsigned)g[i].x, (unsigned)g[i].z};
              }
            }
          }
        }
      }
      TSTAMPB(1);
      if (dead) sh_int = -2;
      lds_barrier();
      if (sh_int == -2) break;
      TSTAMPB(2);
      // ---- partial recurrent gradient over this wave's K quarter → red[wv]
      if (V1 && k > 0) {
        const int wk = wv % NWK;
        const int u0 = 16 * (wv / NWK) + 4 * (lane >> 4);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (r >= B) break;                                  // (B is uniform)
          float o0, o1, o2, o3;
          const float* x = &dgf[r * DROW + (wk * 16 + (lane & 15)) * SP];
          pk_dot4<KSL>(wq, x, o0, o1, o2, o3);
          o0 = row_sum16(o0);
          o1 = row_sum16(o1);
          o2 = row_sum16(o2);
          o3 = row_sum16(o3);
          if ((lane & 15) == 0 && u0 < U) {
            red[wk][r][u0] = o0;
            red[wk][r][u0 + 1] = o1;
            red[wk][r][u0 + 2] = o2;
            red[wk][r][u0 + 3] = o3;
          }
        }
      } else if (k > 0) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          if (mt * 16 >= B) break;
          dca::f32x4 acc = {0.f, 0.f, 0.f, 0.f};
          if constexpr (F32) {
            dca::f32x4 a1 = {0.f, 0.f, 0.f, 0.f}, a2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < KSTEP; ++ks) {
              const bf16x8 a = *reinterpret_cast<const bf16x8*>(&dgl[mt * 16 + col][wv * KW + ks * 32 + 8 * kg]);
              const bf16x8 al = *reinterpret_cast<const bf16x8*>(&dglo[mt * 16 + col][wv * KW + ks * 32 + 8 * kg]);
              acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[ks], acc, 0, 0, 0);
              a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, wf[ks], a1, 0, 0, 0);
              a2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wfl[ks], a2, 0, 0, 0);
            }
            acc += a1 + a2;
          } else {
#pragma unroll
            for (int ks = 0; ks < KSTEP; ++ks) {
              const bf16x8 a = *reinterpret_cast<const bf16x8*>(&dgl[mt * 16 + col][wv * KW + ks * 32 + 8 * kg]);
              acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[ks], acc, 0, 0, 0);
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) red[wv][mt * 16 + kg * 4 + r][col] = acc[r];
        }
      }
      TSTAMPB(3);
      lds_barrier();
      TSTAMPB(4);
      if (t < 0) {
        for (int i = tid; i < B * U; i += NT) {
          const int b = i / U, u = i % U;
          float acc = 0.f;
#pragma unroll
          for (int w = 0; w < NWK; ++w) acc += red[w][b][u];
          // an episode starting at step 0 never read h0
          dh0[(size_t)(b0 + b) * H + j0 + u] = (rst != nullptr && rst[(size_t)(b0 + b) * sb] != 0) ? 0.f : acc;
        }
        break;
      }
      // ---- gate gradients for the owned (row, unit) pairs; publish dG_t, write ∂gates
      const __amdgpu_buffer_rsrc_t ws = uniform_rsrc(xg + (size_t)(t & 1) * Bc * H * CPU_, Bc * H * CPU_ * 16);
      const int tg = (int)(tagbase | (unsigned)(t + 1));
#pragma unroll
      for (int i = 0; i < NPAIR; ++i) {
        const int pi = tid + NT * i;
        if (pi < B * U) {
          const int b = pi / U, u = pi % U;
          float rec = 0.f;
          if (k == 0) {
            rec = dhn ? dhn[(size_t)(b0 + b) * H + j0 + u] : 0.f;
          } else if (!rnext[i]) {
#pragma unroll
            for (int w = 0; w < NWK; ++w) rec += red[w][b][u];
          }
          const float ig = gv[i][0], fg = gv[i][1], gg = gv[i][2], og = gv[i][3];
          const float dht = dv[i] + rec;
          const float tc = tanh_<PREC>(cv[i]);
          const float dc = dcarry[i] + dht * og * (1.f - tc * tc);
          const float d_i = dc * gg * ig * (1.f - ig);
          const float d_f = rcur[i] ? 0.f : dc * cpv[i] * fg * (1.f - fg);
          const float d_g = dc * ig * (1.f - gg * gg);
          const float d_o = dht * tc * og * (1.f - og);
          dcarry[i] = rcur[i] ? 0.f : dc * fg;
          const size_t bt = (size_t)(b0 + b) * sb + (size_t)t * st;
          if constexpr (F32) {
            const int o = (b * H + j0 + u) * 2 * 16;
            __builtin_amdgcn_raw_buffer_store_b128(i32x4{__float_as_int(d_i), tg, __float_as_int(d_f), tg}, ws, o, 0,
                                                   kPlain);
            __builtin_amdgcn_raw_buffer_store_b128(i32x4{__float_as_int(d_g), tg, __float_as_int(d_o), tg}, ws, o + 16,
                                                   0, kPlain);
            *reinterpret_cast<dca::f32x4*>(dgates4 + (bt * H + j0 + u) * 4) = dca::f32x4{d_i, d_f, d_g, d_o};
          } else {
            const unsigned p01 = (unsigned)(unsigned short)dca::f2bf(d_i) | ((unsigned)(unsigned short)dca::f2bf(d_f) << 16);
            const unsigned p23 = (unsigned)(unsigned short)dca::f2bf(d_g) | ((unsigned)(unsigned short)dca::f2bf(d_o) << 16);
            __builtin_amdgcn_raw_buffer_store_b128(i32x4{(int)p01, tg, (int)p23, tg}, ws, (b * H + j0 + u) * 16, 0, kPlain);
            if (dg16) *reinterpret_cast<u32x2*>(dg16 + (bt * H + j0 + u) * 4) = u32x2{p01, p23};
            else *reinterpret_cast<dca::f32x4*>(dgates4 + (bt * H + j0 + u) * 4) = dca::f32x4{d_i, d_f, d_g, d_o};
          }
          dsum[i] += dca::f32x4{d_i, d_f, d_g, d_o};
          if (t == 0) dc0[(size_t)(b0 + b) * H + j0 + u] = dcarry[i];
        }
      }
      TSTAMPB(6);
    }
    if (sh_int == -2) return;
    if (dbpart) {
      // bias gradient of this chain for the owned units: Σ over rows (fixed order) of the per-pair sums
#pragma unroll
      for (int i = 0; i < NPAIR; ++i) {
        const int pi = tid + NT * i;
        if (pi < B * U) *reinterpret_cast<dca::f32x4*>(&dbs[pi * 4]) = dsum[i];
      }
      __syncthreads();
      for (int o = tid; o < U * 4; o += NT) {
        float acc = 0.f;
        for (int b = 0; b < B; ++b) acc += dbs[b * U * 4 + o];
        // PyTorch's gate-major order (gate q of unit j at q·H + j): the partials' chain sum IS ∂b_ih = ∂b_hh
        dbpart[(size_t)chain * 4 * H + (o & 3) * H + j0 + (o >> 2)] = acc;
      }
    }
    __syncthreads();
    if (tid == 0) add_agent(&ctl->done[team], 1u);
  }
#undef TSTAMPB
}

// Half teams (VAR bit 4): 16 workgroups of 512 threads per team, made CU-EXCLUSIVE by LDS — each workgroup holds
// ≥ 159 KB of the CU's 160 KB, so no workgroup of another kernel that uses LDS (every GEMM / encoder / chain kernel
// of the step) can land on a recurrence CU; the other 16 CUs of every XCD stay free for the step's other kernels
// (which would otherwise co-reside and lengthen every hand-off, profiles/r4_chunk_overlap_probe.md).
template <int VAR, int PAD>
__device__ __forceinline__ void claim_cu(int knobs) {
  if constexpr ((VAR & 16) != 0) {
    __shared__ char pad[PAD];
    if (knobs == 0x7fffffff) reinterpret_cast<volatile char*>(pad)[threadIdx.x] = 0;   // (never: keeps the LDS)
  }
}
// pads up to ≈159.5 KB per workgroup: the variants' own LDS (measured from the compiled kernels: forward 4 616 B +
// 4 608 per extra row, backward 25 864 B + 9 216 per extra row) subtracted from the target
constexpr int kHalfLds = 163328;
constexpr int pad_fwd(int var) { return kHalfLds - (4616 + ((1 << ((var >> 5) & 3)) - 1) * 4608); }
constexpr int pad_bwd(int var) { return kHalfLds - (25864 + ((1 << ((var >> 5) & 3)) - 1) * 9216); }
inline int team_threads(int var) { return ((var & 3) == 2 || (var & 16)) ? 512 : kThreads; }
inline int team_size(int var) { return (var & 16) ? 16 : kT; }

template <int MT, int KS, bool F32, int VAR>
__global__ __launch_bounds__(((VAR & 3) == 2 || (VAR & 16)) ? 512 : kThreads, 1) void lstm_team_fwd_kernel(
    const float* __restrict__ xp4, const void* __restrict__ whh, const float* __restrict__ h0,
    const float* __restrict__ c0, short* __restrict__ hs, float* __restrict__ hsf, float* __restrict__ cs,
    float* __restrict__ gates4, float* __restrict__ hn, float* __restrict__ cn, unsigned long long* xg_all,
    TeamCtl* ctl, unsigned* err, int Btot, int Bc, int nch, int S, int sb, int st, unsigned long long* trace,
    int knobs, const float* __restrict__ bias4, const unsigned char* __restrict__ rst) {
  __builtin_amdgcn_s_setprio(3);   // issue priority over co-resident waves of kernels overlapped on other streams
  claim_cu<VAR, pad_fwd(VAR)>(knobs);
  lstm_team_fwd_body<MT, KS, F32, VAR>(xp4, whh, h0, c0, hs, hsf, cs, gates4, hn, cn, xg_all, ctl, err, Btot, Bc, nch, S, sb,
                             st, trace, knobs, bias4, rst);
  team_exit(ctl, err, nch);
}

template <int MT, int KS, bool F32, int VAR>
__global__ __launch_bounds__(((VAR & 3) == 2 || (VAR & 16)) ? 512 : kThreads, 1) void lstm_team_bwd_kernel(
    const float* __restrict__ dhs, const float* __restrict__ gates4, const float* __restrict__ cs,
    const float* __restrict__ c0, const float* __restrict__ dhn, const float* __restrict__ dcn,
    const void* __restrict__ whh, float* __restrict__ dgates4, float* __restrict__ dh0, float* __restrict__ dc0,
    i32x4* xg_all, TeamCtl* ctl, unsigned* err, int Btot, int Bc, int nch, int S, int sb, int st,
    unsigned long long* trace, short* __restrict__ dg16, float* __restrict__ dbpart, int knobs,
    const unsigned char* __restrict__ rst) {
  __builtin_amdgcn_s_setprio(3);
  claim_cu<VAR, pad_bwd(VAR)>(knobs);
  lstm_team_bwd_body<MT, KS, F32, VAR>(dhs, gates4, cs, c0, dhn, dcn, whh, dgates4, dh0, dc0, xg_all, ctl, err, Btot, Bc, nch,
                             S, sb, st, trace, dg16, dbpart, knobs, rst);
  team_exit(ctl, err, nch);
}

// DCA_TEAM_KNOBS = pre_sleep | skip_outputs << 8 | probe_first << 9 | xp_step0 << 10 | no poll back-off sleep << 13
// | three-store forward outputs << 14 (latency experiments only);
// DCA_TEAM_FAIL=1 sets bit 11: no workgroup joins a team (fault injection: every chain left unprocessed → err 3);
// DCA_TEAM_PATIENT=1 sets bit 15: a 60 s instead of 2 s wall-clock hand-off timeout (spin_fail) for runs that share
// the GPU with another process's persistent kernels (bench.py DCA_SHARED_GPU rehearsals: two ranks' recurrences on
// one MI355X); a real lost hand-off still ends in the error, just later
inline int team_knobs() {
  const char* e = getenv("DCA_TEAM_KNOBS");
  const char* f = getenv("DCA_TEAM_FAIL");
  const char* p = getenv("DCA_TEAM_PATIENT");
  return (e ? atoi(e) : 0) | ((f && f[0] == '1') ? (1 << 11) : 0) | ((p && p[0] == '1') ? (1 << 15) : 0);
}

inline void plan(int B, int& nch, int& Bc, int& MT, int f32 = 0) {
  // Spread the sequences over all 8 teams (one chain per XCD) before packing rows into a chain: per-step latency
  // grows with rows per chain (more granules to gather and publish), measured B=8, H=512 fwd/bwd µs per step:
  // 1 chain × 8 rows 2.21/2.82, 2 × 4 2.09/2.57, 4 × 2 2.08/2.41, 8 × 1 2.08/2.26. Chains hold ≤ 32 rows; beyond
  // 8·32 sequences further chains queue behind the running ones.
  nch = B <= kMaxTeams * 32 ? (B < kMaxTeams ? B : kMaxTeams) : (B + 31) / 32;
  // F32 chains hold ≤ 16 rows (the backward's hi + lo gate-gradient images of 16 rows take 132 KB of LDS)
  if (f32 && (B + nch - 1) / nch > 16) nch = (B + 15) / 16;
  Bc = (B + nch - 1) / nch;
  MT = Bc <= 16 ? 1 : 2;
}

}  // namespace

// (F32_, V1_) = (0, 0) bf16 MFMA, (1, 0) bf16x3 MFMA, (1, 1) exact-fp32 VALU for one-row chains
#define DCA_TEAM_DISPATCH(MT_, KS_, F32_, V1_, ...)                                                        \
  switch (((V1_) << 12) | ((F32_) << 8) | ((MT_) << 4) | (KS_)) {   /* V1_ bit 4 (half teams) → 0x10000 */                                          \
    case 0x0011: return __VA_ARGS__(1, 1, false, 0); case 0x0012: return __VA_ARGS__(1, 2, false, 0); \
    case 0x0014: return __VA_ARGS__(1, 4, false, 0); case 0x0021: return __VA_ARGS__(2, 1, false, 0); \
    case 0x0022: return __VA_ARGS__(2, 2, false, 0); case 0x0024: return __VA_ARGS__(2, 4, false, 0); \
    case 0x0111: return __VA_ARGS__(1, 1, true, 0);  case 0x0112: return __VA_ARGS__(1, 2, true, 0);  \
    case 0x0114: return __VA_ARGS__(1, 4, true, 0);                                                      \
    case 0x1111: return __VA_ARGS__(1, 1, true, 1);      case 0x1112: return __VA_ARGS__(1, 2, true, 1);      \
    case 0x1114: return __VA_ARGS__(1, 4, true, 1);      case 0x2114: return __VA_ARGS__(1, 4, true, 2);      \
    case 0x5111: return __VA_ARGS__(1, 1, true, 5);      case 0x5112: return __VA_ARGS__(1, 2, true, 5);      \
    case 0x5114: return __VA_ARGS__(1, 4, true, 5);      case 0x6114: return __VA_ARGS__(1, 4, true, 6);      \
    case 0x11114: return __VA_ARGS__(1, 4, true, 17);                                                       \
    case 0x21111: return __VA_ARGS__(1, 1, true, 33);    case 0x21112: return __VA_ARGS__(1, 2, true, 33);   \
    case 0x21114: return __VA_ARGS__(1, 4, true, 33);    case 0x22114: return __VA_ARGS__(1, 4, true, 34);   \
    case 0x31114: return __VA_ARGS__(1, 4, true, 49);                                                       \
    case 0x41111: return __VA_ARGS__(1, 1, true, 65);    case 0x41112: return __VA_ARGS__(1, 2, true, 65);   \
    case 0x41114: return __VA_ARGS__(1, 4, true, 65);    case 0x42114: return __VA_ARGS__(1, 4, true, 66);   \
    case 0x51114: return __VA_ARGS__(1, 4, true, 81);                                                       \
    default: return hipErrorInvalidValue;                                                                    \
  }

// fp32 chains of ≤ 4 rows take the exact VALU variant; at H = 512 the backward takes its 8-wave form V2 (measured
// B=8, S=1400: backward 2069 vs 2137 µs, while the 8-wave forward was SLOWER, 2056 vs 1778 µs).
// half: the CU-exclusive 16-workgroup teams (V1 form in both directions, H = 512, fast activations).
inline int use_v1(int f32, int Bc, int H, int backward, int precise, int half = -1) {
  if (half < 0) {                        // read per launch (two launches per learner step): tests flip it
    const char* e = getenv("DCA_TEAM_HALF");
    half = e && e[0] == '1';
  }
  if (!(f32 && Bc <= 4)) return 0;
  const int rows = Bc == 1 ? 0 : (Bc == 2 ? 32 : 64);         // VAR bits 5-6: 2 or 4 rows per chain
  if (half && H == 512 && !precise) return 1 | 16 | rows;
  return ((H == 512 && backward) ? 2 : 1) | (precise ? 4 : 0) | rows;
}

// Workspace bytes (control block + per-team exchange buffers) for a launch of (B, H).
extern "C" size_t dca_lstm_team_ctl_bytes() { return 256; }

// Sequence chains a launch of B sequences is split into (rows of the backward's bias-gradient partials).
extern "C" int dca_lstm_team_chains(int B, int f32) {
  int nch, Bc, MT;
  plan(B, nch, Bc, MT, f32);
  return nch;
}

// Exchange-buffer bytes (per-team hand-off rings) for a launch of (B, H). Not zeroed: tags carry the epoch.
extern "C" size_t dca_lstm_team_workspace(int B, int H, int backward, int f32) {
  int nch, Bc, MT;
  plan(B, nch, Bc, MT, f32);
  if (!backward) return (size_t)kMaxTeams * 2 * Bc * (f32 ? H : H / 2) * 8;
  return (size_t)kMaxTeams * 2 * Bc * H * (f32 ? 2 : 1) * 16;
}

// whh: (4H,H) bf16 (f32 = 0) or fp32 (f32 = 1: bf16x3 split MFMA, h exchanged and stored in fp32, hs unused)
extern "C" hipError_t dca_lstm_team_fwd(const float* xp4, const void* whh, const float* h0, const float* c0,
                                        short* hs, float* hsf, float* cs, float* gates4, float* hn, float* cn,
                                        void* ctl_mem, void* ws, size_t ws_bytes, unsigned* err, int B, int S, int H,
                                        int time_major, hipStream_t stream, unsigned long long* trace,
                                        const float* bias4, int f32, int precise, const unsigned char* rst) {
  if (B < 1 || S < 1 || S >= 65535 || (H != 128 && H != 256 && H != 512)) return hipErrorInvalidValue;
  if (ws_bytes < dca_lstm_team_workspace(B, H, 0, f32) || ctl_mem == nullptr) return hipErrorInvalidValue;
  if (f32 && hsf == nullptr) return hipErrorInvalidValue;
  if (!f32 && hs == nullptr) return hipErrorInvalidValue;
  int nch, Bc, MT;
  plan(B, nch, Bc, MT, f32);
  const int sb = time_major ? 1 : S, st = time_major ? B : 1;   // row(b, t) = b·sb + t·st
  TeamCtl* ctl = reinterpret_cast<TeamCtl*>(ctl_mem);
  unsigned long long* xg = reinterpret_cast<unsigned long long*>(ws);
  const int KS = H / 128;
#define DCA_F(mt, ks, f, v)                                                                                     \
  (lstm_team_fwd_kernel<mt, ks, f, v><<<kMaxTeams * team_size(v), team_threads(v), 0, stream>>>(xp4, whh, h0, c0, hs, hsf, cs, gates4, \
                                                                          hn, cn, xg, ctl, err, B, Bc, nch, S, sb, \
                                                                          st, trace, team_knobs(), bias4, rst),    \
   hipGetLastError())
  DCA_TEAM_DISPATCH(MT, KS, f32 ? 1 : 0, use_v1(f32, Bc, H, 0, precise), DCA_F)
#undef DCA_F
}

extern "C" hipError_t dca_lstm_team_bwd(const float* dhs, const float* gates4, const float* cs, const float* c0,
                                        const float* dhn, const float* dcn, const void* whh, float* dgates4,
                                        float* dh0, float* dc0, void* ctl_mem, void* ws, size_t ws_bytes,
                                        unsigned* err, int B, int S, int H, int time_major, hipStream_t stream,
                                        unsigned long long* trace, short* dg16, float* dbpart, int f32, int precise,
                                        const unsigned char* rst) {
  if (B < 1 || S < 1 || S >= 65534 || (H != 128 && H != 256 && H != 512)) return hipErrorInvalidValue;
  if (dgates4 == nullptr && dg16 == nullptr) return hipErrorInvalidValue;
  if (f32 && dgates4 == nullptr) return hipErrorInvalidValue;
  if (ws_bytes < dca_lstm_team_workspace(B, H, 1, f32) || ctl_mem == nullptr) return hipErrorInvalidValue;
  int nch, Bc, MT;
  plan(B, nch, Bc, MT, f32);
  const int sb = time_major ? 1 : S, st = time_major ? B : 1;
  TeamCtl* ctl = reinterpret_cast<TeamCtl*>(ctl_mem);
  i32x4* xb = reinterpret_cast<i32x4*>(ws);
  const int KS = H / 128;
#define DCA_B(mt, ks, f, v)                                                                                        \
  (lstm_team_bwd_kernel<mt, ks, f, v><<<kMaxTeams * team_size(v), team_threads(v), 0, stream>>>(dhs, gates4, cs, c0, dhn, dcn, whh,      \
                                                                          dgates4, dh0, dc0, xb, ctl, err, B, Bc,  \
                                                                          nch, S, sb, st, trace, dg16, dbpart,      \
                                                                          team_knobs(), rst),                      \
   hipGetLastError())
  DCA_TEAM_DISPATCH(MT, KS, f32 ? 1 : 0, use_v1(f32, Bc, H, 1, precise), DCA_B)
#undef DCA_B
}
