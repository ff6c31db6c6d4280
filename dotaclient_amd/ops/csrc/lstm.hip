// Persistent LSTM recurrence kernels for gfx950 (forward and backward), the learner's dominant cost.
//
// North-star feature of BASELINE.json ("LSTM policy (4-gate GEMM + elementwise)"); the reference only sketches it
// (policy.py:67-68, 143-145). Non-recurrent work — the input projection x·W_ihᵀ over all timesteps and the weight
// gradients — are large GEMMs done outside; these kernels do only the strictly sequential part:
//
//   forward : gates_t = xp_t + h_{t-1}·W_hhᵀ ; (i,f,g,o) = (σ,σ,tanh,σ) ; c_t = f c_{t-1} + i g ; h_t = o tanh(c_t)
//   backward: dh_t = dH_t + dG_{t+1}·W_hh ; dc_t = dc_{t+1} f_{t+1} + dh_t o (1-tanh²c_t) ; dG_t = gate grads
//
// Decomposition (one launch for the whole sequence, W_hh resident in VGPRs):
//   * NWG = H/8 workgroups; workgroup w owns hidden units J_w = [8w, 8w+8) and the 32 gate rows {q·H + J_w}.
//     Its 32×H slice of W_hh (32 KB bf16 at H=512) lives in registers for all S steps (32 VGPRs per lane).
//   * forward : each step needs the full h_{t-1} (B×H) — an ALL-GATHER. Every workgroup publishes its B×8 slice of
//     h_t as data-tagged 8-byte granules {tag = t+1, 2×bf16} with agent-scope relaxed stores (write-through);
//     consumers poll the granules they need with agent-scope relaxed loads — the data IS the flag, no fence, no
//     barrier (cdna_hip_programming.md Guideline 16 R2; MI355X_MICROARCH.md 'allgather' price row).
//     Each wave owns a quarter of K and polls only that quarter; the 4 partial gate tiles are summed through LDS.
//   * backward: each step needs Σ over ALL 4H gate rows of dG·W_hh restricted to J_w — we REDUCE-SCATTER instead
//     of all-gathering dG: workgroup w multiplies its own 32 dG columns by its 32 W rows (B×H partial, MFMA) and
//     publishes it as {tag, f32} granules; workgroup w' sums the NWG partials for its 8 units. 4× less traffic
//     than gathering dG (B×H vs B×4H values) and the recurrent gradient is accumulated in fp32.
//   * granule rings are double-buffered by step parity: a workgroup can only write slot t&1 again after every
//     workgroup has consumed step t-1's data (it needs their step-t-1 output first), so no WAR hazard; tags are
//     step-unique so stale data is never mistaken for new. The ring is zeroed before each launch.
//   * every spin is bounded; on timeout a workgroup raises *err and all others bail out, so a residency problem
//     can never hang the GPU. The grid (≤ 64·chains workgroups of 256 threads) is always co-resident.
// MFMA: v_mfma_f32_16x16x32_bf16, batch rows in M (B ≤ 16·MT), gate columns / hidden units in N.
#include "common.h"
#include <cstdio>
#include <cstdlib>

namespace {

using dca::bf16x8;
using gu64 = __attribute__((address_space(1))) unsigned long long;
using gu32 = __attribute__((address_space(1))) unsigned int;

constexpr int kUw = 8;                  // hidden units per workgroup
constexpr int kSc1 = 16;                // buffer-op cache policy: sc1 = agent-coherent (bypasses the per-XCD L2)
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
constexpr unsigned kSpinLimit = 1u << 21;

__device__ __forceinline__ unsigned long long ld_granule(const unsigned long long* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_granule(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned ld_err(const unsigned* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void raise_err(unsigned* p, unsigned code) {
  __hip_atomic_store((gu32*)p, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Bounded-spin bookkeeping shared by all polls of a wave. Returns true when the wave must give up.
__device__ __forceinline__ bool spin_fail(unsigned& spins, unsigned* err, unsigned code) {
  asm volatile("" ::: "memory");   // compiler barrier: the next poll round's buffer loads must be re-issued
  ++spins;
  if ((spins & 255u) == 0) {
    if (ld_err(err) != 0) return true;
    if (spins > kSpinLimit) {
      raise_err(err, code);
      return true;
    }
  }
  if (spins > 64) __builtin_amdgcn_s_sleep(1);
  return false;
}

__device__ __forceinline__ void sleep_n(int n) {
  for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(1);
}

// Buffer resource for a wave-uniform base pointer. readfirstlane makes the uniformity explicit: code inside
// role branches (poller / publisher) is divergent to the compiler, which would otherwise keep the descriptor in
// VGPRs and wrap every buffer load in a waterfall loop.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, int bytes) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// One workgroup-wide rendezvous that orders LDS traffic only. Unlike __syncthreads() it does NOT wait for
// outstanding global stores/loads (no vmcnt(0)), so a wave's in-flight granule or output stores never stall the
// others (cdna_hip_programming.md §5 "Pipelining across barriers"). The "memory" clobber stops the compiler from
// moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// =============================================================================================================
// Forward — 5 waves: waves 0-3 are POLLERS (gather h_{t-1} for their K quarter, prefetch x·W_ihᵀ, MFMA, write
// partial gates to LDS; they never store to global memory, so their polls never wait behind store completion),
// wave 4 is the PUBLISHER (sums the partials, cell update, publishes h_t granules + outputs; it never loads
// global memory inside the loop, so its stores never stall it). One LDS-only barrier per step.
// =============================================================================================================
// xp     (B, S, 4H) f32  input projection incl. both biases
// whh    (4H, H)    bf16 recurrent weights (PyTorch layout, gate order i,f,g,o)
// h0,c0  (B, H)     f32
// hs     (B, S, H)  bf16 out: h_t          hsf (B,S,H) f32 out (optional)
// cs     (B, S, H)  f32  out: c_t          gates (B,S,4H) f32 out: activated i, f, g, o
// hn,cn  (B, H)     f32  out: final state
// ring   (2, B, H/2) u64 granules {tag = t+1, 2×bf16 h} (zeroed before launch)
constexpr int kFwdThreads = 320;
constexpr int kBwdThreads = 512;
constexpr int kMaxPairs = 512;   // B·8 ≤ 512

template <int MT, int KS>
__global__ __launch_bounds__(kFwdThreads) void lstm_fwd_kernel(const float* __restrict__ xp,
                                                               const short* __restrict__ whh,
                                                               const float* __restrict__ h0,
                                                               const float* __restrict__ c0, short* __restrict__ hs,
                                                               float* __restrict__ hsf, float* __restrict__ cs,
                                                               float* __restrict__ gates, float* __restrict__ hn,
                                                               float* __restrict__ cn, unsigned long long* ring,
                                                               unsigned* err, int Btot, int Bc, int S,
                                                               unsigned long long* trace, int pre_sleep,
                                                               int spin_sleep) {
  constexpr int H = 128 * KS;
  constexpr int G4 = 4 * H;
  constexpr int HP = H / 2;
  // optional in-kernel timestamps (s_memrealtime, 100 MHz, chip-wide) for the first 64 steps: trace[wg][wave][t][ev]
#define DCA_TSTAMP(ev)                                                                                   \
  if (trace && lane == 0 && t < 64)                                                                       \
    trace[(((size_t)blockIdx.x * 8 + wv) * 64 + t) * 8 + (ev)] = __builtin_amdgcn_s_memrealtime()
  // independent chains of ≤ 16·MT sequences run side by side in one launch (blockIdx = chain·NWG + w)
  const int chain = blockIdx.x / (H / kUw);
  const int b0 = chain * Bc;
  const int B = min(Bc, Btot - b0);
  xp += (size_t)b0 * S * G4; h0 += (size_t)b0 * H; c0 += (size_t)b0 * H; hs += (size_t)b0 * S * H;
  if (hsf) hsf += (size_t)b0 * S * H;
  cs += (size_t)b0 * S * H; gates += (size_t)b0 * S * G4; hn += (size_t)b0 * H; cn += (size_t)b0 * H;
  ring += (size_t)chain * 2 * Bc * HP;
  const int w = blockIdx.x % (H / kUw);
  const int j0 = w * kUw;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int lrow = lane & 15, lkg = lane >> 4;
  const int P = B * kUw;

  constexpr int PMAX = 128 * MT;        // pairs (B·8) this instantiation supports
  __shared__ float red[2][4][MT][2][16][17];
  __shared__ float xpl[2][4][PMAX];
  __shared__ int abort_flag;
  __shared__ int pub_issued;               // last step whose h granules this workgroup's publisher has issued
  if (tid == 0) { abort_flag = 0; pub_issued = 0; }
  __syncthreads();

  const bool poller = wv < 4;
  bf16x8 wf[2][KS];
  if (poller) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int c = nt * 16 + lrow;
      const int row = (c >> 3) * H + j0 + (c & 7);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int k = wv * (32 * KS) + ks * 32 + 8 * lkg;
        wf[nt][ks] = *reinterpret_cast<const bf16x8*>(whh + (size_t)row * H + k);
      }
    }
  }
  // publisher state: pairs p = lane + 64·r
  constexpr int NPR = PMAX / 64;
  float creg[NPR], hreg[NPR];
  if (!poller) {
#pragma unroll
    for (int r = 0; r < NPR; ++r) {
      const int p = lane + 64 * r;
      creg[r] = hreg[r] = 0.f;
      if (p < P) {
        creg[r] = c0[(p >> 3) * H + j0 + (p & 7)];
        hreg[r] = h0[(p >> 3) * H + j0 + (p & 7)];
      }
    }
  }

  unsigned spins = 0;
  for (int t = 0; t < S; ++t) {
    const int par = t & 1;
    if (poller) {
      DCA_TSTAMP(0);
      // -------- prefetch this step's x·W_ihᵀ values (4 per pair) — issued before the poll, consumed after it
      constexpr int NXV = (4 * PMAX) / 256;
      float xv[NXV];
#pragma unroll
      for (int i = 0; i < NXV; ++i) {
        const int idx = tid + 256 * i;
        xv[i] = 0.f;
        if (idx < 4 * P) {
          const int p = idx >> 2, q = idx & 3;
          xv[i] = xp[((size_t)(p >> 3) * S + t) * G4 + q * H + j0 + (p & 7)];
        }
      }
      // -------- A fragments of h_{t-1} for this wave's K quarter
      bf16x8 af[MT][KS];
      bool dead = false;
      if (t == 0) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            const int b = mt * 16 + lrow;
            const int k = wv * (32 * KS) + ks * 32 + 8 * lkg;
            bf16x8 v;
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = (b < B) ? dca::f2bf(h0[b * H + k + j]) : (short)0;
            af[mt][ks] = v;
          }
      } else {
        const unsigned long long* slot = ring + (size_t)((t - 1) & 1) * B * HP;
        const unsigned tag = (unsigned)t;
        // Data-carrying poll: each fragment (8 h values of one batch row = 4 granules = 32 contiguous bytes, all
        // written by ONE producer store instruction) is read with two 16-byte agent-coherent (sc1) buffer loads —
        // the poll IS the fetch, so a step costs one hand-off round trip, and every load of a round is in flight
        // before any tag is inspected. Buffer loads (unlike atomic/volatile loads) are not serialised by the
        // compiler; the spin loop's side effects keep them inside the loop.
        const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(slot, B * HP * 8);
        i32x4 g2[MT][KS][2];
        // Do not poll before this workgroup's own publisher has ISSUED its step t-1 granule stores: polls queue in
        // the same per-CU vector-memory path and would delay that store — and no other workgroup's data can be
        // expected much earlier, all of them run in lockstep. The wait is LDS-only.
        while (*(volatile int*)&pub_issued < t) __builtin_amdgcn_s_sleep(0);
        sleep_n(pre_sleep);
        while (true) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
              const int b = mt * 16 + lrow;
              const int k = wv * (32 * KS) + ks * 32 + 8 * lkg;
              const int off = (b * HP + (k >> 1)) * 8;
              if (b < B) {
                g2[mt][ks][0] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kSc1);
                g2[mt][ks][1] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, kSc1);
              }
            }
          bool ok = true;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
              if (mt * 16 + lrow < B)
                ok &= ((unsigned)g2[mt][ks][0].y == tag) & ((unsigned)g2[mt][ks][0].w == tag) &
                      ((unsigned)g2[mt][ks][1].y == tag) & ((unsigned)g2[mt][ks][1].w == tag);
          if (__all(ok)) break;
          if (spin_fail(spins, err, 1u)) { dead = true; break; }
          sleep_n(spin_sleep);
        }
        DCA_TSTAMP(1);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            const bool valid = mt * 16 + lrow < B;
            const unsigned pl[4] = {(unsigned)g2[mt][ks][0].x, (unsigned)g2[mt][ks][0].z, (unsigned)g2[mt][ks][1].x,
                                    (unsigned)g2[mt][ks][1].z};
            bf16x8 v;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const unsigned u = valid ? pl[q] : 0u;
              v[2 * q] = (short)(u & 0xffffu);
              v[2 * q + 1] = (short)(u >> 16);
            }
            af[mt][ks] = v;
          }
      }
      DCA_TSTAMP(2);
      if (dead && lane == 0) abort_flag = 1;
      // -------- partial gates over this wave's K quarter → LDS
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          dca::f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt][ks], wf[nt][ks], acc, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) red[par][wv][mt][nt][lkg * 4 + r][lrow] = acc[r];
        }
#pragma unroll
      for (int i = 0; i < NXV; ++i) {
        const int idx = tid + 256 * i;
        if (idx < 4 * P) xpl[par][idx & 3][idx >> 2] = xv[i];
      }
      DCA_TSTAMP(3);
    }
    lds_barrier();
    if (abort_flag) break;
    if (!poller) {
      DCA_TSTAMP(4);
      // -------- cell update for every owned pair; publish the h_t granules FIRST (the next step's critical path),
      // then the bulky per-step outputs, so the hand-off stores are never queued behind them.
      float gi[NPR], gf[NPR], gg_[NPR], go[NPR];
#pragma unroll
      for (int r = 0; r < NPR; ++r) {
        const int p = lane + 64 * r;
        gi[r] = gf[r] = gg_[r] = go[r] = 0.f;
        if (64 * r >= P) continue;                  // wave-uniform
        float hv = 0.f;
        if (p < P) {
          const int b = p >> 3, jj = p & 7;
          const int mt = b >> 4, row = b & 15;
          float pre[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c = q * kUw + jj;
            const int nt = c >> 4, cc = c & 15;
            pre[q] = red[par][0][mt][nt][row][cc] + red[par][1][mt][nt][row][cc] + red[par][2][mt][nt][row][cc] +
                     red[par][3][mt][nt][row][cc] + xpl[par][q][p];
          }
          gi[r] = dca::sigmoidf_(pre[0]);
          gf[r] = dca::sigmoidf_(pre[1]);
          gg_[r] = dca::tanhf_(pre[2]);
          go[r] = dca::sigmoidf_(pre[3]);
          const float c = gf[r] * creg[r] + gi[r] * gg_[r];
          hv = go[r] * dca::tanhf_(c);
          creg[r] = c;
          hreg[r] = hv;
        }
        const float hnext = __shfl_down(hv, 1, 64);
        if (p < P && (p & 1) == 0) {
          const int b = p >> 3, jj = p & 7;
          const unsigned pl = (unsigned)(unsigned short)dca::f2bf(hv) |
                              ((unsigned)(unsigned short)dca::f2bf(hnext) << 16);
          st_granule(ring + (size_t)par * B * HP + (size_t)b * HP + ((j0 + jj) >> 1),
                     ((unsigned long long)(unsigned)(t + 1) << 32) | pl);
        }
      }
      if (lane == 0) *(volatile int*)&pub_issued = t + 1;
      DCA_TSTAMP(6);
#pragma unroll
      for (int r = 0; r < NPR; ++r) {
        const int p = lane + 64 * r;
        if (64 * r >= P) break;                     // wave-uniform
        if (p < P) {
          const int b = p >> 3, jj = p & 7;
          const size_t bt = (size_t)b * S + t;
          hs[bt * H + j0 + jj] = dca::f2bf(hreg[r]);
          if (hsf) hsf[bt * H + j0 + jj] = hreg[r];
          cs[bt * H + j0 + jj] = creg[r];
          float* gp = gates + bt * G4 + j0 + jj;
          gp[0] = gi[r];
          gp[H] = gf[r];
          gp[2 * H] = gg_[r];
          gp[3 * H] = go[r];
        }
      }
      DCA_TSTAMP(5);
    }
  }
#undef DCA_TSTAMP
  if (!poller && !abort_flag) {
#pragma unroll
    for (int r = 0; r < NPR; ++r) {
      const int p = lane + 64 * r;
      if (p < P) {
        hn[(p >> 3) * H + j0 + (p & 7)] = hreg[r];
        cn[(p >> 3) * H + j0 + (p & 7)] = creg[r];
      }
    }
  }
}

// =============================================================================================================
// Backward — 8 waves: waves 0-3 are POLLERS (gather Σ partials of step t+1 for the owned units and prefetch the
// step's saved activations into LDS; no global stores), waves 4-7 are PUBLISHERS (each recomputes the owned units'
// gate gradients from LDS — redundantly, so no publisher-side barrier is needed — then multiplies its own quarter
// of the W slice and publishes the B×H/4 partial as {tag, f32} granules; wave 4 also writes ∂gates).
// =============================================================================================================
// dhs    (B, S, H)  f32  ∂L/∂h_t from everything above the LSTM
// gates  (B, S, 4H) f32  activated gates;  cs (B,S,H) f32 c_t;  c0 (B,H)
// dhn,dcn(B, H)     f32  ∂L/∂(h_S, c_S) (may be null)
// dgates (B, S, 4H) f32  out: ∂L/∂(gate pre-activations);  dh0, dc0 (B,H) out
// ring   (2, B, NWG consumers, NWG producers, 2 quads) 16-byte chunks {2×bf16, tag, 2×bf16, tag} (zeroed)
template <int MT, int KS>
__global__ __launch_bounds__(kBwdThreads) void lstm_bwd_kernel(const float* __restrict__ dhs,
                                                               const float* __restrict__ gates,
                                                               const float* __restrict__ cs,
                                                               const float* __restrict__ c0,
                                                               const float* __restrict__ dhn,
                                                               const float* __restrict__ dcn,
                                                               const short* __restrict__ whh,
                                                               float* __restrict__ dgates, float* __restrict__ dh0,
                                                               float* __restrict__ dc0, unsigned long long* ring,
                                                               unsigned* err, int Btot, int Bc, int S,
                                                               int pre_sleep, int spin_sleep,
                                                               unsigned long long* trace) {
#define DCA_TSTAMPB(ev)                                                                                  \
  if (trace && lane == 0 && k < 64)                                                                       \
    trace[(((size_t)blockIdx.x * 8 + wv) * 64 + k) * 8 + (ev)] = __builtin_amdgcn_s_memrealtime()
  constexpr int H = 128 * KS;
  constexpr int G4 = 4 * H;
  constexpr int NWG = H / kUw;
  constexpr int NT_W = H / 64;          // 16-column N tiles per publisher wave
  const int chain = blockIdx.x / NWG;
  const int b0 = chain * Bc;
  const int B = min(Bc, Btot - b0);
  dhs += (size_t)b0 * S * H; gates += (size_t)b0 * S * G4; cs += (size_t)b0 * S * H; c0 += (size_t)b0 * H;
  if (dhn) dhn += (size_t)b0 * H;
  if (dcn) dcn += (size_t)b0 * H;
  dgates += (size_t)b0 * S * G4; dh0 += (size_t)b0 * H; dc0 += (size_t)b0 * H;
  ring += (size_t)chain * 2 * NWG * Bc * H;
  const int w = blockIdx.x % NWG;
  const int j0 = w * kUw;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int lrow = lane & 15, lkg = lane >> 4;
  const int P = B * kUw;
  const bool poller = wv < 4;
  const int pw = wv - 4;

  constexpr int PMAX = 128 * MT;
  constexpr int NSLOT = (NWG * 2) / 64 > 0 ? (NWG * 2) / 64 : 1;   // LDS partial slots (producer groups per row)
  __shared__ float dpart[2][NSLOT][PMAX];
  __shared__ float inp[2][7][PMAX];        // i, f, g, o, c_t, c_{t-1}, dhs_t
  __shared__ short dgl[4][MT * 16][40];
  constexpr int SC = NT_W * 16 + 8;        // staging row pitch (bf16), padded
  __shared__ unsigned short stg[4][MT * 16][SC];
  __shared__ int abort_flag;
  __shared__ int pub_cnt;                  // publisher waves that issued their partial stores (4 per step)
  if (tid == 0) { abort_flag = 0; pub_cnt = 0; }
  for (int i = tid; i < 4 * MT * 16 * 40; i += kBwdThreads) (&dgl[0][0][0])[i] = 0;
  __syncthreads();

  bf16x8 wf[NT_W];
  constexpr int NPR = PMAX / 64;
  float dcreg[NPR];
  if (!poller) {
#pragma unroll
    for (int n = 0; n < NT_W; ++n) {
      const int col = (pw * NT_W + n) * 16 + lrow;
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = whh[(size_t)(lkg * H + j0 + j) * H + col];
      wf[n] = v;
    }
#pragma unroll
    for (int r = 0; r < NPR; ++r) {
      const int p = lane + 64 * r;
      dcreg[r] = (p < P && dcn) ? dcn[(p >> 3) * H + j0 + (p & 7)] : 0.f;
    }
  }

  unsigned spins = 0;
  for (int k = 0; k <= S; ++k) {
    const int t = S - 1 - k;            // step handled by the publishers this iteration (-1: final gather)
    const int par = k & 1;
    if (poller) {
      // -------- prefetch the saved activations of step t (7 values per pair)
      constexpr int NIN = (7 * PMAX + 255) / 256;
      float iv[NIN];
      if (t >= 0) {
        // branch-free address selection so every load of the prefetch is in flight together
#pragma unroll
        for (int i = 0; i < NIN; ++i) {
          const int idx0 = tid + 256 * i;
          const int idx = idx0 < 7 * P ? idx0 : 0;
          const int p = idx % P, f = idx / P;
          const int b = p >> 3, jj = p & 7;
          const size_t bt = (size_t)b * S + t;
          const float* src = gates + bt * G4 + (f & 3) * H + j0 + jj;
          src = (f == 4) ? cs + bt * H + j0 + jj : src;
          src = (f == 5) ? ((t > 0) ? cs + (bt - 1) * H + j0 + jj : c0 + b * H + j0 + jj) : src;
          src = (f == 6) ? dhs + bt * H + j0 + jj : src;
          iv[i] = *src;
        }
      }
      // -------- recurrent gradient for h_t: Σ_w' partial_{w'} of step t+1 (k = 0: the given ∂L/∂h_S).
      // Ring layout (parity, b, consumer, producer, unit): the NWG×8 partials this workgroup needs for one batch row
      // are one contiguous block, read as 16-byte chunks {2 units of one producer} by all 256 poller lanes with
      // sc1 buffer loads — data-carrying polls, every load of a group of 8 rows in flight at once. The sum over
      // producers is a lane-shuffle tree (producers differ in lane bits 2..5) plus the per-wave LDS slots
      // (dpart[.][pslot]) that the publishers add up.
      DCA_TSTAMPB(0);
      bool dead = false;
      constexpr int CPR = NWG * 2;                    // 16-byte chunks {2 granules, 4 units} per batch row block
      constexpr int RPP = 256 / CPR;                  // rows covered per load slot (2, 4 or 8)
      constexpr int NLD = 8 / RPP;                    // loads per lane per group of 8 rows
      constexpr int LSPAN = CPR < 64 ? CPR : 64;      // lanes of one row inside a wave
      const int chunk = tid % CPR, ro = tid / CPR;
      const int pslot = (tid >> 6) % NSLOT;
      if (k == 0) {
        for (int p = tid; p < P; p += 256) {
          const float v = dhn ? dhn[(p >> 3) * H + j0 + (p & 7)] : 0.f;
#pragma unroll
          for (int sl = 0; sl < NSLOT; ++sl) dpart[par][sl][p] = sl == 0 ? v : 0.f;
        }
      } else {
        const unsigned long long* slot = ring + (size_t)((t + 1) & 1) * B * NWG * NWG * 4 + (size_t)w * NWG * 4;
        const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(slot, ((B - 1) * NWG * NWG * 4 + NWG * 4) * 8);
        const unsigned tag = (unsigned)(t + 2);
        for (int g0 = 0; g0 < B && !dead; g0 += 8) {
          i32x4 g2[NLD];
          if (g0 == 0) {
            while (*(volatile int*)&pub_cnt < 4 * k) __builtin_amdgcn_s_sleep(0);   // see the forward
            sleep_n(pre_sleep);
          }
          while (true) {
#pragma unroll
            for (int i = 0; i < NLD; ++i) {
              const int b = g0 + i * RPP + ro;
              if (b < B) g2[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (b * NWG * NWG * 2 + chunk) * 16, 0, kSc1);
            }
            bool ok = true;
#pragma unroll
            for (int i = 0; i < NLD; ++i)
              if (g0 + i * RPP + ro < B) ok &= ((unsigned)g2[i].y == tag) & ((unsigned)g2[i].w == tag);
            if (__all(ok)) break;
            if (spin_fail(spins, err, 2u)) { dead = true; break; }
            sleep_n(spin_sleep);
          }
#pragma unroll
          for (int i = 0; i < NLD; ++i) {
            float sv[4];
            const unsigned x = (unsigned)g2[i].x, z = (unsigned)g2[i].z;
            sv[0] = __uint_as_float(x << 16); sv[1] = __uint_as_float(x & 0xffff0000u);
            sv[2] = __uint_as_float(z << 16); sv[3] = __uint_as_float(z & 0xffff0000u);
#pragma unroll
            for (int o = 2; o < LSPAN; o <<= 1)
#pragma unroll
              for (int q = 0; q < 4; ++q) sv[q] += __shfl_xor(sv[q], o, 64);
            const int b = g0 + i * RPP + ro;
            if ((lane % LSPAN) < 2 && b < B) {
#pragma unroll
              for (int q = 0; q < 4; ++q) dpart[par][pslot][b * kUw + (lane & 1) * 4 + q] = sv[q];
            }
          }
        }
      }
      DCA_TSTAMPB(1);
      if (dead && lane == 0) abort_flag = 1;
      if (t >= 0) {
#pragma unroll
        for (int i = 0; i < NIN; ++i) {
          const int idx = tid + 256 * i;
          if (idx < 7 * P) inp[par][idx / P][idx % P] = iv[i];
        }
      }
      DCA_TSTAMPB(2);
    }
    lds_barrier();
    if (abort_flag) break;
    if (t < 0) {
      // final gather done: ∂L/∂h0
      if (poller) {
        for (int p = tid; p < P; p += 256)
        {
          float v = 0.f;
#pragma unroll
          for (int sl = 0; sl < NSLOT; ++sl) v += dpart[par][sl][p];
          dh0[(p >> 3) * H + j0 + (p & 7)] = v;
        }
      }
      break;
    }
    if (!poller) {
      DCA_TSTAMPB(3);
      // -------- gate gradients of the owned units (every publisher wave computes all pairs)
      float dgr[NPR][4];
#pragma unroll
      for (int r = 0; r < NPR; ++r) {
        const int p = lane + 64 * r;
        if (64 * r >= P) break;
        if (p < P) {
          const int b = p >> 3, jj = p & 7;
          const float ig = inp[par][0][p], fg = inp[par][1][p], gg = inp[par][2][p], og = inp[par][3][p];
          const float c = inp[par][4][p], cprev = inp[par][5][p];
          float dht = inp[par][6][p];
#pragma unroll
          for (int sl = 0; sl < NSLOT; ++sl) dht += dpart[par][sl][p];
          const float tc = dca::tanhf_(c);
          const float dc = dcreg[r] + dht * og * (1.f - tc * tc);
          dgr[r][3] = dht * tc * og * (1.f - og);
          dgr[r][0] = dc * gg * ig * (1.f - ig);
          dgr[r][1] = dc * cprev * fg * (1.f - fg);
          dgr[r][2] = dc * ig * (1.f - gg * gg);
          dcreg[r] = dc * fg;
#pragma unroll
          for (int q = 0; q < 4; ++q) dgl[pw][b][q * 8 + jj] = dca::f2bf(dgr[r][q]);
        }
      }
      DCA_TSTAMPB(4);
      // -------- partial = dG_blk (B×32) · W_blk (32 × this wave's H/4 columns) → hand-off chunks of step t.
      // Chunk = 16 bytes {bf16 u0,u1 | tag | bf16 u2,u3 | tag} per (row, consumer, producer, unit quad). Store
      // instructions, not bytes, are what a CU's memory path pays for, so the accumulator tiles are transposed
      // through LDS (bf16) and every lane then stores whole chunks: B·H/64/64 full-wave stores instead of 4 per
      // 16-column tile.
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&dgl[pw][mt * 16 + lrow][8 * lkg]);
#pragma unroll
        for (int n = 0; n < NT_W; ++n) {
          dca::f32x4 acc = {0.f, 0.f, 0.f, 0.f};
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[n], acc, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) stg[pw][mt * 16 + lkg * 4 + r][n * 16 + lrow] = (unsigned short)dca::f2bf(acc[r]);
        }
      }
      {
        const __amdgpu_buffer_rsrc_t ws = uniform_rsrc(ring + (size_t)(t & 1) * B * NWG * NWG * 4, B * NWG * NWG * 32);
        const int tg = t + 1;
        constexpr int QPR = NT_W * 4;                 // unit quads per row in this wave's columns
        const int nq = B * QPR;
        for (int qi = lane; qi < nq; qi += 64) {
          const int b = qi / QPR, cq = qi % QPR;
          const uint2 v = *reinterpret_cast<const uint2*>(&stg[pw][b][cq * 4]);
          const int col = pw * NT_W * 16 + cq * 4;
          const i32x4 cv = {(int)v.x, tg, (int)v.y, tg};
          __builtin_amdgcn_raw_buffer_store_b128(cv, ws, (((b * NWG + (col >> 3)) * NWG + w) * 2 + ((col & 7) >> 2)) * 16,
                                                 0, kSc1);
        }
      }
      if (lane == 0) atomicAdd(&pub_cnt, 1);
      DCA_TSTAMPB(5);
      // -------- ∂gates outputs (off the hand-off critical path)
      if (pw == 0) {
#pragma unroll
        for (int r = 0; r < NPR; ++r) {
          const int p = lane + 64 * r;
          if (64 * r >= P) break;
          if (p < P) {
            const int b = p >> 3, jj = p & 7;
            float* dg = dgates + ((size_t)b * S + t) * G4 + j0 + jj;
            dg[0] = dgr[r][0];
            dg[H] = dgr[r][1];
            dg[2 * H] = dgr[r][2];
            dg[3 * H] = dgr[r][3];
            if (t == 0) dc0[b * H + j0 + jj] = dcreg[r];
          }
        }
      }
      DCA_TSTAMPB(6);
    }
  }
#undef DCA_TSTAMPB
}

// Tuning knobs (s_sleep counts before the first poll / after a failed poll round) for fwd and bwd, read from
// DCA_LSTM_KNOBS="fpre,fspin,bpre,bspin" on every launch (default 0 0 0 0) — for latency experiments only.
inline int knob(int i) {
  const char* e = getenv("DCA_LSTM_KNOBS");
  if (!e) return 0;
  int v[4] = {0, 0, 0, 0};
  sscanf(e, "%d,%d,%d,%d", &v[0], &v[1], &v[2], &v[3]);
  return v[i];
}

// Chains: sequences are split into independent groups of Bc ≤ 16·MT (MT ≤ 2 keeps every variant spill-free), all
// run concurrently. Total workgroups = chains·H/8 ≤ 256 so every chain is co-resident.
inline void plan_chains(int B, int H, int& nch, int& Bc, int& MT) {
  const int nwg = H / kUw;
  const int max_ch = 256 / nwg;
  nch = (B + 31) / 32;
  if (nch > max_ch) nch = max_ch;
  Bc = (B + nch - 1) / nch;
  MT = Bc <= 16 ? 1 : 2;
}

template <int MT, int KS>
hipError_t launch_fwd(const float* xp, const short* whh, const float* h0, const float* c0, short* hs, float* hsf,
                      float* cs, float* gates, float* hn, float* cn, unsigned long long* ring, unsigned* err, int B,
                      int Bc, int nch, int S, unsigned long long* trace, hipStream_t st) {
  constexpr int H = 128 * KS;
  hipError_t e = hipMemsetAsync(ring, 0, sizeof(unsigned long long) * (size_t)nch * 2 * Bc * (H / 2), st);
  if (e != hipSuccess) return e;
  lstm_fwd_kernel<MT, KS><<<nch * (H / kUw), kFwdThreads, 0, st>>>(xp, whh, h0, c0, hs, hsf, cs, gates, hn, cn,
                                                                   ring, err, B, Bc, S, trace, knob(0), knob(1));
  return hipGetLastError();
}

template <int MT, int KS>
hipError_t launch_bwd(const float* dhs, const float* gates, const float* cs, const float* c0, const float* dhn,
                      const float* dcn, const short* whh, float* dgates, float* dh0, float* dc0,
                      unsigned long long* ring, unsigned* err, int B, int Bc, int nch, int S,
                      unsigned long long* trace, hipStream_t st) {
  constexpr int H = 128 * KS;
  hipError_t e = hipMemsetAsync(ring, 0, sizeof(unsigned long long) * (size_t)nch * 2 * (H / kUw) * Bc * H, st);
  if (e != hipSuccess) return e;
  lstm_bwd_kernel<MT, KS><<<nch * (H / kUw), kBwdThreads, 0, st>>>(dhs, gates, cs, c0, dhn, dcn, whh, dgates, dh0,
                                                                   dc0, ring, err, B, Bc, S, knob(2), knob(3), trace);
  return hipGetLastError();
}

}  // namespace

#define DCA_DISPATCH_MT_KS(MT_, KS_, ...)                                           \
  switch (((MT_) << 4) | (KS_)) {                                                  \
    case 0x11: return __VA_ARGS__(1, 1); case 0x12: return __VA_ARGS__(1, 2);      \
    case 0x14: return __VA_ARGS__(1, 4); case 0x21: return __VA_ARGS__(2, 1);      \
    case 0x22: return __VA_ARGS__(2, 2); case 0x24: return __VA_ARGS__(2, 4);      \
    default: return hipErrorInvalidValue;                                          \
  }

static bool lstm_shape_ok(int B, int H) {
  if (B < 1 || (H != 128 && H != 256 && H != 512)) return false;
  return B <= 32 * (256 / (H / kUw));
}

// Max batch per launch for hidden size H (chains of ≤ 32 sequences, ≤ 256 workgroups).
extern "C" int dca_lstm_max_batch(int H) { return 32 * (256 / (H / kUw)); }

// Ring sizes (u64 elements) for the chain plan of (B, H).
extern "C" size_t dca_lstm_ring_elems(int B, int H, int backward) {
  int nch, Bc, MT;
  plan_chains(B, H, nch, Bc, MT);
  return backward ? (size_t)nch * 2 * (H / kUw) * Bc * H : (size_t)nch * 2 * Bc * (H / 2);
}

extern "C" hipError_t dca_lstm_fwd(const float* xp, const short* whh, const float* h0, const float* c0, short* hs,
                                   float* hsf, float* cs, float* gates, float* hn, float* cn,
                                   unsigned long long* ring, unsigned* err, int B, int S, int H, hipStream_t st,
                                   unsigned long long* trace) {
  if (!lstm_shape_ok(B, H) || S < 1) return hipErrorInvalidValue;
  int nch, Bc, MT;
  plan_chains(B, H, nch, Bc, MT);
  const int KS = H / 128;
#define DCA_F(mt, ks) launch_fwd<mt, ks>(xp, whh, h0, c0, hs, hsf, cs, gates, hn, cn, ring, err, B, Bc, nch, S, trace, st)
  DCA_DISPATCH_MT_KS(MT, KS, DCA_F)
#undef DCA_F
}

extern "C" hipError_t dca_lstm_bwd(const float* dhs, const float* gates, const float* cs, const float* c0,
                                   const float* dhn, const float* dcn, const short* whh, float* dgates, float* dh0,
                                   float* dc0, unsigned long long* ring, unsigned* err, int B, int S, int H,
                                   hipStream_t st, unsigned long long* trace) {
  if (!lstm_shape_ok(B, H) || S < 1) return hipErrorInvalidValue;
  int nch, Bc, MT;
  plan_chains(B, H, nch, Bc, MT);
  const int KS = H / 128;
#define DCA_B(mt, ks) launch_bwd<mt, ks>(dhs, gates, cs, c0, dhn, dcn, whh, dgates, dh0, dc0, ring, err, B, Bc, nch, S, trace, st)
  DCA_DISPATCH_MT_KS(MT, KS, DCA_B)
#undef DCA_B
}
