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

namespace {

using dca::bf16x8;
using gu64 = __attribute__((address_space(1))) unsigned long long;
using gu32 = __attribute__((address_space(1))) unsigned int;

constexpr int kUw = 8;                  // hidden units per workgroup
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
                                                               unsigned long long* trace) {
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
  if (tid == 0) abort_flag = 0;
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
        // Two-phase poll. (1) PROBE: one granule per fragment (each 8-value fragment comes from exactly one
        // producer workgroup) until every probed tag matches — cheap, so spinning does not flood the memory
        // system. (2) FETCH: issue every granule load before looking at any result (relaxed atomic loads are
        // ordered for the scheduler: interleaved load/use would serialise them), verify, refetch if needed.
        unsigned long long gr[MT][KS][4];
        while (true) {
          bool ok = true;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
              const int b = mt * 16 + lrow;
              const int k = wv * (32 * KS) + ks * 32 + 8 * lkg;
              if (b < B) gr[mt][ks][3] = ld_granule(slot + (size_t)b * HP + (k >> 1) + 3);
            }
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
              if (mt * 16 + lrow < B) ok &= (unsigned)(gr[mt][ks][3] >> 32) == tag;
          if (__all(ok)) break;
          if (spin_fail(spins, err, 1u)) { dead = true; break; }
        }
        DCA_TSTAMP(1);
        while (!dead) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
              const int b = mt * 16 + lrow;
              const int k = wv * (32 * KS) + ks * 32 + 8 * lkg;
              if (b < B) {
                const unsigned long long* g = slot + (size_t)b * HP + (k >> 1);
#pragma unroll
                for (int q = 0; q < 4; ++q) gr[mt][ks][q] = ld_granule(g + q);
              }
            }
          bool ok = true;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
              if (mt * 16 + lrow < B) {
#pragma unroll
                for (int q = 0; q < 4; ++q) ok &= (unsigned)(gr[mt][ks][q] >> 32) == tag;
              }
          if (__all(ok)) break;
          if (spin_fail(spins, err, 1u)) { dead = true; break; }
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            const bool valid = mt * 16 + lrow < B;
            bf16x8 v;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const unsigned pl = valid ? (unsigned)gr[mt][ks][q] : 0u;
              v[2 * q] = (short)(pl & 0xffffu);
              v[2 * q + 1] = (short)(pl >> 16);
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
      // -------- cell update for every owned pair, publish h_t
#pragma unroll
      for (int r = 0; r < NPR; ++r) {
        const int p = lane + 64 * r;
        if (64 * r >= P) break;                     // wave-uniform
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
          const float ig = dca::sigmoidf_(pre[0]);
          const float fg = dca::sigmoidf_(pre[1]);
          const float gg = dca::tanhf_(pre[2]);
          const float og = dca::sigmoidf_(pre[3]);
          const float c = fg * creg[r] + ig * gg;
          hv = og * dca::tanhf_(c);
          creg[r] = c;
          hreg[r] = hv;
          const size_t bt = (size_t)b * S + t;
          hs[bt * H + j0 + jj] = dca::f2bf(hv);
          if (hsf) hsf[bt * H + j0 + jj] = hv;
          cs[bt * H + j0 + jj] = c;
          float* gp = gates + bt * G4 + j0 + jj;
          gp[0] = ig;
          gp[H] = fg;
          gp[2 * H] = gg;
          gp[3 * H] = og;
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
// ring   (2, NWG, B, H) u64 granules {tag = t+1, f32} (zeroed)
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
                                                               unsigned* err, int Btot, int Bc, int S) {
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
  __shared__ float dpart[2][4][PMAX];
  __shared__ float inp[2][7][PMAX];        // i, f, g, o, c_t, c_{t-1}, dhs_t
  __shared__ short dgl[4][MT * 16][40];
  __shared__ int abort_flag;
  if (tid == 0) abort_flag = 0;
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
      // All of this wave's granules (every pass of 64 pairs × its NWG/4 producers) are loaded in ONE poll round, so
      // a step costs one hand-off round trip whatever the batch.
      bool dead = false;
      const int pg = wv;
      constexpr int NPASS = PMAX / 64;
      const int npass = (P + 63) >> 6;
      float ssum[NPASS];
      if (k == 0) {
#pragma unroll
        for (int ps = 0; ps < NPASS; ++ps) {
          const int p = ps * 64 + lane;
          ssum[ps] = (pg == 0 && p < P && dhn) ? dhn[(p >> 3) * H + j0 + (p & 7)] : 0.f;
        }
      } else {
        const unsigned long long* slot = ring + (size_t)((t + 1) & 1) * NWG * B * H;
        const unsigned tag = (unsigned)(t + 2);
        constexpr int NPG = NWG / 4;                 // producers per poller wave
        unsigned long long gr[NPASS][NPG];
        // (1) PROBE: each lane checks ONE producer of its pair (lanes rotate over the producers), so the wave
        //     as a whole samples every producer with a single load per lane per round.
        while (true) {
          bool ok = true;
#pragma unroll
          for (int ps = 0; ps < NPASS; ++ps) {
            const int p = ps * 64 + lane;
            if (ps < npass && p < P) {
              const int wp = pg * NPG + (lane % NPG);
              gr[ps][0] = ld_granule(slot + ((size_t)wp * B + (p >> 3)) * H + j0 + (p & 7));
            }
          }
#pragma unroll
          for (int ps = 0; ps < NPASS; ++ps)
            if (ps < npass && ps * 64 + lane < P) ok &= (unsigned)(gr[ps][0] >> 32) == tag;
          if (__all(ok)) break;
          if (spin_fail(spins, err, 2u)) { dead = true; break; }
        }
        // (2) FETCH every granule of the round, all loads in flight before any use; verify, refetch if needed.
        while (!dead) {
#pragma unroll
          for (int ps = 0; ps < NPASS; ++ps) {
            const int p = ps * 64 + lane;
            if (ps < npass && p < P) {
              const int b = p >> 3, jj = p & 7;
#pragma unroll
              for (int i = 0; i < NPG; ++i)
                gr[ps][i] = ld_granule(slot + ((size_t)(pg * NPG + i) * B + b) * H + j0 + jj);
            }
          }
          bool ok = true;
#pragma unroll
          for (int ps = 0; ps < NPASS; ++ps)
            if (ps < npass && ps * 64 + lane < P) {
#pragma unroll
              for (int i = 0; i < NPG; ++i) ok &= (unsigned)(gr[ps][i] >> 32) == tag;
            }
          if (__all(ok)) break;
          if (spin_fail(spins, err, 2u)) { dead = true; break; }
        }
#pragma unroll
        for (int ps = 0; ps < NPASS; ++ps) {
          float s = 0.f;
#pragma unroll
          for (int i = 0; i < NPG; ++i) s += __uint_as_float((unsigned)gr[ps][i]);
          ssum[ps] = (ps < npass && ps * 64 + lane < P) ? s : 0.f;
        }
      }
#pragma unroll
      for (int ps = 0; ps < NPASS; ++ps) {
        const int p = ps * 64 + lane;
        if (p < P) dpart[par][pg][p] = ssum[ps];
      }
      if (dead && lane == 0) abort_flag = 1;
      if (t >= 0) {
#pragma unroll
        for (int i = 0; i < NIN; ++i) {
          const int idx = tid + 256 * i;
          if (idx < 7 * P) inp[par][idx / P][idx % P] = iv[i];
        }
      }
    }
    lds_barrier();
    if (abort_flag) break;
    if (t < 0) {
      // final gather done: ∂L/∂h0
      if (poller) {
        for (int p = tid; p < P; p += 256)
          dh0[(p >> 3) * H + j0 + (p & 7)] = dpart[par][0][p] + dpart[par][1][p] + dpart[par][2][p] + dpart[par][3][p];
      }
      break;
    }
    if (!poller) {
      // -------- gate gradients of the owned units (every publisher wave computes all pairs)
#pragma unroll
      for (int r = 0; r < NPR; ++r) {
        const int p = lane + 64 * r;
        if (64 * r >= P) break;
        if (p < P) {
          const int b = p >> 3, jj = p & 7;
          const float ig = inp[par][0][p], fg = inp[par][1][p], gg = inp[par][2][p], og = inp[par][3][p];
          const float c = inp[par][4][p], cprev = inp[par][5][p];
          const float dht = inp[par][6][p] + dpart[par][0][p] + dpart[par][1][p] + dpart[par][2][p] +
                            dpart[par][3][p];
          const float tc = dca::tanhf_(c);
          const float dc = dcreg[r] + dht * og * (1.f - tc * tc);
          const float d_o = dht * tc * og * (1.f - og);
          const float d_i = dc * gg * ig * (1.f - ig);
          const float d_f = dc * cprev * fg * (1.f - fg);
          const float d_g = dc * ig * (1.f - gg * gg);
          dcreg[r] = dc * fg;
          dgl[pw][b][0 * 8 + jj] = dca::f2bf(d_i);
          dgl[pw][b][1 * 8 + jj] = dca::f2bf(d_f);
          dgl[pw][b][2 * 8 + jj] = dca::f2bf(d_g);
          dgl[pw][b][3 * 8 + jj] = dca::f2bf(d_o);
          if (pw == 0) {
            float* dg = dgates + ((size_t)b * S + t) * G4 + j0 + jj;
            dg[0] = d_i;
            dg[H] = d_f;
            dg[2 * H] = d_g;
            dg[3 * H] = d_o;
            if (t == 0) dc0[b * H + j0 + jj] = dcreg[r];
          }
        }
      }
      // -------- partial = dG_blk (B×32) · W_blk (32 × this wave's H/4 columns) → granules of step t
      unsigned long long* slot = ring + (size_t)(t & 1) * NWG * B * H + (size_t)w * B * H;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&dgl[pw][mt * 16 + lrow][8 * lkg]);
#pragma unroll
        for (int n = 0; n < NT_W; ++n) {
          dca::f32x4 acc = {0.f, 0.f, 0.f, 0.f};
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[n], acc, 0, 0, 0);
          const int col = (pw * NT_W + n) * 16 + lrow;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int b = mt * 16 + lkg * 4 + r;
            if (b < B)
              st_granule(slot + (size_t)b * H + col,
                         ((unsigned long long)(unsigned)(t + 1) << 32) | __float_as_uint(acc[r]));
          }
        }
      }
    }
  }
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
                                                                   ring, err, B, Bc, S, trace);
  return hipGetLastError();
}

template <int MT, int KS>
hipError_t launch_bwd(const float* dhs, const float* gates, const float* cs, const float* c0, const float* dhn,
                      const float* dcn, const short* whh, float* dgates, float* dh0, float* dc0,
                      unsigned long long* ring, unsigned* err, int B, int Bc, int nch, int S, hipStream_t st) {
  constexpr int H = 128 * KS;
  hipError_t e = hipMemsetAsync(ring, 0, sizeof(unsigned long long) * (size_t)nch * 2 * (H / kUw) * Bc * H, st);
  if (e != hipSuccess) return e;
  lstm_bwd_kernel<MT, KS><<<nch * (H / kUw), kBwdThreads, 0, st>>>(dhs, gates, cs, c0, dhn, dcn, whh, dgates, dh0,
                                                                   dc0, ring, err, B, Bc, S);
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
                                   hipStream_t st) {
  if (!lstm_shape_ok(B, H) || S < 1) return hipErrorInvalidValue;
  int nch, Bc, MT;
  plan_chains(B, H, nch, Bc, MT);
  const int KS = H / 128;
#define DCA_B(mt, ks) launch_bwd<mt, ks>(dhs, gates, cs, c0, dhn, dcn, whh, dgates, dh0, dc0, ring, err, B, Bc, nch, S, st)
  DCA_DISPATCH_MT_KS(MT, KS, DCA_B)
#undef DCA_B
}
