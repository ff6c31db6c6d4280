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

constexpr int kThreads = 256;
constexpr int kUw = 8;                  // hidden units per workgroup
constexpr unsigned kSpinLimit = 1u << 21;

__device__ __forceinline__ unsigned long long ld_granule(const unsigned long long* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_granule(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// XCD-local hand-off: a plain store keeps the line in the producer XCD's L2, where same-XCD consumers' L1-bypassing
// (agent-scope) loads hit it. Only valid when every workgroup of the launch sits on ONE XCD (see LOCAL below).
__device__ __forceinline__ void st_granule_local(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
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

// =============================================================================================================
// Forward
// =============================================================================================================
// xp     (B, S, 4H) f32  input projection incl. both biases
// whh    (4H, H)    bf16 recurrent weights (PyTorch layout, gate order i,f,g,o)
// h0,c0  (B, H)     f32
// hs     (B, S, H)  bf16 out: h_t
// hsf    (B, S, H)  f32  out: h_t (optional, may be null)
// cs     (B, S, H)  f32  out: c_t
// gates  (B, S, 4H) f32  out: activated i, f, g, o
// hn,cn  (B, H)     f32  out: final state
// ring   (2, B, H/2) u64 granules (zeroed)
template <int MT, int KS, bool LOCAL>
__global__ __launch_bounds__(kThreads) void lstm_fwd_kernel(const float* __restrict__ xp, const short* __restrict__ whh,
                                                            const float* __restrict__ h0, const float* __restrict__ c0,
                                                            short* __restrict__ hs, float* __restrict__ hsf,
                                                            float* __restrict__ cs, float* __restrict__ gates,
                                                            float* __restrict__ hn, float* __restrict__ cn,
                                                            unsigned long long* ring, unsigned* err, int B, int S) {
  constexpr int H = 128 * KS;           // each of the 4 waves owns K/4 = 32·KS of the reduction
  constexpr int G4 = 4 * H;
  constexpr int HP = H / 2;             // granules per batch row
  // LOCAL: the grid is 8× oversized and only blocks ≡ 0 (mod 8) — which the dispatcher deals to one XCD — work.
  if (LOCAL && (blockIdx.x & 7) != 0) return;
  const int w = LOCAL ? (blockIdx.x >> 3) : blockIdx.x;
  const int j0 = w * kUw;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int lrow = lane & 15, lkg = lane >> 4;

  __shared__ float red[4][MT][2][16][17];

  // ---- W_hh slice as MFMA B fragments: B[k][c] = W[row(c)][k]; lane holds c = lane&15 (+16·nt), k = 8·lkg + j.
  bf16x8 wf[2][KS];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int c = nt * 16 + lrow;                  // local gate column 0..31
    const int row = (c >> 3) * H + j0 + (c & 7);   // gate q = c/8, unit c%8
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = wv * (32 * KS) + ks * 32 + 8 * lkg;
      wf[nt][ks] = *reinterpret_cast<const bf16x8*>(whh + (size_t)row * H + k);
    }
  }

  // ---- elementwise ownership: pairs p = b*8 + jj; up to 2 per thread (B ≤ 64)
  const int P = B * kUw;
  float creg[2];
  float hreg[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int p = tid + r * kThreads;
    creg[r] = 0.f;
    hreg[r] = 0.f;
    if (p < P) {
      const int b = p >> 3, jj = p & 7;
      creg[r] = c0[b * H + j0 + jj];
      hreg[r] = h0[b * H + j0 + jj];
    }
  }

  unsigned spins = 0;
  bool dead = false;
  for (int t = 0; t < S; ++t) {
    // -------- prefetch this step's input projection (plain loads; written before launch)
    float xv[2][4];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int p = tid + r * kThreads;
      if (p < P) {
        const int b = p >> 3, jj = p & 7;
        const float* x = xp + ((size_t)b * S + t) * G4 + j0 + jj;
#pragma unroll
        for (int q = 0; q < 4; ++q) xv[r][q] = x[q * H];
      }
    }
    // -------- gather h_{t-1} A-fragments (rows = batch, k = hidden) for this wave's K quarter
    bf16x8 af[MT][KS];
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
      const unsigned tag = (unsigned)t;     // h_{t-1} carries tag t
      while (true) {
        bool ok = true;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            const int b = mt * 16 + lrow;
            const int k = wv * (32 * KS) + ks * 32 + 8 * lkg;
            bf16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
            if (b < B) {
              const unsigned long long* g = slot + (size_t)b * HP + (k >> 1);
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const unsigned long long x = ld_granule(g + q);
                ok &= (unsigned)(x >> 32) == tag;
                const unsigned pl = (unsigned)x;
                v[2 * q] = (short)(pl & 0xffffu);
                v[2 * q + 1] = (short)(pl >> 16);
              }
            }
            af[mt][ks] = v;
          }
        if (__all(ok)) break;
        if (spin_fail(spins, err, 1u)) { dead = true; break; }
      }
    }
    // -------- partial gates over this wave's K quarter
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        dca::f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt][ks], wf[nt][ks], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wv][mt][nt][lkg * 4 + r][lrow] = acc[r];
      }
    __syncthreads();
    if (__syncthreads_or(dead)) break;
    // -------- cell update for owned (b, unit) pairs, publish h_t granules
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int p = tid + r * kThreads;
      float hv = 0.f;
      if (p < P) {
        const int b = p >> 3, jj = p & 7;
        const int mt = b >> 4, row = b & 15;
        float pre[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = q * kUw + jj;
          const int nt = c >> 4, cc = c & 15;
          pre[q] = red[0][mt][nt][row][cc] + red[1][mt][nt][row][cc] + red[2][mt][nt][row][cc] +
                   red[3][mt][nt][row][cc] + xv[r][q];
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
      // pair units (jj, jj+1) into one granule: lanes p and p+1 are adjacent in the wave
      const float hnext = __shfl_down(hv, 1, 64);
      if (p < P && (p & 1) == 0) {
        const int b = p >> 3, jj = p & 7;
        const unsigned pl = (unsigned)(unsigned short)dca::f2bf(hv) |
                            ((unsigned)(unsigned short)dca::f2bf(hnext) << 16);
        unsigned long long* gptr = ring + (size_t)(t & 1) * B * HP + (size_t)b * HP + ((j0 + jj) >> 1);
        const unsigned long long gv = ((unsigned long long)(unsigned)(t + 1) << 32) | pl;
        if (LOCAL) st_granule_local(gptr, gv); else st_granule(gptr, gv);
      }
    }
    __syncthreads();   // red[] is rewritten next step
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int p = tid + r * kThreads;
    if (p < P) {
      const int b = p >> 3, jj = p & 7;
      hn[b * H + j0 + jj] = hreg[r];
      cn[b * H + j0 + jj] = creg[r];
    }
  }
}

// =============================================================================================================
// Backward
// =============================================================================================================
// dhs    (B, S, H)  f32  ∂L/∂h_t from everything above the LSTM (not including the recurrence)
// gates  (B, S, 4H) f32  activated gates from the forward
// cs     (B, S, H)  f32  c_t from the forward; c0 (B, H)
// dhn,dcn(B, H)     f32  ∂L/∂(h_S, c_S) (may be null)
// dgates (B, S, 4H) f32  out: ∂L/∂(gate pre-activations) (input to the weight-gradient GEMMs)
// dh0,dc0(B, H)     f32  out
// ring   (2, NWG, B, H) u64 granules {tag, f32} (zeroed)
template <int MT, int KS>
__global__ __launch_bounds__(kThreads) void lstm_bwd_kernel(const float* __restrict__ dhs, const float* __restrict__ gates,
                                                            const float* __restrict__ cs, const float* __restrict__ c0,
                                                            const float* __restrict__ dhn, const float* __restrict__ dcn,
                                                            const short* __restrict__ whh, float* __restrict__ dgates,
                                                            float* __restrict__ dh0, float* __restrict__ dc0,
                                                            unsigned long long* ring, unsigned* err, int B, int S) {
  constexpr int H = 128 * KS;
  constexpr int G4 = 4 * H;
  constexpr int NWG = H / kUw;
  constexpr int NT_W = H / 64;          // N tiles (16 columns) per wave: H/16 tiles over 4 waves
  const int w = blockIdx.x;
  const int j0 = w * kUw;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int lrow = lane & 15, lkg = lane >> 4;

  __shared__ short dgl[MT * 16][40];            // dG_blk (bf16) as the MFMA A operand, padded rows
  __shared__ float dpart[4][512];               // per-wave partial sums of dh_rec (pairs ≤ 512)

  // ---- W slice as B fragments: B[k][col] = W[row(k)][col], row(k) = (k/8)·H + j0 + k%8, k = 8·lkg + j.
  bf16x8 wf[NT_W];
#pragma unroll
  for (int n = 0; n < NT_W; ++n) {
    const int col = (wv * NT_W + n) * 16 + lrow;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = whh[(size_t)(lkg * H + j0 + j) * H + col];
    wf[n] = v;
  }
  // zero the padding rows of the A operand once
  for (int i = tid; i < MT * 16 * 40; i += kThreads) (&dgl[0][0])[i] = 0;

  const int P = B * kUw;
  float dcreg[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int p = tid + r * kThreads;
    dcreg[r] = 0.f;
    if (p < P && dcn) dcreg[r] = dcn[(p >> 3) * H + j0 + (p & 7)];
  }
  __syncthreads();

  unsigned spins = 0;
  bool dead = false, bdead = false;
  // Gather Σ_w' partial_{w'}[b][J_w] of step `ts` (tag ts+1) for every owned pair. Wave pg sums producers
  // [pg·NWG/4, (pg+1)·NWG/4) for 64 pairs per pass; the 4 partial sums meet in LDS (one barrier).
  auto gather = [&](int ts, float (&dh)[2]) {
    const unsigned long long* slot = ring + (size_t)(ts & 1) * NWG * B * H;
    const unsigned tag = (unsigned)(ts + 1);
    const int pg = wv;
    const int npass = (P + 63) >> 6;
    for (int pass = 0; pass < npass; ++pass) {
      const int p = pass * 64 + lane;
      if (p < P) {
        const int b = p >> 3, jj = p & 7;
        float s = 0.f;
        while (true) {
          bool ok = true;
          s = 0.f;
#pragma unroll 4
          for (int i = 0; i < NWG / 4; ++i) {
            const int wp = pg * (NWG / 4) + i;
            const unsigned long long x = ld_granule(slot + ((size_t)wp * B + b) * H + j0 + jj);
            ok &= (unsigned)(x >> 32) == tag;
            s += __uint_as_float((unsigned)x);
          }
          if (__all(ok)) break;
          if (spin_fail(spins, err, 2u)) { dead = true; break; }
        }
        dpart[pg][p] = s;
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int p = tid + r * kThreads;
      dh[r] = (p < P) ? dpart[0][p] + dpart[1][p] + dpart[2][p] + dpart[3][p] : 0.f;
    }
  };

  for (int t = S - 1; t >= 0; --t) {
    float dh[2] = {0.f, 0.f};
    if (t == S - 1) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int p = tid + r * kThreads;
        if (p < P && dhn) dh[r] = dhn[(p >> 3) * H + j0 + (p & 7)];
      }
    } else {
      gather(t + 1, dh);
      if (__syncthreads_or(dead)) { bdead = true; break; }
    }
    // -------- elementwise: dG_t for owned pairs
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int p = tid + r * kThreads;
      if (p < P) {
        const int b = p >> 3, jj = p & 7;
        const size_t bt = (size_t)b * S + t;
        const float* gp = gates + bt * G4 + j0 + jj;
        const float ig = gp[0], fg = gp[H], gg = gp[2 * H], og = gp[3 * H];
        const float c = cs[bt * H + j0 + jj];
        const float cprev = (t > 0) ? cs[(bt - 1) * H + j0 + jj] : c0[b * H + j0 + jj];
        const float tc = dca::tanhf_(c);
        const float dht = dhs[bt * H + j0 + jj] + dh[r];
        const float dc = dcreg[r] + dht * og * (1.f - tc * tc);
        const float d_o = dht * tc * og * (1.f - og);
        const float d_i = dc * gg * ig * (1.f - ig);
        const float d_f = dc * cprev * fg * (1.f - fg);
        const float d_g = dc * ig * (1.f - gg * gg);
        dcreg[r] = dc * fg;
        float* dg = dgates + bt * G4 + j0 + jj;
        dg[0] = d_i;
        dg[H] = d_f;
        dg[2 * H] = d_g;
        dg[3 * H] = d_o;
        dgl[b][0 * 8 + jj] = dca::f2bf(d_i);
        dgl[b][1 * 8 + jj] = dca::f2bf(d_f);
        dgl[b][2 * 8 + jj] = dca::f2bf(d_g);
        dgl[b][3 * 8 + jj] = dca::f2bf(d_o);
      }
    }
    __syncthreads();
    // -------- partial_w = dG_blk (B×32) · W_blk (32×H), publish as {tag=t+1, f32} granules
    unsigned long long* slot = ring + (size_t)(t & 1) * NWG * B * H + (size_t)w * B * H;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(&dgl[mt * 16 + lrow][8 * lkg]);
#pragma unroll
      for (int n = 0; n < NT_W; ++n) {
        dca::f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[n], acc, 0, 0, 0);
        const int col = (wv * NT_W + n) * 16 + lrow;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int b = mt * 16 + lkg * 4 + r;
          if (b < B)
            st_granule(slot + (size_t)b * H + col,
                       ((unsigned long long)(unsigned)(t + 1) << 32) | __float_as_uint(acc[r]));
        }
      }
    }
    __syncthreads();   // dgl[] is rewritten next step
  }
  // -------- dh0 = Σ partials of step 0, dc0 = carried dc
  float dh[2] = {0.f, 0.f};
  if (!bdead) gather(0, dh);
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int p = tid + r * kThreads;
    if (p < P) {
      dh0[(p >> 3) * H + j0 + (p & 7)] = dh[r];
      dc0[(p >> 3) * H + j0 + (p & 7)] = dcreg[r];
    }
  }
}

template <int MT, int KS>
hipError_t launch_fwd(const float* xp, const short* whh, const float* h0, const float* c0, short* hs, float* hsf,
                      float* cs, float* gates, float* hn, float* cn, unsigned long long* ring, unsigned* err, int B,
                      int S, int local, hipStream_t st) {
  constexpr int H = 128 * KS;
  hipError_t e = hipMemsetAsync(ring, 0, sizeof(unsigned long long) * 2 * B * (H / 2), st);
  if (e != hipSuccess) return e;
  if (local)
    lstm_fwd_kernel<MT, KS, true><<<8 * (H / kUw), kThreads, 0, st>>>(xp, whh, h0, c0, hs, hsf, cs, gates, hn, cn,
                                                                      ring, err, B, S);
  else
    lstm_fwd_kernel<MT, KS, false><<<H / kUw, kThreads, 0, st>>>(xp, whh, h0, c0, hs, hsf, cs, gates, hn, cn, ring,
                                                                 err, B, S);
  return hipGetLastError();
}

template <int MT, int KS>
hipError_t launch_bwd(const float* dhs, const float* gates, const float* cs, const float* c0, const float* dhn,
                      const float* dcn, const short* whh, float* dgates, float* dh0, float* dc0,
                      unsigned long long* ring, unsigned* err, int B, int S, hipStream_t st) {
  constexpr int H = 128 * KS;
  hipError_t e = hipMemsetAsync(ring, 0, sizeof(unsigned long long) * 2 * (H / kUw) * B * H, st);
  if (e != hipSuccess) return e;
  lstm_bwd_kernel<MT, KS><<<H / kUw, kThreads, 0, st>>>(dhs, gates, cs, c0, dhn, dcn, whh, dgates, dh0, dc0, ring, err,
                                                        B, S);
  return hipGetLastError();
}

}  // namespace

#define DCA_DISPATCH_MT_KS(MT_, KS_, ...)                                           \
  switch (((MT_) << 4) | (KS_)) {                                                  \
    case 0x11: return __VA_ARGS__(1, 1); case 0x12: return __VA_ARGS__(1, 2);      \
    case 0x14: return __VA_ARGS__(1, 4); case 0x21: return __VA_ARGS__(2, 1);      \
    case 0x22: return __VA_ARGS__(2, 2); case 0x24: return __VA_ARGS__(2, 4);      \
    case 0x41: return __VA_ARGS__(4, 1); case 0x42: return __VA_ARGS__(4, 2);      \
    case 0x44: return __VA_ARGS__(4, 4);                                           \
    default: return hipErrorInvalidValue;                                          \
  }

static int mt_for(int B) { return B <= 16 ? 1 : (B <= 32 ? 2 : 4); }

// Ring sizes (u64 elements): forward 2·B·H/2, backward 2·(H/8)·B·H.
extern "C" size_t dca_lstm_ring_elems(int B, int H, int backward) {
  return backward ? (size_t)2 * (H / kUw) * B * H : (size_t)2 * B * (H / 2);
}

extern "C" hipError_t dca_lstm_fwd(const float* xp, const short* whh, const float* h0, const float* c0, short* hs,
                                   float* hsf, float* cs, float* gates, float* hn, float* cn,
                                   unsigned long long* ring, unsigned* err, int B, int S, int H, int local,
                                   hipStream_t st) {
  if (B < 1 || B > 64 || S < 1 || (H != 128 && H != 256 && H != 512)) return hipErrorInvalidValue;
  const int MT = mt_for(B), KS = H / 128;
#define DCA_F(mt, ks) launch_fwd<mt, ks>(xp, whh, h0, c0, hs, hsf, cs, gates, hn, cn, ring, err, B, S, local, st)
  DCA_DISPATCH_MT_KS(MT, KS, DCA_F)
#undef DCA_F
}

extern "C" hipError_t dca_lstm_bwd(const float* dhs, const float* gates, const float* cs, const float* c0,
                                   const float* dhn, const float* dcn, const short* whh, float* dgates, float* dh0,
                                   float* dc0, unsigned long long* ring, unsigned* err, int B, int S, int H,
                                   hipStream_t st) {
  if (B < 1 || B > 64 || S < 1 || (H != 128 && H != 256 && H != 512)) return hipErrorInvalidValue;
  const int MT = mt_for(B), KS = H / 128;
#define DCA_B(mt, ks) launch_bwd<mt, ks>(dhs, gates, cs, c0, dhn, dcn, whh, dgates, dh0, dc0, ring, err, B, S, st)
  DCA_DISPATCH_MT_KS(MT, KS, DCA_B)
#undef DCA_B
}
