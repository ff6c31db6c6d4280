// Fused ∂X chain of the fp32 learner's pre-RNN layer (gfx950 MFMA), one launch instead of three hipBLASLt /
// elementwise launches on the critical path after the backward recurrence (models/pipelined.py):
//
//   dpre  = (dG · W_ih) ⊙ [x > 0]       dG (N × 4H) = ∂L/∂gates (unit-major), W_ih (4H × P) permuted rows, x = relu
//                                        output of the pre-RNN layer (the ReLU backward, threshold_backward)
//   dx896 = dpre · W_pre                 W_pre (P × X): ∂L/∂(concatenated encoder features)
//
// Reference: policy.py:135-138 (affine_pre_rnn + ReLU) feeding the recurrent layer (policy.py:143-145; the LSTM of
// the north star). N = B·S rows (11 200 at the deploy shape), 4H = 2048, P = 256, X = 896.
//
// One 512-thread workgroup (8 waves) per BM-row tile (BM = 48); the BM × P dpre tile never leaves the workgroup between the
// two products (it is written once to HBM for the pre-RNN weight gradient, and kept in LDS as the second product's
// A operand):
// * stage 1, K = 4H in 32-deep slabs, double-buffered through LDS, loads issued RD slabs ahead into a register ring
//   (one slab of lead left every LDS store waiting out a full memory round trip), one barrier per slab; waves as
//   1 (48 rows) × 8 (32 columns), each 3 × 2 v_mfma_f32_16x16x32_bf16 tiles;
// * ReLU mask + dpre store in the accumulator layout, dpre written into LDS in the stage-1 A layout (8 slabs);
// * stage 2, X in 128-column chunks × K = P in 32-deep slabs (same pipeline), waves as 1 (48 rows) × 8 (16 columns).
// Both weight operands come K-contiguous per output column (W_ihᵀ image (P × 4H), W_preᵀ image (X × P)).
//
// EXACT = false: bf16x3 — x = hi + lo (two bf16), products hi·hi + lo·hi + hi·lo on the bf16 MFMA (≈2⁻¹⁶ relative per
// product, the fp32 learner's accuracy class). The weights arrive PRE-SPLIT (hi / lo bf16 images, split once per
// step by dca_split_bf16x2), so only the dG slab is split while staging. LDS images: 64-B rows (32 bf16) with the
// 16-B chunk index XOR (row>>1)&3 — conflict-free for the fragment reads (ds_read_b128 lane groups), the dG b64
// stores and the weight b128 stores (exhaustive check over the lane→address maps; the first version, 80-B padded
// rows without swizzle and the weights split in-kernel, measured 4.8 bank-conflict cycles per LDS instruction,
// 5 VALU per MFMA and 205 µs at the deploy shape).
// EXACT = true: exact fp32 on v_mfma_f32_16x16x4_f32 — a 16x16x32 fragment's 8 k values per lane feed 8 chained
// 16x16x4 MFMAs (call j takes element j: lane l contributes k = 8·(l/16) + j, so the 8 calls cover all 32 k);
// fp32 LDS rows (144-B pitch), fp32 weights; every launch form (∂X chain, forward chain, heads GEMM + its ∂X
// product) has an exact instance: the IEEE-fp32 learner.
#include "common.h"
#include <cstdlib>

namespace {

using dca::bf16x8;
using dca::f32x4;

// BM = 48 rows per workgroup: 234 workgroups at the deploy shape (N = 11 200) on the 256 CUs (one per CU: LDS- and
// VGPR-bound). BM = 64 left 81 CUs idle (175 workgroups): measured 271 µs for the exact ∂X chain.
constexpr int BM = 48, BK = 32, NT = 512, P = 256, XC = 128, RD = 4;
constexpr int NI1 = BM / 16;                      // 16-row tiles per wave (every wave spans all BM rows)

template <bool EXACT>
struct Lay {
  static constexpr int RP = EXACT ? 144 : 64;             // bytes per operand row of one 32-deep slab
  static constexpr int IMG = EXACT ? 1 : 2;               // images per operand (hi, lo)
  static constexpr int A1 = BM * RP;                       // stage-1 A image bytes
  static constexpr int B1 = P * RP;                        // stage-1 B image bytes
  static constexpr int S1 = IMG * (A1 + B1);               // one stage-1 buffer
  static constexpr int D = IMG * (P / BK) * A1;            // dpre tile: 8 slabs in the A layout
  static constexpr int B2 = XC * RP;                       // stage-2 B image bytes
  static constexpr int S2 = IMG * B2;
  static constexpr int BYTES = (2 * S1 > D + 2 * S2) ? 2 * S1 : D + 2 * S2;
};

// byte offset of 16-B chunk c of row r in a slab image (bf16: 4 chunks per row, swizzled; fp32: 8, padded rows)
template <bool EXACT>
__device__ __forceinline__ int coff(int r, int c) {
  if constexpr (EXACT) return r * Lay<true>::RP + 16 * c;
  else return r * 64 + 16 * (c ^ ((r >> 1) & 3));
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, long long bytes) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int nb = (int)(bytes > 0x7fff0000LL ? 0x7fff0000LL : bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(nb), 0x00020000);
}
__device__ __forceinline__ uint4 ld16(__amdgpu_buffer_rsrc_t r, int off) {   // out of range → zeros
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
constexpr int kOob = 0x7fff8000;

__device__ __forceinline__ unsigned pack2(short a, short b) {
  return (unsigned)(unsigned short)a | ((unsigned)(unsigned short)b << 16);
}
// 4 fp32 → hi / lo bf16 quads
__device__ __forceinline__ void split4(const float4 v, uint2& hi, uint2& lo) {
  const short h0 = dca::f2bf(v.x), h1 = dca::f2bf(v.y), h2 = dca::f2bf(v.z), h3 = dca::f2bf(v.w);
  hi = make_uint2(pack2(h0, h1), pack2(h2, h3));
  lo = make_uint2(pack2(dca::f2bf(v.x - dca::bf2f(h0)), dca::f2bf(v.y - dca::bf2f(h1))),
                  pack2(dca::f2bf(v.z - dca::bf2f(h2)), dca::f2bf(v.w - dca::bf2f(h3))));
}

struct Frag {
  bf16x8 hi, lo;        // bf16x3
  float f[8];           // exact
};
// fragment of row r (chunk q = lane/16 of the 32-deep slab) from a slab image
template <bool EXACT>
__device__ __forceinline__ void get_frag(const char* img, int img_bytes, int r, int q, Frag& fr) {
  if constexpr (EXACT) {
    const float4 a = *reinterpret_cast<const float4*>(img + coff<true>(r, 2 * q));
    const float4 b = *reinterpret_cast<const float4*>(img + coff<true>(r, 2 * q + 1));
    fr.f[0] = a.x; fr.f[1] = a.y; fr.f[2] = a.z; fr.f[3] = a.w;
    fr.f[4] = b.x; fr.f[5] = b.y; fr.f[6] = b.z; fr.f[7] = b.w;
  } else {
    const int o = coff<false>(r, q);
    fr.hi = *reinterpret_cast<const bf16x8*>(img + o);
    fr.lo = *reinterpret_cast<const bf16x8*>(img + img_bytes + o);
  }
}
// all NI × NJ tiles of one slab, one product pass at a time over every tile (the three bf16x3 passes of a tile
// are dependent on its accumulator; interleaving the tiles keeps the MFMA pipe fed instead of waiting out each
// accumulator's latency twice per tile)
template <bool EXACT, int NI, int NJ>
__device__ __forceinline__ void mma_tiles(const Frag (&fa)[NI], const Frag (&fb)[NJ], f32x4 (&acc)[NI][NJ]) {
  if constexpr (EXACT) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i].f[e], fb[j].f[e], acc[i][j], 0, 0, 0);
  } else {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i].lo, fb[j].hi, acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i].hi, fb[j].lo, acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i].hi, fb[j].hi, acc[i][j], 0, 0, 0);
  }
}

// EPI 0: the ∂X chain's ReLU backward (v = [x > 0]·acc, x the layer's output); EPI 1: the forward chain's bias + ReLU
// (v = max(acc + b, 0), `x` = the bias (P)) — pre-RNN layer then input projection, x896 → x → x·W_ihᵀ; EPI 2: bias
// only (the heads GEMM, stage 1 alone). K1 = 0 runs stage 2 alone on A = dG (N, P) (the heads' ∂X product).
template <bool EXACT, int EPI>
__global__ __launch_bounds__(NT, 1) void dpre_dx_kernel(const float* __restrict__ dG, const void* __restrict__ w1h,
                                                        const void* __restrict__ w1l, const float* __restrict__ x,
                                                        const void* __restrict__ w2h, const void* __restrict__ w2l,
                                                        float* __restrict__ dpre, float* __restrict__ dx, int N,
                                                        int K1, int X) {
  using L = Lay<EXACT>;
  constexpr int ES = EXACT ? 4 : 2;                 // bytes per weight element in HBM
  __shared__ __attribute__((aligned(16))) char lds[L::BYTES];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r16 = lane & 15, q = lane >> 4;
  const int r0 = blockIdx.x * BM;
  const __amdgpu_buffer_rsrc_t rA = rsrc(dG, (long long)N * K1 * 4);
  const __amdgpu_buffer_rsrc_t rW1h = rsrc(w1h, (long long)P * K1 * ES);
  const __amdgpu_buffer_rsrc_t rW1l = rsrc(EXACT ? w1h : w1l, (long long)P * K1 * ES);
  const __amdgpu_buffer_rsrc_t rW2h = rsrc(w2h, (long long)X * P * ES);
  const __amdgpu_buffer_rsrc_t rW2l = rsrc(EXACT ? w2h : w2l, (long long)X * P * ES);

  char* dimg = lds;                               // the dpre image aliases the stage-1 buffers
  constexpr int DIMG = (P / BK) * L::A1;          // one image (hi, or fp32) of the dpre tile
  if (K1 > 0) {
  // ================= stage 1: C1 (64 × P) = dG[r0:r0+64] · W_ih =================
  const int ar = tid >> 3, ak = (tid & 7) * 4;              // dG slab: one fp32 quad per thread (threads ≥ 8·BM idle)
  const int arow = r0 + ar;
  const int a_off0 = (ar < BM && arow < N) ? (arow * K1 + ak) * 4 : kOob;
  const int br = tid & 255, bh = tid >> 8;                   // exact W1 slab: 16 k per thread
  const int b_off0 = (br * K1 + 16 * bh) * ES;
  float4 sa[RD];
  uint4 sb[RD][4];
  // Branch-free: a slab past K reads out of range (zeros, no memory traffic) instead of being skipped — a load
  // under an `if` made the compiler wait for every outstanding load at the join (s_waitcnt vmcnt(0) ahead of each
  // slab's loads), which serialised the ring
  auto load1 = [&](int slot, int k0) {
    const bool in = k0 < K1;
    sa[slot] = __builtin_bit_cast(float4, ld16(rA, (in && a_off0 != kOob) ? a_off0 + k0 * 4 : kOob));
    if constexpr (EXACT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) sb[slot][i] = ld16(rW1h, in ? b_off0 + (k0 + 4 * i) * 4 : kOob);
    } else {
      // slab-major images: the 256 × 32 slab is 16 KB contiguous per image, a wave instruction reads 1 KB of it
      const int o = (k0 / BK) * (P * 64) + tid * 16;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        sb[slot][j] = ld16(rW1h, in ? o + 8192 * j : kOob);
        sb[slot][2 + j] = ld16(rW1l, in ? o + 8192 * j : kOob);
      }
    }
  };
  auto store1 = [&](int slot, int buf) {
    char* base = lds + buf * L::S1;
    char* bb = base + L::IMG * L::A1;
    if constexpr (EXACT) {
      if (ar < BM) *reinterpret_cast<float4*>(base + ar * L::RP + ak * 4) = sa[slot];
#pragma unroll
      for (int i = 0; i < 4; ++i) *reinterpret_cast<uint4*>(bb + br * L::RP + (16 * bh + 4 * i) * 4) = sb[slot][i];
    } else {
      uint2 hi, lo;
      split4(sa[slot], hi, lo);
      const int o = coff<false>(ar, ak >> 3) + 8 * ((ak >> 2) & 1);
      if (ar < BM) {
        *reinterpret_cast<uint2*>(base + o) = hi;
        *reinterpret_cast<uint2*>(base + L::A1 + o) = lo;
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {              // 16-B chunk tid & 3 of rows tid / 4 and 128 + tid / 4
        const int ob = coff<false>(128 * j + (tid >> 2), tid & 3);
        *reinterpret_cast<uint4*>(bb + ob) = sb[slot][j];
        *reinterpret_cast<uint4*>(bb + L::B1 + ob) = sb[slot][2 + j];
      }
    }
  };
  const int wc = w;                              // 1 × 8 waves: all BM rows, cols 32·wc
  f32x4 acc[NI1][2];
#pragma unroll
  for (int i = 0; i < NI1; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = K1 / BK;                         // multiple of RD (host check)
#pragma unroll
  for (int d = 0; d < RD; ++d) load1(d, d * BK);
  store1(0, 0);
  __syncthreads();
  for (int ks0 = 0; ks0 < nk; ks0 += RD) {
#pragma unroll
    for (int d = 0; d < RD; ++d) {
      const int ks = ks0 + d;
      const char* base = lds + (d & 1) * L::S1;   // (RD even: slab ks sits in buffer ks & 1 = d & 1)
      const char* bb = base + L::IMG * L::A1;
      Frag fa[NI1], fb[2];
#pragma unroll
      for (int i = 0; i < NI1; ++i) get_frag<EXACT>(base, L::A1, i * 16 + r16, q, fa[i]);
#pragma unroll
      for (int j = 0; j < 2; ++j) get_frag<EXACT>(bb, L::B1, wc * 32 + j * 16 + r16, q, fb[j]);
      mma_tiles<EXACT, NI1, 2>(fa, fb, acc);
      store1((d + 1) % RD, (d + 1) & 1);            // (after the last slab: zeros into a buffer nobody reads)
      load1(d, (ks + RD) * BK);                  // slot d held slab ks, stored at the previous iteration
      __syncthreads();
    }
  }

  // ================= ReLU mask, dpre → HBM and → LDS (stage-2 A operand, 8 slabs in the A layout) =============
  // accumulator layout: acc[i][j][e] = C[row 16·i + 4·q + e][col 32·wc + 16·j + r16]
  // (the dpre image aliases the stage-1 buffers: all their reads are done, barrier above). The ReLU-mask / bias
  // operands are loaded for the whole tile first (buffer loads, rows past N read 0): loads issued between the dpre
  // stores made every element one exposed round trip (load → wait → store, 32 in a row).
  {
    const __amdgpu_buffer_rsrc_t rX = rsrc(x, EPI == 0 ? (long long)N * P * 4 : (long long)P * 4);
    float xv[NI1][2][4];
#pragma unroll
    for (int i = 0; i < NI1; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = i * 16 + 4 * q + e, col = wc * 32 + j * 16 + r16;
          const int grow = r0 + row;
          if constexpr (EPI == 0) {
            xv[i][j][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                              rX, grow < N ? (grow * P + col) * 4 : kOob, 0, 0));
          } else {
            xv[i][j][e] = e == 0 && i == 0 ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                                           rX, col * 4, 0, 0))
                                           : 0.f;
          }
        }
    const __amdgpu_buffer_rsrc_t rD = rsrc(dpre, (long long)N * P * 4);
#pragma unroll
    for (int i = 0; i < NI1; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = i * 16 + 4 * q + e, col = wc * 32 + j * 16 + r16;
          const int grow = r0 + row;
          float v;
          if constexpr (EPI == 0) v = xv[i][j][e] > 0.f ? acc[i][j][e] : 0.f;
          else if constexpr (EPI == 1) v = fmaxf(acc[i][j][e] + xv[0][j][0], 0.f);
          else v = acc[i][j][e] + xv[0][j][0];
          if (grow >= N) v = 0.f;
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rD,
                                                grow < N ? (grow * P + col) * 4 : kOob, 0, 0);
          const int kk = col & (BK - 1);
          char* slab = dimg + (col / BK) * L::A1;
          if constexpr (EXACT) {
            *reinterpret_cast<float*>(slab + coff<true>(row, kk >> 2) + 4 * (kk & 3)) = v;
          } else {
            const int o = coff<false>(row, kk >> 3) + 2 * (kk & 7);
            const short h = dca::f2bf(v);
            *reinterpret_cast<short*>(slab + o) = h;
            *reinterpret_cast<short*>(slab + DIMG + o) = dca::f2bf(v - dca::bf2f(h));
          }
        }
  }

  } else if constexpr (EXACT) {
    // stage-2-only launch (K1 = 0), exact: dG (N, P) fp32 rows straight into the fp32 dpre image (8 slabs)
    for (int i = tid; i < BM * P / 4; i += NT) {
      const int row = i / (P / 4), c4 = (i % (P / 4)) * 4;
      const int grow = r0 + row;
      const float4 v = grow < N ? *reinterpret_cast<const float4*>(dG + (size_t)grow * P + c4)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
      const int kk = c4 & (BK - 1);
      *reinterpret_cast<float4*>(dimg + (c4 / BK) * L::A1 + coff<true>(row, kk >> 2)) = v;
    }
  } else {
    // stage-2-only launch (K1 = 0): the A operand is dG itself, (N, P) fp32 rows, split into the dpre image
    for (int i = tid; i < BM * P / 4; i += NT) {
      const int row = i / (P / 4), c4 = (i % (P / 4)) * 4;
      const int grow = r0 + row;
      const float4 v = grow < N ? *reinterpret_cast<const float4*>(dG + (size_t)grow * P + c4)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
      uint2 hi, lo;
      split4(v, hi, lo);
      const int kk = c4 & (BK - 1);
      char* slab = dimg + (c4 / BK) * L::A1;
      const int o = coff<false>(row, kk >> 3) + 2 * (kk & 7);
      *reinterpret_cast<uint2*>(slab + o) = hi;
      *reinterpret_cast<uint2*>(slab + DIMG + o) = lo;
    }
  }

  // ================= stage 2: dx (64 × X) = dpre · W_pre, 128-column chunks =================
  if (X == 0) return;                             // (stage-1-only launch: X = 0)
  char* s2 = lds + L::D;
  constexpr int nk2 = P / BK;
  const int nchunk = X / XC, total = nchunk * nk2;   // multiple of RD (nk2 = 8)
  const int cr = tid & 127, cq = tid >> 7;        // W2 slab: row, chunk (8 k)
  uint4 sw[RD][2];
  auto load2 = [&](int slot, int it) {             // branch-free like load1 (it ≥ total: zeros)
    const int c0 = (it / nk2) * XC, kb = it % nk2;
    if constexpr (EXACT) {
      const int o = it < total ? ((c0 + cr) * P + kb * BK + 8 * cq) * ES : kOob;
      sw[slot][0] = ld16(rW2h, o);
      sw[slot][1] = ld16(rW2h, o + 16);
    } else {                                      // slab-major images: rows c0 … c0+127 of k-block kb, 8 KB
      const int o = it < total ? (kb * X + c0) * 64 + tid * 16 : kOob;
      sw[slot][0] = ld16(rW2h, o);
      sw[slot][1] = ld16(rW2l, o);
    }
  };
  auto store2 = [&](int slot, int buf) {
    char* bb = s2 + buf * L::S2;
    if constexpr (EXACT) {
      *reinterpret_cast<uint4*>(bb + coff<true>(cr, 2 * cq)) = sw[slot][0];
      *reinterpret_cast<uint4*>(bb + coff<true>(cr, 2 * cq + 1)) = sw[slot][1];
    } else {
      const int o = coff<false>(tid >> 2, tid & 3);
      *reinterpret_cast<uint4*>(bb + o) = sw[slot][0];
      *reinterpret_cast<uint4*>(bb + L::B2 + o) = sw[slot][1];
    }
  };
  const int vc = w;                              // 1 × 8 waves: all BM rows, cols 16·vc of the chunk
  f32x4 acc2[NI1][1];
#pragma unroll
  for (int i = 0; i < NI1; ++i) acc2[i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t rDx = rsrc(dx, (long long)N * X * 4);
#pragma unroll
  for (int d = 0; d < RD; ++d) load2(d, d);
  store2(0, 0);
  __syncthreads();                                // dpre tile and the first W_pre slab are in LDS
  for (int it0 = 0; it0 < total; it0 += RD) {
#pragma unroll
    for (int d = 0; d < RD; ++d) {
      const int it = it0 + d;
      const int chunk = it / nk2, ks = it % nk2;
      const char* bb = s2 + (d & 1) * L::S2;
      Frag fa[NI1], fb[1];
#pragma unroll
      for (int i = 0; i < NI1; ++i) get_frag<EXACT>(dimg + ks * L::A1, DIMG, i * 16 + r16, q, fa[i]);
      get_frag<EXACT>(bb, L::B2, vc * 16 + r16, q, fb[0]);
      mma_tiles<EXACT, NI1, 1>(fa, fb, acc2);
      store2((d + 1) % RD, (d + 1) & 1);
      load2(d, it + RD);
      if (ks == nk2 - 1) {                        // chunk done: store its BM × 128 output tile (rows past N dropped)
#pragma unroll
        for (int i = 0; i < NI1; ++i) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int grow = r0 + i * 16 + 4 * q + e;
            // (through a scalar: __builtin_bit_cast of the vector element itself compiled to element 0 for every e)
            const float v = acc2[i][0][e];
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rDx,
                                                  grow < N ? (grow * X + chunk * XC + vc * 16 + r16) * 4 : kOob, 0, 0);
          }
          acc2[i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      __syncthreads();
    }
  }
}

// fp32 → hi / lo bf16 images (x = hi + lo), 4 elements per thread
__global__ __launch_bounds__(256) void split_bf16x2_kernel(const float4* __restrict__ src, uint2* __restrict__ hi,
                                                           uint2* __restrict__ lo, int n4) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n4) split4(src[i], hi[i], lo[i]);
}

// fp32 (R, K) row-major → hi / lo images in SLAB-MAJOR order [K/32][R][32] (the bf16x3 operand layout of
// dpre_dx_kernel: one 32-deep slab of all R rows is contiguous)
__global__ __launch_bounds__(256) void split_bf16x2_blk_kernel(const float4* __restrict__ src, uint2* __restrict__ hi,
                                                               uint2* __restrict__ lo, int R, int K) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= R * (K / 4)) return;
  const int r = (4 * i) / K, k = (4 * i) % K;
  const int o4 = ((((k >> 5) * R + r) << 5) + (k & 31)) >> 2;
  split4(src[i], hi[o4], lo[o4]);
}

}  // namespace

// src (R, K) fp32 → slab-major hi / lo images [K/32][R][32] (K % 32 == 0)
extern "C" hipError_t dca_split_bf16x2_blk(const float* src, short* hi, short* lo, int R, int K, hipStream_t stream) {
  if (K % 32 != 0 || R < 1) return hipErrorInvalidValue;
  const int n4 = R * (K / 4);
  hipLaunchKernelGGL(split_bf16x2_blk_kernel, dim3((n4 + 255) / 256), dim3(256), 0, stream,
                     reinterpret_cast<const float4*>(src), reinterpret_cast<uint2*>(hi), reinterpret_cast<uint2*>(lo),
                     R, K);
  return hipGetLastError();
}

// src (n fp32, n % 4 == 0) → hi, lo (n bf16 each)
extern "C" hipError_t dca_split_bf16x2(const float* src, short* hi, short* lo, long long n, hipStream_t stream) {
  if (n % 4 != 0) return hipErrorInvalidValue;
  const int n4 = (int)(n / 4);
  if (n4 == 0) return hipSuccess;
  hipLaunchKernelGGL(split_bf16x2_kernel, dim3((n4 + 255) / 256), dim3(256), 0, stream,
                     reinterpret_cast<const float4*>(src), reinterpret_cast<uint2*>(hi), reinterpret_cast<uint2*>(lo),
                     n4);
  return hipGetLastError();
}

// dG (N, K1) f32 row-major; x (N, P) f32 (ReLU outputs). Weights: bf16x3 (exact = 0): w1h / w1l = slab-major
// hi / lo images [K1/32][P][32] of W_ihᵀ (P, K1), w2h / w2l = [P/32][X][32] of W_preᵀ (X, P) (dca_split_bf16x2_blk);
// exact: w1h (P, K1), w2h (X, P) fp32 row-major (w1l / w2l unused). Outputs dpre (N, P), dx (N, X) f32. K1 % 128 == 0, X % 128 == 0.
// epi = 1: the forward chain (dG = x896, x = the pre-RNN bias (P), dpre = relu(x896·W_preᵀ + b), dx = that · W_ihᵀ).
extern "C" hipError_t dca_dpre_dx(const float* dG, const void* w1h, const void* w1l, const float* x, const void* w2h,
                                  const void* w2l, float* dpre, float* dx, int N, int K1, int X, int exact,
                                  int epi, hipStream_t stream) {
  // K1 = 0: stage 2 only (A = dG (N, P)); X = 0: stage 1 only
  if (N < 1 || (K1 == 0 && X == 0) || K1 < 0 || K1 % (RD * BK) != 0 || X < 0 || X % XC != 0 ||
      ((X / XC) * (P / BK)) % RD != 0 || epi < 0 || epi > 2)
    return hipErrorInvalidValue;
  if ((long long)N * K1 * 4 > 0x7fff0000LL) return hipErrorInvalidValue;      // buffer-resource range
  const int grid = (N + BM - 1) / BM;
#define DCA_DX_LAUNCH(EX, EP)                                                                                    \
  hipLaunchKernelGGL((dpre_dx_kernel<EX, EP>), dim3(grid), dim3(NT), 0, stream, dG, w1h, w1l, x, w2h, w2l, dpre, dx, \
                     N, K1, X)
  if (exact) {
    if (epi == 0) DCA_DX_LAUNCH(true, 0);
    else if (epi == 1) DCA_DX_LAUNCH(true, 1);
    else DCA_DX_LAUNCH(true, 2);
  } else {
    if (epi == 0) DCA_DX_LAUNCH(false, 0);
    else if (epi == 1) DCA_DX_LAUNCH(false, 1);
    else DCA_DX_LAUNCH(false, 2);
  }
#undef DCA_DX_LAUNCH
  return hipGetLastError();
}
