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
// One 512-thread workgroup (8 waves) per 64-row tile; the 64 × P dpre tile never leaves the workgroup between the
// two products (it is written once to HBM for the pre-RNN weight gradient, and kept in LDS as the second product's
// A operand):
// * stage 1, K = 4H in 32-deep slabs, double-buffered through LDS (register-staged 16-B loads of the next slab
//   issued before the current slab's MFMAs, one barrier per slab); waves as 2 (32 rows) × 4 (64 columns), each
//   2 × 4 v_mfma_f32_16x16x32_bf16 tiles;
// * ReLU mask + dpre store in the accumulator layout, dpre written into LDS;
// * stage 2, X in 128-column chunks × K = P in 32-deep slabs (same double-buffered pipeline), waves as 4 (16 rows) ×
//   2 (64 columns).
// Operands are fp32; both weight operands come K-contiguous per output column (W_ihᵀ image (P × 4H) and W_preᵀ
// image (X × P), models/pipelined.py WeightImages), so every MFMA fragment is a plain 16-B LDS read.
// EXACT = false: bf16x3 — every fp32 value is split ONCE while staging into hi + lo bf16 LDS images and each product
// is hi·hi + lo·hi + hi·lo on the bf16 MFMA (≈2⁻¹⁶ relative per product, the fp32 learner's accuracy class);
// EXACT = true: exact fp32 on v_mfma_f32_16x16x4_f32 — the 16x16x32 fragment's 8 k values of a lane feed 8 chained
// 16x16x4 MFMAs (call j takes element j: lane l contributes k = 8·(l/16) + j, so the 8 calls cover all 32 k).
#include "common.h"

namespace {

using dca::bf16x8;
using dca::f32x4;

constexpr int BM = 64, BK = 32, NT = 512, P = 256, XC = 128, RD = 4;

template <bool EXACT>
struct Lay {
  // bytes per operand row of one 32-deep slab: hi/lo bf16 (64 B + 16 pad) or fp32 (128 B + 16 pad)
  static constexpr int RP = EXACT ? 144 : 80;
  static constexpr int IMG = EXACT ? 1 : 2;              // images per operand (hi, lo)
  static constexpr int A1 = BM * RP;                      // stage-1 A image bytes
  static constexpr int B1 = P * RP;                       // stage-1 B image bytes
  static constexpr int S1 = IMG * (A1 + B1);              // one stage-1 buffer
  static constexpr int DP = EXACT ? (P * 4 + 16) : (P * 2 + 16);   // dpre row pitch
  static constexpr int D = IMG * BM * DP;                 // dpre tile (A operand of stage 2)
  static constexpr int B2 = XC * RP;                      // stage-2 B image bytes
  static constexpr int S2 = IMG * B2;
  static constexpr int BYTES = (2 * S1 > D + 2 * S2) ? 2 * S1 : D + 2 * S2;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, long long bytes) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int nb = (int)(bytes > 0x7fff0000LL ? 0x7fff0000LL : bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(nb), 0x00020000);
}
__device__ __forceinline__ float4 ld4(__amdgpu_buffer_rsrc_t r, int off) {   // out of range → zeros
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// ---- staging: 4 consecutive fp32 values of one operand row → LDS (hi / lo bf16 images, or fp32)
template <bool EXACT>
__device__ __forceinline__ void put4(char* img, int img_bytes, int row, int k, float4 v) {
  const int off = row * Lay<EXACT>::RP + k * (EXACT ? 4 : 2);
  if constexpr (EXACT) {
    *reinterpret_cast<float4*>(img + off) = v;
  } else {
    const short h0 = dca::f2bf(v.x), h1 = dca::f2bf(v.y), h2 = dca::f2bf(v.z), h3 = dca::f2bf(v.w);
    const short l0 = dca::f2bf(v.x - dca::bf2f(h0)), l1 = dca::f2bf(v.y - dca::bf2f(h1)),
                l2 = dca::f2bf(v.z - dca::bf2f(h2)), l3 = dca::f2bf(v.w - dca::bf2f(h3));
    *reinterpret_cast<uint2*>(img + off) = make_uint2((unsigned)(unsigned short)h0 | ((unsigned)(unsigned short)h1 << 16),
                                                      (unsigned)(unsigned short)h2 | ((unsigned)(unsigned short)h3 << 16));
    *reinterpret_cast<uint2*>(img + img_bytes + off) =
        make_uint2((unsigned)(unsigned short)l0 | ((unsigned)(unsigned short)l1 << 16),
                   (unsigned)(unsigned short)l2 | ((unsigned)(unsigned short)l3 << 16));
  }
}

// one MFMA fragment (row `row` of an image, k chunk q = lane/16 of the 32-deep slab)
struct Frag {
  bf16x8 hi, lo;        // bf16x3
  float f[8];           // exact
};
template <bool EXACT>
__device__ __forceinline__ void get_frag(const char* img, int img_bytes, int row_off, int q, Frag& fr) {
  if constexpr (EXACT) {
    const float4 a = *reinterpret_cast<const float4*>(img + row_off + q * 32);
    const float4 b = *reinterpret_cast<const float4*>(img + row_off + q * 32 + 16);
    fr.f[0] = a.x; fr.f[1] = a.y; fr.f[2] = a.z; fr.f[3] = a.w;
    fr.f[4] = b.x; fr.f[5] = b.y; fr.f[6] = b.z; fr.f[7] = b.w;
  } else {
    fr.hi = *reinterpret_cast<const bf16x8*>(img + row_off + q * 16);
    fr.lo = *reinterpret_cast<const bf16x8*>(img + img_bytes + row_off + q * 16);
  }
}
template <bool EXACT>
__device__ __forceinline__ f32x4 mma(const Frag& a, const Frag& b, f32x4 c) {
  if constexpr (EXACT) {
#pragma unroll
    for (int j = 0; j < 8; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.f[j], b.f[j], c, 0, 0, 0);
    return c;
  } else {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo, b.hi, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.lo, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.hi, c, 0, 0, 0);
  }
}

template <bool EXACT>
__global__ __launch_bounds__(NT, 1) void dpre_dx_kernel(const float* __restrict__ dG, const float* __restrict__ wihT,
                                                        const float* __restrict__ x, const float* __restrict__ wpreT,
                                                        float* __restrict__ dpre, float* __restrict__ dx, int N,
                                                        int K1, int X) {
  using L = Lay<EXACT>;
  __shared__ __attribute__((aligned(16))) char lds[L::BYTES];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r16 = lane & 15, q = lane >> 4;
  const int r0 = blockIdx.x * BM;
  const __amdgpu_buffer_rsrc_t rA = rsrc(dG, (long long)N * K1 * 4);
  const __amdgpu_buffer_rsrc_t rW1 = rsrc(wihT, (long long)P * K1 * 4);
  const __amdgpu_buffer_rsrc_t rW2 = rsrc(wpreT, (long long)X * P * 4);
  constexpr int kOob = 0x7fff8000;

  // ================= stage 1: C1 (64 × P) = dG[r0:r0+64] · W_ih =================
  // staging map: A slab 64 rows × 32 k = 512 float4 (one per thread: row t/8, k 4·(t%8));
  //              B slab P cols × 32 k = 2048 float4 (four per thread: col t/2, k 16·(t%2) + 4·i)
  const int ar = tid >> 3, ak = (tid & 7) * 4;
  const int bc = tid >> 1, bk = (tid & 1) * 16;
  const int arow = r0 + ar;
  const int a_off0 = arow < N ? (arow * K1 + ak) * 4 : kOob;
  const int b_off0 = (bc * K1 + bk) * 4;
  // register ring of RD slabs in flight: the slab stored into LDS at iteration ks was loaded at ks + 1 - RD, so
  // RD - 1 slabs of MFMA work cover each load's latency (one slab of lead was 4x slower: every store waited out a
  // full memory round trip)
  float4 sa[RD], sb[RD][4];
  auto load1 = [&](int slot, int k0) {
    sa[slot] = ld4(rA, a_off0 == kOob ? kOob : a_off0 + k0 * 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) sb[slot][i] = ld4(rW1, b_off0 + (k0 + 4 * i) * 4);
  };
  auto store1 = [&](int slot, int buf) {
    char* base = lds + buf * L::S1;
    put4<EXACT>(base, L::A1, ar, ak, sa[slot]);
    char* bb = base + L::IMG * L::A1;
#pragma unroll
    for (int i = 0; i < 4; ++i) put4<EXACT>(bb, L::B1, bc, bk + 4 * i, sb[slot][i]);
  };
  const int wr = w >> 2, wc = w & 3;             // 2 × 4 waves: rows 32·wr, cols 64·wc
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
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
      Frag fa[2], fb[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) get_frag<EXACT>(base, L::A1, (wr * 32 + i * 16 + r16) * L::RP, q, fa[i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) get_frag<EXACT>(bb, L::B1, (wc * 64 + j * 16 + r16) * L::RP, q, fb[j]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mma<EXACT>(fa[i], fb[j], acc[i][j]);
      if (ks + 1 < nk) store1((d + 1) % RD, (d + 1) & 1);
      if (ks + RD < nk) load1(d, (ks + RD) * BK);  // slot d held slab ks, stored at the previous iteration
      __syncthreads();
    }
  }

  // ================= ReLU mask, dpre → HBM and → LDS (stage-2 A operand) =================
  // accumulator layout: acc[i][j][e] = C[row 32·wr + 16·i + 4·q + e][col 64·wc + 16·j + r16]
  char* dimg = lds;                               // aliases the stage-1 buffers (all reads done: barrier above)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wr * 32 + i * 16 + 4 * q + e, col = wc * 64 + j * 16 + r16;
        const int grow = r0 + row;
        float v = 0.f;
        if (grow < N) {
          v = x[(size_t)grow * P + col] > 0.f ? acc[i][j][e] : 0.f;
          dpre[(size_t)grow * P + col] = v;
        }
        if constexpr (EXACT) {
          *reinterpret_cast<float*>(dimg + row * L::DP + col * 4) = v;
        } else {
          const short h = dca::f2bf(v);
          *reinterpret_cast<short*>(dimg + row * L::DP + col * 2) = h;
          *reinterpret_cast<short*>(dimg + BM * L::DP + row * L::DP + col * 2) = dca::f2bf(v - dca::bf2f(h));
        }
      }

  // ================= stage 2: dx (64 × X) = dpre · W_pre, 128-column chunks =================
  // staging map: B slab 128 cols × 32 k = 1024 float4 (two per thread: col t/4, k 8·(t%4) + 4·i)
  char* s2 = lds + L::D;
  const int cc = tid >> 2, ck = (tid & 3) * 8;
  constexpr int nk2 = P / BK;
  float4 sw[RD][2];
  auto load2 = [&](int slot, int it) {
    const int c0 = (it / nk2) * XC, k0 = (it % nk2) * BK;
#pragma unroll
    for (int i = 0; i < 2; ++i) sw[slot][i] = ld4(rW2, ((c0 + cc) * P + k0 + ck + 4 * i) * 4);
  };
  auto store2 = [&](int slot, int buf) {
    char* bb = s2 + buf * L::S2;
#pragma unroll
    for (int i = 0; i < 2; ++i) put4<EXACT>(bb, L::B2, cc, ck + 4 * i, sw[slot][i]);
  };
  const int vr = w >> 1, vc = w & 1;             // 4 × 2 waves: rows 16·vr, cols 64·vc of the chunk
  const int nchunk = X / XC, total = nchunk * nk2;   // multiple of RD (nk2 = 8)
  f32x4 acc2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc2[j] = f32x4{0.f, 0.f, 0.f, 0.f};
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
      Frag fa, fb[4];
      // A fragment: dpre row 16·vr + r16, k = 32·ks + 8·q … (the dpre image holds the full K = P per row)
      if constexpr (EXACT) {
        get_frag<true>(dimg, 0, (vr * 16 + r16) * L::DP + ks * BK * 4, q, fa);
      } else {
        get_frag<false>(dimg, BM * L::DP, (vr * 16 + r16) * L::DP + ks * BK * 2, q, fa);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) get_frag<EXACT>(bb, L::B2, (vc * 64 + j * 16 + r16) * L::RP, q, fb[j]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc2[j] = mma<EXACT>(fa, fb[j], acc2[j]);
      if (it + 1 < total) store2((d + 1) % RD, (d + 1) & 1);
      if (it + RD < total) load2(d, it + RD);
      if (ks == nk2 - 1) {                        // chunk done: store its 64 × 128 output tile
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int grow = r0 + vr * 16 + 4 * q + e;
            if (grow < N) dx[(size_t)grow * X + chunk * XC + vc * 64 + j * 16 + r16] = acc2[j][e];
          }
          acc2[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      __syncthreads();
    }
  }
}

}  // namespace

extern "C" size_t dca_dpre_dx_lds(int exact) { return exact ? Lay<true>::BYTES : Lay<false>::BYTES; }

// dG (N, K1) f32 row-major; wihT (P=256, K1) f32 (K-contiguous per output column); x (N, P) f32 (ReLU outputs);
// wpreT (X, P) f32; outputs dpre (N, P), dx (N, X) f32. K1 % 32 == 0, X % 128 == 0.
extern "C" hipError_t dca_dpre_dx(const float* dG, const float* wihT, const float* x, const float* wpreT, float* dpre,
                                  float* dx, int N, int K1, int X, int exact, hipStream_t stream) {
  if (N < 1 || K1 < RD * BK || K1 % (RD * BK) != 0 || X < XC || X % XC != 0 || ((X / XC) * (P / BK)) % RD != 0)
    return hipErrorInvalidValue;
  if ((long long)N * K1 * 4 > 0x7fff0000LL) return hipErrorInvalidValue;      // buffer-resource range
  const int grid = (N + BM - 1) / BM;
  if (exact) {
    hipLaunchKernelGGL(dpre_dx_kernel<true>, dim3(grid), dim3(NT), 0, stream, dG, wihT, x, wpreT, dpre, dx, N, K1, X);
  } else {
    hipLaunchKernelGGL(dpre_dx_kernel<false>, dim3(grid), dim3(NT), 0, stream, dG, wihT, x, wpreT, dpre, dx, N, K1, X);
  }
  return hipGetLastError();
}
