// Fused entity encoder for gfx950: unit MLP (10→128, ReLU) → per-type Linear(128→128) → max-pool (+argmax),
// forward and backward. Reference: policy.py:97-138 (affine_env, affine_unit_basic_stats, affine_unit_<type>,
// torch.max over units, concat); SURVEY §2.3 K-env, K-unit-basic, K-unit-type, K-maxpool.
//
// Tiling. A workgroup owns 32 timestep rows = two 16-row groups g. Every MFMA M-tile is (unit type τ, unit slot u,
// 16 rows of group g), so all 16 rows of a tile share one weight matrix W_τ and the max-pool over a type's units is an
// ELEMENT-WISE running max across that type's tiles, kept in registers (no cross-lane or cross-wave reduction).
// Wave jobs (balanced for both 1v1 (1,5,16,16,1,1) and 5v5 (5,5,24,24,3,3) layouts):
//   waves 0,1: types {anh, eh, ath} for groups 0,1     waves 2,3: types {enh, ah, eth} for groups 0,1
// Per tile:
//   layer 1 : 16×10 units · W1ᵀ on v_mfma_f32_16x16x4_f32 (exact fp32, K padded to 12), +b1, ReLU
//   → bf16 C-tile transposed through a per-wave LDS scratch into A-fragments
//   layer 2 : 16×128 · W_τᵀ on v_mfma_f32_16x16x32_bf16 with W_τ held in 128 VGPRs for the whole type job
//   → +b_τ, running max/argmax per (row, column), bf16 embedding tile staged through LDS for 16-B coalesced stores.
// Backward recomputes layer 1, builds ∂emb = dtl⊗q + scatter(∂pool at argmax) in A-fragment layout, computes
// ∂basic = ∂emb·W_τ (MFMA, W_τᵀ in VGPRs), applies ReLU', accumulates ∂W1 in-register on
// v_mfma_f32_16x16x16_bf16 (the C-layout ∂basic tile IS the A operand), and writes ∂emb and basic activations
// (bf16, type-major) so ∂W_τ = ∂emb_τᵀ·basic_τ runs as one large-K hipBLASLt GEMM per type.
#include "common.h"

namespace {

using dca::bf16x8;
using dca::bf16x4;
using dca::f32x4;

constexpr int kD = 128;          // embedding width
constexpr int kF = 10;           // unit features
constexpr int kRows = 32;        // rows per workgroup
constexpr int kLd = kD + 8;      // LDS scratch row stride (bf16): 272 B breaks the 256-B bank period

struct Layout {
  int U;
  int cnt[6];
  int off[6];
};

struct FwdParams {
  const float* units;   // (N, U, 10)
  const float* env;     // (N, 3)
  const float* w1;      // (128, 10)
  const float* b1;      // (128)
  const short* wt;      // (6, 128, 128) bf16  W_τ (out, in)
  const float* bt;      // (6, 128)
  const float* we;      // (128, 3)
  const float* be;      // (128)
  short* x896;          // (N, 896) bf16 out: [env | pool_ah | pool_eh | pool_anh | pool_enh | pool_ath | pool_eth]
  short* emb;           // (N, U, 128) bf16 out
  unsigned char* arg;   // (N, 6, 128) u8 out
  int N;
  int compat;           // reference bug: eth pool = enh pool (policy.py:127)
  Layout L;
};

struct BwdParams {
  const float* units;
  const float* w1;
  const float* b1;
  const short* wtT;     // (6, 128, 128) bf16  W_τᵀ (in, out)
  const float* dtl;     // (N, U) ∂L/∂pointer-logit
  const float* q;       // pointer query, row stride ldq
  int ldq;
  const float* dx;      // (N, 896) f32 ∂L/∂x896
  const unsigned char* arg;
  short* demb;          // type-major bf16: type τ block at rowbase[τ], row m = u·N + n
  short* basic;         // same layout
  float* dw1;           // (128, 10) f32 accumulated with atomics
  float* db1;           // (128)
  int N;
  int compat;
  Layout L;
  long long rowbase[6];
};

__device__ __forceinline__ void type_job(int wv, int j, int& tau, int& g) {
  // wave job list: j-th job of wave wv; returns tau = -1 when done
  const int lists[2][3] = {{2, 1, 4}, {3, 0, 5}};
  g = wv & 1;
  tau = (j < 3) ? lists[wv >> 1][j] : -1;
}

// ------------------------------------------------------------------------------------------------------------
// Layer 1 for a 16-row tile on fp32 MFMA. Returns C-layout (rows (lane>>4)*4+r, col 16n + lane&15) pre-activations.
__device__ __forceinline__ void layer1(const float* __restrict__ units, int U, int N, int row0, int uslot,
                                      const float (&w1f)[8][3], f32x4 (&acc)[8], int lane) {
  const int i = lane & 15, kq = lane >> 4;
  const int row = row0 + i;
  float a[3];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int k = 4 * s + kq;
    a[s] = (row < N && k < kF) ? units[((size_t)row * U + uslot) * kF + k] : 0.f;
  }
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 3; ++s) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], w1f[n][s], c, 0, 0, 0);
    acc[n] = c;
  }
}

__device__ __forceinline__ void load_w1(const float* __restrict__ w1, float (&w1f)[8][3], int lane) {
  const int kq = lane >> 4, j = lane & 15;
#pragma unroll
  for (int n = 0; n < 8; ++n)
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int k = 4 * s + kq;
      w1f[n][s] = (k < kF) ? w1[(16 * n + j) * kF + k] : 0.f;
    }
}

// B fragments of a 128×128 bf16 matrix M stored row-major [col][k] (i.e. B[k][col] = M[col][k]).
__device__ __forceinline__ void load_bfrags(const short* __restrict__ m, bf16x8 (&bf)[8][4], int lane) {
  const int j = lane & 15, kg = lane >> 4;
#pragma unroll
  for (int n = 0; n < 8; ++n)
#pragma unroll
    for (int s = 0; s < 4; ++s)
      bf[n][s] = *reinterpret_cast<const bf16x8*>(m + (size_t)(16 * n + j) * kD + 32 * s + 8 * kg);
}

// ============================================================================================================
__global__ __launch_bounds__(256, 1) void encoder_fwd_kernel(FwdParams P) {
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int rbase = blockIdx.x * kRows;
  const int U = P.L.U, N = P.N;
  __shared__ __attribute__((aligned(16))) short scr[4][16][kLd];

  // ---- env embedding: relu(We·env + be) → x896[:, 0:128] (32 rows × 128 cols over 256 threads)
  {
    const int r = tid >> 3, c0 = (tid & 7) * 16;
    const int row = rbase + r;
    if (row < N) {
      const float e0 = P.env[row * 3], e1 = P.env[row * 3 + 1], e2 = P.env[row * 3 + 2];
      for (int c = c0; c < c0 + 16; ++c) {
        const float v = P.be[c] + P.we[c * 3] * e0 + P.we[c * 3 + 1] * e1 + P.we[c * 3 + 2] * e2;
        P.x896[(size_t)row * 896 + c] = dca::f2bf(fmaxf(v, 0.f));
      }
    }
  }

  float w1f[8][3];
  load_w1(P.w1, w1f, lane);
  float b1v[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) b1v[n] = P.b1[16 * n + (lane & 15)];

  const int i = lane & 15, kg = lane >> 4;
  for (int j = 0; j < 3; ++j) {
    int tau, g;
    type_job(wv, j, tau, g);
    const int cnt = P.L.cnt[tau], uoff = P.L.off[tau];
    if (cnt == 0) continue;
    const int row0 = rbase + 16 * g;
    bf16x8 wf[8][4];
    load_bfrags(P.wt + (size_t)tau * kD * kD, wf, lane);
    float btv[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) btv[n] = P.bt[tau * kD + 16 * n + i];
    f32x4 pmax[8];
    int parg[8][4];
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      pmax[n] = (f32x4){-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
      for (int r = 0; r < 4; ++r) parg[n][r] = 0;
    }
    for (int u = 0; u < cnt; ++u) {
      f32x4 acc[8];
      layer1(P.units, U, N, row0, uoff + u, w1f, acc, lane);
      // basic = relu(acc + b1) → bf16 → scratch [row][col]
#pragma unroll
      for (int n = 0; n < 8; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          scr[wv][kg * 4 + r][16 * n + i] = dca::f2bf(fmaxf(acc[n][r] + b1v[n], 0.f));
      __builtin_amdgcn_wave_barrier();
      bf16x8 af[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) af[s] = *reinterpret_cast<const bf16x8*>(&scr[wv][i][32 * s + 8 * kg]);
      __builtin_amdgcn_wave_barrier();
      // layer 2
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s], wf[n][s], c, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = c[r] + btv[n];
          if (v > pmax[n][r]) { pmax[n][r] = v; parg[n][r] = u; }
          scr[wv][kg * 4 + r][16 * n + i] = dca::f2bf(v);
        }
      }
      __builtin_amdgcn_wave_barrier();
      // coalesced store of the 16×128 bf16 embedding tile: lane → (row lane>>2, 64-B chunk lane&3)
      {
        const int rr = lane >> 2, ch = lane & 3;
        const int row = row0 + rr;
        if (row < N) {
          const bf16x8* src = reinterpret_cast<const bf16x8*>(&scr[wv][rr][32 * ch]);
          bf16x8* dst = reinterpret_cast<bf16x8*>(P.emb + ((size_t)row * U + uoff + u) * kD + 32 * ch);
#pragma unroll
          for (int q = 0; q < 4; ++q) dst[q] = src[q];
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    // ---- flush pool + argmax for this (type, group); compat: eth pool is overwritten by enh (host side)
#pragma unroll
    for (int n = 0; n < 8; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + kg * 4 + r;
        if (row < N) {
          const int col = 16 * n + i;
          P.x896[(size_t)row * 896 + kD + tau * kD + col] = dca::f2bf(pmax[n][r]);
          P.arg[((size_t)row * 6 + tau) * kD + col] = (unsigned char)parg[n][r];
        }
      }
  }
}

// ============================================================================================================
__global__ __launch_bounds__(256, 1) void encoder_bwd_kernel(BwdParams P) {
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int rbase = blockIdx.x * kRows;
  const int U = P.L.U, N = P.N;
  const int i = lane & 15, kg = lane >> 4;
  __shared__ __attribute__((aligned(16))) short scr[4][16][kLd];

  float w1f[8][3];
  load_w1(P.w1, w1f, lane);
  float b1v[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) b1v[n] = P.b1[16 * n + i];
  f32x4 dw1acc[8];
  float db1acc[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    dw1acc[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
    db1acc[n] = 0.f;
  }

  for (int j = 0; j < 3; ++j) {
    int tau, g;
    type_job(wv, j, tau, g);
    const int cnt = P.L.cnt[tau], uoff = P.L.off[tau];
    if (cnt == 0) continue;
    const int row0 = rbase + 16 * g;
    bf16x8 wf[8][4];   // B[k=e][n=j] = W_τ[e][j] = W_τᵀ[j][e]
    load_bfrags(P.wtT + (size_t)tau * kD * kD, wf, lane);
    // per-lane A-layout row data reused across the type's units: q and ∂pool (8 cols × 4 k-steps)
    const int arow = row0 + i;
    const bool rok = arow < N;
    const bool eth_dead = P.compat && tau == 5;   // reference bug: eth pool unused → no pool gradient
    for (int u = 0; u < cnt; ++u) {
      // ---- recompute layer 1 (C layout) → basic f32 + bf16 staged for the type-major store
      f32x4 acc[8];
      layer1(P.units, U, N, row0, uoff + u, w1f, acc, lane);
      f32x4 bas[8];
#pragma unroll
      for (int n = 0; n < 8; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) bas[n][r] = fmaxf(acc[n][r] + b1v[n], 0.f);
      // ---- ∂emb in A layout: lane (row i, cols 32s + 8kg + jj)
      const float dtl = rok ? P.dtl[(size_t)arow * U + uoff + u] : 0.f;
      bf16x8 de[4];
      const size_t mrow = (size_t)u * N + arow;   // row within the type-major block of τ
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int e0 = 32 * s + 8 * kg;
        float v[8];
        if (rok) {
          const float4 qa = *reinterpret_cast<const float4*>(P.q + (size_t)arow * P.ldq + e0);
          const float4 qb = *reinterpret_cast<const float4*>(P.q + (size_t)arow * P.ldq + e0 + 4);
          v[0] = dtl * qa.x; v[1] = dtl * qa.y; v[2] = dtl * qa.z; v[3] = dtl * qa.w;
          v[4] = dtl * qb.x; v[5] = dtl * qb.y; v[6] = dtl * qb.z; v[7] = dtl * qb.w;
          if (!eth_dead) {
            const float* dp = P.dx + (size_t)arow * 896 + kD + tau * kD + e0;
            const unsigned char* ag = P.arg + ((size_t)arow * 6 + tau) * kD + e0;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) v[jj] += (ag[jj] == u) ? dp[jj] : 0.f;
          }
          if (P.compat && tau == 3) {   // eth pool = enh pool: its gradient lands on enh argmax units
            const float* dp = P.dx + (size_t)arow * 896 + kD + 5 * kD + e0;
            const unsigned char* ag = P.arg + ((size_t)arow * 6 + 3) * kD + e0;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) v[jj] += (ag[jj] == u) ? dp[jj] : 0.f;
          }
        } else {
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) v[jj] = 0.f;
        }
        bf16x8 h;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) h[jj] = dca::f2bf(v[jj]);
        de[s] = h;
        if (rok) *reinterpret_cast<bf16x8*>(P.demb + P.rowbase[tau] * kD + mrow * kD + e0) = h;
      }
      // ---- ∂basic = ∂emb · W_τ, ReLU' → C layout
      f32x4 dbp[8];
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(de[s], wf[n][s], c, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) c[r] = bas[n][r] > 0.f ? c[r] : 0.f;
        dbp[n] = c;
      }
      // ---- ∂W1 += ∂basicᵀ · units  (16x16x16 bf16: A[j][m] = ∂basic C-tile, B[m][k] = units)
      bf16x4 ub;
      {
        const int kk = lane & 15;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = row0 + 4 * kg + r;
          const float x = (row < N && kk < kF) ? P.units[((size_t)row * U + uoff + u) * kF + kk] : 0.f;
          ub[r] = dca::f2bf(x);
        }
      }
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        bf16x4 a;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          a[r] = dca::f2bf(dbp[n][r]);
          db1acc[n] += dbp[n][r];
        }
        dw1acc[n] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, ub, dw1acc[n], 0, 0, 0);
      }
      // ---- store basic (bf16, type-major) via the LDS scratch for coalescing
#pragma unroll
      for (int n = 0; n < 8; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) scr[wv][kg * 4 + r][16 * n + i] = dca::f2bf(bas[n][r]);
      __builtin_amdgcn_wave_barrier();
      {
        const int rr = lane >> 2, ch = lane & 3;
        const int row = row0 + rr;
        if (row < N) {
          const bf16x8* src = reinterpret_cast<const bf16x8*>(&scr[wv][rr][32 * ch]);
          bf16x8* dst = reinterpret_cast<bf16x8*>(P.basic + P.rowbase[tau] * kD + ((size_t)u * N + row) * kD + 32 * ch);
#pragma unroll
          for (int q = 0; q < 4; ++q) dst[q] = src[q];
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  // ---- flush ∂W1 (rows j = 16n + 4kg + r, col k = lane&15 < 10) and ∂b1
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    const int k = lane & 15;
    if (k < kF) {
#pragma unroll
      for (int r = 0; r < 4; ++r) atomicAdd(&P.dw1[(16 * n + 4 * kg + r) * kF + k], dw1acc[n][r]);
    }
    float s = db1acc[n];
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    if (kg == 0) atomicAdd(&P.db1[16 * n + i], s);
  }
}

}  // namespace

extern "C" hipError_t dca_encoder_fwd(const float* units, const float* env, const float* w1, const float* b1,
                                      const short* wt, const float* bt, const float* we, const float* be, short* x896,
                                      short* emb, unsigned char* arg, int N, int U, const int* counts, int compat,
                                      hipStream_t st) {
  FwdParams P{units, env, w1, b1, wt, bt, we, be, x896, emb, arg, N, compat, {}};
  P.L.U = U;
  int acc = 0;
  for (int t = 0; t < 6; ++t) { P.L.cnt[t] = counts[t]; P.L.off[t] = acc; acc += counts[t]; }
  if (acc != U || U > 64) return hipErrorInvalidValue;
  encoder_fwd_kernel<<<(N + kRows - 1) / kRows, 256, 0, st>>>(P);
  return hipGetLastError();
}

extern "C" hipError_t dca_encoder_bwd(const float* units, const float* w1, const float* b1, const short* wtT,
                                      const float* dtl, const float* q, int ldq, const float* dx,
                                      const unsigned char* arg, short* demb, short* basic, float* dw1, float* db1,
                                      int N, int U, const int* counts, int compat, hipStream_t st) {
  BwdParams P{units, w1, b1, wtT, dtl, q, ldq, dx, arg, demb, basic, dw1, db1, N, compat, {}, {}};
  P.L.U = U;
  int acc = 0;
  for (int t = 0; t < 6; ++t) {
    P.L.cnt[t] = counts[t];
    P.L.off[t] = acc;
    P.rowbase[t] = (long long)acc * N;
    acc += counts[t];
  }
  if (acc != U || U > 64) return hipErrorInvalidValue;
  encoder_bwd_kernel<<<(N + kRows - 1) / kRows, 256, 0, st>>>(P);
  return hipGetLastError();
}
