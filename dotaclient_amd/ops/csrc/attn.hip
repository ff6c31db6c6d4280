// Entity-attention block of the 5v5 policy (gfx950): pre-LN multi-head self-attention over the unit axis of every
// timestep row, then max-pool per unit type. PyTorch module: models/policy.py EntityAttention (BASELINE config 4);
// the 1v1 reference has no attention (policy.py:97-138), the pooling is the reference's K-maxpool.
//
//   E0  = W_τ·basic + b_τ                       (encoder_fwd; the kernel adds b_τ + b_out, see ln_fwd)
//   Xn  = LN(E0)·γ + β                          ln_fwd_kernel   (16 lanes per unit row, stats saved)
//   QKV = Xn·W_qkvᵀ + b_qkv                     hipBLASLt (bias epilogue)
//   O   = softmax(Q Kᵀ/√d) V   per (row, head)  attn_fwd_kernel (one wave per (row, head): 64×64 scores in
//                                               registers, MFMA 16x16x32, P through LDS, log-sum-exp saved)
//   E1  = E0 + O·W_outᵀ + b_out                 hipBLASLt (residual via beta = 1 on E0 + b_out)
//   pools, argmax per type of E1                pool_kernel
// Backward: demb_kernel (∂E1 = dtl⊗q + ∂pool routed to the argmax unit), attn_bwd_kernel (recomputes P from the
// saved log-sum-exp; dQ, dK, dV), ln_bwd_kernel (∂E0 = ∂E1 + LN'ᵀ∂Xn; ∂γ, ∂β and the per-type ∂b_τ as per-block
// partials), colsum_kernel (fixed-order partial sums: deterministic). The weight-gradient GEMMs over the N·U
// unit rows run on gemm_tn (split-K) with their bias column sums.
//
// MFMA operand images live in per-wave LDS; fragments that need a column of an image come from
// ds_read_b64_tr_b16 transposed reads (cdna_hip_programming.md T10), the others from 16-B row reads.
#include "common.h"

namespace {

using dca::bf16x8;
using dca::f32x4;
typedef short bf16x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4v lds_v4;

constexpr int kU = 64;        // unit slots per row (5v5 layout)
constexpr int kD = 128;       // embedding width
constexpr int kHd = 32;       // head width (4 heads)
constexpr int kP32 = 40;      // LDS pitch (bf16) of a 64×32 image
constexpr int kP64 = 72;      // LDS pitch (bf16) of a 64×64 image

// A[m][k] (m = m0 + lane&15, k = k0 + 8·(lane>>4) … +7) from an image stored [m][k]: one 16-B read
__device__ __forceinline__ bf16x8 frag_row(const short* img, int pitch, int m0, int k0) {
  const int l = threadIdx.x & 63;
  return *reinterpret_cast<const bf16x8*>(img + (m0 + (l & 15)) * pitch + k0 + 8 * (l >> 4));
}

// Fragment whose lane index runs along the image's COLUMNS: element jj of lane l = img[k0 + 8(l>>4) + jj][c0 + (l&15)]
// (two transposed reads: rows k0 + 8g + q and +4, columns c0 + 4p … 4p+3 supplied by lane 4q+p of each group)
__device__ __forceinline__ bf16x8 frag_tr(const short* img, int pitch, int k0, int c0) {
  const int l = threadIdx.x & 63, g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const short* a = img + (k0 + 8 * g + q) * pitch + c0 + 4 * p;
  const bf16x4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)a);
  const bf16x4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a + 4 * pitch));
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

// same fragment as frag_row, straight from global memory (row stride `stride` elements)
__device__ __forceinline__ bf16x8 frag_row_g(const short* __restrict__ src, int stride, int m0, int k0) {
  const int l = threadIdx.x & 63;
  return *reinterpret_cast<const bf16x8*>(src + (size_t)(m0 + (l & 15)) * stride + k0 + 8 * (l >> 4));
}

__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// stage a 64×32 head slice (row stride `stride` elements) into an LDS image [64][kP32]
__device__ __forceinline__ void stage64x32(short* img, const short* __restrict__ src, int stride) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = l + 64 * it, u = idx >> 2, c = idx & 3;
    *reinterpret_cast<bf16x8*>(img + u * kP32 + 8 * c) =
        *reinterpret_cast<const bf16x8*>(src + (size_t)u * stride + 8 * c);
  }
}

// element access for the kernels templated on the activation type (bf16 learner: short, fp32 learner: float)
__device__ __forceinline__ float ldf(short v) { return dca::bf2f(v); }
__device__ __forceinline__ float ldf(float v) { return v; }
__device__ __forceinline__ void stf(short* p, float v) { *p = dca::f2bf(v); }
__device__ __forceinline__ void stf(float* p, float v) { *p = v; }
__device__ __forceinline__ void ld8(const short* p, float* x) {
  const bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = dca::bf2f(v[j]);
}
__device__ __forceinline__ void ld8(const float* p, float* x) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
}
__device__ __forceinline__ void st8(short* p, const float* x) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = dca::f2bf(x[j]);
  *reinterpret_cast<bf16x8*>(p) = o;
}
__device__ __forceinline__ void st8(float* p, const float* x) {
  *reinterpret_cast<float4*>(p) = make_float4(x[0], x[1], x[2], x[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(x[4], x[5], x[6], x[7]);
}

// ============================================================================================================
// LayerNorm forward: x = E0' − b_sub (bf16 learner: E0' carries b_out, folded into the encoder's type bias; fp32
// learner: b_sub = null), 16 lanes × 8 columns.
template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ e0, const float* __restrict__ bsub,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     T* __restrict__ xn, float* __restrict__ mean,
                                                     float* __restrict__ rstd, int R, float eps,
                                                     T* __restrict__ e0_copy) {
  const int row = blockIdx.x * 16 + (threadIdx.x >> 4), c0 = (threadIdx.x & 15) * 8;
  if (row >= R) return;
  float x[8], s = 0.f;
  ld8(e0 + (size_t)row * kD + c0, x);
  if (e0_copy) st8(e0_copy + (size_t)row * kD + c0, x);   // optional copy of the input (saved for the backward)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (bsub) x[j] -= bsub[c0 + j];
    s += x[j];
  }
  s = dca::group_sum<16>(s);
  const float mu = s * (1.f / kD);
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    x[j] -= mu;
    q += x[j] * x[j];
  }
  q = dca::group_sum<16>(q);
  const float rs = rsqrtf(q * (1.f / kD) + eps);
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = x[j] * rs * gamma[c0 + j] + beta[c0 + j];
  st8(xn + (size_t)row * kD + c0, x);
  if ((threadIdx.x & 15) == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// ============================================================================================================
// Attention forward, one wave per (row n, head h) (blockIdx.x = n·4 + h). qkv (N·64, 384) bf16 = [q | k | v],
// each 4 heads × 32. Writes o (N·64, 128) bf16 and lse (N, 4, 64) f32 (natural-log, scaled scores).
__global__ __launch_bounds__(64) void attn_fwd_kernel(const short* __restrict__ qkv, short* __restrict__ o,
                                                      float* __restrict__ lse, float scale) {
  // Q and K fragments are row reads straight from global memory; only V (read by columns) and Pᵀ go through LDS
  // (14 KB per wave → ≈11 waves per CU instead of 6)
  __shared__ __attribute__((aligned(16))) short Vs[kU * kP32];
  __shared__ __attribute__((aligned(16))) short PT[kU * kP64];   // P transposed: [key j][query i]
  const int n = blockIdx.x >> 2, h = blockIdx.x & 3;
  const int l = threadIdx.x, kg = l >> 4, li = l & 15;
  const short* base = qkv + (size_t)n * kU * 384 + h * kHd;
  bf16x8 qa[4], kb[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) qa[a] = frag_row_g(base, 384, 16 * a, 0);
#pragma unroll
  for (int b = 0; b < 4; ++b) kb[b] = frag_row_g(base + 128, 384, 16 * b, 0);
  stage64x32(Vs, base + 256, 384);
  // S = Q Kᵀ: tile (a, b) = queries 16a…, keys 16b…; lane holds rows 16a + 4kg + r, column 16b + li
  f32x4 s[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) s[a][b] = mfma(qa[a], kb[b], f32x4{0.f, 0.f, 0.f, 0.f});
  // row softmax over the 64 keys (4 tiles × 16 lanes)
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float m = fmaxf(fmaxf(s[a][0][r], s[a][1][r]), fmaxf(s[a][2][r], s[a][3][r]));
      m = dca::group_max<16>(m) * scale;
      float e[4], sum = 0.f;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        e[b] = __expf(s[a][b][r] * scale - m);
        sum += e[b];
      }
      sum = dca::group_sum<16>(sum);
      const float inv = 1.f / sum;
#pragma unroll
      for (int b = 0; b < 4; ++b) s[a][b][r] = e[b] * inv;
      if (li == 0) lse[((size_t)n * 4 + h) * kU + 16 * a + 4 * kg + r] = m + __logf(sum);
    }
  // P → PT[j][i]: the lane's 4 consecutive queries of one key are one 8-byte write
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      bf16x4v v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = dca::f2bf(s[a][b][r]);
      *reinterpret_cast<bf16x4v*>(PT + (16 * b + li) * kP64 + 16 * a + 4 * kg) = v;
    }
  __syncthreads();
  // O = P V: A[i][k=j] = PT[j][i] (transposed read), B[k=j][n=d] = V[j][d] (transposed read)
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) acc = mfma(frag_tr(PT, kP64, 32 * ks, 16 * a), frag_tr(Vs, kP32, 32 * ks, 16 * c), acc);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        o[((size_t)n * kU + 16 * a + 4 * kg + r) * kD + h * kHd + 16 * c + li] = dca::f2bf(acc[r]);
    }
}

// ============================================================================================================
// Attention backward, one wave per (row, head). do_ (N·64, 128) bf16 = ∂O; writes dqkv (N·64, 384) bf16.
__global__ __launch_bounds__(64) void attn_bwd_kernel(const short* __restrict__ qkv, const short* __restrict__ o,
                                                      const short* __restrict__ do_, const float* __restrict__ lse,
                                                      short* __restrict__ dqkv, float scale) {
  // V is only read by rows (from global); Q, K and ∂O are also read by columns (transposed reads) → LDS
  __shared__ __attribute__((aligned(16))) short Qs[kU * kP32], Ks[kU * kP32], Ds[kU * kP32];
  __shared__ __attribute__((aligned(16))) short PT[kU * kP64], ST[kU * kP64];   // Pᵀ and (scale·dS)ᵀ, [j][i]
  __shared__ float Dl[kU], Ll[kU];
  const int n = blockIdx.x >> 2, h = blockIdx.x & 3;
  const int l = threadIdx.x, kg = l >> 4, li = l & 15;
  const short* base = qkv + (size_t)n * kU * 384 + h * kHd;
  stage64x32(Qs, base, 384);
  stage64x32(Ks, base + 128, 384);
  stage64x32(Ds, do_ + (size_t)n * kU * kD + h * kHd, kD);
  {  // D_i = Σ_d ∂O[i][d]·O[i][d] (lane = query i), LSE
    const short* orow = o + ((size_t)n * kU + l) * kD + h * kHd;
    const short* drow = do_ + ((size_t)n * kU + l) * kD + h * kHd;
    float d = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bf16x8 ov = *reinterpret_cast<const bf16x8*>(orow + 8 * c);
      const bf16x8 dv = *reinterpret_cast<const bf16x8*>(drow + 8 * c);
#pragma unroll
      for (int j = 0; j < 8; ++j) d += dca::bf2f(ov[j]) * dca::bf2f(dv[j]);
    }
    Dl[l] = d;
    Ll[l] = lse[((size_t)n * 4 + h) * kU + l];
  }
  __syncthreads();
  f32x4 p[4][4], dp[4][4];
  {
    bf16x8 qa[4], kb[4], da[4], vb[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      qa[a] = frag_row(Qs, kP32, 16 * a, 0);
      da[a] = frag_row(Ds, kP32, 16 * a, 0);
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      kb[b] = frag_row(Ks, kP32, 16 * b, 0);
      vb[b] = frag_row_g(base + 256, 384, 16 * b, 0);
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        p[a][b] = mfma(qa[a], kb[b], f32x4{0.f, 0.f, 0.f, 0.f});
        dp[a][b] = mfma(da[a], vb[b], f32x4{0.f, 0.f, 0.f, 0.f});
      }
  }
  // P = exp(scale·S − LSE); scale·dS = scale·P∘(dP − D); both stored transposed
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      bf16x4v pv, sv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * a + 4 * kg + r;
        const float pr = __expf(p[a][b][r] * scale - Ll[i]);
        pv[r] = dca::f2bf(pr);
        sv[r] = dca::f2bf(scale * pr * (dp[a][b][r] - Dl[i]));
      }
      *reinterpret_cast<bf16x4v*>(PT + (16 * b + li) * kP64 + 16 * a + 4 * kg) = pv;
      *reinterpret_cast<bf16x4v*>(ST + (16 * b + li) * kP64 + 16 * a + 4 * kg) = sv;
    }
  __syncthreads();
  short* out = dqkv + (size_t)n * kU * 384 + h * kHd;
  // dV = Pᵀ ∂O and dK = dSᵀ Q: C[j][d]; A[j][k=i] row reads of PT / ST, B[k=i][n=d] transposed reads of ∂O / Q
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 av = {0.f, 0.f, 0.f, 0.f}, ak = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        av = mfma(frag_row(PT, kP64, 16 * b, 32 * ks), frag_tr(Ds, kP32, 32 * ks, 16 * c), av);
        ak = mfma(frag_row(ST, kP64, 16 * b, 32 * ks), frag_tr(Qs, kP32, 32 * ks, 16 * c), ak);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const size_t j = 16 * b + 4 * kg + r;
        out[j * 384 + 256 + 16 * c + li] = dca::f2bf(av[r]);
        out[j * 384 + 128 + 16 * c + li] = dca::f2bf(ak[r]);
      }
    }
  // dQ = dS K: C[i][d]; A[i][k=j] = STᵀ (transposed read), B[k=j][n=d] = K (transposed read)
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 aq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) aq = mfma(frag_tr(ST, kP64, 32 * ks, 16 * a), frag_tr(Ks, kP32, 32 * ks, 16 * c), aq);
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(size_t)(16 * a + 4 * kg + r) * 384 + 16 * c + li] = dca::f2bf(aq[r]);
    }
}

// ============================================================================================================
// Max-pool + argmax per unit type over the attended embeddings E1 (N·64, 128) bf16 → x896[:, 128 + 128τ + c] and
// arg (N, 6, 128) u8 (first maximum, like the fused 1v1 encoder). compat: the enemy-tower pool reuses the
// enemy-nonhero pool (reference policy.py:127). One block of 128 threads (= columns) per row.
struct TypeOff {
  int off[7];
};

template <typename E>
__global__ __launch_bounds__(128) void pool_kernel(const E* __restrict__ e1, TypeOff T, E* __restrict__ x896,
                                                   unsigned char* __restrict__ arg, int compat) {
  const int n = blockIdx.x, c = threadIdx.x;
  const E* rowp = e1 + (size_t)n * kU * kD + c;
#pragma unroll
  for (int t = 0; t < 6; ++t) {
    const int src = (compat && t == 5) ? 3 : t;
    float m = -INFINITY;
    int am = 0;
    for (int u = T.off[src]; u < T.off[src + 1]; ++u) {
      const float v = ldf(rowp[(size_t)u * kD]);
      if (v > m) {
        m = v;
        am = u - T.off[src];
      }
    }
    stf(x896 + (size_t)n * 896 + kD + t * kD + c, m);
    arg[((size_t)n * 6 + t) * kD + c] = (unsigned char)am;
  }
}

// ∂E1[n,u,c] = dtl[n,u]·q[n,c] + Σ_τ [u = off_τ + arg[n,τ,c]]·∂pool_τ[n,c] (compat: the eth pool's gradient goes to
// the enh argmax). One block of 128 threads per row; the row's 64 dtl values via LDS.
template <typename E>
__global__ __launch_bounds__(128) void demb_kernel(const float* __restrict__ dtl, const float* __restrict__ q, int ldq,
                                                   const float* __restrict__ dx, const unsigned char* __restrict__ arg,
                                                   TypeOff T, E* __restrict__ de1, int compat) {
  const int n = blockIdx.x, c = threadIdx.x;
  __shared__ float sd[kU];
  if (c < kU) sd[c] = dtl[(size_t)n * kU + c];
  __syncthreads();
  const float qc = q[(size_t)n * ldq + c];
  int au[6];
  float dp[6];
#pragma unroll
  for (int t = 0; t < 6; ++t) {
    const int src = (compat && t == 5) ? 3 : t;
    au[t] = T.off[src] + arg[((size_t)n * 6 + t) * kD + c];
    dp[t] = dx[(size_t)n * 896 + kD + t * kD + c];
  }
  E* out = de1 + (size_t)n * kU * kD + c;
  for (int u = 0; u < kU; ++u) {
    float v = sd[u] * qc;
#pragma unroll
    for (int t = 0; t < 6; ++t) v += (au[t] == u) ? dp[t] : 0.f;
    stf(out + (size_t)u * kD, v);
  }
}

// ============================================================================================================
// LayerNorm backward + residual: ∂E0 = ∂E1 + rstd·(g − mean(g) − x̂·mean(g∘x̂)), g = ∂Xn∘γ. Per-block partials
// [∂γ (128) | ∂β (128) | ∂b_τ (6×128)]; the type of unit row r is type_of[r % 64]. 16 lanes × 8 columns per row,
// 16 rows per pass, grid-stride over the rows.
constexpr int kLnPart = 2 * kD + 6 * kD;

template <typename E>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const E* __restrict__ dxn, const E* __restrict__ e0,
                                                     const float* __restrict__ bsub, const float* __restrict__ gamma,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const E* __restrict__ de1, const unsigned char* type_of,
                                                     E* __restrict__ de0, float* __restrict__ part, int R) {
  const int lr = threadIdx.x >> 4, c0 = (threadIdx.x & 15) * 8;
  float gacc[8], bacc[8], tacc[6][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    gacc[j] = bacc[j] = 0.f;
#pragma unroll
    for (int t = 0; t < 6; ++t) tacc[t][j] = 0.f;
  }
  float gm[8], bs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    gm[j] = gamma[c0 + j];
    bs[j] = bsub ? bsub[c0 + j] : 0.f;
  }
  for (int row = blockIdx.x * 16 + lr; row < R; row += gridDim.x * 16) {
    float dv[8], ev[8], rv[8];
    ld8(dxn + (size_t)row * kD + c0, dv);
    ld8(e0 + (size_t)row * kD + c0, ev);
    ld8(de1 + (size_t)row * kD + c0, rv);
    const float mu = mean[row], rs = rstd[row];
    float xh[8], g[8], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      xh[j] = (ev[j] - bs[j] - mu) * rs;
      const float d = dv[j];
      g[j] = d * gm[j];
      s1 += g[j];
      s2 += g[j] * xh[j];
      gacc[j] += d * xh[j];
      bacc[j] += d;
    }
    s1 = dca::group_sum<16>(s1) * (1.f / kD);
    s2 = dca::group_sum<16>(s2) * (1.f / kD);
    const int t = type_of[row % kU];
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = rv[j] + rs * (g[j] - s1 - xh[j] * s2);
      o[j] = v;
#pragma unroll
      for (int tt = 0; tt < 6; ++tt) tacc[tt][j] += (tt == t) ? v : 0.f;
    }
    st8(de0 + (size_t)row * kD + c0, o);
  }
  // fixed-order block reduction over the 16 row lanes → one partial per block
  __shared__ float red[16][kLnPart];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[lr][c0 + j] = gacc[j];
    red[lr][kD + c0 + j] = bacc[j];
#pragma unroll
    for (int t = 0; t < 6; ++t) red[lr][2 * kD + t * kD + c0 + j] = tacc[t][j];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kLnPart; e += 256) {
    float v = 0.f;
    for (int k = 0; k < 16; ++k) v += red[k][e];
    part[(size_t)blockIdx.x * kLnPart + e] = v;
  }
}

// out[c] = Σ_b part[b][c] in block order (deterministic); 64 columns × 4 row phases per block.
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ part, int nblk, int W,
                                                     float* __restrict__ out) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), ph = threadIdx.x >> 6;
  float s = 0.f;
  if (c < W) {
    int b = ph;
    for (; b + 12 < nblk; b += 16) {
      const float v0 = part[(size_t)b * W + c], v1 = part[(size_t)(b + 4) * W + c];
      const float v2 = part[(size_t)(b + 8) * W + c], v3 = part[(size_t)(b + 12) * W + c];
      s += v0;
      s += v1;
      s += v2;
      s += v3;
    }
    for (; b < nblk; b += 4) s += part[(size_t)b * W + c];
  }
  __shared__ float red[4][64];
  red[ph][threadIdx.x & 63] = s;
  __syncthreads();
  if (ph == 0 && c < W) out[c] = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

// ============================================================================================================
// fp32 (reference-precision) attention core for the fp32 learner: same math as attn_fwd/bwd_kernel over fp32
// qkv / o / ∂O, every product a bf16x3 split MFMA (x = hi + lo, hi·hi + hi·lo + lo·hi, fp32 accumulation; ≈2⁻¹⁶
// relative per product), softmax and LSE in fp32. Replaces the explicit torch ops whose (N, 4, 64, 64) fp32
// probability tensor (0.73 GB at N = 11 200) was written once and re-read three times per step.
//
// Register-resident layout (no LDS in the forward): Sᵀ = K·Qᵀ comes out of the 16x16x32 MFMA with lane
// (j = 16b + 4kg + r, i = 16a + li), which is EXACTLY the A-operand layout of a 16x16x16 MFMA contracting over j
// (A[m = i][k = j]: m = lane&15, k = 4(lane>>4) + r) — so O = P·V takes P straight from the score registers. The
// backward keeps the i-major S = Q·Kᵀ layout instead (lane (i = 16a + 4kg + r, j = 16b + li) = A[m = j][k = i]) for
// ∂V = Pᵀ∂O and ∂K = ∂Sᵀ Q, and passes ∂S through LDS (hi / lo images, transposed reads) only for ∂Q = ∂S K.
// Measured and not kept: a backward processed per 16-key block that recomputes S and dP in both layouts (no LDS,
// ∂Q accumulated from the j-major tiles) to reach two waves per SIMD — 1392 vs 890 µs at 11 200 rows: the doubled
// MFMA/exp work and 25 spilled registers cost more than the occupancy gains. Nor a backward over two query halves
// of 32 (∂V / ∂K accumulated across the halves, nothing recomputed) bounded to two waves per SIMD (256 registers,
// 8 spilled): 949 vs 868 µs — the re-read operand rows and the spills outweigh the second wave.
__device__ __forceinline__ void split8(const float* __restrict__ p, bf16x8& hi, bf16x8& lo,
                                       const float* bias8 = nullptr) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  if (bias8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += bias8[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hi[j] = dca::f2bf(v[j]);
    lo[j] = dca::f2bf(v[j] - dca::bf2f(hi[j]));
  }
}
__device__ __forceinline__ void split4(const float v0, const float v1, const float v2, const float v3, bf16x4v& hi,
                                       bf16x4v& lo) {
  const float v[4] = {v0, v1, v2, v3};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    hi[j] = dca::f2bf(v[j]);
    lo[j] = dca::f2bf(v[j] - dca::bf2f(hi[j]));
  }
}
// bf16x3 products: 16x16x32 (A, B = 8-element fragments) and 16x16x16 (4-element fragments)
__device__ __forceinline__ f32x4 mfma3(const bf16x8& ah, const bf16x8& al, const bf16x8& bh, const bf16x8& bl,
                                       f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma3k16(const bf16x4v& ah, const bf16x4v& al, const bf16x4v& bh,
                                          const bf16x4v& bl, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bl, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bh, c, 0, 0, 0);
}

// Forward, one wave per (row n, head h) = blockIdx.x · 4 + h. qkv (N·64, 384) f32 → o (N·64, 128) f32, lse (N,4,64).
__global__ __launch_bounds__(64) void attn_fwd_f32_kernel(const float* __restrict__ qkv, const float* __restrict__ bq,
                                                          float* __restrict__ o, float* __restrict__ lse, float scale) {
  const int n = blockIdx.x >> 2, h = blockIdx.x & 3;
  const int l = threadIdx.x, kg = l >> 4, li = l & 15;
  const float* base = qkv + (size_t)n * kU * 384 + h * kHd;
  // QKV projection bias (384, added here: hipBLASLt's bias-epilogue GEMM is 1.7x slower than the plain one)
  float qb[8], kb8[8], vb[2];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    qb[j] = bq[h * kHd + 8 * kg + j];
    kb8[j] = bq[128 + h * kHd + 8 * kg + j];
  }
  vb[0] = bq[256 + h * kHd + li];
  vb[1] = bq[256 + h * kHd + 16 + li];
  // V operand of O = P·V (B[k = j][n = d]): lane needs V[16b + 4kg + r][16c + li] — issued first, used last
  float vr[4][2][4];
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) vr[b][c][r] = base[(size_t)(16 * b + 4 * kg + r) * 384 + 256 + 16 * c + li] + vb[c];
  bf16x8 qh[4], ql[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) split8(base + (size_t)(16 * a + li) * 384 + 8 * kg, qh[a], ql[a], qb);
  // Sᵀ tiles: s[b][a] lane (key j = 16b + 4kg + r, query i = 16a + li)
  f32x4 s[4][4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    bf16x8 kh, kl;
    split8(base + 128 + (size_t)(16 * b + li) * 384 + 8 * kg, kh, kl, kb8);
#pragma unroll
    for (int a = 0; a < 4; ++a) s[b][a] = mfma3(kh, kl, qh[a], ql[a], f32x4{0.f, 0.f, 0.f, 0.f});
  }
  // softmax over the keys of query i = 16a + li: in-lane over (b, r), then across the 4 lane groups (xor 16, 32)
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    float m = -INFINITY;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) m = fmaxf(m, s[b][a][r]);
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    m *= scale;
    float sum = 0.f;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = __expf(s[b][a][r] * scale - m);
        s[b][a][r] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float inv = 1.f / sum;
#pragma unroll
    for (int b = 0; b < 4; ++b) s[b][a] *= inv;
    if (kg == 0) lse[((size_t)n * 4 + h) * kU + 16 * a + li] = m + __logf(sum);
  }
  // O = P·V on 16x16x16: A[m = i][k = j] = s[b][a] as is, B[k = j][n = d] = vr[b][c]
  bf16x4v vh[4][2], vl[4][2];
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int c = 0; c < 2; ++c) split4(vr[b][c][0], vr[b][c][1], vr[b][c][2], vr[b][c][3], vh[b][c], vl[b][c]);
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    bf16x4v ph[4], pl[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) split4(s[b][a][0], s[b][a][1], s[b][a][2], s[b][a][3], ph[b], pl[b]);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int b = 0; b < 4; ++b) acc = mfma3k16(ph[b], pl[b], vh[b][c], vl[b][c], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) o[((size_t)n * kU + 16 * a + 4 * kg + r) * kD + h * kHd + 16 * c + li] = acc[r];
    }
  }
}

// Backward, one wave per (row, head). do_ (N·64, 128) f32 = ∂O; writes dqkv (N·64, 384) f32.
__global__ __launch_bounds__(64) void attn_bwd_f32_kernel(const float* __restrict__ qkv, const float* __restrict__ bq,
                                                          const float* __restrict__ o,
                                                          const float* __restrict__ do_, const float* __restrict__ lse,
                                                          float* __restrict__ dqkv, float scale) {
  __shared__ __attribute__((aligned(16))) short STh[kU * kP64], STl[kU * kP64];   // (scale·∂S)ᵀ hi / lo, [j][i]
  __shared__ float Dl[kU], Ll[kU];
  const int n = blockIdx.x >> 2, h = blockIdx.x & 3;
  const int l = threadIdx.x, kg = l >> 4, li = l & 15;
  const float* base = qkv + (size_t)n * kU * 384 + h * kHd;
  const float* dob = do_ + (size_t)n * kU * kD + h * kHd;
  const float* ob = o + (size_t)n * kU * kD + h * kHd;
  float qb[8], kb8[8], vb8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    qb[j] = bq[h * kHd + 8 * kg + j];
    kb8[j] = bq[128 + h * kHd + 8 * kg + j];
    vb8[j] = bq[256 + h * kHd + 8 * kg + j];
  }
  // D_i = Σ_d ∂O[i][d]·O[i][d] for i = 16a + li (lane group kg sums d = 8kg … 8kg + 7), LSE
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const float* orow = ob + (size_t)(16 * a + li) * kD + 8 * kg;
    const float* drow = dob + (size_t)(16 * a + li) * kD + 8 * kg;
    const float4 o0 = *reinterpret_cast<const float4*>(orow), o1 = *reinterpret_cast<const float4*>(orow + 4);
    const float4 d0 = *reinterpret_cast<const float4*>(drow), d1 = *reinterpret_cast<const float4*>(drow + 4);
    float d = o0.x * d0.x + o0.y * d0.y + o0.z * d0.z + o0.w * d0.w + o1.x * d1.x + o1.y * d1.y + o1.z * d1.z +
              o1.w * d1.w;
    d += __shfl_xor(d, 16, 64);
    d += __shfl_xor(d, 32, 64);
    if (kg == 0) Dl[16 * a + li] = d;
  }
  Ll[l] = lse[((size_t)n * 4 + h) * kU + l];
  // S = Q Kᵀ and dP = ∂O Vᵀ, i-major: p[a][b] lane (query i = 16a + 4kg + r, key j = 16b + li)
  f32x4 p[4][4], dp[4][4];
  {
    bf16x8 qh[4], ql[4], dh[4], dl[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      split8(base + (size_t)(16 * a + li) * 384 + 8 * kg, qh[a], ql[a], qb);
      split8(dob + (size_t)(16 * a + li) * kD + 8 * kg, dh[a], dl[a]);
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      bf16x8 kh, kl, vh, vl;
      split8(base + 128 + (size_t)(16 * b + li) * 384 + 8 * kg, kh, kl, kb8);
      split8(base + 256 + (size_t)(16 * b + li) * 384 + 8 * kg, vh, vl, vb8);
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        p[a][b] = mfma3(qh[a], ql[a], kh, kl, f32x4{0.f, 0.f, 0.f, 0.f});
        dp[a][b] = mfma3(dh[a], dl[a], vh, vl, f32x4{0.f, 0.f, 0.f, 0.f});
      }
    }
  }
  __syncthreads();
  // P = exp(scale·S − LSE); dp ← scale·P∘(dP − D) (= ∂L/∂S_raw); (scale·∂S)ᵀ hi/lo images for ∂Q
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * a + 4 * kg + r;
      const float L = Ll[i], D = Dl[i];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float pr = __expf(p[a][b][r] * scale - L);
        p[a][b][r] = pr;
        dp[a][b][r] = scale * pr * (dp[a][b][r] - D);
      }
    }
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      bf16x4v sh, sl;
      split4(dp[a][b][0], dp[a][b][1], dp[a][b][2], dp[a][b][3], sh, sl);
      *reinterpret_cast<bf16x4v*>(STh + (16 * b + li) * kP64 + 16 * a + 4 * kg) = sh;
      *reinterpret_cast<bf16x4v*>(STl + (16 * b + li) * kP64 + 16 * a + 4 * kg) = sl;
    }
  float* out = dqkv + (size_t)n * kU * 384 + h * kHd;
  // ∂V = Pᵀ∂O and ∂K = ∂Sᵀ Q on 16x16x16: A[m = j][k = i] = p / dp registers (k-chunk a), B[k = i][n = d] = rows
  // 16a + 4kg + r of ∂O / Q at column 16c + li
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const float qbc = bq[h * kHd + 16 * c + li];
    bf16x4v doh[4], dol[4], qh[4], ql[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      float dv[4], qv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dv[r] = dob[(size_t)(16 * a + 4 * kg + r) * kD + 16 * c + li];
        qv[r] = base[(size_t)(16 * a + 4 * kg + r) * 384 + 16 * c + li] + qbc;
      }
      split4(dv[0], dv[1], dv[2], dv[3], doh[a], dol[a]);
      split4(qv[0], qv[1], qv[2], qv[3], qh[a], ql[a]);
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      f32x4 av = {0.f, 0.f, 0.f, 0.f}, ak = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        bf16x4v ph, pl, sh, sl;
        split4(p[a][b][0], p[a][b][1], p[a][b][2], p[a][b][3], ph, pl);
        split4(dp[a][b][0], dp[a][b][1], dp[a][b][2], dp[a][b][3], sh, sl);
        av = mfma3k16(ph, pl, doh[a], dol[a], av);
        ak = mfma3k16(sh, sl, qh[a], ql[a], ak);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const size_t j = 16 * b + 4 * kg + r;
        out[j * 384 + 256 + 16 * c + li] = av[r];
        out[j * 384 + 128 + 16 * c + li] = ak[r];
      }
    }
  }
  __syncthreads();
  // ∂Q = ∂S K on 16x16x32: A[m = i][k = j] = transposed reads of the ∂Sᵀ images, B[k = j][n = d] = K rows
  // 32ks + 8kg … +7 at column 16c + li
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const float kbc = bq[128 + h * kHd + 16 * c + li];
    bf16x8 kh[2], kl[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const float v = base[(size_t)(32 * ks + 8 * kg + jj) * 384 + 128 + 16 * c + li] + kbc;
        kh[ks][jj] = dca::f2bf(v);
        kl[ks][jj] = dca::f2bf(v - dca::bf2f(kh[ks][jj]));
      }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      f32x4 aq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        aq = mfma3(frag_tr(STh, kP64, 32 * ks, 16 * a), frag_tr(STl, kP64, 32 * ks, 16 * a), kh[ks], kl[ks], aq);
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(size_t)(16 * a + 4 * kg + r) * 384 + 16 * c + li] = aq[r];
    }
  }
}

}  // namespace

extern "C" hipError_t dca_attn_fwd_f32(const float* qkv, const float* bq, float* o, float* lse, int N, float scale,
                                       hipStream_t st) {
  hipLaunchKernelGGL(attn_fwd_f32_kernel, dim3(N * 4), dim3(64), 0, st, qkv, bq, o, lse, scale);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}

extern "C" hipError_t dca_attn_bwd_f32(const float* qkv, const float* bq, const float* o, const float* dout,
                                       const float* lse, float* dqkv, int N, float scale, hipStream_t st) {
  hipLaunchKernelGGL(attn_bwd_f32_kernel, dim3(N * 4), dim3(64), 0, st, qkv, bq, o, dout, lse, dqkv, scale);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}

extern "C" int dca_ln_part_width() { return kLnPart; }

extern "C" hipError_t dca_ln_fwd(const void* e0, const float* bsub, const float* gamma, const float* beta, void* xn,
                                 float* mean, float* rstd, int R, float eps, int f32, void* e0_copy, hipStream_t st) {
  if (f32)
    hipLaunchKernelGGL(ln_fwd_kernel<float>, dim3((R + 15) / 16), dim3(256), 0, st, (const float*)e0, bsub, gamma,
                       beta, (float*)xn, mean, rstd, R, eps, (float*)e0_copy);
  else
    hipLaunchKernelGGL(ln_fwd_kernel<short>, dim3((R + 15) / 16), dim3(256), 0, st, (const short*)e0, bsub, gamma,
                       beta, (short*)xn, mean, rstd, R, eps, (short*)e0_copy);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}

extern "C" hipError_t dca_attn_fwd(const short* qkv, short* o, float* lse, int N, float scale, hipStream_t st) {
  hipLaunchKernelGGL(attn_fwd_kernel, dim3(N * 4), dim3(64), 0, st, qkv, o, lse, scale);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}

extern "C" hipError_t dca_attn_bwd(const short* qkv, const short* o, const short* dout, const float* lse, short* dqkv,
                                   int N, float scale, hipStream_t st) {
  hipLaunchKernelGGL(attn_bwd_kernel, dim3(N * 4), dim3(64), 0, st, qkv, o, dout, lse, dqkv, scale);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}

extern "C" hipError_t dca_attn_pool(const void* e1, const int* type_off, void* x896, unsigned char* arg, int N,
                                    int compat, int f32, hipStream_t st) {
  TypeOff T;
  for (int i = 0; i < 7; ++i) T.off[i] = type_off[i];
  if (f32)
    hipLaunchKernelGGL(pool_kernel<float>, dim3(N), dim3(128), 0, st, (const float*)e1, T, (float*)x896, arg, compat);
  else
    hipLaunchKernelGGL(pool_kernel<short>, dim3(N), dim3(128), 0, st, (const short*)e1, T, (short*)x896, arg, compat);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}

extern "C" hipError_t dca_attn_demb(const float* dtl, const float* q, int ldq, const float* dx,
                                    const unsigned char* arg, const int* type_off, void* de1, int N, int compat,
                                    int f32, hipStream_t st) {
  TypeOff T;
  for (int i = 0; i < 7; ++i) T.off[i] = type_off[i];
  if (f32)
    hipLaunchKernelGGL(demb_kernel<float>, dim3(N), dim3(128), 0, st, dtl, q, ldq, dx, arg, T, (float*)de1, compat);
  else
    hipLaunchKernelGGL(demb_kernel<short>, dim3(N), dim3(128), 0, st, dtl, q, ldq, dx, arg, T, (short*)de1, compat);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}

extern "C" hipError_t dca_ln_bwd(const void* dxn, const void* e0, const float* bsub, const float* gamma,
                                 const float* mean, const float* rstd, const void* de1, const unsigned char* type_of,
                                 void* de0, float* part, int nblk, float* out, int R, int f32, hipStream_t st) {
  if (f32)
    hipLaunchKernelGGL(ln_bwd_kernel<float>, dim3(nblk), dim3(256), 0, st, (const float*)dxn, (const float*)e0, bsub,
                       gamma, mean, rstd, (const float*)de1, type_of, (float*)de0, part, R);
  else
    hipLaunchKernelGGL(ln_bwd_kernel<short>, dim3(nblk), dim3(256), 0, st, (const short*)dxn, (const short*)e0, bsub,
                       gamma, mean, rstd, (const short*)de1, type_of, (short*)de0, part, R);
  DCA_CHECK_LAUNCH();
  hipLaunchKernelGGL(colsum_kernel, dim3((kLnPart + 63) / 64), dim3(256), 0, st, part, nblk, kLnPart, out);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}
