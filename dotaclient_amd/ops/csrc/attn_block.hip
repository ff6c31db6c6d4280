// Fused fp32 entity-attention block forward of the 5v5 policy (gfx950, bf16x3 MFMA): ONE launch per step instead of
// LayerNorm + QKV GEMM + attention + out-projection GEMM + pool (attn.hip / hipBLASLt: 1.43 ms at N = 11 200 rows).
// PyTorch module: models/policy.py EntityAttention (BASELINE config 4; the reference's per-unit embed + max-pool,
// policy.py:100-138, extended by pre-LN self-attention over the unit axis).
//
// One 256-thread workgroup (4 waves) per timestep row n (64 unit slots × 128):
//   A  x = E0' − b_out, LayerNorm → Xn (fp32 to HBM for the backward; bf16 hi / lo LDS images), mean / rstd
//   B  wave h = head h: Qᵀ, Kᵀ (d × unit) = W_{q,k}[head rows]·Xnᵀ and V (unit × d) = Xn·W_vᵀ on 16x16x32 bf16x3
//      MFMAs. Computing Qᵀ / Kᵀ (not Q / K) puts them in the C layout lane (d = 16c + 4kg + r, unit = 16a + li),
//      which IS the 4-element operand layout of the 16x16x16 MFMA (m / n = lane&15, k = 4(lane>>4) + r): the
//      attention takes Q and K straight from the accumulators, no LDS transpose; V's C layout is the B operand of
//      P·V as it comes. QKV (without bias) leaves for the backward.
//   C  Sᵀ = K·Qᵀ (16x16x16), softmax over the keys in registers (log-sum-exp saved), O = P·V → HBM and to bf16
//      hi / lo LDS images
//   D  E1 = E0' + O·W_outᵀ (16x16x32, wave w: output columns 32w … 32w+31) → HBM (the heads' pointer keys) and LDS
//   E  max-pool + first argmax per unit type over E1 → x896[:, 128:896], arg (compat: enemy towers pool the enemy
//      non-heroes, reference policy.py:127)
// The per-step weights arrive as bf16 hi / lo images in MFMA fragment order (x = hi + lo, split once per step); products are
// hi·hi + lo·hi + hi·lo with fp32 accumulation (≈2⁻¹⁶ relative per product), softmax / LN / residual in fp32.
// Every workgroup re-reads W_qkv / W_out (256 KB of hi / lo fragments) from L2 for its row — ≈2.9 GB of L2 traffic per
// step, what bounds it (1.02 ms). Not kept: a weight-stationary persistent form (one workgroup per CU holding its
// W_qkv / W_out fragments in registers across rows) needs 256 resident registers per lane next to the QKV
// accumulators and spilled ≈450 registers at the 512-register (one wave per SIMD) budget; at two waves per SIMD the
// resident set cannot fit at all.
#include "common.h"
#include <cstdlib>

namespace {

using dca::bf16x8;
using dca::f32x4;
typedef short bf16x4v __attribute__((ext_vector_type(4)));

constexpr int kU = 64, kD = 128, kHd = 32;
constexpr int kPX = 136;            // bf16 pitch of the 64 × 128 LDS images (272 B rows)
constexpr int kPE = 132;            // fp32 pitch of the E1 image

struct BlockArgs {
  const float* e0;                  // (N·64, 128) E0' = E0 + b_out
  const float* bout; const float* gamma; const float* beta;
  const short* wqh; const short* wql; const float* bq;     // (384, 128) bf16 hi / lo, bias (384)
  const short* woh; const short* wol;                      // (128, 128)
  float* xn; float* mu; float* rs;                         // (N·64, 128), (N·64), (N·64)
  float* qkv; float* o; float* lse;                        // (N·64, 384) without bias, (N·64, 128), (N, 4, 64)
  float* e1;                                               // (N·64, 128)
  float* x896; unsigned char* arg;                         // (N, 896) [128:896], (N, 6, 128)
  int off[7];
  int compat;
  float scale, eps;
};

__device__ __forceinline__ void split8v(const float* v, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hi[j] = dca::f2bf(v[j]);
    lo[j] = dca::f2bf(v[j] - dca::bf2f(hi[j]));
  }
}
__device__ __forceinline__ void split4v(const f32x4 v, bf16x4v& hi, bf16x4v& lo) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    hi[j] = dca::f2bf(v[j]);
    lo[j] = dca::f2bf(v[j] - dca::bf2f(hi[j]));
  }
}
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
// 16x16x32 fragment (m / n = lane&15, k = 8·(lane>>4) … +7) of row m0 + lane&15 at column k0 of a row-major image
__device__ __forceinline__ bf16x8 frag(const short* img, int pitch, int m0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(img + (m0 + (lane & 15)) * pitch + k0 + 8 * (lane >> 4));
}
// weight fragment of rows m0 … m0+15, k-step k0/32 from a FRAGMENT-ORDERED image [row tile][k-step][lane][8] (one
// coalesced 1 KB load per wave; the row-major image cost 16 separate 64-B segments per load instruction)
__device__ __forceinline__ bf16x8 gfrag(const short* __restrict__ w, int m0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(w + ((size_t)((m0 >> 4) * (kD / 32) + (k0 >> 5)) * 64 + lane) * 8);
}

__global__ __launch_bounds__(256, 2) void attn_block_fwd_f32_kernel(BlockArgs P) {
  __shared__ __attribute__((aligned(16))) short img_h[kU * kPX], img_l[kU * kPX];   // Xn, then O (hi / lo)
  __shared__ __attribute__((aligned(16))) float e1s[kU * kPE];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, kg = lane >> 4, li = lane & 15;
  const int n = blockIdx.x;
  const size_t rbase = (size_t)n * kU;

  // ---- A: LayerNorm, 4 threads per unit row (32 columns each)
  {
    const int u = tid >> 2, p = tid & 3;
    const float* src = P.e0 + (rbase + u) * kD + 32 * p;
    float x[32];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float4 v = *reinterpret_cast<const float4*>(src + 4 * i);
      x[4 * i] = v.x - P.bout[32 * p + 4 * i];
      x[4 * i + 1] = v.y - P.bout[32 * p + 4 * i + 1];
      x[4 * i + 2] = v.z - P.bout[32 * p + 4 * i + 2];
      x[4 * i + 3] = v.w - P.bout[32 * p + 4 * i + 3];
    }
#pragma unroll
    for (int j = 0; j < 32; ++j) s += x[j];
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    const float mu = s * (1.f / kD);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      x[j] -= mu;
      q += x[j] * x[j];
    }
    q += __shfl_xor(q, 1, 64);
    q += __shfl_xor(q, 2, 64);
    const float rs = rsqrtf(q * (1.f / kD) + P.eps);
#pragma unroll
    for (int j = 0; j < 32; ++j) x[j] = x[j] * rs * P.gamma[32 * p + j] + P.beta[32 * p + j];
    float* dst = P.xn + (rbase + u) * kD + 32 * p;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      *reinterpret_cast<float4*>(dst + 4 * i) = make_float4(x[4 * i], x[4 * i + 1], x[4 * i + 2], x[4 * i + 3]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bf16x8 hi, lo;
      split8v(x + 8 * i, hi, lo);
      *reinterpret_cast<bf16x8*>(img_h + u * kPX + 32 * p + 8 * i) = hi;
      *reinterpret_cast<bf16x8*>(img_l + u * kPX + 32 * p + 8 * i) = lo;
    }
    if (p == 0) {
      P.mu[rbase + u] = mu;
      P.rs[rbase + u] = rs;
    }
  }
  __syncthreads();

  // ---- B: wave h = head h. qt / kt[c][a]: lane (d = 16c + 4kg + r, unit = 16a + li); v[b][c]: lane (unit =
  //      16b + 4kg + r, d = 16c + li)
  const int h = w;
  f32x4 qt[2][4], kt[2][4], vv[4][2];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      qt[c][a] = f32x4{0.f, 0.f, 0.f, 0.f};
      kt[c][a] = f32x4{0.f, 0.f, 0.f, 0.f};
      vv[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    bf16x8 xh[4], xl[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      xh[a] = frag(img_h, kPX, 16 * a, 32 * ks, lane);
      xl[a] = frag(img_l, kPX, 16 * a, 32 * ks, lane);
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int rq = kHd * h + 16 * c;
      const bf16x8 qwh = gfrag(P.wqh, rq, 32 * ks, lane), qwl = gfrag(P.wql, rq, 32 * ks, lane);
      const bf16x8 kwh = gfrag(P.wqh, 128 + rq, 32 * ks, lane), kwl = gfrag(P.wql, 128 + rq, 32 * ks, lane);
      const bf16x8 vwh = gfrag(P.wqh, 256 + rq, 32 * ks, lane), vwl = gfrag(P.wql, 256 + rq, 32 * ks, lane);
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        qt[c][a] = mfma3(qwh, qwl, xh[a], xl[a], qt[c][a]);    // m = d (weight row), n = unit
        kt[c][a] = mfma3(kwh, kwl, xh[a], xl[a], kt[c][a]);
        vv[a][c] = mfma3(xh[a], xl[a], vwh, vwl, vv[a][c]);    // m = unit, n = d
      }
    }
  }
  // QKV → HBM (no bias): Qᵀ / Kᵀ lanes hold 4 consecutive d of one unit (one 16-B store), V one element
  {
    float* qb = P.qkv + rbase * 384;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int u = 16 * a + li, d = kHd * h + 16 * c + 4 * kg;
        *reinterpret_cast<f32x4*>(qb + (size_t)u * 384 + d) = qt[c][a];
        *reinterpret_cast<f32x4*>(qb + (size_t)u * 384 + 128 + d) = kt[c][a];
#pragma unroll
        for (int r = 0; r < 4; ++r) qb[(size_t)(16 * a + 4 * kg + r) * 384 + 256 + kHd * h + 16 * c + li] = vv[a][c][r];
      }
  }
  __syncthreads();                                        // every wave is done with the Xn images

  // ---- C: attention of head h. Biases first (q / k: per (c, r) row of the lane, v: per column li)
  {
    bf16x4v qh[2][4], ql[2][4], khv[2][4], klv[2][4];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 bqv, bkv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bqv[r] = P.bq[kHd * h + 16 * c + 4 * kg + r];
        bkv[r] = P.bq[128 + kHd * h + 16 * c + 4 * kg + r];
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        split4v(qt[c][a] + bqv, qh[c][a], ql[c][a]);
        split4v(kt[c][a] + bkv, khv[c][a], klv[c][a]);
      }
    }
    // Sᵀ[b][a]: lane (key j = 16b + 4kg + r, query i = 16a + li)
    f32x4 s[4][4];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 2; ++c) acc = mfma3k16(khv[c][b], klv[c][b], qh[c][a], ql[c][a], acc);
        s[b][a] = acc;
      }
    float* lse = P.lse + ((size_t)n * 4 + h) * kU;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      float m = -INFINITY;
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) m = fmaxf(m, s[b][a][r]);
      m = fmaxf(m, __shfl_xor(m, 16, 64));
      m = fmaxf(m, __shfl_xor(m, 32, 64));
      m *= P.scale;
      float sum = 0.f;
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __expf(s[b][a][r] * P.scale - m);
          s[b][a][r] = e;
          sum += e;
        }
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      const float inv = 1.f / sum;
#pragma unroll
      for (int b = 0; b < 4; ++b) s[b][a] *= inv;
      if (kg == 0) lse[16 * a + li] = m + __logf(sum);
    }
    // O = P·V: A[m = i][k = j] = s[b][a], B[k = j][n = d] = v[b][c] (+ bias of column d)
    bf16x4v vh[4][2], vl[4][2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float bv = P.bq[256 + kHd * h + 16 * c + li];
#pragma unroll
      for (int b = 0; b < 4; ++b) split4v(vv[b][c] + bv, vh[b][c], vl[b][c]);
    }
    float* ob = P.o + rbase * kD;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      bf16x4v ph[4], pl[4];
#pragma unroll
      for (int b = 0; b < 4; ++b) split4v(s[b][a], ph[b], pl[b]);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b = 0; b < 4; ++b) acc = mfma3k16(ph[b], pl[b], vh[b][c], vl[b][c], acc);
        const int col = kHd * h + 16 * c + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 16 * a + 4 * kg + r;
          ob[(size_t)i * kD + col] = acc[r];
          const short hi = dca::f2bf(acc[r]);
          img_h[i * kPX + col] = hi;
          img_l[i * kPX + col] = dca::f2bf(acc[r] - dca::bf2f(hi));
        }
      }
    }
  }
  __syncthreads();                                        // O images complete

  // ---- D: E1 = E0' + O·W_outᵀ, wave w: output column tiles 2w, 2w + 1; acc lane (unit = 16a + 4kg + r, col)
  {
    f32x4 acc[4][2];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 wh[2], wl[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        wh[t] = gfrag(P.woh, 16 * (2 * w + t), 32 * ks, lane);
        wl[t] = gfrag(P.wol, 16 * (2 * w + t), 32 * ks, lane);
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const bf16x8 oh = frag(img_h, kPX, 16 * a, 32 * ks, lane), ol = frag(img_l, kPX, 16 * a, 32 * ks, lane);
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[a][t] = mfma3(oh, ol, wh[t], wl[t], acc[a][t]);
      }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int col = 16 * (2 * w + t) + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int u = 16 * a + 4 * kg + r;
          const size_t g = (rbase + u) * kD + col;
          const float v = acc[a][t][r] + P.e0[g];
          P.e1[g] = v;
          e1s[u * kPE + col] = v;
        }
      }
  }
  __syncthreads();

  // ---- E: pools (first maximum, like pool_kernel) — thread t: column t & 127, types 3·(t >> 7) … +2
  {
    const int c = tid & 127, t0 = 3 * (tid >> 7);
#pragma unroll
    for (int t = t0; t < t0 + 3; ++t) {
      const int src = (P.compat && t == 5) ? 3 : t;
      float m = -INFINITY;
      int am = 0;
      for (int u = P.off[src]; u < P.off[src + 1]; ++u) {
        const float v = e1s[u * kPE + c];
        if (v > m) {
          m = v;
          am = u - P.off[src];
        }
      }
      P.x896[(size_t)n * 896 + kD + t * kD + c] = m;
      P.arg[((size_t)n * 6 + t) * kD + c] = (unsigned char)am;
    }
  }
}


}  // namespace

extern "C" hipError_t dca_attn_block_fwd_f32(const float* e0, const float* bout, const float* gamma, const float* beta,
                                             const short* wqh, const short* wql, const float* bq, const short* woh,
                                             const short* wol, float* xn, float* mu, float* rs, float* qkv, float* o,
                                             float* lse, float* e1, float* x896, unsigned char* arg, const int* off,
                                             int compat, int N, float eps, hipStream_t stream) {
  if (N < 1) return hipSuccess;
  BlockArgs a{e0, bout, gamma, beta, wqh, wql, bq, woh, wol, xn, mu, rs, qkv, o, lse, e1, x896, arg, {0}, compat,
              0.17677669529663687f /* 1/sqrt(32) */, eps};
  for (int i = 0; i < 7; ++i) a.off[i] = off[i];
  if (a.off[6] != kU) return hipErrorInvalidValue;
  hipLaunchKernelGGL(attn_block_fwd_f32_kernel, dim3(N), dim3(256), 0, stream, a);
  return hipGetLastError();
}
