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
  const void* wqh; const void* wql; const float* bq;       // (384, 128) bf16 hi / lo (EX: fp32, wql unused), bias
  const void* woh; const void* wol;                        // (128, 128)
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

// Operand abstraction of the two precisions. EX = false: bf16x3 — an operand is a (hi, lo) bf16 pair, a product three
// bf16 MFMAs (hi·hi + lo·hi + hi·lo). EX = true: IEEE fp32 — the operand is the fp32 values themselves and a K = 32
// (K = 16) step is 8 (4) v_mfma_f32_16x16x4_f32 calls: sub-step j takes k = 8·(lane>>4) + j (4·(lane>>4) + j) of
// the lane's k-group, i.e. exactly the elements the bf16 lane layout holds, so every fragment load, accumulator
// layout and LDS image of the bf16x3 form carries over with fp32 in place of the (hi, lo) pair — and the same
// register count (8 floats = a bf16x8 hi + lo pair). Every product is then an fp32 fma (the fp32-exact learner), and
// the softmax takes libm expf / logf instead of the hardware approximations.
template <bool EX> struct F8;
template <> struct F8<false> { bf16x8 h, l; };
template <> struct F8<true> { float v[8]; };
template <bool EX> struct F4;
template <> struct F4<false> { bf16x4v h, l; };
template <> struct F4<true> { f32x4 v; };

template <bool EX>
__device__ __forceinline__ F8<EX> mk8(const float* v) {
  F8<EX> f;
  if constexpr (EX) {
#pragma unroll
    for (int j = 0; j < 8; ++j) f.v[j] = v[j];
  } else {
    split8v(v, f.h, f.l);
  }
  return f;
}
template <bool EX>
__device__ __forceinline__ F4<EX> mk4(const f32x4 v) {
  F4<EX> f;
  if constexpr (EX) f.v = v;
  else split4v(v, f.h, f.l);
  return f;
}
template <bool EX>
__device__ __forceinline__ f32x4 mma8(const F8<EX>& a, const F8<EX>& b, f32x4 c) {
  if constexpr (EX) {
#pragma unroll
    for (int j = 0; j < 8; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[j], b.v[j], c, 0, 0, 0);
    return c;
  } else {
    return mfma3(a.h, a.l, b.h, b.l, c);
  }
}
template <bool EX>
__device__ __forceinline__ f32x4 mma4(const F4<EX>& a, const F4<EX>& b, f32x4 c) {
  if constexpr (EX) {
#pragma unroll
    for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[j], b.v[j], c, 0, 0, 0);
    return c;
  } else {
    return mfma3k16(a.h, a.l, b.h, b.l, c);
  }
}
__device__ __forceinline__ void ld8(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
// weight fragment (gfrag's order) of either precision: EX reads the fp32 image [row tile][k-step][lane][8] from wh
template <bool EX>
__device__ __forceinline__ F8<EX> wfrag8(const void* wh, const void* wl, int m0, int k0, int lane) {
  F8<EX> f;
  if constexpr (EX) {
    ld8(static_cast<const float*>(wh) + ((size_t)((m0 >> 4) * (kD / 32) + (k0 >> 5)) * 64 + lane) * 8, f.v);
  } else {
    f.h = gfrag(static_cast<const short*>(wh), m0, k0, lane);
    f.l = gfrag(static_cast<const short*>(wl), m0, k0, lane);
  }
  return f;
}
// the fwd kernel's Xn / O image: bf16 hi ‖ lo [64][kPX] (EX = false) or fp32 [64][kPE] (EX = true), same footprint
constexpr int kImgBytes = 2 * kU * kPX * 2;
static_assert(kU * kPE * 4 <= kImgBytes, "fp32 image must fit the bf16 pair");
template <bool EX>
__device__ __forceinline__ F8<EX> ifrag(const char* img, int m0, int k0, int lane) {
  F8<EX> f;
  if constexpr (EX) {
    ld8(reinterpret_cast<const float*>(img) + (m0 + (lane & 15)) * kPE + k0 + 8 * (lane >> 4), f.v);
  } else {
    const short* h = reinterpret_cast<const short*>(img);
    f.h = frag(h, kPX, m0, k0, lane);
    f.l = frag(h + kU * kPX, kPX, m0, k0, lane);
  }
  return f;
}
// 8 consecutive values of row u from column c into the image
template <bool EX>
__device__ __forceinline__ void iput8(char* img, int u, int c, const float* x) {
  if constexpr (EX) {
    float* d = reinterpret_cast<float*>(img) + u * kPE + c;
    *reinterpret_cast<float4*>(d) = make_float4(x[0], x[1], x[2], x[3]);
    *reinterpret_cast<float4*>(d + 4) = make_float4(x[4], x[5], x[6], x[7]);
  } else {
    bf16x8 hi, lo;
    split8v(x, hi, lo);
    short* h = reinterpret_cast<short*>(img);
    *reinterpret_cast<bf16x8*>(h + u * kPX + c) = hi;
    *reinterpret_cast<bf16x8*>(h + kU * kPX + u * kPX + c) = lo;
  }
}
template <bool EX>
__device__ __forceinline__ void iput1(char* img, int i, int col, float v) {
  if constexpr (EX) {
    reinterpret_cast<float*>(img)[i * kPE + col] = v;
  } else {
    short* h = reinterpret_cast<short*>(img);
    const short hi = dca::f2bf(v);
    h[i * kPX + col] = hi;
    h[kU * kPX + i * kPX + col] = dca::f2bf(v - dca::bf2f(hi));
  }
}

// Two rows in flight per CU (256 VGPRs). (Measured slower and removed: one row per CU with the phase-B weight
// fragments double-buffered one k-step ahead — 5v5 step 8.45 vs 8.15 ms.) EX: the IEEE-fp32 twin (F8 / F4 above).
template <bool EX>
__global__ __launch_bounds__(256, 2) void attn_block_fwd_f32_kernel(BlockArgs P) {
  __shared__ __attribute__((aligned(16))) char img[kImgBytes];                   // Xn, then O
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
    for (int i = 0; i < 4; ++i) iput8<EX>(img, u, 32 * p + 8 * i, x + 8 * i);
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
  {
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    F8<EX> xf[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) xf[a] = ifrag<EX>(img, 16 * a, 32 * ks, lane);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int rq = kHd * h + 16 * c;
      const F8<EX> qw = wfrag8<EX>(P.wqh, P.wql, rq, 32 * ks, lane);
      const F8<EX> kw = wfrag8<EX>(P.wqh, P.wql, 128 + rq, 32 * ks, lane);
      const F8<EX> vw = wfrag8<EX>(P.wqh, P.wql, 256 + rq, 32 * ks, lane);
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        qt[c][a] = mma8<EX>(qw, xf[a], qt[c][a]);    // m = d (weight row), n = unit
        kt[c][a] = mma8<EX>(kw, xf[a], kt[c][a]);
        vv[a][c] = mma8<EX>(xf[a], vw, vv[a][c]);    // m = unit, n = d
      }
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
    F4<EX> qf[2][4], kf[2][4];
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
        qf[c][a] = mk4<EX>(qt[c][a] + bqv);
        kf[c][a] = mk4<EX>(kt[c][a] + bkv);
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
        for (int c = 0; c < 2; ++c) acc = mma4<EX>(kf[c][b], qf[c][a], acc);
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
          const float e = EX ? expf(s[b][a][r] * P.scale - m) : __expf(s[b][a][r] * P.scale - m);
          s[b][a][r] = e;
          sum += e;
        }
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      const float inv = 1.f / sum;
#pragma unroll
      for (int b = 0; b < 4; ++b) s[b][a] *= inv;
      if (kg == 0) lse[16 * a + li] = m + (EX ? logf(sum) : __logf(sum));
    }
    // O = P·V: A[m = i][k = j] = s[b][a], B[k = j][n = d] = v[b][c] (+ bias of column d)
    F4<EX> vf[4][2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float bv = P.bq[256 + kHd * h + 16 * c + li];
#pragma unroll
      for (int b = 0; b < 4; ++b) vf[b][c] = mk4<EX>(vv[b][c] + bv);
    }
    float* ob = P.o + rbase * kD;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      F4<EX> pf[4];
#pragma unroll
      for (int b = 0; b < 4; ++b) pf[b] = mk4<EX>(s[b][a]);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b = 0; b < 4; ++b) acc = mma4<EX>(pf[b], vf[b][c], acc);
        const int col = kHd * h + 16 * c + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 16 * a + 4 * kg + r;
          ob[(size_t)i * kD + col] = acc[r];
          iput1<EX>(img, i, col, acc[r]);
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
      F8<EX> wf[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) wf[t] = wfrag8<EX>(P.woh, P.wol, 16 * (2 * w + t), 32 * ks, lane);
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const F8<EX> of = ifrag<EX>(img, 16 * a, 32 * ks, lane);
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[a][t] = mma8<EX>(of, wf[t], acc[a][t]);
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

// =============================================================================================================
// Fused fp32 entity-attention block BACKWARD (gfx950, bf16x3 MFMA): ONE launch per step instead of demb + ∂O GEMM +
// attention backward + ∂Xn GEMM + LayerNorm backward (attn.hip / hipBLASLt: ≈1.86 ms of the 5v5 step's critical path
// at N = 11 200 rows). One 256-thread workgroup (4 waves) per timestep row n (64 unit slots × 128):
//   0  ∂E1 = dtl⊗q + ∂pool routed to the argmax unit (demb semantics; compat: the enemy-tower pool's gradient goes to
//      the enemy-non-hero argmax) → HBM (the out-projection's weight gradient) and an fp32 LDS image
//   1  ∂O = ∂E1·W_out, wave h: head h's 32 columns (16x16x32, A split from the LDS image, B = W_outᵀ fragment images)
//   2  attention backward of head h on registers: D = rowsum(∂O∘O) and LSE per query in the accumulator lane layout
//      (DPP row sums, no LDS), S = Q·Kᵀ and dP = ∂O·Vᵀ i-major (∂O row fragments from a per-wave transposed LDS
//      image), P = exp(scale·S − LSE), ∂S = scale·P∘(dP − D); then the TRANSPOSED gradients
//        ∂Vᵀ = ∂Oᵀ·P,  ∂Kᵀ = Qᵀ·∂S  (16x16x16: ∂O's and P / ∂S's accumulators ARE the operands),
//        ∂Qᵀ = Kᵀ·∂Sᵀ  (16x16x32, ∂Sᵀ from a per-wave hi / lo LDS image by transposed reads)
//      whose accumulator lanes (d = 4kg + r, unit = lane&15) are exactly 16x16x16 A fragments over d → ∂QKV to HBM
//      (16-B stores, the QKV weight gradient's operand)
//   3  ∂Xn partial of head h = Σ_{x ∈ q,k,v} ∂Xᵀ_h·W_x[head rows] (16x16x16, B = W_qkv k16-fragment images) → the
//      wave's own fp32 LDS slot; the four slots are summed in a fixed order (deterministic)
//   4  LayerNorm backward + residual: ∂E0 = ∂E1 + rstd·(g − mean(g) − x̂·mean(g∘x̂)), g = ∂Xn∘γ → HBM (the encoder
//      backward's input); the row's [∂γ | ∂β | ∂b_τ per type] partial (1024 floats) → HBM, summed by
//      colsum_rows_kernel in a fixed order.
// LDS: 4 slots of a 64 × 132 fp32 image (135 KB) — phase 0/1 slot 0 = ∂E1, phase 2 slot h = wave h's ∂Oᵀ and ∂Sᵀ
// images, phase 3 slot h = wave h's ∂Xn partial, phase 4 slots 0-2 = the partial sums — one workgroup per CU.
// Measured at N = 11 200 (5v5 learner step): first 1936 µs against 1858 µs for the five launches it replaced; after
// the round-3 operand prefetch and interleaved partial sums 1647 µs, the learner's path since. 405 registers (no spills) and 135 KB of
// LDS leave one wave per SIMD and one row in flight per CU: ≈44 µs per row, the sum of each phase's exposed memory
// round trips (∂E1 inputs, W_out fragments, O / LSE / QKV rows, W_qkv fragments, E0' rows). Making it pay needs
// rows in flight per CU — a persistent form prefetching row n+1's operands during row n, or two waves per head.
constexpr int kPT = 132;                    // fp32 pitch of a 64 × 128 slot image
constexpr int kSlot = kU * kPT;             // floats per slot
constexpr int kPS = 72;                     // bf16 pitch of the per-wave ∂Oᵀ (32 × 64) and ∂Sᵀ (64 × 64) images
constexpr int kLnW = 8 * kD;                // per-row LayerNorm partial: ∂γ | ∂β | ∂b_τ (6 types)

struct BwdArgs {
  const float* dtl; const float* q; const float* dx; const unsigned char* arg;   // demb inputs (q row stride ldq)
  const float* o; const float* qkv; const float* bq; const float* lse;           // saved by the forward
  const float* e0; const float* bout; const float* mu; const float* rs; const float* gamma;
  const void* woth; const void* wotl;       // W_outᵀ (d, c) in 16x16x32 fragment order, bf16 hi / lo (EX: fp32)
  const void* wq4h; const void* wq4l;       // W_qkv (384, 128) in 16x16x16 B-fragment order, bf16 hi / lo (EX: fp32)
  float* de1; float* dqkv; float* de0; float* part;
  unsigned long long* trace;                // optional phase timestamps (s_memrealtime) of rows < 64: [row][wave][8]
  int off[7];
  int ldq, compat;
  float scale;
};

// 16x16x16 B fragment (rows 16·rt + 4·kg + j, column 16·ct + lane&15) of a k16-fragment-ordered (R, 128) image
// [R/16][8][lane][4]: one coalesced 512-B load per wave
__device__ __forceinline__ bf16x4v gfrag4(const short* __restrict__ w, int rt, int ct, int lane) {
  return *reinterpret_cast<const bf16x4v*>(w + ((size_t)(rt * 8 + ct) * 64 + lane) * 4);
}
// Σ over the 16 lanes of this lane's DPP row (xor 1, 2 by quad_perm, half-row and row mirrors), in every lane
__device__ __forceinline__ float row_sum16(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));
  return v;
}
// element jj of lane l = img[k0 + 8(l>>4) + jj][c0 + (l&15)] of a bf16 image [.][kPS] (two transposed reads)
__device__ __forceinline__ bf16x8 frag_tr(const short* img, int k0, int c0, int lane) {
  typedef __attribute__((address_space(3))) bf16x4v lds_v4;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const short* a = img + (k0 + 8 * g + q) * kPS + c0 + 4 * p;
  const bf16x4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)a);
  const bf16x4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a + 4 * kPS));
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}
__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// EX helpers of the backward: the 16x16x16 weight fragment (gfrag4's order) and the per-wave transposed images —
// fp32 [rows][kPF] instead of the bf16 hi / lo pair [rows][kPS] (26 KB of a 33 KB slot), read transposed by scalar
// LDS reads (element jj of lane l = img[k0 + 8(l>>4) + jj][c0 + (l&15)], as frag_tr)
constexpr int kPF = 68;
static_assert(96 * kPF <= kSlot, "fp32 transposed images must fit a slot");
template <bool EX>
__device__ __forceinline__ F4<EX> wfrag4(const void* wh, const void* wl, int rt, int ct, int lane) {
  F4<EX> f;
  if constexpr (EX) {
    f.v = *reinterpret_cast<const f32x4*>(static_cast<const float*>(wh) + ((size_t)(rt * 8 + ct) * 64 + lane) * 4);
  } else {
    f.h = gfrag4(static_cast<const short*>(wh), rt, ct, lane);
    f.l = gfrag4(static_cast<const short*>(wl), rt, ct, lane);
  }
  return f;
}
// one C-layout accumulator (rows 4kg + r of column li at (row0, col0)) transposed into the image: element r goes to
// img[col0 + li][row0 + 4kg + r] — a 16-B store (EX) or two 8-B stores (hi, lo)
template <bool EX>
__device__ __forceinline__ void tput(void* ih, void* il, int col0, int row0, const f32x4& v, int lane) {
  const int li = lane & 15, kg = lane >> 4;
  if constexpr (EX) {
    *reinterpret_cast<f32x4*>(static_cast<float*>(ih) + (col0 + li) * kPF + row0 + 4 * kg) = v;
  } else {
    bf16x4v hi, lo;
    split4v(v, hi, lo);
    *reinterpret_cast<bf16x4v*>(static_cast<short*>(ih) + (col0 + li) * kPS + row0 + 4 * kg) = hi;
    *reinterpret_cast<bf16x4v*>(static_cast<short*>(il) + (col0 + li) * kPS + row0 + 4 * kg) = lo;
  }
}
template <bool EX>
__device__ __forceinline__ F8<EX> tfrag2(const void* ih, const void* il, int k0, int c0, int lane) {
  F8<EX> f;
  if constexpr (EX) {
    const float* b = static_cast<const float*>(ih) + (k0 + 8 * (lane >> 4)) * kPF + c0 + (lane & 15);
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) f.v[jj] = b[jj * kPF];
  } else {
    f.h = frag_tr(static_cast<const short*>(ih), k0, c0, lane);
    f.l = frag_tr(static_cast<const short*>(il), k0, c0, lane);
  }
  return f;
}

template <bool EX>
__global__ __launch_bounds__(256, 1) void attn_block_bwd_f32_kernel(BwdArgs P) {
  __shared__ __attribute__((aligned(16))) float sm[4 * kSlot];
  __shared__ float sd[kU];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, kg = lane >> 4, li = lane & 15;
  const int n = blockIdx.x;
  const size_t rbase = (size_t)n * kU;

#define PSTAMP(ev)                                                                                        \
  if (P.trace && n < 64 && lane == 0) P.trace[((size_t)n * 4 + w) * 8 + (ev)] = __builtin_amdgcn_s_memrealtime()
  PSTAMP(0);
  // phase 1's W_outᵀ fragments (head w) requested first: their round trip runs alongside phase 0's
  F8<EX> wf[4][2];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int t = 0; t < 2; ++t) wf[ks][t] = wfrag8<EX>(P.woth, P.wotl, kHd * w + 16 * t, 32 * ks, lane);
  // ---- 0: ∂E1 (thread: column c, units 32·(tid>>7) … +31)
  if (tid < kU) sd[tid] = P.dtl[(size_t)n * kU + tid];
  {
    // this thread's column operands are requested before the barrier, alongside the ∂logit load
    const int c = tid & 127, uh = tid >> 7;
    const float qc = P.q[(size_t)n * P.ldq + c];
    int au[6];
    float dp[6];
#pragma unroll
    for (int t = 0; t < 6; ++t) {
      const int src = (P.compat && t == 5) ? 3 : t;
      au[t] = P.off[src] + P.arg[((size_t)n * 6 + t) * kD + c];
      dp[t] = P.dx[(size_t)n * 896 + kD + t * kD + c];
    }
    __syncthreads();
#pragma unroll 4
    for (int i = 0; i < 32; ++i) {
      const int u = uh * 32 + i;
      float v = sd[u] * qc;
#pragma unroll
      for (int t = 0; t < 6; ++t) v += (au[t] == u) ? dp[t] : 0.f;
      P.de1[(rbase + u) * kD + c] = v;
      sm[u * kPT + c] = v;
    }
  }
  __syncthreads();

  PSTAMP(1);
  // ---- 1: ∂O of head h = w: dO[a][t] lane (unit i = 16a + 4kg + r, d = 16t + li within the head)
  const int h = w;
  // (Requesting phase 2's Q rows and Q / K / V biases here as well measured slower: kernel 1.698 vs 1.660 ms — the
  // ∂O phase then waits on them through the in-order vector-memory counter.)
  // phase 2's O and LSE operands for D_i (query rows 16a + 4kg + r, this lane's two d columns), requested before the
  // ∂O products so their round trips overlap them
  float opre[4][4][2], Lr[4][4];
  {
    const float* ob = P.o + rbase * kD + kHd * h;
    const float* lb = P.lse + ((size_t)n * 4 + h) * kU;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * a + 4 * kg + r;
        opre[a][r][0] = ob[(size_t)i * kD + li];
        opre[a][r][1] = ob[(size_t)i * kD + 16 + li];
        Lr[a][r] = lb[i];
      }
  }
  f32x4 dO[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int t = 0; t < 2; ++t) dO[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const F8<EX> af = mk8<EX>(&sm[(16 * a + li) * kPT + 32 * ks + 8 * kg]);
#pragma unroll
      for (int t = 0; t < 2; ++t) dO[a][t] = mma8<EX>(af, wf[ks][t], dO[a][t]);
    }
  }
  __syncthreads();                                        // slot 0 (∂E1 image) is wave 0's from here on

  PSTAMP(2);
  // ---- 2: attention backward of head h. Per-wave images in slot h: ∂Oᵀ [32 d] and (scale·∂S)ᵀ [64 j] — bf16 hi / lo
  //      pairs of pitch kPS, or (EX) fp32 of pitch kPF
  void *dTh, *dTl, *STh, *STl;
  if constexpr (EX) {
    dTh = dTl = sm + h * kSlot;
    STh = STl = sm + h * kSlot + 32 * kPF;
  } else {
    short* b = reinterpret_cast<short*>(sm + h * kSlot);
    dTh = b;
    dTl = b + 32 * kPS;
    STh = b + 64 * kPS;
    STl = b + 128 * kPS;
  }
  const float* const base = P.qkv + rbase * 384 + kHd * h;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int t = 0; t < 2; ++t) tput<EX>(dTh, dTl, 16 * t, 16 * a, dO[a][t], lane);
  // D_i = Σ_d ∂O[i][d]·O[i][d] and LSE_i for i = 16a + 4kg + r (the lane's query rows in the S layout below)
  float Dr[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) Dr[a][r] = row_sum16(dO[a][0][r] * opre[a][r][0] + dO[a][1][r] * opre[a][r][1]);
  lds_wait();
  // S = Q·Kᵀ and dP = ∂O·Vᵀ, i-major: p[a][b] lane (query i = 16a + 4kg + r, key j = 16b + li)
  f32x4 p[4][4], dp[4][4];
  {
    float qb[8], kb8[8], vb8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      qb[j] = P.bq[kHd * h + 8 * kg + j];
      kb8[j] = P.bq[128 + kHd * h + 8 * kg + j];
      vb8[j] = P.bq[256 + kHd * h + 8 * kg + j];
    }
    F8<EX> qf[4], df[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      float v[8];
      const float4 x0 = *reinterpret_cast<const float4*>(base + (size_t)(16 * a + li) * 384 + 8 * kg);
      const float4 x1 = *reinterpret_cast<const float4*>(base + (size_t)(16 * a + li) * 384 + 8 * kg + 4);
      v[0] = x0.x + qb[0]; v[1] = x0.y + qb[1]; v[2] = x0.z + qb[2]; v[3] = x0.w + qb[3];
      v[4] = x1.x + qb[4]; v[5] = x1.y + qb[5]; v[6] = x1.z + qb[6]; v[7] = x1.w + qb[7];
      qf[a] = mk8<EX>(v);
      df[a] = tfrag2<EX>(dTh, dTl, 0, 16 * a, lane);
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      float kv[8], vv8[8];
      const float* kr = base + 128 + (size_t)(16 * b + li) * 384 + 8 * kg;
      const float* vr = base + 256 + (size_t)(16 * b + li) * 384 + 8 * kg;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        kv[j] = kr[j] + kb8[j];
        vv8[j] = vr[j] + vb8[j];
      }
      const F8<EX> kf = mk8<EX>(kv), vf = mk8<EX>(vv8);
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        p[a][b] = mma8<EX>(qf[a], kf, f32x4{0.f, 0.f, 0.f, 0.f});
        dp[a][b] = mma8<EX>(df[a], vf, f32x4{0.f, 0.f, 0.f, 0.f});
      }
    }
  }
  // P = exp(scale·S − LSE); dp ← scale·P∘(dP − D) = ∂L/∂(Q·Kᵀ); its transpose to the images for ∂Qᵀ
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float pr = EX ? expf(p[a][b][r] * P.scale - Lr[a][r]) : __expf(p[a][b][r] * P.scale - Lr[a][r]);
        p[a][b][r] = pr;
        dp[a][b][r] = P.scale * pr * (dp[a][b][r] - Dr[a][r]);
      }
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) tput<EX>(STh, STl, 16 * b, 16 * a, dp[a][b], lane);
  // ∂Vᵀ[t][b] = Σ_a ∂Oᵀ(t, a)·P(a, b) and ∂Kᵀ[t][b] = Σ_a Qᵀ(t, a)·∂S(a, b): lanes (d = 16t + 4kg + r, j = 16b + li)
  f32x4 gV[2][4], gK[2][4], gQ[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const float bqc = P.bq[kHd * h + 16 * t + li];
    F4<EX> of[4], qf[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      of[a] = mk4<EX>(dO[a][t]);
      f32x4 qv;
#pragma unroll
      for (int r = 0; r < 4; ++r) qv[r] = base[(size_t)(16 * a + 4 * kg + r) * 384 + 16 * t + li] + bqc;
      qf[a] = mk4<EX>(qv);
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      f32x4 av = {0.f, 0.f, 0.f, 0.f}, ak = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        av = mma4<EX>(of[a], mk4<EX>(p[a][b]), av);
        ak = mma4<EX>(qf[a], mk4<EX>(dp[a][b]), ak);
      }
      gV[t][b] = av;
      gK[t][b] = ak;
    }
  }
  lds_wait();
  // ∂Qᵀ[t][a] = Σ_ks Kᵀ(t, ks)·∂Sᵀ(ks, a): lanes (d = 16t + 4kg + r, i = 16a + li)
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const float kbc = P.bq[128 + kHd * h + 16 * t + li];
    F8<EX> kf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      float kv[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) kv[jj] = base[(size_t)(32 * ks + 8 * kg + jj) * 384 + 128 + 16 * t + li] + kbc;
      kf[ks] = mk8<EX>(kv);
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      f32x4 aq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) aq = mma8<EX>(kf[ks], tfrag2<EX>(STh, STl, 32 * ks, 16 * a, lane), aq);
      gQ[t][a] = aq;
    }
  }
  // ∂QKV → HBM (no bias: the bias gradient is the column sum), 4 consecutive d per lane = one 16-B store
  {
    float* ob = P.dqkv + rbase * 384 + kHd * h;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u4 = 0; u4 < 4; ++u4) {
        float* rowp = ob + (size_t)(16 * u4 + li) * 384 + 16 * t + 4 * kg;
        *reinterpret_cast<f32x4*>(rowp) = gQ[t][u4];
        *reinterpret_cast<f32x4*>(rowp + 128) = gK[t][u4];
        *reinterpret_cast<f32x4*>(rowp + 256) = gV[t][u4];
      }
  }

  PSTAMP(3);
  // the LayerNorm phase's operands — this thread's 32 columns of E0' (HBM), ∂E1 (written in phase 0, L2), μ, rstd
  // — requested now, so their round trips overlap the ∂Xn products (they were two exposed trips of a 9.6 µs phase).
  // Issuing them between the two ∂Xn halves instead (so half 0's weight fragments do not wait behind them in the
  // in-order vector-memory counter) measured the same: 1.656 vs 1.647 ms.
  const int lu = tid >> 2, lc0 = 32 * (tid & 3);
  f32x4 e0pre[8], de1pre[8], gpre[8], bpre[8];
  float mu_pre, rs_pre;
  {
    const size_t row = rbase + lu;
#pragma unroll
    for (int j4 = 0; j4 < 8; ++j4) {
      e0pre[j4] = *reinterpret_cast<const f32x4*>(P.e0 + row * kD + lc0 + 4 * j4);
      de1pre[j4] = *reinterpret_cast<const f32x4*>(P.de1 + row * kD + lc0 + 4 * j4);
      gpre[j4] = *reinterpret_cast<const f32x4*>(P.gamma + lc0 + 4 * j4);
      bpre[j4] = *reinterpret_cast<const f32x4*>(P.bout + lc0 + 4 * j4);
    }
    mu_pre = P.mu[row];
    rs_pre = P.rs[row];
  }
  // ---- 3: ∂Xn partial of head h: A = ∂Xᵀ accumulators (m = unit, k = d), B = W_qkv rows 128x + 32h + 16t + …
  {
    F4<EX> af[3][2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u4 = 0; u4 < 4; ++u4) {
        af[0][t][u4] = mk4<EX>(gQ[t][u4]);
        af[1][t][u4] = mk4<EX>(gK[t][u4]);
        af[2][t][u4] = mk4<EX>(gV[t][u4]);
      }
    float* slot = sm + h * kSlot;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      f32x4 acc[4][4];
#pragma unroll
      for (int u4 = 0; u4 < 4; ++u4)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[u4][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int x = 0; x < 3; ++x)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int rt = 8 * x + 2 * h + t;
          F4<EX> bf[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) bf[c] = wfrag4<EX>(P.wq4h, P.wq4l, rt, 4 * half + c, lane);
#pragma unroll
          for (int u4 = 0; u4 < 4; ++u4)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[u4][c] = mma4<EX>(af[x][t][u4], bf[c], acc[u4][c]);
        }
      // (the wave's own slot: its ∂Oᵀ / ∂Sᵀ images are dead)
#pragma unroll
      for (int u4 = 0; u4 < 4; ++u4)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int r = 0; r < 4; ++r) slot[(16 * u4 + 4 * kg + r) * kPT + 64 * half + 16 * c + li] = acc[u4][c][r];
    }
  }
  __syncthreads();

  PSTAMP(4);
  // ---- 4: LayerNorm backward + residual, 4 threads per unit row (32 columns each)
  {
    const int u = lu, c0 = lc0;
    const size_t row = rbase + u;
    const float mu = mu_pre, rs = rs_pre;
    float dxn[32], xh[32];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j4 = 0; j4 < 8; ++j4) {
      const int c = c0 + 4 * j4;
      const float4 p0 = *reinterpret_cast<const float4*>(&sm[0 * kSlot + u * kPT + c]);
      const float4 p1 = *reinterpret_cast<const float4*>(&sm[1 * kSlot + u * kPT + c]);
      const float4 p2 = *reinterpret_cast<const float4*>(&sm[2 * kSlot + u * kPT + c]);
      const float4 p3 = *reinterpret_cast<const float4*>(&sm[3 * kSlot + u * kPT + c]);
      const float pv[4][4] = {{p0.x, p0.y, p0.z, p0.w}, {p1.x, p1.y, p1.z, p1.w}, {p2.x, p2.y, p2.z, p2.w},
                              {p3.x, p3.y, p3.z, p3.w}};
      const float ev[4] = {e0pre[j4][0], e0pre[j4][1], e0pre[j4][2], e0pre[j4][3]};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float d = ((pv[0][q] + pv[1][q]) + pv[2][q]) + pv[3][q];
        const float x = (ev[q] - bpre[j4][q] - mu) * rs;
        dxn[4 * j4 + q] = d;
        xh[4 * j4 + q] = x;
        const float g = d * gpre[j4][q];
        s1 += g;
        s2 += g * x;
      }
    }
    s1 += __shfl_xor(s1, 1, 64);
    s1 += __shfl_xor(s1, 2, 64);
    s2 += __shfl_xor(s2, 1, 64);
    s2 += __shfl_xor(s2, 2, 64);
    s1 *= (1.f / kD);
    s2 *= (1.f / kD);
    float de0v[32];
#pragma unroll
    for (int j4 = 0; j4 < 8; ++j4) {
      const int c = c0 + 4 * j4;
      const float rv[4] = {de1pre[j4][0], de1pre[j4][1], de1pre[j4][2], de1pre[j4][3]};
      float o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = 4 * j4 + q;
        const float g = dxn[j] * gpre[j4][q];
        o[q] = rv[q] + rs * (g - s1 - xh[j] * s2);
        de0v[j] = o[q];
      }
      *reinterpret_cast<float4*>(P.de0 + row * kD + c) = make_float4(o[0], o[1], o[2], o[3]);
    }
    __syncthreads();                                      // every thread has read the ∂Xn partial slots
#pragma unroll
    for (int j = 0; j < 32; j += 4) {                     // 16-byte LDS stores (kPT and c0 are multiples of 4)
      float* s0 = &sm[0 * kSlot + u * kPT + c0 + j];
      *reinterpret_cast<float4*>(s0) =
          make_float4(dxn[j] * xh[j], dxn[j + 1] * xh[j + 1], dxn[j + 2] * xh[j + 2], dxn[j + 3] * xh[j + 3]);
      *reinterpret_cast<float4*>(s0 + kSlot) = make_float4(dxn[j], dxn[j + 1], dxn[j + 2], dxn[j + 3]);
      *reinterpret_cast<float4*>(s0 + 2 * kSlot) = make_float4(de0v[j], de0v[j + 1], de0v[j + 2], de0v[j + 3]);
    }
  }
  __syncthreads();
  PSTAMP(5);
  // the row's partial [∂γ | ∂β | ∂b_τ]: fixed-order sums over its units (∂b_τ over the units of type τ)
  for (int e = tid; e < kLnW; e += 256) {
    int sl, c, u0, u1;
    if (e < 2 * kD) {
      sl = e >> 7; c = e & 127; u0 = 0; u1 = kU;
    } else {
      const int t = (e - 2 * kD) >> 7;
      sl = 2; c = e & 127; u0 = P.off[t]; u1 = P.off[t + 1];
    }
    // four interleaved accumulators (fixed order): the serial LDS-load → add chain was the phase's latency
    const float* col = sm + sl * kSlot + c;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int u = u0;
#pragma unroll 2
    for (; u + 4 <= u1; u += 4) {
      a0 += col[u * kPT];
      a1 += col[(u + 1) * kPT];
      a2 += col[(u + 2) * kPT];
      a3 += col[(u + 3) * kPT];
    }
    for (; u < u1; ++u) a0 += col[u * kPT];
    P.part[(size_t)n * kLnW + e] = (a0 + a1) + (a2 + a3);
  }
  PSTAMP(6);
#undef PSTAMP
}

// out[g][c] = Σ rows [g·per, min(R, (g+1)·per)) of part (R, W), fixed order: 64 columns × 4 row phases per block,
// grid (W/64, G). Two launches (G groups, then 1) sum the N per-row LayerNorm partials with thousands of threads in
// flight instead of one latency-bound chain per column.
__global__ __launch_bounds__(256) void colsum_rows_kernel(const float* __restrict__ part, int R, int W, int per,
                                                          float* __restrict__ out) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), ph = threadIdx.x >> 6, g = blockIdx.y;
  const int r0 = g * per, r1 = min(R, r0 + per);
  float s = 0.f;
  if (c < W) {
    int r = r0 + ph;
    for (; r + 12 < r1; r += 16) {
      const float v0 = part[(size_t)r * W + c], v1 = part[(size_t)(r + 4) * W + c];
      const float v2 = part[(size_t)(r + 8) * W + c], v3 = part[(size_t)(r + 12) * W + c];
      s += v0;
      s += v1;
      s += v2;
      s += v3;
    }
    for (; r < r1; r += 4) s += part[(size_t)r * W + c];
  }
  __shared__ float red[4][64];
  red[ph][threadIdx.x & 63] = s;
  __syncthreads();
  if (ph == 0 && c < W)
    out[(size_t)g * W + c] = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

// (A fused ∂Xn GEMM + LayerNorm backward kernel for the unfused block backward measured 1033 vs 631 µs for the
// two launches it replaced and was removed in round 5, with that backward chain.)


}  // namespace

// exact = 0: bf16 hi / lo weight images (bf16x3); exact = 1: fp32 images in wqh / woh (wql / wol unused)
extern "C" hipError_t dca_attn_block_fwd_f32(const float* e0, const float* bout, const float* gamma, const float* beta,
                                             const void* wqh, const void* wql, const float* bq, const void* woh,
                                             const void* wol, float* xn, float* mu, float* rs, float* qkv, float* o,
                                             float* lse, float* e1, float* x896, unsigned char* arg, const int* off,
                                             int compat, int N, float eps, hipStream_t stream, int exact) {
  if (N < 1) return hipSuccess;
  BlockArgs a{e0, bout, gamma, beta, wqh, wql, bq, woh, wol, xn, mu, rs, qkv, o, lse, e1, x896, arg, {0}, compat,
              0.17677669529663687f /* 1/sqrt(32) */, eps};
  for (int i = 0; i < 7; ++i) a.off[i] = off[i];
  if (a.off[6] != kU) return hipErrorInvalidValue;
  if (exact) hipLaunchKernelGGL(attn_block_fwd_f32_kernel<true>, dim3(N), dim3(256), 0, stream, a);
  else hipLaunchKernelGGL(attn_block_fwd_f32_kernel<false>, dim3(N), dim3(256), 0, stream, a);
  return hipGetLastError();
}

extern "C" int dca_attn_block_bwd_groups(int N) { return N < 64 ? 1 : 64; }

// part: (N, 1024) per-row partials; tmp: (groups, 1024); sums: (1024) = [∂γ | ∂β | ∂b_τ (6×128)]
extern "C" hipError_t dca_attn_block_bwd_f32(const float* dtl, const float* q, int ldq, const float* dx,
                                             const unsigned char* arg, const int* off, int compat, const float* o,
                                             const float* qkv, const float* bq, const float* lse, const float* e0,
                                             const float* bout, const float* mu, const float* rs, const float* gamma,
                                             const void* woth, const void* wotl, const void* wq4h,
                                             const void* wq4l, float* de1, float* dqkv, float* de0, float* part,
                                             float* tmp, float* sums, int N, hipStream_t stream,
                                             unsigned long long* trace, int exact) {
  if (N < 1) return hipSuccess;
  BwdArgs a{dtl, q, dx, arg, o, qkv, bq, lse, e0, bout, mu, rs, gamma, woth, wotl, wq4h, wq4l, de1, dqkv, de0, part,
            trace, {0}, ldq, compat, 0.17677669529663687f /* 1/sqrt(32) */};
  for (int i = 0; i < 7; ++i) a.off[i] = off[i];
  if (a.off[6] != kU) return hipErrorInvalidValue;
  if (exact) hipLaunchKernelGGL(attn_block_bwd_f32_kernel<true>, dim3(N), dim3(256), 0, stream, a);
  else hipLaunchKernelGGL(attn_block_bwd_f32_kernel<false>, dim3(N), dim3(256), 0, stream, a);
  DCA_CHECK_LAUNCH();
  const int G = dca_attn_block_bwd_groups(N);
  const int per = (N + G - 1) / G;
  hipLaunchKernelGGL(colsum_rows_kernel, dim3(kLnW / 64, G), dim3(256), 0, stream, part, N, kLnW, per, tmp);
  DCA_CHECK_LAUNCH();
  hipLaunchKernelGGL(colsum_rows_kernel, dim3(kLnW / 64, 1), dim3(256), 0, stream, tmp, G, kLnW, G, sums);
  return hipGetLastError();
}

