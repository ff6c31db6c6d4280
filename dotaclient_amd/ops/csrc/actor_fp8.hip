// fp8 actor policy core (gfx950, OCP e4m3fn MFMA): one launch from the encoder's pooled features to the head logits
// of a batch of player slots — the reference actor's per-step policy evaluation (agent.py:641-660 →
// policy.py:135-158: pre-RNN layer, LSTM step, the five heads), BASELINE config 5 (fp8 actor inference).
//
//   x896 (n, 896) bf16  ──►  pre = relu(x·W_preᵀ + b)                       (16 × 256 per workgroup)
//                      ──►  gates = [pre | h]·[W_ih | W_hh]ᵀ + b_ih + b_hh   (16 × 2048, unit-major gate columns)
//                      ──►  LSTM cell (c, h fp32 state in place, resets / inactive slots)
//                      ──►  z = h·W_headsᵀ + b                               (16 × 160 → the sampling kernel)
//
// Quantisation. Weights: per output channel, scaled at hot-swap time (actor/batched.py Fp8ActorPolicy) so the
// channel's max |w| maps to 448, converted by torch to float8_e4m3fn and laid out in MFMA FRAGMENT ORDER
// [col tile][128-deep k-step][lane][32 B]: a wave reads one tile's k-step as one coalesced 2 KB load and the
// weights stream from L2 straight into registers (no LDS staging, no reuse inside a workgroup to stage for).
// Activations: per row, inside the kernel — the row's max |v| over the GEMM's whole K maps to 448 (x896 for the
// pre-RNN layer; [pre | h] jointly for the gates, fp8 keeps 3 mantissa bits at every exponent so the smaller h
// values do not need a scale of their own; h for the heads), converted by v_cvt_pk_fp8_f32 (RNE) into an LDS A
// image. Products run on v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 operands, unit block scales, fp32 accumulation;
// twice the rate of the 16x16x32 fp8 form); the epilogue applies
// scale_row · scale_col + bias. The cell's four gates of a (row, unit) sit in four adjacent lanes of the C layout
// (unit-major columns); a quad transpose by DPP broadcasts hands each lane one (row, unit).
//
// One 512-thread workgroup (8 waves) per 16 slots (n = 4096 slots → 256 workgroups, one per CU). Every workgroup streams all
// weights (1.8 MB of fp8) from L2 once, half the bytes of the bf16 path's operands, through a 4-deep register ring
// per wave that runs across the gate stage's chunk boundaries (1 pair of lookahead measured 61 µs for 4096 slots:
// the stream was latency-bound); the LSTM cell works on c staged in LDS so no global access sits inside the
// stream, and h / c leave in one coalesced pass.
#include "common.h"
#include <hip/hip_fp16.h>

namespace {

using dca::f32x4;

constexpr int BM = 16, NT = 512, NW = NT / 64, TPR = NT / BM;   // 8 waves; 32 staging threads per row
constexpr int XD = 896, PD = 256, HD = 512, GD = 4 * HD, KG = PD + HD, ZD = 160;
constexpr int LDX = XD + 16, LDG = KG + 16, LDF = PD + 4, LDH = HD + 4;   // LDS row pitches (bytes / floats)
constexpr float kQmax = 448.f;                                          // largest finite e4m3fn

// 8 fp32 → 8 e4m3fn bytes (round to nearest even), element j in byte j
__device__ __forceinline__ long long pack8(const float* v) {
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4], v[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6], v[7], hi, true);
  return (long long)(unsigned)lo | ((long long)(unsigned)hi << 32);
}

typedef int i32x8 __attribute__((ext_vector_type(8)));

// One K = 128 step on gfx950's block-scaled f8f6f4 MFMA with e4m3 A and B (format 0) and unit block scales
// (E8M0 127 = 2^0): twice the cycles of the 16x16x32 fp8 form for 4x the K, i.e. twice its rate — the per-row /
// per-channel dequantisation stays in the epilogue. Lane l's 32 operand bytes are k = 128u + 32(l>>4) + j (A rows /
// B columns l & 15); A and B use the same lane → k map, so the product is the sum over k whatever order the
// hardware takes the 32 bytes in.
__device__ __forceinline__ f32x4 mma128(const i32x8& a, const i32x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}

// A fragment of k-step u (128 deep) from a row-major fp8 LDS image: lane l holds A[row l&15][128u + 32(l>>4) + j]
__device__ __forceinline__ i32x8 afrag128(const unsigned char* img, int ld, int u, int lane) {
  const uint4* p = reinterpret_cast<const uint4*>(img + (lane & 15) * ld + 128 * u + 32 * (lane >> 4));
  const uint4 x = p[0], y = p[1];
  return i32x8{(int)x.x, (int)x.y, (int)x.z, (int)x.w, (int)y.x, (int)y.y, (int)y.z, (int)y.w};
}

// one fragment-ordered weight k-step (128 deep) of column tile `tile`: 32 B per lane, a wave's load is 2 KB contiguous
__device__ __forceinline__ i32x8 wfrag128(const i32x8* __restrict__ w, int ku, int tile, int u, int lane) {
  return w[((size_t)tile * ku + u) * 64 + lane];
}

// Streamed weight GEMM: NCH chunks of NTL column tiles (`tile(ch, i)`), each over K = 128·KU. The (chunk, k-step)
// sequence is ONE stream with a D-deep register ring of weight fragments, so the loads of the next chunk are in
// flight during the epilogue of the current one; the epilogue `epi(ch, acc)` runs after a chunk's last k-step (it
// must not touch global memory: every vector memory op counts in the same in-order vmcnt as the ring's loads).
template <int NTL, int KU, int NCH, int D, class TileFn, class Epi>
__device__ __forceinline__ void stream_gemm(const unsigned char* aimg, int lda, const i32x8* __restrict__ w,
                                            TileFn tile, int lane, Epi epi) {
  constexpr int T = NCH * KU;
  i32x8 ring[D][NTL];
  f32x4 acc[NTL];
#pragma unroll
  for (int i = 0; i < NTL; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto issue = [&](int slot, int t) {
    t = t < T ? t : T - 1;                         // past the end: reload the last step (never consumed)
    const int ch = t / KU, u = t - ch * KU;
#pragma unroll
    for (int i = 0; i < NTL; ++i) ring[slot][i] = wfrag128(w, KU, tile(ch, i), u, lane);
  };
#pragma unroll
  for (int d = 0; d < D; ++d) issue(d, d);
  for (int t0 = 0; t0 < T; t0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int t = t0 + d;
      if (t >= T) break;                           // (T need not be a multiple of D; wave-uniform)
      const int ch = t / KU, u = t - ch * KU;
      const i32x8 a = afrag128(aimg, lda, u, lane);
#pragma unroll
      for (int i = 0; i < NTL; ++i) acc[i] = mma128(a, ring[d][i], acc[i]);
      issue(d, t + D);
      if (u == KU - 1) {
        epi(ch, acc);
#pragma unroll
        for (int i = 0; i < NTL; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
}

__device__ __forceinline__ float dpp_quad_bcast(float v, int k) {   // lane (lane & ~3) + k of this lane's quad
  switch (k) {
    case 0: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x00, 0xF, 0xF, false));
    case 1: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x55, 0xF, 0xF, false));
    case 2: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xAA, 0xF, 0xF, false));
    default: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xFF, 0xF, 0xF, false));
  }
}

struct Fp8Args {
  const short* x896;                     // (n, 896) bf16
  const i32x8* wpre; const float* spre; const float* bpre;     // 256 × 896, fragment order
  const i32x8* wg; const float* sg; const float* bg;           // 2048 × 768 unit-major rows ([W_ih | W_hh])
  const i32x8* wh; const float* sh; const float* bh;           // 160 × 512 heads
  float* h; float* c;                    // (n, 512) fp32 state, in place
  const float* keep; const float* active;
  float* z;                              // (n, 160) fp32
  int n;
  long long* bump;                       // the sampler's step counter, += 1 here (null: the caller bumps it)
};

__global__ __launch_bounds__(NT) void actor_fp8_kernel(Fp8Args A) {
  __shared__ __attribute__((aligned(16))) unsigned char a8x[BM * LDX];   // x896 fp8, later h fp8 (heads)
  __shared__ __attribute__((aligned(16))) unsigned char a8g[BM * LDG];   // [pre | h] fp8
  __shared__ __attribute__((aligned(16))) float xf[BM * LDF];            // pre-RNN output fp32
  __shared__ __attribute__((aligned(16))) float hn[BM * LDH];            // new h fp32
  __shared__ __attribute__((aligned(16))) float cs[BM * LDH];            // c·keep, then the new c (active rows)
  __shared__ float s_row[3][BM];                                         // dequant scales per row
  __shared__ float s_keep[BM], s_act[BM];
  // per-column dequant scales and biases (read in the streamed GEMMs' epilogues, which must stay off global memory)
  __shared__ float col_s[PD + GD + ZD], col_b[PD + GD + ZD];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  // the sampling kernel (next launch) reads the counter: bumping it here saves a one-element launch per step
  if (A.bump && blockIdx.x == 0 && tid == 0) A.bump[0] += 1;
  const int q = lane >> 4, cl = lane & 15;
  const int row0 = blockIdx.x * BM;
  const int n = A.n;
  const int r = tid / TPR, sub = tid % TPR;            // staging: TPR threads per row
  const int grow_r = min(row0 + r, n - 1);
  const bool row_ok = row0 + r < n;

  // ---- stage 0: x896 row → fp8 (per-row scale); keep / active flags; column scales / biases
  for (int i = tid; i < PD + GD + ZD; i += NT) {
    const bool p = i < PD, g = !p && i < PD + GD;
    const int k = p ? i : (g ? i - PD : i - PD - GD);
    col_s[i] = p ? A.spre[k] : (g ? A.sg[k] : A.sh[k]);
    col_b[i] = p ? A.bpre[k] : (g ? A.bg[k] : A.bh[k]);
  }
  {
    if (sub == 0) {
      s_keep[r] = A.keep[grow_r];
      s_act[r] = (A.active == nullptr || A.active[grow_r] != 0.f) ? 1.f : 0.f;
    }
    constexpr int NCX = (XD / 8 + TPR - 1) / TPR;      // 8-element chunks per thread (the last one partial)
    float v[NCX][8];
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < NCX; ++i) {
      const int chk = min(sub + TPR * i, XD / 8 - 1);   // (a duplicate of the last chunk past the row's end)
      const dca::bf16x8 b = *reinterpret_cast<const dca::bf16x8*>(A.x896 + (size_t)grow_r * XD + 8 * chk);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[i][j] = dca::bf2f(b[j]);
        amax = fmaxf(amax, fabsf(v[i][j]));
      }
    }
    amax = dca::group_max<TPR>(amax);
    const float qs = amax > 0.f ? kQmax / amax : 1.f;
    if (sub == 0) s_row[0][r] = amax > 0.f ? amax / kQmax : 1.f;
#pragma unroll
    for (int i = 0; i < NCX; ++i) {
      if (sub + TPR * i >= XD / 8) continue;
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = v[i][j] * qs;
      *reinterpret_cast<long long*>(a8x + r * LDX + 8 * (sub + TPR * i)) = pack8(t);
    }
  }
  __syncthreads();

  // ---- stage 1: pre = relu(x·W_preᵀ·scales + b): wave w owns column tiles 2w, 2w+1
  stream_gemm<2, XD / 128, 1, 2>(
      a8x, LDX, A.wpre, [&](int, int i) { return 2 * w + i; }, lane, [&](int, const f32x4 (&acc)[2]) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int col = 16 * (2 * w + i) + cl;
          const float sc = col_s[col], b = col_b[col];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = 4 * q + e;
            xf[row * LDF + col] = fmaxf(acc[i][e] * s_row[0][row] * sc + b, 0.f);
          }
        }
      });
  __syncthreads();

  // ---- stage 2: [pre | keep·h_prev] → fp8 with one per-row scale; keep·c_prev → LDS
  {
    const float kp = s_keep[r];
    constexpr int NCP = PD / 8 / TPR, NCH = HD / 8 / TPR;   // 8-element chunks per thread of pre / h
    float xv[NCP][8], hv[NCH][8];
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < NCP; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xv[i][j] = xf[r * LDF + 8 * (sub + TPR * i) + j];
        amax = fmaxf(amax, fabsf(xv[i][j]));
      }
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const size_t o = (size_t)grow_r * HD + 8 * (sub + TPR * i);
      const float4 a = *reinterpret_cast<const float4*>(A.h + o), b = *reinterpret_cast<const float4*>(A.h + o + 4);
      const float4 ca = *reinterpret_cast<const float4*>(A.c + o), cb = *reinterpret_cast<const float4*>(A.c + o + 4);
      const float t[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        hv[i][j] = t[j] * kp;
        amax = fmaxf(amax, fabsf(hv[i][j]));
      }
      float* cp = cs + r * LDH + 8 * (sub + TPR * i);
      *reinterpret_cast<float4*>(cp) = make_float4(ca.x * kp, ca.y * kp, ca.z * kp, ca.w * kp);
      *reinterpret_cast<float4*>(cp + 4) = make_float4(cb.x * kp, cb.y * kp, cb.z * kp, cb.w * kp);
    }
    amax = dca::group_max<TPR>(amax);
    const float qs = amax > 0.f ? kQmax / amax : 1.f;
    if (sub == 0) s_row[1][r] = amax > 0.f ? amax / kQmax : 1.f;
#pragma unroll
    for (int i = 0; i < NCP; ++i) {
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = xv[i][j] * qs;
      *reinterpret_cast<long long*>(a8g + r * LDG + 8 * (sub + TPR * i)) = pack8(t);
    }
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = hv[i][j] * qs;
      *reinterpret_cast<long long*>(a8g + r * LDG + PD + 8 * (sub + TPR * i)) = pack8(t);
    }
  }
  __syncthreads();

  // ---- stage 3: gates (wave w: units 64w … 64w+63 = tiles 16w … 16w+15, 4 chunks of 4) + LSTM cell in LDS
  stream_gemm<4, KG / 128, 4, 2>(
      a8g, LDG, A.wg, [&](int ch, int i) { return 16 * w + 4 * ch + i; }, lane,
      [&](int ch, const f32x4 (&acc)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int col = 16 * (16 * w + 4 * ch + i) + cl;   // unit-major gate column: unit col/4, gate col%4
          const float sc = col_s[PD + col], b = col_b[PD + col];
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[i][e] * s_row[1][4 * q + e] * sc + b;
          // quad transpose: this lane takes row 4q + g (g = its gate index), the 4 gates of its unit at that row
          const int g = cl & 3;
          float G[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float sel = 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float t = dpp_quad_bcast(v[e], k);
              sel = g == e ? t : sel;
            }
            G[k] = sel;
          }
          const int row = 4 * q + g, unit = col >> 2;
          float* cp = cs + row * LDH + unit;
          const float ig = dca::sigmoidf_(G[0]), fg = dca::sigmoidf_(G[1]), gg = dca::tanhf_(G[2]),
                      og = dca::sigmoidf_(G[3]);
          const float cn = fg * *cp + ig * gg;
          hn[row * LDH + unit] = og * dca::tanhf_(cn);
          if (s_act[row] != 0.f) *cp = cn;
        }
      });
  __syncthreads();

  // ---- stage 3b: state out (coalesced rows): active → new h, c; inactive → only this step's reset
  if (row_ok) {
    const bool act = s_act[r] != 0.f;
    const float kp = s_keep[r];
    if (act || kp != 1.f) {
#pragma unroll
      for (int i = 0; i < HD / 8 / TPR; ++i) {
        const size_t o = (size_t)grow_r * HD + 8 * (sub + TPR * i);
        const float* cp = cs + r * LDH + 8 * (sub + TPR * i);
        *reinterpret_cast<float4*>(A.c + o) = *reinterpret_cast<const float4*>(cp);
        *reinterpret_cast<float4*>(A.c + o + 4) = *reinterpret_cast<const float4*>(cp + 4);
        if (act) {
          const float* hp = hn + r * LDH + 8 * (sub + TPR * i);
          *reinterpret_cast<float4*>(A.h + o) = *reinterpret_cast<const float4*>(hp);
          *reinterpret_cast<float4*>(A.h + o + 4) = *reinterpret_cast<const float4*>(hp + 4);
        } else {
          float4 a = *reinterpret_cast<const float4*>(A.h + o), b = *reinterpret_cast<const float4*>(A.h + o + 4);
          a.x *= kp; a.y *= kp; a.z *= kp; a.w *= kp; b.x *= kp; b.y *= kp; b.z *= kp; b.w *= kp;
          *reinterpret_cast<float4*>(A.h + o) = a;
          *reinterpret_cast<float4*>(A.h + o + 4) = b;
        }
      }
    }
  }

  // ---- stage 4: new h → fp8 (per-row scale) into the x image's space
  {
    constexpr int NCH = HD / 8 / TPR;
    float hv[NCH][8];
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        hv[i][j] = hn[r * LDH + 8 * (sub + TPR * i) + j];
        amax = fmaxf(amax, fabsf(hv[i][j]));
      }
    amax = dca::group_max<TPR>(amax);
    const float qs = amax > 0.f ? kQmax / amax : 1.f;
    if (sub == 0) s_row[2][r] = amax > 0.f ? amax / kQmax : 1.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = hv[i][j] * qs;
      *reinterpret_cast<long long*>(a8x + r * LDX + 8 * (sub + TPR * i)) = pack8(t);
    }
  }
  __syncthreads();

  // ---- stage 5: heads z = h·W_headsᵀ·scales + b (10 column tiles: wave w takes w and w + 8 — waves 2-7 a
  //      duplicate of their first tile as the second, whose result is dropped)
  stream_gemm<2, HD / 128, 1, 2>(
      a8x, LDX, A.wh, [&](int, int i) { return min(w + NW * i, ZD / 16 - 1); }, lane,
      [&](int, const f32x4 (&acc)[2]) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if (w + NW * i >= ZD / 16) continue;
          const int col = 16 * (w + NW * i) + cl;
          const float sc = col_s[PD + GD + col], b = col_b[PD + GD + col];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = 4 * q + e, grow = row0 + row;
            if (grow < n) A.z[(size_t)grow * ZD + col] = acc[i][e] * s_row[2][row] * sc + b;
          }
        }
      });
}


// =============================================================================================================
// fp8 entity encoder of the actor step (BASELINE config 5: the unit-type GEMMs, ≈63 % of the policy's FLOPs, on e4m3
// MFMA). Per slot row and unit u of type τ:
//   basic = relu(W1·u + b1)                 (128, fp32 VALU; K = 10 — W1 rows of the thread's 8 outputs in VGPRs)
//   emb   = (q(basic)·q(W_τ)ᵀ)·s_row·s_col + b_τ   (one v_mfma_scale_f32_16x16x128_f8f6f4 per 16×16 tile: K = 128
//                                                    is exactly one MFMA step) → bf16 (the sampling kernel's input)
//   x896[:, 128 + 128τ + j] = max over the type's units of emb[:, u, j]       (pools, bf16: the fp8 core's input)
//   x896[:, 0:128] = relu(W_env·env + b_env)
// Quantisation as in the core: basic per (row, unit) — its max maps to 448 —, W_τ per output channel at hot-swap
// time (fragment order, actor/batched.py fp8_weight). One 256-thread workgroup per 16 slots: the 16 rows' unit
// features (contiguous, fp16 from the compact staging or fp32) land in LDS once; per unit, every thread computes 8
// basic values of one row and quantises them into a double-buffered fp8 A image (one barrier per unit), then wave w
// runs the MFMAs of output tiles 2w, 2w+1 and keeps the running pool maxima in registers. Replaces the bf16 encoder
// (fp16 units are read as they are).
// buffer resource over [p, p + bytes) (wave-uniform; out-of-range accesses read 0 / are dropped)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, long long bytes) {
  const unsigned long long ad = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)ad);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(ad >> 32));
  const int nb = (int)(bytes > 0x7fff0000LL ? 0x7fff0000LL : bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(nb), 0x00020000);
}

struct EncFp8Args {
  const void* units;                     // (N, U, 10) fp16 or fp32
  const float* env;                      // (N, 3)
  const float* w1; const float* b1;      // (128, 10), (128)
  const i32x8* wt; const float* st; const float* bt;   // (6, 128, 128) e4m3 fragment order, (6, 128), (6, 128)
  const float* we; const float* be;      // (128, 3), (128)
  short* x896;                           // (N, 896) bf16
  short* emb;                            // (N, U, 128) bf16
  int N, U;
  int off[7];                            // type τ owns units off[τ] .. off[τ+1]-1
  int njob;                              // unit jobs per row block (blockIdx.y): whole types, balanced by units
  int nu[3];                             // units of job j, in increasing order (a type's units stay contiguous)
  int ul[3][64];                         // (dwords: wave-uniform scalar loads — byte entries were vector loads, and
                                         // their vmcnt(0) drained every in-flight fetch / store once per unit)
};
constexpr int EBR = 16, ENT = 256, EMAXU = 64;

// max over the 16 lanes of a DPP row (row_ror 8, 4, 2, 1: register-to-register, no LDS round trip)
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xF, 0xF, false)));
  return v;
}

template <bool F16>
__global__ __launch_bounds__(ENT) void encoder_fp8_kernel(EncFp8Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned us[];             // the 16 rows' unit features, raw bytes
  // W1ᵀ (10 × 128) and b1 in LDS (feature-major: a thread's 8 outputs of feature f are one 32-byte run). In VGPRs
  // they took 88 of the kernel's 187 registers — 2 workgroups per CU, so 768 of them ran in 1.5 rounds.
  __shared__ __attribute__((aligned(16))) float w1s[11 * 128];
  __shared__ __attribute__((aligned(16))) unsigned char aimg[2][EBR * 128];  // fp8 basic tile, double-buffered
  __shared__ float rsc[2][EBR];                                             // its row scales
  constexpr int EP = 128 + 8;                                               // emb tile pitch (bf16)
  __shared__ __attribute__((aligned(16))) short etile[2][EBR * EP];          // a unit's emb tile, bf16
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r0 = blockIdx.x * EBR, N = a.N, U = a.U, job = blockIdx.y;
  const int nrows = min(EBR, N - r0);
  {   // unit features → LDS as they are (fp16 / fp32 bytes) by LDS-DMA: every load in flight at once, one drain
      // (a convert-per-element loop waited out one memory round trip per element: most of a first version's time).
      // Rows past N read the last valid dword; their outputs are never stored.
    typedef __attribute__((address_space(1))) void gvoid;
    typedef __attribute__((address_space(3))) void lvoid;
    constexpr int ES = F16 ? 2 : 4;
    const int nd = nrows * U * 10 * ES / 4, total = EBR * U * 10 * ES / 4;    // dwords (U·10 is even)
    const unsigned* src = reinterpret_cast<const unsigned*>(static_cast<const char*>(a.units) +
                                                            (size_t)r0 * U * 10 * ES);
    for (int q0 = 64 * w; q0 < total; q0 += ENT)
      __builtin_amdgcn_global_load_lds((gvoid*)(src + min(q0 + lane, nd - 1)), (lvoid*)(us + q0), 4, 0, 0);
  }
  const int m = tid >> 4, kc = tid & 15;          // phase 1: row m, outputs 8kc … 8kc+7
  if (job == 0) {   // env embedding (job 0 of the row block): row m, 8 columns
    const int row = r0 + m;
    if (row < N) {
      const float e0 = a.env[row * 3], e1 = a.env[row * 3 + 1], e2 = a.env[row * 3 + 2];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = 8 * kc + j;
        a.x896[(size_t)row * 896 + c] = dca::f2bf(fmaxf(a.be[c] + a.we[c * 3] * e0 + a.we[c * 3 + 1] * e1 +
                                                        a.we[c * 3 + 2] * e2, 0.f));
      }
    }
  }
  for (int i = tid; i < 11 * 128; i += ENT) {
    const int f = i >> 7, c = i & 127;
    w1s[i] = f < 10 ? a.w1[c * 10 + f] : a.b1[c];
  }
  f32x4 pm[2];
  // this wave's two weight fragments of the NEXT unit's type, loaded one unit ahead (an L2 round trip per unit
  // right before its MFMAs was most of the kernel's time: 69 µs for 4096 slots)
  auto type_of = [&](int uu) {
    int t = 0;
#pragma unroll
    for (int k = 1; k < 6; ++k) t += uu >= a.off[k] ? 1 : 0;
    return t;
  };
  // Per unit, this wave's two weight fragments of the unit's type (and the lane's columns' dequant scales / biases)
  // are loaded ONE UNIT AHEAD into the other of two register sets (the loop is unrolled by two, so the sets
  // alternate without a copy; an L2 round trip right before each unit's MFMAs was most of a first version's time,
  // 69 µs for 4096 slots).
  struct WSet {
    i32x8 w[2];
    float sw[2], bb[2];
  };
  auto fetch = [&](WSet& S, int tn) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int tile = 2 * w + t, col = 16 * tile + (lane & 15);
      S.w[t] = a.wt[((size_t)tn * 8 + tile) * 64 + lane];
      S.sw[t] = a.st[tn * 128 + col];
      S.bb[t] = a.bt[tn * 128 + col];
    }
  };
  // a unit's 16 × 128 bf16 emb tile leaves through LDS as 16-byte stores (one per thread) after the NEXT unit's
  // barrier — 2-byte C-layout stores straight from the MFMA epilogue were most of the kernel's time (53 µs)
  const int srow = tid >> 4, sch = tid & 15;      // store phase: row, 16-byte chunk (8 columns)
  auto flush = [&](int u, int buf) {
    if (r0 + srow < N)
      *reinterpret_cast<uint4*>(a.emb + ((size_t)(r0 + srow) * U + u) * 128 + 8 * sch) =
          *reinterpret_cast<const uint4*>(etile[buf] + srow * EP + 8 * sch);
  };
  int prev_u = -1;
  auto unit = [&](int u, int buf, const WSet& S) {
    {   // ---- phase 1: basic of (row m, unit u), 8 outputs → e4m3 with the row's scale
      float x[10];
      if constexpr (F16) {
        const __half2* xp = reinterpret_cast<const __half2*>(us) + (m * U + u) * 5;
#pragma unroll
        for (int f = 0; f < 5; ++f) {
          const float2 t2 = __half22float2(xp[f]);
          x[2 * f] = t2.x;
          x[2 * f + 1] = t2.y;
        }
      } else {
        const float* xp = reinterpret_cast<const float*>(us) + (m * U + u) * 10;
#pragma unroll
        for (int f = 0; f < 10; ++f) x[f] = xp[f];
      }
      float v[8];
      {
        const float4* wp = reinterpret_cast<const float4*>(w1s + 8 * kc);
        const float4 b0 = wp[10 * 32], b1 = wp[10 * 32 + 1];
        v[0] = b0.x; v[1] = b0.y; v[2] = b0.z; v[3] = b0.w; v[4] = b1.x; v[5] = b1.y; v[6] = b1.z; v[7] = b1.w;
#pragma unroll
        for (int f = 0; f < 10; ++f) {
          const float4 p0 = wp[f * 32], p1 = wp[f * 32 + 1];
          v[0] = fmaf(p0.x, x[f], v[0]); v[1] = fmaf(p0.y, x[f], v[1]);
          v[2] = fmaf(p0.z, x[f], v[2]); v[3] = fmaf(p0.w, x[f], v[3]);
          v[4] = fmaf(p1.x, x[f], v[4]); v[5] = fmaf(p1.y, x[f], v[5]);
          v[6] = fmaf(p1.z, x[f], v[6]); v[7] = fmaf(p1.w, x[f], v[7]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
      }
      float am = fmaxf(fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])), fmaxf(fmaxf(v[4], v[5]), fmaxf(v[6], v[7])));
      am = row16_max(am);                        // the row's 16 threads (one DPP row)
      const float sc = am > 0.f ? am / kQmax : 1.f, inv = am > 0.f ? kQmax / am : 1.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= inv;
      *reinterpret_cast<long long*>(aimg[buf] + m * 128 + 8 * kc) = pack8(v);
      if (kc == 0) rsc[buf][m] = sc;
    }
    __syncthreads();   // A image of unit u complete (and every wave is past unit u-1's reads of the other buffer)
    if (prev_u >= 0) flush(prev_u, buf ^ 1);       // the previous unit's emb tile (written before this barrier)
    prev_u = u;
    {   // ---- phase 2: wave w → output tiles 2w, 2w + 1
      const int tau = type_of(u);
      const bool first = u == a.off[tau], last = u == a.off[tau + 1] - 1;
      const i32x8 af = afrag128(aimg[buf], 128, 0, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int tile = 2 * w + t, col = 16 * tile + (lane & 15);
        const f32x4 c = mma128(af, S.w[t], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 4 * (lane >> 4) + r;
          const float e = c[r] * rsc[buf][row] * S.sw[t] + S.bb[t];
          pm[t][r] = first ? e : fmaxf(pm[t][r], e);
          etile[buf][row * EP + col] = dca::f2bf(e);
        }
        if (last) {                                // (uniform) the type's pool → x896
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 4 * (lane >> 4) + r;
            if (r0 + row < N) a.x896[(size_t)(r0 + row) * 896 + 128 + 128 * tau + col] = dca::f2bf(pm[t][r]);
          }
        }
      }
    }
  };
  // this workgroup's units: the whole types of job `job` (several workgroups per row block shorten the serial
  // per-unit chain and let 2-3 workgroups share a CU; one type's units keep their order for the running pool)
  const int nu = a.nu[job];
  const int* ul = a.ul[job];
  WSet A, B;
  fetch(A, type_of(ul[0]));
  __builtin_amdgcn_s_waitcnt(0);                  // first fragments landed: no first-iteration waits in the loop
  __syncthreads();                                // unit features staged
  for (int i = 0; i < nu; i += 2) {
    fetch(B, type_of(ul[min(i + 1, nu - 1)]));
    unit(ul[i], i & 1, A);
    if (i + 1 < nu) {                             // (uniform)
      fetch(A, type_of(ul[min(i + 2, nu - 1)]));
      unit(ul[i + 1], (i + 1) & 1, B);
    }
  }
  __syncthreads();
  flush(prev_u, (nu - 1) & 1);                    // the last unit's tile
}

// ---------------------------------------------------------------------------------------------------------------
// Wave-parallel form of the fp8 encoder (the default): one 512-thread workgroup (8 waves) per 16 slot rows and ALL
// unit types. The row block's U units, in type order, are dealt to the 8 waves as contiguous segments (U/8 units each,
// ≤ 3 same-type runs per segment: 1v1 {1, 5, 16, 16, 1, 1} → 5 units per wave), so every wave works through its own
// units with NO per-unit workgroup barrier:
//   basic  lane l computes the 32 outputs 32(l>>4) … +31 of row l&15 (K = 10, W1ᵀ from LDS), the row's max over
//          its 4 lanes (two shuffles), e4m3 — and those 32 bytes ARE the lane's A operand of the 16x16x128 f8f6f4
//          MFMA (A[row l&15][k = 32(l>>4) + j]): no A image, no LDS round trip;
//   GEMM   8 MFMAs (the 128 output columns) against the run's type weights, held in one of two register sets (the
//          next run's set loads while the current run computes);
//   emb    dequantised in the accumulator layout, staged through the wave's own LDS tile, 16-byte row stores;
//   pools  every unit's values folded into the type's LDS pool by integer max on order-preserving keys (exact and
//          order independent across the waves sharing a type; running maxima in registers spilled), written once at
//          the end as 16-byte bf16 stores.
// The per-unit-barrier form above (one unit at a time over the whole workgroup) stays as the fallback for layouts
// whose segments would need more than 3 runs.
struct EncW8Args {
  const void* units; const float* env; const float* w1; const float* b1;
  const i32x8* wt; const float* st; const float* bt; const float* we; const float* be;
  short* x896; short* emb;
  int N, U;
  int nrun[8];                           // same-type runs of wave w's unit segment (≤ 3)
  int rt[8][3], rb[8][3], re[8][3];      // run k: type, first unit, one past the last unit
};
constexpr int EWT = 512, EWP = 136;      // threads; bf16 pitch of a wave's 16 × 128 emb tile

__device__ __forceinline__ int ord_key(float f) {     // float order as signed-int order (an involution)
  const int b = __float_as_int(f);
  return b < 0 ? b ^ 0x7fffffff : b;
}

template <bool F16>
__global__ __launch_bounds__(EWT, 1) void encoder_fp8w_kernel(EncW8Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned us[];          // the 16 rows' unit features, raw bytes
  __shared__ __attribute__((aligned(16))) float w1s[11 * 128];            // W1ᵀ (feature-major), then b1
  __shared__ float cscale[6 * 128], cbias[6 * 128];                       // W_τ dequant scales, b_τ
  __shared__ __attribute__((aligned(16))) short et[8][EBR * EWP];         // each wave's emb tile
  __shared__ __attribute__((aligned(16))) int pool[6 * EBR * 128];        // pool keys [type][row][column]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r0 = blockIdx.x * EBR, N = a.N, U = a.U;
  const int nrows = min(EBR, N - r0);
  {   // unit features → LDS by LDS-DMA (rows past N read the last valid dword; their outputs are never stored)
    typedef __attribute__((address_space(1))) void gvoid;
    typedef __attribute__((address_space(3))) void lvoid;
    constexpr int ES = F16 ? 2 : 4;
    const int nd = nrows * U * 10 * ES / 4, total = EBR * U * 10 * ES / 4;
    const unsigned* src = reinterpret_cast<const unsigned*>(static_cast<const char*>(a.units) +
                                                            (size_t)r0 * U * 10 * ES);
    for (int q0 = 64 * w; q0 < total; q0 += EWT)
      __builtin_amdgcn_global_load_lds((gvoid*)(src + min(q0 + lane, nd - 1)), (lvoid*)(us + q0), 4, 0, 0);
  }
  for (int i = tid; i < 11 * 128; i += EWT) {
    const int f = i >> 7, c = i & 127;
    w1s[i] = f < 10 ? a.w1[c * 10 + f] : a.b1[c];
  }
  for (int i = tid; i < 6 * 128; i += EWT) {
    cscale[i] = a.st[i];
    cbias[i] = a.bt[i];
  }
  for (int i = tid; i < 6 * EBR * 128; i += EWT) pool[i] = (int)0x80000000;
  {   // env embedding: row tid>>5, columns 4(tid&31) … +3
    const int row = r0 + (tid >> 5), c0 = 4 * (tid & 31);
    if (row < N) {
      const float e0 = a.env[row * 3], e1 = a.env[row * 3 + 1], e2 = a.env[row * 3 + 2];
      short o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = c0 + j;
        o[j] = dca::f2bf(fmaxf(a.be[c] + a.we[c * 3] * e0 + a.we[c * 3 + 1] * e1 + a.we[c * 3 + 2] * e2, 0.f));
      }
      *reinterpret_cast<uint2*>(a.x896 + (size_t)row * 896 + c0) =
          make_uint2((unsigned)(unsigned short)o[0] | ((unsigned)(unsigned short)o[1] << 16),
                     (unsigned)(unsigned short)o[2] | ((unsigned)(unsigned short)o[3] << 16));
    }
  }
  const int nr = a.nrun[w];
  i32x8 WA[8], WB[8];
  auto load = [&](i32x8 (&W)[8], int tau) {
#pragma unroll
    for (int t = 0; t < 8; ++t) W[t] = a.wt[((size_t)tau * 8 + t) * 64 + lane];
  };
  if (nr > 0) load(WA, a.rt[w][0]);
  if (nr > 1) load(WB, a.rt[w][1]);
  __builtin_amdgcn_s_waitcnt(0);                  // features (LDS-DMA) and the first weight sets landed
  __syncthreads();

  const int m = lane & 15, kc = lane >> 4;        // basic: row m, outputs 32kc … 32kc+31
  short* const tile = et[w];
  auto unit = [&](int u, const i32x8 (&W)[8], int tau) {
    float x[10];
    if constexpr (F16) {
      const __half2* xp = reinterpret_cast<const __half2*>(us) + (m * U + u) * 5;
#pragma unroll
      for (int f = 0; f < 5; ++f) {
        const float2 t2 = __half22float2(xp[f]);
        x[2 * f] = t2.x;
        x[2 * f + 1] = t2.y;
      }
    } else {
      const float* xp = reinterpret_cast<const float*>(us) + (m * U + u) * 10;
#pragma unroll
      for (int f = 0; f < 10; ++f) x[f] = xp[f];
    }
    const float4* wp = reinterpret_cast<const float4*>(w1s) + 8 * kc;
    float v[32];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float4 b = wp[10 * 32 + i];
      v[4 * i] = b.x; v[4 * i + 1] = b.y; v[4 * i + 2] = b.z; v[4 * i + 3] = b.w;
    }
#pragma unroll
    for (int f = 0; f < 10; ++f)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float4 p = wp[f * 32 + i];
        v[4 * i] = fmaf(p.x, x[f], v[4 * i]);
        v[4 * i + 1] = fmaf(p.y, x[f], v[4 * i + 1]);
        v[4 * i + 2] = fmaf(p.z, x[f], v[4 * i + 2]);
        v[4 * i + 3] = fmaf(p.w, x[f], v[4 * i + 3]);
      }
    float am = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      v[j] = fmaxf(v[j], 0.f);
      am = fmaxf(am, v[j]);
    }
    am = fmaxf(am, __shfl_xor(am, 16, 64));
    am = fmaxf(am, __shfl_xor(am, 32, 64));
    const float sc = am > 0.f ? am / kQmax : 1.f, inv = am > 0.f ? kQmax / am : 1.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] *= inv;
    i32x8 af;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long long p = pack8(v + 8 * q);
      af[2 * q] = (int)(unsigned)p;
      af[2 * q + 1] = (int)(unsigned)(p >> 32);
    }
    float rs[4];                                  // scales of the accumulator rows 4kc + r (lane 4kc + r has them)
#pragma unroll
    for (int r = 0; r < 4; ++r) rs[r] = __shfl(sc, 4 * kc + r, 64);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const f32x4 c = mma128(af, W[t], f32x4{0.f, 0.f, 0.f, 0.f});
      const int col = 16 * t + m;
      const float sw = cscale[tau * 128 + col], bb = cbias[tau * 128 + col];
      int* pk = pool + tau * EBR * 128 + col;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = c[r] * rs[r] * sw + bb;
        atomicMax(pk + (4 * kc + r) * 128, ord_key(e));
        tile[(4 * kc + r) * EWP + col] = dca::f2bf(e);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the wave's tile is complete (cross-lane read below)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 4 * i + kc;
      if (r0 + row < N)
        *reinterpret_cast<uint4*>(a.emb + ((size_t)(r0 + row) * U + u) * 128 + 8 * m) =
            *reinterpret_cast<const uint4*>(tile + row * EWP + 8 * m);
    }
  };
  for (int k = 0; k < nr; ++k) {                  // (wave-uniform)
    const int tau = a.rt[w][k], ub = a.rb[w][k], ue = a.re[w][k];
    if ((k & 1) == 0) {
      for (int u = ub; u < ue; ++u) unit(u, WA, tau);
      if (k + 2 < nr) load(WA, a.rt[w][k + 2]);
    } else {
      for (int u = ub; u < ue; ++u) unit(u, WB, tau);
      if (k + 2 < nr) load(WB, a.rt[w][k + 2]);
    }
  }
  __syncthreads();
  // pools → x896[:, 128 + 128τ + c], 8 columns (16 B) per store
  for (int i = tid; i < 6 * EBR * 16; i += EWT) {
    const int tau = i / (EBR * 16), rem = i - tau * EBR * 16, row = rem >> 4, ch = rem & 15;
    if (r0 + row >= N) continue;
    const int* pk = pool + (tau * EBR + row) * 128 + 8 * ch;
    unsigned o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float lo = __int_as_float(ord_key(__int_as_float(pk[2 * j])));
      const float hi = __int_as_float(ord_key(__int_as_float(pk[2 * j + 1])));
      o[j] = (unsigned)(unsigned short)dca::f2bf(lo) | ((unsigned)(unsigned short)dca::f2bf(hi) << 16);
    }
    *reinterpret_cast<uint4*>(a.x896 + (size_t)(r0 + row) * 896 + 128 + 128 * tau + 8 * ch) =
        make_uint4(o[0], o[1], o[2], o[3]);
  }
}

}  // namespace

// x896 (n,896) bf16; weights fragment-ordered fp8 (see actor/batched.py fp8_weight) with fp32 per-channel scales and
// biases: wpre (256×896), wg (2048×768, unit-major rows, [W_ih | W_hh]), wh (160×512); h, c (n,512) fp32 in place;
// keep (n), active (n or null); z (n,160) fp32.
extern "C" hipError_t dca_actor_fp8(const short* x896, const void* wpre, const float* spre, const float* bpre,
                                    const void* wg, const float* sg, const float* bg, const void* wh, const float* sh,
                                    const float* bh, float* h, float* c, const float* keep, const float* active,
                                    float* z, int n, long long* bump, hipStream_t stream) {
  if (n < 1) return hipSuccess;
  Fp8Args a{x896, reinterpret_cast<const i32x8*>(wpre), spre, bpre, reinterpret_cast<const i32x8*>(wg), sg, bg,
            reinterpret_cast<const i32x8*>(wh), sh, bh, h, c, keep, active, z, n, bump};
  hipLaunchKernelGGL(actor_fp8_kernel, dim3((n + BM - 1) / BM), dim3(NT), 0, stream, a);
  return hipGetLastError();
}

// fp8 entity encoder (actor step): units (N, U, 10) fp16 (f16 = 1) or fp32, env (N, 3); W1 (128, 10), b1; W_τ as
// (6, 128, 128) e4m3 fragment-ordered bytes with per-channel scales st (6, 128) and biases bt (6, 128); W_env (128, 3),
// b_env. Writes x896 (N, 896) bf16 (env embedding + the six pools) and emb (N, U, 128) bf16. counts: units per type.
extern "C" hipError_t dca_encoder_fp8(const void* units, int f16, const float* env, const float* w1, const float* b1,
                                      const void* wt, const float* st, const float* bt, const float* we,
                                      const float* be, short* x896, short* emb, int N, int U, const int* counts,
                                      int per_unit, hipStream_t stream) {
  if (N < 1) return hipSuccess;
  if (U < 1 || U > EMAXU) return hipErrorInvalidValue;
  if (!per_unit) {   // wave-parallel form: U units in type order as 8 contiguous segments of ≤ 3 same-type runs
    EncW8Args b{units, env, w1, b1, reinterpret_cast<const i32x8*>(wt), st, bt, we, be, x896, emb, N, U, {}, {}, {}, {}};
    int tof[EMAXU], acc = 0;
    bool ok = true;
    for (int t = 0; t < 6; ++t) {
      if (counts[t] < 1) return hipErrorInvalidValue;
      for (int j = 0; j < counts[t] && acc < EMAXU; ++j) tof[acc++] = t;
    }
    if (acc != U) return hipErrorInvalidValue;
    for (int w = 0; w < 8 && ok; ++w) {
      const int lo = w * U / 8, hi = (w + 1) * U / 8;
      b.nrun[w] = 0;
      for (int u = lo; u < hi; ++u) {
        if (u == lo || tof[u] != tof[u - 1]) {
          if (b.nrun[w] == 3) { ok = false; break; }
          const int k = b.nrun[w]++;
          b.rt[w][k] = tof[u];
          b.rb[w][k] = u;
        }
        b.re[w][b.nrun[w] - 1] = u + 1;
      }
    }
    if (ok) {
      const size_t lds = ((size_t)EBR * U * 10 * (f16 ? 2 : 4) + 15) / 16 * 16;
      const dim3 grid((N + EBR - 1) / EBR);
      if (f16) hipLaunchKernelGGL(encoder_fp8w_kernel<true>, grid, dim3(EWT), lds, stream, b);
      else hipLaunchKernelGGL(encoder_fp8w_kernel<false>, grid, dim3(EWT), lds, stream, b);
      return hipGetLastError();
    }
  }
  EncFp8Args a{units, env, w1, b1, reinterpret_cast<const i32x8*>(wt), st, bt, we, be, x896, emb, N, U, {}};
  int acc = 0;
  for (int t = 0; t < 6; ++t) {
    a.off[t] = acc;
    acc += counts[t];
    if (counts[t] < 1) return hipErrorInvalidValue;   // every type owns ≥ 1 unit slot (pools have no empty case)
  }
  a.off[6] = acc;
  if (acc != U) return hipErrorInvalidValue;
  // types → 3 jobs, largest first into the lightest job (1v1: {16}, {16}, {1, 5, 1, 1})
  int order[6] = {0, 1, 2, 3, 4, 5};
  for (int i = 0; i < 6; ++i)
    for (int j = i + 1; j < 6; ++j)
      if (counts[order[j]] > counts[order[i]]) { const int t = order[i]; order[i] = order[j]; order[j] = t; }
  int load[3] = {0, 0, 0}, owner[6];
  for (int i = 0; i < 6; ++i) {
    int b = 0;
    for (int j = 1; j < 3; ++j) if (load[j] < load[b]) b = j;
    owner[order[i]] = b;
    load[b] += counts[order[i]];
  }
  a.njob = 0;
  int remap[3] = {-1, -1, -1};
  for (int t = 0; t < 6; ++t) {                   // job ids in order of their first type; units in increasing order
    int& jb = remap[owner[t]];
    if (jb < 0) { jb = a.njob++; a.nu[jb] = 0; }
    for (int u = a.off[t]; u < a.off[t + 1]; ++u) a.ul[jb][a.nu[jb]++] = u;
  }
  const dim3 grid((N + EBR - 1) / EBR, a.njob);
  const size_t lds = ((size_t)EBR * U * 10 * (f16 ? 2 : 4) + 15) / 16 * 16;   // the staged unit features
  if (f16) hipLaunchKernelGGL(encoder_fp8_kernel<true>, grid, dim3(ENT), lds, stream, a);
  else hipLaunchKernelGGL(encoder_fp8_kernel<false>, grid, dim3(ENT), lds, stream, a);
  return hipGetLastError();
}
