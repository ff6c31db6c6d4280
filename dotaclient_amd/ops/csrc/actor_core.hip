// Actor policy core at fp32 (exact) or bf16 (gfx950 MFMA): one launch from the encoder's pooled features to the head
// logits of a batch of player slots — the reference actor's per-step policy evaluation (agent.py:641-660 →
// policy.py:135-158: pre-RNN layer, recurrent layer, the five heads) with no vendor GEMM in the step.
//
//   x896 (n, 896) f32 | bf16  ──►  pre = relu(x·W_preᵀ + b)                       (16 × 256 per workgroup)
//                           ──►  LSTM: gates = [pre | keep·h]·[W_ih | W_hh]ᵀ + b  (16 × 4H, unit-major gate columns)
//                                      → cell (c, h fp32 state in place, resets / inactive slots)
//                                linear (the reference's fake_rnn, policy.py:67-68, 143-145): h = pre·W_fᵀ + b
//                           ──►  z = h·W_headsᵀ + b                               (16 × 160 → the sampling kernel)
//
// MODE 0 — IEEE fp32: every product an fp32 FMA on v_mfma_f32_16x16x4_f32 (the reference actor's torch fp32
// nn.Linear / nn.LSTM precision), fp32 A images in LDS, fp32 weights. MODE 1 — bf16 operands on
// v_mfma_f32_16x16x32_bf16, fp32 accumulation, fp32 state (the default actor step; replaces 3 hipBLASLt GEMMs + the
// state-prep and cell launches).
//
// Layout (actor_fp8.hip's structure): one 512-thread workgroup (8 waves) per 16 slots; weights in MFMA FRAGMENT ORDER
// [col tile][k-group][lane][16 B] so a wave's k-group load is 1 KB contiguous, streamed from L2 through a register
// ring per wave (no LDS staging: every workgroup reads each weight once); activations as padded row-major LDS images
// (row pitch ≡ 8 dwords mod 64: the 16-lane groups of the ds_read_b128 fragment reads hit 16 distinct bank slots).
// A k-group is 16 deep at fp32 (lane l holds k = 16g + 4(l>>4) + j, j < 4: four chained 16x16x4 MFMAs, call j taking
// element j of A and B alike — the product is the sum over k whatever MFMA a k lands in) and 32 deep at bf16 (lane l:
// k = 32g + 8(l>>4) + j, one 16x16x32 MFMA). The cell's four gates of a (row, unit) sit in four adjacent lanes of the
// C layout (unit-major columns); a quad transpose by DPP broadcasts hands each lane one (row, unit). Activations: the
// hardware exp / reciprocal forms (the learner's recurrence uses the same).
//
// Resources: ≤ 148 KB LDS (fp32, H = 512), 512 threads, ≤ 128 VGPRs (launch_bounds 512, 2 → the step's waves fit
// beside a resident learner recurrence wave on each SIMD).
#include "common.h"

namespace {

using dca::bf16x8;
using dca::f32x4;

constexpr int BM = 16, NT = 512, NW = NT / 64, TPR = NT / BM;    // 8 waves; 32 staging threads per row
constexpr int XD = 896, PD = 256, ZD = 160;

template <int MODE>
struct Mma;
template <>
struct Mma<0> {                                  // exact fp32: 16-deep k-group = 4 chained 16x16x4 MFMAs
  static constexpr int KG = 16, ES = 4;
  typedef float T;
  __device__ static __forceinline__ f32x4 run(const uint4& a, const uint4& b, f32x4 c) {
    const float4 af = __builtin_bit_cast(float4, a), bf = __builtin_bit_cast(float4, b);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(af.x, bf.x, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(af.y, bf.y, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(af.z, bf.z, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(af.w, bf.w, c, 0, 0, 0);
    return c;
  }
  __device__ static __forceinline__ void put(void* img, int pitch, int r, int k, float v) {
    static_cast<float*>(img)[r * pitch + k] = v;
  }
};
template <>
struct Mma<1> {                                  // bf16: 32-deep k-group = one 16x16x32 MFMA
  static constexpr int KG = 32, ES = 2;
  typedef short T;
  __device__ static __forceinline__ f32x4 run(const uint4& a, const uint4& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  }
  __device__ static __forceinline__ void put(void* img, int pitch, int r, int k, float v) {
    static_cast<short*>(img)[r * pitch + k] = dca::f2bf(v);
  }
};

// padded row pitch (elements): ≡ 8 dwords mod 64 (conflict-free ds_read_b128 fragment reads, see the header)
template <int MODE>
constexpr int pitch(int k) { return MODE == 0 ? k + 8 : k + 16; }

// A fragment of k-group u from an LDS image: lane l holds row l & 15, 16 B at k = KG·u + (KG/4)·(l >> 4)
template <int MODE>
__device__ __forceinline__ uint4 afrag(const char* img, int pitch_bytes, int u, int lane) {
  return *reinterpret_cast<const uint4*>(img + (lane & 15) * pitch_bytes + 64 * u + 16 * (lane >> 4));
}

// Streamed weight GEMM (actor_fp8.hip stream_gemm): NCH chunks of NTL column tiles (`tile(ch, i)`), each over KU
// k-groups; ONE D-deep register ring of weight fragments runs across the chunk boundaries; the epilogue `epi(ch, acc)`
// runs after a chunk's last k-group and must not touch global memory (the ring's loads share the in-order vmcnt).
template <int MODE, int NTL, int KU, int NCH, int D, class TileFn, class Epi>
__device__ __forceinline__ void stream_gemm(const char* aimg, int pitch_bytes, const uint4* __restrict__ w,
                                            TileFn tile, int lane, Epi epi) {
  constexpr int T = NCH * KU;
  uint4 ring[D][NTL];
  f32x4 acc[NTL];
#pragma unroll
  for (int i = 0; i < NTL; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto issue = [&](int slot, int t) {
    t = t < T ? t : T - 1;                       // past the end: reload the last group (never consumed)
    const int ch = t / KU, u = t - ch * KU;
#pragma unroll
    for (int i = 0; i < NTL; ++i) ring[slot][i] = w[((size_t)tile(ch, i) * KU + u) * 64 + lane];
  };
#pragma unroll
  for (int d = 0; d < D; ++d) issue(d, d);
  for (int t0 = 0; t0 < T; t0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int t = t0 + d;
      if (t >= T) break;
      const int ch = t / KU, u = t - ch * KU;
      const uint4 a = afrag<MODE>(aimg, pitch_bytes, u, lane);
#pragma unroll
      for (int i = 0; i < NTL; ++i) acc[i] = Mma<MODE>::run(a, ring[d][i], acc[i]);
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

struct CoreArgs {
  const void* x896;                      // (n, 896) f32 or bf16
  const uint4* wpre; const float* bpre;  // 256 × 896, fragment order
  const uint4* wg; const float* bg;      // LSTM: 4H × (256 + H) unit-major rows [W_ih | W_hh]; linear: H × 256
  const uint4* wh; const float* bh;      // 160 × H heads
  float* h; float* c;                    // (n, H) fp32 state, in place (c unused by the linear layer)
  const float* keep; const float* active;
  float* z;                              // (n, 160) fp32
  int n;
  long long* bump;                       // the sampler's step counter, += 1 here (null: the caller bumps it)
};

// MODE 0 fp32 / 1 bf16 operands; XF32: x896 arrives fp32 (else bf16); H hidden width; LIN: linear recurrent layer
template <int MODE, bool XF32, int H, bool LIN>
__global__ __launch_bounds__(NT, 2) void actor_core_kernel(CoreArgs A) {
  using M = Mma<MODE>;
  using AT = typename M::T;
  constexpr int KG = M::KG, ES = M::ES;
  constexpr int GK = LIN ? PD : PD + H;          // K of the recurrent product
  constexpr int GN = LIN ? H : 4 * H;            // its output columns
  constexpr int LX = pitch<MODE>(XD), LG = pitch<MODE>(GK), LHB = pitch<MODE>(H);
  constexpr int LH = H + 8;                      // fp32 h / c rows (pitch ≡ 8 mod 64 dwords)
  // LDS: x image | g image | c | h | bias. The x image is dead after stage 1: fp32 keeps the new h (the heads' A
  // image) over it, bf16 the heads' bf16 image (its fp32 h has a region of its own)
  constexpr int OX = 0, SX = BM * LX * ES;
  constexpr int OG = OX + ((SX + 15) & ~15), SG = BM * LG * ES;
  constexpr int OC = OG + ((SG + 15) & ~15), SC = LIN ? 0 : BM * LH * 4;
  constexpr int SH = BM * LH * 4;
  constexpr int OH = MODE == 0 ? OX : OC + SC;
  constexpr int OB = MODE == 0 ? OC + SC : OH + SH, NB = PD + GN + ZD;
  static_assert(MODE == 1 || SH <= SX, "the fp32 h must fit the x image");
  constexpr int BYTES = OB + NB * 4;
  static_assert(BYTES <= 160 * 1024, "LDS budget");
  static_assert(BM * LHB * ES <= SX, "the bf16 heads image must fit the x image");
  __shared__ __attribute__((aligned(16))) char lds[BYTES];
  __shared__ float s_keep[BM], s_act[BM];
  char* ximg = lds + OX;
  char* gimg = lds + OG;
  float* cs = reinterpret_cast<float*>(lds + OC);
  float* hn = reinterpret_cast<float*>(lds + OH);
  float* col_b = reinterpret_cast<float*>(lds + OB);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  if (A.bump && blockIdx.x == 0 && tid == 0) A.bump[0] += 1;
  const int q = lane >> 4, cl = lane & 15;
  const int row0 = blockIdx.x * BM, n = A.n;
  const int r = tid / TPR, sub = tid % TPR;      // staging: TPR threads per row
  const int grow_r = min(row0 + r, n - 1);
  const bool row_ok = row0 + r < n;

  // ---- stage 0: biases; keep / active; the x896 rows → A image
  for (int i = tid; i < NB; i += NT) {
    const bool p = i < PD, g = !p && i < PD + GN;
    col_b[i] = p ? A.bpre[i] : (g ? A.bg[i - PD] : A.bh[i - PD - GN]);
  }
  if (sub == 0) {
    s_keep[r] = A.keep[grow_r];
    s_act[r] = (A.active == nullptr || A.active[grow_r] != 0.f) ? 1.f : 0.f;
  }
  for (int ch = sub; ch < XD / 8; ch += TPR) {   // 8-element chunks of the row
    float v[8];
    if constexpr (XF32) {
      const float* xr = static_cast<const float*>(A.x896) + (size_t)grow_r * XD + 8 * ch;
      const float4 a = *reinterpret_cast<const float4*>(xr), b = *reinterpret_cast<const float4*>(xr + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(static_cast<const short*>(A.x896) + (size_t)grow_r * XD + 8 * ch);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = dca::bf2f(b[j]);
    }
    if constexpr (MODE == 0) {
      float* d = reinterpret_cast<float*>(ximg) + r * LX + 8 * ch;
      *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(d + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = dca::f2bf(v[j]);
      *reinterpret_cast<bf16x8*>(reinterpret_cast<short*>(ximg) + r * LX + 8 * ch) = o;
    }
  }
  // keep·h_prev → the g image's h columns, keep·c_prev → c (LSTM)
  if constexpr (!LIN) {
    const float kp = A.keep[grow_r];
    for (int ch = sub; ch < H / 4; ch += TPR) {
      const size_t o = (size_t)grow_r * H + 4 * ch;
      const float4 hv = *reinterpret_cast<const float4*>(A.h + o), cv = *reinterpret_cast<const float4*>(A.c + o);
      *reinterpret_cast<float4*>(cs + r * LH + 4 * ch) = make_float4(cv.x * kp, cv.y * kp, cv.z * kp, cv.w * kp);
      const float t[4] = {hv.x * kp, hv.y * kp, hv.z * kp, hv.w * kp};
#pragma unroll
      for (int j = 0; j < 4; ++j) M::put(gimg, LG, r, PD + 4 * ch + j, t[j]);
    }
  }
  __syncthreads();

  // ---- stage 1: pre = relu(x·W_preᵀ + b) straight into the g image's first 256 columns; wave w: tiles 2w, 2w+1
  stream_gemm<MODE, 2, XD / KG, 1, 4>(
      ximg, LX * ES, A.wpre, [&](int, int i) { return 2 * w + i; }, lane, [&](int, const f32x4 (&acc)[2]) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int col = 16 * (2 * w + i) + cl;
          const float b = col_b[col];
#pragma unroll
          for (int e = 0; e < 4; ++e) M::put(gimg, LG, 4 * q + e, col, fmaxf(acc[i][e] + b, 0.f));
        }
      });
  __syncthreads();

  // ---- stage 2: the recurrent layer; wave w owns TPW consecutive column tiles, NTL per chunk
  constexpr int TPW = GN / 16 / NW, NTL = TPW < 4 ? TPW : 4, NCH = TPW / NTL;
  static_assert(TPW * 16 * NW == GN && NCH * NTL == TPW, "recurrent tiles per wave");
  stream_gemm<MODE, NTL, GK / KG, NCH, 2>(
      gimg, LG * ES, A.wg, [&](int ch, int i) { return TPW * w + NTL * ch + i; }, lane,
      [&](int ch, const f32x4 (&acc)[NTL]) {
#pragma unroll
        for (int i = 0; i < NTL; ++i) {
          const int col = 16 * (TPW * w + NTL * ch + i) + cl;
          const float b = col_b[PD + col];
          if constexpr (LIN) {
#pragma unroll
            for (int e = 0; e < 4; ++e) hn[(4 * q + e) * LH + col] = acc[i][e] + b;   // fake_rnn: no activation
          } else {
            // unit-major gate column: unit col/4, gate col%4; quad transpose: this lane takes row 4q + g (g = its
            // gate index) with the 4 gates of its unit at that row
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[i][e] + b;
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
            float* cp = cs + row * LH + unit;
            const float ig = dca::sigmoidf_(G[0]), fg = dca::sigmoidf_(G[1]), gg = dca::tanhf_(G[2]),
                        og = dca::sigmoidf_(G[3]);
            const float cn = fg * *cp + ig * gg;
            hn[row * LH + unit] = og * dca::tanhf_(cn);
            if (s_act[row] != 0.f) *cp = cn;
          }
        }
      });
  __syncthreads();

  // ---- stage 3: state out (coalesced rows): active → new h (, c); inactive → only this step's reset
  if (row_ok) {
    const bool act = s_act[r] != 0.f;
    const float kp = s_keep[r];
    if (act || kp != 1.f) {
      for (int ch = sub; ch < H / 4; ch += TPR) {
        const size_t o = (size_t)grow_r * H + 4 * ch;
        if constexpr (!LIN) *reinterpret_cast<float4*>(A.c + o) = *reinterpret_cast<const float4*>(cs + r * LH + 4 * ch);
        float4 hv;
        if (act) {
          hv = *reinterpret_cast<const float4*>(hn + r * LH + 4 * ch);
        } else {
          hv = *reinterpret_cast<const float4*>(A.h + o);
          hv.x *= kp; hv.y *= kp; hv.z *= kp; hv.w *= kp;
        }
        *reinterpret_cast<float4*>(A.h + o) = hv;
      }
    }
  }
  // bf16: the new h → the heads' bf16 image (over the x image, dead since stage 1); fp32: hn IS the A image
  if constexpr (MODE == 1) {
    for (int ch = sub; ch < H / 8; ch += TPR) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = dca::f2bf(hn[r * LH + 8 * ch + j]);
      *reinterpret_cast<bf16x8*>(reinterpret_cast<short*>(ximg) + r * LHB + 8 * ch) = o;
    }
    __syncthreads();
  }

  // ---- stage 4: heads z = h·W_headsᵀ + b (10 column tiles: wave w takes w and w + 8 — waves 2-7 a duplicate of
  //      their first tile as the second, whose result is dropped)
  const char* himg = MODE == 1 ? ximg : reinterpret_cast<const char*>(hn);
  constexpr int HP = MODE == 1 ? LHB * ES : LH * 4;
  stream_gemm<MODE, 2, H / KG, 1, 4>(
      himg, HP, A.wh, [&](int, int i) { return min(w + NW * i, ZD / 16 - 1); }, lane,
      [&](int, const f32x4 (&acc)[2]) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if (w + NW * i >= ZD / 16) continue;
          const int col = 16 * (w + NW * i) + cl;
          const float b = col_b[PD + GN + col];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int grow = row0 + 4 * q + e;
            if (grow < n) A.z[(size_t)grow * ZD + col] = acc[i][e] + b;
          }
        }
      });
}

}  // namespace

// mode 0 fp32 / 1 bf16 weights (fragment order, see actor/batched.py frag_weights); x_f32: x896 dtype; hidden ∈
// {128, 256, 512}; linear: the fake_rnn layer (hidden 256) instead of the LSTM cell.
extern "C" hipError_t dca_actor_core(const void* x896, int x_f32, const void* wpre, const float* bpre, const void* wg,
                                     const float* bg, const void* wh, const float* bh, float* h, float* c,
                                     const float* keep, const float* active, float* z, int n, int hidden, int linear,
                                     int mode, long long* bump, hipStream_t st) {
  if (n < 1 || mode < 0 || mode > 1) return hipErrorInvalidValue;
  CoreArgs a{x896, static_cast<const uint4*>(wpre), bpre, static_cast<const uint4*>(wg), bg,
             static_cast<const uint4*>(wh), bh, h, c, keep, active, z, n, bump};
  const dim3 grid((n + BM - 1) / BM), block(NT);
#define DCA_CORE(MD, XF, HH, LN) hipLaunchKernelGGL((actor_core_kernel<MD, XF, HH, LN>), grid, block, 0, st, a)
#define DCA_CORE_H(MD, XF)                                                   \
  if (linear) {                                                              \
    if (hidden != 256) return hipErrorInvalidValue;                          \
    DCA_CORE(MD, XF, 256, true);                                             \
  } else if (hidden == 512) DCA_CORE(MD, XF, 512, false);                    \
  else if (hidden == 128) DCA_CORE(MD, XF, 128, false);                      \
  else return hipErrorInvalidValue;
  if (mode == 0) {
    if (!x_f32) return hipErrorInvalidValue;       // the fp32 step takes the exact encoder's fp32 features
    DCA_CORE_H(0, true)
  } else if (x_f32) {
    DCA_CORE_H(1, true)
  } else {
    DCA_CORE_H(1, false)
  }
#undef DCA_CORE_H
#undef DCA_CORE
  return hipGetLastError();
}
