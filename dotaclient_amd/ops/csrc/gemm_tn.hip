// Split-K "TN" GEMM for the learner's weight gradients (gfx950 MFMA): C[M×N] (+)= Aᵀ·B with
//   A (K×M) bf16 row-major (row stride lda) — e.g. ∂gates (B·S rows × 4H),
//   B (K×N) bf16 row-major (row stride ldb) — e.g. h_{t-1} / x (B·S rows × H),
// i.e. both operands are K-OUTER: the reduction runs over the B·S = 11 200 rows of a minibatch. hipBLASLt picks a
// 64×64 tile with no split-K for these (24-256 workgroups, 23-280 TF/s, ≈80 µs each); here:
//
// * 128×128 output tile per 256-thread workgroup (4 waves as 2×2, each 64×64 = 4×4 v_mfma_f32_16x16x32_bf16 tiles);
// * the K range is split over workgroups (≈256-512 workgroups in flight), each stages 64-row K slabs of A and B
//   through LDS (double-buffered, coalesced 16-B global loads of whole 256-B rows) and feeds the MFMAs with
//   ds_read_b64_tr_b16 transposed reads — the operands are stored [k][m] / [k][n] and the MFMA wants k-contiguous
//   fragments, the hardware transpose read gives exactly that (cdna_hip_programming.md T10);
// * LDS image swizzle off(row, ch) = 256·row + 16·(ch ^ (((row&3)<<2) | ((row>>2)&3))) (T10 layout (b)): the two
//   16-lane groups of a half read rows 8 apart in the same columns — conflict-free;
// * split-K partials go to an fp32 slab; a second, fully parallel launch sums the slabs in fixed order
//   (deterministic) and writes C, optionally through a row permutation (unit-major → PyTorch gate-major rows) and
//   optionally accumulating into C (the flat grad). (Summing in the last-arriving workgroup of each tile was 5-10×
//   slower: one workgroup's serial, latency-bound pass over all slabs of its tile.)
// * Staging the slabs by LDS-DMA (global_load_lds_dwordx4 with the swizzle applied on the source side, the bias
//   column sum as an extra MFMA against ones) measured SLOWER here: 57 / 33 / 23 / 18 µs vs 47 / 29 / 21 / 15 µs for
//   the four 1v1 weight gradients (the register-staged loads overlap the MFMAs better at this K-slab depth).
// * B may be "row-split": rows k < split come from B0 (e.g. h0), rows ≥ split from B shifted by `split` rows —
//   the LSTM's h_{t-1} operand without materialising the concatenation.
// * fp32 operands (the learner's fp32-accurate mode): "bf16x3" — every value is split once while staging, x = hi +
//   lo (two bf16), into a hi and a lo LDS image, and Aᵀ·B ≈ hiᵀ·hi + loᵀ·hi + hiᵀ·lo on the bf16 MFMA (the dropped
//   lo·lo term and the lo rounding are ≈2⁻¹⁶ relative per product; fp32 accumulation). 3× the bf16 MFMA work is
//   still ≈5× the exact-f32 MFMA rate (v_mfma_f32_16x16x4_f32 runs at 1/16 of bf16). 32-row K slabs keep the four
//   images of a stage within the bf16 kernel's 64 KB of LDS.
#include "common.h"
#include <cstdlib>

namespace {

using dca::bf16x8;
using dca::f32x4;
typedef short bf16x4v __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int kThreads = 256;
constexpr int kTileBytes = BK * 128 * 2;             // one operand stage: 64 rows × 256 B = 16 KB

__device__ __forceinline__ int lds_off(int row, int ch) {   // byte offset of 16-B chunk ch of row
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

// Buffer resource over [p, p + bytes) from wave-uniform values. The staging loads are raw buffer loads with the
// hardware bounds check standing in for the K / M / N edge tests: an out-of-range chunk gets an offset past the end and
// reads 0. (With if-guarded loads the compiler merged each guarded value with its zero default right after the
// load, i.e. waited for every slab load where it was issued instead of behind the MFMAs.)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, long long bytes) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int nb = (int)(bytes < 0 ? 0 : (bytes > 0x7fff0000LL ? 0x7fff0000LL : bytes));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(nb), 0x00020000);
}
constexpr int kOob = 0x7fff8000;   // byte offset past every operand (≤ 0x7fff0000 bytes)

__device__ __forceinline__ uint4 bload16(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

struct Args {
  const void* A; int lda;
  const void* B; int ldb;
  const void* B0; int split;
  float* C; int ldc;
  const int* perm;      // optional output row map (C row perm[m] receives result row m)
  float* slab;          // [splits][M][N] fp32 partials (splits > 1), then [splits][M] column-sum partials
  float* colsum;        // optional: colsum[m] (+)= Σ_k A[k][m] (a bias gradient), computed by the tn == 0 tiles
  int M, N, K, kc, splits, tiles_n, accumulate;
  unsigned* tickets;    // exact kernel, splits > 1: per-tile arrival counters (self-cleaning) — the last workgroup of a
                        // tile sums its slabs in split order (no separate reduce launch); nullptr: gemm_tn_reduce
  int xcd_remap;        // tile_split(): XCD-aware id map (default; DCA_GEMM_XCD=0: the plain map, A/B)
};

struct Rsrc {
  __amdgpu_buffer_rsrc_t A, B, B0;
};

// operand byte counts: A has K rows, B K - split rows, B0 split rows (row strides lda / ldb, es-byte elements)
__device__ __forceinline__ Rsrc make_rsrc(const Args& a, int es) {
  Rsrc r;
  r.A = uniform_rsrc(a.A, ((long long)(a.K - 1) * a.lda + a.M) * es);
  r.B = uniform_rsrc(a.B, a.K > a.split ? ((long long)(a.K - a.split - 1) * a.ldb + a.N) * es : 0);
  r.B0 = uniform_rsrc(a.B0 ? a.B0 : a.B, a.split > 0 ? ((long long)(a.split - 1) * a.ldb + a.N) * es : 0);
  return r;
}

// ---- bf16 operands: 64-row K slabs, one image per operand -------------------------------------------------------
template <bool WITH_B0>
__device__ __forceinline__ void load_stage(const Args& a, const Rsrc& R, int kbase, int kend, int m_base, int n_base,
                                           uint4 (&ra)[4], uint4 (&rb)[4]) {
  const int t = threadIdx.x, ch = t & 15;
  const int m = m_base + ch * 8, n = n_base + ch * 8;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = kbase + (t >> 4) + 16 * i;
    const bool kin = k < kend;
    ra[i] = bload16(R.A, kin && m < a.M ? (k * a.lda + m) * 2 : kOob);
    rb[i] = bload16(R.B, kin && n < a.N && k >= a.split ? ((k - a.split) * a.ldb + n) * 2 : kOob);
  }
  if (WITH_B0 && kbase < a.split) {   // the slab holding B0's rows (the LSTM's h0): a split-K chunk's first slab
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = kbase + (t >> 4) + 16 * i;
      const uint4 v = bload16(R.B0, k < kend && n < a.N && k < a.split ? (k * a.ldb + n) * 2 : kOob);
      rb[i] = make_uint4(rb[i].x | v.x, rb[i].y | v.y, rb[i].z | v.z, rb[i].w | v.w);
    }
  }
}

__device__ __forceinline__ void store_stage(char* As, char* Bs, const uint4 (&ra)[4], const uint4 (&rb)[4]) {
  const int t = threadIdx.x, ch = t & 15;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (t >> 4) + 16 * i;
    *reinterpret_cast<uint4*>(As + lds_off(r, ch)) = ra[i];
    *reinterpret_cast<uint4*>(Bs + lds_off(r, ch)) = rb[i];
  }
}

// running per-thread sums of the 8 A columns this thread stages (ch·8 … ch·8+7), for the optional column sum
__device__ __forceinline__ void colsum_acc(float (&cs)[8], const uint4 (&ra)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const unsigned w[4] = {ra[i].x, ra[i].y, ra[i].z, ra[i].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cs[2 * j] += __uint_as_float(w[j] << 16);
      cs[2 * j + 1] += __uint_as_float(w[j] & 0xffff0000u);
    }
  }
}

// ---- fp32 operands ("bf16x3": x = hi + lo, Aᵀ·B ≈ hiᵀhi + loᵀhi + hiᵀlo, ≈2⁻¹⁶ relative per product, f32
// accumulation): 32-row K slabs, every fp32 value split once while staging into a hi and a lo image ---------------
struct F32Stage {
  float4 a[2][2], b[2][2];   // [row i][half]: 8 consecutive columns of one K row
};

template <bool WITH_B0>
__device__ __forceinline__ void load_stage_f32(const Args& a, const Rsrc& R, int kbase, int kend, int m_base,
                                               int n_base, F32Stage& r) {
  const int t = threadIdx.x, ch = t & 15;
  const int m = m_base + ch * 8, n = n_base + ch * 8;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int k = kbase + (t >> 4) + 16 * i;
    const bool kin = k < kend;
    const int oa = kin && m < a.M ? (k * a.lda + m) * 4 : kOob;
    const int ob = kin && n < a.N && k >= a.split ? ((k - a.split) * a.ldb + n) * 4 : kOob;
    r.a[i][0] = __builtin_bit_cast(float4, bload16(R.A, oa));
    r.a[i][1] = __builtin_bit_cast(float4, bload16(R.A, oa + 16));
    r.b[i][0] = __builtin_bit_cast(float4, bload16(R.B, ob));
    r.b[i][1] = __builtin_bit_cast(float4, bload16(R.B, ob + 16));
  }
  // the slab holding B0's rows: only a split-K chunk's first slab (the host keeps split ≤ the slab depth), loaded
  // in the prologue; the main-loop loads never take this branch, so their results need no merge (which would wait)
  if (WITH_B0 && kbase < a.split) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = kbase + (t >> 4) + 16 * i;
      const int o0 = k < kend && n < a.N && k < a.split ? (k * a.ldb + n) * 4 : kOob;
      const float4 p = __builtin_bit_cast(float4, bload16(R.B0, o0));
      const float4 q = __builtin_bit_cast(float4, bload16(R.B0, o0 + 16));
      r.b[i][0] = make_float4(r.b[i][0].x + p.x, r.b[i][0].y + p.y, r.b[i][0].z + p.z, r.b[i][0].w + p.w);
      r.b[i][1] = make_float4(r.b[i][1].x + q.x, r.b[i][1].y + q.y, r.b[i][1].z + q.z, r.b[i][1].w + q.w);
    }
  }
}

__device__ __forceinline__ unsigned pack_bf2(float x, float y) {
  return (unsigned)(unsigned short)dca::f2bf(x) | ((unsigned)(unsigned short)dca::f2bf(y) << 16);
}

// 8 floats → (hi, lo) bf16 chunks
__device__ __forceinline__ void split8(const float4& p, const float4& q, uint4& hi, uint4& lo) {
  const float v[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
  float l[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) l[j] = v[j] - dca::bf2f(dca::f2bf(v[j]));
  hi = make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7]));
  lo = make_uint4(pack_bf2(l[0], l[1]), pack_bf2(l[2], l[3]), pack_bf2(l[4], l[5]), pack_bf2(l[6], l[7]));
}

// images of one stage: A hi | A lo | B hi | B lo, 32 rows × 256 B each
constexpr int kImgF32 = 32 * 256;
__device__ __forceinline__ void store_stage_f32(char* S, const F32Stage& r) {
  const int t = threadIdx.x, ch = t & 15;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (t >> 4) + 16 * i;
    uint4 hi, lo;
    split8(r.a[i][0], r.a[i][1], hi, lo);
    *reinterpret_cast<uint4*>(S + lds_off(row, ch)) = hi;
    *reinterpret_cast<uint4*>(S + kImgF32 + lds_off(row, ch)) = lo;
    split8(r.b[i][0], r.b[i][1], hi, lo);
    *reinterpret_cast<uint4*>(S + 2 * kImgF32 + lds_off(row, ch)) = hi;
    *reinterpret_cast<uint4*>(S + 3 * kImgF32 + lds_off(row, ch)) = lo;
  }
}

__device__ __forceinline__ void colsum_acc_f32(float (&cs)[8], const F32Stage& r) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    cs[0] += r.a[i][0].x; cs[1] += r.a[i][0].y; cs[2] += r.a[i][0].z; cs[3] += r.a[i][0].w;
    cs[4] += r.a[i][1].x; cs[5] += r.a[i][1].y; cs[6] += r.a[i][1].z; cs[7] += r.a[i][1].w;
  }
}

// 16x16x32 operand fragment (k = 8·(lane>>4) + j, column c0 + (lane&15)) from a [k][128] swizzled image via two
// transposed reads (rows k0 + 8g + 4r + q, columns c0 + 4p … 4p+3).
__device__ __forceinline__ bf16x8 frag_tr(const char* img, int k0, int c0) {
  const int l = threadIdx.x & 63, g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const int ch = (c0 >> 3) + (p >> 1);
  const int row0 = k0 + 8 * g + q;
  typedef __attribute__((address_space(3))) bf16x4v lds_v4;
  const bf16x4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_v4*)(img + lds_off(row0, ch) + 8 * (p & 1)));
  const bf16x4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_v4*)(img + lds_off(row0 + 4, ch) + 8 * (p & 1)));
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

// XCD-aware (tile, split) of this workgroup (1-D grid of tiles × splits). Workgroups are dispatched round-robin over
// the 8 XCDs (each with its own L2): with the plain id → (tile, split) map the M-tiles of one K split — which read the
// SAME B rows (the 5v5 ∂W_qkv: 3 M-tiles over 716 800 × 128 fp32 Xn rows) and, for wide outputs, the same A rows —
// land on different XCDs and each fetch them from HBM. The bijective remap (q = n/8, r = n%8) gives every XCD a
// contiguous id range, so a split's tiles run side by side on one XCD and share its L2.
__device__ __forceinline__ void tile_split(const Args& a, int& tile, int& split) {
  const int tiles = ((a.M + BM - 1) / BM) * a.tiles_n;
  const int n = gridDim.x, orig = blockIdx.x;
  const int q = n >> 3, r = n & 7, x = orig & 7;
  const int id = a.xcd_remap ? (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (orig >> 3) : orig;
  tile = id % tiles;
  split = id / tiles;
}

template <bool F32>
__global__ __launch_bounds__(kThreads) void gemm_tn_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BKx = F32 ? 32 : BK;
  // bf16: [A0 | A1 | B0 | B1] 16 KB images; F32: [stage0: Ahi Alo Bhi Blo | stage1: …] 8 KB images
#define AS(b) (smem + (b) * kTileBytes)
#define BS(b) (smem + (2 + (b)) * kTileBytes)
#define SF(b) (smem + (b) * 4 * kImgF32)
  int tile, split;
  tile_split(a, tile, split);
  const int tm = tile / a.tiles_n, tn = tile % a.tiles_n;
  const int m_base = tm * BM, n_base = tn * BN;
  const int k_lo = split * a.kc, k_hi = min(a.K, k_lo + a.kc);
  const int w = threadIdx.x >> 6, wm = w & 1, wn = w >> 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[4], rb[4];
  F32Stage rf;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool do_cs = a.colsum != nullptr && tn == 0;
  int buf = 0;
  const Rsrc R = make_rsrc(a, F32 ? 4 : 2);
  if (k_lo < k_hi) {
    if constexpr (F32) {
      load_stage_f32<true>(a, R, k_lo, k_hi, m_base, n_base, rf);
      store_stage_f32(SF(0), rf);
      if (do_cs) colsum_acc_f32(cs, rf);
    } else {
      load_stage<true>(a, R, k_lo, k_hi, m_base, n_base, ra, rb);
      store_stage(AS(0), BS(0), ra, rb);
      if (do_cs) colsum_acc(cs, ra);
    }
  }
  __syncthreads();
  for (int kb = k_lo; kb < k_hi; kb += BKx) {
    const bool more = kb + BKx < k_hi;
    if constexpr (F32) {
      if (more) load_stage_f32<false>(a, R, kb + BKx, k_hi, m_base, n_base, rf);   // in flight during the MFMAs
      const char* S = SF(buf);
      bf16x8 fah[4], fal[4], fbh[4], fbl[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fah[i] = frag_tr(S, 0, wm * 64 + i * 16);
        fal[i] = frag_tr(S + kImgF32, 0, wm * 64 + i * 16);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        fbh[j] = frag_tr(S + 2 * kImgF32, 0, wn * 64 + j * 16);
        fbl[j] = frag_tr(S + 3 * kImgF32, 0, wn * 64 + j * 16);
      }
      // small terms first, the hi·hi product last (16 independent accumulators interleave the chains)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fal[i], fbh[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fah[i], fbl[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fah[i], fbh[j], acc[i][j], 0, 0, 0);
      if (more) {
        store_stage_f32(SF(buf ^ 1), rf);
        if (do_cs) colsum_acc_f32(cs, rf);
      }
    } else {
      if (more) load_stage<false>(a, R, kb + BK, k_hi, m_base, n_base, ra, rb);   // in flight during the MFMAs
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        bf16x8 fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = frag_tr(AS(buf), ks * 32, wm * 64 + i * 16);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = frag_tr(BS(buf), ks * 32, wn * 64 + j * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
      if (more) {
        store_stage(AS(buf ^ 1), BS(buf ^ 1), ra, rb);
        if (do_cs) colsum_acc(cs, ra);
      }
    }
    __syncthreads();
    buf ^= 1;
  }
  if (do_cs) {       // 16 row groups share each column chunk: fixed-order LDS fold, then one value per column
    float* red = reinterpret_cast<float*>(smem);       // [16][128] (the LDS images are dead after the barrier)
    const int t = threadIdx.x, ch = t & 15, rg = t >> 4;
#pragma unroll
    for (int j = 0; j < 8; ++j) red[rg * 128 + ch * 8 + j] = cs[j];
    __syncthreads();
    if (t < 128) {
      float v = 0.f;
      for (int g = 0; g < 16; ++g) v += red[g * 128 + t];
      const int m = m_base + t;
      if (m < a.M) {
        if (a.splits == 1) {
          float* cp = a.colsum + (a.perm ? a.perm[m] : m);
          *cp = a.accumulate ? *cp + v : v;
        } else {
          a.slab[(size_t)a.splits * a.M * a.N + (size_t)split * a.M + m] = v;
        }
      }
    }
  }

  // accumulator element (i, j, e): row m = wm*64 + 16i + 4(l>>4) + e, column n = wn*64 + 16j + (l&15)
  const int l = threadIdx.x & 63;
  if (a.splits == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m_base + wm * 64 + 16 * i + 4 * (l >> 4) + e;
        if (m >= a.M) continue;
        float* crow = a.C + (size_t)(a.perm ? a.perm[m] : m) * a.ldc;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n_base + wn * 64 + 16 * j + (l & 15);
          if (n < a.N) crow[n] = a.accumulate ? crow[n] + acc[i][j][e] : acc[i][j][e];
        }
      }
    return;
  }
  float* slab = a.slab + (size_t)split * a.M * a.N;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m_base + wm * 64 + 16 * i + 4 * (l >> 4) + e;
      if (m >= a.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n_base + wn * 64 + 16 * j + (l & 15);
        if (n < a.N) slab[(size_t)m * a.N + n] = acc[i][j][e];
      }
    }
#undef AS
#undef BS
#undef SF
}

// ---- exact fp32 (the IEEE-fp32 learner): v_mfma_f32_16x16x4_f32, one f32 per operand per lane, no split -------
// Same 128×128 tile / split-K / reduce organisation as above, 32-row K slabs staged as fp32 [k][m] images (row pitch
// 144 floats: the two 16-lane halves of a ds_read_b32 group read rows k and k+1 → banks 0-15 / 16-31, conflict-free).
// The 16x16x4 A fragment is A[m = l&15][k = l>>4] and B[k = l>>4][n = l&15]: with K-outer [k][m] images that is one
// plain dword read per lane, no transpose. Call c of a slab takes rows 4c … 4c+3.
// Two-level summation: every 32-row slab is accumulated from zero on the MFMA (a 32-long fma chain), then added into
// the running sum on the VALU — a split's outputs are sums of ≤ kc/32 slab partials instead of one kc-long chain
// (the round-off of a 1 400-long chain measured 1.8e-5 relative on the enum head's ∂W against float64; the split-K
// partials then go through the fixed-order reduce as before).
constexpr int kXP = 144;                          // fp32 image row pitch (floats)
constexpr int kXImg = 32 * kXP * 4;               // one 32-row operand image (bytes)

struct XStage {
  float4 a[4], b[4];                              // rows (t>>5) + 8i, columns 4·(t&31) … +3
};

template <bool WITH_B0>
__device__ __forceinline__ void load_stage_x(const Args& a, const Rsrc& R, int kbase, int kend, int m_base, int n_base,
                                             XStage& r) {
  const int t = threadIdx.x, c4 = 4 * (t & 31);
  const int m = m_base + c4, n = n_base + c4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = kbase + (t >> 5) + 8 * i;
    const bool kin = k < kend;
    r.a[i] = __builtin_bit_cast(float4, bload16(R.A, kin && m < a.M ? (k * a.lda + m) * 4 : kOob));
    r.b[i] = __builtin_bit_cast(float4, bload16(R.B, kin && n < a.N && k >= a.split ? ((k - a.split) * a.ldb + n) * 4
                                                                                    : kOob));
  }
  if (WITH_B0 && kbase < a.split) {               // prologue only (host keeps split ≤ 32 = one slab)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = kbase + (t >> 5) + 8 * i;
      const float4 p = __builtin_bit_cast(float4, bload16(R.B0, k < kend && n < a.N && k < a.split ? (k * a.ldb + n) * 4
                                                                                                  : kOob));
      r.b[i] = make_float4(r.b[i].x + p.x, r.b[i].y + p.y, r.b[i].z + p.z, r.b[i].w + p.w);
    }
  }
}

__device__ __forceinline__ void store_stage_x(char* S, const XStage& r) {
  const int t = threadIdx.x, c4 = 4 * (t & 31);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (t >> 5) + 8 * i;
    *reinterpret_cast<float4*>(S + (row * kXP + c4) * 4) = r.a[i];
    *reinterpret_cast<float4*>(S + kXImg + (row * kXP + c4) * 4) = r.b[i];
  }
}

// column sums (bias gradients) two-level like the products: the thread's 4 rows of a 32-row slab summed pairwise,
// then added into the running sum — a chain of kc/32 slab sums instead of kc/8 single rows (a 175-long fp32 chain per
// column measured 1.0e-5 relative on the 5v5 pointer head's bias gradient against float64, torch fp32 6e-7)
// (and Kahan-compensated: cc carries each add's rounding error into the next)
__device__ __forceinline__ void kahan_add(float& s, float& c, float v) {
  const float y = v - c, t = s + y;
  c = (t - s) - y;
  s = t;
}
__device__ __forceinline__ void add_slab_colsum(float (&cs)[4], float (&cc)[4], const XStage& st) {
  kahan_add(cs[0], cc[0], (st.a[0].x + st.a[1].x) + (st.a[2].x + st.a[3].x));
  kahan_add(cs[1], cc[1], (st.a[0].y + st.a[1].y) + (st.a[2].y + st.a[3].y));
  kahan_add(cs[2], cc[2], (st.a[0].z + st.a[1].z) + (st.a[2].z + st.a[3].z));
  kahan_add(cs[3], cc[3], (st.a[0].w + st.a[1].w) + (st.a[2].w + st.a[3].w));
}

__global__ __launch_bounds__(kThreads, 2) void gemm_tn_exact_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) char smem[4 * kXImg];   // [stage][A image | B image], 72 KB
  int tile, split;
  tile_split(a, tile, split);
  const int tm = tile / a.tiles_n, tn = tile % a.tiles_n;
  const int m_base = tm * BM, n_base = tn * BN;
  const int k_lo = split * a.kc, k_hi = min(a.K, k_lo + a.kc);
  const int w = threadIdx.x >> 6, wm = w & 1, wn = w >> 1, l = threadIdx.x & 63;
  const int fr = l >> 4, fc = l & 15;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float cs[4] = {0.f, 0.f, 0.f, 0.f}, cc[4] = {0.f, 0.f, 0.f, 0.f};
  const bool do_cs = a.colsum != nullptr && tn == 0;
  const Rsrc R = make_rsrc(a, 4);
  XStage st;
  int buf = 0;
  if (k_lo < k_hi) {
    load_stage_x<true>(a, R, k_lo, k_hi, m_base, n_base, st);
    store_stage_x(smem, st);
    if (do_cs) add_slab_colsum(cs, cc, st);
  }
  __syncthreads();
  for (int kb = k_lo; kb < k_hi; kb += 32) {
    const bool more = kb + 32 < k_hi;
    if (more) load_stage_x<false>(a, R, kb + 32, k_hi, m_base, n_base, st);   // in flight during the MFMAs
    const float* As = reinterpret_cast<const float*>(smem + buf * 2 * kXImg);
    const float* Bs = As + kXImg / 4;
    f32x4 part[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) part[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int row = 4 * c + fr;
      float fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = As[row * kXP + wm * 64 + 16 * i + fc];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = Bs[row * kXP + wn * 64 + 16 * j + fc];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) part[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], part[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] += part[i][j];
    if (more) {
      store_stage_x(smem + (buf ^ 1) * 2 * kXImg, st);
      if (do_cs) add_slab_colsum(cs, cc, st);
    }
    __syncthreads();
    buf ^= 1;
  }
  if (do_cs) {       // 8 row phases share each column quad: fixed-order LDS fold, one value per column
    float* red = reinterpret_cast<float*>(smem);       // [8][128] (the images are dead after the barrier)
    const int t = threadIdx.x, c4 = 4 * (t & 31), rg = t >> 5;
#pragma unroll
    for (int j = 0; j < 4; ++j) red[rg * 128 + c4 + j] = cs[j];
    __syncthreads();
    if (t < 128) {
      float v = 0.f;
      for (int g = 0; g < 8; ++g) v += red[g * 128 + t];
      const int m = m_base + t;
      if (m < a.M) {
        if (a.splits == 1) {
          float* cp = a.colsum + (a.perm ? a.perm[m] : m);
          *cp = a.accumulate ? *cp + v : v;
        } else {
          a.slab[(size_t)a.splits * a.M * a.N + (size_t)split * a.M + m] = v;
        }
      }
    }
  }
  // accumulator element (i, j, e): row m = wm*64 + 16i + 4(l>>4) + e, column n = wn*64 + 16j + (l&15)
  float* slab = a.slab + (size_t)split * a.M * a.N;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m_base + wm * 64 + 16 * i + 4 * fr + e;
      if (m >= a.M) continue;
      if (a.splits == 1) {
        float* crow = a.C + (size_t)(a.perm ? a.perm[m] : m) * a.ldc;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n_base + wn * 64 + 16 * j + fc;
          if (n < a.N) crow[n] = a.accumulate ? crow[n] + acc[i][j][e] : acc[i][j][e];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n_base + wn * 64 + 16 * j + fc;
          if (n < a.N) slab[(size_t)m * a.N + n] = acc[i][j][e];
        }
      }
    }
  if (a.splits == 1 || a.tickets == nullptr) return;
  // ---- split-K fold: the LAST workgroup of this tile to finish sums the tile's slabs in split order (deterministic
  // whichever workgroup arrives last) and writes C (and the column sums). Release: this workgroup's slab stores are
  // made visible device-wide (cross-XCD: the L2s are per XCD) before it takes its ticket; acquire before the reads.
  __shared__ unsigned s_last;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(a.tickets + tile, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == (unsigned)(a.splits - 1) ? 1u : 0u;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  const size_t plane = (size_t)a.M * a.N;
  const int n4t = BN / 4;                                   // float4 columns of a full tile
  for (int q = threadIdx.x; q < BM * n4t; q += kThreads) {
    const int m = m_base + q / n4t, n = n_base + 4 * (q % n4t);
    if (m >= a.M || n >= a.N) continue;                     // (N % 4 == 0: checked by the host)
    const f32x4* src = reinterpret_cast<const f32x4*>(a.slab + (size_t)m * a.N + n);
    const size_t pl4 = plane / 4;
    f32x4 sum = {0.f, 0.f, 0.f, 0.f};
    int sp = 0;
    for (; sp + 3 < a.splits; sp += 4) {                    // 4 loads in flight, summed in split order
      const f32x4 v0 = __builtin_nontemporal_load(src + (size_t)(sp + 0) * pl4);
      const f32x4 v1 = __builtin_nontemporal_load(src + (size_t)(sp + 1) * pl4);
      const f32x4 v2 = __builtin_nontemporal_load(src + (size_t)(sp + 2) * pl4);
      const f32x4 v3 = __builtin_nontemporal_load(src + (size_t)(sp + 3) * pl4);
      sum += v0;
      sum += v1;
      sum += v2;
      sum += v3;
    }
    for (; sp < a.splits; ++sp) sum += __builtin_nontemporal_load(src + (size_t)sp * pl4);
    float* cp = a.C + (size_t)(a.perm ? a.perm[m] : m) * a.ldc + n;
    if (a.accumulate) {
      sum[0] += cp[0]; sum[1] += cp[1]; sum[2] += cp[2]; sum[3] += cp[3];
    }
    cp[0] = sum[0]; cp[1] = sum[1]; cp[2] = sum[2]; cp[3] = sum[3];
  }
  if (do_cs && threadIdx.x < BM) {
    const int m = m_base + threadIdx.x;
    if (m < a.M) {
      const float* cs_part = a.slab + (size_t)a.splits * plane + m;
      float v = 0.f;
      for (int sp = 0; sp < a.splits; ++sp) v += cs_part[(size_t)sp * a.M];
      float* cp = a.colsum + (a.perm ? a.perm[m] : m);
      *cp = a.accumulate ? *cp + v : v;
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(a.tickets + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Fixed-order (deterministic) sum of the split-K slabs, optional row map / accumulate. A block of 256 threads owns
// 256/P float4 outputs × P split phases (P = power of two ≤ min(16, splits)): thread (phase p, output o) sums splits
// p, p+P, … with 4 loads in flight, then a fixed LDS fold over the phases — a long split list (K = 716 800 unit rows
// of the 5v5 attention weight gradients → ≈380 splits of one tile) is not one latency-bound chain per output, and
// a short one (6-25 splits of the 1v1 gradients) keeps every thread busy.
__global__ __launch_bounds__(256) void gemm_tn_reduce(const float* __restrict__ slab, int splits, int M, int N,
                                                      float* __restrict__ C, int ldc, const int* __restrict__ perm,
                                                      int accumulate, float* __restrict__ colsum, int lp) {
  const int P = 1 << lp, OPB = 256 >> lp;
  const int n4 = N >> 2;
  const size_t plane4 = (size_t)M * N / 4;
  const int ph = threadIdx.x >> (8 - lp), oi = threadIdx.x & (OPB - 1);
  __shared__ f32x4 red[256];
  const int nout = M * n4;
  for (int base = blockIdx.x * OPB; base < nout; base += gridDim.x * OPB) {
    const int idx = base + oi;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    if (idx < nout) {
      const int m = idx / n4, n = (idx % n4) * 4;
      const f32x4* src = reinterpret_cast<const f32x4*>(slab + (size_t)m * N + n);
      int sp = ph;
      for (; sp + 3 * P < splits; sp += 4 * P) {
        const f32x4 v0 = __builtin_nontemporal_load(src + (size_t)(sp + 0 * P) * plane4);
        const f32x4 v1 = __builtin_nontemporal_load(src + (size_t)(sp + 1 * P) * plane4);
        const f32x4 v2 = __builtin_nontemporal_load(src + (size_t)(sp + 2 * P) * plane4);
        const f32x4 v3 = __builtin_nontemporal_load(src + (size_t)(sp + 3 * P) * plane4);
        s += v0;
        s += v1;
        s += v2;
        s += v3;
      }
      for (; sp < splits; sp += P) s += __builtin_nontemporal_load(src + (size_t)sp * plane4);
    }
    if (P > 1) {
      red[threadIdx.x] = s;
      __syncthreads();
    }
    if (ph == 0 && idx < nout) {
      for (int k = 1; k < P; ++k) s += red[k * OPB + oi];
      const int m = idx / n4, n = (idx % n4) * 4;
      float* cp = C + (size_t)(perm ? perm[m] : m) * ldc + n;
      if (accumulate) {
        s[0] += cp[0]; s[1] += cp[1]; s[2] += cp[2]; s[3] += cp[3];
      }
      cp[0] = s[0]; cp[1] = s[1]; cp[2] = s[2]; cp[3] = s[3];
    }
    if (P > 1) __syncthreads();
  }
  if (colsum != nullptr) {       // same phase split for the column sums
    const float* cs = slab + (size_t)splits * plane4 * 4;
    __shared__ float cred[256];
    for (int base = blockIdx.x * OPB; base < M; base += gridDim.x * OPB) {
      const int m = base + oi;
      float v = 0.f;
      if (m < M) {
        int sp = ph;
        for (; sp + 3 * P < splits; sp += 4 * P) {
          const float v0 = cs[(size_t)(sp + 0 * P) * M + m], v1 = cs[(size_t)(sp + 1 * P) * M + m];
          const float v2 = cs[(size_t)(sp + 2 * P) * M + m], v3 = cs[(size_t)(sp + 3 * P) * M + m];
          v += v0;
          v += v1;
          v += v2;
          v += v3;
        }
        for (; sp < splits; sp += P) v += cs[(size_t)sp * M + m];
      }
      cred[threadIdx.x] = v;
      __syncthreads();
      if (ph == 0 && m < M) {
        for (int k = 1; k < P; ++k) v += cred[k * OPB + oi];
        float* cp = colsum + (perm ? perm[m] : m);
        *cp = accumulate ? *cp + v : v;
      }
      __syncthreads();
    }
  }
}

}  // namespace

// f32: 0 bf16, 1 fp32 bf16x3, 2 exact fp32
extern "C" void dca_gemm_tn_plan(int M, int N, int K, int* splits, int* kc, int* tiles, int f32) {
  const int bk = f32 ? 32 : BK;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  const int t = tm * tn;
  // ≈1.5 workgroups per CU; exact: ≈2 (MFMA-bound at 1/16 of the bf16 rate, two 64 KB workgroups fit a CU)
  // (exact workgroup target swept in round 4, learner step, two passes each: 256 → 5.55, 512 → 5.48, 768 → 5.53,
  // 1024 → 5.59 ms; profiles/r4_gemm_tn_target_sweep.txt)
  // (round 6: the split count is rounded DOWN — t·s never exceeds the target: with 2 workgroups per CU the exact
  // kernel's 512 slots hold the whole grid, where ceil(512 / t) left a straggler round for a handful of workgroups,
  // e.g. the 5v5 ∂W_qkv at t = 3 → 513 workgroups took 984 µs, twice its per-workgroup time; 1v1 ∂W_pre t = 14 → 518)
  const int target = f32 == 2 ? 512 : 384;
  int s = t >= target ? 1 : target / t;
  const int kmax = (K + bk - 1) / bk;                     // at least one K slab per split
  if (s > kmax) s = kmax;
  if (s < 1) s = 1;
  int c = (K + s - 1) / s;
  c = (c + bk - 1) / bk * bk;
  s = (K + c - 1) / c;
  *splits = s;
  *kc = c;
  *tiles = t;
}

// Split-K fold tickets: one persistent, zero-initialised pool of per-tile counters; every launch takes the next
// region round-robin (each tile's last workgroup resets its counter, so a region is clean again when its kernel ends).
// Regions are baked into captured graphs: 1 M counters are ≈ 5 000 step captures before a region is handed out again,
// and only kernels running at the same time could collide.
constexpr int kFoldMaxSplits = 64;
constexpr size_t kTicketPool = 1u << 20;
static unsigned* fold_tickets(int tiles) {
  static unsigned* pool = nullptr;
  static size_t next = 0;
  if (pool == nullptr) {
    if (hipMalloc(reinterpret_cast<void**>(&pool), kTicketPool * sizeof(unsigned)) != hipSuccess) return nullptr;
    if (hipMemset(pool, 0, kTicketPool * sizeof(unsigned)) != hipSuccess) return nullptr;
  }
  if (next + (size_t)tiles > kTicketPool) next = 0;
  unsigned* r = pool + next;
  next += (size_t)(tiles + 63) / 64 * 64;
  return r;
}

// f32 = 0: A, B, B0 bf16; f32 = 1: fp32 operands (bf16x3 split MFMA); f32 = 2: fp32 operands, exact fp32 MFMA
extern "C" hipError_t dca_gemm_tn(const void* A, int lda, const void* B, int ldb, const void* B0, int split_rows,
                                  float* C, int ldc, const int* perm, int accumulate, int M, int N, int K, float* slab,
                                  float* colsum, hipStream_t st, int f32) {
  if (B0 && split_rows > (f32 ? 32 : BK)) return hipErrorInvalidValue;   // B0 is read by a chunk's first slab only
  int splits, kc, tiles;
  dca_gemm_tn_plan(M, N, K, &splits, &kc, &tiles, f32);
  // exact kernel, DCA_GEMM_FOLD=1: the slabs are folded by each tile's last workgroup (no reduce launch) when the
  // split list is short. Measured SLOWER and therefore off by default (round 6, same box: learner step 5.88 vs 5.55 ms,
  // 5v5 exact 10.94 vs 10.63 ms — every workgroup's release fence writes its XCD's dirty L2 lines back before taking
  // a ticket, and the last workgroup's serial pass over the slabs lands on the step's tail; the separate reduce kernel
  // overlaps the encoder backward instead; profiles/r6_split_k_fold.md)
  static const bool fold_on = [] { const char* e = getenv("DCA_GEMM_FOLD"); return e && e[0] == '1'; }();
  unsigned* tickets = nullptr;
  if (f32 == 2 && splits > 1 && splits <= kFoldMaxSplits && (N % 4) == 0 && fold_on) {
    tickets = fold_tickets(tiles);
    if (tickets == nullptr) return hipErrorOutOfMemory;
  }
  static const int xcd_remap = [] { const char* e = getenv("DCA_GEMM_XCD"); return (e && e[0] == '0') ? 0 : 1; }();
  Args a{A, lda, B, ldb, B0 ? B0 : B, B0 ? split_rows : 0, C, ldc, perm, slab, colsum, M, N, K, kc, splits,
         (N + BN - 1) / BN, accumulate, tickets, xcd_remap};
  const dim3 grid(tiles * splits);                          // 1-D: tile_split() maps it XCD-aware
  if (f32 == 2) hipLaunchKernelGGL(gemm_tn_exact_kernel, grid, dim3(kThreads), 0, st, a);
  else if (f32) hipLaunchKernelGGL(gemm_tn_kernel<true>, grid, dim3(kThreads), 8 * kImgF32, st, a);
  else hipLaunchKernelGGL(gemm_tn_kernel<false>, grid, dim3(kThreads), 4 * kTileBytes, st, a);
  DCA_CHECK_LAUNCH();
  if (splits > 1 && tickets == nullptr) {
    int lp = 0;
    while (lp < 4 && (2 << lp) <= splits) ++lp;            // P = 2^lp ≤ min(16, splits)
    const int n = M * (N / 4), opb = 256 >> lp;
    int blocks = (n + opb - 1) / opb;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(gemm_tn_reduce, dim3(blocks), dim3(256), 0, st, slab, splits, M, N, C, ldc, perm, accumulate,
                       colsum, lp);
    DCA_CHECK_LAUNCH();
  }
  return hipSuccess;
}
