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
//   layer 1 : 16×10 units · W1ᵀ + b1 on ONE v_mfma_f32_16x16x32_bf16 per column tile (bf16 hi/lo split of x, W1
//             and b1, ≈2⁻¹⁶ relative; layer1_split), ReLU
//   → bf16 C-tile written transposed into a per-wave LDS image (ds_write_b64), read back as A fragments with
//     ds_read_b64_tr_b16
//   layer 2 : 16×128 · W_τᵀ on v_mfma_f32_16x16x32_bf16 with W_τ held in 128 VGPRs for the whole type job
//   → +b_τ, running max/argmax per (row, column), bf16 embedding tile through the same image for 16-B row stores.
// Unit features reach LDS by LDS-DMA (stage_units), so a type job has one memory round trip before its tiles.
// Backward recomputes layer 1 (same split form), builds ∂emb = dtl⊗q + scatter(∂pool at argmax) in A-fragment layout, computes
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
constexpr int kJobs = 3;         // type jobs per wave; grid.y splits them over workgroups

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
  const void* wt;       // (6, 128, 128) W_τ (out, in): bf16, or fp32 in the F32 variant
  const float* bt;      // (6, 128)
  const float* we;      // (128, 3)
  const float* be;      // (128)
  void* x896;           // (N, 896) out (bf16 / F32: fp32): [env | pool_ah | pool_eh | pool_anh | pool_enh | pool_ath | pool_eth]
  void* emb;            // (N, U, 128) out (bf16 / F32: fp32)
  unsigned char* arg;   // (N, 6, 128) u8 out
  int N;
  int compat;           // reference bug: eth pool = enh pool (policy.py:127)
  Layout L;
};

struct BwdParams {
  const float* units;
  const float* w1;
  const float* b1;
  const void* wtT;      // (6, 128, 128) bf16 W_τᵀ (in, out)
  const float* dtl;     // (N, U) ∂L/∂pointer-logit
  const float* q;       // pointer query, row stride ldq
  int ldq;
  const float* dx;      // (N, 896) f32 ∂L/∂x896
  const unsigned char* arg;
  short* demb;          // K-blocked bf16 (see kBlk): block (τ, u, 16-row block rb) at blkbase[τ] + u·NB + rb
  short* basic;         // same layout
  float* w1part;        // (gridDim.y·gridDim.x, 128·10 + 128) f32 per-workgroup ∂W1 ‖ ∂b1 partials
  int N;
  int compat;
  Layout L;
  long long blkbase[6];
  int NB;               // 16-row blocks per unit slot = ⌈N/16⌉
  const void* demb_in;  // optional (N, U, 128) bf16 ∂emb given (entity-attention path) —
                        // dtl/q/dx/arg unused
};

__device__ __forceinline__ void type_job(int wv, int j, int& tau, int& g) {
  // wave job list: j-th job of wave wv; returns tau = -1 when done
  const int lists[2][3] = {{2, 1, 4}, {3, 0, 5}};
  g = wv & 1;
  tau = (j < 3) ? lists[wv >> 1][j] : -1;
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

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// buffer resource over [p, p + bytes) from wave-uniform values (no waterfall loops around the buffer loads)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, int bytes) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

__device__ __forceinline__ short bf_lo(float v) { return dca::f2bf(v - dca::bf2f(dca::f2bf(v))); }

// LDS staging of a type job's unit features (shared by forward and backward, see the backward's notes).
constexpr int kStage = 24;                  // units staged per chunk (1v1 max 16, 5v5 max 24 per type)
constexpr int kUP = 4 * 64 + 1;            // LDS pitch (floats) of a staged row (see stage_units)
constexpr int kDP = 64;                    // LDS pitch (floats) of a staged dtl row
constexpr int kW1 = kD * kF + kD;           // ∂W1 (128×10) ‖ ∂b1 (128) floats per partial

// Layer 1 on ONE v_mfma_f32_16x16x32_bf16 per 16-column tile (16 cycles) instead of three exact-f32 16x16x4 MFMAs
// (96 cycles): split x = x_hi + x_lo and W1 = W_hi + W_lo into bf16 pairs and lay the K = 32 slots out as
//   k 0-9: x_hi·W_hi   k 10-19: x_lo·W_hi   k 20-29: x_hi·W_lo   k 30: 1·b_hi   k 31: 1·b_lo
// which is x·W1ᵀ + b1 up to the dropped x_lo·W_lo and the bf16 rounding of the lo parts (≈2⁻¹⁶ relative; the
// result is rounded to bf16 for layer 2 anyway). Slot → (feature, part) depends on the lane's k-group only.
__device__ __forceinline__ int l1_feat(int slot) { return slot < 30 ? slot % 10 : -1; }
__device__ __forceinline__ bool l1_xlo(int slot) { return slot >= 10 && slot < 20; }
__device__ __forceinline__ bool l1_wlo(int slot) { return slot >= 20; }   // slot 31 = b_lo (30 = b_hi)

__device__ __forceinline__ void load_w1_split(const float* __restrict__ w1, const float* __restrict__ b1,
                                              bf16x8 (&wb)[8], int lane) {
  const int j = lane & 15, kg = lane >> 4;
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    const int col = 16 * n + j;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int slot = 8 * kg + jj, f = l1_feat(slot);
      const float w = f >= 0 ? w1[col * kF + f] : b1[col];
      const short hi = dca::f2bf(w);
      const short lo = dca::f2bf(w - dca::bf2f(hi));
      wb[n][jj] = (slot == 31 || (f >= 0 && l1_wlo(slot))) ? lo : hi;
    }
  }
}

// A fragment of one unit for the 16 staged rows (row = lane & 15), slots 8·kg … 8·kg + 7.
__device__ __forceinline__ bf16x8 l1_afrag(const float* __restrict__ ur, int u, int lane) {
  const int i = lane & 15, kg = lane >> 4;
  const float* x = ur + i * kUP + u * kF;
  bf16x8 a;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    const int slot = 8 * kg + jj, f = l1_feat(slot);
    const float v = x[f < 0 ? 0 : f];
    const short hi = dca::f2bf(v);
    const short lo = dca::f2bf(v - dca::bf2f(hi));
    a[jj] = f < 0 ? (short)0x3F80 : (l1_xlo(slot) ? lo : hi);   // 0x3F80 = bf16 1.0 (bias slots)
  }
  return a;
}

__device__ __forceinline__ void layer1_split(const float* __restrict__ ur, int u, const bf16x8 (&wb)[8],
                                             f32x4 (&acc)[8], int lane) {
  const bf16x8 a = l1_afrag(ur, u, lane);
#pragma unroll
  for (int n = 0; n < 8; ++n)
    acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wb[n], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
}

// 16×128 bf16 tile image in LDS, TRANSPOSED ([column][row], 32-B image rows): a C-layout fragment (rows 4kg … 4kg+3
// of one column) is one ds_write_b64, and tile_frag reads it back as A fragments / row-major 16-B chunks with
// ds_read_b64_tr_b16. Image row R sits at R·16 + (R/8)·64 shorts (a 128-B skew between 8-row groups) with its four
// 8-B chunks XOR-swizzled by 2·((R/8)&1): both the writes (16 rows × 2 chunks per half-wave) and the transposed reads
// (rows 8g + q and 8g + q + 4, 4 chunks) then hit 32 distinct bank pairs per half-wave.
constexpr int kImg = 128 * 16 + 16 * 64;   // shorts per tile image
__device__ __forceinline__ int img_off(int R, int c) { return R * 16 + (R >> 3) * 64 + 4 * (c ^ (2 * ((R >> 3) & 1))); }
typedef short lds_bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void tile_put(short* img, int n, const f32x4& v, int lane) {
  const int i = lane & 15, kg = lane >> 4;
  bf16x4 h;
  h[0] = dca::f2bf(v[0]); h[1] = dca::f2bf(v[1]); h[2] = dca::f2bf(v[2]); h[3] = dca::f2bf(v[3]);
  *reinterpret_cast<bf16x4*>(img + img_off(16 * n + i, kg)) = h;
}
// the lo bf16 halves (v - bf16(v)) of a C-layout fragment, same image layout (F32 variant)
__device__ __forceinline__ void tile_put_lo(short* img, int n, const f32x4& v, int lane) {
  const int i = lane & 15, kg = lane >> 4;
  bf16x4 h;
  h[0] = bf_lo(v[0]); h[1] = bf_lo(v[1]); h[2] = bf_lo(v[2]); h[3] = bf_lo(v[3]);
  *reinterpret_cast<bf16x4*>(img + img_off(16 * n + i, kg)) = h;
}
// element jj of lane l = image[k0 + 8(l>>4) + jj][l & 15] (= tile row l&15, columns k0 + 8(l>>4) … +7); k0 % 16 == 0
__device__ __forceinline__ bf16x8 tile_frag(const short* img, int k0, int lane) {
  typedef __attribute__((address_space(3))) lds_bf16x4 lds_v4;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const short* a = img + img_off(k0 + 8 * g + q, p);
  const lds_bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)a);
  const lds_bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a + 4 * 16));   // row + 4: same group
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

// Stage units[row0 .. row0+15][uoff+c0 .. +cc][0..9] and dtl for the same (row, unit) block into LDS (one wave) with
// LDS-DMA (global_load_lds_dword: no VGPRs, every load of the job in flight at once, one drain). Each instruction moves
// 64 consecutive floats of one row, so rows sit kUP = 4·64 + 1 floats apart (the +1 skews the banks of the 16 rows a
// fragment read touches). Rows past N load row N-1: their results are never stored and their gradients are zero.
// (Register-staged conditional loads made the compiler wait out each load before the next: ≈40 serialised round
// trips per 16-unit job, then most of the encoder's time.)
__device__ __forceinline__ void stage_units(const float* __restrict__ units, const float* __restrict__ dtl, int U,
                                            int N, int row0, int ubase, int cc, float* ur, float* dr, int lane) {
  typedef __attribute__((address_space(1))) void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;
  const int per = cc * kF;                       // floats per row (contiguous in global memory)
  const int nk = (per + 63) >> 6;
#pragma unroll 4
  for (int r = 0; r < 16; ++r) {
    const float* src = units + ((size_t)min(row0 + r, N - 1) * U + ubase) * kF;
    for (int k = 0; k < nk; ++k)
      __builtin_amdgcn_global_load_lds((gvoid*)(src + min(64 * k + lane, per - 1)), (lvoid*)(ur + r * kUP + 64 * k),
                                       4, 0, 0);
  }
  if (dtl) {
#pragma unroll 4
    for (int r = 0; r < 16; ++r)
      __builtin_amdgcn_global_load_lds((gvoid*)(dtl + (size_t)min(row0 + r, N - 1) * U + ubase + min(lane, cc - 1)),
                                       (lvoid*)(dr + r * kDP), 4, 0, 0);
  }
  // drain here, once: later unit iterations then carry no vmcnt waits (which would also wait out their own stores)
  __builtin_amdgcn_s_waitcnt(0);
}

// ============================================================================================================
__global__ __launch_bounds__(256, 1) void encoder_fwd_kernel(FwdParams P) {
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int rbase = blockIdx.x * kRows;
  const int U = P.L.U, N = P.N;
  short* const x896 = static_cast<short*>(P.x896);
  short* const embo = static_cast<short*>(P.emb);
  __shared__ __attribute__((aligned(16))) short scr[4][kImg];
  __shared__ __attribute__((aligned(16))) float ust[4][16 * kUP];

  // ---- env embedding: relu(We·env + be) → x896[:, 0:128] (32 rows × 128 cols over 256 threads; job 0's workgroups)
  if (blockIdx.y == 0) {
    const int r = tid >> 3, c0 = (tid & 7) * 16;
    const int row = rbase + r;
    if (row < N) {
      const float e0 = P.env[row * 3], e1 = P.env[row * 3 + 1], e2 = P.env[row * 3 + 2];
      for (int c = c0; c < c0 + 16; ++c) {
        const float v = P.be[c] + P.we[c * 3] * e0 + P.we[c * 3 + 1] * e1 + P.we[c * 3 + 2] * e2;
        x896[(size_t)row * 896 + c] = dca::f2bf(fmaxf(v, 0.f));
      }
    }
  }

  bf16x8 wb[8];
  load_w1_split(P.w1, P.b1, wb, lane);
  short* img = &scr[wv][0];

  const int i = lane & 15, kg = lane >> 4;
  // job split over blockIdx.y (gridDim.y == 3: one type job per wave per workgroup; 1: all three)
  const int jlo = gridDim.y == 3 ? (int)blockIdx.y : 0, jhi = gridDim.y == 3 ? jlo + 1 : 3;
  for (int j = jlo; j < jhi; ++j) {
    int tau, g;
    type_job(wv, j, tau, g);
    const int cnt = P.L.cnt[tau], uoff = P.L.off[tau];
    if (cnt == 0) continue;
    const int row0 = rbase + 16 * g;
    bf16x8 wf[8][4];
    load_bfrags(static_cast<const short*>(P.wt) + (size_t)tau * kD * kD, wf, lane);
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
    float* ur = &ust[wv][0];
    for (int c0 = 0; c0 < cnt; c0 += kStage) {
     const int cc = min(kStage, cnt - c0);
     // stage the next ≤ kStage units of this job (all loads in flight at once; also drains the W_τ loads)
     __builtin_amdgcn_wave_barrier();
     stage_units(P.units, nullptr, U, N, row0, uoff + c0, cc, ur, nullptr, lane);
     __builtin_amdgcn_wave_barrier();
     for (int uc = 0; uc < cc; ++uc) {
      const int u = c0 + uc;
      // layer 1 (bias folded into the MFMA) → ReLU → bf16 transposed tile image → layer-2 A fragments
      f32x4 acc[8];
      layer1_split(ur, uc, wb, acc, lane);
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        f32x4 b;
#pragma unroll
        for (int r = 0; r < 4; ++r) b[r] = fmaxf(acc[n][r], 0.f);
        tile_put(img, n, b, lane);
      }
      __builtin_amdgcn_wave_barrier();
      bf16x8 af[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) af[s] = tile_frag(img, 32 * s, lane);
      // layer 2 (LDS ops of a wave execute in order: the writes below cannot overtake the reads above)
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s], wf[n][s], c, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = c[r] + btv[n];
          if (v > pmax[n][r]) { pmax[n][r] = v; parg[n][r] = u; }
          c[r] = v;
        }
        tile_put(img, n, c, lane);
      }
      __builtin_amdgcn_wave_barrier();
      // embedding tile → row-major: lane → row i, columns 32s + 8kg … +7 (16-B stores, 64 B contiguous per row)
      {
        const int row = row0 + i;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const bf16x8 f = tile_frag(img, 32 * s, lane);
          if (row < N) *reinterpret_cast<bf16x8*>(embo + ((size_t)row * U + uoff + u) * kD + 32 * s + 8 * kg) = f;
        }
      }
      __builtin_amdgcn_wave_barrier();
     }
    }
    // ---- flush pool + argmax for this (type, group); compat: eth pool is overwritten by enh (host side)
#pragma unroll
    for (int n = 0; n < 8; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + kg * 4 + r;
        if (row < N) {
          const int col = 16 * n + i;
          x896[(size_t)row * 896 + kD + tau * kD + col] = dca::f2bf(pmax[n][r]);
          P.arg[((size_t)row * 6 + tau) * kD + col] = (unsigned char)parg[n][r];
        }
      }
  }
}

// ============================================================================================================
// Backward. Latency structure: one wave per SIMD (W_τ lives in 128 VGPRs), so every global load a unit iteration
// waits on is exposed. Per type job the wave therefore (1) stages the job's unit features and pointer-logit
// gradients for its 16 rows in LDS with all loads in flight at once, and (2) hoists the per-(row, type) operands —
// pointer query q, pool gradient ∂pool and the argmax bytes — into registers; a unit iteration then touches
// global memory only for its output stores. ∂W1/∂b1 are reduced over the workgroup's waves in LDS and written as
// one partial per workgroup; encoder_w1_reduce sums the partials in a fixed order (deterministic, no atomics).
// K-blocked layout of ∂emb and basic for the weight-gradient GEMM (∂W_τ = Σ ∂embᵀ·basic over all rows and units):
// element (row r of 16-row block blk, column e) at (blk·128 + e)·16 + r. A 16x16x32 MFMA fragment (8 consecutive k
// of one column) is then one 16-byte load, and a (τ, u, row block) tile is 4 KB contiguous.
// The tile is transposed through a padded per-wave LDS image: column e at element e·16 + (e/8)·16 (32-B pad every
// 8 columns spreads the four 8-column groups of a store over different banks).
constexpr int kTile = 128 * 16 + 16 * 16;
__device__ __forceinline__ int toff(int e, int r) { return e * 16 + (e >> 3) * 16 + r; }
__device__ __forceinline__ void store_tile(const short* tw, short* dst, int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = lane + 64 * q;                  // 16-byte chunk: column c/2, rows 8·(c&1) …
    *reinterpret_cast<bf16x8*>(dst + c * 8) = *reinterpret_cast<const bf16x8*>(tw + toff(c >> 1, 8 * (c & 1)));
  }
}

__global__ __launch_bounds__(256, 1) void encoder_bwd_kernel(BwdParams P) {
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int rbase = blockIdx.x * kRows;
  const int U = P.L.U, N = P.N;
  const int i = lane & 15, kg = lane >> 4;
  __shared__ __attribute__((aligned(16))) short tsc[4][kTile];
  __shared__ __attribute__((aligned(16))) float ust[4][16 * kUP];
  __shared__ float dst_[4][16 * kDP];
  __shared__ float wred[kW1];
  short* tw = &tsc[wv][0];

  bf16x8 wb[8];                                   // layer 1 exactly as the forward computed it (layer1_split)
  load_w1_split(P.w1, P.b1, wb, lane);
  f32x4 dw1acc[8];
  float db1acc[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    dw1acc[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
    db1acc[n] = 0.f;
  }
  for (int e = tid; e < kW1; e += 256) wred[e] = 0.f;

  // job split over blockIdx.y (gridDim.y == 3: one type job per wave per workgroup; 1: all three)
  const int jlo = gridDim.y == 3 ? (int)blockIdx.y : 0, jhi = gridDim.y == 3 ? jlo + 1 : 3;
  for (int j = jlo; j < jhi; ++j) {
    int tau, g;
    type_job(wv, j, tau, g);
    const int cnt = P.L.cnt[tau], uoff = P.L.off[tau];
    if (cnt == 0) continue;
    const int row0 = rbase + 16 * g;
    if (row0 >= N) continue;                      // wave-uniform: no rows in this group
    const int rb = row0 / 16;
    bf16x8 wf[8][4];   // B[k=e][n=j] = W_τ[e][j] = W_τᵀ[j][e]
    load_bfrags(static_cast<const short*>(P.wtT) + (size_t)tau * kD * kD, wf, lane);
    const int arow = row0 + i;
    const bool rok = arow < N;
    const bool eth_dead = P.compat && tau == 5;   // reference bug: eth pool unused → no pool gradient
    const bool given = P.demb_in != nullptr;       // wave-uniform
    // ---- per-(row, type) operands in A layout (row i, cols 32s + 8kg + jj), loaded once per type job
    float qv[4][8], dpv[4][8];
    unsigned agv[4][2];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int e0 = 32 * s + 8 * kg;
      if (rok && !given) {
        const float4 qa = *reinterpret_cast<const float4*>(P.q + (size_t)arow * P.ldq + e0);
        const float4 qb = *reinterpret_cast<const float4*>(P.q + (size_t)arow * P.ldq + e0 + 4);
        qv[s][0] = qa.x; qv[s][1] = qa.y; qv[s][2] = qa.z; qv[s][3] = qa.w;
        qv[s][4] = qb.x; qv[s][5] = qb.y; qv[s][6] = qb.z; qv[s][7] = qb.w;
        const float* dp = P.dx + (size_t)arow * 896 + kD + tau * kD + e0;
        const float4 da = *reinterpret_cast<const float4*>(dp);
        const float4 db = *reinterpret_cast<const float4*>(dp + 4);
        dpv[s][0] = da.x; dpv[s][1] = da.y; dpv[s][2] = da.z; dpv[s][3] = da.w;
        dpv[s][4] = db.x; dpv[s][5] = db.y; dpv[s][6] = db.z; dpv[s][7] = db.w;
        const uint2 ag = *reinterpret_cast<const uint2*>(P.arg + ((size_t)arow * 6 + tau) * kD + e0);
        agv[s][0] = eth_dead ? 0xffffffffu : ag.x;
        agv[s][1] = eth_dead ? 0xffffffffu : ag.y;
      } else {
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) { qv[s][jj] = 0.f; dpv[s][jj] = 0.f; }
        agv[s][0] = agv[s][1] = 0xffffffffu;
      }
    }
    float* ur = &ust[wv][0];
    float* dr = &dst_[wv][0];
    for (int c0 = 0; c0 < cnt; c0 += kStage) {
      const int cc = min(kStage, cnt - c0);
      __builtin_amdgcn_wave_barrier();
      stage_units(P.units, given ? nullptr : P.dtl, U, N, row0, uoff + c0, cc, ur, dr, lane);
      __builtin_amdgcn_wave_barrier();
      for (int uc = 0; uc < cc; ++uc) {
        const int u = c0 + uc;
        // ---- recompute layer 1 (C layout) → basic f32
        f32x4 acc[8];
        layer1_split(ur, uc, wb, acc, lane);
        f32x4 bas[8];
#pragma unroll
        for (int n = 0; n < 8; ++n)
#pragma unroll
          for (int r = 0; r < 4; ++r) bas[n][r] = fmaxf(acc[n][r], 0.f);
        // ---- ∂emb in A layout: dtl·q + ∂pool where this unit is the argmax (or given)
        const float dtl = given ? 0.f : dr[i * kDP + uc];
        bf16x8 de[4];
        if (given) {
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            bf16x8 h = {0, 0, 0, 0, 0, 0, 0, 0};
            if (rok)
              h = *reinterpret_cast<const bf16x8*>(static_cast<const short*>(P.demb_in) +
                                                   ((size_t)arow * U + uoff + u) * kD + 32 * s + 8 * kg);
            de[s] = h;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) tw[toff(32 * s + 8 * kg + jj, i)] = h[jj];
          }
        }
#pragma unroll
        for (int s = 0; s < 4 && !given; ++s) {
          float v[8];
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            const unsigned ab = (agv[s][jj >> 2] >> (8 * (jj & 3))) & 0xffu;
            v[jj] = dtl * qv[s][jj] + (ab == (unsigned)u ? dpv[s][jj] : 0.f);
          }
          if (P.compat && tau == 3 && rok) {   // eth pool = enh pool: its gradient lands on enh argmax units
            const int e0 = 32 * s + 8 * kg;
            const float* dp = P.dx + (size_t)arow * 896 + kD + 5 * kD + e0;
            const unsigned char* ag = P.arg + ((size_t)arow * 6 + 3) * kD + e0;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) v[jj] += (ag[jj] == u) ? dp[jj] : 0.f;
          }
          bf16x8 h;
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) h[jj] = dca::f2bf(v[jj]);
          de[s] = h;
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) tw[toff(32 * s + 8 * kg + jj, i)] = h[jj];
        }
        // ---- ∂emb tile → K-blocked image (4 KB contiguous per (τ, u, row block))
        const size_t blk = (size_t)(P.blkbase[tau] + (long long)u * P.NB + rb) * (kD * 16);
        __builtin_amdgcn_wave_barrier();
        store_tile(tw, P.demb + blk, lane);
        __builtin_amdgcn_wave_barrier();
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
        // ---- ∂W1 += ∂basicᵀ · units  (16x16x16 bf16: A[j][m] = ∂basic C-tile, B[m][k] = units from LDS)
        bf16x4 ub;
        {
          const int kk = lane & 15;
#pragma unroll
          for (int r = 0; r < 4; ++r) ub[r] = dca::f2bf(kk < kF ? ur[(4 * kg + r) * kUP + uc * kF + kk] : 0.f);
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
        // ---- basic tile (C layout: rows 4kg + r, column 16n + i) → K-blocked image
#pragma unroll
        for (int n = 0; n < 8; ++n) {
          bf16x4 v4;
#pragma unroll
          for (int r = 0; r < 4; ++r) v4[r] = dca::f2bf(bas[n][r]);
          *reinterpret_cast<bf16x4*>(&tw[toff(16 * n + i, 4 * kg)]) = v4;
        }
        __builtin_amdgcn_wave_barrier();
        store_tile(tw, P.basic + blk, lane);
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
  // ---- ∂W1 (rows j = 16n + 4kg + r, col k = lane&15 < 10) and ∂b1: waves → LDS (fixed order) → one partial
  for (int w = 0; w < 4; ++w) {
    __syncthreads();
    if (wv == w) {
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        const int k = lane & 15;
        if (k < kF) {
#pragma unroll
          for (int r = 0; r < 4; ++r) wred[(16 * n + 4 * kg + r) * kF + k] += dw1acc[n][r];
        }
        float s = db1acc[n];
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        if (kg == 0) wred[kD * kF + 16 * n + i] += s;
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < kW1; e += 256) P.w1part[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * kW1 + e] = wred[e];
}

// ============================================================================================================
// F32 variants (the learner's fp32-accurate mode, "bf16x3"): every MFMA operand x is split once into two bf16,
// x = hi + lo, and a product is hi·hi + lo·hi + hi·lo on three independent accumulation chains (the dropped lo·lo
// term and the rounding of lo are ≈2⁻¹⁶ relative; f32 accumulation). Outputs are fp32. Both F32 kernels run
// 8-wave workgroups over ranges of (16-row group, unit) items of one type, wave w owning 16 output columns (its
// hi + lo weight fragments: 32 VGPRs), so that two waves share a SIMD.
// bf16x3 16×16 tile over K = 128: Σ_s a·w + al·w + a·wl (three chains)
__device__ __forceinline__ f32x4 mfma3_k128(const bf16x8 (&a)[4], const bf16x8 (&al)[4], const bf16x8 (&w)[4],
                                            const bf16x8 (&wl)[4]) {
  f32x4 c = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f}, c2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s], w[s], c, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[s], w[s], c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s], wl[s], c2, 0, 0, 0);
  }
  return c + (c1 + c2);
}

// F32 backward, fused ∂W_τ. The bf16 path writes ∂emb and basic as K-blocked images for a separate GEMM; at bf16x3
// that is four bf16 images (≈460 MB at the 1v1 learner shape) written and read back. Here a workgroup of 8 waves
// owns a contiguous range of (16-row group, unit) items of ONE type τ and keeps ∂W_τ in registers across the range:
//   * wave w builds e-tile w of the item's ∂emb (C layout, fp32 → hi / lo bf16) into a double-buffered transposed
//     LDS image (tile_put layout), one item ahead, between its MFMAs of the current item; one LDS-only barrier per
//     item;
//   * wave w owns basic columns j ∈ tile w: layer 1 (recomputed), ∂basic = ∂emb·W_τ[:, j] (bf16x3, A fragments
//     by ds_read_b64_tr_b16), ReLU', ∂W1 rows j, and ∂W_τᵀ[j][e] += basicᵀ·∂emb on 16x16x16 MFMAs whose A operand
//     is the C-layout basic tile and whose B operand is the C-layout ∂emb tile read back as written;
//   * an item's unit features and dtl (identical for all 8 waves) are staged once into LDS two items ahead; the per-row q / ∂pool / argmax of the wave's e-tile are raw buffer loads (hardware bounds check: rows
//     past N read 0), issued one item ahead and only when the row group changes.
// 2 waves per SIMD (≤ 256 VGPRs) overlap one wave's loads / VALU with the other's MFMAs.
// Each workgroup writes one tile-linear 128×128 ∂W_τ partial and one ∂W1‖∂b1 partial; fixed-order reduces follow.
struct FbParams {
  const float* units;
  const float* w1;
  const float* b1;
  const float* wtT;      // (6, 128, 128) fp32 W_τᵀ (in, out)
  const float* dtl;
  const float* q;
  int ldq;
  const float* dx;
  const unsigned char* arg;
  const float* demb_in;  // optional fp32 (N, U, 128)
  float* w1part;         // (jobs, kW1)
  float* dwtpart;        // (jobs, 128·128) tile-linear
  int N;
  int compat;
  int items;             // items per job
  Layout L;
  int jbase[7];
};

struct FbBuild {   // per-row-group data the ∂emb build needs (e = 16·wv + i, rows 4kg + r); GIVEN: the item's ∂emb
  float q[4];      // q[row][e]                              (GIVEN: ∂emb[row][u][e])
  float ds[4];     // ∂pool[row][e] routed to this type (compat: + the eth slot for enh; none for a dead eth)
  unsigned ab[4];  // argmax byte of each row (unpacked: packing would wait for the loads where they are issued)
};

__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

struct FbRsrc {
  __amdgpu_buffer_rsrc_t q, x, a, g;
};

// Build loads of item k (raw buffer loads: 32-bit offsets, rows past N read 0). rg: item k starts a new row group —
// q / ∂pool / argmax are per row, shared by the type's units, so they are re-read only then.
template <bool GIVEN, bool COMPAT>
__device__ __forceinline__ void fb_load_build(FbBuild& p, const FbRsrc& R, int ldq, int k, bool rg, int cnt, int uoff,
                                              int U, int tau, int wv, int i, int kg) {
  const int rb = k / cnt, u = k - rb * cnt, row0 = 16 * rb;
  const int e = 16 * wv + i;
  if constexpr (GIVEN) {
#pragma unroll
    for (int r = 0; r < 4; ++r) p.q[r] = bload(R.g, (((row0 + 4 * kg + r) * U + uoff + u) * kD + e) * 4);
  } else if (rg) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * kg + r;
      p.q[r] = bload(R.q, (row * ldq + e) * 4);
      const int xo = (row * 896 + kD + tau * kD + e) * 4;
      p.ds[r] = tau == 5 && COMPAT ? 0.f : bload(R.x, xo);
      if constexpr (COMPAT) p.ds[r] += tau == 3 ? bload(R.x, xo + 2 * kD * 4) : 0.f;
      p.ab[r] = __builtin_amdgcn_raw_buffer_load_b8(R.a, (row * 6 + tau) * kD + e, 0, 0);
    }
  }
}

// Per-item staging (LDS, 3 slots): units[row0 .. row0+15][u][0..9] (160 floats) ‖ dtl[row0 .. row0+15][u] (16) — the
// same for all 8 waves, so waves 0-2 load it once (one dword per lane, rows past N read row N-1, whose ∂emb is zero),
// hold it in a register for an item and write it to the slot two items ahead of its use. (An LDS-DMA load instead
// made the compiler wait for it before every later read of the staging array: one exposed round trip per item.)
constexpr int kStg = 192;
__device__ __forceinline__ float fb_stage_load(const FbParams& P, int k, int cnt, int uoff, int wv, int lane) {
  const int U = P.L.U, N = P.N;
  const int rb = k / cnt, u = k - rb * cnt, row0 = 16 * rb;
  const int idx = 64 * min(wv, 2) + lane;
  // one load per lane, address selected (two loads under divergent branches wrote the same register: the second
  // had to wait for the first, a full memory round trip in the item loop)
  const bool isu = idx < 16 * kF;
  const int row = isu ? min(row0 + idx / kF, N - 1) : min(row0 + min(idx - 16 * kF, 15), N - 1);
  // (no dtl — the given-∂emb variant, which never reads the dtl slots: any valid address; no select on the loaded
  // value either, which would make the wave wait for the load right here)
  const float* src = isu ? P.units + ((size_t)row * U + uoff + u) * kF + idx % kF
                         : (P.dtl ? P.dtl + (size_t)row * U + uoff + u : P.units);
  return *src;
}

// ∂emb e-tile wv of item k (C layout) → hi / lo image
template <bool GIVEN>
__device__ __forceinline__ void fb_build(const FbBuild& b, const float* slot, int u, short* ih, short* il, int wv,
                                         int lane) {
  const int kg = lane >> 4;
  f32x4 v;
  if constexpr (GIVEN) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = b.q[r];
  } else {
    const f32x4 d4 = *reinterpret_cast<const f32x4*>(slot + 16 * kF + 4 * kg);   // dtl of rows 4kg … 4kg + 3
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = d4[r] * b.q[r] + (b.ab[r] == (unsigned)u ? b.ds[r] : 0.f);
  }
  tile_put(ih, wv, v, lane);
  tile_put_lo(il, wv, v, lane);
}

template <bool GIVEN, bool COMPAT>
__global__ __launch_bounds__(512, 1) void encoder_bwd_f32_fused_kernel(FbParams P) {
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int i = lane & 15, kg = lane >> 4;
  const int job = blockIdx.x;
  int tau = 0;
#pragma unroll
  for (int t = 1; t < 6; ++t) tau += job >= P.jbase[t] ? 1 : 0;
  const int cnt = P.L.cnt[tau], uoff = P.L.off[tau], N = P.N, U = P.L.U;
  const int NB = (N + 15) >> 4;
  const int k0 = (job - P.jbase[tau]) * P.items, k1 = min(k0 + P.items, cnt * NB);
  __shared__ __attribute__((aligned(16))) short img[2][2][kImg];   // [buffer][hi, lo]
  __shared__ __attribute__((aligned(16))) float stg[3][kStg];
  FbRsrc R;
  if constexpr (GIVEN) {
    R.g = uniform_rsrc(P.demb_in, N * U * kD * 4);
  } else {
    R.q = uniform_rsrc(P.q, N * P.ldq * 4);
    R.x = uniform_rsrc(P.dx, N * 896 * 4);
    R.a = uniform_rsrc(P.arg, N * 6 * kD);
  }

  // ---- weights of this wave's basic-column tile: B[k = e][n = j] = W_τ[e][j] (bf16x3 halves) and the split W1 row
  const int col = 16 * wv + i;
  bf16x8 wf[4], wfl[4], wb;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const float* p = P.wtT + ((size_t)tau * kD + col) * kD + 32 * s + 8 * kg;
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      wf[s][jj] = dca::f2bf(v[jj]);
      wfl[s][jj] = dca::f2bf(v[jj] - dca::bf2f(wf[s][jj]));
    }
  }
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    const int slot = 8 * kg + jj, f = l1_feat(slot);
    const float w = f >= 0 ? P.w1[col * kF + f] : P.b1[col];
    const short hi = dca::f2bf(w);
    const short lo = dca::f2bf(w - dca::bf2f(hi));
    wb[jj] = (slot == 31 || (f >= 0 && l1_wlo(slot))) ? lo : hi;
  }
  f32x4 acc[8], dw1acc = {0.f, 0.f, 0.f, 0.f};
  float db1acc = 0.f;
#pragma unroll
  for (int et = 0; et < 8; ++et) acc[et] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Software pipeline, per item k: [barrier: image k built, staging slot of k+1 written] → waves 0-2 write the
  // staging of k+2 (loaded one item earlier) and load k+3 → item k's MFMAs with the ∂emb of k+1 built in between
  // (its row data were loaded one item earlier) → build loads of k+2. No barrier waits on global memory.
  FbBuild bn;
  const int kl = max(k1 - 1, 0);
  float pre = 0.f;
  if (wv < 3) {
    stg[k0 % 3][64 * wv + lane] = fb_stage_load(P, min(k0, kl), cnt, uoff, wv, lane);
    stg[(k0 + 1) % 3][64 * wv + lane] = fb_stage_load(P, min(k0 + 1, kl), cnt, uoff, wv, lane);
    pre = fb_stage_load(P, min(k0 + 2, kl), cnt, uoff, wv, lane);
  }
  fb_load_build<GIVEN, COMPAT>(bn, R, P.ldq, min(k0, kl), true, cnt, uoff, U, tau, wv, i, kg);
  lds_barrier();
  fb_build<GIVEN>(bn, stg[k0 % 3], k0 % cnt, &img[0][0][0], &img[0][1][0], wv, lane);
  fb_load_build<GIVEN, COMPAT>(bn, R, P.ldq, min(k0 + 1, kl), min(k0 + 1, kl) % cnt == 0, cnt, uoff, U, tau, wv, i,
                               kg);
  int buf = 0;
  for (int k = k0; k < k1; ++k) {
    lds_barrier();
    if (wv < 3) {
      stg[(k + 2) % 3][64 * wv + lane] = pre;
      pre = fb_stage_load(P, min(k + 3, kl), cnt, uoff, wv, lane);
    }
    const float* sl = stg[k % 3];
    bf16x8 a1;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int slot = 8 * kg + jj;
      const float x = sl[i * kF + max(l1_feat(slot), 0)];
      const short hi = dca::f2bf(x);
      const short lo = dca::f2bf(x - dca::bf2f(hi));
      a1[jj] = l1_feat(slot) < 0 ? (short)0x3F80 : (l1_xlo(slot) ? lo : hi);
    }
    bf16x4 ub, ubl;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float x = i < kF ? sl[(4 * kg + r) * kF + i] : 0.f;
      ub[r] = dca::f2bf(x);
      ubl[r] = dca::f2bf(x - dca::bf2f(ub[r]));
    }
    const short* ih = &img[buf][0][0];
    const short* il = &img[buf][1][0];
    bf16x8 de[4], del[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      de[s] = tile_frag(ih, 32 * s, lane);
      del[s] = tile_frag(il, 32 * s, lane);
    }
    bf16x4 eh[8], el[8];
#pragma unroll
    for (int et = 0; et < 8; ++et) {
      eh[et] = *reinterpret_cast<const bf16x4*>(ih + img_off(16 * et + i, kg));
      el[et] = *reinterpret_cast<const bf16x4*>(il + img_off(16 * et + i, kg));
    }
    const f32x4 l1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, wb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    f32x4 c = mfma3_k128(de, del, wf, wfl);
    // item k + 1's ∂emb into the other image (every wave has passed this item's barrier, so none still reads it;
    // past the range's end this rewrites the last item, which nobody reads)
    fb_build<GIVEN>(bn, stg[(k + 1) % 3], min(k + 1, kl) % cnt, &img[buf ^ 1][0][0], &img[buf ^ 1][1][0], wv, lane);
    fb_load_build<GIVEN, COMPAT>(bn, R, P.ldq, min(k + 2, kl), k + 2 <= kl && (k + 2) % cnt == 0, cnt, uoff, U, tau,
                                 wv, i, kg);
    bf16x4 bh, bl;
    f32x4 bas;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bas[r] = fmaxf(l1[r], 0.f);
      bh[r] = dca::f2bf(bas[r]);
      bl[r] = dca::f2bf(bas[r] - dca::bf2f(bh[r]));
    }
    // ∂W_τᵀ[j][e] += Σ_rows basic[row][j] · ∂emb[row][e]
#pragma unroll
    for (int et = 0; et < 8; ++et) {
      acc[et] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(bl, eh[et], acc[et], 0, 0, 0);
      acc[et] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(bh, el[et], acc[et], 0, 0, 0);
      acc[et] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(bh, eh[et], acc[et], 0, 0, 0);
    }
    bf16x4 a, al;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      c[r] = bas[r] > 0.f ? c[r] : 0.f;
      a[r] = dca::f2bf(c[r]);
      al[r] = dca::f2bf(c[r] - dca::bf2f(a[r]));
      db1acc += c[r];
    }
    // ∂W1[j][f] += Σ_rows ∂basic[row][j] · units[row][f]
    dw1acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(al, ub, dw1acc, 0, 0, 0);
    dw1acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, ubl, dw1acc, 0, 0, 0);
    dw1acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, ub, dw1acc, 0, 0, 0);
    buf ^= 1;
  }
  // ---- partials: ∂W_τ tile-linear ((wv·8 + et)·64 + lane)·4 + r; ∂W1 rows j of this wave's tile, ∂b1
  float* dst = P.dwtpart + (size_t)job * (kD * kD);
#pragma unroll
  for (int et = 0; et < 8; ++et) *reinterpret_cast<f32x4*>(dst + ((8 * wv + et) * 64 + lane) * 4) = acc[et];
  float* wp = P.w1part + (size_t)job * kW1;
  if (i < kF) {
#pragma unroll
    for (int r = 0; r < 4; ++r) wp[(16 * wv + 4 * kg + r) * kF + i] = dw1acc[r];
  }
  float s = db1acc;
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  if (kg == 0) wp[kD * kF + 16 * wv + i] = s;
}

// F32 forward over item ranges (same organisation as the fused backward): a workgroup of 8 waves owns whole 16-row
// groups of ONE type τ and walks its (row group, unit) items; per item
//   * wave w computes basic tile w (layer 1, one 16x16x32 MFMA on the bf16-split unit features staged in LDS two
//     items ahead) → ReLU → hi / lo transposed image (double-buffered, one item ahead);
//   * wave w computes output columns 16w … 16w+15 of emb = basic·W_τᵀ + b_τ (bf16x3 over K = 128, A fragments by
//     ds_read_b64_tr_b16), stores them (fp32) and keeps the running max / argmax over the group's units in
//     registers, flushed to x896 / arg after the group's last unit.
struct FfParams {
  const float* units;
  const float* env;
  const float* w1;
  const float* b1;
  const float* wt;       // (6, 128, 128) fp32 W_τ (out, in)
  const float* bt;
  const float* we;
  const float* be;
  float* x896;
  float* emb;
  unsigned char* arg;
  int N;
  Layout L;
  int gpj[6];            // row groups per job of each type
  int jbase[7];
};

__device__ __forceinline__ float ff_stage_load(const FfParams& P, __amdgpu_buffer_rsrc_t Ru, int k, int cnt, int uoff,
                                              int wv, int lane) {
  const int idx = min(64 * min(wv, 2) + lane, 16 * kF - 1);
  const int rb = k / cnt, u = k - rb * cnt;
  const int row = min(16 * rb + idx / kF, P.N - 1);
  return bload(Ru, ((row * P.L.U + uoff + u) * kF + idx % kF) * 4);
}

// layer 1 of basic tile wv for the staged item → ReLU → hi / lo image
__device__ __forceinline__ void ff_layer1(const float* sl, const bf16x8& wb, short* ih, short* il, int wv, int lane) {
  const int i = lane & 15, kg = lane >> 4;
  bf16x8 a1;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    const int slot = 8 * kg + jj;
    const float x = sl[i * kF + max(l1_feat(slot), 0)];
    const short hi = dca::f2bf(x);
    const short lo = dca::f2bf(x - dca::bf2f(hi));
    a1[jj] = l1_feat(slot) < 0 ? (short)0x3F80 : (l1_xlo(slot) ? lo : hi);
  }
  const f32x4 l1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, wb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  f32x4 b;
#pragma unroll
  for (int r = 0; r < 4; ++r) b[r] = fmaxf(l1[r], 0.f);
  tile_put(ih, wv, b, lane);
  tile_put_lo(il, wv, b, lane);
}

__global__ __launch_bounds__(512, 1) void encoder_fwd_f32_items_kernel(FfParams P) {
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int i = lane & 15, kg = lane >> 4;
  const int job = blockIdx.x, N = P.N, U = P.L.U;
  // env embedding (fp32 VALU): 32-row blocks strided over the jobs
  for (int rbase = 32 * job; rbase < N; rbase += 32 * (int)gridDim.x) {
    const int row = rbase + (tid >> 4), c0 = (tid & 15) * 8;
    if (row < N) {
      const float e0 = P.env[row * 3], e1 = P.env[row * 3 + 1], e2 = P.env[row * 3 + 2];
#pragma unroll
      for (int c = c0; c < c0 + 8; ++c)
        P.x896[(size_t)row * 896 + c] = fmaxf(P.be[c] + P.we[c * 3] * e0 + P.we[c * 3 + 1] * e1 + P.we[c * 3 + 2] * e2, 0.f);
    }
  }
  int tau = 0;
#pragma unroll
  for (int t = 1; t < 6; ++t) tau += job >= P.jbase[t] ? 1 : 0;
  if (job >= P.jbase[6]) return;
  const int cnt = P.L.cnt[tau], uoff = P.L.off[tau];
  const int NB = (N + 15) >> 4;
  const int g0 = (job - P.jbase[tau]) * P.gpj[tau], g1 = min(g0 + P.gpj[tau], NB);
  const int k0 = g0 * cnt, k1 = g1 * cnt, kl = k1 - 1;
  __shared__ __attribute__((aligned(16))) short img[2][2][kImg];
  __shared__ __attribute__((aligned(16))) float stg[3][kStg];

  const int col = 16 * wv + i;
  bf16x8 wf[4], wfl[4], wb;
#pragma unroll
  for (int s = 0; s < 4; ++s) {   // B[k = j][n = out] = W_τ[out][j]
    const float* p = P.wt + ((size_t)tau * kD + col) * kD + 32 * s + 8 * kg;
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      wf[s][jj] = dca::f2bf(v[jj]);
      wfl[s][jj] = dca::f2bf(v[jj] - dca::bf2f(wf[s][jj]));
    }
  }
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    const int slot = 8 * kg + jj, f = l1_feat(slot);
    const float w = f >= 0 ? P.w1[col * kF + f] : P.b1[col];
    const short hi = dca::f2bf(w);
    const short lo = dca::f2bf(w - dca::bf2f(hi));
    wb[jj] = (slot == 31 || (f >= 0 && l1_wlo(slot))) ? lo : hi;
  }
  const float btv = P.bt[tau * kD + col];
  const __amdgpu_buffer_rsrc_t Ru = uniform_rsrc(P.units, N * U * kF * 4),
                               Re = uniform_rsrc(P.emb, N * U * kD * 4);
  f32x4 pmax = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  int parg[4] = {0, 0, 0, 0};

  // staging as in the fused backward: waves 0-2 write item k+2's unit rows at item k, loaded one item earlier
  float pre = 0.f;
  if (wv < 3) {
    stg[k0 % 3][64 * wv + lane] = ff_stage_load(P, Ru, k0, cnt, uoff, wv, lane);
    stg[(k0 + 1) % 3][64 * wv + lane] = ff_stage_load(P, Ru, min(k0 + 1, kl), cnt, uoff, wv, lane);
    pre = ff_stage_load(P, Ru, min(k0 + 2, kl), cnt, uoff, wv, lane);
  }
  lds_barrier();
  ff_layer1(stg[k0 % 3], wb, &img[0][0][0], &img[0][1][0], wv, lane);
  int buf = 0;
  for (int k = k0; k < k1; ++k) {
    lds_barrier();   // image k complete; staging slot of k + 1 written
    if (wv < 3) {
      stg[(k + 2) % 3][64 * wv + lane] = pre;
      pre = ff_stage_load(P, Ru, min(k + 3, kl), cnt, uoff, wv, lane);
    }
    const int rb = k / cnt, u = k - rb * cnt, row0 = 16 * rb;
    const short* ih = &img[buf][0][0];
    const short* il = &img[buf][1][0];
    bf16x8 af[4], afl[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      af[s] = tile_frag(ih, 32 * s, lane);
      afl[s] = tile_frag(il, 32 * s, lane);
    }
    const f32x4 c = mfma3_k128(af, afl, wf, wfl);
    // next item's basic tile into the other image (past the range's end: a rewrite nobody reads)
    ff_layer1(stg[(k + 1) % 3], wb, &img[buf ^ 1][0][0], &img[buf ^ 1][1][0], wv, lane);
    // emb stores are bounds-checked buffer stores (rows past N are dropped): no per-row branches
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = c[r] + btv;
      if (v > pmax[r]) { pmax[r] = v; parg[r] = u; }
      const int row = row0 + 4 * kg + r;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), Re, ((row * U + uoff + u) * kD + col) * 4,
                                            0, 0);
    }
    if (u == cnt - 1) {   // the group's last unit: pools + argmax
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 4 * kg + r;
        if (row < N) {
          P.x896[(size_t)row * 896 + kD + tau * kD + col] = pmax[r];
          P.arg[((size_t)row * 6 + tau) * kD + col] = (unsigned char)parg[r];
        }
        pmax[r] = -INFINITY;
        parg[r] = 0;
      }
    }
    buf ^= 1;
  }
}

// ============================================================================================================
// EXACT variants (the IEEE-fp32 learner, precision='fp32-exact'): the same item-range organisation as the F32 kernels
// above, but every product is an IEEE fp32 fma on v_mfma_f32_16x16x4_f32 (bit-for-bit a k-ordered fmaf chain) —
// no bf16 split anywhere. A 16x16x4 f32 fragment is ONE float per lane, A[m = l&15][k = l>>4] / B[k = l>>4][n = l&15],
// so:
//   * layer 1 (K = 10 features + bias) is 3 calls, call c taking feature 4c + (l>>4) (slot 10 = the bias against a
//     1.0 operand, slot 11 = 0);
//   * layer 2 (K = 128) is 32 calls: call (s, jj) takes k = 32s + 8·(l>>4) + jj, so the A operand of a lane is 8
//     consecutive floats of ONE basic row per s — two ds_read_b128 from a row-major fp32 tile image — and the weight
//     operand is 32 floats per lane held in VGPRs for the whole job (the bf16x3 kernels' hi + lo images: same 32 VGPRs);
//   * the C-layout tiles (column on the lane, rows 4(l>>4) … +3 in the registers) are directly the A / B operands of
//     the row-reduction products (∂W_τᵀ = basicᵀ·∂emb, ∂W1 = ∂basicᵀ·units): call r takes row 4(l>>4) + r.
// Weight-gradient sums are two-level: each item's 16-row product starts from zero and is added into the job's running
// sum (a 16-long fma chain per item, then one add per item), then the per-job partials go through the fixed-order
// reduces shared with the F32 kernels. MFMA work per item is 5.3x the bf16x3 kernels' (the f32 MFMA rate is 1/16 of
// bf16), so these are MFMA-bound where the bf16x3 ones are latency-bound.
constexpr int kXP = 132;                     // row pitch (floats) of the row-major fp32 tile image [16 rows][128]
constexpr int kXT = 20;                      // row pitch (floats) of the transposed image [128 columns][16 rows]

// layer 1 of the staged item for basic tile wv (exact): 3 f32 MFMAs, C layout (rows 4kg + r, column 16wv + i)
__device__ __forceinline__ f32x4 x_layer1(const float* sl, const float (&w1x)[3], int i, int kg) {
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int cc = 0; cc < 3; ++cc) {
    const int f = 4 * cc + kg;
    const float a = f < kF ? sl[i * kF + f] : (f == kF ? 1.f : 0.f);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w1x[cc], c, 0, 0, 0);
  }
  return c;
}

__device__ __forceinline__ void x_load_w1(const float* w1, const float* b1, int col, int kg, float (&w1x)[3]) {
#pragma unroll
  for (int cc = 0; cc < 3; ++cc) {
    const int f = 4 * cc + kg;
    w1x[cc] = f < kF ? w1[col * kF + f] : (f == kF ? b1[col] : 0.f);
  }
}

// A operand of a 16×128 row-major fp32 image for 32 calls: lane (row i, kg) gets columns 32s + 8kg … +7 per s
__device__ __forceinline__ void x_afrags(const float* img, int i, int kg, float (&a)[32]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const float4 p = *reinterpret_cast<const float4*>(img + i * kXP + 32 * s + 8 * kg);
    const float4 q = *reinterpret_cast<const float4*>(img + i * kXP + 32 * s + 8 * kg + 4);
    a[8 * s + 0] = p.x; a[8 * s + 1] = p.y; a[8 * s + 2] = p.z; a[8 * s + 3] = p.w;
    a[8 * s + 4] = q.x; a[8 * s + 5] = q.y; a[8 * s + 6] = q.z; a[8 * s + 7] = q.w;
  }
}

// 16 × 128 product over K = 128 against the weight fragments: two interleaved accumulators (the f32 MFMA's
// dependent latency is 40 cycles against a 32-cycle issue), summed at the end
__device__ __forceinline__ f32x4 x_mma_k128(const float (&a)[32], const float (&w)[32]) {
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 32; k += 2) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[k], w[k], c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[k + 1], w[k + 1], c1, 0, 0, 0);
  }
  return c0 + c1;
}

// C-layout fragment (rows 4kg + r, column 16n + i) → row-major image (4 dword stores)
__device__ __forceinline__ void x_put(float* img, int n, const f32x4& v, int i, int kg) {
#pragma unroll
  for (int r = 0; r < 4; ++r) img[(4 * kg + r) * kXP + 16 * n + i] = v[r];
}

__global__ __launch_bounds__(512, 1) void encoder_fwd_x_kernel(FfParams P) {
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int i = lane & 15, kg = lane >> 4;
  const int job = blockIdx.x, N = P.N, U = P.L.U;
  for (int rbase = 32 * job; rbase < N; rbase += 32 * (int)gridDim.x) {     // env embedding (fp32 VALU)
    const int row = rbase + (tid >> 4), c0 = (tid & 15) * 8;
    if (row < N) {
      const float e0 = P.env[row * 3], e1 = P.env[row * 3 + 1], e2 = P.env[row * 3 + 2];
#pragma unroll
      for (int c = c0; c < c0 + 8; ++c)
        P.x896[(size_t)row * 896 + c] = fmaxf(P.be[c] + P.we[c * 3] * e0 + P.we[c * 3 + 1] * e1 + P.we[c * 3 + 2] * e2, 0.f);
    }
  }
  int tau = 0;
#pragma unroll
  for (int t = 1; t < 6; ++t) tau += job >= P.jbase[t] ? 1 : 0;
  if (job >= P.jbase[6]) return;
  const int cnt = P.L.cnt[tau], uoff = P.L.off[tau];
  const int NB = (N + 15) >> 4;
  const int g0 = (job - P.jbase[tau]) * P.gpj[tau], g1 = min(g0 + P.gpj[tau], NB);
  const int k0 = g0 * cnt, k1 = g1 * cnt, kl = k1 - 1;
  __shared__ __attribute__((aligned(16))) float img[2][16 * kXP];
  __shared__ __attribute__((aligned(16))) float stg[3][kStg];

  const int col = 16 * wv + i;
  float wx[32], w1x[3];
#pragma unroll
  for (int s = 0; s < 4; ++s) {   // B[k = j][n = out] = W_τ[out][j], k = 32s + 8kg + jj
    const float* p = P.wt + ((size_t)tau * kD + col) * kD + 32 * s + 8 * kg;
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    wx[8 * s + 0] = a.x; wx[8 * s + 1] = a.y; wx[8 * s + 2] = a.z; wx[8 * s + 3] = a.w;
    wx[8 * s + 4] = b.x; wx[8 * s + 5] = b.y; wx[8 * s + 6] = b.z; wx[8 * s + 7] = b.w;
  }
  x_load_w1(P.w1, P.b1, col, kg, w1x);
  const float btv = P.bt[tau * kD + col];
  const __amdgpu_buffer_rsrc_t Ru = uniform_rsrc(P.units, N * U * kF * 4),
                               Re = uniform_rsrc(P.emb, N * U * kD * 4);
  f32x4 pmax = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  int parg[4] = {0, 0, 0, 0};

  float pre = 0.f;
  if (wv < 3) {
    stg[k0 % 3][64 * wv + lane] = ff_stage_load(P, Ru, k0, cnt, uoff, wv, lane);
    stg[(k0 + 1) % 3][64 * wv + lane] = ff_stage_load(P, Ru, min(k0 + 1, kl), cnt, uoff, wv, lane);
    pre = ff_stage_load(P, Ru, min(k0 + 2, kl), cnt, uoff, wv, lane);
  }
  lds_barrier();
  {
    f32x4 b = x_layer1(stg[k0 % 3], w1x, i, kg);
#pragma unroll
    for (int r = 0; r < 4; ++r) b[r] = fmaxf(b[r], 0.f);
    x_put(img[0], wv, b, i, kg);
  }
  // the weight / bias loads have landed: no first-iteration wait left inside the loop (where it would stay as a
  // vmcnt(0) before the emb stores of every item, waiting out the previous item's stores)
  __builtin_amdgcn_s_waitcnt(0);
  int buf = 0;
  for (int k = k0; k < k1; ++k) {
    lds_barrier();   // image k complete; staging slot of k + 1 written
    const int rb = k / cnt, u = k - rb * cnt, row0 = 16 * rb;
    float a[32];
    x_afrags(img[buf], i, kg, a);
    const f32x4 c = x_mma_k128(a, wx);
    // staging of item k + 2 (slot (k - 1) % 3, free in this iteration), loaded at the end of the previous iteration
    // AFTER its emb stores: waiting for it does not wait for stores issued later (vmcnt also counts stores on
    // gfx950), and the next load is issued after this item's stores for the same reason
    if (wv < 3) stg[(k + 2) % 3][64 * wv + lane] = pre;
    {   // next item's basic tile into the other image (past the range's end: a rewrite nobody reads)
      f32x4 b = x_layer1(stg[(k + 1) % 3], w1x, i, kg);
#pragma unroll
      for (int r = 0; r < 4; ++r) b[r] = fmaxf(b[r], 0.f);
      x_put(img[buf ^ 1], wv, b, i, kg);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = c[r] + btv;
      if (v > pmax[r]) { pmax[r] = v; parg[r] = u; }
      const int row = row0 + 4 * kg + r;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), Re, ((row * U + uoff + u) * kD + col) * 4,
                                            0, 0);
    }
    if (u == cnt - 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 4 * kg + r;
        if (row < N) {
          P.x896[(size_t)row * 896 + kD + tau * kD + col] = pmax[r];
          P.arg[((size_t)row * 6 + tau) * kD + col] = (unsigned char)parg[r];
        }
        pmax[r] = -INFINITY;
        parg[r] = 0;
      }
    }
    if (wv < 3) pre = ff_stage_load(P, Ru, min(k + 3, kl), cnt, uoff, wv, lane);
    buf ^= 1;
  }
}

// ∂emb e-tile wv of item k (C layout) → row-major image (∂basic's A operand) and transposed image (the ∂W_τ
// products' B operand: one b128 of rows 4kg … 4kg+3 per lane and tile). GIVEN: the item's ∂emb as loaded (the
// entity-attention path hands the encoder ∂E0 instead of the pointer / pool gradients)
template <bool GIVEN>
__device__ __forceinline__ void xb_build(const FbBuild& b, const float* slot, int u, float* im, float* it, int wv,
                                         int lane) {
  const int i = lane & 15, kg = lane >> 4;
  f32x4 v;
  if constexpr (GIVEN) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = b.q[r];
  } else {
    const f32x4 d4 = *reinterpret_cast<const f32x4*>(slot + 16 * kF + 4 * kg);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = d4[r] * b.q[r] + (b.ab[r] == (unsigned)u ? b.ds[r] : 0.f);
  }
  x_put(im, wv, v, i, kg);
  *reinterpret_cast<f32x4*>(it + (16 * wv + i) * kXT + 4 * kg) = v;
}

// Exact encoder backward, 4-wave form (two workgroups per CU; an 8-wave one-per-CU form measured slower and was
// removed in round 5): wave w owns basic-column tiles 2w, 2w+1 and builds
// e-tiles 2w, 2w+1 of the item's ∂emb images. The item's A fragments (∂emb rows) and transposed ∂emb tiles are read
// once per wave for two column tiles (half the LDS traffic per MFMA), and the two resident workgroups work on
// different items, so one's barrier / staging phases overlap the other's MFMAs (the 8-wave form keeps both waves of
// a SIMD in lockstep: ≈55 % MFMA busy). Same products, same per-item two-level sums, same partial layouts.
// GIVEN: ∂emb read from P.demb_in (the 5v5 entity-attention step, ∂E0 of the attention block) instead of built from
// the pointer / pool gradients.
template <bool GIVEN, bool COMPAT>
__global__ __launch_bounds__(256, 2) void encoder_bwd_x2_kernel(FbParams P) {
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int i = lane & 15, kg = lane >> 4;
  const int job = blockIdx.x;
  int tau = 0;
#pragma unroll
  for (int t = 1; t < 6; ++t) tau += job >= P.jbase[t] ? 1 : 0;
  const int cnt = P.L.cnt[tau], uoff = P.L.off[tau], N = P.N, U = P.L.U;
  const int NB = (N + 15) >> 4;
  const int k0 = (job - P.jbase[tau]) * P.items, k1 = min(k0 + P.items, cnt * NB);
  __shared__ __attribute__((aligned(16))) float img[2][16 * kXP];
  __shared__ __attribute__((aligned(16))) float imt[2][128 * kXT];
  __shared__ __attribute__((aligned(16))) float stg[3][kStg];
  FbRsrc R;
  if constexpr (GIVEN) {
    R.g = uniform_rsrc(P.demb_in, N * U * kD * 4);
  } else {
    R.q = uniform_rsrc(P.q, N * P.ldq * 4);
    R.x = uniform_rsrc(P.dx, N * 896 * 4);
    R.a = uniform_rsrc(P.arg, N * 6 * kD);
  }

  float wx[2][32], w1x[2][3];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int col = 16 * (2 * w + t) + i;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float* p = P.wtT + ((size_t)tau * kD + col) * kD + 32 * s + 8 * kg;
      const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
      wx[t][8 * s + 0] = a.x; wx[t][8 * s + 1] = a.y; wx[t][8 * s + 2] = a.z; wx[t][8 * s + 3] = a.w;
      wx[t][8 * s + 4] = b.x; wx[t][8 * s + 5] = b.y; wx[t][8 * s + 6] = b.z; wx[t][8 * s + 7] = b.w;
    }
    x_load_w1(P.w1, P.b1, col, kg, w1x[t]);
  }
  f32x4 acc[2][8], dw1acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  float db1acc[2] = {0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int et = 0; et < 8; ++et) acc[t][et] = f32x4{0.f, 0.f, 0.f, 0.f};

  FbBuild bn[2];
  const int kl = max(k1 - 1, 0);
  float pre = 0.f;
  if (w < 3) {
    stg[k0 % 3][64 * w + lane] = fb_stage_load(P, min(k0, kl), cnt, uoff, w, lane);
    stg[(k0 + 1) % 3][64 * w + lane] = fb_stage_load(P, min(k0 + 1, kl), cnt, uoff, w, lane);
    pre = fb_stage_load(P, min(k0 + 2, kl), cnt, uoff, w, lane);
  }
#pragma unroll
  for (int t = 0; t < 2; ++t)
    fb_load_build<GIVEN, COMPAT>(bn[t], R, P.ldq, min(k0, kl), true, cnt, uoff, U, tau, 2 * w + t, i, kg);
  lds_barrier();
#pragma unroll
  for (int t = 0; t < 2; ++t) xb_build<GIVEN>(bn[t], stg[k0 % 3], k0 % cnt, img[0], imt[0], 2 * w + t, lane);
#pragma unroll
  for (int t = 0; t < 2; ++t)
    fb_load_build<GIVEN, COMPAT>(bn[t], R, P.ldq, min(k0 + 1, kl), min(k0 + 1, kl) % cnt == 0, cnt, uoff, U, tau,
                                 2 * w + t, i, kg);
  float l1n[3], ubn[4];
  auto l1_read = [&](const float* sl) {
#pragma unroll
    for (int cc = 0; cc < 3; ++cc) {
      const int f = 4 * cc + kg;
      l1n[cc] = f < kF ? sl[i * kF + f] : (f == kF ? 1.f : 0.f);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) ubn[r] = i < kF ? sl[(4 * kg + r) * kF + i] : 0.f;
  };
  l1_read(stg[k0 % 3]);
  int buf = 0;
  for (int k = k0; k < k1; ++k) {
    lds_barrier();
    float a[32];
    x_afrags(img[buf], i, kg, a);                 // ∂emb[row i][e], e = 32s + 8kg + jj (both column tiles)
    const float ub[4] = {ubn[0], ubn[1], ubn[2], ubn[3]};
    f32x4 bas[2], c[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      bas[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) bas[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(l1n[cc], w1x[t][cc], bas[t], 0, 0, 0);
    }
    {   // ∂basic (before ReLU') of both tiles: the two tiles' chains interleaved (even / odd k summed at the end, as
        // the 8-wave form does)
      f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, d0 = c0, d1 = c0;
#pragma unroll
      for (int kk = 0; kk < 32; kk += 2) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kk], wx[0][kk], c0, 0, 0, 0);
        d0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kk], wx[1][kk], d0, 0, 0, 0);
      }
#pragma unroll
      for (int kk = 1; kk < 32; kk += 2) {
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kk], wx[0][kk], c1, 0, 0, 0);
        d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kk], wx[1][kk], d1, 0, 0, 0);
      }
      c[0] = c0 + c1;
      c[1] = d0 + d1;
    }
    f32x4 et4[8];
#pragma unroll
    for (int et = 0; et < 8; ++et) et4[et] = *reinterpret_cast<const f32x4*>(imt[buf] + (16 * et + i) * kXT + 4 * kg);
    if (w < 3) stg[(k + 2) % 3][64 * w + lane] = pre;
#pragma unroll
    for (int t = 0; t < 2; ++t)
      xb_build<GIVEN>(bn[t], stg[(k + 1) % 3], min(k + 1, kl) % cnt, img[buf ^ 1], imt[buf ^ 1], 2 * w + t, lane);
#pragma unroll
    for (int t = 0; t < 2; ++t)
      fb_load_build<GIVEN, COMPAT>(bn[t], R, P.ldq, min(k + 2, kl), k + 2 <= kl && (k + 2) % cnt == 0, cnt, uoff, U,
                                   tau, 2 * w + t, i, kg);
    l1_read(stg[(k + 1) % 3]);
    if (w < 3) pre = fb_stage_load(P, min(k + 3, kl), cnt, uoff, w, lane);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) bas[t][r] = fmaxf(bas[t][r], 0.f);
    // ∂W_τᵀ[j][e] += Σ_rows basic[row][j]·∂emb[row][e], per item from zero then added; the two tiles' chains of an
    // e-tile interleaved
#pragma unroll
    for (int et = 0; et < 8; ++et) {
      f32x4 p0 = __builtin_amdgcn_mfma_f32_16x16x4f32(bas[0][0], et4[et][0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      f32x4 p1 = __builtin_amdgcn_mfma_f32_16x16x4f32(bas[1][0], et4[et][0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
      for (int r = 1; r < 4; ++r) {
        p0 = __builtin_amdgcn_mfma_f32_16x16x4f32(bas[0][r], et4[et][r], p0, 0, 0, 0);
        p1 = __builtin_amdgcn_mfma_f32_16x16x4f32(bas[1][r], et4[et][r], p1, 0, 0, 0);
      }
      acc[0][et] += p0;
      acc[1][et] += p1;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        c[t][r] = bas[t][r] > 0.f ? c[t][r] : 0.f;
        db1acc[t] += c[t][r];
      }
      f32x4 p1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) p1 = __builtin_amdgcn_mfma_f32_16x16x4f32(c[t][r], ub[r], p1, 0, 0, 0);
      dw1acc[t] += p1;
    }
    buf ^= 1;
  }
  float* dst = P.dwtpart + (size_t)job * (kD * kD);
  float* wp = P.w1part + (size_t)job * kW1;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int jt = 2 * w + t;
#pragma unroll
    for (int et = 0; et < 8; ++et) *reinterpret_cast<f32x4*>(dst + ((8 * jt + et) * 64 + lane) * 4) = acc[t][et];
    if (i < kF) {
#pragma unroll
      for (int r = 0; r < 4; ++r) wp[(16 * jt + 4 * kg + r) * kF + i] = dw1acc[t][r];
    }
    float s = db1acc[t];
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    if (kg == 0) wp[kD * kF + 16 * jt + i] = s;
  }
}

// Fixed-order sum of a type's fused-backward partials (tile-linear → ∂W_τ[e][j]); 4 job phases per block as dwt_reduce.
__global__ __launch_bounds__(256) void fb_dwt_reduce(const float* __restrict__ part, FbParams P, float* __restrict__ dwt) {
  __shared__ float red[4][64];
  const int tau = blockIdx.y, ph = threadIdx.x >> 6;
  const int xi = blockIdx.x * 64 + (threadIdx.x & 63);
  float s = 0.f;
#pragma unroll 4
  for (int j = P.jbase[tau] + ph; j < P.jbase[tau + 1]; j += 4) s += part[(size_t)j * (kD * kD) + xi];
  red[ph][threadIdx.x & 63] = s;
  __syncthreads();
  if (ph) return;
  s = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
  const int r = xi & 3, lane = (xi >> 2) & 63, tile = xi >> 8;
  const int j = 16 * (tile >> 3) + 4 * (lane >> 4) + r;
  const int e = 16 * (tile & 7) + (lane & 15);
  dwt[(size_t)tau * kD * kD + e * kD + j] = s;
}

// Fixed-order sum of the per-workgroup ∂W1‖∂b1 partials: block of 256 = 16 columns × 16 row phases (88 blocks;
// 64 × 4 gave 22 blocks whose threads each walked ~90 partials: 23 µs, latency-bound).
__global__ __launch_bounds__(256) void encoder_w1_reduce(const float* __restrict__ part, int nblk,
                                                          float* __restrict__ dw1, float* __restrict__ db1) {
  __shared__ float red[16][16];
  const int c = blockIdx.x * 16 + (threadIdx.x & 15), ph = threadIdx.x >> 4;
  float s = 0.f;
  if (c < kW1) {
#pragma unroll 4
    for (int b = ph; b < nblk; b += 16) s += part[(size_t)b * kW1 + c];
  }
  red[ph][threadIdx.x & 15] = s;
  __syncthreads();
  if (ph == 0 && c < kW1) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) v += red[k][threadIdx.x];
    if (c < kD * kF) dw1[c] = v;
    else db1[c - kD * kF] = v;
  }
}


// ============================================================================================================
// ∂W_τ = Σ_k ∂emb[k]ᵀ · basic[k] over the K-blocked images (K = units of τ × rows): split-K over jobs of kJobBlk
// 16-row blocks; a workgroup's 4 waves own the four 64×64 quadrants of the 128×128 output (16 MFMA tiles each,
// operands straight from HBM/L2 as 16-B fragments, next k-step prefetched into registers). Each job writes its
// partial tile-linearly; dwt_reduce sums a type's partials in job order (deterministic).
constexpr int kJobBlk = 64;
struct DwtJobs {
  long long blkbase[6];
  int nblk[6];
  int jbase[7];
};

__device__ __forceinline__ void dwt_load(const short* __restrict__ A, const short* __restrict__ Bm, long long b,
                                         long long bend, int mq, int nq, int lane, bf16x8 (&a)[4], bf16x8 (&bb)[4]) {
  const long long blk = b + (lane >> 5);
  const bool ok = blk < bend;
  const int kh = 8 * ((lane >> 4) & 1);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const size_t oa = ((size_t)blk * kD + 64 * mq + 16 * t + (lane & 15)) * 16 + kh;
    const size_t ob = ((size_t)blk * kD + 64 * nq + 16 * t + (lane & 15)) * 16 + kh;
    a[t] = ok ? *reinterpret_cast<const bf16x8*>(A + oa) : bf16x8{};
    bb[t] = ok ? *reinterpret_cast<const bf16x8*>(Bm + ob) : bf16x8{};
  }
}

__global__ __launch_bounds__(256, 2) void dwt_blocked_kernel(const short* __restrict__ A, const short* __restrict__ Bm,
                                                             DwtJobs J, float* __restrict__ part) {
  const int job = blockIdx.x, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int tau = 0;
  while (tau < 5 && job >= J.jbase[tau + 1]) ++tau;
  const long long b0 = J.blkbase[tau] + (long long)(job - J.jbase[tau]) * kJobBlk;
  const long long bend = min(b0 + kJobBlk, J.blkbase[tau] + J.nblk[tau]);
  const int mq = wv >> 1, nq = wv & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[4], bb[4], an[4], bn[4];
  dwt_load(A, Bm, b0, bend, mq, nq, lane, a, bb);
  for (long long b = b0; b < bend; b += 2) {
    if (b + 2 < bend) dwt_load(A, Bm, b + 2, bend, mq, nq, lane, an, bn);
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[x], bb[y], acc[x][y], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      a[t] = an[t];
      bb[t] = bn[t];
    }
  }
  // tile-linear partial: ((wave·16 + 4x + y)·64 + lane)·4 + r
  float* dst = part + (size_t)job * (kD * kD) + (size_t)wv * 16 * 256;
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) *reinterpret_cast<f32x4*>(dst + ((4 * x + y) * 64 + lane) * 4) = acc[x][y];
}

// 64 elements × 4 job phases per block (a phase sums every 4th job, the phases combine in a fixed order through LDS):
// 4× the parallelism of one thread per element over up to 175 jobs, still deterministic.
__global__ __launch_bounds__(256) void dwt_reduce(const float* __restrict__ part, DwtJobs J, float* __restrict__ dwt) {
  __shared__ float red[4][64];
  const int tau = blockIdx.y, ph = threadIdx.x >> 6;
  const int xi = blockIdx.x * 64 + (threadIdx.x & 63);  // tile-linear element
  float s = 0.f;
#pragma unroll 4
  for (int j = J.jbase[tau] + ph; j < J.jbase[tau + 1]; j += 4) s += part[(size_t)j * (kD * kD) + xi];
  red[ph][threadIdx.x & 63] = s;
  __syncthreads();
  if (ph) return;
  s = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
  const int r = xi & 3, lane = (xi >> 2) & 63, tile = (xi >> 8) & 15, wv = xi >> 12;
  const int m = 64 * (wv >> 1) + 16 * (tile >> 2) + 4 * (lane >> 4) + r;
  const int n = 64 * (wv & 1) + 16 * (tile & 3) + (lane & 15);
  dwt[(size_t)tau * kD * kD + m * kD + n] = s;
}

}  // namespace

// f32 = 1: wt fp32, x896 / emb fp32 (bf16x3 layer 2); f32 = 2: the same, exact fp32 MFMA; f32 = 0: wt, x896, emb bf16
extern "C" hipError_t dca_encoder_fwd(const float* units, const float* env, const float* w1, const float* b1,
                                      const void* wt, const float* bt, const float* we, const float* be, void* x896,
                                      void* emb, unsigned char* arg, int N, int U, const int* counts, int compat,
                                      hipStream_t st, int f32) {
  FwdParams P{units, env, w1, b1, wt, bt, we, be, x896, emb, arg, N, compat, {}};
  P.L.U = U;
  int acc = 0;
  for (int t = 0; t < 6; ++t) { P.L.cnt[t] = counts[t]; P.L.off[t] = acc; acc += counts[t]; }
  if (acc != U || U > 64) return hipErrorInvalidValue;
  // (row block, type job) grid: 3× the workgroups of a row-block grid, so small batches (the actor's few thousand
  // rows) still fill the 256 CUs, and heavy jobs (16-unit types, dispatched first) are balanced by the light ones
  if (f32) {
    FfParams F{units, env, w1, b1, static_cast<const float*>(wt), bt, we, be, static_cast<float*>(x896),
               static_cast<float*>(emb), arg, N, P.L, {}, {}};
    const long long NB = (N + 15) / 16;
    long long total = 0;
    for (int t = 0; t < 6; ++t) total += counts[t] * NB;
    const long long target = std::max<long long>(1, (total + 499) / 500);   // ≈500 equal jobs (cf. fb_plan)
    int jobs = 0;
    for (int t = 0; t < 6; ++t) {
      F.jbase[t] = jobs;
      F.gpj[t] = (int)((target + std::max(1, counts[t]) - 1) / std::max(1, counts[t]));
      if (counts[t] > 0) jobs += (int)((NB + F.gpj[t] - 1) / F.gpj[t]);
    }
    F.jbase[6] = jobs;
    // every launch also covers the env embedding (32-row blocks strided over the grid)
    if (f32 == 2) encoder_fwd_x_kernel<<<std::max(jobs, 1), 512, 0, st>>>(F);
    else encoder_fwd_f32_items_kernel<<<std::max(jobs, 1), 512, 0, st>>>(F);
    return hipGetLastError();
  }
  const dim3 grid((N + kRows - 1) / kRows, kJobs);
  encoder_fwd_kernel<<<grid, 256, 0, st>>>(P);
  return hipGetLastError();
}

namespace {
void dwt_plan(int N, const int* counts, DwtJobs& J, int& NB) {
  NB = (N + 15) / 16;
  long long acc = 0;
  int jobs = 0;
  for (int t = 0; t < 6; ++t) {
    J.blkbase[t] = acc;
    J.nblk[t] = counts[t] * NB;
    J.jbase[t] = jobs;
    acc += J.nblk[t];
    jobs += (J.nblk[t] + kJobBlk - 1) / kJobBlk;
  }
  J.jbase[6] = jobs;
}

void fb_plan(int N, const int* counts, FbParams& P) {
  const long long NB = (N + 15) / 16;
  long long total = 0;
  for (int t = 0; t < 6; ++t) total += counts[t] * NB;
  // ≈500 equal jobs: two rounds of one workgroup per CU (VGPR-bound occupancy), + at most one tail job per type
  P.items = (int)std::max<long long>(1, (total + 499) / 500);
  int jobs = 0;
  for (int t = 0; t < 6; ++t) {
    P.jbase[t] = jobs;
    jobs += (int)((counts[t] * NB + P.items - 1) / P.items);
  }
  P.jbase[6] = jobs;
}
}  // namespace

// Workspace. bf16: ∂W1 partials ‖ K-blocked ∂emb and basic images ‖ ∂W_τ split-K partials. F32 (fused ∂W_τ):
// per job one ∂W1‖∂b1 partial and one 128×128 ∂W_τ partial.
extern "C" size_t dca_encoder_bwd_workspace(int N, int U, const int* counts, int f32) {
  if (f32) {
    FbParams F{};
    fb_plan(N, counts, F);
    return (size_t)F.jbase[6] * (kW1 + kD * kD) * sizeof(float);
  }
  DwtJobs J;
  int NB;
  dwt_plan(N, counts, J, NB);
  const size_t w1 = (size_t)((N + kRows - 1) / kRows) * kJobs * kW1 * sizeof(float);
  const size_t img = (size_t)U * NB * kD * 16 * sizeof(short);
  const size_t parts = (size_t)J.jbase[6] * kD * kD * sizeof(float);
  return w1 + 2 * img + parts;
}

extern "C" hipError_t dca_encoder_bwd(const float* units, const float* w1, const float* b1, const void* wtT,
                                      const float* dtl, const float* q, int ldq, const float* dx,
                                      const unsigned char* arg, float* dwt, float* dw1, float* db1, void* ws,
                                      size_t ws_bytes, int N, int U, const int* counts, int compat, hipStream_t st,
                                      const void* demb_in, int f32) {
  if (ws_bytes < dca_encoder_bwd_workspace(N, U, counts, f32)) return hipErrorInvalidValue;
  int acc = 0;
  for (int t = 0; t < 6; ++t) acc += counts[t];
  if (acc != U || U > 64) return hipErrorInvalidValue;
  if (f32) {
    FbParams F{units, w1, b1, static_cast<const float*>(wtT), dtl, q, ldq, dx, arg,
               static_cast<const float*>(demb_in), nullptr, nullptr, N, compat, 0, {}, {}};
    fb_plan(N, counts, F);
    F.L.U = U;
    for (int t = 0, o = 0; t < 6; ++t) { F.L.cnt[t] = counts[t]; F.L.off[t] = o; o += counts[t]; }
    const int jobs = F.jbase[6];
    F.w1part = static_cast<float*>(ws);
    F.dwtpart = F.w1part + (size_t)jobs * kW1;
    if (jobs > 0 && f32 == 2) {
      // the 4-wave two-workgroups-per-CU form: 369.7 vs 373.6 µs alone for the 8-wave form, and in the exact learner
      // step 5.498 / 5.483 vs 5.518 / 5.513 ms (two same-box pairs) — beside the side stream's weight-gradient GEMMs
      // two smaller workgroups per CU schedule better
      if (demb_in) encoder_bwd_x2_kernel<true, false><<<jobs, 256, 0, st>>>(F);
      else if (compat) encoder_bwd_x2_kernel<false, true><<<jobs, 256, 0, st>>>(F);
      else encoder_bwd_x2_kernel<false, false><<<jobs, 256, 0, st>>>(F);
    } else if (jobs > 0) {
      if (demb_in) encoder_bwd_f32_fused_kernel<true, false><<<jobs, 512, 0, st>>>(F);
      else if (compat) encoder_bwd_f32_fused_kernel<false, true><<<jobs, 512, 0, st>>>(F);
      else encoder_bwd_f32_fused_kernel<false, false><<<jobs, 512, 0, st>>>(F);
    }
    encoder_w1_reduce<<<(kW1 + 15) / 16, 256, 0, st>>>(F.w1part, jobs, dw1, db1);
    fb_dwt_reduce<<<dim3(kD * kD / 64, 6), 256, 0, st>>>(F.dwtpart, F, dwt);
    return hipGetLastError();
  }
  DwtJobs J;
  int NB;
  dwt_plan(N, counts, J, NB);
  const int nblk = (N + kRows - 1) / kRows;
  char* p = static_cast<char*>(ws);
  float* w1part = reinterpret_cast<float*>(p);
  p += (size_t)nblk * kJobs * kW1 * sizeof(float);
  const size_t img = (size_t)U * NB * kD * 16;
  short* demb = reinterpret_cast<short*>(p);
  short* basic = demb + img;
  float* parts = reinterpret_cast<float*>(basic + img);
  BwdParams P{units, w1, b1, wtT, dtl, q, ldq, dx, arg, demb, basic, w1part, N, compat, {}, {}, NB, demb_in};
  P.L.U = U;
  acc = 0;
  for (int t = 0; t < 6; ++t) {
    P.L.cnt[t] = counts[t];
    P.L.off[t] = acc;
    P.blkbase[t] = J.blkbase[t];
    acc += counts[t];
  }
  encoder_bwd_kernel<<<dim3(nblk, kJobs), 256, 0, st>>>(P);
  encoder_w1_reduce<<<(kW1 + 15) / 16, 256, 0, st>>>(w1part, nblk * kJobs, dw1, db1);
  if (J.jbase[6] > 0) dwt_blocked_kernel<<<J.jbase[6], 256, 0, st>>>(demb, basic, J, parts);
  dwt_reduce<<<dim3(kD * kD / 64, 6), 256, 0, st>>>(parts, J, dwt);
  return hipGetLastError();
}
