// Small fused "glue" kernels of the learner step (gfx950). Each replaces a chain of 10-40 tiny PyTorch launches
// whose cost is launch/dependency latency, not bytes:
//
//   loss_prep_kernel     experience-only loss normalisers from the one-hot action rows (was ≈35 torch ops:
//                        column sums, amax, four clamp/reciprocal/where chains, cat). Multi-block partial counts,
//                        the last block to arrive (agent-scope counter, self-resetting → hipGraph-replayable)
//                        folds them into norms[8] = [1/n_valid, 1/total_sel, 1/n_sel[enum,x,y,target], 0, 0].
//   loss_assemble_kernel loss scalar + metrics from the heads/loss kernel's per-block partials (was a torch sum +
//                        ≈20 scalar ops) — reference optimizer.py:640-672 formulas, see ops/heads.py:assemble_loss.
//   enc_small_grads      ∂b_τ (6×128), ∂W_env (128×3), ∂b_env (128) of the entity encoder in one pass over the rows
//                        (was ≈15 launches: dtl·seg GEMM, a split-K bmm, column sums, the env ReLU mask and a
//                        128×3 fp32 GEMM that hipBLASLt ran at 55 µs), deterministic per-block partials +
//                        enc_small_reduce.
//   replay_gather_kernel the learner minibatch straight from the HBM replay pool in TIME-MAJOR row order, every
//                        field in one launch (was a row-index computation + one index_select per field).
//   weight_prep_kernel   every per-step working copy of the weights in one gather pass over the flat fp32 buffer:
//                        bf16 images (stacked / permuted / transposed / zero-padded, via an int32 source map) and
//                        fp32 images (optionally the sum of two sources: b_ih + b_hh), and bf16 hi / lo split images
//                        (x = hi + lo) for the bf16x3 operands of the fp32 learner's chain kernels.
#include "common.h"

namespace {

constexpr int kPrepThreads = 256;
constexpr int kPrepBlocks = 256;

// One wave per row: lane j reads byte j of the row (coalesced), ballots give the per-head selection counts
// (one-hot 0/1 entries) and the row's validity (any entry set). Per-block partial counts
// [n_valid, sel_enum, sel_x, sel_y, sel_target]; the last block to arrive folds them.
__global__ __launch_bounds__(kPrepThreads) void loss_prep_kernel(const unsigned char* __restrict__ act, int N, int A,
                                                                 int* __restrict__ partial,
                                                                 unsigned* __restrict__ counter,
                                                                 float* __restrict__ norms) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nw = gridDim.x * (kPrepThreads / dca::kWave);
  // lane → head masks over the first 64 columns (enum 0-2, x 3-11, y 12-20, target 21..)
  const unsigned long long m_enum = 0x7ull, m_x = 0x1ffull << 3, m_y = 0x1ffull << 12;
  const unsigned long long m_t = ~(m_enum | m_x | m_y);
  int c[5] = {0, 0, 0, 0, 0};
  for (int r = blockIdx.x * (kPrepThreads / dca::kWave) + w; r < N; r += nw) {
    const unsigned char* row = act + (size_t)r * A;
    const bool v0 = lane < A && row[lane] != 0;
    const bool v1 = lane + 64 < A && row[lane + 64] != 0;          // target columns beyond 64 (A ≤ 128)
    const unsigned long long b0 = __ballot(v0), b1 = __ballot(v1);
    c[0] += (b0 | b1) != 0ull;
    c[1] += __popcll(b0 & m_enum);
    c[2] += __popcll(b0 & m_x);
    c[3] += __popcll(b0 & m_y);
    c[4] += __popcll(b0 & m_t) + __popcll(b1);
  }
  __shared__ int red[kPrepThreads / dca::kWave][5];
  __shared__ bool last;
  if (lane == 0)
    for (int i = 0; i < 5; ++i) red[w][i] = c[i];
  __syncthreads();
  if (threadIdx.x < 5) {
    int v = 0;
#pragma unroll
    for (int k = 0; k < kPrepThreads / dca::kWave; ++k) v += red[k][threadIdx.x];
    partial[blockIdx.x * 5 + threadIdx.x] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();                                             // release this block's partials
    const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == gridDim.x - 1);
  }
  __syncthreads();
  if (!last) return;
  __threadfence();                                               // acquire every block's partials
  // parallel fold: thread b loads block b's five counts (all loads in flight at once), then a fixed LDS tree
  __shared__ int fold[kPrepBlocks][5];
  for (int b = threadIdx.x; b < kPrepBlocks; b += kPrepThreads)
    for (int i = 0; i < 5; ++i)
      fold[b][i] = b < (int)gridDim.x
                       ? __hip_atomic_load(partial + b * 5 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  __syncthreads();
  for (int o = kPrepBlocks / 2; o > 0; o >>= 1) {
    for (int b = threadIdx.x; b < o; b += kPrepThreads)
      for (int i = 0; i < 5; ++i) fold[b][i] += fold[b + o][i];
    __syncthreads();
  }
  if (threadIdx.x < 5) red[0][threadIdx.x] = fold[0][threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    auto inv = [](long long x) { return x > 0 ? 1.f / (float)x : 0.f; };
    const long long n_valid = red[0][0];
    long long tot = 0;
    for (int h = 0; h < 4; ++h) tot += red[0][1 + h];
    norms[0] = inv(n_valid);
    norms[1] = inv(tot);
    for (int h = 0; h < 4; ++h) norms[2 + h] = inv(red[0][1 + h]);
    norms[6] = 0.f;
    norms[7] = 0.f;
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // ready for the next launch
  }
}

constexpr int kAsmThreads = 1024;

// out[0..11] = [loss, policy_loss, entropy_loss, advantage_loss, entropy, advantage, approx_kl, clipfrac,
//               entropy/enum, entropy/x, entropy/y, entropy/target_unit]; out[12..15] = 0
// Column sums of part (R,16): thread t sums column t&15 over rows t>>4, +64, … (8 loads in flight), then a fixed
// LDS tree over the 64 row groups (deterministic).
__global__ __launch_bounds__(kAsmThreads) void loss_assemble_kernel(const float* __restrict__ part, int nrows,
                                                                    const float* __restrict__ norms, int N, int algo,
                                                                    float ent_coef, float vf_coef,
                                                                    float* __restrict__ out, int S, int vbug) {
  const int t = threadIdx.x, col = t & 15, rg = t >> 4;
  float s = 0.f;
  int r = rg;
  for (; r + 7 * 64 < nrows; r += 8 * 64) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = part[(size_t)(r + k * 64) * 16 + col];
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
  }
  for (; r < nrows; r += 64) s += part[(size_t)r * 16 + col];
  __shared__ float red[64][17];
  red[rg][col] = s;
  __syncthreads();
  for (int o = 32; o > 0; o >>= 1) {
    if (rg < o) red[rg][col] += red[rg + o][col];
    __syncthreads();
  }
  if (t != 0) return;
  float p[16];
  for (int i = 0; i < 16; ++i) p[i] = red[0][i];
  float eh[4], ent = 0.f;
  for (int h = 0; h < 4; ++h) {
    eh[h] = p[2 + h] * norms[2 + h];
    ent += eh[h];
  }
  float pol, val, entl, adv, kl = 0.f, cf = 0.f;
  const float invN = 1.f / (float)(N > 0 ? N : 1);
  if (algo != 1) {   // PPO clipped surrogate (0) or truncated-IS off-policy PG (2)
    pol = -p[0] * norms[0];
    val = vf_coef * p[1] * norms[0];
    entl = -ent_coef * ent;
    adv = p[8] * norms[0];
    kl = p[6] * norms[0];
    cf = p[7] * norms[0];
  } else {
    pol = p[0] * norms[1];
    entl = ent_coef > 0.f ? -ent_coef * ent : 0.f;
    val = vf_coef > 0.f ? vf_coef * p[1] * invN : 0.f;
    adv = p[8] * invN;
    if (vbug && vf_coef > 0.f && S > 0) {
      // the reference's value bug (optimizer.py:603): mean over (B, S, S) of (V[b,s] − G_last[s'])², from ΣV (p[9]),
      // ΣV² (p[10]) and ΣG_last / ΣG_last² (norms[6], norms[7]) — ops/heads.py assemble_loss
      const float Sf = (float)S, Bf = (float)(N / S);
      val = vf_coef * (Sf * p[10] - 2.f * p[9] * norms[6] + (float)N * norms[7]) / (Bf * Sf * Sf);
      adv = p[9] * invN - norms[6] / Sf;
    }
  }
  out[0] = pol + val + entl;
  out[1] = pol;
  out[2] = entl;
  out[3] = val;
  out[4] = ent;
  out[5] = adv;
  out[6] = kl;
  out[7] = cf;
  for (int h = 0; h < 4; ++h) out[8 + h] = eh[h];
  for (int i = 12; i < 16; ++i) out[i] = 0.f;
}

__global__ __launch_bounds__(256) void weight_prep_kernel(const float* __restrict__ src, const int* __restrict__ map16,
                                                          short* __restrict__ dst16, int n16,
                                                          const int2* __restrict__ map32, float* __restrict__ dst32,
                                                          int n32, const int* __restrict__ maps,
                                                          short* __restrict__ dsth, short* __restrict__ dstl, int ns) {
  const int stride = gridDim.x * blockDim.x;
  // bf16x3 operand images: x = hi + lo (the slab-major weight images of the fp32 learner's hand-written chains)
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += stride) {
    const int m = maps[i];
    const float v = m >= 0 ? src[m] : 0.f;          // (-1: zero padding rows)
    const short h = dca::f2bf(v);
    dsth[i] = h;
    dstl[i] = dca::f2bf(v - dca::bf2f(h));
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const int m = map16[i];
    dst16[i] = dca::f2bf(m >= 0 ? src[m] : 0.f);
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n32; i += stride) {
    const int2 m = map32[i];
    dst32[i] = (m.x >= 0 ? src[m.x] : 0.f) + (m.y >= 0 ? src[m.y] : 0.f);
  }
}

constexpr int kSgBlocks = 256;
constexpr int kSgPhases = 4;                  // row phases per block (128 columns each)
constexpr int kSgRows = 32;                       // rows per LDS tile
constexpr int kSgOut = 6 * 128 + 128 * 3 + 128;   // [dbt | dWe | dbe] per partial

// Thread (row phase ph = tid >> 7, column d = tid & 127). Per row n:
//   ∂b_τ[d] += q[n,d]·Σ_{u∈τ} dtl[n,u] + dx[n, 128 + 128τ' + d]   (τ' = pool column routed to τ; compat: 5 → 3)
//   de = dx[n,d]·[env[n]·W_env[d] + b_env[d] > 0];  ∂W_env[d,c] += de·env[n,c];  ∂b_env[d] += de
__global__ __launch_bounds__(128 * kSgPhases) void enc_small_grads_kernel(const float* __restrict__ z, int ldz,
                                                              const float* __restrict__ dtl, int U,
                                                              const int* __restrict__ type_off,
                                                              const float* __restrict__ dx, const float* __restrict__ env,
                                                              const float* __restrict__ we, const float* __restrict__ be,
                                                              int N, int compat, float* __restrict__ part) {
  const int d = threadIdx.x & 127, ph = threadIdx.x >> 7;
  __shared__ float s_seg[kSgRows][6];
  __shared__ float s_env[kSgRows][3];
  __shared__ float red[kSgPhases - 1][kSgOut];
  float adbt[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, adwe[3] = {0.f, 0.f, 0.f}, adbe = 0.f;
  const float w0 = we[d * 3 + 0], w1 = we[d * 3 + 1], w2 = we[d * 3 + 2], bd = be[d];
  const int rows_per = (N + gridDim.x - 1) / gridDim.x;
  const int r_lo = blockIdx.x * rows_per, r_hi = min(N, r_lo + rows_per);
  for (int t0 = r_lo; t0 < r_hi; t0 += kSgRows) {
    const int nt = min(kSgRows, r_hi - t0);
    __syncthreads();
    for (int i = threadIdx.x; i < nt * 6; i += 128 * kSgPhases) {   // per-(row, type) pointer-gradient sums
      const int r = i / 6, ty = i % 6;
      const float* dr = dtl + (size_t)(t0 + r) * U;
      float sacc = 0.f;
      for (int u = type_off[ty]; u < type_off[ty + 1]; ++u) sacc += dr[u];
      s_seg[r][ty] = sacc;
    }
    for (int i = threadIdx.x; i < nt * 3; i += 128 * kSgPhases)
      s_env[i / 3][i % 3] = env[(size_t)(t0 + i / 3) * 3 + i % 3];
    __syncthreads();
    for (int r = ph; r < nt; r += kSgPhases) {
      const size_t n = t0 + r;
      const float q = z[n * ldz + d];
      const float* dxr = dx + n * 896;
      float pool[6];
#pragma unroll
      for (int ty = 0; ty < 6; ++ty) pool[ty] = dxr[128 + 128 * ty + d];
      if (compat) {
        pool[3] += pool[5];
        pool[5] = 0.f;
      }
#pragma unroll
      for (int ty = 0; ty < 6; ++ty) adbt[ty] += q * s_seg[r][ty] + pool[ty];
      const float e0 = s_env[r][0], e1 = s_env[r][1], e2 = s_env[r][2];
      const float pre = e0 * w0 + e1 * w1 + e2 * w2 + bd;
      const float de = pre > 0.f ? dxr[d] : 0.f;
      adwe[0] += de * e0;
      adwe[1] += de * e1;
      adwe[2] += de * e2;
      adbe += de;
    }
  }
  // combine the row phases in a fixed order, one partial per block
  __syncthreads();
  if (ph > 0) {
    float* rr = red[ph - 1];
    for (int ty = 0; ty < 6; ++ty) rr[ty * 128 + d] = adbt[ty];
    for (int c = 0; c < 3; ++c) rr[768 + d * 3 + c] = adwe[c];
    rr[1152 + d] = adbe;
  }
  __syncthreads();
  if (ph == 0) {
    float* o = part + (size_t)blockIdx.x * kSgOut;
    for (int ty = 0; ty < 6; ++ty) {
      float v = adbt[ty];
      for (int k = 0; k < kSgPhases - 1; ++k) v += red[k][ty * 128 + d];
      o[ty * 128 + d] = v;
    }
    for (int c = 0; c < 3; ++c) {
      float v = adwe[c];
      for (int k = 0; k < kSgPhases - 1; ++k) v += red[k][768 + d * 3 + c];
      o[768 + d * 3 + c] = v;
    }
    float v = adbe;
    for (int k = 0; k < kSgPhases - 1; ++k) v += red[k][1152 + d];
    o[1152 + d] = v;
  }
}

// out[c] = Σ_b part[b][c] in block order (deterministic): 64 columns × 4 row phases per block.
__global__ __launch_bounds__(256) void enc_small_reduce(const float* __restrict__ part, int nblk,
                                                        float* __restrict__ out) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), ph = threadIdx.x >> 6;
  float s = 0.f;
  if (c < kSgOut) {
    int b = ph;
    for (; b + 12 < nblk; b += 16) {
      const float v0 = part[(size_t)b * kSgOut + c], v1 = part[(size_t)(b + 4) * kSgOut + c];
      const float v2 = part[(size_t)(b + 8) * kSgOut + c], v3 = part[(size_t)(b + 12) * kSgOut + c];
      s += v0;
      s += v1;
      s += v2;
      s += v3;
    }
    for (; b < nblk; b += 4) s += part[(size_t)b * kSgOut + c];
  }
  __shared__ float red[4][64];
  red[ph][threadIdx.x & 63] = s;
  __syncthreads();
  if (ph == 0 && c < kSgOut) out[c] = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) +
                                       red[3][threadIdx.x];
}

constexpr int kMaxGather = 12;
struct GatherField {
  const char* src;      // pool base: (capacity, S, …) per-step field or (capacity, …) per-sequence field
  char* dst;            // (S·B, …) time-major rows, or (B, …)
  long long row_bytes;  // bytes per time step (per-step) or per sequence
  int per_step;
  int unit;             // copy granule: 16, 4 or 1 bytes (divides row_bytes and the alignment)
};
struct GatherArgs {
  GatherField f[kMaxGather];
  const long long* idx;
  int S, B;
};

template <typename T>
__device__ __forceinline__ void gather_rows(const GatherField& F, const long long* __restrict__ idx, int S, int B) {
  const long long wpr = F.row_bytes / (long long)sizeof(T);
  const long long rows = F.per_step ? (long long)S * B : B;
  const long long total = rows * wpr;
  const T* src = reinterpret_cast<const T*>(F.src);
  T* dst = reinterpret_cast<T*>(F.dst);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / wpr, w = i - r * wpr;
    long long srow;
    if (F.per_step) {
      const long long t = r / B, b = r - t * B;
      srow = idx[b] * S + t;
    } else {
      srow = idx[r];
    }
    dst[r * wpr + w] = src[srow * wpr + w];
  }
}

__global__ __launch_bounds__(256) void replay_gather_kernel(GatherArgs a) {
  const GatherField& F = a.f[blockIdx.y];
  if (F.unit == 16) gather_rows<uint4>(F, a.idx, a.S, a.B);
  else if (F.unit == 4) gather_rows<unsigned>(F, a.idx, a.S, a.B);
  else gather_rows<unsigned char>(F, a.idx, a.S, a.B);
}

}  // namespace

extern "C" hipError_t dca_replay_gather(const void* const* src, void* const* dst, const long long* row_bytes,
                                        const int* per_step, int nf, const long long* idx, int S, int B,
                                        hipStream_t st) {
  if (nf < 1 || nf > kMaxGather) return hipErrorInvalidValue;
  GatherArgs a{};
  for (int i = 0; i < nf; ++i) {
    const unsigned long long align = (unsigned long long)src[i] | (unsigned long long)dst[i];
    int unit = 1;
    if (row_bytes[i] % 16 == 0 && align % 16 == 0) unit = 16;
    else if (row_bytes[i] % 4 == 0 && align % 4 == 0) unit = 4;
    a.f[i] = GatherField{static_cast<const char*>(src[i]), static_cast<char*>(dst[i]), row_bytes[i], per_step[i], unit};
  }
  a.idx = idx;
  a.S = S;
  a.B = B;
  hipLaunchKernelGGL(replay_gather_kernel, dim3(256, nf), dim3(256), 0, st, a);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}

extern "C" int dca_enc_small_out() { return kSgOut; }
extern "C" int dca_enc_small_blocks() { return kSgBlocks; }

extern "C" hipError_t dca_enc_small_grads(const float* z, int ldz, const float* dtl, int U, const int* type_off,
                                          const float* dx, const float* env, const float* we, const float* be, int N,
                                          int compat, float* part, float* out, hipStream_t st) {
  hipLaunchKernelGGL(enc_small_grads_kernel, dim3(kSgBlocks), dim3(128 * kSgPhases), 0, st, z, ldz, dtl, U, type_off, dx, env, we,
                     be, N, compat, part);
  DCA_CHECK_LAUNCH();
  hipLaunchKernelGGL(enc_small_reduce, dim3((kSgOut + 63) / 64), dim3(256), 0, st, part, kSgBlocks, out);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}

extern "C" int dca_loss_prep_blocks() { return kPrepBlocks; }

extern "C" hipError_t dca_loss_prep(const unsigned char* act, int N, int A, int* partial, unsigned* counter,
                                    float* norms, hipStream_t st) {
  hipLaunchKernelGGL(loss_prep_kernel, dim3(kPrepBlocks), dim3(kPrepThreads), 0, st, act, N, A, partial, counter,
                     norms);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}

extern "C" hipError_t dca_loss_assemble(const float* part, int nrows, const float* norms, int N, int algo,
                                        float ent_coef, float vf_coef, float* out, int S, int vbug, hipStream_t st) {
  hipLaunchKernelGGL(loss_assemble_kernel, dim3(1), dim3(kAsmThreads), 0, st, part, nrows, norms, N, algo, ent_coef, vf_coef,
                     out, S, vbug);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}

extern "C" hipError_t dca_weight_prep(const float* src, const int* map16, short* dst16, int n16, const int* map32,
                                      float* dst32, int n32, const int* maps, short* dsth, short* dstl, int ns,
                                      hipStream_t st) {
  int n = n16 > n32 ? n16 : n32;
  if (ns > n) n = ns;
  int blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(weight_prep_kernel, dim3(blocks), dim3(256), 0, st, src, map16, dst16, n16,
                     reinterpret_cast<const int2*>(map32), dst32, n32, maps, dsth, dstl, ns);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}

// ---- test utility: occupy CUs of ONE XCD -------------------------------------------------------------------------
// Workgroups that land on XCD `xcd` (HW_REG_XCC_ID) hold their CU for `ticks` of the 100 MHz s_memrealtime clock
// with a 160 KB LDS allocation (no other LDS-using workgroup can share the CU); every other workgroup exits at once.
// Every wave ends when its own deadline passes (no flag to wait for), and writes one vector store of where it ran
// (`seen[blockIdx.x]` = XCC id + 1 on the target XCD, 0 elsewhere). Used by tests/test_team_residency.py to check
// that the XCD-team recurrence forms its teams on the remaining XCDs when part of one XCD is already occupied.
namespace {
constexpr int kOccupyLds = 160 * 1024;
__global__ __launch_bounds__(64) void occupy_xcd_kernel(int xcd, unsigned long long ticks, int* seen) {
  extern __shared__ __attribute__((aligned(16))) float occ_lds[];
  const unsigned x = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xf;
  if ((int)x != xcd) {
    if (threadIdx.x == 0) seen[blockIdx.x] = 0;
    return;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  occ_lds[threadIdx.x] = 0.f;                                  // touch the allocation
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
  if (threadIdx.x == 0) seen[blockIdx.x] = (int)x + 1 + (int)occ_lds[threadIdx.x];
}
}  // namespace

extern "C" hipError_t dca_occupy_xcd(int xcd, int blocks, double seconds, int* seen, hipStream_t st) {
  if (blocks < 1 || blocks > 4096 || seconds <= 0.0 || seconds > 10.0) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(occupy_xcd_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kOccupyLds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const unsigned long long ticks = (unsigned long long)(seconds * 1e8);
  hipLaunchKernelGGL(occupy_xcd_kernel, dim3(blocks), dim3(64), kOccupyLds, st, xcd, ticks, seen);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}
