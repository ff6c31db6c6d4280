// Fused global-norm gradient clip + Adam over one flat fp32 parameter buffer (gfx950).
//
// Replaces clip_grad_norm_(0.5) + torch.optim.Adam (reference optimizer.py:281, 680-681) with two launches over the
// flat buffers of dotaclient_amd.parallel.dp.FlatParams:
//   1. adam_norm_kernel   : per-block partial sums of g^2 (float4 loads, grid-stride), written to partials[blk];
//                           block 0 also snapshots the per-parameter step counters into partials[kMaxBlocks + p].
//   2. adam_update_kernel : every block re-reduces the (<=1024) partials itself — no third launch, no cross-block
//                           hand-off — then applies clip + Adam to its float4 groups with t = snapshot + 1. Parameters
//                           with DP has-grad count 0 are skipped (sparse-param semantics, reference
//                           distributed.py:40-42). Block 0 advances the step counters (from the snapshot, so no block
//                           reads a counter another block is writing) only when the step is APPLIED: a skipped or
//                           non-finite step leaves Adam's bias correction where it was.
// Memory-bound: ~28 B/element moved. Offsets are 64-element aligned so a float4 group never straddles parameters.
// The first h4 float4 groups are the flat buffer's header (has-grad counts + the kernel-error flag, see
// parallel/dp.py), never part of the gradient norm. `skip` (optional, device): when *skip != 0 — a persistent
// recurrence kernel failed on some rank this step — neither the step counters nor any parameter / moment changes
// (the reference raises before optimizer.step(), optimizer.py:674-676; here the decision stays on the device).
// `nonfinite` (optional, device, sticky): set to 1 when a step is dropped because its gradient norm is not finite, so
// the learner raises at the iteration boundary like the reference's NaN check instead of training on silently.
#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxBlocks = 1024;

// divide: the gradient buffer holds DP SUMS; the has-grad average g / count[param] is taken here (count 0 → 0)
// instead of by a separate pass over the buffer after the all-reduce.
__device__ __forceinline__ float grad_scale(const int* seg, const float* counts, int i, int divide) {
  if (!divide) return 1.f;
  const int s = seg[i * 4];
  return (s >= 0 && counts[s] > 0.f) ? 1.f / counts[s] : 0.f;
}

__global__ __launch_bounds__(kThreads) void adam_norm_kernel(const float4* __restrict__ g, int n4,
                                                             float* __restrict__ partials,
                                                             const float* __restrict__ counts,
                                                             float* __restrict__ steps, int n_params,
                                                             const int* __restrict__ seg, int divide, int h4) {
  float acc = 0.f;
  for (int i = h4 + blockIdx.x * kThreads + threadIdx.x; i < n4; i += gridDim.x * kThreads) {
    float4 v = g[i];
    const float sc = grad_scale(seg, counts, i, divide);
    acc += sc * sc * (v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w);
  }
  __shared__ float red[kThreads / dca::kWave];
  acc = dca::wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kThreads / dca::kWave; ++w) s += red[w];
    partials[blockIdx.x] = s;
  }
  if (blockIdx.x == 0)
    for (int p = threadIdx.x; p < n_params; p += kThreads) partials[kMaxBlocks + p] = steps[p];
}

__global__ __launch_bounds__(kThreads) void adam_update_kernel(
    float4* __restrict__ param, const float4* __restrict__ grad, float4* __restrict__ m, float4* __restrict__ v,
    const int* __restrict__ seg, int n4, const float* __restrict__ partials, int nparts,
    const float* __restrict__ counts, float* __restrict__ steps, int n_params, float* __restrict__ norm_out,
    float lr, float b1, float b2, float eps, float max_norm, int divide, const float* __restrict__ skip,
    float* __restrict__ nonfinite) {
  __shared__ float red[kThreads / dca::kWave];
  __shared__ float s_coef;
  __shared__ bool s_bad;
  float acc = 0.f;
  for (int i = threadIdx.x; i < nparts; i += kThreads) acc += partials[i];
  acc = dca::wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kThreads / dca::kWave; ++w) s += red[w];
    const float norm = sqrtf(s);
    float coef = 1.f;
    if (max_norm > 0.f) coef = fminf(1.f, max_norm / (norm + 1e-6f));
    s_coef = coef;
    // a non-finite gradient (NaN / Inf loss) never reaches the weights: the reference raises before
    // optimizer.step() (optimizer.py:674-676); the learner raises when it reads the loss, which with deferred
    // metrics is an iteration later — the weights published meanwhile stay the last finite ones
    s_bad = !__builtin_isfinite(norm);
    if (blockIdx.x == 0) *norm_out = norm;
  }
  __syncthreads();
  if (skip && *skip != 0.f) return;          // failed step: the norm is reported, nothing is applied
  if (s_bad) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && nonfinite) *nonfinite = 1.f;
    return;
  }
  const float* snap = partials + kMaxBlocks;
  if (blockIdx.x == 0)
    for (int p = threadIdx.x; p < n_params; p += kThreads)
      if (counts[p] > 0.f) steps[p] = snap[p] + 1.f;
  const float coef = s_coef;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < n4; i += gridDim.x * kThreads) {
    const int s = seg[i * 4];
    if (s < 0) continue;
    if (!(counts[s] > 0.f)) continue;
    const float t = snap[s] + 1.f;
    const float gcoef = divide ? coef / counts[s] : coef;
    const float bc1 = 1.f - powf(b1, t);
    const float bc2s = sqrtf(1.f - powf(b2, t));
    const float step_size = lr / bc1;
    float4 gg = grad[i], mm = m[i], vv = v[i], pp = param[i];
#define DCA_ADAM_LANE(c)                                          \
    {                                                             \
      const float gc = gg.c * gcoef;                              \
      mm.c = b1 * mm.c + (1.f - b1) * gc;                         \
      vv.c = b2 * vv.c + (1.f - b2) * gc * gc;                    \
      pp.c -= step_size * mm.c / (sqrtf(vv.c) / bc2s + eps);      \
    }
    DCA_ADAM_LANE(x) DCA_ADAM_LANE(y) DCA_ADAM_LANE(z) DCA_ADAM_LANE(w)
#undef DCA_ADAM_LANE
    m[i] = mm;
    v[i] = vv;
    param[i] = pp;
  }
}

}  // namespace

// n must be a multiple of 4 (FlatParams pads every parameter to 64 elements). `partials` holds
// >= kMaxBlocks + n_params floats (dca_adam_partials_len).
extern "C" int dca_adam_partials_len(int n_params) { return kMaxBlocks + n_params; }

extern "C" hipError_t dca_adam_step(float* param, const float* grad, float* m, float* v, const int* seg, int64_t n,
                                    const float* counts, float* steps, int n_params, float* partials,
                                    float* norm_out, float lr, float b1, float b2, float eps, float max_norm,
                                    hipStream_t stream, int divide, int64_t header, const float* skip,
                                    float* nonfinite) {
  if (header < 0 || header % 4 != 0 || header > n) return hipErrorInvalidValue;
  const int n4 = (int)(n / 4);
  int blocks = (n4 + kThreads - 1) / kThreads;
  blocks = blocks < 1 ? 1 : (blocks > kMaxBlocks ? kMaxBlocks : blocks);
  adam_norm_kernel<<<blocks, kThreads, 0, stream>>>(reinterpret_cast<const float4*>(grad), n4, partials, counts,
                                                    steps, n_params, seg, divide, (int)(header / 4));
  DCA_CHECK_LAUNCH();
  adam_update_kernel<<<blocks, kThreads, 0, stream>>>(
      reinterpret_cast<float4*>(param), reinterpret_cast<const float4*>(grad), reinterpret_cast<float4*>(m),
      reinterpret_cast<float4*>(v), seg, n4, partials, blocks, counts, steps, n_params, norm_out, lr, b1, b2, eps,
      max_norm, divide, skip, nonfinite);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}

// ------------------------------------------------------------------------------------------------------------
// Multi-tensor "dst_i += s · src_i" for up to kMaxAxpy tensors in ONE launch. The tensor table travels by value in
// the kernel arguments (no host-side metadata buffer), so the launch is safe to capture in a hipGraph and replay
// (the fused learner step adds its 30 precomputed parameter gradients into the flat gradient buffer with it).
namespace {
constexpr int kMaxAxpy = 64;
struct AxpyTable {
  float* dst[kMaxAxpy];
  const float* src[kMaxAxpy];
  long long start[kMaxAxpy + 1];   // prefix sum of element counts
  int n;
};

__global__ __launch_bounds__(256) void multi_axpy_kernel(AxpyTable tab, const float* __restrict__ scale) {
  const float s = scale ? *scale : 1.f;
  const long long total = tab.start[tab.n];
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    int lo = 0, hi = tab.n - 1;                    // tensor containing element e (binary search, ≤ 6 steps)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tab.start[mid] <= e) lo = mid; else hi = mid - 1;
    }
    const long long k = e - tab.start[lo];
    tab.dst[lo][k] += s * tab.src[lo][k];
  }
}
}  // namespace

extern "C" hipError_t dca_multi_axpy(float* const* dst, const float* const* src, const long long* numel, int n,
                                     const float* scale, hipStream_t st) {
  if (n < 0 || n > kMaxAxpy) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  AxpyTable tab;
  tab.n = n;
  tab.start[0] = 0;
  for (int i = 0; i < n; ++i) {
    tab.dst[i] = dst[i];
    tab.src[i] = src[i];
    tab.start[i + 1] = tab.start[i] + numel[i];
  }
  const long long total = tab.start[n];
  int blocks = (int)((total + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  multi_axpy_kernel<<<blocks, 256, 0, st>>>(tab, scale);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------------------
// Multi-tensor copy: up to kMaxCopy (dst, src, bytes) segments in ONE launch (16-byte chunks, byte tail), table by
// value in the kernel arguments. The learner's per-iteration pool fill was a dozen separate copy launches.
namespace {
constexpr int kMaxCopy = 64;
struct CopyTable {
  unsigned char* dst[kMaxCopy];
  const unsigned char* src[kMaxCopy];
  long long bytes[kMaxCopy];
  long long start[kMaxCopy + 1];   // prefix sum of 16-byte chunk counts
  int n;
};

__global__ __launch_bounds__(256) void multi_copy_kernel(CopyTable tab) {
  const long long total = tab.start[tab.n];
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    int lo = 0, hi = tab.n - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tab.start[mid] <= e) lo = mid; else hi = mid - 1;
    }
    const long long off = (e - tab.start[lo]) * 16;
    const long long nb = tab.bytes[lo];
    if (off + 16 <= nb) {
      *reinterpret_cast<uint4*>(tab.dst[lo] + off) = *reinterpret_cast<const uint4*>(tab.src[lo] + off);
    } else {
      for (long long b = off; b < nb; ++b) tab.dst[lo][b] = tab.src[lo][b];
    }
  }
}
}  // namespace

extern "C" hipError_t dca_multi_copy(void* const* dst, const void* const* src, const long long* bytes, int n,
                                     hipStream_t st) {
  if (n < 0 || n > kMaxCopy) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  CopyTable tab;
  tab.n = n;
  tab.start[0] = 0;
  for (int i = 0; i < n; ++i) {
    // 16-byte chunks need 16-byte aligned segments (torch allocations and their leading slices are)
    if ((reinterpret_cast<unsigned long long>(dst[i]) | reinterpret_cast<unsigned long long>(src[i])) & 15ull)
      return hipErrorInvalidValue;
    tab.dst[i] = static_cast<unsigned char*>(dst[i]);
    tab.src[i] = static_cast<const unsigned char*>(src[i]);
    tab.bytes[i] = bytes[i];
    tab.start[i + 1] = tab.start[i] + (bytes[i] + 15) / 16;
  }
  const long long total = tab.start[n];
  long long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  multi_copy_kernel<<<(int)blocks, 256, 0, st>>>(tab);
  return hipGetLastError();
}

