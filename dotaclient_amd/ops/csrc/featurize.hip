// GPU-side unit featurization (gfx950): the per-unit features of the reference featurizer (agent.py:496-562,
// features/featurizer.py unit_matrix) computed on the device from a compact raw record, so the host (the native
// engine's observe, native/core.h featurize_one_raw) no longer evaluates the distance / sincos / range test of every
// unit of every player-step, and the policy step's staged observation crosses PCIe as 32 B per unit instead of 48 B
// (40 B of fp32 features + an 8 B handle).
//
// Raw unit record (8 × 32-bit words, two 16-B loads per unit):
//   w0 x, w1 y, w2 z, w3 facing (degrees) — fp32 as observed (CMsgBotWorldState.Unit)
//   w4 1 − health / health_max — the first feature itself, evaluated in double and rounded once on the host (it also
//      decides the handle's denial rule, so the host needs it anyway)
//   w5 the unit's action handle, −1 = not targetable (the host's validity rules, agent.py:540-552)
//   w6 flags: bit 0 present (a unit fills the slot), bit 1 it attacks the hero, bit 2 the hero attacks it
//      (attack target or an incoming attack projectile, agent.py:250-259: a scan of projectile lists that stays on
//      the host)
//   w7 0
// Hero record per observation (4 × fp32): the observing hero's x, y, attack range, 0.
//
// Every feature is computed in double and rounded once, in the host featurizer's operation order, with FMA
// contraction off — bit-identical to native/core.h unit_rows / featurizer.py for the same record (sqrt is correctly
// rounded in both; the double sincos agrees to an ulp, far below the float rounding). An empty slot gives ten zeros
// and handle −1 (featurizer.py's zero rows).
//
// One thread per (row, unit) slot; outputs fp32 features + int64 handles (bf16 / fp32 actor steps, the learner's
// ingest — which needs no handles) or fp16 features + int32 handles (the fp8 actor step's staged dtypes).
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include "common.h"
#include "launchers.h"

namespace {

template <typename UT>
__device__ __forceinline__ UT to_out(float v);
template <>
__device__ __forceinline__ float to_out<float>(float v) { return v; }
template <>
__device__ __forceinline__ __half to_out<__half>(float v) { return __float2half_rn(v); }

template <typename UT, typename HT>
__global__ __launch_bounds__(256) void featurize_raw_kernel(const int4* __restrict__ raw, const float4* __restrict__ hero,
                                                           UT* __restrict__ units, HT* __restrict__ handles, int rows,
                                                           int U) {
#pragma clang fp contract(off)
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)rows * U) return;
  const long row = i / U;
  const int4 a = raw[2 * i], b = raw[2 * i + 1];
  UT* o = units + i * 10;
  const int flags = b.z;
  if (!(flags & 1)) {
#pragma unroll
    for (int k = 0; k < 10; ++k) o[k] = to_out<UT>(0.f);
    if (handles) handles[i] = (HT)-1;
    return;
  }
  const float4 h = hero[row];
  const double x = (double)__int_as_float(a.x), y = (double)__int_as_float(a.y), z = (double)__int_as_float(a.z);
  const double facing = (double)__int_as_float(a.w);
  const double dx = (double)h.x - x, dy = (double)h.y - y;
  const double dist = sqrt(dx * dx + dy * dy);
  const double tau = 2.0 * 3.14159265358979323846;
  double sf, cf;
  sincos(facing * tau / 360.0, &sf, &cf);
  float f[10];
  f[0] = __int_as_float(b.x);
  f[1] = (float)(x / 7000.0);
  f[2] = (float)(y / 7000.0);
  f[3] = (float)(z / 512.0 - 0.5);
  f[4] = (float)(dist / 7000.0 - 0.5);
  f[5] = (float)sf;
  f[6] = (float)cf;
  f[7] = (dist <= (double)h.z ? 1.f : 0.f) - 0.5f;
  f[8] = ((flags >> 1) & 1 ? 1.f : 0.f) - 0.5f;
  f[9] = ((flags >> 2) & 1 ? 1.f : 0.f) - 0.5f;
#pragma unroll
  for (int k = 0; k < 10; ++k) o[k] = to_out<UT>(f[k]);
  if (handles) handles[i] = (HT)b.y;
}

// fp8 policy step (its features are fp16): the 16-byte record — x | y, z | facing, (1 − hp) | flags as binary16 pairs,
// then the handle — featurized in fp32 arithmetic (hero record fp32) and rounded to fp16 once per feature.
__global__ __launch_bounds__(256) void featurize_raw16_kernel(const int4* __restrict__ raw, const float4* __restrict__ hero,
                                                             __half* __restrict__ units, int32_t* __restrict__ handles,
                                                             int rows, int U) {
#pragma clang fp contract(off)
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)rows * U) return;
  const int4 r = raw[i];
  const int flags = (int)((unsigned)r.z >> 16);
  __half* o = units + i * 10;
  if (!(flags & 1)) {
#pragma unroll
    for (int k = 0; k < 10; ++k) o[k] = __float2half_rn(0.f);
    if (handles) handles[i] = -1;
    return;
  }
  auto lo = [](int w) { return __half2float(__ushort_as_half((unsigned short)((unsigned)w & 0xffffu))); };
  auto hi = [](int w) { return __half2float(__ushort_as_half((unsigned short)((unsigned)w >> 16))); };
  const float4 h = hero[i / U];
  const float x = lo(r.x), y = hi(r.x), z = lo(r.y), facing = hi(r.y);
  const float dx = h.x - x, dy = h.y - y;
  const float dist = sqrtf(dx * dx + dy * dy);
  float sf, cf;
  sincosf(facing * (2.f * 3.14159265358979f) / 360.f, &sf, &cf);
  const float f[10] = {lo(r.z), x / 7000.f, y / 7000.f, z / 512.f - 0.5f, dist / 7000.f - 0.5f, sf, cf,
                       (dist <= h.z ? 1.f : 0.f) - 0.5f, ((flags >> 1) & 1 ? 1.f : 0.f) - 0.5f,
                       ((flags >> 2) & 1 ? 1.f : 0.f) - 0.5f};
#pragma unroll
  for (int k = 0; k < 10; ++k) o[k] = __float2half_rn(f[k]);
  if (handles) handles[i] = r.w;
}

}  // namespace

// half_out: fp16 features + int32 handles; else fp32 features + int64 handles
// 16-byte records (rows, U, 4) → fp16 features + int32 handles (may be null)
extern "C" hipError_t dca_featurize_raw16(const void* raw16, const float* hero, void* units, void* handles, int rows,
                                          int U, hipStream_t st) {
  const long n = (long)rows * U;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(featurize_raw16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     static_cast<const int4*>(raw16), reinterpret_cast<const float4*>(hero),
                     static_cast<__half*>(units), static_cast<int32_t*>(handles), rows, U);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}

extern "C" hipError_t dca_featurize_raw(const void* raw, const float* hero, void* units, void* handles, int rows, int U,
                                        int half_out, hipStream_t st) {
  const long n = (long)rows * U;
  if (n <= 0) return hipSuccess;
  const int blocks = (int)((n + 255) / 256);
  if (half_out) {
    hipLaunchKernelGGL((featurize_raw_kernel<__half, int32_t>), dim3(blocks), dim3(256), 0, st,
                       static_cast<const int4*>(raw), reinterpret_cast<const float4*>(hero),
                       static_cast<__half*>(units), static_cast<int32_t*>(handles), rows, U);
  } else {
    hipLaunchKernelGGL((featurize_raw_kernel<float, int64_t>), dim3(blocks), dim3(256), 0, st,
                       static_cast<const int4*>(raw), reinterpret_cast<const float4*>(hero),
                       static_cast<float*>(units), static_cast<int64_t*>(handles), rows, U);
  }
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}
