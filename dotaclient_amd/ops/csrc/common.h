// Shared device helpers for the dotaclient_amd HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define DCA_CHECK_LAUNCH() do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return e__; } while (0)

namespace dca {

constexpr int kWave = 64;   // CDNA wavefront width

typedef short bf16x8 __attribute__((ext_vector_type(8)));   // 8 bf16 = one 16x16x32 MFMA A/B fragment
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));      // 16x16 MFMA accumulator fragment
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Sum over a group of `W` consecutive lanes (W power of two, <= 64).
template <int W>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <int W>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// bf16 <-> f32 (round-to-nearest-even), as raw 16-bit patterns.
__device__ __forceinline__ short f2bf(float f) {
  // round-to-nearest-even in one v_cvt_pk_bf16_f32 (gfx950); NaN stays NaN
  return __builtin_bit_cast(short, (__bf16)f);
}
__device__ __forceinline__ float bf2f(short h) { return __uint_as_float(((uint32_t)(uint16_t)h) << 16); }

// v_rcp_f32 (1 ulp) instead of an IEEE division (a ~10-instruction sequence on the recurrence's critical path)
__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanhf_(float x) {
  // tanh via exp: accurate to ~2e-7 relative for |x| < 9, saturates beyond.
  float e = __expf(-2.f * fabsf(x));
  float t = (1.f - e) * __builtin_amdgcn_rcpf(1.f + e);
  return copysignf(t, x);
}

// XCD-aware bijective remap of a 1-D block id (cdna_hip_programming.md §5 'XCD swizzle must be bijective'):
// consecutive logical tiles land on the same XCD (shared L2).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

}  // namespace dca
