// Issue rate of v_dot2_f32_bf16 vs v_fma_f32 vs v_mfma_f32_16x16x32_bf16 for ONE wave per SIMD (a latency-bound
// persistent kernel's situation): cycles per instruction from s_memtime around an unrolled loop of independent chains.
// Measured (MI355X): v_dot2_f32_bf16 9.0, v_fma_f32 5.5, v_mfma_f32_16x16x32_bf16 18.0 cycles — a one-row (B = 1)
// recurrent mat-vec on dot2 VALU (64 per lane) costs ≈2× the 16 MFMAs it would replace.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef short bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2r __attribute__((ext_vector_type(2)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k_dot2(float* out, long long* cyc, int iters) {
  bf16x2r a = {(__bf16)1.0f, (__bf16)0.5f}, b = {(__bf16)0.25f, (__bf16)(float)threadIdx.x};
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_fdot2_f32_bf16(a, b, acc[j], false);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int j = 0; j < 8; ++j) s += acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_fma(float* out, long long* cyc, int iters) {
  float a = 1.0001f, b = (float)threadIdx.x;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_fmaf(a, acc[j], b);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int j = 0; j < 8; ++j) s += acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_mfma(float* out, long long* cyc, int iters) {
  bf16x8 a = {1, 2, 3, 4, 5, 6, 7, (short)threadIdx.x}, b = a;
  f32x4 acc = {0, 0, 0, 0};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out;
  long long* cyc;
  hipMalloc(&out, 256 * 64 * sizeof(float));
  hipMalloc(&cyc, 256 * sizeof(long long));
  const int iters = 4096;
  long long h[256];
  const char* names[3] = {"v_dot2_f32_bf16", "v_fma_f32", "v_mfma_f32_16x16x32_bf16"};
  for (int k = 0; k < 3; ++k) {
    for (int rep = 0; rep < 2; ++rep) {
      // 256 blocks of ONE wave each: one wave per SIMD on a quarter of the SIMDs
      if (k == 0) k_dot2<<<256, 64>>>(out, cyc, iters);
      if (k == 1) k_fma<<<256, 64>>>(out, cyc, iters);
      if (k == 2) k_mfma<<<256, 64>>>(out, cyc, iters);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    long long mn = h[0];
    for (int i = 1; i < 256; ++i) mn = h[i] < mn ? h[i] : mn;
    printf("%-28s %.2f cycles per instruction (one wave)\n", names[k], (double)mn / (iters * 8.0));
  }
  return 0;
}
