// Microbenchmark: per-step latency of an all-gather among T workgroups of ONE XCD through its L2 (tagged 8-B
// granules, plain stores, sc1 polls), no compute. Workgroups are placed with blockIdx ≡ 0 (mod 8) so they share
// XCD 0 under the observed round-robin dispatch (verified with HW_REG_XCC_ID).
// Build: hipcc --offload-arch=gfx950 -O3 scripts/ubench/xcd_allgather.hip -o scripts/ubench/xcd_allgather
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xf; }

// T members; each publishes G granules (8 B) per step; every member gathers T*G granules.
__global__ __launch_bounds__(256, 1) void allgather(unsigned long long* buf, int T, int G, int steps,
                                                    unsigned long long* out, unsigned* xcc, int store_pol) {
  if (blockIdx.x % 8 != 0) return;
  const int m = blockIdx.x / 8;
  if (m >= T) return;
  if (threadIdx.x == 0) xcc[m] = xcc_id();
  const int tid = threadIdx.x;
  const int total = T * G;                     // granules per step
  const int nchunk = total / 2;                // 16-B chunks
  unsigned long long t0 = 0;
  for (int t = 1; t <= steps; ++t) {
    if (t == 2) t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* slot = buf + (size_t)(t & 1) * total;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slot, 0, total * 8, 0x00020000);
    // publish my G granules
    for (int g = tid; g < G; g += 256) {
      const u32x2 v = {(unsigned)(m * 1000 + g), (unsigned)t};
      if (store_pol) __builtin_amdgcn_raw_buffer_store_b64(v, rs, (m * G + g) * 8, 0, 16);
      else __builtin_amdgcn_raw_buffer_store_b64(v, rs, (m * G + g) * 8, 0, 0);
    }
    // gather all
    const int per = (nchunk + 255) / 256;
    for (int i = 0; i < per; ++i) {
      const int ci = tid + 256 * i;
      if (ci >= nchunk) break;
      unsigned spins = 0;
      while (true) {
        i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, ci * 16, 0, 16);
        if ((unsigned)v.y == (unsigned)t && (unsigned)v.w == (unsigned)t) break;
        if (++spins > (1u << 22)) { out[1] = 1; return; }
        asm volatile("" ::: "memory");
      }
    }
    __syncthreads();
  }
  if (m == 0 && tid == 0) out[0] = __builtin_amdgcn_s_memrealtime() - t0;
}

int main() {
  unsigned long long *buf, *out;
  unsigned* xcc;
  hipMalloc(&buf, 1 << 24);
  hipMalloc(&out, 64);
  hipMalloc(&xcc, 256);
  const int steps = 2000;
  for (int pol : {0, 16}) {
    for (int T : {4, 8, 16, 32}) {
      for (int bytes_per_member : {64, 256, 512, 2048}) {
        const int G = bytes_per_member / 8;
        hipMemset(buf, 0, 1 << 24);
        hipMemset(out, 0, 64);
        allgather<<<256, 256>>>(buf, T, G, steps, out, xcc, pol);
        hipDeviceSynchronize();
        unsigned long long h[2];
        hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
        unsigned hx[32];
        hipMemcpy(hx, xcc, 128, hipMemcpyDeviceToHost);
        bool same = true;
        for (int i = 1; i < T; ++i) same &= hx[i] == hx[0];
        printf("store=%s T=%2d publish=%5d B/member gather=%6d B: %s %.0f ns/step\n", pol ? "sc1  " : "plain", T,
               bytes_per_member, bytes_per_member * T, same ? "same-xcc" : "MIXED", h[1] ? -1.0 : h[0] * 10.0 / (steps - 1));
      }
    }
  }
  return 0;
}
