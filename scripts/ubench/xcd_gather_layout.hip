// Microbenchmark: does the L2 placement of a team's exchange buffer bound the per-step all-gather latency?
// T workgroups of ONE XCD (blockIdx ≡ 0 mod 8 under the round-robin dispatch; checked with HW_REG_XCC_ID) each
// publish G tagged 8-B granules per step (plain stores) and gather all T·G granules (sc1 16-B polls, one chunk per
// thread per round, re-polling only missing chunks — the lstm_team.hip protocol), then __syncthreads. No compute.
// The gathered region is laid out as 128-B lines (8 chunks) placed `stride` bytes apart: stride 128 = contiguous
// (today's layout), larger strides put consecutive lines in other L2 channels / pages if the channel hash uses those
// address bits. Also: T = 16 vs 32 members at the same gathered bytes (team-size question, lstm_team.hip kT).
// Build: hipcc --offload-arch=gfx950 -O3 scripts/ubench/xcd_gather_layout.hip -o scripts/ubench/xcd_gather_layout
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xf; }

__device__ __forceinline__ unsigned chunk_off(int ci, int stride) { return (unsigned)((ci >> 3) * stride + (ci & 7) * 16); }

template <int NL, int POL>
__global__ __launch_bounds__(256, 1) void gather(unsigned char* buf, int T, int G, int steps, int stride,
                                                 unsigned long long* out, unsigned* xcc) {
  if (blockIdx.x % 8 != 0) return;
  const int m = blockIdx.x / 8;
  if (m >= T) return;
  if (threadIdx.x == 0) xcc[m] = xcc_id();
  const int tid = threadIdx.x;
  const int nchunk = T * G / 2;                          // 16-B chunks per step
  const int span = ((nchunk + 7) / 8) * stride;          // bytes per parity slot
  unsigned long long t0 = 0;
  for (int t = 1; t <= steps; ++t) {
    if (t == 2) t0 = __builtin_amdgcn_s_memrealtime();
    unsigned char* slot = buf + (size_t)(t & 1) * span;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slot, 0, span, 0x00020000);
    // publish: member m owns chunks [m·G/2, (m+1)·G/2); a lane stores one 8-B granule (half a chunk)
    for (int g = tid; g < G; g += 256) {
      const int ci = m * (G / 2) + g / 2;
      const u32x2 v = {(unsigned)(m * 1000 + g), (unsigned)t};
      __builtin_amdgcn_raw_buffer_store_b64(v, rs, chunk_off(ci, stride) + (g & 1) * 8, 0, 0);
    }
    i32x4 v[NL];
    bool ok[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) ok[i] = tid + 256 * i >= nchunk;
    unsigned spins = 0;
    while (true) {
#pragma unroll
      for (int i = 0; i < NL; ++i)
        if (!ok[i]) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, chunk_off(tid + 256 * i, stride), 0, POL);
      bool all = true;
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        ok[i] = ok[i] || (((unsigned)v[i].y == (unsigned)t) & ((unsigned)v[i].w == (unsigned)t));
        all &= ok[i];
      }
      if (__all(all)) break;
      if (++spins > (1u << 22)) { out[1] = 1; return; }
      asm volatile("" ::: "memory");
    }
    __syncthreads();
  }
  if (m == 0 && tid == 0) out[0] = __builtin_amdgcn_s_memrealtime() - t0;
}

int main() {
  unsigned char* buf;
  unsigned long long* out;
  unsigned* xcc;
  const size_t bytes = 64u << 20;
  hipMalloc(&buf, bytes);
  hipMalloc(&out, 64);
  hipMalloc(&xcc, 256);
  const int steps = 4000;
  struct Cfg { int T, G; } cfgs[] = {{32, 16}, {16, 32}, {32, 32}, {16, 64}, {8, 64}};
  for (const Cfg& c : cfgs) {
    for (int pol : {16, 17}) {
      for (int stride : {128, 256, 512, 1024, 2048, 4096, 8192}) {
        hipMemset(buf, 0, bytes);
        hipMemset(out, 0, 64);
        const int nchunk = c.T * c.G / 2;
        auto k = nchunk <= 256 ? (pol == 16 ? gather<1, 16> : gather<1, 17>) : (pol == 16 ? gather<2, 16> : gather<2, 17>);
        k<<<256, 256>>>(buf, c.T, c.G, steps, stride, out, xcc);
        hipDeviceSynchronize();
        unsigned long long h[2];
        hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
        unsigned hx[32];
        hipMemcpy(hx, xcc, 128, hipMemcpyDeviceToHost);
        bool same = true;
        for (int i = 1; i < c.T; ++i) same &= hx[i] == hx[0];
        printf("T=%2d G=%2d gather=%5d B pollpol=%2d stride=%5d: %s %.1f ns/step\n", c.T, c.G, c.T * c.G * 8, pol,
               stride, same ? "same-xcc" : "MIXED", h[1] ? -1.0 : h[0] * 10.0 / (steps - 1));
        fflush(stdout);
      }
    }
  }
  return 0;
}
