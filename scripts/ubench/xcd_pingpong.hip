// Microbenchmark: workgroup→XCC placement and intra- vs cross-XCD hand-off round trip on gfx950.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/ubench/xcd_pingpong.hip -o xcd_pingpong
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xf; }

__global__ void placement(unsigned* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = xcc_id();
}

typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int STORE_POL, int LOAD_POL>
__global__ void pingpong(unsigned* flags, int a, int b, int iters, unsigned long long* out, unsigned* xcc) {
  const int me = blockIdx.x;
  if (threadIdx.x != 0) return;
  if (me != a && me != b) return;
  xcc[me] = xcc_id();
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(flags, 0, 4096, 0x00020000);
  const int mine = (me == a) ? 0 : 64, theirs = (me == a) ? 64 : 0;   // different 256-B lines
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 1; i <= iters; ++i) {
    if (me == a) {
      __builtin_amdgcn_raw_buffer_store_b32(i, rs, mine * 4, 0, STORE_POL);
      unsigned spins = 0;
      while (__builtin_amdgcn_raw_buffer_load_b32(rs, theirs * 4, 0, LOAD_POL) != (unsigned)i) {
        if (++spins > (1u << 24)) { out[2] = 1; return; }
        asm volatile("" ::: "memory");   // the poll must be re-issued every iteration
      }
    } else {
      unsigned spins = 0;
      while (__builtin_amdgcn_raw_buffer_load_b32(rs, theirs * 4, 0, LOAD_POL) != (unsigned)i) {
        if (++spins > (1u << 24)) { out[2] = 1; return; }
        asm volatile("" ::: "memory");   // the poll must be re-issued every iteration
      }
      __builtin_amdgcn_raw_buffer_store_b32(i, rs, mine * 4, 0, STORE_POL);
    }
  }
  if (me == a) out[0] = __builtin_amdgcn_s_memrealtime() - t0;
}

template <int SP, int LP>
double run(int a, int b, unsigned* flags, unsigned long long* out, unsigned* xcc, int iters, unsigned* xa, unsigned* xb) {
  hipMemset(flags, 0, 4096);
  hipMemset(out, 0, 64);
  pingpong<SP, LP><<<64, 64>>>(flags, a, b, iters, out, xcc);
  hipDeviceSynchronize();
  unsigned long long h[3];
  hipMemcpy(h, out, 24, hipMemcpyDeviceToHost);
  unsigned hx[64];
  hipMemcpy(hx, xcc, sizeof(hx), hipMemcpyDeviceToHost);
  *xa = hx[a]; *xb = hx[b];
  if (h[2]) return -1;
  return h[0] * 10.0 / iters;   // ns per round trip (100 MHz clock)
}

int main() {
  unsigned* d;
  hipMalloc(&d, 4096 * 4);
  placement<<<256, 64>>>(d);
  hipDeviceSynchronize();
  std::vector<unsigned> h(256);
  hipMemcpy(h.data(), d, 256 * 4, hipMemcpyDeviceToHost);
  printf("placement (block: xcc) first 24:");
  for (int i = 0; i < 24; ++i) printf(" %d:%u", i, h[i]);
  int cnt[16] = {0};
  bool rr = true;
  for (int i = 0; i < 256; ++i) { cnt[h[i] & 15]++; if (h[i] != h[i % 8]) rr = false; }
  printf("\nper-xcc counts:");
  for (int i = 0; i < 8; ++i) printf(" %d", cnt[i]);
  printf("\nround-robin-by-8 consistent: %s\n", rr ? "yes" : "no");
  unsigned* flags; unsigned long long* out; unsigned* xcc;
  hipMalloc(&flags, 4096); hipMalloc(&out, 64); hipMalloc(&xcc, 256);
  const int iters = 20000;
  struct { int a, b; const char* name; } pairs[] = {{0, 8, "same-xcc"}, {0, 1, "cross-xcc"}};
  for (auto& p : pairs) {
    unsigned xa, xb;
    double t;
    t = run<0, 16>(p.a, p.b, flags, out, xcc, iters, &xa, &xb);
    printf("%-9s (xcc %u,%u) store plain / load sc1 : %.0f ns round trip\n", p.name, xa, xb, t);
    t = run<16, 16>(p.a, p.b, flags, out, xcc, iters, &xa, &xb);
    printf("%-9s (xcc %u,%u) store sc1   / load sc1 : %.0f ns round trip\n", p.name, xa, xb, t);
    t = run<1, 16>(p.a, p.b, flags, out, xcc, iters, &xa, &xb);
    printf("%-9s (xcc %u,%u) store sc0   / load sc1 : %.0f ns round trip\n", p.name, xa, xb, t);
  }
  return 0;
}
