// Device side of the learner's look-ahead ingest (learner/ingest.py IngestPipeline.expand, learner/optimizer.py
// _normalize_advantages), each a chain of small PyTorch launches before:
//
//   ingest_scatter_kernel  the staged iteration's packed valid rows → the zero-padded [L rows] layout of every field
//                          in ONE launch, plus the validity mask: padded row r takes valid row inv[r] (or zeros when
//                          inv[r] < 0). Was a zero_() and an index_copy_() per field and a zero_() + index_fill_() for
//                          the mask (16 launches).
//   adv_normalize_kernel   PPO advantage normalisation over the valid rows, (adv − mean) / (std + eps) · valid, in one
//                          single-workgroup launch with fp64 sums in a fixed order (was ≈10 launches: masked sums,
//                          mean, squared deviations, sqrt, the affine map).
#include "common.h"

namespace {

constexpr int kMaxFields = 16;
struct ScatterTable {
  unsigned char* dst[kMaxFields];
  const unsigned char* src[kMaxFields];
  int row_bytes[kMaxFields];
  int chunks[kMaxFields];          // 16-byte chunks per row
  long long start[kMaxFields + 1]; // prefix sum of L · chunks
  int n;
};

__global__ __launch_bounds__(256) void ingest_scatter_kernel(ScatterTable tab, const int* __restrict__ inv, int L,
                                                             int nsrc, float* __restrict__ valid) {
  const long long total = tab.start[tab.n];
  const long long stride = (long long)gridDim.x * 256;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += stride) {
    int lo = 0, hi = tab.n - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tab.start[mid] <= e) lo = mid; else hi = mid - 1;
    }
    const long long k = e - tab.start[lo];
    const int r = (int)(k / tab.chunks[lo]), c = (int)(k % tab.chunks[lo]);
    const int rb = tab.row_bytes[lo];
    const int j = inv[r] < nsrc ? inv[r] : -1;      // (a source row out of range reads nothing: zeros)
    const int b0 = 16 * c, nb = min(16, rb - b0);
    unsigned char* d = tab.dst[lo] + (size_t)r * rb + b0;
    if (j < 0) {
      if (nb == 16 && ((reinterpret_cast<unsigned long long>(d) & 15ull) == 0)) {
        *reinterpret_cast<uint4*>(d) = make_uint4(0u, 0u, 0u, 0u);
      } else {
        for (int b = 0; b < nb; ++b) d[b] = 0;
      }
    } else {
      const unsigned char* s = tab.src[lo] + (size_t)j * rb + b0;
      if (nb == 16 && (((reinterpret_cast<unsigned long long>(d) | reinterpret_cast<unsigned long long>(s)) & 15ull) == 0)) {
        *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(s);
      } else {
        for (int b = 0; b < nb; ++b) d[b] = s[b];
      }
    }
  }
  if (valid) {
    for (long long r = (long long)blockIdx.x * 256 + threadIdx.x; r < L; r += stride) valid[r] = (inv[r] >= 0 && inv[r] < nsrc) ? 1.f : 0.f;
  }
}

// one workgroup of 1024 threads: fixed-order fp64 partial sums (thread t owns rows t, t + 1024, …), then a fixed tree
__global__ __launch_bounds__(1024) void adv_normalize_kernel(const float* __restrict__ adv,
                                                             const float* __restrict__ valid, float* __restrict__ out,
                                                             int L, float eps) {
  __shared__ double red[1024];
  const int t = threadIdx.x;
  double sv = 0.0, sa = 0.0;
  for (int r = t; r < L; r += 1024) {
    const double v = valid[r];
    sv += v;
    sa += (double)adv[r] * v;
  }
  auto tree = [&](double x) {
    red[t] = x;
    __syncthreads();
    for (int s = 512; s > 0; s >>= 1) {
      if (t < s) red[t] += red[t + s];
      __syncthreads();
    }
    const double r = red[0];
    __syncthreads();
    return r;
  };
  const double n = fmax(tree(sv), 1.0);
  const double mu = tree(sa) / n;
  double sq = 0.0;
  for (int r = t; r < L; r += 1024) {
    const double d = (double)adv[r] - mu;
    sq += d * d * (double)valid[r];
  }
  const double sd = sqrt(tree(sq) / n);
  const float muf = (float)mu, den = (float)sd + eps;     // the torch expression's fp32 operations, in its order
  for (int r = t; r < L; r += 1024) out[r] = ((adv[r] - muf) / den) * valid[r];
}

}  // namespace

extern "C" hipError_t dca_ingest_scatter(void* const* dst, const void* const* src, const int* row_bytes, int n,
                                         const int* inv, int L, int nsrc, float* valid, hipStream_t st) {
  if (n < 0 || n > kMaxFields || L < 0) return hipErrorInvalidValue;
  ScatterTable tab;
  tab.n = n;
  tab.start[0] = 0;
  for (int i = 0; i < n; ++i) {
    if (row_bytes[i] <= 0) return hipErrorInvalidValue;
    tab.dst[i] = static_cast<unsigned char*>(dst[i]);
    tab.src[i] = static_cast<const unsigned char*>(src[i]);
    tab.row_bytes[i] = row_bytes[i];
    tab.chunks[i] = (row_bytes[i] + 15) / 16;
    tab.start[i + 1] = tab.start[i] + (long long)L * tab.chunks[i];
  }
  long long blocks = (tab.start[n] + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  ingest_scatter_kernel<<<(int)blocks, 256, 0, st>>>(tab, inv, L, nsrc, valid);
  return hipGetLastError();
}

extern "C" hipError_t dca_adv_normalize(const float* adv, const float* valid, float* out, int L, float eps,
                                        hipStream_t st) {
  if (L < 0) return hipErrorInvalidValue;
  adv_normalize_kernel<<<1, 1024, 0, st>>>(adv, valid, out, L, eps);
  return hipGetLastError();
}
