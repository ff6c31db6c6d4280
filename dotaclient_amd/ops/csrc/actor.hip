// Actor-side inference kernels (gfx950): fused LSTM cell and fused masked hierarchical action sampling.
//
// Reference actor step (agent.py:641-660, policy.py:171-283): policy.single → action_masks → select_actions
// (enum first, then x,y for MOVE or target_unit for ATTACK, each a masked categorical) → head_masks ∧ action masks.
// Here one launch does it for a whole batch of players, one wave per player row:
//   * pointer logits q·embᵀ over the unit slots, validity from unit handles (self slot 0 never targetable; ATTACK
//     disabled when no unit is targetable — policy.py:272-283);
//   * masked log-softmax of the 4 heads, Gumbel-max sampling with a counter-based hash RNG (seed, step counter,
//     row, head, entry) — deterministic for a given seed/counter, graph-capturable (the counter lives in device
//     memory and is bumped by the caller);
//   * hierarchical selection, joint log-prob of the sampled action, one-hot actions and selected-heads masks
//     (the experience record), and V(s).
#include "common.h"

namespace {

constexpr int kQ = 128;

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ float gumbel(unsigned long long seed, unsigned long long ctr, int row, int head, int e) {
  const unsigned long long h =
      mix64(seed ^ mix64(ctr ^ mix64(((unsigned long long)row << 24) ^ ((unsigned long long)head << 16) ^ e)));
  const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);   // (0,1)
  return -__logf(-__logf(u));
}

// arg-max over lanes of (v); ties → lowest lane
__device__ __forceinline__ int wave_argmax(float v, int lane) {
  int idx = lane;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
  }
  return idx;
}

__device__ __forceinline__ void load8(const short* p, float* v) {
  const dca::bf16x8 b = *reinterpret_cast<const dca::bf16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = dca::bf2f(b[j]);
}
__device__ __forceinline__ void load8(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// HT: unit handles int64 (the reference's layout) or int32 (the fp8 step's compact staging); ET: the unit embeddings
// bf16 (short) or fp32 (the IEEE-fp32 actor step and the 5v5 attention block's output)
template <typename HT, typename ET>
__global__ __launch_bounds__(256) void sample_kernel(const float* __restrict__ z, int ldz,
                                                     const ET* __restrict__ emb,
                                                     const HT* __restrict__ handles, int N, int U,
                                                     unsigned long long seed, const long long* __restrict__ ctr,
                                                     int* __restrict__ idx_out, unsigned char* __restrict__ act_out,
                                                     unsigned char* __restrict__ msk_out, float* __restrict__ logp_out,
                                                     float* __restrict__ value_out) {
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int n = blockIdx.x * 4 + wv;
  if (n >= N) return;
  const int A = 21 + U;
  const float* zr = z + (size_t)n * ldz;
  // ---- pointer logits (4 units per wave instruction, 16 lanes per unit)
  const int ks = lane & 15, ug = lane >> 4;
  float q8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) q8[j] = zr[8 * ks + j];
  float tl = -INFINITY;   // lane u holds target logit u
  for (int it = 0; it * 4 < U; ++it) {
    const int u = it * 4 + ug;
    float d = 0.f;
    if (u < U) {
      float v[8];
      load8(emb + ((size_t)n * U + u) * kQ + 8 * ks, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) d += q8[j] * v[j];
    }
    d = dca::group_sum<16>(d);
    // lane (16·g) holds unit it*4+g; move it to lane u
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float dv = __shfl(d, 16 * g, 64);
      if (lane == it * 4 + g) tl = dv;
    }
  }
  // ---- validity
  const bool tvalid = lane < U && lane != 0 && handles[(size_t)n * U + lane] != -1;
  const bool any_target = __any(tvalid);
  const unsigned long long c = *ctr;
  const int hoff[4] = {0, 3, 12, 21};
  const int hw[4] = {3, 9, 9, U};
  int pick[4];
  float plogp[4];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const bool in = lane < hw[h];
    float lg = 0.f;
    bool m = false;
    if (h == 3) { lg = tl; m = tvalid; }
    else if (in) { lg = zr[kQ + hoff[h] + lane]; m = (h == 0 && lane == 2) ? any_target : true; }
    const float v = m ? lg : -INFINITY;
    float mx = dca::wave_max(v);
    const bool any = mx > -INFINITY;
    if (!any) mx = 0.f;
    float s = dca::wave_sum(m ? __expf(lg - mx) : 0.f);
    if (!(s > 0.f)) s = 1.f;
    const float lp = lg - mx - __logf(s);
    const float key = m ? lp + gumbel(seed, c, n, h, lane) : -INFINITY;
    int k = wave_argmax(key, lane);
    if (!any) k = 0;
    pick[h] = k;
    plogp[h] = __shfl(lp, k, 64);
    // selected-heads mask (head sampled ∧ valid) and one-hot action, written after the enum is known
    if (h == 3) {
      const int e = pick[0];
      const bool mv = e == 1, at = e == 2;
      for (int hh = 0; hh < 4; ++hh) {
        const bool head_on = hh == 0 || ((hh == 1 || hh == 2) && mv) || (hh == 3 && at);
        for (int j = lane; j < hw[hh]; j += 64) {
          bool valid = true;
          if (hh == 3) valid = j != 0 && handles[(size_t)n * U + j] != -1;
          if (hh == 0 && j == 2) valid = any_target;
          msk_out[(size_t)n * A + hoff[hh] + j] = (head_on && valid) ? 1 : 0;
          act_out[(size_t)n * A + hoff[hh] + j] = (head_on && j == pick[hh]) ? 1 : 0;
        }
      }
      if (lane == 0) {
        idx_out[n * 4 + 0] = pick[0];
        idx_out[n * 4 + 1] = pick[1];
        idx_out[n * 4 + 2] = pick[2];
        idx_out[n * 4 + 3] = pick[3];
        logp_out[n] = plogp[0] + (mv ? plogp[1] + plogp[2] : 0.f) + (at ? plogp[3] : 0.f);
        value_out[n] = zr[kQ + 21];
      }
    }
  }
}

// gates (N, 4H) pre-activations (x·W_ihᵀ + h·W_hhᵀ + b, fp32) → h, c (fp32) in place + h bf16 copy
__global__ __launch_bounds__(256) void lstm_cell_kernel(const float* __restrict__ g, float* __restrict__ h,
                                                        float* __restrict__ c, short* __restrict__ h16,
                                                        const float* __restrict__ active, int N, int H) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N * H) return;
  const int n = i / H, j = i % H;
  if (active && active[n] == 0.f) return;   // slot not stepped this call: its state is left untouched
  const float* gr = g + (size_t)n * 4 * H;
  const float ig = dca::sigmoidf_(gr[j]), fg = dca::sigmoidf_(gr[H + j]), gg = dca::tanhf_(gr[2 * H + j]),
              og = dca::sigmoidf_(gr[3 * H + j]);
  const float cn = fg * c[i] + ig * gg;
  const float hn = og * dca::tanhf_(cn);
  c[i] = cn;
  h[i] = hn;
  h16[i] = dca::f2bf(hn);
}

// Actor step input staging: episode resets (h, c *= keep) and the combined gate-GEMM operand xh = [x | bf16(h)]
// (N, P + H) bf16, so x·W_ihᵀ + h·W_hhᵀ + b is ONE GEMM (K = P + H, bias in its epilogue). pre: the pre-RNN
// activations (N, P) bf16 (hipBLASLt ReLU epilogue). Replaces three elementwise passes, a cast and two GEMM-output adds.
__global__ __launch_bounds__(256) void actor_state_prep_kernel(const short* __restrict__ pre, float* __restrict__ h,
                                                               float* __restrict__ c, const float* __restrict__ keep,
                                                               short* __restrict__ xh, int N, int P, int H,
                                                               long long* __restrict__ bump) {
  const int per = (P > H ? P : H) / 4;            // one 4-column quad of the row per thread
  const int i = blockIdx.x * 256 + threadIdx.x;
  // the sampling kernel (later in the step) reads the counter: bumping it here saves a one-element launch
  if (bump && i == 0) bump[0] += 1;
  if (i >= N * per) return;
  const int n = i / per, j = (i % per) * 4;
  short* xr = xh + (size_t)n * (P + H);
  if (j < P) *reinterpret_cast<uint2*>(xr + j) = *reinterpret_cast<const uint2*>(pre + (size_t)n * P + j);
  if (j < H) {
    const float k = keep[n];
    float4 hv = *reinterpret_cast<const float4*>(h + (size_t)n * H + j);
    if (k != 1.f) {
      float4 cv = *reinterpret_cast<const float4*>(c + (size_t)n * H + j);
      hv.x *= k; hv.y *= k; hv.z *= k; hv.w *= k;
      cv.x *= k; cv.y *= k; cv.z *= k; cv.w *= k;
      *reinterpret_cast<float4*>(h + (size_t)n * H + j) = hv;
      *reinterpret_cast<float4*>(c + (size_t)n * H + j) = cv;
    }
    const unsigned lo = (unsigned)(unsigned short)dca::f2bf(hv.x) | ((unsigned)(unsigned short)dca::f2bf(hv.y) << 16);
    const unsigned hi = (unsigned)(unsigned short)dca::f2bf(hv.z) | ((unsigned)(unsigned short)dca::f2bf(hv.w) << 16);
    *reinterpret_cast<uint2*>(xr + P + j) = make_uint2(lo, hi);
  }
}

}  // namespace

extern "C" hipError_t dca_actor_state_prep(const short* pre, float* h, float* c, const float* keep, short* xh, int N,
                                           int P, int H, long long* bump, hipStream_t st) {
  if (H % 4 || P % 4) return hipErrorInvalidValue;
  const int per = (P > H ? P : H) / 4;
  actor_state_prep_kernel<<<(N * per + 255) / 256, 256, 0, st>>>(pre, h, c, keep, xh, N, P, H, bump);
  return hipGetLastError();
}

extern "C" hipError_t dca_sample_actions(const float* z, int ldz, const void* emb, int emb_f32, const void* handles,
                                         int h32, int N, int U, unsigned long long seed, const long long* ctr,
                                         int* idx, unsigned char* act, unsigned char* msk, float* logp, float* value,
                                         hipStream_t st) {
  if (U < 1 || U > 64 || ldz < kQ + 22) return hipErrorInvalidValue;
  const dim3 grid((N + 3) / 4), block(256);
#define DCA_SAMPLE(HT, ET)                                                                                   \
  hipLaunchKernelGGL((sample_kernel<HT, ET>), grid, block, 0, st, z, ldz, static_cast<const ET*>(emb),    \
                     static_cast<const HT*>(handles), N, U, seed, ctr, idx, act, msk, logp, value)
  if (h32) {
    if (emb_f32) DCA_SAMPLE(int, float); else DCA_SAMPLE(int, short);
  } else {
    if (emb_f32) DCA_SAMPLE(long long, float); else DCA_SAMPLE(long long, short);
  }
#undef DCA_SAMPLE
  return hipGetLastError();
}

extern "C" hipError_t dca_lstm_cell(const float* gates, float* h, float* c, short* h16, const float* active, int N,
                                    int H, hipStream_t st) {
  lstm_cell_kernel<<<(N * H + 255) / 256, 256, 0, st>>>(gates, h, c, h16, active, N, H);
  return hipGetLastError();
}
