// Device return / advantage computation over a batch of rollouts (gfx950): segmented reverse linear scan +
// per-segment statistics + per-team EMA reward normalisation.
//
// Reference semantics (SURVEY §2.3 K-return / K-norm):
//   * discounted return over the whole padded rollout, G_t = r_t + γ·G_{t+1}, r_t = Σ_k subreward_k
//     (optimizer.py:52-53, 382 — scipy lfilter);
//   * per-team EMA(0.99) of the batch mean / std of those returns, updated once per rollout in arrival order, and the
//     normalised return (G − μ)/(σ + eps) (optimizer.py:335-343, 185-186);
//   * the PPO path (north star): GAE(γ, λ) over the valid prefix, A_t = δ_t + γλ·A_{t+1},
//     δ_t = r_t + γ·V_{t+1} − V_t (bootstrapped with the actor's V at the cut, 0 at a terminal), returns = A + V.
//   * mode 2, V-trace GAE (off-policy experience; Espeholt et al. 2018): the values are the LEARNER's (its forward at
//     the iteration's weights) and lr_t = log π(a_t) − log μ(a_t) against the actor's behaviour log-prob;
//     ρ_t = min(ρ̄, e^{lr_t}), c_t = λ·min(c̄, e^{lr_t}), A_t = ρ_t·δ_t + γ·c_t·A_{t+1}: the value target
//     v_t = V_t + A_t is the V-trace target and A_t the advantage (the off-policy-corrected GAE — at π = μ, weight
//     age 0, exactly mode 1's GAE(γ, λ)).
//
// Layout: all rollouts of an iteration are concatenated, each padded to a multiple of seq_len (segment s spans
// [off[s], off[s+1]) with T_s valid steps), so the learner's sequences are a plain reshape of the outputs.
//
//   1. returns_scan_kernel   — one 256-thread workgroup per rollout. Each thread owns a contiguous chunk, reduces it
//      to an affine map y ↦ X + p·y (the chunk's recurrence with the carry y coming from later steps), the 256 maps
//      are composed by a wave-level suffix scan (DPP shuffles) and a 4-entry LDS scan across waves, then every
//      thread replays its chunk from its exact carry. The forcing terms are computed once (pass 1) and parked in the
//      output buffer, which the same thread reads back in pass 2 (no cross-thread hazards). A third pass over the
//      thread's own outputs gives the two-pass mean / population std of the returns.
//   2. ema_normalize_kernel  — grid (segments × blocks-per-segment). Thread 0 of each block folds the statistics of
//      every earlier segment of the same team into the EMA state (rollouts are few, the fold is O(n_seg)), the block
//      normalises its slice, and the block that owns a team's last segment writes that team's final EMA state.
#include "common.h"

namespace {

constexpr int kT = 256;
constexpr int kWaves = kT / dca::kWave;

__device__ __forceinline__ float forcing(const float* __restrict__ rew, int K, const float* __restrict__ val,
                                         size_t row, int t, int T, float vboot, float gamma, int mode) {
  const float* rr = rew + row * K;
  float r = 0.f;
  for (int k = 0; k < K; ++k) r += rr[k];
  if (mode >= 1) {
    const float vn = (t + 1 < T) ? val[row + 1] : vboot;
    return r + gamma * vn - val[row];
  }
  return r;
}

// V-trace truncated importance weights of row i (mode 2): ρ = min(ρ̄, e^{lr}), the trace coefficient min(c̄, e^{lr})
__device__ __forceinline__ void vtrace_w(const float* __restrict__ lr, size_t i, float rho_bar, float c_bar,
                                         float& rho, float& cw) {
  const float r = __expf(fminf(lr[i], 30.f));
  rho = fminf(rho_bar, r);
  cw = fminf(c_bar, r);
}

__global__ __launch_bounds__(kT) void returns_scan_kernel(
    const float* __restrict__ rew, int K, const float* __restrict__ val, const float* __restrict__ lr,
    const int* __restrict__ off, const int* __restrict__ seglen, const float* __restrict__ boot,
    const unsigned char* __restrict__ done, float* __restrict__ ret, float* __restrict__ adv,
    float* __restrict__ stats, int mode, float gamma, float lam, float rho_bar, float c_bar) {
  const int s = blockIdx.x;
  const int base = off[s];
  const int P = off[s + 1] - base;
  const int T = min(seglen[s], P);
  const int n = (mode >= 1) ? T : P;                 // GAE: the padded tail is zero
  const float c0 = (mode >= 1) ? gamma * lam : gamma;
  const float vboot = (mode >= 1 && !done[s]) ? boot[s] : 0.f;
  float* acc_out = (mode >= 1) ? adv : ret;          // the scanned quantity
  const int per = (n + kT - 1) / kT;
  const int lo = min((int)threadIdx.x * per, n), hi = min(lo + per, n);

  // pass 1: forcing terms (parked in acc_out) and this chunk's map y -> X + p*y
  float X = 0.f, p = 1.f;
  for (int t = hi - 1; t >= lo; --t) {
    float d = forcing(rew, K, val, (size_t)base + t, t, T, vboot, gamma, mode);
    float c = c0;
    if (mode == 2) {
      float rho, cw;
      vtrace_w(lr, (size_t)base + t, rho_bar, c_bar, rho, cw);
      d *= rho;
      c = c0 * cw;
    }
    acc_out[base + t] = d;
    X = d + c * X;
    p *= c;
  }

  // suffix scan of the maps: lane l ends with the composition of lanes l..63 of its wave
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float xo = __shfl_down(X, o, 64), po = __shfl_down(p, o, 64);
    if (lane + o < 64) {
      X = X + p * xo;
      p = p * po;
    }
  }
  __shared__ float wx[kWaves], wp[kWaves], red[kWaves];
  if (lane == 0) {
    wx[w] = X;
    wp[w] = p;
  }
  __syncthreads();
  float y = 0.f;                                      // carry entering this wave from later waves
  for (int k = kWaves - 1; k > w; --k) y = wx[k] + wp[k] * y;
  const float x1 = __shfl_down(X, 1, 64), p1 = __shfl_down(p, 1, 64);
  float carry = (lane == 63) ? y : x1 + p1 * y;     // value of the recurrence just after this chunk

  // pass 2: replay the chunk from its carry; returns and the running sum for the statistics
  float sum = 0.f;
  for (int t = hi - 1; t >= lo; --t) {
    const size_t i = (size_t)base + t;
    const float d = acc_out[i];
    if (mode == 2) {
      float rho, cw;
      vtrace_w(lr, i, rho_bar, c_bar, rho, cw);
      carry = d + c0 * cw * carry;                    // A_t = ρ_t·δ_t + γλ·min(c̄, w_t)·A_{t+1}
      acc_out[i] = carry;
    } else {
      carry = d + c0 * carry;
      acc_out[i] = carry;
    }
    float g = carry;
    if (mode >= 1) {
      g = carry + val[i];
      ret[i] = g;
    }
    sum += g;
  }
  if (mode >= 1) {                                    // zero tail of a GAE segment
    for (int t = T + threadIdx.x; t < P; t += kT) {
      ret[base + t] = 0.f;
      adv[base + t] = 0.f;
    }
  }

  // two-pass mean / population std of the returns over the scanned range
  sum = dca::wave_sum(sum);
  if (lane == 0) red[w] = sum;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int k = 0; k < kWaves; ++k) tot += red[k];
  const float mean = tot / (float)max(n, 1);
  __syncthreads();
  float sq = 0.f;
  for (int t = lo; t < hi; ++t) {
    const float dlt = ret[base + t] - mean;
    sq += dlt * dlt;
  }
  sq = dca::wave_sum(sq);
  if (lane == 0) red[w] = sq;
  __syncthreads();
  if (threadIdx.x == 0) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) v += red[k];
    stats[2 * s] = mean;
    stats[2 * s + 1] = sqrtf(v / (float)max(n, 1));
  }
}

__global__ __launch_bounds__(kT) void ema_normalize_kernel(
    const float* __restrict__ ret, const int* __restrict__ off, const int* __restrict__ keys,
    const float* __restrict__ stats, int nseg, const float* __restrict__ ema_in, float* __restrict__ ema_out,
    float* __restrict__ norm, int normalize, float factor, float eps) {
  const int s = blockIdx.x;
  const int key = keys[s];
  __shared__ float sm, ss;
  if (threadIdx.x == 0) {
    float m = ema_in[3 * key], sd = ema_in[3 * key + 1];
    bool init = ema_in[3 * key + 2] != 0.f;
    for (int j = 0; j <= s; ++j) {
      if (keys[j] != key) continue;
      const float bm = stats[2 * j], bs = stats[2 * j + 1];
      if (!init) {
        m = bm;
        sd = bs;
        init = true;
      } else {
        m = m * factor + bm * (1.f - factor);
        sd = sd * factor + bs * (1.f - factor);
      }
    }
    sm = m;
    ss = sd;
    bool last = true;
    for (int j = s + 1; j < nseg && last; ++j) last = keys[j] != key;
    if (last && blockIdx.y == 0) {
      ema_out[3 * key] = m;
      ema_out[3 * key + 1] = sd;
      ema_out[3 * key + 2] = 1.f;
    }
  }
  if (!normalize) return;
  __syncthreads();
  const float m = sm, inv = 1.f / (ss + eps);
  const int base = off[s], P = off[s + 1] - base;
  for (int t = blockIdx.y * kT + threadIdx.x; t < P; t += gridDim.y * kT) norm[base + t] = (ret[base + t] - m) * inv;
}


// ---- V-trace inside the learner step (time-major rows r = t·B + b of one minibatch) ------------------------------
// The advantages and value targets of a minibatch from the step's OWN forward: V_t = z[r][vcol] (the heads GEMM's
// value column) and log π(a_t) = lp[r] (the heads kernel's selected-action log-prob) at the weights of this very
// step, against the actor's behaviour log-prob mu[r]. vt[r] = {reward, bootstrap, valid, last}: `last` marks the last
// row of an episode segment inside its sequence (the episode's end — bootstrap 0 if done, else the actor's
// bootstrap value — or a sequence boundary the rollout continues past — bootstrap the actor's value of the next
// row). ρ_t = min(ρ̄, w_t), w_t = e^{lp − mu}; A_t = ρ_t·δ_t + γλ·min(c̄, w_t)·A_{t+1} (A_{t+1} = 0 at `last`);
// adv = A, ret = A + V (V-trace target; GAE(γ, λ) exactly when π = μ). One workgroup per sequence: each thread owns
// a chunk of steps, the chunks' affine maps are composed by a wave suffix scan + an LDS pass over the 4 waves.
// stats[b] = Σ over valid rows of {ρ, [w > ρ̄], mu − lp, 1}.
__global__ __launch_bounds__(kT) void vtrace_step_kernel(
    const float* __restrict__ z, int ldz, int vcol, const float* __restrict__ lp, const float* __restrict__ mu,
    const float* __restrict__ vt, float* __restrict__ adv, float* __restrict__ ret, float* __restrict__ stats, int B,
    int S, float gamma, float lam, float rho_bar, float c_bar) {
  const int b = blockIdx.x;
  const int per = (S + kT - 1) / kT;
  const int lo = min((int)threadIdx.x * per, S), hi = min(lo + per, S);
  float X = 0.f, p = 1.f;
  float s_rho = 0.f, s_tr = 0.f, s_kl = 0.f, s_n = 0.f;
  for (int t = hi - 1; t >= lo; --t) {
    const size_t r = (size_t)t * B + b;
    const float4 v4 = *reinterpret_cast<const float4*>(vt + 4 * r);       // reward, bootstrap, valid, last
    const bool valid = v4.z > 0.f, last = v4.w > 0.f || t == S - 1;
    const float V = z[r * ldz + vcol];
    const float nextV = last ? v4.y : z[(r + B) * ldz + vcol];
    const float dl = lp[r] - mu[r];
    const float w = __expf(fminf(dl, 30.f));
    const float rho = fminf(rho_bar, w), cw = fminf(c_bar, w);
    const float d = valid ? rho * (v4.x + gamma * nextV - V) : 0.f;
    const float k = (valid && !last) ? gamma * lam * cw : 0.f;
    adv[r] = d;                                       // parked: the forcing term and the coefficient
    ret[r] = k;
    X = d + k * X;
    p *= k;
    if (valid) {
      s_rho += rho;
      s_tr += w > rho_bar * (1.f + 1e-6f) ? 1.f : 0.f;
      s_kl += -dl;
      s_n += 1.f;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float xo = __shfl_down(X, o, 64), po = __shfl_down(p, o, 64);
    if (lane + o < 64) {
      X = X + p * xo;
      p = p * po;
    }
  }
  __shared__ float wx[kWaves], wp[kWaves], red[4][kWaves];
  if (lane == 0) {
    wx[w] = X;
    wp[w] = p;
  }
  __syncthreads();
  float y = 0.f;
  for (int k = kWaves - 1; k > w; --k) y = wx[k] + wp[k] * y;
  const float x1 = __shfl_down(X, 1, 64), p1 = __shfl_down(p, 1, 64);
  float carry = (lane == 63) ? y : x1 + p1 * y;
  for (int t = hi - 1; t >= lo; --t) {
    const size_t r = (size_t)t * B + b;
    const float d = adv[r], k = ret[r];
    carry = d + k * carry;
    adv[r] = carry;
    ret[r] = vt[4 * r + 2] > 0.f ? carry + z[r * ldz + vcol] : 0.f;
  }
  s_rho = dca::wave_sum(s_rho);
  s_tr = dca::wave_sum(s_tr);
  s_kl = dca::wave_sum(s_kl);
  s_n = dca::wave_sum(s_n);
  if (lane == 0) {
    red[0][w] = s_rho;
    red[1][w] = s_tr;
    red[2][w] = s_kl;
    red[3][w] = s_n;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) v += red[threadIdx.x][k];
    stats[4 * b + threadIdx.x] = v;
  }
}
}  // namespace

extern "C" hipError_t dca_returns(const float* rew, int K, const float* val, const float* lr, const int* off,
                                  const int* seglen, const float* boot, const unsigned char* done, const int* keys,
                                  int nseg, int max_len, float* ret, float* adv, float* norm, float* stats,
                                  const float* ema_in, float* ema_out, int mode, int normalize, float gamma, float lam,
                                  float rho_bar, float c_bar, float factor, float eps, hipStream_t st) {
  if (nseg <= 0) return hipSuccess;
  hipLaunchKernelGGL(returns_scan_kernel, dim3(nseg), dim3(kT), 0, st, rew, K, val, lr, off, seglen, boot, done, ret,
                     adv, stats, mode, gamma, lam, rho_bar, c_bar);
  DCA_CHECK_LAUNCH();
  const int by = normalize ? max(1, min(64, (max_len + 4 * kT - 1) / (4 * kT))) : 1;
  hipLaunchKernelGGL(ema_normalize_kernel, dim3(nseg, by), dim3(kT), 0, st, ret, off, keys, stats, nseg, ema_in,
                     ema_out, norm, normalize, factor, eps);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}

extern "C" hipError_t dca_vtrace_step(const float* z, int ldz, int vcol, const float* lp, const float* mu,
                                      const float* vt, float* adv, float* ret, float* stats, int B, int S,
                                      float gamma, float lam, float rho_bar, float c_bar, hipStream_t st) {
  if (B <= 0 || S <= 0) return hipSuccess;
  hipLaunchKernelGGL(vtrace_step_kernel, dim3(B), dim3(kT), 0, st, z, ldz, vcol, lp, mu, vt, adv, ret, stats, B, S,
                     gamma, lam, rho_bar, c_bar);
  DCA_CHECK_LAUNCH();
  return hipSuccess;
}
