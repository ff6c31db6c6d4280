// Python bindings for the dotaclient_amd HIP kernels.
//
// Kernels live in *.hip translation units that know nothing about torch (raw pointers + hipStream_t, extern "C"
// launchers); this file only validates tensors, picks the current HIP stream (so every op composes with torch
// streams and hipGraph capture) and forwards. Keeping torch headers out of the device TUs keeps their rebuilds fast.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "launchers.h"

namespace {

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

inline void hip_check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, " failed: ", hipGetErrorString(e));
}

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_DT(t, dt) TORCH_CHECK((t).scalar_type() == (dt), #t " must be " #dt)
#define CHECK_F32(t) CHECK_DEV(t); CHECK_CONTIG(t); CHECK_DT(t, at::kFloat)
#define CHECK_BF16(t) CHECK_DEV(t); CHECK_CONTIG(t); CHECK_DT(t, at::kBFloat16)
#define CHECK_I32(t) CHECK_DEV(t); CHECK_CONTIG(t); CHECK_DT(t, at::kInt)
#define CHECK_U8(t) CHECK_DEV(t); CHECK_CONTIG(t); CHECK_DT(t, at::kByte)

template <typename T>
inline T* ptr(const torch::Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }

// ------------------------------------------------------------------------------------------------------------
// header: leading elements of the flat buffers that are not parameters (excluded from the norm); skip: optional
// 1-element f32 device flag — nonzero → the step changes nothing (failed recurrence on some DP rank).
void adam_step(torch::Tensor param, torch::Tensor grad, torch::Tensor m, torch::Tensor v, torch::Tensor seg,
               torch::Tensor counts, torch::Tensor steps, torch::Tensor norm_out, double lr, double b1, double b2,
               double eps, double max_norm, bool divide, int64_t header, c10::optional<torch::Tensor> skip,
               c10::optional<torch::Tensor> nonfinite) {
  CHECK_F32(param); CHECK_F32(grad); CHECK_F32(m); CHECK_F32(v); CHECK_I32(seg); CHECK_F32(counts);
  CHECK_F32(steps); CHECK_F32(norm_out);
  const int64_t n = param.numel();
  TORCH_CHECK(n % 4 == 0 && grad.numel() == n && m.numel() == n && v.numel() == n && seg.numel() == n,
              "adam_step: flat buffers must share a length that is a multiple of 4");
  TORCH_CHECK(counts.numel() == steps.numel(), "adam_step: counts/steps length mismatch");
  const float* sk = nullptr;
  if (skip.has_value() && skip->defined()) {
    CHECK_F32((*skip));
    TORCH_CHECK(skip->numel() >= 1, "adam_step: skip must hold one float");
    sk = ptr<float>(*skip);
  }
  float* nf = nullptr;
  if (nonfinite.has_value() && nonfinite->defined()) {
    CHECK_F32((*nonfinite));
    TORCH_CHECK(nonfinite->numel() >= 1, "adam_step: nonfinite must hold one float");
    nf = ptr<float>(*nonfinite);
  }
  auto partials = torch::empty({dca_adam_partials_len((int)counts.numel())}, param.options());
  hip_check(dca_adam_step(ptr<float>(param), ptr<float>(grad), ptr<float>(m), ptr<float>(v), ptr<int>(seg), n,
                          ptr<float>(counts), ptr<float>(steps), (int)counts.numel(), ptr<float>(partials),
                          ptr<float>(norm_out), (float)lr, (float)b1, (float)b2, (float)eps, (float)max_norm,
                          cur_stream(), divide ? 1 : 0, header, sk, nf),
            "dca_adam_step");
}

// dst_i += scale · src_i over a list of fp32 tensors in one graph-capturable launch (scale: 1-element device
// tensor or None = 1).
// the look-ahead ingest's expand (learner/ingest.py): padded row r of every field takes packed valid row inv[r]
// (zeros when inv[r] < 0); valid[r] = inv[r] >= 0
void ingest_scatter(std::vector<torch::Tensor> dst, std::vector<torch::Tensor> src, torch::Tensor inv,
                    torch::Tensor valid) {
  TORCH_CHECK(dst.size() == src.size() && dst.size() <= 16, "ingest_scatter: at most 16 (dst, src) pairs");
  CHECK_DEV(inv); CHECK_CONTIG(inv); CHECK_DT(inv, at::kInt);
  CHECK_F32(valid);
  const int64_t L = inv.numel();
  TORCH_CHECK(valid.numel() == L, "ingest_scatter: valid must have one entry per padded row");
  std::vector<void*> d;
  std::vector<const void*> s;
  std::vector<int> rb;
  int64_t nsrc = INT32_MAX;
  for (size_t i = 0; i < dst.size(); ++i) {
    CHECK_DEV(dst[i]); CHECK_DEV(src[i]); CHECK_CONTIG(dst[i]); CHECK_CONTIG(src[i]);
    TORCH_CHECK(dst[i].scalar_type() == src[i].scalar_type(), "ingest_scatter: dtype mismatch at ", i);
    nsrc = std::min<int64_t>(nsrc, src[i].size(0));
    TORCH_CHECK(dst[i].dim() >= 1 && dst[i].size(0) == L, "ingest_scatter: dst ", i, " must have L rows");
    const int64_t row = dst[i].numel() / std::max<int64_t>(1, L) * dst[i].element_size();
    TORCH_CHECK(src[i].dim() >= 1 && src[i].numel() / std::max<int64_t>(1, src[i].size(0)) * src[i].element_size() == row,
                "ingest_scatter: row size mismatch at ", i);
    d.push_back(dst[i].data_ptr());
    s.push_back(src[i].data_ptr());
    rb.push_back((int)row);
  }
  // inv entries beyond the shortest source read nothing (the kernel zero-fills those rows): no out-of-range reads
  if (d.empty()) nsrc = 0;
  hip_check(dca_ingest_scatter(d.data(), s.data(), rb.data(), (int)d.size(), ptr<int>(inv), (int)L, (int)nsrc,
                               ptr<float>(valid), cur_stream()), "dca_ingest_scatter");
}

void adv_normalize(torch::Tensor adv, torch::Tensor valid, torch::Tensor out, double eps) {
  CHECK_F32(adv); CHECK_F32(valid); CHECK_F32(out);
  TORCH_CHECK(adv.numel() == valid.numel() && out.numel() == adv.numel(), "adv_normalize: size mismatch");
  hip_check(dca_adv_normalize(ptr<float>(adv), ptr<float>(valid), ptr<float>(out), (int)adv.numel(), (float)eps,
                              cur_stream()), "dca_adv_normalize");
}

void multi_copy(std::vector<torch::Tensor> dst, std::vector<torch::Tensor> src) {
  TORCH_CHECK(dst.size() == src.size(), "multi_copy: list length mismatch");
  TORCH_CHECK(dst.size() <= 64, "multi_copy: at most 64 tensors");
  std::vector<void*> d;
  std::vector<const void*> s;
  std::vector<long long> n;
  for (size_t i = 0; i < dst.size(); ++i) {
    CHECK_DEV(dst[i]); CHECK_DEV(src[i]); CHECK_CONTIG(dst[i]); CHECK_CONTIG(src[i]);
    TORCH_CHECK(dst[i].nbytes() == src[i].nbytes(), "multi_copy: byte size mismatch at ", i);
    d.push_back(dst[i].data_ptr());
    s.push_back(src[i].data_ptr());
    n.push_back((long long)dst[i].nbytes());
  }
  hip_check(dca_multi_copy(d.data(), s.data(), n.data(), (int)d.size(), cur_stream()), "dca_multi_copy");
}

void multi_axpy(std::vector<torch::Tensor> dst, std::vector<torch::Tensor> src, c10::optional<torch::Tensor> scale) {
  TORCH_CHECK(dst.size() == src.size(), "multi_axpy: list length mismatch");
  TORCH_CHECK(dst.size() <= 64, "multi_axpy: at most 64 tensors");
  std::vector<float*> d;
  std::vector<const float*> s;
  std::vector<long long> n;
  for (size_t i = 0; i < dst.size(); ++i) {
    CHECK_F32(dst[i]); CHECK_F32(src[i]);
    TORCH_CHECK(dst[i].numel() == src[i].numel(), "multi_axpy: numel mismatch at ", i);
    d.push_back(ptr<float>(dst[i]));
    s.push_back(ptr<float>(src[i]));
    n.push_back(dst[i].numel());
  }
  const float* sp = nullptr;
  if (scale.has_value() && scale->defined()) { CHECK_F32((*scale)); sp = ptr<float>(*scale); }
  hip_check(dca_multi_axpy(d.data(), s.data(), n.data(), (int)d.size(), sp, cur_stream()), "dca_multi_axpy");
}

// ------------------------------------------------------------------------------------------------------------
// Optional in-kernel timestamp buffers: checked contiguous int64 GPU tensors of at least `need` values (the kernels
// write without bounds checks). Team LSTM: 32 members × 4 waves × 64 steps × 8 events.
constexpr int64_t kTeamTraceElems = 32LL * 4 * 64 * 8;
inline unsigned long long* trace_ptr(const c10::optional<torch::Tensor>& t, int64_t need, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  CHECK_DEV(*t); CHECK_CONTIG(*t);
  TORCH_CHECK(t->scalar_type() == at::kLong && t->numel() >= need, name,
              ": trace must be a contiguous int64 GPU tensor with >= ", need, " elements");
  return ptr<unsigned long long>(*t);
}


// ------------------------------------------------------------------------------------------------------------
// XCD-team LSTM recurrence (lstm_team.hip). Gates in unit-major (·,·,H,4) layout; see the kernel header.
// whh bf16: bf16 MFMA, h exchanged in bf16 (hs bf16, optional f32 copy); whh fp32: the fp32-accurate variant
// (bf16x3 split MFMA, h exchanged in fp32; returns hs f32 in both hs slots).
// time_major=false: xp4 (B,S,H,4) and outputs (B,S,…); time_major=true: xp4 (S,B,H,4) and outputs (S,B,…) — a
// time chunk [t0,t1) of a time-major tensor is then a contiguous slice, which the pipelined learner step uses.
// Outputs may be passed in (e.g. slices of a whole-sequence tensor) to avoid copies.
namespace {
inline torch::Tensor out_or_new(const c10::optional<torch::Tensor>& o, at::IntArrayRef shape,
                                const at::TensorOptions& opt, const char* name) {
  if (o.has_value() && o->defined()) {
    TORCH_CHECK(o->is_cuda() && o->is_contiguous() && o->sizes() == shape && o->scalar_type() == opt.dtype(),
                name, ": preallocated output has the wrong shape/dtype/layout");
    return *o;
  }
  return torch::empty(shape, opt);
}
}  // namespace

// sequence-packing reset flags: (S, B) time-major or (B, S) u8, 1 where an episode starts (h, c := 0 before that step)
inline const unsigned char* reset_ptr(const c10::optional<torch::Tensor>& r, int B, int S) {
  if (!r.has_value() || !r->defined()) return nullptr;
  CHECK_DEV(*r); CHECK_CONTIG(*r);
  TORCH_CHECK(r->scalar_type() == at::kByte && r->numel() == (int64_t)B * S, "reset must be B*S uint8 flags");
  return r->data_ptr<unsigned char>();
}

inline void check_ctl(const torch::Tensor& ctl) {
  CHECK_DEV(ctl); CHECK_CONTIG(ctl);
  TORCH_CHECK(ctl.numel() * ctl.element_size() >= (int64_t)dca_lstm_team_ctl_bytes(),
              "team control block too small (use ops.lstm.team_ctl())");
}

std::vector<torch::Tensor> lstm_team_fwd(torch::Tensor xp4, torch::Tensor whh, torch::Tensor h0, torch::Tensor c0,
                                         torch::Tensor err, torch::Tensor ctl, bool want_f32_h,
                                         c10::optional<torch::Tensor> trace,
                                         bool time_major, c10::optional<torch::Tensor> hs_out,
                                         c10::optional<torch::Tensor> cs_out, c10::optional<torch::Tensor> gates_out,
                                         c10::optional<torch::Tensor> bias4, bool precise,
                                         c10::optional<torch::Tensor> reset) {
  CHECK_F32(xp4); CHECK_DEV(whh); CHECK_CONTIG(whh); CHECK_F32(h0); CHECK_F32(c0); CHECK_I32(err); check_ctl(ctl);
  const bool f32w = whh.scalar_type() == at::kFloat;
  TORCH_CHECK(f32w || whh.scalar_type() == at::kBFloat16, "whh must be bf16 or f32");
  TORCH_CHECK(xp4.dim() == 4 && xp4.size(3) == 4, "xp4 must be (B,S,H,4) or (S,B,H,4)");
  const int B = time_major ? xp4.size(1) : xp4.size(0), S = time_major ? xp4.size(0) : xp4.size(1);
  const int H = xp4.size(2);
  TORCH_CHECK(whh.size(0) == 4 * H && whh.size(1) == H, "whh must be (4H,H)");
  TORCH_CHECK(h0.size(0) == B && h0.size(1) == H && c0.size(0) == B && c0.size(1) == H, "h0/c0 must be (B,H)");
  TORCH_CHECK(H == 128 || H == 256 || H == 512, "lstm_team_fwd: H in {128,256,512}");
  auto f32 = xp4.options();
  const int64_t d0 = time_major ? S : B, d1 = time_major ? B : S;
  auto hs = out_or_new(hs_out, {d0, d1, H}, f32w ? f32 : f32.dtype(at::kBFloat16), "hs_out");
  torch::Tensor hsf = (want_f32_h && !f32w) ? torch::empty({d0, d1, H}, f32) : torch::Tensor();
  auto cs = out_or_new(cs_out, {d0, d1, H}, f32, "cs_out");
  auto gates4 = out_or_new(gates_out, {d0, d1, H, 4}, f32, "gates_out");
  auto hn = torch::empty({B, H}, f32);
  auto cn = torch::empty({B, H}, f32);
  const float* bias_p = nullptr;
  if (bias4.has_value() && bias4->defined()) {
    CHECK_F32((*bias4));
    TORCH_CHECK(bias4->numel() == 4 * H, "bias4 must hold 4H floats (unit-major)");
    bias_p = ptr<float>(*bias4);
  }
  const size_t wsb = dca_lstm_team_workspace(B, H, 0, f32w ? 1 : 0);
  auto ws = torch::empty({(int64_t)wsb}, f32.dtype(at::kByte));
  hip_check(dca_lstm_team_fwd(ptr<float>(xp4), whh.data_ptr(), ptr<float>(h0), ptr<float>(c0),
                              f32w ? nullptr : ptr<short>(hs),
                              f32w ? ptr<float>(hs) : (want_f32_h ? ptr<float>(hsf) : nullptr), ptr<float>(cs),
                              ptr<float>(gates4), ptr<float>(hn), ptr<float>(cn), ctl.data_ptr(), ws.data_ptr(), wsb,
                              ptr<unsigned>(err), B, S, H, time_major ? 1 : 0, cur_stream(),
                              trace_ptr(trace, kTeamTraceElems, "lstm_team_fwd"),
                              bias_p, f32w ? 1 : 0, precise ? 1 : 0, reset_ptr(reset, B, S)),
            "dca_lstm_team_fwd");
  if (f32w) return {hs, hs, cs, gates4, hn, cn};
  return {hs, want_f32_h ? hsf : hs, cs, gates4, hn, cn};
}

std::vector<torch::Tensor> lstm_team_bwd(torch::Tensor dhs, torch::Tensor gates4, torch::Tensor cs,
                                         torch::Tensor c0, c10::optional<torch::Tensor> dhn,
                                         c10::optional<torch::Tensor> dcn, torch::Tensor whh, torch::Tensor err,
                                         torch::Tensor ctl, c10::optional<torch::Tensor> trace, bool time_major,
                                         c10::optional<torch::Tensor> dg_out, bool dg_bf16, bool want_dbias,
                                         bool precise, c10::optional<torch::Tensor> reset) {
  CHECK_F32(dhs); CHECK_F32(gates4); CHECK_F32(cs); CHECK_F32(c0); CHECK_DEV(whh); CHECK_CONTIG(whh); CHECK_I32(err);
  check_ctl(ctl);
  const bool f32w = whh.scalar_type() == at::kFloat;
  TORCH_CHECK(f32w || whh.scalar_type() == at::kBFloat16, "whh must be bf16 or f32");
  TORCH_CHECK(!(f32w && dg_bf16), "lstm_team_bwd: the fp32 variant writes fp32 gate gradients");
  const int B = time_major ? dhs.size(1) : dhs.size(0), S = time_major ? dhs.size(0) : dhs.size(1);
  const int H = dhs.size(2);
  TORCH_CHECK(gates4.dim() == 4 && gates4.size(0) == dhs.size(0) && gates4.size(1) == dhs.size(1) &&
                  gates4.size(2) == H && gates4.size(3) == 4, "gates4 must match dhs with a trailing 4");
  TORCH_CHECK(cs.sizes() == dhs.sizes(), "cs must match dhs");
  TORCH_CHECK(c0.size(0) == B && c0.size(1) == H, "c0 must be (B,H)");
  TORCH_CHECK(whh.size(0) == 4 * H && whh.size(1) == H, "whh must be (4H,H)");
  TORCH_CHECK(H == 128 || H == 256 || H == 512, "lstm_team_bwd: H in {128,256,512}");
  const float* dhn_p = nullptr;
  const float* dcn_p = nullptr;
  if (dhn.has_value() && dhn->defined()) { CHECK_F32((*dhn)); dhn_p = ptr<float>(*dhn); }
  if (dcn.has_value() && dcn->defined()) { CHECK_F32((*dcn)); dcn_p = ptr<float>(*dcn); }
  auto f32 = dhs.options();
  // ∂gates in f32, or in bf16 (half the bytes; what the weight-gradient GEMMs consume)
  auto dgates4 = out_or_new(dg_out, {dhs.size(0), dhs.size(1), H, 4}, dg_bf16 ? f32.dtype(at::kBFloat16) : f32,
                            "dg_out");
  auto dh0 = torch::empty({B, H}, f32);
  auto dc0 = torch::empty({B, H}, f32);
  // per-chain bias-gradient partials (Σ over the chain's rows and steps), summed in chain order below
  torch::Tensor dbp = want_dbias ? torch::empty({dca_lstm_team_chains(B, f32w ? 1 : 0), 4 * H}, f32) : torch::Tensor();
  const size_t wsb = dca_lstm_team_workspace(B, H, 1, f32w ? 1 : 0);
  auto ws = torch::empty({(int64_t)wsb}, f32.dtype(at::kByte));
  hip_check(dca_lstm_team_bwd(ptr<float>(dhs), ptr<float>(gates4), ptr<float>(cs), ptr<float>(c0), dhn_p, dcn_p,
                              whh.data_ptr(), dg_bf16 ? nullptr : ptr<float>(dgates4), ptr<float>(dh0),
                              ptr<float>(dc0), ctl.data_ptr(), ws.data_ptr(), wsb, ptr<unsigned>(err), B, S, H,
                              time_major ? 1 : 0, cur_stream(),
                              trace_ptr(trace, kTeamTraceElems, "lstm_team_bwd"),
                              dg_bf16 ? ptr<short>(dgates4) : nullptr, want_dbias ? ptr<float>(dbp) : nullptr,
                              f32w ? 1 : 0, precise ? 1 : 0, reset_ptr(reset, B, S)),
            "dca_lstm_team_bwd");
  if (want_dbias) return {dgates4, dh0, dc0, dbp.sum(0)};
  return {dgates4, dh0, dc0};
}

// ------------------------------------------------------------------------------------------------------------
// Fused heads + loss. Returns (dz (N,ldz) f32 — bf16 with dz_bf16 —, dtl (N,U) f32, partials (nblk,16) f32, logp (N) f32).
std::vector<torch::Tensor> heads_loss(torch::Tensor z, torch::Tensor emb, torch::Tensor act, torch::Tensor msk,
                                      torch::Tensor adv, torch::Tensor ret, torch::Tensor logp_old,
                                      torch::Tensor nret, torch::Tensor norms, int64_t algo, bool compat_value_bug,
                                      int64_t S_bug, int64_t B_bug, double clip_eps, double ent_coef,
                                      double vf_coef, bool dz_bf16, bool precise) {
  CHECK_F32(z); CHECK_DEV(emb); CHECK_CONTIG(emb); CHECK_U8(act); CHECK_U8(msk); CHECK_F32(adv); CHECK_F32(ret);
  CHECK_F32(logp_old); CHECK_F32(nret); CHECK_F32(norms);
  const bool ef32 = emb.scalar_type() == at::kFloat;
  TORCH_CHECK(ef32 || emb.scalar_type() == at::kBFloat16, "emb must be bf16 or f32");
  TORCH_CHECK(z.dim() == 2 && emb.dim() == 3 && emb.size(2) == 128, "z (N,ldz), emb (N,U,128)");
  const int N = z.size(0), ldz = z.size(1), U = emb.size(1);
  TORCH_CHECK(emb.size(0) == N && act.size(0) == N && msk.size(0) == N, "row count mismatch");
  TORCH_CHECK(act.size(1) == 21 + U && msk.size(1) == 21 + U, "actions/masks must be (N, 21+U)");
  TORCH_CHECK(adv.numel() == N && ret.numel() == N && logp_old.numel() == N && nret.numel() == N, "per-row inputs");
  TORCH_CHECK(norms.numel() >= 8, "norms must hold 8 floats");
  TORCH_CHECK(ldz % 4 == 0 && ldz >= 150 && U <= 64, "ldz must be a multiple of 4 and >= 150; U <= 64");
  auto dz = dz_bf16 ? torch::empty_like(z, z.options().dtype(at::kBFloat16)) : torch::empty_like(z);
  auto dtl = torch::empty({N, U}, z.options());
  const int nb = dca_heads_loss_nblocks(N);
  auto part = torch::empty({nb, 16}, z.options());
  auto logp = torch::empty({N}, z.options());
  hip_check(dca_heads_loss(ptr<float>(z), ldz, emb.data_ptr(), ptr<unsigned char>(act), ptr<unsigned char>(msk),
                           21 + U, ptr<float>(adv), ptr<float>(ret), ptr<float>(logp_old), ptr<float>(nret),
                           ptr<float>(norms), dz_bf16 ? nullptr : ptr<float>(dz), ptr<float>(dtl), ptr<float>(part),
                           ptr<float>(logp), N, U, (int)algo, compat_value_bug ? 1 : 0, (int)S_bug, (int)B_bug,
                           (float)clip_eps, (float)ent_coef, (float)vf_coef, cur_stream(),
                           dz_bf16 ? ptr<short>(dz) : nullptr, ef32 ? 1 : 0, precise && ef32 ? 1 : 0),
            "dca_heads_loss");
  return {dz, dtl, part, logp};
}

// ------------------------------------------------------------------------------------------------------------
// Fused entity encoder. units (N,U,10) f32, env (N,3) f32, w1 (128,10), b1 (128), wt (6,128,128) bf16 or f32,
// bt (6,128), we (128,3), be (128); counts = 6 unit counts. Returns (x896 (N,896), emb (N,U,128), argmax u8
// (N,6,128)); x896 / emb have wt's dtype (f32: the fp32-accurate bf16x3 variant).
std::vector<torch::Tensor> encoder_fwd(torch::Tensor units, torch::Tensor env, torch::Tensor w1, torch::Tensor b1,
                                       torch::Tensor wt, torch::Tensor bt, torch::Tensor we, torch::Tensor be,
                                       std::vector<int64_t> counts, bool compat, bool exact,
                                       c10::optional<torch::Tensor> x896_out, c10::optional<torch::Tensor> emb_out,
                                       c10::optional<torch::Tensor> arg_out) {
  CHECK_F32(units); CHECK_F32(env); CHECK_F32(w1); CHECK_F32(b1); CHECK_DEV(wt); CHECK_CONTIG(wt); CHECK_F32(bt);
  CHECK_F32(we); CHECK_F32(be);
  const bool f32w = wt.scalar_type() == at::kFloat;
  TORCH_CHECK(f32w || wt.scalar_type() == at::kBFloat16, "wt must be bf16 or f32");
  TORCH_CHECK(!exact || f32w, "encoder_fwd: exact mode needs fp32 weights");
  TORCH_CHECK(units.dim() == 3 && units.size(2) == 10, "units must be (N,U,10)");
  const int N = units.size(0), U = units.size(1);
  TORCH_CHECK(env.size(0) == N && env.size(1) == 3, "env must be (N,3)");
  TORCH_CHECK(w1.size(0) == 128 && w1.size(1) == 10 && wt.size(0) == 6 && wt.size(1) == 128 && wt.size(2) == 128,
              "weight shapes");
  TORCH_CHECK(counts.size() == 6, "counts must have 6 entries");
  int c[6];
  int64_t tot = 0;
  for (int i = 0; i < 6; ++i) { c[i] = (int)counts[i]; tot += counts[i]; }
  TORCH_CHECK(tot == U && U <= 64, "counts must sum to U <= 64");
  auto o = units.options();
  const auto adt = f32w ? at::kFloat : at::kBFloat16;
  auto x896 = out_or_new(x896_out, {N, 896}, o.dtype(adt), "x896_out");
  auto emb = out_or_new(emb_out, {N, U, 128}, o.dtype(adt), "emb_out");
  auto arg = out_or_new(arg_out, {N, 6, 128}, o.dtype(at::kByte), "arg_out");
  hip_check(dca_encoder_fwd(ptr<float>(units), ptr<float>(env), ptr<float>(w1), ptr<float>(b1), wt.data_ptr(),
                            ptr<float>(bt), ptr<float>(we), ptr<float>(be), x896.data_ptr(), emb.data_ptr(),
                            ptr<unsigned char>(arg), N, U, c, compat ? 1 : 0, cur_stream(), exact ? 2 : (f32w ? 1 : 0)),
            "dca_encoder_fwd");
  return {x896, emb, arg};
}

// Returns (demb bf16 (U*N,128) type-major, basic bf16 (U*N,128) type-major, dw1 (128,10) f32, db1 (128) f32).
std::vector<torch::Tensor> encoder_bwd(torch::Tensor units, torch::Tensor w1, torch::Tensor b1, torch::Tensor wtT,
                                       torch::Tensor dtl, torch::Tensor q, torch::Tensor dx, torch::Tensor arg,
                                       std::vector<int64_t> counts, bool compat,
                                       c10::optional<torch::Tensor> demb_in, bool exact) {
  CHECK_F32(units); CHECK_F32(w1); CHECK_F32(b1); CHECK_DEV(wtT); CHECK_CONTIG(wtT); CHECK_F32(dtl); CHECK_F32(dx);
  CHECK_U8(arg); CHECK_DEV(q); CHECK_DT(q, at::kFloat);
  const bool f32w = wtT.scalar_type() == at::kFloat;
  TORCH_CHECK(f32w || wtT.scalar_type() == at::kBFloat16, "wtT must be bf16 or f32");
  TORCH_CHECK(!exact || f32w, "encoder_bwd: exact mode needs fp32 weights");
  const int N = units.size(0), U = units.size(1);
  TORCH_CHECK(q.dim() == 2 && q.size(0) == N && q.size(1) >= 128 && q.stride(1) == 1 && q.stride(0) % 4 == 0,
              "q must be (N, >=128) with unit column stride and 16-B aligned rows");
  TORCH_CHECK(dtl.size(0) == N && dtl.size(1) == U && dx.size(0) == N && dx.size(1) == 896, "dtl/dx shapes");
  TORCH_CHECK(arg.size(0) == N && arg.size(1) == 6 && arg.size(2) == 128, "arg shape");
  int c[6];
  int64_t tot = 0;
  for (int i = 0; i < 6; ++i) { c[i] = (int)counts[i]; tot += counts[i]; }
  TORCH_CHECK(tot == U && U <= 64, "counts must sum to U <= 64");
  auto o = units.options();
  auto dwt = torch::empty({6, 128, 128}, o);
  auto dw1 = torch::empty({128, 10}, o);
  auto db1 = torch::empty({128}, o);
  const size_t wsb = dca_encoder_bwd_workspace(N, U, c, f32w ? 1 : 0);
  auto ws = torch::empty({(int64_t)((wsb + 3) / 4)}, o);
  const void* dein = nullptr;
  if (demb_in && demb_in->defined()) {
    CHECK_DEV(*demb_in); CHECK_CONTIG(*demb_in);
    // the given ∂emb has the variant's activation dtype: bf16, or fp32 with fp32 weights (bf16x3 variant)
    TORCH_CHECK(demb_in->scalar_type() == (f32w ? at::kFloat : at::kBFloat16), "encoder_bwd: demb_in dtype");
    TORCH_CHECK(demb_in->numel() == (int64_t)N * U * 128, "demb_in must be (N, U, 128)");
    dein = demb_in->data_ptr();
  }
  hip_check(dca_encoder_bwd(ptr<float>(units), ptr<float>(w1), ptr<float>(b1), wtT.data_ptr(), ptr<float>(dtl),
                            ptr<float>(q), (int)q.stride(0), ptr<float>(dx), ptr<unsigned char>(arg), ptr<float>(dwt),
                            ptr<float>(dw1), ptr<float>(db1), ws.data_ptr(), wsb, N, U, c, compat ? 1 : 0,
                            cur_stream(), dein, exact ? 2 : (f32w ? 1 : 0)),
            "dca_encoder_bwd");
  return {dwt, dw1, db1};
}

// ------------------------------------------------------------------------------------------------------------
// Actor inference. Fused masked hierarchical sampling: z (N,ldz) f32 head logits [q|enum|x|y|v|pad], emb (N,U,128)
// bf16, handles (N,U) int64, ctr (1) int64 device step counter; writes idx (N,4) i32, act/msk (N,21+U) u8,
// logp (N) f32, value (N) f32 (all preallocated so the op is hipGraph-capturable).
void sample_actions(torch::Tensor z, torch::Tensor emb, torch::Tensor handles, int64_t seed, torch::Tensor ctr,
                    torch::Tensor idx, torch::Tensor act, torch::Tensor msk, torch::Tensor logp, torch::Tensor value) {
  CHECK_F32(z); CHECK_DEV(emb); CHECK_CONTIG(emb); CHECK_DEV(handles); CHECK_CONTIG(handles);
  const bool e32 = emb.scalar_type() == at::kFloat;
  TORCH_CHECK(e32 || emb.scalar_type() == at::kBFloat16, "sample_actions: emb bf16 or fp32");
  const bool h32 = handles.scalar_type() == at::kInt;
  TORCH_CHECK(h32 || handles.scalar_type() == at::kLong, "sample_actions: handles int64 or int32");
  CHECK_DEV(ctr); CHECK_DT(ctr, at::kLong); CHECK_I32(idx); CHECK_U8(act); CHECK_U8(msk); CHECK_F32(logp);
  CHECK_F32(value);
  TORCH_CHECK(z.dim() == 2 && emb.dim() == 3 && emb.size(2) == 128, "z (N,ldz), emb (N,U,128)");
  const int N = z.size(0), ldz = z.size(1), U = emb.size(1);
  TORCH_CHECK(emb.size(0) == N && handles.size(0) == N && handles.size(1) == U, "row/unit count mismatch");
  TORCH_CHECK(idx.size(0) == N && idx.size(1) == 4 && logp.numel() == N && value.numel() == N, "output shapes");
  TORCH_CHECK(act.size(0) == N && act.size(1) == 21 + U && msk.sizes() == act.sizes(), "act/msk (N,21+U)");
  TORCH_CHECK(U <= 64 && ldz >= 150, "U <= 64, ldz >= 150");
  hip_check(dca_sample_actions(ptr<float>(z), ldz, emb.data_ptr(), e32 ? 1 : 0, handles.data_ptr(), h32 ? 1 : 0, N,
                               U, (unsigned long long)seed, ptr<long long>(ctr), ptr<int>(idx),
                               ptr<unsigned char>(act), ptr<unsigned char>(msk), ptr<float>(logp), ptr<float>(value),
                               cur_stream()),
            "dca_sample_actions");
}

// Actor step staging: h, c *= keep (N) in place; xh (N, P + H) bf16 = [pre | bf16(h)] for the one-GEMM gates.
static long long* bump_ptr(const c10::optional<torch::Tensor>& bump) {   // optional (1) int64 device counter
  if (!bump || !bump->defined()) return nullptr;
  CHECK_DEV(*bump); CHECK_DT(*bump, at::kLong);
  TORCH_CHECK(bump->numel() >= 1, "bump: (1) int64 counter");
  return ptr<long long>(*bump);
}

void actor_state_prep(torch::Tensor pre, torch::Tensor h, torch::Tensor c, torch::Tensor keep, torch::Tensor xh,
                      c10::optional<torch::Tensor> bump) {
  CHECK_BF16(pre); CHECK_F32(h); CHECK_F32(c); CHECK_F32(keep); CHECK_BF16(xh);
  const int N = h.size(0), H = h.size(1), P = pre.size(1);
  TORCH_CHECK(pre.dim() == 2 && pre.size(0) == N && c.sizes() == h.sizes() && keep.numel() == N && xh.dim() == 2 &&
              xh.size(0) == N && xh.size(1) == P + H && H % 4 == 0 && P % 4 == 0, "actor_state_prep shapes");
  hip_check(dca_actor_state_prep(ptr<short>(pre), ptr<float>(h), ptr<float>(c), ptr<float>(keep), ptr<short>(xh), N, P,
                                 H, bump_ptr(bump), cur_stream()), "dca_actor_state_prep");
}

// LSTM cell from fp32 pre-activation gates (N,4H): updates h, c (N,H) f32 in place, writes h16 (N,H) bf16.
// Optional ``active`` (N) f32: rows with active == 0 keep their h / c / h16 (slots not stepped this call).
void lstm_cell(torch::Tensor gates, torch::Tensor h, torch::Tensor c, torch::Tensor h16,
               c10::optional<torch::Tensor> active) {
  CHECK_F32(gates); CHECK_F32(h); CHECK_F32(c); CHECK_BF16(h16);
  const int N = h.size(0), H = h.size(1);
  TORCH_CHECK(gates.size(0) == N && gates.size(1) == 4 * H && c.sizes() == h.sizes() && h16.sizes() == h.sizes(),
              "lstm_cell shapes");
  const float* act = nullptr;
  if (active && active->defined()) {
    CHECK_F32(*active);
    TORCH_CHECK(active->numel() == N, "lstm_cell: active must have one entry per row");
    act = ptr<float>(*active);
  }
  hip_check(dca_lstm_cell(ptr<float>(gates), ptr<float>(h), ptr<float>(c), ptr<short>(h16), act, N, H, cur_stream()),
            "dca_lstm_cell");
}

// fp8 actor policy core (actor_fp8.hip): x896 (n,896) bf16 → pre-RNN → gates + LSTM cell (h, c in place) → z (n,160).
// Weights are fragment-ordered e4m3fn bytes (uint8) with fp32 per-channel scales (actor/batched.py fp8_weight).
void actor_fp8(torch::Tensor x896, torch::Tensor wpre, torch::Tensor spre, torch::Tensor bpre, torch::Tensor wg,
               torch::Tensor sg, torch::Tensor bg, torch::Tensor wh, torch::Tensor sh, torch::Tensor bh,
               torch::Tensor h, torch::Tensor c, torch::Tensor keep, torch::Tensor z,
               c10::optional<torch::Tensor> active, c10::optional<torch::Tensor> bump) {
  CHECK_BF16(x896); CHECK_U8(wpre); CHECK_U8(wg); CHECK_U8(wh);
  CHECK_F32(spre); CHECK_F32(bpre); CHECK_F32(sg); CHECK_F32(bg); CHECK_F32(sh); CHECK_F32(bh);
  CHECK_F32(h); CHECK_F32(c); CHECK_F32(keep); CHECK_F32(z);
  const int n = x896.size(0);
  TORCH_CHECK(x896.dim() == 2 && x896.size(1) == 896, "actor_fp8: x896 (n, 896)");
  TORCH_CHECK(wpre.numel() == 256 * 896 && spre.numel() == 256 && bpre.numel() == 256, "actor_fp8: pre-RNN 256x896");
  TORCH_CHECK(wg.numel() == 2048 * 768 && sg.numel() == 2048 && bg.numel() == 2048, "actor_fp8: gates 2048x768");
  TORCH_CHECK(wh.numel() == 160 * 512 && sh.numel() == 160 && bh.numel() == 160, "actor_fp8: heads 160x512");
  TORCH_CHECK(h.dim() == 2 && h.size(0) == n && h.size(1) == 512 && c.sizes() == h.sizes() && keep.numel() == n,
              "actor_fp8: h, c (n, 512), keep (n)");
  TORCH_CHECK(z.dim() == 2 && z.size(0) == n && z.size(1) == 160, "actor_fp8: z (n, 160)");
  const float* act = nullptr;
  if (active && active->defined()) {
    CHECK_F32(*active);
    TORCH_CHECK(active->numel() == n, "actor_fp8: active (n)");
    act = ptr<float>(*active);
  }
  hip_check(dca_actor_fp8(ptr<short>(x896), wpre.data_ptr(), ptr<float>(spre), ptr<float>(bpre), wg.data_ptr(),
                          ptr<float>(sg), ptr<float>(bg), wh.data_ptr(), ptr<float>(sh), ptr<float>(bh), ptr<float>(h),
                          ptr<float>(c), ptr<float>(keep), act, ptr<float>(z), n, bump_ptr(bump), cur_stream()),
            "dca_actor_fp8");
}

// fp32 / bf16 actor policy core (actor_core.hip): x896 (n,896) f32 or bf16 → pre-RNN → LSTM step (h, c in place) or
// the linear fake_rnn layer → z (n,160). Weights in fragment order (actor/batched.py frag_weight): fp32 (mode 0, IEEE
// fp32 on the f32 MFMA) or bf16 (mode 1); wg = [W_ih | W_hh] rows in unit-major gate order (LSTM) or W_f (linear).
void actor_core(torch::Tensor x896, torch::Tensor wpre, torch::Tensor bpre, torch::Tensor wg, torch::Tensor bg,
                torch::Tensor wh, torch::Tensor bh, torch::Tensor h, torch::Tensor c, torch::Tensor keep,
                torch::Tensor z, int64_t mode, bool linear, c10::optional<torch::Tensor> active,
                c10::optional<torch::Tensor> bump) {
  CHECK_DEV(x896); CHECK_CONTIG(x896); CHECK_DEV(wpre); CHECK_CONTIG(wpre); CHECK_DEV(wg); CHECK_CONTIG(wg);
  CHECK_DEV(wh); CHECK_CONTIG(wh); CHECK_F32(bpre); CHECK_F32(bg); CHECK_F32(bh); CHECK_F32(h); CHECK_F32(c);
  CHECK_F32(keep); CHECK_F32(z);
  TORCH_CHECK(mode == 0 || mode == 1, "actor_core: mode 0 (fp32) or 1 (bf16)");
  const auto wdt = mode == 0 ? at::kFloat : at::kBFloat16;
  TORCH_CHECK(wpre.scalar_type() == wdt && wg.scalar_type() == wdt && wh.scalar_type() == wdt,
              "actor_core: weights must be fp32 (mode 0) or bf16 (mode 1)");
  const bool x32 = x896.scalar_type() == at::kFloat;
  TORCH_CHECK(x32 || (x896.scalar_type() == at::kBFloat16 && mode == 1), "actor_core: x896 fp32 (or bf16, mode 1)");
  const int n = x896.size(0), H = h.size(1);
  TORCH_CHECK(x896.dim() == 2 && x896.size(1) == 896, "actor_core: x896 (n, 896)");
  TORCH_CHECK(linear ? H == 256 : (H == 512 || H == 128), "actor_core: hidden 512 / 128 (LSTM) or 256 (linear)");
  const int64_t gn = linear ? H : 4 * H, gk = linear ? 256 : 256 + H;
  TORCH_CHECK(wpre.numel() == 256 * 896 && bpre.numel() == 256, "actor_core: pre-RNN 256x896");
  TORCH_CHECK(wg.numel() == gn * gk && bg.numel() == gn, "actor_core: recurrent weights");
  TORCH_CHECK(wh.numel() == 160 * H && bh.numel() == 160, "actor_core: heads 160 x hidden");
  TORCH_CHECK(h.dim() == 2 && h.size(0) == n && c.sizes() == h.sizes() && keep.numel() == n,
              "actor_core: h, c (n, hidden), keep (n)");
  TORCH_CHECK(z.dim() == 2 && z.size(0) == n && z.size(1) == 160, "actor_core: z (n, 160)");
  const float* act = nullptr;
  if (active && active->defined()) {
    CHECK_F32(*active);
    TORCH_CHECK(active->numel() == n, "actor_core: active (n)");
    act = ptr<float>(*active);
  }
  hip_check(dca_actor_core(x896.data_ptr(), x32 ? 1 : 0, wpre.data_ptr(), ptr<float>(bpre), wg.data_ptr(),
                           ptr<float>(bg), wh.data_ptr(), ptr<float>(bh), ptr<float>(h), ptr<float>(c),
                           ptr<float>(keep), act, ptr<float>(z), n, H, linear ? 1 : 0, (int)mode, bump_ptr(bump),
                           cur_stream()),
            "dca_actor_core");
}

// fp8 entity encoder of the actor step (actor_fp8.hip): units (N, U, 10) fp16 or fp32, env (N, 3) → x896 (N, 896) bf16
// (env embedding + pools) and emb (N, U, 128) bf16. W_τ: (6 × 128 × 128) e4m3 bytes in fragment order (fp8_weight per
// type) with per-channel scales st (6, 128); bt (6, 128).
std::vector<torch::Tensor> encoder_fp8(torch::Tensor units, torch::Tensor env, torch::Tensor w1, torch::Tensor b1,
                                       torch::Tensor wt, torch::Tensor st, torch::Tensor bt, torch::Tensor we,
                                       torch::Tensor be, std::vector<int64_t> counts, bool per_unit) {
  CHECK_DEV(units); CHECK_CONTIG(units); CHECK_F32(env); CHECK_F32(w1); CHECK_F32(b1); CHECK_U8(wt);
  CHECK_F32(st); CHECK_F32(bt); CHECK_F32(we); CHECK_F32(be);
  const bool f16 = units.scalar_type() == at::kHalf;
  TORCH_CHECK(f16 || units.scalar_type() == at::kFloat, "encoder_fp8: units fp16 or fp32");
  TORCH_CHECK(units.dim() == 3 && units.size(2) == 10, "encoder_fp8: units (N, U, 10)");
  const int N = units.size(0), U = units.size(1);
  TORCH_CHECK(env.dim() == 2 && env.size(0) == N && env.size(1) == 3, "encoder_fp8: env (N, 3)");
  TORCH_CHECK(w1.numel() == 128 * 10 && b1.numel() == 128 && we.numel() == 128 * 3 && be.numel() == 128,
              "encoder_fp8: W1 (128, 10), W_env (128, 3)");
  TORCH_CHECK(wt.numel() == 6 * 128 * 128 && st.numel() == 6 * 128 && bt.numel() == 6 * 128,
              "encoder_fp8: W_τ (6, 128, 128) e4m3, scales / biases (6, 128)");
  TORCH_CHECK(counts.size() == 6, "encoder_fp8: six unit counts");
  int c[6];
  int64_t tot = 0;
  for (int i = 0; i < 6; ++i) { c[i] = (int)counts[i]; tot += counts[i]; }
  TORCH_CHECK(tot == U && U <= 64, "encoder_fp8: counts must sum to U <= 64");
  auto o = env.options();
  auto x896 = torch::empty({N, 896}, o.dtype(at::kBFloat16));
  auto emb = torch::empty({N, U, 128}, o.dtype(at::kBFloat16));
  hip_check(dca_encoder_fp8(units.data_ptr(), f16 ? 1 : 0, ptr<float>(env), ptr<float>(w1), ptr<float>(b1),
                            wt.data_ptr(), ptr<float>(st), ptr<float>(bt), ptr<float>(we), ptr<float>(be),
                            ptr<short>(x896), ptr<short>(emb), N, U, c, per_unit ? 1 : 0, cur_stream()),
            "dca_encoder_fp8");
  return {x896, emb};
}

// Fused fp32 entity-attention block forward (attn_block.hip): e0 = E0' (N·64, 128) → xn, mean, rstd, qkv (no bias), o,
// lse, e1 (all for the backward / heads), and the pools into x896[:, 128:896] + arg (N, 6, 128). Weights: bf16 hi / lo
// images of W_qkv (384, 128) and W_out (128, 128) (split_bf16x2), bq (384).
std::vector<torch::Tensor> attn_block_fwd(torch::Tensor e0, torch::Tensor bout, torch::Tensor gamma, torch::Tensor beta,
                                          torch::Tensor wqh, torch::Tensor wql, torch::Tensor bq, torch::Tensor woh,
                                          torch::Tensor wol, std::vector<int64_t> type_off, torch::Tensor x896,
                                          torch::Tensor arg, bool compat, double eps) {
  CHECK_F32(e0); CHECK_F32(bout); CHECK_F32(gamma); CHECK_F32(beta); CHECK_F32(bq); CHECK_F32(x896); CHECK_U8(arg);
  // fp32 weight images (wql / wol ignored): the IEEE-fp32 kernel; bf16 hi / lo images: bf16x3
  const bool exact = wqh.scalar_type() == at::kFloat;
  CHECK_DEV(wqh); CHECK_CONTIG(wqh); CHECK_DEV(woh); CHECK_CONTIG(woh);
  if (exact) {
    CHECK_F32(woh);
  } else {
    CHECK_BF16(wqh); CHECK_BF16(wql); CHECK_BF16(woh); CHECK_BF16(wol);
  }
  TORCH_CHECK(e0.numel() % (64 * 128) == 0 && e0.size(-1) == 128, "attn_block_fwd: e0 (N·64, 128)");
  const int64_t N = e0.numel() / (64 * 128);
  TORCH_CHECK(wqh.numel() == 384 * 128 && (exact || wql.numel() == 384 * 128) && woh.numel() == 128 * 128 &&
              (exact || wol.numel() == 128 * 128) && bq.numel() == 384 && bout.numel() == 128 && gamma.numel() == 128 &&
              beta.numel() == 128, "attn_block_fwd: weight shapes");
  TORCH_CHECK(x896.dim() == 2 && x896.size(0) == N && x896.size(1) == 896, "attn_block_fwd: x896 (N, 896)");
  TORCH_CHECK(arg.numel() == N * 6 * 128, "attn_block_fwd: arg (N, 6, 128)");
  TORCH_CHECK(type_off.size() == 7 && type_off[0] == 0 && type_off[6] == 64, "attn_block_fwd: 7 type offsets 0 … 64");
  int off[7];
  for (int i = 0; i < 7; ++i) off[i] = (int)type_off[i];
  auto o32 = e0.options();
  auto xn = torch::empty({N * 64, 128}, o32);
  auto mu = torch::empty({N * 64}, o32);
  auto rs = torch::empty({N * 64}, o32);
  auto qkv = torch::empty({N * 64, 384}, o32);
  auto o = torch::empty({N * 64, 128}, o32);
  auto lse = torch::empty({N, 4, 64}, o32);
  auto e1 = torch::empty({N * 64, 128}, o32);
  hip_check(dca_attn_block_fwd_f32(ptr<float>(e0), ptr<float>(bout), ptr<float>(gamma), ptr<float>(beta),
                                   wqh.data_ptr(), exact ? nullptr : wql.data_ptr(), ptr<float>(bq), woh.data_ptr(),
                                   exact ? nullptr : wol.data_ptr(), ptr<float>(xn), ptr<float>(mu), ptr<float>(rs),
                                   ptr<float>(qkv), ptr<float>(o), ptr<float>(lse), ptr<float>(e1), ptr<float>(x896),
                                   ptr<unsigned char>(arg), off, compat ? 1 : 0, (int)N, (float)eps, cur_stream(),
                                   exact ? 1 : 0),
            "dca_attn_block_fwd_f32");
  return {xn, mu, rs, qkv, o, lse, e1};
}

static void check_type_off(const std::vector<int64_t>& t) {
  TORCH_CHECK(t.size() == 7 && t[0] == 0 && t[6] == 64, "type offsets must be 7 values from 0 to 64");
  for (int i = 0; i < 6; ++i) TORCH_CHECK(t[i + 1] >= t[i], "type offsets must be non-decreasing");
}

// Fused fp32 entity-attention block backward (attn_block.hip). q = the heads' z rows (row stride q.stride(0)), dx =
// ∂x896; o / qkv / lse / mu / rs from attn_block_fwd, e0 = E0' (N·64, 128); W_outᵀ images in 16x16x32 fragment
// order, W_qkv images in 16x16x16 B-fragment order (bf16 hi / lo). Returns (∂E1, ∂QKV (no bias), ∂E0,
// [∂γ | ∂β | ∂b_τ (6×128)] (1024)).
std::vector<torch::Tensor> attn_block_bwd(torch::Tensor dtl, torch::Tensor q, torch::Tensor dx, torch::Tensor arg,
                                          std::vector<int64_t> type_off, bool compat, torch::Tensor o,
                                          torch::Tensor qkv, torch::Tensor bq, torch::Tensor lse, torch::Tensor e0,
                                          torch::Tensor bout, torch::Tensor mu, torch::Tensor rs, torch::Tensor gamma,
                                          torch::Tensor woth, torch::Tensor wotl, torch::Tensor wq4h,
                                          torch::Tensor wq4l, c10::optional<torch::Tensor> trace) {
  CHECK_F32(dtl); CHECK_DEV(q); CHECK_DT(q, at::kFloat); CHECK_F32(dx); CHECK_U8(arg); CHECK_F32(o); CHECK_F32(qkv);
  CHECK_F32(bq); CHECK_F32(lse); CHECK_F32(e0); CHECK_F32(bout); CHECK_F32(mu); CHECK_F32(rs); CHECK_F32(gamma);
  const bool exact = woth.scalar_type() == at::kFloat;     // fp32 images: the IEEE-fp32 kernel
  CHECK_DEV(woth); CHECK_CONTIG(woth); CHECK_DEV(wq4h); CHECK_CONTIG(wq4h);
  if (exact) {
    CHECK_F32(wq4h);
  } else {
    CHECK_BF16(woth); CHECK_BF16(wotl); CHECK_BF16(wq4h); CHECK_BF16(wq4l);
  }
  check_type_off(type_off);
  const int64_t N = dtl.size(0);
  TORCH_CHECK(dtl.dim() == 2 && dtl.size(1) == 64, "attn_block_bwd: dtl (N, 64)");
  TORCH_CHECK(q.dim() == 2 && q.size(0) == N && q.size(1) >= 128 && q.stride(1) == 1, "attn_block_bwd: q (N, >=128)");
  TORCH_CHECK(dx.dim() == 2 && dx.size(0) == N && dx.size(1) == 896, "attn_block_bwd: dx (N, 896)");
  TORCH_CHECK(arg.numel() == N * 6 * 128, "attn_block_bwd: arg (N, 6, 128)");
  TORCH_CHECK(o.numel() == N * 64 * 128 && e0.numel() == N * 64 * 128 && qkv.numel() == N * 64 * 384 &&
              lse.numel() == N * 4 * 64 && mu.numel() == N * 64 && rs.numel() == N * 64, "attn_block_bwd: saved shapes");
  TORCH_CHECK(bq.numel() == 384 && bout.numel() == 128 && gamma.numel() == 128 && woth.numel() == 128 * 128 &&
              (exact || wotl.numel() == 128 * 128) && wq4h.numel() == 384 * 128 &&
              (exact || wq4l.numel() == 384 * 128), "attn_block_bwd: weight shapes");
  int off[7];
  for (int i = 0; i < 7; ++i) off[i] = (int)type_off[i];
  auto o32 = e0.options();
  auto de1 = torch::empty({N * 64, 128}, o32);
  auto dqkv = torch::empty({N * 64, 384}, o32);
  auto de0 = torch::empty({N * 64, 128}, o32);
  auto part = torch::empty({N, 1024}, o32);
  auto tmp = torch::empty({(int64_t)dca_attn_block_bwd_groups((int)N), 1024}, o32);
  auto sums = torch::empty({1024}, o32);
  if (trace.has_value() && trace->defined()) {
    // the kernel writes trace[(n·4 + w)·8 + ev] for rows n < 64 (4 waves, 8 events): 2048 u64 values
    CHECK_DEV(*trace); CHECK_CONTIG(*trace);
    TORCH_CHECK(trace->scalar_type() == at::kLong && trace->numel() >= 64 * 4 * 8,
                "attn_block_bwd: trace must be a contiguous int64 GPU tensor with >= 2048 elements");
  }
  hip_check(dca_attn_block_bwd_f32(ptr<float>(dtl), ptr<float>(q), (int)q.stride(0), ptr<float>(dx),
                                   ptr<unsigned char>(arg), off, compat ? 1 : 0, ptr<float>(o), ptr<float>(qkv),
                                   ptr<float>(bq), ptr<float>(lse), ptr<float>(e0), ptr<float>(bout), ptr<float>(mu),
                                   ptr<float>(rs), ptr<float>(gamma), woth.data_ptr(),
                                   exact ? nullptr : wotl.data_ptr(), wq4h.data_ptr(),
                                   exact ? nullptr : wq4l.data_ptr(), ptr<float>(de1), ptr<float>(dqkv),
                                   ptr<float>(de0), ptr<float>(part), ptr<float>(tmp), ptr<float>(sums), (int)N,
                                   cur_stream(),
                                   (trace.has_value() && trace->defined()) ? ptr<unsigned long long>(*trace) : nullptr,
                                   exact ? 1 : 0),
            "dca_attn_block_bwd_f32");
  return {de1, dqkv, de0, sums};
}


// Returns / advantages over concatenated padded rollouts. rew (L,K) f32 and val (L) f32 (GAE; ignored for mode 0)
// live on the GPU; the per-segment metadata is host data — off (nseg+1) i32 row offsets, seglen (nseg) i32 valid
// steps, keys (nseg) i32 team key, boot (nseg) f32 bootstrap values, done (nseg) u8 — validated here and uploaded in
// one copy. ema (n_keys,3) f32 [mean, std, initialised] is read and replaced by the state after this batch.
// mode 0 = discounted return + EMA normalisation (reference VPG), 1 = GAE(γ, λ). Writes ret/adv/norm (L) and
// stats (nseg,2) [mean, std of the returns].
void returns_scan(torch::Tensor rew, torch::Tensor val, torch::Tensor off, torch::Tensor seglen, torch::Tensor boot,
                  torch::Tensor done, torch::Tensor keys, torch::Tensor ema, torch::Tensor ret, torch::Tensor adv,
                  torch::Tensor norm, torch::Tensor stats, int64_t mode, bool normalize, double gamma, double lam,
                  double factor, double eps, c10::optional<torch::Tensor> lr, double rho_bar, double c_bar) {
  CHECK_F32(rew); CHECK_F32(ema); CHECK_F32(ret); CHECK_F32(adv); CHECK_F32(norm); CHECK_F32(stats);
  TORCH_CHECK(rew.dim() == 2, "rew must be (L, K)");
  const int64_t L = rew.size(0);
  const int nseg = seglen.numel();
  for (auto* t : {&off, &seglen, &keys, &boot, &done})
    TORCH_CHECK(!t->is_cuda() && t->is_contiguous(), "returns_scan: segment metadata must be contiguous host tensors");
  TORCH_CHECK(off.scalar_type() == at::kInt && seglen.scalar_type() == at::kInt && keys.scalar_type() == at::kInt &&
              boot.scalar_type() == at::kFloat && done.scalar_type() == at::kByte, "returns_scan: metadata dtypes");
  TORCH_CHECK(off.numel() == nseg + 1 && boot.numel() == nseg && done.numel() == nseg && keys.numel() == nseg,
              "returns_scan: per-segment tensor lengths");
  TORCH_CHECK(ret.numel() == L && adv.numel() == L && norm.numel() == L && stats.numel() == 2 * nseg,
              "returns_scan: output lengths");
  TORCH_CHECK(ema.dim() == 2 && ema.size(1) == 3, "ema must be (n_keys, 3)");
  TORCH_CHECK(mode == 0 || mode == 1 || mode == 2, "mode must be 0 (discount), 1 (gae) or 2 (v-trace gae)");
  TORCH_CHECK(rew.size(1) <= 64, "returns_scan: at most 64 sub-rewards");
  const float* vp = nullptr;
  const float* lp = nullptr;
  if (mode >= 1) {
    CHECK_F32(val);
    TORCH_CHECK(val.numel() == L, "returns_scan: values must have one entry per row");
    vp = ptr<float>(val);
  }
  if (mode == 2) {
    TORCH_CHECK(lr.has_value() && lr->defined(), "returns_scan: v-trace needs the per-row log ratios");
    CHECK_F32((*lr));
    TORCH_CHECK(lr->numel() == L, "returns_scan: log ratios must have one entry per row");
    lp = ptr<float>(*lr);
  }
  if (nseg == 0) return;
  const int* o = off.data_ptr<int>();
  const int* k = keys.data_ptr<int>();
  TORCH_CHECK(o[0] == 0 && o[nseg] == L, "returns_scan: offsets must span [0, L]");
  int max_len = 0;
  for (int i = 0; i < nseg; ++i) {
    TORCH_CHECK(o[i + 1] >= o[i], "returns_scan: decreasing offsets at segment ", i);
    TORCH_CHECK(k[i] >= 0 && k[i] < ema.size(0), "returns_scan: key out of range at segment ", i);
    max_len = std::max(max_len, o[i + 1] - o[i]);
  }
  // one upload of the packed metadata: [off | seglen | keys | boot | done] — from pinned memory, non-blocking. (A
  // pageable upload is a synchronous copy that waits for everything already queued on the stream: in the node loop's
  // look-ahead ingest that was the whole iteration's training steps, with the GIL held by this call, so the stager
  // and decode threads stalled behind it. The caching host allocator keeps the pinned block until the copy is done.)
  auto meta = torch::empty({(int64_t)(4 * nseg + 1 + (nseg + 3) / 4)}, torch::dtype(at::kInt).pinned_memory(true));
  int* mp = meta.data_ptr<int>();
  std::memcpy(mp, o, sizeof(int) * (nseg + 1));
  std::memcpy(mp + nseg + 1, seglen.data_ptr<int>(), sizeof(int) * nseg);
  std::memcpy(mp + 2 * nseg + 1, k, sizeof(int) * nseg);
  std::memcpy(mp + 3 * nseg + 1, boot.data_ptr<float>(), sizeof(float) * nseg);
  std::memcpy(mp + 4 * nseg + 1, done.data_ptr<uint8_t>(), nseg);
  auto md = meta.to(rew.device(), /*non_blocking=*/true);
  int* d = md.data_ptr<int>();
  auto ema_out = ema.clone();
  hip_check(dca_returns(ptr<float>(rew), (int)rew.size(1), vp, lp, d, d + nseg + 1,
                        reinterpret_cast<float*>(d + 3 * nseg + 1), reinterpret_cast<unsigned char*>(d + 4 * nseg + 1),
                        d + 2 * nseg + 1, nseg, max_len, ptr<float>(ret), ptr<float>(adv), ptr<float>(norm),
                        ptr<float>(stats), ptr<float>(ema), ptr<float>(ema_out), (int)mode, normalize ? 1 : 0,
                        (float)gamma, (float)lam, (float)rho_bar, (float)c_bar, (float)factor, (float)eps,
                        cur_stream()),
            "dca_returns");
  ema.copy_(ema_out);
}

// Loss normalisers from the one-hot action rows act (N,A) u8 → norms (8) f32. ws: int32 workspace of
// 5·loss_prep_blocks() + 1 elements whose last element (the arrival counter) must be zero before the first call
// (the kernel leaves it zero again, so the op is hipGraph-replayable).
void loss_prep(torch::Tensor act, torch::Tensor ws, torch::Tensor norms) {
  CHECK_U8(act); CHECK_I32(ws); CHECK_F32(norms);
  TORCH_CHECK(act.dim() == 2 && act.size(1) >= 22 && act.size(1) <= 128, "act must be (N, 21+U), U <= 107");
  const int nb = dca_loss_prep_blocks();
  TORCH_CHECK(ws.numel() >= 5 * nb + 1 && norms.numel() >= 8, "loss_prep: workspace / norms too small");
  int* w = ptr<int>(ws);
  hip_check(dca_loss_prep(ptr<unsigned char>(act), (int)act.size(0), (int)act.size(1), w,
                          reinterpret_cast<unsigned*>(w + 5 * nb), ptr<float>(norms), cur_stream()),
            "dca_loss_prep");
}

int64_t loss_prep_ws_elems() { return 5 * dca_loss_prep_blocks() + 1; }

// Loss scalar + metrics (out (16) f32) from the heads/loss partials part (R,16).
// V-trace inside the learner step (scan.hip vtrace_step_kernel): z (N, ldz) heads logits with the value in column
// vcol, lp / mu (N) the step's and the behaviour log-probs, vt (N, 4) {reward, bootstrap, valid, last}, time-major rows
// of B sequences × S steps. Returns (adv (N), ret (N), stats (B, 4) = Σ valid {ρ, truncated, mu − lp, 1}).
std::vector<torch::Tensor> vtrace_step(torch::Tensor z, int64_t vcol, torch::Tensor lp, torch::Tensor mu,
                                       torch::Tensor vt, int64_t B, int64_t S, double gamma, double lam,
                                       double rho_bar, double c_bar) {
  CHECK_DEV(z); CHECK_DT(z, at::kFloat); CHECK_F32(lp); CHECK_F32(mu); CHECK_F32(vt);
  const int64_t N = B * S;
  TORCH_CHECK(z.dim() == 2 && z.size(0) == N && z.stride(1) == 1 && vcol >= 0 && vcol < z.size(1),
              "vtrace_step: z (B·S, ldz) with the value column inside");
  TORCH_CHECK(lp.numel() == N && mu.numel() == N && vt.numel() == 4 * N, "vtrace_step: per-row inputs");
  auto adv = torch::empty({N}, z.options());
  auto ret = torch::empty({N}, z.options());
  auto stats = torch::empty({B, 4}, z.options());
  hip_check(dca_vtrace_step(ptr<float>(z), (int)z.stride(0), (int)vcol, ptr<float>(lp), ptr<float>(mu),
                            ptr<float>(vt), ptr<float>(adv), ptr<float>(ret), ptr<float>(stats), (int)B, (int)S,
                            (float)gamma, (float)lam, (float)rho_bar, (float)c_bar, cur_stream()),
            "dca_vtrace_step");
  return {adv, ret, stats};
}

// GPU unit featurization (featurize.hip): raw records (rows, U, 8) int32 + hero (rows, 4) fp32 → features (rows, U, 10)
// fp32 + handles (rows, U) int64, or fp16 + int32 (the fp8 actor's staged dtypes); handles optional
void featurize_raw(torch::Tensor raw, torch::Tensor hero, torch::Tensor units, c10::optional<torch::Tensor> handles) {
  CHECK_DEV(raw); CHECK_CONTIG(raw); CHECK_DT(raw, at::kInt);
  CHECK_F32(hero);
  CHECK_DEV(units); CHECK_CONTIG(units);
  TORCH_CHECK(raw.dim() == 3 && (raw.size(2) == 8 || raw.size(2) == 4),
              "featurize_raw: raw must be (rows, U, 8) int32, or (rows, U, 4) — the 16-byte records (fp16 out)");
  const int64_t rows = raw.size(0), U = raw.size(1);
  TORCH_CHECK(hero.numel() == rows * 4, "featurize_raw: hero must be (rows, 4)");
  TORCH_CHECK(units.numel() == rows * U * 10, "featurize_raw: units must be (rows, U, 10)");
  const bool half = units.scalar_type() == at::kHalf;
  TORCH_CHECK(half || units.scalar_type() == at::kFloat, "featurize_raw: units fp32 or fp16");
  void* hp = nullptr;
  if (handles.has_value() && handles->defined()) {
    CHECK_DEV(*handles); CHECK_CONTIG(*handles);
    TORCH_CHECK(handles->numel() == rows * U, "featurize_raw: handles must be (rows, U)");
    TORCH_CHECK(handles->scalar_type() == (half ? at::kInt : at::kLong),
                "featurize_raw: handles int64 with fp32 features, int32 with fp16");
    hp = handles->data_ptr();
  }
  TORCH_CHECK(rows * U < (int64_t)1 << 31, "featurize_raw: too many unit slots");
  if (raw.size(2) == 4) {
    TORCH_CHECK(half, "featurize_raw: 16-byte records featurize to fp16 (+ int32 handles)");
    hip_check(dca_featurize_raw16(raw.data_ptr(), ptr<float>(hero), units.data_ptr(), hp, (int)rows, (int)U,
                                  cur_stream()),
              "dca_featurize_raw16");
    return;
  }
  hip_check(dca_featurize_raw(raw.data_ptr(), ptr<float>(hero), units.data_ptr(), hp, (int)rows, (int)U, half ? 1 : 0,
                              cur_stream()),
            "dca_featurize_raw");
}

// Test utility (glue.hip): hold `blocks`·(1/8) CUs of XCD `xcd` for `seconds` on the current stream; returns the
// per-workgroup placement record (XCC id + 1 where it held a CU, 0 elsewhere).
torch::Tensor occupy_xcd(int64_t xcd, int64_t blocks, double seconds, torch::Tensor like) {
  TORCH_CHECK(xcd >= 0 && xcd < 8 && blocks >= 1 && blocks <= 4096 && seconds > 0.0 && seconds <= 10.0,
              "occupy_xcd: xcd in [0, 8), 1..4096 blocks, 0 < seconds <= 10");
  auto seen = torch::zeros({blocks}, like.options().dtype(at::kInt));
  hip_check(dca_occupy_xcd((int)xcd, (int)blocks, seconds, ptr<int>(seen), cur_stream()), "dca_occupy_xcd");
  return seen;
}

void loss_assemble(torch::Tensor part, torch::Tensor norms, int64_t N, int64_t algo, double ent_coef, double vf_coef,
                   torch::Tensor out, int64_t S, bool compat_value_bug) {
  CHECK_F32(part); CHECK_F32(norms); CHECK_F32(out);
  TORCH_CHECK(part.dim() == 2 && part.size(1) == 16 && out.numel() >= 16 && norms.numel() >= 8,
              "loss_assemble shapes");
  hip_check(dca_loss_assemble(ptr<float>(part), (int)part.size(0), ptr<float>(norms), (int)N, (int)algo,
                              (float)ent_coef, (float)vf_coef, ptr<float>(out), (int)S, compat_value_bug ? 1 : 0,
                              cur_stream()),
            "dca_loss_assemble");
}

// Working copies of the weights: dst16[i] = bf16(src[map16[i]]) (0 where map16 < 0),
// dst32[i] = src[map32[i,0]] + src[map32[i,1]] (negative index = 0 term).
void weight_prep(torch::Tensor src, torch::Tensor map16, torch::Tensor dst16, torch::Tensor map32,
                 torch::Tensor dst32, c10::optional<torch::Tensor> maps, c10::optional<torch::Tensor> dsth,
                 c10::optional<torch::Tensor> dstl) {
  CHECK_F32(src); CHECK_I32(map16); CHECK_BF16(dst16); CHECK_I32(map32); CHECK_F32(dst32);
  TORCH_CHECK(map16.numel() == dst16.numel() && map32.numel() == 2 * dst32.numel(), "weight_prep: map sizes");
  const int* ms = nullptr;
  short *dh = nullptr, *dl = nullptr;
  int ns = 0;
  if (maps && maps->defined()) {
    TORCH_CHECK(dsth && dsth->defined() && dstl && dstl->defined(), "weight_prep: split map needs both hi / lo outputs");
    CHECK_I32(*maps); CHECK_BF16(*dsth); CHECK_BF16(*dstl);
    TORCH_CHECK(maps->numel() == dsth->numel() && dstl->numel() == dsth->numel(), "weight_prep: split map sizes");
    ms = ptr<int>(*maps); dh = ptr<short>(*dsth); dl = ptr<short>(*dstl); ns = (int)maps->numel();
  }
  hip_check(dca_weight_prep(ptr<float>(src), ptr<int>(map16), ptr<short>(dst16), (int)dst16.numel(), ptr<int>(map32),
                            ptr<float>(dst32), (int)dst32.numel(), ms, dh, dl, ns, cur_stream()),
            "dca_weight_prep");
}

// C (+)= Aᵀ·B for K-outer operands (split-K MFMA, ops/csrc/gemm_tn.hip). A (K,M) and B (K-split_rows,N) are
// row-major with unit column stride (any row stride), both bf16 or both fp32 (fp32: bf16x3 split MFMA, ≈fp32
// accuracy); optional B0 (split_rows,N) supplies rows k < split_rows of the B operand. C (M',N) f32 with unit column
// stride; optional perm (M) i32 maps result row m → C row perm[m].
void gemm_tn(torch::Tensor A, torch::Tensor B, torch::Tensor C, c10::optional<torch::Tensor> perm, bool accumulate,
             c10::optional<torch::Tensor> B0, c10::optional<torch::Tensor> colsum, bool exact) {
  CHECK_DEV(A); CHECK_DEV(B); CHECK_DEV(C);
  const bool f32 = A.scalar_type() == at::kFloat;
  TORCH_CHECK((A.scalar_type() == at::kBFloat16 || f32) && B.scalar_type() == A.scalar_type() &&
                  C.scalar_type() == at::kFloat, "gemm_tn: A, B both bf16 or both f32; C f32");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2 && A.stride(1) == 1 && B.stride(1) == 1 &&
              C.stride(1) == 1, "gemm_tn: 2-D operands with unit column stride");
  const int K = A.size(0), M = A.size(1), N = B.size(1);
  int split_rows = 0;
  const void* b0 = nullptr;
  if (B0 && B0->defined()) {
    CHECK_DEV(*B0);
    TORCH_CHECK(B0->scalar_type() == A.scalar_type() && B0->dim() == 2 && B0->size(1) == N && B0->stride(1) == 1 &&
                B0->stride(0) == B.stride(0), "gemm_tn: B0 must match B's dtype, columns and row stride");
    split_rows = B0->size(0);
    b0 = B0->data_ptr();
  }
  TORCH_CHECK(B.size(0) + split_rows == K, "gemm_tn: K mismatch between A and [B0; B]");
  const int al = f32 ? 4 : 8;   // elements per 16-B load
  TORCH_CHECK(M % 8 == 0 && N % 8 == 0 && A.stride(0) % al == 0 && B.stride(0) % al == 0,
              "gemm_tn: M, N multiples of 8 and row strides 16-B aligned");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(A.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(B.data_ptr()) & 15) == 0 &&
              (b0 == nullptr || (reinterpret_cast<uintptr_t>(b0) & 15) == 0), "gemm_tn: operands must be 16-B aligned");
  const int* pp = nullptr;
  int64_t crow = M;
  if (perm && perm->defined()) {
    CHECK_I32(*perm);
    TORCH_CHECK(perm->numel() == M, "gemm_tn: perm must have M entries");
    pp = ptr<int>(*perm);
    crow = C.size(0);
  }
  TORCH_CHECK(C.size(0) >= crow && C.size(1) == N, "gemm_tn: C shape");
  float* csp = nullptr;
  if (colsum && colsum->defined()) {
    CHECK_F32(*colsum);
    TORCH_CHECK(colsum->numel() >= crow, "gemm_tn: colsum must have one entry per C row");
    csp = ptr<float>(*colsum);
  }
  if (K == 0) {
    if (!accumulate) {
      C.zero_();
      if (csp) colsum->zero_();
    }
    return;
  }
  int splits, kc, tiles;
  TORCH_CHECK(!exact || f32, "gemm_tn: exact mode needs fp32 operands");
  const int mode = exact ? 2 : (f32 ? 1 : 0);
  dca_gemm_tn_plan(M, N, K, &splits, &kc, &tiles, mode);
  torch::Tensor slab;
  if (splits > 1) slab = torch::empty({(int64_t)splits * M * N + (csp ? (int64_t)splits * M : 0)}, C.options());
  hip_check(dca_gemm_tn(A.data_ptr(), (int)A.stride(0), B.data_ptr(), (int)B.stride(0), b0, split_rows,
                        ptr<float>(C), (int)C.stride(0), pp, accumulate ? 1 : 0, M, N, K,
                        splits > 1 ? ptr<float>(slab) : nullptr, csp, cur_stream(), mode),
            "dca_gemm_tn");
}

// Entity-encoder small gradients in one pass: returns (dbt (6,128), dWe (128,3), dbe (128)). z (N,ldz) f32 with the
// pointer query in columns 0..127, dtl (N,U) f32, type_off (7) i32 device unit-slot offsets per type, dx (N,896) f32
// (∂ of the encoder output x896), env (N,3) f32, we (128,3), be (128) f32.
std::vector<torch::Tensor> enc_small_grads(torch::Tensor z, torch::Tensor dtl, torch::Tensor type_off, torch::Tensor dx,
                                           torch::Tensor env, torch::Tensor we, torch::Tensor be, bool compat) {
  CHECK_DEV(z); CHECK_DT(z, at::kFloat); TORCH_CHECK(z.stride(1) == 1 && z.size(1) >= 128, "z (N, ldz>=128)");
  CHECK_F32(dtl); CHECK_I32(type_off); CHECK_F32(dx); CHECK_F32(env); CHECK_F32(we); CHECK_F32(be);
  const int N = z.size(0), U = dtl.size(1);
  TORCH_CHECK(dtl.size(0) == N && dx.size(0) == N && dx.size(1) == 896 && env.size(0) == N && env.size(1) == 3 &&
              we.size(0) == 128 && we.size(1) == 3 && be.numel() == 128 && type_off.numel() == 7,
              "enc_small_grads shapes");
  auto o = z.options();
  auto part = torch::empty({(int64_t)dca_enc_small_blocks() * dca_enc_small_out()}, o);
  auto out = torch::empty({(int64_t)dca_enc_small_out()}, o);
  hip_check(dca_enc_small_grads(ptr<float>(z), (int)z.stride(0), ptr<float>(dtl), U, ptr<int>(type_off),
                                ptr<float>(dx), ptr<float>(env), ptr<float>(we), ptr<float>(be), N, compat ? 1 : 0,
                                ptr<float>(part), ptr<float>(out), cur_stream()),
            "dca_enc_small_grads");
  return {out.narrow(0, 0, 768).view({6, 128}), out.narrow(0, 768, 384).view({128, 3}), out.narrow(0, 1152, 128)};
}

// fp32 → (hi, lo) bf16 images, x = hi + lo (the bf16x3 operand split, done once per step for a weight image)
std::vector<torch::Tensor> split_bf16x2(torch::Tensor src, bool slab_major) {
  CHECK_F32(src);
  TORCH_CHECK(src.numel() % 4 == 0, "split_bf16x2: numel % 4 == 0");
  if (slab_major) {
    TORCH_CHECK(src.dim() == 2 && src.size(1) % 32 == 0, "split_bf16x2: slab-major images need (R, K), K % 32 == 0");
    const int R = src.size(0), K = src.size(1);
    auto hi = torch::empty({K / 32, R, 32}, src.options().dtype(at::kBFloat16));
    auto lo = torch::empty({K / 32, R, 32}, src.options().dtype(at::kBFloat16));
    hip_check(dca_split_bf16x2_blk(ptr<float>(src), ptr<short>(hi), ptr<short>(lo), R, K, cur_stream()),
              "dca_split_bf16x2_blk");
    return {hi, lo};
  }
  auto hi = torch::empty(src.sizes(), src.options().dtype(at::kBFloat16));
  auto lo = torch::empty(src.sizes(), src.options().dtype(at::kBFloat16));
  hip_check(dca_split_bf16x2(ptr<float>(src), ptr<short>(hi), ptr<short>(lo), src.numel(), cur_stream()),
            "dca_split_bf16x2");
  return {hi, lo};
}

// Fused ∂X chain of the fp32 pre-RNN layer (ops/csrc/dx_chain.hip): dpre = (dG · W_ih) ⊙ [x > 0], dx = dpre · W_pre.
// dG (N, K1) f32, x (N, 256) f32 ReLU outputs; weights K-contiguous per output column: w1 = W_ihᵀ image (256, K1),
// w2 = W_preᵀ image (X, 256) — bf16 hi / lo images (bf16x3), or fp32 with w1l / w2l empty (exact).
// Returns (dpre (N, 256), dx (N, X)).
std::vector<torch::Tensor> dpre_dx(torch::Tensor dG, torch::Tensor w1h, torch::Tensor w1l, torch::Tensor x,
                                   torch::Tensor w2h, torch::Tensor w2l) {
  CHECK_F32(dG); CHECK_F32(x); CHECK_DEV(w1h); CHECK_CONTIG(w1h); CHECK_DEV(w2h); CHECK_CONTIG(w2h);
  const bool exact = w1h.scalar_type() == at::kFloat;
  if (exact) {
    TORCH_CHECK(w2h.scalar_type() == at::kFloat, "dpre_dx: both weights fp32 (exact) or bf16 hi/lo pairs");
  } else {
    CHECK_DT(w1h, at::kBFloat16); CHECK_DT(w2h, at::kBFloat16); CHECK_DEV(w1l); CHECK_CONTIG(w1l);
    CHECK_DEV(w2l); CHECK_CONTIG(w2l); CHECK_DT(w1l, at::kBFloat16); CHECK_DT(w2l, at::kBFloat16);
    TORCH_CHECK(w1l.sizes() == w1h.sizes() && w2l.sizes() == w2h.sizes(), "dpre_dx: hi / lo image shapes");
  }
  const int N = dG.size(0), K1 = dG.size(1);
  TORCH_CHECK(dG.dim() == 2 && x.dim() == 2, "dpre_dx: 2-D dG and x");
  int X;
  if (exact) {
    TORCH_CHECK(w1h.dim() == 2 && w2h.dim() == 2, "dpre_dx: exact weights (256,K1) (X,256)");
    X = w2h.size(0);
    TORCH_CHECK(w1h.size(0) == 256 && w1h.size(1) == K1 && w2h.size(1) == 256, "dpre_dx: shapes (256,K1) (X,256)");
  } else {
    // slab-major images (split_bf16x2(..., slab_major=True)): (K1/32, 256, 32) and (256/32, X, 32)
    TORCH_CHECK(w1h.dim() == 3 && w2h.dim() == 3 && w1h.size(0) * 32 == K1 && w1h.size(1) == 256 &&
                w1h.size(2) == 32 && w2h.size(0) == 8 && w2h.size(2) == 32,
                "dpre_dx: bf16x3 weights are slab-major images (K1/32,256,32) and (8,X,32)");
    X = w2h.size(1);
  }
  TORCH_CHECK(x.size(0) == N && x.size(1) == 256, "dpre_dx: x (N,256)");
  TORCH_CHECK(K1 % 128 == 0 && X % 128 == 0, "dpre_dx: K1 % 128 == 0 and X % 128 == 0");
  TORCH_CHECK((long long)N * K1 * 4 <= 0x7fff0000LL, "dpre_dx: dG too large for one launch");
  auto o = dG.options();
  auto dpre = torch::empty({N, 256}, o);
  auto dx = torch::empty({N, X}, o);
  hip_check(dca_dpre_dx(ptr<float>(dG), w1h.data_ptr(), exact ? nullptr : w1l.data_ptr(), ptr<float>(x),
                        w2h.data_ptr(), exact ? nullptr : w2l.data_ptr(), ptr<float>(dpre), ptr<float>(dx), N, K1, X,
                        exact ? 1 : 0, 0, cur_stream()),
            "dca_dpre_dx");
  return {dpre, dx};
}

// The chain kernel's stages alone (dx_chain.hip). bf16x3: slab-major bf16 hi / lo weight images; exact (IEEE fp32
// products, v_mfma_f32_16x16x4_f32): the fp32 weight itself with wl empty.
// rowmm_out256: C (N, 256) = A (N, K) · Wᵀ + b with W (256, K) → images (K/32, 256, 32) — stage 1, bias epilogue;
// rowmm_in256:  C (N, X) = A (N, 256) · Wᵀ with W (X, 256) → images (8, X, 32) — stage 2 on A read from HBM.
// The 1v1 heads GEMM (W_cat zero-padded to 256 rows) and its ∂X product.
static bool chain_exact(const torch::Tensor& wh, const torch::Tensor& wl, const char* what) {
  CHECK_DEV(wh); CHECK_CONTIG(wh);
  if (wh.scalar_type() == at::kFloat) {
    TORCH_CHECK(wh.dim() == 2 && wl.numel() == 0, what, ": exact weights are 2-D fp32 with an empty lo image");
    return true;
  }
  CHECK_BF16(wh); CHECK_BF16(wl);
  TORCH_CHECK(wl.sizes() == wh.sizes(), what, ": hi / lo image shapes");
  return false;
}

torch::Tensor rowmm_out256(torch::Tensor A, torch::Tensor wh, torch::Tensor wl, torch::Tensor bias) {
  CHECK_F32(A); CHECK_F32(bias);
  const bool exact = chain_exact(wh, wl, "rowmm_out256");
  const int N = A.size(0), K = A.size(1);
  TORCH_CHECK(A.dim() == 2 && K % 128 == 0 && bias.numel() == 256, "rowmm_out256: A (N, K % 128 == 0), bias (256)");
  if (exact) {
    TORCH_CHECK(wh.size(0) == 256 && wh.size(1) == K, "rowmm_out256: exact W (256, K)");
  } else {
    TORCH_CHECK(wh.dim() == 3 && wh.size(0) * 32 == K && wh.size(1) == 256 && wh.size(2) == 32,
                "rowmm_out256: slab-major images (K/32, 256, 32)");
  }
  TORCH_CHECK((long long)N * K * 4 <= 0x7fff0000LL, "rowmm_out256: A too large for one launch");
  auto out = torch::empty({N, 256}, A.options());
  hip_check(dca_dpre_dx(ptr<float>(A), wh.data_ptr(), exact ? nullptr : wl.data_ptr(), ptr<float>(bias), nullptr,
                        nullptr, ptr<float>(out), nullptr, N, K, 0, exact ? 1 : 0, 2, cur_stream()),
            "dca_dpre_dx(stage 1)");
  return out;
}

torch::Tensor rowmm_in256(torch::Tensor A, torch::Tensor wh, torch::Tensor wl) {
  CHECK_F32(A);
  const bool exact = chain_exact(wh, wl, "rowmm_in256");
  const int N = A.size(0);
  TORCH_CHECK(A.dim() == 2 && A.size(1) == 256, "rowmm_in256: A (N, 256)");
  int X;
  if (exact) {
    TORCH_CHECK(wh.size(1) == 256 && wh.size(0) % 128 == 0, "rowmm_in256: exact W (X, 256), X % 128 == 0");
    X = wh.size(0);
  } else {
    TORCH_CHECK(wh.dim() == 3 && wh.size(0) == 8 && wh.size(2) == 32 && wh.size(1) % 128 == 0,
                "rowmm_in256: slab-major images (8, X, 32), X % 128 == 0");
    X = wh.size(1);
  }
  auto out = torch::empty({N, X}, A.options());
  hip_check(dca_dpre_dx(ptr<float>(A), nullptr, nullptr, nullptr, wh.data_ptr(), exact ? nullptr : wl.data_ptr(),
                        nullptr, ptr<float>(out), N, 0, X, exact ? 1 : 0, 0, cur_stream()),
            "dca_dpre_dx(stage 2)");
  return out;
}

// The forward twin of dpre_dx (same kernel, bias + ReLU epilogue): x = relu(x896·W_preᵀ + b) (N, 256) and
// xp = x·W_ihᵀ (N, X) in one launch. bf16x3: slab-major hi / lo weight images (split_bf16x2(w, True) of W_pre
// (256, K1) and of W_ih (X, 256)); exact: W_pre (256, K1) and W_ih (X, 256) fp32 with empty lo images.
std::vector<torch::Tensor> pre_rnn_chain(torch::Tensor x896, torch::Tensor w1h, torch::Tensor w1l, torch::Tensor bias,
                                         torch::Tensor w2h, torch::Tensor w2l, c10::optional<torch::Tensor> x_out,
                                         c10::optional<torch::Tensor> xp_out) {
  CHECK_F32(x896); CHECK_F32(bias);
  const bool exact = chain_exact(w1h, w1l, "pre_rnn_chain");
  TORCH_CHECK(chain_exact(w2h, w2l, "pre_rnn_chain") == exact, "pre_rnn_chain: both weights exact or both bf16x3");
  const int N = x896.size(0), K1 = x896.size(1);
  TORCH_CHECK(x896.dim() == 2 && bias.numel() == 256, "pre_rnn_chain: x896 (N, K1), bias (256)");
  int X;
  if (exact) {
    TORCH_CHECK(w1h.size(0) == 256 && w1h.size(1) == K1 && w2h.size(1) == 256, "pre_rnn_chain: exact W_pre (256, K1), "
                "W_ih (X, 256)");
    X = w2h.size(0);
  } else {
    TORCH_CHECK(w1h.dim() == 3 && w1h.size(0) * 32 == K1 && w1h.size(1) == 256 && w1h.size(2) == 32 &&
                w2h.dim() == 3 && w2h.size(0) == 8 && w2h.size(2) == 32,
                "pre_rnn_chain: slab-major images (K1/32,256,32) and (8,X,32)");
    X = w2h.size(1);
  }
  TORCH_CHECK(K1 % 128 == 0 && X % 128 == 0, "pre_rnn_chain: K1 % 128 == 0 and X % 128 == 0");
  TORCH_CHECK((long long)N * K1 * 4 <= 0x7fff0000LL, "pre_rnn_chain: x896 too large for one launch");
  auto o = x896.options();
  auto x = out_or_new(x_out, {N, 256}, o, "x_out");
  auto xp = out_or_new(xp_out, {N, X}, o, "xp_out");
  hip_check(dca_dpre_dx(ptr<float>(x896), w1h.data_ptr(), exact ? nullptr : w1l.data_ptr(), ptr<float>(bias),
                        w2h.data_ptr(), exact ? nullptr : w2l.data_ptr(), ptr<float>(x), ptr<float>(xp), N, K1, X,
                        exact ? 1 : 0, 1, cur_stream()),
            "dca_dpre_dx(forward)");
  return {x, xp};
}


// Minibatch gather from an HBM replay pool into time-major rows (one launch for all fields). pools: per-step
// fields (capacity, S, …) then per-sequence fields (capacity, …) (n_step of them are per-step); idx (B) int64 device.
// Returns the gathered tensors: per-step fields as (S·B, …), per-sequence fields as (B, …).
std::vector<torch::Tensor> replay_gather(std::vector<torch::Tensor> pools, int64_t n_step, torch::Tensor idx) {
  CHECK_DEV(idx); CHECK_CONTIG(idx); CHECK_DT(idx, at::kLong);
  TORCH_CHECK(!pools.empty() && pools.size() <= 12, "replay_gather: 1..12 fields");
  const int B = idx.numel();
  const int S = n_step > 0 ? pools[0].size(1) : 1;
  std::vector<torch::Tensor> out;
  std::vector<const void*> src;
  std::vector<void*> dst;
  std::vector<long long> rb;
  std::vector<int> ps;
  for (size_t i = 0; i < pools.size(); ++i) {
    const torch::Tensor& p = pools[i];
    CHECK_DEV(p); CHECK_CONTIG(p);
    const bool step = (int64_t)i < n_step;
    TORCH_CHECK(!step || (p.dim() >= 2 && p.size(1) == S), "replay_gather: per-step pools must be (capacity, S, ...)");
    std::vector<int64_t> shape;
    if (step) {
      shape.push_back((int64_t)S * B);
      for (int d = 2; d < p.dim(); ++d) shape.push_back(p.size(d));
    } else {
      shape.push_back(B);
      for (int d = 1; d < p.dim(); ++d) shape.push_back(p.size(d));
    }
    auto o = torch::empty(shape, p.options());
    const int64_t per = step ? p.numel() / (p.size(0) * S) : p.numel() / p.size(0);
    src.push_back(p.data_ptr());
    dst.push_back(o.data_ptr());
    rb.push_back((long long)(per * p.element_size()));
    ps.push_back(step ? 1 : 0);
    out.push_back(o);
  }
  hip_check(dca_replay_gather(src.data(), dst.data(), rb.data(), ps.data(), (int)pools.size(), ptr<long long>(idx), S,
                              B, cur_stream()),
            "dca_replay_gather");
  return out;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "dotaclient_amd gfx950 HIP kernels";
  m.def("adam_step", &adam_step, "fused global-norm clip + Adam over a flat fp32 buffer (divide: grad holds DP sums, "
        "averaged by the has-grad counts in-kernel)", py::arg("param"), py::arg("grad"), py::arg("m"), py::arg("v"),
        py::arg("seg"), py::arg("counts"), py::arg("steps"), py::arg("norm_out"), py::arg("lr"), py::arg("b1"),
        py::arg("b2"), py::arg("eps"), py::arg("max_norm"), py::arg("divide") = false, py::arg("header") = 0,
        py::arg("skip") = py::none(), py::arg("nonfinite") = py::none());
  m.def("ingest_scatter", &ingest_scatter, "packed valid rows -> zero-padded rows of every field + validity mask");
  m.def("adv_normalize", &adv_normalize, "PPO advantage normalisation over the valid rows (one workgroup)");
  m.def("multi_copy", &multi_copy, "dst_i <- src_i (same byte sizes, contiguous, 16-B aligned) in one launch");
  m.def("multi_axpy", &multi_axpy, "dst_i += scale * src_i for a list of fp32 tensors (one graph-safe launch)",
        py::arg("dst"), py::arg("src"), py::arg("scale") = py::none());
  m.def("lstm_team_ctl_bytes", &dca_lstm_team_ctl_bytes, "bytes of a persistent team-LSTM control block");
  m.def("heads_loss", &heads_loss, "fused heads + pointer + masked log-softmax + PPO/VPG loss + gradients",
        py::arg("z"), py::arg("emb"), py::arg("act"), py::arg("msk"), py::arg("adv"), py::arg("ret"),
        py::arg("logp_old"), py::arg("nret"), py::arg("norms"), py::arg("algo"), py::arg("compat_value_bug"),
        py::arg("S_bug"), py::arg("B_bug"), py::arg("clip_eps"), py::arg("ent_coef"), py::arg("vf_coef"),
        py::arg("dz_bf16") = false, py::arg("precise") = false);
  m.def("encoder_fwd", &encoder_fwd, "fused entity encoder forward (unit MLP, per-type GEMM, max-pool+argmax)",
        py::arg("units"), py::arg("env"), py::arg("w1"), py::arg("b1"), py::arg("wt"), py::arg("bt"), py::arg("we"),
        py::arg("be"), py::arg("counts"), py::arg("compat"), py::arg("exact") = false,
        py::arg("x896_out") = py::none(), py::arg("emb_out") = py::none(), py::arg("arg_out") = py::none());
  m.def("encoder_bwd", &encoder_bwd, "fused entity encoder backward: dW_type (K-blocked split-K MFMA GEMM), dW1, db1",
        py::arg("units"), py::arg("w1"), py::arg("b1"), py::arg("wtT"), py::arg("dtl"), py::arg("q"), py::arg("dx"),
        py::arg("arg"), py::arg("counts"), py::arg("compat"), py::arg("demb_in") = py::none(),
        py::arg("exact") = false);
  m.def("lstm_team_fwd", &lstm_team_fwd, "XCD-team persistent LSTM forward (L2-local hand-off), unit-major gates",
        py::arg("xp4"), py::arg("whh"), py::arg("h0"), py::arg("c0"), py::arg("err"), py::arg("ctl"),
        py::arg("want_f32_h"), py::arg("trace") = py::none(), py::arg("time_major") = false, py::arg("hs_out") = py::none(),
        py::arg("cs_out") = py::none(), py::arg("gates_out") = py::none(), py::arg("bias4") = py::none(),
        py::arg("precise") = false, py::arg("reset") = py::none());
  m.def("lstm_team_bwd", &lstm_team_bwd, "XCD-team persistent LSTM backward (L2-local reduce-scatter)",
        py::arg("dhs"), py::arg("gates4"), py::arg("cs"), py::arg("c0"), py::arg("dhn"), py::arg("dcn"),
        py::arg("whh"), py::arg("err"), py::arg("ctl"), py::arg("trace") = py::none(),
        py::arg("time_major") = false, py::arg("dg_out") = py::none(), py::arg("dg_bf16") = false,
        py::arg("want_dbias") = false, py::arg("precise") = false, py::arg("reset") = py::none());
  m.def("lstm_team_chains", [](int64_t B, bool f32) { return dca_lstm_team_chains((int)B, f32 ? 1 : 0); },
        "sequence chains of a team-recurrence launch of B sequences", py::arg("B"), py::arg("f32"));
  m.def("sample_actions", &sample_actions, "fused masked hierarchical Gumbel-max action sampling (actor)");
  m.def("actor_state_prep", &actor_state_prep, "actor step: state resets + [x | bf16(h)] gate-GEMM operand",
        py::arg("pre"), py::arg("h"), py::arg("c"), py::arg("keep"), py::arg("xh"), py::arg("bump") = py::none());
  m.def("lstm_cell", &lstm_cell, "LSTM cell nonlinearity from fp32 gates (actor single step)", py::arg("gates"),
        py::arg("h"), py::arg("c"), py::arg("h16"), py::arg("active") = py::none());
  m.def("encoder_fp8", &encoder_fp8, "fp8 (e4m3) entity encoder of the actor step: unit MLP, per-type GEMMs, pools "
        "(per_unit: the one-unit-at-a-time workgroup form instead of the wave-parallel one)", py::arg("units"),
        py::arg("env"), py::arg("w1"), py::arg("b1"), py::arg("wt"), py::arg("st"), py::arg("bt"), py::arg("we"),
        py::arg("be"), py::arg("counts"), py::arg("per_unit") = false);
  m.def("actor_core", &actor_core, "fp32 / bf16 actor policy core: pre-RNN + LSTM step (or linear layer) + heads",
        py::arg("x896"), py::arg("wpre"), py::arg("bpre"), py::arg("wg"), py::arg("bg"), py::arg("wh"), py::arg("bh"),
        py::arg("h"), py::arg("c"), py::arg("keep"), py::arg("z"), py::arg("mode"), py::arg("linear") = false,
        py::arg("active") = py::none(), py::arg("bump") = py::none());
  m.def("actor_fp8", &actor_fp8, "fp8 (e4m3) actor policy core: pre-RNN + LSTM step + heads from x896",
        py::arg("x896"), py::arg("wpre"), py::arg("spre"), py::arg("bpre"), py::arg("wg"), py::arg("sg"), py::arg("bg"),
        py::arg("wh"), py::arg("sh"), py::arg("bh"), py::arg("h"), py::arg("c"), py::arg("keep"), py::arg("z"),
        py::arg("active") = py::none(), py::arg("bump") = py::none());
  m.def("attn_block_fwd", &attn_block_fwd, "fused fp32 entity-attention block forward: LN + QKV + attention + "
        "out-projection + residual + pools (-> xn, mean, rstd, qkv, o, lse, e1)");
  m.def("attn_block_bwd", &attn_block_bwd, "fused fp32 entity-attention block backward: demb + dO + attention "
        "backward + dXn + LayerNorm backward (-> de1, dqkv, de0, [dgamma | dbeta | dbt])");
    m.def("loss_prep", &loss_prep, "loss normalisers from one-hot action rows (graph-replayable)");
  m.def("loss_prep_ws_elems", &loss_prep_ws_elems, "int32 workspace elements of loss_prep");
  m.def("loss_assemble", &loss_assemble, "loss scalar + metrics from heads/loss partials", py::arg("part"),
        py::arg("norms"), py::arg("N"), py::arg("algo"), py::arg("ent_coef"), py::arg("vf_coef"), py::arg("out"),
        py::arg("S") = 0, py::arg("compat_value_bug") = false);
  m.def("weight_prep", &weight_prep, "gather the flat fp32 params into bf16 / fp32 working weight images (+ bf16 "
        "hi / lo split images)", py::arg("src"), py::arg("map16"), py::arg("dst16"), py::arg("map32"), py::arg("dst32"),
        py::arg("maps") = py::none(), py::arg("dsth") = py::none(), py::arg("dstl") = py::none());
  m.def("gemm_tn", &gemm_tn, "C (+)= A^T B for K-outer bf16 or fp32 (bf16x3) operands (split-K MFMA, LDS transposed reads)",
        py::arg("A"), py::arg("B"), py::arg("C"), py::arg("perm") = py::none(), py::arg("accumulate") = false,
        py::arg("B0") = py::none(), py::arg("colsum") = py::none(), py::arg("exact") = false);
  m.def("dpre_dx", &dpre_dx, "fused pre-RNN dX chain: (dG·W_ih)*[x>0] -> dpre, dpre·W_pre -> dx (bf16x3 with pre-split "
        "bf16 hi/lo weights, or exact-f32 MFMA with fp32 weights)", py::arg("dG"), py::arg("w1h"), py::arg("w1l"),
        py::arg("x"), py::arg("w2h"), py::arg("w2l"));
  m.def("pre_rnn_chain", &pre_rnn_chain, "fused forward chain x = relu(x896·W_pre^T + b), xp = x·W_ih^T (bf16x3)",
        py::arg("x896"), py::arg("w1h"), py::arg("w1l"), py::arg("bias"), py::arg("w2h"), py::arg("w2l"),
        py::arg("x_out") = py::none(), py::arg("xp_out") = py::none());
  m.def("rowmm_out256", &rowmm_out256, "C (N,256) = A (N,K)·W^T + b on the chain kernel's stage 1 (bf16x3)",
        py::arg("A"), py::arg("wh"), py::arg("wl"), py::arg("bias"));
  m.def("rowmm_in256", &rowmm_in256, "C (N,X) = A (N,256)·W^T on the chain kernel's stage 2 (bf16x3)", py::arg("A"),
        py::arg("wh"), py::arg("wl"));
  m.def("split_bf16x2", &split_bf16x2, "fp32 -> (hi, lo) bf16 images with x = hi + lo (slab_major: (R,K) -> "
        "[K/32][R][32] images, the dpre_dx operand layout)", py::arg("src"), py::arg("slab_major") = false);
  m.def("enc_small_grads", &enc_small_grads, "entity-encoder type-bias and env-layer gradients in one pass");
  m.def("replay_gather", &replay_gather, "minibatch gather from an HBM replay pool into time-major rows (one launch)");
  m.def("vtrace_step", &vtrace_step, "V-trace advantages / value targets of a minibatch from the step's own values",
        py::arg("z"), py::arg("vcol"), py::arg("lp"), py::arg("mu"), py::arg("vt"), py::arg("B"), py::arg("S"),
        py::arg("gamma"), py::arg("lam"), py::arg("rho_bar") = 1.0, py::arg("c_bar") = 1.0);
  m.def("featurize_raw", &featurize_raw, "GPU unit featurization from raw unit records (featurize.hip)",
        py::arg("raw"), py::arg("hero"), py::arg("units"), py::arg("handles") = py::none());
  m.def("occupy_xcd", &occupy_xcd, "test utility: hold CUs of one XCD for a while (160 KB LDS per workgroup)",
        py::arg("xcd"), py::arg("blocks"), py::arg("seconds"), py::arg("like"));
  m.def("returns_scan", &returns_scan, "segmented reverse scan: discounted returns / GAE / V-trace GAE + per-team EMA "
        "normalisation (positional: ..., factor, eps, lr or None, rho_bar, c_bar)");
}
