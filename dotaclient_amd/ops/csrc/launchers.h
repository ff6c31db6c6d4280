// extern "C" launchers exported by the *.hip kernel translation units (raw pointers + stream; no torch types).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" {

hipError_t dca_split_bf16x2(const float* src, short* hi, short* lo, long long n, hipStream_t stream);
hipError_t dca_split_bf16x2_blk(const float* src, short* hi, short* lo, int R, int K, hipStream_t stream);
// attn_block.hip
hipError_t dca_attn_block_fwd_f32(const float* e0, const float* bout, const float* gamma, const float* beta,
                                  const void* wqh, const void* wql, const float* bq, const void* woh,
                                  const void* wol, float* xn, float* mu, float* rs, float* qkv, float* o, float* lse,
                                  float* e1, float* x896, unsigned char* arg, const int* off, int compat, int N,
                                  float eps, hipStream_t stream, int exact);
int dca_attn_block_bwd_groups(int N);
hipError_t dca_attn_block_bwd_f32(const float* dtl, const float* q, int ldq, const float* dx, const unsigned char* arg,
                                  const int* off, int compat, const float* o, const float* qkv, const float* bq,
                                  const float* lse, const float* e0, const float* bout, const float* mu,
                                  const float* rs, const float* gamma, const void* woth, const void* wotl,
                                  const void* wq4h, const void* wq4l, float* de1, float* dqkv, float* de0,
                                  float* part, float* tmp, float* sums, int N, hipStream_t stream,
                                  unsigned long long* trace, int exact);
// actor_fp8.hip
hipError_t dca_actor_fp8(const short* x896, const void* wpre, const float* spre, const float* bpre, const void* wg,
                         const float* sg, const float* bg, const void* wh, const float* sh, const float* bh, float* h,
                         float* c, const float* keep, const float* active, float* z, int n, long long* bump,
                         hipStream_t stream);
hipError_t dca_encoder_fp8(const void* units, int f16, const float* env, const float* w1, const float* b1,
                           const void* wt, const float* st, const float* bt, const float* we, const float* be,
                           short* x896, short* emb, int N, int U, const int* counts, int per_unit,
                           hipStream_t stream);

hipError_t dca_dpre_dx(const float* dG, const void* w1h, const void* w1l, const float* x, const void* w2h,
                       const void* w2l, float* dpre, float* dx, int N, int K1, int X, int exact, int epi, hipStream_t stream);

hipError_t dca_adam_step(float* param, const float* grad, float* m, float* v, const int* seg, int64_t n,
                         const float* counts, float* steps, int n_params, float* partials, float* norm_out, float lr,
                         float b1, float b2, float eps, float max_norm, hipStream_t st, int divide, int64_t header,
                         const float* skip, float* nonfinite);
int dca_adam_partials_len(int n_params);

hipError_t dca_ingest_scatter(void* const* dst, const void* const* src, const int* row_bytes, int n, const int* inv,
                              int L, int nsrc, float* valid, hipStream_t st);
hipError_t dca_adv_normalize(const float* adv, const float* valid, float* out, int L, float eps, hipStream_t st);
hipError_t dca_multi_copy(void* const* dst, const void* const* src, const long long* bytes, int n, hipStream_t st);
hipError_t dca_multi_axpy(float* const* dst, const float* const* src, const long long* numel, int n,
                          const float* scale, hipStream_t st);

int dca_heads_loss_nblocks(int N);
hipError_t dca_heads_loss(const float* z, int ldz, const void* emb, const unsigned char* act, const unsigned char* msk,
                          int A, const float* adv, const float* ret, const float* logp_old, const float* nret,
                          const float* norms, float* dz, float* dtl, float* part, float* logp_out, int N, int U,
                          int algo, int compat_value_bug, int S_bug, int B_bug, float clip_eps, float ent_coef,
                          float vf_coef, hipStream_t st, short* dz16, int emb_f32, int precise = 0);

hipError_t dca_encoder_fwd(const float* units, const float* env, const float* w1, const float* b1, const void* wt,
                           const float* bt, const float* we, const float* be, void* x896, void* emb,
                           unsigned char* arg, int N, int U, const int* counts, int compat, hipStream_t st, int f32);
size_t dca_encoder_bwd_workspace(int N, int U, const int* counts, int f32);
hipError_t dca_encoder_bwd(const float* units, const float* w1, const float* b1, const void* wtT, const float* dtl,
                           const float* q, int ldq, const float* dx, const unsigned char* arg, float* dwt, float* dw1,
                           float* db1, void* ws, size_t ws_bytes, int N, int U, const int* counts, int compat,
                           hipStream_t st, const void* demb_in, int f32);

size_t dca_lstm_team_ctl_bytes();
size_t dca_lstm_team_workspace(int B, int H, int backward, int f32);
hipError_t dca_lstm_team_fwd(const float* xp4, const void* whh, const float* h0, const float* c0, short* hs,
                             float* hsf, float* cs, float* gates4, float* hn, float* cn, void* ctl, void* ws,
                             size_t ws_bytes, unsigned* err, int B, int S, int H, int time_major, hipStream_t st,
                             unsigned long long* trace, const float* bias4, int f32, int precise = 0,
                             const unsigned char* rst = nullptr);
int dca_lstm_team_chains(int B, int f32);
hipError_t dca_lstm_team_bwd(const float* dhs, const float* gates4, const float* cs, const float* c0,
                             const float* dhn, const float* dcn, const void* whh, float* dgates4, float* dh0,
                             float* dc0, void* ctl, void* ws, size_t ws_bytes, unsigned* err, int B, int S, int H,
                             int time_major, hipStream_t st, unsigned long long* trace, short* dg16, float* dbpart,
                             int f32, int precise = 0, const unsigned char* rst = nullptr);

hipError_t dca_sample_actions(const float* z, int ldz, const void* emb, int emb_f32, const void* handles, int h32,
                              int N, int U, unsigned long long seed, const long long* ctr, int* idx,
                              unsigned char* act, unsigned char* msk, float* logp, float* value, hipStream_t st);
hipError_t dca_actor_core(const void* x896, int x_f32, const void* wpre, const float* bpre, const void* wg,
                          const float* bg, const void* wh, const float* bh, float* h, float* c, const float* keep,
                          const float* active, float* z, int n, int hidden, int linear, int mode, long long* bump,
                          hipStream_t st);
hipError_t dca_actor_state_prep(const short* pre, float* h, float* c, const float* keep, short* xh, int N, int P,
                                int H, long long* bump, hipStream_t st);
hipError_t dca_lstm_cell(const float* gates, float* h, float* c, short* h16, const float* active, int N, int H,
                         hipStream_t st);

hipError_t dca_vtrace_step(const float* z, int ldz, int vcol, const float* lp, const float* mu, const float* vt,
                           float* adv, float* ret, float* stats, int B, int S, float gamma, float lam, float rho_bar,
                           float c_bar, hipStream_t st);
hipError_t dca_returns(const float* rew, int K, const float* val, const float* lr, const int* off, const int* seglen,
                       const float* boot, const unsigned char* done, const int* keys, int nseg, int max_len,
                       float* ret, float* adv, float* norm, float* stats, const float* ema_in, float* ema_out,
                       int mode, int normalize, float gamma, float lam, float rho_bar, float c_bar, float factor,
                       float eps, hipStream_t st);

int dca_loss_prep_blocks();
hipError_t dca_loss_prep(const unsigned char* act, int N, int A, int* partial, unsigned* counter, float* norms,
                         hipStream_t st);
hipError_t dca_occupy_xcd(int xcd, int blocks, double seconds, int* seen, hipStream_t st);
// raw unit records (rows, U, 8) i32 + hero (rows, 4) f32 → features (rows, U, 10) + handles (rows, U) (may be null);
// half_out: fp16 features / int32 handles, else fp32 / int64 (featurize.hip)
hipError_t dca_featurize_raw(const void* raw, const float* hero, void* units, void* handles, int rows, int U,
                             int half_out, hipStream_t st);
hipError_t dca_featurize_raw16(const void* raw16, const float* hero, void* units, void* handles, int rows, int U,
                               hipStream_t st);
hipError_t dca_loss_assemble(const float* part, int nrows, const float* norms, int N, int algo, float ent_coef,
                             float vf_coef, float* out, int S, int vbug, hipStream_t st);
hipError_t dca_weight_prep(const float* src, const int* map16, short* dst16, int n16, const int* map32, float* dst32,
                           int n32, const int* maps, short* dsth, short* dstl, int ns, hipStream_t st);

void dca_gemm_tn_plan(int M, int N, int K, int* splits, int* kc, int* tiles, int f32);
hipError_t dca_gemm_tn(const void* A, int lda, const void* B, int ldb, const void* B0, int split_rows, float* C,
                       int ldc, const int* perm, int accumulate, int M, int N, int K, float* slab, float* colsum,
                       hipStream_t st, int f32);

int dca_enc_small_out();
int dca_enc_small_blocks();
hipError_t dca_enc_small_grads(const float* z, int ldz, const float* dtl, int U, const int* type_off, const float* dx,
                               const float* env, const float* we, const float* be, int N, int compat, float* part,
                               float* out, hipStream_t st);

hipError_t dca_replay_gather(const void* const* src, void* const* dst, const long long* row_bytes, const int* per_step,
                             int nf, const long long* idx, int S, int B, hipStream_t st);

}  // extern "C"
