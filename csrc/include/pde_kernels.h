// extern "C" launchers of the framework's HIP kernels (device TUs include no torch headers; the
// torch binding layer in csrc/ops_bindings.cpp calls these with raw pointers + the current stream).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// ---- LeNet (toy CNN) fused kernels: csrc/kernels/lenet.hip ----
hipError_t pde_lenet_conv_fwd(const float* X, const int* idx, int n_idx, const long long* step, int nbatches,
                              int stride, const long long* labels_all, int B, const float* w1, const float* b1,
                              const float* Wt2, const float* b2, float* P1, uint8_t* A1, float* P2, uint8_t* A2,
                              int* cur_row, long long* cur_lbl, float* zero_ptr, int zero_n, int dbg, hipStream_t st);
hipError_t pde_lenet_fc1_fwd(const float* P2, int B, const float* W, const float* bias, float* H1, long long* ctr,
                             int nctr, hipStream_t st);
hipError_t pde_lenet_head(const float* H1, int B, const float* W2, const float* b2, const long long* labels,
                          float inv_b, float* logp_out, float* dZ2, float* dZ1, float* row_loss, int* row_hit,
                          double* loss_sum, unsigned long long* correct, hipStream_t st);
hipError_t pde_lenet_head2(const float* H1, int B, const float* W2, const float* b2, const long long* labels,
                           float inv_b, float* logp_out, float* dZ2, float* dZ1, float* row_loss, int* row_hit,
                           double* loss_sum, unsigned long long* correct, hipStream_t st);
hipError_t pde_lenet_head_bwd(const float* H1, int B, const float* W2, const float* logp, const float* g, float* dZ2,
                              float* dZ1, hipStream_t st);
hipError_t pde_lenet_fc_bwd(const float* P2, const float* H1, const float* dZ1, const float* dZ2, const float* W1,
                            int B, float* dP2m, float* gW1, float* gb1, float* gW2, float* gb2, const float* row_loss,
                            const int* row_hit, double* loss_sum, unsigned long long* correct, int dbg, int part,
                            hipStream_t st);
hipError_t pde_lenet_conv_bwd(const float* X, const int* rows, const float* P1, const uint8_t* A1,
                              const float* dP2m, const uint8_t* A2, const float* W2c, int B, float* gW1c,
                              float* gb1c, float* gW2c, float* gb2c, int c1_nrep, int c1_rep_stride,
                              const float* row_loss, const int* row_hit, double* loss_sum,
                              unsigned long long* correct, int dbg, const void* peer_dev, float* ar_buf, int64_t ar_n, int ar_two,
                              hipStream_t st);

void pde_lenet_set_prof(unsigned long long* buf);
unsigned long long* pde_lenet_prof_slot(int kid);

// ---- optimizers: csrc/kernels/optim.hip ----
// fold_*: gradient replicas folded before the update: for e in [fold_off, fold_off + fold_len),
// g[e] = sum_{r < fold_nrep} g[e + r * fold_stride] (written back); replica storage r >= 1 is skipped.
hipError_t pde_adam_flat(float* p, float* g, float* m, float* v, long long n, float lr, float b1, float b2,
                         float eps, float wd, int decoupled, float grad_scale, long long* step, unsigned* arrive,
                         int bump, long long pack_off, float* pack_dst, long long fold_off, int fold_len,
                         int fold_nrep, int fold_stride, const void* peer_dev, long long ar_off,
                         long long* ar_epoch, int ar_two, int pack_mode, long long fold2_off, int fold2_len,
                         int fold2_nrep, int fold2_stride, hipStream_t st);
hipError_t pde_sgd_flat(float* p, float* g, float* buf, long long n, float lr, float momentum, float dampening,
                        float wd, int nesterov, float grad_scale, long long* step, unsigned* arrive, int bump,
                        long long pack_off, float* pack_dst, long long fold_off, int fold_len, int fold_nrep,
                        int fold_stride, int pack_mode, long long fold2_off, int fold2_len, int fold2_nrep,
                        int fold2_stride, hipStream_t st);
hipError_t pde_lenet_pack_w2(const float* w2, float* dst, hipStream_t st);

// ---- LeNet step v2: csrc/kernels/lenet_v2.hip ----
hipError_t pde_lenet_conv_fwd2(const float* Xb, int B, const float* w1, const float* b1, const float* Wp,
                               const float* b2, float* P1, uint8_t* A1, float* P2, uint8_t* A2, float* zero_ptr,
                               int zero_n, hipStream_t st);
hipError_t pde_lenet_gather(const float* X, const long long* labels, const int* idx, int n_idx, const long long* ctr,
                            int nbatches, int B, float* Xdst, long long* Ydst, int* rows_dst, hipStream_t st);
hipError_t pde_lenet_pack_w2_v2(const float* w2, float* dst, hipStream_t st);
// Gradient reduction of the v2 conv backward (lenet_v2.hip): deferred to the optimizer, or in-launch.
struct PdeLenetBwdOpt {
  float* slab;              // [16][25088] conv2 wgrad slabs
  long long* c1rep;         // [16][576] int64 conv1 wgrad replicas (zeroed once; kept zero by the kernel)
  float* c1part;            // defer mode: [16][576] float conv1 wgrad replicas (atomics)
  unsigned* tick;           // [32] arrival counters (zeroed once)
  float* g;                 // flat gradient buffer (canonical conv gradients written here)
  long long c1w, c1b, c2w, c2b;
  const void* peer_dev;     // fused fc-bucket all-reduce (nullptr: none)
  float* ar_buf;
  long long ar_n;
  int ar_two;
  int defer;                // 0: fold in the launch; 1: leave slabs / replicas for the flat optimizer to fold;
                            // 2 (ext): slabs + per-image conv1 partials, folded by pde_lenet_conv_grad_fold
  float* c1img;             // ext: [B][520] per-image conv1 partials
};
// ext-mode fold fused with the in-place one-shot (two = 0) or two-shot (two = 1) all-reduce of the
// registered flat gradient buffer
// (ipdev: PeerIpDev bytes of that registration; [lo, hi) the conv range the fold writes; sync: two
// zero-initialised device counters, left zero by every launch).  hipErrorInvalidValue when the buffer
// does not fit one one-shot grid (the grid cap of ranks sharing a GPU).
hipError_t pde_lenet_conv_fold_ar(const void* ipdev, const float* slab, const float* c1img, int B, long long c1w,
                                 long long c1b, long long c2w, long long c2b, long long n, long long lo, long long hi,
                                 unsigned* sync, float scale, int two, hipStream_t st);
hipError_t pde_lenet_conv_grad_fold(const float* slab, const float* c1img, int B, float* g, long long c1w, long long c1b,
                                    long long c2w, long long c2b, hipStream_t st);
hipError_t pde_lenet_conv_bwd2(const float* Xb, const float* P1, const uint8_t* A1, const float* dP2m,
                               const uint8_t* A2, const float* W2c, int B, const PdeLenetBwdOpt* o,
                               const float* row_loss, const int* row_hit, double* loss_sum, unsigned long long* correct,
                               const float* gX, const long long* glabels, const int* gidx, int gn_idx,
                               const long long* gctr, int gnbatches, int gstride, float* gXdst, long long* gYdst,
                               int* grows, int dbg, hipStream_t st);
hipError_t pde_scale(float* x, long long n, float s, hipStream_t st);

// ---- generic ops: csrc/kernels/generic.hip ----
hipError_t pde_gemm_f32(const float* A, const float* B, float* C, const float* bias, int M, int N, int K, int lda,
                        int ldb, int ldc, int transA, int transB, long long sA, long long sB, long long sC, int batch,
                        float alpha, float beta, int bias_mode, int relu, int atomic, hipStream_t st);
hipError_t pde_xent_fwd(const float* x, const long long* y, int B, int C, float* row_loss, float* lse, hipStream_t st);
hipError_t pde_xent_fwd_bf16(const void* x, const long long* y, int B, int C, float* row_loss, float* lse,
                             hipStream_t st);
hipError_t pde_xent_bwd_bf16(const void* x, const long long* y, const float* lse, const float* gscale, int per_row,
                             float mul, int B, int C, void* dx, hipStream_t st);
hipError_t pde_xent_bwd(const float* x, const long long* y, const float* lse, const float* gscale, int per_row,
                        float mul, int B, int C, float* dx, hipStream_t st);
hipError_t pde_log_softmax_fwd(const float* x, int B, int C, float* out, hipStream_t st);
hipError_t pde_log_softmax_bwd(const float* out, const float* g, int B, int C, float* dx, hipStream_t st);
hipError_t pde_relu_fwd(const float* x, float* y, long long n, hipStream_t st);
hipError_t pde_relu_bwd(const float* y, const float* g, float* dx, long long n, hipStream_t st);
hipError_t pde_pool2_fwd(const float* x, int NC, int H, int W, float* y, uint8_t* code, hipStream_t st);
hipError_t pde_pool2_bwd(const float* g, const uint8_t* code, int NC, int H, int W, float* dx, hipStream_t st);
hipError_t pde_im2col(const float* x, int B, int C, int H, int W, int KH, int KW, int stride, int pad, int OH, int OW,
                      float* col, hipStream_t st);
hipError_t pde_col2im(const float* col, int B, int C, int H, int W, int KH, int KW, int stride, int pad, int OH,
                      int OW, float* dx, hipStream_t st);
hipError_t pde_bias_grad_nchw(const float* dy, int B, int O, long long P, float* db, hipStream_t st);
hipError_t pde_colsum(const float* x, int M, int N, float* out, hipStream_t st);
hipError_t pde_gather_rows(const float* src, const long long* idx, int n, int row_floats, float* out, hipStream_t st);


// ---- transformer (transformer.hip) ----
hipError_t pde_ln_fwd(const void* X, const void* D, void* S, const void* G, const void* B, void* Y, float* mean,
                      float* rstd, int N, int C, float eps, hipStream_t st);
int pde_ln_bwd_blocks(int N);
hipError_t pde_ln_bwd(const void* dY, const void* X, const float* mean, const float* rstd, const void* G,
                      const void* dRes, void* dX, float* part, void* dG, void* dB, int N, int C, int accumulate,
                      hipStream_t st);
hipError_t pde_gelu_fwd(const void* X, void* Y, int64_t n, hipStream_t st);
hipError_t pde_gelu_bwd(const void* dY, const void* X, void* dX, int64_t n, hipStream_t st);
hipError_t pde_xent_bf16(void* logits, const int64_t* tgt, int N, int Vp, int V, float scale, float* loss_rows,
                         int write_grad, hipStream_t st);
hipError_t pde_embed_fwd(const int64_t* idx, const void* wte, const void* wpe, void* out, int N, int T, int C,
                         hipStream_t st);
hipError_t pde_embed_bwd(const void* dX, const int64_t* idx, void* dwte, void* dwpe, float* acc, uint8_t* touched,
                         int N, int T, int C, int Vp, int accumulate_pos, hipStream_t st);
hipError_t pde_sumsq_bf16(const void* g, int64_t n, float scale, float* out, float* step_inc, hipStream_t st);
hipError_t pde_adamw_master(float* master, void* p16, const void* g16, float* m, float* v, int64_t n, float lr,
                            float b1, float b2, float eps, float wd, float grad_scale, int step,
                            const uint8_t* decay_blk, const float* clip_sumsq, float max_norm, const float* step_dev,
                            hipStream_t st);
hipError_t pde_f32_to_bf16(const float* x, void* y, int64_t n, hipStream_t st);
hipError_t pde_scale_bf16(void* x, const float* s, int64_t n, hipStream_t st);   // x *= s[0], n % 8 == 0
hipError_t pde_sum_f32(const float* x, int n, float* out, float scale, hipStream_t st);
hipError_t pde_token_batch(const int64_t* pool, const int64_t* rows, int B, int T, int64_t* x, int64_t* y,
                           hipStream_t st);
int pde_colsum_bf16_splits(int C);
hipError_t pde_colsum_bf16(const void* x, int N, int C, float* part, void* out, hipStream_t st);

// ---- implicit-GEMM bf16 convolutions, NHWC (conv.hip) ----
void pde_conv_set_stages(int nst);
int pde_conv_fprop_mtiles(int M, int N);
int pde_conv_stats_rows(int Bn, int H, int W, int C, int N, int R, int S, int stride, int pad, int OH, int OW);
// ResNet stem (7x7 / stride 2 / pad 3, 3 -> 64 ch, NHWC bf16): stem.hip
int pde_stem_stats_blocks(int Bn, int OH);
hipError_t pde_stem_fwd(const void* X, const void* W, void* Wp, void* Y, float* stats, int Bn, int H, int Wd,
                        hipStream_t st);
int pde_stem_wgrad_blocks(int Bn, int OH);
hipError_t pde_stem_wgrad(const void* X, const void* dY, float* part, void* dW, int Bn, int H, int Wd,
                          hipStream_t st);
hipError_t pde_conv_fprop(const void* x, const void* w, void* y, float* stats, int Bn, int H, int W, int C, int N,
                          int R, int S, int stride, int pad, int OH, int OW, hipStream_t st);
hipError_t pde_conv_wtrans(const void* w, void* wt, int N, int T, int C, hipStream_t st);
hipError_t pde_conv_wtrans_batch(const void* desc, int nconv, int total, long long* ctr, int ncnt, hipStream_t st);
int pde_conv_wtdesc_bytes();
// bx..bpart (optional, stride 1): BN-backward partials of dx fused into the epilogue (conv.hip BnbArgs)
int pde_conv_dgrad_bnb_rows(int Bn, int H, int W, int C, int N, int R, int S, int stride, int pad);
hipError_t pde_conv_dgrad(const void* dy, const void* wt, void* dx, const void* res, const void* dy2, const void* wt2,
                          int Bn, int H, int W, int C, int N, int R, int S, int stride, int pad, int OH, int OW,
                          const void* bx, const float* bsc, const float* bsh, const float* bmu, const float* brs,
                          float* bpart, hipStream_t st);
int pde_conv_wgrad_splits2(int Bn, int H, int W, int C, int N, int R, int S, int stride, int pad, int OH, int OW);
int pde_conv_wgrad_splits(int Bn, int OH, int OW, int N, int T, int C);
hipError_t pde_sum_slabs_bf16(const float* part, int S, int64_t n, void* out, hipStream_t st);
hipError_t pde_conv_wgrad(const void* dy, const void* x, float* part, int splits, void* dw, int Bn, int H, int W,
                          int C, int N, int R, int S, int stride, int pad, int OH, int OW, hipStream_t st);

// ---- bf16 MFMA GEMM with fused epilogues (gemm.hip) ----
int pde_gemm_num_cfgs();
void pde_gemm_tile(int cfg, int* bm, int* bn);
int pde_gemm_splits(int K, int splits);
void pde_gemm_set_dbg(int d);
hipError_t pde_gemm(const void* A, const void* B, void* C, void* C2, const void* bias, const void* aux, float* colsum,
                    int ta, int tb, int epi, int M, int N, int K, int lda, int ldb, int ldc, int splits, int cfg,
                    const float* scale, hipStream_t st);
hipError_t pde_gemm_reduce(const float* part, int S, int M, int N, void* dw, const float* cs, void* db,
                           const float* scale, hipStream_t st);

// ---- attention (attention.hip) ----
void pde_attn_set_variant(int v);
hipError_t pde_attn_fwd(const void* q, const void* k, const void* v, int ldq, void* o, int ldo, float* lse, int B,
                        int T, int H, float scale, hipStream_t st);
hipError_t pde_attn_bwd(const void* q, const void* k, const void* v, int ldq, const void* o, const void* dout,
                        int ldo, const float* lse, float* Dd, void* dq, void* dk, void* dv, int B, int T, int H,
                        float scale, hipStream_t st);


// ---- resnet (resnet.hip) ----
int pde_bn_blocks(int M, int C);
int pde_bn_part_rows(int pre_nblk);
hipError_t pde_bn_fwd(const void* x, const void* res, void* y, int M, int C, const void* gamma, const void* beta,
                      float eps, float momentum, float* run_mean, float* run_var, float* part, float* mean,
                      float* rstd, float* scale, float* shift, int relu, int training, int pre_nblk,
                      const float* res_scale, const float* res_shift, hipStream_t st);
hipError_t pde_bn_bwd(const void* dy, const void* y, const void* x, int M, int C, const void* gamma, const float* mean,
                      const float* rstd, const float* scale, const float* shift, float* part, float* coef,
                      void* dgamma, void* dbeta, void* dx, void* dres, int relu, int pre_nblk, hipStream_t st);
int pde_bnpool_part_floats(int N, int H, int W, int C);
hipError_t pde_bnpool_fwd(const void* y, const float* scale, const float* shift, void* p, void* arg, void* ysel,
                          int N, int C, int H, int W, int OH, int OW, hipStream_t st);
hipError_t pde_bnpool_bwd(const void* dp, const void* arg, const void* y, const void* ysel, const float* scale,
                          const float* shift, const void* gamma, const float* mean, const float* rstd, float* part,
                          float* coef, void* dgamma, void* dbeta, void* dy, int N, int C, int H, int W, int OH, int OW,
                          hipStream_t st);
hipError_t pde_maxpool3s2_fwd(const void* x, void* y, void* arg, int N, int C, int H, int W, int OH, int OW,
                              hipStream_t st);
hipError_t pde_maxpool3s2_bwd(const void* dy, const void* arg, void* dx, int N, int C, int H, int W, int OH, int OW,
                              hipStream_t st);
hipError_t pde_avgpool_fwd(const void* x, void* out, int N, int HW, int C, hipStream_t st);
hipError_t pde_avgpool_bwd(const void* dout, void* dx, int N, int HW, int C, hipStream_t st);
hipError_t pde_sgd_master(float* master, void* p16, const void* g16, float* buf, int64_t n, float lr, float momentum,
                          float wd, int nesterov, float grad_scale, const uint8_t* decay_blk, hipStream_t st);

#ifdef __cplusplus
}
#endif
