// torch bindings of the ResNet kernels (csrc/kernels/resnet.hip): fused BatchNorm(+residual)+ReLU
// over channels-last bf16 activations, and the SGD step with fp32 master weights.
#include "pde_bind.h"
#include "pde_kernels.h"

namespace pde {
namespace {

int64_t nhwc_rows(const at::Tensor& x, const char* name) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == BF16, name, " must be a bf16 GPU tensor");
  if (x.dim() == 4) {
    TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), name, " must be channels-last");
    return x.size(0) * x.size(2) * x.size(3);
  }
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), name, " must be [N, C] contiguous or 4-D channels-last");
  return x.size(0);
}

void check_same(const at::Tensor& a, const at::Tensor& b, const char* name) {
  TORCH_CHECK(a.sizes() == b.sizes() && a.strides() == b.strides() && a.scalar_type() == b.scalar_type(), name,
              " must match the input's shape / layout / dtype");
}

void check_c(int64_t C) {
  TORCH_CHECK(C % 8 == 0 && 256 % (C / 8) == 0, "batchnorm kernel: C must be 8 * a power of two <= 2048");
}

int64_t bn_blocks(int64_t M, int64_t C) { return pde_bn_blocks((int)M, (int)C); }

// y None: statistics / finalize only (mean, rstd, scale, shift and the running stats; no apply pass)
// res_scale / res_shift (optional, with res): the residual is a BatchNorm input normalised on the fly,
// y = relu(x*scale + shift + res*res_scale + res_shift) (a ResNet downsample branch, never materialised)
void bn_fwd(const at::Tensor& x, const OptT& res, const OptT& y, const at::Tensor& gamma, const at::Tensor& beta,
            double eps, double momentum, const OptT& run_mean, const OptT& run_var, const at::Tensor& part,
            const at::Tensor& mean, const at::Tensor& rstd, const at::Tensor& scale, const at::Tensor& shift, bool relu,
            bool training, int64_t pre_nblk, const OptT& res_scale, const OptT& res_shift) {
  const int64_t M = nhwc_rows(x, "x"), C = x.size(1);
  check_c(C);
  void* yp = nullptr;
  if (y.has_value() && y->defined()) {
    check_same(x, *y, "y");
    yp = y->data_ptr();
  }
  TORCH_CHECK(yp || training, "bn_fwd: eval mode needs y");
  const void* r = nullptr;
  if (res.has_value() && res->defined()) {
    check_same(x, *res, "residual");
    r = res->data_ptr();
  }
  const float* rsc = optr<float>(res_scale, "res_scale", F32, C);
  const float* rsh = optr<float>(res_shift, "res_shift", F32, C);
  TORCH_CHECK(!(rsc || rsh) || (r && rsc && rsh), "bn_fwd: res_scale / res_shift need res and each other");
  check_cuda(gamma, "gamma", BF16, C);
  check_cuda(beta, "beta", BF16, C);
  float* rm = optr<float>(run_mean, "running_mean", F32, C);
  float* rv = optr<float>(run_var, "running_var", F32, C);
  if (training)
    check_cuda(part, "part", F32,
               (pre_nblk > 0 ? pde_bn_part_rows((int)pre_nblk) : (int64_t)pde_bn_blocks((int)M, (int)C)) * 2 * C);
  for (auto* t : {&mean, &rstd, &scale, &shift}) check_cuda(*t, "bn stats", F32, C);
  hip_check(pde_bn_fwd(x.data_ptr(), r, yp, (int)M, (int)C, gamma.data_ptr(), beta.data_ptr(), (float)eps,
                       (float)momentum, rm, rv, ptr<float>(part), ptr<float>(mean), ptr<float>(rstd), ptr<float>(scale),
                       ptr<float>(shift), relu, training, (int)pre_nblk, rsc, rsh, cur_stream()),
            "bn_fwd");
}

// y: the forward output (ReLU mask y > 0), or None with scale / shift of the forward: the mask is
// recomputed from x (only valid without a residual), one tensor less to read
void bn_bwd(const at::Tensor& dy, const OptT& y, const at::Tensor& x, const at::Tensor& gamma, const at::Tensor& mean,
            const at::Tensor& rstd, const at::Tensor& part, const at::Tensor& coef, const at::Tensor& dgamma,
            const at::Tensor& dbeta, const at::Tensor& dx, const OptT& dres, bool relu, const OptT& scale,
            const OptT& shift, int64_t pre_nblk) {
  const int64_t M = nhwc_rows(x, "x"), C = x.size(1);
  check_c(C);
  check_same(x, dy, "dy");
  check_same(x, dx, "dx");
  const void* yp = nullptr;
  if (y.has_value() && y->defined()) {
    check_same(x, *y, "y");
    yp = y->data_ptr();
  }
  const float* sc = optr<float>(scale, "scale", F32, C);
  const float* sf = optr<float>(shift, "shift", F32, C);
  TORCH_CHECK(!relu || yp || (sc && sf), "bn_bwd: a ReLU needs y or the forward's scale / shift");
  void* dr = nullptr;
  if (dres.has_value() && dres->defined()) {
    check_same(x, *dres, "dres");
    dr = dres->data_ptr();
  }
  check_cuda(gamma, "gamma", BF16, C);
  check_cuda(mean, "mean", F32, C);
  check_cuda(rstd, "rstd", F32, C);
  // pre_nblk > 0: part holds the dgrad epilogue's reduction partials (conv_dgrad bn_* arguments)
  TORCH_CHECK(pre_nblk <= 0 || (relu && !yp && !dr), "bn_bwd: pre-summed partials need relu, y=None and no dres");
  check_cuda(part, "part", F32,
             (pre_nblk > 0 ? pde_bn_part_rows((int)pre_nblk) : (int64_t)pde_bn_blocks((int)M, (int)C)) * 2 * C);
  check_cuda(coef, "coef", F32, 3 * C);
  check_cuda(dgamma, "dgamma", BF16, C);
  check_cuda(dbeta, "dbeta", BF16, C);
  hip_check(pde_bn_bwd(dy.data_ptr(), yp, x.data_ptr(), (int)M, (int)C, gamma.data_ptr(), ptr<float>(mean),
                       ptr<float>(rstd), sc, sf, ptr<float>(part), ptr<float>(coef), dgamma.data_ptr(),
                       dbeta.data_ptr(), dx.data_ptr(), dr, relu, (int)pre_nblk, cur_stream()),
            "bn_bwd");
}

// global average pool: x channels-last [N, C, H, W] -> out [N, C] (and back)
void avgpool_fwd(const at::Tensor& x, const at::Tensor& out) {
  nhwc_rows(x, "x");
  const int64_t N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  check_cuda(out, "out", BF16, N * C);
  TORCH_CHECK(C % 8 == 0, "avgpool: C % 8 == 0");
  hip_check(pde_avgpool_fwd(x.data_ptr(), out.data_ptr(), (int)N, (int)HW, (int)C, cur_stream()), "avgpool_fwd");
}

void avgpool_bwd(const at::Tensor& dout, const at::Tensor& dx) {
  nhwc_rows(dx, "dx");
  const int64_t N = dx.size(0), C = dx.size(1), HW = dx.size(2) * dx.size(3);
  check_cuda(dout, "dout", BF16, N * C);
  TORCH_CHECK(C % 8 == 0, "avgpool: C % 8 == 0");
  hip_check(pde_avgpool_bwd(dout.data_ptr(), dx.data_ptr(), (int)N, (int)HW, (int)C, cur_stream()), "avgpool_bwd");
}

void maxpool3s2_fwd(const at::Tensor& x, const at::Tensor& y, const at::Tensor& arg) {
  nhwc_rows(x, "x");
  nhwc_rows(y, "y");
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.size(1) % 8 == 0, "maxpool: 4-D channels-last, C % 8 == 0");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(y.size(0) == N && y.size(1) == C && y.size(2) == (H - 1) / 2 + 1 && y.size(3) == (W - 1) / 2 + 1,
              "maxpool: y must be [N, C, (H-1)/2+1, (W-1)/2+1]");
  TORCH_CHECK(arg.is_cuda() && arg.scalar_type() == U8 && arg.numel() == y.numel() && arg.is_contiguous(),
              "maxpool: arg must be a uint8 buffer of y.numel()");
  hip_check(pde_maxpool3s2_fwd(x.data_ptr(), y.data_ptr(), arg.data_ptr(), (int)N, (int)C, (int)H, (int)W,
                               (int)y.size(2), (int)y.size(3), cur_stream()),
            "maxpool3s2_fwd");
}

void maxpool3s2_bwd(const at::Tensor& dy, const at::Tensor& arg, const at::Tensor& dx) {
  nhwc_rows(dy, "dy");
  nhwc_rows(dx, "dx");
  const int64_t N = dx.size(0), C = dx.size(1), H = dx.size(2), W = dx.size(3);
  TORCH_CHECK(dy.size(0) == N && dy.size(1) == C && dy.size(2) == (H - 1) / 2 + 1 && dy.size(3) == (W - 1) / 2 + 1 &&
                  C % 8 == 0,
              "maxpool bwd: shape mismatch");
  TORCH_CHECK(arg.is_cuda() && arg.scalar_type() == U8 && arg.numel() == dy.numel(), "maxpool bwd: arg");
  hip_check(pde_maxpool3s2_bwd(dy.data_ptr(), arg.data_ptr(), dx.data_ptr(), (int)N, (int)C, (int)H, (int)W,
                               (int)dy.size(2), (int)dy.size(3), cur_stream()),
            "maxpool3s2_bwd");
}

// ---- stem BN + ReLU + max-pool as one pass (k_bnpool_*): the post-BN map is never materialised ----
void check_pool_shapes(const at::Tensor& y, const at::Tensor& p, const at::Tensor& arg) {
  nhwc_rows(y, "y");
  nhwc_rows(p, "pooled");
  TORCH_CHECK(y.dim() == 4 && p.dim() == 4, "bnpool: 4-D channels-last tensors");
  const int64_t N = y.size(0), C = y.size(1), H = y.size(2), W = y.size(3);
  TORCH_CHECK(C % 8 == 0 && ((C / 8) & (C / 8 - 1)) == 0 && C / 8 <= 64, "bnpool: C must be 8 * a power of two <= 512");
  TORCH_CHECK(p.size(0) == N && p.size(1) == C && p.size(2) == (H - 1) / 2 + 1 && p.size(3) == (W - 1) / 2 + 1,
              "bnpool: pooled must be [N, C, (H-1)/2+1, (W-1)/2+1]");
  TORCH_CHECK(arg.is_cuda() && arg.scalar_type() == U8 && arg.numel() == p.numel() && arg.is_contiguous(),
              "bnpool: arg must be a uint8 buffer of pooled.numel()");
  TORCH_CHECK(y.numel() * 2 < (int64_t(1) << 31), "bnpool: y must be < 2 GiB");
}

int64_t bnpool_part_floats(int64_t N, int64_t H, int64_t W, int64_t C) {
  return pde_bnpool_part_floats((int)N, (int)H, (int)W, (int)C);
}

// training forward: batch statistics from the conv-epilogue partials (part, pre_nblk), running-stat
// update, then the fused BN-apply + ReLU + max-pool pass writing pooled, argmax and y at the argmax
void bnpool_fwd(const at::Tensor& y, const at::Tensor& gamma, const at::Tensor& beta, double eps, double momentum,
                const at::Tensor& run_mean, const at::Tensor& run_var, const at::Tensor& part, int64_t pre_nblk,
                const at::Tensor& mean, const at::Tensor& rstd, const at::Tensor& scale, const at::Tensor& shift,
                const at::Tensor& pooled, const at::Tensor& arg, const at::Tensor& ysel) {
  check_pool_shapes(y, pooled, arg);
  check_same(pooled, ysel, "ysel");
  const int64_t M = nhwc_rows(y, "y"), C = y.size(1);
  check_cuda(gamma, "gamma", BF16, C);
  check_cuda(beta, "beta", BF16, C);
  check_cuda(run_mean, "running_mean", F32, C);
  check_cuda(run_var, "running_var", F32, C);
  TORCH_CHECK(pre_nblk > 0, "bnpool_fwd: needs the producing convolution's statistics partials");
  check_cuda(part, "part", F32, pde_bn_part_rows((int)pre_nblk) * 2 * C);
  for (auto* t : {&mean, &rstd, &scale, &shift}) check_cuda(*t, "bn stats", F32, C);
  hip_check(pde_bn_fwd(y.data_ptr(), nullptr, nullptr, (int)M, (int)C, gamma.data_ptr(), beta.data_ptr(), (float)eps,
                       (float)momentum, ptr<float>(run_mean), ptr<float>(run_var), ptr<float>(part), ptr<float>(mean),
                       ptr<float>(rstd), ptr<float>(scale), ptr<float>(shift), 1, 1, (int)pre_nblk, nullptr, nullptr,
                       cur_stream()),
            "bnpool_fwd (finalize)");
  hip_check(pde_bnpool_fwd(y.data_ptr(), ptr<float>(scale), ptr<float>(shift), pooled.data_ptr(), arg.data_ptr(),
                           ysel.data_ptr(), (int)y.size(0), (int)C, (int)y.size(2), (int)y.size(3), (int)pooled.size(2),
                           (int)pooled.size(3), cur_stream()),
            "bnpool_fwd");
}

void bnpool_bwd(const at::Tensor& dp, const at::Tensor& arg, const at::Tensor& y, const at::Tensor& ysel,
                const at::Tensor& gamma,
                const at::Tensor& mean, const at::Tensor& rstd, const at::Tensor& scale, const at::Tensor& shift,
                const at::Tensor& part, const at::Tensor& coef, const at::Tensor& dgamma, const at::Tensor& dbeta,
                const at::Tensor& dy) {
  check_pool_shapes(y, dp, arg);
  check_same(y, dy, "dy");
  check_same(dp, ysel, "ysel");
  const int64_t C = y.size(1);
  check_cuda(gamma, "gamma", BF16, C);
  for (auto* t : {&mean, &rstd, &scale, &shift}) check_cuda(*t, "bn stats", F32, C);
  check_cuda(part, "part", F32, bnpool_part_floats(y.size(0), y.size(2), y.size(3), C));
  check_cuda(coef, "coef", F32, 3 * C);
  check_cuda(dgamma, "dgamma", BF16, C);
  check_cuda(dbeta, "dbeta", BF16, C);
  hip_check(pde_bnpool_bwd(dp.data_ptr(), arg.data_ptr(), y.data_ptr(), ysel.data_ptr(), ptr<float>(scale),
                           ptr<float>(shift),
                           gamma.data_ptr(), ptr<float>(mean), ptr<float>(rstd), ptr<float>(part), ptr<float>(coef),
                           dgamma.data_ptr(), dbeta.data_ptr(), dy.data_ptr(), (int)y.size(0), (int)C, (int)y.size(2),
                           (int)y.size(3), (int)dp.size(2), (int)dp.size(3), cur_stream()),
            "bnpool_bwd");
}

void sgd_master(const at::Tensor& master, const at::Tensor& p16, const at::Tensor& g16, const at::Tensor& buf,
                double lr, double momentum, double wd, bool nesterov, double grad_scale, const OptT& decay_blk) {
  const int64_t n = master.numel();
  TORCH_CHECK(n % 64 == 0, "sgd_master: flat buffers are padded to 64 elements");
  check_cuda(master, "master", F32);
  check_cuda(p16, "param_bf16", BF16, n);
  check_cuda(g16, "grad_bf16", BF16, n);
  check_cuda(buf, "momentum_buffer", F32, n);
  const uint8_t* db = optr<uint8_t>(decay_blk, "decay_blk", U8, n / 64);
  hip_check(pde_sgd_master(ptr<float>(master), p16.data_ptr(), g16.data_ptr(), ptr<float>(buf), n, (float)lr,
                           (float)momentum, (float)wd, nesterov, (float)grad_scale, db, cur_stream()),
            "sgd_master");
}

// ---- implicit-GEMM convolutions (conv.hip) ----
struct ConvGeom {
  int64_t Bn, C, H, W, N, R, S, OH, OW;
};

ConvGeom conv_geom(const at::Tensor& x, const at::Tensor& w, int64_t stride, int64_t pad) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == BF16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv: x must be a 4-D channels-last bf16 GPU tensor");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == BF16 && w.dim() == 4 &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv: weight must be a 4-D channels-last bf16 GPU tensor");
  ConvGeom g{x.size(0), x.size(1), x.size(2), x.size(3), w.size(0), w.size(2), w.size(3), 0, 0};
  TORCH_CHECK(w.size(1) == g.C, "conv: weight in-channels ", w.size(1), " != input channels ", g.C);
  TORCH_CHECK(g.C % 64 == 0 && g.N % 64 == 0 && g.R * g.S <= 9 && (stride == 1 || stride == 2) && pad >= 0 &&
                  pad < g.R,
              "conv: needs C % 64 == 0, Cout % 64 == 0, kernel <= 3x3, stride 1 or 2");
  g.OH = (g.H + 2 * pad - g.R) / stride + 1;
  g.OW = (g.W + 2 * pad - g.S) / stride + 1;
  TORCH_CHECK(g.OH > 0 && g.OW > 0, "conv: empty output");
  TORCH_CHECK(g.Bn * std::max(g.H * g.W * g.C, g.OH * g.OW * g.N) * 2 < (int64_t(1) << 31),
              "conv: tensors must be < 2 GiB (32-bit buffer offsets)");
  return g;
}

int64_t conv_stats_blocks(int64_t M, int64_t N) { return pde_conv_fprop_mtiles((int)M, (int)N); }
// rows of BN partials conv_fprop writes for this convolution (the halo-tiled kernel tiles by image rows)
int64_t conv_stats_rows(const at::Tensor& x, const at::Tensor& w, int64_t stride, int64_t pad) {
  const ConvGeom g = conv_geom(x, w, stride, pad);
  return pde_conv_stats_rows((int)g.Bn, (int)g.H, (int)g.W, (int)g.C, (int)g.N, (int)g.R, (int)g.S, (int)stride,
                             (int)pad, (int)g.OH, (int)g.OW);
}
// rows to allocate for a conv-stats buffer that feeds bn_fwd (partials + the finalize's pre-fold)
int64_t bn_part_rows(int64_t nblk) { return pde_bn_part_rows((int)nblk); }

void conv_fprop(const at::Tensor& x, const at::Tensor& w, const at::Tensor& y, const OptT& stats, int64_t stride,
                int64_t pad) {
  const ConvGeom g = conv_geom(x, w, stride, pad);
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == BF16 && y.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  y.size(0) == g.Bn && y.size(1) == g.N && y.size(2) == g.OH && y.size(3) == g.OW,
              "conv: y must be channels-last bf16 [B, Cout, OH, OW]");
  const int64_t M = g.Bn * g.OH * g.OW;
  float* sp = optr<float>(stats, "stats", F32, conv_stats_rows(x, w, stride, pad) * 2 * g.N);
  hip_check(pde_conv_fprop(x.data_ptr(), w.data_ptr(), y.data_ptr(), sp, (int)g.Bn, (int)g.H, (int)g.W, (int)g.C,
                           (int)g.N, (int)g.R, (int)g.S, (int)stride, (int)pad, (int)g.OH, (int)g.OW, cur_stream()),
            "conv_fprop");
}

// ds_dy / ds_w / ds_wt (optional): the gradient of a 1x1 / stride-2 / pad-0 downsample conv of the same
// input (dy [B, Cout, OH, OW], weight [Cout, C, 1, 1], bf16 scratch for its transpose) accumulated into dx
// in the same pass (extra K stages of the even-pixel phase) instead of a second dgrad + residual add
// wt_ready: wt (and ds_wt) already hold the transposed weights (conv_wtrans_batch), no transpose here
// rows of BN-backward partials conv_dgrad(..., bn_x=...) writes (0: not available for this conv)
int64_t conv_dgrad_bn_rows(const at::Tensor& dx, const at::Tensor& w, int64_t stride, int64_t pad) {
  const ConvGeom g = conv_geom(dx, w, stride, pad);
  return pde_conv_dgrad_bnb_rows((int)g.Bn, (int)g.H, (int)g.W, (int)g.C, (int)g.N, (int)g.R, (int)g.S, (int)stride,
                                 (int)pad);
}

// bn_x / bn_scale / bn_shift / bn_mean / bn_rstd / bn_part (optional, stride 1): dx is the gradient of
// relu(bn(bn_x)); the epilogue also sums that BN's backward partials (sum d, sum d * xhat) into
// bn_part [bn_part_rows(conv_dgrad_bn_rows)][2][C], consumed by bn_bwd(..., pre_nblk=rows)
void conv_dgrad(const at::Tensor& dy, const at::Tensor& w, const at::Tensor& wt, const at::Tensor& dx,
                int64_t stride, int64_t pad, const OptT& res, const OptT& ds_dy, const OptT& ds_w, const OptT& ds_wt,
                bool wt_ready, const OptT& bn_x, const OptT& bn_scale, const OptT& bn_shift, const OptT& bn_mean,
                const OptT& bn_rstd, const OptT& bn_part) {
  const ConvGeom g = conv_geom(dx, w, stride, pad);
  const void* bx = nullptr;
  const float *bsc = nullptr, *bsh = nullptr, *bmu = nullptr, *brs = nullptr;
  float* bpart = nullptr;
  if (bn_x.has_value() && bn_x->defined()) {
    check_same(dx, *bn_x, "bn_x");
    const int64_t rows = conv_dgrad_bn_rows(dx, w, stride, pad);
    TORCH_CHECK(rows > 0, "conv dgrad: fused BN-backward partials need a stride-1 convolution");
    bsc = optr<float>(bn_scale, "bn_scale", F32, g.C);
    bsh = optr<float>(bn_shift, "bn_shift", F32, g.C);
    bmu = optr<float>(bn_mean, "bn_mean", F32, g.C);
    brs = optr<float>(bn_rstd, "bn_rstd", F32, g.C);
    bpart = optr<float>(bn_part, "bn_part", F32, pde_bn_part_rows((int)rows) * 2 * g.C);
    TORCH_CHECK(bsc && bsh && bmu && brs && bpart, "conv dgrad: bn_x needs bn_scale / shift / mean / rstd / part");
    TORCH_CHECK(!(ds_dy.has_value() && ds_dy->defined()) && !(res.has_value() && res->defined()),
                "conv dgrad: bn_x excludes a downsample source and a residual");
    bx = bn_x->data_ptr();
  }
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == BF16 && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  dy.size(0) == g.Bn && dy.size(1) == g.N && dy.size(2) == g.OH && dy.size(3) == g.OW,
              "conv dgrad: dy must be channels-last bf16 [B, Cout, OH, OW]");
  check_cuda(wt, "wt", BF16, g.N * g.C * g.R * g.S);
  if (!wt_ready)
    hip_check(pde_conv_wtrans(w.data_ptr(), wt.data_ptr(), (int)g.N, (int)(g.R * g.S), (int)g.C, cur_stream()),
              "conv_wtrans");
  const void* rp = nullptr;
  if (res.has_value() && res->defined()) {
    TORCH_CHECK(res->is_cuda() && res->scalar_type() == BF16 && res->is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    res->sizes() == dx.sizes(),
                "conv dgrad: res must be a channels-last bf16 tensor shaped like dx");
    rp = res->data_ptr();
  }
  const void* dy2 = nullptr;
  const void* wt2 = nullptr;
  if (ds_dy.has_value() && ds_dy->defined()) {
    TORCH_CHECK(ds_w.has_value() && ds_wt.has_value(), "conv dgrad: ds_dy needs ds_w and ds_wt");
    TORCH_CHECK(stride == 2, "conv dgrad: the downsample source needs a stride-2 convolution");
    TORCH_CHECK(ds_dy->is_cuda() && ds_dy->scalar_type() == BF16 &&
                    ds_dy->is_contiguous(at::MemoryFormat::ChannelsLast) && ds_dy->sizes() == dy.sizes(),
                "conv dgrad: ds_dy must be a channels-last bf16 tensor shaped like dy");
    TORCH_CHECK(g.OH == (g.H - 1) / 2 + 1 && g.OW == (g.W - 1) / 2 + 1,
                "conv dgrad: the downsample (1x1 / s2 / p0) output must match this convolution's output");
    const at::Tensor& w2 = *ds_w;
    TORCH_CHECK(w2.is_cuda() && w2.scalar_type() == BF16 && w2.dim() == 4 && w2.size(0) == g.N && w2.size(1) == g.C &&
                    w2.size(2) == 1 && w2.size(3) == 1 && w2.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv dgrad: ds_w must be a channels-last bf16 [Cout, C, 1, 1] weight");
    check_cuda(*ds_wt, "ds_wt", BF16, g.N * g.C);
    if (!wt_ready)
      hip_check(pde_conv_wtrans(w2.data_ptr(), ds_wt->data_ptr(), (int)g.N, 1, (int)g.C, cur_stream()),
                "conv_wtrans (downsample)");
    dy2 = ds_dy->data_ptr();
    wt2 = ds_wt->data_ptr();
  }
  hip_check(pde_conv_dgrad(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), rp, dy2, wt2, (int)g.Bn, (int)g.H, (int)g.W,
                           (int)g.C, (int)g.N, (int)g.R, (int)g.S, (int)stride, (int)pad, (int)g.OH, (int)g.OW, bx,
                           bsc, bsh, bmu, brs, bpart, cur_stream()),
            "conv_dgrad");
}

// desc: int64 GPU tensor [nconv][4] = (w ptr, wt ptr, N | T << 32, C | tile0 << 32), the WtDesc table
void conv_wtrans_batch(const at::Tensor& desc, int64_t total, const OptT& counters) {
  TORCH_CHECK(pde_conv_wtdesc_bytes() == 32, "conv_wtrans_batch: descriptor layout mismatch");
  TORCH_CHECK(desc.is_cuda() && desc.scalar_type() == at::kLong && desc.is_contiguous() && desc.dim() == 2 &&
                  desc.size(1) == 4,
              "conv_wtrans_batch: desc must be a contiguous int64 GPU tensor [nconv, 4]");
  long long* ctr = nullptr;
  int ncnt = 0;
  if (counters.has_value()) {
    const at::Tensor& c = *counters;
    TORCH_CHECK(c.is_cuda() && c.scalar_type() == at::kLong && c.is_contiguous() && c.numel() <= 256,
                "conv_wtrans_batch: counters must be a contiguous int64 GPU tensor of <= 256 elements");
    ctr = reinterpret_cast<long long*>(c.data_ptr());
    ncnt = (int)c.numel();
  }
  hip_check(pde_conv_wtrans_batch(desc.data_ptr(), (int)desc.size(0), (int)total, ctr, ncnt, cur_stream()),
            "conv_wtrans_batch");
}

int64_t conv_wgrad_splits(const at::Tensor& x, const at::Tensor& w, int64_t stride, int64_t pad) {
  const ConvGeom g = conv_geom(x, w, stride, pad);
  return pde_conv_wgrad_splits2((int)g.Bn, (int)g.H, (int)g.W, (int)g.C, (int)g.N, (int)g.R, (int)g.S, (int)stride,
                                (int)pad, (int)g.OH, (int)g.OW);
}

void conv_wgrad(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w, const at::Tensor& part,
                int64_t splits, const at::Tensor& dw, int64_t stride, int64_t pad) {
  const ConvGeom g = conv_geom(x, w, stride, pad);
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == BF16 && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  dy.size(0) == g.Bn && dy.size(1) == g.N && dy.size(2) == g.OH && dy.size(3) == g.OW,
              "conv wgrad: dy must be channels-last bf16 [B, Cout, OH, OW]");
  TORCH_CHECK(dw.is_cuda() && dw.scalar_type() == BF16 && dw.sizes() == w.sizes() &&
                  dw.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv wgrad: dw must be a channels-last bf16 tensor shaped like the weight");
  check_cuda(part, "part", F32, splits * g.N * g.R * g.S * g.C);
  hip_check(pde_conv_wgrad(dy.data_ptr(), x.data_ptr(), ptr<float>(part), (int)splits, dw.data_ptr(), (int)g.Bn,
                           (int)g.H, (int)g.W, (int)g.C, (int)g.N, (int)g.R, (int)g.S, (int)stride, (int)pad,
                           (int)g.OH, (int)g.OW, cur_stream()),
            "conv_wgrad");
}

int64_t stem_stats_blocks(int64_t Bn, int64_t OH) { return pde_stem_stats_blocks((int)Bn, (int)OH); }

// ResNet stem: y = conv7x7/s2/p3(x, w) with x NHWC bf16 [B, 3, H, W], w channels-last [64, 3, 7, 7];
// wp: bf16 scratch >= 64*224 (packed weights); stats: optional BN partials [stem_stats_blocks][2][64]
void stem_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& wp, const at::Tensor& y,
              const OptT& stats) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == BF16 && x.dim() == 4 && x.size(1) == 3 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem: x must be channels-last bf16 [B, 3, H, W]");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == BF16 && w.size(0) == 64 && w.size(1) == 3 && w.size(2) == 7 &&
                  w.size(3) == 7 && w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem: w must be channels-last bf16 [64, 3, 7, 7]");
  const int64_t Bn = x.size(0), H = x.size(2), W = x.size(3), OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(OW <= 112, "stem: input width must be <= 224");
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == BF16 && y.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  y.size(0) == Bn && y.size(1) == 64 && y.size(2) == OH && y.size(3) == OW,
              "stem: y must be channels-last bf16 [B, 64, OH, OW]");
  TORCH_CHECK(Bn * std::max(H * W * 3, OH * OW * 64) * 2 < (int64_t(1) << 31), "stem: tensors must be < 2 GiB");
  check_cuda(wp, "wp", BF16, 64 * 224);
  float* sp = optr<float>(stats, "stats", F32, stem_stats_blocks(Bn, OH) * 2 * 64);
  hip_check(pde_stem_fwd(x.data_ptr(), w.data_ptr(), wp.data_ptr(), y.data_ptr(), sp, (int)Bn, (int)H, (int)W,
                         cur_stream()),
            "stem_fwd");
}

int64_t stem_wgrad_blocks(int64_t Bn, int64_t OH) { return pde_stem_wgrad_blocks((int)Bn, (int)OH); }

// dW (bf16, channels-last [64, 3, 7, 7]) of the stem from x and dy; part: fp32 scratch
// >= stem_wgrad_blocks(B, OH) * 64 * 147
void stem_wgrad(const at::Tensor& x, const at::Tensor& dy, const at::Tensor& part, const at::Tensor& dw) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == BF16 && x.dim() == 4 && x.size(1) == 3 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem wgrad: x must be channels-last bf16 [B, 3, H, W]");
  const int64_t Bn = x.size(0), H = x.size(2), W = x.size(3), OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(OW <= 112, "stem: input width must be <= 224");
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == BF16 && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  dy.size(0) == Bn && dy.size(1) == 64 && dy.size(2) == OH && dy.size(3) == OW,
              "stem wgrad: dy must be channels-last bf16 [B, 64, OH, OW]");
  TORCH_CHECK(dw.is_cuda() && dw.scalar_type() == BF16 && dw.numel() == 64 * 147 &&
                  dw.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem wgrad: dw must be channels-last bf16 [64, 3, 7, 7]");
  check_cuda(part, "part", F32, stem_wgrad_blocks(Bn, OH) * 64 * 147);
  hip_check(pde_stem_wgrad(x.data_ptr(), dy.data_ptr(), ptr<float>(part), dw.data_ptr(), (int)Bn, (int)H, (int)W,
                           cur_stream()),
            "stem_wgrad");
}

}  // namespace

void register_resnet(pybind11::module& m) {
  m.def("bn_blocks", &bn_blocks);
  m.def("bn_fwd", &bn_fwd, py::arg("x"), py::arg("res"), py::arg("y"), py::arg("gamma"), py::arg("beta"), py::arg("eps"),
        py::arg("momentum"), py::arg("run_mean"), py::arg("run_var"), py::arg("part"), py::arg("mean"), py::arg("rstd"),
        py::arg("scale"), py::arg("shift"), py::arg("relu"), py::arg("training"), py::arg("pre_nblk"),
        py::arg("res_scale") = py::none(), py::arg("res_shift") = py::none());
  m.def("bn_bwd", &bn_bwd, py::arg("dy"), py::arg("y"), py::arg("x"), py::arg("gamma"), py::arg("mean"),
        py::arg("rstd"), py::arg("part"), py::arg("coef"), py::arg("dgamma"), py::arg("dbeta"), py::arg("dx"),
        py::arg("dres"), py::arg("relu"), py::arg("scale") = py::none(), py::arg("shift") = py::none(),
        py::arg("pre_nblk") = 0);
  m.def("sgd_master", &sgd_master);
  m.def("maxpool3s2_fwd", &maxpool3s2_fwd);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("maxpool3s2_bwd", &maxpool3s2_bwd);
  m.def("bnpool_part_floats", &bnpool_part_floats);
  m.def("bnpool_fwd", &bnpool_fwd);
  m.def("bnpool_bwd", &bnpool_bwd);
  m.def("conv_stats_blocks", &conv_stats_blocks);
  m.def("conv_stats_rows", &conv_stats_rows);
  m.def("stem_stats_blocks", &stem_stats_blocks);
  m.def("stem_fwd", &stem_fwd);
  m.def("stem_wgrad_blocks", &stem_wgrad_blocks);
  m.def("stem_wgrad", &stem_wgrad);
  m.def("bn_part_rows", &bn_part_rows);
  m.def("conv_set_stages", [](int64_t n) { pde_conv_set_stages((int)n); });
  m.def("conv_fprop", &conv_fprop);
  m.def("conv_dgrad", &conv_dgrad, py::arg("dy"), py::arg("w"), py::arg("wt"), py::arg("dx"), py::arg("stride"),
        py::arg("pad"), py::arg("res") = py::none(), py::arg("ds_dy") = py::none(), py::arg("ds_w") = py::none(),
        py::arg("ds_wt") = py::none(), py::arg("wt_ready") = false, py::arg("bn_x") = py::none(),
        py::arg("bn_scale") = py::none(), py::arg("bn_shift") = py::none(), py::arg("bn_mean") = py::none(),
        py::arg("bn_rstd") = py::none(), py::arg("bn_part") = py::none());
  m.def("conv_dgrad_bn_rows", &conv_dgrad_bn_rows);
  m.def("conv_wtrans_batch", &conv_wtrans_batch, py::arg("desc"), py::arg("total"), py::arg("counters") = py::none());
  m.def("conv_wgrad_splits", &conv_wgrad_splits);
  m.def("conv_wgrad", &conv_wgrad);
}

}  // namespace pde
