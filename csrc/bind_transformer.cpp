// torch bindings of the transformer kernels (csrc/kernels/transformer.hip, attention.hip).
// Every entry validates device / dtype / contiguity / shape before launching on the current stream.
#include "pde_bind.h"
#include "pde_kernels.h"

namespace pde {
namespace {

void ln_fwd(const at::Tensor& X, const at::Tensor& G, const at::Tensor& B, const at::Tensor& Y,
            const at::Tensor& mean, const at::Tensor& rstd, double eps, const OptT& D, const OptT& S) {
  const int64_t C = X.size(-1), N = X.numel() / C;
  TORCH_CHECK(C % 4 == 0 && C <= 2048, "ln: C must be a multiple of 4 and <= 2048");
  check_cuda(X, "X", BF16);
  check_cuda(G, "gamma", BF16, C);
  check_cuda(B, "beta", BF16, C);
  check_cuda(Y, "Y", BF16, N * C);
  check_cuda(mean, "mean", F32, N);
  check_cuda(rstd, "rstd", F32, N);
  const void* dp = optr<void>(D, "D", BF16, N * C);
  void* sp = optr<void>(S, "S", BF16, N * C);
  TORCH_CHECK((dp == nullptr) == (sp == nullptr), "ln_fwd: D (residual input) and S (sum output) go together");
  hip_check(pde_ln_fwd(X.data_ptr(), dp, sp, G.data_ptr(), B.data_ptr(), Y.data_ptr(), ptr<float>(mean), ptr<float>(rstd),
                       (int)N, (int)C, (float)eps, cur_stream()),
            "ln_fwd");
}

int64_t ln_bwd_blocks(int64_t N) { return pde_ln_bwd_blocks((int)N); }

void ln_bwd(const at::Tensor& dY, const at::Tensor& X, const at::Tensor& mean, const at::Tensor& rstd,
            const at::Tensor& G, const OptT& dRes, const at::Tensor& dX, const at::Tensor& part, const at::Tensor& dG,
            const at::Tensor& dB, bool accumulate) {
  const int64_t C = X.size(-1), N = X.numel() / C;
  TORCH_CHECK(C % 4 == 0 && C <= 2048, "ln: C must be a multiple of 4 and <= 2048");
  check_cuda(dY, "dY", BF16, N * C);
  check_cuda(X, "X", BF16);
  check_cuda(mean, "mean", F32, N);
  check_cuda(rstd, "rstd", F32, N);
  check_cuda(G, "gamma", BF16, C);
  check_cuda(dX, "dX", BF16, N * C);
  check_cuda(part, "part", F32, (int64_t)pde_ln_bwd_blocks((int)N) * 2 * C);
  check_cuda(dG, "dgamma", BF16, C);
  check_cuda(dB, "dbeta", BF16, C);
  const void* dr = optr<at::BFloat16>(dRes, "dRes", BF16, N * C);
  hip_check(pde_ln_bwd(dY.data_ptr(), X.data_ptr(), ptr<float>(mean), ptr<float>(rstd), G.data_ptr(), dr,
                       dX.data_ptr(), ptr<float>(part), dG.data_ptr(), dB.data_ptr(), (int)N, (int)C, accumulate,
                       cur_stream()),
            "ln_bwd");
}

// out (bf16, contiguous) = sum of the S fp32 slabs of part ([S, *out.shape]) -- split-K reduction
void sum_slabs_bf16(const at::Tensor& part, const at::Tensor& out) {
  const int64_t n = out.numel();
  check_cuda(out, "out", BF16);
  check_cuda(part, "part", F32);
  TORCH_CHECK(n % 4 == 0 && part.numel() % n == 0, "sum_slabs_bf16: part must hold S x out.numel() floats");
  hip_check(pde_sum_slabs_bf16(ptr<float>(part), (int)(part.numel() / n), n, out.data_ptr(), cur_stream()),
            "sum_slabs_bf16");
}

void gelu_fwd(const at::Tensor& X, const at::Tensor& Y) {
  check_cuda(X, "X", BF16);
  check_cuda(Y, "Y", BF16, X.numel());
  TORCH_CHECK(X.numel() % 8 == 0, "gelu: numel must be a multiple of 8");
  hip_check(pde_gelu_fwd(X.data_ptr(), Y.data_ptr(), X.numel(), cur_stream()), "gelu_fwd");
}

void gelu_bwd(const at::Tensor& dY, const at::Tensor& X, const at::Tensor& dX) {
  check_cuda(X, "X", BF16);
  check_cuda(dY, "dY", BF16, X.numel());
  check_cuda(dX, "dX", BF16, X.numel());
  TORCH_CHECK(X.numel() % 8 == 0, "gelu: numel must be a multiple of 8");
  hip_check(pde_gelu_bwd(dY.data_ptr(), X.data_ptr(), dX.data_ptr(), X.numel(), cur_stream()), "gelu_bwd");
}

void xent_bf16(const at::Tensor& logits, const at::Tensor& tgt, int64_t V, double scale, const at::Tensor& loss_rows,
               bool write_grad) {
  check_cuda(logits, "logits", BF16);
  TORCH_CHECK(logits.dim() == 2 && logits.size(1) % 8 == 0, "logits must be [N, Vp] with Vp % 8 == 0");
  const int64_t N = logits.size(0), Vp = logits.size(1);
  TORCH_CHECK(V <= Vp, "V > padded vocab");
  check_cuda(tgt, "targets", I64, N);
  check_cuda(loss_rows, "loss_rows", F32, N);
  hip_check(pde_xent_bf16(logits.data_ptr(), ptr<int64_t>(tgt), (int)N, (int)Vp, (int)V, (float)scale,
                          ptr<float>(loss_rows), write_grad, cur_stream()),
            "xent_bf16");
}

void embed_fwd(const at::Tensor& idx, const at::Tensor& wte, const at::Tensor& wpe, const at::Tensor& out, int64_t T) {
  check_cuda(idx, "idx", I64);
  const int64_t N = idx.numel(), C = wte.size(1);
  TORCH_CHECK(C % 4 == 0 && N % T == 0 && wpe.size(0) >= T, "embed: bad shapes");
  check_cuda(wte, "wte", BF16);
  check_cuda(wpe, "wpe", BF16);
  check_cuda(out, "out", BF16, N * C);
  hip_check(pde_embed_fwd(ptr<int64_t>(idx), wte.data_ptr(), wpe.data_ptr(), out.data_ptr(), (int)N, (int)T, (int)C,
                          cur_stream()),
            "embed_fwd");
}

void embed_bwd(const at::Tensor& dX, const at::Tensor& idx, const at::Tensor& dwte, const at::Tensor& dwpe,
               const at::Tensor& acc, const at::Tensor& touched, int64_t T, bool accumulate_pos) {
  check_cuda(idx, "idx", I64);
  const int64_t N = idx.numel(), C = dwte.size(1), Vp = dwte.size(0);
  check_cuda(dX, "dX", BF16, N * C);
  check_cuda(dwte, "dwte", BF16);
  check_cuda(dwpe, "dwpe", BF16, T * C);
  check_cuda(acc, "acc", F32, Vp * C);
  check_cuda(touched, "touched", U8, Vp);
  hip_check(pde_embed_bwd(dX.data_ptr(), ptr<int64_t>(idx), dwte.data_ptr(), dwpe.data_ptr(), ptr<float>(acc),
                          ptr<uint8_t>(touched), (int)N, (int)T, (int)C, (int)Vp, accumulate_pos, cur_stream()),
            "embed_bwd");
}

void sumsq_bf16(const at::Tensor& g, double scale, const at::Tensor& out, const OptT& step_inc) {
  check_cuda(g, "g", BF16);
  check_cuda(out, "out", F32, 1025);      // [0] result, [1..1024] per-block partials
  TORCH_CHECK(g.numel() % 8 == 0 && reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 == 0,
              "sumsq: numel % 8 and a 16-byte aligned buffer");
  hip_check(pde_sumsq_bf16(g.data_ptr(), g.numel(), (float)scale, ptr<float>(out),
                           optr<float>(step_inc, "step_inc", F32, 1), cur_stream()),
            "sumsq_bf16");
}

void adamw_master(const at::Tensor& master, const at::Tensor& p16, const at::Tensor& g16, const at::Tensor& m,
                  const at::Tensor& v, double lr, double b1, double b2, double eps, double wd, double grad_scale,
                  int64_t step, const OptT& decay_blk, const OptT& clip_sumsq, double max_norm, const OptT& step_dev) {
  const int64_t n = master.numel();
  TORCH_CHECK(n % 64 == 0, "adamw_master: flat buffers are padded to 64 elements");
  check_cuda(master, "master", F32);
  check_cuda(p16, "param_bf16", BF16, n);
  check_cuda(g16, "grad_bf16", BF16, n);
  check_cuda(m, "exp_avg", F32, n);
  check_cuda(v, "exp_avg_sq", F32, n);
  const uint8_t* db = optr<uint8_t>(decay_blk, "decay_blk", U8, n / 64);
  const float* cs = optr<float>(clip_sumsq, "clip_sumsq", F32, 1);
  const float* sd = optr<float>(step_dev, "step_dev", F32, 1);
  hip_check(pde_adamw_master(ptr<float>(master), p16.data_ptr(), g16.data_ptr(), ptr<float>(m), ptr<float>(v), n,
                             (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (float)grad_scale, (int)step, db,
                             cs, (float)max_norm, sd, cur_stream()),
            "adamw_master");
}

void f32_to_bf16(const at::Tensor& x, const at::Tensor& y) {
  check_cuda(x, "x", F32);
  check_cuda(y, "y", BF16, x.numel());
  TORCH_CHECK(x.numel() % 4 == 0, "numel % 4");
  hip_check(pde_f32_to_bf16(ptr<float>(x), y.data_ptr(), x.numel(), cur_stream()), "f32_to_bf16");
}

void scale_bf16(const at::Tensor& x, const at::Tensor& s) {
  check_cuda(x, "x", BF16);
  check_cuda(s, "s", F32, 1);
  TORCH_CHECK(x.numel() % 8 == 0, "scale_bf16: numel % 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "scale_bf16: x must be 16-byte aligned (uint4 accesses)");
  hip_check(pde_scale_bf16(x.data_ptr(), ptr<float>(s), x.numel(), cur_stream()), "scale_bf16");
}

int64_t colsum_bf16_splits(int64_t C) { return pde_colsum_bf16_splits((int)C); }

void colsum_bf16(const at::Tensor& x, const at::Tensor& part, const at::Tensor& out) {
  check_cuda(x, "x", BF16);
  const int64_t C = x.size(-1), N = x.numel() / C;
  TORCH_CHECK(C % 8 == 0, "colsum_bf16: C % 8");
  check_cuda(part, "part", F32, (int64_t)pde_colsum_bf16_splits((int)C) * C);
  check_cuda(out, "out", BF16, C);
  hip_check(pde_colsum_bf16(x.data_ptr(), (int)N, (int)C, ptr<float>(part), out.data_ptr(), cur_stream()),
            "colsum_bf16");
}

void sum_f32(const at::Tensor& x, const at::Tensor& out, double scale) {
  check_cuda(x, "x", F32);
  check_cuda(out, "out", F32, 1);
  hip_check(pde_sum_f32(ptr<float>(x), (int)x.numel(), ptr<float>(out), (float)scale, cur_stream()), "sum_f32");
}

void token_batch(const at::Tensor& pool, const at::Tensor& rows, const at::Tensor& x, const at::Tensor& y) {
  check_cuda(pool, "pool", I64);
  check_cuda(rows, "rows", I64);
  TORCH_CHECK(pool.dim() == 2 && pool.size(1) >= 2, "token_batch: pool must be [P, T+1]");
  const int64_t B = rows.numel(), T = pool.size(1) - 1;
  check_cuda(x, "x", I64, B * T);
  check_cuda(y, "y", I64, B * T);
  hip_check(pde_token_batch(ptr<int64_t>(pool), ptr<int64_t>(rows), (int)B, (int)T, ptr<int64_t>(x), ptr<int64_t>(y),
                            cur_stream()),
            "token_batch");
}

// q/k/v: views into a [B, T, ld] bf16 buffer (column offset = section start); o: [B, T, H*64]
void check_qkv(const at::Tensor& t, const char* name, int64_t B, int64_t T, int64_t H) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == BF16, name, " must be a bf16 GPU tensor");
  TORCH_CHECK(t.dim() == 3 && t.size(0) == B && t.size(1) == T && t.size(2) == H * 64, name, " must be [B, T, H*64]");
  TORCH_CHECK(t.stride(2) == 1 && t.stride(1) >= H * 64 && t.stride(0) == T * t.stride(1), name,
              " must have unit inner stride and packed rows");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0 && t.stride(1) % 8 == 0, name,
              " must be 16-byte aligned");
}

void attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const at::Tensor& o,
              const at::Tensor& lse, int64_t H, double scale) {
  const int64_t B = q.size(0), T = q.size(1);
  TORCH_CHECK(T % 128 == 0, "attention: T must be a multiple of 128");
  check_qkv(q, "q", B, T, H);
  check_qkv(k, "k", B, T, H);
  check_qkv(v, "v", B, T, H);
  TORCH_CHECK(k.stride(1) == q.stride(1) && v.stride(1) == q.stride(1), "q/k/v must share the row stride");
  check_qkv(o, "o", B, T, H);
  check_cuda(lse, "lse", F32, B * H * T);
  hip_check(pde_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), (int)q.stride(1), o.data_ptr(), (int)o.stride(1),
                         ptr<float>(lse), (int)B, (int)T, (int)H, (float)scale, cur_stream()),
            "attn_fwd");
}

void attn_bwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const at::Tensor& o,
              const at::Tensor& dout, const at::Tensor& lse, const at::Tensor& Dd, const at::Tensor& dq,
              const at::Tensor& dk, const at::Tensor& dv, int64_t H, double scale) {
  const int64_t B = q.size(0), T = q.size(1);
  TORCH_CHECK(T % 128 == 0, "attention: T must be a multiple of 128");
  for (auto* p : {&q, &k, &v, &dq, &dk, &dv}) check_qkv(*p, "q/k/v/dq/dk/dv", B, T, H);
  for (auto* p : {&k, &v, &dq, &dk, &dv})
    TORCH_CHECK(p->stride(1) == q.stride(1), "q/k/v and dq/dk/dv must share the row stride");
  check_qkv(o, "o", B, T, H);
  check_qkv(dout, "dout", B, T, H);
  TORCH_CHECK(dout.stride(1) == o.stride(1), "o / dout row strides differ");
  check_cuda(lse, "lse", F32, B * H * T);
  check_cuda(Dd, "D", F32, B * H * T);
  hip_check(pde_attn_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), (int)q.stride(1), o.data_ptr(), dout.data_ptr(),
                         (int)o.stride(1), ptr<float>(lse), ptr<float>(Dd), dq.data_ptr(), dk.data_ptr(),
                         dv.data_ptr(), (int)B, (int)T, (int)H, (float)scale, cur_stream()),
            "attn_bwd");
}

// ---- own GEMM (gemm.hip).  Operand conventions: C[m][n] = sum_k A(m,k) B(k,n) with
// A(m,k) = A[m*lda+k] (ta=0) or A[k*lda+m] (ta=1), B(k,n) = B[n*ldb+k] (tb=0) or B[k*ldb+n] (tb=1).
void gemm(const at::Tensor& A, const at::Tensor& B, const at::Tensor& C, int64_t ta, int64_t tb, int64_t epi,
          int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int64_t splits, int64_t cfg,
          const OptT& C2, const OptT& bias, const OptT& aux, const OptT& colsum, const OptT& scale) {
  check_cuda(A, "A", BF16, (ta ? K : M - 1) * lda + (ta ? 0 : K));
  check_cuda(B, "B", BF16, (tb ? K : N - 1) * ldb + (tb ? 0 : K));
  TORCH_CHECK(ta ? lda >= M : lda >= K, "gemm: lda too small");
  TORCH_CHECK(tb ? ldb >= N : ldb >= K, "gemm: ldb too small");
  TORCH_CHECK(ldc >= N, "gemm: ldc too small");
  const int S = pde_gemm_splits((int)K, (int)splits);
  if (epi == 3) check_cuda(C, "C", F32, (int64_t)S * M * ldc);
  else check_cuda(C, "C", BF16, (M - 1) * ldc + N);
  void* c2 = optr<void>(C2, "C2", BF16, (M - 1) * ldc + N);
  const void* bp = optr<void>(bias, "bias", BF16, N);
  const void* xp = optr<void>(aux, "aux", BF16, (M - 1) * ldc + N);
  float* cs = optr<float>(colsum, "colsum", F32, (int64_t)S * M);
  TORCH_CHECK(epi != 1 || c2 != nullptr, "gemm: the GELU epilogue needs C2 (activation output)");
  TORCH_CHECK(epi != 2 || xp != nullptr, "gemm: the GELU-backward epilogue needs aux (pre-activation)");
  const float* sp = optr<float>(scale, "scale", F32, 1);
  TORCH_CHECK(sp == nullptr || epi == 0, "gemm: a device scale needs the plain bf16 epilogue");
  hip_check(pde_gemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), c2, bp, xp, cs, (int)ta, (int)tb, (int)epi, (int)M,
                     (int)N, (int)K, (int)lda, (int)ldb, (int)ldc, (int)splits, (int)cfg, sp, cur_stream()),
            "gemm");
}

// dw = sum of the S fp32 slabs of part; db = sum of the S bias-gradient partials cs (part / dw may
// be None: db only)
void gemm_reduce(const OptT& part, int64_t S, int64_t M, int64_t N, const OptT& dw, const OptT& cs,
                 const OptT& db, const OptT& scale) {
  const float* p = optr<float>(part, "part", F32, S * M * N);
  void* w = optr<void>(dw, "dw", BF16, M * N);
  const float* c = optr<float>(cs, "cs", F32, S * M);
  void* d = optr<void>(db, "db", BF16, M);
  hip_check(pde_gemm_reduce(p, (int)S, (int)M, (int)N, w, c, d, optr<float>(scale, "scale", F32, 1), cur_stream()),
            "gemm_reduce");
}

std::vector<int64_t> gemm_tile(int64_t cfg) {
  int bm = 0, bn = 0;
  pde_gemm_tile((int)cfg, &bm, &bn);
  return {bm, bn};
}

int64_t gemm_splits(int64_t K, int64_t splits) { return pde_gemm_splits((int)K, (int)splits); }
int64_t gemm_num_cfgs() { return pde_gemm_num_cfgs(); }

}  // namespace

void register_transformer(pybind11::module& m) {
  namespace py = pybind11;
  m.def("ln_fwd", &ln_fwd, py::arg("X"), py::arg("G"), py::arg("B"), py::arg("Y"), py::arg("mean"), py::arg("rstd"),
        py::arg("eps"), py::arg("D") = py::none(), py::arg("S") = py::none());
  m.def("ln_bwd_blocks", &ln_bwd_blocks);
  m.def("ln_bwd", &ln_bwd);
  m.def("sum_slabs_bf16", &sum_slabs_bf16);
  m.def("gemm_bf16", &gemm, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("ta"), py::arg("tb"), py::arg("epi"),
        py::arg("M"), py::arg("N"), py::arg("K"), py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("splits") = 1,
        py::arg("cfg") = 0, py::arg("C2") = py::none(), py::arg("bias") = py::none(), py::arg("aux") = py::none(),
        py::arg("colsum") = py::none(), py::arg("scale") = py::none());
  m.def("gemm_reduce", &gemm_reduce, py::arg("part"), py::arg("S"), py::arg("M"), py::arg("N"), py::arg("dw"),
        py::arg("cs") = py::none(), py::arg("db") = py::none(), py::arg("scale") = py::none());
  m.def("gemm_tile", &gemm_tile);
  m.def("gemm_splits", &gemm_splits);
  m.def("gemm_num_cfgs", &gemm_num_cfgs);
  m.def("gemm_set_dbg", [](int64_t d) { pde_gemm_set_dbg((int)d); });
  m.def("gelu_fwd", &gelu_fwd);
  m.def("gelu_bwd", &gelu_bwd);
  m.def("xent_bf16", &xent_bf16);
  m.def("embed_fwd", &embed_fwd);
  m.def("embed_bwd", &embed_bwd);
  m.def("sumsq_bf16", &sumsq_bf16, py::arg("g"), py::arg("scale"), py::arg("out"), py::arg("step_inc") = py::none());
  m.def("adamw_master", &adamw_master, py::arg("master"), py::arg("p16"), py::arg("g16"), py::arg("m"), py::arg("v"),
        py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("grad_scale"),
        py::arg("step"), py::arg("decay_blk") = py::none(), py::arg("clip_sumsq") = py::none(),
        py::arg("max_norm") = 1.0, py::arg("step_dev") = py::none());
  m.def("f32_to_bf16", &f32_to_bf16);
  m.def("scale_bf16", &scale_bf16);
  m.def("sum_f32", &sum_f32, py::arg("x"), py::arg("out"), py::arg("scale") = 1.0);
  m.def("token_batch", &token_batch);
  m.def("colsum_bf16_splits", &colsum_bf16_splits);
  m.def("colsum_bf16", &colsum_bf16);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd);
  m.def("attn_set_variant", [](int64_t v) { pde_attn_set_variant((int)v); });
}

}  // namespace pde
