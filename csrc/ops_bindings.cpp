// torch <-> HIP kernel binding layer for the `_kernels` extension.
//
// Every function takes preallocated tensors (the Python engine owns all workspaces so the whole
// training step is capturable in a hipGraph), validates device / dtype / contiguity / size, and
// launches on the caller's current HIP stream.  Device code lives in csrc/kernels/*.hip and is
// reached through the extern "C" launchers of pde_kernels.h.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPGuard.h>

#include <cmath>
#include <cstring>
#include <optional>

#include "pde_kernels.h"
#include "pde_lenet.h"
#include "pde_bind.h"
#include "pde_peer.h"

namespace {

using OptT = std::optional<at::Tensor>;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_cuda(const at::Tensor& t, const char* name, at::ScalarType dt, int64_t min_numel = 0) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.numel() >= min_numel, name, " has ", t.numel(), " elements, needs >= ", min_numel);
}

template <typename T>
T* ptr(const at::Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }

template <typename T>
T* optr(const OptT& t, const char* name, at::ScalarType dt, int64_t min_numel = 0) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_cuda(*t, name, dt, min_numel);
  return ptr<T>(*t);
}

void hip_check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, " failed: ", hipGetErrorString(e));
}

constexpr auto F32 = at::kFloat;
constexpr auto I32 = at::kInt;
constexpr auto I64 = at::kLong;
constexpr auto U8 = at::kByte;
constexpr auto F64 = at::kDouble;

// ------------------------------------------------------------------------------------------------
void lenet_conv_fwd(const at::Tensor& X, const OptT& idx, const OptT& step, int64_t nbatches, int64_t stride,
                    const OptT& labels_all, int64_t B, const at::Tensor& w1, const at::Tensor& b1, const at::Tensor& Wt2,
                    const at::Tensor& b2, const at::Tensor& P1, const at::Tensor& A1, const at::Tensor& P2,
                    const at::Tensor& A2, const OptT& cur_row, const OptT& cur_lbl, const OptT& zero, int64_t dbg) {
  TORCH_CHECK(B >= 1, "batch must be >= 1");
  check_cuda(X, "X", F32);
  TORCH_CHECK(X.numel() % 784 == 0, "X must be [N,1,28,28]");
  if (!idx.has_value()) TORCH_CHECK(X.numel() >= B * 784, "X smaller than batch");
  check_cuda(w1, "conv1.weight", F32, 500);
  check_cuda(b1, "conv1.bias", F32, 20);
  check_cuda(Wt2, "Wt2", F32, 500 * 64);
  check_cuda(b2, "conv2.bias", F32, 50);
  check_cuda(P1, "P1", F32, B * 2880);
  check_cuda(A1, "A1", U8, B * 2880);
  check_cuda(P2, "P2", F32, B * 800);
  check_cuda(A2, "A2", U8, B * 800);
  const int* ip = optr<int>(idx, "idx", I32, step.has_value() ? 1 : B);
  const long long* sp = optr<long long>(step, "step", I64, 1);
  const int64_t st = stride > 0 ? stride : B;
  if (sp) TORCH_CHECK(ip && nbatches >= 1, "step-indexed batches need idx");
  float* zp = optr<float>(zero, "zero", F32);
  hip_check(pde_lenet_conv_fwd(ptr<float>(X), ip, ip ? (int)idx->numel() : 0, sp, (int)nbatches, (int)st,
                               optr<long long>(labels_all, "labels", I64), (int)B, ptr<float>(w1), ptr<float>(b1),
                               ptr<float>(Wt2), ptr<float>(b2), ptr<float>(P1), ptr<uint8_t>(A1), ptr<float>(P2),
                               ptr<uint8_t>(A2), optr<int>(cur_row, "cur_row", I32, B),
                               optr<long long>(cur_lbl, "cur_lbl", I64, B), zp, zp ? (int)zero->numel() : 0,
                               (int)dbg, cur_stream()),
            "lenet_conv_fwd");
}

void lenet_fc1_fwd(const at::Tensor& P2, int64_t B, const at::Tensor& W, const at::Tensor& bias, const at::Tensor& H1,
                   const OptT& ctr) {
  check_cuda(P2, "P2", F32, B * 800);
  check_cuda(W, "fc1.weight", F32, 500 * 800);
  check_cuda(bias, "fc1.bias", F32, 500);
  check_cuda(H1, "H1", F32, B * 500);
  long long* cp = optr<long long>(ctr, "counters", I64, 1);
  hip_check(pde_lenet_fc1_fwd(ptr<float>(P2), (int)B, ptr<float>(W), ptr<float>(bias), ptr<float>(H1), cp,
                              cp ? (int)ctr->numel() : 0, cur_stream()),
            "lenet_fc1_fwd");
}

void lenet_head(const at::Tensor& H1, int64_t B, const at::Tensor& W2, const at::Tensor& b2, const at::Tensor& labels,
                double inv_b, const OptT& logp, const OptT& dZ2, const OptT& dZ1, const OptT& row_loss,
                const OptT& row_hit, const OptT& loss_sum, const OptT& correct) {
  check_cuda(H1, "H1", F32, B * 500);
  check_cuda(W2, "fc2.weight", F32, 5000);
  check_cuda(b2, "fc2.bias", F32, 10);
  check_cuda(labels, "labels", I64, B);
  float* dz1 = optr<float>(dZ1, "dZ1", F32, B * 500);
  float* dz2 = optr<float>(dZ2, "dZ2", F32, B * 10);
  TORCH_CHECK((dz1 == nullptr) == (dz2 == nullptr), "dZ1 and dZ2 go together");
  float* rl = optr<float>(row_loss, "row_loss", F32, B);
  int* rh = optr<int>(row_hit, "row_hit", I32, B);
  TORCH_CHECK((rl == nullptr) == (rh == nullptr), "row_loss and row_hit go together");
  hip_check(pde_lenet_head(ptr<float>(H1), (int)B, ptr<float>(W2), ptr<float>(b2), ptr<long long>(labels), (float)inv_b,
                           optr<float>(logp, "logp", F32, B * 10), dz2, dz1, rl, rh,
                           optr<double>(loss_sum, "loss_sum", F64, 1),
                           optr<unsigned long long>(correct, "correct", I64, 1), cur_stream()),
            "lenet_head");
}

void lenet_head_bwd(const at::Tensor& H1, int64_t B, const at::Tensor& W2, const at::Tensor& logp, const at::Tensor& g,
                    const at::Tensor& dZ2, const at::Tensor& dZ1) {
  check_cuda(H1, "H1", F32, B * 500);
  check_cuda(W2, "fc2.weight", F32, 5000);
  check_cuda(logp, "logp", F32, B * 10);
  check_cuda(g, "grad_logp", F32, B * 10);
  check_cuda(dZ2, "dZ2", F32, B * 10);
  check_cuda(dZ1, "dZ1", F32, B * 500);
  hip_check(pde_lenet_head_bwd(ptr<float>(H1), (int)B, ptr<float>(W2), ptr<float>(logp), ptr<float>(g), ptr<float>(dZ2),
                               ptr<float>(dZ1), cur_stream()),
            "lenet_head_bwd");
}

void lenet_fc_bwd(const at::Tensor& P2, const at::Tensor& H1, const at::Tensor& dZ1, const at::Tensor& dZ2,
                  const at::Tensor& W1, int64_t B, const at::Tensor& dP2m, const at::Tensor& gW1, const at::Tensor& gb1,
                  const at::Tensor& gW2, const at::Tensor& gb2, const OptT& row_loss, const OptT& row_hit,
                  const OptT& loss_sum, const OptT& correct, int64_t dbg, int64_t part) {
  TORCH_CHECK(part >= 0 && part <= 2, "lenet_fc_bwd: part must be 0 (all), 1 (dP2) or 2 (weight grads)");
  check_cuda(P2, "P2", F32, B * 800);
  check_cuda(H1, "H1", F32, B * 500);
  check_cuda(dZ1, "dZ1", F32, B * 500);
  check_cuda(dZ2, "dZ2", F32, B * 10);
  check_cuda(W1, "fc1.weight", F32, 400000);
  check_cuda(dP2m, "dP2m", F32, B * 800);
  check_cuda(gW1, "gW1", F32, 400000);
  check_cuda(gb1, "gb1", F32, 500);
  check_cuda(gW2, "gW2", F32, 5000);
  check_cuda(gb2, "gb2", F32, 10);
  hip_check(pde_lenet_fc_bwd(ptr<float>(P2), ptr<float>(H1), ptr<float>(dZ1), ptr<float>(dZ2), ptr<float>(W1), (int)B,
                             ptr<float>(dP2m), ptr<float>(gW1), ptr<float>(gb1), ptr<float>(gW2), ptr<float>(gb2),
                             optr<float>(row_loss, "row_loss", F32, B), optr<int>(row_hit, "row_hit", I32, B),
                             optr<double>(loss_sum, "loss_sum", F64, 1),
                             optr<unsigned long long>(correct, "correct", I64, 1), (int)dbg, (int)part,
                             cur_stream()),
            "lenet_fc_bwd");
}

void lenet_conv_bwd(const at::Tensor& X, const at::Tensor& rows, const at::Tensor& P1, const at::Tensor& A1,
                    const at::Tensor& dP2m, const at::Tensor& A2, const at::Tensor& W2c, int64_t B,
                    const at::Tensor& gW1c, const at::Tensor& gb1c, const at::Tensor& gW2c, const at::Tensor& gb2c,
                    int64_t c1_nrep, int64_t c1_rep_stride, const OptT& row_loss, const OptT& row_hit,
                    const OptT& loss_sum, const OptT& correct, int64_t dbg, const OptT& peer_dev,
                    const OptT& ar_buf, int64_t ar_two) {
  check_cuda(X, "X", F32);
  check_cuda(rows, "rows", I32, B);
  // fused all-reduce side blocks: peer_dev = CPU uint8 bytes of a pde::PeerDev, ar_buf = fc bucket
  const void* pdev = nullptr;
  float* arp = nullptr;
  int64_t arn = 0;
  if (peer_dev.has_value() && peer_dev->defined()) {
    TORCH_CHECK(!peer_dev->is_cuda() && peer_dev->scalar_type() == at::kByte &&
                    peer_dev->numel() == (int64_t)sizeof(pde::PeerDev) && peer_dev->is_contiguous(),
                "peer_dev must be the CPU uint8 bytes of PeerAllReduce.device_args()");
    TORCH_CHECK(ar_buf.has_value() && ar_buf->defined(), "ar_buf required with peer_dev");
    check_cuda(*ar_buf, "ar_buf", F32, 1);
    TORCH_CHECK(reinterpret_cast<uintptr_t>(ar_buf->data_ptr()) % 16 == 0, "ar_buf must be 16-byte aligned");
    pdev = peer_dev->data_ptr();
    arp = ar_buf->data_ptr<float>();
    arn = ar_buf->numel();
    const auto* pd = static_cast<const pde::PeerDev*>(pdev);
    TORCH_CHECK(arn * 4 <= pd->cap, "ar_buf exceeds the peer all-reduce capacity");
  }
  check_cuda(P1, "P1", F32, B * 2880);
  check_cuda(A1, "A1", U8, B * 2880);
  check_cuda(dP2m, "dP2m", F32, B * 800);
  check_cuda(A2, "A2", U8, B * 800);
  check_cuda(W2c, "conv2.weight", F32, 25000);
  TORCH_CHECK(c1_nrep >= 1 && (c1_nrep == 1 || c1_rep_stride >= 520), "bad conv1 replica layout");
  check_cuda(gW1c, "gW1c", F32, 500 + (c1_nrep - 1) * c1_rep_stride);
  check_cuda(gb1c, "gb1c", F32, 20);
  if (c1_nrep > 1)
    TORCH_CHECK(gb1c.data_ptr<float>() + (c1_nrep - 1) * c1_rep_stride + 20 <=
                    gW1c.data_ptr<float>() + gW1c.numel(), "conv1 replicas must fit in the gW1c storage view");
  check_cuda(gW2c, "gW2c", F32, 25000);
  check_cuda(gb2c, "gb2c", F32, 50);
  hip_check(pde_lenet_conv_bwd(ptr<float>(X), ptr<int>(rows), ptr<float>(P1), ptr<uint8_t>(A1), ptr<float>(dP2m),
                               ptr<uint8_t>(A2), ptr<float>(W2c), (int)B, ptr<float>(gW1c), ptr<float>(gb1c),
                               ptr<float>(gW2c), ptr<float>(gb2c), (int)c1_nrep, (int)c1_rep_stride,
                               optr<float>(row_loss, "row_loss", F32, B), optr<int>(row_hit, "row_hit", I32, B),
                               optr<double>(loss_sum, "loss_sum", F64, 1),
                               optr<unsigned long long>(correct, "correct", I64, 1), (int)dbg, pdev, arp, arn,
                               (int)ar_two, cur_stream()),
            "lenet_conv_bwd");
}

// ------------------------------------------------------------------------------------------------
void adam_flat(const at::Tensor& p, const at::Tensor& g, const at::Tensor& m, const at::Tensor& v, double lr,
               double b1, double b2, double eps, double wd, bool decoupled, double grad_scale, const at::Tensor& step,
               const at::Tensor& arrive, int64_t bump, int64_t pack_off, const OptT& pack_dst, int64_t fold_off,
               int64_t fold_len, int64_t fold_nrep, int64_t fold_stride, const OptT& peer_dev, int64_t ar_off,
               const OptT& ar_epoch, int64_t ar_two, int64_t pack_mode, int64_t fold2_off, int64_t fold2_len,
               int64_t fold2_nrep, int64_t fold2_stride) {
  const int64_t n = p.numel();
  // fused all-reduce of [ar_off, n) by side blocks (peer_dev = CPU bytes of PeerAllReduce.device_args())
  const void* pdev = nullptr;
  long long* ep = nullptr;
  if (peer_dev.has_value() && peer_dev->defined()) {
    TORCH_CHECK(!peer_dev->is_cuda() && peer_dev->scalar_type() == at::kByte &&
                    peer_dev->numel() == (int64_t)sizeof(pde::PeerDev) && peer_dev->is_contiguous(),
                "peer_dev must be the CPU uint8 bytes of PeerAllReduce.device_args()");
    TORCH_CHECK(ar_off >= 0 && ar_off < n && ar_off % 4 == 0, "bad fused all-reduce offset");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(g.data_ptr<float>() + ar_off) % 16 == 0, "fused range must be 16-B aligned");
    const auto* pd = static_cast<const pde::PeerDev*>(peer_dev->data_ptr());
    TORCH_CHECK((n - ar_off) * 4 <= pd->cap, "fused range exceeds the peer all-reduce capacity");
    TORCH_CHECK(ar_epoch.has_value() && ar_epoch->defined(), "ar_epoch required with peer_dev");
    check_cuda(*ar_epoch, "ar_epoch", I64, 1);
    pdev = peer_dev->data_ptr();
    ep = ptr<long long>(*ar_epoch);
  }
  check_cuda(p, "params", F32);
  check_cuda(g, "grads", F32, n);
  check_cuda(m, "exp_avg", F32, n);
  if (fold_off >= 0 && fold_nrep > 1)
    TORCH_CHECK(fold_off % 4 == 0 && fold_len % 4 == 0 && fold_stride % 4 == 0 && fold_len <= fold_stride &&
                    fold_off + fold_stride * fold_nrep <= n && fold_nrep <= 16,
                "bad gradient fold layout (at most 16 replicas)");
  if (fold2_off >= 0 && fold2_nrep > 1)
    TORCH_CHECK(fold2_off % 4 == 0 && fold2_len % 4 == 0 && fold2_stride % 4 == 0 && fold2_len <= fold2_stride &&
                    fold2_off + fold2_stride * fold2_nrep <= n && fold2_nrep <= 16,
                "bad second gradient fold layout (at most 16 replicas)");
  check_cuda(v, "exp_avg_sq", F32, n);
  check_cuda(step, "step", I64, std::max<int64_t>(1, bump));
  TORCH_CHECK(bump >= -1, "bump must be >= -1");
  check_cuda(arrive, "arrive", I32, 1);
  TORCH_CHECK(n % 4 == 0, "flat buffer length must be a multiple of 4");
  TORCH_CHECK(pack_mode == 1 || pack_mode == 2, "pack_mode must be 1 ([500][64]) or 2 (lenet_v2 image)");
  float* pd = optr<float>(pack_dst, "pack_dst", F32, pack_mode == 2 ? kPdeWpFloats : 500 * 64);
  if (pack_off >= 0) TORCH_CHECK(pd && pack_off + 25000 <= n, "bad pack target");
  hip_check(pde_adam_flat(ptr<float>(p), ptr<float>(g), ptr<float>(m), ptr<float>(v), n, (float)lr, (float)b1,
                          (float)b2, (float)eps, (float)wd, decoupled ? 1 : 0, (float)grad_scale, ptr<long long>(step),
                          ptr<unsigned>(arrive), (int)bump, pd ? pack_off : -1, pd, fold_off, (int)fold_len,
                          (int)fold_nrep, (int)fold_stride, pdev, ar_off, ep, (int)ar_two, (int)pack_mode, fold2_off,
                          (int)fold2_len, (int)fold2_nrep, (int)fold2_stride, cur_stream()),
            "adam_flat");
}

void sgd_flat(const at::Tensor& p, const at::Tensor& g, const at::Tensor& buf, double lr, double momentum,
              double dampening, double wd, bool nesterov, double grad_scale, const at::Tensor& step,
              const at::Tensor& arrive, int64_t bump, int64_t pack_off, const OptT& pack_dst, int64_t fold_off,
              int64_t fold_len, int64_t fold_nrep, int64_t fold_stride, int64_t pack_mode, int64_t fold2_off,
              int64_t fold2_len, int64_t fold2_nrep, int64_t fold2_stride) {
  const int64_t n = p.numel();
  check_cuda(p, "params", F32);
  check_cuda(g, "grads", F32, n);
  check_cuda(buf, "momentum_buffer", F32, momentum != 0.0 ? n : 0);
  if (fold_off >= 0 && fold_nrep > 1)
    TORCH_CHECK(fold_off % 4 == 0 && fold_len % 4 == 0 && fold_stride % 4 == 0 && fold_len <= fold_stride &&
                    fold_off + fold_stride * fold_nrep <= n && fold_nrep <= 16,
                "bad gradient fold layout (at most 16 replicas)");
  if (fold2_off >= 0 && fold2_nrep > 1)
    TORCH_CHECK(fold2_off % 4 == 0 && fold2_len % 4 == 0 && fold2_stride % 4 == 0 && fold2_len <= fold2_stride &&
                    fold2_off + fold2_stride * fold2_nrep <= n && fold2_nrep <= 16,
                "bad second gradient fold layout (at most 16 replicas)");
  check_cuda(step, "step", I64, std::max<int64_t>(1, bump));
  TORCH_CHECK(bump >= -1, "bump must be >= -1");
  check_cuda(arrive, "arrive", I32, 1);
  TORCH_CHECK(n % 4 == 0, "flat buffer length must be a multiple of 4");
  TORCH_CHECK(pack_mode == 1 || pack_mode == 2, "pack_mode must be 1 ([500][64]) or 2 (lenet_v2 image)");
  float* pd = optr<float>(pack_dst, "pack_dst", F32, pack_mode == 2 ? kPdeWpFloats : 500 * 64);
  if (pack_off >= 0) TORCH_CHECK(pd && pack_off + 25000 <= n, "bad pack target");
  hip_check(pde_sgd_flat(ptr<float>(p), ptr<float>(g), ptr<float>(buf), n, (float)lr, (float)momentum,
                         (float)dampening, (float)wd, nesterov ? 1 : 0, (float)grad_scale, ptr<long long>(step),
                         ptr<unsigned>(arrive), (int)bump, pd ? pack_off : -1, pd, fold_off, (int)fold_len,
                         (int)fold_nrep, (int)fold_stride, (int)pack_mode, fold2_off, (int)fold2_len,
                         (int)fold2_nrep, (int)fold2_stride, cur_stream()),
            "sgd_flat");
}

void lenet_pack_w2_v2(const at::Tensor& w2, const at::Tensor& dst) {
  check_cuda(w2, "conv2.weight", F32, 25000);
  check_cuda(dst, "Wp", F32, kPdeWpFloats);
  hip_check(pde_lenet_pack_w2_v2(ptr<float>(w2), ptr<float>(dst), cur_stream()), "lenet_pack_w2_v2");
}

void lenet_conv_fwd2(const at::Tensor& Xb, int64_t B, const at::Tensor& w1, const at::Tensor& b1, const at::Tensor& Wp,
                     const at::Tensor& b2, const at::Tensor& P1, const at::Tensor& A1, const at::Tensor& P2,
                     const at::Tensor& A2, const OptT& zero) {
  TORCH_CHECK(B >= 1 && B <= 65535, "batch must be in [1, 65535]");
  check_cuda(Xb, "Xb", F32, B * 784);
  check_cuda(w1, "conv1.weight", F32, 500);
  check_cuda(b1, "conv1.bias", F32, 20);
  check_cuda(Wp, "Wp", F32, kPdeWpFloats);
  check_cuda(b2, "conv2.bias", F32, 50);
  check_cuda(P1, "P1", F32, B * 2880);
  check_cuda(A1, "A1", U8, B * 2880);
  check_cuda(P2, "P2", F32, B * 800);
  check_cuda(A2, "A2", U8, B * 800);
  for (const at::Tensor* t : {&Xb, &w1, &Wp, &P1})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "conv_fwd2 operands must be 16-B aligned");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(A1.data_ptr()) % 4 == 0, "A1 must be 4-B aligned");
  float* zp = optr<float>(zero, "zero", F32);
  hip_check(pde_lenet_conv_fwd2(ptr<float>(Xb), (int)B, ptr<float>(w1), ptr<float>(b1), ptr<float>(Wp), ptr<float>(b2),
                                ptr<float>(P1), ptr<uint8_t>(A1), ptr<float>(P2), ptr<uint8_t>(A2), zp,
                                zp ? (int)zero->numel() : 0, cur_stream()),
            "lenet_conv_fwd2");
}

void lenet_gather(const at::Tensor& X, const at::Tensor& labels, const OptT& idx, const OptT& ctr, int64_t nbatches,
                  int64_t B, const at::Tensor& Xdst, const at::Tensor& Ydst, const OptT& rows_dst) {
  check_cuda(X, "X", F32);
  TORCH_CHECK(X.numel() % 784 == 0, "X must be [N,1,28,28]");
  check_cuda(labels, "labels", I64, X.numel() / 784);
  const int* ip = optr<int>(idx, "idx", I32, 1);
  if (!ip) TORCH_CHECK(X.numel() >= B * 784, "X smaller than batch");
  const long long* cp = optr<long long>(ctr, "ctr", I64, 1);
  if (cp) TORCH_CHECK(ip && nbatches >= 1, "counter-indexed batches need idx");
  check_cuda(Xdst, "Xdst", F32, B * 784);
  check_cuda(Ydst, "Ydst", I64, B);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(X.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(Xdst.data_ptr()) % 16 == 0,
              "gather buffers must be 16-B aligned");
  hip_check(pde_lenet_gather(ptr<float>(X), ptr<long long>(labels), ip, ip ? (int)idx->numel() : 0, cp, (int)nbatches,
                             (int)B, ptr<float>(Xdst), ptr<long long>(Ydst), optr<int>(rows_dst, "rows_dst", I32, B),
                             cur_stream()),
            "lenet_gather");
}

void lenet_conv_grad_fold(const at::Tensor& slab, const at::Tensor& c1img, int64_t B, const at::Tensor& g, int64_t c1w,
                          int64_t c1b, int64_t c2w, int64_t c2b) {
  TORCH_CHECK(B >= 1 && B <= 128, "conv_grad_fold: batch must be in [1, 128]");
  check_cuda(slab, "slab", F32, 16 * 25088);
  check_cuda(c1img, "c1img", F32, B * 520);
  check_cuda(g, "grads", F32);
  const int64_t n = g.numel();
  TORCH_CHECK(c1w >= 0 && c1w + 500 <= n && c1b >= 0 && c1b + 20 <= n && c2w >= 0 && c2w + 25000 <= n && c2b >= 0 &&
                  c2b + 50 <= n, "conv_grad_fold: conv gradient slots outside the flat buffer");
  hip_check(pde_lenet_conv_grad_fold(ptr<float>(slab), ptr<float>(c1img), (int)B, ptr<float>(g), c1w, c1b, c2w, c2b,
                                     cur_stream()),
            "lenet_conv_grad_fold");
}

void lenet_conv_fold_ar(const at::Tensor& ipdev, const at::Tensor& slab, const at::Tensor& c1img, int64_t B,
                        const at::Tensor& g, int64_t c1w, int64_t c1b, int64_t c2w, int64_t c2b, int64_t lo, int64_t hi,
                        const at::Tensor& sync, double scale, int64_t two) {
  TORCH_CHECK(B >= 1 && B <= 128, "conv_fold_ar: batch must be in [1, 128]");
  TORCH_CHECK(ipdev.device().is_cpu() && ipdev.scalar_type() == at::kByte && ipdev.numel() == sizeof(pde::PeerIpDev),
              "conv_fold_ar: ipdev must be the bytes of PeerAllReduce.registered_device_args()");
  check_cuda(slab, "slab", F32, 16 * 25088);
  check_cuda(c1img, "c1img", F32, B * 520);
  check_cuda(g, "grads", F32);
  check_cuda(sync, "sync", at::kInt, 2);
  pde::PeerIpDev d;
  std::memcpy(&d, ipdev.data_ptr(), sizeof(d));
  TORCH_CHECK(d.data[d.rank] == g.data_ptr(), "conv_fold_ar: g must be the registered buffer (from its start)");
  hip_check(pde_lenet_conv_fold_ar(ipdev.data_ptr(), ptr<float>(slab), ptr<float>(c1img), (int)B, c1w, c1b, c2w, c2b,
                                   g.numel(), lo, hi, reinterpret_cast<unsigned*>(sync.data_ptr()), (float)scale,
                                   (int)two, cur_stream()),
            "lenet_conv_fold_ar");
}

void lenet_conv_bwd2(const at::Tensor& Xb, const at::Tensor& P1, const at::Tensor& A1, const at::Tensor& dP2m,
                     const at::Tensor& A2, const at::Tensor& W2c, int64_t B, const at::Tensor& slab,
                     const at::Tensor& c1rep, const at::Tensor& c1part, const at::Tensor& tick, const at::Tensor& g, int64_t c1w, int64_t c1b,
                     int64_t c2w, int64_t c2b, const OptT& row_loss, const OptT& row_hit,
                     const OptT& loss_sum, const OptT& correct, const OptT& gX, const OptT& glabels, const OptT& gidx,
                     const OptT& gctr, int64_t gnbatches, int64_t gstride, const OptT& gXdst, const OptT& gYdst,
                     const OptT& grows, const OptT& peer_dev, const OptT& ar_buf, int64_t ar_two, int64_t defer,
                     int64_t dbg, const OptT& c1img) {
  TORCH_CHECK(B >= 1 && B <= 128, "conv_bwd2: batch must be in [1, 128] (16 image groups of <= 8 images)");
  check_cuda(Xb, "Xb", F32, B * 784);
  check_cuda(P1, "P1", F32, B * 2880);
  check_cuda(A1, "A1", U8, B * 2880);
  check_cuda(dP2m, "dP2m", F32, B * 800);
  check_cuda(A2, "A2", U8, B * 800);
  check_cuda(W2c, "conv2.weight", F32, 25000);
  check_cuda(slab, "slab", F32, 15 * 25088 + 25074);
  check_cuda(c1rep, "c1rep", I64, 16 * 576);
  check_cuda(c1part, "c1part", F32, 16 * 576);
  check_cuda(tick, "tick", I32, 32);
  check_cuda(g, "grads", F32);
  const int64_t n = g.numel();
  TORCH_CHECK(c1w >= 0 && c1w + 500 <= n && c1b >= 0 && c1b + 20 <= n && c2w >= 0 && c2w + 25000 <= n && c2b >= 0 &&
                  c2b + 50 <= n, "conv_bwd2: conv gradient slots outside the flat buffer");
  for (const at::Tensor* t : {&Xb, &P1, &dP2m, &g})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "conv_bwd2 operands must be 16-B aligned");
  PdeLenetBwdOpt o{};
  o.slab = ptr<float>(slab);
  o.c1rep = ptr<long long>(c1rep);
  o.c1part = ptr<float>(c1part);
  o.tick = reinterpret_cast<unsigned*>(tick.data_ptr<int32_t>());
  o.g = ptr<float>(g);
  o.c1w = c1w; o.c1b = c1b; o.c2w = c2w; o.c2b = c2b;
  TORCH_CHECK(defer >= 0 && defer <= 2, "conv_bwd2: defer must be 0 (fold), 1 (defer) or 2 (ext)");
  o.defer = (int)defer;
  if (defer == 2) {
    TORCH_CHECK(c1img.has_value(), "conv_bwd2: ext mode needs the per-image conv1 partial buffer");
    check_cuda(*c1img, "c1img", F32, B * 520);
    o.c1img = ptr<float>(*c1img);
  }
  if (peer_dev.has_value()) {
    TORCH_CHECK(peer_dev->numel() == (int64_t)sizeof(pde::PeerDev), "bad peer device args");
    check_cuda(*ar_buf, "ar_buf", F32);
    TORCH_CHECK(reinterpret_cast<uintptr_t>(ar_buf->data_ptr()) % 16 == 0, "ar_buf must be 16-B aligned");
    o.peer_dev = peer_dev->data_ptr();
    o.ar_buf = ptr<float>(*ar_buf);
    o.ar_n = ar_buf->numel();
    o.ar_two = (int)ar_two;
  }
  const bool meters = row_loss.has_value() && row_hit.has_value() && loss_sum.has_value() && correct.has_value();
  const bool gather = gX.has_value();
  if (gather) {
    TORCH_CHECK(glabels.has_value() && gidx.has_value() && gctr.has_value() && gXdst.has_value() &&
                    gYdst.has_value() && grows.has_value() && gnbatches >= 1 && gstride >= B,
                "conv_bwd2 prefetch needs labels, idx, counter, destinations");
    check_cuda(*gX, "gX", F32);
    check_cuda(*gXdst, "gXdst", F32, B * 784);
    check_cuda(*gYdst, "gYdst", I64, B);
  }
  hip_check(pde_lenet_conv_bwd2(ptr<float>(Xb), ptr<float>(P1), ptr<uint8_t>(A1), ptr<float>(dP2m), ptr<uint8_t>(A2),
                                ptr<float>(W2c), (int)B, &o,
                                meters ? ptr<float>(*row_loss) : nullptr, meters ? ptr<int>(*row_hit) : nullptr,
                                meters ? ptr<double>(*loss_sum) : nullptr,
                                meters ? reinterpret_cast<unsigned long long*>(correct->data_ptr<int64_t>()) : nullptr,
                                gather ? ptr<float>(*gX) : nullptr, gather ? ptr<long long>(*glabels) : nullptr,
                                gather ? ptr<int>(*gidx) : nullptr, gather ? (int)gidx->numel() : 0,
                                gather ? ptr<long long>(*gctr) : nullptr, (int)gnbatches, (int)gstride,
                                gather ? ptr<float>(*gXdst) : nullptr, gather ? ptr<long long>(*gYdst) : nullptr,
                                gather ? ptr<int>(*grows) : nullptr, (int)dbg, cur_stream()),
            "lenet_conv_bwd2");
}

void lenet_set_prof(const OptT& buf) {
  if (buf.has_value()) {
    check_cuda(*buf, "prof", I64, 6 * 4096 * 8);
    pde_lenet_set_prof(reinterpret_cast<unsigned long long*>(buf->data_ptr<int64_t>()));
  } else {
    pde_lenet_set_prof(nullptr);
  }
}

void lenet_pack_w2(const at::Tensor& w2, const at::Tensor& dst) {
  check_cuda(w2, "conv2.weight", F32, 25000);
  check_cuda(dst, "Wt2", F32, 500 * 64);
  hip_check(pde_lenet_pack_w2(ptr<float>(w2), ptr<float>(dst), cur_stream()), "lenet_pack_w2");
}

void scale_(const at::Tensor& x, double s) {
  check_cuda(x, "x", F32);
  hip_check(pde_scale(ptr<float>(x), x.numel(), (float)s, cur_stream()), "scale_");
}

// ------------------------------------------------------------------------------------------------
// generic ops
void gemm(const at::Tensor& A, const at::Tensor& B, const at::Tensor& C, const OptT& bias, int64_t M, int64_t N,
          int64_t K, int64_t lda, int64_t ldb, int64_t ldc, bool transA, bool transB, int64_t sA, int64_t sB,
          int64_t sC, int64_t batch, double alpha, double beta, int64_t bias_mode, bool relu, bool atomic) {
  check_cuda(A, "A", F32);
  check_cuda(B, "B", F32);
  check_cuda(C, "C", F32);
  TORCH_CHECK(M > 0 && N > 0 && K > 0 && batch > 0, "empty gemm");
  const int64_t needA = (batch - 1) * sA + (transA ? (K - 1) * lda + M : (M - 1) * lda + K);
  const int64_t needB = (batch - 1) * sB + (transB ? (N - 1) * ldb + K : (K - 1) * ldb + N);
  const int64_t needC = (batch - 1) * sC + (M - 1) * ldc + N;
  TORCH_CHECK(A.numel() >= needA && B.numel() >= needB && C.numel() >= needC, "gemm operand too small");
  const float* bp = optr<float>(bias, "bias", F32, bias_mode == 1 ? N : (bias_mode == 2 ? M : 0));
  TORCH_CHECK(bias_mode == 0 || bp, "bias_mode needs a bias");
  hip_check(pde_gemm_f32(ptr<float>(A), ptr<float>(B), ptr<float>(C), bp, (int)M, (int)N, (int)K, (int)lda, (int)ldb,
                         (int)ldc, transA, transB, sA, sB, sC, (int)batch, (float)alpha, (float)beta, (int)bias_mode,
                         relu, atomic, cur_stream()),
            "gemm");
}

void xent_fwd(const at::Tensor& x, const at::Tensor& y, const at::Tensor& row_loss, const at::Tensor& lse) {
  TORCH_CHECK(x.dim() == 2, "logits must be [B, C]");
  const bool bf = x.scalar_type() == at::kBFloat16;
  check_cuda(x, "logits", bf ? at::kBFloat16 : F32);
  const int64_t B = x.size(0), C = x.size(1);
  check_cuda(y, "target", I64, B);
  check_cuda(row_loss, "row_loss", F32, B);
  check_cuda(lse, "lse", F32, B);
  if (bf)
    hip_check(pde_xent_fwd_bf16(x.data_ptr(), ptr<long long>(y), (int)B, (int)C, ptr<float>(row_loss), ptr<float>(lse),
                                cur_stream()),
              "xent_fwd");
  else
    hip_check(pde_xent_fwd(ptr<float>(x), ptr<long long>(y), (int)B, (int)C, ptr<float>(row_loss), ptr<float>(lse),
                           cur_stream()),
              "xent_fwd");
}

void xent_bwd(const at::Tensor& x, const at::Tensor& y, const at::Tensor& lse, const at::Tensor& gscale, bool per_row,
              double mul, const at::Tensor& dx) {
  const bool bf = x.scalar_type() == at::kBFloat16;
  check_cuda(x, "logits", bf ? at::kBFloat16 : F32);
  const int64_t B = x.size(0), C = x.size(1);
  check_cuda(y, "target", I64, B);
  check_cuda(lse, "lse", F32, B);
  check_cuda(gscale, "grad", F32, per_row ? B : 1);
  check_cuda(dx, "dx", bf ? at::kBFloat16 : F32, B * C);
  if (bf)
    hip_check(pde_xent_bwd_bf16(x.data_ptr(), ptr<long long>(y), ptr<float>(lse), ptr<float>(gscale), per_row,
                                (float)mul, (int)B, (int)C, dx.data_ptr(), cur_stream()),
              "xent_bwd");
  else
    hip_check(pde_xent_bwd(ptr<float>(x), ptr<long long>(y), ptr<float>(lse), ptr<float>(gscale), per_row, (float)mul,
                           (int)B, (int)C, ptr<float>(dx), cur_stream()),
              "xent_bwd");
}

void log_softmax_fwd(const at::Tensor& x, const at::Tensor& out) {
  check_cuda(x, "x", F32);
  TORCH_CHECK(x.dim() == 2, "log_softmax kernel takes [B, C] (dim=1)");
  check_cuda(out, "out", F32, x.numel());
  hip_check(pde_log_softmax_fwd(ptr<float>(x), (int)x.size(0), (int)x.size(1), ptr<float>(out), cur_stream()),
            "log_softmax_fwd");
}

void log_softmax_bwd(const at::Tensor& out, const at::Tensor& g, const at::Tensor& dx) {
  check_cuda(out, "out", F32);
  check_cuda(g, "grad", F32, out.numel());
  check_cuda(dx, "dx", F32, out.numel());
  hip_check(pde_log_softmax_bwd(ptr<float>(out), ptr<float>(g), (int)out.size(0), (int)out.size(1), ptr<float>(dx),
                                cur_stream()),
            "log_softmax_bwd");
}

void relu_fwd(const at::Tensor& x, const at::Tensor& y) {
  check_cuda(x, "x", F32);
  check_cuda(y, "y", F32, x.numel());
  hip_check(pde_relu_fwd(ptr<float>(x), ptr<float>(y), x.numel(), cur_stream()), "relu_fwd");
}

void relu_bwd(const at::Tensor& y, const at::Tensor& g, const at::Tensor& dx) {
  check_cuda(y, "y", F32);
  check_cuda(g, "grad", F32, y.numel());
  check_cuda(dx, "dx", F32, y.numel());
  hip_check(pde_relu_bwd(ptr<float>(y), ptr<float>(g), ptr<float>(dx), y.numel(), cur_stream()), "relu_bwd");
}

void pool2_fwd(const at::Tensor& x, int64_t NC, int64_t H, int64_t W, const at::Tensor& y, const at::Tensor& code) {
  check_cuda(x, "x", F32, NC * H * W);
  check_cuda(y, "y", F32, NC * (H / 2) * (W / 2));
  check_cuda(code, "code", U8, NC * (H / 2) * (W / 2));
  hip_check(pde_pool2_fwd(ptr<float>(x), (int)NC, (int)H, (int)W, ptr<float>(y), ptr<uint8_t>(code), cur_stream()),
            "pool2_fwd");
}

void pool2_bwd(const at::Tensor& g, const at::Tensor& code, int64_t NC, int64_t H, int64_t W, const at::Tensor& dx) {
  check_cuda(g, "grad", F32, NC * (H / 2) * (W / 2));
  check_cuda(code, "code", U8, NC * (H / 2) * (W / 2));
  check_cuda(dx, "dx", F32, NC * H * W);
  hip_check(pde_pool2_bwd(ptr<float>(g), ptr<uint8_t>(code), (int)NC, (int)H, (int)W, ptr<float>(dx), cur_stream()),
            "pool2_bwd");
}

void im2col(const at::Tensor& x, int64_t B, int64_t C, int64_t H, int64_t W, int64_t KH, int64_t KW, int64_t stride,
            int64_t pad, int64_t OH, int64_t OW, const at::Tensor& col) {
  check_cuda(x, "x", F32, B * C * H * W);
  check_cuda(col, "col", F32, B * C * KH * KW * OH * OW);
  hip_check(pde_im2col(ptr<float>(x), (int)B, (int)C, (int)H, (int)W, (int)KH, (int)KW, (int)stride, (int)pad, (int)OH,
                       (int)OW, ptr<float>(col), cur_stream()),
            "im2col");
}

void col2im(const at::Tensor& col, int64_t B, int64_t C, int64_t H, int64_t W, int64_t KH, int64_t KW, int64_t stride,
            int64_t pad, int64_t OH, int64_t OW, const at::Tensor& dx) {
  check_cuda(col, "col", F32, B * C * KH * KW * OH * OW);
  check_cuda(dx, "dx", F32, B * C * H * W);
  hip_check(pde_col2im(ptr<float>(col), (int)B, (int)C, (int)H, (int)W, (int)KH, (int)KW, (int)stride, (int)pad,
                       (int)OH, (int)OW, ptr<float>(dx), cur_stream()),
            "col2im");
}

void bias_grad_nchw(const at::Tensor& dy, int64_t B, int64_t O, int64_t P, const at::Tensor& db) {
  check_cuda(dy, "dy", F32, B * O * P);
  check_cuda(db, "db", F32, O);
  hip_check(pde_bias_grad_nchw(ptr<float>(dy), (int)B, (int)O, P, ptr<float>(db), cur_stream()), "bias_grad_nchw");
}

void colsum(const at::Tensor& x, int64_t M, int64_t N, const at::Tensor& out) {
  check_cuda(x, "x", F32, M * N);
  check_cuda(out, "out", F32, N);
  hip_check(pde_colsum(ptr<float>(x), (int)M, (int)N, ptr<float>(out), cur_stream()), "colsum");
}

void gather_rows(const at::Tensor& src, const at::Tensor& idx, const at::Tensor& out) {
  check_cuda(src, "src", F32);
  check_cuda(idx, "idx", I64);
  check_cuda(out, "out", F32);
  const int64_t n = idx.numel(), row = src.numel() / std::max<int64_t>(1, src.size(0));
  TORCH_CHECK(out.numel() >= n * row && row % 4 == 0, "gather_rows: bad sizes");
  hip_check(pde_gather_rows(ptr<float>(src), ptr<long long>(idx), (int)n, (int)row, ptr<float>(out), cur_stream()),
            "gather_rows");
}

}  // namespace

PYBIND11_MODULE(_kernels, m) {
  m.doc() = "CDNA4 (gfx950) HIP kernels of pytorch_distributed_example_amd";
  m.attr("arch") = "gfx950";
  namespace py = pybind11;
  pde::register_transformer(m);
  pde::register_resnet(m);
  m.def("lenet_conv_fwd", &lenet_conv_fwd, py::arg("X"), py::arg("idx"), py::arg("step"), py::arg("nbatches"),
        py::arg("stride"), py::arg("labels_all"), py::arg("B"), py::arg("w1"), py::arg("b1"), py::arg("Wt2"),
        py::arg("b2"), py::arg("P1"), py::arg("A1"), py::arg("P2"), py::arg("A2"), py::arg("cur_row"),
        py::arg("cur_lbl"), py::arg("zero"), py::arg("dbg") = 0);
  m.def("lenet_fc1_fwd", &lenet_fc1_fwd);
  m.def("lenet_head", &lenet_head);
  m.def("lenet_head_bwd", &lenet_head_bwd);
  m.def("lenet_fc_bwd", &lenet_fc_bwd, py::arg("P2"), py::arg("H1"), py::arg("dZ1"), py::arg("dZ2"), py::arg("W1"),
        py::arg("B"), py::arg("dP2m"), py::arg("gW1"), py::arg("gb1"), py::arg("gW2"), py::arg("gb2"),
        py::arg("row_loss"), py::arg("row_hit"), py::arg("loss_sum"), py::arg("correct"), py::arg("dbg") = 0,
        py::arg("part") = 0);
  m.def("lenet_conv_bwd", &lenet_conv_bwd, py::arg("X"), py::arg("rows"), py::arg("P1"), py::arg("A1"), py::arg("dP2m"),
        py::arg("A2"), py::arg("W2c"), py::arg("B"), py::arg("gW1c"), py::arg("gb1c"), py::arg("gW2c"), py::arg("gb2c"),
        py::arg("c1_nrep") = 1, py::arg("c1_rep_stride") = 0, py::arg("row_loss") = py::none(),
        py::arg("row_hit") = py::none(), py::arg("loss_sum") = py::none(), py::arg("correct") = py::none(),
        py::arg("dbg") = 0, py::arg("peer_dev") = py::none(), py::arg("ar_buf") = py::none(), py::arg("ar_two") = 1);
  m.def("adam_flat", &adam_flat, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("lr"), py::arg("b1"),
        py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("decoupled"), py::arg("grad_scale"), py::arg("step"),
        py::arg("arrive"), py::arg("bump"), py::arg("pack_off") = -1, py::arg("pack_dst") = py::none(),
        py::arg("fold_off") = -1, py::arg("fold_len") = 0, py::arg("fold_nrep") = 1, py::arg("fold_stride") = 0,
        py::arg("peer_dev") = py::none(), py::arg("ar_off") = 0, py::arg("ar_epoch") = py::none(),
        py::arg("ar_two") = 0, py::arg("pack_mode") = 1, py::arg("fold2_off") = -1, py::arg("fold2_len") = 0,
        py::arg("fold2_nrep") = 1, py::arg("fold2_stride") = 0);
  m.def("sgd_flat", &sgd_flat, py::arg("p"), py::arg("g"), py::arg("buf"), py::arg("lr"), py::arg("momentum"),
        py::arg("dampening"), py::arg("wd"), py::arg("nesterov"), py::arg("grad_scale"), py::arg("step"),
        py::arg("arrive"), py::arg("bump"), py::arg("pack_off") = -1, py::arg("pack_dst") = py::none(),
        py::arg("fold_off") = -1, py::arg("fold_len") = 0, py::arg("fold_nrep") = 1, py::arg("fold_stride") = 0,
        py::arg("pack_mode") = 1, py::arg("fold2_off") = -1, py::arg("fold2_len") = 0, py::arg("fold2_nrep") = 1,
        py::arg("fold2_stride") = 0);
  m.def("lenet_pack_w2", &lenet_pack_w2);
  m.def("lenet_pack_w2_v2", &lenet_pack_w2_v2);
  m.def("lenet_conv_fwd2", &lenet_conv_fwd2, py::arg("Xb"), py::arg("B"), py::arg("w1"), py::arg("b1"), py::arg("Wp"),
        py::arg("b2"), py::arg("P1"), py::arg("A1"), py::arg("P2"), py::arg("A2"), py::arg("zero") = py::none());
  m.def("lenet_conv_grad_fold", &lenet_conv_grad_fold);
  m.def("lenet_conv_fold_ar", &lenet_conv_fold_ar);
  m.def("lenet_conv_bwd2", &lenet_conv_bwd2, py::arg("Xb"), py::arg("P1"), py::arg("A1"), py::arg("dP2m"),
        py::arg("A2"), py::arg("W2c"), py::arg("B"), py::arg("slab"), py::arg("c1rep"), py::arg("c1part"), py::arg("tick"),
        py::arg("g"),
        py::arg("c1w"), py::arg("c1b"), py::arg("c2w"), py::arg("c2b"), py::arg("row_loss") = py::none(), py::arg("row_hit") = py::none(), py::arg("loss_sum") = py::none(),
        py::arg("correct") = py::none(), py::arg("gX") = py::none(), py::arg("glabels") = py::none(),
        py::arg("gidx") = py::none(), py::arg("gctr") = py::none(), py::arg("gnbatches") = 1, py::arg("gstride") = 0,
        py::arg("gXdst") = py::none(), py::arg("gYdst") = py::none(), py::arg("grows") = py::none(),
        py::arg("peer_dev") = py::none(), py::arg("ar_buf") = py::none(), py::arg("ar_two") = 0, py::arg("defer") = 0,
        py::arg("dbg") = 0, py::arg("c1img") = py::none());
  m.def("lenet_gather", &lenet_gather, py::arg("X"), py::arg("labels"), py::arg("idx"), py::arg("ctr"),
        py::arg("nbatches"), py::arg("B"), py::arg("Xdst"), py::arg("Ydst"), py::arg("rows_dst"));
  m.def("lenet_set_prof", &lenet_set_prof, py::arg("buf") = py::none());
  m.def("scale_", &scale_);
  m.def("gemm", &gemm, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("bias"), py::arg("M"), py::arg("N"),
        py::arg("K"), py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("transA") = false,
        py::arg("transB") = false, py::arg("sA") = 0, py::arg("sB") = 0, py::arg("sC") = 0, py::arg("batch") = 1,
        py::arg("alpha") = 1.0, py::arg("beta") = 0.0, py::arg("bias_mode") = 0, py::arg("relu") = false,
        py::arg("atomic") = false);
  m.def("xent_fwd", &xent_fwd);
  m.def("xent_bwd", &xent_bwd);
  m.def("log_softmax_fwd", &log_softmax_fwd);
  m.def("log_softmax_bwd", &log_softmax_bwd);
  m.def("relu_fwd", &relu_fwd);
  m.def("relu_bwd", &relu_bwd);
  m.def("pool2_fwd", &pool2_fwd);
  m.def("pool2_bwd", &pool2_bwd);
  m.def("im2col", &im2col);
  m.def("col2im", &col2im);
  m.def("bias_grad_nchw", &bias_grad_nchw);
  m.def("colsum", &colsum);
  m.def("gather_rows", &gather_rows);
}
