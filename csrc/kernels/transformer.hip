// Transformer (GPT-2) kernels for gfx950: LayerNorm fwd/bwd, tanh-GELU fwd/bwd, fused vocab
// softmax-cross-entropy (loss + dlogits in one pass pair), token+position embedding fwd/bwd, and
// the AdamW step on bf16 model weights with fp32 master weights (+ device-side grad-norm clipping).
//
// All activations/weights are bf16 (raw uint16); statistics and optimizer state are fp32.  Rows are
// processed one wave (64 lanes) per row with 8- or 16-byte vector accesses; per-lane columns are
// fixed (chunk c = lane + 64 j) so LayerNorm's dgamma/dbeta accumulate in registers across rows.
#include "pde_hip.h"
#include "pde_act.h"
#include "pde_bf16.h"
#include "pde_kernels.h"

namespace {

// ---------------------------------------------------------------------------------- LayerNorm
template <int NCH>
// With D != nullptr the row is first summed with D (the residual add of a pre-LN block), rounded to
// bf16 exactly like a separate bf16 add would, written to S, and normalised: one pass instead of an
// elementwise add kernel (read 2, write 1) followed by the LayerNorm (read 1).
__global__ __launch_bounds__(256) void k_ln_fwd(const bf16_t* __restrict__ X, const bf16_t* __restrict__ D,
                                                bf16_t* __restrict__ S, const bf16_t* __restrict__ G,
                                                const bf16_t* __restrict__ Bt, bf16_t* __restrict__ Y,
                                                float* __restrict__ mean_out, float* __restrict__ rstd_out, int N,
                                                int C, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;  // wave-uniform
  const int nc = C >> 2;
  const uint2* xr = reinterpret_cast<const uint2*>(X + (size_t)row * C);
  const uint2* g4 = reinterpret_cast<const uint2*>(G);
  const uint2* b4 = reinterpret_cast<const uint2*>(Bt);
  float v[NCH][4], gg[NCH][4], bb[NCH][4];
  uint2 wx[NCH], wd[NCH], wg[NCH], wb[NCH];
  const uint2* dr = D ? reinterpret_cast<const uint2*>(D + (size_t)row * C) : nullptr;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {  // issue every load first (clamped index, no branch)
    const int c = min(lane + 64 * j, nc - 1);
    wx[j] = xr[c];
    wd[j] = dr ? dr[c] : make_uint2(0u, 0u);
    wg[j] = g4[c];
    wb[j] = b4[c];
  }
  if (D) {  // residual add, rounded to bf16 (the stored residual stream is bf16)
    uint2* sr = reinterpret_cast<uint2*>(S + (size_t)row * C);
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      float a[4], b[4];
      unpack4(wx[j], a);
      unpack4(wd[j], b);
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] += b[e];
      wx[j] = pack4(a);
      if (lane + 64 * j < nc) sr[lane + 64 * j] = wx[j];
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const bool ok = lane + 64 * j < nc;
    unpack4(wx[j], v[j]);
#pragma unroll
    for (int e = 0; e < 4; ++e) s += ok ? v[j][e] : 0.f;
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const bool ok = lane + 64 * j < nc;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[j][e] - mean;
      q += ok ? d * d : 0.f;
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)C + eps);
  uint2* yr = reinterpret_cast<uint2*>(Y + (size_t)row * C);
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = lane + 64 * j;
    unpack4(wg[j], gg[j]);
    unpack4(wb[j], bb[j]);
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (v[j][e] - mean) * rstd * gg[j][e] + bb[j][e];
    if (c < nc) yr[c] = pack4(o);
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// dX = rstd * (gy - mean(gy) - xhat * mean(gy * xhat)) (+ dRes), gy = dY * gamma.
// Block = 4 waves x RPW rows each; dgamma / dbeta partial sums per block -> part[blk][2][C].
template <int NCH>
__global__ __launch_bounds__(256) void k_ln_bwd(const bf16_t* __restrict__ dY, const bf16_t* __restrict__ X,
                                                const float* __restrict__ mean, const float* __restrict__ rstd,
                                                const bf16_t* __restrict__ G, const bf16_t* __restrict__ dRes,
                                                bf16_t* __restrict__ dX, float* __restrict__ part, int N, int C,
                                                int rpw) {
  extern __shared__ float sh[];  // [4][2][C]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nc = C >> 2;
  float gg[NCH][4], dg[NCH][4], db[NCH][4];
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = min(lane + 64 * j, nc - 1);
    unpack4(reinterpret_cast<const uint2*>(G)[c], gg[j]);
#pragma unroll
    for (int e = 0; e < 4; ++e) dg[j][e] = db[j][e] = 0.f;
  }
  const int row0 = blockIdx.x * 4 * rpw;
  // register double buffer: row i+1's loads are in flight while row i is reduced and written
  uint2 wdy[NCH], wx[NCH], wr[NCH];
  float mu = 0.f, rs = 0.f;
  auto load_row = [&](int row, uint2 (&ldy)[NCH], uint2 (&lx)[NCH], uint2 (&lr)[NCH], float& lmu, float& lrs) {
    const uint2* dyr = reinterpret_cast<const uint2*>(dY + (size_t)row * C);
    const uint2* xr = reinterpret_cast<const uint2*>(X + (size_t)row * C);
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int c = min(lane + 64 * j, nc - 1);
      ldy[j] = dyr[c];
      lx[j] = xr[c];
      lr[j] = dRes ? reinterpret_cast<const uint2*>(dRes + (size_t)row * C)[c] : make_uint2(0u, 0u);
    }
    lmu = mean[row];
    lrs = rstd[row];
  };
  if (row0 + w < N) load_row(row0 + w, wdy, wx, wr, mu, rs);
  for (int i = 0; i < rpw; ++i) {
    const int row = row0 + w + 4 * i;
    if (row >= N) break;  // wave-uniform
    uint2 ndy[NCH], nx[NCH], nr[NCH];
    float nmu = 0.f, nrs = 0.f;
    const bool more = i + 1 < rpw && row + 4 < N;  // wave-uniform
    if (more) load_row(row + 4, ndy, nx, nr, nmu, nrs);
    float xh[NCH][4], gy[NCH][4];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const bool ok = lane + 64 * j < nc;
      float dy[4], x[4];
      unpack4(wdy[j], dy);
      unpack4(wx[j], x);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xh[j][e] = (x[e] - mu) * rs;
        gy[j][e] = ok ? dy[e] * gg[j][e] : 0.f;
        a += gy[j][e];
        b += gy[j][e] * xh[j][e];
        dg[j][e] += ok ? dy[e] * xh[j][e] : 0.f;
        db[j][e] += ok ? dy[e] : 0.f;
      }
    }
    a = wave_sum(a) / (float)C;
    b = wave_sum(b) / (float)C;
    uint2* dxr = reinterpret_cast<uint2*>(dX + (size_t)row * C);
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int c = lane + 64 * j;
      float r[4], o[4];
      unpack4(wr[j], r);
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = rs * (gy[j][e] - a - xh[j][e] * b) + r[e];
      if (c < nc) dxr[c] = pack4(o);
    }
    if (more) {
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        wdy[j] = ndy[j];
        wx[j] = nx[j];
        wr[j] = nr[j];
      }
      mu = nmu;
      rs = nrs;
    }
  }
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = lane + 64 * j;
    if (c < nc) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sh[(w * 2 + 0) * C + 4 * c + e] = dg[j][e];
        sh[(w * 2 + 1) * C + 4 * c + e] = db[j][e];
      }
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 2 * C; k += 256) {
    const float s = sh[k] + sh[2 * C + k] + sh[4 * C + k] + sh[6 * C + k];
    part[(size_t)blockIdx.x * 2 * C + k] = s;
  }
}

// Sum per-block partials: out[k] = sum_b part[b][k], k < 2C; writes dgamma | dbeta as bf16 (or
// accumulates into them when accumulate != 0).  Block = 64 columns x 16 row-groups (16 waves, 8
// independent loads each in flight: the pass is latency-bound, it has only 2C/64 blocks).
__global__ __launch_bounds__(1024) void k_ln_reduce(const float* __restrict__ part, int nblk, int C2,
                                                    bf16_t* __restrict__ dG, bf16_t* __restrict__ dB, int C,
                                                    int accumulate) {
  __shared__ float sh[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + lane;
  const int kc = min(k, C2 - 1);
  float a[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) a[u] = 0.f;
  int b = w;
  for (; b + 112 < nblk; b += 128) {    // 8 rows in flight: 512 partial rows in 4 round trips
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(b + 16 * u) * C2 + kc];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += v[u];
  }
  {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = b + 16 * u < nblk ? part[(size_t)(b + 16 * u) * C2 + kc] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += v[u];
  }
  sh[w][lane] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (w == 0 && k < C2) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) t += sh[r][lane];
    bf16_t* dst = k < C ? dG + k : dB + (k - C);
    if (accumulate) t += bf2f(*dst);
    *dst = f2bf(t);
  }
}

// ---------------------------------------------------------------------------------- GELU (tanh)
__global__ __launch_bounds__(256) void k_gelu_fwd(const uint4* __restrict__ X, uint4* __restrict__ Y, int64_t n8) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8];
    unpack8(X[i], v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = gelu_t(v[e], nullptr);
    Y[i] = pack8(v);
  }
}

__global__ __launch_bounds__(256) void k_gelu_bwd(const uint4* __restrict__ dY, const uint4* __restrict__ X,
                                                  uint4* __restrict__ dX, int64_t n8) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float x[8], g[8];
    unpack8(X[i], x);
    unpack8(dY[i], g);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float d;
      gelu_t(x[e], &d);
      g[e] *= d;
    }
    dX[i] = pack8(g);
  }
}

// ---------------------------------------------------------------------------------- softmax-CE
// One block per row of logits [N, Vp] (bf16).  Pass 1: online max / sum-exp over the V real columns;
// pass 2 overwrites the row IN PLACE with dlogits = (softmax - onehot) * scale (padding columns -> 0).
// Target < 0 = ignore_index: loss 0, zero gradient.
__device__ __forceinline__ void ms_combine(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
  m = mn;
}

// Register-resident variant (rows of <= 256 * NJ 16-byte chunks: GPT-2's 50304-wide padded vocab is
// 6288): a thread's NJ chunks of the row are loaded ONCE, all in flight together, and both the
// softmax statistics and the dlogits come from registers -- the two-pass kernel below reads each
// 100 KB row twice (the second time mostly from the last-level cache) for 3 row-sized transfers;
// this one moves 2 (read + write).
template <int NJ>
__global__ __launch_bounds__(256) void k_xent_bf16_reg(bf16_t* __restrict__ L, const int64_t* __restrict__ tgt,
                                                       int Vp, int V, float scale, float* __restrict__ loss_rows,
                                                       int write_grad) {
  __shared__ float shm[4], shs[4];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint4* Lr = reinterpret_cast<uint4*>(L + (size_t)row * Vp);
  const int nch = Vp >> 3;
  const int64_t t = tgt[row];
  const int t32 = (t >= 0 && t < V) ? (int)t : -1;
  uint4 q[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = tid + 256 * j;
    q[j] = c < nch ? Lr[c] : make_uint4(0u, 0u, 0u, 0u);
  }
  float m = -INFINITY, s = 0.f, xt = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col0 = (tid + 256 * j) * 8;
    float v[8];
    unpack8(q[j], v);
    float bm = -INFINITY;
#pragma unroll
    for (int e = 0; e < 8; ++e) bm = fmaxf(bm, col0 + e < V ? v[e] : -INFINITY);
    float bs = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bs += col0 + e < V ? __expf(v[e] - bm) : 0.f;
      xt += col0 + e == t32 ? v[e] : 0.f;
    }
    ms_combine(m, s, bm, bs);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    ms_combine(m, s, m2, s2);
    xt += __shfl_xor(xt, o, 64);
  }
  __shared__ float shx[4];
  if (lane == 0) {
    shm[w] = m;
    shs[w] = s;
    shx[w] = xt;
  }
  __syncthreads();
  m = shm[0];
  s = shs[0];
#pragma unroll
  for (int k = 1; k < 4; ++k) ms_combine(m, s, shm[k], shs[k]);
  xt = (shx[0] + shx[1]) + (shx[2] + shx[3]);
  const float lse = m + __logf(s);
  const bool valid = t >= 0 && t < V;
  if (tid == 0) loss_rows[row] = valid ? lse - xt : 0.f;
  if (!write_grad) return;
  const float sc = valid ? scale : 0.f;
  // opaque to the optimiser: the pass-1 unpacked floats are re-derived from the packed words
  // (2 VGPRs per 4 values) instead of being kept live across the reduction (248 -> fewer VGPRs)
#pragma unroll
  for (int j = 0; j < NJ; ++j) asm volatile("" : "+v"(q[j].x), "+v"(q[j].y), "+v"(q[j].z), "+v"(q[j].w));
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = tid + 256 * j;
    if (c < nch) {
      float v[8];
      unpack8(q[j], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int col = c * 8 + e;
        const float p = col < V ? __expf(v[e] - lse) : 0.f;
        v[e] = (p - (col == t32 ? 1.f : 0.f)) * sc;
      }
      Lr[c] = pack8(v);
    }
  }
}

// One exp per logit instead of ~2.25 (k_xent_bf16_reg: an online max/sum with per-chunk rescaling,
// then exp(v - lse) again for the gradient; v_exp_f32 is a quarter-rate op and the kernel was
// VALU-bound above its 3.3 GB HBM floor).  Pass 0 takes the row max M from the register-resident
// row; pass 1 forms q = 2^15 exp(v - M) once (raw v_exp_f32 of v log2e - M log2e + 15 <= 15), sums it
// (S = 2^15 s), and keeps it as packed fp16 in the row's registers: q <= 2^15 < the fp16 maximum, and
// the 2^15 shift keeps every p >= 2^-39 out of fp16's subnormal range (p ~ 2e-5 of a near-uniform
// 50257-way row would otherwise sit below 6.1e-5 with a 6e-8 spacing and, rounded toward zero, bias the
// non-target gradients low); pass 2 writes q * (scale / S) -- no exp -- and the owner of the
// target column then rewrites that one gradient exactly, exp(x_t - lse) - 1 (no cancellation through
// the fp16 copy).  No per-element masking: k_xent_pad_fill first sets the vocab padding [V, Vp) of
// every row to -inf (exp -> 0, ignored by the max), and the launcher requires Vp - V >= 8 so the
// clamped duplicate loads of lanes past the row end are copies of a fully padded chunk.
__global__ __launch_bounds__(256) void k_xent_pad_fill(bf16_t* __restrict__ L, int N, int Vp, int V) {
  const int pad = Vp - V;
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= (int64_t)N * pad) return;
  const int64_t row = i / pad;
  L[row * Vp + V + (i - row * pad)] = (bf16_t)0xFF80u;   // -inf
}

template <int NJ>
__global__ __launch_bounds__(256, 2) void k_xent_bf16_reg2(bf16_t* __restrict__ L, const int64_t* __restrict__ tgt,
                                                           int Vp, int V, float scale, float* __restrict__ loss_rows,
                                                           int write_grad) {
  __shared__ float shr[4], shx;
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint4* Lr = reinterpret_cast<uint4*>(L + (size_t)row * Vp);
  const int nch = Vp >> 3;
  const int64_t t = tgt[row];
  const bool valid = t >= 0 && t < V;
  const int t32 = valid ? (int)t : -1;
  const bool owner = valid && (t32 >> 3) % 256 == tid;   // this thread holds the target column
  uint4 q[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j)   // unconditional (see above); 32-bit offsets from the uniform row base
    q[j] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(Lr) +
                                           (uint32_t)min(tid + 256 * j, nch - 1) * 16u);
  // pass 0: row max
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    float v[8];
    unpack8(q[j], v);
#pragma unroll
    for (int e = 0; e < 8; ++e) mx = fmaxf(mx, v[e]);
    __builtin_amdgcn_sched_barrier(0);               // chunk by chunk: the row stays packed (q only)
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if (lane == 0) shr[w] = mx;
  float xt = 0.f;
  if (owner) {   // the target logit: one (L2-hit) load -- selecting it from q would index q dynamically
    xt = bf2f(L[(size_t)row * Vp + t32]);                // and push the whole row array to scratch
    shx = xt;
  }
  __syncthreads();
  const float M = fmaxf(fmaxf(shr[0], shr[1]), fmaxf(shr[2], shr[3]));
  const float L2E = 1.4426950408889634f, mb = M * L2E;
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    float v[8];
    unpack8(q[j], v);
    float pj[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      pj[e] = __builtin_amdgcn_exp2f(fmaf(v[e], L2E, 15.f - mb));   // 2^15 p
      sum += pj[e];
    }
    uint32_t h[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      h[k] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(pj[2 * k], pj[2 * k + 1]));
    q[j] = make_uint4(h[0], h[1], h[2], h[3]);
    __builtin_amdgcn_sched_barrier(0);
  }
  // lanes past the row end summed a duplicate of the last (fully padded, p = 0) chunk: no correction
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  __syncthreads();                                   // every wave has read the max from shr
  if (lane == 0) shr[w] = sum;
  __syncthreads();
  const float s = (shr[0] + shr[1]) + (shr[2] + shr[3]);        // 2^15 x the softmax denominator
  const float lse = M + __logf(s) - 10.397207708399179f;         // - 15 ln 2
  if (tid == 0) loss_rows[row] = valid ? lse - shx : 0.f;
  if (!write_grad) return;
  const float sc = valid ? scale : 0.f, f = sc / s;
  int tid2 = tid;                                    // opaque copy: the store offsets are recomputed
  asm volatile("" : "+v"(tid2));                     // here, not kept live (spilled) from the loads
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = tid2 + 256 * j;
    float g[8];
    const uint32_t hw[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const auto hv = __builtin_bit_cast(__fp16 __attribute__((ext_vector_type(2))), hw[k]);
      g[2 * k] = (float)hv[0] * f;
      g[2 * k + 1] = (float)hv[1] * f;
    }
    if (c < nch) Lr[c] = pack8(g);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (owner) L[(size_t)row * Vp + t32] = f2bf((__expf(xt - lse) - 1.f) * sc);   // program order: after its chunk
}

__global__ __launch_bounds__(256) void k_xent_bf16(bf16_t* __restrict__ L, const int64_t* __restrict__ tgt, int Vp,
                                                   int V, float scale, float* __restrict__ loss_rows,
                                                   int write_grad) {
  __shared__ float shm[4], shs[4];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint4* Lr = reinterpret_cast<uint4*>(L + (size_t)row * Vp);
  const int nch = Vp >> 3;
  const int64_t t = tgt[row];
  const float xt = (t >= 0 && t < V) ? bf2f(L[(size_t)row * Vp + t]) : 0.f;
  float m = -INFINITY, s = 0.f;
  int c = tid;
  for (; c + 768 < nch; c += 1024) {  // 4 loads in flight per thread
    uint4 q[4] = {Lr[c], Lr[c + 256], Lr[c + 512], Lr[c + 768]};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float v[8];
      unpack8(q[u], v);
      const int col0 = (c + 256 * u) * 8;
      float bm = -INFINITY;
#pragma unroll
      for (int e = 0; e < 8; ++e) bm = fmaxf(bm, col0 + e < V ? v[e] : -INFINITY);
      float bs = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) bs += col0 + e < V ? __expf(v[e] - bm) : 0.f;
      ms_combine(m, s, bm, bs);
    }
  }
  for (; c < nch; c += 256) {
    float v[8];
    unpack8(Lr[c], v);
    const int col0 = c * 8;
    float bm = -INFINITY;
#pragma unroll
    for (int e = 0; e < 8; ++e) bm = fmaxf(bm, col0 + e < V ? v[e] : -INFINITY);
    float bs = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) bs += col0 + e < V ? __expf(v[e] - bm) : 0.f;
    ms_combine(m, s, bm, bs);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    ms_combine(m, s, m2, s2);
  }
  if (lane == 0) {
    shm[w] = m;
    shs[w] = s;
  }
  __syncthreads();
  m = shm[0];
  s = shs[0];
#pragma unroll
  for (int k = 1; k < 4; ++k) ms_combine(m, s, shm[k], shs[k]);
  const float lse = m + __logf(s);
  const bool valid = t >= 0 && t < V;
  if (tid == 0) loss_rows[row] = valid ? lse - xt : 0.f;
  if (!write_grad) return;
  const float sc = valid ? scale : 0.f;
  for (c = tid; c < nch; c += 256) {
    float v[8];
    unpack8(Lr[c], v);
    const int col0 = c * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int col = col0 + e;
      const float p = col < V ? __expf(v[e] - lse) : 0.f;
      v[e] = (p - (col == t ? 1.f : 0.f)) * sc;
    }
    Lr[c] = pack8(v);
  }
}

// ---------------------------------------------------------------------------------- embeddings
__global__ __launch_bounds__(256) void k_embed_fwd(const int64_t* __restrict__ idx, const bf16_t* __restrict__ wte,
                                                   const bf16_t* __restrict__ wpe, bf16_t* __restrict__ out, int N,
                                                   int T, int C) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const int64_t tok = idx[row];
  const int pos = row % T;
  const uint2* a = reinterpret_cast<const uint2*>(wte + (size_t)tok * C);
  const uint2* b = reinterpret_cast<const uint2*>(wpe + (size_t)pos * C);
  uint2* o = reinterpret_cast<uint2*>(out + (size_t)row * C);
  for (int c = lane; c < (C >> 2); c += 64) {
    float x[4], y[4];
    unpack4(a[c], x);
    unpack4(b[c], y);
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] += y[e];
    o[c] = pack4(x);
  }
}

// dwpe[t, :] = sum_b dX[b*T + t, :]  (thread per (t, 4-column chunk); no atomics)
__global__ __launch_bounds__(256) void k_embed_bwd_pos(const bf16_t* __restrict__ dX, bf16_t* __restrict__ dwpe,
                                                       int N, int T, int C, int accumulate) {
  const int nc = C >> 2;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= T * nc) return;
  const int t = i / nc, c = i % nc;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int r = t; r < N; r += T) {
    float x[4];
    unpack4(reinterpret_cast<const uint2*>(dX + (size_t)r * C)[c], x);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] += x[e];
  }
  uint2* d = reinterpret_cast<uint2*>(dwpe + (size_t)t * C) + c;
  if (accumulate) {
    float o[4];
    unpack4(*d, o);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] += o[e];
  }
  *d = pack4(acc);
}

// token rows: fp32 atomics into a scratch table + a per-row touched flag
__global__ __launch_bounds__(256) void k_embed_bwd_tok(const bf16_t* __restrict__ dX, const int64_t* __restrict__ idx,
                                                       float* __restrict__ acc, uint8_t* __restrict__ touched, int N,
                                                       int C) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const int64_t tok = idx[row];
  if (lane == 0) touched[tok] = 1;
  float* a = acc + (size_t)tok * C;
  // one float per lane and instruction, lanes on consecutive addresses: every atomic wave-instruction
  // adds 256 contiguous bytes (full atomic rate; the 4-values-per-lane form hit 16-byte strides)
  const bf16_t* x = dX + (size_t)row * C;
  for (int c = lane; c < C; c += 64) atomicAdd(a + c, bf2f(x[c]));
}

// dwte[v] += acc[v] for touched rows; resets acc / touched for the next step (no memset needed)
__global__ __launch_bounds__(256) void k_embed_tok_merge(float* __restrict__ acc, uint8_t* __restrict__ touched,
                                                         bf16_t* __restrict__ dwte, int Vp, int C) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= Vp || !touched[row]) return;
  float4* a = reinterpret_cast<float4*>(acc + (size_t)row * C);
  uint2* d = reinterpret_cast<uint2*>(dwte + (size_t)row * C);
  for (int c = lane; c < (C >> 2); c += 64) {
    float4 v = a[c];
    float o[4];
    unpack4(d[c], o);
    o[0] += v.x; o[1] += v.y; o[2] += v.z; o[3] += v.w;
    d[c] = pack4(o);
    a[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (lane == 0) touched[row] = 0;
}

// ---------------------------------------------------------------------------------- optimizer
// sum of squares of a bf16 buffer (times scale^2) -> out[0].  Deterministic (bit-identical run to
// run and across data-parallel ranks holding identical gradients, so clipped replicas never drift):
// block b writes its partial to out[1 + b], one block then sums the partials in a fixed order.
constexpr int kSumsqMaxBlocks = 1024;

__global__ __launch_bounds__(256) void k_sumsq_bf16(const uint4* __restrict__ g, int64_t n8, float* __restrict__ out) {
  // 16-byte loads, four in flight per thread before any is reduced (the 8-byte serial version ran
  // at ~3.3 TB/s over GPT-2's 249 MB of gradients)
  __shared__ float sh[4];
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += 4 * stride) {
    uint4 w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) w[u] = i + u * stride < n8 ? g[i + u * stride] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float v[8];
      unpack8(w[u], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[u] += v[e] * v[e];
    }
  }
  float t = (s[0] + s[1]) + (s[2] + s[3]);
  t = wave_sum(t);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) out[1 + blockIdx.x] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// step_inc (nullable): the optimizer's device step count, advanced here (the launch right before the
// optimizer's, one block) instead of by a separate ATen add kernel per step
__global__ __launch_bounds__(256) void k_sumsq_finish(float* __restrict__ out, int nparts, float scale,
                                                      float* __restrict__ step_inc) {
  __shared__ float sh[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) s += out[1 + i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = ((sh[0] + sh[1]) + (sh[2] + sh[3])) * scale * scale;
    if (step_inc) *step_inc += 1.f;
  }
}

// AdamW (torch semantics, decoupled decay) on fp32 master weights; writes the bf16 model copy.
// decay_blk (nullable): per-64-element flag (flat layouts align every parameter to 64 elements).
// clip_sumsq (nullable): device sum of squared (scaled) grads -> coef = min(1, max_norm / (norm + 1e-6)).
__global__ __launch_bounds__(256) void k_adamw_master(float* __restrict__ master, uint2* __restrict__ p16,
                                                      const uint2* __restrict__ g16, float4* __restrict__ m4,
                                                      float4* __restrict__ v4, int64_t n4, float lr, float b1,
                                                      float b2, float eps, float wd, float grad_scale, int step,
                                                      const uint8_t* __restrict__ decay_blk,
                                                      const float* __restrict__ clip_sumsq, float max_norm,
                                                      const float* __restrict__ step_dev) {
  float gs = grad_scale;
  if (step_dev) step = (int)*step_dev;               // capturable mode: the step count lives on the device
  if (clip_sumsq) {
    const float norm = sqrtf(*clip_sumsq);
    gs *= fminf(1.f, max_norm / (norm + 1e-6f));
  }
  const float bc1 = 1.f - powf(b1, (float)step);
  const float bc2 = 1.f - powf(b2, (float)step);
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  // 28 B of HBM traffic per parameter, each byte touched once (the state is GBs, far past L2 / MALL):
  // two elements' loads are issued before either is used (more bytes in flight per thread), and the
  // fp32 streams bypass the caches (non-temporal); the bf16 weights are read by the next forward.
  typedef float nt4 __attribute__((ext_vector_type(4)));
  typedef unsigned int nt2 __attribute__((ext_vector_type(2)));
  nt4* mp = reinterpret_cast<nt4*>(master);
  nt4* mq = reinterpret_cast<nt4*>(m4);
  nt4* vq = reinterpret_cast<nt4*>(v4);
  const nt2* gq = reinterpret_cast<const nt2*>(g16);
  auto update = [&](int64_t i, nt4 p, nt4 m, nt4 v, nt2 graw) {
    float g[4];
    unpack4(make_uint2(graw.x, graw.y), g);
    const float dec = (decay_blk == nullptr || decay_blk[i >> 4]) ? (1.f - lr * wd) : 1.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gg = g[e] * gs;
      p[e] *= dec;
      m[e] = m[e] + (gg - m[e]) * (1.f - b1);
      v[e] = v[e] * b2 + (1.f - b2) * gg * gg;
      const float denom = sqrtf(v[e]) / bc2s + eps;
      p[e] -= step_size * m[e] / denom;
    }
    __builtin_nontemporal_store(p, mp + i);
    __builtin_nontemporal_store(m, mq + i);
    __builtin_nontemporal_store(v, vq + i);
    const float pf[4] = {p[0], p[1], p[2], p[3]};
    p16[i] = pack4(pf);
  };
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += 2 * stride) {
    const int64_t j = i + stride;
    const nt4 p0 = __builtin_nontemporal_load(mp + i), m0 = __builtin_nontemporal_load(mq + i),
              v0 = __builtin_nontemporal_load(vq + i);
    const nt2 g0 = __builtin_nontemporal_load(gq + i);
    if (j < n4) {
      const nt4 p1 = __builtin_nontemporal_load(mp + j), m1 = __builtin_nontemporal_load(mq + j),
                v1 = __builtin_nontemporal_load(vq + j);
      const nt2 g1 = __builtin_nontemporal_load(gq + j);
      update(i, p0, m0, v0, g0);
      update(j, p1, m1, v1, g1);
    } else {
      update(i, p0, m0, v0, g0);
    }
  }
}

__global__ __launch_bounds__(256) void k_f32_to_bf16(const float4* __restrict__ x, uint2* __restrict__ y, int64_t n4) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 v = x[i];
    y[i] = pack4(&v.x);
  }
}

// x *= s[0] in place (bf16, 8 elements per thread; the scale is a device scalar -- a loss gradient --
// so there is no host read). Replaces torch's `mul_(0-dim fp32 cuda tensor)`, which takes the
// non-vectorised mixed-dtype path (41 us on the 12.6 MB GPT-2 LM-head dgrad vs ~4 us here).
__global__ __launch_bounds__(256) void k_scale_bf16(uint4* __restrict__ x, const float* __restrict__ s, int64_t n8) {
  const float a = *s;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8];
    unpack8(x[i], v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= a;
    x[i] = pack8(v);
  }
}

// Column sums of a [N, C] bf16 matrix (bias gradients): grid (ceil(C/256), RS); a block sums 256
// columns (32 x 8-column chunks) over its N/RS rows with 8 row-lanes -> part[RS][C] fp32; then
// k_colsum_finish folds the RS partial rows into bf16.
__global__ __launch_bounds__(256) void k_colsum_bf16_part(const uint4* __restrict__ X, int N, int C,
                                                          float* __restrict__ part) {
  __shared__ float sh[8][256];
  const int CP = C >> 3;
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c8 = min(blockIdx.x * 32 + cl, CP - 1);
  const int rows = (N + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * rows, r1 = min(N, r0 + rows);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int r = r0 + rl;
  for (; r + 24 < r1; r += 32) {
    uint4 q[4] = {X[(size_t)r * CP + c8], X[(size_t)(r + 8) * CP + c8], X[(size_t)(r + 16) * CP + c8],
                  X[(size_t)(r + 24) * CP + c8]};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float v[8];
      unpack8(q[u], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
  }
  for (; r < r1; r += 8) {
    float v[8];
    unpack8(X[(size_t)r * CP + c8], v);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += v[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) sh[rl][cl * 8 + e] = acc[e];
  __syncthreads();
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col < C) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += sh[k][threadIdx.x];
    part[(size_t)blockIdx.y * C + col] = s;
  }
}

// 64 columns per block; the 4 waves stride over the RS partial rows with 4 independent
// accumulators each (a single thread walking all RS rows was a 64-deep dependent-load chain).
__global__ __launch_bounds__(256) void k_colsum_finish(const float* __restrict__ part, int RS, int C,
                                                       bf16_t* __restrict__ out) {
  __shared__ float sh[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = min(blockIdx.x * 64 + lane, C - 1);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int k = w;
  for (; k + 12 < RS; k += 16) {
    s0 += part[(size_t)k * C + c];
    s1 += part[(size_t)(k + 4) * C + c];
    s2 += part[(size_t)(k + 8) * C + c];
    s3 += part[(size_t)(k + 12) * C + c];
  }
  for (; k < RS; k += 4) s0 += part[(size_t)k * C + c];
  sh[w][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (w == 0 && blockIdx.x * 64 + lane < C) out[c] = f2bf(sh[0][lane] + sh[1][lane] + sh[2][lane] + sh[3][lane]);
}

// out[0] = sum(x[0..n)) (one 1024-thread block; n up to a few 1e5 -- loss rows)
__global__ __launch_bounds__(1024) void k_sum_f32(const float* __restrict__ x, int n, float* __restrict__ out,
                                                  float scale) {
  __shared__ float sh[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 1024) s += x[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = threadIdx.x < 16 ? sh[threadIdx.x] : 0.f;
    t = wave_sum(t);
    if (threadIdx.x == 0) out[0] = t * scale;
  }
}

// Next-token batch of a [P][T+1] token pool: x[b] = pool[rows[b]][0:T], y[b] = pool[rows[b]][1:T+1]
// (contiguous model inputs / targets straight from the sampler's rows, one pass, no index_select)
__global__ __launch_bounds__(256) void k_token_batch(const int64_t* __restrict__ pool, const int64_t* __restrict__ rows,
                                                     int T, int64_t* __restrict__ x, int64_t* __restrict__ y) {
  const int b = blockIdx.y;
  const int64_t* src = pool + rows[b] * (int64_t)(T + 1);
  for (int t = blockIdx.x * 256 + threadIdx.x; t < T; t += gridDim.x * 256) {
    x[(int64_t)b * T + t] = src[t];
    y[(int64_t)b * T + t] = src[t + 1];
  }
}

inline int grid_for(int64_t n, int per_block, int cap = 4096) {
  int64_t g = (n + per_block - 1) / per_block;
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

}  // namespace

// ------------------------------------------------------------------------------------ launchers
extern "C" {

hipError_t pde_ln_fwd(const void* X, const void* D, void* S, const void* G, const void* B, void* Y, float* mean,
                      float* rstd, int N, int C, float eps, hipStream_t st) {
  const int nch = (C / 4 + 63) / 64;
  dim3 grid((N + 3) / 4);
#define LNF(K)                                                                                          \
  case K:                                                                                               \
    hipLaunchKernelGGL(k_ln_fwd<K>, grid, dim3(256), 0, st, (const bf16_t*)X, (const bf16_t*)D,          \
                       (bf16_t*)S, (const bf16_t*)G,                                                    \
                       (const bf16_t*)B, (bf16_t*)Y, mean, rstd, N, C, eps);                            \
    break;
  switch (nch) {
    LNF(1) LNF(2) LNF(3) LNF(4) LNF(5) LNF(6) LNF(7) LNF(8)
    default: return hipErrorInvalidValue;
  }
#undef LNF
  return hipGetLastError();
}

// Rows per wave: ~512 blocks of 4 waves (2 blocks per CU) so the memory-bound backward has enough
// waves in flight; the per-block dgamma/dbeta partials (2C floats each) stay small next to dY / X.
static int ln_bwd_rpw(int N) { return (N + 4 * 512 - 1) / (4 * 512); }

int pde_ln_bwd_blocks(int N) {
  const int rpw = ln_bwd_rpw(N);
  return (N + 4 * rpw - 1) / (4 * rpw);
}

hipError_t pde_ln_bwd(const void* dY, const void* X, const float* mean, const float* rstd, const void* G,
                      const void* dRes, void* dX, float* part, void* dG, void* dB, int N, int C, int accumulate,
                      hipStream_t st) {
  const int nch = (C / 4 + 63) / 64;
  const int rpw = ln_bwd_rpw(N);
  const int nblk = (N + 4 * rpw - 1) / (4 * rpw);
  const size_t lds = (size_t)8 * C * sizeof(float);
#define LNB(K)                                                                                          \
  case K:                                                                                               \
    hipLaunchKernelGGL(k_ln_bwd<K>, dim3(nblk), dim3(256), lds, st, (const bf16_t*)dY, (const bf16_t*)X, \
                       mean, rstd, (const bf16_t*)G, (const bf16_t*)dRes, (bf16_t*)dX, part, N, C, rpw); \
    break;
  switch (nch) {
    LNB(1) LNB(2) LNB(3) LNB(4) LNB(5) LNB(6) LNB(7) LNB(8)
    default: return hipErrorInvalidValue;
  }
#undef LNB
  hipLaunchKernelGGL(k_ln_reduce, dim3((2 * C + 63) / 64), dim3(1024), 0, st, part, nblk, 2 * C, (bf16_t*)dG,
                     (bf16_t*)dB, C, accumulate);
  return hipGetLastError();
}

hipError_t pde_gelu_fwd(const void* X, void* Y, int64_t n, hipStream_t st) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(k_gelu_fwd, dim3(grid_for(n8, 256)), dim3(256), 0, st, (const uint4*)X, (uint4*)Y, n8);
  return hipGetLastError();
}

hipError_t pde_gelu_bwd(const void* dY, const void* X, void* dX, int64_t n, hipStream_t st) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(k_gelu_bwd, dim3(grid_for(n8, 256)), dim3(256), 0, st, (const uint4*)dY, (const uint4*)X,
                     (uint4*)dX, n8);
  return hipGetLastError();
}

hipError_t pde_xent_bf16(void* logits, const int64_t* tgt, int N, int Vp, int V, float scale, float* loss_rows,
                         int write_grad, hipStream_t st) {
  if ((Vp >> 3) <= 256 * 25 && Vp >= 256 * 8 * 16) {   // wide rows (GPT-2 vocab): one read, one write
    const char* env = getenv("PDE_XENT_V");            // 1: the two-exp online-softmax kernel (A/B)
    // loss-only calls (write_grad = 0) keep the logits unmodified: the old kernel (no padding fill)
    if ((env && atoi(env) == 1) || Vp - V < 8 || !write_grad)
      hipLaunchKernelGGL(k_xent_bf16_reg<25>, dim3(N), dim3(256), 0, st, (bf16_t*)logits, tgt, Vp, V, scale,
                         loss_rows, write_grad);
    else {
      const int64_t np = (int64_t)N * (Vp - V);
      hipLaunchKernelGGL(k_xent_pad_fill, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, st, (bf16_t*)logits, N, Vp,
                         V);
      hipLaunchKernelGGL(k_xent_bf16_reg2<25>, dim3(N), dim3(256), 0, st, (bf16_t*)logits, tgt, Vp, V, scale,
                         loss_rows, write_grad);
    }
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_xent_bf16, dim3(N), dim3(256), 0, st, (bf16_t*)logits, tgt, Vp, V, scale, loss_rows,
                     write_grad);
  return hipGetLastError();
}

hipError_t pde_embed_fwd(const int64_t* idx, const void* wte, const void* wpe, void* out, int N, int T, int C,
                         hipStream_t st) {
  hipLaunchKernelGGL(k_embed_fwd, dim3((N + 3) / 4), dim3(256), 0, st, idx, (const bf16_t*)wte, (const bf16_t*)wpe,
                     (bf16_t*)out, N, T, C);
  return hipGetLastError();
}

hipError_t pde_embed_bwd(const void* dX, const int64_t* idx, void* dwte, void* dwpe, float* acc, uint8_t* touched,
                         int N, int T, int C, int Vp, int accumulate_pos, hipStream_t st) {
  hipLaunchKernelGGL(k_embed_bwd_pos, dim3((T * (C / 4) + 255) / 256), dim3(256), 0, st, (const bf16_t*)dX,
                     (bf16_t*)dwpe, N, T, C, accumulate_pos);
  hipLaunchKernelGGL(k_embed_bwd_tok, dim3((N + 3) / 4), dim3(256), 0, st, (const bf16_t*)dX, idx, acc, touched, N,
                     C);
  hipLaunchKernelGGL(k_embed_tok_merge, dim3((Vp + 3) / 4), dim3(256), 0, st, acc, touched, (bf16_t*)dwte, Vp, C);
  return hipGetLastError();
}

hipError_t pde_sumsq_bf16(const void* g, int64_t n, float scale, float* out, float* step_inc, hipStream_t st) {
  if (n % 8) return hipErrorInvalidValue;
  const int64_t n8 = n / 8;
  const int grid = grid_for(n8, 256 * 4, kSumsqMaxBlocks);
  hipLaunchKernelGGL(k_sumsq_bf16, dim3(grid), dim3(256), 0, st, (const uint4*)g, n8, out);
  hipLaunchKernelGGL(k_sumsq_finish, dim3(1), dim3(256), 0, st, out, grid, scale, step_inc);
  return hipGetLastError();
}

hipError_t pde_adamw_master(float* master, void* p16, const void* g16, float* m, float* v, int64_t n, float lr,
                            float b1, float b2, float eps, float wd, float grad_scale, int step,
                            const uint8_t* decay_blk, const float* clip_sumsq, float max_norm, const float* step_dev,
                            hipStream_t st) {
  const int64_t n4 = n / 4;
  hipLaunchKernelGGL(k_adamw_master, dim3(grid_for(n4, 256, 2048)), dim3(256), 0, st, master, (uint2*)p16,
                     (const uint2*)g16, (float4*)m, (float4*)v, n4, lr, b1, b2, eps, wd, grad_scale, step, decay_blk,
                     clip_sumsq, max_norm, step_dev);
  return hipGetLastError();
}

int pde_colsum_bf16_splits(int C) {
  const int cb = (C + 255) / 256;
  const int rs = 512 / cb;
  return rs < 1 ? 1 : (rs > 128 ? 128 : rs);
}

hipError_t pde_colsum_bf16(const void* x, int N, int C, float* part, void* out, hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  const int rs = pde_colsum_bf16_splits(C);
  hipLaunchKernelGGL(k_colsum_bf16_part, dim3((C + 255) / 256, rs), dim3(256), 0, st, (const uint4*)x, N, C, part);
  hipLaunchKernelGGL(k_colsum_finish, dim3((C + 63) / 64), dim3(256), 0, st, part, rs, C, (bf16_t*)out);
  return hipGetLastError();
}

hipError_t pde_sum_f32(const float* x, int n, float* out, float scale, hipStream_t st) {
  hipLaunchKernelGGL(k_sum_f32, dim3(1), dim3(1024), 0, st, x, n, out, scale);
  return hipGetLastError();
}

hipError_t pde_token_batch(const int64_t* pool, const int64_t* rows, int B, int T, int64_t* x, int64_t* y,
                           hipStream_t st) {
  hipLaunchKernelGGL(k_token_batch, dim3((T + 255) / 256, B), dim3(256), 0, st, pool, rows, T, x, y);
  return hipGetLastError();
}

hipError_t pde_f32_to_bf16(const float* x, void* y, int64_t n, hipStream_t st) {
  const int64_t n4 = n / 4;
  hipLaunchKernelGGL(k_f32_to_bf16, dim3(grid_for(n4, 256)), dim3(256), 0, st, (const float4*)x, (uint2*)y, n4);
  return hipGetLastError();
}

hipError_t pde_scale_bf16(void* x, const float* s, int64_t n, hipStream_t st) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(k_scale_bf16, dim3(grid_for(n8, 256)), dim3(256), 0, st, (uint4*)x, s, n8);
  return hipGetLastError();
}

}  // extern "C"
