// Fused optimizers over flat fp32 buffers (one launch per step for ALL parameters).
//
// Adam / AdamW reproduce torch.optim.Adam's single-tensor math (torch/optim/adam.py:347-460):
//   m = lerp(m, g, 1-b1); v = v*b2 + (1-b2)*g*g
//   p -= (lr / (1-b1^t)) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
// The step counter lives on the device: every block reads t = *step + 1 and the last block to
// arrive publishes *step = t (arrival counter reset in the same block), so the whole optimizer
// step is capturable in a hipGraph and replayable without host involvement.  `bump` = number of
// consecutive int64 counters advanced by the last block (0: none; [0] is the optimizer step);
// bump < 0: the caller's earlier kernel already advanced the counter, t = *step, no fan-in at all.
// grad_scale folds the DDP 1/world_size average (or any loss scale) into the update.
// Optional fused all-reduce (Adam only, the W > 1 "fused" LeNet schedule): the first ar_nvb blocks
// all-reduce the flat range [ar_lo4, n4) (the conv-gradient bucket) across ranks with the xGMI peer
// protocol while the other blocks update [0, ar_lo4); those blocks then wait for the reduction (the
// completing side block publishes the optimizer step t in *ar_epoch) before updating the rest.
// Side blocks have the lowest block ids, so they are dispatched first: no wait can starve them.
// Optional epilogue: repack the LeNet conv2 weight [50][20][5][5] into the [k'][64] layout the
// conv2 forward kernel streams (k' = (kh*5+kw)*20+ci), so no separate repack launch exists.
#include "pde_hip.h"
#include "pde_kernels.h"
#include "pde_lenet.h"
#include "pde_peer_dev.h"
#include "pde_adam.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace {

struct Pack {
  long long off;   // flat offset of conv2.weight, -1 = no repack
  float* dst;      // mode 1: [500][64] (lenet.hip F1); mode 2: the LDS-DMA image of lenet_v2.hip
  int mode;
};

struct Fold1 {
  long long off;   // first element of the canonical gradient (replica 0); -1 = none
  int len;         // elements per replica unit (multiple of 4)
  int nrep;        // replicas (1 = nothing to fold)
  int stride;      // floats between replicas (multiple of 4)
};
struct Fold {      // up to two replicated gradient ranges (LeNet: conv1 atomic replicas, conv2 wgrad slabs)
  Fold1 f[2];
};

// Folded ranges (whole replica sets [off, off + nrep*stride)) are holes of the main index space;
// appended fold blocks own them.  Each canonical float4 gets kLS lanes: lane l sums replicas
// l, l+kLS, ... (all loads in flight at once), a 2-step xor shuffle combines the lanes, and lane l
// then updates element l of the float4 (the old one-thread-per-float4 fold issued 19 loads per
// thread on the last ~27 blocks and ended the kernel 2 us after every other block).
constexpr int kMaxFold = 16;
constexpr int kLS = 4;

struct Holes {
  long long lo[2], len[2];   // in float4 units, sorted, lo = huge when unused
};

__host__ __device__ __forceinline__ bool fold_on(const Fold1& f) { return f.off >= 0 && f.nrep > 1; }

__host__ __device__ __forceinline__ Holes make_holes(const Fold& fd) {
  Holes h{{(long long)1 << 60, (long long)1 << 60}, {0, 0}};
  for (int k = 0; k < 2; ++k) {
    const Fold1& f = fd.f[k];
    if (fold_on(f)) {
      h.lo[k] = f.off / 4;
      h.len[k] = (long long)f.nrep * f.stride / 4;
    }
  }
  if (h.lo[1] < h.lo[0]) {
    const long long a = h.lo[0], b = h.len[0];
    h.lo[0] = h.lo[1]; h.len[0] = h.len[1];
    h.lo[1] = a; h.len[1] = b;
  }
  return h;
}

__device__ __forceinline__ long long hole_map(const Holes& h, long long c) {   // compressed -> real index
  if (c >= h.lo[0]) c += h.len[0];
  if (c >= h.lo[1]) c += h.len[1];
  return c;
}

// fold blocks per range: kLS lanes for each float4 of the canonical slot (stride / 4 float4s)
__host__ __device__ __forceinline__ int fold_blocks(const Fold1& f) {
  return fold_on(f) ? (int)(((long long)f.stride / 4 * kLS + 255) / 256) : 0;
}

struct FoldLane {
  long long e;   // flat element this lane updates (-1: none)
  float g;       // its folded gradient (before grad_scale)
};

// The flat element fold lane (fb, threadIdx.x) updates (-1: none) -- known before any load, so the
// optimizer state of that element is fetched in the same round trip as the replicas.
__device__ __forceinline__ long long fold_elem(const Fold& fd, int fb) {
  const int nb0 = fold_blocks(fd.f[0]);
  const int k = fb < nb0 ? 0 : 1;
  const Fold1& f = fd.f[k];
  const long long j = ((long long)(k ? fb - nb0 : fb) * 256 + threadIdx.x) / kLS;
  return j < f.stride / 4 ? f.off + 4 * j + threadIdx.x % kLS : -1;
}

// fb = fold-block index (0-based over both ranges).  All lanes of the wave take part in the shuffles.
__device__ __forceinline__ FoldLane fold_lane(const Fold& fd, float* __restrict__ g, int fb) {
  const int nb0 = fold_blocks(fd.f[0]);
  const int k = fb < nb0 ? 0 : 1;
  const Fold1& f = fd.f[k];
  const long long j = ((long long)(k ? fb - nb0 : fb) * 256 + threadIdx.x) / kLS;   // float4 in the slot
  const int lane = threadIdx.x % kLS;
  const bool valid = j < f.stride / 4;
  const int nrep = (valid && 4 * j < f.len) ? f.nrep : 1;            // past len: no replicas to add
  const float4* g4 = reinterpret_cast<const float4*>(g) + f.off / 4 + (valid ? j : 0);
  const int s4 = f.stride / 4;
  float4 x[kMaxFold / kLS];
#pragma unroll
  for (int q = 0; q < kMaxFold / kLS; ++q) {
    const int r = lane + q * kLS;
    x[q] = (valid && r < nrep) ? g4[(long long)r * s4] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float4 a = x[0];
#pragma unroll
  for (int q = 1; q < kMaxFold / kLS; ++q) { a.x += x[q].x; a.y += x[q].y; a.z += x[q].z; a.w += x[q].w; }
#pragma unroll
  for (int o = 1; o < kLS; o <<= 1) {
    a.x += __shfl_xor(a.x, o); a.y += __shfl_xor(a.y, o); a.z += __shfl_xor(a.z, o); a.w += __shfl_xor(a.w, o);
  }
  const float mine = lane == 0 ? a.x : lane == 1 ? a.y : lane == 2 ? a.z : a.w;
  return FoldLane{valid ? f.off + 4 * j + lane : -1, mine};
}

__device__ __forceinline__ void pack_store(const Pack& pk, long long i, float v) {
  const long long e64 = i - pk.off;
  if (pk.off >= 0 && e64 >= 0 && e64 < 25000) {
    const int e = (int)e64;                 // 32-bit index math (64-bit division is ~100 instructions)
    if (pk.mode == 2) {
      pk.dst[pde_lenet_wp_index(e)] = v;
    } else {
      const int co = e / 500, k = e - co * 500, ci = k / 25, r = k - ci * 25;
      pk.dst[(r * 20 + ci) * 64 + co] = v;
    }
  }
}

// The arrival add carries a data dependency on the step value this block read, so it cannot be
// issued before that read returned: no block can observe the bumped counter.
__device__ __forceinline__ bool last_block(unsigned* arrive, long long t) {
  __shared__ int is_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = atomicAdd(arrive, t > 0 ? 1u : 2u);
    is_last = (prev == gridDim.x - 1);
  }
  __syncthreads();
  return is_last != 0;
}

struct FusedAR {
  pde::PeerDev pd;
  long long lo4;            // first float4 of the all-reduced range (range = [lo4, n4))
  long long* epoch;         // completion word: the optimizer step t of the reduced call
  int nvb;                  // side blocks (0 = no fused all-reduce)
  int two;
};

__device__ __forceinline__ void wait_epoch(const long long* epoch, long long t, const pde::PeerDev& pd) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    // relaxed polling (an acquire per poll would invalidate the L2 under the side blocks' feet),
    // one acquire once the completion word is seen
    while (__hip_atomic_load(epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != t) {
      __builtin_amdgcn_s_sleep(2);
      if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > 2 * pd.timeout) break;   // failure latched by the side blocks
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

template <bool PROF, bool NTP>
__global__ __launch_bounds__(256) void k_adam(float* __restrict__ p, float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v, long long n4,
                                              float lr, float b1, float b2, float eps, float wd, int decoupled,
                                              float grad_scale, long long* __restrict__ step,
                                              unsigned* __restrict__ arrive, int bump, Pack pk, Fold fd, FusedAR ar,
                                              unsigned long long* __restrict__ prof) {
  if constexpr (PROF) {
    if (threadIdx.x == 0) prof[(size_t)blockIdx.x * 8] = __builtin_amdgcn_s_memrealtime();
  }
  const long long t = bump < 0 ? *step : *step + 1;   // bump < 0: counter pre-advanced by an earlier kernel
  __shared__ uint32_t lds2[2];
  const Holes holes = make_holes(fd);
  const long long n4c = n4 - holes.len[0] - holes.len[1];   // compressed index space (replicas skipped)
  const int nmain = (int)gridDim.x - fold_blocks(fd.f[0]) - fold_blocks(fd.f[1]);
  long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x, istride = (long long)nmain * blockDim.x;
  long long lo = 0, hi = n4c;                         // pass 1 range; pass 2 = [ar.lo4, n4c) after the wait
  if (ar.nvb > 0) {
    if ((int)blockIdx.x < ar.nvb) {
      if (pde::peer_ar_f32_vblock(ar.pd, g + 4 * ar.lo4, g + 4 * ar.lo4, 4 * (n4 - ar.lo4), 1.f, blockIdx.x,
                                  ar.nvb, ar.two != 0, lds2))
        __hip_atomic_store(ar.epoch, t, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      i0 = n4;                                        // no parameter work in side blocks
    } else {
      i0 = (long long)(blockIdx.x - ar.nvb) * blockDim.x + threadIdx.x;
      istride = (long long)(nmain - ar.nvb) * blockDim.x;
      hi = ar.lo4;
    }
  }
  const float bc1 = 1.f - powf(b1, (float)t);
  const float bc2 = 1.f - powf(b2, (float)t);
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  const float omb1 = 1.f - b1, omb2 = 1.f - b2;
  float4* p4 = reinterpret_cast<float4*>(p);
  float4* g4 = reinterpret_cast<float4*>(g);
  float4* m4 = reinterpret_cast<float4*>(m);
  float4* v4 = reinterpret_cast<float4*>(v);
  const int nfb = fold_blocks(fd.f[0]) + fold_blocks(fd.f[1]);
  const int fb = (int)blockIdx.x - ((int)gridDim.x - nfb);   // >= 0: fold block
  for (int pass = 0; pass < 2; ++pass) {
  if (pass == 1 && fb < 0) {
    if (ar.nvb == 0 || (int)blockIdx.x < ar.nvb) break;   // block-uniform: wait_epoch has barriers
    wait_epoch(ar.epoch, t, ar.pd);                   // the all-reduced range is ready
    lo = ar.lo4;
    hi = n4c;
  }
  if (fb >= 0) {                                     // fold block: its own range, one pass
    if (pass == 1) break;
    if (ar.nvb > 0) wait_epoch(ar.epoch, t, ar.pd);   // the reduced replicas must be complete
    const long long e0 = fold_elem(fd, fb);
    float pa = 0.f, ma = 0.f, va = 0.f;
    if (e0 >= 0) {                                   // issued before the replica loads: one round trip
      pa = p[e0];
      ma = m[e0];
      va = v[e0];
    }
    const FoldLane fl = fold_lane(fd, g, fb);
    if (fl.e >= 0) {
      adam_elem(pa, ma, va, fl.g * grad_scale, lr, wd, decoupled, omb1, omb2, b2, step_size, bc2s, eps);
      if constexpr (NTP) {     // NTP: nothing of this launch is left dirty in the XCD L2s (see below)
        __builtin_nontemporal_store(pa, p + fl.e);
        __builtin_nontemporal_store(ma, m + fl.e);
        __builtin_nontemporal_store(va, v + fl.e);
        __builtin_nontemporal_store(fl.g, g + fl.e);   // p.grad holds the true (folded) gradient
      } else {
        p[fl.e] = pa; m[fl.e] = ma; v[fl.e] = va;
        g[fl.e] = fl.g;                                // p.grad holds the true (folded) gradient
      }
      pack_store(pk, fl.e, pa);
    }
    continue;
  }
  for (long long ic = lo + i0; ic < hi; ic += istride) {
    const long long i = hole_map(holes, ic);
    float4 pp = p4[i], gg = g4[i], mm = m4[i], vv = v4[i];
    float* pa = &pp.x; float* ga = &gg.x; float* ma = &mm.x; float* va = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      adam_elem(pa[j], ma[j], va[j], ga[j] * grad_scale, lr, wd, decoupled, omb1, omb2, b2, step_size, bc2s, eps);
      pack_store(pk, 4 * i + j, pa[j]);
    }
    // the moments are read again only by the next step's Adam: streamed out (non-temporal) rather than
    // left dirty in the XCD L2s for the end-of-kernel write-back that the next kernel waits behind.
    // NTP: the parameters too -- their next readers (the next step's forward kernels) run on other
    // XCDs' L2s anyway, so a dirty line here only lengthens this kernel's end-of-kernel write-back
    typedef float nt_f4 __attribute__((ext_vector_type(4)));
    if constexpr (NTP) __builtin_nontemporal_store(*reinterpret_cast<nt_f4*>(&pp), reinterpret_cast<nt_f4*>(p4 + i));
    else p4[i] = pp;
    __builtin_nontemporal_store(*reinterpret_cast<nt_f4*>(&mm), reinterpret_cast<nt_f4*>(m4 + i));
    __builtin_nontemporal_store(*reinterpret_cast<nt_f4*>(&vv), reinterpret_cast<nt_f4*>(v4 + i));
  }
  }
  if (bump > 0 && last_block(arrive, t) && threadIdx.x == 0) {
    step[0] = t;
    for (int c = 1; c < bump; ++c) step[c] += 1;   // extra device counters (e.g. batch position)
    *arrive = 0u;
  }
  if constexpr (PROF) {
    if (threadIdx.x == 0) prof[(size_t)blockIdx.x * 8 + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

__device__ __forceinline__ void sgd_elem(float& p, float& b, float d, float lr, float momentum, float dampening,
                                         float wd, int nesterov, long long t) {
  if (wd != 0.f) d = d + wd * p;
  if (momentum != 0.f) {
    b = (t == 1) ? d : momentum * b + (1.f - dampening) * d;
    d = nesterov ? d + momentum * b : b;
  }
  p = p - lr * d;
}

// torch.optim.SGD semantics (torch/optim/sgd.py): d_p = g + wd*p; buf = momentum*buf + (1-dampening)*d_p
// (buf = d_p on the first step); d_p = nesterov ? d_p + momentum*buf : buf; p -= lr*d_p.
__global__ __launch_bounds__(256) void k_sgd(float* __restrict__ p, float* __restrict__ g, float* __restrict__ buf,
                                             long long n4, float lr, float momentum, float dampening, float wd,
                                             int nesterov, float grad_scale, long long* __restrict__ step,
                                             unsigned* __restrict__ arrive, int bump, Pack pk, Fold fd) {
  const long long t = bump < 0 ? *step : *step + 1;
  float4* p4 = reinterpret_cast<float4*>(p);
  float4* g4 = reinterpret_cast<float4*>(g);
  float4* b4 = reinterpret_cast<float4*>(buf);
  const Holes holes = make_holes(fd);
  const long long n4c = n4 - holes.len[0] - holes.len[1];
  const int nfb = fold_blocks(fd.f[0]) + fold_blocks(fd.f[1]);
  const int fb = (int)blockIdx.x - ((int)gridDim.x - nfb);
  if (fb >= 0) {                                       // fold block (see fold_lane)
    const FoldLane fl = fold_lane(fd, g, fb);
    if (fl.e >= 0) {
      float pa = p[fl.e], ba = momentum != 0.f ? buf[fl.e] : 0.f;
      sgd_elem(pa, ba, fl.g * grad_scale, lr, momentum, dampening, wd, nesterov, t);
      p[fl.e] = pa;
      if (momentum != 0.f) buf[fl.e] = ba;
      g[fl.e] = fl.g;
      pack_store(pk, fl.e, pa);
    }
  } else {
    const long long istride = (long long)(gridDim.x - nfb) * blockDim.x;
    for (long long ic = (long long)blockIdx.x * blockDim.x + threadIdx.x; ic < n4c; ic += istride) {
      const long long i = hole_map(holes, ic);
      float4 pp = p4[i], gg = g4[i];
      float4 bb = momentum != 0.f ? b4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      float* pa = &pp.x; float* ga = &gg.x; float* ba = &bb.x;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sgd_elem(pa[j], ba[j], ga[j] * grad_scale, lr, momentum, dampening, wd, nesterov, t);
        pack_store(pk, 4 * i + j, pa[j]);
      }
      p4[i] = pp;
      if (momentum != 0.f) b4[i] = bb;
    }
  }
  if (bump > 0 && last_block(arrive, t) && threadIdx.x == 0) {
    step[0] = t;
    for (int c = 1; c < bump; ++c) step[c] += 1;   // extra device counters (e.g. batch position)
    *arrive = 0u;
  }
}

__global__ void k_lenet_pack_w2(const float* __restrict__ w2, float* __restrict__ dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 500 * 64) {
    const int kp = i >> 6, co = i & 63, r = kp / 20, ci = kp % 20;
    dst[i] = co < 50 ? w2[co * 500 + ci * 25 + r] : 0.f;
  }
}

__global__ void k_scale(float* __restrict__ x, long long n, float s) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    x[i] *= s;
}

inline int grid_for(long long n4) {
  long long blocks = (n4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  return (int)blocks;
}

}  // namespace

extern "C" {

hipError_t pde_adam_flat(float* p, float* g, float* m, float* v, long long n, float lr, float b1, float b2,
                         float eps, float wd, int decoupled, float grad_scale, long long* step, unsigned* arrive,
                         int bump, long long pack_off, float* pack_dst, long long fold_off, int fold_len,
                         int fold_nrep, int fold_stride, const void* peer_dev, long long ar_off, long long* ar_epoch,
                         int ar_two, int pack_mode, long long fold2_off, int fold2_len, int fold2_nrep,
                         int fold2_stride, hipStream_t st) {
  if (n % 4) return hipErrorInvalidValue;
  const long long n4 = n / 4;
  FusedAR ar{};
  if (peer_dev != nullptr && ar_epoch != nullptr) {
    if (ar_off % 4 || ar_off < 0 || ar_off >= n) return hipErrorInvalidValue;
    std::memcpy(&ar.pd, peer_dev, sizeof(ar.pd));
    ar.lo4 = ar_off / 4;
    ar.epoch = ar_epoch;
    ar.two = ar_two;
    const long long m4 = n4 - ar.lo4, work = ar_two ? (m4 + ar.pd.world - 1) / ar.pd.world : m4;
    ar.nvb = (int)std::min<long long>(32, std::max<long long>(1, (work + 255) / 256));
  }
  const Fold fdh{{Fold1{fold_off, fold_len, fold_nrep, fold_stride}, Fold1{fold2_off, fold2_len, fold2_nrep, fold2_stride}}};
  const Holes hh = make_holes(fdh);
  const long long n4c = n4 - hh.len[0] - hh.len[1];
  if (ar.nvb > 0 && (hh.len[0] || hh.len[1]) && hh.lo[0] < ar.lo4) return hipErrorInvalidValue;   // holes above ar range start
  for (int k = 0; k < 2; ++k)
    if (fold_on(fdh.f[k]) && (fdh.f[k].off % 4 || fdh.f[k].stride % 4 || fdh.f[k].nrep > kMaxFold ||
                              fdh.f[k].off + (long long)fdh.f[k].nrep * fdh.f[k].stride > n))
      return hipErrorInvalidValue;
  const int nfb = fold_blocks(fdh.f[0]) + fold_blocks(fdh.f[1]);
  unsigned long long* prof = pde_lenet_prof_slot(5);
  static const bool ntp = [] {
    const char* e = getenv("PDE_ADAM_NT_P");
    return e != nullptr && e[0] == '1';   // default off: neutral in a same-box A/B (profiles/r5_lenet/)
  }();
#define PDE_ADAM_LAUNCH(P, N)                                                                                   \
  hipLaunchKernelGGL((k_adam<P, N>), dim3(grid_for(n4c) + ar.nvb + nfb), dim3(256), 0, st, p, g, m, v, n4, lr, b1, \
                     b2, eps, wd, decoupled, grad_scale, step, arrive, bump, Pack{pack_off, pack_dst, pack_mode},    \
                     Fold{{Fold1{fold_off, fold_len, fold_nrep, fold_stride},                                      \
                           Fold1{fold2_off, fold2_len, fold2_nrep, fold2_stride}}},                                \
                     ar, P ? prof : nullptr)
  if (prof) {
    if (ntp) PDE_ADAM_LAUNCH(true, true); else PDE_ADAM_LAUNCH(true, false);
  } else {
    if (ntp) PDE_ADAM_LAUNCH(false, true); else PDE_ADAM_LAUNCH(false, false);
  }
#undef PDE_ADAM_LAUNCH
  return hipGetLastError();
}

hipError_t pde_sgd_flat(float* p, float* g, float* buf, long long n, float lr, float momentum, float dampening,
                        float wd, int nesterov, float grad_scale, long long* step, unsigned* arrive, int bump,
                        long long pack_off, float* pack_dst, long long fold_off, int fold_len, int fold_nrep,
                        int fold_stride, int pack_mode, long long fold2_off, int fold2_len, int fold2_nrep,
                        int fold2_stride, hipStream_t st) {
  if (n % 4) return hipErrorInvalidValue;
  const long long n4 = n / 4;
  const Fold fdh{{Fold1{fold_off, fold_len, fold_nrep, fold_stride}, Fold1{fold2_off, fold2_len, fold2_nrep, fold2_stride}}};
  const Holes hh = make_holes(fdh);
  for (int k = 0; k < 2; ++k)
    if (fold_on(fdh.f[k]) && (fdh.f[k].off % 4 || fdh.f[k].stride % 4 || fdh.f[k].nrep > kMaxFold ||
                              fdh.f[k].off + (long long)fdh.f[k].nrep * fdh.f[k].stride > n))
      return hipErrorInvalidValue;
  const int nfb = fold_blocks(fdh.f[0]) + fold_blocks(fdh.f[1]);
  hipLaunchKernelGGL(k_sgd, dim3(grid_for(n4 - hh.len[0] - hh.len[1]) + nfb), dim3(256), 0, st, p, g, buf, n4, lr, momentum, dampening, wd,
                     nesterov, grad_scale, step, arrive, bump, Pack{pack_off, pack_dst, pack_mode},
                     Fold{{Fold1{fold_off, fold_len, fold_nrep, fold_stride}, Fold1{fold2_off, fold2_len, fold2_nrep, fold2_stride}}});
  return hipGetLastError();
}

hipError_t pde_lenet_pack_w2(const float* w2, float* dst, hipStream_t st) {
  hipLaunchKernelGGL(k_lenet_pack_w2, dim3((500 * 64 + 255) / 256), dim3(256), 0, st, w2, dst);
  return hipGetLastError();
}

hipError_t pde_scale(float* x, long long n, float s, hipStream_t st) {
  hipLaunchKernelGGL(k_scale, dim3(grid_for((n + 3) / 4)), dim3(256), 0, st, x, n, s);
  return hipGetLastError();
}

}  // extern "C"
