// Causal flash attention (head_dim 64) forward + backward for gfx950, bf16 in / fp32 accumulate,
// on v_mfma_f32_32x32x16_bf16.  Used by the GPT-2 model (models/gpt2.py).
//
// Layout: q/k/v are row-major [B, T, *] with a row stride `ld` (elements) and head h at column
// h*64, so the fused c_attn output [B, T, 3, H, 64] is read in place and dq/dk/dv are written in
// place into a [B, T, 3, H, 64] gradient buffer; O / dO are [B, T, H, 64].
//
// MFMA 32x32x16 bf16 fragments (cdna_hip_programming.md §3): lane l (r = l&31, h = l>>5) holds
// A[r][8h+j] and B[8h+j][r] (j < 8); accumulator reg i is at row (i&3)+8(i>>2)+4h, col r.
//
// Forward / dQ kernels compute the TRANSPOSED score tile S^T = K Q^T (keys on registers, queries on
// lanes): every query's running max / sum lives in one lane (plus its mirror half), the rescale of
// the output accumulator O^T is a per-lane multiply, and P^T feeds the next MFMA (O^T += V^T P^T)
// straight from registers (regs 8s..8s+7 -> bf16 fragment of k-step s, whose K index j of lane
// half h is key 16s + 8(j>>2) + 4h + (j&3)).  The dK/dV kernel keeps S = Q K^T (queries on
// registers) so that dV += P^T dO and dK += dS^T Q take P / dS as the A operand.
//
// Every 64-row tile a block needs (K and V; or Q and dO) is staged ONCE per block in LDS as a
// row-major, XOR-swizzled image (cdna_hip_programming.md T10 layout (a), 8 KB): the row-operand
// fragments are ds_read_b128 row reads and the transposed operands (V^T, K^T, dO^T, Q^T) are
// ds_read_b64_tr_b16 hardware-transposed reads of the same image -- conflict-free for both (checked
// with the bank model of §2).  Tiles are staged by LDS-DMA (buffer_load ... lds, pde_lds.h) into a
// ring of NST stage buffers, NST-1 tiles in flight ahead of the MFMAs: per tile a counted vmcnt
// wait, one raw s_barrier, the next issue, then compute.  (The first version staged through
// registers; hipcc placed the staging registers in scratch and waited vmcnt(0) after every load,
// leaving the waves parked 65% of their cycles.)  Transposed reads are inline asm with immediate
// offsets (the builtin makes hipcc drain the DMA queue before each one).  exp2 is the bare
// v_exp_f32 (inputs <= 0; no denormal fix-up), and the O rescale is skipped when no query's
// running max grew (cdna_hip_programming.md T13 with threshold 0: exact).
#include <type_traits>

#include "pde_hip.h"
#include "pde_bf16.h"
#include "pde_kernels.h"
#include "pde_lds.h"

namespace {

using namespace pde_lds;

constexpr int HD = 64;        // head dim
constexpr int TILE = 8192;    // bytes of one 64 x 64 bf16 tile image
constexpr int kNstDefault = 4;   // LDS stage ring depth (template parameter NST of the kernels)

__device__ __forceinline__ bf16x8 ld16(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
// max of three with no NaN canonicalisation (fmaxf on MFMA results costs a v_max x,x per operand)
__device__ __forceinline__ float max3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// accumulator regs 8s..8s+7 -> bf16 fragment
template <int S>
__device__ __forceinline__ bf16x8 frag_of(const f32x16& a) {
  uint4 u = make_uint4(pack_bf2(a[8 * S + 0], a[8 * S + 1]), pack_bf2(a[8 * S + 2], a[8 * S + 3]),
                       pack_bf2(a[8 * S + 4], a[8 * S + 5]), pack_bf2(a[8 * S + 6], a[8 * S + 7]));
  return __builtin_bit_cast(bf16x8, u);
}

// LDS-DMA of the 64-row tile starting at row0 of a [T][ld] bf16 matrix (resource r) into img:
// wave w fills the 8-row groups w and w + 4 (two wave-instructions).
__device__ __forceinline__ void issue_tile(rsrc_t r, int ld, int row0, const char* img, int w, int lrow, int lch) {
#pragma unroll
  for (int gg = 0; gg < 2; ++gg) {
    const int g = w + 4 * gg;
    glds16(r, img + g * 1024, (uint32_t)(((row0 + 8 * g + lrow) * ld + lch * 8) * 2));
  }
}

// wait until at most `ahead` younger stages (of PER glds per wave) are in flight
template <int PER>
__device__ __forceinline__ void wait_stages(int ahead) {
  if (ahead >= 2) wait_vm<2 * PER>();
  else if (ahead == 1) wait_vm<PER>();
  else wait_vm<0>();
}

// V^T / K^T / dO^T / Q^T fragment of k-step S, dims half C (0/1) from a transposed-read base
template <int S, int C>
__device__ __forceinline__ bf16x8 tfrag(uint2 base) {
  return trpair<2048 * S + colblk_off(C)>(base);
}

// write a [dim x query] accumulator pair (dims 0..31 / 32..63) of one lane's query as 8-byte rows
__device__ __forceinline__ void store_dimrows(bf16_t* dst, const f32x16& a0, const f32x16& a1, float mul, int h) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    float v0[4] = {a0[4 * g] * mul, a0[4 * g + 1] * mul, a0[4 * g + 2] * mul, a0[4 * g + 3] * mul};
    float v1[4] = {a1[4 * g] * mul, a1[4 * g + 1] * mul, a1[4 * g + 2] * mul, a1[4 * g + 3] * mul};
    *reinterpret_cast<uint2*>(dst + 8 * g + 4 * h) = pack4(v0);
    *reinterpret_cast<uint2*>(dst + 32 + 8 * g + 4 * h) = pack4(v1);
  }
}

// ------------------------------------------------------------------------------------ block map
// (tile, batch*head) of this block.  The dispatcher deals blocks to the 8 XCDs round-robin, so with a
// plain 2-D grid the tiles of one (batch, head) land on every XCD and each XCD re-fetches that head's
// K/V (or Q/dO) tiles through its own L2 -- the kernels then run at the fabric rate of those
// re-fetches.  Instead: XCD-contiguous ids (pde_hip.h xcd_remap), cut into groups of kAttnGroup heads
// whose tiles stay L2-resident while the group runs, heaviest causal tiles first inside a group.
// G = 0 keeps the plain order (no remap, one head per group) for A/B runs.
constexpr int kAttnGroup = 8;
__device__ __forceinline__ void attn_block(int nt, int nbh, int G, bool heavy_high, int& t, int& bh) {
  const int id = G ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  G = G ? G : 1;
  const int grp = id / (G * nt), r = id - grp * G * nt;
  const int gsz = min(G, nbh - grp * G);
  const int k = r / gsz;
  bh = grp * G + (r - k * gsz);
  t = heavy_high ? nt - 1 - k : k;
}

// ------------------------------------------------------------------------------------ forward
// grid (T/128 * B*H), 256 threads: wave w owns queries qt*128 + 32w + (0..31)
template <int NST, int OCC>
__global__ __launch_bounds__(256, OCC) void k_attn_fwd(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K,
                                                     const bf16_t* __restrict__ V, int ldq, bf16_t* __restrict__ O,
                                                     int ldo, float* __restrict__ LSE, int T, int H, float sl2,
                                                     float scale, int G) {
  __shared__ __attribute__((aligned(16))) char lds[NST * 2 * TILE];  // stage: K | V
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), h = lane >> 5, r = lane & 31;
  int qt, bh;
  attn_block(T / 128, gridDim.x / (T / 128), G, true, qt, bh);   // longest (most keys) tiles first
  const int b = bh / H, hh = bh % H;
  const size_t boff = (size_t)b * T * ldq + hh * HD;
  const uint32_t tbytes = (uint32_t)T * ldq * 2;
  const rsrc_t kr = make_rsrc(K + boff, tbytes), vr = make_rsrc(V + boff, tbytes);
  const int lrow = glds_row(lane), lch = glds_chunk(lane, w & 1);
  const int q0 = qt * 128 + w * 32, myq = q0 + r;
  const int nkt = (qt * 128 + 127) / 64 + 1;
  const int last_kt = (q0 + 31) / 64;
  auto issue = [&](int kt) {
    const char* st = lds + (kt % NST) * 2 * TILE;
    issue_tile(kr, ldq, kt * 64, st, w, lrow, lch);
    issue_tile(vr, ldq, kt * 64, st + TILE, w, lrow, lch);
  };
  bf16x8 qf[4];                        // issued before the DMA prologue: waiting for them later
#pragma unroll                          // does not drain the prefetched stages (in-order vmcnt)
  for (int s = 0; s < 4; ++s) qf[s] = ld16(Q + boff + (size_t)myq * ldq + 16 * s + 8 * h);
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nkt) issue(s);
  const uint2 tl = tr_lane_off();
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_char*)lds;
  f32x16 o0 = {}, o1 = {};
  float m = -INFINITY, l = 0.f;
  for (int kt = 0; kt < nkt; ++kt) {
    wait_stages<4>(min(NST - 2, nkt - 1 - kt));
    __builtin_amdgcn_s_barrier();
    if (kt + NST - 1 < nkt) issue(kt + NST - 1);
    if (kt <= last_kt) {
      const int sb = kt % NST;
      const char* Ks = lds + sb * 2 * TILE;
      const uint2 vb = add2(tl, lds0 + sb * 2 * TILE + TILE);
      const int k0 = kt * 64;
      f32x16 s0 = {}, s1 = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        s0 = mfma_bf16(row_frag(Ks, r, 2 * s + h), qf[s], s0);
        s1 = mfma_bf16(row_frag(Ks, 32 + r, 2 * s + h), qf[s], s1);
      }
      // V^T fragments in flight while the softmax runs
      const bf16x8 v00 = tfrag<0, 0>(vb), v01 = tfrag<0, 1>(vb), v10 = tfrag<1, 0>(vb), v11 = tfrag<1, 1>(vb);
      const bf16x8 v20 = tfrag<2, 0>(vb), v21 = tfrag<2, 1>(vb), v30 = tfrag<3, 0>(vb), v31 = tfrag<3, 1>(vb);
      if (k0 + 63 > q0) {  // tile crosses the diagonal of this wave
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = k0 + (i & 3) + 8 * (i >> 2) + 4 * h;
          s0[i] = key > myq ? -INFINITY : s0[i];
          s1[i] = key + 32 > myq ? -INFINITY : s1[i];
        }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) mx = max3(mx, s0[i], s1[i]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m, mx);
      if (__any(mn > m)) {                 // some query's running max grew: rescale O and l
        const float alpha = fexp2((m - mn) * sl2);
        l *= alpha;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          o0[i] *= alpha;
          o1[i] *= alpha;
        }
        m = mn;
      }
      const float mb = m * sl2;
      float ls = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s0[i] = fexp2(s0[i] * sl2 - mb);
        s1[i] = fexp2(s1[i] * sl2 - mb);
        ls += s0[i] + s1[i];
      }
      l += ls;
      const bf16x8 p0 = frag_of<0>(s0), p1 = frag_of<1>(s0), p2 = frag_of<0>(s1), p3 = frag_of<1>(s1);
      lgkm_fence();
      o0 = mfma_bf16(v00, p0, o0);
      o1 = mfma_bf16(v01, p0, o1);
      o0 = mfma_bf16(v10, p1, o0);
      o1 = mfma_bf16(v11, p1, o1);
      o0 = mfma_bf16(v20, p2, o0);
      o1 = mfma_bf16(v21, p2, o1);
      o0 = mfma_bf16(v30, p3, o0);
      o1 = mfma_bf16(v31, p3, o1);
    }
  }
  const float lt = l + __shfl_xor(l, 32, 64);
  store_dimrows(O + (size_t)b * T * ldo + (size_t)myq * ldo + hh * HD, o0, o1, 1.f / lt, h);
  // log-sum-exp in base-2 units of the scaled scores (what the backward's exp2 consumes directly)
  if (h == 0) LSE[(size_t)bh * T + myq] = m * sl2 + __log2f(lt);
}

// ------------------------------------------------------------------------------------ backward
// dQ: grid (T/128 * B*H); transposed-score structure of the forward; K, V tiles staged in LDS
// (K rows for S^T, V rows for dP^T, K^T via transposed reads for dQ^T += K^T dS^T).
// Dd[bh, t] = sum_d dO * O of its query rows is computed here, from the dO fragments it loads anyway
// plus the O rows (each lane pair holds a row's 64 dims), and written for k_attn_bwd_dkdv, which runs
// after it: no separate pre-pass over dO and O (14.6 us per layer at the GPT-2 shape).
template <int NST, int OCC>
__global__ __launch_bounds__(256, OCC) void k_attn_bwd_dq(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K,
                                                        const bf16_t* __restrict__ V, int ldq,
                                                        const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO,
                                                        int ldo, const float* __restrict__ LSE,
                                                        float* __restrict__ Dd, bf16_t* __restrict__ dQ, int T, int H,
                                                        float sl2, float scale, int G) {
  __shared__ __attribute__((aligned(16))) char lds[NST * 2 * TILE];  // stage: K | V
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), h = lane >> 5, r = lane & 31;
  int qt, bh;
  attn_block(T / 128, gridDim.x / (T / 128), G, true, qt, bh);   // longest (most keys) tiles first
  const int b = bh / H, hh = bh % H;
  const size_t boff = (size_t)b * T * ldq + hh * HD;
  const uint32_t tbytes = (uint32_t)T * ldq * 2;
  const rsrc_t kr = make_rsrc(K + boff, tbytes), vr = make_rsrc(V + boff, tbytes);
  const int lrow = glds_row(lane), lch = glds_chunk(lane, w & 1);
  const bf16_t* dOb = dO + (size_t)b * T * ldo + hh * HD;
  const int q0 = qt * 128 + w * 32, myq = q0 + r;
  const int nkt = (qt * 128 + 127) / 64 + 1;
  const int last_kt = (q0 + 31) / 64;
  auto issue = [&](int kt) {
    const char* st = lds + (kt % NST) * 2 * TILE;
    issue_tile(kr, ldq, kt * 64, st, w, lrow, lch);
    issue_tile(vr, ldq, kt * 64, st + TILE, w, lrow, lch);
  };
  bf16x8 qf[4], gf[4], of[4];
  const bf16_t* Ob = O + (size_t)b * T * ldo + hh * HD;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = ld16(Q + boff + (size_t)myq * ldq + 16 * s + 8 * h);
    gf[s] = ld16(dOb + (size_t)myq * ldo + 16 * s + 8 * h);
    of[s] = ld16(Ob + (size_t)myq * ldo + 16 * s + 8 * h);
  }
  const float lse2 = LSE[(size_t)bh * T + myq];        // base-2 units (k_attn_fwd)
  float dq_d = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int e = 0; e < 8; ++e) dq_d += bf2f((uint16_t)gf[s][e]) * bf2f((uint16_t)of[s][e]);
  dq_d += __shfl_xor(dq_d, 32, 64);                    // the row's other 32 dims (lane half h ^ 1)
  if (h == 0) Dd[(size_t)bh * T + myq] = dq_d;
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nkt) issue(s);
  const uint2 tl = tr_lane_off();
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_char*)lds;
  f32x16 a0 = {}, a1 = {};
  for (int kt = 0; kt < nkt; ++kt) {
    wait_stages<4>(min(NST - 2, nkt - 1 - kt));
    __builtin_amdgcn_s_barrier();
    if (kt + NST - 1 < nkt) issue(kt + NST - 1);
    if (kt <= last_kt) {
      const int sb = kt % NST;
      const char* Ks = lds + sb * 2 * TILE;
      const char* Vs = Ks + TILE;
      const uint2 kb = add2(tl, lds0 + sb * 2 * TILE);
      const int k0 = kt * 64;
      f32x16 s0 = {}, s1 = {}, d0 = {}, d1 = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        s0 = mfma_bf16(row_frag(Ks, r, 2 * s + h), qf[s], s0);
        s1 = mfma_bf16(row_frag(Ks, 32 + r, 2 * s + h), qf[s], s1);
        d0 = mfma_bf16(row_frag(Vs, r, 2 * s + h), gf[s], d0);
        d1 = mfma_bf16(row_frag(Vs, 32 + r, 2 * s + h), gf[s], d1);
      }
      const bf16x8 k00 = tfrag<0, 0>(kb), k01 = tfrag<0, 1>(kb), k10 = tfrag<1, 0>(kb), k11 = tfrag<1, 1>(kb);
      const bf16x8 k20 = tfrag<2, 0>(kb), k21 = tfrag<2, 1>(kb), k30 = tfrag<3, 0>(kb), k31 = tfrag<3, 1>(kb);
      const bool diag = k0 + 63 > q0;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = k0 + (i & 3) + 8 * (i >> 2) + 4 * h;
        float p0 = fexp2(fmaf(s0[i], sl2, -lse2));
        float p1 = fexp2(fmaf(s1[i], sl2, -lse2));
        if (diag) {
          p0 = key > myq ? 0.f : p0;
          p1 = key + 32 > myq ? 0.f : p1;
        }
        s0[i] = p0 * (d0[i] - dq_d);
        s1[i] = p1 * (d1[i] - dq_d);
      }
      const bf16x8 p0 = frag_of<0>(s0), p1 = frag_of<1>(s0), p2 = frag_of<0>(s1), p3 = frag_of<1>(s1);
      lgkm_fence();
      a0 = mfma_bf16(k00, p0, a0);
      a1 = mfma_bf16(k01, p0, a1);
      a0 = mfma_bf16(k10, p1, a0);
      a1 = mfma_bf16(k11, p1, a1);
      a0 = mfma_bf16(k20, p2, a0);
      a1 = mfma_bf16(k21, p2, a1);
      a0 = mfma_bf16(k30, p3, a0);
      a1 = mfma_bf16(k31, p3, a1);
    }
  }
  store_dimrows(dQ + boff + (size_t)myq * ldq, a0, a1, scale, h);
}

// dK, dV: grid (T/128 * B*H); wave w owns keys kb*128 + 32w + (0..31); loops over 64-query tiles
// with Q / dO / LSE / D staged in LDS (rows for S / dP, transposed reads for dK / dV).
constexpr int kDkdvStage = 2 * TILE + 512;           // Q | dO | LSE[64] | D[64]
template <int NST, int OCC>
__global__ __launch_bounds__(256, OCC) void k_attn_bwd_dkdv(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K,
                                                          const bf16_t* __restrict__ V, int ldq,
                                                          const bf16_t* __restrict__ dO, int ldo,
                                                          const float* __restrict__ LSE,
                                                          const float* __restrict__ Dd, bf16_t* __restrict__ dK,
                                                          bf16_t* __restrict__ dV, int T, int H, float sl2,
                                                          float scale, int G) {
  __shared__ __attribute__((aligned(16))) char lds[NST * kDkdvStage];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), h = lane >> 5, r = lane & 31;
  int kb, bh;
  attn_block(T / 128, gridDim.x / (T / 128), G, false, kb, bh);  // key tile 0 sees the most queries
  const int b = bh / H, hh = bh % H;
  const size_t boff = (size_t)b * T * ldq + hh * HD;
  const rsrc_t qr = make_rsrc(Q + boff, (uint32_t)T * ldq * 2);
  const rsrc_t gr = make_rsrc(dO + (size_t)b * T * ldo + hh * HD, (uint32_t)T * ldo * 2);
  // wave w & 1 == 0 stages LSE, == 1 stages D (two waves write each: identical bytes)
  const rsrc_t vecr = make_rsrc((w & 1) ? Dd + (size_t)bh * T : LSE + (size_t)bh * T, (uint32_t)T * 4);
  const int lrow = glds_row(lane), lch = glds_chunk(lane, w & 1);
  const int k0 = kb * 128 + w * 32, myk = k0 + r;
  const int qt0 = (kb * 128) / 64, nqt = T / 64;
  auto issue = [&](int qt) {
    const char* st = lds + ((qt - qt0) % NST) * kDkdvStage;
    issue_tile(qr, ldq, qt * 64, st, w, lrow, lch);
    issue_tile(gr, ldo, qt * 64, st + TILE, w, lrow, lch);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(vecr, (__attribute__((address_space(3))) void*)(st + 2 * TILE +
                                                                                              256 * (w & 1)),
                                             4, (uint32_t)(qt * 64 + lane) * 4, 0, 0, 0);
  };
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = ld16(K + boff + (size_t)myk * ldq + 16 * s + 8 * h);
    vf[s] = ld16(V + boff + (size_t)myk * ldq + 16 * s + 8 * h);
  }
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (qt0 + s < nqt) issue(qt0 + s);
  const uint2 tl = tr_lane_off();
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_char*)lds;
  f32x16 dv0 = {}, dv1 = {}, dk0 = {}, dk1 = {};
  for (int qt = qt0; qt < nqt; ++qt) {
    wait_stages<5>(min(NST - 2, nqt - 1 - qt));
    __builtin_amdgcn_s_barrier();
    if (qt + NST - 1 < nqt) issue(qt + NST - 1);
    const int qbase = qt * 64;
    if (k0 <= qbase + 63) {  // some query of this tile sees some key of this wave
      const int sb = (qt - qt0) % NST;
      const char* Qs = lds + sb * kDkdvStage;
      const char* Gs = Qs + TILE;
      const float* Ls = reinterpret_cast<const float*>(Qs + 2 * TILE);
      const float* Ds = Ls + 64;
      const uint2 qbv = add2(tl, lds0 + sb * kDkdvStage), gbv = add2(tl, lds0 + sb * kDkdvStage + TILE);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        f32x16 S = {}, dP = {};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          S = mfma_bf16(row_frag(Qs, 32 * u + r, 2 * s + h), kf[s], S);
          dP = mfma_bf16(row_frag(Gs, 32 * u + r, 2 * s + h), vf[s], dP);
        }
        bf16x8 g00, g01, g10, g11, q00, q01, q10, q11;
        if (u == 0) {
          g00 = tfrag<0, 0>(gbv); g01 = tfrag<0, 1>(gbv); g10 = tfrag<1, 0>(gbv); g11 = tfrag<1, 1>(gbv);
          q00 = tfrag<0, 0>(qbv); q01 = tfrag<0, 1>(qbv); q10 = tfrag<1, 0>(qbv); q11 = tfrag<1, 1>(qbv);
        } else {
          g00 = tfrag<2, 0>(gbv); g01 = tfrag<2, 1>(gbv); g10 = tfrag<3, 0>(gbv); g11 = tfrag<3, 1>(gbv);
          q00 = tfrag<2, 0>(qbv); q01 = tfrag<2, 1>(qbv); q10 = tfrag<3, 0>(qbv); q11 = tfrag<3, 1>(qbv);
        }
        // the causal mask only matters where this wave's keys reach past the half's first query
        // (wave-uniform): the other tiles skip the per-element compare / select
        const bool need_mask = k0 + 31 > qbase + 32 * u;
        auto softmax_grad = [&](auto MASK_) {
          constexpr bool MASK = decltype(MASK_)::value;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const float4 l4 = *reinterpret_cast<const float4*>(&Ls[32 * u + 8 * g + 4 * h]);
            const float4 d4 = *reinterpret_cast<const float4*>(&Ds[32 * u + 8 * g + 4 * h]);
            const float lv[4] = {l4.x, l4.y, l4.z, l4.w};   // base-2 log-sum-exp (k_attn_fwd)
            const float dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int i = 4 * g + e;
              float p = fexp2(fmaf(S[i], sl2, -lv[e]));
              if constexpr (MASK) {
                const int q = qbase + 32 * u + 8 * g + 4 * h + e;
                p = myk > q ? 0.f : p;
              }
              S[i] = p;
              dP[i] = p * (dP[i] - dv[e]);
            }
          }
        };
        if (need_mask) softmax_grad(std::true_type{});
        else softmax_grad(std::false_type{});
        const bf16x8 p0 = frag_of<0>(S), p1 = frag_of<1>(S);
        const bf16x8 d0 = frag_of<0>(dP), d1 = frag_of<1>(dP);
        lgkm_fence();
        dv0 = mfma_bf16(p0, g00, dv0);
        dv1 = mfma_bf16(p0, g01, dv1);
        dv0 = mfma_bf16(p1, g10, dv0);
        dv1 = mfma_bf16(p1, g11, dv1);
        dk0 = mfma_bf16(d0, q00, dk0);
        dk1 = mfma_bf16(d0, q01, dk1);
        dk0 = mfma_bf16(d1, q10, dk0);
        dk1 = mfma_bf16(d1, q11, dk1);
      }
    }
  }
  // acc rows = keys (regs), cols = dims (lanes): 2-byte stores, coalesced across the 32 lanes of a half
  bf16_t* dKb = dK + boff;
  bf16_t* dVb = dV + boff;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int key = k0 + (i & 3) + 8 * (i >> 2) + 4 * h;
    dKb[(size_t)key * ldq + r] = f2bf(dk0[i] * scale);
    dKb[(size_t)key * ldq + 32 + r] = f2bf(dk1[i] * scale);
    dVb[(size_t)key * ldq + r] = f2bf(dv0[i]);
    dVb[(size_t)key * ldq + 32 + r] = f2bf(dv1[i]);
  }
}

int g_attn_variant = 5;   // pde_attn_set_variant: LDS ring depth / occupancy (default: measured best)
int g_attn_group = kAttnGroup;   // heads per L2 group of the block map (0: plain order)

template <int NST, int OCC>
void launch_fwd(const void* q, const void* k, const void* v, int ldq, void* o, int ldo, float* lse, int B, int T,
                int H, float scale, hipStream_t st) {
  hipLaunchKernelGGL((k_attn_fwd<NST, OCC>), dim3(T / 128 * B * H), dim3(256), 0, st, (const bf16_t*)q,
                     (const bf16_t*)k, (const bf16_t*)v, ldq, (bf16_t*)o, ldo, lse, T, H, scale * 1.4426950408889634f,
                     scale, g_attn_group);
}

template <int NST, int OCC>
void launch_dq(const void* q, const void* k, const void* v, int ldq, const void* o, const void* dout, int ldo,
               const float* lse, float* Dd, void* dq, int B, int T, int H, float sl2, float scale, hipStream_t st) {
  hipLaunchKernelGGL((k_attn_bwd_dq<NST, OCC>), dim3(T / 128 * B * H), dim3(256), 0, st, (const bf16_t*)q,
                     (const bf16_t*)k, (const bf16_t*)v, ldq, (const bf16_t*)o, (const bf16_t*)dout, ldo, lse, Dd,
                     (bf16_t*)dq, T, H, sl2, scale, g_attn_group);
}

template <int NST, int OCC>
void launch_dkdv(const void* q, const void* k, const void* v, int ldq, const void* dout, int ldo, const float* lse,
                 const float* Dd, void* dk, void* dv, int B, int T, int H, float sl2, float scale, hipStream_t st) {
  hipLaunchKernelGGL((k_attn_bwd_dkdv<NST, OCC>), dim3(T / 128 * B * H), dim3(256), 0, st, (const bf16_t*)q,
                     (const bf16_t*)k, (const bf16_t*)v, ldq, (const bf16_t*)dout, ldo, lse, Dd, (bf16_t*)dk,
                     (bf16_t*)dv, T, H, sl2, scale, g_attn_group);
}

}  // namespace

extern "C" {

// variant bits: 1 = forward with a 3-deep ring at 3 blocks per CU, 2 = dQ likewise (spills: slower),
//               4 = dK/dV with a 3-deep ring (2 blocks per CU).  Default 5, measured on MI355X at the
//               GPT-2 shape (tools/attn_bench.py, profiles/r2_attn/): fwd 85.3 -> 71.3 us, bwd 263.8 -> 241.0 us
//               bits 8..15: heads per L2 group of the block map (attn_block), 0 = default, 255 = plain order
void pde_attn_set_variant(int v) {
  g_attn_variant = v & 0xff;
  const int g = (v >> 8) & 0xff;
  g_attn_group = g == 0 ? kAttnGroup : g == 255 ? 0 : g;
}

hipError_t pde_attn_fwd(const void* q, const void* k, const void* v, int ldq, void* o, int ldo, float* lse, int B,
                        int T, int H, float scale, hipStream_t st) {
  if (T % 128 != 0) return hipErrorInvalidValue;
  if (g_attn_variant & 1) launch_fwd<3, 3>(q, k, v, ldq, o, ldo, lse, B, T, H, scale, st);
  else launch_fwd<kNstDefault, 2>(q, k, v, ldq, o, ldo, lse, B, T, H, scale, st);
  return hipGetLastError();
}

hipError_t pde_attn_bwd(const void* q, const void* k, const void* v, int ldq, const void* o, const void* dout,
                        int ldo, const float* lse, float* Dd, void* dq, void* dk, void* dv, int B, int T, int H,
                        float scale, hipStream_t st) {
  if (T % 128 != 0) return hipErrorInvalidValue;
  const float sl2 = scale * 1.4426950408889634f;
  // dQ first: it computes and writes Dd (= rowsum dO * O), which the dK / dV kernel reads
  if (g_attn_variant & 2) launch_dq<3, 3>(q, k, v, ldq, o, dout, ldo, lse, Dd, dq, B, T, H, sl2, scale, st);
  else launch_dq<kNstDefault, 2>(q, k, v, ldq, o, dout, ldo, lse, Dd, dq, B, T, H, sl2, scale, st);
  if (g_attn_variant & 4) launch_dkdv<3, 2>(q, k, v, ldq, dout, ldo, lse, Dd, dk, dv, B, T, H, sl2, scale, st);
  else launch_dkdv<kNstDefault, 2>(q, k, v, ldq, dout, ldo, lse, Dd, dk, dv, B, T, H, sl2, scale, st);
  return hipGetLastError();
}

}  // extern "C"
