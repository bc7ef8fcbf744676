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
// with the bank model of §2).  Tiles are double-buffered: global loads of tile t+1 are issued before
// the MFMA work on tile t and written to the other buffer after it; one barrier per tile.
#include "pde_hip.h"
#include "pde_bf16.h"
#include "pde_kernels.h"

namespace {

constexpr int HD = 64;        // head dim
constexpr int TILE = 8192;    // bytes of one 64 x 64 bf16 tile image

typedef short s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v lds_s4v;

__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 ld16(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

// byte offset of 16-byte chunk `ch` (0..7) of row `row` (0..63) in a tile image
__device__ __forceinline__ int toff(int row, int ch) {
  return 1024 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}

// accumulator regs 8s..8s+7 -> bf16 fragment
template <int S>
__device__ __forceinline__ bf16x8 frag_of(const f32x16& a) {
  uint4 u = make_uint4(pack_bf2(a[8 * S + 0], a[8 * S + 1]), pack_bf2(a[8 * S + 2], a[8 * S + 3]),
                       pack_bf2(a[8 * S + 4], a[8 * S + 5]), pack_bf2(a[8 * S + 6], a[8 * S + 7]));
  return __builtin_bit_cast(bf16x8, u);
}

// row operand: row `row` of the tile, dims 8*ch .. 8*ch+7
__device__ __forceinline__ bf16x8 row_frag(const char* tile, int row, int ch) {
  return *reinterpret_cast<const bf16x8*>(tile + toff(row, ch));
}

// transposed operand: lane (r, h) gets column col0 + r of rows row0 + {4h..4h+3, 8+4h..8+4h+3}
// (= the permuted K order of a 32x32x16 k-step), via two ds_read_b64_tr_b16.  EXEC must be full.
__device__ __forceinline__ bf16x8 tr_frag(const char* tile, int row0, int col0) {
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, h = g >> 1;
  const int ch = (col0 >> 3) + 2 * (g & 1) + (p >> 1);
  const int r = row0 + 4 * h + q;
  const char* a0 = tile + toff(r, ch) + 8 * (p & 1);
  const char* a1 = tile + toff(r + 8, ch) + 8 * (p & 1);
  const s4v v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)a0);
  const s4v v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)a1);
  bf16x8 out;
  out[0] = v0[0]; out[1] = v0[1]; out[2] = v0[2]; out[3] = v0[3];
  out[4] = v1[0]; out[5] = v1[1]; out[6] = v1[2]; out[7] = v1[3];
  return out;
}

// 64 rows x 64 dims starting at `row0` of a [*, ld] matrix: 512 16-byte chunks, two per thread
__device__ __forceinline__ void tile_load(const bf16_t* src, size_t ld, int row0, uint4* reg) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = threadIdx.x + 256 * u;
    reg[u] = *reinterpret_cast<const uint4*>(src + (size_t)(row0 + (c >> 3)) * ld + (c & 7) * 8);
  }
}
__device__ __forceinline__ void tile_store(char* tile, const uint4* reg) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = threadIdx.x + 256 * u;
    *reinterpret_cast<uint4*>(tile + toff(c >> 3, c & 7)) = reg[u];
  }
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

// ------------------------------------------------------------------------------------ forward
// grid (T/128, B*H), 256 threads: wave w owns queries qt*128 + 32w + (0..31)
__global__ __launch_bounds__(256, 2) void k_attn_fwd(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K,
                                                     const bf16_t* __restrict__ V, int ldq, bf16_t* __restrict__ O,
                                                     int ldo, float* __restrict__ LSE, int T, int H, float sl2,
                                                     float scale) {
  __shared__ __attribute__((aligned(16))) char lds[4 * TILE];  // K[2] | V[2]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, r = lane & 31;
  const int qt = gridDim.x - 1 - blockIdx.x;  // longest (most keys) tiles first
  const int bh = blockIdx.y, b = bh / H, hh = bh % H;
  const size_t boff = (size_t)b * T * ldq + hh * HD;
  const bf16_t* Kb = K + boff;
  const bf16_t* Vb = V + boff;
  const int q0 = qt * 128 + w * 32, myq = q0 + r;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = ld16(Q + boff + (size_t)myq * ldq + 16 * s + 8 * h);
  f32x16 o0 = {}, o1 = {};
  float m = -INFINITY, l = 0.f;
  const int nkt = (qt * 128 + 127) / 64 + 1;
  const int last_kt = (q0 + 31) / 64;
  uint4 kr[2], vr[2];
  tile_load(Kb, ldq, 0, kr);
  tile_load(Vb, ldq, 0, vr);
  tile_store(lds, kr);
  tile_store(lds + 2 * TILE, vr);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const bool more = kt + 1 < nkt;
    if (more) {
      tile_load(Kb, ldq, (kt + 1) * 64, kr);
      tile_load(Vb, ldq, (kt + 1) * 64, vr);
    }
    if (kt <= last_kt) {
      const char* Ks = lds + (kt & 1) * TILE;
      const char* Vs = lds + 2 * TILE + (kt & 1) * TILE;
      const int k0 = kt * 64;
      f32x16 s0 = {}, s1 = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        s0 = mfma_bf16(row_frag(Ks, r, 2 * s + h), qf[s], s0);
        s1 = mfma_bf16(row_frag(Ks, 32 + r, 2 * s + h), qf[s], s1);
      }
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
      for (int i = 0; i < 16; ++i) mx = fmaxf(mx, fmaxf(s0[i], s1[i]));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m, mx);
      const float alpha = exp2f((m - mn) * sl2);
      const float mb = mn * sl2;
      float ls = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s0[i] = exp2f(s0[i] * sl2 - mb);
        s1[i] = exp2f(s1[i] * sl2 - mb);
        ls += s0[i] + s1[i];
      }
      l = l * alpha + ls;
      m = mn;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        o0[i] *= alpha;
        o1[i] *= alpha;
      }
      const bf16x8 p0 = frag_of<0>(s0), p1 = frag_of<1>(s0), p2 = frag_of<0>(s1), p3 = frag_of<1>(s1);
      o0 = mfma_bf16(tr_frag(Vs, 0, 0), p0, o0);
      o1 = mfma_bf16(tr_frag(Vs, 0, 32), p0, o1);
      o0 = mfma_bf16(tr_frag(Vs, 16, 0), p1, o0);
      o1 = mfma_bf16(tr_frag(Vs, 16, 32), p1, o1);
      o0 = mfma_bf16(tr_frag(Vs, 32, 0), p2, o0);
      o1 = mfma_bf16(tr_frag(Vs, 32, 32), p2, o1);
      o0 = mfma_bf16(tr_frag(Vs, 48, 0), p3, o0);
      o1 = mfma_bf16(tr_frag(Vs, 48, 32), p3, o1);
    }
    if (more) {
      tile_store(lds + ((kt + 1) & 1) * TILE, kr);
      tile_store(lds + 2 * TILE + ((kt + 1) & 1) * TILE, vr);
    }
    __syncthreads();
  }
  const float lt = l + __shfl_xor(l, 32, 64);
  store_dimrows(O + (size_t)b * T * ldo + (size_t)myq * ldo + hh * HD, o0, o1, 1.f / lt, h);
  if (h == 0) LSE[(size_t)bh * T + myq] = m * scale + __logf(lt);
}

// ------------------------------------------------------------------------------------ backward
// Dd[bh, t] = sum_d dO[b, t, h, d] * O[b, t, h, d]   (thread per (row, head))
__global__ __launch_bounds__(256) void k_attn_bwd_pre(const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO,
                                                      int ldo, float* __restrict__ Dd, int N, int T, int H) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N * H) return;
  const int row = i / H, hh = i % H;
  const uint4* o = reinterpret_cast<const uint4*>(O + (size_t)row * ldo + hh * HD);
  const uint4* g = reinterpret_cast<const uint4*>(dO + (size_t)row * ldo + hh * HD);
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    float a[8], bq[8];
    unpack8(o[c], a);
    unpack8(g[c], bq);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += a[e] * bq[e];
  }
  const int b = row / T, t = row % T;
  Dd[((size_t)b * H + hh) * T + t] = acc;
}

// dQ: grid (T/128, B*H); transposed-score structure of the forward; K, V tiles staged in LDS
// (K rows for S^T, V rows for dP^T, K^T via transposed reads for dQ^T += K^T dS^T).
__global__ __launch_bounds__(256, 2) void k_attn_bwd_dq(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K,
                                                        const bf16_t* __restrict__ V, int ldq,
                                                        const bf16_t* __restrict__ dO, int ldo,
                                                        const float* __restrict__ LSE, const float* __restrict__ Dd,
                                                        bf16_t* __restrict__ dQ, int T, int H, float sl2,
                                                        float scale) {
  __shared__ __attribute__((aligned(16))) char lds[4 * TILE];  // K[2] | V[2]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, r = lane & 31;
  const int qt = gridDim.x - 1 - blockIdx.x;
  const int bh = blockIdx.y, b = bh / H, hh = bh % H;
  const size_t boff = (size_t)b * T * ldq + hh * HD;
  const bf16_t* Kb = K + boff;
  const bf16_t* Vb = V + boff;
  const bf16_t* dOb = dO + (size_t)b * T * ldo + hh * HD;
  const int q0 = qt * 128 + w * 32, myq = q0 + r;
  bf16x8 qf[4], gf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = ld16(Q + boff + (size_t)myq * ldq + 16 * s + 8 * h);
    gf[s] = ld16(dOb + (size_t)myq * ldo + 16 * s + 8 * h);
  }
  const float lse2 = LSE[(size_t)bh * T + myq] * 1.4426950408889634f;
  const float dq_d = Dd[(size_t)bh * T + myq];
  f32x16 a0 = {}, a1 = {};
  const int nkt = (qt * 128 + 127) / 64 + 1;
  const int last_kt = (q0 + 31) / 64;
  uint4 kr[2], vr[2];
  tile_load(Kb, ldq, 0, kr);
  tile_load(Vb, ldq, 0, vr);
  tile_store(lds, kr);
  tile_store(lds + 2 * TILE, vr);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const bool more = kt + 1 < nkt;
    if (more) {
      tile_load(Kb, ldq, (kt + 1) * 64, kr);
      tile_load(Vb, ldq, (kt + 1) * 64, vr);
    }
    if (kt <= last_kt) {
      const char* Ks = lds + (kt & 1) * TILE;
      const char* Vs = lds + 2 * TILE + (kt & 1) * TILE;
      const int k0 = kt * 64;
      f32x16 s0 = {}, s1 = {}, d0 = {}, d1 = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        s0 = mfma_bf16(row_frag(Ks, r, 2 * s + h), qf[s], s0);
        s1 = mfma_bf16(row_frag(Ks, 32 + r, 2 * s + h), qf[s], s1);
        d0 = mfma_bf16(row_frag(Vs, r, 2 * s + h), gf[s], d0);
        d1 = mfma_bf16(row_frag(Vs, 32 + r, 2 * s + h), gf[s], d1);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = k0 + (i & 3) + 8 * (i >> 2) + 4 * h;
        const float p0 = key > myq ? 0.f : exp2f(s0[i] * sl2 - lse2);
        const float p1 = key + 32 > myq ? 0.f : exp2f(s1[i] * sl2 - lse2);
        s0[i] = p0 * (d0[i] - dq_d);
        s1[i] = p1 * (d1[i] - dq_d);
      }
      const bf16x8 p0 = frag_of<0>(s0), p1 = frag_of<1>(s0), p2 = frag_of<0>(s1), p3 = frag_of<1>(s1);
      a0 = mfma_bf16(tr_frag(Ks, 0, 0), p0, a0);
      a1 = mfma_bf16(tr_frag(Ks, 0, 32), p0, a1);
      a0 = mfma_bf16(tr_frag(Ks, 16, 0), p1, a0);
      a1 = mfma_bf16(tr_frag(Ks, 16, 32), p1, a1);
      a0 = mfma_bf16(tr_frag(Ks, 32, 0), p2, a0);
      a1 = mfma_bf16(tr_frag(Ks, 32, 32), p2, a1);
      a0 = mfma_bf16(tr_frag(Ks, 48, 0), p3, a0);
      a1 = mfma_bf16(tr_frag(Ks, 48, 32), p3, a1);
    }
    if (more) {
      tile_store(lds + ((kt + 1) & 1) * TILE, kr);
      tile_store(lds + 2 * TILE + ((kt + 1) & 1) * TILE, vr);
    }
    __syncthreads();
  }
  store_dimrows(dQ + boff + (size_t)myq * ldq, a0, a1, scale, h);
}

// dK, dV: grid (T/128, B*H); wave w owns keys kb*128 + 32w + (0..31); loops over 64-query tiles
// with Q / dO (+ lse, D) staged in LDS (rows for S / dP, transposed reads for dK / dV).
__global__ __launch_bounds__(256, 2) void k_attn_bwd_dkdv(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K,
                                                          const bf16_t* __restrict__ V, int ldq,
                                                          const bf16_t* __restrict__ dO, int ldo,
                                                          const float* __restrict__ LSE,
                                                          const float* __restrict__ Dd, bf16_t* __restrict__ dK,
                                                          bf16_t* __restrict__ dV, int T, int H, float sl2,
                                                          float scale) {
  __shared__ __attribute__((aligned(16))) char lds[4 * TILE];  // Q[2] | dO[2]
  __shared__ __attribute__((aligned(16))) float Ls[2][64], Ds[2][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, r = lane & 31;
  const int kb = blockIdx.x;  // tile 0 has the most queries: natural order is heavy-first
  const int bh = blockIdx.y, b = bh / H, hh = bh % H;
  const size_t boff = (size_t)b * T * ldq + hh * HD;
  const bf16_t* Qb = Q + boff;
  const bf16_t* dOb = dO + (size_t)b * T * ldo + hh * HD;
  const float* Lb = LSE + (size_t)bh * T;
  const float* Db = Dd + (size_t)bh * T;
  const int k0 = kb * 128 + w * 32, myk = k0 + r;
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = ld16(K + boff + (size_t)myk * ldq + 16 * s + 8 * h);
    vf[s] = ld16(V + boff + (size_t)myk * ldq + 16 * s + 8 * h);
  }
  f32x16 dv0 = {}, dv1 = {}, dk0 = {}, dk1 = {};
  const int qt0 = (kb * 128) / 64, nqt = T / 64;
  const int tid = threadIdx.x;
  uint4 qr[2], gr[2];
  float lsv = 0.f;
  tile_load(Qb, ldq, qt0 * 64, qr);
  tile_load(dOb, ldo, qt0 * 64, gr);
  lsv = tid < 64 ? Lb[qt0 * 64 + tid] : (tid < 128 ? Db[qt0 * 64 + tid - 64] : 0.f);
  tile_store(lds, qr);
  tile_store(lds + 2 * TILE, gr);
  if (tid < 64) Ls[0][tid] = lsv * 1.4426950408889634f;
  else if (tid < 128) Ds[0][tid - 64] = lsv;
  __syncthreads();
  for (int qt = qt0; qt < nqt; ++qt) {
    const int buf = (qt - qt0) & 1;
    const bool more = qt + 1 < nqt;
    if (more) {
      tile_load(Qb, ldq, (qt + 1) * 64, qr);
      tile_load(dOb, ldo, (qt + 1) * 64, gr);
      lsv = tid < 64 ? Lb[(qt + 1) * 64 + tid] : (tid < 128 ? Db[(qt + 1) * 64 + tid - 64] : 0.f);
    }
    const int qbase = qt * 64;
    if (k0 <= qbase + 63) {  // some query of this tile sees some key of this wave
      const char* Qs = lds + buf * TILE;
      const char* Gs = lds + 2 * TILE + buf * TILE;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        f32x16 S = {}, dP = {};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          S = mfma_bf16(row_frag(Qs, 32 * u + r, 2 * s + h), kf[s], S);
          dP = mfma_bf16(row_frag(Gs, 32 * u + r, 2 * s + h), vf[s], dP);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 l4 = *reinterpret_cast<const float4*>(&Ls[buf][32 * u + 8 * g + 4 * h]);
          const float4 d4 = *reinterpret_cast<const float4*>(&Ds[buf][32 * u + 8 * g + 4 * h]);
          const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
          const float dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int i = 4 * g + e;
            const int q = qbase + 32 * u + 8 * g + 4 * h + e;
            const float p = myk > q ? 0.f : exp2f(S[i] * sl2 - lv[e]);
            S[i] = p;
            dP[i] = p * (dP[i] - dv[e]);
          }
        }
        const bf16x8 p0 = frag_of<0>(S), p1 = frag_of<1>(S);
        const bf16x8 g0 = frag_of<0>(dP), g1 = frag_of<1>(dP);
        dv0 = mfma_bf16(p0, tr_frag(Gs, 32 * u, 0), dv0);
        dv1 = mfma_bf16(p0, tr_frag(Gs, 32 * u, 32), dv1);
        dv0 = mfma_bf16(p1, tr_frag(Gs, 32 * u + 16, 0), dv0);
        dv1 = mfma_bf16(p1, tr_frag(Gs, 32 * u + 16, 32), dv1);
        dk0 = mfma_bf16(g0, tr_frag(Qs, 32 * u, 0), dk0);
        dk1 = mfma_bf16(g0, tr_frag(Qs, 32 * u, 32), dk1);
        dk0 = mfma_bf16(g1, tr_frag(Qs, 32 * u + 16, 0), dk0);
        dk1 = mfma_bf16(g1, tr_frag(Qs, 32 * u + 16, 32), dk1);
      }
    }
    if (more) {
      tile_store(lds + (buf ^ 1) * TILE, qr);
      tile_store(lds + 2 * TILE + (buf ^ 1) * TILE, gr);
      if (tid < 64) Ls[buf ^ 1][tid] = lsv * 1.4426950408889634f;
      else if (tid < 128) Ds[buf ^ 1][tid - 64] = lsv;
    }
    __syncthreads();
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

}  // namespace

extern "C" {

hipError_t pde_attn_fwd(const void* q, const void* k, const void* v, int ldq, void* o, int ldo, float* lse, int B,
                        int T, int H, float scale, hipStream_t st) {
  if (T % 128 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_attn_fwd, dim3(T / 128, B * H), dim3(256), 0, st, (const bf16_t*)q, (const bf16_t*)k,
                     (const bf16_t*)v, ldq, (bf16_t*)o, ldo, lse, T, H, scale * 1.4426950408889634f, scale);
  return hipGetLastError();
}

hipError_t pde_attn_bwd(const void* q, const void* k, const void* v, int ldq, const void* o, const void* dout,
                        int ldo, const float* lse, float* Dd, void* dq, void* dk, void* dv, int B, int T, int H,
                        float scale, hipStream_t st) {
  if (T % 128 != 0) return hipErrorInvalidValue;
  const int N = B * T;
  hipLaunchKernelGGL(k_attn_bwd_pre, dim3((N * H + 255) / 256), dim3(256), 0, st, (const bf16_t*)o,
                     (const bf16_t*)dout, ldo, Dd, N, T, H);
  const float sl2 = scale * 1.4426950408889634f;
  hipLaunchKernelGGL(k_attn_bwd_dkdv, dim3(T / 128, B * H), dim3(256), 0, st, (const bf16_t*)q, (const bf16_t*)k,
                     (const bf16_t*)v, ldq, (const bf16_t*)dout, ldo, lse, Dd, (bf16_t*)dk, (bf16_t*)dv, T, H, sl2,
                     scale);
  hipLaunchKernelGGL(k_attn_bwd_dq, dim3(T / 128, B * H), dim3(256), 0, st, (const bf16_t*)q, (const bf16_t*)k,
                     (const bf16_t*)v, ldq, (const bf16_t*)dout, ldo, lse, Dd, (bf16_t*)dq, T, H, sl2, scale);
  return hipGetLastError();
}

}  // extern "C"
