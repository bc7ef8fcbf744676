// Device side of the xGMI peer all-reduce for use inside another kernel ("side blocks").
//
// peer_ar_f32_vblock(d, in, out, count, scale, vb, nvb, two_shot, lds2) runs virtual block vb of nvb of
// one all-reduce call (fp32 SUM * scale, in == out allowed) with exactly the protocol of the
// standalone kernel in csrc/runtime/peer_allreduce.hip (same flag slots, call counter and parity
// double-buffering), so fused and standalone calls interleave freely on one stream.  All threads of
// the block must call it; the host kernel must run the SAME nvb virtual blocks on every rank.
#pragma once
#include <hip/hip_runtime.h>

#include "pde_peer.h"

namespace pde {

typedef unsigned int peer_vec_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t* peer_flag(uint8_t* region, int phase, int vb, int src) {
  return reinterpret_cast<uint32_t*>(region) + (phase * kPeerMaxBlocks + vb) * kPeerMaxRanks + src;
}

// Block barrier with virtual block vb of every rank (see peer_allreduce.hip: peer_barrier).
// *bad (the caller's LDS word, block-uniform after the closing __syncthreads): set on a time-out, so
// the virtual block writes NaN instead of a partial sum (see peer_allreduce.hip: peer_barrier).
__device__ __forceinline__ void peer_vbarrier(const PeerDev& d, int phase, int vb, uint32_t target, bool failed,
                                              uint32_t* bad) {
  __builtin_amdgcn_s_waitcnt(0x0F70);          // vmcnt(0): this wave's stores have landed
  __syncthreads();
  const int t = threadIdx.x;
  if (t < d.world) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope: write back this XCD's L2
    __hip_atomic_store(peer_flag(d.flags[t], phase, vb, d.rank), target, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = peer_flag(d.flags[d.rank], phase, vb, t);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    int spins = 0;
    while (!failed && __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins == 256) {
        spins = 0;
        if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > d.timeout) {
          __hip_atomic_fetch_add(d.ctrl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (d.err_host) __hip_atomic_store(d.err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          *bad = 1u;
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
}

__device__ __forceinline__ peer_vec_t peer_sum(const peer_vec_t (&v)[kPeerMaxRanks], int W, float s) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
  for (int p = 0; p < kPeerMaxRanks; ++p) {
    if (p < W) {                                  // fixed rank order: bit-identical on every rank
      a0 += __uint_as_float(v[p].x);
      a1 += __uint_as_float(v[p].y);
      a2 += __uint_as_float(v[p].z);
      a3 += __uint_as_float(v[p].w);
    }
  }
  peer_vec_t r = {__float_as_uint(a0 * s), __float_as_uint(a1 * s), __float_as_uint(a2 * s), __float_as_uint(a3 * s)};
  return r;
}

// lds2: two words of the caller's LDS (no __shared__ object of our own: a second LDS object next to a
// kernel's single staging array can change how hipcc schedules that kernel).
__device__ bool peer_ar_f32_vblock(const PeerDev& d, const float* in_f, float* out_f, int64_t count, float scale,
                                   int vb, int nvb, bool two_shot, uint32_t* lds2) {
  const int T = blockDim.x;
  __syncthreads();                                // lds2 may alias LDS the caller just used
  if (threadIdx.x == 0) {
    lds2[0] = __hip_atomic_load(d.ctrl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lds2[1] = __hip_atomic_load(d.ctrl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const uint32_t call = lds2[0], par = call & 1u, target = call + 1u;
  const bool failed = lds2[1] != 0;
  const int W = d.world;
  const peer_vec_t* in = reinterpret_cast<const peer_vec_t*>(in_f);
  peer_vec_t* out = reinterpret_cast<peer_vec_t*>(out_f);
  const int64_t n4 = count / 4, tail = count - n4 * 4, last = n4 - 1;
  const int NC = two_shot ? W : 1;
  const int64_t chunk4 = two_shot ? (n4 + W - 1) / W : n4;
  const int64_t stride = (int64_t)nvb * T, t0 = (int64_t)vb * T + threadIdx.x;
  peer_vec_t* stage[kPeerMaxRanks];
  peer_vec_t* res[kPeerMaxRanks];
#pragma unroll
  for (int p = 0; p < kPeerMaxRanks; ++p) {
    const int q = p < W ? p : 0;
    stage[p] = reinterpret_cast<peer_vec_t*>(d.data[q] + par * d.cap);
    res[p] = reinterpret_cast<peer_vec_t*>(d.data[q] + (2 + par) * d.cap);
  }
  peer_vec_t* my_stage = reinterpret_cast<peer_vec_t*>(d.data[d.rank] + par * d.cap);
  // 1. stage the input: vector i of every chunk (chunk-relative) belongs to virtual block (i / T) % nvb
  for (int64_t i = t0; i < chunk4; i += stride) {
    peer_vec_t v[kPeerMaxRanks];
#pragma unroll
    for (int c = 0; c < kPeerMaxRanks; ++c) {      // c < NC is wave-uniform: scalar branches
      const int64_t g = (int64_t)c * chunk4 + i;
      if (c < NC) v[c] = in[g < last ? g : last];
    }
#pragma unroll
    for (int c = 0; c < kPeerMaxRanks; ++c) {
      const int64_t g = (int64_t)c * chunk4 + i;
      // own slice only: a clamped duplicate store would re-stage a value that the in-place output
      // of the owning virtual block may already have overwritten with the reduced sum
      if (c < NC && g <= last) my_stage[g] = v[c];
    }
  }
  if (vb == 0 && threadIdx.x < tail) reinterpret_cast<float*>(my_stage)[n4 * 4 + threadIdx.x] = in_f[n4 * 4 + threadIdx.x];
  peer_vbarrier(d, 0, vb, target, failed, lds2 + 1);
  bool bad = lds2[1] != 0;                        // poisoned before, or a wait of this block timed out
  const peer_vec_t vnan = {0x7FC00000u, 0x7FC00000u, 0x7FC00000u, 0x7FC00000u};
  if (vb == 0 && threadIdx.x < tail) {
    float acc = 0.f;
    for (int p = 0; p < W; ++p) acc += reinterpret_cast<const float*>(stage[p])[n4 * 4 + threadIdx.x];
    out_f[n4 * 4 + threadIdx.x] = bad ? __builtin_nanf("") : acc * scale;
  }
  const int64_t lo = two_shot ? (int64_t)d.rank * chunk4 : 0;
  const int64_t len = two_shot ? ((lo + chunk4 <= n4) ? chunk4 : (n4 > lo ? n4 - lo : 0)) : n4;
  // 2. reduce [lo, lo + len) over every rank's stage (own chunk when two-shot)
  for (int64_t i = t0; i < len; i += stride) {
    peer_vec_t v[kPeerMaxRanks];
#pragma unroll
    for (int p = 0; p < kPeerMaxRanks; ++p)
      if (p < W) v[p] = stage[p][lo + i];
    const peer_vec_t r = bad ? vnan : peer_sum(v, W, scale);
    out[lo + i] = r;
    if (two_shot) reinterpret_cast<peer_vec_t*>(d.data[d.rank] + (2 + par) * d.cap)[lo + i] = r;
  }
  if (two_shot) {
    peer_vbarrier(d, 1, vb, target, failed, lds2 + 1);
    bad = lds2[1] != 0;
    // 3. gather every other chunk from its owner's res[par]
    for (int64_t i = t0; i < chunk4; i += stride) {
      peer_vec_t v[kPeerMaxRanks];
#pragma unroll
      for (int q = 0; q < kPeerMaxRanks; ++q) {
        const int64_t g = (int64_t)q * chunk4 + i;
        if (q < W) v[q] = res[q][g < last ? g : last];
      }
#pragma unroll
      for (int q = 0; q < kPeerMaxRanks; ++q) {
        const int64_t g = (int64_t)q * chunk4 + i;
        if (q < W && q != d.rank && g <= last) out[g] = bad ? vnan : v[q];
      }
    }
  }
  // call bookkeeping: the last virtual block of this call advances the call number.  Every wave
  // drains its output stores first, so a consumer in the SAME kernel that sees the call complete
  // (agent-scope acquire) reads the reduced values.  Returns true in the thread that completed it.
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();
  bool completed = false;
  if (threadIdx.x == 0) {
    if (__hip_atomic_fetch_add(d.ctrl + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)nvb - 1) {
      __hip_atomic_store(d.ctrl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(d.ctrl, target, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      completed = true;
    }
  }
  return completed;
}


// ---- in-place (registered buffer) one-shot inside another kernel ------------------------------------
// Exactly peer_inplace_kernel's protocol (peer_allreduce.hip) with the rank count at run time: virtual
// block vb of every rank owns the same vectors; the arrival signal is an atomic add into this rank's
// phase-0 slot of every rank's flag region (the add on the own region returns the calls so far of slot
// vb: per-slot call numbers agree across ranks because every rank makes the same calls); barrier B
// (phase 1) publishes the call number once every buffer has been read.  Inputs must be in memory
// (earlier kernels, or system-scope write-through stores drained before the arrival).
__device__ __forceinline__ uint32_t* ipd_flag(uint8_t* region, int phase, int vb, int src) {
  return reinterpret_cast<uint32_t*>(region) + (phase * kPeerMaxBlocks + vb) * kPeerMaxRanks + src;
}

// lanes t < world: arrival add on this rank's slot in rank t's region; *s_call (LDS) <- calls so far
__device__ __forceinline__ void ipd_arrive(const PeerIpDev& d, int vb, uint32_t* s_call) {
  const int t = threadIdx.x;
  if (t < d.world) {
    uint32_t* slot = ipd_flag(d.flags[t], 0, vb, d.rank);
    const uint32_t old = __hip_atomic_fetch_add(slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (t == d.rank) *s_call = old;
  }
}

// wait (and with SIGNAL first publish `target` into every rank's slot for this rank) until every rank's
// slot in the own region holds `target`; skip_own: no signal to / poll of the own slot (barrier A: the
// arrival add already put `target` there; B / C: no other rank reads it, the drain orders own accesses)
template <bool SIGNAL>
__device__ __forceinline__ void ipd_barrier(const PeerIpDev& d, int phase, int vb, uint32_t target, bool failed,
                                            bool skip_own, uint32_t* bad) {
  if constexpr (SIGNAL) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const int t = threadIdx.x;
  if (t < d.world && !(skip_own && t == d.rank)) {
    if constexpr (SIGNAL)
      __hip_atomic_store(ipd_flag(d.flags[t], phase, vb, d.rank), target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = ipd_flag(d.flags[d.rank], phase, vb, t);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    int spins = 0;
    while (!failed && __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins == 256) {
        spins = 0;
        if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > d.timeout) {
          __hip_atomic_fetch_add(d.errc + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(d.err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          *bad = 1u;
          break;
        }
      }
    }
  }
  __syncthreads();
}

// 16-byte system-coherent (sc0 sc1) load / store through a buffer resource: served from memory, never
// from this CU's or XCD's caches (peers' data arrives over xGMI; own write-through stores land there)
constexpr int kIpdAuxSys = 1 | 16;
__device__ __forceinline__ peer_vec_t ipd_ld(__amdgpu_buffer_rsrc_t r, int64_t i) {
  return __builtin_bit_cast(peer_vec_t, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i * 16), 0, kIpdAuxSys));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ipd_rsrc(const uint8_t* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p), (short)0, (int)bytes, 0x00020000);
}

}  // namespace pde
