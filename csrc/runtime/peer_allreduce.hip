// Peer all-reduce over xGMI-mapped peer memory (design notes in peer_allreduce.h).
#include "peer_allreduce.h"
#include "pde_peer_dev.h"

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

namespace pde {

namespace {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP ") + what + " failed: " + hipGetErrorString(e));
}

constexpr int kThreads = 512;                 // 8 waves per block
constexpr int64_t kFlagBytes = kPeerFlagBytes;   // flags[2 phases][kPeerMaxBlocks][kPeerMaxRanks] u32 (16 KB used)
constexpr int kHandle = sizeof(hipIpcMemHandle_t);
// 16-byte vector as a clang vector type: arrays of HIP's struct vec_t defeat SROA and land in scratch
typedef unsigned int vec_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ vec_t mkvec(unsigned a, unsigned b, unsigned c, unsigned d) {
  vec_t v = {a, b, c, d};
  return v;
}

struct Args {
  uint8_t* flags[kPeerMaxRanks];  // every rank's flag region (uncached; [rank] = own)
  uint8_t* data[kPeerMaxRanks];   // every rank's stage0 | stage1 | res0 | res1 region
  const vec_t* in;
  vec_t* out;
  uint32_t* ctrl;                 // [0] completed calls, [1] blocks done in this call, [2] timeouts
  uint32_t* err_host;             // host-mapped mirror of ctrl[2] != 0 (read by the host without a sync)
  int64_t n4;                     // 16-byte vectors
  int64_t tail;                   // trailing elements (< elements per vector)
  int64_t chunk4;                 // two-shot chunk (vectors); == n4 for one-shot
  int64_t cap;                    // bytes per stage / res buffer
  int64_t timeout;                // s_memrealtime ticks
  float scale;
  int rank;
  int skip_stage;                 // test hook: leave own stage[par] as it is (a stale-buffer injection)
};

__device__ __forceinline__ uint32_t* flag_ptr(uint8_t* region, int phase, int block, int src) {
  return reinterpret_cast<uint32_t*>(region) + (phase * kPeerMaxBlocks + block) * kPeerMaxRanks + src;
}
__device__ __forceinline__ uint8_t* stage_ptr(uint8_t* region, int64_t cap, uint32_t par) {
  return region + par * cap;
}
__device__ __forceinline__ uint8_t* res_ptr(uint8_t* region, int64_t cap, uint32_t par) {
  return region + (2 + par) * cap;
}

// Block-level barrier between block b of every rank: publish `target` into every peer's flag slot
// for this rank, wait until every peer published it into ours.  Every thread first drains its own
// stores (vmcnt(0)); the signalling store is a system-scope release after the block barrier.
// *bad (LDS, block-uniform after the closing __syncthreads): set when this call's communicator was
// already poisoned or a wait timed out here -- the block then writes NaN instead of a partial sum,
// so a rank that went on without its peers never hands out plausible-looking wrong gradients.
template <int W>
__device__ __forceinline__ void peer_barrier(const Args& a, int phase, uint32_t target, bool failed,
                                             uint32_t* bad) {
  __builtin_amdgcn_s_waitcnt(0x0F70);          // vmcnt(0): this wave's stores have landed
  __syncthreads();
  const int t = threadIdx.x;
  if (t < W) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope: write back this XCD's L2
    __hip_atomic_store(flag_ptr(a.flags[t], phase, blockIdx.x, a.rank), target, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = flag_ptr(a.flags[a.rank], phase, blockIdx.x, t);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    int spins = 0;
    // after a time-out the communicator is poisoned: signal, never wait again (fail fast, no hang)
    while (!failed && __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins == 256) {
        spins = 0;
        if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > a.timeout) {   // dead / hung peer
          __hip_atomic_fetch_add(a.ctrl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          *bad = 1u;
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
}

struct F32Op {
  static __device__ __forceinline__ void zero(float* acc) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = 0.f;
  }
  static __device__ __forceinline__ void add(float* acc, vec_t v) {
    acc[0] += __uint_as_float(v.x); acc[1] += __uint_as_float(v.y);
    acc[2] += __uint_as_float(v.z); acc[3] += __uint_as_float(v.w);
  }
  static __device__ __forceinline__ vec_t pack(const float* acc, float s) {
    return mkvec(__float_as_uint(acc[0] * s), __float_as_uint(acc[1] * s), __float_as_uint(acc[2] * s),
                      __float_as_uint(acc[3] * s));
  }
  static __device__ __forceinline__ vec_t nan_vec() { return mkvec(0x7FC00000u, 0x7FC00000u, 0x7FC00000u, 0x7FC00000u); }
  static constexpr int kAcc = 4;
  static constexpr int kPerVec = 4;
  static __device__ __forceinline__ void tail_add(float& acc, const uint8_t* p, int64_t i) {
    acc += reinterpret_cast<const float*>(p)[i];
  }
  static __device__ __forceinline__ void tail_store(uint8_t* p, int64_t i, float v) {
    reinterpret_cast<float*>(p)[i] = v;
  }
  static __device__ __forceinline__ void tail_copy(uint8_t* d, const uint8_t* s, int64_t i) {
    reinterpret_cast<float*>(d)[i] = reinterpret_cast<const float*>(s)[i];
  }
};

struct BF16Op {
  static __device__ __forceinline__ void zero(float* acc) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  }
  static __device__ __forceinline__ void add(float* acc, vec_t v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[2 * i] += __uint_as_float(w[i] << 16);
      acc[2 * i + 1] += __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ uint32_t pk(float a, float b) {
    typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
    bf2 v;
    v[0] = (__bf16)a;
    v[1] = (__bf16)b;
    return __builtin_bit_cast(uint32_t, v);
  }
  static __device__ __forceinline__ vec_t pack(const float* acc, float s) {
    return mkvec(pk(acc[0] * s, acc[1] * s), pk(acc[2] * s, acc[3] * s), pk(acc[4] * s, acc[5] * s),
                      pk(acc[6] * s, acc[7] * s));
  }
  static __device__ __forceinline__ vec_t nan_vec() { return mkvec(0x7FC07FC0u, 0x7FC07FC0u, 0x7FC07FC0u, 0x7FC07FC0u); }
  static constexpr int kAcc = 8;
  static constexpr int kPerVec = 8;
  static __device__ __forceinline__ void tail_add(float& acc, const uint8_t* p, int64_t i) {
    acc += __uint_as_float(uint32_t(reinterpret_cast<const uint16_t*>(p)[i]) << 16);
  }
  static __device__ __forceinline__ void tail_store(uint8_t* p, int64_t i, float v) {
    reinterpret_cast<uint16_t*>(p)[i] = uint16_t(pk(v, 0.f) & 0xffffu);
  }
  static __device__ __forceinline__ void tail_copy(uint8_t* d, const uint8_t* s, int64_t i) {
    reinterpret_cast<uint16_t*>(d)[i] = reinterpret_cast<const uint16_t*>(s)[i];
  }
};

// Sum vector i over every rank's stage[par] in fixed rank order (bit-identical on every rank).
template <int W, typename Op>
__device__ __forceinline__ vec_t sum_ranks(const vec_t (&v)[W], float scale) {
  float acc[Op::kAcc];
  Op::zero(acc);
#pragma unroll
  for (int p = 0; p < W; ++p) Op::add(acc, v[p]);
  return Op::pack(acc, scale);
}

// out[i] (and res[i] when given) = sum over ranks of stage_p[i] for i in [lo, lo + len), this
// thread's grid-stride share, two vectors per iteration: 2W independent loads in flight.
template <int W, typename Op>
__device__ __forceinline__ void reduce_range(const Args& a, uint32_t par, int64_t lo, int64_t len, int64_t t0,
                                             int64_t stride, vec_t* res, bool bad) {
  const vec_t* st[W];
#pragma unroll
  for (int p = 0; p < W; ++p) st[p] = reinterpret_cast<const vec_t*>(stage_ptr(a.data[p], a.cap, par)) + lo;
  for (int64_t i = t0; i < len; i += 2 * stride) {
    const int64_t j = i + stride;
    const int64_t jj = j < len ? j : i;
    vec_t v0[W], v1[W];
#pragma unroll
    for (int p = 0; p < W; ++p) {
      v0[p] = st[p][i];
      v1[p] = st[p][jj];
    }
    const vec_t r0 = bad ? Op::nan_vec() : sum_ranks<W, Op>(v0, a.scale);
    const vec_t r1 = bad ? Op::nan_vec() : sum_ranks<W, Op>(v1, a.scale);
    a.out[lo + i] = r0;
    if (res) res[lo + i] = r0;
    if (j < len) {
      a.out[lo + j] = r1;
      if (res) res[lo + j] = r1;
    }
  }
}

template <int W, bool TWO, typename Op>
__global__ void __launch_bounds__(kThreads) peer_allreduce_kernel(Args a) {
  __shared__ uint32_t s_call, s_failed, s_bad;
  if (threadIdx.x == 0) {
    s_call = __hip_atomic_load(a.ctrl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_failed = __hip_atomic_load(a.ctrl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_bad = s_failed;
  }
  __syncthreads();
  const uint32_t call = s_call;
  const bool failed = s_failed != 0;
  const uint32_t par = call & 1u, target = call + 1u;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  const int64_t t0 = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  constexpr int NC = TWO ? W : 1;                    // chunks
  constexpr int U = NC >= 8 ? 1 : 8 / NC;            // vectors per chunk per iteration: ~8 loads in flight
  vec_t* my_stage = reinterpret_cast<vec_t*>(stage_ptr(a.data[a.rank], a.cap, par));
  const int64_t last = a.n4 - 1;

  // 1. stage this rank's input.  Slices are chunk-relative (vector i of every chunk belongs to block
  //    (i / kThreads) % gridDim.x on every rank), so a block-level barrier suffices below.
  for (int64_t i = a.skip_stage ? a.chunk4 : t0; i < a.chunk4; i += U * stride) {
    vec_t v[NC * U];
#pragma unroll
    for (int k = 0; k < NC * U; ++k) {
      const int64_t g = (int64_t)(k / U) * a.chunk4 + i + (k % U) * stride;
      v[k] = a.in[g < last ? g : last];             // clamped: every load unconditional
    }
    // stores only for this block's own slice (index inside its chunk and inside the buffer).  (An
    // earlier version also stored clamped / next-chunk indices, "rewriting an element with the same
    // input" -- but the all-reduce runs in place: the block owning that element may already have
    // passed its barrier and written the REDUCED value into a.in, and the lagging block then staged
    // that sum over the peers' input: a wrong last vector on every rank, seen with 4 ranks
    // time-sharing one GPU.)
#pragma unroll
    for (int k = 0; k < NC * U; ++k) {
      const int64_t idx = i + (k % U) * stride, g = (int64_t)(k / U) * a.chunk4 + idx;
      if (idx < a.chunk4 && g <= last) my_stage[g] = v[k];
    }
  }
  const int64_t tail_off = a.n4 * Op::kPerVec;
  if (blockIdx.x == 0 && threadIdx.x < a.tail && !a.skip_stage)
    Op::tail_copy(reinterpret_cast<uint8_t*>(my_stage), reinterpret_cast<const uint8_t*>(a.in),
                  tail_off + threadIdx.x);
  peer_barrier<W>(a, 0, target, failed, &s_bad);
  bool bad = s_bad != 0;

  if (blockIdx.x == 0 && threadIdx.x < a.tail) {   // tail: every rank reduces it itself, same order
    float acc = 0.f;
    for (int p = 0; p < W; ++p) Op::tail_add(acc, stage_ptr(a.data[p], a.cap, par), tail_off + threadIdx.x);
    Op::tail_store(reinterpret_cast<uint8_t*>(a.out), tail_off + threadIdx.x, bad ? __builtin_nanf("") : acc * a.scale);
  }
  if (!TWO) {
    reduce_range<W, Op>(a, par, 0, a.n4, t0, stride, nullptr, bad);
  } else {
    // 2. reduce this rank's chunk from every peer's stage into own res[par] (+ own output)
    const int64_t lo = (int64_t)a.rank * a.chunk4;
    const int64_t len = (lo + a.chunk4 <= a.n4) ? a.chunk4 : (a.n4 > lo ? a.n4 - lo : 0);
    reduce_range<W, Op>(a, par, lo, len, t0, stride, reinterpret_cast<vec_t*>(res_ptr(a.data[a.rank], a.cap, par)),
                        bad);
    peer_barrier<W>(a, 1, target, failed, &s_bad);
    bad = s_bad != 0;
    // 3. gather every chunk from its owner's res[par] (W loads in flight; own chunk already in out)
    for (int64_t i = t0; i < a.chunk4; i += stride) {
      vec_t v[W];
#pragma unroll
      for (int q = 0; q < W; ++q) {
        const int64_t g = (int64_t)q * a.chunk4 + i;
        v[q] = reinterpret_cast<const vec_t*>(res_ptr(a.data[q], a.cap, par))[g < last ? g : last];
      }
#pragma unroll
      for (int q = 0; q < W; ++q) {
        const int64_t g = (int64_t)q * a.chunk4 + i;
        if (q != a.rank && g <= last) a.out[g] = bad ? Op::nan_vec() : v[q];
      }
    }
  }
  // call bookkeeping: the last block of this call advances the call number
  __syncthreads();
  if (threadIdx.x == 0) {
    if (__hip_atomic_fetch_add(a.ctrl + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      __hip_atomic_store(a.ctrl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.ctrl, target, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// The device-side protocol of pde_peer_dev.h (run by side blocks of the fused LeNet / Adam kernels)
// as a kernel of its own: every block is one virtual block.  Used by the self-test, so that path is
// checked across devices before any schedule that uses it is timed.
__global__ void __launch_bounds__(kThreads) peer_dev_probe_kernel(PeerDev d, const float* in, float* out,
                                                                  int64_t count, float scale, int two) {
  __shared__ uint32_t lds2[2];
  peer_ar_f32_vblock(d, in, out, count, scale, blockIdx.x, gridDim.x, two != 0, lds2);
}


// ============================================================================ in-place (registered)
// See peer_allreduce.h.  Block b of every rank owns the same vectors; barriers are per block index.
struct IpArgs {
  uint8_t* data[kPeerMaxRanks];    // every rank's buffer at this call's first element (mapped here)
  uint8_t* flags[kPeerMaxRanks];   // every rank's in-place flag region
  uint32_t* errc;                  // the staged protocol's ctrl: [2] = time-out count (shared latch)
  uint32_t* err_host;
  int64_t n4, tail, chunk4, bytes;
  int64_t timeout;
  float scale;
  int rank;
};
constexpr int kAuxSys = 1 | 16;    // sc0 sc1: system-scope (coherent across GPUs) load / write-through store

__device__ __forceinline__ uint32_t* ip_flag(uint8_t* region, int phase, int block, int src) {
  return reinterpret_cast<uint32_t*>(region) + (phase * kPeerMaxBlocks + block) * kPeerMaxRanks + src;
}
__device__ __forceinline__ vec_t ld_sys(__amdgpu_buffer_rsrc_t r, int64_t i) {
  return __builtin_bit_cast(vec_t, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i * 16), 0, kAuxSys));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ip_rsrc(const uint8_t* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p), (short)0, (int)bytes, 0x00020000);
}

// Flag barrier of block b across ranks, NO fences: every wave drains its memory operations (loads
// consumed, write-through stores acknowledged), then lane t < W stores the call number into rank t's
// slot for this rank and waits for rank t's store into ours (relaxed system-scope accesses to
// uncached memory).  A time-out poisons the call (NaN results) and latches the error words.
// SKIP_OWN: no signal to and no poll of this rank's own slot.  Barrier A: the slot already holds
// `target` (its signal is an atomic add whose return value this block waited for).  Barriers B / C:
// nobody else reads a rank's own slot, and the drain above already orders this block's own accesses;
// the store-then-poll round trip on uncached memory was pure latency (-0.54 us per one-shot call and
// -1.08 us per two-shot call at W = 1, profiles/r6_comm/skip_own_bc/).
template <int W, bool SIGNAL = true, bool SKIP_OWN = false>
__device__ __forceinline__ void ip_barrier(const IpArgs& a, int phase, uint32_t target, bool failed, uint32_t* bad) {
  if constexpr (SIGNAL) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const int t = threadIdx.x;
  if (t < W && !(SKIP_OWN && t == a.rank)) {
    if constexpr (SIGNAL)
      __hip_atomic_store(ip_flag(a.flags[t], phase, blockIdx.x, a.rank), target, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = ip_flag(a.flags[a.rank], phase, blockIdx.x, t);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    int spins = 0;
    while (!failed && __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins == 256) {
        spins = 0;
        if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > a.timeout) {
          __hip_atomic_fetch_add(a.errc + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          *bad = 1u;
          break;
        }
      }
    }
  }
  __syncthreads();
}

// Call numbers are per block index: block b of every rank runs in the same calls (same sizes on every
// rank), so its count agrees across ranks with no grid-wide "last block" atomic (the former done
// counter serialised every block's exit on one uncached address).  The count lives in barrier A's
// own flag slots: at the start lane t < W adds 1 to this rank's slot in rank t's region -- the arrival
// signal -- and the add on this rank's OWN region returns the calls so far, so no separate counter
// load precedes the signal (one memory round trip less per call; the remote adds are posted).  (The
// staged protocol keeps its global counter: its stage parity must flip for ALL blocks between calls
// whose grids differ.)  U: 16-byte vectors per thread in the one-shot form (held across barrier B).
template <int W, bool TWO, int U, typename Op>
__global__ void __launch_bounds__(kThreads) peer_inplace_kernel(IpArgs a) {
  __shared__ uint32_t s_call, s_bad;
  {
    const int t = threadIdx.x;
    if (t < W) {
      uint32_t* slot = ip_flag(a.flags[t], 0, blockIdx.x, a.rank);
      if (t == a.rank) s_call = __hip_atomic_fetch_add(slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      else (void)__hip_atomic_fetch_add(slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (t == 64) s_bad = __hip_atomic_load(a.errc + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  constexpr int ESZ = 16 / Op::kPerVec;                  // element bytes (4: fp32, 2: bf16)
  const uint32_t target = s_call + 1u;
  const bool failed = s_bad != 0;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  const int64_t t0 = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  __amdgpu_buffer_rsrc_t rs[W];
#pragma unroll
  for (int p = 0; p < W; ++p) rs[p] = ip_rsrc(a.data[p], a.bytes);
  uint8_t* own = a.data[a.rank];
  const int64_t tail_off = a.n4 * Op::kPerVec;           // first trailing element
  const bool tail_lane = blockIdx.x == 0 && threadIdx.x < a.tail;
  float tail_sum = 0.f;

  // A: every rank's buffer holds its input.  No release is needed in front of the signal: the input was
  // written by EARLIER kernels of this stream, and the kernel boundary between them and this launch is
  // at least an agent-scope release -- on gfx950 `buffer_wbl2 sc1`, which writes every XCD L2's dirty
  // lines back to memory (the eight XCD L2s are not coherent with each other, so agent scope already
  // means memory-side visibility: MI355X_MICROARCH.md, inter-workgroup visibility).  Peers read with
  // sc0 sc1 (system-coherent) loads that are served from memory / MALL over xGMI, never from this
  // rank's L2.  (A fence here would only write back the XCD this block runs on, not the producer's.)
  // The results are plain stores: their readers are this rank's own later kernels, and the peers read
  // this range again only after the next call's barrier A, behind the same kernel-boundary release.
  // The registration self-test (dist/peer.py) exercises exactly this producer -> in-place hand-off.
  ip_barrier<W, false, true>(a, 0, target, failed, &s_bad);
  if (tail_lane) {                                      // trailing elements: read now, written after B
    const int tb = (int)((tail_off + threadIdx.x) * ESZ);
#pragma unroll
    for (int p = 0; p < W; ++p) {
      if constexpr (ESZ == 4)
        tail_sum += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs[p], tb, 0, kAuxSys));
      else
        tail_sum += __uint_as_float((uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rs[p], tb, 0, kAuxSys) << 16);
    }
  }
  if (!TWO) {
    // host guarantees gridDim * kThreads * U >= n4
    float acc[U][Op::kAcc];
    vec_t v[U][W];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = t0 + u * stride;
#pragma unroll
      for (int p = 0; p < W; ++p) v[u][p] = ld_sys(rs[p], i < a.n4 ? i : 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      Op::zero(acc[u]);
#pragma unroll
      for (int p = 0; p < W; ++p) Op::add(acc[u], v[u][p]);  // fixed rank order: bit-identical on every rank
    }
    ip_barrier<W, true, true>(a, 1, target, failed, &s_bad);   // B: every rank has read every buffer
    const bool bad = s_bad != 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = t0 + u * stride;
      if (i < a.n4) reinterpret_cast<vec_t*>(own)[i] = bad ? Op::nan_vec() : Op::pack(acc[u], a.scale);
    }
    if (tail_lane) Op::tail_store(own, tail_off + threadIdx.x, bad ? __builtin_nanf("") : tail_sum * a.scale);
  } else {
    // reduce-scatter: my chunk from every rank, written through into my own buffer
    const int64_t lo = (int64_t)a.rank * a.chunk4;
    const int64_t len = lo + a.chunk4 <= a.n4 ? a.chunk4 : (a.n4 > lo ? a.n4 - lo : 0);
    const __amdgpu_buffer_rsrc_t ro = rs[a.rank];
    // R vectors per thread per iteration: R * W uncached loads in flight (one per iteration was
    // latency-bound: ~0.75 TB/s on a 248 MB GPT-2 gradient at W = 1)
    constexpr int R = W <= 2 ? 4 : (W <= 4 ? 2 : 1);
    for (int64_t i0 = t0; i0 < len; i0 += R * stride) {
      vec_t v[R][W];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int64_t i = i0 + r * stride;
#pragma unroll
        for (int p = 0; p < W; ++p) v[r][p] = ld_sys(rs[p], lo + (i < len ? i : i0));
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int64_t i = i0 + r * stride;
        float acc[Op::kAcc];
        Op::zero(acc);
#pragma unroll
        for (int p = 0; p < W; ++p) Op::add(acc, v[r][p]);
        const vec_t o = s_bad ? Op::nan_vec() : Op::pack(acc, a.scale);
        if (i < len) __builtin_amdgcn_raw_buffer_store_b128(o, ro, (int)((lo + i) * 16), 0, kAuxSys);
      }
    }
    ip_barrier<W, true, true>(a, 1, target, failed, &s_bad);   // B: every chunk reduced, every input read
    const bool bad = s_bad != 0;
    if (tail_lane) Op::tail_store(own, tail_off + threadIdx.x, bad ? __builtin_nanf("") : tail_sum * a.scale);
    // all-gather: chunk q from its owner q (W-1 loads in flight per lane)
    const int64_t last = a.n4 - 1;
    constexpr int RG = W <= 2 ? 4 : (W <= 4 ? 2 : 1);
    for (int64_t i0 = t0; i0 < a.chunk4; i0 += RG * stride) {
      vec_t v[RG][W];
#pragma unroll
      for (int r = 0; r < RG; ++r) {
        const int64_t i = i0 + r * stride;
#pragma unroll
        for (int q = 0; q < W; ++q) {
          const int64_t g = (int64_t)q * a.chunk4 + i;
          v[r][q] = (q == a.rank) ? vec_t{0u, 0u, 0u, 0u} : ld_sys(rs[q], g < last ? g : last);
        }
      }
#pragma unroll
      for (int r = 0; r < RG; ++r) {
        const int64_t i = i0 + r * stride;
#pragma unroll
        for (int q = 0; q < W; ++q) {
          const int64_t g = (int64_t)q * a.chunk4 + i;
          if (q != a.rank && i < a.chunk4 && g <= last) reinterpret_cast<vec_t*>(own)[g] = bad ? Op::nan_vec() : v[r][q];
        }
      }
    }
    ip_barrier<W, true, true>(a, 2, target, failed, &s_bad);   // C: every rank has gathered from every owner
  }
}

template <bool TWO, int U, typename Op>
void ip_launch(int world, const IpArgs& a, int nb, hipStream_t s) {
  switch (world) {
#define PDE_IP_CASE(W) \
    case W: hipLaunchKernelGGL((peer_inplace_kernel<W, TWO, U, Op>), dim3(nb), dim3(kThreads), 0, s, a); break;
    PDE_IP_CASE(1) PDE_IP_CASE(2) PDE_IP_CASE(3) PDE_IP_CASE(4) PDE_IP_CASE(5) PDE_IP_CASE(6) PDE_IP_CASE(7)
    PDE_IP_CASE(8)
#undef PDE_IP_CASE
    default: throw std::invalid_argument("peer all-reduce supports 1..8 ranks");
  }
}

template <typename Op>
void ip_dispatch(int world, const IpArgs& a, bool two, int64_t u, int nb, hipStream_t s) {
  if (two) ip_launch<true, 1, Op>(world, a, nb, s);
  else if (u == 1) ip_launch<false, 1, Op>(world, a, nb, s);
  else if (u == 2) ip_launch<false, 2, Op>(world, a, nb, s);
  else ip_launch<false, 4, Op>(world, a, nb, s);
}


template <int W, typename Op>
void launch_w(const Args& a, bool two, int nb, hipStream_t s) {
  if (two)
    hipLaunchKernelGGL((peer_allreduce_kernel<W, true, Op>), dim3(nb), dim3(kThreads), 0, s, a);
  else
    hipLaunchKernelGGL((peer_allreduce_kernel<W, false, Op>), dim3(nb), dim3(kThreads), 0, s, a);
}

template <typename Op>
void launch_any(int world, const Args& a, bool two, int nb, hipStream_t s) {
  switch (world) {
    case 1: launch_w<1, Op>(a, two, nb, s); break;
    case 2: launch_w<2, Op>(a, two, nb, s); break;
    case 3: launch_w<3, Op>(a, two, nb, s); break;
    case 4: launch_w<4, Op>(a, two, nb, s); break;
    case 5: launch_w<5, Op>(a, two, nb, s); break;
    case 6: launch_w<6, Op>(a, two, nb, s); break;
    case 7: launch_w<7, Op>(a, two, nb, s); break;
    case 8: launch_w<8, Op>(a, two, nb, s); break;
    default: throw std::invalid_argument("peer all-reduce supports 1..8 ranks");
  }
}

}  // namespace

PeerAllReduce::PeerAllReduce(int rank, int world, int device, int64_t capacity_bytes, bool uncached_data)
    : rank_(rank), world_(world), device_(device), uncached_data_(uncached_data) {
  if (world < 1 || world > kPeerMaxRanks) throw std::invalid_argument("peer all-reduce supports 1..8 ranks");
  if (rank < 0 || rank >= world) throw std::invalid_argument("bad rank");
  cap_ = (capacity_bytes + 65535) / 65536 * 65536;
  region_bytes_ = 4 * cap_;
  hip_check(hipSetDevice(device), "hipSetDevice");
  void* f = nullptr;
  hip_check(hipExtMallocWithFlags(&f, kFlagBytes, hipDeviceMallocUncached), "hipExtMallocWithFlags(flags)");
  flags_ = static_cast<uint8_t*>(f);
  hip_check(hipMemset(flags_, 0, kFlagBytes), "hipMemset");
  void* p = nullptr;
  if (uncached_data)
    hip_check(hipExtMallocWithFlags(&p, region_bytes_, hipDeviceMallocUncached), "hipExtMallocWithFlags(data)");
  else
    hip_check(hipMalloc(&p, region_bytes_), "hipMalloc(data)");
  region_ = static_cast<uint8_t*>(p);
  hip_check(hipMemset(region_, 0, region_bytes_), "hipMemset");
  void* c = nullptr;
  hip_check(hipExtMallocWithFlags(&c, 256, hipDeviceMallocUncached), "hipExtMallocWithFlags(ctrl)");
  ctrl_ = static_cast<uint32_t*>(c);
  hip_check(hipMemset(ctrl_, 0, 256), "hipMemset");
  void* eh = nullptr;
  hip_check(hipHostMalloc(&eh, 64, hipHostMallocCoherent | hipHostMallocMapped), "hipHostMalloc(err)");
  err_host_ = static_cast<volatile uint32_t*>(eh);
  std::memset(eh, 0, 64);
  void* ed = nullptr;
  hip_check(hipHostGetDevicePointer(&ed, eh, 0), "hipHostGetDevicePointer(err)");
  err_dev_ = static_cast<uint32_t*>(ed);
  void* ipf = nullptr;
  hip_check(hipExtMallocWithFlags(&ipf, kFlagBytes, hipDeviceMallocUncached), "hipExtMallocWithFlags(ipflags)");
  ipflags_ = static_cast<uint8_t*>(ipf);
  hip_check(hipMemset(ipflags_, 0, kFlagBytes), "hipMemset");
  if (const char* e = std::getenv("PDE_PEER_IP_VPT")) ip_vpt_ = std::atoi(e) < 1 ? 1 : std::atoi(e);
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  peers_[rank_] = region_;
  peer_flags_[rank_] = flags_;
  peer_ipflags_[rank_] = ipflags_;
}

PeerAllReduce::~PeerAllReduce() {
  try {
    close();
  } catch (...) {
  }
}

void PeerAllReduce::close() {
  if (region_ == nullptr) return;
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) continue;
    if (peers_[p] != nullptr) (void)hipIpcCloseMemHandle(peers_[p]);
    if (peer_flags_[p] != nullptr) (void)hipIpcCloseMemHandle(peer_flags_[p]);
    if (peer_ipflags_[p] != nullptr) (void)hipIpcCloseMemHandle(peer_ipflags_[p]);
  }
  for (auto& kv : ipc_open_) (void)hipIpcCloseMemHandle(kv.second);
  ipc_open_.clear();
  regs_.clear();
  for (auto& q : peers_) q = nullptr;
  for (auto& q : peer_flags_) q = nullptr;
  for (auto& q : peer_ipflags_) q = nullptr;
  (void)hipFree(ipflags_);
  ipflags_ = nullptr;
  (void)hipFree(region_);
  (void)hipFree(flags_);
  (void)hipFree(ctrl_);
  if (err_host_ != nullptr) (void)hipHostFree(const_cast<uint32_t*>(err_host_));
  err_host_ = nullptr;
  err_dev_ = nullptr;
  region_ = nullptr;
  flags_ = nullptr;
  ctrl_ = nullptr;
  opened_ = false;
}

std::string PeerAllReduce::handle() const {
  hipIpcMemHandle_t h[3];
  hip_check(hipIpcGetMemHandle(&h[0], flags_), "hipIpcGetMemHandle(flags)");
  hip_check(hipIpcGetMemHandle(&h[1], region_), "hipIpcGetMemHandle(data)");
  hip_check(hipIpcGetMemHandle(&h[2], ipflags_), "hipIpcGetMemHandle(in-place flags)");
  return std::string(reinterpret_cast<const char*>(h), sizeof(h));
}

void PeerAllReduce::open(const std::vector<std::string>& handles) {
  if ((int)handles.size() != world_) throw std::invalid_argument("need one IPC handle per rank");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) continue;
    if (handles[p].size() != 3 * kHandle) throw std::invalid_argument("bad IPC handle size");
    hipIpcMemHandle_t h[3];
    std::memcpy(h, handles[p].data(), sizeof(h));
    void* fp = nullptr;
    void* dp = nullptr;
    void* ip = nullptr;
    hip_check(hipIpcOpenMemHandle(&fp, h[0], hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(flags)");
    peer_flags_[p] = static_cast<uint8_t*>(fp);
    hip_check(hipIpcOpenMemHandle(&dp, h[1], hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(data)");
    peers_[p] = static_cast<uint8_t*>(dp);
    hip_check(hipIpcOpenMemHandle(&ip, h[2], hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(in-place flags)");
    peer_ipflags_[p] = static_cast<uint8_t*>(ip);
  }
  opened_ = true;
}

void PeerAllReduce::launch(uintptr_t in, uintptr_t out, int64_t count, float scale, int algo, uintptr_t stream,
                           bool bf16) {
  if (!opened_) throw std::runtime_error("peer all-reduce used before open()");
  const int esize = bf16 ? 2 : 4;
  const int per_vec = 16 / esize;
  if (count <= 0) return;
  if (count * esize > cap_) throw std::invalid_argument("peer all-reduce buffer exceeds the registered capacity");
  if ((in | out) & 15) throw std::invalid_argument("peer all-reduce needs 16-byte aligned buffers");
  Args a;
  for (int p = 0; p < kPeerMaxRanks; ++p) {
    a.data[p] = p < world_ ? peers_[p] : nullptr;
    a.flags[p] = p < world_ ? peer_flags_[p] : nullptr;
  }
  a.in = reinterpret_cast<const vec_t*>(in);
  a.out = reinterpret_cast<vec_t*>(out);
  a.ctrl = ctrl_;
  a.err_host = err_dev_;
  a.n4 = count / per_vec;
  a.tail = count - a.n4 * per_vec;
  a.cap = cap_;
  a.timeout = timeout_ticks_;
  a.scale = scale;
  a.rank = rank_;
  a.skip_stage = 0;
  if (debug_skip_stage_ > 0) {
    a.skip_stage = 1;
    --debug_skip_stage_;
  }
  const bool two = algo == 2 || (algo == 0 && world_ > 2 && count * esize > one_shot_max_);
  a.chunk4 = two ? (a.n4 + world_ - 1) / world_ : a.n4;
  int64_t work = two ? a.chunk4 : a.n4;
  int64_t nb = (work + kThreads - 1) / kThreads;
  if (nb < 1) nb = 1;
  if (nb > max_blocks_) nb = max_blocks_;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (bf16)
    launch_any<BF16Op>(world_, a, two, (int)nb, s);
  else
    launch_any<F32Op>(world_, a, two, (int)nb, s);
  hip_check(hipGetLastError(), "peer all-reduce launch");
}

void PeerAllReduce::all_reduce_f32(uintptr_t in, uintptr_t out, int64_t count, float scale, int algo,
                                   uintptr_t stream) {
  launch(in, out, count, scale, algo, stream, false);
}

void PeerAllReduce::all_reduce_bf16(uintptr_t in, uintptr_t out, int64_t count, float scale, int algo,
                                    uintptr_t stream) {
  launch(in, out, count, scale, algo, stream, true);
}

std::string PeerAllReduce::device_args() const {
  if (!opened_) throw std::runtime_error("peer all-reduce used before open()");
  PeerDev d{};
  for (int p = 0; p < kPeerMaxRanks; ++p) {
    d.flags[p] = p < world_ ? peer_flags_[p] : nullptr;
    d.data[p] = p < world_ ? peers_[p] : nullptr;
  }
  d.ctrl = ctrl_;
  d.err_host = err_dev_;
  d.cap = cap_;
  d.timeout = timeout_ticks_;
  d.rank = rank_;
  d.world = world_;
  return std::string(reinterpret_cast<const char*>(&d), sizeof(d));
}

void PeerAllReduce::device_probe_f32(uintptr_t in, uintptr_t out, int64_t count, float scale, int two,
                                     uintptr_t stream) {
  if (!opened_) throw std::runtime_error("peer all-reduce used before open()");
  if (count <= 0) return;
  if (count * 4 > cap_) throw std::invalid_argument("peer all-reduce buffer exceeds the registered capacity");
  if ((in | out) & 15) throw std::invalid_argument("peer all-reduce needs 16-byte aligned buffers");
  PeerDev d{};
  for (int p = 0; p < kPeerMaxRanks; ++p) {
    d.flags[p] = p < world_ ? peer_flags_[p] : nullptr;
    d.data[p] = p < world_ ? peers_[p] : nullptr;
  }
  d.ctrl = ctrl_;
  d.err_host = err_dev_;
  d.cap = cap_;
  d.timeout = timeout_ticks_;
  d.rank = rank_;
  d.world = world_;
  const int64_t n4 = count / 4;
  const int64_t work = two ? (n4 + world_ - 1) / world_ : n4;
  int64_t nb = (work + kThreads - 1) / kThreads;
  nb = nb < 1 ? 1 : (nb > 16 ? 16 : nb);
  hipLaunchKernelGGL(peer_dev_probe_kernel, dim3((int)nb), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream), d,
                     reinterpret_cast<const float*>(in), reinterpret_cast<float*>(out), count, scale, two);
  hip_check(hipGetLastError(), "peer device-path probe launch");
}

std::string PeerAllReduce::registered_device_args(int id) const {
  if (id < 0 || id >= (int)regs_.size() || !regs_[id].open) throw std::runtime_error("registration not open");
  const Reg& r = regs_[id];
  PeerIpDev d{};
  for (int p = 0; p < kPeerMaxRanks; ++p) {
    d.data[p] = p < world_ ? r.base[p] : nullptr;
    d.flags[p] = p < world_ ? peer_ipflags_[p] : nullptr;
  }
  d.errc = ctrl_;
  d.err_host = err_dev_;
  d.bytes = r.bytes;
  d.timeout = timeout_ticks_;
  d.rank = rank_;
  d.world = world_;
  d.block_cap = ip_block_cap_;
  return std::string(reinterpret_cast<const char*>(&d), sizeof(d));
}

std::string PeerAllReduce::register_buffer(uintptr_t ptr, int64_t bytes, int* id) {
  if (ptr & 15) throw std::invalid_argument("registered buffers must be 16-byte aligned");
  if (bytes <= 0 || bytes > 0x7fffffffLL) throw std::invalid_argument("registered buffer size must be in (0, 2 GB)");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  void* base = nullptr;
  size_t size = 0;
  hip_check(hipMemGetAddressRange(&base, &size, reinterpret_cast<void*>(ptr)), "hipMemGetAddressRange");
  const int64_t off = (int64_t)(ptr - reinterpret_cast<uintptr_t>(base));
  if (off < 0 || off + bytes > (int64_t)size) throw std::invalid_argument("buffer outside its allocation");
  hipIpcMemHandle_t h;
  hip_check(hipIpcGetMemHandle(&h, base), "hipIpcGetMemHandle(registered)");   // the allocation's base: offset 0
  Reg r;
  r.base[rank_] = reinterpret_cast<uint8_t*>(ptr);
  r.bytes = bytes;
  regs_.push_back(r);
  *id = (int)regs_.size() - 1;
  std::string out(reinterpret_cast<const char*>(&h), sizeof(h));
  out.append(reinterpret_cast<const char*>(&off), sizeof(off));
  out.append(reinterpret_cast<const char*>(&bytes), sizeof(bytes));
  return out;
}

void PeerAllReduce::open_registered(int id, const std::vector<std::string>& handles) {
  if (id < 0 || id >= (int)regs_.size()) throw std::invalid_argument("unknown registration");
  if ((int)handles.size() != world_) throw std::invalid_argument("need one registration handle per rank");
  if (!opened_) throw std::runtime_error("open() the peer regions before registered buffers");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  Reg& r = regs_[id];
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) continue;
    const std::string& s = handles[p];
    if (s.size() != kHandle + 16) throw std::invalid_argument("bad registration handle size");
    hipIpcMemHandle_t h;
    int64_t off = 0, bytes = 0;
    std::memcpy(&h, s.data(), kHandle);
    std::memcpy(&off, s.data() + kHandle, 8);
    std::memcpy(&bytes, s.data() + kHandle + 8, 8);
    if (bytes != r.bytes) throw std::invalid_argument("registered buffers differ in size across ranks");
    if (off & 15) throw std::invalid_argument("a peer's registered buffer is not 16-byte aligned");
    const auto key = std::make_pair(p, std::string(s.data(), kHandle));
    auto it = ipc_open_.find(key);
    if (it == ipc_open_.end()) {
      void* m = nullptr;
      hip_check(hipIpcOpenMemHandle(&m, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(registered)");
      it = ipc_open_.emplace(key, static_cast<uint8_t*>(m)).first;
    }
    r.base[p] = it->second + off;
  }
  r.open = true;
}

int64_t PeerAllReduce::registered_bytes(int id) const {
  if (id < 0 || id >= (int)regs_.size()) throw std::invalid_argument("unknown registration");
  return regs_[id].bytes;
}

void PeerAllReduce::all_reduce_registered_f32(int id, int64_t off, int64_t count, float scale, int algo,
                                              uintptr_t stream) {
  all_reduce_registered(id, off, count, 4, scale, algo, stream);
}

void PeerAllReduce::all_reduce_registered(int id, int64_t off, int64_t count, int esz, float scale, int algo,
                                          uintptr_t stream) {
  if (id < 0 || id >= (int)regs_.size() || !regs_[id].open) throw std::runtime_error("registration not open");
  if (esz != 4 && esz != 2) throw std::invalid_argument("in-place all-reduce: fp32 (4) or bf16 (2) elements");
  const Reg& r = regs_[id];
  if (count <= 0) return;
  if (off < 0 || (off + count) * esz > r.bytes) throw std::invalid_argument("range outside the registered buffer");
  if ((off * esz) & 15) throw std::invalid_argument("in-place range must start 16-byte aligned");
  const int per = 16 / esz;
  IpArgs a{};
  for (int p = 0; p < world_; ++p) {
    a.data[p] = r.base[p] + off * esz;
    a.flags[p] = peer_ipflags_[p];
  }
  a.errc = ctrl_;
  a.err_host = err_dev_;
  a.n4 = count / per;
  a.tail = count - a.n4 * per;
  a.bytes = count * esz;
  a.timeout = timeout_ticks_;
  a.scale = scale;
  a.rank = rank_;
  // one-shot: U vectors per thread held across barrier B; U > 1 trades flag traffic (one barrier pair
  // per block) for a longer per-thread load chain
  const int64_t u_max = ip_vpt_;
  const int64_t one_shot_max_vec = (int64_t)kPeerMaxBlocks * kThreads * 4;
  bool two = algo == 2 || (algo == 0 && world_ > 2 && count * esz > one_shot_max_);
  if (!two && a.n4 > one_shot_max_vec) {
    if (algo == 1) throw std::invalid_argument("in-place one-shot holds at most 8 MB per call");
    two = true;
  }
  if (!two && a.n4 > (int64_t)ip_block_cap_ * kThreads * 4) two = true;   // shared-GPU grid cap (header)
  a.chunk4 = two ? (a.n4 + world_ - 1) / world_ : a.n4;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int64_t u = 1, nb;
  if (two) {
    // capped like the staged path (64 blocks by default): the two-shot is link-bound well below that,
    // and spinning blocks on every CU starve a peer's full-LDS kernels when ranks share a GPU (a
    // ResNet-18 DDP step deadlocked that way with 256 blocks)
    nb = (a.chunk4 + kThreads - 1) / kThreads;
    nb = nb < 1 ? 1 : (nb > max_blocks_ ? max_blocks_ : nb);
  } else {
    while (u < 4 && (u < u_max || a.n4 > (int64_t)ip_block_cap_ * kThreads * u)) u *= 2;
    nb = (a.n4 + kThreads * u - 1) / (kThreads * u);
    nb = nb < 1 ? 1 : nb;
  }
  if (esz == 4) ip_dispatch<F32Op>(world_, a, two, u, (int)nb, s);
  else ip_dispatch<BF16Op>(world_, a, two, u, (int)nb, s);
  hip_check(hipGetLastError(), "peer in-place all-reduce launch");
}

int64_t PeerAllReduce::error() {
  uint32_t v = 0;
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hip_check(hipMemcpy(&v, ctrl_ + 2, 4, hipMemcpyDeviceToHost), "hipMemcpy");
  return v;
}

int64_t PeerAllReduce::error_async() const {
  return err_host_ != nullptr ? (int64_t)*err_host_ : 0;
}

void PeerAllReduce::reset_error() {
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hip_check(hipMemset(ctrl_ + 2, 0, 4), "hipMemset");
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  if (err_host_ != nullptr) *err_host_ = 0;
}

}  // namespace pde
