// Peer all-reduce: a latency-optimised all-reduce for SMALL buffers over xGMI peer memory.
//
// Why: the toy CNN's gradient buckets are 1.62 MB + 0.10 MB per step and a step
// is ~65 us, so the all-reduce is latency-bound.  A ring all-reduce over 8 GPUs does 14 dependent
// hops and drives one xGMI link per direction; here every GPU instead loads its peers' data straight
// out of their HBM over all 7 point-to-point xGMI links at once (hipIpc-mapped peer buffers), with
// one (one-shot) or two (two-shot) flag barriers per call:
//
//   one-shot  (small):  copy input -> own stage[par]  | barrier | out = sum_p stage_p[par]
//   two-shot  (large):  copy input -> own stage[par]  | barrier | res_self[par][my chunk] = sum_p stage_p[par][my chunk]
//                       | barrier | out[chunk q] = res_q[par][chunk q] for every q
//
// Each GPU moves (W-1)/W * bytes per phase in the two-shot form, spread evenly over the W-1 links.
// stage/res are double-buffered by call parity, which makes a trailing barrier unnecessary: a rank
// rewrites stage[par] two calls later, and it can only get there after every peer has passed the
// next call's first barrier, i.e. finished this call.  Barriers are per block index (block b of
// every rank owns the same slices), flags hold the monotonically increasing global call number.
// Flags live in uncached memory (hipDeviceMallocUncached: a spinning load always sees the peer's
// store).  stage/res are ordinary device memory by default: the signalling store is a system-scope
// release (L2 write-back of this XCD after every wave drained its stores) and the waiter does a
// system-scope acquire (L2 invalidate) before touching peer data, so no stale line is read on any
// of the 8 per-XCD L2s; ``uncached_data`` allocates them uncached instead (slower local traffic).
// Spins are bounded by a wall-clock timeout (s_memrealtime): a dead peer latches an error word
// instead of hanging the GPU.
//
// In-place form over REGISTERED buffers (the engines' persistent flat gradient buffers): every rank
// IPC-maps its peers' buffer once (register_buffer / open_registered), and a call reads the peers'
// gradients where the backward left them -- no stage copy, no fence:
//
//   one-shot:  barrier A | v = sum_p buf_p[i] (system-coherent loads) | barrier B | buf_self[i] = v
//   two-shot:  barrier A | buf_self[my chunk] = sum_p buf_p[my chunk] (write-through stores) | barrier B
//              | buf_self[chunk q] = buf_q[chunk q] for every q | barrier C
//
// Barrier A needs no release: the gradients were written by earlier kernels, whose end-of-kernel
// release already made them visible in memory; the peers' reads are system-scope loads (no stale L1 /
// L2 line), and the only bytes published inside the call (the two-shot partial sums) are written
// through with system-scope stores and drained (vmcnt(0)) before the flag store.  B keeps every rank
// from overwriting its buffer while a peer may still read it; C (two-shot) the same for the gathered
// chunks.  One-shot sums are held in registers across B: at most 256 blocks x 512 lanes x 16 B = 2 MB
// per call.
//
// Calls on one PeerAllReduce must be ordered on a single stream (the engine's comm stream) and be
// issued by every rank in the same order with the same sizes (collective semantics); launches are
// hipGraph-capturable (the call number lives in device memory).
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "pde_peer.h"

namespace pde {

class PeerAllReduce {
 public:
  PeerAllReduce(int rank, int world, int device, int64_t capacity_bytes, bool uncached_data = false);
  ~PeerAllReduce();
  // IPC handles (bytes: flags | data) of this rank's shared regions; exchanged through the store.
  std::string handle() const;
  // Map every peer's region (handles indexed by rank; this rank's own entry is ignored).
  void open(const std::vector<std::string>& handles);
  // out = sum over ranks of in (fp32), scaled by `scale`; in == out allowed. algo: 0 auto, 1 one-shot, 2 two-shot.
  void all_reduce_f32(uintptr_t in, uintptr_t out, int64_t count, float scale, int algo, uintptr_t stream);
  // bf16 variant (fp32 accumulation).
  void all_reduce_bf16(uintptr_t in, uintptr_t out, int64_t count, float scale, int algo, uintptr_t stream);
  int64_t capacity_bytes() const { return cap_; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  bool is_open() const { return opened_; }
  // 0 = healthy; otherwise the number of timed-out barrier waits since the last reset (synchronises).
  // Device-side view (flags/data of every rank, ctrl) for kernels that run the algorithm in side
  // blocks (pde_peer_dev.h); raw bytes of a PeerDev struct.
  std::string device_args() const;
  // The device-side protocol (pde_peer_dev.h) run as its own kernel, fp32: self-test of that path.
  void device_probe_f32(uintptr_t in, uintptr_t out, int64_t count, float scale, int two, uintptr_t stream);
  // Test hook: the next n host-kernel calls of this rank skip staging their input (peers then read
  // this rank's stage buffer as it was two calls ago): the self-test must catch it.
  void debug_skip_stage(int n) { debug_skip_stage_ = n; }
  int64_t error();
  // Host-mapped mirror of the time-out latch: non-zero once any barrier wait of this rank timed out.
  // A plain host load, no device synchronisation (a kernel still queued has not reported yet).
  int64_t error_async() const;
  void reset_error();
  void set_timeout_ms(int64_t ms) { timeout_ticks_ = ms * 100000; }   // s_memrealtime runs at 100 MHz
  void set_one_shot_max_bytes(int64_t b) { one_shot_max_ = b; }
  void set_max_blocks(int b) { max_blocks_ = b < 1 ? 1 : (b > kPeerMaxBlocks ? kPeerMaxBlocks : b); }
  // in-place one-shot grid cap: ranks time-sharing ONE GPU need every rank's spinning grid co-resident
  // (a grid that cannot be placed until another rank's spinning blocks exit deadlocks until the barrier
  // time-out), so dist/peer.py sets 256 / (ranks on this device) there; a call that does not fit runs
  // two-shot (same fixed rank order: bit-identical results)
  void set_ip_block_cap(int b) { ip_block_cap_ = b < 1 ? 1 : (b > kPeerMaxBlocks ? kPeerMaxBlocks : b); }
  // In-place registered form.  register_buffer returns the bytes (IPC handle of the allocation's base |
  // int64 offset of `ptr` in it) peers pass to open_registered; returns the registration id through
  // `id` (the same on every rank when every rank registers in the same order).
  std::string register_buffer(uintptr_t ptr, int64_t bytes, int* id);
  void open_registered(int id, const std::vector<std::string>& handles);
  // buf[off, off + count) of registration `id` = scale * sum over ranks, in place (elements of esz
  // bytes: 4 fp32, 2 bf16 with fp32 accumulation and one rounding).  algo: 1 one-shot (<= 8 MB),
  // 2 two-shot, 0 auto.
  void all_reduce_registered(int id, int64_t off, int64_t count, int esz, float scale, int algo, uintptr_t stream);
  void all_reduce_registered_f32(int id, int64_t off, int64_t count, float scale, int algo, uintptr_t stream);
  int64_t registered_bytes(int id) const;
  // Raw bytes of a PeerIpDev (pde_peer.h) for registration `id`: kernels that run the in-place one-shot
  // protocol in their own launch (csrc/kernels/lenet_v2.hip: k_conv_fold_ar).
  std::string registered_device_args(int id) const;
  void close();

 private:
  void launch(uintptr_t in, uintptr_t out, int64_t count, float scale, int algo, uintptr_t stream, bool bf16);
  int rank_, world_, device_;
  int64_t cap_;                 // bytes per stage / res buffer
  int64_t region_bytes_ = 0;
  bool uncached_data_ = false;
  uint8_t* flags_ = nullptr;    // own flag region (uncached)
  uint8_t* region_ = nullptr;   // own data region: stage0 | stage1 | res0 | res1
  uint32_t* ctrl_ = nullptr;    // local (not shared): [0] call counter, [1] done counter, [2] error count
  volatile uint32_t* err_host_ = nullptr;   // pinned host word: 1 once a barrier timed out (kernel-written)
  uint32_t* err_dev_ = nullptr;             // its device address
  uint8_t* peers_[kPeerMaxRanks] = {};
  uint8_t* peer_flags_[kPeerMaxRanks] = {};
  uint8_t* ipflags_ = nullptr;                  // own in-place flag region (uncached): [3][blocks][ranks] u32;
                                                // phase 0 slots count the calls (see peer_inplace_kernel)
  uint8_t* peer_ipflags_[kPeerMaxRanks] = {};
  int ip_vpt_ = 2;                              // one-shot vectors per thread (PDE_PEER_IP_VPT; 2 measured best)
  struct Reg {
    uint8_t* base[kPeerMaxRanks] = {};          // every rank's registered buffer, mapped here ([rank] = own)
    int64_t bytes = 0;
    bool open = false;
  };
  std::vector<Reg> regs_;
  // peer allocations opened for registrations, by (peer, IPC handle bytes): two registered buffers in
  // one peer allocation (one caching-allocator segment) share a single mapping, closed once
  std::map<std::pair<int, std::string>, uint8_t*> ipc_open_;
  bool opened_ = false;
  int64_t timeout_ticks_ = 10LL * 100000000;   // 10 s
  int64_t one_shot_max_ = 256 * 1024;
  int max_blocks_ = 64;
  int ip_block_cap_ = kPeerMaxBlocks;
  int debug_skip_stage_ = 0;
};

}  // namespace pde
