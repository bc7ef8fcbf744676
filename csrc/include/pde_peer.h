// Shared layout of the xGMI peer all-reduce (csrc/runtime/peer_allreduce.{h,hip}) for code that
// runs the algorithm INSIDE another kernel (pde_peer_dev.h: e.g. the LeNet conv backward reduces
// the fc-gradient bucket in side blocks while its other blocks compute, with no extra launch and no
// cross-stream edge).  Host-safe: no HIP device code here.
#pragma once
#include <stdint.h>

namespace pde {

constexpr int kPeerMaxRanks = 8;
constexpr int kPeerMaxBlocks = 256;           // flag slots per phase (virtual blocks)
constexpr int64_t kPeerFlagBytes = 64 * 1024; // flags[2 phases][kPeerMaxBlocks][kPeerMaxRanks] u32

// Everything a device-side participant needs (POD, passed by value as a kernel argument).
// flags[p] / data[p]: rank p's flag region (uncached) and data region (stage0|stage1|res0|res1,
// `cap` bytes each), mapped into this process; ctrl: this rank's call counter / done counter /
// time-out count.  Produced by PeerAllReduce::device_args().
struct PeerDev {
  uint8_t* flags[kPeerMaxRanks];
  uint8_t* data[kPeerMaxRanks];
  uint32_t* ctrl;
  uint32_t* err_host;   // host-mapped time-out flag (PeerAllReduce::error_async)
  int64_t cap;
  int64_t timeout;   // s_memrealtime ticks (100 MHz)
  int32_t rank;
  int32_t world;
};

// The in-place (registered-buffer) protocol's view of one registration, for kernels that run the
// in-place one-shot all-reduce inside their own launch (the LeNet engine's fused conv-gradient fold +
// all-reduce): every rank's registered buffer and in-place flag region mapped here, the shared
// time-out latch, and the one-shot grid cap.  Produced by PeerAllReduce::registered_device_args(id).
// Flag slots and per-slot call counting are exactly peer_inplace_kernel's (peer_allreduce.hip), so
// fused and standalone in-place calls interleave freely.
struct PeerIpDev {
  uint8_t* data[kPeerMaxRanks];
  uint8_t* flags[kPeerMaxRanks];
  uint32_t* errc;       // the staged protocol's ctrl: [2] = time-out count (shared latch)
  uint32_t* err_host;
  int64_t bytes;        // registered bytes
  int64_t timeout;      // s_memrealtime ticks (100 MHz)
  int32_t rank;
  int32_t world;
  int32_t block_cap;    // in-place one-shot grid cap (ranks sharing one GPU)
  int32_t pad;
};

}  // namespace pde
