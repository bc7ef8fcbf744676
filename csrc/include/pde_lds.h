// LDS tile images, LDS-DMA staging and MFMA fragment reads shared by the bf16 MFMA kernels
// (conv.hip, attention.hip).  gfx950 only.
//
// Tile image: [rows][64 bf16] with 128-byte rows in 8-row groups of 1 KB, 16-byte chunks XOR-swizzled
// (cdna_hip_programming.md T10 layout (a)): conflict-free ds_read_b128 row reads of 32x32x16
// operands AND ds_read_b64_tr_b16 transposed reads of the same image.  Stages are filled by
// buffer_load ... lds (LDS-DMA): a wave-instruction writes 64 x 16 B lane-linearly into one 8-row
// group, so the swizzle goes into the per-lane SOURCE address (glds_row / glds_chunk).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pde_bf16.h"
#include "pde_hip.h"

namespace pde_lds {

typedef short s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v lds_s4v;

// Bounds-checked buffer loads: an offset past the resource's size returns zeros, so image padding
// and ragged tiles cost no branch around the load (cdna_hip_programming.md T8 / §5.5 trap (c)).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kOOB = 0x80000000u;
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 bload16(rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// byte offset of 16-byte chunk `ch` (0..7) of row `row` in a [rows][64 bf16] image
__device__ __forceinline__ int toff(int row, int ch) {
  return 1024 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}
__device__ __forceinline__ bf16x8 row_frag(const char* img, int row, int ch) {
  return *reinterpret_cast<const bf16x8*>(img + toff(row, ch));
}
// Transposed reads (ds_read_b64_tr_b16) are issued as inline asm in loops with LDS-DMA in flight:
// hipcc puts a blanket `s_waitcnt vmcnt(0)` before every ds_read_b64_tr_b16 BUILTIN there (no
// memory operand to prove it does not alias the DMA), which drains the prefetched stages.  The asm
// form is not tracked: the caller waits with `lgkm_fence()` before using the fragments.
typedef __attribute__((address_space(3))) char lds_char;
// wait for this wave's outstanding LDS reads; the sched_barrier keeps the MFMAs that consume
// asm-loaded fragments from being hoisted above the wait (cdna_hip_programming.md §5.4 rule 18)
__device__ __forceinline__ void lgkm_fence() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// 16-byte buffer load straight into LDS (LDS-DMA): lane l of the wave writes lds + 16*l, the LDS
// base must be wave-uniform; a global offset past the resource returns zeros.
__device__ __forceinline__ void glds16(rsrc_t r, const char* lds, uint32_t off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, off, 0, 0, 0);
}
// The lane -> (row, chunk) map that makes a glds wave-instruction (64 x 16 B, lane-linear in LDS)
// fill one 8-row group of the toff() image: lane l writes 8-row group offset 16*l, i.e. row
// (l>>2)&7 of the group and the chunk whose swizzled slot that is (g1 = parity of the group index).
__device__ __forceinline__ int glds_row(int l) { return (l >> 2) & 7; }
__device__ __forceinline__ int glds_chunk(int l, int g1) {
  return 4 * (l >> 5) + ((l & 3) ^ ((((l >> 2) & 7) >> 2) | (g1 << 1)));
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Transposed-read fragment pair at a compile-time offset from two per-wave base addresses (the rows
// 4h+q and 8+4h+q of a k-step sit in differently swizzled slots, hence two bases): every
// ds_read_b64_tr_b16 of a wgrad stage is base + immediate (k-step 2048*S, fragment column half 512),
// so the K loop spends no VALU on LDS addresses.
template <int OFF>
__device__ __forceinline__ bf16x8 trpair(uint2 a) {
  s4v v0, v1;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v0) : "v"(a.x), "n"(OFF));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v1) : "v"(a.y), "n"(OFF));
  bf16x8 out;
  out[0] = v0[0]; out[1] = v0[1]; out[2] = v0[2]; out[3] = v0[3];
  out[4] = v1[0]; out[5] = v1[1]; out[6] = v1[2]; out[7] = v1[3];
  return out;
}
// byte offset of fragment column block x (32 columns each) inside a stage's 64-column images
__host__ __device__ constexpr int colblk_off(int x) { return (x >> 1) * 8192 + (x & 1) * 512; }
// lane part of the two transposed reads (column 0 of an image, rows 4h+q / 8+4h+q of k-step 0,
// 8-B half p&1)
__device__ __forceinline__ uint2 tr_lane_off() {
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, h = g >> 1;
  const int ch = 2 * (g & 1) + (p >> 1);
  return make_uint2(toff(4 * h + q, ch) + 8 * (p & 1), toff(8 + 4 * h + q, ch) + 8 * (p & 1));
}
__device__ __forceinline__ uint2 add2(uint2 a, uint32_t b) { return make_uint2(a.x + b, a.y + b); }
}  // namespace pde_lds
