// Shared device helpers of the hand-written MFMA GEMMs (gemm.hip: K-major x K-major weight
// gradients; gemm_nt.hip: forward / dgrad with fused epilogues).  gfx950 only.
#pragma once
#include "common.h"

#pragma clang diagnostic ignored "-Winline-asm"  // m0 is clobbered on purpose (dma16)

namespace mx {
namespace gemm {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __attribute__((address_space(3))) bf16x8 lds_bf16x8;

// K-major image ([k][n] rows of >= 256 B): the 16-B chunks of k-row k are XOR-swizzled by
// (k & 3, k >> 3 & 1) so the 16 row segments of one transposed read spread over all 8 32-B
// slots of a bank row
__device__ __forceinline__ int gsw(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }
// physical 16-B chunk of logical chunk c in k-row k (an involution: also logical <- physical)
__device__ __forceinline__ int pchunk(int k, int c) { return (((c >> 1) ^ gsw(k)) << 1) | (c & 1); }

__device__ __forceinline__ bf16x4 tr_read(const char* lds, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(lds + byte_off));
}
__device__ __forceinline__ bf16x8 lds_read8(const char* lds, int byte_off) {
  return *(const lds_bf16x8*)(lds + byte_off);
}
__device__ __forceinline__ bf16x8 cat(bf16x4 a, bf16x4 b) {
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
// one 1-KiB LDS-DMA piece: lane i's 16 B from `g` land at lds_base + 16 i.  Issued from
// inline asm on purpose: for the builtin, the compiler's wait-count pass cannot prove that a
// later ds_read of ANOTHER ring slot does not alias the in-flight DMA (the accesses carry no
// alias-scope info) and drains the whole queue (vmcnt(0)) before the first read of every
// K-step, which serialises load and compute; the kernels order DMA and reads themselves with
// counted vmcnt waits + barriers.  M0 = LDS base; one wait state between the M0 write and
// the DMA.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const lds_void_t*)p;
}
__device__ __forceinline__ void dma16(const void* g, uint32_t lds_base) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :: "v"(g), "s"(lds_base) : "memory", "m0");
}
// The same piece addressed as a 32-bit byte offset from a wave-uniform base (saddr form): the
// per-lane address math stays 32-bit (no 64-bit adds / multiplies per piece).
__device__ __forceinline__ void dma16_sbase(const void* sbase, uint32_t voff, uint32_t lds_base) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(voff), "s"(sbase), "s"(lds_base) : "memory", "m0");
}
// Buffer-resource form: a byte offset >= the resource's size reads zeros (padding rows of an
// implicit-GEMM gather without a select between two 64-bit addresses).  Raw buffer, stride 0.
typedef int i32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4_t buffer_rsrc(const void* base, uint32_t bytes) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  return i32x4_t{(int)(uint32_t)b, (int)(uint32_t)(b >> 32), (int)bytes, 0x00020000};
}
constexpr uint32_t kOOB = 0x80000000u;   // out-of-range offset (resources stay < 2 GiB)
__device__ __forceinline__ void dma16_buf(i32x4_t rsrc, uint32_t voff, uint32_t lds_base) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :: "v"(voff), "s"(rsrc), "s"(lds_base) : "memory", "m0");
}
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}

// Epilogue re-deal of two 16-column MFMA subtiles: (x0, x1) = lane's 4 columns 4G..4G+3
// of subtile u0 (bf16 pairs), (y0, y1) the same of u1.  permlane32_swap exchanges the
// upper half of x with the lower half of y, permlane16_swap the odd 16-lane rows of x with
// the even rows of y; afterwards lane group G holds the 8 consecutive columns 8G .. 8G + 7
// of the 32-column pair as (x0, x1, y0, y1).  undeal is the inverse (each swap is an
// involution, applied in reverse order).
__device__ __forceinline__ void swap32(uint32_t& x, uint32_t& y) {
  auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}
__device__ __forceinline__ void swap16(uint32_t& x, uint32_t& y) {
  auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}
__device__ __forceinline__ void deal(uint32_t& x0, uint32_t& x1, uint32_t& y0, uint32_t& y1) {
  swap32(x0, y0);
  swap32(x1, y1);
  swap16(x0, y0);
  swap16(x1, y1);
}
__device__ __forceinline__ void undeal(uint32_t& x0, uint32_t& x1, uint32_t& y0, uint32_t& y1) {
  swap16(x0, y0);
  swap16(x1, y1);
  swap32(x0, y0);
  swap32(x1, y1);
}

}  // namespace gemm
}  // namespace mx
