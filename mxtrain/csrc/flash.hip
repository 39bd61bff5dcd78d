// Flash attention v3 for gfx950 (CDNA4): forward, atomics-free backward, attention dropout.
//
// Replaces the Megatron fused `scaled_upper_triang_masked_softmax` + two batched GEMMs +
// attention dropout (GPT, causal) and the HF BERT padded-softmax attention + dropout the
// reference runs upstream (containers/megatron-deepspeed/Dockerfile:13, examples/
// megatron-deepspeed/gpt2_345m/pretrain-ddp-zero1.yaml:39-53 -- Megatron's default
// --attention-dropout 0.1 --; examples/accelerate/bert-glue-mrpc/pretrain.yaml:45;
// SURVEY §2.8 K1/K2).  No S x S matrix is materialised.
//
// Layout: Q/K/V are read in place from the packed QKV projection output ([tokens, heads, D]
// with a token stride), O / dQ / dK / dV are written token-major, so the model needs no
// transposes.  lse is base-2: lse2 = max*c + log2(sum), c = scale*log2(e).
//
// Three kernels, 4-wave workgroups (two per CU = 2 waves per SIMD), one barrier per tile.
// One 128-row block per workgroup: every wave is busy on every tile it waits for (a
// mirrored causal pair in one workgroup left half of the waves idle for most tiles), the two
// workgroups of a CU hide each other's barriers, and under a causal mask the heaviest blocks
// are dispatched first so the hardware dispatcher balances the tail; the blocks of one head
// are dealt to one XCD, so its K/V (or Q/dO) stream is shared in that XCD's L2.
//   qmajor<FWD>  each wave owns 32 query rows (query on the MFMA lane: S^T = K Q^T,
//                O^T = V^T P^T, the row statistics are lane-local plus one permlane32 swap).  K/V tiles of 128 keys arrive by LDS-DMA
//                (global_load_lds_dwordx4: no staging registers, no ds_write) into a two-slot
//                ring; the swizzle is applied on the SOURCE addresses so the 1-KiB DMA pieces
//                land in the conflict-free image the row reads (ds_read_b128) and transposed
//                reads (ds_read_b64_tr_b16) both use.
//   qmajor<DQ>   same skeleton for dQ: recomputes S^T and dP^T = V dO^T per 32-key subtile,
//                dS^T = P^T (dP^T - delta) -> dQ^T += K^T dS^T (K^T by transposed LDS reads).
//                delta = rowsum(dO O) is computed in the prologue (no pre-pass kernel) and
//                published for kmajor; dQ is written once in bf16 (no fp32 accumulator, no
//                atomics, no convert kernel).
//   kmajor       each wave keeps dK^T / dV^T of its 32 keys in accumulators (key on the lane: P and dS are
//                ready-made B operands) while Q / dO / lse / delta tiles of 64 rows stream
//                through an LDS-DMA ring (32 rows for D = 128).
//   kmajor128    D = 128 in one pass: 8 waves, two per 32 keys -- one computes S -> P, its
//                partner dP -> dP - delta, the halves are swapped through LDS and each wave
//                accumulates half of the dK/dV columns (the accumulators of all 128 columns
//                do not fit two waves per SIMD; the earlier two column-half passes recomputed
//                S and dP twice: 323 -> 275 us at GPT-3 shapes).
// The 5-GEMM single backward would need dQ summed across key blocks: with fp32 atomics that
// is bounded by the ~1.3 TB/s chip atomic rate (MI355X_MICROARCH.md "Global float atomics"),
// 33 MB / 26 us per GPT-2 layer; the recompute costs 1.4x the MFMA work but no atomics.
//
// Attention dropout: keep-mask M[b,h,q,k] is a pure function of (seed, global row, key):
// per (row, 32-key block, lane half) one hash32 seeds an xorshift32 stream whose 16-bit
// halves are the draws (drop_stream_bits; keep <=> draw >= thr16), row = (b * Hg + h_global)
// * S + q (16-bit threshold: p exact to 2^-16; ops/attention.py::dropout_keep_mask is the
// reference).
// flash_dropmask_kernel evaluates it once per forward (on a side stream, concurrent with the
// QKV GEMM) into two lane-bit images laid out so that each packed bf16 pair is masked with
// three VALU ops (shift, v_pk_ashrrev_i16, and): 16 bits per lane per 32x32 block, element
// 2j at bit sh+j and 2j+1 at bit sh+16+j of a 32-bit word holding two blocks (sh = 0 / 8).
#include "common.h"

#include <type_traits>

#pragma clang diagnostic ignored "-Winline-asm"  // m0 is clobbered on purpose (dma16 / dma4)

using namespace mx;

namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef short short2_t __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------------------ helpers
// Chunk swizzle for a [rows][D] bf16 tile (D*2-byte rows, 16-B chunks).
//  D=64 (128-B rows, two rows per 256-B bank row): f = x ^ ((x&1)<<2), x = (row>>1)&7
//  D=128 (256-B rows): f = ((row&3)<<2) | ((row>>2)&3)
// Both keep the row reads (ds_read_b128, 32 rows) and the transposed reads (4 consecutive
// rows x 32 columns per half-wave) conflict-free; f depends on row bits 0-3 only, so a
// 32-row step is an immediate offset.
template <int D>
__device__ __forceinline__ int swz(int row) {
  if constexpr (D == 64) {
    int x = (row >> 1) & 7;
    return x ^ ((x & 1) << 2);
  } else {
    return ((row & 3) << 2) | ((row >> 2) & 3);
  }
}
template <int D>
__device__ __forceinline__ int toff(int row, int chunk) {
  return row * (D * 2) + ((chunk ^ swz<D>(row)) << 4);
}
__device__ __forceinline__ bf16x4 tr_read(const char* lds, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(lds + byte_off));
}
__device__ __forceinline__ bf16x8 cat(bf16x4 a, bf16x4 b) {
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
__device__ __forceinline__ bf16x8 ld8(const uint16_t* p) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p));
}
__device__ __forceinline__ bf16x8 lds8(const char* base, int off) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(base + off));
}
__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int crow(int e, int hh) { return (e & 3) + 8 * (e >> 2) + 4 * hh; }
// sum over the 32 lanes of the caller's half-wave (every lane gets it): 16-lane row sum by
// DPP, then the two rows of the half through v_permlane16_swap
__device__ __forceinline__ float half_sum(float v) {
  v += MX_DPP(v, 0xB1);
  v += MX_DPP(v, 0x4E);
  v += MX_DPP(v, 0x124);
  v += MX_DPP(v, 0x128);
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// Bias-gradient column partials of a 32-row MFMA output block (QKV bias = column sums of
// dQ / dK / dV): acc[dt][e] holds column 32 dt + crow(e, hh) of the lane's row; the 32 rows
// of a half-wave are summed and lanes 0 / 32 store them (fp32, unrounded) into partial row
// `prow` at column col0 + d.  The caller guarantees all 32 rows exist (S % 32 == 0).
template <int N>
__device__ __forceinline__ void bias_partial_store(const f32x16 (&acc)[N], float sc, float* __restrict__ bp,
                                                   int ldbp, int prow, int col0, int dt0, int lane) {
  const int hh = lane >> 5;
  float* row = bp + (size_t)prow * ldbp + col0;
#pragma unroll
  for (int dt = 0; dt < N; ++dt) {
    float sums[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) sums[e] = half_sum(acc[dt][e] * sc);
    if ((lane & 31) == 0) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        *reinterpret_cast<float4*>(row + 32 * (dt + dt0) + 8 * g4 + 4 * hh) =
            make_float4(sums[4 * g4], sums[4 * g4 + 1], sums[4 * g4 + 2], sums[4 * g4 + 3]);
    }
  }
}
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

// One 32-column group of a row-per-lane 32x32 MFMA result (lane r and r + 32 hold row r:
// columns 8 k + 4 hh .. +3 of each group k) stored as bf16 with 16-B stores: for each pair of
// groups (k, k + 1) one v_permlane32_swap per dword gives the lower half-wave columns
// 8 k .. 8 k + 7 and the upper one 8 k + 8 .. 8 k + 15 -- 2 dwordx4 stores per lane instead of
// 4 dwordx2 (the epilogue store tail is issue-bound: MI355X guide T21).  Both lanes of a row
// must be active.
__device__ __forceinline__ void store_row32(uint16_t* rowp, const f32x16& acc, float sc, int hh) {
#pragma unroll
  for (int k = 0; k < 4; k += 2) {
    const uint32_t ax = pack2(acc[4 * k + 0] * sc, acc[4 * k + 1] * sc);
    const uint32_t ay = pack2(acc[4 * k + 2] * sc, acc[4 * k + 3] * sc);
    const uint32_t bx = pack2(acc[4 * k + 4] * sc, acc[4 * k + 5] * sc);
    const uint32_t by = pack2(acc[4 * k + 6] * sc, acc[4 * k + 7] * sc);
    const auto rx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
    const auto ry = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
    *reinterpret_cast<uint4*>(rowp + 8 * k + 8 * hh) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
  }
}

// one 1-KiB LDS-DMA piece: lane i's 16 B from `g` land at lds_base + 16 i.  Issued from
// inline asm: for the builtin, the compiler cannot prove that a later ds_read of another
// ring slot does not alias the in-flight DMA (no alias-scope info on either access) and
// waits vmcnt(0) before the first LDS read after every issue -- the next tile's DMA was
// drained before the current tile's first MFMA, serialising load and compute.  The kernels
// order DMA and reads themselves (vm_drain + barrier at the top of every tile).  M0 = LDS
// base (wave-uniform); one wait state between the M0 write and the DMA.
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const lds_void_t*)p);
}
__device__ __forceinline__ void dma16(const void* g, char* lds_base) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :: "v"(g), "s"(lds_u32(lds_base)) : "memory", "m0");
}
__device__ __forceinline__ void dma4(const void* g, char* lds_base) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off"
               :: "v"(g), "s"(lds_u32(lds_base)) : "memory", "m0");
}
// vmcnt(0) through the builtin (expcnt / lgkmcnt fields at their "no wait" maxima), not asm:
// the waitcnt pass then knows every compiler-visible load (e.g. the dropout words of the
// previous step) is complete, instead of re-waiting for them mid-tile with a vmcnt(N) that
// the hardware also applies to the asm-issued DMA of the next tile.
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// dropout: all-ones halves for the kept elements of packed pair j (elements 2j, 2j+1)
__device__ __forceinline__ uint32_t pair_keep(uint32_t w, int sh, int j) {
  short2_t v = __builtin_bit_cast(short2_t, w << (15 - sh - j));
  v = v >> (short2_t){15, 15};
  return __builtin_bit_cast(uint32_t, v);
}
// all-ones if element e is kept
__device__ __forceinline__ uint32_t elem_keep(uint32_t w, int sh, int e) {
  return (uint32_t)__builtin_amdgcn_sbfe((int)w, (uint32_t)(sh + 16 * (e & 1) + (e >> 1)), 1u);
}
__device__ __forceinline__ bf16x8 pack8(const f32x16& acc, int base) {
  uint4 u;
  u.x = pack2(acc[base + 0], acc[base + 1]);
  u.y = pack2(acc[base + 2], acc[base + 3]);
  u.z = pack2(acc[base + 4], acc[base + 5]);
  u.w = pack2(acc[base + 6], acc[base + 7]);
  return __builtin_bit_cast(bf16x8, u);
}
__device__ __forceinline__ bf16x8 pack8_keep(const f32x16& acc, int base, uint32_t w, int sh) {
  const int j0 = base >> 1;
  uint4 u;
  u.x = pack2(acc[base + 0], acc[base + 1]) & pair_keep(w, sh, j0 + 0);
  u.y = pack2(acc[base + 2], acc[base + 3]) & pair_keep(w, sh, j0 + 1);
  u.z = pack2(acc[base + 4], acc[base + 5]) & pair_keep(w, sh, j0 + 2);
  u.w = pack2(acc[base + 6], acc[base + 7]) & pair_keep(w, sh, j0 + 3);
  return __builtin_bit_cast(bf16x8, u);
}

// workgroup id -> (block rank, head): block ranks in dispatch order (rank 0 first, so the
// caller maps rank 0 to the heaviest causal block), and, when the head count is a multiple
// of 8, every block of a head on one XCD (workgroups are dealt round-robin over the 8 XCDs,
// id % 8): its K/V (Q/dO) stream is then read once into that XCD's L2.
__device__ __forceinline__ void block_map(int nheads, int& rank, int& head) {
  const int L = blockIdx.x;
  if ((nheads & 7) == 0) {
    const int x = L & 7, idx = L >> 3, nh8 = nheads >> 3;
    rank = idx / nh8;
    head = (idx - rank * nh8) * 8 + x;
  } else {
    rank = L / nheads;
    head = L - rank * nheads;
  }
}

// ============================================================================ dropout mask
// The random bits of one (query row, 32-key block, lane half hh) -- the 16 keys
// crow(e, hh) of a lane -- come from ONE hash and an xorshift32 stream: x0 = hash32(row *
// 0x85EBCA6B + 2 kb + hh, seed) (| 1: never the all-zero fixed point), x_{j+1} = xorshift(x_j);
// x_j holds the 16-bit draws of the lane's pair j (elements 2j, 2j+1 = keys crow(2j, hh) and
// +1) in its low / high half.  Returns the lane's 16 keep bits in pair layout: element 2j at
// bit j, 2j+1 at bit 8 + j -- so a 32-bit word of two blocks holds (sh = 0 / 8) element 2j
// at sh + j and 2j+1 at sh + 16 + j after the second block is shifted in by 8.
__device__ __forceinline__ uint32_t drop_stream_bits(uint32_t rbase, uint32_t kb, int hh,
                                                     uint32_t seed, uint32_t thr16) {
  uint32_t x = hash32(rbase + 2u * kb + (uint32_t)hh, seed) | 1u;
  // both 16-bit draws of x at once: sat(x - (thr-1)) is non-zero iff draw >= thr, min(., 1)
  // leaves the keep bit at bit 0 / 16 (v_pk_sub_u16 clamp + v_pk_min_u16), then shift-or
  // (thr16 == 0: thr2 = 0xFFFF'FFFF subtracts to 0 only for 0xFFFF draws -- p = 0 never
  // reaches here, the host only generates masks for p > 0)
  const uint32_t thr2 = ((thr16 - 1) & 0xFFFFu) * 0x00010001u;
  const uint32_t one2 = 0x00010001u;
  uint32_t bits = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (j) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; }
    uint32_t t;
    asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(t) : "v"(x), "v"(thr2));
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(t) : "v"(t), "v"(one2));
    bits |= t << j;
  }
  return bits;
}

// One wave per 64x64 group (query blocks 2qb2, 2qb2+1 x key blocks 2kb2, 2kb2+1).
// fwd image (query on lane): u64 [B*Hq][NB][NKT][64 lanes], 16 bits per 32-key subtile,
//   subtile t of a 128-key tile in word t>>1 at sh = 8 (t & 1).
// bwd image (key on lane):   u32 [B*Hq][NB][NQT][64 lanes], 16 bits per 32-query half of a
//   64-query tile at sh = 8 u.
// blockIdx.z = layer * BH + bh: the images of several layers (salt + layer, images at
// layer * stride) in one launch -- every layer's masks of a step depend only on the seed, so
// the model generates them all up front (one launch instead of one per layer).
__global__ __launch_bounds__(256) void flash_dropmask_kernel(
    const uint32_t* __restrict__ seed_ptr, uint32_t salt, uint32_t thr16, int S, int Hq,
    int h_off, int Hg, int NB, int NKT, int NQT, int causal, uint32_t* __restrict__ fwd_bits,
    uint32_t* __restrict__ bwd_bits, int BH, long long fwd_stride, long long bwd_stride) {
  const int lane = threadIdx.x & 63, w = uni(threadIdx.x >> 6);
  const int layer = blockIdx.z / BH;
  const int qb2 = blockIdx.x, kb2 = blockIdx.y * 4 + w, bh = blockIdx.z - layer * BH;
  salt += (uint32_t)layer;
  fwd_bits += (size_t)layer * fwd_stride;
  bwd_bits += (size_t)layer * bwd_stride;
  const int NB2 = (NB + 1) >> 1;
  __shared__ uint32_t fw[4][2][64];
  const bool live = kb2 < NB2 && !(causal && kb2 > qb2);
  const int b = bh / Hq, h = bh - b * Hq;
  const int r = lane & 31, hh = lane >> 5;
  if (live) {
    const uint32_t seed = *seed_ptr + salt;
    uint32_t fb[2][2];
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      const uint32_t row = (uint32_t)(((long long)b * Hg + h_off + h) * S + (2 * qb2 + qq) * 32 + r);
      const uint32_t rbase = row * 0x85EBCA6Bu;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        fb[qq][kk] = drop_stream_bits(rbase, (uint32_t)(2 * kb2 + kk), hh, seed, thr16);
      // forward word of query block 2 qb2 + qq: key blocks 2 kb2 (sh 0) and 2 kb2 + 1 (sh 8)
      const int qb = 2 * qb2 + qq;
      if (qb < NB)
        fwd_bits[(((size_t)bh * NB + qb) * NKT + (kb2 >> 1)) * 128 + lane * 2 + (kb2 & 1)] =
            fb[qq][0] | (fb[qq][1] << 8);
      fw[w][qq][lane] = fb[qq][0] | (fb[qq][1] << 8);
    }
  }
  __syncthreads();
  if (!live) return;
  // backward image: lane = key kl of key block 2 kb2 + kk; element e -> query crow(e, hh) of
  // query block 2 qb2 + u, read from forward lane crow(e, hh) + 32 ((kl >> 2) & 1), whose
  // element ef = (kl & 3) + 4 (kl >> 3) sits at bit 8 kk + 16 (ef & 1) + (ef >> 1)
  const int kl = r;
  const int ef = (kl & 3) + 4 * (kl >> 3), fhi = 32 * ((kl >> 2) & 1);
  const int fpos = 16 * (ef & 1) + (ef >> 1);
  uint32_t wb[2] = {0u, 0u};
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const uint32_t src = fw[w][u][crow(e, hh) + fhi];
      const int pos = 8 * u + 16 * (e & 1) + (e >> 1);
      wb[0] |= __builtin_amdgcn_ubfe(src, (uint32_t)fpos, 1u) << pos;
      wb[1] |= __builtin_amdgcn_ubfe(src, (uint32_t)(8 + fpos), 1u) << pos;
    }
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int kb = 2 * kb2 + kk;
    if (kb < NB) bwd_bits[(((size_t)bh * NB + kb) * NQT + qb2) * 64 + lane] = wb[kk];
  }
}

// The same images from a fixed grid of waves that walk the LIVE 64x64 groups of every
// (layer, batch x head) -- a causal mask has NB2 (NB2 + 1) / 2 of NB2^2 -- instead of one
// 4-wave workgroup per (query group, 4 key groups, layer x head): that grid launched ~98k
// workgroups per GPT-2 step, half of them dead above the diagonal, each running ~600
// instructions -- dispatch-bound at ~3x the VALU time of the hashing (312 us per step,
// profiles/r4_s1/gpt2_kernel_table.txt).  Bit-identical images: the same per-group code.
__global__ __launch_bounds__(256) void flash_dropmask_waves_kernel(
    const uint32_t* __restrict__ seed_ptr, uint32_t salt0, uint32_t thr16, int S, int Hq,
    int h_off, int Hg, int NB, int NKT, int NQT, int causal, uint32_t* __restrict__ fwd_bits0,
    uint32_t* __restrict__ bwd_bits0, int BH, int L, long long fwd_stride, long long bwd_stride) {
  const int lane = threadIdx.x & 63, w = uni(threadIdx.x >> 6);
  __shared__ uint32_t fwl[4][2][64];
  const int NB2 = (NB + 1) >> 1;
  const int per = causal ? NB2 * (NB2 + 1) / 2 : NB2 * NB2;   // live groups per (layer, bh)
  const long long total = (long long)L * BH * per;
  const int r = lane & 31, hh = lane >> 5;
  const uint32_t seed0 = *seed_ptr;
  // bwd-image gather constants (see flash_dropmask_kernel)
  const int kl = r;
  const int ef = (kl & 3) + 4 * (kl >> 3), fhi = 32 * ((kl >> 2) & 1);
  const int fpos = 16 * (ef & 1) + (ef >> 1);
  for (long long it = (long long)blockIdx.x * 4 + w; it < total; it += (long long)gridDim.x * 4) {
    const int z = uni((int)(it / per));
    const int pi = uni((int)(it - (long long)z * per));
    int qb2, kb2;
    if (causal) {   // row qb2 of the lower triangle holds qb2 + 1 groups
      int q = (int)((sqrtf(8.f * (float)pi + 1.f) - 1.f) * 0.5f);
      while ((q + 1) * (q + 2) / 2 <= pi) ++q;
      while (q * (q + 1) / 2 > pi) --q;
      qb2 = uni(q);
      kb2 = uni(pi - q * (q + 1) / 2);
    } else {
      qb2 = uni(pi / NB2);
      kb2 = uni(pi - (pi / NB2) * NB2);
    }
    const int layer = z / BH, bh = z - layer * BH;
    uint32_t* fwd_bits = fwd_bits0 + (size_t)layer * fwd_stride;
    uint32_t* bwd_bits = bwd_bits0 + (size_t)layer * bwd_stride;
    const uint32_t seed = seed0 + salt0 + (uint32_t)layer;
    const int b = bh / Hq, h = bh - b * Hq;
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      const uint32_t row = (uint32_t)(((long long)b * Hg + h_off + h) * S + (2 * qb2 + qq) * 32 + r);
      const uint32_t rbase = row * 0x85EBCA6Bu;
      uint32_t fb0 = drop_stream_bits(rbase, (uint32_t)(2 * kb2), hh, seed, thr16);
      uint32_t fb1 = drop_stream_bits(rbase, (uint32_t)(2 * kb2 + 1), hh, seed, thr16);
      const int qb = 2 * qb2 + qq;
      const uint32_t word = fb0 | (fb1 << 8);
      if (qb < NB) fwd_bits[(((size_t)bh * NB + qb) * NKT + (kb2 >> 1)) * 128 + lane * 2 + (kb2 & 1)] = word;
      fwl[w][qq][lane] = word;
    }
    __builtin_amdgcn_wave_barrier();   // (LDS ops of one wave run in order; keep the compiler's too)
    uint32_t wb[2] = {0u, 0u};
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const uint32_t src = fwl[w][u][crow(e, hh) + fhi];
        const int pos = 8 * u + 16 * (e & 1) + (e >> 1);
        wb[0] |= __builtin_amdgcn_ubfe(src, (uint32_t)fpos, 1u) << pos;
        wb[1] |= __builtin_amdgcn_ubfe(src, (uint32_t)(8 + fpos), 1u) << pos;
      }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int kb = 2 * kb2 + kk;
      if (kb < NB) bwd_bits[(((size_t)bh * NB + kb) * NQT + qb2) * 64 + lane] = wb[kk];
    }
    __builtin_amdgcn_wave_barrier();   // this group's reads before the next group's writes
  }
}

// ============================================================================ query-major
// DQ false: forward (o, lse out).  DQ true: dQ (o, dout, lse in; delta, dq out).
//
// PAIR (D = 64): one 8-wave workgroup = two 4-wave teams with a K/V ring each.  Causal: the
// mirrored block pair (L = i, H = n-1-i) holds n+1 key tiles of work; team 0 takes H's first
// T = ceil(total/2) tiles, team 1 takes all of L and H's remaining tiles, so both teams run
// T steps (one shared barrier per step) and every workgroup does the same work.  Team 1
// hands its partial (m, l, O^T) -- or dQ^T -- of H to team 0 through LDS at the end (same
// lane <-> (row, column) mapping in both teams: an element-wise merge).  Non-causal: team
// t takes block 2i+t whole.  The critical path is ~half the heaviest block's tiles.
// !PAIR (D = 128): one 4-wave workgroup per block (two per CU), heaviest block first.

// In-kernel keep bits (DGEN, forward only; the measured alternative to the mask pre-pass,
// profiles/r6/attn_inkernel_dropout_ab.txt): every wave hashes its own 32 rows x 128 keys per
// tile with drop_stream_bits, bit-identical to the pre-pass images.
struct DGen {
  const uint32_t* seed;
  uint32_t salt, thr16;
  int hoff, hg;
};

template <int D, bool CAUSAL, bool DROP, bool DQ, bool PAIR, int BKT = 64, bool DGEN = false>
__global__ __launch_bounds__(PAIR ? 512 : 256) __attribute__((amdgpu_waves_per_eu(2, 2))) void flash_qmajor_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, int ldq, int ldk, int ldv,
    const uint16_t* __restrict__ dout, int lddo, uint16_t* __restrict__ o, int ldo,
    float* __restrict__ lse, float* __restrict__ delta, uint16_t* __restrict__ dq, int lddq,
    int S, int Hq, int Hkv, const int* __restrict__ klen, float c,
    float oscale /* FWD 1/(1-p); DQ scale/(1-p) */, float dkeep /* 1-p */,
    const uint64_t* __restrict__ dbits, int NB, int NKT, float* __restrict__ bpart, int ldbp, DGen dg) {
  constexpr int BQ = 128, BK = BKT, NSUB = BK / 32, NKK = D / 16, NDT = D / 32;
  constexpr int RB = D * 2, CPR = D / 8, RPP = 64 / CPR;
  constexpr int TILE = BK * RB, PIECES = TILE / 1024, PPW = PIECES / 4;
  constexpr int T2 = PAIR ? TILE : 16;
  constexpr int NREG = NDT * 16 + 2;                       // merged registers per lane
  constexpr int MRG = PAIR ? 4 * NREG * 64 : 4;
  __shared__ __attribute__((aligned(16))) char k0[TILE];
  __shared__ __attribute__((aligned(16))) char k1[TILE];
  __shared__ __attribute__((aligned(16))) char v0[TILE];
  __shared__ __attribute__((aligned(16))) char v1[TILE];
  // team 1's tiles; the end-of-loop merge area aliases them (written after a barrier that
  // team 1 reaches only once its last tile is consumed): 4 x 16 KB tiles at BK 128 + the
  // 34 KB merge area would not fit next to team 0's 64 KB otherwise
  constexpr int T1B = 4 * T2 > MRG * 4 ? 4 * T2 : MRG * 4;
  __shared__ __attribute__((aligned(16))) char t1buf[T1B];
  char* const k2 = t1buf;
  char* const k3 = t1buf + T2;
  char* const v2 = t1buf + 2 * T2;
  char* const v3 = t1buf + 3 * T2;
  float* const mrg = reinterpret_cast<float*>(t1buf);

  const int tid = threadIdx.x, lane = tid & 63, w = uni(tid >> 6);
  const int team = PAIR ? (w >> 2) : 0, wl = w & 3;
  const int r = lane & 31, hh = lane >> 5, g = lane >> 4, gi = lane & 15;
  const int nqb = (S + BQ - 1) / BQ;
  const int nunits = PAIR ? (nqb + 1) / 2 : nqb;
  int rank, head;
  block_map((int)gridDim.x / nunits, rank, head);   // grid = nunits x (B * Hq)
  const int hq = head % Hq, b = head / Hq;
  const int hk = hq / (Hq / Hkv);
  const int kl = klen ? klen[b] : S;
  auto ntiles = [&](int qb_) __attribute__((always_inline)) {
    const int lim = CAUSAL ? min(kl, min(S, (qb_ + 1) * BQ)) : kl;
    return (lim + BK - 1) / BK;
  };
  // ---- schedule: this team's items (block, key tile) for steps 0..T-1
  int blk0, cnt, sw = 1 << 30, blk1 = -1, t1 = 0, T;
  bool merge = false;
  if (!PAIR) {
    blk0 = CAUSAL ? nqb - 1 - rank : rank;          // causal: heaviest block first
    cnt = T = ntiles(blk0);
  } else if (CAUSAL) {
    const int H = nqb - 1 - rank, L = rank;
    const int tH = ntiles(H), tL = L != H ? ntiles(L) : 0;
    const int tot = tH + tL;
    T = (tot + 1) / 2;
    merge = tot - T > tL;                            // team 1 computed part of H
    if (team == 0) { blk0 = H; cnt = T; }
    else { blk0 = tL > 0 ? L : H; cnt = tot - T; sw = tL > 0 ? tL : (1 << 30); blk1 = H; t1 = T; }
    if (team == 1 && tL == 0) t1 = T;                // middle block: H tiles from T on
  } else {
    blk0 = 2 * rank + team;
    T = ntiles(2 * rank);
    cnt = blk0 < nqb ? ntiles(blk0) : 0;
  }
  T = uni(T); cnt = uni(cnt);
  // key tile of step t
  auto tile_of = [&](int t) __attribute__((always_inline)) -> int {
    if (!PAIR || !CAUSAL || team == 0) return t;
    if (t < sw) return blk0 == blk1 ? t1 + t : t;    // (middle block: starts at T)
    return t1 + (t - sw);
  };

  // ---- per-wave row state
  int qb, qw, qrow;
  bool row_ok;
  bf16x8 qf[NKK];
  bf16x8 dof[DQ ? NKK : 1];
  float lse2 = 0.f, dl = 0.f;
  const uint64_t* dmrow = dbits;
  auto load_rows = [&](int qb_) __attribute__((always_inline)) {
    qb = qb_;
    qw = qb * BQ + 32 * wl;
    qrow = qw + r;
    row_ok = qw < S;
    const int qrow_c = min(qrow, S - 1);
    const uint16_t* qp = q + (size_t)(b * S + qrow_c) * ldq + hq * D + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) qf[kk] = ld8(qp + 16 * kk);
    if constexpr (DQ) {
      const uint16_t* dp = dout + (size_t)(b * S + qrow_c) * lddo + hq * D + 8 * hh;
      const uint16_t* op = o + (size_t)(b * S + qrow_c) * ldo + hq * D + 8 * hh;
      float a = 0.f;
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        dof[kk] = ld8(dp + 16 * kk);
        const uint4 ov = *reinterpret_cast<const uint4*>(op + 16 * kk);
        const uint4 dv = __builtin_bit_cast(uint4, dof[kk]);
        a += lo_bf(ov.x) * lo_bf(dv.x) + hi_bf(ov.x) * hi_bf(dv.x);
        a += lo_bf(ov.y) * lo_bf(dv.y) + hi_bf(ov.y) * hi_bf(dv.y);
        a += lo_bf(ov.z) * lo_bf(dv.z) + hi_bf(ov.z) * hi_bf(dv.z);
        a += lo_bf(ov.w) * lo_bf(dv.w) + hi_bf(ov.w) * hi_bf(dv.w);
      }
      const float dsum = xhalf_sum(a);     // delta = rowsum(dO * O)
      const size_t li = ((size_t)b * Hq + hq) * S + qrow_c;
      lse2 = lse[li];
      dl = dsum * dkeep;                   // delta (1 - p): the dropped branch of dS
      // published for kmajor (both teams of a split block write the same value)
      if (row_ok && hh == 0 && qrow < S) delta[li] = dl;
    }
    dmrow = dbits + ((size_t)(b * Hq + hq) * NB + (min(qw, S - 1) >> 5)) * NKT * 64 + lane;
  };
  float m_i = -INFINITY, l_i = 0.f;
  f32x16 acc[NDT];   // FWD: O^T, DQ: dQ^T
  auto reset = [&]() __attribute__((always_inline)) {
    m_i = -INFINITY;
    l_i = 0.f;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) acc[dt] = f32x16{};
  };
  auto finalize = [&]() __attribute__((always_inline)) {
    if (!(row_ok && qrow < S)) return;
    float sc = oscale;
    if constexpr (!DQ) {
      const float lt = xhalf_sum(l_i);
      sc = lt > 0.f ? oscale / lt : 0.f;
      if (hh == 0) lse[((size_t)b * Hq + hq) * S + qrow] = lt > 0.f ? m_i * c + __log2f(lt) : INFINITY;
    }
    uint16_t* op = DQ ? dq + (size_t)(b * S + qrow) * lddq + hq * D : o + (size_t)(b * S + qrow) * ldo + hq * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) store_row32(op + 32 * dt, acc[dt], sc, hh);
    // dQ's bias-gradient column partials (S % 32 == 0: every row of the wave is valid)
    if (DQ && bpart) bias_partial_store<NDT>(acc, sc, bpart, ldbp, (b * S + qw) >> 5, hq * D, 0, lane);
  };
  reset();
  load_rows(blk0);
  // The row operands (Q, dO, O, lse) are complete before the tile loop.  This must be the
  // compiler-visible builtin, not asm: the waitcnt pass does not see the LDS-DMA issued
  // from inline asm, so without it the pass keeps these pre-loop loads "in flight" and
  // puts vmcnt(3..0) waits in front of the loop's MFMAs -- which the hardware counter
  // resolves by waiting for the NEXT tile's DMA too (load latency exposed every tile).
  __builtin_amdgcn_s_waitcnt(0);

  // lane-constant LDS offsets (the 32-row subtile steps are immediates)
  int offK[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) offK[kk] = toff<D>(r, 2 * kk + hh);
  int offT[NDT][2];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    const int col = 32 * dt + 16 * (g & 1) + 4 * (gi & 3);
    const int row0 = 4 * hh + (gi >> 2);
    offT[dt][0] = toff<D>(row0, col >> 3) + (col & 7) * 2;
    offT[dt][1] = toff<D>(row0 + 8, col >> 3) + (col & 7) * 2;
  }
  // causal diagonal: element e of a lane is dead when crow(e, 0) > r - 4 hh
  const int rr = r - 4 * hh;

  const uint16_t* kbase = k + (size_t)b * S * ldk + hk * D;
  const uint16_t* vbase = v + (size_t)b * S * ldv + hk * D;
  const int prow = lane / CPR, slot = lane % CPR;
  auto issue = [&](char* kd, char* vd, int j) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = wl + 4 * i;
      const int R = p * RPP + prow;
      const int key = min(j * BK + R, S - 1);  // tail rows: finite duplicates, masked later
      const int ch = slot ^ swz<D>(R);
      dma16(kbase + (size_t)key * ldk + ch * 8, kd + p * 1024);
      dma16(vbase + (size_t)key * ldv + ch * 8, vd + p * 1024);
    }
  };
  uint64_t dm_cur = 0, dm_next = 0;
  // dropout words of step t (the rows of the block that step belongs to)
  auto dmload = [&](int t) __attribute__((always_inline)) -> uint64_t {
    if (!DROP) return 0;
    const int qb_ = (PAIR && CAUSAL && team == 1 && t >= sw) ? blk1 : blk0;
    const int qw_ = qb_ * BQ + 32 * wl;
    if (qw_ >= S) return 0;
    if constexpr (DGEN) {   // the pre-pass's words for (row block qw_, 128-key tile j), hashed here
      const uint32_t j = (uint32_t)((tile_of(t) * BK) >> 7);
      const uint32_t row = (uint32_t)(((long long)b * dg.hg + dg.hoff + hq) * S + qw_ + r);
      const uint32_t rbase = row * 0x85EBCA6Bu, seed = *dg.seed + dg.salt;
      const uint32_t lo = drop_stream_bits(rbase, 4 * j, hh, seed, dg.thr16) |
                          (drop_stream_bits(rbase, 4 * j + 1, hh, seed, dg.thr16) << 8);
      const uint32_t hi = drop_stream_bits(rbase, 4 * j + 2, hh, seed, dg.thr16) |
                          (drop_stream_bits(rbase, 4 * j + 3, hh, seed, dg.thr16) << 8);
      return (uint64_t)lo | ((uint64_t)hi << 32);
    }
    const uint64_t* row = dbits + ((size_t)(b * Hq + hq) * NB + (qw_ >> 5)) * NKT * 64 + lane;
    return row[(size_t)((tile_of(t) * BK) >> 7) * 64];
  };

  // FULL: every key of the tile is visible to every row of the wave (below the causal
  // diagonal, no padded tail): the tile body is straight-line code with no per-subtile
  // guards or masks, so the compiler can hoist the LDS reads ahead of their MFMAs and
  // interleave one subtile's softmax VALU with the neighbouring subtile's MFMAs (the
  // guarded form compiles to one basic block per subtile: read -> wait -> MFMA in series).
  auto compute_body = [&](const char* Kt, const char* Vt, int kv0, int nsub, int tdiag, bool tail,
                          auto fullc) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(fullc)::value;
    if constexpr (!DQ) {
      f32x16 sacc[NSUB];
#pragma unroll
      for (int t = 0; t < NSUB; ++t) {
        if (FULL || t < nsub) {
          bf16x8 kr[NKK];
#pragma unroll
          for (int kk = 0; kk < NKK; ++kk) kr[kk] = lds8(Kt + 32 * t * RB, offK[kk]);
          sacc[t] = f32x16{};
#pragma unroll
          for (int kk = 0; kk < NKK; ++kk) sacc[t] = mfma32(kr[kk], qf[kk], sacc[t]);
        }
      }
#pragma unroll
      for (int t = 0; t < NSUB; ++t) {
        // (a wave-uniform branch: only the diagonal subtile pays the per-element select)
        if (!FULL && CAUSAL && uni(t == tdiag ? 1 : 0)) {
          asm volatile("" ::: "memory");   // a real branch, not per-element selects
#pragma unroll
          for (int e = 0; e < 16; ++e) sacc[t][e] = crow(e, 0) > rr ? -INFINITY : sacc[t][e];
        }
        if (!FULL && !CAUSAL && tail && t < nsub) {
          const int lim = kl - kv0 - 32 * t - 4 * hh;
#pragma unroll
          for (int e = 0; e < 16; ++e) sacc[t][e] = crow(e, 0) >= lim ? -INFINITY : sacc[t][e];
        }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < NSUB; ++t)
        if (FULL || t < nsub) {
#pragma unroll
          for (int e = 0; e < 16; ++e) mx = fmaxf(mx, sacc[t][e]);
        }
      mx = xhalf_max(mx);
      // exact deferred rescale (T13, threshold 0): skipped when no row raised its max
      if (!__all(mx <= m_i)) {
        const float m_new = fmaxf(m_i, mx);
        const float alpha = m_new == -INFINITY ? 1.f : __builtin_amdgcn_exp2f((m_i - m_new) * c);
        l_i *= alpha;
        m_i = m_new;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[dt][e] *= alpha;
      }
      const float mc = m_i == -INFINITY ? 0.f : m_i * c;
      // packed fp32 (v_pk_fma_f32 / v_pk_add_f32: two elements per issue) for the exponent
      // argument and the row sum -- the forward is VALU-issue bound (profiles/r4_s1)
      const f32x2_t c2 = {c, c}, nmc2 = {-mc, -mc};
      f32x2_t rs2 = {0.f, 0.f};
#pragma unroll
      for (int t = 0; t < NSUB; ++t)
        if (FULL || t < nsub) {
#pragma unroll
          for (int e = 0; e < 16; e += 2) {
            const f32x2_t a = __builtin_elementwise_fma((f32x2_t){sacc[t][e], sacc[t][e + 1]}, c2, nmc2);
            const f32x2_t p = {__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
            sacc[t][e] = p.x;
            sacc[t][e + 1] = p.y;
            rs2 += p;
          }
        }
      l_i += rs2.x + rs2.y;
#pragma unroll
      for (int t = 0; t < NSUB; ++t)
        if (FULL || t < nsub) {
          const uint32_t wd = (uint32_t)(dm_cur >> (32 * ((((kv0 >> 5) + t) >> 1) & 1)));
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            bf16x8 vr[NDT];
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt)
              vr[dt] = cat(tr_read(Vt + (32 * t + 16 * s) * RB, offT[dt][0]),
                           tr_read(Vt + (32 * t + 16 * s) * RB, offT[dt][1]));
            const bf16x8 pb = DROP ? pack8_keep(sacc[t], 8 * s, wd, 8 * (t & 1)) : pack8(sacc[t], 8 * s);
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) acc[dt] = mfma32(vr[dt], pb, acc[dt]);
          }
        }
    } else {
#pragma unroll
      for (int t = 0; t < NSUB; ++t) {
        if (FULL || t < nsub) {
          bf16x8 kr[NKK], vr[NKK];
#pragma unroll
          for (int kk = 0; kk < NKK; ++kk) {
            kr[kk] = lds8(Kt + 32 * t * RB, offK[kk]);
            vr[kk] = lds8(Vt + 32 * t * RB, offK[kk]);
          }
          f32x16 s_ = f32x16{}, dp = f32x16{};
#pragma unroll
          for (int kk = 0; kk < NKK; ++kk) {
            s_ = mfma32(kr[kk], qf[kk], s_);
            dp = mfma32(vr[kk], dof[kk], dp);
          }
          const uint32_t wd = (uint32_t)(dm_cur >> (32 * ((((kv0 >> 5) + t) >> 1) & 1)));
          const int lim = kl - kv0 - 32 * t - 4 * hh;
          float pv[16];
          const f32x2_t c2 = {c, c}, nl2 = {-lse2, -lse2};
#pragma unroll
          for (int e = 0; e < 16; e += 2) {   // packed exponent arguments (v_pk_fma_f32)
            const f32x2_t a = __builtin_elementwise_fma((f32x2_t){s_[e], s_[e + 1]}, c2, nl2);
            pv[e] = __builtin_amdgcn_exp2f(a.x);
            pv[e + 1] = __builtin_amdgcn_exp2f(a.y);
          }
          // (only the diagonal / padded-tail subtile is masked: a wave-uniform branch)
          if (!FULL && uni((CAUSAL && t == tdiag) || (!CAUSAL && tail) ? 1 : 0)) {
            asm volatile("" ::: "memory");   // a real branch, not per-element selects
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              if (CAUSAL) pv[e] = crow(e, 0) > rr ? 0.f : pv[e];
              else pv[e] = crow(e, 0) >= lim ? 0.f : pv[e];
            }
          }
          const f32x2_t ndl2 = {-dl, -dl};
#pragma unroll
          for (int e = 0; e < 16; e += 2) {
            f32x2_t x = {dp[e], dp[e + 1]};
            if (DROP) {   // (keep ? dP : 0) - delta
              x.x = __uint_as_float(__float_as_uint(x.x) & elem_keep(wd, 8 * (t & 1), e));
              x.y = __uint_as_float(__float_as_uint(x.y) & elem_keep(wd, 8 * (t & 1), e + 1));
            }
            const f32x2_t d = (f32x2_t){pv[e], pv[e + 1]} * (x + ndl2);   // dS^T (1/(1-p) in oscale)
            s_[e] = d.x;
            s_[e + 1] = d.y;
          }
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const bf16x8 db = pack8(s_, 8 * s);
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
              const bf16x8 ktr = cat(tr_read(Kt + (32 * t + 16 * s) * RB, offT[dt][0]),
                                     tr_read(Kt + (32 * t + 16 * s) * RB, offT[dt][1]));
              acc[dt] = mfma32(ktr, db, acc[dt]);
            }
          }
        }
      }
    }
  };
  auto compute = [&](const char* Kt, const char* Vt, int j) __attribute__((always_inline)) {
    const int kv0 = j * BK;
    int nsub = NSUB;
    // (qw, kv0 are 32-aligned: subtiles up to and including the diagonal one)
    if (CAUSAL) nsub = qw >= kv0 ? min(NSUB, (qw - kv0) / 32 + 1) : 0;
    nsub = uni(row_ok ? nsub : 0);
    if (nsub == 0) return;
    // the subtile on the causal diagonal (qw is 32-aligned) and the padded-key tail
    const int tdiag = CAUSAL ? uni((qw - kv0) >> 5) : -1;
    const bool tail = uni(kv0 + BK > kl ? 1 : 0);
    // forward only: the FULL dQ body measured slower at D = 64 (38.3 vs 36.0 us per GPT-2
    // layer; profiles/r4_s2/) and spills at D = 128, so dQ keeps the guarded form
    if (!DQ && uni((!CAUSAL || kv0 + BK <= qw) && !tail ? 1 : 0))
      compute_body(Kt, Vt, kv0, NSUB, tdiag, false, std::integral_constant<bool, !DQ>{});
    else
      compute_body(Kt, Vt, kv0, nsub, tdiag, tail, std::false_type{});
  };

  // one step: wait for this step's tile, hand the other slot to the next step's DMA, compute
  auto step = [&](char* Kc, char* Vc, char* Kn, char* Vn, int t) __attribute__((always_inline)) {
    vm_drain();
    __syncthreads();
    if (t + 1 < cnt) {
      issue(Kn, Vn, tile_of(t + 1));
      dm_next = dmload(t + 1);
    }
    if (t < cnt) {
      if (PAIR && CAUSAL && team == 1 && t == sw) {   // team 1: L done, continue with H
        finalize();
        reset();
        load_rows(blk1);
        __builtin_amdgcn_s_waitcnt(0);   // (see after the first load_rows)
      }
      compute(Kc, Vc, tile_of(t));
    }
    dm_cur = dm_next;
  };
  auto run = [&](char* ka, char* kb_, char* va, char* vb) __attribute__((always_inline)) {
    if (cnt > 0) {
      issue(ka, va, tile_of(0));
      dm_cur = dmload(0);
    }
    for (int t = 0; t < T; t += 2) {
      step(ka, va, kb_, vb, t);
      if (t + 1 < T) step(kb_, vb, ka, va, t + 1);
    }
  };
  if (!PAIR || team == 0) run(k0, k1, v0, v1);
  else run(k2, k3, v2, v3);

  if constexpr (PAIR) {
    if (CAUSAL && merge) {
      // team 1's partial of block H -> team 0 (identical lane mapping: element-wise)
      float* mw = mrg + wl * NREG * 64 + lane;
      __syncthreads();   // the merge area aliases team 1's tiles
      if (team == 1) {
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int e = 0; e < 16; ++e) mw[(dt * 16 + e) * 64] = acc[dt][e];
        mw[(NDT * 16) * 64] = m_i;
        mw[(NDT * 16 + 1) * 64] = l_i;
      }
      __syncthreads();
      if (team == 0) {
        if constexpr (DQ) {
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[dt][e] += mw[(dt * 16 + e) * 64];
        } else {
          const float mB = mw[(NDT * 16) * 64], lB = mw[(NDT * 16 + 1) * 64];
          const float m = fmaxf(m_i, mB);
          const float aA = m_i == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m_i - m) * c);
          const float aB = mB == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((mB - m) * c);
          l_i = l_i * aA + lB * aB;
          m_i = m;
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[dt][e] = acc[dt][e] * aA + mw[(dt * 16 + e) * 64] * aB;
        }
      }
      if (team == 0) finalize();
      return;
    }
    if (cnt > 0 || team == 0) finalize();
    return;
  }
  finalize();
}

// ============================================================================ key-major
// dK, dV.  DP: 0 = every dK/dV column in one pass (D = 64, K and V rows in registers);
// 1 / 2 = columns [0, D/2) / [D/2, D) (D = 128: K rows read from LDS, S and dP recomputed
// by the second pass -- the accumulators of all 128 columns plus the operands exceed the
// 256-register budget of two waves per SIMD).
// PAIR (D = 64): two 4-wave teams as in qmajor; the heavy key block (most query rows, the
// smallest index under a causal mask) is split between the teams and team 1's partial
// dK^T / dV^T are summed into team 0's through LDS.
template <int D, bool CAUSAL, bool DROP, int DP, bool PAIR, bool RAGGED>
__global__ __launch_bounds__(PAIR ? 512 : 256) __attribute__((amdgpu_waves_per_eu(2, 2))) void flash_kmajor_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, int ldq, int ldk, int ldv,
    const uint16_t* __restrict__ dout, int lddo, const float* __restrict__ lse,
    const float* __restrict__ delta, uint16_t* __restrict__ dk, uint16_t* __restrict__ dv,
    int lddk, int lddv, int S, int Hq, int Hkv, const int* __restrict__ klen, float c,
    float dkscale, float dvscale, const uint32_t* __restrict__ dbits, int NB, int NQT,
    float* __restrict__ bpart, int ldbp, int bcol) {
  // 64-row Q/dO tiles (32 for D = 128: K image + ring = 65 KB, two workgroups per CU)
  constexpr int KB = 128, KW = 128, QT = D == 64 ? 64 : 32, NQS = QT / 32, NKK = D / 16, NDT = D / 32;
  constexpr int NDL = DP == 0 ? NDT : NDT / 2;
  constexpr int DT0 = DP == 2 ? NDT / 2 : 0;
  constexpr int RB = D * 2, CPR = D / 8, RPP = 64 / CPR;
  constexpr int QTILE = QT * RB, PIECES = QTILE / 1024, PPW = (2 * PIECES) / 4;
  constexpr bool KREG = D <= 64;
  static_assert(KREG || !PAIR, "PAIR needs K rows in registers");
  constexpr int KT_BYTES = KREG ? 16 : KW * RB;
  constexpr int Q2 = PAIR ? QTILE : 16, L2 = PAIR ? 64 : 4;
  constexpr int NREG = 2 * NDL * 16;
  constexpr int MRG = PAIR ? 4 * NREG * 64 : 4;
  __shared__ __attribute__((aligned(16))) char q0[QTILE];
  __shared__ __attribute__((aligned(16))) char q1[QTILE];
  __shared__ __attribute__((aligned(16))) char o0[QTILE];
  __shared__ __attribute__((aligned(16))) char o1[QTILE];
  __shared__ __attribute__((aligned(16))) float l0[64];   // one dword-DMA wave instruction
  __shared__ __attribute__((aligned(16))) float l1[64];
  __shared__ __attribute__((aligned(16))) float d0[64];
  __shared__ __attribute__((aligned(16))) float d1[64];
  __shared__ __attribute__((aligned(16))) char q2[Q2];
  __shared__ __attribute__((aligned(16))) char q3[Q2];
  __shared__ __attribute__((aligned(16))) char o2[Q2];
  __shared__ __attribute__((aligned(16))) char o3[Q2];
  __shared__ __attribute__((aligned(16))) float l2[L2];
  __shared__ __attribute__((aligned(16))) float l3[L2];
  __shared__ __attribute__((aligned(16))) float d2[L2];
  __shared__ __attribute__((aligned(16))) float d3[L2];
  __shared__ __attribute__((aligned(16))) char kt_lds[KT_BYTES];
  __shared__ __attribute__((aligned(16))) float mrg[MRG];

  const int tid = threadIdx.x, lane = tid & 63, w = uni(tid >> 6);
  const int team = PAIR ? (w >> 2) : 0, wl = w & 3;
  const int r = lane & 31, hh = lane >> 5, g = lane >> 4, gi = lane & 15;
  const int nkb = (S + KB - 1) / KB;
  const int nunits = PAIR ? (nkb + 1) / 2 : nkb;
  int rank, head;
  block_map((int)gridDim.x / nunits, rank, head);   // grid = nunits x (B * Hkv)
  const int hk = head % Hkv, b = head / Hkv;
  const int grp = Hq / Hkv;
  const int kl = klen ? klen[b] : S;
  const int nqt = (S + QT - 1) / QT;
  auto qt0_of = [&](int kb_) __attribute__((always_inline)) { return CAUSAL ? kb_ * KB / QT : 0; };
  auto items_of = [&](int kb_) __attribute__((always_inline)) { return (nqt - qt0_of(kb_)) * grp; };
  // ---- schedule (items = (query head, query tile) of a key block)
  int blk0, cnt, sw = 1 << 30, blk1 = -1, t1 = 0, T;
  bool merge = false;
  if (!PAIR) {
    blk0 = rank;                                     // causal: block 0 (most rows) first
    cnt = T = items_of(blk0);
  } else if (CAUSAL) {
    const int Hb = rank, Lb = nkb - 1 - rank;        // heavy = small index
    const int tH = items_of(Hb), tL = Lb != Hb ? items_of(Lb) : 0;
    const int tot = tH + tL;
    T = (tot + 1) / 2;
    merge = tot - T > tL;
    if (team == 0) { blk0 = Hb; cnt = T; }
    else { blk0 = tL > 0 ? Lb : Hb; cnt = tot - T; sw = tL > 0 ? tL : (1 << 30); blk1 = Hb; t1 = T; }
  } else {
    blk0 = 2 * rank + team;
    T = items_of(2 * rank);
    cnt = blk0 < nkb ? items_of(blk0) : 0;
  }
  T = uni(T); cnt = uni(cnt);
  auto item_of = [&](int t) __attribute__((always_inline)) -> int {               // item index within the block of step t
    if (!PAIR || !CAUSAL || team == 0) return t;
    if (t < sw) return blk0 == blk1 ? t1 + t : t;
    return t1 + (t - sw);
  };
  auto blk_of = [&](int t) __attribute__((always_inline)) -> int {
    return (PAIR && CAUSAL && team == 1 && t >= sw) ? blk1 : blk0;
  };

  // ---- per-wave key state
  int kb, kw0, key;
  bool key_ok, wave_on;
  bf16x8 kf[KREG ? NKK : 1], vf[NKK];
  f32x16 dvacc[NDL], dkacc[NDL];
  auto load_keys = [&](int kb_) __attribute__((always_inline)) {
    kb = kb_;
    kw0 = kb * KB + 32 * wl;
    key = kw0 + r;
    key_ok = key < kl;
    wave_on = kw0 < S;
    const int key_c = min(key, S - 1);
    const uint16_t* kp = k + (size_t)(b * S + key_c) * ldk + hk * D + 8 * hh;
    const uint16_t* vp = v + (size_t)(b * S + key_c) * ldv + hk * D + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      if constexpr (KREG) kf[kk] = ld8(kp + 16 * kk);
      vf[kk] = ld8(vp + 16 * kk);
    }
#pragma unroll
    for (int dt = 0; dt < NDL; ++dt) { dvacc[dt] = f32x16{}; dkacc[dt] = f32x16{}; }
  };
  auto finalize = [&]() __attribute__((always_inline)) {
    if (!(key < S)) return;
    uint16_t* dkp = dk + (size_t)(b * S + key) * lddk + hk * D;
    uint16_t* dvp = dv + (size_t)(b * S + key) * lddv + hk * D;
#pragma unroll
    for (int dt = 0; dt < NDL; ++dt) {
      store_row32(dkp + 32 * (dt + DT0), dkacc[dt], dkscale, hh);
      store_row32(dvp + 32 * (dt + DT0), dvacc[dt], dvscale, hh);
    }
    // dK / dV bias-gradient column partials (S % 32 == 0: every key of the wave is valid)
    if (bpart) {
      bias_partial_store<NDL>(dkacc, dkscale, bpart, ldbp, (b * S + kw0) >> 5, bcol + hk * D, DT0, lane);
      bias_partial_store<NDL>(dvacc, dvscale, bpart, ldbp, (b * S + kw0) >> 5, bcol + (Hkv + hk) * D, DT0, lane);
    }
  };
  load_keys(blk0);
  __builtin_amdgcn_s_waitcnt(0);  // K / V rows complete before the loop (see qmajor)
  const int krow = 32 * wl + r;   // this lane's row of the K image (D = 128)
  if constexpr (!KREG) {
    constexpr int KCH = KW * CPR / 256;
#pragma unroll
    for (int i = 0; i < KCH; ++i) {
      const int ci = tid + 256 * i, row = ci / CPR, ch = ci % CPR;
      const int kk_ = min(kb * KB + row, S - 1);
      *reinterpret_cast<uint4*>(kt_lds + toff<D>(row, ch)) =
          *reinterpret_cast<const uint4*>(k + (size_t)(b * S + kk_) * ldk + hk * D + ch * 8);
    }
  }

  int offQ[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) offQ[kk] = toff<D>(r, 2 * kk + hh);
  int offKl[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) offKl[kk] = KREG ? 0 : toff<D>(krow, 2 * kk + hh);
  int offT[NDL][2];
#pragma unroll
  for (int dt = 0; dt < NDL; ++dt) {
    const int col = 32 * (dt + DT0) + 16 * (g & 1) + 4 * (gi & 3);
    const int row0 = 4 * hh + (gi >> 2);
    offT[dt][0] = toff<D>(row0, col >> 3) + (col & 7) * 2;
    offT[dt][1] = toff<D>(row0 + 8, col >> 3) + (col & 7) * 2;
  }
  const int rr = r - 4 * hh;   // diagonal: element e dead when r - 4hh > crow(e, 0)

  const int prow = lane / CPR, slot = lane % CPR;
  auto decode = [&](int t, int& hq, int& qs) __attribute__((always_inline)) {
    const int kb_ = blk_of(t), it = item_of(t);
    const int ph = nqt - qt0_of(kb_);
    hq = hk * grp + it / ph;
    qs = (qt0_of(kb_) + it % ph) * QT;
  };
  auto issue = [&](char* qd, char* od, float* ld, float* dd, int t) __attribute__((always_inline)) {
    int hq, qs;
    decode(t, hq, qs);
    const uint16_t* qb_ = q + (size_t)b * S * ldq + hq * D;
    const uint16_t* ob_ = dout + (size_t)b * S * lddo + hq * D;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = wl + 4 * i;                // 0 .. 2*PIECES-1: Q pieces then dO pieces
      const bool isq = p < PIECES;
      const int pp = isq ? p : p - PIECES;
      const int R = pp * RPP + prow;
      const int row = min(qs + R, S - 1);
      const int ch = slot ^ swz<D>(R);
      if (isq) dma16(qb_ + (size_t)row * ldq + ch * 8, qd + pp * 1024);
      else dma16(ob_ + (size_t)row * lddo + ch * 8, od + pp * 1024);
    }
    if (wl < 2) {
      const size_t li = ((size_t)b * Hq + hq) * S + min(qs + lane, S - 1);
      if (wl == 0) dma4(lse + li, (char*)ld);
      else dma4(delta + li, (char*)dd);
    }
  };
  auto dmload = [&](int t) __attribute__((always_inline)) -> uint32_t {
    if (!DROP) return 0u;
    int hq, qs;
    decode(t, hq, qs);
    const int kw = blk_of(t) * KB + 32 * wl;
    if (kw >= S) return 0u;
    return dbits[(((size_t)(b * Hq + hq) * NB + (kw >> 5)) * NQT + (qs >> 6)) * 64 + lane];
  };
  uint32_t dm_cur = 0, dm_next = 0;

  // FULL: every query subtile of the step active, none on the causal diagonal, no query
  // tail -- straight-line code (see qmajor's compute_body)
  auto compute_body = [&](const char* Qt, const char* Ot, const float* Lt, const float* Dt, int qs,
                          auto fullc) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
    for (int u = 0; u < NQS; ++u) {
      const int qsu = qs + 32 * u;
      if constexpr (!FULL) {
        const bool act = uni(wave_on && qsu < S && (!CAUSAL || qsu + 31 >= kw0) ? 1 : 0);
        if (!act) continue;
      }
      f32x16 sacc = f32x16{}, dpacc = f32x16{};
      const char* Qu = Qt + 32 * u * RB;
      const char* Ou = Ot + 32 * u * RB;
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        const bf16x8 qa = lds8(Qu, offQ[kk]);
        const bf16x8 oa = lds8(Ou, offQ[kk]);
        const bf16x8 kb_ = KREG ? kf[kk] : lds8(kt_lds, offKl[kk]);
        sacc = mfma32(qa, kb_, sacc);
        dpacc = mfma32(oa, vf[kk], dpacc);
      }
      const bool diag = !FULL && CAUSAL && qsu == kw0;
      const bool qtail = !FULL && qsu + 32 > S;
      // P of the subtile, unmasked; the causal diagonal subtile (wave-uniform branch) and, in
      // RAGGED launches only, the query tail / invalid keys are zeroed afterwards
      float pv[16];
      const f32x2_t c2 = {c, c};
#pragma unroll
      for (int e = 0; e < 16; e += 4) {
        // row constants of the lane's query rows, 4 consecutive per e >> 2 (one ds_read_b128);
        // exponent arguments two at a time (v_pk_fma_f32)
        const float4 lsq = *reinterpret_cast<const float4*>(Lt + 32 * u + 8 * (e >> 2) + 4 * hh);
        const f32x2_t a0 = __builtin_elementwise_fma((f32x2_t){sacc[e], sacc[e + 1]}, c2, (f32x2_t){-lsq.x, -lsq.y});
        const f32x2_t a1 = __builtin_elementwise_fma((f32x2_t){sacc[e + 2], sacc[e + 3]}, c2, (f32x2_t){-lsq.z, -lsq.w});
        pv[e] = __builtin_amdgcn_exp2f(a0.x);
        pv[e + 1] = __builtin_amdgcn_exp2f(a0.y);
        pv[e + 2] = __builtin_amdgcn_exp2f(a1.x);
        pv[e + 3] = __builtin_amdgcn_exp2f(a1.y);
      }
      if (!FULL && uni(diag ? 1 : 0)) {
        asm volatile("" ::: "memory");   // keeps this a real (scalar) branch: not if-converted into selects
#pragma unroll
        for (int e = 0; e < 16; ++e) pv[e] = rr > crow(e, 0) ? 0.f : pv[e];
      }
      if constexpr (RAGGED) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          if (qtail) pv[e] = qsu + crow(e, hh) >= S ? 0.f : pv[e];
          pv[e] = key_ok ? pv[e] : 0.f;
        }
      }
#pragma unroll
      for (int e = 0; e < 16; e += 2) {
        float4 dlq;
        if ((e & 3) == 0) dlq = *reinterpret_cast<const float4*>(Dt + 32 * u + 8 * (e >> 2) + 4 * hh);
        const f32x2_t ndl = (e & 3) == 0 ? (f32x2_t){-dlq.x, -dlq.y} : (f32x2_t){-dlq.z, -dlq.w};
        const f32x2_t p = {pv[e], pv[e + 1]};
        // dS = P (keep ? dP - delta : -delta) = P ((keep ? dP : 0) - delta); the dropped P is 0
        // in dV's operand: one sign-extended bit-field extract serves both
        f32x2_t x = {dpacc[e], dpacc[e + 1]};
        if (DROP) {
          const uint32_t mk0 = elem_keep(dm_cur, 8 * ((qsu >> 5) & 1), e);
          const uint32_t mk1 = elem_keep(dm_cur, 8 * ((qsu >> 5) & 1), e + 1);
          x.x = __uint_as_float(__float_as_uint(x.x) & mk0);
          x.y = __uint_as_float(__float_as_uint(x.y) & mk1);
          sacc[e] = __uint_as_float(__float_as_uint(p.x) & mk0);
          sacc[e + 1] = __uint_as_float(__float_as_uint(p.y) & mk1);
        } else {
          sacc[e] = p.x;
          sacc[e + 1] = p.y;
        }
        const f32x2_t d = p * (x + ndl);   // dS (1/(1-p) in dkscale), v_pk_add_f32 + v_pk_mul_f32
        dpacc[e] = d.x;
        dpacc[e + 1] = d.y;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pb = pack8(sacc, 8 * s);
        const bf16x8 db = pack8(dpacc, 8 * s);
        const int rofs = (32 * u + 16 * s) * RB;
#pragma unroll
        for (int dt = 0; dt < NDL; ++dt) {
          const bf16x8 dot = cat(tr_read(Ot + rofs, offT[dt][0]), tr_read(Ot + rofs, offT[dt][1]));
          dvacc[dt] = mfma32(dot, pb, dvacc[dt]);
          const bf16x8 qtr = cat(tr_read(Qt + rofs, offT[dt][0]), tr_read(Qt + rofs, offT[dt][1]));
          dkacc[dt] = mfma32(qtr, db, dkacc[dt]);
        }
      }
    }
  };
  auto compute = [&](const char* Qt, const char* Ot, const float* Lt, const float* Dt, int t) __attribute__((always_inline)) {
    int hq, qs;
    decode(t, hq, qs);
    (void)hq;
    // (the straight-line FULL body spills at D = 64 -- dK/dV accumulators plus hoisted
    // operands exceed the two-waves-per-SIMD register budget -- so it is not instantiated)
    compute_body(Qt, Ot, Lt, Dt, qs, std::false_type{});
  };

  auto step = [&](char* Qc, char* Oc, float* Lc, float* Dc, char* Qn, char* On, float* Ln, float* Dn,
                  int t) __attribute__((always_inline)) {
    vm_drain();
    __syncthreads();
    if (t + 1 < cnt) {
      issue(Qn, On, Ln, Dn, t + 1);
      dm_next = dmload(t + 1);
    }
    if (t < cnt) {
      if (PAIR && CAUSAL && team == 1 && t == sw) {   // team 1: light block done, on to the heavy one
        finalize();
        load_keys(blk1);
        __builtin_amdgcn_s_waitcnt(0);   // (see qmajor)
      }
      compute(Qc, Oc, Lc, Dc, t);
    }
    dm_cur = dm_next;
  };
  auto run = [&](char* qa, char* qb_, char* oa, char* ob, float* la, float* lb, float* da, float* db) __attribute__((always_inline)) {
    if (cnt > 0) {
      issue(qa, oa, la, da, 0);
      dm_cur = dmload(0);
    }
    for (int t = 0; t < T; t += 2) {
      step(qa, oa, la, da, qb_, ob, lb, db, t);
      if (t + 1 < T) step(qb_, ob, lb, db, qa, oa, la, da, t + 1);
    }
  };
  if (!PAIR || team == 0) run(q0, q1, o0, o1, l0, l1, d0, d1);
  else run(q2, q3, o2, o3, l2, l3, d2, d3);

  if constexpr (PAIR) {
    if (CAUSAL && merge) {
      float* mw = mrg + wl * NREG * 64 + lane;
      __syncthreads();   // the merge area aliases team 1's tiles
      if (team == 1) {
#pragma unroll
        for (int dt = 0; dt < NDL; ++dt)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            mw[(dt * 16 + e) * 64] = dkacc[dt][e];
            mw[((NDL + dt) * 16 + e) * 64] = dvacc[dt][e];
          }
      }
      __syncthreads();
      if (team == 0) {
#pragma unroll
        for (int dt = 0; dt < NDL; ++dt)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            dkacc[dt][e] += mw[(dt * 16 + e) * 64];
            dvacc[dt][e] += mw[((NDL + dt) * 16 + e) * 64];
          }
        finalize();
      }
      return;
    }
    if (cnt > 0 || team == 0) finalize();
    return;
  }
  finalize();
}

// ====================================================================== key-major, D = 128
// dK, dV of D = 128 in ONE pass (S and dP computed once per subtile, not once per half of
// the columns).  One 8-wave workgroup per 128-key block, two waves per SIMD: waves w and
// w + 4 (same SIMD) own the same 32 keys.  Team 0 (w < 4) holds the keys' K rows and
// computes S^T -> P; team 1 holds their V rows and computes dP^T -> x = (keep ? dP : 0) -
// delta.  The two fp32 16-element lane images are swapped through LDS (identical MFMA
// output layout in both waves: an element-wise exchange, conflict-free 16-B lane slots),
// then both form dS = P x and the dropped P, and each accumulates its own half of the
// dK^T / dV^T columns ([0, 64) team 0, [64, 128) team 1).  Per 32 x 32 subtile and key
// group: 32 MFMAs (8 S + 8 dP + 16 dK/dV) instead of the two-pass 48, and one exp2 per
// element instead of two.  Q / dO tiles of 32 rows stream through the LDS-DMA ring as in
// flash_kmajor_kernel; two barriers per tile (ring, exchange), executed by every wave
// whatever its causal / tail state, so the barrier counts of all waves match.
template <bool CAUSAL, bool DROP, bool RAGGED>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void flash_kmajor128_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, int ldq, int ldk, int ldv,
    const uint16_t* __restrict__ dout, int lddo, const float* __restrict__ lse,
    const float* __restrict__ delta, uint16_t* __restrict__ dk, uint16_t* __restrict__ dv,
    int lddk, int lddv, int S, int Hq, int Hkv, const int* __restrict__ klen, float c,
    float dkscale, float dvscale, const uint32_t* __restrict__ dbits, int NB, int NQT,
    float* __restrict__ bpart, int ldbp, int bcol) {
  // 32 query rows per step (NQS = 1 subtile; 64 rows per step spilled at 256 VGPRs and
  // measured 349.9 vs 299.7 us).  One exchange buffer: a wave writes it after the ring
  // barrier of step t + 1, and every partner read of step t precedes that barrier (two
  // alternating buffers measured the same, 300.2 vs 299.7 us on one box).
  constexpr int D = 128, KB = 128, QT = 32, NQS = QT / 32, NKK = D / 16, NDL = 2;
  constexpr int RB = D * 2, CPR = D / 8, RPP = 64 / CPR;
  constexpr int QTILE = QT * RB, PIECES = QTILE / 1024, PPW = (2 * PIECES) / 8;
  static_assert(PPW * 8 == 2 * PIECES, "8 waves issue the Q + dO pieces");
  __shared__ __attribute__((aligned(16))) char q0[QTILE];
  __shared__ __attribute__((aligned(16))) char q1[QTILE];
  __shared__ __attribute__((aligned(16))) char o0[QTILE];
  __shared__ __attribute__((aligned(16))) char o1[QTILE];
  __shared__ __attribute__((aligned(16))) float l0[64];
  __shared__ __attribute__((aligned(16))) float l1[64];
  __shared__ __attribute__((aligned(16))) float d0[64];
  __shared__ __attribute__((aligned(16))) float d1[64];
  // [wave][subtile][4 chunks][64 lanes][4 floats]: a wave's 16 elements of a subtile as four
  // 16-B slots
  __shared__ __attribute__((aligned(16))) float xch[8 * NQS * 1024];

  const int tid = threadIdx.x, lane = tid & 63, w = uni(tid >> 6);
  const int team = w >> 2, wl = w & 3;
  const int r = lane & 31, hh = lane >> 5, g = lane >> 4, gi = lane & 15;
  const int nkb = (S + KB - 1) / KB;
  int rank, head;
  block_map((int)gridDim.x / nkb, rank, head);   // grid = nkb x (B * Hkv)
  const int hk = head % Hkv, b = head / Hkv;
  const int grp = Hq / Hkv;
  const int kl = klen ? klen[b] : S;
  const int nqt = (S + QT - 1) / QT;
  const int kb = rank;                            // causal: block 0 (most rows) first
  const int qt0 = CAUSAL ? kb * KB / QT : 0;
  const int ph = nqt - qt0;
  const int cnt = uni(ph * grp);

  const int kw0 = kb * KB + 32 * wl;
  const int key = kw0 + r;
  const bool key_ok = key < kl;
  const bool wave_on = kw0 < S;
  const int DT0 = 2 * team;
  // team 0: K rows of the lane's key; team 1: V rows (the B operands of S^T / dP^T)
  bf16x8 kv[NKK];
  {
    const int key_c = min(key, S - 1);
    const uint16_t* src = team == 0 ? k + (size_t)(b * S + key_c) * ldk : v + (size_t)(b * S + key_c) * ldv;
    src += hk * D + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) kv[kk] = ld8(src + 16 * kk);
  }
  f32x16 dvacc[NDL], dkacc[NDL];
#pragma unroll
  for (int dt = 0; dt < NDL; ++dt) { dvacc[dt] = f32x16{}; dkacc[dt] = f32x16{}; }
  __builtin_amdgcn_s_waitcnt(0);  // K / V rows complete before the loop (see qmajor)

  int offQ[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) offQ[kk] = toff<D>(r, 2 * kk + hh);
  int offT[NDL][2];
#pragma unroll
  for (int dt = 0; dt < NDL; ++dt) {
    const int col = 32 * (dt + DT0) + 16 * (g & 1) + 4 * (gi & 3);
    const int row0 = 4 * hh + (gi >> 2);
    offT[dt][0] = toff<D>(row0, col >> 3) + (col & 7) * 2;
    offT[dt][1] = toff<D>(row0 + 8, col >> 3) + (col & 7) * 2;
  }
  const int rr = r - 4 * hh;   // diagonal: element e dead when r - 4hh > crow(e, 0)
  float* const xmine = xch + w * NQS * 1024 + lane * 4;
  const float* const xother = xch + (w ^ 4) * NQS * 1024 + lane * 4;

  const int prow = lane / CPR, slot = lane % CPR;
  auto decode = [&](int t, int& hq, int& qs) __attribute__((always_inline)) {
    hq = hk * grp + t / ph;
    qs = (qt0 + t % ph) * QT;
  };
  auto issue = [&](char* qd, char* od, float* ld, float* dd, int t) __attribute__((always_inline)) {
    int hq, qs;
    decode(t, hq, qs);
    const uint16_t* qb_ = q + (size_t)b * S * ldq + hq * D;
    const uint16_t* ob_ = dout + (size_t)b * S * lddo + hq * D;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = w + 8 * i;                 // 0 .. 2*PIECES-1: Q pieces then dO pieces
      const bool isq = p < PIECES;
      const int pp = isq ? p : p - PIECES;
      const int R = pp * RPP + prow;
      const int row = min(qs + R, S - 1);
      const int ch = slot ^ swz<D>(R);
      if (isq) dma16(qb_ + (size_t)row * ldq + ch * 8, qd + pp * 1024);
      else dma16(ob_ + (size_t)row * lddo + ch * 8, od + pp * 1024);
    }
    if (w < 2) {
      const size_t li = ((size_t)b * Hq + hq) * S + min(qs + lane, S - 1);
      if (w == 0) dma4(lse + li, (char*)ld);
      else dma4(delta + li, (char*)dd);
    }
  };
  auto dmload = [&](int t) __attribute__((always_inline)) -> uint32_t {
    if (!DROP || !wave_on) return 0u;
    int hq, qs;
    decode(t, hq, qs);
    return dbits[(((size_t)(b * Hq + hq) * NB + (kw0 >> 5)) * NQT + (qs >> 6)) * 64 + lane];
  };
  uint32_t dm_cur = 0, dm_next = 0;

  auto compute = [&](const char* Qt, const char* Ot, const float* Lt, const float* Dt, int t)
      __attribute__((always_inline)) {
    int hq, qs;
    decode(t, hq, qs);
    (void)hq;
    bool act[NQS];
    f32x16 acc[NQS];
#pragma unroll
    for (int u = 0; u < NQS; ++u) {
      const int qsu = qs + 32 * u;
      act[u] = uni(wave_on && qsu < S && (!CAUSAL || qsu + 31 >= kw0) ? 1 : 0);
    }
    // S^T (team 0) / dP^T (team 1) of every subtile first: the MFMAs of subtile u + 1 can
    // run under the vector work of subtile u
    const char* X = team == 0 ? Qt : Ot;
#pragma unroll
    for (int u = 0; u < NQS; ++u) {
      acc[u] = f32x16{};
      if (act[u]) {
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) acc[u] = mfma32(lds8(X + 32 * u * RB, offQ[kk]), kv[kk], acc[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < NQS; ++u) {
      if (!act[u]) continue;
      const int qsu = qs + 32 * u;
      if (team == 0) {
        // P of the subtile; the causal diagonal (wave-uniform branch) and, in RAGGED
        // launches only, the query tail / invalid keys are zeroed afterwards
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          float4 lsq;
          if ((e & 3) == 0) lsq = *reinterpret_cast<const float4*>(Lt + 32 * u + 8 * (e >> 2) + 4 * hh);
          const float lse_e = (e & 3) == 0 ? lsq.x : (e & 3) == 1 ? lsq.y : (e & 3) == 2 ? lsq.z : lsq.w;
          acc[u][e] = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[u][e], c, -lse_e));
        }
        if (uni(CAUSAL && qsu == kw0 ? 1 : 0)) {
          asm volatile("" ::: "memory");   // a real (scalar) branch, not per-element selects
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[u][e] = rr > crow(e, 0) ? 0.f : acc[u][e];
        }
        if constexpr (RAGGED) {
          const bool qtail = qsu + 32 > S;
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            if (qtail) acc[u][e] = qsu + crow(e, hh) >= S ? 0.f : acc[u][e];
            acc[u][e] = key_ok ? acc[u][e] : 0.f;
          }
        }
      } else {
        // x = (keep ? dP : 0) - delta
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          float4 dlq;
          if ((e & 3) == 0) dlq = *reinterpret_cast<const float4*>(Dt + 32 * u + 8 * (e >> 2) + 4 * hh);
          const float dl_e = (e & 3) == 0 ? dlq.x : (e & 3) == 1 ? dlq.y : (e & 3) == 2 ? dlq.z : dlq.w;
          float x = acc[u][e];
          if (DROP) x = __uint_as_float(__float_as_uint(x) & elem_keep(dm_cur, 8 * ((qsu >> 5) & 1), e));
          acc[u][e] = x - dl_e;
        }
      }
#pragma unroll
      for (int ch = 0; ch < 4; ++ch)
        *reinterpret_cast<float4*>(xmine + u * 1024 + ch * 256) =
            make_float4(acc[u][4 * ch], acc[u][4 * ch + 1], acc[u][4 * ch + 2], acc[u][4 * ch + 3]);
    }
    __syncthreads();   // every wave, active or not: the barrier counts of all waves match
#pragma unroll
    for (int u = 0; u < NQS; ++u) {
      if (!act[u]) continue;
      const int qsu = qs + 32 * u;
      float o[16];
#pragma unroll
      for (int ch = 0; ch < 4; ++ch) {
        const float4 f = *reinterpret_cast<const float4*>(xother + u * 1024 + ch * 256);
        o[4 * ch] = f.x; o[4 * ch + 1] = f.y; o[4 * ch + 2] = f.z; o[4 * ch + 3] = f.w;
      }
      f32x16 pd, ds;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float p = team == 0 ? acc[u][e] : o[e];
        const float x = team == 0 ? o[e] : acc[u][e];
        ds[e] = p * x;   // dS (1/(1-p) in dkscale)
        pd[e] = DROP ? __uint_as_float(__float_as_uint(p) & elem_keep(dm_cur, 8 * ((qsu >> 5) & 1), e)) : p;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pb = pack8(pd, 8 * s);
        const bf16x8 db = pack8(ds, 8 * s);
        const int rofs = (32 * u + 16 * s) * RB;
#pragma unroll
        for (int dt = 0; dt < NDL; ++dt) {
          const bf16x8 dot = cat(tr_read(Ot + rofs, offT[dt][0]), tr_read(Ot + rofs, offT[dt][1]));
          dvacc[dt] = mfma32(dot, pb, dvacc[dt]);
          const bf16x8 qtr = cat(tr_read(Qt + rofs, offT[dt][0]), tr_read(Qt + rofs, offT[dt][1]));
          dkacc[dt] = mfma32(qtr, db, dkacc[dt]);
        }
      }
    }
  };

  auto step = [&](char* Qc, char* Oc, float* Lc, float* Dc, char* Qn, char* On, float* Ln, float* Dn,
                  int t) __attribute__((always_inline)) {
    vm_drain();
    __syncthreads();
    if (t + 1 < cnt) {
      issue(Qn, On, Ln, Dn, t + 1);
      dm_next = dmload(t + 1);
    }
    compute(Qc, Oc, Lc, Dc, t);
    dm_cur = dm_next;
  };
  if (cnt > 0) {
    issue(q0, o0, l0, d0, 0);
    dm_cur = dmload(0);
  }
  for (int t = 0; t < cnt; t += 2) {
    step(q0, o0, l0, d0, q1, o1, l1, d1, t);
    if (t + 1 < cnt) step(q1, o1, l1, d1, q0, o0, l0, d0, t + 1);
  }

  if (!(key < S)) return;
  uint16_t* dkp = dk + (size_t)(b * S + key) * lddk + hk * D;
  uint16_t* dvp = dv + (size_t)(b * S + key) * lddv + hk * D;
#pragma unroll
  for (int dt = 0; dt < NDL; ++dt) {
    store_row32(dkp + 32 * (dt + DT0), dkacc[dt], dkscale, hh);
    store_row32(dvp + 32 * (dt + DT0), dvacc[dt], dvscale, hh);
  }
  if (bpart) {   // dK / dV bias-gradient column partials (S % 32 == 0)
    bias_partial_store<NDL>(dkacc, dkscale, bpart, ldbp, (b * S + kw0) >> 5, bcol + hk * D, DT0, lane);
    bias_partial_store<NDL>(dvacc, dvscale, bpart, ldbp, (b * S + kw0) >> 5, bcol + (Hkv + hk) * D, DT0, lane);
  }
}

// ------------------------------------------------------------------------------ launch
// key-tile rows of the D 64 query-major kernels (rocprofv3, GPT-2 shapes, dropout 0.1, one
// box: forward 25.8 us at 64 / 24.4 at 128; dQ 32.5 at 64 / 34.0 at 128 -- the dQ step
// holds S, dP and dQ^T, and its longer per-tile chain already covers the next tile's DMA)
int g_qbk_fwd = 128, g_qbk_dq = 64;
// D 128 dK/dV: 0 = single-pass 8-wave kernel (default), 1 = the two column-half passes
// (bit-identical; kept for the equality test and A/B runs).  Measured and dropped (GPT-3
// shapes, dropout 0.1, one MI355X, profiles/r3_s4): static s_setprio 1 for the team-1 half
// 280.1 vs 280.2 us; a ping-pong schedule (teams offset by one of four barrier-separated
// segments per tile, 3-slot ring) 452.7 vs 275.3 us -- four barriers per 32-row tile cost
// more than the matrix / vector pairing recovers, and it spilled at 256 VGPRs.
int g_kmajor128_variant = 0;

template <int D, bool DQ>
hipError_t launch_qmajor(bool causal, bool drop, int S, int B, hipStream_t s,
                         const uint16_t* q, const uint16_t* k, const uint16_t* v, int ldq, int ldk,
                         int ldv, const uint16_t* dout, int lddo, uint16_t* o, int ldo, float* lse,
                         float* delta, uint16_t* dq, int lddq, int Hq, int Hkv,
                         const int* klen, float c, float oscale, float dkeep,
                         const uint64_t* dbits, int NB, int NKT, float* bpart = nullptr, int ldbp = 0,
                         const DGen* dgen = nullptr) {
  constexpr bool PAIR = D == 64;
  const int nqb = (S + 127) / 128;
  const dim3 grid((PAIR ? (nqb + 1) / 2 : nqb) * Hq * B);
  const DGen dg = dgen ? *dgen : DGen{nullptr, 0u, 0u, 0, 0};
#define MX_QM(C, DR, BKT)                                                                              \
  do {                                                                                                 \
    if constexpr (!DQ && DR && D == 64) {                                                              \
      if (dgen) {                                                                                      \
        hipLaunchKernelGGL((flash_qmajor_kernel<D, C, DR, DQ, PAIR, BKT, true>), grid,                 \
                           dim3(PAIR ? 512 : 256), 0, s, q, k, v, ldq, ldk, ldv, dout, lddo, o, ldo,     \
                           lse, delta, dq, lddq, S, Hq, Hkv, klen, c, oscale, dkeep, dbits, NB, NKT,     \
                           bpart, ldbp, dg);                                                           \
        break;                                                                                         \
      }                                                                                                \
    }                                                                                                  \
    hipLaunchKernelGGL((flash_qmajor_kernel<D, C, DR, DQ, PAIR, BKT>), grid, dim3(PAIR ? 512 : 256),    \
                       0, s, q, k, v, ldq, ldk, ldv, dout, lddo, o, ldo, lse, delta, dq, lddq, S, Hq,    \
                       Hkv, klen, c, oscale, dkeep, dbits, NB, NKT, bpart, ldbp, dg);                  \
  } while (0)
#define MX_QM_B(BKT)                                                          \
  {                                                                           \
    if (causal) { if (drop) MX_QM(true, true, BKT); else MX_QM(true, false, BKT); } \
    else { if (drop) MX_QM(false, true, BKT); else MX_QM(false, false, BKT); }    \
  }
  // D 64 forward: 128-key tiles (half the steps, each with twice the compute under the
  // next tile's DMA; the GPT-2 shapes run only ~9 dependent steps per team).  D 128 keeps
  // 64 (two waves per SIMD need the registers).
  if constexpr (PAIR) {
    if ((DQ ? g_qbk_dq : g_qbk_fwd) == 128) MX_QM_B(128)
    else MX_QM_B(64)
  } else {
    MX_QM_B(64)
  }
#undef MX_QM_B
#undef MX_QM
  return hipGetLastError();
}

template <int D>
hipError_t launch_kmajor(bool causal, bool drop, int S, int B, hipStream_t s,
                         const uint16_t* q, const uint16_t* k, const uint16_t* v, int ldq, int ldk,
                         int ldv, const uint16_t* dout, int lddo, const float* lse,
                         const float* delta, uint16_t* dk, uint16_t* dv, int lddk, int lddv,
                         int Hq, int Hkv, const int* klen, float c, float dkscale, float dvscale,
                         const uint32_t* dbits, int NB, int NQT, float* bpart, int ldbp, int bcol) {
  constexpr bool PAIR = D == 64;
  const int nkb = (S + 127) / 128;
  const dim3 grid((PAIR ? (nkb + 1) / 2 : nkb) * Hkv * B);
  // RAGGED: padded keys (klen) or a sequence that does not fill the last key block; the
  // common launch (every key valid, S a multiple of 128) carries no per-element key mask
  const bool ragged = klen != nullptr || S % 128 != 0;
#define MX_KM(C, DR, P)                                                                                  \
  do {                                                                                                   \
    if (ragged)                                                                                          \
      hipLaunchKernelGGL((flash_kmajor_kernel<D, C, DR, P, PAIR, true>), grid, dim3(PAIR ? 512 : 256), 0, \
                         s, q, k, v, ldq, ldk, ldv, dout, lddo, lse, delta, dk, dv, lddk, lddv, S, Hq,    \
                         Hkv, klen, c, dkscale, dvscale, dbits, NB, NQT, bpart, ldbp, bcol);              \
    else                                                                                                 \
      hipLaunchKernelGGL((flash_kmajor_kernel<D, C, DR, P, PAIR, false>), grid, dim3(PAIR ? 512 : 256), 0, \
                         s, q, k, v, ldq, ldk, ldv, dout, lddo, lse, delta, dk, dv, lddk, lddv, S, Hq,    \
                         Hkv, klen, c, dkscale, dvscale, dbits, NB, NQT, bpart, ldbp, bcol);              \
  } while (0)
#define MX_KM_P(P)                                                                   \
  {                                                                                  \
    if (causal) { if (drop) MX_KM(true, true, P); else MX_KM(true, false, P); }      \
    else { if (drop) MX_KM(false, true, P); else MX_KM(false, false, P); }           \
  }
  if constexpr (D <= 64) {
    MX_KM_P(0)
  } else if (g_kmajor128_variant == 1) {
    MX_KM_P(1)
    MX_KM_P(2)
  } else {
#define MX_K8(C, DR)                                                                                \
  do {                                                                                              \
    if (ragged)                                                                                     \
      hipLaunchKernelGGL((flash_kmajor128_kernel<C, DR, true>), grid, dim3(512), 0, s, q, k, v, ldq, \
                         ldk, ldv, dout, lddo, lse, delta, dk, dv, lddk, lddv, S, Hq, Hkv, klen, c, \
                         dkscale, dvscale, dbits, NB, NQT, bpart, ldbp, bcol);                      \
    else                                                                                            \
      hipLaunchKernelGGL((flash_kmajor128_kernel<C, DR, false>), grid, dim3(512), 0, s, q, k, v,    \
                         ldq, ldk, ldv, dout, lddo, lse, delta, dk, dv, lddk, lddv, S, Hq, Hkv,     \
                         klen, c, dkscale, dvscale, dbits, NB, NQT, bpart, ldbp, bcol);             \
  } while (0)
    if (causal) { if (drop) MX_K8(true, true); else MX_K8(true, false); }
    else { if (drop) MX_K8(false, true); else MX_K8(false, false); }
#undef MX_K8
  }
#undef MX_KM_P
#undef MX_KM
  return hipGetLastError();
}

}  // namespace

// key-tile rows (64 or 128) of the D 64 forward / dQ kernels; returns the old values
// (fwd * 1000 + dq).  A value of 0 keeps the current setting.
MX_EXPORT int mx_flash_qmajor_bk(int fwd, int dq) {
  const int old = g_qbk_fwd * 1000 + g_qbk_dq;
  if (fwd == 64 || fwd == 128) g_qbk_fwd = fwd;
  if (dq == 64 || dq == 128) g_qbk_dq = dq;
  return old;
}

// D 128 dK/dV kernel choice (g_kmajor128_variant); a negative value keeps the setting.
// Returns the old one.
MX_EXPORT int mx_flash_kmajor128_variant(int variant) {
  const int old = g_kmajor128_variant;
  if (variant == 0 || variant == 1) g_kmajor128_variant = variant;
  return old;
}

namespace {
// 0: the per-group grid (flash_dropmask_kernel), 1 (default): the wave-walk kernel
int g_dropmask_variant = 1;
int launch_dropmask(const uint32_t* seed, uint32_t salt, uint32_t thr16, int S, int Hq, int h_off, int Hg, int NB,
                    int NKT, int NQT, int causal, void* fwd_bits, void* bwd_bits, int BH, int L, long long fwd_words,
                    long long bwd_words, hipStream_t s) {
  const int NB2 = (NB + 1) / 2;
  if (g_dropmask_variant == 0) {
    if ((long long)BH * L > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(flash_dropmask_kernel, dim3(NB2, (NB2 + 3) / 4, BH * L), dim3(256), 0, s, seed, salt, thr16,
                       S, Hq, h_off, Hg, NB, NKT, NQT, causal, (uint32_t*)fwd_bits, (uint32_t*)bwd_bits, BH,
                       fwd_words, bwd_words);
    return hipGetLastError();
  }
  const long long per = causal ? (long long)NB2 * (NB2 + 1) / 2 : (long long)NB2 * NB2;
  const long long waves = per * BH * L;
  long long blocks = (waves + 3) / 4;
  if (blocks > 2048) blocks = 2048;   // 8 waves per CU, each walking its share of the groups
  hipLaunchKernelGGL(flash_dropmask_waves_kernel, dim3((unsigned)blocks), dim3(256), 0, s, seed, salt, thr16, S, Hq,
                     h_off, Hg, NB, NKT, NQT, causal, (uint32_t*)fwd_bits, (uint32_t*)bwd_bits, BH, L, fwd_words,
                     bwd_words);
  return hipGetLastError();
}
}  // namespace

// dropout-mask kernel choice (0 per-group grid, 1 wave walk); returns the previous setting
MX_EXPORT int mx_flash_dropmask_variant(int v) {
  const int old = g_dropmask_variant;
  if (v >= 0) g_dropmask_variant = v;
  return old;
}

// Dropout keep-mask images for one attention call (layouts in flash_dropmask_kernel).
// fwd_bits: u64 [B*Hq][NB][NKT][64]; bwd_bits: u32 [B*Hq][NB][NQT][64], NB = ceil(S/32),
// NKT = ceil(S/128), NQT = ceil(S/64).  h_off / Hg: this rank's first global head / the
// model's head count (tensor/context-parallel shards draw the single-GPU mask).
MX_EXPORT int mx_flash_dropmask(const uint32_t* seed, uint32_t salt, float p, int B, int S,
                                int Hq, int h_off, int Hg, int causal, void* fwd_bits,
                                void* bwd_bits, hipStream_t s) {
  const int NB = (S + 31) / 32, NKT = (S + 127) / 128, NQT = (S + 63) / 64;
  const int NB2 = (NB + 1) / 2;
  const uint32_t thr16 = (uint32_t)(p * 65536.0f + 0.5f);
  return launch_dropmask(seed, salt, thr16, S, Hq, h_off, Hg, NB, NKT, NQT, causal, fwd_bits, bwd_bits, B * Hq, 1,
                         0ll, 0ll, s);
}

// the images of L layers (salts salt, salt + 1, ...) in one launch; layer l's images start
// at fwd_bits + l * fwd_words (uint32 words) and bwd_bits + l * bwd_words
MX_EXPORT int mx_flash_dropmask_layers(const uint32_t* seed, uint32_t salt, float p, int B, int S, int Hq,
                                       int h_off, int Hg, int causal, int L, void* fwd_bits, void* bwd_bits,
                                       long long fwd_words, long long bwd_words, hipStream_t s) {
  if (L < 1) return hipErrorInvalidValue;
  const int NB = (S + 31) / 32, NKT = (S + 127) / 128, NQT = (S + 63) / 64;
  const int NB2 = (NB + 1) / 2;
  const uint32_t thr16 = (uint32_t)(p * 65536.0f + 0.5f);
  return launch_dropmask(seed, salt, thr16, S, Hq, h_off, Hg, NB, NKT, NQT, causal, fwd_bits, bwd_bits, B * Hq, L,
                         fwd_words, bwd_words, s);
}

// Q/K/V/O bf16 with token strides ld*; head h at column h*D.  lse: fp32 [B, Hq, S] (base 2).
// klen: int32 [B] valid key count or null.  fwd_bits: dropout image or null; keep_scale =
// 1/(1-p).
MX_EXPORT int mx_flash_fwd(const void* q, const void* k, const void* v, int ldq, int ldk, int ldv,
                           void* o, int ldo, float* lse, int B, int S, int Hq, int Hkv, int D,
                           int causal, const int* klen, float scale, const void* fwd_bits,
                           float keep_scale, hipStream_t s) {
  if (Hq % Hkv || S <= 0) return hipErrorInvalidValue;
  const float c = scale * 1.4426950408889634f;
  const int NB = (S + 31) / 32, NKT = (S + 127) / 128;
  const bool drop = fwd_bits != nullptr;
  const float osc = drop ? keep_scale : 1.f;
  if (D == 64)
    return launch_qmajor<64, false>(causal, drop, S, B, s, (const uint16_t*)q, (const uint16_t*)k,
                                    (const uint16_t*)v, ldq, ldk, ldv, nullptr, 0, (uint16_t*)o, ldo,
                                    lse, nullptr, nullptr, 0, Hq, Hkv, klen, c, osc, 1.f,
                                    (const uint64_t*)fwd_bits, NB, NKT);
  if (D == 128)
    return launch_qmajor<128, false>(causal, drop, S, B, s, (const uint16_t*)q, (const uint16_t*)k,
                                     (const uint16_t*)v, ldq, ldk, ldv, nullptr, 0, (uint16_t*)o, ldo,
                                     lse, nullptr, nullptr, 0, Hq, Hkv, klen, c, osc, 1.f,
                                     (const uint64_t*)fwd_bits, NB, NKT);
  return hipErrorInvalidValue;
}

// A/B only (profiles/r6/attn_inkernel_dropout_ab.txt): the forward with its keep bits hashed
// in-kernel from (seed, salt, p, h_off, Hg) instead of read from the pre-pass image.  Output
// bit-identical to mx_flash_fwd with the image of mx_flash_dropmask(seed, salt, p, ...).
MX_EXPORT int mx_flash_fwd_dgen(const void* q, const void* k, const void* v, int ldq, int ldk, int ldv,
                                void* o, int ldo, float* lse, int B, int S, int Hq, int Hkv, int D, int causal,
                                const int* klen, float scale, const uint32_t* seed, uint32_t salt, float p,
                                int h_off, int Hg, hipStream_t s) {
  if (Hq % Hkv || S <= 0 || D != 64 || !(p > 0.f) || seed == nullptr) return hipErrorInvalidValue;
  const float c = scale * 1.4426950408889634f;
  const int NB = (S + 31) / 32, NKT = (S + 127) / 128;
  const DGen dg{seed, salt, (uint32_t)(p * 65536.0f + 0.5f), h_off, Hg};
  return launch_qmajor<64, false>(causal, true, S, B, s, (const uint16_t*)q, (const uint16_t*)k,
                                  (const uint16_t*)v, ldq, ldk, ldv, nullptr, 0, (uint16_t*)o, ldo, lse, nullptr,
                                  nullptr, 0, Hq, Hkv, klen, c, (float)(65536.0 / (65536.0 - dg.thr16)), 1.f, nullptr, NB, NKT, nullptr,
                                  0, &dg);
}

// delta: fp32 [B, Hq, S] workspace (written by the dQ kernel, read by the dK/dV kernel).
// fwd_bits / bwd_bits: the forward's dropout images (both null without dropout).
MX_EXPORT int mx_flash_bwd(const void* q, const void* k, const void* v, int ldq, int ldk, int ldv,
                           const void* o, int ldo, const void* dout, int lddo, const float* lse,
                           float* delta, void* dq, int lddq, void* dk, void* dv, int lddk,
                           int lddv, int B, int S, int Hq, int Hkv, int D, int causal,
                           const int* klen, float scale, const void* fwd_bits,
                           const void* bwd_bits, float keep_scale, float* bias_part, int ldbp,
                           hipStream_t s) {
  if (Hq % Hkv || S <= 0 || (D != 64 && D != 128)) return hipErrorInvalidValue;
  // bias-gradient partials need whole 32-row groups and room for [dq | dk | dv] columns
  if (bias_part && (S % 32 || ldbp < (Hq + 2 * Hkv) * D)) return hipErrorInvalidValue;
  if ((fwd_bits == nullptr) != (bwd_bits == nullptr)) return hipErrorInvalidValue;
  const float c = scale * 1.4426950408889634f;
  const bool drop = fwd_bits != nullptr;
  const float ks = drop ? keep_scale : 1.f;
  const float dkeep = drop ? 1.f / keep_scale : 1.f;
  const int NB = (S + 31) / 32, NKT = (S + 127) / 128, NQT = (S + 63) / 64;
  hipError_t e;
  if (D == 64)
    e = launch_qmajor<64, true>(causal, drop, S, B, s, (const uint16_t*)q, (const uint16_t*)k,
                                (const uint16_t*)v, ldq, ldk, ldv, (const uint16_t*)dout, lddo,
                                (uint16_t*)o, ldo, (float*)lse, delta, (uint16_t*)dq, lddq, Hq, Hkv,
                                klen, c, scale * ks, dkeep, (const uint64_t*)fwd_bits, NB, NKT, bias_part,
                                ldbp);
  else
    e = launch_qmajor<128, true>(causal, drop, S, B, s, (const uint16_t*)q, (const uint16_t*)k,
                                 (const uint16_t*)v, ldq, ldk, ldv, (const uint16_t*)dout, lddo,
                                 (uint16_t*)o, ldo, (float*)lse, delta, (uint16_t*)dq, lddq, Hq, Hkv,
                                 klen, c, scale * ks, dkeep, (const uint64_t*)fwd_bits, NB, NKT, bias_part,
                                 ldbp);
  if (e != hipSuccess) return e;
  if (D == 64)
    e = launch_kmajor<64>(causal, drop, S, B, s, (const uint16_t*)q, (const uint16_t*)k,
                          (const uint16_t*)v, ldq, ldk, ldv, (const uint16_t*)dout, lddo, lse, delta,
                          (uint16_t*)dk, (uint16_t*)dv, lddk, lddv, Hq, Hkv, klen, c, scale * ks, ks,
                          (const uint32_t*)bwd_bits, NB, NQT, bias_part, ldbp, Hq * D);
  else
    e = launch_kmajor<128>(causal, drop, S, B, s, (const uint16_t*)q, (const uint16_t*)k,
                           (const uint16_t*)v, ldq, ldk, ldv, (const uint16_t*)dout, lddo, lse, delta,
                           (uint16_t*)dk, (uint16_t*)dv, lddk, lddv, Hq, Hkv, klen, c, scale * ks, ks,
                           (const uint32_t*)bwd_bits, NB, NQT, bias_part, ldbp, Hq * D);
  return e;
}
