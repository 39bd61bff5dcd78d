// Flash attention forward + backward for gfx950 (CDNA4), bf16 in/out, fp32 softmax.
//
// Replaces the Megatron fused `scaled_upper_triang_masked_softmax` + two batched
// GEMMs (GPT, causal) and the HF BERT padded-softmax attention the reference runs
// upstream (containers/megatron-deepspeed/Dockerfile:13, examples/accelerate/
// bert-glue-mrpc/pretrain.yaml:45).  No S x S matrix is ever
// materialised.
//
// Layout: Q/K/V are read in place from the packed QKV projection output
// ([tokens, 3, heads, D] with a token stride), O is written [tokens, heads, D], so the
// model needs no transposes.  lse is base-2: lse2 = max*c + log2(sum), c = scale*log2(e).
//
// Forward (one workgroup = 8 waves = two 128-row query blocks of one (batch, head) --
// for causal masks the mirrored pair (i, n-1-i), so every workgroup does identical work
// and the grid is one workgroup per CU; K/V tiles of 64 keys double-buffered in LDS by
// register staging, T14, shared by both halves):
//   S^T = K * Q^T with v_mfma_f32_32x32x16_bf16 ("swapped" product: the query is on
//   the lane, so the row max / row sum are lane-local plus one lane^32 exchange);
//   O^T = V^T * P^T where the P accumulator registers feed the B operand directly
//   (cdna_hip_programming.md §3 "accumulator tile as the next MFMA's operand") and V^T
//   fragments come from ds_read_b64_tr_b16 (T10).  O stays query-on-lane, so the
//   online-softmax rescale is lane-local.
// Backward (one workgroup = 8 waves = 256 keys, again a mirrored causal pair of 128-key
// blocks; each wave keeps dK^T/dV^T of its 32 keys in accumulators while sweeping 32-row
// query tiles): S and dP are computed key-on-lane with -lse and -delta preloaded into
// the accumulators, so P and dS are ready-made B operands of dV^T += dO^T P and
// dK^T += Q^T dS; dS crosses LDS once for dQ = dS K (v_mfma_f32_16x16x32_bf16) over all
// 256 keys, staged through LDS and summed over key blocks with row-contiguous fp32
// global atomics (one 256-B wave-instruction per row: the full-rate shape of
// MI355X_MICROARCH.md "Global float atomics"), converted to bf16 once.
//
// Attention dropout (Megatron --attention-dropout, HF attention_probs_dropout_prob): the
// keep-mask M[b,h,q,k] is a pure function of (seed, global row, key) --
//   keep <=> ((hash32(row * 0x85EBCA6B + (k >> 1), seed) >> 16 * (k & 1)) & 0xFFFF) >= thr16,
//   row = (b * Hg + h_global) * S + q
// (16-bit threshold: p is exact to 2^-16).  attn_dropmask_kernel evaluates it once per
// forward into two lane-bit images, one per MFMA accumulator layout: the forward's
// query-on-lane image (one 8-B word per lane per 128-key tile) and the backward's
// key-on-lane image (one 2-B word per lane per 32x32 block).  The main loops then pay two
// VALU ops per element (v_bfe_i32 + v_and on P); dS = P (Z dP~ - delta) with Z = M/(1-p)
// is formed with one v_bfi per element from a -delta(1-p) accumulator preload, and the
// 1/(1-p) factors are folded into the O / dK / dV / dQ epilogue scales.
//
// Every LDS tile uses a 16-B chunk XOR swizzle chosen so that both the row reads
// (ds_read_b128 of 32 different rows) and the transposed reads (4 consecutive rows x
// 32 columns per half-wave) are bank-conflict free (derivation in Swz below).
#include "common.h"

using namespace mx;

namespace {

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// Chunk swizzle for a [rows][D] bf16 tile (D*2-byte rows, 16-B chunks).
//  D=64 (128-B rows, two rows per 256-B bank row): f = x ^ ((x&1)<<2), x = (row>>1)&7
//    - rows {0-3,12-15,20-27} (one ds_read_b128 lane group) map to distinct slots
//    - rows R..R+3 (R%4==0) read transposed over 4 chunks land in disjoint chunk quads
//  D=128 (256-B rows): f = ((row&3)<<2) | ((row>>2)&3)
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
// Swizzle for the backward K tile, read only transposed by 8 rows {R..R+3, R+8..R+11}
// x 2 chunks per half-wave (the 16x16x32 B operand of dQ = dS K).
template <int D>
__device__ __forceinline__ int toff_k(int row, int chunk) {
  int f;
  if constexpr (D == 64) f = (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2);
  else f = ((row & 3) << 1) | (((row >> 3) & 1) << 3);
  return row * (D * 2) + ((chunk ^ f) << 4);
}

// dS^T image [keys][32 q] bf16 (64-B rows): XOR of the 8-B unit with key bits {3, 2, 1^3}
// makes both the 16-row ds_write_b64 groups and the transposed dQ-operand reads
// conflict-free (checked by scripts/lds_banks.py).
__device__ __forceinline__ int ds_off(int krow, int qbytes) {
  const int f = ((krow >> 3) & 1) | (((krow >> 2) & 1) << 1) | ((((krow >> 1) ^ (krow >> 3)) & 1) << 2);
  return krow * 64 + ((((qbytes >> 3) ^ f) << 3) | (qbytes & 7));
}

__device__ __forceinline__ bf16x4 tr_read(const char* lds, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(lds + byte_off));
}
__device__ __forceinline__ bf16x8 cat(bf16x4 a, bf16x4 b) {
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
__device__ __forceinline__ bf16x8 pack_acc8(const f32x16& acc, int base) {
  uint4 u;
  u.x = pack2(acc[base + 0], acc[base + 1]);
  u.y = pack2(acc[base + 2], acc[base + 3]);
  u.z = pack2(acc[base + 4], acc[base + 5]);
  u.w = pack2(acc[base + 6], acc[base + 7]);
  return __builtin_bit_cast(bf16x8, u);
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
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ============================================================================ dropout mask
// One wave per 32x32 (query block, key block).  Lane (r, hh) owns query 32qb + r and, in
// the forward image, keys crow(e, hh) = (e&3) + 8(e>>2) + 4hh of the block (e = 0..15, the
// 32x32 accumulator rows of a lane); its 16 keep bits are 8 hashes.  The backward image
// (lane = key, e -> query crow(e, hh)) is the transpose, formed through LDS.
__device__ __forceinline__ int crow(int e, int hh) { return (e & 3) + 8 * (e >> 2) + 4 * hh; }

__global__ __launch_bounds__(64) void attn_dropmask_kernel(
    const uint32_t* __restrict__ seed_ptr, uint32_t salt, uint32_t thr16, int S, int Hq,
    int h_off, int Hg, int NB, int NKT, int causal, uint16_t* __restrict__ fwd_bits,
    uint16_t* __restrict__ bwd_bits) {
  const int qb = blockIdx.x, kb = blockIdx.y, bh = blockIdx.z;
  if (causal && kb > qb) return;  // never read (whole block above the diagonal)
  const int b = bh / Hq, h = bh - b * Hq;
  const uint32_t seed = *seed_ptr + salt;
  const int lane = threadIdx.x, r = lane & 31, hh = lane >> 5;
  const uint32_t row = (uint32_t)(((long long)b * Hg + h_off + h) * S + qb * 32 + r);
  const uint32_t rbase = row * 0x85EBCA6Bu;
  uint32_t fbits = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const uint32_t kp = (uint32_t)(kb * 16 + 4 * j + 2 * hh + half);
      const uint32_t hv = hash32(rbase + kp, seed);
      const int e = 4 * j + 2 * half;
      fbits |= (uint32_t)((hv & 0xFFFFu) >= thr16) << e;
      fbits |= (uint32_t)((hv >> 16) >= thr16) << (e + 1);
    }
  // forward image: [bh][qb][kt = kb/4][lane] u64, 16 bits per key block (kb % 4)
  fwd_bits[((((size_t)bh * NB + qb) * NKT + (kb >> 2)) * 64 + lane) * 4 + (kb & 3)] = (uint16_t)fbits;
  __shared__ uint16_t fw[64];
  fw[lane] = (uint16_t)fbits;
  __syncthreads();
  // backward image: lane = key kl; element e = query crow(e, hh) -> forward lane
  // crow(e, hh) + 32 * ((kl >> 2) & 1), forward bit (kl & 3) + 4 (kl >> 3)
  const int kl = r;
  const int fbit = (kl & 3) + 4 * (kl >> 3), fhi = 32 * ((kl >> 2) & 1);
  uint32_t bbits = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) bbits |= (((uint32_t)fw[crow(e, hh) + fhi] >> fbit) & 1u) << e;
  bwd_bits[(((size_t)bh * NB + kb) * NB + qb) * 64 + lane] = (uint16_t)bbits;
}

// p if element bit `bit` of `m` is set, else +0 (v_bfe_i32 + v_and)
__device__ __forceinline__ float keep_or_zero(float p, uint32_t m, int bit) {
  return __uint_as_float(__float_as_uint(p) & (uint32_t)__builtin_amdgcn_sbfe((int)m, (uint32_t)bit, 1u));
}
// x if the bit is set else y (v_bfe_i32 + v_bfi_b32)
__device__ __forceinline__ float keep_sel(float x, float y, uint32_t m, int bit) {
  const uint32_t mk = (uint32_t)__builtin_amdgcn_sbfe((int)m, (uint32_t)bit, 1u);
  return __uint_as_float((__float_as_uint(x) & mk) | (__float_as_uint(y) & ~mk));
}

// ============================================================================ forward
// Workgroup = 8 waves = two 128-row query blocks.  Causal: the pair (i, nqb-1-i), so every
// workgroup does the same number of K/V tiles (light block + its mirrored heavy block)
// and the grid is exactly one workgroup per CU with no tail; the two halves share every
// K/V tile staged in LDS.  Non-causal: blocks (2i, 2i+1).
template <int D, bool CAUSAL, bool DROP>
// waves_per_eu(2,2): one 8-wave workgroup per CU is the design point, so let the
// scheduler spend the full 256-VGPR budget on read batching instead of occupancy.
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn_fwd_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, int ldq, int ldk, int ldv, uint16_t* __restrict__ o,
    int ldo, float* __restrict__ lse, int S, int Hq, int Hkv, const int* __restrict__ klen,
    float c /* scale*log2(e) */, const uint64_t* __restrict__ dbits, int NB, int NKT,
    float oscale /* 1/(1-p) */) {
  // 128-key K/V tiles: one tile of compute per wave must cover the HBM latency of the
  // next tile's register-staged prefetch (64-key tiles left the loop latency-bound)
  constexpr int BQ = 128, BK = 128, NSUB = BK / 32, NKK = D / 16, NDT = D / 32;
  constexpr int TILE = BK * D * 2;           // bytes of one K (or V) tile
  constexpr int CPR = D / 8;                 // 16-B chunks per row
  constexpr int CH = BK * CPR / 512;         // chunks per thread per tile
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wl = w & 3, half = w >> 2;
  const int r = lane & 31, hh = lane >> 5, g = lane >> 4, gi = lane & 15;
  const int nqb = (S + BQ - 1) / BQ;
  const int pair = blockIdx.x;
  int qb_mine, qb_other;
  if (CAUSAL) {
    const int a = pair, bq = nqb - 1 - pair;
    qb_mine = half ? bq : a;
    qb_other = half ? a : bq;
  } else {
    qb_mine = 2 * pair + half;
    qb_other = 2 * pair + (half ^ 1);
  }
  const bool half_on = qb_mine < nqb && !(CAUSAL && half == 1 && qb_mine == qb_other);
  const int hq = blockIdx.y, b = blockIdx.z;
  const int hk = hq / (Hq / Hkv);
  const int qw = qb_mine * BQ + 32 * wl;
  const int kl = klen ? klen[b] : S;
  const int qrow = qw + r;

  bf16x8 qf[NKK];
  {
    const uint16_t* qp = q + (size_t)(b * S + qrow) * ldq + hq * D + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk)
      qf[kk] = (half_on && qrow < S) ? ld8(qp + 16 * kk) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  int kv_end = kl;
  if (CAUSAL) {
    const int last_q = (max(qb_mine, qb_other < nqb ? qb_other : 0) + 1) * BQ;
    kv_end = min(kv_end, min(S, last_q));
  }
  const int nt = (kv_end + BK - 1) / BK;

  const uint16_t* kbase = k + (size_t)b * S * ldk + hk * D;
  const uint16_t* vbase = v + (size_t)b * S * ldv + hk * D;
  // Staging: rows past S are clamped to S-1 (their scores are masked to -inf, so the
  // duplicate rows only need to be finite) -> unconditional 16-B loads, no exec branches.
  // Staging registers are named scalars (k0..k3 / v0..v3), not arrays: hipcc promoted the
  // uint4 arrays to LDS / scratch instead of registers.
  static_assert(CH == 2 || CH == 4, "staging assumes 2 or 4 chunks per thread");
  uint4 k0, k1, k2, k3, v0, v1, v2, v3;
  const int srow = tid / CPR, sch = tid % CPR;       // chunk i: row srow + i*512/CPR
  constexpr int RSTEP = 512 / CPR;
  const int so0 = toff<D>(srow, sch), so1 = toff<D>(srow + RSTEP, sch);
  const int so2 = toff<D>(srow + 2 * RSTEP, sch), so3 = toff<D>(srow + 3 * RSTEP, sch);
#define FWD_LD1(I, T)                                                                    \
  {                                                                                      \
    const int key = min((T) * BK + srow + (I) * RSTEP, S - 1);                           \
    k##I = *reinterpret_cast<const uint4*>(kbase + (size_t)key * ldk + sch * 8);         \
    v##I = *reinterpret_cast<const uint4*>(vbase + (size_t)key * ldv + sch * 8);         \
  }
#define FWD_ST1(I, BUF)                                                                  \
  {                                                                                      \
    *reinterpret_cast<uint4*>(smem + (BUF) * 2 * TILE + so##I) = k##I;                   \
    *reinterpret_cast<uint4*>(smem + (BUF) * 2 * TILE + TILE + so##I) = v##I;            \
  }
#define FWD_GLOAD(T)                                                                     \
  {                                                                                      \
    FWD_LD1(0, T) FWD_LD1(1, T)                                                          \
    if constexpr (CH == 4) { FWD_LD1(2, T) FWD_LD1(3, T) }                               \
  }
#define FWD_SWRITE(BUF)                                                                  \
  {                                                                                      \
    FWD_ST1(0, BUF) FWD_ST1(1, BUF)                                                      \
    if constexpr (CH == 4) { FWD_ST1(2, BUF) FWD_ST1(3, BUF) }                           \
  }

  float m_i = -INFINITY, l_i = 0.f;
  f32x16 oacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) oacc[dt] = f32x16{};

  // dropout bits of this lane's query row: one 8-B word per 128-key tile (4 x 16 bits)
  const uint64_t* dmrow = DROP ? dbits + ((size_t)(b * Hq + hq) * NB + (qw >> 5)) * NKT * 64 + lane : nullptr;
  uint64_t dm_cur = 0, dm_next = 0;
  if constexpr (DROP) {
    if (nt > 0 && half_on && qw < S) dm_cur = dmrow[0];
  }
  if (nt > 0) {
    FWD_GLOAD(0);
    FWD_SWRITE(0);
  }
  __syncthreads();
  for (int j = 0; j < nt; ++j) {
    const char* Kt = smem + (j & 1) * 2 * TILE;
    const char* Vt = Kt + TILE;
    const int kv0 = j * BK;
    // causal: 32-key subtiles past this wave's last query are skipped outright
    // (wave-uniform), so a 128-key tile costs only the subtiles it really needs
    int nsub = NSUB;
    if (CAUSAL) nsub = min(NSUB, max(0, (qw + 31 - kv0) / 32 + 1));
    const bool active = half_on && qw < S && nsub > 0;
    f32x16 sacc[NSUB];
    if (active) {
#pragma unroll
      for (int t = 0; t < NSUB; ++t) {
        if (t < nsub) {
          bf16x8 kr[NKK];  // batch the subtile's K fragment reads ahead of its MFMAs
#pragma unroll
          for (int kk = 0; kk < NKK; ++kk) kr[kk] = lds8(Kt, toff<D>(32 * t + r, 2 * kk + hh));
          sacc[t] = f32x16{};
#pragma unroll
          for (int kk = 0; kk < NKK; ++kk) sacc[t] = mfma32(kr[kk], qf[kk], sacc[t]);
        }
      }
    }
    // T14: the next tile's global loads are issued only after QK^T, so their latency
    // hides under softmax + PV and no wait lands in front of the first MFMA
    if (j + 1 < nt) {
      FWD_GLOAD(j + 1);
      if constexpr (DROP) {
        if (half_on && qw < S && (!CAUSAL || qw + 31 >= (j + 1) * BK)) dm_next = dmrow[(size_t)(j + 1) * 64];
      }
    }
    if (active) {
      const bool need_mask = (CAUSAL && kv0 + 32 * nsub - 1 > qw) || (kv0 + BK > kl);
      if (need_mask) {
#pragma unroll
        for (int t = 0; t < NSUB; ++t) {
          if (t < nsub) {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int key = kv0 + 32 * t + (e & 3) + 8 * (e >> 2) + 4 * hh;
              const bool dead = key >= kl || (CAUSAL && key > qrow);
              sacc[t][e] = dead ? -INFINITY : sacc[t][e];
            }
          }
        }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < NSUB; ++t)
        if (t < nsub) {
#pragma unroll
          for (int e = 0; e < 16; ++e) mx = fmaxf(mx, sacc[t][e]);
        }
      mx = xhalf_max(mx);
      // Exact deferred rescale (T13 with threshold 0): when no row of the wave raised its
      // running max, alpha == 1 for every lane and the O / l rescale is skipped outright.
      if (!__all(mx <= m_i)) {
        const float m_new = fmaxf(m_i, mx);
        const float alpha = m_new == -INFINITY ? 1.f : __builtin_amdgcn_exp2f((m_i - m_new) * c);
        l_i *= alpha;
        m_i = m_new;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int e = 0; e < 16; ++e) oacc[dt][e] *= alpha;
      }
      const float mc = m_i == -INFINITY ? 0.f : m_i * c;
      float rs = 0.f;
#pragma unroll
      for (int t = 0; t < NSUB; ++t)
        if (t < nsub) {
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const float p = __builtin_amdgcn_exp2f(sacc[t][e] * c - mc);
            rs += p;  // the normaliser sums the undropped probabilities
            sacc[t][e] = DROP ? keep_or_zero(p, (uint32_t)(dm_cur >> (16 * t)), e) : p;
          }
        }
      l_i += rs;
#pragma unroll
      for (int t = 0; t < NSUB; ++t)
        if (t < nsub) {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const int row0 = 32 * t + 16 * s + 4 * hh + (gi >> 2);
            bf16x8 vr[NDT];  // batch the V^T fragment reads ahead of the MFMAs
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
              const int col = 32 * dt + 16 * (g & 1) + 4 * (gi & 3);
              const int within = (col & 7) * 2;
              vr[dt] = cat(tr_read(Vt, toff<D>(row0, col >> 3) + within),
                           tr_read(Vt, toff<D>(row0 + 8, col >> 3) + within));
            }
            const bf16x8 pb = pack_acc8(sacc[t], 8 * s);
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) oacc[dt] = mfma32(vr[dt], pb, oacc[dt]);
          }
        }
    }
    if (j + 1 < nt) { FWD_SWRITE((j + 1) & 1); }
    if constexpr (DROP) dm_cur = dm_next;
    __syncthreads();
  }

  const float lt = xhalf_sum(l_i);
  const float inv = lt > 0.f ? oscale / lt : 0.f;
  if (half_on && qrow < S) {
    uint16_t* op = o + (size_t)(b * S + qrow) * ldo + hq * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * dt + 8 * g4 + 4 * hh;
        uint2 u;
        u.x = pack2(oacc[dt][4 * g4 + 0] * inv, oacc[dt][4 * g4 + 1] * inv);
        u.y = pack2(oacc[dt][4 * g4 + 2] * inv, oacc[dt][4 * g4 + 3] * inv);
        *reinterpret_cast<uint2*>(op + d) = u;
      }
    if (hh == 0)
      lse[((size_t)b * Hq + hq) * S + qrow] = lt > 0.f ? m_i * c + __log2f(lt) : INFINITY;
  }
}

// ============================================================================ backward
// delta[b,h,q] = sum_d dO*O  (fp32)
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(
    const uint16_t* __restrict__ o, int ldo, const uint16_t* __restrict__ dout, int lddo,
    float* __restrict__ delta, int B, int S, int Hq, float* __restrict__ dq_zero) {
  constexpr int LPR = D / 8;  // lanes per (token, head) row
  const int gid = (blockIdx.x * 256 + threadIdx.x);
  const int row = gid / LPR, sub = gid % LPR;  // row = (b*S + s)*Hq + h
  const int nrows = B * S * Hq;
  float acc = 0.f;
  if (row < nrows) {
    const int h = row % Hq, tok = row / Hq;
    float a[8], bb[8];
    unpack8(*reinterpret_cast<const uint4*>(o + (size_t)tok * ldo + h * D + sub * 8), a);
    unpack8(*reinterpret_cast<const uint4*>(dout + (size_t)tok * lddo + h * D + sub * 8), bb);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += a[j] * bb[j];
    if (dq_zero) {  // the dQ atomics accumulator starts at zero (saves a separate fill)
      float4* z = reinterpret_cast<float4*>(dq_zero + (size_t)tok * Hq * D + h * D + sub * 8);
      z[0] = make_float4(0.f, 0.f, 0.f, 0.f);
      z[1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (row < nrows && sub == 0) {
    const int h = row % Hq, tok = row / Hq, bi = tok / S, s = tok % S;
    delta[((size_t)bi * Hq + h) * S + s] = acc;
  }
}

// Workgroup = 8 waves = 256 keys: two 128-key blocks, causal pair (i, nkb-1-i) for equal
// work per workgroup.  Each wave owns 32 keys (dK^T, dV^T in accumulators) and sweeps
// 32-row query tiles.  Per tile:
//   phase A  S, dP (key on the lane, -lse / -delta preloaded), P, dS, dV^T += dO^T P,
//            dK^T += Q^T dS, dS^T -> LDS image                              | barrier
//   phase B  dQ_tile = dS K over the 256 keys (16x16x32, one 16x16 tile per wave per
//            16 d-columns) -> fp32 LDS image                                   | barrier
//   phase C  row-contiguous fp32 atomics of the dQ image (one 256-B wave-instruction
//            per row, the full-rate atomic shape) + staging of the next Q/dO tile | barrier
// DP (D-pass): 0 = whole head dim in one pass (D = 64).  D = 128 keeps dK^T/dV^T for all
// 128 columns + K/V rows + Q/dO fragments = ~370 live VGPRs at 2 waves/SIMD (256 max:
// ~100 spilled to scratch, 7.5x the forward time), so it runs as two passes that each
// accumulate half of the dK/dV columns: DP = 1 (columns 0-63, plus dQ), DP = 2 (columns
// 64-127, S and dP recomputed, no dQ).  1.4x the MFMA work, no scratch traffic.
template <int D, bool CAUSAL, int DP, bool DROP>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn_bwd_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
    const uint16_t* __restrict__ v, int ldq, int ldk, int ldv,
    const uint16_t* __restrict__ dout, int lddo, const float* __restrict__ lse,
    const float* __restrict__ delta, float* __restrict__ dq_acc, int lddq,
    uint16_t* __restrict__ dk, uint16_t* __restrict__ dv, int lddk, int lddv, int S, int Hq,
    int Hkv, const int* __restrict__ klen, float c, float dkscale, float dvscale,
    const uint16_t* __restrict__ dbitsT, int NB, float dkeep /* 1-p */) {
  constexpr int KB = 128, KW = 256, QT = 32, NKK = D / 16, NDT = D / 32;
  constexpr int NDL = DP == 0 ? NDT : NDT / 2;      // dK/dV column tiles of this pass
  constexpr int DT0 = DP == 2 ? NDT / 2 : 0;        // first column tile of this pass
  constexpr bool DO_DQ = DP != 2;
  constexpr int KTILE = KW * D * 2;  // bytes
  constexpr int QTILE = QT * D * 2;
  constexpr int CPR = D / 8;
  constexpr int QCH = (QT * CPR + 511) / 512;  // chunks per thread for a Q (or dO) tile
  constexpr int KCH = KW * CPR / 512;
  constexpr int DQT = D / 64;                  // 16x16 dQ tiles per wave (8 waves, 2 q-halves)
  // LDS carve (one array, 16-B aligned offsets)
  constexpr int OFF_K = 0;
  constexpr int OFF_Q = OFF_K + KTILE;            // [2][QTILE]
  constexpr int OFF_DO = OFF_Q + 2 * QTILE;       // [2][QTILE]
  constexpr int OFF_DS = OFF_DO + 2 * QTILE;      // [KW keys][QT q] bf16, 64-B rows
  constexpr int OFF_DQ = OFF_DS + KW * QT * 2;    // [QT][D+4] fp32
  constexpr int DQS = D + 4;                      // padded dQ image row (2-way -> 1-way)
  constexpr int OFF_L = OFF_DQ + QT * DQS * 4;    // [2][QT] float  (-lse2/c)
  constexpr int OFF_DL = OFF_L + 2 * QT * 4;      // [2][QT] float  (-delta)
  constexpr int LDS_BYTES = OFF_DL + 2 * QT * 4;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wl = w & 3, half = w >> 2;
  const int r = lane & 31, hh = lane >> 5, g = lane >> 4, gi = lane & 15;
  const int nkb = (S + KB - 1) / KB;
  const int pair = blockIdx.x;
  int kb_mine, kb_other;
  if (CAUSAL) {
    kb_mine = half ? nkb - 1 - pair : pair;
    kb_other = half ? pair : nkb - 1 - pair;
  } else {
    kb_mine = 2 * pair + half;
    kb_other = 2 * pair + (half ^ 1);
  }
  const bool half_on = kb_mine < nkb && !(CAUSAL && half == 1 && kb_mine == kb_other);
  const int hk = blockIdx.y, b = blockIdx.z;
  const int grp = Hq / Hkv;
  const int kl = klen ? klen[b] : S;
  const int kw0 = kb_mine * KB + 32 * wl;  // first key of this wave
  const int key = kw0 + r;                 // this lane's key (column of S / dP)
  const bool key_ok = half_on && key < kl;

  // D = 128: the lane's K row is NOT kept in registers (it is read back from the K tile
  // in LDS per use) and Q/dO rows are read per MFMA step -- keeping all of them resident
  // (kf + vf + qr + orr = 128 VGPRs next to 128 accumulator VGPRs) spilled ~170 VGPRs.
  constexpr bool KREG = D <= 64;
  bf16x8 kf[KREG ? NKK : 1], vf[NKK];
  {
    const bool in = half_on && key < S;
    const uint16_t* kp = k + (size_t)(b * S + key) * ldk + hk * D + 8 * hh;
    const uint16_t* vp = v + (size_t)(b * S + key) * ldv + hk * D + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      if constexpr (KREG) kf[kk] = in ? ld8(kp + 16 * kk) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      vf[kk] = in ? ld8(vp + 16 * kk) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  // K tile of both key blocks in LDS (rows 0-127: first block of the pair, 128-255: second)
#pragma unroll
  for (int i = 0; i < KCH; ++i) {
    const int ci = tid + 512 * i, row = ci / CPR, ch = ci % CPR;
    const int blk = (row < KB) ? (CAUSAL ? pair : 2 * pair) : (CAUSAL ? nkb - 1 - pair : 2 * pair + 1);
    const int kk = blk * KB + (row & (KB - 1));
    uint4 val = make_uint4(0, 0, 0, 0);
    const bool dup = CAUSAL && row >= KB && blk == pair;
    if (blk < nkb && kk < S && !dup)
      val = *reinterpret_cast<const uint4*>(k + (size_t)(b * S + kk) * ldk + hk * D + ch * 8);
    *reinterpret_cast<uint4*>(smem + OFF_K + toff_k<D>(row, ch)) = val;
  }

  f32x16 dvacc[NDL], dkacc[NDL];
#pragma unroll
  for (int dt = 0; dt < NDL; ++dt) { dvacc[dt] = f32x16{}; dkacc[dt] = f32x16{}; }

  const int nqt = (S + QT - 1) / QT;
  const int first_kb = CAUSAL ? pair : 2 * pair;
  const int qt0 = CAUSAL ? (first_kb * KB / QT) : 0;
  const int per_head = nqt - qt0;
  const int total = per_head * grp;

  uint4 qreg[QCH], dreg[QCH];
  float lreg = 0.f, dlreg = 0.f;
  int lq = 0;
  uint32_t dm_next = 0;
  auto gload = [&](int it) {
    const int hq = hk * grp + it / per_head;
    const int qs = (qt0 + it % per_head) * QT;
    if constexpr (DROP) {  // key-on-lane dropout bits of this wave's 32x32 block
      if (half_on && kw0 < S && (!CAUSAL || qs + QT - 1 >= kw0))
        dm_next = dbitsT[(((size_t)(b * Hq + hq) * NB + (kw0 >> 5)) * NB + (qs >> 5)) * 64 + lane];
    }
    // rows past S are clamped (finite duplicates; their P is forced to 0 via lse=-inf)
#pragma unroll
    for (int i = 0; i < QCH; ++i) {
      const int ci = tid + 512 * i, row = ci / CPR, ch = ci % CPR;
      const int qq = min(qs + row, S - 1);
      if (row < QT) {
        qreg[i] = *reinterpret_cast<const uint4*>(q + (size_t)(b * S + qq) * ldq + hq * D + ch * 8);
        dreg[i] = *reinterpret_cast<const uint4*>(dout + (size_t)(b * S + qq) * lddo + hq * D + ch * 8);
      }
    }
    // raw loads only: any arithmetic on a just-loaded value here would make the compiler
    // wait vmcnt(0) and serialise the whole prefetch; the conversion happens in swrite
    if (tid < QT) {
      const int qq = qs + tid;
      const size_t li = ((size_t)b * Hq + hq) * S + min(qq, S - 1);
      lreg = lse[li];
      dlreg = delta[li];
      lq = qq;
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < QCH; ++i) {
      const int ci = tid + 512 * i, row = ci / CPR, ch = ci % CPR;
      if (row < QT) {
        *reinterpret_cast<uint4*>(smem + OFF_Q + buf * QTILE + toff<D>(row, ch)) = qreg[i];
        *reinterpret_cast<uint4*>(smem + OFF_DO + buf * QTILE + toff<D>(row, ch)) = dreg[i];
      }
    }
    if (tid < QT) {
      reinterpret_cast<float*>(smem + OFF_L)[buf * QT + tid] = lq < S ? -lreg / c : -INFINITY;
      reinterpret_cast<float*>(smem + OFF_DL)[buf * QT + tid] = lq < S ? -dlreg * dkeep : 0.f;
    }
  };

  if (total > 0) {
    gload(0);
    swrite(0);
  }
  __syncthreads();
  char* dsimg = smem + OFF_DS;
  float* dqimg = reinterpret_cast<float*>(smem + OFF_DQ);
  const int krow = KB * half + 32 * wl + r;  // this lane's row in the dS^T image / K tile
  uint32_t dm = 0;
  for (int it = 0; it < total; ++it) {
    const int hq = hk * grp + it / per_head;
    const int qs = (qt0 + it % per_head) * QT;
    if constexpr (DROP) dm = dm_next;
    if (it + 1 < total) gload(it + 1);
    const int buf = it & 1;
    const char* Qt = smem + OFF_Q + buf * QTILE;
    const char* Ot = smem + OFF_DO + buf * QTILE;
    const float* Ls = reinterpret_cast<const float*>(smem + OFF_L) + buf * QT;
    const float* DLs = reinterpret_cast<const float*>(smem + OFF_DL) + buf * QT;
    const bool active = half_on && kw0 < S && (!CAUSAL || qs + QT - 1 >= kw0);
    // ---------------- phase A
    if (active) {
      f32x16 sacc, dpacc;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int ql = (e & 3) + 8 * (e >> 2) + 4 * hh;
        sacc[e] = Ls[ql];
        dpacc[e] = DLs[ql];
      }
      if constexpr (KREG) {
        bf16x8 qr[NKK], orr[NKK];  // batch the row reads ahead of the MFMAs
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) {
          qr[kk] = lds8(Qt, toff<D>(r, 2 * kk + hh));
          orr[kk] = lds8(Ot, toff<D>(r, 2 * kk + hh));
        }
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) {
          sacc = mfma32(qr[kk], kf[kk], sacc);
          dpacc = mfma32(orr[kk], vf[kk], dpacc);
        }
      } else {
#pragma unroll
        for (int kk = 0; kk < NKK; kk += 2) {   // two steps of row reads in flight
          const bf16x8 q0 = lds8(Qt, toff<D>(r, 2 * kk + hh));
          const bf16x8 o0 = lds8(Ot, toff<D>(r, 2 * kk + hh));
          const bf16x8 k0 = lds8(smem + OFF_K, toff_k<D>(krow, 2 * kk + hh));
          const bf16x8 q1 = lds8(Qt, toff<D>(r, 2 * kk + 2 + hh));
          const bf16x8 o1 = lds8(Ot, toff<D>(r, 2 * kk + 2 + hh));
          const bf16x8 k1 = lds8(smem + OFF_K, toff_k<D>(krow, 2 * kk + 2 + hh));
          sacc = mfma32(q0, k0, sacc);
          dpacc = mfma32(o0, vf[kk], dpacc);
          sacc = mfma32(q1, k1, sacc);
          dpacc = mfma32(o1, vf[kk + 1], dpacc);
        }
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) sacc[e] = __builtin_amdgcn_exp2f(c * sacc[e]);
      // masking only on diagonal / padded tiles (wave-uniform test), as selects
      if ((CAUSAL && qs < kw0 + 31) || kw0 + 32 > kl) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int qq = qs + (e & 3) + 8 * (e >> 2) + 4 * hh;
          const bool dead = !key_ok || (CAUSAL && key > qq);
          sacc[e] = dead ? 0.f : sacc[e];
        }
      }
      if constexpr (DROP) {
        // dpacc = dP~ - delta(1-p): kept -> P * dpacc, dropped -> P * (-delta(1-p)) (the
        // common 1/(1-p) is in dkscale / the dQ scale); dV^T takes the dropped P
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float p = sacc[e];
          const int ql = (e & 3) + 8 * (e >> 2) + 4 * hh;
          dpacc[e] = p * keep_sel(dpacc[e], DLs[ql], dm, e);
          sacc[e] = keep_or_zero(p, dm, e);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float p = sacc[e];
          dpacc[e] = p * dpacc[e];
        }
      }
      constexpr int SUNROLL = D <= 64 ? 2 : 1;   // D=128: don't hoist both halves' reads
#pragma unroll SUNROLL
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pb = pack_acc8(sacc, 8 * s);
        const bf16x8 db = pack_acc8(dpacc, 8 * s);
        const int row0 = 16 * s + 4 * hh + (gi >> 2);
#pragma unroll
        for (int dt = 0; dt < NDL; ++dt) {
          const int col = 32 * (dt + DT0) + 16 * (g & 1) + 4 * (gi & 3);
          const int within = (col & 7) * 2;
          const bf16x8 dot = cat(tr_read(Ot, toff<D>(row0, col >> 3) + within),
                                 tr_read(Ot, toff<D>(row0 + 8, col >> 3) + within));
          dvacc[dt] = mfma32(dot, pb, dvacc[dt]);
          const bf16x8 qtr = cat(tr_read(Qt, toff<D>(row0, col >> 3) + within),
                                 tr_read(Qt, toff<D>(row0 + 8, col >> 3) + within));
          dkacc[dt] = mfma32(qtr, db, dkacc[dt]);
        }
      }
#pragma unroll
      for (int g4 = 0; g4 < (DO_DQ ? 4 : 0); ++g4) {
        const int ql = 8 * g4 + 4 * hh;
        uint2 u;
        u.x = pack2(dpacc[4 * g4 + 0], dpacc[4 * g4 + 1]);
        u.y = pack2(dpacc[4 * g4 + 2], dpacc[4 * g4 + 3]);
        *reinterpret_cast<uint2*>(dsimg + ds_off(krow, ql * 2)) = u;
      }
    } else if (DO_DQ) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int ql = 8 * g4 + 4 * hh;
        *reinterpret_cast<uint2*>(dsimg + ds_off(krow, ql * 2)) = make_uint2(0, 0);
      }
    }
    __syncthreads();
    // ---------------- phase B: dQ[q][d] = sum over 256 keys dS[q][key] K[key][d]
    if constexpr (DO_DQ) {
      const int qtile = w & 1;
      f32x4 dq[DQT];
#pragma unroll
      for (int i = 0; i < DQT; ++i) dq[i] = f32x4{};
#pragma unroll
      for (int ks = 0; ks < KW / 32; ++ks) {
        const int kr = 32 * ks + 8 * g + (gi >> 2);
        const int qcol = 16 * qtile + 4 * (gi & 3);
        const bf16x8 a = cat(tr_read(dsimg, ds_off(kr, qcol * 2)),
                             tr_read(dsimg, ds_off(kr + 4, qcol * 2)));
#pragma unroll
        for (int i = 0; i < DQT; ++i) {
          const int dtile = (w >> 1) * DQT + i;
          const int dcol = 16 * dtile + 4 * (gi & 3);
          const int within = (dcol & 7) * 2;
          const bf16x8 bk = cat(tr_read(smem + OFF_K, toff_k<D>(kr, dcol >> 3) + within),
                                tr_read(smem + OFF_K, toff_k<D>(kr + 4, dcol >> 3) + within));
          dq[i] = mfma16(a, bk, dq[i]);
        }
      }
      // C layout 16x16: col = lane&15 (d), row = (lane>>4)*4 + e (q)
#pragma unroll
      for (int i = 0; i < DQT; ++i) {
        const int dtile = (w >> 1) * DQT + i;
#pragma unroll
        for (int e = 0; e < 4; ++e) dqimg[(16 * qtile + 4 * g + e) * DQS + 16 * dtile + gi] = dq[i][e];
      }
    }
    __syncthreads();
    // ---------------- phase C: next-tile staging FIRST (its vmcnt wait must not cover the
    // atomics), then row-contiguous fp32 atomics that stay in flight across the barrier
    if (it + 1 < total) swrite((it + 1) & 1);
    if constexpr (DO_DQ) {
      constexpr int RPW = QT / 8;       // rows per wave
      constexpr int IPR = D / 64;       // 64-lane instructions per row
      float vals[RPW][IPR];
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
        for (int ii = 0; ii < IPR; ++ii) vals[rr][ii] = dqimg[(w * RPW + rr) * DQS + 64 * ii + lane];
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) {
        const int qq = qs + w * RPW + rr;
        if (qq < S) {
#pragma unroll
          for (int ii = 0; ii < IPR; ++ii)
            atomicAdd(dq_acc + (size_t)(b * S + qq) * lddq + hq * D + 64 * ii + lane,
                      vals[rr][ii]);
        }
      }
    }
    __syncthreads();
  }
  // write dK (scaled) and dV for this lane's key: rows d = 32dt + 8g4 + 4hh + 0..3
  if (half_on && key < S) {
    uint16_t* dkp = dk + (size_t)(b * S + key) * lddk + hk * D;
    uint16_t* dvp = dv + (size_t)(b * S + key) * lddv + hk * D;
#pragma unroll
    for (int dt = 0; dt < NDL; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * (dt + DT0) + 8 * g4 + 4 * hh;
        uint2 u;
        u.x = pack2(dkacc[dt][4 * g4 + 0] * dkscale, dkacc[dt][4 * g4 + 1] * dkscale);
        u.y = pack2(dkacc[dt][4 * g4 + 2] * dkscale, dkacc[dt][4 * g4 + 3] * dkscale);
        *reinterpret_cast<uint2*>(dkp + d) = u;
        u.x = pack2(dvacc[dt][4 * g4 + 0] * dvscale, dvacc[dt][4 * g4 + 1] * dvscale);
        u.y = pack2(dvacc[dt][4 * g4 + 2] * dvscale, dvacc[dt][4 * g4 + 3] * dvscale);
        *reinterpret_cast<uint2*>(dvp + d) = u;
      }
  }
}

// dq (bf16, strided into the packed dqkv) = dq_acc * scale
__global__ __launch_bounds__(256) void dq_convert_kernel(const float* __restrict__ acc,
                                                         int ldacc, uint16_t* __restrict__ dq,
                                                         int lddq, int ntok, int width,
                                                         float scale) {
  const int64_t v = blockIdx.x * 256ll + threadIdx.x;
  const int per_row = width / 8;
  if (v >= (int64_t)ntok * per_row) return;
  const int t = (int)(v / per_row), c = (int)(v % per_row) * 8;
  const float4 a = *reinterpret_cast<const float4*>(acc + (size_t)t * ldacc + c);
  const float4 bq = *reinterpret_cast<const float4*>(acc + (size_t)t * ldacc + c + 4);
  float f[8] = {a.x * scale, a.y * scale, a.z * scale, a.w * scale,
                bq.x * scale, bq.y * scale, bq.z * scale, bq.w * scale};
  *reinterpret_cast<uint4*>(dq + (size_t)t * lddq + c) = pack8(f);
}

template <int D>
hipError_t fwd_dispatch(bool causal, bool drop, dim3 grid, hipStream_t s, const uint16_t* q,
                        const uint16_t* k, const uint16_t* v, int ldq, int ldk, int ldv,
                        uint16_t* o, int ldo, float* lse, int S, int Hq, int Hkv,
                        const int* klen, float c, const uint64_t* dbits, int NB, int NKT,
                        float oscale) {
#define MX_ATTN_FWD(C, DR)                                                                  \
  hipLaunchKernelGGL((attn_fwd_kernel<D, C, DR>), grid, dim3(512), 0, s, q, k, v, ldq, ldk, ldv, o, \
                     ldo, lse, S, Hq, Hkv, klen, c, dbits, NB, NKT, oscale)
  if (causal) {
    if (drop) MX_ATTN_FWD(true, true); else MX_ATTN_FWD(true, false);
  } else {
    if (drop) MX_ATTN_FWD(false, true); else MX_ATTN_FWD(false, false);
  }
#undef MX_ATTN_FWD
  return hipGetLastError();
}

template <int D>
hipError_t bwd_dispatch(bool causal, bool drop, dim3 grid, hipStream_t s, const uint16_t* q,
                        const uint16_t* k, const uint16_t* v, int ldq, int ldk, int ldv,
                        const uint16_t* dout, int lddo, const float* lse, const float* delta,
                        float* dq_acc, int lddq, uint16_t* dk, uint16_t* dv, int lddk, int lddv,
                        int S, int Hq, int Hkv, const int* klen, float c, float dkscale,
                        float dvscale, const uint16_t* dbitsT, int NB, float dkeep) {
#define MX_ATTN_BWD(C, P, DR)                                                              \
  hipLaunchKernelGGL((attn_bwd_kernel<D, C, P, DR>), grid, dim3(512), 0, s, q, k, v, ldq, ldk,  \
                     ldv, dout, lddo, lse, delta, dq_acc, lddq, dk, dv, lddk, lddv, S, Hq, Hkv,   \
                     klen, c, dkscale, dvscale, dbitsT, NB, dkeep)
#define MX_ATTN_BWD_P(C, P) \
  { if (drop) MX_ATTN_BWD(C, P, true); else MX_ATTN_BWD(C, P, false); }
  if constexpr (D <= 64) {
    if (causal) MX_ATTN_BWD_P(true, 0)
    else MX_ATTN_BWD_P(false, 0)
  } else {
    if (causal) { MX_ATTN_BWD_P(true, 1) MX_ATTN_BWD_P(true, 2) }
    else { MX_ATTN_BWD_P(false, 1) MX_ATTN_BWD_P(false, 2) }
  }
#undef MX_ATTN_BWD_P
#undef MX_ATTN_BWD
  return hipGetLastError();
}

}  // namespace

// Dropout keep-mask images for one attention call (see the header comment).
// fwd_bits: u16 [B*Hq][NB][NKT*4][64] (NB = ceil(S/32), NKT = ceil(NB/4));
// bwd_bits: u16 [B*Hq][NB][NB][64].  h_off / Hg: this rank's first global head / the
// model's head count (so tensor/context-parallel shards draw the single-GPU mask).
MX_EXPORT int mx_attn_dropmask(const uint32_t* seed, uint32_t salt, float p, int B, int S, int Hq,
                               int h_off, int Hg, int causal, void* fwd_bits, void* bwd_bits,
                               hipStream_t s) {
  const int NB = (S + 31) / 32, NKT = (NB + 3) / 4;
  const uint32_t thr16 = (uint32_t)(p * 65536.0f + 0.5f);
  hipLaunchKernelGGL(attn_dropmask_kernel, dim3(NB, NB, B * Hq), dim3(64), 0, s, seed, salt, thr16,
                     S, Hq, h_off, Hg, NB, NKT, causal, (uint16_t*)fwd_bits, (uint16_t*)bwd_bits);
  return hipGetLastError();
}

// Q/K/V/O are bf16 with token strides ld*; head h lives at column h*D.
// lse: fp32 [B, Hq, S] (base 2).  klen: int32 [B] valid key count or null.
// fwd_bits: dropout image from mx_attn_dropmask or null (no dropout); keep_scale = 1/(1-p).
MX_EXPORT int mx_attn_fwd(const void* q, const void* k, const void* v, int ldq, int ldk,
                          int ldv, void* o, int ldo, float* lse, int B, int S, int Hq, int Hkv,
                          int D, int causal, const int* klen, float scale, const void* fwd_bits,
                          float keep_scale, hipStream_t s) {
  if (Hq % Hkv) return hipErrorInvalidValue;
  const float c = scale * 1.4426950408889634f;
  const int nqb = (S + 127) / 128;
  const int NB = (S + 31) / 32, NKT = (NB + 3) / 4;
  dim3 grid((nqb + 1) / 2, Hq, B);
  const bool drop = fwd_bits != nullptr;
  const float osc = drop ? keep_scale : 1.f;
  if (D == 64)
    return fwd_dispatch<64>(causal, drop, grid, s, (const uint16_t*)q, (const uint16_t*)k,
                            (const uint16_t*)v, ldq, ldk, ldv, (uint16_t*)o, ldo, lse, S, Hq,
                            Hkv, klen, c, (const uint64_t*)fwd_bits, NB, NKT, osc);
  if (D == 128)
    return fwd_dispatch<128>(causal, drop, grid, s, (const uint16_t*)q, (const uint16_t*)k,
                             (const uint16_t*)v, ldq, ldk, ldv, (uint16_t*)o, ldo, lse, S, Hq,
                             Hkv, klen, c, (const uint64_t*)fwd_bits, NB, NKT, osc);
  return hipErrorInvalidValue;
}

// dq_acc: fp32 [B*S, Hq*D] workspace (zeroed here); delta: fp32 [B, Hq, S] workspace.
// bwd_bits: the dropout image of the forward (or null); keep_scale = 1/(1-p).
MX_EXPORT int mx_attn_bwd(const void* q, const void* k, const void* v, int ldq, int ldk,
                          int ldv, const void* o, int ldo, const void* dout, int lddo,
                          const float* lse, float* delta, float* dq_acc, void* dq, int lddq,
                          void* dk, void* dv, int lddk, int lddv, int B, int S, int Hq,
                          int Hkv, int D, int causal, const int* klen, float scale,
                          const void* bwd_bits, float keep_scale, hipStream_t s) {
  if (Hq % Hkv) return hipErrorInvalidValue;
  const float c = scale * 1.4426950408889634f;
  {
    const int64_t threads = (int64_t)B * S * Hq * (D / 8);
    if (D == 64)
      hipLaunchKernelGGL(attn_bwd_pre_kernel<64>, dim3((unsigned)((threads + 255) / 256)),
                         dim3(256), 0, s, (const uint16_t*)o, ldo, (const uint16_t*)dout, lddo,
                         delta, B, S, Hq, dq_acc);
    else if (D == 128)
      hipLaunchKernelGGL(attn_bwd_pre_kernel<128>, dim3((unsigned)((threads + 255) / 256)),
                         dim3(256), 0, s, (const uint16_t*)o, ldo, (const uint16_t*)dout, lddo,
                         delta, B, S, Hq, dq_acc);
    else
      return hipErrorInvalidValue;
  }
  const int nkb = (S + 127) / 128;
  const int NB = (S + 31) / 32;
  dim3 grid((nkb + 1) / 2, Hkv, B);
  const int lddq_acc = Hq * D;
  const bool drop = bwd_bits != nullptr;
  const float ks = drop ? keep_scale : 1.f;
  const float dkeep = drop ? 1.f / keep_scale : 1.f;
  hipError_t e;
  if (D == 64)
    e = bwd_dispatch<64>(causal, drop, grid, s, (const uint16_t*)q, (const uint16_t*)k,
                         (const uint16_t*)v, ldq, ldk, ldv, (const uint16_t*)dout, lddo, lse,
                         delta, dq_acc, lddq_acc, (uint16_t*)dk, (uint16_t*)dv, lddk, lddv, S,
                         Hq, Hkv, klen, c, scale * ks, ks, (const uint16_t*)bwd_bits, NB, dkeep);
  else
    e = bwd_dispatch<128>(causal, drop, grid, s, (const uint16_t*)q, (const uint16_t*)k,
                          (const uint16_t*)v, ldq, ldk, ldv, (const uint16_t*)dout, lddo, lse,
                          delta, dq_acc, lddq_acc, (uint16_t*)dk, (uint16_t*)dv, lddk, lddv, S,
                          Hq, Hkv, klen, c, scale * ks, ks, (const uint16_t*)bwd_bits, NB, dkeep);
  if (e != hipSuccess) return e;
  const int64_t nv = (int64_t)B * S * Hq * D / 8;
  hipLaunchKernelGGL(dq_convert_kernel, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s,
                     dq_acc, lddq_acc, (uint16_t*)dq, lddq, B * S, Hq * D, scale * ks);
  return hipGetLastError();
}
