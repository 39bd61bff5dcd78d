// Direct peer-to-peer collectives over xGMI for one MI355X node.
//
// RCCL's ring moves every byte over ONE outbound xGMI link per GPU (~153 GB/s), so a
// ring all-reduce is per-link bound.  Here every rank maps every peer's registered
// buffer (hipIpcGetMemHandle / hipIpcOpenMemHandle, handles exchanged through the c10d
// store) and a kernel reads all 7 peers at once, so all 7 links carry traffic:
//
//   one-shot all-reduce (small messages):  copy-in -> barrier -> every rank reads the
//       whole message from every peer and reduces it locally -> barrier
//   two-shot all-reduce (large):  copy-in -> barrier -> rank r reduces shard r from all
//       peers into its own buffer -> barrier -> every rank gathers all shards -> barrier
//   reduce-scatter (ZeRO-1 gradient shard) and all-gather (parameter shard): halves
//       of the two-shot algorithm
//   direct reduce-scatter / all-gather on REGISTERED buffers (the flat gradient buffer,
//       the ZeRO-1 parameter shard): every peer's buffer is IPC-mapped once, so the
//       kernel reads the peers' bucket in place -- no copy-in through a staging buffer
//       (one HBM read + write less per byte), barrier -> read -> barrier
//
// Synchronisation is per workgroup, never grid-wide: workgroup b of every rank
// copies exactly the pieces that workgroup b of the other ranks read next (the
// piece partition is the same on every rank), so a barrier between the b-th
// workgroups of all ranks is enough.  Barrier = release fence (system scope; writes
// the L2 back so peers reading over xGMI see the data) -> one lane per peer stores
// the epoch into that peer's flag slot [b][my rank] (uncached memory) -> one lane per
// peer polls our own slot [b][peer] -> acquire fence.  Epochs are per-workgroup
// counters kept in device memory and advanced by the kernel itself, so the same
// launch can be replayed from a hipGraph.  Every poll is bounded (s_memrealtime,
// 100 MHz): on timeout the kernel records an error word and exits, so a rank that
// never arrives cannot hang the GPU; the host checks the word (mx_xgmi_error).
#include <cstring>

#include "../common.h"

using namespace mx;

namespace {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 128;
constexpr int kThreads = 512;

struct Flags {                                  // one per rank, uncached device memory
  uint32_t slot[3][kMaxBlocks][kMaxRanks];      // [phase][workgroup][source rank]
  uint32_t counter[kMaxBlocks];                 // last completed epoch per workgroup
  uint32_t error;                               // nonzero after a barrier timeout / mismatch
  uint32_t sig[4];                              // validation: op, bytes lo/hi, host sequence no.
};

// error word: 1 + phase for a barrier timeout; kErrSig + peer for a call-signature
// mismatch (validation mode: ranks are not in the same collective call)
constexpr uint32_t kErrSig = 0x100;

struct Peers {
  char* data[kMaxRanks];
  Flags* flags[kMaxRanks];
};

__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

// cross-rank barrier between the b-th workgroups; false on timeout
__device__ bool xbarrier(const Peers& pp, int phase, int rank, int world, uint32_t epoch,
                         uint64_t timeout_ticks) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope: drain + L2 write-back
  __syncthreads();
  const int b = blockIdx.x, t = threadIdx.x;
  __shared__ int ok_s;
  if (t == 0) ok_s = 1;
  __syncthreads();
  if (t < world) {
    __hip_atomic_store(&pp.flags[t]->slot[phase][b][rank], epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = &pp.flags[rank]->slot[phase][b][t];
    const uint64_t t0 = now_ticks();
    while (__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      if (now_ticks() - t0 > timeout_ticks) {
        __hip_atomic_store(&pp.flags[rank]->error, 1u + (uint32_t)phase, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        ok_s = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // drop stale lines before peer reads
  return ok_s != 0;
}

// 16-byte vector accumulate helpers (bf16 x 8 or fp32 x 4)
template <bool kBF16>
struct Vec;
template <>
struct Vec<true> {
  float f[8];
  __device__ void zero() {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = 0.f;
  }
  __device__ void add(const uint4& v) {
    float g[8];
    unpack8(v, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] += g[j];
  }
  __device__ uint4 pack() const { return pack8(f); }
};
template <>
struct Vec<false> {
  float f[4];
  __device__ void zero() { f[0] = f[1] = f[2] = f[3] = 0.f; }
  __device__ void add(const uint4& v) {
    f[0] += __uint_as_float(v.x); f[1] += __uint_as_float(v.y);
    f[2] += __uint_as_float(v.z); f[3] += __uint_as_float(v.w);
  }
  __device__ uint4 pack() const {
    return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]),
                      __float_as_uint(f[3]));
  }
};

template <bool kBF16>
__device__ __forceinline__ uint4 reduce_at(const Peers& pp, int64_t v, int rank, int world) {
  Vec<kBF16> acc;
  acc.zero();
  uint4 x[kMaxRanks];
#pragma unroll
  for (int i = 0; i < kMaxRanks; ++i)   // issue all peer loads before using any (7 links)
    if (i < world) x[i] = reinterpret_cast<const uint4*>(pp.data[(rank + i) % world])[v];
#pragma unroll
  for (int i = 0; i < kMaxRanks; ++i)
    if (i < world) acc.add(x[i]);
  return acc.pack();
}

// piece partition of [lo, hi): workgroup b, thread t take lo + b*T + t, stride G*T
#define FOR_PIECE(v, lo, hi) \
  for (int64_t v = (lo) + (int64_t)blockIdx.x * kThreads + threadIdx.x; v < (hi); \
       v += (int64_t)gridDim.x * kThreads)

enum Op {
  kAllReduce1 = 0, kAllReduce2 = 1, kReduceScatter = 2, kAllGather = 3,
  kReduceScatterDirect = 4,   // pp.data[i] = peer i's registered input (the full message)
  kAllGatherDirect = 5        // pp.data[i] = peer i's registered shard (hi(i) - lo(i) vectors)
};

// validation mode: workgroup 0 publishes this call's signature before the first barrier
// and compares every peer's after it (peers cannot start their next call before the last
// barrier of this one, so the slot is stable while it is read)
__device__ __forceinline__ void publish_sig(Flags* self, const uint32_t* sig) {
  if (blockIdx.x == 0 && threadIdx.x < 4)
    __hip_atomic_store(&self->sig[threadIdx.x], sig[threadIdx.x], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void check_sig(const Peers& pp, int rank, int world, const uint32_t* sig) {
  if (blockIdx.x != 0 || threadIdx.x >= world) return;
  const int peer = threadIdx.x;
  bool same = true;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    same &= __hip_atomic_load(&pp.flags[peer]->sig[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == sig[j];
  if (!same)
    __hip_atomic_store(&pp.flags[rank]->error, kErrSig + (uint32_t)peer, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// nvec = 16-B vectors of the FULL message (all-gather: of the gathered output);
// shard = ceil(nvec / world) vectors (shards 0..world-2 full, last may be short)
struct Sig {
  uint32_t v[4];
};

template <bool kBF16>
__global__ __launch_bounds__(kThreads) void xgmi_kernel(Peers pp, const uint4* in,
                                                         uint4* out, int64_t nvec,
                                                         int rank, int world, int op,
                                                         uint64_t timeout_ticks, Sig sig,
                                                         int validate) {
  Flags* self = pp.flags[rank];
  const int b = blockIdx.x;
  const uint32_t epoch = self->counter[b] + 1;
  uint4* mine = reinterpret_cast<uint4*>(pp.data[rank]);
  const int64_t shard = (nvec + world - 1) / world;
  auto lo = [&](int q) { return min((int64_t)q * shard, nvec); };
  auto hi = [&](int q) { return min((int64_t)(q + 1) * shard, nvec); };
  bool ok = true;
  if (validate) publish_sig(self, sig.v);

  if (op == kReduceScatterDirect) {
    ok = xbarrier(pp, 0, rank, world, epoch, timeout_ticks);
    if (validate) check_sig(pp, rank, world, sig.v);
    if (ok) FOR_PIECE(v, lo(rank), hi(rank)) out[v - lo(rank)] = reduce_at<kBF16>(pp, v, rank, world);
  } else if (op == kAllGatherDirect) {
    ok = xbarrier(pp, 0, rank, world, epoch, timeout_ticks);
    if (validate) check_sig(pp, rank, world, sig.v);
    if (ok)
      for (int i = 0; i < world; ++i) {
        const int q = (rank + i) % world;
        const uint4* src = reinterpret_cast<const uint4*>(pp.data[q]);
        FOR_PIECE(v, lo(q), hi(q)) out[v] = src[v - lo(q)];
      }
  } else if (op == kAllReduce1) {
    FOR_PIECE(v, 0, nvec) mine[v] = in[v];
    ok = xbarrier(pp, 0, rank, world, epoch, timeout_ticks);
    if (validate) check_sig(pp, rank, world, sig.v);
    if (ok) FOR_PIECE(v, 0, nvec) out[v] = reduce_at<kBF16>(pp, v, rank, world);
  } else if (op == kAllGather) {
    // in = my shard (hi(rank) - lo(rank) vectors); out = full [nvec]
    FOR_PIECE(v, lo(rank), hi(rank)) mine[v] = in[v - lo(rank)];
    ok = xbarrier(pp, 0, rank, world, epoch, timeout_ticks);
    if (validate) check_sig(pp, rank, world, sig.v);
    if (ok)
      for (int i = 0; i < world; ++i) {
        const int q = (rank + i) % world;
        const uint4* src = reinterpret_cast<const uint4*>(pp.data[q]);
        FOR_PIECE(v, lo(q), hi(q)) out[v] = src[v];
      }
  } else {
    // reduce-scatter / two-shot: copy pieces of every shard, reduce my shard
    for (int q = 0; q < world; ++q) FOR_PIECE(v, lo(q), hi(q)) mine[v] = in[v];
    ok = xbarrier(pp, 0, rank, world, epoch, timeout_ticks);
    if (validate) check_sig(pp, rank, world, sig.v);
    if (ok) {
      if (op == kReduceScatter) {
        FOR_PIECE(v, lo(rank), hi(rank)) out[v - lo(rank)] = reduce_at<kBF16>(pp, v, rank, world);
      } else {
        FOR_PIECE(v, lo(rank), hi(rank)) mine[v] = reduce_at<kBF16>(pp, v, rank, world);
        ok = xbarrier(pp, 1, rank, world, epoch, timeout_ticks);
        if (ok)
          for (int i = 0; i < world; ++i) {
            const int q = (rank + i) % world;
            const uint4* src = reinterpret_cast<const uint4*>(pp.data[q]);
            FOR_PIECE(v, lo(q), hi(q)) out[v] = src[v];
          }
      }
    }
  }
  // nobody may overwrite its buffer (next call) while a peer still reads it
  if (ok) ok = xbarrier(pp, 2, rank, world, epoch, timeout_ticks);
  if (threadIdx.x == 0) self->counter[b] = epoch;
}

// ------------------------------------------------------------------ point-to-point
// Pipeline-parallel 1F1B transfers (one activation / activation gradient per message)
// between two ranks of one node.  Same memory model as the collectives above: the WRITER
// of a buffer writes it locally and releases it at system scope (L2 write-back) before it
// signals; the reader acquires and then reads it over xGMI.  Per directed channel:
//   * the sender owns a ring of kP2PRing slots (registered, IPC-mapped by the receiver);
//   * message n goes to slot n % kP2PRing: the sender waits until the receiver has freed
//     the slot (message n - kP2PRing consumed), copies the payload into it, releases, and
//     stores n + 1 into the receiver's FULL word of that slot (remote store);
//   * the receiver polls its own FULL word, acquires, copies the slot into its output
//     tensor (reads over xGMI), drains its loads, and stores n + 1 into the sender's FREE
//     word (remote store) -- the sender's next use of the slot waits for it.
// Every workgroup b handles the same strided share of the message on both sides and has
// its own FULL / FREE words and its own sequence counter, so no grid-wide sync is needed.
// The counters live in device memory and are advanced by the kernels (hipGraph replays stay
// in step); every wait is bounded (error word, as above).
constexpr int kP2PRing = 4;
constexpr int kP2PBlocks = 64;

struct P2PCtl {                                 // one per rank per peer, uncached memory
  uint32_t full[kP2PRing][kP2PBlocks];          // receiver side: message seq + 1 is in slot
  uint32_t free_[kP2PRing][kP2PBlocks];         // sender side: message seq + 1 was consumed
  uint32_t send_seq[kP2PBlocks];
  uint32_t recv_seq[kP2PBlocks];
  uint32_t error;                               // 1: send wait timed out, 2: recv wait timed out
};

__device__ __forceinline__ bool p2p_wait(const uint32_t* word, uint32_t target, uint64_t timeout_ticks) {
  const uint64_t t0 = now_ticks();
  while ((int32_t)(__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - target) < 0) {
    if (now_ticks() - t0 > timeout_ticks) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// mine: this rank's ctl for the channel; peer: the receiver's ctl (mapped); ring: this
// rank's own send ring (local); src: the payload (nvec 16-B vectors, nvec <= slot_vec)
__global__ __launch_bounds__(kThreads) void p2p_send_kernel(P2PCtl* mine, P2PCtl* peer, uint4* ring,
                                                            int64_t slot_vec, const uint4* src, int64_t nvec,
                                                            uint64_t timeout_ticks) {
  const int b = blockIdx.x, t = threadIdx.x;
  __shared__ int ok_s;
  const uint32_t n = mine->send_seq[b];
  const int slot = (int)(n % kP2PRing);
  if (t == 0) {
    ok_s = 1;
    // slot free: message n - kP2PRing consumed (the first kP2PRing messages find it free)
    if (n >= (uint32_t)kP2PRing && !p2p_wait(&mine->free_[slot][b], n - kP2PRing + 1, timeout_ticks)) {
      __hip_atomic_store(&mine->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      ok_s = 0;
    }
  }
  __syncthreads();
  // (the receiver's last reads of this slot completed before it freed it: no acquire needed
  // before overwriting; a failed wait still writes nothing)
  if (ok_s) {
    uint4* dst = ring + (int64_t)slot * slot_vec;
    for (int64_t v = (int64_t)b * kThreads + t; v < nvec; v += (int64_t)gridDim.x * kThreads) dst[v] = src[v];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope: drain + L2 write-back
  __syncthreads();
  if (t == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (ok_s) __hip_atomic_store(&peer->full[slot][b], n + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    mine->send_seq[b] = n + 1;
  }
}

// mine: this rank's ctl (its FULL words are written by the sender); peer: the sender's ctl
// (mapped: FREE words); ring: the SENDER's ring (mapped); dst: the output tensor
__global__ __launch_bounds__(kThreads) void p2p_recv_kernel(P2PCtl* mine, P2PCtl* peer, const uint4* ring,
                                                            int64_t slot_vec, uint4* dst, int64_t nvec,
                                                            uint64_t timeout_ticks) {
  const int b = blockIdx.x, t = threadIdx.x;
  __shared__ int ok_s;
  const uint32_t n = mine->recv_seq[b];
  const int slot = (int)(n % kP2PRing);
  if (t == 0) {
    ok_s = 1;
    if (!p2p_wait(&mine->full[slot][b], n + 1, timeout_ticks)) {
      __hip_atomic_store(&mine->error, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      ok_s = 0;
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // drop stale lines before the peer reads
  if (ok_s) {
    const uint4* src = ring + (int64_t)slot * slot_vec;
    for (int64_t v = (int64_t)b * kThreads + t; v < nvec; v += (int64_t)gridDim.x * kThreads) dst[v] = src[v];
  }
  // every load of the slot has returned (its data is in registers / stored) before the
  // sender may overwrite the slot
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    if (ok_s) __hip_atomic_store(&peer->free_[slot][b], n + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    mine->recv_seq[b] = n + 1;
  }
}

}  // namespace

MX_EXPORT int mx_xgmi_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }
MX_EXPORT int mx_xgmi_flags_bytes() { return (int)((sizeof(Flags) + 255) / 256 * 256); }
MX_EXPORT int mx_xgmi_max_ranks() { return kMaxRanks; }

// data: plain device memory (cached in the owner's L2; the barrier writes it back);
// flags: uncached device memory (polled across GPUs).  Both zeroed.
MX_EXPORT int mx_xgmi_alloc(int64_t data_bytes, void** data, void** flags) {
  hipError_t e = hipMalloc(data, (size_t)data_bytes);
  if (e != hipSuccess) return e;
  e = hipExtMallocWithFlags(flags, (size_t)mx_xgmi_flags_bytes(), hipDeviceMallocUncached);
  if (e != hipSuccess) return e;
  e = hipMemset(*flags, 0, (size_t)mx_xgmi_flags_bytes());
  if (e != hipSuccess) return e;
  e = hipMemset(*data, 0, (size_t)data_bytes);
  if (e != hipSuccess) return e;
  return hipDeviceSynchronize();
}

MX_EXPORT int mx_xgmi_free(void* data, void* flags) {
  hipError_t e = hipFree(data);
  hipError_t f = hipFree(flags);
  return e != hipSuccess ? e : f;
}

MX_EXPORT int mx_xgmi_get_handle(void* ptr, void* out) {
  return hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(out), ptr);
}

MX_EXPORT int mx_xgmi_open_handle(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

MX_EXPORT int mx_xgmi_close_handle(void* ptr) { return hipIpcCloseMemHandle(ptr); }

// Registration of an existing device allocation (e.g. a torch tensor from the caching
// allocator): the IPC handle names the whole underlying allocation, so the byte offset of
// ``ptr`` inside it travels with the handle and the peer adds it to its mapping.
MX_EXPORT int mx_xgmi_register(void* ptr, void* handle_out, int64_t* offset_out, int64_t* alloc_bytes) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(ptr));
  if (e != hipSuccess) return e;
  *offset_out = reinterpret_cast<char*>(ptr) - reinterpret_cast<char*>(base);
  *alloc_bytes = (int64_t)size;
  return hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle_out), reinterpret_cast<void*>(base));
}

// error word of this rank's flags (synchronous read; 0 = healthy)
MX_EXPORT int mx_xgmi_error(void* flags, uint32_t* out) {
  return hipMemcpy(out, &reinterpret_cast<Flags*>(flags)->error, 4, hipMemcpyDeviceToHost);
}

// datas / flagss: world device pointers (this rank's own + mapped peers), in rank order.
// nbytes: bytes of the full message (% 16 == 0).  bf16: reduce in bf16 (else fp32).
// Direct ops (4, 5): datas are the registered regions of this call (offset-adjusted by the
// caller); ``in`` is unused.  seq / validate: the call signature check (validation mode).
MX_EXPORT int mx_xgmi_collective(void* const* datas, void* const* flagss, int world, int rank,
                                 const void* in, void* out, int64_t nbytes, int bf16, int op,
                                 int blocks, double timeout_s, uint32_t seq, int validate,
                                 hipStream_t stream) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || nbytes % 16 || op < 0 ||
      op > kAllGatherDirect)
    return hipErrorInvalidValue;
  Sig sig = {{(uint32_t)op, (uint32_t)(nbytes & 0xffffffffu), (uint32_t)(nbytes >> 32), seq}};
  Peers pp = {};
  for (int i = 0; i < world; ++i) {
    pp.data[i] = reinterpret_cast<char*>(datas[i]);
    pp.flags[i] = reinterpret_cast<Flags*>(flagss[i]);
  }
  const int64_t nvec = nbytes / 16;
  if (blocks <= 0) {
    const int64_t want = (nvec + kThreads - 1) / kThreads;
    blocks = (int)(want < 64 ? (want < 1 ? 1 : want) : 64);
  }
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  const uint64_t ticks = (uint64_t)(timeout_s * 1e8);   // s_memrealtime: 100 MHz
  if (bf16)
    hipLaunchKernelGGL(xgmi_kernel<true>, dim3(blocks), dim3(kThreads), 0, stream, pp,
                       (const uint4*)in, (uint4*)out, nvec, rank, world, op, ticks, sig, validate);
  else
    hipLaunchKernelGGL(xgmi_kernel<false>, dim3(blocks), dim3(kThreads), 0, stream, pp,
                       (const uint4*)in, (uint4*)out, nvec, rank, world, op, ticks, sig, validate);
  return hipGetLastError();
}

// ---- point-to-point channel (see p2p_send_kernel): ring of kP2PRing slots of slot_bytes
MX_EXPORT int mx_xgmi_p2p_ring() { return kP2PRing; }
MX_EXPORT int mx_xgmi_p2p_ctl_bytes() { return (int)((sizeof(P2PCtl) + 255) / 256 * 256); }

// ring: plain device memory (kP2PRing * slot_bytes); ctl: uncached; both zeroed
MX_EXPORT int mx_xgmi_p2p_alloc(int64_t slot_bytes, void** ring, void** ctl) {
  hipError_t e = hipMalloc(ring, (size_t)slot_bytes * kP2PRing);
  if (e != hipSuccess) return e;
  e = hipExtMallocWithFlags(ctl, (size_t)mx_xgmi_p2p_ctl_bytes(), hipDeviceMallocUncached);
  if (e != hipSuccess) return e;
  e = hipMemset(*ctl, 0, (size_t)mx_xgmi_p2p_ctl_bytes());
  if (e != hipSuccess) return e;
  return hipDeviceSynchronize();
}

MX_EXPORT int mx_xgmi_p2p_error(void* ctl, uint32_t* out) {
  return hipMemcpy(out, &reinterpret_cast<P2PCtl*>(ctl)->error, 4, hipMemcpyDeviceToHost);
}

// send: mine = own ctl, peer = receiver's ctl (mapped), ring = own ring
// recv: mine = own ctl, peer = sender's ctl (mapped), ring = sender's ring (mapped)
MX_EXPORT int mx_xgmi_p2p(int is_send, void* mine, void* peer, void* ring, int64_t slot_bytes, void* buf,
                          int64_t nbytes, int blocks, double timeout_s, hipStream_t stream) {
  if (nbytes % 16 || slot_bytes % 16 || nbytes > slot_bytes || nbytes <= 0) return hipErrorInvalidValue;
  if (blocks <= 0 || blocks > kP2PBlocks) blocks = kP2PBlocks;
  const uint64_t ticks = (uint64_t)(timeout_s * 1e8);
  if (is_send)
    hipLaunchKernelGGL(p2p_send_kernel, dim3(blocks), dim3(kThreads), 0, stream, (P2PCtl*)mine, (P2PCtl*)peer,
                       (uint4*)ring, slot_bytes / 16, (const uint4*)buf, nbytes / 16, ticks);
  else
    hipLaunchKernelGGL(p2p_recv_kernel, dim3(blocks), dim3(kThreads), 0, stream, (P2PCtl*)mine, (P2PCtl*)peer,
                       (const uint4*)ring, slot_bytes / 16, (uint4*)buf, nbytes / 16, ticks);
  return hipGetLastError();
}
