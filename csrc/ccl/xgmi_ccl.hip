// Intra-node collectives over xGMI peer memory for MI355X (gfx950).
//
// The reference's allreduce jobs rely on Horovod + NCCL inside the user image (SURVEY §2.10,
// §2.12: DistributedOptimizer gradient allreduce every step). On an 8x MI355X node every GPU has a
// direct xGMI link to every other GPU, so instead of a ring (one link busy per hop) each rank
// reads its 1/W chunk from ALL peers at once, reduces it, and then every rank reads every reduced
// chunk from its owner: a "two-shot" allreduce (reduce-scatter + all-gather) in ONE kernel, using
// all W-1 links in both directions, with no host involvement (graph-capturable).
//
// Buffers are plain hipMalloc allocations shared through hipIpc handles; the barrier flags live
// in uncached memory (hipDeviceMallocUncached). Block b of every rank owns sub-range b of every
// chunk, and synchronises only with block b of the other ranks.
//
// PULL ONLY (default): no kernel stores into a peer's buffer. Data crosses xGMI only as loads of
// a peer's memory issued after a barrier whose release side (buffer_wbl2 + flag store at system
// scope) the owner passed after writing it, and whose acquire side (buffer_inv at system scope)
// the reader passed before loading it. A remote GPU's write into a cacheable allocation that the
// owner's XCD L2 may already hold is therefore never relied on -- that case cannot be exercised
// by same-GPU rehearsals, so the design avoids it instead of testing it:
//
//   copy-in (own sub-range b of every chunk) -> barrier 0 -> reduce chunk[rank] sub-range b from
//   all ranks into MY buffer -> barrier 1 -> pull chunk[q] sub-range b from rank q for every q
//   -> barrier 2 (peers finished reading my chunk before my next copy-in overwrites it)
//
// The fused optimizer kernels (Adam, sharded SGD) end on the same third barrier: without it a rank
// could leave the kernel and rewrite its buffer (a host-side copy, a checkpoint load) while a
// slower peer still pulls from it -- the per-kernel self-test caught exactly that at W = 8.
// That last barrier of every pull kernel only has to order the peers' finished loads before the
// owner's later writes, so it runs without the release / acquire fences (xbarrier<W, false>): no
// L2 write-back or invalidate on the way out of the kernel.
// The push form (owner stores its chunk into every peer's buffer, two barriers) is kept behind
// ArenaXgmiPeers::push and used only when the communicator's self-test of it passed.
//
// Why that is race-free: every remote access to a rank's buffer by block b of another rank
// happens between barriers that rank's block b also takes part in, and within a phase the
// accessed ranges (chunk[owner] sub-range b) are disjoint between ranks. Flag values are
// per-block call counters (no reset between calls).
//
// xgmi_adam fuses the gradient reduce-scatter, a sharded Adam step and the parameter all-gather:
// rank r sums chunk r of every rank's gradient, applies Adam to that chunk only (its optimizer
// state shard), writes the updated parameters into its own parameter buffer, and every rank pulls
// the other ranks' updated chunks after barrier 1 (push form: the owner stores them). Bytes on
// the wire equal one two-shot allreduce, but the optimizer pass runs on 1/W of the vector and
// the separate all-reduce + Adam launches disappear.
//
// Small vectors (<= ARENA_CCL_ONESHOT_ELEMS floats: metrics, tail buckets) take a one-shot path
// with ONE barrier instead of two: every rank stages its vector in a double-buffered tail region,
// and after the barrier reads the whole vector from all peers and reduces it locally (see
// xgmi_allreduce_oneshot_kernel for why the second barrier is not needed).
//
// Broadcast and all-gather (Horovod's broadcast_global_variables / allgather) are pure copies
// over the same registered buffers:
//   * broadcast, small vectors: direct pull -- the root stages its vector, barrier, every other
//     rank reads it over its own link, barrier. Each link carries n bytes.
//   * broadcast, large vectors: scatter + all-gather -- rank c pulls chunk c from the root into its
//     own buffer, barrier, every rank pulls chunk q from rank q, barrier. Each link carries 2n/W
//     bytes (4x less than direct pull at W = 8), for one extra barrier.
//   * all-gather: every rank stages its shard, barrier, reads shard q from rank q for all q (W
//     loads in flight per thread), barrier. Each link carries one shard.
// The last barrier of each call keeps a rank from restaging its buffer while a peer still reads
// it (the same argument as for the two-shot allreduce).
//
// Barrier waits are bounded (timeout_cycles of the 100 MHz s_memrealtime clock): a peer that never
// arrives sets *err and the kernel drains instead of hanging the GPU; the host checks err.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "abi.h"
#include "adam.h"

using namespace arena;

namespace {

constexpr int kThreads = 256;
constexpr int kMaxB = ARENA_CCL_MAX_BLOCKS;
constexpr int kMaxR = ARENA_CCL_MAX_RANKS;

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// FENCE = false: a "readers are done" barrier (the last one of a pull kernel). It publishes
// nothing -- no peer reads anything this rank wrote since the previous barrier before the next
// call's first barrier, which has its own release -- and acquires nothing, so it skips the L2
// write-back and invalidate and only orders every peer's completed loads of this rank's buffers
// before this rank's later writes to them. Its loads have all returned when the flag goes out:
// each pulled value was stored before the block's s_barrier, which waits for vmcnt(0).
template <int W, bool FENCE = true>
__device__ __forceinline__ void xbarrier(const ArenaXgmiPeers& P, int phase, int b, uint32_t e) {
  // every wave's stores have completed (hipcc emits vmcnt(0) before s_barrier)
  __syncthreads();
  if (threadIdx.x < 64) {
    // ONE system-scope release per block (buffer_wbl2: our stores reach memory before the flags),
    // flags written and polled with relaxed system-scope accesses to uncached memory, then ONE
    // acquire (buffer_inv). An acquire per poll would invalidate L2 on every spin iteration.
    if constexpr (FENCE) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      // the write-back must complete before the flag goes out: hipcc drops the vmcnt(0) after
      // buffer_wbl2 whenever the scoreboard is provably empty (MI355X_MICROARCH.md, compiler
      // hazard)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const int t = threadIdx.x;
    if (t < W) {
      const int slot = (phase * kMaxB + b) * kMaxR;
      __hip_atomic_store(P.sig[t] + slot + P.rank, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const uint32_t* mine = P.sig[P.rank] + slot + t;
      const long long t0 = wall_clock64();
      while ((int)(__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
        if (wall_clock64() - t0 > P.timeout_cycles) {
          __hip_atomic_store(P.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if constexpr (FENCE) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      // buffer_inv completes asynchronously: hold the barrier until it has, or the block's other
      // waves could load the peers' data through a not-yet-invalidated L1 (MI355X_MICROARCH.md)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
}

// float4 slots per thread per reduce round: a block of kThreads covers kU * 4 * kThreads floats
// with one xGMI round trip per thread (g_block_elems = 4096 -> one round). At W = 8 the fused
// Adam kernel holds kU * (W + 3) float4 operands in flight: 256 VGPRs, no scratch (checked with
// -Rpass-analysis=kernel-resource-usage).
constexpr int kU = 4;

// dst[c*L + o] = src[c*L + o] for all chunks c, W loads in flight per thread.
template <int W>
__device__ __forceinline__ void copy_chunks(float* __restrict__ dst, const float* __restrict__ src,
                                            long long n, long long L, long long lo, long long hi) {
  for (long long o = lo + threadIdx.x * 4; o < hi; o += kThreads * 4) {
    float4 v[W];
#pragma unroll
    for (int c = 0; c < W; ++c) {
      const long long i = (long long)c * L + o;
      if (i < n) v[c] = ld4(src + i);
    }
#pragma unroll
    for (int c = 0; c < W; ++c) {
      const long long i = (long long)c * L + o;
      if (i < n) st4(dst + i, v[c]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Copies between registered buffers: U float4 slots per thread, all loads before any store.
template <int NSRC>
__device__ __forceinline__ void pull_range(float* const* dst, const float* const* src,
                                           const long long* dst_off, const long long* src_off,
                                           long long lo, long long hi, const long long* lim) {
  constexpr int U = kU;
  for (long long o0 = lo + threadIdx.x * 4; o0 < hi; o0 += (long long)kThreads * 4 * U) {
    float4 v[U][NSRC];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long o = o0 + (long long)u * kThreads * 4;
#pragma unroll
      for (int q = 0; q < NSRC; ++q)
        if (o < hi && o < lim[q]) v[u][q] = ld4(src[q] + src_off[q] + o);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long o = o0 + (long long)u * kThreads * 4;
#pragma unroll
      for (int q = 0; q < NSRC; ++q)
        if (o < hi && o < lim[q]) st4(dst[q] + dst_off[q] + o, v[u][q]);
    }
  }
}

// Phase 2 of the pull protocol: after barrier 1 every owner q holds its finished chunk q in its
// OWN buffer `src[q] + base`; this rank copies chunk q (sub-range [lo, hi) of it) from rank q
// into `dst + base` for every q, skipping its own chunk when dst is its own buffer. Chunks are L
// units long; elements at or past n do not exist. One load per link in flight per slot.
template <int W>
__device__ __forceinline__ void pull_chunks(float* dst, float* const* src, long long base,
                                            long long n, long long L, long long lo, long long hi,
                                            int rank, bool skip_own) {
  float* d[W];
  const float* sp[W];
  long long off[W], lim[W];
#pragma unroll
  for (int q = 0; q < W; ++q) {
    d[q] = dst;
    sp[q] = src[q];
    off[q] = base + (long long)q * L;
    lim[q] = (skip_own && q == rank) ? 0 : n - (long long)q * L;
  }
  pull_range<W>(d, sp, off, off, lo, hi, lim);
}

template <int W>
__global__ __launch_bounds__(kThreads) void xgmi_allreduce_kernel(ArenaXgmiPeers P,
                                                                   const float* __restrict__ in,
                                                                   float* __restrict__ out,
                                                                   long long n, long long L,
                                                                   long long S, float scale) {
  const int b = blockIdx.x;
  const uint32_t e = P.epoch[b] + 1;
  float* mine = P.buf[P.rank];
  const long long lo = (long long)b * S;
  const long long hi = std::min(lo + S, L);
  if (in != mine) copy_chunks<W>(mine, in, n, L, lo, hi);
  xbarrier<W>(P, 0, b, e);
  const long long base = (long long)P.rank * L;
  constexpr int U = kU;
  for (long long o0 = lo + threadIdx.x * 4; o0 < hi; o0 += (long long)kThreads * 4 * U) {
    // every remote load of this thread's U float4 slots is issued before the first store (the
    // stores may alias the loads, so the compiler cannot hoist the next slot's loads above them):
    // ONE xGMI round trip per thread instead of one per slot
    float4 v[U][W];
    bool ok[U];
    long long idx[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long o = o0 + (long long)u * kThreads * 4;
      ok[u] = o < hi && base + o < n;
      idx[u] = ok[u] ? base + o : 0;  // clamped, branch-free loads
#pragma unroll
      for (int q = 0; q < W; ++q) v[u][q] = ld4(P.buf[q] + idx[u]);  // one load per link
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float4 acc = v[u][0];
#pragma unroll
      for (int q = 1; q < W; ++q) acc = add4(acc, v[u][q]);  // fixed order: same on all ranks
      acc.x *= scale; acc.y *= scale; acc.z *= scale; acc.w *= scale;
      if (ok[u]) {
        if (P.push) {
#pragma unroll
          for (int q = 0; q < W; ++q) st4(P.buf[q] + idx[u], acc);
        } else {
          st4(mine + idx[u], acc);  // the owner's chunk stays home; peers pull it below
        }
      }
    }
  }
  xbarrier<W>(P, 1, b, e);
  if (P.push) {
    if (out != mine) copy_chunks<W>(out, mine, n, L, lo, hi);
  } else {
    pull_chunks<W>(out, P.buf, 0, n, L, lo, hi, P.rank, out == mine);
    // peers read my chunk until here: the next call's copy-in must not overwrite it earlier
    xbarrier<W, false>(P, 2, b, e);
  }
  if (threadIdx.x == 0) P.epoch[b] = e;
}

// One-shot: block b owns floats [b*kOneSub, (b+1)*kOneSub) of the vector, one float4 per thread.
// Stage into tail half (e & 1), barrier, read that slot from all W ranks, reduce, store locally.
//
// Why one barrier is enough: block b of every rank reads my half-p slot b only between its
// barrier of call e and its exit. I write that slot again at call e + 2 at the earliest (the half
// flips every call of block b), and between the two I pass block b's barrier of call e + 1 (of
// whatever kind), which needs block b of every peer to have arrived there, i.e. to have finished
// call e. Only block b ever touches slot b of the tail; the two-shot and Adam kernels stay below
// buf_elems. Per-block counters are equal on all ranks because every rank issues the same calls.
constexpr int kOneSub = kThreads * 4;

template <int W>
__global__ __launch_bounds__(kThreads) void xgmi_allreduce_oneshot_kernel(ArenaXgmiPeers P,
                                                                           const float* __restrict__ in,
                                                                           float* __restrict__ out,
                                                                           long long n, float scale) {
  const int b = blockIdx.x;
  const uint32_t e = P.epoch[b] + 1;
  const long long tail = P.buf_elems + (long long)(e & 1) * ARENA_CCL_ONESHOT_ELEMS;
  const long long o = (long long)b * kOneSub + threadIdx.x * 4;
  const bool ok = o < n;
  if (ok) st4(P.buf[P.rank] + tail + o, ld4(in + o));
  xbarrier<W>(P, 0, b, e);
  if (ok) {
    float4 v[W];
#pragma unroll
    for (int q = 0; q < W; ++q) v[q] = ld4(P.buf[q] + tail + o);  // W loads in flight
    float4 acc = v[0];
#pragma unroll
    for (int q = 1; q < W; ++q) acc = add4(acc, v[q]);  // same order as the two-shot kernel
    acc.x *= scale; acc.y *= scale; acc.z *= scale; acc.w *= scale;
    st4(out + o, acc);
  }
  if (threadIdx.x == 0) P.epoch[b] = e;
}

template <int W>
__global__ __launch_bounds__(kThreads) void xgmi_adam_kernel(ArenaXgmiPeers P, float* __restrict__ M,
                                                              float* __restrict__ V, long long n,
                                                              long long L, long long S, ArenaAdam a,
                                                              ArenaCounterOp ctr) {
  const int b = blockIdx.x;
  const uint32_t e = P.epoch[b] + 1;
  const AdamCoef co = adam_coef(a);  // t / lr loads issued before the barrier wait
  const long long lo = (long long)b * S;
  const long long hi = std::min(lo + S, L);
  xbarrier<W>(P, 0, b, e);
  const long long base = (long long)P.rank * L;
  float* Pm = P.buf2[P.rank];
  constexpr int U = kU;
  for (long long o0 = lo + threadIdx.x * 4; o0 < hi; o0 += (long long)kThreads * 4 * U) {
    // all loads of the thread's U slots (W remote gradients + local P/M/V each) before any store
    float4 v[U][W], p[U], m[U], s[U];
    bool ok[U];
    long long idx[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long o = o0 + (long long)u * kThreads * 4;
      ok[u] = o < hi && base + o < n;
      idx[u] = ok[u] ? base + o : 0;
#pragma unroll
      for (int q = 0; q < W; ++q) v[u][q] = ld4(P.buf[q] + idx[u]);
      p[u] = ld4(Pm + idx[u]);
      m[u] = ld4(M + idx[u]);
      s[u] = ld4(V + idx[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float4 g = v[u][0];
#pragma unroll
      for (int q = 1; q < W; ++q) g = add4(g, v[u][q]);
      adam_apply(co, g.x, p[u].x, m[u].x, s[u].x);
      adam_apply(co, g.y, p[u].y, m[u].y, s[u].y);
      adam_apply(co, g.z, p[u].z, m[u].z, s[u].z);
      adam_apply(co, g.w, p[u].w, m[u].w, s[u].w);
      if (ok[u]) {
        st4(M + idx[u], m[u]);
        st4(V + idx[u], s[u]);
        if (P.push) {
#pragma unroll
          for (int q = 0; q < W; ++q) st4(P.buf2[q] + idx[u], p[u]);
        } else {
          st4(Pm + idx[u], p[u]);
        }
      }
    }
  }
  xbarrier<W>(P, 1, b, e);
  // pull: every other chunk from its owner, then a third barrier, so that when this kernel ends on
  // any rank no peer still reads its buffers (the owner may rewrite them by any means afterwards:
  // the next step's gradients, a checkpoint load, a host-side copy)
  if (!P.push) {
    pull_chunks<W>(Pm, P.buf2, 0, n, L, lo, hi, P.rank, true);
    xbarrier<W, false>(P, 2, b, e);
  }
  counter_op(ctr);
  if (threadIdx.x == 0) P.epoch[b] = e;
}

// Direct-pull broadcast: block b moves floats [b*S, b*S+S) of the vector.
template <int W>
__global__ __launch_bounds__(kThreads) void xgmi_bcast_direct_kernel(ArenaXgmiPeers P,
                                                                      const float* __restrict__ in,
                                                                      float* __restrict__ out,
                                                                      long long n, int root,
                                                                      long long S) {
  const int b = blockIdx.x;
  const uint32_t e = P.epoch[b] + 1;
  const long long lo = (long long)b * S;
  const long long hi = std::min(lo + S, n);
  const long long zero = 0;
  const float* src_in = in;  // (restrict-qualified parameters do not bind to T* const*)
  float* dst_out = out;
  if (P.rank == root && in != P.buf[root]) {
    float* d = P.buf[root];
    pull_range<1>(&d, &src_in, &zero, &zero, lo, hi, &n);
  }
  xbarrier<W>(P, 0, b, e);
  if (P.rank != root) {
    const float* src = P.buf[root];
    pull_range<1>(&dst_out, &src, &zero, &zero, lo, hi, &n);   // over the link to the root
  } else if (out != in) {
    pull_range<1>(&dst_out, &src_in, &zero, &zero, lo, hi, &n);
  }
  xbarrier<W, false>(P, 1, b, e);
  if (threadIdx.x == 0) P.epoch[b] = e;
}

// Scatter + all-gather broadcast: chunk c = [c*L, (c+1)*L); block b owns sub-range
// [b*S, b*S+S) of every chunk.
template <int W>
__global__ __launch_bounds__(kThreads) void xgmi_bcast_twoshot_kernel(ArenaXgmiPeers P,
                                                                       const float* __restrict__ in,
                                                                       float* __restrict__ out,
                                                                       long long n, int root,
                                                                       long long L, long long S) {
  const int b = blockIdx.x;
  const uint32_t e = P.epoch[b] + 1;
  const long long lo = (long long)b * S;
  const long long hi = std::min(lo + S, L);
  const int r = P.rank;
  if (r == root && in != P.buf[root]) copy_chunks<W>(P.buf[root], in, n, L, lo, hi);
  xbarrier<W>(P, 0, b, e);
  if (r != root) {  // scatter: my chunk from the root, into my own buffer
    float* d = P.buf[r];
    const float* src = P.buf[root];
    const long long off = (long long)r * L;
    const long long lim = n - off;
    pull_range<1>(&d, &src, &off, &off, lo, hi, &lim);
  }
  xbarrier<W>(P, 1, b, e);
  if (r != root) {  // all-gather: chunk q from rank q (the root's chunk from the root)
    float* dst[W];
    const float* src[W];
    long long off[W], lim[W];
#pragma unroll
    for (int q = 0; q < W; ++q) {
      dst[q] = out;
      src[q] = P.buf[q];
      off[q] = (long long)q * L;
      // my own chunk is already in place when the destination is my staging buffer
      lim[q] = (q == r && out == P.buf[r]) ? 0 : n - off[q];
    }
    pull_range<W>(dst, src, off, off, lo, hi, lim);
  } else if (out != in) {
    copy_chunks<W>(out, in, n, L, lo, hi);
  }
  xbarrier<W, false>(P, 2, b, e);
  if (threadIdx.x == 0) P.epoch[b] = e;
}

// All-gather: out[q*m + j] = shard of rank q; block b moves floats [b*S, b*S+S) of every shard.
template <int W>
__global__ __launch_bounds__(kThreads) void xgmi_allgather_kernel(ArenaXgmiPeers P,
                                                                   const float* __restrict__ in,
                                                                   float* __restrict__ out,
                                                                   long long m, long long S) {
  const int b = blockIdx.x;
  const uint32_t e = P.epoch[b] + 1;
  const long long lo = (long long)b * S;
  const long long hi = std::min(lo + S, m);
  const long long zero = 0;
  float* mine = P.buf[P.rank];
  const float* src_in = in;
  if (in != mine) pull_range<1>(&mine, &src_in, &zero, &zero, lo, hi, &m);
  xbarrier<W>(P, 0, b, e);
  float* dst[W];
  const float* src[W];
  long long doff[W], soff[W], lim[W];
#pragma unroll
  for (int q = 0; q < W; ++q) {
    dst[q] = out;
    src[q] = P.buf[q];
    doff[q] = (long long)q * m;
    soff[q] = 0;
    lim[q] = m;
  }
  pull_range<W>(dst, src, doff, soff, lo, hi, lim);
  xbarrier<W, false>(P, 1, b, e);
  if (threadIdx.x == 0) P.epoch[b] = e;
}

// ---------------------------------------------------------------------------------------------
// Sharded momentum SGD on bf16 weights with fp32 masters (data-parallel CNN training):
//   reduce-scatter of the bf16 gradients (fp32 sums, fixed rank order) -> SGD on the owned chunk
//   of the fp32 master weights and momentum -> all-gather of the rounded bf16 weights into every
//   rank's weight buffer (buf2), one kernel per gradient bucket.
// Element units are bf16; a bucket [off, off + n) is split into W chunks of L (multiple of 8),
// block b owns sub-range [b*S, b*S + S) of every chunk. Same update as mt_sgd_master
// (torch.optim.SGD, dampening 0): d = g + wd*w; m = mu*m + d; w -= lr*m. Masters/momentum are
// full-length arrays of which each rank only ever updates its own chunks.
__device__ __forceinline__ float bf_lo(uint32_t v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf_hi(uint32_t v) { return __uint_as_float(v & 0xffff0000u); }
__device__ __forceinline__ uint32_t to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);                                  // round to nearest even
  return u >> 16;
}

struct SgdCoef {
  float lr, mu, wd, scale;
};

__device__ __forceinline__ void sgd1(const SgdCoef& c, float g, float& w, float& m) {
  const float d = g * c.scale + c.wd * w;
  m = c.mu * m + d;
  w = w - c.lr * m;
}

template <int W>
__global__ __launch_bounds__(kThreads) void xgmi_sgd_bf16_kernel(ArenaXgmiPeers P,
                                                                  float* __restrict__ master,
                                                                  float* __restrict__ mom,
                                                                  long long off, long long n,
                                                                  long long L, long long S,
                                                                  SgdCoef c) {
  const int b = blockIdx.x;
  const uint32_t e = P.epoch[b] + 1;
  const long long lo = (long long)b * S;
  const long long hi = std::min(lo + S, L);
  xbarrier<W>(P, 0, b, e);
  const long long base = (long long)P.rank * L;
  constexpr int U = 2;  // 8 bf16 per slot: U * (W + 4) 16-byte operands in flight per thread
  for (long long o0 = lo + threadIdx.x * 8; o0 < hi; o0 += (long long)kThreads * 8 * U) {
    uint4 g[U][W];
    float4 w[U][2], m[U][2];
    bool ok[U];
    long long idx[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long o = o0 + (long long)u * kThreads * 8;
      ok[u] = o < hi && base + o < n;
      idx[u] = off + (ok[u] ? base + o : 0);
#pragma unroll
      for (int q = 0; q < W; ++q)
        g[u][q] = *reinterpret_cast<const uint4*>(
            reinterpret_cast<const uint16_t*>(P.buf[q]) + idx[u]);
      w[u][0] = ld4(master + idx[u]);
      w[u][1] = ld4(master + idx[u] + 4);
      m[u][0] = ld4(mom + idx[u]);
      m[u][1] = ld4(mom + idx[u] + 4);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float acc[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t x = (&g[u][0].x)[k];
        acc[2 * k] = bf_lo(x);
        acc[2 * k + 1] = bf_hi(x);
      }
#pragma unroll
      for (int q = 1; q < W; ++q) {  // fixed order: identical on every rank
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t x = (&g[u][q].x)[k];
          acc[2 * k] += bf_lo(x);
          acc[2 * k + 1] += bf_hi(x);
        }
      }
      float* wv = &w[u][0].x;
      float* mv = &m[u][0].x;
#pragma unroll
      for (int k = 0; k < 8; ++k) sgd1(c, acc[k], wv[k], mv[k]);
      uint4 packed;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        (&packed.x)[k] = to_bf16(wv[2 * k]) | (to_bf16(wv[2 * k + 1]) << 16);
      if (ok[u]) {
        st4(master + idx[u], w[u][0]);
        st4(master + idx[u] + 4, w[u][1]);
        st4(mom + idx[u], m[u][0]);
        st4(mom + idx[u] + 4, m[u][1]);
        if (P.push) {
#pragma unroll
          for (int q = 0; q < W; ++q)
            *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(P.buf2[q]) + idx[u]) = packed;
        } else {
          *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(P.buf2[P.rank]) + idx[u]) = packed;
        }
      }
    }
  }
  xbarrier<W>(P, 1, b, e);
  // pull the other chunks in float units (off, n, L, S are multiples of 8 bf16 = 4 floats), then
  // the end barrier (see xgmi_adam_kernel)
  if (!P.push) {
    pull_chunks<W>(P.buf2[P.rank], P.buf2, off / 2, n / 2, L / 2, lo / 2, hi / 2, P.rank, true);
    xbarrier<W, false>(P, 2, b, e);
  }
  if (threadIdx.x == 0) P.epoch[b] = e;
}

// The fp32 tail of the same optimizer (BatchNorm scales/shifts, biases: ~0.1 M values in a
// ResNet-50): fp32 gradients staged at buf[off, off + n) of every rank are reduce-scattered (fixed
// rank order), momentum SGD runs on the owned chunk of the fp32 weights -- which live in buf2 and
// ARE the masters (no rounding on the way out) -- and the chunk is written to every rank's buf2.
// `mom` is indexed relative to the bucket (mom[0] <-> element off). Element units are floats.
template <int W>
__global__ __launch_bounds__(kThreads) void xgmi_sgd_f32_kernel(ArenaXgmiPeers P,
                                                                 float* __restrict__ mom,
                                                                 long long off, long long n,
                                                                 long long L, long long S,
                                                                 SgdCoef c) {
  const int b = blockIdx.x;
  const uint32_t e = P.epoch[b] + 1;
  const long long lo = (long long)b * S;
  const long long hi = std::min(lo + S, L);
  xbarrier<W>(P, 0, b, e);
  const long long base = (long long)P.rank * L;
  const float* wmine = P.buf2[P.rank];
  constexpr int U = kU;
  for (long long o0 = lo + threadIdx.x * 4; o0 < hi; o0 += (long long)kThreads * 4 * U) {
    float4 v[U][W], w[U], m[U];
    bool ok[U];
    long long idx[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long o = o0 + (long long)u * kThreads * 4;
      ok[u] = o < hi && base + o < n;
      idx[u] = ok[u] ? base + o : 0;
#pragma unroll
      for (int q = 0; q < W; ++q) v[u][q] = ld4(P.buf[q] + off + idx[u]);
      w[u] = ld4(wmine + off + idx[u]);
      m[u] = ld4(mom + idx[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float4 g = v[u][0];
#pragma unroll
      for (int q = 1; q < W; ++q) g = add4(g, v[u][q]);  // fixed order: identical on every rank
      sgd1(c, g.x, w[u].x, m[u].x);
      sgd1(c, g.y, w[u].y, m[u].y);
      sgd1(c, g.z, w[u].z, m[u].z);
      sgd1(c, g.w, w[u].w, m[u].w);
      if (ok[u]) {
        st4(mom + idx[u], m[u]);
        if (P.push) {
#pragma unroll
          for (int q = 0; q < W; ++q) st4(P.buf2[q] + off + idx[u], w[u]);
        } else {
          st4(P.buf2[P.rank] + off + idx[u], w[u]);
        }
      }
    }
  }
  xbarrier<W>(P, 1, b, e);
  if (!P.push) {   // pull, then the end barrier (see xgmi_adam_kernel)
    pull_chunks<W>(P.buf2[P.rank], P.buf2, off, n, L, lo, hi, P.rank, true);
    xbarrier<W, false>(P, 2, b, e);
  }
  if (threadIdx.x == 0) P.epoch[b] = e;
}

// Floats of a chunk per block. Every block pays two cross-rank barriers (one L2 writeback + one
// invalidate each), so blocks are made fat rather than numerous; tunable for sweeps.
long long g_block_elems = 4096;
// Blocks per collective launch (<= kMaxB, the flag slots). Every block of a launch meets the
// blocks of the same index on every rank at its barriers, so all ranks' blocks must be able to
// run at once. With one rank per GPU that is each GPU's own launch; when several ranks share a
// GPU (same-device rehearsals of a W-GPU node) their launches must fit on it TOGETHER: XgmiComm
// lowers the cap to 128 / W there (8 ranks x 256 blocks starved each other until the barrier
// timeouts -- a 32 MB broadcast at W = 8 hung for minutes and returned partial copies).
int g_max_blocks = kMaxB;
// Crossover measured on 1x MI355X, 2 ranks (profiles/r1_ccl_oneshot_ab.jsonl): one-shot 3.0 vs
// 3.7 us at 4 KB, 3.56 vs 3.97 us at 16 KB, but 4.5 vs 4.26 us at 64 KB. One-shot also moves
// (W-1) x n bytes per rank over the links instead of 2 (W-1)/W x n, so the default stays at 32 KB.
long long g_oneshot_max = ARENA_CCL_ONESHOT_ELEMS / 2;
static_assert(ARENA_CCL_ONESHOT_ELEMS / kOneSub <= kMaxB, "one-shot blocks exceed the flag slots");

// Broadcasts up to this many floats pull directly from the root (one barrier less); above it the
// scatter + all-gather form moves 2/W of the bytes per link. W = 2 always pulls directly.
long long g_bcast_direct_max = 128 << 10;

void range_geometry(long long n, long long* S, int* nb) {
  int blocks = (int)std::min<long long>(
      g_max_blocks, std::max<long long>(1, (n + g_block_elems - 1) / g_block_elems));
  long long s = (n + blocks - 1) / blocks;
  s = (s + 3) / 4 * 4;
  *S = s;
  *nb = blocks;
}

void geometry(long long n, int W, long long* L, long long* S, int* nb) {
  long long l = (n + W - 1) / W;
  l = (l + 3) / 4 * 4;
  int blocks = (int)std::min<long long>(
      g_max_blocks, std::max<long long>(1, (l + g_block_elems - 1) / g_block_elems));
  long long s = (l + blocks - 1) / blocks;
  s = (s + 3) / 4 * 4;
  *L = l;
  *S = s;
  *nb = blocks;
}

}  // namespace

extern "C" {

hipError_t arena_ccl_malloc(void** p, size_t bytes, int uncached) {
  if (uncached) return hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached);
  return hipMalloc(p, bytes);
}

hipError_t arena_ccl_free(void* p) { return hipFree(p); }

hipError_t arena_ccl_memset(void* p, int v, size_t bytes) {
  hipError_t e = hipMemset(p, v, bytes);
  if (e != hipSuccess) return e;
  return hipDeviceSynchronize();
}

hipError_t arena_ccl_ipc_get(void* p, void* handle) {
  return hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle), p);
}

hipError_t arena_ccl_ipc_open(const void* handle, void** p) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof h);
  return hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess);
}

hipError_t arena_ccl_ipc_close(void* p) { return hipIpcCloseMemHandle(p); }

#define ARENA_CCL_DISPATCH(W, KERNEL, ...)                                                   \
  switch (W) {                                                                               \
    case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;                              \
    case 3: hipLaunchKernelGGL(KERNEL<3>, __VA_ARGS__); break;                              \
    case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;                              \
    case 5: hipLaunchKernelGGL(KERNEL<5>, __VA_ARGS__); break;                              \
    case 6: hipLaunchKernelGGL(KERNEL<6>, __VA_ARGS__); break;                              \
    case 7: hipLaunchKernelGGL(KERNEL<7>, __VA_ARGS__); break;                              \
    case 8: hipLaunchKernelGGL(KERNEL<8>, __VA_ARGS__); break;                              \
    default: return hipErrorInvalidValue;                                                    \
  }

hipError_t arena_ccl_allreduce(const ArenaXgmiPeers* P, const float* in, float* out, long long n,
                               float scale, hipStream_t stream) {
  const int W = P->world;
  if (W < 2 || W > kMaxR || n <= 0 || n % 4 || n > P->buf_elems) return hipErrorInvalidValue;
  if (n <= g_oneshot_max) {
    const int nb = (int)((n + kOneSub - 1) / kOneSub);
    ARENA_CCL_DISPATCH(W, xgmi_allreduce_oneshot_kernel, dim3(nb), dim3(kThreads), 0, stream, *P,
                       in, out, n, scale);
    return hipGetLastError();
  }
  long long L, S;
  int nb;
  geometry(n, W, &L, &S, &nb);
  ARENA_CCL_DISPATCH(W, xgmi_allreduce_kernel, dim3(nb), dim3(kThreads), 0, stream, *P, in, out,
                     n, L, S, scale);
  return hipGetLastError();
}

// Largest vector (floats) that takes the one-shot kernel; 0 forces two-shot (for A/B sweeps).
void arena_ccl_set_oneshot_max(long long e) {
  g_oneshot_max = e < 0 ? 0 : std::min<long long>(e, ARENA_CCL_ONESHOT_ELEMS);
}
long long arena_ccl_get_oneshot_max() { return g_oneshot_max; }

hipError_t arena_ccl_adam(const ArenaXgmiPeers* P, float* M, float* V, long long n, ArenaAdam a,
                          ArenaCounterOp ctr, hipStream_t stream) {
  const int W = P->world;
  if (W < 2 || W > kMaxR || n <= 0 || n % 4 || n > P->buf_elems || n > P->buf2_elems)
    return hipErrorInvalidValue;
  long long L, S;
  int nb;
  geometry(n, W, &L, &S, &nb);
  ARENA_CCL_DISPATCH(W, xgmi_adam_kernel, dim3(nb), dim3(kThreads), 0, stream, *P, M, V, n, L, S,
                     a, ctr);
  return hipGetLastError();
}

void arena_ccl_set_block_elems(long long e) { g_block_elems = e < 256 ? 256 : e; }
void arena_ccl_set_max_blocks(int b) { g_max_blocks = b < 1 ? 1 : (b > kMaxB ? kMaxB : b); }

// Broadcast n floats (n % 4 == 0, n <= buf_elems) from `root`: in = the root's source, out =
// every rank's destination (in == out is allowed; non-roots ignore in).
hipError_t arena_ccl_broadcast(const ArenaXgmiPeers* P, const float* in, float* out, long long n,
                               int root, hipStream_t stream) {
  const int W = P->world;
  if (W < 2 || W > kMaxR || n <= 0 || n % 4 || n > P->buf_elems || root < 0 || root >= W)
    return hipErrorInvalidValue;
  if (W == 2 || n <= g_bcast_direct_max) {
    long long S;
    int nb;
    range_geometry(n, &S, &nb);
    ARENA_CCL_DISPATCH(W, xgmi_bcast_direct_kernel, dim3(nb), dim3(kThreads), 0, stream, *P, in,
                       out, n, root, S);
    return hipGetLastError();
  }
  long long L, S;
  int nb;
  geometry(n, W, &L, &S, &nb);
  ARENA_CCL_DISPATCH(W, xgmi_bcast_twoshot_kernel, dim3(nb), dim3(kThreads), 0, stream, *P, in,
                     out, n, root, L, S);
  return hipGetLastError();
}

void arena_ccl_set_bcast_direct_max(long long e) { g_bcast_direct_max = e < 0 ? 0 : e; }

// Chunking of a sharded-SGD bucket (bf16 elements): L per rank (multiple of 8), S per block.
void sgd_geometry(long long n, int W, long long* L, long long* S, int* nb) {
  long long l = (n + W - 1) / W;
  l = (l + 7) / 8 * 8;
  const long long per_block = std::max<long long>(8, g_block_elems * 2);  // bytes as the fp32 path
  int blocks = (int)std::min<long long>(g_max_blocks,
                                        std::max<long long>(1, (l + per_block - 1) / per_block));
  long long s = (l + blocks - 1) / blocks;
  s = (s + 7) / 8 * 8;
  *L = l;
  *S = s;
  *nb = blocks;
}

// One bucket [off, off + n) (bf16 elements, off and n multiples of 8) of the sharded SGD: bf16
// grads staged in every rank's buf, bf16 weights in every rank's buf2, fp32 master/mom local.
hipError_t arena_ccl_sgd_bf16(const ArenaXgmiPeers* P, float* master, float* mom, long long off,
                              long long n, float lr, float momentum, float wd, float scale,
                              hipStream_t stream) {
  const int W = P->world;
  if (W < 2 || W > kMaxR || n <= 0 || off < 0 || n % 8 || off % 8 || P->buf2[0] == nullptr)
    return hipErrorInvalidValue;
  if ((off + n + 1) / 2 > P->buf_elems || (off + n + 1) / 2 > P->buf2_elems)
    return hipErrorInvalidValue;
  long long L, S;
  int nb;
  sgd_geometry(n, W, &L, &S, &nb);
  SgdCoef c{lr, momentum, wd, scale};
  ARENA_CCL_DISPATCH(W, xgmi_sgd_bf16_kernel, dim3(nb), dim3(kThreads), 0, stream, *P, master, mom,
                     off, n, L, S, c);
  return hipGetLastError();
}

// The [lo, hi) bf16 elements of bucket [off, off + n) whose masters rank r updates.
void arena_ccl_sgd_shard(long long off, long long n, int world, int r, long long* lo,
                         long long* hi) {
  long long L, S;
  int nb;
  sgd_geometry(n, world, &L, &S, &nb);
  *lo = off + std::min(n, (long long)r * L);
  *hi = off + std::min(n, (long long)(r + 1) * L);
}

// One fp32 bucket [off, off + n) (floats, multiples of 4) of the sharded SGD: fp32 grads staged in
// every rank's buf, fp32 weights (= masters) in every rank's buf2, momentum local (bucket-relative).
hipError_t arena_ccl_sgd_f32(const ArenaXgmiPeers* P, float* mom, long long off, long long n,
                             float lr, float momentum, float wd, float scale, hipStream_t stream) {
  const int W = P->world;
  if (W < 2 || W > kMaxR || n <= 0 || off < 0 || n % 4 || off % 4 || P->buf2[0] == nullptr)
    return hipErrorInvalidValue;
  if (off + n > P->buf_elems || off + n > P->buf2_elems) return hipErrorInvalidValue;
  long long L, S;
  int nb;
  geometry(n, W, &L, &S, &nb);
  SgdCoef c{lr, momentum, wd, scale};
  ARENA_CCL_DISPATCH(W, xgmi_sgd_f32_kernel, dim3(nb), dim3(kThreads), 0, stream, *P, mom, off, n,
                     L, S, c);
  return hipGetLastError();
}

// The [lo, hi) floats of fp32 bucket [off, off + n) whose weights/momentum rank r updates.
void arena_ccl_sgd_f32_shard(long long off, long long n, int world, int r, long long* lo,
                             long long* hi) {
  long long L, S;
  int nb;
  geometry(n, world, &L, &S, &nb);
  *lo = off + std::min(n, (long long)r * L);
  *hi = off + std::min(n, (long long)(r + 1) * L);
}

// All-gather m floats per rank (m % 4 == 0, m <= buf_elems) into out[W * m].
hipError_t arena_ccl_allgather(const ArenaXgmiPeers* P, const float* in, float* out, long long m,
                               hipStream_t stream) {
  const int W = P->world;
  if (W < 2 || W > kMaxR || m <= 0 || m % 4 || m > P->buf_elems) return hipErrorInvalidValue;
  long long S;
  int nb;
  range_geometry(m, &S, &nb);
  ARENA_CCL_DISPATCH(W, xgmi_allgather_kernel, dim3(nb), dim3(kThreads), 0, stream, *P, in, out,
                     m, S);
  return hipGetLastError();
}

// The slice of the flat vector whose optimizer state rank `r` owns under arena_ccl_adam.
void arena_ccl_shard(long long n, int world, int r, long long* lo, long long* hi) {
  long long L, S;
  int nb;
  geometry(n, world, &L, &S, &nb);
  *lo = std::min(n, (long long)r * L);
  *hi = std::min(n, (long long)(r + 1) * L);
}

}  // extern "C"
