// Fused training BatchNorm (+ residual add) (+ ReLU) for NHWC activations on gfx950 (MI355X).
//
// The ResNet workload of the Horovod demo family (arena_amd/examples/cnn_bench.py) spends more
// than half of its GPU time outside the convolutions when BatchNorm, ReLU and the residual add
// run as separate library/elementwise kernels (profiles/r1_resnet50_steady_kernels.csv: MIOpen
// BN 34 %, elementwise 21 %). Every one of those ops is HBM-bound, so the win is in passes over
// memory. Per BN layer these kernels make:
//
//   forward   stats      1 read of x            -> per-channel mean / invstd (+ running stats)
//             apply      1 read of x (+ res), 1 write of y = act(x*scale + shift (+ res))
//   backward  reduce     1 read of dy, x (+ mask bits) -> dgamma, dbeta and the dx coefficients
//             dx         1 read of dy, x (+ mask bits), 1 write of dx (+ 1 write of dres = the
//                        masked dy)
//
// The ReLU mask (y > 0) is written by the apply pass as one bit per element (a byte per 8-channel
// vector): the backward passes read M*C/8 bytes instead of re-reading the bf16 output y, which
// removes one of the three input streams of the reduction and one of the four of the dx pass.
//
// Layout: x is [M][C] with M = N*H*W (a channels_last tensor) and C % 8 == 0, C <= 2048.
// A thread owns 8 consecutive channels: one 16-byte load for bf16, two for fp32.
// A 256-thread block covers 256 / (C/8) rows per round.
// Reductions:
//   * per-thread Welford (stats) or plain fp32 sums (backward: x - mean uses the exact forward
//     mean, so nothing cancels);
//   * Chan merges across the block's row slots in LDS;
//   * per-block partials in a workspace;
//   * a finalize kernel with one block per 8 channels: 32 threads per channel merge strided
//     subsets of the partials in fp64, then a 5-level LDS tree. A single "last block" doing
//     the whole merge serially was latency-bound (hundreds of dependent L2 loads per channel)
//     and cost more than the data passes themselves.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "abi.h"

namespace {

constexpr int kT = 256;      // threads per block
constexpr int kVec = 8;      // channels per thread
constexpr int kMaxC = 2048;  // C / kVec <= kT


// 8 channels of row `r`, group `g` (channels 8g..8g+7) as fp32.
template <typename T>
struct V8;
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

template <>
struct V8<uint16_t> {
  // non-temporal (last read of a streamed tensor in this pass sequence)
  static __device__ __forceinline__ void loadnt(const uint16_t* p, float v[kVec]) {
    const u32x4_t q = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(q[i] << 16);
      v[2 * i + 1] = __uint_as_float(q[i] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void load(const uint16_t* p, float v[kVec]) {
    const uint4 q = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  // round to nearest even, two per v_cvt_pk_bf16_f32 (NaN stays NaN, quieted)
  static __device__ __forceinline__ uint32_t pack2(float a, float b) {
    const f32x2_t v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
  }
  static __device__ __forceinline__ void store(uint16_t* p, const float v[kVec]) {
    *reinterpret_cast<uint4*>(p) = make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]),
                                              pack2(v[4], v[5]), pack2(v[6], v[7]));
  }
  // store, and return the bits of the stored (rounded) values that are > 0 (not NaN)
  static __device__ __forceinline__ uint32_t store_pos(uint16_t* p, const float v[kVec]) {
    const uint32_t w[4] = {pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]),
                           pack2(v[6], v[7])};
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
    uint32_t b = 0;
#pragma unroll
    for (int i = 0; i < kVec; ++i) {
      const uint32_t h = (i & 1) ? (w[i >> 1] >> 16) : (w[i >> 1] & 0xffffu);
      const bool pos = (h & 0x8000u) == 0 && (h & 0x7fffu) != 0 && (h & 0x7fffu) <= 0x7f80u;
      b |= (pos ? 1u : 0u) << i;
    }
    return b;
  }
};
template <>
struct V8<float> {
  static __device__ __forceinline__ void loadnt(const float* p, float v[kVec]) {
    const f32x4_t a = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(p));
    const f32x4_t b = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(p + 4));
#pragma unroll
    for (int i = 0; i < 4; ++i) { v[i] = a[i]; v[4 + i] = b[i]; }
  }
  static __device__ __forceinline__ void load(const float* p, float v[kVec]) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float v[kVec]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
  static __device__ __forceinline__ uint32_t store_pos(float* p, const float v[kVec]) {
    store(p, v);
    uint32_t b = 0;
#pragma unroll
    for (int i = 0; i < kVec; ++i) b |= (v[i] > 0.f ? 1u : 0u) << i;
    return b;
  }
};

// 8 per-channel fp32 coefficients (two 16-byte loads; the arrays are tiny and stay in L1/L2)
__device__ __forceinline__ void load8f(const float* p, float v[kVec]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// ------------------------------------------------------------------ accumulated statistics
// "acc mode": the statistics pass, the backward reduction and the producing conv's epilogue
// (conv_kernels.hip ConvArgs::bn_acc) add their per-block fp64 sums straight into acc [2][C] with
// fire-and-forget memory-side atomics (consecutive threads on consecutive channels: contiguous
// 512-byte wave instructions). The CONSUMING pass (apply forward, dx backward) derives each
// thread's per-channel coefficients from the sums in its prologue, so no finalize launch sits
// between producer and consumer; a later kernel of the same layer zeroes the set again (block 0,
// plain stores: its last reader has finished by stream order). That replaces the two-level merge
// of per-block partials (up to 3136 per channel) in the partial-based finalize kernels below.

// Replicated sets (abi.h ARENA_ACC_REP): the BN passes' reductions emit at most 512 block sums
// per channel and add into replica 0; the conv epilogues spread over all replicas. Readers sum
// every replica in replica order.
constexpr int kAccRep = ARENA_ACC_REP;

__device__ __forceinline__ void acc_sums(const double* __restrict__ acc, int C, int c, double& s1,
                                         double& s2) {
  s1 = acc[c];
  s2 = acc[C + c];
#pragma unroll
  for (int r = 1; r < kAccRep; ++r) {
    s1 += acc[(size_t)r * 2 * C + c];
    s2 += acc[(size_t)r * 2 * C + C + c];
  }
}

// Reduction geometry. A block covers `cg` channel groups (all C / 8 of them, or a 32-group slice
// for C > 256: blockIdx.y picks the slice) and kT / cg row slots. The channel split keeps the
// number of (row block, channel) pairs -- the per-block sums a reduction emits -- at <= 512 x 256
// for every C, so the acc-mode atomics stay ~2 MB per pass (a 2048-channel layer used to emit 1 M
// pairs from 512 full-width blocks).
struct Geo {
  int cg;    // channel groups of this block
  int rip;   // rows in parallel per block round
  int g;     // this thread's channel group (global index)
  int gl;    // ... within the block's slice
  int slot;  // this thread's row slot (active iff slot < rip)
  int cw;    // channels of the block's slice (8 cg)
  int cb;    // first channel of the slice
};
__device__ __forceinline__ Geo geo(int C) {
  Geo q;
  q.cg = C / kVec / (int)gridDim.y;
  q.rip = kT / q.cg;
  q.gl = threadIdx.x % q.cg;
  q.slot = threadIdx.x / q.cg;
  q.cw = q.cg * kVec;
  q.cb = (int)blockIdx.y * q.cw;
  q.g = (int)blockIdx.y * q.cg + q.gl;
  return q;
}

// Rows [r0, r1) of block b.
__device__ __forceinline__ void block_rows(long long M, long long rpb, long long* r0,
                                           long long* r1) {
  *r0 = (long long)blockIdx.x * rpb;
  *r1 = min(M, *r0 + rpb);
}

// ------------------------------------------------------------------------------------ stats
// part: [nblk][2][C] (block mean, block M2)
// acc != null: the block's (sum x, sum x^2) go to acc [2][C] (acc mode) instead of part.
template <typename T>
__global__ __launch_bounds__(kT) void bn_stats_kernel(const T* __restrict__ x, long long M, int C,
                                                      long long rpb, float* __restrict__ part,
                                                      double* __restrict__ acc) {
  const Geo q = geo(C);
  long long r0, r1;
  block_rows(M, rpb, &r0, &r1);
  float mean[kVec], m2[kVec];
#pragma unroll
  for (int i = 0; i < kVec; ++i) mean[i] = m2[i] = 0.f;
  float n = 0.f;
  if (q.slot < q.rip) {
    const T* base = x + (long long)q.g * kVec;
    long long r = r0 + q.slot;
    // 4 rows per step: all loads issued before the Welford updates
    for (; r + 3LL * q.rip < r1; r += 4LL * q.rip) {
      float v[4][kVec];
#pragma unroll
      for (int u = 0; u < 4; ++u) V8<T>::load(base + (r + (long long)u * q.rip) * C, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        n += 1.f;
        const float inv = 1.f / n;
#pragma unroll
        for (int i = 0; i < kVec; ++i) {
          const float d = v[u][i] - mean[i];
          mean[i] += d * inv;
          m2[i] += d * (v[u][i] - mean[i]);
        }
      }
    }
    for (; r < r1; r += q.rip) {
      float v[kVec];
      V8<T>::load(base + r * C, v);
      n += 1.f;
      const float inv = 1.f / n;
#pragma unroll
      for (int i = 0; i < kVec; ++i) {
        const float d = v[i] - mean[i];
        mean[i] += d * inv;
        m2[i] += d * (v[i] - mean[i]);
      }
    }
  }
  // Chan merge over the row slots of each channel group (LDS: [slot][C] mean, m2; [slot] n)
  __shared__ float s_mean[kT * kVec], s_m2[kT * kVec], s_n[kT];
  if (q.slot < q.rip) {
#pragma unroll
    for (int i = 0; i < kVec; ++i) {
      s_mean[q.slot * q.cw + q.gl * kVec + i] = mean[i];
      s_m2[q.slot * q.cw + q.gl * kVec + i] = m2[i];
    }
    if (q.gl == 0) s_n[q.slot] = n;
  }
  __syncthreads();
  for (int cl = threadIdx.x; cl < q.cw; cl += kT) {
    const int c = q.cb + cl;
    float na = s_n[0], ma = s_mean[cl], sa = s_m2[cl];
    for (int s = 1; s < q.rip; ++s) {
      const float nb = s_n[s];
      if (nb == 0.f) continue;
      const float nab = na + nb;
      const float d = s_mean[s * q.cw + cl] - ma;
      ma += d * (nb / nab);
      sa += s_m2[s * q.cw + cl] + d * d * (na * nb / nab);
      na = nab;
    }
    if (acc != nullptr) {
      const double nd = (double)na, mu = (double)ma;
      unsafeAtomicAdd(acc + c, nd * mu);                        // sum x
      unsafeAtomicAdd(acc + C + c, (double)sa + nd * mu * mu);  // sum x^2
    } else {
      part[(long long)blockIdx.x * 2 * C + c] = ma;
      part[(long long)blockIdx.x * 2 * C + C + c] = sa;
    }
  }
}

// Finalize = merge of the per-block (or per-conv-tile) partials, [nblk][2][C] floats, into the
// per-channel outputs. Up to 3136 partials per channel arrive from a conv epilogue, so the merge is
// a two-level parallel reduction: block (g, p) of a (C/64) x P grid gives each of its 4 waves one
// channel per lane (coalesced 256-byte reads of a partial row) and a strided share of the
// partials, with 8 loads in flight per lane and no division in the loop; the block's sums go to
// `lvl2` and the last of the P blocks of channel group g (ticket counter) merges them in a fixed
// order and writes the outputs. Statistics use shifted fp64 sums: with K = the first partial's
// mean, S1 = sum n_b (m_b - K), S2 = sum (M2_b + n_b (m_b - K)^2), so mean = K + S1/N and
// M2 = S2 - S1^2/N without cancellation. (The previous form, a serial fp64 Chan merge per thread,
// was latency-bound: 13.5 us per layer on average, 43 us behind a 56x56 conv.)
constexpr int kFinWaves = kT / 64;
constexpr int kFinU = 16;       // partials per lane per load batch (one batch up to 4096 partials)
int g_fin_max_p = 64;           // level-1 blocks per channel group (runtime-tunable; 1 = no tickets)

int fin_blocks_per_group(int nblk) {
  int p = (nblk + kFinWaves * kFinU - 1) / (kFinWaves * kFinU);
  return p < 1 ? 1 : (p > g_fin_max_p ? g_fin_max_p : p);
}

// Sum of the 4 waves' (a, b, c) in LDS, fixed order, into wave 0's lanes. Returns false on the
// other waves (they are done).
__device__ __forceinline__ bool fin_block_sum(double& a, double& b, double& c) {
  __shared__ double sh[3][kFinWaves][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  sh[0][wv][lane] = a; sh[1][wv][lane] = b; sh[2][wv][lane] = c;
  __syncthreads();
  if (wv != 0) return false;
  a = ((sh[0][0][lane] + sh[0][1][lane]) + (sh[0][2][lane] + sh[0][3][lane]));
  b = ((sh[1][0][lane] + sh[1][1][lane]) + (sh[1][2][lane] + sh[1][3][lane]));
  c = ((sh[2][0][lane] + sh[2][1][lane]) + (sh[2][2][lane] + sh[2][3][lane]));
  return true;
}

// Wave 0 of a level-1 block: publish (a, b, c) and take a ticket. Returns true on the last block
// of the group, with (a, b, c) replaced by the merge over all P blocks (fixed order).
__device__ __forceinline__ bool fin_level2(double& a, double& b, double& c, double* __restrict__ lvl2,
                                           unsigned* __restrict__ tickets) {
  const int lane = threadIdx.x & 63, g = blockIdx.x, p = blockIdx.y, P = gridDim.y;
  double* mine = lvl2 + ((long long)g * P + p) * 3 * 64;
  mine[lane] = a; mine[64 + lane] = b; mine[128 + lane] = c;
  // release: this wave's stores reach device scope before the ticket (the explicit vmcnt(0):
  // hipcc may drop the wait after the L2 write-back when its scoreboard looks empty)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(tickets + g, 1u, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
  old = __shfl(old, 0);
  if (old != (unsigned)(P - 1)) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate has landed before the reads
  const double* base = lvl2 + (long long)g * P * 3 * 64;
  double sa = 0.0, sb = 0.0, sc = 0.0;
  int q = 0;
  // 16 published rows per batch (48 loads in flight per lane): the level-2 merge of P <= 64 rows
  // is 4 dependent round trips instead of 16 (same summation order)
  for (; q + 16 <= P; q += 16) {
    double va[16], vb[16], vc[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const double* r = base + (long long)(q + u) * 3 * 64;
      va[u] = r[lane]; vb[u] = r[64 + lane]; vc[u] = r[128 + lane];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) { sa += va[u]; sb += vb[u]; sc += vc[u]; }
  }
  for (; q + 4 <= P; q += 4) {
    double va[4], vb[4], vc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double* r = base + (long long)(q + u) * 3 * 64;
      va[u] = r[lane]; vb[u] = r[64 + lane]; vc[u] = r[128 + lane];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) { sa += va[u]; sb += vb[u]; sc += vc[u]; }
  }
  for (; q < P; ++q) {
    const double* r = base + (long long)q * 3 * 64;
    sa += r[lane]; sb += r[64 + lane]; sc += r[128 + lane];
  }
  if (lane == 0) __hip_atomic_store(tickets + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  a = sa; b = sb; c = sc;
  return true;
}

__global__ __launch_bounds__(kT) void bn_stats_finalize_kernel(const float* __restrict__ part,
                                                               int nblk, long long M, int C,
                                                               long long rpb,
                                                               double* __restrict__ lvl2,
                                                               unsigned* __restrict__ tickets,
                                                               ArenaBNStats out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int ci = c < C ? c : C - 1;
  const float* pc = part + ci;
  const double K = (double)pc[0];
  double n = 0.0, s1 = 0.0, s2 = 0.0;
  const int stride = kFinWaves * (int)gridDim.y;
  for (int b = (int)blockIdx.y * kFinWaves + wv; b < nblk; b += kFinU * stride) {
    float mb[kFinU], sb[kFinU];
    double nb[kFinU];
#pragma unroll
    for (int u = 0; u < kFinU; ++u) {
      const int bb = b + u * stride;
      const bool ok = bb < nblk;
      const long long o = (long long)(ok ? bb : 0) * 2 * C;
      mb[u] = pc[o];
      sb[u] = pc[o + C];
      const long long r0 = (long long)bb * rpb;
      nb[u] = ok ? (double)(min(M, r0 + rpb) - r0) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kFinU; ++u) {
      const double d = (double)mb[u] - K;
      n += nb[u];
      s1 += nb[u] * d;
      s2 += (nb[u] > 0.0 ? (double)sb[u] : 0.0) + nb[u] * d * d;
    }
  }
  if (!fin_block_sum(n, s1, s2)) return;
  if (gridDim.y > 1 && !fin_level2(n, s1, s2, lvl2, tickets)) return;
  // the module's batch counter rides along (one launch fewer per BN layer than a separate add)
  if (out.batches != nullptr && blockIdx.x == 0 && lane == 0) *out.batches += 1;
  if (c >= C) return;
  const double mean = K + s1 / n;
  double m2 = s2 - s1 * s1 / n;
  m2 = m2 > 0.0 ? m2 : 0.0;
  const double var = m2 / n;  // biased: what training normalises with
  const float invstd = (float)(1.0 / sqrt(var + (double)out.eps));
  out.mean[c] = (float)mean;
  out.invstd[c] = invstd;
  const float gam = out.gamma ? out.gamma[c] : 1.f;
  const float bet = out.beta ? out.beta[c] : 0.f;
  out.scale[c] = gam * invstd;
  out.shift[c] = bet;  // y = (x - mean) * scale + shift: no cancellation when |mean| >> std
  if (out.running_mean) {
    const float mom = out.momentum;
    out.running_mean[c] = (1.f - mom) * out.running_mean[c] + mom * (float)mean;
    const double unbiased = n > 1.0 ? m2 / (n - 1.0) : var;
    out.running_var[c] = (1.f - mom) * out.running_var[c] + mom * (float)unbiased;
  }
}

// ------------------------------------------------------------------------------------ apply
// y = act((x - mean) * scale + shift (+ res)), 2 vectors per thread per round for load ILP.
// The mask bits are those of the stored (rounded) outputs that are > 0: exactly "saved y > 0"
// (V8::store_pos).

// Block 0 clears `zero` [nzero] doubles: the accumulator set of an earlier pass whose last reader
// has finished (kernel order on the stream), made ready for its next producer without a launch.
__device__ __forceinline__ void zero_duty(double* zero, int nzero) {
  if (zero == nullptr || blockIdx.x != 0 || blockIdx.y != 0) return;
  for (int i = threadIdx.x; i < nzero; i += kT) zero[i] = 0.0;
}

// Per-channel coefficients of the apply / dx passes are computed ONCE PER BLOCK, one thread per
// channel, into LDS (`s_co`, [k][C] floats, dynamic shared memory), and each thread then reads its
// 8 channels from there. Every thread loading its own 8 channels from global memory put up to
// 4096 x 256 requests for the same few hundred bytes on one L2 channel per layer: with the 176
// bytes per thread the fp64 sums need, the dx pass ran at half speed (51 vs 27 us per layer).
__device__ __forceinline__ void lds8(const float* p, float v[kVec]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// FIN: the batch statistics arrive as the fp64 sums (sum x, sum x^2) of acc mode in `fin` [2][C]
// (from the producing conv's epilogue or the acc-mode statistics pass) and the block derives mean,
// invstd, scale and shift itself -- the work of a finalize launch, which this replaces. Block 0
// also writes st's outputs (mean / invstd for the backward, scale / shift, running statistics,
// the batch counter). The sums stay in place: the backward's dx pass of this layer zeroes them
// (arena_bn_bwd `zero`), after their last reader here has finished.
// [c_lo, c_lo + cs): the channels this block covers (all C, or one 256-channel slice of a
// channel-sliced grid, see Slice); s_co holds them at local indices [k][cs].
// writer: this block writes st's outputs for its channels (one block per channel).
template <bool FIN>
__device__ __forceinline__ void apply_coefs(int C, long long M, const double* fin,
                                            const ArenaBNStats& st, float* s_co, int c_lo,
                                            int cs, bool writer) {
  const double inv_m = 1.0 / (double)M;
  for (int cl = threadIdx.x; cl < cs; cl += kT) {
    const int c = c_lo + cl;
    float mu, sc, sh;
    if constexpr (!FIN) {
      mu = st.mean[c];
      sc = st.scale[c];
      sh = st.shift[c];
    } else {
      double s1, s2;
      acc_sums(fin, C, c, s1, s2);
      const double mean = s1 * inv_m;
      const double d = s2 - s1 * mean;
      const double m2 = d > 0.0 ? d : 0.0;
      const float inv = (float)(1.0 / sqrt(m2 * inv_m + (double)st.eps));
      mu = (float)mean;
      sc = (st.gamma ? st.gamma[c] : 1.f) * inv;
      sh = st.beta ? st.beta[c] : 0.f;
      if (writer) {
        st.mean[c] = mu;
        st.invstd[c] = inv;
        st.scale[c] = sc;
        st.shift[c] = sh;
        if (st.running_mean) {
          const float mom = st.momentum;
          const double unbiased = M > 1 ? m2 / (double)(M - 1) : m2 * inv_m;
          st.running_mean[c] = (1.f - mom) * st.running_mean[c] + mom * mu;
          st.running_var[c] = (1.f - mom) * st.running_var[c] + mom * (float)unbiased;
        }
        if (c == 0 && st.batches != nullptr) *st.batches += 1;
      }
    }
    s_co[cl] = mu;
    s_co[cs + cl] = sc;
    s_co[2 * cs + cl] = sh;
  }
  __syncthreads();
}

// Thread -> vector mapping of the streaming passes (apply, dx). Every vector a thread touches has
// the same channel group, so its coefficients load once. Flat grid (gridDim.y == 1): vector
// blockIdx.x * kT + tid, stride gridDim.x * kT (cg | kT, host-checked). Channel-sliced grid
// (gridDim.y = cg / 32 slices of 256 channels, for C > 256): a block covers 32 groups x 8 rows of
// its slice, so its coefficient prologue derives 256 channels instead of all C -- with C = 2048
// and ~6 vectors per thread that prologue was most of the pass (the 7x7 dx ran at 1.9 TB/s).
struct Slice {
  long long v0, stride;   // first vector, vector stride
  int c_lo, cs;           // channel range of the block (coefficients)
  int c0;                 // the thread's first channel, local to [c_lo, c_lo + cs)
};
constexpr int kSliceG = 32;   // channel groups per slice

__device__ __forceinline__ Slice slice_of(int cg) {
  Slice q;
  if (gridDim.y == 1) {
    q.v0 = (long long)blockIdx.x * kT + threadIdx.x;
    q.stride = (long long)gridDim.x * kT;
    q.c_lo = 0;
    q.cs = cg * kVec;
    q.c0 = (int)(q.v0 & (cg - 1)) * kVec;
  } else {
    constexpr int kRows = kT / kSliceG;
    const int gl = threadIdx.x & (kSliceG - 1);
    const long long row0 = (long long)blockIdx.x * kRows + threadIdx.x / kSliceG;
    q.v0 = row0 * cg + (long long)blockIdx.y * kSliceG + gl;
    q.stride = (long long)gridDim.x * kRows * cg;
    q.c_lo = blockIdx.y * kSliceG * kVec;
    q.cs = kSliceG * kVec;
    q.c0 = gl * kVec;
  }
  return q;
}

// NT: non-temporal loads of x (and res) -- their last read before the backward pass
// dynamic shared memory: 3 * C floats
template <typename T, bool RELU, bool RES, bool NT, bool FIN>
__global__ __launch_bounds__(kT) void bn_apply_kernel(const T* __restrict__ x,
                                                      const T* __restrict__ res,
                                                      T* __restrict__ y,
                                                      uint8_t* __restrict__ mask,
                                                      ArenaBNStats st,
                                                      const double* __restrict__ fin,
                                                      long long M, long long nvec, int cg,
                                                      double* __restrict__ zero, int nzero) {
  extern __shared__ __attribute__((aligned(16))) float s_co[];
  const Slice q = slice_of(cg);
  const long long stride = q.stride;
  const int C = cg * kVec;
  // the loads of x (and res) do not depend on the coefficients: each thread issues its first two
  // vectors before the coefficient prologue and the next two before computing the current ones,
  // so the prologue's round trip to the sums overlaps the first data round trip (most threads of
  // the 14x14 / 7x7 passes only ever touch two to six vectors)
  float a[2][kVec], b[2][kVec];
  bool ok[2];
  long long vv[2];
  auto issue = [&](long long v0, float (&ta)[2][kVec], float (&tb)[2][kVec], bool (&tok)[2],
                   long long (&tvv)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      tvv[u] = v0 + u * stride;
      tok[u] = tvv[u] < nvec;
      const long long vc = tok[u] ? tvv[u] : v0;
      if (NT) {
        V8<T>::loadnt(x + vc * kVec, ta[u]);
        if (RES) V8<T>::loadnt(res + vc * kVec, tb[u]);
      } else {
        V8<T>::load(x + vc * kVec, ta[u]);
        if (RES) V8<T>::load(res + vc * kVec, tb[u]);
      }
    }
  };
  if (q.v0 < nvec) issue(q.v0, a, b, ok, vv);
  apply_coefs<FIN>(C, M, fin, st, s_co, q.c_lo, q.cs, blockIdx.x == 0);   // one per slice
  float mu[kVec], sc[kVec], sh[kVec];
  lds8(s_co + q.c0, mu);
  lds8(s_co + q.cs + q.c0, sc);
  lds8(s_co + 2 * q.cs + q.c0, sh);
  zero_duty(zero, nzero);
  for (long long v0 = q.v0; v0 < nvec; v0 += 2 * stride) {
    float na[2][kVec], nb[2][kVec];
    bool nok[2] = {false, false};
    long long nvv[2];
    const bool more = v0 + 2 * stride < nvec;
    if (more) issue(v0 + 2 * stride, na, nb, nok, nvv);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float o[kVec];
#pragma unroll
      for (int i = 0; i < kVec; ++i) {
        float t = fmaf(a[u][i] - mu[i], sc[i], sh[i]);
        if (RES) t += b[u][i];
        o[i] = RELU ? fmaxf(t, 0.f) : t;
      }
      if (ok[u]) {
        if (RELU && mask != nullptr)
          mask[vv[u]] = (uint8_t)V8<T>::store_pos(y + vv[u] * kVec, o);
        else
          V8<T>::store(y + vv[u] * kVec, o);
      }
    }
    if (more) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        ok[u] = nok[u];
        vv[u] = nvv[u];
#pragma unroll
        for (int i = 0; i < kVec; ++i) {
          a[u][i] = na[u][i];
          if (RES) b[u][i] = nb[u][i];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------- backward sums
// g = RELU ? dy * mask : dy;  per channel: sum g, sum g * (x - mean).  part: [nblk][2][C]
// bn_bwd_finish: the backward finalize of channel c from its sums (sum g, sum g (x - mean)).
__device__ __forceinline__ void bn_bwd_finish(const ArenaBNBwd& out, int c, double a, double b,
                                              long long M) {
  const float invstd = out.invstd[c];
  const float gam = out.gamma ? out.gamma[c] : 1.f;
  if (out.dgamma) out.dgamma[c] = (float)(b * invstd);
  if (out.dbeta) out.dbeta[c] = (float)a;
  // dx = gamma*invstd * (g - sum_g/M - (x - mean) * invstd^2 * sum_gx/M)
  out.ca[c] = gam * invstd;
  out.cb[c] = (float)(a / (double)M);
  out.cc[c] = (float)(b / (double)M) * invstd * invstd;
}

// acc != null (acc mode): the block sums go to acc [2][C]; else the per-block partials to part.
template <typename T, bool RELU>
__global__ __launch_bounds__(kT) void bn_bwd_reduce_kernel(const T* __restrict__ dy,
                                                           const uint8_t* __restrict__ mask,
                                                           const T* __restrict__ x, long long M,
                                                           int C, long long rpb,
                                                           float* __restrict__ part,
                                                           ArenaBNBwd out,
                                                           double* __restrict__ acc) {
  const Geo q = geo(C);
  long long r0, r1;
  block_rows(M, rpb, &r0, &r1);
  float sg[kVec], sgx[kVec], mu[kVec];
#pragma unroll
  for (int i = 0; i < kVec; ++i) sg[i] = sgx[i] = 0.f;
  if (q.slot < q.rip) {
#pragma unroll
    for (int i = 0; i < kVec; ++i) mu[i] = out.mean[q.g * kVec + i];
    const long long off = (long long)q.g * kVec;
    long long r = r0 + q.slot;
    for (; r + q.rip < r1; r += 2LL * q.rip) {  // 2 rows per step: all loads in flight
      float d[2][kVec], v[2][kVec];
      uint32_t mb[2] = {0xffu, 0xffu};
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const long long rr = r + (long long)u * q.rip;
        const long long p = rr * C + off;
        V8<T>::load(dy + p, d[u]);
        if (RELU) mb[u] = mask[rr * (C / kVec) + q.g];
        V8<T>::load(x + p, v[u]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < kVec; ++i) {
          const float g = ((mb[u] >> i) & 1u) ? d[u][i] : 0.f;
          sg[i] += g;
          sgx[i] = fmaf(g, v[u][i] - mu[i], sgx[i]);
        }
    }
    for (; r < r1; r += q.rip) {
      float d[kVec], v[kVec];
      const long long p = r * C + off;
      V8<T>::load(dy + p, d);
      const uint32_t mb = RELU ? (uint32_t)mask[r * (C / kVec) + q.g] : 0xffu;
      V8<T>::load(x + p, v);
#pragma unroll
      for (int i = 0; i < kVec; ++i) {
        const float g = ((mb >> i) & 1u) ? d[i] : 0.f;
        sg[i] += g;
        sgx[i] = fmaf(g, v[i] - mu[i], sgx[i]);
      }
    }
  }
  __shared__ float s_g[kT * kVec], s_gx[kT * kVec];
  if (q.slot < q.rip) {
#pragma unroll
    for (int i = 0; i < kVec; ++i) {
      s_g[q.slot * q.cw + q.gl * kVec + i] = sg[i];
      s_gx[q.slot * q.cw + q.gl * kVec + i] = sgx[i];
    }
  }
  __syncthreads();
  for (int cl = threadIdx.x; cl < q.cw; cl += kT) {
    const int c = q.cb + cl;
    float a = 0.f, b = 0.f;
    for (int s = 0; s < q.rip; ++s) {
      a += s_g[s * q.cw + cl];
      b += s_gx[s * q.cw + cl];
    }
    if (acc != nullptr) {
      unsafeAtomicAdd(acc + c, (double)a);
      unsafeAtomicAdd(acc + C + c, (double)b);
    } else {
      part[(long long)blockIdx.x * 2 * C + c] = a;
      part[(long long)blockIdx.x * 2 * C + C + c] = b;
    }
  }
}

// Backward finalize of acc mode: one thread per channel, accumulators zeroed again.
__global__ __launch_bounds__(kT) void bn_bwd_acc_finalize_kernel(double* __restrict__ acc,
                                                                 long long M, int C,
                                                                 ArenaBNBwd out) {
  const int c = blockIdx.x * kT + threadIdx.x;
  if (c >= C) return;
  double a = 0.0, b = 0.0;
#pragma unroll
  for (int r = 0; r < kAccRep; ++r) {
    a += __hip_atomic_exchange(acc + (size_t)r * 2 * C + c, 0.0, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    b += __hip_atomic_exchange(acc + (size_t)r * 2 * C + C + c, 0.0, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
  }
  bn_bwd_finish(out, c, a, b, M);
}

__global__ __launch_bounds__(kT) void bn_bwd_finalize_kernel(const float* __restrict__ part,
                                                             int nblk, long long M, int C,
                                                             double* __restrict__ lvl2,
                                                             unsigned* __restrict__ tickets,
                                                             ArenaBNBwd out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const float* pc = part + (c < C ? c : C - 1);
  double a = 0.0, b = 0.0, unused = 0.0;
  const int stride = kFinWaves * (int)gridDim.y;
  for (int blk = (int)blockIdx.y * kFinWaves + wv; blk < nblk; blk += kFinU * stride) {
    float va[kFinU], vb[kFinU];
#pragma unroll
    for (int u = 0; u < kFinU; ++u) {
      const int bb = blk + u * stride;
      const bool ok = bb < nblk;
      const long long o = (long long)(ok ? bb : 0) * 2 * C;
      const float x0 = pc[o], x1 = pc[o + C];  // clamped address: unconditional loads
      va[u] = ok ? x0 : 0.f;
      vb[u] = ok ? x1 : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kFinU; ++u) { a += (double)va[u]; b += (double)vb[u]; }
  }
  if (!fin_block_sum(a, b, unused)) return;
  if (gridDim.y > 1 && !fin_level2(a, b, unused, lvl2, tickets)) return;
  if (c >= C) return;
  bn_bwd_finish(out, c, a, b, M);
}

// --------------------------------------------------------------------------------- backward dx
// NT: non-temporal loads of dy and x (their last read in the step)
// FIN: the reduction ran in acc mode into `acc` [2][C] (sum g, sum g (x - mean)) and the block
// derives the coefficients, one thread per channel (bn_bwd_finish's arithmetic, with 1/M
// multiplied instead of divided); block 0 writes dgamma / dbeta. The sums are left in place: the layer's
// next forward apply pass zeroes them (arena_bn_fwd `zero`).
// dynamic shared memory: 4 * C floats
// S2 (RELU, FIN, no RES): the same pass also sums (g, g (x2 - mean2)) per channel into acc2
// [ARENA_ACC_REP][2][C] -- the backward sums of a second BN whose gradient is this layer's masked
// dy g: a downsample block's down_bn, the residual of this bn3 (see batchnorm.ResidualMask). Its
// own reduction pass (dy, mask and x2 read again) then does not run.
template <typename T, bool RELU, bool RES, bool NT, bool FIN, bool S2 = false>
__global__ __launch_bounds__(kT) void bn_bwd_dx_kernel(const T* __restrict__ dy,
                                                       const uint8_t* __restrict__ mask,
                                                       const T* __restrict__ x,
                                                       T* __restrict__ dx, T* __restrict__ dres,
                                                       long long nvec, int cg, ArenaBNBwd co,
                                                       const double* __restrict__ acc, long long M,
                                                       double* __restrict__ zero, int nzero,
                                                       const T* __restrict__ x2,
                                                       const float* __restrict__ mean2,
                                                       double* __restrict__ acc2) {
  extern __shared__ __attribute__((aligned(16))) float s_co[];
  const Slice q = slice_of(cg);   // fixed channel group per thread: coefficients once
  const long long stride = q.stride;
  const int c0 = q.c0, cs = q.cs;
  const int C = cg * kVec;
  const double inv_m = 1.0 / (double)M;
  // the first vector's loads (dy, mask, x) are issued before the coefficient prologue and each
  // next vector's before the current one is computed (as in bn_apply_kernel)
  float d[kVec], xv[kVec], x2v[S2 ? kVec : 1];
  uint32_t mb = 0xffu;
  auto issue = [&](long long v, float (&td)[kVec], float (&tx)[kVec], float (&tx2)[S2 ? kVec : 1],
                   uint32_t& tm) {
    if (NT) V8<T>::loadnt(dy + v * kVec, td); else V8<T>::load(dy + v * kVec, td);
    tm = RELU ? (uint32_t)mask[v] : 0xffu;
    if (NT) V8<T>::loadnt(x + v * kVec, tx); else V8<T>::load(x + v * kVec, tx);
    if constexpr (S2) {
      if (NT) V8<T>::loadnt(x2 + v * kVec, tx2); else V8<T>::load(x2 + v * kVec, tx2);
    }
  };
  if (q.v0 < nvec) issue(q.v0, d, xv, x2v, mb);
  for (int cl = threadIdx.x; cl < cs; cl += kT) {   // one thread per channel (see lds8)
    const int c = q.c_lo + cl;
    float a_, b_, c_;
    if constexpr (FIN) {
      double a, b;
      acc_sums(acc, C, c, a, b);
      const float invstd = co.invstd[c];
      const float gam = co.gamma ? co.gamma[c] : 1.f;
      a_ = gam * invstd;
      b_ = (float)(a * inv_m);
      c_ = (float)(b * inv_m) * invstd * invstd;
      if (blockIdx.x == 0) {
        if (co.dgamma) co.dgamma[c] = (float)(b * invstd);
        if (co.dbeta) co.dbeta[c] = (float)a;
      }
    } else {
      a_ = co.ca[c];
      b_ = co.cb[c];
      c_ = co.cc[c];
    }
    s_co[cl] = a_;
    s_co[cs + cl] = b_;
    s_co[2 * cs + cl] = c_;
    s_co[3 * cs + cl] = co.mean[c];
  }
  __syncthreads();
  float ca[kVec], cb[kVec], cc[kVec], mu[kVec];
  lds8(s_co + c0, ca);
  lds8(s_co + cs + c0, cb);
  lds8(s_co + 2 * cs + c0, cc);
  lds8(s_co + 3 * cs + c0, mu);
  zero_duty(zero, nzero);
  float mu2[S2 ? kVec : 1], sa2[S2 ? kVec : 1], sb2[S2 ? kVec : 1];
  if constexpr (S2) {
#pragma unroll
    for (int i = 0; i < kVec; ++i) {
      mu2[i] = mean2[q.c_lo + c0 + i];
      sa2[i] = sb2[i] = 0.f;
    }
  }
  for (long long v = q.v0; v < nvec; v += stride) {
    float dn[kVec], xn[kVec], x2n[S2 ? kVec : 1];
    uint32_t mn = 0xffu;
    const bool more = v + stride < nvec;
    if (more) issue(v + stride, dn, xn, x2n, mn);
    float g[kVec], o[kVec];
#pragma unroll
    for (int i = 0; i < kVec; ++i) {
      g[i] = ((mb >> i) & 1u) ? d[i] : 0.f;
      o[i] = ca[i] * (g[i] - cb[i] - (xv[i] - mu[i]) * cc[i]);
    }
    if constexpr (S2) {
#pragma unroll
      for (int i = 0; i < kVec; ++i) {
        sa2[i] += g[i];
        sb2[i] = fmaf(g[i], x2v[i] - mu2[i], sb2[i]);
      }
    }
    V8<T>::store(dx + v * kVec, o);
    if (RES) V8<T>::store(dres + v * kVec, g);
    if (more) {
      mb = mn;
#pragma unroll
      for (int i = 0; i < kVec; ++i) {
        d[i] = dn[i];
        xv[i] = xn[i];
        if constexpr (S2) x2v[i] = x2n[i];
      }
    }
  }
  if constexpr (S2) {
    // the block's partial sums per channel: thread t holds channel group t % cgl of row t / cgl
    // (flat grid: cgl = cg, cg | kT; sliced: 32), summed over the rows in LDS, then one fp64
    // atomic per (channel, sum) into replica blockIdx.x % ARENA_ACC_REP
    __shared__ float s_a2[kT * kVec], s_b2[kT * kVec];
#pragma unroll
    for (int i = 0; i < kVec; ++i) {
      s_a2[threadIdx.x * kVec + i] = sa2[i];
      s_b2[threadIdx.x * kVec + i] = sb2[i];
    }
    __syncthreads();
    const int cgl = cs / kVec;
    if ((int)threadIdx.x < cs) {
      const int gq = threadIdx.x / kVec, i = threadIdx.x % kVec;
      float a = 0.f, b = 0.f;
      for (int r = 0; r < kT / cgl; ++r) {
        a += s_a2[(r * cgl + gq) * kVec + i];
        b += s_b2[(r * cgl + gq) * kVec + i];
      }
      double* dst = acc2 + (size_t)(blockIdx.x % kAccRep) * 2 * C;
      unsafeAtomicAdd(dst + q.c_lo + threadIdx.x, (double)a);
      unsafeAtomicAdd(dst + C + q.c_lo + threadIdx.x, (double)b);
    }
  }
}

// ------------------------------------------------------------------------ fused stem: BN + ReLU + max pool
// The ResNet stem's BatchNorm + ReLU feeds a 3x3 / 2 max pool and nothing else, so the pool reads
// the BN input x and normalises on the fly: the forward writes only the pooled output and its
// in-window argmax (no y, no mask bits: 205 MB written and read back less at batch 128), and the
// backward gathers each input's gradient from the windows that picked it (maxpool_bwd's rule,
// pool_kernels.hip) inside the BN reduction and dx passes, recomputing the ReLU mask from x,
// instead of materialising the pool's dx (another 205 MB write + 2 reads). Values, argmax ties and
// gradients are those of bn_apply + maxpool_fwd / maxpool_bwd + bn_bwd on the rounded output.
struct PoolG {
  int N, H, W, C, OH, OW, k, s, p;
};

template <typename T>
__device__ __forceinline__ float stored_val(float v) {   // the value bn_apply would have stored
  if constexpr (sizeof(T) == 2) return __uint_as_float(V8<uint16_t>::pack2(v, 0.f) << 16);
  else return v;
}

// dynamic shared memory: 3 * C floats. grid: (N * OH output rows, ceil(OW * C/8 / kT)).
// FIN: coefficients from the fp64 sums `fin`; else from st (a partial-merge finalize ran first).
template <typename T, bool FIN>
__global__ __launch_bounds__(kT) void bn_pool_fwd_kernel(const T* __restrict__ x,
                                                         T* __restrict__ y,
                                                         uint8_t* __restrict__ pos,
                                                         T* __restrict__ xsel,
                                                         ArenaBNStats st,
                                                         const double* __restrict__ fin,
                                                         long long M, PoolG g,
                                                         double* __restrict__ zero, int nzero) {
  extern __shared__ __attribute__((aligned(16))) float s_co[];
  const int C = g.C, cg = C / kVec;
  apply_coefs<FIN>(C, M, fin, st, s_co, 0, C, blockIdx.x == 0 && blockIdx.y == 0);
  zero_duty(zero, nzero);
  const int row = blockIdx.x;
  const int t = blockIdx.y * kT + threadIdx.x;
  if (t >= g.OW * cg) return;
  const int ow = t / cg, c8 = t - ow * cg;
  float mu[kVec], sc[kVec], sh[kVec];
  lds8(s_co + c8 * kVec, mu);
  lds8(s_co + C + c8 * kVec, sc);
  lds8(s_co + 2 * C + c8 * kVec, sh);
  const int n32 = row / g.OH, oh = row - n32 * g.OH;
  const long long n = n32;
  const int h0 = oh * g.s - g.p, w0 = ow * g.s - g.p;
  float m[kVec], xb[kVec];
  int best[kVec];
#pragma unroll
  for (int i = 0; i < kVec; ++i) { m[i] = -INFINITY; best[i] = -1; xb[i] = 0.f; }
  for (int kh = 0; kh < g.k; ++kh) {
    const int h = h0 + kh;
    if (h < 0 || h >= g.H) continue;
    for (int kw = 0; kw < g.k; ++kw) {
      const int w = w0 + kw;
      if (w < 0 || w >= g.W) continue;
      float a[kVec];
      V8<T>::load(x + (((n * g.H + h) * g.W + w) * C + (long long)c8 * kVec), a);
      const int q = kh * g.k + kw;
#pragma unroll
      for (int i = 0; i < kVec; ++i) {
        const float v = stored_val<T>(fmaxf(fmaf(a[i] - mu[i], sc[i], sh[i]), 0.f));
        if (v > m[i] || __builtin_isnan(v) || best[i] < 0) { m[i] = v; best[i] = q; xb[i] = a[i]; }
      }
    }
  }
  const long long v = (long long)row * g.OW * cg + t;
  V8<T>::store(y + v * kVec, m);
  uint2 pk;
  pk.x = (uint32_t)(best[0] & 0xff) | ((uint32_t)(best[1] & 0xff) << 8) |
         ((uint32_t)(best[2] & 0xff) << 16) | ((uint32_t)(best[3] & 0xff) << 24);
  pk.y = (uint32_t)(best[4] & 0xff) | ((uint32_t)(best[5] & 0xff) << 8) |
         ((uint32_t)(best[6] & 0xff) << 16) | ((uint32_t)(best[7] & 0xff) << 24);
  *reinterpret_cast<uint2*>(pos + v * kVec) = pk;
  if (xsel != nullptr) V8<T>::store(xsel + v * kVec, xb);   // x at the argmax (exact: x is T)
}

// The pool's gradient at input pixel r (row-major n, h, w), channels 8 c8 .. 8 c8 + 7: the sum of
// dy over the (at most 2 x 2 for the 3x3 / 2 pool) windows whose saved argmax is this pixel.
template <typename T>
__device__ __forceinline__ void pool_grad8(const T* __restrict__ dy,
                                           const uint8_t* __restrict__ pos, const PoolG& g,
                                           long long r, int c8, float out[kVec]) {
  constexpr int CW = 2;
  // 32-bit index math (M < 2^31, host-checked): a 64-bit division is a ~100-instruction
  // software sequence, and these run once per 8-channel vector
  const unsigned ru = (unsigned)r;
  const unsigned nh = ru / (unsigned)g.W;
  const int w = (int)(ru - nh * (unsigned)g.W);
  const unsigned n32 = nh / (unsigned)g.H;
  const int h = (int)(nh - n32 * (unsigned)g.H);
  const long long n = n32;
  const int th = h + g.p - g.k + 1, tw = w + g.p - g.k + 1;
  const int oh_lo = th <= 0 ? 0 : (th + g.s - 1) / g.s;
  const int ow_lo = tw <= 0 ? 0 : (tw + g.s - 1) / g.s;
  const int oh_hi = min(g.OH - 1, (h + g.p) / g.s);
  const int ow_hi = min(g.OW - 1, (w + g.p) / g.s);
  long long off[CW * CW];
  int q[CW * CW];
  uint2 pk[CW * CW];
#pragma unroll
  for (int a = 0; a < CW; ++a)
#pragma unroll
    for (int b = 0; b < CW; ++b) {
      const int j = a * CW + b;
      const bool ok = oh_lo + a <= oh_hi && ow_lo + b <= ow_hi;
      const int oh = ok ? oh_lo + a : min(oh_lo, g.OH - 1);
      const int ow = ok ? ow_lo + b : min(ow_lo, g.OW - 1);
      q[j] = ok ? (h - (oh * g.s - g.p)) * g.k + (w - (ow * g.s - g.p)) : 0xff;
      off[j] = ((n * g.OH + oh) * g.OW + ow) * g.C + (long long)c8 * kVec;
      pk[j] = *reinterpret_cast<const uint2*>(pos + off[j]);
    }
  float d[CW * CW][kVec];
#pragma unroll
  for (int j = 0; j < CW * CW; ++j) V8<T>::load(dy + off[j], d[j]);
#pragma unroll
  for (int i = 0; i < kVec; ++i) out[i] = 0.f;
#pragma unroll
  for (int j = 0; j < CW * CW; ++j) {
    const uint32_t ps[2] = {pk[j].x, pk[j].y};
#pragma unroll
    for (int i = 0; i < kVec; ++i)
      out[i] += ((ps[i >> 2] >> (8 * (i & 3))) & 0xff) == (uint32_t)q[j] ? d[j][i] : 0.f;
  }
}

// Backward reduction of the fused stem (acc mode into `acc`, zero on entry): g = pool gradient
// masked by the recomputed ReLU bit; per channel sum g, sum g (x - mean). Rows r of x are split
// over blocks like bn_bwd_reduce_kernel (C <= 256: one channel slice).
template <typename T>
__global__ __launch_bounds__(kT) void bn_pool_bwd_reduce_kernel(const T* __restrict__ dy,
                                                                const uint8_t* __restrict__ pos,
                                                                const T* __restrict__ x,
                                                                long long M, long long rpb,
                                                                PoolG g, ArenaBNBwd co,
                                                                double* __restrict__ acc) {
  __shared__ __attribute__((aligned(16))) float s_c[3 * 256];
  const int C = g.C;
  for (int c = threadIdx.x; c < C; c += kT) {
    s_c[c] = co.mean[c];
    s_c[C + c] = co.scale[c];
    s_c[2 * C + c] = co.shift[c];
  }
  __syncthreads();
  const Geo q = geo(C);
  long long r0, r1;
  block_rows(M, rpb, &r0, &r1);
  float sg[kVec], sgx[kVec], mu[kVec], sc[kVec], sh[kVec];
#pragma unroll
  for (int i = 0; i < kVec; ++i) sg[i] = sgx[i] = 0.f;
  lds8(s_c + q.g * kVec, mu);
  lds8(s_c + C + q.g * kVec, sc);
  lds8(s_c + 2 * C + q.g * kVec, sh);
  if (q.slot < q.rip) {
    // two rows per step: both rows' gathers (8 position + 8 gradient loads) and x loads are in
    // flight together (one row per step: 170 us at batch 128, two: 151 us)
    long long r = r0 + q.slot;
    for (; r + q.rip < r1; r += 2LL * q.rip) {
      float gv[2][kVec], v[2][kVec];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        V8<T>::load(x + (r + u * q.rip) * C + (long long)q.g * kVec, v[u]);
        pool_grad8<T>(dy, pos, g, r + u * q.rip, q.g, gv[u]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < kVec; ++i) {
          const bool on = stored_val<T>(fmaxf(fmaf(v[u][i] - mu[i], sc[i], sh[i]), 0.f)) > 0.f;
          const float gg = on ? gv[u][i] : 0.f;
          sg[i] += gg;
          sgx[i] = fmaf(gg, v[u][i] - mu[i], sgx[i]);
        }
    }
    for (; r < r1; r += q.rip) {
      float gv[kVec], v[kVec];
      V8<T>::load(x + r * C + (long long)q.g * kVec, v);
      pool_grad8<T>(dy, pos, g, r, q.g, gv);
#pragma unroll
      for (int i = 0; i < kVec; ++i) {
        const bool on = stored_val<T>(fmaxf(fmaf(v[i] - mu[i], sc[i], sh[i]), 0.f)) > 0.f;
        const float gg = on ? gv[i] : 0.f;
        sg[i] += gg;
        sgx[i] = fmaf(gg, v[i] - mu[i], sgx[i]);
      }
    }
  }
  __shared__ float s_g[kT * kVec], s_gx[kT * kVec];
  if (q.slot < q.rip) {
#pragma unroll
    for (int i = 0; i < kVec; ++i) {
      s_g[q.slot * q.cw + q.gl * kVec + i] = sg[i];
      s_gx[q.slot * q.cw + q.gl * kVec + i] = sgx[i];
    }
  }
  __syncthreads();
  for (int cl = threadIdx.x; cl < q.cw; cl += kT) {
    float a = 0.f, b = 0.f;
    for (int s2 = 0; s2 < q.rip; ++s2) {
      a += s_g[s2 * q.cw + cl];
      b += s_gx[s2 * q.cw + cl];
    }
    unsafeAtomicAdd(acc + q.cb + cl, (double)a);
    unsafeAtomicAdd(acc + C + q.cb + cl, (double)b);
  }
}

// dx of the fused stem from the reduction's sums (FIN as in bn_bwd_dx_kernel); dynamic shared
// memory: 6 * C floats
template <typename T>
__global__ __launch_bounds__(kT) void bn_pool_bwd_dx_kernel(const T* __restrict__ dy,
                                                            const uint8_t* __restrict__ pos,
                                                            const T* __restrict__ x,
                                                            T* __restrict__ dx, long long nvec,
                                                            PoolG g, ArenaBNBwd co,
                                                            const double* __restrict__ acc,
                                                            long long M,
                                                            double* __restrict__ zero, int nzero) {
  extern __shared__ __attribute__((aligned(16))) float s_co[];
  const int C = g.C, cg = C / kVec;
  const long long stride = (long long)gridDim.x * kT;
  const int c8 = (int)(((long long)blockIdx.x * kT + threadIdx.x) & (cg - 1));
  const double inv_m = 1.0 / (double)M;
  for (int c = threadIdx.x; c < C; c += kT) {
    double a, b;
    acc_sums(acc, C, c, a, b);
    const float invstd = co.invstd[c];
    const float gam = co.gamma ? co.gamma[c] : 1.f;
    s_co[c] = gam * invstd;
    s_co[C + c] = (float)(a * inv_m);
    s_co[2 * C + c] = (float)(b * inv_m) * invstd * invstd;
    s_co[3 * C + c] = co.mean[c];
    s_co[4 * C + c] = co.scale[c];
    s_co[5 * C + c] = co.shift[c];
    if (blockIdx.x == 0) {
      if (co.dgamma) co.dgamma[c] = (float)(b * invstd);
      if (co.dbeta) co.dbeta[c] = (float)a;
    }
  }
  __syncthreads();
  zero_duty(zero, nzero);
  float ca[kVec], cb[kVec], cc[kVec], mu[kVec], sc[kVec], sh[kVec];
  lds8(s_co + c8 * kVec, ca);
  lds8(s_co + C + c8 * kVec, cb);
  lds8(s_co + 2 * C + c8 * kVec, cc);
  lds8(s_co + 3 * C + c8 * kVec, mu);
  lds8(s_co + 4 * C + c8 * kVec, sc);
  lds8(s_co + 5 * C + c8 * kVec, sh);
  const int sh_cg = __builtin_ctz(cg);   // cg is a power of two
  // (two vectors per step measured slower here: 146 vs 131 us at batch 128)
  for (long long v = (long long)blockIdx.x * kT + threadIdx.x; v < nvec; v += stride) {
    float gv[kVec], xv[kVec], o[kVec];
    V8<T>::load(x + v * kVec, xv);
    pool_grad8<T>(dy, pos, g, (long long)((unsigned long long)v >> sh_cg), c8, gv);
#pragma unroll
    for (int i = 0; i < kVec; ++i) {
      const bool on = stored_val<T>(fmaxf(fmaf(xv[i] - mu[i], sc[i], sh[i]), 0.f)) > 0.f;
      const float gg = on ? gv[i] : 0.f;
      o[i] = ca[i] * (gg - cb[i] - (xv[i] - mu[i]) * cc[i]);
    }
    V8<T>::store(dx + v * kVec, o);
  }
}

// ---- the ResNet stem's 3x3 / stride 2 / pad 1 pool: gradients per 2x2 input quad ----
// Input row 2i is in window row i only, row 2i+1 in rows i and i+1 (same for columns), so the
// quad {2i, 2i+1} x {2j, 2j+1} needs exactly the 4 windows (i..i+1) x (j..j+1), and the window
// position each pixel has in each of them is fixed: one gather of 4 windows serves 4 pixels.
// Per pixel that is 24 bytes of position + gradient reads instead of 96 (4 clamped windows each
// in pool_grad8) -- the generic path was gather-bound at ~3x its x-stream time.
struct Quad8 {
  float g[4][kVec];   // pixel (2i + a, 2j + b) -> g[2a + b]
};

template <typename T>
__device__ __forceinline__ void quad_grad8(const T* __restrict__ dy,
                                           const uint8_t* __restrict__ pos, const PoolG& g,
                                           int n, int i, int j, int c8, Quad8& o) {
  uint2 pk[4];
  float d[4][kVec];
  bool ok[4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int w = 2 * a + b;
      ok[w] = i + a < g.OH && j + b < g.OW;
      const int oh = ok[w] ? i + a : i, ow = ok[w] ? j + b : j;   // clamped: always a window
      const long long off = (((long long)n * g.OH + oh) * g.OW + ow) * g.C + (long long)c8 * kVec;
      pk[w] = *reinterpret_cast<const uint2*>(pos + off);
      V8<T>::load(dy + off, d[w]);
    }
  // (window, in-window position) that points at each pixel of the quad
  constexpr int kPosOf[4][4] = {{4, -1, -1, -1}, {5, 3, -1, -1}, {7, -1, 1, -1}, {8, 6, 2, 0}};
#pragma unroll
  for (int px = 0; px < 4; ++px)
#pragma unroll
    for (int e = 0; e < kVec; ++e) o.g[px][e] = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t ps[2] = {pk[w].x, pk[w].y};
#pragma unroll
    for (int px = 0; px < 4; ++px) {
      const int want = kPosOf[px][w];
      if (want < 0) continue;
#pragma unroll
      for (int e = 0; e < kVec; ++e)
        o.g[px][e] += (ok[w] && ((ps[e >> 2] >> (8 * (e & 3))) & 0xff) == (uint32_t)want)
                          ? d[w][e] : 0.f;
    }
  }
}

__device__ __forceinline__ void quad_of(unsigned qd, int QH, int QW, int* n, int* i, int* j) {
  const unsigned nq = qd / (unsigned)QW;
  *j = (int)(qd - nq * (unsigned)QW);
  const unsigned nn = nq / (unsigned)QH;
  *i = (int)(nq - nn * (unsigned)QH);
  *n = (int)nn;
}

// Backward reduction over quads (rows of the Geo layout are quads; 4 pixel vectors each).
template <typename T>
__global__ __launch_bounds__(kT) void bn_pool_bwd_reduce_q_kernel(const T* __restrict__ dy,
                                                                  const uint8_t* __restrict__ pos,
                                                                  const T* __restrict__ x,
                                                                  long long NQ, long long rpb,
                                                                  PoolG g, ArenaBNBwd co,
                                                                  double* __restrict__ acc) {
  __shared__ __attribute__((aligned(16))) float s_c[3 * 256];
  const int C = g.C;
  for (int c = threadIdx.x; c < C; c += kT) {
    s_c[c] = co.mean[c];
    s_c[C + c] = co.scale[c];
    s_c[2 * C + c] = co.shift[c];
  }
  __syncthreads();
  const Geo q = geo(C);
  long long r0, r1;
  block_rows(NQ, rpb, &r0, &r1);
  const int QH = (g.H + 1) / 2, QW = (g.W + 1) / 2;
  float sg[kVec], sgx[kVec], mu[kVec], sc[kVec], sh[kVec];
#pragma unroll
  for (int e = 0; e < kVec; ++e) sg[e] = sgx[e] = 0.f;
  lds8(s_c + q.g * kVec, mu);
  lds8(s_c + C + q.g * kVec, sc);
  lds8(s_c + 2 * C + q.g * kVec, sh);
  if (q.slot < q.rip) {
    for (long long r = r0 + q.slot; r < r1; r += q.rip) {
      int n, i, j;
      quad_of((unsigned)r, QH, QW, &n, &i, &j);
      Quad8 gq;
      quad_grad8<T>(dy, pos, g, n, i, j, q.g, gq);
#pragma unroll
      for (int px = 0; px < 4; ++px) {
        const int h = 2 * i + (px >> 1), w = 2 * j + (px & 1);
        if (h >= g.H || w >= g.W) continue;
        float v[kVec];
        V8<T>::load(x + (((long long)n * g.H + h) * g.W + w) * C + (long long)q.g * kVec, v);
#pragma unroll
        for (int e = 0; e < kVec; ++e) {
          const bool on = stored_val<T>(fmaxf(fmaf(v[e] - mu[e], sc[e], sh[e]), 0.f)) > 0.f;
          const float gg = on ? gq.g[px][e] : 0.f;
          sg[e] += gg;
          sgx[e] = fmaf(gg, v[e] - mu[e], sgx[e]);
        }
      }
    }
  }
  __shared__ float s_g[kT * kVec], s_gx[kT * kVec];
  if (q.slot < q.rip) {
#pragma unroll
    for (int e = 0; e < kVec; ++e) {
      s_g[q.slot * q.cw + q.gl * kVec + e] = sg[e];
      s_gx[q.slot * q.cw + q.gl * kVec + e] = sgx[e];
    }
  }
  __syncthreads();
  for (int cl = threadIdx.x; cl < q.cw; cl += kT) {
    float a = 0.f, b = 0.f;
    for (int s2 = 0; s2 < q.rip; ++s2) {
      a += s_g[s2 * q.cw + cl];
      b += s_gx[s2 * q.cw + cl];
    }
    unsafeAtomicAdd(acc + q.cb + cl, (double)a);
    unsafeAtomicAdd(acc + C + q.cb + cl, (double)b);
  }
}

// Backward reduction from the forward's selected inputs. Window o's gradient reaches only its
// argmax pixel, whose x the forward saved as xsel[o] (and whose ReLU bit follows from it), so
//   sum g = sum_o dy[o] on(xsel[o]),   sum g (x - mean) = sum_o dy[o] on(xsel[o]) (xsel[o] - mean)
// -- the per-pixel sums of bn_pool_bwd_reduce_q_kernel regrouped by window: two pooled-size
// streams (dy, xsel) instead of x (4x the pooled size) plus the argmax gather. Rows: pooled pixels.
template <typename T>
__global__ __launch_bounds__(kT) void bn_pool_bwd_reduce_sel_kernel(const T* __restrict__ dy,
                                                                    const T* __restrict__ xsel,
                                                                    long long MO, long long rpb,
                                                                    int C, ArenaBNBwd co,
                                                                    double* __restrict__ acc) {
  __shared__ __attribute__((aligned(16))) float s_c[3 * 256];
  for (int c = threadIdx.x; c < C; c += kT) {
    s_c[c] = co.mean[c];
    s_c[C + c] = co.scale[c];
    s_c[2 * C + c] = co.shift[c];
  }
  __syncthreads();
  const Geo q = geo(C);
  long long r0, r1;
  block_rows(MO, rpb, &r0, &r1);
  float sg[kVec], sgx[kVec], mu[kVec], sc[kVec], sh[kVec];
#pragma unroll
  for (int e = 0; e < kVec; ++e) sg[e] = sgx[e] = 0.f;
  lds8(s_c + q.g * kVec, mu);
  lds8(s_c + C + q.g * kVec, sc);
  lds8(s_c + 2 * C + q.g * kVec, sh);
  if (q.slot < q.rip) {
    constexpr int U = 4;   // rows in flight per thread
    for (long long r = r0 + q.slot; r < r1; r += U * q.rip) {
      float d[U][kVec], v[U][kVec];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long ru = r + u * q.rip;
        const long long rc = ru < r1 ? ru : r;   // clamped: branch-free loads
        V8<T>::load(dy + rc * C + (long long)q.g * kVec, d[u]);
        V8<T>::load(xsel + rc * C + (long long)q.g * kVec, v[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool row_ok = r + u * q.rip < r1;
#pragma unroll
        for (int e = 0; e < kVec; ++e) {
          const bool on = row_ok &&
                          stored_val<T>(fmaxf(fmaf(v[u][e] - mu[e], sc[e], sh[e]), 0.f)) > 0.f;
          const float gg = on ? d[u][e] : 0.f;
          sg[e] += gg;
          sgx[e] = fmaf(gg, v[u][e] - mu[e], sgx[e]);
        }
      }
    }
  }
  __shared__ float s_g[kT * kVec], s_gx[kT * kVec];
  if (q.slot < q.rip) {
#pragma unroll
    for (int e = 0; e < kVec; ++e) {
      s_g[q.slot * q.cw + q.gl * kVec + e] = sg[e];
      s_gx[q.slot * q.cw + q.gl * kVec + e] = sgx[e];
    }
  }
  __syncthreads();
  for (int cl = threadIdx.x; cl < q.cw; cl += kT) {
    float a = 0.f, b = 0.f;
    for (int s2 = 0; s2 < q.rip; ++s2) {
      a += s_g[s2 * q.cw + cl];
      b += s_gx[s2 * q.cw + cl];
    }
    unsafeAtomicAdd(acc + q.cb + cl, (double)a);
    unsafeAtomicAdd(acc + C + q.cb + cl, (double)b);
  }
}

// dx over quads; dynamic shared memory: 6 * C floats (as bn_pool_bwd_dx_kernel)
template <typename T>
__global__ __launch_bounds__(kT) void bn_pool_bwd_dx_q_kernel(const T* __restrict__ dy,
                                                              const uint8_t* __restrict__ pos,
                                                              const T* __restrict__ x,
                                                              T* __restrict__ dx, long long nqv,
                                                              PoolG g, ArenaBNBwd co,
                                                              const double* __restrict__ acc,
                                                              long long M,
                                                              double* __restrict__ zero,
                                                              int nzero) {
  extern __shared__ __attribute__((aligned(16))) float s_co[];
  const int C = g.C, cg = C / kVec;
  const long long stride = (long long)gridDim.x * kT;
  const int c8 = (int)(((long long)blockIdx.x * kT + threadIdx.x) & (cg - 1));
  const double inv_m = 1.0 / (double)M;
  for (int c = threadIdx.x; c < C; c += kT) {
    double a, b;
    acc_sums(acc, C, c, a, b);
    const float invstd = co.invstd[c];
    const float gam = co.gamma ? co.gamma[c] : 1.f;
    s_co[c] = gam * invstd;
    s_co[C + c] = (float)(a * inv_m);
    s_co[2 * C + c] = (float)(b * inv_m) * invstd * invstd;
    s_co[3 * C + c] = co.mean[c];
    s_co[4 * C + c] = co.scale[c];
    s_co[5 * C + c] = co.shift[c];
    if (blockIdx.x == 0) {
      if (co.dgamma) co.dgamma[c] = (float)(b * invstd);
      if (co.dbeta) co.dbeta[c] = (float)a;
    }
  }
  __syncthreads();
  zero_duty(zero, nzero);
  float ca[kVec], cb[kVec], cc[kVec], mu[kVec], sc[kVec], sh[kVec];
  lds8(s_co + c8 * kVec, ca);
  lds8(s_co + C + c8 * kVec, cb);
  lds8(s_co + 2 * C + c8 * kVec, cc);
  lds8(s_co + 3 * C + c8 * kVec, mu);
  lds8(s_co + 4 * C + c8 * kVec, sc);
  lds8(s_co + 5 * C + c8 * kVec, sh);
  const int sh_cg = __builtin_ctz(cg);
  const int QH = (g.H + 1) / 2, QW = (g.W + 1) / 2;
  for (long long v = (long long)blockIdx.x * kT + threadIdx.x; v < nqv; v += stride) {
    int n, i, j;
    quad_of((unsigned)((unsigned long long)v >> sh_cg), QH, QW, &n, &i, &j);
    Quad8 gq;
    quad_grad8<T>(dy, pos, g, n, i, j, c8, gq);
#pragma unroll
    for (int px = 0; px < 4; ++px) {
      const int h = 2 * i + (px >> 1), w = 2 * j + (px & 1);
      if (h >= g.H || w >= g.W) continue;
      const long long off = (((long long)n * g.H + h) * g.W + w) * C + (long long)c8 * kVec;
      float xv[kVec], o[kVec];
      V8<T>::load(x + off, xv);
#pragma unroll
      for (int e = 0; e < kVec; ++e) {
        const bool on = stored_val<T>(fmaxf(fmaf(xv[e] - mu[e], sc[e], sh[e]), 0.f)) > 0.f;
        const float gg = on ? gq.g[px][e] : 0.f;
        o[e] = ca[e] * (gg - cb[e] - (xv[e] - mu[e]) * cc[e]);
      }
      V8<T>::store(dx + off, o);
    }
  }
}

// Blocks for a reduction over M rows: >= 8 row rounds per thread (the loops issue 4 or 2 rounds
// of loads at once), as many blocks as that allows up to 512 partials. The 7x7 ResNet layers
// (M = 6272) need the small per-thread share to fill the chip: at 32 rounds per thread they ran
// 49 blocks and reached ~1 TB/s.
// Both limits are runtime-tunable for sweeps (scripts/bn_bench.py); the workspace size follows.
long long g_max_reduce_blocks = 512;
int g_bn_nt = 1;           // non-temporal loads in the apply / dx passes (runtime switch for A/Bs)
// stem-pool quad reduction grid, x the usual (A/B switch): 1-2x measured ~15 us/step faster than
// 4x, 8x 56 us slower (profiles/r3_stem_quad_grid_ab.jsonl): fewer blocks, fewer same-address atomics
long long g_pool_quad_mult = 2;
long long g_min_rounds = 8;

// acc mode pays one fp64 (a, b) atomic pair per block and channel at the end of the pass; above
// this many pairs their drain would cost more than the partial merge. With the channel-sliced
// grid (Geo) a reduction emits at most 512 x 256 pairs, so every layer takes acc mode.
long long g_acc_max_pairs = 1 << 18;

// Channel slices of a reduction block row (Geo): one up to 256 channels, else 32-group slices.
int chan_slices(int C) {
  const int cg = C / kVec;
  return cg > 32 ? cg / 32 : 1;
}

// Row blocks of a reduction over M rows (the grid is row blocks x chan_slices(C)).
long long reduce_blocks(long long M, int C, long long* rpb) {
  const int ns = chan_slices(C);
  const int rip = kT / (C / kVec / ns);
  long long rounds = (M + rip - 1) / rip;
  long long nb = (rounds + g_min_rounds - 1) / g_min_rounds;
  long long maxb = g_max_reduce_blocks / ns;
  maxb = maxb < 1 ? 1 : maxb;
  nb = nb < 1 ? 1 : (nb > maxb ? maxb : nb);
  long long r = (M + nb - 1) / nb;
  r = (r + rip - 1) / rip * rip;  // whole rounds per block
  *rpb = r;
  return (M + r - 1) / r;
}

// Grid of the streaming passes (apply, dx): at most g_elem_max_blocks blocks, each thread then
// loops over its vectors. Every block derives its per-channel coefficients in its prologue (from
// the fp64 sums: ARENA_ACC_REP replicas x 2 x C loads), so fewer, fatter blocks pay that less
// often: ResNet-50 step 11.718 / 11.677 / 11.578 / 11.811 ms at 4096 / 2048 / 1024 / 512
// (profiles/r5_ebk_ab.jsonl, same process). Going further on the small layers -- a floor of 8 or
// 16 vectors per thread down to 256 blocks -- lost on every shape (25088 x 256 apply 8.3 -> 8.7 /
// 10.1 us; step 11.411 -> 11.446 / 11.580 ms, profiles/r6_bn_min_vpt_ab.jsonl): those passes are
// latency-bound by their few µs of issue, not by the coefficient prologue.
int g_elem_max_blocks = 1024;

int elementwise_blocks(long long nvec) {
  long long b = (nvec + 2LL * kT - 1) / (2LL * kT);
  return (int)(b < 1 ? 1 : (b > g_elem_max_blocks ? g_elem_max_blocks : b));
}

// The dx pass's grid (one vector per thread per iteration): at most g_dx_max_blocks blocks.
// Channel-sliced grids (Slice) for the apply / dx passes of layers with C > 256. ResNet-50 step,
// interleaved replays (profiles/r5_slice_ab.jsonl): flat grids with 4096 dx blocks 11.990 ms,
// sliced 11.651, sliced + 1024 dx blocks 11.502 (flat + 1024: 11.723).
int g_dx_max_blocks = 1024;
int g_bn_slice = 1;

// (x, y) grid of a streaming pass with `total` blocks wanted: flat, or row blocks x channel
// slices when slicing is on and C > 256 (the same number of blocks in all).
dim3 stream_grid(long long total, int C) {
  const int cg = C / kVec;
  if (!g_bn_slice || cg <= kSliceG) return dim3((unsigned)total);
  const int ns = cg / kSliceG;
  const long long bx = total / ns;
  return dim3((unsigned)(bx < 1 ? 1 : bx), (unsigned)ns);
}

int stream_lds_channels(int C) { return (g_bn_slice && C / kVec > kSliceG) ? kSliceG * kVec : C; }

bool bad_shape(long long M, int C) {
  return M <= 0 || C <= 0 || C % kVec != 0 || C > kMaxC || (kT % (C / kVec)) != 0;
}

}  // namespace

extern "C" {

void arena_bn_set_fin_max_blocks(int p) { g_fin_max_p = p < 1 ? 1 : (p > 64 ? 64 : p); }

void arena_bn_set_nt(int on) { g_bn_nt = on ? 1 : 0; }

void arena_bn_set_elem_max_blocks(int b) { g_elem_max_blocks = b < 64 ? 64 : (b > 65536 ? 65536 : b); }

void arena_bn_set_dx_max_blocks(int b) { g_dx_max_blocks = b < 64 ? 64 : (b > 65536 ? 65536 : b); }

void arena_bn_set_slice(int on) { g_bn_slice = on ? 1 : 0; }

void arena_bn_set_pool_quad_mult(int m) { g_pool_quad_mult = m < 1 ? 1 : (m > 16 ? 16 : m); }

void arena_bn_set_acc_max_pairs(long long p) { g_acc_max_pairs = p < 0 ? 0 : p; }
long long arena_bn_acc_max_pairs() { return g_acc_max_pairs; }

// 1 when a pass over M x C takes acc mode (its reduction emits few enough sums).
int arena_bn_acc_ok(long long M, int C) {
  if (bad_shape(M, C)) return 0;
  long long rpb;
  return reduce_blocks(M, C, &rpb) * C <= g_acc_max_pairs ? 1 : 0;
}

void arena_bn_set_reduce_geometry(long long max_blocks, long long min_rounds) {
  g_max_reduce_blocks = max_blocks < 1 ? 1 : (max_blocks > 4096 ? 4096 : max_blocks);
  g_min_rounds = min_rounds < 1 ? 1 : min_rounds;
}

// Level-2 workspace of the finalize kernels for `nblk` partials of C channels (doubles), and the
// ticket counters they need: ARENA_BN_TICKETS_PER_SET per launch, zero on entry and left zero.
long long arena_bn_lvl2_doubles(long long nblk, int C) {
  return (long long)((C + 63) / 64) * fin_blocks_per_group((int)nblk) * 3 * 64;
}

long long arena_bn_workspace_floats(long long M, int C) {
  if (bad_shape(M, C)) return 0;
  long long rpb;
  return reduce_blocks(M, C, &rpb) * 2LL * C;
}

// dtype: 0 = f32, 1 = bf16 (all activation tensors share it)
// ext_nblk > 0: `part` already holds the statistics partials of x ([ext_nblk][2][C], ext_rpb rows
// each), written by the producing convolution's epilogue (conv_kernels.hip): no statistics pass.
// mask (optional, relu only): [M * C / 8] bytes, bit i of byte v = (y[v * 8 + i] > 0)
// acc (training, optional): fp64 [2][C] accumulators, zero on entry. acc_ready: the producing
// convolution already added the statistics of x (no statistics pass); else the statistics pass
// runs in acc mode. Either way the apply pass derives the coefficients from the sums (no finalize
// launch) and LEAVES THEM IN PLACE: the caller hands `acc` to this layer's arena_bn_bwd as its
// `zero` set (or zeroes it itself when no backward follows).
// zero / nzero (optional): doubles block 0 of the apply pass clears (this layer's backward
// accumulators of the previous step, see arena_bn_bwd fin_dx).
hipError_t arena_bn_fwd(int dtype, const void* x, const void* res, void* y, uint8_t* mask,
                        long long M, int C, int relu, int training, float* part, int ext_nblk,
                        long long ext_rpb,
                        double* lvl2, unsigned* tickets, ArenaBNStats st, double* acc,
                        int acc_ready, double* zero, int nzero, hipStream_t stream) {
  if (bad_shape(M, C)) return hipErrorInvalidValue;
  const int groups = (C + 63) / 64;
  const int ns = chan_slices(C);
  if (training && acc != nullptr && !acc_ready) {
    long long rpb;
    if (reduce_blocks(M, C, &rpb) * C > g_acc_max_pairs) acc = nullptr;   // partials instead
  }
  const bool fin = training && acc != nullptr;
  if (fin) {
    if (!acc_ready) {
      long long rpb;
      const long long nb = reduce_blocks(M, C, &rpb);
      if (dtype == 1)
        hipLaunchKernelGGL(bn_stats_kernel<uint16_t>, dim3(nb, ns), dim3(kT), 0, stream,
                           static_cast<const uint16_t*>(x), M, C, rpb, nullptr, acc);
      else
        hipLaunchKernelGGL(bn_stats_kernel<float>, dim3(nb, ns), dim3(kT), 0, stream,
                           static_cast<const float*>(x), M, C, rpb, nullptr, acc);
    }
  } else if (training && ext_nblk > 0) {
    if (ext_rpb <= 0 || (long long)ext_nblk * ext_rpb < M) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3(groups, fin_blocks_per_group(ext_nblk)),
                       dim3(kT), 0, stream, part, ext_nblk, M, C, ext_rpb, lvl2, tickets, st);
  } else if (training) {
    long long rpb;
    const long long nb = reduce_blocks(M, C, &rpb);
    if (dtype == 1)
      hipLaunchKernelGGL(bn_stats_kernel<uint16_t>, dim3(nb, ns), dim3(kT), 0, stream,
                         static_cast<const uint16_t*>(x), M, C, rpb, part, nullptr);
    else
      hipLaunchKernelGGL(bn_stats_kernel<float>, dim3(nb, ns), dim3(kT), 0, stream,
                         static_cast<const float*>(x), M, C, rpb, part, nullptr);
    hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3(groups, fin_blocks_per_group((int)nb)),
                       dim3(kT), 0, stream, part, (int)nb, M, C, rpb, lvl2, tickets, st);
  }
  const long long nvec = M * (C / kVec);
  const dim3 agrid = stream_grid(elementwise_blocks(nvec), C);
  const int acs = stream_lds_channels(C);
  const int cg = C / kVec;
#define ARENA_BN_APPLY_NT(TT, R, S, NT, F)                                                   \
  hipLaunchKernelGGL((bn_apply_kernel<TT, R, S, NT, F>), agrid, dim3(kT), 3 * acs * 4, stream, \
                     static_cast<const TT*>(x), static_cast<const TT*>(res), static_cast<TT*>(y), \
                     mask, st, acc, M, nvec, cg, zero, nzero)
#define ARENA_BN_APPLY_F(TT, R, S, F)                                                        \
  do { if (g_bn_nt) ARENA_BN_APPLY_NT(TT, R, S, true, F);                                    \
       else ARENA_BN_APPLY_NT(TT, R, S, false, F); } while (0)
#define ARENA_BN_APPLY(TT, R, S)                                                             \
  do { if (fin) ARENA_BN_APPLY_F(TT, R, S, true); else ARENA_BN_APPLY_F(TT, R, S, false); }  \
  while (0)
  const bool r = relu != 0, s = res != nullptr;
  if (dtype == 1) {
    if (r && s) ARENA_BN_APPLY(uint16_t, true, true);
    else if (r) ARENA_BN_APPLY(uint16_t, true, false);
    else if (s) ARENA_BN_APPLY(uint16_t, false, true);
    else ARENA_BN_APPLY(uint16_t, false, false);
  } else {
    if (r && s) ARENA_BN_APPLY(float, true, true);
    else if (r) ARENA_BN_APPLY(float, true, false);
    else if (s) ARENA_BN_APPLY(float, false, true);
    else ARENA_BN_APPLY(float, false, false);
  }
#undef ARENA_BN_APPLY
#undef ARENA_BN_APPLY_F
#undef ARENA_BN_APPLY_NT
  return hipGetLastError();
}

// ext_nblk > 0: `part` already holds the backward partials of (dy, x) ([ext_nblk][2][C]), written
// by the epilogue of the backward-data convolution that produced dy (conv_kernels.hip, EPI 2):
// no reduction pass.
// acc != null (and no external partials): the reduction runs in acc mode. fin_dx: the dx pass
// derives the coefficients from the sums (no finalize launch) and leaves them in place -- the
// caller owns `acc` per layer and hands it to the layer's next arena_bn_fwd as its `zero` set;
// else a one-thread-per-channel finalize writes the coefficients and zeroes `acc`.
// zero / nzero (optional): doubles block 0 of the dx pass clears (the forward's statistics sums
// of this layer, whose last reader -- the apply pass -- has finished).
// x2 / mean2 / acc2 (optional): the second BN's input, batch mean and backward sums (S2 in
// bn_bwd_dx_kernel); only with relu, no dres and sums fed or summed here (fin_dx).
hipError_t arena_bn_bwd(int dtype, const void* dy, const uint8_t* mask, const void* x, void* dx,
                        void* dres, long long M, int C, int relu, float* part, int ext_nblk,
                        double* lvl2, unsigned* tickets, ArenaBNBwd co, double* acc, int fin_dx,
                        double* zero, int nzero, const void* x2, const float* mean2,
                        double* acc2, hipStream_t stream) {
  if (bad_shape(M, C)) return hipErrorInvalidValue;
  if (relu && mask == nullptr) return hipErrorInvalidValue;
  long long rpb;
  long long nb = reduce_blocks(M, C, &rpb);
  const int ns = chan_slices(C);
  // ext_nblk < 0: the producer already summed into acc (fin_dx required): no reduction
  const bool pre = ext_nblk < 0;
  if (pre && (acc == nullptr || !fin_dx)) return hipErrorInvalidValue;
  const bool acc_mode = acc != nullptr && (pre || (ext_nblk == 0 && nb * C <= g_acc_max_pairs));
  double* am = acc_mode ? acc : nullptr;
  if (ext_nblk > 0) {
    nb = ext_nblk;
  } else if (!pre) {
#define ARENA_BN_RED(TT, R)                                                                  \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<TT, R>), dim3(nb, ns), dim3(kT), 0, stream,     \
                     static_cast<const TT*>(dy), mask, static_cast<const TT*>(x), M, C, rpb, \
                     part, co, am)
    if (dtype == 1) {
      if (relu) ARENA_BN_RED(uint16_t, true);
      else ARENA_BN_RED(uint16_t, false);
    } else {
      if (relu) ARENA_BN_RED(float, true);
      else ARENA_BN_RED(float, false);
    }
#undef ARENA_BN_RED
  }
  const bool fin = acc_mode && fin_dx;
  if (acc_mode && !fin)
    hipLaunchKernelGGL(bn_bwd_acc_finalize_kernel, dim3((C + kT - 1) / kT), dim3(kT), 0, stream,
                       acc, M, C, co);
  else if (!acc_mode)
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64, fin_blocks_per_group((int)nb)),
                       dim3(kT), 0, stream, part, (int)nb, M, C, lvl2, tickets, co);
  const long long nvec = M * (C / kVec);
  long long ne = (nvec + kT - 1) / kT;
  ne = ne < 1 ? 1 : (ne > g_dx_max_blocks ? g_dx_max_blocks : ne);
  const dim3 dgrid = stream_grid(ne, C);
  const int dcs = stream_lds_channels(C);
  const int cg = C / kVec;
#define ARENA_BN_DX_NT(TT, R, S, NT, F)                                                      \
  hipLaunchKernelGGL((bn_bwd_dx_kernel<TT, R, S, NT, F>), dgrid, dim3(kT), 4 * dcs * 4,     \
                     stream, static_cast<const TT*>(dy), mask, static_cast<const TT*>(x),    \
                     static_cast<TT*>(dx), static_cast<TT*>(dres), nvec, cg, co, acc, M,     \
                     zero, nzero, nullptr, nullptr, nullptr)
#define ARENA_BN_DX_F(TT, R, S, F)                                                           \
  do { if (g_bn_nt) ARENA_BN_DX_NT(TT, R, S, true, F);                                       \
       else ARENA_BN_DX_NT(TT, R, S, false, F); } while (0)
#define ARENA_BN_DX(TT, R, S)                                                                \
  do { if (fin) ARENA_BN_DX_F(TT, R, S, true); else ARENA_BN_DX_F(TT, R, S, false); }        \
  while (0)
  const bool r = relu != 0, s = dres != nullptr;
  if (x2 != nullptr) {
    if (!(fin && r && !s) || mean2 == nullptr || acc2 == nullptr)
      return hipErrorInvalidValue;
#define ARENA_BN_DX_S2(TT, NT)                                                                 \
  hipLaunchKernelGGL((bn_bwd_dx_kernel<TT, true, false, NT, true, true>), dgrid,              \
                     dim3(kT), 4 * dcs * 4, stream, static_cast<const TT*>(dy), mask,           \
                     static_cast<const TT*>(x), static_cast<TT*>(dx), nullptr, nvec, cg, co,    \
                     acc, M, zero, nzero, static_cast<const TT*>(x2), mean2, acc2)
    if (dtype == 1) {
      if (g_bn_nt) ARENA_BN_DX_S2(uint16_t, true); else ARENA_BN_DX_S2(uint16_t, false);
    } else {
      if (g_bn_nt) ARENA_BN_DX_S2(float, true); else ARENA_BN_DX_S2(float, false);
    }
#undef ARENA_BN_DX_S2
  } else if (dtype == 1) {
    if (r && s) ARENA_BN_DX(uint16_t, true, true);
    else if (r) ARENA_BN_DX(uint16_t, true, false);
    else if (s) ARENA_BN_DX(uint16_t, false, true);
    else ARENA_BN_DX(uint16_t, false, false);
  } else {
    if (r && s) ARENA_BN_DX(float, true, true);
    else if (r) ARENA_BN_DX(float, true, false);
    else if (s) ARENA_BN_DX(float, false, true);
    else ARENA_BN_DX(float, false, false);
  }
#undef ARENA_BN_DX
#undef ARENA_BN_DX_F
#undef ARENA_BN_DX_NT
  return hipGetLastError();
}

// Fused stem forward (training): y = the max pool of relu(bn(x)), pos = its in-window argmax.
// Statistics: acc-mode sums `fin` from the producing conv, or (fin == null) its per-tile partials
// `part` [ext_nblk][2][C] (ext_rpb rows each), merged first by the finalize kernel (lvl2 /
// tickets as in arena_bn_fwd). Only the 3x3 / 2 style pools whose inputs have <= 2 x 2 candidate
// windows, C % 8 == 0, C <= 256. zero / nzero: see arena_bn_fwd.
hipError_t arena_bn_pool_fwd(int dtype, const void* x, void* y, uint8_t* pos, void* xsel, int N,
                             int H, int W,
                             int C, int k, int s, int p, ArenaBNStats st, const double* fin,
                             const float* part, int ext_nblk, long long ext_rpb, double* lvl2,
                             unsigned* tickets, double* zero, int nzero, hipStream_t stream) {
  PoolG g{N, H, W, C, (H + 2 * p - k) / s + 1, (W + 2 * p - k) / s + 1, k, s, p};
  const long long M = (long long)N * H * W;
  if (bad_shape(M, C) || C > 256 || (k + s - 1) / s != 2 || 2 * p > k || g.OH <= 0 || g.OW <= 0)
    return hipErrorInvalidValue;
  if (fin == nullptr) {
    if (part == nullptr || ext_nblk <= 0 || ext_rpb <= 0 || (long long)ext_nblk * ext_rpb < M ||
        lvl2 == nullptr || tickets == nullptr)
      return hipErrorInvalidValue;
    hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3((C + 63) / 64, fin_blocks_per_group(ext_nblk)),
                       dim3(kT), 0, stream, part, ext_nblk, M, C, ext_rpb, lvl2, tickets, st);
  }
  const int cg = C / kVec;
  const dim3 grid((unsigned)(N * g.OH), (unsigned)((g.OW * cg + kT - 1) / kT));
#define ARENA_BN_POOL(TT, F)                                                                   \
  hipLaunchKernelGGL((bn_pool_fwd_kernel<TT, F>), grid, dim3(kT), 3 * C * 4, stream,          \
                     static_cast<const TT*>(x), static_cast<TT*>(y), pos,                     \
                     static_cast<TT*>(xsel), st, fin, M, g, zero, nzero)
  if (dtype == 1) {
    if (fin) ARENA_BN_POOL(uint16_t, true); else ARENA_BN_POOL(uint16_t, false);
  } else {
    if (fin) ARENA_BN_POOL(float, true); else ARENA_BN_POOL(float, false);
  }
#undef ARENA_BN_POOL
  return hipGetLastError();
}

// Fused stem backward: dy is the pooled output's gradient, pos the forward's argmax; the
// reduction adds into acc (fp64 [2][C], zero on entry: the layer's own backward set, left in
// place for its next forward to zero) and the dx pass derives its coefficients from it.
// co.scale / co.shift: the forward's (ReLU mask recomputed from x). zero / nzero: see arena_bn_bwd.
hipError_t arena_bn_pool_bwd(int dtype, const void* dy, const uint8_t* pos, const void* x,
                             const void* xsel, void* dx, int N, int H, int W, int C, int k, int s,
                             int p, ArenaBNBwd co, double* acc, double* zero, int nzero,
                             hipStream_t stream) {
  PoolG g{N, H, W, C, (H + 2 * p - k) / s + 1, (W + 2 * p - k) / s + 1, k, s, p};
  const long long M = (long long)N * H * W;
  if (bad_shape(M, C) || C > 256 || M >= (1LL << 31) || acc == nullptr || co.scale == nullptr ||
      co.shift == nullptr || (k + s - 1) / s != 2 || 2 * p > k || g.OH <= 0 || g.OW <= 0)
    return hipErrorInvalidValue;
  // up to 4x the usual reduction grid: the stem's C = 64 leaves 512 row blocks latency-bound
  // on their gathers, and 2048 x 64 sums are still few atomics
  const long long saved_max = g_max_reduce_blocks;
  g_max_reduce_blocks = saved_max * 4;
  long long rpb;
  const long long nb = reduce_blocks(M, C, &rpb);
  g_max_reduce_blocks = saved_max;
  const long long nvec = M * (C / kVec);
  long long ne = (nvec + kT - 1) / kT;
  ne = ne < 1 ? 1 : (ne > 4096 ? 4096 : ne);
  if (xsel != nullptr) {   // the sums from the forward's selected inputs (pooled-size streams)
    const long long MO = (long long)N * g.OH * g.OW;
    long long orpb;
    const long long onb = reduce_blocks(MO, C, &orpb);
    if (dtype == 1)
      hipLaunchKernelGGL(bn_pool_bwd_reduce_sel_kernel<uint16_t>, dim3(onb, 1), dim3(kT), 0,
                         stream, static_cast<const uint16_t*>(dy),
                         static_cast<const uint16_t*>(xsel), MO, orpb, C, co, acc);
    else
      hipLaunchKernelGGL(bn_pool_bwd_reduce_sel_kernel<float>, dim3(onb, 1), dim3(kT), 0, stream,
                         static_cast<const float*>(dy), static_cast<const float*>(xsel), MO, orpb,
                         C, co, acc);
  }
  if (k == 3 && s == 2 && p == 1) {   // the ResNet stem pool: 2x2 input quads per gather
    const long long NQ = (long long)N * ((H + 1) / 2) * ((W + 1) / 2);
    g_max_reduce_blocks = saved_max * g_pool_quad_mult;
    long long qrpb;
    const long long qnb = reduce_blocks(NQ, C, &qrpb);
    g_max_reduce_blocks = saved_max;
    const long long nqv = NQ * (C / kVec);
    long long qne = (nqv + kT - 1) / kT;
    qne = qne < 1 ? 1 : (qne > 4096 ? 4096 : qne);
#define ARENA_BN_POOL_Q(TT)                                                                     \
    if (xsel == nullptr)                                                                        \
      hipLaunchKernelGGL(bn_pool_bwd_reduce_q_kernel<TT>, dim3(qnb, 1), dim3(kT), 0, stream,   \
                         static_cast<const TT*>(dy), pos, static_cast<const TT*>(x), NQ, qrpb, \
                         g, co, acc);                                                           \
    hipLaunchKernelGGL(bn_pool_bwd_dx_q_kernel<TT>, dim3(qne), dim3(kT), 6 * C * 4, stream,    \
                       static_cast<const TT*>(dy), pos, static_cast<const TT*>(x),              \
                       static_cast<TT*>(dx), nqv, g, co, acc, M, zero, nzero)
    if (dtype == 1) { ARENA_BN_POOL_Q(uint16_t); } else { ARENA_BN_POOL_Q(float); }
#undef ARENA_BN_POOL_Q
    return hipGetLastError();
  }
  if (dtype == 1) {
    if (xsel == nullptr)
      hipLaunchKernelGGL(bn_pool_bwd_reduce_kernel<uint16_t>, dim3(nb, 1), dim3(kT), 0, stream,
                         static_cast<const uint16_t*>(dy), pos, static_cast<const uint16_t*>(x),
                         M, rpb, g, co, acc);
    hipLaunchKernelGGL(bn_pool_bwd_dx_kernel<uint16_t>, dim3(ne), dim3(kT), 6 * C * 4, stream,
                       static_cast<const uint16_t*>(dy), pos, static_cast<const uint16_t*>(x),
                       static_cast<uint16_t*>(dx), nvec, g, co, acc, M, zero, nzero);
  } else {
    if (xsel == nullptr)
      hipLaunchKernelGGL(bn_pool_bwd_reduce_kernel<float>, dim3(nb, 1), dim3(kT), 0, stream,
                         static_cast<const float*>(dy), pos, static_cast<const float*>(x), M, rpb,
                         g, co, acc);
    hipLaunchKernelGGL(bn_pool_bwd_dx_kernel<float>, dim3(ne), dim3(kT), 6 * C * 4, stream,
                       static_cast<const float*>(dy), pos, static_cast<const float*>(x),
                       static_cast<float*>(dx), nvec, g, co, acc, M, zero, nzero);
  }
  return hipGetLastError();
}

}  // extern "C"
