// Fused fp32 MLP training kernels for gfx950 (MI355X).
//
// The reference (mark1222/arena) only *launches* MNIST training images (TF1.5 mnist_with_summaries,
// dist-mnist, Horovod): see docs/userguide/1-tfjob-standalone.md:178-186 and SURVEY.md §2.11. Their
// hot ops -- GEMM+bias+ReLU, dropout, softmax-cross-entropy, Adam -- are implemented here natively:
//
//   linear_fwd      Y = dropout(act(X·Wᵀ + b))      X rows gathered from the dataset in-kernel
//   xent_head       logits = H·W2ᵀ + b2 -> loss, accuracy, dlogits, dZ = (dlogits·W2)⊙mask
//   wgrad_grouped   dW = dZᵀ·X, db = dZᵀ·1 for up to 4 layers in ONE launch, epilogue either
//                   writes the (scaled) gradient into the flat all-reduce bucket or applies Adam
//   adam_flat       Adam over the whole flat parameter buffer (after the gradient all-reduce)
//   softmax_xent    generic row softmax-cross-entropy forward+backward
//   mt_copy_scale   multi-tensor flatten/unflatten with scale (gradient buckets)
//
// All matmul work uses the exact-fp32 MFMA v_mfma_f32_16x16x4_f32 (no TF32 on gfx950), so numerics
// equal an fp32 fmaf chain. Weights are [out][in] (nn.Linear layout), activations row-major.
#include "common.h"
#include "adam.h"

#include <algorithm>
#include <cmath>

using namespace arena;

#ifndef ARENA_EXP
#define ARENA_EXP 0
#endif
#ifdef ARENA_TIMELINE
__device__ long long arena::arena_tl_buf[4 * ARENA_TL_BLOCKS * ARENA_TL_SLOTS];
extern "C" hipError_t arena_timeline_read(long long* host, int clear) {
  const size_t bytes = sizeof(long long) * 4 * ARENA_TL_BLOCKS * ARENA_TL_SLOTS;
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(host, HIP_SYMBOL(arena::arena_tl_buf), bytes);
  if (e == hipSuccess && clear) {
    void* p = nullptr;
    e = hipGetSymbolAddress(&p, HIP_SYMBOL(arena::arena_tl_buf));
    if (e == hipSuccess) e = hipMemset(p, 0, bytes);
  }
  return e;
}
#endif

namespace {

// softmax via the hardware exp2/log2 (v_exp_f32 / v_log_f32, see adam.h): exp(x) = 2^(x log2 e)
constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;

template <int XT>
__device__ __forceinline__ void load4(const ArenaRowSource& s, long long prow, int k, float out[4]) {
  if constexpr (XT == 1) {
    const uint32_t u = *reinterpret_cast<const uint32_t*>(
        static_cast<const uint8_t*>(s.ptr) + prow * (long long)s.ld + k);
#pragma unroll
    for (int j = 0; j < 4; ++j) out[j] = (float)((u >> (8 * j)) & 0xffu) * s.scale;
  } else {
    const float4 v = *reinterpret_cast<const float4*>(static_cast<const float*>(s.ptr) +
                                                      prow * (long long)s.ld + k);
    out[0] = v.x * s.scale; out[1] = v.y * s.scale; out[2] = v.z * s.scale; out[3] = v.w * s.scale;
  }
}

template <int XT>
__device__ __forceinline__ float load1(const ArenaRowSource& s, long long prow, int k) {
  if constexpr (XT == 1) {
    return (float)(static_cast<const uint8_t*>(s.ptr)[prow * (long long)s.ld + k]) * s.scale;
  } else {
    return static_cast<const float*>(s.ptr)[prow * (long long)s.ld + k] * s.scale;
  }
}

// Batch gather: logical row r of this step -> dataset row idx[(cursor*batch + r) % len]. The
// 64-bit modulo (a ~100-instruction software routine on CDNA) is done ONCE per wave on the
// wave-uniform base; per row it is one add + one conditional subtract (host guarantees r < len).
// x mod n for 0 <= x < 2^53 (exact in fp64) and 0 < n < 2^31 via fp64 division + correction:
// branch-free, unlike the ~100-instruction 64-bit integer division routine.
__device__ __forceinline__ long long mod_fp64(double x, long long n) {
  const double dn = (double)n;
  double r = x - floor(x / dn) * dn;
  r = (r < 0.0) ? r + dn : r;
  r = (r >= dn) ? r - dn : r;
  return (long long)r;
}

struct Gather {
  const int* idx;
  long long base, len;
};
__device__ __forceinline__ Gather make_gather(const ArenaRowSource& s) {
  Gather gt{s.idx, 0, s.idx_len};
  if (s.idx != nullptr) {
    const long long cur = (s.cursor ? *s.cursor : 0) + s.cursor_off;
    gt.base = mod_fp64((double)cur * (double)s.batch, s.idx_len);
  }
  return gt;
}
__device__ __forceinline__ int gather_row(const Gather& gt, int r) {
  if (gt.idx == nullptr) return r;
  long long p = gt.base + r;
  p = (p >= gt.len) ? p - gt.len : p;
  return gt.idx[p];
}

// ---------------------------------------------------------------------------------------------
// linear_fwd: Y[M][N] = dropout(act(X·Wᵀ + b)), W stored [N][K] (out x in, nn.Linear layout).
// One 16x16 output tile per workgroup; K split across WAVES waves, partial tiles reduced through
// LDS. Lane (g = l>>4, c = l&15) loads 4 consecutive k of its A row (X) and of its B column (a W
// row) with ONE vector load each; MFMA j consumes k = 16s + 4g + j (a K permutation shared by A
// and B). Every load is unconditional on a clamped address (out-of-range operands are zeroed
// AFTER the load): a branch around a load makes hipcc drain vmcnt per element.
// Grid: (ceil(N/16), ceil(M/16)).
// ---------------------------------------------------------------------------------------------
template <int XT, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void linear_fwd_kernel(
    ArenaRowSource src, const float* __restrict__ W, const float* __restrict__ bias,
    float* __restrict__ Y, int M, int N, int K, int act, uint32_t keep_thr, float inv_keep,
    uint32_t seed, const long long* step_src) {
  constexpr int CH = 8;
  const int lane = lane_id(), w = wave_id();
  const int g = lane >> 4, c = lane & 15;
  const int n0 = blockIdx.x * 16, m0 = blockIdx.y * 16;
  const int rowc = min(m0 + c, M - 1), colc = min(n0 + c, N - 1);
  const Gather gt = make_gather(src);
  const uint32_t step = step_src ? (uint32_t)(*step_src) : 0u;  // early: off the epilogue's path
  const float bv = bias ? bias[min(n0 + (int)(threadIdx.x & 15), N - 1)] : 0.f;  // epilogue t&15
  const long long prow = gather_row(gt, rowc);
  const float* wrow = W + (long long)colc * K;
  const int nsteps = (K + 15) >> 4;
  const int s0 = (nsteps * w) / WAVES, s1 = (nsteps * (w + 1)) / WAVES;

  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int sb = s0; sb < s1; sb += CH) {
    float a[CH][4], b[CH][4];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int k = (sb + i) * 16 + 4 * g;
      const int kc = min(k, K - 4);
      load4<XT>(src, prow, kc, a[i]);
      const float4 wv = *reinterpret_cast<const float4*>(wrow + kc);
      b[i][0] = wv.x; b[i][1] = wv.y; b[i][2] = wv.z; b[i][3] = wv.w;
    }
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const bool kv = ((sb + i) * 16 + 4 * g) < K;
#pragma unroll
      for (int j = 0; j < 4; ++j) a[i][j] = kv ? a[i][j] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (sb + i < s1) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = mfma_16x16x4(a[i][j], b[i][j], acc);
      }
    }
  }

  __shared__ float red[WAVES][16][17];
#pragma unroll
  for (int r = 0; r < 4; ++r) red[w][4 * g + r][c] = acc[r];
  __syncthreads();
  for (int t = threadIdx.x; t < 256; t += WAVES * 64) {
    const int rr = t >> 4, cc = t & 15;
    const int gm = m0 + rr, gn = n0 + cc;
    if (gm < M && gn < N) {
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) v += red[ww][rr][cc];
      v += bv;  // thread t's prefetched bias[n0 + (t & 15)] == bias[gn]
      if (act == 1) v = fmaxf(v, 0.f);
      if (keep_thr != 0xFFFFFFFFu) {
        const uint32_t h = hash4(seed, step, (uint32_t)gm, (uint32_t)gn);
        v = (h < keep_thr) ? v * inv_keep : 0.f;
      }
      Y[(long long)gm * N + gn] = v;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// xent_head: one wave per batch row, 4 rows per workgroup; W2 [C][D] staged in LDS by float4
// loads that are all in flight at once (one round trip), concurrently with the row's H loads and
// the label gather chain.
//   logits = h·W2ᵀ + b2; loss = lse - logit[y]; dlogits = (softmax - onehot) * loss_scale
//   dZ[j] = (Σ_c dlogits[c]·W2[c][j]) * (h[j] > 0 ? inv_keep : 0)      (ReLU + dropout backward)
// Loss/correct go (one atomic per row) into slot (*hist_step % hist_len); block 0 zeroes the NEXT
// slot, so a graph-replayed loop keeps a ring of per-step metrics on the device.
// ---------------------------------------------------------------------------------------------
constexpr int kHeadMaxT = 16;  // hidden <= 1024
constexpr int kHeadMaxC = 16;  // classes <= 16
constexpr int kHeadStage = 16; // max float4 staging loads per thread (D*C <= 16384)

// CB/TB: compile-time bounds on classes and hidden/64 so the inner loops are straight-line code
// (runtime C/D guards become selects on clamped LDS addresses, not branches).
template <int LT, int STAGE, int CB, int TB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 4))) void xent_head_kernel(
    const float* __restrict__ H, int M, int D, const float* __restrict__ W2,
    const float* __restrict__ b2, int C, ArenaRowSource lab, float* __restrict__ dlogits,
    float* __restrict__ dZ, float inv_keep, int relu_mask, float loss_scale,
    float* __restrict__ loss_acc, int* __restrict__ correct_acc, int hist_len,
    const long long* hist_step, ArenaCounterOp ctr) {
  extern __shared__ __attribute__((aligned(16))) float ws[];  // [C][D] + one dummy float4
  const int lane = lane_id();
  const int r = blockIdx.x * 4 + wave_id();
  const int rc = min(r, M - 1);
  // (1) issue every independent global load up front
  const long long pr = gather_row(make_gather(lab), rc);
  int y;
  if constexpr (LT == 1) y = (int)static_cast<const uint8_t*>(lab.ptr)[pr];
  else if constexpr (LT == 2) y = static_cast<const int*>(lab.ptr)[pr];
  else y = (int)static_cast<const long long*>(lab.ptr)[pr];
  float h[TB];
#pragma unroll
  for (int t = 0; t < TB; ++t) h[t] = H[(long long)rc * D + min(lane + 64 * t, D - 1)];
  const int n4 = (D * C) >> 2;  // host guarantees (D*C) % 4 == 0
  float4 st[STAGE];
#pragma unroll
  for (int i = 0; i < STAGE; ++i)
    st[i] = reinterpret_cast<const float4*>(W2)[min((int)threadIdx.x + 256 * i, n4 - 1)];
  // b2: one vector load (lane cc holds b2[cc]); broadcast later with readlane (no scalar chain)
  const float bl = b2 ? b2[min(lane, C - 1)] : 0.f;
  const long long hs = hist_step ? *hist_step : 0;
  // (2) stage W2; unconditional stores (out-of-range items go to the dummy slot ws[4*n4]): a
  //     store guarded by a branch lets hipcc sink each load into it and wait there, serialising.
#pragma unroll
  for (int i = 0; i < STAGE; ++i) {
    const int q = threadIdx.x + 256 * i;
    reinterpret_cast<float4*>(ws)[q < n4 ? q : n4] = st[i];
  }
  counter_op(ctr);
  const int hmask = hist_len - 1;  // hist_len is a power of two (host-checked)
  const int slot = (int)hs & hmask;
  if (hist_len > 1 && blockIdx.x == 0 && threadIdx.x == 0) {
    const int nxt = (int)(hs + 1) & hmask;
    loss_acc[nxt] = 0.f;
    correct_acc[nxt] = 0;
  }
  __syncthreads();
  if (r >= M) return;
  int jo[TB];  // clamped LDS column per t; h zeroed past D
#pragma unroll
  for (int t = 0; t < TB; ++t) {
    const int j = lane + 64 * t;
    jo[t] = min(j, D - 1);
    h[t] = (j < D) ? h[t] : 0.f;
  }

  // (3) logits: per-lane partial dot products, then 64-lane reductions (independent chains)
  float lg[CB];
#pragma unroll
  for (int cc = 0; cc < CB; ++cc) {
    const float* wr = ws + min(cc, C - 1) * D;
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < TB; ++t) s += h[t] * wr[jo[t]];
    lg[cc] = s;
  }
#pragma unroll
  for (int cc = 0; cc < CB; ++cc) {  // all CB reductions unconditional -> interleaved DPP chains
    const float tot = wave_sum_fast(lg[cc]) +
                      __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bl), cc));
    lg[cc] = (cc < C) ? tot : -INFINITY;
  }
  float mx = lg[0];
  int arg = 0;
#pragma unroll
  for (int cc = 1; cc < CB; ++cc) {
    const bool gt = lg[cc] > mx;
    mx = gt ? lg[cc] : mx;
    arg = gt ? cc : arg;
  }
  float se = 0.f;
#pragma unroll
  for (int cc = 0; cc < CB; ++cc) se += (cc < C) ? hw_exp2((lg[cc] - mx) * kLog2e) : 0.f;
  const float lse = mx + hw_log2(se) * kLn2;
  float ly = 0.f;
#pragma unroll
  for (int cc = 0; cc < CB; ++cc) ly = (cc == y) ? lg[cc] : ly;
  if (lane == 0) {
    atomicAdd(&loss_acc[slot], (lse - ly) * loss_scale);
    atomicAdd(&correct_acc[slot], arg == y ? 1 : 0);
  }
  if (dlogits == nullptr) return;

  float gcl[CB];
#pragma unroll
  for (int cc = 0; cc < CB; ++cc)
    gcl[cc] = (cc < C) ? (hw_exp2((lg[cc] - lse) * kLog2e) - (cc == y ? 1.f : 0.f)) * loss_scale
                       : 0.f;
  if (lane < C) {
    float v = 0.f;
#pragma unroll
    for (int cc = 0; cc < CB; ++cc) v = (cc == lane) ? gcl[cc] : v;
    dlogits[(long long)r * C + lane] = v;
  }
  if (dZ == nullptr) return;
  float o[TB];
#pragma unroll
  for (int t = 0; t < TB; ++t) {
    float s = 0.f;
#pragma unroll
    for (int cc = 0; cc < CB; ++cc) s += gcl[cc] * ws[min(cc, C - 1) * D + jo[t]];
    o[t] = relu_mask ? ((h[t] > 0.f) ? s * inv_keep : 0.f) : s;
  }
#pragma unroll
  for (int t = 0; t < TB; ++t) {
    const int j = lane + 64 * t;
    if (j < D) dZ[(long long)r * D + j] = o[t];
  }
}

// ---------------------------------------------------------------------------------------------
// wgrad_grouped: dW[N][K] = dZᵀ·X (+ db = dZᵀ·1) for up to kMaxProblems layers in one launch.
// Workgroup = 4 waves = a 16(n) x 64(k) tile of dW. Per 128-row chunk: (1) the gathered row ids
// go to LDS (one dependent chain per row, once), (2) the X block [m][64] and the dZ slice [m][16]
// are staged through LDS with every load of the block in flight at once, (3) 4 waves run the MFMA
// K-loop over m. The Adam state of the tile is prefetched at kernel entry so its latency hides
// under the staging.
//   A operand (dZᵀ): lane l -> Zs[m = 4s + (l>>4)][n = l&15]         (stride 16: conflict-free)
//   B operand (X)  : lane l -> Xs[m = 4s + (l>>4)][k = 16w + (l&15)] (stride 80 ≡ 16 mod 32 banks:
//                    the two 16-lane groups of each half-wave hit disjoint banks)
//   D              : lane l, reg r -> dW[n0 + 4(l>>4) + r][k0 + 16w + (l&15)]   (coalesced rows)
// ---------------------------------------------------------------------------------------------
constexpr int kMaxProblems = 2;  // kernarg stays small (launch latency)
struct WGradArgs {
  ArenaWGradProblem p[kMaxProblems];
  int nprob;
  ArenaAdam adam;
  float grad_scale;  // mode 0
  ArenaCounterOp ctr;
  ArenaHead head;    // used by problems with hd_mode != 0
  int head_block;    // first block of the first head-mode problem: zeroes + records metrics
};

constexpr int kMC = 128;       // rows per LDS chunk
constexpr int kXsStride = 80;  // floats
constexpr int kXItems = (kMC * 16) / 256;  // X staging items per thread (16 per row)
constexpr int kZItems = (kMC * 4) / 256;   // dZ staging items per thread (4 float4 per row)
constexpr int kDItems = (kMC * 16) / 256;  // head logits items per thread ([m][16])

// Raw workgroup barrier for LDS hand-offs: waits only for this wave's LDS ops (lgkmcnt), NOT for
// its outstanding global loads (__syncthreads() would emit vmcnt(0) and drain the prefetches).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int XT>
__device__ __forceinline__ void load_x_items(const ArenaWGradProblem& P, const Gather& gt, int mc0,
                                             int mcn, int k0, float4 (&v)[kXItems]) {
  // 16 items per row, item q = 4 consecutive k (one u32 of u8 pixels or one float4). Rows past
  // mcn re-read row mcn-1 (finite data; their A operand is zeroed in the K-loop).
  int prow[kXItems];
#pragma unroll
  for (int i = 0; i < kXItems; ++i) {
    const int t = threadIdx.x + 256 * i;
    prow[i] = gather_row(gt, mc0 + min(t >> 4, mcn - 1));
  }
#pragma unroll
  for (int i = 0; i < kXItems; ++i) {
    const int q = (threadIdx.x + 256 * i) & 15;
    float f[4];
    load4<XT>(P.x, prow[i], min(k0 + 4 * q, P.K - 4), f);
    v[i] = make_float4(f[0], f[1], f[2], f[3]);
  }
}

__device__ __forceinline__ int load_label(const ArenaRowSource& lab, long long pr) {
  if (lab.dtype == 1) return (int)static_cast<const uint8_t*>(lab.ptr)[pr];
  if (lab.dtype == 2) return static_cast<const int*>(lab.ptr)[pr];
  return (int)static_cast<const long long*>(lab.ptr)[pr];
}

// ---------------------------------------------------------------------------------------------
// wgrad_grouped: dW[N][K] = dZᵀ·X (+ db = dZᵀ·1) for up to kMaxProblems layers in one launch.
// Workgroup = 4 waves = a 16(n) x 64(k) tile of dW. Per 128-row chunk: (1) every global load of the
// chunk is issued at once (gathered X block, dZ slice -- or the softmax head's raw logits, labels
// and the W2/H slices dZ is derived from -- then the tile's Adam state), (2) LDS images, (3) in
// head mode each workgroup recomputes softmax-xent for the chunk's rows (cheap, removes a kernel)
// and derives dZ, (4) 4 waves run the MFMA K-loop over m; the Adam update is the epilogue.
//   A operand (dZᵀ): lane l -> Zs[m = 4s + (l>>4)][n = l&15]         (stride 16: conflict-free)
//   B operand (X)  : lane l -> Xs[m = 4s + (l>>4)][k = 16w + (l&15)] (stride 80 ≡ 16 mod 32 banks:
//                    the two 16-lane groups of each half-wave hit disjoint banks)
//   D              : lane l, reg r -> dW[n0 + 4(l>>4) + r][k0 + 16w + (l&15)]   (coalesced rows)
// >= 2 waves/SIMD so all 424 workgroups x 4 waves are co-resident in ONE round on 1024 SIMDs.
// ---------------------------------------------------------------------------------------------
// Per-problem compile-time specialisation. SPEC == 0: every property of the problem is read at run
// time (generic path). Otherwise SPEC - 1 = xt | hd_mode << 1 | gather << 3 | mode << 4 |
// static_parity << 5 (the head's logits buffer index comes from the launch, not the counter), so hipcc
// sees straight-line code: no branch around a load, and every independent global load of the
// chunk is issued before the first wait (measured with scripts/timeline.py: the generic path
// drained vmcnt between the label, index, row and step loads).
template <int SPEC>
struct WSpec {
  static constexpr bool known = SPEC != 0;
  static constexpr int s = SPEC - 1;
  static constexpr int xt = s & 1, hm = (s >> 1) & 3, gather = (s >> 3) & 1, mode = (s >> 4) & 1;
  static constexpr bool sp = known && ((s >> 5) & 1);
};


constexpr int wgrad_spec(int xt, int hm, int gather, int mode, int sp = 0) {
  return 1 + xt + 2 * hm + 8 * gather + 16 * mode + 32 * sp;
}

template <int CB, int SPEC, int LG, int LDT>  // CB: bound on head classes (C <= CB); LG: labels
                                              // gathered, LDT: label dtype (-1: run time)
// (LDS images come in as plain pointers: __restrict__ here would let hipcc move LDS accesses
// across the raw s_barrier in lds_barrier(), whose memory clobber noalias memory escapes)
__device__ __forceinline__ void wgrad_body(const WGradArgs& args, int pi, float* Xs, float* Zs,
                                           float* Ds, float* W2s, int* Ys, float* B2s) {
  using WS = WSpec<SPEC>;
  const ArenaWGradProblem& P = args.p[pi];
  const ArenaHead& HD = args.head;
  const int local = blockIdx.x - P.block_begin;
  // XCD-aware tile order: workgroups are dealt to the 8 XCDs round-robin by linear block id, and
  // the forward kernel's n-tile x runs on XCD x % 8. Giving this problem's n-tile tn to a block
  // with blockIdx % 8 == tn % 8 keeps each 16-row slice of W (written here by Adam, read next by
  // the forward) and of H / the W2 snapshot (written by the forward, read here) inside one XCD's L2.
  int tn, tk;
  if ((P.tiles_n & 7) == 0 && (P.block_begin & 7) == 0) {
    const int xcd = local & 7, slot = local >> 3;
    tn = xcd + 8 * (slot / P.tiles_k);
    tk = slot % P.tiles_k;
  } else {
    tn = local / P.tiles_k;
    tk = local % P.tiles_k;
  }
  const int n0 = tn * 16, k0 = tk * 64;
  const int lane = lane_id(), w = wave_id();
  const int g = lane >> 4, c = lane & 15;
  const int kk = k0 + 16 * w + c;
  const int kkc = min(kk, P.K - 1);
  const bool bias_wave = (tk == 0) && (w == 0);
  const int mode = WS::known ? WS::mode : P.mode;
  const int xt = WS::known ? WS::xt : P.xt;
  const int hmode = WS::known ? WS::hm : P.hd_mode;
  const bool has_bias = mode == 1 ? P.pB != nullptr : P.gB != nullptr;
  const Gather gt = (WS::known && !WS::gather) ? Gather{nullptr, 0, P.M} : make_gather(P.x);
  const bool zvec = (P.N & 3) == 0;
  ARENA_TL(1, 0);
  // step counter and Adam scalars: loads issued now, first used after the chunk's other loads
  // are in flight (in-order vmcnt: waiting on these oldest loads leaves the younger ones going)
  // Loaded now, first used after every other load of the chunk is issued. Two hipcc habits are
  // defeated here: (1) a load under a branch is drained at the branch, so the spec path loads
  // unconditionally (the host guarantees the pointers); (2) a uniform loaded value is moved into an
  // SGPR (v_readfirstlane) right after its load, draining vmcnt at once, so the values are made
  // lane-varying by adding a lane-dependent zero the compiler cannot see through.
  int lz;  // an opaque zero in a VGPR (hipcc cannot fold it or prove the sums below uniform)
  asm volatile("v_mov_b32 %0, 0" : "=v"(lz));
  long long hstep_raw = 0, adam_t = 1;
  float adam_lr = args.adam.lr;
  if constexpr (WS::known) {
    // 32-bit loads of the counters' low words (< 2^31 steps): a 64-bit destination whose dead
    // high half is reused would force an early wait (register write-after-read on the load)
    if (WS::hm) hstep_raw = *reinterpret_cast<const int*>(HD.step) + lz;
    if (WS::mode == 1) {
      adam_t = *reinterpret_cast<const int*>(args.adam.t_ptr) + lz;
      adam_lr = *args.adam.lr_ptr + __int_as_float(lz);
    }
  } else {
    if (hmode) hstep_raw = *HD.step;
    if (mode == 1) {
      adam_t = args.adam.t_ptr ? *args.adam.t_ptr : 1;
      adam_lr = args.adam.lr_ptr ? *args.adam.lr_ptr : args.adam.lr;
    }
  }
  const float* logits = nullptr;
  long long hstep = 0;

  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  f32x4 accb = {0.f, 0.f, 0.f, 0.f};
  float pw[4], mw[4], vw[4], pb[4], mb[4], vb[4];
  // spec path: the host guarantees M <= kMC, so the chunk loop (and every mc0 == 0 test) folds away
  const int nchunks = WS::known ? 1 : (P.M + kMC - 1) / kMC;
  for (int ci = 0; ci < nchunks; ++ci) {
    const int mc0 = ci * kMC;
    const int mcn = min(kMC, P.M - mc0);
    // (1) issue the chunk's loads
    float4 xv[kXItems];
    if (ARENA_EXP & 2) {
#pragma unroll
      for (int i = 0; i < kXItems; ++i) xv[i] = make_float4(0.5f, 0.25f, 0.f, 1.f);
    } else if (xt == 1) {
      load_x_items<1>(P, gt, mc0, mcn, k0, xv);
    } else {
      load_x_items<0>(P, gt, mc0, mcn, k0, xv);
    }
    ARENA_TL(1, 8);
    float4 zv[kZItems];
    float dv[kDItems];
    float wv = 0.f, bv = 0.f;
    int yv = 0;
    if (hmode == 0) {
#pragma unroll
      for (int i = 0; i < kZItems; ++i) {
        const int t = threadIdx.x + 256 * i;
        const int rr = min(t >> 2, mcn - 1), q = t & 3;
        const int n = n0 + 4 * q;
        const float* srcp = P.dz + (long long)(mc0 + rr) * P.N;
        if (zvec) {
          zv[i] = *reinterpret_cast<const float4*>(srcp + min(n, P.N - 4));
        } else {
          zv[i] = make_float4(srcp[min(n, P.N - 1)], srcp[min(n + 1, P.N - 1)],
                              srcp[min(n + 2, P.N - 1)], srcp[min(n + 3, P.N - 1)]);
        }
      }
    } else {
      const int C = HD.C;
      if ((int)threadIdx.x < kMC) {
        // labels share the layer input's gather (same rows); no gather -> direct
        const Gather lg = (LG == 0) ? Gather{nullptr, 0, P.M} : make_gather(HD.lab);
        const long long pr = gather_row(lg, mc0 + min((int)threadIdx.x, mcn - 1));
        if constexpr (LDT == 1) yv = static_cast<const uint8_t*>(HD.lab.ptr)[pr];
        else if constexpr (LDT == 2) yv = static_cast<const int*>(HD.lab.ptr)[pr];
        else yv = load_label(HD.lab, pr);
      }
      {
        const float* b2p = HD.b2 ? HD.b2 : P.hd_w2 ? P.hd_w2 : HD.logits2;  // any valid address
        const float b2v = b2p[min((int)threadIdx.x & 15, C - 1)];
        bv = HD.b2 ? b2v : 0.f;
      }
      if (hmode == 2) {
#pragma unroll
        for (int i = 0; i < kZItems; ++i) {  // mask source (post-dropout activation)
          const int t = threadIdx.x + 256 * i;
          const int rr = min(t >> 2, mcn - 1), q = t & 3;
          if (ARENA_EXP & 4) zv[i] = make_float4(1.f, 0.f, 1.f, 1.f);
          else zv[i] = *reinterpret_cast<const float4*>(P.hd_h + (long long)(mc0 + rr) * P.N +
                                                        min(n0 + 4 * q, P.N - 4));
        }
        wv = P.hd_w2[(long long)min((int)threadIdx.x >> 4, C - 1) * P.N +
                     min(n0 + ((int)threadIdx.x & 15), P.N - 1)];
      }
      ARENA_TL(1, 9);
      if (mc0 == 0) {
        if constexpr (WS::sp) {
          // buffer index known at launch: the logits loads go out now and the step counter is
          // first waited for where the metric slot / next-step bookkeeping needs it
          logits = HD.logits2 + (long long)HD.parity * P.M * HD.C;
          ARENA_TL(1, 1);
        } else {  // first use of the step counter: every other load of the chunk is issued
          if (ARENA_EXP & 16) hstep_raw = 7;
          hstep = hstep_raw + HD.step_off;
          logits = HD.logits2 + (long long)(hstep & 1) * P.M * HD.C;
          ARENA_TL_DEP((int)hstep);
          ARENA_TL(1, 1);
        }
      }
#pragma unroll
      for (int i = 0; i < kDItems; ++i) {  // raw logits rows: item t -> (m = t>>4, c = t&15)
        const int t = threadIdx.x + 256 * i;
        if (ARENA_EXP & 1) dv[i] = 0.01f * (float)(t & 15);
        else dv[i] = logits[(long long)(mc0 + min(t >> 4, mcn - 1)) * C + min(t & 15, C - 1)];
      }
      ARENA_TL(1, 10);
      if (mc0 == 0 && (int)blockIdx.x == args.head_block) {  // zero the other buffer + next slot
        if constexpr (WS::sp) hstep = hstep_raw + HD.step_off;  // this block only waits here
        float* nxt = HD.logits2 + (long long)((hstep + 1) & 1) * P.M * HD.C;
        for (int i = threadIdx.x; i < P.M * HD.C; i += 256) nxt[i] = 0.f;
        if (HD.nr_out != nullptr && (int)threadIdx.x < HD.nr_batch) {
          long long q = mod_fp64((double)(hstep + 1) * (double)HD.nr_batch, HD.nr_len) +
                        (long long)threadIdx.x;
          q = (q >= HD.nr_len) ? q - HD.nr_len : q;
          HD.nr_out[threadIdx.x] = HD.nr_perm[q];
        }
        if (threadIdx.x == 0 && HD.hist_len > 1) {
          const int ns = (int)(hstep + 1) & (HD.hist_len - 1);
          HD.loss_acc[ns] = 0.f;
          HD.correct_acc[ns] = 0;
        }
      }
    }
    // (2) on the first chunk, prefetch the tile's Adam state behind them (in-order vmcnt lets the
    //     staging waits below leave these in flight through the K-loop)
    if (mc0 == 0 && mode == 1 && (ARENA_EXP & 32)) {  // ablation: no Adam state loads
#pragma unroll
      for (int r = 0; r < 4; ++r) { pw[r] = 0.1f; mw[r] = 0.01f; vw[r] = 0.001f; }
#pragma unroll
      for (int r = 0; r < 4; ++r) { pb[r] = 0.1f; mb[r] = 0.01f; vb[r] = 0.001f; }
    } else if (mc0 == 0 && mode == 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long long off = (long long)min(n0 + 4 * g + r, P.N - 1) * P.K + kkc;
        pw[r] = P.pW[off]; mw[r] = P.mW[off]; vw[r] = P.vW[off];
      }
      {  // every wave loads (a branch around loads drains vmcnt); only the bias wave uses them
        const float* pbp = has_bias ? P.pB : P.pW;
        const float* mbp = has_bias ? P.mB : P.mW;
        const float* vbp = has_bias ? P.vB : P.vW;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = min(n0 + 4 * g + r, P.N - 1);
          pb[r] = pbp[n]; mb[r] = mbp[n]; vb[r] = vbp[n];
        }
      }
    }
    // (3) LDS images; every store unconditional (no branch for hipcc to sink a load into)
#pragma unroll
    for (int i = 0; i < kXItems; ++i) {
      const int t = threadIdx.x + 256 * i;
      const int rr = t >> 4, q = t & 15;
      const float4 o = (k0 + 4 * q < P.K) ? xv[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(&Xs[rr * kXsStride + 4 * q]) = o;
    }
    if (hmode == 0) {
#pragma unroll
      for (int i = 0; i < kZItems; ++i) {
        const int t = threadIdx.x + 256 * i;
        const int rr = t >> 2, q = t & 3;
        const int n = n0 + 4 * q;
        float4 o = zv[i];
        o.x = (n + 0 < P.N) ? o.x : 0.f;
        o.y = (n + 1 < P.N) ? o.y : 0.f;
        o.z = (n + 2 < P.N) ? o.z : 0.f;
        o.w = (n + 3 < P.N) ? o.w : 0.f;
        if (rr >= mcn) o = make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4*>(&Zs[rr * 16 + 4 * q]) = o;
      }
    } else {
      const int C = HD.C;
#pragma unroll
      for (int i = 0; i < kDItems; ++i) Ds[threadIdx.x + 256 * i] = dv[i];
      if ((int)threadIdx.x < kMC) Ys[threadIdx.x] = yv;
      if (threadIdx.x < 16) B2s[threadIdx.x] = bv;
      W2s[threadIdx.x] = (((int)threadIdx.x >> 4) < C) ? wv : 0.f;
      lds_barrier();
      ARENA_TL(1, 2);
      // softmax-xent per row (thread = row): Ds row -> dlogits; block 0 also records metrics
      float loss = 0.f, corr = 0.f;
      if ((int)threadIdx.x < mcn) {
        float* row = &Ds[threadIdx.x * 16];
        const int y = Ys[threadIdx.x];
        float lgv[CB];
        float mx = -INFINITY;
        int arg = 0;
#pragma unroll
        for (int cc = 0; cc < CB; ++cc) {
          lgv[cc] = row[cc] + B2s[cc];
          const bool better = cc < C && lgv[cc] > mx;
          mx = better ? lgv[cc] : mx;
          arg = better ? cc : arg;
        }
        float pe[CB];
        float se = 0.f;
#pragma unroll
        for (int cc = 0; cc < CB; ++cc) {
          pe[cc] = (cc < C) ? hw_exp2((lgv[cc] - mx) * kLog2e) : 0.f;  // x <= 0: no overflow
          se += pe[cc];
        }
        const float inv = hw_rcp(se);                  // se >= 1 (the max term is exp(0))
        const float lse = mx + hw_log2(se) * kLn2;
        float ly = 0.f;
#pragma unroll
        for (int cc = 0; cc < CB; ++cc) {
          ly = (cc == y) ? lgv[cc] : ly;
          row[cc] = (pe[cc] * inv - (cc == y ? 1.f : 0.f)) * HD.loss_scale;
        }
        loss = (lse - ly) * HD.loss_scale;
        corr = (arg == y) ? 1.f : 0.f;
      }
      if ((int)blockIdx.x == args.head_block) {
        const float ls = wave_sum_fast(loss), cs = wave_sum_fast(corr);
        if (lane == 0 && w * 64 < mcn) {
          const int slot = (int)hstep & (HD.hist_len - 1);
          atomicAdd(&HD.loss_acc[slot], ls);
          atomicAdd(&HD.correct_acc[slot], (int)(cs + 0.5f));
        }
      }
      lds_barrier();
      ARENA_TL(1, 3);
      // derive dZ for this tile into the Zs image
#pragma unroll
      for (int i = 0; i < kZItems; ++i) {
        const int t = threadIdx.x + 256 * i;
        const int rr = t >> 2, q = t & 3;
        const int n = n0 + 4 * q;
        float z[4];
        if (hmode == 1) {  // output layer: dz = dlogits (N == C <= 16, single n tile)
          const float4 d4 = *reinterpret_cast<const float4*>(&Ds[rr * 16 + 4 * q]);
          z[0] = d4.x; z[1] = d4.y; z[2] = d4.z; z[3] = d4.w;
        } else {           // hidden layer: dz = (dlogits · W2) ⊙ (h > 0) / keep
          z[0] = z[1] = z[2] = z[3] = 0.f;
#pragma unroll
          for (int cc = 0; cc < CB; ++cc) {
            const float d = Ds[rr * 16 + cc];
            const float4 w4 = *reinterpret_cast<const float4*>(&W2s[cc * 16 + 4 * q]);
            z[0] += d * w4.x; z[1] += d * w4.y; z[2] += d * w4.z; z[3] += d * w4.w;
          }
          const float4 hm = zv[i];
          const float ik = P.hd_inv_keep;
          z[0] = hm.x > 0.f ? z[0] * ik : 0.f;
          z[1] = hm.y > 0.f ? z[1] * ik : 0.f;
          z[2] = hm.z > 0.f ? z[2] * ik : 0.f;
          z[3] = hm.w > 0.f ? z[3] * ik : 0.f;
        }
        float4 o = make_float4((n + 0 < P.N) ? z[0] : 0.f, (n + 1 < P.N) ? z[1] : 0.f,
                               (n + 2 < P.N) ? z[2] : 0.f, (n + 3 < P.N) ? z[3] : 0.f);
        if (rr >= mcn) o = make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4*>(&Zs[rr * 16 + 4 * q]) = o;
      }
    }
    lds_barrier();
    ARENA_TL(1, 4);
    // (4) K-loop over all kMC rows of the image (rows >= mcn: Zs zero, Xs finite). Four
    //     independent accumulator chains (the f32 MFMA's dependent latency is 40 cycles, its
    //     issue 8): a quarter of the serial depth. Bias columns (db = dZᵀ·1) run in the same
    //     loop in the k-tile-0 blocks only (a block-uniform branch outside the loop).
    if (mcn > kMC / 2) {
      f32x4 ch[4] = {acc, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      if (tk == 0) {
        f32x4 chb[4] = {accb, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int s = 0; s < kMC / 4; s += 4) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int m = 4 * (s + j) + g;
            const float a = Zs[m * 16 + c];
            const float b = Xs[m * kXsStride + 16 * w + c];
            ch[j] = mfma_16x16x4(a, b, ch[j]);
            chb[j] = mfma_16x16x4(a, 1.f, chb[j]);
          }
        }
        accb = (chb[0] + chb[1]) + (chb[2] + chb[3]);
      } else {
#pragma unroll
        for (int s = 0; s < kMC / 4; s += 4) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int m = 4 * (s + j) + g;
            const float a = Zs[m * 16 + c];
            const float b = Xs[m * kXsStride + 16 * w + c];
            ch[j] = mfma_16x16x4(a, b, ch[j]);
          }
        }
      }
      acc = (ch[0] + ch[1]) + (ch[2] + ch[3]);
    } else {
      const int nst = (mcn + 3) >> 2;
      for (int s = 0; s < nst; ++s) {
        const int m = 4 * s + g;
        const float a = Zs[m * 16 + c];
        const float b = Xs[m * kXsStride + 16 * w + c];
        acc = mfma_16x16x4(a, b, acc);
        if (bias_wave) accb = mfma_16x16x4(a, 1.f, accb);
      }
    }
    if (ci + 1 < nchunks) lds_barrier();  // before the next chunk overwrites the images
  }
  ARENA_TL_DEP(acc[0]);
  ARENA_TL(1, 5);
  AdamCoef co{};
  if (mode == 1) co = adam_coef_tl(args.adam, (float)adam_t, adam_lr);

  if (mode == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + 4 * g + r;
      if (kk < P.K && n < P.N) P.gW[(long long)n * P.K + kk] = acc[r] * args.grad_scale;
    }
    if (bias_wave && has_bias && c == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + 4 * g + r;
        if (n < P.N) P.gB[n] = accb[r] * args.grad_scale;
      }
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + 4 * g + r;
      if (kk < P.K && n < P.N) {
        const long long off = (long long)n * P.K + kk;
        adam_apply(co, acc[r], pw[r], mw[r], vw[r]);
        P.pW[off] = pw[r]; P.mW[off] = mw[r]; P.vW[off] = vw[r];
      }
    }
    if (bias_wave && has_bias && c == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + 4 * g + r;
        if (n < P.N) {
          adam_apply(co, accb[r], pb[r], mb[r], vb[r]);
          P.pB[n] = pb[r]; P.mB[n] = mb[r]; P.vB[n] = vb[r];
        }
      }
    }
  }
  ARENA_TL(1, 6);
  ARENA_TL_DRAIN();
  ARENA_TL(1, 7);
}

// S0 / S1: specs of problems 0 / 1 (both nonzero = the fused MLP step's fixed pair; 0 = generic).
template <int CB, int S0, int S1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 4))) void wgrad_grouped_kernel(
    WGradArgs args) {
  __shared__ __attribute__((aligned(16))) float Xs[kMC * kXsStride];
  __shared__ __attribute__((aligned(16))) float Zs[kMC * 16];
  __shared__ __attribute__((aligned(16))) float Ds[kMC * 16];  // head: logits -> dlogits [m][c]
  __shared__ __attribute__((aligned(16))) float W2s[16 * 16];  // head: W2 slice [c][n]
  __shared__ int Ys[kMC];                                      // head: labels
  __shared__ float B2s[16];
  int pi = 0;
#pragma unroll
  for (int i = 1; i < kMaxProblems; ++i)
    if (i < args.nprob && (int)blockIdx.x >= args.p[i].block_begin) pi = i;
  if constexpr (S0 != 0 && S1 != 0) {
    // the head's labels follow problem 0's gather (the binding shares it with the label source)
    // (published batch: int32 labels; dataset gather: the dataset's uint8 labels)
    constexpr int LG = WSpec<S0>::gather;
    constexpr int LDT = LG ? 1 : 2;
    if (pi == 0) wgrad_body<CB, S0, LG, LDT>(args, 0, Xs, Zs, Ds, W2s, Ys, B2s);
    else wgrad_body<CB, S1, LG, LDT>(args, 1, Xs, Zs, Ds, W2s, Ys, B2s);
  } else {
    wgrad_body<CB, 0, -1, -1>(args, pi, Xs, Zs, Ds, W2s, Ys, B2s);
  }
  counter_op(args.ctr);  // A = B last: nothing in this kernel reads A
}


// ---------------------------------------------------------------------------------------------
// mlp_fwd_logits: linear_fwd of the hidden layer (bias, ReLU, dropout) that also emits the
// output layer's logits: each (m, n) tile multiplies its 16x16 H tile by the matching 16-column
// slice of W2 and atomically adds the 16 x C partial into logits2[step&1] (no-return f32 atomics;
// 32 hidden tiles per logit, so the sum order -- and the last bit -- may vary run to run). The
// m-tile-0 workgroups also snapshot W2 for the backward pass (which updates W2 in place). The
// softmax itself is recomputed by every wgrad workgroup: no intra-kernel hand-off anywhere.
// ---------------------------------------------------------------------------------------------
// FM: 0 = generic; 1 = training-step fast path gathering rows from the step counter; 2 = fast
// path reading this step's rows precomputed by the previous backward kernel.
template <int XT, int WAVES, int FM>
__global__ __launch_bounds__(WAVES * 64) void mlp_fwd_logits_kernel(
    ArenaRowSource src, const float* __restrict__ W, const float* __restrict__ bias,
    float* __restrict__ Y, int M, int N, int K, uint32_t keep_thr, float inv_keep, uint32_t seed,
    const long long* step_src, const float* __restrict__ W2, float* __restrict__ W2_copy, int C,
    float* __restrict__ logits2, uint8_t* __restrict__ xb, const void* __restrict__ lab_ptr,
    int lab_dtype, int* __restrict__ yb, ArenaCounterOp ctr, const int* __restrict__ rows) {
  constexpr int CH = 8;
  const int lane = lane_id(), w = wave_id();
  const int g = lane >> 4, c = lane & 15;
  const int n0 = blockIdx.x * 16, m0 = blockIdx.y * 16;
  ARENA_TL(0, 0);
  const int rowc = min(m0 + c, M - 1), colc = min(n0 + c, N - 1);
  const float* wrow = W + (long long)colc * K;
  const int nsteps = (K + 15) >> 4;
  const int s0 = (nsteps * w) / WAVES, s1 = (nsteps * (w + 1)) / WAVES;
  // n-tile-0 workgroups publish the step's gathered batch (u8 rows + labels) so the backward
  // kernel reads them directly instead of repeating the cursor -> index -> row chain
  const bool publish = (xb != nullptr) && blockIdx.x == 0;
  __shared__ float w2s[16][17];
  __shared__ float hs[16][17];
  __shared__ float red[WAVES][16][17];
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  long long stepv;
  long long prow;
  float w2v, bv;
  constexpr bool FAST = FM != 0;
  if constexpr (FAST) {
    // The fused training step (host-checked: cursor == step counter == counter-op source, one
    // K chunk per wave, gather on, publishing on). One straight load stream: the step counter
    // (oldest), then everything independent of it (this wave's W rows, the W2 slice, bias), then
    // the cursor -> index -> row chain, whose waits leave the W loads in flight. The counter is
    // kept lane-varying (opaque zero) so hipcc does not drain it into an SGPR at once, and the
    // label publication and the counter update move to the end.
    int lz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(lz));
    // FM 2: the row index is the oldest load, so waiting for it leaves the W loads in flight
    int prow2 = 0;
    if constexpr (FM == 2) prow2 = rows[rowc] + lz;
    const int A = *reinterpret_cast<const int*>(step_src) + lz;
    __builtin_amdgcn_sched_barrier(0);
    float b[CH][4];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int kc = min((s0 + i) * 16 + 4 * g, K - 4);
      const float4 wv = *reinterpret_cast<const float4*>(wrow + kc);
      b[i][0] = wv.x; b[i][1] = wv.y; b[i][2] = wv.z; b[i][3] = wv.w;
    }
    w2v = W2[(long long)min((int)(threadIdx.x >> 4) & 15, C - 1) * N +
             min(n0 + ((int)threadIdx.x & 15), N - 1)];
    bv = bias[min(n0 + ((int)threadIdx.x & 15), N - 1)];
    __builtin_amdgcn_sched_barrier(0);  // keep the independent loads above the counter's first use
    if constexpr (FM == 2) {  // this step's rows, precomputed by the previous backward kernel
      prow = prow2;
    } else {
      long long p = mod_fp64((double)A * (double)src.batch, src.idx_len) + rowc;
      p = (p >= src.idx_len) ? p - src.idx_len : p;
      prow = src.idx[p];
    }
    stepv = A;
    ARENA_TL_DEP((int)prow);
    ARENA_TL(0, 1);
    float a[CH][4];
    uint32_t raw[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int kc = min((s0 + i) * 16 + 4 * g, K - 4);
      if constexpr (XT == 1) {
        raw[i] = *reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(src.ptr) +
                                                    prow * (long long)src.ld + kc);
#pragma unroll
        for (int j = 0; j < 4; ++j) a[i][j] = (float)((raw[i] >> (8 * j)) & 0xffu) * src.scale;
      } else {
        load4<XT>(src, prow, kc, a[i]);
        raw[i] = 0;
      }
    }
    if constexpr (XT == 1) {
      if (publish && m0 + c < M) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int k = (s0 + i) * 16 + 4 * g;
          if (s0 + i < s1 && k < K)  // stores only: the branch holds no load
            *reinterpret_cast<uint32_t*>(xb + (long long)(m0 + c) * K + k) = raw[i];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < CH; ++i) {  // steps past this wave's range contribute zero (no branch)
      const bool kv = ((s0 + i) * 16 + 4 * g) < K && (s0 + i) < s1;
#pragma unroll
      for (int j = 0; j < 4; ++j) a[i][j] = kv ? a[i][j] : 0.f;
    }
    // four independent accumulator chains (40-cycle dependent MFMA latency, 8-cycle issue)
    f32x4 ch[4] = {acc, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int i = 0; i < CH; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) ch[j] = mfma_16x16x4(a[i][j], b[i][j], ch[j]);
    }
    acc = (ch[0] + ch[1]) + (ch[2] + ch[3]);
  } else {
  const Gather gt = make_gather(src);
  stepv = step_src ? *step_src : 0;
  prow = gather_row(gt, rowc);
  ARENA_TL_DEP((int)prow);
  ARENA_TL(0, 1);
  if (publish && w == 0 && g == 0 && m0 + c < M) {
    const int y = (lab_dtype == 1) ? (int)static_cast<const uint8_t*>(lab_ptr)[prow]
                : (lab_dtype == 2) ? static_cast<const int*>(lab_ptr)[prow]
                                   : (int)static_cast<const long long*>(lab_ptr)[prow];
    yb[m0 + c] = y;
  }
  w2v = 0.f;
  bv = 0.f;
  if (threadIdx.x < 256) {
    w2v = W2[(long long)min((int)threadIdx.x >> 4, C - 1) * N + min(n0 + ((int)threadIdx.x & 15), N - 1)];
    bv = bias[min(n0 + ((int)threadIdx.x & 15), N - 1)];
  }
  counter_op(ctr);

  for (int sb = s0; sb < s1; sb += CH) {
    float a[CH][4], b[CH][4];
    uint32_t raw[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int k = (sb + i) * 16 + 4 * g;
      const int kc = min(k, K - 4);
      if constexpr (XT == 1) {
        raw[i] = *reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(src.ptr) +
                                                    prow * (long long)src.ld + kc);
#pragma unroll
        for (int j = 0; j < 4; ++j) a[i][j] = (float)((raw[i] >> (8 * j)) & 0xffu) * src.scale;
      } else {
        load4<XT>(src, prow, kc, a[i]);
      }
      const float4 wv = *reinterpret_cast<const float4*>(wrow + kc);
      b[i][0] = wv.x; b[i][1] = wv.y; b[i][2] = wv.z; b[i][3] = wv.w;
    }
    if constexpr (XT == 1) {
      if (publish && m0 + c < M) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int k = (sb + i) * 16 + 4 * g;
          if (sb + i < s1 && k < K)  // stores only: the branch holds no load
            *reinterpret_cast<uint32_t*>(xb + (long long)(m0 + c) * K + k) = raw[i];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const bool kv = ((sb + i) * 16 + 4 * g) < K;
#pragma unroll
      for (int j = 0; j < 4; ++j) a[i][j] = kv ? a[i][j] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (sb + i < s1) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = mfma_16x16x4(a[i][j], b[i][j], acc);
      }
    }
  }
  }
  const uint32_t step = (uint32_t)stepv;
  ARENA_TL_DEP(acc[0]);
  ARENA_TL(0, 2);
#pragma unroll
  for (int r = 0; r < 4; ++r) red[w][4 * g + r][c] = acc[r];
  if (threadIdx.x < 256)
    w2s[threadIdx.x >> 4][threadIdx.x & 15] = ((int)(threadIdx.x >> 4) < C) ? w2v : 0.f;
  __syncthreads();
  ARENA_TL(0, 3);
  if (threadIdx.x < 256) {
    const int rr = threadIdx.x >> 4, cc = threadIdx.x & 15;
    const int gm = m0 + rr, gn = n0 + cc;
    float v = bv;
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) v += red[ww][rr][cc];
    v = fmaxf(v, 0.f);
    if (keep_thr != 0xFFFFFFFFu) {
      const uint32_t h = hash4(seed, step, (uint32_t)gm, (uint32_t)gn);
      v = (h < keep_thr) ? v * inv_keep : 0.f;
    }
    const bool ok = gm < M && gn < N;
    if (ok) Y[(long long)gm * N + gn] = v;
    hs[rr][cc] = ok ? v : 0.f;
    if (W2_copy != nullptr && blockIdx.y == 0 && rr < C && gn < N)
      W2_copy[(long long)rr * N + gn] = w2v;  // thread (rr, cc) holds W2[rr][n0 + cc]
  }
  __syncthreads();
  ARENA_TL(0, 4);
  float* lg = logits2 + (long long)(stepv & 1) * M * C;
  if ((int)threadIdx.x < 16 * C) {
    const int rr = threadIdx.x / C, cl = threadIdx.x % C;
    float p = 0.f;
#pragma unroll
    for (int n = 0; n < 16; ++n) p += hs[rr][n] * w2s[cl][n];
    if (ARENA_EXP & 8) {
      if (m0 + rr < M) lg[(long long)(m0 + rr) * C + cl] = p;
    } else {
      if (m0 + rr < M) atomicAdd(&lg[(long long)(m0 + rr) * C + cl], p);
    }
  }
  if constexpr (FAST) {
    if (publish && w == 0 && g == 0 && m0 + c < M) {
      const int y = (lab_dtype == 1) ? (int)static_cast<const uint8_t*>(lab_ptr)[prow]
                  : (lab_dtype == 2) ? static_cast<const int*>(lab_ptr)[prow]
                                     : (int)static_cast<const long long*>(lab_ptr)[prow];
      yb[m0 + c] = y;
    }
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *ctr.dst = stepv + ctr.add;
  }
  ARENA_TL(0, 5);
  ARENA_TL_DRAIN();
  ARENA_TL(0, 6);
}

// ---------------------------------------------------------------------------------------------
// adam_flat: float4-vectorised Adam over the flat parameter buffer; n must be a multiple of 4.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void adam_flat_kernel(float* __restrict__ P, float* __restrict__ Mm,
                                                        float* __restrict__ V,
                                                        const float* __restrict__ G, long long n4,
                                                        ArenaAdam a, ArenaCounterOp ctr) {
  counter_op(ctr);
  const AdamCoef co = adam_coef(a);
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    float4 p = reinterpret_cast<float4*>(P)[i];
    float4 m = reinterpret_cast<float4*>(Mm)[i];
    float4 v = reinterpret_cast<float4*>(V)[i];
    const float4 g = reinterpret_cast<const float4*>(G)[i];
    adam_apply(co, g.x, p.x, m.x, v.x);
    adam_apply(co, g.y, p.y, m.y, v.y);
    adam_apply(co, g.z, p.z, m.z, v.z);
    adam_apply(co, g.w, p.w, m.w, v.w);
    reinterpret_cast<float4*>(P)[i] = p;
    reinterpret_cast<float4*>(Mm)[i] = m;
    reinterpret_cast<float4*>(V)[i] = v;
  }
}

__global__ __launch_bounds__(256) void sgd_flat_kernel(float* __restrict__ P,
                                                       const float* __restrict__ G, long long n4,
                                                       float lr, const float* lr_ptr, float gscale) {
  const float l = lr_ptr ? *lr_ptr : lr;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    float4 p = reinterpret_cast<float4*>(P)[i];
    const float4 g = reinterpret_cast<const float4*>(G)[i];
    p.x -= l * g.x * gscale; p.y -= l * g.y * gscale; p.z -= l * g.z * gscale; p.w -= l * g.w * gscale;
    reinterpret_cast<float4*>(P)[i] = p;
  }
}

// ---------------------------------------------------------------------------------------------
// softmax_xent: generic rows (any C), one wave per row; writes per-row loss and dlogits.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void softmax_xent_kernel(const float* __restrict__ logits,
                                                           const long long* __restrict__ labels,
                                                           int M, int C, float* __restrict__ loss,
                                                           float* __restrict__ dlogits,
                                                           float grad_scale) {
  const int lane = lane_id();
  const int r = blockIdx.x * 4 + wave_id();
  if (r >= M) return;
  const float* x = logits + (long long)r * C;
  float mx = -INFINITY;
  for (int cc = lane; cc < C; cc += 64) mx = fmaxf(mx, x[cc]);
  mx = wave_max_fast(mx);
  float se = 0.f;
  for (int cc = lane; cc < C; cc += 64) se += hw_exp2((x[cc] - mx) * kLog2e);
  se = wave_sum_fast(se);
  const float lse = mx + hw_log2(se) * kLn2;
  const long long y = labels[r];
  if (lane == 0) loss[r] = lse - x[y];
  if (dlogits) {
    float* d = dlogits + (long long)r * C;
    for (int cc = lane; cc < C; cc += 64)
      d[cc] = (hw_exp2((x[cc] - lse) * kLog2e) - (cc == y ? 1.f : 0.f)) * grad_scale;
  }
}

// ---------------------------------------------------------------------------------------------
// mt_copy_scale: multi-tensor gather/scatter between a list of tensors and one flat bucket.
//   dir 0: flat[off_i + j] = src_i[j] * scale      (flatten gradients into the all-reduce bucket)
//   dir 1: dst_i[j] = flat[off_i + j] * scale      (unflatten reduced gradients)
// ---------------------------------------------------------------------------------------------
constexpr int kMtMax = 48;
struct MtArgs {
  float* ptr[kMtMax];
  long long off[kMtMax];
  long long n[kMtMax];
  int blk_begin[kMtMax + 1];
  int count;
};

__global__ __launch_bounds__(256) void mt_copy_scale_kernel(MtArgs a, float* __restrict__ flat,
                                                            float scale, int dir) {
  int ti = 0;
  for (int i = 1; i < a.count; ++i)
    if ((int)blockIdx.x >= a.blk_begin[i]) ti = i;
  const long long base = (long long)(blockIdx.x - a.blk_begin[ti]) * 1024;
  float* t = a.ptr[ti];
  float* f = flat + a.off[ti];
  for (int k = 0; k < 4; ++k) {
    const long long j = base + k * 256 + threadIdx.x;
    if (j < a.n[ti]) {
      if (dir == 0) f[j] = t[j] * scale;
      else t[j] = f[j] * scale;
    }
  }
}


// Momentum SGD over bf16 weights with fp32 master copies (mixed-precision CNN training).
// Tensor i: bf16 gradient at a.ptr[i] (autograd-owned, same storage order as the parameter),
// master/momentum/bf16-param segments at a.off[i] of the flat buffers. One pass reads the bf16
// grad + fp32 master + fp32 momentum and writes master, momentum and the rounded bf16 weight
// the next forward consumes, so autocast needs no per-step weight/grad casts.
// Matches torch.optim.SGD (dampening 0, no nesterov): d = g + wd*w; m = mu*m + d; w -= lr*m.
__device__ inline float bf16_to_f32(uint32_t v) { return __uint_as_float(v << 16); }
__device__ inline uint32_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);                                  // round to nearest even
  return u >> 16;
}

__global__ __launch_bounds__(256) void mt_sgd_master_kernel(MtArgs a, float* __restrict__ master,
                                                            float* __restrict__ mom,
                                                            uint16_t* __restrict__ wbf, float lr,
                                                            float mu, float wd) {
  int ti = 0;
  for (int i = 1; i < a.count; ++i)
    if ((int)blockIdx.x >= a.blk_begin[i]) ti = i;
  const long long j = (long long)(blockIdx.x - a.blk_begin[ti]) * 1024 + threadIdx.x * 4;
  if (j >= a.n[ti]) return;  // n % 4 == 0 (host-checked): a live thread owns 4 whole elements
  const long long o = a.off[ti] + j;
  const uint2 g2 = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(a.ptr[ti]) + j);
  float4 w4 = *reinterpret_cast<const float4*>(master + o);
  float4 m4 = *reinterpret_cast<const float4*>(mom + o);
  const float g[4] = {bf16_to_f32(g2.x & 0xffffu), bf16_to_f32(g2.x >> 16),
                      bf16_to_f32(g2.y & 0xffffu), bf16_to_f32(g2.y >> 16)};
  float* w = &w4.x;
  float* m = &m4.x;
  uint32_t r[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    m[k] = mu * m[k] + (g[k] + wd * w[k]);
    w[k] = w[k] - lr * m[k];
    r[k] = f32_to_bf16(w[k]);
  }
  *reinterpret_cast<float4*>(master + o) = w4;
  *reinterpret_cast<float4*>(mom + o) = m4;
  *reinterpret_cast<uint2*>(wbf + o) = make_uint2(r[0] | (r[1] << 16), r[2] | (r[3] << 16));
}

// Momentum SGD over ONE flat range: a data-parallel rank's shard of a gradient bucket after the
// RCCL reduce-scatter (ShardedMasterSGD's off-node backend). Same arithmetic, in the same order,
// as the xGMI kernels' shard update (csrc/ccl/xgmi_ccl.hip xgmi_sgd_*): d = g * scale + wd * w,
// m = mu * m + d, w = w - lr * m. BF16: bf16 summed gradient, fp32 master, rounded bf16 weight
// written to wbf; else fp32 gradient and the fp32 weights are their own masters. n % 4 == 0 and
// 16-byte aligned fp32 pointers (host-checked): one thread owns 4 elements per grid-stride step.
template <bool BF16>
__global__ __launch_bounds__(256) void shard_sgd_kernel(const void* __restrict__ grad,
                                                        float* __restrict__ w32,
                                                        float* __restrict__ mom,
                                                        uint16_t* __restrict__ wbf, long long n,
                                                        float lr, float mu, float wd,
                                                        float scale) {
  const long long stride = (long long)gridDim.x * 1024;
  for (long long j = ((long long)blockIdx.x * 256 + threadIdx.x) * 4; j < n; j += stride) {
    float g[4];
    if constexpr (BF16) {
      const uint2 g2 = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(grad) + j);
      g[0] = bf16_to_f32(g2.x & 0xffffu);
      g[1] = bf16_to_f32(g2.x >> 16);
      g[2] = bf16_to_f32(g2.y & 0xffffu);
      g[3] = bf16_to_f32(g2.y >> 16);
    } else {
      const float4 g4 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(grad) + j);
      g[0] = g4.x;
      g[1] = g4.y;
      g[2] = g4.z;
      g[3] = g4.w;
    }
    float4 w4 = *reinterpret_cast<const float4*>(w32 + j);
    float4 m4 = *reinterpret_cast<const float4*>(mom + j);
    float* w = &w4.x;
    float* m = &m4.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float d = g[k] * scale + wd * w[k];
      m[k] = mu * m[k] + d;
      w[k] = w[k] - lr * m[k];
    }
    *reinterpret_cast<float4*>(w32 + j) = w4;
    *reinterpret_cast<float4*>(mom + j) = m4;
    if constexpr (BF16) {
      *reinterpret_cast<uint2*>(wbf + j) = make_uint2(f32_to_bf16(w[0]) | (f32_to_bf16(w[1]) << 16),
                                                      f32_to_bf16(w[2]) | (f32_to_bf16(w[3]) << 16));
    }
  }
}

}  // namespace

// =============================================================================================
// Host launchers (plain C ABI; the torch binding TU validates shapes before calling these).
// =============================================================================================
extern "C" {

hipError_t arena_linear_fwd(ArenaRowSource src, const float* W, const float* bias, float* Y, int M,
                            int N, int K, int act, float keep_prob, uint32_t seed,
                            const long long* step_src, hipStream_t stream) {
  uint32_t thr = 0xFFFFFFFFu;
  float inv_keep = 1.f;
  if (keep_prob < 1.f) {
    thr = (uint32_t)((double)keep_prob * 4294967296.0);
    inv_keep = 1.f / keep_prob;
  }
  dim3 grid((N + 15) / 16, (M + 15) / 16);
  if (src.dtype == 1)
    hipLaunchKernelGGL((linear_fwd_kernel<1, 8>), grid, dim3(512), 0, stream, src, W, bias, Y, M,
                       N, K, act, thr, inv_keep, seed, step_src);
  else
    hipLaunchKernelGGL((linear_fwd_kernel<0, 8>), grid, dim3(512), 0, stream, src, W, bias, Y, M,
                       N, K, act, thr, inv_keep, seed, step_src);
  return hipGetLastError();
}

hipError_t arena_mlp_fwd_logits(ArenaRowSource src, const float* W, const float* bias, float* Y,
                                int M, int N, int K, float keep_prob, uint32_t seed,
                                const long long* step_src, const float* W2, float* W2_copy, int C,
                                float* logits2, uint8_t* xb, const void* lab_ptr, int lab_dtype,
                                int* yb, ArenaCounterOp ctr, const int* rows, hipStream_t stream) {
  if (C < 1 || C > 16 || K % 4) return hipErrorInvalidValue;
  uint32_t thr = 0xFFFFFFFFu;
  float inv_keep = 1.f;
  if (keep_prob < 1.f) {
    thr = (uint32_t)((double)keep_prob * 4294967296.0);
    inv_keep = 1.f / keep_prob;
  }
  dim3 grid((N + 15) / 16, (M + 15) / 16);
  // the training step's configuration gets the straight-line variant (see the kernel)
  const int nsteps = (K + 15) / 16;
  const bool fast = src.dtype == 1 && src.idx != nullptr && src.cursor != nullptr &&
                    src.cursor == step_src && src.cursor_off == 0 && ctr.dst != nullptr &&
                    ctr.src == step_src && xb != nullptr && lab_ptr != nullptr &&
                    (nsteps + 7) / 8 <= 8 && src.idx_len < (1LL << 31);
  if (fast && rows != nullptr)
    hipLaunchKernelGGL((mlp_fwd_logits_kernel<1, 8, 2>), grid, dim3(512), 0, stream, src, W,
                       bias, Y, M, N, K, thr, inv_keep, seed, step_src, W2, W2_copy, C, logits2,
                       xb, lab_ptr, lab_dtype, yb, ctr, rows);
  else if (fast)
    hipLaunchKernelGGL((mlp_fwd_logits_kernel<1, 8, 1>), grid, dim3(512), 0, stream, src, W,
                       bias, Y, M, N, K, thr, inv_keep, seed, step_src, W2, W2_copy, C, logits2,
                       xb, lab_ptr, lab_dtype, yb, ctr, rows);
  else if (src.dtype == 1)
    hipLaunchKernelGGL((mlp_fwd_logits_kernel<1, 8, 0>), grid, dim3(512), 0, stream, src, W,
                       bias, Y, M, N, K, thr, inv_keep, seed, step_src, W2, W2_copy, C, logits2,
                       xb, lab_ptr, lab_dtype, yb, ctr, nullptr);
  else
    hipLaunchKernelGGL((mlp_fwd_logits_kernel<0, 8, 0>), grid, dim3(512), 0, stream, src, W,
                       bias, Y, M, N, K, thr, inv_keep, seed, step_src, W2, W2_copy, C, logits2,
                       nullptr, lab_ptr, lab_dtype, yb, ctr, nullptr);
  return hipGetLastError();
}

hipError_t arena_xent_head(const float* H, int M, int D, const float* W2, const float* b2, int C,
                           ArenaRowSource lab, float* dlogits, float* dZ, float keep_prob,
                           int relu_mask, float loss_scale, float* loss_acc, int* correct_acc,
                           int hist_len, const long long* hist_step, ArenaCounterOp ctr,
                           hipStream_t stream) {
  if (D > 64 * kHeadMaxT || C > kHeadMaxC || D * C > 1024 * kHeadStage || (D * C) % 4)
    return hipErrorInvalidValue;
  const float inv_keep = keep_prob < 1.f ? 1.f / keep_prob : 1.f;
  dim3 grid((M + 3) / 4);
  const size_t smem = sizeof(float) * ((size_t)D * C + 4);  // + dummy float4 slot
  const bool big = D * C > 1024 * 8;
  const bool small = C <= 10 && D <= 512 && !big;
#define ARENA_HEAD(LT, ST, CB, TB)                                                               \
  hipLaunchKernelGGL((xent_head_kernel<LT, ST, CB, TB>), grid, dim3(256), smem, stream, H, M, D, \
                     W2, b2, C, lab, dlogits, dZ, inv_keep, relu_mask, loss_scale, loss_acc,     \
                     correct_acc, hist_len, hist_step, ctr)
#define ARENA_HEAD_LT(LT)                \
  if (small) ARENA_HEAD(LT, 8, 10, 8);   \
  else if (big) ARENA_HEAD(LT, 16, 16, 16); \
  else ARENA_HEAD(LT, 8, 16, 16);
  switch (lab.dtype) {
    case 1: ARENA_HEAD_LT(1) break;
    case 2: ARENA_HEAD_LT(2) break;
    default: ARENA_HEAD_LT(3)
  }
#undef ARENA_HEAD_LT
#undef ARENA_HEAD
  return hipGetLastError();
}

hipError_t arena_wgrad_grouped(ArenaWGradProblem* probs, int nprob, ArenaAdam adam,
                               float grad_scale, ArenaCounterOp ctr, ArenaHead head,
                               hipStream_t stream) {
  if (nprob < 1 || nprob > kMaxProblems) return hipErrorInvalidValue;
  WGradArgs a;
  int blocks = 0;
  for (int i = 0; i < nprob; ++i) {
    probs[i].tiles_k = (probs[i].K + 63) / 64;
    probs[i].tiles_n = (probs[i].N + 15) / 16;
    probs[i].block_begin = blocks;
    blocks += probs[i].tiles_k * probs[i].tiles_n;
    a.p[i] = probs[i];
  }
  a.nprob = nprob;
  a.head_block = -1;
  for (int i = 0; i < nprob; ++i)
    if (probs[i].hd_mode != 0) { a.head_block = probs[i].block_begin; break; }
  a.adam = adam;
  a.grad_scale = grad_scale;
  a.ctr = ctr;
  a.head = head;
  // the fused MLP step: problem 0 = u8 dataset rows + hidden head, problem 1 = f32 H + output head
  const bool g0 = probs[0].x.idx != nullptr;
  const bool sp = head.parity == 0 || head.parity == 1;
  const bool mlp_pair = nprob == 2 && head.C <= 10 && probs[0].xt == 1 && probs[0].hd_mode == 2 &&
                        probs[1].xt == 0 && probs[1].hd_mode == 1 && probs[1].x.idx == nullptr &&
                        probs[0].mode == probs[1].mode && probs[0].M <= kMC &&
                        (probs[0].mode == 0 || (adam.t_ptr && adam.lr_ptr)) && head.step &&
                        probs[1].M <= kMC && head.lab.dtype == (g0 ? 1 : 2);
  const dim3 grid(blocks), block(256);
  if (mlp_pair) {
    const int m = probs[0].mode & 1;
#define ARENA_WG_PAIR(G, M, SP)                                                                \
  hipLaunchKernelGGL((wgrad_grouped_kernel<10, wgrad_spec(1, 2, G, M, SP),                     \
                                           wgrad_spec(0, 1, 0, M, SP)>), grid, block, 0, stream, a)
    if (sp) {
      if (g0 == 0 && m == 0) ARENA_WG_PAIR(0, 0, 1);
      else if (g0 == 0 && m == 1) ARENA_WG_PAIR(0, 1, 1);
      else if (g0 == 1 && m == 0) ARENA_WG_PAIR(1, 0, 1);
      else ARENA_WG_PAIR(1, 1, 1);
    } else {
      if (g0 == 0 && m == 0) ARENA_WG_PAIR(0, 0, 0);
      else if (g0 == 0 && m == 1) ARENA_WG_PAIR(0, 1, 0);
      else if (g0 == 1 && m == 0) ARENA_WG_PAIR(1, 0, 0);
      else ARENA_WG_PAIR(1, 1, 0);
    }
#undef ARENA_WG_PAIR
  } else if (head.C <= 10) {
    hipLaunchKernelGGL((wgrad_grouped_kernel<10, 0, 0>), grid, block, 0, stream, a);
  } else {
    hipLaunchKernelGGL((wgrad_grouped_kernel<16, 0, 0>), grid, block, 0, stream, a);
  }
  return hipGetLastError();
}

hipError_t arena_adam_flat(float* P, float* M, float* V, const float* G, long long n,
                           ArenaAdam adam, ArenaCounterOp ctr, hipStream_t stream) {
  if (n % 4) return hipErrorInvalidValue;
  const long long n4 = n / 4;
  const int blocks = (int)std::min<long long>((n4 + 255) / 256, 2048);
  hipLaunchKernelGGL(adam_flat_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, stream, P, M, V,
                     G, n4, adam, ctr);
  return hipGetLastError();
}

hipError_t arena_sgd_flat(float* P, const float* G, long long n, float lr, const float* lr_ptr,
                          float gscale, hipStream_t stream) {
  if (n % 4) return hipErrorInvalidValue;
  const long long n4 = n / 4;
  const int blocks = (int)std::min<long long>((n4 + 255) / 256, 2048);
  hipLaunchKernelGGL(sgd_flat_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, stream, P, G, n4,
                     lr, lr_ptr, gscale);
  return hipGetLastError();
}

hipError_t arena_softmax_xent(const float* logits, const long long* labels, int M, int C,
                              float* loss, float* dlogits, float grad_scale, hipStream_t stream) {
  hipLaunchKernelGGL(softmax_xent_kernel, dim3((M + 3) / 4), dim3(256), 0, stream, logits, labels,
                     M, C, loss, dlogits, grad_scale);
  return hipGetLastError();
}

// ptrs/offs/ns arrays of length count (any count; chunked into launches of kMtMax tensors).
hipError_t arena_mt_copy_scale(float* const* ptrs, const long long* offs, const long long* ns,
                               int count, float* flat, float scale, int dir, hipStream_t stream) {
  for (int base = 0; base < count; base += kMtMax) {
    MtArgs a;
    const int cnt = std::min(kMtMax, count - base);
    int blocks = 0;
    for (int i = 0; i < cnt; ++i) {
      a.ptr[i] = ptrs[base + i];
      a.off[i] = offs[base + i];
      a.n[i] = ns[base + i];
      a.blk_begin[i] = blocks;
      blocks += (int)((ns[base + i] + 1023) / 1024);
    }
    a.blk_begin[cnt] = blocks;
    a.count = cnt;
    if (blocks == 0) continue;
    hipLaunchKernelGGL(mt_copy_scale_kernel, dim3(blocks), dim3(256), 0, stream, a, flat, scale,
                       dir);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// grads[i]: bf16 gradient pointers; offs/ns: segment offsets (multiples of 4) and sizes (n % 4 == 0).
hipError_t arena_mt_sgd_master(const void* const* grads, const long long* offs, const long long* ns,
                               int count, float* master, float* mom, void* wbf, float lr, float mu,
                               float wd, hipStream_t stream) {
  for (int base = 0; base < count; base += kMtMax) {
    MtArgs a;
    const int cnt = std::min(kMtMax, count - base);
    int blocks = 0;
    for (int i = 0; i < cnt; ++i) {
      if (ns[base + i] % 4 || offs[base + i] % 4) return hipErrorInvalidValue;
      a.ptr[i] = const_cast<float*>(reinterpret_cast<const float*>(grads[base + i]));
      a.off[i] = offs[base + i];
      a.n[i] = ns[base + i];
      a.blk_begin[i] = blocks;
      blocks += (int)((ns[base + i] + 1023) / 1024);
    }
    a.blk_begin[cnt] = blocks;
    a.count = cnt;
    if (blocks == 0) continue;
    hipLaunchKernelGGL(mt_sgd_master_kernel, dim3(blocks), dim3(256), 0, stream, a, master, mom,
                       reinterpret_cast<uint16_t*>(wbf), lr, mu, wd);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t arena_shard_sgd(const void* grad, int grad_bf16, float* w32, float* mom, void* wbf,
                           long long n, float lr, float mu, float wd, float scale,
                           hipStream_t stream) {
  if (n % 4 || (grad_bf16 && !wbf)) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  const long long blocks = std::min<long long>((n + 1023) / 1024, 4096);
  if (grad_bf16)
    hipLaunchKernelGGL(shard_sgd_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, stream, grad,
                       w32, mom, reinterpret_cast<uint16_t*>(wbf), n, lr, mu, wd, scale);
  else
    hipLaunchKernelGGL(shard_sgd_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, stream, grad,
                       w32, mom, nullptr, n, lr, mu, wd, scale);
  return hipGetLastError();
}

}  // extern "C"
