// NHWC bf16 convolution as an implicit GEMM on the gfx950 matrix cores.
//
// Workload: the convolutions of the ResNet family that the reference's Horovod image benchmarks
// (charts/tf-horovod/README.md:66-69, SURVEY §2.11 "Horovod TF image"); MIOpen/CK run them at
// 100-550 TFLOP/s on MI355X (profiles/r2_conv_roofline.jsonl). Here one kernel computes
//
//     Y[m][co] = sum_{r,s,ci} X[n, ho*st-pad+r, wo*st-pad+s, ci] * W[co][r][s][ci]
//
// with m = (n, ho, wo) the output pixel: a GEMM of M = N*Ho*Wo rows, K = R*S*C (tap-major,
// channel-minor, i.e. the channels_last weight's own memory order) and Cout columns. Both operands
// are K-contiguous, so every 64-deep K step of a tile is one filter tap and 64 channels: a 128-byte
// run of one input pixel (A) or of one weight row (B).
//
// Design (MI355X-first, cdna_hip_programming.md §5):
//  * global_load_lds (16 B per lane) stages A and B straight into LDS: no VGPR round trip, no
//    ds_write. Padded taps and rows past M read a 16-byte zero page instead (the source address is
//    per lane, so the halo costs nothing extra).
//  * LDS rows are 128 B; the 16-byte chunk p of row r holds global chunk p ^ ((r >> 1) & 7). The
//    permutation is applied on the SOURCE address (glds writes lane-linearly) and undone on the
//    ds_read_b128 fragment read, which makes the 16 rows a 16x16x32 fragment read touches land on
//    16 distinct 16-byte bank slots (conflict-free).
//  * 4 waves (2 x 2), v_mfma_f32_16x16x32_bf16, two LDS buffers: tile t+1 is in flight while tile
//    t is multiplied; one vmcnt(0) + barrier per K step.
//  * The MFMA is issued as W-fragment x X-fragment, so a lane's accumulator holds 4 consecutive
//    output channels of one pixel: the epilogue stores 8-byte packed bf16 runs of an NHWC row.
//  * blockIdx is remapped so consecutive output tiles (sharing their A rows) run on one XCD.
//
// The backward-data pass of a stride-1 convolution is the same kernel on (dY, flipped/transposed
// W); see arena_amd/ops/conv.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kThreads = 256;
constexpr int kBK = 64;           // K elements per step (= 128 bytes of bf16)
constexpr int kRowBytes = kBK * 2;

__device__ uint4 g_zero_page[4] = {};  // 64 zero bytes: the source of every padded chunk

struct ConvArgs {
  const uint16_t* x;   // [N][H][W][C] bf16
  const uint16_t* w;   // [Cout][R][S][C] bf16
  uint16_t* y;         // [N][Ho][Wo][Cout] bf16
  float* part;         // optional BatchNorm partials [m_tiles][2][Cout] (tile mean, tile M2)
  const uint16_t* add; // optional [M][Cout] bf16 added to the fp32 sums before rounding (the
                       // other gradient of a tensor with two consumers: the residual join)
  // optional bit mask of the addend, [M][Cout / 8] bytes, bit i of byte v <-> element 8v + i:
  // only set elements are added. The residual join's other gradient is dY of a ReLU'd BatchNorm
  // times its ReLU mask; taking (dY, mask) spares the BN backward writing that product.
  const uint8_t* addmask;
  // BatchNorm-backward partials of the output (EPI 2, a backward-data pass whose output dY is the
  // gradient of a BN layer's output): g = dY (* ReLU mask bit); part[tile][0][c] = sum g,
  // part[tile][1][c] = sum g * (bnx - bnmean[c]) -- the bn_bwd_reduce partial format.
  const uint16_t* bnx;     // [M][Cout] the BN layer's input
  const uint8_t* bnmask;   // [M][Cout / 8] ReLU bits of the BN output, or null (no ReLU)
  const float* bnmean;     // [Cout] the BN layer's batch mean
  int N, H, W, C, Cout, R, S, stride, pad, Ho, Wo;
  int M;               // N * Ho * Wo
  int Ktot;            // R * S * C
  int m_tiles, n_tiles;
  int pad_w;           // left padding (pad is the top one)
  // Output placement: output pixel (n, ho, wo) is stored at (n, ho*osh + ooh, wo*osw + oow) of a
  // [N][Hy][Wy][Cout] tensor (mapped != 0; else dense [N][Ho][Wo][Cout]). The phases of a
  // stride-2 backward-data pass each write one parity class of dX this way.
  int mapped, Hy, Wy, osh, osw, ooh, oow;
  // fill_sib (mapped, ooh == oow == 0, the only phase with filter taps: 1x1 stride-2 backward
  // data): each output pixel also stores its osh*osw - 1 sibling pixels of the [Hy][Wy] image,
  // which receive no taps -- the addend there (add != null) or zero. One pass writes all of dX.
  int fill_sib;
  // coal: stage the output tile through LDS (fp32, half a tile at a time) and store whole 16-byte
  // chunks with consecutive lanes on consecutive chunks of a pixel row (the MFMA layout alone
  // stores 8 bytes per lane, 16 rows per instruction). Needed off only for EPI != 0 with an addend.
  int coal;
  // c16: C == 16 and a 64-deep K step is one filter row and FOUR consecutive filter columns
  // (4 pixels x 16 channels = 128 contiguous bytes of an NHWC row). S is a multiple of 4. The
  // space-to-depth form of the 7x7/2 stem runs on it.
  int c16;
  // EPI 1, accumulated statistics (bn_acc != null, part unused): every tile adds its moment
  // sums (n*mean = sum y, M2 + n*mean^2 = sum y^2 over its rows) into fp64 accumulators
  // bn_acc [ARENA_ACC_REP][2][Cout] (replica mt % ARENA_ACC_REP) with memory-side atomics, fire-and-forget (the persistent form: once per
  // block). The consuming BN apply pass derives its coefficients from the sums (bn_kernels.hip
  // apply_coefs) and the layer's backward zeroes them: no finalize launch, where per-tile
  // partials (3136 per channel for a 56x56 layer at batch 128) need a two-level merge.
  double* bn_acc;
  // Split-K (ksplit > 1): the K steps of every output tile are divided over ksplit blocks. Each
  // writes its fp32 accumulators to kws [tile][slice][acc][thread] (16-byte stores, thread-
  // contiguous), publishes them (agent release, then a relaxed ticket on kcnt[tile]), and the
  // block drawing the last ticket sums all slices in slice order -- the same order whichever
  // block arrives last, so results are bit-reproducible -- resets the ticket and runs the
  // epilogue. For the layers whose tile count leaves CUs idle (14x14 and 7x7 stages at batch 128).
  int ksplit;
  float4* kws;
  unsigned* kcnt;
  int xbytes, wbytes;  // buffer-descriptor ranges of x and w (both < 2^31 bytes, host-checked)
  int st1p;            // EPI 1 statistics in one pass (sum, sum of squares) instead of two
  // ablation switches of the halo K loop for timing studies only (tools/halo_ablation.py; the
  // output is garbage with any bit set): 1 no weight loads after the first chunk's prologue,
  // 2 no window loads after the first chunk, 4 no barriers in the tap loop, 8 no MFMAs
  int dbg;
  // Several phase convolutions of a strided backward-data pass in ONE launch (v2 tiles, plain
  // mapped epilogue): phase p owns blocks [ph[p].blk0, ph[p + 1].blk0) (starts on multiples of 8,
  // so the XCD-aware tile order holds within each phase) and overrides the per-phase fields.
  struct Phase {
    const uint16_t* w;
    int R, S, pad, pad_w, Ho, Wo, ooh, oow, wbytes, blk0;
  };
  int nph;             // 0: a single convolution
  Phase ph[4];
};

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS accesses (lgkmcnt) but not
// for its outstanding global stores. __syncthreads() also waits vmcnt(0), which in an epilogue
// that stores in two halves exposes the first half's store latency on every block.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---- split-K slab hand-off inside a launch (cdna_hip_programming.md §6 Guideline 16, form R1) --
// The slabs are stored write-through (sc1) and drained by every storing wave before the block's
// barrier; one lane then takes a relaxed agent-scope ticket. No release fence: an agent-scope
// release writes back the whole XCD L2 (buffer_wbl2), and with every split block of a launch
// doing one, the v2 split tiles ran ~2x slower than unsplit (profiles/r5_split_plan_fenced.log).
// The reducer reads every slab with sc1 loads, so it needs no acquire either.
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void slab_store(__amdgpu_buffer_rsrc_t r, int off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), r, off, 0, 16);
}

__device__ __forceinline__ float4 slab_load(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}

// After this block's slab stores: true (in every thread) for the block that drew the last of
// ks tickets on *cnt, which it resets for the next launch. `flag_lds`: 4 bytes of the block's LDS
// that no wave reads or writes at this point (the stage buffers after the K loop's last barrier).
__device__ __forceinline__ bool slab_ticket(unsigned* cnt, int ks, uint8_t* flag_lds) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave: its slab is out
  __syncthreads();
  volatile unsigned* flag = reinterpret_cast<volatile unsigned*>(flag_lds);
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned last = old == (unsigned)(ks - 1) ? 1u : 0u;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = last;
  }
  __syncthreads();
  const bool last = flag[0] != 0u;
  __syncthreads();   // every wave has read the flag before the epilogue reuses the LDS
  return last;
}

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)lds_wave_base, 16, 0, 0);
}

// the same with the non-temporal cache policy (aux bit 1: nt)
__device__ __forceinline__ void glds16nt(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)lds_wave_base, 16, 0, 2);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// 8 bf16 addend elements at element offset `off` (a multiple of 8), zeroed where the mask bit is 0
__device__ __forceinline__ uint4 masked_add8(const uint16_t* add, const uint8_t* mask,
                                             size_t off) {
  uint4 q = *reinterpret_cast<const uint4*>(add + off);
  if (mask != nullptr) {
    const uint32_t mk = mask[off >> 3];
    uint32_t* w = reinterpret_cast<uint32_t*>(&q);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w[e] &= ((mk >> (2 * e)) & 1u ? 0x0000ffffu : 0u) | ((mk >> (2 * e + 1)) & 1u ? 0xffff0000u : 0u);
  }
  return q;
}

// 4 bf16 addend elements at element offset `off` (a multiple of 4), masked likewise
__device__ __forceinline__ uint2 masked_add4(const uint16_t* add, const uint8_t* mask,
                                             size_t off) {
  uint2 q = *reinterpret_cast<const uint2*>(add + off);
  if (mask != nullptr) {
    const uint32_t mk = (uint32_t)mask[off >> 3] >> (off & 7);
    q.x &= ((mk & 1u) ? 0x0000ffffu : 0u) | ((mk & 2u) ? 0xffff0000u : 0u);
    q.y &= ((mk & 4u) ? 0x0000ffffu : 0u) | ((mk & 8u) ? 0xffff0000u : 0u);
  }
  return q;
}

// bf16 round-to-nearest-even of two floats, packed (lo = a): ONE v_cvt_pk_bf16_f32 on gfx950.
// The integer form (add 0x7fff + lsb, shift) took ~9 VALU ops per pair, which on the streaming-
// bound 1x1 convolutions was a visible share of the epilogue (and turned some NaNs into Inf).
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  const f32x2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

__device__ __forceinline__ float bf16_round(float f) {
  return __uint_as_float(pack_bf16x2(f, 0.f) << 16);
}

// sum over the 16 lanes of a DPP row (lane bits 0..3); every lane of the row gets the sum
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, false));
  return v;
}

// The accumulator replica (abi.h ARENA_ACC_REP) that row tile `mt` adds its BatchNorm sums into:
// tiles of one column range differ in mt, so the same-address fp64 atomics of up to 3136 tiles per
// channel spread over every replica.
__device__ __forceinline__ double* acc_replica(const ConvArgs& a, int mt) {
  return a.bn_acc + (size_t)(mt % ARENA_ACC_REP) * 2 * a.Cout;
}

// EPI 1 accumulated-statistics tail (see ConvArgs::bn_acc). `emit(add)` calls add(c, mean, m2)
// for the block's channels c in [0, BN) whose tile statistics this thread holds. The values are
// restaged in LDS so that consecutive lanes add to consecutive channels: 64 fp64 adds = 512
// contiguous bytes per wave instruction (scattered few-lane atomics cost one 64-B memory-side
// request each). No wait and no fence: the kernel's end makes the sums visible to the finalize.
template <int BM, int BN, int NT, typename Emit>
__device__ __forceinline__ void bn_acc_epilogue(const ConvArgs& a, int mt, int n0, int nrows,
                                                Emit&& emit) {
  __shared__ float s_st[2][BN];
  emit([&](int c, float mean, float m2) {
    s_st[0][c] = mean;
    s_st[1][c] = m2;
  });
  // LDS-only barrier: __syncthreads() would also wait for the tile's output stores (vmcnt(0)),
  // holding the CU slot for their whole latency (measured +16 us on a 56x56 1x1 layer)
  lds_barrier();
  double* acc = acc_replica(a, mt) + n0;
  const double n = (double)nrows;
  for (int c = threadIdx.x; c < BN; c += NT) {
    const double mu = (double)s_st[0][c];
    const double s1 = n * mu, s2 = (double)s_st[1][c] + n * mu * mu;
    unsafeAtomicAdd(acc + c, s1);             // sum y
    unsafeAtomicAdd(acc + a.Cout + c, s2);    // sum y^2
  }
}

// NBUF = LDS stage buffers: 2 (double-buffered K loop) or 1 for a single 64-deep K step (1x1
// convolutions over 64 channels): half the LDS, so twice the blocks per CU overlap their loads
// with other blocks' epilogues -- those shapes are bound by the output write.
// EPI: 0 = plain, 1 = BatchNorm statistics of Y (forward), 2 = BatchNorm-backward partials of Y
// (see ConvArgs::bnx).
// NWM x NWN waves (NT = 64 NWM NWN threads): 2 x 2 for the 128- and 64-wide tiles, 4 x 2 for the
// 256-row tiles (per-wave 64 x BN/2), so a block's MFMA work per staged byte grows with the tile.
//
// C16 selects the staging form: false (every C % 64 shape) stages through buffer descriptors --
// each glds slot's byte offset is fixed per block, a 64-deep K step moves only scalars (tap and
// channel-block offsets, kept incrementally: no divisions in the loop), and a padded tap or a
// row past M gets an out-of-range offset, which the descriptor's range check turns into zeros.
// That leaves ~3 VALU per A slot per filter tap and none per weight slot, where the address
// arithmetic of the flat form (a tap division, bounds checks and 64-bit addresses per slot per
// step) issued ~115 VALU and ~140 SALU per K step against 16 MFMAs (the kernels were
// issue-bound, not load-bound). C16 = true is the stem's space-to-depth form on flat loads.
template <int BM, int BN, int EPI, int NBUF = 2, int NWM = 2, int NWN = 2, bool C16 = false>
__device__ __forceinline__ void conv_fwd_body(const ConvArgs& a) {
  constexpr int NT = 64 * NWM * NWN;
  constexpr int WM = BM / NWM, WN = BN / NWN;    // per-wave output tile
  constexpr int MI = WM / 16, NI = WN / 16;      // 16x16 MFMA tiles per wave
  constexpr int AI = BM * 8 / NT;                // A staging instructions per thread
  constexpr int BI = BN * 8 / NT;
  static_assert(AI >= 1 && BI >= 1 && MI >= 1 && NI >= 1, "tile too small for the wave grid");
  constexpr int kBufBytes = (BM + BN) * kRowBytes;
  __shared__ __attribute__((aligned(16))) uint8_t lds[NBUF * kBufBytes];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // XCD-aware tile order: blocks b and b+8 share an XCD (round-robin dispatch), so give each XCD
  // a contiguous range of tiles (bijective for any grid size).
  const int ks = a.ksplit;
  const int nwg = a.m_tiles * a.n_tiles * ks;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r8 = nwg & 7;
  const int lin = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (bid >> 3);
  // a tile's K slices are consecutive in the XCD order: the last arriver reads same-XCD slabs
  const int tile0 = ks > 1 ? lin / ks : lin;
  const int slice = ks > 1 ? lin - tile0 * ks : 0;
  const int nt = tile0 % a.n_tiles;
  const int mt0 = tile0 / a.n_tiles;
  const int n0 = nt * BN;

  {
    const int mt = mt0;
    const int tile = mt * a.n_tiles + nt;
    const int m0 = mt * BM;

    // ---- per-thread staging descriptors: row and (swizzled) source chunk of every glds ----
    // slot s = (wave*AI + i)*64 + lane -> LDS row s/8, chunk position s%8 (= lane%8)
    const int pos = lane & 7;
    int a_hb[AI], a_wb[AI], a_nb[AI], a_chunk[AI];
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int row = (wave * AI + i) * 8 + (lane >> 3);
      a_chunk[i] = pos ^ swz(row);
      const int m = m0 + row;
      if (m < a.M) {
        const int hw = a.Ho * a.Wo;
        const int n = m / hw, rem = m - n * hw;
        const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
        a_hb[i] = ho * a.stride - a.pad;
        a_wb[i] = wo * a.stride - a.pad_w;
        a_nb[i] = n * a.H;
      } else {
        a_hb[i] = -(1 << 28);  // every tap invalid -> zero page
        a_wb[i] = 0;
        a_nb[i] = 0;
      }
    }
    const uint16_t* b_src[BI];
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int row = (wave * BI + i) * 8 + (lane >> 3);
      b_src[i] = a.w + (size_t)(n0 + row) * a.Ktot + (pos ^ swz(row)) * 8;
    }
    const int CB = C16 ? 1 : a.C / kBK;  // 64-channel blocks per tap
    // this block's K steps: [t0, t0 + T) of the Ktot / kBK (split-K: slice `slice` of ks)
    const int Tall = a.Ktot / kBK;
    const int t0 = (int)((long long)Tall * slice / ks);
    const int T = (int)((long long)Tall * (slice + 1) / ks) - t0;

    // ---- descriptor staging state (C16 == false) ----
    constexpr uint32_t kOOB = 0x80000000u;   // >= num_records: the load returns zeros
    const __amdgpu_buffer_rsrc_t xrsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wrsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.wbytes, 0x00020000);
    int a_lane[AI];          // byte offset of the slot's 16-byte chunk at tap (0, 0), channel block 0
    uint32_t a_mask[AI];     // bit r*S+s: tap (r, s) inside the image for this slot's pixel
    uint32_t a_cur[AI];      // the current tap's offset, or kOOB
    uint32_t b_voff[BI];
    int s_tap = 0, s_cb = 0, s_s = 0, s_tapoff = 0, s_t = t0;   // scalar K-step state
    if constexpr (!C16) {
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const int row = (wave * AI + i) * 8 + (lane >> 3);
        uint32_t mk = 0u;
        int off = 0;
        if (a_hb[i] > -(1 << 27)) {
          for (int r = 0; r < a.R; ++r) {
            if ((unsigned)(a_hb[i] + r) >= (unsigned)a.H) continue;
            for (int s2 = 0; s2 < a.S; ++s2)
              if ((unsigned)(a_wb[i] + s2) < (unsigned)a.W) mk |= 1u << (r * a.S + s2);
          }
          off = (((a_nb[i] + a_hb[i]) * a.W + a_wb[i]) * a.C + a_chunk[i] * 8) * 2;
        }
        (void)row;
        a_lane[i] = off;
        a_mask[i] = mk;
      }
#pragma unroll
      for (int i = 0; i < BI; ++i) {
        const int row = (wave * BI + i) * 8 + (lane >> 3);
        b_voff[i] = (uint32_t)(((n0 + row) * a.Ktot + (pos ^ swz(row)) * 8) * 2);
      }
      s_tap = t0 / CB;
      s_cb = t0 - s_tap * CB;
      const int r0 = s_tap / a.S;
      s_s = s_tap - r0 * a.S;
      s_tapoff = (r0 * a.W + s_s) * a.C * 2;
#pragma unroll
      for (int i = 0; i < AI; ++i)
        a_cur[i] = ((a_mask[i] >> s_tap) & 1u) ? (uint32_t)(a_lane[i] + s_tapoff) : kOOB;
    }

    auto stage = [&](int tl, int buf) {
      const int t = t0 + tl;
      uint8_t* base = lds + buf * kBufBytes;
      if constexpr (!C16) {
        (void)t;
        const int coff = s_cb * kRowBytes;   // channel block within the tap (scalar)
#pragma unroll
        for (int i = 0; i < AI; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, (lds_ptr_t)(base + (wave * AI + i) * 64 * 16),
                                                   16, a_cur[i], coff, 0, 0);
        uint8_t* bb = base + BM * kRowBytes;
#pragma unroll
        for (int i = 0; i < BI; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(wrsrc, (lds_ptr_t)(bb + (wave * BI + i) * 64 * 16),
                                                   16, b_voff[i], s_t * kRowBytes, 0, 0);
        // advance the scalar state to the next K step
        ++s_t;
        if (++s_cb == CB) {
          s_cb = 0;
          ++s_tap;
          s_tapoff += a.C * 2;
          if (++s_s == a.S) {
            s_s = 0;
            s_tapoff += (a.W - a.S) * a.C * 2;
          }
#pragma unroll
          for (int i = 0; i < AI; ++i)
            a_cur[i] = ((a_mask[i] >> s_tap) & 1u) ? (uint32_t)(a_lane[i] + s_tapoff) : kOOB;
        }
        return;
      }
      if (C16) {
        // K step t = filter row r, columns 4*sb .. 4*sb+3; 16-byte chunk c = pixel c/2, half c%2
        const int SB = a.S >> 2;
        const int r = t / SB, sb = t - r * SB;
#pragma unroll
        for (int i = 0; i < AI; ++i) {
          const int c = a_chunk[i];
          const int hi = a_hb[i] + r, wi = a_wb[i] + sb * 4 + (c >> 1);
          const bool ok = (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
          const void* src = ok ? (const void*)(a.x + ((size_t)(a_nb[i] + hi) * a.W + wi) * 16 +
                                               (c & 1) * 8)
                               : (const void*)g_zero_page;
          glds16(src, base + (wave * AI + i) * 64 * 16);
        }
      } else {
        const int tap = t / CB, cb = t - tap * CB;
        const int r = tap / a.S, s = tap - r * a.S;
#pragma unroll
        for (int i = 0; i < AI; ++i) {
          const int hi = a_hb[i] + r, wi = a_wb[i] + s;
          const bool ok = (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
          const void* src = ok ? (const void*)(a.x + ((size_t)(a_nb[i] + hi) * a.W + wi) * a.C +
                                               cb * kBK + a_chunk[i] * 8)
                               : (const void*)g_zero_page;
          glds16(src, base + (wave * AI + i) * 64 * 16);
        }
      }
      uint8_t* bbase = base + BM * kRowBytes;
#pragma unroll
      for (int i = 0; i < BI; ++i) glds16(b_src[i] + (size_t)t * kBK, bbase + (wave * BI + i) * 64 * 16);
    };
    (void)a_cur;

    f32x4v acc[MI][NI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

    const int wm = wave / NWN, wn = wave % NWN;
    const int fr = lane & 15, fq = lane >> 4;

    auto compute = [&](int buf) {
      const uint8_t* abuf = lds + buf * kBufBytes;
      const uint8_t* bbuf = abuf + BM * kRowBytes;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[MI], bfr[NI];
        const int c = kk * 4 + fq;  // global 16-byte chunk of this lane's 8 k values
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int row = wm * WM + i * 16 + fr;
          af[i] = *reinterpret_cast<const bf16x8*>(abuf + row * kRowBytes + ((c ^ swz(row)) << 4));
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int row = wn * WN + j * 16 + fr;
          bfr[j] = *reinterpret_cast<const bf16x8*>(bbuf + row * kRowBytes + ((c ^ swz(row)) << 4));
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
    };

    if constexpr (NBUF >= 3) {
      // NBUF stage buffers, S = NBUF - 1 K steps in flight: the glds of steps t+2 .. t+S stay
      // outstanding across the barrier that publishes step t+1 (counted vmcnt = this thread's glds
      // of S - 1 stages, raw s_barrier: __syncthreads() would drain every outstanding LDS-DMA
      // with a vmcnt(0)). The deep-K layers (3x3 at 14x14 / 7x7: 36-72 K steps of ~500 MFMA
      // cycles each) wait ~700 ns per staged step, so one step in flight leaves them latency-bound.
      // RAW: stage t+1 is read in iteration t+1, after the vmcnt that retired it and a barrier.
      // WAR: stage t+S overwrites buffer (t-1) % NBUF, whose reads finished before iteration
      // t-1's barrier.
      constexpr int S = NBUF - 1;
      constexpr int kLps = AI + BI;   // glds per thread per stage
#pragma unroll
      for (int i = 0; i < S; ++i)
        if (i < T) stage(i, i);
      if (T >= S)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((S - 1) * kLps) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      int cur = 0;
      for (int t = 0; t < T; ++t) {
        if (t + S < T) stage(t + S, cur == 0 ? NBUF - 1 : cur - 1);
        compute(cur);
        if (t + S < T)
          asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((S - 1) * kLps) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        cur = cur == NBUF - 1 ? 0 : cur + 1;
      }
    } else {
      stage(0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();

      for (int t = 0; t < T; ++t) {
        const int cur = NBUF == 1 ? 0 : (t & 1);
        if (NBUF == 2 && t + 1 < T) stage(t + 1, cur ^ 1);
        compute(cur);
        if (NBUF == 1 && t + 1 < T) {   // serial: every wave is done with the buffer, restage it
          __syncthreads();
          stage(t + 1, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }

    if (ks > 1) {
      // ---- split-K hand-off (slab_store / slab_ticket: write-through slabs, relaxed ticket,
      // sc1 reads; the flag travels through the stage LDS, free after the K loop's barrier -- a
      // second __shared__ object would perturb the K loop's waits, cdna_hip_programming.md §5
      // item 4a) ----
      constexpr int NA = MI * NI;
      const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.kws + (size_t)tile * ks * NA * NT), (short)0, ks * NA * NT * 16, 0x00020000);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          slab_store(srs, ((slice * NA + i * NI + j) * NT + tid) * 16,
                     make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]));
      if (!slab_ticket(a.kcnt + tile, ks, lds)) return;
      // sum the slices in slice order (this block's own slab re-read from memory: the order, and
      // so the rounding, is independent of which block arrived last)
#pragma unroll
      for (int i = 0; i < MI; ++i) {
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const float4 v = slab_load(srs, ((i * NI + j) * NT + tid) * 16);
          acc[i][j] = f32x4v{v.x, v.y, v.z, v.w};
        }
        for (int s = 1; s < ks; ++s) {
          float4 v[NI];
#pragma unroll
          for (int j = 0; j < NI; ++j) v[j] = slab_load(srs, ((s * NA + i * NI + j) * NT + tid) * 16);
#pragma unroll
          for (int j = 0; j < NI; ++j) acc[i][j] += f32x4v{v[j].x, v[j].y, v[j].z, v[j].w};
        }
      }
    }

    // ---- epilogue: lane holds channels n0+wn*WN+j*16+4*fq .. +3 of pixel m0+wm*WM+i*16+fr ----
    // EPI 2 operands, issued before the stores so their latency overlaps them (clamped addresses)
    uint2 bx[EPI == 2 ? MI : 1][EPI == 2 ? NI : 1];
    uint32_t bm[EPI == 2 ? MI : 1][EPI == 2 ? NI : 1];
    float4 bmu[EPI == 2 ? NI : 1];
    if constexpr (EPI == 2) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = min(m0 + wm * WM + i * 16 + fr, a.M - 1);
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int c0 = n0 + wn * WN + j * 16 + 4 * fq;
          bx[i][j] = *reinterpret_cast<const uint2*>(a.bnx + (size_t)m * a.Cout + c0);
          bm[i][j] = a.bnmask ? ((uint32_t)a.bnmask[(size_t)m * (a.Cout >> 3) + (c0 >> 3)] >>
                                 (c0 & 7)) : 0xfu;
          if (m0 + wm * WM + i * 16 + fr >= a.M) bm[i][j] = 0u;   // rows past M: no contribution
        }
      }
#pragma unroll
      for (int j = 0; j < NI; ++j)
        bmu[j] = *reinterpret_cast<const float4*>(a.bnmean + n0 + wn * WN + j * 16 + 4 * fq);
    }
    // EPI 1: round the accumulators to their stored bf16 values once; the stores (whose own
    // rounding is then exact) and the statistics below both read them.
    if constexpr (EPI == 1) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            const uint32_t u = pack_bf16x2(acc[i][j][r], acc[i][j][r + 1]);
            acc[i][j][r] = __uint_as_float(u << 16);
            acc[i][j][r + 1] = __uint_as_float(u & 0xffff0000u);
          }
    }
    if (a.coal && !(EPI != 0 && a.add != nullptr)) {
      // ---- coalesced store through LDS (stage buffers are free: the K loop ended on a barrier) ----
      float* stg = reinterpret_cast<float*>(lds);
      constexpr int F4R = BN / 4;   // float4 slots per staged row (>= 16: the XOR below stays inside)
      constexpr int CPR = BN / 8;   // 16-byte bf16 output chunks per row
#pragma unroll
      for (int h = 0; h < NWM; ++h) {
        if (h) lds_barrier();       // every reader of the first half is done
        if (wm == h) {
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const int row = i * 16 + fr;
#pragma unroll
            for (int j = 0; j < NI; ++j) {
              const int slot = (wn * WN + j * 16) / 4 + fq;
              *reinterpret_cast<f32x4v*>(stg + (row * F4R + (slot ^ (row & 7))) * 4) = acc[i][j];
            }
          }
        }
        lds_barrier();              // the staged half is complete (global stores may be in flight)
        for (int q = tid; q < WM * CPR; q += NT) {
          const int row = q / CPR, cc = q - row * CPR;
          const int m = m0 + h * WM + row;
          if (m >= a.M) continue;
          const f32x4v lo = *reinterpret_cast<const f32x4v*>(stg + (row * F4R + ((2 * cc) ^ (row & 7))) * 4);
          const f32x4v hi =
              *reinterpret_cast<const f32x4v*>(stg + (row * F4R + ((2 * cc + 1) ^ (row & 7))) * 4);
          float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          size_t pix = (size_t)m;
          int n = 0, ho = 0, wo = 0;
          if (a.mapped) {
            const int hw = a.Ho * a.Wo;
            n = m / hw;
            const int rem = m - n * hw;
            ho = rem / a.Wo;
            wo = rem - ho * a.Wo;
            pix = ((size_t)n * a.Hy + ho * a.osh + a.ooh) * a.Wy + wo * a.osw + a.oow;
          }
          const size_t off = pix * a.Cout + n0 + cc * 8;
          if (a.add != nullptr) {
            const uint4 qa = masked_add8(a.add, a.addmask, off);
            const uint32_t u[4] = {qa.x, qa.y, qa.z, qa.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[2 * e] += __uint_as_float(u[e] << 16);
              v[2 * e + 1] += __uint_as_float(u[e] & 0xffff0000u);
            }
          }
          *reinterpret_cast<uint4*>(a.y + off) =
              make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                         pack_bf16x2(v[6], v[7]));
          if (a.fill_sib) {
            for (int da = 0; da < a.osh; ++da) {
              const int hy = ho * a.osh + da;
              if (hy >= a.Hy) break;
              for (int db = 0; db < a.osw; ++db) {
                const int wy = wo * a.osw + db;
                if ((da == 0 && db == 0) || wy >= a.Wy) continue;
                const size_t so = (((size_t)n * a.Hy + hy) * a.Wy + wy) * a.Cout + n0 + cc * 8;
                *reinterpret_cast<uint4*>(a.y + so) =
                    a.add ? masked_add8(a.add, a.addmask, so) : make_uint4(0u, 0u, 0u, 0u);
              }
            }
          }
        }
      }
    } else {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * WM + i * 16 + fr;
      if (m >= a.M) continue;
      size_t pix = (size_t)m;
      int n = 0, ho = 0, wo = 0;
      if (a.mapped) {
        const int hw = a.Ho * a.Wo;
        n = m / hw;
        const int rem = m - n * hw;
        ho = rem / a.Wo;
        wo = rem - ho * a.Wo;
        pix = ((size_t)n * a.Hy + ho * a.osh + a.ooh) * a.Wy + wo * a.osw + a.oow;
      }
      uint16_t* yrow = a.y + pix * a.Cout + n0 + wn * WN + 4 * fq;
      if (a.fill_sib) {
        for (int da = 0; da < a.osh; ++da) {
          const int hy = ho * a.osh + da;
          if (hy >= a.Hy) break;
          for (int db = 0; db < a.osw; ++db) {
            const int wy = wo * a.osw + db;
            if ((da == 0 && db == 0) || wy >= a.Wy) continue;
            const size_t off = (((size_t)n * a.Hy + hy) * a.Wy + wy) * a.Cout + n0 + wn * WN + 4 * fq;
#pragma unroll
            for (int j = 0; j < NI; ++j) {
              const uint2 v = a.add ? masked_add4(a.add, a.addmask, off + j * 16)
                                    : make_uint2(0u, 0u);
              *reinterpret_cast<uint2*>(a.y + off + j * 16) = v;
            }
          }
        }
      }
      if (a.add != nullptr) {
        const size_t aoff = (size_t)(yrow - a.y);
        uint2 q[NI];
#pragma unroll
        for (int j = 0; j < NI; ++j) q[j] = masked_add4(a.add, a.addmask, aoff + j * 16);
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          acc[i][j][0] += __uint_as_float(q[j].x << 16);
          acc[i][j][1] += __uint_as_float(q[j].x & 0xffff0000u);
          acc[i][j][2] += __uint_as_float(q[j].y << 16);
          acc[i][j][3] += __uint_as_float(q[j].y & 0xffff0000u);
        }
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        uint2 v;
        v.x = pack_bf16x2(acc[i][j][0], acc[i][j][1]);
        v.y = pack_bf16x2(acc[i][j][2], acc[i][j][3]);
        *reinterpret_cast<uint2*>(yrow + j * 16) = v;
      }
    }
    }
    if constexpr (EPI == 2) {
      // per channel over the tile's valid rows: sum g, sum g * (x - mean), g = stored dY * mask.
      // Per element: the stored (bf16-rounded) value via one v_cvt_pk_bf16_f32 per pair, the mask
      // select (rows past M were cleared from the mask bits at load), packed fp32 sums.
      float* red = reinterpret_cast<float*>(lds);   // [NWM][2][BN]
      float s1[NI][4], s2[NI][4];
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const f32x2 mu01 = {bmu[j].x, bmu[j].y}, mu23 = {bmu[j].z, bmu[j].w};
        f32x2 a01 = {0.f, 0.f}, a23 = {0.f, 0.f}, b01 = {0.f, 0.f}, b23 = {0.f, 0.f};
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const uint32_t u01 = pack_bf16x2(acc[i][j][0], acc[i][j][1]);
          const uint32_t u23 = pack_bf16x2(acc[i][j][2], acc[i][j][3]);
          const uint32_t mk = bm[i][j];
          const f32x2 g01 = {(mk & 1u) ? __uint_as_float(u01 << 16) : 0.f,
                             (mk & 2u) ? __uint_as_float(u01 & 0xffff0000u) : 0.f};
          const f32x2 g23 = {(mk & 4u) ? __uint_as_float(u23 << 16) : 0.f,
                             (mk & 8u) ? __uint_as_float(u23 & 0xffff0000u) : 0.f};
          const f32x2 x01 = {__uint_as_float(bx[i][j].x << 16),
                             __uint_as_float(bx[i][j].x & 0xffff0000u)};
          const f32x2 x23 = {__uint_as_float(bx[i][j].y << 16),
                             __uint_as_float(bx[i][j].y & 0xffff0000u)};
          a01 += g01;
          a23 += g23;
          b01 = __builtin_elementwise_fma(g01, x01 - mu01, b01);
          b23 = __builtin_elementwise_fma(g23, x23 - mu23, b23);
        }
        s1[j][0] = row16_sum(a01.x); s1[j][1] = row16_sum(a01.y);
        s1[j][2] = row16_sum(a23.x); s1[j][3] = row16_sum(a23.y);
        s2[j][0] = row16_sum(b01.x); s2[j][1] = row16_sum(b01.y);
        s2[j][2] = row16_sum(b23.x); s2[j][3] = row16_sum(b23.y);
      }
      lds_barrier();   // every wave is past its last read of the staging LDS (stores may be in flight)
      if (fr == 0) {
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int c = wn * WN + j * 16 + 4 * fq + r;
            red[wm * 2 * BN + c] = s1[j][r];
            red[wm * 2 * BN + BN + c] = s2[j][r];
          }
      }
      lds_barrier();
      if (wm == 0 && fr == 0) {
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int c = wn * WN + j * 16 + 4 * fq + r;
            float r1 = red[c], r2 = red[BN + c];
#pragma unroll
            for (int h = 1; h < NWM; ++h) {
              r1 += red[h * 2 * BN + c];
              r2 += red[h * 2 * BN + BN + c];
            }
            if (a.bn_acc != nullptr) {   // acc mode: the BN layer's fp64 backward sums
              double* acc = acc_replica(a, mt) + n0;
              unsafeAtomicAdd(acc + c, (double)r1);
              unsafeAtomicAdd(acc + a.Cout + c, (double)r2);
            } else {
              a.part[(size_t)mt * 2 * a.Cout + n0 + c] = r1;
              a.part[(size_t)mt * 2 * a.Cout + a.Cout + n0 + c] = r2;
            }
          }
      }
    }
    if constexpr (EPI == 1) {
      // BatchNorm statistics of this tile's (rounded) outputs, two-pass -- mean, then sum of
      // squared deviations -- over the valid rows: the partial format of bn_stats_kernel with
      // rpb = BM, so the BN layer that consumes this output skips its statistics pass over HBM.
      // Every output element passes through it, which on the streaming-bound 1x1 shapes made its
      // scalar per-element math (a rounding sequence per pass, selects) a measurable cost: the
      // values are rounded once before the stores, the sums are packed fp32 (two channels per op)
      // and the row-validity selects only run on the last, partial tile (1x1 64->256 @56x56,
      // batch 128: 94 -> 85 us; profiles/r2_conv_epi_{before,after}.jsonl).
      const int nrows = min(BM, a.M - m0);
      const bool full = nrows == BM;
      float* red = reinterpret_cast<float*>(lds);   // [NWM][BN] ([NWM][2][BN] single-pass)
      float mean[NI][4], s[NI][4];
      auto exchange = [&](bool first) {   // s (row-16 sums of this wave) -> per-block channel sums
        if (!first) lds_barrier();        // every wave has read the previous sums
        if (fr == 0) {
#pragma unroll
          for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[wm * BN + wn * WN + j * 16 + 4 * fq + r] = s[j][r];
        }
        lds_barrier();
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int c = wn * WN + j * 16 + 4 * fq + r;
            float v = red[c];
#pragma unroll
            for (int h = 1; h < NWM; ++h) v += red[h * BN + c];
            s[j][r] = v;
          }
      };
      const float inv_n = 1.f / (float)nrows;
      if (a.st1p) {
        // single pass (ConvArgs::st1p): sums and sums of squares together, ONE LDS exchange;
        // M2 = sum y^2 - n mean^2 over the tile's <= 256 rows in fp32 (the cross-tile merge is
        // fp64): the two-pass form's second exchange and barrier are the epilogue's cost
        float ss[NI][4];
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          f32x2 t0 = {0.f, 0.f}, t1 = {0.f, 0.f}, q0 = {0.f, 0.f}, q1 = {0.f, 0.f};
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            f32x2 v0 = {acc[i][j][0], acc[i][j][1]}, v1 = {acc[i][j][2], acc[i][j][3]};
            if (!full && m0 + wm * WM + i * 16 + fr >= a.M) v0 = v1 = f32x2{0.f, 0.f};
            t0 += v0;
            t1 += v1;
            q0 = __builtin_elementwise_fma(v0, v0, q0);
            q1 = __builtin_elementwise_fma(v1, v1, q1);
          }
          s[j][0] = row16_sum(t0.x); s[j][1] = row16_sum(t0.y);
          s[j][2] = row16_sum(t1.x); s[j][3] = row16_sum(t1.y);
          ss[j][0] = row16_sum(q0.x); ss[j][1] = row16_sum(q0.y);
          ss[j][2] = row16_sum(q1.x); ss[j][3] = row16_sum(q1.y);
        }
        lds_barrier();   // the coalesced store path's last reads of the staging LDS are done
        if (fr == 0) {
#pragma unroll
          for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int c = wn * WN + j * 16 + 4 * fq + r;
              red[wm * 2 * BN + c] = s[j][r];
              red[wm * 2 * BN + BN + c] = ss[j][r];
            }
        }
        lds_barrier();
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int c = wn * WN + j * 16 + 4 * fq + r;
            float v = red[c], q = red[BN + c];
#pragma unroll
            for (int h = 1; h < NWM; ++h) {
              v += red[h * 2 * BN + c];
              q += red[h * 2 * BN + BN + c];
            }
            mean[j][r] = v * inv_n;
            s[j][r] = fmaxf(q - v * mean[j][r], 0.f);
          }
      } else {
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        f32x2 t0 = {0.f, 0.f}, t1 = {0.f, 0.f};
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          f32x2 v0 = {acc[i][j][0], acc[i][j][1]}, v1 = {acc[i][j][2], acc[i][j][3]};
          if (!full && m0 + wm * WM + i * 16 + fr >= a.M) v0 = v1 = f32x2{0.f, 0.f};
          t0 += v0;
          t1 += v1;
        }
        s[j][0] = row16_sum(t0.x); s[j][1] = row16_sum(t0.y);
        s[j][2] = row16_sum(t1.x); s[j][3] = row16_sum(t1.y);
      }
      lds_barrier();   // the coalesced store path's last reads of the staging LDS are done
      exchange(true);
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) mean[j][r] = s[j][r] * inv_n;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const f32x2 mu0 = {mean[j][0], mean[j][1]}, mu1 = {mean[j][2], mean[j][3]};
        f32x2 t0 = {0.f, 0.f}, t1 = {0.f, 0.f};
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          f32x2 d0 = f32x2{acc[i][j][0], acc[i][j][1]} - mu0;
          f32x2 d1 = f32x2{acc[i][j][2], acc[i][j][3]} - mu1;
          if (!full && m0 + wm * WM + i * 16 + fr >= a.M) d0 = d1 = f32x2{0.f, 0.f};
          t0 = __builtin_elementwise_fma(d0, d0, t0);
          t1 = __builtin_elementwise_fma(d1, d1, t1);
        }
        s[j][0] = row16_sum(t0.x); s[j][1] = row16_sum(t0.y);
        s[j][2] = row16_sum(t1.x); s[j][3] = row16_sum(t1.y);
      }
      exchange(false);
      }
      if (a.bn_acc == nullptr) {
        if (wm == 0 && fr == 0) {
#pragma unroll
          for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int c = wn * WN + j * 16 + 4 * fq + r;
              a.part[(size_t)mt * 2 * a.Cout + n0 + c] = mean[j][r];
              a.part[(size_t)mt * 2 * a.Cout + a.Cout + n0 + c] = s[j][r];
            }
        }
      } else {
        bn_acc_epilogue<BM, BN, NT>(a, mt, n0, nrows, [&](auto&& add) {
          if (wm == 0 && fr == 0) {
#pragma unroll
            for (int j = 0; j < NI; ++j)
#pragma unroll
              for (int r = 0; r < 4; ++r) add(wn * WN + j * 16 + 4 * fq + r, mean[j][r], s[j][r]);
          }
        });
      }
    }
  }
}

template <int BM, int BN, int EPI, int NBUF, bool C16>
__global__ __launch_bounds__(kThreads) void conv_fwd_kernel(ConvArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)   // the body uses device-only builtins
  conv_fwd_body<BM, BN, EPI, NBUF, 2, 2, C16>(a);
#endif
}

// Single stage buffer (one K step -- 1x1 over 64 channels -- or the serial variants 8..11): the
// shapes that want it are bound by streaming the output, so it trades registers for occupancy --
// four waves per SIMD (<= 128 VGPRs) instead of two, up to five blocks per CU by LDS.
template <int BM, int BN, int EPI, bool C16>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4)))
void conv_fwd_kernel_occ4(ConvArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)   // the body uses device-only builtins
  conv_fwd_body<BM, BN, EPI, 1, 2, 2, C16>(a);
#endif
}

// 256-row tiles on 8 waves (4 x 2, per-wave 64 x BN/2): twice the MFMA work of a 128-row tile per
// staged weight byte, 2 waves per SIMD at one block per CU (96 KB of LDS double-buffered, 144 KB
// triple-buffered at BN = 128).
template <int BM, int BN, int EPI, int NBUF>
__global__ __launch_bounds__(512) void conv_fwd_kernel_w8(ConvArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)   // the body uses device-only builtins
  conv_fwd_body<BM, BN, EPI, NBUF, 4, 2, false>(a);
#endif
}

template <int BM, int BN>
hipError_t launch_w8(const ConvArgs& a0, int nb, hipStream_t st) {
  ConvArgs a = a0;
  if (a.c16) return hipErrorInvalidValue;
  a.m_tiles = (a.M + BM - 1) / BM;
  a.n_tiles = a.Cout / BN;
  const int nwg = a.m_tiles * a.n_tiles * a.ksplit;
  if (a.Ktot == kBK) nb = 1;
  const int epi = (a.part == nullptr && a.bn_acc == nullptr) ? 0 : (a.bnx != nullptr ? 2 : 1);
#define ARENA_CONV_W8(E) \
  do { if (nb == 1) hipLaunchKernelGGL((conv_fwd_kernel_w8<BM, BN, E, 1>), dim3(nwg), dim3(512), 0, st, a); \
       else if (nb == 2) hipLaunchKernelGGL((conv_fwd_kernel_w8<BM, BN, E, 2>), dim3(nwg), dim3(512), 0, st, a); \
       else hipLaunchKernelGGL((conv_fwd_kernel_w8<BM, BN, E, 3>), dim3(nwg), dim3(512), 0, st, a); } while (0)
  if (epi == 0) ARENA_CONV_W8(0);
  else if (epi == 1) ARENA_CONV_W8(1);
  else ARENA_CONV_W8(2);
#undef ARENA_CONV_W8
  return hipGetLastError();
}

template <int BM, int BN, bool C16>
hipError_t launch_t(const ConvArgs& a0, int pipe, hipStream_t st) {
  ConvArgs a = a0;
  a.m_tiles = (a.M + BM - 1) / BM;
  a.n_tiles = a.Cout / BN;
  const int nwg = a.m_tiles * a.n_tiles * a.ksplit;
  // stage buffers: pipe 0 (variants 0..3) two, pipe 1 (4..7) three, pipe 2 (8..11) one (serial,
  // high occupancy); a single K step always one
  const int nb = a.Ktot == kBK || pipe == 2 ? 1 : (pipe == 1 ? 4 : 2);
  const int epi = (a.part == nullptr && a.bn_acc == nullptr) ? 0 : (a.bnx != nullptr ? 2 : 1);
#define ARENA_CONV_LAUNCH(E, NB) \
  hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, E, NB, C16>), dim3(nwg), dim3(kThreads), 0, st, a)
#define ARENA_CONV_NB(E) \
  do { if (nb == 1 && (E == 0 || BM * BN < 128 * 128)) /* fits 128 VGPRs without spills */ \
         hipLaunchKernelGGL((conv_fwd_kernel_occ4<BM, BN, E, C16>), dim3(nwg), dim3(kThreads), 0, st, a); \
       else if (nb == 1) ARENA_CONV_LAUNCH(E, 1); \
       else if (nb == 2) ARENA_CONV_LAUNCH(E, 2); \
       else ARENA_CONV_LAUNCH(E, 4); } while (0)
  if (epi == 0) ARENA_CONV_NB(0);
  else if (epi == 1) ARENA_CONV_NB(1);
  else if constexpr (!C16) ARENA_CONV_NB(2);
  else return hipErrorInvalidValue;
#undef ARENA_CONV_NB
#undef ARENA_CONV_LAUNCH
  return hipGetLastError();
}

// ================================================================================================
// Tile kernel v2 (variant codes 4096 + i): 32x32x16 MFMAs on 256-row tiles, a deeper LDS-DMA
// pipeline, and an epilogue that works on an fp32 copy of the output tile in LDS.
//
// Why (docs/perf.md "Where the ResNet-50 step stands"): the v1 kernel issues 16x16x32 MFMAs on
// 128x128 tiles and stages 32 KB per 2 MFLOP. v2 stages (256 + BN) rows per 64-deep K step --
// 48 KB per 4.2 MFLOP at 256x128 -- and its 32x32x16 MFMA reads half the LDS bytes per FLOP of
// the 16x16x32 one (per wave and k16 step MI + NI fragments of 1 KB feed MI * NI MFMAs of
// 32 K-FLOP). With NBUF = 3 two K steps are in flight across each barrier (counted vmcnt, raw
// s_barrier: __syncthreads() would drain the LDS-DMA, cdna_hip_programming.md §5).
//
// Operands are staged exactly as in v1 (descriptor-based buffer_load ... lds, 128-byte rows with
// the chunk ^ ((row >> 1) & 7) swizzle, which also makes the 32x32 fragment reads conflict-free:
// every 16-lane ds_read_b128 group covers 16 distinct (row & 1, (row >> 1) & 7) pairs).
//
// The MFMA runs as W-fragment x X-fragment: D[row = channel][col = pixel], so lane l, register r
// holds pixel (l & 31) and channel 8 (r >> 2) + 4 (l >> 5) + (r & 3) of its 32x32 block. The
// epilogue writes those to an fp32 [row][channel] tile in LDS (16-byte slots, slot ^ (row & 7):
// conflict-free ds_write_b128), then every feature reads the tile in a layout of its own:
// coalesced 16-byte bf16 stores (+ optional masked addend, the residual join), and the BatchNorm
// statistics (EPI 1) as column sums over the tile's valid rows -- per-tile partials (mean, M2) or
// fp64 acc-mode atomics, the formats the v1 kernel emits. Tiles that do not fit LDS at once are
// processed in bands of one wave-row (EH = WM rows), statistics merged across bands (Chan).
// Mapped outputs (strided dgrad phases, incl. fill_sib) are stored by the plain epilogue. EPI 2
// (BN-backward partials of a dgrad output) rides on the coalesced store loop: each thread owns one
// 8-channel column chunk, so g and g * (x - mean) accumulate in registers across its rows/bands.
// Not covered (v1 handles them): c16 and split-K.
// ================================================================================================
typedef float f32x16v __attribute__((ext_vector_type(16)));

constexpr int kLdsMax = 160 * 1024;

// HALO (3x3, stride 1, pad 1, W <= kHaloMaxW): the A operand of a BM-pixel tile is the window of
// input pixels [m0 - W - 1, m0 + BM + W] (NHW-linear), staged ONCE per 64-channel chunk; the nine
// taps read it at row offsets r*W + s, and taps that fall outside the image (row/column padding or
// a neighbouring image) are zeroed on the fragment. A is staged once instead of nine times.
constexpr int kHaloMaxW = 63;
constexpr int kHaloSmallW = 31;   // HALO & 3 == 2: a window sized for <= 31-wide images
// HALO & 4: two window buffers -- chunk cb + 1's window is staged while chunk cb's taps run, and
// the weight ring runs on across chunk boundaries (no pipeline drain per 64-channel chunk)
constexpr int kHaloWin2 = 4;
// HALO & 8: two groups of four waves (512 threads, two waves per SIMD) split the 64-channel chunks
// by parity, each with its own window and weight ring and the whole BM x BN tile in its
// accumulators; at the end group 1 hands its sums to group 0 through LDS and exits, and group 0
// runs the epilogue. With one wave per SIMD the MFMA pipe idles whenever the wave waits on an LDS
// read or a barrier; the partner wave fills those gaps (needs an even chunk count).
constexpr int kHaloSplit2 = 8;

template <int BM, int BN, int NWM, int NWN, int NBUF, int EPI, bool BAND = false,
          int HALO = 0>
struct Conv2Geo {
  static constexpr int kBM = BM, kBN = BN;
  static constexpr int NT = 64 * NWM * NWN;
  static constexpr int WM = BM / NWM, WN = BN / NWN;
  static constexpr int MI = WM / 32, NI = WN / 32;
  static constexpr int AI = BM * 8 / NT, BI = BN * 8 / NT;
  static constexpr int kBufBytes = (BM + BN) * kRowBytes;
  // window rows (max W: kHaloMaxW, or kHaloSmallW for HALO & 3 == 2)
  static constexpr int kHaloRows = BM + 2 * ((HALO & 3) == 2 ? kHaloSmallW : kHaloMaxW) + 2;
  static constexpr int AIH = (kHaloRows * 8 + NT - 1) / NT;  // window loads per thread
  static constexpr int kWinBytes = AIH * NT / 8 * kRowBytes;
  static constexpr int kWins = (HALO & kHaloWin2) ? 2 : 1;
  static constexpr int kGroups = (HALO & kHaloSplit2) ? 2 : 1;
  // HALO: per wave group the window(s) + a ring of NBUF per-tap weight buffers (NBUF - 1 taps in
  // flight)
  static constexpr int kGroupStage = kWins * kWinBytes + NBUF * BN * kRowBytes;
  static constexpr int kStage = HALO ? kGroups * kGroupStage : NBUF * kBufBytes;
  static constexpr int SL = BN / 4;       // float4 slots per tile row
  static constexpr int RG = NT / SL;      // row groups of the statistics passes
  static constexpr int kRed = 0;   // EPI 1's partials reuse the band's tile (2 RG rows)
  // rows per epilogue band: the whole tile when it fits, else one wave-row; BAND forces the
  // wave-row bands to keep the block's LDS small (the high-occupancy serial variants)
  static constexpr int EH = !BAND && BM * BN * 4 + kRed <= kLdsMax - 1024 ? BM : WM;
  static constexpr int kEpi = EH * BN * 4 + kRed;
  static constexpr int kLds = kStage > kEpi ? kStage : kEpi;
  static_assert(MI >= 1 && NI >= 1 && AI >= 1 && BI >= 1, "tile too small for the wave grid");
  static_assert(AI * NT == BM * 8 && BI * NT == BN * 8, "staging slots must cover the tile");
  static_assert(SL >= 8 && NT % SL == 0, "epilogue layout");
  static_assert(EPI != 1 || 2 * RG <= EH, "EPI 1 partials fit the band's tile");
  static_assert(kLds <= kLdsMax, "LDS budget");
};

// s_waitcnt vmcnt(k * BI) lgkmcnt(0) for a k that is a constant after unrolling (the "n" operand
// needs a constant expression, so the cases are spelled out; the switch folds to one of them)
template <int BI>
__device__ __forceinline__ void vm_wait_groups(int k) {
  switch (k) {
    case 0: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(1 * BI) : "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * BI) : "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(3 * BI) : "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(4 * BI) : "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(5 * BI) : "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(6 * BI) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(7 * BI) : "memory"); break;
  }
}

// The v2 epilogue: the accumulators through an fp32 LDS tile at `lds` (EH x BN floats, bands of
// EH rows), coalesced bf16 stores (+ addend, mapped placement, fill_sib), and the EPI 1 / EPI 2
// BatchNorm sums (their partials reuse the tile).
template <class G, int EPI>
__device__ __forceinline__ void conv2_epilogue(const ConvArgs& a,
                                               f32x16v (&acc)[G::MI][G::NI], uint8_t* lds,
                                               int m0, int n0, int mt, int tid, int wm, int wn,
                                               int fr, int hh) {
  constexpr int BM = G::kBM, BN = G::kBN, NT = G::NT, WM = G::WM, WN = G::WN;
  constexpr int MI = G::MI, NI = G::NI, SL = G::SL, RG = G::RG, EH = G::EH;
  // ---- epilogue through the fp32 LDS tile (the stage buffers are free: the loop ended on a
  // barrier after every wave's last read) ----
  float* tile = reinterpret_cast<float*>(lds);
  constexpr int CPR = BN / 8;           // 16-byte bf16 output chunks per row
  if constexpr (EPI == 1) {
    // statistics of the stored (bf16-rounded) values: round once, the stores re-round exactly
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const uint32_t u = pack_bf16x2(acc[i][j][r], acc[i][j][r + 1]);
          acc[i][j][r] = __uint_as_float(u << 16);
          acc[i][j][r + 1] = __uint_as_float(u & 0xffff0000u);
        }
  }
  float st_n = 0.f, st_mean = 0.f, st_m2 = 0.f;   // running statistics of channel tid (< BN)
  // EPI 2: this thread's 8 channels (n0 + (tid % CPR) * 8 + e: the store loop below keeps a
  // thread on one 16-byte column chunk) -- sum g and sum g * (x - mean) over its rows
  float e1[EPI == 2 ? 8 : 1], e2[EPI == 2 ? 8 : 1], emu[EPI == 2 ? 8 : 1];
  if constexpr (EPI == 2) {
    static_assert(NT % CPR == 0, "EPI 2: a thread's column chunk is fixed");
    const float* mp = a.bnmean + n0 + (tid % CPR) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      e1[e] = 0.f;
      e2[e] = 0.f;
      emu[e] = mp[e];
    }
  }
#pragma unroll
  for (int band = 0; band < BM / EH; ++band) {
    if (band > 0) lds_barrier();   // every reader of the previous band is done
    if (EH == BM || wm == band) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = wm * WM + i * 32 + fr - band * EH;
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int slot = (wn * WN + j * 32 + 8 * g + 4 * hh) >> 2;
            *reinterpret_cast<f32x4v*>(tile + (row * SL + (slot ^ (row & 7))) * 4) =
                f32x4v{acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2],
                       acc[i][j][4 * g + 3]};
          }
      }
    }
    lds_barrier();
    const int rbase = m0 + band * EH;
    const int nvalid = min(EH, a.M - rbase);
    // coalesced stores: consecutive lanes on consecutive 16-byte chunks of a row
    for (int qq = tid; qq < EH * CPR; qq += NT) {
      const int row = qq / CPR, cc = qq - row * CPR;
      if (row >= nvalid) break;
      const f32x4v lo = *reinterpret_cast<const f32x4v*>(tile + (row * SL + ((2 * cc) ^ (row & 7))) * 4);
      const f32x4v hi = *reinterpret_cast<const f32x4v*>(tile + (row * SL + ((2 * cc + 1) ^ (row & 7))) * 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      size_t pix = (size_t)(rbase + row);
      int n = 0, ho = 0, wo = 0;
      if (EPI == 0 && a.mapped) {   // a strided-dgrad phase: scatter into the full dX image
        const int m = rbase + row, hw = a.Ho * a.Wo;
        n = m / hw;
        const int rem = m - n * hw;
        ho = rem / a.Wo;
        wo = rem - ho * a.Wo;
        pix = ((size_t)n * a.Hy + ho * a.osh + a.ooh) * a.Wy + wo * a.osw + a.oow;
      }
      const size_t off = pix * a.Cout + n0 + cc * 8;
      uint4 bxq;
      uint32_t bmk = 0xffu;
      if constexpr (EPI == 2) {   // the BN layer's input and ReLU bits at the same pixel/channels
        bxq = *reinterpret_cast<const uint4*>(a.bnx + off);
        if (a.bnmask)
          bmk = a.bnmask[(size_t)(rbase + row) * (a.Cout >> 3) + (n0 >> 3) + cc];
      }
      if (EPI != 1 && a.add != nullptr) {
        const uint4 qa = masked_add8(a.add, a.addmask, off);
        const uint32_t u[4] = {qa.x, qa.y, qa.z, qa.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] += __uint_as_float(u[e] << 16);
          v[2 * e + 1] += __uint_as_float(u[e] & 0xffff0000u);
        }
      }
      const uint4 yq = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                  pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
      *reinterpret_cast<uint4*>(a.y + off) = yq;
      if constexpr (EPI == 2) {
        // g = the stored dY (bf16) where the BN output's ReLU passed it
        const uint32_t yu[4] = {yq.x, yq.y, yq.z, yq.w}, xu[4] = {bxq.x, bxq.y, bxq.z, bxq.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float glo = (bmk >> (2 * e)) & 1u ? __uint_as_float(yu[e] << 16) : 0.f;
          const float ghi = (bmk >> (2 * e + 1)) & 1u ? __uint_as_float(yu[e] & 0xffff0000u) : 0.f;
          e1[2 * e] += glo;
          e1[2 * e + 1] += ghi;
          e2[2 * e] = fmaf(glo, __uint_as_float(xu[e] << 16) - emu[2 * e], e2[2 * e]);
          e2[2 * e + 1] =
              fmaf(ghi, __uint_as_float(xu[e] & 0xffff0000u) - emu[2 * e + 1], e2[2 * e + 1]);
        }
      }
      if (EPI == 0 && a.fill_sib) {   // 1x1 stride-2 dgrad: the tapless pixels get add (or 0)
        for (int da = 0; da < a.osh; ++da) {
          const int hy = ho * a.osh + da;
          if (hy >= a.Hy) break;
          for (int db = 0; db < a.osw; ++db) {
            const int wy = wo * a.osw + db;
            if ((da == 0 && db == 0) || wy >= a.Wy) continue;
            const size_t so = (((size_t)n * a.Hy + hy) * a.Wy + wy) * a.Cout + n0 + cc * 8;
            *reinterpret_cast<uint4*>(a.y + so) =
                a.add ? masked_add8(a.add, a.addmask, so) : make_uint4(0u, 0u, 0u, 0u);
          }
        }
      }
    }
    if constexpr (EPI == 1) {
      if (nvalid > 0) {
        // one pass over the band's valid rows, shifted by the band's first row k (the same shift
        // for every thread of a channel): thread = (row group, slot) sums d = x - k and d^2; the
        // band's mean is k + s / n and its M2 = q - s^2 / n. The partials then overwrite the
        // tile (every read of it is done), so EPI 1 needs no LDS of its own.
        const int sl = tid % SL, rg = tid / SL;
        const f32x4v k4 = *reinterpret_cast<const f32x4v*>(tile + sl * 4);   // row 0, slot sl
        const float kc = tid < BN ? tile[tid] : 0.f;                         // channel tid's k
        f32x4v s4 = {0.f, 0.f, 0.f, 0.f}, q4 = {0.f, 0.f, 0.f, 0.f};
        for (int row = rg; row < nvalid; row += RG) {
          const f32x4v d = *reinterpret_cast<const f32x4v*>(tile + (row * SL + (sl ^ (row & 7))) * 4) - k4;
          s4 += d;
          q4 += d * d;
        }
        lds_barrier();   // every thread is done reading the band: its tile takes the partials
        *reinterpret_cast<f32x4v*>(tile + rg * BN + sl * 4) = s4;
        *reinterpret_cast<f32x4v*>(tile + (RG + rg) * BN + sl * 4) = q4;
        lds_barrier();
        if (tid < BN) {
          float sd = 0.f, m2 = 0.f;
#pragma unroll 8
          for (int g2 = 0; g2 < RG; ++g2) {
            sd += tile[g2 * BN + tid];
            m2 += tile[(RG + g2) * BN + tid];
          }
          const float nb = (float)nvalid;
          const float bmean = kc + sd / nb;
          m2 = fmaxf(m2 - sd * sd / nb, 0.f);
          if (st_n == 0.f) {
            st_n = nb; st_mean = bmean; st_m2 = m2;
          } else {   // Chan's merge of two bands
            const float ntot = st_n + nb, d = bmean - st_mean;
            st_mean += d * nb / ntot;
            st_m2 += m2 + d * d * st_n * nb / ntot;
            st_n = ntot;
          }
        }
      }
    }
  }
  if constexpr (EPI == 2) {
    // per-tile BN-backward partials (bn_bwd_reduce's format, rpb = BM): the RG2 row groups'
    // sums reduced through the (free) epilogue tile, one quantity at a time
    constexpr int RG2 = NT / CPR;
    static_assert(EH >= RG2, "EPI 2 reduction fits the epilogue tile");
    const int cc = tid % CPR, rg = tid / CPR;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      lds_barrier();   // every reader of the last band (or of the previous quantity) is done
      float* dst = tile + rg * BN + cc * 8;
      const float* src = q == 0 ? e1 : e2;
      *reinterpret_cast<f32x4v*>(dst) = f32x4v{src[0], src[1], src[2], src[3]};
      *reinterpret_cast<f32x4v*>(dst + 4) = f32x4v{src[4], src[5], src[6], src[7]};
      lds_barrier();
      if (tid < BN) {
        float sum = 0.f;
#pragma unroll
        for (int g2 = 0; g2 < RG2; ++g2) sum += tile[g2 * BN + tid];
        if (a.bn_acc != nullptr)   // acc mode: the BN layer's fp64 backward sums
          unsafeAtomicAdd(acc_replica(a, mt) + q * a.Cout + n0 + tid, (double)sum);
        else
          a.part[(size_t)mt * 2 * a.Cout + q * a.Cout + n0 + tid] = sum;
      }
    }
  }
  if constexpr (EPI == 1) {
    if (tid < BN) {
      const int c = n0 + tid;
      if (a.bn_acc == nullptr) {
        a.part[(size_t)mt * 2 * a.Cout + c] = st_mean;
        a.part[(size_t)mt * 2 * a.Cout + a.Cout + c] = st_m2;
      } else {
        const double n = (double)st_n, mu = (double)st_mean;
        double* acc = acc_replica(a, mt);
        unsafeAtomicAdd(acc + c, n * mu);                                 // sum y
        unsafeAtomicAdd(acc + a.Cout + c, (double)st_m2 + n * mu * mu);   // sum y^2
      }
    }
  }
}

template <int BM, int BN, int NWM, int NWN, int NBUF, int EPI, bool BAND = false,
          int HALO = 0>
__device__ __forceinline__ void conv2_body(const ConvArgs& a, int bid) {
  using G = Conv2Geo<BM, BN, NWM, NWN, NBUF, EPI, BAND, HALO>;
  constexpr int NT = G::NT, WM = G::WM, WN = G::WN, MI = G::MI, NI = G::NI;
  constexpr int AI = G::AI, BI = G::BI, kBufBytes = G::kBufBytes;
  constexpr int SL = G::SL, RG = G::RG, EH = G::EH;
  __shared__ __attribute__((aligned(16))) uint8_t lds[G::kLds];

  // kHaloSplit2: wave group grp = threadIdx.x / 256, each group laid out as a 4-wave block
  constexpr int kGroups = HALO ? G::kGroups : 1;
  const int grp = kGroups == 2 ? (int)(threadIdx.x >> 8) : 0;
  const int tid = kGroups == 2 ? (int)(threadIdx.x & 255) : (int)threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  // XCD-aware order (as v1): each XCD gets a contiguous range of tiles, column tiles of one row
  // tile consecutive (their A rows stay in that XCD's L2)
  const int nblk = a.m_tiles * a.n_tiles;
  const int xcd = bid & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int nt = tile % a.n_tiles, mt = tile / a.n_tiles;
  const int n0 = nt * BN, m0 = mt * BM;

  f32x16v acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int wm = wave / NWN, wn = wave % NWN;
  const int fr = lane & 31, hh = lane >> 5;

  // ---- staging descriptors (v1's descriptor form): slot s = (wave*AI + i)*64 + lane -> LDS row
  // s / 8, chunk position s % 8 = lane % 8 ----
  const int pos = lane & 7;
  constexpr uint32_t kOOB = 0x80000000u;
  const __amdgpu_buffer_rsrc_t xrsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.wbytes, 0x00020000);
  if constexpr (HALO) {
    // ---- window staging: row j of the window = input pixel org + j (zero outside [0, M)) ----
    constexpr int AIH = G::AIH, kWin = G::kWinBytes;
    const int Wd = a.W;
    const int WR = BM + 2 * Wd + 2;
    const int org = m0 - Wd - 1;
    uint32_t w_off[AIH];
#pragma unroll
    for (int i = 0; i < AIH; ++i) {
      const int j = (wave * AIH + i) * 8 + (lane >> 3);
      const int pix = org + j;
      w_off[i] = (j < WR && pix >= 0 && pix < a.M)
                     ? (uint32_t)(((size_t)pix * a.C + (pos ^ swz(j)) * 8) * 2)
                     : kOOB;
    }
    uint32_t b_voff[BI];
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int row = (wave * BI + i) * 8 + (lane >> 3);
      b_voff[i] = (uint32_t)(((n0 + row) * a.Ktot + (pos ^ swz(row)) * 8) * 2);
    }
    // in-image taps of this lane's fragment rows: bit r*3 + s
    uint32_t tmask[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * WM + i * 32 + fr;
      uint32_t mk = 0u;
      if (m < a.M) {
        const int hw = a.Ho * a.Wo;
        const int n = m / hw, rem = m - n * hw;
        const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int s2 = 0; s2 < 3; ++s2)
            if ((unsigned)(ho + r - 1) < (unsigned)a.H && (unsigned)(wo + s2 - 1) < (unsigned)Wd)
              mk |= 1u << (r * 3 + s2);
      }
      tmask[i] = mk;
    }
    constexpr int kWins = G::kWins;
    uint8_t* const gbase = lds + grp * G::kGroupStage;   // this wave group's buffers
    uint8_t* const ring = gbase + kWins * kWin;
    auto stage_win = [&](int cb, int wb) {
#pragma unroll
      for (int i = 0; i < AIH; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            xrsrc, (lds_ptr_t)(gbase + wb * kWin + (wave * AIH + i) * 64 * 16), 16, w_off[i],
            cb * kRowBytes, 0, 0);
    };
    // the group's chunk sequence: cb = kGroups * j + grp
    // the weights of the group's global tap g = 9 j + tap into ring buffer g % NBUF
    auto stage_w = [&](int g) {
      const int jj = g / 9, tap = g - 9 * jj;
      const int cb = kGroups * jj + grp;
      uint8_t* bb = ring + (g % NBUF) * BN * kRowBytes;
#pragma unroll
      for (int i = 0; i < BI; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wrsrc, (lds_ptr_t)(bb + (wave * BI + i) * 64 * 16),
                                                 16, b_voff[i], (tap * a.C + cb * kBK) * 2, 0, 0);
    };
    auto compute_tap = [&](int tap, const uint8_t* win, int buf) {
      const int r = tap / 3, s2 = tap - 3 * r;
      const int shift = r * Wd + s2;
      const uint8_t* bbuf = ring + buf * BN * kRowBytes;
      bool ok[MI];
#pragma unroll
      for (int i = 0; i < MI; ++i) ok[i] = (tmask[i] >> tap) & 1u;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        bf16x8 af[MI], bfr[NI];
        const int c = kk * 2 + hh;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int j = wm * WM + i * 32 + fr + shift;
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(win + j * kRowBytes + ((c ^ swz(j)) << 4));
          af[i] = ok[i] ? v : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
#pragma unroll
        for (int jn = 0; jn < NI; ++jn) {
          const int row = wn * WN + jn * 32 + fr;
          bfr[jn] = *reinterpret_cast<const bf16x8*>(bbuf + row * kRowBytes + ((c ^ swz(row)) << 4));
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int jn = 0; jn < NI; ++jn)
            acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[jn], af[i], acc[i][jn], 0, 0, 0);
      }
    };
    // ---- K loop over the 9 CB global taps g = 9 cb + tap: the weights run D = NBUF - 1 taps
    // ahead in a ring of NBUF buffers, across chunk boundaries. Window: one buffer (restaged at
    // each chunk start, after the barrier that ended the previous chunk's last tap), or two
    // (kHaloWin2: chunk cb + 1's window issued at chunk cb's first tap, into the buffer chunk
    // cb - 1 used). Only loads are in flight, in issue order, so every counted vmcnt is exact:
    // before tap g + 1 the loads younger than its weights W(g + 1) are W(g + 2 .. g + D) and, for
    // the first D taps of a chunk with two windows, the next chunk's window. ----
    constexpr int D = NBUF - 1;
    static_assert(D >= 1 && D < 9, "weight ring depth");
    const int CB = a.C / kBK / kGroups;   // this group's chunks (host-checked: C / 64 divisible)
    const int T = 9 * CB;
    const int dbg = a.dbg;
    stage_win(grp, 0);
#pragma unroll
    for (int d = 0; d < D; ++d) stage_w(d);   // T >= 9 > D
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * BI) : "memory");   // window 0 + tap 0
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int cb = 0; cb < CB; ++cb) {
      const bool last = cb == CB - 1;
      const int wb = kWins == 2 ? (cb & 1) : 0;
      if (kWins == 1 && cb > 0) {
        // the previous chunk's last tap ended on a barrier: the window is free. Its loads are the
        // youngest, so waiting for them drains the (older, mostly landed) weights too.
        if (!(dbg & 2)) stage_win(kGroups * cb + grp, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      const uint8_t* win = gbase + wb * kWin;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int g = 9 * cb + t;
        // buffer (g + D) % NBUF was last read by tap g - 1, before the barrier that ended it
        if (g + D < T && !(dbg & 1)) stage_w(g + D);
        if (kWins == 2 && t == 0 && !last && !(dbg & 2))   // (its buffer: chunk cb - 1's, done)
          stage_win(kGroups * (cb + 1) + grp, wb ^ 1);
        if (!(dbg & 8)) compute_tap(t, win, g % NBUF);
        // (t is a constant of the unrolled loop: every branch below folds to one s_waitcnt)
        if (!last) {
          // W(g + 1) landed (with two windows and t == 8, the older next-chunk window too)
          if (kWins == 2 && t + 1 <= D)
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((D - 1) * BI + AIH) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((D - 1) * BI) : "memory");
        } else {
          // last chunk: W(g + 2 .. min(g + D, T - 1)) may stay in flight
          vm_wait_groups<BI>(t < 8 ? ((D - 1) < (7 - t) ? (D - 1) : (7 - t)) : 0);
        }
        if (!(dbg & 4)) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
    }
    if constexpr (kGroups == 2) {
      // group 1 hands its sums to group 0 through LDS (the stage buffers are free: the loop ended
      // on a barrier after every wave's last read), 16-byte lane-contiguous slots, the same
      // fragment layout in both groups; fixed order (group 0 + group 1): bit-reproducible
      float4* xs = reinterpret_cast<float4*>(lds) + (size_t)wave * (MI * NI * 4) * 64 + lane;
      if (grp == 1) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q)
              xs[((i * NI + j) * 4 + q) * 64] =
                  make_float4(acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2],
                              acc[i][j][4 * q + 3]);
      }
      lds_barrier();
      // group 1 is done; a terminated wave no longer counts toward the workgroup's barriers, so
      // the epilogue's barriers synchronise group 0 alone
      if (grp == 1) return;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 v = xs[((i * NI + j) * 4 + q) * 64];
            acc[i][j][4 * q] += v.x;
            acc[i][j][4 * q + 1] += v.y;
            acc[i][j][4 * q + 2] += v.z;
            acc[i][j][4 * q + 3] += v.w;
          }
      lds_barrier();   // every read of the hand-off is done before the epilogue reuses the LDS
    }
  } else {
    int a_lane[AI];
    uint32_t a_mask[AI], a_cur[AI], b_voff[BI];
  #pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int row = (wave * AI + i) * 8 + (lane >> 3);
      const int m = m0 + row;
      uint32_t mk = 0u;
      int off = 0;
      if (m < a.M) {
        const int hw = a.Ho * a.Wo;
        const int n = m / hw, rem = m - n * hw;
        const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
        const int hb = ho * a.stride - a.pad, wb = wo * a.stride - a.pad_w;
        for (int r = 0; r < a.R; ++r) {
          if ((unsigned)(hb + r) >= (unsigned)a.H) continue;
          for (int s2 = 0; s2 < a.S; ++s2)
            if ((unsigned)(wb + s2) < (unsigned)a.W) mk |= 1u << (r * a.S + s2);
        }
        off = (((n * a.H + hb) * a.W + wb) * a.C + (pos ^ swz(row)) * 8) * 2;
      }
      a_lane[i] = off;
      a_mask[i] = mk;
    }
  #pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int row = (wave * BI + i) * 8 + (lane >> 3);
      b_voff[i] = (uint32_t)(((n0 + row) * a.Ktot + (pos ^ swz(row)) * 8) * 2);
    }
    const int CB = a.C / kBK;
    // staging cursor: tap (r, s) sits (r*W + s)*C elements from tap 0
    const int T = a.Ktot / kBK;
    int s_tap = 0, s_cb = 0, s_s = 0, s_t = 0;
    int s_tapoff = 0;
  #pragma unroll
    for (int i = 0; i < AI; ++i)
      a_cur[i] = ((a_mask[i] >> s_tap) & 1u) ? (uint32_t)(a_lane[i] + s_tapoff) : kOOB;

    auto stage = [&](int buf) {
      uint8_t* base = lds + buf * kBufBytes;
      const int coff = s_cb * kRowBytes;
  #pragma unroll
      for (int i = 0; i < AI; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, (lds_ptr_t)(base + (wave * AI + i) * 64 * 16),
                                                 16, a_cur[i], coff, 0, 0);
      uint8_t* bb = base + BM * kRowBytes;
  #pragma unroll
      for (int i = 0; i < BI; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wrsrc, (lds_ptr_t)(bb + (wave * BI + i) * 64 * 16),
                                                 16, b_voff[i], s_t * kRowBytes, 0, 0);
      ++s_t;
      if (++s_cb == CB) {
        s_cb = 0;
        ++s_tap;
        s_tapoff += a.C * 2;
        if (++s_s == a.S) {
          s_s = 0;
          s_tapoff += (a.W - a.S) * a.C * 2;
        }
  #pragma unroll
        for (int i = 0; i < AI; ++i)
          a_cur[i] = ((a_mask[i] >> s_tap) & 1u) ? (uint32_t)(a_lane[i] + s_tapoff) : kOOB;
      }
    };


    auto compute = [&](int buf) {
      const uint8_t* abuf = lds + buf * kBufBytes;
      const uint8_t* bbuf = abuf + BM * kRowBytes;
  #pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        bf16x8 af[MI], bfr[NI];
        const int c = kk * 2 + hh;   // 16-byte chunk of this lane's 8 k values
  #pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int row = wm * WM + i * 32 + fr;
          af[i] = *reinterpret_cast<const bf16x8*>(abuf + row * kRowBytes + ((c ^ swz(row)) << 4));
        }
  #pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int row = wn * WN + j * 32 + fr;
          bfr[j] = *reinterpret_cast<const bf16x8*>(bbuf + row * kRowBytes + ((c ^ swz(row)) << 4));
        }
  #pragma unroll
        for (int i = 0; i < MI; ++i)
  #pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
    };

    // ---- K loop: S = NBUF - 1 steps in flight ----
    if constexpr (NBUF == 1) {
      // serial form (high occupancy: several blocks per CU overlap each other's staging)
      if (T > 0) stage(0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int t = 0; t < T; ++t) {
        compute(0);
        if (t + 1 < T) {
          __syncthreads();   // every wave is done reading the buffer: restage it
          stage(0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    } else {
      constexpr int S = NBUF - 1;
      constexpr int kLps = AI + BI;   // LDS-DMA instructions per thread per stage
  #pragma unroll
      for (int i = 0; i < S; ++i)
        if (i < T) stage(i);
      if (T >= S)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((S - 1) * kLps) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      int cur = 0;
      for (int t = 0; t < T; ++t) {
        // RAW: stage t + 1 was retired by the vmcnt before the last barrier. WAR: stage t + S
        // overwrites buffer (t - 1) % NBUF, whose reads completed before that barrier.
        if (t + S < T) stage(cur == 0 ? NBUF - 1 : cur - 1);
        compute(cur);
        if (t + S < T)
          asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((S - 1) * kLps) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        cur = cur == NBUF - 1 ? 0 : cur + 1;
      }
    }
  }

  conv2_epilogue<G, EPI>(a, acc, lds, m0, n0, mt, tid, wm, wn, fr, hh);
}

// The multi-phase launch: this block's phase, its arguments and its block index within it
// (false: a padding block past the phase's tiles, which exits before any barrier).
template <int BM>
__device__ __forceinline__ bool conv2_phase(const ConvArgs& a, ConvArgs& b, int& bid) {
  int p = 0;
  while (p + 1 < a.nph && (int)blockIdx.x >= a.ph[p + 1].blk0) ++p;
  const ConvArgs::Phase& ph = a.ph[p];
  b = a;
  b.w = ph.w;
  b.R = ph.R; b.S = ph.S; b.pad = ph.pad; b.pad_w = ph.pad_w;
  b.Ho = ph.Ho; b.Wo = ph.Wo; b.ooh = ph.ooh; b.oow = ph.oow; b.wbytes = ph.wbytes;
  b.M = a.N * ph.Ho * ph.Wo;
  b.Ktot = ph.R * ph.S * a.C;
  b.m_tiles = (b.M + BM - 1) / BM;
  bid = (int)blockIdx.x - ph.blk0;
  return bid < b.m_tiles * b.n_tiles;
}

template <int BM, int BN, int NWM, int NWN, int NBUF, int EPI>
__global__ __launch_bounds__(64 * NWM * NWN) void conv2_kernel(ConvArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)   // the body uses device-only builtins
  if constexpr (EPI == 0) {
    if (a.nph > 0) {
      ConvArgs b;
      int bid;
      if (conv2_phase<BM>(a, b, bid)) conv2_body<BM, BN, NWM, NWN, NBUF, EPI>(b, bid);
      return;
    }
  }
  conv2_body<BM, BN, NWM, NWN, NBUF, EPI>(a, blockIdx.x);
#endif
}

// serial, wave-row epilogue bands, <= 128 VGPRs: four waves per SIMD (up to four 4-wave blocks
// per CU by LDS), the structure that wins the streaming-bound layers in v1 (variants 8..11)
// (EPI 2 on the 128x128 tile: three waves per SIMD -- its 24 extra live registers spill at four)
template <int BM, int BN, int EPI>
__global__ __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(EPI == 2 && BM * BN >= 128 * 128 ? 3 : 4)))
void conv2_kernel_occ4(ConvArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (EPI == 0) {
    if (a.nph > 0) {
      ConvArgs b;
      int bid;
      if (conv2_phase<BM>(a, b, bid)) conv2_body<BM, BN, 2, 2, 1, EPI, true>(b, bid);
      return;
    }
  }
  conv2_body<BM, BN, 2, 2, 1, EPI, true>(a, blockIdx.x);
#endif
}

// the 3x3 halo form (see Conv2Geo::HALO): 4 waves, a ring of NBR per-tap weight buffers --
// 128x128: three (80 KB, two blocks per CU); 128x64: two (48 KB, three blocks per CU; with the
// small window of <= 31-wide images 40 KB, four blocks per CU)
template <int BM, int BN, int EPI, int HW, int NB, int NWM = 2, int NWN = 2>
__global__ __launch_bounds__((HW & kHaloSplit2) ? 512 : 64 * NWM * NWN)
void conv2_kernel_halo(ConvArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  conv2_body<BM, BN, NWM, NWN, NB, EPI, false, HW>(a, blockIdx.x);
#endif
}

// HW: window size class (1: <= 63 wide, 2: <= 31) | kHaloWin2; NB: weight ring buffers; NWM x NWN
// waves (8-wave forms: a 256-pixel or 256-channel tile per block, so each weight tap staged into
// LDS feeds twice the MFMAs of a 128x128 tile)
template <int BM, int BN, int HW, int NB, int NWM = 2, int NWN = 2>
hipError_t launch2_halo(const ConvArgs& a0, hipStream_t st) {
  ConvArgs a = a0;
  if (a.c16 || a.Cout % BN || a.R != 3 || a.S != 3 ||
      a.stride != 1 || a.pad != 1 || a.pad_w != 1 || a.Ho != a.H || a.Wo != a.W ||
      a.W > ((HW & 3) == 2 ? kHaloSmallW : kHaloMaxW) || a.mapped ||
      ((HW & kHaloSplit2) && (a.C / kBK) % 2))
    return hipErrorInvalidValue;
  const int nthr = (HW & kHaloSplit2) ? 512 : 64 * NWM * NWN;
  if (a.ksplit != 1) return hipErrorInvalidValue;
  if (a.bnx == nullptr && (a.part != nullptr || a.bn_acc != nullptr) && a.add != nullptr)
    return hipErrorInvalidValue;
  a.m_tiles = (a.M + BM - 1) / BM;
  a.n_tiles = a.Cout / BN;
  const int nwg = a.m_tiles * a.n_tiles;
  if (a.bnx != nullptr)
    hipLaunchKernelGGL((conv2_kernel_halo<BM, BN, 2, HW, NB, NWM, NWN>), dim3(nwg), dim3(nthr), 0,
                       st, a);
  else if (a.part != nullptr || a.bn_acc != nullptr)
    hipLaunchKernelGGL((conv2_kernel_halo<BM, BN, 1, HW, NB, NWM, NWN>), dim3(nwg), dim3(nthr), 0,
                       st, a);
  else
    hipLaunchKernelGGL((conv2_kernel_halo<BM, BN, 0, HW, NB, NWM, NWN>), dim3(nwg), dim3(nthr), 0,
                       st, a);
  return hipGetLastError();
}

template <int BM, int BN, int NWM, int NWN, int NBUF, bool OCC4 = false>
hipError_t launch2_t(const ConvArgs& a0, hipStream_t st) {
  ConvArgs a = a0;
  if (a.c16 || a.Cout % BN) return hipErrorInvalidValue;
  if (a.ksplit != 1) return hipErrorInvalidValue;   // split-K: the v1 tiles only
  const bool bwd_bn = a.bnx != nullptr;   // EPI 2 (the caller checked part / bnmean / no map)
  if (!bwd_bn && (a.part != nullptr || a.bn_acc != nullptr) && (a.add != nullptr || a.mapped))
    return hipErrorInvalidValue;
  a.m_tiles = (a.M + BM - 1) / BM;
  a.n_tiles = a.Cout / BN;
  int nwg = a.m_tiles * a.n_tiles;
  const bool stats = a.part != nullptr || a.bn_acc != nullptr;
  if (a.nph > 0) {   // phases back to back, each starting on a multiple of 8 blocks
    if (stats || bwd_bn) return hipErrorInvalidValue;
    int b0 = 0;
    for (int p = 0; p < a.nph; ++p) {
      a.ph[p].blk0 = b0;
      const long long mp = (long long)a.N * a.ph[p].Ho * a.ph[p].Wo;
      b0 += ((int)((mp + BM - 1) / BM) * a.n_tiles + 7) / 8 * 8;
    }
    nwg = b0;
  }
  if constexpr (OCC4) {
    if (bwd_bn)
      hipLaunchKernelGGL((conv2_kernel_occ4<BM, BN, 2>), dim3(nwg), dim3(256), 0, st, a);
    else if (stats)
      hipLaunchKernelGGL((conv2_kernel_occ4<BM, BN, 1>), dim3(nwg), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((conv2_kernel_occ4<BM, BN, 0>), dim3(nwg), dim3(256), 0, st, a);
  } else if (bwd_bn) {
    hipLaunchKernelGGL((conv2_kernel<BM, BN, NWM, NWN, NBUF, 2>), dim3(nwg),
                       dim3(64 * NWM * NWN), 0, st, a);
  } else if (stats) {
    hipLaunchKernelGGL((conv2_kernel<BM, BN, NWM, NWN, NBUF, 1>), dim3(nwg),
                       dim3(64 * NWM * NWN), 0, st, a);
  } else {
    hipLaunchKernelGGL((conv2_kernel<BM, BN, NWM, NWN, NBUF, 0>), dim3(nwg),
                       dim3(64 * NWM * NWN), 0, st, a);
  }
  return hipGetLastError();
}

// v2 variant table (code 1024 + index): BM x BN tile, waves NWM x NWN, stage buffers
constexpr int kV2Base = 4096;   // above every v1 code (base + 16 (k - 1), split-K k <= 16)
constexpr int kV2Count = 19;
constexpr int kV2Tiles[kV2Count][2] = {{256, 128}, {256, 256}, {128, 128}, {256, 64}, {128, 256},
                                       {128, 64}, {64, 64}, {64, 128},
                                       {128, 128}, {128, 64}, {64, 128}, {64, 64},
                                       {128, 128}, {128, 64}, {128, 64},
                                       {128, 128},
                                       {256, 128}, {128, 256}, {256, 64}};

hipError_t launch2(const ConvArgs& a, int idx, hipStream_t st) {
  switch (idx) {
    case 0: return launch2_t<256, 128, 4, 2, 3>(a, st);
    case 1: return launch2_t<256, 256, 2, 4, 2>(a, st);
    case 2: return launch2_t<128, 128, 2, 2, 2>(a, st);
    case 3: return launch2_t<256, 64, 4, 2, 3>(a, st);
    case 4: return launch2_t<128, 256, 2, 4, 3>(a, st);
    // 4-wave small tiles: several blocks per CU (48 / 32 / 48 KB of LDS) for the 64-channel
    // layers, where the 8-wave 256-row tiles leave each SIMD with two waves to hide latency
    case 5: return launch2_t<128, 64, 2, 2, 2>(a, st);
    case 6: return launch2_t<64, 64, 2, 2, 2>(a, st);
    case 7: return launch2_t<64, 128, 2, 2, 2>(a, st);
    // serial high-occupancy forms of the 4-wave tiles (conv2_kernel_occ4)
    case 8: return launch2_t<128, 128, 2, 2, 1, true>(a, st);
    case 9: return launch2_t<128, 64, 2, 2, 1, true>(a, st);
    case 10: return launch2_t<64, 128, 2, 2, 1, true>(a, st);
    case 11: return launch2_t<64, 64, 2, 2, 1, true>(a, st);
    // 3x3 / stride 1 / pad 1 halo forms (conv2_kernel_halo); LDS per block in comments
    case 12: return launch2_halo<128, 128, 1, 3>(a, st);   // 80 KB
    case 13: return launch2_halo<128, 64, 1, 2>(a, st);    // 48 KB
    case 14: return launch2_halo<128, 64, 2, 2>(a, st);    // <= 31 wide: 40 KB, 4 blocks per CU
    // two wave groups splitting the channel chunks (512 threads, two waves per SIMD): 144 KB.
    // Measured and not kept (profiles/r6_halo_variants.jsonl): 128x128 with two groups and two
    // ring buffers, 128x64 with two groups, four- and six-deep rings, a second window buffer.
    case 15: return launch2_halo<128, 128, 2 | kHaloSplit2, 3>(a, st);
    // 8-wave halo forms (one block per CU, two waves per SIMD): the L2 -> LDS weight stream is
    // what bounds the 4-wave forms (16 KB per tap per 128x128 block ~ 30 B/clk per CU at full MFMA
    // rate, the measured L2 -> LDS rate; MI355X_MICROARCH.md "gather into LDS"). A 256-pixel or
    // 256-channel block halves the weight bytes per MFMA.
    case 16: return launch2_halo<256, 128, 1, 3, 4, 2>(a, st);   // 128 KB (epilogue tile)
    case 17: return launch2_halo<128, 256, 1, 3, 2, 4>(a, st);   // 128 KB
    case 18: return launch2_halo<256, 64, 1, 3, 4, 2>(a, st);    // 72 KB, two blocks per CU
    // (a four-buffer ring on 16 / 18, three taps in flight, measured no faster:
    // profiles/r6_halo_wide_ring4.jsonl)
    default: return hipErrorInvalidValue;
  }
}

// the stem's c16 form only exists for 64-wide tiles (its Cout is 64)
template <int BM, int BN>
hipError_t launch(const ConvArgs& a, int pipe, hipStream_t st) {
  if (a.c16) {
    if constexpr (BN == 64) return launch_t<BM, BN, true>(a, pipe, st);
    else return hipErrorInvalidValue;
  }
  return launch_t<BM, BN, false>(a, pipe, st);
}

}  // namespace

int g_conv_st1p = 0;   // see ConvArgs::st1p (runtime switch: arena_conv_set_stats_one_pass)

extern "C" {

void arena_conv_set_stats_one_pass(int on) { g_conv_st1p = on ? 1 : 0; }

int g_conv_dbg = 0;   // ConvArgs::dbg (timing ablations only)
void arena_conv_set_dbg(int bits) { g_conv_dbg = bits; }

// Returns hipErrorInvalidValue for shapes the kernel does not cover (the caller falls back to
// MIOpen): C % 64 != 0, Cout % 64 != 0, or an unknown tile variant.
// variant: 0 = 128x128, 1 = 128x64, 2 = 64x128, 3 = 64x64 (BM x BN output tile per block);
// variant + 4: the same tile with a four-stage K pipeline (three glds steps in flight);
// variant + 8: one stage buffer, serial K loop, high occupancy (streaming-bound 1x1 shapes).
// 12 / 13: 256x128 / 256x64 on 8 waves, two stage buffers; 14 / 15: the same, three.
// part (optional): BatchNorm partials of y, [ceil(M / BM)][2][Cout] (EPI 1 / EPI 2 epilogues).
// General form. pad_h/pad_w: top/left padding; Ho/Wo: output size (<= 0: derived from a symmetric
// padding); y_map {Hy, Wy, osh, osw, ooh, oow, fill_sib} (null: dense output); c16, fill_sib:
// see ConvArgs.
// bnx/bnmask/bnmean (optional, with part): the backward-data form, part = BatchNorm-backward
// partials of y instead of forward statistics (see ConvArgs).
// bn_acc (optional, instead of part): accumulated BatchNorm statistics, see ConvArgs::bn_acc;
// [2][Cout] doubles, zero on entry (the BN layer that consumes them zeroes them again).
hipError_t arena_conv_fwd_ex(const void* x, const void* w, void* y, float* part, const void* add,
                             const uint8_t* addmask,
                             const void* bnx, const uint8_t* bnmask, const float* bnmean, int N,
                             int H, int W, int C, int Cout, int R, int S, int stride, int pad_h,
                             int pad_w, int Ho, int Wo, const int* y_map, int c16, int variant,
                             double* bn_acc, int ksplit, void* kws, unsigned* kcnt,
                             hipStream_t st) {
  if (Cout % 64 || N <= 0 || R <= 0 || S <= 0 || stride <= 0) return hipErrorInvalidValue;
  if (c16 ? (C != 16 || S % 4) : (C % kBK)) return hipErrorInvalidValue;
  ConvArgs a{};
  a.x = (const uint16_t*)x;
  a.w = (const uint16_t*)w;
  a.y = (uint16_t*)y;
  a.part = part;
  a.add = (const uint16_t*)add;
  a.addmask = add != nullptr ? addmask : nullptr;
  if (addmask != nullptr && Cout % 8) return hipErrorInvalidValue;
  a.bnx = (const uint16_t*)bnx;
  a.bnmask = bnmask;
  a.bnmean = bnmean;
  if (bnx != nullptr &&
      ((part == nullptr) == (bn_acc == nullptr) || bnmean == nullptr || y_map != nullptr))
    return hipErrorInvalidValue;
  // forward statistics are taken from the accumulators before the epilogue adds an addend
  if (part != nullptr && bnx == nullptr && add != nullptr) return hipErrorInvalidValue;
  if (bn_acc != nullptr) {   // forward statistics without an addend, or the EPI 2 sums
    if (part != nullptr || (bnx == nullptr && add != nullptr)) return hipErrorInvalidValue;
    a.bn_acc = bn_acc;
  }
  a.N = N; a.H = H; a.W = W; a.C = C; a.Cout = Cout; a.R = R; a.S = S;
  a.stride = stride; a.pad = pad_h; a.pad_w = pad_w;
  a.Ho = Ho > 0 ? Ho : (H + 2 * pad_h - R) / stride + 1;
  a.Wo = Wo > 0 ? Wo : (W + 2 * pad_w - S) / stride + 1;
  if (a.Ho <= 0 || a.Wo <= 0) return hipErrorInvalidValue;
  a.c16 = c16;
  static const int coal = [] {
    const char* e = getenv("ARENA_CONV_COAL");
    return e == nullptr || e[0] != '0' ? 1 : 0;
  }();
  a.coal = coal;
  if (y_map != nullptr) {
    a.mapped = 1;
    a.Hy = y_map[0]; a.Wy = y_map[1]; a.osh = y_map[2]; a.osw = y_map[3];
    a.ooh = y_map[4]; a.oow = y_map[5]; a.fill_sib = y_map[6];
    if (a.fill_sib && (a.ooh || a.oow || a.Ho != (a.Hy + a.osh - 1) / a.osh ||
                       a.Wo != (a.Wy + a.osw - 1) / a.osw))
      return hipErrorInvalidValue;
    // every mapped output pixel inside the [Hy][Wy] image (the caller checked the sizes too)
    if ((a.Ho - 1) * a.osh + a.ooh >= a.Hy || (a.Wo - 1) * a.osw + a.oow >= a.Wy || a.ooh < 0 ||
        a.oow < 0 || a.osh <= 0 || a.osw <= 0)
      return hipErrorInvalidValue;
  }
  const long long M = (long long)N * a.Ho * a.Wo;
  if (M >= (1LL << 31) || (long long)N * H * W * C >= (1LL << 40)) return hipErrorInvalidValue;
  a.M = (int)M;
  a.Ktot = R * S * C;
  const bool v2 = variant >= kV2Base && variant < kV2Base + kV2Count;
  if (!v2 && (variant < 0 || variant > 15)) return hipErrorInvalidValue;
  if (!c16) {   // descriptor staging: 31-bit byte offsets, a 32-bit tap mask
    const long long xb = (long long)N * H * W * C * 2, wb = (long long)Cout * a.Ktot * 2;
    if (xb >= (1LL << 31) || wb >= (1LL << 31) || R * S > 32) return hipErrorInvalidValue;
    a.xbytes = (int)xb;
    a.wbytes = (int)wb;
  }
  // split-K: every slice gets at least one K step; the caller sized kws with
  // arena_conv_fwd_ksplit_floats and zeroed kcnt once (the kernel re-zeroes what it uses)
  if (ksplit < 1 || ksplit > a.Ktot / kBK || (ksplit > 1 && (kws == nullptr || kcnt == nullptr)))
    return hipErrorInvalidValue;
  a.ksplit = ksplit;
  a.kws = (float4*)kws;
  a.kcnt = kcnt;
  a.st1p = g_conv_st1p;
  a.dbg = g_conv_dbg;
  if (v2) {
    if (c16) return hipErrorInvalidValue;
    return launch2(a, variant - kV2Base, st);
  }
  if (variant >= 12) {   // 256-row tiles, 8 waves: 12/13 two stage buffers, 14/15 three
    const int nb = variant >= 14 ? 3 : 2;
    if ((variant & 1) == 0)
      return Cout % 128 ? hipErrorInvalidValue : launch_w8<256, 128>(a, nb, st);
    return launch_w8<256, 64>(a, nb, st);
  }
  const int pipe = variant >> 2;
  switch (variant & 3) {
    case 0: return Cout % 128 ? hipErrorInvalidValue : launch<128, 128>(a, pipe, st);
    case 1: return launch<128, 64>(a, pipe, st);
    case 2: return Cout % 128 ? hipErrorInvalidValue : launch<64, 128>(a, pipe, st);
    case 3: return launch<64, 64>(a, pipe, st);
    default: return hipErrorInvalidValue;
  }
}

// All phase convolutions of a strided backward-data pass in one launch of v2 tile `variant`
// (kV2Base + i, not the halo forms): x = dY [N][H][W][C], phase p's weights w[p]
// [Cout][R[p]][S[p]][C] with top/left padding pad_h/pad_w[p] over a Ho[p] x Wo[p] phase grid,
// stored at (ho*osh + ooh[p], wo*osw + oow[p]) of y [N][Hy][Wy][Cout] (+ add, same shape; add may
// alias y). nph <= 4.
hipError_t arena_conv_fwd_phases(const void* x, void* y, const void* add, int N, int H, int W,
                                 int C, int Cout, int Hy, int Wy, int osh, int osw, int nph,
                                 const void* const* w, const int* R, const int* S,
                                 const int* pad_h, const int* pad_w, const int* Ho, const int* Wo,
                                 const int* ooh, const int* oow, int variant, hipStream_t st) {
  const int idx = variant - kV2Base;
  if (idx < 0 || idx >= 12 || nph < 1 || nph > 4 || C % kBK || Cout % 64 || N <= 0)
    return hipErrorInvalidValue;
  ConvArgs a{};
  a.x = (const uint16_t*)x;
  a.y = (uint16_t*)y;
  a.add = (const uint16_t*)add;
  a.N = N; a.H = H; a.W = W; a.C = C; a.Cout = Cout; a.stride = 1;
  a.mapped = 1; a.Hy = Hy; a.Wy = Wy; a.osh = osh; a.osw = osw;
  a.coal = 1;
  a.ksplit = 1;
  const long long xb = (long long)N * H * W * C * 2;
  if (xb >= (1LL << 31) || osh <= 0 || osw <= 0) return hipErrorInvalidValue;
  a.xbytes = (int)xb;
  a.nph = nph;
  for (int p = 0; p < nph; ++p) {
    ConvArgs::Phase& ph = a.ph[p];
    ph.w = (const uint16_t*)w[p];
    ph.R = R[p]; ph.S = S[p]; ph.pad = pad_h[p]; ph.pad_w = pad_w[p];
    ph.Ho = Ho[p]; ph.Wo = Wo[p]; ph.ooh = ooh[p]; ph.oow = oow[p];
    const long long wb = (long long)Cout * R[p] * S[p] * C * 2;
    if (wb >= (1LL << 31) || R[p] * S[p] > 32 || R[p] <= 0 || S[p] <= 0 || Ho[p] <= 0 ||
        Wo[p] <= 0 || ooh[p] < 0 || oow[p] < 0 || (Ho[p] - 1) * osh + ooh[p] >= Hy ||
        (Wo[p] - 1) * osw + oow[p] >= Wy || (long long)N * Ho[p] * Wo[p] >= (1LL << 31))
      return hipErrorInvalidValue;
    ph.wbytes = (int)wb;
  }
  // the single-convolution fields stay consistent with phase 0 (launch2_t's checks read them)
  a.w = a.ph[0].w; a.R = R[0]; a.S = S[0]; a.pad = pad_h[0]; a.pad_w = pad_w[0];
  a.Ho = Ho[0]; a.Wo = Wo[0]; a.ooh = ooh[0]; a.oow = oow[0]; a.wbytes = a.ph[0].wbytes;
  a.M = N * Ho[0] * Wo[0];
  a.Ktot = R[0] * S[0] * C;
  a.st1p = g_conv_st1p;
  a.dbg = g_conv_dbg;
  return launch2(a, idx, st);
}

hipError_t arena_conv_fwd(const void* x, const void* w, void* y, float* part, const void* add,
                          const void* bnx, const uint8_t* bnmask, const float* bnmean,
                          int N, int H, int W, int C, int Cout, int R, int S, int stride, int pad,
                          int variant, hipStream_t st) {
  return arena_conv_fwd_ex(x, w, y, part, add, nullptr, bnx, bnmask, bnmean, N, H, W, C, Cout, R, S,
                           stride, pad, pad, 0, 0, nullptr, 0, variant, nullptr, 1, nullptr, nullptr,
                           st);
}

// Split-K workspace of one launch, in floats (0 when ksplit == 1), and its ticket count (tiles).
static void conv_tile(int variant, int* bm, int* bn) {
  static const int tm[4] = {128, 128, 64, 64}, tn[4] = {128, 64, 128, 64};
  if (variant >= kV2Base && variant < kV2Base + kV2Count) {
    *bm = kV2Tiles[variant - kV2Base][0];
    *bn = kV2Tiles[variant - kV2Base][1];
  } else if (variant >= 12) {
    *bm = 256;
    *bn = (variant & 1) ? 64 : 128;
  } else {
    *bm = tm[variant & 3];
    *bn = tn[variant & 3];
  }
}

long long arena_conv_fwd_ksplit_floats(long long M, int Cout, int variant, int ksplit) {
  if (ksplit <= 1 || variant < 0 || variant > 15) return 0;   // split-K: the v1 tiles only
  int bm, bn;
  conv_tile(variant, &bm, &bn);
  return ((M + bm - 1) / bm) * (Cout / bn) * ksplit * bm * bn;
}

long long arena_conv_fwd_tiles(long long M, int Cout, int variant) {
  if (variant < 0 || (variant > 15 && !(variant >= kV2Base && variant < kV2Base + kV2Count)))
    return 0;
  int bm, bn;
  conv_tile(variant, &bm, &bn);
  return ((M + bm - 1) / bm) * (Cout / bn);
}

int arena_conv_fwd_tile_rows(int variant) {
  int bm, bn;
  conv_tile(variant, &bm, &bn);
  return bm;
}

}  // extern "C"

// ================================================================================================
// The backward-data pass runs the forward kernel on W'[ci][r][s][co] = W[co][R-1-r][S-1-s][ci]
// (arena_amd/ops/conv.py). Per tap that is a transpose of the [Cout][C] slice: one 64x64 bf16 tile
// per block through LDS (a 2-byte pad per row keeps the column reads on distinct banks), 16-byte
// loads and stores. One launch instead of torch's flip + strided copy (two kernels per dgrad, and
// a memcpy for 1x1 weights).
// A stride-s backward-data pass splits into s*s phase convolutions (conv2d_bwd_data_strided), each
// with the flipped sub-filter of the taps r = r0 (mod s): one launch writes every phase's weights,
// packed phase after phase, from a per-tap table (blockIdx.z = destination tap).
// ================================================================================================
namespace {

constexpr int kMaxFlipTaps = 64;

struct FlipTaps {
  int src[kMaxFlipTaps];    // source tap r * S + s of W
  int dtap[kMaxFlipTaps];   // destination tap u * Sp + v within its phase
  int ntap[kMaxFlipTaps];   // Rp * Sp of that phase
  int off[kMaxFlipTaps];    // element offset of that phase's [C][Rp][Sp][Cout] block
};

__global__ __launch_bounds__(256) void conv_flip_weight_kernel(const uint16_t* __restrict__ w,
                                                               uint16_t* __restrict__ wt, int Cout,
                                                               int C, int RS, FlipTaps tp) {
  __shared__ uint16_t tile[64][64 + 2];
  const int ci0 = blockIdx.x * 64, co0 = blockIdx.y * 64, z = blockIdx.z;
  const int src_tap = tp.src[z], dtap = tp.dtap[z], ntap = tp.ntap[z];
  uint16_t* dst = wt + tp.off[z];
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; ++k) {   // 64 rows (co) x 8 chunks of 8 ci
    const int q = t + k * 256, row = q >> 3, ch = q & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(
        w + ((size_t)(co0 + row) * RS + src_tap) * C + ci0 + ch * 8);
    const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      tile[row][ch * 8 + 2 * e] = (uint16_t)(u[e] & 0xffffu);
      tile[row][ch * 8 + 2 * e + 1] = (uint16_t)(u[e] >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {   // 64 rows (ci) x 8 chunks of 8 co
    const int q = t + k * 256, row = q >> 3, ch = q & 7;
    uint32_t u[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      u[e] = (uint32_t)tile[ch * 8 + 2 * e][row] | ((uint32_t)tile[ch * 8 + 2 * e + 1][row] << 16);
    *reinterpret_cast<uint4*>(dst + ((size_t)(ci0 + row) * ntap + dtap) * Cout + co0 + ch * 8) =
        make_uint4(u[0], u[1], u[2], u[3]);
  }
}

// Many stride-1 flips in one launch (a ResNet step flips every stride-1 conv weight once, at the
// start of its forward: one launch instead of one per backward-data pass). Block b belongs to the
// tensor whose [start, next start) range holds b; within it, b -> (ci tile, co tile, tap).
constexpr int kMaxFlipTensors = 64;
struct FlipMulti {
  const uint16_t* src[kMaxFlipTensors];
  uint16_t* dst[kMaxFlipTensors];
  int cout[kMaxFlipTensors], cin[kMaxFlipTensors], rs[kMaxFlipTensors];
  int start[kMaxFlipTensors + 1];
  int n;
};

__global__ __launch_bounds__(256) void conv_flip_multi_kernel(FlipMulti fm) {
  __shared__ uint16_t tile[64][64 + 2];
  const int b = blockIdx.x;
  int k = 0;
  while (k + 1 < fm.n && b >= fm.start[k + 1]) ++k;   // <= 64 uniform scalar steps
  const int Cout = fm.cout[k], C = fm.cin[k], RS = fm.rs[k];
  int rem = b - fm.start[k];
  const int cit = C >> 6, cot = Cout >> 6;
  const int ci0 = (rem % cit) * 64;
  rem /= cit;
  const int co0 = (rem % cot) * 64, dtap = rem / cot, src_tap = RS - 1 - dtap;
  const uint16_t* w = fm.src[k];
  uint16_t* dst = fm.dst[k];
  const int t = threadIdx.x;
#pragma unroll
  for (int s = 0; s < 2; ++s) {   // 64 rows (co) x 8 chunks of 8 ci
    const int q = t + s * 256, row = q >> 3, ch = q & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(
        w + ((size_t)(co0 + row) * RS + src_tap) * C + ci0 + ch * 8);
    const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      tile[row][ch * 8 + 2 * e] = (uint16_t)(u[e] & 0xffffu);
      tile[row][ch * 8 + 2 * e + 1] = (uint16_t)(u[e] >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < 2; ++s) {   // 64 rows (ci) x 8 chunks of 8 co
    const int q = t + s * 256, row = q >> 3, ch = q & 7;
    uint32_t u[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      u[e] = (uint32_t)tile[ch * 8 + 2 * e][row] | ((uint32_t)tile[ch * 8 + 2 * e + 1][row] << 16);
    *reinterpret_cast<uint4*>(dst + ((size_t)(ci0 + row) * RS + dtap) * Cout + co0 + ch * 8) =
        make_uint4(u[0], u[1], u[2], u[3]);
  }
}

}  // namespace

extern "C" {

// W'[ci][r][s][co] = W[co][R-1-r][S-1-s][ci] for n weights in one launch (see conv_flip_multi_kernel).
// Every Cout and C a multiple of 64, R*S <= 64, n <= 64.
hipError_t arena_conv_flip_multi(int n, const void* const* src, void* const* dst, const int* cout,
                                 const int* cin, const int* rs, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (n > kMaxFlipTensors) return hipErrorInvalidValue;
  FlipMulti fm{};
  long long blocks = 0;
  for (int i = 0; i < n; ++i) {
    if (cout[i] % 64 || cin[i] % 64 || cout[i] <= 0 || cin[i] <= 0 || rs[i] <= 0 ||
        rs[i] > kMaxFlipTaps)
      return hipErrorInvalidValue;
    fm.src[i] = (const uint16_t*)src[i];
    fm.dst[i] = (uint16_t*)dst[i];
    fm.cout[i] = cout[i];
    fm.cin[i] = cin[i];
    fm.rs[i] = rs[i];
    fm.start[i] = (int)blocks;
    blocks += (long long)(cin[i] / 64) * (cout[i] / 64) * rs[i];
    if (blocks >= (1LL << 31)) return hipErrorInvalidValue;
  }
  fm.start[n] = (int)blocks;
  fm.n = n;
  hipLaunchKernelGGL(conv_flip_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, st, fm);
  return hipGetLastError();
}

// Phase weights of a stride-`stride`, top/left-`pad` convolution's backward-data pass, packed in
// phase order (a, b) = (0, 0), (0, 1), ... skipping phases without taps:
//   Wp[ci][u][v][co] = W[co][r0 + s*(Rp-1-u)][c0 + s*(Sp-1-v)][ci],  r0 = (a + pad) % s, ...
// stride 1 is the plain flip. Returns the number of elements written via *total (may be null).
hipError_t arena_conv_phase_weights(const void* w, void* wt, int Cout, int C, int R, int S,
                                    int stride, int pad, long long* total, hipStream_t st) {
  if (Cout % 64 || C % 64 || R <= 0 || S <= 0 || stride <= 0 || pad < 0)
    return hipErrorInvalidValue;
  FlipTaps tp{};
  int nz = 0;
  long long off = 0;
  for (int a = 0; a < stride; ++a) {
    const int r0 = (a + pad) % stride;
    if (r0 >= R) continue;
    const int Rp = (R - r0 + stride - 1) / stride;
    for (int b = 0; b < stride; ++b) {
      const int c0 = (b + pad) % stride;
      if (c0 >= S) continue;
      const int Sp = (S - c0 + stride - 1) / stride;
      if (nz + Rp * Sp > kMaxFlipTaps || off + (long long)C * Rp * Sp * Cout >= (1LL << 31))
        return hipErrorInvalidValue;
      for (int u = 0; u < Rp; ++u)
        for (int v = 0; v < Sp; ++v) {
          tp.src[nz] = (r0 + stride * (Rp - 1 - u)) * S + c0 + stride * (Sp - 1 - v);
          tp.dtap[nz] = u * Sp + v;
          tp.ntap[nz] = Rp * Sp;
          tp.off[nz] = (int)off;
          ++nz;
        }
      off += (long long)C * Rp * Sp * Cout;
    }
  }
  if (total != nullptr) *total = off;
  if (wt == nullptr) return hipSuccess;   // size query
  if (nz == 0) return hipSuccess;
  hipLaunchKernelGGL(conv_flip_weight_kernel, dim3(C / 64, Cout / 64, nz), dim3(256), 0, st,
                     (const uint16_t*)w, (uint16_t*)wt, Cout, C, R * S, tp);
  return hipGetLastError();
}

hipError_t arena_conv_flip_weight(const void* w, void* wt, int Cout, int C, int R, int S,
                                  hipStream_t st) {
  if (R * S > kMaxFlipTaps) return hipErrorInvalidValue;
  return arena_conv_phase_weights(w, wt, Cout, C, R, S, 1, 0, nullptr, st);
}

}  // extern "C"

// ================================================================================================
// Space-to-depth for the 7x7/2 stem: x [N][H][W][C] (C <= 4) -> z [N][H/2][W/2][16] with
// z[n][i][j][(dy*2 + dx)*C + c] = x[n][2i+dy][2j+dx][c] and channels 4C..15 zero. The stride-2
// 7x7 convolution over x is then a stride-1 4x4 convolution over z (arena_amd/ops/conv.py
// StemConv2d), which the MFMA kernel runs in its c16 mode.
// ================================================================================================
namespace {

// TIn = uint16_t (bf16) or float: an fp32 input batch is rounded to bf16 here, which under
// autocast replaces the separate cast pass over the whole batch (a 77 MB read + 38 MB write at
// ResNet-50 batch 128).
__device__ __forceinline__ uint16_t s2d_in(uint16_t v) { return v; }
__device__ __forceinline__ uint16_t s2d_in(float v) {
  const f32x2 p = {v, 0.f};
  return (uint16_t)(__builtin_bit_cast(uint32_t, __builtin_convertvector(p, bf16x2_t)) & 0xffffu);
}

// x's two pixels (2j, 2j+1) of one row are 2C contiguous elements, and in z they are channels
// dy*2C .. dy*2C + 2C-1: each thread copies two runs, as C 8-byte (fp32) or 4-byte (bf16) loads --
// both aligned because W is even. Index math in 32 bits when the pixel count allows (two 64-bit
// divisions per thread cost more than its loads).
template <typename TIn, int C, typename I>
__global__ __launch_bounds__(256) void s2d_stem_kernel(const TIn* __restrict__ x,
                                                       uint16_t* __restrict__ z, int N, int H,
                                                       int W) {
  const I Hz = (I)(H >> 1), Wz = (I)(W >> 1);
  const I p = (I)blockIdx.x * 256 + (I)threadIdx.x;
  if (p >= (I)N * Hz * Wz) return;
  const I t = p / Wz;
  const I j = p - t * Wz;
  const I n = t / Hz;
  const I i = t - n * Hz;
  uint16_t v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = 0;
#pragma unroll
  for (int dy = 0; dy < 2; ++dy) {
    const TIn* src = x + (((size_t)n * H + 2 * (size_t)i + dy) * W + 2 * (size_t)j) * C;
#pragma unroll
    for (int q = 0; q < C; ++q) {
      if constexpr (sizeof(TIn) == 4) {
        const float2 f = reinterpret_cast<const float2*>(src)[q];
        v[dy * 2 * C + 2 * q] = s2d_in(f.x);
        v[dy * 2 * C + 2 * q + 1] = s2d_in(f.y);
      } else {
        const uint32_t u = reinterpret_cast<const uint32_t*>(src)[q];
        v[dy * 2 * C + 2 * q] = (uint16_t)(u & 0xffffu);
        v[dy * 2 * C + 2 * q + 1] = (uint16_t)(u >> 16);
      }
    }
  }
  uint4 o0, o1;
  o0.x = v[0] | ((uint32_t)v[1] << 16); o0.y = v[2] | ((uint32_t)v[3] << 16);
  o0.z = v[4] | ((uint32_t)v[5] << 16); o0.w = v[6] | ((uint32_t)v[7] << 16);
  o1.x = v[8] | ((uint32_t)v[9] << 16); o1.y = v[10] | ((uint32_t)v[11] << 16);
  o1.z = v[12] | ((uint32_t)v[13] << 16); o1.w = v[14] | ((uint32_t)v[15] << 16);
  uint4* dst = reinterpret_cast<uint4*>(z + (size_t)p * 16);
  dst[0] = o0;
  dst[1] = o1;
}

// The stem weight in its space-to-depth form, one thread per W16 element (and its backward, one
// thread per W element: every W tap has exactly one W16 slot):
//   W16[co][u][v][(dy*2+dx)*C + c] = W[co][c][2u+dy-1][2v+dx-1]  (0 outside the 7x7 filter)
// W is [Cout][C][7][7] in any memory layout (element strides given), fp32 or bf16; W16 is the
// channels_last bf16 [Cout][16][4][4] the c16 conv reads, i.e. memory [co][u][v][16].
template <typename TW>
__global__ __launch_bounds__(256) void stem_weight_kernel(const TW* __restrict__ w,
                                                          uint16_t* __restrict__ w16, int Cout,
                                                          int C, long long sco, long long sc,
                                                          long long sr, long long ss) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= Cout * 256) return;
  const int ch = e & 15, v = (e >> 4) & 3, u = (e >> 6) & 3, co = e >> 8;
  float val = 0.f;
  if (ch < 4 * C) {
    const int d = ch / C, c = ch - d * C;
    const int r = 2 * u + (d >> 1) - 1, s = 2 * v + (d & 1) - 1;
    if (r >= 0 && r < 7 && s >= 0 && s < 7) {
      const TW q = w[co * sco + c * sc + r * sr + s * ss];
      if constexpr (sizeof(TW) == 2) val = __uint_as_float((uint32_t)q << 16);
      else val = q;
    }
  }
  const f32x2 pr = {val, 0.f};
  w16[e] = (uint16_t)(__builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2_t)) & 0xffffu);
}

// dW[co][c][r][s] = dW16 at W's slot; dW [Cout][C][7][7] with element strides (dco, dc, dr, ds),
// fp32 or bf16 (the parameter's own dtype and layout: no copy in autograd's accumulation)
template <typename TW>
__global__ __launch_bounds__(256) void stem_weight_grad_kernel(const uint16_t* __restrict__ dw16,
                                                               TW* __restrict__ dw, int Cout,
                                                               int C, long long dco, long long dc,
                                                               long long dr, long long ds) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= Cout * C * 49) return;
  const int s = e % 7, r = (e / 7) % 7, c = (e / 49) % C, co = e / (49 * C);
  const int u = (r + 1) >> 1, dy = (r + 1) & 1, v = (s + 1) >> 1, dx = (s + 1) & 1;
  const int ch = (dy * 2 + dx) * C + c;
  const uint16_t g = dw16[((co * 4 + u) * 4 + v) * 16 + ch];
  TW* o = dw + co * dco + c * dc + r * dr + s * ds;
  if constexpr (sizeof(TW) == 2) *o = g;
  else *o = __uint_as_float((uint32_t)g << 16);
}

}  // namespace

// in_f32: x is fp32 (rounded to bf16 on the way), else bf16
extern "C" hipError_t arena_s2d_stem(const void* x, void* z, int N, int H, int W, int C,
                                     int in_f32, hipStream_t st) {
  if (N <= 0 || H % 2 || W % 2 || C < 1 || C > 4) return hipErrorInvalidValue;
  const long long P = (long long)N * (H / 2) * (W / 2);
  const dim3 g((unsigned)((P + 255) / 256));
  const bool small = P < (1ll << 31);
#define S2D_LAUNCH(TIn, CC)                                                                    \
  do {                                                                                         \
    if (small)                                                                                 \
      hipLaunchKernelGGL((s2d_stem_kernel<TIn, CC, unsigned>), g, dim3(256), 0, st,            \
                         (const TIn*)x, (uint16_t*)z, N, H, W);                                \
    else                                                                                       \
      hipLaunchKernelGGL((s2d_stem_kernel<TIn, CC, long long>), g, dim3(256), 0, st,           \
                         (const TIn*)x, (uint16_t*)z, N, H, W);                                \
  } while (0)
#define S2D_C(TIn)                  \
  switch (C) {                      \
    case 1: S2D_LAUNCH(TIn, 1); break; \
    case 2: S2D_LAUNCH(TIn, 2); break; \
    case 3: S2D_LAUNCH(TIn, 3); break; \
    default: S2D_LAUNCH(TIn, 4); break; \
  }
  if (in_f32) S2D_C(float) else S2D_C(uint16_t)
#undef S2D_C
#undef S2D_LAUNCH
  return hipGetLastError();
}

// W [Cout][C][7][7] (element strides sco, sc, sr, ss; fp32 if w_f32 else bf16) -> W16
extern "C" hipError_t arena_stem_weight(const void* w, void* w16, int Cout, int C, long long sco,
                                        long long sc, long long sr, long long ss, int w_f32,
                                        hipStream_t st) {
  if (Cout <= 0 || C < 1 || C > 4) return hipErrorInvalidValue;
  const dim3 g((unsigned)((Cout * 256 + 255) / 256));
  if (w_f32)
    hipLaunchKernelGGL(stem_weight_kernel<float>, g, dim3(256), 0, st, (const float*)w,
                       (uint16_t*)w16, Cout, C, sco, sc, sr, ss);
  else
    hipLaunchKernelGGL(stem_weight_kernel<uint16_t>, g, dim3(256), 0, st, (const uint16_t*)w,
                       (uint16_t*)w16, Cout, C, sco, sc, sr, ss);
  return hipGetLastError();
}

extern "C" hipError_t arena_stem_weight_grad(const void* dw16, void* dw, int Cout, int C,
                                             long long dco, long long dc, long long dr,
                                             long long ds, int dw_f32, hipStream_t st) {
  if (Cout <= 0 || C < 1 || C > 4) return hipErrorInvalidValue;
  const dim3 g((unsigned)((Cout * C * 49 + 255) / 256));
  if (dw_f32)
    hipLaunchKernelGGL(stem_weight_grad_kernel<float>, g, dim3(256), 0, st,
                       (const uint16_t*)dw16, (float*)dw, Cout, C, dco, dc, dr, ds);
  else
    hipLaunchKernelGGL(stem_weight_grad_kernel<uint16_t>, g, dim3(256), 0, st,
                       (const uint16_t*)dw16, (uint16_t*)dw, Cout, C, dco, dc, dr, ds);
  return hipGetLastError();
}

// ================================================================================================
// Backward-weight: dW[co][r][s][ci] = sum_m dY[m][co] * X[pix(m, r, s)][ci]
//
// A GEMM of Cout rows, R*S*C columns and N*Ho*Wo (up to 400k) reduction steps, so the reduction
// is split over blocks: block (split, co-tile, k-tile) sums 64-pixel steps [split*SPS, ...) into
// an fp32 slab ws[split][Cout][R*S*C] with plain stores, and conv_wgrad_reduce sums the slabs in
// a fixed order (bit-reproducible, no float atomics: those run at ~1.3 TB/s, MI355X_MICROARCH.md).
//
// Both operands are reduction-strided (a pixel row holds 64..2048 consecutive channels), so the
// tiles are staged pixel-major ([64 pixels][BM or BN channels], glds, 16-byte chunks permuted per
// row) and the MFMA fragments are read with ds_read_b64_tr_b16, which hands each lane one channel
// of 4 consecutive pixels. The permutation moves 32-byte chunk pairs so that the 8 rows one
// 32-lane half of a transposed read touches sit in 8 distinct 32-byte bank slots.
// ================================================================================================
namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4* lds_s4_t;

struct FastDiv {  // n / d for 0 <= n < 2^31 (Granlund-Montgomery, 32-bit)
  uint32_t mul, shift, d;
};

__device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv f) {
  return (__umulhi(n, f.mul) + n) >> f.shift;
}

struct WgradArgs {
  const uint16_t* x;   // [N][H][W][C]
  const uint16_t* dy;  // [N][Ho][Wo][Cout]
  float* ws;           // [splits][Cout][Ktot]
  int N, H, W, C, Cout, R, S, stride, pad, Ho, Wo;
  int M, Ktot;
  int m_tiles, n_tiles, splits, sps;  // sps = 64-pixel steps per split
  FastDiv div_hw, div_w;
  int pad_w;           // left padding (pad is the top one)
  int c16;             // C == 16, a BN = 64 column tile = one filter row x 4 columns x 16 channels
  int xbytes, dybytes; // buffer-descriptor ranges (both < 2^31 bytes, host-checked)
  int aff;             // 1x1, stride 1, no padding: X pixel m is output pixel m (affine staging)
};

// chunk permutation of a pixel row of RB bytes (bit 0 of the chunk index is kept: 32-B pairs)
template <int RB>
__device__ __forceinline__ int wswz(int row) {
  if constexpr (RB == 256) return 2 * ((row & 3) | (((row >> 3) & 1) << 2));
  else return 2 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1));
}

// NBUF 2: double-buffered pixel steps; NBUF 1 (variants 4..7): one buffer, serial steps, four
// waves per SIMD -- more blocks per CU hide the staging latency instead (see conv_fwd_kernel_occ4).
template <int BM, int BN, int NBUF>
__device__ __forceinline__ void conv_wgrad_body(const WgradArgs& a) {
  constexpr int RA = BM * 2, RBB = BN * 2;        // row bytes of the A (dY) and B (X) images
  constexpr int CA = RA / 16, CB = RBB / 16;       // 16-byte chunks per row
  constexpr int kPix = 64;                         // pixels per step
  constexpr int AI = kPix * CA / kThreads, BI = kPix * CB / kThreads;
  constexpr int kBuf = kPix * (RA + RBB);
  constexpr int WM = BM / 2, WN = BN / 2, MI = WM / 16, NI = WN / 16;
  __shared__ __attribute__((aligned(16))) uint8_t lds[NBUF * kBuf];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles = a.m_tiles * a.n_tiles;
  const int nwg = tiles * a.splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  // split-major order: the blocks of one XCD share a pixel range (dY and X rows hit its L2)
  const int split = lin / tiles, t2 = lin - split * tiles;
  const int mt = t2 / a.n_tiles, nt = t2 - mt * a.n_tiles;
  const int co0 = mt * BM, kk0 = nt * BN;
  int tap, ci0, rr, ss;
  if (a.c16) {   // column tile nt = filter row rr, columns 4*sb .. 4*sb+3 (BN == 64, host-checked)
    const int SB = a.S >> 2;
    rr = nt / SB;
    ss = (nt - rr * SB) * 4;
    tap = 0;
    ci0 = 0;
  } else {
    tap = kk0 / a.C;
    ci0 = kk0 - tap * a.C;
    rr = tap / a.S;
    ss = tap - rr * a.S;
  }
  const int step0 = split * a.sps;
  const int nsteps = min(a.sps, (a.M + kPix - 1) / kPix - step0);

  // staging: wave-instruction i of this wave fills rows [(wave*I + i) * RPI, +RPI) of the image
  constexpr int RPI_A = 64 / CA, RPI_B = 64 / CB;  // rows per wave-instruction
  const int a_row_l = lane / CA, a_pos = lane % CA;
  const int b_row_l = lane / CB, b_pos = lane % CB;

  // Staging through buffer descriptors (see conv_fwd_body): a dY row is affine in the pixel
  // index, so its slot offset is fixed and the step moves the scalar soffset; rows past M get an
  // out-of-range offset (zeros). X rows are affine too for 1x1 stride-1 unpadded convolutions
  // (a.aff); otherwise the pixel is decomposed per slot and padded taps go out of range.
  constexpr uint32_t kOOB = 0x80000000u;
  const __amdgpu_buffer_rsrc_t dyr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, a.dybytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.xbytes, 0x00020000);
  uint32_t a_voff[AI], b_voff[BI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int row = (wave * AI + i) * RPI_A + a_row_l;
    a_voff[i] = (uint32_t)((row * a.Cout + co0 + (a_pos ^ wswz<RA>(row)) * 8) * 2);
  }
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int row = (wave * BI + i) * RPI_B + b_row_l;
    b_voff[i] = (uint32_t)((row * a.C + ci0 + (b_pos ^ wswz<RBB>(row)) * 8) * 2);
  }

  auto stage = [&](int step, int buf) {
    uint8_t* base = lds + buf * kBuf;
    const int p0 = (step0 + step) * kPix;
    const bool full = p0 + kPix <= a.M;   // no row of this step is past M (uniform)
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int row = (wave * AI + i) * RPI_A + a_row_l;
      const uint32_t vo = (full || p0 + row < a.M) ? a_voff[i] : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(dyr, (lds_ptr_t)(base + (wave * AI + i) * 1024), 16,
                                               vo, p0 * a.Cout * 2, 0, 0);
    }
    uint8_t* bb = base + kPix * RA;
    if (a.aff) {
#pragma unroll
      for (int i = 0; i < BI; ++i) {
        const int row = (wave * BI + i) * RPI_B + b_row_l;
        const uint32_t vo = (full || p0 + row < a.M) ? b_voff[i] : kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_ptr_t)(bb + (wave * BI + i) * 1024), 16,
                                                 vo, p0 * a.C * 2, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int row = (wave * BI + i) * RPI_B + b_row_l;
      const int m = p0 + row;
      uint32_t vo = kOOB;
      if (m < a.M) {
        const int n = (int)fdiv((uint32_t)m, a.div_hw);
        const int rem = m - n * a.Ho * a.Wo;
        const int ho = (int)fdiv((uint32_t)rem, a.div_w);
        const int wo = rem - ho * a.Wo;
        const int cch = b_pos ^ wswz<RBB>(row);   // this slot's global 16-byte chunk
        const int hi = ho * a.stride - a.pad + rr;
        const int wi = wo * a.stride - a.pad_w + ss + (a.c16 ? (cch >> 1) : 0);
        if ((unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W)
          vo = a.c16 ? (uint32_t)((((n * a.H + hi) * a.W + wi) * 16 + (cch & 1) * 8) * 2)
                     : (uint32_t)((((n * a.H + hi) * a.W + wi) * a.C + ci0 + cch * 8) * 2);
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_ptr_t)(bb + (wave * BI + i) * 1024), 16, vo,
                                               0, 0, 0);
    }
  };

  f32x4v acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;

  // BN fold: the X image of step `step` in buffer `buf` through relu(fma(x - mean, scale, shift));
  // thread = one logical chunk of rows tid / CB + k * kThreads / CB (one chunk's coefficients)

  if (nsteps > 0) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int t = 0; t < nsteps; ++t) {
    const int cur = NBUF == 1 ? 0 : (t & 1);
    if (NBUF == 2 && t + 1 < nsteps) stage(t + 1, cur ^ 1);
    const uint8_t* abuf = lds + cur * kBuf;
    const uint8_t* bbuf = abuf + kPix * RA;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = kk * 32 + 8 * g + 4 * h + qq;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int byte = 2 * (wm * WM + i * 16 + 4 * pp);
          const int off = row * RA + (((byte >> 4) ^ wswz<RA>(row)) << 4) + (byte & 15);
          const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t)(abuf + off));
          af[i][4 * h + 0] = v[0]; af[i][4 * h + 1] = v[1];
          af[i][4 * h + 2] = v[2]; af[i][4 * h + 3] = v[3];
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int byte = 2 * (wn * WN + j * 16 + 4 * pp);
          const int off = row * RBB + (((byte >> 4) ^ wswz<RBB>(row)) << 4) + (byte & 15);
          const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t)(bbuf + off));
          bfr[j][4 * h + 0] = v[0]; bfr[j][4 * h + 1] = v[1];
          bfr[j][4 * h + 2] = v[2]; bfr[j][4 * h + 3] = v[3];
        }
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (NBUF == 1 && t + 1 < nsteps) {   // serial: every wave is done with the buffer
      __syncthreads();
      stage(t + 1, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // lane holds D[co = .. + 4*g + reg][kk = .. + (lane & 15)]
  float* slab = a.ws + (size_t)split * a.Cout * a.Ktot;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int col = kk0 + wn * WN + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * WM + i * 16 + 4 * g + r;
        slab[(size_t)co * a.Ktot + col] = acc[i][j][r];
      }
    }
}

template <int BM, int BN>
__global__ __launch_bounds__(kThreads) void conv_wgrad_kernel(WgradArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)   // the body uses device-only builtins
  conv_wgrad_body<BM, BN, 2>(a);
#endif
}

template <int BM, int BN>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4)))
void conv_wgrad_kernel_occ4(WgradArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  conv_wgrad_body<BM, BN, 1>(a);
#endif
}

// out = sum over splits of ws, bf16 and/or fp32. Thread (col, grp) of a block sums float4 column
// blockIdx.x * 32 + col over splits grp, grp + 8, ... (8 float4 loads in flight), and the 8 groups
// are combined in LDS in a fixed order (bit-reproducible). Splitting the split dimension over the
// block's waves keeps a small dW (4096 floats for a 64x64 1x1 conv, summed over hundreds of slabs)
// from being a serial chain of dependent load batches (16 us per layer on average before).
// COLS x GROUPS = 256 threads. Small weights (a 64x64 1x1 conv has 1024 float4 columns) use the
// 8 x 32 shape: 32 blocks of the 32 x 8 shape left 224 CUs idle and each thread summed 64 slabs
// behind one another (7+ us per layer); 8 columns per block give 4x the blocks and a quarter of
// the chain. The sum order is fixed per shape (bit-reproducible).
constexpr int kRedU = 8;

template <int COLS, int GROUPS>
__global__ __launch_bounds__(256) void conv_wgrad_reduce_kernel(const float4* __restrict__ ws,
                                                                int splits, long long n4,
                                                                uint2* __restrict__ out_bf,
                                                                float4* __restrict__ out_f,
                                                                float scale) {
  static_assert(COLS * GROUPS == 256, "one block is 256 threads");
  const int col = threadIdx.x % COLS, grp = threadIdx.x / COLS;
  const long long i = (long long)blockIdx.x * COLS + col;
  const float4* src = ws + (i < n4 ? i : 0);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int k = grp;
  for (; k + (kRedU - 1) * GROUPS < splits; k += kRedU * GROUPS) {
    float4 v[kRedU];
#pragma unroll
    for (int u = 0; u < kRedU; ++u) v[u] = src[(long long)(k + u * GROUPS) * n4];
#pragma unroll
    for (int u = 0; u < kRedU; ++u) {
      acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
    }
  }
  for (; k < splits; k += GROUPS) {
    const float4 v = src[(long long)k * n4];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  __shared__ float4 red[GROUPS][COLS];
  red[grp][col] = acc;
  __syncthreads();
  if (grp != 0 || i >= n4) return;
  float4 s = red[0][col];
#pragma unroll
  for (int g = 1; g < GROUPS; ++g) {
    const float4 v = red[g][col];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  s.x *= scale; s.y *= scale; s.z *= scale; s.w *= scale;
  if (out_f) out_f[i] = s;
  if (out_bf) {
    uint2 b;
    b.x = pack_bf16x2(s.x, s.y);
    b.y = pack_bf16x2(s.z, s.w);
    out_bf[i] = b;
  }
}

FastDiv make_fastdiv(uint32_t d) {
  FastDiv f{};
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.shift = l;
  f.mul = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
  return f;
}

// ------------------------------------------------------------------------------------------------
// Backward-weight v2 (variants 8..11): 32x32x16 MFMAs on 128/256-wide tiles, two K steps... the
// same split-K slab scheme as v1, the same pixel-major staging by LDS-DMA, but the fragments of
// the 32x32x16 operands: lane l of a 16-lane group g needs channel l & 31 of pixels
// 8 (l >> 5) + 0..7, i.e. two ds_read_b64_tr_b16 per fragment whose 4-row x 16-column blocks are
// rows 8 (g >> 1) + 4 h + q and columns 16 (g & 1) + 4 p (lane 4q + p of the group). A 32-lane
// half then reads 4 pixel rows x 64 bytes, so the image permutes 64-byte granules per row
// (16-byte chunk c -> c ^ 4 (row & 3)): the 4 rows land on 4 distinct granules of the 256-byte
// bank row (rows need >= 256 bytes: tiles of >= 128 channels). The permutation is applied on the
// LDS-DMA source address and undone on the read, as everywhere in this file.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int wswz2(int row) { return 4 * (row & 3); }

// GRP > 1: GRP groups of NWM x NWN waves in one block split the block's pixel steps (group g takes
// steps t = g (mod GRP)) with their own stage buffers and a whole tile of accumulators each; at
// the end groups 1 .. GRP-1 hand their sums to group 0 through LDS in group order (fixed order:
// bit-reproducible) and exit, and group 0 writes the slab. A block then covers GRP times the
// pixels of a one-group block with the same waves per CU, so the launch needs 1 / GRP of the
// split slabs (fp32 [splits][Cout][Ktot], written here and read back by the reduce pass: 1.8 GB
// per ResNet-50 step at one group).
template <int BM, int BN, int NWM, int NWN, int NBUF, int GRP = 1>
__device__ __forceinline__ void conv_wgrad2_body(const WgradArgs& a) {
  constexpr int NT = 64 * NWM * NWN;
  constexpr int RA = BM * 2, RBB = BN * 2;        // row bytes of the dY and X images
  constexpr int CA = RA / 16, CB = RBB / 16;
  constexpr int kPix = 64;
  constexpr int AI = kPix * CA / NT, BI = kPix * CB / NT;
  constexpr int kBuf = kPix * (RA + RBB);
  constexpr int WM = BM / NWM, WN = BN / NWN, MI = WM / 32, NI = WN / 32;
  static_assert(CA >= 16 && CB >= 16, "the 64-byte granule permutation needs >= 256-byte rows");
  static_assert(AI >= 1 && BI >= 1 && MI >= 1 && NI >= 1, "tile too small for the wave grid");
  static_assert(AI * NT == kPix * CA && BI * NT == kPix * CB, "staging slots must cover the tile");
  constexpr int kHand = GRP > 1 ? NT * MI * NI * 16 * 4 : 0;   // one group's accumulators
  constexpr int kLdsW = GRP * NBUF * kBuf > kHand ? GRP * NBUF * kBuf : kHand;
  static_assert(kLdsW <= kLdsMax, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint8_t lds_all[kLdsW];

  const int grp = GRP > 1 ? (int)(threadIdx.x / NT) : 0;
  const int tid = GRP > 1 ? (int)(threadIdx.x % NT) : (int)threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  uint8_t* const lds = lds_all + grp * NBUF * kBuf;   // this group's stage buffers
  const int tiles = a.m_tiles * a.n_tiles;
  const int nwg = tiles * a.splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int split = lin / tiles, t2 = lin - split * tiles;
  const int mt = t2 / a.n_tiles, nt = t2 - mt * a.n_tiles;
  const int co0 = mt * BM, kk0 = nt * BN;
  const int tap = kk0 / a.C, ci0 = kk0 - tap * a.C;
  const int rr = tap / a.S, ss = tap - rr * a.S;
  // this group's steps: step0 + grp, step0 + grp + GRP, ... (a.sps steps per block)
  const int step0 = split * a.sps + grp;
  const int nblk_steps = min(a.sps, (a.M + kPix - 1) / kPix - split * a.sps);
  const int nsteps = nblk_steps > grp ? (nblk_steps - grp + GRP - 1) / GRP : 0;

  constexpr int RPI_A = 64 / CA, RPI_B = 64 / CB;   // rows per wave-instruction (1 KB)
  const int a_row_l = lane / CA, a_pos = lane % CA;
  const int b_row_l = lane / CB, b_pos = lane % CB;
  constexpr uint32_t kOOB = 0x80000000u;
  const __amdgpu_buffer_rsrc_t dyr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, a.dybytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.xbytes, 0x00020000);
  uint32_t a_voff[AI], b_voff[BI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int row = (wave * AI + i) * RPI_A + a_row_l;
    a_voff[i] = (uint32_t)((row * a.Cout + co0 + (a_pos ^ wswz2(row)) * 8) * 2);
  }
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int row = (wave * BI + i) * RPI_B + b_row_l;
    b_voff[i] = (uint32_t)((row * a.C + ci0 + (b_pos ^ wswz2(row)) * 8) * 2);
  }

  auto stage = [&](int step, int buf) {
    uint8_t* base = lds + buf * kBuf;
    const int p0 = (step0 + step * GRP) * kPix;
    const bool full = p0 + kPix <= a.M;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int row = (wave * AI + i) * RPI_A + a_row_l;
      const uint32_t vo = (full || p0 + row < a.M) ? a_voff[i] : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(dyr, (lds_ptr_t)(base + (wave * AI + i) * 1024), 16,
                                               vo, p0 * a.Cout * 2, 0, 0);
    }
    uint8_t* bb = base + kPix * RA;
    if (a.aff) {
#pragma unroll
      for (int i = 0; i < BI; ++i) {
        const int row = (wave * BI + i) * RPI_B + b_row_l;
        const uint32_t vo = (full || p0 + row < a.M) ? b_voff[i] : kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_ptr_t)(bb + (wave * BI + i) * 1024), 16,
                                                 vo, p0 * a.C * 2, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int row = (wave * BI + i) * RPI_B + b_row_l;
      const int m = p0 + row;
      uint32_t vo = kOOB;
      if (m < a.M) {
        const int n = (int)fdiv((uint32_t)m, a.div_hw);
        const int rem = m - n * a.Ho * a.Wo;
        const int ho = (int)fdiv((uint32_t)rem, a.div_w);
        const int wo = rem - ho * a.Wo;
        const int cch = b_pos ^ wswz2(row);
        const int hi = ho * a.stride - a.pad + rr;
        const int wi = wo * a.stride - a.pad_w + ss;
        if ((unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W)
          vo = (uint32_t)((((n * a.H + hi) * a.W + wi) * a.C + ci0 + cch * 8) * 2);
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_ptr_t)(bb + (wave * BI + i) * 1024), 16, vo,
                                               0, 0, 0);
    }
  };

  f32x16v acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int wm = wave / NWN, wn = wave % NWN;
  const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;


  auto compute = [&](int buf) {
    const uint8_t* abuf = lds + buf * kBuf;
    const uint8_t* bbuf = abuf + kPix * RA;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {   // 16 pixels per 32x32x16 MFMA
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = kk * 16 + 8 * (g >> 1) + 4 * h + qq;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int byte = 2 * (wm * WM + i * 32 + 16 * (g & 1) + 4 * pp);
          const int off = row * RA + (((byte >> 4) ^ wswz2(row)) << 4) + (byte & 15);
          const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t)(abuf + off));
          af[i][4 * h + 0] = v[0]; af[i][4 * h + 1] = v[1];
          af[i][4 * h + 2] = v[2]; af[i][4 * h + 3] = v[3];
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int byte = 2 * (wn * WN + j * 32 + 16 * (g & 1) + 4 * pp);
          const int off = row * RBB + (((byte >> 4) ^ wswz2(row)) << 4) + (byte & 15);
          const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t)(bbuf + off));
          bfr[j][4 * h + 0] = v[0]; bfr[j][4 * h + 1] = v[1];
          bfr[j][4 * h + 2] = v[2]; bfr[j][4 * h + 3] = v[3];
        }
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // every group runs the same trip count (barriers are workgroup-wide); a group past its last
  // step only takes part in the barriers
  const int trips = GRP > 1 ? (nblk_steps + GRP - 1) / GRP : nsteps;
  if (NBUF == 1 && trips > 0) {
    // serial form (high occupancy): stage, wait, compute, restage
    if (nsteps > 0) stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < trips; ++t) {
      if (t < nsteps) compute(0);
      if (t + 1 < trips) {
        __syncthreads();
        if (t + 1 < nsteps) stage(t + 1, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else if (nsteps > 0) {
    static_assert(GRP == 1 || NBUF == 1, "wave groups: serial form only");
    constexpr int S = NBUF > 1 ? NBUF - 1 : 1;
    constexpr int kLps = AI + BI;
#pragma unroll
    for (int i = 0; i < S; ++i)
      if (i < nsteps) stage(i, i);
    if (nsteps >= S)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((S - 1) * kLps) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    int cur = 0;
    for (int t = 0; t < nsteps; ++t) {
      if (t + S < nsteps) stage(t + S, cur == 0 ? NBUF - 1 : cur - 1);
      compute(cur);
      if (t + S < nsteps)
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((S - 1) * kLps) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      cur = cur == NBUF - 1 ? 0 : cur + 1;
    }
  }

  if constexpr (GRP > 1) {
    // groups 1 .. GRP-1 hand their sums to group 0, one group per round, in group order (the
    // stage buffers are free: the loop ended on a barrier after every wave's last read)
    float4* xs = reinterpret_cast<float4*>(lds_all) + (size_t)wave * (MI * NI * 4) * 64 + lane;
    for (int q = 1; q < GRP; ++q) {
      if (grp == q) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int k = 0; k < 4; ++k)
              xs[((i * NI + j) * 4 + k) * 64] =
                  make_float4(acc[i][j][4 * k], acc[i][j][4 * k + 1], acc[i][j][4 * k + 2],
                              acc[i][j][4 * k + 3]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (grp == 0) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const float4 v = xs[((i * NI + j) * 4 + k) * 64];
              acc[i][j][4 * k] += v.x;
              acc[i][j][4 * k + 1] += v.y;
              acc[i][j][4 * k + 2] += v.z;
              acc[i][j][4 * k + 3] += v.w;
            }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();   // group 0's reads done before the next group writes
      asm volatile("" ::: "memory");
    }
    if (grp != 0) return;
  }
  // D[row = co][col = k column]: lane holds column (lane & 31), rows (r & 3) + 8 (r >> 2) +
  // 4 (lane >> 5): 32 consecutive floats per half-wave store
  float* slab = a.ws + (size_t)split * a.Cout * a.Ktot;
  const int hh = lane >> 5;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int col = kk0 + wn * WN + j * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        slab[(size_t)co * a.Ktot + col] = acc[i][j][r];
      }
    }
}

template <int BM, int BN, int NWM, int NWN, int NBUF>
__global__ __launch_bounds__(64 * NWM * NWN) void conv_wgrad2_kernel(WgradArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  conv_wgrad2_body<BM, BN, NWM, NWN, NBUF>(a);
#endif
}

// serial single-buffer form, <= 128 VGPRs: four waves per SIMD (v1's variants 4..7 structure)
template <int BM, int BN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
void conv_wgrad2_kernel_occ4(WgradArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  conv_wgrad2_body<BM, BN, 2, 2, 1>(a);
#endif
}

// serial single-buffer form with GRP wave groups (2: 512 threads, 4: 1024) splitting the steps
template <int BM, int BN, int GRP>
__global__ __launch_bounds__(256 * GRP) void conv_wgrad2_kernel_grp(WgradArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  conv_wgrad2_body<BM, BN, 2, 2, 1, GRP>(a);
#endif
}

// v2 wgrad variant table (variant 8 + i): BM x BN (Cout x R*S*C), waves, stage buffers;
// 13 / 14: the serial 128x128 form with two / four wave groups per block
constexpr int kWg2Count = 7;
constexpr int kWg2Tiles[kWg2Count][2] = {{128, 128}, {256, 128}, {128, 256}, {256, 256},
                                         {128, 128}, {128, 128}, {128, 128}};

template <int BM, int BN, int NWM, int NWN, int NBUF, bool OCC4 = false, int GRP = 1>
hipError_t launch_wgrad2(WgradArgs a, int splits_hint, hipStream_t st) {
  a.m_tiles = a.Cout / BM;
  a.n_tiles = a.Ktot / BN;
  const int tiles = a.m_tiles * a.n_tiles;
  const int total = (a.M + 63) / 64;
  int splits = splits_hint > 0 ? splits_hint : std::max(1, (1024 + tiles / 2) / tiles);
  splits = std::min(splits, total);
  a.sps = (total + splits - 1) / splits;
  a.splits = (total + a.sps - 1) / a.sps;
  if constexpr (GRP > 1) {
    hipLaunchKernelGGL((conv_wgrad2_kernel_grp<BM, BN, GRP>), dim3(tiles * a.splits),
                       dim3(256 * GRP), 0, st, a);
  } else if constexpr (OCC4) {
    hipLaunchKernelGGL((conv_wgrad2_kernel_occ4<BM, BN>), dim3(tiles * a.splits), dim3(256), 0,
                       st, a);
  } else {
    hipLaunchKernelGGL((conv_wgrad2_kernel<BM, BN, NWM, NWN, NBUF>), dim3(tiles * a.splits),
                       dim3(64 * NWM * NWN), 0, st, a);
  }
  return hipGetLastError();
}

template <int BM, int BN>
hipError_t launch_wgrad(WgradArgs a, int splits_hint, bool serial, hipStream_t st) {
  a.m_tiles = a.Cout / BM;
  a.n_tiles = a.Ktot / BN;
  const int tiles = a.m_tiles * a.n_tiles;
  const int total = (a.M + 63) / 64;
  int splits = splits_hint > 0 ? splits_hint : std::max(1, (1024 + tiles / 2) / tiles);
  splits = std::min(splits, total);
  a.sps = (total + splits - 1) / splits;
  a.splits = (total + a.sps - 1) / a.sps;
  if (serial)
    hipLaunchKernelGGL((conv_wgrad_kernel_occ4<BM, BN>), dim3(tiles * a.splits), dim3(kThreads), 0,
                       st, a);
  else
    hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN>), dim3(tiles * a.splits), dim3(kThreads), 0, st,
                       a);
  return hipGetLastError();
}

}  // namespace


extern "C" {


// Number of split slabs the wgrad launch will use (the caller sizes the workspace with it).
int arena_conv_wgrad_splits(int N, int Ho, int Wo, int Cout, int Ktot, int variant,
                            int splits_hint) {
  static const int bm[4] = {128, 128, 64, 64}, bn[4] = {128, 64, 128, 64};
  if (variant < 0 || variant >= 8 + kWg2Count) return -1;
  const int tbm = variant >= 8 ? kWg2Tiles[variant - 8][0] : bm[variant & 3];
  const int tbn = variant >= 8 ? kWg2Tiles[variant - 8][1] : bn[variant & 3];
  const int tiles = (Cout / tbm) * (Ktot / tbn);
  const long long M = (long long)N * Ho * Wo;
  const int total = (int)((M + 63) / 64);
  int splits = splits_hint > 0 ? splits_hint : std::max(1, (1024 + tiles / 2) / tiles);
  splits = std::min(splits, total);
  const int sps = (total + splits - 1) / splits;
  return (total + sps - 1) / sps;
}

// variant: 0 = 128x128, 1 = 128x64, 2 = 64x128, 3 = 64x64 (Cout x R*S*C tile); + 4: serial
// single-buffer high-occupancy form of the same tile. Needs C % BN == 0
// (a tile never straddles two filter taps) and Cout % BM == 0; c16 mode: C == 16, S % 4 == 0 and
// BN == 64 (variants 1 and 3). Ho/Wo <= 0: derived from a symmetric padding.
hipError_t arena_conv_wgrad_ex(const void* x, const void* dy, float* ws, void* dw_bf16,
                               float* dw_f32, int N, int H, int W, int C, int Cout, int R, int S,
                               int stride, int pad_h, int pad_w, int Ho, int Wo, int c16,
                               int variant, int splits_hint, float scale, hipStream_t st) {
  static const int bm[4] = {128, 128, 64, 64}, bn[4] = {128, 64, 128, 64};
  if (variant < 0 || variant >= 8 + kWg2Count) return hipErrorInvalidValue;
  const bool v2 = variant >= 8;
  const int tv = variant & 3;
  const bool serial = !v2 && variant >= 4;
  const int tbm = v2 ? kWg2Tiles[variant - 8][0] : bm[tv];
  const int tbn = v2 ? kWg2Tiles[variant - 8][1] : bn[tv];
  if (v2 && c16) return hipErrorInvalidValue;
  if (c16 ? (C != 16 || S % 4 || tbn != 64) : (C % tbn != 0)) return hipErrorInvalidValue;
  if (Cout % tbm || N <= 0 || stride <= 0) return hipErrorInvalidValue;
  WgradArgs a{};
  a.x = (const uint16_t*)x;
  a.dy = (const uint16_t*)dy;
  a.ws = ws;
  a.N = N; a.H = H; a.W = W; a.C = C; a.Cout = Cout; a.R = R; a.S = S;
  a.stride = stride; a.pad = pad_h; a.pad_w = pad_w; a.c16 = c16;
  {
    const long long xb = (long long)N * H * W * C * 2;
    const long long Ho_ = Ho > 0 ? Ho : (H + 2 * pad_h - R) / stride + 1;
    const long long Wo_ = Wo > 0 ? Wo : (W + 2 * pad_w - S) / stride + 1;
    const long long db = (long long)N * Ho_ * Wo_ * Cout * 2;
    if (xb >= (1LL << 31) || db >= (1LL << 31)) return hipErrorInvalidValue;
    a.xbytes = (int)xb;
    a.dybytes = (int)db;
    a.aff = (!c16 && R == 1 && S == 1 && stride == 1 && pad_h == 0 && pad_w == 0 &&
             Ho_ == H && Wo_ == W) ? 1 : 0;
  }
  a.Ho = Ho > 0 ? Ho : (H + 2 * pad_h - R) / stride + 1;
  a.Wo = Wo > 0 ? Wo : (W + 2 * pad_w - S) / stride + 1;
  if (a.Ho <= 0 || a.Wo <= 0) return hipErrorInvalidValue;
  const long long M = (long long)N * a.Ho * a.Wo;
  if (M >= (1LL << 31)) return hipErrorInvalidValue;
  a.M = (int)M;
  a.Ktot = R * S * C;
  a.div_hw = make_fastdiv((uint32_t)(a.Ho * a.Wo));
  a.div_w = make_fastdiv((uint32_t)a.Wo);
  hipError_t e;
  if (v2) {
    switch (variant - 8) {
      case 0: e = launch_wgrad2<128, 128, 2, 2, 2>(a, splits_hint, st); break;
      case 1: e = launch_wgrad2<256, 128, 4, 2, 2>(a, splits_hint, st); break;
      case 2: e = launch_wgrad2<128, 256, 2, 4, 2>(a, splits_hint, st); break;
      case 3: e = launch_wgrad2<256, 256, 2, 4, 2>(a, splits_hint, st); break;
      case 5: e = launch_wgrad2<128, 128, 2, 2, 1, false, 2>(a, splits_hint, st); break;
      case 6: e = launch_wgrad2<128, 128, 2, 2, 1, false, 4>(a, splits_hint, st); break;
      default: e = launch_wgrad2<128, 128, 2, 2, 1, true>(a, splits_hint, st); break;
    }
  } else switch (tv) {
    case 0: e = launch_wgrad<128, 128>(a, splits_hint, serial, st); break;
    case 1: e = launch_wgrad<128, 64>(a, splits_hint, serial, st); break;
    case 2: e = launch_wgrad<64, 128>(a, splits_hint, serial, st); break;
    default: e = launch_wgrad<64, 64>(a, splits_hint, serial, st); break;
  }
  if (e != hipSuccess) return e;
  const int splits = arena_conv_wgrad_splits(N, a.Ho, a.Wo, Cout, a.Ktot, variant, splits_hint);
  const long long n4 = (long long)Cout * a.Ktot / 4;  // Cout % 64 == 0
  // the 8 x 32 shape while 32-column blocks would not give every CU a block
  if (n4 < 32LL * 256 && splits >= 64)
    hipLaunchKernelGGL((conv_wgrad_reduce_kernel<8, 32>), dim3((unsigned)((n4 + 7) / 8)), dim3(256),
                       0, st, reinterpret_cast<const float4*>(ws), splits, n4,
                       reinterpret_cast<uint2*>(dw_bf16), reinterpret_cast<float4*>(dw_f32), scale);
  else
    hipLaunchKernelGGL((conv_wgrad_reduce_kernel<32, 8>), dim3((unsigned)((n4 + 31) / 32)),
                       dim3(256), 0, st, reinterpret_cast<const float4*>(ws), splits, n4,
                       reinterpret_cast<uint2*>(dw_bf16), reinterpret_cast<float4*>(dw_f32), scale);
  return hipGetLastError();
}

hipError_t arena_conv_wgrad(const void* x, const void* dy, float* ws, void* dw_bf16, float* dw_f32,
                            int N, int H, int W, int C, int Cout, int R, int S, int stride,
                            int pad, int variant, int splits_hint, float scale, hipStream_t st) {
  return arena_conv_wgrad_ex(x, dy, ws, dw_bf16, dw_f32, N, H, W, C, Cout, R, S, stride, pad, pad,
                             0, 0, 0, variant, splits_hint, scale, st);
}

}  // extern "C"
