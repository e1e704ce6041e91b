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
  int N, H, W, C, Cout, R, S, stride, pad, Ho, Wo;
  int M;               // N * Ho * Wo
  int Ktot;            // R * S * C
  int m_tiles, n_tiles;
};

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)lds_wave_base, 16, 0, 0);
}

// bf16 round-to-nearest-even of two floats, packed (lo = a)
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  uint32_t ua = __float_as_uint(a), ub = __float_as_uint(b);
  ua = (ua + 0x7FFFu + ((ua >> 16) & 1u)) >> 16;
  ub = (ub + 0x7FFFu + ((ub >> 16) & 1u)) & 0xFFFF0000u;
  return ua | ub;
}

template <int BM, int BN>
__global__ __launch_bounds__(kThreads) void conv_fwd_kernel(ConvArgs a) {
  constexpr int WM = BM / 2, WN = BN / 2;        // per-wave output tile (2 x 2 waves)
  constexpr int MI = WM / 16, NI = WN / 16;      // 16x16 MFMA tiles per wave
  constexpr int AI = BM * 8 / kThreads;          // A staging instructions per thread
  constexpr int BI = BN * 8 / kThreads;
  constexpr int kBufBytes = (BM + BN) * kRowBytes;
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * kBufBytes];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // XCD-aware tile order: blocks b and b+8 share an XCD (round-robin dispatch), so give each XCD
  // a contiguous range of tiles (bijective for any grid size).
  const int nwg = a.m_tiles * a.n_tiles;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (bid >> 3);
  const int mt = tile / a.n_tiles, nt = tile - mt * a.n_tiles;
  const int m0 = mt * BM, n0 = nt * BN;

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
      a_wb[i] = wo * a.stride - a.pad;
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
  const int CB = a.C / kBK;  // 64-channel blocks per tap

  auto stage = [&](int t, int buf) {
    const int tap = t / CB, cb = t - tap * CB;
    const int r = tap / a.S, s = tap - r * a.S;
    uint8_t* base = lds + buf * kBufBytes;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int hi = a_hb[i] + r, wi = a_wb[i] + s;
      const bool ok = (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
      const void* src = ok ? (const void*)(a.x + ((size_t)(a_nb[i] + hi) * a.W + wi) * a.C +
                                           cb * kBK + a_chunk[i] * 8)
                           : (const void*)g_zero_page;
      glds16(src, base + (wave * AI + i) * 64 * 16);
    }
    uint8_t* bbase = base + BM * kRowBytes;
#pragma unroll
    for (int i = 0; i < BI; ++i) glds16(b_src[i] + (size_t)t * kBK, bbase + (wave * BI + i) * 64 * 16);
  };

  f32x4v acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fq = lane >> 4;
  const int T = a.Ktot / kBK;

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    const int cur = t & 1;
    if (t + 1 < T) stage(t + 1, cur ^ 1);
    const uint8_t* abuf = lds + cur * kBufBytes;
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
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: lane holds channels n0+wn*WN+j*16+4*fq .. +3 of pixel m0+wm*WM+i*16+fr ----
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int m = m0 + wm * WM + i * 16 + fr;
    if (m >= a.M) continue;
    uint16_t* yrow = a.y + (size_t)m * a.Cout + n0 + wn * WN + 4 * fq;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      uint2 v;
      v.x = pack_bf16x2(acc[i][j][0], acc[i][j][1]);
      v.y = pack_bf16x2(acc[i][j][2], acc[i][j][3]);
      *reinterpret_cast<uint2*>(yrow + j * 16) = v;
    }
  }
}

template <int BM, int BN>
hipError_t launch(const ConvArgs& a0, hipStream_t st) {
  ConvArgs a = a0;
  a.m_tiles = (a.M + BM - 1) / BM;
  a.n_tiles = a.Cout / BN;
  const int nwg = a.m_tiles * a.n_tiles;
  hipLaunchKernelGGL((conv_fwd_kernel<BM, BN>), dim3(nwg), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

}  // namespace

extern "C" {

// Returns hipErrorInvalidValue for shapes the kernel does not cover (the caller falls back to
// MIOpen): C % 64 != 0, Cout % 64 != 0, or an unknown tile variant.
// variant: 0 = 128x128, 1 = 128x64, 2 = 64x128, 3 = 64x64 (BM x BN output tile per block).
hipError_t arena_conv_fwd(const void* x, const void* w, void* y, int N, int H, int W, int C,
                          int Cout, int R, int S, int stride, int pad, int variant,
                          hipStream_t st) {
  if (C % kBK || Cout % 64 || N <= 0 || R <= 0 || S <= 0 || stride <= 0 || pad < 0)
    return hipErrorInvalidValue;
  ConvArgs a{};
  a.x = (const uint16_t*)x;
  a.w = (const uint16_t*)w;
  a.y = (uint16_t*)y;
  a.N = N; a.H = H; a.W = W; a.C = C; a.Cout = Cout; a.R = R; a.S = S;
  a.stride = stride; a.pad = pad;
  a.Ho = (H + 2 * pad - R) / stride + 1;
  a.Wo = (W + 2 * pad - S) / stride + 1;
  if (a.Ho <= 0 || a.Wo <= 0) return hipErrorInvalidValue;
  const long long M = (long long)N * a.Ho * a.Wo;
  if (M >= (1LL << 31) || (long long)N * H * W * C >= (1LL << 40)) return hipErrorInvalidValue;
  a.M = (int)M;
  a.Ktot = R * S * C;
  switch (variant) {
    case 0: return Cout % 128 ? hipErrorInvalidValue : launch<128, 128>(a, st);
    case 1: return launch<128, 64>(a, st);
    case 2: return Cout % 128 ? hipErrorInvalidValue : launch<64, 128>(a, st);
    case 3: return launch<64, 64>(a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // extern "C"
