// NHWC max pooling forward/backward for gfx950 (MI355X): the ResNet stem's 3x3 / stride 2 pool.
//
// The library backward (at::native::max_pool_backward_nhwc) took 305 us per ResNet-50 batch-128
// step on MI355X (profiles/r1_resnet50_fusedbn_steady_kernels.csv), ~7x its HBM floor: it
// re-derives each input's window membership with a divide-heavy per-element loop. Here:
//
//   forward   one thread = 8 channels of one output pixel: k*k 16-byte loads (neighbouring
//             threads share them through L1/L2), max with PyTorch's rule (first strict maximum in
//             kh-major order, NaN wins), 16-byte store of y, 8-byte store of the argmax as the
//             in-window position (uint8, 0..k*k-1);
//   backward  one thread = 8 channels of one INPUT pixel: gather dy from the (at most
//             ceil(k/s)^2) windows that contain it where the saved position points back at it,
//             sum in fp32, one 16-byte store. No atomics, no zero-fill of dx, and dx is written
//             exactly once.
//
// Layout: x [N][H][W][C] (channels_last), C % 8 == 0, dilation 1, floor mode, k <= 15.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kT = 256;
constexpr int kVec = 8;
// backward: input rows per block (57K one-row blocks of the stem pool were dispatch-bound)
constexpr int kRowsPerBlock = 4;

template <typename T>
struct P8;
template <>
struct P8<uint16_t> {  // bf16
  static __device__ __forceinline__ void load(const uint16_t* p, float v[kVec]) {
    const uint4 q = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ uint16_t bf(float f) {  // RNE, NaN stays NaN
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
  }
  static __device__ __forceinline__ void store(uint16_t* p, const float v[kVec]) {
    uint4 q;
    q.x = bf(v[0]) | ((uint32_t)bf(v[1]) << 16);
    q.y = bf(v[2]) | ((uint32_t)bf(v[3]) << 16);
    q.z = bf(v[4]) | ((uint32_t)bf(v[5]) << 16);
    q.w = bf(v[6]) | ((uint32_t)bf(v[7]) << 16);
    *reinterpret_cast<uint4*>(p) = q;
  }
};
template <>
struct P8<float> {
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
};

struct PoolGeo {
  int N, H, W, C, OH, OW, k, s, p;
};

template <typename T>
__global__ __launch_bounds__(kT) void maxpool_fwd_kernel(const T* __restrict__ x,
                                                         T* __restrict__ y,
                                                         uint8_t* __restrict__ pos,
                                                         PoolGeo g, long long nvec) {
  const int cg = g.C / kVec;
  // blockIdx.x = output row (n, oh), blockIdx.y * kT + tid = (ow, c8): two 32-bit divides per
  // thread instead of a chain of 64-bit ones (those cost more than the memory traffic)
  const int row = blockIdx.x;
  const int t = blockIdx.y * kT + threadIdx.x;
  if (t < g.OW * cg) {
    const int ow = t / cg, c8 = t - ow * cg;
    const int n32 = row / g.OH, oh = row - n32 * g.OH;
    const long long n = n32;
    const long long v = (long long)row * g.OW * cg + t;
    const int h0 = oh * g.s - g.p, w0 = ow * g.s - g.p;
    float m[kVec];
    int best[kVec];
#pragma unroll
    for (int i = 0; i < kVec; ++i) { m[i] = -INFINITY; best[i] = -1; }
    for (int kh = 0; kh < g.k; ++kh) {
      const int h = h0 + kh;
      if (h < 0 || h >= g.H) continue;
      for (int kw = 0; kw < g.k; ++kw) {
        const int w = w0 + kw;
        if (w < 0 || w >= g.W) continue;
        float a[kVec];
        P8<T>::load(x + (((n * g.H + h) * g.W + w) * g.C + (long long)c8 * kVec), a);
        const int q = kh * g.k + kw;
#pragma unroll
        for (int i = 0; i < kVec; ++i) {
          // PyTorch's rule: (val > max) || isnan(val) (so the last NaN wins); the first in-bounds
          // element always counts, so an all -inf window still points at a real input
          if (a[i] > m[i] || __builtin_isnan(a[i]) || best[i] < 0) { m[i] = a[i]; best[i] = q; }
        }
      }
    }
    P8<T>::store(y + v * kVec, m);
    uint2 pk;
    pk.x = (uint32_t)(best[0] & 0xff) | ((uint32_t)(best[1] & 0xff) << 8) |
           ((uint32_t)(best[2] & 0xff) << 16) | ((uint32_t)(best[3] & 0xff) << 24);
    pk.y = (uint32_t)(best[4] & 0xff) | ((uint32_t)(best[5] & 0xff) << 8) |
           ((uint32_t)(best[6] & 0xff) << 16) | ((uint32_t)(best[7] & 0xff) << 24);
    *reinterpret_cast<uint2*>(pos + v * kVec) = pk;
  }
}

// CW = ceil(k / s) candidate windows per spatial dimension (2 for the 3x3 / 2 stem pool). All
// CW*CW position loads, then all dy loads, are issued before any is used: a data-dependent
// "skip the dy load" branch per window serialised them into 2*CW*CW round trips.
template <typename T, int CW>
__global__ __launch_bounds__(kT) void maxpool_bwd_kernel(const T* __restrict__ dy,
                                                         const uint8_t* __restrict__ pos,
                                                         T* __restrict__ dx, PoolGeo g,
                                                         long long nvec) {
  const int cg = g.C / kVec;
  // blockIdx.x = group of kRowsPerBlock input rows (n, h), blockIdx.y * kT + tid = (w, c8)
  const int t = blockIdx.y * kT + threadIdx.x;
  const int rows = g.N * g.H;
#pragma unroll 1
  for (int row = blockIdx.x * kRowsPerBlock; row < min(rows, (int)(blockIdx.x + 1) * kRowsPerBlock);
       ++row) {
    if (t >= g.W * cg) break;
    const int w = t / cg, c8 = t - w * cg;
    const int n32 = row / g.H, h = row - n32 * g.H;
    const long long n = n32;
    const long long v = (long long)row * g.W * cg + t;
    // windows oh with oh*s - p <= h <= oh*s - p + k - 1
    const int th = h + g.p - g.k + 1, tw = w + g.p - g.k + 1;
    const int oh_lo = th <= 0 ? 0 : (th + g.s - 1) / g.s;
    const int ow_lo = tw <= 0 ? 0 : (tw + g.s - 1) / g.s;
    const int oh_hi = min(g.OH - 1, (h + g.p) / g.s);
    const int ow_hi = min(g.OW - 1, (w + g.p) / g.s);
    long long off[CW * CW];
    int q[CW * CW];
    uint2 pk[CW * CW];
#pragma unroll
    for (int a = 0; a < CW; ++a) {
#pragma unroll
      for (int b = 0; b < CW; ++b) {
        const int j = a * CW + b;
        const bool ok = oh_lo + a <= oh_hi && ow_lo + b <= ow_hi;
        // not-a-window slots read a clamped in-bounds address (an input no window covers, when
        // k < s, has oh_lo = OH)
        const int oh = ok ? oh_lo + a : min(oh_lo, g.OH - 1);
        const int ow = ok ? ow_lo + b : min(ow_lo, g.OW - 1);
        q[j] = ok ? (h - (oh * g.s - g.p)) * g.k + (w - (ow * g.s - g.p)) : 0xff;  // 0xff: none
        off[j] = ((n * g.OH + oh) * g.OW + ow) * g.C + (long long)c8 * kVec;
        pk[j] = *reinterpret_cast<const uint2*>(pos + off[j]);
      }
    }
    float d[CW * CW][kVec];
#pragma unroll
    for (int j = 0; j < CW * CW; ++j) P8<T>::load(dy + off[j], d[j]);
    float acc[kVec];
#pragma unroll
    for (int i = 0; i < kVec; ++i) acc[i] = 0.f;
#pragma unroll
    for (int j = 0; j < CW * CW; ++j) {
      const uint32_t ps[2] = {pk[j].x, pk[j].y};
#pragma unroll
      for (int i = 0; i < kVec; ++i)
        acc[i] += ((ps[i >> 2] >> (8 * (i & 3))) & 0xff) == (uint32_t)q[j] ? d[j][i] : 0.f;
    }
    P8<T>::store(dx + v * kVec, acc);
  }
}

// rows (n, h) on x, the (w, channel-group) vectors of a row on y
dim3 grid_for(long long rows, long long row_vecs) {
  return dim3((unsigned)rows, (unsigned)((row_vecs + kT - 1) / kT));
}

bool bad(const PoolGeo& g) {
  return g.N <= 0 || g.H <= 0 || g.W <= 0 || g.C <= 0 || g.C % kVec || g.k < 1 || g.k > 15 ||
         g.s < 1 || g.p < 0 || 2 * g.p > g.k || g.OH != (g.H + 2 * g.p - g.k) / g.s + 1 ||
         g.OW != (g.W + 2 * g.p - g.k) / g.s + 1 || g.OH <= 0 || g.OW <= 0 ||
         (long long)g.N * g.H >= (1LL << 31) ||
         ((long long)g.W * (g.C / kVec) + kT - 1) / kT > 65535;
}

}  // namespace

extern "C" {

// dtype: 0 = f32, 1 = bf16. pos: uint8 [N][OH][OW][C] in-window argmax positions.
hipError_t arena_maxpool_fwd(int dtype, const void* x, void* y, uint8_t* pos, int N, int H, int W,
                             int C, int k, int s, int p, hipStream_t stream) {
  const PoolGeo g{N, H, W, C, (H + 2 * p - k) / s + 1, (W + 2 * p - k) / s + 1, k, s, p};
  if (bad(g)) return hipErrorInvalidValue;
  const long long nvec = (long long)N * g.OH * g.OW * (C / kVec);
  const dim3 grid = grid_for((long long)N * g.OH, (long long)g.OW * (C / kVec));
  if (dtype == 1)
    hipLaunchKernelGGL(maxpool_fwd_kernel<uint16_t>, grid, dim3(kT), 0, stream,
                       static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), pos, g, nvec);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, grid, dim3(kT), 0, stream,
                       static_cast<const float*>(x), static_cast<float*>(y), pos, g, nvec);
  return hipGetLastError();
}

hipError_t arena_maxpool_bwd(int dtype, const void* dy, const uint8_t* pos, void* dx, int N, int H,
                             int W, int C, int k, int s, int p, hipStream_t stream) {
  const PoolGeo g{N, H, W, C, (H + 2 * p - k) / s + 1, (W + 2 * p - k) / s + 1, k, s, p};
  if (bad(g)) return hipErrorInvalidValue;
  const long long nvec = (long long)N * H * W * (C / kVec);
  const dim3 grid = grid_for((long long)N * H, (long long)W * (C / kVec));
  const dim3 grid_b((unsigned)((N * H + kRowsPerBlock - 1) / kRowsPerBlock), grid.y);
  const int cw = (k + s - 1) / s;
#define ARENA_POOL_BWD(TT, CW)                                                               \
  hipLaunchKernelGGL((maxpool_bwd_kernel<TT, CW>), grid_b, dim3(kT), 0, stream,            \
                     static_cast<const TT*>(dy), pos, static_cast<TT*>(dx), g, nvec)
  if (cw < 1 || cw > 3) return hipErrorInvalidValue;
  if (dtype == 1) {
    if (cw == 1) ARENA_POOL_BWD(uint16_t, 1);
    else if (cw == 2) ARENA_POOL_BWD(uint16_t, 2);
    else ARENA_POOL_BWD(uint16_t, 3);
  } else {
    if (cw == 1) ARENA_POOL_BWD(float, 1);
    else if (cw == 2) ARENA_POOL_BWD(float, 2);
    else ARENA_POOL_BWD(float, 3);
  }
#undef ARENA_POOL_BWD
  return hipGetLastError();
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// Softmax cross-entropy of the classifier head (mean over rows), fp32 arithmetic on bf16 or fp32
// logits: F.cross_entropy's result in three launches (forward, mean, backward) instead of its seven
// (upcast copy, log_softmax, nll forward, two fills, nll backward, log_softmax backward, downcast
// copy: ~45 us per ResNet-50 bs128 step, profiles/r6_kernel_neighbors.txt).
// forward: one wave per row, every sum in a fixed order (deterministic); writes each row's loss and
// log-sum-exp (the mean is taken by the caller, also deterministic). backward: one elementwise pass,
// dlogits = g * (exp(x - lse) - onehot) / rows, in the logits' dtype.
// ------------------------------------------------------------------------------------------------
namespace {

template <typename T>
__device__ __forceinline__ float xent_ld(const T* p, long long i) {
  if constexpr (sizeof(T) == 2) return __uint_as_float((uint32_t)p[i] << 16);
  else return p[i];
}

// One wave per row, four rows per block. NPL > 0: the row (<= 64 * NPL classes) is loaded into
// registers once, all NPL loads in flight, and max / sum-exp run from registers; NPL == 0: any
// width, three passes over memory. Writes the row's log-sum-exp and loss; the mean over rows is a
// separate deterministic reduction (the caller's). (A single-block form -- one block walking all
// rows, the mean in LDS -- took 60 us per ResNet-50 bs128 step at 1000 classes: eight rows per
// wave, each waiting out its loads serially, profiles/r6_xent_fwd_before_after.txt.)
template <typename T, int NPL>
__global__ __launch_bounds__(256) void xent_fwd_kernel(const T* __restrict__ x,
                                                       const long long* __restrict__ y,
                                                       float* __restrict__ rowloss,
                                                       float* __restrict__ lse, int rows,
                                                       int classes) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const T* xr = x + (long long)r * classes;
  float m = -INFINITY, s = 0.f;
  if constexpr (NPL > 0) {
    float v[NPL];
#pragma unroll
    for (int j = 0; j < NPL; ++j) {
      const int c = lane + 64 * j;
      v[j] = c < classes ? xent_ld(xr, c) : -INFINITY;
    }
#pragma unroll
    for (int j = 0; j < NPL; ++j) m = fmaxf(m, v[j]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
#pragma unroll
    for (int j = 0; j < NPL; ++j) s += lane + 64 * j < classes ? __expf(v[j] - m) : 0.f;
  } else {
    for (int c = lane; c < classes; c += 64) m = fmaxf(m, xent_ld(xr, c));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    for (int c = lane; c < classes; c += 64) s += __expf(xent_ld(xr, c) - m);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) {
    const float l = m + __logf(s);
    long long t = y[r];
    t = t < 0 ? 0 : (t >= classes ? classes - 1 : t);
    lse[r] = l;
    rowloss[r] = l - xent_ld(xr, t);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void xent_bwd_kernel(const T* __restrict__ x,
                                                       const long long* __restrict__ y,
                                                       const float* __restrict__ lse,
                                                       const float* __restrict__ gout,
                                                       T* __restrict__ dx, int rows, int classes) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)rows * classes) return;
  const int r = (int)(i / classes), c = (int)(i - (long long)r * classes);
  long long t = y[r];
  t = t < 0 ? 0 : (t >= classes ? classes - 1 : t);
  const float p = __expf(xent_ld(x, i) - lse[r]);
  const float v = (*gout) * (p - (c == t ? 1.f : 0.f)) / (float)rows;
  if constexpr (sizeof(T) == 2) {
    const uint32_t u = __float_as_uint(v);
    dx[i] = (T)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);   // round to nearest even
  } else {
    dx[i] = v;
  }
}

}  // namespace

extern "C" {

// dtype: 0 = f32, 1 = bf16 logits [rows][classes]; y: int64 [rows]; rowloss, lse: fp32 [rows]
hipError_t arena_xent_fwd(int dtype, const void* x, const long long* y, float* rowloss,
                          float* lse, int rows, int classes, hipStream_t stream) {
  if (rows <= 0 || classes <= 0) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
#define XENT_LAUNCH(T, NPL)                                                                     \
  hipLaunchKernelGGL((xent_fwd_kernel<T, NPL>), grid, block, 0, stream,                         \
                     static_cast<const T*>(x), y, rowloss, lse, rows, classes)
  if (dtype == 1) {
    if (classes <= 64 * 16) XENT_LAUNCH(uint16_t, 16);
    else XENT_LAUNCH(uint16_t, 0);
  } else {
    if (classes <= 64 * 16) XENT_LAUNCH(float, 16);
    else XENT_LAUNCH(float, 0);
  }
#undef XENT_LAUNCH
  return hipGetLastError();
}

hipError_t arena_xent_bwd(int dtype, const void* x, const long long* y, const float* lse,
                          const float* gout, void* dx, int rows, int classes, hipStream_t stream) {
  if (rows <= 0 || classes <= 0) return hipErrorInvalidValue;
  const long long n = (long long)rows * classes;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (dtype == 1)
    hipLaunchKernelGGL(xent_bwd_kernel<uint16_t>, grid, dim3(256), 0, stream,
                       static_cast<const uint16_t*>(x), y, lse, gout, static_cast<uint16_t*>(dx),
                       rows, classes);
  else
    hipLaunchKernelGGL(xent_bwd_kernel<float>, grid, dim3(256), 0, stream,
                       static_cast<const float*>(x), y, lse, gout, static_cast<float*>(dx), rows,
                       classes);
  return hipGetLastError();
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// Backward of the global average pool: dx[n, p, c] = g[n, c] / HW for every pixel p of a
// channels_last [N, HW, C] tensor, 8 channels (16 bytes of bf16) per thread -- one write pass
// (the stock broadcast-and-copy wrote it at ~1.2 TB/s through torch's non-vectorised copy kernel).
// ------------------------------------------------------------------------------------------------
namespace {

template <typename T>
__global__ __launch_bounds__(256) void gap_bwd_kernel(const T* __restrict__ g, T* __restrict__ dx,
                                                      long long nvec, int hw, int cg, float scale) {
  const long long v = (long long)blockIdx.x * 256 + threadIdx.x;
  if (v >= nvec) return;
  const int c8 = (int)(v % cg);
  const long long n = v / ((long long)cg * hw);
  float a[kVec];
  P8<T>::load(g + (n * cg + c8) * kVec, a);
#pragma unroll
  for (int i = 0; i < kVec; ++i) a[i] *= scale;
  P8<T>::store(dx + v * kVec, a);
}

}  // namespace

extern "C" {

// dtype: 0 = f32, 1 = bf16. g: [N][C]; dx: channels_last [N][HW][C]; C % 8 == 0
hipError_t arena_gap_bwd(int dtype, const void* g, void* dx, int N, int HW, int C, float scale,
                         hipStream_t stream) {
  if (N <= 0 || HW <= 0 || C <= 0 || C % kVec) return hipErrorInvalidValue;
  const long long nvec = (long long)N * HW * (C / kVec);
  const dim3 grid((unsigned)((nvec + 255) / 256));
  if (dtype == 1)
    hipLaunchKernelGGL(gap_bwd_kernel<uint16_t>, grid, dim3(256), 0, stream,
                       static_cast<const uint16_t*>(g), static_cast<uint16_t*>(dx), nvec, HW,
                       C / kVec, scale);
  else
    hipLaunchKernelGGL(gap_bwd_kernel<float>, grid, dim3(256), 0, stream,
                       static_cast<const float*>(g), static_cast<float*>(dx), nvec, HW, C / kVec,
                       scale);
  return hipGetLastError();
}

}  // extern "C"
