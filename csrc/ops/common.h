// Shared device-side definitions for the arena_amd HIP kernels (gfx950 / CDNA4 only).
//
// Design notes (MI355X-first):
//  * wave64 everywhere: lane = threadIdx.x & 63, 64-bit ballots, shfl over 64 lanes.
//  * fp32 matmul-shaped work goes to the exact-f32 MFMA (v_mfma_f32_16x16x4_f32):
//      A operand: lane l holds A[i = l&15][k = l>>4]
//      B operand: lane l holds B[k = l>>4][j = l&15]
//      C/D      : lane l, reg r holds D[row = 4*(l>>4) + r][col = l&15]
//  * Per-step scalars that change across hipGraph replays (data cursor, Adam step t,
//    learning rate) live in device memory and are read in-kernel, never baked in.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "abi.h"

namespace arena {

// Optional in-kernel phase timeline (build with -DARENA_TIMELINE; scripts/timeline.py): thread 0
// of every block stamps the 100 MHz s_memrealtime clock at phase points of a kernel, so phase
// costs and launch skew can be read per block. Compiles to nothing in normal builds.
#ifdef ARENA_TIMELINE
#define ARENA_TL_SLOTS 16
#define ARENA_TL_BLOCKS 1024
extern __device__ long long arena_tl_buf[];
#define ARENA_TL(kid, i)                                                                      \
  do {                                                                                        \
    if (threadIdx.x == 0) {                                                                   \
      const int tl_b_ = (int)(blockIdx.x + gridDim.x * blockIdx.y);                           \
      if (tl_b_ < ARENA_TL_BLOCKS)                                                            \
        arena_tl_buf[((kid) * ARENA_TL_BLOCKS + tl_b_) * ARENA_TL_SLOTS + (i)] = wall_clock64(); \
    }                                                                                         \
  } while (0)
#define ARENA_TL_DRAIN() __builtin_amdgcn_s_waitcnt(0)
// make the next stamp wait until value x has arrived (loads) / been computed (MFMA)
#define ARENA_TL_DEP(x) asm volatile("" ::"v"(x))
#else
#define ARENA_TL_DEP(x) \
  do {                  \
  } while (0)
#define ARENA_TL(kid, i) \
  do {                   \
  } while (0)
#define ARENA_TL_DRAIN() \
  do {                   \
  } while (0)
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

__device__ __forceinline__ f32x4 mfma_16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Full-wave reductions without LDS round trips: DPP quad_perm (xor 1, xor 2) and row_ror (4, 8)
// inside each 16-lane row, ds_swizzle xor 16 across row pairs, then two v_readlane for the
// halves. Result is wave-uniform. (The __shfl_xor form is 6 dependent ds_bpermute_b32.)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float swz_xor16(float v) {
  // ds_swizzle bit-mode: offset = xor_mask<<10 | or_mask<<5 | and_mask  (within 32-lane halves)
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (0x10 << 10) | 0x1F));
}
__device__ __forceinline__ float wave_sum_fast(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x124>(v);  // row_ror:4
  v += dpp_f<0x128>(v);  // row_ror:8
  v += swz_xor16(v);
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
         __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
}
__device__ __forceinline__ float wave_max_fast(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x124>(v));
  v = fmaxf(v, dpp_f<0x128>(v));
  v = fmaxf(v, swz_xor16(v));
  return fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)),
               __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Counter-based hash used for dropout masks: a pure function of (seed, step, row, col) so the
// mask never has to be stored and a PyTorch reference can reproduce it bit-exactly
// (arena_amd/ops/reference.py::dropout_keep_mask).
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t h) {
  h ^= h >> 16; h *= 0x7FEB352Du;
  h ^= h >> 15; h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}
__host__ __device__ __forceinline__ uint32_t hash4(uint32_t seed, uint32_t step, uint32_t row,
                                                   uint32_t col) {
  uint32_t h = mix32(seed ^ 0x9E3779B9u);
  h = mix32(h ^ (step * 0x85EBCA77u));
  h = mix32(h ^ (row * 0xC2B2AE3Du));
  h = mix32(h ^ (col * 0x27D4EB2Fu));
  return h;
}

}  // namespace arena

