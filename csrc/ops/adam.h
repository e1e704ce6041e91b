// Device-side optimizer + step-counter helpers shared by the MLP kernels (mlp_kernels.hip) and
// the fused xGMI reduce-scatter/Adam/all-gather collective (csrc/ccl/xgmi_ccl.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "abi.h"

namespace arena {

__device__ __forceinline__ void counter_op(const ArenaCounterOp& c) {
  if (c.dst != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    *c.dst = (c.src ? *c.src : 0) + c.add;
  }
}

__device__ __forceinline__ float adam_lr(const ArenaAdam& a) { return a.lr_ptr ? *a.lr_ptr : a.lr; }

// Hardware transcendentals (v_exp_f32 / v_log_f32 / v_sqrt_f32 / v_rcp_f32, ~1 ulp) instead of
// the IEEE-exact library sequences (denormal pre-scaling + Newton corrections + div_fixup). The
// exact versions made the fused Adam epilogue of the MNIST backward kernel ~1 µs of its 8 µs
// (profiles/r1_timeline_phases*.json, ISA of wgrad_grouped_kernel); a 1-ulp difference in Adam's
// update is far below fp32 training noise (tests compare against torch.optim.Adam at rtol 1e-5).
__device__ __forceinline__ float hw_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float hw_log2(float x) { return __builtin_amdgcn_logf(x); }
__device__ __forceinline__ float hw_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float hw_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

struct AdamCoef {
  float step_size, inv_sqrt_bc2, eps, b1, b2, wd, gscale;
  int tf;
};

// coefficients from already-loaded step t and learning rate (lets a kernel issue those loads early
// and do the math late)
__device__ __forceinline__ AdamCoef adam_coef_tl(const ArenaAdam& a, float t, float lr) {
  AdamCoef c;
  const float bc1 = 1.0f - hw_exp2(t * hw_log2(a.beta1));
  const float bc2 = 1.0f - hw_exp2(t * hw_log2(a.beta2));
  c.tf = a.tf_style;
  if (a.tf_style) {
    c.step_size = lr * hw_sqrt(bc2) * hw_rcp(bc1);
    c.inv_sqrt_bc2 = 1.0f;
  } else {
    c.step_size = lr * hw_rcp(bc1);
    c.inv_sqrt_bc2 = hw_rcp(hw_sqrt(bc2));
  }
  c.eps = a.eps; c.b1 = a.beta1; c.b2 = a.beta2; c.wd = a.weight_decay; c.gscale = a.grad_scale;
  return c;
}

__device__ __forceinline__ AdamCoef adam_coef(const ArenaAdam& a) {
  return adam_coef_tl(a, a.t_ptr ? (float)(*a.t_ptr) : 1.0f, adam_lr(a));
}

__device__ __forceinline__ void adam_apply(const AdamCoef& c, float g, float& p, float& m, float& v) {
  g = g * c.gscale + c.wd * p;
  m = c.b1 * m + (1.0f - c.b1) * g;
  v = c.b2 * v + (1.0f - c.b2) * g * g;
  // torch: p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps);  tf: p -= lr_t * m / (sqrt(v) + eps)
  p -= c.step_size * m * hw_rcp(hw_sqrt(v) * c.inv_sqrt_bc2 + c.eps);
}

}  // namespace arena
