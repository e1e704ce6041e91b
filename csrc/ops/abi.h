// Plain-C ABI shared by the HIP kernel TUs and the host binding TU (no device code here).
#pragma once
#include <stdint.h>

// ----------------------------------------------------------------------------------------------
// Host-visible plain-C ABI structs shared with the torch binding TU (bindings.cpp).
// ----------------------------------------------------------------------------------------------
extern "C" {

// Where the rows of an A operand (or the labels) come from. Row r of the logical batch is
//   phys = idx ? idx[((*cursor + cursor_off) * batch + r) % idx_len] : r
// which fuses the data-loader gather (dataset permutation + per-step cursor) into the GEMM.
struct ArenaRowSource {
  const void* ptr;
  int dtype;            // 0 = f32, 1 = u8, 2 = i32, 3 = i64
  int ld;               // row stride in elements
  float scale;          // multiplied on load (1/255 for u8 pixels)
  const int* idx;       // optional gather permutation (device)
  long long idx_len;
  const long long* cursor;  // optional device counter (completed steps)
  int cursor_off;       // added to *cursor (lets a kernel read the step counter it does not commit)
  int batch;            // rows consumed per cursor step
};

// Device step counters: dst = (src ? *src : 0) + add, executed by one lane of block 0.
struct ArenaCounterOp {
  long long* dst;
  const long long* src;
  int add;
};

struct ArenaAdam {
  float lr;               // used when lr_ptr == nullptr
  const float* lr_ptr;    // optional device learning rate (schedules under graph replay)
  float beta1, beta2, eps, weight_decay;
  const long long* t_ptr; // device Adam step t (1-based) for bias correction
  float grad_scale;       // e.g. 1/world_size for averaged all-reduce gradients
  int tf_style;           // 1: TF AdamOptimizer epsilon placement, 0: torch.optim.Adam
};

// One layer of a grouped weight-gradient launch (wgrad_grouped).
struct ArenaWGradProblem {
  ArenaRowSource x;       // rows m of the layer input
  int xt;                 // 0 f32, 1 u8
  const float* dz;        // [M][N] upstream gradient (null when recomputed from the head below)
  // dz recomputed in-kernel from the softmax head (fused MLP step):
  //   dz[m][n] = (Σ_c hd_dl[m][c] * hd_w2[c][n]) * (hd_h[m][n] > 0 ? hd_inv_keep : 0)
  const float* hd_dl;     // [M][hd_c] dlogits
  const float* hd_w2;     // [hd_c][N] next-layer weight
  const float* hd_h;      // [M][N] this layer's (post-dropout) activation, for the ReLU/drop mask
  int hd_c;
  float hd_inv_keep;
  int M, K, N;
  int mode;               // 0: write grad (scaled), 1: Adam in place
  float* gW; float* gB;   // mode 0 outputs ([K][N], [N]); gB may be null
  float* pW; float* mW; float* vW;  // mode 1
  float* pB; float* mB; float* vB;
  int tiles_k, tiles_n, block_begin;
};

// Fused forward + loss head of a 1-hidden-layer MLP (mlp_fwd_head).
struct ArenaFwdHead {
  const float* W2;        // [C][N] output layer
  const float* b2;        // [C]
  int C;
  ArenaRowSource lab;     // labels (same gather as x)
  float* slabs;           // workspace [mtiles][ntiles][16][C] partial logits
  int* counters;          // workspace [mtiles], zero-initialised once; reset by the last arriver
  float* dlogits;         // [M][C] out (null: metrics only)
  float* W2_copy;         // optional [C][N] snapshot of W2 (backward reads it while Adam updates W2)
  float loss_scale;
  float* loss_acc; int* correct_acc; int hist_len; const long long* hist_step;
};

}  // extern "C"
