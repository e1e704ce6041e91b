// Plain-C ABI shared by the HIP kernel TUs and the host binding TU (no device code here).
#pragma once
#include <stdint.h>

// BatchNorm statistics accumulators ("acc mode", bn_kernels.hip / conv_kernels.hip): every fp64
// set is ARENA_ACC_REP consecutive [2][C] replicas; a consumer sums all of them, in replica order.
// The conv epilogues (up to 3136 tiles per channel at batch 128) add row tile mt's sums into
// replica mt % ARENA_ACC_REP, so their same-address fp64 atomics do not serialize; the BN passes'
// reductions (at most 512 block sums per channel) add into replica 0.
#define ARENA_ACC_REP 4

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
  const float* dz;        // [M][N] upstream gradient (null when derived from the softmax head)
  // Softmax-head modes (fused MLP step, see ArenaHead):
  //   hd_mode 1: dz = dlogits                               (output layer, N == C)
  //   hd_mode 2: dz = (dlogits · hd_w2) ⊙ (hd_h > 0) / keep  (hidden layer: ReLU+dropout bwd)
  int hd_mode;
  const float* hd_w2;     // [C][N] W2 snapshot (mode 2)
  const float* hd_h;      // [M][N] post-dropout activation, mask source (mode 2)
  float hd_inv_keep;
  int M, K, N;
  int mode;               // 0: write grad (scaled), 1: Adam in place
  float* gW; float* gB;   // mode 0 outputs ([N][K], [N]); gB may be null
  float* pW; float* mW; float* vW;  // mode 1
  float* pB; float* mB; float* vB;
  int tiles_k, tiles_n, block_begin;
};

// Softmax-cross-entropy head recomputed inside every wgrad workgroup from the raw logits that the
// forward kernel accumulated (100 x 10 for MNIST: cheaper than any inter-workgroup hand-off).
// logits2 is double-buffered by step parity: step t accumulates into buffer t&1 while the wgrad
// of step t zeroes buffer (t+1)&1 for the next forward.
struct ArenaHead {
  float* logits2;           // [2][M][C] Σ over hidden tiles of H·W2ᵀ (no bias)
  const long long* step;    // device step counter: (*step + step_off) = index of this step
  int step_off;
  int parity;               // -1: buffer (*step + step_off) & 1; 0/1: known at launch, so the
                            // logits loads need not wait for the step counter
  const float* b2;          // [C]
  int C;
  ArenaRowSource lab;       // labels (same gather as the layer input)
  float loss_scale;         // 1/batch (mean loss)
  float* loss_acc; int* correct_acc; int hist_len;  // metric ring (block 0), power of two
  // optional: the NEXT step's dataset rows, nr_out[r] = nr_perm[((step + 1) * nr_batch + r) %
  // nr_len], written by the head block so the next forward skips the cursor -> permutation hop
  const int* nr_perm; long long nr_len; int nr_batch; int* nr_out;
};


// Fused training BatchNorm (csrc/ops/bn_kernels.hip). Per-channel fp32 arrays of length C.
struct ArenaBNStats {
  float eps, momentum;
  const float* gamma;     // optional (affine off -> 1)
  const float* beta;      // optional (-> 0)
  float* mean;            // out (training) / in (eval: running mean): batch mean
  float* invstd;          // out: 1 / sqrt(biased var + eps)
  float* scale;           // out (training) / in (eval): gamma * invstd
  float* shift;           // out (training) / in (eval): beta;  y = (x - mean) * scale + shift
  float* running_mean;    // optional, updated in place with momentum (unbiased variance)
  float* running_var;
  long long* batches;     // optional nn.BatchNorm num_batches_tracked, += 1 by the finalize kernel
};

struct ArenaBNBwd {
  const float* mean;      // saved batch statistics of the forward
  const float* invstd;
  const float* gamma;     // optional
  float* dgamma;          // optional outputs
  float* dbeta;
  float* ca; float* cb; float* cc;  // workspace [C] each: dx = ca * (g - cb - (x - mean) * cc)
  // the forward's y = act((x - mean) * scale + shift): the fused stem (BN + ReLU + max pool,
  // arena_bn_pool_bwd) recomputes its ReLU mask from x with them
  const float* scale; const float* shift;
};

// Intra-node xGMI collective (csrc/ccl/xgmi_ccl.hip): every rank's registered buffers, mapped into
// this process through hipIpc handles (buf[rank] / sig[rank] are the local allocations).
#define ARENA_CCL_MAX_RANKS 8
#define ARENA_CCL_MAX_BLOCKS 256
// One-shot allreduce region: 2 x ONESHOT_ELEMS floats (double-buffered by call parity) that sit
// right after the buf_elems floats of every staging buffer (the host allocates them).
#define ARENA_CCL_ONESHOT_ELEMS 16384
// barrier phases per call (the scatter + all-gather broadcast uses three)
#define ARENA_CCL_PHASES 3
struct ArenaXgmiPeers {
  float* buf[ARENA_CCL_MAX_RANKS];    // staging / gradient buffer of each rank (+ one-shot tail)
  float* buf2[ARENA_CCL_MAX_RANKS];   // second buffer (parameters for the fused Adam step)
  uint32_t* sig[ARENA_CCL_MAX_RANKS]; // uncached flags: [3 phases][MAX_BLOCKS][MAX_RANKS]
  uint32_t* epoch;                    // local, per block: calls completed
  int* err;                           // local: set to 1 when a barrier wait timed out
  long long buf_elems;                // capacity of buf[] (floats)
  long long buf2_elems;
  int rank, world;
  // 0 (default): every kernel stores only into this rank's own buffers and peers PULL the owner's
  // chunk after a barrier; 1: the owner pushes its chunk into every peer's buffer (one barrier
  // less for the two-shot allreduce; used only when its own construction-time self-test passed)
  int push;
  long long timeout_cycles;           // barrier wait bound in s_memrealtime ticks (100 MHz)
};
}  // extern "C"
