// PyTorch binding for the arena_amd HIP kernels. Validates every shape/dtype/device on the host
// BEFORE launching (a kernel that faults on an MI355X can reset the node), then calls the plain-C
// launchers in mlp_kernels.hip on the current HIP stream (so hipGraph capture via torch works).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>

#include <cstring>
#include <string>
#include <vector>

#include "abi.h"

extern "C" {
hipError_t arena_linear_fwd(ArenaRowSource, const float*, const float*, float*, int, int, int, int,
                            float, uint32_t, const long long*, hipStream_t);
hipError_t arena_mlp_fwd_logits(ArenaRowSource, const float*, const float*, float*, int, int, int,
                                float, uint32_t, const long long*, const float*, float*, int,
                                float*, uint8_t*, const void*, int, int*, ArenaCounterOp,
                                const int*, hipStream_t);
hipError_t arena_xent_head(const float*, int, int, const float*, const float*, int, ArenaRowSource,
                           float*, float*, float, int, float, float*, int*, int, const long long*,
                           ArenaCounterOp, hipStream_t);
hipError_t arena_wgrad_grouped(ArenaWGradProblem*, int, ArenaAdam, float, ArenaCounterOp, ArenaHead,
                               hipStream_t);
hipError_t arena_adam_flat(float*, float*, float*, const float*, long long, ArenaAdam,
                           ArenaCounterOp, hipStream_t);
hipError_t arena_sgd_flat(float*, const float*, long long, float, const float*, float, hipStream_t);
hipError_t arena_softmax_xent(const float*, const long long*, int, int, float*, float*, float,
                              hipStream_t);
hipError_t arena_mt_copy_scale(float* const*, const long long*, const long long*, int, float*, float,
                               int, hipStream_t);
hipError_t arena_mt_sgd_master(const void* const*, const long long*, const long long*, int,
                               float*, float*, void*, float, float, float, hipStream_t);
hipError_t arena_shard_sgd(const void*, int, float*, float*, void*, long long, float, float, float,
                           float, hipStream_t);
// csrc/ccl/xgmi_ccl.hip
hipError_t arena_ccl_malloc(void**, size_t, int);
hipError_t arena_ccl_free(void*);
hipError_t arena_ccl_memset(void*, int, size_t);
hipError_t arena_ccl_ipc_get(void*, void*);
hipError_t arena_ccl_ipc_open(const void*, void**);
hipError_t arena_ccl_ipc_close(void*);
hipError_t arena_ccl_allreduce(const ArenaXgmiPeers*, const float*, float*, long long, float,
                               hipStream_t);
hipError_t arena_ccl_adam(const ArenaXgmiPeers*, float*, float*, long long, ArenaAdam,
                          ArenaCounterOp, hipStream_t);
void arena_ccl_shard(long long, int, int, long long*, long long*);
hipError_t arena_ccl_broadcast(const ArenaXgmiPeers*, const float*, float*, long long, int,
                               hipStream_t);
hipError_t arena_ccl_allgather(const ArenaXgmiPeers*, const float*, float*, long long,
                               hipStream_t);
void arena_ccl_set_bcast_direct_max(long long);
hipError_t arena_ccl_sgd_bf16(const ArenaXgmiPeers*, float*, float*, long long, long long, float,
                              float, float, float, hipStream_t);
void arena_ccl_sgd_shard(long long, long long, int, int, long long*, long long*);
hipError_t arena_ccl_sgd_f32(const ArenaXgmiPeers*, float*, long long, long long, float, float,
                             float, float, hipStream_t);
void arena_ccl_sgd_f32_shard(long long, long long, int, int, long long*, long long*);
void arena_ccl_set_block_elems(long long);
void arena_ccl_set_max_blocks(int);
void arena_bn_set_elem_max_blocks(int);
void arena_bn_set_dx_max_blocks(int);
void arena_bn_set_slice(int);
void arena_ccl_set_oneshot_max(long long);
long long arena_ccl_get_oneshot_max();
// csrc/ops/conv_kernels.hip
hipError_t arena_conv_fwd(const void*, const void*, void*, float*, const void*, const void*,
                          const uint8_t*, const float*, int, int, int, int, int, int, int, int,
                          int, int, hipStream_t);
hipError_t arena_conv_flip_weight(const void*, void*, int, int, int, int, hipStream_t);
hipError_t arena_conv_flip_multi(int, const void* const*, void* const*, const int*, const int*,
                                 const int*, hipStream_t);
hipError_t arena_conv_fwd_ex(const void*, const void*, void*, float*, const void*, const uint8_t*,
                             const void*, const uint8_t*, const float*, int, int, int, int, int,
                             int, int, int, int, int, int, int, const int*, int, int, double*,
                             int, void*, unsigned*, hipStream_t);
hipError_t arena_conv_fwd_phases(const void*, void*, const void*, int, int, int, int, int, int,
                                 int, int, int, int, const void* const*, const int*, const int*,
                                 const int*, const int*, const int*, const int*, const int*,
                                 const int*, int, hipStream_t);
long long arena_conv_fwd_ksplit_floats(long long, int, int, int);
void arena_conv_set_stats_one_pass(int);
void arena_conv_set_dbg(int);
long long arena_conv_fwd_tiles(long long, int, int);
int arena_conv_fwd_tile_rows(int);
hipError_t arena_conv_wgrad_ex(const void*, const void*, float*, void*, float*, int, int, int, int,
                               int, int, int, int, int, int, int, int, int, int, int, float,
                               hipStream_t);
hipError_t arena_s2d_stem(const void*, void*, int, int, int, int, int, hipStream_t);
hipError_t arena_stem_weight(const void*, void*, int, int, long long, long long, long long,
                             long long, int, hipStream_t);
hipError_t arena_stem_weight_grad(const void*, void*, int, int, long long, long long, long long,
                                  long long, int, hipStream_t);
hipError_t arena_conv_phase_weights(const void*, void*, int, int, int, int, int, int, long long*,
                                    hipStream_t);
int arena_conv_wgrad_splits(int, int, int, int, int, int, int);
hipError_t arena_conv_wgrad(const void*, const void*, float*, void*, float*, int, int, int, int,
                            int, int, int, int, int, int, int, float, hipStream_t);
// csrc/ops/bn_kernels.hip
long long arena_bn_workspace_floats(long long, int);
long long arena_bn_lvl2_doubles(long long, int);
void arena_bn_set_reduce_geometry(long long, long long);
void arena_bn_set_fin_max_blocks(int);
void arena_bn_set_nt(int);
void arena_bn_set_pool_quad_mult(int);
// csrc/ops/pool_kernels.hip
hipError_t arena_maxpool_fwd(int, const void*, void*, uint8_t*, int, int, int, int, int, int, int,
                             hipStream_t);
hipError_t arena_maxpool_bwd(int, const void*, const uint8_t*, void*, int, int, int, int, int, int,
                             int, hipStream_t);
hipError_t arena_xent_fwd(int, const void*, const long long*, float*, float*, int, int,
                          hipStream_t);
hipError_t arena_gap_bwd(int, const void*, void*, int, int, int, float, hipStream_t);
hipError_t arena_xent_bwd(int, const void*, const long long*, const float*, const float*, void*,
                          int, int, hipStream_t);
hipError_t arena_bn_fwd(int, const void*, const void*, void*, uint8_t*, long long, int, int, int,
                        float*, int, long long, double*, unsigned*, ArenaBNStats, double*, int,
                        double*, int, hipStream_t);
hipError_t arena_bn_bwd(int, const void*, const uint8_t*, const void*, void*, void*, long long, int,
                        int, float*, int, double*, unsigned*, ArenaBNBwd, double*, int, double*,
                        int, const void*, const float*, double*, hipStream_t);
int arena_bn_acc_ok(long long, int);
hipError_t arena_bn_pool_fwd(int, const void*, void*, uint8_t*, void*, int, int, int, int, int, int,
                             int, ArenaBNStats, const double*, const float*, int, long long,
                             double*, unsigned*, double*, int, hipStream_t);
hipError_t arena_bn_pool_bwd(int, const void*, const uint8_t*, const void*, const void*, void*, int,
                             int, int, int, int, int, int, ArenaBNBwd, double*, double*, int,
                             hipStream_t);
#ifdef ARENA_TIMELINE
hipError_t arena_timeline_read(long long*, int);
#endif
}

namespace {

using torch::Tensor;
using OptT = c10::optional<Tensor>;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_hip(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "arena_amd HIP launch failed in ", what, ": ", hipGetErrorString(e));
}

void check_dev(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void check_f32(const Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be float32");
}

const long long* opt_i64_scalar(const OptT& t, const char* name) {
  if (!t.has_value()) return nullptr;
  check_dev(*t, name);
  TORCH_CHECK(t->scalar_type() == torch::kInt64 && t->numel() >= 1, name,
              " must be an int64 device tensor with >=1 element");
  return reinterpret_cast<const long long*>(t->data_ptr<int64_t>());
}

int dtype_code(const Tensor& t) {
  switch (t.scalar_type()) {
    case torch::kFloat32: return 0;
    case torch::kUInt8: return 1;
    case torch::kInt32: return 2;
    case torch::kInt64: return 3;
    default: TORCH_CHECK(false, "unsupported dtype ", t.scalar_type());
  }
  return -1;
}

// x: [rows, ld] (2-D) or [rows] (1-D labels). Logical row r reads physical row
// idx[(cursor*batch + r) % len(idx)] when idx is given, else row r (checked against rows).
ArenaRowSource make_src(const Tensor& x, double scale, const OptT& idx, const OptT& cursor,
                        int64_t batch, int64_t logical_rows, const char* name,
                        int64_t cursor_off = 0) {
  check_dev(x, name);
  ArenaRowSource s{};
  s.ptr = x.data_ptr();
  s.dtype = dtype_code(x);
  s.ld = x.dim() >= 2 ? (int)x.size(1) : 1;
  s.scale = (float)scale;
  s.idx = nullptr;
  s.idx_len = 0;
  s.cursor = opt_i64_scalar(cursor, "cursor");
  s.batch = (int)batch;
  s.cursor_off = (int)cursor_off;
  if (idx.has_value()) {
    check_dev(*idx, "idx");
    TORCH_CHECK(idx->scalar_type() == torch::kInt32, "idx must be int32");
    TORCH_CHECK(idx->numel() > 0, "idx must be non-empty");
    s.idx = idx->data_ptr<int>();
    s.idx_len = idx->numel();
    TORCH_CHECK(logical_rows <= s.idx_len, name, ": batch rows (", logical_rows,
                ") must not exceed the gather index length (", s.idx_len, ")");
    TORCH_CHECK(batch >= 0, "batch must be >= 0");
    // Every index value must be a valid row: checked once on the host when the permutation is
    // installed (arena_amd/data/device_loader.py), not per launch (launches are graph-captured).
  } else {
    TORCH_CHECK(logical_rows <= x.size(0), name, ": ", logical_rows, " rows requested but tensor has ",
                x.size(0));
  }
  return s;
}

// Y = dropout(act(X·W + b)); X rows optionally gathered (dataset permutation + device cursor).
void linear_fwd(Tensor x, double x_scale, OptT idx, OptT cursor, int64_t batch, Tensor W, OptT bias,
                Tensor Y, int64_t act, double keep_prob, int64_t seed, OptT step) {
  check_f32(W, "W");
  check_f32(Y, "Y");
  TORCH_CHECK(W.dim() == 2 && Y.dim() == 2 && x.dim() == 2, "linear_fwd: 2-D tensors required");
  // W is [out, in] (nn.Linear layout)
  const int64_t M = Y.size(0), N = Y.size(1), K = W.size(1);
  TORCH_CHECK(W.size(0) == N, "W.shape[0] must equal Y.shape[1]");
  TORCH_CHECK(x.size(1) == K, "x.shape[1] must equal W.shape[1]");
  TORCH_CHECK(K % 4 == 0, "linear_fwd: K must be a multiple of 4 (got ", K, ")");
  TORCH_CHECK(x.scalar_type() == torch::kFloat32 || x.scalar_type() == torch::kUInt8,
              "x must be float32 or uint8");
  TORCH_CHECK(M > 0 && N > 0, "empty linear");
  const float* b = nullptr;
  if (bias.has_value()) {
    check_f32(*bias, "bias");
    TORCH_CHECK(bias->numel() == N, "bias size mismatch");
    b = bias->data_ptr<float>();
  }
  TORCH_CHECK(keep_prob > 0.0 && keep_prob <= 1.0, "keep_prob must be in (0, 1]");
  ArenaRowSource s = make_src(x, x_scale, idx, cursor, batch, M, "x");
  check_hip(arena_linear_fwd(s, W.data_ptr<float>(), b, Y.data_ptr<float>(), (int)M, (int)N, (int)K,
                             (int)act, (float)keep_prob, (uint32_t)seed, opt_i64_scalar(step, "step"),
                             cur_stream()),
            "linear_fwd");
}

// Hidden layer forward that also accumulates the output layer's logits (mlp_fwd_logits_kernel).
// logits2 [2, M, C] must be zero in buffer (step & 1) before the launch (the fused wgrad zeroes
// the other buffer each step; zero both once at setup).
void mlp_fwd_logits(Tensor x, double x_scale, OptT idx, OptT cursor, int64_t batch, Tensor W1,
                    Tensor b1, Tensor H, double keep_prob, int64_t seed, OptT step, Tensor W2,
                    OptT W2_copy, Tensor logits2, OptT xb, OptT labels, OptT yb, OptT ctr_dst,
                    OptT ctr_src, int64_t ctr_add, OptT rows) {
  for (auto* t : {&W1, &b1, &H, &W2, &logits2}) check_f32(*t, "mlp_fwd_logits operand");
  const int64_t M = H.size(0), N = H.size(1), K = W1.size(1), C = W2.size(0);
  TORCH_CHECK(W1.dim() == 2 && W1.size(0) == N && x.dim() == 2 && x.size(1) == K,
              "mlp_fwd_logits: W1 [N, K], x [*, K], H [M, N]");
  TORCH_CHECK(K % 4 == 0, "K must be a multiple of 4");
  TORCH_CHECK(b1.numel() == N, "b1 size");
  TORCH_CHECK(W2.dim() == 2 && W2.size(1) == N && C >= 1 && C <= 16, "W2 must be [C<=16, N]");
  TORCH_CHECK(logits2.numel() == 2 * M * C, "logits2 must be [2, M, C]");
  TORCH_CHECK(x.scalar_type() == torch::kFloat32 || x.scalar_type() == torch::kUInt8, "x dtype");
  TORCH_CHECK(keep_prob > 0.0 && keep_prob <= 1.0, "keep_prob in (0, 1]");
  float* w2c = nullptr;
  if (W2_copy.has_value()) {
    check_f32(*W2_copy, "W2_copy");
    TORCH_CHECK(W2_copy->numel() == C * N, "W2_copy size");
    w2c = W2_copy->data_ptr<float>();
  }
  ArenaCounterOp ctr{};
  if (ctr_dst.has_value()) {
    ctr.dst = const_cast<long long*>(opt_i64_scalar(ctr_dst, "ctr_dst"));
    ctr.src = opt_i64_scalar(ctr_src, "ctr_src");
    ctr.add = (int)ctr_add;
  }
  // optional publication of the gathered batch (u8 rows -> xb [M, K], labels -> yb [M] int32)
  uint8_t* pxb = nullptr;
  int* pyb = nullptr;
  const void* plab = nullptr;
  int lab_dtype = 0;
  if (xb.has_value()) {
    check_dev(*xb, "xb");
    TORCH_CHECK(x.scalar_type() == torch::kUInt8 && xb->scalar_type() == torch::kUInt8 &&
                    xb->numel() == M * K,
                "xb must be uint8 [M, K] (u8 input only)");
    TORCH_CHECK(labels.has_value() && yb.has_value(), "xb requires labels and yb");
    check_dev(*labels, "labels");
    check_dev(*yb, "yb");
    TORCH_CHECK(yb->scalar_type() == torch::kInt32 && yb->numel() == M, "yb must be int32 [M]");
    TORCH_CHECK(labels->dim() == 1 && labels->size(0) >= x.size(0) &&
                    labels->scalar_type() != torch::kFloat32,
                "labels must be integer [rows of x]");
    pxb = xb->data_ptr<uint8_t>();
    pyb = yb->data_ptr<int>();
    plab = labels->data_ptr();
    lab_dtype = dtype_code(*labels);
  }
  ArenaRowSource s = make_src(x, x_scale, idx, cursor, batch, M, "x");
  const int* prows = nullptr;
  if (rows.has_value()) {  // this step's dataset rows (each must index x)
    check_dev(*rows, "rows");
    TORCH_CHECK(rows->scalar_type() == torch::kInt32 && rows->numel() == M,
                "rows must be int32 [M]");
    TORCH_CHECK(idx.has_value(), "rows replaces the idx/cursor gather: pass idx too");
    prows = rows->data_ptr<int>();
  }
  check_hip(arena_mlp_fwd_logits(s, W1.data_ptr<float>(), b1.data_ptr<float>(),
                                 H.data_ptr<float>(), (int)M, (int)N, (int)K, (float)keep_prob,
                                 (uint32_t)seed, opt_i64_scalar(step, "step"), W2.data_ptr<float>(),
                                 w2c, (int)C, logits2.data_ptr<float>(), pxb, plab, lab_dtype, pyb,
                                 ctr, prows, cur_stream()),
            "mlp_fwd_logits");
}

void xent_head(Tensor H, Tensor W2, OptT b2, Tensor labels, OptT idx, OptT cursor, int64_t batch,
               OptT dlogits, OptT dZ, double keep_prob, bool relu_mask, double loss_scale,
               Tensor loss_acc, Tensor correct_acc, OptT hist_step, OptT ctr_dst, OptT ctr_src,
               int64_t ctr_add) {
  check_f32(H, "H");
  check_f32(W2, "W2");
  // W2 is [classes, hidden]
  const int64_t M = H.size(0), D = H.size(1), C = W2.size(0);
  TORCH_CHECK(W2.size(1) == D, "W2.shape[1] must equal H.shape[1]");
  TORCH_CHECK(D <= 1024 && C <= 16 && D * C <= 16384 && (D * C) % 4 == 0,
              "xent_head: D<=1024, C<=16, D*C<=16384, D*C % 4 == 0");
  TORCH_CHECK(labels.dim() == 1, "labels must be 1-D");
  const float* pb2 = nullptr;
  if (b2.has_value()) {
    check_f32(*b2, "b2");
    TORCH_CHECK(b2->numel() == C, "b2 size");
    pb2 = b2->data_ptr<float>();
  }
  float* pdl = nullptr;
  float* pdz = nullptr;
  if (dlogits.has_value()) {
    check_f32(*dlogits, "dlogits");
    TORCH_CHECK(dlogits->numel() == M * C, "dlogits size");
    pdl = dlogits->data_ptr<float>();
  }
  if (dZ.has_value()) {
    TORCH_CHECK(pdl != nullptr, "dZ requires dlogits");
    check_f32(*dZ, "dZ");
    TORCH_CHECK(dZ->numel() == M * D, "dZ size");
    pdz = dZ->data_ptr<float>();
  }
  check_f32(loss_acc, "loss_acc");
  check_dev(correct_acc, "correct_acc");
  TORCH_CHECK(correct_acc.scalar_type() == torch::kInt32, "correct_acc must be int32");
  TORCH_CHECK(loss_acc.numel() == correct_acc.numel() && loss_acc.numel() >= 1, "acc sizes");
  TORCH_CHECK((loss_acc.numel() & (loss_acc.numel() - 1)) == 0,
              "metric history length must be a power of two");
  TORCH_CHECK(labels.scalar_type() != torch::kFloat32, "labels must be integer");
  ArenaRowSource lab = make_src(labels, 1.0, idx, cursor, batch, M, "labels");
  ArenaCounterOp ctr{};
  if (ctr_dst.has_value()) {
    ctr.dst = const_cast<long long*>(opt_i64_scalar(ctr_dst, "ctr_dst"));
    ctr.src = opt_i64_scalar(ctr_src, "ctr_src");
    ctr.add = (int)ctr_add;
  }
  check_hip(arena_xent_head(H.data_ptr<float>(), (int)M, (int)D, W2.data_ptr<float>(), pb2, (int)C,
                            lab, pdl, pdz, (float)keep_prob, relu_mask ? 1 : 0, (float)loss_scale,
                            loss_acc.data_ptr<float>(), correct_acc.data_ptr<int>(),
                            (int)loss_acc.numel(), opt_i64_scalar(hist_step, "hist_step"), ctr,
                            cur_stream()),
            "xent_head");
}

ArenaAdam make_adam(double lr, OptT lr_t, double b1, double b2, double eps, double wd, OptT t_step,
                    double grad_scale, bool tf_style) {
  ArenaAdam a{};
  a.lr = (float)lr;
  a.lr_ptr = nullptr;
  if (lr_t.has_value()) {
    check_f32(*lr_t, "lr");
    a.lr_ptr = lr_t->data_ptr<float>();
  }
  a.beta1 = (float)b1; a.beta2 = (float)b2; a.eps = (float)eps; a.weight_decay = (float)wd;
  a.t_ptr = opt_i64_scalar(t_step, "t_step");
  a.grad_scale = (float)grad_scale;
  a.tf_style = tf_style ? 1 : 0;
  return a;
}

// problems: list of dicts is awkward across pybind; use parallel lists of tensors instead.
// Each layer i: x_i (f32 or u8 [rows, K]), x_scale_i, dz_i [M, N]; mode 0 -> gW_i/gB_i views,
// mode 1 -> (pW,mW,vW,pB,mB,vB) views. One shared gather (idx, cursor, batch) is applied to
// layers flagged gather=True (the dataset-fed first layer).
void wgrad_grouped(std::vector<Tensor> xs, std::vector<double> x_scales, std::vector<bool> gather,
                   OptT idx, OptT cursor, int64_t cursor_off, int64_t batch,
                   std::vector<OptT> dzs, std::vector<int64_t> hd_modes,
                   std::vector<OptT> hd_w2, std::vector<OptT> hd_h, double hd_keep_prob,
                   OptT hd_logits2, OptT hd_step, int64_t hd_step_off, OptT hd_b2,
                   OptT hd_labels, double hd_loss_scale, OptT hd_loss_acc,
                   OptT hd_correct_acc, int64_t mode,
                   std::vector<Tensor> outW, std::vector<OptT> outB, std::vector<OptT> mW,
                   std::vector<OptT> vW, std::vector<OptT> mB, std::vector<OptT> vB, double lr,
                   OptT lr_t, double b1, double b2, double eps, double wd, OptT t_step,
                   double grad_scale, bool tf_style, OptT ctr_dst, OptT ctr_src, int64_t ctr_add,
                   OptT next_rows, OptT next_rows_perm, int64_t hd_parity) {
  const size_t n = xs.size();
  TORCH_CHECK(hd_parity >= -1 && hd_parity <= 1, "hd_parity must be -1 (from the counter), 0 or 1");
  TORCH_CHECK(n >= 1 && n <= 2, "wgrad_grouped: 1..2 problems");
  TORCH_CHECK(x_scales.size() == n && gather.size() == n && dzs.size() == n && outW.size() == n &&
                  outB.size() == n && hd_modes.size() == n && hd_w2.size() == n &&
                  hd_h.size() == n,
              "wgrad_grouped: list lengths differ");
  if (mode == 1)
    TORCH_CHECK(mW.size() == n && vW.size() == n && mB.size() == n && vB.size() == n,
                "adam state lists");
  std::vector<ArenaWGradProblem> probs(n);
  for (size_t i = 0; i < n; ++i) {
    ArenaWGradProblem& P = probs[i];
    P = ArenaWGradProblem{};
    const Tensor& x = xs[i];
    int64_t M = 0, N = 0;
    if (hd_modes[i] == 0) {
      TORCH_CHECK(dzs[i].has_value(), "wgrad_grouped: problem ", i, " needs dz");
      const Tensor& dz = *dzs[i];
      check_f32(dz, "dz");
      TORCH_CHECK(dz.dim() == 2, "dz must be 2-D");
      M = dz.size(0);
      N = dz.size(1);
      P.dz = dz.data_ptr<float>();
    } else {
      TORCH_CHECK(hd_logits2.has_value() && hd_labels.has_value() && hd_step.has_value() &&
                      hd_loss_acc.has_value() && hd_correct_acc.has_value(),
                  "head mode needs logits2, labels, step and metric buffers");
      const int64_t C = hd_logits2->size(-1);
      M = hd_logits2->size(-2);
      TORCH_CHECK(hd_logits2->dim() == 3 && hd_logits2->size(0) == 2 && C >= 1 && C <= 16,
                  "hd_logits2 must be [2, M, C<=16]");
      P.dz = nullptr;
      P.hd_mode = (int)hd_modes[i];
      if (hd_modes[i] == 1) {
        N = C;
      } else {
        TORCH_CHECK(hd_modes[i] == 2 && hd_w2[i].has_value() && hd_h[i].has_value(),
                    "hd_mode 2 needs hd_w2 and hd_h");
        const Tensor& w2 = *hd_w2[i];
        const Tensor& h = *hd_h[i];
        check_f32(w2, "hd_w2");
        check_f32(h, "hd_h");
        TORCH_CHECK(h.dim() == 2 && h.size(0) == M, "hd_h must be [M, N]");
        N = h.size(1);
        TORCH_CHECK(w2.dim() == 2 && w2.size(0) == C && w2.size(1) == N, "hd_w2 must be [C, N]");
        TORCH_CHECK(N % 4 == 0, "head mode 2 needs N % 4 == 0");
        P.hd_w2 = w2.data_ptr<float>();
        P.hd_h = h.data_ptr<float>();
      }
      TORCH_CHECK(hd_keep_prob > 0.0 && hd_keep_prob <= 1.0, "hd_keep_prob in (0, 1]");
      P.hd_inv_keep = (float)(1.0 / hd_keep_prob);
    }
    const int64_t K = x.size(1);
    TORCH_CHECK(K % 4 == 0, "wgrad: K must be a multiple of 4");
    TORCH_CHECK(x.scalar_type() == torch::kFloat32 || x.scalar_type() == torch::kUInt8,
                "x must be f32/u8");
    P.x = gather[i] ? make_src(x, x_scales[i], idx, cursor, batch, M, "x", cursor_off)
                    : make_src(x, x_scales[i], c10::nullopt, c10::nullopt, 0, M, "x");
    P.xt = x.scalar_type() == torch::kUInt8 ? 1 : 0;
    P.M = (int)M; P.K = (int)K; P.N = (int)N;
    P.mode = (int)mode;
    check_f32(outW[i], "W");
    TORCH_CHECK(outW[i].numel() == K * N, "W/grad size mismatch for problem ", i);
    if (outB[i].has_value()) {
      check_f32(*outB[i], "b");
      TORCH_CHECK(outB[i]->numel() == N, "bias size");
    }
    if (mode == 0) {
      P.gW = outW[i].data_ptr<float>();
      P.gB = outB[i].has_value() ? outB[i]->data_ptr<float>() : nullptr;
    } else {
      P.pW = outW[i].data_ptr<float>();
      TORCH_CHECK(mW[i].has_value() && vW[i].has_value(), "adam: mW/vW required");
      check_f32(*mW[i], "mW");
      check_f32(*vW[i], "vW");
      TORCH_CHECK(mW[i]->numel() == K * N && vW[i]->numel() == K * N, "adam W state size");
      P.mW = mW[i]->data_ptr<float>();
      P.vW = vW[i]->data_ptr<float>();
      if (outB[i].has_value()) {
        TORCH_CHECK(mB[i].has_value() && vB[i].has_value(), "adam: mB/vB required");
        check_f32(*mB[i], "mB");
        check_f32(*vB[i], "vB");
        TORCH_CHECK(mB[i]->numel() == N && vB[i]->numel() == N, "adam b state size");
        P.pB = outB[i]->data_ptr<float>();
        P.mB = mB[i]->data_ptr<float>();
        P.vB = vB[i]->data_ptr<float>();
      }
    }
  }
  ArenaAdam a = make_adam(lr, lr_t, b1, b2, eps, wd, t_step, grad_scale, tf_style);
  ArenaCounterOp ctr{};
  if (ctr_dst.has_value()) {
    ctr.dst = const_cast<long long*>(opt_i64_scalar(ctr_dst, "ctr_dst"));
    ctr.src = opt_i64_scalar(ctr_src, "ctr_src");
    ctr.add = (int)ctr_add;
  }
  ArenaHead head{};
  bool any_head = false;
  for (auto m : hd_modes) any_head |= (m != 0);
  if (any_head) {
    check_f32(*hd_logits2, "hd_logits2");
    head.logits2 = hd_logits2->data_ptr<float>();
    head.step = opt_i64_scalar(hd_step, "hd_step");
    head.step_off = (int)hd_step_off;
    head.parity = (int)hd_parity;
    head.C = (int)hd_logits2->size(-1);
    head.b2 = nullptr;
    if (hd_b2.has_value()) {
      check_f32(*hd_b2, "hd_b2");
      TORCH_CHECK(hd_b2->numel() == head.C, "hd_b2 size");
      head.b2 = hd_b2->data_ptr<float>();
    }
    const int64_t Mh = hd_logits2->size(1);
    TORCH_CHECK(hd_labels->dim() == 1 && hd_labels->scalar_type() != torch::kFloat32, "labels");
    // labels share the layer-input gather (first problem with gather=True), same cursor offset
    int gi = -1;
    for (size_t i = 0; i < n; ++i)
      if (gather[i]) { gi = (int)i; break; }
    head.lab = gi >= 0 ? make_src(*hd_labels, 1.0, idx, cursor, batch, Mh, "labels", cursor_off)
                       : make_src(*hd_labels, 1.0, c10::nullopt, c10::nullopt, 0, Mh, "labels");
    head.loss_scale = (float)hd_loss_scale;
    check_f32(*hd_loss_acc, "hd_loss_acc");
    check_dev(*hd_correct_acc, "hd_correct_acc");
    TORCH_CHECK(hd_correct_acc->scalar_type() == torch::kInt32 &&
                    hd_correct_acc->numel() == hd_loss_acc->numel(),
                "metric buffers");
    TORCH_CHECK((hd_loss_acc->numel() & (hd_loss_acc->numel() - 1)) == 0,
                "metric history length must be a power of two");
    head.loss_acc = hd_loss_acc->data_ptr<float>();
    head.correct_acc = hd_correct_acc->data_ptr<int>();
    head.hist_len = (int)hd_loss_acc->numel();
    if (next_rows.has_value()) {
      TORCH_CHECK(next_rows_perm.has_value(), "next_rows needs next_rows_perm");
      check_dev(*next_rows, "next_rows");
      check_dev(*next_rows_perm, "next_rows_perm");
      TORCH_CHECK(next_rows->scalar_type() == torch::kInt32 &&
                      next_rows_perm->scalar_type() == torch::kInt32,
                  "next_rows / next_rows_perm must be int32");
      TORCH_CHECK(next_rows->numel() <= 256 && next_rows->numel() <= next_rows_perm->numel(),
                  "next_rows: at most 256 rows, not more than the permutation");
      head.nr_out = next_rows->data_ptr<int>();
      head.nr_perm = next_rows_perm->data_ptr<int>();
      head.nr_len = next_rows_perm->numel();
      head.nr_batch = (int)next_rows->numel();
    }
  }
  check_hip(arena_wgrad_grouped(probs.data(), (int)n, a, (float)grad_scale, ctr, head,
                                cur_stream()),
            "wgrad_grouped");
}

void adam_flat(Tensor P, Tensor M, Tensor V, Tensor G, double lr, OptT lr_t, double b1, double b2,
               double eps, double wd, OptT t_step, double grad_scale, bool tf_style, OptT ctr_dst,
               OptT ctr_src, int64_t ctr_add) {
  for (auto* t : {&P, &M, &V, &G}) check_f32(*t, "adam_flat operand");
  const int64_t n = P.numel();
  TORCH_CHECK(M.numel() == n && V.numel() == n && G.numel() == n, "adam_flat size mismatch");
  TORCH_CHECK(n % 4 == 0, "adam_flat: numel must be a multiple of 4");
  ArenaAdam a = make_adam(lr, lr_t, b1, b2, eps, wd, t_step, grad_scale, tf_style);
  ArenaCounterOp ctr{};
  if (ctr_dst.has_value()) {
    ctr.dst = const_cast<long long*>(opt_i64_scalar(ctr_dst, "ctr_dst"));
    ctr.src = opt_i64_scalar(ctr_src, "ctr_src");
    ctr.add = (int)ctr_add;
  }
  check_hip(arena_adam_flat(P.data_ptr<float>(), M.data_ptr<float>(), V.data_ptr<float>(),
                            G.data_ptr<float>(), n, a, ctr, cur_stream()),
            "adam_flat");
}

void sgd_flat(Tensor P, Tensor G, double lr, OptT lr_t, double grad_scale) {
  check_f32(P, "P");
  check_f32(G, "G");
  TORCH_CHECK(P.numel() == G.numel() && P.numel() % 4 == 0, "sgd_flat sizes");
  const float* lp = nullptr;
  if (lr_t.has_value()) {
    check_f32(*lr_t, "lr");
    lp = lr_t->data_ptr<float>();
  }
  check_hip(arena_sgd_flat(P.data_ptr<float>(), G.data_ptr<float>(), P.numel(), (float)lr, lp,
                           (float)grad_scale, cur_stream()),
            "sgd_flat");
}

std::vector<Tensor> softmax_xent(Tensor logits, Tensor labels, double grad_scale, bool need_grad) {
  check_f32(logits, "logits");
  check_dev(labels, "labels");
  TORCH_CHECK(logits.dim() == 2, "logits must be 2-D");
  TORCH_CHECK(labels.scalar_type() == torch::kInt64 && labels.numel() == logits.size(0),
              "labels must be int64 [M]");
  const int64_t M = logits.size(0), C = logits.size(1);
  auto loss = torch::empty({M}, logits.options());
  Tensor dl;
  if (need_grad) dl = torch::empty_like(logits);
  // Labels outside [0, C) would read out of bounds: validated by the Python wrapper in debug mode
  // and by construction of the data pipeline (labels are class ids).
  check_hip(arena_softmax_xent(logits.data_ptr<float>(),
                               reinterpret_cast<const long long*>(labels.data_ptr<int64_t>()),
                               (int)M, (int)C, loss.data_ptr<float>(),
                               need_grad ? dl.data_ptr<float>() : nullptr, (float)grad_scale,
                               cur_stream()),
            "softmax_xent");
  if (need_grad) return {loss, dl};
  return {loss};
}

// dir 0: flat[off_i:off_i+n_i] = t_i * scale; dir 1: t_i = flat[...] * scale.
void mt_copy_scale(std::vector<Tensor> tensors, std::vector<int64_t> offsets, Tensor flat,
                   double scale, int64_t dir) {
  check_f32(flat, "flat");
  TORCH_CHECK(tensors.size() == offsets.size(), "offsets length");
  std::vector<float*> ptrs;
  std::vector<long long> offs, ns;
  for (size_t i = 0; i < tensors.size(); ++i) {
    check_f32(tensors[i], "tensor");
    TORCH_CHECK(offsets[i] >= 0 && offsets[i] + tensors[i].numel() <= flat.numel(),
                "mt_copy_scale: segment ", i, " out of bounds");
    ptrs.push_back(tensors[i].data_ptr<float>());
    offs.push_back(offsets[i]);
    ns.push_back(tensors[i].numel());
  }
  check_hip(arena_mt_copy_scale(ptrs.data(), offs.data(), ns.data(), (int)ptrs.size(),
                                flat.data_ptr<float>(), (float)scale, (int)dir, cur_stream()),
            "mt_copy_scale");
}

void mt_sgd_master(std::vector<Tensor> grads, std::vector<int64_t> offsets, Tensor master,
                   Tensor mom, Tensor wbf, double lr, double momentum, double weight_decay) {
  check_f32(master, "master");
  check_f32(mom, "mom");
  check_dev(wbf, "wbf");
  TORCH_CHECK(wbf.scalar_type() == torch::kBFloat16 && wbf.is_contiguous() &&
                  mom.numel() == master.numel() && wbf.numel() == master.numel(),
              "mt_sgd_master: flat buffers must be fp32/fp32/bf16 of equal size");
  TORCH_CHECK(grads.size() == offsets.size(), "offsets length");
  std::vector<const void*> ptrs;
  std::vector<long long> offs, ns;
  for (size_t i = 0; i < grads.size(); ++i) {
    const Tensor& g = grads[i];
    TORCH_CHECK(g.is_cuda() && g.device() == master.device(), "grad ", i,
                " must be on the master buffer's GPU");
    TORCH_CHECK(g.scalar_type() == torch::kBFloat16 && g.is_non_overlapping_and_dense(),
                "mt_sgd_master: grad ", i, " must be dense bf16");
    TORCH_CHECK(g.numel() % 4 == 0 && offsets[i] % 4 == 0 && offsets[i] >= 0 &&
                    offsets[i] + g.numel() <= master.numel(),
                "mt_sgd_master: segment ", i, " misaligned or out of bounds");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(g.data_ptr()) % 8 == 0, "grad ", i, " not 8B aligned");
    ptrs.push_back(g.data_ptr());
    offs.push_back(offsets[i]);
    ns.push_back(g.numel());
  }
  check_hip(arena_mt_sgd_master(ptrs.data(), offs.data(), ns.data(), (int)ptrs.size(),
                                master.data_ptr<float>(), mom.data_ptr<float>(), wbf.data_ptr(),
                                (float)lr, (float)momentum, (float)weight_decay, cur_stream()),
            "mt_sgd_master");
}

void shard_sgd(Tensor grad, Tensor w32, Tensor mom, c10::optional<Tensor> wbf, double lr,
               double momentum, double weight_decay, double scale) {
  check_f32(w32, "w32");
  check_f32(mom, "mom");
  check_dev(grad, "grad");
  const bool bf = grad.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(bf || grad.scalar_type() == torch::kFloat32, "shard_sgd: grad must be bf16 or fp32");
  TORCH_CHECK(grad.is_contiguous() && w32.is_contiguous() && mom.is_contiguous() &&
                  grad.device() == w32.device() && mom.device() == w32.device(),
              "shard_sgd: contiguous tensors on one GPU");
  const int64_t n = w32.numel();
  TORCH_CHECK(grad.numel() == n && mom.numel() == n && n % 4 == 0,
              "shard_sgd: equal sizes, a multiple of 4");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(w32.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(mom.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(grad.data_ptr()) % (bf ? 8 : 16) == 0,
              "shard_sgd: misaligned range");
  void* wp = nullptr;
  if (bf) {
    TORCH_CHECK(wbf.has_value(), "shard_sgd: bf16 gradients need the bf16 weight range");
    check_dev(*wbf, "wbf");
    TORCH_CHECK(wbf->scalar_type() == torch::kBFloat16 && wbf->is_contiguous() &&
                    wbf->numel() == n && reinterpret_cast<uintptr_t>(wbf->data_ptr()) % 8 == 0,
                "shard_sgd: wbf must be a dense, 8-byte aligned bf16 range of the same size");
    wp = wbf->data_ptr();
  } else {
    TORCH_CHECK(!wbf.has_value(), "shard_sgd: fp32 weights are their own masters (no wbf)");
  }
  check_hip(arena_shard_sgd(grad.data_ptr(), bf ? 1 : 0, w32.data_ptr<float>(),
                            mom.data_ptr<float>(), wp, n, (float)lr, (float)momentum,
                            (float)weight_decay, (float)scale, cur_stream()),
            "shard_sgd");
}

// ------------------------------------------------------------------------------ xGMI collective
int64_t ccl_malloc(int64_t bytes, bool uncached) {
  TORCH_CHECK(bytes > 0, "ccl_malloc: bytes must be positive");
  void* p = nullptr;
  check_hip(arena_ccl_malloc(&p, (size_t)bytes, uncached ? 1 : 0), "ccl_malloc");
  return reinterpret_cast<int64_t>(p);
}
void ccl_free(int64_t p) { check_hip(arena_ccl_free(reinterpret_cast<void*>(p)), "ccl_free"); }
void ccl_memset(int64_t p, int64_t v, int64_t bytes) {
  check_hip(arena_ccl_memset(reinterpret_cast<void*>(p), (int)v, (size_t)bytes), "ccl_memset");
}
py::bytes ccl_ipc_get(int64_t p) {
  char h[64];
  check_hip(arena_ccl_ipc_get(reinterpret_cast<void*>(p), h), "hipIpcGetMemHandle");
  return py::bytes(h, 64);
}
int64_t ccl_ipc_open(py::bytes handle) {
  std::string h = handle;
  TORCH_CHECK(h.size() == 64, "IPC handle must be 64 bytes");
  void* p = nullptr;
  check_hip(arena_ccl_ipc_open(h.data(), &p), "hipIpcOpenMemHandle");
  return reinterpret_cast<int64_t>(p);
}
void ccl_ipc_close(int64_t p) {
  check_hip(arena_ccl_ipc_close(reinterpret_cast<void*>(p)), "hipIpcCloseMemHandle");
}
// A float32 view of registered memory (no ownership: the communicator frees it).
Tensor ccl_tensor(int64_t p, int64_t numel, int64_t device) {
  auto opts = torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, device);
  return torch::from_blob(reinterpret_cast<void*>(p), {numel}, [](void*) {}, opts);
}
std::vector<int64_t> ccl_shard(int64_t n, int64_t world, int64_t rank) {
  long long lo = 0, hi = 0;
  arena_ccl_shard(n, (int)world, (int)rank, &lo, &hi);
  return {lo, hi};
}

// ---------------------------------------------------------------------- fused BatchNorm (NHWC)
// Activations are [M][C] rows: a 4-D channels_last tensor (M = N*H*W) or a 2-D [M][C] tensor.
struct BNGeom {
  long long M;
  int C;
  int dtype;  // 0 f32, 1 bf16
};

BNGeom bn_geom(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16 || t.scalar_type() == torch::kFloat32, name,
              " must be bfloat16 or float32");
  BNGeom g{};
  if (t.dim() == 4) {
    TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), name,
                " must be channels_last contiguous (NHWC)");
    g.C = (int)t.size(1);
  } else {
    TORCH_CHECK(t.dim() == 2 && t.is_contiguous(), name, " must be 4-D NHWC or 2-D [M][C]");
    g.C = (int)t.size(1);
  }
  g.M = g.C ? t.numel() / g.C : 0;
  g.dtype = t.scalar_type() == torch::kBFloat16 ? 1 : 0;
  TORCH_CHECK(arena_bn_workspace_floats(g.M, g.C) > 0, name, ": C=", g.C,
              " unsupported (need C % 8 == 0, C <= 2048, C/8 dividing 256) or empty tensor");
  return g;
}

void bn_same(const Tensor& a, const Tensor& b, const char* name) {
  TORCH_CHECK(a.sizes() == b.sizes() && a.scalar_type() == b.scalar_type(), name,
              " must match x in shape and dtype");
  bn_geom(b, name);
}

const float* bn_vec(const OptT& t, int C, const char* name) {
  if (!t.has_value()) return nullptr;
  check_f32(*t, name);
  TORCH_CHECK(t->numel() == C, name, " must have C=", C, " elements");
  return t->data_ptr<float>();
}

// Ticket counters of the BN finalize kernels (bn_kernels.hip, fin_level2): zero-initialised once
// per device and left zero by every launch. Consecutive launches take different sets, so two
// finalizes that overlap on different streams never share a counter.
constexpr int kTicketSets = 64, kTicketsPerSet = 32;  // 32 groups of 64 channels = C <= 2048

unsigned* bn_tickets(const Tensor& like) {
  static std::vector<Tensor> pools;
  static std::vector<unsigned> next;
  const int dev = like.get_device();
  if ((int)pools.size() <= dev) {
    pools.resize(dev + 1);
    next.resize(dev + 1, 0);
  }
  if (!pools[dev].defined()) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    check_hip(hipStreamIsCapturing(cur_stream(), &cs), "bn_tickets");
    TORCH_CHECK(cs == hipStreamCaptureStatusNone,
                "arena BatchNorm: run one eager step before capturing a graph (its ticket "
                "counters are allocated and zeroed on first use)");
    pools[dev] = torch::zeros({kTicketSets * kTicketsPerSet}, like.options().dtype(torch::kInt32));
    check_hip(hipStreamSynchronize(cur_stream()), "bn_tickets zero");
  }
  const unsigned set = next[dev]++ % kTicketSets;
  return reinterpret_cast<unsigned*>(pools[dev].data_ptr<int32_t>()) + set * kTicketsPerSet;
}

// Statistics accumulators of acc mode (conv_kernels.hip ConvArgs::bn_acc, bn_kernels.hip): a
// rotating pool of fp64 [kRep][2][C] sets (abi.h ARENA_ACC_REP replicas), zero when handed out.
// A forward set (conv epilogue or statistics pass -> apply pass) is zeroed by its layer's
// backward dx pass (bn_bwd zero_f); a backward set from the pool by its finalize. The host tracks which sets may still hold sums (a
// training forward whose backward never ran): such a set is zeroed on the stream before it is
// handed out again. Graph replays stay valid because every captured step zeroes the sets it
// dirtied (forward and backward are captured together).
constexpr int kAccSets = 128, kAccC = 2048;
constexpr int64_t kRep = ARENA_ACC_REP;   // replicas per set (abi.h): a set is [kRep][2][C]
struct AccPool {
  Tensor t;
  unsigned next = 0;
  std::vector<char> dirty;
};
std::vector<AccPool>& acc_pools() {
  static std::vector<AccPool> pools;
  return pools;
}

// Scratch mode (conv autotuning, ops/conv.py plan_for): every request gets one fixed set that is
// never zeroed -- timed launches only need somewhere to add, and must not dirty the pool.
bool g_acc_scratch = false;

Tensor bn_acc_set(const Tensor& like, int64_t C) {
  TORCH_CHECK(C > 0 && C <= kAccC, "BatchNorm acc mode: C must be <= ", kAccC);
  auto& pools = acc_pools();
  const int dev = like.get_device();
  if ((int)pools.size() <= dev) pools.resize(dev + 1);
  AccPool& p = pools[dev];
  if (g_acc_scratch) {
    static std::vector<Tensor> scratch;
    if ((int)scratch.size() <= dev) scratch.resize(dev + 1);
    if (!scratch[dev].defined())
      scratch[dev] = torch::zeros({kRep * 2 * kAccC}, like.options().dtype(torch::kFloat64));
    return scratch[dev].narrow(0, 0, kRep * 2 * C).view({kRep, 2, C});
  }
  if (!p.t.defined()) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    check_hip(hipStreamIsCapturing(cur_stream(), &cs), "bn_acc_set");
    TORCH_CHECK(cs == hipStreamCaptureStatusNone,
                "arena BatchNorm: run one eager step before capturing a graph (its statistics "
                "accumulators are allocated and zeroed on first use)");
    p.t = torch::zeros({kAccSets, kRep * 2 * kAccC}, like.options().dtype(torch::kFloat64));
    p.dirty.assign(kAccSets, 0);
    check_hip(hipStreamSynchronize(cur_stream()), "bn_acc_set zero");
  }
  const int64_t set = p.next++ % kAccSets;
  Tensor row = p.t[set];
  if (p.dirty[set]) row.zero_();
  p.dirty[set] = 1;
  return row.narrow(0, 0, kRep * 2 * C).view({kRep, 2, C});
}

// A kernel that zeroes `t` (a pool set) has been enqueued: the set is clean for its next user.
void bn_acc_clean(const Tensor& t) {
  auto& pools = acc_pools();
  const int dev = t.get_device();
  if (dev < 0 || (int)pools.size() <= dev || !pools[dev].t.defined()) return;
  const AccPool& p = pools[dev];
  const int64_t off = (const double*)t.data_ptr() - (const double*)p.t.data_ptr();
  if (off < 0 || off >= (int64_t)kAccSets * kRep * 2 * kAccC) return;
  pools[dev].dirty[off / (kRep * 2 * kAccC)] = 0;
}

// Split-K tickets of the conv kernel (ConvArgs::kcnt): one ring of zeroed counters per device;
// each launch takes `tiles` consecutive counters from a cursor and its last-arriving blocks zero
// them again, so the ring needs no memset and graph replays stay valid. Consecutive launches get
// disjoint ranges, so launches on concurrent streams do not share tickets unless more than
// kConvTickets / 65536 of them are in flight at once.
constexpr int64_t kConvTickets = 1 << 22, kConvMaxTiles = 1 << 16;
unsigned* conv_tickets(const Tensor& like, int64_t tiles) {
  static std::vector<Tensor> pools;
  static std::vector<int64_t> next;
  TORCH_CHECK(tiles > 0 && tiles <= kConvMaxTiles, "conv split-K: too many output tiles");
  const int dev = like.get_device();
  if ((int)pools.size() <= dev) {
    pools.resize(dev + 1);
    next.resize(dev + 1, 0);
  }
  if (!pools[dev].defined()) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    check_hip(hipStreamIsCapturing(cur_stream(), &cs), "conv_tickets");
    TORCH_CHECK(cs == hipStreamCaptureStatusNone,
                "arena conv split-K: run one eager step before capturing a graph (its ticket "
                "counters are allocated and zeroed on first use)");
    pools[dev] = torch::zeros({kConvTickets}, like.options().dtype(torch::kInt32));
    check_hip(hipStreamSynchronize(cur_stream()), "conv_tickets zero");
  }
  if (next[dev] + tiles > kConvTickets) next[dev] = 0;
  unsigned* p = reinterpret_cast<unsigned*>(pools[dev].data_ptr<int32_t>()) + next[dev];
  next[dev] += (tiles + 63) / 64 * 64;
  return p;
}

// conv variant code: v1 tile/pipeline variant (0..15) + 16 * (ksplit - 1); 4096 + i: the v2 tile
// kernel's variant i (never split)
struct ConvSplit {
  int base = 0, ks = 1;
  Tensor ws;
  unsigned* cnt = nullptr;
};

ConvSplit conv_split(const Tensor& x, int64_t variant, int64_t M, int64_t Cout, int64_t Ktot) {
  ConvSplit s;
  TORCH_CHECK(variant >= 0, "conv: bad variant ", variant);
  if (variant >= 4096) {   // v2 tile kernel (conv_kernels.hip conv2_body): 4096 + i
    TORCH_CHECK(variant - 4096 < 19, "conv: unknown v2 variant ", variant);
    s.base = (int)variant;
  } else {   // v1 tile i (0..15), its K steps split over ks blocks: i + 16 (ks - 1)
    TORCH_CHECK(variant < 256, "conv: unknown variant ", variant);
    s.base = (int)(variant % 16);
    s.ks = (int)(variant / 16) + 1;
    TORCH_CHECK((s.base & 1) || Cout % 128 == 0, "conv: variant ", variant,
                " needs Cout % 128 == 0 (Cout = ", Cout, ")");
  }
  if (s.ks > 1) {
    TORCH_CHECK(s.ks <= Ktot / 64, "conv: split-K ", s.ks, " exceeds the ", Ktot / 64,
                " K steps");
    const long long nf = arena_conv_fwd_ksplit_floats(M, (int)Cout, s.base, s.ks);
    s.ws = torch::empty({nf}, x.options().dtype(torch::kFloat32));
    s.cnt = conv_tickets(x, arena_conv_fwd_tiles(M, (int)Cout, s.base));
  }
  return s;
}

// finished statistics / acc-mode reductions in the BN kernels (runtime switch for A/Bs)
bool g_bn_acc = [] {
  const char* e = getenv("ARENA_BN_FINAL");
  return e == nullptr || e[0] != '0';
}();

Tensor bn_lvl2(int64_t nblk, int64_t C, const Tensor& like) {
  return torch::empty({arena_bn_lvl2_doubles(nblk, (int)C)}, like.options().dtype(torch::kFloat64));
}

// Returns (y, mean, invstd, mask, acc). Eval mode normalises with the running statistics. mask (relu
// in training, else empty): uint8 [M * C / 8], bit i of byte v = (y.flat[8 v + i] > 0).
// acc: the fp64 [2][C] statistics sums the apply pass derived its coefficients from (acc mode), or
// empty. They stay in place: pass it to this layer's bn_bwd as zero_f, which zeroes it.
// zero_b (optional): fp64 tensor the apply pass zeroes (this layer's backward sums, bn_bwd acc_b).
// stats_part/stats_rpb: BatchNorm partials of x from conv_fwd(with_stats=True) (training only).
// stats_fin (training): the fp64 [2][C] accumulators conv_fwd(..., stats_final=True) filled: no
// statistics pass and no finalize (the apply pass derives its coefficients from the sums).
std::vector<Tensor> bn_fwd(Tensor x, OptT res, OptT gamma, OptT beta, OptT running_mean,
                           OptT running_var, bool training, double momentum, double eps,
                           bool relu, OptT num_batches, OptT stats_part, int64_t stats_rpb,
                           OptT stats_fin, OptT zero_b) {
  const BNGeom g = bn_geom(x, "x");
  if (res.has_value()) bn_same(x, *res, "residual");
  auto f32 = x.options().dtype(torch::kFloat32);
  Tensor mean = torch::empty({g.C}, f32), invstd = torch::empty({g.C}, f32);
  Tensor scale = torch::empty({g.C}, f32), shift = torch::empty({g.C}, f32);
  ArenaBNStats st{};
  st.eps = (float)eps;
  st.momentum = (float)momentum;
  st.gamma = bn_vec(gamma, g.C, "weight");
  st.beta = bn_vec(beta, g.C, "bias");
  st.mean = mean.data_ptr<float>();
  st.invstd = invstd.data_ptr<float>();
  st.scale = scale.data_ptr<float>();
  st.shift = shift.data_ptr<float>();
  Tensor part;
  if (training) {
    if (running_mean.has_value() || running_var.has_value()) {
      TORCH_CHECK(running_mean.has_value() && running_var.has_value(),
                  "running_mean and running_var go together");
      st.running_mean = const_cast<float*>(bn_vec(running_mean, g.C, "running_mean"));
      st.running_var = const_cast<float*>(bn_vec(running_var, g.C, "running_var"));
    }
    if (num_batches.has_value()) {
      check_dev(*num_batches, "num_batches_tracked");
      TORCH_CHECK(num_batches->scalar_type() == torch::kInt64 && num_batches->numel() == 1,
                  "num_batches_tracked must be an int64 scalar tensor");
      st.batches = reinterpret_cast<long long*>(num_batches->data_ptr<int64_t>());
    }
    if (stats_fin.has_value()) {
      TORCH_CHECK(stats_fin->is_cuda() && stats_fin->device() == x.device() &&
                      stats_fin->scalar_type() == torch::kFloat64 && stats_fin->is_contiguous() &&
                      stats_fin->numel() == kRep * 2 * g.C && !stats_part.has_value(),
                  "stats_fin must be a contiguous fp64 [kRep, 2, C] set (and excludes stats_part)");
    } else if (stats_part.has_value()) {
      check_f32(*stats_part, "stats_part");
      TORCH_CHECK(stats_rpb > 0 && stats_part->is_contiguous(), "stats_part: bad layout");
      const int64_t nblk = (g.M + stats_rpb - 1) / stats_rpb;
      TORCH_CHECK(stats_part->numel() == nblk * 2 * g.C, "stats_part has ", stats_part->numel(),
                  " floats, expected ", nblk * 2 * g.C);
      part = *stats_part;
    } else {
      // (acc mode may still fall back to partials for layers with many blocks x channels)
      part = torch::empty({arena_bn_workspace_floats(g.M, g.C)}, f32);
    }
  } else {
    TORCH_CHECK(running_mean.has_value() && running_var.has_value(),
                "eval-mode BatchNorm needs running statistics");
    bn_vec(running_mean, g.C, "running_mean");
    bn_vec(running_var, g.C, "running_var");
    mean.copy_(*running_mean);
    invstd.copy_(torch::rsqrt(*running_var + eps));
    scale.copy_(gamma.has_value() ? *gamma * invstd : invstd);
    if (beta.has_value()) shift.copy_(*beta); else shift.zero_();
  }
  Tensor y = torch::empty_like(x);
  Tensor mask = (training && relu) ? torch::empty({g.M * g.C / 8}, x.options().dtype(torch::kUInt8))
                                   : Tensor();
  const int ext_nblk = training && stats_part.has_value()
                           ? (int)((g.M + stats_rpb - 1) / stats_rpb) : 0;
  Tensor lvl2, acc;
  unsigned* tickets = nullptr;
  int acc_ready = 0;
  double* zb = nullptr;
  int nzb = 0;
  if (zero_b.has_value()) {
    TORCH_CHECK(zero_b->is_cuda() && zero_b->device() == x.device() &&
                    zero_b->scalar_type() == torch::kFloat64 && zero_b->is_contiguous(),
                "zero_b must be a contiguous fp64 tensor on x's device");
    zb = zero_b->data_ptr<double>();
    nzb = (int)zero_b->numel();
  }
  if (training && stats_fin.has_value()) {
    acc = *stats_fin;
    acc_ready = 1;
  } else if (training) {
    if (!stats_part.has_value() && g_bn_acc && arena_bn_acc_ok(g.M, (int)g.C))
      acc = bn_acc_set(x, g.C);
    const int64_t nblk = ext_nblk > 0 ? ext_nblk : part.numel() / (2 * g.C);
    lvl2 = bn_lvl2(nblk, g.C, x);
    tickets = bn_tickets(x);
  }
  check_hip(arena_bn_fwd(g.dtype, x.data_ptr(), res.has_value() ? res->data_ptr() : nullptr,
                         y.data_ptr(), mask.defined() ? mask.data_ptr<uint8_t>() : nullptr, g.M,
                         g.C, relu ? 1 : 0, training ? 1 : 0,
                         part.defined() ? part.data_ptr<float>() : nullptr, ext_nblk,
                         (long long)stats_rpb, lvl2.defined() ? lvl2.data_ptr<double>() : nullptr,
                         tickets, st, acc.defined() ? acc.data_ptr<double>() : nullptr, acc_ready,
                         zb, nzb, cur_stream()),
            "bn_fwd");
  return {y, mean, invstd, mask, acc};
}

// Returns (dx, dres or empty, dgamma or empty, dbeta or empty). mask: bn_fwd's ReLU bits (relu).
// ext_part/ext_rpb: the (dy, x) partials from conv_fwd(..., bn_x=x, ...) that produced dy.
// acc_b (optional): this layer's own fp64 [2][C] backward sums, zero on entry: the reduction adds
// into it and the dx pass derives its coefficients from it (no finalize launch); the sums stay in
// place until the layer's next bn_fwd(zero_b=acc_b). Without it a pool set and a finalize are used.
// zero_f (optional): the forward's statistics sums (bn_fwd's acc output), zeroed by the dx pass.
// x2 / mean2 / acc2 (optional): the dx pass also adds the backward sums of a second BN whose input
// is x2 and whose gradient is this layer's masked dy (a downsample block's down_bn) into acc2,
// that layer's own [kRep, 2, C] set -- where the pass derives its coefficients from sums, with
// ReLU and no residual output. Returns (dx, dres, dgamma, dbeta, acc2 if it was filled).
std::vector<Tensor> bn_bwd(Tensor dy, OptT mask, Tensor x, Tensor mean, Tensor invstd, OptT gamma,
                           bool relu, bool with_res, bool affine_grads, OptT ext_part,
                           int64_t ext_rpb, OptT acc_b, OptT zero_f, bool acc_ready, OptT x2,
                           OptT mean2, OptT acc2) {
  const BNGeom g = bn_geom(x, "x");
  bn_same(x, dy, "grad_output");
  const bool sum2 = x2.has_value() && x2->defined();
  if (sum2) {
    bn_same(x, *x2, "x2");
    TORCH_CHECK(mean2.has_value() && acc2.has_value(), "bn_bwd: x2 needs mean2 and acc2");
    check_f32(*mean2, "mean2");
    TORCH_CHECK(mean2->numel() == g.C, "bn_bwd: mean2 must have C elements");
    TORCH_CHECK(acc2->is_cuda() && acc2->device() == x.device() &&
                    acc2->scalar_type() == torch::kFloat64 && acc2->is_contiguous() &&
                    acc2->numel() == kRep * 2 * g.C,
                "bn_bwd: acc2 must be a contiguous fp64 [kRep, 2, C] set on x's device");
  }
  if (relu) {
    TORCH_CHECK(mask.has_value() && mask->is_cuda() && mask->scalar_type() == torch::kUInt8 &&
                    mask->is_contiguous() && mask->numel() == g.M * g.C / 8 &&
                    mask->device() == x.device(),
                "bn_bwd: relu needs the forward's uint8 mask of M*C/8 bytes");
  }
  check_f32(mean, "mean");
  check_f32(invstd, "invstd");
  TORCH_CHECK(mean.numel() == g.C && invstd.numel() == g.C, "saved statistics must have C elements");
  auto f32 = x.options().dtype(torch::kFloat32);
  Tensor co = torch::empty({3, g.C}, f32);
  Tensor dgamma, dbeta;
  ArenaBNBwd b{};
  b.mean = mean.data_ptr<float>();
  b.invstd = invstd.data_ptr<float>();
  b.gamma = bn_vec(gamma, g.C, "weight");
  if (affine_grads) {
    dgamma = torch::empty({g.C}, f32);
    dbeta = torch::empty({g.C}, f32);
    b.dgamma = dgamma.data_ptr<float>();
    b.dbeta = dbeta.data_ptr<float>();
  }
  b.ca = co.data_ptr<float>();
  b.cb = b.ca + g.C;
  b.cc = b.cb + g.C;
  Tensor part;
  int ext_nblk = 0;
  if (ext_part.has_value()) {
    check_f32(*ext_part, "ext_part");
    TORCH_CHECK(ext_rpb > 0, "bn_bwd: ext_rpb must be positive");
    const int64_t nblk = (g.M + ext_rpb - 1) / ext_rpb;
    TORCH_CHECK(ext_part->numel() == nblk * 2 * g.C, "bn_bwd: ext_part has ", ext_part->numel(),
                " floats, expected ", nblk * 2 * g.C);
    part = *ext_part;
    ext_nblk = (int)nblk;
  } else {
    part = torch::empty({arena_bn_workspace_floats(g.M, g.C)}, f32);
  }
  Tensor lvl2, acc;
  unsigned* tickets = nullptr;
  lvl2 = bn_lvl2(part.numel() / (2 * g.C), g.C, x);
  tickets = bn_tickets(x);
  // acc mode: atomics in the reduction + per-channel finalize (the kernel side keeps the
  // partials for layers with many blocks x channels)
  int fin_dx = 0;
  // acc_ready: the producing conv's backward-data epilogue already summed into acc_b (BNGradLink
  // acc mode): no reduction pass, the dx pass derives its coefficients from the sums
  TORCH_CHECK(!acc_ready || (acc_b.has_value() && !ext_part.has_value()),
              "bn_bwd: acc_ready needs acc_b and no ext_part");
  if (acc_ready) {
    TORCH_CHECK(acc_b->is_cuda() && acc_b->device() == x.device() &&
                    acc_b->scalar_type() == torch::kFloat64 && acc_b->is_contiguous() &&
                    acc_b->numel() == kRep * 2 * g.C,
                "acc_b must be a contiguous fp64 tensor of 2*C elements on x's device");
    acc = *acc_b;
    fin_dx = 1;
    ext_nblk = -1;
  } else if (!ext_part.has_value() && g_bn_acc && arena_bn_acc_ok(g.M, (int)g.C)) {
    if (acc_b.has_value()) {
      TORCH_CHECK(acc_b->is_cuda() && acc_b->device() == x.device() &&
                      acc_b->scalar_type() == torch::kFloat64 && acc_b->is_contiguous() &&
                      acc_b->numel() == kRep * 2 * g.C,
                  "acc_b must be a contiguous fp64 tensor of 2*C elements on x's device");
      acc = *acc_b;
      fin_dx = 1;
    } else {
      acc = bn_acc_set(x, g.C);
    }
  }
  double* zf = nullptr;
  int nzf = 0;
  if (zero_f.has_value() && zero_f->defined() && zero_f->numel() > 0) {
    TORCH_CHECK(zero_f->is_cuda() && zero_f->device() == x.device() &&
                    zero_f->scalar_type() == torch::kFloat64 && zero_f->is_contiguous(),
                "zero_f must be a contiguous fp64 tensor on x's device");
    zf = zero_f->data_ptr<double>();
    nzf = (int)zero_f->numel();
  }
  Tensor dx = torch::empty_like(x);
  Tensor dres = with_res ? torch::empty_like(x) : Tensor();
  // the second BN's sums ride along only where the dx pass derives its coefficients from sums
  // (fin_dx) on the plain ReLU path; else the caller's second BN reduces itself
  const bool use2 = sum2 && fin_dx == 1 && relu && !with_res;
  check_hip(arena_bn_bwd(g.dtype, dy.data_ptr(),
                         relu ? mask->data_ptr<uint8_t>() : nullptr, x.data_ptr(),
                         dx.data_ptr(), with_res ? dres.data_ptr() : nullptr, g.M, g.C,
                         relu ? 1 : 0, part.defined() ? part.data_ptr<float>() : nullptr, ext_nblk,
                         lvl2.defined() ? lvl2.data_ptr<double>() : nullptr, tickets, b,
                         acc.defined() ? acc.data_ptr<double>() : nullptr, fin_dx, zf, nzf,
                         use2 ? x2->data_ptr() : nullptr,
                         use2 ? mean2->data_ptr<float>() : nullptr,
                         use2 ? acc2->data_ptr<double>() : nullptr, cur_stream()),
            "bn_bwd");
  if (acc.defined() && !fin_dx) bn_acc_clean(acc);   // the finalize zeroed the pool set
  if (zf != nullptr) bn_acc_clean(*zero_f);
  return {dx, dres, dgamma, dbeta, use2 ? *acc2 : Tensor()};
}

// Fused stem BatchNorm + ReLU + k x k / s max pool (training; bn_kernels.hip arena_bn_pool_fwd):
// x is the BN input with its statistics from the producing conv: summed (fin, fp64 [2][C]) or as
// per-tile partials (stats_part, stats_rpb rows per partial; fin then empty).
// Returns (y, pos, mean, invstd, scale, shift, xsel): the pooled output, its uint8 in-window
// argmax, the saved statistics, and (with_xsel; else empty) x at each window's argmax, from which
// the backward takes its sums. fin stays in place until bn_pool_bwd(zero_f=fin) zeroes it;
// zero_b: as in bn_fwd.
std::vector<Tensor> bn_pool_fwd(Tensor x, OptT gamma, OptT beta, OptT running_mean,
                                OptT running_var, double momentum, double eps, OptT num_batches,
                                OptT fin, OptT stats_part, int64_t stats_rpb, int64_t k, int64_t s,
                                int64_t p, OptT zero_b, bool with_xsel) {
  const BNGeom g = bn_geom(x, "x");
  TORCH_CHECK(fin.has_value() != stats_part.has_value(),
              "bn_pool_fwd: give the statistics as fin sums or as stats_part partials");
  if (fin.has_value())
    TORCH_CHECK(fin->is_cuda() && fin->device() == x.device() &&
                    fin->scalar_type() == torch::kFloat64 && fin->is_contiguous() &&
                    fin->numel() == kRep * 2 * g.C,
                "bn_pool_fwd: fin must be the fp64 [kRep, 2, C] statistics sums");
  int ext_nblk = 0;
  Tensor lvl2;
  unsigned* tickets = nullptr;
  if (stats_part.has_value()) {
    check_f32(*stats_part, "stats_part");
    TORCH_CHECK(stats_rpb > 0 && stats_part->is_contiguous(), "stats_part: bad layout");
    const int64_t nblk = (g.M + stats_rpb - 1) / stats_rpb;
    TORCH_CHECK(stats_part->numel() == nblk * 2 * g.C, "stats_part has ", stats_part->numel(),
                " floats, expected ", nblk * 2 * g.C);
    ext_nblk = (int)nblk;
    lvl2 = bn_lvl2(nblk, g.C, x);
    tickets = bn_tickets(x);
  }
  auto f32 = x.options().dtype(torch::kFloat32);
  Tensor mean = torch::empty({g.C}, f32), invstd = torch::empty({g.C}, f32);
  Tensor scale = torch::empty({g.C}, f32), shift = torch::empty({g.C}, f32);
  ArenaBNStats st{};
  st.eps = (float)eps;
  st.momentum = (float)momentum;
  st.gamma = bn_vec(gamma, g.C, "weight");
  st.beta = bn_vec(beta, g.C, "bias");
  st.mean = mean.data_ptr<float>();
  st.invstd = invstd.data_ptr<float>();
  st.scale = scale.data_ptr<float>();
  st.shift = shift.data_ptr<float>();
  if (running_mean.has_value() || running_var.has_value()) {
    TORCH_CHECK(running_mean.has_value() && running_var.has_value(),
                "running_mean and running_var go together");
    st.running_mean = const_cast<float*>(bn_vec(running_mean, g.C, "running_mean"));
    st.running_var = const_cast<float*>(bn_vec(running_var, g.C, "running_var"));
  }
  if (num_batches.has_value()) {
    check_dev(*num_batches, "num_batches_tracked");
    st.batches = reinterpret_cast<long long*>(num_batches->data_ptr<int64_t>());
  }
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  const int64_t OH = (H + 2 * p - k) / s + 1, OW = (W + 2 * p - k) / s + 1;
  TORCH_CHECK(OH > 0 && OW > 0, "bn_pool_fwd: bad pool geometry");
  Tensor y = torch::empty({N, g.C, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor pos = torch::empty({N * OH * OW * g.C}, x.options().dtype(torch::kUInt8));
  Tensor xsel = with_xsel ? torch::empty_like(y) : Tensor();
  double* zb = nullptr;
  int nzb = 0;
  if (zero_b.has_value()) {
    TORCH_CHECK(zero_b->is_cuda() && zero_b->device() == x.device() &&
                    zero_b->scalar_type() == torch::kFloat64 && zero_b->is_contiguous(),
                "zero_b must be a contiguous fp64 tensor on x's device");
    zb = zero_b->data_ptr<double>();
    nzb = (int)zero_b->numel();
  }
  check_hip(arena_bn_pool_fwd(g.dtype, x.data_ptr(), y.data_ptr(), pos.data_ptr<uint8_t>(),
                              with_xsel ? xsel.data_ptr() : nullptr, (int)N, (int)H, (int)W,
                              (int)g.C, (int)k, (int)s, (int)p, st,
                              fin.has_value() ? fin->data_ptr<double>() : nullptr,
                              stats_part.has_value() ? stats_part->data_ptr<float>() : nullptr,
                              ext_nblk, (long long)stats_rpb,
                              lvl2.defined() ? lvl2.data_ptr<double>() : nullptr, tickets, zb, nzb,
                              cur_stream()),
            "bn_pool_fwd");
  return {y, pos, mean, invstd, scale, shift, xsel};
}

// Backward of bn_pool_fwd: returns (dx, dgamma or empty, dbeta or empty). acc_b: the layer's own
// fp64 [2, C] backward sums (zero on entry, left for the next forward's zero_b); zero_f: the
// forward's fin, zeroed by the dx pass; xsel: the forward's selected inputs (the reduction then
// reads them and dy instead of x).
std::vector<Tensor> bn_pool_bwd(Tensor dy, Tensor pos, Tensor x, Tensor mean, Tensor invstd,
                                Tensor scale, Tensor shift, OptT gamma, bool affine_grads,
                                int64_t k, int64_t s, int64_t p, Tensor acc_b, OptT zero_f,
                                OptT xsel) {
  const BNGeom g = bn_geom(x, "x");
  for (const Tensor* t : {&mean, &invstd, &scale, &shift}) {
    check_f32(*t, "saved statistics");
    TORCH_CHECK(t->numel() == g.C, "saved statistics must have C elements");
  }
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == x.scalar_type() && dy.size(0) == x.size(0) &&
                  dy.size(1) == g.C && dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "bn_pool_bwd: dy must be a channels_last tensor like the pooled output");
  TORCH_CHECK(pos.scalar_type() == torch::kUInt8 && pos.numel() == dy.numel() && pos.is_contiguous(),
              "bn_pool_bwd: pos must be the forward's argmax bytes");
  const bool has_xsel = xsel.has_value() && xsel->defined();
  if (has_xsel)
    TORCH_CHECK(xsel->is_cuda() && xsel->device() == x.device() &&
                    xsel->scalar_type() == x.scalar_type() && xsel->sizes() == dy.sizes() &&
                    xsel->is_contiguous(at::MemoryFormat::ChannelsLast),
                "bn_pool_bwd: xsel must be the forward's selected inputs (dy's shape and layout)");
  TORCH_CHECK(acc_b.is_cuda() && acc_b.device() == x.device() &&
                  acc_b.scalar_type() == torch::kFloat64 && acc_b.is_contiguous() &&
                  acc_b.numel() == kRep * 2 * g.C,
              "acc_b must be a contiguous fp64 tensor of 2*C elements on x's device");
  auto f32 = x.options().dtype(torch::kFloat32);
  ArenaBNBwd b{};
  b.mean = mean.data_ptr<float>();
  b.invstd = invstd.data_ptr<float>();
  b.scale = scale.data_ptr<float>();
  b.shift = shift.data_ptr<float>();
  b.gamma = bn_vec(gamma, g.C, "weight");
  Tensor dgamma, dbeta;
  if (affine_grads) {
    dgamma = torch::empty({g.C}, f32);
    dbeta = torch::empty({g.C}, f32);
    b.dgamma = dgamma.data_ptr<float>();
    b.dbeta = dbeta.data_ptr<float>();
  }
  double* zf = nullptr;
  int nzf = 0;
  if (zero_f.has_value() && zero_f->defined() && zero_f->numel() > 0) {
    TORCH_CHECK(zero_f->is_cuda() && zero_f->device() == x.device() &&
                    zero_f->scalar_type() == torch::kFloat64 && zero_f->is_contiguous(),
                "zero_f must be a contiguous fp64 tensor on x's device");
    zf = zero_f->data_ptr<double>();
    nzf = (int)zero_f->numel();
  }
  Tensor dx = torch::empty_like(x);
  check_hip(arena_bn_pool_bwd(g.dtype, dy.data_ptr(), pos.data_ptr<uint8_t>(), x.data_ptr(),
                              has_xsel ? xsel->data_ptr() : nullptr, dx.data_ptr(), (int)x.size(0), (int)x.size(2), (int)x.size(3),
                              (int)g.C, (int)k, (int)s, (int)p, b, acc_b.data_ptr<double>(), zf,
                              nzf, cur_stream()),
            "bn_pool_bwd");
  if (zf != nullptr) bn_acc_clean(*zero_f);
  return {dx, dgamma, dbeta};
}

// ------------------------------------------------------------------- NHWC max pooling
void pool_check(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4, name, " must be a 4-D GPU tensor");
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16 || t.scalar_type() == torch::kFloat32, name,
              " must be bfloat16 or float32");
  TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), name,
              " must be channels_last contiguous (NHWC)");
  TORCH_CHECK(t.size(1) % 8 == 0, name, ": C must be a multiple of 8");
}

// Returns (y, pos): pos = uint8 in-window argmax, same NHWC layout as y.
// NHWC bf16 implicit-GEMM convolution (csrc/ops/conv_kernels.hip). x: [N,C,H,W] channels_last,
// w: [Cout,C,R,S] channels_last (memory order [Cout][R][S][C]).
// with_stats: also returns the BatchNorm partials of y ([ceil(M/BM)][2][Cout] fp32, BM rows per
// partial) for bn_fwd(..., stats_part, BM): the BN layer after the conv skips its stats pass.
// addend (optional): bf16 tensor shaped like y (channels_last) added to the fp32 sums before the
// bf16 rounding: the second gradient of a tensor with two consumers (arena_amd.ops.conv.GradJoin).
// bn_x/bn_mask/bn_mean (optional, backward-data use): y is the gradient of a BatchNorm layer's
// output; with with_stats the returned partials are that BN's backward partials (g = y * mask,
// sum g, sum g * (bn_x - bn_mean)) for bn_bwd(..., ext_part, BM) instead of forward statistics.
// stats_final (with with_stats, forward statistics only): the second output is the fp64 [2][Cout]
// accumulator set (sum y, sum y^2) the epilogue added into, for bn_fwd(stats_fin=...), instead of
// the per-tile partials.
std::vector<Tensor> conv_fwd(Tensor x, Tensor w, int64_t stride, int64_t pad, int64_t variant,
                             bool with_stats, OptT addend, OptT bn_x, OptT bn_mask,
                             OptT bn_mean, OptT addmask, bool stats_final, OptT bn_acc) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && x.dim() == 4 && w.dim() == 4,
              "conv_fwd: x and w must be 4-D GPU tensors");
  TORCH_CHECK(x.scalar_type() == torch::kBFloat16 && w.scalar_type() == torch::kBFloat16,
              "conv_fwd: bfloat16 only");
  TORCH_CHECK(x.device() == w.device(), "conv_fwd: x and w on different devices");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_fwd: x and w must be channels_last contiguous");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Cout = w.size(0), R = w.size(2), S = w.size(3);
  TORCH_CHECK(w.size(1) == C, "conv_fwd: weight has ", w.size(1), " input channels, x has ", C);
  TORCH_CHECK(C % 64 == 0 && Cout % 64 == 0, "conv_fwd: C and Cout must be multiples of 64");
  TORCH_CHECK(stride >= 1 && pad >= 0 && H + 2 * pad >= R && W + 2 * pad >= S,
              "conv_fwd: bad stride/padding");
  const int64_t Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(N * Ho * Wo < (int64_t(1) << 31), "conv_fwd: too many output pixels");
  const ConvSplit ks = conv_split(x, variant, N * Ho * Wo, Cout, R * S * C);
  Tensor y = torch::empty({N, Cout, Ho, Wo},
                          x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int rows = arena_conv_fwd_tile_rows(ks.base);
  const int64_t m_tiles = (N * Ho * Wo + rows - 1) / rows;
  const bool fin = with_stats && stats_final;
  TORCH_CHECK(!fin || (!bn_x.has_value() && !addend.has_value() && Cout <= kAccC),
              "conv_fwd: stats_final is forward statistics without an addend");
  // bn_acc (backward-data form): the BN layer's fp64 [2][Cout] backward sums, added into
  const bool bacc = bn_acc.has_value() && bn_acc->defined();
  if (bacc) {
    TORCH_CHECK(bn_x.has_value() && with_stats && !fin, "conv_fwd: bn_acc is the bn_x form's");
    TORCH_CHECK(bn_acc->is_cuda() && bn_acc->device() == x.device() &&
                    bn_acc->scalar_type() == torch::kFloat64 && bn_acc->is_contiguous() &&
                    bn_acc->numel() == kRep * 2 * Cout,
                "conv_fwd: bn_acc must be a contiguous fp64 [kRep, 2, Cout] set");
  }
  Tensor part = with_stats && !fin && !bacc
                    ? torch::empty({m_tiles * 2 * Cout}, x.options().dtype(torch::kFloat32))
                    : Tensor();
  Tensor acc_t = fin ? bn_acc_set(x, Cout) : (bacc ? *bn_acc : Tensor());
  if (addend.has_value()) {
    TORCH_CHECK(addend->sizes() == y.sizes() && addend->scalar_type() == torch::kBFloat16 &&
                    addend->device() == y.device() &&
                    addend->is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_fwd: addend must be a channels_last bf16 tensor shaped like the output");
  }
  if (bn_x.has_value()) {
    TORCH_CHECK(with_stats && bn_mean.has_value(), "conv_fwd: bn_x needs with_stats and bn_mean");
    TORCH_CHECK(bn_x->sizes() == y.sizes() && bn_x->scalar_type() == torch::kBFloat16 &&
                    bn_x->device() == y.device() &&
                    bn_x->is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_fwd: bn_x must be a channels_last bf16 tensor shaped like the output");
    check_f32(*bn_mean, "bn_mean");
    TORCH_CHECK(bn_mean->numel() == Cout, "conv_fwd: bn_mean must have Cout elements");
    if (bn_mask.has_value()) {
      TORCH_CHECK(bn_mask->scalar_type() == torch::kUInt8 && bn_mask->is_contiguous() &&
                      bn_mask->device() == y.device() && bn_mask->numel() == y.numel() / 8,
                  "conv_fwd: bn_mask must be uint8 with numel(y) / 8 bytes");
    }
  }
  if (addmask.has_value()) {
    TORCH_CHECK(addend.has_value() && addmask->scalar_type() == torch::kUInt8 &&
                    addmask->is_contiguous() && addmask->device() == y.device() &&
                    addmask->numel() == y.numel() / 8,
                "conv_fwd: addmask needs an addend and numel(y) / 8 uint8 bytes");
  }
  check_hip(arena_conv_fwd_ex(x.data_ptr(), w.data_ptr(), y.data_ptr(),
                              part.defined() ? part.data_ptr<float>() : nullptr,
                              addend.has_value() ? addend->data_ptr() : nullptr,
                              addmask.has_value() ? addmask->data_ptr<uint8_t>() : nullptr,
                              bn_x.has_value() ? bn_x->data_ptr() : nullptr,
                              bn_x.has_value() && bn_mask.has_value()
                                  ? bn_mask->data_ptr<uint8_t>()
                                  : nullptr,
                              bn_x.has_value() ? bn_mean->data_ptr<float>() : nullptr,
                              (int)N, (int)H, (int)W, (int)C, (int)Cout, (int)R, (int)S,
                              (int)stride, (int)pad, (int)pad, 0, 0, nullptr, 0, ks.base,
                              acc_t.defined() ? acc_t.data_ptr<double>() : nullptr, ks.ks,
                              ks.ks > 1 ? ks.ws.data_ptr() : nullptr, ks.cnt, cur_stream()),
            "conv_fwd");
  if (acc_t.defined()) return {y, acc_t};
  if (with_stats) return {y, part};
  return {y};
}

// W'[ci][co][r][s] = W[co][ci][R-1-r][S-1-s] as a channels_last [C, Cout, R, S] bf16 tensor: the
// weight of the backward-data pass run through conv_fwd.
Tensor conv_flip_weight(Tensor w) {
  TORCH_CHECK(w.is_cuda() && w.dim() == 4 && w.scalar_type() == torch::kBFloat16 &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_flip_weight: w must be a channels_last bf16 GPU tensor [Cout, C, R, S]");
  const int64_t Cout = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
  TORCH_CHECK(Cout % 64 == 0 && C % 64 == 0, "conv_flip_weight: C and Cout must be multiples of 64");
  Tensor wt = torch::empty({C, Cout, R, S}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
  check_hip(arena_conv_flip_weight(w.data_ptr(), wt.data_ptr(), (int)Cout, (int)C, (int)R, (int)S,
                                   cur_stream()),
            "conv_flip_weight");
  return wt;
}

// conv_flip_weight for many weights in one launch per 64 tensors, into caller-owned outputs
// (dst[i]: channels_last [C, Cout, R, S] of src[i]'s shape).
void conv_flip_multi(std::vector<Tensor> src, std::vector<Tensor> dst) {
  TORCH_CHECK(src.size() == dst.size(), "conv_flip_multi: src and dst lengths differ");
  std::vector<const void*> sp;
  std::vector<void*> dp;
  std::vector<int> co, ci, rs;
  for (size_t i = 0; i < src.size(); ++i) {
    const Tensor& w = src[i];
    const Tensor& d = dst[i];
    TORCH_CHECK(w.is_cuda() && w.dim() == 4 && w.scalar_type() == torch::kBFloat16 &&
                    w.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_flip_multi: src must be channels_last bf16 GPU tensors [Cout, C, R, S]");
    TORCH_CHECK(d.is_cuda() && d.scalar_type() == torch::kBFloat16 && d.dim() == 4 &&
                    d.size(0) == w.size(1) && d.size(1) == w.size(0) && d.size(2) == w.size(2) &&
                    d.size(3) == w.size(3) && d.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    d.get_device() == w.get_device(),
                "conv_flip_multi: dst must be a channels_last bf16 [C, Cout, R, S] tensor");
    TORCH_CHECK(w.size(0) % 64 == 0 && w.size(1) % 64 == 0 && w.size(2) * w.size(3) <= 64,
                "conv_flip_multi: C and Cout must be multiples of 64, R*S <= 64");
    sp.push_back(w.data_ptr());
    dp.push_back(d.data_ptr());
    co.push_back((int)w.size(0));
    ci.push_back((int)w.size(1));
    rs.push_back((int)(w.size(2) * w.size(3)));
  }
  for (size_t b = 0; b < sp.size(); b += 64) {
    const int n = (int)std::min<size_t>(64, sp.size() - b);
    check_hip(arena_conv_flip_multi(n, sp.data() + b, dp.data() + b, co.data() + b, ci.data() + b,
                                    rs.data() + b, cur_stream()),
              "conv_flip_multi");
  }
}

// Phase weights of a stride-`stride` backward-data pass (arena_conv_phase_weights): one launch,
// one buffer; returns one channels_last [C, Cout, Rp, Sp] view per phase with taps, in phase
// order (a, b) row-major (phases without taps are absent).
std::vector<Tensor> conv_phase_weights(Tensor w, int64_t stride, int64_t pad) {
  TORCH_CHECK(w.is_cuda() && w.dim() == 4 && w.scalar_type() == torch::kBFloat16 &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_phase_weights: w must be a channels_last bf16 GPU tensor [Cout, C, R, S]");
  const int64_t Cout = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
  TORCH_CHECK(Cout % 64 == 0 && C % 64 == 0 && stride >= 1 && pad >= 0,
              "conv_phase_weights: C and Cout must be multiples of 64");
  long long total = 0;
  check_hip(arena_conv_phase_weights(w.data_ptr(), nullptr, (int)Cout, (int)C, (int)R, (int)S,
                                     (int)stride, (int)pad, &total, cur_stream()),
            "conv_phase_weights (geometry)");
  Tensor flat = torch::empty({std::max<long long>(total, 1)}, w.options());
  check_hip(arena_conv_phase_weights(w.data_ptr(), flat.data_ptr(), (int)Cout, (int)C, (int)R,
                                     (int)S, (int)stride, (int)pad, nullptr, cur_stream()),
            "conv_phase_weights");
  std::vector<Tensor> out;
  int64_t off = 0;
  for (int64_t a = 0; a < stride; ++a) {
    const int64_t r0 = (a + pad) % stride;
    if (r0 >= R) continue;
    const int64_t Rp = (R - r0 + stride - 1) / stride;
    for (int64_t b = 0; b < stride; ++b) {
      const int64_t c0 = (b + pad) % stride;
      if (c0 >= S) continue;
      const int64_t Sp = (S - c0 + stride - 1) / stride;
      out.push_back(flat.as_strided({C, Cout, Rp, Sp}, {Rp * Sp * Cout, 1, Sp * Cout, Cout}, off));
      off += C * Rp * Sp * Cout;
    }
  }
  return out;
}

// General NHWC convolution on the MFMA kernel (csrc/ops/conv_kernels.hip arena_conv_fwd_ex):
// top/left padding, explicit output size, optional placement of the output pixels into a larger
// preallocated tensor (y_out with y_map = [osh, osw, ooh, oow]: output (ho, wo) -> (ho*osh+ooh,
// wo*osw+oow) of y_out; an optional 5th entry fill_sib = 1 also writes the untapped sibling pixels
// of phase (0, 0) with the addend or zero), c16 mode (C == 16, S % 4 == 0). addend may alias y_out
// (in-place accumulate: each element is read and written by the same lane).
std::vector<Tensor> conv_fwd_ex(Tensor x, Tensor w, int64_t stride, int64_t pad_h, int64_t pad_w,
                                int64_t Ho, int64_t Wo, int64_t variant, bool with_stats,
                                OptT addend, OptT y_out, std::vector<int64_t> y_map, bool c16,
                                bool stats_final) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && x.dim() == 4 && w.dim() == 4 &&
                  x.scalar_type() == torch::kBFloat16 && w.scalar_type() == torch::kBFloat16 &&
                  x.device() == w.device(),
              "conv_fwd_ex: x and w must be 4-D bf16 tensors on one GPU");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_fwd_ex: x and w must be channels_last contiguous");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Cout = w.size(0), R = w.size(2), S = w.size(3);
  TORCH_CHECK(w.size(1) == C, "conv_fwd_ex: weight/input channel mismatch");
  TORCH_CHECK(Cout % 64 == 0 && (c16 ? (C == 16 && S % 4 == 0) : C % 64 == 0),
              "conv_fwd_ex: Cout % 64, and C % 64 (or C == 16, S % 4 == 0 in c16 mode)");
  TORCH_CHECK(stride >= 1 && Ho >= 1 && Wo >= 1, "conv_fwd_ex: bad geometry");
  TORCH_CHECK(N * Ho * Wo < (int64_t(1) << 31), "conv_fwd_ex: too many output pixels");
  const ConvSplit ks = conv_split(x, variant, N * Ho * Wo, Cout, R * S * C);
  Tensor y;
  std::vector<int> map6;
  if (y_out.has_value()) {
    y = *y_out;
    TORCH_CHECK(y.is_cuda() && y.device() == x.device() && y.dim() == 4 &&
                    y.scalar_type() == torch::kBFloat16 && y.size(0) == N && y.size(1) == Cout &&
                    y.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_fwd_ex: y_out must be a channels_last bf16 [N, Cout, Hy, Wy] tensor");
    TORCH_CHECK((y_map.size() == 4 || y_map.size() == 5) && y_map[0] >= 1 && y_map[1] >= 1 &&
                    y_map[2] >= 0 && y_map[3] >= 0 && (Ho - 1) * y_map[0] + y_map[2] < y.size(2) &&
                    (Wo - 1) * y_map[1] + y_map[3] < y.size(3),
                "conv_fwd_ex: y_map must place every output pixel inside y_out");
    const bool fill = y_map.size() == 5 && y_map[4] != 0;
    // sibling fill: phase (0, 0) whose pixels' siblings tile all of y_out
    TORCH_CHECK(!fill || (y_map[2] == 0 && y_map[3] == 0 &&
                          Ho == (y.size(2) + y_map[0] - 1) / y_map[0] &&
                          Wo == (y.size(3) + y_map[1] - 1) / y_map[1]),
                "conv_fwd_ex: fill_sib needs phase (0, 0) covering y_out");
    map6 = {(int)y.size(2), (int)y.size(3), (int)y_map[0], (int)y_map[1], (int)y_map[2],
            (int)y_map[3], fill ? 1 : 0};
  } else {
    y = torch::empty({N, Cout, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  }
  if (addend.has_value()) {
    TORCH_CHECK(addend->sizes() == y.sizes() && addend->scalar_type() == torch::kBFloat16 &&
                    addend->device() == y.device() &&
                    addend->is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_fwd_ex: addend must be shaped like the output tensor");
  }
  const int rows = arena_conv_fwd_tile_rows(ks.base);
  const int64_t m_tiles = (N * Ho * Wo + rows - 1) / rows;
  TORCH_CHECK(!(with_stats && y_out.has_value()), "conv_fwd_ex: statistics need a dense output");
  const bool fin = with_stats && stats_final;
  TORCH_CHECK(!fin || (!addend.has_value() && Cout <= kAccC),
              "conv_fwd_ex: stats_final is forward statistics without an addend");
  Tensor part = with_stats && !fin
                    ? torch::empty({m_tiles * 2 * Cout}, x.options().dtype(torch::kFloat32))
                    : Tensor();
  Tensor acc_t = fin ? bn_acc_set(x, Cout) : Tensor();
  check_hip(arena_conv_fwd_ex(x.data_ptr(), w.data_ptr(), y.data_ptr(),
                              with_stats && !fin ? part.data_ptr<float>() : nullptr,
                              addend.has_value() ? addend->data_ptr() : nullptr, nullptr, nullptr,
                              nullptr, nullptr, (int)N, (int)H, (int)W, (int)C, (int)Cout, (int)R,
                              (int)S,
                              (int)stride, (int)pad_h, (int)pad_w, (int)Ho, (int)Wo,
                              y_out.has_value() ? map6.data() : nullptr, c16 ? 1 : 0,
                              ks.base, fin ? acc_t.data_ptr<double>() : nullptr, ks.ks,
                              ks.ks > 1 ? ks.ws.data_ptr() : nullptr, ks.cnt, cur_stream()),
            "conv_fwd_ex");
  if (fin) return {y, acc_t};
  if (with_stats) return {y, part};
  return {y};
}

// Every phase convolution of a stride-`stride` backward-data pass in one launch (v2 tile
// `variant`): dy [N, C, H, W] (channels_last bf16), phase weights wps[p] [Cout, C, R_p, S_p]
// (conv_phase_weights' views), geometry[p] = {pad_h, pad_w, Ho, Wo, ooh, oow}; phase p writes
// pixel (ho, wo) of its grid to (ho*stride + ooh, wo*stride + oow) of dx_out [N, Cout, Hy, Wy]
// (+ addend shaped like dx_out, which may alias it).
void conv_dgrad_phases(Tensor dy, std::vector<Tensor> wps, std::vector<std::vector<int64_t>> geom,
                       Tensor dx_out, OptT addend, int64_t stride, int64_t variant) {
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 4 && dy.scalar_type() == torch::kBFloat16 &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_dgrad_phases: dy must be a channels_last bf16 GPU tensor");
  const int64_t np = (int64_t)wps.size();
  TORCH_CHECK(np >= 1 && np <= 4 && (int64_t)geom.size() == np, "conv_dgrad_phases: 1..4 phases");
  const int64_t N = dy.size(0), C = dy.size(1), H = dy.size(2), W = dy.size(3);
  TORCH_CHECK(dx_out.is_cuda() && dx_out.device() == dy.device() && dx_out.dim() == 4 &&
                  dx_out.scalar_type() == torch::kBFloat16 && dx_out.size(0) == N &&
                  dx_out.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_dgrad_phases: dx_out must be a channels_last bf16 [N, Cout, Hy, Wy] tensor");
  const int64_t Cout = dx_out.size(1);
  if (addend.has_value()) {
    TORCH_CHECK(addend->sizes() == dx_out.sizes() && addend->scalar_type() == torch::kBFloat16 &&
                    addend->device() == dx_out.device() &&
                    addend->is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_dgrad_phases: addend must be shaped like dx_out");
  }
  std::vector<const void*> wp(np);
  std::vector<int> R(np), S(np), ph(np), pw(np), Ho(np), Wo(np), oh(np), ow(np);
  for (int64_t p = 0; p < np; ++p) {
    const Tensor& w = wps[p];
    TORCH_CHECK(w.is_cuda() && w.device() == dy.device() && w.dim() == 4 &&
                    w.scalar_type() == torch::kBFloat16 && w.size(0) == Cout && w.size(1) == C &&
                    w.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_dgrad_phases: phase weights must be channels_last bf16 [Cout, C, R, S]");
    TORCH_CHECK(geom[p].size() == 6, "conv_dgrad_phases: geometry is {pad_h, pad_w, Ho, Wo, ooh, oow}");
    wp[p] = w.data_ptr();
    R[p] = (int)w.size(2); S[p] = (int)w.size(3);
    ph[p] = (int)geom[p][0]; pw[p] = (int)geom[p][1]; Ho[p] = (int)geom[p][2];
    Wo[p] = (int)geom[p][3]; oh[p] = (int)geom[p][4]; ow[p] = (int)geom[p][5];
    TORCH_CHECK(ph[p] >= 0 && pw[p] >= 0 && ph[p] < R[p] && pw[p] < S[p] &&
                    (Ho[p] - 1) * stride + oh[p] < dx_out.size(2) &&
                    (Wo[p] - 1) * stride + ow[p] < dx_out.size(3),
                "conv_dgrad_phases: phase ", p, " geometry outside dx_out");
  }
  check_hip(arena_conv_fwd_phases(dy.data_ptr(), dx_out.data_ptr(),
                                  addend.has_value() ? addend->data_ptr() : nullptr, (int)N, (int)H,
                                  (int)W, (int)C, (int)Cout, (int)dx_out.size(2),
                                  (int)dx_out.size(3), (int)stride, (int)stride, (int)np, wp.data(),
                                  R.data(), S.data(), ph.data(), pw.data(), Ho.data(), Wo.data(),
                                  oh.data(), ow.data(), (int)variant, cur_stream()),
            "conv_dgrad_phases");
}

// dW [Cout, C, R, S] (channels_last) of a convolution with top/left padding and an explicit
// output size (dy's), c16 mode as conv_fwd_ex.
// wgrad tile (Cout x R*S*C) of a variant: 0..3 (+4 serial) v1, 8..11 the v2 32x32x16 kernel
static bool wgrad_tile(int64_t variant, int* tbm, int* tbn) {
  static const int bm[4] = {128, 128, 64, 64}, bn[4] = {128, 64, 128, 64};
  static const int bm2[7] = {128, 256, 128, 256, 128, 128, 128};
  static const int bn2[7] = {128, 128, 256, 256, 128, 128, 128};
  if (variant >= 0 && variant <= 7) {
    *tbm = bm[variant & 3];
    *tbn = bn[variant & 3];
    return true;
  }
  if (variant >= 8 && variant <= 14) {
    *tbm = bm2[variant - 8];
    *tbn = bn2[variant - 8];
    return true;
  }
  return false;
}

Tensor conv_wgrad_ex(Tensor x, Tensor dy, int64_t R, int64_t S, int64_t stride, int64_t pad_h,
                     int64_t pad_w, int64_t variant, int64_t splits_hint, bool out_fp32,
                     double scale, bool c16) {
  TORCH_CHECK(x.is_cuda() && dy.is_cuda() && x.dim() == 4 && dy.dim() == 4 &&
                  x.scalar_type() == torch::kBFloat16 && dy.scalar_type() == torch::kBFloat16 &&
                  x.device() == dy.device(),
              "conv_wgrad_ex: x and dy must be 4-D bf16 tensors on one GPU");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_wgrad_ex: x and dy must be channels_last contiguous");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Cout = dy.size(1), Ho = dy.size(2), Wo = dy.size(3);
  TORCH_CHECK(dy.size(0) == N && R >= 1 && S >= 1 && stride >= 1, "conv_wgrad_ex: bad geometry");
  int tbm = 0, tbn = 0;
  TORCH_CHECK(wgrad_tile(variant, &tbm, &tbn) && Cout % tbm == 0 &&
                  (c16 ? (variant <= 7 && C == 16 && S % 4 == 0 && tbn == 64) : C % tbn == 0),
              "conv_wgrad_ex: variant ", variant, " does not fit C=", C, " Cout=", Cout);
  TORCH_CHECK(N * Ho * Wo < (int64_t(1) << 31), "conv_wgrad_ex: too many output pixels");
  const int64_t Ktot = R * S * C;
  const int splits = arena_conv_wgrad_splits((int)N, (int)Ho, (int)Wo, (int)Cout, (int)Ktot,
                                             (int)variant, (int)splits_hint);
  TORCH_CHECK(splits >= 1, "conv_wgrad_ex: bad split count");
  Tensor ws = torch::empty({(int64_t)splits * Cout * Ktot}, x.options().dtype(torch::kFloat32));
  Tensor dw = torch::empty({Cout, C, R, S}, x.options()
                                                .dtype(out_fp32 ? torch::kFloat32 : torch::kBFloat16)
                                                .memory_format(at::MemoryFormat::ChannelsLast));
  check_hip(arena_conv_wgrad_ex(x.data_ptr(), dy.data_ptr(), ws.data_ptr<float>(),
                                out_fp32 ? nullptr : dw.data_ptr(),
                                out_fp32 ? dw.data_ptr<float>() : nullptr, (int)N, (int)H, (int)W,
                                (int)C, (int)Cout, (int)R, (int)S, (int)stride, (int)pad_h,
                                (int)pad_w, (int)Ho, (int)Wo, c16 ? 1 : 0, (int)variant,
                                (int)splits_hint, (float)scale, cur_stream()),
            "conv_wgrad_ex");
  return dw;
}

// Space-to-depth of a channels_last [N, C<=4, H, W] bf16 image: [N, 16, H/2, W/2] (see kernel).
// x: channels_last [N, C<=4, H, W], bf16 or fp32 (rounded to bf16: the autocast cast, fused)
Tensor s2d_stem(Tensor x) {
  const bool f32 = x.scalar_type() == torch::kFloat32;
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 &&
                  (f32 || x.scalar_type() == torch::kBFloat16) &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast) && x.size(1) <= 4 &&
                  x.size(2) % 2 == 0 && x.size(3) % 2 == 0,
              "s2d_stem: channels_last bf16/fp32 [N, C<=4, H, W] with even H, W");
  // the kernel loads a pixel pair's 2C values as C 8-byte (fp32) / 4-byte (bf16) words
  if (reinterpret_cast<uintptr_t>(x.data_ptr()) % (f32 ? 8 : 4))
    x = x.clone(at::MemoryFormat::ChannelsLast);
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  Tensor z = torch::empty({N, 16, H / 2, W / 2}, x.options().dtype(torch::kBFloat16).memory_format(
                                                     at::MemoryFormat::ChannelsLast));
  check_hip(arena_s2d_stem(x.data_ptr(), z.data_ptr(), (int)N, (int)H, (int)W, (int)C, f32 ? 1 : 0,
                           cur_stream()),
            "s2d_stem");
  return z;
}

// The 7x7 stem weight [Cout, C<=4, 7, 7] (fp32 or bf16, any strides) -> its space-to-depth form,
// channels_last bf16 [Cout, 16, 4, 4] (ops/conv.py stem_weight).
Tensor stem_weight(Tensor w) {
  const bool f32 = w.scalar_type() == torch::kFloat32;
  TORCH_CHECK(w.is_cuda() && w.dim() == 4 && (f32 || w.scalar_type() == torch::kBFloat16) &&
                  w.size(1) >= 1 && w.size(1) <= 4 && w.size(2) == 7 && w.size(3) == 7,
              "stem_weight: [Cout, C<=4, 7, 7] fp32/bf16 GPU tensor");
  const int64_t Cout = w.size(0);
  Tensor w16 = torch::empty({Cout, 16, 4, 4}, w.options().dtype(torch::kBFloat16).memory_format(
                                                  at::MemoryFormat::ChannelsLast));
  check_hip(arena_stem_weight(w.data_ptr(), w16.data_ptr(), (int)Cout, (int)w.size(1),
                              w.stride(0), w.stride(1), w.stride(2), w.stride(3), f32 ? 1 : 0,
                              cur_stream()),
            "stem_weight");
  return w16;
}

// dW of the stem weight from dW16 (channels_last bf16 [Cout, 16, 4, 4]), allocated like `w`
// (its dtype and strides, so autograd accumulates it without a layout copy)
Tensor stem_weight_grad(Tensor dw16, Tensor w) {
  TORCH_CHECK(dw16.is_cuda() && dw16.dim() == 4 && dw16.scalar_type() == torch::kBFloat16 &&
                  dw16.size(1) == 16 && dw16.size(2) == 4 && dw16.size(3) == 4 &&
                  dw16.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_weight_grad: dw16 must be channels_last bf16 [Cout, 16, 4, 4]");
  const bool f32 = w.scalar_type() == torch::kFloat32;
  TORCH_CHECK(w.dim() == 4 && w.size(0) == dw16.size(0) && w.size(1) >= 1 && w.size(1) <= 4 &&
                  w.size(2) == 7 && w.size(3) == 7 &&
                  (f32 || w.scalar_type() == torch::kBFloat16),
              "stem_weight_grad: w must be [Cout, C<=4, 7, 7] fp32/bf16");
  Tensor dw = torch::empty_like(w);
  TORCH_CHECK(dw.is_non_overlapping_and_dense(), "stem_weight_grad: dense weight layout needed");
  check_hip(arena_stem_weight_grad(dw16.data_ptr(), dw.data_ptr(), (int)w.size(0),
                                   (int)w.size(1), dw.stride(0), dw.stride(1), dw.stride(2),
                                   dw.stride(3), f32 ? 1 : 0, cur_stream()),
            "stem_weight_grad");
  return dw;
}

// dW of an NHWC convolution: [Cout, C, R, S] channels_last, bf16 (for MasterSGD) or fp32.
Tensor conv_wgrad(Tensor x, Tensor dy, int64_t R, int64_t S, int64_t stride, int64_t pad,
                  int64_t variant, int64_t splits_hint, bool out_fp32, double scale) {
  TORCH_CHECK(x.is_cuda() && dy.is_cuda() && x.dim() == 4 && dy.dim() == 4,
              "conv_wgrad: x and dy must be 4-D GPU tensors");
  TORCH_CHECK(x.scalar_type() == torch::kBFloat16 && dy.scalar_type() == torch::kBFloat16,
              "conv_wgrad: bfloat16 only");
  TORCH_CHECK(x.device() == dy.device(), "conv_wgrad: x and dy on different devices");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_wgrad: x and dy must be channels_last contiguous");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Cout = dy.size(1);
  TORCH_CHECK(stride >= 1 && pad >= 0 && R >= 1 && S >= 1 && H + 2 * pad >= R && W + 2 * pad >= S,
              "conv_wgrad: bad geometry");
  const int64_t Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == Ho && dy.size(3) == Wo,
              "conv_wgrad: dy shape does not match the convolution geometry");
  int tbm = 0, tbn = 0;
  TORCH_CHECK(wgrad_tile(variant, &tbm, &tbn), "conv_wgrad: variant must be 0..14");
  TORCH_CHECK(C % tbn == 0 && Cout % tbm == 0, "conv_wgrad: variant ", variant, " needs C % ",
              tbn, " == 0 and Cout % ", tbm, " == 0");
  TORCH_CHECK(N * Ho * Wo < (int64_t(1) << 31), "conv_wgrad: too many output pixels");
  const int64_t Ktot = R * S * C;
  const int splits = arena_conv_wgrad_splits((int)N, (int)Ho, (int)Wo, (int)Cout, (int)Ktot,
                                             (int)variant, (int)splits_hint);
  TORCH_CHECK(splits >= 1, "conv_wgrad: bad split count");
  Tensor ws = torch::empty({(int64_t)splits * Cout * Ktot}, x.options().dtype(torch::kFloat32));
  Tensor dw = torch::empty({Cout, C, R, S}, x.options()
                                                .dtype(out_fp32 ? torch::kFloat32 : torch::kBFloat16)
                                                .memory_format(at::MemoryFormat::ChannelsLast));
  check_hip(arena_conv_wgrad_ex(x.data_ptr(), dy.data_ptr(), ws.data_ptr<float>(),
                                out_fp32 ? nullptr : dw.data_ptr(),
                                out_fp32 ? dw.data_ptr<float>() : nullptr, (int)N, (int)H, (int)W,
                                (int)C, (int)Cout, (int)R, (int)S, (int)stride, (int)pad, (int)pad,
                                0, 0, 0, (int)variant, (int)splits_hint, (float)scale,
                                cur_stream()),
            "conv_wgrad");
  return dw;
}

// Softmax cross-entropy, mean over rows (pool_kernels.hip): (loss, per-row log-sum-exp).
static void xent_check(const Tensor& x, const Tensor& y) {
  TORCH_CHECK(x.is_cuda() && y.is_cuda() && x.device() == y.device(), "xent: GPU tensors");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && x.size(0) > 0 && x.size(1) > 0 &&
                  (x.scalar_type() == torch::kBFloat16 || x.scalar_type() == torch::kFloat32),
              "xent: logits must be a contiguous 2-D bf16/fp32 tensor");
  TORCH_CHECK(y.dim() == 1 && y.is_contiguous() && y.scalar_type() == torch::kInt64 &&
                  y.size(0) == x.size(0), "xent: labels must be int64 [rows]");
  TORCH_CHECK(x.numel() < (int64_t(1) << 31), "xent: too many logits");
}

std::vector<Tensor> xent_fwd(Tensor x, Tensor y) {
  xent_check(x, y);
  // one buffer: [0, rows) log-sum-exp, [rows, 2 rows) per-row loss
  Tensor buf = torch::empty({2, x.size(0)}, x.options().dtype(torch::kFloat32));
  Tensor lse = buf[0], rowloss = buf[1];
  check_hip(arena_xent_fwd(x.scalar_type() == torch::kBFloat16 ? 1 : 0, x.data_ptr(),
                           reinterpret_cast<const long long*>(y.data_ptr<int64_t>()),
                           rowloss.data_ptr<float>(), lse.data_ptr<float>(),
                           (int)x.size(0), (int)x.size(1), cur_stream()),
            "xent_fwd");
  return {rowloss.mean(), lse};
}

Tensor xent_bwd(Tensor x, Tensor y, Tensor lse, Tensor gout) {
  xent_check(x, y);
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == torch::kFloat32 && lse.numel() == x.size(0) &&
                  gout.is_cuda() && gout.scalar_type() == torch::kFloat32 && gout.numel() == 1,
              "xent_bwd: lse fp32 [rows], grad fp32 scalar");
  Tensor dx = torch::empty_like(x);
  check_hip(arena_xent_bwd(x.scalar_type() == torch::kBFloat16 ? 1 : 0, x.data_ptr(),
                           reinterpret_cast<const long long*>(y.data_ptr<int64_t>()),
                           lse.data_ptr<float>(),
                           gout.contiguous().data_ptr<float>(), dx.data_ptr(), (int)x.size(0),
                           (int)x.size(1), cur_stream()),
            "xent_bwd");
  return dx;
}

// Global-average-pool backward: g [N, C] -> channels_last [N, C, H, W] filled with g / (H W).
Tensor gap_bwd(Tensor g, int64_t H, int64_t W) {
  TORCH_CHECK(g.is_cuda() && g.dim() == 2 && g.is_contiguous() &&
                  (g.scalar_type() == torch::kBFloat16 || g.scalar_type() == torch::kFloat32) &&
                  g.size(1) % 8 == 0 && H > 0 && W > 0,
              "gap_bwd: g must be a contiguous [N, C % 8 == 0] bf16/fp32 GPU tensor");
  TORCH_CHECK(g.size(0) * H * W * g.size(1) < (int64_t(1) << 34), "gap_bwd: too large");
  Tensor dx = torch::empty({g.size(0), g.size(1), H, W},
                           g.options().memory_format(at::MemoryFormat::ChannelsLast));
  check_hip(arena_gap_bwd(g.scalar_type() == torch::kBFloat16 ? 1 : 0, g.data_ptr(), dx.data_ptr(),
                          (int)g.size(0), (int)(H * W), (int)g.size(1), 1.0f / (float)(H * W),
                          cur_stream()),
            "gap_bwd");
  return dx;
}

std::vector<Tensor> maxpool_fwd(Tensor x, int64_t k, int64_t s, int64_t p) {
  pool_check(x, "x");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  TORCH_CHECK(k >= 1 && k <= 15 && s >= 1 && p >= 0 && 2 * p <= k && H + 2 * p >= k &&
                  W + 2 * p >= k,
              "maxpool: unsupported kernel/stride/padding");
  const int OH = (int)((H + 2 * p - k) / s + 1), OW = (int)((W + 2 * p - k) / s + 1);
  Tensor y = torch::empty({N, C, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor pos = torch::empty({N, C, OH, OW},
                            x.options().dtype(torch::kUInt8).memory_format(at::MemoryFormat::ChannelsLast));
  check_hip(arena_maxpool_fwd(x.scalar_type() == torch::kBFloat16 ? 1 : 0, x.data_ptr(),
                              y.data_ptr(), pos.data_ptr<uint8_t>(), N, H, W, C, (int)k, (int)s,
                              (int)p, cur_stream()),
            "maxpool_fwd");
  return {y, pos};
}

Tensor maxpool_bwd(Tensor dy, Tensor pos, int64_t H, int64_t W, int64_t k, int64_t s, int64_t p) {
  pool_check(dy, "grad_output");
  TORCH_CHECK(pos.scalar_type() == torch::kUInt8 && pos.sizes() == dy.sizes() &&
                  pos.is_contiguous(at::MemoryFormat::ChannelsLast),
              "maxpool_bwd: positions must be uint8 NHWC shaped like grad_output");
  const int N = (int)dy.size(0), C = (int)dy.size(1);
  TORCH_CHECK(dy.size(2) == (H + 2 * p - k) / s + 1 && dy.size(3) == (W + 2 * p - k) / s + 1,
              "maxpool_bwd: grad_output shape does not match the input geometry");
  Tensor dx = torch::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  check_hip(arena_maxpool_bwd(dy.scalar_type() == torch::kBFloat16 ? 1 : 0, dy.data_ptr(),
                              pos.data_ptr<uint8_t>(), dx.data_ptr(), N, (int)H, (int)W, C, (int)k,
                              (int)s, (int)p, cur_stream()),
            "maxpool_bwd");
  return dx;
}

class XgmiPeers {
 public:
  XgmiPeers(std::vector<int64_t> bufs, std::vector<int64_t> bufs2, std::vector<int64_t> sigs,
            Tensor epoch, Tensor err, int64_t buf_elems, int64_t buf2_elems, int64_t rank,
            double timeout_s)
      : epoch_(epoch), err_(err) {
    const int64_t w = (int64_t)bufs.size();
    TORCH_CHECK(w >= 2 && w <= ARENA_CCL_MAX_RANKS, "xGMI collective: world size must be 2..",
                ARENA_CCL_MAX_RANKS);
    TORCH_CHECK((int64_t)sigs.size() == w, "one signal buffer per rank");
    TORCH_CHECK(bufs2.empty() || (int64_t)bufs2.size() == w, "one second buffer per rank");
    TORCH_CHECK(rank >= 0 && rank < w, "rank out of range");
    check_dev(epoch, "epoch");
    check_dev(err, "err");
    TORCH_CHECK(epoch.scalar_type() == torch::kInt32 && epoch.numel() >= ARENA_CCL_MAX_BLOCKS,
                "epoch must be int32[", ARENA_CCL_MAX_BLOCKS, "]");
    TORCH_CHECK(err.scalar_type() == torch::kInt32 && err.numel() >= 1, "err must be int32[1]");
    std::memset(&p_, 0, sizeof p_);
    for (int64_t i = 0; i < w; ++i) {
      TORCH_CHECK(bufs[i] != 0 && sigs[i] != 0, "null peer pointer for rank ", i);
      p_.buf[i] = reinterpret_cast<float*>(bufs[i]);
      p_.sig[i] = reinterpret_cast<uint32_t*>(sigs[i]);
      if (!bufs2.empty()) p_.buf2[i] = reinterpret_cast<float*>(bufs2[i]);
    }
    p_.epoch = reinterpret_cast<uint32_t*>(epoch.data_ptr<int32_t>());
    p_.err = err.data_ptr<int32_t>();
    p_.buf_elems = buf_elems;
    p_.buf2_elems = bufs2.empty() ? 0 : buf2_elems;
    p_.rank = (int)rank;
    p_.world = (int)w;
    p_.timeout_cycles = (long long)(timeout_s * 1e8);  // s_memrealtime runs at 100 MHz
  }

  void allreduce(Tensor in, Tensor out, double scale) {
    check_f32(in, "in");
    check_f32(out, "out");
    const int64_t n = in.numel();
    TORCH_CHECK(out.numel() == n, "allreduce: in/out size mismatch");
    TORCH_CHECK(n % 4 == 0 && n <= p_.buf_elems, "allreduce: numel must be a multiple of 4 and <= ",
                p_.buf_elems);
    check_hip(arena_ccl_allreduce(&p_, in.data_ptr<float>(), out.data_ptr<float>(), n,
                                  (float)scale, cur_stream()),
              "xgmi_allreduce");
  }

  void adam(Tensor M, Tensor V, int64_t n, double lr, OptT lr_t, double b1, double b2, double eps,
            double wd, OptT t_step, double grad_scale, bool tf_style, OptT ctr_dst, OptT ctr_src,
            int64_t ctr_add) {
    check_f32(M, "M");
    check_f32(V, "V");
    TORCH_CHECK(p_.buf2[0] != nullptr, "xgmi adam needs the parameter buffers (buf2)");
    TORCH_CHECK(M.numel() >= n && V.numel() >= n && n % 4 == 0 && n <= p_.buf_elems &&
                    n <= p_.buf2_elems,
                "xgmi adam: bad sizes");
    ArenaAdam a = make_adam(lr, lr_t, b1, b2, eps, wd, t_step, grad_scale, tf_style);
    ArenaCounterOp ctr{};
    if (ctr_dst.has_value()) {
      ctr.dst = const_cast<long long*>(opt_i64_scalar(ctr_dst, "ctr_dst"));
      ctr.src = opt_i64_scalar(ctr_src, "ctr_src");
      ctr.add = (int)ctr_add;
    }
    check_hip(arena_ccl_adam(&p_, M.data_ptr<float>(), V.data_ptr<float>(), n, a, ctr, cur_stream()),
              "xgmi_adam");
  }

  // Pure copies: the tensors are raw 4-byte words (any dtype viewed as float32 by the caller).
  void broadcast(Tensor in, Tensor out, int64_t root) {
    check_f32(in, "in");
    check_f32(out, "out");
    const int64_t n = out.numel();
    TORCH_CHECK(in.numel() == n, "broadcast: in/out size mismatch");
    TORCH_CHECK(n % 4 == 0 && n <= p_.buf_elems, "broadcast: numel must be a multiple of 4 and <= ",
                p_.buf_elems);
    TORCH_CHECK(root >= 0 && root < p_.world, "broadcast: root out of range");
    TORCH_CHECK(in.data_ptr<float>() != nullptr && ((uintptr_t)in.data_ptr() % 16) == 0 &&
                    ((uintptr_t)out.data_ptr() % 16) == 0,
                "broadcast: 16-byte aligned tensors required");
    check_hip(arena_ccl_broadcast(&p_, in.data_ptr<float>(), out.data_ptr<float>(), n, (int)root,
                                  cur_stream()),
              "xgmi_broadcast");
  }

  void allgather(Tensor in, Tensor out) {
    check_f32(in, "in");
    check_f32(out, "out");
    const int64_t m = in.numel();
    TORCH_CHECK(out.numel() == m * p_.world, "allgather: out must hold world * numel(in)");
    TORCH_CHECK(m % 4 == 0 && m <= p_.buf_elems, "allgather: numel must be a multiple of 4 and <= ",
                p_.buf_elems);
    TORCH_CHECK(((uintptr_t)in.data_ptr() % 16) == 0 && ((uintptr_t)out.data_ptr() % 16) == 0,
                "allgather: 16-byte aligned tensors required");
    check_hip(arena_ccl_allgather(&p_, in.data_ptr<float>(), out.data_ptr<float>(), m,
                                  cur_stream()),
              "xgmi_allgather");
  }

  // Sharded momentum SGD over one bucket [off, off + n) of bf16 elements (see xgmi_ccl.hip).
  void sgd_bf16(Tensor master, Tensor mom, int64_t off, int64_t n, double lr, double momentum,
                double wd, double scale) {
    check_f32(master, "master");
    check_f32(mom, "mom");
    TORCH_CHECK(p_.buf2[0] != nullptr, "sgd_bf16 needs the weight buffers (buf2)");
    TORCH_CHECK(off >= 0 && n > 0 && off % 8 == 0 && n % 8 == 0, "sgd_bf16: off/n must be "
                "multiples of 8");
    TORCH_CHECK(master.numel() >= off + n && mom.numel() >= off + n, "sgd_bf16: master/mom too "
                "short");
    TORCH_CHECK((off + n + 1) / 2 <= p_.buf_elems && (off + n + 1) / 2 <= p_.buf2_elems,
                "sgd_bf16: bucket exceeds the registered buffers");
    check_hip(arena_ccl_sgd_bf16(&p_, master.data_ptr<float>(), mom.data_ptr<float>(), off, n,
                                 (float)lr, (float)momentum, (float)wd, (float)scale, cur_stream()),
              "xgmi_sgd_bf16");
  }

  // The fp32 tail bucket [off, off + n) (floats) of the same optimizer; `mom` holds the bucket's
  // momentum (bucket-relative, n floats).
  void sgd_f32(Tensor mom, int64_t off, int64_t n, double lr, double momentum, double wd,
               double scale) {
    check_f32(mom, "mom");
    TORCH_CHECK(p_.buf2[0] != nullptr, "sgd_f32 needs the weight buffers (buf2)");
    TORCH_CHECK(off >= 0 && n > 0 && off % 4 == 0 && n % 4 == 0, "sgd_f32: off/n must be "
                "multiples of 4");
    TORCH_CHECK(mom.numel() >= n, "sgd_f32: mom too short");
    TORCH_CHECK(off + n <= p_.buf_elems && off + n <= p_.buf2_elems,
                "sgd_f32: bucket exceeds the registered buffers");
    check_hip(arena_ccl_sgd_f32(&p_, mom.data_ptr<float>(), off, n, (float)lr, (float)momentum,
                                (float)wd, (float)scale, cur_stream()),
              "xgmi_sgd_f32");
  }

  int64_t world() const { return p_.world; }
  bool push() const { return p_.push != 0; }
  void set_push(bool on) { p_.push = on ? 1 : 0; }

 private:
  ArenaXgmiPeers p_;
  Tensor epoch_, err_;  // keep the device state alive
};

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "arena_amd native HIP kernels (gfx950)";
  m.def("linear_fwd", &linear_fwd);
  m.def("bn_fwd", &bn_fwd, py::arg("x"), py::arg("res"), py::arg("gamma"), py::arg("beta"),
        py::arg("running_mean"), py::arg("running_var"), py::arg("training"),
        py::arg("momentum"), py::arg("eps"), py::arg("relu"), py::arg("num_batches"),
        py::arg("stats_part"), py::arg("stats_rpb"), py::arg("stats_fin") = py::none(),
        py::arg("zero_b") = py::none());
  m.def("conv_flip_weight", &conv_flip_weight);
  m.def("conv_flip_multi", &conv_flip_multi);
  m.def("conv_phase_weights", &conv_phase_weights);
  m.def("conv_fwd_ex", &conv_fwd_ex, py::arg("x"), py::arg("w"), py::arg("stride"),
        py::arg("pad_h"), py::arg("pad_w"), py::arg("Ho"), py::arg("Wo"), py::arg("variant"),
        py::arg("with_stats"), py::arg("addend"), py::arg("y_out"), py::arg("y_map"),
        py::arg("c16"), py::arg("stats_final") = false);
  m.def("conv_wgrad_ex", &conv_wgrad_ex);
  m.def("conv_dgrad_phases", &conv_dgrad_phases, py::arg("dy"), py::arg("wps"), py::arg("geom"),
        py::arg("dx_out"), py::arg("addend"), py::arg("stride"), py::arg("variant"));
  m.def("s2d_stem", &s2d_stem);
  m.def("stem_weight", &stem_weight);
  m.def("stem_weight_grad", &stem_weight_grad);
  m.def("bn_bwd", &bn_bwd, py::arg("dy"), py::arg("mask"), py::arg("x"), py::arg("mean"),
        py::arg("invstd"), py::arg("gamma"), py::arg("relu"), py::arg("with_res"),
        py::arg("affine_grads"), py::arg("ext_part") = py::none(), py::arg("ext_rpb") = 0,
        py::arg("acc_b") = py::none(), py::arg("zero_f") = py::none(),
        py::arg("acc_ready") = false, py::arg("x2") = py::none(),
        py::arg("mean2") = py::none(), py::arg("acc2") = py::none());
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("w"), py::arg("stride"), py::arg("pad"),
        py::arg("variant"), py::arg("with_stats"), py::arg("addend") = py::none(),
        py::arg("bn_x") = py::none(), py::arg("bn_mask") = py::none(),
        py::arg("bn_mean") = py::none(), py::arg("addmask") = py::none(),
        py::arg("stats_final") = false, py::arg("bn_acc") = py::none());
  m.def("conv_wgrad", &conv_wgrad, py::arg("x"), py::arg("dy"), py::arg("R"), py::arg("S"),
        py::arg("stride"), py::arg("pad"), py::arg("variant"), py::arg("splits_hint"),
        py::arg("out_fp32"), py::arg("scale"));
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("xent_fwd", &xent_fwd);
  m.def("xent_bwd", &xent_bwd);
  m.def("gap_bwd", &gap_bwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("bn_set_fin_max_blocks", [](int64_t p) { arena_bn_set_fin_max_blocks((int)p); });
  m.def("bn_set_nt", [](int64_t on) { arena_bn_set_nt((int)on); });
  m.def("bn_set_pool_quad_mult", [](int64_t m) { arena_bn_set_pool_quad_mult((int)m); });
  m.def("bn_set_acc", [](bool on) { g_bn_acc = on; });
  m.def("bn_acc_scratch", [](bool on) { g_acc_scratch = on; });
  m.def("bn_pool_fwd", &bn_pool_fwd);
  m.attr("acc_rep") = (int)ARENA_ACC_REP;   // replicas per BatchNorm accumulator set
  m.def("conv_set_stats_one_pass", [](bool on) { arena_conv_set_stats_one_pass(on ? 1 : 0); });
  m.def("conv_set_dbg", [](int64_t bits) { arena_conv_set_dbg((int)bits); });
  m.def("bn_pool_bwd", &bn_pool_bwd);
  m.def("bn_set_reduce_geometry", [](int64_t max_blocks, int64_t min_rounds) {
    arena_bn_set_reduce_geometry(max_blocks, min_rounds);
  });
  m.def("xent_head", &xent_head);
  m.def("mlp_fwd_logits", &mlp_fwd_logits);
  m.def("wgrad_grouped", &wgrad_grouped);
  m.def("adam_flat", &adam_flat);
  m.def("sgd_flat", &sgd_flat);
  m.def("softmax_xent", &softmax_xent);
  m.def("mt_copy_scale", &mt_copy_scale);
  m.def("mt_sgd_master", &mt_sgd_master);
  m.def("shard_sgd", &shard_sgd, py::arg("grad"), py::arg("w32"), py::arg("mom"),
        py::arg("wbf") = py::none(), py::arg("lr"), py::arg("momentum"),
        py::arg("weight_decay"), py::arg("scale"));
  m.def("ccl_malloc", &ccl_malloc);
  m.def("ccl_free", &ccl_free);
  m.def("ccl_memset", &ccl_memset);
  m.def("ccl_ipc_get", &ccl_ipc_get);
  m.def("ccl_ipc_open", &ccl_ipc_open);
  m.def("ccl_ipc_close", &ccl_ipc_close);
  m.def("ccl_tensor", &ccl_tensor);
  m.def("ccl_shard", &ccl_shard);
  m.def("ccl_set_block_elems", [](int64_t e) { arena_ccl_set_block_elems(e); });
  m.def("ccl_set_max_blocks", [](int64_t b) { arena_ccl_set_max_blocks((int)b); });
  m.def("bn_set_elem_max_blocks", [](int64_t b) { arena_bn_set_elem_max_blocks((int)b); });
  m.def("bn_set_dx_max_blocks", [](int64_t b) { arena_bn_set_dx_max_blocks((int)b); });
  m.def("bn_set_slice", [](int64_t on) { arena_bn_set_slice((int)on); });
  m.def("ccl_set_oneshot_max", [](int64_t e) { arena_ccl_set_oneshot_max(e); });
  m.def("ccl_get_oneshot_max", []() { return (int64_t)arena_ccl_get_oneshot_max(); });
  m.def("ccl_set_bcast_direct_max", [](int64_t e) { arena_ccl_set_bcast_direct_max(e); });
  m.def("ccl_sgd_shard", [](int64_t off, int64_t n, int64_t world, int64_t rank) {
    long long lo = 0, hi = 0;
    arena_ccl_sgd_shard(off, n, (int)world, (int)rank, &lo, &hi);
    return std::vector<int64_t>{lo, hi};
  });
  m.def("ccl_sgd_f32_shard", [](int64_t off, int64_t n, int64_t world, int64_t rank) {
    long long lo = 0, hi = 0;
    arena_ccl_sgd_f32_shard(off, n, (int)world, (int)rank, &lo, &hi);
    return std::vector<int64_t>{lo, hi};
  });
  py::class_<XgmiPeers>(m, "XgmiPeers")
      .def(py::init<std::vector<int64_t>, std::vector<int64_t>, std::vector<int64_t>, Tensor,
                    Tensor, int64_t, int64_t, int64_t, double>())
      .def("allreduce", &XgmiPeers::allreduce)
      .def("adam", &XgmiPeers::adam)
      .def("broadcast", &XgmiPeers::broadcast)
      .def("allgather", &XgmiPeers::allgather)
      .def("sgd_bf16", &XgmiPeers::sgd_bf16)
      .def("sgd_f32", &XgmiPeers::sgd_f32)
      .def_property_readonly("world", &XgmiPeers::world)
      .def_property("push", &XgmiPeers::push, &XgmiPeers::set_push);
#ifdef ARENA_TIMELINE
  m.def("timeline_read", [](bool clear) {
    auto t = torch::empty({4, 1024, 16}, torch::TensorOptions().dtype(torch::kInt64));
    check_hip(arena_timeline_read(reinterpret_cast<long long*>(t.data_ptr<int64_t>()), clear ? 1 : 0),
              "timeline_read");
    return t;
  });
#endif
  m.attr("ccl_max_blocks") = ARENA_CCL_MAX_BLOCKS;
  m.attr("ccl_max_ranks") = ARENA_CCL_MAX_RANKS;
  m.attr("ccl_oneshot_elems") = ARENA_CCL_ONESHOT_ELEMS;
  m.attr("ccl_phases") = ARENA_CCL_PHASES;
  m.attr("arch") = "gfx950";
#ifndef ARENA_SRC_HASH
#define ARENA_SRC_HASH "unknown"
#endif
  m.attr("src_hash") = ARENA_SRC_HASH;
}
