// torch dispatcher kernels (CUDA key = HIP on PyTorch-ROCm) for the quantized-linear ops that run
// once per linear per forward: int4_weight_only_linear, int8_weight_only_linear,
// int8_quantize_per_token, int8_scaled_mm, int8_dyn_linear.
//
// The schemas stay defined in torchao/ops.py (the reference's registration pattern,
// torchao/ops.py:12-21); this library only supplies their CUDA kernels, so a call goes
// dispatcher -> C++ -> the C-ABI (include/torchao_mi355x.h) with no Python frame. The Python
// impls it replaces cost ~19 µs of host time per call at M = 1, four times the 4096x4096 GEMV
// (experiments/eager_overhead.py, profiles/r2_eager_overhead*.json); aten._weight_int4pack_mm,
// which the reference calls here (tensor_core_tiled_layout.py:104), is a C++ kernel too.
//
// Argument checks and messages are those of the Python impls (ops.py), raised as RuntimeError.
// Host-only code: built with g++ against the torch headers (Makefile target `ops`).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "../../include/torchao_mi355x.h"

namespace {

using at::Tensor;

void check_rc(int rc, const char* name) {
  TORCH_CHECK(rc == 0, name, " failed (status ", rc, "): ", tao_last_error());
}

hipStream_t stream_of(const Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

// x reshaped to [M, K], contiguous and 16-B aligned (the kernels' vector loads)
Tensor rows_of(const Tensor& x, int64_t K) {
  Tensor x2 = x.reshape({-1, K});
  if (!x2.is_contiguous() || reinterpret_cast<uintptr_t>(x2.data_ptr()) % 16) x2 = x2.contiguous();
  return x2;
}

std::vector<int64_t> out_shape(const Tensor& x, int64_t N) {
  std::vector<int64_t> s(x.sizes().begin(), x.sizes().end() - 1);
  s.push_back(N);
  return s;
}

template <class T>
const T* cptr(const Tensor& t) {
  return reinterpret_cast<const T*>(t.data_ptr());
}
template <class T>
T* mptr(const Tensor& t) {
  return reinterpret_cast<T*>(t.data_ptr());
}

// Every operand must live on x's device: the kernels take raw device pointers, so a weight left
// on another GPU (e.g. after a partial .to()) or on the host would reach the launch as a foreign
// pointer. The reference's aten ops raise on such inputs; so does this.
void check_device(const Tensor& x, const Tensor& t, const char* name) {
  TORCH_CHECK(x.is_cuda(), "expected x on a HIP device, got ", x.device());
  TORCH_CHECK(t.device() == x.device(), name, " is on ", t.device(), " but x is on ", x.device(),
              ": all operands must be on the same device");
}
void check_device(const Tensor& x, const std::optional<Tensor>& t, const char* name) {
  if (t.has_value()) check_device(x, *t, name);
}

std::optional<Tensor> bf16_bias(const std::optional<Tensor>& bias) {
  if (!bias.has_value()) return std::nullopt;
  return bias->to(at::kBFloat16).contiguous();
}

// ---- int4 weight-only (ops.py _int4_linear_cuda) ----------------------------------------------
Tensor int4_weight_only_linear(const Tensor& x, const Tensor& packed_w, const Tensor& sz,
                               int64_t group_size, const std::optional<Tensor>& bias) {
  TORCH_CHECK(packed_w.dim() == 2 && packed_w.scalar_type() == at::kInt,
              "packed weight must be a 2D int32 [N, K/8] tensor");
  const int64_t N = packed_w.size(0), K = packed_w.size(1) * 8;
  TORCH_CHECK(group_size == 32 || group_size == 64 || group_size == 128 || group_size == 256,
              "qGroupSize must be 32, 64, 128, or 256");
  TORCH_CHECK(K % group_size == 0, "K (", K, ") must be divisible by qGroupSize");
  TORCH_CHECK(sz.scalar_type() == at::kBFloat16, "scales_and_zeros must be bfloat16");
  TORCH_CHECK(sz.dim() == 3 && sz.size(0) == N && sz.size(1) == K / group_size && sz.size(2) == 2,
              "scales_and_zeros must be [N, K/g, 2] = (", N, ", ", K / group_size, ", 2), got ",
              sz.sizes());
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, "int4 weight-only linear needs bf16 input");
  TORCH_CHECK(x.size(-1) == K, "x last dim ", x.size(-1), " != K ", K);
  TORCH_CHECK(packed_w.is_contiguous(), "packed_w must be contiguous");
  TORCH_CHECK(sz.is_contiguous(), "scales_and_zeros must be contiguous");
  check_device(x, packed_w, "packed_w");
  check_device(x, sz, "scales_and_zeros");
  check_device(x, bias, "bias");
  const Tensor x2 = rows_of(x, K);
  const int64_t M = x2.size(0);
  const std::optional<Tensor> b = bf16_bias(bias);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = at::empty({M, N}, x.options().dtype(at::kBFloat16));
  check_rc(tao_int4wo_linear_bf16(cptr<uint16_t>(x2), cptr<uint32_t>(packed_w), cptr<uint16_t>(sz),
                                  b ? cptr<uint16_t>(*b) : nullptr, mptr<uint16_t>(y), M, N, K,
                                  group_size, stream_of(x)),
           "tao_int4wo_linear_bf16");
  return y.reshape(out_shape(x, N));
}

// ---- int8 ------------------------------------------------------------------------------------
void check_int8_weight(const Tensor& w, const Tensor& scale) {
  TORCH_CHECK(w.dim() == 2 && w.scalar_type() == at::kChar, "w must be a 2D int8 tensor");
  TORCH_CHECK(scale.numel() == w.size(0), "scale must have N elements");
}

Tensor int8_weight_only_linear(const Tensor& x, const Tensor& w_int8, const Tensor& scale,
                               const std::optional<Tensor>& bias) {
  check_int8_weight(w_int8, scale);
  const int64_t N = w_int8.size(0), K = w_int8.size(1);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, "int8 weight-only linear (HIP) needs bf16 x");
  TORCH_CHECK(x.size(-1) == K, "x last dim ", x.size(-1), " != K ", K);
  check_device(x, w_int8, "w_int8");
  check_device(x, scale, "scale");
  check_device(x, bias, "bias");
  const Tensor x2 = rows_of(x, K);
  const int64_t M = x2.size(0);
  const Tensor w = w_int8.contiguous();
  const Tensor s = scale.reshape({-1}).to(at::kBFloat16).contiguous();
  const std::optional<Tensor> b = bf16_bias(bias);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = at::empty({M, N}, x.options().dtype(at::kBFloat16));
  check_rc(tao_int8wo_linear_bf16(cptr<uint16_t>(x2), cptr<int8_t>(w), cptr<uint16_t>(s),
                                  b ? cptr<uint16_t>(*b) : nullptr, mptr<uint16_t>(y), M, N, K,
                                  stream_of(x)),
           "tao_int8wo_linear_bf16");
  return y.reshape(out_shape(x, N));
}

std::tuple<Tensor, Tensor> int8_quantize_per_token(const Tensor& x) {
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, "int8 per-token quant (HIP) needs bf16 x");
  const int64_t K = x.size(-1);
  const Tensor x2 = rows_of(x, K);
  const int64_t M = x2.size(0);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor q = at::empty({M, K}, x.options().dtype(at::kChar));
  Tensor s = at::empty({M, 1}, x.options().dtype(at::kBFloat16));
  check_rc(tao_int8_quant_per_token(cptr<uint16_t>(x2), mptr<int8_t>(q), mptr<uint16_t>(s), M, K,
                                    stream_of(x)),
           "tao_int8_quant_per_token");
  std::vector<int64_t> ss(x.sizes().begin(), x.sizes().end() - 1);
  ss.push_back(1);
  return {q.reshape(x.sizes()), s.reshape(ss)};
}

Tensor int8_scaled_mm(const Tensor& x_int8, const Tensor& x_scale, const Tensor& w_int8,
                      const Tensor& w_scale, const std::optional<Tensor>& bias) {
  check_int8_weight(w_int8, w_scale);
  const int64_t N = w_int8.size(0), K = w_int8.size(1);
  TORCH_CHECK(x_int8.scalar_type() == at::kChar, "x_int8 must be int8");
  TORCH_CHECK(x_int8.size(-1) == K, "x last dim ", x_int8.size(-1), " != K ", K);
  check_device(x_int8, x_scale, "x_scale");
  check_device(x_int8, w_int8, "w_int8");
  check_device(x_int8, w_scale, "w_scale");
  check_device(x_int8, bias, "bias");
  const Tensor x2 = x_int8.reshape({-1, K}).contiguous();
  const int64_t M = x2.size(0);
  const Tensor xs = x_scale.reshape({-1}).to(at::kBFloat16).contiguous();
  TORCH_CHECK(xs.numel() == M, "x_scale must have one entry per row");
  const Tensor ws = w_scale.reshape({-1}).to(at::kBFloat16).contiguous();
  const Tensor w = w_int8.contiguous();
  const std::optional<Tensor> b = bf16_bias(bias);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x_int8.device());
  Tensor y = at::empty({M, N}, x_int8.options().dtype(at::kBFloat16));
  check_rc(tao_int8_scaled_mm_bf16(cptr<int8_t>(x2), cptr<uint16_t>(xs), cptr<int8_t>(w),
                                   cptr<uint16_t>(ws), b ? cptr<uint16_t>(*b) : nullptr,
                                   mptr<uint16_t>(y), M, N, K, stream_of(x_int8)),
           "tao_int8_scaled_mm_bf16");
  return y.reshape(out_shape(x_int8, N));
}

Tensor int8_dyn_linear(const Tensor& x, const Tensor& w_int8, const Tensor& w_scale,
                       const std::optional<Tensor>& bias) {
  check_int8_weight(w_int8, w_scale);
  const int64_t N = w_int8.size(0), K = w_int8.size(1);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, "int8_dyn_linear (HIP) needs bf16 x");
  TORCH_CHECK(x.size(-1) == K, "x last dim ", x.size(-1), " != K ", K);
  TORCH_CHECK(x.numel() == K, "int8_dyn_linear is one token (x.numel() == K)");
  check_device(x, w_int8, "w_int8");
  check_device(x, w_scale, "w_scale");
  check_device(x, bias, "bias");
  const Tensor x2 = rows_of(x, K);
  const Tensor ws = w_scale.reshape({-1}).to(at::kBFloat16).contiguous();
  const Tensor w = w_int8.contiguous();
  const std::optional<Tensor> b = bf16_bias(bias);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = at::empty({1, N}, x.options().dtype(at::kBFloat16));
  check_rc(tao_int8_dyn_linear_bf16(cptr<uint16_t>(x2), cptr<int8_t>(w), cptr<uint16_t>(ws),
                                    b ? cptr<uint16_t>(*b) : nullptr, mptr<uint16_t>(y), 1, N, K,
                                    stream_of(x)),
           "tao_int8_dyn_linear_bf16");
  return y.reshape(out_shape(x, N));
}

}  // namespace

TORCH_LIBRARY_IMPL(torchao, CUDA, m) {
  m.impl("int4_weight_only_linear", &int4_weight_only_linear);
  m.impl("int8_weight_only_linear", &int8_weight_only_linear);
  m.impl("int8_quantize_per_token", &int8_quantize_per_token);
  m.impl("int8_scaled_mm", &int8_scaled_mm);
  m.impl("int8_dyn_linear", &int8_dyn_linear);
}

// Probe for torchao.ops (which ops this library serves).
extern "C" const char* tao_torch_ops_served(void) {
  return "int4_weight_only_linear,int8_weight_only_linear,int8_quantize_per_token,"
         "int8_scaled_mm,int8_dyn_linear";
}
