// PyTorch custom-op registration of the C-ABI ("C-ABI op
// set ... registered through TORCH_LIBRARY").
//
// libd3rlpy_amd_torch.so registers namespace `d3rlpy_amd` with tensor-level
// schemas over the plain-pointer entry points of include/d3rlpy_amd.h, so the
// HIP kernels are visible to torch: callable as torch.ops.d3rlpy_amd.*,
// usable from TorchScript (torch.jit.script / save / load with the library
// loaded), and traceable by torch.export / torch.compile through the Meta
// (shape-only) implementations.  The ops run on the caller's current HIP
// stream, allocate their outputs with the caching allocator and never
// synchronise.  Errors are TORCH_CHECKs (Python RuntimeError), with the
// library's d3a_last_error() text for a rejected launch.
//
// Ops (reference call sites they replace):
//   linear(x, W, b, relu)          nn.Linear (+ ReLU) of every ensemble member in
//                                  one launch (encoders.py:265-275, 328-339)
//   mlp_forward(x, Ws, bs)         VectorEncoder(WithAction) trunk + linear head
//                                  (encoders.py:290-296 + mean_q_function.py:255)
//   gather_batch(...)              TransitionMiniBatch of vector transitions
//                                  (dataset.pyx:1139-1342)
//   standardize(x, mean, std, eps) StandardScaler.transform (scalers.py:350-354)
//   soft_update_(targ, src, tau)   soft_sync (torch_utility.py:27-33)
//   adam_step_(p, m, v, g, step, lr, beta1, beta2, eps)
//                                  torch.optim.Adam single-tensor step; `step`
//                                  is a device int64[1] holding the completed steps
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <torch/library.h>

#include <cmath>
#include <vector>

#include "d3rlpy_amd.h"

namespace {

void* cur_stream() { return (void*)at::hip::getCurrentHIPStream().stream(); }

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " failed: ", d3a_last_error());
}

void check_f32_gpu(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a HIP (cuda) tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

// x: [R, in] (shared by the members) or [C, R, in]; W: [C, out, in] or
// [out, in]; b: [C, out] or [out] -> y: [C, R, out] (or [R, out] for 2-D W)
at::Tensor linear_hip(const at::Tensor& x, const at::Tensor& W, const at::Tensor& b, bool relu) {
  check_f32_gpu(x, "x");
  check_f32_gpu(W, "W");
  check_f32_gpu(b, "b");
  const bool single = W.dim() == 2;
  const at::Tensor W3 = single ? W.unsqueeze(0) : W;
  const at::Tensor b2 = single ? b.unsqueeze(0) : b;
  TORCH_CHECK(W3.dim() == 3 && b2.dim() == 2, "linear: W [C, out, in], b [C, out]");
  const int64_t C = W3.size(0), out = W3.size(1), in = W3.size(2);
  TORCH_CHECK(b2.size(0) == C && b2.size(1) == out, "linear: bias shape mismatch");
  const bool shared = x.dim() == 2;
  TORCH_CHECK(shared || (x.dim() == 3 && x.size(0) == C), "linear: x [R, in] or [C, R, in]");
  const int64_t R = x.size(shared ? 0 : 1);
  TORCH_CHECK(x.size(shared ? 1 : 2) == in, "linear: x has ", x.size(shared ? 1 : 2),
              " features, W expects ", in);
  at::Tensor y = at::empty({C, R, out}, x.options());
  d3a_gemm_desc d{};
  d.A = x.data_ptr<float>();
  d.B = W3.data_ptr<float>();
  d.C = y.data_ptr<float>();
  d.bias = b2.data_ptr<float>();
  d.M = R; d.N = out; d.K = in; d.batch = C;
  d.sAb = shared ? 0 : R * in; d.sAm = in; d.sAk = 1;
  d.sBb = out * in; d.sBk = 1; d.sBn = in;   // B(k, n) = W[n][k]
  d.sCb = R * out; d.sCm = out; d.sCn = 1;
  d.sbias_b = out;
  d.splits = 1;
  d.alpha = 1.f;
  d.relu = relu ? 1 : 0;
  d.variant = -1;
  d.batch2 = 1;
  if (R > 0 && out > 0) check_rc(d3a_gemm_f32(&d, cur_stream()), "d3rlpy_amd::linear");
  return single ? y.squeeze(0) : y;
}

at::Tensor linear_meta(const at::Tensor& x, const at::Tensor& W, const at::Tensor& b, bool) {
  const bool single = W.dim() == 2;
  const int64_t C = single ? 1 : W.size(0), out = W.size(single ? 0 : 1);
  const int64_t R = x.size(x.dim() == 2 ? 0 : 1);
  return single ? at::empty({R, out}, x.options()) : at::empty({C, R, out}, x.options());
}

at::Tensor mlp_forward_hip(const at::Tensor& x, at::TensorList Ws, at::TensorList bs) {
  TORCH_CHECK(!Ws.empty() && Ws.size() == bs.size(), "mlp_forward: one bias per weight");
  at::Tensor h = x;
  for (size_t l = 0; l < Ws.size(); ++l) h = linear_hip(h, Ws[l], bs[l], l + 1 < Ws.size());
  return h;
}

at::Tensor mlp_forward_meta(const at::Tensor& x, at::TensorList Ws, at::TensorList bs) {
  at::Tensor h = x;
  for (size_t l = 0; l < Ws.size(); ++l) h = linear_meta(h, Ws[l], bs[l], false);
  return h;
}

at::Tensor standardize_hip(const at::Tensor& x, const at::Tensor& mean, const at::Tensor& std,
                           double eps) {
  check_f32_gpu(x, "x");
  check_f32_gpu(mean, "mean");
  check_f32_gpu(std, "std");
  TORCH_CHECK(x.dim() == 2 && mean.numel() == x.size(1) && std.numel() == x.size(1),
              "standardize: x [rows, D], mean / std [D]");
  at::Tensor y = at::empty_like(x);
  if (x.numel() > 0)
    check_rc(d3a_standardize_f32(x.data_ptr<float>(), y.data_ptr<float>(), x.size(0),
                                 (int32_t)x.size(1), x.size(1), mean.data_ptr<float>(),
                                 std.data_ptr<float>(), (float)eps, cur_stream()),
             "d3rlpy_amd::standardize");
  return y;
}

at::Tensor standardize_meta(const at::Tensor& x, const at::Tensor&, const at::Tensor&, double) {
  return at::empty_like(x);
}

void soft_update_hip(at::Tensor& targ, const at::Tensor& src, double tau) {
  check_f32_gpu(targ, "targ");
  check_f32_gpu(src, "src");
  TORCH_CHECK(targ.numel() == src.numel(), "soft_update_: size mismatch");
  check_rc(d3a_soft_update_f32(targ.data_ptr<float>(), src.data_ptr<float>(), targ.numel(), tau,
                               cur_stream()),
           "d3rlpy_amd::soft_update_");
}

void soft_update_meta(at::Tensor&, const at::Tensor&, double) {}

void adam_step_hip(at::Tensor& p, at::Tensor& m, at::Tensor& v, const at::Tensor& g,
                   const at::Tensor& step, double lr, double beta1, double beta2, double eps) {
  check_f32_gpu(p, "param");
  check_f32_gpu(m, "exp_avg");
  check_f32_gpu(v, "exp_avg_sq");
  check_f32_gpu(g, "grad");
  TORCH_CHECK(m.numel() == p.numel() && v.numel() == p.numel() && g.numel() == p.numel(),
              "adam_step_: size mismatch");
  TORCH_CHECK(step.is_cuda() && step.scalar_type() == at::kLong && step.numel() == 1,
              "adam_step_: step must be a HIP int64 tensor of one element");
  if (p.numel() == 0) return;
  d3a_adam_segment seg{};
  seg.param = p.data_ptr<float>();
  seg.exp_avg = m.data_ptr<float>();
  seg.exp_avg_sq = v.data_ptr<float>();
  seg.grad = g.data_ptr<float>();
  seg.numel = p.numel();
  seg.n_partials = 1;
  seg.partial_stride = p.numel();
  // the segment table is a device array (the kernel reads it)
  at::Tensor host = at::empty({(int64_t)sizeof(seg)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(host.data_ptr(), &seg, sizeof(seg));
  at::Tensor table = host.to(p.device(), /*non_blocking=*/false);
  const int64_t blocks = (p.numel() + 255) / 256;
  check_rc(d3a_adam_f32(reinterpret_cast<const d3a_adam_segment*>(table.data_ptr()), 1, blocks,
                        step.data_ptr<int64_t>(), lr, beta1, beta2, eps, 1.0, cur_stream()),
           "d3rlpy_amd::adam_step_");
  // commit the step count (d3a_step_end's counter increment)
  check_rc(d3a_step_end(nullptr, 0, nullptr, 0, nullptr, const_cast<int64_t*>(
                            step.data_ptr<int64_t>()), 1u, nullptr, nullptr, 0, 0.0, 1.f,
                        cur_stream()),
           "d3rlpy_amd::adam_step_");
}

void adam_step_meta(at::Tensor&, at::Tensor&, at::Tensor&, const at::Tensor&, const at::Tensor&,
                    double, double, double, double) {}

// Vector-observation gather (continuous actions): the dataset's structure of
// arrays and transition table as DeviceDataset holds them (d3rlpy_amd/dataset.py).
std::vector<at::Tensor> gather_batch_hip(const at::Tensor& obs, const at::Tensor& act,
                                         const at::Tensor& rew, const at::Tensor& t_row,
                                         const at::Tensor& t_ep_start,
                                         const at::Tensor& t_ep_last,
                                         const at::Tensor& t_terminal, const at::Tensor& idx,
                                         int64_t n_steps, double gamma) {
  check_f32_gpu(obs, "obs");
  check_f32_gpu(act, "act");
  check_f32_gpu(rew, "rew");
  for (const at::Tensor* t : {&t_row, &t_ep_start, &t_ep_last, &idx})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kLong && t->is_contiguous(),
                "gather_batch: transition table / indices must be contiguous HIP int64");
  TORCH_CHECK(t_terminal.is_cuda() && t_terminal.scalar_type() == at::kByte,
              "gather_batch: t_terminal must be HIP uint8");
  TORCH_CHECK(obs.dim() == 2 && act.dim() == 2, "gather_batch: obs [rows, D], act [rows, A]");
  TORCH_CHECK(n_steps >= 1 && n_steps <= D3A_MAX_NSTEP, "gather_batch: n_steps out of range");
  const int64_t B = idx.numel(), D = obs.size(1), A = act.size(1);
  auto f = obs.options();
  at::Tensor o_obs = at::empty({B, D}, f), o_next = at::empty({B, D}, f);
  at::Tensor o_act = at::empty({B, A}, f);
  at::Tensor o_rew = at::empty({B}, f), o_term = at::empty({B}, f), o_ns = at::empty({B}, f);
  if (B == 0) return {o_obs, o_act, o_rew, o_next, o_term, o_ns};
  d3a_gather_desc d{};
  d.obs = obs.data_ptr<float>();
  d.act = act.data_ptr<float>();
  d.rew = rew.data_ptr<float>();
  d.t_row = t_row.data_ptr<int64_t>();
  d.t_ep_start = t_ep_start.data_ptr<int64_t>();
  d.t_ep_last = t_ep_last.data_ptr<int64_t>();
  d.t_terminal = t_terminal.data_ptr<uint8_t>();
  d.n_trans = t_row.numel();
  d.D = (int32_t)D;
  d.A = (int32_t)A;
  d.n_frames = 1;
  d.n_steps = (int32_t)n_steps;
  d.gamma = (float)gamma;
  // powf(gamma, i): the reference's Cython 0.29 power (see d3a_gather_desc)
  for (int64_t i = 0; i < n_steps; ++i) d.gamma_pow[i] = powf((float)gamma, (float)i);
  d.idx = idx.data_ptr<int64_t>();
  d.B = (int32_t)B;
  d.o_obs = o_obs.data_ptr<float>();
  d.o_act = o_act.data_ptr<float>();
  d.o_rew = o_rew.data_ptr<float>();
  d.o_next_obs = o_next.data_ptr<float>();
  d.o_term = o_term.data_ptr<float>();
  d.o_n_steps = o_ns.data_ptr<float>();
  check_rc(d3a_gather_batch(&d, cur_stream()), "d3rlpy_amd::gather_batch");
  return {o_obs, o_act, o_rew, o_next, o_term, o_ns};
}

std::vector<at::Tensor> gather_batch_meta(const at::Tensor& obs, const at::Tensor& act,
                                          const at::Tensor&, const at::Tensor&, const at::Tensor&,
                                          const at::Tensor&, const at::Tensor&,
                                          const at::Tensor& idx, int64_t, double) {
  const int64_t B = idx.numel(), D = obs.size(1), A = act.size(1);
  auto f = obs.options();
  return {at::empty({B, D}, f), at::empty({B, A}, f), at::empty({B}, f), at::empty({B, D}, f),
          at::empty({B}, f), at::empty({B}, f)};
}

}  // namespace

TORCH_LIBRARY(d3rlpy_amd, m) {
  m.def("linear(Tensor x, Tensor W, Tensor b, bool relu) -> Tensor");
  m.def("mlp_forward(Tensor x, Tensor[] Ws, Tensor[] bs) -> Tensor");
  m.def("standardize(Tensor x, Tensor mean, Tensor std, float eps) -> Tensor");
  m.def("soft_update_(Tensor(a!) targ, Tensor src, float tau) -> ()");
  m.def("adam_step_(Tensor(a!) param, Tensor(b!) exp_avg, Tensor(c!) exp_avg_sq, Tensor grad, "
        "Tensor(d!) step, float lr, float beta1, float beta2, float eps) -> ()");
  m.def("gather_batch(Tensor obs, Tensor act, Tensor rew, Tensor t_row, Tensor t_ep_start, "
        "Tensor t_ep_last, Tensor t_terminal, Tensor idx, int n_steps, float gamma) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(d3rlpy_amd, CUDA, m) {
  m.impl("linear", &linear_hip);
  m.impl("mlp_forward", &mlp_forward_hip);
  m.impl("standardize", &standardize_hip);
  m.impl("soft_update_", &soft_update_hip);
  m.impl("adam_step_", &adam_step_hip);
  m.impl("gather_batch", &gather_batch_hip);
}

TORCH_LIBRARY_IMPL(d3rlpy_amd, Meta, m) {
  m.impl("linear", &linear_meta);
  m.impl("mlp_forward", &mlp_forward_meta);
  m.impl("standardize", &standardize_meta);
  m.impl("soft_update_", &soft_update_meta);
  m.impl("adam_step_", &adam_step_meta);
  m.impl("gather_batch", &gather_batch_meta);
}
