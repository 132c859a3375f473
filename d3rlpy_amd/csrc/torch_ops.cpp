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
//   linear_backward(g, x, W, y?)   nn.Linear (+ ReLU when y, its output, is
//                                  given) backward: (dx, dW, db) of every member
//   mlp_backward(g, x, Ws, hs)     the VectorEncoder trunk + head backward
//                                  (encoders.py:265-275): [dx, dW_0.., db_0..]
//   logsumexp(x) / _backward       torch.logsumexp(x, -1) (cql_impl.py:208-213)
//   td_mse_loss(q, r, t, d, gamma) / _backward
//                                  mean-Q TD error (mean_q_function.py:74-87)
//   quantile_huber_loss(q, y, taus) / _backward
//                                  q_functions/utility.py:27-46
//   iqn_cos_embed(taus, W, b) / _backward
//                                  relu(embed(cos(pi i tau))) (iqn_q_function.py:33-47)
//   squashed_gaussian_sample(mu, logstd, eps, lo, hi) / _backward
//                                  SquashedNormalPolicy.sample_with_log_prob
//                                  (distributions.py:112-135, policies.py:196-216)
//   cql_update_step(graph, state)  one whole CQLImpl update (CQL._update,
//                                  algos/cql.py:234-258 over cql_impl.py:119-243,
//                                  sac_impl.py, ddpg_impl.py): the step's HIP
//                                  kernels as the update pipeline's captured HIP
//                                  graph, launched on the current stream; `state`
//                                  lists the tensors the step mutates (parameters,
//                                  targets, optimiser state, metric ring) so the
//                                  dispatcher sees the effect.  update_step: the
//                                  same for the TD3+BC, BCQ and DiscreteCQL Impls.
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


at::Tensor contig(const at::Tensor& t) { return t.is_contiguous() ? t : t.contiguous(); }

// ---- linear / MLP backward ---------------------------------------------------
// g: [C, R, out] (or [R, out] with a 2-D W); x: [R, in] shared or [C, R, in];
// y (optional, undefined = none): the layer's ReLU output, masks g first.
std::vector<at::Tensor> linear_backward_hip(const at::Tensor& g_in, const at::Tensor& x_in,
                                            const at::Tensor& W_in,
                                            const c10::optional<at::Tensor>& y_in) {
  const at::Tensor g0 = contig(g_in), x = contig(x_in), W = contig(W_in);
  check_f32_gpu(g0, "grad");
  check_f32_gpu(x, "x");
  check_f32_gpu(W, "W");
  const bool single = W.dim() == 2;
  const at::Tensor W3 = single ? W.unsqueeze(0) : W;
  const int64_t C = W3.size(0), out = W3.size(1), in = W3.size(2);
  const bool shared = x.dim() == 2;
  const int64_t R = x.size(shared ? 0 : 1);
  TORCH_CHECK(g0.numel() == C * R * out, "linear_backward: grad must be [C, R, out]");
  at::Tensor g = g0;
  if (y_in.has_value() && y_in->defined()) {
    const at::Tensor y = contig(*y_in);
    check_f32_gpu(y, "y");
    TORCH_CHECK(y.numel() == g.numel(), "linear_backward: y must have grad's shape");
    g = at::empty_like(g0);
    check_rc(d3a_relu_mask_f32(g0.data_ptr<float>(), y.data_ptr<float>(), g0.numel(),
                               g.data_ptr<float>(), cur_stream()),
             "d3rlpy_amd::linear_backward");
  }
  at::Tensor dx = at::empty({C, R, in}, x.options());
  at::Tensor dW = at::empty({C, out, in}, x.options());
  at::Tensor db = at::empty({C, out}, x.options());
  if (R > 0) {
    // dx = g W: A = g [R, out] (k-contiguous), B(k = o, n = i) = W[o][i]
    d3a_gemm_desc a{};
    a.A = g.data_ptr<float>(); a.B = W3.data_ptr<float>(); a.C = dx.data_ptr<float>();
    a.M = R; a.N = in; a.K = out; a.batch = C;
    a.sAb = R * out; a.sAm = out; a.sAk = 1;
    a.sBb = out * in; a.sBk = in; a.sBn = 1;
    a.sCb = R * in; a.sCm = in; a.sCn = 1;
    a.splits = 1; a.alpha = 1.f; a.variant = -1; a.batch2 = 1;
    check_rc(d3a_gemm_f32(&a, cur_stream()), "d3rlpy_amd::linear_backward");
    // dW = g^T x (one split), db = row sums of g^T
    d3a_gemm_desc b{};
    b.A = g.data_ptr<float>(); b.B = x.data_ptr<float>(); b.C = dW.data_ptr<float>();
    b.rowsum = db.data_ptr<float>();
    b.M = out; b.N = in; b.K = R; b.batch = C;
    b.sAb = R * out; b.sAm = 1; b.sAk = out;
    b.sBb = shared ? 0 : R * in; b.sBk = in; b.sBn = 1;
    b.sCb = out * in; b.sCm = in; b.sCn = 1;
    b.sRb = out; b.sRs = C * out;
    b.splits = 1; b.alpha = 1.f; b.variant = -1; b.batch2 = 1;
    check_rc(d3a_gemm_f32(&b, cur_stream()), "d3rlpy_amd::linear_backward");
  } else {
    dW.zero_();
    db.zero_();
  }
  if (single) return {dx.squeeze(0), dW.squeeze(0), db.squeeze(0)};
  return {dx, dW, db};
}

std::vector<at::Tensor> linear_backward_meta(const at::Tensor& g, const at::Tensor& x,
                                             const at::Tensor& W,
                                             const c10::optional<at::Tensor>&) {
  const bool single = W.dim() == 2;
  const int64_t C = single ? 1 : W.size(0), out = W.size(single ? 0 : 1),
                in = W.size(single ? 1 : 2);
  const int64_t R = x.size(x.dim() == 2 ? 0 : 1);
  if (single)
    return {at::empty({R, in}, x.options()), at::empty({out, in}, x.options()),
            at::empty({out}, x.options())};
  return {at::empty({C, R, in}, x.options()), at::empty({C, out, in}, x.options()),
          at::empty({C, out}, x.options())};
}

// ReLU MLP (hidden layers hs[l] = relu(...), last layer linear): g is
// dL/d(output); returns [dx, dW_0 .. dW_{L-1}, db_0 .. db_{L-1}]
std::vector<at::Tensor> mlp_backward_hip(const at::Tensor& g, const at::Tensor& x,
                                         at::TensorList Ws, at::TensorList hs) {
  const size_t L = Ws.size();
  TORCH_CHECK(L >= 1 && hs.size() + 1 == L, "mlp_backward: one activation per hidden layer");
  std::vector<at::Tensor> dWs(L), dbs(L);
  at::Tensor cur = g;
  c10::optional<at::Tensor> none;
  for (size_t k = L; k-- > 0;) {
    const at::Tensor& xin = k == 0 ? x : hs[k - 1];
    // layer k's output gradient is masked by its ReLU output (hidden layers)
    c10::optional<at::Tensor> y = k + 1 < L ? c10::optional<at::Tensor>(hs[k]) : none;
    auto r = linear_backward_hip(cur, xin, Ws[k], y);
    dWs[k] = r[1];
    dbs[k] = r[2];
    cur = r[0];
  }
  std::vector<at::Tensor> out{cur};
  out.insert(out.end(), dWs.begin(), dWs.end());
  out.insert(out.end(), dbs.begin(), dbs.end());
  return out;
}

std::vector<at::Tensor> mlp_backward_meta(const at::Tensor& g, const at::Tensor& x,
                                          at::TensorList Ws, at::TensorList) {
  std::vector<at::Tensor> out{at::empty_like(x)};
  for (const auto& W : Ws) out.push_back(at::empty_like(W));
  for (const auto& W : Ws) out.push_back(at::empty({W.size(W.dim() - 2)}, W.options()));
  return out;
}

// ---- logsumexp over the last dimension -----------------------------------------
at::Tensor logsumexp_hip(const at::Tensor& x_in) {
  const at::Tensor x = contig(x_in);
  check_f32_gpu(x, "x");
  TORCH_CHECK(x.dim() >= 1 && x.size(-1) >= 1, "logsumexp: empty last dimension");
  const int64_t n = x.size(-1), rows = x.numel() / n;
  auto shape = x.sizes().vec();
  shape.pop_back();
  at::Tensor out = at::empty(shape, x.options());
  check_rc(d3a_logsumexp_f32(x.data_ptr<float>(), rows, n, n, out.data_ptr<float>(),
                             cur_stream()),
           "d3rlpy_amd::logsumexp");
  return out;
}

at::Tensor logsumexp_meta(const at::Tensor& x) {
  auto shape = x.sizes().vec();
  shape.pop_back();
  return at::empty(shape, x.options());
}

at::Tensor logsumexp_backward_hip(const at::Tensor& g_in, const at::Tensor& x_in,
                                  const at::Tensor& lse_in) {
  const at::Tensor g = contig(g_in), x = contig(x_in), lse = contig(lse_in);
  check_f32_gpu(x, "x");
  const int64_t n = x.size(-1), rows = x.numel() / n;
  TORCH_CHECK(g.numel() == rows && lse.numel() == rows, "logsumexp_backward: shape mismatch");
  at::Tensor dx = at::empty_like(x);
  check_rc(d3a_logsumexp_bwd_f32(x.data_ptr<float>(), rows, n, n, lse.data_ptr<float>(),
                                 g.data_ptr<float>(), dx.data_ptr<float>(), n, cur_stream()),
           "d3rlpy_amd::logsumexp_backward");
  return dx;
}

at::Tensor logsumexp_backward_meta(const at::Tensor&, const at::Tensor& x, const at::Tensor&) {
  return at::empty_like(x);
}

// ---- TD mean-squared error ------------------------------------------------------
// q: [C, B] (or [B]); rew, term, gamma: [B]; target: q's shape -> (loss [C] / [], diff)
std::vector<at::Tensor> td_mse_loss_hip(const at::Tensor& q_in, const at::Tensor& rew_in,
                                        const at::Tensor& target_in, const at::Tensor& term_in,
                                        const at::Tensor& gamma_in) {
  const at::Tensor q = contig(q_in), rew = contig(rew_in), target = contig(target_in),
                   term = contig(term_in), gamma = contig(gamma_in);
  for (const at::Tensor* t : {&q, &rew, &target, &term, &gamma}) check_f32_gpu(*t, "td_mse_loss input");
  const int64_t n = rew.numel();
  TORCH_CHECK(n >= 1 && q.numel() % n == 0 && target.numel() == q.numel() &&
                  term.numel() == n && gamma.numel() == n,
              "td_mse_loss: q / target [C, B], rew / term / gamma [B]");
  const int64_t C = q.numel() / n;
  at::Tensor diff = at::empty_like(q);
  at::Tensor loss = at::empty({C}, q.options());
  check_rc(d3a_td_mse_f32(q.data_ptr<float>(), rew.data_ptr<float>(), target.data_ptr<float>(),
                          term.data_ptr<float>(), gamma.data_ptr<float>(), C, n,
                          diff.data_ptr<float>(), loss.data_ptr<float>(), cur_stream()),
           "d3rlpy_amd::td_mse_loss");
  return {q.dim() == 1 ? loss.squeeze(0) : loss, diff};
}

std::vector<at::Tensor> td_mse_loss_meta(const at::Tensor& q, const at::Tensor& rew,
                                         const at::Tensor&, const at::Tensor&, const at::Tensor&) {
  const int64_t C = q.numel() / std::max<int64_t>(rew.numel(), 1);
  return {q.dim() == 1 ? at::empty({}, q.options()) : at::empty({C}, q.options()),
          at::empty_like(q)};
}

at::Tensor td_mse_loss_backward_hip(const at::Tensor& g_in, const at::Tensor& diff_in) {
  const at::Tensor g = contig(g_in), diff = contig(diff_in);
  check_f32_gpu(diff, "diff");
  const int64_t C = std::max<int64_t>(g.numel(), 1), n = diff.numel() / C;
  at::Tensor dq = at::empty_like(diff);
  check_rc(d3a_td_mse_bwd_f32(diff.data_ptr<float>(), g.data_ptr<float>(), C, n,
                              dq.data_ptr<float>(), cur_stream()),
           "d3rlpy_amd::td_mse_loss_backward");
  return dq;
}

at::Tensor td_mse_loss_backward_meta(const at::Tensor&, const at::Tensor& diff) {
  return at::empty_like(diff);
}

// ---- quantile Huber loss ----------------------------------------------------------
at::Tensor quantile_huber_loss_hip(const at::Tensor& q_in, const at::Tensor& y_in,
                                   const at::Tensor& taus_in) {
  const at::Tensor q = contig(q_in), y = contig(y_in), taus = contig(taus_in);
  for (const at::Tensor* t : {&q, &y, &taus}) check_f32_gpu(*t, "quantile_huber_loss input");
  TORCH_CHECK(q.dim() == 2 && y.dim() == 2 && taus.sizes() == q.sizes() && y.size(0) == q.size(0),
              "quantile_huber_loss: q [B, N], y [B, M], taus [B, N]");
  const int64_t B = q.size(0), N = q.size(1), M = y.size(1);
  at::Tensor loss = at::empty({B}, q.options());
  check_rc(d3a_quantile_huber_f32(q.data_ptr<float>(), N, y.data_ptr<float>(), M,
                                  taus.data_ptr<float>(), N, B, N, M, loss.data_ptr<float>(),
                                  cur_stream()),
           "d3rlpy_amd::quantile_huber_loss");
  return loss;
}

at::Tensor quantile_huber_loss_meta(const at::Tensor& q, const at::Tensor&, const at::Tensor&) {
  return at::empty({q.size(0)}, q.options());
}

at::Tensor quantile_huber_loss_backward_hip(const at::Tensor& g_in, const at::Tensor& q_in,
                                            const at::Tensor& y_in, const at::Tensor& taus_in) {
  const at::Tensor g = contig(g_in), q = contig(q_in), y = contig(y_in), taus = contig(taus_in);
  const int64_t B = q.size(0), N = q.size(1), M = y.size(1);
  TORCH_CHECK(g.numel() == B, "quantile_huber_loss_backward: grad [B]");
  at::Tensor dq = at::empty_like(q);
  check_rc(d3a_quantile_huber_bwd_f32(q.data_ptr<float>(), N, y.data_ptr<float>(), M,
                                      taus.data_ptr<float>(), N, B, N, M, g.data_ptr<float>(),
                                      dq.data_ptr<float>(), N, cur_stream()),
           "d3rlpy_amd::quantile_huber_loss_backward");
  return dq;
}

at::Tensor quantile_huber_loss_backward_meta(const at::Tensor&, const at::Tensor& q,
                                             const at::Tensor&, const at::Tensor&) {
  return at::empty_like(q);
}

// ---- IQN cosine embedding ------------------------------------------------------
// taus: any shape (R elements); W [F, E]; b [F] -> phi [R, F] = relu(cos(pi (i+1) tau) W^T + b)
at::Tensor iqn_prior(const at::Tensor& taus, int64_t E) {
  at::Tensor prior = at::empty({taus.numel(), E}, taus.options());
  d3a_iqn_prior_desc d{};
  d.taus = taus.data_ptr<float>();
  d.prior = prior.data_ptr<float>();
  d.rows = taus.numel();
  d.E = (int32_t)E;
  if (d.rows > 0) check_rc(d3a_iqn_prior(&d, cur_stream()), "d3rlpy_amd::iqn_cos_embed");
  return prior;
}

at::Tensor iqn_cos_embed_hip(const at::Tensor& taus_in, const at::Tensor& W, const at::Tensor& b) {
  const at::Tensor taus = contig(taus_in);
  check_f32_gpu(taus, "taus");
  TORCH_CHECK(W.dim() == 2 && b.dim() == 1 && b.size(0) == W.size(0), "iqn_cos_embed: W [F, E], b [F]");
  const at::Tensor prior = iqn_prior(taus, W.size(1));
  return linear_hip(prior, contig(W), contig(b), true);
}

at::Tensor iqn_cos_embed_meta(const at::Tensor& taus, const at::Tensor& W, const at::Tensor&) {
  return at::empty({taus.numel(), W.size(0)}, taus.options());
}

// -> (dW, db); taus carry no gradient (random fractions, iqn_q_function.py:15-30)
std::vector<at::Tensor> iqn_cos_embed_backward_hip(const at::Tensor& g, const at::Tensor& taus_in,
                                                   const at::Tensor& phi, const at::Tensor& W) {
  const at::Tensor taus = contig(taus_in);
  const at::Tensor prior = iqn_prior(taus, W.size(1));
  auto r = linear_backward_hip(g, prior, W, c10::optional<at::Tensor>(phi));
  return {r[1], r[2]};
}

std::vector<at::Tensor> iqn_cos_embed_backward_meta(const at::Tensor&, const at::Tensor&,
                                                    const at::Tensor&, const at::Tensor& W) {
  return {at::empty_like(W), at::empty({W.size(0)}, W.options())};
}

// ---- squashed Gaussian sample + log-prob -----------------------------------------
std::vector<at::Tensor> squashed_gaussian_sample_hip(const at::Tensor& mu_in,
                                                     const at::Tensor& logstd_in,
                                                     const at::Tensor& eps_in, double lo,
                                                     double hi) {
  const at::Tensor mu = contig(mu_in), logstd = contig(logstd_in), eps = contig(eps_in);
  for (const at::Tensor* t : {&mu, &logstd, &eps}) check_f32_gpu(*t, "squashed_gaussian_sample input");
  TORCH_CHECK(mu.dim() == 2 && logstd.sizes() == mu.sizes() && eps.sizes() == mu.sizes(),
              "squashed_gaussian_sample: mu, logstd, eps [B, A]");
  const int64_t B = mu.size(0), A = mu.size(1);
  at::Tensor act = at::empty_like(mu), logp = at::empty({B, 1}, mu.options());
  check_rc(d3a_squashed_gauss_f32(mu.data_ptr<float>(), logstd.data_ptr<float>(),
                                  eps.data_ptr<float>(), B, (int32_t)A, (float)lo, (float)hi,
                                  act.data_ptr<float>(), logp.data_ptr<float>(), cur_stream()),
           "d3rlpy_amd::squashed_gaussian_sample");
  return {act, logp};
}

std::vector<at::Tensor> squashed_gaussian_sample_meta(const at::Tensor& mu, const at::Tensor&,
                                                      const at::Tensor&, double, double) {
  return {at::empty_like(mu), at::empty({mu.size(0), 1}, mu.options())};
}

std::vector<at::Tensor> squashed_gaussian_sample_backward_hip(
    const at::Tensor& ga_in, const at::Tensor& gl_in, const at::Tensor& mu_in,
    const at::Tensor& logstd_in, const at::Tensor& eps_in, double lo, double hi) {
  const at::Tensor mu = contig(mu_in), logstd = contig(logstd_in), eps = contig(eps_in);
  const at::Tensor ga = contig(ga_in), gl = contig(gl_in);
  const int64_t B = mu.size(0), A = mu.size(1);
  TORCH_CHECK(ga.numel() == B * A && gl.numel() == B, "squashed_gaussian_sample_backward: shapes");
  at::Tensor dmu = at::empty_like(mu), dls = at::empty_like(mu);
  check_rc(d3a_squashed_gauss_bwd_f32(mu.data_ptr<float>(), logstd.data_ptr<float>(),
                                      eps.data_ptr<float>(), B, (int32_t)A, (float)lo, (float)hi,
                                      ga.data_ptr<float>(), gl.data_ptr<float>(),
                                      dmu.data_ptr<float>(), dls.data_ptr<float>(), cur_stream()),
           "d3rlpy_amd::squashed_gaussian_sample_backward");
  return {dmu, dls};
}

std::vector<at::Tensor> squashed_gaussian_sample_backward_meta(
    const at::Tensor&, const at::Tensor&, const at::Tensor& mu, const at::Tensor&,
    const at::Tensor&, double, double) {
  return {at::empty_like(mu), at::empty_like(mu)};
}

// the captured update pipeline (a hipGraphExec_t owned by the caller's
// torch.cuda.CUDAGraph, CUDAGraph.raw_cuda_graph_exec()) launched on the
// current stream.  The graph draws its noise from the library's own Philox
// stream (no torch generator state to advance), so the launch is the whole
// replay.
void update_step_hip(int64_t graph_exec, at::TensorList state) {
  TORCH_CHECK(graph_exec != 0, "update_step: null graph");
  for (const at::Tensor& t : state) TORCH_CHECK(t.is_cuda(), "update_step: state tensors must be on the GPU");
  const hipError_t e =
      hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(graph_exec), at::hip::getCurrentHIPStream().stream());
  TORCH_CHECK(e == hipSuccess, "update_step: hipGraphLaunch failed: ", hipGetErrorString(e));
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
  m.def("linear_backward(Tensor grad, Tensor x, Tensor W, Tensor? y) -> Tensor[]");
  m.def("mlp_backward(Tensor grad, Tensor x, Tensor[] Ws, Tensor[] hs) -> Tensor[]");
  m.def("logsumexp(Tensor x) -> Tensor");
  m.def("logsumexp_backward(Tensor grad, Tensor x, Tensor result) -> Tensor");
  m.def("td_mse_loss(Tensor q, Tensor rew, Tensor target, Tensor term, Tensor gamma) -> Tensor[]");
  m.def("td_mse_loss_backward(Tensor grad, Tensor diff) -> Tensor");
  m.def("quantile_huber_loss(Tensor q, Tensor y, Tensor taus) -> Tensor");
  m.def("quantile_huber_loss_backward(Tensor grad, Tensor q, Tensor y, Tensor taus) -> Tensor");
  m.def("iqn_cos_embed(Tensor taus, Tensor W, Tensor b) -> Tensor");
  m.def("iqn_cos_embed_backward(Tensor grad, Tensor taus, Tensor phi, Tensor W) -> Tensor[]");
  m.def("squashed_gaussian_sample(Tensor mu, Tensor logstd, Tensor eps, float min_logstd, "
        "float max_logstd) -> Tensor[]");
  m.def("squashed_gaussian_sample_backward(Tensor grad_action, Tensor grad_log_prob, Tensor mu, "
        "Tensor logstd, Tensor eps, float min_logstd, float max_logstd) -> Tensor[]");
  m.def("cql_update_step(int graph_exec, Tensor(a!)[] state) -> ()");
  m.def("update_step(int graph_exec, Tensor(a!)[] state) -> ()");
}

TORCH_LIBRARY_IMPL(d3rlpy_amd, CUDA, m) {
  m.impl("linear", &linear_hip);
  m.impl("mlp_forward", &mlp_forward_hip);
  m.impl("standardize", &standardize_hip);
  m.impl("soft_update_", &soft_update_hip);
  m.impl("adam_step_", &adam_step_hip);
  m.impl("gather_batch", &gather_batch_hip);
  m.impl("linear_backward", &linear_backward_hip);
  m.impl("mlp_backward", &mlp_backward_hip);
  m.impl("logsumexp", &logsumexp_hip);
  m.impl("logsumexp_backward", &logsumexp_backward_hip);
  m.impl("td_mse_loss", &td_mse_loss_hip);
  m.impl("td_mse_loss_backward", &td_mse_loss_backward_hip);
  m.impl("quantile_huber_loss", &quantile_huber_loss_hip);
  m.impl("quantile_huber_loss_backward", &quantile_huber_loss_backward_hip);
  m.impl("iqn_cos_embed", &iqn_cos_embed_hip);
  m.impl("iqn_cos_embed_backward", &iqn_cos_embed_backward_hip);
  m.impl("squashed_gaussian_sample", &squashed_gaussian_sample_hip);
  m.impl("squashed_gaussian_sample_backward", &squashed_gaussian_sample_backward_hip);
  m.impl("cql_update_step", &update_step_hip);
  m.impl("update_step", &update_step_hip);
}

TORCH_LIBRARY_IMPL(d3rlpy_amd, Meta, m) {
  m.impl("linear", &linear_meta);
  m.impl("mlp_forward", &mlp_forward_meta);
  m.impl("standardize", &standardize_meta);
  m.impl("soft_update_", &soft_update_meta);
  m.impl("adam_step_", &adam_step_meta);
  m.impl("gather_batch", &gather_batch_meta);
  m.impl("linear_backward", &linear_backward_meta);
  m.impl("mlp_backward", &mlp_backward_meta);
  m.impl("logsumexp", &logsumexp_meta);
  m.impl("logsumexp_backward", &logsumexp_backward_meta);
  m.impl("td_mse_loss", &td_mse_loss_meta);
  m.impl("td_mse_loss_backward", &td_mse_loss_backward_meta);
  m.impl("quantile_huber_loss", &quantile_huber_loss_meta);
  m.impl("quantile_huber_loss_backward", &quantile_huber_loss_backward_meta);
  m.impl("iqn_cos_embed", &iqn_cos_embed_meta);
  m.impl("iqn_cos_embed_backward", &iqn_cos_embed_backward_meta);
  m.impl("squashed_gaussian_sample", &squashed_gaussian_sample_meta);
  m.impl("squashed_gaussian_sample_backward", &squashed_gaussian_sample_backward_meta);
}
