// DiscreteCQL with an IQN Q-function on pixel observations (K5): the conv
// encoder's data movement (col2im / layout transposes; im2col is kept in the
// ABI for reference-layout checks) and the IQN head, loss and head backward.
// The conv forward and weight gradient are implicit GEMMs (conv.hip); the
// conv input gradient is a GEMM into the column matrix + col2im.
//
// Reference (restated op for op, fp32):
//   PixelEncoder._conv_encode / forward      models/torch/encoders.py:130-162
//   PixelScaler.transform (x / 255)          preprocessing/scalers.py:109-110
//   compute_iqn_feature                       q_functions/iqn_q_function.py:33-47
//   DiscreteIQNQFunction._compute_quantiles   q_functions/iqn_q_function.py:82-88
//   DoubleDQNImpl.compute_target              algos/torch/dqn_impl.py:162-171
//   compute_quantile_loss (per-sample taus)   q_functions/utility.py:35-61
//   DiscreteCQLImpl._compute_conservative_loss algos/torch/cql_impl.py:291-302
//
// Activation layout: conv outputs are NHWC ([sample][y][x][channel], the
// row-major output of the im2col GEMM); the flatten before the encoder's fc
// uses the reference's NCHW order, so the last conv output is transposed
// (d3a_iqn_transpose) before the fc and its gradient transposed back.
#include "common.hpp"
#include "iqn_cos.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

inline unsigned blocks256(int64_t n) { return (unsigned)((n + 255) / 256); }

// col[(b, oy, ox)][c*KH*KW + kh*KW + kw] = x[b, c, S*oy+kh, S*ox+kw]
// x is NCHW uint8 (scaled by 1/255) or NHWC f32
__global__ __launch_bounds__(256) void im2col_kernel(d3a_im2col_desc d) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int KK = d.KH * d.KW;
  const int64_t Kc = (int64_t)d.C * KK;
  const int64_t P = (int64_t)d.OH * d.OW;
  if (i >= (int64_t)d.B * P * Kc) return;
  const int64_t row = i / Kc;
  const int k = (int)(i - row * Kc);
  const int64_t b = row / P;
  const int p = (int)(row - b * P);
  const int oy = p / d.OW, ox = p - oy * d.OW;
  const int c = k / KK, r = k - c * KK;
  const int kh = r / d.KW, kw = r - kh * d.KW;
  const int y = oy * d.S + kh, x = ox * d.S + kw;
  float v;
  if (d.x_u8) {
    // PixelScaler: x.float() / 255.0
    v = __fdiv_rn((float)d.x_u8[((b * d.C + c) * d.H + y) * d.W + x], 255.f);
  } else {
    v = d.x_f32[((b * d.H + y) * d.W + x) * d.C + c];
  }
  d.col[row * d.ldcol + k] = v;
}

// gather-form col2im (deterministic): dx[b][y][x][c] = sum over the output
// positions covering (y, x) of dcol[(b, oy, ox)][c, kh, kw]; times
// [mask[b][y][x][c] > 0] (the ReLU of the layer that produced x)
__global__ __launch_bounds__(256) void col2im_kernel(d3a_col2im_desc d) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n = (int64_t)d.B * d.H * d.W * d.C;
  if (i >= n) return;
  const int c = (int)(i % d.C);
  int64_t t = i / d.C;
  const int x = (int)(t % d.W);
  t /= d.W;
  const int y = (int)(t % d.H);
  const int64_t b = t / d.H;
  if (d.mask && !(d.mask[i] > 0.f)) {
    d.dx[i] = 0.f;
    return;
  }
  const int KK = d.KH * d.KW;
  float s = 0.f;
  for (int kh = 0; kh < d.KH; ++kh) {
    const int yy = y - kh;
    if (yy < 0 || yy % d.S) continue;
    const int oy = yy / d.S;
    if (oy >= d.OH) continue;
    for (int kw = 0; kw < d.KW; ++kw) {
      const int xx = x - kw;
      if (xx < 0 || xx % d.S) continue;
      const int ox = xx / d.S;
      if (ox >= d.OW) continue;
      const int64_t row = (b * d.OH + oy) * d.OW + ox;
      s += d.dcol[row * d.ldcol + c * KK + kh * d.KW + kw];
    }
  }
  d.dx[i] = s;
}

// per-sample [P][C] <-> [C][P] transpose, optionally masked by [mask > 0]
// (mask in the destination layout)
__global__ __launch_bounds__(256) void transpose_kernel(d3a_transpose_desc d) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t PC = (int64_t)d.P * d.C;
  if (i >= (int64_t)d.B * PC) return;
  const int64_t b = i / PC;
  const int64_t j = i - b * PC;
  int64_t src;
  if (d.to_cp) {  // dst [C][P]: j = c*P + p
    const int64_t c = j / d.P, p = j - c * d.P;
    src = b * PC + p * d.C + c;
  } else {        // dst [P][C]: j = p*C + c
    const int64_t p = j / d.C, c = j - p * d.C;
    src = b * PC + c * d.P + p;
  }
  const float v = d.src[src];
  d.dst[i] = (d.mask && !(d.mask[i] > 0.f)) ? 0.f : v;
}

// prior[r][i] = cos(pi * (i + 1) * tau[r])   (fp32 ops in torch's order; the
// cosine is iqn_cos, iqn_cos.hpp, shared with the fused head kernels)
__global__ __launch_bounds__(256) void iqn_prior_kernel(d3a_iqn_prior_desc d) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= d.rows * d.E) return;
  const int64_t r = i / d.E;
  const int e = (int)(i - r * d.E);
  const float ps = __fmul_rn(3.14159265358979323846f, (float)(e + 1));
  d.prior[i] = iqn_cos(__fmul_rn(ps, d.taus[r]));
}

// q[r][a] = (h[b(r)] * phi[r]) . Wf[a] + bf[a]; one wave per row.
// rows are grouped: group g covers rows [g*group_rows, (g+1)*group_rows) and
// reads its feature rows from h_group[g] (b = (r mod group_rows) / K)
__global__ __launch_bounds__(256) void iqn_head_fwd_kernel(d3a_iqn_head_desc d) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= d.rows) return;
  const int g = (int)(r / d.group_rows);
  const int64_t b = (r - (int64_t)g * d.group_rows) / d.K;
  const float* h = d.h[g] + b * d.F;
  const float* phi = d.phi + r * d.F;
  float acc[D3A_IQN_MAX_ACTIONS];
#pragma unroll
  for (int a = 0; a < D3A_IQN_MAX_ACTIONS; ++a) acc[a] = 0.f;
  for (int n = lane; n < d.F; n += 64) {
    const float pv = __fmul_rn(h[n], phi[n]);  // prod = h * phi
#pragma unroll
    for (int a = 0; a < D3A_IQN_MAX_ACTIONS; ++a)
      if (a < d.A) acc[a] = fmaf(pv, d.Wf[(int64_t)a * d.F + n], acc[a]);
  }
#pragma unroll
  for (int a = 0; a < D3A_IQN_MAX_ACTIONS; ++a) {
    if (a >= d.A) break;
    const float s = wave_sum(acc[a]);
    if (lane == 0) d.q[r * d.A + a] = s + d.bf[a];
  }
}

// Same head, 16 lanes per row and 16-byte loads (F % 4 == 0): Wf staged in
// LDS once per workgroup, each lane multiplies 4 features per load and the 16
// lanes of a row are summed with a butterfly.  Bandwidth-bound on phi.
__global__ __launch_bounds__(256) void iqn_head_fwd4_kernel(d3a_iqn_head_desc d) {
  __shared__ __attribute__((aligned(16))) float sW[D3A_IQN_MAX_ACTIONS * 512];
  const int F = d.F, A = d.A;
  for (int i = threadIdx.x; i < A * F; i += 256) sW[i] = d.Wf[i];
  __syncthreads();
  const int sl = threadIdx.x & 15;
  const int64_t r = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  if (r >= d.rows) return;
  const int g = (int)(r / d.group_rows);
  const int64_t b = (r - (int64_t)g * d.group_rows) / d.K;
  const float4* h = reinterpret_cast<const float4*>(d.h[g] + b * F);
  const float4* phi = reinterpret_cast<const float4*>(d.phi + r * F);
  float acc[D3A_IQN_MAX_ACTIONS];
#pragma unroll
  for (int a = 0; a < D3A_IQN_MAX_ACTIONS; ++a) acc[a] = 0.f;
  for (int n4 = sl; n4 < F / 4; n4 += 16) {
    const float4 hv = h[n4], pv4 = phi[n4];
    const float p0 = __fmul_rn(hv.x, pv4.x), p1 = __fmul_rn(hv.y, pv4.y);
    const float p2 = __fmul_rn(hv.z, pv4.z), p3 = __fmul_rn(hv.w, pv4.w);
#pragma unroll
    for (int a = 0; a < D3A_IQN_MAX_ACTIONS; ++a) {
      if (a < A) {
        const float4 wv = *reinterpret_cast<const float4*>(&sW[a * F + 4 * n4]);
        acc[a] = fmaf(p3, wv.w, fmaf(p2, wv.z, fmaf(p1, wv.y, fmaf(p0, wv.x, acc[a]))));
      }
    }
  }
#pragma unroll
  for (int a = 0; a < D3A_IQN_MAX_ACTIONS; ++a) {
    if (a >= A) break;
    float v = acc[a];
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (sl == 0) d.q[r * A + a] = v + d.bf[a];
  }
}

// One workgroup per batch row b: Double-DQN target, quantile Huber TD loss
// with the sample's taus, conservative term; dL/dq of the three gradient
// passes (rows [0, 3BK) of dq: loss | logsumexp | data), per-row loss.
//   q_loss  : online quantiles of the three gradient passes [3][B*K][A]
//   q_next  : online quantiles on next_obs (taus_next_online) [B*K][A]
//   q_targ  : target quantiles on next_obs                    [B*K][A]
__global__ __launch_bounds__(256) void iqn_loss_kernel(d3a_iqn_loss_desc d) {
  __shared__ float ys[1024];
  __shared__ float s_means[D3A_IQN_MAX_ACTIONS];
  __shared__ float scratch[16];
  __shared__ int s_arg;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t b = blockIdx.x;
  const int K = d.K, A = d.A;
  const int64_t BK = (int64_t)d.B * K;
  // argmax_a mean_k q_next(b, k, a)  (torch argmax: first maximal index)
  if (w < A) {
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s += d.q_next[(b * K + k) * A + w];
    s = wave_sum(s);
    if (lane == 0) s_means[w] = s / (float)K;
  }
  __syncthreads();
  if (t == 0) {
    int arg = 0;
    float best = s_means[0];
    for (int a = 1; a < A; ++a)
      if (s_means[a] > best) { best = s_means[a]; arg = a; }
    s_arg = arg;
  }
  __syncthreads();
  const int act = d.act[b];
  const float gam = powf(d.gamma, d.n_steps[b]);
  const float nt = __fsub_rn(1.f, d.term[b]);
  for (int i = t; i < K; i += 256) {
    const float tq = d.q_targ[(b * K + i) * A + s_arg];
    ys[i] = __fadd_rn(d.rew[b], __fmul_rn(__fmul_rn(gam, tq), nt));
  }
  __syncthreads();
  // TD: quantiles of the data action under the loss taus
  const float* q3 = d.q_loss;                 // pass 0 rows
  const float gscale = -1.f / ((float)d.B * (float)K);
  float lsum = 0.f;
  for (int j = t; j < K; j += 256) {
    const float qj = q3[(b * K + j) * A + act];
    const float tau = d.taus_loss[b * K + j];
    float l = 0.f, g = 0.f;
    for (int i = 0; i < K; ++i) {
      const float diff = __fsub_rn(ys[i], qj);
      const float ad = fabsf(diff);
      const float wgt = fabsf(__fsub_rn(tau, diff < 0.f ? 1.f : 0.f));
      const float hub = ad < 1.f ? __fmul_rn(0.5f, __fmul_rn(diff, diff)) : __fsub_rn(ad, 0.5f);
      l += __fmul_rn(wgt, hub);
      g = fmaf(wgt, ad < 1.f ? diff : (diff < 0.f ? -1.f : 1.f), g);
    }
    lsum += l;
    for (int a = 0; a < A; ++a)
      d.dq[(b * K + j) * A + a] = a == act ? __fmul_rn(g, gscale) : 0.f;
  }
  const float td = block_sum(lsum, scratch) / (float)K;
  // conservative term: logsumexp_a Q_lse(b, a) - Q_data(b, act)
  const float* q4 = d.q_loss + BK * A;
  const float* q5 = d.q_loss + 2 * BK * A;
  __syncthreads();
  if (w < A) {
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s += q4[(b * K + k) * A + w];
    s = wave_sum(s);
    if (lane == 0) s_means[w] = s / (float)K;
  }
  __syncthreads();
  float mx = -INFINITY;
  for (int a = 0; a < A; ++a) mx = fmaxf(mx, s_means[a]);
  if (isinf(mx)) mx = 0.f;
  float se = 0.f;
  for (int a = 0; a < A; ++a) se += expf(s_means[a] - mx);
  const float lse = logf(se) + mx;
  float qd = 0.f;
  if (w == 0) {
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s += q5[(b * K + k) * A + act];
    s = wave_sum(s);
    qd = s / (float)K;
  }
  // dL/dq: logsumexp pass alpha softmax / (B K), data pass -alpha / (B K)
  const float cs = d.alpha / ((float)d.B * (float)K);
  for (int64_t e = t; e < (int64_t)K * A; e += 256) {
    const int k = (int)(e / A), a = (int)(e - (int64_t)k * A);
    d.dq[BK * A + (b * K + k) * A + a] = __fmul_rn(cs, expf(s_means[a] - lse));
    d.dq[2 * BK * A + (b * K + k) * A + a] = a == act ? -cs : 0.f;
  }
  if (t == 0) {
    d.loss_b[b] = td;
    d.cons_b[b] = lse - qd;
  }
}

// metrics[0] = mean_b td + alpha * mean_b cons  (one workgroup)
__global__ __launch_bounds__(1024) void iqn_loss_reduce_kernel(d3a_iqn_loss_desc d) {
  __shared__ double sd[16];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  double a = 0.0, c = 0.0;
  for (int b = t; b < d.B; b += 1024) { a += d.loss_b[b]; c += d.cons_b[b]; }
  for (int o = 32; o > 0; o >>= 1) { a += __shfl_xor(a, o, 64); }
  if (lane == 0) sd[wid] = a;
  __syncthreads();
  double ta = 0.0;
  if (t == 0) for (int i = 0; i < 16; ++i) ta += sd[i];
  __syncthreads();
  for (int o = 32; o > 0; o >>= 1) { c += __shfl_xor(c, o, 64); }
  if (lane == 0) sd[wid] = c;
  __syncthreads();
  if (t == 0) {
    double tc = 0.0;
    for (int i = 0; i < 16; ++i) tc += sd[i];
    const float td = (float)(ta / d.B), cons = (float)(tc / d.B);
    d.metrics[0] = __fadd_rn(td, __fmul_rn(d.alpha, cons));
    d.metrics[1] = td;
    d.metrics[2] = cons;
  }
}

// Head backward, one workgroup per batch row b (threads over the feature
// index n), over the b's rows of the G gradient passes:
//   dprod = sum_a dq[r][a] Wf[a][n]
//   dphi_pre[r][n] = dprod * h[b][n] * [phi > 0]
//   dh[b][n] = (sum_r dprod * phi[r][n]) * [h[b][n] > 0]   (encoder fc ReLU)
//   dWf partial[b][a][n] = sum_r dq[r][a] h[b][n] phi[r][n], dbf partial[b][a]
__global__ __launch_bounds__(512) void iqn_head_bwd_kernel(d3a_iqn_head_bwd_desc d) {
  // dq rows of this b (G passes x K quantiles x A), staged once: every thread
  // reads them as LDS broadcasts
  __shared__ float sdq[D3A_IQN_HEAD_BWD_MAX_ROWS * D3A_IQN_MAX_ACTIONS];
  const int64_t b = blockIdx.x;
  const int K = d.K, A = d.A, F = d.F;
  const int64_t BK = (int64_t)d.B * K;
  const float* __restrict__ phi = d.phi;
  float* __restrict__ dphi = d.dphi;
  for (int i = threadIdx.x; i < d.G * K * A; i += 512) {
    const int gk = i / A, a = i - gk * A;
    const int g = gk / K, k = gk - g * K;
    sdq[i] = d.dq[(g * BK + b * K + k) * A + a];
  }
  __syncthreads();
  constexpr int UR = 8;  // rows loaded before any is processed
  for (int n = threadIdx.x; n < F; n += 512) {
    const float hv = d.h[b * F + n];
    float wv[D3A_IQN_MAX_ACTIONS];
#pragma unroll
    for (int a = 0; a < D3A_IQN_MAX_ACTIONS; ++a) wv[a] = a < A ? d.Wf[(int64_t)a * F + n] : 0.f;
    float dh = 0.f;
    float dw[D3A_IQN_MAX_ACTIONS];
#pragma unroll
    for (int a = 0; a < D3A_IQN_MAX_ACTIONS; ++a) dw[a] = 0.f;
    for (int g = 0; g < d.G; ++g) {
      const int64_t rbase = g * BK + b * K;
      for (int k0 = 0; k0 < K; k0 += UR) {
        float ph[UR];
#pragma unroll
        for (int u = 0; u < UR; ++u) ph[u] = k0 + u < K ? phi[(rbase + k0 + u) * F + n] : 0.f;
#pragma unroll
        for (int u = 0; u < UR; ++u) {
          if (k0 + u >= K) break;
          const int64_t r = rbase + k0 + u;
          const float* sq = &sdq[(g * K + k0 + u) * A];
          float dp = 0.f;
#pragma unroll
          for (int a = 0; a < D3A_IQN_MAX_ACTIONS; ++a) {
            if (a >= A) break;
            const float q = sq[a];
            dp = fmaf(q, wv[a], dp);
            dw[a] = fmaf(q, __fmul_rn(hv, ph[u]), dw[a]);
          }
          dphi[r * F + n] = ph[u] > 0.f ? __fmul_rn(dp, hv) : 0.f;
          dh = fmaf(dp, ph[u], dh);
        }
      }
    }
    d.dh[b * F + n] = hv > 0.f ? dh : 0.f;
#pragma unroll
    for (int a = 0; a < D3A_IQN_MAX_ACTIONS; ++a)
      if (a < A) d.dWf_part[(b * A + a) * F + n] = dw[a];
  }
  if (threadIdx.x < (unsigned)A) {
    const int a = threadIdx.x;
    double s = 0.0;
    for (int gk = 0; gk < d.G * K; ++gk) s += (double)sdq[gk * A + a];
    d.dbf_part[b * A + a] = (float)s;
  }
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_im2col(const d3a_im2col_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->col && ((d->x_u8 != nullptr) != (d->x_f32 != nullptr)),
                "d3a_im2col: need col and exactly one input");
  D3A_CHECK_ARG(d->B >= 1 && d->C >= 1 && d->S >= 1 && d->OH == (d->H - d->KH) / d->S + 1 &&
                d->OW == (d->W - d->KW) / d->S + 1 && d->ldcol >= (int64_t)d->C * d->KH * d->KW,
                "d3a_im2col: inconsistent geometry");
  const int64_t n = (int64_t)d->B * d->OH * d->OW * d->C * d->KH * d->KW;
  hipLaunchKernelGGL(im2col_kernel, dim3(blocks256(n)), dim3(256), 0, (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_im2col");
  return 0;
}

extern "C" int d3a_col2im(const d3a_col2im_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->dcol && d->dx, "d3a_col2im: null pointer");
  D3A_CHECK_ARG(d->OH == (d->H - d->KH) / d->S + 1 && d->OW == (d->W - d->KW) / d->S + 1,
                "d3a_col2im: inconsistent geometry");
  const int64_t n = (int64_t)d->B * d->H * d->W * d->C;
  hipLaunchKernelGGL(col2im_kernel, dim3(blocks256(n)), dim3(256), 0, (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_col2im");
  return 0;
}

extern "C" int d3a_iqn_transpose(const d3a_transpose_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->src && d->dst && d->src != d->dst, "d3a_iqn_transpose: bad pointers");
  hipLaunchKernelGGL(transpose_kernel, dim3(blocks256((int64_t)d->B * d->P * d->C)), dim3(256),
                     0, (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_iqn_transpose");
  return 0;
}

extern "C" int d3a_iqn_prior(const d3a_iqn_prior_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->taus && d->prior && d->E >= 1, "d3a_iqn_prior: bad args");
  hipLaunchKernelGGL(iqn_prior_kernel, dim3(blocks256(d->rows * d->E)), dim3(256), 0,
                     (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_iqn_prior");
  return 0;
}

extern "C" int d3a_iqn_head_fwd(const d3a_iqn_head_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->phi && d->Wf && d->bf && d->q, "d3a_iqn_head_fwd: null pointer");
  D3A_CHECK_ARG(d->A >= 1 && d->A <= D3A_IQN_MAX_ACTIONS && d->K >= 1 && d->group_rows >= 1,
                "d3a_iqn_head_fwd: bad sizes");
  const int64_t groups = (d->rows + d->group_rows - 1) / d->group_rows;
  D3A_CHECK_ARG(groups <= D3A_IQN_MAX_GROUPS, "d3a_iqn_head_fwd: too many row groups");
  for (int64_t g = 0; g < groups; ++g) D3A_CHECK_ARG(d->h[g], "d3a_iqn_head_fwd: null h group");
  const bool vec = d->F % 4 == 0 && d->F <= 512 &&
                   (reinterpret_cast<uintptr_t>(d->phi) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(d->Wf) & 15) == 0;
  bool hvec = true;
  for (int64_t g = 0; g < groups; ++g) hvec = hvec && (reinterpret_cast<uintptr_t>(d->h[g]) & 15) == 0;
  if (vec && hvec)
    hipLaunchKernelGGL(iqn_head_fwd4_kernel, dim3((unsigned)((d->rows + 15) / 16)), dim3(256), 0,
                       (hipStream_t)stream, *d);
  else
    hipLaunchKernelGGL(iqn_head_fwd_kernel, dim3((unsigned)((d->rows + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_iqn_head_fwd");
  return 0;
}

extern "C" int d3a_iqn_loss(const d3a_iqn_loss_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->q_loss && d->q_next && d->q_targ && d->act && d->rew && d->term &&
                d->n_steps && d->taus_loss && d->dq && d->loss_b && d->cons_b && d->metrics,
                "d3a_iqn_loss: null pointer");
  D3A_CHECK_ARG(d->K >= 1 && d->K <= 1024 && d->A >= 1 && d->A <= D3A_IQN_MAX_ACTIONS,
                "d3a_iqn_loss: bad sizes");
  hipLaunchKernelGGL(iqn_loss_kernel, dim3((unsigned)d->B), dim3(256), 0, (hipStream_t)stream, *d);
  hipLaunchKernelGGL(iqn_loss_reduce_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_iqn_loss");
  return 0;
}

extern "C" int d3a_iqn_head_bwd(const d3a_iqn_head_bwd_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->h && d->phi && d->dq && d->Wf && d->dphi && d->dh && d->dWf_part &&
                d->dbf_part, "d3a_iqn_head_bwd: null pointer");
  D3A_CHECK_ARG(d->A >= 1 && d->A <= D3A_IQN_MAX_ACTIONS && d->G >= 1, "d3a_iqn_head_bwd: bad sizes");
  D3A_CHECK_ARG((int64_t)d->G * d->K <= D3A_IQN_HEAD_BWD_MAX_ROWS,
                "d3a_iqn_head_bwd: G * K exceeds D3A_IQN_HEAD_BWD_MAX_ROWS");
  hipLaunchKernelGGL(iqn_head_bwd_kernel, dim3((unsigned)d->B), dim3(512), 0, (hipStream_t)stream,
                     *d);
  D3A_LAUNCH_CHECK("d3a_iqn_head_bwd");
  return 0;
}
