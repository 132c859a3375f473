// Backward of the single-output Q head q = relu(h) . w + b, fused.
//
// Reference: ContinuousMeanQFunction._fc (q_functions/mean_q_function.py:255-256)
// and its autograd backward.  For every row r of an ensemble member c:
//   dz[c][r][j] = g[c][r] * w[c][j] * [h[c][r][j] > 0]        (dL/d pre-relu)
//   dW[s][c][j] = sum_{r in split s} g[c][r] * h[c][r][j]      (head weight grad)
//   db[s][c]    = sum_{r in split s} g[c][r]                   (head bias grad)
// In "argmin" mode the row gradient is not read but derived from the
// ensemble's Q values: g[c][r] = scale if c is the first argmin over members
// of q[.][r], else 0 — the backward of ``min`` over critics in
// SACImpl.compute_actor_loss (sac_impl.py:114-121; torch's min routes the
// gradient to one index).
//
// One launch replaces the column reductions and the masked outer product of
// the head backward; h is read once.  Grid: (column tiles of 64, row splits,
// members); 4 waves stride the split's rows, lanes cover columns (coalesced).
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

__global__ __launch_bounds__(1024) void head1_bwd_kernel(d3a_head1_bwd_desc d) {
  constexpr int NW = 16;  // waves per workgroup (latency hiding: many rows in flight)
  __shared__ double sw[NW][64];
  __shared__ double sb[NW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t j = (int64_t)blockIdx.x * 64 + lane;
  const int64_t s = blockIdx.y, c = blockIdx.z;
  const int64_t chunk = (d.rows + d.splits - 1) / d.splits;
  const int64_t r0 = s * chunk;
  const int64_t r1 = (r0 + chunk < d.rows) ? r0 + chunk : d.rows;
  const bool colok = j < d.n;
  const float wj = colok ? d.w[c * d.swb + j] : 0.f;
  const float* h = d.h + c * d.shb;
  float* dz = d.dz + c * d.sdzb;
  const float gs = d.gscale ? *d.gscale : 1.f;
  double accw = 0.0, accb = 0.0;
  // 8 rows per wave per iteration: all loads issued before any use
  constexpr int U = 8;
  for (int64_t rb = r0 + w; rb < r1; rb += NW * U) {
    float g[U], hv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = rb + NW * u;
      g[u] = 0.f;
      hv[u] = 0.f;
      if (r < r1) {
        if (d.q_min) {
          // first argmin over members of q[.][r]
          int arg = 0;
          float mn = d.q_min[r];
          for (int k = 1; k < d.C; ++k) {
            const float v = d.q_min[k * d.sqb + r];
            if (v < mn) { mn = v; arg = k; }
          }
          g[u] = (arg == c) ? d.scale : 0.f;
        } else {
          g[u] = d.g[c * d.sgb + r];
          if (r < d.n_scaled) g[u] *= gs;
        }
        if (colok) hv[u] = h[r * d.ldh + j];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = rb + NW * u;
      if (r < r1) {
        if (d.q_min && d.g_out && lane == 0 && blockIdx.x == 0) d.g_out[c * d.sgb + r] = g[u];
        if (colok) {
          dz[r * d.lddz + j] = hv[u] > 0.f ? g[u] * wj : 0.f;
          accw += (double)(g[u] * hv[u]);
        }
        accb += (double)g[u];
      }
    }
  }
  if (d.dW) {
    sw[w][lane] = accw;
    if (lane == 0) sb[w] = accb;
    __syncthreads();
    if (w == 0) {
      if (colok) {
        double t = 0.0;
        for (int q = 0; q < NW; ++q) t += sw[q][lane];
        d.dW[s * d.sWs + c * d.n + j] = (float)t;
      }
      if (lane == 0 && blockIdx.x == 0 && d.db)
      {
        double tb = 0.0;
        for (int q = 0; q < NW; ++q) tb += sb[q];
        d.db[s * d.sbs + c] = (float)tb;
      }
    }
  }
}

// d3a_head1_min: one wave per row; lane l holds columns 4l..4l+3 of every
// member's activation row (loaded once, used for the dot and the mask).
__global__ __launch_bounds__(256) void head1_min_kernel(d3a_head1_min_desc d) {
  constexpr int MAXC = 8;
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= d.rows) return;
  const int64_t k = (int64_t)lane * 4;
  const bool on = k < d.n;
  float4 hv[MAXC], wv[MAXC];
  float q[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    if (c >= d.C) break;
    hv[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    wv[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (on) {
      hv[c] = *reinterpret_cast<const float4*>(d.h + c * d.shb + r * d.ldh + k);
      wv[c] = *reinterpret_cast<const float4*>(d.w + c * d.swb + k);
    }
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    if (c >= d.C) break;
    // the fmaf chain of d3a_rowdot_f32 (n <= 256: one float4 per lane)
    const float a = fmaf(hv[c].w, wv[c].w,
                         fmaf(hv[c].z, wv[c].z, fmaf(hv[c].y, wv[c].y, fmaf(hv[c].x, wv[c].x, 0.f))));
    q[c] = wave_sum(a) + d.b[c * d.sbb];
  }
  int arg = 0;
  float mn = q[0];
#pragma unroll
  for (int c = 1; c < MAXC; ++c) {
    if (c >= d.C) break;
    if (q[c] < mn) { mn = q[c]; arg = c; }
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    if (c >= d.C) break;
    const float g = (arg == c) ? d.scale : 0.f;
    if (lane == 0) {
      d.q[c * d.sqb + r] = q[c];
      if (d.g_out) d.g_out[c * d.sgb + r] = g;
    }
    if (on) {
      float4 z;
      z.x = hv[c].x > 0.f ? g * wv[c].x : 0.f;
      z.y = hv[c].y > 0.f ? g * wv[c].y : 0.f;
      z.z = hv[c].z > 0.f ? g * wv[c].z : 0.f;
      z.w = hv[c].w > 0.f ? g * wv[c].w : 0.f;
      *reinterpret_cast<float4*>(d.dz + c * d.sdzb + r * d.lddz + k) = z;
    }
  }
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_head1_bwd(const d3a_head1_bwd_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->h && d->w && d->dz, "d3a_head1_bwd: null operand");
  D3A_CHECK_ARG((d->g != nullptr) != (d->q_min != nullptr),
                "d3a_head1_bwd: exactly one of g / q_min");
  D3A_CHECK_ARG(d->C >= 1 && d->rows >= 0 && d->n >= 1 && d->splits >= 1,
                "d3a_head1_bwd: bad sizes");
  D3A_CHECK_ARG(!d->dW || d->db, "d3a_head1_bwd: dW requires db");
  if (d->rows == 0) return 0;
  dim3 grid((unsigned)((d->n + 63) / 64), (unsigned)d->splits, (unsigned)d->C);
  hipLaunchKernelGGL(head1_bwd_kernel, grid, dim3(1024), 0, (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_head1_bwd");
  return 0;
}

extern "C" int d3a_head1_min(const d3a_head1_min_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->h && d->w && d->b && d->q && d->dz, "d3a_head1_min: null operand");
  D3A_CHECK_ARG(d->C >= 1 && d->C <= 8 && d->rows >= 0, "d3a_head1_min: 1..8 members");
  D3A_CHECK_ARG(d->n >= 4 && d->n <= 256 && d->n % 4 == 0, "d3a_head1_min: n must be 4..256, %4");
  D3A_CHECK_ARG(d->ldh % 4 == 0 && d->lddz % 4 == 0 && d->shb % 4 == 0 && d->sdzb % 4 == 0 &&
                    d->swb % 4 == 0 &&
                    ((reinterpret_cast<uintptr_t>(d->h) | reinterpret_cast<uintptr_t>(d->w) |
                      reinterpret_cast<uintptr_t>(d->dz)) & 15) == 0,
                "d3a_head1_min: 16-byte aligned rows");
  if (d->rows == 0) return 0;
  hipLaunchKernelGGL(head1_min_kernel, dim3((unsigned)((d->rows + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_head1_min");
  return 0;
}
