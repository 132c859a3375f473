// The whole backward of a small-batch two-hidden-layer MLP, [n_in <= 64 ->
// 256 -> 256 -> n_out <= 256] with ReLU hidden layers, in two launches: what the
// per-layer path ran as 4-5 split-K / input-gradient GEMM launches of a few
// hundred rows each (each at the launch floor: K3's VAE decoder / encoder,
// QR critics, actor critic pass and residual policy, bcq_impl.py:132-161,
// ddpg_impl.py:138-165 through encoders.py:265-275, 328-339 and the heads
// qr_q_function.py:126-128, policies.py:94-97, imitators.py:63-86).
//
// Given dz3 = dL/d(out) [C][rows][n_out] and the forward's kept h1, h2:
//   dz2 = (dz3 W3) * [h2 > 0]        dW3 = dz3^T h2,  db3 = sum dz3
//   dz1 = (dz2 W2) * [h1 > 0]        dW2 = dz2^T h1,  db2 = sum dz2
//   dx  = dz1 W1 (optional)          dW1 = dz1^T x,   db1 = sum dz1
// A workgroup owns 32 rows (row block rb) x 32 units (slice s of the 256) of
// one member: dz2 for its units needs only W3's 32 columns, so dW3 / dW2 /
// db2 of the slice and the slice's share of dz2 W2 (K = its 32 units) are
// independent per workgroup.  The eight slices' dz2 W2 shares go to a scratch
// [8][C][rows][256]; a second launch of 32-row workgroups sums them in slice
// order, applies the h1 mask and forms dW1 / db1 / dx.  (One launch with the
// last slice of a row block running that stage behind a ticket, as
// cql_lse_loss_kernel, measured 50-78 us: each workgroup's device-scope fence
// writes back its XCD's L2, and the slices of a row block sit on different
// XCDs.)  Weight gradients are partials per row block [rows / 32][C][out][in],
// summed in order by the Adam kernel.  Exact fp32 arithmetic (VALU fma
// chains), operands staged in LDS.
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

constexpr int SB_H = 256;      // hidden width
constexpr int SB_RB = 32;      // rows per workgroup
constexpr int SB_US = 32;      // units per slice
constexpr int SB_NS = SB_H / SB_US;
constexpr int SB_OMAX = 256;   // n_out
constexpr int SB_IMAX = 64;    // n_in
constexpr int SB_LH = SB_H + 4;     // float stride of a 256-wide row image
constexpr int SB_LS = SB_US + 4;    // float stride of a 32-wide slice image
constexpr int SB_LX = SB_IMAX + 4;

struct SbLds {
  union {
    struct {
      float dz3[SB_RB][SB_OMAX + 4];   // dL/d(out) rows
      float w3[SB_OMAX][SB_LS];        // W3[:, slice]
    } a;
    float w1[SB_H][SB_IMAX + 1];       // phase B: W1 rows (dx)
  } u;
  float h2[SB_RB][SB_LS];    // h2[:, slice]
  float dz2[SB_RB][SB_LS];   // dz2[:, slice]
  float h1[SB_RB][SB_LH];
  float w2[SB_US][SB_LH];    // W2[slice, :]; phase B: dz1 rows
  float x[SB_RB][SB_LX];
};

__global__ __launch_bounds__(512) void mlp_bwd_small_a_kernel(d3a_mlp_bwd_small_desc d) {
  __shared__ __attribute__((aligned(16))) SbLds L;
  const int t = threadIdx.x;
  const int s = blockIdx.x, rb = blockIdx.y, c = blockIdx.z;
  const int C = d.C, R = d.rows, n_out = d.n_out;
  const int r0 = rb * SB_RB;
  const int nr = R - r0 < SB_RB ? R - r0 : SB_RB;
  const int u0 = s * SB_US;
  const float* dz3g = d.dout + c * d.sdout + (int64_t)r0 * d.ld_dout;
  const float* h1g = d.h1 + c * d.sh + (int64_t)r0 * SB_H;
  const float* h2g = d.h2 + c * d.sh + (int64_t)r0 * SB_H;
  const float* W2 = d.W2 + c * d.sW2;
  const float* W3 = d.W3 + c * d.sW3;
  const bool wg = d.dW1 != nullptr;

  // ---- stage: dz3 rows, W3[:, slice], h2[:, slice], h1 rows, W2[slice, :]
  for (int i = t; i < SB_RB * n_out; i += 512) {
    const int m = i / n_out, o = i - m * n_out;
    L.u.a.dz3[m][o] = m < nr ? dz3g[(int64_t)m * d.ld_dout + o] : 0.f;
  }
  for (int i = t; i < n_out * (SB_US / 4); i += 512) {
    const int o = i >> 3, u4 = 4 * (i & 7);
    *reinterpret_cast<float4*>(&L.u.a.w3[o][u4]) = *reinterpret_cast<const float4*>(W3 + o * SB_H + u0 + u4);
  }
  for (int i = t; i < SB_RB * (SB_H / 4); i += 512) {
    const int m = i >> 6, i4 = 4 * (i & 63);
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(&L.h1[m][i4]) = m < nr ? *reinterpret_cast<const float4*>(h1g + m * SB_H + i4) : z;
    if (i < SB_US * (SB_H / 4))
      *reinterpret_cast<float4*>(&L.w2[m][i4]) = *reinterpret_cast<const float4*>(W2 + (u0 + m) * SB_H + i4);
    if ((i4 >> 5) == s)  // this slice's 32 columns of h2
      *reinterpret_cast<float4*>(&L.h2[m][i4 - u0]) =
          m < nr ? *reinterpret_cast<const float4*>(h2g + m * SB_H + i4) : z;
  }
  __syncthreads();

  // ---- dz2 of the slice: thread (m, 4 units), K = n_out
  if (t < SB_RB * (SB_US / 4)) {
    const int m = t >> 3, u4 = 4 * (t & 7);
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll 8
    for (int o = 0; o < n_out; ++o) {
      const float g = L.u.a.dz3[m][o];
      const float4 w = *reinterpret_cast<const float4*>(&L.u.a.w3[o][u4]);
      a0 = fmaf(g, w.x, a0);
      a1 = fmaf(g, w.y, a1);
      a2 = fmaf(g, w.z, a2);
      a3 = fmaf(g, w.w, a3);
    }
    const float4 hv = *reinterpret_cast<const float4*>(&L.h2[m][u4]);
    *reinterpret_cast<float4*>(&L.dz2[m][u4]) =
        make_float4(hv.x > 0.f ? a0 : 0.f, hv.y > 0.f ? a1 : 0.f, hv.z > 0.f ? a2 : 0.f, hv.w > 0.f ? a3 : 0.f);
  }
  __syncthreads();

  const int64_t pw = (int64_t)rb * C + c;  // this row block's partial, member c
  if (wg) {
    // dW3[:, slice] = dz3^T h2[:, slice] (K = the block's rows); db3 on slice 0
    float* dW3 = d.dW3 + pw * n_out * SB_H;
    for (int g = t; g < n_out * (SB_US / 4); g += 512) {
      const int o = g >> 3, u4 = 4 * (g & 7);
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll 8
      for (int m = 0; m < SB_RB; ++m) {
        const float q = L.u.a.dz3[m][o];
        const float4 hv = *reinterpret_cast<const float4*>(&L.h2[m][u4]);
        a0 = fmaf(q, hv.x, a0);
        a1 = fmaf(q, hv.y, a1);
        a2 = fmaf(q, hv.z, a2);
        a3 = fmaf(q, hv.w, a3);
      }
      *reinterpret_cast<float4*>(dW3 + o * SB_H + u0 + u4) = make_float4(a0, a1, a2, a3);
    }
    if (s == 0) {
      for (int o = t; o < n_out; o += 512) {
        float a = 0.f;
        for (int m = 0; m < SB_RB; ++m) a += L.u.a.dz3[m][o];
        d.db3[pw * n_out + o] = a;
      }
    }
    // dW2[slice, :] = dz2[:, slice]^T h1; db2[slice]
    {
      const int u = t >> 4, i16 = 16 * (t & 15);
      float a[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) a[j] = 0.f;
#pragma unroll 4
      for (int m = 0; m < SB_RB; ++m) {
        const float g = L.dz2[m][u];
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
          const float4 hv = *reinterpret_cast<const float4*>(&L.h1[m][i16 + 4 * j4]);
          a[4 * j4 + 0] = fmaf(g, hv.x, a[4 * j4 + 0]);
          a[4 * j4 + 1] = fmaf(g, hv.y, a[4 * j4 + 1]);
          a[4 * j4 + 2] = fmaf(g, hv.z, a[4 * j4 + 2]);
          a[4 * j4 + 3] = fmaf(g, hv.w, a[4 * j4 + 3]);
        }
      }
      float* dW2 = d.dW2 + pw * SB_H * SB_H + (int64_t)(u0 + u) * SB_H + i16;
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4)
        *reinterpret_cast<float4*>(dW2 + 4 * j4) =
            make_float4(a[4 * j4], a[4 * j4 + 1], a[4 * j4 + 2], a[4 * j4 + 3]);
      if (t < SB_US) {
        float b = 0.f;
        for (int m = 0; m < SB_RB; ++m) b += L.dz2[m][t];
        d.db2[pw * SB_H + u0 + t] = b;
      }
    }
  }
  // the slice's share of dz2 W2: P[s][c][row][i] = sum_{u in slice} dz2[row][u] W2[u][i]
  {
    const int m = t >> 4, i16 = 16 * (t & 15);
    float a[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = 0.f;
#pragma unroll 4
    for (int u = 0; u < SB_US; ++u) {
      const float g = L.dz2[m][u];
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const float4 wv = *reinterpret_cast<const float4*>(&L.w2[u][i16 + 4 * j4]);
        a[4 * j4 + 0] = fmaf(g, wv.x, a[4 * j4 + 0]);
        a[4 * j4 + 1] = fmaf(g, wv.y, a[4 * j4 + 1]);
        a[4 * j4 + 2] = fmaf(g, wv.z, a[4 * j4 + 2]);
        a[4 * j4 + 3] = fmaf(g, wv.w, a[4 * j4 + 3]);
      }
    }
    if (m < nr) {
      float* P = d.scratch + (((int64_t)s * C + c) * R + r0 + m) * SB_H + i16;
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4)
        *reinterpret_cast<float4*>(P + 4 * j4) = make_float4(a[4 * j4], a[4 * j4 + 1], a[4 * j4 + 2], a[4 * j4 + 3]);
    }
  }

}

// stage B: one workgroup per (row block, member)
__global__ __launch_bounds__(512) void mlp_bwd_small_b_kernel(d3a_mlp_bwd_small_desc d) {
  __shared__ __attribute__((aligned(16))) SbLds L;
  const int t = threadIdx.x;
  const int rb = blockIdx.y, c = blockIdx.z;
  const int C = d.C, R = d.rows, n_in = d.n_in;
  const int r0 = rb * SB_RB;
  const int nr = R - r0 < SB_RB ? R - r0 : SB_RB;
  const float* h1g = d.h1 + c * d.sh + (int64_t)r0 * SB_H;
  const float* xg = d.x + c * d.sxb + (int64_t)r0 * d.ldx;
  const float* W1 = d.W1 + c * d.sW1;
  const bool wg = d.dW1 != nullptr;
  const int64_t pw = (int64_t)rb * C + c;
  for (int i = t; i < SB_RB * (SB_H / 4); i += 512) {
    const int m = i >> 6, i4 = 4 * (i & 63);
    *reinterpret_cast<float4*>(&L.h1[m][i4]) =
        m < nr ? *reinterpret_cast<const float4*>(h1g + m * SB_H + i4) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (wg) {
    for (int i = t; i < SB_RB * n_in; i += 512) {
      const int m = i / n_in, k = i - m * n_in;
      L.x[m][k] = m < nr ? xg[(int64_t)m * d.ldx + k] : 0.f;
    }
  }
  __syncthreads();  // h1 staged
  // dz1 = (sum_s P[s]) * [h1 > 0] into the w2 image
  {
    const int m = t >> 4, i16 = 16 * (t & 15);
    float a[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = 0.f;
    if (m < nr) {
      for (int q = 0; q < SB_NS; ++q) {
        const float* P = d.scratch + (((int64_t)q * C + c) * R + r0 + m) * SB_H + i16;
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
          const float4 v = *reinterpret_cast<const float4*>(P + 4 * j4);
          a[4 * j4 + 0] += v.x;
          a[4 * j4 + 1] += v.y;
          a[4 * j4 + 2] += v.z;
          a[4 * j4 + 3] += v.w;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) L.w2[m][i16 + j] = L.h1[m][i16 + j] > 0.f ? a[j] : 0.f;
  }
  // W1 rows for dx
  if (d.dx) {
    for (int i = t; i < SB_H * n_in; i += 512) {
      const int r = i / n_in, k = i - r * n_in;
      L.u.w1[r][k] = W1[i];
    }
  }
  __syncthreads();
  if (wg) {
    // dW1 = dz1^T x, db1
    float* dW1 = d.dW1 + pw * SB_H * n_in;
    for (int g = t; g < SB_H * n_in; g += 512) {
      const int i = g / n_in, k = g - i * n_in;
      float a = 0.f;
#pragma unroll 8
      for (int m = 0; m < SB_RB; ++m) a = fmaf(L.w2[m][i], L.x[m][k], a);
      dW1[g] = a;
    }
    if (t < SB_H) {
      float b = 0.f;
      for (int m = 0; m < SB_RB; ++m) b += L.w2[m][t];
      d.db1[pw * SB_H + t] = b;
    }
  }
  if (d.dx) {
    // dx[row][k] = sum_i dz1[row][i] W1[i][k]
    float* dx = d.dx + ((int64_t)c * R + r0) * n_in;
    for (int g = t; g < SB_RB * n_in; g += 512) {
      const int m = g / n_in, k = g - m * n_in;
      if (m >= nr) continue;
      float a = 0.f;
#pragma unroll 8
      for (int i = 0; i < SB_H; ++i) a = fmaf(L.w2[m][i], L.u.w1[i][k], a);
      dx[(int64_t)m * n_in + k] = a;
    }
  }
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_mlp_bwd_small(const d3a_mlp_bwd_small_desc* dp, void* stream) {
  D3A_CHECK_ARG(dp, "d3a_mlp_bwd_small: null desc");
  const d3a_mlp_bwd_small_desc& d = *dp;
  D3A_CHECK_ARG(d.x && d.h1 && d.h2 && d.dout && d.W1 && d.W2 && d.W3 && d.scratch,
                "d3a_mlp_bwd_small: null operand");
  const bool wg = d.dW1 != nullptr;
  D3A_CHECK_ARG(!wg || (d.db1 && d.dW2 && d.db2 && d.dW3 && d.db3),
                "d3a_mlp_bwd_small: weight gradients all or none");
  D3A_CHECK_ARG(wg || d.dx, "d3a_mlp_bwd_small: nothing to compute");
  D3A_CHECK_ARG(d.n_in >= 1 && d.n_in <= SB_IMAX && d.n_out >= 1 && d.n_out <= SB_OMAX && d.C >= 1 &&
                    d.rows >= 1 && d.rows <= 65536,
                "d3a_mlp_bwd_small: needs [n_in <= 64, 256, 256, n_out <= 256]");
  auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  D3A_CHECK_ARG(a16(d.h1) && a16(d.h2) && a16(d.W2) && a16(d.W3) && a16(d.scratch) && d.sh % 4 == 0 &&
                    d.sW2 % 4 == 0 && d.sW3 % 4 == 0 && (!wg || (a16(d.dW2) && a16(d.dW3))),
                "d3a_mlp_bwd_small: h / W2 / W3 / scratch / dW2 / dW3 must be 16-byte aligned");
  const int NRB = (d.rows + SB_RB - 1) / SB_RB;
  hipLaunchKernelGGL(mlp_bwd_small_a_kernel, dim3(SB_NS, NRB, d.C), dim3(512), 0, (hipStream_t)stream, d);
  hipLaunchKernelGGL(mlp_bwd_small_b_kernel, dim3(1, NRB, d.C), dim3(512), 0, (hipStream_t)stream, d);
  D3A_LAUNCH_CHECK("d3a_mlp_bwd_small");
  return 0;
}
