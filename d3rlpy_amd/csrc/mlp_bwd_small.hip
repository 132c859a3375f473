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
// summed in order by the Adam kernel.  The products run on the fp32 matrix
// cores (v_mfma_f32_32x32x2_f32: fp32 products and sums), operands staged in
// LDS; round 5's first version ran them as VALU fma chains at 30 + 13 us.
#include <cstdlib>
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

typedef float f32x16 __attribute__((ext_vector_type(16)));

// one 32 x 32 x 2 fp32 matrix-core step: lane l supplies A[l & 31][l >> 5] and
// B[l >> 5][l & 31]; the accumulator holds column l & 31, rows 8 R + 4 (l >> 5)
// + i in element 4 R + i (fp32 products and sums: the fp32-exact path)
__device__ __forceinline__ f32x16 mf32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
// NK steps of mf32 with every operand read (fa(p), fb(p): LDS or registers)
// before the first MFMA: the reads of a step no longer wait in front of it
template <int NK, typename FA, typename FB>
__device__ __forceinline__ f32x16 mf32_run(f32x16 acc, FA fa, FB fb) {
  float a[NK], b[NK];
#pragma unroll
  for (int p = 0; p < NK; ++p) {
    a[p] = fa(p);
    b[p] = fb(p);
  }
#pragma unroll
  for (int p = 0; p < NK; ++p) acc = mf32(a[p], b[p], acc);
  return acc;
}
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// diagnostic phase stamps (STAMPS, D3A_SB_STAMPS=1; d3a_small_bwd_stamps):
// wave 0 of each workgroup, [stage][workgroup][4]: stage A 0 start, 1 staged,
// 2 dz2 formed, 3 end; stage B 0 start, 1 staged, 2 dz1 formed, 3 end
constexpr int SB_NST = 4, SB_MAXWG = 1024;
__device__ unsigned long long sb_stamps[2 * SB_MAXWG * SB_NST];

struct SbLdsA {
  float dz3[SB_RB][SB_OMAX + 4];   // dL/d(out) rows
  float w3[SB_OMAX][SB_LS];        // W3[:, slice]
  float h2[SB_RB][SB_LS];          // h2[:, slice]
  float dz2[SB_RB][SB_LS];         // dz2[:, slice]
  float h1[SB_RB][SB_LH];
  float w2[SB_US][SB_LH];          // W2[slice, :]
  float red[4][SB_RB * SB_US];     // dz2's four K-quarter partial tiles
};

struct SbLdsB {
  float h1[SB_RB][SB_LH];
  float dz1[SB_RB][SB_LH];
  float x[SB_RB][SB_LX];
  float red[8][SB_RB * 32];        // dx's K-chunk partial tiles
};

// stage A: one workgroup per (slice, row block, member).  Waves 0-3 form the
// slice's dz2 over K-quarters of n_out, waves 4-7 meanwhile dW3[:, slice];
// then dz2 (quarters summed in order, h2's mask) and per wave one 32-column
// tile each of dW2[slice, :] and of the slice's dz2 W2 share.
template <bool STAMPS>
__global__ __launch_bounds__(512) void mlp_bwd_small_a_kernel(d3a_mlp_bwd_small_desc d) {
  __shared__ __attribute__((aligned(16))) SbLdsA L;
  const int t = threadIdx.x;
  const int wgi = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  auto stamp = [&](int k) {
    if constexpr (STAMPS) {
      __builtin_amdgcn_sched_barrier(0);
      if (t == 0 && wgi < SB_MAXWG) sb_stamps[wgi * SB_NST + k] = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  stamp(0);
  const int w = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63, li = lane & 31, lh = lane >> 5;
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

  // ---- stage: dz3 rows, W3[:, slice], h2[:, slice], h1 rows, W2[slice, :].
  // Every load is issued (from clamped, always valid addresses) before any is
  // stored: a load under a branch makes the compiler wait for all in flight.
  // dz3: thread (row t >> 4, outputs (t & 15) + 16 j)
  const int jn = (n_out + 15) / 16;  // uniform
  const int mz = t >> 4, oz = t & 15;
  const int mzc = mz < nr ? mz : nr - 1;
  float vz[SB_OMAX / 16];
#pragma unroll
  for (int j = 0; j < SB_OMAX / 16; ++j)
    if (j < jn) vz[j] = dz3g[(int64_t)mzc * d.ld_dout + min(oz + 16 * j, n_out - 1)];
  // W3[:, slice]: (output o, 4 units) pieces, up to four a thread
  constexpr int QW = SB_OMAX * (SB_US / 4) / 512;
  float4 vw[QW];
#pragma unroll
  for (int q = 0; q < QW; ++q) {
    const int i = min(t + 512 * q, n_out * (SB_US / 4) - 1);
    vw[q] = *reinterpret_cast<const float4*>(W3 + (i >> 3) * SB_H + u0 + 4 * (i & 7));
  }
  // h1 rows, W2[slice, :], h2[:, slice]: four 16-byte pieces a thread each
  float4 vh[4], v2[4], vh2[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = t + 512 * q;
    const int m = i >> 6, i4 = 4 * (i & 63);
    const int mc = m < nr ? m : nr - 1;
    vh[q] = *reinterpret_cast<const float4*>(h1g + mc * SB_H + i4);
    v2[q] = *reinterpret_cast<const float4*>(W2 + (u0 + (m & (SB_US - 1))) * SB_H + i4);
    vh2[q] = *reinterpret_cast<const float4*>(h2g + mc * SB_H + u0 + 4 * (i & 7));
  }
#pragma unroll
  for (int j = 0; j < SB_OMAX / 16; ++j)
    if (j < jn && oz + 16 * j < n_out) L.dz3[mz][oz + 16 * j] = mz < nr ? vz[j] : 0.f;
#pragma unroll
  for (int q = 0; q < QW; ++q) {
    const int i = t + 512 * q;
    if (i < n_out * (SB_US / 4)) *reinterpret_cast<float4*>(&L.w3[i >> 3][4 * (i & 7)]) = vw[q];
  }
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = t + 512 * q;
    const int m = i >> 6, i4 = 4 * (i & 63);
    *reinterpret_cast<float4*>(&L.h1[m][i4]) = m < nr ? vh[q] : z;
    if (i < SB_US * (SB_H / 4)) *reinterpret_cast<float4*>(&L.w2[m][i4]) = v2[q];
    if ((i & 63) < 8) {  // (row m, pieces 0-7 of the slice): h2[:, slice]
      *reinterpret_cast<float4*>(&L.h2[m][4 * (i & 7)]) = m < nr ? vh2[q] : z;
    }
  }
  __syncthreads();
  stamp(1);

  const int64_t pw = (int64_t)rb * C + c;  // this row block's partial, member c
  if (w < 4) {
    // dz2 partial over k pairs p = w, w + 4, ..: A = dz3[row][k], B = W3[k][u]
    f32x16 acc = zero16();
    const int np = (n_out + 1) / 2;
    for (int p0 = w; p0 < np; p0 += 4 * 8) {  // eight steps a batch (pairs p0 + 4 q)
      acc = mf32_run<8>(
          acc,
          [&](int q) {
            const int k = 2 * (p0 + 4 * q) + lh;
            return k < n_out ? L.dz3[li][k] : 0.f;
          },
          [&](int q) {
            const int k = 2 * (p0 + 4 * q) + lh;
            return k < n_out ? L.w3[k < n_out ? k : 0][li] : 0.f;
          });
    }
#pragma unroll
    for (int R = 0; R < 4; ++R)
#pragma unroll
      for (int i = 0; i < 4; ++i) L.red[w][(8 * R + 4 * lh + i) * SB_US + li] = acc[4 * R + i];
  } else if (wg) {
    // dW3[:, slice] = dz3^T h2[:, slice], K = the block's rows: tiles of 32 o
    float* dW3 = d.dW3 + pw * n_out * SB_H;
    for (int tt = w - 4; tt < (n_out + 31) / 32; tt += 4) {
      const int o = 32 * tt + li;
      const f32x16 acc = mf32_run<SB_RB / 2>(
          zero16(), [&](int p) { return o < n_out ? L.dz3[2 * p + lh][o] : 0.f; },
          [&](int p) { return L.h2[2 * p + lh][li]; });
#pragma unroll
      for (int R = 0; R < 4; ++R)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int oo = 32 * tt + 8 * R + 4 * lh + i;
          if (oo < n_out) dW3[oo * SB_H + u0 + li] = acc[4 * R + i];
        }
    }
  }
  if (wg && s == 0) {
    for (int o = t; o < n_out; o += 512) {
      float a = 0.f;
      for (int m = 0; m < SB_RB; ++m) a += L.dz3[m][o];
      d.db3[pw * n_out + o] = a;
    }
  }
  __syncthreads();
  // dz2 = (the four quarters in order) * [h2 > 0]
  for (int e = t; e < SB_RB * SB_US; e += 512) {
    const int m = e / SB_US, u = e - m * SB_US;
    const float v = ((L.red[0][e] + L.red[1][e]) + L.red[2][e]) + L.red[3][e];
    L.dz2[m][u] = L.h2[m][u] > 0.f ? v : 0.f;
  }
  __syncthreads();
  stamp(2);

  if (wg) {
    // dW2[slice, 32 w ..] = dz2[:, slice]^T h1[:, 32 w ..]: A = dz2[m][u], B = h1[m][j]
    const f32x16 acc = mf32_run<SB_RB / 2>(
        zero16(), [&](int p) { return L.dz2[2 * p + lh][li]; },
        [&](int p) { return L.h1[2 * p + lh][32 * w + li]; });
    float* dW2 = d.dW2 + pw * SB_H * SB_H;
#pragma unroll
    for (int R = 0; R < 4; ++R)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        dW2[(int64_t)(u0 + 8 * R + 4 * lh + i) * SB_H + 32 * w + li] = acc[4 * R + i];
    if (t < SB_US) {
      float b = 0.f;
      for (int m = 0; m < SB_RB; ++m) b += L.dz2[m][t];
      d.db2[pw * SB_H + u0 + t] = b;
    }
  }
  // the slice's share of dz2 W2, columns 32 w ..: A = dz2[row][u], B = W2[u][j]
  {
    const f32x16 acc = mf32_run<SB_US / 2>(
        zero16(), [&](int p) { return L.dz2[li][2 * p + lh]; },
        [&](int p) { return L.w2[2 * p + lh][32 * w + li]; });
    float* P = d.scratch + ((int64_t)s * C + c) * R * SB_H;
#pragma unroll
    for (int R = 0; R < 4; ++R)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = 8 * R + 4 * lh + i;
        if (m < nr) P[(int64_t)(r0 + m) * SB_H + 32 * w + li] = acc[4 * R + i];
      }
  }
  stamp(3);
}

// stage B: one workgroup per (row block, member): dz1 = (the eight shares in
// slice order) * [h1 > 0], then dW1 (tiles of 32 units x 32 inputs over the
// block's rows), db1, and dx (K = 256 in eight chunks, summed in order)
template <bool STAMPS>
__global__ __launch_bounds__(512) void mlp_bwd_small_b_kernel(d3a_mlp_bwd_small_desc d) {
  __shared__ __attribute__((aligned(16))) SbLdsB L;
  const int t = threadIdx.x;
  const int wgi = blockIdx.y + gridDim.y * blockIdx.z;
  auto stamp = [&](int k) {
    if constexpr (STAMPS) {
      __builtin_amdgcn_sched_barrier(0);
      if (t == 0 && wgi < SB_MAXWG) sb_stamps[(SB_MAXWG + wgi) * SB_NST + k] = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  stamp(0);
  const int w = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63, li = lane & 31, lh = lane >> 5;
  const int rb = blockIdx.y, c = blockIdx.z;
  const int C = d.C, R = d.rows, n_in = d.n_in;
  const int r0 = rb * SB_RB;
  const int nr = R - r0 < SB_RB ? R - r0 : SB_RB;
  const float* h1g = d.h1 + c * d.sh + (int64_t)r0 * SB_H;
  const float* xg = d.x + c * d.sxb + (int64_t)r0 * d.ldx;
  const float* W1 = d.W1 + c * d.sW1;
  const bool wg = d.dW1 != nullptr;
  const int64_t pw = (int64_t)rb * C + c;
  const int NT = (n_in + 31) / 32;  // input tiles (1 or 2)
  // (loads first, from clamped addresses; then the LDS stores)
  float4 vh[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = t + 512 * q;
    const int m = i >> 6, mc = m < nr ? m : nr - 1;
    vh[q] = *reinterpret_cast<const float4*>(h1g + mc * SB_H + 4 * (i & 63));
  }
  // x: thread (row t >> 4, inputs (t & 15) + 16 j), j < 4
  float vx[4];
  const int mx = t >> 4, kx = t & 15, mxc = mx < nr ? mx : nr - 1;
#pragma unroll
  for (int j = 0; j < 4; ++j) vx[j] = xg[(int64_t)mxc * d.ldx + min(kx + 16 * j, n_in - 1)];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = t + 512 * q;
    const int m = i >> 6;
    *reinterpret_cast<float4*>(&L.h1[m][4 * (i & 63)]) = m < nr ? vh[q] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) L.x[mx][kx + 16 * j] = (mx < nr && kx + 16 * j < n_in) ? vx[j] : 0.f;
  __syncthreads();  // h1 and x staged
  stamp(1);
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
    for (int j = 0; j < 16; ++j) L.dz1[m][i16 + j] = L.h1[m][i16 + j] > 0.f ? a[j] : 0.f;
  }
  __syncthreads();
  stamp(2);
  if (wg) {
    // dW1[32 ti .. + 31][32 tj .. + 31] = dz1^T x: A = dz1[m][unit], B = x[m][k]
    float* dW1 = d.dW1 + pw * SB_H * n_in;
    for (int job = w; job < 8 * NT; job += 8) {
      const int ti = job % 8, tj = job / 8;
      const f32x16 acc = mf32_run<SB_RB / 2>(
          zero16(), [&](int p) { return L.dz1[2 * p + lh][32 * ti + li]; },
          [&](int p) { return L.x[2 * p + lh][32 * tj + li]; });
      const int k = 32 * tj + li;
      if (k < n_in) {
#pragma unroll
        for (int R = 0; R < 4; ++R)
#pragma unroll
          for (int i = 0; i < 4; ++i) dW1[(int64_t)(32 * ti + 8 * R + 4 * lh + i) * n_in + k] = acc[4 * R + i];
      }
    }
    if (t < SB_H) {
      float b = 0.f;
      for (int m = 0; m < SB_RB; ++m) b += L.dz1[m][t];
      d.db1[pw * SB_H + t] = b;
    }
  }
  if (d.dx) {
    // dx[row][32 tj ..] over units: wave w takes tile tj = w % NT and the
    // unit chunk w / NT of 8 / NT; B = W1[unit][k] from global memory
    const int tj = w % NT, nck = 8 / NT, ck = w / NT;
    const int ulen = SB_H / nck;
    const int k = 32 * tj + li;
    const int kc = k < n_in ? k : n_in - 1;
    // this lane's W1 column over the chunk, all loads issued before the MFMAs
    // (up to 32: 64 units for two input tiles)
    float wb[32];
#pragma unroll
    for (int p = 0; p < 32; ++p) wb[p] = W1[(ck * ulen + min(2 * p, ulen - 2) + lh) * n_in + kc];
    f32x16 acc = zero16();
    if (ulen == 32) {  // uniform: one input tile, eight 32-unit chunks
      acc = mf32_run<16>(acc, [&](int p) { return L.dz1[li][ck * ulen + 2 * p + lh]; },
                         [&](int p) { return k < n_in ? wb[p] : 0.f; });
    } else {
      acc = mf32_run<32>(acc, [&](int p) { return L.dz1[li][ck * ulen + 2 * p + lh]; },
                         [&](int p) { return k < n_in ? wb[p] : 0.f; });
    }
#pragma unroll
    for (int R = 0; R < 4; ++R)
#pragma unroll
      for (int i = 0; i < 4; ++i) L.red[w][(8 * R + 4 * lh + i) * 32 + li] = acc[4 * R + i];
    __syncthreads();  // uniform: dx is a kernel argument
    float* dx = d.dx + ((int64_t)c * R + r0) * n_in;
    for (int e = t; e < NT * SB_RB * 32; e += 512) {
      const int tjj = e / (SB_RB * 32), rem = e - tjj * (SB_RB * 32);
      const int m = rem / 32, kk = 32 * tjj + (rem % 32);
      if (m >= nr || kk >= n_in) continue;
      float v = L.red[tjj][rem];
      for (int q = 1; q < nck; ++q) v += L.red[q * NT + tjj][rem];
      dx[(int64_t)m * n_in + kk] = v;
    }
  }
  stamp(3);
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
  static const bool stamps = [] {
    const char* e = getenv("D3A_SB_STAMPS");
    return e && atoi(e) != 0;
  }();
  if (stamps) {
    hipLaunchKernelGGL(mlp_bwd_small_a_kernel<true>, dim3(SB_NS, NRB, d.C), dim3(512), 0, (hipStream_t)stream, d);
    hipLaunchKernelGGL(mlp_bwd_small_b_kernel<true>, dim3(1, NRB, d.C), dim3(512), 0, (hipStream_t)stream, d);
  } else {
    hipLaunchKernelGGL(mlp_bwd_small_a_kernel<false>, dim3(SB_NS, NRB, d.C), dim3(512), 0, (hipStream_t)stream, d);
    hipLaunchKernelGGL(mlp_bwd_small_b_kernel<false>, dim3(1, NRB, d.C), dim3(512), 0, (hipStream_t)stream, d);
  }
  D3A_LAUNCH_CHECK("d3a_mlp_bwd_small");
  return 0;
}

// diagnostic (synchronous, not for graphs): the stamps of the last
// D3A_SB_STAMPS=1 launch, [stage][workgroup][4]
extern "C" int d3a_small_bwd_stamps(unsigned long long* dst, int n) {
  D3A_CHECK_ARG(dst && n >= 0 && n <= 2 * SB_MAXWG * SB_NST, "d3a_small_bwd_stamps: bad arguments");
  if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(d3a::sb_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) !=
      hipSuccess) {
    set_error("d3a_small_bwd_stamps: copy failed");
    return -1;
  }
  return 0;
}
