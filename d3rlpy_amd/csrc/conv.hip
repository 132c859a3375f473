// Implicit-GEMM convolutions of the Nature-DQN PixelEncoder on the gfx950
// f32-input matrix cores: no im2col matrix is ever written to HBM.
//
// Replaces nn.Conv2d forward and weight gradient in PixelEncoder._conv_encode
// (d3rlpy/models/torch/encoders.py:130-162; no padding, square stride), with
// PixelScaler.transform (preprocessing/scalers.py:109-110, x.float() / 255)
// fused into the first layer's operand load.
//
// A conv is the GEMM  y[row][co] = sum_k col(row, k) * W[co][k] + b[co], with
// row = (b, oy, ox) and k = (c, kh, kw).  Here col(row, k) is read straight
// from the layer input when the MFMA operand is loaded:
//   * uint8 NCHW frames (first layer): k in the reference's (c, kh, kw) order;
//     four consecutive kw of one kernel row are one aligned 32-bit load
//     (KW % 4 == 0, W % 4 == 0, S % 4 == 0) scaled by 1/255 (correctly
//     rounded, as the reference's fp32 division);
//   * fp32 NHWC activations (later layers): k walked in (kh, kw, c) order so
//     that four consecutive k are four consecutive channels (one 16-byte
//     load); the weight is first re-laid in that order (conv_pack_kernel).
// The sum over k is a reduction, so walking it in another order only changes
// the fp32 rounding order (the reference's CPU conv has its own order too).
//
// Forward: a wave owns 32 output rows x CO channels (CO = 32 * WN),
// v_mfma_f32_32x32x2_f32; lane l covers row / channel l & 31 and
// k = 4 * (l >> 5) + {0..3} of each 8-k group.  The input operand goes
// straight into registers; the weight is staged per 32-k chunk in LDS and
// shared by the workgroup's four waves.  The per-k-group input offsets are
// tabulated in LDS once per workgroup.
//
// Weight gradient: dW[co][k] = sum_rows dy[row][co] * col(row, k) and
// db[co] = sum_rows dy[row][co] (ReLU already applied to dy).  A wave owns a
// 32 (co) x 32*WNK (k) tile over a slice of rows; KWV waves of a workgroup
// take consecutive slices of the split and are summed through LDS in wave
// order; the split's partial goes to dW[split] (summed in order by the Adam
// kernel), so the result is run-to-run deterministic.
#include <cstdlib>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"
#include "x6.hpp"

namespace d3a {
namespace {

using x6::f32x16;
constexpr int kMaxKGroups = 1024;  // C*KH*KW <= 4096

// x / 255 correctly rounded (== torch's x.float() / 255.0) for x in 0..255
// without a full IEEE division: q = x * fl(1/255), one Newton residual step
// with exact fma (checked exhaustively, tests/test_gpu_conv.py)
__device__ __forceinline__ float px(uint32_t byte) {
  const float x = (float)byte, r = 1.f / 255.f;
  const float q = __fmul_rn(x, r);
  const float e = fmaf(-q, 255.f, x);
  return fmaf(e, r, q);
}

// input offset of k-group g (4 consecutive k) relative to the row's window
// origin (walk order: (c, kh, kw) for uint8 input, (kh, kw, c) for fp32)
template <bool U8>
__device__ __forceinline__ int kgroup_offset(const d3a_conv_desc& d, int g) {
  const int k = 4 * g, KK = d.KH * d.KW;
  if (U8) {
    const int c = k / KK, r = k - c * KK, kh = r / d.KW, kw = r - kh * d.KW;
    return (c * d.H + kh) * d.W + kw;
  }
  const int c = k % d.C, t = k / d.C, kw = t % d.KW, kh = t / d.KW;
  return (kh * d.W + kw) * d.C + c;
}

template <bool U8>
__device__ __forceinline__ int64_t window_origin(const d3a_conv_desc& d, int64_t b, int oy, int ox) {
  if (U8) return (b * d.C * d.H + (int64_t)oy * d.S) * d.W + (int64_t)ox * d.S;
  return ((b * d.H + (int64_t)oy * d.S) * d.W + (int64_t)ox * d.S) * d.C;
}

// weight [CO][C][KH][KW] -> wpack [CO][KH][KW][C] (the fp32 walk order)
__global__ __launch_bounds__(256) void conv_pack_kernel(const float* __restrict__ w,
                                                        float* __restrict__ wp, int C, int KH,
                                                        int KW, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int Kc = C * KH * KW;
  const int64_t co = i / Kc;
  const int kp = (int)(i - co * Kc);
  const int c = kp % C, t = kp / C, kw = t % KW, kh = t / KW;
  wp[i] = w[co * Kc + (c * KH + kh) * KW + kw];
}

// Forward.  Workgroup: 4 waves x 32 rows; each wave 32 rows x CO channels.
// K is walked in chunks of 32: the workgroup stages the chunk's weights
// (CO x 32, from the walk-ordered weight, coalesced) into LDS, double
// buffered, one barrier per chunk; the input operand is loaded straight into
// registers one chunk ahead.
template <int WN, bool U8, bool ALIGNED>
__global__ __launch_bounds__(256) void conv_fwd_kernel(d3a_conv_desc d, const float* __restrict__ wk) {
  constexpr int CO = 32 * WN, BK = 32, LDW = BK + 4, U = BK / 8;
  __shared__ int ta[kMaxKGroups];
  __shared__ __attribute__((aligned(16))) float Ws[2][CO * LDW];
  const int KK = d.KH * d.KW;
  const int Kc = d.C * KK;
  const int G = Kc / 4;
  for (int g = threadIdx.x; g < G; g += 256) ta[g] = kgroup_offset<U8>(d, g);

  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const int li = lane & 31, lg = lane >> 5;
  const int P = d.OH * d.OW;
  const int64_t M = (int64_t)d.B * P;
  const int64_t m0 = ((int64_t)blockIdx.x * 4 + w) * 32;
  const int64_t m = m0 + li;
  const bool valid = m < M;
  int64_t org = 0;
  if (valid) {
    const int64_t b = m / P;
    const int p = (int)(m - b * P);
    const int oy = p / d.OW, ox = p - oy * d.OW;
    org = window_origin<U8>(d, b, oy, ox);
  }

  // weight chunk loader: WN float4 per thread (CO rows x 8 float4)
  float4 wr[WN];
  auto wload = [&](int k0) {
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int v = t + 256 * j, co = v >> 3, q = v & 7;
      const int k = k0 + 4 * q;
      wr[j] = k < Kc ? *reinterpret_cast<const float4*>(wk + (int64_t)co * Kc + k)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto wstore = [&](int buf) {
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int v = t + 256 * j, co = v >> 3, q = v & 7;
      *reinterpret_cast<float4*>(&Ws[buf][co * LDW + 4 * q]) = wr[j];
    }
  };
  float4 ra[U];
  auto aload = [&](int k0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int g = k0 / 4 + 2 * u + lg;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      if (valid && g < G) {
        if (U8) {
          const uint8_t* s = d.x_u8 + org + ta[g];
          if (ALIGNED) {
            const uint32_t x = *reinterpret_cast<const uint32_t*>(s);
            a = make_float4(px(x & 255u), px((x >> 8) & 255u), px((x >> 16) & 255u), px(x >> 24));
          } else {
            a = make_float4(px(s[0]), px(s[1]), px(s[2]), px(s[3]));
          }
        } else {
          a = *reinterpret_cast<const float4*>(d.x_f32 + org + ta[g]);
        }
      }
      ra[u] = a;
    }
  };

  f32x16 acc[WN];
#pragma unroll
  for (int j = 0; j < WN; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  wload(0);
  wstore(0);
  __syncthreads();  // also publishes the offset table
  aload(0);
  int cur = 0;
  for (int k0 = 0; k0 < Kc; k0 += BK) {
    const bool more = k0 + BK < Kc;
    if (more) wload(k0 + BK);
    float4 ca[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ca[u] = ra[u];
    if (more) aload(k0 + BK);
    const float* Wc = Ws[cur];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        const float4 bv = *reinterpret_cast<const float4*>(&Wc[(32 * j + li) * LDW + 8 * u + 4 * lg]);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ca[u].x, bv.x, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ca[u].y, bv.y, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ca[u].z, bv.z, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ca[u].w, bv.w, acc[j], 0, 0, 0);
      }
    }
    if (more) wstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  if (m0 >= M) return;
  // epilogue: acc[j][r] -> row m0 + (r&3) + 8*(r>>2) + 4*lg, channel 32*j + li
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    const int n = 32 * j + li;
    const float bn = d.bias ? d.bias[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t mm = m0 + (r & 3) + 8 * (r >> 2) + 4 * lg;
      if (mm < M) {
        float v = acc[j][r] + bn;
        if (d.relu) v = fmaxf(v, 0.f);
        d.y[mm * CO + n] = v;
      }
    }
  }
}

// Forward on the bf16 matrix cores at fp32 accuracy (x6.hpp): the same
// implicit GEMM, 16 k per v_mfma_f32_32x32x16_bf16.  Weights are staged per
// 32-k chunk as three exact bf16 parts, read from nn.Conv2d's layout in the
// walk order directly (no conv_pack launch).  fp32 input: the activation is
// split into three parts too, six part products.  uint8 input (the first
// layer): the byte x itself is the A operand -- an integer 0..255, exact in
// one bf16 part -- so a tap is three products, and the pixel scale is applied
// to the sum, fl(sum x W) / 255 (correctly rounded), against the reference's
// sum fl(x / 255) W: the same value up to fp32 rounding, and bit for bit the
// reference's x / 255 where one tap carries the output (tests/test_gpu_conv.py:
// the one-hot pixel-scale test and the 2e-5 bar against fp64).
// PACKED (fp32 input): the weight was re-laid in the walk order into d.wpack
// (conv_pack_kernel), so a chunk row is 32 consecutive floats
template <int WN, bool U8, bool ALIGNED = false, bool PACKED = false>
__global__ __launch_bounds__(256) void conv_fwd_x6_kernel(d3a_conv_desc d) {
  using namespace x6;
  constexpr int CO = 32 * WN, BK = 32, LDB = BK + 8;
  __shared__ int ta[kMaxKGroups];
  __shared__ __attribute__((aligned(16))) __bf16 Ws[2][3][CO * LDB];
  const int KK = d.KH * d.KW;
  const int Kc = d.C * KK;
  const int G = Kc / 4;
  for (int g = threadIdx.x; g < G; g += 256) ta[g] = kgroup_offset<U8>(d, g);
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const int li = lane & 31, lg = lane >> 5;
  const int P = d.OH * d.OW;
  const int64_t M = (int64_t)d.B * P;
  const int64_t m0 = ((int64_t)blockIdx.x * 4 + w) * 32;
  const int64_t m = m0 + li;
  const bool valid = m < M;
  int64_t org = 0;
  if (valid) {
    const int64_t b = m / P;
    const int p = (int)(m - b * P);
    const int oy = p / d.OW, ox = p - oy * d.OW;
    org = window_origin<U8>(d, b, oy, ox);
  }
  // weight chunk: CO x 32 walk-ordered values, WN x 4 per thread (co = e >> 5,
  // kk = e & 31), read from [CO][C][KH][KW]
  float wv[4 * WN];
  auto wload = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 4 * WN; ++j) {
      const int e = t + 256 * j, co = e >> 5, kk = e & 31;
      const int k = k0 + kk;
      float v = 0.f;
      if (k < Kc) {
        int src = k;  // (c, kh, kw) order for uint8 input = the native layout
        if (!U8 && !PACKED) {
          const int c = k % d.C, tt = k / d.C, kw = tt % d.KW, kh = tt / d.KW;
          src = (c * d.KH + kh) * d.KW + kw;
        }
        v = (PACKED ? d.wpack : d.weight)[(int64_t)co * Kc + src];
      }
      wv[j] = v;
    }
  };
  auto wstore = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 4 * WN; ++j) {
      const int e = t + 256 * j, co = e >> 5, kk = e & 31;
      __bf16 q0, q1, q2;
      split1(wv[j], q0, q1, q2);
      Ws[buf][0][co * LDB + kk] = q0;
      Ws[buf][1][co * LDB + kk] = q1;
      Ws[buf][2][co * LDB + kk] = q2;
    }
  };
  // the A operand of a chunk: per k step s, this lane's 8 k (16 s + 8 lg ..),
  // two k groups; raw (uint32 bytes or float4) one chunk ahead
  uint32_t ru[2][2];
  float4 rf[2][2];
  auto aload = [&](int k0) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int g = (k0 + 16 * s + 8 * lg) / 4 + h;
        if (U8) {
          uint32_t x = 0u;
          if (valid && g < G) {
            const uint8_t* sp = d.x_u8 + org + ta[g];
            if (ALIGNED) x = *reinterpret_cast<const uint32_t*>(sp);
            else x = (uint32_t)sp[0] | ((uint32_t)sp[1] << 8) | ((uint32_t)sp[2] << 16) | ((uint32_t)sp[3] << 24);
          }
          ru[s][h] = x;
        } else {
          rf[s][h] = (valid && g < G) ? *reinterpret_cast<const float4*>(d.x_f32 + org + ta[g])
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
  };
  f32x16 acc[WN];
#pragma unroll
  for (int j = 0; j < WN; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  wload(0);
  wstore(0);
  __syncthreads();  // also publishes the offset table
  aload(0);
  int cur = 0;
  for (int k0 = 0; k0 < Kc; k0 += BK) {
    const bool more = k0 + BK < Kc;
    if (more) wload(k0 + BK);
    uint32_t cu[2][2];
    float4 cf[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        cu[s][h] = ru[s][h];
        cf[s][h] = rf[s][h];
      }
    if (more) aload(k0 + BK);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 a[3];
      if (U8) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < 4; ++i) a[0][4 * h + i] = (__bf16)(float)((cu[s][h] >> (8 * i)) & 255u);
      } else {
        const float v[8] = {cf[s][0].x, cf[s][0].y, cf[s][0].z, cf[s][0].w,
                            cf[s][1].x, cf[s][1].y, cf[s][1].z, cf[s][1].w};
        split8(v, a);
      }
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        bf16x8 bq[3];
#pragma unroll
        for (int q = 0; q < 3; ++q)
          bq[q] = *reinterpret_cast<const bf16x8*>(&Ws[cur][q][(32 * j + li) * LDB + 16 * s + 8 * lg]);
        if (U8) {
          // the byte is exact in one part: three products, smallest first
          acc[j] = mfma16(a[0], bq[2], acc[j]);
          acc[j] = mfma16(a[0], bq[1], acc[j]);
          acc[j] = mfma16(a[0], bq[0], acc[j]);
        } else {
          acc[j] = prod6(a, bq, acc[j]);
        }
      }
    }
    if (more) wstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  if (m0 >= M) return;
  // epilogue: acc[j][r] -> row m0 + (r&3) + 8*(r>>2) + 4*lg, channel 32*j + li
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    const int n = 32 * j + li;
    const float bn = d.bias ? d.bias[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t mm = m0 + (r & 3) + 8 * (r >> 2) + 4 * lg;
      if (mm < M) {
        float v = (U8 ? __fdiv_rn(acc[j][r], 255.f) : acc[j][r]) + bn;
        if (d.relu) v = fmaxf(v, 0.f);
        d.y[mm * CO + n] = v;
      }
    }
  }
}

// row -> (b, oy, ox) cursor that advances one row at a time
struct RowCursor {
  int64_t b;
  int oy, ox;
  __device__ __forceinline__ void set(int64_t row, int P, int OW) {
    b = row / P;
    const int p = (int)(row - b * P);
    oy = p / OW;
    ox = p - oy * OW;
  }
  __device__ __forceinline__ void next(int OH, int OW) {
    if (++ox == OW) {
      ox = 0;
      if (++oy == OH) { oy = 0; ++b; }
    }
  }
};

template <int WNK, int KWV, bool U8>
__global__ __launch_bounds__(64 * KWV) void conv_bwd_w_kernel(d3a_conv_desc d) {
  __shared__ float red[(KWV - 1) * WNK * 16 * 64];
  __shared__ double rsum[KWV * 32];
  constexpr int U = 2;  // 8-row steps loaded before any is multiplied
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 31, lg = lane >> 5;
  const int KK = d.KH * d.KW;
  const int Kc = d.C * KK;
  const int P = d.OH * d.OW;
  const int64_t M = (int64_t)d.B * P;
  const int k0 = blockIdx.x * 32 * WNK;
  const int co0 = blockIdx.y * 32;
  const int s = blockIdx.z;
  // split s: rows [sb, se); wave w: a multiple-of-8 sub-slice
  const int64_t chunk = (M + d.splits - 1) / d.splits;
  const int64_t sb = s * chunk;
  const int64_t se = sb + chunk < M ? sb + chunk : M;
  int64_t wch = (se - sb + KWV - 1) / KWV;
  wch = (wch + 7) / 8 * 8;
  const int64_t rb = sb + w * wch;
  const int64_t re = rb + wch < se ? rb + wch : se;
  const bool do_bias = d.db != nullptr && blockIdx.x == 0;

  // this lane's k columns (walk order) -> input offset and output column
  int koff[WNK], kout[WNK];
  bool kok[WNK];
#pragma unroll
  for (int j = 0; j < WNK; ++j) {
    const int k = k0 + 32 * j + li;
    kok[j] = k < Kc;
    const int kk = kok[j] ? k : 0;
    if (U8) {
      const int c = kk / KK, r = kk - c * KK, kh = r / d.KW, kw = r - kh * d.KW;
      koff[j] = (c * d.H + kh) * d.W + kw;
      kout[j] = kk;
    } else {
      const int c = kk % d.C, t = kk / d.C, kw = t % d.KW, kh = t / d.KW;
      koff[j] = (kh * d.W + kw) * d.C + c;
      kout[j] = c * KK + kh * d.KW + kw;
    }
  }

  f32x16 acc[WNK];
#pragma unroll
  for (int j = 0; j < WNK; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  double bs = 0.0;

  RowCursor cur;
  if (rb < re) cur.set(rb + 4 * lg, P, d.OW);
  for (int64_t r0 = rb; r0 < re; r0 += 8 * U) {
    float ra[U][4], rv[U][WNK][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      RowCursor c = cur;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t row = r0 + 8 * u + 4 * lg + q;
        const bool ok = row < re;
        ra[u][q] = ok ? d.dy[row * d.CO + co0 + li] : 0.f;
        const int64_t org = window_origin<U8>(d, c.b, c.oy, c.ox);
#pragma unroll
        for (int j = 0; j < WNK; ++j) {
          float v = 0.f;
          if (ok && kok[j]) v = U8 ? px(d.x_u8[org + koff[j]]) : d.x_f32[org + koff[j]];
          rv[u][j][q] = v;
        }
        c.next(d.OH, d.OW);
      }
      // advance the cursor by 8 rows (4 consumed above + 4 of the other lane group)
#pragma unroll
      for (int q = 0; q < 4; ++q) c.next(d.OH, d.OW);
      cur = c;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (do_bias) bs += (double)ra[u][0] + (double)ra[u][1] + (double)ra[u][2] + (double)ra[u][3];
#pragma unroll
      for (int j = 0; j < WNK; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[u][q], rv[u][j][q], acc[j], 0, 0, 0);
    }
  }

  if (w > 0) {
#pragma unroll
    for (int j = 0; j < WNK; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(((w - 1) * WNK + j) * 16 + r) * 64 + lane] = acc[j][r];
  }
  if (do_bias) {
    bs += __shfl_xor(bs, 32, 64);
    if (lg == 0) rsum[w * 32 + li] = bs;
  }
  __syncthreads();
  if (w != 0) return;
#pragma unroll
  for (int v = 1; v < KWV; ++v)
#pragma unroll
    for (int j = 0; j < WNK; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] += red[(((v - 1) * WNK + j) * 16 + r) * 64 + lane];
  float* dW = d.dW + (int64_t)s * d.CO * Kc;
#pragma unroll
  for (int j = 0; j < WNK; ++j) {
    if (!kok[j]) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + (r & 3) + 8 * (r >> 2) + 4 * lg;
      dW[(int64_t)co * Kc + kout[j]] = acc[j][r];
    }
  }
  if (do_bias && lg == 0) {
    double tot = 0.0;
    for (int v = 0; v < KWV; ++v) tot += rsum[v * 32 + li];
    d.db[(int64_t)s * d.CO + co0 + li] = (float)tot;
  }
}

// Weight gradient on the bf16 matrix cores at fp32 accuracy (x6.hpp):
// dW[co][k] = sum_rows dy[row][co] col(row, k) as v_mfma_f32_32x32x16_bf16
// over 16-row steps (M = co, N = k, K = rows).  Lane (li, lg) holds rows
// 8 lg .. 8 lg + 7 of a step: dy[row][co0 + li] (A, three exact bf16 parts)
// and col(row, k0 + 32 j + li) (B: an fp32 activation in three parts, six
// products; a uint8 byte exact in one part, three products, the pixel scale
// applied to the sum as in conv_fwd_x6_kernel).  A wave owns 32 co x 32 NK k
// over a row sub-slice, the next step's operands loaded while the current one
// multiplies; the 8 waves of a workgroup are summed by a fixed tree through
// LDS and the split's partial goes to dW[split] (summed in order by Adam).
template <int NK, bool U8>
__global__ __launch_bounds__(512) void conv_bwd_w_x6_kernel(d3a_conv_desc d) {
  using namespace x6;
  constexpr int NW = 8;
  __shared__ float red[4 * NK * 16 * 64];
  __shared__ double rsum[NW * 32];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 31, lg = lane >> 5;
  const int KK = d.KH * d.KW;
  const int Kc = d.C * KK;
  const int P = d.OH * d.OW;
  const int64_t M = (int64_t)d.B * P;
  const int k0 = blockIdx.x * 32 * NK;
  const int co0 = blockIdx.y * 32;
  const int s = blockIdx.z;
  const int64_t chunk = (M + d.splits - 1) / d.splits;
  const int64_t sb = s * chunk;
  const int64_t se = sb + chunk < M ? sb + chunk : M;
  int64_t wch = (se - sb + NW - 1) / NW;
  wch = (wch + 15) / 16 * 16;
  const int64_t rb = sb + w * wch;
  const int64_t re = rb + wch < se ? rb + wch : se;
  const bool do_bias = d.db != nullptr && blockIdx.x == 0;

  int koff[NK], kout[NK];
  bool kok[NK];
#pragma unroll
  for (int j = 0; j < NK; ++j) {
    const int k = k0 + 32 * j + li;
    kok[j] = k < Kc;
    const int kk = kok[j] ? k : 0;
    if (U8) {
      const int c = kk / KK, r = kk - c * KK, kh = r / d.KW, kw = r - kh * d.KW;
      koff[j] = (c * d.H + kh) * d.W + kw;
      kout[j] = kk;
    } else {
      const int c = kk % d.C, t = kk / d.C, kw = t % d.KW, kh = t / d.KW;
      koff[j] = (kh * d.W + kw) * d.C + c;
      kout[j] = c * KK + kh * d.KW + kw;
    }
  }

  f32x16 acc[NK];
#pragma unroll
  for (int j = 0; j < NK; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  double bs = 0.0;

  // this lane's 8 rows of a step: r0 + 8 lg + i
  float ny[8], nx[NK][8];
  RowCursor cur;
  if (rb < re) cur.set(rb + 8 * lg, P, d.OW);
  auto load = [&](int64_t r0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t row = r0 + 8 * lg + i;
      const bool ok = row < re;
      ny[i] = ok ? d.dy[row * d.CO + co0 + li] : 0.f;
      const int64_t org = window_origin<U8>(d, cur.b, cur.oy, cur.ox);
#pragma unroll
      for (int j = 0; j < NK; ++j) {
        float v = 0.f;
        if (ok && kok[j]) v = U8 ? (float)d.x_u8[org + koff[j]] : d.x_f32[org + koff[j]];
        nx[j][i] = v;
      }
      cur.next(d.OH, d.OW);
    }
    // skip the other lane group's 8 rows
#pragma unroll
    for (int i = 0; i < 8; ++i) cur.next(d.OH, d.OW);
  };
  if (rb < re) load(rb);
  for (int64_t r0 = rb; r0 < re; r0 += 16) {
    float cy[8], cx[NK][8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      cy[i] = ny[i];
#pragma unroll
      for (int j = 0; j < NK; ++j) cx[j][i] = nx[j][i];
    }
    if (r0 + 16 < re) load(r0 + 16);
    if (do_bias) {
#pragma unroll
      for (int i = 0; i < 8; ++i) bs += (double)cy[i];
    }
    bf16x8 a[3];
    split8(cy, a);
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      if (U8) {
        bf16x8 b;
#pragma unroll
        for (int i = 0; i < 8; ++i) b[i] = (__bf16)cx[j][i];
        // the byte is exact in one part: three products, smallest first
        acc[j] = mfma16(a[2], b, acc[j]);
        acc[j] = mfma16(a[1], b, acc[j]);
        acc[j] = mfma16(a[0], b, acc[j]);
      } else {
        bf16x8 b[3];
        split8(cx[j], b);
        acc[j] = prod6(a, b, acc[j]);
      }
    }
  }

  // fixed-order tree over the 8 waves: (w, w + 4), then (w, w + 2), then (0, 1)
#pragma unroll
  for (int half = 4; half >= 1; half >>= 1) {
    if (w >= half && w < 2 * half) {
#pragma unroll
      for (int j = 0; j < NK; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) red[(((w - half) * NK + j) * 16 + r) * 64 + lane] = acc[j][r];
    }
    __syncthreads();
    if (w < half) {
#pragma unroll
      for (int j = 0; j < NK; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] += red[((w * NK + j) * 16 + r) * 64 + lane];
    }
    __syncthreads();
  }
  if (do_bias) {
    bs += __shfl_xor(bs, 32, 64);
    if (lg == 0) rsum[w * 32 + li] = bs;
  }
  __syncthreads();
  if (w != 0) return;
  float* dW = d.dW + (int64_t)s * d.CO * Kc;
#pragma unroll
  for (int j = 0; j < NK; ++j) {
    if (!kok[j]) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + (r & 3) + 8 * (r >> 2) + 4 * lg;
      dW[(int64_t)co * Kc + kout[j]] = U8 ? __fdiv_rn(acc[j][r], 255.f) : acc[j][r];
    }
  }
  if (do_bias && lg == 0) {
    double tot = 0.0;
    for (int v = 0; v < NW; ++v) tot += rsum[v * 32 + li];
    d.db[(int64_t)s * d.CO + co0 + li] = (float)tot;
  }
}

// The uint8 stride-4, 8-wide first layer (Nature DQN conv1) weight gradient:
// the generic kernels above gather one byte per lane and row, 52 MB of single-
// byte loads at K5's shape (122 us).  Here the GEMM's K (rows) is walked in
// runs of 4 consecutive output columns ox = 4 q .. 4 q + 3 of one (b, oy):
// for a tap (c, kh, kw = 4 j + dx) their pixels x[b][c][4 oy + kh][16 q + 4 j
// + 4 u + dx], u = 0..3, are byte dx of the 4 dwords at 16 q + 4 j.  The 4
// lanes of a quad (dx = 0..3, one (c, kh, j)) load one dword each (u = dx)
// and transpose the 4 x 4 bytes with two DPP exchanges + v_perm, so lane dx
// ends with its 4 pixels.  A 16-row MFMA step is four runs; lane (li, lg)
// holds runs 2 lg, 2 lg + 1 (its 8 k slots): B = the pixels of k = 32 t + li
// (k-tile t; kout order c KH KW + kh KW + kw, 4 (c, kh) pairs x 8 kw per
// tile), exact in one bf16 part; A = dy[row][co0 + li] in three parts: three
// products, the pixel scale applied to the sum (as conv_bwd_w_x6_kernel).  A
// wave keeps all NKT k-tiles (Kc = 32 NKT <= 256): dy is read once; the
// k-tiles' loads are double-buffered in halves.  Waves take K-steps w, w + 8,
// .. of their workgroup's chunk; the 8 waves meet in a fixed-order LDS tree,
// the split's partial goes to dW[split].
template <int NKT>
__global__ __launch_bounds__(512) void conv1_bwd_w_u8s4_kernel(d3a_conv_desc d) {
  using namespace x6;
  constexpr int NW = 8, HK = NKT / 2;  // k-tiles per half
  __shared__ float red[4 * HK * 16 * 64];
  __shared__ double rsum[NW * 32];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 31, lg = lane >> 5;
  const int QW = d.OW / 4;
  const int64_t NR = (int64_t)d.B * d.OH * QW;  // runs
  const int64_t NKS = (NR + 3) / 4;             // 16-row steps
  const int co0 = blockIdx.y * 32;
  const int s = blockIdx.z;
  const int64_t chunk = (NKS + d.splits - 1) / d.splits;
  const int64_t kb = s * chunk;
  const int64_t ke = kb + chunk < NKS ? kb + chunk : NKS;
  const bool do_bias = d.db != nullptr;
  const int64_t plane = (int64_t)d.H * d.W;
  // this lane's tap in k-tile t: pair 4 t + (li >> 3) = (c, kh), kw = li & 7
  // = 4 j + dx; it loads dword u = dx of the tap's 16 bytes
  const int dx = li & 3;
  int toff[NKT];
#pragma unroll
  for (int t = 0; t < NKT; ++t) {
    const int pr = 4 * t + (li >> 3), c = pr / d.KH, kh = pr - c * d.KH;
    toff[t] = (int)(c * plane + (int64_t)kh * d.W) + 4 * ((li & 7) >> 2) + 4 * dx;
  }
  // quad byte transpose selectors (own dword = bytes 0-3, the partner's 4-7)
  const uint32_t sel1 = (dx & 1) ? 0x03070105u : 0x06020400u;  // with lane ^ 1
  const uint32_t sel2 = (dx & 2) ? 0x03020706u : 0x05040100u;  // with lane ^ 2

  f32x16 acc[NKT];
#pragma unroll
  for (int t = 0; t < NKT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  double bs = 0.0;

  // a step's two runs for this lane half: image base offsets and dy rows
  struct Runs {
    int64_t xo[2], row[2];
    bool ok[2];
  };
  auto runs_of = [&](int64_t ks) {
    Runs R;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t rho = 4 * ks + 2 * lg + h;
      R.ok[h] = rho < NR;
      const int64_t rr = R.ok[h] ? rho : 0;
      const int64_t line = rr / QW;
      const int q = (int)(rr - line * QW);
      const int64_t b = line / d.OH;
      const int oy = (int)(line - b * d.OH);
      R.xo[h] = b * d.C * plane + (int64_t)(4 * oy) * d.W + 16 * q;
      R.row[h] = line * d.OW + 4 * q;
    }
    return R;
  };
  uint32_t xa[HK][2], xb[HK][2];  // [k-tile of the half][run]
  float dyv[8];
  auto load_half = [&](const Runs& R, int half, uint32_t (*xv)[2]) {
#pragma unroll
    for (int t = 0; t < HK; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        xv[t][h] = R.ok[h] ? *reinterpret_cast<const uint32_t*>(d.x_u8 + R.xo[h] + toff[half * HK + t])
                           : 0u;
  };
  auto load_dy = [&](const Runs& R) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int u = 0; u < 4; ++u) dyv[4 * h + u] = R.ok[h] ? d.dy[(R.row[h] + u) * d.CO + co0 + li] : 0.f;
  };
  auto mul_half = [&](const bf16x8* a, uint32_t (*xv)[2], int half) {
#pragma unroll
    for (int t = 0; t < HK; ++t) {
      bf16x8 b;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        // 4 x 4 byte transpose across the quad: byte u of the result = dword u's byte dx
        const uint32_t v = xv[t][h];
        const uint32_t p1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
        const uint32_t t1 = __builtin_amdgcn_perm(p1, v, sel1);
        const uint32_t p2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)t1, 0x4E, 0xF, 0xF, false);
        const uint32_t px = __builtin_amdgcn_perm(p2, t1, sel2);
#pragma unroll
        for (int u = 0; u < 4; ++u) b[4 * h + u] = (__bf16)(float)((px >> (8 * u)) & 0xffu);
      }
      f32x16& c = acc[half * HK + t];
      c = mfma16(a[2], b, c);
      c = mfma16(a[1], b, c);
      c = mfma16(a[0], b, c);
    }
  };

  int64_t ks = kb + w;
  if (ks < ke) {
    const Runs R = runs_of(ks);
    load_dy(R);
    load_half(R, 0, xa);
    load_half(R, 1, xb);
  }
  for (; ks < ke; ks += NW) {
    const bool more = ks + NW < ke;
    const Runs Rn = runs_of(more ? ks + NW : ks);
    bf16x8 a[3];
    split8(dyv, a);
    if (do_bias) {
#pragma unroll
      for (int i = 0; i < 8; ++i) bs += (double)dyv[i];
    }
    __builtin_amdgcn_sched_barrier(0);
    mul_half(a, xa, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (more) {
      load_dy(Rn);
      load_half(Rn, 0, xa);
    }
    __builtin_amdgcn_sched_barrier(0);
    mul_half(a, xb, 1);
    __builtin_amdgcn_sched_barrier(0);
    if (more) load_half(Rn, 1, xb);
  }

  // fixed-order tree over the 8 waves per half of the k-tiles: (w, w + 4),
  // then (w, w + 2), then (0, 1)
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int m = 4; m >= 1; m >>= 1) {
      if (w >= m && w < 2 * m) {
#pragma unroll
        for (int t = 0; t < HK; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) red[(((w - m) * HK + t) * 16 + r) * 64 + lane] = acc[half * HK + t][r];
      }
      __syncthreads();
      if (w < m) {
#pragma unroll
        for (int t = 0; t < HK; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[half * HK + t][r] += red[((w * HK + t) * 16 + r) * 64 + lane];
      }
      __syncthreads();
    }
  }
  if (do_bias) {
    bs += __shfl_xor(bs, 32, 64);
    if (lg == 0) rsum[w * 32 + li] = bs;
  }
  __syncthreads();
  if (w != 0) return;
  const int Kc = 32 * NKT;
  float* dW = d.dW + (int64_t)s * d.CO * Kc;
#pragma unroll
  for (int t = 0; t < NKT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + (r & 3) + 8 * (r >> 2) + 4 * lg;
      dW[(int64_t)co * Kc + 32 * t + li] = __fdiv_rn(acc[t][r], 255.f);
    }
  if (do_bias && lg == 0) {
    double tot = 0.0;
    for (int v = 0; v < NW; ++v) tot += rsum[v * 32 + li];
    d.db[(int64_t)s * d.CO + co0 + li] = (float)tot;
  }
}

// the first-layer fast path's geometry: uint8 input, stride 4, 8-wide
// kernel (two 4-byte column groups), whole 4-column runs, Kc = C KH 8 a
// multiple of 64 up to 256
inline bool conv1_u8s4_ok(const d3a_conv_desc* d) {
  const int64_t Kc = (int64_t)d->C * d->KH * d->KW;
  return d->x_u8 != nullptr && d->S == 4 && d->KW == 8 && d->OW % 4 == 0 && d->W % 4 == 0 &&
         (reinterpret_cast<uintptr_t>(d->x_u8) & 3) == 0 && Kc % 64 == 0 && Kc <= 256 &&
         d->CO % 32 == 0 && (int64_t)d->C * d->H * d->W < (int64_t)1 << 31;
}

// Input gradient on the bf16 matrix cores at fp32 accuracy: dx[b][y][x][c] =
// [x > 0] sum over the output positions (oy, ox) whose window covers (y, x) of
// sum_co dy[b][oy][ox][co] W[co][c][y - S oy][x - S ox] -- im2col's transpose
// (col2im of dy W) as one implicit GEMM, no column matrix in HBM.  Rows are
// walked per stride phase (py, px) = (y % S, x % S): every row of a phase
// takes the same taps kh = py + S ih, kw = px + S iw, at oy = y / S - ih,
// ox = x / S - iw, so a workgroup's weight chunk is shared by its 128 rows
// (M = phase rows, N = c, K = (ih, iw, co), a missing position a zero
// operand).  dy is read as float4 runs of 8 co (CO % 16 == 0); the weight is
// staged per 32-k chunk in three bf16 parts, six products.
// weight [CO][C][KH][KW] -> [KH][KW][CO][C] (d3a_conv_bwd_x's chunk order: a
// 32-k chunk, one tap x 32 co x all c, is one contiguous run)
__global__ __launch_bounds__(256) void conv_pack_tap_kernel(const float* __restrict__ w,
                                                            float* __restrict__ wt, int CO, int C,
                                                            int KH, int KW) {
  const int64_t n = (int64_t)CO * C * KH * KW;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int kw = (int)(i % KW);
  int64_t r = i / KW;
  const int kh = (int)(r % KH);
  r /= KH;
  const int c = (int)(r % C);
  const int co = (int)(r / C);
  wt[(((int64_t)kh * KW + kw) * CO + co) * C + c] = w[i];
}

// F32: the products on v_mfma_f32_32x32x2_f32 instead (exact fp32 products,
// fp32 accumulation: the column-matrix GEMM's arithmetic), the weight chunk
// kept in fp32 in LDS -- the kernel is bound by its loads, not the matrix cores
// several layers' weight copies in one launch (d3a_conv_pack_weights)
struct PackJobs {
  const float* w[8];
  float* dst[8];
  int CO[8], C[8], KH[8], KW[8], layout[8];
  int64_t end[8];  // running element count through job i
  int n;
  // (d3a_conv_pack_weights_philox) a Philox fill on the blocks past the
  // copies' (pk_blocks of them): d3a_philox_fill's body and counter ticket
  d3a_philox_job ph;
  int pk_blocks;
};

__global__ __launch_bounds__(256) void conv_pack_multi_kernel(PackJobs J) {
  if ((int)blockIdx.x >= J.pk_blocks) {
    const int64_t total = J.ph.n_normal + J.ph.n_uniform;
    const int64_t nwp = (int64_t)gridDim.x - J.pk_blocks;
    const int64_t wgi = (int64_t)blockIdx.x - J.pk_blocks;
    const int64_t step = *J.ph.ctr;
    const int64_t e0 = (wgi * 256 + threadIdx.x) * 4;
    if (e0 < total) {
      for (int q = 0; q < 4; ++q) {
        const int64_t e = e0 + q;
        if (e < total)
          J.ph.out[e] = philox_elem(J.ph.seed, (uint64_t)step, e, J.ph.n_normal, J.ph.lo, J.ph.hi);
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned prev = atomicAdd(J.ph.ticket, 1u);
      if (prev == (unsigned)(nwp - 1)) {
        *J.ph.ctr = step + 1;
        *J.ph.ticket = 0u;
      }
    }
    return;
  }
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int j = 0;
  while (j < J.n && g >= J.end[j]) ++j;
  if (j >= J.n) return;
  const int64_t i = g - (j > 0 ? J.end[j - 1] : 0);  // source index in [CO][C][KH][KW]
  const int KW = J.KW[j], KH = J.KH[j], C = J.C[j], CO = J.CO[j];
  const int kw = (int)(i % KW);
  int64_t r = i / KW;
  const int kh = (int)(r % KH);
  r /= KH;
  const int c = (int)(r % C);
  const int co = (int)(r / C);
  const int64_t o = J.layout[j] == 0 ? (((int64_t)co * KH + kh) * KW + kw) * C + c
                                     : (((int64_t)kh * KW + kw) * CO + co) * C + c;
  J.dst[j][o] = J.w[j][i];
}

template <int WN, bool PACKED, bool F32 = false>
__global__ __launch_bounds__(256) void conv_bwd_x_x6_kernel(d3a_conv_desc d) {
  using namespace x6;
  constexpr int C = 32 * WN, BK = 32, LDB = BK + 8, LDF = BK + 4;
  __shared__ __attribute__((aligned(16))) __bf16 Ws[F32 ? 1 : 2][3][F32 ? 8 : C * LDB];
  __shared__ __attribute__((aligned(16))) float Wf[F32 ? 2 : 1][F32 ? C * LDF : 4];
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const int li = lane & 31, lg = lane >> 5;
  const int S = d.S, CO = d.CO;
  const int py = blockIdx.y / S, px = blockIdx.y - py * S;
  const int nyp = (d.H - py + S - 1) / S, nxp = (d.W - px + S - 1) / S;
  const int NTH = (d.KH - py + S - 1) / S, NTW = (d.KW - px + S - 1) / S;
  const int Kc = NTH * NTW * CO;
  const int64_t Mp = (int64_t)d.B * nyp * nxp;
  if ((int64_t)blockIdx.x * 128 >= Mp) return;  // whole workgroup, before any barrier
  const int64_t m0 = ((int64_t)blockIdx.x * 4 + w) * 32;
  const int64_t m = m0 + li;
  const bool valid = m < Mp;
  int64_t bimg = 0;
  int yi = 0, xi = 0;
  if (valid) {
    bimg = m / (nyp * nxp);
    const int r = (int)(m - bimg * nyp * nxp);
    yi = r / nxp;
    xi = r - yi * nxp;
  }
  const float* dyb = d.dy + bimg * d.OH * d.OW * CO;
  // weight chunk: C x 32 values, WN x 4 per thread: packed, one contiguous run
  // of [32 co][C] (co = e / C, c = e % C); else gathered from nn.Conv2d's
  // layout (c = e >> 5, kk = e & 31)
  float wv[4 * WN];
  auto wload = [&](int k0) {
    if constexpr (PACKED) {
      const int tap = k0 / CO, co0 = k0 - tap * CO;
      const int ih = tap / NTW, iw = tap - ih * NTW;
      const int kh = py + S * ih, kw = px + S * iw;
      const float* src = d.wpack + (((int64_t)kh * d.KW + kw) * CO + co0) * C;
#pragma unroll
      for (int j = 0; j < 4 * WN; ++j) wv[j] = k0 < Kc ? src[t + 256 * j] : 0.f;
      return;
    }
#pragma unroll
    for (int j = 0; j < 4 * WN; ++j) {
      const int e = t + 256 * j, c = e >> 5, kk = e & 31;
      const int k = k0 + kk;
      float v = 0.f;
      if (k < Kc) {
        const int tap = k / CO, co = k - tap * CO;
        const int ih = tap / NTW, iw = tap - ih * NTW;
        const int kh = py + S * ih, kw = px + S * iw;
        v = d.weight[(((int64_t)co * d.C + c) * d.KH + kh) * d.KW + kw];
      }
      wv[j] = v;
    }
  };
  auto wstore = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 4 * WN; ++j) {
      const int e = t + 256 * j;
      const int c = PACKED ? e % C : e >> 5, kk = PACKED ? e / C : e & 31;
      if constexpr (F32) {
        Wf[buf][c * LDF + kk] = wv[j];
      } else {
        __bf16 q0, q1, q2;
        split1(wv[j], q0, q1, q2);
        Ws[buf][0][c * LDB + kk] = q0;
        Ws[buf][1][c * LDB + kk] = q1;
        Ws[buf][2][c * LDB + kk] = q2;
      }
    }
  };
  // the A operand of a chunk: per k step s, this lane's 8 k = 8 co of one tap
  float4 rf[2][2];
  auto aload = [&](int k0) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int k = k0 + 16 * s2 + 8 * lg;
      float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0;
      if (valid && k < Kc) {
        const int tap = k / CO, co = k - tap * CO;
        const int ih = tap / NTW, iw = tap - ih * NTW;
        const int oy = yi - ih, ox = xi - iw;
        if (oy >= 0 && oy < d.OH && ox >= 0 && ox < d.OW) {
          const float4* src = reinterpret_cast<const float4*>(dyb + ((int64_t)oy * d.OW + ox) * CO + co);
          v0 = src[0];
          v1 = src[1];
        }
      }
      rf[s2][0] = v0;
      rf[s2][1] = v1;
    }
  };
  f32x16 acc[WN];
#pragma unroll
  for (int j = 0; j < WN; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  wload(0);
  wstore(0);
  __syncthreads();
  aload(0);
  int cur = 0;
  for (int k0 = 0; k0 < Kc; k0 += BK) {
    const bool more = k0 + BK < Kc;
    if (more) wload(k0 + BK);
    float4 cf[2][2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      cf[s2][0] = rf[s2][0];
      cf[s2][1] = rf[s2][1];
    }
    if (more) aload(k0 + BK);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const float v[8] = {cf[s2][0].x, cf[s2][0].y, cf[s2][0].z, cf[s2][0].w,
                          cf[s2][1].x, cf[s2][1].y, cf[s2][1].z, cf[s2][1].w};
      if constexpr (F32) {
        // MFMA i covers k = 16 s2 + i (lane group 0) and 16 s2 + 8 + i (group 1)
#pragma unroll
        for (int j = 0; j < WN; ++j) {
          const float* wr = &Wf[cur][(32 * j + li) * LDF + 16 * s2 + 8 * lg];
          const float4 w0 = *reinterpret_cast<const float4*>(wr);
          const float4 w1 = *reinterpret_cast<const float4*>(wr + 4);
          const float wk[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
          for (int i = 0; i < 8; ++i)
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(v[i], wk[i], acc[j], 0, 0, 0);
        }
        continue;
      }
      bf16x8 a[3];
      split8(v, a);
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        bf16x8 bq[3];
#pragma unroll
        for (int q = 0; q < 3; ++q)
          bq[q] = *reinterpret_cast<const bf16x8*>(&Ws[cur][q][(32 * j + li) * LDB + 16 * s2 + 8 * lg]);
        acc[j] = prod6(a, bq, acc[j]);
      }
    }
    if (more) wstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  if (m0 >= Mp) return;
  // epilogue: acc[j][r] -> phase row m0 + (r&3) + 8*(r>>2) + 4*lg, channel 32*j + li
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t mm = m0 + (r & 3) + 8 * (r >> 2) + 4 * lg;
    if (mm >= Mp) continue;
    const int64_t bb = mm / (nyp * nxp);
    const int rr = (int)(mm - bb * nyp * nxp);
    const int yy = py + S * (rr / nxp), xx = px + S * (rr - (rr / nxp) * nxp);
    const int64_t o = ((bb * d.H + yy) * d.W + xx) * C;
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int n = 32 * j + li;
      float v = acc[j][r];
      if (d.relu && !(d.x_f32[o + n] > 0.f)) v = 0.f;
      d.y[o + n] = v;
    }
  }
}

int check_geometry(const d3a_conv_desc* d, const char* name) {
  D3A_CHECK_ARG(d != nullptr, "%s: null descriptor", name);
  D3A_CHECK_ARG((d->x_u8 != nullptr) != (d->x_f32 != nullptr),
                "%s: exactly one of x_u8 / x_f32 must be set", name);
  D3A_CHECK_ARG(d->weight, "%s: null weight", name);
  D3A_CHECK_ARG(d->B >= 0 && d->C >= 1 && d->KH >= 1 && d->KW >= 1 && d->S >= 1 &&
                    d->H >= d->KH && d->W >= d->KW,
                "%s: bad geometry", name);
  D3A_CHECK_ARG(d->OH == (d->H - d->KH) / d->S + 1 && d->OW == (d->W - d->KW) / d->S + 1,
                "%s: inconsistent output size", name);
  D3A_CHECK_ARG(d->CO == 32 || d->CO == 64, "%s: CO must be 32 or 64", name);
  const int64_t Kc = (int64_t)d->C * d->KH * d->KW;
  D3A_CHECK_ARG(Kc % 4 == 0 && Kc / 4 <= kMaxKGroups, "%s: C*KH*KW must be a multiple of 4, <= 4096",
                name);
  if (d->x_u8) D3A_CHECK_ARG(d->KW % 4 == 0, "%s: uint8 input needs KW %% 4 == 0", name);
  else D3A_CHECK_ARG(d->C % 4 == 0, "%s: fp32 NHWC input needs C %% 4 == 0", name);
  return 0;
}

}  // namespace
}  // namespace d3a

namespace d3a {
namespace {
// the split-bf16 forward of an fp32-input layer reads a walk-ordered copy of
// the weight (one conv_pack launch: coalesced chunk loads instead of 32
// scattered channels) unless D3A_CONV_FWD_PACK=0 (K5 768 -> 803 steps/s)
bool conv_fwd_pack() {
  static const bool on = [] {
    const char* e = getenv("D3A_CONV_FWD_PACK");
    return !(e && atoi(e) == 0);
  }();
  return on;
}
}  // namespace
}  // namespace d3a

extern "C" int d3a_conv_fwd(const d3a_conv_desc* d, void* stream) {
  using namespace d3a;
  if (check_geometry(d, "d3a_conv_fwd")) return -1;
  D3A_CHECK_ARG(d->y, "d3a_conv_fwd: null output");
  D3A_CHECK_ARG(d->x_u8 || d->wpack, "d3a_conv_fwd: fp32 input needs the wpack scratch");
  const int64_t M = (int64_t)d->B * d->OH * d->OW;
  if (M == 0) return 0;
  const int64_t blocks = (M + 127) / 128;
  D3A_CHECK_ARG(blocks < (1ll << 31), "d3a_conv_fwd: too many rows");
  D3A_CHECK_ARG((reinterpret_cast<uintptr_t>(d->weight) & 15) == 0,
                "d3a_conv_fwd: weight must be 16-byte aligned");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)blocks), block(256);
  // split-bf16 (fp32-accurate) implicit GEMM unless D3A_CONV_X6=0
  static const bool use_x6 = [] {
    const char* e = getenv("D3A_CONV_X6");
    return !(e && atoi(e) == 0);
  }();
  if (use_x6) {
    if (d->x_u8) {
      const bool al = d->W % 4 == 0 && d->S % 4 == 0 && (reinterpret_cast<uintptr_t>(d->x_u8) & 3) == 0;
      if (d->CO == 32 && al) hipLaunchKernelGGL((conv_fwd_x6_kernel<1, true, true>), grid, block, 0, st, *d);
      else if (d->CO == 32) hipLaunchKernelGGL((conv_fwd_x6_kernel<1, true>), grid, block, 0, st, *d);
      else if (al) hipLaunchKernelGGL((conv_fwd_x6_kernel<2, true, true>), grid, block, 0, st, *d);
      else hipLaunchKernelGGL((conv_fwd_x6_kernel<2, true>), grid, block, 0, st, *d);
    } else {
      D3A_CHECK_ARG((reinterpret_cast<uintptr_t>(d->x_f32) & 15) == 0,
                    "d3a_conv_fwd: fp32 input must be 16-byte aligned");
      if (conv_fwd_pack()) {
        // the weight re-laid in the walk order first: coalesced chunk loads
        const int64_t n = (int64_t)d->CO * d->C * d->KH * d->KW;
        if (!d->wpack_ready)
          hipLaunchKernelGGL(conv_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                             d->weight, d->wpack, d->C, d->KH, d->KW, n);
        if (d->CO == 32) hipLaunchKernelGGL((conv_fwd_x6_kernel<1, false, false, true>), grid, block, 0, st, *d);
        else hipLaunchKernelGGL((conv_fwd_x6_kernel<2, false, false, true>), grid, block, 0, st, *d);
      } else {
        if (d->CO == 32) hipLaunchKernelGGL((conv_fwd_x6_kernel<1, false>), grid, block, 0, st, *d);
        else hipLaunchKernelGGL((conv_fwd_x6_kernel<2, false>), grid, block, 0, st, *d);
      }
    }
    D3A_LAUNCH_CHECK("d3a_conv_fwd");
    return 0;
  }
  if (d->x_u8) {
    const bool aligned = d->W % 4 == 0 && d->S % 4 == 0 &&
                         (reinterpret_cast<uintptr_t>(d->x_u8) & 3) == 0;
    const float* wk = d->weight;  // (c, kh, kw) walk order == nn.Conv2d layout
    if (d->CO == 32) {
      if (aligned) hipLaunchKernelGGL((conv_fwd_kernel<1, true, true>), grid, block, 0, st, *d, wk);
      else hipLaunchKernelGGL((conv_fwd_kernel<1, true, false>), grid, block, 0, st, *d, wk);
    } else {
      if (aligned) hipLaunchKernelGGL((conv_fwd_kernel<2, true, true>), grid, block, 0, st, *d, wk);
      else hipLaunchKernelGGL((conv_fwd_kernel<2, true, false>), grid, block, 0, st, *d, wk);
    }
  } else {
    D3A_CHECK_ARG((reinterpret_cast<uintptr_t>(d->x_f32) & 15) == 0 &&
                      (reinterpret_cast<uintptr_t>(d->wpack) & 15) == 0,
                  "d3a_conv_fwd: fp32 input and wpack must be 16-byte aligned");
    const int64_t n = (int64_t)d->CO * d->C * d->KH * d->KW;
    hipLaunchKernelGGL(conv_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       d->weight, d->wpack, d->C, d->KH, d->KW, n);
    if (d->CO == 32)
      hipLaunchKernelGGL((conv_fwd_kernel<1, false, true>), grid, block, 0, st, *d, d->wpack);
    else
      hipLaunchKernelGGL((conv_fwd_kernel<2, false, true>), grid, block, 0, st, *d, d->wpack);
  }
  D3A_LAUNCH_CHECK("d3a_conv_fwd");
  return 0;
}

namespace d3a {
namespace {
// the split-bf16 weight-gradient kernel unless D3A_CONV_BWD_X6=0
bool conv_bwd_x6() {
  static const bool on = [] {
    const char* e = getenv("D3A_CONV_BWD_X6");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

// the first-layer weight-gradient kernel (conv1_bwd_w_u8s4_kernel);
// D3A_CONV1_U8S4=0 keeps the generic fp32-MFMA kernel (A/B)
bool conv1_u8s4() {
  static const bool on = [] {
    const char* e = getenv("D3A_CONV1_U8S4");
    return !(e && atoi(e) == 0);
  }();
  return on;
}
// d3a_conv_bwd_x's products on fp32 MFMA (packed weights) unless
// D3A_CONV_BWD_X_F32=0 (split-bf16: 64 / 59 us against 69 / 71 on K5's layers,
// but with the split-bf16 weight gradients of the same layers the B = 512
// arbiter measures the first conv's bias gradient at 1.03e-5 of fp64 -- over
// its 1e-5 bar -- where the fp32-MFMA input gradient keeps it at 4.3e-6)
bool conv_bwd_x_f32() {
  static const bool on = [] {
    const char* e = getenv("D3A_CONV_BWD_X_F32");
    return !(e && atoi(e) == 0);
  }();
  return on;
}
}  // namespace
}  // namespace d3a

// the weight-gradient split count that fills the chip for this geometry (the
// caller sizes its dW / db partial space with it): about 512 workgroups of the
// split-bf16 kernel, at least 16 rows a wave
extern "C" int32_t d3a_conv_bwd_w_splits(const d3a_conv_desc* d) {
  using namespace d3a;
  if (d == nullptr) return -1;
  const int64_t M = (int64_t)d->B * d->OH * d->OW;
  const int64_t Kc = (int64_t)d->C * d->KH * d->KW;
  if (conv1_u8s4_ok(d) && conv1_u8s4()) {
    // the first-layer kernel: ~256 workgroups over the CO / 32 column blocks,
    // >= 32 16-row steps (4 a wave) each
    const int64_t steps = (M / 4 + 3) / 4;
    int64_t s = 256 / (d->CO / 32);
    if (s > steps / 32) s = steps / 32;
    return (int32_t)(s > 1 ? s : 1);
  }
  if (d->x_u8 || !conv_bwd_x6()) {
    // the fp32-MFMA kernel: >= 32 rows a split, at most 32 splits
    const int64_t s = M / 32 < 32 ? M / 32 : 32;
    return (int32_t)(s > 1 ? s : 1);
  }
  const int64_t tiles = ((Kc + 63) / 64) * (d->CO / 32 > 0 ? d->CO / 32 : 1);
  int64_t s = (512 + tiles - 1) / tiles;
  const int64_t cap = M / 128 > 1 ? M / 128 : 1;  // >= 16 rows for each of 8 waves
  if (s > cap) s = cap;
  if (s < 1) s = 1;
  if (s > 1024) s = 1024;
  return (int32_t)s;
}

extern "C" int d3a_conv_bwd_w(const d3a_conv_desc* d, void* stream) {
  using namespace d3a;
  if (check_geometry(d, "d3a_conv_bwd_w")) return -1;
  D3A_CHECK_ARG(d->dy && d->dW, "d3a_conv_bwd_w: null dy / dW");
  D3A_CHECK_ARG(d->splits >= 1 && d->splits < 65536, "d3a_conv_bwd_w: bad splits");
  const int64_t Kc = (int64_t)d->C * d->KH * d->KW;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (conv1_u8s4_ok(d) && conv1_u8s4()) {
    const dim3 grid(1u, (unsigned)(d->CO / 32), (unsigned)d->splits);
    switch (Kc / 32) {
      case 2: hipLaunchKernelGGL(conv1_bwd_w_u8s4_kernel<2>, grid, dim3(512), 0, st, *d); break;
      case 4: hipLaunchKernelGGL(conv1_bwd_w_u8s4_kernel<4>, grid, dim3(512), 0, st, *d); break;
      case 6: hipLaunchKernelGGL(conv1_bwd_w_u8s4_kernel<6>, grid, dim3(512), 0, st, *d); break;
      default: hipLaunchKernelGGL(conv1_bwd_w_u8s4_kernel<8>, grid, dim3(512), 0, st, *d); break;
    }
    D3A_LAUNCH_CHECK("d3a_conv_bwd_w");
    return 0;
  }
  if (conv_bwd_x6() && !d->x_u8) {
    // split-bf16 weight gradient: 32 (co) x 64 (k) per wave, 8 waves a workgroup
    // (fp32 input; the uint8 layer stays on the fp32-MFMA kernel: both are bound
    // by the byte gathers there, measured 133 us at 128 splits either way, 119
    // for the fp32 kernel at 32)
    constexpr int NK = 2;
    const dim3 grid((unsigned)((Kc + 32 * NK - 1) / (32 * NK)), (unsigned)(d->CO / 32), (unsigned)d->splits);
    if (d->x_u8) hipLaunchKernelGGL((conv_bwd_w_x6_kernel<NK, true>), grid, dim3(512), 0, st, *d);
    else hipLaunchKernelGGL((conv_bwd_w_x6_kernel<NK, false>), grid, dim3(512), 0, st, *d);
    D3A_LAUNCH_CHECK("d3a_conv_bwd_w");
    return 0;
  }
  // 32 (co) x 32 (k) per wave, 16 waves per workgroup over consecutive row slices
  const dim3 grid((unsigned)((Kc + 31) / 32), (unsigned)(d->CO / 32), (unsigned)d->splits);
  if (d->x_u8) hipLaunchKernelGGL((conv_bwd_w_kernel<1, 16, true>), grid, dim3(1024), 0, st, *d);
  else hipLaunchKernelGGL((conv_bwd_w_kernel<1, 16, false>), grid, dim3(1024), 0, st, *d);
  D3A_LAUNCH_CHECK("d3a_conv_bwd_w");
  return 0;
}

extern "C" int d3a_conv_bwd_x(const d3a_conv_desc* d, void* stream) {
  using namespace d3a;
  if (check_geometry(d, "d3a_conv_bwd_x")) return -1;
  D3A_CHECK_ARG(d->dy && d->y, "d3a_conv_bwd_x: null dy / dx (y)");
  D3A_CHECK_ARG(d->x_f32 || !d->relu, "d3a_conv_bwd_x: the ReLU gate reads x_f32");
  D3A_CHECK_ARG(d->C == 32 || d->C == 64, "d3a_conv_bwd_x: C must be 32 or 64");
  D3A_CHECK_ARG(d->CO % 16 == 0 && (reinterpret_cast<uintptr_t>(d->dy) & 15) == 0,
                "d3a_conv_bwd_x: dy must be 16-byte aligned rows of CO %% 16 == 0 floats");
  D3A_CHECK_ARG(d->S <= 8, "d3a_conv_bwd_x: stride must be <= 8");
  const int64_t nyp = (d->H + d->S - 1) / d->S, nxp = (d->W + d->S - 1) / d->S;
  const int64_t Mp = (int64_t)d->B * nyp * nxp;  // the largest phase
  if (Mp == 0) return 0;
  const int64_t blocks = (Mp + 127) / 128;
  D3A_CHECK_ARG(blocks < (1ll << 31), "d3a_conv_bwd_x: too many rows");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)blocks, (unsigned)(d->S * d->S)), block(256);
  if (d->wpack && d->CO % 32 == 0) {
    // the weight re-laid [KH][KW][CO][C] into the wpack scratch first (unless
    // the caller did: wpack_ready): each chunk is then one coalesced run
    // instead of 32 co x C scattered floats
    const int64_t n = (int64_t)d->CO * d->C * d->KH * d->KW;
    if (!d->wpack_ready)
      hipLaunchKernelGGL(conv_pack_tap_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                         d->weight, d->wpack, d->CO, d->C, d->KH, d->KW);
    if (conv_bwd_x_f32()) {
      if (d->C == 32) hipLaunchKernelGGL((conv_bwd_x_x6_kernel<1, true, true>), grid, block, 0, st, *d);
      else hipLaunchKernelGGL((conv_bwd_x_x6_kernel<2, true, true>), grid, block, 0, st, *d);
    } else {
      if (d->C == 32) hipLaunchKernelGGL((conv_bwd_x_x6_kernel<1, true>), grid, block, 0, st, *d);
      else hipLaunchKernelGGL((conv_bwd_x_x6_kernel<2, true>), grid, block, 0, st, *d);
    }
  } else {
    if (d->C == 32) hipLaunchKernelGGL((conv_bwd_x_x6_kernel<1, false>), grid, block, 0, st, *d);
    else hipLaunchKernelGGL((conv_bwd_x_x6_kernel<2, false>), grid, block, 0, st, *d);
  }
  D3A_LAUNCH_CHECK("d3a_conv_bwd_x");
  return 0;
}

extern "C" int d3a_conv_pack_weights_philox(const d3a_conv_desc* descs, const int32_t* layouts,
                                            int32_t n, const d3a_philox_job* ph, void* stream) {
  using namespace d3a;
  D3A_CHECK_ARG(descs && layouts && n >= 1 && n <= 8, "d3a_conv_pack_weights: 1..8 descriptors");
  D3A_CHECK_ARG(ph == nullptr || (ph->out && ph->ctr && ph->ticket && ph->n_normal >= 0 &&
                                  ph->n_uniform >= 0),
                "d3a_conv_pack_weights_philox: the philox job needs out, ctr and ticket");
  PackJobs J{};
  int64_t tot = 0;
  for (int i = 0; i < n; ++i) {
    const d3a_conv_desc& d = descs[i];
    D3A_CHECK_ARG(d.weight && d.wpack && d.CO >= 1 && d.C >= 1 && d.KH >= 1 && d.KW >= 1,
                  "d3a_conv_pack_weights: null weight / wpack or bad geometry");
    D3A_CHECK_ARG(layouts[i] == 0 || layouts[i] == 1, "d3a_conv_pack_weights: layout must be 0 or 1");
    J.w[i] = d.weight;
    J.dst[i] = d.wpack;
    J.CO[i] = d.CO;
    J.C[i] = d.C;
    J.KH[i] = d.KH;
    J.KW[i] = d.KW;
    J.layout[i] = layouts[i];
    tot += (int64_t)d.CO * d.C * d.KH * d.KW;
    J.end[i] = tot;
  }
  J.n = n;
  D3A_CHECK_ARG(tot < (1ll << 31), "d3a_conv_pack_weights: too many elements");
  J.pk_blocks = (int)((tot + 255) / 256);
  int64_t ph_blocks = 0;
  if (ph != nullptr && ph->n_normal + ph->n_uniform > 0) {
    J.ph = *ph;
    ph_blocks = ((ph->n_normal + ph->n_uniform + 3) / 4 + 255) / 256;
  }
  hipLaunchKernelGGL(conv_pack_multi_kernel, dim3((unsigned)(J.pk_blocks + ph_blocks)), dim3(256), 0,
                     (hipStream_t)stream, J);
  D3A_LAUNCH_CHECK("d3a_conv_pack_weights");
  return 0;
}

extern "C" int d3a_conv_pack_weights(const d3a_conv_desc* descs, const int32_t* layouts, int32_t n,
                                     void* stream) {
  return d3a_conv_pack_weights_philox(descs, layouts, n, nullptr, stream);
}
