// fp32-accurate forward of a two-hidden-layer ensemble MLP with a wide head,
// [n_in <= 64 -> 256 -> 256 -> n_out <= 256], on the bf16 matrix cores
// (exact three-way split-bf16 operands, the six part products above fp32
// resolution, fp32 accumulation: x6.hpp, q2_x6.hip).
//
// The pass it is for: BCQ's target step (bcq_impl.py:215-226 through
// compute_max_with_n_actions, q_functions/__init__.py:8-63) evaluates the
// target QR critics [obs + act -> 256 -> 256 -> 200 quantiles]
// (encoders.py:265-275, 328-339; qr_q_function.py:97-161) over B * N = 25,600
// sampled actions per member -- 12.56 GFLOP per K3 step, the largest GEMM of
// the BCQ update -- and the target residual policy [obs + act -> 256 -> 256 ->
// act] over the same rows.  d3a_mlp_fwd's contract (kept activations optional,
// no aux pass, out [C][rows][ldout]).
//
// A workgroup owns 64 rows of one member; eight waves (two per SIMD).
//   layer 1: in 64-unit chunks, each a 64 x 64 block of sixteen 16 x 16 tiles
//     (v_mfma_f32_16x16x32_bf16), two per wave -- every wave produces its share
//     of the next chunk while layer 2 consumes the current one (a two-slot LDS
//     ring of the three bf16 parts, [row][k]; fp32 kept rows to h[0])
//   layer 2: wave w owns units 32 w .. + 31 over the 64 rows (two transposed
//     32 x 32 tiles C^T[unit][row], W1 the A operand split from fp32 loads one
//     chunk ahead, the ring the B operand)
//   head: the layer-2 activations are written once as parts over the ring
//     ([row][unit], 528-byte rows), then wave w < ceil(n_out / 32) computes
//     outputs 32 w .. + 31 for the 64 rows over K = 256 (Wh rows split from
//     fp32 loads two k steps ahead); lane = row, four runs of four outputs:
//     16-byte stores.
#include <cstdlib>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"
#include "x6.hpp"

namespace d3a {
namespace {

using namespace x6;

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int W_H = 256;    // hidden width
constexpr int W_RB = 64;    // rows per workgroup
constexpr int W_CK = 64;    // layer-2 k per chunk (= layer-1 units per chunk)
constexpr int W_NCK = W_H / W_CK;
constexpr int W_KS = W_CK / 16;
constexpr int W_LDB = 72;   // bf16 stride of a ring row (144 B)
constexpr int W_LDH = 264;  // bf16 stride of an h2 image row (528 B)

__device__ __forceinline__ f32x4 mfma16x16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 prod6_16(const bf16x8* a, const bf16x8* b, f32x4 c) {
  c = mfma16x16(a[2], b[0], c);
  c = mfma16x16(a[1], b[1], c);
  c = mfma16x16(a[0], b[2], c);
  c = mfma16x16(a[1], b[0], c);
  c = mfma16x16(a[0], b[1], c);
  c = mfma16x16(a[0], b[0], c);
  return c;
}

template <int XL>
struct WideLds {
  union {
    struct {
      __bf16 ring[2][3][W_RB * W_LDB];
      __bf16 x[3][W_RB * (XL + 8)];
    } a;
    __bf16 h2[3][W_RB * W_LDH];  // after layer 2
  } u;
  float rs[8][W_RB];  // row_mean: per-wave output sums [wave][row]
};

// XL: n_in rounded up to 32 (32 or 64)
template <int XL>
__global__ __launch_bounds__(512) void mlp_x6_wide_kernel(d3a_mlp_fwd_desc d) {
  constexpr int XLD = XL + 8;
  constexpr int NS0 = XL / 32;  // layer-1 k steps (16x16x32)
  __shared__ __attribute__((aligned(16))) WideLds<XL> L;
  static_assert(sizeof(WideLds<XL>) <= 163840, "LDS");
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int l16 = lane & 15, lq = lane >> 4;
  const int c = blockIdx.z;
  const int m0 = (int)d.r0 + (int)blockIdx.x * W_RB;
  const int rend = (int)(d.r0 + d.rows);
  const int h_from = (int)d.h_from;
  const int nin = d.n_in, nout = d.n_out;
  float* const outp = d.out + c * d.sout;
  float* const h0g = d.h[0] ? d.h[0] + c * d.sh : nullptr;
  float* const h1g = d.h[1] ? d.h[1] + c * d.sh : nullptr;
  const float* W0 = d.W[0] + c * d.sW[0];
  const float* b0 = d.b[0] + c * d.sb[0];
  const float* W1 = d.W[1] + c * d.sW[1] + (32 * w + li) * W_H + 8 * lh;
  const float* Wh = d.W[2] + c * d.sW[2];
  const float* bh = d.b[2] + c * d.sb[2];

  // ---- prologue: the first W1 chunk in flight, input rows split into LDS
  float4 wr[W_KS][2];
  auto load_w1 = [&](int j) {
#pragma unroll
    for (int s = 0; s < W_KS; ++s) {
      wr[s][0] = *reinterpret_cast<const float4*>(W1 + W_CK * j + 16 * s);
      wr[s][1] = *reinterpret_cast<const float4*>(W1 + W_CK * j + 16 * s + 4);
    }
  };
  load_w1(0);
  {
    const float* xb = d.x + c * d.sxb;
    const int64_t ldx = d.ldx;
    constexpr int X4 = XL / 4;
    for (int e = t; e < W_RB * X4; e += 512) {
      const int m = e / X4, k4 = (e - m * X4) * 4;
      const int r = m0 + m;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (r < rend && k4 + j < nin) ? input_at(d, xb, ldx, r, k4 + j) : 0.f;
      bf16x4 p[3];
      split4(v, p);
#pragma unroll
      for (int q = 0; q < 3; ++q) *reinterpret_cast<bf16x4*>(&L.u.a.x[q][m * XLD + k4]) = p[q];
    }
  }
  __syncthreads();  // x parts staged

  // ---- layer 1, chunk j: sixteen 16 x 16 tiles (unit tile ut = w >> 1 of 16
  // units, row tiles rt0 + {0, 1}, rt0 = 2 (w & 1)); lane: row 16 rt + l16,
  // units 16 ut + 4 lq + i.  W0 rows and bias of the next chunk loaded one
  // production ahead.
  const int ut = w >> 1, rt0 = 2 * (w & 1);
  float w0n[NS0][8];
  float4 b0n;
  auto load_w0 = [&](int j) {
    const int u = W_CK * j + 16 * ut + l16;
#pragma unroll
    for (int s = 0; s < NS0; ++s)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int k = 32 * s + 8 * lq + i;
        w0n[s][i] = k < nin ? W0[u * nin + k] : 0.f;
      }
    b0n = *reinterpret_cast<const float4*>(b0 + W_CK * j + 16 * ut + 4 * lq);
  };
  load_w0(0);
  auto produce = [&](int j) {
    f32x4 a[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) a[r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS0; ++s) {
      bf16x8 wp[3];
      split8(w0n[s], wp);
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        bf16x8 xp[3];
#pragma unroll
        for (int q = 0; q < 3; ++q)
          xp[q] = *reinterpret_cast<const bf16x8*>(
              &L.u.a.x[q][(16 * (rt0 + r) + l16) * XLD + 32 * s + 8 * lq]);
        a[r] = prod6_16(wp, xp, a[r]);
      }
    }
    const float4 bv = b0n;
    if (j + 1 < W_NCK) load_w0(j + 1);
    const int k = 16 * ut + 4 * lq;  // local k of the chunk
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int rl = 16 * (rt0 + r) + l16;
      const int row = m0 + rl;
      float v[4] = {fmaxf(a[r][0] + bv.x, 0.f), fmaxf(a[r][1] + bv.y, 0.f),
                    fmaxf(a[r][2] + bv.z, 0.f), fmaxf(a[r][3] + bv.w, 0.f)};
      if (h0g != nullptr && row >= h_from && row < rend)
        *reinterpret_cast<float4*>(h0g + row * W_H + W_CK * j + k) = make_float4(v[0], v[1], v[2], v[3]);
      bf16x4 p[3];
      split4(v, p);
#pragma unroll
      for (int q = 0; q < 3; ++q)
        *reinterpret_cast<bf16x4*>(&L.u.a.ring[j & 1][q][rl * W_LDB + k]) = p[q];
    }
  };
  produce(0);
  __syncthreads();  // chunk 0 in slot 0

  // ---- layer 2: acc[rt] = C^T[units 32 w ..][rows 32 rt ..]
  f32x16 acc[2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[rt][r] = 0.f;
#pragma unroll 1
  for (int j = 0; j < W_NCK; ++j) {
    float4 wc[W_KS][2];
#pragma unroll
    for (int s = 0; s < W_KS; ++s) {
      wc[s][0] = wr[s][0];
      wc[s][1] = wr[s][1];
    }
    if (j + 1 < W_NCK) load_w1(j + 1);
    const int slot = j & 1;
#pragma unroll
    for (int s = 0; s < W_KS; ++s) {
      bf16x8 wa[3];
      const float v[8] = {wc[s][0].x, wc[s][0].y, wc[s][0].z, wc[s][0].w,
                          wc[s][1].x, wc[s][1].y, wc[s][1].z, wc[s][1].w};
      split8(v, wa);
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        bf16x8 bp[3];
#pragma unroll
        for (int q = 0; q < 3; ++q)
          bp[q] = *reinterpret_cast<const bf16x8*>(
              &L.u.a.ring[slot][q][(32 * rt + li) * W_LDB + 16 * s + 8 * lh]);
        acc[rt] = prod6(wa, bp, acc[rt]);
      }
      if (s == 1 && j + 1 < W_NCK) produce(j + 1);
    }
    __syncthreads();  // slot j & 1 free; chunk j + 1 in slot (j + 1) & 1
  }

  // ---- layer-2 epilogue: bias, ReLU, kept rows to h[1], parts to the h2
  // image (over the ring: every wave passed the loop's last barrier)
  {
    const float* b1 = d.b[1] + c * d.sb[1];
#pragma unroll
    for (int R = 0; R < 4; ++R) {
      const int u = 32 * w + 8 * R + 4 * lh;
      const float4 bv = *reinterpret_cast<const float4*>(b1 + u);
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const int rl = 32 * rt + li;
        const int row = m0 + rl;
        float v[4] = {fmaxf(acc[rt][4 * R + 0] + bv.x, 0.f), fmaxf(acc[rt][4 * R + 1] + bv.y, 0.f),
                      fmaxf(acc[rt][4 * R + 2] + bv.z, 0.f), fmaxf(acc[rt][4 * R + 3] + bv.w, 0.f)};
        if (h1g != nullptr && row >= h_from && row < rend)
          *reinterpret_cast<float4*>(h1g + row * W_H + u) = make_float4(v[0], v[1], v[2], v[3]);
        bf16x4 p[3];
        split4(v, p);
#pragma unroll
        for (int q = 0; q < 3; ++q) *reinterpret_cast<bf16x4*>(&L.u.h2[q][rl * W_LDH + u]) = p[q];
      }
    }
  }
  __syncthreads();  // h2 image complete

  // ---- head: wave w computes outputs 32 w .. + 31 (A = Wh rows, B = h2 image)
  const int nkt = (nout + 31) / 32;
  if (w < nkt) {
    const int kout = 32 * w + li;  // A-operand row (output) of this lane
    const bool kok = kout < nout;
    const float* whr = Wh + (kok ? kout : 0) * W_H + 8 * lh;
    f32x16 o[2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[rt][r] = 0.f;
    // raw fp32 Wh of k steps s .. s + HD - 1 in flight (an L2 round trip is
    // longer than two steps' twelve MFMAs)
    constexpr int HD = 4;
    float4 hr[HD][2];
    auto load_h = [&](int s, int slot) {
      hr[slot][0] = kok ? *reinterpret_cast<const float4*>(whr + 16 * s) : make_float4(0.f, 0.f, 0.f, 0.f);
      hr[slot][1] = kok ? *reinterpret_cast<const float4*>(whr + 16 * s + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    };
#pragma unroll
    for (int s = 0; s < HD; ++s) load_h(s, s);
#pragma unroll
    for (int s = 0; s < W_H / 16; ++s) {
      bf16x8 wa[3];
      const int sl = s % HD;
      const float v[8] = {hr[sl][0].x, hr[sl][0].y, hr[sl][0].z, hr[sl][0].w,
                          hr[sl][1].x, hr[sl][1].y, hr[sl][1].z, hr[sl][1].w};
      split8(v, wa);
      if (s + HD < W_H / 16) load_h(s + HD, sl);
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        bf16x8 bp[3];
#pragma unroll
        for (int q = 0; q < 3; ++q)
          bp[q] = *reinterpret_cast<const bf16x8*>(&L.u.h2[q][(32 * rt + li) * W_LDH + 16 * s + 8 * lh]);
        o[rt] = prod6(wa, bp, o[rt]);
      }
    }
    // lane: row 32 rt + li, outputs 32 w + 8 R + 4 lh + i
    const int64_t ldo = d.ldout;
    float rsum[2] = {0.f, 0.f};  // row_mean: this lane's outputs, in output order
    const bool vec = ((reinterpret_cast<uintptr_t>(outp) & 15) == 0) && (ldo & 3) == 0;
#pragma unroll
    for (int R = 0; R < 4; ++R) {
      const int k0 = 32 * w + 8 * R + 4 * lh;
      float bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) bv[i] = k0 + i < nout ? bh[k0 + i] : 0.f;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const int row = m0 + 32 * rt + li;
        if (row >= rend) continue;
        float* op = outp + (int64_t)row * ldo + k0;
        const float v0 = o[rt][4 * R] + bv[0], v1 = o[rt][4 * R + 1] + bv[1];
        const float v2 = o[rt][4 * R + 2] + bv[2], v3 = o[rt][4 * R + 3] + bv[3];
        if (k0 + 0 < nout) rsum[rt] += v0;
        if (k0 + 1 < nout) rsum[rt] += v1;
        if (k0 + 2 < nout) rsum[rt] += v2;
        if (k0 + 3 < nout) rsum[rt] += v3;
        if (k0 + 3 < nout && vec) {
          *reinterpret_cast<float4*>(op) = make_float4(v0, v1, v2, v3);
        } else {
          if (k0 + 0 < nout) op[0] = v0;
          if (k0 + 1 < nout) op[1] = v1;
          if (k0 + 2 < nout) op[2] = v2;
          if (k0 + 3 < nout) op[3] = v3;
        }
      }
    }
    if (d.row_mean != nullptr) {
      // the two lane halves hold interleaved runs of four outputs: the wave's
      // 32 outputs of a row as (lane half 0's 16) + (lane half 1's 16)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const float other = __shfl_xor(rsum[rt], 32, 64);
        if (lh == 0) L.rs[w][32 * rt + li] = rsum[rt] + other;
      }
    }
  }
  if (d.row_mean != nullptr) {
    __syncthreads();  // uniform: row_mean is a kernel argument
    if (t < W_RB) {
      float s = L.rs[0][t];
      for (int v = 1; v < nkt; ++v) s += L.rs[v][t];
      const int row = m0 + t;
      if (row < rend) d.row_mean[c * d.s_mean + row] = s / (float)nout;
    }
  }
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_mlp_fwd_x6(const d3a_mlp_fwd_desc* dp, void* stream) {
  D3A_CHECK_ARG(dp, "d3a_mlp_fwd_x6: null desc");
  const d3a_mlp_fwd_desc& d = *dp;
  D3A_CHECK_ARG(d.n_hidden == 2 && d.H == W_H && d.n_out >= 1 && d.n_out <= 256 && d.n_in >= 1 &&
                    d.n_in <= 64,
                "d3a_mlp_fwd_x6: needs [n_in <= 64, 256, 256, n_out <= 256]");
  D3A_CHECK_ARG((d.x || d.xg_mode) && d.out && d.W[0] && d.W[1] && d.W[2] && d.b[0] && d.b[1] &&
                    d.b[2],
                "d3a_mlp_fwd_x6: null operand");
  D3A_CHECK_ARG(xgen_ok(d), "d3a_mlp_fwd_x6: bad input-row builder (xg_*)");
  D3A_CHECK_ARG(d.hmask == nullptr, "d3a_mlp_fwd_x6: hmask is d3a_q2_fwd_x6 only");
  D3A_CHECK_ARG(d.aux_rows == 0 && d.parts <= 1, "d3a_mlp_fwd_x6: no aux pass / parts");
  D3A_CHECK_ARG(d.C >= 1 && d.rows >= 0 && d.r0 >= 0 && d.h_from >= 0, "d3a_mlp_fwd_x6: bad sizes");
  auto a16 = [](const void* p, int64_t stride) {
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && stride % 4 == 0;
  };
  D3A_CHECK_ARG(a16(d.W[1], d.sW[1]) && a16(d.W[2], d.sW[2]) && a16(d.b[0], d.sb[0]) &&
                    a16(d.b[1], d.sb[1]),
                "d3a_mlp_fwd_x6: W1, Wh, b0 and b1 must be 16-byte aligned");
  D3A_CHECK_ARG((d.h[0] == nullptr || (reinterpret_cast<uintptr_t>(d.h[0]) & 15) == 0) &&
                    (d.h[1] == nullptr || (reinterpret_cast<uintptr_t>(d.h[1]) & 15) == 0) &&
                    d.sh % 4 == 0,
                "d3a_mlp_fwd_x6: kept activations must be 16-byte aligned rows of 256");
  D3A_CHECK_ARG((d.r0 + d.rows) * (int64_t)(d.ldout > W_H ? d.ldout : W_H) < (int64_t(1) << 31) &&
                    (d.r0 + d.rows) * d.ldx < (int64_t(1) << 31),
                "d3a_mlp_fwd_x6: rows x row stride exceeds 2^31");
  D3A_CHECK_ARG(d.ldout >= d.n_out, "d3a_mlp_fwd_x6: ldout < n_out");
  D3A_CHECK_ARG(d.row_mean == nullptr || (d.s_mean >= d.r0 + d.rows &&
                                          d.s_mean * (int64_t)d.C < (int64_t(1) << 31)),
                "d3a_mlp_fwd_x6: row_mean member stride must cover the rows");
  if (d.rows == 0) return 0;
  const dim3 grid((unsigned)((d.rows + W_RB - 1) / W_RB), 1, (unsigned)d.C);
  const hipStream_t st = (hipStream_t)stream;
  if (d.n_in <= 32)
    hipLaunchKernelGGL(mlp_x6_wide_kernel<32>, grid, dim3(512), 0, st, d);
  else
    hipLaunchKernelGGL(mlp_x6_wide_kernel<64>, grid, dim3(512), 0, st, d);
  D3A_LAUNCH_CHECK("d3a_mlp_fwd_x6");
  return 0;
}
