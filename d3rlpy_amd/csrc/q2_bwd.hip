// Critic backward of a two-hidden-layer, single-output Q ensemble in one launch:
// every weight / bias gradient of the head and both trunk layers.
//
// Replaces, for update_critic (d3rlpy/algos/torch/ddpg_impl.py:119-133 via
// cql_impl.py:110-125), the autograd backward of
//   VectorEncoderWithAction [n_in -> 256 -> 256]  (encoders.py:265-275, 328-339)
//   + ContinuousMeanQFunction._fc                  (q_functions/mean_q_function.py:255-256)
// for the weight gradients (no input gradient).  Per member c and row r:
//   g'   = g[r] (* gscale for r < n_scaled)
//   dz2  = g' w3 * [h2 > 0]            dW3 = g'^T h2,  db3 = sum g'
//   dz1  = (dz2 W2) * [h1 > 0]         dW2 = dz2^T h1, db2 = sum dz2
//                                      dW1 = dz1^T x,  db1 = sum dz1
//
// Why one kernel: the two large products of this backward, dz2 W2 (the input
// gradient of layer 2) and dz2^T h1 (its weight gradient), read the same dz2
// and h1 rows.  A workgroup owns 256 rows of one member and a quarter (64
// units) of layer 1: it stages W2[:, quarter] in LDS once, then for each
// 64-row sub-block generates dz2 (64 x 256) into LDS from h2 and stages the
// h1 and x tiles beside it.  Four waves, one per SIMD (so each has the whole
// 512-entry register file: accumulators, the next sub-block's loads and the
// operand pipeline never spill); wave w computes, per sub-block,
//   dh1 tile (rows 32 (w & 1).., units 32 (w >> 1)..) = dz2 W2[:, quarter]
//       (K = 256), its ReLU mask, and the first layer's dW1 / db1 from the
//       masked tile in registers
//   dW2[64 w .. 64 w + 63][quarter] += dz2^T h1[:, quarter]  (K = 64 rows)
// with the two independent MFMA chains interleaved (272 MFMAs per wave per
// sub-block).  The next sub-block's loads are in flight during the MFMAs.  Gradients leave as one partial per 256-row block
// (the optimiser sums them in order, like split-K partials); every other
// reduction is in a fixed order, so the result is run-to-run bit-identical.
// MFMA: v_mfma_f32_32x32x2_f32 (exact fp32), operands from LDS with
// conflict-free strides (dz2 rows 257 floats apart: its rows and its columns
// are both read as 32 consecutive banks).
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int Q2_H = 256;    // hidden width
constexpr int Q2_RB = 256;   // rows per workgroup (one gradient partial)
constexpr int Q2_SB = 64;    // rows per LDS sub-block
constexpr int Q2_NSB = Q2_RB / Q2_SB;
constexpr int Q2_QW = 64;    // layer-1 units per workgroup
constexpr int Q2_LDZ = 257;  // dz2 row stride
constexpr int Q2_XMAX = 48;  // widest first-layer input staged in LDS
constexpr int Q2_NT = 256;   // threads: four waves, one per SIMD

struct Q2Lds {
  float w2[Q2_H * Q2_QW];    // W2[o][i0 + i]
  float dz[Q2_SB * Q2_LDZ];  // dz2[r][o]
  float h1[Q2_SB * Q2_QW];   // h1[r][i0 + i]
  float x[Q2_SB * Q2_XMAX];  // x[r][d]
};
static_assert(sizeof(Q2Lds) <= 163840, "LDS");

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// XL: the first layer's input width rounded up to 4 (16, 32 or 48), fixed at
// compile time so the LDS addresses of the x operand are immediates
template <int XL>
__global__ __launch_bounds__(Q2_NT) void q2_bwd_kernel(d3a_q2_bwd_desc d) {
  __shared__ __attribute__((aligned(16))) Q2Lds L;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);  // wave-uniform
  const int li = lane & 31, lk = lane >> 5;
  // XCD-aware decode: the four quarters of one (row block, member) unit get
  // block ids 8 apart, i.e. the same XCD under round-robin dispatch, so the
  // h2 rows all four read are fetched into one L2 (speed only)
  const int64_t P = (d.rows + Q2_RB - 1) / Q2_RB;
  const int64_t nunits = P * d.C;
  const int bid = blockIdx.x;
  const int kx = bid >> 3;
  const int q = kx & 3;
  const int64_t u = (int64_t)(kx >> 2) * 8 + (bid & 7);
  if (u >= nunits) return;  // whole workgroup: no barrier has been passed
  const int64_t p = u / d.C;
  const int c = (int)(u - p * d.C);
  const int64_t rows = d.rows;
  const int64_t rb0 = p * Q2_RB;
  const int ldx = (int)d.ldx;
  constexpr int ldh = Q2_H;  // h1 / h2 rows are [C][rows][256] (checked)
  const float* h1g = d.h1 + c * d.sh;
  const float* h2g = d.h2 + c * d.sh;
  const float* gg = d.g + c * d.sgb;
  const float* xg = d.x + c * d.sxb;
  const float* W2g = d.W2 + c * d.sW2;
  const float* w3g = d.w3 + c * d.sw3;
  const float gs = d.gscale ? *d.gscale : 1.f;
  const int i0 = q * Q2_QW;
  const int nin = d.n_in, xr4 = (nin + 3) / 4;  // float4 pieces of an x row
  constexpr int x4 = XL / 4;
  constexpr int XV = (Q2_SB * x4 + Q2_NT - 1) / Q2_NT;  // x pieces per thread
  const int64_t rlast = rows - 1;

  // ---- W2[:, quarter] -> LDS (once), w3 for this lane's columns
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const int idx = t + Q2_NT * v, o = idx >> 4, c4 = (idx & 15) * 4;
    const float4 wv = *reinterpret_cast<const float4*>(W2g + o * Q2_H + i0 + c4);
    *reinterpret_cast<float4*>(&L.w2[o * Q2_QW + c4]) = wv;
  }
  float w3v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) w3v[j] = w3g[lane + 64 * j];

  // ---- sub-block loads (unconditional, clamped rows; validity applied at staging)
  // thread (w, lane): h2 rows w + 4s, columns lane + 64j; h1 / x as float4 pieces
  float hv[16][4], gv[16];
  float h1v[4][4], xv[XV][4];  // float4 pieces kept as scalars (registers)
  auto prefetch = [&](int sb) {
    const int64_t base = rb0 + sb * Q2_SB;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      int64_t r = base + w + 4 * s;
      r = r < rlast ? r : rlast;
      gv[s] = gg[r];
#pragma unroll
      for (int j = 0; j < 4; ++j) hv[s][j] = h2g[(int)r * ldh + lane + 64 * j];
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int idx = t + Q2_NT * v;
      int64_t r = base + (idx >> 4);
      r = r < rlast ? r : rlast;
      const float4 a = *reinterpret_cast<const float4*>(h1g + (int)r * ldh + i0 + (idx & 15) * 4);
      h1v[v][0] = a.x; h1v[v][1] = a.y; h1v[v][2] = a.z; h1v[v][3] = a.w;
    }
#pragma unroll
    for (int v = 0; v < XV; ++v) {
      const int idx = t + Q2_NT * v;
      const int ix = idx < Q2_SB * x4 ? idx : Q2_SB * x4 - 1;
      int64_t rx = base + ix / x4;
      rx = rx < rlast ? rx : rlast;
      const int cx = ix % x4 < xr4 ? ix % x4 : 0;  // pieces past n_in: staged as 0
      const float4 a = *reinterpret_cast<const float4*>(xg + (int)rx * ldx + cx * 4);
      xv[v][0] = a.x; xv[v][1] = a.y; xv[v][2] = a.z; xv[v][3] = a.w;
    }
  };

  // fp64 running sums: db2 / dW3 of column i0 + lane (every thread), db3
  // (lane 0 of each wave), db1 of this wave's dh1 column
  double acc_db2 = 0.0, acc_dw3 = 0.0, acc_db3 = 0.0, acc_db1 = 0.0;
  const int rh = w & 1, ib = w >> 1;  // dh1 tile: row half, 32-unit block
  // accumulators: A1 dh1 of the sub-block, W1[db] dW1 (input block db),
  // W2t[ob][bb] dW2 tile (o block 64 w + 32 ob, unit block 32 bb)
  f32x16 A1, W1[2], W2t[2][2];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    W1[0][r] = W1[1][r] = 0.f;
    W2t[0][0][r] = W2t[0][1][r] = W2t[1][0][r] = W2t[1][1][r] = 0.f;
  }
  const int ndb = (nin + 31) / 32;  // 32-wide input blocks of dW1 (1 or 2)

  auto stage = [&](int sb) {
    const int64_t base = rb0 + sb * Q2_SB;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int rl = w + 4 * s;
      const int64_t r = base + rl;
      const bool ok = r < rows;
      float gp = gv[s];
      if (r < d.n_scaled) gp *= gs;  // as d3a_head1_bwd forms g'
      if (!ok) gp = 0.f;
      float hq = 0.f, dq = 0.f;  // this workgroup's quarter column (j == q)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float hval = ok ? hv[s][j] : 0.f;
        const float dzv = hval > 0.f ? gp * w3v[j] : 0.f;
        L.dz[rl * Q2_LDZ + lane + 64 * j] = dzv;
        hq = j == q ? hval : hq;
        dq = j == q ? dzv : dq;
      }
      acc_db2 += (double)dq;
      acc_dw3 += (double)(gp * hq);
      if (lane == 0) acc_db3 += (double)gp;
    }
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int idx = t + Q2_NT * v, rl = idx >> 4;
      *reinterpret_cast<float4*>(&L.h1[rl * Q2_QW + (idx & 15) * 4]) =
          base + rl < rows ? make_float4(h1v[v][0], h1v[v][1], h1v[v][2], h1v[v][3]) : z;
    }
#pragma unroll
    for (int v = 0; v < XV; ++v) {
      const int idx = t + Q2_NT * v;
      if (idx < Q2_SB * x4) {
        const int rx = idx / x4;
        *reinterpret_cast<float4*>(&L.x[rx * XL + (idx % x4) * 4]) =
            (base + rx < rows && idx % x4 < xr4)
                ? make_float4(xv[v][0], xv[v][1], xv[v][2], xv[v][3]) : z;
      }
    }
  };

  prefetch(0);
#pragma unroll 1
  for (int sb = 0; sb < Q2_NSB; ++sb) {
    stage(sb);
    __syncthreads();
    if (sb + 1 < Q2_NSB) prefetch(sb + 1);  // in flight during the MFMAs
#pragma unroll
    for (int r = 0; r < 16; ++r) A1[r] = 0.f;
    // dh1: A = dz2[rows of half rh][o], B = W2[o][units of block ib]
    const float* Ax = &L.dz[(32 * rh + li) * Q2_LDZ + lk];
    const float* Bx = &L.w2[lk * Q2_QW + 32 * ib + li];
    // dW2: A = dz2[r][o of this wave's block], B = h1[r][units]
    const float* Aw = &L.dz[lk * Q2_LDZ + 64 * w + li];
    const float* Bw = &L.h1[lk * Q2_QW + li];
    // 32 steps, each: 4 k-steps of dh1 (8 o) + 1 k-step of dW2 (2 rows, 4 tiles)
#pragma unroll 2
    for (int it = 0; it < 32; ++it) {
      float a[4], b[4], aw[2], bw[2];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] = Ax[8 * it + 2 * e];
        b[e] = Bx[(8 * it + 2 * e) * Q2_QW];
      }
      aw[0] = Aw[(2 * it) * Q2_LDZ];
      aw[1] = Aw[(2 * it) * Q2_LDZ + 32];
      bw[0] = Bw[(2 * it) * Q2_QW];
      bw[1] = Bw[(2 * it) * Q2_QW + 32];
      A1 = mfma(a[0], b[0], A1);
      W2t[0][0] = mfma(aw[0], bw[0], W2t[0][0]);
      A1 = mfma(a[1], b[1], A1);
      W2t[0][1] = mfma(aw[0], bw[1], W2t[0][1]);
      A1 = mfma(a[2], b[2], A1);
      W2t[1][0] = mfma(aw[1], bw[0], W2t[1][0]);
      A1 = mfma(a[3], b[3], A1);
      W2t[1][1] = mfma(aw[1], bw[1], W2t[1][1]);
    }
    // ReLU mask -> dz1 (in registers), its column sum, and dW1 from it: MFMA
    // k-step s pairs accumulator row (s, lk) with that row of x
    float z[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = 32 * rh + (r & 3) + 8 * (r >> 2) + 4 * lk;
      z[r] = L.h1[rl * Q2_QW + 32 * ib + li] > 0.f ? A1[r] : 0.f;
      acc_db1 += (double)z[r];
    }
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      if (db < ndb) {
        const int dcol = 32 * db + li;
        const bool okd = dcol < XL;
        const int dc = okd ? dcol : 0;
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const int rl = 32 * rh + (s & 3) + 8 * (s >> 2) + 4 * lk;
          const float xval = L.x[rl * XL + dc];
          W1[db] = mfma(z[s], okd ? xval : 0.f, W1[db]);
        }
      }
    }
    __syncthreads();  // the next stage overwrites dz2 / h1 / x
  }

  // ---- epilogue: partial of this 256-row block (index p)
  const int64_t pc = p * d.C + c;
  float* scr = L.dz;                                // dW1 of the rh = 1 waves
  double* dscr = reinterpret_cast<double*>(L.w2);   // [4 waves][64] x {db2, dW3}
  double* dscr1 = reinterpret_cast<double*>(L.h1);  // db1 of the rh = 1 waves
  dscr[(w * 64 + lane) * 2 + 0] = acc_db2;
  dscr[(w * 64 + lane) * 2 + 1] = acc_dw3;
  if (lane == 0) dscr[512 + w] = acc_db3;
  if (rh == 1) {
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) scr[((ib * 2 + db) * 16 + r) * 64 + lane] = W1[db][r];
    dscr1[ib * 64 + lane] = acc_db1;
  }
  {
    float* dW2 = d.dW2 + pc * (Q2_H * Q2_H);
#pragma unroll
    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
      for (int bb = 0; bb < 2; ++bb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int o = 64 * w + 32 * ob + (r & 3) + 8 * (r >> 2) + 4 * lk;
          dW2[o * Q2_H + i0 + 32 * bb + li] = W2t[ob][bb][r];
        }
  }
  __syncthreads();
  if (rh == 0) {
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      if (db < ndb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float v = W1[db][r] + scr[((ib * 2 + db) * 16 + r) * 64 + lane];
          const int i = 32 * ib + (r & 3) + 8 * (r >> 2) + 4 * lk;
          const int dcol = 32 * db + li;
          if (dcol < nin) d.dW1[(pc * Q2_H + i0 + i) * nin + dcol] = v;
        }
      }
    }
    // column 32 ib + li: (rh 0 + rh 1) per row half, then the two halves
    double s1 = acc_db1 + dscr1[ib * 64 + lane];
    s1 += __shfl_xor(s1, 32, 64);
    if (lk == 0) d.db1[pc * Q2_H + i0 + 32 * ib + li] = (float)s1;
  }
  if (t < 64) {
    double s2 = 0.0, s3 = 0.0;
    for (int v = 0; v < 4; ++v) {
      s2 += dscr[(v * 64 + t) * 2 + 0];
      s3 += dscr[(v * 64 + t) * 2 + 1];
    }
    d.db2[pc * Q2_H + i0 + t] = (float)s2;
    d.dW3[pc * Q2_H + i0 + t] = (float)s3;
  } else if (t == 64 && q == 0) {
    double s = 0.0;
    for (int v = 0; v < 4; ++v) s += dscr[512 + v];
    d.db3[pc] = (float)s;
  }
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_q2_bwd(const d3a_q2_bwd_desc* dp, void* stream) {
  D3A_CHECK_ARG(dp, "d3a_q2_bwd: null desc");
  const d3a_q2_bwd_desc& d = *dp;
  D3A_CHECK_ARG(d.x && d.h1 && d.h2 && d.g && d.W2 && d.w3, "d3a_q2_bwd: null input");
  D3A_CHECK_ARG(d.dW1 && d.db1 && d.dW2 && d.db2 && d.dW3 && d.db3, "d3a_q2_bwd: null output");
  D3A_CHECK_ARG(d.n_in >= 1 && d.n_in <= Q2_XMAX, "d3a_q2_bwd: n_in must be 1..48");
  D3A_CHECK_ARG(d.C >= 1 && d.rows >= 0 && d.n_scaled >= 0, "d3a_q2_bwd: bad sizes");
  // float4 loads of h1, x and W2 rows
  auto a16 = [](const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; };
  D3A_CHECK_ARG(a16(d.h1) && a16(d.h2) && d.ldh == Q2_H && d.sh % 4 == 0,
                "d3a_q2_bwd: h1 / h2 must be 16-byte aligned rows of 256 floats");
  D3A_CHECK_ARG(a16(d.x) && d.ldx % 4 == 0 && d.ldx >= ((d.n_in + 3) & ~3) && d.sxb % 4 == 0,
                "d3a_q2_bwd: x rows must be 16-byte aligned with ldx >= n_in rounded to 4");
  D3A_CHECK_ARG(a16(d.W2) && d.sW2 % 4 == 0, "d3a_q2_bwd: W2 must be 16-byte aligned");
  D3A_CHECK_ARG(d.rows * (d.ldh > d.ldx ? d.ldh : d.ldx) < (int64_t(1) << 31),
                "d3a_q2_bwd: rows x row stride exceeds 2^31");
  if (d.rows == 0) return 0;
  const int64_t units = ((d.rows + Q2_RB - 1) / Q2_RB) * d.C;
  const int64_t blocks = (units + 7) / 8 * 32;
  D3A_CHECK_ARG(blocks < (int64_t(1) << 31), "d3a_q2_bwd: too many rows");
  const int xl = (d.n_in + 3) & ~3;
  const dim3 grid((unsigned)blocks), block(Q2_NT);
  if (xl <= 16)
    hipLaunchKernelGGL(q2_bwd_kernel<16>, grid, block, 0, (hipStream_t)stream, d);
  else if (xl <= 32)
    hipLaunchKernelGGL(q2_bwd_kernel<32>, grid, block, 0, (hipStream_t)stream, d);
  else
    hipLaunchKernelGGL(q2_bwd_kernel<48>, grid, block, 0, (hipStream_t)stream, d);
  D3A_LAUNCH_CHECK("d3a_q2_bwd");
  return 0;
}
