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
// units) of layer 1 and walks its rows in 32-row sub-blocks through LDS tiles
// (dz2 32 x 256 generated from h2, double-buffered; h1[:, quarter] and x,
// triple-buffered).  Eight waves, two per SIMD, split by role so each SIMD
// holds one wave of each (waves w and w + 4 share a SIMD):
//   waves 0-3  dh1 (32 rows x units 32 (w & 1)..) over half of K (o in
//              128 (w >> 1)..), with their W2 slice held in registers; the
//              half-K partials meet in LDS and the w < 2 waves apply the ReLU
//              mask and form the first layer's dW1 / db1 from the masked tile
//              (one sub-block later, overlapping the next sub-block's MFMAs)
//   waves 4-7  dW2[64 (w - 4) .. + 63][quarter] += dz2^T h1[:, quarter]
//              (K = 32 rows; four 32 x 32 accumulators)
// 64 MFMAs per wave per sub-block.  While a sub-block is multiplied, every
// wave also stages the next one into the other buffers (from registers loaded
// one sub-block earlier) and issues the loads of the one after, spread over
// the MFMA loop, so the matrix pipe is not idle while tiles are built; one
// barrier per sub-block.  Gradients leave as one partial per 256-row block
// (the optimiser sums them in order, like split-K partials); every other
// reduction is in a fixed order, so the result is run-to-run bit-identical.
// MFMA: v_mfma_f32_32x32x2_f32 (exact fp32), operands from LDS with
// conflict-free strides (dz2 rows 257 floats apart: its rows and its columns
// are both read as 32 consecutive banks).
#include <cstdlib>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int Q2_H = 256;    // hidden width
constexpr int Q2_SB = 32;    // rows per LDS sub-block
constexpr int Q2_NSB8 = 8;   // sub-blocks per workgroup: 256 rows (one gradient partial)
constexpr int Q2_QW = 64;    // layer-1 units per workgroup
constexpr int Q2_LDZ = 257;  // dz2 row stride
constexpr int Q2_NT = 512;   // threads: eight waves, two per SIMD

template <int XL>
struct Q2Lds {
  float dz[2][Q2_SB * Q2_LDZ];      // dz2[r][o]
  float h1[3][Q2_SB * Q2_QW];       // h1[r][i0 + i]
  float x[3][Q2_SB * XL];           // x[r][d]
  float ex[2][2 * 16 * 64];         // dh1 half-K partials of waves 2, 3
};

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// A value of the policy head given as np partial sums (cql.hip's head_val:
// parts summed in order)
__device__ __forceinline__ float head_part_sum(const float* h, int64_t sp, int np, int64_t j) {
  if (np == D3A_MLP_PARTS) {
    const float a = h[j], b = h[sp + j], c = h[2 * sp + j], e = h[3 * sp + j];
    return ((a + b) + c) + e;
  }
  float v = h[j];
  for (int p = 1; p < np; ++p) v += h[p * sp + j];
  return v;
}

// XL: the first layer's input width rounded up to 4 (16, 32 or 48), fixed at
// compile time so the LDS addresses of the x operand are immediates
// NOSTAGE (timing probe only, tools/bench_q2.py --probe): the sub-block
// staging and loads are skipped, every sub-block reuses the first one's tiles
// NSB: 32-row sub-blocks per workgroup (8: 256-row partials; 1: 32-row
// partials for passes of a few hundred rows, e.g. the K2 policy's 256)
// DZIN: dz2 is given (d.dz2, already masked: a caller's head kernel formed
// it, e.g. d3a_sac_actor_head for the policy) instead of generated from g, w3
// and h2; no head gradients
// HEADIN (with DZIN, one 32-row sub-block): the SAC / CQL actor head itself
// (d3a_sac_actor_head's dq_min arithmetic, descriptor hd) runs in this
// launch's prologue: each workgroup forms dhead of its 32 rows and their dz2
// from it (the same fma order: bitwise the head kernel's dz), quarter-0
// workgroups write dhead and the head's per-row weight / bias partials, and
// workgroup 0 the actor-loss metric -- one launch fewer in the actor phase
template <int XL, bool NOSTAGE = false, int Q2_NSB = Q2_NSB8, bool DZIN = false, bool HEADIN = false>
__global__ __launch_bounds__(Q2_NT) void q2_bwd_kernel(d3a_q2_bwd_desc d, d3a_sac_actor_head_desc hd) {
  constexpr int Q2_RB = Q2_NSB * Q2_SB;
  static_assert(!HEADIN || (DZIN && Q2_NSB == 1), "HEADIN is the one-sub-block dz2 instantiation");
  __shared__ __attribute__((aligned(16))) Q2Lds<XL> L;
  __shared__ float sdh[HEADIN ? Q2_SB : 1][HEADIN ? 33 : 1];  // dhead rows [row][2A]
  __shared__ float hscr[HEADIN ? Q2_NT / 64 : 1];
  static_assert(sizeof(Q2Lds<XL>) <= 163840, "LDS");
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
  // DZIN: h2g walks dz2 (same [rows][256] row layout), gg unused
  const float* h2g = HEADIN ? nullptr : DZIN ? d.dz2 + c * d.sdz : d.h2 + c * d.sh;
  const float* gg = DZIN ? nullptr : d.g + c * d.sgb;
  const float* xg = d.x + c * d.sxb;
  const float* W2g = d.W2 + c * d.sW2;
  const float* w3g = DZIN ? nullptr : d.w3 + c * d.sw3;
  const float gs = d.gscale ? *d.gscale : 1.f;
  const int i0 = q * Q2_QW;
  const int nin = d.n_in, xr4 = (nin + 3) / 4;  // float4 pieces of an x row
  // x rows as 16-byte pieces, or (ldx % 4 != 0) element by element
  // (the 256-row critic instantiation is always handed padded rows: checked)
  const bool xal = !DZIN || ((reinterpret_cast<uintptr_t>(d.x) | (uintptr_t)(d.ldx * 4) |
                              (uintptr_t)(d.sxb * 4)) & 15) == 0;
  constexpr int x4 = XL / 4;
  const int64_t rlast = rows - 1;
  const bool role_dx = w < 4;
  const int ib = w & 1, kh = (w >> 1) & 1;  // dX waves: unit block, K half
  const int ob0 = 64 * (w - 4);             // dW2 waves: o block

  if constexpr (HEADIN) {
    const int A = hd.A, Cq = hd.C;
    const int np = hd.dq_min ? hd.n_part : 1;
    const int hp = hd.head_parts > 1 ? hd.head_parts : 1;
    const float et = hd.scalars[0];
    auto qv = [&](int cc, int64_t r) {
      float v = hd.q[cc * hd.sqc + r];
      for (int pp = 1; pp < np; ++pp) v += hd.q[pp * hd.sq_part + cc * hd.sqc + r];
      return v;
    };
    if (t < Q2_SB * A) {
      const int rl = t / A, j = t - rl * A;
      const int64_t b = rb0 + rl;
      float dmu = 0.f, dls = 0.f;
      if (b < rows) {
        // backward of min over the members (the first of least q), parts in order
        int arg = 0;
        float mn = qv(0, b);
        for (int cc = 1; cc < Cq; ++cc) {
          const float v = qv(cc, b);
          if (v < mn) { mn = v; arg = cc; }
        }
        const float* jp = hd.dq_da + arg * hd.sda_c + b * hd.ld_da + hd.da_off + j;
        float jv = jp[0];
        for (int pp = 1; pp < np; ++pp) jv += jp[pp * hd.sda_part];
        const float da = hd.dq_scale * jv;
        const float dlogp = et / (float)hd.B;
        const float* hrow = hd.head + b * 2 * A;
        const float mu = head_part_sum(hrow, hd.s_head_part, hp, j);
        const float lsr = head_part_sum(hrow, hd.s_head_part, hp, A + j);
        const float l = fminf(fmaxf(lsr, hd.min_logstd), hd.max_logstd);
        const float sd = expf(l);
        const float u = hd.u[b * A + j];
        const float e = hd.eps[b * A + j];
        const float th = tanhf(u);
        const float dm = u - mu;
        const float var = sd * sd;
        const float dlp_du = -dm / var + 2.f - 4.f * sigmoidf_t(-2.f * u);
        const float du = da * (1.f - th * th) + dlogp * dlp_du;
        dmu = du + dlogp * (dm / var);
        const float dsd = du * e + dlogp * ((dm * dm) / (var * sd) - 1.f / sd);
        const bool pass = (lsr >= hd.min_logstd) && (lsr <= hd.max_logstd);
        dls = pass ? dsd * sd : 0.f;
        if (q == 0) {
          hd.dhead[b * 2 * A + j] = dmu;
          hd.dhead[b * 2 * A + A + j] = dls;
          if (hd.db_part) {
            hd.db_part[b * 2 * A + j] = dmu;
            hd.db_part[b * 2 * A + A + j] = dls;
          }
        }
      }
      sdh[rl][j] = dmu;
      sdh[rl][A + j] = dls;
    }
    if (q == 0 && p == 0) {
      // the actor loss mean(exp(log_temp) * logp - min_c Q) (the head kernel's
      // last workgroup: rows strided by 256, the same block sum -- waves 4..7
      // add zeros)
      float lsum = 0.f;
      if (t < 256) {
        for (int64_t r = t; r < hd.B; r += 256) {
          float qmin = qv(0, r);
          for (int cc = 1; cc < Cq; ++cc) qmin = fminf(qmin, qv(cc, r));
          lsum += et * hd.logp[r] - qmin;
        }
      }
      const float tot = block_sum(lsum, hscr);
      if (t == 0) hd.metrics[5] = tot / (float)hd.B;
    }
    __syncthreads();  // dhead rows in LDS
    if (q == 0 && hd.dW_part) {
      // the head's per-row weight partials dW[k][n] = dhead[k] h[n], n = t & 255
      const int n = t & (Q2_H - 1);
      for (int rl = t >> 8; rl < Q2_SB; rl += Q2_NT / Q2_H) {
        const int64_t b = rb0 + rl;
        if (b >= rows) continue;
        const float hv = hd.h[b * hd.ldh + n];
        float* pw = hd.dW_part + b * 2 * A * hd.H + n;
        for (int k = 0; k < 2 * A; ++k) pw[(int64_t)k * hd.H] = sdh[rl][k] * hv;
      }
    }
  }

  float w3v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) w3v[j] = DZIN ? 0.f : w3g[lane + 64 * j];

  // ---- staging registers of one sub-block (unconditional loads, clamped
  // rows; validity applied when staged).  Thread (w, lane): h2 rows w + 8s
  // (s < 4), columns lane + 64j; one float4 piece of h1 and of x
  float hv[4][4], gv[4], h1v[4], xv[4];
  auto load_row = [&](int sb, int s) {
    int64_t r = rb0 + sb * Q2_SB + w + 8 * s;
    r = r < rlast ? r : rlast;
    gv[s] = DZIN ? 0.f : gg[r];
    if constexpr (HEADIN) {
      // dz2[r][n] = (sum_k dhead[r][k] w_head[k][n]) * [h[r][n] > 0], the head
      // kernel's fma order (rows past the end: staged as zero later)
      const int rl = (int)(r - rb0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = lane + 64 * j;
        float v = 0.f;
        for (int k = 0; k < 2 * hd.A; ++k) v = fmaf(sdh[rl][k], hd.w_head[(int64_t)k * hd.H + n], v);
        hv[s][j] = hd.h[r * hd.ldh + n] > 0.f ? v : 0.f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) hv[s][j] = h2g[(int)r * ldh + lane + 64 * j];
    }
  };
  auto load_tiles = [&](int sb) {
    const int64_t base = rb0 + sb * Q2_SB;
    {
      int64_t r = base + (t >> 4);
      r = r < rlast ? r : rlast;
      const float4 a = *reinterpret_cast<const float4*>(h1g + (int)r * ldh + i0 + (t & 15) * 4);
      h1v[0] = a.x; h1v[1] = a.y; h1v[2] = a.z; h1v[3] = a.w;
    }
    {
      const int ix = t < Q2_SB * x4 ? t : Q2_SB * x4 - 1;
      int64_t rx = base + ix / x4;
      rx = rx < rlast ? rx : rlast;
      const int cx = ix % x4 < xr4 ? ix % x4 : 0;  // pieces past n_in: staged as 0
      const float* px = xg + (int)rx * ldx + cx * 4;
      if (xal) {
        const float4 a = *reinterpret_cast<const float4*>(px);
        xv[0] = a.x; xv[1] = a.y; xv[2] = a.z; xv[3] = a.w;
      } else {  // unpadded rows (e.g. the policy's [obs; next_obs], ldx = n_in)
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[e] = cx * 4 + e < nin ? px[e] : 0.f;
      }
    }
  };

  // fp64 running sums: db2 / dW3 of column i0 + lane (every thread), db3
  // (lane 0 of each wave), db1 of a w < 2 wave's column
  double acc_db2 = 0.0, acc_dw3 = 0.0, acc_db3 = 0.0, acc_db1 = 0.0;
  auto stage_row = [&](int sb, int s) {
    const int buf = sb & 1;
    const int rl = w + 8 * s;
    const int64_t r = rb0 + sb * Q2_SB + rl;
    const bool ok = r < rows && sb < Q2_NSB;  // (the loop's one-past-the-end stage is all zero)
    float gp = gv[s];
    if (r < d.n_scaled) gp *= gs;  // as d3a_head1_bwd forms g'
    if (!ok) gp = 0.f;
    float hq = 0.f, dq = 0.f;  // this workgroup's quarter column (j == q)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float hval = ok ? hv[s][j] : 0.f;
      const float dzv = DZIN ? hval : (hval > 0.f ? gp * w3v[j] : 0.f);
      L.dz[buf][rl * Q2_LDZ + lane + 64 * j] = dzv;
      hq = j == q ? hval : hq;
      dq = j == q ? dzv : dq;
    }
    acc_db2 += (double)dq;
    if (!DZIN) {
      acc_dw3 += (double)(gp * hq);
      if (lane == 0) acc_db3 += (double)gp;
    }
  };
  auto stage_tiles = [&](int sb) {
    const int buf = sb % 3;
    const int64_t base = rb0 + sb * Q2_SB;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    const int rl = t >> 4;
    *reinterpret_cast<float4*>(&L.h1[buf][rl * Q2_QW + (t & 15) * 4]) =
        (base + rl < rows && sb < Q2_NSB) ? make_float4(h1v[0], h1v[1], h1v[2], h1v[3]) : z;
    if (t < Q2_SB * x4) {
      const int rx = t / x4;
      *reinterpret_cast<float4*>(&L.x[buf][rx * XL + (t % x4) * 4]) =
          (base + rx < rows && sb < Q2_NSB && t % x4 < xr4) ? make_float4(xv[0], xv[1], xv[2], xv[3]) : z;
    }
  };
  // pipelined staging step it < 8 of sub-block sb's MFMA loop: the next
  // sub-block's rows / tiles staged from registers, the registers reloaded
  // with the sub-block after it
  // Branch-free, so the wait-count pass sees the same straight-line
  // schedule every iteration: past the end a zero sub-block is staged into a
  // free buffer and the last one is reloaded (both unused).
  auto pipe = [&](int sb, int it) {
    if constexpr (NOSTAGE) return;
    const int ld = sb + 2 < Q2_NSB ? sb + 2 : Q2_NSB - 1;
    if (it < 4) {
      stage_row(sb + 1, it);
      load_row(ld, it);
    } else if (it == 4) {
      stage_tiles(sb + 1);
      load_tiles(ld);
    }
  };

  constexpr int ndb = XL > 32 ? 2 : 1;  // 32-wide input blocks of dW1 (n_in <= XL)
  const int64_t pc = p * d.C + c;   // this workgroup's partial index

  // prologue: sub-block 0 staged, sub-block 1 in registers
#pragma unroll
  for (int s = 0; s < 4; ++s) load_row(0, s);
  load_tiles(0);
#pragma unroll
  for (int s = 0; s < 4; ++s) stage_row(0, s);
  stage_tiles(0);
#pragma unroll
  for (int s = 0; s < 4; ++s) load_row(1, s);
  load_tiles(1);
  __syncthreads();

  // The two roles run separate loops (same barrier count: one per sub-block),
  // so their register sets do not have to coexist.
  f32x16 W1[2];  // dX waves: dW1 over the rows they finish (input blocks 0, 1)
  if (role_dx) {
    // W2 operand in registers, B[k = o][n = unit] of the 64 k-steps of this
    // wave's K half (lane: o = 128 kh + 2 s + lk, unit 32 ib + li)
    float wreg[64];
#pragma unroll
    for (int s = 0; s < 64; ++s)
      wreg[s] = W2g[(128 * kh + 2 * s + lk) * Q2_H + i0 + 32 * ib + li];
    // dh1 half-K partials of this and of the previous sub-block; dW1 over the
    // rows this wave finishes (accumulator registers 8 kh .. 8 kh + 7 of
    // every sub-block; the partner wave (kh ^ 1) finishes the others)
    f32x16 acc, accp;
#pragma unroll
    for (int r = 0; r < 16; ++r) W1[0][r] = W1[1][r] = accp[r] = 0.f;
    float z[8];
#pragma unroll
    for (int r2 = 0; r2 < 8; ++r2) z[r2] = 0.f;  // sub-block -1: nothing to add
    // the masked dh1 of sub-block sb's rows this wave finishes: its own half-K
    // partial (accp) and the partner's from LDS, o < 128 first (fixed order)
    auto mask = [&](int sb) {
      const int eb = sb & 1, tb = sb % 3;
#pragma unroll
      for (int r2 = 0; r2 < 8; ++r2) {
        const int r = 8 * kh + r2;
        const int rl = (r & 3) + 8 * (r >> 2) + 4 * lk;
        const float o = L.ex[eb][((ib * 2 + (kh ^ 1)) * 8 + r2) * 64 + lane];
        const float v = kh == 0 ? __fadd_rn(accp[r], o) : __fadd_rn(o, accp[r]);
        z[r2] = L.h1[tb][rl * Q2_QW + 32 * ib + li] > 0.f ? v : 0.f;
        acc_db1 += (double)z[r2];
      }
    };
    // dW1 k-step r2 of sub-block sb: accumulator row (8 kh + r2, lk) x that row of x
    auto w1step = [&](int sb, int r2) {
      const int tb = sb % 3;
      const int r = 8 * kh + r2;
      const int rl = (r & 3) + 8 * (r >> 2) + 4 * lk;
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        if (db < ndb) {
          const int dcol = 32 * db + li;
          const bool okd = dcol < XL;
          const float xval = L.x[tb][rl * XL + (okd ? dcol : 0)];
          W1[db] = mfma(z[r2], okd ? xval : 0.f, W1[db]);
        }
      }
    };
#pragma unroll 1
    for (int sb = 0; sb < Q2_NSB; ++sb) {
      const int cb = sb & 1;
      if (sb > 0) mask(sb - 1);  // the previous sub-block's partials met at the barrier
      // two independent accumulation chains (even / odd k-steps), summed at
      // the end of the sub-block: more MFMA issue freedom beside the partner wave
      f32x16 acc1;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = acc1[r] = 0.f;
      // dh1 half-K: A = dz2[row li][o = 128 kh + 2 s + lk], B = wreg[s]; the
      // previous sub-block's dW1 k-steps ride along (independent accumulators)
      const float* A = &L.dz[cb][li * Q2_LDZ + 128 * kh + lk];
      // operand reads one step ahead of their MFMAs
      float a[2][8];
#pragma unroll
      for (int e = 0; e < 8; ++e) a[0][e] = A[2 * e];
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        if (it + 1 < 8) {
#pragma unroll
          for (int e = 0; e < 8; ++e) a[(it + 1) & 1][e] = A[16 * (it + 1) + 2 * e];
        }
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          acc = mfma(a[it & 1][e], wreg[8 * it + e], acc);
          acc1 = mfma(a[it & 1][e + 1], wreg[8 * it + e + 1], acc1);
        }
        w1step(sb > 0 ? sb - 1 : 0, it);  // z = 0 at sb = 0: adds nothing
        pipe(sb, it);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = __fadd_rn(acc[r], acc1[r]);
      // the half of this partial the partner finishes, to LDS
#pragma unroll
      for (int r2 = 0; r2 < 8; ++r2)
        L.ex[cb][((ib * 2 + kh) * 8 + r2) * 64 + lane] = acc[8 * (kh ^ 1) + r2];
      accp = acc;
      __syncthreads();  // sub-block sb + 1 staged; sb's half-K partials in LDS
    }
    mask(Q2_NSB - 1);
#pragma unroll
    for (int it = 0; it < 8; ++it) w1step(Q2_NSB - 1, it);
  } else {
    f32x16 R[4];  // dW2 tiles R[2 ob + bb]: o block ob0 + 32 ob, unit block 32 bb
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) R[k][r] = 0.f;
#pragma unroll 1
    for (int sb = 0; sb < Q2_NSB; ++sb) {
      const int cb = sb & 1;
      // dW2[o block][quarter] += dz2[rows][o]^T h1[rows][quarter], K = 32 rows
      const float* A = &L.dz[cb][lk * Q2_LDZ + ob0 + li];
      const float* B = &L.h1[sb % 3][lk * Q2_QW + li];
      // operand reads one step ahead of their MFMAs
      float a[2][2][2], b[2][2][2];
      auto rd = [&](int it, int buf) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          a[buf][e][0] = A[(4 * it + 2 * e) * Q2_LDZ];
          a[buf][e][1] = A[(4 * it + 2 * e) * Q2_LDZ + 32];
          b[buf][e][0] = B[(4 * it + 2 * e) * Q2_QW];
          b[buf][e][1] = B[(4 * it + 2 * e) * Q2_QW + 32];
        }
      };
      rd(0, 0);
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        if (it + 1 < 8) rd(it + 1, (it + 1) & 1);
        const int u = it & 1;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          R[0] = mfma(a[u][e][0], b[u][e][0], R[0]);
          R[1] = mfma(a[u][e][0], b[u][e][1], R[1]);
          R[2] = mfma(a[u][e][1], b[u][e][0], R[2]);
          R[3] = mfma(a[u][e][1], b[u][e][1], R[3]);
        }
        pipe(sb, it);
      }
      __syncthreads();  // sub-block sb + 1 staged
    }
    float* dW2 = d.dW2 + pc * (Q2_H * Q2_H);
#pragma unroll
    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
      for (int bb = 0; bb < 2; ++bb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int o = ob0 + 32 * ob + (r & 3) + 8 * (r >> 2) + 4 * lk;
          dW2[o * Q2_H + i0 + 32 * bb + li] = R[2 * ob + bb][r];
        }
  }

  // ---- epilogue (after the loops' last barrier every LDS tile is free):
  // dW1 / db1 halves of the two K-half waves summed kh 0 first; the head's and
  // layer 2's bias / weight partials summed over the waves in order (fp64)
  float* w1s = &L.dz[0][0];                                  // [ib][db][16][64]
  double* db1s = reinterpret_cast<double*>(&L.dz[0][0] + 4096);  // [ib][64]
  double* dscr = reinterpret_cast<double*>(&L.dz[1][0]);     // [8 waves][64] x 2
  if (role_dx && kh == 1) {
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) w1s[((ib * 2 + db) * 16 + r) * 64 + lane] = W1[db][r];
    db1s[ib * 64 + lane] = acc_db1;
  }
  dscr[(w * 64 + lane) * 2 + 0] = acc_db2;
  dscr[(w * 64 + lane) * 2 + 1] = acc_dw3;
  if (lane == 0) dscr[1024 + w] = acc_db3;
  __syncthreads();
  if (role_dx && kh == 0) {
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      if (db < ndb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float v = __fadd_rn(W1[db][r], w1s[((ib * 2 + db) * 16 + r) * 64 + lane]);
          const int i = 32 * ib + (r & 3) + 8 * (r >> 2) + 4 * lk;
          const int dcol = 32 * db + li;
          if (dcol < nin) d.dW1[(pc * Q2_H + i0 + i) * nin + dcol] = v;
        }
      }
    }
    // column 32 ib + li: (kh 0 + kh 1) per row group, then the two row groups
    double s1 = acc_db1 + db1s[ib * 64 + lane];
    s1 += __shfl_xor(s1, 32, 64);
    if (lk == 0) d.db1[pc * Q2_H + i0 + 32 * ib + li] = (float)s1;
  }
  if (t >= 256 && t < 320) {  // a dW2 wave: the column sums
    const int tt = t - 256;
    double s2 = 0.0, s3 = 0.0;
    for (int v = 0; v < 8; ++v) {
      s2 += dscr[(v * 64 + tt) * 2 + 0];
      s3 += dscr[(v * 64 + tt) * 2 + 1];
    }
    d.db2[pc * Q2_H + i0 + tt] = (float)s2;
    if (!DZIN) d.dW3[pc * Q2_H + i0 + tt] = (float)s3;
  } else if (!DZIN && t == 320 && q == 0) {
    double sg = 0.0;
    for (int v = 0; v < 8; ++v) sg += dscr[1024 + v];
    d.db3[pc] = (float)sg;
  }
}

}  // namespace
}  // namespace d3a

using namespace d3a;

namespace d3a {
int q2_bwd_launch(const d3a_q2_bwd_desc& d, const d3a_sac_actor_head_desc* head, void* stream);
}

extern "C" int d3a_q2_bwd(const d3a_q2_bwd_desc* dp, void* stream) {
  D3A_CHECK_ARG(dp, "d3a_q2_bwd: null desc");
  const d3a_q2_bwd_desc& d = *dp;
  D3A_CHECK_ARG(d.m2 == nullptr, "d3a_q2_bwd: the mask image is d3a_q2_bwd_x6 only");
  const bool dzin = d.dz2 != nullptr;
  D3A_CHECK_ARG(d.x && d.h1 && d.W2 && (dzin || (d.h2 && d.g && d.w3)), "d3a_q2_bwd: null input");
  D3A_CHECK_ARG(d.dW1 && d.db1 && d.dW2 && d.db2 && (dzin || (d.dW3 && d.db3)),
                "d3a_q2_bwd: null output");
  D3A_CHECK_ARG(d.block_rows == 0 || d.block_rows == 256 || (d.block_rows == 32 && dzin),
                "d3a_q2_bwd: block_rows must be 0 / 256, or 32 with dz2");
  D3A_CHECK_ARG(!dzin || (d.block_rows == 32), "d3a_q2_bwd: dz2 needs block_rows 32");
  D3A_CHECK_ARG(d.n_in >= 1 && d.n_in <= 48, "d3a_q2_bwd: n_in must be 1..48");
  D3A_CHECK_ARG(d.C >= 1 && d.rows >= 0 && d.n_scaled >= 0, "d3a_q2_bwd: bad sizes");
  // float4 loads of h1, x and W2 rows
  auto a16 = [](const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; };
  D3A_CHECK_ARG(a16(d.h1) && (dzin || a16(d.h2)) && d.ldh == Q2_H && d.sh % 4 == 0,
                "d3a_q2_bwd: h1 / h2 must be 16-byte aligned rows of 256 floats");
  D3A_CHECK_ARG(!dzin || (a16(d.dz2) && d.sdz % 4 == 0),
                "d3a_q2_bwd: dz2 must be 16-byte aligned rows of 256 floats");
  D3A_CHECK_ARG(d.ldx >= d.n_in, "d3a_q2_bwd: ldx < n_in");
  D3A_CHECK_ARG(dzin || (a16(d.x) && d.ldx % 4 == 0 && d.sxb % 4 == 0),
                "d3a_q2_bwd: x rows must be 16-byte aligned with ldx % 4 == 0 (without dz2)");
  D3A_CHECK_ARG(a16(d.W2) && d.sW2 % 4 == 0, "d3a_q2_bwd: W2 must be 16-byte aligned");
  D3A_CHECK_ARG(d.rows * (d.ldh > d.ldx ? d.ldh : d.ldx) < (int64_t(1) << 31),
                "d3a_q2_bwd: rows x row stride exceeds 2^31");
  if (d.rows == 0) return 0;
  return q2_bwd_launch(d, nullptr, stream);
}

// The policy trunk backward with the SAC actor head in its prologue: the
// work of d3a_sac_actor_head (dq_min form, dz not written) followed by
// d3a_q2_bwd with dz2, in one launch -- the same dhead, head partials, metric
// and trunk gradients bit for bit
extern "C" int d3a_q2_bwd_actor_head(const d3a_q2_bwd_desc* dp, const d3a_sac_actor_head_desc* hp,
                                     void* stream) {
  D3A_CHECK_ARG(dp && hp, "d3a_q2_bwd_actor_head: null desc");
  const d3a_q2_bwd_desc& d = *dp;
  const d3a_sac_actor_head_desc& h = *hp;
  D3A_CHECK_ARG(d.m2 == nullptr && d.dz2 == nullptr,
                "d3a_q2_bwd_actor_head: dz2 is formed here (no dz2, no mask image)");
  D3A_CHECK_ARG(d.C == 1 && d.block_rows == 32, "d3a_q2_bwd_actor_head: one trunk, block_rows 32");
  D3A_CHECK_ARG(d.x && d.h1 && d.W2 && d.dW1 && d.db1 && d.dW2 && d.db2,
                "d3a_q2_bwd_actor_head: null trunk operand");
  D3A_CHECK_ARG(d.n_in >= 1 && d.n_in <= 48 && d.ldx >= d.n_in && d.rows == h.B,
                "d3a_q2_bwd_actor_head: bad sizes (n_in 1..48, rows == B)");
  auto a16 = [](const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; };
  D3A_CHECK_ARG(a16(d.h1) && d.ldh == Q2_H && a16(d.W2) && d.sW2 % 4 == 0,
                "d3a_q2_bwd_actor_head: h1 / W2 must be 16-byte aligned rows of 256 floats");
  D3A_CHECK_ARG(d.rows * (d.ldh > d.ldx ? d.ldh : d.ldx) < (int64_t(1) << 31),
                "d3a_q2_bwd_actor_head: rows x row stride exceeds 2^31");
  D3A_CHECK_ARG(h.B >= 1 && h.A >= 1 && h.A <= 16 && h.C >= 1 && h.dq_min && h.dq_da && h.q &&
                    h.n_part >= 1 && !h.dq_dz,
                "d3a_q2_bwd_actor_head: the head's dq_min form (dq_da and q in n_part parts)");
  D3A_CHECK_ARG(h.h && h.w_head && h.H == Q2_H && h.head && h.eps && h.u && h.logp && h.dhead &&
                    h.metrics && h.scalars,
                "d3a_q2_bwd_actor_head: null head operand, or H != 256");
  return q2_bwd_launch(d, &h, stream);
}

// the launch of a checked descriptor (d3a_q2_bwd, d3a_q2_bwd_actor_head)
int d3a::q2_bwd_launch(const d3a_q2_bwd_desc& d, const d3a_sac_actor_head_desc* head, void* stream) {
  const bool dzin = d.dz2 != nullptr || head != nullptr;
  const int64_t rb = dzin ? 32 : 256;
  const int64_t units = ((d.rows + rb - 1) / rb) * d.C;
  const int64_t blocks = (units + 7) / 8 * 32;
  D3A_CHECK_ARG(blocks < (int64_t(1) << 31), "d3a_q2_bwd: too many rows");
  const int xl = (d.n_in + 3) & ~3;
  const dim3 grid((unsigned)blocks), block(Q2_NT);
  const d3a_sac_actor_head_desc hz{};
  static const bool probe = [] {
    const char* e = getenv("D3A_Q2_PROBE");
    return e && e[0] == '1';
  }();
  if (probe && xl <= 16) {
    hipLaunchKernelGGL((q2_bwd_kernel<16, true>), grid, block, 0, (hipStream_t)stream, d, hz);
    D3A_LAUNCH_CHECK("d3a_q2_bwd");
    return 0;
  }
  if (head != nullptr) {
    const d3a_sac_actor_head_desc h = *head;
    if (xl <= 16)
      hipLaunchKernelGGL((q2_bwd_kernel<16, false, 1, true, true>), grid, block, 0, (hipStream_t)stream, d, h);
    else if (xl <= 32)
      hipLaunchKernelGGL((q2_bwd_kernel<32, false, 1, true, true>), grid, block, 0, (hipStream_t)stream, d, h);
    else
      hipLaunchKernelGGL((q2_bwd_kernel<48, false, 1, true, true>), grid, block, 0, (hipStream_t)stream, d, h);
    D3A_LAUNCH_CHECK("d3a_q2_bwd_actor_head");
    return 0;
  }
  if (dzin) {
    if (xl <= 16)
      hipLaunchKernelGGL((q2_bwd_kernel<16, false, 1, true>), grid, block, 0, (hipStream_t)stream, d, hz);
    else if (xl <= 32)
      hipLaunchKernelGGL((q2_bwd_kernel<32, false, 1, true>), grid, block, 0, (hipStream_t)stream, d, hz);
    else
      hipLaunchKernelGGL((q2_bwd_kernel<48, false, 1, true>), grid, block, 0, (hipStream_t)stream, d, hz);
    D3A_LAUNCH_CHECK("d3a_q2_bwd");
    return 0;
  }
  if (xl <= 16)
    hipLaunchKernelGGL(q2_bwd_kernel<16>, grid, block, 0, (hipStream_t)stream, d, hz);
  else if (xl <= 32)
    hipLaunchKernelGGL(q2_bwd_kernel<32>, grid, block, 0, (hipStream_t)stream, d, hz);
  else
    hipLaunchKernelGGL(q2_bwd_kernel<48>, grid, block, 0, (hipStream_t)stream, d, hz);
  D3A_LAUNCH_CHECK("d3a_q2_bwd");
  return 0;
}
