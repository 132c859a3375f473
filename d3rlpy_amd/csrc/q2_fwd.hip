// Forward of a two-hidden-layer, single-output Q ensemble over a large row
// pass, with the second layer's weights held in registers.
//
// The specialised instantiation of d3a_mlp_fwd (mlp_fused.hip) for the shape
// of the critic passes of the hot path,
//   VectorEncoderWithAction [n_in -> 256 -> 256]  (encoders.py:265-275, 328-339)
//   + ContinuousMeanQFunction._fc [256 -> 1]       (q_functions/mean_q_function.py:255-256),
// over thousands of rows per member (the CQL critic pass: 15,616 Q rows + 256
// target rows per member at K2).  Same contract as d3a_mlp_fwd: h[0] / h[1]
// kept for rows in [h_from, r0 + rows), out for every row, an optional aux
// pass over a second parameter buffer.
//
// Why a second kernel: the generic fused forward runs each layer of a
// 128-row block as a phase (MFMAs, barrier, epilogue to LDS, barrier, copy
// out), so the matrix pipe idles through every epilogue and operand latency --
// 52 % MFMA-busy on the K2 pass (profiles/r03_pmc_fwd.txt).  Here a workgroup
// of eight waves (one per 32 hidden units, two per SIMD) keeps W1[its 32
// units][256] in registers (128 VGPRs), computes layer 1 of all 128 rows in
// the prologue (W0 in registers, x and the result in LDS), and then runs
// layer 2 over four 32-row sub-blocks with no barrier: the epilogue of
// sub-block s - 1 (bias, ReLU, h[1] stores, head dot) and the copy-out of
// h[0] rows (whole 1 KB rows from LDS) are spread over sub-block s's MFMA
// stream.  The MFMAs compute the transposed tile C^T[unit][row] (W as the A
// operand), so a lane owns four runs of four consecutive units of one row:
// 16-byte stores and a 16-unit head dot in registers (then the two lane halves
// and the eight waves, in order).  K2 critic pass: 54.8 -> 49.9 us
// (tools/bench_fwd.py; profiles/r03_fwd_ab.jsonl).
//
// Numerics: every hidden unit is the same exact-f32 MFMA chain as the generic
// kernel (k groups of 8 in order, lane half lk taking k = 8m + 4lk + j), bias
// and ReLU after the chain; the head is an fp32 sum in a fixed order
// (deterministic, not the generic kernel's order).
#include <cstdlib>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int F_H = 256;    // hidden width
constexpr int F_RB = 128;   // rows per workgroup
constexpr int F_SB = 32;    // rows per sub-block
constexpr int F_NSB = F_RB / F_SB;
constexpr int F_LDK = 260;  // h1 row stride in LDS (conflict-free ds_read_b128 rows)

template <int XL>
struct FwdLds {
  float h[F_RB * F_LDK];  // layer-1 activations of the workgroup's rows
  union {
    float x[F_RB * (XL + 4)];  // input rows, zero-padded to XL (prologue)
    float hp[F_NSB][8][F_SB];  // head partials [sub-block][wave][row] (after)
  } u;
};

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float pick(const float4& v, int j) {
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}

// XL: n_in rounded up to 16 (16, 32 or 48) -- the layer-1 K padding of the
// generic kernel, so both run the same MFMA chain
// PROBE (timing probes only, tools/bench_fwd.py with D3A_FWD_PROBE): bit 0
// drops the kept-activation stores, bit 1 feeds layer 2 a register operand
// instead of LDS reads
template <int XL, int PROBE = 0>
__global__ __launch_bounds__(512) void q2_fwd_kernel(d3a_mlp_fwd_desc d) {
  constexpr int LDX = XL + 4;
  constexpr int NG0 = XL / 8;  // layer-1 k groups
  __shared__ __attribute__((aligned(16))) FwdLds<XL> L;
  static_assert(sizeof(FwdLds<XL>) <= 163840, "LDS");
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int li = lane & 31, lk = lane >> 5;
  const int c = blockIdx.z;
  const int nb_main = (int)((d.rows + F_RB - 1) / F_RB);
  const bool aux = (int)blockIdx.x >= nb_main;
  // row indices fit 32 bits (checked on the host)
  const int m0 = aux ? ((int)blockIdx.x - nb_main) * F_RB : (int)d.r0 + (int)blockIdx.x * F_RB;
  const int rend = aux ? (int)d.aux_rows : (int)(d.r0 + d.rows);
  const int h_from = aux ? rend : (int)d.h_from;
  const int64_t wdel = aux ? d.aux_wdelta : 0;
  float* const outp = aux ? d.aux_out + c * d.aux_sout : d.out + c * d.sout;
  const int nin = d.n_in;
  const int col = 32 * w + li;  // this lane's hidden unit (both layers)
  float* const h0g = (!aux && d.h[0] && !(PROBE & 1)) ? d.h[0] + c * d.sh : nullptr;
  float* const h1g = (!aux && d.h[1] && !(PROBE & 1)) ? d.h[1] + c * d.sh : nullptr;

  // ---- prologue: W1 / W0 to registers (W1 first: the longest latency,
  // overlapped with the x staging and layer 1), x rows to LDS
  const float* W1 = d.W[1] + wdel + c * d.sW[1];
  float w1r[128];  // step 4m + j: W1[col][8m + 4lk + j]
#pragma unroll
  for (int m = 0; m < 32; ++m) {
    const float4 v = *reinterpret_cast<const float4*>(W1 + col * F_H + 8 * m + 4 * lk);
    w1r[4 * m + 0] = v.x; w1r[4 * m + 1] = v.y; w1r[4 * m + 2] = v.z; w1r[4 * m + 3] = v.w;
  }
  const float* W0 = d.W[0] + wdel + c * d.sW[0];
  float w0r[4 * NG0];  // step 4g + j: W0[col][8g + 4lk + j] (0 past n_in)
#pragma unroll
  for (int i = 0; i < 4 * NG0; ++i) {
    const int k = 8 * (i >> 2) + 4 * lk + (i & 3);
    w0r[i] = k < nin ? W0[col * nin + k] : 0.f;
  }
  const float b2v = (d.b[2] + wdel + c * d.sb[2])[0];
  {
    const float* xb = aux ? d.aux_x + c * d.aux_sxb : d.x + c * d.sxb;
    const int64_t ldx = aux ? d.aux_ldx : d.ldx;
    constexpr int X4 = XL / 4;
    for (int e = t; e < F_RB * X4; e += 512) {
      const int m = e / X4, k4 = (e - m * X4) * 4;
      const int r = m0 + m;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < rend) {
        const float* p = xb + r * ldx + k4;
        if (k4 + 3 < nin) {
          v = make_float4(p[0], p[1], p[2], p[3]);
        } else {
          v.x = k4 + 0 < nin ? p[0] : 0.f;
          v.y = k4 + 1 < nin ? p[1] : 0.f;
          v.z = k4 + 2 < nin ? p[2] : 0.f;
        }
      }
      *reinterpret_cast<float4*>(&L.u.x[m * LDX + k4]) = v;
    }
  }
  __syncthreads();  // x staged

  // The MFMAs compute the transposed tile, C^T[unit][row] = W[unit] . act[row]
  // (W as the A operand from registers, the activation rows as B from LDS):
  // lane (li, lk) holds row li and units 32 w + 8 R + 4 lk + j of accumulator
  // element r = 4 R + j, so each lane owns four runs of four consecutive units
  // of one row -- 16-byte stores, a 16-unit head dot in registers.  The products
  // and their k order are those of the untransposed tile (bitwise the same).
  auto unit_of = [&](int R) { return 32 * w + 8 * R + 4 * lk; };
  float bb[16], ww[16];  // layer-1 bias / head weights of this lane's units
  auto load_units = [&](const float* src, float* dst) {
#pragma unroll
    for (int R = 0; R < 4; ++R) {
      const float4 v = *reinterpret_cast<const float4*>(src + unit_of(R));
      dst[4 * R] = v.x; dst[4 * R + 1] = v.y; dst[4 * R + 2] = v.z; dst[4 * R + 3] = v.w;
    }
  };
  // row rb + li kept in h[l]
  auto kept = [&](const float* base, int rb) {
    const int row = rb + li;
    return base != nullptr && row >= h_from && row < rend;
  };
  // ---- layer 1 over the four 32-row tiles: this wave's 32 units, to LDS
  // (and, rows kept, to h[0])
  load_units(d.b[0] + wdel + c * d.sb[0], bb);
#pragma unroll 1
  for (int tt = 0; tt < F_NSB; ++tt) {
    f32x16 a0;
#pragma unroll
    for (int r = 0; r < 16; ++r) a0[r] = 0.f;
    float4 xo[NG0];
#pragma unroll
    for (int g = 0; g < NG0; ++g)
      xo[g] = *reinterpret_cast<const float4*>(&L.u.x[(tt * F_SB + li) * LDX + 8 * g + 4 * lk]);
#pragma unroll
    for (int i = 0; i < 4 * NG0; ++i) a0 = mfma(w0r[i], pick(xo[i >> 2], i & 3), a0);
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = fmaxf(a0[r] + bb[r], 0.f);
    float* hl = &L.h[(tt * F_SB + li) * F_LDK];
#pragma unroll
    for (int R = 0; R < 4; ++R)
      *reinterpret_cast<float4*>(hl + unit_of(R)) =
          make_float4(v[4 * R], v[4 * R + 1], v[4 * R + 2], v[4 * R + 3]);
  }
  load_units(d.b[1] + wdel + c * d.sb[1], bb);
  load_units(d.W[2] + wdel + c * d.sW[2], ww);
  __syncthreads();  // h1 of every row in LDS; x dead (hp aliases it)

  // ---- layer 2, sub-block by sub-block with no barrier.  Spread over each
  // sub-block's MFMA stream: the previous sub-block's epilogue (bias, ReLU,
  // kept rows to h[1], the head dot of the lane's 16 units in order) and four
  // rows of h[0] copied out of LDS (wave w: rows 16 w .. 16 w + 15, one whole
  // 1 KB row per instruction).  The last sub-block's epilogue drains alone.
  f32x16 accp;
#pragma unroll
  for (int r = 0; r < 16; ++r) accp[r] = 0.f;
  bool kp = false;  // row rbp + li of the previous sub-block kept in h[1]
  int rbp = 0;
  float hs = 0.f;
  auto epi_at = [&](int m) {
    if (m < 16) {
      accp[m] = fmaxf(accp[m] + bb[m], 0.f);
      if ((m & 3) == 3 && kp) {
        const int R = m >> 2;
        *reinterpret_cast<float4*>(h1g + (rbp + li) * F_H + unit_of(R)) =
            make_float4(accp[m - 3], accp[m - 2], accp[m - 1], accp[m]);
      }
    } else {
      const int r = m - 16;
      hs = r == 0 ? accp[0] * ww[0] : fmaf(accp[r], ww[r], hs);
    }
  };
  auto head_part = [&](int sp) {  // the two lane halves, to LDS per wave
    const float o = __shfl_xor(hs, 32, 64);
    if (lk == 0) L.u.hp[sp][w][li] = hs + o;
  };
  // (read from LDS two groups before the store, so the store's wait is on
  // that read only, not on the operand prefetches behind it)
  float4 hc;
  auto h0_read = [&](int j) { hc = *reinterpret_cast<const float4*>(&L.h[(16 * w + j) * F_LDK + 4 * lane]); };
  auto h0_store = [&](int j) {
    const int row = m0 + 16 * w + j;  // wave-uniform
    if (h0g && row >= h_from && row < rend)
      *reinterpret_cast<float4*>(h0g + row * F_H + 4 * lane) = hc;
  };
#pragma unroll 1
  for (int s = 0; s < F_NSB; ++s) {
    const float* Bp = &L.h[(s * F_SB + li) * F_LDK + 4 * lk];
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // operand reads two k groups ahead of their MFMAs
    float4 av[3];
    av[0] = *reinterpret_cast<const float4*>(Bp);
    av[1] = *reinterpret_cast<const float4*>(Bp + 8);
#pragma unroll
    for (int m = 0; m < 32; ++m) {
      if (!(PROBE & 2) && m + 2 < 32) av[(m + 2) % 3] = *reinterpret_cast<const float4*>(Bp + 8 * (m + 2));
      // keep the prefetch two groups ahead (the scheduler would otherwise
      // sink it next to its use and expose the LDS latency every group)
      __builtin_amdgcn_sched_barrier(0);
      const float4 a = (PROBE & 2) ? av[0] : av[m % 3];
      acc = mfma(w1r[4 * m + 0], a.x, acc);
      acc = mfma(w1r[4 * m + 1], a.y, acc);
      acc = mfma(w1r[4 * m + 2], a.z, acc);
      acc = mfma(w1r[4 * m + 3], a.w, acc);
      epi_at(m);  // (sub-block 0: on zeros, nothing stored, result dropped)
      if ((m & 7) == 1) h0_read(4 * s + (m >> 3));
      if ((m & 7) == 3) h0_store(4 * s + (m >> 3));
    }
    if (s > 0) head_part(s - 1);
    accp = acc;
    rbp = m0 + s * F_SB;
    kp = kept(h1g, rbp);
  }
#pragma unroll
  for (int m = 0; m < 32; ++m) epi_at(m);
  head_part(F_NSB - 1);
  __syncthreads();  // every head partial in LDS
  // out[row] = sum over the eight waves (in order) + b2
  if (t < F_RB) {
    const int sb = t / F_SB, rl = t % F_SB;
    float q = L.u.hp[sb][0][rl];
#pragma unroll
    for (int v = 1; v < 8; ++v) q += L.u.hp[sb][v][rl];
    const int row = m0 + t;
    if (row < rend) outp[(int64_t)row * d.ldout] = q + b2v;
  }
}

}  // namespace

// d3a_mlp_fwd's dispatch: true when this kernel took the launch
bool q2_fwd_launch(const d3a_mlp_fwd_desc& d, hipStream_t st) {
  if (d.n_hidden != 2 || d.H != F_H || d.n_out != 1 || d.n_in < 1 || d.n_in > 48) return false;
  // float4 loads of W1 rows, of the layer-1 / layer-2 biases and the head row
  auto a16 = [](const void* p, int64_t stride) {
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && stride % 4 == 0;
  };
  if (!a16(d.W[1], d.sW[1]) || !a16(d.b[0], d.sb[0]) || !a16(d.b[1], d.sb[1]) ||
      !a16(d.W[2], d.sW[2]))
    return false;
  if (d.aux_rows > 0 && d.aux_wdelta % 4) return false;
  const int64_t nb = (d.rows + F_RB - 1) / F_RB + (d.aux_rows + F_RB - 1) / F_RB;
  const dim3 grid((unsigned)nb, 1, (unsigned)d.C);
  const int xl = (d.n_in + 15) / 16 * 16;
  static const int probe = [] {
    const char* e = getenv("D3A_FWD_PROBE");
    return e ? atoi(e) : 0;
  }();
  if (probe && xl == 16) {
    if (probe == 1)
      hipLaunchKernelGGL((q2_fwd_kernel<16, 1>), grid, dim3(512), 0, st, d);
    else
      hipLaunchKernelGGL((q2_fwd_kernel<16, 2>), grid, dim3(512), 0, st, d);
    return true;
  }
  if (xl == 16)
    hipLaunchKernelGGL(q2_fwd_kernel<16>, grid, dim3(512), 0, st, d);
  else if (xl == 32)
    hipLaunchKernelGGL(q2_fwd_kernel<32>, grid, dim3(512), 0, st, d);
  else
    hipLaunchKernelGGL(q2_fwd_kernel<48>, grid, dim3(512), 0, st, d);
  return true;
}

}  // namespace d3a
