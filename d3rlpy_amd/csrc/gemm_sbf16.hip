// Split-bf16 GEMM: fp32 operands evaluated on the bf16 matrix cores.
//
// The throughput instantiation of the ensemble-Q layer GEMM (the nn.Linear of
// encoders.py:265-275 over every critic at once; SURVEY §7 step 4, "fp32 for
// parity, bf16 for throughput").  Each fp32 operand x is split into bf16
// parts x = x0 + x1 (+ x2) — x0 = bf16(x), x1 = bf16(x - x0), x2 =
// bf16(x - x0 - x1), each subtraction exact in fp32 — and a product is the sum
// of the part products whose order is below fp32's resolution:
//   TERMS 3 (hi/lo):      x0 y0 + x0 y1 + x1 y0                  ~2^-16 relative
//   TERMS 6 (hi/mid/lo):  + x0 y2 + x1 y1 + x2 y0                ~2^-24 relative
// on v_mfma_f32_32x32x16_bf16 (16 k per instruction, 32 cycles per SIMD:
// 3 or 6 of them per 16 k against 8 x 64 cycles of v_mfma_f32_32x32x2_f32),
// accumulated in fp32.
//
// Operands are split once, when a K tile is staged into LDS (one split per
// element per workgroup, not per use): a 128x128 output tile, sixteen 32x32
// waves, BK 32, LDS rows [m][k] of bf16 parts so that a lane's fragment
// (A[row r][k = 8h + j], B[k = 8h + j][col r], j < 8) is one ds_read_b128 per
// part.  A and B must be k-contiguous (the forward GEMM y = x W^T + b: x rows
// and W rows both run along k); epilogue bias / ReLU as d3a_gemm_f32.
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int SB_BM = 128, SB_BN = 128, SB_BK = 32, SB_NT = 1024;
constexpr int SB_LD = SB_BK + 8;  // bf16 row stride (80 B: 16-B aligned, bank-staggered)

template <int PARTS>
struct SbLds {
  __bf16 A[2][PARTS][SB_BM * SB_LD];
  __bf16 B[2][PARTS][SB_BN * SB_LD];
};

__device__ __forceinline__ void split4(float4 v, bf16x4* out, int parts) {
  float x[4] = {v.x, v.y, v.z, v.w};
  bf16x4 p0, p1, p2;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const __bf16 h0 = (__bf16)x[i];
    const float r1 = x[i] - (float)h0;  // exact
    const __bf16 h1 = (__bf16)r1;
    const float r2 = r1 - (float)h1;    // exact
    p0[i] = h0;
    p1[i] = h1;
    p2[i] = (__bf16)r2;
  }
  out[0] = p0;
  out[1] = p1;
  if (parts > 2) out[2] = p2;
}

// BT: B is n-contiguous (B(k, n) = W[k][n], the input-gradient GEMM dx = dy W):
// its tile is transposed into the [n][k] LDS rows while staging (thread t
// takes k = t % 32, n = 4 (t / 32) .. +3, so consecutive threads write
// consecutive bf16 of one row).
// AT: A is m-contiguous (A(m, k) = dY[k][m], the weight-gradient GEMM
// dW = dY^T X over the rows k), staged transposed like BT; its fp32 row sums
// (the bias gradient, d3a_gemm_desc.rowsum) are accumulated in fp64 by the
// staging threads and reduced over each 32-lane group in a fixed order.
// Split-K: blockIdx.z = batch * splits + s covers rows [s*kchunk, ...).
template <int TERMS, bool AT, bool BT>
__global__ __launch_bounds__(SB_NT) void gemm_sbf16_kernel(d3a_gemm_desc p, int64_t kchunk) {
  constexpr int PARTS = TERMS == 3 ? 2 : 3;
  __shared__ __attribute__((aligned(16))) SbLds<PARTS> L;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t n0 = (int64_t)blockIdx.x * SB_BN, m0 = (int64_t)blockIdx.y * SB_BM;
  const int64_t splits = p.splits > 1 ? p.splits : 1;
  const int64_t b = blockIdx.z / splits, sp = blockIdx.z % splits;
  const int64_t kbeg = sp * kchunk;
  const int64_t kend = kbeg + kchunk < p.K ? kbeg + kchunk : p.K;
  const float* A = p.A + b * p.sAb;
  const float* B = p.B + b * p.sBb;
  // staging: one float4 of A and one of B per thread per K tile
  const int srow = t / (SB_BK / 4), sk = (t % (SB_BK / 4)) * 4;
  const int wm = (w / 4) * 32, wn = (w % 4) * 32;

  auto gload = [&](const float* base, int64_t ld, int64_t x, int64_t X, int64_t k) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (x < X) {
      const float* q = base + x * ld + k;
      if (k + 3 < kend) {
        v = *reinterpret_cast<const float4*>(q);
      } else {
        if (k + 0 < kend) v.x = q[0];
        if (k + 1 < kend) v.y = q[1];
        if (k + 2 < kend) v.z = q[2];
      }
    }
    return v;
  };
  // transposed staging coordinates (k along the thread, 4 consecutive x)
  const int tk = t % SB_BK, tn = (t / SB_BK) * 4;
  auto gload_t = [&](const float* base, int64_t sk_, int64_t x0, int64_t X, int64_t k) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t x = x0 + tn;
    if (k < kend) {
      const float* q = base + k * sk_ + x;
      if (x + 3 < X) {
        v = *reinterpret_cast<const float4*>(q);
      } else {
        if (x + 0 < X) v.x = q[0];
        if (x + 1 < X) v.y = q[1];
        if (x + 2 < X) v.z = q[2];
      }
    }
    return v;
  };
  auto loadA = [&](int64_t k0) {
    return AT ? gload_t(A, p.sAk, m0, p.M, k0 + tk) : gload(A, p.sAm, m0 + srow, p.M, k0 + sk);
  };
  auto loadB = [&](int64_t k0) {
    return BT ? gload_t(B, p.sBk, n0, p.N, k0 + tk) : gload(B, p.sBn, n0 + srow, p.N, k0 + sk);
  };
  const bool do_rowsum = AT && p.rowsum != nullptr && blockIdx.x == 0;
  double rs0 = 0.0, rs1 = 0.0, rs2 = 0.0, rs3 = 0.0;
  auto stage = [&](int buf, float4 va, float4 vb) {
    bf16x4 pa[3], pb[3];
    split4(va, pa, PARTS);
    split4(vb, pb, PARTS);
    if (do_rowsum) {
      rs0 += (double)va.x;
      rs1 += (double)va.y;
      rs2 += (double)va.z;
      rs3 += (double)va.w;
    }
#pragma unroll
    for (int q = 0; q < PARTS; ++q) {
      if (AT) {
#pragma unroll
        for (int i = 0; i < 4; ++i) L.A[buf][q][(tn + i) * SB_LD + tk] = pa[q][i];
      } else {
        *reinterpret_cast<bf16x4*>(&L.A[buf][q][srow * SB_LD + sk]) = pa[q];
      }
      if (BT) {
#pragma unroll
        for (int i = 0; i < 4; ++i) L.B[buf][q][(tn + i) * SB_LD + tk] = pb[q][i];
      } else {
        *reinterpret_cast<bf16x4*>(&L.B[buf][q][srow * SB_LD + sk]) = pb[q];
      }
    }
  };

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  float4 va = loadA(kbeg);
  float4 vb = loadB(kbeg);
  stage(0, va, vb);
  __syncthreads();
  int cur = 0;
  for (int64_t k0 = kbeg; k0 < kend; k0 += SB_BK) {
    const bool more = k0 + SB_BK < kend;
    if (more) {
      va = loadA(k0 + SB_BK);
      vb = loadB(k0 + SB_BK);
    }
#pragma unroll
    for (int ks = 0; ks < SB_BK; ks += 16) {
      bf16x8 a[PARTS], bb[PARTS];
#pragma unroll
      for (int q = 0; q < PARTS; ++q) {
        a[q] = *reinterpret_cast<const bf16x8*>(&L.A[cur][q][(wm + r) * SB_LD + ks + 8 * h]);
        bb[q] = *reinterpret_cast<const bf16x8*>(&L.B[cur][q][(wn + r) * SB_LD + ks + 8 * h]);
      }
      // smallest terms first
      if (TERMS == 6) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bb[2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], bb[1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], bb[0], acc, 0, 0, 0);
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bb[1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], bb[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bb[0], acc, 0, 0, 0);
    }
    if (more) stage(cur ^ 1, va, vb);
    __syncthreads();
    cur ^= 1;
  }

  if (do_rowsum) {
    // the 32 lanes of a group hold the same 4 rows at k = tk: fixed butterfly
    for (int o = 16; o > 0; o >>= 1) {
      rs0 += __shfl_xor(rs0, o, 64);
      rs1 += __shfl_xor(rs1, o, 64);
      rs2 += __shfl_xor(rs2, o, 64);
      rs3 += __shfl_xor(rs3, o, 64);
    }
    if (tk == 0) {
      float* rsum = p.rowsum + b * p.sRb + sp * p.sRs;
      const double v[4] = {rs0, rs1, rs2, rs3};
      for (int i = 0; i < 4; ++i)
        if (m0 + tn + i < p.M) rsum[m0 + tn + i] = (float)v[i];
    }
  }
  float* C = p.C + b * p.sCb + sp * p.sCs;
  const float* bias = p.bias ? p.bias + b * p.sbias_b : nullptr;
  const float* mask = p.mask ? p.mask + b * p.sMb : nullptr;
  const int64_t n = n0 + wn + r;
  if (n >= p.N) return;
  const float bn = bias ? bias[n] : 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t m = m0 + wm + (i & 3) + 8 * (i >> 2) + 4 * h;
    if (m < p.M) {
      float v = acc[i] * p.alpha;
      if (bias) v += bn;
      if (p.relu) v = fmaxf(v, 0.f);
      if (mask && !(mask[m * p.sMm + n * p.sMn] > 0.f)) v = 0.f;
      C[m * p.sCm + n * p.sCn] = v;
    }
  }
}

}  // namespace
}  // namespace d3a

namespace d3a {
namespace {
// y[m][n] = act(sum_s part[s][m][n] + bias[n]), the split-K partials of a
// d3a_gemm_sbf16 launch added in split order (four n per thread)
__global__ __launch_bounds__(256) void splitk_epilogue_kernel(const float* __restrict__ part,
                                                              int32_t S, int64_t sS, float* y,
                                                              const float* bias, int64_t M,
                                                              int64_t N, int32_t relu) {
  const int64_t i4 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n4 = N / 4;
  if (i4 >= M * n4) return;
  const int64_t m = i4 / n4, n = 4 * (i4 - m * n4);
  const int64_t o = m * N + n;
  float4 a = *reinterpret_cast<const float4*>(part + o);
  for (int s = 1; s < S; ++s) {
    const float4 v = *reinterpret_cast<const float4*>(part + s * sS + o);
    a.x += v.x;
    a.y += v.y;
    a.z += v.z;
    a.w += v.w;
  }
  if (bias) {
    a.x += bias[n];
    a.y += bias[n + 1];
    a.z += bias[n + 2];
    a.w += bias[n + 3];
  }
  if (relu) {
    a.x = fmaxf(a.x, 0.f);
    a.y = fmaxf(a.y, 0.f);
    a.z = fmaxf(a.z, 0.f);
    a.w = fmaxf(a.w, 0.f);
  }
  *reinterpret_cast<float4*>(y + o) = a;
}
}  // namespace
}  // namespace d3a

extern "C" int d3a_splitk_epilogue_f32(const float* part, int32_t S, int64_t sS, float* y,
                                       const float* bias, int64_t M, int64_t N, int32_t relu,
                                       void* stream) {
  using namespace d3a;
  D3A_CHECK_ARG(part && y && S >= 1 && M >= 0 && N >= 0, "d3a_splitk_epilogue_f32: bad args");
  D3A_CHECK_ARG(N % 4 == 0 && sS % 4 == 0 &&
                    ((reinterpret_cast<uintptr_t>(part) | reinterpret_cast<uintptr_t>(y)) & 15) == 0,
                "d3a_splitk_epilogue_f32: 16-byte aligned rows of N %% 4 == 0 floats");
  const int64_t n = M * (N / 4);
  if (n == 0) return 0;
  hipLaunchKernelGGL(splitk_epilogue_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, part, S, sS, y, bias, M, N, relu);
  D3A_LAUNCH_CHECK("d3a_splitk_epilogue_f32");
  return 0;
}

extern "C" int d3a_gemm_sbf16(const d3a_gemm_desc* d, int32_t terms, void* stream) {
  using namespace d3a;
  D3A_CHECK_ARG(d && d->A && d->B && d->C, "d3a_gemm_sbf16: null operand");
  D3A_CHECK_ARG(terms == 3 || terms == 6, "d3a_gemm_sbf16: terms must be 3 or 6");
  const bool at = d->sAk != 1, bt = d->sBk != 1;
  D3A_CHECK_ARG((d->sAk == 1 || d->sAm == 1) && (d->sBk == 1 || d->sBn == 1),
                "d3a_gemm_sbf16: every operand k- or row-contiguous");
  D3A_CHECK_ARG((at ? d->sAk % 4 == 0 && d->M % 4 == 0 : d->sAm % 4 == 0 && d->K % 4 == 0) &&
                    (bt ? d->sBk % 4 == 0 && d->N % 4 == 0 : d->sBn % 4 == 0 && d->K % 4 == 0) &&
                    ((reinterpret_cast<uintptr_t>(d->A) | reinterpret_cast<uintptr_t>(d->B)) & 15) == 0,
                "d3a_gemm_sbf16: 16-byte aligned vectors along the contiguous dimensions");
  D3A_CHECK_ARG(!d->agen, "d3a_gemm_sbf16: no generated A");
  D3A_CHECK_ARG(!d->accumulate && d->batch2 <= 1 && (!d->rowsum || at),
                "d3a_gemm_sbf16: no accumulate / batch2; rowsum only with an m-contiguous A");
  if (d->M == 0 || d->N == 0 || d->batch == 0) return 0;
  const int64_t splits = d->splits > 1 ? d->splits : 1;
  int64_t kchunk = (d->K + splits - 1) / splits;
  kchunk = (kchunk + SB_BK - 1) / SB_BK * SB_BK;
  D3A_CHECK_ARG(d->batch * splits < 65536, "d3a_gemm_sbf16: batch * splits too large");
  const dim3 grid((unsigned)((d->N + SB_BN - 1) / SB_BN), (unsigned)((d->M + SB_BM - 1) / SB_BM),
                  (unsigned)(d->batch * splits));
  hipStream_t st = (hipStream_t)stream;
#define D3A_SB_LAUNCH(T, A_, B_) \
  hipLaunchKernelGGL((gemm_sbf16_kernel<T, A_, B_>), grid, dim3(SB_NT), 0, st, *d, kchunk)
  if (terms == 3) {
    if (at) { if (bt) D3A_SB_LAUNCH(3, true, true); else D3A_SB_LAUNCH(3, true, false); }
    else { if (bt) D3A_SB_LAUNCH(3, false, true); else D3A_SB_LAUNCH(3, false, false); }
  } else {
    if (at) { if (bt) D3A_SB_LAUNCH(6, true, true); else D3A_SB_LAUNCH(6, true, false); }
    else { if (bt) D3A_SB_LAUNCH(6, false, true); else D3A_SB_LAUNCH(6, false, false); }
  }
#undef D3A_SB_LAUNCH
  D3A_LAUNCH_CHECK("d3a_gemm_sbf16");
  return 0;
}
