// Whole-MLP forward in one launch: the ReLU trunk + linear head of an
// ensemble member over a block of rows, activations staged in LDS.
//
// Replaces, for the vector encoders of the hot path, the per-layer
// nn.Linear + ReLU chain of VectorEncoder / VectorEncoderWithAction
// (d3rlpy/models/torch/encoders.py:265-275, 328-339) followed by the head
// (q_functions/mean_q_function.py:255-256 `_fc`, policies.py:57-59,170-176).
//
// One workgroup = BM rows of one member (blockIdx.z).  The input rows are
// copied to LDS once; every hidden layer reads its input tile from LDS and
// writes relu(x W^T + b) to the other LDS buffer (and, when requested, to
// global memory for the backward pass); the head reads the last tile from
// LDS.  No intermediate activation makes an HBM round trip and the whole
// forward is one launch instead of one per layer (the per-launch cost
// dominates the 100-256-row policy / target passes).
//
// MFMA mapping (v_mfma_f32_32x32x2_f32, exact fp32): each wave owns 32-wide
// output column tiles (ct = wave, wave+4, ...) for all BM rows; lane l covers
// column / row l&31 and k = k0 + 4*(l>>5) + {0..3}: the activation operand
// is one ds_read_b128 per 32-row tile, the weight operand one 16-byte global
// load (W rows are k-contiguous, L2-resident across workgroups), four MFMAs
// per 8 k.
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// W[n][k] row-major (row stride ldw), k..k+3 (zero beyond kend / n >= N)
__device__ __forceinline__ float4 wload(const float* W, int64_t ldw, int n, int N, int k,
                                        int kend) {
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n >= N) return r;
  const float* p = W + (int64_t)n * ldw + k;
  if (k + 3 < kend && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) {
    r = *reinterpret_cast<const float4*>(p);
  } else {
    if (k + 0 < kend) r.x = p[0];
    if (k + 1 < kend) r.y = p[1];
    if (k + 2 < kend) r.z = p[2];
    if (k + 3 < kend) r.w = p[3];
  }
  return r;
}

// LDS row stride: widest input (256) + 4 floats, so consecutive rows start 4
// banks apart and the ds_read_b128 lane groups are conflict-free
constexpr int LDK = 260;

template <int BM, int NW>
__global__ __launch_bounds__(64 * NW) void mlp_fwd_kernel(d3a_mlp_fwd_desc d) {
  constexpr int NT = 64 * NW;
  constexpr int RT = BM / 32;  // 32-row MFMA tiles per workgroup
  constexpr int U = 4;         // 8-k groups whose weight loads are in flight together
  __shared__ __attribute__((aligned(16))) float lds[2 * BM * LDK];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int li = lane & 31, lg = lane >> 5;
  const int c = blockIdx.z;
  const int64_t m0 = d.r0 + (int64_t)blockIdx.x * BM;
  const int64_t rend = d.r0 + d.rows;
  const int H = d.H;
  const int K0 = d.n_in;
  const int K0p = (K0 + 7) / 8 * 8;
  float* bufA = lds;
  float* bufB = lds + BM * LDK;

  // stage the input rows (zero-padded to a multiple of 8 columns)
  const float* xb = d.x + c * d.sxb;
  for (int i = t; i < BM * K0p; i += NT) {
    const int m = i / K0p, k = i - m * K0p;
    const int64_t r = m0 + m;
    bufA[m * LDK + k] = (r < rend && k < K0) ? xb[r * d.ldx + k] : 0.f;
  }
  __syncthreads();

  // hidden layers, and the head too when it is wide (a quantile head:
  // J > 64 columns go through the MFMA loop, narrow heads through VALU dots)
  const int J = d.n_out;
  const int n_mfma = d.n_hidden + (J > 64 ? 1 : 0);
  for (int l = 0; l < n_mfma; ++l) {
    const bool head = l == d.n_hidden;
    const int N = head ? J : H;
    const int Kin = l == 0 ? K0p : H;
    const int Kreal = l == 0 ? K0 : H;
    const float* W = d.W[l] + c * d.sW[l];
    const float* bias = d.b[l] + c * d.sb[l];
    float* gout = head ? d.out + c * d.sout : (d.h[l] ? d.h[l] + c * d.sh : nullptr);
    const int64_t ldg = head ? d.ldout : H;
    for (int ct = w; ct < (N + 31) / 32; ct += NW) {
      const int n = ct * 32 + li;
      f32x16 acc[RT];
#pragma unroll
      for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
      // weight operand double-buffered in registers: the loads of the next
      // 8U-deep k slice are in flight while the current one is multiplied
      float4 bv[U], bnx[U];
#pragma unroll
      for (int u = 0; u < U; ++u) bv[u] = wload(W, Kreal, n, N, 8 * u + 4 * lg, Kreal);
      for (int k0 = 0; k0 < Kin; k0 += 8 * U) {
        if (k0 + 8 * U < Kin) {
#pragma unroll
          for (int u = 0; u < U; ++u)
            bnx[u] = wload(W, Kreal, n, N, k0 + 8 * U + 8 * u + 4 * lg, Kreal);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int k = k0 + 8 * u + 4 * lg;
          if (k0 + 8 * u >= Kin) break;
#pragma unroll
          for (int i = 0; i < RT; ++i) {
            const float4 av = *reinterpret_cast<const float4*>(&bufA[(i * 32 + li) * LDK + k]);
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv[u].x, acc[i], 0, 0, 0);
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv[u].y, acc[i], 0, 0, 0);
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bv[u].z, acc[i], 0, 0, 0);
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bv[u].w, acc[i], 0, 0, 0);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) bv[u] = bnx[u];
      }
      if (n < N) {
        const float bn = bias[n];
#pragma unroll
        for (int i = 0; i < RT; ++i) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lg;
            const float v = head ? acc[i][r] + bn : fmaxf(acc[i][r] + bn, 0.f);
            if (!head) bufB[m * LDK + n] = v;
            if (gout && m0 + m < rend) gout[(m0 + m) * ldg + n] = v;
          }
        }
      }
    }
    if (head) return;
    __syncthreads();
    float* tmp = bufA; bufA = bufB; bufB = tmp;
  }

  // narrow head: out[r][j] = h[r] . Wh[j] + bh[j]
  const float* Wh = d.W[d.n_hidden] + c * d.sW[d.n_hidden];
  const float* bh = d.b[d.n_hidden] + c * d.sb[d.n_hidden];
  float* outb = d.out + c * d.sout;
  if (J == 1) {
    // TPR lanes per row, interleaved columns, then a shuffle reduction
    constexpr int TPR = NT / BM;
    const int m = t / TPR, q = t % TPR;
    float s = 0.f;
    for (int n = q * 4; n < H; n += TPR * 4) {
      const float4 hv = *reinterpret_cast<const float4*>(&bufA[m * LDK + n]);
      const float4 wv = *reinterpret_cast<const float4*>(&Wh[n]);
      s = fmaf(hv.x, wv.x, s);
      s = fmaf(hv.y, wv.y, s);
      s = fmaf(hv.z, wv.z, s);
      s = fmaf(hv.w, wv.w, s);
    }
#pragma unroll
    for (int o = TPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (q == 0 && m0 + m < rend) outb[(m0 + m) * d.ldout] = s + bh[0];
  } else {
    for (int p = t; p < BM * J; p += NT) {
      const int m = p / J, j = p - m * J;
      if (m0 + m >= rend) continue;
      const float* wr = Wh + (int64_t)j * H;
      float s = 0.f;
      for (int n = 0; n < H; n += 4) {
        const float4 hv = *reinterpret_cast<const float4*>(&bufA[m * LDK + n]);
        const float4 wv = *reinterpret_cast<const float4*>(&wr[n]);
        s = fmaf(hv.x, wv.x, s);
        s = fmaf(hv.y, wv.y, s);
        s = fmaf(hv.z, wv.z, s);
        s = fmaf(hv.w, wv.w, s);
      }
      outb[(m0 + m) * d.ldout + j] = s + bh[j];
    }
  }
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_mlp_fwd(const d3a_mlp_fwd_desc* d_in, void* stream) {
  D3A_CHECK_ARG(d_in, "d3a_mlp_fwd: null desc");
  d3a_mlp_fwd_desc d = *d_in;
  D3A_CHECK_ARG(d.x && d.out, "d3a_mlp_fwd: null input / output");
  D3A_CHECK_ARG(d.n_hidden >= 1 && d.n_hidden <= D3A_MLP_MAX_HIDDEN,
                "d3a_mlp_fwd: 1..D3A_MLP_MAX_HIDDEN hidden layers");
  D3A_CHECK_ARG(d.H % 32 == 0 && d.H >= 32 && d.H <= 256, "d3a_mlp_fwd: H must be 32..256, %32");
  D3A_CHECK_ARG(d.n_in >= 1 && d.n_in <= 256, "d3a_mlp_fwd: n_in must be 1..256");
  D3A_CHECK_ARG(d.n_out >= 1 && d.n_out <= 1024, "d3a_mlp_fwd: n_out must be 1..1024");
  D3A_CHECK_ARG(d.C >= 1 && d.rows >= 0, "d3a_mlp_fwd: bad sizes");
  for (int l = 0; l <= d.n_hidden; ++l)
    D3A_CHECK_ARG(d.W[l] && d.b[l], "d3a_mlp_fwd: null layer parameters");
  // the head reads W rows with 16-byte loads
  D3A_CHECK_ARG((reinterpret_cast<uintptr_t>(d.W[d.n_hidden]) & 15) == 0 && d.sW[d.n_hidden] % 4 == 0,
                "d3a_mlp_fwd: head weights must be 16-byte aligned");
  if (d.rows == 0) return 0;
  // 64-row blocks for the large critic passes (each weight load feeds two
  // row tiles), 32-row blocks otherwise (more workgroups for 100-256 rows);
  // 8 waves: one 32-column tile per wave at H = 256
  const int bm = d.block_rows > 0 ? d.block_rows : (d.rows * d.C >= 4096 ? 64 : 32);
  D3A_CHECK_ARG(bm == 32 || bm == 64, "d3a_mlp_fwd: block_rows must be 0, 32 or 64");
  dim3 grid((unsigned)((d.rows + bm - 1) / bm), 1, (unsigned)d.C);
  if (bm == 32)
    hipLaunchKernelGGL((mlp_fwd_kernel<32, 8>), grid, dim3(512), 0, (hipStream_t)stream, d);
  else
    hipLaunchKernelGGL((mlp_fwd_kernel<64, 8>), grid, dim3(512), 0, (hipStream_t)stream, d);
  D3A_LAUNCH_CHECK("d3a_mlp_fwd");
  return 0;
}

// ---------------------------------------------------------------------------
// Backward-data of the same MLP in one launch: the chain of pre-activation
// gradients dz_l (written for the weight-gradient GEMMs) and optionally
// dL/dx, each row block independent.  Replaces the autograd backward of
// the encoder / head chain (encoders.py:265-275, mean_q_function.py:255-256)
// up to the weight gradients, which stay split-K GEMMs over all rows.
namespace d3a {
namespace {

template <int BM, int NW>
__global__ __launch_bounds__(64 * NW) void mlp_bwd_kernel(d3a_mlp_bwd_desc d) {
  constexpr int NT = 64 * NW;
  constexpr int RT = BM / 32;
  constexpr int U = 4;
  __shared__ __attribute__((aligned(16))) float lds[2 * BM * LDK];
  __shared__ float s_g[BM];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int li = lane & 31, lg = lane >> 5;
  const int c = blockIdx.z;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int64_t rows = d.rows;
  const int H = d.H, L = d.n_hidden, J = d.n_out;
  float* bufA = lds;
  float* bufB = lds + BM * LDK;
  const float* hl = d.h[L - 1] + c * d.sh;

  // ---- head: dz_{L-1} = (dL/dout W_head) * [h_{L-1} > 0] ----
  const float* Wh = d.W[L] + c * d.sW[L];
  if (J == 1) {
    if (t < BM) {
      const int64_t r = m0 + t;
      float g = 0.f;
      if (r < rows) {
        if (d.q_min) {
          // backward of min over the ensemble: `scale` on the first argmin
          int arg = 0;
          float mn = d.q_min[r];
          for (int k = 1; k < d.C; ++k) {
            const float v = d.q_min[k * d.sqb + r];
            if (v < mn) { mn = v; arg = k; }
          }
          g = arg == c ? d.scale : 0.f;
        } else {
          g = d.g[c * d.sgb + r];
          if (d.gscale && r < d.n_scaled) g *= *d.gscale;
        }
        if (d.g_eff) d.g_eff[c * d.sgeb + r] = g;
      }
      s_g[t] = g;
    }
    __syncthreads();
    for (int i = t; i < BM * H; i += NT) {
      const int m = i / H, n = i - m * H;
      const int64_t r = m0 + m;
      float v = 0.f;
      if (r < rows && hl[r * d.ldh + n] > 0.f) v = s_g[m] * Wh[n];
      bufA[m * LDK + n] = v;
      if (r < rows) d.dz[L - 1][c * d.sdz + r * H + n] = v;
    }
  } else {
    const float* dh = d.dhead + c * d.sdhb;
    for (int i = t; i < BM * H; i += NT) {
      const int m = i / H, n = i - m * H;
      const int64_t r = m0 + m;
      float v = 0.f;
      if (r < rows && hl[r * d.ldh + n] > 0.f) {
        for (int j = 0; j < J; ++j) v = fmaf(dh[r * d.lddh + j], Wh[(int64_t)j * H + n], v);
      }
      bufA[m * LDK + n] = v;
      if (r < rows) d.dz[L - 1][c * d.sdz + r * H + n] = v;
    }
  }
  __syncthreads();

  // ---- trunk: dz_{l-1} = (dz_l W_l) * [h_{l-1} > 0]; then dx = dz_0 W_0 ----
  for (int l = L - 1; l >= 0; --l) {
    const bool to_x = l == 0;
    if (to_x && !d.dx) break;
    const int Kout = to_x ? d.n_in : H;  // columns of the product
    const float* W = d.W[l] + c * d.sW[l];
    const int ldw = to_x ? d.n_in : H;
    const float* hm = to_x ? nullptr : d.h[l - 1] + c * d.sh;
    float* dzo = to_x ? nullptr : d.dz[l - 1] + c * d.sdz;
    for (int ct = w; ct < (Kout + 31) / 32; ct += NW) {
      const int k = ct * 32 + li;
      f32x16 acc[RT];
#pragma unroll
      for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
      // B(n, k) = W[n][k]: four rows, one column per lane (coalesced over
      // lanes); double-buffered like the forward's weight operand
      auto bload = [&](int n0_, float4* dst) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int n = n0_ + 8 * u + 4 * lg;
          const float* p = W + (int64_t)n * ldw + k;
          const bool ok = k < Kout;
          dst[u].x = ok ? p[0] : 0.f;
          dst[u].y = ok ? p[ldw] : 0.f;
          dst[u].z = ok ? p[2 * ldw] : 0.f;
          dst[u].w = ok ? p[3 * ldw] : 0.f;
        }
      };
      float4 bv[U], bnx[U];
      bload(0, bv);
      for (int n0 = 0; n0 < H; n0 += 8 * U) {
        if (n0 + 8 * U < H) bload(n0 + 8 * U, bnx);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int n = n0 + 8 * u + 4 * lg;
#pragma unroll
          for (int i = 0; i < RT; ++i) {
            const float4 av = *reinterpret_cast<const float4*>(&bufA[(i * 32 + li) * LDK + n]);
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv[u].x, acc[i], 0, 0, 0);
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv[u].y, acc[i], 0, 0, 0);
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bv[u].z, acc[i], 0, 0, 0);
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bv[u].w, acc[i], 0, 0, 0);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) bv[u] = bnx[u];
      }
      if (k < Kout) {
#pragma unroll
        for (int i = 0; i < RT; ++i) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lg;
            const int64_t row = m0 + m;
            if (to_x) {
              if (row < rows) d.dx[c * d.sdxb + row * d.lddx + k] = acc[i][r];
            } else {
              const float v = (row < rows && hm[row * d.ldh + k] > 0.f) ? acc[i][r] : 0.f;
              bufB[m * LDK + k] = v;
              if (row < rows) dzo[row * H + k] = v;
            }
          }
        }
      }
    }
    __syncthreads();
    float* tmp = bufA; bufA = bufB; bufB = tmp;
  }
}

}  // namespace
}  // namespace d3a

extern "C" int d3a_mlp_bwd(const d3a_mlp_bwd_desc* dp, void* stream) {
  D3A_CHECK_ARG(dp, "d3a_mlp_bwd: null desc");
  const d3a_mlp_bwd_desc& d = *dp;
  D3A_CHECK_ARG(d.n_hidden >= 1 && d.n_hidden <= D3A_MLP_MAX_HIDDEN,
                "d3a_mlp_bwd: 1..D3A_MLP_MAX_HIDDEN hidden layers");
  D3A_CHECK_ARG(d.H % 32 == 0 && d.H >= 32 && d.H <= 256, "d3a_mlp_bwd: H must be 32..256, %32");
  D3A_CHECK_ARG(d.n_in >= 1 && d.n_in <= 256 && d.n_out >= 1 && d.n_out <= 64 && d.C >= 1,
                "d3a_mlp_bwd: bad sizes");
  for (int l = 0; l <= d.n_hidden; ++l) D3A_CHECK_ARG(d.W[l], "d3a_mlp_bwd: null weights");
  for (int l = 0; l < d.n_hidden; ++l)
    D3A_CHECK_ARG(d.h[l] && d.dz[l], "d3a_mlp_bwd: activations and dz outputs required");
  D3A_CHECK_ARG(d.n_out == 1 ? (d.g != nullptr || d.q_min != nullptr) : d.dhead != nullptr,
                "d3a_mlp_bwd: missing output gradient");
  if (d.rows <= 0) return 0;
  const int bm = d.block_rows > 0 ? d.block_rows : (d.rows * d.C >= 4096 ? 64 : 32);
  D3A_CHECK_ARG(bm == 32 || bm == 64, "d3a_mlp_bwd: block_rows must be 0, 32 or 64");
  dim3 grid((unsigned)((d.rows + bm - 1) / bm), 1, (unsigned)d.C);
  if (bm == 32)
    hipLaunchKernelGGL((mlp_bwd_kernel<32, 8>), grid, dim3(512), 0, (hipStream_t)stream, d);
  else
    hipLaunchKernelGGL((mlp_bwd_kernel<64, 8>), grid, dim3(512), 0, (hipStream_t)stream, d);
  D3A_LAUNCH_CHECK("d3a_mlp_bwd");
  return 0;
}
