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
#include <cstdlib>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"
#include "x6.hpp"

namespace d3a {
// q2_fwd.hip: the register-resident instantiation for [n_in, 256, 256, 1]
bool q2_fwd_launch(const d3a_mlp_fwd_desc& d, hipStream_t st);
// mlp_small.hip: 16-row workgroups for small passes (block_rows == 16)
bool mlp_small_launch(const d3a_mlp_fwd_desc& d, hipStream_t st);
bool mlp_parts_launch(const d3a_mlp_fwd_desc& d, hipStream_t st);

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// LDS row stride: widest input (256) + 4 floats, so consecutive rows start 4
// banks apart and the ds_read_b128 lane groups are conflict-free
constexpr int LDK = 260;

// One 32-column output tile over all RT row tiles:
//   acc[i] += A[i*32.., 0:Kin] (LDS, row stride LDK) x B[0:Kin][this column]
// Kin is a multiple of 8U (the LDS operand is zero-padded up to it);
// load(k) returns the lane's B operand B[k..k+3][column].  The B operand is
// double-buffered in registers: the loads of the next 32-deep k slice are
// issued before the MFMAs of the current one.  Loaders must be
// unconditional (clamped addresses, no guarded loads) so the compiler can
// keep them in flight across the MFMAs -- a guarded load makes it drain the
// whole queue first.
template <int RT, int U, class LoadB>
__device__ __forceinline__ void tile_mfma(f32x16* acc, const float* A, int Kin, int li, int lg,
                                          LoadB load) {
  // multiply one 32-deep slice at k0 with its weights b; every activation
  // operand of the slice is read before its MFMAs
  auto slice = [&](int k0, const float4* b) {
    float4 av[U][RT];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < RT; ++i)
        av[u][i] = *reinterpret_cast<const float4*>(&A[(i * 32 + li) * LDK + k0 + 8 * u + 4 * lg]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int i = 0; i < RT; ++i) {
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u][i].x, b[u].x, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u][i].y, b[u].y, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u][i].z, b[u].z, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u][i].w, b[u].w, acc[i], 0, 0, 0);
      }
    }
  };
  // ping-pong between two register sets (no copies, so no wait on the
  // prefetch before its slice); prefetch addresses past the end clamp to
  // the last slice and are never used
  float4 b0[U], b1[U];
#pragma unroll
  for (int u = 0; u < U; ++u) b0[u] = load(8 * u + 4 * lg);
  const int klast = Kin - 8 * U;
  int k0 = 0;
  for (; k0 + 16 * U <= Kin; k0 += 16 * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) b1[u] = load(k0 + 8 * U + 8 * u + 4 * lg);
    __builtin_amdgcn_sched_barrier(0);
    slice(k0, b0);
#pragma unroll
    for (int u = 0; u < U; ++u) b0[u] = load(min(k0 + 16 * U, klast) + 8 * u + 4 * lg);
    __builtin_amdgcn_sched_barrier(0);
    slice(k0 + 8 * U, b1);
  }
  if (k0 < Kin) slice(k0, b0);  // odd number of 32-deep slices
}

// RTW = 32-row tiles per wave: the waves split the BM rows into RT / RTW
// groups and each group's waves split the output columns.  32-row blocks use
// half the LDS, so two workgroups share a CU.
template <int BM, int NW, int RTW>
__global__ __launch_bounds__(64 * NW)
__attribute__((amdgpu_waves_per_eu((NW / 4) * (BM == 32 ? 2 : 1))))
void mlp_fwd_kernel(d3a_mlp_fwd_desc d) {
  constexpr int NT = 64 * NW;
  constexpr int RT = BM / 32;  // 32-row MFMA tiles per workgroup
  constexpr int RG = RT / RTW;  // row groups
  constexpr int NCW = NW / RG;  // waves per row group
  static_assert(RT % RTW == 0 && NW % RG == 0, "bad wave split");
  // 128-row blocks keep one activation buffer (133 KB) and update it in place
  constexpr bool INPLACE = BM == 128;
  static_assert(!INPLACE || (RG == 1 && NW * 32 >= 256), "in-place needs a column tile per wave");
  __shared__ __attribute__((aligned(16))) float lds[(INPLACE ? 1 : 2) * BM * LDK];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int li = lane & 31, lg = lane >> 5;
  const int c = blockIdx.z;
  // workgroups past the main pass's row blocks run the aux pass (the same
  // network at W + aux_wdelta over aux_rows rows of aux_x, no activations kept)
  const int64_t nb_main = (d.rows + BM - 1) / BM;
  const bool aux = (int64_t)blockIdx.x >= nb_main;
  const int64_t m0 = aux ? ((int64_t)blockIdx.x - nb_main) * BM : d.r0 + (int64_t)blockIdx.x * BM;
  const int64_t rend = aux ? d.aux_rows : d.r0 + d.rows;
  const int64_t h_from = aux ? rend : d.h_from;
  const int64_t wdel = aux ? d.aux_wdelta : 0;
  float* const outp = aux ? d.aux_out + c * d.aux_sout : d.out + c * d.sout;
  const int H = d.H;
  const int K0 = d.n_in;
  // zero-padded to whole k slices: 16-deep (U = 2) for the narrow first layer
  // (K2: 14 inputs -> 16 instead of 32), 32-deep for the hidden layers
  const int K0p = (K0 + 15) / 16 * 16;
  float* bufA = lds;
  float* bufB = INPLACE ? lds : lds + BM * LDK;

  // stage the input rows (zero-padded to a multiple of 8 columns)
  const float* xb = aux ? d.aux_x + c * d.aux_sxb : d.x + c * d.sxb;
  const int64_t ldx = aux ? d.aux_ldx : d.ldx;
  for (int i = t; i < BM * K0p; i += NT) {
    const int m = i / K0p, k = i - m * K0p;
    const int64_t r = m0 + m;
    bufA[m * LDK + k] = (r < rend && k < K0) ? xb[r * ldx + k] : 0.f;
  }
  __syncthreads();

  // hidden layers, and the head too when it is wide (a quantile head:
  // J > 64 columns go through the MFMA loop, narrow heads through VALU dots)
  const int J = d.n_out;
  const int n_mfma = d.n_hidden + (J > 64 ? 1 : 0);
  // per-lane row-validity bit masks over the RTW x 16 accumulator rows:
  // v_out rows < rend, v_h rows also >= h_from (activations kept)
  uint64_t v_out = 0, v_h = 0;
  {
    const int64_t lr = m0 + (w % RG) * RTW * 32 + 4 * lg;
#pragma unroll
    for (int i = 0; i < RTW; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = lr + i * 32 + (r & 3) + 8 * (r >> 2);
        const uint64_t bit = uint64_t(1) << (i * 16 + r);
        if (row < rend) {
          v_out |= bit;
          if (row >= h_from) v_h |= bit;
        }
      }
  }
  for (int l = 0; l < n_mfma; ++l) {
    const bool head = l == d.n_hidden;
    const int N = head ? J : H;
    const int Kin = l == 0 ? K0p : H;
    const int Kreal = l == 0 ? K0 : H;
    const float* W = d.W[l] + wdel + c * d.sW[l];
    const float* bias = d.b[l] + wdel + c * d.sb[l];
    float* gout = head ? outp : (!aux && d.h[l] ? d.h[l] + c * d.sh : nullptr);
    const int ldg = head ? (int)d.ldout : H;
    const int rg = w % RG;
    const float* Ag = bufA + rg * RTW * 32 * LDK;
    auto mma = [&](f32x16* acc, int n) {
#pragma unroll
      for (int i = 0; i < RTW; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
      // columns >= N are computed from a clamped row and dropped; 32-bit
      // offsets from the uniform base keep the addresses in one VGPR each
      const int wo = min(n, N - 1) * Kreal;
      if (l == 0) {
        // k beyond the real inputs clamps to the last one; its product with
        // the zero padding of the LDS operand is an exact zero
        tile_mfma<RTW, 2>(acc, Ag, Kin, li, lg, [&](int k) {
          float4 r;
          r.x = W[wo + min(k + 0, Kreal - 1)];
          r.y = W[wo + min(k + 1, Kreal - 1)];
          r.z = W[wo + min(k + 2, Kreal - 1)];
          r.w = W[wo + min(k + 3, Kreal - 1)];
          return r;
        });
      } else {
        tile_mfma<RTW, 4>(acc, Ag, Kin, li, lg,
                       [&](int k) { return *reinterpret_cast<const float4*>(W + (wo + k)); });
      }
    };
    auto epi = [&](const f32x16* acc, int n, float* dst, bool store_h) {
      if (n >= N) return;
      const float bn = bias[n];
      // this lane's rows: lrow + mo(i, r); row validity from the masks
      const int lrow = rg * RTW * 32 + 4 * lg;
      float* gp = gout ? gout + (int64_t)(m0 + lrow) * ldg + n : nullptr;
      const uint64_t vm = head ? v_out : v_h;
#pragma unroll
      for (int i = 0; i < RTW; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int mo = i * 32 + (r & 3) + 8 * (r >> 2);
          const bool ok = (vm >> (i * 16 + r)) & 1;
          if (head) {
            if (ok) gp[mo * ldg] = acc[i][r] + bn;
          } else {
            const float v = fmaxf(acc[i][r] + bn, 0.f);
            dst[(lrow + mo) * LDK + n] = v;
            // the global copy for the backward pass leaves with the
            // epilogue (overlapping the other waves' MFMAs)
            if (store_h && gp && ok) gp[mo * ldg] = v;
          }
        }
      }
    };
    if (INPLACE && !head) {
      // one column tile per wave (H <= 32 * NW); the layer's output
      // overwrites its input once every wave has finished reading it
      const int n = w * 32 + li;
      const bool act = w * 32 < N;
      f32x16 acc[RTW];
      if (act) mma(acc, n);
      __syncthreads();
      if (act) epi(acc, n, bufA, false);
      __syncthreads();
      // the activations kept for the backward leave from LDS as whole
      // 16-byte row pieces (8 stores per thread instead of 16 scalar stores
      // per row tile per lane); the next layer only reads bufA meanwhile
      if (gout) {
        const int n4 = N / 4;
        for (int e = t; e < BM * n4; e += NT) {
          const int rr = e / n4, c4 = (e - rr * n4) * 4;
          const int64_t row = m0 + rr;
          if (row >= h_from && row < rend)
            *reinterpret_cast<float4*>(&gout[row * ldg + c4]) =
                *reinterpret_cast<const float4*>(&bufA[rr * LDK + c4]);
        }
      }
      continue;
    }
    for (int ct = w / RG; ct < (N + 31) / 32; ct += NCW) {
      const int n = ct * 32 + li;
      f32x16 acc[RTW];
      mma(acc, n);
      epi(acc, n, bufB, true);
    }
    if (head) return;
    __syncthreads();
    float* tmp = bufA; bufA = bufB; bufB = tmp;  // (INPLACE never gets here for hidden layers)
  }

  // narrow head: out[r][j] = h[r] . Wh[j] + bh[j]
  const float* Wh = d.W[d.n_hidden] + wdel + c * d.sW[d.n_hidden];
  const float* bh = d.b[d.n_hidden] + wdel + c * d.sb[d.n_hidden];
  float* outb = outp;
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
  D3A_CHECK_ARG(d_in->row_mean == nullptr, "d3a_mlp_fwd: row_mean is d3a_mlp_fwd_x6 only");
  // the input-row builder (xg_*) only on the small-pass paths (block_rows 16:
  // mlp_small.hip), without an aux pass
  D3A_CHECK_ARG(d_in->xg_mode == 0 || (d_in->block_rows == 16 && d_in->aux_rows == 0 && x6::xgen_ok(*d_in)),
                "d3a_mlp_fwd: the input-row builder (xg_mode) needs block_rows 16, no aux pass and a "
                "valid builder");
  D3A_CHECK_ARG(d_in->xg_mode != 0 || (d_in->xg_xout == nullptr && d_in->xg_eout == nullptr),
                "d3a_mlp_fwd: xg_xout / xg_eout need the input-row builder (xg_mode)");
  D3A_CHECK_ARG(d_in->hmask == nullptr, "d3a_mlp_fwd: hmask is d3a_q2_fwd_x6 only");
  d3a_mlp_fwd_desc d = *d_in;
  D3A_CHECK_ARG((d.x || d.xg_mode) && d.out, "d3a_mlp_fwd: null input / output");
  D3A_CHECK_ARG(d.n_hidden >= 1 && d.n_hidden <= D3A_MLP_MAX_HIDDEN,
                "d3a_mlp_fwd: 1..D3A_MLP_MAX_HIDDEN hidden layers");
  D3A_CHECK_ARG(d.H % 32 == 0 && d.H >= 32 && d.H <= 256, "d3a_mlp_fwd: H must be 32..256, %32");
  D3A_CHECK_ARG(d.n_in >= 1 && d.n_in <= 256, "d3a_mlp_fwd: n_in must be 1..256");
  D3A_CHECK_ARG(d.n_out >= 1 && d.n_out <= 1024, "d3a_mlp_fwd: n_out must be 1..1024");
  D3A_CHECK_ARG(d.C >= 1 && d.rows >= 0, "d3a_mlp_fwd: bad sizes");
  D3A_CHECK_ARG(d.h_from >= 0, "d3a_mlp_fwd: h_from must be >= 0");
  for (int l = 0; l <= d.n_hidden; ++l)
    D3A_CHECK_ARG(d.W[l] && d.b[l], "d3a_mlp_fwd: null layer parameters");
  // layers after the first (and the head) read W rows with 16-byte loads
  for (int l = 1; l <= d.n_hidden; ++l)
    D3A_CHECK_ARG((reinterpret_cast<uintptr_t>(d.W[l]) & 15) == 0 && d.sW[l] % 4 == 0,
                  "d3a_mlp_fwd: weights after layer 0 must be 16-byte aligned");
  // in-kernel row offsets are 32-bit
  D3A_CHECK_ARG((d.r0 + d.rows) * (int64_t)(d.ldout > d.H ? d.ldout : d.H) < (int64_t(1) << 31),
                "d3a_mlp_fwd: rows x row stride exceeds 2^31");
  D3A_CHECK_ARG(d.aux_rows >= 0, "d3a_mlp_fwd: aux_rows must be >= 0");
  if (d.aux_rows > 0) {
    D3A_CHECK_ARG(d.aux_x && d.aux_out, "d3a_mlp_fwd: aux pass needs aux_x and aux_out");
    D3A_CHECK_ARG(d.aux_wdelta % 4 == 0, "d3a_mlp_fwd: aux_wdelta must keep 16-byte alignment");
    D3A_CHECK_ARG(d.aux_rows * (int64_t)(d.ldout > d.H ? d.ldout : d.H) < (int64_t(1) << 31),
                  "d3a_mlp_fwd: aux rows x row stride exceeds 2^31");
  }
  if (d.rows == 0 && d.aux_rows == 0) return 0;
  // Rows per workgroup, from bench A/B runs (profiles/r01_fused_ab.log):
  // 128 (in-place activations, four row tiles per weight load) for large
  // passes with narrow heads -- 55.8 us against 69.5 (32) / 77.6 (64) on the
  // K2 critic pass, 2 x 15616 rows; 32 (two workgroups per CU) otherwise --
  // 164.9 us against 173.5 (128) / 194.9 (64) on the K3 200-quantile target
  // pass, 2 x 25600 rows, and more workgroups for the 100-2560-row passes
  // [n_in <= 48, 256, 256, 1] over >= 8,192 member-rows: W1 in registers,
  // sub-block pipelined (q2_fwd.hip); block_rows > 0 forces the generic kernel
  static const bool q2_on = [] {
    const char* e = getenv("D3A_FWD_Q2");
    return !(e && e[0] == '0');
  }();
  if (q2_on && d.block_rows == 0 && (d.rows + d.aux_rows) * d.C >= 8192 &&
      q2_fwd_launch(d, (hipStream_t)stream)) {
    D3A_LAUNCH_CHECK("d3a_mlp_fwd");
    return 0;
  }
  D3A_CHECK_ARG(d.presplit.n_jobs == 0 || (d.parts > 1 && x6::x6_split_ok(d.presplit)),
                "d3a_mlp_fwd: presplit jobs only on the parts path, each with src, 16-byte aligned "
                "dst, 1 <= k <= kpad and kpad % 16 == 0");
  D3A_CHECK_ARG((d.philox.n_normal == 0 && d.philox.n_uniform == 0) ||
                    (d.parts > 1 && d.philox.out && d.philox.ctr && d.philox.ticket &&
                     d.philox.n_normal >= 0 && d.philox.n_uniform >= 0),
                "d3a_mlp_fwd: a philox job only on the parts path, with out, ctr and ticket");
  if (d.parts > 1) {
    D3A_CHECK_ARG(d.parts == D3A_MLP_PARTS && d.block_rows == 16 && d.n_hidden == 2 &&
                      d.H == 256 && d.n_in <= 64 && d.n_out <= 32 && d.aux_rows == 0 &&
                      d.s_part >= (int64_t)d.C * d.sout,
                  "d3a_mlp_fwd: parts needs parts == D3A_MLP_PARTS, block_rows 16, two hidden "
                  "layers of 256, n_in <= 64, n_out <= 32, no aux pass, s_part >= C * sout");
    D3A_CHECK_ARG(mlp_parts_launch(d, (hipStream_t)stream),
                  "d3a_mlp_fwd: parts needs 16-byte aligned W[1], biases and activation rows");
    D3A_LAUNCH_CHECK("d3a_mlp_fwd");
    return 0;
  }
  if (d.block_rows == 16) {
    D3A_CHECK_ARG(mlp_small_launch(d, (hipStream_t)stream),
                  "d3a_mlp_fwd: block_rows 16 needs H == 256, n_in <= 256, n_out <= 64 (<= 256 with "
                  "two hidden layers and a 16-byte aligned head) and "
                  "16-byte aligned W[1..], biases and activation rows");
    D3A_LAUNCH_CHECK("d3a_mlp_fwd");
    return 0;
  }
  const int bm = d.block_rows > 0
                     ? d.block_rows
                     : (d.n_out <= 64 && d.rows * d.C >= 16384 ? 128 : 32);
  D3A_CHECK_ARG(bm == 32 || bm == 64 || bm == 128,
                "d3a_mlp_fwd: block_rows must be 0, 16, 32, 64 or 128");
  dim3 grid((unsigned)((d.rows + bm - 1) / bm + (d.aux_rows + bm - 1) / bm), 1, (unsigned)d.C);
  hipStream_t st = (hipStream_t)stream;
  if (bm == 128)
    hipLaunchKernelGGL((mlp_fwd_kernel<128, 8, 4>), grid, dim3(512), 0, st, d);
  else if (bm == 64)
    hipLaunchKernelGGL((mlp_fwd_kernel<64, 8, 2>), grid, dim3(512), 0, st, d);
  else
    hipLaunchKernelGGL((mlp_fwd_kernel<32, 8, 1>), grid, dim3(512), 0, st, d);
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
    float* dxb = to_x ? d.dx + c * d.sdxb : nullptr;
    for (int ct = w; ct < (Kout + 31) / 32; ct += NW) {
      const int k = ct * 32 + li;
      f32x16 acc[RT];
#pragma unroll
      for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
      // B(n, k) = W[n][k]: four rows, one column per lane (coalesced over
      // lanes); columns >= Kout read a clamped column and are dropped
      const int kc = min(k, Kout - 1);
      tile_mfma<RT, 4>(acc, bufA, H, li, lg, [&](int n) {
        float4 r;
        r.x = W[kc + (n + 0) * ldw];
        r.y = W[kc + (n + 1) * ldw];
        r.z = W[kc + (n + 2) * ldw];
        r.w = W[kc + (n + 3) * ldw];
        return r;
      });
      if (k < Kout) {
#pragma unroll
        for (int i = 0; i < RT; ++i) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lg;
            const int64_t row = m0 + m;
            if (to_x) {
              if (row < rows) dxb[(int)(row * d.lddx) + k] = acc[i][r];
            } else {
              const float v = (row < rows && hm[(int)(row * d.ldh) + k] > 0.f) ? acc[i][r] : 0.f;
              bufB[m * LDK + k] = v;
              if (row < rows) dzo[(int)row * H + k] = v;
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
  // in-kernel row offsets are 32-bit
  {
    int64_t ld = d.H;
    if (d.ldh > ld) ld = d.ldh;
    if (d.dx && d.lddx > ld) ld = d.lddx;
    D3A_CHECK_ARG(d.rows * ld < (int64_t(1) << 31), "d3a_mlp_bwd: rows x row stride exceeds 2^31");
  }
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
