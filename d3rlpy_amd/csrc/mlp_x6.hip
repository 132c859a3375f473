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
// A workgroup owns 64 rows of one member; eight waves (two per SIMD).  Every
// layer is the same product shape: wave w computes a transposed 32 x 64 block
// C^T[32 outputs][64 rows] (two v_mfma_f32_32x32x16_bf16 tiles; A = 32 weight
// rows, split from fp32 loads, B = an LDS image of the layer input's parts,
// [row][k]):
//   layer 1: units 32 w .. + 31 over K = n_in (the staged input parts), written
//     as parts to the 64 x 256 activation image;
//   layer 2: units 32 w .. + 31 over K = 256 of that image -- a stream of
//     16 k steps with no barrier, the weight rows four steps ahead;
//   head: after one barrier the layer-2 activations replace the image, and
//     wave w < ceil(n_out / 32) streams outputs 32 w .. + 31 the same way.
// Barriers: input staged, image 1 written, layer 2 read out, image 2 written
// (+ one for row_mean).  Round 5 measured the previous design (layer 1
// produced chunk by chunk inside the layer-2 loop, a barrier per chunk) at
// 71k cycles per workgroup, of which 12.5k were the interleaved production
// and 3.4k its barriers (tools/bench_wide.py ablations).
#include <cstdlib>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"
#include "x6.hpp"

namespace d3a {
namespace {

using namespace x6;

constexpr int W_H = 256;    // hidden width
constexpr int W_RB = 64;    // rows per workgroup
constexpr int W_LDH = 264;  // bf16 stride of an image row (528 B)
constexpr int W_HD = 4;     // weight k steps in flight

template <int XL>
struct WideLds {
  __bf16 x[3][W_RB * (XL + 8)];  // input parts [row][k]
  __bf16 img[3][W_RB * W_LDH];   // layer-1, then layer-2 activation parts [row][unit]
  float rs[8][W_RB];             // row_mean: per-wave output sums [wave][row]
};

// diagnostic phase stamps (STAMPS, D3A_WIDE_STAMPS=1; read with
// d3a_wide_stamps): wave 0 of each workgroup records s_memtime at 0 start,
// 1 input staged, 2 its barrier passed, 3 image 1 written, 4 layer-2 products
// issued, 5 image 2 written, 6 head products issued, 7 outputs stored
constexpr int W_NST = 8;
__device__ unsigned long long wide_stamps[1024 * W_NST];

// o[rt] += W[32 rows][256] x img[64 rows][256]^T for this lane's weight row
// (wrow = row + 8 lh): hr holds the raw fp32 of k steps 0 .. W_HD - 1 on entry;
// each step splits its slot, refills it W_HD steps ahead, then issues twelve
// MFMAs.  With next != nullptr the freed slots are refilled with steps
// 0 .. W_HD - 1 of the next stream (the head's rows) instead.
__device__ __forceinline__ void stream256(const float* wrow, const float* next, float4 (&hr)[W_HD][2],
                                          const __bf16 (&img)[3][W_RB * W_LDH], int li, int lh,
                                          f32x16 (&o)[2]) {
#pragma unroll
  for (int s = 0; s < W_H / 16; ++s) {
    bf16x8 wa[3];
    const int sl = s % W_HD;
    const float v[8] = {hr[sl][0].x, hr[sl][0].y, hr[sl][0].z, hr[sl][0].w,
                        hr[sl][1].x, hr[sl][1].y, hr[sl][1].z, hr[sl][1].w};
    split8(v, wa);
    if (s + W_HD < W_H / 16) {
      hr[sl][0] = *reinterpret_cast<const float4*>(wrow + 16 * (s + W_HD));
      hr[sl][1] = *reinterpret_cast<const float4*>(wrow + 16 * (s + W_HD) + 4);
    } else if (next != nullptr) {
      const int s2 = s + W_HD - W_H / 16;
      hr[sl][0] = *reinterpret_cast<const float4*>(next + 16 * s2);
      hr[sl][1] = *reinterpret_cast<const float4*>(next + 16 * s2 + 4);
    }
    // keep the refill here: the scheduler would sink it to its first use
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      bf16x8 bp[3];
#pragma unroll
      for (int q = 0; q < 3; ++q)
        bp[q] = *reinterpret_cast<const bf16x8*>(&img[q][(32 * rt + li) * W_LDH + 16 * s + 8 * lh]);
      o[rt] = prod6(wa, bp, o[rt]);
    }
  }
}

// bias, ReLU, kept rows to hg, parts into the image: lane holds rows
// 32 rt + li, units 32 w + 8 R + 4 lh + i
template <bool KEEP>
__device__ __forceinline__ void act_to_image(const f32x16 (&o)[2], const float4 (&bv)[4], float* hg, int m0,
                                             int h_from, int rend, int w, int li, int lh,
                                             __bf16 (&img)[3][W_RB * W_LDH]) {
#pragma unroll
  for (int R = 0; R < 4; ++R) {
    const int u = 32 * w + 8 * R + 4 * lh;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int rl = 32 * rt + li;
      const int row = m0 + rl;
      float v[4] = {fmaxf(o[rt][4 * R + 0] + bv[R].x, 0.f), fmaxf(o[rt][4 * R + 1] + bv[R].y, 0.f),
                    fmaxf(o[rt][4 * R + 2] + bv[R].z, 0.f), fmaxf(o[rt][4 * R + 3] + bv[R].w, 0.f)};
      if (KEEP && hg != nullptr && row >= h_from && row < rend)
        *reinterpret_cast<float4*>(hg + row * W_H + u) = make_float4(v[0], v[1], v[2], v[3]);
      bf16x4 p[3];
      split4(v, p);
#pragma unroll
      for (int q = 0; q < 3; ++q) *reinterpret_cast<bf16x4*>(&img[q][rl * W_LDH + u]) = p[q];
    }
  }
}

// XL: n_in rounded up to 32 (32 or 64); KEEP: some kept activations (h[0] /
// h[1]) are written (without them no store precedes the head's)
template <int XL, bool KEEP, bool STAMPS = false>
__global__ __launch_bounds__(512) void mlp_x6_wide_kernel(d3a_mlp_fwd_desc d) {
  constexpr int XLD = XL + 8;
  constexpr int NS1 = XL / 16;  // layer-1 k steps
  __shared__ __attribute__((aligned(16))) WideLds<XL> L;
  static_assert(sizeof(WideLds<XL>) <= 163840, "LDS");
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int c = blockIdx.z;
  const int m0 = (int)d.r0 + (int)blockIdx.x * W_RB;
  const int rend = (int)(d.r0 + d.rows);
  const int h_from = (int)d.h_from;
  const int nin = d.n_in, nout = d.n_out;
  float* const outp = d.out + c * d.sout;
  float* const h0g = KEEP && d.h[0] ? d.h[0] + c * d.sh : nullptr;
  float* const h1g = KEEP && d.h[1] ? d.h[1] + c * d.sh : nullptr;
  const int u0 = 32 * w + li;  // this lane's weight row in layers 1 and 2
  const float* W0r = d.W[0] + c * d.sW[0] + u0 * nin;
  const float* W1r = d.W[1] + c * d.sW[1] + u0 * W_H + 8 * lh;
  const float* b0 = d.b[0] + c * d.sb[0];
  const float* b1 = d.b[1] + c * d.sb[1];
  const float* Wh = d.W[2] + c * d.sW[2];
  const float* bh = d.b[2] + c * d.sb[2];
  const int nkt = (nout + 31) / 32;
  const int kout = 32 * w + li;  // head: this lane's output row (rows past n_out read row 0:
  const float* whr = Wh + (kout < nout ? kout : 0) * W_H + 8 * lh;  // never stored)
  const int wgi = blockIdx.x + blockIdx.z * gridDim.x;
  auto stamp = [&](int k) {
    if constexpr (STAMPS) {
      __builtin_amdgcn_sched_barrier(0);
      if (t == 0 && wgi < 1024) wide_stamps[wgi * W_NST + k] = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  stamp(0);

  // ---- prologue: layer-2 weight steps 0 .. W_HD - 1, the layer-1 weight row
  // (clamped k, masked at use) and both biases in flight; input rows split
  // into LDS (input4_at: every load issued before any is used)
  float4 hr[W_HD][2];
#pragma unroll
  for (int s = 0; s < W_HD; ++s) {
    hr[s][0] = *reinterpret_cast<const float4*>(W1r + 16 * s);
    hr[s][1] = *reinterpret_cast<const float4*>(W1r + 16 * s + 4);
  }
  float w0r[NS1][8];
#pragma unroll
  for (int s = 0; s < NS1; ++s)
#pragma unroll
    for (int i = 0; i < 8; ++i) w0r[s][i] = W0r[min(16 * s + 8 * lh + i, nin - 1)];
  float4 b0v[4], b1v[4];
#pragma unroll
  for (int R = 0; R < 4; ++R) {
    b0v[R] = *reinterpret_cast<const float4*>(b0 + 32 * w + 8 * R + 4 * lh);
    b1v[R] = *reinterpret_cast<const float4*>(b1 + 32 * w + 8 * R + 4 * lh);
  }
  {
    const float* xb = d.x + c * d.sxb;
    const int64_t ldx = d.ldx;
    constexpr int X4 = XL / 4;
    for (int e = t; e < W_RB * X4; e += 512) {
      const int m = e / X4, k4 = (e - m * X4) * 4;
      float v[4];
      input4_at(d, xb, ldx, m0 + m, k4, rend, nin, v);
      bf16x4 p[3];
      split4(v, p);
#pragma unroll
      for (int q = 0; q < 3; ++q) *reinterpret_cast<bf16x4*>(&L.x[q][m * XLD + k4]) = p[q];
    }
  }
  stamp(1);
  __syncthreads();  // input parts staged
  stamp(2);

  // ---- layer 1: units 32 w .. over K = XL (x parts past n_in are zero, the
  // weights there masked to zero)
  f32x16 o[2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[rt][r] = 0.f;
#pragma unroll
  for (int s = 0; s < NS1; ++s) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 16 * s + 8 * lh + i < nin ? w0r[s][i] : 0.f;
    bf16x8 wa[3];
    split8(v, wa);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      bf16x8 bp[3];
#pragma unroll
      for (int q = 0; q < 3; ++q)
        bp[q] = *reinterpret_cast<const bf16x8*>(&L.x[q][(32 * rt + li) * XLD + 16 * s + 8 * lh]);
      o[rt] = prod6(wa, bp, o[rt]);
    }
  }
  act_to_image<KEEP>(o, b0v, h0g, m0, h_from, rend, w, li, lh, L.img);
  __syncthreads();  // image 1 complete
  stamp(3);

  // ---- layer 2: units 32 w .. over the image; the head's first weight
  // steps follow in the freed slots
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[rt][r] = 0.f;
  stream256(W1r, w < nkt ? whr : nullptr, hr, L.img, li, lh, o);
  stamp(4);
  __syncthreads();  // every wave done reading image 1
  act_to_image<KEEP>(o, b1v, h1g, m0, h_from, rend, w, li, lh, L.img);
  // head bias of this lane's outputs 32 w + 8 R + 4 lh + i (clamped index)
  float bhv[4][4];
#pragma unroll
  for (int R = 0; R < 4; ++R)
#pragma unroll
    for (int i = 0; i < 4; ++i) bhv[R][i] = bh[min(32 * w + 8 * R + 4 * lh + i, nout - 1)];
  __syncthreads();  // image 2 complete
  stamp(5);

  // ---- head: wave w < nkt computes outputs 32 w .. + 31
  if (w < nkt) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[rt][r] = 0.f;
    stream256(whr, nullptr, hr, L.img, li, lh, o);
    stamp(6);
    // lane: row 32 rt + li, outputs 32 w + 8 R + 4 lh + i
    const int64_t ldo = d.ldout;
    float rsum[2] = {0.f, 0.f};  // row_mean: this lane's outputs, in output order
    const bool vec = ((reinterpret_cast<uintptr_t>(outp) & 15) == 0) && (ldo & 3) == 0;
#pragma unroll
    for (int R = 0; R < 4; ++R) {
      const int k0 = 32 * w + 8 * R + 4 * lh;
      float bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) bv[i] = k0 + i < nout ? bhv[R][i] : 0.f;
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
  stamp(7);
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
  static const bool stamps = [] {
    const char* e = getenv("D3A_WIDE_STAMPS");
    return e && atoi(e) != 0;
  }();
  const bool keep = d.h[0] != nullptr || d.h[1] != nullptr;
  if (stamps && d.n_in <= 32 && !keep)
    hipLaunchKernelGGL((mlp_x6_wide_kernel<32, false, true>), grid, dim3(512), 0, st, d);
  else if (d.n_in <= 32 && keep)
    hipLaunchKernelGGL((mlp_x6_wide_kernel<32, true>), grid, dim3(512), 0, st, d);
  else if (d.n_in <= 32)
    hipLaunchKernelGGL((mlp_x6_wide_kernel<32, false>), grid, dim3(512), 0, st, d);
  else if (keep)
    hipLaunchKernelGGL((mlp_x6_wide_kernel<64, true>), grid, dim3(512), 0, st, d);
  else
    hipLaunchKernelGGL((mlp_x6_wide_kernel<64, false>), grid, dim3(512), 0, st, d);
  D3A_LAUNCH_CHECK("d3a_mlp_fwd_x6");
  return 0;
}

// diagnostic (synchronous, not for graphs): the stamps of the last
// D3A_WIDE_STAMPS=1 launch, [workgroup][8]
extern "C" int d3a_wide_stamps(unsigned long long* dst, int n) {
  D3A_CHECK_ARG(dst && n >= 0 && n <= 1024 * W_NST, "d3a_wide_stamps: bad arguments");
  if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(d3a::wide_stamps), (size_t)n * 8, 0,
                          hipMemcpyDeviceToHost) != hipSuccess) {
    set_error("d3a_wide_stamps: copy failed");
    return -1;
  }
  return 0;
}
