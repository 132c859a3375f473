// Bandwidth-bound helpers: 1-output heads, column reductions (bias / head
// weight gradients), relu-masked outer products, Adam, soft target update and
// the Philox noise generator.  All loads are coalesced along the contiguous
// (feature) dimension; reductions are in a fixed order (deterministic).
#include <cstdarg>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

namespace {

// ---- rowdot: one wave per row, 4 floats per lane per step -------------------
// out[r][j] = x[r] . w[j] + bias[j] for the J (<= 16) outputs of a narrow head;
// w is [J][n] (nn.Linear layout), out rows have stride J.
__global__ __launch_bounds__(256) void rowdot_kernel(const float* X, int64_t sXb, int64_t sXr,
                                                     const float* w, int64_t swb,
                                                     const float* bias, int64_t sbb, float* out,
                                                     int64_t sOb, int64_t rows, int64_t n, int J,
                                                     int64_t dX, int64_t dw, int64_t dbias,
                                                     int64_t dout) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t b = blockIdx.y, t = blockIdx.z;
  if (r >= rows) return;
  const float* x = X + b * sXb + t * dX + r * sXr;
  const float* wb = w + b * swb + t * dw;
  out += t * dout;
  if (bias) bias += t * dbias;
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  const bool vec = ((n & 3) == 0) && ((reinterpret_cast<uintptr_t>(x) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(wb) & 15) == 0);
  if (vec) {
    for (int64_t k = (int64_t)lane * 4; k < n; k += 256) {
      const float4 a = *reinterpret_cast<const float4*>(x + k);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (j >= J) break;
        const float4 c = *reinterpret_cast<const float4*>(wb + j * n + k);
        acc[j] = fmaf(a.w, c.w, fmaf(a.z, c.z, fmaf(a.y, c.y, fmaf(a.x, c.x, acc[j]))));
      }
    }
  } else {
    for (int64_t k = lane; k < n; k += 64) {
      const float a = x[k];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (j >= J) break;
        acc[j] = fmaf(a, wb[j * n + k], acc[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (j >= J) break;
    const float v = wave_sum(acc[j]);
    if (lane == 0) out[b * sOb + r * J + j] = v + (bias ? bias[b * sbb + j] : 0.f);
  }
}

// ---- colreduce: column tile of TW columns x RL row lanes per 256-thread block
// thread t: column (t % TW), row lane (t / TW) walks rows r0+rl, r0+rl+RL, ...;
// the RL partial sums are combined through LDS in a fixed order (deterministic).
__global__ __launch_bounds__(256) void colreduce_kernel(const float* X, int64_t sXb, int64_t sXr,
                                                        const float* w, int64_t swb, float* out,
                                                        int64_t sOb, int64_t sOs, int64_t rows,
                                                        int64_t n, int64_t splits, int TW) {
  __shared__ double part[256];
  const int t = threadIdx.x;
  const int RL = 256 / TW;
  const int cl = t % TW, rl = t / TW;
  const int64_t j = (int64_t)blockIdx.x * TW + cl;
  const int64_t s = blockIdx.y, b = blockIdx.z;
  const int64_t chunk = (rows + splits - 1) / splits;
  const int64_t r0 = s * chunk;
  const int64_t r1 = (r0 + chunk < rows) ? r0 + chunk : rows;
  // fp64 accumulation: bias / head gradients sum thousands of mixed-sign rows
  double acc = 0.0;
  if (j < n) {
    const float* x = X + b * sXb + j;
    const float* wb = w ? w + b * swb : nullptr;
    if (wb) {
      for (int64_t r = r0 + rl; r < r1; r += RL) acc += (double)(wb[r] * x[r * sXr]);
    } else {
      for (int64_t r = r0 + rl; r < r1; r += RL) acc += (double)x[r * sXr];
    }
  }
  part[t] = acc;
  __syncthreads();
  if (rl == 0 && j < n) {
    double tot = 0.0;
    for (int q = 0; q < RL; ++q) tot += part[q * TW + cl];
    out[b * sOb + s * sOs + j] = (float)tot;
  }
}

// ---- outer_mask: out[r][j] = g[r] * w[j] * (h[r][j] > 0) ------------------
__global__ __launch_bounds__(256) void outer_mask_kernel(const float* g, int64_t sgb,
                                                         const float* w, int64_t swb,
                                                         const float* h, int64_t shb, float* out,
                                                         int64_t sob, int64_t rows, int64_t n) {
  const int64_t b = blockIdx.y;
  const int64_t total = rows * n;
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= total) return;
  const float* hb = h + b * shb;
  float* ob = out + b * sob;
  const float* wb = w + b * swb;
  const float* gb = g + b * sgb;
  if ((n & 3) == 0) {
    const int64_t r = i / n, j = i % n;
    const float4 hv = *reinterpret_cast<const float4*>(hb + i);
    const float4 wv = *reinterpret_cast<const float4*>(wb + j);
    const float gv = gb[r];
    float4 o;
    o.x = hv.x > 0.f ? gv * wv.x : 0.f;
    o.y = hv.y > 0.f ? gv * wv.y : 0.f;
    o.z = hv.z > 0.f ? gv * wv.z : 0.f;
    o.w = hv.w > 0.f ? gv * wv.w : 0.f;
    *reinterpret_cast<float4*>(ob + i) = o;
  } else {
    for (int q = 0; q < 4 && i + q < total; ++q) {
      const int64_t e = i + q, r = e / n, j = e % n;
      ob[e] = hb[e] > 0.f ? gb[r] * wb[j] : 0.f;
    }
  }
}

// ---- split-K partials: sum_q grad[q][i] in fp64 in a fixed order (run-to-run
// bit-identical).  A segment with many partials (>= 64, e.g. one per batch
// row) gives each element a group of L = 16 lanes: lane j sums partials
// q = j, j + L, ... in order, then the group is summed by a fixed butterfly.
// A lane issues up to 32 loads before it adds (clamped addresses, so short
// segments take one memory round trip too); the addition order is q ascending.
// lanes per element summing a segment's partials: 16 (strided over the
// partials, combined in a fixed order) for >= 64 partials, else 1 (measured
// on K5's 32,768-element embedding weight with 256 partials: one lane per
// element walking them coalesced, 32 loads in flight, took the Adam launch
// from 80.4 to 85.6 us -- the 16-lane walk keeps more loads in flight)
__host__ __device__ __forceinline__ int seg_lanes(int64_t n_partials, int64_t numel) {
  (void)numel;
  return n_partials >= 64 ? 16 : 1;
}

// elements per thread: 4 for large one-lane segments whose size is a
// multiple of 4 (16-byte state / partial loads where the pointers allow --
// K5's 1.6 M fc weights were a thread each: its Adam 41.6 -> 34.4 us), else 1
// (K2's 65 K-weight critic segments at 4 a thread filled a third of the
// chip: 6.6 -> 7.2 us); threads per segment = numel * L / V (nets.py
// AdamGroup counts the blocks by the same rule)
__host__ __device__ __forceinline__ int seg_vec(int64_t n_partials, int64_t numel) {
  return (seg_lanes(n_partials, numel) == 1 && numel % 4 == 0 && numel >= (1 << 18)) ? 4 : 1;
}
__host__ __device__ __forceinline__ int64_t seg_threads(int64_t n_partials, int64_t numel) {
  return numel * seg_lanes(n_partials, numel) / seg_vec(n_partials, numel);
}

// Offsets are 32-bit bytes from the segment's (uniform) base: one VGPR per
// load address instead of two (a segment's partials are < 4 GiB: nets.py
// AdamGroup checks), which took adam_kernel from 142 VGPRs (3 waves a SIMD,
// every launch a dozen latency rounds) to the 8-wave range.
// Lt: lanes of the closing butterfly (L, or 1 where the caller combines the
// L slots itself: the slot-major 16-lane blocks)
template <int U>
__device__ __forceinline__ double sum_partials_u(const float* g, int64_t n, int64_t stride,
                                                 int64_t i, int j, int L, int Lt) {
  double gd = 0.0;
  const char* gb = reinterpret_cast<const char*>(g);
  const uint32_t n32 = (uint32_t)n, s4 = (uint32_t)stride * 4u, i4 = (uint32_t)i * 4u;
  for (uint32_t q = (uint32_t)j; q < n32; q += (uint32_t)(U * L)) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // a clamped (always valid) address: the loads stay unconditional, so
      // none of them is fenced behind a branch and all are in flight at once
      const uint32_t qq = q + (uint32_t)(u * L);
      v[u] = *reinterpret_cast<const float*>(gb + ((qq < n32 ? qq : n32 - 1u) * s4 + i4));
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (q + (uint32_t)(u * L) < n32) gd += (double)v[u];
  }
  for (int o = Lt >> 1; o > 0; o >>= 1) gd += __shfl_xor(gd, o, 64);
  return gd;
}

// The 16-lane groups (>= 64 partials) run slot-major: in a 256-thread block
// slot j = thread / 16 of element base + thread % 16, so one load instruction
// of a wave reads 64 contiguous bytes of each of four partial rows (the
// element-major groups read 16 bytes of each of sixteen); the block combines
// the sixteen slot sums through LDS with the butterfly's pairing -- the same
// additions, so the same value (fp64 addition commutes).
__device__ __forceinline__ double slot_tree16(const double (&r)[16][16], int e) {
  double a8[8], b4[4];
#pragma unroll
  for (int k = 0; k < 8; ++k) a8[k] = r[k][e] + r[k + 8][e];
#pragma unroll
  for (int k = 0; k < 4; ++k) b4[k] = a8[k] + a8[k + 4];
  return (b4[0] + b4[2]) + (b4[1] + b4[3]);
}

// four consecutive elements' partial sums (one lane, q ascending, fp64: the
// one-lane order of sum_partials_u), 16-byte loads; at most 8 in flight
__device__ __forceinline__ void sum_partials4(const float* g, int64_t n, int64_t stride,
                                              int64_t i, double (&gd)[4]) {
  const char* gb = reinterpret_cast<const char*>(g);
  const uint32_t n32 = (uint32_t)n, s4 = (uint32_t)stride * 4u, i4 = (uint32_t)i * 4u;
  constexpr int U = 8;
  for (uint32_t q = 0; q < n32; q += U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t qq = q + (uint32_t)u;
      v[u] = *reinterpret_cast<const float4*>(gb + ((qq < n32 ? qq : n32 - 1u) * s4 + i4));
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (q + (uint32_t)u < n32) {
        gd[0] += (double)v[u].x;
        gd[1] += (double)v[u].y;
        gd[2] += (double)v[u].z;
        gd[3] += (double)v[u].w;
      }
  }
}

// the partial sum of element i in index order; the batch of loads in flight is
// sized to the partial count (8 for the critic's slice-backward row blocks: a
// 32-load batch would issue 24 clamped duplicates per element), the same
// order and sum for every batch size
// (the batch: the lane's partial count rounded up to a power of two, at most
// 16 -- K5's 128 embedding-weight partials over 16 lanes are eight a lane: a
// 32-load batch issued 24 clamped duplicates each; the fc's 4 split-K
// partials 4 of 8)
__device__ __forceinline__ double sum_partials(const float* g, int64_t n, int64_t stride,
                                               int64_t i, int j, int L, int Lt) {
  const int64_t per = (n + L - 1) / L;  // uniform over the segment
  if (per <= 1) return sum_partials_u<1>(g, n, stride, i, j, L, Lt);
  if (per <= 2) return sum_partials_u<2>(g, n, stride, i, j, L, Lt);
  if (per <= 4) return sum_partials_u<4>(g, n, stride, i, j, L, Lt);
  if (per <= 8) return sum_partials_u<8>(g, n, stride, i, j, L, Lt);
  return sum_partials_u<16>(g, n, stride, i, j, L, Lt);
}

// ---- Adam (torch.optim.adam._single_tensor_adam, weight_decay = 0) ---------
// The grid is flat over the segments: segment s owns ceil(numel_s * L_s / 256)
// consecutive blocks, in table order (no idle blocks for small segments).
// Wave 0 finds the block's segment: lane s reads segment s's block count and a
// wave prefix sum gives every segment's first block (one memory round trip for
// up to 64 segments, instead of one per segment walked).
__device__ __forceinline__ void locate_block(const d3a_adam_segment* segs, int n_seg, int* s_seg,
                                             int64_t* s_first) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  const long long b = blockIdx.x;
  long long base = 0;
  for (int c = 0; c < n_seg; c += 64) {
    const int s = c + lane;
    long long nb = 0;
    if (s < n_seg) nb = (seg_threads(segs[s].n_partials, segs[s].numel) + 255) / 256;
    long long incl = nb;
    for (int o = 1; o < 64; o <<= 1) {
      const long long t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    const long long first = base + incl - nb;
    // the last segment also owns any block past the end (as the serial walk did)
    const bool own = s < n_seg && b >= first && (b < base + incl || s == n_seg - 1);
    if (own) {
      *s_seg = s;
      *s_first = first;
    }
    if (__ballot(own)) break;
    base += __shfl(incl, 63, 64);
  }
}

template <bool VEC>
__global__ __launch_bounds__(256, VEC ? 6 : 8) void adam_kernel(d3a_adam_desc a) {
  __shared__ float s_step_size, s_bc2_sqrt;
  __shared__ int s_seg;
  __shared__ int64_t s_first;
  const d3a_adam_segment* segs = a.segs;
  const int n_seg = a.n_seg;
  const double beta1 = a.beta1, beta2 = a.beta2;
  const float grad_scale = (float)a.grad_scale;
  // t: the optimiser's step for this update (*step completed steps + 1, or a
  // counter another kernel of the update already advanced: step_add 0)
  const int64_t t = *a.step + a.step_add;
  // block 0 also does the update's bookkeeping (d3a_step_end's, for counters
  // this launch does not read): the metric ring push and counter increments
  const bool tail = blockIdx.x == 0;
  int64_t rc0 = 0;
  if (tail && a.ring && (int)threadIdx.x < a.n_metrics) {
    const float mk = a.metrics[threadIdx.x];
    rc0 = *a.ring_ctr;
    a.ring[(rc0 % a.ring_cap) * a.n_metrics + threadIdx.x] =
        a.metric_scale == 1.f ? mk : mk * a.metric_scale;
  }
  if (a.blocks == nullptr) locate_block(segs, n_seg, &s_seg, &s_first);
  if (threadIdx.x == 64) {  // wave 1, concurrently with wave 0's segment search
    // bias corrections in fp64 exactly as torch computes them in Python floats
    const double bc1 = 1.0 - pow(beta1, (double)t);
    const double bc2 = 1.0 - pow(beta2, (double)t);
    s_step_size = (float)(a.lr / bc1);
    s_bc2_sqrt = (float)sqrt(bc2);
  }
  // per-block table: the segment is one (scalar) load, and the state and
  // partial loads go out before the barrier (the bias-correction pows of wave
  // 1 run under them); else the search's result after the barrier
  const bool tab = a.blocks != nullptr;
  if (!tab) __syncthreads();  // (block 0: every ring writer has read *ring_ctr)
  const d3a_adam_segment sg = tab ? a.blocks[blockIdx.x].seg : segs[s_seg];
  const int64_t first = tab ? a.blocks[blockIdx.x].first : s_first;
  const int L = seg_lanes(sg.n_partials, sg.numel);
  // (VEC false: the host's one_elem -- no segment has seg_vec 4)
  const int V = VEC ? seg_vec(sg.n_partials, sg.numel) : 1;
  const int64_t lt = ((int64_t)blockIdx.x - first) * 256 + threadIdx.x;
  const bool smj = L == 16;  // slot-major 16-lane block (uniform)
  // the thread's first element, and its partial slot
  const int64_t i = V == 4 ? lt * 4 : smj ? ((int64_t)blockIdx.x - first) * 16 + (threadIdx.x & 15) : lt / L;
  const int slot = smj ? (int)(threadIdx.x >> 4) : (int)(lt % L);
  const bool act = i < sg.numel;
  float* tg = a.soft ? sg.param + a.targ_delta : nullptr;
  // 16-byte accesses when every stream is 16-byte aligned (a flat store's
  // segment offsets need not be), else four scalar ones
  const bool v4 = V == 4 && sg.partial_stride % 4 == 0 &&
                  ((reinterpret_cast<uintptr_t>(sg.param) | reinterpret_cast<uintptr_t>(sg.exp_avg) |
                    reinterpret_cast<uintptr_t>(sg.exp_avg_sq) | reinterpret_cast<uintptr_t>(sg.grad) |
                    reinterpret_cast<uintptr_t>(sg.grad_out) | reinterpret_cast<uintptr_t>(tg)) & 15) == 0;
  const bool lead = V == 4 || slot == 0;
  float m[4] = {}, v[4] = {}, p[4] = {}, tv[4] = {};
  double gd[4] = {};
  if (act) {
    // the state loads go out with the partial loads (one round trip for both)
    if (v4) {
      const float4 m4 = *reinterpret_cast<const float4*>(sg.exp_avg + i);
      const float4 v4_ = *reinterpret_cast<const float4*>(sg.exp_avg_sq + i);
      const float4 p4 = *reinterpret_cast<const float4*>(sg.param + i);
      m[0] = m4.x, m[1] = m4.y, m[2] = m4.z, m[3] = m4.w;
      v[0] = v4_.x, v[1] = v4_.y, v[2] = v4_.z, v[3] = v4_.w;
      p[0] = p4.x, p[1] = p4.y, p[2] = p4.z, p[3] = p4.w;
      if (tg) {
        const float4 t4 = *reinterpret_cast<const float4*>(tg + i);
        tv[0] = t4.x, tv[1] = t4.y, tv[2] = t4.z, tv[3] = t4.w;
      }
      sum_partials4(sg.grad, sg.n_partials, sg.partial_stride, i, gd);
    } else {
      for (int e = 0; e < V; ++e) {
        if (lead) {
          m[e] = sg.exp_avg[i + e];
          v[e] = sg.exp_avg_sq[i + e];
          p[e] = sg.param[i + e];
          if (tg) tv[e] = tg[i + e];
        }
        gd[e] = sum_partials(sg.grad, sg.n_partials, sg.partial_stride, i + e,
                             V == 4 ? 0 : slot, V == 4 ? 1 : L, V == 4 || smj ? 1 : L);
      }
    }
  }
  if (smj) {  // uniform: the sixteen slots' sums meet in LDS
    __shared__ double s_red[16][16];
    s_red[slot][threadIdx.x & 15] = gd[0];
    __syncthreads();
    if (lead) gd[0] = slot_tree16(s_red, threadIdx.x & 15);
  }
  if (tab) __syncthreads();  // s_step_size; block 0: every ring writer has read *ring_ctr
  if (tail) {
    if (a.ring && threadIdx.x == 0) *a.ring_ctr = rc0 + 1;
    if (threadIdx.x < 32 && (a.inc_mask >> threadIdx.x & 1u)) a.counters[threadIdx.x] += 1;
    // the scalar state an earlier launch staged (d3a_cql_loss_desc.stage)
    if ((int)threadIdx.x < a.n_commit) *a.commit_dst[threadIdx.x] = a.commit_src[threadIdx.x];
    if (threadIdx.x >= 64 && threadIdx.x < 66 && a.commit_step[threadIdx.x - 64])
      *a.commit_step[threadIdx.x - 64] += 1;
  }
  if (act) {  // uniform over each lane group
    if (!lead) return;
    const float step_size = s_step_size;
    const float bc2_sqrt = s_bc2_sqrt;
    float gs[4] = {}, tn[4] = {};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e >= V) break;
      // grad_scale: 1, or 1/world after a data-parallel SUM all-reduce (exact
      // for power-of-two worlds)
      const float g = grad_scale == 1.f ? (float)gd[e] : __fmul_rn((float)gd[e], grad_scale);
      gs[e] = g;
      // exp_avg.lerp_(grad, 1 - beta1): weight < 0.5 -> self + w * (end - self)
      // (ATen's vectorised CPU lerp: fmadd(weight, end - self, self))
      const float w = (float)(1.0 - beta1);
      m[e] = fmaf(w, __fsub_rn(g, m[e]), m[e]);
      // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
      v[e] = __fmul_rn(v[e], (float)beta2);
      const float omb2 = (float)(1.0 - beta2);
      v[e] = __fadd_rn(v[e], __fmul_rn(__fmul_rn(omb2, g), g));
      const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(v[e]), bc2_sqrt), (float)a.eps);
      p[e] = __fadd_rn(p[e], __fmul_rn(-step_size, __fdiv_rn(m[e], denom)));
      // soft_sync of the target copy from the updated parameter, the three
      // separately rounded ops of d3a_soft_update_f32 (torch_utility.py:27-33)
      if (tg) tn[e] = __fadd_rn(__fmul_rn(tv[e], (float)(1.0 - a.tau)), __fmul_rn((float)a.tau, p[e]));
    }
    if (v4) {
      if (sg.grad_out) *reinterpret_cast<float4*>(sg.grad_out + i) = make_float4(gs[0], gs[1], gs[2], gs[3]);
      *reinterpret_cast<float4*>(sg.exp_avg + i) = make_float4(m[0], m[1], m[2], m[3]);
      *reinterpret_cast<float4*>(sg.exp_avg_sq + i) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(sg.param + i) = make_float4(p[0], p[1], p[2], p[3]);
      if (tg) *reinterpret_cast<float4*>(tg + i) = make_float4(tn[0], tn[1], tn[2], tn[3]);
    } else {
      for (int e = 0; e < V; ++e) {
        if (sg.grad_out) sg.grad_out[i + e] = gs[e];
        sg.exp_avg[i + e] = m[e];
        sg.exp_avg_sq[i + e] = v[e];
        sg.param[i + e] = p[e];
        if (tg) tg[i + e] = tn[e];
      }
    }
  }
  // the step counter this launch reads is committed by another kernel
  // (d3a_step_end, or a later d3a_adam_step's inc_mask)
}

// ---- split-K partials -> one gradient (the data-parallel path reduces
// before the all-reduce, so the collective moves one copy, not S partials)
__global__ __launch_bounds__(256) void grad_reduce_kernel(const d3a_adam_segment* segs,
                                                          int n_seg) {
  __shared__ int s_seg;
  __shared__ int64_t s_first;
  locate_block(segs, n_seg, &s_seg, &s_first);
  __syncthreads();
  const d3a_adam_segment sg = segs[s_seg];
  const int L = seg_lanes(sg.n_partials, sg.numel);
  const int V = seg_vec(sg.n_partials, sg.numel);
  const int64_t lt = ((int64_t)blockIdx.x - s_first) * 256 + threadIdx.x;
  if (L == 16) {  // slot-major (uniform), as adam_kernel
    __shared__ double s_red[16][16];
    const int e = threadIdx.x & 15, slot = threadIdx.x >> 4;
    const int64_t i = ((int64_t)blockIdx.x - s_first) * 16 + e;
    s_red[slot][e] = i < sg.numel ? sum_partials(sg.grad, sg.n_partials, sg.partial_stride, i, slot, 16, 1) : 0.0;
    __syncthreads();
    if (slot == 0 && i < sg.numel) sg.grad_out[i] = (float)slot_tree16(s_red, e);
    return;
  }
  const int64_t i = V == 4 ? lt * 4 : lt / L;
  if (i >= sg.numel) return;  // uniform over each lane group
  if (V == 4) {
    const bool v4 = sg.partial_stride % 4 == 0 &&
                    ((reinterpret_cast<uintptr_t>(sg.grad) |
                      reinterpret_cast<uintptr_t>(sg.grad_out)) & 15) == 0;
    double gd[4] = {};
    if (v4) {
      sum_partials4(sg.grad, sg.n_partials, sg.partial_stride, i, gd);
      *reinterpret_cast<float4*>(sg.grad_out + i) =
          make_float4((float)gd[0], (float)gd[1], (float)gd[2], (float)gd[3]);
    } else {
      for (int e = 0; e < 4; ++e)
        sg.grad_out[i + e] = (float)sum_partials(sg.grad, sg.n_partials, sg.partial_stride, i + e, 0, 1, 1);
    }
    return;
  }
  const double gd = sum_partials(sg.grad, sg.n_partials, sg.partial_stride, i, (int)(lt % L), L, L);
  if (lt % L) return;
  sg.grad_out[i] = (float)gd;
}

// ---- soft update: fl(fl(p_t * (1 - tau)) + fl(tau * p)) -------------------
__global__ __launch_bounds__(256) void soft_update_kernel(float* targ, const float* src,
                                                          int64_t n, float omt, float tau) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) targ[i] = __fadd_rn(__fmul_rn(targ[i], omt), __fmul_rn(tau, src[i]));
}

// ---- StandardScaler.transform: y = (x - mean) / (std + eps), each op rounded
// as torch's separate fp32 ops (scalers.py:350-354) --------------------------
__global__ __launch_bounds__(256) void standardize_kernel(const float* x, float* y, int64_t rows,
                                                          int D, int64_t ldx, const float* mean,
                                                          const float* std, float eps) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * D) return;
  const int64_t r = i / D;
  const int j = (int)(i - r * D);
  y[r * ldx + j] = __fdiv_rn(__fsub_rn(x[r * ldx + j], mean[j]), __fadd_rn(std[j], eps));
}

// ---- Philox noise ----------------------------------------------------------
__global__ __launch_bounds__(256) void philox_kernel(float* out, int64_t n_normal,
                                                     int64_t n_uniform, float lo, float hi,
                                                     uint64_t seed, int64_t* ctr,
                                                     unsigned int* ticket) {
  const int64_t step = *ctr;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;  // one Philox call -> 4 outputs
  const int64_t total = n_normal + n_uniform;
  const int64_t e0 = g * 4;
  if (e0 < total) {
    for (int q = 0; q < 4; ++q) {
      const int64_t e = e0 + q;
      if (e < total) out[e] = philox_elem(seed, (uint64_t)step, e, n_normal, lo, hi);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = atomicAdd(ticket, 1u);
    if (prev == gridDim.x - 1) {
      *ctr = step + 1;
      *ticket = 0u;
    }
  }
}

// End of an update: soft target update over the whole flat parameter buffer
// (fl(fl(p_t*(1-tau)) + fl(tau*p)), torch_utility.py:27-33) + metric ring push
// + optimiser step counters, in one launch.
__global__ __launch_bounds__(256) void step_end_kernel(const float* m, int n, float* ring,
                                                       int64_t cap, int64_t* ctr,
                                                       int64_t* counters, unsigned inc_mask,
                                                       float* targ, const float* src, int64_t ns,
                                                       float omt, float tau, float mscale) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (targ && i < ns) targ[i] = __fadd_rn(__fmul_rn(targ[i], omt), __fmul_rn(tau, src[i]));
  if (blockIdx.x != 0) return;
  // counters: one lane each, in parallel with the ring push
  if (threadIdx.x < 32 && (inc_mask >> threadIdx.x & 1u)) counters[threadIdx.x] += 1;
  int64_t c0 = 0;
  if (ring) {
    const float mk = threadIdx.x < n ? m[threadIdx.x] : 0.f;  // issued with the ctr load
    c0 = *ctr;
    const int64_t slot = c0 % cap;
    if (threadIdx.x < n) ring[slot * n + threadIdx.x] = mscale == 1.f ? mk : mk * mscale;
    for (int k = threadIdx.x + blockDim.x; k < n; k += blockDim.x)
      ring[slot * n + k] = mscale == 1.f ? m[k] : m[k] * mscale;
  }
  __syncthreads();  // every thread has read *ctr before it moves
  if (ring && threadIdx.x == 0) *ctr = c0 + 1;
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_step_end(const float* metrics, int32_t n, float* ring, int64_t cap,
                            int64_t* ring_ctr, int64_t* counters, uint32_t inc_mask, float* targ,
                            const float* src, int64_t n_soft, double tau, float metric_scale,
                            void* stream) {
  D3A_CHECK_ARG(!ring || (metrics && ring_ctr && n > 0 && cap > 0), "d3a_step_end: bad ring");
  D3A_CHECK_ARG(!inc_mask || counters, "d3a_step_end: counters required");
  D3A_CHECK_ARG(!targ || (src && n_soft >= 0), "d3a_step_end: bad soft-update operands");
  const int64_t ns = targ ? n_soft : 0;
  const unsigned blocks = (unsigned)(ns > 0 ? (ns + 255) / 256 : 1);
  hipLaunchKernelGGL(step_end_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, metrics,
                     n, ring, cap, ring_ctr, counters, inc_mask, targ, src, ns,
                     (float)(1.0 - tau), (float)tau, metric_scale);
  D3A_LAUNCH_CHECK("d3a_step_end");
  return 0;
}

extern "C" int d3a_abi_version(void) { return 1; }

extern "C" const char* d3a_last_error(void) { return d3a::g_err; }

extern "C" int d3a_device_count(int* count) {
  D3A_CHECK_ARG(count != nullptr, "d3a_device_count: null");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  (void)hipGetLastError();
  return 0;
}

extern "C" int d3a_rowdot_f32(const float* X, int64_t sXb, int64_t sXr, const float* w,
                              int64_t swb, const float* bias, int64_t sbb, float* out,
                              int64_t sOb, int64_t batch, int64_t rows, int64_t n,
                              void* stream) {
  return d3a_rowdot2_f32(X, sXb, sXr, w, swb, bias, sbb, out, sOb, batch, rows, n, 1, 1, 0, 0, 0,
                         0, stream);
}

extern "C" int d3a_rowdot2_f32(const float* X, int64_t sXb, int64_t sXr, const float* w,
                               int64_t swb, const float* bias, int64_t sbb, float* out,
                               int64_t sOb, int64_t batch, int64_t rows, int64_t n, int32_t J,
                               int64_t batch2, int64_t dX, int64_t dw, int64_t dbias,
                               int64_t dout, void* stream) {
  D3A_CHECK_ARG(X && w && out, "d3a_rowdot_f32: null pointer");
  D3A_CHECK_ARG(batch2 >= 1, "d3a_rowdot2_f32: batch2 >= 1");
  D3A_CHECK_ARG(J >= 1 && J <= 16, "d3a_rowdot2_f32: 1 <= J <= 16");
  if (batch <= 0 || rows <= 0) return 0;
  dim3 grid((unsigned)((rows + 3) / 4), (unsigned)batch, (unsigned)batch2);
  hipLaunchKernelGGL(rowdot_kernel, grid, dim3(256), 0, (hipStream_t)stream, X, sXb, sXr, w, swb,
                     bias, sbb, out, sOb, rows, n, (int)J, dX, dw, dbias, dout);
  D3A_LAUNCH_CHECK("d3a_rowdot2_f32");
  return 0;
}

extern "C" int d3a_colreduce_f32(const float* X, int64_t sXb, int64_t sXr, const float* w,
                                 int64_t swb, float* out, int64_t sOb, int64_t sOs,
                                 int64_t batch, int64_t rows, int64_t n, int64_t splits,
                                 void* stream) {
  D3A_CHECK_ARG(X && out, "d3a_colreduce_f32: null pointer");
  D3A_CHECK_ARG(splits >= 1, "d3a_colreduce_f32: splits >= 1");
  if (batch <= 0 || n <= 0) return 0;
  int TW = 1;
  while (TW < n && TW < 64) TW <<= 1;  // columns per block (power of two <= 64)
  dim3 grid((unsigned)((n + TW - 1) / TW), (unsigned)splits, (unsigned)batch);
  hipLaunchKernelGGL(colreduce_kernel, grid, dim3(256), 0, (hipStream_t)stream, X, sXb, sXr, w,
                     swb, out, sOb, sOs, rows, n, splits, TW);
  D3A_LAUNCH_CHECK("d3a_colreduce_f32");
  return 0;
}

extern "C" int d3a_outer_mask_f32(const float* g, int64_t sgb, const float* w, int64_t swb,
                                  const float* h, int64_t shb, float* out, int64_t sob,
                                  int64_t batch, int64_t rows, int64_t n, void* stream) {
  D3A_CHECK_ARG(g && w && h && out, "d3a_outer_mask_f32: null pointer");
  if (batch <= 0 || rows <= 0 || n <= 0) return 0;
  const int64_t total4 = (rows * n + 3) / 4;
  dim3 grid((unsigned)((total4 + 255) / 256), (unsigned)batch);
  hipLaunchKernelGGL(outer_mask_kernel, grid, dim3(256), 0, (hipStream_t)stream, g, sgb, w, swb,
                     h, shb, out, sob, rows, n);
  D3A_LAUNCH_CHECK("d3a_outer_mask_f32");
  return 0;
}

extern "C" int d3a_adam_step(const d3a_adam_desc* a, void* stream) {
  D3A_CHECK_ARG(a && a->segs && a->step, "d3a_adam_step: null pointer");
  D3A_CHECK_ARG(a->n_seg > 0 && a->n_seg < 65536, "d3a_adam_step: bad segment count");
  D3A_CHECK_ARG(a->n_blocks >= a->n_seg && a->n_blocks < (1ll << 31),
                "d3a_adam_step: bad n_blocks");
  D3A_CHECK_ARG(a->step_add == 0 || a->step_add == 1, "d3a_adam_step: step_add must be 0 or 1");
  D3A_CHECK_ARG(!a->inc_mask || a->counters, "d3a_adam_step: counters required");
  D3A_CHECK_ARG(a->n_commit >= 0 && a->n_commit <= 8 && (a->n_commit == 0 || a->commit_src),
                "d3a_adam_step: n_commit in [0, 8] with commit_src");
  D3A_CHECK_ARG(!a->ring || (a->metrics && a->ring_ctr && a->n_metrics >= 1 &&
                             a->n_metrics <= 256 && a->ring_cap > 0),
                "d3a_adam_step: bad metric ring");
  D3A_CHECK_ARG(!a->soft || a->targ_delta != 0, "d3a_adam_step: soft update needs targ_delta");
  if (a->one_elem)
    hipLaunchKernelGGL(adam_kernel<false>, dim3((unsigned)a->n_blocks), dim3(256), 0,
                       (hipStream_t)stream, *a);
  else
    hipLaunchKernelGGL(adam_kernel<true>, dim3((unsigned)a->n_blocks), dim3(256), 0,
                       (hipStream_t)stream, *a);
  D3A_LAUNCH_CHECK("d3a_adam_step");
  return 0;
}

extern "C" int d3a_adam_f32(const d3a_adam_segment* segs, int32_t n_seg, int64_t n_blocks,
                            const int64_t* step, double lr, double beta1, double beta2,
                            double eps, double grad_scale, void* stream) {
  d3a_adam_desc a;
  memset(&a, 0, sizeof(a));
  a.segs = segs;
  a.n_seg = n_seg;
  a.n_blocks = n_blocks;
  a.step = step;
  a.step_add = 1;
  a.lr = lr;
  a.beta1 = beta1;
  a.beta2 = beta2;
  a.eps = eps;
  a.grad_scale = grad_scale;
  a.metric_scale = 1.f;
  if (segs == nullptr || step == nullptr) {
    set_error("d3a_adam_f32: null pointer");
    return -1;
  }
  const int rc = d3a_adam_step(&a, stream);
  if (rc != 0) {
    // report under this entry point's name
    char buf[512];
    snprintf(buf, sizeof(buf), "%s", d3a_last_error());
    set_error("d3a_adam_f32: %s", buf);
  }
  return rc;
}

extern "C" int d3a_grad_reduce_f32(const d3a_adam_segment* segs, int32_t n_seg,
                                   int64_t n_blocks, void* stream) {
  D3A_CHECK_ARG(segs, "d3a_grad_reduce_f32: null pointer");
  D3A_CHECK_ARG(n_seg > 0 && n_seg < 65536, "d3a_grad_reduce_f32: bad segment count");
  D3A_CHECK_ARG(n_blocks >= n_seg && n_blocks < (1ll << 31), "d3a_grad_reduce_f32: bad n_blocks");
  hipLaunchKernelGGL(grad_reduce_kernel, dim3((unsigned)n_blocks), dim3(256), 0,
                     (hipStream_t)stream, segs, (int)n_seg);
  D3A_LAUNCH_CHECK("d3a_grad_reduce_f32");
  return 0;
}

extern "C" int d3a_standardize_f32(const float* x, float* y, int64_t rows, int32_t D,
                                   int64_t ldx, const float* mean, const float* std, float eps,
                                   void* stream) {
  D3A_CHECK_ARG(x && y && mean && std, "d3a_standardize_f32: null pointer");
  D3A_CHECK_ARG(D >= 1 && ldx >= D && rows >= 0, "d3a_standardize_f32: bad sizes");
  if (rows == 0) return 0;
  hipLaunchKernelGGL(standardize_kernel, dim3((unsigned)((rows * D + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, x, y, rows, D, ldx, mean, std, eps);
  D3A_LAUNCH_CHECK("d3a_standardize_f32");
  return 0;
}

extern "C" int d3a_soft_update_f32(float* targ, const float* src, int64_t n, double tau,
                                   void* stream) {
  D3A_CHECK_ARG(targ && src, "d3a_soft_update_f32: null pointer");
  if (n <= 0) return 0;
  const float omt = (float)(1.0 - tau);
  hipLaunchKernelGGL(soft_update_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, targ, src, n, omt, (float)tau);
  D3A_LAUNCH_CHECK("d3a_soft_update_f32");
  return 0;
}

extern "C" int d3a_philox_fill(float* out, int64_t n_normal, int64_t n_uniform, float lo,
                               float hi, uint64_t seed, int64_t* ctr, unsigned int* ticket,
                               void* stream) {
  D3A_CHECK_ARG(out && ctr && ticket, "d3a_philox_fill: null pointer");
  const int64_t total = n_normal + n_uniform;
  if (total <= 0) return 0;
  const int64_t groups = (total + 3) / 4;
  hipLaunchKernelGGL(philox_kernel, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, out, n_normal, n_uniform, lo, hi, seed, ctr, ticket);
  D3A_LAUNCH_CHECK("d3a_philox_fill");
  return 0;
}
