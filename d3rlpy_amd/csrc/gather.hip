// Minibatch gather from a device-resident MDP dataset.
//
// Reference: TransitionMiniBatch.__cinit__ / _assign_to_batch /
// _assign_observation / _stack_frames (d3rlpy/dataset.pyx:1053-1342) and the
// index stream of RandomIterator._next (d3rlpy/iterators/random_iterator.py:38-41).
//
// Dataset layout in HBM (structure of arrays, built once by
// d3rlpy_amd/dataset.py DeviceDataset):
//   obs[n_rows][D] f32  or  frames[n_rows][frame_bytes] u8   (one row per step)
//   act[n_rows][A] f32  or  act_i[n_rows] i32, rew[n_rows] f32
//   per transition i: t_row (its step row), t_ep_start (first row of its
//   episode), t_ep_last (last transition index of its episode),
//   t_terminal (1 iff its next observation is the all-zero dummy).
// Transitions of one episode have consecutive indices, so next_transition is
// i + 1 unless i == t_ep_last[i].
//
// One workgroup per batch row: lane 0 walks the n-step chain (at most
// n_steps dependent loads), then the whole workgroup copies observation /
// frame bytes with 16-byte accesses.
#include <cstdlib>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

struct RowMeta {
  int64_t t;          // transition index
  int64_t row;        // its step row
  int64_t ep_start;
  int64_t next_row;   // row of next observation (t+n), or -1 for zeros
  int64_t next_t;     // transition index at t+n-1
};

__device__ __forceinline__ void copy_bytes(uint8_t* dst, const uint8_t* src, int64_t n,
                                           int tid, int nt) {
  // 16-byte path when both ends are aligned
  if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0) {
    const int64_t n16 = n >> 4;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (int64_t k = tid; k < n16; k += nt) d4[k] = s4[k];
    for (int64_t k = (n16 << 4) + tid; k < n; k += nt) dst[k] = src[k];
  } else {
    for (int64_t k = tid; k < n; k += nt) dst[k] = src[k];
  }
}

__device__ __forceinline__ void zero_bytes(uint8_t* dst, int64_t n, int tid, int nt) {
  for (int64_t k = tid; k < n; k += nt) dst[k] = 0;
}

__global__ __launch_bounds__(256) void gather_kernel(d3a_gather_desc d, bool batched) {
  __shared__ RowMeta meta;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int64_t b = blockIdx.x;

  if (tid == 0) {
    int64_t t;
    if (d.idx) {
      t = d.idx[b];
    } else {
      uint32_t r[4];
      Philox::gen(d.seed, (uint64_t)(*d.ctr), (uint64_t)(d.row_offset + b), r);
      const uint64_t x = ((uint64_t)r[0] << 32) | r[1];
      t = (int64_t)(x % (uint64_t)d.n_trans);
      d.idx_out[b] = t;
    }
    // every table entry of transition t is requested at once (one memory
    // round trip instead of one per field)
    const int64_t row_t = d.t_row[t], last_t = d.t_ep_last[t], ep_t = d.t_ep_start[t];
    const uint8_t term_t = d.t_terminal[t];
    // n-step return (dataset.pyx:1323-1330)
    float ret = 0.f;
    int64_t nt_i = t, row_i = row_t, last_i = last_t;
    int k = 0;
    for (k = 0; k < d.n_steps; ++k) {
      // n_step_return += reward * gamma ** i   (dataset.pyx:1325): the host's
      // powf(gamma, i) from the descriptor, then one fp32 multiply and one fp32
      // add (no contraction) — the Cython 0.29 codegen, see d3a_gather_desc
      const float gp = d.gamma_pow[k];
      ret = __fadd_rn(ret, __fmul_rn(d.rew[row_i], gp));
      if (nt_i == last_i || k == d.n_steps - 1) break;
      // successor slot; wraps at n_trans for the online replay ring (an
      // offline table never steps past its last transition here)
      nt_i = nt_i + 1 == d.n_trans ? 0 : nt_i + 1;
      row_i = d.t_row[nt_i];
      last_i = d.t_ep_last[nt_i];
    }
    d.o_rew[b] = ret;
    const bool term = (nt_i == t ? term_t : d.t_terminal[nt_i]) != 0;
    d.o_term[b] = d.t_term_value ? d.t_term_value[nt_i] : (term ? 1.f : 0.f);
    d.o_n_steps[b] = (float)(k + 1);
    meta.t = t;
    meta.row = row_t;
    meta.ep_start = ep_t;
    meta.next_t = nt_i;
    meta.next_row = term ? -1 : row_i + 1;
    // actions
    if (d.act_i) d.o_act_i[b] = d.act_i[meta.row];
  }
  __syncthreads();
  const int64_t row = meta.row, nrow = meta.next_row, ep0 = meta.ep_start;

  if (d.act) {
    for (int j = tid; j < d.A; j += nt) d.o_act[b * d.A + j] = d.act[row * d.A + j];
  }
  if (d.obs) {
    const int D = d.D;
    for (int j = tid; j < D; j += nt) {
      d.o_obs[b * D + j] = d.obs[row * D + j];
      d.o_next_obs[b * D + j] = nrow >= 0 ? d.obs[nrow * D + j] : 0.f;
    }
  } else {
    // image observations with frame stacking (dataset.pyx:1053-1096)
    const int64_t fb = d.frame_bytes, nf = d.n_frames;
    uint8_t* o = d.o_frames + b * nf * fb;
    uint8_t* on = d.o_next_frames + b * nf * fb;
    const int64_t n16 = fb >> 4;
    const bool al = ((reinterpret_cast<uintptr_t>(d.frames) | reinterpret_cast<uintptr_t>(o) |
                      reinterpret_cast<uintptr_t>(on) | (uintptr_t)fb) & 15) == 0;
    if (batched && al && nf <= 4 && n16 <= 2 * nt) {
      // every 16-byte piece of the 2 nf frames loaded before any is stored (a
      // copy loop's store would otherwise wait on its load, frame by frame)
      uint4 v[8][2];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int q = i & 3;
        const bool nx = i >= 4;
        const bool live = q < nf && !(nx && nrow < 0);
        const int64_t base = nx ? nrow : row;
        const int64_t r = (base - q > ep0) ? base - q : ep0;
        const uint4* s4 = reinterpret_cast<const uint4*>(d.frames + r * fb);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int64_t k = tid + (int64_t)j * nt;
          v[i][j] = (live && k < n16) ? s4[k] : make_uint4(0u, 0u, 0u, 0u);
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int q = i & 3;
        if (q >= nf) continue;
        uint4* d4 = reinterpret_cast<uint4*>((i >= 4 ? on : o) + (nf - 1 - q) * fb);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int64_t k = tid + (int64_t)j * nt;
          if (k < n16) d4[k] = v[i][j];
        }
      }
    } else {
    for (int64_t q = 0; q < nf; ++q) {
      // slot nf-1-q holds the frame q steps back, clamped at the episode start
      const int64_t r = (row - q > ep0) ? row - q : ep0;
      copy_bytes(o + (nf - 1 - q) * fb, d.frames + r * fb, fb, tid, nt);
      if (nrow < 0) {
        zero_bytes(on + (nf - 1 - q) * fb, fb, tid, nt);
      } else {
        const int64_t rn = (nrow - q > ep0) ? nrow - q : ep0;
        copy_bytes(on + (nf - 1 - q) * fb, d.frames + rn * fb, fb, tid, nt);
      }
    }
    }
  }

  // advance the sampler counter once every block has drawn its index
  if (!d.idx) {
    __syncthreads();
    if (tid == 0) {
      const unsigned prev = atomicAdd(d.ticket, 1u);
      if (prev == gridDim.x - 1) {
        *d.ctr = *d.ctr + 1;
        *d.ticket = 0u;
      }
    }
  }
}

// Vector observations: one wave per batch row, four rows per workgroup.  The
// index draw is lane-uniform (every lane computes the same Philox output), the
// transition's table entries arrive in one round trip, and the observation,
// action and reward loads that depend only on its row go out together in the
// next one (the next observation too when n_steps == 1); longer n-step walks
// follow the chain lane-uniformly as the generic kernel does.
__global__ __launch_bounds__(256) void gather_vec_kernel(d3a_gather_desc d) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= d.B) return;
  int64_t t;
  if (d.idx) {
    t = d.idx[b];
  } else {
    const uint64_t c = d.ctr ? (uint64_t)(*d.ctr) : (uint64_t)d.ctr_value;
    uint32_t r[4];
    Philox::gen(d.seed, c, (uint64_t)(d.row_offset + b), r);
    const uint64_t x = ((uint64_t)r[0] << 32) | r[1];
    t = (int64_t)(x % (uint64_t)d.n_trans);
    if (lane == 0) d.idx_out[b] = t;
  }
  const int64_t row_t = d.t_row[t], last_t = d.t_ep_last[t];
  const uint8_t term_t = d.t_terminal[t];
  const int D = d.D, A = d.A;
  // row-only loads first (they do not wait for the n-step walk)
  const float rew_t = d.rew[row_t];
  float ov = 0.f, av = 0.f;
  if (lane < D) ov = d.obs[row_t * D + lane];
  if (d.act && lane < A) av = d.act[row_t * A + lane];
  int32_t ai = 0;
  if (d.act_i && lane == 0) ai = d.act_i[row_t];
  // n-step return (dataset.pyx:1323-1330), the generic kernel's arithmetic
  float ret = __fmul_rn(rew_t, d.gamma_pow[0]);
  ret = __fadd_rn(0.f, ret);
  int64_t nt_i = t, row_i = row_t, last_i = last_t;
  int k = 0;
  for (k = 0; k < d.n_steps; ++k) {
    if (k > 0) ret = __fadd_rn(ret, __fmul_rn(d.rew[row_i], d.gamma_pow[k]));
    if (nt_i == last_i || k == d.n_steps - 1) break;
    nt_i = nt_i + 1 == d.n_trans ? 0 : nt_i + 1;
    row_i = d.t_row[nt_i];
    last_i = d.t_ep_last[nt_i];
  }
  const bool term = (nt_i == t ? term_t : d.t_terminal[nt_i]) != 0;
  const int64_t nrow = term ? -1 : row_i + 1;
  float nv = 0.f;
  if (nrow >= 0 && lane < D) nv = d.obs[nrow * D + lane];
  if (lane < D) {
    d.o_obs[b * D + lane] = ov;
    d.o_next_obs[b * D + lane] = nv;
  }
  // observations wider than a wave (rare): the remaining columns
  for (int j = lane + 64; j < D; j += 64) {
    d.o_obs[b * D + j] = d.obs[row_t * D + j];
    d.o_next_obs[b * D + j] = nrow >= 0 ? d.obs[nrow * D + j] : 0.f;
  }
  if (d.act) {
    if (lane < A) d.o_act[b * A + lane] = av;
    for (int j = lane + 64; j < A; j += 64) d.o_act[b * A + j] = d.act[row_t * A + j];
  }
  if (lane == 0) {
    if (d.act_i) d.o_act_i[b] = ai;
    d.o_rew[b] = ret;
    d.o_term[b] = d.t_term_value ? d.t_term_value[nt_i] : (term ? 1.f : 0.f);
    d.o_n_steps[b] = (float)(k + 1);
  }
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_gather_batch(const d3a_gather_desc* d, void* stream) {
  D3A_CHECK_ARG(d, "d3a_gather_batch: null desc");
  D3A_CHECK_ARG(d->B >= 1, "d3a_gather_batch: batch size must be >= 1");
  D3A_CHECK_ARG(d->n_trans >= 1, "d3a_gather_batch: empty dataset");
  D3A_CHECK_ARG(d->rew && d->t_row && d->t_ep_start && d->t_ep_last && d->t_terminal,
                "d3a_gather_batch: missing transition table");
  D3A_CHECK_ARG((d->obs != nullptr) != (d->frames != nullptr),
                "d3a_gather_batch: exactly one of obs / frames");
  D3A_CHECK_ARG((d->act != nullptr) != (d->act_i != nullptr),
                "d3a_gather_batch: exactly one of act / act_i");
  D3A_CHECK_ARG(d->n_steps >= 1 && d->n_frames >= 1, "d3a_gather_batch: n_steps, n_frames >= 1");
  D3A_CHECK_ARG(d->n_steps <= D3A_MAX_NSTEP, "d3a_gather_batch: n_steps > D3A_MAX_NSTEP");
  D3A_CHECK_ARG(d->idx || (d->idx_out && ((d->ctr && d->ticket) || (!d->ctr && d->ctr_value >= 0))),
                "d3a_gather_batch: indices must be given or drawn (idx_out and ctr + ticket, "
                "or ctr_value)");
  D3A_CHECK_ARG(d->obs || d->ctr || d->idx, "d3a_gather_batch: ctr_value needs vector obs");
  D3A_CHECK_ARG(d->obs ? (d->o_obs && d->o_next_obs) : (d->o_frames && d->o_next_frames),
                "d3a_gather_batch: missing observation outputs");
  D3A_CHECK_ARG(d->o_rew && d->o_term && d->o_n_steps && (d->act ? d->o_act != nullptr
                                                                 : d->o_act_i != nullptr),
                "d3a_gather_batch: missing outputs");
  if (d->obs && !d->idx && !d->ctr) {
    // counter by value: the vector kernel (no ticket)
    hipLaunchKernelGGL(gather_vec_kernel, dim3((unsigned)((d->B + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, *d);
  } else if (d->obs && d->idx) {
    hipLaunchKernelGGL(gather_vec_kernel, dim3((unsigned)((d->B + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, *d);
  } else {
    // all frame pieces loaded before any is stored, unless D3A_GATHER_BATCHED=0
    static const bool batched = [] {
      const char* e = getenv("D3A_GATHER_BATCHED");
      return !(e && e[0] == '0');
    }();
    hipLaunchKernelGGL(gather_kernel, dim3((unsigned)d->B), dim3(256), 0, (hipStream_t)stream,
                       *d, batched);
  }
  D3A_LAUNCH_CHECK("d3a_gather_batch");
  return 0;
}
