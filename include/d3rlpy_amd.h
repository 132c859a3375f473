/*
 * d3rlpy_amd — C-ABI of the MI355X (gfx950) offline-RL update engine.
 *
 * Boundary: this library replaces the *arithmetic* that the reference d3rlpy
 * v1.1.0 performs through eager PyTorch inside the Impl update methods and the
 * Cython minibatch gather.  The Python host layer (d3rlpy_amd/) keeps the
 * reference's Algo/Impl plugin surface (fit / update / predict,
 * update_critic / update_actor / update_temp / update_alpha ...) and calls
 * these entry points through ctypes with raw device pointers.
 *
 * Conventions
 *   - every pointer is a device pointer unless stated otherwise;
 *   - `stream` is a hipStream_t passed as void* (torch's current stream);
 *   - nothing here allocates, frees or synchronises: every entry point only
 *     enqueues kernels, so all of them are legal inside stream capture;
 *   - return value 0 = enqueued, < 0 = argument or launch error; the message
 *     is available from d3a_last_error() (thread-local).
 *   - all math is fp32 (the reference's dtype); strides are in elements.
 *
 * The reference interface each entry point replaces is cited per function
 * (paths relative to the reference repository root).
 */
#ifndef D3RLPY_AMD_H_
#define D3RLPY_AMD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- library ------------------------------------------------------------ */
int d3a_abi_version(void);
const char* d3a_last_error(void);
/* number of visible HIP devices (0 when none). */
int d3a_device_count(int* count);

/* ---- dense layers (replaces nn.Linear forward/backward as used by
 *      d3rlpy/models/torch/encoders.py:265-275 _fc_encode, the heads in
 *      policies.py:57,170-176, q_functions/mean_q_function.py:255-256, and the
 *      autograd backward of those layers) ---------------------------------- */

/* Batched strided fp32 GEMM on MFMA (v_mfma_f32_32x32x2_f32):
 *   for b < batch, s < splits:
 *     P = alpha * sum_{k in split s} A_b(m,k) * B_b(k,n)
 *     v = P (+ bias_b[n]) ; relu ; (* [mask_b(m,n) > 0])
 *     C_b,s(m,n) = v   (or += v when accumulate)
 *   A_b(m,k) = A[b*sAb + m*sAm + k*sAk], B_b(k,n) = B[b*sBb + k*sBk + n*sBn],
 *   C_b,s(m,n) = C[b*sCb + s*sCs + m*sCm + n*sCn].
 * A forward nn.Linear is (A = x [rows,in], B = W^T i.e. sBk=1,sBn=in),
 * dX = dY W is (A = dY, B = W), dW = dY^T X is (A = dY^T, B = X). */
/* Next-layer weight-gradient epilogue of an input-gradient GEMM (see
 * d3a_gemm_desc.wnext). */
typedef struct d3a_gemm_wnext {
  const float* x; int64_t ldx, sxb;  /* layer input rows x[b*sxb + r*ldx + d] */
  int64_t n_in;                      /* d < n_in <= 64                       */
  float* dW;  /* [ceil(M/128)][batch][N][n_in] partials                      */
  float* db;  /* [ceil(M/128)][batch][N] partials                            */
} d3a_gemm_wnext;

typedef struct d3a_gemm_desc {
  const float* A;
  const float* B;
  float* C;
  const float* bias;  /* may be NULL */
  const float* mask;  /* may be NULL */
  float* rowsum;      /* may be NULL: rowsum[b*sRb + s*sRs + m] = sum_{k in s} A_b(m,k)
                         (the bias gradient when A = dY^T), fp64-accumulated */
  int64_t M, N, K, batch;
  int64_t sAb, sAm, sAk;
  int64_t sBb, sBk, sBn;
  int64_t sCb, sCm, sCn;
  int64_t sbias_b;
  int64_t sMb, sMm, sMn;
  int64_t splits, sCs;
  int64_t sRb, sRs;
  float alpha;
  int32_t relu;
  int32_t accumulate;
  int32_t variant;    /* tile configuration, -1 = automatic */
  /* Optional second batch dimension t < batch2 (0 or 1 = none): operands of
   * (b, t) at A + b*sAb + t*sAb2, B + b*sBb + t*sBb2, C + b*sCb + t*sCb2,
   * bias + b*sbias_b + t*sbias_b2, mask + b*sMb + t*sMb2 -- an independent
   * pass of the same shape in the same launch (the target networks beside
   * the online ones, DDPGBaseImpl._targ_q_func).  Not with rowsum. */
  int64_t batch2, sAb2, sBb2, sCb2, sbias_b2, sMb2;
  /* Optional (may be NULL): A is not read but generated as the masked input
   * gradient of a single-output head, exactly as d3a_head1_bwd writes dz
   * (its g / gscale / n_scaled / h / w fields; A = NULL, batch = members):
   *   A_b(r, j) = g'[b][r] * w[b][j] * [h[b][r][j] > 0]     (A k-contiguous)
   *   A_b(j, r) = the same                                  (A m-contiguous)
   * With A m-contiguous (the weight-gradient GEMM dW = dz^T h_prev) and
   * agen->dW / db set, the launch also writes the head's weight / bias
   * gradient partials agen->dW[s][b][j] = sum_{r in split s} g'[r] h[r][j],
   * agen->db[s][b] = sum g'[r] (fp64-accumulated, as d3a_head1_bwd does) —
   * the head backward needs no launch of its own. */
  const struct d3a_head1_bwd_desc* agen;
  /* Optional (may be NULL) on an input-gradient GEMM whose output C_b(r, j)
   * is the masked gradient dz of the layer below (A k-contiguous, no split,
   * bias, ReLU or rowsum): C is not written (may be NULL); instead, per
   * 128-row tile t, the weight / bias gradient partials of the layer whose
   * input is x:  wnext->dW[t][b][j][d] = sum_{r in t} C_b(r, j) x[r][d],
   * wnext->db[t][b][j] = sum_{r in t} C_b(r, j) (fp64-accumulated) — the
   * first layer's weight gradient without a launch of its own or a dz
   * round trip through HBM. */
  const d3a_gemm_wnext* wnext;
} d3a_gemm_desc;
int d3a_gemm_f32(const d3a_gemm_desc* desc, void* stream);

/* Two independent GEMMs (no data dependence between them; the weight- and
 * input-gradient GEMMs of one backward layer) enqueued as ONE launch when both
 * resolve to the register-direct kernel, one with one-wave tiles and one with
 * eight-wave K-split tiles (each tile then computes exactly what its own
 * d3a_gemm_f32 launch computes); otherwise as two d3a_gemm_f32 launches. */
int d3a_gemm_f32_pair(const d3a_gemm_desc* d1, const d3a_gemm_desc* d2, void* stream);

/* The same GEMM (A k-contiguous; B k-contiguous, y = x W^T (+ bias, ReLU),
 * or n-contiguous, dx = (dy W) * mask) evaluated on the bf16 matrix cores with
 * each fp32 operand split into bf16 parts: terms = 3 (hi/lo, ~2^-16 relative
 * per product) or 6 (hi/mid/lo, ~fp32).  The throughput instantiation of the
 * ensemble-Q layer GEMMs; no split-K / rowsum / batch2. */
int d3a_gemm_sbf16(const d3a_gemm_desc* desc, int32_t terms, void* stream);
/* y[m][n] = act(sum_s part[s][m][n] + bias[n]) over the S split-K partials
 * (split stride sS) of a d3a_gemm_sbf16 launch, added in split order (relu:
 * max(., 0)); the bias / activation of nn.Linear + ReLU (encoders.py:157-160). */
int d3a_splitk_epilogue_f32(const float* part, int32_t S, int64_t sS, float* y,
                            const float* bias, int64_t M, int64_t N, int32_t relu,
                            void* stream);

/* out[b*sOb + r] = sum_j X[b*sXb + r*sXr + j] * w[b*swb + j] + bias[b*sbb]
 * (the 256->1 head of ContinuousMeanQFunction, mean_q_function.py:255-256) */
int d3a_rowdot_f32(const float* X, int64_t sXb, int64_t sXr, const float* w,
                   int64_t swb, const float* bias, int64_t sbb, float* out,
                   int64_t sOb, int64_t batch, int64_t rows, int64_t n,
                   void* stream);
/* the same for a narrow head of J <= 16 outputs (w [J][n], bias [J], out
 * rows of stride J: out[b*sOb + r*J + j]; the nn.Linear heads of
 * policies.py:57-59 / 170-176) over a second batch dimension t < batch2,
 * offsets t * (dX, dw, dbias, dout) on top of the above (an independent pass
 * of the same shape, e.g. the target networks) */
int d3a_rowdot2_f32(const float* X, int64_t sXb, int64_t sXr, const float* w,
                    int64_t swb, const float* bias, int64_t sbb, float* out,
                    int64_t sOb, int64_t batch, int64_t rows, int64_t n, int32_t J,
                    int64_t batch2, int64_t dX, int64_t dw, int64_t dbias, int64_t dout,
                    void* stream);

/* out[b*sOb + s*sOs + j] = sum_{r in split s} (w ? w[b*swb + r] : 1) *
 *                          X[b*sXb + r*sXr + j]
 * (bias gradients and the weight gradient of a 1-output head) */
int d3a_colreduce_f32(const float* X, int64_t sXb, int64_t sXr,
                      const float* w, int64_t swb, float* out, int64_t sOb,
                      int64_t sOs, int64_t batch, int64_t rows, int64_t n,
                      int64_t splits, void* stream);

/* out[b][r][j] = g[b*sgb + r] * w[b*swb + j] * (h[b][r][j] > 0)
 * (backward of relu(h) -> 1-output head; h, out row-major [rows][n]) */
int d3a_outer_mask_f32(const float* g, int64_t sgb, const float* w,
                       int64_t swb, const float* h, int64_t shb, float* out,
                       int64_t sob, int64_t batch, int64_t rows, int64_t n,
                       void* stream);

/* Fused backward of the 1-output Q head q = relu(h).w + b
 * (ContinuousMeanQFunction._fc, mean_q_function.py:255-256), per member c:
 *   dz[c][r][j] = g[c][r] * w[c][j] * [h[c][r][j] > 0]
 *   dW[s][c][j] = sum_{r in split s} g[c][r] h[c][r][j],  db[s][c] = sum g
 * With q_min != NULL the row gradient is `scale` on the first argmin member of
 * q_min[.][r] and 0 elsewhere (backward of min over critics in
 * SACImpl.compute_actor_loss, sac_impl.py:114-121), optionally stored to g_out.
 * dW/db may be NULL (input gradient only). */
typedef struct d3a_head1_bwd_desc {
  const float* g;      int64_t sgb;            /* [C] x rows (or NULL)      */
  const float* gscale; int64_t n_scaled;       /* g[r] *= *gscale for r < n_scaled
                                                  (gscale may be NULL)      */
  const float* q_min;  int64_t sqb;            /* [C] x rows (or NULL)      */
  float scale;
  float* g_out;                                /* optional, stride sgb      */
  const float* h;      int64_t shb, ldh;       /* [C][rows][ldh]            */
  const float* w;      int64_t swb;            /* [C][n]                    */
  float* dz;           int64_t sdzb, lddz;     /* [C][rows][lddz]           */
  float* dW;           int64_t sWs;            /* [splits][C][n] or NULL    */
  float* db;           int64_t sbs;            /* [splits][C]                */
  int64_t rows, n, splits;
  int32_t C;
} d3a_head1_bwd_desc;
int d3a_head1_bwd(const d3a_head1_bwd_desc* desc, void* stream);

/* The single-output Q head of an ensemble evaluated and differentiated
 * through min over the members in one launch (the actor loss of
 * SACImpl.compute_actor_loss, sac_impl.py:114-121: q = min_c Q_c(s, a)).
 * One wave per row r:
 *   q[c*sqb + r] = h[c][r] . w[c] + b[c]        (the order of d3a_rowdot_f32)
 *   g_c = scale if c is the first argmin over c of q[.][r] else 0
 *   dz[c][r][j] = g_c * w[c][j] * [h[c][r][j] > 0],  g_out[c*sgb + r] = g_c
 * i.e. d3a_rowdot_f32 followed by d3a_head1_bwd in argmin mode; n <= 256,
 * n % 4 == 0, C <= 8. */
typedef struct d3a_head1_min_desc {
  const float* h; int64_t shb, ldh;   /* [C][rows][ldh]                     */
  const float* w; int64_t swb;        /* [C][n]                             */
  const float* b; int64_t sbb;        /* [C]                                */
  float* q; int64_t sqb;              /* [C] x rows (out)                   */
  float scale;
  float* g_out; int64_t sgb;          /* [C] x rows (out, may be NULL)      */
  float* dz; int64_t sdzb, lddz;      /* [C][rows][lddz] (out)              */
  int64_t rows, n;
  int32_t C;
} d3a_head1_min_desc;
int d3a_head1_min(const d3a_head1_min_desc* desc, void* stream);

/* ---- split-bf16 operand images of critic weights ------------------------ */

/* Exact three-way split of fp32 weights into bf16 parts, laid out as the
 * split-bf16 critic forward's MFMA A operand (d3a_mlp_fwd_desc.wp): for row
 * r < rows and 8-wide k block kb < kpad / 8, dst + (r * (kpad / 8) + kb) * 48
 * bytes holds parts 0, 1, 2 of src[r][8 kb .. 8 kb + 7] (8 bf16 each; x = p0
 * + p1 + p2 exactly: p0 = bf16(x), p1 = bf16(x - p0), p2 = bf16(x - p0 -
 * p1)), columns k .. kpad zero.  src is row-major [rows][k] (nn.Linear's
 * weight, members stacked); kpad a multiple of 16, >= k; dst 16-byte aligned.
 * No reference counterpart: the reference multiplies the fp32 weights
 * (encoders.py:265-275, 328-339); this is the same product's operand. */
typedef struct d3a_x6_split_job {
  const float* src;
  void* dst;
  int32_t rows, k, kpad, pad_;
} d3a_x6_split_job;
#define D3A_X6_SPLIT_MAX_JOBS 4
typedef struct d3a_x6_split_desc {
  d3a_x6_split_job job[D3A_X6_SPLIT_MAX_JOBS];
  int32_t n_jobs;
} d3a_x6_split_desc;
int d3a_x6_split(const d3a_x6_split_desc* d, void* stream);

/* Whole-MLP forward, one launch (replaces the per-layer nn.Linear + ReLU
 * chain of VectorEncoder / VectorEncoderWithAction, encoders.py:265-275,
 * 328-339, and the linear head: mean_q_function.py:255-256 `_fc`,
 * policies.py:57-59 / 170-176).  Per member c < C, rows r in [r0, r0+rows):
 *   a_0 = x[c*sxb + r*ldx + 0:n_in]
 *   a_l = relu(a_{l-1} W_{l-1}^T + b_{l-1}),  l = 1..n_hidden   (width H)
 *   out[c*sout + r*ldout + j] = a_{n_hidden} . W_head[j] + b_head[j]
 * W[l] row-major [out][in] (member stride sW[l]), W[n_hidden] is the head
 * (16-byte aligned; every layer after the first too).  h[l] (optional)
 * receives a_{l+1} as [C][R][H] (member stride sh, absolute row index) for
 * the backward pass, for rows r >= h_from only (rows no backward reads are
 * not stored).  Activations stay in LDS between layers; block_rows (0 =
 * automatic, 16, 32, 64 or 128) rows per workgroup.  Heads wider than 64
 * (quantile heads) run on MFMA as well.  block_rows 16: the small-pass
 * kernel (hundreds of rows; H == 256, n_out <= 64, 16-byte aligned W[1..],
 * biases and h rows).  Automatic on [n_in <= 48, 256, 256, 1] over >= 8,192
 * member-rows: the register-resident critic kernel (csrc/q2_fwd.hip). */
#define D3A_MLP_MAX_HIDDEN 4
/* A Philox fill -- d3a_philox_fill's stream, arithmetic and counter ticket --
 * run by extra workgroups of another launch (d3a_mlp_fwd_desc.philox, the
 * parts path); enabled when n_normal + n_uniform > 0. */
typedef struct d3a_philox_job {
  float* out; int64_t n_normal, n_uniform; float lo, hi; uint64_t seed;
  int64_t* ctr; unsigned int* ticket;
} d3a_philox_job;

typedef struct d3a_mlp_fwd_desc {
  const float* x; int64_t ldx, sxb;
  int32_t n_in, n_hidden, H, n_out;
  const float* W[D3A_MLP_MAX_HIDDEN + 1];
  const float* b[D3A_MLP_MAX_HIDDEN + 1];
  int64_t sW[D3A_MLP_MAX_HIDDEN + 1], sb[D3A_MLP_MAX_HIDDEN + 1];
  float* h[D3A_MLP_MAX_HIDDEN]; int64_t sh;
  float* out; int64_t sout, ldout;
  int64_t r0, rows, h_from;
  int32_t C, block_rows;
  /* Optional second, independent pass in the same launch (aux_rows > 0):
   * the same network shape with its parameters at W[l] + aux_wdelta and
   * b[l] + aux_wdelta (a second parameter buffer of the same layout, e.g.
   * the target networks of DDPGBaseImpl._targ_q_func), input rows
   * [0, aux_rows) of aux_x (row stride aux_ldx, member stride aux_sxb),
   * output aux_out (member stride aux_sout, row stride ldout), no
   * activations kept.  Its workgroups follow the main pass's in the grid and
   * run on the CUs the main pass leaves idle. */
  const float* aux_x; int64_t aux_ldx, aux_sxb, aux_wdelta;
  float* aux_out; int64_t aux_sout, aux_rows;
  /* Optional (parts = D3A_MLP_PARTS, block_rows 16, two hidden layers of 256,
   * n_in <= 64, n_out <= 16, no aux pass): the second hidden layer's units
   * are split into parts of 64, one workgroup per 16 rows, member and part,
   * so a few-hundred-row pass spreads over four times the CUs.  The head is
   * linear in the parts: out + p*s_part holds part p's sum over its units
   * (the head bias in part 0); a consumer sums the parts in order.  h[0] is
   * written by part 0, h[1] unit-slice by slice.  parts 0 / 1: off.       */
  int32_t parts;
  int64_t s_part;
  /* Optional (d3a_mlp_fwd_x6 only; null elsewhere): row_mean[c * s_mean + r]
   * = the mean of row r's n_out outputs (a fixed summation order), written
   * beside out -- e.g. the per-(critic, sampled action) quantile mean of
   * compute_max_with_n_actions (q_functions/__init__.py:37-39), so that
   * d3a_bcq_target does not re-read every quantile row.                  */
  float* row_mean; int64_t s_mean;
  /* Optional input-row builder (d3a_q2_fwd_x6 / d3a_mlp_fwd_x6 only, no aux
   * pass; xg_mode 0: off, read x): the kernel forms input row r itself as
   * d3a_bcq_rows would have written it -- (xg_obs[r / xg_rep][0..xg_D),
   * f(xg_a[r][0..xg_E))), f by xg_mode: 1 clamp(a, -clip, clip), 2 tanh(a),
   * 3 clamp(base + scale tanh(a), -1, 1), 4 as 3 with base = tanh(xg_base)
   * (the raw decoder output; xg_base rows of xg_E) -- so BCQ's target chain
   * (bcq_impl.py:215-226) needs no row-building launches.                */
  int32_t xg_mode, xg_D, xg_rep, xg_E;
  const float* xg_obs; const float* xg_a; int64_t xg_lda;
  const float* xg_base; float xg_clip, xg_scale;
  /* Optional (d3a_q2_fwd_x6 with one output only): the ReLU mask of the last
   * hidden layer of the kept rows (>= h_from) as bits, [C][rows][256 / 32]
   * uint32 (bit o & 31 of word o >> 5; member stride s_hmask words) -- what
   * d3a_q2_bwd_x6 builds its mask operand from (d3a_q2_bwd_desc.m2).       */
  void* hmask; int64_t s_hmask;
  /* Optional (with hmask, r0 % 32 == 0): the same mask transposed, [C][rows
   * / 32][256] uint32 -- word [r >> 5][o], bit r & 31 = [h_last[r][o] > 0] --
   * for every 32-row group holding a kept row (member stride s_hmaskT words):
   * the operand of d3a_q2_bwd_x6's slice kernel (d3a_q2_bwd_desc.m2t).     */
  void* hmaskT; int64_t s_hmaskT;
  /* Optional, with xg_mode: xg_a given as xg_a_parts > 1 partial sums (a
   * parts-path head, d3a_mlp_fwd_desc.parts), part q at xg_a + q *
   * xg_s_apart, summed in order (d3a_bcq_rows_desc.a_parts's arithmetic).
   * 0 / 1: one array.                                                      */
  int32_t xg_a_parts; int64_t xg_s_apart;
  /* Optional, with xg_mode on the parts path (parts > 1): the part-0
   * workgroups also write the rows they form to xg_xout (row stride xg_ldxo,
   * a multiple of 4, 16-byte aligned; columns past n_in zero) and f(a) to
   * xg_eout ([rows][xg_E]) -- d3a_bcq_rows's x and e_out, so a pass whose rows
   * a later stage reads (a backward's dW1) needs no d3a_bcq_rows launch.
   * xg_mode 5: f(a) = a (d3a_bcq_rows mode 0). */
  float* xg_xout; int64_t xg_ldxo; float* xg_eout;
  /* Optional (d3a_q2_fwd_x6 with one output and n_in <= 32; all four set or
   * all null): W[0] and W[1] of the main pass (wp) and of the aux pass
   * (aux_wp) as split-bf16 operand images -- d3a_x6_split's layout with kpad
   * = n_in rounded up to 16 (W[0]) and 256 (W[1]), every member's rows --
   * formed by an earlier launch from the same weights.  The kernel streams the
   * parts instead of splitting the fp32 weights in every workgroup; its
   * results are bitwise those of the in-kernel split.                       */
  const void* wp[2];
  const void* aux_wp[2];
  /* Optional (the parts path only): presplit.n_jobs > 0 appends workgroups
   * that run those d3a_x6_split jobs -- on the CUs the few-hundred-row pass
   * leaves idle (the CQL step's critic weight images, formed by the policy
   * forward that precedes the critic forward). */
  d3a_x6_split_desc presplit;
  /* Optional (the parts path only, round 6): a Philox fill on further
   * appended workgroups (BCQ's step noise in the VAE encoder's launch, which
   * precedes every reader of the noise). */
  d3a_philox_job philox;
} d3a_mlp_fwd_desc;
#define D3A_MLP_PARTS 4
int d3a_mlp_fwd(const d3a_mlp_fwd_desc* d, void* stream);

/* Backward-data of the same MLP, one launch (the autograd backward of the
 * encoder / head chain up to the weight gradients).  Rows r < rows of each
 * member c (all row pointers already at the first row):
 *   head, n_out == 1:  g_eff = g (* *gscale for r < n_scaled), or with
 *                      q_min: `scale` on the first argmin member of
 *                      q_min[.][r] (backward of min over the ensemble,
 *                      sac_impl.py:114-121), 0 on the others; stored to
 *                      g_eff when given;  dz_{L-1} = g_eff w_head * [h > 0]
 *   head, n_out > 1:   dz_{L-1} = dhead W_head * [h_{L-1} > 0]
 *   trunk:             dz_{l-1} = dz_l W_l * [h_{l-1} > 0]
 *   input (dx given):  dx = dz_0 W_0
 * dz[l] is [C][rows][H] (member stride sdz); h[l] the forward activations
 * (member stride sh, row stride ldh).  Weight gradients are not formed here:
 * they are split-K GEMMs over all rows (d3a_gemm_f32 with row sums). */
typedef struct d3a_mlp_bwd_desc {
  int32_t n_in, n_hidden, H, n_out, C;
  const float* W[D3A_MLP_MAX_HIDDEN + 1];
  int64_t sW[D3A_MLP_MAX_HIDDEN + 1];
  const float* h[D3A_MLP_MAX_HIDDEN]; int64_t sh, ldh;
  const float* g; int64_t sgb; const float* gscale; int64_t n_scaled;
  const float* q_min; int64_t sqb; float scale;
  float* g_eff; int64_t sgeb;
  const float* dhead; int64_t sdhb, lddh;
  float* dz[D3A_MLP_MAX_HIDDEN]; int64_t sdz;
  float* dx; int64_t sdxb, lddx;
  int64_t rows;
  int32_t block_rows;
} d3a_mlp_bwd_desc;
int d3a_mlp_bwd(const d3a_mlp_bwd_desc* d, void* stream);

/* The whole backward of a small-batch [n_in <= 64, 256, 256, n_out <= 256]
 * ReLU MLP in two launches on one stream (csrc/mlp_bwd_small.hip: stage A,
 * one workgroup per 32 rows x 32 units of the second hidden layer -- dW3 /
 * dW2 / db2 of its unit slice and its share of dz2 W2 into scratch; stage B,
 * one workgroup per 32-row block -- the eight shares summed in order, dz1,
 * dW1 / db1 / dx; replaces the per-layer
 * split-K / input-gradient GEMMs of the autograd of encoders.py:265-275,
 * 328-339 and the heads -- K3's VAE, QR critics and residual policy,
 * bcq_impl.py:132-161, ddpg_impl.py:138-165).  dout = dL/d(out) [C][rows]
 * [ld_dout] (member stride sdout), h1 / h2 the forward's kept activations
 * ([C][.][256], member stride sh, row 0 = the first row here), x [C][rows]
 * [ldx] (sxb 0: shared).  Weight / bias gradients (all or none) as one
 * partial per 32-row block, [ceil(rows / 32)][C][out][in]; dx (optional)
 * [C][rows][n_in].  scratch: [8][C][rows][256] floats (stage A -> stage B);
 * tickets: reserved, not read (may be NULL; the one-launch ticketed form was
 * measured slower and removed).  Exact fp32 arithmetic. */
typedef struct d3a_mlp_bwd_small_desc {
  const float* x; int64_t ldx, sxb;
  const float* h1; const float* h2; int64_t sh;
  const float* dout; int64_t ld_dout, sdout;
  const float* W1; const float* W2; const float* W3;
  int64_t sW1, sW2, sW3;
  float* dW1; float* db1; float* dW2; float* db2; float* dW3; float* db3;
  float* dx;
  float* scratch; int32_t* tickets;
  int32_t rows, n_in, n_out, C;
} d3a_mlp_bwd_small_desc;
int d3a_mlp_bwd_small(const d3a_mlp_bwd_small_desc* d, void* stream);
/* Diagnostic (synchronous, not for graphs): the phase stamps ([launch 0/1:
 * stage A/B][workgroup][4] s_memtime values) of the last d3a_mlp_bwd_small
 * launch made with D3A_SB_STAMPS=1 in the environment. */
int d3a_small_bwd_stamps(unsigned long long* dst, int n);

/* Weight gradients of a single-output Q ensemble with two hidden layers of
 * width 256 (VectorEncoderWithAction [n_in -> 256 -> 256], encoders.py:265-275,
 * 328-339, + ContinuousMeanQFunction._fc, mean_q_function.py:255-256), one
 * launch — the backward of update_critic's loss (ddpg_impl.py:119-133,
 * cql_impl.py:110-125).  Per member c, rows r < rows (pointers at row 0):
 *   g' = g[c*sgb + r] (* *gscale for r < n_scaled; gscale may be NULL)
 *   dz2 = g' w3 * [h2 > 0],  dz1 = (dz2 W2) * [h1 > 0]
 *   dW3 = g'^T h2, db3 = sum g', dW2 = dz2^T h1, db2 = sum dz2,
 *   dW1 = dz1^T x, db1 = sum dz1
 * as one partial per 256-row block p < P = ceil(rows / 256) (block_rows), laid out like
 * the split-K partials d3a_adam_f32 sums: dW1 [P][C][256][n_in], db1
 * [P][C][256], dW2 [P][C][256][256], db2 [P][C][256], dW3 [P][C][256], db3
 * [P][C].  h1 / h2 [C][rows][ldh] (member stride sh), x [rows][ldx] (member
 * stride sxb, 0 = shared), W2 [C][256][256] (stride sW2), w3 [C][256] (stride
 * sw3); h1, h2, W2 16-byte aligned, ldx >= n_in (16-byte x pieces when x is
 * aligned and ldx % 4 == 0, else element loads), n_in <= 48. */
typedef struct d3a_q2_bwd_desc {
  const float* x; int64_t ldx, sxb;
  const float* h1; const float* h2; int64_t sh, ldh;
  const float* g; int64_t sgb;
  const float* gscale; int64_t n_scaled;
  const float* W2; int64_t sW2;
  const float* w3; int64_t sw3;
  float* dW1; float* db1; float* dW2; float* db2; float* dW3; float* db3;
  int64_t rows;
  int32_t n_in, C;
  /* dz2 != NULL (fp32 only): the trunk backward of a two-hidden-layer net
   * whose head a caller already differentiated -- dz2 [C][rows][256] (member
   * stride sdz) is the masked pre-activation gradient of the second hidden
   * layer (e.g. d3a_sac_actor_head's dz for the policy, sac_impl.py:164-176);
   * g, w3, h2 are unused and dW3 / db3 not written.  block_rows: rows per
   * partial, 0 or 256 (default), or 32 (required with dz2: the few-hundred-row
   * actor pass spread over ceil(rows / 32) * 4 workgroups). */
  const float* dz2; int64_t sdz;
  int32_t block_rows;
  /* Optional (d3a_q2_bwd_x6 only): the forward's mask bits of h2
   * (d3a_mlp_fwd_desc.hmask; rows at the same base as h1 / h2, member stride
   * sm2 words) -- the ReLU-mask operand is expanded from them, not built
   * from h2.                                                              */
  const void* m2; int64_t sm2;
  /* Optional (d3a_q2_bwd_x6 only, with m2): the forward's transposed mask bits
   * (d3a_mlp_fwd_desc.hmaskT; word [r / 32][o] of the rows at the base of
   * h1, member stride sm2t words) and the layer-2 bias b2 [C][256] (stride
   * sb2).  Selects the slice kernel (csrc/q2_x6_bwd2.hip): h2 is not read
   * (dW3 = W2 . (m^T g' h1) + b2 (m^T g'), the forward's h2 identity), and
   * the partials are P = row_splits (0: d3a_q2_bwd_x6t_splits(rows, C)) row
   * blocks of ceil(rows / P) rows rounded up to 32: dW1 / db1 / dW2 / db2 /
   * db3 [P][C][..] as above, dW3 [16 P][C][256] (one per row block and
   * 16-unit slice of layer 1).                                              */
  const void* m2t; int64_t sm2t;
  const float* b2; int64_t sb2;
  int32_t row_splits;
} d3a_q2_bwd_desc;
/* Row blocks P of d3a_q2_bwd_x6's slice kernel for `rows` rows of C members
 * (about 256 workgroups of C * P * 16; the caller sizes the partials with it). */
int32_t d3a_q2_bwd_x6t_splits(int64_t rows, int32_t C);
int d3a_q2_bwd(const d3a_q2_bwd_desc* d, void* stream);


/* bf16 throughput instantiation of the critic forward / backward (the
 * `--precision bf16` bench line, never the parity path): the same contracts
 * as d3a_mlp_fwd on [n_in <= 48, 256, 256, 1] and d3a_q2_bwd, with every GEMM
 * operand rounded to bf16 and fp32 accumulation (v_mfma_f32_32x32x16_bf16);
 * the kept activations h[0] / h[1] (forward) and h1 / h2 (backward) are bf16
 * rows ([C][rows][256] __bf16, 16-byte aligned), everything else fp32. */
int d3a_q2_fwd_bf16(const d3a_mlp_fwd_desc* d, void* stream);
int d3a_q2_bwd_bf16(const d3a_q2_bwd_desc* d, void* stream);

/* fp32-accurate critic forward / backward on the bf16 matrix cores (csrc/
 * q2_x6.hip): the contracts of d3a_mlp_fwd on [n_in <= 48, 256, 256, 1]
 * (fp32 kept activations) and d3a_q2_bwd (block_rows 0 / 256), every GEMM
 * product x*y formed from an exact three-way bf16 split of both operands as
 * the six part products above fp32 resolution, accumulated in fp32
 * (v_mfma_f32_32x32x16_bf16): within fp32 rounding of the exact product, not
 * a reduced-precision path.  Replaces, like d3a_mlp_fwd / d3a_q2_bwd, the
 * critic passes of cql_impl.py:110-223 / ddpg_impl.py:119-133 through
 * encoders.py:265-275, 328-339 and mean_q_function.py:255-256. */
int d3a_q2_fwd_x6(const d3a_mlp_fwd_desc* d, void* stream);
int d3a_q2_bwd_x6(const d3a_q2_bwd_desc* d, void* stream);
/* The bf16 throughput line's critic forward: d3a_q2_fwd_x6's contract (fp32
 * kept activations) with one bf16 rounding per operand (fp32 accumulation);
 * its backward is d3a_q2_bwd_x6 (ReLU-mask operands exact, the other operand
 * split in three parts). */
int d3a_q2_fwd_x1(const d3a_mlp_fwd_desc* d, void* stream);
/* The same split-bf16 forward for a wide head, [n_in <= 64, 256, 256,
 * n_out <= 256] (csrc/mlp_x6.hip): d3a_mlp_fwd's contract without the aux pass
 * and parts; e.g. BCQ's target QR critics over B*N sampled actions
 * (bcq_impl.py:215-226, qr_q_function.py:97-161). */
int d3a_mlp_fwd_x6(const d3a_mlp_fwd_desc* d, void* stream);
/* The input-gradient chain of two 256 x 256 ReLU layers on split-bf16
 * streams (round 6; the CQL reproduction critic's backward between its head
 * and its first layer): per member c, rows [0, rows),
 *   dz_mid = (dz_top Wa) * [h_mid > 0],  dz_bot = (dz_mid Wb) * [h_bot > 0]
 * (Wa, Wb nn.Linear [out][in] weights, member stride sW; dz rows of stride ld,
 * member stride sdz; h rows of stride ldh, member stride sh).  dz_bot may
 * alias dz_top (each workgroup reads its rows of dz_top before it writes
 * them), dz_mid may not.  Replaces the two input-gradient GEMMs of the
 * trunk's autograd backward (encoders.py:265-275). */
typedef struct d3a_mlp_bwd_chain_desc {
  const float* dz_top; float* dz_mid; float* dz_bot;
  const float* h_mid; const float* h_bot;
  const float* Wa; const float* Wb;
  int64_t sW, ld, sdz, ldh, sh, rows;
  int32_t C;
} d3a_mlp_bwd_chain_desc;
int d3a_mlp_bwd_chain(const d3a_mlp_bwd_chain_desc* d, void* stream);
/* Diagnostic (synchronous, not for graphs): the phase stamps ([workgroup][9]
 * s_memtime values) of the last d3a_mlp_fwd_x6 launch made with
 * D3A_WIDE_STAMPS=1 in the environment. */
int d3a_wide_stamps(unsigned long long* dst, int n);
/* diagnostic: every wave's phase stamps of the last three-hidden-layer
 * D3A_WIDE_STAMPS=1 d3a_mlp_fwd_x6 launch, [workgroup < 512][wave][8]
 * (s_memtime at tile start, the input barrier, image 1, layer 2 issued,
 * image 2, layer 3 issued, head written) */
int d3a_wide_wave_stamps(unsigned long long* dst, int n);
/* Diagnostic (synchronous, not for graphs): the phase-boundary s_memtime
 * stamps of the last d3a_q2_fwd_x6 launch built with D3A_X6_PROBE bit 4. */
int d3a_x6_stamps(unsigned long long* dst, int n);

/* ---- optimiser and target networks ------------------------------------- */

/* One parameter tensor inside a flat buffer, with its gradient given as
 * `n_partials` partial sums laid out `partial_stride` apart (summed in order
 * 0..n_partials-1 before the update; n_partials=1 for a plain gradient).   */
typedef struct d3a_adam_segment {
  float* param;
  float* exp_avg;
  float* exp_avg_sq;
  const float* grad;
  int64_t numel;
  int64_t n_partials;
  int64_t partial_stride;
  float* grad_out; /* optional: reduced gradient is stored here (may be NULL) */
} d3a_adam_segment;

/* torch.optim.Adam single-tensor step (torch/optim/adam.py, weight_decay=0,
 * amsgrad=False) as created by AdamFactory (d3rlpy/models/optimizers.py:106-138):
 *   m = lerp(m, g, 1-b1); v = v*b2 + (1-b2)*g*g; t = *step + 1
 *   p += -(lr/(1-b1^t)) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
 * `segs` is a DEVICE array of n_seg segments; the launch is flat over them:
 * n_blocks = sum_s ceil(numel_s * L_s / 256), L_s = 16 if n_partials_s >= 64
 * else 1 (segment s owns the next ceil(numel_s * L_s / 256) blocks, in table
 * order; L_s lanes share one element's partial sum).  *step (device int64, the
 * optimiser's completed steps) is only read; commit it with d3a_step_end.
 * The reduced gradient is multiplied by grad_scale (1, or 1/world after a
 * data-parallel SUM all-reduce). */
int d3a_adam_f32(const d3a_adam_segment* segs, int32_t n_seg,
                 int64_t n_blocks, const int64_t* step,
                 double lr, double beta1, double beta2, double eps,
                 double grad_scale, void* stream);

/* d3a_adam_f32 with the update's end-of-step bookkeeping folded in (one
 * launch instead of Adam + d3a_step_end):
 *   t = *step + step_add (1: *step counts completed steps; 0: an earlier
 *       launch of the same update already advanced it);
 *   soft != 0: after each element's step the target copy at
 *       param + targ_delta (elements; a second buffer of the same layout) is
 *       soft-synced from the new value, targ = targ*(1-tau) + tau*p, the three
 *       rounded ops of d3a_soft_update_f32 (soft_sync, torch_utility.py:27-33:
 *       DDPGBaseImpl.update_critic_target / update_actor_target run after the
 *       parameter's last change of the step, so the fusion is exact);
 *   block 0: counters[i] += 1 for each bit i of inc_mask, and with ring !=
 *       NULL metrics[0:n_metrics] (* metric_scale) appended to
 *       ring[*ring_ctr % ring_cap], *ring_ctr += 1 — as d3a_step_end; the
 *       counters incremented must not include the one `step` points at. */
/* One workgroup's share of a flat Adam launch: its segment and the
 * segment's first block (a table of n_blocks of these, built once per
 * optimiser, saves the in-kernel segment search: one memory round trip). */
typedef struct d3a_adam_block {
  d3a_adam_segment seg;
  int64_t first;
} d3a_adam_block;

typedef struct d3a_adam_desc {
  const d3a_adam_segment* segs; int32_t n_seg; int64_t n_blocks;
  const int64_t* step; int32_t step_add;
  double lr, beta1, beta2, eps, grad_scale;
  int32_t soft; int64_t targ_delta; double tau;
  int64_t* counters; uint32_t inc_mask;
  const float* metrics; int32_t n_metrics;
  float* ring; int64_t ring_cap; int64_t* ring_ctr; float metric_scale;
  /* optional (may be NULL): DEVICE table of n_blocks d3a_adam_block, block b
   * = the segment owning flat block b in the layout above and its first
   * block; segs is then not read */
  const d3a_adam_block* blocks;
  /* optional, block 0 (n_commit <= 8): *commit_dst[i] = commit_src[i], and
   * *commit_step[k] += 1 where commit_step[k] != NULL -- a scalar optimiser
   * state an earlier launch of the update computed but could not write in
   * place (d3a_cql_loss_desc.stage) */
  const float* commit_src; float* commit_dst[8]; int32_t n_commit;
  int64_t* commit_step[2];
  /* 1: no segment takes four elements a thread (>= 2^18 elements, a multiple
   * of 4, < 64 partials) -- the launch runs the one-element kernel (fewer
   * registers); 0: either */
  int32_t one_elem;
} d3a_adam_desc;
int d3a_adam_step(const d3a_adam_desc* d, void* stream);

/* grad_out = sum of the n_partials split-K partials of each segment (fp64
 * accumulation, same order and flat grid as d3a_adam_f32) — the data-parallel path's
 * reduction before the gradient all-reduce. */
int d3a_grad_reduce_f32(const d3a_adam_segment* segs, int32_t n_seg,
                        int64_t n_blocks, void* stream);

/* StandardScaler.transform (preprocessing/scalers.py:350-354) as applied to a
 * minibatch by TorchMiniBatch (torch_utility.py:179-181): y[r][j] =
 * (x[r][j] - mean[j]) / (std[j] + eps), separately rounded fp32 ops; x and y
 * rows of stride ldx (may alias). */
int d3a_standardize_f32(const float* x, float* y, int64_t rows, int32_t D, int64_t ldx,
                        const float* mean, const float* std, float eps, void* stream);

/* soft_sync (d3rlpy/torch_utility.py:27-33): targ = targ*(1-tau) + tau*src,
 * three separately rounded fp32 ops (mul_, tau*p, add_), bit-exact. */
int d3a_soft_update_f32(float* targ, const float* src, int64_t n, double tau,
                        void* stream);

/* End of one update, one launch: (1) when targ != NULL the soft target
 * update targ = targ*(1-tau) + tau*src over n_soft elements (soft_sync,
 * d3rlpy/torch_utility.py:27-33, bit-exact as d3a_soft_update_f32);
 * (2) when ring != NULL append metrics[0:n] to ring[(*ring_ctr % cap)] and
 * increment *ring_ctr (per-step loss history kept on device and read once per
 * epoch instead of one device->host sync per update, cf. base.py:645-657);
 * (3) increment counters[i] for every bit i of inc_mask (optimiser steps).
 * Ring entries are metrics * metric_scale (1, or 1/world for metrics summed
 * over data-parallel ranks). */
int d3a_step_end(const float* metrics, int32_t n, float* ring, int64_t cap,
                 int64_t* ring_ctr, int64_t* counters, uint32_t inc_mask,
                 float* targ, const float* src, int64_t n_soft, double tau,
                 float metric_scale, void* stream);

/* ---- stand-alone loss / sampling blocks (csrc/ops_generic.hip): the op set
 *      behind the PyTorch custom ops of csrc/torch_ops.cpp; the update
 *      pipelines run fused versions of the same arithmetic ------------------ */

/* out[r] = logsumexp(x[r*ldx + 0:n]) (torch.logsumexp over the last dim; the
 * CQL conservative term, d3rlpy/algos/torch/cql_impl.py:208-213), and its
 * backward dx[r*lddx + j] = gout[r] * exp(x[r][j] - out[r]). */
int d3a_logsumexp_f32(const float* x, int64_t rows, int64_t n, int64_t ldx, float* out,
                      void* stream);
int d3a_logsumexp_bwd_f32(const float* x, int64_t rows, int64_t n, int64_t ldx,
                          const float* lse, const float* gout, float* dx, int64_t lddx,
                          void* stream);

/* TD error of ContinuousMeanQFunction.compute_error (q_functions/
 * mean_q_function.py:74-87) per member c < C over n rows:
 *   y = rew + gamma[r] * target[c][r] * (1 - term[r]),  diff[c][r] = q[c][r] - y
 *   loss[c] = mean_r diff^2   (gamma[r] = gamma ** n_steps[r], ddpg_impl.py:123)
 * and its backward dq[c][r] = 2 * diff[c][r] * gout[c] / n. */
int d3a_td_mse_f32(const float* q, const float* rew, const float* target, const float* term,
                   const float* gamma, int64_t C, int64_t n, float* diff, float* loss,
                   void* stream);
int d3a_td_mse_bwd_f32(const float* diff, const float* gout, int64_t C, int64_t n, float* dq,
                       void* stream);

/* compute_quantile_huber_loss (q_functions/utility.py:27-46) of quantiles
 * q[b][0:N] against targets y[b][0:M] at fractions taus[b][0:N]:
 *   loss[b] = (1/M) sum_j sum_i |taus_i - [y_j - q_i < 0]| * huber(y_j - q_i)
 * (huber with beta 1; the QR / IQN losses of utility.py:49-64,
 * iqn_q_function.py), and its backward dq[b][i] = gout[b] * d loss[b]/d q_i
 * (the indicator is detached, as in the reference). */
int d3a_quantile_huber_f32(const float* q, int64_t ldq, const float* y, int64_t ldy,
                           const float* taus, int64_t ldt, int64_t B, int64_t N, int64_t M,
                           float* loss, void* stream);
int d3a_quantile_huber_bwd_f32(const float* q, int64_t ldq, const float* y, int64_t ldy,
                               const float* taus, int64_t ldt, int64_t B, int64_t N, int64_t M,
                               const float* gout, float* dq, int64_t lddq, void* stream);

/* SquashedNormalPolicy.sample_with_log_prob (policies.py:196-216 +
 * distributions.py:112-135) for rows b < B of A actions given the noise:
 *   s = exp(clamp(logstd, min, max)), raw = mu + eps * s, action = tanh(raw),
 *   logp[b] = sum_a Normal(mu, s).log_prob(raw) - 2 (log 2 - raw - softplus(-2 raw))
 * and its backward (grad_action and / or grad_logp may be NULL = 0) to dmu and
 * dlogstd (zero where the clamp is active). */
int d3a_squashed_gauss_f32(const float* mu, const float* logstd, const float* eps, int64_t B,
                           int32_t A, float min_logstd, float max_logstd, float* action,
                           float* logp, void* stream);
int d3a_squashed_gauss_bwd_f32(const float* mu, const float* logstd, const float* eps,
                               int64_t B, int32_t A, float min_logstd, float max_logstd,
                               const float* grad_action, const float* grad_logp, float* dmu,
                               float* dlogstd, void* stream);

/* ReLU backward: dz[i] = y[i] > 0 ? dy[i] : 0 (y the ReLU output). */
int d3a_relu_mask_f32(const float* dy, const float* y, int64_t n, float* dz, void* stream);

/* ---- random numbers ----------------------------------------------------- */

/* Philox4x32-10: out[0:n_normal] ~ N(0,1) (Box-Muller), then
 * out[n_normal:n_normal+n_uniform] ~ U(lo, hi).  The device counter *ctr is
 * read by every block and incremented once per call, so a captured graph
 * draws fresh numbers on every replay (replaces torch.randn / rsample /
 * uniform_ in policies.py:202-216, cql_impl.py:186, td3_impl.py:67). */
int d3a_philox_fill(float* out, int64_t n_normal, int64_t n_uniform, float lo,
                    float hi, uint64_t seed, int64_t* ctr,
                    unsigned int* ticket, void* stream);



/* ---- CQL / SAC fused stages (d3rlpy/algos/torch/cql_impl.py,
 *      sac_impl.py) ------------------------------------------------------- */

/* Sampling stage of one CQL update.  Inputs: policy head outputs for the
 * stacked batch [obs; next_obs] (`head`, [2B][2A] = mu | raw logstd), the
 * observations, and the step's noise.  Produces every Q-function input row
 * and every log-probability of the step; see d3rlpy_amd/algos/cql.py for the
 * row layout.  Mirrors SquashedNormalPolicy.sample_with_log_prob /
 * sample_n_with_log_prob (policies.py:160-216, distributions.py:112-135). */
typedef struct d3a_cql_sample_desc {
  const float* head;      /* [2B][2A] */
  const float* obs;       /* [B][D]   */
  const float* next_obs;  /* [B][D]   */
  const float* act;       /* [B][A]   */
  const float* eps_temp;  /* [B][A]            update_temp sample        */
  const float* eps_pi;    /* [2 sets][2][N][B][A] conservative samples   */
  const float* u_rand;    /* [2 sets][B*N][A]  uniform(-1,1) actions     */
  const float* eps_actor; /* [B][A]            update_actor sample       */
  float* x_q;             /* [2 sets * 3*N*B + B][D+A] Q inputs           */
  float* x_targ;          /* [B][D+A] target-Q inputs (next_obs, tanh mu') */
  float* x_actor;         /* [B][D+A] actor Q inputs                      */
  float* logp_temp;       /* [B]                                         */
  float* logp_is;         /* [2 sets][2][B*N] log-probs of the IS samples */
  float* actor_u;         /* [B][A]  pre-tanh actor sample                */
  float* actor_logp;      /* [B]                                         */
  int32_t B, D, A, N;
  int32_t ldx;            /* row stride of x_q / x_targ / x_actor (>= D + A;
                             padded to a multiple of 4 for 16-byte rows)   */
  float min_logstd, max_logstd;
  /* soft_target != 0: the target action is a policy sample at next_obs
   * (SACImpl.compute_target, sac_impl.py:148-162; CQL soft_q_backup,
   * cql_impl.py:225-230) from eps_targ [B][A], its log-prob -> logp_targ [B];
   * otherwise tanh(mu(next_obs)) (cql_impl.py:232-243).  N = 0 (SAC: no
   * conservative samples) leaves x_q = the B data rows. */
  const float* eps_targ;
  float* logp_targ;
  int32_t soft_target;
  /* gen_noise != 0: the draws are not read from eps_* / u_rand but computed
   * here as the elements (pointer - noise_base) of the d3a_philox_fill stream
   * (seed, *rng_ctr; the first n_normal normal, the rest uniform in [-1, 1)),
   * bit-identical to filling the buffer first; the actor draws are written
   * to eps_actor_out for d3a_sac_actor_head.  The caller advances *rng_ctr. */
  const float* noise_base;
  const int64_t* rng_ctr;
  float* eps_actor_out;
  uint64_t seed;
  int64_t n_normal;
  int32_t gen_noise;
  /* head_parts >= 2: the policy head rows are head_parts partial sums at
   * head + p*s_head_part (d3a_mlp_fwd parts), summed in order here */
  int32_t head_parts;
  int64_t s_head_part;
  /* presplit.n_jobs > 0: this launch also runs those d3a_x6_split jobs (the
   * critic weights the step's critic forward streams as parts, formed by the
   * launch before it -- no launch of their own). */
  d3a_x6_split_desc presplit;
} d3a_cql_sample_desc;
int d3a_cql_sample(const d3a_cql_sample_desc* d, void* stream);

/* Loss stage of one CQL update (two launches: a wave-per-row logsumexp
 * kernel, then one workgroup for the scalars): update_temp
 * (sac_impl.py:123-146) incl. its Adam step on log_temp, update_alpha
 * (cql_impl.py:119-141) incl. its Adam step on log_alpha, the TD target
 * (cql_impl.py:232-243, mean_q_function.py:268-270) and dL/dQ of every
 * critic row of update_critic (cql_impl.py:110-117,196-223). */
typedef struct d3a_cql_loss_desc {
  const float* q;          /* [C][R] Q of every x_q row                    */
  const float* q_targ;     /* [C][B] target Q at (next_obs, tanh mu')      */
  const float* logp_temp;  /* [B]                                         */
  const float* logp_is;    /* [2][2][B*N]                                 */
  const float* rew;        /* [B] */
  const float* term;       /* [B] */
  const float* n_steps;    /* [B] */
  float* log_temp;         /* [1] parameter, updated in place              */
  float* temp_m; float* temp_v; int64_t* temp_step;
  float* log_alpha;        /* [1] parameter, updated in place              */
  float* alpha_m; float* alpha_v; int64_t* alpha_step;
  float* dq;               /* [C][R] dL_critic/dQ (alpha rows set to 0)    */
  float* lse;              /* [2][C][B] workspace: logsumexp per set       */
  float* metrics;          /* [8]: temp_loss temp alpha_loss alpha critic_loss
                              td_loss conservative_loss (reserved)          */
  float* scalars;          /* [4]: exp(log_temp_new) exp(log_alpha_new) .. */
  int32_t B, A, N, C;
  int64_t R;               /* rows per critic in q / dq                    */
  float gamma;
  double temp_lr, alpha_lr, beta1, beta2, adam_eps;
  float alpha_threshold, conservative_weight;
  int32_t update_temp, update_alpha, update_critic;
  /* data parallel (K4): 0 = single device; 1 = write the temp /
   * alpha gradients to scalar_grads[0:2] and stop; 2 = Adam on the
   * all-reduced scalar_grads * grad_scale, then the critic stage */
  int32_t dp_phase;
  float* scalar_grads;
  float grad_scale;
  /* soft_target: y uses min_c Q_targ - exp(log_temp_new) * logp_targ[b]
   * (sac_impl.py:148-162); conservative = 0: plain TD loss (SACImpl, no
   * logsumexp stage, no alpha) */
  const float* logp_targ;
  int32_t soft_target, conservative;
  /* ticket (optional, a zero-initialised device counter): the logsumexp stage
   * and the loss stage in one launch -- the last workgroup of the first runs
   * the second (same sums, same order) and resets the counter */
  uint32_t* ticket;
  /* split != 0 (the loss stage inside the critic backward, d3a_q2_bwd_x6_cql;
   * single device, conservative, no soft target, update_critic): this entry
   * launches only the logsumexp stage, which also writes every data row's
   * alpha-free gradient dq[c][6NB + b] = 2 (q - y) / B (the backward
   * subtracts the conservative term), td2[c][b] = (q - y)^2 and bc[0:4] =
   * the coming temperature step's (float) lr / (1 - beta1^t) and (float)
   * sqrt(1 - beta2^t), then alpha's (fp64 pows, the loss stage's constants).
   * stage [6]: the new log_temp, temp_m, temp_v, log_alpha, alpha_m, alpha_v
   * the backward computes; the critic Adam's tail commits them
   * (d3a_adam_desc.commit_*). */
  int32_t split;
  float* td2;
  double* bc;
  float* stage;
} d3a_cql_loss_desc;
int d3a_cql_loss(const d3a_cql_loss_desc* d, void* stream);
/* d3a_q2_bwd_x6's slice kernel with the CQL loss stage in every workgroup's
 * prologue (no launch of its own): from the logsumexp stage's outputs (loss
 * with split set; d.g = dq at the critic set's first row, n_scaled = 3NB) each
 * workgroup forms the alpha Adam step of update_alpha (cql_impl.py:119-141)
 * itself -- the same sums in the same order in every workgroup -- and so the
 * conservative scale ca cw / (C B): the 3NB importance-sampled rows' softmax
 * weights are multiplied by it, the data rows' alpha-free gradients have it
 * subtracted (ddpg_impl.py:138-165 with cql_impl.py:110-117).  Workgroup 0
 * also takes update_temp's step (sac_impl.py:123-146), writes metrics[0:8]
 * (but 5) and scalars[0:3] as d3a_cql_loss does, and the new scalar optimiser
 * state to loss.stage (committed by a later launch: every workgroup reads the
 * old state).  gscale is not read. */
int d3a_q2_bwd_x6_cql(const d3a_q2_bwd_desc* d, const d3a_cql_loss_desc* loss, void* stream);
/* Diagnostic (synchronous, not for graphs): the phase stamps ([workgroup
 * < 256][wave 0 / 4][8] s_memtime values) of the last slice-backward launch
 * made with D3A_BWD_STAMPS=1 in the environment. */
int d3a_bwd_stamps(unsigned long long* dst, int n);

/* Actor stage helpers (SACImpl.compute_actor_loss, sac_impl.py:114-121):
 * from the critics' Q at (s, tanh u) and the policy head, the per-row
 * gradient seed for the critics (dq = -1/B on the argmin critic) ...        */
int d3a_sac_actor_dq(const float* q, int64_t sqc, int32_t C, int32_t B,
                     float* dq, int64_t sdq, void* stream);
/* ... and, given dQ/da summed over critics, the policy-head gradient
 * [B][2A] (dmu | dlogstd_raw) of mean(exp(log_temp)*logp - min_c Q).   */
typedef struct d3a_sac_actor_head_desc {
  const float* head;      /* [>=B][2A] policy head rows for obs           */
  const float* eps;       /* [B][A] */
  const float* u;         /* [B][A] pre-tanh sample                       */
  const float* logp;      /* [B] */
  const float* dq_da;     /* [C][B][ld_da] dQ_c/d(input); action columns at
                             offset da_off                                */
  int64_t ld_da, da_off, sda_c;
  const float* q;         /* [C] x [B], stride sqc */
  int64_t sqc;
  const float* scalars;   /* scalars[0] = exp(log_temp) (after update_temp) */
  float* dhead;           /* [B][2A] */
  float* metrics;         /* metrics[5] = actor_loss                       */
  int32_t B, A, C;
  float min_logstd, max_logstd;
  /* optional (dz != NULL): the head's input gradient for the trunk backward,
   * dz[b*lddz + n] = (sum_k dhead[b][k] w_head[k*H + n]) * [h[b*ldh + n] > 0] */
  const float* w_head;    /* [2A][H] head weight (_mu rows, then _logstd)   */
  const float* h;         /* [B][ldh] last hidden activation of the policy  */
  int64_t ldh;
  float* dz;
  int64_t lddz;
  int32_t H;              /* <= 256 */
  /* optional (with dz): one partial per row of the head's weight / bias
   * gradients, dW_part[b][k][n] = dhead[b][k] h[b][n], db_part[b][k] =
   * dhead[b][k] (summed over b, in row order, by d3a_adam_f32) */
  float* dW_part;
  float* db_part;
  /* optional (dq_dz != NULL, C <= 4, C * A <= 32): dQ_c/da formed here from the critic's
   * first-layer pre-activation gradient instead of read from dq_da (the
   * critic backward's last input-gradient launch is skipped):
   * dQ_c/da_j = sum_k dq_dz[c*sdz_c + b*lddqz + k] * w0[c*sw0_c + k*ldw0 + da_off + j],
   * k < H0 <= 256 (w0: the critic's first layer, nn.Linear [H0][in] per member) */
  const float* dq_dz;
  int64_t lddqz, sdz_c;
  const float* w0;
  int64_t ldw0, sw0_c;
  int32_t H0;
  /* dq_min != 0 (with dq_da, not dq_dz): dq_da holds each critic's UNSCALED
   * dQ_c/da as n_part partial sums (d3a_sac_actor_q), q likewise:
   *   Q_c(b)      = sum_{p < n_part} q[p*sq_part + c*sqc + b]
   *   dQ_c/da_j   = sum_{p < n_part} dq_da[p*sda_part + c*sda_c + b*ld_da + da_off + j]
   * (parts summed in order); the backward of min over the ensemble is
   * applied here: dQ/da = dq_scale * dQ_m/da with m the first member of
   * least Q (`y.min(dim=0).values`, d3rlpy/models/torch/q_functions/
   * ensemble_q_function.py:12-13) and dq_scale = -1/B the actor loss's d/dq
   * ((entropy - q_t).mean(), d3rlpy/algos/torch/sac_impl.py:114-121)      */
  int32_t dq_min;
  float dq_scale;
  int32_t n_part;
  int64_t sq_part, sda_part;
  /* head_parts >= 2: the policy head rows as partial sums, as in
   * d3a_cql_sample_desc */
  int32_t head_parts;
  int64_t s_head_part;
} d3a_sac_actor_head_desc;
int d3a_sac_actor_head(const d3a_sac_actor_head_desc* d, void* stream);
/* The policy trunk backward (d3a_q2_bwd with dz2, C == 1, block_rows 32)
 * with d3a_sac_actor_head's dq_min work in its prologue: dz2 is formed per
 * workgroup from dhead (not written), dhead / db_part / dW_part / metrics[5]
 * as the head kernel writes them.  Replaces the two launches that follow
 * torch autograd through the policy's `_mu` / `_logstd` heads and encoder
 * (d3rlpy/models/torch/policies.py:170-176, encoders.py:165-176). */
int d3a_q2_bwd_actor_head(const d3a_q2_bwd_desc* d, const d3a_sac_actor_head_desc* head,
                          void* stream);

/* ---- the actor phase's critic pass in one launch (CQL / SAC actor update,
 *      d3rlpy/algos/torch/sac_impl.py:120 `self._q_func(obs, action, "min")`
 *      and its autograd back to the action input):
 * for an ensemble [n_in, 256, 256, 1] of C members and B rows x[b] = (s, a),
 * with the second hidden layer's units split into D3A_ACTOR_Q_PARTS parts p
 * of 64 (Q and dQ/da are linear in the parts' contributions):
 *   q[(p*C + c)*B + b]               = part p of Q_c(x[b]) (+ the head bias in p = 0)
 *   dq_da[((p*C + c)*B + b)*A + j]   = part p of dQ_c/dx_(da_off+j) at x[b], j < A,
 * UNSCALED (dL/dQ_c = 1); d3a_sac_actor_head (dq_min = 1, n_part =
 * D3A_ACTOR_Q_PARTS) sums the parts, selects the argmin member and scales.
 * Replaces the per-layer forward, d3a_head1_min and the input-gradient
 * launches of the actor phase.  One workgroup per 16 rows, member and part;
 * exact-fp32 MFMA chains.  Requires n_in <= 64, A <= 16, da_off + A <= n_in,
 * W1 / b rows 16-byte aligned.                                             */
#define D3A_ACTOR_Q_PARTS 4
typedef struct d3a_sac_actor_q_desc {
  const float* x;         /* [B][ldx] critic input rows (obs | action | pad) */
  int64_t ldx;
  const float* W0; const float* b0;   /* [C][256][n_in], [C][256] */
  const float* W1; const float* b1;   /* [C][256][256],  [C][256] */
  const float* wh; const float* bh;   /* [C][1][256],    [C][1]   */
  float* q;               /* [D3A_ACTOR_Q_PARTS][C][B]                      */
  float* dq_da;           /* [D3A_ACTOR_Q_PARTS][C][B][A]                   */
  int32_t B, C, n_in, A, da_off;
} d3a_sac_actor_q_desc;
int d3a_sac_actor_q(const d3a_sac_actor_q_desc* d, void* stream);

/* ---- device-resident dataset gather (replaces TransitionMiniBatch /
 *      _assign_to_batch, d3rlpy/dataset.pyx:1139-1342, and the index draw of
 *      RandomIterator._next, d3rlpy/iterators/random_iterator.py:38-41) ---- */
#define D3A_MAX_NSTEP 64
typedef struct d3a_gather_desc {
  /* dataset (device resident, structure of arrays over all stored steps) */
  const float* obs;          /* [n_rows][D] float observations (or NULL)   */
  const uint8_t* frames;     /* [n_rows][frame_bytes] image observations   */
  const float* act;          /* [n_rows][A] continuous actions (or NULL)   */
  const int32_t* act_i;      /* [n_rows] discrete actions (or NULL)        */
  const float* rew;          /* [n_rows] */
  const int64_t* t_row;      /* [n_trans] row of transition i              */
  const int64_t* t_ep_start; /* [n_trans] first row of its episode         */
  const int64_t* t_ep_last;  /* [n_trans] last transition index of episode */
  const uint8_t* t_terminal; /* [n_trans] 1 iff next obs is the zero dummy */
  int64_t n_trans;
  int32_t D, A, frame_bytes, n_frames, n_steps;
  float gamma;
  /* indices: either given (idx != NULL) or drawn on device (idx_out) */
  const int64_t* idx;
  int64_t* idx_out;
  uint64_t seed;
  int64_t* ctr;
  unsigned int* ticket;
  /* batch outputs */
  int32_t B;
  float* o_obs; uint8_t* o_frames;
  float* o_act; int32_t* o_act_i;
  float* o_rew; float* o_next_obs; uint8_t* o_next_frames;
  float* o_term; float* o_n_steps;
  /* drawn indices: row b takes draw number row_offset + b of the step, so
   * data-parallel ranks slice one global index stream */
  int64_t row_offset;
  /* optional [n_trans] terminal flag reported in o_term (NULL: t_terminal).
   * The online ReplayBuffer needs it: its transition into the terminal state
   * has terminal = 1 but a real next observation (online/buffers.py:268-281) */
  const float* t_term_value;
  /* gamma_pow[i] = powf(gamma, (float)i) for i < n_steps, filled by the host
   * with its C library's powf: the reference's n-step accumulation
   * `n_step_return += reward * gamma ** i` (dataset.pyx:1325; float gamma,
   * int i) is compiled by its pinned Cython 0.29.21 into
   * `acc = acc + reward * powf(gamma, (float)i)` — all fp32 — and powf is
   * not always the correctly rounded power, so the kernel reads the host's */
  float gamma_pow[D3A_MAX_NSTEP];
  /* drawn indices with ctr == NULL: the step's counter value is ctr_value
   * (the caller counts its draws; no device counter, no ticket) */
  int64_t ctr_value;
} d3a_gather_desc;
int d3a_gather_batch(const d3a_gather_desc* d, void* stream);

/* ---- TD3+BC stages (K1).  The layer GEMMs use d3a_gemm_f32 / d3a_rowdot_f32
 * / d3a_head1_bwd; these produce the layer inputs and loss gradients. ---- */

/* Standard-scaled Q inputs (replaces scaler.transform in TorchMiniBatch,
 * torch_utility.py:179-181 / preprocessing/scalers.py:350-354, plus the
 * torch.cat([x, action]) of ContinuousQFunction.forward):
 * x_q[b] = ((obs_b - mean) / (std + eps), act_b); x_targ[b][0:D) = scaled
 * next_obs_b.  mean == NULL: no scaler. */
typedef struct d3a_td3_prep_desc {
  const float* obs; const float* next_obs; const float* act;
  const float* mean; const float* std; float eps;
  float* x_q; float* x_targ;
  int32_t B, D, A, ldx;
} d3a_td3_prep_desc;
int d3a_td3_prep(const d3a_td3_prep_desc* d, void* stream);

/* Target policy smoothing (replaces TD3Impl.compute_target,
 * algos/torch/td3_impl.py:61-78): x_targ[b][D+j] =
 * clamp(tanh(head) + clamp(sigma * noise, -clip, clip), -1, 1). */
typedef struct d3a_td3_target_desc {
  const float* head; const float* noise; float sigma, clip;
  float* x_targ; int32_t ldx, D, B, A;
} d3a_td3_target_desc;
int d3a_td3_target(const d3a_td3_target_desc* d, void* stream);

/* Critic TD loss (replaces DDPGBaseImpl.compute_critic_loss,
 * algos/torch/ddpg_impl.py:154-167 -> EnsembleQFunction.compute_error with
 * the mean Q function's mse): dq[c][b] = dL/dq, metrics[0] = critic loss;
 * metrics[1] (actor loss) is set to NaN when actor_step == 0 (no actor
 * update at this step: TD3PlusBC._update, algos/td3_plus_bc.py:177-192). */
typedef struct d3a_td3_critic_loss_desc {
  const float* q; const float* q_targ;   /* [C][B] */
  const float* rew; const float* term; const float* n_steps;
  float* dq; float* metrics;
  int32_t B, C; float gamma; int32_t actor_step;
} d3a_td3_critic_loss_desc;
int d3a_td3_critic_loss(const d3a_td3_critic_loss_desc* d, void* stream);

/* TD3+BC actor loss (replaces TD3PlusBCImpl.compute_actor_loss,
 * algos/torch/td3_plus_bc_impl.py:64-70), in three stages around the
 * critic-0 forward / input backward:
 *   d3a_td3bc_actor_input  x_actor = (x_q[:, :D], tanh(head)), pi_act = tanh(head)
 *   d3a_td3bc_actor_seed   scalars[0] = lam = alpha / mean|q0|,
 *                          scalars[1] = -lam mean(q0), g = -lam / B
 *   d3a_td3bc_actor_head   dhead = (dq_da + d mse/da)(1 - a^2), metrics[1] = loss */
typedef struct d3a_td3bc_actor_desc {
  const float* head; const float* x_q; float* x_actor; float* pi_act;
  const float* q0; float* g; float* scalars;
  const float* dq_da; int32_t ld_da, da_off;
  const float* act; float* dhead; float* metrics;
  float alpha;
  int32_t B, D, A, ldx;
  /* 1: TD3+BC loss (lam = alpha / mean|Q0|, + BC term); 0: the DDPG / TD3
   * actor loss -mean Q0 (ddpg_impl.py:244-249), lam = 1, no BC term */
  int32_t bc;
} d3a_td3bc_actor_desc;
int d3a_td3bc_actor_input(const d3a_td3bc_actor_desc* d, void* stream);
int d3a_td3bc_actor_seed(const d3a_td3bc_actor_desc* d, void* stream);
int d3a_td3bc_actor_head(const d3a_td3bc_actor_desc* d, void* stream);

/* ---- BCQ stages (K3: continuous BCQ, quantile-regression critics).  The MLP
 * layers use d3a_mlp_fwd / d3a_gemm_f32; these build their input rows and
 * the loss gradients. ---- */

/* x[r] = (obs[r / rep], f(a[r])), r < rows; f by mode: 0 copy, 1 clamp(a,
 * -clip, clip) (the clipped latent of bcq_impl.py:139,180), 2 tanh(a)
 * (ConditionalVAE.decode, imitators.py:70-72), 3 clamp(base + scale *
 * tanh(a), -1, 1) (DeterministicResidualPolicy.forward, policies.py:94-97),
 * 4 as 3 with base = tanh(base) (the raw decoder output);
 * e_out (optional) also receives f(a).  Replaces _repeat_observation +
 * torch.cat of VectorEncoderWithAction (bcq_impl.py:163-187). */
typedef struct d3a_bcq_rows_desc {
  const float* obs; int32_t D, rep;
  const float* a; int32_t E; int64_t lda;
  const float* base;
  int32_t mode; float clip, scale;
  float* x; int64_t ldx;
  float* e_out;
  int64_t rows;
  /* a as head parts (d3a_mlp_fwd_desc.parts): a_parts > 1 sums a[q * s_a_part
   * + i] over q in order (part 0 holds the bias) */
  int32_t a_parts; int64_t s_a_part;
} d3a_bcq_rows_desc;
int d3a_bcq_rows(const d3a_bcq_rows_desc* d, void* stream);

/* ConditionalVAE.compute_error (imitators.py:80-86) around the encoder /
 * decoder MLPs, three stages:
 *   d3a_bcq_vae_sample    head_e = [mu | logstd] -> std = exp(clamp(logstd)),
 *                         z = mu + eps std, x_dec = (obs, z), scalars[0] = mean KL
 *   d3a_bcq_vae_loss      head_d -> y = tanh, metrics[0] = mse(y, act) + beta KL,
 *                         dhead_d = dL/dhead_d
 *   d3a_bcq_vae_enc_grad  dhead_e from dz = dx_dec[:, D:] and the KL term */
typedef struct d3a_bcq_vae_desc {
  const float* obs; const float* act; const float* eps;
  const float* head_e; float* std_out; float* x_dec; int64_t ldx;
  const float* head_d; float* dhead_d;
  const float* dx_dec; int64_t lddx; float* dhead_e;
  float* scalars; float* metrics;
  int32_t B, D, A, L;
  float beta, min_logstd, max_logstd;
  /* head_e / head_d as head parts of the encoder / decoder (head_parts > 1:
   * summed in part order, part strides s_e_part / s_d_part; a stride of 0
   * leaves that head a plain [B][.] matrix) */
  int32_t head_parts; int64_t s_e_part, s_d_part;
  /* optional: [B][L] per-element KL terms.  When set, d3a_bcq_vae_sample runs
   * one thread per (row, latent) over many workgroups and writes them, and
   * d3a_bcq_vae_loss forms the KL mean of the logged loss from them (in a
   * fixed order); null: one workgroup forms it into scalars[0]. */
  float* kl;
} d3a_bcq_vae_desc;
int d3a_bcq_vae_sample(const d3a_bcq_vae_desc* d, void* stream);
int d3a_bcq_vae_loss(const d3a_bcq_vae_desc* d, void* stream);
int d3a_bcq_vae_enc_grad(const d3a_bcq_vae_desc* d, void* stream);

/* compute_max_with_n_actions (q_functions/__init__.py:8-72): q = target
 * quantiles [C][B*N][K] (row b*N + n) -> target[b] = (1 - lam) q[cmax][b, n*]
 * + lam q[cmin][b, n*], n* = argmax_n mix of the per-critic quantile means. */
typedef struct d3a_bcq_target_desc {
  const float* q; float* target;
  int32_t B, N, K, C; float lam;
  /* optional: the quantile means [C][B*N] (d3a_mlp_fwd_x6's row_mean); when
   * null the kernel forms them from q */
  const float* means;
} d3a_bcq_target_desc;
int d3a_bcq_target(const d3a_bcq_target_desc* d, void* stream);

/* Quantile Huber TD loss of every critic (ContinuousQRQFunction.compute_error,
 * qr_q_function.py:130-150, q_functions/utility.py:27-61): dq = dL/dq
 * [C][B][K], loss_cb[c][b] = per-row loss (summed over critics and averaged
 * over rows by d3a_bcq_actor_head into metrics[1]). */
typedef struct d3a_bcq_qr_desc {
  const float* q; const float* target;
  const float* rew; const float* term; const float* n_steps;
  float* dq; float* loss_cb;
  int32_t B, K, C; float gamma;
  /* optional: the target formed in the loss launch (d3a_bcq_target's
   * arithmetic, bitwise) from the target pass's quantiles tg_q
   * [tg_C][B*tg_N][K] and their means tg_means [tg_C][B*tg_N]; target is then
   * not read (one launch fewer) */
  const float* tg_q; const float* tg_means; int32_t tg_N, tg_C; float tg_lam;
} d3a_bcq_qr_desc;
int d3a_bcq_qr_loss(const d3a_bcq_qr_desc* d, void* stream);

/* BCQImpl.compute_actor_loss backward through the residual policy
 * (bcq_impl.py:132-146): dhead = dq_da[:, da_off:] * [clamp pass] * scale *
 * (1 - tanh(head)^2); metrics[2] = -mean q0 (q0: member-0 quantiles [B][K]),
 * metrics[1] = sum_c mean_b loss_cb. */
typedef struct d3a_bcq_actor_desc {
  const float* head; const float* a_dec;
  const float* dq_da; int32_t ld_da, da_off;
  float* dhead; const float* q0; const float* loss_cb; float* metrics;
  int32_t B, A, K, C; float scale;
  int32_t head_parts; int64_t s_head_part;  /* head as parts (summed in order) */
} d3a_bcq_actor_desc;
int d3a_bcq_actor_head(const d3a_bcq_actor_desc* d, void* stream);

/* ---- DiscreteCQL + IQN on pixels (K5).  Convolutions are d3a_gemm_f32 over
 * im2col matrices; activations are NHWC (the GEMM's row-major output). ---- */

/* col[(b, oy, ox)][c*KH*KW + kh*KW + kw] = x[b, c, S*oy + kh, S*ox + kw]:
 * x_u8 NCHW uint8 scaled by 1/255 (PixelScaler.transform, scalers.py:109-110;
 * the first conv of PixelEncoder, encoders.py:130-136) or x_f32 NHWC. */
typedef struct d3a_im2col_desc {
  const uint8_t* x_u8; const float* x_f32;
  int32_t B, C, H, W, KH, KW, S, OH, OW;
  float* col; int64_t ldcol;
} d3a_im2col_desc;
int d3a_im2col(const d3a_im2col_desc* d, void* stream);

/* Deterministic (gather-form) col2im: dx[b][y][x][c] = sum of the dcol
 * entries whose window covers (y, x), times [mask > 0] (the producing
 * layer's ReLU) — the autograd of nn.Conv2d's input (encoders.py:130-136). */
typedef struct d3a_col2im_desc {
  const float* dcol; int64_t ldcol;
  const float* mask;
  float* dx;
  int32_t B, C, H, W, KH, KW, S, OH, OW;
} d3a_col2im_desc;
int d3a_col2im(const d3a_col2im_desc* d, void* stream);

/* Implicit-GEMM convolution (nn.Conv2d without padding) of PixelEncoder
 * (encoders.py:130-136): no im2col matrix in HBM.  Input x_u8 NCHW uint8,
 * scaled by 1/255 on load (PixelScaler.transform, scalers.py:109-110; needs
 * KW % 4 == 0) or x_f32 NHWC (the previous conv's output; needs C % 4 == 0);
 * weight [CO][C][KH][KW] (nn.Conv2d layout), CO = 32 or 64.
 *   d3a_conv_fwd:   y[(b, oy, ox)][co] = act(conv(x, weight) + bias)
 *                   (act = ReLU when relu != 0), NHWC.  fp32 input needs
 *                   `wpack`, CO*C*KH*KW floats of scratch (the weight is
 *                   re-laid [CO][KH][KW][C] there first, in the same stream).
 *   d3a_conv_bwd_w: dW[s][co][c][kh][kw] = sum over rows of split s of
 *                   dy[row][co] * x-window(row)[c][kh][kw]; db[s][co] (optional)
 *                   = sum of dy over the split's rows.  dy is the gradient at
 *                   the pre-activation, NHWC [B*OH*OW][CO]; rows are cut into
 *                   `splits` equal consecutive chunks (the Adam kernel sums the
 *                   split partials in order). */
typedef struct d3a_conv_desc {
  const uint8_t* x_u8; const float* x_f32;
  const float* weight; const float* bias;
  float* y; float* wpack;
  const float* dy; float* dW; float* db;
  int32_t B, C, H, W, KH, KW, S, OH, OW, CO;
  int32_t relu, splits;
  /* wpack_ready: wpack already holds the layout the entry reads (written by
   * d3a_conv_pack_weights earlier on the stream); 0: the entry packs it */
  int32_t wpack_ready;
} d3a_conv_desc;
int d3a_conv_fwd(const d3a_conv_desc* d, void* stream);
int d3a_conv_bwd_w(const d3a_conv_desc* d, void* stream);
/* The split count d3a_conv_bwd_w fills the chip with for this geometry (reads
 * B, C, KH, KW, OH, OW, CO only); callers size the dW / db partials with it. */
int32_t d3a_conv_bwd_w_splits(const d3a_conv_desc* d);
/* Input gradient of the convolution (autograd of nn.Conv2d's input,
 * encoders.py:130-136, through the previous layer's ReLU): y (as dx, NHWC
 * [B][H][W][C]) = [x_f32 > 0 when relu] * sum over the output positions whose
 * window covers the pixel of dy W -- one implicit GEMM per stride phase
 * (replaces the column-matrix GEMM + d3a_col2im pair).  Needs fp32 x
 * geometry with C = 32 or 64, CO % 16 == 0, dy 16-byte aligned.  With wpack
 * (CO * C * KH * KW floats of scratch) and CO % 32 == 0 the weight is first
 * re-laid [KH][KW][CO][C] there so every chunk load is coalesced. */
int d3a_conv_bwd_x(const d3a_conv_desc* d, void* stream);
/* The weight copies of up to 8 fp32-input layers in one launch: descs[i].weight
 * re-laid into descs[i].wpack in the order layouts[i] names -- 0: d3a_conv_fwd's
 * walk order [CO][KH][KW][C], 1: d3a_conv_bwd_x's tap-major [KH][KW][CO][C]. */
int d3a_conv_pack_weights(const d3a_conv_desc* descs, const int32_t* layouts, int32_t n,
                          void* stream);
/* The same, with a Philox fill (d3a_philox_fill's stream, arithmetic and
 * counter ticket; ph may be NULL) on appended workgroups: K5's tau draw for
 * the step's IQN evaluations in the weight copies' launch (round 6). */
int d3a_conv_pack_weights_philox(const d3a_conv_desc* descs, const int32_t* layouts, int32_t n,
                                 const d3a_philox_job* ph, void* stream);

/* Per-sample [P][C] (NHWC) <-> [C][P] (NCHW) transpose, optional [mask > 0]
 * in the destination layout: the flatten before PixelEncoder._fc
 * (encoders.py:157) and its gradient. */
typedef struct d3a_transpose_desc {
  const float* src; float* dst; const float* mask;
  int32_t B, P, C, to_cp;
} d3a_transpose_desc;
int d3a_iqn_transpose(const d3a_transpose_desc* d, void* stream);

/* prior[r][i] = cos(pi (i + 1) tau[r]), i < E (compute_iqn_feature,
 * iqn_q_function.py:33-44). */
typedef struct d3a_iqn_prior_desc {
  const float* taus; float* prior; int64_t rows; int32_t E;
} d3a_iqn_prior_desc;
int d3a_iqn_prior(const d3a_iqn_prior_desc* d, void* stream);

/* TD loss + gradient of the DQN family with the mean Q-function
 * (DiscreteMeanQFunction.compute_error, mean_q_function.py:25-40, Huber,
 * beta 1; DQNImpl / DoubleDQNImpl.compute_target, dqn_impl.py:128-171;
 * DiscreteCQLImpl.compute_loss, cql_impl.py:279-302, when alpha != 0).
 * q [B][A] = Q(s, .), q_next [B][A] = Q(s', .) (online; read when double_q),
 * q_targ [B][A] = Q_targ(s', .).  dq [B][A] = dL/dQ(s, .);
 * metrics[0..2] = loss, td loss, conservative loss. */
typedef struct d3a_dqn_loss_desc {
  const float* q;
  const float* q_next;
  const float* q_targ;
  const int32_t* act;
  const float* rew;
  const float* term;
  const float* n_steps;
  float* dq;
  float* metrics;
  int32_t B, A, double_q;
  float gamma, alpha;
} d3a_dqn_loss_desc;
int d3a_dqn_loss(const d3a_dqn_loss_desc* d, void* stream);

#define D3A_IQN_MAX_ACTIONS 18
#define D3A_IQN_MAX_GROUPS 8
#define D3A_IQN_HEAD_BWD_MAX_ROWS 512 /* G * K of d3a_iqn_head_bwd */
/* q[r][a] = (h[b] * phi[r]) . Wf[a] + bf[a] (compute_iqn_feature's product
 * + DiscreteIQNQFunction._fc, iqn_q_function.py:45-47, 82-88).  Rows come in
 * groups of group_rows = B*K; group g reads its features from h[g]
 * (b = (r mod group_rows) / K). */
typedef struct d3a_iqn_head_desc {
  const float* h[D3A_IQN_MAX_GROUPS];
  const float* phi; const float* Wf; const float* bf; float* q;
  int64_t rows, group_rows;
  int32_t K, F, A;
} d3a_iqn_head_desc;
int d3a_iqn_head_fwd(const d3a_iqn_head_desc* d, void* stream);

/* DiscreteCQL loss on IQN quantiles, one workgroup per row b
 * (DoubleDQNImpl.compute_target dqn_impl.py:162-171; DiscreteIQNQFunction.
 * compute_error iqn_q_function.py:95-118 with per-sample taus; DiscreteCQLImpl.
 * compute_loss / _compute_conservative_loss cql_impl.py:279-302):
 *   q_loss [3][B*K][A] online quantiles on obs (loss | logsumexp | data taus)
 *   q_next [B*K][A] online on next_obs (argmax), q_targ [B*K][A] target
 * -> dq [3][B*K][A], loss_b / cons_b per row, metrics[0] = loss,
 * metrics[1] = td, metrics[2] = conservative term. */
typedef struct d3a_iqn_loss_desc {
  const float* q_loss; const float* q_next; const float* q_targ;
  const int32_t* act; const float* rew; const float* term; const float* n_steps;
  const float* taus_loss;
  float* dq; float* loss_b; float* cons_b; float* metrics;
  int32_t B, K, A; float gamma, alpha;
} d3a_iqn_loss_desc;
int d3a_iqn_loss(const d3a_iqn_loss_desc* d, void* stream);

/* Backward of the IQN head over G gradient passes (rows g*B*K + b*K + k),
 * one workgroup per b: dphi = (dq Wf) * h * [phi > 0] (the embed ReLU),
 * dh = (sum_r (dq Wf) * phi) * [h > 0] (the encoder fc ReLU), and per-b
 * partials of dWf / dbf (summed in order by d3a_adam_f32). */
typedef struct d3a_iqn_head_bwd_desc {
  const float* h; const float* phi; const float* dq; const float* Wf;
  float* dphi; float* dh; float* dWf_part; float* dbf_part;
  int32_t B, K, F, A, G;
} d3a_iqn_head_bwd_desc;
int d3a_iqn_head_bwd(const d3a_iqn_head_bwd_desc* d, void* stream);

/* The IQN head forward in one launch (d3a_iqn_prior + the embed Linear + ReLU
 * + d3a_iqn_head_fwd): prior[r][e] = cos(pi (e + 1) taus[r]), phi[r] =
 * relu(prior[r] We^T + be), q[r][a] = (h[g][b] * phi[r]) . Wf[a] + bf[a] with
 * the row groups of d3a_iqn_head_desc (compute_iqn_feature + _compute_
 * quantiles, iqn_q_function.py:33-47, 82-88).  The embed product on the bf16
 * matrix cores with exact split-bf16 operands (fp32-accurate).  prior_out /
 * phi_out (optional) receive rows [0, n_keep) for a backward.  E == 64,
 * F <= 512 (multiple of 64), A <= 8, K a multiple of 32. */
typedef struct d3a_iqn_embed_head_desc {
  const float* taus;
  const float* We; const float* be;
  const float* h[D3A_IQN_MAX_GROUPS];
  const float* Wf; const float* bf;
  float* q;
  float* prior_out; float* phi_out;
  int64_t rows, group_rows, n_keep;
  int32_t K, E, F, A;
} d3a_iqn_embed_head_desc;
int d3a_iqn_embed_head(const d3a_iqn_embed_head_desc* d, void* stream);

/* The IQN head backward and the embed weight gradient in one launch (d3a_iqn_
 * head_bwd + the dWe = dphi^T prior GEMM, without the dphi round trip): over
 * the G gradient passes (rows g*B*K + b*K + k; phi / prior as the forward kept
 * them), NB batch rows per workgroup p = b / NB:
 *   dh[b] = (sum_r dprod * phi) * [h > 0], dprod = sum_a dq[r][a] Wf[a],
 *   dWf_part[p][a] / dbf_part[p][a], dWe_part[p][F][E] = sum_r dphi^T prior,
 *   dbe_part[p][F] = sum_r dphi, dphi = dprod * h * [phi > 0]
 * (the backward of compute_iqn_feature + _compute_quantiles, iqn_q_function.py:
 * 33-47, 82-88).  F == 512, E == 64, A <= 8, K a multiple of 32; the dWe
 * product on the bf16 matrix cores with exact split-bf16 operands. */
typedef struct d3a_iqn_head_bwd_fused_desc {
  const float* h; const float* phi; const float* prior; const float* dq; const float* Wf;
  float* dh; float* dWf_part; float* dbf_part; float* dWe_part; float* dbe_part;
  int32_t B, K, F, E, A, G, NB;
  /* recompute mode (taus set; phi / prior unused, may be null): the backward
   * rebuilds prior and phi = relu(We prior + be) of its rows from tau (row r's
   * tau at taus[r], the forward's rows) with the forward's ops; F 256 or 512 */
  const float* taus; const float* We; const float* be;
  /* optional (recompute mode, tests / diagnostics): the recomputed phi rows,
   * [rows][F] in the forward's row order -- what the backward's ReLU mask and
   * dh use, to compare with d3a_iqn_embed_head's phi_out */
  float* phi_dbg;
} d3a_iqn_head_bwd_fused_desc;
int d3a_iqn_head_bwd_fused(const d3a_iqn_head_bwd_fused_desc* d, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* D3RLPY_AMD_H_ */
