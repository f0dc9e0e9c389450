// HBM-bound and latency-bound pieces of the TransformerVAE step:
//   embedding gather / scatter-add      transformer_language_model.py:40-48 (tied head, :62-63)
//   reparameterise + KL (wave per sample) conditional_gaussian.py:18-28, continuous_autoencoder.py:42-52
//   cross-entropy finalize / gradient   language_model.py:98-113, 161-170
//   dropout-backward cast, splice-row extraction, dq finalize (inverse rotary, attention.py:194-208)
//   RAdam + clip (fused, one pass)      rectified_adam.py:16-88, language_model.py:120-122
#include "common.h"
#include "../../include/svae.h"

using namespace svae;

namespace {

// ------------------------------------------------------------------ embedding
__global__ __launch_bounds__(256) void emb_fwd_kernel(const int* __restrict__ ids, const float* __restrict__ table,
                                                      float* __restrict__ out, bf16* __restrict__ out_bf, int rows,
                                                      int D, float* __restrict__ out2) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const long long src = (long long)ids[row] * D;
  for (int c = lane * 4; c < D; c += 256) {
    const f32x4 v = *(const f32x4*)(table + src + c);
    *(f32x4*)(out + (long long)row * D + c) = v;
    if (out2) *(f32x4*)(out2 + (long long)row * D + c) = v;
    if (out_bf)
      *(bf16x4*)(out_bf + (long long)row * D + c) = (bf16x4){f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
  }
}

__global__ __launch_bounds__(256) void emb_bwd_kernel(const int* __restrict__ ids, const float* __restrict__ dout,
                                                      float* __restrict__ dtable, int rows, int D) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const long long dst = (long long)ids[row] * D;
  for (int c = lane; c < D; c += 64) atomicAdd(dtable + dst + c, dout[(long long)row * D + c]);
}

// Embedding backward fused with the one-hot part of the vocabulary head's dW (P-head, see ce_prob_*): dlogits =
// r (x) P - q (x) onehot(labels) puts -q[t] * hh[t] into table row labels[t]; labels[t] = ids[t + 1] inside a
// sequence (the head predicts the next token), so row ids[t] also receives -q[t-1] hh[t-1] (t % seq != 0): one
// atomic pass for both (q = 0 where the label is ignored).
__global__ __launch_bounds__(256) void emb_bwd_ce_kernel(const int* __restrict__ ids, const float* __restrict__ dout,
                                                         float* __restrict__ dtable, int rows, int D, int seq,
                                                         const bf16* __restrict__ hh, const float* __restrict__ q) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const long long dst = (long long)ids[row] * D;
  const float qp = (row % seq != 0) ? q[row - 1] : 0.f;
  const bf16* hp = hh + (long long)(row - 1) * D;
  for (int c = lane; c < D; c += 64) {
    float g = dout[(long long)row * D + c];
    if (qp != 0.f) g -= qp * (float)hp[c];
    atomicAdd(dtable + dst + c, g);
  }
}

// ------------------------------------------------------------------ reparameterise + KL
// One block of 16 waves; wave w takes samples w, w + 16, ... (latent index on the lane), 4 samples' loads in flight
// per wave, so B = 64 is one pass of 16 waves instead of 16 dependent iterations of 4 (21 -> ~4 us); the batch means
// come out of the same launch (a fixed-order sum over the waves' partials: deterministic).
constexpr int REPARAM_WAVES = 16;

__global__ __launch_bounds__(1024) void reparam_fwd_kernel(const float* __restrict__ stats, const float* __restrict__ eps_in,
                                                           unsigned long long seed, const long long* __restrict__ ntok,
                                                           float* __restrict__ z, bf16* __restrict__ z_bf,
                                                           float* __restrict__ eps_out, float* __restrict__ raw_kl,
                                                           float* __restrict__ kl_out, int B, int Z) {
  __shared__ float red[2][REPARAM_WAVES];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc_norm = 0.f, acc_raw = 0.f;
  constexpr int NB = 4;                       // samples per wave in flight
  for (int b0 = wave; b0 < B; b0 += NB * REPARAM_WAVES) {
    float klsum[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) klsum[k] = 0.f;
    for (int j = lane; j < Z; j += 64) {
      float mu[NB], lv[NB], e[NB];
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        const int b = b0 + k * REPARAM_WAVES;
        if (b < B) {
          mu[k] = stats[(long long)b * 2 * Z + j];
          lv[k] = stats[(long long)b * 2 * Z + Z + j];
          if (eps_in) {
            e[k] = eps_in[(long long)b * Z + j];
          } else {  // Box-Muller over two counter-based uniforms
            const unsigned long long idx = ((unsigned long long)b * Z + j) * 2ull;
            const float u1 = rand_uniform(seed, idx), u2 = rand_uniform(seed, idx + 1);
            e[k] = sqrtf(-2.f * __logf(u1)) * __cosf(6.283185307179586f * u2);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        const int b = b0 + k * REPARAM_WAVES;
        if (b < B) {
          const float var = __expf(lv[k]);
          const float zz = mu[k] + e[k] * sqrtf(var);
          if (eps_out) eps_out[(long long)b * Z + j] = e[k];
          z[(long long)b * Z + j] = zz;
          if (z_bf) z_bf[(long long)b * Z + j] = f2bf(zz);
          klsum[k] += 0.5f * (mu[k] * mu[k] + var - lv[k] - 1.0f);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int b = b0 + k * REPARAM_WAVES;
      if (b < B) {                            // wave-uniform
        const float ks = wave_sum(klsum[k]);
        if (lane == 0) raw_kl[b] = ks;
        acc_raw += ks;
        acc_norm += ks / (float)ntok[b];
      }
    }
  }
  if (lane == 0) { red[0][wave] = acc_norm; red[1][wave] = acc_raw; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float n = 0.f, r = 0.f;
#pragma unroll
    for (int w = 0; w < REPARAM_WAVES; ++w) { n += red[0][w]; r += red[1][w]; }
    kl_out[0] = n / B;
    kl_out[1] = r / B;
  }
}

__global__ __launch_bounds__(256) void reparam_bwd_kernel(const float* __restrict__ stats, const float* __restrict__ eps,
                                                          const float* __restrict__ dz, const long long* __restrict__ ntok,
                                                          const float* __restrict__ gkl, float* __restrict__ dstats,
                                                          int B, int Z) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * Z) return;
  const int b = i / Z, j = i % Z;
  const float mu = stats[(long long)b * 2 * Z + j];
  const float lv = stats[(long long)b * 2 * Z + Z + j];
  const float var = __expf(lv), sd = sqrtf(var);
  const float w = gkl[0] / ((float)B * (float)ntok[b]);   // d loss / d raw_kl[b]
  const float g = dz ? dz[i] : 0.f;
  dstats[(long long)b * 2 * Z + j] = g + w * mu;
  dstats[(long long)b * 2 * Z + Z + j] = g * eps[i] * sd * 0.5f + w * 0.5f * (var - 1.0f);
}

// ------------------------------------------------------------------ cross entropy
// Row pass: lse from the per-128-column (max, sumexp) partials of the logits GEMM, per-row loss.
__global__ __launch_bounds__(256) void ce_rows_kernel(const float* __restrict__ part, int ntile,
                                                      const float* __restrict__ label_logit, const int* __restrict__ labels,
                                                      int rows, float* __restrict__ lse, float* __restrict__ row_loss) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float2* pr = (const float2*)part + (long long)row * ntile;
  float mx = -INFINITY;
  for (int t = lane; t < ntile; t += 64) mx = fmaxf(mx, pr[t].x);
  mx = wave_max(mx);
  float se = 0.f;
  for (int t = lane; t < ntile; t += 64) {
    const float2 v = pr[t];
    se += (v.x == -INFINITY) ? 0.f : v.y * __expf(v.x - mx);
  }
  se = wave_sum(se);
  if (lane == 0) {
    const float l = mx + __logf(se);
    lse[row] = l;
    row_loss[row] = labels[row] != 0 ? l - label_logit[row] : 0.f;
  }
}

// ---- P-head cross entropy (training): the vocabulary GEMM stores P = exp(logit - c) with c = the row's label
// logit (SVAE_EPI_CE_PROB) instead of the logits, so the backward needs no exponential and no dlogits pass:
//   dlogits = r (x) P - q (x) onehot,  q = g * w_chunk (0 for ignored rows),  r = q * exp(c - lse)
//   dX = r . (P W) - q W[label]   (SVAE_EPI_ROWSCALE_GATHER)
//   dW = P^T (r . hh) + [one-hot part, folded into the embedding backward], d bias = sum_t r_t P[t] - hist(q)
// c from ce_label_logit: one wave per row, f32 dot of the bf16 operands + bias (0 for ignored rows).
__global__ __launch_bounds__(256) void ce_label_logit_kernel(const bf16* __restrict__ hh, long long ldh,
                                                             const bf16* __restrict__ W, long long ldw,
                                                             const float* __restrict__ bias,
                                                             const int* __restrict__ labels, int rows, int D,
                                                             float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lab = labels[row];
  if (lab == 0) {
    if (lane == 0) out[row] = 0.f;
    return;
  }
  float acc = 0.f;
  for (int c = lane * 8; c < D; c += 512) {
    const bf16x8 a = *(const bf16x8*)(hh + (long long)row * ldh + c);
    const bf16x8 b = *(const bf16x8*)(W + (long long)lab * ldw + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc = fmaf((float)a[e], (float)b[e], acc);
  }
  acc = wave_sum(acc);
  if (lane == 0) out[row] = acc + (bias ? bias[lab] : 0.f);
}

// lse = c + log(sum of the row's per-tile sums of P); row loss = lse - c (labelled rows; 0 and lse = 0 otherwise).
// part is tile-major [ntile][rows]. Block = 32 rows x 8 tile slices (thread (r, s) sums tiles s, s + 8, ..., 8 loads in
// flight), the 8 slice sums combined in LDS in a fixed order. (One thread per row walking all 256 tiles: 512 waves
// on the chip, 37.6 us at C2.)
// A labelled row whose sum reaches 2^100 (a logit more than ~69 nats above the label logit, or a non-finite one) is
// appended to sat[1..] (count in sat[0]) for ce_prob_fixup: the GEMM epilogue's exp2 overflows to +inf past 88 nats, so
// such a row's P and lse are recomputed with the row maximum as the offset.
__global__ __launch_bounds__(256) void ce_prob_rows_kernel(const float* __restrict__ part, int ntile,
                                                           const float* __restrict__ off, const int* __restrict__ labels,
                                                           int rows, float* __restrict__ lse, float* __restrict__ row_loss,
                                                           int* __restrict__ sat) {
  __shared__ float red[8][33];
  const int r = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int row = blockIdx.x * 32 + r;
  float acc = 0.f;
  if (row < rows) {
    int t = sl;
    for (; t + 56 < ntile; t += 64) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(long long)(t + 8 * u) * rows + row];
      acc += ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
    }
    for (; t < ntile; t += 8) acc += part[(long long)t * rows + row];
  }
  red[sl][r] = acc;
  __syncthreads();
  if (sl != 0 || row >= rows) return;
  float se = red[0][r];
#pragma unroll
  for (int k = 1; k < 8; ++k) se += red[k][r];
  const bool live = labels[row] != 0;
  const float l = live ? __logf(se) : 0.f;
  lse[row] = live ? off[row] + l : 0.f;
  row_loss[row] = l;
  if (sat && live && !(se < 0x1p100f)) sat[1 + atomicAdd(sat, 1)] = row;
}

// The rows ce_prob_rows flagged, one block per row (blocks stride over the list; an empty list costs one launch):
// logit = hh . W[col] + bias[col] over the whole vocabulary (bf16 operands, f32 accumulation, as the GEMM), m = the
// row maximum; P[row] = exp(logit - m) (bf16), lse = m + log sum, row_loss = lse - c (c = the label logit, the old
// offset), and the offset becomes m, so the backward's r = q exp(off - lse) stays consistent with the new P.
__global__ __launch_bounds__(256) void ce_prob_fixup_kernel(const int* __restrict__ sat, const bf16* __restrict__ hh,
                                                            long long ldh, const bf16* __restrict__ W, long long ldw,
                                                            const float* __restrict__ bias, bf16* __restrict__ P,
                                                            long long ldp, int V, int D, float* __restrict__ off,
                                                            float* __restrict__ lse, float* __restrict__ row_loss) {
  __shared__ float h[1024];
  __shared__ float red[4];
  // Every flagged row is recomputed (each costs 2 V D MACs on one block, ~0.3 ms at V = 32768, D = 512: a handful of
  // rows costs one round of the grid; a diverging step that saturates every row of C2 ~40 ms) -- an overflowed P left
  // in place would feed inf / NaN gradients to clip and RAdam, where the reference's log-softmax stays finite.
  // sat[0] counts the flagged rows (out['ce_saturated']).
  const int n = sat[0];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    const int row = sat[1 + i];
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += 256) h[c] = (float)hh[(long long)row * ldh + c];
    __syncthreads();
    float mx = -INFINITY;
    for (int col = threadIdx.x; col < V; col += 256) {
      const bf16* wr = W + (long long)col * ldw;
      float acc = 0.f;
      for (int c = 0; c < D; c += 8) {
        const bf16x8 b = *(const bf16x8*)(wr + c);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc = fmaf(h[c + e], (float)b[e], acc);
      }
      mx = fmaxf(mx, acc + (bias ? bias[col] : 0.f));
    }
    mx = wave_max(mx);
    if (lane == 0) red[w] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    float se = 0.f;
    for (int col = threadIdx.x; col < V; col += 256) {
      const bf16* wr = W + (long long)col * ldw;
      float acc = 0.f;
      for (int c = 0; c < D; c += 8) {
        const bf16x8 b = *(const bf16x8*)(wr + c);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc = fmaf(h[c + e], (float)b[e], acc);
      }
      const float p = __expf(acc + (bias ? bias[col] : 0.f) - mx);
      P[(long long)row * ldp + col] = f2bf(p);
      se += p;
    }
    se = wave_sum(se);
    if (lane == 0) red[w] = se;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float l = mx + __logf(red[0] + red[1] + red[2] + red[3]);
      row_loss[row] = l - off[row];
      lse[row] = l;
      off[row] = mx;
    }
  }
}

// Backward prologue of the P-head, one wave per row: q = g * w_chunk, r = q * exp(c - lse) (0 for ignored rows),
// hh_out = r * hh (the B operand of dW = P^T (r . hh)), d bias[label] -= q (the one-hot column sums).
__global__ __launch_bounds__(256) void ce_prob_bwd_prep_kernel(const bf16* __restrict__ hh, long long ldh,
                                                               const float* __restrict__ lse,
                                                               const float* __restrict__ off,
                                                               const float* __restrict__ chunk_w,
                                                               const int* __restrict__ labels,
                                                               const float* __restrict__ gscale, int rows, int seq,
                                                               int nchunks, int chunk_len, int D,
                                                               bf16* __restrict__ hh_out, float* __restrict__ r_out,
                                                               float* __restrict__ q_out, float* __restrict__ dbias) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lab = labels[row];
  float q = 0.f, r = 0.f;
  if (lab != 0) {
    const int ch = min((row % seq) / chunk_len, nchunks - 1);
    q = gscale[0] * chunk_w[ch];
    r = q * __expf(off[row] - lse[row]);
  }
  for (int c = lane * 8; c < D; c += 512) {
    const bf16x8 a = *(const bf16x8*)(hh + (long long)row * ldh + c);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(r * (float)a[e]);
    *(bf16x8*)(hh_out + (long long)row * D + c) = o;
  }
  if (lane == 0) {
    r_out[row] = r;
    q_out[row] = q;
    if (lab != 0 && dbias) atomicAdd(dbias + lab, -q);
  }
}

// log p(x|z) summed over each sequence (continuous_autoencoder.py:82-88): one block of 4 waves per sequence;
// a wave finalises one row's logsumexp from the per-tile partials at a time. Label 0 rows add 0.
__global__ __launch_bounds__(256) void ce_seq_logprob_kernel(const float* __restrict__ part, int ntile,
                                                             const float* __restrict__ label_logit,
                                                             const int* __restrict__ labels, int seq,
                                                             float* __restrict__ out) {
  __shared__ float ws[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long r0 = (long long)blockIdx.x * seq;
  float acc = 0.f;
  for (int i = w; i < seq; i += 4) {
    const long long row = r0 + i;
    if (labels[row] == 0) continue;                 // wave-uniform
    const float2* pr = (const float2*)part + row * ntile;
    float mx = -INFINITY;
    for (int t = lane; t < ntile; t += 64) mx = fmaxf(mx, pr[t].x);
    mx = wave_max(mx);
    float se = 0.f;
    for (int t = lane; t < ntile; t += 64) {
      const float2 v = pr[t];
      se += (v.x == -INFINITY) ? 0.f : v.y * __expf(v.x - mx);
    }
    se = wave_sum(se);
    acc += label_logit[row] - (mx + __logf(se));
  }
  if (lane == 0) ws[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// ------------------------------------------------------------------ marginal KL (mutual-information log)
// math_utils.py:51-58: S posterior samples x[s][i] = mu_i + eps * scale_i; log q_j(x) summed over the latent;
// marginal[s][i] = logsumexp_j log q_j(x[s][i]) - log B. One block per (s, i), a thread per posterior j; the block
// also sums x^2. Partials go to ws[s*B + i] (marginal) and ws[S*B + s*B + i] (sum x^2); mi_final reduces them in
// a fixed order: mi = kl - (sample_prob - mean(marginal)), sample_prob = -0.5 (mean sum x^2 + Z log 2 pi).
__global__ __launch_bounds__(256) void mi_marginal_kernel(const float* __restrict__ stats, const float* __restrict__ eps,
                                                          unsigned long long seed, int B, int Z,
                                                          float* __restrict__ ws) {
  extern __shared__ float xs[];            // [Z] the sample
  __shared__ float red[8];
  const int si = blockIdx.x, i = si % B, tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  float sq = 0.f;
  for (int z = tid; z < Z; z += 256) {
    const float mu = stats[(long long)i * 2 * Z + z];
    const float sd = sqrtf(__expf(stats[(long long)i * 2 * Z + Z + z]));
    float e;
    if (eps) {
      e = eps[(long long)si * Z + z];
    } else {
      const unsigned long long idx = ((unsigned long long)si * Z + z) * 2ull;
      const float u1 = rand_uniform(seed, idx), u2 = rand_uniform(seed, idx + 1);
      e = sqrtf(-2.f * __logf(u1)) * __cosf(6.283185307179586f * u2);
    }
    const float x = mu + e * sd;
    xs[z] = x;
    sq += x * x;
  }
  __syncthreads();
  // log q_j(x) = sum_z -(x - mu)^2 / (2 var) - log(sd) - log(sqrt(2 pi)); a thread's j's fold into an online
  // logsumexp (m, e), then the block combines the 256 pairs
  const float lsq2pi = 0.91893853320467274f;   // log(sqrt(2 pi))
  float m = -INFINITY, e = 0.f;
  for (int j = tid; j < B; j += 256) {
    const float* st = stats + (long long)j * 2 * Z;
    float acc = 0.f;
    for (int z = 0; z < Z; ++z) {
      const float lv = st[Z + z];
      const float d = xs[z] - st[z];
      acc += -(d * d) * (0.5f * __expf(-lv)) - 0.5f * lv - lsq2pi;
    }
    const float nm = fmaxf(m, acc);
    e = e * __expf(m - nm) + __expf(acc - nm);
    m = nm;
  }
  float mx = wave_max(m);
  if (lane == 0) red[w] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float se = wave_sum(m == -INFINITY ? 0.f : e * __expf(m - mx));
  sq = wave_sum(sq);
  if (lane == 0) { red[w] = se; red[4 + w] = sq; }
  __syncthreads();
  if (tid == 0) {
    ws[si] = mx + __logf(red[0] + red[1] + red[2] + red[3]) - __logf((float)B);
    ws[gridDim.x + si] = red[4] + red[5] + red[6] + red[7];
  }
}

__global__ __launch_bounds__(256) void mi_final_kernel(const float* __restrict__ ws, int n, int Z,
                                                       const float* __restrict__ kl, float* __restrict__ out) {
  __shared__ float red[8];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float m = 0.f, q = 0.f;
  for (int k = tid; k < n; k += 256) { m += ws[k]; q += ws[n + k]; }
  m = wave_sum(m);
  q = wave_sum(q);
  if (lane == 0) { red[w] = m; red[4 + w] = q; }
  __syncthreads();
  if (tid == 0) {
    const float mm = (red[0] + red[1] + red[2] + red[3]) / n;
    const float qq = (red[4] + red[5] + red[6] + red[7]) / n;
    const float sample_prob = -0.5f * (qq + Z * 1.8378770664093453f);   // log(2 pi)
    out[0] = kl[0] - (sample_prob - mm);
  }
}

// Chunked mean-of-means (robust_cross_entropy, language_model.py:163-170): grid (CE_RED_BLOCKS, nchunks); block
// (b, c) sums the loss and count of chunk c's rows (positions c*chunk_len .. of every sequence; the last chunk runs
// to the end of the sequence) into part[c][b]; one small block adds them in a fixed order and writes nll and the
// per-chunk row weights (deterministic). tok_w (optional, f32 [V]): per-target class weights, F.cross_entropy's
// `weight` (the val_bpb metric, language_model.py:106-110): sum w[y] l / sum w[y] per chunk.
constexpr int CE_RED_BLOCKS = 64;
constexpr int CE_MAX_CHUNKS = 1024;

__global__ __launch_bounds__(256) void ce_reduce_part_kernel(const float* __restrict__ row_loss,
                                                             const int* __restrict__ labels,
                                                             const float* __restrict__ tok_w, int rows, int seq,
                                                             int nchunks, int chunk_len, float* __restrict__ part) {
  __shared__ float red[8];
  const int ch = blockIdx.y;
  const int p0 = ch * chunk_len;
  const int clen = ch == nchunks - 1 ? seq - p0 : chunk_len;
  const int n = (rows / seq) * clen;
  float s = 0.f, c = 0.f;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += CE_RED_BLOCKS * 256) {
    const int r = (i / clen) * seq + p0 + i % clen;
    const int lab = labels[r];
    if (lab != 0) {
      const float w = tok_w ? tok_w[lab] : 1.f;
      s += w * row_loss[r];
      c += w;
    }
  }
  s = wave_sum(s);
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = s; red[4 + (threadIdx.x >> 6)] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float* o = part + ((long long)ch * CE_RED_BLOCKS + blockIdx.x) * 2;
    o[0] = (red[0] + red[1]) + (red[2] + red[3]);
    o[1] = (red[4] + red[5]) + (red[6] + red[7]);
  }
}

__global__ __launch_bounds__(256) void ce_reduce_final_kernel(const float* __restrict__ part, int nchunks,
                                                              float* __restrict__ chunk_w, float* __restrict__ nll_out) {
  __shared__ float mean[CE_MAX_CHUNKS];
  for (int k = threadIdx.x; k < nchunks; k += 256) {
    float ts = 0.f, tc = 0.f;
    for (int b = 0; b < CE_RED_BLOCKS; ++b) {
      ts += part[((long long)k * CE_RED_BLOCKS + b) * 2];
      tc += part[((long long)k * CE_RED_BLOCKS + b) * 2 + 1];
    }
    mean[k] = ts / tc;
    if (chunk_w) chunk_w[k] = 1.0f / (tc * (float)nchunks);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float nll = 0.f;
    for (int j = 0; j < nchunks; ++j) nll += mean[j];
    nll_out[0] = nll / nchunks;
  }
}

// dlogits = g * w_chunk * (softmax - onehot), in place on bf16 logits, fused with the output-bias gradient
// db[v] += sum_rows dlogits[row][v] (the reference's autograd sums it separately). Block = 256 threads x 8
// columns = a 2048-column strip, walking `rows_per_block` rows: every row is one contiguous 4 KiB read+write.
// logits are read once and dlogits are consumed by the next GEMMs from HBM (2 GiB at C2, far beyond the caches):
// nontemporal loads/stores (797 vs 869 us in the C2 step, scripts/ce_probe.py and scripts/_ab_run.sh); 2 rows in
// flight per thread measured best (4: 814, 8: 818 us)
#define CE_U 2
#define CE_LOAD(p) __builtin_nontemporal_load(p)
#define CE_STORE(v, p) __builtin_nontemporal_store(v, p)
__global__ __launch_bounds__(256) void ce_grad_kernel(bf16* __restrict__ logits, long long ld, const float* __restrict__ lse,
                                                      const float* __restrict__ chunk_w, const int* __restrict__ labels,
                                                      const float* __restrict__ gscale, float* __restrict__ dbias, int rows,
                                                      int V, int seq, int nchunks, int chunk_len, int rows_per_block) {
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * 8;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  const float g = gscale[0];
  float db[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < V) {
    // CE_U rows per iteration with all loads issued before any store (the stores would otherwise order the next
    // row's load behind them: one HBM round trip per row)
    for (int row = r0; row < r1; row += CE_U) {
      bf16x8 v[CE_U];
#pragma unroll
      for (int u = 0; u < CE_U; ++u)
        if (row + u < r1) v[u] = CE_LOAD((const bf16x8*)(logits + (long long)(row + u) * ld + c0));
#pragma unroll
      for (int u = 0; u < CE_U; ++u) {
        const int rr = row + u;
        if (rr >= r1) break;
        bf16x8* ptr = (bf16x8*)(logits + (long long)rr * ld + c0);
        const int lab = labels[rr];
        bf16x8 o;
        if (lab == 0) {
          o = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
        } else {
          const int ch = min((rr % seq) / chunk_len, nchunks - 1);
          const float w = g * chunk_w[ch];
          const float l = lse[rr];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float pr = __expf((float)v[u][e] - l);
            if (c0 + e == lab) pr -= 1.0f;
            const float d = w * pr;
            db[e] += d;
            o[e] = f2bf(d);
          }
        }
        CE_STORE(o, ptr);
      }
    }
    if (dbias) {
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(dbias + c0 + e, db[e]);
    }
  }
}

// ------------------------------------------------------------------ misc elementwise
__global__ __launch_bounds__(256) void dropout_bwd_cast_kernel(const float* __restrict__ g, bf16* __restrict__ out, float p,
                                                               unsigned long long seed, long long n, int cols, long long ld_in) {
  const float scale = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  for (long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += (long long)gridDim.x * 1024) {
    const long long r = i / cols;
    const int c = (int)(i % cols);
    const f32x4 v = *(const f32x4*)(g + r * ld_in + c);
    bf16x4 o;
    float u[4] = {1.f, 1.f, 1.f, 1.f};
    if (p > 0.f) rand_uniform4(seed, (unsigned long long)i >> 2, u);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x = v[e];
      if (p > 0.f) x = (u[e] >= p) ? x * scale : 0.f;
      o[e] = f2bf(x);
    }
    *(bf16x4*)(out + i) = o;
  }
}

// The step's token inputs in one pass (engine.forward): ids32 = int32(ids), labels = ids shifted left by one within
// each sequence with 0 at its last position (language_model.py: the next-token targets), the uint8 key-padding mask
// (pad_mode 1: ids == 0, 2: from the caller's bool mask, 0: none) and the per-sequence token counts.
__global__ __launch_bounds__(256) void prep_tokens_kernel(const int64_t* __restrict__ ids, const unsigned char* __restrict__ pad,
                                                          int pad_mode, int rows, int L, int32_t* __restrict__ ids32,
                                                          int32_t* __restrict__ labels, unsigned char* __restrict__ padm,
                                                          const int64_t* __restrict__ ntok, int64_t* __restrict__ ntok_out,
                                                          int B) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t < B && ntok) ntok_out[t] = ntok[t];
  if (t >= rows) return;
  const int64_t v = ids[t];
  ids32[t] = (int32_t)v;
  labels[t] = (t % L == L - 1) ? 0 : (int32_t)ids[t + 1];
  if (pad_mode == 1) padm[t] = v == 0;
  else if (pad_mode == 2) padm[t] = pad[t] != 0;
}

// loss = nll + kl_weight * kl (transformer_vae.py:55) and the backward's gradient scales gs = (gloss, gloss *
// kl_weight), each op rounded as the torch expressions it replaces (no contraction into an fma)
__global__ __launch_bounds__(64) void step_scalars_kernel(const float* __restrict__ nll, const float* __restrict__ kl,
                                                          const float* __restrict__ gloss, float kw,
                                                          float* __restrict__ loss, float* __restrict__ gs) {
  if (threadIdx.x != 0) return;
  if (loss) loss[0] = __fadd_rn(nll[0], __fmul_rn(kw, kl[0]));
  if (gs) {
    const float g = gloss[0];
    gs[0] = g;
    gs[1] = __fmul_rn(g, kw);
  }
}

__global__ __launch_bounds__(256) void gelu_bwd_kernel(const float* __restrict__ dx, const bf16* __restrict__ gp,
                                                       bf16* __restrict__ out, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    out[i] = f2bf(dx[i] * (float)gp[i]);
}

__global__ __launch_bounds__(256) void cast_kernel(const float* __restrict__ in, bf16* __restrict__ out, long long n) {
  for (long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += (long long)gridDim.x * 1024) {
    if (i + 4 <= n) {
      const f32x4 v = *(const f32x4*)(in + i);
      *(bf16x4*)(out + i) = (bf16x4){f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
    } else {
      for (long long j = i; j < n; ++j) out[j] = f2bf(in[j]);
    }
  }
}

__global__ __launch_bounds__(256) void extract_rows_kernel(float* __restrict__ x, long long ld, int nout, int mod, int D,
                                                           float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= nout * D) return;
  const int r = i / D, c = i % D;
  float* src = x + (long long)r * mod * ld + c;
  out[(long long)r * D + c] = *src;
  *src = 0.f;
}

__global__ __launch_bounds__(256) void dq_finalize_kernel(const float* __restrict__ dq, bf16* __restrict__ out, long long ldo,
                                                          int rows, int D, const float* __restrict__ rot, int seq) {
  const long long n2 = (long long)rows * (D / 2);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long long)gridDim.x * 256) {
    const int row = (int)(i / (D / 2));
    const int pr = (int)(i % (D / 2));
    const float2 v = *(const float2*)(dq + (long long)row * D + 2 * pr);
    float a = v.x, b = v.y;
    if (rot) {  // inverse of (a c - b s, b c + a s)
      const float2 cs = ((const float2*)rot)[(long long)(row % seq) * (D / 2) + pr];
      a = v.x * cs.x + v.y * cs.y;
      b = -v.x * cs.y + v.y * cs.x;
    }
    bf16* o = out + (long long)row * ldo + 2 * pr;
    o[0] = f2bf(a);
    o[1] = f2bf(b);
  }
}


// Transposed bf16 weight shadows: for each block b of table[b] = (offset, rows, cols, first_tile),
// dst[offset + c * rows + r] = src[offset + r * cols + c]. One 64 x 64 tile per workgroup through a padded LDS
// tile; 16-B loads and stores (rows, cols % 8 == 0).
__global__ __launch_bounds__(256) void transpose_blocks_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst,
                                                               const long long* __restrict__ table, int nb) {
  __shared__ unsigned short t[64][66];
  __shared__ int sfirst[256];
  const int tile = blockIdx.x;
  // the block this tile belongs to: the first tiles of up to 256 blocks come in one coalesced load and are searched
  // in LDS (a dependent global load per table entry cost the last tiles ~100 L2 round trips); more blocks: a binary
  // search over the table in global memory
  int b = 0;
  if (nb <= 256) {
    for (int i = threadIdx.x; i < nb; i += 256) sfirst[i] = (int)table[i * 4 + 3];
    __syncthreads();
    int lo = 0, hi = nb - 1;   // last b with first_tile[b] <= tile
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (sfirst[mid] <= tile) lo = mid; else hi = mid - 1;
    }
    b = lo;
  } else {
    int lo = 0, hi = nb - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (table[mid * 4 + 3] <= tile) lo = mid; else hi = mid - 1;
    }
    b = lo;
  }
  const long long off = table[b * 4], rows = table[b * 4 + 1], cols = table[b * 4 + 2];
  const int local = tile - (int)table[b * 4 + 3];
  const int tcols = (int)((cols + 63) / 64);
  const int r0 = (local / tcols) * 64, c0 = (local % tcols) * 64;
  const int tid = threadIdx.x, c8 = (tid & 7) * 8;
  const unsigned short* s = (const unsigned short*)src + off;
  unsigned short* d = (unsigned short*)dst + off;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (tid >> 3) + 32 * i;
    if (r0 + r < rows && c0 + c8 < cols) {
      const u32x4 v = *(const u32x4*)(s + (r0 + r) * cols + c0 + c8);
      const unsigned short* e = (const unsigned short*)&v;
#pragma unroll
      for (int j = 0; j < 8; ++j) t[r][c8 + j] = e[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = (tid >> 3) + 32 * i;   // output row = input column
    if (c0 + c < cols && r0 + c8 < rows) {
      u32x4 v;
      unsigned short* e = (unsigned short*)&v;
#pragma unroll
      for (int j = 0; j < 8; ++j) e[j] = t[c8 + j][c];
      *(u32x4*)(d + (c0 + c) * rows + r0 + c8) = v;
    }
  }
}

// ------------------------------------------------------------------ optimiser
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, long long n, float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  // four 16-B loads in flight per thread (one per iteration left a single load in flight: 36.8 us for 185 MB)
  const long long stride = (long long)gridDim.x * 1024;
  long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  for (; i + 3 * stride + 4 <= n; i += 4 * stride) {
    const f32x4 v0 = *(const f32x4*)(g + i), v1 = *(const f32x4*)(g + i + stride);
    const f32x4 v2 = *(const f32x4*)(g + i + 2 * stride), v3 = *(const f32x4*)(g + i + 3 * stride);
    const f32x4 q = (v0 * v0 + v1 * v1) + (v2 * v2 + v3 * v3);
    s += (q[0] + q[1]) + (q[2] + q[3]);
  }
  for (; i < n; i += stride) {
    if (i + 4 <= n) {
      const f32x4 v = *(const f32x4*)(g + i);
      s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
    } else {
      for (long long j = i; j < n; ++j) s += g[j] * g[j];
    }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// scal: {lr_eff, bcm, bcv, rho_ok, beta1, beta2, eps, wd, max_norm}
template <int U, bool NTIN>
__global__ __launch_bounds__(256) void radam_kernel(float* __restrict__ p, bf16* __restrict__ pbf, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, long long n,
                                                    const float* __restrict__ part, int nblk, const float* __restrict__ scal,
                                                    float* __restrict__ norm_out) {
  __shared__ float red[4];
  __shared__ float s_coef;
  float s = 0.f;
  for (int i = threadIdx.x; i < nblk; i += 256) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float norm = sqrtf(red[0] + red[1] + red[2] + red[3]);
    const float max_norm = scal[8];
    s_coef = fminf(1.0f, max_norm / (norm + 1e-6f));
    if (blockIdx.x == 0 && norm_out) norm_out[0] = norm;
  }
  __syncthreads();
  const float coef = s_coef;
  const float lr = scal[0], bcm = scal[1], bcv = scal[2], rho_ok = scal[3], b1 = scal[4], b2 = scal[5], eps = scal[6],
              wd = scal[7];
  const float step = lr / bcm, decay = 1.0f - lr * wd;
  const long long n4 = n / 4;   // n % 4 == 0 (checked on the host): 16-B vectors
  auto update = [&](long long i, f32x4 gi, f32x4 m0, f32x4 v0, f32x4 p0) {
    gi *= coef;
    const f32x4 mi = m0 * b1 + (1.0f - b1) * gi;
    const f32x4 vi = v0 * b2 + (1.0f - b2) * gi * gi;
    // the moments are read again only by the next step's update: nontemporal
    __builtin_nontemporal_store(mi, (f32x4*)m + i);
    __builtin_nontemporal_store(vi, (f32x4*)v + i);
    f32x4 pi = p0 * decay;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (rho_ok != 0.f) pi[e] -= step * (mi[e] / (sqrtf(vi[e]) / bcv + eps));
      else pi[e] -= step * mi[e];
    }
    ((f32x4*)p)[i] = pi;
    if (pbf) ((bf16x4*)pbf)[i] = (bf16x4){f2bf(pi[0]), f2bf(pi[1]), f2bf(pi[2]), f2bf(pi[3])};
  };
  // U vectors per thread per iteration: all 4 U 16-B loads issued before the first update (NTIN: the gradient and
  // parameter loads nontemporal too)
  const long long stride = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 gg[U], mm[U], vv[U], pp[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long j = i + u * stride;
      gg[u] = NTIN ? __builtin_nontemporal_load((const f32x4*)g + j) : ((const f32x4*)g)[j];
      mm[u] = __builtin_nontemporal_load((const f32x4*)m + j);
      vv[u] = __builtin_nontemporal_load((const f32x4*)v + j);
      pp[u] = NTIN ? __builtin_nontemporal_load((const f32x4*)p + j) : ((const f32x4*)p)[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) update(i + u * stride, gg[u], mm[u], vv[u], pp[u]);
  }
  for (; i < n4; i += stride)
    update(i, ((const f32x4*)g)[i], ((const f32x4*)m)[i], ((const f32x4*)v)[i], ((const f32x4*)p)[i]);
}

// In-place clip_grad_norm_ (language_model.py:120-122) for a micro-step that is not followed by an optimiser step
// (gradient accumulation): g *= min(1, max_norm / (norm + 1e-6)), norm from the svae_sumsq partials.
__global__ __launch_bounds__(256) void clip_scale_kernel(float* __restrict__ g, long long n, const float* __restrict__ part,
                                                         int nblk, float max_norm, float* __restrict__ norm_out) {
  __shared__ float red[4];
  __shared__ float s_coef;
  float s = 0.f;
  for (int i = threadIdx.x; i < nblk; i += 256) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float norm = sqrtf(red[0] + red[1] + red[2] + red[3]);
    s_coef = fminf(1.0f, max_norm / (norm + 1e-6f));
    if (blockIdx.x == 0 && norm_out) norm_out[0] = norm;
  }
  __syncthreads();
  const float coef = s_coef;
  if (coef == 1.0f) return;                  // block-uniform: nothing to scale
  const long long n4 = n / 4;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256)
    ((f32x4*)g)[i] = ((const f32x4*)g)[i] * coef;
}

inline int grid_for(long long work, int per_block, int cap = 4096) {
  long long g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace

SVAE_EXPORT int svae_embedding_fwd(const int32_t* ids, const void* table, float* out, void* out_bf, int32_t rows,
                                   int32_t D, svae_stream_t stream) {
  if (!ids || !table || !out || rows <= 0 || D % 4) return SVAE_EINVAL;
  hipLaunchKernelGGL(emb_fwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, ids, (const float*)table,
                     out, (bf16*)out_bf, rows, D, (float*)nullptr);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_embedding_fwd_dual(const int32_t* ids, const void* table, float* out, float* out2, int32_t rows,
                                        int32_t D, svae_stream_t stream) {
  if (!ids || !table || !out || !out2 || rows <= 0 || D % 4) return SVAE_EINVAL;
  hipLaunchKernelGGL(emb_fwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, ids, (const float*)table,
                     out, (bf16*)nullptr, rows, D, out2);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_embedding_bwd(const int32_t* ids, const float* dout, float* dtable, int32_t rows, int32_t D,
                                   svae_stream_t stream) {
  if (!ids || !dout || !dtable || rows <= 0 || D <= 0) return SVAE_EINVAL;
  hipLaunchKernelGGL(emb_bwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, ids, dout, dtable, rows, D);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_embedding_bwd_ce(const int32_t* ids, const float* dout, float* dtable, int32_t rows, int32_t D,
                                      int32_t seq, const void* hh, const float* q, svae_stream_t stream) {
  if (!ids || !dout || !dtable || !hh || !q || rows <= 0 || D <= 0 || seq <= 0 || rows % seq) return SVAE_EINVAL;
  hipLaunchKernelGGL(emb_bwd_ce_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, ids, dout, dtable, rows,
                     D, seq, (const bf16*)hh, q);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_ce_label_logit(const void* hh, int64_t ldh, const void* W, int64_t ldw, const float* bias,
                                    const int32_t* labels, int32_t rows, int32_t D, float* out, svae_stream_t stream) {
  if (!hh || !W || !labels || !out || rows <= 0 || D <= 0 || D % 8 || ldh % 8 || ldw % 8) return SVAE_EINVAL;
  if (((uintptr_t)hh | (uintptr_t)W) & 15) return SVAE_EINVAL;
  hipLaunchKernelGGL(ce_label_logit_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, (const bf16*)hh,
                     (long long)ldh, (const bf16*)W, (long long)ldw, bias, labels, rows, D, out);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_ce_prob_finalize(const float* part, int32_t ntile, const float* row_off, const int32_t* labels,
                                      int32_t rows, int32_t seq, int32_t nchunks, int32_t chunk_len, float* lse,
                                      float* row_loss, float* chunk_w, float* nll_out, float* red_ws,
                                      svae_stream_t stream) {
  return svae_ce_prob_finalize_fix(part, ntile, (float*)row_off, labels, rows, seq, nchunks, chunk_len, lse, row_loss,
                                   chunk_w, nll_out, red_ws, nullptr, 0, nullptr, 0, nullptr, nullptr, 0, 0, 0, nullptr,
                                   stream);
}

SVAE_EXPORT int svae_ce_prob_finalize_fix(const float* part, int32_t ntile, float* row_off, const int32_t* labels,
                                          int32_t rows, int32_t seq, int32_t nchunks, int32_t chunk_len, float* lse,
                                          float* row_loss, float* chunk_w, float* nll_out, float* red_ws,
                                          const void* hh, int64_t ldh, const void* W, int64_t ldw, const float* bias,
                                          void* P, int64_t ldp, int32_t V, int32_t D, int32_t* sat_ws,
                                          svae_stream_t stream) {
  if (!part || !row_off || !labels || !lse || !row_loss || !chunk_w || !nll_out || !red_ws) return SVAE_EINVAL;
  if (rows <= 0 || ntile <= 0 || seq <= 0 || rows % seq || nchunks <= 0 || nchunks > CE_MAX_CHUNKS ||
      chunk_len <= 0 || (long long)(nchunks - 1) * chunk_len >= seq)
    return SVAE_EINVAL;
  const bool fix = sat_ws != nullptr;
  if (fix && (!hh || !W || !P || V <= 0 || D <= 0 || D > 1024 || D % 8 || ldh % 8 || ldw % 8 ||
              (((uintptr_t)hh | (uintptr_t)W) & 15)))
    return SVAE_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (fix && hipMemsetAsync(sat_ws, 0, sizeof(int32_t), s) != hipSuccess) return SVAE_ELAUNCH;
  hipLaunchKernelGGL(ce_prob_rows_kernel, dim3((rows + 31) / 32), dim3(256), 0, s, part, ntile, row_off, labels, rows,
                     lse, row_loss, (int*)sat_ws);
  if (fix)
    hipLaunchKernelGGL(ce_prob_fixup_kernel, dim3(64), dim3(256), 0, s, (const int*)sat_ws, (const bf16*)hh,
                       (long long)ldh, (const bf16*)W, (long long)ldw, bias, (bf16*)P, (long long)ldp, V, D, row_off,
                       lse, row_loss);
  hipLaunchKernelGGL(ce_reduce_part_kernel, dim3(CE_RED_BLOCKS, nchunks), dim3(256), 0, s, row_loss, labels,
                     (const float*)nullptr, rows, seq, nchunks, chunk_len, red_ws);
  hipLaunchKernelGGL(ce_reduce_final_kernel, dim3(1), dim3(256), 0, s, red_ws, nchunks, chunk_w, nll_out);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_ce_prob_bwd_prep(const void* hh, int64_t ldh, const float* lse, const float* row_off,
                                      const float* chunk_w, const int32_t* labels, const float* gscale, int32_t rows,
                                      int32_t seq, int32_t nchunks, int32_t chunk_len, int32_t D, void* hh_out,
                                      float* r_out, float* q_out, float* dbias, svae_stream_t stream) {
  if (!hh || !lse || !row_off || !chunk_w || !labels || !gscale || !hh_out || !r_out || !q_out) return SVAE_EINVAL;
  if (rows <= 0 || seq <= 0 || nchunks <= 0 || chunk_len <= 0 || D <= 0 || D % 8 || ldh % 8) return SVAE_EINVAL;
  if (((uintptr_t)hh | (uintptr_t)hh_out) & 15) return SVAE_EINVAL;
  hipLaunchKernelGGL(ce_prob_bwd_prep_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, (const bf16*)hh,
                     (long long)ldh, lse, row_off, chunk_w, labels, gscale, rows, seq, nchunks, chunk_len, D,
                     (bf16*)hh_out, r_out, q_out, dbias);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_reparam_kl_fwd(const float* stats, const float* eps, uint64_t seed, const int64_t* ntok, float* z,
                                    void* z_bf, float* eps_out, float* raw_kl, float* kl_out, int32_t B, int32_t Z,
                                    svae_stream_t stream) {
  if (!stats || !ntok || !z || !raw_kl || !kl_out || B <= 0 || Z <= 0) return SVAE_EINVAL;
  hipLaunchKernelGGL(reparam_fwd_kernel, dim3(1), dim3(64 * REPARAM_WAVES), 0, (hipStream_t)stream, stats, eps, seed,
                     (const long long*)ntok, z, (bf16*)z_bf, eps_out, raw_kl, kl_out, B, Z);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_reparam_kl_bwd(const float* stats, const float* eps, const float* dz, const int64_t* ntok,
                                    const float* gkl, float* dstats, int32_t B, int32_t Z, svae_stream_t stream) {
  if (!stats || !eps || !ntok || !gkl || !dstats || B <= 0 || Z <= 0) return SVAE_EINVAL;
  hipLaunchKernelGGL(reparam_bwd_kernel, dim3((B * Z + 255) / 256), dim3(256), 0, (hipStream_t)stream, stats, eps, dz,
                     (const long long*)ntok, gkl, dstats, B, Z);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_ce_finalize(const float* part, int32_t ntile, const float* label_logit, const int32_t* labels,
                                 int32_t rows, int32_t seq, int32_t nchunks, int32_t chunk_len, float* lse,
                                 float* row_loss, float* chunk_w, float* nll_out, float* red_ws, svae_stream_t stream) {
  if (!part || !label_logit || !labels || !lse || !row_loss || !chunk_w || !nll_out || !red_ws) return SVAE_EINVAL;
  if (rows <= 0 || ntile <= 0 || seq <= 0 || rows % seq || nchunks <= 0 || nchunks > CE_MAX_CHUNKS ||
      chunk_len <= 0 || (long long)(nchunks - 1) * chunk_len >= seq)
    return SVAE_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(ce_rows_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, part, ntile, label_logit, labels, rows, lse,
                     row_loss);
  hipLaunchKernelGGL(ce_reduce_part_kernel, dim3(CE_RED_BLOCKS, nchunks), dim3(256), 0, s, row_loss, labels,
                     (const float*)nullptr, rows, seq, nchunks, chunk_len, red_ws);
  hipLaunchKernelGGL(ce_reduce_final_kernel, dim3(1), dim3(256), 0, s, red_ws, nchunks, chunk_w, nll_out);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_ce_weighted_nll(const float* row_loss, const int32_t* labels, const float* tok_w, int32_t rows,
                                     int32_t seq, int32_t nchunks, int32_t chunk_len, float* out, float* red_ws,
                                     svae_stream_t stream) {
  if (!row_loss || !labels || !tok_w || !out || !red_ws) return SVAE_EINVAL;
  if (rows <= 0 || seq <= 0 || rows % seq || nchunks <= 0 || nchunks > CE_MAX_CHUNKS || chunk_len <= 0 ||
      (long long)(nchunks - 1) * chunk_len >= seq)
    return SVAE_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(ce_reduce_part_kernel, dim3(CE_RED_BLOCKS, nchunks), dim3(256), 0, s, row_loss, labels, tok_w, rows,
                     seq, nchunks, chunk_len, red_ws);
  hipLaunchKernelGGL(ce_reduce_final_kernel, dim3(1), dim3(256), 0, s, red_ws, nchunks, (float*)nullptr, out);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int32_t svae_ce_red_ws_elems(int32_t nchunks) { return nchunks * CE_RED_BLOCKS * 2; }

SVAE_EXPORT int svae_mutual_info(const float* stats, const float* eps, uint64_t seed, const float* kl, int32_t B,
                                 int32_t Z, int32_t S, float* ws, float* out, svae_stream_t stream) {
  if (!stats || !kl || !ws || !out || B <= 0 || Z <= 0 || S <= 0 || Z > 4096) return SVAE_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(mi_marginal_kernel, dim3(S * B), dim3(256), (size_t)Z * sizeof(float), s, stats, eps,
                     (unsigned long long)seed, B, Z, ws);
  hipLaunchKernelGGL(mi_final_kernel, dim3(1), dim3(256), 0, s, ws, S * B, Z, kl, out);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_ce_seq_logprob(const float* part, int32_t ntile, const float* label_logit, const int32_t* labels,
                                    int32_t rows, int32_t seq, float* out, svae_stream_t stream) {
  if (!part || !label_logit || !labels || !out || rows <= 0 || ntile <= 0 || seq <= 0 || rows % seq) return SVAE_EINVAL;
  hipLaunchKernelGGL(ce_seq_logprob_kernel, dim3(rows / seq), dim3(256), 0, (hipStream_t)stream, part, ntile,
                     label_logit, labels, seq, out);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_ce_grad(void* logits, int64_t ld, const float* lse, const float* chunk_w, const int32_t* labels,
                             const float* gscale, float* dbias, int32_t rows, int32_t V, int32_t seq, int32_t nchunks,
                             int32_t chunk_len, svae_stream_t stream) {
  if (!logits || !lse || !chunk_w || !labels || !gscale || rows <= 0 || V % 8 || ld % 8) return SVAE_EINVAL;
  const int strips = (V + 2047) / 2048;
  int rpb = 256;
  while (rpb > 16 && (long long)strips * ((rows + rpb - 1) / rpb) < 1024) rpb /= 2;
  dim3 grid(strips, (rows + rpb - 1) / rpb);
  hipLaunchKernelGGL(ce_grad_kernel, grid, dim3(256), 0, (hipStream_t)stream, (bf16*)logits, ld, lse, chunk_w, labels,
                     gscale, dbias, rows, V, seq, nchunks, chunk_len, rpb);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_dropout_bwd_cast(const float* g, void* out, float p, uint64_t seed, int64_t n, int32_t cols,
                                      int64_t ld_in, svae_stream_t stream) {
  if (!g || !out || n <= 0 || cols <= 0 || cols % 4 || n % cols || ld_in % 4) return SVAE_EINVAL;
  hipLaunchKernelGGL(dropout_bwd_cast_kernel, dim3(grid_for(n, 1024)), dim3(256), 0, (hipStream_t)stream, g, (bf16*)out,
                     p, seed, n, cols, ld_in);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_gelu_bwd(const float* dx, const void* gp, void* out, int64_t n, svae_stream_t stream) {
  if (!dx || !gp || !out || n <= 0) return SVAE_EINVAL;
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, dx, (const bf16*)gp,
                     (bf16*)out, n);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_prep_tokens(const int64_t* ids, const void* pad, int32_t pad_mode, int32_t B, int32_t L,
                                 int32_t* ids32, int32_t* labels, void* padm, const int64_t* ntok, int64_t* ntok_out,
                                 svae_stream_t stream) {
  if (!ids || !ids32 || !labels || B <= 0 || L <= 0 || pad_mode < 0 || pad_mode > 2) return SVAE_EINVAL;
  if ((pad_mode && !padm) || (pad_mode == 2 && !pad) || (!ntok != !ntok_out)) return SVAE_EINVAL;
  const long long rows = (long long)B * L;
  if (rows > 0x7FFFFFFFLL - 256) return SVAE_EINVAL;
  const long long work = rows > B ? rows : B;
  hipLaunchKernelGGL(prep_tokens_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ids,
                     (const unsigned char*)pad, pad_mode, (int)rows, L, ids32, labels, (unsigned char*)padm, ntok,
                     ntok_out, B);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_step_scalars(const float* nll, const float* kl, const float* gloss, float kl_weight, float* loss,
                                  float* gs, svae_stream_t stream) {
  if ((!loss && !gs) || (loss && (!nll || !kl)) || (gs && !gloss)) return SVAE_EINVAL;
  hipLaunchKernelGGL(step_scalars_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, nll, kl, gloss, kl_weight, loss, gs);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_cast_bf16(const float* in, void* out, int64_t n, svae_stream_t stream) {
  if (!in || !out || n <= 0) return SVAE_EINVAL;
  hipLaunchKernelGGL(cast_kernel, dim3(grid_for(n, 1024)), dim3(256), 0, (hipStream_t)stream, in, (bf16*)out, n);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_transpose_blocks(const void* src, void* dst, const int64_t* table, int32_t nblocks,
                                      int32_t total_tiles, svae_stream_t stream) {
  if (!src || !dst || !table || nblocks <= 0 || total_tiles <= 0) return SVAE_EINVAL;
  hipLaunchKernelGGL(transpose_blocks_kernel, dim3(total_tiles), dim3(256), 0, (hipStream_t)stream, (const bf16*)src,
                     (bf16*)dst, (const long long*)table, nblocks);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

// z_projections[i] backward (svae.h): 1024-thread blocks. Blocks [0, nbw) own 16 rows m of dW (one wave per row,
// lanes over n; the wave's lane-strided sum over b gives db[m]); blocks [nbw, nbw + B) own one row b of dz (16 waves
// over slices of m, combined in LDS in a fixed order). Every output has one writer: no atomics. Operands are staged
// through LDS in 64-row chunks. (256-thread blocks: 10.7 us per launch at C2, the dz row's 128 dependent steps.)
__global__ __launch_bounds__(1024) void zproj_bwd_kernel(const float* __restrict__ g, const bf16* __restrict__ z,
                                                         const bf16* __restrict__ W, float* __restrict__ dW,
                                                         float* __restrict__ db, float* __restrict__ dz, int B, int d,
                                                         int Z, int nbw) {
  __shared__ float zs[64][65];
  __shared__ float gs[1024];
  __shared__ float red[16][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if ((int)blockIdx.x < nbw) {
    const int m0 = blockIdx.x * 16, m = m0 + wave;
    for (int n0 = 0; n0 < Z; n0 += 64) {
      const int n = n0 + lane;
      float acc = 0.f;
      for (int b0 = 0; b0 < B; b0 += 64) {
        const int nb = min(64, B - b0);
        for (int e = tid; e < 64 * 64; e += 1024) {
          const int i = e >> 6, j = e & 63;
          zs[i][j] = (i < nb && n0 + j < Z) ? (float)z[(long long)(b0 + i) * Z + n0 + j] : 0.f;
        }
        {
          const int i = tid >> 4, w = tid & 15;
          gs[tid] = (i < nb && m0 + w < d) ? g[(long long)(b0 + i) * d + m0 + w] : 0.f;
        }
        __syncthreads();
#pragma unroll 16
        for (int i = 0; i < 64; ++i) acc = fmaf(gs[16 * i + wave], zs[i][lane], acc);
        __syncthreads();
      }
      if (m < d && n < Z) dW[(long long)m * Z + n] += acc;
    }
    if (m < d) {
      float s = 0.f;
      for (int b = lane; b < B; b += 64) s += g[(long long)b * d + m];
      s = wave_sum(s);
      if (lane == 0) db[m] += s;
    }
  } else {
    const int b = blockIdx.x - nbw;
    const float* gb = g + (long long)b * d;
    for (int n0 = 0; n0 < Z; n0 += 64) {
      const int n = n0 + lane;
      float acc = 0.f;
      for (int c0 = 0; c0 < d; c0 += 1024) {   // the row's g in LDS, 1024 columns at a time
        const int nc = min(1024, d - c0);
        if (tid < nc) gs[tid] = gb[c0 + tid];
        __syncthreads();
        if (n < Z) {
#pragma unroll 8
          for (int mm = wave; mm < nc; mm += 16) acc = fmaf(gs[mm], (float)W[(long long)(c0 + mm) * Z + n], acc);
        }
        __syncthreads();
      }
      red[wave][lane] = acc;
      __syncthreads();
      if (wave == 0 && n < Z) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < 16; ++w) t += red[w][lane];
        dz[(long long)b * Z + n] += t;
      }
      __syncthreads();
    }
  }
}

// The backward of n z projections in one launch (svae_zproj_bwd_multi): blocks [0, n * nbw) take the dW / db part of
// segment blk / nbw; the B blocks after them sum dz[b] += g_i[b] W_i over the segments in list order, each segment's
// partial reduced exactly as zproj_bwd_kernel reduces it and added in the same order as n separate launches would.
struct ZprojSegs {
  svae_zproj_seg s[SVAE_ZPROJ_MAX];
};

__global__ __launch_bounds__(1024) void zproj_bwd_multi_kernel(ZprojSegs segs, int nseg, const bf16* __restrict__ z,
                                                               float* __restrict__ dz, int B, int d, int Z, int nbw) {
  __shared__ float gs[1024];
  __shared__ float red[16][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int blk = blockIdx.x;
  if (blk < nseg * nbw) {
    __shared__ float zs[64][65];
    const svae_zproj_seg& sg = segs.s[blk / nbw];
    const float* g = sg.g;
    float* dW = sg.dW;
    const int m0 = (blk % nbw) * 16, m = m0 + wave;
    for (int n0 = 0; n0 < Z; n0 += 64) {
      const int n = n0 + lane;
      float acc = 0.f;
      for (int b0 = 0; b0 < B; b0 += 64) {
        const int nb = min(64, B - b0);
        for (int e = tid; e < 64 * 64; e += 1024) {
          const int i = e >> 6, j = e & 63;
          zs[i][j] = (i < nb && n0 + j < Z) ? (float)z[(long long)(b0 + i) * Z + n0 + j] : 0.f;
        }
        {
          const int i = tid >> 4, w = tid & 15;
          gs[tid] = (i < nb && m0 + w < d) ? g[(long long)(b0 + i) * d + m0 + w] : 0.f;
        }
        __syncthreads();
#pragma unroll 16
        for (int i = 0; i < 64; ++i) acc = fmaf(gs[16 * i + wave], zs[i][lane], acc);
        __syncthreads();
      }
      if (m < d && n < Z) dW[(long long)m * Z + n] += acc;
    }
    if (m < d) {
      float s = 0.f;
      for (int b = lane; b < B; b += 64) s += g[(long long)b * d + m];
      s = wave_sum(s);
      if (lane == 0) sg.db[m] += s;
    }
    return;
  }
  const int b = blk - nseg * nbw;
  for (int n0 = 0; n0 < Z; n0 += 64) {
    const int n = n0 + lane;
    float out = (wave == 0 && n < Z) ? dz[(long long)b * Z + n] : 0.f;
    for (int si = 0; si < nseg; ++si) {
      const float* gb = segs.s[si].g + (long long)b * d;
      const bf16* W = (const bf16*)segs.s[si].W;
      float acc = 0.f;
      for (int c0 = 0; c0 < d; c0 += 1024) {
        const int nc = min(1024, d - c0);
        if (tid < nc) gs[tid] = gb[c0 + tid];
        __syncthreads();
        if (n < Z) {
#pragma unroll 8
          for (int mm = wave; mm < nc; mm += 16) acc = fmaf(gs[mm], (float)W[(long long)(c0 + mm) * Z + n], acc);
        }
        __syncthreads();
      }
      red[wave][lane] = acc;
      __syncthreads();
      if (wave == 0 && n < Z) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < 16; ++w) t += red[w][lane];
        out += t;
      }
      __syncthreads();
    }
    if (wave == 0 && n < Z) dz[(long long)b * Z + n] = out;
  }
}

// Forward of n z projections (transformer_vae.py:89: z_projections[i](z)) in one launch: out_i [B][d] f32 =
// z W_i^T + b_i, z bf16 [B][Z], W_i bf16 [d][Z]; one block per (segment, sequence), z's row in LDS, 4 outputs per thread
// per pass (f32 FMAs over k in order).
struct ZfwdSegs {
  svae_zproj_fwd_seg s[SVAE_ZPROJ_MAX];
};

__global__ __launch_bounds__(256) void zproj_fwd_multi_kernel(ZfwdSegs segs, const bf16* __restrict__ z, int B, int d,
                                                              int Z) {
  __shared__ float zr[1024];
  const int si = blockIdx.x / B, b = blockIdx.x - si * B;
  const svae_zproj_fwd_seg& sg = segs.s[si];
  for (int k = threadIdx.x; k < Z; k += 256) zr[k] = (float)z[(long long)b * Z + k];
  __syncthreads();
  const bf16* W = (const bf16*)sg.W;
  for (int m = threadIdx.x; m < d; m += 256) {
    const bf16* wr = W + (long long)m * Z;
    float acc = 0.f;
    for (int k = 0; k < Z; ++k) acc = fmaf(zr[k], (float)wr[k], acc);
    sg.out[(long long)b * d + m] = acc + sg.bias[m];
  }
}

SVAE_EXPORT int svae_zproj_fwd_multi(const svae_zproj_fwd_seg* segs, int32_t n, const void* z, int32_t B, int32_t d,
                                     int32_t Z, svae_stream_t stream) {
  if (!segs || n <= 0 || n > SVAE_ZPROJ_MAX || !z || B <= 0 || d <= 0 || Z <= 0 || Z > 1024) return SVAE_EINVAL;
  ZfwdSegs a;
  for (int i = 0; i < n; ++i) {
    if (!segs[i].W || !segs[i].bias || !segs[i].out) return SVAE_EINVAL;
    a.s[i] = segs[i];
  }
  hipLaunchKernelGGL(zproj_fwd_multi_kernel, dim3((unsigned)(n * B)), dim3(256), 0, (hipStream_t)stream, a,
                     (const bf16*)z, B, d, Z);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_zproj_bwd_multi(const svae_zproj_seg* segs, int32_t n, const void* z, float* dz, int32_t B,
                                     int32_t d, int32_t Z, svae_stream_t stream) {
  if (!segs || n <= 0 || n > SVAE_ZPROJ_MAX || !z || !dz || B <= 0 || d <= 0 || Z <= 0) return SVAE_EINVAL;
  ZprojSegs a;
  for (int i = 0; i < n; ++i) {
    if (!segs[i].g || !segs[i].W || !segs[i].dW || !segs[i].db) return SVAE_EINVAL;
    a.s[i] = segs[i];
  }
  const int nbw = (d + 15) / 16;
  hipLaunchKernelGGL(zproj_bwd_multi_kernel, dim3(n * nbw + B), dim3(1024), 0, (hipStream_t)stream, a, (int)n,
                     (const bf16*)z, dz, B, d, Z, nbw);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_zproj_bwd(const float* g, const void* z, const void* W, float* dW, float* db, float* dz,
                               int32_t B, int32_t d, int32_t Z, svae_stream_t stream) {
  if (!g || !z || !W || !dW || !db || !dz || B <= 0 || d <= 0 || Z <= 0) return SVAE_EINVAL;
  const int nbw = (d + 15) / 16;
  hipLaunchKernelGGL(zproj_bwd_kernel, dim3(nbw + B), dim3(1024), 0, (hipStream_t)stream, g, (const bf16*)z,
                     (const bf16*)W, dW, db, dz, B, d, Z, nbw);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_extract_rows(float* x, int64_t ld, int32_t rows, int32_t mod, int32_t D, float* out,
                                  svae_stream_t stream) {
  if (!x || !out || rows <= 0 || mod <= 0 || rows % mod || D <= 0) return SVAE_EINVAL;
  const int nout = rows / mod;
  hipLaunchKernelGGL(extract_rows_kernel, dim3((nout * D + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, ld, nout,
                     mod, D, out);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_dq_finalize(const float* dq, void* out, int64_t ldo, int32_t rows, int32_t D, const float* rot_tab,
                                 int32_t seq, svae_stream_t stream) {
  if (!dq || !out || rows <= 0 || D <= 0 || D % 2 || (rot_tab && seq <= 0)) return SVAE_EINVAL;
  const long long work = (long long)rows * (D / 2);
  hipLaunchKernelGGL(dq_finalize_kernel, dim3(grid_for(work, 256)), dim3(256), 0, (hipStream_t)stream, dq, (bf16*)out,
                     ldo, rows, D, rot_tab, seq);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_sumsq(const float* g, int64_t n, float* part, int32_t nblk, svae_stream_t stream) {
  if (!g || !part || n <= 0 || nblk <= 0 || nblk > 4096) return SVAE_EINVAL;
  hipLaunchKernelGGL(sumsq_kernel, dim3(nblk), dim3(256), 0, (hipStream_t)stream, g, n, part);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_radam(float* p, void* pbf, const float* g, float* m, float* v, int64_t n, const float* part,
                           int32_t nblk, const float* scal, float* norm_out, svae_stream_t stream) {
  if (!p || !g || !m || !v || !part || !scal || n <= 0 || n % 4 || nblk <= 0) return SVAE_EINVAL;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15 || ((uintptr_t)pbf & 7)) return SVAE_EINVAL;
  // the gradient and parameter loads nontemporal as well (C2's 45 M parameters 263 -> 223-227 us; at C4's 162 M all
  // variants run 4.6-5.0 TB/s: profiles/r05ra_radam_variants.log). SVAE_RADAM_U / _NT / _GRID: A/B variants
  static const int u_env = [] { const char* e = getenv("SVAE_RADAM_U"); return e ? atoi(e) : 2; }();
  static const int nt_env = [] { const char* e = getenv("SVAE_RADAM_NT"); return e ? atoi(e) : 1; }();
  static const int grid_env = [] { const char* e = getenv("SVAE_RADAM_GRID"); return e ? atoi(e) : 2048; }();
  const dim3 grid(grid_for(n / 4, 256, grid_env)), blk(256);
  hipStream_t s = (hipStream_t)stream;
  if (u_env == 4 && nt_env) hipLaunchKernelGGL((radam_kernel<4, true>), grid, blk, 0, s, p, (bf16*)pbf, g, m, v, n, part, nblk, scal, norm_out);
  else if (u_env == 4) hipLaunchKernelGGL((radam_kernel<4, false>), grid, blk, 0, s, p, (bf16*)pbf, g, m, v, n, part, nblk, scal, norm_out);
  else if (nt_env) hipLaunchKernelGGL((radam_kernel<2, true>), grid, blk, 0, s, p, (bf16*)pbf, g, m, v, n, part, nblk, scal, norm_out);
  else hipLaunchKernelGGL((radam_kernel<2, false>), grid, blk, 0, s, p, (bf16*)pbf, g, m, v, n, part, nblk, scal, norm_out);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_clip_grad(float* g, int64_t n, const float* part, int32_t nblk, float max_norm, float* norm_out,
                               svae_stream_t stream) {
  if (!g || !part || n <= 0 || n % 4 || nblk <= 0 || ((uintptr_t)g & 15)) return SVAE_EINVAL;
  hipLaunchKernelGGL(clip_scale_kernel, dim3(grid_for(n / 4, 256, 2048)), dim3(256), 0, (hipStream_t)stream, g, n, part,
                     nblk, max_norm, norm_out);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT const char* svae_version(void) { return "libsvae 0.1 gfx950"; }
