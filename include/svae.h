/*
 * svae.h — C ABI of libsvae.so, the MI355X (gfx950) kernels behind the sparse-vae TransformerVAE
 * training step.
 *
 * The reference (norabelrose/sparse-vae) has NO native layer: its hot path is PyTorch ATen ops called
 * from nn.Modules. Each entry point below replaces the ATen op sequence of one
 * reference call site (cited per function); the Python host package (sparse-vae_amd/sparse_vae) keeps
 * the reference's nn.Module / LightningModule surface and calls these through ctypes.
 *
 * Conventions (all entry points):
 *   - device pointers are plain addresses of memory owned by the caller (PyTorch's caching allocator);
 *     the library never allocates, frees or synchronises;
 *   - element types: bf16 = 16-bit bfloat16 storage, f32 = IEEE float;
 *   - `stream` is a hipStream_t; work is enqueued asynchronously on it;
 *   - return 0 on success, SVAE_EINVAL (1) on a bad argument (nothing launched), SVAE_ELAUNCH (2) if
 *     the launch failed. The Python layer raises RuntimeError on any non-zero status.
 */
#ifndef SVAE_H
#define SVAE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef void* svae_stream_t; /* hipStream_t */

/* ---- GEMM: C[M,N] = epi(alpha * A[M,K] . B[K,N]) ------------------------------------------------
 * Replaces nn.Linear forward (addmm) and its autograd backward (mm for dX and dW) at every Linear of
 * the path: attention.py:33-38,60,67,103; transformer_layer.py:17-21; transformer_language_model.py:55-63;
 * conditional_gaussian.py:18; transformer_vae.py:37-40,89.
 * a_t = 0: A stored [M][K] (lda >= K); a_t = 1: A stored [K][M] (lda >= M).
 * b_t = 0: B stored [N][K] (nn.Linear weight layout); b_t = 1: B stored [K][N].
 * Requirements: K % 8 == 0 unless a_t && b_t; for a_t: M % 8 == 0; for b_t: N % 8 == 0; lda, ldb % 8 == 0;
 * A, B 16-byte aligned; N, ldc (and ldr, ldaux) % 4 == 0 and C 8-byte aligned (vectorised epilogue). */
enum svae_epi {
  SVAE_EPI_BF16 = 0,          /* C bf16 = alpha*acc + bias                                            */
  SVAE_EPI_F32 = 1,           /* C f32  = alpha*acc + bias (+ resid); with aux != NULL (batch 1, ldaux %
                                 8 == 0) also aux bf16 = bf16(keep(seed, m*N+n) * C / (1 - p)) -- what
                                 svae_dropout_bwd_cast makes of C (drop_p 0: bf16(C))                  */
  SVAE_EPI_F32_ACC = 2,       /* C f32 += alpha*acc                                                   */
  SVAE_EPI_F32_ATOMIC = 3,    /* atomicAdd(C f32, alpha*acc)   (split-K / shared destinations); with
                                 splits > 1 and aux != NULL: each split stores its partial tile into the
                                 f32 workspace aux [splits][M][N] and a reduce pass adds them into C     */
  SVAE_EPI_GELU = 4,          /* C bf16 = gelu(acc + bias);  aux bf16 = gelu'(acc + bias)              */
  SVAE_EPI_GELU_BWD = 5,      /* C bf16 = acc * aux  (aux = the gelu' saved by SVAE_EPI_GELU)          */
  SVAE_EPI_DROPOUT_RESID = 6, /* C f32 = resid + keep(seed, m*N+n) * acc / (1 - p); with aux != NULL
                                 (batch 1, ldaux % 8 == 0) also aux bf16 = bf16(C)                    */
  SVAE_EPI_ROTARY_BF16 = 7,   /* C bf16 = rotary(acc + bias) on cols < rot_cols (attention.py:194-208) */
  SVAE_EPI_CE_STATS = 8,      /* C bf16 = acc + bias; per (row, 128-col tile) online (max, sumexp) to
                                 aux f32 [M][ceil(N/128)][2]; label logit (f32) to resid-as-out [M]   */
  SVAE_EPI_CE_PROB = 9,       /* vocab head, training: C bf16 = exp(acc + bias - row_a[m]) for rows with
                                 labels[m] != 0, else 0 (exponent clamped at 2^127); aux f32
                                 [ceil(N/128)][M] (tile-major) = per (128-col tile, row) sums of them  */
  SVAE_EPI_ROWSCALE_GATHER = 10 /* C bf16 = alpha * row_a[m] * acc - row_b[m] * gather[labels[m]][n]
                                 (the gather term is skipped where labels[m] == 0)                    */
};

typedef struct svae_gemm_desc {
  const void* A;
  const void* B;
  int64_t lda, ldb, batch_stride_a, batch_stride_b;
  int32_t M, N, K;
  int32_t batch, splits;
  int32_t a_t, b_t;
  int32_t epi;
  void* C;
  int64_t ldc, batch_stride_c;
  const float* bias;        /* [N] f32 or NULL */
  const float* resid;       /* f32 [M][ldr] or NULL (DROPOUT_RESID / F32); may alias C */
  int64_t ldr;
  void* aux;                /* see svae_epi */
  int64_t ldaux;
  float alpha;
  float drop_p;
  uint64_t seed;
  const float* rot_tab;     /* [rot_seq][rot_d/2] x (cos, sin) f32 */
  int32_t rot_cols, rot_d, rot_seq;
  const int32_t* labels;    /* CE_STATS: [M] target column per row (0 = ignored) */
  float* label_logit;       /* CE_STATS: [M] f32 out */
  float* a_rowsum;          /* a_t only, optional: a_rowsum[m] += sum_k A[m][k] (bias grad of a dW GEMM) */
  /* optional with a_rowsum (a_t && b_t; splits 1 with F32_ACC, or split-K slab mode: F32_ATOMIC with aux):  */
  /* a_rowsum[m] += sum_k A[m][k] * k_weight[k]                                                            */
  const float* k_weight;
  const float* row_a;       /* CE_PROB / ROWSCALE_GATHER: [M] f32 (see svae_epi)                        */
  const float* row_b;       /* ROWSCALE_GATHER: [M] f32                                                  */
  const void* gather;       /* ROWSCALE_GATHER: bf16 rows [*][ldg], row labels[m] gathered; 16-B aligned */
  int64_t ldg;
  /* optional with SVAE_EPI_BF16 (the attention output projection's dO GEMM under autograd, attention.py:51-105):
   * also write the attention backward's row constants delta[(b * (N / delta_hd) + h) * delta_seq + q] = sum over
   * the head's delta_hd columns of bf16(C)[m][h * delta_hd + c] * delta_o32[m * ld_o32 + h * delta_hd + c], m = b *
   * delta_seq + q (delta_o32: the forward's f32 copy of O). delta is overwritten; svae_attn_bwd with delta_ready = 1
   * then skips its own delta pass. splits 1, batch 1, a_t 0; N % delta_hd == 0, delta_hd % 16 == 0, M % delta_seq == 0. */
  float* delta;
  const float* delta_o32;
  int64_t ld_o32;
  int32_t delta_hd, delta_seq;
} svae_gemm_desc;

int svae_gemm(const svae_gemm_desc* d, svae_stream_t stream);

/* Two weight-gradient GEMMs in one launch (engine.layer_bwd pairs the two dW GEMMs of the FFN, and the output
 * projection's with the QKV / K-V projection's: the nn.Linear weight gradients of transformer_layer.py:56-61 and
 * attention.py:51-105 under loss.backward()). Each desc as for svae_gemm with a_t = b_t = 1, epi
 * SVAE_EPI_F32_ATOMIC, splits >= 2 and a slab workspace in aux (aux[split][M][N] f32, then C += the sum of the
 * splits); the results equal two svae_gemm calls with the same descs. */
int svae_gemm_pair(const svae_gemm_desc* d0, const svae_gemm_desc* d1, svae_stream_t stream);

/* ---- LayerNorm ---------------------------------------------------------------------------------
 * nn.LayerNorm(d, eps=1e-5) forward/backward: transformer_layer.py:23-24,39-40,47,52,56;
 * transformer_language_model.py:59. x_dtype: 0 = f32 input, 1 = bf16 input. y is bf16.
 * Backward: dx = dres + LN'(dy) (dres may be NULL), written f32 to dx and (optionally) bf16 to dx_bf;
 * per-block partial (dw, db) sums go to part[nblk][2][D] (reduce with svae_colsum). Rows with
 * (row % zero_mod == 0) get dx = 0 when zero_mod > 0 (position-0 overwrite, transformer_vae.py:89-90). */
/* Residual add + dropout + LayerNorm forward (transformer_layer.py:49-50, :58-61 and the following LayerNorm, :47 / :56),
 * one pass: v = x[r] + dropout(y[r]) (x f32 [rows][D] or NULL; y bf16 [rows][ldy] -- the projection's output -- or
 * NULL; y_dtype 0 = f32, 1 = bf16; dropout with the counter RNG of SVAE_EPI_DROPOUT_RESID: seed, index (r * D + c) / 4),
 * or v = zrows[r / zmod]
 * where zrows != NULL and r % zmod == 0 (the z splice, transformer_vae.py:89-90); xo f32 = v (may be NULL);
 * h bf16 = LayerNorm(v) * w + b with mean / rstd, or h = bf16(v) when w == b == NULL. D % 8 == 0, D <= 1024. */
int svae_resid_ln_fwd(const float* x, const void* y, int32_t y_dtype, int64_t ldy, float drop_p, uint64_t seed,
                      const float* zrows, int32_t zmod, const float* w, const float* b, float* xo, void* h, float* mean,
                      float* rstd, int32_t rows, int32_t D, svae_stream_t stream);
int svae_layernorm_fwd(const void* x, int32_t x_dtype, const float* w, const float* b, void* y,
                       float* mean, float* rstd, int32_t rows, int32_t D, svae_stream_t stream);
int svae_layernorm_bwd(const void* dy, const void* x, int32_t x_dtype, const float* w, const float* mean,
                       const float* rstd, const float* dres, float* dx, void* dx_bf, float* part,
                       int32_t nblk, int32_t rows, int32_t D, int32_t zero_mod, svae_stream_t stream);
/* svae_layernorm_bwd for the last LayerNorm of a decoder layer's backward, with the two passes that followed it
 * fused in: (1) the bf16 copy dx_bf carries the NEXT layer's dropout backward (replaces svae_dropout_bwd_cast of
 * dx): dx_bf = bf16(keep(bf_seed, (row*D + c)/4) * dx / (1 - bf_drop_p)), the mask of the forward's
 * SVAE_EPI_DROPOUT_RESID epilogue with the same seed (transformer_layer.py:61, nn.Dropout), and dx_bf = 0 on rows
 * with row % bf_zero_mod == 0 (bf_zero_mod > 0); bf_drop_p in [0, 1). (2) with zero_mod > 0, the rows it zeroes in
 * dx are first written to zrow[row / zero_mod] (f32) and zrow_bf (bf16), either may be NULL: the gradient of the
 * position-0 z splice (transformer_vae.py:89-90; replaces svae_extract_rows + svae_cast_bf16). */
int svae_layernorm_bwd_drop(const void* dy, const void* x, int32_t x_dtype, const float* w, const float* mean,
                            const float* rstd, const float* dres, float* dx, void* dx_bf, float* part, int32_t nblk,
                            int32_t rows, int32_t D, int32_t zero_mod, float bf_drop_p, uint64_t bf_seed,
                            int32_t bf_zero_mod, float* zrow, void* zrow_bf, svae_stream_t stream);
/* svae_layernorm_bwd of the vocabulary head's LayerNorm (transformer_vae.py output_layer[2]) fused with the GELU
 * backward of the linear before it (output_layer[0..1]): out_bf = bf16(LN'(dy) * gp), gp the bf16 GELU' the forward's
 * SVAE_EPI_GELU epilogue saved; no f32 dx is written (replaces svae_layernorm_bwd + svae_gelu_bwd). part as above. */
int svae_layernorm_bwd_gelu(const void* dy, const void* x, int32_t x_dtype, const float* w, const float* mean,
                            const float* rstd, const void* gp, void* out_bf, float* part, int32_t nblk, int32_t rows,
                            int32_t D, svae_stream_t stream);
/* svae_layernorm_fwd (f32 x, D % 8 == 0, 16-B aligned x / zrows) with the z splice of transformer_vae.py:89-90: rows
 * r % zmod == 0 are taken from zrows[r / zmod] (f32 [rows / zmod][D]) and also written into x (the residual stream). */
int svae_layernorm_fwd_z(float* x, const float* zrows, int32_t zmod, const float* w, const float* b, void* y,
                         float* mean, float* rstd, int32_t rows, int32_t D, svae_stream_t stream);
int svae_layernorm_nblk(int32_t rows);
/* n <= SVAE_LN_MULTI_MAX LayerNorms of ONE input with their own affines: the encoder middle layers'
 * context_layer_norm(context) over the same x_emb (transformer_layer.py:52, one per middle layer, perceiver.py:43-46).
 * svae_layernorm_fwd_multi: one pass over f32 x writes y[j] = bf16(LN(x) * w[j] + b[j]) (bit-identical to n
 * svae_layernorm_fwd calls) and the shared mean / rstd. svae_layernorm_bwd_multi: the n backwards in one pass,
 * dx = dres + sum_j LN'_j(dy[j]) (dres may alias dx), the affine-gradient partials of LayerNorm j into part[j]
 * ([nblk][2][D] each, as svae_layernorm_bwd's part). f32 x, D % 4 == 0, D <= 1024. */
#define SVAE_LN_MULTI_MAX 4
int svae_layernorm_fwd_multi(const float* x, const float* const* w, const float* const* b, void* const* y, int32_t n,
                             float* mean, float* rstd, int32_t rows, int32_t D, svae_stream_t stream);
int svae_layernorm_bwd_multi(const void* const* dy, const float* x, const float* const* w, const float* mean,
                             const float* rstd, const float* dres, float* dx, float* const* part, int32_t nblk,
                             int32_t n, int32_t rows, int32_t D, svae_stream_t stream);

/* ---- column sums: out[j] (+)= sum_i in[i*ld + j] (bias grads, LN affine grads, batch sums) ----------
 * in_dtype 0 = f32, 1 = bf16. accumulate: 0 = overwrite, 1 = add into out. */
int svae_colsum(const void* in, int32_t in_dtype, int32_t rows, int32_t cols, int64_t ld, float* out,
                int32_t accumulate, svae_stream_t stream);

/* Up to SVAE_COLSUM_MAX f32 column sums in one launch, each added into its own out (the LayerNorm-affine gradients
 * of one layer's LayerNorm backwards). in / out 16-B aligned, cols and ld multiples of 4. */
#define SVAE_COLSUM_MAX 8
typedef struct svae_colsum_seg {
  const float* in;
  float* out;
  int64_t ld;
  int32_t rows, cols;
} svae_colsum_seg;
int svae_colsum_multi(const svae_colsum_seg* segs, int32_t n, svae_stream_t stream);

/* ---- Flash attention (dense path of Attention.forward, attention.py:51-105) ------------------------
 * q/k/v/o: bf16 rows of H*hd (token-major, head-interleaved, exactly the nn.Linear output layout),
 * row strides sq/sk/sv/so elements, batch strides bq/bk/bv/bo elements (bq = 0 for learned queries).
 * key_pad: uint8 [B][Lk] (1 = masked, padded_tensor.py:16) or NULL. causal: mask key > query
 * (attention.py:85-95). lse: f32 [B][H][Lq]. scale = hd^-0.5 (attention.py:83). */
typedef struct svae_attn_desc {
  const void* q; const void* k; const void* v; void* o;
  int64_t sq, sk, sv, so, bq, bk, bv, bo;
  const uint8_t* key_pad;
  float* lse;
  int32_t B, H, Lq, Lk, hd, causal;
  float scale;
  /* backward only */
  const void* dout; int64_t sdo, bdo;
  float* delta;             /* [B][H][Lq] f32 workspace */
  float* dq;                /* f32 [B][Lq][H*hd] output (written), batch stride bdq; used when dq_bf is NULL */
  int64_t bdq;
  void* dk; void* dv;       /* bf16 outputs, row stride sdk/sdv, batch stride bdk/bdv */
  int64_t sdk, sdv, bdk, bdv;
  const float* rot_tab;     /* inverse rotary applied to dk when non-NULL ([Lk][d/2] (cos, sin)) */
  int32_t rot_d;
  /* optional f32 copy of O (forward writes it, backward's delta = rowsum(dO . O) reads it): keeps delta
     free of the bf16 rounding of O, which otherwise cancels badly when the keys are nearly alike */
  float* o32;
  int64_t so32, bo32;
  /* dQ is summed over key blocks without atomics: the backward writes one f32 partial per 128-key block
     into dq_part ([svae_attn_dq_part_elems] floats), then a second kernel sums them (times scale) into dq_bf
     (bf16, row stride ldq_bf, inverse rotary with rot_tab at pos = query row when rot_tab is set) or, when
     dq_bf is NULL, into dq (f32, no rotary). */
  float* dq_part;
  void* dq_bf;
  int64_t ldq_bf;
  /* > 0 (causal only): block-sparse sliding window of SparseAttention (sparse_attention.py:39-60 with
     block_size 32, include_cls): query q sees key k <= q iff k < 32 or k / 32 >= q / 32 - (window - 1).
     0 = dense. */
  int32_t window;
  /* backward: 1 = delta already holds rowsum(dO . O) (svae_gemm's delta epilogue on the dO GEMM): the delta pass is
     skipped */
  int32_t delta_ready;
  /* optional bf16 residual of O (the alternative to o32, 2 B per element instead of 4): the forward writes
     o_lo = bf16(O - bf16(O)) (row stride so_lo, batch stride bo_lo), the backward's delta pass reads dO . (o + o_lo):
     O to ~16 significant bits, where the f32-accumulated O itself carries ~19 */
  void* o_lo;
  int64_t so_lo, bo_lo;
  /* forward, few queries over many keys (<= 128 queries, non-causal, >= 2048 keys, < 128 query tiles in all): optional
     f32 workspace of svae_attn_fwd_ws_elems floats (16-B aligned); when given, the keys are cut into slices (one launch,
     the slice a grid dimension) whose partial O / lse are combined (split-KV), so a long key sequence fills the chip.
     NULL: one pass. */
  float* fwd_ws;
  int64_t fwd_ws_elems;
} svae_attn_desc;

int svae_attn_fwd(const svae_attn_desc* d, svae_stream_t stream);
/* floats of the split-KV forward's workspace for a shape (0: that shape runs in one pass) */
int64_t svae_attn_fwd_ws_elems(int32_t B, int32_t H, int32_t Lq, int32_t Lk, int32_t hd, int32_t causal, int32_t window);
int svae_attn_bwd(const svae_attn_desc* d, svae_stream_t stream);
/* floats of the dq_part workspace: ceil(Lk / 128) * B * Lq * H * hd (+ the sliding window's [CLS] slabs) -- enough for
   every mode */
int64_t svae_attn_dq_part_elems(int32_t B, int32_t H, int32_t Lq, int32_t Lk, int32_t hd);
/* the same for a given sliding window (0 = dense): in window mode the 8-wave backward keeps dQ planes >= 1 to their
   band's rows, O(Lq) floats instead of O(Lq^2 / 512) (2 x 16384 tokens at hd 64: 36 MB instead of 8.6 GB) */
int64_t svae_attn_dq_part_elems_w(int32_t B, int32_t H, int32_t Lq, int32_t Lk, int32_t hd, int32_t window);
/* dq f32 [rows][H*hd] -> bf16 out (row stride ldo) with optional inverse rotary (pos = row % seq). */
int svae_dq_finalize(const float* dq, void* out, int64_t ldo, int32_t rows, int32_t D, const float* rot_tab,
                     int32_t seq, svae_stream_t stream);

/* ---- embedding (transformer_language_model.py:40-48): gather rows / scatter-add grads ------------- */
int svae_embedding_fwd(const int32_t* ids, const void* table_bf, float* out, void* out_bf, int32_t rows,
                       int32_t D, svae_stream_t stream);
/* the same gather into two f32 destinations (the encoder's input and the decoder's, whose position-0 rows the z
 * splice overwrites): replaces a device copy of the [rows, D] result */
int svae_embedding_fwd_dual(const int32_t* ids, const void* table, float* out, float* out2, int32_t rows, int32_t D,
                            svae_stream_t stream);
int svae_embedding_bwd(const int32_t* ids, const float* dout, float* dtable, int32_t rows, int32_t D,
                       svae_stream_t stream);

/* ---- reparameterise + KL (conditional_gaussian.py:18-28, continuous_autoencoder.py:42-52) -----------
 * stats: f32 [B][2*Z] (mu | logvar). eps: f32 [B][Z] or NULL (then drawn from (seed) in-kernel).
 * z out bf16 [B][Z] and f32 copy; raw_kl f32 [B]; kl_out f32[2] = {mean(raw_kl / ntok), mean(raw_kl)}.
 * Backward: dstats from dz (bf16 or f32) and the scalar kl gradient weight. */
int svae_reparam_kl_fwd(const float* stats, const float* eps, uint64_t seed, const int64_t* ntok,
                        float* z, void* z_bf, float* eps_out, float* raw_kl, float* kl_out, int32_t B,
                        int32_t Z, svae_stream_t stream);
int svae_reparam_kl_bwd(const float* stats, const float* eps, const float* dz, const int64_t* ntok,
                        const float* gkl, float* dstats, int32_t B, int32_t Z, svae_stream_t stream);

/* ---- cross entropy over materialised bf16 logits (robust_cross_entropy, language_model.py:161-170) --
 * part: f32 [rows][ntile][2] (max, sumexp) from SVAE_EPI_CE_STATS; label_logit f32 [rows].
 * Row r is position (r % seq) of its sequence (rows % seq == 0); label 0 = ignore_index. The sequence
 * positions are cut into nchunks chunks of chunk_len (torch.chunk along the sequence dim, :168; the last
 * chunk runs to the end of the sequence) and nll = mean over chunks of the per-chunk mean loss (a single
 * F.cross_entropy when nchunks == 1, :164-165). 1 <= nchunks <= 1024, (nchunks - 1) * chunk_len < seq.
 * finalize: lse[rows], row_loss[rows] (lse - label logit, 0 for ignored rows), chunk_w[nchunks]
 * (= 1 / (count_c * nchunks)), nll_out[1]; red_ws: f32 workspace of svae_ce_red_ws_elems(nchunks) floats
 * (per-block chunk partials, added in a fixed order: deterministic).
 * weighted_nll: the same chunked mean with F.cross_entropy's class weights (the val_bpb metric,
 * language_model.py:106-110): per chunk sum tok_w[y] * row_loss / sum tok_w[y]; tok_w f32 [V].
 * grad: in place, logits -> gscale[0] * chunk_w[c] * (softmax - onehot) in bf16 (0 for ignored rows);
 * dbias (optional, f32 [V]) += column sums of dlogits (output-bias gradient). */
int svae_ce_finalize(const float* part, int32_t ntile, const float* label_logit, const int32_t* labels,
                     int32_t rows, int32_t seq, int32_t nchunks, int32_t chunk_len, float* lse, float* row_loss,
                     float* chunk_w, float* nll_out, float* red_ws, svae_stream_t stream);
int svae_ce_weighted_nll(const float* row_loss, const int32_t* labels, const float* tok_w, int32_t rows,
                         int32_t seq, int32_t nchunks, int32_t chunk_len, float* out, float* red_ws,
                         svae_stream_t stream);
int32_t svae_ce_red_ws_elems(int32_t nchunks);
int svae_ce_grad(void* logits, int64_t ld, const float* lse, const float* chunk_w, const int32_t* labels,
                 const float* gscale, float* dbias, int32_t rows, int32_t V, int32_t seq, int32_t nchunks,
                 int32_t chunk_len, svae_stream_t stream);

/* ---- P-head cross entropy (training path of the tied vocabulary head + robust_cross_entropy) -----------
 * The head GEMM (SVAE_EPI_CE_PROB, row_a = c) stores P = exp(logit - c), c = the row's label logit, instead of
 * the logits; the backward then needs neither an exponential nor a dlogits pass:
 *   dlogits = r (x) P - q (x) onehot(label),  q = gscale * chunk_w[chunk] (0 for ignored rows),
 *   r = q * exp(c - lse);  dX = r . (P W) - q W[label] (SVAE_EPI_ROWSCALE_GATHER);
 *   dW = P^T (r . hh) (+ the one-hot part, svae_embedding_bwd_ce); d bias = sum_t r_t P[t] (k_weight row sums
 *   of the dW GEMM) - q scattered to the labels (bwd_prep).
 * ce_label_logit: out[r] = hh[r] . W[labels[r]] + bias[labels[r]] (f32 dot of bf16 rows; 0 where labels[r] = 0).
 * ce_prob_finalize: part f32 [ntile][rows] (the per-tile sums of P) -> lse = c + log sum, row_loss = lse - c,
 *   chunk_w, nll_out: the chunked mean of means of svae_ce_finalize.
 * ce_prob_bwd_prep: r_out, q_out [rows]; hh_out bf16 [rows][D] = r * hh; dbias[label] -= q (atomics; may be NULL).
 * The GEMM's exponent overflows to +inf for a logit more than 88 nats above the label logit; ce_prob_finalize_fix
 * finds every labelled row whose sum of P reaches 2^100 (or is not finite), lists it in sat_ws (int32 [1 + rows]:
 * count, then rows; the count stays readable after the call) and recomputes it exactly: the row's logits from hh, W
 * and bias, P[row] = exp(logit - max) (bf16, into P with leading dimension ldp), lse = max + log sum, row_loss =
 * lse - c, and row_off[row] = max -- so the backward (which reads P, row_off and lse) stays consistent. At most 1024
 * rows are recomputed (~5 ms worst case at V = 32768, D = 512); past that the step is diverging, the remaining rows
 * keep their overflowed P (their loss is infinite) and the count still lists every flagged row.
 * ce_prob_finalize = ce_prob_finalize_fix without the check (sat_ws = NULL). */
int svae_ce_label_logit(const void* hh, int64_t ldh, const void* W, int64_t ldw, const float* bias,
                        const int32_t* labels, int32_t rows, int32_t D, float* out, svae_stream_t stream);
int svae_ce_prob_finalize(const float* part, int32_t ntile, const float* row_off, const int32_t* labels,
                          int32_t rows, int32_t seq, int32_t nchunks, int32_t chunk_len, float* lse, float* row_loss,
                          float* chunk_w, float* nll_out, float* red_ws, svae_stream_t stream);
int svae_ce_prob_finalize_fix(const float* part, int32_t ntile, float* row_off, const int32_t* labels, int32_t rows,
                              int32_t seq, int32_t nchunks, int32_t chunk_len, float* lse, float* row_loss,
                              float* chunk_w, float* nll_out, float* red_ws, const void* hh, int64_t ldh, const void* W,
                              int64_t ldw, const float* bias, void* P, int64_t ldp, int32_t V, int32_t D,
                              int32_t* sat_ws, svae_stream_t stream);
int svae_ce_prob_bwd_prep(const void* hh, int64_t ldh, const float* lse, const float* row_off, const float* chunk_w,
                          const int32_t* labels, const float* gscale, int32_t rows, int32_t seq, int32_t nchunks,
                          int32_t chunk_len, int32_t D, void* hh_out, float* r_out, float* q_out, float* dbias,
                          svae_stream_t stream);
/* Embedding backward fused with the one-hot part of the P-head's dW: dtable[ids[t]] += dout[t] - q[t-1] * hh[t-1]
 * (the second term where t % seq != 0; valid because labels[t-1] = ids[t] inside a sequence). */
int svae_embedding_bwd_ce(const int32_t* ids, const float* dout, float* dtable, int32_t rows, int32_t D, int32_t seq,
                          const void* hh, const float* q, svae_stream_t stream);

/* ---- elementwise helpers ------------------------------------------------------------------------ */
/* dropout backward + cast: out bf16 = keep(seed, idx) * g / (1-p) (p = 0: plain cast). */
int svae_dropout_bwd_cast(const float* g, void* out, float p, uint64_t seed, int64_t n, int32_t cols,
                          int64_t ld_in, svae_stream_t stream);
/* GELU backward (transformer_language_model.py:57 head GELU): out bf16 = dx * gp, gp = gelu' saved by the
   forward's SVAE_EPI_GELU epilogue. */
int svae_gelu_bwd(const float* dx, const void* gp, void* out, int64_t n, svae_stream_t stream);
/* The training step's token inputs (transformer_vae.py:42-55 / language_model.py's next-token targets), one pass:
 * ids32[t] = int32(ids[t]), labels[t] = ids[t + 1] inside a sequence of L and 0 at its last position, padm[t]
 * (uint8) = (ids[t] == 0) for pad_mode 1 or pad[t] (bool bytes) for pad_mode 2 (pad_mode 0: no mask), and
 * ntok_out[b] = ntok[b] for b < B when both are given. ids int64 [B][L] contiguous. */
int svae_prep_tokens(const int64_t* ids, const void* pad, int32_t pad_mode, int32_t B, int32_t L, int32_t* ids32,
                     int32_t* labels, void* padm, const int64_t* ntok, int64_t* ntok_out, svae_stream_t stream);
/* The step's scalars (transformer_vae.py:55 and its autograd backward): loss[0] = nll[0] + kl_weight * kl[0] when
 * loss != NULL; gs[0] = gloss[0], gs[1] = gloss[0] * kl_weight when gs != NULL (f32, each op rounded separately). */
int svae_step_scalars(const float* nll, const float* kl, const float* gloss, float kl_weight, float* loss, float* gs,
                      svae_stream_t stream);
/* cast f32 -> bf16 (n elements). */
int svae_cast_bf16(const float* in, void* out, int64_t n, svae_stream_t stream);
/* Transposed bf16 weight shadows (the K-contiguous B operand of the dX GEMMs): for each of nblocks
 * blocks, table[4b..4b+3] = (element offset, rows, cols, first tile) on the device, rows and cols % 8 == 0,
 * dst[offset + c * rows + r] = src[offset + r * cols + c]; one workgroup per 64 x 64 tile. */
int svae_transpose_blocks(const void* src, void* dst, const int64_t* table, int32_t nblocks, int32_t total_tiles,
                          svae_stream_t stream);
/* rows of x (f32 [rows][D], stride ld) whose (row % mod == 0) are copied to out [rows/mod][D] and zeroed
 * (the position-0 gradient of the z-projection splice, transformer_vae.py:89-90). */
int svae_extract_rows(float* x, int64_t ld, int32_t rows, int32_t mod, int32_t D, float* out,
                      svae_stream_t stream);
/* z_projections[i] backward (transformer_vae.py:89-90, x[:, 0] = nn.Linear(Z, d)(z)) from the position-0 gradient
 * g f32 [B][d]: dW f32 [d][Z] += g^T z, db f32 [d] += sum_b g[b], dz f32 [B][Z] += g W, with z bf16 [B][Z] and
 * W bf16 [d][Z] the forward's operands; f32 accumulation in a fixed order (deterministic), one launch (replaces the
 * dW GEMM with fused bias row sums and the split-K dz GEMM of a decoder layer). */
int svae_zproj_bwd(const float* g, const void* z, const void* W, float* dW, float* db, float* dz, int32_t B,
                   int32_t d, int32_t Z, svae_stream_t stream);
/* n (<= SVAE_ZPROJ_MAX) z-projection backwards sharing z and dz in one launch: for each segment, dW += g^T z and
 * db += sum_b g as svae_zproj_bwd; dz += g_0 W_0, then += g_1 W_1, ... in list order -- the same f32 results as n
 * svae_zproj_bwd calls in that order. */
#define SVAE_ZPROJ_MAX 32
typedef struct svae_zproj_seg {
  const float* g;   /* [B][d] f32 */
  const void* W;    /* [d][Z] bf16 */
  float* dW;        /* [d][Z] f32 */
  float* db;        /* [d] f32 */
} svae_zproj_seg;
int svae_zproj_bwd_multi(const svae_zproj_seg* segs, int32_t n, const void* z, float* dz, int32_t B, int32_t d,
                         int32_t Z, svae_stream_t stream);
/* The forward of n (<= SVAE_ZPROJ_MAX) z projections in one launch (transformer_vae.py:89, z_projections[i](z)):
 * out_i [B][d] f32 = z W_i^T + bias_i, z bf16 [B][Z] (Z <= 1024), W_i bf16 [d][Z]; f32 FMAs over k in order. */
typedef struct svae_zproj_fwd_seg {
  const void* W;       /* [d][Z] bf16 */
  const float* bias;   /* [d] f32 */
  float* out;          /* [B][d] f32 */
} svae_zproj_fwd_seg;
int svae_zproj_fwd_multi(const svae_zproj_fwd_seg* segs, int32_t n, const void* z, int32_t B, int32_t d, int32_t Z,
                         svae_stream_t stream);

/* ---- optimiser (RAdam, rectified_adam.py:16-88; clip_grad_norm_, language_model.py:120-122) -------
 * sumsq: partial sums of g^2 over n elements into part[nblk]; radam: reads part to form the global
 * norm, clips, updates m, v, p (f32) and the bf16 shadow pbf in one pass. scal: {lr_eff, bcm, bcv,
 * rho_ok, beta1, beta2, eps, wd_lr, max_norm}. norm_out[0] = total grad norm (pre-clip). */
int svae_sumsq(const float* g, int64_t n, float* part, int32_t nblk, svae_stream_t stream);
int svae_radam(float* p, void* pbf, const float* g, float* m, float* v, int64_t n, const float* part,
               int32_t nblk, const float* scal, float* norm_out, svae_stream_t stream);
/* In-place clip_grad_norm_ of a micro-step that no optimiser step follows (gradient accumulation): g *=
 * min(1, max_norm / (norm + 1e-6)) with norm from the sumsq partials; norm_out[0] = norm (may be NULL).
 * n % 4 == 0, g 16-byte aligned. */
int svae_clip_grad(float* g, int64_t n, const float* part, int32_t nblk, float max_norm, float* norm_out,
                   svae_stream_t stream);

/* ---- fp32 kernel mode (argmax-reconstruction parity; TransformerVAE.reconstruct in exact f32) ---------
 * svae_gemm_f32: C[M,N] = epi(A[M,K] . W[N,K]^T) on f32-input MFMA; epi in {SVAE_EPI_F32 (+bias, +resid),
 * SVAE_EPI_ROTARY_BF16 (rotary on cols < rot_cols, f32 out), SVAE_EPI_GELU (f32 out)}.
 * svae_attn_fwd_f32: attention forward in f32 (same strides / masks / window as svae_attn_desc).
 * svae_layernorm_fwd_f32: LayerNorm with f32 output. */
int svae_gemm_f32(const float* A, const float* W, float* C, int32_t M, int32_t N, int32_t K, int64_t lda, int64_t ldw,
                  int64_t ldc, const float* bias, const float* resid, int64_t ldr, int32_t epi, const float* rot_tab,
                  int32_t rot_cols, int32_t rot_d, int32_t rot_seq, svae_stream_t stream);
int svae_attn_fwd_f32(const float* q, const float* k, const float* v, float* o, int64_t sq, int64_t sk, int64_t sv,
                      int64_t so, int64_t bq, int64_t bk, int64_t bv, int64_t bo, const uint8_t* key_pad, int32_t B,
                      int32_t H, int32_t Lq, int32_t Lk, int32_t hd, int32_t causal, int32_t window, float scale,
                      svae_stream_t stream);
int svae_layernorm_fwd_f32(const float* x, const float* w, const float* b, float* y, int32_t rows, int32_t D,
                           svae_stream_t stream);

/* ---- mutual-information log (transformer_vae.py:59-61, math_utils.py:51-58) ---------------------------
 * out[0] = kl[0] - marginal_kl(q), q = N(mu, exp(logvar)) from stats [B][2Z] (mu | logvar), with S posterior
 * samples per sequence: eps f32 [S][B][Z] or NULL (counter-based normals from seed). ws: f32 workspace of
 * >= 2 * S * B floats. Log-only diagnostic (not in the loss). */
int svae_mutual_info(const float* stats, const float* eps, uint64_t seed, const float* kl, int32_t B, int32_t Z,
                     int32_t S, float* ws, float* out, svae_stream_t stream);

/* ---- evaluation: log p(x|z) per sequence (continuous_autoencoder.py:82-88) ---------------------------
 * From the SVAE_EPI_CE_STATS partials of the head GEMM (which may run with C = NULL: no logits stored):
 * out[s] = sum over the rows r of sequence s (rows s*seq .. s*seq+seq-1) with labels[r] != 0 of
 * (label_logit[r] - logsumexp_r); labels 0 add 0 (the reference zeroes log_softmax column 0). */
int svae_ce_seq_logprob(const float* part, int32_t ntile, const float* label_logit, const int32_t* labels,
                        int32_t rows, int32_t seq, float* out, svae_stream_t stream);

/* ---- autoregressive decoding (TransformerVAE.sample, transformer_vae.py:95-128; the KV cache of
 * attention.py:107-168; GenerationState, generation.py). All f32. `cur` is a device int32 holding
 * GenerationState.current_index: kernels read it at run time, so a captured step graph replays for every
 * position. out_ids: int64 [B][T] (GenerationState.output_ids); live: uint8 [B].
 * dec_linear: Y[M,N] = epi(X[M,K] . W[N,K]^T + bias) + resid; epi SVAE_EPI_F32 / SVAE_EPI_GELU /
 *   SVAE_EPI_ROTARY_BF16 (rotary of rot_tab row cur-1 on columns < rot_cols, pairs within rot_d; f32 out).
 *   K % 4 == 0, X and W 16-byte aligned. part_ws (f32, part_elems floats, may be NULL): split-K partials for
 *   narrow N (the library picks the split count that fits; NULL = no split).
 * dec_attn: qkv f32 [B][ldq] = q | k | v (rotary applied); appends k, v at position cur-1 to the caches
 *   [B][H][T][hd] and writes O[b][h*hd ..] = softmax(q k^T * scale) v over the visible keys: 0..cur-1, or with
 *   window > 0 the sliding-window cache's set ([CLS] block, window-1 previous 32-blocks, current block).
 * dec_embed: x[b] = table[out_ids[b][cur-1]].
 * dec_penalty: repetition penalty on logits rows (row r is sequence row_map[r], or r): the ids
 *   out_ids[b][max(cur-512,0) .. cur-1] get logit * penalty if < 0 else logit / penalty (generation.py:35-41).
 * dec_sample: per live row: greedy (temperature <= 0 or top_k == 1) or temperature / top-k / nucleus top-p +
 *   multinomial from (seed, cur, b); writes out_ids[b][cur]; clears live[b] (and decrements *live_count)
 *   when the token is end_token or cur + 1 >= T (generation.py:43-77). V <= 32768.
 * dec_advance: *cur += 1. */
int svae_dec_linear(const float* X, int64_t ldx, const float* W, int64_t ldw, const float* bias, float* Y, int64_t ldy,
                    const float* resid, int64_t ldr, int32_t M, int32_t N, int32_t K, int32_t epi, const float* rot_tab,
                    int32_t rot_cols, int32_t rot_d, const int32_t* cur, float* part_ws, int64_t part_elems,
                    svae_stream_t stream);
int svae_dec_attn(const float* qkv, int64_t ldq, float* kcache, float* vcache, int32_t B, int32_t H, int32_t hd,
                  int32_t T, const int32_t* cur, int32_t window, float scale, float* O, int64_t ldo,
                  svae_stream_t stream);
int svae_dec_embed(const int64_t* out_ids, int32_t T, const int32_t* cur, const float* table, float* x, int32_t B,
                   int32_t D, svae_stream_t stream);
int svae_dec_penalty(float* logits, int64_t ldl, int32_t rows, const int32_t* row_map, const int64_t* out_ids,
                     int32_t T, const int32_t* cur, const uint8_t* live, float penalty, svae_stream_t stream);
int svae_dec_sample(const float* logits, int64_t ldl, int32_t V, int32_t rows, const int32_t* row_map,
                    int64_t* out_ids, int32_t T, const int32_t* cur, uint8_t* live, int32_t end_token,
                    float temperature, int32_t top_k, float top_p, uint64_t seed, int32_t* live_count,
                    svae_stream_t stream);
int svae_dec_advance(int32_t* cur, svae_stream_t stream);

/* library identification: returns a static string (build id, target arch). */
const char* svae_version(void);

#ifdef __cplusplus
}
#endif
#endif
