// fp32 kernel mode: the decoder + head forward of TransformerVAE.reconstruct (transformer_vae.py:85-93) in
// exact f32, for the bit-exact argmax-reconstruction check against the fp32 reference (the bf16 path keeps
// ~96% argmax agreement at init). Not a throughput path.
//
//   svae_gemm_f32:     C = epi(A[M,K] . W[N,K]^T) on v_mfma_f32_16x16x4_f32 (f32 in, f32 accumulate: a
//                      k-ordered fmaf chain), 64x64 tiles, epilogues F32 (+bias, +resid), ROTARY, GELU.
//   svae_attn_fwd_f32: softmax(q k^T * scale - 1e7 * mask) v per (batch, head, query), two-pass in LDS.
#include "common.h"
#include "../../include/svae.h"

using namespace svae;

namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));

// 64x64 output tile, 256 threads = 4 waves (2x2), each wave 32x32 = 2x2 MFMA 16x16x4 tiles; K step 16.
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ A, const float* __restrict__ W,
                                                       float* __restrict__ C, int M, int N, int K, long long lda,
                                                       long long ldw, long long ldc, const float* __restrict__ bias,
                                                       const float* __restrict__ resid, long long ldr, int epi,
                                                       const float* __restrict__ rot, int rot_cols, int rot_d,
                                                       int rot_seq) {
  __shared__ float As[64][17];
  __shared__ float Ws[64][17];
  __shared__ float Cs[64][65];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  f32x4v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4v){0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 16) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int idx = tid + 256 * t, r = idx >> 4, c = idx & 15;
      As[r][c] = (m0 + r < M && k0 + c < K) ? A[(long long)(m0 + r) * lda + k0 + c] : 0.f;
      Ws[r][c] = (n0 + r < N && k0 + c < K) ? W[(long long)(n0 + r) * ldw + k0 + c] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; kk += 4) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float a = As[wm * 32 + i * 16 + (lane & 15)][kk + (lane >> 4)];
          const float b = Ws[wn * 32 + j * 16 + (lane & 15)][kk + (lane >> 4)];
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i][j], 0, 0, 0);
        }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) Cs[wm * 32 + i * 16 + 4 * (lane >> 4) + r][wn * 32 + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  for (int e = tid; e < 64 * 32; e += 256) {        // pairs of adjacent columns (rotary pairs)
    const int r = e >> 5, c = (e & 31) * 2, m = m0 + r, n = n0 + c;
    if (m >= M || n >= N) continue;
    float x0 = Cs[r][c] + (bias ? bias[n] : 0.f);
    float x1 = (n + 1 < N) ? Cs[r][c + 1] + (bias ? bias[n + 1] : 0.f) : 0.f;
    if (epi == SVAE_EPI_ROTARY_BF16 && n < rot_cols) {
      const float2 cs = ((const float2*)rot)[(long long)(m % rot_seq) * (rot_d / 2) + (n % rot_d) / 2];
      const float a = x0, b = x1;
      x0 = a * cs.x + (-b) * cs.y;
      x1 = b * cs.x + a * cs.y;
    } else if (epi == SVAE_EPI_GELU) {
      x0 = gelu_f(x0);
      x1 = gelu_f(x1);
    }
    if (resid) {
      x0 += resid[(long long)m * ldr + n];
      if (n + 1 < N) x1 += resid[(long long)m * ldr + n + 1];
    }
    C[(long long)m * ldc + n] = x0;
    if (n + 1 < N) C[(long long)m * ldc + n + 1] = x1;
  }
}

// One wave per (batch, head, query); scores for every key in LDS, softmax, then o[d] = sum_j p_j v[j][d]. WPB waves
// (queries) per block: 4 up to 8192 keys, fewer beyond (each wave's score row is Lk floats of the 160 KiB LDS).
template <int WPB>
__global__ __launch_bounds__(64 * WPB) void attn_fwd_f32_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                           const float* __restrict__ v, float* __restrict__ o,
                                                           long long sq, long long sk, long long sv, long long so,
                                                           long long bq, long long bk, long long bv, long long bo,
                                                           const unsigned char* __restrict__ pad, int B, int H,
                                                           int Lq, int Lk, int hd, int causal, int window,
                                                           float scale) {
  extern __shared__ float sc[];   // [4 waves][Lk]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long gid_raw = (long long)blockIdx.x * WPB + wave;
  const bool valid = gid_raw < (long long)B * H * Lq;
  const long long gid = valid ? gid_raw : 0;
  const int qi = (int)(gid % Lq), h = (int)((gid / Lq) % H), b = (int)(gid / ((long long)Lq * H));
  float* s = sc + wave * Lk;
  const float* qp = q + b * bq + (long long)qi * sq + (long long)h * hd;
  float mx = -INFINITY;
  for (int j = lane; j < Lk && valid; j += 64) {
    const float* kp = k + b * bk + (long long)j * sk + (long long)h * hd;
    float dot = 0.f;
    for (int dd = 0; dd < hd; ++dd) dot = fmaf(qp[dd], kp[dd], dot);
    float x = dot * scale;
    // window > 0: keys outside SparseAttention's causal band + [CLS] block (sparse_attention.py:39-60) are
    // absent from the reference's block-sparse softmax; the -1e7 shift gives them exactly zero weight too
    const bool out_of_band = window > 0 && j >= 32 && j / 32 < qi / 32 - (window - 1);
    const bool m = (pad && pad[(long long)b * Lk + j]) || (causal && j > qi) || out_of_band;
    if (m) x = x - 1e7f;          // attention.py:98 (score - mask * 1e7)
    s[j] = x;
    mx = fmaxf(mx, x);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j < Lk && valid; j += 64) {
    const float e = expf(s[j] - mx);
    s[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  __syncthreads();
  if (!valid) return;
  for (int dd = lane; dd < hd; dd += 64) {
    float acc = 0.f;
    for (int j = 0; j < Lk; ++j) acc = fmaf(s[j], v[b * bv + (long long)j * sv + (long long)h * hd + dd], acc);
    o[b * bo + (long long)qi * so + (long long)h * hd + dd] = acc / sum;
  }
}

__global__ __launch_bounds__(256) void ln_fwd_f32_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ bb, float* __restrict__ y, int rows,
                                                         int D) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + (long long)row * D;
  float s = 0.f;
  for (int c = lane; c < D; c += 64) s += xr[c];
  const float mean = wave_sum(s) / D;
  float sq = 0.f;
  for (int c = lane; c < D; c += 64) { const float t = xr[c] - mean; sq += t * t; }
  const float rstd = 1.0f / sqrtf(wave_sum(sq) / D + 1e-5f);
  for (int c = lane; c < D; c += 64) y[(long long)row * D + c] = (xr[c] - mean) * rstd * w[c] + bb[c];
}

}  // namespace

SVAE_EXPORT int svae_gemm_f32(const float* A, const float* W, float* C, int32_t M, int32_t N, int32_t K, int64_t lda,
                              int64_t ldw, int64_t ldc, const float* bias, const float* resid, int64_t ldr, int32_t epi,
                              const float* rot_tab, int32_t rot_cols, int32_t rot_d, int32_t rot_seq,
                              svae_stream_t stream) {
  if (!A || !W || !C || M <= 0 || N <= 0 || K <= 0) return SVAE_EINVAL;
  if (epi != SVAE_EPI_F32 && epi != SVAE_EPI_ROTARY_BF16 && epi != SVAE_EPI_GELU) return SVAE_EINVAL;
  if (epi == SVAE_EPI_ROTARY_BF16 && (!rot_tab || rot_d <= 0 || rot_seq <= 0 || rot_cols % 2)) return SVAE_EINVAL;
  dim3 grid((N + 63) / 64, (M + 63) / 64);
  hipLaunchKernelGGL(gemm_f32_kernel, grid, dim3(256), 0, (hipStream_t)stream, A, W, C, M, N, K, lda, ldw, ldc, bias,
                     resid, ldr, epi, rot_tab, rot_cols, rot_d, rot_seq);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_attn_fwd_f32(const float* q, const float* k, const float* v, float* o, int64_t sq, int64_t sk,
                                  int64_t sv, int64_t so, int64_t bq, int64_t bk, int64_t bv, int64_t bo,
                                  const uint8_t* key_pad, int32_t B, int32_t H, int32_t Lq, int32_t Lk, int32_t hd,
                                  int32_t causal, int32_t window, float scale, svae_stream_t stream) {
  if (!q || !k || !v || !o || B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0 || hd <= 0 || Lk > 32768) return SVAE_EINVAL;
  if (window < 0 || (window > 0 && !causal)) return SVAE_EINVAL;
  const long long n = (long long)B * H * Lq;
  hipStream_t st = (hipStream_t)stream;
  if (Lk <= 8192)
    hipLaunchKernelGGL(attn_fwd_f32_kernel<4>, dim3((unsigned)((n + 3) / 4)), dim3(256), 4 * Lk * sizeof(float), st, q, k,
                       v, o, sq, sk, sv, so, bq, bk, bv, bo, key_pad, B, H, Lq, Lk, hd, causal, window, scale);
  else if (Lk <= 16384)
    hipLaunchKernelGGL(attn_fwd_f32_kernel<2>, dim3((unsigned)((n + 1) / 2)), dim3(128), 2 * Lk * sizeof(float), st, q, k,
                       v, o, sq, sk, sv, so, bq, bk, bv, bo, key_pad, B, H, Lq, Lk, hd, causal, window, scale);
  else
    hipLaunchKernelGGL(attn_fwd_f32_kernel<1>, dim3((unsigned)n), dim3(64), Lk * sizeof(float), st, q, k, v, o, sq, sk,
                       sv, so, bq, bk, bv, bo, key_pad, B, H, Lq, Lk, hd, causal, window, scale);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_layernorm_fwd_f32(const float* x, const float* w, const float* b, float* y, int32_t rows,
                                       int32_t D, svae_stream_t stream) {
  if (!x || !w || !b || !y || rows <= 0 || D <= 0) return SVAE_EINVAL;
  hipLaunchKernelGGL(ln_fwd_f32_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, x, w, b, y, rows, D);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}
