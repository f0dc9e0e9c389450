// Autoregressive decoding of TransformerVAE.sample (transformer_vae.py:95-128) with a KV cache
// (attention.py:107-168) and GenerationState.process_logits (generation.py:27-77), in f32.
//
// Decode is latency-bound: one token per sequence per step, M = batch rows. Every kernel here reads the step's
// position from a device scalar (`cur` = GenerationState.current_index) instead of a launch argument, so one
// captured step graph (hipGraph via torch.cuda.CUDAGraph) replays for every position.
//
//   svae_dec_linear:  Y[M,N] = epi(X[M,K] . W[N,K]^T + b) (+ resid): weight-streaming skinny GEMM on
//                     v_mfma_f32_16x16x4_f32, 16 output columns per workgroup, K split over its 16 waves (LDS
//                     reduction) and, for narrow N, over workgroups (partials + an ordered finalize); epilogues
//                     plain / GELU / rotary at position cur-1.
//   svae_dec_attn:    one workgroup per (sequence, head): appends k, v at position cur-1 to the cache
//                     [B][H][T][hd] and attends over the visible keys (dense causal, or the sliding-window
//                     cache's key set: [CLS] block + window-1 previous blocks + the current block).
//   svae_dec_embed:   x[b] = W_emb[out_ids[b][cur-1]]   (the previous token, generation.py:27-28).
//   svae_dec_penalty: repetition penalty over the last 512 generated ids (generation.py:35-41).
//   svae_dec_sample:  greedy / temperature / top-k / top-p (nucleus) + multinomial with a counter-based RNG,
//                     writes out_ids[b][cur], updates the live mask (generation.py:43-77).
//   svae_dec_advance: cur += 1.
#include "common.h"
#include "../../include/svae.h"

using namespace svae;

namespace {

// ------------------------------------------------------------------ skinny f32 linear
// 16 output columns x up to 64 rows per workgroup of 16 waves; the waves split the workgroup's K range and meet in
// LDS. Narrow outputs (a d x d weight is only N / 16 = 32 workgroups wide) also split K over workgroups
// (gridDim.z = splits): each writes its partial sums to a caller-owned workspace and a finalize pass adds the
// splits in a fixed order and applies the epilogue (deterministic, no atomics).
constexpr int DL_MROWS = 64;   // rows per workgroup (4 MFMA m-tiles)
constexpr int DL_WAVES = 16;

struct DL {
  const float* X; long long ldx;
  const float* W; long long ldw;
  const float* bias;
  float* Y; long long ldy;
  const float* resid; long long ldr;
  int M, N, K, kslice;
  const float* rot; int rot_cols, rot_d;
  const int* cur;
  float* part;        // [splits][M][N] partial sums (split-K), or nullptr
};

template <int EPI>
__device__ __forceinline__ void dl_epilogue(const DL& p, int m, int nn, float x0, float x1, int pos) {
  if (p.bias) {
    x0 += p.bias[nn];
    if (nn + 1 < p.N) x1 += p.bias[nn + 1];
  }
  if constexpr (EPI == SVAE_EPI_GELU) {
    x0 = gelu_f(x0);
    x1 = gelu_f(x1);
  } else if constexpr (EPI == SVAE_EPI_ROTARY_BF16) {
    if (nn < p.rot_cols) {
      const float2 cs = ((const float2*)p.rot)[(long long)pos * (p.rot_d / 2) + (nn % p.rot_d) / 2];
      const float a = x0, b = x1;
      x0 = a * cs.x + (-b) * cs.y;
      x1 = b * cs.x + a * cs.y;
    }
  }
  if (p.resid) {
    x0 += p.resid[(long long)m * p.ldr + nn];
    if (nn + 1 < p.N) x1 += p.resid[(long long)m * p.ldr + nn + 1];
  }
  p.Y[(long long)m * p.ldy + nn] = x0;
  if (nn + 1 < p.N) p.Y[(long long)m * p.ldy + nn + 1] = x1;
}

template <int EPI>
__global__ __launch_bounds__(1024) void dec_linear_kernel(DL p) {
  __shared__ float red[DL_WAVES][DL_MROWS][17];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16, m0 = blockIdx.y * DL_MROWS, split = blockIdx.z;
  const int mrows = min(DL_MROWS, p.M - m0);
  const int mt = (mrows + 15) >> 4;
  // this wave's K range inside the split's: a multiple of 16 (one float4 per lane per step)
  const int sb = split * p.kslice, se = min(p.K, sb + p.kslice);
  const int kq = ((se - sb + 16 * DL_WAVES - 1) / (16 * DL_WAVES)) * 16;
  const int kb = sb + wave * kq, ke = min(se, kb + kq);
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int n = n0 + r;
  const float* wrow = p.W + (long long)min(n, p.N - 1) * p.ldw;
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  for (int k = kb; k < ke; k += 32) {     // two K-steps per iteration: all loads issued before the MFMAs
    const int kk0 = k + 4 * g, kk1 = kk0 + 16;
    const bool in0 = kk0 < ke && n < p.N, in1 = kk1 < ke && n < p.N;
    const f32x4 w0 = in0 ? *(const f32x4*)(wrow + kk0) : zero;
    const f32x4 w1 = in1 ? *(const f32x4*)(wrow + kk1) : zero;
    f32x4 x0[4], x1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = i * 16 + r;
      const bool mok = i < mt && m < mrows;
      const float* xr = p.X + (long long)(m0 + (mok ? m : 0)) * p.ldx;
      x0[i] = (mok && kk0 < ke) ? *(const f32x4*)(xr + kk0) : zero;
      x1[i] = (mok && kk1 < ke) ? *(const f32x4*)(xr + kk1) : zero;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i < mt) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(x0[i][e], w0[e], acc[i], 0, 0, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(x1[i][e], w1[e], acc[i], 0, 0, 0);
      }
    }
  }
  // C/D layout: row = 4 * (lane >> 4) + e, col = lane & 15
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (i < mt)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[wave][i * 16 + 4 * g + e][r] = acc[i][e];
  __syncthreads();
  // epilogue: thread = (row, column pair); 64 rows x 8 pairs = 512 threads
  if (tid >= DL_MROWS * 8) return;
  const int row = tid >> 3, c = (tid & 7) * 2;
  if (row >= mrows) return;
  const int m = m0 + row, nn = n0 + c;
  if (nn >= p.N) return;
  float x0 = 0.f, x1 = 0.f;
#pragma unroll
  for (int w = 0; w < DL_WAVES; ++w) {
    x0 += red[w][row][c];
    x1 += red[w][row][c + 1];
  }
  if (p.part) {
    float* pp = p.part + ((long long)split * p.M + m) * p.N + nn;
    pp[0] = x0;
    if (nn + 1 < p.N) pp[1] = x1;
    return;
  }
  dl_epilogue<EPI>(p, m, nn, x0, x1, p.cur ? *p.cur - 1 : 0);
}

// split-K finalize: thread = (row, column pair), the splits added in order, then the epilogue
template <int EPI>
__global__ __launch_bounds__(256) void dec_linear_finalize_kernel(DL p, int splits) {
  const int half = (p.N + 1) / 2;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= p.M * half) return;
  const int m = i / half, nn = (i % half) * 2;
  float x0 = 0.f, x1 = 0.f;
  for (int s2 = 0; s2 < splits; ++s2) {
    const float* pp = p.part + ((long long)s2 * p.M + m) * p.N + nn;
    x0 += pp[0];
    if (nn + 1 < p.N) x1 += pp[1];
  }
  dl_epilogue<EPI>(p, m, nn, x0, x1, p.cur ? *p.cur - 1 : 0);
}

// ------------------------------------------------------------------ block reductions (256 / 1024 threads)
template <int NW>
__device__ __forceinline__ float block_max(float v, float* sh) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float r = sh[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) r = fmaxf(r, sh[i]);
  return r;
}
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) r += sh[i];
  return r;
}

// ------------------------------------------------------------------ decode attention
// grid (H, B), 256 threads. qkv f32 [B][ldq] with q | k | v (rotary already applied to q, k); caches
// [B][H][T][hd] f32; O [B][ldo]. Dynamic LDS: one score per visible key.
// 16 waves per (sequence, head): the P.V sweep runs 16 key groups (hd = 64) in parallel, so a workgroup keeps 4x
// more cache rows in flight than with 4 waves (the sweep is load-latency bound)
constexpr int DA_THREADS = 1024, DA_WAVES = DA_THREADS / 64;

__global__ __launch_bounds__(DA_THREADS) void dec_attn_kernel(const float* __restrict__ qkv, long long ldq,
                                                       float* __restrict__ kc, float* __restrict__ vc, int H, int hd,
                                                       int T, const int* __restrict__ cur, int window, float scale,
                                                       float* __restrict__ O, long long ldo) {
  extern __shared__ float sc[];
  __shared__ float qs[128], ks[128], vs[128], red[2 * DA_WAVES], osum[DA_THREADS];
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int d = H * hd;
  const int p = *cur - 1;
  const float* qrow = qkv + (long long)b * ldq + h * hd;
  const long long cbase = ((long long)b * H + h) * T * hd;
  if (tid < hd) {
    qs[tid] = qrow[tid];
    ks[tid] = qrow[d + tid];
    vs[tid] = qrow[2 * d + tid];
    kc[cbase + (long long)p * hd + tid] = ks[tid];
    vc[cbase + (long long)p * hd + tid] = vs[tid];
  }
  __syncthreads();
  // visible keys: [0, n1) then [lo2, p]
  int n1, lo2, n;
  if (window > 0) {
    n1 = min(p + 1, 32);
    lo2 = max(32, (p / 32 - (window - 1)) * 32);
    n = n1 + max(0, p + 1 - lo2);
  } else {
    n1 = p + 1;
    lo2 = 0;
    n = p + 1;
  }
  float mx = -INFINITY;
  for (int t = tid; t < n; t += DA_THREADS) {
    const int j = t < n1 ? t : lo2 + (t - n1);
    const float* kr = (j == p) ? ks : kc + cbase + (long long)j * hd;
    float s = 0.f;
    for (int c = 0; c < hd; c += 4) {
      const f32x4 k4 = (j == p) ? *(const f32x4*)(ks + c) : *(const f32x4*)(kr + c);
      s += qs[c] * k4[0] + qs[c + 1] * k4[1] + qs[c + 2] * k4[2] + qs[c + 3] * k4[3];
    }
    s *= scale;
    sc[t] = s;
    mx = fmaxf(mx, s);
  }
  mx = block_max<DA_WAVES>(mx, red);
  float se = 0.f;
  for (int t = tid; t < n; t += DA_THREADS) {
    const float e = __expf(sc[t] - mx);
    sc[t] = e;
    se += e;
  }
  se = block_sum<DA_WAVES>(se, red + DA_WAVES);
  // O[c] = sum_t sc[t] v[key(t)][c]: thread = (column c, key group gi)
  const int G = DA_THREADS / hd, c = tid % hd, gi = tid / hd;
  float acc = 0.f;
  if (gi < G) {
    for (int t = gi; t < n; t += G) {
      const int j = t < n1 ? t : lo2 + (t - n1);
      const float v = (j == p) ? vs[c] : vc[cbase + (long long)j * hd + c];
      acc += sc[t] * v;
    }
  }
  osum[tid] = acc;
  __syncthreads();
  if (tid < hd) {
    float o = 0.f;
    for (int i = 0; i < G; ++i) o += osum[i * hd + tid];
    O[(long long)b * ldo + h * hd + tid] = o / se;
  }
}

// ------------------------------------------------------------------ embedding of the previous token
__global__ __launch_bounds__(256) void dec_embed_kernel(const long long* __restrict__ out_ids, int T,
                                                        const int* __restrict__ cur, const float* __restrict__ table,
                                                        float* __restrict__ x, int B, int D) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= B) return;
  const long long tok = out_ids[(long long)b * T + *cur - 1];
  for (int c = lane * 4; c < D; c += 256) *(f32x4*)(x + (long long)b * D + c) = *(const f32x4*)(table + tok * D + c);
}

// ------------------------------------------------------------------ repetition penalty
// One block per logits row; the gathers all happen before any write, so a token repeated in the window is
// penalised once from its original value (torch gather then scatter_, generation.py:38-41).
__global__ __launch_bounds__(512) void dec_penalty_kernel(float* __restrict__ logits, long long ldl,
                                                          const int* __restrict__ row_map,
                                                          const long long* __restrict__ out_ids, int T,
                                                          const int* __restrict__ cur,
                                                          const unsigned char* __restrict__ live, float penalty) {
  const int r = blockIdx.x, b = row_map ? row_map[r] : r;
  if (live && !live[b]) return;
  const int c = *cur, left = max(c - 512, 0), nprev = c - left;
  float* row = logits + (long long)r * ldl;
  const int i = threadIdx.x;
  long long tok = 0;
  float v = 0.f;
  if (i < nprev) {
    tok = out_ids[(long long)b * T + left + i];
    v = row[tok];
  }
  __syncthreads();
  if (i < nprev) row[tok] = v < 0.f ? v * penalty : v / penalty;
}

// ------------------------------------------------------------------ sampling
constexpr int DS_T = 1024;          // threads per row
constexpr int DS_E = 32;            // elements per thread (V <= 32768)

__device__ __forceinline__ unsigned fkey(float x) {     // order-preserving float -> uint
  const unsigned u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Thread t holds vocabulary entries t + 1024 e (e < 32): coalesced row loads, and index order = (e, t).
__global__ __launch_bounds__(1024) void dec_sample_kernel(const float* __restrict__ logits, long long ldl, int V,
                                                          const int* __restrict__ row_map, long long* __restrict__ out_ids,
                                                          int T, const int* __restrict__ cur,
                                                          unsigned char* __restrict__ live, int end_token,
                                                          float temperature, int top_k, float top_p, uint64_t seed,
                                                          int* __restrict__ live_count) {
  __shared__ float shf[32 * (DS_T / 64)];
  __shared__ int shi[DS_T / 64];
  __shared__ float colsum[DS_E];
  __shared__ int chosen;
  __shared__ float xchosen;
  const int r = blockIdx.x, b = row_map ? row_map[r] : r;
  if (live && !live[b]) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = *cur;
  const float* row = logits + (long long)r * ldl;
  float x[DS_E];
#pragma unroll
  for (int e = 0; e < DS_E; ++e) {
    const int i = tid + DS_T * e;
    x[e] = i < V ? row[i] : -INFINITY;
  }
  // global max and its first index
  float mx = -INFINITY;
  int mi = 0x7fffffff;
#pragma unroll
  for (int e = 0; e < DS_E; ++e)
    if (x[e] > mx) { mx = x[e]; mi = tid + DS_T * e; }
  {
    float m2 = wave_max(mx);
    int i2 = (mx == m2) ? mi : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) i2 = min(i2, __shfl_xor(i2, o, 64));
    __syncthreads();
    if (lane == 0) { shf[w] = m2; shi[w] = i2; }
    __syncthreads();
    float bm = -INFINITY;
    int bi = 0x7fffffff;
    for (int k = 0; k < DS_T / 64; ++k) {
      if (shf[k] > bm) { bm = shf[k]; bi = shi[k]; }
      else if (shf[k] == bm) bi = min(bi, shi[k]);
    }
    mx = bm;
    mi = bi;
  }
  long long token;
  if (temperature <= 0.f || top_k == 1) {          // generation.py:44-45 (max over the row)
    token = mi;
  } else {
    const float invt = 1.0f / temperature;         // :49
#pragma unroll
    for (int e = 0; e < DS_E; ++e) x[e] *= invt;
    const float mt = mx * invt;
    bool keep[DS_E];
#pragma unroll
    for (int e = 0; e < DS_E; ++e) keep[e] = x[e] > -INFINITY;
    if (top_k > 0) {                               // :52-54, threshold = k-th largest (radix bisection)
      unsigned thr = 0;
      for (int bit = 31; bit >= 0; --bit) {
        const unsigned cand = thr | (1u << bit);
        int cnt = 0;
#pragma unroll
        for (int e = 0; e < DS_E; ++e) cnt += (keep[e] && fkey(x[e]) >= cand) ? 1 : 0;
        cnt = (int)block_sum<DS_T / 64>((float)cnt, shf);
        if (cnt >= top_k) thr = cand;
      }
#pragma unroll
      for (int e = 0; e < DS_E; ++e) keep[e] = keep[e] && fkey(x[e]) >= thr;
    }
    float q[DS_E];
    float qs = 0.f;
#pragma unroll
    for (int e = 0; e < DS_E; ++e) {
      q[e] = keep[e] ? __expf(x[e] - mt) : 0.f;
      qs += q[e];
    }
    const float Q = block_sum<DS_T / 64>(qs, shf);
    if (top_p < 1.0f) {                            // :58-66, nucleus: keep p_i with mass(p >= p_i) <= top_p
      const float lim = top_p * Q;
      unsigned lo = 0, hi = 0x7f800000u;           // smallest bit pattern u with S(u) <= lim
      while (lo < hi) {
        const unsigned mid = lo + ((hi - lo) >> 1);
        const float v = __uint_as_float(mid);
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < DS_E; ++e) s += (q[e] >= v && q[e] > 0.f) ? q[e] : 0.f;
        s = block_sum<DS_T / 64>(s, shf);
        if (s <= lim) hi = mid; else lo = mid + 1;
      }
      const float v = __uint_as_float(lo);
#pragma unroll
      for (int e = 0; e < DS_E; ++e) {
        const bool k2 = (q[e] >= v && q[e] > 0.f) || (tid + DS_T * e == mi);   // the most probable stays (:63)
        if (!k2) q[e] = 0.f;
      }
    }
    // multinomial (:68): u in [0, sum q); column sums over t for each e, then a scan inside the hit column
    float cs[DS_E];
#pragma unroll
    for (int e = 0; e < DS_E; ++e) cs[e] = wave_sum(q[e]);
    __syncthreads();
    if (lane == 0)
#pragma unroll
      for (int e = 0; e < DS_E; ++e) shf[w * DS_E + e] = cs[e];
    __syncthreads();
    if (tid < DS_E) {
      float s = 0.f;
      for (int k = 0; k < DS_T / 64; ++k) s += shf[k * DS_E + tid];
      colsum[tid] = s;
    }
    __syncthreads();
    float tot = 0.f;
    for (int e = 0; e < DS_E; ++e) tot += colsum[e];
    const float u = rand_uniform(seed, (uint64_t)c * 0x100000000ull + (uint64_t)b) * tot;
    int ec = DS_E - 1;
    float before = 0.f;
    for (int e = 0; e < DS_E; ++e) {
      if (u < before + colsum[e] || e == DS_E - 1) { ec = e; break; }
      before += colsum[e];
    }
    // column ec: inclusive scan over t of q[ec] (wave scan + wave offsets)
    float mine = 0.f;
#pragma unroll
    for (int e = 0; e < DS_E; ++e)
      if (e == ec) mine = q[e];
    float inc = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float t2 = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t2;
    }
    __syncthreads();
    if (lane == 63) shf[w] = inc;
    __syncthreads();
    float off = before;
    for (int k = 0; k < w; ++k) off += shf[k];
    const bool hit = mine > 0.f && u >= off + inc - mine && u < off + inc;
    if (tid == 0) chosen = -1;
    __syncthreads();
    if (hit) atomicMax(&chosen, tid + DS_T * ec);
    __syncthreads();
    if (chosen < 0) {                             // u fell in a rounding gap: take the last kept element
      int last = -1;
#pragma unroll
      for (int e = 0; e < DS_E; ++e)
        if (q[e] > 0.f) last = max(last, tid + DS_T * e);
      if (last >= 0) atomicMax(&chosen, last);
      __syncthreads();
    }
    const int pick = chosen;
    token = pick;
    if (top_k > 0 && top_p < 1.0f) {
      // generation.py:53-60 re-binds token_ids to the sort permutation of the top-k values, so the reference
      // emits the sampled element's rank among the top k (descending), not its vocabulary id.
#pragma unroll
      for (int e = 0; e < DS_E; ++e)
        if (tid + DS_T * e == pick) xchosen = x[e];
      __syncthreads();
      const float xsel = xchosen;
      int gt = 0;
#pragma unroll
      for (int e = 0; e < DS_E; ++e)
        gt += (keep[e] && (x[e] > xsel || (x[e] == xsel && tid + DS_T * e < pick))) ? 1 : 0;
      token = (long long)block_sum<DS_T / 64>((float)gt, shf);
    }
  }
  if (tid == 0) {
    out_ids[(long long)b * T + c] = token;           // :71
    const bool cont = token != end_token && c + 1 < T;   // :73-74 (current_index incremented first)
    if (live && !cont) {
      live[b] = 0;
      if (live_count) atomicSub(live_count, 1);
    }
  }
}

__global__ void dec_advance_kernel(int* cur) { *cur += 1; }

}  // namespace

SVAE_EXPORT int svae_dec_linear(const float* X, int64_t ldx, const float* W, int64_t ldw, const float* bias, float* Y,
                                int64_t ldy, const float* resid, int64_t ldr, int32_t M, int32_t N, int32_t K,
                                int32_t epi, const float* rot_tab, int32_t rot_cols, int32_t rot_d, const int32_t* cur,
                                float* part_ws, int64_t part_elems, svae_stream_t stream) {
  if (!X || !W || !Y || M <= 0 || N <= 0 || K <= 0 || K % 4 || ldx % 4 || ldw % 4) return SVAE_EINVAL;
  if (((uintptr_t)X | (uintptr_t)W) & 15) return SVAE_EINVAL;
  if (epi == SVAE_EPI_ROTARY_BF16 && (!rot_tab || !cur || rot_d <= 0 || rot_d % 2 || rot_cols % 2)) return SVAE_EINVAL;
  if (epi != SVAE_EPI_F32 && epi != SVAE_EPI_GELU && epi != SVAE_EPI_ROTARY_BF16) return SVAE_EINVAL;
  const int cols = (N + 15) / 16, mblk = (M + DL_MROWS - 1) / DL_MROWS;
  // split K over workgroups until ~512 workgroups are in flight (slices of >= 256 K-elements), if a workspace
  // of splits * M * N floats was given
  int splits = 1;
  while (splits < 16 && (long long)cols * mblk * splits * 2 <= 512 && K / (splits * 2) >= 256 &&
         part_ws && (long long)splits * 2 * M * N <= part_elems)
    splits *= 2;
  DL p;
  p.X = X; p.ldx = ldx; p.W = W; p.ldw = ldw; p.bias = bias; p.Y = Y; p.ldy = ldy; p.resid = resid; p.ldr = ldr;
  p.M = M; p.N = N; p.K = K; p.kslice = ((K + splits - 1) / splits + 15) / 16 * 16;
  p.rot = rot_tab; p.rot_cols = rot_cols; p.rot_d = rot_d; p.cur = cur;
  p.part = splits > 1 ? part_ws : nullptr;
  dim3 grid(cols, mblk, splits);
  hipStream_t s = (hipStream_t)stream;
  const int fin_blocks = (M * ((N + 1) / 2) + 255) / 256;
#define SVAE_DL_CASE(E)                                                                               \
  case E:                                                                                             \
    hipLaunchKernelGGL((dec_linear_kernel<E>), grid, dim3(1024), 0, s, p);                            \
    if (splits > 1) hipLaunchKernelGGL((dec_linear_finalize_kernel<E>), dim3(fin_blocks), dim3(256), 0, s, p, splits); \
    break;
  switch (epi) {
    SVAE_DL_CASE(SVAE_EPI_F32)
    SVAE_DL_CASE(SVAE_EPI_GELU)
    SVAE_DL_CASE(SVAE_EPI_ROTARY_BF16)
  }
#undef SVAE_DL_CASE
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_dec_attn(const float* qkv, int64_t ldq, float* kcache, float* vcache, int32_t B, int32_t H,
                              int32_t hd, int32_t T, const int32_t* cur, int32_t window, float scale, float* O,
                              int64_t ldo, svae_stream_t stream) {
  if (!qkv || !kcache || !vcache || !cur || !O || B <= 0 || H <= 0 || T <= 0) return SVAE_EINVAL;
  if (hd <= 0 || hd > 128 || hd % 4 || window < 0 || T > 32768) return SVAE_EINVAL;
  if ((((uintptr_t)kcache | (uintptr_t)vcache) & 15) || ldq % 4) return SVAE_EINVAL;
  hipLaunchKernelGGL(dec_attn_kernel, dim3(H, B), dim3(DA_THREADS), (size_t)T * sizeof(float), (hipStream_t)stream, qkv, ldq,
                     kcache, vcache, H, hd, T, cur, window, scale, O, ldo);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_dec_embed(const int64_t* out_ids, int32_t T, const int32_t* cur, const float* table, float* x,
                               int32_t B, int32_t D, svae_stream_t stream) {
  if (!out_ids || !cur || !table || !x || B <= 0 || D <= 0 || D % 4) return SVAE_EINVAL;
  hipLaunchKernelGGL(dec_embed_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     (const long long*)out_ids, T, cur, table, x, B, D);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_dec_penalty(float* logits, int64_t ldl, int32_t rows, const int32_t* row_map,
                                 const int64_t* out_ids, int32_t T, const int32_t* cur, const uint8_t* live,
                                 float penalty, svae_stream_t stream) {
  if (!logits || !out_ids || !cur || rows <= 0 || T <= 0) return SVAE_EINVAL;
  hipLaunchKernelGGL(dec_penalty_kernel, dim3(rows), dim3(512), 0, (hipStream_t)stream, logits, ldl, row_map,
                     (const long long*)out_ids, T, cur, live, penalty);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_dec_sample(const float* logits, int64_t ldl, int32_t V, int32_t rows, const int32_t* row_map,
                                int64_t* out_ids, int32_t T, const int32_t* cur, uint8_t* live, int32_t end_token,
                                float temperature, int32_t top_k, float top_p, uint64_t seed, int32_t* live_count,
                                svae_stream_t stream) {
  if (!logits || !out_ids || !cur || rows <= 0 || V <= 0 || V > DS_T * DS_E || T <= 0) return SVAE_EINVAL;
  hipLaunchKernelGGL(dec_sample_kernel, dim3(rows), dim3(DS_T), 0, (hipStream_t)stream, logits, ldl, V, row_map,
                     (long long*)out_ids, T, cur, live, end_token, temperature, top_k, top_p, seed, live_count);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_dec_advance(int32_t* cur, svae_stream_t stream) {
  if (!cur) return SVAE_EINVAL;
  hipLaunchKernelGGL(dec_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, cur);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}
