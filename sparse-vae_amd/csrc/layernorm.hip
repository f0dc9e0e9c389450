// LayerNorm (eps 1e-5, affine) forward / backward, one wave64 per row, and the column-sum reduction used
// for bias / LayerNorm-affine gradients.
//
// Reference: nn.LayerNorm(d) in TransformerLayer (transformer_layer.py:23-24, 39-40, 47, 52, 56) and the
// output head (transformer_language_model.py:59). HBM-bound: forward moves 4d (f32 in) + 2d (bf16 out)
// bytes per row; backward reads dy (2d), x (4d), dres (4d) and writes dx (4d + 2d).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "../../include/svae.h"

using namespace svae;

namespace {

// MAXV = float4 chunks per lane: D <= 64 * 4 * MAXV (instantiated for 2, 3, 4: D <= 512 / 768 / 1024, so the
// per-lane arrays, and the registers, fit the model width: the D <= 1024 copy held 112-136 VGPRs, 3-4 waves / SIMD)

template <typename T>
__device__ __forceinline__ f32x4 load4(const T* p);
template <>
__device__ __forceinline__ f32x4 load4<float>(const float* p) { return *(const f32x4*)p; }
template <>
__device__ __forceinline__ f32x4 load4<bf16>(const bf16* p) {
  bf16x4 v = *(const bf16x4*)p;
  return (f32x4){(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
__device__ __forceinline__ void store4_bf(bf16* p, f32x4 v) {
  *(bf16x4*)p = (bf16x4){f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
}

// column of the lane's k-th float4 in a row: even MAXV = runs of 8 columns (two float4 each), odd = runs of 4
template <int MAXV>
__device__ __forceinline__ int ln_col(int lane, int k) {
  return MAXV % 2 == 0 ? (lane + 64 * (k >> 1)) * 8 + 4 * (k & 1) : (lane + 64 * k) * 4;
}
template <typename T, int MAXV>
__device__ __forceinline__ void ln_load_row(const T* __restrict__ xr, int lane, int D, f32x4 (&dst)[MAXV]) {
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int c = ln_col<MAXV>(lane, k);
    dst[k] = (c < D) ? load4<T>(xr + c) : (f32x4){0.f, 0.f, 0.f, 0.f};
  }
}

// y = bf16((v - mean) * rstd * w + b) of one row held by a wave (the ln_col layout of MAXV)
template <int MAXV>
__device__ __forceinline__ void ln_store_row(const f32x4 (&v)[MAXV], float mean, float rstd, const float* __restrict__ w,
                                             const float* __restrict__ b, bf16* __restrict__ yr, int lane, int D) {
  if constexpr (MAXV % 2 == 0) {
#pragma unroll
    for (int j = 0; j < MAXV / 2; ++j) {
      const int c = ln_col<MAXV>(lane, 2 * j);
      if (c < D) {
        bf16x8 o;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 ww = *(const f32x4*)(w + c + 4 * h), bb = *(const f32x4*)(b + c + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) o[4 * h + e] = f2bf((v[2 * j + h][e] - mean) * rstd * ww[e] + bb[e]);
        }
        *(bf16x8*)(yr + c) = o;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int c = ln_col<MAXV>(lane, k);
      if (c < D) {
        const f32x4 ww = *(const f32x4*)(w + c), bb = *(const f32x4*)(b + c);
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (v[k][e] - mean) * rstd * ww[e] + bb[e];
        store4_bf(yr + c, o);
      }
    }
  }
}

// A wave walks rows wave, wave + waves, ... (the launcher sizes the grid so a few rows fall to each wave) with the
// next row's loads issued before the current row's reductions and stores: the loads stay in flight across rows
// instead of one load round trip per wave launch.
// ZR (f32 x only): rows r % zmod == 0 are taken from zrows[r / zmod] and written into x (xw) -- the z splice of
// transformer_vae.py:89-90 applied by the layer's first LayerNorm, so the z projections of all layers run as one
// launch ahead of the decoder
template <typename T, int MAXV, bool ZR = false>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ b, bf16* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int rows, int D, const float* __restrict__ zrows = nullptr,
                                                     int zmod = 0, float* __restrict__ xw = nullptr) {
  // even MAXV: D % 8 == 0 (checked by the launcher), each lane owns runs of 8 consecutive columns, so the bf16 output
  // is one 16-B store per run (the 4-column layout stores 8 B per lane); odd MAXV: runs of 4 columns
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * 4;
  int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  f32x4 v[MAXV], vn[MAXV];
  auto src = [&](int r) -> const T* {
    if constexpr (ZR) {
      if (r % zmod == 0) return (const T*)(zrows + (long long)(r / zmod) * D);
    }
    return x + (long long)r * D;
  };
  ln_load_row<T, MAXV>(src(row), lane, D, v);
#pragma nounroll
  while (true) {
    const int next = row + nw;
    if (next < rows) ln_load_row<T, MAXV>(src(next), lane, D, vn);
    if constexpr (ZR) {
      if (row % zmod == 0) {   // the spliced row into x (the residual stream)
#pragma unroll
        for (int k = 0; k < MAXV; ++k) {
          const int c = ln_col<MAXV>(lane, k);
          if (c < D) *(f32x4*)(xw + (long long)row * D + c) = v[k];
        }
      }
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) s += (v[k][0] + v[k][1]) + (v[k][2] + v[k][3]);
    const float mean = wave_sum(s) / D;
    float sq = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const bool in = ln_col<MAXV>(lane, k) < D;
#pragma unroll
      for (int e = 0; e < 4; ++e) { const float t = in ? v[k][e] - mean : 0.f; sq += t * t; }
    }
    const float rstd = rsqrtf(wave_sum(sq) / D + 1e-5f);
    ln_store_row<MAXV>(v, mean, rstd, w, b, y + (long long)row * D, lane, D);
    if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
    if (next >= rows) break;
    for (int k = 0; k < MAXV; ++k) v[k] = vn[k];   // (register renames once unrolled by the optimiser)
    row = next;
  }
}

// Residual add + dropout + LayerNorm, fused (the TransformerLayer's "x = x + y" followed by the next LayerNorm,
// transformer_layer.py:49-50 / :56 and :58-61 + the next layer's :47): one wave per row, 8 consecutive columns per lane.
//   v = x[r] + dropout(y[r])          (x may be NULL: no residual; y f32 or bf16, the projection GEMM's output; dropout with the
//                                      counter RNG of the GEMM epilogues: index (r * D + c) / 4, keep u >= p, scale 1/(1-p))
//   v = zrows[r / zmod]  when zrows and r % zmod == 0   (the z splice of transformer_vae.py:89-90)
//   xo[r] = v (f32, when xo); h[r] = LN(v) * w + b (bf16) and mean / rstd when w, else h[r] = bf16(v).
// Moves 14 B per element with an f32 y (x, y in; xo, h out): the residual add and the dropout leave the GEMM epilogue (which ran with
// no MFMA beside it: the f32 + residual epilogue cost 2x a bf16 store at the C2 FFN2 shape) for this HBM-bound pass.
// CPL = columns per lane per run (8: one 16-B bf16 store per run, D % 512 == 0 fills every lane; 4: D = 768 as 3 runs of
// 256 columns, every lane busy -- the 8-column layout left half the lanes idle in its second run), NR runs.
template <int NR, int CPL, typename TY>
__global__ __launch_bounds__(256) void resid_ln_fwd_kernel(const float* __restrict__ x, const TY* __restrict__ y,
                                                           long long ldy, float drop_p, unsigned long long seed,
                                                           const float* __restrict__ zrows, int zmod,
                                                           const float* __restrict__ w, const float* __restrict__ b,
                                                           float* __restrict__ xo, bf16* __restrict__ h,
                                                           float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                           int rows, int D) {
  constexpr int NV = CPL / 4;                    // f32x4 per run
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bool zr = zrows && row % zmod == 0;      // wave-uniform
  const float sc = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  f32x4 v[NR][NV];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int c = (lane + 64 * j) * CPL;
#pragma unroll
    for (int q = 0; q < NV; ++q) v[j][q] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (c < D) {
      if (zr) {
        const float* zp = zrows + (long long)(row / zmod) * D + c;
#pragma unroll
        for (int q = 0; q < NV; ++q) v[j][q] = *(const f32x4*)(zp + 4 * q);
      } else {
        if (x) {
#pragma unroll
          for (int q = 0; q < NV; ++q) v[j][q] = *(const f32x4*)(x + (long long)row * D + c + 4 * q);
        }
        if (y) {
          float yy[CPL];
          if constexpr (sizeof(TY) == 2) {
            if constexpr (CPL == 8) {
              const bf16x8 t = *(const bf16x8*)(y + (long long)row * ldy + c);
#pragma unroll
              for (int e = 0; e < 8; ++e) yy[e] = (float)t[e];
            } else {
              const bf16x4 t = *(const bf16x4*)(y + (long long)row * ldy + c);
#pragma unroll
              for (int e = 0; e < 4; ++e) yy[e] = (float)t[e];
            }
          } else {
#pragma unroll
            for (int q = 0; q < NV; ++q) {
              const f32x4 t = *(const f32x4*)(y + (long long)row * ldy + c + 4 * q);
#pragma unroll
              for (int e = 0; e < 4; ++e) yy[4 * q + e] = t[e];
            }
          }
#pragma unroll
          for (int q = 0; q < NV; ++q) {
            float u[4] = {1.f, 1.f, 1.f, 1.f};
            if (drop_p > 0.f) rand_uniform4(seed, ((unsigned long long)row * D + c + 4 * q) >> 2, u);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float t = yy[4 * q + e];
              v[j][q][e] += drop_p > 0.f ? (u[e] >= drop_p ? t * sc : 0.f) : t;
            }
          }
        }
      }
#pragma unroll
      for (int q = 0; q < NV; ++q) s += (v[j][q][0] + v[j][q][1]) + (v[j][q][2] + v[j][q][3]);
      if (xo) {
#pragma unroll
        for (int q = 0; q < NV; ++q) *(f32x4*)(xo + (long long)row * D + c + 4 * q) = v[j][q];
      }
    }
  }
  auto store_h = [&](int c, const float (&o)[CPL]) {
    if constexpr (CPL == 8) {
      bf16x8 t;
#pragma unroll
      for (int e = 0; e < 8; ++e) t[e] = f2bf(o[e]);
      *(bf16x8*)(h + (long long)row * D + c) = t;
    } else {
      *(bf16x4*)(h + (long long)row * D + c) = (bf16x4){f2bf(o[0]), f2bf(o[1]), f2bf(o[2]), f2bf(o[3])};
    }
  };
  if (!w) {                                      // no LayerNorm: the bf16 copy of v
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int c = (lane + 64 * j) * CPL;
      if (c < D) {
        float o[CPL];
#pragma unroll
        for (int e = 0; e < CPL; ++e) o[e] = v[j][e >> 2][e & 3];
        store_h(c, o);
      }
    }
    return;
  }
  const float mean = wave_sum(s) / D;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int c = (lane + 64 * j) * CPL;
    if (c < D) {
#pragma unroll
      for (int e = 0; e < CPL; ++e) { const float t = v[j][e >> 2][e & 3] - mean; sq += t * t; }
    }
  }
  const float rstd = rsqrtf(wave_sum(sq) / D + 1e-5f);
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int c = (lane + 64 * j) * CPL;
    if (c < D) {
      float o[CPL];
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const f32x4 ww = *(const f32x4*)(w + c + 4 * q), bb = *(const f32x4*)(b + c + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) o[4 * q + e] = (v[j][q][e] - mean) * rstd * ww[e] + bb[e];
      }
      store_h(c, o);
    }
  }
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// GMUL: only the bf16 dx_bf = bf16(dx * gmul) is written (no f32 dx): the vocabulary head's LayerNorm backward fused
// with the GELU backward of the linear before it (gmul = the GELU' its forward epilogue saved)
template <typename T, int MAXV, bool GMUL = false>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const bf16* __restrict__ dy, const T* __restrict__ x,
                                                     const float* __restrict__ w, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, const float* __restrict__ dres,
                                                     float* __restrict__ dx, bf16* __restrict__ dx_bf,
                                                     float* __restrict__ part, int rows, int D, int zero_mod,
                                                     float bf_drop_p, unsigned long long bf_seed, int bf_zero_mod,
                                                     float* __restrict__ zrow, bf16* __restrict__ zrow_bf,
                                                     const bf16* __restrict__ gmul = nullptr) {
  __shared__ float red[4][2][256 * MAXV];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  f32x4 adw[MAXV], adb[MAXV];
#pragma unroll
  for (int j = 0; j < MAXV; ++j) { adw[j] = (f32x4){0.f, 0.f, 0.f, 0.f}; adb[j] = adw[j]; }
  for (int row = blockIdx.x * 4 + wave; row < rows; row += gridDim.x * 4) {
    const long long base = (long long)row * D;
    const float mean = mean_in[row], rstd = rstd_in[row];
    f32x4 xh[MAXV], g[MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      const int c = (lane + 64 * j) * 4;
      if (c < D) {
        const f32x4 xv = load4<T>(x + base + c);
        const f32x4 dv = load4<bf16>(dy + base + c);
        const f32x4 ww = *(const f32x4*)(w + c);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xh[j][e] = (xv[e] - mean) * rstd;
          g[j][e] = dv[e] * ww[e];
          s1 += g[j][e];
          s2 += g[j][e] * xh[j][e];
          adw[j][e] += dv[e] * xh[j][e];
          adb[j][e] += dv[e];
        }
      }
    }
    const float m1 = wave_sum(s1) / D, m2 = wave_sum(s2) / D;
    const bool zero = zero_mod > 0 && (row % zero_mod) == 0;
    const bool bf_zero = bf_zero_mod > 0 && (row % bf_zero_mod) == 0;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      const int c = (lane + 64 * j) * 4;
      if (c < D) {
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = rstd * (g[j][e] - m1 - xh[j][e] * m2);
        if constexpr (GMUL) {
          const f32x4 gv = load4<bf16>(gmul + base + c);
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] *= gv[e];
          store4_bf(dx_bf + base + c, o);
          continue;
        }
        if (dres) {
          const f32x4 r = *(const f32x4*)(dres + base + c);
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] += r[e];
        }
        if (zero) {   // (the row's value first goes to zrow[row / zero_mod]: the z splice's gradient)
          if (zrow) *(f32x4*)(zrow + (long long)(row / zero_mod) * D + c) = o;
          if (zrow_bf) store4_bf(zrow_bf + (long long)(row / zero_mod) * D + c, o);
          o = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
        *(f32x4*)(dx + base + c) = o;
        if (dx_bf) {
          // the bf16 copy may carry the next consumer's dropout backward (mask of the forward's DROPOUT_RESID
          // epilogue: counter (row * D + c) / 4 of bf_seed) and its position-0 zeroing
          if (bf_zero) o = (f32x4){0.f, 0.f, 0.f, 0.f};
          else if (bf_drop_p > 0.f) {
            float u[4];
            rand_uniform4(bf_seed, ((unsigned long long)row * D + c) >> 2, u);
            const float sc = 1.0f / (1.0f - bf_drop_p);
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = u[e] >= bf_drop_p ? o[e] * sc : 0.f;
          }
          store4_bf(dx_bf + base + c, o);
        }
      }
    }
  }
  // reduce the 4 waves' affine-gradient partials, write this block's slab
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int c = (lane + 64 * j) * 4;
    if (c < D) {
      *(f32x4*)&red[wave][0][c] = adw[j];
      *(f32x4*)&red[wave][1][c] = adb[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * D; c += 256) {
    const int which = c / D, col = c % D;
    const float s = red[0][which][col] + red[1][which][col] + red[2][which][col] + red[3][which][col];
    part[((long long)blockIdx.x * 2 + which) * D + col] = s;
  }
}

// The encoder middle layers' context LayerNorms: n <= SVAE_LN_MULTI_MAX affines of one normalised input
struct LnMulti {
  const float* w[SVAE_LN_MULTI_MAX];
  const float* b[SVAE_LN_MULTI_MAX];
  bf16* y[SVAE_LN_MULTI_MAX];
  const bf16* dy[SVAE_LN_MULTI_MAX];
  float* part[SVAE_LN_MULTI_MAX];
  int n;
};

// ln_fwd_kernel (f32 x, no z splice) writing m.n outputs from one read of the row: the statistics and every output
// element are computed as ln_fwd_kernel computes them (bit-identical to m.n separate passes)
template <int MAXV>
__global__ __launch_bounds__(256) void ln_fwd_multi_kernel(const float* __restrict__ x, LnMulti m,
                                                           float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                           int rows, int D) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * 4;
  int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  f32x4 v[MAXV], vn[MAXV];
  ln_load_row<float, MAXV>(x + (long long)row * D, lane, D, v);
#pragma nounroll
  while (true) {
    const int next = row + nw;
    if (next < rows) ln_load_row<float, MAXV>(x + (long long)next * D, lane, D, vn);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) s += (v[k][0] + v[k][1]) + (v[k][2] + v[k][3]);
    const float mean = wave_sum(s) / D;
    float sq = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const bool in = ln_col<MAXV>(lane, k) < D;
#pragma unroll
      for (int e = 0; e < 4; ++e) { const float t = in ? v[k][e] - mean : 0.f; sq += t * t; }
    }
    const float rstd = rsqrtf(wave_sum(sq) / D + 1e-5f);
#pragma unroll
    for (int j = 0; j < SVAE_LN_MULTI_MAX; ++j)
      if (j < m.n) ln_store_row<MAXV>(v, mean, rstd, m.w[j], m.b[j], m.y[j] + (long long)row * D, lane, D);
    if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
    if (next >= rows) break;
    for (int k = 0; k < MAXV; ++k) v[k] = vn[k];
    row = next;
  }
}

// m.n LayerNorm backwards of one input in one pass (ln_bwd_kernel's row program): LN' is linear in g = dy * w, so
// dx = dres + rstd (G - mean(G) - xh mean(G xh)) with G = sum_j dy[j] * w[j]; the affine partials per LayerNorm j
// (sum dy[j] * xh, sum dy[j]) into m.part[j]. Moves 4 (x) + 2 n (dy) + 8 (dres, dx) bytes per element instead of
// n (2 + 4 + 8). (dres may alias dx: no __restrict__.)
template <int MAXV>
__global__ __launch_bounds__(256) void ln_bwd_multi_kernel(LnMulti m, const float* __restrict__ x,
                                                           const float* __restrict__ mean_in,
                                                           const float* __restrict__ rstd_in, const float* dres,
                                                           float* dx, int rows, int D) {
  constexpr int NM = SVAE_LN_MULTI_MAX;
  __shared__ float red[4][2][256 * MAXV];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  f32x4 adw[NM][MAXV], adb[NM][MAXV];
#pragma unroll
  for (int i = 0; i < NM; ++i)
#pragma unroll
    for (int j = 0; j < MAXV; ++j) { adw[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f}; adb[i][j] = adw[i][j]; }
  // a row's inputs, loaded one row ahead (two rows' loads in flight per wave: at 192+ VGPRs two waves per SIMD fit, and
  // one row in flight per wave ran the four-LayerNorm pass at 2.7 TB/s)
  struct RowIn {
    f32x4 xv[MAXV], rr[MAXV];
    bf16x4 dv[NM][MAXV];
    float mean, rstd;
  };
  auto load_row = [&](int row, RowIn& in) {
    const long long base = (long long)row * D;
    in.mean = mean_in[row];
    in.rstd = rstd_in[row];
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      const int c = (lane + 64 * j) * 4;
      const bool ok = c < D;
      in.xv[j] = ok ? *(const f32x4*)(x + base + c) : (f32x4){0.f, 0.f, 0.f, 0.f};
      in.rr[j] = ok && dres ? *(const f32x4*)(dres + base + c) : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        if (i >= m.n) break;
        in.dv[i][j] = ok ? *(const bf16x4*)(m.dy[i] + base + c) : (bf16x4){};
      }
    }
  };
  const int stride = gridDim.x * 4;
  int row = blockIdx.x * 4 + wave;
  RowIn cur, nxt;
  if (row < rows) load_row(row, cur);
  for (; row < rows; row += stride) {
    if (row + stride < rows) load_row(row + stride, nxt);
    const long long base = (long long)row * D;
    const float mean = cur.mean, rstd = cur.rstd;
    f32x4 xh[MAXV], g[MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      const int c = (lane + 64 * j) * 4;
      g[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      xh[j] = g[j];
      if (c < D) {
#pragma unroll
        for (int e = 0; e < 4; ++e) xh[j][e] = (cur.xv[j][e] - mean) * rstd;
#pragma unroll
        for (int i = 0; i < NM; ++i) {
          if (i >= m.n) break;
          const f32x4 ww = *(const f32x4*)(m.w[i] + c);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float dv = (float)cur.dv[i][j][e];
            g[j][e] += dv * ww[e];
            adw[i][j][e] += dv * xh[j][e];
            adb[i][j][e] += dv;
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) { s1 += g[j][e]; s2 += g[j][e] * xh[j][e]; }
      }
    }
    const float m1 = wave_sum(s1) / D, m2 = wave_sum(s2) / D;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      const int c = (lane + 64 * j) * 4;
      if (c < D) {
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = rstd * (g[j][e] - m1 - xh[j][e] * m2) + cur.rr[j][e];
        *(f32x4*)(dx + base + c) = o;
      }
    }
    cur = nxt;
  }
  // per LayerNorm: reduce the 4 waves' affine partials, write this block's slab of m.part[i]
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    if (i >= m.n) break;
    if (i > 0) __syncthreads();   // (the previous LayerNorm's reads of red are done)
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      const int c = (lane + 64 * j) * 4;
      if (c < D) {
        *(f32x4*)&red[wave][0][c] = adw[i][j];
        *(f32x4*)&red[wave][1][c] = adb[i][j];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 2 * D; c += 256) {
      const int which = c / D, col = c % D;
      const float s = red[0][which][col] + red[1][which][col] + red[2][which][col] + red[3][which][col];
      m.part[i][((long long)blockIdx.x * 2 + which) * D + col] = s;
    }
  }
}

// out[j] += sum_i in[i*ld + j]. Block = 64 columns (16 column threads x 4) x 16 row threads, grid (column blocks,
// row splits): every thread keeps 8 rows' loads in flight, the block reduces its 16 row threads in LDS and adds
// its 64 sums with one atomic each. (Row-wave blocks with a serial row loop ran 7.9 us on the LayerNorm slabs'
// 1024 x 1024 floats; with 4x the splits, 8.6 us: same-address atomics from many blocks serialise.)
template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const T* __restrict__ in, int rows, int cols, long long ld,
                                                     float* __restrict__ out, int rows_per_split) {
  __shared__ f32x4 red[16][17];
  const int ct = threadIdx.x & 15, rt = threadIdx.x >> 4;
  const int c = (blockIdx.x * 16 + ct) * 4;
  const int r0 = blockIdx.y * rows_per_split;
  const int r1 = min(rows, r0 + rows_per_split);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
    int r = r0 + rt;
    for (; r + 112 < r1; r += 128) {
      f32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = load4<T>(in + (long long)(r + 16 * i) * ld + c);
      acc += ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
    }
    for (; r < r1; r += 16) acc += load4<T>(in + (long long)r * ld + c);
  }
  red[rt][ct] = acc;
  __syncthreads();
  if (threadIdx.x < 16 && c < cols) {
    f32x4 s = red[0][ct];
#pragma unroll
    for (int i = 1; i < 16; ++i) s += red[i][ct];
#pragma unroll
    for (int e = 0; e < 4; ++e) atomicAdd(out + c + e, s[e]);
  }
}

// Up to SVAE_COLSUM_MAX f32 column sums in one launch (the LayerNorm backwards of one layer: one launch instead of
// one per LayerNorm, each ~1.6 us of launch cost for ~1 us of work). Segment s owns blocks [first[s], first[s+1]).
struct ColsumSegs {
  const float* in[SVAE_COLSUM_MAX];
  float* out[SVAE_COLSUM_MAX];
  long long ld[SVAE_COLSUM_MAX];
  int rows[SVAE_COLSUM_MAX], cols[SVAE_COLSUM_MAX], rps[SVAE_COLSUM_MAX], colblocks[SVAE_COLSUM_MAX];
  int first[SVAE_COLSUM_MAX + 1];
  int n;
};
__global__ __launch_bounds__(256) void colsum_multi_kernel(ColsumSegs sg) {
  __shared__ f32x4 red[16][17];
  int sgi = 0;
  while (sgi + 1 < sg.n && (int)blockIdx.x >= sg.first[sgi + 1]) ++sgi;   // (block-uniform, <= 8 steps)
  const int local = blockIdx.x - sg.first[sgi];
  const int cb = local % sg.colblocks[sgi], split = local / sg.colblocks[sgi];
  const float* in = sg.in[sgi];
  const int rows = sg.rows[sgi], cols = sg.cols[sgi];
  const long long ld = sg.ld[sgi];
  const int ct = threadIdx.x & 15, rt = threadIdx.x >> 4;
  const int c = (cb * 16 + ct) * 4;
  const int r0 = split * sg.rps[sgi];
  const int r1 = min(rows, r0 + sg.rps[sgi]);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
    int r = r0 + rt;
    for (; r + 112 < r1; r += 128) {
      f32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = *(const f32x4*)(in + (long long)(r + 16 * i) * ld + c);
      acc += ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
    }
    for (; r < r1; r += 16) acc += *(const f32x4*)(in + (long long)r * ld + c);
  }
  red[rt][ct] = acc;
  __syncthreads();
  if (threadIdx.x < 16 && c < cols) {
    f32x4 s = red[0][ct];
#pragma unroll
    for (int i = 1; i < 16; ++i) s += red[i][ct];
#pragma unroll
    for (int e = 0; e < 4; ++e) atomicAdd(sg.out[sgi] + c + e, s[e]);
  }
}

// grid of one column sum (shared by svae_colsum and svae_colsum_multi): ~256 blocks, >= 128 rows per split
static void colsum_grid(int rows, int cols, int& colblocks, int& splits, int& rps) {
  colblocks = (cols + 63) / 64;
  splits = (256 + colblocks - 1) / colblocks;
  const int max_splits = (rows + 127) / 128;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  rps = (rows + splits - 1) / splits;
  splits = (rows + rps - 1) / rps;
}

}  // namespace

SVAE_EXPORT int svae_colsum_multi(const svae_colsum_seg* segs, int32_t n, svae_stream_t stream) {
  if (!segs || n <= 0 || n > SVAE_COLSUM_MAX) return SVAE_EINVAL;
  ColsumSegs sg;
  sg.n = n;
  int total = 0;
  for (int i = 0; i < n; ++i) {
    const svae_colsum_seg& q = segs[i];
    if (!q.in || !q.out || q.rows <= 0 || q.cols <= 0 || q.cols % 4 || q.ld % 4) return SVAE_EINVAL;
    if (((uintptr_t)q.in | (uintptr_t)q.out) & 15) return SVAE_EINVAL;
    int cb, sp, rps;
    colsum_grid(q.rows, q.cols, cb, sp, rps);
    sg.in[i] = q.in; sg.out[i] = q.out; sg.ld[i] = q.ld;
    sg.rows[i] = q.rows; sg.cols[i] = q.cols; sg.rps[i] = rps; sg.colblocks[i] = cb;
    sg.first[i] = total;
    total += cb * sp;
  }
  sg.first[n] = total;
  hipLaunchKernelGGL(colsum_multi_kernel, dim3((unsigned)total), dim3(256), 0, (hipStream_t)stream, sg);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_layernorm_fwd(const void* x, int32_t x_dtype, const float* w, const float* b, void* y,
                                   float* mean, float* rstd, int32_t rows, int32_t D, svae_stream_t stream) {
  if (!x || !w || !b || !y || !mean || !rstd || rows <= 0 || D <= 0 || D % 4 || D > 1024) return SVAE_EINVAL;
  // rows per wave: the grid holds at most SVAE_LN_FWD_BLOCKS blocks of 4 waves (0: one row per wave)
  // (default: 2048 blocks for D <= 512, 1024 above -- where 2048 measured slower with the 8-column layout)
  static const int cap_env = [] { const char* e = getenv("SVAE_LN_FWD_BLOCKS"); return e ? atoi(e) : -1; }();
  static const int c4 = [] { const char* e = getenv("SVAE_LN_FWD_4COL"); return e ? atoi(e) : 1; }();
  // (the 4-column layout at 512 < D <= 768 runs 2048 blocks too)
  const int cap = cap_env >= 0 ? cap_env : ((D <= 512 || (c4 && D <= 768)) ? 2048 : 1024);
  const int need = (rows + 3) / 4;
  dim3 grid((unsigned)(cap > 0 ? std::min(need, cap) : need));
  hipStream_t s = (hipStream_t)stream;
#define SVAE_LN_FWD(MV)                                                                                            \
  do {                                                                                                             \
    if (x_dtype == 0)                                                                                              \
      hipLaunchKernelGGL((ln_fwd_kernel<float, MV>), grid, dim3(256), 0, s, (const float*)x, w, b, (bf16*)y, mean, \
                         rstd, rows, D);                                                                           \
    else                                                                                                           \
      hipLaunchKernelGGL((ln_fwd_kernel<bf16, MV>), grid, dim3(256), 0, s, (const bf16*)x, w, b, (bf16*)y, mean,   \
                         rstd, rows, D);                                                                           \
  } while (0)
  // (even MAXV = the 8-column layout, which needs D % 8 == 0 and 16-B aligned rows. The 4-column layout for 512 < D <=
  // 768 (SVAE_LN_FWD_4COL=0 turns it off): every lane busy in every run; with 2048 blocks the C4 / C5 row shape runs
  // 59.7 -> 55.5 us, its z-splice form 76 -> 62.6 us (profiles/r05ln_ln_fwd_probe.log). Round 5 kept it off because its
  // other fp32 summation order moved an encoder k_linear weight gradient's norm ratio to 0.979 against a 2 % bar; that bar
  // sat inside the bf16 noise floor of those gradients (sigma 1.4-2.0 %, tests/golden/noise_floor_c4shape.json), and on
  // that floor the 4-column build is no less accurate: norm-ratio deviations rms 0.56-0.79 sigma against 0.61-0.98 for
  // the 8-column one over the C2 / C4 / C5 step-parity cases (profiles/r06m_ln4col_parity.log))
  if (c4 && D > 512 && D <= 768) SVAE_LN_FWD(3);
  else if (D % 8 == 0 && D <= 512) SVAE_LN_FWD(2);
  else if (D % 8 == 0) SVAE_LN_FWD(4);
  else if (D <= 768) SVAE_LN_FWD(3);
  else SVAE_LN_FWD(5);
#undef SVAE_LN_FWD
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_layernorm_fwd_z(float* x, const float* zrows, int32_t zmod, const float* w, const float* b, void* y,
                                     float* mean, float* rstd, int32_t rows, int32_t D, svae_stream_t stream) {
  if (!x || !zrows || zmod <= 0 || !w || !b || !y || !mean || !rstd || rows <= 0 || D <= 0 || D % 8 || D > 1024)
    return SVAE_EINVAL;
  if (((uintptr_t)x | (uintptr_t)zrows) & 15) return SVAE_EINVAL;
  // (default: 2048 blocks for D <= 512, 1024 above -- where 2048 measured slower with the 8-column layout)
  static const int cap_env = [] { const char* e = getenv("SVAE_LN_FWD_BLOCKS"); return e ? atoi(e) : -1; }();
  static const int c4 = [] { const char* e = getenv("SVAE_LN_FWD_4COL"); return e ? atoi(e) : 1; }();
  // (the 4-column layout at 512 < D <= 768 runs 2048 blocks too)
  const int cap = cap_env >= 0 ? cap_env : ((D <= 512 || (c4 && D <= 768)) ? 2048 : 1024);
  const int need = (rows + 3) / 4;
  dim3 grid((unsigned)(cap > 0 ? std::min(need, cap) : need));
  hipStream_t s = (hipStream_t)stream;
  if (D <= 512)
    hipLaunchKernelGGL((ln_fwd_kernel<float, 2, true>), grid, dim3(256), 0, s, (const float*)x, w, b, (bf16*)y, mean,
                       rstd, rows, D, zrows, zmod, x);
  else if (c4 && D <= 768)
    hipLaunchKernelGGL((ln_fwd_kernel<float, 3, true>), grid, dim3(256), 0, s, (const float*)x, w, b, (bf16*)y, mean,
                       rstd, rows, D, zrows, zmod, x);
  else
    hipLaunchKernelGGL((ln_fwd_kernel<float, 4, true>), grid, dim3(256), 0, s, (const float*)x, w, b, (bf16*)y, mean,
                       rstd, rows, D, zrows, zmod, x);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_resid_ln_fwd(const float* x, const void* y, int32_t y_dtype, int64_t ldy, float drop_p,
                                  uint64_t seed, const float* zrows, int32_t zmod, const float* w, const float* b,
                                  float* xo, void* h, float* mean, float* rstd, int32_t rows, int32_t D,
                                  svae_stream_t stream) {
  if (!h || rows <= 0 || D <= 0 || D % 8 || D > 1024 || (!x && !y && !zrows) || (y_dtype != 0 && y_dtype != 1))
    return SVAE_EINVAL;
  if ((w == nullptr) != (b == nullptr) || (w && (!mean || !rstd)) || (zrows && zmod <= 0)) return SVAE_EINVAL;
  if (drop_p < 0.f || drop_p >= 1.f || (y && ldy % 8) || (((uintptr_t)y | (uintptr_t)h) & 15)) return SVAE_EINVAL;
  // x, xo, zrows, w, b are read / written as f32x4 rows of stride D: 16-byte aligned
  if (((uintptr_t)x | (uintptr_t)xo | (uintptr_t)zrows | (uintptr_t)w | (uintptr_t)b) & 15) return SVAE_EINVAL;
  dim3 grid((rows + 3) / 4);
  hipStream_t s = (hipStream_t)stream;
#define SVAE_RLN(NR, CPL, TY)                                                                                     \
  hipLaunchKernelGGL((resid_ln_fwd_kernel<NR, CPL, TY>), grid, dim3(256), 0, s, x, (const TY*)y, (long long)ldy,     \
                     drop_p, (unsigned long long)seed, zrows, zmod, w, b, xo, (bf16*)h, mean, rstd, rows, D)
  if (D <= 512) {
    if (y_dtype == 0) SVAE_RLN(1, 8, float); else SVAE_RLN(1, 8, bf16);
  } else if (D <= 768) {
    if (y_dtype == 0) SVAE_RLN(3, 4, float); else SVAE_RLN(3, 4, bf16);
  } else {
    if (y_dtype == 0) SVAE_RLN(2, 8, float); else SVAE_RLN(2, 8, bf16);
  }
#undef SVAE_RLN
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_layernorm_fwd_multi(const float* x, const float* const* w, const float* const* b, void* const* y,
                                         int32_t n, float* mean, float* rstd, int32_t rows, int32_t D,
                                         svae_stream_t stream) {
  if (!x || !w || !b || !y || !mean || !rstd || n <= 0 || n > SVAE_LN_MULTI_MAX || rows <= 0 || D <= 0 || D % 4 ||
      D > 1024)
    return SVAE_EINVAL;
  LnMulti m = {};
  m.n = n;
  for (int i = 0; i < n; ++i) {
    if (!w[i] || !b[i] || !y[i]) return SVAE_EINVAL;
    m.w[i] = w[i]; m.b[i] = b[i]; m.y[i] = (bf16*)y[i];
  }
  // the grid and the row layout of svae_layernorm_fwd (so the outputs are bit-identical to its)
  static const int cap_env = [] { const char* e = getenv("SVAE_LN_FWD_BLOCKS"); return e ? atoi(e) : -1; }();
  static const int c4 = [] { const char* e = getenv("SVAE_LN_FWD_4COL"); return e ? atoi(e) : 1; }();
  const int cap = cap_env >= 0 ? cap_env : ((D <= 512 || (c4 && D <= 768)) ? 2048 : 1024);
  const int need = (rows + 3) / 4;
  dim3 grid((unsigned)(cap > 0 ? std::min(need, cap) : need));
  hipStream_t s = (hipStream_t)stream;
#define SVAE_LN_FWDM(MV) hipLaunchKernelGGL((ln_fwd_multi_kernel<MV>), grid, dim3(256), 0, s, x, m, mean, rstd, rows, D)
  if (c4 && D > 512 && D <= 768) SVAE_LN_FWDM(3);
  else if (D % 8 == 0 && D <= 512) SVAE_LN_FWDM(2);
  else if (D % 8 == 0) SVAE_LN_FWDM(4);
  else if (D <= 768) SVAE_LN_FWDM(3);
  else SVAE_LN_FWDM(5);
#undef SVAE_LN_FWDM
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_layernorm_bwd_multi(const void* const* dy, const float* x, const float* const* w, const float* mean,
                                         const float* rstd, const float* dres, float* dx, float* const* part,
                                         int32_t nblk, int32_t n, int32_t rows, int32_t D, svae_stream_t stream) {
  if (!dy || !x || !w || !mean || !rstd || !dx || !part || n <= 0 || n > SVAE_LN_MULTI_MAX || rows <= 0 || D <= 0 ||
      D % 4 || D > 1024 || nblk <= 0)
    return SVAE_EINVAL;
  LnMulti m = {};
  m.n = n;
  for (int i = 0; i < n; ++i) {
    if (!dy[i] || !w[i] || !part[i]) return SVAE_EINVAL;
    m.dy[i] = (const bf16*)dy[i]; m.w[i] = w[i]; m.part[i] = part[i];
  }
  hipStream_t s = (hipStream_t)stream;
#define SVAE_LN_BWDM(MV) \
  hipLaunchKernelGGL((ln_bwd_multi_kernel<MV>), dim3(nblk), dim3(256), 0, s, m, x, mean, rstd, dres, dx, rows, D)
  if (D <= 512) SVAE_LN_BWDM(2);
  else if (D <= 768) SVAE_LN_BWDM(3);
  else SVAE_LN_BWDM(4);
#undef SVAE_LN_BWDM
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_layernorm_nblk(int32_t rows) {
  int n = (rows + 3) / 4;
  return n < 1024 ? n : 1024;
}

SVAE_EXPORT int svae_layernorm_bwd_drop(const void* dy, const void* x, int32_t x_dtype, const float* w,
                                        const float* mean, const float* rstd, const float* dres, float* dx, void* dx_bf,
                                        float* part, int32_t nblk, int32_t rows, int32_t D, int32_t zero_mod,
                                        float bf_drop_p, uint64_t bf_seed, int32_t bf_zero_mod, float* zrow,
                                        void* zrow_bf, svae_stream_t stream) {
  if (!dy || !x || !w || !mean || !rstd || !dx || !part || rows <= 0 || D <= 0 || D % 4 || D > 1024 || nblk <= 0)
    return SVAE_EINVAL;
  if (bf_drop_p < 0.f || bf_drop_p >= 1.f || ((bf_drop_p > 0.f || bf_zero_mod > 0) && !dx_bf)) return SVAE_EINVAL;
  if ((zrow || zrow_bf) && zero_mod <= 0) return SVAE_EINVAL;
  hipStream_t s = (hipStream_t)stream;
#define SVAE_LN_BWD(MV)                                                                                            \
  do {                                                                                                             \
    if (x_dtype == 0)                                                                                              \
      hipLaunchKernelGGL((ln_bwd_kernel<float, MV>), dim3(nblk), dim3(256), 0, s, (const bf16*)dy, (const float*)x, \
                         w, mean, rstd, dres, dx, (bf16*)dx_bf, part, rows, D, zero_mod, bf_drop_p,                 \
                         (unsigned long long)bf_seed, bf_zero_mod, zrow, (bf16*)zrow_bf);                           \
    else                                                                                                           \
      hipLaunchKernelGGL((ln_bwd_kernel<bf16, MV>), dim3(nblk), dim3(256), 0, s, (const bf16*)dy, (const bf16*)x,   \
                         w, mean, rstd, dres, dx, (bf16*)dx_bf, part, rows, D, zero_mod, bf_drop_p,                 \
                         (unsigned long long)bf_seed, bf_zero_mod, zrow, (bf16*)zrow_bf);                           \
  } while (0)
  if (D <= 512) SVAE_LN_BWD(2);
  else if (D <= 768) SVAE_LN_BWD(3);
  else SVAE_LN_BWD(4);
#undef SVAE_LN_BWD
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_layernorm_bwd(const void* dy, const void* x, int32_t x_dtype, const float* w, const float* mean,
                                   const float* rstd, const float* dres, float* dx, void* dx_bf, float* part,
                                   int32_t nblk, int32_t rows, int32_t D, int32_t zero_mod, svae_stream_t stream) {
  return svae_layernorm_bwd_drop(dy, x, x_dtype, w, mean, rstd, dres, dx, dx_bf, part, nblk, rows, D, zero_mod, 0.f, 0,
                                 0, nullptr, nullptr, stream);
}

SVAE_EXPORT int svae_layernorm_bwd_gelu(const void* dy, const void* x, int32_t x_dtype, const float* w,
                                        const float* mean, const float* rstd, const void* gp, void* out_bf, float* part,
                                        int32_t nblk, int32_t rows, int32_t D, svae_stream_t stream) {
  if (!dy || !x || !w || !mean || !rstd || !gp || !out_bf || !part || rows <= 0 || D <= 0 || D % 4 || D > 1024 ||
      nblk <= 0)
    return SVAE_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const bf16* g = (const bf16*)gp;
#define SVAE_LN_BWD_G(MV)                                                                                          \
  do {                                                                                                             \
    if (x_dtype == 0)                                                                                              \
      hipLaunchKernelGGL((ln_bwd_kernel<float, MV, true>), dim3(nblk), dim3(256), 0, s, (const bf16*)dy,            \
                         (const float*)x, w, mean, rstd, nullptr, nullptr, (bf16*)out_bf, part, rows, D, 0, 0.f, 0ULL, \
                         0, nullptr, nullptr, g);                                                                  \
    else                                                                                                           \
      hipLaunchKernelGGL((ln_bwd_kernel<bf16, MV, true>), dim3(nblk), dim3(256), 0, s, (const bf16*)dy,             \
                         (const bf16*)x, w, mean, rstd, nullptr, nullptr, (bf16*)out_bf, part, rows, D, 0, 0.f, 0ULL,  \
                         0, nullptr, nullptr, g);                                                                  \
  } while (0)
  if (D <= 512) SVAE_LN_BWD_G(2);
  else if (D <= 768) SVAE_LN_BWD_G(3);
  else SVAE_LN_BWD_G(4);
#undef SVAE_LN_BWD_G
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_colsum(const void* in, int32_t in_dtype, int32_t rows, int32_t cols, int64_t ld, float* out,
                            int32_t accumulate, svae_stream_t stream) {
  if (!in || !out || rows <= 0 || cols <= 0 || cols % 4 || ld % 4) return SVAE_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (!accumulate && hipMemsetAsync(out, 0, sizeof(float) * cols, s) != hipSuccess) return SVAE_ELAUNCH;
  // ~256 blocks, >= 128 rows (one unrolled group of loads per thread) per split
  int colblocks, splits, rps;
  colsum_grid(rows, cols, colblocks, splits, rps);
  dim3 grid(colblocks, splits);
  if (in_dtype == 0)
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, s, (const float*)in, rows, cols, ld, out, rps);
  else
    hipLaunchKernelGGL(colsum_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)in, rows, cols, ld, out, rps);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}
