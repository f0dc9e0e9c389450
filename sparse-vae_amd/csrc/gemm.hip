// MFMA bf16 GEMM family for gfx950 with fused epilogues.
//
// C[M,N] = epi(alpha * A[M,K] . B[K,N]); A is [M][K] (a_t=0) or [K][M] (a_t=1); B is [N][K] (b_t=0,
// the nn.Linear weight layout) or [K][N] (b_t=1). The three layout pairs cover every nn.Linear of the
// TransformerVAE step: forward Y = X W^T (0,0), dX = dY W (0,1), dW = dY^T X (1,1).
//
// Tile 128x128x64, 256 threads = 4 waves (2x2), each wave 64x64 = 4x4 v_mfma_f32_16x16x32_bf16.
// Operands staged HBM -> registers -> LDS (issue-early / write-late, double-buffered LDS, one barrier per
// K-tile). K-contiguous tiles are read with ds_read_b128 (XOR-swizzled 16-B chunks, conflict-free for the
// b128 lane groups); M/N-contiguous tiles with ds_read_b64_tr_b16 (XOR-swizzled 8-B units).
#include "common.h"
#include "../../include/svae.h"

using namespace svae;

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = BM * BK * 2;  // 16 KiB per operand tile

struct GP {
  const bf16* A; const bf16* B;
  long long lda, ldb, sA, sB;
  int M, N, K, splits, kchunk, tiles_n, tiles_m;
  void* C; long long ldc, sC;
  const float* bias;
  const float* resid; long long ldr;
  void* aux; long long ldaux;
  float alpha, drop_p;
  unsigned long long seed;
  const float* rot_tab; int rot_cols, rot_d, rot_seq;
  const int* labels; float* label_logit;
  int epi;
};

// byte offset of (row, 16-B chunk c) in a K-contiguous [128][64] bf16 tile (128-B rows)
__device__ __forceinline__ int kc_off(int row, int c) { return row * 128 + ((c ^ ((row >> 1) & 7)) << 4); }
// byte offset of (k row, 8-B unit u) in an MN-contiguous [64][128] bf16 tile (256-B rows)
__device__ __forceinline__ int mn_off(int k, int u) {
  const int s = (k & 3) | (((k >> 3) & 1) << 2);
  return k * 256 + ((u ^ (s << 2)) << 3);
}

// Load one operand tile (rows x 64 k) into 4 x 16-B registers per thread with buffer loads: lanes outside
// the matrix get an out-of-range offset and read zeros from the hardware range check (no branches).
// TRANS = false: global [rows][K] (ld), TRANS = true: global [K][rows] (ld).
template <bool TRANS>
__device__ __forceinline__ void load_tile(const bf16* __restrict__ g, long long ld, int row0, int nrows, int k0,
                                          int kend, u32x4 (&r)[4], int tid) {
  const bf16* base = TRANS ? g + (long long)k0 * ld + row0 : g + (long long)row0 * ld + k0;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + 256 * i;
    int row, k;
    if (!TRANS) { row = idx >> 3; k = (idx & 7) * 8; }
    else { k = idx >> 4; row = (idx & 15) * 8; }
    const bool ok = (row0 + row < nrows) && (k0 + k < kend);
    const int off = TRANS ? (k * (int)ld + row) * 2 : (row * (int)ld + k) * 2;
    r[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, ok ? off : 0x7FFFFFF0, 0, 0));
  }
}

template <bool TRANS>
__device__ __forceinline__ void store_tile(char* lds, const u32x4 (&r)[4], int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + 256 * i;
    int off;
    if (!TRANS) off = kc_off(idx >> 3, idx & 7);
    else off = mn_off(idx >> 4, (idx & 15) * 2);
    *(u32x4*)(lds + off) = r[i];
  }
}

// Fragment (16 rows x 32 k) for MFMA 16x16x32: lane l holds X[row = base + (l&15)][k = 32kk + 8(l>>4) + j].
template <bool TRANS>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int base, int kk, int lane) {
  if (!TRANS) {
    const int row = base + (lane & 15);
    const int c = (lane >> 4) + 4 * kk;
    return *(const bf16x8*)(lds + kc_off(row, c));
  } else {
    const int q = (lane & 15) >> 2, p = lane & 3;
    const int kb = 32 * kk + 8 * (lane >> 4) + q;
    const int u = (base >> 2) + p;
    short4v lo = lds_read_tr(lds + mn_off(kb, u));
    short4v hi = lds_read_tr(lds + mn_off(kb + 4, u));
    return cat44(lo, hi);
  }
}

template <bool AT, bool BT, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GP p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // tile coordinates: consecutive blocks walk N first (A panel reuse in L2)
  const int bid = blockIdx.x;
  const int bn = bid % p.tiles_n, bm = bid / p.tiles_n;
  const int z = blockIdx.z;
  const int batch = z / p.splits, split = z % p.splits;
  const int m0 = bm * BM, n0 = bn * BN;
  const int kbeg = split * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const bf16* A = p.A + batch * p.sA;
  const bf16* B = p.B + batch * p.sB;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + BK - 1) / BK;
  u32x4 ra[4], rb[4];
  if (nk > 0) {
    load_tile<AT>(A, p.lda, m0, p.M, kbeg, kend, ra, tid);
    load_tile<BT>(B, p.ldb, n0, p.N, kbeg, kend, rb, tid);
    store_tile<AT>(smem, ra, tid);
    store_tile<BT>(smem + TILE_BYTES, rb, tid);
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const char* la = smem + cur * 2 * TILE_BYTES;
    const char* lb = la + TILE_BYTES;
    const bool more = kt + 1 < nk;
    if (more) {
      const int kn = kbeg + (kt + 1) * BK;
      load_tile<AT>(A, p.lda, m0, p.M, kn, kend, ra, tid);
      load_tile<BT>(B, p.ldb, n0, p.N, kn, kend, rb, tid);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<AT>(la, wm * 64 + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag<BT>(lb, wn * 64 + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    if (more) {
      char* nb = smem + (cur ^ 1) * 2 * TILE_BYTES;
      store_tile<AT>(nb, ra, tid);
      store_tile<BT>(nb + TILE_BYTES, rb, tid);
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
  const long long cofs = (long long)batch * p.sC;
  if constexpr (EPI == SVAE_EPI_CE_STATS) {
    // logits tile -> bf16 store, per-row (max, sumexp) over this block's 128 columns, label logit.
    // Each wave covers 64 columns; reduce the 2 waves (wn) through LDS.
    float* red = (float*)smem;  // [2 wn][128 rows][2]
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ml = wm * 64 + i * 16 + 4 * (lane >> 4) + r;
        const int m = m0 + ml;
        float mx = -INFINITY;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + wn * 64 + j * 16 + (lane & 15);
          float x = -INFINITY;
          if (n < p.N) {
            x = p.alpha * acc[i][j][r] + (p.bias ? p.bias[n] : 0.f);
            if (m < p.M) {
              ((bf16*)p.C)[cofs + (long long)m * p.ldc + n] = f2bf(x);
              if (p.labels[m] == n) p.label_logit[m] = x;
            }
          }
          v[j] = x;
          mx = fmaxf(mx, x);
        }
        // reduce over the 16 lanes sharing this row (lane & 15 varies)
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        float se = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) se += (v[j] == -INFINITY) ? 0.f : __expf(v[j] - mx);
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) se += __shfl_xor(se, o, 64);
        if ((lane & 15) == 0) {
          red[(wn * 128 + ml) * 2 + 0] = mx;
          red[(wn * 128 + ml) * 2 + 1] = se;
        }
      }
    }
    __syncthreads();
    if (tid < 128) {
      const int m = m0 + tid;
      if (m < p.M) {
        const float a0 = red[tid * 2], s0 = red[tid * 2 + 1];
        const float a1 = red[(128 + tid) * 2], s1 = red[(128 + tid) * 2 + 1];
        const float mx = fmaxf(a0, a1);
        const float se = (a0 == -INFINITY ? 0.f : s0 * __expf(a0 - mx)) + (a1 == -INFINITY ? 0.f : s1 * __expf(a1 - mx));
        float* part = (float*)p.aux + ((long long)m * p.tiles_n + bn) * 2;
        part[0] = mx;
        part[1] = se;
      }
    }
    return;
  }

#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + (lane & 15);
      const float bias = (p.bias && n < p.N) ? p.bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + 4 * (lane >> 4) + r;
        float x = p.alpha * acc[i][j][r];
        if constexpr (EPI == SVAE_EPI_ROTARY_BF16) {
          x += bias;
          const float partner = __shfl_xor(x, 1, 64);
          if (n < p.rot_cols && m < p.M) {
            const int pair = (n % p.rot_d) >> 1;
            const int pos = m % p.rot_seq;
            const float2 cs = ((const float2*)p.rot_tab)[(long long)pos * (p.rot_d >> 1) + pair];
            x = (n & 1) ? (x * cs.x + partner * cs.y) : (x * cs.x + (-partner) * cs.y);
          }
        }
        if (m >= p.M || n >= p.N) continue;
        const long long ci = cofs + (long long)m * p.ldc + n;
        if constexpr (EPI == SVAE_EPI_BF16) {
          ((bf16*)p.C)[ci] = f2bf(x + bias);
        } else if constexpr (EPI == SVAE_EPI_ROTARY_BF16) {
          ((bf16*)p.C)[ci] = f2bf(x);
        } else if constexpr (EPI == SVAE_EPI_F32) {
          float y = x + bias;
          if (p.resid) y += p.resid[(long long)m * p.ldr + n];
          ((float*)p.C)[ci] = y;
        } else if constexpr (EPI == SVAE_EPI_F32_ACC) {
          ((float*)p.C)[ci] += x;
        } else if constexpr (EPI == SVAE_EPI_F32_ATOMIC) {
          atomicAdd(&((float*)p.C)[ci], x);
        } else if constexpr (EPI == SVAE_EPI_GELU) {
          const float pre = x + bias;
          ((bf16*)p.aux)[(long long)m * p.ldaux + n] = f2bf(pre);
          ((bf16*)p.C)[ci] = f2bf(gelu_f(pre));
        } else if constexpr (EPI == SVAE_EPI_GELU_BWD) {
          const float pre = bf2f(((const bf16*)p.aux)[(long long)m * p.ldaux + n]);
          ((bf16*)p.C)[ci] = f2bf(x * gelu_grad_f(pre));
        } else if constexpr (EPI == SVAE_EPI_DROPOUT_RESID) {
          float y = x;
          if (p.drop_p > 0.f) {
            const float u = rand_uniform(p.seed, (unsigned long long)m * p.N + n);
            y = (u >= p.drop_p) ? y * (1.0f / (1.0f - p.drop_p)) : 0.f;
          }
          ((float*)p.C)[ci] = p.resid[(long long)m * p.ldr + n] + y;
        }
      }
    }
  }
}

}  // namespace

SVAE_EXPORT int svae_gemm(const svae_gemm_desc* d, svae_stream_t stream) {
  if (!d || !d->A || !d->B || !d->C) return SVAE_EINVAL;
  if (d->M <= 0 || d->N <= 0 || d->K <= 0 || d->batch <= 0 || d->splits <= 0) return SVAE_EINVAL;
  if ((d->K % 8 && !(d->a_t && d->b_t)) || d->lda % 8 || d->ldb % 8) return SVAE_EINVAL;
  if (d->a_t && d->M % 8) return SVAE_EINVAL;
  if (d->b_t && d->N % 8) return SVAE_EINVAL;
  if (((uintptr_t)d->A | (uintptr_t)d->B) & 15) return SVAE_EINVAL;
  if (d->batch_stride_a % 8 || d->batch_stride_b % 8) return SVAE_EINVAL;
  if (d->epi < 0 || d->epi > SVAE_EPI_CE_STATS) return SVAE_EINVAL;
  if (d->epi == SVAE_EPI_ROTARY_BF16 && (!d->rot_tab || d->rot_d <= 0 || d->rot_seq <= 0)) return SVAE_EINVAL;
  if ((d->epi == SVAE_EPI_GELU || d->epi == SVAE_EPI_GELU_BWD || d->epi == SVAE_EPI_CE_STATS) && !d->aux)
    return SVAE_EINVAL;
  if (d->epi == SVAE_EPI_DROPOUT_RESID && !d->resid) return SVAE_EINVAL;
  if (d->epi == SVAE_EPI_CE_STATS && (!d->labels || !d->label_logit || d->splits != 1)) return SVAE_EINVAL;
  if (d->splits > 1 && d->epi != SVAE_EPI_F32_ATOMIC) return SVAE_EINVAL;

  GP p;
  p.A = (const bf16*)d->A; p.B = (const bf16*)d->B;
  p.lda = d->lda; p.ldb = d->ldb; p.sA = d->batch_stride_a; p.sB = d->batch_stride_b;
  p.M = d->M; p.N = d->N; p.K = d->K; p.splits = d->splits;
  int kchunk = (d->K + d->splits - 1) / d->splits;
  kchunk = (kchunk + BK - 1) / BK * BK;
  p.kchunk = kchunk;
  p.tiles_n = (d->N + BN - 1) / BN;
  p.tiles_m = (d->M + BM - 1) / BM;
  p.C = d->C; p.ldc = d->ldc; p.sC = d->batch_stride_c;
  p.bias = d->bias; p.resid = d->resid; p.ldr = d->ldr;
  p.aux = d->aux; p.ldaux = d->ldaux;
  p.alpha = d->alpha; p.drop_p = d->drop_p; p.seed = d->seed;
  p.rot_tab = d->rot_tab; p.rot_cols = d->rot_cols; p.rot_d = d->rot_d; p.rot_seq = d->rot_seq;
  p.labels = d->labels; p.label_logit = d->label_logit;
  p.epi = d->epi;

  dim3 grid(p.tiles_n * p.tiles_m, 1, d->batch * d->splits);
  hipStream_t s = (hipStream_t)stream;
  const int lay = (d->a_t ? 2 : 0) | (d->b_t ? 1 : 0);
#define SVAE_GEMM_CASE(E)                                                                             \
  case E:                                                                                             \
    if (lay == 0) hipLaunchKernelGGL((gemm_kernel<false, false, E>), grid, dim3(256), 0, s, p);        \
    else if (lay == 1) hipLaunchKernelGGL((gemm_kernel<false, true, E>), grid, dim3(256), 0, s, p);    \
    else if (lay == 2) hipLaunchKernelGGL((gemm_kernel<true, false, E>), grid, dim3(256), 0, s, p);    \
    else hipLaunchKernelGGL((gemm_kernel<true, true, E>), grid, dim3(256), 0, s, p);                   \
    break;
  switch (d->epi) {
    SVAE_GEMM_CASE(SVAE_EPI_BF16)
    SVAE_GEMM_CASE(SVAE_EPI_F32)
    SVAE_GEMM_CASE(SVAE_EPI_F32_ACC)
    SVAE_GEMM_CASE(SVAE_EPI_F32_ATOMIC)
    SVAE_GEMM_CASE(SVAE_EPI_GELU)
    SVAE_GEMM_CASE(SVAE_EPI_GELU_BWD)
    SVAE_GEMM_CASE(SVAE_EPI_DROPOUT_RESID)
    SVAE_GEMM_CASE(SVAE_EPI_ROTARY_BF16)
    SVAE_GEMM_CASE(SVAE_EPI_CE_STATS)
    default: return SVAE_EINVAL;
  }
#undef SVAE_GEMM_CASE
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}
