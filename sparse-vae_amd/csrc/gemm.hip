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
#include <stdlib.h>
#include <algorithm>

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
  float* a_rowsum;   // optional: += sum_k A[m][k] (bias gradient fused into the dW GEMM); a_t layout only
  const float* k_weight;   // optional with a_rowsum: a_rowsum[m] += sum_k A[m][k] * k_weight[k] (gemm256 only)
  const float* row_a; const float* row_b;   // CE_PROB offset / ROWSCALE_GATHER scale and gather weight, per row
  const bf16* gather; long long ldg;        // ROWSCALE_GATHER: bf16 rows, row labels[m] gathered
  int epi;
  int tn2, tm2;      // 256-tile counts (gemm256)
  int group;         // L2 grouping: consecutive tiles walk `group` tile rows (M) before the next tile column
  int total3;        // gemm256: tiles x batch x splits (blocks loop over tiles with stride gridDim.x)
  int relaxed;       // gemm256 persistent: allow the vmcnt(G3_EPI_STORES) first wait after interior epilogues
  int dma_stagger;   // gemm256: the M-half-1 waves issue their next-K-tile DMA after their first MFMA quadrant
  long long slab;    // split-K slab mode: split s writes its partial tile at C + s * slab (0 = off)
  float* delta; const float* delta_o32; long long ld_o32; int delta_hd, delta_seq;   // see svae_gemm_desc.delta
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

// f32 staging tile [128][128] for the epilogue: 16-B unit index XOR ((row >> 2) & 3) << 2
__device__ __forceinline__ int cs_swz(int row, int col) { return (((col >> 2) ^ (((row >> 2) & 3) << 2)) << 2) | (col & 3); }
// gemm256's staging (16-B writes of 8 consecutive rows per lane group): unit index XOR (row & 7)
__device__ __forceinline__ int cs_swz8(int row, int col) { return (((col >> 2) ^ (row & 7)) << 2) | (col & 3); }
template <bool SW8>
__device__ __forceinline__ int cs_at(int row, int col) { return SW8 ? cs_swz8(row, col) : cs_swz(row, col); }

// Tile index -> (bm, bn). group <= 1: N-fastest rows of tiles. group = G: tiles run in bands of G tile rows,
// M-fastest inside a band, so the ~32 tiles an XCD holds at once cover a G x (32/G) patch whose A and B panels
// fit its 4 MiB L2 (instead of 32 different B panels that miss it on every tile).
__device__ __forceinline__ void group_tile(int t, int tiles_m, int tiles_n, int group, int& bm, int& bn) {
  if (group <= 1) {
    bn = t % tiles_n;
    bm = t / tiles_n;
    return;
  }
  const int per = group * tiles_n, grp = t / per, first = grp * group;
  const int gs = min(group, tiles_m - first), r = t - grp * per;
  bm = first + r % gs;
  bn = r / gs;
}

// Block -> (tile, batch, split). The hardware deals consecutive block ids round-robin over the 8 XCDs; the
// bijective remap gives each XCD one contiguous range of the (batch, split)-major / N-fastest logical order,
// so blocks that share A rows, B columns or a K-chunk run together on one L2.
__device__ __forceinline__ void tile_coords(const GP& p, int& bm, int& bn, int& batch, int& split) {
  const int tiles = p.tiles_n * p.tiles_m;
  const int nwg = gridDim.x;
  int bid = blockIdx.x;
  if (nwg >= 16) {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, idx = bid / 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int z = bid / tiles, t = bid - z * tiles;
  group_tile(t, p.tiles_m, p.tiles_n, p.group, bm, bn);
  batch = z / p.splits;
  split = z - batch * p.splits;
}

__device__ __forceinline__ void store_bf16(bf16* dst, const f32x4& a, const f32x4& b, bool full) {
  if (full)
    *(bf16x8*)dst = (bf16x8){f2bf(a[0]), f2bf(a[1]), f2bf(a[2]), f2bf(a[3]), f2bf(b[0]), f2bf(b[1]), f2bf(b[2]), f2bf(b[3])};
  else
    *(bf16x4*)dst = (bf16x4){f2bf(a[0]), f2bf(a[1]), f2bf(a[2]), f2bf(a[3])};
}

// rotary on the interleaved pairs (n, n+1), (n+2, n+3) of 4 columns: (a, b) -> (a c - b s, b c + a s)
__device__ __forceinline__ void rotary4(const GP& p, f32x4& x, int m, int n) {
  if (n >= p.rot_cols) return;
  const int pos = m % p.rot_seq;
  const int pair = (n % p.rot_d) >> 1;
  const f32x4 cs2 = *(const f32x4*)(p.rot_tab + ((long long)pos * (p.rot_d >> 1) + pair) * 2);
  const float a0 = x[0], b0 = x[1], a1 = x[2], b1 = x[3];
  x[0] = a0 * cs2[0] + (-b0) * cs2[1];
  x[1] = b0 * cs2[0] + a0 * cs2[1];
  x[2] = a1 * cs2[2] + (-b1) * cs2[3];
  x[3] = b1 * cs2[2] + a1 * cs2[3];
}

__device__ __forceinline__ void dropout4(const GP& p, f32x4& x, int m, int n) {
  const float sc = 1.0f / (1.0f - p.drop_p);
  float u[4];
  rand_uniform4(p.seed, ((unsigned long long)m * p.N + n) >> 2, u);   // n % 4 == 0, N % 4 == 0
#pragma unroll
  for (int e = 0; e < 4; ++e) x[e] = (u[e] >= p.drop_p) ? x[e] * sc : 0.f;
}

// Epilogue over 64 rows x 128 columns of the f32 staging tile cs (local rows; global row m0 + rbase + row).
// Thread = 8 consecutive columns x 4 rows (16 threads per row): 16-B bf16 / 2 x 16-B f32 global vectors.
// N % 4 == 0, so a thread's group is either fully inside N or holds exactly 4 valid columns ("full").
template <int EPI, bool BIAS_DONE = false, bool SW8 = false>
__device__ __forceinline__ void epilogue_half(const GP& p, const float* cs, int m0, int n0, int bn, int rbase,
                                              long long cofs, int tid, int label_pre = -1) {
  if constexpr (EPI == SVAE_EPI_F32_ATOMIC) {
    // one column per lane: each wave-wide atomic covers 256 contiguous bytes (the full-rate shape)
    const int col = tid & 127, n = n0 + col;
    if (n < p.N) {
      for (int it = 0; it < 32; ++it) {
        const int row = (tid >> 7) + 2 * it, m = m0 + rbase + row;
        if (m < p.M) atomicAdd((float*)p.C + cofs + (long long)m * p.ldc + n, cs[row * 128 + cs_at<SW8>(row, col)]);
      }
    }
    return;
  }
  const int cc = (tid & 15) * 8, n = n0 + cc;
  const bool ncol = n < p.N, full = n + 8 <= p.N;
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  f32x4 b0 = zero, b1 = zero;
  if (!BIAS_DONE && p.bias && ncol) {
    b0 = *(const f32x4*)(p.bias + n);
    if (full) b1 = *(const f32x4*)(p.bias + n + 4);
  }
  if constexpr (EPI == SVAE_EPI_CE_STATS) {
    // one pass: thread = (row, quarter qd); its 32 columns are 32u + 8qd + (0..7), u < 4, so each of the 4
    // bf16 stores of a row covers 64 contiguous bytes across the row's 4 lanes. Per row: (max, sumexp) over
    // the tile's 128 columns and the label logit.
    const int row = tid >> 2, qd = tid & 3, m = m0 + rbase + row;
    float v[32];
    float mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = 32 * u + 8 * qd;
      f32x4 x0 = *(const f32x4*)(cs + row * 128 + cs_at<SW8>(row, c));
      f32x4 x1 = *(const f32x4*)(cs + row * 128 + cs_at<SW8>(row, c + 4));
      if (!BIAS_DONE && p.bias) {
        x0 += (n0 + c < p.N) ? *(const f32x4*)(p.bias + n0 + c) : zero;
        x1 += (n0 + c + 4 < p.N) ? *(const f32x4*)(p.bias + n0 + c + 4) : zero;
      }
      if (p.C && m < p.M && n0 + c < p.N)   // C == nullptr: statistics only (the IW-NLL evaluation)
        store_bf16((bf16*)p.C + cofs + (long long)m * p.ldc + n0 + c, x0, x1, n0 + c + 8 <= p.N);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float y0 = (n0 + c + e < p.N) ? x0[e] : -INFINITY;
        const float y1 = (n0 + c + 4 + e < p.N) ? x1[e] : -INFINITY;
        v[8 * u + e] = y0;
        v[8 * u + 4 + e] = y1;
        mx = fmaxf(mx, fmaxf(y0, y1));
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
    float se = 0.f;
#pragma unroll
    for (int e = 0; e < 32; ++e) se += __expf(v[e] - mx);
    se += __shfl_xor(se, 1, 64);
    se += __shfl_xor(se, 2, 64);
    if (m < p.M) {
      const int lc = (BIAS_DONE ? label_pre : p.labels[m]) - n0;   // label column within the tile (gemm256: preloaded)
      if (lc >= 0 && lc < 128 && ((lc >> 3) & 3) == qd) {
        const int idx = 8 * (lc >> 5) + (lc & 7);
#pragma unroll
        for (int e = 0; e < 32; ++e)
          if (e == idx) p.label_logit[m] = v[e];
      }
      if (qd == 0) {
        float* part = (float*)p.aux + ((long long)m * p.tiles_n + bn) * 2;
        part[0] = mx;
        part[1] = se;
      }
    }
    return;
  }
  if (!ncol) return;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int row = (tid >> 4) + 16 * it, m = m0 + rbase + row;
    if (m >= p.M) break;
    f32x4 x0 = *(const f32x4*)(cs + row * 128 + cs_at<SW8>(row, cc));
    f32x4 x1 = full ? *(const f32x4*)(cs + row * 128 + cs_at<SW8>(row, cc + 4)) : zero;
    const long long ci = cofs + (long long)m * p.ldc + n;
    if constexpr (EPI == SVAE_EPI_BF16) {
      store_bf16((bf16*)p.C + ci, x0 + b0, x1 + b1, full);
    } else if constexpr (EPI == SVAE_EPI_ROTARY_BF16) {
      x0 += b0;
      x1 += b1;
      rotary4(p, x0, m, n);
      if (full) rotary4(p, x1, m, n + 4);
      store_bf16((bf16*)p.C + ci, x0, x1, full);
    } else if constexpr (EPI == SVAE_EPI_F32 || EPI == SVAE_EPI_F32_ACC || EPI == SVAE_EPI_DROPOUT_RESID) {
      float* c = (float*)p.C + ci;
      if constexpr (EPI == SVAE_EPI_F32) {
        x0 += b0;
        x1 += b1;
        if (p.resid) {
          const float* r = p.resid + (long long)m * p.ldr + n;
          x0 += *(const f32x4*)r;
          if (full) x1 += *(const f32x4*)(r + 4);
        }
      } else if constexpr (EPI == SVAE_EPI_F32_ACC) {
        x0 += *(const f32x4*)c;
        if (full) x1 += *(const f32x4*)(c + 4);
      } else {
        if (p.drop_p > 0.f) {
          dropout4(p, x0, m, n);
          if (full) dropout4(p, x1, m, n + 4);
        }
        const float* r = p.resid + (long long)m * p.ldr + n;
        x0 += *(const f32x4*)r;
        if (full) x1 += *(const f32x4*)(r + 4);
      }
      *(f32x4*)c = x0;
      if (full) *(f32x4*)(c + 4) = x1;
      if constexpr (EPI == SVAE_EPI_DROPOUT_RESID) {   // the bf16 copy (the vocabulary head's input)
        if (p.aux) store_bf16((bf16*)p.aux + (long long)m * p.ldaux + n, x0, x1, full);
      } else if constexpr (EPI == SVAE_EPI_F32) {      // the dropout-masked bf16 copy (a layer backward's input)
        if (p.aux) {
          if (p.drop_p > 0.f) {
            dropout4(p, x0, m, n);
            if (full) dropout4(p, x1, m, n + 4);
          }
          store_bf16((bf16*)p.aux + (long long)m * p.ldaux + n, x0, x1, full);
        }
      }
    } else if constexpr (EPI == SVAE_EPI_GELU) {
      // C = gelu(acc + bias), aux = gelu'(acc + bias): the backward multiplies by aux, no erf recomputed
      x0 += b0;
      x1 += b1;
      f32x4 g0, g1, d0, d1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float g, dg;
        gelu_pair(x0[e], g, dg);
        g0[e] = g;
        d0[e] = dg;
        gelu_pair(x1[e], g, dg);
        g1[e] = g;
        d1[e] = dg;
      }
      store_bf16((bf16*)p.C + ci, g0, g1, full);
      store_bf16((bf16*)p.aux + (long long)m * p.ldaux + n, d0, d1, full);
    } else if constexpr (EPI == SVAE_EPI_GELU_BWD) {
      const bf16* a = (const bf16*)p.aux + (long long)m * p.ldaux + n;
      bf16x8 d;
      if (full) d = *(const bf16x8*)a;
      else {
        const bf16x4 h = *(const bf16x4*)a;
        d = (bf16x8){h[0], h[1], h[2], h[3], h[0], h[1], h[2], h[3]};
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x0[e] *= (float)d[e];
        x1[e] *= (float)d[e + 4];
      }
      store_bf16((bf16*)p.C + ci, x0, x1, full);
    }
  }
}

template <bool AT, bool BT, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GP p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // tile coordinates: XCD-aware remap (see gemm_glds_kernel), then N first inside an XCD's range
  int bm, bn, batch, split;
  tile_coords(p, bm, bn, batch, split);
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
  float rsum[4] = {0.f, 0.f, 0.f, 0.f};
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
    if constexpr (AT) {
      if (p.a_rowsum && bn == 0) {   // this block's share of sum_k A[m][k]: 4 columns x 8 k-rows per thread
        const int mu = tid & 31, kg = tid >> 5;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const short4v v = *(const short4v*)(la + mn_off(kg * 8 + r, mu));
          const bf16x4 b = __builtin_bit_cast(bf16x4, v);
#pragma unroll
          for (int e = 0; e < 4; ++e) rsum[e] += (float)b[e];
        }
      }
    }
    if (more) {
      char* nb = smem + (cur ^ 1) * 2 * TILE_BYTES;
      store_tile<AT>(nb, ra, tid);
      store_tile<BT>(nb + TILE_BYTES, rb, tid);
    }
    __syncthreads();
  }

  if constexpr (AT) {
    if (p.a_rowsum && bn == 0) {
      const int m = m0 + (tid & 31) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (m + e < p.M) atomicAdd(p.a_rowsum + m + e, rsum[e]);
    }
  }
  // ---------------------------------------------------------------- epilogue
  // Stage the 128x128 f32 tile through LDS (16-B units XOR-swizzled by row so the fragment writes spread over
  // the banks), then run the shared vectorised epilogue on each 64-row half.
  float* cs = (float*)smem;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 64 + i * 16 + 4 * (lane >> 4) + r;
        const int col = wn * 64 + j * 16 + (lane & 15);
        cs[row * 128 + cs_swz(row, col)] = p.alpha * acc[i][j][r];
      }
  __syncthreads();
  const long long cofs = (long long)batch * p.sC + split * p.slab;
  epilogue_half<EPI>(p, cs, m0, n0, bn, 0, cofs, tid);
  epilogue_half<EPI>(p, cs + 64 * 128, m0, n0, bn, 64, cofs, tid);
}

// ===================================================================================================
// gemm_glds: same contract, deeper pipeline. BK = 32, a 3-stage LDS ring filled by LDS-DMA
// (buffer_load ... lds, 16 B per lane; out-of-range lanes read zeros from the buffer range check), so two
// K-tiles are in flight while a third is consumed, with no staging registers and no ds_write pass.
// 48 KiB of LDS and <= 168 VGPRs per block -> 3 blocks (12 waves) per CU overlap each other's prologue and
// epilogue. The LDS image is lane-linear per wave instruction (1 KiB); the bank swizzle is applied on the
// SOURCE address and undone on the fragment reads (K-contiguous: 64-B rows, chunk ^ ((row >> 1) & 3);
// M/N-contiguous: 256-B rows, 16-B chunk ^ 2 s(k)).
constexpr int BK2 = 32;
constexpr int T2 = 128 * BK2 * 2;          // 8 KiB per operand tile
constexpr int STAGE2 = 2 * T2;             // A + B
constexpr int NSTAGE = 3;

__device__ __forceinline__ int kc2_off(int row, int c) { return row * 64 + ((c ^ ((row >> 1) & 3)) << 4); }

// LDS-DMA pieces (1 KiB wave-instructions) each of the 4 waves issues per operand K-tile: 8 KiB / 4 waves / 1 KiB
constexpr int G2_PIECES = T2 / 1024 / 4;
// the ring's counted wait: tile kt has landed while the next tile's pieces (both operands) may still fly
constexpr int G2_WAIT_NEXT = 2 * G2_PIECES;
static_assert(G2_PIECES * 4 * 1024 == T2, "issue_tile2 covers the operand tile exactly");

template <bool TRANS>
__device__ __forceinline__ void issue_tile2(const bf16* __restrict__ g, long long ld, int row0, int nrows, int k0,
                                            int kend, char* lds_tile, int wave, int lane) {
  const bf16* base = TRANS ? g + (long long)k0 * ld + row0 : g + (long long)row0 * ld + k0;
  const u32x4 rsrc = buffer_rsrc(base, 0x7FFFFFF0u);
  int o[G2_PIECES];
#pragma unroll
  for (int j = 0; j < G2_PIECES; ++j) {
    const int inst = wave * G2_PIECES + j;
    const int slot = inst * 64 + lane;
    int off;
    bool ok;
    if (!TRANS) {
      const int row = slot >> 2, c = (slot & 3) ^ ((row >> 1) & 3);
      off = (row * (int)ld + c * 8) * 2;
      ok = (row0 + row < nrows) && (k0 + c * 8 < kend);
    } else {
      const int kr = slot >> 4;
      const int sk = (kr & 3) | (((kr >> 3) & 1) << 2);
      const int v = (slot & 15) ^ (sk << 1);
      off = (kr * (int)ld + v * 8) * 2;
      ok = (k0 + kr < kend) && (row0 + v * 8 < nrows);
    }
    o[j] = ok ? off : 0x7FFFFFF0;
  }
  // the wave's consecutive pieces in one statement
  if constexpr (G2_PIECES == 2) dma16x2_lds(rsrc, lds_tile + wave * G2_PIECES * 1024, o[0], o[1]);
  else {
#pragma unroll
    for (int j = 0; j < G2_PIECES; ++j) dma16_lds(rsrc, lds_tile + (wave * G2_PIECES + j) * 1024, o[j]);
  }
}

template <bool TRANS>
__device__ __forceinline__ bf16x8 read_frag2(const char* lds, int base, int lane) {
  if (!TRANS) {
    return *(const bf16x8*)(lds + kc2_off(base + (lane & 15), lane >> 4));
  } else {
    const int q = (lane & 15) >> 2, p = lane & 3;
    const int kb = 8 * (lane >> 4) + q;
    const int u = (base >> 2) + p;
    return cat44(lds_read_tr(lds + mn_off(kb, u)), lds_read_tr(lds + mn_off(kb + 4, u)));
  }
}

template <bool AT, bool BT, int EPI>
__global__ __launch_bounds__(256, 3) void gemm_glds_kernel(GP p) {
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * STAGE2];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int bm, bn, batch, split;
  tile_coords(p, bm, bn, batch, split);
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
  float rsum[4] = {0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + BK2 - 1) / BK2;
  if (nk > 0) {
    issue_tile2<AT>(A, p.lda, m0, p.M, kbeg, kend, smem, wave, lane);
    issue_tile2<BT>(B, p.ldb, n0, p.N, kbeg, kend, smem + T2, wave, lane);
  }
  if (nk > 1) {
    issue_tile2<AT>(A, p.lda, m0, p.M, kbeg + BK2, kend, smem + STAGE2, wave, lane);
    issue_tile2<BT>(B, p.ldb, n0, p.N, kbeg + BK2, kend, smem + STAGE2 + T2, wave, lane);
  }
  int stage = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt landed (this wave's 4 DMA pieces of tile kt+1 may still fly), then everyone's pieces + the
    // ring slot of tile kt+2 (last read in iteration kt-1) is free
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G2_WAIT_NEXT) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) {
      int s2 = stage + 2;
      if (s2 >= NSTAGE) s2 -= NSTAGE;
      char* st2 = smem + s2 * STAGE2;
      issue_tile2<AT>(A, p.lda, m0, p.M, kbeg + (kt + 2) * BK2, kend, st2, wave, lane);
      issue_tile2<BT>(B, p.ldb, n0, p.N, kbeg + (kt + 2) * BK2, kend, st2 + T2, wave, lane);
    }
    const char* la = smem + stage * STAGE2;
    const char* lb = la + T2;
    bf16x8 af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = read_frag2<AT>(la, wm * 64 + i * 16, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = read_frag2<BT>(lb, wn * 64 + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    if constexpr (AT) {
      if (p.a_rowsum && bn == 0) {   // sum_k A[m][k]: 4 columns x 4 k-rows per thread
        const int mu = tid & 31, kg = tid >> 5;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const short4v v = *(const short4v*)(la + mn_off(kg * 4 + r, mu));
          const bf16x4 b = __builtin_bit_cast(bf16x4, v);
#pragma unroll
          for (int e = 0; e < 4; ++e) rsum[e] += (float)b[e];
        }
      }
    }
    stage = stage + 1 == NSTAGE ? 0 : stage + 1;
  }
  if constexpr (AT) {
    if (p.a_rowsum && bn == 0) {
      const int m = m0 + (tid & 31) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (m + e < p.M) atomicAdd(p.a_rowsum + m + e, rsum[e]);
    }
  }
  __syncthreads();
  // epilogue in two halves of 64 rows (the ring holds 48 KiB; a half tile of f32 is 32 KiB)
  float* cs = (float*)smem;
  const long long cofs = (long long)batch * p.sC + split * p.slab;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = i * 16 + 4 * (lane >> 4) + r;
            const int col = wn * 64 + j * 16 + (lane & 15);
            cs[row * 128 + cs_swz(row, col)] = p.alpha * acc[i][j][r];
          }
    }
    __syncthreads();
    epilogue_half<EPI>(p, cs, m0, n0, bn, h * 64, cofs, tid);
    __syncthreads();
  }
}

// ===================================================================================================
// gemm256: 256x256 output tile per 512-thread block (8 waves as 2 (M) x 4 (N), each wave 128 x 64 =
// 8 x 4 accumulator tiles), BK = 64, A and B K-tiles double-buffered in LDS (2 x 64 KiB) and filled by
// LDS-DMA one whole K-tile ahead: the next tile's 64 DMA pieces are issued right after the barrier that
// frees its buffer, so they fly under the current tile's 128 MFMAs per wave. One counted wait + raw barrier
// per K-tile. Inside a K-tile the wave walks its four 64 x 32 quadrants (A fragments reused across two,
// B fragments across the turn), 16 MFMAs each. Layouts: A [M][K] (K-contiguous, 128-B rows, kc_off
// swizzle); B [N][K] likewise, or B [K][N] (b_t) as two [64][128] MN-contiguous halves read with
// ds_read_b64_tr_b16 (mn_off swizzle). All swizzles are applied on the DMA SOURCE address (the LDS image is
// lane-linear per 1-KiB piece) and undone by the fragment reads. Epilogues run straight from the
// accumulator registers (g3_reg_epilogue / g3_reg_epilogue_ld below); float-atomic split-K without a slab
// workspace is left to the 128-tile kernels.
constexpr int G3_T = 256 * 64 * 2;   // 32 KiB per operand K-tile
constexpr int G3_STAGE = 2 * G3_T;
// internal instantiation: SVAE_EPI_BF16 that also writes the attention backward's delta (svae_gemm_desc.delta)
constexpr int G3_EPI_BF16_DELTA = 65;
// internal instantiation: SVAE_EPI_F32_ACC whose fused bias-gradient row sums are weighted by k_weight (the
// vocabulary head's dW, where the per-token weight r folds the softmax normalisation into the row sums)
constexpr int G3_EPI_ACC_KW = 64;
// internal: the split-K slab form of the same (each split stores its partial tile, slab_reduce adds them into C;
// the k-weighted row sums of each split's K range go to a_rowsum by atomics as in every split-K row sum)
constexpr int G3_EPI_F32_KW = 66;
// internal: the split-K slab store (plain f32 partial tile: no residual, no bf16 copy) -- SVAE_EPI_F32 without the
// operand loads and branches of its optional inputs, whose registers spilled in the heaviest instantiations
constexpr int G3_EPI_SLAB = 67;

// Per-lane DMA source offsets of one operand's K-tile relative to the tile base (a scalar that moves with m0 / n0 and
// k0): they do not depend on the tile, so they are computed once per kernel and are the only per-lane DMA state kept
// across the tile loop (8 VGPRs). A tile that is interior (its 256 rows / columns inside M / N) and a full K-tile
// issue them as they are; an edge tile or the K tail recomputes its offsets from a fresh lane id with the bound
// checks (out-of-range -> OOB offset, the piece reads zeros). Keeping per-tile checked offsets (and the compiler's
// unchecked copies) live across the tile loop spilled them in the register-heaviest instantiations, and a spill
// reload's vmcnt(0) inside the K loop drains the DMA ring.
struct G3Src {
  int off[4];
};

// K-contiguous operand [rows][K] (128-B rows of the tile): piece = 8 rows x 128 B; lane -> (row r, 16-B chunk c)
__device__ __forceinline__ void g3_piece_k(int piece, int lane, int& r, int& c) {
  r = piece * 8 + (lane >> 3);
  c = (lane & 7) ^ ((r >> 1) & 7);
}
// MN-contiguous operand [K][cols] as two [64][128] halves: piece = 4 k-rows x 256 B; lane -> (k-row kr, column col)
__device__ __forceinline__ void g3_piece_mn(int piece, int lane, int& kr, int& col) {
  const int half = piece >> 4;
  kr = (piece & 15) * 4 + (lane >> 4);
  const int sk = (kr & 3) | (((kr >> 3) & 1) << 2);
  col = half * 128 + (((lane & 15) ^ (sk << 1)) * 8);
}

template <bool MN>
__device__ __forceinline__ G3Src g3_src(long long ld, int wave, int lane) {
  G3Src s;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int x, y;
    if constexpr (MN) { g3_piece_mn(wave * 4 + i, lane, x, y); s.off[i] = (x * (int)ld + y) * 2; }
    else { g3_piece_k(wave * 4 + i, lane, x, y); s.off[i] = (x * (int)ld + y * 8) * 2; }
  }
  return s;
}

// One operand's K-tile: full = interior tile and a whole K-tile (wave-uniform); otherwise the checked offsets
// (row / column bound nb - base0, K bound krem) from a fresh lane id
template <bool MN>
__device__ __forceinline__ void g3_issue_one(const bf16* tile_base, const G3Src& src, bool full, long long ld, int nrem,
                                             int krem, char* dst, int wave) {
  const u32x4 rs = buffer_rsrc(tile_base, 0x7FFFFFF0u);
  if (full) {
    dma16x4_lds(rs, dst + wave * 4 * 1024, src.off[0], src.off[1], src.off[2], src.off[3]);
  } else {
    const int lane = lane_id_fresh();
    int o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int x, y, off;
      bool ok;
      if constexpr (MN) {   // x = k-row, y = column
        g3_piece_mn(wave * 4 + i, lane, x, y);
        ok = y < nrem && x < krem;
        off = (x * (int)ld + y) * 2;
      } else {              // x = row, y = 16-B chunk
        g3_piece_k(wave * 4 + i, lane, x, y);
        ok = x < nrem && y * 8 < krem;
        off = (x * (int)ld + y * 8) * 2;
      }
      o[i] = ok ? off : 0x7FFFFFF0;
    }
    dma16x4_lds(rs, dst + wave * 4 * 1024, o[0], o[1], o[2], o[3]);
  }
}

template <bool AT, bool BT>
__device__ __forceinline__ void g3_issue(const GP& p, const bf16* A, const bf16* B, const G3Src& sa, const G3Src& sb,
                                         int m0, int n0, int k0, int kend, char* stage, int wave) {
  const int krem = kend - k0;
  const bool fa = krem >= 64 && m0 + 256 <= p.M, fb = krem >= 64 && n0 + 256 <= p.N;
  if constexpr (AT) g3_issue_one<true>(A + (long long)k0 * p.lda + m0, sa, fa, p.lda, p.M - m0, krem, stage, wave);
  else g3_issue_one<false>(A + (long long)m0 * p.lda + k0, sa, fa, p.lda, p.M - m0, krem, stage, wave);
  if constexpr (BT) g3_issue_one<true>(B + (long long)k0 * p.ldb + n0, sb, fb, p.ldb, p.N - n0, krem, stage + G3_T, wave);
  else g3_issue_one<false>(B + (long long)n0 * p.ldb + k0, sb, fb, p.ldb, p.N - n0, krem, stage + G3_T, wave);
}

// B fragment (16 n x 32 k) of n-tile at column cb (0..255) of the B tile, k-step ks
template <bool BT>
__device__ __forceinline__ bf16x8 g3_bfrag(const char* lb, int cb, int ks, int lane) {
  if constexpr (!BT) return *(const bf16x8*)(lb + kc_off(cb + (lane & 15), (lane >> 4) + 4 * ks));
  else return read_frag<true>(lb + (cb >> 7) * (G3_T / 2), cb & 127, ks, lane);
}

// A fragment (16 m x 32 k) of the m-tile at row rb (0..255), k-step ks
template <bool AT>
__device__ __forceinline__ bf16x8 g3_afrag(const char* la, int rb, int ks, int lane) {
  if constexpr (!AT) return *(const bf16x8*)(la + kc_off(rb + (lane & 15), (lane >> 4) + 4 * ks));
  else return read_frag<true>(la + (rb >> 7) * (G3_T / 2), rb & 127, ks, lane);
}

// gemm256 accumulators are C^T fragments (MFMA operands swapped): acc[i][j] lane l holds row
// wr*128 + 16i + (l & 15), columns wc*64 + 16j + 4(l >> 4) + (0..3) -- one row, 4 consecutive columns.

// Register epilogue (bf16 out, GELU, rotary, CE statistics): straight from the C^T fragments, no staging. Each fragment
// is one 8-B bf16x4 store per lane (16 rows x 32 B per instruction; a row's 128-B line completes over the 4 j).
// CE: per-row (max, sum exp) over the wave's 64 columns by permlane reductions, combined across the 4 column
// waves through the side area into the 128-column partials ce_rows_kernel expects; the label logit is written
// by the lane holding it.
constexpr float G3_LOG2E = 1.4426950408889634f;


// Store the bf16 of two fragments' column groups x (cols 16ja + 4g..) and y (cols 16ja + 16 + 4g..) of one row
// as 16-B vectors: a permlane16 swap gives lane group g 8 consecutive columns (g0: 0-7, g2: 8-15, g1: 16-23,
// g3: 24-31 of the pair), so each instruction writes 16 rows x 64 contiguous bytes.
template <bool NT = false>
__device__ __forceinline__ void store_pair_bf16(bf16* row_base, int colbase, int ncols_left, const f32x4& x,
                                                const f32x4& y, int g) {
  const unsigned x0 = pack_bf16x2(x[0], x[1]), x1 = pack_bf16x2(x[2], x[3]);
  const unsigned y0 = pack_bf16x2(y[0], y[1]), y1 = pack_bf16x2(y[2], y[3]);
  const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
  const int c = colbase + ((g & 1) ? 16 : 0) + ((g & 2) ? 8 : 0);
  const u32x4 w = {s0[0], s1[0], s0[1], s1[1]};
  if (c + 8 <= ncols_left) {
    if constexpr (NT) __builtin_nontemporal_store(w, (u32x4*)(row_base + c));
    else *(u32x4*)(row_base + c) = w;
  } else if (c < ncols_left) *(u32x2*)(row_base + c) = (u32x2){w[0], w[1]};
}

template <bool B>
struct BoolC {
  static constexpr bool value = B;
};

template <int EPI>
__device__ __forceinline__ void g3_reg_epilogue(const GP& p, const f32x4 (&acc)[8][4], const float* sbias,
                                                const int* slabel, float* sstat, int m0, int n0, int bn, int batch,
                                                int split, int wr, int wc, int tid, int lane) {
  const long long cofs = (long long)batch * p.sC + split * p.slab;
  const int g = lane >> 4, li = lane & 15;
  f32x4 b4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) b4[j] = *(const f32x4*)(sbias + wc * 64 + j * 16 + 4 * g);
  f32x4 bl4[4];   // CE_PROB: bias * log2(e)
#pragma unroll
  for (int j = 0; j < 4; ++j) bl4[j] = b4[j] * G3_LOG2E;
  // ROTARY: a lane's 4 consecutive columns are two whole (2i, 2i+1) rotary pairs, rotated in registers. The table
  // offsets of its 4 column groups are per tile, the table row (position m mod rot_seq) steps by 16 per fragment
  // row, and row i + 1's (cos, sin) are loaded before row i is rotated (columns >= rot_cols get the identity).
  int rofs[4] = {0, 0, 0, 0};
  bool rot_on[4] = {false, false, false, false};
  int pos = 0, pstep = 0;
  f32x4 cs_cur[4], cs_nxt[4];
  auto rot_load = [&](int ps, f32x4 (&cs)[4]) {
    const float* t = p.rot_tab + (long long)ps * p.rot_d;
#pragma unroll
    for (int j = 0; j < 4; ++j) cs[j] = rot_on[j] ? *(const f32x4*)(t + rofs[j]) : (f32x4){1.f, 0.f, 1.f, 0.f};
  };
  if constexpr (EPI == SVAE_EPI_ROTARY_BF16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wc * 64 + j * 16 + 4 * g;
      rot_on[j] = n < p.rot_cols;
      rofs[j] = ((n % p.rot_d) >> 1) * 2;
    }
    pos = (m0 + wr * 128 + li) % p.rot_seq;
    pstep = 16 % p.rot_seq;
    rot_load(pos, cs_cur);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int rl = wr * 128 + i * 16 + li, m = m0 + rl;
    f32x4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = p.alpha * acc[i][j] + b4[j];
    if constexpr (EPI == SVAE_EPI_ROTARY_BF16) {
      int pn = pos + pstep;
      if (pn >= p.rot_seq) pn -= p.rot_seq;
      if (i + 1 < 8) rot_load(pn, cs_nxt);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 cs2 = cs_cur[j];
        const float a0 = v[j][0], b0 = v[j][1], a1 = v[j][2], b1 = v[j][3];
        v[j][0] = a0 * cs2[0] + (-b0) * cs2[1];
        v[j][1] = b0 * cs2[0] + a0 * cs2[1];
        v[j][2] = a1 * cs2[2] + (-b1) * cs2[3];
        v[j][3] = b1 * cs2[2] + a1 * cs2[3];
      }
      pos = pn;
      if (i + 1 < 8) {
#pragma unroll
        for (int j = 0; j < 4; ++j) cs_cur[j] = cs_nxt[j];
      }
    }
    {
      // (the permlane swaps and DPP moves need every lane: the bounds are applied to the stores only)
      if constexpr (EPI == SVAE_EPI_GELU) {
        f32x4 gg[4], dg[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            f32x2 ge, de;
            gelu_pair2((f32x2){v[j][e], v[j][e + 1]}, ge, de);
            gg[j][e] = ge[0];
            gg[j][e + 1] = ge[1];
            dg[j][e] = de[0];
            dg[j][e + 1] = de[1];
          }
        store_rows_bf16<false>((bf16*)p.C + cofs, p.ldc, m0 + wr * 128 + i * 16, p.M, n0 + wc * 64, p.N, gg, g, li);
        // GELU' (read only by the FFN backward): nontemporal
        store_rows_bf16<true>((bf16*)p.aux, p.ldaux, m0 + wr * 128 + i * 16, p.M, n0 + wc * 64, p.N, dg, g, li);
      } else if constexpr (EPI == SVAE_EPI_CE_PROB) {
        // p = exp(logit - c_row) for rows with a target (0 elsewhere); the f32 values feed the per-tile sums below
        // exponent in packed f32 pairs: x = acc (alpha log2e) + (bias log2e - off), one v_pk_fma_f32 per two logits
        // (the row's offset folded into the per-column constants with one v_pk_add_f32 per pair), sums by v_pk_add
        const float off = sstat[1024 + rl] * G3_LOG2E;   // +inf for rows without a target: P = 0
        const f32x2 sa2 = {p.alpha * G3_LOG2E, p.alpha * G3_LOG2E}, noff = {-off, -off};
        f32x2 se2 = {0.f, 0.f};
        // the column bound is checked per element only on a wave whose 64 columns cross N (a scalar branch between
        // two copies: if-converted into the one loop it cost 4 VALU per element, as much as the exp's arithmetic)
        auto body = [&](auto rag) {
          f32x4 xs[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
              for (int e = 0; e < 4; e += 2) {
                const f32x2 a2 = {acc[i][j][e], acc[i][j][e + 1]};
                const f32x2 c2 = (f32x2){bl4[j][e], bl4[j][e + 1]} + noff;
                const f32x2 t2 = a2 * sa2 + c2;
                // (no clamp: a logit more than 88 nats above the label logit gives +inf here, which svae_ce_prob_finalize_fix finds
                // in the row's sum and recomputes exactly)
                f32x2 x = {__builtin_amdgcn_exp2f(t2[0]), __builtin_amdgcn_exp2f(t2[1])};
                if constexpr (decltype(rag)::value) {
                  const int n = n0 + wc * 64 + j * 16 + 4 * g + e;
                  if (n >= p.N) x[0] = 0.f;
                  if (n + 1 >= p.N) x[1] = 0.f;
                }
                xs[j][e] = x[0];
                xs[j][e + 1] = x[1];
                se2 += x;
              }
          // P [T, V] bf16 (2 GiB at C2): whole lines, nontemporal
          store_rows_bf16<true>((bf16*)p.C + cofs, p.ldc, m0 + wr * 128 + i * 16, p.M, n0 + wc * 64, p.N, xs, g, li);
        };
        if (__builtin_amdgcn_readfirstlane((int)(n0 + wc * 64 + 64 > p.N))) body(BoolC<true>{});
        else body(BoolC<false>{});
        float se = sum_x16_x32(se2[0] + se2[1]);
        if (g == 0) sstat[rl * 4 + wc] = se;
      } else if (EPI != SVAE_EPI_CE_STATS || p.C) {   // CE statistics with C == nullptr: no logits stored
        // (vocab logits of the statistics head, 2 GiB at C2: nontemporal)
        store_rows_bf16<EPI == SVAE_EPI_CE_STATS>((bf16*)p.C + cofs, p.ldc, m0 + wr * 128 + i * 16, p.M, n0 + wc * 64,
                                                  p.N, v, g, li);
      }
    }
    if constexpr (EPI == SVAE_EPI_CE_STATS) {
      const bool ragged = n0 + wc * 64 + 64 > p.N;   // wave-uniform
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (ragged && n0 + wc * 64 + j * 16 + 4 * g + e >= p.N) v[j][e] = -INFINITY;
          mx = fmaxf(mx, v[j][e]);
        }
      mx = max_x16_x32(mx);
      const float mc = mx == -INFINITY ? 0.f : mx * G3_LOG2E;
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) se += __builtin_amdgcn_exp2f(fmaf(v[j][e], G3_LOG2E, -mc));
      se = sum_x16_x32(se);
      if (g == 0) {
        sstat[(rl * 4 + wc) * 2] = mx;
        sstat[(rl * 4 + wc) * 2 + 1] = se;
      }
      const int lc = slabel[rl] - (n0 + wc * 64);   // label column within this wave's 64
      if (m < p.M && lc >= 0 && lc < 64 && ((lc >> 2) & 3) == g) {
        float x = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (j == (lc >> 4) && e == (lc & 3)) x = v[j][e];
        p.label_logit[m] = x;
      }
    }
  }
  if constexpr (EPI == SVAE_EPI_CE_STATS) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int row = tid >> 1, hf = tid & 1, m = m0 + row;   // 512 threads: (row, 128-column half)
    if (m < p.M && n0 + 128 * hf < p.N) {
      const float* s = sstat + (row * 4 + 2 * hf) * 2;
      const float m1 = s[0], s1 = s[1], m2 = s[2], s2 = s[3];
      const float mm = fmaxf(m1, m2);
      const float e1 = m1 == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m1 - mm) * G3_LOG2E);
      const float e2 = m2 == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m2 - mm) * G3_LOG2E);
      float* part = (float*)p.aux + ((long long)m * p.tiles_n + bn * 2 + hf) * 2;
      part[0] = mm;
      part[1] = s1 * e1 + s2 * e2;
    }
  }
  if constexpr (EPI == SVAE_EPI_CE_PROB) {
    // tile-major partial sums aux[128-column tile][M]: a wave writes 64 consecutive rows of one tile (256 B runs;
    // a row-major [M][tiles] layout scatters 4-B writes 1 KiB apart, each a partial-line write)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int row = tid & 255, hf = tid >> 8, m = m0 + row;   // 512 threads: (128-column half, row)
    if (m < p.M && n0 + 128 * hf < p.N)
      ((float*)p.aux)[(long long)(bn * 2 + hf) * p.M + m] = sstat[row * 4 + 2 * hf] + sstat[row * 4 + 2 * hf + 1];
  }
}

// ROWSCALE_GATHER (the vocabulary head's dX = dlogits . W with dlogits = r (x) P - q (x) onehot, never stored):
// C bf16 [m][n] = row_a[m] * acc - row_b[m] * gather[labels[m]][n]. The permlane-swapped 8-column layout of
// store_pair_bf16 with 16-B gather loads of the same 8 columns; row i + 1's gather rows are loaded before row i's
// stores (vmcnt retires in issue order).
__device__ __forceinline__ void g3_rowscale_gather_epilogue(const GP& p, const f32x4 (&acc)[8][4], const int* slabel,
                                                            const float* sra, const float* srb, int m0, int n0, int wr,
                                                            int wc, int lane) {
  const int g = lane >> 4, li = lane & 15;
  const int nb = n0 + wc * 64;
  const int cs = ((g & 1) ? 16 : 0) + ((g & 2) ? 8 : 0);
  auto ld_row = [&](int i, u32x4 (&r)[2]) {
    const int rl = wr * 128 + i * 16 + li, m = m0 + rl, lab = slabel[rl];
    const bool on = m < p.M && lab != 0 && srb[rl] != 0.f;
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      const int n = nb + 32 * jp + cs;
      r[jp] = (on && n + 8 <= p.N) ? *(const u32x4*)(p.gather + (long long)lab * p.ldg + n) : (u32x4){0u, 0u, 0u, 0u};
    }
  };
  u32x4 cur[2], nxt[2];
  ld_row(0, cur);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i + 1 < 8) ld_row(i + 1, nxt);
    const int rl = wr * 128 + i * 16 + li, m = m0 + rl;
    const float ra = sra[rl] * p.alpha, rb = srb[rl];
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      const f32x4 x = acc[i][2 * jp], y = acc[i][2 * jp + 1];
      float w[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(x[e]), __float_as_uint(y[e]), false, false);
        w[e] = __uint_as_float(sw[0]);
        w[4 + e] = __uint_as_float(sw[1]);
      }
      const bf16x8 gv = __builtin_bit_cast(bf16x8, cur[jp]);
      const u32x4 o = {pack_bf16x2(ra * w[0] - rb * (float)gv[0], ra * w[1] - rb * (float)gv[1]),
                       pack_bf16x2(ra * w[2] - rb * (float)gv[2], ra * w[3] - rb * (float)gv[3]),
                       pack_bf16x2(ra * w[4] - rb * (float)gv[4], ra * w[5] - rb * (float)gv[5]),
                       pack_bf16x2(ra * w[6] - rb * (float)gv[6], ra * w[7] - rb * (float)gv[7])};
      // (half lines: the whole-line merge cost the head dX a spill and ~8 us)
      const int n = nb + 32 * jp + cs;
      if (m < p.M && n + 8 <= p.N) *(u32x4*)((bf16*)p.C + (long long)m * p.ldc + n) = o;
      else if (m < p.M && n < p.N) *(u32x2*)((bf16*)p.C + (long long)m * p.ldc + n) = (u32x2){o[0], o[1]};
    }
    if (i + 1 < 8) {
      cur[0] = nxt[0];
      cur[1] = nxt[1];
    }
  }
}

// Register epilogue for the epilogues that read another tensor: f32 out (+resid), f32 accumulate, dropout +
// resid, and bf16 x GELU' (the FFN backward). The operand rows for fragment row i + 1 are loaded before row i's
// stores are issued, so the compiler's counted waits never drain the stores (vmcnt retires in issue order).
// (A two-row-ahead variant measured no faster in the step.)
// f32 rows: one 16-B load per fragment (16 rows x 64 B per instruction), whole-line stores (store_rows_f32); GELU':
// the permlane-swapped 8-column layout of store_pair_bf16, with the matching 16-B aux loads, whole-line stores.
template <int EPI>
__device__ __forceinline__ void g3_reg_epilogue_ld(const GP& p, const f32x4 (&acc)[8][4], const float* sbias, int m0,
                                                   int n0, int batch, int split, int wr, int wc, int lane) {
  const long long cofs = (long long)batch * p.sC + split * p.slab;
  const int g = lane >> 4, li = lane & 15;
  const int nb = n0 + wc * 64;                  // this wave's first column
  f32x4 b4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) b4[j] = *(const f32x4*)(sbias + wc * 64 + j * 16 + 4 * g);
  if constexpr (EPI == G3_EPI_BF16_DELTA) {
    // bf16 out, and per (row, head) the sum of bf16(C) * O32 over the head's columns (the attention backward's delta,
    // attention.py:51-105). A wave's 64 columns hold at most two heads (hd 64 / 96 / 128, head bounds on 16-column
    // fragments): one partial per head, reduced over the 4 lane groups, added by f32 atomics into the zeroed delta
    // -- at most two contributions per (row, head) onto 0, so the order does not change the sum. The O32 rows of
    // fragment row i + 1 are loaded before row i's stores (vmcnt retires in issue order).
    const int H = p.N / p.delta_hd;
    const int hA = nb / p.delta_hd;
    auto ld_row = [&](int i, f32x4 (&r)[4]) {
      const int m = m0 + wr * 128 + i * 16 + li;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nb + j * 16 + 4 * g;
        r[j] = (m < p.M && n < p.N) ? *(const f32x4*)(p.delta_o32 + (long long)m * p.ld_o32 + n)
                                    : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    };
    f32x4 cur[4], nxt[4];
    ld_row(0, cur);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i + 1 < 8) ld_row(i + 1, nxt);
      const int m = m0 + wr * 128 + i * 16 + li;
      f32x4 x[4];
      float sA = 0.f, sB = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[j] = p.alpha * acc[i][j] + b4[j];
        float dj = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) dj = fmaf((float)f2bf(x[j][e]), cur[j][e], dj);
        if ((nb + 16 * j) / p.delta_hd == hA) sA += dj;
        else sB += dj;
      }
      store_rows_bf16<false>((bf16*)p.C + cofs, p.ldc, m0 + wr * 128 + i * 16, p.M, nb, p.N, x, g, li);
      sA = sum_x16_x32(sA);
      sB = sum_x16_x32(sB);
      if (g == 0 && m < p.M && nb < p.N) {
        const int b = m / p.delta_seq, q = m - b * p.delta_seq;
        atomicAdd(p.delta + ((long long)b * H + hA) * p.delta_seq + q, sA);
        if ((nb + 63) / p.delta_hd != hA && hA + 1 < H) atomicAdd(p.delta + ((long long)b * H + hA + 1) * p.delta_seq + q, sB);
      }
      if (i + 1 < 8) {
#pragma unroll
        for (int j = 0; j < 4; ++j) cur[j] = nxt[j];
      }
    }
    return;
  } else if constexpr (EPI == SVAE_EPI_GELU_BWD) {
    const int cs = ((g & 1) ? 16 : 0) + ((g & 2) ? 8 : 0);   // column of this lane's 8 within a 32-column pair
    auto ld_row = [&](int i, u32x4 (&r)[2]) {
      const int m = m0 + wr * 128 + i * 16 + li;
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int n = nb + 32 * jp + cs;
        r[jp] = (m < p.M && n + 8 <= p.N) ? *(const u32x4*)((const bf16*)p.aux + (long long)m * p.ldaux + n)
                                          : (u32x4){0u, 0u, 0u, 0u};
      }
    };
    u32x4 cur[2], nxt[2];
    ld_row(0, cur);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i + 1 < 8) ld_row(i + 1, nxt);
      u32x4 o[2];
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const f32x4 x = p.alpha * acc[i][2 * jp] + b4[2 * jp], y = p.alpha * acc[i][2 * jp + 1] + b4[2 * jp + 1];
        float w[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(x[e]), __float_as_uint(y[e]), false, false);
          w[e] = __uint_as_float(s[0]);
          w[4 + e] = __uint_as_float(s[1]);
        }
        const bf16x8 a = __builtin_bit_cast(bf16x8, cur[jp]);
        o[jp] = (u32x4){pack_bf16x2(w[0] * (float)a[0], w[1] * (float)a[1]), pack_bf16x2(w[2] * (float)a[2], w[3] * (float)a[3]),
                        pack_bf16x2(w[4] * (float)a[4], w[5] * (float)a[5]), pack_bf16x2(w[6] * (float)a[6], w[7] * (float)a[7])};
      }
      store_rows_w16<false>((bf16*)p.C + cofs, p.ldc, m0 + wr * 128 + i * 16, p.M, nb, p.N, o, g, li);
      if (i + 1 < 8) {
        cur[0] = nxt[0];
        cur[1] = nxt[1];
      }
    }
    return;
  } else {
    // f32 out: F32 (+resid when given), F32_ACC (+C), DROPOUT_RESID (dropout then +resid), SLAB (nothing added)
    const float* src = EPI == SVAE_EPI_F32_ACC ? (const float*)p.C + cofs : p.resid;
    const long long lds_ = EPI == SVAE_EPI_F32_ACC ? p.ldc : p.ldr;
    const bool ld = EPI != G3_EPI_SLAB && src != nullptr;
    auto ld_row = [&](int i, f32x4 (&r)[4]) {
      const int m = m0 + wr * 128 + i * 16 + li;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nb + j * 16 + 4 * g;
        r[j] = (ld && m < p.M && n < p.N) ? *(const f32x4*)(src + (long long)m * lds_ + n) : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    };
    f32x4 cur[4], nxt[4];
    if constexpr (EPI != G3_EPI_SLAB) ld_row(0, cur);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (EPI != G3_EPI_SLAB && i + 1 < 8) ld_row(i + 1, nxt);
      const int m = m0 + wr * 128 + i * 16 + li;
      f32x4 x[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nb + j * 16 + 4 * g;
        x[j] = p.alpha * acc[i][j] + b4[j];
        if constexpr (EPI == SVAE_EPI_DROPOUT_RESID) {
          if (p.drop_p > 0.f) dropout4(p, x[j], m, n);
        }
        if constexpr (EPI != G3_EPI_SLAB) x[j] += cur[j];
      }
      if constexpr (EPI == SVAE_EPI_F32_ACC) {   // (the head dW: the merge's registers cost spills, 1185 -> 1211 us)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = nb + j * 16 + 4 * g;
          if (m < p.M && n < p.N) *(f32x4*)((float*)p.C + cofs + (long long)m * p.ldc + n) = x[j];
        }
      } else {
        store_rows_f32((float*)p.C + cofs, p.ldc, m0 + wr * 128 + i * 16, p.M, nb, p.N, x, g, li);
        // DROPOUT_RESID with aux: also the bf16 copy (the last decoder layer's output = the vocabulary head's input,
        // which then needs no separate cast pass over [T, d])
        if constexpr (EPI == SVAE_EPI_DROPOUT_RESID) {
          if (p.aux) store_rows_bf16<false>((bf16*)p.aux, p.ldaux, m0 + wr * 128 + i * 16, p.M, nb, p.N, x, g, li);
        } else if constexpr (EPI == SVAE_EPI_F32) {
          // F32 with aux: also bf16(dropout(C)) (the vocabulary head's d x -> the top decoder layer's FFN-output
          // gradient, as svae_dropout_bwd_cast would make it from C)
          if (p.aux) {
            if (p.drop_p > 0.f) {
#pragma unroll
              for (int j = 0; j < 4; ++j) dropout4(p, x[j], m, nb + j * 16 + 4 * g);
            }
            store_rows_bf16<false>((bf16*)p.aux, p.ldaux, m0 + wr * 128 + i * 16, p.M, nb, p.N, x, g, li);
          }
        }
      }
      if (EPI != G3_EPI_SLAB && i + 1 < 8) {
#pragma unroll
        for (int j = 0; j < 4; ++j) cur[j] = nxt[j];
      }
    }
  }
}

struct G3Tile {
  int m0, n0, bn, batch, split, kbeg, kend, nk;
  const bf16* A; const bf16* B;
};

__device__ __forceinline__ G3Tile g3_tile(const GP& p, int t3) {
  G3Tile T;
  const int tiles = p.tn2 * p.tm2;
  const int z = t3 / tiles, t = t3 - z * tiles;
  T.batch = z / p.splits;
  T.split = z - T.batch * p.splits;
  int bm, bn;
  group_tile(t, p.tm2, p.tn2, p.group, bm, bn);
  T.bn = bn;
  T.m0 = bm * 256;
  T.n0 = bn * 256;
  T.kbeg = T.split * p.kchunk;
  T.kend = min(p.K, T.kbeg + p.kchunk);
  T.nk = T.kend > T.kbeg ? (T.kend - T.kbeg + 63) / 64 : 0;
  T.A = p.A + T.batch * p.sA;
  T.B = p.B + T.batch * p.sB;
  return T;
}

// stores issued by every wave of an interior tile's epilogue (lower bound over the epilogues): the next tile's first
// K-step waits vmcnt(G3_EPI_STORES) instead of 0, so those stores drain under its MFMAs
constexpr int G3_EPI_STORES = 16;

#ifdef SVAE_STAMPS
// diagnostic build only (make STAMPS=1 -> libsvae_stamps.so): s_memtime at tile start / after the K loop / after
// the epilogue, for blocks 0..7 and their first 96 tiles
__device__ unsigned long long svae_stamps[8][96][3];
__device__ unsigned long long svae_rt[1024][2];   // per block: entry, exit (s_memrealtime, 100 MHz)
#define G3_STAMP(k) \
  do { if (blockIdx.x < 8 && tid == 0 && ntile < 96) svae_stamps[blockIdx.x][ntile][k] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define G3_STAMP(k) ((void)0)
#endif
#ifndef SVAE_KW_FORM
#define SVAE_KW_FORM 0
#endif
#ifndef SVAE_KW_PRE
#define SVAE_KW_PRE 1   // form 0's weights loaded at the K-tile top by counted asm loads (0: at the use, no DMA stagger)
#endif

// Vector-memory operations every wave issues unconditionally in the epilogue of an interior 256 x 256 tile (stores
// and atomics only: loads a lane may branch around are not counted), i.e. after the next tile's first K-tile DMA.
// The next tile's relaxed first wait, vmcnt(G3_EPI_STORES), covers that DMA only if at least G3_EPI_STORES of them
// are younger (vmcnt retires in issue order); gemm256_run static_asserts it per instantiation.
template <int EPI>
constexpr int g3_epi_vmem_ops() {
  switch (EPI) {
    case SVAE_EPI_BF16:
    case G3_EPI_BF16_DELTA:
    case SVAE_EPI_ROTARY_BF16:
    case SVAE_EPI_CE_STATS:           // with C (the host clears p.relaxed when C == NULL: no logits stored)
    case SVAE_EPI_ROWSCALE_GATHER:
    case SVAE_EPI_GELU_BWD:
      return 8 * 2;                   // 8 fragment rows x 2 permlane-paired 16-B stores
    case SVAE_EPI_CE_PROB:
      return 8 * 2 + 1;               // + the tile's per-row partial sums
    case SVAE_EPI_GELU:
      return 8 * 2 * 2;               // + the GELU' aux
    case SVAE_EPI_F32:
    case SVAE_EPI_F32_ACC:
    case SVAE_EPI_DROPOUT_RESID:
    case G3_EPI_ACC_KW:
    case G3_EPI_F32_KW:
    case G3_EPI_SLAB:
      return 8 * 4;                   // 8 fragment rows x 4 16-B f32 stores
    default:
      return 0;
  }
}

// The gemm256 block program over the tiles of one GEMM: block `blk` of `nwg` blocks working on p (the plain kernel
// passes blockIdx.x / gridDim.x; the paired kernel gives each GEMM its own range of blocks).
template <bool AT, bool BT, int EPI>
__device__ __forceinline__ void gemm256_run(const GP& p, int blk, int nwg) {
  // 2 ring stages + a side area: the epilogue's per-tile bias (256 f32), CE labels (256 i32) and CE row statistics
  // ([256 rows][4 column waves][max, sum]); one array
  static_assert(g3_epi_vmem_ops<EPI>() >= G3_EPI_STORES, "the relaxed first wait would not cover the prefetch DMA");
  // ACC_KW with SVAE_KW_FORM > 0 (diagnostic builds; the product, form 0, loads the weights from global memory):
  // [stage][wave] k-weight slots, each wave DMAs the weights of a K-tile into its OWN slot -- form 1: 64 dwords
  // (buffer_load_dword lds) after the side area (138 KiB); form 2: 16-B pieces (buffer_load_dwordx4 lds, lanes 0-15)
  // after the side area; form 3: 64 dwords at offset 0, the ring moved up by 4 KiB (all DMA below 132 KiB)
  constexpr bool IS_KW = EPI == G3_EPI_ACC_KW || EPI == G3_EPI_F32_KW;
  constexpr int KW_FORM = IS_KW ? SVAE_KW_FORM : 0;
  constexpr int KW_SLOT = KW_FORM == 2 ? 1024 : 256;
  constexpr int KW_BYTES = KW_FORM ? 2 * 8 * KW_SLOT : 0;
  constexpr int RING_OFF = KW_FORM == 3 ? KW_BYTES : 0;
  constexpr int KW_OFF = KW_FORM == 3 ? 0 : 2 * G3_STAGE + 2048 + 8192;
  __shared__ __attribute__((aligned(16))) char smem[2 * G3_STAGE + 2048 + 8192 + KW_BYTES];
  char* ring = smem + RING_OFF;
  float* sbias = (float*)(ring + 2 * G3_STAGE);
  int* slabel = (int*)(ring + 2 * G3_STAGE + 1024);
  float* sstat = (float*)(ring + 2 * G3_STAGE + 2048);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  // XCD-aware bijective remap of the block id; block b then walks tiles b, b + G, b + 2G, ... (G = nwg):
  // with G = 256 every XCD runs one contiguous N-fastest range of tiles at a time. (blk % 8 is the XCD: the paired
  // kernel's block ranges start at multiples of 8.)
  int bid = blk;
  if (nwg >= 16) {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, idx = bid / 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  int t3 = bid;
  if (t3 >= p.total3) return;
  G3Tile T = g3_tile(p, t3);
  // ACC_KW: the 64 k-weights of a K-tile ride along with its operand pieces, one dword per lane into this wave's own
  // slot of the K-tile's stage; read after the same counted wait + barrier as the operands (no cross-wave hand-off)
  char* skw = smem + KW_OFF;
  auto kw_issue = [&](int k0, int kend, int stage) {
    if constexpr (KW_FORM == 1 || KW_FORM == 3) {
      const u32x4 kwr = buffer_rsrc(p.k_weight, 0x7FFFFFF0u);
      const int kk = k0 + lane_id_fresh();
      dma4_lds(kwr, skw + (stage * 8 + wave) * KW_SLOT, kk < kend ? kk * 4 : 0x7FFFFFF0);
    } else if constexpr (KW_FORM == 2) {
      const u32x4 kwr = buffer_rsrc(p.k_weight, 0x7FFFFFF0u);
      const int l = lane_id_fresh(), kk = k0 + 4 * l;
      dma16_lds(kwr, skw + (stage * 8 + wave) * KW_SLOT, l < 16 && kk < kend ? kk * 4 : 0x7FFFFFF0);
    }
  };
  const G3Src sa = g3_src<AT>(p.lda, wave, lane), sb = g3_src<BT>(p.ldb, wave, lane);
  int g = 0;   // K-tiles consumed so far by this block: the stage of K-tile g is g & 1
  if (T.nk > 0) {
    g3_issue<AT, BT>(p, T.A, T.B, sa, sb, T.m0, T.n0, T.kbeg, T.kend, ring, wave);
    kw_issue(T.kbeg, T.kend, 0);
  }

  bool relaxed = false;   // the previous tile was interior: its epilogue issued >= G3_EPI_STORES stores per wave
  int ntile = 0;
  (void)ntile;
  while (true) {
    G3_STAMP(0);
    const int t3n = t3 + nwg;
    const bool has_next = t3n < p.total3;
    float rsum[4] = {0.f, 0.f, 0.f, 0.f};
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    // the next tile's first K-tile is prefetched by the last K-tile of this one (8 DMA pieces per wave)
    const bool next_dma = has_next && g3_tile(p, t3n).nk > 0;
    for (int kt = 0; kt < T.nk; ++kt, ++g) {
      // this wave's pieces of K-tile g landed (after an interior epilogue, up to G3_EPI_STORES younger stores may
      // still be in flight: vmcnt retires in issue order)
      if (kt == 0 && relaxed) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G3_EPI_STORES) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();                      // everyone's landed; K-tile g-1 (other stage) consumed
      const char* la = ring + (g & 1) * G3_STAGE;
      const char* lb = la + G3_T;
      char* nxt = ring + ((g + 1) & 1) * G3_STAGE;
      const bool do_rs = AT && p.a_rowsum && T.bn < 2;
      // p.dma_stagger: the two waves of a SIMD (wr 0 and 1, same wc) issue their pieces of the next K-tile at different
      // times -- wr 0 here, wr 1 after its first MFMA quadrant -- so one wave's DMA issue runs beside the other's MFMAs
      // (the k-weighted forms: form 0 loads the weights from global memory at the use, whose wait would also wait for
      // the late pieces, so no stagger; the LDS-slot diagnostic forms stagger)
      // ACC_KW form 0: the K-tile's 64 weights are loaded here, one dword per lane, BEFORE this K-tile's 8 DMA pieces
      // (issued next, or after the first quadrant by a late wave; the block's very last K-tile issues 8 out-of-range
      // pieces instead, so the count holds), by an asm buffer load the compiler does not track; the use waits vmcnt(8)
      // -- those pieces may stay in flight, so the DMA stagger applies to the k-weighted GEMM too -- and takes each
      // lane's 8 weights of a k-step by ds_bpermute (1 VGPR live across the quadrants instead of 8 or 16; a
      // compiler-visible load made hipcc wait vmcnt(0), draining the DMA, and the wider live forms spilled)
      const int ks0 = p.tn2 >= 2 ? T.bn : 0, ks1 = p.tn2 >= 2 ? T.bn + 1 : 2;
      const bool kw_pre = IS_KW && KW_FORM == 0 && SVAE_KW_PRE && do_rs;   // (block-uniform)
      float kw1 = 0.f;
      if (kw_pre) {
        const int kk = T.kbeg + kt * 64 + lane_id_fresh();
        const int off = kk < T.kend ? kk * 4 : 0x7FFFFFF0;
        const u32x4 kwr = buffer_rsrc(p.k_weight, 0x7FFFFFF0u);
        asm volatile("s_nop 4\n\tbuffer_load_dword %0, %1, %2, 0 offen" : "=&v"(kw1) : "v"(off), "s"(kwr) : "memory");
      }
      const bool late = (!IS_KW || KW_FORM > 0 || kw_pre) && p.dma_stagger && wr == 1 && kt + 1 < T.nk;   // (uniform)
      if (kt + 1 < T.nk) {
        if (!late) g3_issue<AT, BT>(p, T.A, T.B, sa, sb, T.m0, T.n0, T.kbeg + (kt + 1) * 64, T.kend, nxt, wave);
        kw_issue(T.kbeg + (kt + 1) * 64, T.kend, (g + 1) & 1);   // (every wave here, late or not)
      } else if (next_dma) {   // the next tile's first K-tile, in flight during this tile's epilogue
        const G3Tile TN = g3_tile(p, t3n);
        g3_issue<AT, BT>(p, TN.A, TN.B, sa, sb, TN.m0, TN.n0, TN.kbeg, TN.kend, nxt, wave);
        kw_issue(TN.kbeg, TN.kend, (g + 1) & 1);
      } else if (kw_pre) {   // (see kw_pre: 8 pieces that read nothing, into the idle stage)
        const u32x4 rs = buffer_rsrc(p.A, 0x7FFFFFF0u);
#pragma unroll
        for (int i = 0; i < 8; ++i) dma16_lds(rs, nxt + (wave * 8 + i) * 1024, 0x7FFFFFF0);
      }
      // Quadrant walk (mh, nh) = (0,0) (0,1) (1,1) (1,0): A fragments of a half reused by two quadrants, B
      // fragments of a half by the turn. The next quadrant's fragment reads are issued ahead of the current
      // quadrant's MFMAs.
      bf16x8 a0[4][2], a1[4][2], b0[2][2], b1[2][2];
      // AT: sum_k A[m][k] (* k_weight[k]) from the A fragments already in registers (no extra LDS reads): lane l of
      // a fragment holds row 16i + (l & 15), k = 32 ks + 8 (l >> 4) + (0..7); column wave wc takes row groups
      // 2 wc, 2 wc + 1 of its wave row's eight (balanced over the SIMDs; a0's right after their last MFMA use),
      // summed over the lane groups at the end of the tile. ACC_KW: the lane's 8 weights per k-step are global loads
      // at the use (L2-resident; the compiler's wait for them also drains the next K-tile's DMA pieces issued before
      // them). Every LDS form measured (a ring filled by wave 0; each wave's own slot DMA'd with the K-tile's pieces,
      // forms 1-3 of SVAE_KW_FORM, kept for diagnostic builds) read stale weights now and then in the bit-exact test
      // (DESIGN §6); registers loaded a K-tile ahead spilled (34 VGPRs). The first two column tiles (blocks bn = 0, 1
      // hold the same A rows) split the work by k-step, so neither runs much longer than the blocks without row sums.
      auto rowsum2 = [&](const bf16x8 (&x)[2], const bf16x8 (&y)[2]) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          if (ks < ks0 || ks >= ks1) continue;   // (block-uniform)
          f32x4 k0 = {1.f, 1.f, 1.f, 1.f}, k1 = k0;
          if constexpr (KW_FORM > 0) {   // this wave's slot of the stage (zeros past kend)
            const float* kws = (const float*)(skw + ((g & 1) * 8 + wave) * KW_SLOT) + 32 * ks + 8 * (lane >> 4);
            k0 = *(const f32x4*)kws;
            k1 = *(const f32x4*)(kws + 4);
          } else if constexpr (IS_KW) {
            if (kw_pre) {   // (kw1 landed: the wait after the second quadrant)
              const int src0 = (32 * ks + 8 * (lane_id_fresh() >> 4)) * 4;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                k0[e] = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src0 + 4 * e, __builtin_bit_cast(int, kw1)));
                k1[e] = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src0 + 16 + 4 * e, __builtin_bit_cast(int, kw1)));
              }
            } else {        // (SVAE_KW_PRE=0 builds: loads at the use, the wait drains the DMA too: no stagger)
              const int kk = T.kbeg + kt * 64 + 32 * ks + 8 * (lane_id_fresh() >> 4);
              const int off = kk < T.kend ? kk * 4 : 0x7FFFFFF0;
              const u32x4 kwr = buffer_rsrc(p.k_weight, 0x7FFFFFF0u);
              asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %2, %3, 0 offen\n\t"
                           "buffer_load_dwordx4 %1, %2, %3, 0 offen offset:16\n\ts_waitcnt vmcnt(0)"
                           : "=&v"(k0), "=&v"(k1) : "v"(off), "s"(kwr) : "memory");
            }
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float kwe = e < 4 ? k0[e] : k1[e - 4];
            rsum[0] = fmaf((float)x[ks][e], kwe, rsum[0]);
            rsum[1] = fmaf((float)y[ks][e], kwe, rsum[1]);
          }
        }
      };
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) a0[i][ks] = g3_afrag<AT>(la, wr * 128 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) b0[j][ks] = g3_bfrag<BT>(lb, wc * 64 + j * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) b1[j][ks] = g3_bfrag<BT>(lb, wc * 64 + 32 + j * 16, ks, lane);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(b0[j][ks], a0[i][ks], acc[i][j]);
      if (late) {
        __builtin_amdgcn_sched_barrier(0);
        g3_issue<AT, BT>(p, T.A, T.B, sa, sb, T.m0, T.n0, T.kbeg + (kt + 1) * 64, T.kend, nxt, wave);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (!AT) {   // (AT: transposed A reads need the registers; load after the a0 quadrants)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) a1[i][ks] = g3_afrag<AT>(la, wr * 128 + 64 + i * 16, ks, lane);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][2 + j] = mfma16(b1[j][ks], a0[i][ks], acc[i][2 + j]);
      if constexpr (AT) {
        // kw1's one wait, for every wave here (a wait per use site let hipcc copy kw1 before the data landed)
        if (kw_pre) asm volatile("s_waitcnt vmcnt(8)" : "+v"(kw1) :: "memory");
        if (do_rs) {
          if (wc == 0) rowsum2(a0[0], a0[1]);
          else if (wc == 1) rowsum2(a0[2], a0[3]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) a1[i][ks] = g3_afrag<AT>(la, wr * 128 + 64 + i * 16, ks, lane);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[4 + i][2 + j] = mfma16(b1[j][ks], a1[i][ks], acc[4 + i][2 + j]);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[4 + i][j] = mfma16(b0[j][ks], a1[i][ks], acc[4 + i][j]);
      if constexpr (AT) {
        if (do_rs) {
          if (wc == 2) rowsum2(a1[0], a1[1]);
          else if (wc == 3) rowsum2(a1[2], a1[3]);
        }
      }
    }
    G3_STAMP(1);
    // epilogue operands into the side area, loaded before any store of this tile (the previous epilogue's reads of
    // the side area finished before this tile's first barrier)
    if (tid < 256) {
      const int n = T.n0 + tid, m = T.m0 + tid;
      sbias[tid] = (p.bias && n < p.N) ? p.bias[n] : 0.f;
      if (EPI == SVAE_EPI_CE_STATS || EPI == SVAE_EPI_CE_PROB || EPI == SVAE_EPI_ROWSCALE_GATHER)
        slabel[tid] = m < p.M ? p.labels[m] : 0;
      // CE_PROB: a row without a target gets offset +inf, so its P comes out exactly 0 from the exp2 (no select per
      // element)
      if (EPI == SVAE_EPI_CE_PROB) sstat[1024 + tid] = (m < p.M && p.labels[m] != 0) ? p.row_a[m] : INFINITY;
      if (EPI == SVAE_EPI_ROWSCALE_GATHER) sstat[1024 + tid] = m < p.M ? p.row_a[m] : 0.f;
      if (EPI == SVAE_EPI_ROWSCALE_GATHER) sstat[1280 + tid] = m < p.M ? p.row_b[m] : 0.f;
    }
    // every wave's reads of the last K-tile's stage are done: it becomes the epilogue's staging area
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if constexpr (AT) {
      if (p.a_rowsum && T.bn < 2) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float t = sum_x16_x32(rsum[h]);
          const int m = T.m0 + wr * 128 + (2 * wc + h) * 16 + (lane & 15);
          if ((lane >> 4) == 0 && m < p.M) atomicAdd(p.a_rowsum + m, t);
        }
      }
    }
    if constexpr (EPI == SVAE_EPI_BF16 || EPI == SVAE_EPI_GELU || EPI == SVAE_EPI_CE_STATS ||
                  EPI == SVAE_EPI_ROTARY_BF16 || EPI == SVAE_EPI_CE_PROB)
      g3_reg_epilogue<EPI>(p, acc, sbias, slabel, sstat, T.m0, T.n0, T.bn, T.batch, T.split, wr, wc, tid, lane);
    else if constexpr (EPI == SVAE_EPI_ROWSCALE_GATHER)
      g3_rowscale_gather_epilogue(p, acc, slabel, sstat + 1024, sstat + 1280, T.m0, T.n0, wr, wc, lane);
    else if constexpr (EPI == SVAE_EPI_F32 || EPI == SVAE_EPI_F32_ACC || EPI == SVAE_EPI_DROPOUT_RESID ||
                       EPI == SVAE_EPI_GELU_BWD || EPI == G3_EPI_BF16_DELTA)
      g3_reg_epilogue_ld<EPI>(p, acc, sbias, T.m0, T.n0, T.batch, T.split, wr, wc, lane);
    else if constexpr (EPI == G3_EPI_ACC_KW)
      g3_reg_epilogue_ld<SVAE_EPI_F32_ACC>(p, acc, sbias, T.m0, T.n0, T.batch, T.split, wr, wc, lane);
    else if constexpr (EPI == G3_EPI_F32_KW || EPI == G3_EPI_SLAB)
      g3_reg_epilogue_ld<G3_EPI_SLAB>(p, acc, sbias, T.m0, T.n0, T.batch, T.split, wr, wc, lane);
    else
      static_assert(EPI == G3_EPI_SLAB, "no gemm256 epilogue for this EPI");
    relaxed = p.relaxed && T.m0 + 256 <= p.M && T.n0 + 256 <= p.N;
    G3_STAMP(2);
    ++ntile;
    if (!has_next) break;
    const bool prefetched = T.nk > 0;
    t3 = t3n;
    T = g3_tile(p, t3);
    if (!prefetched && T.nk > 0) {   // (an empty split-K slice prefetched nothing)
      g3_issue<AT, BT>(p, T.A, T.B, sa, sb, T.m0, T.n0, T.kbeg, T.kend, ring + (g & 1) * G3_STAGE, wave);
      kw_issue(T.kbeg, T.kend, g & 1);
    }
  }
}

template <bool AT, bool BT, int EPI>
__global__ __launch_bounds__(512, 1) void gemm256_kernel(GP p) {
#ifdef SVAE_STAMPS
  // (diagnostic) every block's entry and exit on the chip-wide 100 MHz clock: the launch's start skew and tail
  if (threadIdx.x == 0 && blockIdx.x < 1024) svae_rt[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
#endif
  gemm256_run<AT, BT, EPI>(p, blockIdx.x, gridDim.x);
#ifdef SVAE_STAMPS
  if (threadIdx.x == 0 && blockIdx.x < 1024) svae_rt[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
#endif
}

// Two independent GEMMs in one launch (the weight gradients of two layers of one transformer block, split-K slab
// mode): blocks [0, nb0) run p[0], the rest p[1]. Each GEMM then needs only half the split-K slices to fill the
// chip, which halves its slab bytes (written by the epilogue, read by slab_reduce) and shares one launch's
// ramp-up and tail between the two.
struct GP2 {
  GP p[2];
  int nb0;   // a multiple of 8
};

template <bool AT, bool BT, int EPI>
__global__ __launch_bounds__(512, 1) void gemm256_pair_kernel(GP2 q) {
  // one inlined copy of the block program over the selected GEMM's parameters (two copies, one per GEMM, kept both
  // parameter sets in SGPRs: 185 SGPR spills)
  const int b = blockIdx.x;
  const int sel = b < q.nb0 ? 0 : 1;
  gemm256_run<AT, BT, EPI>(q.p[sel], sel ? b - q.nb0 : b, sel ? (int)gridDim.x - q.nb0 : q.nb0);
}

// ===================================================================================================
// gemm_skinny: M <= 64 rows (the encoder bottleneck layer, q(z|x), the z projections: one row per sequence).
// A 128-row tile leaves such a GEMM to a handful of blocks that walk all of K serially (a 64 x 512 x 2048 dropout +
// residual GEMM took 33 us). Here a block owns 32 columns, its 16 waves split K into contiguous slices (fragments
// loaded straight from global memory, the next k-step's loads issued before the current MFMAs), the 16 partial
// 64 x 32 tiles are summed in LDS in a fixed order and 512 threads run the epilogue (4 columns of one row each).
// (8 waves: 20.8 us for the 64 x 512 x 2048 dropout + residual GEMM, the k-step latency chain.)
// A [M][K] and B [N][K] K-contiguous, K % 8 == 0.
constexpr int SK_BN = 32, SK_WAVES = 16;

template <int EPI>
__global__ __launch_bounds__(1024) void gemm_skinny_kernel(GP p) {
  __shared__ __attribute__((aligned(16))) float red[SK_WAVES][64][SK_BN + 4];
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n0 = blockIdx.x * SK_BN;
  const int nks = (p.K + 31) / 32;                       // k-steps of 32
  const int per = (nks + SK_WAVES - 1) / SK_WAVES;
  const int ks0 = wave * per, ks1 = min(nks, ks0 + per);
  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // lane's fragment rows / columns and the k offset of its 8 elements
  auto load = [&](int ks, bf16x8 (&a)[4], bf16x8 (&b)[2]) {
    const int k = ks * 32 + 8 * g;
    const bool kok = k < p.K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = 16 * i + li;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (kok && m < p.M) v = *(const u32x4*)(p.A + (long long)m * p.lda + k);
      a[i] = __builtin_bit_cast(bf16x8, v);
    }
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int n = n0 + 16 * jj + li;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (kok && n < p.N) v = *(const u32x4*)(p.B + (long long)n * p.ldb + k);
      b[jj] = __builtin_bit_cast(bf16x8, v);
    }
  };
  if (ks0 < ks1) {
    bf16x8 a[4], b[2], an[4], bn[2];
    load(ks0, a, b);
    for (int ks = ks0; ks < ks1; ++ks) {
      if (ks + 1 < ks1) load(ks + 1, an, bn);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) acc[i][jj] = mfma16(b[jj], a[i], acc[i][jj]);
      if (ks + 1 < ks1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = an[i];
        b[0] = bn[0];
        b[1] = bn[1];
      }
    }
  }
  // acc[i][jj]: row 16 i + li, columns 16 jj + 4 g + (0..3)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) *(f32x4*)&red[wave][16 * i + li][16 * jj + 4 * g] = acc[i][jj];
  __syncthreads();
  const int row = tid >> 3, c4 = (tid & 7) * 4, m = row, n = n0 + c4;
  if (tid >= 512 || m >= p.M || n >= p.N) return;
  f32x4 x = *(const f32x4*)&red[0][row][c4];
#pragma unroll
  for (int w = 1; w < SK_WAVES; ++w) x += *(const f32x4*)&red[w][row][c4];
  x *= p.alpha;
  if (p.bias) x += *(const f32x4*)(p.bias + n);
  if constexpr (EPI == SVAE_EPI_F32 || EPI == SVAE_EPI_DROPOUT_RESID) {
    if constexpr (EPI == SVAE_EPI_DROPOUT_RESID) {
      if (p.drop_p > 0.f) dropout4(p, x, m, n);
    }
    if (p.resid) x += *(const f32x4*)(p.resid + (long long)m * p.ldr + n);
    *(f32x4*)((float*)p.C + (long long)m * p.ldc + n) = x;
    if (p.aux) {   // DROPOUT_RESID: bf16(C); F32: bf16(dropout(C))
      if (EPI == SVAE_EPI_F32 && p.drop_p > 0.f) dropout4(p, x, m, n);
      *(bf16x4*)((bf16*)p.aux + (long long)m * p.ldaux + n) = (bf16x4){f2bf(x[0]), f2bf(x[1]), f2bf(x[2]), f2bf(x[3])};
    }
  } else if constexpr (EPI == SVAE_EPI_GELU) {
    f32x2 g0, d0, g1, d1;
    gelu_pair2((f32x2){x[0], x[1]}, g0, d0);
    gelu_pair2((f32x2){x[2], x[3]}, g1, d1);
    *(bf16x4*)((bf16*)p.C + (long long)m * p.ldc + n) = (bf16x4){f2bf(g0[0]), f2bf(g0[1]), f2bf(g1[0]), f2bf(g1[1])};
    *(bf16x4*)((bf16*)p.aux + (long long)m * p.ldaux + n) = (bf16x4){f2bf(d0[0]), f2bf(d0[1]), f2bf(d1[0]), f2bf(d1[1])};
  } else if constexpr (EPI == SVAE_EPI_GELU_BWD) {
    const bf16x4 a4 = *(const bf16x4*)((const bf16*)p.aux + (long long)m * p.ldaux + n);
    *(bf16x4*)((bf16*)p.C + (long long)m * p.ldc + n) =
        (bf16x4){f2bf(x[0] * (float)a4[0]), f2bf(x[1] * (float)a4[1]), f2bf(x[2] * (float)a4[2]), f2bf(x[3] * (float)a4[3])};
  } else {
    *(bf16x4*)((bf16*)p.C + (long long)m * p.ldc + n) = (bf16x4){f2bf(x[0]), f2bf(x[1]), f2bf(x[2]), f2bf(x[3])};
  }
}

// C[m][n] += sum over splits of slab[s][m][n] (slab rows of N floats); 4 columns per thread
struct SlabRed {
  const float* slab;
  float* C;
  int M, N;
  long long ldc;
  int splits;
};
__device__ __forceinline__ void slab_reduce_range(const SlabRed& r, int blk, int nblk) {
  const int N4 = r.N / 4;
  const long long total = (long long)r.M * N4, plane = (long long)r.M * r.N;
  for (long long i = (long long)blk * 256 + threadIdx.x; i < total; i += (long long)nblk * 256) {
    const long long m = i / N4;
    const int n = (int)(i - m * N4) * 4;
    const float* src = r.slab + m * r.N + n;
    f32x4 acc = *(const f32x4*)src;
    for (int s = 1; s < r.splits; ++s) acc += *(const f32x4*)(src + s * plane);
    f32x4* dst = (f32x4*)(r.C + m * r.ldc + n);
    *dst = *dst + acc;
  }
}
__global__ __launch_bounds__(256) void slab_reduce_kernel(SlabRed r) { slab_reduce_range(r, blockIdx.x, gridDim.x); }
// the two slab reductions of a paired dW launch in one launch: blocks [0, nb0) take r0, the rest r1 (one launch
// fewer per pair: ~1.6 us of GPU-side launch cost each, scripts/bubble_probe.py)
__global__ __launch_bounds__(256) void slab_reduce2_kernel(SlabRed r0, SlabRed r1, int nb0) {
  if ((int)blockIdx.x < nb0) slab_reduce_range(r0, blockIdx.x, nb0);
  else slab_reduce_range(r1, blockIdx.x - nb0, (int)gridDim.x - nb0);
}

}  // namespace

static SlabRed slab_red(const svae_gemm_desc* d) {
  return SlabRed{(const float*)d->aux, (float*)d->C, d->M, d->N, (long long)d->ldc, d->splits};
}
static long long slab_blocks(const svae_gemm_desc* d) {
  return std::min(4096LL, ((long long)d->M * (d->N / 4) + 255) / 256);
}
static int launch_slab_reduce(const svae_gemm_desc* d, hipStream_t s) {
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)slab_blocks(d)), dim3(256), 0, s, slab_red(d));
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

static int validate_desc(const svae_gemm_desc* d) {
  if (!d || !d->A || !d->B || (!d->C && d->epi != SVAE_EPI_CE_STATS)) return SVAE_EINVAL;
  const bool epi_new = d->epi == SVAE_EPI_CE_PROB || d->epi == SVAE_EPI_ROWSCALE_GATHER;
  if (d->M <= 0 || d->N <= 0 || d->K <= 0 || d->batch <= 0 || d->splits <= 0) return SVAE_EINVAL;
  if ((d->K % 8 && !(d->a_t && d->b_t)) || d->lda % 8 || d->ldb % 8) return SVAE_EINVAL;
  if (d->a_t && d->M % 8) return SVAE_EINVAL;
  if (d->b_t && d->N % 8) return SVAE_EINVAL;
  if (((uintptr_t)d->A | (uintptr_t)d->B) & 15) return SVAE_EINVAL;
  if (d->batch_stride_a % 8 || d->batch_stride_b % 8) return SVAE_EINVAL;
  if (d->epi < 0 || d->epi > SVAE_EPI_ROWSCALE_GATHER) return SVAE_EINVAL;
  // the P-head epilogues (CE_PROB, ROWSCALE_GATHER) and weighted row sums exist in the 256x256 kernel only
  if (epi_new && (d->a_t || d->splits != 1 || d->batch != 1 || !d->labels || !d->row_a)) return SVAE_EINVAL;
  if (d->epi == SVAE_EPI_CE_PROB && !d->aux) return SVAE_EINVAL;
  if (d->epi == SVAE_EPI_ROWSCALE_GATHER && (!d->row_b || !d->gather || d->ldg % 8 || ((uintptr_t)d->gather & 15)))
    return SVAE_EINVAL;
  // k-weighted row sums: one split (F32_ACC), or split-K slab mode (F32_ATOMIC with aux)
  if (d->k_weight && (!d->a_rowsum || !d->a_t || (d->splits != 1 && !(d->epi == SVAE_EPI_F32_ATOMIC && d->aux))))
    return SVAE_EINVAL;
  if (d->epi == SVAE_EPI_ROTARY_BF16 && (!d->rot_tab || d->rot_d <= 0 || d->rot_seq <= 0)) return SVAE_EINVAL;
  if ((d->epi == SVAE_EPI_GELU || d->epi == SVAE_EPI_GELU_BWD || d->epi == SVAE_EPI_CE_STATS) && !d->aux)
    return SVAE_EINVAL;
  if (d->epi == SVAE_EPI_DROPOUT_RESID && !d->resid) return SVAE_EINVAL;
  // DROPOUT_RESID's / F32's optional bf16 copy in aux: one batch, 16-B aligned rows
  if ((d->epi == SVAE_EPI_DROPOUT_RESID || d->epi == SVAE_EPI_F32) && d->aux &&
      (d->batch != 1 || d->ldaux % 8 || ((uintptr_t)d->aux & 15)))
    return SVAE_EINVAL;
  if (d->epi == SVAE_EPI_CE_STATS && (!d->labels || !d->label_logit || d->splits != 1)) return SVAE_EINVAL;
  if (d->splits > 1 && d->epi != SVAE_EPI_F32_ATOMIC) return SVAE_EINVAL;
  if (d->a_rowsum && !d->a_t) return SVAE_EINVAL;
  // vectorised epilogue: 16-B aligned rows of C / resid / aux
  if (d->N % 4 || d->ldc % 8 || ((uintptr_t)d->C & 15) || (d->resid && (d->ldr % 4 || ((uintptr_t)d->resid & 15))))
    return SVAE_EINVAL;
  if ((d->epi == SVAE_EPI_GELU || d->epi == SVAE_EPI_GELU_BWD) && (d->ldaux % 8 || ((uintptr_t)d->aux & 15)))
    return SVAE_EINVAL;
  if (d->epi == SVAE_EPI_ROTARY_BF16 && (d->rot_d % 4 || d->rot_cols % 4)) return SVAE_EINVAL;

  return SVAE_OK;
}

static void fill_gp(const svae_gemm_desc* d, GP& p) {
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
  p.a_rowsum = d->a_rowsum;
  p.k_weight = d->k_weight;
  p.row_a = d->row_a; p.row_b = d->row_b;
  p.gather = (const bf16*)d->gather; p.ldg = d->ldg;
  p.epi = d->epi;
  p.slab = 0;
  p.dma_stagger = 0;
  p.delta = d->delta; p.delta_o32 = d->delta_o32; p.ld_o32 = d->ld_o32;
  p.delta_hd = d->delta_hd; p.delta_seq = d->delta_seq;
}

// delta[(b * H + h) * seq + q] = sum_c bf16 C[m][h * hd + c] * o32[m][h * hd + c] (m = b * seq + q), one wave per
// (row, head) -- svae_gemm's delta for the GEMMs that do not run the 256 x 256 kernel (its epilogue does it there)
__global__ __launch_bounds__(256) void gemm_delta_kernel(const bf16* __restrict__ C, long long ldc,
                                                         const float* __restrict__ o32, long long ldo, int M, int H,
                                                         int hd, int seq, float* __restrict__ delta) {
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (gw >= M * H) return;
  const int m = gw / H, h = gw - m * H;
  float s = 0.f;
  for (int c = lane * 4; c < hd; c += 256) {
    const bf16x4 a = *(const bf16x4*)(C + (long long)m * ldc + h * hd + c);
    const f32x4 o = *(const f32x4*)(o32 + (long long)m * ldo + h * hd + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) s = fmaf((float)a[e], o[e], s);
  }
  s = wave_sum(s);
  const int b = m / seq, q = m - b * seq;
  if (lane == 0) delta[((long long)b * H + h) * seq + q] = s;
}

static int gemm_run(const svae_gemm_desc* d, svae_stream_t stream, bool* fused_delta);

SVAE_EXPORT int svae_gemm(const svae_gemm_desc* d, svae_stream_t stream) {
  if (!d || !d->delta) return gemm_run(d, stream, nullptr);
  // the attention backward's delta alongside the dO GEMM (svae_gemm_desc.delta)
  if (d->epi != SVAE_EPI_BF16 || d->splits != 1 || d->batch != 1 || d->a_t || !d->delta_o32 || !d->C ||
      d->delta_hd <= 0 || d->delta_hd % 16 || d->N % d->delta_hd || d->delta_seq <= 0 || d->M % d->delta_seq ||
      d->ld_o32 < d->N || d->ld_o32 % 4 || ((uintptr_t)d->delta_o32 & 15) || ((uintptr_t)d->C & 7))
    return SVAE_EINVAL;
  bool fused = false;
  if (const int rc = gemm_run(d, stream, &fused)) return rc;
  if (!fused) {
    const int H = d->N / d->delta_hd;
    hipLaunchKernelGGL(gemm_delta_kernel, dim3((unsigned)(((long long)d->M * H + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, (const bf16*)d->C, (long long)d->ldc, d->delta_o32, (long long)d->ld_o32,
                       d->M, H, d->delta_hd, d->delta_seq, d->delta);
    SVAE_LAUNCH_CHECK();
  }
  return SVAE_OK;
}

static int gemm_run(const svae_gemm_desc* d, svae_stream_t stream, bool* fused_delta) {
  if (const int rc = validate_desc(d)) return rc;
  const bool epi_new = d->epi == SVAE_EPI_CE_PROB || d->epi == SVAE_EPI_ROWSCALE_GATHER;
  GP p;
  fill_gp(d, p);
  // split-K slab mode (F32_ATOMIC with aux): every split stores its partial tile with plain stores into
  // aux[split][M][N], then slab_reduce adds the splits into C (no float atomics on C).
  const bool slab = d->epi == SVAE_EPI_F32_ATOMIC && d->splits > 1 && d->aux;
  int epi_run = d->epi;
  if (slab) {
    if (d->batch != 1 || ((uintptr_t)d->aux & 15) || d->N % 4) return SVAE_EINVAL;
    p.C = d->aux; p.ldc = d->N; p.sC = 0; p.slab = (long long)d->M * d->N;
    p.bias = nullptr; p.resid = nullptr; p.aux = nullptr;   // (aux is the slab: no bf16 copy of the F32 epilogue)
    epi_run = SVAE_EPI_F32;
  }

  const long long nblocks = (long long)p.tiles_n * p.tiles_m * d->batch * d->splits;
  if (nblocks > 0x7FFFFFFF) return SVAE_EINVAL;
  dim3 grid((unsigned)nblocks);
  hipStream_t s = (hipStream_t)stream;
  // M <= 64 (one row per sequence): the skinny kernel (SVAE_GEMM_SKINNY=0 turns it off for A/B runs)
  static const int skinny_env = [] { const char* e = getenv("SVAE_GEMM_SKINNY"); return e ? atoi(e) : 1; }();
  if (skinny_env && d->M <= 64 && !d->a_t && !d->b_t && d->batch == 1 && d->splits == 1 && !d->a_rowsum &&
      d->C && d->K % 8 == 0 && d->lda % 8 == 0 && d->ldb % 8 == 0 && ((uintptr_t)d->A & 15) == 0 &&
      ((uintptr_t)d->B & 15) == 0 &&
      (d->epi == SVAE_EPI_BF16 || d->epi == SVAE_EPI_F32 || d->epi == SVAE_EPI_GELU || d->epi == SVAE_EPI_GELU_BWD ||
       d->epi == SVAE_EPI_DROPOUT_RESID)) {
    const dim3 gs((unsigned)((d->N + SK_BN - 1) / SK_BN));
    switch (d->epi) {
      case SVAE_EPI_BF16: hipLaunchKernelGGL(gemm_skinny_kernel<SVAE_EPI_BF16>, gs, dim3(1024), 0, s, p); break;
      case SVAE_EPI_F32: hipLaunchKernelGGL(gemm_skinny_kernel<SVAE_EPI_F32>, gs, dim3(1024), 0, s, p); break;
      case SVAE_EPI_GELU: hipLaunchKernelGGL(gemm_skinny_kernel<SVAE_EPI_GELU>, gs, dim3(1024), 0, s, p); break;
      case SVAE_EPI_GELU_BWD: hipLaunchKernelGGL(gemm_skinny_kernel<SVAE_EPI_GELU_BWD>, gs, dim3(1024), 0, s, p); break;
      default: hipLaunchKernelGGL(gemm_skinny_kernel<SVAE_EPI_DROPOUT_RESID>, gs, dim3(1024), 0, s, p); break;
    }
    SVAE_LAUNCH_CHECK();
    return SVAE_OK;
  }
  const int lay = (d->a_t ? 2 : 0) | (d->b_t ? 1 : 0);
  // short-K GEMMs: the 3-stage LDS-DMA kernel (3 blocks/CU overlap prologues/epilogues); long-K GEMMs: the
  // BK=64 register-staged kernel (half the barriers per MFMA). SVAE_GEMM_IMPL=1/2 forces one (A/B runs).
  static const int forced = [] { const char* e = getenv("SVAE_GEMM_IMPL"); return e ? atoi(e) : 0; }();
  const int kslice = (d->K + d->splits - 1) / d->splits;
  p.tn2 = (d->N + 255) / 256;
  p.tm2 = (d->M + 255) / 256;
  static const int group_env = [] { const char* e = getenv("SVAE_GEMM_GROUP"); return e ? atoi(e) : -1; }();
  // wide N (the vocab head, 128 column tiles): groups of 4 tile rows, so each XCD's 32 concurrent tiles are 4 rows x
  // 8 columns (12 operand strips in its L2 instead of 33): head fwd 1385 -> 1314 us (scripts/gemm_probe.py). No
  // effect measured on the narrow (<= 8 column tiles) C2 shapes.
  p.group = group_env >= 0 ? group_env : (p.tn2 >= 32 ? 4 : 0);
  const long long blocks256 = (long long)p.tn2 * p.tm2 * d->batch * d->splits;
  // (a_t with a K-contiguous B: the gemm256 copy exists for the f32-accumulate epilogues only -- the vocabulary head's
  // dW with a transposed B operand)
  const bool acc_epi = d->epi == SVAE_EPI_F32_ACC;
  const bool ok3 = !(d->a_t && !d->b_t) || acc_epi;
  int impl = forced ? forced : ((ok3 && blocks256 >= 192) ? 3 : ((kslice <= 2048 && !(d->a_t && d->b_t)) ? 2 : 1));
  if (epi_new || d->k_weight || (d->a_t && !d->b_t && acc_epi && blocks256 >= 192)) impl = 3;
  if (d->k_weight) {
    if (d->epi == SVAE_EPI_F32_ACC && d->splits == 1) epi_run = G3_EPI_ACC_KW;
    else if (slab) epi_run = G3_EPI_F32_KW;
    else return SVAE_EINVAL;
  }
  if (impl == 3 && !ok3) impl = 1;
  // float-atomic split-K (no slab workspace) is not a gemm256 epilogue: its staged 4-pass atomics cost 67-88 spilled
  // VGPRs there; the 128-tile kernels run it (the product's split-K weight gradients use the slab form)
  if (impl == 3 && epi_run == SVAE_EPI_F32_ATOMIC) impl = (kslice <= 2048 && !(d->a_t && d->b_t)) ? 2 : 1;
  if (impl == 3) {
    // the weight-gradient slab layout stores through the plain slab epilogue (other layouts keep SVAE_EPI_F32)
    if (slab && epi_run == SVAE_EPI_F32 && d->a_t && d->b_t) epi_run = G3_EPI_SLAB;
    int kc3 = (d->K + d->splits - 1) / d->splits;
    p.kchunk = (kc3 + 63) / 64 * 64;
    // persistent above one block per CU (1 block of 8 waves fits a CU): blocks walk their tiles and prefetch the
    // next tile's first K-tile under the current tile's epilogue. SVAE_GEMM_PERSIST=0 restores 1 block per tile.
    static const int persist_env = [] { const char* e = getenv("SVAE_GEMM_PERSIST"); return e ? atoi(e) : 1; }();
    static const int ncu = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        n = 256;
      return n > 0 ? n : 256;
    }();
    p.total3 = (int)blocks256;
    const long long nb3 = persist_env ? std::min<long long>(blocks256, ncu) : blocks256;
    static const int relax_env = [] { const char* e = getenv("SVAE_GEMM_RELAX"); return e ? atoi(e) : 1; }();
    // (the CE-statistics epilogue without a logits store issues too few stores for the counted first wait)
    p.relaxed = relax_env && !(d->epi == SVAE_EPI_CE_STATS && !d->C);
    // (SVAE_GEMM_STAGGER=0 for A/B: C2 step 12.89 / 12.99 -> 12.75 / 12.73 ms, head forward 1.12 -> 1.07 ms)
    static const int stagger_env = [] { const char* e = getenv("SVAE_GEMM_STAGGER"); return e ? atoi(e) : 1; }();
    p.dma_stagger = stagger_env;
    dim3 grid3((unsigned)nb3);
    // the delta epilogue (a wave's 64 columns hold at most two heads: hd >= 64) adds into a zeroed delta (svae_gemm)
    if (fused_delta && epi_run == SVAE_EPI_BF16 && d->delta_hd >= 64) {
      const long long n = (long long)d->M * (d->N / d->delta_hd);
      if (hipMemsetAsync(d->delta, 0, n * sizeof(float), s) != hipSuccess) return SVAE_ELAUNCH;
      epi_run = G3_EPI_BF16_DELTA;
      *fused_delta = true;
    }
#define SVAE_GEMM3_CASE(E)                                                                                   \
  case E:                                                                                                    \
    if (d->a_t && !d->b_t) {                                                                                 \
      if constexpr (E == SVAE_EPI_F32_ACC) hipLaunchKernelGGL((gemm256_kernel<true, false, E>), grid3, dim3(512), 0, s, p); \
      else return SVAE_EINVAL;                                                                               \
    } else if (d->a_t) hipLaunchKernelGGL((gemm256_kernel<true, true, E>), grid3, dim3(512), 0, s, p);       \
    else if (d->b_t) hipLaunchKernelGGL((gemm256_kernel<false, true, E>), grid3, dim3(512), 0, s, p);        \
    else hipLaunchKernelGGL((gemm256_kernel<false, false, E>), grid3, dim3(512), 0, s, p);                   \
    break;
    switch (epi_run) {
      SVAE_GEMM3_CASE(SVAE_EPI_BF16)
      SVAE_GEMM3_CASE(SVAE_EPI_F32)
      SVAE_GEMM3_CASE(SVAE_EPI_F32_ACC)
      SVAE_GEMM3_CASE(SVAE_EPI_GELU)
      SVAE_GEMM3_CASE(SVAE_EPI_GELU_BWD)
      SVAE_GEMM3_CASE(SVAE_EPI_DROPOUT_RESID)
      SVAE_GEMM3_CASE(SVAE_EPI_ROTARY_BF16)
      SVAE_GEMM3_CASE(SVAE_EPI_CE_STATS)
      case G3_EPI_ACC_KW:
        if (d->b_t) hipLaunchKernelGGL((gemm256_kernel<true, true, G3_EPI_ACC_KW>), grid3, dim3(512), 0, s, p);
        else hipLaunchKernelGGL((gemm256_kernel<true, false, G3_EPI_ACC_KW>), grid3, dim3(512), 0, s, p);
        break;
      case G3_EPI_SLAB:
        hipLaunchKernelGGL((gemm256_kernel<true, true, G3_EPI_SLAB>), grid3, dim3(512), 0, s, p);
        break;
      case G3_EPI_F32_KW:
        if (!d->b_t) return SVAE_EINVAL;
        hipLaunchKernelGGL((gemm256_kernel<true, true, G3_EPI_F32_KW>), grid3, dim3(512), 0, s, p);
        break;
      case SVAE_EPI_CE_PROB:
        hipLaunchKernelGGL((gemm256_kernel<false, false, SVAE_EPI_CE_PROB>), grid3, dim3(512), 0, s, p);
        break;
      case G3_EPI_BF16_DELTA:
        if (d->b_t) hipLaunchKernelGGL((gemm256_kernel<false, true, G3_EPI_BF16_DELTA>), grid3, dim3(512), 0, s, p);
        else hipLaunchKernelGGL((gemm256_kernel<false, false, G3_EPI_BF16_DELTA>), grid3, dim3(512), 0, s, p);
        break;
      case SVAE_EPI_ROWSCALE_GATHER:
        if (d->b_t) hipLaunchKernelGGL((gemm256_kernel<false, true, SVAE_EPI_ROWSCALE_GATHER>), grid3, dim3(512), 0, s, p);
        else hipLaunchKernelGGL((gemm256_kernel<false, false, SVAE_EPI_ROWSCALE_GATHER>), grid3, dim3(512), 0, s, p);
        break;
      default: return SVAE_EINVAL;
    }
#undef SVAE_GEMM3_CASE
    SVAE_LAUNCH_CHECK();
    return slab ? launch_slab_reduce(d, s) : SVAE_OK;
  }
  if (impl == 2) {
    int kchunk2 = (d->K + d->splits - 1) / d->splits;
    p.kchunk = (kchunk2 + BK2 - 1) / BK2 * BK2;
#define SVAE_GEMM2_CASE(E)                                                                             \
  case E:                                                                                              \
    if (lay == 0) hipLaunchKernelGGL((gemm_glds_kernel<false, false, E>), grid, dim3(256), 0, s, p);    \
    else if (lay == 1) hipLaunchKernelGGL((gemm_glds_kernel<false, true, E>), grid, dim3(256), 0, s, p); \
    else if (lay == 2) hipLaunchKernelGGL((gemm_glds_kernel<true, false, E>), grid, dim3(256), 0, s, p); \
    else hipLaunchKernelGGL((gemm_glds_kernel<true, true, E>), grid, dim3(256), 0, s, p);                \
    break;
    switch (epi_run) {
      SVAE_GEMM2_CASE(SVAE_EPI_BF16)
      SVAE_GEMM2_CASE(SVAE_EPI_F32)
      SVAE_GEMM2_CASE(SVAE_EPI_F32_ACC)
      SVAE_GEMM2_CASE(SVAE_EPI_F32_ATOMIC)
      SVAE_GEMM2_CASE(SVAE_EPI_GELU)
      SVAE_GEMM2_CASE(SVAE_EPI_GELU_BWD)
      SVAE_GEMM2_CASE(SVAE_EPI_DROPOUT_RESID)
      SVAE_GEMM2_CASE(SVAE_EPI_ROTARY_BF16)
      SVAE_GEMM2_CASE(SVAE_EPI_CE_STATS)
      default: return SVAE_EINVAL;
    }
#undef SVAE_GEMM2_CASE
    SVAE_LAUNCH_CHECK();
    return slab ? launch_slab_reduce(d, s) : SVAE_OK;
  }
#define SVAE_GEMM_CASE(E)                                                                             \
  case E:                                                                                             \
    if (lay == 0) hipLaunchKernelGGL((gemm_kernel<false, false, E>), grid, dim3(256), 0, s, p);        \
    else if (lay == 1) hipLaunchKernelGGL((gemm_kernel<false, true, E>), grid, dim3(256), 0, s, p);    \
    else if (lay == 2) hipLaunchKernelGGL((gemm_kernel<true, false, E>), grid, dim3(256), 0, s, p);    \
    else hipLaunchKernelGGL((gemm_kernel<true, true, E>), grid, dim3(256), 0, s, p);                   \
    break;
  switch (epi_run) {
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
  return slab ? launch_slab_reduce(d, s) : SVAE_OK;
}

SVAE_EXPORT int svae_gemm_pair(const svae_gemm_desc* d0, const svae_gemm_desc* d1, svae_stream_t stream) {
  const svae_gemm_desc* d[2] = {d0, d1};
  GP2 q;
  long long nb[2];
  for (int i = 0; i < 2; ++i) {
    if (const int rc = validate_desc(d[i])) return rc;
    // the weight-gradient shape only: A and B transposed (row-major [K][M] and [K][N]), split-K slab mode
    if (!d[i]->a_t || !d[i]->b_t || d[i]->epi != SVAE_EPI_F32_ATOMIC || d[i]->splits < 2 || !d[i]->aux ||
        d[i]->batch != 1 || d[i]->k_weight || ((uintptr_t)d[i]->aux & 15))
      return SVAE_EINVAL;
    GP& p = q.p[i];
    fill_gp(d[i], p);
    p.C = d[i]->aux; p.ldc = d[i]->N; p.sC = 0; p.slab = (long long)d[i]->M * d[i]->N;
    p.bias = nullptr; p.resid = nullptr; p.aux = nullptr;
    const int kc3 = (d[i]->K + d[i]->splits - 1) / d[i]->splits;
    p.kchunk = (kc3 + 63) / 64 * 64;
    p.tn2 = (d[i]->N + 255) / 256;
    p.tm2 = (d[i]->M + 255) / 256;
    p.group = 0;
    nb[i] = (long long)p.tn2 * p.tm2 * d[i]->splits;
    if (nb[i] > (1 << 24)) return SVAE_EINVAL;
    p.total3 = (int)nb[i];
    p.relaxed = 1;   // (p.dma_stagger stays 0: on the paired dW launches it measured 12.72 / 12.77 -> 12.79 / 12.93 ms)
  }
  q.nb0 = (int)((nb[0] + 7) / 8 * 8);   // block ranges start on an XCD boundary (block id % 8)
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL((gemm256_pair_kernel<true, true, G3_EPI_SLAB>), dim3((unsigned)(q.nb0 + nb[1])), dim3(512), 0, s,
                     q);
  SVAE_LAUNCH_CHECK();
  static const int two_env = [] { const char* e = getenv("SVAE_SLAB2"); return e ? atoi(e) : 1; }();
  if (!two_env) {   // (A/B: one launch per GEMM)
    if (const int rc = launch_slab_reduce(d0, s)) return rc;
    return launch_slab_reduce(d1, s);
  }
  const long long b0 = slab_blocks(d0), b1 = slab_blocks(d1);
  hipLaunchKernelGGL(slab_reduce2_kernel, dim3((unsigned)(b0 + b1)), dim3(256), 0, s, slab_red(d0), slab_red(d1), (int)b0);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

#ifdef SVAE_STAMPS
extern "C" __attribute__((visibility("default"))) int svae_debug_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(svae_stamps), sizeof(svae_stamps)) == hipSuccess ? 0 : -1;
}
extern "C" __attribute__((visibility("default"))) int svae_debug_rt(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(svae_rt), sizeof(svae_rt)) == hipSuccess ? 0 : -1;
}
extern "C" __attribute__((visibility("default"))) int svae_debug_stamps_clear() {
  static unsigned long long zeros[8 * 96 * 3];
  return hipMemcpyToSymbol(HIP_SYMBOL(svae_stamps), zeros, sizeof(zeros)) == hipSuccess ? 0 : -1;
}
#endif
