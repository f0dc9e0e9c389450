// Flash attention forward / backward for the dense path of Attention.forward (attention.py:51-105):
//   scores = q k^T * hd^-0.5 (:83); scores -= 1e7 * (key_pad | causal) (:85-98); softmax . v (:100).
// A masked score contributes exactly 0 after exp (as the reference's -1e7 shift underflows to 0).
//
// Layout: q/k/v/o are token-major rows of H*hd bf16 (the nn.Linear output layout, heads interleaved),
// so no head-split copies exist. Head dim is padded to HDP = 64 or 128 inside the kernel.
//
// Forward: one block = 64 queries of one (batch, head), 4 waves x 16 queries. "Swapped" products keep the
// query on the MFMA lane: S^T = K . Q^T (K tile ds_read_b128, Q fragment in registers), then
// O^T += V^T . P^T where P^T is the S^T accumulator converted in place (key order permuted to match the
// ds_read_b64_tr_b16 reads of V). Online softmax per lane, no P round trip through LDS.
//
// Backward: one block = 64 keys, 4 waves x 16 keys, sweeping query tiles (key on the lane: S = Q K^T and
// dP = dO V^T accumulators are already the B operands of dV^T += dO^T P and dK^T += Q^T dS). dS^T goes
// through LDS once for dQ = dS K, which is summed across key blocks with f32 atomics.
#include "common.h"
#include "../../include/svae.h"

using namespace svae;

namespace {

struct AP {
  const bf16* q; const bf16* k; const bf16* v; bf16* o;
  long long sq, sk, sv, so, bq, bk, bv, bo;
  const unsigned char* pad;
  float* lse;
  int B, H, Lq, Lk, hd, causal;
  float scale;
  const bf16* dout; long long sdo, bdo;
  const float* delta;
  float* dq; long long bdq;
  bf16* dk; bf16* dv; long long sdk, sdv, bdk, bdv;
  const float* rot; int rot_d;
  float* o32; long long so32, bo32;
};

// [64 rows][HDP] bf16 tile in LDS, 16-B chunks XOR-swizzled by (row & (chunks-1)): conflict-free for the
// row-wise ds_read_b128 fragment reads, <= 2-way for the ds_read_b64_tr_b16 reads.
template <int HDP>
struct Tile {
  static constexpr int NCH = HDP / 8;
  static constexpr int PITCH = HDP * 2;
  static constexpr int BYTES = 64 * PITCH;
  __device__ static __forceinline__ int off(int r, int c) { return r * PITCH + ((c ^ (r & (NCH - 1))) << 4); }
  __device__ static __forceinline__ int uoff(int r, int u) { return off(r, u >> 1) + ((u & 1) << 3); }
};

// Load rows [row0, row0+64) of a token-major matrix (row stride ld, head column offset folded into g)
// into registers: NCH/4 16-B vectors per thread. Rows >= nrows and dims >= hd read as zero.
template <int HDP>
__device__ __forceinline__ void load_rows(const bf16* g, long long ld, int row0, int nrows, int hd, u32x4* r,
                                          int tid) {
  constexpr int NV = Tile<HDP>::NCH / 4;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int idx = tid + 256 * i;
    const int row = idx / Tile<HDP>::NCH, c = idx % Tile<HDP>::NCH;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (row0 + row < nrows && c * 8 < hd) v = *(const u32x4*)(g + (long long)(row0 + row) * ld + c * 8);
    r[i] = v;
  }
}

template <int HDP>
__device__ __forceinline__ void store_rows(char* lds, const u32x4* r, int tid) {
  constexpr int NV = Tile<HDP>::NCH / 4;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int idx = tid + 256 * i;
    *(u32x4*)(lds + Tile<HDP>::off(idx / Tile<HDP>::NCH, idx % Tile<HDP>::NCH)) = r[i];
  }
}

__device__ __forceinline__ bf16x8 pack8(const f32x4& a, const f32x4& b) {
  return (bf16x8){f2bf(a[0]), f2bf(a[1]), f2bf(a[2]), f2bf(a[3]), f2bf(b[0]), f2bf(b[1]), f2bf(b[2]), f2bf(b[3])};
}

// ===================================================================================== forward
template <int HDP>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(AP p) {
  using T = Tile<HDP>;
  constexpr int NKK = HDP / 32, NT = HDP / 16, NV = T::NCH / 4;
  __shared__ __attribute__((aligned(16))) char smem[4 * T::BYTES + 128];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  const int q0 = blockIdx.x * 64, h = blockIdx.y, b = blockIdx.z;
  const bf16* Q = p.q + b * p.bq + (long long)h * p.hd;
  const bf16* K = p.k + b * p.bk + (long long)h * p.hd;
  const bf16* V = p.v + b * p.bv + (long long)h * p.hd;
  const unsigned char* pad = p.pad ? p.pad + (long long)b * p.Lk : nullptr;
  unsigned char* pm = (unsigned char*)(smem + 4 * T::BYTES);

  const int qrow = q0 + 16 * w + li;
  bf16x8 qf[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    const int d = 32 * kk + 8 * g;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (qrow < p.Lq && d < p.hd) v = *(const u32x4*)(Q + (long long)qrow * p.sq + d);
    qf[kk] = __builtin_bit_cast(bf16x8, v);
  }
  f32x4 o[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) o[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = -1e30f, lsum = 0.f;
  const int kv_end = p.causal ? min(p.Lk, q0 + 64) : p.Lk;
  const int ntiles = (kv_end + 63) / 64;
  const float sl2 = p.scale;

  u32x4 rk[NV], rv[NV];
  unsigned char rpm = 0;
  load_rows<HDP>(K, p.sk, 0, p.Lk, p.hd, rk, tid);
  load_rows<HDP>(V, p.sv, 0, p.Lk, p.hd, rv, tid);
  if (tid < 64) rpm = (pad && tid < p.Lk) ? pad[tid] : 0;
  store_rows<HDP>(smem, rk, tid);
  store_rows<HDP>(smem + T::BYTES, rv, tid);
  if (tid < 64) pm[tid] = rpm;
  __syncthreads();

  for (int kt = 0; kt < ntiles; ++kt) {
    const int buf = kt & 1;
    const char* Ks = smem + buf * 2 * T::BYTES;
    const char* Vs = Ks + T::BYTES;
    const unsigned char* pms = pm + buf * 64;
    const bool more = kt + 1 < ntiles;
    if (more) {
      const int kn = (kt + 1) * 64;
      load_rows<HDP>(K, p.sk, kn, p.Lk, p.hd, rk, tid);
      load_rows<HDP>(V, p.sv, kn, p.Lk, p.hd, rv, tid);
      if (tid < 64) rpm = (pad && kn + tid < p.Lk) ? pad[kn + tid] : 0;
    }
    // S^T = K . Q^T : s[st][r] = score(key = 16st + 4g + r, query = qrow)
    f32x4 s[4];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      s[st] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        const bf16x8 kf = *(const bf16x8*)(Ks + T::off(16 * st + li, g + 4 * kk));
        s[st] = mfma16(kf, qf[kk], s[st]);
      }
    }
    const int kbase = kt * 64;
    float mx = -1e30f;
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kl = 16 * st + 4 * g + r, key = kbase + kl;
        const bool masked = key >= p.Lk || pms[kl] || (p.causal && key > qrow);
        const float x = masked ? -INFINITY : s[st][r] * sl2;
        s[st][r] = x;
        mx = fmaxf(mx, x);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float alpha = __expf(m - mn);
    m = mn;
    lsum *= alpha;
#pragma unroll
    for (int t = 0; t < NT; ++t) o[t] *= alpha;
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = __expf(s[st][r] - m);
        s[st][r] = pv;
        lsum += pv;
      }
    // O^T += V^T . P^T  (keys of k-step kk: 32kk + 16(j>>2) + 4g + (j&3))
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const bf16x8 pf = pack8(s[2 * kk], s[2 * kk + 1]);
      const int r0 = 32 * kk + 4 * g + (li >> 2);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int u = 4 * t + (li & 3);
        const short4v lo = lds_read_tr(Vs + T::uoff(r0, u));
        const short4v hi = lds_read_tr(Vs + T::uoff(r0 + 16, u));
        o[t] = mfma16(cat44(lo, hi), pf, o[t]);
      }
    }
    if (more) {
      char* nb = smem + (buf ^ 1) * 2 * T::BYTES;
      store_rows<HDP>(nb, rk, tid);
      store_rows<HDP>(nb + T::BYTES, rv, tid);
      if (tid < 64) pm[(buf ^ 1) * 64 + tid] = rpm;
    }
    __syncthreads();
  }

  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  if (qrow < p.Lq) {
    const float inv = 1.0f / lsum;
    bf16* O = p.o + b * p.bo + (long long)h * p.hd + (long long)qrow * p.so;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int d = 16 * t + 4 * g;
      if (d < p.hd) {
        *(bf16x4*)(O + d) = (bf16x4){f2bf(o[t][0] * inv), f2bf(o[t][1] * inv), f2bf(o[t][2] * inv), f2bf(o[t][3] * inv)};
        if (p.o32)
          *(f32x4*)(p.o32 + b * p.bo32 + (long long)h * p.hd + (long long)qrow * p.so32 + d) = o[t] * inv;
      }
    }
    if (g == 0) p.lse[((long long)b * p.H + h) * p.Lq + qrow] = m + __logf(lsum);
  }
}

// ===================================================================================== backward
// delta[b][h][q] = sum_d dO . O   (16 lanes per (q, h) row)
__global__ __launch_bounds__(256) void attn_delta_kernel(AP p) {
  const int gid = blockIdx.x * 16 + (threadIdx.x >> 4);
  const int li = threadIdx.x & 15;
  const int total = p.B * p.Lq * p.H;
  if (gid >= total) return;
  const int h = gid % p.H, q = (gid / p.H) % p.Lq, b = gid / (p.H * p.Lq);
  const bf16* dO = p.dout + b * p.bdo + (long long)q * p.sdo + (long long)h * p.hd;
  float s = 0.f;
  if (p.o32) {
    const float* O = p.o32 + b * p.bo32 + (long long)q * p.so32 + (long long)h * p.hd;
    for (int d = li * 8; d < p.hd; d += 128) {
      const bf16x8 c = *(const bf16x8*)(dO + d);
      const f32x4 a0 = *(const f32x4*)(O + d), a1 = *(const f32x4*)(O + d + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) s += a0[e] * (float)c[e] + a1[e] * (float)c[e + 4];
    }
  } else {
    const bf16* O = p.o + b * p.bo + (long long)q * p.so + (long long)h * p.hd;
    for (int d = li * 8; d < p.hd; d += 128) {
      const bf16x8 a = *(const bf16x8*)(O + d), c = *(const bf16x8*)(dO + d);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += (float)a[e] * (float)c[e];
    }
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
  if (li == 0) ((float*)p.delta)[((long long)b * p.H + h) * p.Lq + q] = s;
}

template <int HDP>
__global__ __launch_bounds__(256, 2) void attn_bwd_kernel(AP p) {
  using T = Tile<HDP>;
  using TS = Tile<64>;   // dS^T tile [64 keys][64 queries]
  constexpr int NKK = HDP / 32, NT = HDP / 16, NV = T::NCH / 4;
  __shared__ __attribute__((aligned(16))) char smem[3 * T::BYTES + TS::BYTES + 2 * 64 * 4];
  char* Qs = smem;
  char* dOs = smem + T::BYTES;
  char* Ks = smem + 2 * T::BYTES;
  char* dSs = smem + 3 * T::BYTES;
  float* lse_s = (float*)(smem + 3 * T::BYTES + TS::BYTES);
  float* del_s = lse_s + 64;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  const int k0 = blockIdx.x * 64, h = blockIdx.y, b = blockIdx.z;
  const bf16* Q = p.q + b * p.bq + (long long)h * p.hd;
  const bf16* K = p.k + b * p.bk + (long long)h * p.hd;
  const bf16* V = p.v + b * p.bv + (long long)h * p.hd;
  const bf16* dO = p.dout + b * p.bdo + (long long)h * p.hd;
  const float* lse = p.lse + ((long long)b * p.H + h) * p.Lq;
  const float* delta = p.delta + ((long long)b * p.H + h) * p.Lq;
  const int kw = k0 + 16 * w;
  const int key = kw + li;                       // this lane's key (column of S / dP)
  const bool key_ok = key < p.Lk && !(p.pad && p.pad[(long long)b * p.Lk + key]);

  // K and V fragments of this wave's 16 keys (B operands of S = Q K^T and dP = dO V^T)
  bf16x8 kf[NKK], vf[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    const int d = 32 * kk + 8 * g;
    u32x4 a = {0u, 0u, 0u, 0u}, c = a;
    if (key < p.Lk && d < p.hd) {
      a = *(const u32x4*)(K + (long long)key * p.sk + d);
      c = *(const u32x4*)(V + (long long)key * p.sv + d);
    }
    kf[kk] = __builtin_bit_cast(bf16x8, a);
    vf[kk] = __builtin_bit_cast(bf16x8, c);
  }
  {  // K tile for dQ = dS . K (transposed reads)
    u32x4 rk[NV];
    load_rows<HDP>(K, p.sk, k0, p.Lk, p.hd, rk, tid);
    store_rows<HDP>(Ks, rk, tid);
  }
  f32x4 dk[NT], dv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) { dk[t] = (f32x4){0.f, 0.f, 0.f, 0.f}; dv[t] = dk[t]; }

  const int qt0 = p.causal ? k0 / 64 : 0;
  const int nqt = (p.Lq + 63) / 64;
  for (int qt = qt0; qt < nqt; ++qt) {
    const int qb = qt * 64;
    {
      u32x4 rq[NV], ro[NV];
      load_rows<HDP>(Q, p.sq, qb, p.Lq, p.hd, rq, tid);
      load_rows<HDP>(dO, p.sdo, qb, p.Lq, p.hd, ro, tid);
      __syncthreads();   // previous tile's readers are done
      store_rows<HDP>(Qs, rq, tid);
      store_rows<HDP>(dOs, ro, tid);
      if (tid < 64) {
        const int q = qb + tid;
        lse_s[tid] = q < p.Lq ? lse[q] : 0.f;
        del_s[tid] = q < p.Lq ? delta[q] : 0.f;
      }
      __syncthreads();
    }
    // S (q x key) and dP, key on the lane: s[t][r] -> q = qb + 16t + 4g + r
    f32x4 s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
      dp[t] = s[t];
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        const bf16x8 qa = *(const bf16x8*)(Qs + T::off(16 * t + li, g + 4 * kk));
        const bf16x8 oa = *(const bf16x8*)(dOs + T::off(16 * t + li, g + 4 * kk));
        s[t] = mfma16(qa, kf[kk], s[t]);
        dp[t] = mfma16(oa, vf[kk], dp[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = 16 * t + 4 * g + r, q = qb + ql;
        const bool ok = key_ok && q < p.Lq && !(p.causal && key > q);
        const float pr = ok ? __expf(s[t][r] * p.scale - lse_s[ql]) : 0.f;
        s[t][r] = pr;
        dp[t][r] = pr * (dp[t][r] - del_s[ql]);
      }
    // dV^T += dO^T P ; dK^T += Q^T dS   (query order of k-step kk: 32kk + 16(j>>2) + 4g + (j&3))
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const bf16x8 pf = pack8(s[2 * kk], s[2 * kk + 1]);
      const bf16x8 df = pack8(dp[2 * kk], dp[2 * kk + 1]);
      const int r0 = 32 * kk + 4 * g + (li >> 2);
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const int uu = 4 * u + (li & 3);
        const bf16x8 ao = cat44(lds_read_tr(dOs + T::uoff(r0, uu)), lds_read_tr(dOs + T::uoff(r0 + 16, uu)));
        dv[u] = mfma16(ao, pf, dv[u]);
        const bf16x8 aq = cat44(lds_read_tr(Qs + T::uoff(r0, uu)), lds_read_tr(Qs + T::uoff(r0 + 16, uu)));
        dk[u] = mfma16(aq, df, dk[u]);
      }
    }
    // dS^T -> LDS [key][q]: this lane holds q = 16t + 4g + (0..3) at key row 16w + li
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const bf16x4 v4 = (bf16x4){f2bf(dp[t][0]), f2bf(dp[t][1]), f2bf(dp[t][2]), f2bf(dp[t][3])};
      *(bf16x4*)(dSs + TS::uoff(16 * w + li, 4 * t + g)) = v4;
    }
    __syncthreads();
    // dQ[q = qb + 16w + 4g + r][d = 16u + li] = scale * sum_key dS[q][key] K[key][d]
    f32x4 dq[NT];
#pragma unroll
    for (int u = 0; u < NT; ++u) dq[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int kr = 32 * kk + 8 * g + (li >> 2);
      const int uq = 4 * w + (li & 3);
      const bf16x8 a = cat44(lds_read_tr(dSs + TS::uoff(kr, uq)), lds_read_tr(dSs + TS::uoff(kr + 4, uq)));
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const int uk = 4 * u + (li & 3);
        const bf16x8 bk = cat44(lds_read_tr(Ks + T::uoff(kr, uk)), lds_read_tr(Ks + T::uoff(kr + 4, uk)));
        dq[u] = mfma16(a, bk, dq[u]);
      }
    }
    float* DQ = p.dq + b * p.bdq + (long long)h * p.hd;
    const long long ldq = (long long)p.H * p.hd;
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      const int d = 16 * u + li;
      if (d < p.hd) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = qb + 16 * w + 4 * g + r;
          if (q < p.Lq) atomicAdd(DQ + (long long)q * ldq + d, dq[u][r] * p.scale);
        }
      }
    }
  }

  // epilogue: dK (scaled, inverse rotary) and dV for key = kw + li, dims 16u + 4g + (0..3)
  if (key < p.Lk) {
    bf16* DK = p.dk + b * p.bdk + (long long)key * p.sdk + (long long)h * p.hd;
    bf16* DV = p.dv + b * p.bdv + (long long)key * p.sdv + (long long)h * p.hd;
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      const int d = 16 * u + 4 * g;
      if (d >= p.hd) continue;
      float x[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) x[r] = dk[u][r] * p.scale;
      if (p.rot) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int pair = (h * p.hd + d) / 2 + e;
          const float2 cs = ((const float2*)p.rot)[(long long)key * (p.rot_d / 2) + pair];
          const float a = x[2 * e], c = x[2 * e + 1];
          x[2 * e] = a * cs.x + c * cs.y;
          x[2 * e + 1] = -a * cs.y + c * cs.x;
        }
      }
      *(bf16x4*)(DK + d) = (bf16x4){f2bf(x[0]), f2bf(x[1]), f2bf(x[2]), f2bf(x[3])};
      *(bf16x4*)(DV + d) = (bf16x4){f2bf(dv[u][0]), f2bf(dv[u][1]), f2bf(dv[u][2]), f2bf(dv[u][3])};
    }
  }
}

bool fill(const svae_attn_desc* d, AP& p) {
  if (!d || !d->q || !d->k || !d->v || !d->o || !d->lse) return false;
  if (d->B <= 0 || d->H <= 0 || d->Lq <= 0 || d->Lk <= 0 || d->hd <= 0 || d->hd > 128 || d->hd % 8) return false;
  if ((d->sq | d->sk | d->sv | d->so | d->bq | d->bk | d->bv | d->bo) % 8) return false;
  p.q = (const bf16*)d->q; p.k = (const bf16*)d->k; p.v = (const bf16*)d->v; p.o = (bf16*)d->o;
  p.sq = d->sq; p.sk = d->sk; p.sv = d->sv; p.so = d->so;
  p.bq = d->bq; p.bk = d->bk; p.bv = d->bv; p.bo = d->bo;
  p.pad = d->key_pad; p.lse = d->lse;
  p.B = d->B; p.H = d->H; p.Lq = d->Lq; p.Lk = d->Lk; p.hd = d->hd; p.causal = d->causal;
  p.scale = d->scale;
  p.dout = (const bf16*)d->dout; p.sdo = d->sdo; p.bdo = d->bdo;
  p.delta = d->delta; p.dq = d->dq; p.bdq = d->bdq;
  p.dk = (bf16*)d->dk; p.dv = (bf16*)d->dv; p.sdk = d->sdk; p.sdv = d->sdv; p.bdk = d->bdk; p.bdv = d->bdv;
  p.rot = d->rot_tab; p.rot_d = d->rot_d;
  p.o32 = d->o32; p.so32 = d->so32; p.bo32 = d->bo32;
  if (p.o32 && ((p.so32 | p.bo32) % 4)) return false;
  return true;
}

}  // namespace

SVAE_EXPORT int svae_attn_fwd(const svae_attn_desc* d, svae_stream_t stream) {
  AP p;
  if (!fill(d, p)) return SVAE_EINVAL;
  if (d->causal && d->Lq != d->Lk) return SVAE_EINVAL;
  dim3 grid((d->Lq + 63) / 64, d->H, d->B);
  hipStream_t s = (hipStream_t)stream;
  if (d->hd <= 64) hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(attn_fwd_kernel<128>, grid, dim3(256), 0, s, p);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_attn_bwd(const svae_attn_desc* d, svae_stream_t stream) {
  AP p;
  if (!fill(d, p)) return SVAE_EINVAL;
  if (!d->dout || !d->delta || !d->dq || !d->dk || !d->dv) return SVAE_EINVAL;
  if ((d->sdo | d->bdo | d->sdk | d->sdv | d->bdk | d->bdv) % 4) return SVAE_EINVAL;
  if (d->causal && d->Lq != d->Lk) return SVAE_EINVAL;
  if (d->rot_tab && d->rot_d <= 0) return SVAE_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int rows = d->B * d->Lq * d->H;
  hipLaunchKernelGGL(attn_delta_kernel, dim3((rows + 15) / 16), dim3(256), 0, s, p);
  dim3 grid((d->Lk + 63) / 64, d->H, d->B);
  if (d->hd <= 64) hipLaunchKernelGGL(attn_bwd_kernel<64>, grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(attn_bwd_kernel<128>, grid, dim3(256), 0, s, p);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}
