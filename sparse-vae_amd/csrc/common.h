// Shared device helpers for the sparse-vae MI355X (gfx950 / CDNA4) kernels.
// wave64 everywhere; bf16 storage via clang's __bf16 (conversion lowers to v_cvt_pk_bf16_f32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

#define SVAE_EXPORT extern "C" __attribute__((visibility("default")))

namespace svae {

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Transposed LDS read (gfx950 ds_read_b64_tr_b16): within each 16-lane group, lane 4q+p supplies the
// address of row q (4 contiguous 16-bit elements); lane i receives column i of the 4 rows.
__device__ __forceinline__ short4v lds_read_tr(const void* lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) short4v*)(uintptr_t)(lds_addr));
}

// The lane id recomputed where it is used (volatile: never hoisted or shared): per-lane DMA offsets derived from it
// stay cheap to rematerialise instead of being computed once at kernel entry and spilled around the loop (a spill
// reload's compiler-inserted vmcnt(0) drains the hand-counted DMA).
__device__ __forceinline__ int lane_id_fresh() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// The same read from an address-space-3 pointer: base + compile-time offset folds into the instruction's offset field
// (through the generic-pointer form the compiler materialised every offset in a VGPR of its own).
typedef __attribute__((address_space(3))) char lds_char;
__device__ __forceinline__ const lds_char* lds_ptr(const void* p) { return (const lds_char*)(uintptr_t)p; }
__device__ __forceinline__ short4v lds_read_tr3(const lds_char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)p);
}

// LDS-DMA of 16 B per lane (buffer_load_dwordx4 ... lds) into lds_base + 16 * lane, from rsrc + voff (bytes;
// out-of-range offsets land as zeros). Issued through inline asm on purpose: the compiler's wait-count pass
// would otherwise treat every later ds_read_b64_tr_b16 as a possible reader of the DMA destination and put a
// vmcnt(0) in front of it, draining the prefetched tiles of every ring that uses transposed LDS reads. The
// callers wait for the DMA explicitly (counted s_waitcnt vmcnt + barrier) before reading a stage.
// rsrc: the 4 descriptor words (base lo, base hi, num_records, flags), wave-uniform.
__device__ __forceinline__ u32x4 buffer_rsrc(const void* base, unsigned num_records) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  return (u32x4){(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)a),
                 (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)(a >> 32) & 0xFFFFu)), num_records,
                 0x00020000u};
}
__device__ __forceinline__ void dma16_lds(const u32x4& rsrc, const void* lds_base, int voff) {
  const int m = __builtin_amdgcn_readfirstlane((int)(unsigned)(uintptr_t)lds_base);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(m), "v"(voff), "s"(rsrc)
               : "memory");  // (m0 is reserved: the compiler sets it before each of its own uses)
}

// 4 B per lane (buffer_load_dword ... lds) into lds_base + 4 * lane, same conventions as dma16_lds.
__device__ __forceinline__ void dma4_lds(const u32x4& rsrc, const void* lds_base, int voff) {
  const int m = __builtin_amdgcn_readfirstlane((int)(unsigned)(uintptr_t)lds_base);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds"
               :
               : "s"(m), "v"(voff), "s"(rsrc)
               : "memory");  // (m0 is reserved: the compiler sets it before each of its own uses)
}

// 1 B per lane (buffer_load_ubyte ... lds) into a dword slot per lane (lds_base + 4 * lane; the byte is the low
// 8 bits of the slot), same conventions as dma16_lds.
__device__ __forceinline__ void dma1_lds(const u32x4& rsrc, const void* lds_base, int voff) {
  const int m = __builtin_amdgcn_readfirstlane((int)(unsigned)(uintptr_t)lds_base);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_ubyte %1, %2, 0 offen lds"
               :
               : "s"(m), "v"(voff), "s"(rsrc)
               : "memory");  // (m0 is reserved: the compiler sets it before each of its own uses)
}

__device__ __forceinline__ bf16x8 cat44(short4v lo, short4v hi) {
  typedef short short8v __attribute__((ext_vector_type(8)));
  short8v s = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, s);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// erf-GELU (nn.GELU default) and its derivative, in fp32.
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad_f(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// cross-lane reductions over the 4 lane groups (lane ^ 16, lane ^ 32) with VALU permlane swaps (no LDS)
__device__ __forceinline__ float max_x16_x32(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto c = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(c[0]), __uint_as_float(c[1]));
}
__device__ __forceinline__ float sum_x16_x32(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto c = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(c[0]) + __uint_as_float(c[1]);
}

// GELU and GELU' together for the GEMM epilogues: Phi(x) from erfc(|x|/sqrt2) by Abramowitz-Stegun 7.1.26
// (|erf error| <= 1.5e-7, branchless: one v_rcp, one v_exp, 7 FMAs), and phi(x) = exp(-x^2/2)/sqrt(2 pi)
// reusing the same exponential. ~1/5 of the instructions of the erff-based pair above.
__device__ __forceinline__ void gelu_pair(float x, float& g, float& gp) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  const float poly =
      t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f), 0.254829592f);
  const float e = __expf(-z * z);             // exp(-x^2 / 2)
  const float half_erfc = 0.5f * poly * e;    // Phi(-|x|)
  const float cdf = x >= 0.f ? 1.0f - half_erfc : half_erfc;
  g = x * cdf;
  gp = fmaf(x * 0.3989422804014327f, e, cdf);
}

// gelu_pair on two elements with the packed f32 VALU ops (v_pk_fma/mul_f32: two lanes' worth per instruction):
// the same A-S 7.1.26 formula with 0.5 folded into the coefficients; cdf = step(x) - sign(x) * Phi(-|x|) (one
// rounding, no cancellation for x << 0). ~9 VALU + 2 transcendental per element instead of ~17 + 2.
__device__ __forceinline__ void gelu_pair2(f32x2 x, f32x2& g, f32x2& gp) {
  const f32x2 z = {fabsf(x[0]) * 0.70710678118654752f, fabsf(x[1]) * 0.70710678118654752f};
  const f32x2 d = z * 0.3275911f + 1.0f;
  const f32x2 t = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  const f32x2 poly = t * (((((t * 0.5307027145f) + -0.7265760135f) * t + 0.7107068705f) * t + -0.142248368f) * t +
                          0.127414796f);                                   // 0.5 * A-S polynomial
  const f32x2 w = (x * x) * -0.72134752044448170f;                        // -x^2/2 * log2(e)
  const f32x2 e = {__builtin_amdgcn_exp2f(w[0]), __builtin_amdgcn_exp2f(w[1])};   // exp(-x^2 / 2)
  const f32x2 h = poly * e;                                                 // Phi(-|x|)
  const f32x2 sg = __builtin_elementwise_copysign((f32x2){1.0f, 1.0f}, x);
  const f32x2 step = sg * 0.5f + 0.5f;
  const f32x2 cdf = (-sg) * h + step;
  g = x * cdf;
  gp = (x * 0.3989422804014327f) * e + cdf;
}

// Counter-based RNG (splitmix64 finaliser over (seed, counter)): stateless, so the backward pass
// regenerates exactly the forward's dropout mask / noise from the same (seed, index).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float rand_uniform(uint64_t seed, uint64_t idx) {
  uint64_t r = mix64(seed * 0x9E3779B97F4A7C15ull + idx + 0x632BE59BD9B4E019ull);
  return ((uint32_t)(r >> 40) + 0.5f) * (1.0f / 16777216.0f);
}
// Dropout: the four uniforms of elements 4q..4q+3 (row-major index / 4) from ONE hash, 16 bits each
// (keep-probability resolution 2^-16). Shared by the forward epilogue and the backward mask kernel.
__device__ __forceinline__ void rand_uniform4(uint64_t seed, uint64_t q, float (&u)[4]) {
  const uint64_t r = mix64(seed * 0x9E3779B97F4A7C15ull + q + 0x632BE59BD9B4E019ull);
  const uint32_t lo = (uint32_t)r, hi = (uint32_t)(r >> 32);
  const float s = 1.0f / 65536.0f;
  u[0] = ((lo & 0xffffu) + 0.5f) * s;
  u[1] = ((lo >> 16) + 0.5f) * s;
  u[2] = ((hi & 0xffffu) + 0.5f) * s;
  u[3] = ((hi >> 16) + 0.5f) * s;
}

}  // namespace svae

// Status codes returned by every C-ABI entry point.
#define SVAE_OK 0
#define SVAE_EINVAL 1
#define SVAE_ELAUNCH 2

#define SVAE_LAUNCH_CHECK()                                  \
  do {                                                       \
    hipError_t _e = hipGetLastError();                       \
    if (_e != hipSuccess) return SVAE_ELAUNCH;               \
  } while (0)
