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
//
// The statement is self-contained in two ways hipcc cannot provide for inline asm (cdna_hip_programming.md §5.7):
//  * wait states: a VALU write of an SGPR needs 5 wait states before a VMEM instruction reads it as descriptor.
//    hipcc pads only its own instructions, and it does put such writes right in front of these statements (an
//    SGPR-spill reload `v_readlane_b32 s19, v208, 33` of a descriptor word, a `v_readfirstlane` recomputing a
//    base: 2-4 states before the load in attn_bwd8 / attn_bwd / the k-weighted gemm256, scripts/isa_audit.py).
//    The buffer_load then reads the descriptor's OLD words: silently wrong source data whenever the register held
//    something else before (the same descriptor re-loaded is harmless, which is why it hid). The string opens with
//    enough states (keep copy 1 + s_nop 1 (2) + m0 write 1 + s_nop 0 (1) = 5) so no instruction placed in front
//    of it can be inside the window.
//  * m0: compiler-reserved ("m0" in the clobber list is not honoured, only warned about); the statement saves it
//    and restores it after the issue (the DMA reads m0 at issue).
// scripts/isa_audit.py checks both on the built ISA (tests/test_isa_audit.py).
__device__ __forceinline__ u32x4 buffer_rsrc(const void* base, unsigned num_records) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  return (u32x4){(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)a),
                 (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)(a >> 32) & 0xFFFFu)), num_records,
                 0x00020000u};
}
__device__ __forceinline__ void dma16_lds(const u32x4& rsrc, const void* lds_base, int voff) {
  const int m = __builtin_amdgcn_readfirstlane((int)(unsigned)(uintptr_t)lds_base);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_nop 1\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "s"(m), "v"(voff), "s"(rsrc)
               : "memory");
}

// Four 1-KiB pieces to lds_base, + 1 KiB, + 2 KiB, + 3 KiB in ONE statement (same conventions as dma16_lds): m0 is
// saved, set and restored once and stepped by s_add between the loads (one wait state after each m0 write), 15
// instructions for the four pieces instead of 24 -- the GEMM K loop issues 8 pieces per wave per K-tile and its
// scalar issue (SQ_ACTIVE_INST_SCA ~0.1 of the wave cycles) was mostly these statements.
__device__ __forceinline__ void dma16x4_lds(const u32x4& rsrc, const void* lds_base, int v0, int v1, int v2, int v3) {
  const int m = __builtin_amdgcn_readfirstlane((int)(unsigned)(uintptr_t)lds_base);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_nop 1\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %2, %6, 0 offen lds\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %3, %6, 0 offen lds\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %4, %6, 0 offen lds\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %5, %6, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "s"(m), "v"(v0), "v"(v1), "v"(v2), "v"(v3), "s"(rsrc)
               : "memory", "scc");
}

// Two / three consecutive 1-KiB pieces in one statement (as dma16x4_lds).
__device__ __forceinline__ void dma16x2_lds(const u32x4& rsrc, const void* lds_base, int v0, int v1) {
  const int m = __builtin_amdgcn_readfirstlane((int)(unsigned)(uintptr_t)lds_base);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_nop 1\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %2, %4, 0 offen lds\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %3, %4, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "s"(m), "v"(v0), "v"(v1), "s"(rsrc)
               : "memory", "scc");
}
__device__ __forceinline__ void dma16x3_lds(const u32x4& rsrc, const void* lds_base, int v0, int v1, int v2) {
  const int m = __builtin_amdgcn_readfirstlane((int)(unsigned)(uintptr_t)lds_base);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_nop 1\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %2, %5, 0 offen lds\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %3, %5, 0 offen lds\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %4, %5, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "s"(m), "v"(v0), "v"(v1), "v"(v2), "s"(rsrc)
               : "memory", "scc");
}
// Two dword slots 256 B apart from two tensors (the attention backward's lse and delta rows of a query tile).
__device__ __forceinline__ void dma4x2_lds(const u32x4& rs_a, const u32x4& rs_b, const void* lds_base, int va, int vb) {
  const int m = __builtin_amdgcn_readfirstlane((int)(unsigned)(uintptr_t)lds_base);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_nop 1\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
               "buffer_load_dword %2, %4, 0 offen lds\n\ts_add_u32 m0, m0, 0x100\n\ts_nop 0\n\t"
               "buffer_load_dword %3, %5, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "s"(m), "v"(va), "v"(vb), "s"(rs_a), "s"(rs_b)
               : "memory", "scc");
}

// 4 B per lane (buffer_load_dword ... lds) into lds_base + 4 * lane, same conventions as dma16_lds.
__device__ __forceinline__ void dma4_lds(const u32x4& rsrc, const void* lds_base, int voff) {
  const int m = __builtin_amdgcn_readfirstlane((int)(unsigned)(uintptr_t)lds_base);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_nop 1\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dword %2, %3, 0 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "s"(m), "v"(voff), "s"(rsrc)
               : "memory");
}

// 1 B per lane (buffer_load_ubyte ... lds) into a dword slot per lane (lds_base + 4 * lane; the byte is the low
// 8 bits of the slot), same conventions as dma16_lds.
__device__ __forceinline__ void dma1_lds(const u32x4& rsrc, const void* lds_base, int voff) {
  const int m = __builtin_amdgcn_readfirstlane((int)(unsigned)(uintptr_t)lds_base);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_nop 1\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_ubyte %2, %3, 0 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "s"(m), "v"(voff), "s"(rsrc)
               : "memory");
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


// Status codes returned by every C-ABI entry point.
#define SVAE_OK 0
#define SVAE_EINVAL 1
#define SVAE_ELAUNCH 2

#define SVAE_LAUNCH_CHECK()                                  \
  do {                                                       \
    hipError_t _e = hipGetLastError();                       \
    if (_e != hipSuccess) return SVAE_ELAUNCH;               \
  } while (0)

__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
  typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, (bf16x2v){f2bf(a), f2bf(b)});
}

// Whole-line bf16 stores of one 16-row fragment row group straight from registers. After the permlane16 swap
// (gemm.hip's store_pair_bf16) lane (g, li) holds 8 consecutive columns of row li for each 32-column half jp: w0 (chunk cg) and
// w1 (chunk cg + 4) of the wave's 64 columns, so a store instruction would cover 16 rows x 64 B (half lines). A DPP
// row rotation by 8 swaps w1 between lanes li and li +- 8 (the bank mask keeps w0 in the other half): instruction
// 0 then writes rows 0-7 and instruction 1 rows 8-15, each 8 whole 128-B lines. No LDS, 12 VALU per row group.
// Nontemporal (NT) for the tensors read back only much later or by one streaming pass: the P-head's P (2 GiB at C2:
// head forward 1225 -> 1185 us; whole lines cached 1246, half lines nontemporal wrote 3.0 GB instead of 2.15) and the
// FFN's GELU' (its FFN-output GEMM, which reads the GELU output next, 110 -> 93 us: the MALL keeps the GELU output).
// The DPP merge of two 8-column chunks per lane (w[0]: chunk cg, w[1]: chunk cg + 4 of row li) and the two stores.
template <bool NT>
__device__ __forceinline__ void store_rows_w16(bf16* C, long long ldc, int mrow0, int M, int ncol0, int N,
                                               const u32x4 (&w)[2], int g, int li) {
  u32x4 h[2];
#pragma unroll
  for (int d = 0; d < 4; ++d) {   // row_ror:8 (dpp_ctrl 0x128); bank mask 0xC: lanes 8-15 of a row, 0x3: lanes 0-7
    h[0][d] = __builtin_amdgcn_update_dpp(w[0][d], w[1][d], 0x128, 0xF, 0xC, false);
    h[1][d] = __builtin_amdgcn_update_dpp(w[0][d], w[1][d], 0x128, 0xF, 0x3, false);
  }
  const int cg = ((g & 1) ? 2 : 0) + ((g & 2) ? 1 : 0), hi = li >> 3;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int m = mrow0 + 8 * hh + (li & 7), c = cg + 4 * (hi ^ hh), nleft = N - ncol0 - 8 * c;
    bf16* dst = C + (long long)(m < M ? m : 0) * ldc + ncol0 + 8 * c;
    if (m < M && nleft >= 8) {
      if constexpr (NT) __builtin_nontemporal_store(h[hh], (u32x4*)dst);
      else *(u32x4*)dst = h[hh];
    } else if (m < M && nleft > 0) *(u32x2*)dst = (u32x2){h[hh][0], h[hh][1]};
  }
}

template <bool NT>
__device__ __forceinline__ void store_rows_bf16(bf16* C, long long ldc, int mrow0, int M, int ncol0, int N,
                                                const f32x4 (&x)[4], int g, int li) {
  u32x4 w[2];
#pragma unroll
  for (int jp = 0; jp < 2; ++jp) {
    const f32x4 a = x[2 * jp], b = x[2 * jp + 1];
    const auto s0 = __builtin_amdgcn_permlane16_swap(pack_bf16x2(a[0], a[1]), pack_bf16x2(b[0], b[1]), false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(pack_bf16x2(a[2], a[3]), pack_bf16x2(b[2], b[3]), false, false);
    w[jp] = (u32x4){s0[0], s1[0], s0[1], s1[1]};
  }
  store_rows_w16<NT>(C, ldc, mrow0, M, ncol0, N, w, g, li);
}

// f32 rows: lane (g, li) holds columns 16 j + 4 g .. + 3 of row li; fragments j = 2 jp, 2 jp + 1 are the two halves
// of the 128-B line at columns 32 jp .. 32 jp + 31, merged the same way (chunk g and g + 4). N % 4 == 0. NPAIR
// fragment pairs (64 columns: 2; an hd-96 attention row: 3).
template <bool NT = false, int NPAIR = 2>
__device__ __forceinline__ void store_rows_f32(float* C, long long ldc, int mrow0, int M, int ncol0, int N,
                                               const f32x4 (&x)[2 * NPAIR], int g, int li) {
  const int hi = li >> 3;
#pragma unroll
  for (int jp = 0; jp < NPAIR; ++jp) {
    f32x4 h[2];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      h[0][d] = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x[2 * jp][d]), __float_as_int(x[2 * jp + 1][d]),
                                                           0x128, 0xF, 0xC, false));
      h[1][d] = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x[2 * jp][d]), __float_as_int(x[2 * jp + 1][d]),
                                                           0x128, 0xF, 0x3, false));
    }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int m = mrow0 + 8 * hh + (li & 7), n = ncol0 + 32 * jp + 4 * (g + 4 * (hi ^ hh));
      if (m < M && n < N) {
        if constexpr (NT) __builtin_nontemporal_store(h[hh], (f32x4*)(C + (long long)m * ldc + n));
        else *(f32x4*)(C + (long long)m * ldc + n) = h[hh];
      }
    }
  }
}

}  // namespace svae
