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
