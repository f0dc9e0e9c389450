// Microbenchmark of the LDS-DMA slot pattern that read stale in the k-weighted head dW with the DMA stagger:
// 8 waves per block, a 2-stage ring of 64 KiB operand stages and per-wave 256-B slots. Per K-tile t every wave DMAs
// the 64 floats w[64 (t+1) .. +63] into its own slot of stage (t+1)&1 (dword LDS-DMA, one per lane) and 8 operand
// pieces (1 KiB each) into ring stage (t+1)&1; with LATE the wave-row-1 waves issue their pieces after the first MFMA
// quadrant instead of right after the barrier. After the next K-tile's vmcnt(0) + barrier each wave reads its slot of
// stage t&1 (column waves 0/1 after the second quadrant, 2/3 after the fourth; READ_EARLY = 0: all after the fourth)
// and counts the values that are not w[64 t + i]. Fragment reads of the current ring stage feed the MFMAs, as in the
// GEMM. Diagnostic only (scripts/dma_slot_race.py); not part of the library.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared scripts/dma_slot_race.hip -o scripts/libdmarace.so
#include "../sparse-vae_amd/csrc/common.h"

using namespace svae;

namespace {

constexpr int STAGE = 65536;
constexpr int SLOT_BASE_HI = 2 * STAGE + 10240;   // the GEMM's form-1 slot offset (138 KiB)

__device__ __forceinline__ void pieces(const u32x4& rs, char* stage, int wave, int t, int src_pieces) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int piece = (t * 64 + wave * 8 + i) % src_pieces;
    dma16_lds(rs, stage + (wave * 8 + i) * 1024, piece * 1024 + lane_id_fresh() * 16);
  }
}

template <bool LATE, bool READ_EARLY, bool SLOT_LOW, bool TR = false>
__global__ __launch_bounds__(512, 1) void race_kernel(const float* __restrict__ w, const bf16* __restrict__ src,
                                                      int src_pieces, int ntiles, unsigned* __restrict__ bad,
                                                      float* __restrict__ sink) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 10240 + 4096];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  char* ring = smem + (SLOT_LOW ? 4096 : 0);
  char* slots = smem + (SLOT_LOW ? 0 : SLOT_BASE_HI);
  const u32x4 wrs = buffer_rsrc(w, (unsigned)(ntiles * 64 * 4));
  const u32x4 srs = buffer_rsrc(src, (unsigned)(src_pieces * 1024));
  dma4_lds(wrs, slots + wave * 256, lane_id_fresh() * 4);
  pieces(srs, ring, wave, 0, src_pieces);
  f32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  unsigned nbad = 0;
  auto check = [&](int t) {
    const float* s = (const float*)(slots + ((t & 1) * 8 + wave) * 256) + 8 * (lane >> 4);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const f32x4 k0 = *(const f32x4*)(s + 32 * ks), k1 = *(const f32x4*)(s + 32 * ks + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float base = (float)(t * 64 + 32 * ks + 8 * (lane >> 4));
        nbad += (k0[e] != base + e) + (k1[e] != base + 4 + e);
      }
    }
  };
  auto quadrant = [&](const char* st, int q) {
    bf16x8 a[4], b;
    if constexpr (TR) {   // transposed reads (ds_read_b64_tr_b16 pairs), as the k-weighted GEMM's A operand
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const char* base = st + ((wave * 4 + i + q) % 64) * 1024 + (lane & 15) * 64 + (lane >> 4) * 8;
        a[i] = cat44(lds_read_tr(base), lds_read_tr(base + 32));
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *(const bf16x8*)(st + ((wave * 4 + i + q) % 64) * 1024 + lane * 16);
    }
    b = *(const bf16x8*)(st + ((wave + 32 + q) % 64) * 1024 + lane * 16);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[(i + r) & 7] = mfma16(b, a[i], acc[(i + r) & 7]);
  };
  for (int t = 0; t < ntiles; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const char* cur = ring + (t & 1) * STAGE;
    char* nxt = ring + ((t + 1) & 1) * STAGE;
    const bool more = t + 1 < ntiles;
    const bool late = LATE && wr == 1 && more;
    if (more) {
      dma4_lds(wrs, slots + (((t + 1) & 1) * 8 + wave) * 256, ((t + 1) * 64 + lane_id_fresh()) * 4);
      if (!late) pieces(srs, nxt, wave, t + 1, src_pieces);
    }
    quadrant(cur, 0);
    if (late) {
      __builtin_amdgcn_sched_barrier(0);
      pieces(srs, nxt, wave, t + 1, src_pieces);
      __builtin_amdgcn_sched_barrier(0);
    }
    quadrant(cur, 1);
    if (READ_EARLY && wc < 2) check(t);
    quadrant(cur, 2);
    quadrant(cur, 3);
    if (!READ_EARLY || wc >= 2) check(t);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) atomicAdd(bad + wave, nbad);
  float z = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) z += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (z == 12345.678f) sink[tid] = z;   // keeps the MFMAs
}

}  // namespace

extern "C" __attribute__((visibility("default"))) int dma_race_run(int variant, const float* w, const void* src,
                                                                   int src_pieces, int ntiles, int nblocks,
                                                                   unsigned* bad, float* sink, void* stream) {
  if (!w || !src || !bad || src_pieces < 64 || ntiles < 1 || nblocks < 1 || nblocks > 4096) return 1;
  const dim3 g((unsigned)nblocks), b(512);
  hipStream_t s = (hipStream_t)stream;
  const bf16* sp = (const bf16*)src;
  switch (variant) {
    case 0: hipLaunchKernelGGL((race_kernel<false, true, false>), g, b, 0, s, w, sp, src_pieces, ntiles, bad, sink); break;
    case 1: hipLaunchKernelGGL((race_kernel<true, true, false>), g, b, 0, s, w, sp, src_pieces, ntiles, bad, sink); break;
    case 2: hipLaunchKernelGGL((race_kernel<true, false, false>), g, b, 0, s, w, sp, src_pieces, ntiles, bad, sink); break;
    case 3: hipLaunchKernelGGL((race_kernel<true, true, true>), g, b, 0, s, w, sp, src_pieces, ntiles, bad, sink); break;
    case 4: hipLaunchKernelGGL((race_kernel<true, true, false, true>), g, b, 0, s, w, sp, src_pieces, ntiles, bad, sink); break;
    case 5: hipLaunchKernelGGL((race_kernel<false, true, false, true>), g, b, 0, s, w, sp, src_pieces, ntiles, bad, sink); break;
    default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
