// Flash attention forward / backward for the dense path of Attention.forward (attention.py:51-105):
//   scores = q k^T * hd^-0.5 (:83); scores -= 1e7 * (key_pad | causal) (:85-98); softmax . v (:100).
// A masked score contributes exactly 0 after exp (as the reference's -1e7 shift underflows to 0).
//
// Layout: q/k/v/o are token-major rows of H*hd bf16 (the nn.Linear output layout, heads interleaved),
// so no head-split copies exist. Head dim is padded to HDP = 64 or 128 inside the kernel.
//
// Forward: one block = 128 queries of one (batch, head), 4 waves x 32 queries. "Swapped" products keep the
// query on the MFMA lane: S^T = K . Q^T (K tile ds_read_b128, Q fragments in registers), then
// O^T += V^T . P^T where P^T is the S^T accumulator converted in place (key order permuted to match the
// ds_read_b64_tr_b16 reads of V). Online softmax per lane, no P round trip through LDS. K/V tiles of 64 keys by
// LDS-DMA one tile ahead.
//
// Backward: one block = 128 keys, 4 waves x 32 keys, sweeping 64-query tiles (key on the lane: S = Q K^T and
// dP = dO V^T accumulators are already the B operands of dV^T += dO^T P and dK^T += Q^T dS). dS^T goes
// through LDS once for dQ = dS K: each key block stores its f32 partial dQ into its own slice of dq_part (no
// atomics) and attn_dq_reduce_kernel sums the slices in a fixed order (deterministic).
#include "common.h"
#include <algorithm>
#include <type_traits>
#include "../../include/svae.h"

using namespace svae;

namespace {

struct AP {
  const bf16* q; const bf16* k; const bf16* v; bf16* o;
  long long sq, sk, sv, so, bq, bk, bv, bo;
  const unsigned char* pad; long long ldpad;   // key_pad [B][ldpad] (a key slice of a longer row: ldpad > Lk)
  float* lse;
  int B, H, Lq, Lk, hd, causal;
  float scale;
  const bf16* dout; long long sdo, bdo;
  const float* delta;
  float* dq; long long bdq;
  bf16* dk; bf16* dv; long long sdk, sdv, bdk, bdv;
  const float* rot; int rot_d;
  float* o32; long long so32, bo32;
  float* dq_part; void* dq_bf; long long ldq_bf;
  bf16* olo; long long solo, bolo;   // bf16 residual O - bf16(O) (alternative to o32)
  int window;        // > 0: causal sliding window of `window` 32-key blocks plus key block 0 (SparseAttention)
  int kblk;          // backward: keys per dQ partial (the key block of the kernel that wrote dq_part)
  int dq_direct;     // backward (attn_bwd8, causal): the final dQ of queries < dq_direct is stored by attn_bwd8 itself
  // backward, sliding window (attn_bwd8 path): queries >= cls_q0 see nothing of dQ plane 0 but the [CLS] block (keys
  // 0-31); plane 0's key blocks sweep only the queries below it, attn_bwd_cls_kernel takes the rest, and the [CLS]
  // keys' dK / dV go as f32 partial slabs into cls_part (slab 0 from attn_bwd8) summed by attn_cls_finalize_kernel.
  // 0 = off.
  int cls_q0;
  float* cls_part;
  // backward (attn_bwd8, hd <= 64, o_lo given): delta = rowsum(dO . O) computed inside the kernel (no attn_delta_kernel)
  int delta_inkernel;
  // backward, sliding window on the attn_bwd8 path: dQ planes pk >= 1 hold only their band's wrows query rows
  // (queries pk kblk .. + wrows - 1), after plane 0's B x Lq rows: O(L) instead of O(L^2 / kblk) floats. 0 = dense.
  int wrows;
  // forward, split-KV (svae_attn_fwd for few queries over many keys): grid z = B nsplit, slice sl = z % nsplit takes keys
  // sl kc .. + kc - 1 and writes its O / o_lo / lse into the split workspace (fwd_slice); 1 = off
  int nsplit, kc;
  bf16* split_o; bf16* split_olo; float* split_lse;
};

// The split-KV forward's view of one slice: batch b of a grid of B nsplit batches is (b / nsplit, slice b % nsplit); the
// slice's keys (pointers, padding row, length) and its outputs (the workspace's per-slice O, o_lo [B][Lq][H hd] and lse
// [B][H][Lq]) replace the problem's in p
__device__ __forceinline__ void fwd_slice(AP& p, int& b) {
  const int sl = b % p.nsplit;
  b /= p.nsplit;
  const int k0 = sl * p.kc;
  p.k += (long long)k0 * p.sk;
  p.v += (long long)k0 * p.sv;
  if (p.pad) p.pad += k0;   // (ldpad stays the full row)
  p.Lk = min(p.kc, p.Lk - k0);
  const long long D = (long long)p.H * p.hd, slice_o = (long long)p.B * p.Lq * D;
  p.o = p.split_o + sl * slice_o; p.so = D; p.bo = (long long)p.Lq * D;
  p.olo = p.split_olo + sl * slice_o; p.solo = D; p.bolo = (long long)p.Lq * D;
  p.o32 = nullptr;
  p.lse = p.split_lse + (long long)sl * p.B * p.H * p.Lq;
}

// Start of the (batch b) partial dQ of plane pk, indexed by ABSOLUTE query row: plane 0 and the dense layout [pk][B][Lq][D];
// the window's compact planes [pk - 1][B][wrows][D] after plane 0 (rows pk kblk .. ; the returned base is offset back by
// pk kblk rows, so base + q D addresses query q of the band)
__device__ __forceinline__ float* dq_plane(const AP& p, int pk, int b) {
  const long long D = (long long)p.H * p.hd;
  if (p.wrows > 0 && pk > 0)
    return p.dq_part + (long long)p.B * p.Lq * D + ((long long)(pk - 1) * p.B + b) * p.wrows * D - (long long)pk * p.kblk * D;
  return p.dq_part + ((long long)pk * p.B + b) * p.Lq * D;
}

// Block-sparse sliding window of SparseAttention (sparse_attention.py:39-60, causal, block 32): query q sees
// key k <= q iff k < 32 (the [CLS] block, layout[:, 0] = 1) or k / 32 >= q / 32 - (window - 1).
constexpr int SBLK = 32;
__device__ __forceinline__ int band_lo(int q, int window) {   // first in-band key of query q's 32-block
  return window > 0 ? max(0, (q / SBLK - (window - 1)) * SBLK) : 0;
}
__device__ __forceinline__ bool band_hidden(int key, int q, int window) {
  return window > 0 && key >= SBLK && key < band_lo(q, window);
}

// [64 rows][HDP] bf16 tile in LDS, 16-B chunks XOR-swizzled by (row & (chunks-1)): conflict-free for the
// row-wise ds_read_b128 fragment reads, <= 2-way for the ds_read_b64_tr_b16 reads.
template <int HDP>
struct Tile {
  static constexpr int NCH = HDP / 8;
  static constexpr int PITCH = HDP * 2;
  static constexpr int BYTES = 64 * PITCH;
  __device__ static __forceinline__ int off(int r, int c) { return r * PITCH + ((c ^ (r & (NCH - 1))) << 4); }
  __device__ static __forceinline__ int uoff(int r, int u) { return off(r, u >> 1) + ((u & 1) << 3); }
  // byte distance between rows r and r + 1 for 4-dim unit u; the swizzle sees row bits below log2(NCH) only, so
  // uoff(r + 16 k, u) = uoff(r, u) + 16 k row_pitch(u) (k >= 0)
  __device__ static constexpr int row_pitch(int) { return PITCH; }
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

// LDS-DMA (buffer_load ... lds, 16 B per lane) of rows [row0, row0+64) into a Tile<HDP> image: each wave
// instruction writes 1 KiB lane-linearly, so the chunk swizzle is applied to the SOURCE address. Rows >= nrows
// and dims >= hd get an out-of-range offset and land as zeros. No staging registers.
template <int HDP>
__device__ __forceinline__ void dma_rows(const bf16* g, long long ld, int row0, int nrows, int hd, char* lds, int w,
                                         int lane) {
  using T = Tile<HDP>;
  constexpr int NI = 64 * T::PITCH / 1024;   // wave instructions per tile: 8 (HDP 64) / 16 (HDP 128)
  const u32x4 rsrc = buffer_rsrc(g + (long long)row0 * ld, 0x7FFFFFF0u);
#pragma unroll
  for (int i = 0; i < NI / 4; ++i) {
    const int inst = w * (NI / 4) + i;
    const int byte = inst * 1024 + lane * 16;
    const int r = byte / T::PITCH, c = ((byte % T::PITCH) >> 4) ^ (r & (T::NCH - 1));
    const bool ok = row0 + r < nrows && c * 8 < hd;
    dma16_lds(rsrc, lds + inst * 1024, ok ? (r * (int)ld + c * 8) * 2 : 0x7FFFFFF0);
  }
}

// RowImg<HDC>: 64 rows x HDC bf16. Dims 0-63: the Tile<64> image (128-B rows, chunk c ^ (r & 7)). HDC = 96: dims
// 64-95 follow as [64 rows][4 chunks] (64-B rows) with chunk swizzle c ^ tail_swz(r): rows r, r + 4, r + 8, r + 12
// share banks, so tail_swz takes 4 distinct values over bits 2-3 of r (the 16-row b128 reads) and differs in bit 1
// between r and r + 4 and between r and r + 8 (the transposed reads of rows 4g + q and 8g + q): conflict-free.
template <int HDC>
struct RowImg {
  static_assert(HDC == 64 || HDC == 96, "RowImg: 64 or 96 dims");
  static constexpr int NCH = HDC / 8;               // 16-B chunks per row
  static constexpr int BYTES = 64 * HDC * 2;        // 8 or 12 KiB
  static constexpr int PIECES = BYTES / 1024;       // LDS-DMA wave-instructions per image
  __device__ static __forceinline__ int tail_swz(int r) { return ((((r >> 2) ^ (r >> 3)) & 1) << 1) | ((r >> 2) & 1); }
  // byte offset of (row r < 64, logical chunk c)
  __device__ static __forceinline__ int off(int r, int c) {
    if (HDC == 64 || c < 8) return r * 128 + ((c ^ (r & 7)) << 4);
    return 8192 + r * 64 + (((c - 8) ^ tail_swz(r)) << 4);
  }
  // 8-B unit u (dims 4u .. 4u + 3) of row r
  __device__ static __forceinline__ int uoff(int r, int u) { return off(r, u >> 1) + ((u & 1) << 3); }
  // as Tile::row_pitch (the swizzles see row bits 0-3 only)
  __device__ static constexpr int row_pitch(int u) { return (HDC == 64 || u < 16) ? 128 : 64; }
  // the LDS slot of lane `lane` in DMA piece i: row r and logical chunk c it receives (swizzle undone)
  __device__ static __forceinline__ void piece_src(int i, int lane, int& r, int& c) {
    if (HDC == 64 || i < 8) {
      r = 8 * i + (lane >> 3);
      c = (lane & 7) ^ (r & 7);
    } else {
      r = 16 * (i - 8) + (lane >> 2);
      c = ((lane & 3) ^ tail_swz(r)) + 8;
    }
  }
};

// LDS-DMA of piece i of the RowImg of rows [row0, row0 + 64) of a token-major matrix whose row 0 the descriptor
// addresses (offsets stay below 2^31 bytes: checked by svae_attn_bwd); rows >= nrows and dims >= hd land as zeros
// (out-of-range source offset)
template <int HDC>
__device__ __forceinline__ void dma_img_piece(const u32x4& rsrc, long long ld, int row0, int nrows, int hd, char* img,
                                              int i, int lane) {
  int r, c;
  RowImg<HDC>::piece_src(i, lane, r, c);
  const bool ok = row0 + r < nrows && c * 8 < hd;
  dma16_lds(rsrc, img + i * 1024, ok ? ((row0 + r) * (int)ld + c * 8) * 2 : 0x7FFFFFF0);
}

// The forward's K / V tile layout: RowImg for hd <= 96 (64 or 96 dims per row: hd 96 no longer pays 128-wide rows, so
// three workgroups fit a CU), Tile<128> for hd 128.
template <int HDP, int HDC>
struct FwdTile {
  using type = Tile<HDP>;
};
template <>
struct FwdTile<64, 64> {
  using type = RowImg<64>;
};
template <>
struct FwdTile<128, 96> {
  using type = RowImg<96>;
};
// rows [row0, row0 + 64) of a token-major matrix (row 0 at g) into the LDS image; the 4 waves split the pieces
template <int HDP>
__device__ __forceinline__ void dma_tile(const Tile<HDP>*, const bf16* g, long long ld, int row0, int nrows, int hd,
                                         char* lds, int w, int lane) {
  dma_rows<HDP>(g, ld, row0, nrows, hd, lds, w, lane);
}
template <int HDC>
__device__ __forceinline__ void dma_tile(const RowImg<HDC>*, const bf16* g, long long ld, int row0, int nrows, int hd,
                                         char* lds, int w, int lane) {
  constexpr int PW = RowImg<HDC>::PIECES / 4;
  static_assert(PW * 4 == RowImg<HDC>::PIECES, "pieces split over the 4 waves");
  const u32x4 rs = buffer_rsrc(g, 0x7FFFFFF0u);
  const int ln = lane_id_fresh();   // (offsets recomputed here, not kept live across the key loop)
  if constexpr (PW == 2 || PW == 3) {   // the wave's consecutive pieces in one statement
    int o[3];
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      int r, c;
      RowImg<HDC>::piece_src(w * PW + i, ln, r, c);
      const bool ok = row0 + r < nrows && c * 8 < hd;
      o[i] = ok ? ((row0 + r) * (int)ld + c * 8) * 2 : 0x7FFFFFF0;
    }
    if constexpr (PW == 2) dma16x2_lds(rs, lds + w * PW * 1024, o[0], o[1]);
    else dma16x3_lds(rs, lds + w * PW * 1024, o[0], o[1], o[2]);
  } else {
#pragma unroll
    for (int i = 0; i < PW; ++i) dma_img_piece<HDC>(rs, ld, row0, nrows, hd, lds, w * PW + i, ln);
  }
}
template <int HDP>
constexpr int tile_pieces(const Tile<HDP>*) { return 64 * Tile<HDP>::PITCH / 1024; }
template <int HDC>
constexpr int tile_pieces(const RowImg<HDC>*) { return RowImg<HDC>::PIECES; }

__device__ __forceinline__ bf16x8 pack8(const f32x4& a, const f32x4& b) {
  return (bf16x8){f2bf(a[0]), f2bf(a[1]), f2bf(a[2]), f2bf(a[3]), f2bf(b[0]), f2bf(b[1]), f2bf(b[2]), f2bf(b[3])};
}


constexpr float LOG2E = 1.4426950408889634f;


// ===================================================================================== forward
// One block = 128 queries of one (batch, head): 4 waves x 32 queries (two 16-query MFMA column tiles), so
// every K fragment and V^T fragment read from LDS feeds two MFMAs. K/V tiles arrive by LDS-DMA one tile ahead
// (asm-issued, so the compiler adds no drain before the transposed V reads) with one counted wait + barrier per
// tile; 3 blocks per CU for hd <= 64. Softmax in the exp2 domain with the raw
// (unscaled) running max: p = exp2(s c - m c), c = scale log2(e). Masks only on edge tiles (causal diagonal,
// ragged end, padded keys present); causal tiles entirely above a wave's queries are skipped.
// s_waitcnt vmcnt(n) for a run-time n (the immediate must be a constant): n = vector-memory ops allowed to stay in
// flight (vmcnt retires in issue order, so this waits for everything older than the n youngest).
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
    case 32: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    case 34: asm volatile("s_waitcnt vmcnt(34)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// XCD-aware block order: hardware dispatch sends block i to XCD i % 8; remap so that logically consecutive blocks
// (the query tiles, or key blocks, of one (batch, head)) run on the same XCD and share its L2 for K/V (Q/dO).
// C2 decoder shape (scripts/attn_probe.py): fwd 71.7 -> 67.5 us, bwd 227.6 -> 222.5 us; L = 1024: fwd 208 -> 171 us.
// Causal work order (lpt != 0): a block's work grows with x (lpt = 1: forward query tiles) or shrinks with x
// (lpt = 2: backward key blocks). Inside an XCD's range of whole (batch, head) pairs the blocks are then dispatched
// longest first, x-major per chunk of pairs (the pair-major order put the longest blocks of the last pairs at the
// end: a tail of idle CUs; list-scheduling model of the C2 decoder shape: backward makespan 29 -> 24 block-tiles,
// forward 21 -> 17; measured at C2: forward 59.3 -> 52.6 us, backward + delta + dQ reduce 202 -> 182 us).
__device__ __forceinline__ void xcd_block(int& x, int& y, int& z, int lpt = 0) {
  const int gx = gridDim.x, gy = gridDim.y;
  const int n = gx * gy * gridDim.z;
  const int lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  int l = lin;
  if (n >= 16) {
    const int q = n / 8, r = n % 8, xcd = lin % 8, idx = lin / 8;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q, cnt = xcd < r ? q + 1 : q;
    l = base + idx;
    if (lpt && gx > 1 && base % gx == 0 && cnt % gx == 0) {
      // in chunks of 32 pairs (their K/V, or Q/dO, stay L2-resident while the chunk runs; x-major over all the
      // XCD's pairs made the B = 256 forward 7 % slower)
      constexpr int CH = 32;
      const int np = cnt / gx, c = idx / (CH * gx), local = idx - c * CH * gx, cp = min(CH, np - c * CH);
      const int rank = local / cp, pair = base / gx + c * CH + (local - rank * cp);
      x = lpt == 1 ? gx - 1 - rank : rank;
      y = pair % gy;
      z = pair / gy;
      return;
    }
  }
  x = l % gx;
  y = (l / gx) % gy;
  z = l / (gx * gy);
}

#ifdef SVAE_STAMPS
// diagnostic build only (make stamps): s_memtime at block start / after the first K/V tile's wait / after the key
// loop / at the end, for the first 1024 hardware block ids, plus the block's tile count and query tile
__device__ unsigned long long svae_attn_stamps[1024][6];
#define ATTN_STAMP(k, v) \
  do { if (lin_id < 1024 && threadIdx.x == 0) svae_attn_stamps[lin_id][k] = (v); } while (0)
#else
#define ATTN_STAMP(k, v) ((void)0)
#endif

constexpr int ATTN_NS = 2;   // K/V ring stages (3 stages with the XCD order: 70.7 vs 67.5 us)


// One 128-query tile of one (batch, head). smem: the K/V ring + key-padding ring of the kernel. HDP: the LDS row
// width (64 or 128 dims); HDC <= HDP: the dims the MFMAs cover (hd 96 runs HDC = 96 on 128-wide rows: no work on the
// zero padding).
template <int HDP, int HDC = HDP>
__device__ __forceinline__ void attn_fwd_tile(const AP& p, char* smem, int bx, int h, int b) {
  using T = typename FwdTile<HDP, HDC>::type;
  constexpr int NKK = HDC / 32, NT = HDC / 16;
  // K/V ring: NS stages of (K, V) tiles filled NS - 1 key tiles ahead; the key-padding bytes ride along in an
  // [NS][64] ring. Measured at the C2 shape (hd 64): 2 stages at 3 blocks / CU (33 KB LDS, <= 170 VGPRs) beat
  // 3 or 4 stages at 2 blocks / CU (73.5 vs 78.4 / 92 us): blocks in flight, not prefetch depth, set the time.
  constexpr int NS = ATTN_NS;
  constexpr int DMA_OPS = 2 * tile_pieces((const T*)nullptr) / 4;   // buffer_load_lds per wave per (K, V) tile
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar branches, not exec masks
  const int q0 = bx * 128;
#ifdef SVAE_STAMPS
  const int lin_id = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  ATTN_STAMP(0, __builtin_amdgcn_s_memtime());
#endif
  const bf16* Q = p.q + b * p.bq + (long long)h * p.hd;
  const bf16* K = p.k + b * p.bk + (long long)h * p.hd;
  const bf16* V = p.v + b * p.bv + (long long)h * p.hd;
  const unsigned char* pad = p.pad ? p.pad + b * p.ldpad : nullptr;
  // key-padding ring: one dword per key (LDS-DMA writes a dword slot per lane; the byte is its low 8 bits), one ring
  // per wave ([wave][NS][64]): every wave DMAs the bytes it reads itself (no wave reads another wave's DMA)
  unsigned* pm = (unsigned*)(smem + NS * 2 * T::BYTES);

  const int qw = q0 + 32 * w;
  bf16x8 qf[2][NKK];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      const int qrow = qw + 16 * j + li, d = 32 * kk + 8 * g;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (qrow < p.Lq && d < p.hd) v = *(const u32x4*)(Q + (long long)qrow * p.sq + d);
      qf[j][kk] = __builtin_bit_cast(bf16x8, v);
    }
  f32x4 o[2][NT];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < NT; ++t) o[j][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // (Row sums of P by MFMA against a ones column of V^T -- 4 MFMAs per tile instead of 32 VALU adds -- sum the
  // bf16-rounded P; measured: that moves a gradient norm ratio of the windowed small6_pad parity case from < 2 %
  // to 2.03 %, so the row sums stay f32 VALU adds.)
  float m[2] = {-1e30f, -1e30f}, ls[2] = {0.f, 0.f};
  const int kv_end = p.causal ? min(p.Lk, q0 + 128) : p.Lk;
  const int ntiles = (kv_end + 63) / 64;
  const float c = p.scale * LOG2E;
  // key tiles visited: tile 0, then the band from the tile holding the block's first in-band key (dense: all)
  const int kt1 = max(1, band_lo(q0, p.window) / 64);
  const int nvisit = 1 + max(0, ntiles - kt1);
  const int lo_w = band_lo(qw, p.window);          // this wave's 32 queries share one 32-block
  // vector-memory ops one tile issue adds per wave: the K and V pieces, and the key-padding bytes (DMA'd into the
  // wave's own [NS][64] ring like the tiles: no register round trip, no compiler-visible load to wait for)
  const int ops = DMA_OPS + (pad ? 1 : 0);
  const u32x4 prs = buffer_rsrc(pad ? (const void*)pad : (const void*)p.q, pad ? (unsigned)p.Lk : 0u);
  auto issue = [&](int it2) {
    const int kn = (it2 == 0 ? 0 : kt1 + it2 - 1) * 64;
    char* nb = smem + (it2 % NS) * 2 * T::BYTES;
    dma_tile((const T*)nullptr, K, p.sk, kn, p.Lk, p.hd, nb, w, lane);
    dma_tile((const T*)nullptr, V, p.sv, kn, p.Lk, p.hd, nb + T::BYTES, w, lane);
    if (pad) dma1_lds(prs, pm + (w * NS + it2 % NS) * 64, kn + lane < p.Lk ? kn + lane : 0x7FFFFFF0);
  };
  if (!pad)
    for (int i = tid; i < 4 * NS * 64; i += 256) pm[i] = 0;
#pragma unroll
  for (int s2 = 0; s2 < NS - 1; ++s2)
    if (s2 < nvisit) issue(s2);
  // Consume the Q fragments here (after the ring's first DMA is in flight, so the two latencies overlap): the
  // compiler cannot see the DMA, so its wait for them is a vmcnt(0); here that costs nothing (tile 0 is needed
  // next anyway), inside the loop it would drain the ring.
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) asm volatile("" ::"v"(__builtin_bit_cast(u32x4, qf[j][kk])));

  for (int it = 0; it < nvisit; ++it) {
    const int kt = it == 0 ? 0 : kt1 + it - 1;
    const int st = it % NS;
    const char* Ks = smem + st * 2 * T::BYTES;
    const char* Vs = Ks + T::BYTES;
    const unsigned* pms = pm + (w * NS + st) * 64;
    wait_vmcnt(min(NS - 2, nvisit - 1 - it) * ops);   // this wave's pieces of tile it have landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // everyone's have; stage (it - 1) % NS is free (a raw barrier: __syncthreads
                                    // would also drain the younger tiles' DMA with its vmcnt(0))
    if (it + NS - 1 < nvisit) issue(it + NS - 1);
#ifdef SVAE_STAMPS
    if (it == 0) ATTN_STAMP(1, __builtin_amdgcn_s_memtime());
#endif
    const int kbase = kt * 64;
    if ((!p.causal || kbase <= qw + 31) && (kbase < SBLK || kbase + 63 >= lo_w)) {
      // S^T = K . Q^T : s[j][st][r] = score(key = kbase + 16st + 4g + r, query = qw + 16j + li)
      f32x4 s[2][4];
#pragma unroll
      for (int sx = 0; sx < 4; ++sx) {
        s[0][sx] = (f32x4){0.f, 0.f, 0.f, 0.f};
        s[1][sx] = s[0][sx];
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) {
          const bf16x8 kf = *(const bf16x8*)(Ks + T::off(16 * sx + li, g + 4 * kk));
          s[0][sx] = mfma16(kf, qf[0][kk], s[0][sx]);
          s[1][sx] = mfma16(kf, qf[1][kk], s[1][sx]);
        }
      }
      const bool pad_any = pad && __builtin_amdgcn_ballot_w64((pms[lane] & 0xFFu) != 0) != 0;
      const bool band_edge = kbase + 63 >= SBLK && kbase < lo_w;
      if (HDC == 64 && !pad_any && !band_edge && (kbase + 64 > p.Lk || (p.causal && kbase + 63 > qw))) {
        // The causal diagonal / ragged end alone (the common edge tile): key kl = 16 sx + 4 g + r is visible iff
        // kl < lim_j, i.e. 16 sx + r < lim_j - 4 g -- one compare against an inline constant and one select per score
        // instead of ~5 VALU + 2 hazard nops (the general form below). hd 64 only: at hd 96 the second path raised the
        // forward's spills from 1 to 17 VGPRs.
        const int t0 = (p.causal ? min(p.Lk, qw + li + 1) : p.Lk) - kbase - 4 * g;
        const int t1 = (p.causal ? min(p.Lk, qw + 16 + li + 1) : p.Lk) - kbase - 4 * g;
#pragma unroll
        for (int sx = 0; sx < 4; ++sx)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s[0][sx][r] = 16 * sx + r < t0 ? s[0][sx][r] : -INFINITY;
            s[1][sx][r] = 16 * sx + r < t1 ? s[1][sx][r] : -INFINITY;
          }
      } else if (pad_any || kbase + 64 > p.Lk || (p.causal && kbase + 63 > qw) || band_edge) {
        // Edge tile (wave-uniform branch). The per-key tests are branch-free: bitwise ORs of compares feeding one
        // select per score (short-circuit || compiled to an exec-mask branch per score, ~5 scalar instructions each).
        // This lane's keys are kl = 16 sx + 4 g + r; its key-padding bits come from 4 16-B LDS reads.
        unsigned pbits = 0;
        if (pad_any) {
#pragma unroll
          for (int sx = 0; sx < 4; ++sx) {
            const u32x4 pw = *(const u32x4*)(pms + 16 * sx + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r) pbits |= (unsigned)((pw[r] & 0xFFu) != 0u) << (4 * sx + r);
          }
        }
        // visible iff kl < lim_j (ragged end; causal: key <= query) and not (hlo <= kl < hhi) (outside the window band)
        const int lim0 = (p.causal ? min(p.Lk, qw + li + 1) : p.Lk) - kbase;
        const int lim1 = (p.causal ? min(p.Lk, qw + 16 + li + 1) : p.Lk) - kbase;
        const int hlo = SBLK - kbase, hhi = lo_w - kbase;
#pragma unroll
        for (int sx = 0; sx < 4; ++sx)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int kl = 16 * sx + 4 * g + r;
            const unsigned hid = ((pbits >> (4 * sx + r)) & 1u) | ((unsigned)(kl >= hlo) & (unsigned)(kl < hhi));
            s[0][sx][r] = (hid | (unsigned)(kl >= lim0)) ? -INFINITY : s[0][sx][r];
            s[1][sx][r] = (hid | (unsigned)(kl >= lim1)) ? -INFINITY : s[1][sx][r];
          }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float mx = -INFINITY;
#pragma unroll
        for (int sx = 0; sx < 4; ++sx) {   // (v_max3_f32 chains: 8 per 16 scores)
          mx = fmaxf(fmaxf(mx, s[j][sx][0]), s[j][sx][1]);
          mx = fmaxf(fmaxf(mx, s[j][sx][2]), s[j][sx][3]);
        }
        mx = max_x16_x32(mx);
        // rescale O and the row sum only when some row's max grew (wave-uniform branch; alpha would be exactly 1
        // for every other row, so the result is bit-identical to rescaling every tile)
        if (__builtin_amdgcn_ballot_w64(mx > m[j]) != 0) {
          const float mn = fmaxf(m[j], mx);
          const float alpha = __builtin_amdgcn_exp2f((m[j] - mn) * c);
          m[j] = mn;
          ls[j] *= alpha;
#pragma unroll
          for (int t = 0; t < NT; ++t) o[j][t] *= alpha;
        }
        const float mc = m[j] * c;
#pragma unroll
        for (int sx = 0; sx < 4; ++sx)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float pv = __builtin_amdgcn_exp2f(fmaf(s[j][sx][r], c, -mc));
            s[j][sx][r] = pv;
            ls[j] += pv;
          }
      }
      // O^T += V^T . P^T  (keys of k-step kk: 32kk + 16(jj>>2) + 4g + (jj&3))
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 pf0 = pack8(s[0][2 * kk], s[0][2 * kk + 1]);
        const bf16x8 pf1 = pack8(s[1][2 * kk], s[1][2 * kk + 1]);
        const int rq = 4 * g + (li >> 2);   // row 32 kk + rq: a constant offset from row rq (folded into the ds_read)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int u = 4 * t + (li & 3);
          const int pt = T::row_pitch(4 * t);
          const lds_char* pv = lds_ptr(Vs) + T::uoff(rq, u) + 32 * kk * pt;
          const bf16x8 vf = cat44(lds_read_tr3(pv), lds_read_tr3(pv + 16 * pt));
          o[0][t] = mfma16(vf, pf0, o[0][t]);
          o[1][t] = mfma16(vf, pf1, o[1][t]);
        }
      }
    }
  }

#ifdef SVAE_STAMPS
  ATTN_STAMP(2, __builtin_amdgcn_s_memtime());
  ATTN_STAMP(4, (unsigned long long)nvisit);
  ATTN_STAMP(5, (unsigned long long)bx);
#endif
  if ((HDC == 64 || HDC == 96) && p.hd == HDC) {
    // whole-line stores (common.h): O's first 64 dims as 8 rows x 128 B per instruction (hd 96: the last 32 dims as
    // before), its f32 copy nontemporal (read only by the backward's delta pass): 55 -> 51 us at the C2 decoder shape
    constexpr int NP = HDC / 32;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float lsum = sum_x16_x32(ls[j]);
      const float inv = lsum > 0.f ? 1.0f / lsum : 0.f;
      f32x4 v[2 * NP];
#pragma unroll
      for (int t = 0; t < 2 * NP; ++t) v[t] = o[j][t < NT ? t : 0] * inv;
      bf16* O = p.o + b * p.bo + (long long)h * HDC;
      store_rows_bf16<false>(O, p.so, qw + 16 * j, p.Lq, 0, 64, *(const f32x4(*)[4])v, g, li);
      const int qrow = qw + 16 * j + li;
      if (HDC == 96 && qrow < p.Lq) {
#pragma unroll
        for (int t = 4; t < 2 * NP; ++t) {
          const int d = 16 * t + 4 * g;
          *(bf16x4*)(O + (long long)qrow * p.so + d) = (bf16x4){f2bf(v[t][0]), f2bf(v[t][1]), f2bf(v[t][2]), f2bf(v[t][3])};
        }
      }
      if (p.o32)
        store_rows_f32<true, NP>(p.o32 + b * p.bo32 + (long long)h * HDC, p.so32, qw + 16 * j, p.Lq, 0, HDC, v, g, li);
      if (p.olo) {   // bf16 residual O - bf16(O)
        f32x4 lo[2 * NP];
#pragma unroll
        for (int t = 0; t < 2 * NP; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) lo[t][e] = v[t][e] - (float)f2bf(v[t][e]);
        bf16* OL = p.olo + b * p.bolo + (long long)h * HDC;
        store_rows_bf16<false>(OL, p.solo, qw + 16 * j, p.Lq, 0, 64, *(const f32x4(*)[4])lo, g, li);
        if (HDC == 96 && qrow < p.Lq) {
#pragma unroll
          for (int t = 4; t < 2 * NP; ++t) {
            const int d = 16 * t + 4 * g;
            *(bf16x4*)(OL + (long long)qrow * p.solo + d) =
                (bf16x4){f2bf(lo[t][0]), f2bf(lo[t][1]), f2bf(lo[t][2]), f2bf(lo[t][3])};
          }
        }
      }
      if (g == 0 && qrow < p.Lq) p.lse[((long long)b * p.H + h) * p.Lq + qrow] = m[j] * p.scale + __logf(lsum);
    }
  } else {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float lsum = sum_x16_x32(ls[j]);
    const int qrow = qw + 16 * j + li;
    if (qrow < p.Lq) {
      const float inv = lsum > 0.f ? 1.0f / lsum : 0.f;
      bf16* O = p.o + b * p.bo + (long long)h * p.hd + (long long)qrow * p.so;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int d = 16 * t + 4 * g;
        if (d < p.hd) {
          const f32x4 v = o[j][t] * inv;
          *(bf16x4*)(O + d) = (bf16x4){f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
          if (p.o32) *(f32x4*)(p.o32 + b * p.bo32 + (long long)h * p.hd + (long long)qrow * p.so32 + d) = v;
          if (p.olo)
            *(bf16x4*)(p.olo + b * p.bolo + (long long)h * p.hd + (long long)qrow * p.solo + d) =
                (bf16x4){f2bf(v[0] - (float)f2bf(v[0])), f2bf(v[1] - (float)f2bf(v[1])), f2bf(v[2] - (float)f2bf(v[2])),
                         f2bf(v[3] - (float)f2bf(v[3]))};
        }
      }
      if (g == 0) p.lse[((long long)b * p.H + h) * p.Lq + qrow] = m[j] * p.scale + __logf(lsum);
    }
  }
  }
#ifdef SVAE_STAMPS
  ATTN_STAMP(3, __builtin_amdgcn_s_memtime());
#endif
}

// One query tile per workgroup. (Running query tiles x and nqt - 1 - x in one workgroup, to even out the causal
// work, measured 68 -> 73 us at the C2 shape on two boxes out of three, scripts/attn_probe.py: half the workgroups
// in flight cost more than the imbalance.)
template <int HDP, int HDC = HDP>
__global__ __launch_bounds__(256, HDC <= 96 ? 3 : 2) void attn_fwd_kernel(AP p) {
  __shared__ __attribute__((aligned(16))) char smem[ATTN_NS * 2 * FwdTile<HDP, HDC>::type::BYTES + 4 * ATTN_NS * 64 * 4];
  int bx, h, b;
  xcd_block(bx, h, b, p.causal ? 1 : 0);
  if (p.nsplit > 1) fwd_slice(p, b);
  attn_fwd_tile<HDP, HDC>(p, smem, bx, h, b);
}

// ===================================================================================== forward, 32 x 32 MFMA form
// attn_fwd32_kernel<HDC> (HDC = 64: hd <= 64, zero-padded; HDC = 96): the same flash forward as attn_fwd_kernel, with
// v_mfma_f32_32x32x16_bf16 instead of 16x16x32 and a deferred running max. Why (the forward is issue-bound: per 64-key
// tile a wave issues ~930 cycles of VALU + MFMA beside 512 cycles of MFMA work, §6):
//  * a 32x32x16 MFMA holds the SIMD's vector issue for 8 of its 32 cycles, the 16x16x32 form for 8 of 16: half the
//    MFMA issue cost for the same flops (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost');
//  * S^T = K . Q^T puts ONE query on each lane (column = lane & 31) with 16 keys per 32-key tile in the registers, so a
//    row reduction is in-lane plus one permlane32 swap, and the accumulator is the B operand of O^T += V^T . P^T with no
//    lane movement (cdna_hip_programming.md §3, 'An accumulator tile as the next MFMA's operand');
//  * no per-tile row max: p = exp2(s c - m c) against the running reference m, and only when some lane's tile sum
//    exceeds 2^16 (or is not finite) does the wave take the rescale path (recompute S, true max, rescale O and l).
//    Every p then stays <= 2^16 (bf16 keeps its relative precision at any magnitude; O and l accumulate in f32), and
//    the lse = m scale + ln l is exact for any reference m. A wave's first live tile sets m to the true max.
// K / V images: 64 key rows, 16-B chunks XOR-swizzled so that both the row-wise ds_read_b128 K reads (lane = key row
// 0..31) and the transposed ds_read_b64_tr_b16 V reads (4 consecutive rows x 4 chunks per 32 lanes) are conflict-free.
template <int HDC>
struct KVImg {
  static_assert(HDC == 64 || HDC == 96, "KVImg: 64 or 96 dims");
  static constexpr int BYTES = 64 * HDC * 2;         // 8 / 12 KiB
  static constexpr int PIECES = BYTES / 1024;        // LDS-DMA wave-instructions per image
  // dims 0-63: 128-B rows, chunk c at c ^ F(r). b128 reads: the 8 even (odd) rows of a 16-lane group get 8 distinct
  // chunks; tr reads: rows r0, r0 + 2 (r0 % 4 == 0) differ in bit 2 of F, so their 4-chunk groups are disjoint.
  __device__ static __forceinline__ int F(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
  // dims 64-95 (HDC 96): 64-B rows at 8192, chunk c at c ^ T(r): the 4 rows of each r % 4 class in a 16-lane b128 group
  // get 4 distinct chunks
  __device__ static __forceinline__ int T(int r) { return ((r >> 2) ^ (r >> 3)) & 3; }
  __device__ static __forceinline__ int off(int r, int c) {
    if (HDC == 64 || c < 8) return r * 128 + ((c ^ F(r)) << 4);
    return 8192 + r * 64 + (((c - 8) ^ T(r)) << 4);
  }
  // the source row r and logical chunk c of lane `lane`'s 16-B slot in DMA piece i
  __device__ static __forceinline__ void piece_src(int i, int lane, int& r, int& c) {
    if (HDC == 64 || i < 8) {
      r = 8 * i + (lane >> 3);
      c = (lane & 7) ^ F(r);
    } else {
      r = 16 * (i - 8) + (lane >> 2);
      c = 8 + ((lane & 3) ^ T(r));
    }
  }
};

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 lds_read_b128(const lds_char* p) {
  return *(const __attribute__((address_space(3))) bf16x8*)p;
}
// registers 8 s .. 8 s + 7 of a 32x32 accumulator as a bf16 fragment (k-step s of the next product)
__device__ __forceinline__ bf16x8 pack_acc8(const f32x16& x, int s) {
  return (bf16x8){f2bf(x[8 * s]), f2bf(x[8 * s + 1]), f2bf(x[8 * s + 2]), f2bf(x[8 * s + 3]),
                  f2bf(x[8 * s + 4]), f2bf(x[8 * s + 5]), f2bf(x[8 * s + 6]), f2bf(x[8 * s + 7])};
}
// reductions over the lane pair (l, l ^ 32) (one permlane32 swap: each lane gets its own and its partner's value)
__device__ __forceinline__ float max_x32(float v) {
  auto c = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(c[0]), __uint_as_float(c[1]));
}
__device__ __forceinline__ float sum_x32(float v) {
  auto c = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(c[0]) + __uint_as_float(c[1]);
}

#ifndef SVAE_FWD32_DIAG
#define SVAE_FWD32_DIAG 0   // diagnostic builds only (scripts/build_variant.sh ... -DSVAE_FWD32_DIAG=n): 1 no tile body, 2 no
#endif                      // exp2 / fma, 3 one S MFMA per subtile, 4 one PV MFMA per k-step; results are wrong
constexpr int FWD32_MAXPAD = 4096;    // keys whose padding bits fit the block's LDS bit mask
constexpr float FWD32_THRESH = 65536.f;

template <int HDC, int OCC, int NS>
__global__ __launch_bounds__(256, OCC) void attn_fwd32_kernel(AP p) {
  using I = KVImg<HDC>;                 // NS: K / V ring stages (NS - 1 tiles ahead)
  constexpr int KS = HDC / 16;          // k-steps of S = Q K^T
  constexpr int DT = HDC / 32;          // 32-dim tiles of O^T
  constexpr int PW = I::PIECES / 4;     // DMA pieces per wave per image
  __shared__ __attribute__((aligned(16))) char smem[NS * 2 * I::BYTES + FWD32_MAXPAD / 8];
  int bx, h, b;
  xcd_block(bx, h, b, p.causal ? 1 : 0);
  if (p.nsplit > 1) fwd_slice(p, b);
  const int tid = threadIdx.x, lane = tid & 63, r32 = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q0 = bx * 128, qw = q0 + 32 * w, qrow = qw + r32;
  const bf16* Q = p.q + b * p.bq + (long long)h * p.hd;
  const bf16* K = p.k + b * p.bk + (long long)h * p.hd;
  const bf16* V = p.v + b * p.bv + (long long)h * p.hd;

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[qrow][16 ks + 8 hh .. + 7]
  bf16x8 qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int d = 16 * ks + 8 * hh;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (qrow < p.Lq && d < p.hd) v = *(const u32x4*)(Q + (long long)qrow * p.sq + d);
    qf[ks] = __builtin_bit_cast(bf16x8, v);
  }
  // key padding as a bit mask in LDS (bit k of word k / 64), built once per block by ballots: plain loads, read after
  // the first tile's barrier (no per-tile DMA ring, no wave reading another wave's DMA)
  const unsigned char* pad = p.pad ? p.pad + b * p.ldpad : nullptr;
  unsigned long long* pbits = (unsigned long long*)(smem + NS * 2 * I::BYTES);
  if (pad) {
    for (int k0 = 64 * w; k0 < p.Lk; k0 += 256) {
      const int key = k0 + lane;
      const unsigned long long bal = __builtin_amdgcn_ballot_w64(key < p.Lk && pad[key] != 0);
      if (lane == 0) pbits[k0 >> 6] = bal;
    }
  }

  const int kv_end = p.causal ? min(p.Lk, q0 + 128) : p.Lk;
  const int ntiles = (kv_end + 63) / 64;
  const int kt1 = max(1, band_lo(q0, p.window) / 64);   // tile 0, then the band from kt1 (dense: all tiles)
  const int nvisit = 1 + max(0, ntiles - kt1);
  const int lo_w = band_lo(qw, p.window);
  const u32x4 krs = buffer_rsrc(K, 0x7FFFFFF0u), vrs = buffer_rsrc(V, 0x7FFFFFF0u);
  auto issue = [&](int it2) {
    const int kn = (it2 == 0 ? 0 : kt1 + it2 - 1) * 64;
    char* kb = smem + (it2 % NS) * 2 * I::BYTES;
    const int ln = lane_id_fresh();   // (offsets recomputed at the issue, never kept live across the key loop)
    if constexpr (PW == 2) {   // K's two pieces in one statement, V's in another
      int ko[2], vo[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        int r, c;
        I::piece_src(w * PW + i, ln, r, c);
        const bool ok = kn + r < p.Lk && c * 8 < p.hd;
        ko[i] = ok ? ((kn + r) * (int)p.sk + c * 8) * 2 : 0x7FFFFFF0;
        vo[i] = ok ? ((kn + r) * (int)p.sv + c * 8) * 2 : 0x7FFFFFF0;
      }
      dma16x2_lds(krs, kb + w * PW * 1024, ko[0], ko[1]);
      dma16x2_lds(vrs, kb + I::BYTES + w * PW * 1024, vo[0], vo[1]);
    } else {
#pragma unroll
      for (int i = 0; i < PW; ++i) {
        int r, c;
        I::piece_src(w * PW + i, ln, r, c);
        const bool ok = kn + r < p.Lk && c * 8 < p.hd;
        dma16_lds(krs, kb + (w * PW + i) * 1024, ok ? ((kn + r) * (int)p.sk + c * 8) * 2 : 0x7FFFFFF0);
        dma16_lds(vrs, kb + I::BYTES + (w * PW + i) * 1024, ok ? ((kn + r) * (int)p.sv + c * 8) * 2 : 0x7FFFFFF0);
      }
    }
  };
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nvisit) issue(t);
  // consume the Q fragments after the first DMA is in flight (the compiler's wait for them is a vmcnt(0): here it costs
  // nothing, inside the loop it would drain the ring)
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(__builtin_bit_cast(u32x4, qf[ks])));

  // per-lane LDS offsets (stage 0, key subtile 0). K (A operand of S^T, ds_read_b128): row r32, chunk 2 ks + hh.
  int koff[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) koff[ks] = I::off(r32, 2 * ks + hh);
  // V (A operand of O^T, ds_read_b64_tr_b16): lane 16 G + 4 q + p reads row 16 s + 8 j2 + 4 (G >> 1) + q, dims
  // 32 dt + 16 (G & 1) + 4 p; dims < 64 need one offset per (dt, j2), the 96-dim tail one per (s, j2)
  const int G = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  int voff[2][2], vtail[2][2];
#pragma unroll
  for (int j2 = 0; j2 < 2; ++j2) {
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      const int row = 8 * j2 + 4 * (G >> 1) + qq;
      voff[dt][j2] = I::off(row, 4 * dt + 2 * (G & 1) + (pp >> 1)) + 8 * (pp & 1);
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int row = 16 * s2 + 8 * j2 + 4 * (G >> 1) + qq;
      vtail[s2][j2] = HDC == 96 ? I::off(row, 8 + 2 * (G & 1) + (pp >> 1)) + 8 * (pp & 1) : 0;
    }
  }

  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[dt][i] = 0.f;
  const float c = p.scale * LOG2E;
  float m = -1e30f, mc = m * c, ls = 0.f;   // reference point of this lane's query (raw score units), row sum
  bool started = false;                      // wave-uniform: the first live tile sets m to the true max

  auto tile = [&](auto STC, int kbase, bool edge, bool diag_only, unsigned long long pm) {
    constexpr int ST = decltype(STC)::value;
    const lds_char* Ks = lds_ptr(smem) + ST * 2 * I::BYTES;
    const lds_char* Vs = Ks + I::BYTES;
    // the limits of this lane's keys kl = 32 kt2 + (i & 3) + 8 (i >> 2) + 4 hh: visible iff kl < lim
    const int lim = (p.causal ? min(p.Lk, qrow + 1) : p.Lk) - kbase - 4 * hh;
    const int hlo = SBLK - kbase - 4 * hh, hhi = lo_w - kbase - 4 * hh;
    const unsigned long long pml = pm >> (4 * hh);
    auto compute_s = [&](f32x16 (&s)[2]) {
#pragma unroll
      for (int kt2 = 0; kt2 < 2; ++kt2) {
#pragma unroll
        for (int i = 0; i < 16; ++i) s[kt2][i] = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
#if SVAE_FWD32_DIAG == 3
          if (ks) break;   // diagnostic build: one S MFMA per subtile
#endif
          s[kt2] = mfma32(lds_read_b128(Ks + koff[ks] + kt2 * 32 * (2 * ks < 8 ? 128 : 64)), qf[ks], s[kt2]);
        }
      }
      // (wave-uniform branches outside the unrolled element loops: inside them the compiler kept a branch per score)
      if (edge && diag_only) {
#pragma unroll
        for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int kc = 32 * kt2 + (i & 3) + 8 * (i >> 2);   // kl - 4 hh
            s[kt2][i] = kc < lim ? s[kt2][i] : -INFINITY;
          }
      } else if (edge) {
        const unsigned plo = (unsigned)pml, phi = (unsigned)(pml >> 32);
#pragma unroll
        for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int kc = 32 * kt2 + (i & 3) + 8 * (i >> 2);
            const unsigned pb = kc < 32 ? (plo >> kc) & 1u : (phi >> (kc - 32)) & 1u;
            const unsigned hid = pb | ((unsigned)(kc >= hlo) & (unsigned)(kc < hhi)) | (unsigned)(kc >= lim);
            s[kt2][i] = hid ? -INFINITY : s[kt2][i];
          }
      }
    };
    auto row_max = [&](const f32x16 (&s)[2]) {
      float mx = -INFINITY;
#pragma unroll
      for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
        for (int i = 0; i < 16; i += 2) mx = fmaxf(fmaxf(mx, s[kt2][i]), s[kt2][i + 1]);
      return max_x32(mx);
    };
    auto exps = [&](f32x16 (&s)[2]) {
      float l0 = 0.f, l1 = 0.f;
#pragma unroll
      for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
#if SVAE_FWD32_DIAG == 2
          const float e0 = s[kt2][i] * 1e-3f, e1 = s[kt2][i + 1] * 1e-3f;   // diagnostic build: no exp2 / fma
#else
          const float e0 = __builtin_amdgcn_exp2f(fmaf(s[kt2][i], c, -mc));
          const float e1 = __builtin_amdgcn_exp2f(fmaf(s[kt2][i + 1], c, -mc));
#endif
          s[kt2][i] = e0;
          s[kt2][i + 1] = e1;
          l0 += e0;
          l1 += e1;
        }
      return l0 + l1;
    };
#if SVAE_FWD32_DIAG == 1
    return;   // diagnostic build: DMA, barriers, prologue and epilogue only
#endif
    f32x16 s[2];
    compute_s(s);
    if (!started) {
      m = fmaxf(m, row_max(s));
      mc = m * c;
      started = true;
    }
    float lt = exps(s);
    if (__builtin_amdgcn_ballot_w64(!(lt <= FWD32_THRESH)) != 0) {
      // the max grew by more than 16 (log2 units) on some row: recompute S, move the reference to the true max (the
      // clobber makes the compiler re-read the K fragments here instead of keeping 32 VGPRs of them live across the
      // exponentials of the common path)
      asm volatile("" ::: "memory");
      compute_s(s);
      const float mn = fmaxf(m, row_max(s));
      const float alpha = __builtin_amdgcn_exp2f((m - mn) * c);
      m = mn;
      mc = m * c;
      ls *= alpha;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
      lt = exps(s);
    }
    ls += lt;
    // O^T += V^T . P^T over the 4 k-steps of 16 keys (key order of k-step (kt2, s2): 32 kt2 + 16 s2 + 8 (j >> 2) +
    // 4 hh + (j & 3), matched by the two transposed V reads j2 = 0, 1)
#pragma unroll
    for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pf = pack_acc8(s[kt2], s2);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const lds_char *a0, *a1;
          if (dt < 2) {
            const int ro = (32 * kt2 + 16 * s2) * 128;
            a0 = Vs + voff[dt][0] + ro;
            a1 = Vs + voff[dt][1] + ro;
          } else {
            a0 = Vs + vtail[s2][0] + 32 * kt2 * 64;
            a1 = Vs + vtail[s2][1] + 32 * kt2 * 64;
          }
#if SVAE_FWD32_DIAG == 4
          if (dt) continue;   // diagnostic build: one PV MFMA per k-step
#endif
          o[dt] = mfma32(cat44(lds_read_tr3(a0), lds_read_tr3(a1)), pf, o[dt]);
        }
      }
  };

  for (int it = 0; it < nvisit; ++it) {
    const int kt = it == 0 ? 0 : kt1 + it - 1;
    wait_vmcnt(min(NS - 2, nvisit - 1 - it) * 2 * PW);   // this wave's pieces of tile it have landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                        // everyone's have; stage (it - 1) % NS is free
    if (it + NS - 1 < nvisit) issue(it + NS - 1);
    const int kbase = kt * 64;
    if ((!p.causal || kbase <= qw + 31) && (kbase < SBLK || kbase + 63 >= lo_w)) {
      const unsigned long long pm = pad ? pbits[kt] : 0ull;
      const bool band_edge = kbase + 63 >= SBLK && kbase < lo_w;
      const bool edge = pm != 0ull || kbase + 64 > p.Lk || (p.causal && kbase + 63 > qw) || band_edge;
      const bool diag_only = pm == 0ull && !band_edge;
      const int st = it % NS;
      if (st == 0) tile(std::integral_constant<int, 0>(), kbase, edge, diag_only, pm);
      else if (NS == 2 || st == 1) tile(std::integral_constant<int, 1>(), kbase, edge, diag_only, pm);
      else tile(std::integral_constant<int, NS == 3 ? 2 : 1>(), kbase, edge, diag_only, pm);
    }
  }

  // epilogue: O = O^T / l (lane: query qrow, dims 32 dt + 8 j + 4 hh + (0..3)), lse = m scale + ln l
  const float lsum = sum_x32(ls);
  const float inv = lsum > 0.f ? 1.0f / lsum : 0.f;
  const bool qok = qrow < p.Lq;
  const __amdgpu_buffer_rsrc_t ors =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.o + b * p.bo + (long long)h * p.hd), 0, 0x7FFFFFF0, 0x00020000);
  const __amdgpu_buffer_rsrc_t olrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.olo ? p.olo + b * p.bolo + (long long)h * p.hd : p.o), 0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    const f32x16 v = o[dt] * inv;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      // lanes hh = 0 / 1 hold dims +0..3 / +4..7 (j = 2a) and +8..11 / +12..15 (j = 2a + 1): one swap per dword gives
      // each lane 8 consecutive dims, 32 dt + 16 a + 8 hh
      const unsigned x0 = pack_bf16x2(v[8 * a], v[8 * a + 1]), x1 = pack_bf16x2(v[8 * a + 2], v[8 * a + 3]);
      const unsigned y0 = pack_bf16x2(v[8 * a + 4], v[8 * a + 5]), y1 = pack_bf16x2(v[8 * a + 6], v[8 * a + 7]);
      const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
      const int d = 32 * dt + 16 * a + 8 * hh;
      const int off = qok && d < p.hd ? (qrow * (int)p.so + d) * 2 : 0x7FFFFFF0;
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){s0[0], s1[0], s0[1], s1[1]}, ors, off, 0, 0);
      if (p.olo) {   // the bf16 residual, same layout
        float r[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) r[e] = v[8 * a + e] - (float)f2bf(v[8 * a + e]);
        const auto t0 = __builtin_amdgcn_permlane32_swap(pack_bf16x2(r[0], r[1]), pack_bf16x2(r[4], r[5]), false, false);
        const auto t1 = __builtin_amdgcn_permlane32_swap(pack_bf16x2(r[2], r[3]), pack_bf16x2(r[6], r[7]), false, false);
        const int offl = qok && d < p.hd ? (qrow * (int)p.solo + d) * 2 : 0x7FFFFFF0;
        __builtin_amdgcn_raw_buffer_store_b128((u32x4){t0[0], t1[0], t0[1], t1[1]}, olrs, offl, 0, 0);
      }
    }
    if (p.o32) {
      float* O32 = p.o32 + b * p.bo32 + (long long)h * p.hd;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int d = 32 * dt + 8 * j + 4 * hh;
        if (qok && d < p.hd)
          __builtin_nontemporal_store((f32x4){v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]},
                                      (f32x4*)(O32 + (long long)qrow * p.so32 + d));
      }
    }
  }
  if (hh == 0 && qok) p.lse[((long long)b * p.H + h) * p.Lq + qrow] = m * p.scale + __logf(lsum);
}

// ===================================================================================== backward
// delta[b][h][q] = sum_d dO . O   (LPR = hd / 8 lanes per (q, h) row: 8 for hd <= 64, 16 for hd <= 128, so no
// lane idles)
template <int LPR>
__global__ __launch_bounds__(256) void attn_delta_kernel(AP p) {
  const int gid = blockIdx.x * (256 / LPR) + (threadIdx.x / LPR);
  const int li = threadIdx.x % LPR;
  const int total = p.B * p.Lq * p.H;
  if (gid >= total) return;
  const int h = gid % p.H, q = (gid / p.H) % p.Lq, b = gid / (p.H * p.Lq);
  const bf16* dO = p.dout + b * p.bdo + (long long)q * p.sdo + (long long)h * p.hd;
  float s = 0.f;
  if (p.olo) {
    const bf16* O = p.o + b * p.bo + (long long)q * p.so + (long long)h * p.hd;
    const bf16* OL = p.olo + b * p.bolo + (long long)q * p.solo + (long long)h * p.hd;
    for (int d = li * 8; d < p.hd; d += 8 * LPR) {
      const bf16x8 a = *(const bf16x8*)(O + d), l = *(const bf16x8*)(OL + d), c = *(const bf16x8*)(dO + d);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += ((float)a[e] + (float)l[e]) * (float)c[e];
    }
  } else if (p.o32) {
    const float* O = p.o32 + b * p.bo32 + (long long)q * p.so32 + (long long)h * p.hd;
    for (int d = li * 8; d < p.hd; d += 8 * LPR) {
      const bf16x8 c = *(const bf16x8*)(dO + d);
      const f32x4 a0 = *(const f32x4*)(O + d), a1 = *(const f32x4*)(O + d + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) s += a0[e] * (float)c[e] + a1[e] * (float)c[e + 4];
    }
  } else {
    const bf16* O = p.o + b * p.bo + (long long)q * p.so + (long long)h * p.hd;
    for (int d = li * 8; d < p.hd; d += 8 * LPR) {
      const bf16x8 a = *(const bf16x8*)(O + d), c = *(const bf16x8*)(dO + d);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += (float)a[e] * (float)c[e];
    }
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, LPR);
  if (li == 0) ((float*)p.delta)[((long long)b * p.H + h) * p.Lq + q] = s;
}

// Main backward: one block = 128 keys of one (batch, head) = 4 waves x 32 keys (two 16-key MFMA column
// tiles), sweeping 64-query tiles (causal: from the tile holding the block's first key). Key on the lane:
// S = Q K^T and dP = dO V^T accumulators are the B operands of dV^T += dO^T P and dK^T += Q^T dS; every
// dO^T / Q^T fragment read feeds both key tiles. Row constants start the accumulators: S' = S - lse/scale,
// dP' = dP - delta, so p = exp2(c S') and dS = p dP' with no per-element subtraction.
// dQ: dS^T goes through LDS once, the block's 64 x hd partial dQ (over its 128 keys) is STORED to its own
// slice of dq_part (no atomics); attn_dq_reduce_kernel sums the slices.
constexpr int BWD_KEYS = 128;

template <int HDP>
__device__ __forceinline__ void attn_bwd_tile(const AP& p, char* smem, int kb, int h, int b) {
  using T = Tile<HDP>;          // [rows][HDP] bf16
  using TS = Tile<64>;          // dS^T [128 keys][64 queries]
  constexpr int NKK = HDP / 32, NT = HDP / 16;
  char* QO = smem;                                  // [buf][Q, dO] tiles
  char* Ks = smem + 4 * T::BYTES;                   // 128 key rows
  char* dSs = smem + 6 * T::BYTES;                  // 128 key rows x 64 queries
  float* cst = (float*)(smem + 6 * T::BYTES + 2 * TS::BYTES);   // [buf][wave][lse, delta][64] (DMA'd with the tile)
  constexpr int NWB = 4;

  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar branches, not exec masks
  const int k0 = kb * BWD_KEYS;
  const bf16* Q = p.q + b * p.bq + (long long)h * p.hd;
  const bf16* K = p.k + b * p.bk + (long long)h * p.hd;
  const bf16* V = p.v + b * p.bv + (long long)h * p.hd;
  const bf16* dO = p.dout + b * p.bdo + (long long)h * p.hd;
  const float* lse = p.lse + ((long long)b * p.H + h) * p.Lq;
  const float* delta = p.delta + ((long long)b * p.H + h) * p.Lq;
  const int kw = k0 + 32 * w;                       // this wave's first key
  // V fragments of this wave's 32 keys stay in registers (B operands of dP = dO V^T); K fragments are read
  // from the block's K tile in LDS each query tile (it is there anyway for dQ = dS K).
  bool key_ok[2];
  bf16x8 vf[2][NKK];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = kw + 16 * j + li;
    key_ok[j] = key < p.Lk && !(p.pad && p.pad[b * p.ldpad + key]);
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      const int d = 32 * kk + 8 * g;
      u32x4 c = {0u, 0u, 0u, 0u};
      if (key < p.Lk && d < p.hd) c = *(const u32x4*)(V + (long long)key * p.sv + d);
      vf[j][kk] = __builtin_bit_cast(bf16x8, c);
    }
  }
  const bool keys_all_ok = __builtin_amdgcn_ballot_w64(!(key_ok[0] && key_ok[1])) == 0;
  {  // K tile (128 rows) for dQ = dS . K
    dma_rows<HDP>(K, p.sk, k0, p.Lk, p.hd, Ks, w, lane);
    dma_rows<HDP>(K, p.sk, k0 + 64, p.Lk, p.hd, Ks + T::BYTES, w, lane);
  }
  f32x4 dk[2][NT], dv[2][NT];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < NT; ++t) { dk[j][t] = (f32x4){0.f, 0.f, 0.f, 0.f}; dv[j][t] = dk[j][t]; }

  const float inv_scale = 1.0f / p.scale, c = p.scale * LOG2E;
  const int qt0 = p.causal ? k0 / 64 : 0;
  // sliding window: queries past the last in-band query of the block's last key block see none of its keys
  // (block 0 holds the [CLS] keys, which every later query sees)
  const int q_end = (p.window > 0 && k0 > 0) ? min(p.Lq, k0 + BWD_KEYS - SBLK + SBLK * p.window) : p.Lq;
  const int nqt = (q_end + 63) / 64;
  const int band_end = p.window > 0 && kw >= SBLK ? kw + SBLK * p.window : 0x7FFFFFFF;   // first query past kw's band
  float* part = p.dq_part + ((long long)kb * p.B + b) * p.Lq * p.H * p.hd + (long long)h * p.hd;
  const long long ldp = (long long)p.H * p.hd;
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc((void*)part, 0, 0x7FFFFFF0, 0x00020000);
  // Every wave issues exactly DQ_STORES dQ-partial stores (16 B per lane) per query tile after the next tile's DMA,
  // so the end-of-tile wait can leave exactly those in flight (vmcnt retires in issue order).
  constexpr int DQ_STORES = NT;

  // the row constants (lse, delta) of a query tile ride along with its Q / dO DMA into cst[buf][wave][lse | delta]
  const u32x4 lser = buffer_rsrc(lse, (unsigned)p.Lq * 4u), der = buffer_rsrc(delta, (unsigned)p.Lq * 4u);
  auto fetch = [&](int qb, int buf) {
    dma_rows<HDP>(Q, p.sq, qb, p.Lq, p.hd, QO + buf * 2 * T::BYTES, w, lane);
    dma_rows<HDP>(dO, p.sdo, qb, p.Lq, p.hd, QO + buf * 2 * T::BYTES + T::BYTES, w, lane);
    const int qo = qb + lane < p.Lq ? (qb + lane) * 4 : 0x7FFFFFF0;
    // every wave DMAs the tile's lse and delta rows into its OWN slot; it reads them only after its own
    // end-of-tile vmcnt (+ the block barrier), so no wave depends on another wave's DMA count
    dma4_lds(lser, cst + (buf * NWB + w) * 128, qo);
    dma4_lds(der, cst + (buf * NWB + w) * 128 + 64, qo);
  };
  if (qt0 < nqt) fetch(qt0 * 64, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int qt = qt0; qt < nqt; ++qt) {
    const int buf = (qt - qt0) & 1;
    const int qb = qt * 64;
    const char* Qs = QO + buf * 2 * T::BYTES;
    const char* dOs = Qs + T::BYTES;
    const float* nl = cst + (buf * NWB + w) * 128;
    const bool more = qt + 1 < nqt;
    if (more) fetch(qb + 64, buf ^ 1);
    const bool live = (!p.causal || kw <= qb + 63) && qb < band_end;   // some key of this wave visible to some query
    if (live) {
      bf16x8 kf[2][NKK];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) kf[j][kk] = *(const bf16x8*)(Ks + T::off(32 * w + 16 * j + li, g + 4 * kk));
      // Masks only on edge tiles (wave-uniform): a masked score's accumulator starts at -inf, so the MFMA sum stays
      // -inf and exp2 gives exactly 0; the tests are branch-free compares + one select per score (short-circuit ||
      // compiled to an exec-mask branch per score, ~5 scalar instructions each).
      const bool edge = !keys_all_ok || qb + 64 > p.Lq || (p.causal && kw + 31 > qb) || qb + 63 >= band_end;
      const int qlim = min(p.Lq, band_end) - qb;   // queries ql >= qlim see nothing (ragged end, window)
      // Two passes of TPP = 2 16-query row tiles: S and dP of a pass, its softmax, its dV / dK MFMAs (one k-step of
      // 32 queries) and its dS^T stores, then the next pass (half the S / dP accumulators live at a time: 256 VGPRs
      // without spills at 2 blocks / CU).
      constexpr int TPP = 2;
#pragma unroll
      for (int pass = 0; pass < 4 / TPP; ++pass) {
        f32x4 s[2][TPP], dp[2][TPP];
#pragma unroll
        for (int th = 0; th < TPP; ++th) {
          const int t = pass * TPP + th;
          const f32x4 sl = *(const f32x4*)(nl + 16 * t + 4 * g) * -inv_scale;   // -lse / scale
          const f32x4 dl = -*(const f32x4*)(nl + 64 + 16 * t + 4 * g);          // -delta
          s[0][th] = sl; s[1][th] = sl;
          dp[0][th] = dl; dp[1][th] = dl;
          if (edge) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const int kmin = p.causal ? kw + 16 * j + li - qb : -0x40000000;   // causal: query ql >= kmin sees it
              const unsigned kbad = key_ok[j] ? 0u : 1u;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int ql = 16 * t + 4 * g + r;
                s[j][th][r] = (kbad | (unsigned)(ql >= qlim) | (unsigned)(ql < kmin)) ? -INFINITY : s[j][th][r];
              }
            }
          }
#pragma unroll
          for (int k2 = 0; k2 < NKK; ++k2) {
            const bf16x8 qa = *(const bf16x8*)(Qs + T::off(16 * t + li, g + 4 * k2));
            const bf16x8 oa = *(const bf16x8*)(dOs + T::off(16 * t + li, g + 4 * k2));
            s[0][th] = mfma16(qa, kf[0][k2], s[0][th]);
            s[1][th] = mfma16(qa, kf[1][k2], s[1][th]);
            dp[0][th] = mfma16(oa, vf[0][k2], dp[0][th]);
            dp[1][th] = mfma16(oa, vf[1][k2], dp[1][th]);
          }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int th = 0; th < TPP; ++th)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float pr = __builtin_amdgcn_exp2f(s[j][th][r] * c);
              s[j][th][r] = pr;
              dp[j][th][r] = pr * dp[j][th][r];
            }
        // dV^T += dO^T P ; dK^T += Q^T dS   (query order of k-step kk: 32kk + 16(jj>>2) + 4g + (jj&3))
#pragma unroll
        for (int k2 = 0; k2 < TPP / 2; ++k2) {
          const int kk = pass * (TPP / 2) + k2;
          const bf16x8 pf0 = pack8(s[0][2 * k2], s[0][2 * k2 + 1]), pf1 = pack8(s[1][2 * k2], s[1][2 * k2 + 1]);
          const bf16x8 df0 = pack8(dp[0][2 * k2], dp[0][2 * k2 + 1]), df1 = pack8(dp[1][2 * k2], dp[1][2 * k2 + 1]);
          const int r0 = 32 * kk + 4 * g + (li >> 2);
#pragma unroll
          for (int u = 0; u < NT; ++u) {
            const int uu = 4 * u + (li & 3);
            const bf16x8 ao = cat44(lds_read_tr(dOs + T::uoff(r0, uu)), lds_read_tr(dOs + T::uoff(r0 + 16, uu)));
            dv[0][u] = mfma16(ao, pf0, dv[0][u]);
            dv[1][u] = mfma16(ao, pf1, dv[1][u]);
            const bf16x8 aq = cat44(lds_read_tr(Qs + T::uoff(r0, uu)), lds_read_tr(Qs + T::uoff(r0 + 16, uu)));
            dk[0][u] = mfma16(aq, df0, dk[0][u]);
            dk[1][u] = mfma16(aq, df1, dk[1][u]);
          }
        }
        // dS^T -> LDS [key][q]: lane holds q = 16t + 4g + (0..3) at key row 32w + 16j + li
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int th = 0; th < TPP; ++th)
            *(bf16x4*)(dSs + TS::uoff(32 * w + 16 * j + li, 4 * (pass * TPP + th) + g)) =
                (bf16x4){f2bf(dp[j][th][0]), f2bf(dp[j][th][1]), f2bf(dp[j][th][2]), f2bf(dp[j][th][3])};
      }
    } else {
      const bf16x4 z = {f2bf(0.f), f2bf(0.f), f2bf(0.f), f2bf(0.f)};
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) *(bf16x4*)(dSs + TS::uoff(32 * w + 16 * j + li, 4 * t + g)) = z;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // dS^T complete (a raw barrier: __syncthreads' vmcnt(0) would drain the DMA)
    // partial dQ[q = qb + 16w + li][d = 16u + 4g + r] = sum over the block's 128 keys of dS[q][key] K[key][d]
    // (K fragment as the MFMA's first operand: a lane holds 4 consecutive dims of one query, one 16-B store each)
    f32x4 dq[NT];
#pragma unroll
    for (int u = 0; u < NT; ++u) dq[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int kvis = p.causal ? min(BWD_KEYS, qb + 64 - k0) : BWD_KEYS;   // keys past the tile's last query: dS = 0
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (32 * kk >= kvis) break;
      const int kr = 32 * kk + 8 * g + (li >> 2);
      const int uq = 4 * w + (li & 3);
      const bf16x8 a = cat44(lds_read_tr(dSs + TS::uoff(kr, uq)), lds_read_tr(dSs + TS::uoff(kr + 4, uq)));
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const int uk = 4 * u + (li & 3);
        const bf16x8 bk = cat44(lds_read_tr(Ks + T::uoff(kr, uk)), lds_read_tr(Ks + T::uoff(kr + 4, uk)));
        dq[u] = mfma16(bk, a, dq[u]);
      }
    }
    // buffer stores, always DQ_STORES per wave: rows past Lq / dims past hd get an out-of-range offset and are dropped
    // by the range check (no branches, and a fixed count for the wait below)
    {
      const bool qok = qb + 16 * w + li < p.Lq;
      const int qrow = (qb + 16 * w + li) * (int)ldp + 4 * g;
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const int off = (qok && 16 * u + 4 * g < p.hd) ? (qrow + 16 * u) * 4 : 0x7FFFFFF0;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, dq[u]), prs, off, 0, 0);
      }
    }
    // the next tile's DMA (issued before this tile's stores) has landed; the stores stay in flight
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DQ_STORES) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  // epilogue: dK (scaled, inverse rotary) and dV for key = kw + 16j + li, dims 16u + 4g + (0..3)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = kw + 16 * j + li;
    if (key >= p.Lk) continue;
    bf16* DK = p.dk + b * p.bdk + (long long)key * p.sdk + (long long)h * p.hd;
    bf16* DV = p.dv + b * p.bdv + (long long)key * p.sdv + (long long)h * p.hd;
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      const int d = 16 * u + 4 * g;
      if (d >= p.hd) continue;
      float x[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) x[r] = dk[j][u][r] * p.scale;
      if (p.rot) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int pair = (h * p.hd + d) / 2 + e;
          const float2 cs = ((const float2*)p.rot)[(long long)key * (p.rot_d / 2) + pair];
          const float a = x[2 * e], cc = x[2 * e + 1];
          x[2 * e] = a * cs.x + cc * cs.y;
          x[2 * e + 1] = -a * cs.y + cc * cs.x;
        }
      }
      *(bf16x4*)(DK + d) = (bf16x4){f2bf(x[0]), f2bf(x[1]), f2bf(x[2]), f2bf(x[3])};
      *(bf16x4*)(DV + d) = (bf16x4){f2bf(dv[j][u][0]), f2bf(dv[j][u][1]), f2bf(dv[j][u][2]), f2bf(dv[j][u][3])};
    }
  }
}

// hd 128 (hd 96 padded): the same algorithm in one pass of 64 queries with the original mask / store code, one wave
// per SIMD (512 registers); the restructured attn_bwd_tile spills there (46 spills against 7).
template <int HDP, int HDC = HDP>
__device__ __forceinline__ void attn_bwd_tile_wide(const AP& p, char* smem, int kb, int h, int b) {
  using T = Tile<HDP>;          // [rows][HDP] bf16
  using TS = Tile<64>;          // dS^T [128 keys][64 queries]
  constexpr int NKK = HDC / 32, NT = HDC / 16;   // the MFMAs cover HDC <= HDP dims (hd 96: HDC = 96)
  char* QO = smem;                                  // [buf][Q, dO] tiles
  char* Ks = smem + 4 * T::BYTES;                   // 128 key rows
  char* dSs = smem + 6 * T::BYTES;                  // 128 key rows x 64 queries
  float* cst = (float*)(smem + 6 * T::BYTES + 2 * TS::BYTES);   // [buf][wave][lse, delta][64] (DMA'd with the tile)
  constexpr int NWB = 4;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  const int k0 = kb * BWD_KEYS;
  const bf16* Q = p.q + b * p.bq + (long long)h * p.hd;
  const bf16* K = p.k + b * p.bk + (long long)h * p.hd;
  const bf16* V = p.v + b * p.bv + (long long)h * p.hd;
  const bf16* dO = p.dout + b * p.bdo + (long long)h * p.hd;
  const float* lse = p.lse + ((long long)b * p.H + h) * p.Lq;
  const float* delta = p.delta + ((long long)b * p.H + h) * p.Lq;
  const int kw = k0 + 32 * w;                       // this wave's first key
  // V fragments of this wave's 32 keys stay in registers (B operands of dP = dO V^T); K fragments are read
  // from the block's K tile in LDS each query tile (it is there anyway for dQ = dS K).
  bool key_ok[2];
  bf16x8 vf[2][NKK];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = kw + 16 * j + li;
    key_ok[j] = key < p.Lk && !(p.pad && p.pad[b * p.ldpad + key]);
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      const int d = 32 * kk + 8 * g;
      u32x4 c = {0u, 0u, 0u, 0u};
      if (key < p.Lk && d < p.hd) c = *(const u32x4*)(V + (long long)key * p.sv + d);
      vf[j][kk] = __builtin_bit_cast(bf16x8, c);
    }
  }
  const bool keys_all_ok = __builtin_amdgcn_ballot_w64(!(key_ok[0] && key_ok[1])) == 0;
  {  // K tile (128 rows) for dQ = dS . K
    dma_rows<HDP>(K, p.sk, k0, p.Lk, p.hd, Ks, w, lane);
    dma_rows<HDP>(K, p.sk, k0 + 64, p.Lk, p.hd, Ks + T::BYTES, w, lane);
  }
  f32x4 dk[2][NT], dv[2][NT];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < NT; ++t) { dk[j][t] = (f32x4){0.f, 0.f, 0.f, 0.f}; dv[j][t] = dk[j][t]; }

  const float inv_scale = 1.0f / p.scale, c = p.scale * LOG2E;
  const int qt0 = p.causal ? k0 / 64 : 0;
  // sliding window: queries past the last in-band query of the block's last key block see none of its keys
  // (block 0 holds the [CLS] keys, which every later query sees)
  const int q_end = (p.window > 0 && k0 > 0) ? min(p.Lq, k0 + BWD_KEYS - SBLK + SBLK * p.window) : p.Lq;
  const int nqt = (q_end + 63) / 64;
  const int band_end = p.window > 0 && kw >= SBLK ? kw + SBLK * p.window : 0x7FFFFFFF;   // first query past kw's band
  float* part = p.dq_part + ((long long)kb * p.B + b) * p.Lq * p.H * p.hd + (long long)h * p.hd;
  const long long ldp = (long long)p.H * p.hd;
  // On a full query tile (all 64 queries < Lq, hd == HDC) every wave issues exactly DQ_STORES dQ-partial stores
  // after the next tile's DMA, so the end-of-tile wait can leave exactly those in flight (vmcnt retires in
  // issue order); edge tiles wait for everything.
  constexpr int DQ_STORES = NT;

  // the row constants (lse, delta) of a query tile ride along with its Q / dO DMA into cst[buf][wave][lse | delta]
  const u32x4 lser = buffer_rsrc(lse, (unsigned)p.Lq * 4u), der = buffer_rsrc(delta, (unsigned)p.Lq * 4u);
  auto fetch = [&](int qb, int buf) {
    dma_rows<HDP>(Q, p.sq, qb, p.Lq, p.hd, QO + buf * 2 * T::BYTES, w, lane);
    dma_rows<HDP>(dO, p.sdo, qb, p.Lq, p.hd, QO + buf * 2 * T::BYTES + T::BYTES, w, lane);
    const int qo = qb + lane < p.Lq ? (qb + lane) * 4 : 0x7FFFFFF0;
    // every wave DMAs the tile's lse and delta rows into its OWN slot; it reads them only after its own
    // end-of-tile vmcnt (+ the block barrier), so no wave depends on another wave's DMA count
    dma4_lds(lser, cst + (buf * NWB + w) * 128, qo);
    dma4_lds(der, cst + (buf * NWB + w) * 128 + 64, qo);
  };
  if (qt0 < nqt) fetch(qt0 * 64, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int qt = qt0; qt < nqt; ++qt) {
    const int buf = (qt - qt0) & 1;
    const int qb = qt * 64;
    const char* Qs = QO + buf * 2 * T::BYTES;
    const char* dOs = Qs + T::BYTES;
    const float* nl = cst + (buf * NWB + w) * 128;
    const bool more = qt + 1 < nqt;
    if (more) fetch(qb + 64, buf ^ 1);
    const bool live = (!p.causal || kw <= qb + 63) && qb < band_end;   // some key of this wave visible to some query
    if (live) {
      f32x4 s[2][4], dp[2][4];
      bf16x8 kf[2][NKK];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) kf[j][kk] = *(const bf16x8*)(Ks + T::off(32 * w + 16 * j + li, g + 4 * kk));
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const f32x4 sl = *(const f32x4*)(nl + 16 * t + 4 * g) * -inv_scale;   // -lse / scale
        const f32x4 dl = -*(const f32x4*)(nl + 64 + 16 * t + 4 * g);          // -delta
        s[0][t] = sl; s[1][t] = sl;
        dp[0][t] = dl; dp[1][t] = dl;
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) {
          const bf16x8 qa = *(const bf16x8*)(Qs + T::off(16 * t + li, g + 4 * kk));
          const bf16x8 oa = *(const bf16x8*)(dOs + T::off(16 * t + li, g + 4 * kk));
          s[0][t] = mfma16(qa, kf[0][kk], s[0][t]);
          s[1][t] = mfma16(qa, kf[1][kk], s[1][t]);
          dp[0][t] = mfma16(oa, vf[0][kk], dp[0][t]);
          dp[1][t] = mfma16(oa, vf[1][kk], dp[1][t]);
        }
      }
      const bool edge = !keys_all_ok || qb + 64 > p.Lq || (p.causal && kw + 31 > qb) || qb + 63 >= band_end;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float pr = __builtin_amdgcn_exp2f(s[j][t][r] * c);
            if (edge) {
              const int q = qb + 16 * t + 4 * g + r, key = kw + 16 * j + li;
              if (!key_ok[j] || q >= p.Lq || (p.causal && key > q) || q >= band_end) pr = 0.f;
            }
            s[j][t][r] = pr;
            dp[j][t][r] = pr * dp[j][t][r];
          }
      // dV^T += dO^T P ; dK^T += Q^T dS   (query order of k-step kk: 32kk + 16(jj>>2) + 4g + (jj&3))
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 pf0 = pack8(s[0][2 * kk], s[0][2 * kk + 1]), pf1 = pack8(s[1][2 * kk], s[1][2 * kk + 1]);
        const bf16x8 df0 = pack8(dp[0][2 * kk], dp[0][2 * kk + 1]), df1 = pack8(dp[1][2 * kk], dp[1][2 * kk + 1]);
        const int r0 = 32 * kk + 4 * g + (li >> 2);
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          const int uu = 4 * u + (li & 3);
          const bf16x8 ao = cat44(lds_read_tr(dOs + T::uoff(r0, uu)), lds_read_tr(dOs + T::uoff(r0 + 16, uu)));
          dv[0][u] = mfma16(ao, pf0, dv[0][u]);
          dv[1][u] = mfma16(ao, pf1, dv[1][u]);
          const bf16x8 aq = cat44(lds_read_tr(Qs + T::uoff(r0, uu)), lds_read_tr(Qs + T::uoff(r0 + 16, uu)));
          dk[0][u] = mfma16(aq, df0, dk[0][u]);
          dk[1][u] = mfma16(aq, df1, dk[1][u]);
        }
      }
      // dS^T -> LDS [key][q]: lane holds q = 16t + 4g + (0..3) at key row 32w + 16j + li
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          *(bf16x4*)(dSs + TS::uoff(32 * w + 16 * j + li, 4 * t + g)) =
              (bf16x4){f2bf(dp[j][t][0]), f2bf(dp[j][t][1]), f2bf(dp[j][t][2]), f2bf(dp[j][t][3])};
    } else {
      const bf16x4 z = {f2bf(0.f), f2bf(0.f), f2bf(0.f), f2bf(0.f)};
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) *(bf16x4*)(dSs + TS::uoff(32 * w + 16 * j + li, 4 * t + g)) = z;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // dS^T complete (a raw barrier: __syncthreads' vmcnt(0) would drain the DMA)
    // partial dQ[q = qb + 16w + li][d = 16u + 4g + r] = sum over the block's 128 keys of dS[q][key] K[key][d]
    f32x4 dq[NT];
#pragma unroll
    for (int u = 0; u < NT; ++u) dq[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int kvis = p.causal ? min(BWD_KEYS, qb + 64 - k0) : BWD_KEYS;   // keys past the tile's last query: dS = 0
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (32 * kk >= kvis) break;
      const int kr = 32 * kk + 8 * g + (li >> 2);
      const int uq = 4 * w + (li & 3);
      const bf16x8 a = cat44(lds_read_tr(dSs + TS::uoff(kr, uq)), lds_read_tr(dSs + TS::uoff(kr + 4, uq)));
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const int uk = 4 * u + (li & 3);
        const bf16x8 bk = cat44(lds_read_tr(Ks + T::uoff(kr, uk)), lds_read_tr(Ks + T::uoff(kr + 4, uk)));
        dq[u] = mfma16(bk, a, dq[u]);
      }
    }
    {
      const int q = qb + 16 * w + li;
      if (q < p.Lq) {
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          const int d = 16 * u + 4 * g;
          if (d < p.hd) *(f32x4*)(part + (long long)q * ldp + d) = dq[u];
        }
      }
    }
    // the next tile's DMA (issued before this tile's stores) has landed; on full tiles the stores stay in flight
    if (qb + 64 <= p.Lq && p.hd == HDC) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DQ_STORES) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  // epilogue: dK (scaled, inverse rotary) and dV for key = kw + 16j + li, dims 16u + 4g + (0..3)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = kw + 16 * j + li;
    if (key >= p.Lk) continue;
    bf16* DK = p.dk + b * p.bdk + (long long)key * p.sdk + (long long)h * p.hd;
    bf16* DV = p.dv + b * p.bdv + (long long)key * p.sdv + (long long)h * p.hd;
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      const int d = 16 * u + 4 * g;
      if (d >= p.hd) continue;
      float x[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) x[r] = dk[j][u][r] * p.scale;
      if (p.rot) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int pair = (h * p.hd + d) / 2 + e;
          const float2 cs = ((const float2*)p.rot)[(long long)key * (p.rot_d / 2) + pair];
          const float a = x[2 * e], cc = x[2 * e + 1];
          x[2 * e] = a * cs.x + cc * cs.y;
          x[2 * e + 1] = -a * cs.y + cc * cs.x;
        }
      }
      *(bf16x4*)(DK + d) = (bf16x4){f2bf(x[0]), f2bf(x[1]), f2bf(x[2]), f2bf(x[3])};
      *(bf16x4*)(DV + d) = (bf16x4){f2bf(dv[j][u][0]), f2bf(dv[j][u][1]), f2bf(dv[j][u][2]), f2bf(dv[j][u][3])};
    }
  }
}

// ===================================================================================== backward, 8 waves
// One workgroup = 256 keys of one (batch, head) = 8 waves x 32 keys, sweeping 64-query tiles: the same key-on-the-lane
// algorithm as attn_bwd_tile, but twice the keys per dQ partial (the partial planes and the reduction's reads halve:
// at C4, hd 96, they were 0.9 GB written and read per launch) and, for hd 96, two waves per SIMD instead of one (the
// 4-wave kernel needed 128-wide LDS rows and 256-register waves). LDS rows of HDC = 64 or 96 dims (RowImg: 96 = a
// 64-dim Tile plus a 32-dim tail image), so hd 96 keeps K, dS^T and double-buffered Q / dO in 129 KiB.
//
constexpr int BWD8_KEYS = 256;
#ifndef SVAE_BWD8_DIAG
#define SVAE_BWD8_DIAG 0   // diagnostic build only (-DSVAE_BWD8_DIAG=1): no S / dP / dV / dK / dQ products (DMA, barriers,
#endif                     // zero dS^T writes and every store kept): the kernel's memory and synchronisation skeleton

#ifdef SVAE_STAMPS
// diagnostic build only: per (hardware block < 1024, wave) cycle sums of the q-tile phases of attn_bwd8 --
// [0] prologue (block start -> loop), [1] S / dP / dV / dK + dS^T writes, [2] wait at the dS^T barrier, [3] dQ MFMAs
// + stores, [4] end-of-tile DMA wait + barrier, [5] epilogue (dK / dV stores, drained), [6] live q-tiles, [7] q-tiles
__device__ unsigned long long svae_bwd8_stamps[1024][8][8];
#define BWD8_T(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#define BWD8_ACC(k, a, b) (st_acc[k] += (b) - (a))
#endif

// The [CLS] keys' f32 dK / dV partials of one wave (keys 16 j + li, dims 16 u + 4 g ..): slab layout [2][B][32][H hd]
// (dK, then dV), unscaled and before the inverse rotary (attn_cls_finalize_kernel applies both to the slabs' sum)
template <int NT>
__device__ __forceinline__ void bwd_cls_store_slab(const AP& p, float* slab, int b, int h, const f32x4 (&dk)[2][NT],
                                                   const f32x4 (&dv)[2][NT]) {
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const long long D = (long long)p.H * p.hd, half = (long long)p.B * 32 * D;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    float* row = slab + ((long long)b * 32 + 16 * j + li) * D + (long long)h * p.hd;
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      const int d = 16 * u + 4 * g;
      if (d >= p.hd) continue;
      *(f32x4*)(row + d) = dk[j][u];
      *(f32x4*)(row + half + d) = dv[j][u];
    }
  }
}

#ifndef SVAE_BWD8_KEYMAP
#define SVAE_BWD8_KEYMAP 1
#endif
template <int HDC, int NSUB, bool RMW>
__device__ __forceinline__ void attn_bwd8_tile(const AP& p, char* smem, int kb, int h, int b, int nsub) {
  using R = RowImg<HDC>;
  using TS = Tile<64>;          // dS^T [256 keys][64 queries]
  constexpr int NKK = HDC / 32, NT = HDC / 16;
  constexpr int NW = 8;
  // LDS: [buf][Q, dO] images | K: 4 images (256 keys) | dS^T | [buf][lse, delta][64]
  char* QO = smem;
  char* Ks = smem + 4 * R::BYTES;
  char* dSs = Ks + 4 * R::BYTES;
  float* cst = (float*)(dSs + 4 * TS::BYTES);   // [buf][wave][lse, delta][64] (DMA'd with the tile)
  constexpr int NWB = 8;
  char* rslots = (char*)(cst + 2 * NWB * 128);    // [wave][DQ_NT KiB]: the first sub-block's dQ partial (see rmw)
  // [wave][DQ_NT KiB]: the direct tiles' rotary cos / sin. hd 96 has no LDS left for a second slot array: there the
  // direct tiles are key block 0's (queries < 256, never rmw) and share the rmw slots (the host's dq_direct limit)
  char* cslots = HDC == 64 && NSUB == 2 ? rslots + NWB * (HDC / 32) * 1024 : rslots;
  // LDS-DMA pieces per wave: one query tile's Q + dO images, and the K tile
  constexpr int QO_PW = 2 * R::PIECES / NW;
  constexpr int K_PW = 4 * R::PIECES / NW;
  static_assert(QO_PW * NW == 2 * R::PIECES && K_PW * NW == 4 * R::PIECES, "pieces split evenly over the waves");

  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int k0 = kb * BWD8_KEYS;
#ifdef SVAE_STAMPS
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  BWD8_T(t_start);
#endif
  const bf16* Q = p.q + b * p.bq + (long long)h * p.hd;
  const bf16* K = p.k + b * p.bk + (long long)h * p.hd;
  const bf16* V = p.v + b * p.bv + (long long)h * p.hd;
  const bf16* dO = p.dout + b * p.bdo + (long long)h * p.hd;
  const float* lse = p.lse + ((long long)b * p.H + h) * p.Lq;
  const float* delta = p.delta + ((long long)b * p.H + h) * p.Lq;
  // this wave's 32 keys: slot wk of the block's 8 (SVAE_BWD8_KEYMAP, default 1: waves w and w + 4 -- the two waves of
  // one SIMD -- take slots w and 7 - w, an early and a late key group, so every SIMD carries the same causal work on
  // the diagonal key blocks (live query tiles 4 + 1, 4 + 1, 3 + 2, 3 + 2 of a 4-tile sweep, instead of 4 + 2, 4 + 2,
  // 3 + 1, 3 + 1 with slot = w); 0: slot = w)
  const int wk = SVAE_BWD8_KEYMAP ? (w < 4 ? w : 11 - w) : w;
  const int kw = k0 + 32 * wk;                      // this wave's first key
  bool key_ok[2];
  bf16x8 vf[2][NKK];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = kw + 16 * j + li;
    key_ok[j] = key < p.Lk && !(p.pad && p.pad[b * p.ldpad + key]);
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      const int d = 32 * kk + 8 * g;
      u32x4 c = {0u, 0u, 0u, 0u};
      if (key < p.Lk && d < p.hd) c = *(const u32x4*)(V + (long long)key * p.sv + d);
      vf[j][kk] = __builtin_bit_cast(bf16x8, c);
    }
  }
  const bool keys_all_ok = __builtin_amdgcn_ballot_w64(!(key_ok[0] && key_ok[1])) == 0;
  {  // K tile: 4 images of 64 keys
    const u32x4 krs = buffer_rsrc(K, 0x7FFFFFF0u);
#pragma unroll
    for (int i = 0; i < K_PW; ++i) {
      const int pc = w * K_PW + i, img = pc / R::PIECES;
      dma_img_piece<HDC>(krs, p.sk, k0 + 64 * img, p.Lk, p.hd, Ks + img * R::BYTES, pc % R::PIECES, lane);
    }
  }
  f32x4 dk[2][NT], dv[2][NT];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < NT; ++t) { dk[j][t] = (f32x4){0.f, 0.f, 0.f, 0.f}; dv[j][t] = dk[j][t]; }

  const float inv_scale = 1.0f / p.scale, c = p.scale * LOG2E;
  const int qt0 = p.causal ? k0 / 64 : 0;
  // (key block 0 in window mode: every query sees its [CLS] keys; with the [CLS] split it stops at cls_q0)
  const int q_end = (p.window > 0 && k0 > 0) ? min(p.Lq, k0 + BWD8_KEYS - SBLK + SBLK * p.window)
                                             : (p.cls_q0 > 0 ? min(p.Lq, p.cls_q0) : p.Lq);
  const int nqt = (q_end + 63) / 64;
  const int band_end = p.window > 0 && kw >= SBLK ? kw + SBLK * p.window : 0x7FFFFFFF;   // first query past kw's band
  // dQ partial plane pk: nsub = 2 consecutive 256-key sub-blocks (kb = 2 pk, 2 pk + 1) share one plane, swept one
  // after the other by the same workgroup; the second adds the first's partial (read back by LDS-DMA into its own
  // per-wave slot, `rmw`) before storing, so the planes -- and attn_dq_reduce's reads of them -- halve
  const int pk = nsub == 2 ? kb >> 1 : kb;
  constexpr bool rmw = RMW;   // (the second sub-block: kb odd, NSUB = nsub = 2)
  // query tiles the first sub-block (keys k0 - 256 ..) stored: every tile from its qt0 (<= this qt0) to its q_end
  const int nqt_prev = !rmw ? 0
                       : (((p.window > 0 && k0 - BWD8_KEYS > 0)
                               ? min(p.Lq, k0 - SBLK + SBLK * p.window) : p.Lq) + 63) >> 6;
  float* part = dq_plane(p, pk, b) + (long long)h * p.hd;
  const long long ldp = (long long)p.H * p.hd;
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc((void*)part, 0, 0x7FFFFFF0, 0x00020000);
  // final dQ of the direct tiles (see the dQ stores): row 0 of this (batch, head) in dq_bf (bf16) or dq (f32)
  void* dbase = p.dq_bf ? (void*)((bf16*)p.dq_bf + (long long)b * p.Lq * p.ldq_bf + (long long)h * p.hd)
                        : (void*)(p.dq + b * p.bdq + (long long)h * p.hd);
  const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(dbase, 0, 0x7FFFFFF0, 0x00020000);
  // dQ partial of a query tile (64 queries x HDC dims): wave w owns queries 16 (w & 3) .. + 15 and dims
  // (w >> 2) HDC / 2 .. + HDC / 2 - 1, i.e. NT / 2 fragments, stored as NT / 2 16-B buffer stores per lane (a fixed
  // count: the end-of-tile wait leaves exactly those in flight)
  constexpr int DQ_NT = NT / 2;
  constexpr int DQ_STORES = DQ_NT;
  const int dq_q16 = w & 3, dq_u0 = (w >> 2) * DQ_NT;

  const u32x4 qrs = buffer_rsrc(Q, 0x7FFFFFF0u), ors = buffer_rsrc(dO, 0x7FFFFFF0u);
  const u32x4 lser = buffer_rsrc(lse, (unsigned)p.Lq * 4u), der = buffer_rsrc(delta, (unsigned)p.Lq * 4u);
  auto fetch = [&](int qb, int buf) {
    char* base = QO + buf * 2 * R::BYTES;
    const int ln = lane_id_fresh();
    // a wave's QO_PW pieces are consecutive pieces of ONE image (Q for waves 0-3, dO for 4-7: 2 R::PIECES split over
    // 8 waves), issued in one statement
    static_assert(R::PIECES % QO_PW == 0 && (QO_PW == 2 || QO_PW == 3), "a wave's pieces within one image");
    const bool isq = w * QO_PW < R::PIECES;   // (wave-uniform)
    const int pc0 = isq ? w * QO_PW : w * QO_PW - R::PIECES;
    char* img = isq ? base : base + R::BYTES;
    const long long ld = isq ? p.sq : p.sdo;
    const u32x4 irs = isq ? qrs : ors;
    int po[3];
#pragma unroll
    for (int i = 0; i < QO_PW; ++i) {
      int r, c;
      R::piece_src(pc0 + i, ln, r, c);
      const bool ok = qb + r < p.Lq && c * 8 < p.hd;
      po[i] = ok ? ((qb + r) * (int)ld + c * 8) * 2 : 0x7FFFFFF0;
    }
    if constexpr (QO_PW == 2) dma16x2_lds(irs, img + pc0 * 1024, po[0], po[1]);
    else dma16x3_lds(irs, img + pc0 * 1024, po[0], po[1], po[2]);
    const int qo = qb + ln < p.Lq ? (qb + ln) * 4 : 0x7FFFFFF0;
    // every wave DMAs the tile's lse and delta rows into its OWN slot; it reads them only after its own
    // end-of-tile vmcnt (+ the block barrier), so no wave depends on another wave's DMA count
    dma4x2_lds(lser, der, cst + (buf * NWB + w) * 128, qo, qo);
  };
  // In-kernel delta (hd 64, p.delta_inkernel): waves 4-7, which DMA the dO image of a tile (rows 16 (w - 4) .. + 15),
  // DMA the same rows of O and of its bf16 residual o_lo into a slot of their own with the tile (4 more LDS-DMA pieces,
  // retired by the same end-of-tile wait) and reduce delta = sum_d dO . (O + o_lo) of their 16 rows into the shared
  // slot dsh[buf] before the end-of-tile barrier that publishes the tile. This replaces the attn_delta_kernel pass
  // (which re-read O, o_lo and dO: 100 MB per launch at C2, 19 us). (Register loads instead -- compiler-visible ones --
  // made hipcc put a vmcnt(0) in front of them on every tile, behind the next tile's DMA.)
  constexpr bool DIK_OK = HDC == 64;
  const bool dik = DIK_OK && p.delta_inkernel != 0;   // (uniform)
  float* dsh = (float*)(rslots + (HDC == 64 && NSUB == 2 ? 2 : 1) * NWB * (HDC / 32) * 1024);   // [2][64]
  char* dslot = (char*)(dsh + 128) + (w - 4) * 4096;   // waves 4-7: [O 16 x 64 | o_lo 16 x 64] bf16, row-major
  const u32x4 ors_o = buffer_rsrc(p.o + b * p.bo + (long long)h * p.hd, 0x7FFFFFF0u);
  const u32x4 ors_l = buffer_rsrc(p.olo ? p.olo + b * p.bolo + (long long)h * p.hd : p.o, 0x7FFFFFF0u);
  auto dik_issue = [&](int qb) {   // piece i, lane l: row 8 i + (l >> 3) of the wave's 16, dims 8 (l & 7) .. + 7
    const int ln = lane_id_fresh();
    int oo[2], ol[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = 16 * (w - 4) + 8 * i + (ln >> 3), dd = 8 * (ln & 7);
      const bool ok = qb + r < p.Lq && dd < p.hd;   // (dims >= hd land as zeros, as in the dO image)
      oo[i] = ok ? ((qb + r) * (int)p.so + dd) * 2 : 0x7FFFFFF0;
      ol[i] = ok ? ((qb + r) * (int)p.solo + dd) * 2 : 0x7FFFFFF0;
    }
    dma16x2_lds(ors_o, dslot, oo[0], oo[1]);
    dma16x2_lds(ors_l, dslot + 2048, ol[0], ol[1]);
  };
  // hd 64: p.scale for the direct tiles' dQ, re-read from LDS at the use. (Kept in a register across the q-tile loop,
  // SGPR pressure -- 231 SGPR spills since the window / [CLS] / in-kernel-delta fields -- put it in scratch, and its
  // reload's vmcnt(0) in the dQ phase waited for the next tile's DMA on every direct tile.)
  float* sscl = nullptr;
  if constexpr (HDC == 64) {
    sscl = (float*)(dslot - (w - 4) * 4096 + 4 * 4096);
    if (tid == 0) *sscl = p.scale;
  }
  auto dik_reduce = [&](int buf, int qb) {   // after this wave's wait for the tile's DMA and its O / o_lo pieces
    const int ln = lane_id_fresh();
    const int rl = ln >> 2, r = 16 * (w - 4) + rl, c0 = 2 * (ln & 3);
    const char* dimg = QO + buf * 2 * R::BYTES + R::BYTES;
    float sacc = 0.f;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const bf16x8 dv8 = *(const bf16x8*)(dimg + R::off(r, c0 + hh));
      const bf16x8 o8 = *(const bf16x8*)(dslot + rl * 128 + (c0 + hh) * 16);
      const bf16x8 l8 = *(const bf16x8*)(dslot + 2048 + rl * 128 + (c0 + hh) * 16);
#pragma unroll
      for (int e = 0; e < 8; ++e) sacc += ((float)o8[e] + (float)l8[e]) * (float)dv8[e];
    }
    sacc += __shfl_xor(sacc, 1);
    sacc += __shfl_xor(sacc, 2);
    if ((ln & 3) == 0) {
      dsh[buf * 64 + r] = sacc;
      // (also to the delta buffer, as the separate pass writes it: every workgroup that sweeps the tile stores the
      // same value)
      if (qb + r < p.Lq) ((float*)p.delta)[((long long)b * p.H + h) * p.Lq + qb + r] = sacc;
    }
  };
  if (qt0 < nqt) fetch(qt0 * 64, 0);
  if (dik && w >= 4 && qt0 < nqt) dik_issue(qt0 * 64);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (dik) {
    if (w >= 4 && qt0 < nqt) dik_reduce(0, qt0 * 64);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // the V fragments' loads counted as complete here (an empty statement reading them: the compiler's own wait lands
  // in front of it): left pending into the loop they got a vmcnt(0) before their first MFMA inside it (the second
  // sub-block's instance), which waited for the next tile's DMA on every tile
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) asm volatile("" : "+v"(vf[j][kk]));

#ifdef SVAE_STAMPS
  { BWD8_T(t1); BWD8_ACC(0, t_start, t1); }
#endif
  for (int qt = qt0; qt < nqt; ++qt) {
#ifdef SVAE_STAMPS
    BWD8_T(ta);
    st_acc[7] += 1;
#endif
    const int buf = (qt - qt0) & 1;
    const int qb = qt * 64;
    const char* Qs = QO + buf * 2 * R::BYTES;
    const char* dOs = Qs + R::BYTES;
    const float* nl = cst + (buf * NWB + w) * 128;
    const bool rmw_t = rmw && qt < nqt_prev;   // (wave-uniform)
    if (rmw_t) {
      // this wave's dQ fragments of the first sub-block's partial (the layout of the stores below: piece u, lane l =
      // query 16 dq_q16 + (l & 15), dims 16 (dq_u0 + u) + 4 (l >> 4) .. + 3) into its own slot; issued before the next
      // tile's DMA, so the dQ phase's counted wait covers it. The first sub-block's stores were drained by the
      // workgroup barrier between the sub-blocks.
      const int lf = lane_id_fresh();
      const bool qok = qb + 16 * dq_q16 + (lf & 15) < p.Lq;
      const int qrow = (qb + 16 * dq_q16 + (lf & 15)) * (int)ldp + 4 * (lf >> 4);
      const u32x4 prs4 = buffer_rsrc(part, 0x7FFFFFF0u);
      int ro[DQ_NT];
#pragma unroll
      for (int u = 0; u < DQ_NT; ++u) {
        const int d = 16 * (dq_u0 + u);
        ro[u] = (qok && d + 4 * (lf >> 4) < p.hd) ? (qrow + d) * 4 : 0x7FFFFFF0;
      }
      static_assert(DQ_NT == 2 || DQ_NT == 3, "dQ fragments per wave");
      if constexpr (DQ_NT == 2) dma16x2_lds(prs4, rslots + w * DQ_NT * 1024, ro[0], ro[1]);
      else dma16x3_lds(prs4, rslots + w * DQ_NT * 1024, ro[0], ro[1], ro[2]);
    }
    // direct tiles (see the dQ stores): plane 0 (its sub-blocks hold every key of these causal queries), below the
    // host's limit dq_direct, and below this sub-block's last key (a later sub-block of the plane adds to the others)
    // (hd 96: dq_direct <= 256, so the second sub-block has no direct tiles)
    const bool direct_t = !(RMW && HDC == 96) && pk == 0 && qb + 64 <= p.dq_direct && qb + 64 <= k0 + BWD8_KEYS;
    const bool rot_t = direct_t && p.dq_bf && p.rot;
    if (rot_t) {
      // the inverse rotary's cos / sin of this wave's dQ fragments (query, dim pair 2 j, 2 j + 1 per 16 B), by
      // LDS-DMA with the tile: a plain load at the use waited for it (and for the next tile's DMA) in the dQ phase
      const int lf = lane_id_fresh();
      const int q = qb + 16 * dq_q16 + (lf & 15);
      const bool qok = q < p.Lq;
      const u32x4 crs = buffer_rsrc(p.rot, 0x7FFFFFF0u);
      int co[DQ_NT];
#pragma unroll
      for (int u = 0; u < DQ_NT; ++u) {
        const int d = 16 * (dq_u0 + u) + 4 * (lf >> 4);
        co[u] = (qok && d < p.hd) ? (q * (p.rot_d / 2) + (h * p.hd + d) / 2) * 8 : 0x7FFFFFF0;
      }
      if constexpr (DQ_NT == 2) dma16x2_lds(crs, cslots + w * DQ_NT * 1024, co[0], co[1]);
      else dma16x3_lds(crs, cslots + w * DQ_NT * 1024, co[0], co[1], co[2]);
    }
    if (qt + 1 < nqt) fetch(qb + 64, buf ^ 1);
    if (dik && w >= 4 && qt + 1 < nqt) dik_issue(qb + 64);
    const float* dlp = dik ? dsh + buf * 64 : nl + 64;   // the tile's delta rows
    const bool live = (!p.causal || kw <= qb + 63) && qb < band_end && kw < p.Lk;
#ifdef SVAE_STAMPS
    if (live) st_acc[6] += 1;
#endif
    if (live && SVAE_BWD8_DIAG != 1) {
      const char* Kw = Ks + (wk >> 1) * R::BYTES;    // this wave's 32 keys: rows 32 (wk & 1) .. of image wk / 2
      const bool edge = !keys_all_ok || qb + 64 > p.Lq || (p.causal && kw + 31 > qb) || qb + 63 >= band_end;
      const int qlim = min(p.Lq, band_end) - qb;
      constexpr int TPP = 2;
#pragma unroll
      for (int pass = 0; pass < 4 / TPP; ++pass) {
        // the K fragments are re-read per pass (live only through its S products: 4 NKK registers fewer at the
        // dV / dK peak, which is what keeps hd 96 at 256 registers without spills)
        bf16x8 kf[2][NKK];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kk = 0; kk < NKK; ++kk) kf[j][kk] = *(const bf16x8*)(Kw + R::off(32 * (wk & 1) + 16 * j + li, g + 4 * kk));
        f32x4 s[2][TPP], dp[2][TPP];
#pragma unroll
        for (int th = 0; th < TPP; ++th) {
          const int t = pass * TPP + th;
          const f32x4 sl = *(const f32x4*)(nl + 16 * t + 4 * g) * -inv_scale;   // -lse / scale
          const f32x4 dl = -*(const f32x4*)(dlp + 16 * t + 4 * g);              // -delta
          s[0][th] = sl; s[1][th] = sl;
          dp[0][th] = dl; dp[1][th] = dl;
          if (edge) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const int kmin = p.causal ? kw + 16 * j + li - qb : -0x40000000;
              const unsigned kbad = key_ok[j] ? 0u : 1u;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int ql = 16 * t + 4 * g + r;
                s[j][th][r] = (kbad | (unsigned)(ql >= qlim) | (unsigned)(ql < kmin)) ? -INFINITY : s[j][th][r];
              }
            }
          }
#pragma unroll
          for (int k2 = 0; k2 < NKK; ++k2) {
            const bf16x8 qa = *(const bf16x8*)(Qs + R::off(16 * t + li, g + 4 * k2));
            const bf16x8 oa = *(const bf16x8*)(dOs + R::off(16 * t + li, g + 4 * k2));
            s[0][th] = mfma16(qa, kf[0][k2], s[0][th]);
            s[1][th] = mfma16(qa, kf[1][k2], s[1][th]);
            dp[0][th] = mfma16(oa, vf[0][k2], dp[0][th]);
            dp[1][th] = mfma16(oa, vf[1][k2], dp[1][th]);
          }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int th = 0; th < TPP; ++th)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float pr = __builtin_amdgcn_exp2f(s[j][th][r] * c);
              s[j][th][r] = pr;
              dp[j][th][r] = pr * dp[j][th][r];
            }
#pragma unroll
        for (int k2 = 0; k2 < TPP / 2; ++k2) {
          const int kk = pass * (TPP / 2) + k2;
          const bf16x8 pf0 = pack8(s[0][2 * k2], s[0][2 * k2 + 1]), pf1 = pack8(s[1][2 * k2], s[1][2 * k2 + 1]);
          const bf16x8 df0 = pack8(dp[0][2 * k2], dp[0][2 * k2 + 1]), df1 = pack8(dp[1][2 * k2], dp[1][2 * k2 + 1]);
          // rows r0 = 32 kk + 4g + (li >> 2) and r0 + 16: the swizzles see row bits 0-3 only, so the address is the
          // lane's row-(4g + (li >> 2)) address plus a constant (folded into the ds_read offset)
          const int rq = 4 * g + (li >> 2);
#pragma unroll
          for (int u = 0; u < NT; ++u) {
            const int uu = 4 * u + (li & 3);
            const int pitch = 16 * u < 64 ? 128 : 64;
            const int lo = R::uoff(rq, uu);
            const int ro = 32 * kk * pitch;
            const lds_char* po = lds_ptr(dOs) + lo + ro;
            const lds_char* pq = lds_ptr(Qs) + lo + ro;
            const bf16x8 ao = cat44(lds_read_tr3(po), lds_read_tr3(po + 16 * pitch));
            dv[0][u] = mfma16(ao, pf0, dv[0][u]);
            dv[1][u] = mfma16(ao, pf1, dv[1][u]);
            const bf16x8 aq = cat44(lds_read_tr3(pq), lds_read_tr3(pq + 16 * pitch));
            dk[0][u] = mfma16(aq, df0, dk[0][u]);
            dk[1][u] = mfma16(aq, df1, dk[1][u]);
          }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int th = 0; th < TPP; ++th)
            *(bf16x4*)(dSs + TS::uoff(32 * wk + 16 * j + li, 4 * (pass * TPP + th) + g)) =
                (bf16x4){f2bf(dp[j][th][0]), f2bf(dp[j][th][1]), f2bf(dp[j][th][2]), f2bf(dp[j][th][3])};
      }
    } else {
      const bf16x4 z = {f2bf(0.f), f2bf(0.f), f2bf(0.f), f2bf(0.f)};
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) *(bf16x4*)(dSs + TS::uoff(32 * wk + 16 * j + li, 4 * t + g)) = z;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#ifdef SVAE_STAMPS
    BWD8_T(tb);
    BWD8_ACC(1, ta, tb);
#endif
    __builtin_amdgcn_s_barrier();   // dS^T complete (a raw barrier: __syncthreads' vmcnt(0) would drain the DMA)
    asm volatile("" ::: "memory");
    // in-kernel delta of the NEXT tile, by waves 4-7 beside the other waves' dQ phase (its DMA, issued at the top of
    // this step, has landed by now; their only older vector-memory operations are the last step's dQ stores); written
    // to dsh[buf ^ 1], published by the end-of-tile barrier. (At the end of the step it held every wave at that barrier.)
    if (dik && w >= 4 && qt + 1 < nqt) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      dik_reduce(buf ^ 1, qb + 64);
    }
#ifdef SVAE_STAMPS
    BWD8_T(tc);
    BWD8_ACC(2, tb, tc);
#endif
    // partial dQ[q = qb + 16 dq_q16 + li][d = 16 (dq_u0 + u) + 4g + r] over the block's keys (K fragment as the first
    // MFMA operand: a lane holds 4 consecutive dims of one query)
    f32x4 dq[DQ_NT];
#pragma unroll
    for (int u = 0; u < DQ_NT; ++u) dq[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int kvis = p.causal ? min(BWD8_KEYS, qb + 64 - k0) : min(BWD8_KEYS, p.Lk - k0);   // keys with dS != 0
    // Addresses: row kr = 32 kk + 8g + (li >> 2) (and kr + 4) of the dS^T and K images. The swizzles depend on row
    // bits 0-3 only, which do not move with kk, so a lane's address is its kk = 0 address plus a constant per kk
    // (folded into the ds_read offset field): per-kk addresses computed in full were spilled (76 VGPRs at hd 96).
    {
      const int q4 = 8 * g + (li >> 2);
      const int uq = 4 * dq_q16 + (li & 3);
      const lds_char* sp0 = lds_ptr(dSs) + TS::uoff(q4, uq);
      const lds_char* sp4 = lds_ptr(dSs) + TS::uoff(q4 + 4, uq);
      const lds_char* kp0[DQ_NT];
      const lds_char* kp4[DQ_NT];
#pragma unroll
      for (int u = 0; u < DQ_NT; ++u) {
        const int uk = 4 * (dq_u0 + u) + (li & 3);
        kp0[u] = lds_ptr(Ks) + R::uoff(q4, uk);
        kp4[u] = lds_ptr(Ks) + R::uoff(q4 + 4, uk);
      }
#pragma unroll
      for (int kk = 0; kk < BWD8_KEYS / 32; ++kk) {
        if (32 * kk >= kvis || SVAE_BWD8_DIAG == 1) break;
        const int so = kk * 32 * TS::PITCH;
        const bf16x8 a = cat44(lds_read_tr3(sp0 + so), lds_read_tr3(sp4 + so));
#pragma unroll
        for (int u = 0; u < DQ_NT; ++u) {
          // the fragment's part of the row image (dims < 64: 128-B rows; the 96-dim tail: 64-B rows) is wave-uniform
          const int pitch = 16 * (dq_u0 + u) < 64 ? 128 : 64;
          const int ko = (kk >> 1) * R::BYTES + (kk & 1) * 32 * pitch;
          const bf16x8 bk = cat44(lds_read_tr3(kp0[u] + ko), lds_read_tr3(kp4[u] + ko));
          dq[u] = mfma16(bk, a, dq[u]);
        }
      }
    }
    if (rmw_t || rot_t) {
      // the slot DMAs landed once only the next tile's DMA (its QO_PW + 2 loads, issued after them) can be in flight
      // (+ the 4 O / o_lo loads of waves 4-7 with the in-kernel delta)
      if (qt + 1 < nqt) {
        if (dik && w >= 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QO_PW + 6) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QO_PW + 2) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    if (rmw_t) {
      const lds_char* sl = lds_ptr(rslots + w * DQ_NT * 1024) + 16 * lane_id_fresh();
#pragma unroll
      for (int u = 0; u < DQ_NT; ++u) dq[u] += *(const f32x4*)(sl + 1024 * u);
    }
    if (direct_t) {
      // causal, plane 0, queries below this sub-block's last key: plane 0's sub-blocks hold every key these queries
      // see (the first sub-block's share added above), so dQ is final here
      // (scale, inverse rotary, bf16 or f32 out) -- no partial plane, and attn_dq_reduce skips these rows. The same
      // number of store instructions as the partial path (out-of-range offsets for masked lanes): the end-of-tile wait
      // counts them.
      // lane terms from a fresh v_mbcnt: offsets derived from the hoisted lane id were kept across the q-tile loop
      // and spilled (hd 96), and each reload's vmcnt(0) would wait on the next tile's DMA
      const int lf = lane_id_fresh();
      const int q = qb + 16 * dq_q16 + (lf & 15);
      const bool qok = q < p.Lq;
#pragma unroll
      for (int u = 0; u < DQ_NT; ++u) {
        const int d = 16 * (dq_u0 + u) + 4 * (lf >> 4);
        const bool ok = qok && d < p.hd;
        float scl = p.scale;
        if constexpr (HDC == 64) scl = *(volatile const float*)sscl;
        f32x4 v = dq[u] * scl;
        if (p.dq_bf) {
          if (p.rot) {
            // (the tile's cos / sin slot; a masked lane's DMA wrote zeros and its store is dropped)
            const f32x4 cs = *(const f32x4*)(lds_ptr(cslots + w * DQ_NT * 1024) + 16 * lf + 1024 * u);
            const float a0 = v[0], b0 = v[1], a1 = v[2], b1 = v[3];
            v[0] = a0 * cs[0] + b0 * cs[1];
            v[1] = -a0 * cs[1] + b0 * cs[0];
            v[2] = a1 * cs[2] + b1 * cs[3];
            v[3] = -a1 * cs[3] + b1 * cs[2];
          }
          const bf16x4 pd = {f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, pd), drs,
                                                ok ? (q * (int)p.ldq_bf + d) * 2 : 0x7FFFFFF0, 0, 0);
        } else {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), drs, ok ? (q * (int)ldp + d) * 4 : 0x7FFFFFF0,
                                                 0, 0);
        }
      }
    } else {
      const bool qok = qb + 16 * dq_q16 + li < p.Lq;
      const int qrow = (qb + 16 * dq_q16 + li) * (int)ldp + 4 * g;
#pragma unroll
      for (int u = 0; u < DQ_NT; ++u) {
        const int d = 16 * (dq_u0 + u);
        const int off = (qok && d + 4 * g < p.hd) ? (qrow + d) * 4 : 0x7FFFFFF0;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, dq[u]), prs, off, 0, 0);
      }
    }
#ifdef SVAE_STAMPS
    BWD8_T(td);
    BWD8_ACC(3, tc, td);
#endif
    // the next tile's DMA (issued before this tile's stores) has landed; the stores stay in flight
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DQ_STORES) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#ifdef SVAE_STAMPS
    { BWD8_T(te); BWD8_ACC(4, td, te); }
#endif
  }
#ifdef SVAE_STAMPS
  BWD8_T(t_ep);
#endif

  // epilogue: dK (scaled, inverse rotary) and dV for key = kw + 16j + li, dims 16u + 4g + (0..3)
  if (p.cls_q0 > 0 && kw == 0) {
    // the [CLS] keys with the window's [CLS] split: their dK / dV so far (queries < cls_q0) as slab 0 of the f32
    // partials attn_cls_finalize_kernel sums (unscaled, before the inverse rotary)
    bwd_cls_store_slab<NT>(p, p.cls_part, b, h, dk, dv);
  } else {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = kw + 16 * j + li;
    if (key >= p.Lk) continue;
    bf16* DK = p.dk + b * p.bdk + (long long)key * p.sdk + (long long)h * p.hd;
    bf16* DV = p.dv + b * p.bdv + (long long)key * p.sdv + (long long)h * p.hd;
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      const int d = 16 * u + 4 * g;
      if (d >= p.hd) continue;
      float x[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) x[r] = dk[j][u][r] * p.scale;
      if (p.rot) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int pair = (h * p.hd + d) / 2 + e;
          const float2 cs = ((const float2*)p.rot)[(long long)key * (p.rot_d / 2) + pair];
          const float a = x[2 * e], cc = x[2 * e + 1];
          x[2 * e] = a * cs.x + cc * cs.y;
          x[2 * e + 1] = -a * cs.y + cc * cs.x;
        }
      }
      *(bf16x4*)(DK + d) = (bf16x4){f2bf(x[0]), f2bf(x[1]), f2bf(x[2]), f2bf(x[3])};
      *(bf16x4*)(DV + d) = (bf16x4){f2bf(dv[j][u][0]), f2bf(dv[j][u][1]), f2bf(dv[j][u][2]), f2bf(dv[j][u][3])};
    }
  }
  }
#ifdef SVAE_STAMPS
  {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    BWD8_T(t_end);
    BWD8_ACC(5, t_ep, t_end);
    const int lin_id = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    unsigned long long x = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) x = lane == k ? st_acc[k] : x;   // (static indices: no scratch array)
    if (lin_id < 1024 && lane < 8) svae_bwd8_stamps[lin_id][w][lane] = x;
  }
#endif
}

template <int HDC, int NSUB>
__global__ __launch_bounds__(512, 1) void attn_bwd8_kernel(AP p) {
  // + the per-wave dQ slots of the second sub-block (8 waves x HDC / 32 KiB: hd 96 fills the CU's 160 KiB exactly)
  // and, hd 64, the rotary slots of the direct tiles
  __shared__ __attribute__((aligned(16))) char smem[8 * RowImg<HDC>::BYTES + 4 * Tile<64>::BYTES + 2 * 8 * 128 * 4 +
                                                    (HDC == 64 && NSUB == 2 ? 2 : 1) * 8 * (HDC / 32) * 1024 +
                                                    (HDC == 64 ? 2 * 64 * 4 + 4 * 4096 + 16 : 0)];   // (+ in-kernel delta, scale)
  int kb, h, b;
  xcd_block(kb, h, b, p.causal ? 2 : 0);
  // NSUB 256-key sub-blocks per workgroup and dQ plane (1, or 2 as two instances of the sweep: the loop form spilled
  // 42 VGPRs into the q-tile loop at hd 96; nsub = p.kblk / 256 = NSUB, a run-time value on purpose -- the
  // compile-time one changed the register allocation and spilled inside the hd 96 loop)
  if constexpr (NSUB == 1) {
    attn_bwd8_tile<HDC, 1, false>(p, smem, kb, h, b, 1);
  } else {
    const int nsub = p.kblk / BWD8_KEYS;
    attn_bwd8_tile<HDC, 2, false>(p, smem, nsub * kb, h, b, nsub);
    if (nsub == 2 && (2 * kb + 1) * BWD8_KEYS < p.Lk) {
      // the first sub-block's dQ plane stores drained before the second reads them back by LDS-DMA (an explicit
      // vmcnt(0): a workgroup barrier only waits lgkmcnt on gfx950, and the read-back need not come from the same
      // wave and lane that stored), then its LDS reads done
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      attn_bwd8_tile<HDC, 2, true>(p, smem, 2 * kb + 1, h, b, 2);
    }
  }
}


// ===================================================================================== backward, sliding window: [CLS]
// With SparseAttention's window every query sees the [CLS] block (keys 0-31, sparse_attention.py:39-60 include_cls), so
// key block 0 of attn_bwd8 would sweep ALL Lq / 64 query tiles while every other key block sweeps the ~6 of its band:
// at 2 x 16384 tokens that one workgroup per (batch, head) took 810 us of 6 layers' 17 ms step
// (profiles/r06i_c2s16k_kernel_summary.txt). With cls_q0 set, plane 0's key blocks stop at cls_q0 (past it they hold
// nothing but the [CLS] keys for any query) and this kernel takes the queries >= cls_q0 against the 32 [CLS] keys:
// 4 independent waves per workgroup, each sweeping CLS_TW query tiles with the bwd8 wave program for one 32-key slice
// (key on the MFMA lane; its own Q / dO / lse / delta LDS images and its own dS^T image, so no workgroup barrier in
// the loop), dQ of its tiles straight into plane 0 (no other writer there), dK / dV of the [CLS] keys into its own f32
// slab; attn_cls_finalize_kernel sums the slabs in a fixed order (deterministic).
constexpr int CLS_TW = 8;   // query tiles per wave

template <int HDC>
__global__ __launch_bounds__(256, 1) void attn_bwd_cls_kernel(AP p) {
  using R = RowImg<HDC>;
  using TS = Tile<64>;
  constexpr int NKK = HDC / 32, NT = HDC / 16;
  constexpr int WAVE_LDS = 2 * R::BYTES + 32 * TS::PITCH + 512;
  __shared__ __attribute__((aligned(16))) char smem[R::BYTES + 4 * WAVE_LDS];
  const int chunk = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  char* Ks = smem;   // the [CLS] keys' K rows (rows 32-63 read as zeros)
  char* Qs = smem + R::BYTES + w * WAVE_LDS;
  char* dOs = Qs + R::BYTES;
  char* dSs = dOs + R::BYTES;                  // dS^T [32 keys][64 queries]
  float* nl = (float*)(dSs + 32 * TS::PITCH);  // [lse 64 | delta 64]
  const long long hc = (long long)h * p.hd;
  const bf16* Q = p.q + b * p.bq + hc;
  const bf16* K = p.k + b * p.bk + hc;
  const bf16* V = p.v + b * p.bv + hc;
  const bf16* dO = p.dout + b * p.bdo + hc;
  const float* lse = p.lse + ((long long)b * p.H + h) * p.Lq;
  const float* delta = p.delta + ((long long)b * p.H + h) * p.Lq;
  const int nk = min(p.Lk, 32);
  {  // K image: the 4 waves split its pieces
    const u32x4 krs = buffer_rsrc(K, 0x7FFFFFF0u);
    for (int i = w; i < R::PIECES; i += 4) dma_img_piece<HDC>(krs, p.sk, 0, nk, p.hd, Ks, i, lane);
  }
  bool key_ok[2];
  bf16x8 vf[2][NKK];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = 16 * j + li;
    key_ok[j] = key < nk && !(p.pad && p.pad[b * p.ldpad + key]);
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      const int d = 32 * kk + 8 * g;
      u32x4 c = {0u, 0u, 0u, 0u};
      if (key < nk && d < p.hd) c = *(const u32x4*)(V + (long long)key * p.sv + d);
      vf[j][kk] = __builtin_bit_cast(bf16x8, c);
    }
  }
  const bool keys_all_ok = __builtin_amdgcn_ballot_w64(!(key_ok[0] && key_ok[1])) == 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  f32x4 dk[2][NT], dv[2][NT];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < NT; ++t) { dk[j][t] = (f32x4){0.f, 0.f, 0.f, 0.f}; dv[j][t] = dk[j][t]; }
  const float inv_scale = 1.0f / p.scale, c = p.scale * LOG2E;
  const int ntile = (p.Lq + 63) / 64;
  const int t0 = p.cls_q0 / 64 + (chunk * 4 + w) * CLS_TW, t1 = min(ntile, t0 + CLS_TW);
  float* part = p.dq_part + (long long)b * p.Lq * p.H * p.hd + hc;   // dQ plane 0
  const long long ldp = (long long)p.H * p.hd;
  const u32x4 qrs = buffer_rsrc(Q, 0x7FFFFFF0u), ors = buffer_rsrc(dO, 0x7FFFFFF0u);
  const u32x4 lser = buffer_rsrc(lse, (unsigned)p.Lq * 4u), der = buffer_rsrc(delta, (unsigned)p.Lq * 4u);
  for (int qt = t0; qt < t1; ++qt) {
    const int qb = qt * 64;
    for (int i = 0; i < R::PIECES; ++i) {
      dma_img_piece<HDC>(qrs, p.sq, qb, p.Lq, p.hd, Qs, i, lane);
      dma_img_piece<HDC>(ors, p.sdo, qb, p.Lq, p.hd, dOs, i, lane);
    }
    const int qo = qb + lane < p.Lq ? (qb + lane) * 4 : 0x7FFFFFF0;
    dma4x2_lds(lser, der, nl, qo, qo);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // every query of the tile is past the [CLS] keys (qb >= cls_q0 > 31) and inside their window: masks only for
    // padded keys and the ragged end
    const bool edge = !keys_all_ok || qb + 64 > p.Lq;
    const int qlim = p.Lq - qb;
    constexpr int TPP = 2;
#pragma unroll
    for (int pass = 0; pass < 4 / TPP; ++pass) {
      bf16x8 kf[2][NKK];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) kf[j][kk] = *(const bf16x8*)(Ks + R::off(16 * j + li, g + 4 * kk));
      f32x4 s[2][TPP], dp[2][TPP];
#pragma unroll
      for (int th = 0; th < TPP; ++th) {
        const int t = pass * TPP + th;
        const f32x4 sl = *(const f32x4*)(nl + 16 * t + 4 * g) * -inv_scale;
        const f32x4 dl = -*(const f32x4*)(nl + 64 + 16 * t + 4 * g);
        s[0][th] = sl; s[1][th] = sl;
        dp[0][th] = dl; dp[1][th] = dl;
        if (edge) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const unsigned kbad = key_ok[j] ? 0u : 1u;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int ql = 16 * t + 4 * g + r;
              s[j][th][r] = (kbad | (unsigned)(ql >= qlim)) ? -INFINITY : s[j][th][r];
            }
          }
        }
#pragma unroll
        for (int k2 = 0; k2 < NKK; ++k2) {
          const bf16x8 qa = *(const bf16x8*)(Qs + R::off(16 * t + li, g + 4 * k2));
          const bf16x8 oa = *(const bf16x8*)(dOs + R::off(16 * t + li, g + 4 * k2));
          s[0][th] = mfma16(qa, kf[0][k2], s[0][th]);
          s[1][th] = mfma16(qa, kf[1][k2], s[1][th]);
          dp[0][th] = mfma16(oa, vf[0][k2], dp[0][th]);
          dp[1][th] = mfma16(oa, vf[1][k2], dp[1][th]);
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int th = 0; th < TPP; ++th)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float pr = __builtin_amdgcn_exp2f(s[j][th][r] * c);
            s[j][th][r] = pr;
            dp[j][th][r] = pr * dp[j][th][r];
          }
#pragma unroll
      for (int k2 = 0; k2 < TPP / 2; ++k2) {
        const int kk = pass * (TPP / 2) + k2;
        const bf16x8 pf0 = pack8(s[0][2 * k2], s[0][2 * k2 + 1]), pf1 = pack8(s[1][2 * k2], s[1][2 * k2 + 1]);
        const bf16x8 df0 = pack8(dp[0][2 * k2], dp[0][2 * k2 + 1]), df1 = pack8(dp[1][2 * k2], dp[1][2 * k2 + 1]);
        const int rq = 4 * g + (li >> 2);
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          const int uu = 4 * u + (li & 3);
          const int pitch = 16 * u < 64 ? 128 : 64;
          const lds_char* po = lds_ptr(dOs) + R::uoff(rq, uu) + 32 * kk * pitch;
          const lds_char* pq = lds_ptr(Qs) + R::uoff(rq, uu) + 32 * kk * pitch;
          const bf16x8 ao = cat44(lds_read_tr3(po), lds_read_tr3(po + 16 * pitch));
          dv[0][u] = mfma16(ao, pf0, dv[0][u]);
          dv[1][u] = mfma16(ao, pf1, dv[1][u]);
          const bf16x8 aq = cat44(lds_read_tr3(pq), lds_read_tr3(pq + 16 * pitch));
          dk[0][u] = mfma16(aq, df0, dk[0][u]);
          dk[1][u] = mfma16(aq, df1, dk[1][u]);
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int th = 0; th < TPP; ++th)
          *(bf16x4*)(dSs + TS::uoff(16 * j + li, 4 * (pass * TPP + th) + g)) =
              (bf16x4){f2bf(dp[j][th][0]), f2bf(dp[j][th][1]), f2bf(dp[j][th][2]), f2bf(dp[j][th][3])};
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (the wave's own dS^T writes, read back below)
    // dQ of the tile over the 32 [CLS] keys: query 16 q16 + li, dims 16 u + 4 g .. (plane 0, unscaled)
    const int q4 = 8 * g + (li >> 2);
#pragma unroll
    for (int q16 = 0; q16 < 4; ++q16) {
      const int uq = 4 * q16 + (li & 3);
      const bf16x8 a = cat44(lds_read_tr3(lds_ptr(dSs) + TS::uoff(q4, uq)), lds_read_tr3(lds_ptr(dSs) + TS::uoff(q4 + 4, uq)));
      const int q = qb + 16 * q16 + li;
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const int uk = 4 * u + (li & 3);
        const bf16x8 bk = cat44(lds_read_tr3(lds_ptr(Ks) + R::uoff(q4, uk)), lds_read_tr3(lds_ptr(Ks) + R::uoff(q4 + 4, uk)));
        const f32x4 dq = mfma16(bk, a, (f32x4){0.f, 0.f, 0.f, 0.f});
        const int d = 16 * u + 4 * g;
        if (q < p.Lq && d < p.hd) *(f32x4*)(part + (long long)q * ldp + d) = dq;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (the LDS reads done before the next tile's DMA)
  }
  bwd_cls_store_slab<NT>(p, p.cls_part + (long long)(1 + chunk * 4 + w) * 2 * p.B * 32 * p.H * p.hd, b, h, dk, dv);
}

// dK / dV of the [CLS] keys = the sum of the nslab f32 slabs (slab 0 from attn_bwd8's key block 0, the rest from
// attn_bwd_cls_kernel) in a fixed order; dK scaled and inverse-rotated (pos = key) like attn_bwd8's epilogue
__global__ __launch_bounds__(256) void attn_cls_finalize_kernel(AP p, int nslab) {
  const int D = p.H * p.hd, D4 = D / 4;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= p.B * 32 * D4) return;
  const int row = i / D4, c4 = i - row * D4;   // row = b * 32 + key
  const int b = row / 32, key = row - b * 32;
  if (key >= p.Lk) return;
  const long long half = (long long)p.B * 32 * D;
  const float* src = p.cls_part + (long long)row * D + 4 * c4;
  f32x4 k4 = {0.f, 0.f, 0.f, 0.f}, v4 = k4;
  for (int s = 0; s < nslab; ++s) {
    k4 += *(const f32x4*)(src + s * 2 * half);
    v4 += *(const f32x4*)(src + s * 2 * half + half);
  }
  k4 *= p.scale;
  if (p.rot) {
    const f32x4 cs = *(const f32x4*)(p.rot + ((long long)key * (p.rot_d / 2) + 2 * c4) * 2);
    const float a0 = k4[0], b0 = k4[1], a1 = k4[2], b1 = k4[3];
    k4[0] = a0 * cs[0] + b0 * cs[1];
    k4[1] = -a0 * cs[1] + b0 * cs[0];
    k4[2] = a1 * cs[2] + b1 * cs[3];
    k4[3] = -a1 * cs[3] + b1 * cs[2];
  }
  *(bf16x4*)(p.dk + b * p.bdk + (long long)key * p.sdk + 4 * c4) = (bf16x4){f2bf(k4[0]), f2bf(k4[1]), f2bf(k4[2]), f2bf(k4[3])};
  *(bf16x4*)(p.dv + b * p.bdv + (long long)key * p.sdv + 4 * c4) = (bf16x4){f2bf(v4[0]), f2bf(v4[1]), f2bf(v4[2]), f2bf(v4[3])};
}

// One key block per workgroup. (Pairing key blocks x and nkb - 1 - x per workgroup, to even out the causal
// sweeps, measured slower: 219 -> 247 us at the C2 shape, 629 -> 771 us at L = 1024 -- half the workgroups and
// two serial prologues per workgroup cost more than the imbalance.)
template <int HDP, int HDC = HDP>
__global__ __launch_bounds__(256, HDP == 64 ? 2 : 1) void attn_bwd_kernel(AP p) {
  __shared__ __attribute__((aligned(16))) char smem[6 * Tile<HDP>::BYTES + 2 * Tile<64>::BYTES + 2 * 4 * 128 * 4];
  int kb, h, b;
  xcd_block(kb, h, b, p.causal ? 2 : 0);
  if constexpr (HDP == 64) attn_bwd_tile<HDP>(p, smem, kb, h, b);
  else attn_bwd_tile_wide<HDP, HDC>(p, smem, kb, h, b);
}

// dQ = scale * sum over the key blocks that can see the query (causal: kb <= q / 128) of the partials;
// bf16 out with inverse rotary (pos = query) or f32 out. One thread per 4 columns of one (batch, query).
__global__ __launch_bounds__(256) void attn_dq_reduce_kernel(AP p) {
  // one thread per 4 columns of one (batch, query) row: 32-bit index math only (the former 64-bit div / mod per
  // element of a grid-stride loop cost more than the memory traffic), all partial-plane loads of a thread issued
  // before the adds
  const int D = p.H * p.hd, D4 = D / 4;
  const int rows = p.B * p.Lq;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * D4) return;
  const int row = i / D4, c4 = i - row * D4;      // row = b * Lq + q
  const int b = row / p.Lq, q = row - b * p.Lq;
  const int KB = p.kblk;
  const int nkb = (p.Lk + KB - 1) / KB;
  const long long plane = (long long)rows * D;
  const int nk = p.causal ? min(nkb, q / KB + 1) : nkb;
  if (q < p.dq_direct) return;   // written final by attn_bwd8 (causal: plane 0 holds every key these queries see)
  // sliding window: key block k >= 1 wrote partials only for the query tiles it swept (see attn_bwd_kernel)
  int k1 = 1;
  if (p.window > 0)
    while (k1 < nk && q >= (min(p.Lq, k1 * KB + KB - SBLK + SBLK * p.window) + 63) / 64 * 64) ++k1;
  const float* src = p.dq_part + (long long)row * D + 4 * c4;
  f32x4 acc = *(const f32x4*)src;
  int k = k1;
  if (p.wrows > 0) {   // the window's compact planes (a query sees at most a few)
    for (; k < nk; ++k) acc += *(const f32x4*)(dq_plane(p, k, b) + (long long)q * D + 4 * c4);
    k = nk;
  }
  for (; k + 4 <= nk; k += 4) {
    const f32x4 v0 = *(const f32x4*)(src + k * plane), v1 = *(const f32x4*)(src + (k + 1) * plane);
    const f32x4 v2 = *(const f32x4*)(src + (k + 2) * plane), v3 = *(const f32x4*)(src + (k + 3) * plane);
    acc += v0;
    acc += v1;
    acc += v2;
    acc += v3;
  }
  for (; k < nk; ++k) acc += *(const f32x4*)(src + k * plane);
  acc *= p.scale;
  if (p.dq_bf) {
    if (p.rot) {   // inverse of (a c - b s, b c + a s) on the pairs (4c4, 4c4+1), (4c4+2, 4c4+3)
      const f32x4 cs = *(const f32x4*)(p.rot + ((long long)q * (p.rot_d / 2) + 2 * c4) * 2);
      const float a0 = acc[0], b0 = acc[1], a1 = acc[2], b1 = acc[3];
      acc[0] = a0 * cs[0] + b0 * cs[1];
      acc[1] = -a0 * cs[1] + b0 * cs[0];
      acc[2] = a1 * cs[2] + b1 * cs[3];
      acc[3] = -a1 * cs[3] + b1 * cs[2];
    }
    *(bf16x4*)((bf16*)p.dq_bf + (long long)row * p.ldq_bf + 4 * c4) = (bf16x4){f2bf(acc[0]), f2bf(acc[1]), f2bf(acc[2]), f2bf(acc[3])};
  } else {
    *(f32x4*)(p.dq + b * p.bdq + (long long)q * D + 4 * c4) = acc;
  }
}

bool fill(const svae_attn_desc* d, AP& p) {
  if (!d || !d->q || !d->k || !d->v || !d->o || !d->lse) return false;
  if (d->B <= 0 || d->H <= 0 || d->Lq <= 0 || d->Lk <= 0 || d->hd <= 0 || d->hd > 128 || d->hd % 8) return false;
  if ((d->sq | d->sk | d->sv | d->so | d->bq | d->bk | d->bv | d->bo) % 8) return false;
  p.q = (const bf16*)d->q; p.k = (const bf16*)d->k; p.v = (const bf16*)d->v; p.o = (bf16*)d->o;
  p.sq = d->sq; p.sk = d->sk; p.sv = d->sv; p.so = d->so;
  p.bq = d->bq; p.bk = d->bk; p.bv = d->bv; p.bo = d->bo;
  p.pad = d->key_pad; p.ldpad = d->Lk; p.lse = d->lse;
  p.B = d->B; p.H = d->H; p.Lq = d->Lq; p.Lk = d->Lk; p.hd = d->hd; p.causal = d->causal;
  p.scale = d->scale;
  p.dout = (const bf16*)d->dout; p.sdo = d->sdo; p.bdo = d->bdo;
  p.delta = d->delta; p.dq = d->dq; p.bdq = d->bdq;
  p.dk = (bf16*)d->dk; p.dv = (bf16*)d->dv; p.sdk = d->sdk; p.sdv = d->sdv; p.bdk = d->bdk; p.bdv = d->bdv;
  p.rot = d->rot_tab; p.rot_d = d->rot_d;
  p.o32 = d->o32; p.so32 = d->so32; p.bo32 = d->bo32;
  p.dq_part = d->dq_part; p.dq_bf = d->dq_bf; p.ldq_bf = d->ldq_bf;
  p.window = d->window;
  p.olo = (bf16*)d->o_lo; p.solo = d->so_lo; p.bolo = d->bo_lo;
  if (p.olo && ((p.solo | p.bolo) % 8)) return false;
  p.kblk = BWD_KEYS;
  p.dq_direct = 0;
  p.cls_q0 = 0;
  p.cls_part = nullptr;
  p.delta_inkernel = 0;
  p.wrows = 0;
  p.nsplit = 1; p.kc = p.Lk;
  p.split_o = nullptr; p.split_olo = nullptr; p.split_lse = nullptr;
  if (p.window < 0 || (p.window > 0 && !p.causal)) return false;
  if (p.o32 && ((p.so32 | p.bo32) % 4)) return false;
  return true;
}

// The backward's kernel choice and dQ-partial layout for a shape (svae_attn_bwd and the workspace-size queries agree on
// it). hd <= 96: the 8-wave 256-key kernel, two 256-key sub-blocks per dQ plane from 512 queries on; hd 128 and the
// encoder's <= 64 latent queries at hd <= 64: the 4-wave 128-key one. Environment switches (A/B runs only):
// SVAE_ATTN_BWD8=0 (the 4-wave kernels everywhere), SVAE_ATTN_BWD_SMALLQ=0 (the 8-wave kernel for <= 64 queries too),
// SVAE_BWD8_SUB=1 (one sub-block per plane), SVAE_ATTN_WINDOW_COMPACT=0 (dense planes in window mode).
struct BwdLayout {
  bool use8;
  int nsub, kblk, wrows;
  long long plane_elems;   // floats of the dQ partial planes (the [CLS] slabs follow them)
};
BwdLayout bwd_layout(int B, int H, int Lq, int Lk, int hd, bool causal, int window) {
  static const int bwd8_env = [] { const char* e = getenv("SVAE_ATTN_BWD8"); return e ? atoi(e) : 1; }();
  // one query tile (the encoder's 64 latent / learned queries) at hd <= 64: the 4-wave 128-key kernel, two workgroups
  // per CU, hides more of the per-workgroup prologue / epilogue that such a sweep is made of (C2 encoder shape 64 -> 58
  // us, C4's 180 -> 171 us: profiles/r05enc_attn_bwd_smallq_probe.log)
  static const int smallq_env = [] { const char* e = getenv("SVAE_ATTN_BWD_SMALLQ"); return e ? atoi(e) : 1; }();
  // two 256-key sub-blocks per workgroup and dQ plane for >= 512 queries; fewer query tiles per key block (the
  // encoder's latent queries) keep one: there the two serial sweeps of one workgroup cost more than the halved planes
  static const int sub_env = [] { const char* e = getenv("SVAE_BWD8_SUB"); return e && atoi(e) == 1 ? 1 : 2; }();
  static const int compact_env = [] { const char* e = getenv("SVAE_ATTN_WINDOW_COMPACT"); return e ? atoi(e) : 1; }();
  BwdLayout l;
  l.use8 = bwd8_env && hd <= 96 && !(smallq_env && Lq <= 64 && hd <= 64);
  l.nsub = l.use8 && sub_env == 2 && Lq >= 512 ? 2 : 1;
  l.kblk = l.use8 ? BWD8_KEYS * l.nsub : BWD_KEYS;
  const long long D = (long long)H * hd;
  l.wrows = 0;
  l.plane_elems = (long long)((Lk + BWD_KEYS - 1) / BWD_KEYS) * B * Lq * D;   // dense: the 128-key planes (either kernel)
  if (l.use8 && window > 0 && causal && compact_env) {
    // a plane's band: its keys pk kblk .. + kblk - 1 are seen by queries up to pk kblk + kblk - 32 + 32 window (whole
    // query tiles); plane 0 keeps every row (the [CLS] keys are seen by all queries)
    const int R = (std::min(Lq, l.kblk - SBLK + SBLK * window) + 63) / 64 * 64;
    const int np = (Lk + l.kblk - 1) / l.kblk;
    if (np > 1 && R < Lq) {
      l.wrows = R;
      l.plane_elems = (long long)B * Lq * D + (long long)(np - 1) * B * R * D;
    }
  }
  return l;
}

// floats of the [CLS] split's dK / dV slabs: at most 1 + 4 ceil(tiles / (4 CLS_TW)) of [2][B][32][H hd]
long long cls_slab_elems(int B, int H, int Lq, int hd) {
  const long long nslab = 1 + 4 * (((Lq + 63) / 64 + 4 * CLS_TW - 1) / (4 * CLS_TW));
  return nslab * 2 * B * 32 * H * hd;
}

}  // namespace

namespace {

// the forward's kernel choice for the problem p (split-KV, p.nsplit > 1: one launch over B nsplit batches, the kernel
// choice made for a slice's kc keys)
void launch_fwd(const AP& p, hipStream_t s) {
  dim3 grid((p.Lq + 127) / 128, p.H, p.B * p.nsplit);
  const int Lk = p.nsplit > 1 ? p.kc : p.Lk;
  // the 32x32-MFMA kernel for hd <= 64 (hd 96 spilled; SVAE_ATTN_FWD32=0: the 16x16 kernels, for A/B runs); its padding
  // bit mask holds FWD32_MAXPAD keys and its DMA / store offsets are 32-bit byte offsets from a sequence's row 0
  static const int fwd32_env = [] { const char* e = getenv("SVAE_ATTN_FWD32"); return e ? atoi(e) : 1; }();
  static const int occ_env = [] { const char* e = getenv("SVAE_ATTN_FWD32_OCC"); return e ? atoi(e) : 3; }();
  static const int ns_env = [] { const char* e = getenv("SVAE_ATTN_FWD32_NS"); return e ? atoi(e) : 2; }();
  const long long so = p.nsplit > 1 ? (long long)p.H * p.hd : p.so, solo = p.nsplit > 1 ? so : p.solo;
  const bool fit32 = ((long long)Lk + 64) * std::max(p.sk, p.sv) * 2 < 0x7FFFFFF0LL &&
                     ((long long)p.Lq + 128) * so * 2 < 0x7FFFFFF0LL && (!p.pad || Lk <= FWD32_MAXPAD) &&
                     (!p.olo || ((long long)p.Lq + 128) * solo * 2 < 0x7FFFFFF0LL);   // (o_lo's 32-bit offsets too)
  if (fwd32_env && fit32 && p.hd <= 64) {
    if (ns_env == 3) hipLaunchKernelGGL((attn_fwd32_kernel<64, 3, 3>), grid, dim3(256), 0, s, p);
    else if (occ_env == 4) hipLaunchKernelGGL((attn_fwd32_kernel<64, 4, 2>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((attn_fwd32_kernel<64, 3, 2>), grid, dim3(256), 0, s, p);
  } else if (p.hd <= 64) hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(256), 0, s, p);
  else if (p.hd <= 96) hipLaunchKernelGGL((attn_fwd_kernel<128, 96>), grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(attn_fwd_kernel<128>, grid, dim3(256), 0, s, p);
}

// Split-KV forward for few queries over many keys (the encoder's 64 learned / latent queries against a long sequence:
// at 2 x 16384 tokens one 128-query tile per (batch, head) gave 16 workgroups for the whole chip, 312 us per launch,
// profiles/r06i_c2s16k_kernel_summary.txt): the keys are cut into nsplit slices of kc keys, each slice's attention runs
// as its own problem into the workspace (O in bf16 + its bf16 residual, lse; one launch, the slice a grid dimension:
// fwd_slice), and this kernel combines them:
// lse = log sum_s exp(lse_s), O = sum_s exp(lse_s - lse) O_s (a slice whose keys are all padding has lse_s = -inf and no
// weight). One thread per 4 dims of one (batch, query, head).
__global__ __launch_bounds__(256) void attn_fwd_combine_kernel(AP p, const bf16* so_hi, const bf16* so_lo,
                                                              const float* slse, int nsplit) {
  const int D4 = p.hd / 4;
  const long long n = (long long)p.B * p.Lq * p.H * D4;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int c4 = (int)(i % D4);
  const long long r = i / D4;                 // ((b * Lq + q) * H + h)
  const int h = (int)(r % p.H), q = (int)((r / p.H) % p.Lq), b = (int)(r / ((long long)p.H * p.Lq));
  const long long D = (long long)p.H * p.hd;
  const long long slice_o = (long long)p.B * p.Lq * D, slice_l = (long long)p.B * p.H * p.Lq;
  const long long lrow = ((long long)b * p.H + h) * p.Lq + q;
  float m = -INFINITY;
  for (int sl = 0; sl < nsplit; ++sl) {
    const float l = slse[sl * slice_l + lrow];
    if (l > m) m = l;   // (NaN / -inf slices never raise it)
  }
  float wsum = 0.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const long long orow = ((long long)b * p.Lq + q) * D + (long long)h * p.hd + 4 * c4;
  for (int sl = 0; sl < nsplit; ++sl) {
    const float l = slse[sl * slice_l + lrow];
    if (!(l > -INFINITY)) continue;           // all-padding slice (or none): no weight, its O is 0 / 0
    const float wgt = __expf(l - m);
    const bf16x4 hi = *(const bf16x4*)(so_hi + sl * slice_o + orow), lo = *(const bf16x4*)(so_lo + sl * slice_o + orow);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] += wgt * ((float)hi[e] + (float)lo[e]);
    wsum += wgt;
  }
  const float inv = wsum > 0.f ? 1.0f / wsum : 0.f;
  acc *= inv;
  const bf16x4 oh = {f2bf(acc[0]), f2bf(acc[1]), f2bf(acc[2]), f2bf(acc[3])};
  const long long od = (long long)q * p.so + (long long)h * p.hd + 4 * c4;
  *(bf16x4*)(p.o + b * p.bo + od) = oh;
  if (p.olo) {
    const long long ol = (long long)q * p.solo + (long long)h * p.hd + 4 * c4;
    *(bf16x4*)(p.olo + b * p.bolo + ol) = (bf16x4){f2bf(acc[0] - (float)oh[0]), f2bf(acc[1] - (float)oh[1]),
                                                   f2bf(acc[2] - (float)oh[2]), f2bf(acc[3] - (float)oh[3])};
  }
  if (p.o32) *(f32x4*)(p.o32 + b * p.bo32 + (long long)q * p.so32 + (long long)h * p.hd + 4 * c4) = acc;
  if (c4 == 0) p.lse[lrow] = m + __logf(wsum);
}

// the split for a shape: slices of kc keys (a multiple of 64), nsplit of them; 1 = no split
void fwd_split(int B, int H, int Lq, int Lk, bool causal, int window, int& nsplit, int& kc) {
  // SVAE_ATTN_FWD_SPLIT: 0 = off, 1 = on (about 512 workgroups), N > 1 = about N workgroups (A/B runs)
  static const int env = [] { const char* e = getenv("SVAE_ATTN_FWD_SPLIT"); return e ? atoi(e) : 1; }();
  nsplit = 1;
  kc = Lk;
  const long long nwg = (long long)((Lq + 127) / 128) * H * B;
  if (!env || causal || window > 0 || Lq > 128 || nwg >= 128 || Lk < 2048) return;
  const long long target = env > 1 ? env : 512;
  int sp = (int)std::min<long long>((target + nwg - 1) / nwg, (Lk + 255) / 256);
  if (sp < 2) return;
  kc = ((Lk + sp - 1) / sp + 63) / 64 * 64;
  nsplit = (Lk + kc - 1) / kc;
}

}  // namespace

SVAE_EXPORT int64_t svae_attn_fwd_ws_elems(int32_t B, int32_t H, int32_t Lq, int32_t Lk, int32_t hd, int32_t causal,
                                           int32_t window) {
  if (B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0 || hd <= 0) return 0;
  int nsplit, kc;
  fwd_split(B, H, Lq, Lk, causal != 0, window, nsplit, kc);
  if (nsplit <= 1) return 0;
  // per slice: O and its residual, bf16 [B][Lq][H hd] each (one float per element for both), lse f32 [B][H][Lq]
  return (int64_t)nsplit * ((int64_t)B * Lq * H * hd + (int64_t)B * H * Lq);
}

SVAE_EXPORT int svae_attn_fwd(const svae_attn_desc* d, svae_stream_t stream) {
  AP p;
  if (!fill(d, p)) return SVAE_EINVAL;
  if (d->causal && d->Lq != d->Lk) return SVAE_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  int nsplit, kc;
  fwd_split(d->B, d->H, d->Lq, d->Lk, d->causal != 0, d->window, nsplit, kc);
  if (nsplit > 1 && d->fwd_ws &&
      d->fwd_ws_elems >= svae_attn_fwd_ws_elems(d->B, d->H, d->Lq, d->Lk, d->hd, d->causal, d->window) &&
      !((uintptr_t)d->fwd_ws & 15) && d->hd % 4 == 0) {
    const long long D = (long long)d->H * d->hd, slice_o = (long long)d->B * d->Lq * D;
    bf16* ohi = (bf16*)d->fwd_ws;
    bf16* olo = ohi + (long long)nsplit * slice_o;
    float* lse = (float*)(olo + (long long)nsplit * slice_o);
    AP q = p;
    q.nsplit = nsplit; q.kc = kc;
    q.split_o = ohi; q.split_olo = olo; q.split_lse = lse;
    launch_fwd(q, s);
    const long long n = (long long)d->B * d->Lq * d->H * (d->hd / 4);
    hipLaunchKernelGGL(attn_fwd_combine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, ohi, olo, lse,
                       nsplit);
  } else {
    launch_fwd(p, s);
  }
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int svae_attn_bwd(const svae_attn_desc* d, svae_stream_t stream) {
  AP p;
  if (!fill(d, p)) return SVAE_EINVAL;
  if (!d->dout || !d->delta || !d->dq_part || !d->dk || !d->dv || (!d->dq && !d->dq_bf)) return SVAE_EINVAL;
  if ((d->sdo | d->bdo | d->sdk | d->sdv | d->bdk | d->bdv) % 4) return SVAE_EINVAL;
  if (d->causal && d->Lq != d->Lk) return SVAE_EINVAL;
  if (d->rot_tab && d->rot_d <= 0) return SVAE_EINVAL;
  if (d->hd % 4 || (d->dq_bf && d->ldq_bf % 4) || (!d->dq_bf && d->bdq % 4)) return SVAE_EINVAL;
  if (d->dq_bf && d->rot_tab && d->rot_d != d->H * d->hd) return SVAE_EINVAL;
  if ((long long)d->B * d->Lq * (d->H * d->hd / 4) > 0x7FFFFF00LL) return SVAE_EINVAL;   // (32-bit dQ-reduce index)
  // (the 8-wave kernel's DMA offsets are 32-bit byte offsets from a sequence's row 0)
  if (((long long)std::max(d->Lq, d->Lk) + 64) * std::max(std::max(d->sq, d->sk), d->sdo) * 2 > 0x7FFFFFF0LL) return SVAE_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int rows = d->B * d->Lq * d->H;
  const BwdLayout lay = bwd_layout(d->B, d->H, d->Lq, d->Lk, d->hd, d->causal != 0, d->window);
  const bool use8 = lay.use8;
  const int nsub = lay.nsub;
  // SVAE_ATTN_DQ_DIRECT=0: every query tile through the partial planes (A/B runs)
  static const int direct_env = [] { const char* e = getenv("SVAE_ATTN_DQ_DIRECT"); return e ? atoi(e) : 1; }();
  if (use8) {
    p.kblk = lay.kblk;
    p.wrows = lay.wrows;
    // causal: attn_bwd8 stores the final dQ of the queries below dq_direct itself (hd 96: key block 0's, < 256;
    // hd 64 with two sub-blocks: plane 0's, < 512)
    p.dq_direct = (d->causal && direct_env) ? (nsub == 2 && d->hd <= 64 ? 2 : 1) * BWD8_KEYS : 0;
    // sliding window: queries from cls_q0 on see nothing of dQ plane 0 but the [CLS] block -> attn_bwd_cls_kernel
    // (SVAE_ATTN_CLS_SPLIT=0: key block 0 sweeps every query, A/B runs)
    static const int cls_env = [] { const char* e = getenv("SVAE_ATTN_CLS_SPLIT"); return e ? atoi(e) : 1; }();
    if (cls_env && d->window > 0 && d->causal && (!d->rot_tab || d->rot_d == d->H * d->hd)) {
      const int q0 = (std::min(d->Lq, p.kblk - SBLK + SBLK * d->window) + 63) / 64 * 64;
      if (q0 < d->Lq) {
        p.cls_q0 = q0;
        p.cls_part = d->dq_part + lay.plane_elems;
      }
    }
    // in-kernel delta (SVAE_ATTN_DELTA_INKERNEL=0: the separate pass, A/B runs): the 8-wave kernel at hd <= 64 reads O
    // and o_lo itself; not with the [CLS] split (attn_bwd_cls_kernel reads delta from memory)
    static const int dik_env = [] { const char* e = getenv("SVAE_ATTN_DELTA_INKERNEL"); return e ? atoi(e) : 1; }();
    // (with the [CLS] split too: every query row >= cls_q0 lies in the band of the key block holding its own key, whose
    // workgroup stores its delta for attn_bwd_cls_kernel, launched after this kernel on the same stream)
    if (dik_env && d->hd <= 64 && !d->delta_ready && d->o_lo &&
        ((long long)d->Lq + 64) * std::max(d->so, d->so_lo) * 2 < 0x7FFFFFF0LL)
      p.delta_inkernel = 1;
  }
  // delta_ready: the dO GEMM's epilogue already wrote delta (svae_gemm_desc.delta)
  if (!d->delta_ready && !p.delta_inkernel) {
    if (d->hd <= 64) hipLaunchKernelGGL(attn_delta_kernel<8>, dim3((rows + 31) / 32), dim3(256), 0, s, p);
    else hipLaunchKernelGGL(attn_delta_kernel<16>, dim3((rows + 15) / 16), dim3(256), 0, s, p);
  }
  if (use8) {
    dim3 grid8((d->Lk + p.kblk - 1) / p.kblk, d->H, d->B);
    if (d->hd <= 64) {
      if (nsub == 2) hipLaunchKernelGGL((attn_bwd8_kernel<64, 2>), grid8, dim3(512), 0, s, p);
      else hipLaunchKernelGGL((attn_bwd8_kernel<64, 1>), grid8, dim3(512), 0, s, p);
    } else {
      if (nsub == 2) hipLaunchKernelGGL((attn_bwd8_kernel<96, 2>), grid8, dim3(512), 0, s, p);
      else hipLaunchKernelGGL((attn_bwd8_kernel<96, 1>), grid8, dim3(512), 0, s, p);
    }
  } else {
    p.kblk = BWD_KEYS;
    dim3 grid((d->Lk + BWD_KEYS - 1) / BWD_KEYS, d->H, d->B);
    if (d->hd <= 64) hipLaunchKernelGGL(attn_bwd_kernel<64>, grid, dim3(256), 0, s, p);
    else if (d->hd <= 96) hipLaunchKernelGGL((attn_bwd_kernel<128, 96>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(attn_bwd_kernel<128>, grid, dim3(256), 0, s, p);
  }
  if (p.cls_q0 > 0) {
    const int nfar = (d->Lq + 63) / 64 - p.cls_q0 / 64, nchunk = (nfar + 4 * CLS_TW - 1) / (4 * CLS_TW);
    const dim3 gc(nchunk, d->H, d->B);
    if (d->hd <= 64) hipLaunchKernelGGL(attn_bwd_cls_kernel<64>, gc, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(attn_bwd_cls_kernel<96>, gc, dim3(256), 0, s, p);
    const long long nf = (long long)d->B * 32 * (d->H * d->hd / 4);
    hipLaunchKernelGGL(attn_cls_finalize_kernel, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, s, p, 1 + 4 * nchunk);
  }
  const long long work = (long long)d->B * d->Lq * (d->H * d->hd / 4);
  // (causal with every query below kblk: attn_bwd8 stored the whole dQ itself)
  if (d->Lq > p.dq_direct)
    hipLaunchKernelGGL(attn_dq_reduce_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s, p);
  SVAE_LAUNCH_CHECK();
  return SVAE_OK;
}

SVAE_EXPORT int64_t svae_attn_dq_part_elems(int32_t B, int32_t H, int32_t Lq, int32_t Lk, int32_t hd) {
  if (B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0 || hd <= 0) return 0;
  // the dense planes (enough for any mode) + the sliding window's [CLS] dK / dV slabs (attn_bwd_cls_kernel)
  return (int64_t)((Lk + BWD_KEYS - 1) / BWD_KEYS) * B * Lq * H * hd + cls_slab_elems(B, H, Lq, hd);
}

SVAE_EXPORT int64_t svae_attn_dq_part_elems_w(int32_t B, int32_t H, int32_t Lq, int32_t Lk, int32_t hd, int32_t window) {
  if (B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0 || hd <= 0 || window < 0) return 0;
  return bwd_layout(B, H, Lq, Lk, hd, window > 0, window).plane_elems + cls_slab_elems(B, H, Lq, hd);
}

#ifdef SVAE_STAMPS
extern "C" __attribute__((visibility("default"))) int svae_debug_attn_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(svae_attn_stamps), sizeof(svae_attn_stamps)) == hipSuccess ? 0 : -1;
}
extern "C" __attribute__((visibility("default"))) int svae_debug_bwd8_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(svae_bwd8_stamps), sizeof(svae_bwd8_stamps)) == hipSuccess ? 0 : -1;
}
#endif
