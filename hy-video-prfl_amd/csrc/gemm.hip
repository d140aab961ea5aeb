// bf16 MFMA GEMM for the Wan DiT projections (QKV / O / cross-attn / FFN) and their backward.
//
//   C[m][n] = sum_k A(m,k) * B(n,k)     (+ fused epilogue)
//
// Operand layouts (chosen per call so no transpose kernel is ever needed):
//   A_KC: A(m,k) = A[m*lda + k]   (token-major activations, forward / dX)
//  !A_KC: A(m,k) = A[k*lda + m]   (dW: A = dY^T read straight from dY [L, N])
//   B_KC: B(n,k) = B[n*ldb + k]   (nn.Linear weight [out, in] in the forward)
//  !B_KC: B(n,k) = B[k*ldb + n]   (dX: weight read as [out][in] with k = out; dW: X [L, in])
//
// Three bf16 kernels, chosen by shape and epilogue (launch()): every element is summed in the
// same k order (32-deep MFMA k-steps in sequence), so their outputs are bit-identical (tested):
//   * gemm4w_kernel (the 720p projections, every epilogue): 256x256 tile,
//     4 waves = one per SIMD, each wave 128x128 with its 256 fp32 accumulators in AGPRs,
//     operands by buffer LDS-DMA into a 4-slot ring of 32-deep K-slices (details at the kernel);
//   * gemm256s_kernel (operands past 4 GiB, the fp8 path, tile code 512): 256x256 tile,
//     8 waves, staggered 4-phase LDS-DMA schedule (details at the kernel);
//   * gemm_kernel (small / ragged shapes): 128x128x64 tile, 4 waves (2x2), each 64x64 = 4x4
//     MFMA 16x16x32 tiles, register-staged double buffer, one barrier per K step.
// K-contiguous tiles live in LDS as rows with an XOR-swizzled 16-B chunk order and feed
// ds_read_b128; MN-contiguous tiles live as [k][128] rows (256 B, 32-B XOR swz_mn(k)) and feed
// ds_read_b64_tr_b16 (hardware transpose), so both layouts reach the same MFMA fragment.
// The MFMA is issued as D = B.A^T so each lane owns 4 consecutive n of one row m: epilogue stores
// are 8-16 B contiguous per lane.
// The fp8 path (C5) runs gemm256s_kernel<.., F8 = true>.
#include <stdlib.h>

#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = BM * BK * 2;  // 16 KiB per operand per stage

enum { EPI_BF16 = 0, EPI_GELU = 1, EPI_RESID = 2, EPI_F32 = 3, EPI_DGELU = 4 };

struct GemmArgs {
  const bf16* A; int64_t lda;
  const bf16* B; int64_t ldb;
  void* C; int64_t ldc;
  int M, N, K;
  const bf16* bias;     // [N] or null
  const float* gate;    // [N] or null (EPI_RESID)
  const void* res;      // EPI_RESID residual input (fp32 or bf16), may alias C
  int64_t ldr; int res_bf16;
  bf16* aux; int64_t ldaux;  // GELU: pre-activation out; RESID: y out; DGELU: pre-activation in
  int accumulate;       // EPI_F32: C += acc
  const float* sa = nullptr;   // fp8 path: per-row dequant scales of A [M]
  const float* sb = nullptr;   //           per-row dequant scales of B [N]
};

typedef __attribute__((ext_vector_type(8))) int i32x8;

// two 16-B K-major fragments (bf16 kernel's k-steps s = 0, 1 of one 128-B row chunk pair) as one
// 32-element e4m3 operand: lane (g = lane>>4) holds bytes [16g, 16g+16) and [64+16g, 64+16g+16)
// of its row.  A and B use the same k permutation, so the dot product is unchanged.
__device__ __forceinline__ i32x8 cat_fp8(bf16x8 lo, bf16x8 hi) {
  const u32x4 a = __builtin_bit_cast(u32x4, lo), b = __builtin_bit_cast(u32x4, hi);
  return (i32x8){(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2],
                 (int)b[3]};
}

// block-scaled MFMA 16x16x128 e4m3 (2x the bf16 rate; the unscaled fp8 forms run at the bf16
// rate): cbsz = blgp = 0 (both e4m3), opsel 0 -> byte 0 of each scale word = 127 = 2^0
__device__ __forceinline__ f32x4 mfma_fp8(i32x8 a, i32x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 0x7f7f7f7f, 0,
                                                          0x7f7f7f7f);
}

// 32-B granule swizzle of MN-major rows: k bits {0,1,3} -> the 8 k-rows one ds_read_b64_tr_b16
// lane group touches (q = k&3, g&1 = k>>3 bit) land on 8 different granules (conflict-free)
__device__ __forceinline__ int swz_mn(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

// ---- staging: global -> registers -----------------------------------------------------------
template <bool KC>
__device__ __forceinline__ void load_tile(u32x4 (&r)[4], const bf16* __restrict__ P, int64_t ld,
                                          int rows, int K, int r0, int k0) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + NT * i;
    if (KC) {  // [128 rows][8 chunks of 8 k]
      const int row = c >> 3, kc = c & 7;
      const int gr = min(r0 + row, rows - 1);
      const int gk = k0 + kc * 8;
      if (gk < K)
        r[i] = *(const u32x4*)(P + (int64_t)gr * ld + gk);
      else
        r[i] = (u32x4){0u, 0u, 0u, 0u};
    } else {   // [64 k][16 chunks of 8 rows]
      const int kr = c >> 4, mc = c & 15;
      const int gk = k0 + kr, gm = r0 + mc * 8;
      if (gk < K && gm < rows)
        r[i] = *(const u32x4*)(P + (int64_t)gk * ld + gm);
      else
        r[i] = (u32x4){0u, 0u, 0u, 0u};
    }
  }
}

template <bool KC>
__device__ __forceinline__ void store_tile(char* lds, const u32x4 (&r)[4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + NT * i;
    int off;
    if (KC) {
      const int row = c >> 3, kc = c & 7;
      off = row * 128 + ((kc ^ (row & 7)) << 4);
    } else {
      const int kr = c >> 4, mc = c & 15;
      off = kr * 256 + ((mc << 4) ^ (swz_mn(kr) << 5));
    }
    *(u32x4*)(lds + off) = r[i];
  }
}

// fragment for MFMA 16x16x32: lane l holds X[row = base + (l&15)][k = 32*s + 8*(l>>4) + 0..7]
template <bool KC>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int base, int s, int lane) {
  if (KC) {
    const int row = base + (lane & 15);
    const int kc = s * 4 + (lane >> 4);
    return *(const bf16x8*)(lds + row * 128 + ((kc ^ (row & 7)) << 4));
  } else {
    const int g = lane >> 4, l16 = lane & 15, q = l16 >> 2, p = l16 & 3;
    const int col = (base + 4 * p) * 2;
    const int k0 = s * 32 + g * 8 + q;
    const int k1 = k0 + 4;
    bf16x4 lo = lds_read_tr(lds + k0 * 256 + (col ^ (swz_mn(k0) << 5)));
    bf16x4 hi = lds_read_tr(lds + k1 * 256 + (col ^ (swz_mn(k1) << 5)));
    return cat8(lo, hi);
  }
}

__device__ __forceinline__ void tile_coords(int bid, int M, int N, int& tm, int& tn) {
  const int ntm = (M + BM - 1) / BM, ntn = (N + BN - 1) / BN;
  const int nwg = ntm * ntn;
  // XCD-aware remap (bijective): blocks b, b+8, ... share an XCD; give each XCD a contiguous
  // range of tiles so neighbouring tiles (shared A rows / B cols) hit the same L2.
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  int w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  // grouped ordering: GM tile-rows sweep all tile-columns together
  const int GM = 8;
  const int group = w / (GM * ntn);
  const int first_m = group * GM;
  const int gsz = min(ntm - first_m, GM);
  const int within = w - group * GM * ntn;
  tm = first_m + within % gsz;
  tn = within / gsz;
}

template <bool A_KC, bool B_KC, int EPI>
__device__ __forceinline__ void epilogue_tile(const GemmArgs& g, f32x4 v, int m, int n) {
#pragma clang diagnostic push
      if (EPI == EPI_F32) {
        float* cp = (float*)g.C + (int64_t)m * g.ldc + n;
        if (g.accumulate) {
          f32x4 o = *(f32x4*)cp;
          v = v + o;
        }
        *(f32x4*)cp = v;
        return;
      }
      if (EPI == EPI_DGELU) {
        const bf16x4 pre = *(const bf16x4*)(g.aux + (int64_t)m * g.ldaux + n);
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(bfr(v[r]) * gelu_tanh_grad(bf2f(pre[r])));
        *(bf16x4*)((bf16*)g.C + (int64_t)m * g.ldc + n) = o;
        return;
      }
      float y[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) y[r] = bfr(v[r] + (g.bias ? bf2f(g.bias[n + r]) : 0.f));
      if (EPI == EPI_BF16) {
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(y[r]);
        *(bf16x4*)((bf16*)g.C + (int64_t)m * g.ldc + n) = o;
      } else if (EPI == EPI_GELU) {
        bf16x4 o, pre;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pre[r] = f2bf(y[r]);
          o[r] = f2bf(gelu_tanh(y[r]));
        }
        if (g.aux) *(bf16x4*)(g.aux + (int64_t)m * g.ldaux + n) = pre;
        *(bf16x4*)((bf16*)g.C + (int64_t)m * g.ldc + n) = o;
      } else if (EPI == EPI_RESID) {
        if (g.aux) {
          bf16x4 yo;
#pragma unroll
          for (int r = 0; r < 4; ++r) yo[r] = f2bf(y[r]);
          *(bf16x4*)(g.aux + (int64_t)m * g.ldaux + n) = yo;
        }
        float rv[4];
        if (g.res_bf16) {
          const bf16x4 rr = *(const bf16x4*)((const bf16*)g.res + (int64_t)m * g.ldr + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) rv[r] = bf2f(rr[r]);
        } else {
          const f32x4 rr = *(const f32x4*)((const float*)g.res + (int64_t)m * g.ldr + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) rv[r] = rr[r];
        }
        f32x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gt = g.gate ? g.gate[n + r] : 1.f;
          o[r] = rv[r] + mul_rn(y[r], gt);  // x + y*e (two roundings, as in torch)
        }
        *(f32x4*)((float*)g.C + (int64_t)m * g.ldc + n) = o;
      }
#pragma clang diagnostic pop
}

template <bool A_KC, bool B_KC, int EPI>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];
  // stage st: A at smem + st*2*TILE_BYTES, B right after it
#define AS(st) (smem + (st) * 2 * TILE_BYTES)
#define BS(st) (smem + (st) * 2 * TILE_BYTES + TILE_BYTES)

  int tm, tn;
  tile_coords(blockIdx.x, g.M, g.N, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (g.K + BK - 1) / BK;
  u32x4 ra[4], rb[4];
  load_tile<A_KC>(ra, g.A, g.lda, g.M, g.K, m0, 0);
  load_tile<B_KC>(rb, g.B, g.ldb, g.N, g.K, n0, 0);
  store_tile<A_KC>(AS(0), ra);
  store_tile<B_KC>(BS(0), rb);
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) {
      load_tile<A_KC>(ra, g.A, g.lda, g.M, g.K, m0, (t + 1) * BK);
      load_tile<B_KC>(rb, g.B, g.ldb, g.N, g.K, n0, (t + 1) * BK);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[4], bfr_[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<A_KC>(AS(cur), wm * 64 + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr_[j] = read_frag<B_KC>(BS(cur), wn * 64 + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr_[j], af[i], acc[i][j]);
    }
    if (t + 1 < nk) {
      store_tile<A_KC>(AS(cur ^ 1), ra);
      store_tile<B_KC>(BS(cur ^ 1), rb);
    }
    __syncthreads();
  }

#undef AS
#undef BS
  // ---- epilogue: lane owns D[n = nb + 4*(lane>>4) + r][m = mb + (lane&15)], r = 0..3 ----
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    if (m >= g.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
      if (n >= g.N) continue;
      epilogue_tile<A_KC, B_KC, EPI>(g, acc[i][j], m, n);
    }
  }
}

// =========================================================================== 256x256 tile ===
// 8 waves (2 along M x 4 along N), each 128x64 = 8x4 MFMA 16x16x32 tiles; BK = 64; operands
// land in LDS by LDS-DMA (global_load_lds_dwordx4, one 1-KiB piece per wave instruction) and
// stay in flight across the barriers (counted `s_waitcnt vmcnt(N)` + raw s_barrier; no
// __syncthreads in the loop, one __shared__ array), per MI355X guide §5 "Pipelining across
// barriers".  The LDS images are the swizzled layouts above, produced by permuting each lane's
// SOURCE address (the DMA destination is lane-linear).  Requires K % 64 == 0 and MN-major
// extents % 256 == 0.
constexpr int BM2 = 256, BN2 = 256, NT2 = 512;
constexpr int TILE2 = BM2 * BK * 2;                    // 32 KiB per operand per stage


#ifndef GEMM_GROUP_M
#define GEMM_GROUP_M 4        // 256-row blocks walked together per XCD (L2 / MALL reuse of B)
#endif
__device__ __forceinline__ void tile_coords2(int bid, int M, int N, int& tm, int& tn) {
  const int ntm = (M + BM2 - 1) / BM2, ntn = (N + BN2 - 1) / BN2;
  const int nwg = ntm * ntn;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  int w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int GM = GEMM_GROUP_M;
  const int group = w / (GM * ntn);
  const int first_m = group * GM;
  const int gsz = min(ntm - first_m, GM);
  const int within = w - group * GM * ntn;
  tm = first_m + within % gsz;
  tn = within / gsz;
}

// ------------------------------------------------------------ 256x256, staggered 4-phase ---
// The 256x256 tile and 8-wave grid above, scheduled after the MI355X guide's 8-phase
// template (cdna_hip_programming.md §5): every K-tile is four phases, one C-quadrant (16 MFMAs)
// each; a phase = {fragment reads for its quadrant + one half-tile LDS-DMA} | barrier |
// {lgkmcnt(0), MFMA cluster, counted vmcnt} | barrier.  Waves 4-7 (wr = 1) run one barrier
// behind waves 0-3, so on every SIMD one partner's MFMA cluster overlaps the other's reads.
// The operand stream is cut into half-tiles, each holding exactly the fragments one phase reads:
//   A_h0: rows wr*128 + {0..63}   (quadrants 0, 1)    B_h0: cols wc*64 + {0..31}  (quadrants 0, 2)
//   A_h1: rows wr*128 + {64..127} (quadrants 2, 3)    B_h1: cols wc*64 + {32..63} (quadrants 1, 3)
// Half-tile h (tile h/4, part order A_h0, B_h0, B_h1, A_h1) is issued in phase h-6 into a 2-deep
// ring, retired by the counted vmcnt at the end of phase h-3 and first read in phase h-1 (A_h0:
// phase h).  Barrier numbering: wave group wr runs phase k between barriers 2k+1+wr and
// 2k+2+wr, so a writer of group wr retires h before barrier 2h-4+wr and a reader of group wr'
// reads it after barrier 2h-2+wr' >= 2h-3: every half-tile is retired by BOTH groups one
// barrier before its first reader passes (the guide's 'Read a staged buffer one phase AFTER
// the wait that retires it', with the stagger's extra barrier).  Half-tiles 0-2 are read in
// phases 0-1, before any in-loop wait: the prologue must retire all three (round 1 retired only
// 0-1, so waves 0-3 could read waves 4-7's half of B_h1 of tile 0 before it landed).  WAR: a
// slot is re-filled in phase h-6, >= 2 phases after its last read (phase h-8).
constexpr int HALF = 16384;

template <bool KC, bool IS_A>
__device__ __forceinline__ void dma_half(char* lds, const bf16* __restrict__ P, int64_t ld, int rows,
                                         int r0, int k0, int half, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = wid * 2 + i;                     // 16 pieces of 1 KiB
    const bf16* src;
    if (KC) {          // [128 local rows][64 k], 128-B rows, chunk ^ (row & 7)
      const int lr = piece * 8 + (lane >> 3), pc = lane & 7;
      const int grow = IS_A ? ((lr >> 6) * 128 + ((((lr >> 4) & 3) + 4 * half) << 4) + (lr & 15))
                            : ((lr >> 5) * 64 + ((((lr >> 4) & 1) + 2 * half) << 4) + (lr & 15));
      const int gr = min(r0 + grow, rows - 1);
      src = P + (int64_t)gr * ld + k0 + ((pc ^ (lr & 7)) << 3);
    } else {           // [64 k][128 local cols], 256-B rows, 32-B granule ^ swz_mn(k)
      const int kr = piece * 4 + (lane >> 4), pb = (lane & 15) << 4;
      const int lc = (pb ^ (swz_mn(kr) << 5)) >> 1;
      const int gcol = IS_A ? ((lc >> 6) * 128 + half * 64 + (lc & 63))
                            : ((lc >> 5) * 64 + half * 32 + (lc & 31));
      src = P + (int64_t)(k0 + kr) * ld + r0 + gcol;
    }
    dma16(src, lds_addr(lds + piece * 1024));
  }
}

template <bool A_KC, bool B_KC, int EPI, bool F8 = false>
__global__ __launch_bounds__(NT2, 1) void gemm256s_kernel(GemmArgs g) {
  // F8: A / B are e4m3 [rows][K8] passed as bf16 [rows][K8/2] (same bytes: the LDS images and
  // LDS-DMA of the bf16 schedule move exactly the right bytes); each phase issues 8 block-scaled
  // 16x16x128 MFMAs (same MFMA cycles as the 16 bf16 16x16x32 ones, 2x the FLOPs)
  static_assert(!F8 || (A_KC && B_KC), "fp8 operands are K-major");
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE2];   // [stage][A_h0|A_h1|B_h0|B_h1]
  int tm, tn;
  tile_coords2(blockIdx.x, g.M, g.N, tm, tn);
  const int m0 = tm * BM2, n0 = tn * BN2;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = g.K / BK, nph = 4 * nk;
  // stream part: 0 = A_h0, 1 = B_h0, 2 = B_h1, 3 = A_h1 ; slot offsets inside a 64-KiB stage
  auto issue = [&](int T, int part) {
    char* st = smem + (T & 1) * 2 * TILE2;
    if (part == 0) dma_half<A_KC, true>(st, g.A, g.lda, g.M, m0, T * BK, 0, wid, lane);
    if (part == 3) dma_half<A_KC, true>(st + HALF, g.A, g.lda, g.M, m0, T * BK, 1, wid, lane);
    if (part == 1) dma_half<B_KC, false>(st + 2 * HALF, g.B, g.ldb, g.N, n0, T * BK, 0, wid, lane);
    if (part == 2) dma_half<B_KC, false>(st + 3 * HALF, g.B, g.ldb, g.N, n0, T * BK, 1, wid, lane);
  };
  const int pro = min(6, nph);           // nph % 4 == 0: pro is 4 or 6 half-tiles
  for (int h = 0; h < pro; ++h) issue(h >> 2, h & 3);
  // retire half-tiles 0, 1, 2 (2 DMA instructions per wave each); leave the rest in flight
  if (pro == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // phase reads: 0: A_h0 + B_h0 | 1: B_h1 | 2: A_h1 (into the A_h0 registers) | 3: none
  bf16x8 af[4][2], bl[2][2], bh[2][2];
  i32x8 af8[4], bl8[2], bh8[2];          // F8: the two k-steps' chunks as one e4m3 operand
  for (int t = 0; t < nk; ++t) {
    const char* st = smem + (t & 1) * 2 * TILE2;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int k = 4 * t + p;
      if (p == 0 || p == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if constexpr (F8) {
            const char* base = st + (p == 0 ? 0 : HALF);
            af8[i] = cat_fp8(read_frag<A_KC>(base, wr * 64 + i * 16, 0, lane),
                             read_frag<A_KC>(base, wr * 64 + i * 16, 1, lane));
          } else {
#pragma unroll
            for (int s = 0; s < 2; ++s)
              af[i][s] = read_frag<A_KC>(st + (p == 0 ? 0 : HALF), wr * 64 + i * 16, s, lane);
          }
        }
      }
      if (p == 0 || p == 1) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if constexpr (F8) {
            const char* base = st + (p == 0 ? 2 : 3) * HALF;
            const i32x8 f = cat_fp8(read_frag<B_KC>(base, wc * 32 + j * 16, 0, lane),
                                    read_frag<B_KC>(base, wc * 32 + j * 16, 1, lane));
            if (p == 0) bl8[j] = f; else bh8[j] = f;
          } else {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
              const bf16x8 f = read_frag<B_KC>(st + (p == 0 ? 2 : 3) * HALF, wc * 32 + j * 16, s, lane);
              if (p == 0) bl[j][s] = f; else bh[j][s] = f;
            }
          }
        }
      }
      if (k + 6 < nph) issue(t + 1 + ((p + 2) >> 2), (p + 2) & 3);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
      if constexpr (F8) {
        // pin the cluster between its barriers: hipcc otherwise hoists the (register-only)
        // scaled MFMAs across them; the empty asm statements make the operands "defined" after
        // the lgkmcnt wait and the accumulators "used" before the vmcnt wait
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(af8[i]));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (p & 1) asm volatile("" : "+v"(bh8[j]));
          else asm volatile("" : "+v"(bl8[j]));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int ai = (p >> 1) * 4 + i, bj = (p & 1) * 2 + j;
            acc[ai][bj] = mfma_fp8((p & 1) ? bh8[j] : bl8[j], af8[i], acc[ai][bj]);
          }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[(p >> 1) * 4 + i][(p & 1) * 2 + j]));
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
              const int ai = (p >> 1) * 4 + i, bj = (p & 1) * 2 + j;
              acc[ai][bj] = mfma16((p & 1) ? bh[j][s] : bl[j][s], af[i][s], acc[ai][bj]);
            }
      }
      __builtin_amdgcn_s_setprio(0);
      const int out = nph - 4 - k;          // half-tiles allowed in flight after this phase
      if (out >= 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if (out == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (out == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wr * 128 + i * 16 + (lane & 15);
    if (m >= g.M) continue;
    const float s_m = F8 ? g.sa[m] : 1.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wc * 64 + j * 16 + 4 * (lane >> 4);
      if (n >= g.N) continue;
      f32x4 v = acc[i][j];
      if constexpr (F8) {
        const f32x4 s_n = *(const f32x4*)(g.sb + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] * (s_m * s_n[r]);
      }
      epilogue_tile<A_KC, B_KC, EPI>(g, v, m, n);
    }
  }
}

// ------------------------------------------------- 256x256, four waves, one wave per SIMD ---
// The 256x256 tile on 4 waves (2 x 2), each wave 128x128 = 8x8 MFMA 16x16x32 tiles: 256 fp32
// accumulators per lane (the AGPR half of the 512-entry register file at one wave per SIMD) and
// half the LDS read bytes per MFMA of the 8-wave kernel (16 fragments feed 64 MFMAs).  With no
// partner wave on the SIMD, each wave overlaps its own fragment reads with its MFMAs: the
// fragments of K-slice j+1 (32 deep) are read while the 64 MFMAs of slice j run.
// K-slices of 32 land by LDS-DMA in a 4-slot ring (slot = A 16 KiB | B 16 KiB):
//   iteration j: counted vmcnt (own DMA of slice j+1 done) -> barrier M_j -> issue slice j+3
//   into slot (j+3)%4 = (j-1)%4 -> MFMAs of slice j || reads of slice j+1.
// RAW: slice j+1 is read only after M_j, which every wave passes after retiring its own part of
// it.  WAR: slot (j-1)%4 was last read (slice j-1's fragments) before iteration j-1's MFMAs
// consumed them, i.e. before every wave's M_j.  DMA latency budget: 3 slices (~3 x 1024 MFMA
// cycles) per slice.
// K-major slice image: [256 rows][32 k], 64-B rows, 16-B chunk c of row r at position
// c ^ ((r >> 2) & 2) (conflict-free for the 16x16x32 fragment read: the four row quads of a
// b128 lane group land on four different chunk columns).  MN-major slice image: two [32 k][128]
// halves with 256-B rows and the swz_mn granule swizzle of the 128 kernel.
constexpr int BK4 = 32, SLICE4 = 32768, HALF4 = 16384;

__device__ __forceinline__ int kc_pos(int row, int c) { return row * 64 + ((c ^ ((row >> 2) & 2)) << 4); }

// byte offset (from the operand's SRD base: the tile's first row for K-major, its first column
// for MN-major) of this lane's 16 B of piece i (< 4) of the wave's quarter of a slice at k0 = 0
template <bool KC>
__device__ __forceinline__ uint32_t piece_off4(int64_t ld, int wid, int lane, int i) {
  const int piece = wid * 4 + i;                       // 16 pieces of 1 KiB per operand
  if (KC) {          // 16 rows x 64 B per piece
    const int row = piece * 16 + (lane >> 2), pos = lane & 3;
    return (uint32_t)(row * ld * 2) + ((pos ^ ((row >> 2) & 2)) << 4);
  }
  // half piece>>3, 4 k-rows x 256 B per piece
  const int kr = (piece & 7) * 4 + (lane >> 4), pb = (lane & 15) << 4;
  const int lc = (pb ^ (swz_mn(kr) << 5)) >> 1;
  return (uint32_t)(kr * ld * 2) + (uint32_t)(((piece >> 3) * 128 + lc) * 2);
}

template <bool KC>
__device__ __forceinline__ bf16x8 read_frag4(const char* lds, int base, int lane) {
  if (KC) return *(const bf16x8*)(lds + kc_pos(base + (lane & 15), lane >> 4));
  return read_frag<false>(lds + (base >> 7) * 8192, base & 127, 0, lane);
}

// Epilogue of the four-wave kernel: lane owns rows mb + 16 i (i < 8) and columns nb + 16 j + r
// (j < 8, r < 4).  With one wave per SIMD nothing hides a load's latency, so (1) the per-column
// bias / gate values are loaded once per lane (not once per row block), and (2) the per-element
// inputs (fp32 / bf16 residual, fp32 accumulator, dGELU pre-activation) run EPI4_AHEAD row blocks
// ahead of their use, kept in registers as loaded (bf16 inputs are widened only at their use, so
// the prefetch is not drained by a conversion).  The main loop's fragment registers are dead
// here, which leaves room for (EPI4_AHEAD + 1) x 32 input VGPRs.  The in-place residual
// (res == C) stays correct: a row block is read before anything of it is written.  Same
// arithmetic, in the same order, as epilogue_tile (outputs bit-identical to the 128 kernel).
#ifndef EPI4_AHEAD
#define EPI4_AHEAD 2
#endif
// FULL (round 5): a tile whose 256 x 256 outputs are all in range, with 16-B aligned output rows
// and 8 / 16-B aligned bias / gate (every tile of the 720p / 480p shapes), takes an epilogue with
// no per-lane bounds test.  With the tests, every coefficient, residual and store sat in its own
// exec-masked block (s_cbranch_execz per fragment): the waitcnt pass could not count across them
// and drained vmcnt(0) at the joins, and each bias load (bf16, converted at once) was waited alone.
// FULL: one batch of coefficient loads, counted waits; GELU / dGELU / biased forward 1-4 % faster
// on the 720p shapes, the gated residual 0-2 % (profiles/r05_ab_gemm_full.txt).  Same arithmetic
// in the same order: bit-identical.
//
// Measured and dropped: the whole residual tile issued before the first store (row blocks 0-4 by
// LDS-DMA into the ring's 160 KiB, 5-7 into registers, one vmcnt(0), then no memory wait at all,
// since vmcnt also counts stores): bit-identical and no faster than FULL alone
// (profiles/r05_ab_gemm_stage.txt), so the residual's latency is not what the epilogue waits on.
//
// SH (EPI4_SHUFFLE, FULL tiles): the outputs leave through LDS.  In the MFMA layout a lane holds 4
// columns of one row, so every store instruction wrote 16 rows x 64 B: 16 half cache lines per
// instruction, and the per-CU store stream (not the residual loads, not the bandwidth) set the
// epilogue's time -- fp32 C alone cost 14 us per tile more than bf16 C, at 32 tiles as at 5 760
// (profiles/r05_gemm_epi_probe.txt).  SH writes each pass of 32 rows (two row blocks) of the
// wave's 128 columns into a wave-private LDS image (rows padded 16 B: conflict-free both ways) and
// reads it back row-major, so a store instruction writes 2 rows x 512 B (fp32) or 4 rows x 256 B
// (bf16): whole lines.  Per wave 25 KiB: [32 rows x 528 B] fp32 / bf16 C | [32 x 272 B] bf16 aux.
// Same values: bit-identical.
#ifndef EPI4_SHUFFLE
#define EPI4_SHUFFLE 1
#endif
constexpr int EPI4_WLDS = 32 * 528 + 32 * 272;    // 25 600 B of LDS per wave
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
template <int EPI, bool IN_BF16, bool FULL, bool SH = false>
__device__ __forceinline__ void epilogue4w(const GemmArgs& g, const f32x4 (&acc)[8][8], int mb, int nb,
                                           char* wl = nullptr) {
  static_assert(!SH || FULL, "the LDS shuffle serves whole tiles only");
  constexpr int AHEAD = EPI4_AHEAD;
  constexpr bool F32C = EPI == EPI_F32 || EPI == EPI_RESID;          // C is fp32
  constexpr bool HAS_AUX = EPI == EPI_GELU || EPI == EPI_RESID;
  constexpr int RSF = 528, RSB = 272, AUX0 = 32 * 528;              // SH image strides / aux offset
  constexpr bool HAS_IN = EPI == EPI_RESID || EPI == EPI_F32 || EPI == EPI_DGELU;
  constexpr bool HAS_BIAS = EPI != EPI_F32 && EPI != EPI_DGELU, HAS_GATE = EPI == EPI_RESID;
  using InT = typename std::conditional<IN_BF16, bf16x4, f32x4>::type;
  // FULL: the bias kept as loaded (bf16, widened at use, so the batch of loads is not drained
  // one by one by its conversion)
  f32x4 bias[8], gate[8];
  bf16x4 braw[8];
  const bool fbias = FULL && HAS_BIAS && g.bias;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    bias[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    gate[j] = (f32x4){1.f, 1.f, 1.f, 1.f};
    braw[j] = bf16x4{};
  }
  if (FULL) {                    // uniform tests only: one batch of vector loads
    if (fbias) {
#pragma unroll
      for (int j = 0; j < 8; ++j) braw[j] = *(const bf16x4*)(g.bias + nb + 16 * j);
    }
    if (HAS_GATE && g.gate) {
#pragma unroll
      for (int j = 0; j < 8; ++j) gate[j] = *(const f32x4*)(g.gate + nb + 16 * j);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = nb + 16 * j;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bias[j][r] = (HAS_BIAS && g.bias && n < g.N) ? bf2f(g.bias[n + r]) : 0.f;
        gate[j][r] = (HAS_GATE && g.gate && n < g.N) ? g.gate[n + r] : 1.f;
      }
    }
  }
  const void* src = EPI == EPI_F32 ? (const void*)g.C : EPI == EPI_DGELU ? (const void*)g.aux : g.res;
  const int64_t lds_in = EPI == EPI_F32 ? g.ldc : EPI == EPI_DGELU ? g.ldaux : g.ldr;
  const bool any_in = HAS_IN && (EPI != EPI_F32 || g.accumulate);
  auto load_in = [&](int i, InT (&in)[8]) {
    const int m = mb + 16 * i;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = nb + 16 * j;
      in[j] = InT{};
      if (!any_in || (!FULL && (m >= g.M || n >= g.N))) continue;
      in[j] = *(const InT*)((const char*)src + ((int64_t)m * lds_in + n) * sizeof(in[j][0]));
    }
  };
  auto widen = [](InT x) {
    f32x4 f;
#pragma unroll
    for (int r = 0; r < 4; ++r) f[r] = (float)x[r];
    return f;
  };
  InT buf[8][8];
  const int lane = threadIdx.x & 63;
  if (HAS_IN) {
#pragma unroll
    for (int i = 0; i < AHEAD; ++i) load_in(i, buf[i]);
  }
  // bf16 outputs of fragments j, j+1 leave as ONE 16-B store per lane (MI355X guide T21, with
  // v_permlane16_swap: lane group g holds columns 4g..4g+3 of a 16-column fragment; swapping
  // groups 1 <-> 0 and 3 <-> 2 between the two fragments gives every lane 8 contiguous columns,
  // at column offset 16 (g & 1) + 8 (g >> 1) of the pair) when the wave's 128 columns are in
  // range and the rows 16-B aligned; else the two 8-B stores as computed
  const int gq = lane >> 4, nw = nb - 4 * gq;
  const int woff = 16 * (gq & 1) + 8 * (gq >> 1);
  const bool cols_in = nw + 128 <= g.N;
  const bool wide_c = FULL || (cols_in && (g.ldc % 8) == 0 && (((uintptr_t)g.C) & 15) == 0);
  const bool wide_x = FULL || (cols_in && (g.ldaux % 8) == 0 && (((uintptr_t)g.aux) & 15) == 0);
  auto st_pair = [&](bf16* base, int64_t ld, bool wide, int m, int j, bf16x4 a, bf16x4 b) {
    bf16* row = base + (int64_t)m * ld;
    if (wide) {
      const u32x2 ua = __builtin_bit_cast(u32x2, a), ub = __builtin_bit_cast(u32x2, b);
      const auto r0 = __builtin_amdgcn_permlane16_swap(ua[0], ub[0], false, false);
      const auto r1 = __builtin_amdgcn_permlane16_swap(ua[1], ub[1], false, false);
      *(u32x4*)(row + nw + 16 * j + woff) = (u32x4){r0[0], r1[0], r0[1], r1[1]};
    } else {
      if (nb + 16 * j < g.N) *(bf16x4*)(row + nb + 16 * j) = a;
      if (nb + 16 * j + 16 < g.N) *(bf16x4*)(row + nb + 16 * j + 16) = b;
    }
  };
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (HAS_IN && i + AHEAD < 8) load_in(i + AHEAD, buf[i + AHEAD]);
    const int m = mb + 16 * i;
    if (FULL || m < g.M) {
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        bf16x4 oc[2], ox[2];          // bf16 results for C / aux of fragments j, j + 1
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int jj = j + h, n = nb + 16 * jj;
          const f32x4 v = acc[i][jj];
          if (EPI == EPI_F32) {
            const f32x4 o = g.accumulate ? v + widen(buf[i][jj]) : v;
            if (SH) *(f32x4*)(wl + ((i & 1) * 16 + (lane & 15)) * RSF + (16 * jj + 4 * gq) * 4) = o;
            else if (FULL || n < g.N) *(f32x4*)((float*)g.C + (int64_t)m * g.ldc + n) = o;
          } else if (EPI == EPI_DGELU) {
            const f32x4 pre = widen(buf[i][jj]);
#pragma unroll
            for (int r = 0; r < 4; ++r) oc[h][r] = f2bf(bfr(v[r]) * gelu_tanh_grad(pre[r]));
          } else {
            float y[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) y[r] = bfr(v[r] + (FULL ? (float)braw[jj][r] : bias[jj][r]));
            if (EPI == EPI_BF16) {
#pragma unroll
              for (int r = 0; r < 4; ++r) oc[h][r] = f2bf(y[r]);
            } else if (EPI == EPI_GELU) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                ox[h][r] = f2bf(y[r]);
                oc[h][r] = f2bf(gelu_tanh(y[r]));
              }
            } else {    // EPI_RESID: x + y*gate (two roundings, as torch)
#pragma unroll
              for (int r = 0; r < 4; ++r) ox[h][r] = f2bf(y[r]);
              const f32x4 res = widen(buf[i][jj]);
              f32x4 o;
#pragma unroll
              for (int r = 0; r < 4; ++r) o[r] = res[r] + mul_rn(y[r], gate[jj][r]);
              if (SH) *(f32x4*)(wl + ((i & 1) * 16 + (lane & 15)) * RSF + (16 * jj + 4 * gq) * 4) = o;
              else if (FULL || n < g.N) *(f32x4*)((float*)g.C + (int64_t)m * g.ldc + n) = o;
            }
          }
          if (SH) {          // bf16 C / aux of this fragment into the pass image
            const int rr = (i & 1) * 16 + (lane & 15), cb = (16 * jj + 4 * gq) * 2;
            if (!F32C) *(bf16x4*)(wl + rr * RSB + cb) = oc[h];
            if (HAS_AUX && g.aux) *(bf16x4*)(wl + AUX0 + rr * RSB + cb) = ox[h];
          }
        }
        if (!SH) {
          if (EPI == EPI_BF16 || EPI == EPI_GELU || EPI == EPI_DGELU)
            st_pair((bf16*)g.C, g.ldc, wide_c, m, j, oc[0], oc[1]);
          if ((EPI == EPI_GELU || EPI == EPI_RESID) && g.aux)
            st_pair(g.aux, g.ldaux, wide_x, m, j, ox[0], ox[1]);
        }
      }
    }
    if (SH && (i & 1)) {     // the pass's 32 rows leave row-major: whole cache lines per store
      wave_lds_sync();
      const int64_t r0 = (int64_t)(mb - (lane & 15)) + 16 * (i - 1);   // first row of the pass
      const int c0 = nb - 4 * gq;                                         // the wave's first column
      if (F32C) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int row = 2 * k + (lane >> 5), c4 = lane & 31;
          const f32x4 o = *(const f32x4*)(wl + row * RSF + c4 * 16);
          *(f32x4*)((float*)g.C + (r0 + row) * g.ldc + c0 + 4 * c4) = o;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int row = 4 * k + (lane >> 4), c8 = lane & 15;
          const u32x4 o = *(const u32x4*)(wl + row * RSB + c8 * 16);
          *(u32x4*)((bf16*)g.C + (r0 + row) * g.ldc + c0 + 8 * c8) = o;
        }
      }
      if (HAS_AUX && g.aux) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int row = 4 * k + (lane >> 4), c8 = lane & 15;
          const u32x4 o = *(const u32x4*)(wl + AUX0 + row * RSB + c8 * 16);
          *(u32x4*)(g.aux + (r0 + row) * g.ldaux + c0 + 8 * c8) = o;
        }
      }
      wave_lds_sync();       // the next pass rewrites the image
    }
  }
}

// the FULL epilogue's preconditions (uniform per workgroup): the whole 256 x 256 tile in range and
// every vector access of the FULL path aligned
__device__ __forceinline__ bool epi4_full(const GemmArgs& g, int m0, int n0, int epi) {
  const bool bf16_c = epi == EPI_BF16 || epi == EPI_GELU || epi == EPI_DGELU;
  return m0 + 256 <= g.M && n0 + 256 <= g.N &&
         (!bf16_c || ((g.ldc % 8) == 0 && (((uintptr_t)g.C) & 15) == 0)) &&
         (!g.aux || ((g.ldaux % 8) == 0 && (((uintptr_t)g.aux) & 15) == 0)) &&
         (!g.bias || (((uintptr_t)g.bias) & 7) == 0) && (!g.gate || (((uintptr_t)g.gate) & 15) == 0);
}

#ifndef GEMM4_PREWAIT
#define GEMM4_PREWAIT 1
#endif
// 1: every non-MFMA instruction of the four-wave loop between two MFMAs, as hipBLASLt's TN
// loop places them (one LDS-DMA piece after MFMA 0, the A / B fragment reads after MFMAs 1 / 2 of
// each 8-MFMA chunk) instead of a [piece, reads, 8 MFMAs] burst: bit-identical, forward +0.2-1.7 %,
// dX +1.1-6.7 % on the 720p shapes (profiles/r04_ab_gemm_il.txt)
#ifndef GEMM4_IL
#define GEMM4_IL 1
#endif
// the same placement in the 32x32x16 weight-gradient kernel: dW +5.3-9.5 %, bit-identical
// (profiles/r04_ab_gemm4x_il.txt)
#ifndef GEMM4X_IL
#define GEMM4X_IL 1
#endif
// AGPR-accumulator MFMA as inline asm ("+a" keeps hipcc from moving the accumulators to VGPRs)
__device__ __forceinline__ void mfma16(f32x4& acc, bf16x8 b, bf16x8 a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

// A64: a K-major A operand staged 64 deep.  A 32-deep K-major slice moves each A row as a 64-B
// run (one LDS-DMA piece = 16 rows x 64 B = 16 half cache lines); staged 64 deep, a piece is 8
// rows x 128 B = 8 whole lines, as hipBLASLt's MT256x256x64 TN loop fetches its operands.  The A
// operand gets its own ring of three 64-deep slots (3 x 32 KiB) beside the B operand's ring of
// four 32-deep slots (4 x 16 KiB): exactly the 160 KiB of LDS.  The 32-deep step schedule is
// unchanged (one barrier per 32-deep sub-slice, fragments of sub-slice j+1 read during the MFMAs
// of sub-slice j, 8 DMA pieces per wave per step, vmcnt(8)); A slice J (sub-slices 2J, 2J+1) is
// issued half per step in steps 2J-4 and 2J-3 into slot J % 3, whose previous slice J-3 was last
// read in step 2J-6, and it is retired by the vmcnt(8) + barrier at the top of step 2J-1, the
// first that reads it.  Same MFMAs in the same k order: outputs bit-identical.
// A 64-deep slot image: row r (0..255) at r * 128 B, 16-B chunk c (k 8c..8c+7) at c ^ (r & 7)
// (the 128 kernel's conflict-free K-major layout).
#ifndef GEMM4_A64
#define GEMM4_A64 1
#endif
constexpr int A64SLOT = 32768;
// diagnostic builds only (wrong results): the A64 loop without its barrier (1), its LDS-DMA and
// vmcnt waits (2), its fragment reads (4), its vmcnt waits only (8)
// (Measured and dropped: B fragments of the next sub-slice read in the step's first half, A in its
// second -- chunk 0 of a step consumes every B fragment -- tied or lost up to 2 %,
// profiles/r05_ab_gemm_rorder.txt.)
// (Measured and dropped, profiles/r05_ab_gemm_dpos.txt: each wave issuing its LDS-DMA piece at a
// different MFMA gap of the chunk -- after MFMA {0, 3, 5, 7}[wave] or 2 x wave -- so the four
// waves' pieces do not reach the texture-address unit together: 0.5-2.5 % slower.  A build without
// the DMA runs 14 % faster and one without its vmcnt waits no faster (profiles/r05_ab_gemm_diag.txt):
// what the pieces cost is neither the data's arrival nor the four waves' collision.  Moving every
// wave's piece to MFMA gap 3, 5 or 7 of the chunk ties within 0.5 %, profiles/r05_ab_gemm_dgap.txt.
// Also measured and dropped: the TN forward with B staged 64 deep too (hipBLASLt's operand format,
// one ds_read_b128 per B fragment; A's three 64-deep slots + B's two fill the 160 KiB, so a B slice
// has one step to land instead of two): bit-identical, 4-8 % SLOWER than the 32-deep forms,
// profiles/r05_ab_gemm_b64.txt.)
#ifndef GEMM4_DIAG
#define GEMM4_DIAG 0
#endif

// byte offset of this lane's 16 B in A piece i (< 4) of half 0 of the wave's 64 rows of a 64-deep
// slice at k0 = 0 (half 1 = rows + 32: the same lane offsets plus a wave-uniform soffset)
__device__ __forceinline__ uint32_t piece_off_a64(int64_t ld, int wid, int lane, int i) {
  const int row = (wid * 8 + i) * 8 + (lane >> 3), p = lane & 7;
  return (uint32_t)(row * ld * 2) + ((p ^ (row & 7)) << 4);
}

// 16x16x32 A fragment of half h (k 32h..32h+31) of a 64-deep slot: lane l gets row
// base + (l & 15), k = 32h + 8 (l >> 4) + 0..7
__device__ __forceinline__ bf16x8 read_frag_a64(const char* slot, int h, int base, int lane) {
  const int row = base + (lane & 15), kc = 4 * h + (lane >> 4);
  return *(const bf16x8*)(slot + row * 128 + ((kc ^ (row & 7)) << 4));
}

// Start stagger: all 256 first-wave workgroups start together, so every CU reaches its epilogue
// (the residual / pre-activation reads and the output writes) at the same moment and the chip's
// HBM serves 256 epilogues at once while every matrix pipe idles; the next wave inherits the same
// phase.  With GEMM4_STAGGER = S > 0 the first-wave workgroup of slot s = (bid >> 3) & 31 on its
// XCD first waits s/32 * S * K shader cycles (S ~ 54 cycles per K is one tile's main loop at
// 1.3 PF), so the CUs' epilogues fall at spread-out times from then on.  Grids of >= 2 waves only.
// Measured (one process, 720p shapes, profiles/r05_ab_gemm_stagger.txt): S = 7 gains 1-2.6 % on
// the o-projection shape, loses up to 2.1 % on FFN-down and dX, and the dW kernel (K = L) loses
// 10-17 % to the start delay; larger S lose more.  The epilogue's cost does not follow the
// chip-wide burst, so the stagger stays off
#ifndef GEMM4_STAGGER
#define GEMM4_STAGGER 0
#endif
__device__ __forceinline__ void gemm_start_stagger(int K) {
  if (GEMM4_STAGGER && blockIdx.x < 256 && gridDim.x >= 512) {
    const uint64_t wait = (uint64_t)((blockIdx.x >> 3) & 31) * (uint64_t)K * GEMM4_STAGGER / 32;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < wait) __builtin_amdgcn_s_sleep(4);
  }
}

template <bool A_KC, bool B_KC, int EPI>
__global__ __launch_bounds__(256, 1) void gemm4w_kernel(GemmArgs g) {
  constexpr bool A64 = A_KC && GEMM4_A64;
  __shared__ __attribute__((aligned(16))) char smem[A64 ? 3 * A64SLOT + 4 * HALF4 : 4 * SLICE4];
  char* const smB = smem + 3 * A64SLOT;      // A64: the B ring (4 x 16 KiB) after the A ring
  gemm_start_stagger(g.K);
  int tm, tn;
  tile_coords2(blockIdx.x, g.M, g.N, tm, tn);
  const int m0 = tm * BM2, n0 = tn * BN2;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // ns = K / 32 is even and >= 4 (host check).  Branch-free body: past the last slice the DMA
  // re-fetches slice ns-1 into the free slot and the reads fetch fragments nobody uses, so every
  // iteration issues the same 8 DMA instructions per wave and `vmcnt(8)` is always the count
  const int ns = g.K / BK4;
  // operand SRDs (host guarantees every byte offset fits 32 bits); K-major rows past the
  // operand's end are out of the SRD's range and load zeros
  const i32x4 srd_a = A_KC ? make_srd(g.A + (int64_t)m0 * g.lda, (uint32_t)((int64_t)(g.M - m0) * g.lda * 2))
                           : make_srd(g.A + m0, (uint32_t)((int64_t)g.K * g.lda * 2 - (int64_t)m0 * 2));
  const i32x4 srd_b = B_KC ? make_srd(g.B + (int64_t)n0 * g.ldb, (uint32_t)((int64_t)(g.N - n0) * g.ldb * 2))
                           : make_srd(g.B + n0, (uint32_t)((int64_t)g.K * g.ldb * 2 - (int64_t)n0 * 2));
  // DMA pieces: the wave's 4 pieces of an operand are consecutive KiB of LDS, so one m0 (the
  // first piece's LDS address) serves all four, piece i adding i KiB through the instruction
  // offset; that offset also adds to the global address, so it is pre-subtracted from the per-lane
  // offsets (never below zero: K-major ld >= K >= 128, MN-major ld >= 256 under fits256).
  // One m0 write per 4 pieces instead of a save / set / nop / restore per piece: dX +3-7 %,
  // forward +0.2-2.8 %, bit-identical (profiles/r03_gemm_m0group_ab.txt)
  uint32_t offa[4], offb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    offa[i] = (A64 ? piece_off_a64(g.lda, wid, lane, i) : piece_off4<A_KC>(g.lda, wid, lane, i)) - i * 1024;
    offb[i] = piece_off4<B_KC>(g.ldb, wid, lane, i) - i * 1024;
  }
  unsigned m0keep = 0;
  // k0 -> soffset: 2 B per k for K-major operands, one row (ld elements) per k for MN-major
  auto soff_a = [&](int j) { return (uint32_t)(A_KC ? j * BK4 * 2 : (int64_t)j * BK4 * g.lda * 2); };
  auto soff_b = [&](int j) { return (uint32_t)(B_KC ? j * BK4 * 2 : (int64_t)j * BK4 * g.ldb * 2); };
  // A64: piece i (< 4) of half hh of 64-deep A slice J into the A slot at sa; B piece i (< 4) of
  // 32-deep sub-slice j into the B slot at sb
  auto piece_a64 = [&](int i, int J, int hh, char* sa) {
    if (i == 0) m0_set(lds_addr(sa + wid * 8192 + hh * 4096), m0keep);
    dma16_buf_m0(srd_a, offa[i], (uint32_t)(J * 128 + (int64_t)hh * 32 * g.lda * 2), i);
    if (i == 3) m0_restore(m0keep);
  };
  auto piece_b = [&](int i, int j, char* sb) {
    if (i == 0) m0_set(lds_addr(sb + wid * 4096), m0keep);
    dma16_buf_m0(srd_b, offb[i], soff_b(j), i);
    if (i == 3) m0_restore(m0keep);
  };
  // piece i (< 8: A pieces 0-3, B pieces 4-7) of slice j into ring slot sd
  auto piece = [&](int i, int j, char* sd) {
    if (i == 0 || i == 4) m0_set(lds_addr(sd + (i ? HALF4 : 0) + wid * 4096), m0keep);
    if (i < 4) dma16_buf_m0(srd_a, offa[i], soff_a(j), i);
    else dma16_buf_m0(srd_b, offb[i - 4], soff_b(j), i - 4);
    if (i == 3 || i == 7) m0_restore(m0keep);
  };
  auto issue = [&](int j) {
    j = min(j, ns - 1);
#pragma unroll
    for (int i = 0; i < 8; ++i) piece(i, j, smem + (j & 3) * SLICE4);
  };
  auto read = [&](int j, bf16x8 (&af)[8], bf16x8 (&bf)[8]) {
    const char* st = smem + (j & 3) * SLICE4;
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = read_frag4<A_KC>(st, wm * 128 + i * 16, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) bf[i] = read_frag4<B_KC>(st + HALF4, wn * 128 + i * 16, lane);
  };
  auto step = [&](int j, bf16x8 (&ca)[8], bf16x8 (&cb)[8], bf16x8 (&na)[8], bf16x8 (&nb)[8]) {
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // own part of slice j+1 landed
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int jd = min(j + 3, ns - 1);
    char* sd = smem + ((j + 3) & 3) * SLICE4;
    const char* st = smem + ((j + 1) & 3) * SLICE4;
    // eight chunks: row i's 8 MFMAs beside one LDS-DMA piece of slice j+3 and the reads of
    // fragments i of slice j+1, pinned in place by sched_barrier so the non-MFMA work spreads
    // over the slice (one wave per SIMD: nothing else fills the matrix pipe)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (GEMM4_IL == 2) {    // the slice's 8 pieces in its first half, two per chunk
        mfma16(acc[i][0], cb[0], ca[i]);
        if (i < 4) piece(2 * i, jd, sd);
        mfma16(acc[i][1], cb[1], ca[i]);
        if (i < 4) piece(2 * i + 1, jd, sd);
        mfma16(acc[i][2], cb[2], ca[i]);
        __builtin_amdgcn_sched_barrier(0);
        na[i] = read_frag4<A_KC>(st, wm * 128 + i * 16, lane);
        __builtin_amdgcn_sched_barrier(0);
        mfma16(acc[i][3], cb[3], ca[i]);
        __builtin_amdgcn_sched_barrier(0);
        nb[i] = read_frag4<B_KC>(st + HALF4, wn * 128 + i * 16, lane);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int jj = 4; jj < 8; ++jj) mfma16(acc[i][jj], cb[jj], ca[i]);
        __builtin_amdgcn_sched_barrier(0);
        continue;
      }
      if (GEMM4_IL) {
        // hipBLASLt's placement (its TN loop, disassembled): every non-MFMA instruction sits
        // BETWEEN two MFMAs, so the matrix pipe has the next product queued behind it
        mfma16(acc[i][0], cb[0], ca[i]);
        piece(i, jd, sd);
        mfma16(acc[i][1], cb[1], ca[i]);
        __builtin_amdgcn_sched_barrier(0);
        na[i] = read_frag4<A_KC>(st, wm * 128 + i * 16, lane);
        __builtin_amdgcn_sched_barrier(0);
        mfma16(acc[i][2], cb[2], ca[i]);
        __builtin_amdgcn_sched_barrier(0);
        nb[i] = read_frag4<B_KC>(st + HALF4, wn * 128 + i * 16, lane);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int jj = 3; jj < 8; ++jj) mfma16(acc[i][jj], cb[jj], ca[i]);
        __builtin_amdgcn_sched_barrier(0);
        continue;
      }
      piece(i, jd, sd);
      na[i] = read_frag4<A_KC>(st, wm * 128 + i * 16, lane);
      nb[i] = read_frag4<B_KC>(st + HALF4, wn * 128 + i * 16, lane);
#pragma unroll
      for (int jj = 0; jj < 8; ++jj)   // AGPR accumulators: the MFMA as inline asm ("+a") keeps
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"   // hipcc from switching them to
                     : "+a"(acc[i][jj]) : "v"(cb[jj]), "v"(ca[i]));   // VGPRs and spilling
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // A64 step j: MFMAs of sub-slice j || reads of sub-slice j+1 (A: half hr of the slot at ra; B:
  // slot (j+1) & 3) || DMA of half hh of A slice J into the slot at sa and of B sub-slice j+3
  auto step64 = [&](int j, bf16x8 (&ca)[8], bf16x8 (&cb)[8], bf16x8 (&na)[8], bf16x8 (&nb)[8],
                    char* sa, int J, int hh, const char* ra, int hr) {
    if (!(GEMM4_DIAG & 10)) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // own pieces of sub-slice j+1 landed
    if (!(GEMM4_DIAG & 1)) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int jb = min(j + 3, ns - 1);
    char* sb = smB + ((j + 3) & 3) * HALF4;
    const char* rb = smB + ((j + 1) & 3) * HALF4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      mfma16(acc[i][0], cb[0], ca[i]);
      if (!(GEMM4_DIAG & 2)) {
        if (i < 4) piece_a64(i, J, hh, sa);
        else piece_b(i - 4, jb, sb);
      }
      mfma16(acc[i][1], cb[1], ca[i]);
      __builtin_amdgcn_sched_barrier(0);
      na[i] = (GEMM4_DIAG & 4) ? ca[i] : read_frag_a64(ra, hr, wm * 128 + i * 16, lane);
      __builtin_amdgcn_sched_barrier(0);
      mfma16(acc[i][2], cb[2], ca[i]);
      __builtin_amdgcn_sched_barrier(0);
      nb[i] = (GEMM4_DIAG & 4) ? cb[i] : read_frag4<B_KC>(rb, wn * 128 + i * 16, lane);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int jj = 3; jj < 8; ++jj) mfma16(acc[i][jj], cb[jj], ca[i]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  asm volatile("s_nop 7" ::: "memory");    // accumulator zeroing (VALU) -> first asm MFMA
  bf16x8 fa[8], fb[8], ga[8], gb[8];
  if constexpr (A64) {
    // prologue: A slice 0, B 0, B 1, A slice 1, B 2; retire A 0 + B 0 (the last 16 pieces stay
    // in flight) and read sub-slice 0
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int i = 0; i < 4; ++i) piece_a64(i, 0, hh, smem);
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int i = 0; i < 4; ++i) piece_b(i, jb, smB + jb * HALF4);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int i = 0; i < 4; ++i) piece_a64(i, 1, hh, smem + A64SLOT);
#pragma unroll
    for (int i = 0; i < 4; ++i) piece_b(i, 2, smB + 2 * HALF4);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      fa[i] = read_frag_a64(smem, 0, wm * 128 + i * 16, lane);
      fb[i] = read_frag4<B_KC>(smB, wn * 128 + i * 16, lane);
    }
    if (GEMM4_PREWAIT) __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
    // A slots of A slices q, q+1, q+2 (q = j / 2), rotated every two steps
    int s0 = 0, s1 = A64SLOT, s2 = 2 * A64SLOT;
    const int nA = ns >> 1;
    for (int j = 0; j < ns; j += 2) {
      const int J = min((j >> 1) + 2, nA - 1);   // past the end: re-fetch the last slice
      step64(j, fa, fb, ga, gb, smem + s2, J, 0, smem + s0, 1);
      step64(j + 1, ga, gb, fa, fb, smem + s2, J, 1, smem + s1, 0);
      const int t = s0;
      s0 = s1;
      s1 = s2;
      s2 = t;
    }
  } else {
  issue(0);
  issue(1);
  issue(2);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  read(0, fa, fb);
  // GEMM4_PREWAIT: retire every LDS / scalar load before the loop with a wait the compiler's
  // waitcnt pass sees (the builtin, not asm): else a kernel-argument load still in flight from
  // the preheader (scalar loads complete out of order) made the pass drain every LDS read
  // (lgkmcnt(0)) before the first MFMA of every other slice.  Measured neutral (+-0.5 %,
  // bit-identical: profiles/r04_gemm_lgkm_ab.txt) -- that drain was not a stall; kept as the
  // cleaner loop
  if (GEMM4_PREWAIT) __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
  for (int j = 0; j < ns; j += 2) {
    step(j, fa, fb, ga, gb);
    step(j + 1, ga, gb, fa, fb);
  }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // the MFMAs are inline asm: the compiler does not see their AGPR writes, so pad the
  // MFMA-write -> v_accvgpr_read distance by hand before the epilogue
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  const int mb = m0 + wm * 128 + (lane & 15), nb = n0 + wn * 128 + 4 * (lane >> 4);
  const bool full = epi4_full(g, m0, n0, EPI);
  // the shuffle where it measured faster: the fp32 gated residual (2-3 % over FULL) and dGELU
  // (0.3-1 %); GELU's two bf16 outputs and the fp32 C without input ran slower through it, the
  // plain bf16 C tied (profiles/r05_ab_gemm_sh.txt, r05_gemm_epi_probe.txt)
  constexpr bool SH = EPI4_SHUFFLE && sizeof(smem) >= 4 * EPI4_WLDS && (EPI == EPI_RESID || EPI == EPI_DGELU);
  if (SH && full) {          // the shuffle images reuse the ring: every wave's DMA has landed
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  char* const wl = smem + wid * EPI4_WLDS;
  if (EPI == EPI_DGELU || (EPI == EPI_RESID && g.res_bf16)) {
    if (full) epilogue4w<EPI, true, true, SH>(g, acc, mb, nb, wl);
    else epilogue4w<EPI, true, false>(g, acc, mb, nb);
  } else {
    if (full) epilogue4w<EPI, false, true, SH>(g, acc, mb, nb, wl);
    else epilogue4w<EPI, false, false>(g, acc, mb, nb);
  }
}

// ---------------------------------------- 256x256, four waves, MFMA 32x32x16 (gemm4x) -------
// gemm4w_kernel's tile, 4-slot ring, DMA schedule and one barrier per 32-deep K-slice, with each
// wave's 128x128 computed as 4 x 4 MFMA 32x32x16 tiles (32 MFMAs of 32 cycles per slice instead
// of 64 of 16): an MFMA holds the SIMD's vector issue for 8 cycles either way, so the slice's
// issue slots spent on MFMAs halve (512 -> 256 of 1024 cycles) and the eight LDS-DMA pieces
// and sixteen fragment reads no longer compete with the matrix pipe for issue (MI355X guide,
// constants table: vector-instruction issue cost).  Same operand bytes and LDS reads per MFMA
// FLOP.  Outputs are not bit-identical to the 16x16x32 kernels: one 32x32x16 MFMA rounds its
// accumulator after 16 products, a 16x16x32 one after 32.
// K-major slice image: [256 rows][32 k], 64-B rows, 16-B chunk c of row r at c ^ ((r >> 2) & 3)
// (every 16-lane quarter of a b128 read — 16 rows x one chunk column — lands on 16 distinct
// 16-B bank groups).  MN-major: two [32 k][128] halves, 256-B rows, 64-B chunk ^ (k & 3) (the 32
// lanes of a b64 transposed read — 4 k-rows x 32 columns — cover the 256-B bank window once).
__device__ __forceinline__ int kc_pos32(int row, int c) { return row * 64 + ((c ^ ((row >> 2) & 3)) << 4); }

template <bool KC>
__device__ __forceinline__ uint32_t piece_off32(int64_t ld, int wid, int lane, int i) {
  const int piece = wid * 4 + i;                       // 16 pieces of 1 KiB per operand
  if (KC) {          // 16 rows x 64 B per piece: LDS slot (row, pos) <- global chunk pos ^ swz(row)
    const int row = piece * 16 + (lane >> 2), pos = lane & 3;
    return (uint32_t)(row * ld * 2) + ((pos ^ ((row >> 2) & 3)) << 4);
  }
  // half piece>>3, 4 k-rows x 256 B per piece: LDS byte pb of row kr <- column byte pb ^ 64 (kr & 3)
  const int kr = (piece & 7) * 4 + (lane >> 4), pb = (lane & 15) << 4;
  const int lc = (pb ^ ((kr & 3) << 6)) >> 1;
  return (uint32_t)(kr * ld * 2) + (uint32_t)(((piece >> 3) * 128 + lc) * 2);
}

// MFMA 32x32x16 operand of k-step s (16 k) of a slice: lane l gets row `base + (l & 31)` at
// k = 16 s + 8 (l >> 5) + 0..7 (the A and the B operand have the same form).
template <bool KC>
__device__ __forceinline__ bf16x8 read_frag32(const char* lds, int base, int s, int lane) {
  if (KC) return *(const bf16x8*)(lds + kc_pos32(base + (lane & 31), 2 * s + (lane >> 5)));
  const char* h = lds + (base >> 7) * 8192;
  const int g = lane >> 4, l16 = lane & 15, q = l16 >> 2, p = l16 & 3;
  const int cb = ((base & 127) + 16 * (g & 1) + 4 * p) * 2;
  const int k0 = 16 * s + 8 * (g >> 1) + q, k1 = k0 + 4;
  return cat8(lds_read_tr(h + k0 * 256 + (cb ^ ((k0 & 3) << 6))),
              lds_read_tr(h + k1 * 256 + (cb ^ ((k1 & 3) << 6))));
}

// Epilogue of gemm4x: the 16 (row block i, column tile jj) pieces in turn, each 4 column vectors
// (register group q of acc[i][jj]: columns 32 jj + 8 q + 0..3 of the lane's group, rows 32 i +
// (lane & 31)); per piece the per-element inputs and the bias / gate of its columns are loaded one
// piece ahead.  Same arithmetic, in the same order, as epilogue_tile.
template <int EPI, bool IN_BF16>
__device__ __forceinline__ void epilogue4x(const GemmArgs& g, const f32x16 (&acc)[4][4], int mb, int nb) {
  constexpr bool HAS_IN = EPI == EPI_RESID || EPI == EPI_F32 || EPI == EPI_DGELU;
  using InT = typename std::conditional<IN_BF16, bf16x4, f32x4>::type;
  const void* src = EPI == EPI_F32 ? (const void*)g.C : EPI == EPI_DGELU ? (const void*)g.aux : g.res;
  const int64_t lds_in = EPI == EPI_F32 ? g.ldc : EPI == EPI_DGELU ? g.ldaux : g.ldr;
  const bool any_in = HAS_IN && (EPI != EPI_F32 || g.accumulate);
  struct Piece { InT in[4]; f32x4 bias[4], gate[4]; };
  auto load = [&](int b, Piece& p) {
    const int m = mb + 32 * (b >> 2);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = nb + 32 * (b & 3) + 8 * q;
      p.in[q] = InT{};
      p.bias[q] = (f32x4){0.f, 0.f, 0.f, 0.f};
      p.gate[q] = (f32x4){1.f, 1.f, 1.f, 1.f};
      if (n >= g.N) continue;
      if (EPI != EPI_F32 && EPI != EPI_DGELU && g.bias) {
        const bf16x4 bb = *(const bf16x4*)(g.bias + n);
        p.bias[q] = (f32x4){bf2f(bb[0]), bf2f(bb[1]), bf2f(bb[2]), bf2f(bb[3])};
      }
      if (EPI == EPI_RESID && g.gate) p.gate[q] = *(const f32x4*)(g.gate + n);
      if (any_in && m < g.M)
        p.in[q] = *(const InT*)((const char*)src + ((int64_t)m * lds_in + n) * sizeof(p.in[q][0]));
    }
  };
  auto widen = [](InT x) {
    f32x4 f;
#pragma unroll
    for (int r = 0; r < 4; ++r) f[r] = (float)x[r];
    return f;
  };
  Piece cur, nxt;
  load(0, cur);
#pragma unroll
  for (int b = 0; b < 16; ++b) {
    __builtin_amdgcn_sched_barrier(0);
    if (b + 1 < 16) load(b + 1, nxt);
    const int m = mb + 32 * (b >> 2);
    if (m < g.M) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = nb + 32 * (b & 3) + 8 * q;
        if (n >= g.N) continue;
        const f32x16& t = acc[b >> 2][b & 3];
        const f32x4 v = {t[4 * q], t[4 * q + 1], t[4 * q + 2], t[4 * q + 3]};
        if (EPI == EPI_F32) {   // in = 0 unless accumulating: one branch-free form (-0 -> +0)
          *(f32x4*)((float*)g.C + (int64_t)m * g.ldc + n) = v + widen(cur.in[q]);
        } else if (EPI == EPI_DGELU) {
          const f32x4 pre = widen(cur.in[q]);
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bf(bfr(v[r]) * gelu_tanh_grad(pre[r]));
          *(bf16x4*)((bf16*)g.C + (int64_t)m * g.ldc + n) = o;
        } else {
          float y[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) y[r] = bfr(v[r] + cur.bias[q][r]);
          if (EPI == EPI_BF16) {
            bf16x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = f2bf(y[r]);
            *(bf16x4*)((bf16*)g.C + (int64_t)m * g.ldc + n) = o;
          } else if (EPI == EPI_GELU) {
            bf16x4 o, pre;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              pre[r] = f2bf(y[r]);
              o[r] = f2bf(gelu_tanh(y[r]));
            }
            if (g.aux) *(bf16x4*)(g.aux + (int64_t)m * g.ldaux + n) = pre;
            *(bf16x4*)((bf16*)g.C + (int64_t)m * g.ldc + n) = o;
          } else {    // EPI_RESID: x + y*gate (two roundings, as torch)
            if (g.aux) {
              bf16x4 yo;
#pragma unroll
              for (int r = 0; r < 4; ++r) yo[r] = f2bf(y[r]);
              *(bf16x4*)(g.aux + (int64_t)m * g.ldaux + n) = yo;
            }
            const f32x4 res = widen(cur.in[q]);
            f32x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = res[r] + mul_rn(y[r], cur.gate[q][r]);
            *(f32x4*)((float*)g.C + (int64_t)m * g.ldc + n) = o;
          }
        }
      }
    }
    cur = nxt;
  }
}

template <bool A_KC, bool B_KC, int EPI>
__global__ __launch_bounds__(256, 1) void gemm4x_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[4 * SLICE4];
  gemm_start_stagger(g.K);
  int tm, tn;
  tile_coords2(blockIdx.x, g.M, g.N, tm, tn);
  const int m0 = tm * BM2, n0 = tn * BN2;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;

  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // ring / DMA exactly as gemm4w_kernel (see there): ns = K / 32 even and >= 4 (host check)
  const int ns = g.K / BK4;
  const i32x4 srd_a = A_KC ? make_srd(g.A + (int64_t)m0 * g.lda, (uint32_t)((int64_t)(g.M - m0) * g.lda * 2))
                           : make_srd(g.A + m0, (uint32_t)((int64_t)g.K * g.lda * 2 - (int64_t)m0 * 2));
  const i32x4 srd_b = B_KC ? make_srd(g.B + (int64_t)n0 * g.ldb, (uint32_t)((int64_t)(g.N - n0) * g.ldb * 2))
                           : make_srd(g.B + n0, (uint32_t)((int64_t)g.K * g.ldb * 2 - (int64_t)n0 * 2));
  // grouped DMA pieces (one m0 per operand, piece i at instruction offset i KiB), as gemm4w_kernel
  uint32_t offa[4], offb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    offa[i] = piece_off32<A_KC>(g.lda, wid, lane, i) - i * 1024;
    offb[i] = piece_off32<B_KC>(g.ldb, wid, lane, i) - i * 1024;
  }
  unsigned m0keep = 0;
  auto soff_a = [&](int j) { return (uint32_t)(A_KC ? j * BK4 * 2 : (int64_t)j * BK4 * g.lda * 2); };
  auto soff_b = [&](int j) { return (uint32_t)(B_KC ? j * BK4 * 2 : (int64_t)j * BK4 * g.ldb * 2); };
  auto piece = [&](int i, int j, char* sd) {
    if (i == 0 || i == 4) m0_set(lds_addr(sd + (i ? HALF4 : 0) + wid * 4096), m0keep);
    if (i < 4) dma16_buf_m0(srd_a, offa[i], soff_a(j), i);
    else dma16_buf_m0(srd_b, offb[i - 4], soff_b(j), i - 4);
    if (i == 3 || i == 7) m0_restore(m0keep);
  };
  auto issue = [&](int j) {
    j = min(j, ns - 1);
#pragma unroll
    for (int i = 0; i < 8; ++i) piece(i, j, smem + (j & 3) * SLICE4);
  };
  // fragment c = 4 s + i: k-step s, 32-row block i of the wave's 128 rows (A) / columns (B)
  auto read = [&](int j, bf16x8 (&af)[8], bf16x8 (&bf)[8]) {
    const char* st = smem + (j & 3) * SLICE4;
#pragma unroll
    for (int c = 0; c < 8; ++c) af[c] = read_frag32<A_KC>(st, wm * 128 + (c & 3) * 32, c >> 2, lane);
#pragma unroll
    for (int c = 0; c < 8; ++c) bf[c] = read_frag32<B_KC>(st + HALF4, wn * 128 + (c & 3) * 32, c >> 2, lane);
  };
  auto step = [&](int j, bf16x8 (&ca)[8], bf16x8 (&cb)[8], bf16x8 (&na)[8], bf16x8 (&nb)[8]) {
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // own part of slice j+1 landed
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int jd = min(j + 3, ns - 1);
    char* sd = smem + ((j + 3) & 3) * SLICE4;
    const char* st = smem + ((j + 1) & 3) * SLICE4;
    // eight chunks: chunk c = (k-step s, A block i) runs its 4 MFMAs beside one LDS-DMA piece of
    // slice j+3 and the reads of fragments c of slice j+1
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int s = c >> 2, i = c & 3;
      if (GEMM4X_IL) {       // the four-wave kernel's GEMM4_IL placement: each between two MFMAs
        auto mf = [&](int jj) {
          asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0"
                       : "+a"(acc[i][jj]) : "v"(cb[4 * s + jj]), "v"(ca[c]));
        };
        mf(0);
        piece(c, jd, sd);
        mf(1);
        __builtin_amdgcn_sched_barrier(0);
        na[c] = read_frag32<A_KC>(st, wm * 128 + (c & 3) * 32, c >> 2, lane);
        __builtin_amdgcn_sched_barrier(0);
        mf(2);
        __builtin_amdgcn_sched_barrier(0);
        nb[c] = read_frag32<B_KC>(st + HALF4, wn * 128 + (c & 3) * 32, c >> 2, lane);
        __builtin_amdgcn_sched_barrier(0);
        mf(3);
        __builtin_amdgcn_sched_barrier(0);
        continue;
      }
      piece(c, jd, sd);
      na[c] = read_frag32<A_KC>(st, wm * 128 + (c & 3) * 32, c >> 2, lane);
      nb[c] = read_frag32<B_KC>(st + HALF4, wn * 128 + (c & 3) * 32, c >> 2, lane);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)   // D = B . A^T: lanes own consecutive n of one row m
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0"
                     : "+a"(acc[i][jj]) : "v"(cb[4 * s + jj]), "v"(ca[c]));
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  asm volatile("s_nop 7" ::: "memory");    // accumulator zeroing (VALU) -> first asm MFMA
  issue(0);
  issue(1);
  issue(2);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  bf16x8 fa[8], fb[8], ga[8], gb[8];
  read(0, fa, fb);
  for (int j = 0; j < ns; j += 2) {
    step(j, fa, fb, ga, gb);
    step(j + 1, ga, gb, fa, fb);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // inline-asm MFMAs: pad the last MFMA write -> v_accvgpr_read distance by hand (32x32: 16 passes)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  const int mb = m0 + wm * 128 + (lane & 31), nb = n0 + wn * 128 + 4 * (lane >> 5);
  if (EPI == EPI_DGELU || (EPI == EPI_RESID && g.res_bf16))
    epilogue4x<EPI, true>(g, acc, mb, nb);
  else
    epilogue4x<EPI, false>(g, acc, mb, nb);
}

// tile: 0 = by shape (the 256 tile wherever it applies and fills >= 96 CUs), 128 / 256 = forced,
// 512 = the 256 tile on the 8-wave kernel
// (parity tests: both kernels accumulate every element in the same k order, so their outputs
// are bit-identical)
// GELU / gated-residual epilogues on the four-wave kernel (1) or the 8-wave one (0): with the
// sigmoid-form GELU and the 3-row-block-ahead epilogue inputs the four-wave kernel is level on
// FFN-up GELU (8.91 vs 8.92 ms) and 1-4 % faster on the residual (o-proj 3.66 vs 3.80 ms) at 720p
// (profiles/r02_gemm_epi4w_ab.txt); round 2's first four-wave epilogue was 1-6 % slower there.
#ifndef GEMM_GELU_4W
#define GEMM_GELU_4W 1
#endif
#ifndef GEMM_RESID_4W
#define GEMM_RESID_4W 1
#endif
// the four-wave tile on MFMA 32x32x16 (gemm4x_kernel) for every epilogue (1), or only for the
// weight gradients dW = dY^T X (0): there it is 1.3-6 % faster, on the forward / dX shapes 1-7 %
// slower (720p x 81f, one process, 5 interleaved reps: profiles/r03_gemm_mfma32_ab.txt); the
// outputs of the two kernels are bit-identical on every shape measured
#ifndef GEMM_MFMA32
#define GEMM_MFMA32 0
#endif
template <bool A_KC, bool B_KC, int EPI>
int launch(const GemmArgs& g, hipStream_t s, int tile) {
  const int nt256 = ((g.M + BM2 - 1) / BM2) * ((g.N + BN2 - 1) / BN2);
  // the 256 tiles need whole 64-deep K steps and whole 256-wide MN-major extents
  const bool fits256 = (g.K % BK) == 0 && g.K >= 128 && (A_KC || g.M % BM2 == 0) &&
                       (B_KC || g.N % BN2 == 0);
  if ((tile == 256 || tile == 512) && !fits256) return (int)hipErrorInvalidValue;
  if (tile == 512) {       // forced: the 8-wave 256 kernel (parity tests)
    hipLaunchKernelGGL((gemm256s_kernel<A_KC, B_KC, EPI>), dim3(nt256), dim3(NT2), 0, s, g);
  } else if (tile == 256 || (tile == 0 && fits256 && nt256 >= 96)) {
    // the four-wave kernel (each operand addressed through a 32-bit buffer offset) wherever
    // the operands fit 4 GiB; the 8-wave kernel otherwise (and for the epilogues switched back
    // by GEMM_GELU_4W / GEMM_RESID_4W = 0)
    const int64_t bytes_a = (A_KC ? (int64_t)g.M : (int64_t)g.K) * g.lda * 2;
    const int64_t bytes_b = (B_KC ? (int64_t)g.N : (int64_t)g.K) * g.ldb * 2;
    const bool four = (GEMM_GELU_4W || EPI != EPI_GELU) && (GEMM_RESID_4W || EPI != EPI_RESID) &&
                      bytes_a < (1ll << 32) && bytes_b < (1ll << 32);
    if (four && (GEMM_MFMA32 || (EPI == EPI_F32 && !A_KC && !B_KC)))
      hipLaunchKernelGGL((gemm4x_kernel<A_KC, B_KC, EPI>), dim3(nt256), dim3(256), 0, s, g);
    else if (four)
      hipLaunchKernelGGL((gemm4w_kernel<A_KC, B_KC, EPI>), dim3(nt256), dim3(256), 0, s, g);
    else
      hipLaunchKernelGGL((gemm256s_kernel<A_KC, B_KC, EPI>), dim3(nt256), dim3(NT2), 0, s, g);
  } else {
    const int ntm = (g.M + BM - 1) / BM, ntn = (g.N + BN - 1) / BN;
    hipLaunchKernelGGL((gemm_kernel<A_KC, B_KC, EPI>), dim3(ntm * ntn), dim3(NT), 0, s, g);
  }
  PRFL_LAUNCH_CHECK();
  return 0;
}

}  // namespace

extern "C" int prfl_gemm_bf16_tiled(const void* A, int64_t lda, int a_kmajor, const void* B,
                                    int64_t ldb, int b_kmajor, void* C, int64_t ldc, int64_t M,
                                    int64_t N, int64_t K, int epilogue, const void* bias,
                                    const float* gate, const void* res, int64_t ldr, int res_bf16,
                                    void* aux, int64_t ldaux, int accumulate, int tile,
                                    void* stream) {
  if (M <= 0 || N <= 0) return 0;
  if (tile != 0 && tile != 128 && tile != 256 && tile != 512) return (int)hipErrorInvalidValue;
  // K is a contiguous extent only for K-major operands; MN-major operands take any K (row tail)
  if (K <= 0 || ((a_kmajor || b_kmajor) && (K % 8) != 0) || (N % 4) != 0)
    return (int)hipErrorInvalidValue;
  if ((lda % 8) || (ldb % 8) || ((uintptr_t)A & 15) || ((uintptr_t)B & 15))
    return (int)hipErrorInvalidValue;
  if (!a_kmajor && (M % 8)) return (int)hipErrorInvalidValue;
  if (!b_kmajor && (N % 8)) return (int)hipErrorInvalidValue;
  if (M > 0x7fffffff || N > 0x7fffffff || K > 0x7fffffff) return (int)hipErrorInvalidValue;
  GemmArgs g{(const bf16*)A, lda, (const bf16*)B, ldb, C, ldc, (int)M, (int)N, (int)K,
             (const bf16*)bias, gate, res, ldr, res_bf16, (bf16*)aux, ldaux, accumulate};
  hipStream_t s = (hipStream_t)stream;
  prfl_prof::begin(KID_GEMM, s);
  int rc = (int)hipErrorInvalidValue;
  // weight gradients with a token count K that is not a multiple of 64: the bulk of K goes
  // through the 256-tile kernel, the < 64-row tail is accumulated by a second (128-tile) launch
  if (tile != 128 && epilogue == EPI_F32 && !a_kmajor && !b_kmajor && (K % BK) != 0 && K > BK &&
      (M % BM2) == 0 && (N % BN2) == 0) {
    const int64_t Kmain = K - K % BK;
    GemmArgs gm = g;
    gm.K = (int)Kmain;
    rc = launch<false, false, EPI_F32>(gm, s, tile);
    if (rc == 0) {
      GemmArgs gt = g;
      gt.A = g.A + Kmain * lda;
      gt.B = g.B + Kmain * ldb;
      gt.K = (int)(K - Kmain);
      gt.accumulate = 1;
      const int ntm = (gt.M + BM - 1) / BM, ntn = (gt.N + BN - 1) / BN;
      hipLaunchKernelGGL((gemm_kernel<false, false, EPI_F32>), dim3(ntm * ntn), dim3(NT), 0, s, gt);
      rc = (int)hipGetLastError();
    }
    prfl_prof::set_work(2.0 * (double)M * (double)N * (double)K);
    prfl_prof::end(KID_GEMM, s);
    return rc;
  }
#define GEMM_CASE(AK, BK_, E) \
  if (a_kmajor == AK && b_kmajor == BK_ && epilogue == E) rc = launch<AK, BK_, E>(g, s, tile);
  GEMM_CASE(1, 1, EPI_BF16)
  GEMM_CASE(1, 1, EPI_GELU)
  GEMM_CASE(1, 1, EPI_RESID)
  GEMM_CASE(1, 1, EPI_F32)
  GEMM_CASE(1, 1, EPI_DGELU)
  GEMM_CASE(1, 0, EPI_BF16)
  GEMM_CASE(1, 0, EPI_GELU)
  GEMM_CASE(1, 0, EPI_RESID)
  GEMM_CASE(1, 0, EPI_DGELU)
  GEMM_CASE(1, 0, EPI_F32)
  GEMM_CASE(0, 0, EPI_F32)
  GEMM_CASE(0, 0, EPI_BF16)   // both operands MN-major (tools/gemm_run_probe.py: DMA row runs)
  GEMM_CASE(0, 1, EPI_F32)
#undef GEMM_CASE
  prfl_prof::set_work(2.0 * (double)M * (double)N * (double)K);
  prfl_prof::end(KID_GEMM, s);
  return rc;
}

extern "C" int prfl_gemm_bf16(const void* A, int64_t lda, int a_kmajor, const void* B, int64_t ldb,
                              int b_kmajor, void* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                              int epilogue, const void* bias, const float* gate, const void* res,
                              int64_t ldr, int res_bf16, void* aux, int64_t ldaux, int accumulate,
                              void* stream) {
  return prfl_gemm_bf16_tiled(A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, M, N, K, epilogue, bias,
                              gate, res, ldr, res_bf16, aux, ldaux, accumulate, 0, stream);
}

// ================================================================ fp8 (C5: I2V 720p fp8 path) ===
// C[m][n] = sa[m] * sb[n] * sum_k A8(m,k) B8(n,k)   (+ the bf16 kernel's epilogues)
// A8 / B8 are OCP e4m3 (gfx950 `e4m3fn`), both K-major, quantised per row (prfl_quant_rows_fp8).
// The MFMA is the block-scaled `v_mfma_scale_f32_16x16x128_f8f6f4` (2x the bf16 MFMA rate; the
// unscaled fp8 forms run at the bf16 rate) with every E8M0 block scale = 2^0: the per-row /
// per-column dequantisation happens once, in fp32, in the epilogue.
// It runs on gemm256s_kernel<.., F8 = true>: the staggered bf16 schedule over the same BYTES (an
// e4m3 [rows][K] operand passed as bf16 [rows][K/2]).
namespace {
// ---- per-row e4m3 quantisation: scale[m] = amax_m / 448, q = e4m3(x * (448 / amax_m)) ------
constexpr int QNT = 256, QMAXC = 8;     // <= 8 chunks of 8 per thread: K <= 16384
constexpr float E4M3_MAX = 448.f;

__device__ __forceinline__ float ldf(const float* p, int64_t i) { return p[i]; }
__device__ __forceinline__ float ldf(const bf16* p, int64_t i) { return bf2f(p[i]); }

template <typename T>
__global__ __launch_bounds__(QNT) void quant_rows_fp8_kernel(const T* __restrict__ x, int64_t ldx,
                                                             int K, uint8_t* __restrict__ q,
                                                             int64_t ldq,
                                                             float* __restrict__ scale) {
  __shared__ float red[QNT / 64];
  const int64_t m = blockIdx.x;
  const T* xr = x + m * ldx;
  const int nch = K / 8;
  float v[QMAXC][8];
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < QMAXC; ++c) {
    const int ch = threadIdx.x + c * QNT;
    if (ch < nch) {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        v[c][r] = ldf(xr, (int64_t)ch * 8 + r);
        amax = fmaxf(amax, fabsf(v[c][r]));
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float inv = amax > 0.f ? E4M3_MAX / amax : 1.f;
  if (threadIdx.x == 0) scale[m] = amax > 0.f ? amax / E4M3_MAX : 1.f;
  uint8_t* qr = q + m * ldq;
#pragma unroll
  for (int c = 0; c < QMAXC; ++c) {
    const int ch = threadIdx.x + c * QNT;
    if (ch < nch) {
      int lo = 0, hi = 0;
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][0] * inv, v[c][1] * inv, lo, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][2] * inv, v[c][3] * inv, lo, true);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][4] * inv, v[c][5] * inv, hi, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][6] * inv, v[c][7] * inv, hi, true);
      *(uint2*)(qr + (int64_t)ch * 8) = make_uint2((unsigned)lo, (unsigned)hi);
    }
  }
}
}  // namespace

extern "C" int prfl_quant_rows_fp8(const void* x, int x_f32, int64_t ldx, int64_t M, int64_t K,
                                   void* q, int64_t ldq, float* scale, void* stream) {
  if (M <= 0) return 0;
  if (K <= 0 || K % 8 || K > 8LL * QNT * QMAXC || ldx % 8 || ldq % 8 || M > 0x7fffffff)
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  prfl_prof::begin(KID_ELTWISE, s);
  if (x_f32)
    hipLaunchKernelGGL(quant_rows_fp8_kernel<float>, dim3(M), dim3(QNT), 0, s, (const float*)x,
                       ldx, (int)K, (uint8_t*)q, ldq, scale);
  else
    hipLaunchKernelGGL(quant_rows_fp8_kernel<bf16>, dim3(M), dim3(QNT), 0, s, (const bf16*)x,
                       ldx, (int)K, (uint8_t*)q, ldq, scale);
  prfl_prof::set_work((double)M * K * ((x_f32 ? 4 : 2) + 1));
  prfl_prof::end(KID_ELTWISE, s);
  PRFL_LAUNCH_CHECK();
  return 0;
}

extern "C" int prfl_gemm_fp8(const void* A, int64_t lda, const float* sa, const void* B,
                             int64_t ldb, const float* sb, void* C, int64_t ldc, int64_t M,
                             int64_t N, int64_t K, int epilogue, const void* bias,
                             const float* gate, const void* res, int64_t ldr, int res_bf16,
                             void* aux, int64_t ldaux, void* stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K <= 0 || K % 128 || N % 4 || lda % 16 || ldb % 16 || ((uintptr_t)A & 15) ||
      ((uintptr_t)B & 15) || ((uintptr_t)sb & 15) || !sa || !sb)
    return (int)hipErrorInvalidValue;
  if (M > 0x7fffffff || N > 0x7fffffff || K > 0x7fffffff) return (int)hipErrorInvalidValue;
  if (epilogue != EPI_BF16 && epilogue != EPI_GELU && epilogue != EPI_RESID)
    return (int)hipErrorInvalidValue;
  GemmArgs g{(const bf16*)A, lda, (const bf16*)B, ldb, C, ldc, (int)M, (int)N, (int)K,
             (const bf16*)bias, gate, res, ldr, res_bf16, (bf16*)aux, ldaux, 0};
  hipStream_t s = (hipStream_t)stream;
  const int nt = (int)(((M + BM2 - 1) / BM2) * ((N + BN2 - 1) / BN2));
  prfl_prof::begin(KID_GEMM, s);
  // the staggered 4-phase bf16 schedule over the same bytes: K8 e4m3 = K8/2 "bf16" columns
  GemmArgs g2 = g;
  g2.lda = lda / 2;
  g2.ldb = ldb / 2;
  g2.K = (int)(K / 2);
  g2.sa = sa;
  g2.sb = sb;
  if (epilogue == EPI_BF16)
    hipLaunchKernelGGL((gemm256s_kernel<true, true, EPI_BF16, true>), dim3(nt), dim3(NT2), 0, s, g2);
  else if (epilogue == EPI_GELU)
    hipLaunchKernelGGL((gemm256s_kernel<true, true, EPI_GELU, true>), dim3(nt), dim3(NT2), 0, s, g2);
  else
    hipLaunchKernelGGL((gemm256s_kernel<true, true, EPI_RESID, true>), dim3(nt), dim3(NT2), 0, s, g2);
  prfl_prof::set_work(2.0 * (double)M * (double)N * (double)K);
  prfl_prof::end(KID_GEMM, s);
  PRFL_LAUNCH_CHECK();
  return 0;
}
