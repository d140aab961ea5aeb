// Row-wise normalisation kernels of the Wan block, forward and backward.
//
//  ln_mod      : WanLayerNorm (no affine, eps 1e-6) + AdaLN  y = LN(x)*(1+scale)+shift  -> bf16
//                (`model.py:125-135, 345, 353`); or affine LN y = LN(x)*w+b -> bf16 (norm3, :352)
//  rms_rope    : WanRMSNorm over all C channels (`model.py:106-122`): n = bf16(x*rsqrt(mean x^2+eps)),
//                y = n*w, then the 3-D RoPE of `model.py:61-103` (pairs 0..21 rotate with the frame
//                index, 22..42 with the row, 43..63 with the column) -> bf16 attention operand,
//                times out_scale (1, or softmax_scale * log2 e for a q that the attention kernels
//                take in log2 units: the *_l2q entries of attention.hip); the backward scales the
//                incoming gradient by the same out_scale.
//
// One workgroup (256 threads) per row (C <= 5120); the forward holds the row in registers, the
// backward re-reads it from L1/L2 in a second pass instead of spilling.
// The column reductions of the backward passes (d scale, d shift, d w, d b) are written as
// per-workgroup partial rows and summed by colsum_reduce (elementwise.hip) — no float atomics,
// bitwise reproducible.
#include "common.h"

namespace {
constexpr int NT = 256;
constexpr int MAXV = 5;  // float4 chunks per thread -> C <= 5120 (Wan 14B width)

__device__ __forceinline__ f32x4 ld4(const void* p, int64_t i, int is_bf16) {
  if (is_bf16) {
    const bf16x4 v = *(const bf16x4*)((const bf16*)p + i);
    return (f32x4){bf2f(v[0]), bf2f(v[1]), bf2f(v[2]), bf2f(v[3])};
  }
  return *(const f32x4*)((const float*)p + i);
}
__device__ __forceinline__ f32x4 ldf4(const float* p, int i) { return *(const f32x4*)(p + i); }

// --------------------------------------------------------------------------- LN + modulate --
constexpr int WV = 20;  // float4 chunks per lane -> C <= 5120

// dx (+)= LN backward; partial column sums: part0 = sum dy*xhat_used (d scale / d w),
// part1 = sum dy (d shift / d b).  ROWS rows per workgroup.
template <int ROWS>
__global__ __launch_bounds__(NT) void ln_mod_bwd_kernel(
    const bf16* __restrict__ dy, int64_t lddy, const void* __restrict__ x, int x_bf16, int64_t ldx,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, int L, int C,
    const float* __restrict__ scale, const float* __restrict__ w, float* __restrict__ dx,
    int64_t lddx, int dx_accumulate, float* __restrict__ part0, float* __restrict__ part1) {
  __shared__ float red[NT / 64];
  const int nc = C / 4;
  f32x4 p0[MAXV], p1[MAXV];
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    p0[j] = (f32x4){0, 0, 0, 0};
    p1[j] = (f32x4){0, 0, 0, 0};
  }
  const int r0 = blockIdx.x * ROWS;
  for (int rr = 0; rr < ROWS; ++rr) {
    const int64_t row = r0 + rr;
    if (row >= L) break;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      const int c = threadIdx.x + j * NT;
      if (c < nc) {
        const f32x4 xv = ld4(x, row * ldx + c * 4, x_bf16);
        const bf16x4 dv = *(const bf16x4*)(dy + row * lddy + c * 4);
        const f32x4 m = w ? ldf4(w, c * 4) : ldf4(scale, c * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float xhat = (xv[r] - mean) * rstd;
          const float d = bf2f(dv[r]);
          const float xu = (!w && x_bf16) ? bfr(xhat) : xhat;
          p0[j][r] += d * xu;
          p1[j][r] += d;
          const float gg = w ? d * m[r] : d * (1.f + m[r]);
          s1 += gg;
          s2 += gg * xhat;
        }
      }
    }
    const float m1 = block_sum<NT>(s1, red) / C;
    const float m2 = block_sum<NT>(s2, red) / C;
    // second pass re-reads the (L1/L2-resident) row instead of holding it in registers
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      const int c = threadIdx.x + j * NT;
      if (c < nc) {
        const f32x4 xv = ld4(x, row * ldx + c * 4, x_bf16);
        const bf16x4 dv = *(const bf16x4*)(dy + row * lddy + c * 4);
        const f32x4 m = w ? ldf4(w, c * 4) : ldf4(scale, c * 4);
        f32x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float xhat = (xv[r] - mean) * rstd;
          const float d = bf2f(dv[r]);
          const float gg = w ? d * m[r] : d * (1.f + m[r]);
          o[r] = rstd * (gg - m1 - xhat * m2);
        }
        float* dp = dx + row * lddx + c * 4;
        if (dx_accumulate) o = o + *(f32x4*)dp;
        *(f32x4*)dp = o;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int c = threadIdx.x + j * NT;
    if (c < nc) {
      *(f32x4*)(part0 + (int64_t)blockIdx.x * C + c * 4) = p0[j];
      *(f32x4*)(part1 + (int64_t)blockIdx.x * C + c * 4) = p1[j];
    }
  }
}

// --------------------------------------------------------------------------- RMSNorm + RoPE --
// rope: table [1024][64] of (cos, sin) fp32; grid (F, Hg, Wg); rows >= F*Hg*Wg pass through.
__device__ __forceinline__ void rope_pos(int64_t row, int F, int Hg, int Wg, int& pf, int& ph,
                                         int& pw, bool& rot) {
  const int64_t n = (int64_t)F * Hg * Wg;
  rot = row < n;
  pf = (int)(row / ((int64_t)Hg * Wg));
  ph = (int)((row / Wg) % Hg);
  pw = (int)(row % Wg);
}
__device__ __forceinline__ int rope_index(int pair, int pf, int ph, int pw) {
  // split [22, 21, 21] of the 64 complex pairs of a head (model.py:65)
  return pair < 22 ? pf : (pair < 43 ? ph : pw);
}

__global__ __launch_bounds__(NT) void rms_rope_fwd_kernel(
    const bf16* __restrict__ x, int64_t ldx, int C, const float* __restrict__ w, float eps,
    const float2* __restrict__ tab, int F, int Hg, int Wg, int64_t row0, bf16* __restrict__ out,
    int64_t ldo, float* __restrict__ rstd_out, float oscale) {
  __shared__ float red[NT / 64];
  const int64_t row = blockIdx.x;
  const int nc = C / 4;
  f32x4 v[MAXV];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int c = threadIdx.x + j * NT;
    if (c < nc) {
      v[j] = ld4(x, row * ldx + c * 4, 1);
#pragma unroll
      for (int r = 0; r < 4; ++r) ss += v[j][r] * v[j][r];
    }
  }
  const float rstd = rsqrtf(block_sum<NT>(ss, red) / C + eps);
  int pf, ph, pw;
  bool rot;
  rope_pos(row0 + row, F, Hg, Wg, pf, ph, pw, rot);
  rot = rot && tab != nullptr;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int c = threadIdx.x + j * NT;
    if (c < nc) {
      const f32x4 wv = ldf4(w, c * 4);
      float y[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) y[r] = mul_rn(bfr(v[j][r] * rstd), wv[r]);
      bf16x4 o;
      if (rot) {
        const int e0 = (c * 4) & 127;  // element within the head
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int pair = (e0 >> 1) + pp;
          const float2 cs = tab[rope_index(pair, pf, ph, pw) * 64 + pair];
          const float a = y[2 * pp], bq = y[2 * pp + 1];
          o[2 * pp] = f2bf(__fmul_rn(__fsub_rn(__fmul_rn(a, cs.x), __fmul_rn(bq, cs.y)), oscale));
          o[2 * pp + 1] = f2bf(__fmul_rn(__fadd_rn(__fmul_rn(a, cs.y), __fmul_rn(bq, cs.x)), oscale));
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(__fmul_rn(y[r], oscale));
      }
      *(bf16x4*)(out + row * ldo + c * 4) = o;
    }
  }
  if (threadIdx.x == 0) rstd_out[row] = rstd;
}

// dx = RMSNorm backward of (RoPE^T dout); part0 = sum dy*n (d w).
template <int ROWS>
__global__ __launch_bounds__(NT) void rms_rope_bwd_kernel(
    const bf16* __restrict__ dout, int64_t lddo, const bf16* __restrict__ x, int64_t ldx,
    const float* __restrict__ rstd_in, int L, int C, const float* __restrict__ w,
    const float2* __restrict__ tab, int F, int Hg, int Wg, int64_t row0, bf16* __restrict__ dx,
    int64_t lddx, float* __restrict__ part0, float oscale) {
  __shared__ float red[NT / 64];
  const int nc = C / 4;
  f32x4 p0[MAXV];
#pragma unroll
  for (int j = 0; j < MAXV; ++j) p0[j] = (f32x4){0, 0, 0, 0};
  const int r0 = blockIdx.x * ROWS;
  for (int rr = 0; rr < ROWS; ++rr) {
    const int64_t row = r0 + rr;
    if (row >= L) break;
    const float rstd = rstd_in[row];
    int pf, ph, pw;
    bool rot;
    rope_pos(row0 + row, F, Hg, Wg, pf, ph, pw, rot);
    rot = rot && tab != nullptr;
    float s = 0.f;
    // pass 1: s = sum(dn * xhat); pass 2 recomputes dn from the re-read row
    for (int pass = 0; pass < 2; ++pass) {
      const float m = pass ? block_sum<NT>(s, red) / C : 0.f;
#pragma unroll
      for (int j = 0; j < MAXV; ++j) {
        const int c = threadIdx.x + j * NT;
        if (c < nc) {
          const f32x4 xv = ld4(x, row * ldx + c * 4, 1);
          const f32x4 gv = ld4(dout, row * lddo + c * 4, 1) * oscale;
          const f32x4 wv = ldf4(w, c * 4);
          float dy[4];
          if (rot) {
            const int e0 = (c * 4) & 127;
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
              const int pair = (e0 >> 1) + pp;
              const float2 cs = tab[rope_index(pair, pf, ph, pw) * 64 + pair];
              const float ga = gv[2 * pp], gb = gv[2 * pp + 1];
              dy[2 * pp] = ga * cs.x + gb * cs.y;       // conj rotation
              dy[2 * pp + 1] = gb * cs.x - ga * cs.y;
            }
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) dy[r] = gv[r];
          }
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float xhat = xv[r] * rstd;
            const float d = bfr(dy[r] * wv[r]);  // grad of the bf16 normalised tensor
            if (pass == 0) {
              p0[j][r] += dy[r] * bfr(xhat);
              s += d * xhat;
            } else {
              o[r] = f2bf(rstd * (d - xhat * m));
            }
          }
          if (pass == 1) *(bf16x4*)(dx + row * lddx + c * 4) = o;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int c = threadIdx.x + j * NT;
    if (c < nc) *(f32x4*)(part0 + (int64_t)blockIdx.x * C + c * 4) = p0[j];
  }
}

// ---- RMSNorm + RoPE, one wave per row (round 6, RMS_WAVE) ------------------------------------
// 16-B loads and stores (8 bf16 per chunk, chunk c = lane + 64 j), the row held in registers, the
// sum of squares a wave shuffle (no workgroup barrier per row), w staged once per workgroup in LDS
// (the 256-thread form re-read 20 KB of fp32 w from L2 for every 10 KB row), and the RoPE
// multipliers loaded once per row: a lane's chunks all start at the same element of a head
// ((lane * 8) & 127), so its 4 (cos, sin) pairs are the same for every chunk of the row.
// Per-element arithmetic as rms_rope_fwd_kernel; only the order of the row's sum of squares
// differs (fp32 rounding of rstd).
#ifndef RMS_WAVE
#define RMS_WAVE 1
#endif
#ifndef RMS_WAVE_RPW
#define RMS_WAVE_RPW 4
#endif
// forward row prefetch: 0 none (one row in flight per wave, 90 VGPRs), 1 the next row into a
// second register set (unrolled), 2 the same in a rolled loop, the prefetched set copied into the
// working one; 720p 0.337 / 0.332 / 0.313 ms, bit-identical (profiles/r06_ab_rms_prefetch.txt)
#ifndef RMS_WAVE_PF
#define RMS_WAVE_PF 2
#endif
constexpr int RW_RPW = RMS_WAVE_RPW;     // rows per wave in the forward (16 rows per workgroup)
constexpr int RW_NJ = 10;     // 16-B chunks per lane: C <= 64 * 10 * 8 = 5120

__device__ __forceinline__ void rope_cs4(const float2* __restrict__ tab, int pair0, int pf, int ph,
                                         int pw, float2 (&cs)[4]) {
#pragma unroll
  for (int pp = 0; pp < 4; ++pp) cs[pp] = tab[rope_index(pair0 + pp, pf, ph, pw) * 64 + pair0 + pp];
}

__global__ __launch_bounds__(NT) void rms_rope_fwd_wave_kernel(
    const bf16* __restrict__ x, int64_t ldx, int L, int C, const float* __restrict__ w, float eps,
    const float2* __restrict__ tab, int F, int Hg, int Wg, int64_t row0, bf16* __restrict__ out,
    int64_t ldo, float* __restrict__ rstd_out, float oscale) {
  __shared__ f32x4 ws[RW_NJ * 64 * 2];
  const int lane = threadIdx.x & 63, nc = C / 8, pair0 = ((lane * 8) & 127) >> 1;
  const int64_t rbase = ((int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6)) * RW_RPW;
  // RMS_WAVE_PF: the next row's chunks are loaded before this row's normalise / store, and the
  // first row's before the w staging and its barrier
  bf16x8 v[2][RW_NJ];
  auto load = [&](int64_t row, bf16x8 (&d)[RW_NJ]) {
#pragma unroll
    for (int j = 0; j < RW_NJ; ++j) {
      const int c = lane + 64 * j;
      if (c < nc && row < L) d[j] = *(const bf16x8*)(x + row * ldx + c * 8);
    }
  };
  if (RMS_WAVE_PF) load(rbase, v[0]);
  for (int c = threadIdx.x; c < C / 4; c += NT) ws[c] = ldf4(w, c * 4);
  __syncthreads();
#if RMS_WAVE_PF == 2
#pragma unroll 1
#else
#pragma unroll
#endif
  for (int rr = 0; rr < RW_RPW; ++rr) {
    const int64_t row = rbase + rr;
    if (row >= L) return;
    // PF 2: rolled loop, the prefetched set copied into the working one (fewer live registers)
    bf16x8 (&cur)[RW_NJ] = v[RMS_WAVE_PF == 1 ? (rr & 1) : 0];
    if (!RMS_WAVE_PF) {
      load(row, cur);
    } else if (RMS_WAVE_PF == 2) {
      if (rr > 0) {
#pragma unroll
        for (int j = 0; j < RW_NJ; ++j) cur[j] = v[1][j];
      }
      if (rr + 1 < RW_RPW) load(row + 1, v[1]);
    } else if (rr + 1 < RW_RPW) {
      load(row + 1, v[(rr + 1) & 1]);
    }
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < RW_NJ; ++j) {
      const int c = lane + 64 * j;
      if (c < nc) {
#pragma unroll
        for (int r = 0; r < 8; ++r) ss += bf2f(cur[j][r]) * bf2f(cur[j][r]);
      }
    }
    const float rstd = rsqrtf(wave_sum(ss) / C + eps);
    int pf, ph, pw;
    bool rot;
    rope_pos(row0 + row, F, Hg, Wg, pf, ph, pw, rot);
    rot = rot && tab != nullptr;
    float2 cs[4];
    if (rot) rope_cs4(tab, pair0, pf, ph, pw, cs);
#pragma unroll
    for (int j = 0; j < RW_NJ; ++j) {
      const int c = lane + 64 * j;
      if (c < nc) {
        const f32x4 w0 = ws[2 * c], w1 = ws[2 * c + 1];
        float y[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          y[r] = mul_rn(bfr(bf2f(cur[j][r]) * rstd), w0[r]);
          y[r + 4] = mul_rn(bfr(bf2f(cur[j][r + 4]) * rstd), w1[r]);
        }
        bf16x8 o;
        if (rot) {
#pragma unroll
          for (int pp = 0; pp < 4; ++pp) {
            const float a = y[2 * pp], bq = y[2 * pp + 1];
            o[2 * pp] = f2bf(__fmul_rn(__fsub_rn(__fmul_rn(a, cs[pp].x), __fmul_rn(bq, cs[pp].y)), oscale));
            o[2 * pp + 1] = f2bf(__fmul_rn(__fadd_rn(__fmul_rn(a, cs[pp].y), __fmul_rn(bq, cs[pp].x)), oscale));
          }
        } else {
#pragma unroll
          for (int r = 0; r < 8; ++r) o[r] = f2bf(__fmul_rn(y[r], oscale));
        }
        *(bf16x8*)(out + row * ldo + c * 8) = o;
      }
    }
    if (lane == 0) rstd_out[row] = rstd;
  }
}

// backward: the workgroup's BWD_ROWS rows, wave k taking rows k, k + 4, ...; 16-B chunks, the
// d w partial kept per lane (80 registers) and summed over
// the four waves in LDS in a fixed order (deterministic), one partial row per workgroup as before
template <int ROWS>
__global__ __launch_bounds__(NT) void rms_rope_bwd_wave_kernel(
    const bf16* __restrict__ dout, int64_t lddo, const bf16* __restrict__ x, int64_t ldx,
    const float* __restrict__ rstd_in, int L, int C, const float* __restrict__ w,
    const float2* __restrict__ tab, int F, int Hg, int Wg, int64_t row0, bf16* __restrict__ dx,
    int64_t lddx, float* __restrict__ part0, float oscale) {
  __shared__ f32x4 ws[RW_NJ * 64 * 2];
  __shared__ f32x4 acc[RW_NJ * 64 * 2];
  for (int c = threadIdx.x; c < C / 4; c += NT) ws[c] = ldf4(w, c * 4);
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nc = C / 8;
  const int pair0 = ((lane * 8) & 127) >> 1;
  float p0[RW_NJ][8];
#pragma unroll
  for (int j = 0; j < RW_NJ; ++j)
#pragma unroll
    for (int r = 0; r < 8; ++r) p0[j][r] = 0.f;
  for (int rr = wv; rr < ROWS; rr += NT / 64) {
    const int64_t row = (int64_t)blockIdx.x * ROWS + rr;
    if (row >= L) break;
    const float rstd = rstd_in[row];
    int pf, ph, pw;
    bool rot;
    rope_pos(row0 + row, F, Hg, Wg, pf, ph, pw, rot);
    rot = rot && tab != nullptr;
    float2 cs[4];
    if (rot) rope_cs4(tab, pair0, pf, ph, pw, cs);
    // pass 1 streams the row from HBM; pass 2 re-reads it (L1 / L2) rather than holding both
    // operands across the row reduction beside the 80 partial sums (305 registers, 1 wave / SIMD)
    auto dyv = [&](const bf16x8& gq, float (&dy)[8]) {
#pragma unroll
      for (int r = 0; r < 8; ++r) dy[r] = bf2f(gq[r]) * oscale;
      if (rot) {
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {
          const float ga = dy[2 * pp], gb = dy[2 * pp + 1];
          dy[2 * pp] = ga * cs[pp].x + gb * cs[pp].y;
          dy[2 * pp + 1] = gb * cs[pp].x - ga * cs[pp].y;
        }
      }
    };
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < RW_NJ; ++j) {
      const int c = lane + 64 * j;
      if (c < nc) {
        const bf16x8 gq = *(const bf16x8*)(dout + row * lddo + c * 8);
        const bf16x8 xq = *(const bf16x8*)(x + row * ldx + c * 8);
        float dy[8];
        dyv(gq, dy);
        const f32x4 w0 = ws[2 * c], w1 = ws[2 * c + 1];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const float xhat = bf2f(xq[r]) * rstd;
          const float d = bfr(dy[r] * (r < 4 ? w0[r] : w1[r - 4]));
          p0[j][r] += dy[r] * bfr(xhat);
          s += d * xhat;
        }
      }
    }
    const float m = wave_sum(s) / C;
#pragma unroll
    for (int j = 0; j < RW_NJ; ++j) {
      const int c = lane + 64 * j;
      if (c < nc) {
        const bf16x8 gq = *(const bf16x8*)(dout + row * lddo + c * 8);
        const bf16x8 xq = *(const bf16x8*)(x + row * ldx + c * 8);
        float dy[8];
        dyv(gq, dy);
        const f32x4 w0 = ws[2 * c], w1 = ws[2 * c + 1];
        bf16x8 o;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const float xhat = bf2f(xq[r]) * rstd;
          const float d = bfr(dy[r] * (r < 4 ? w0[r] : w1[r - 4]));
          o[r] = f2bf(rstd * (d - xhat * m));
        }
        *(bf16x8*)(dx + row * lddx + c * 8) = o;
      }
    }
  }
  // sum the four waves' partials in a fixed order: wave 0 stores, waves 1..3 add in turn
  for (int k = 0; k < NT / 64; ++k) {
    if (wv == k) {
#pragma unroll
      for (int j = 0; j < RW_NJ; ++j) {
        const int c = lane + 64 * j;
        if (c < nc) {
          const f32x4 a = {p0[j][0], p0[j][1], p0[j][2], p0[j][3]};
          const f32x4 b = {p0[j][4], p0[j][5], p0[j][6], p0[j][7]};
          if (k == 0) {
            acc[2 * c] = a;
            acc[2 * c + 1] = b;
          } else {
            acc[2 * c] = acc[2 * c] + a;
            acc[2 * c + 1] = acc[2 * c + 1] + b;
          }
        }
      }
    }
    __syncthreads();
  }
  for (int c = threadIdx.x; c < C / 4; c += NT)
    *(f32x4*)(part0 + (int64_t)blockIdx.x * C + c * 4) = acc[c];
}

// ---- RMSNorm + RoPE, column-fixed (round 6, RMS_COLS) -----------------------------------------
// Thread t of a C/16-thread workgroup owns columns [8t, 8t + 8) and [8(t + C/16), +8) of EVERY row:
// its 16 w values and its 4 RoPE pair indices are loaded once, and a workgroup streams a block of
// RC_ROWS rows RC_R at a time (2 x 16-B loads per thread per row, RC_R rows in flight), the rows'
// sums of squares reduced across the workgroup through LDS with one barrier per RC_R rows
// (double-buffered partial array).  The backward keeps its 16 d w partial sums in registers across
// the block of rows and holds each row's dout / x between its two passes.  Same per-element
// arithmetic as the kernels above; the sum of squares of a row is added in another order.
#ifndef RMS_COLS
#define RMS_COLS 2          // bit 0: forward, bit 1: backward (profiles/r06_ab_norms_cols.txt: the
#endif                      // forward runs 0.41 ms here vs 0.33 ms one-wave-per-row, 0.50 ms with
                            // the next rows prefetched before the barrier)
constexpr int RC_R = 4;             // rows in flight per workgroup (forward)
constexpr int RC_RB = 2;            // (backward: two operands held per row)
constexpr int RC_ROWS = 32;         // rows per workgroup (= prfl_norm_rows_per_part for the partial rows)
constexpr int RC_MAXT = 512;        // C <= 8192

template <bool BWD>
__device__ __forceinline__ void rc_cols(int C, int& nt, int& t, bool& act) {
  nt = C / 16;
  t = threadIdx.x;
  act = t < nt;
}

__global__ __launch_bounds__(RC_MAXT) void rms_rope_fwd_cols_kernel(
    const bf16* __restrict__ x, int64_t ldx, int L, int C, const float* __restrict__ w, float eps,
    const float2* __restrict__ tab, int F, int Hg, int Wg, int64_t row0, bf16* __restrict__ out,
    int64_t ldo, float* __restrict__ rstd_out, float oscale) {
  __shared__ float red[2][RC_R][RC_MAXT / 64];
  int nt, t;
  bool act;
  rc_cols<false>(C, nt, t, act);
  const int nw = (blockDim.x + 63) >> 6, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c0 = t * 8, c1 = (t + nt) * 8;           // element offsets of the two chunks
  const int pair0 = (c0 & 127) >> 1;                  // == (c1 & 127) >> 1: C / 16 * 8 = C / 2 % 128 == 0
  float wr[16];
  if (act) {
    const f32x4 a0 = ldf4(w, c0), a1 = ldf4(w, c0 + 4), b0 = ldf4(w, c1), b1 = ldf4(w, c1 + 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      wr[r] = a0[r];
      wr[4 + r] = a1[r];
      wr[8 + r] = b0[r];
      wr[12 + r] = b1[r];
    }
  }
  const int64_t rb = (int64_t)blockIdx.x * RC_ROWS;
  for (int it = 0; it < RC_ROWS / RC_R; ++it) {
    const int buf = it & 1;
    bf16x8 v[RC_R][2];
    float ss[RC_R];
#pragma unroll
    for (int j = 0; j < RC_R; ++j) {
      const int64_t row = rb + it * RC_R + j;
      ss[j] = 0.f;
      if (act && row < L) {
        v[j][0] = *(const bf16x8*)(x + row * ldx + c0);
        v[j][1] = *(const bf16x8*)(x + row * ldx + c1);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 8; ++r) ss[j] += bf2f(v[j][h][r]) * bf2f(v[j][h][r]);
      }
    }
#pragma unroll
    for (int j = 0; j < RC_R; ++j) {
      const float sw = wave_sum(ss[j]);
      if (lane == 0) red[buf][j][wv] = sw;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RC_R; ++j) {
      const int64_t row = rb + it * RC_R + j;
      if (row >= L) break;
      float tot = 0.f;
      for (int k = 0; k < nw; ++k) tot += red[buf][j][k];
      const float rstd = rsqrtf(tot / C + eps);
      if (threadIdx.x == 0) rstd_out[row] = rstd;
      if (!act) continue;
      int pf, ph, pw;
      bool rot;
      rope_pos(row0 + row, F, Hg, Wg, pf, ph, pw, rot);
      rot = rot && tab != nullptr;
      float2 cs[4];
      if (rot) rope_cs4(tab, pair0, pf, ph, pw, cs);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float y[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) y[r] = mul_rn(bfr(bf2f(v[j][h][r]) * rstd), wr[8 * h + r]);
        bf16x8 o;
        if (rot) {
#pragma unroll
          for (int pp = 0; pp < 4; ++pp) {
            const float a = y[2 * pp], bq = y[2 * pp + 1];
            o[2 * pp] = f2bf(__fmul_rn(__fsub_rn(__fmul_rn(a, cs[pp].x), __fmul_rn(bq, cs[pp].y)), oscale));
            o[2 * pp + 1] = f2bf(__fmul_rn(__fadd_rn(__fmul_rn(a, cs[pp].y), __fmul_rn(bq, cs[pp].x)), oscale));
          }
        } else {
#pragma unroll
          for (int r = 0; r < 8; ++r) o[r] = f2bf(__fmul_rn(y[r], oscale));
        }
        *(bf16x8*)(out + row * ldo + (h ? c1 : c0)) = o;
      }
    }
  }
}

__global__ __launch_bounds__(RC_MAXT) void rms_rope_bwd_cols_kernel(
    const bf16* __restrict__ dout, int64_t lddo, const bf16* __restrict__ x, int64_t ldx,
    const float* __restrict__ rstd_in, int L, int C, const float* __restrict__ w,
    const float2* __restrict__ tab, int F, int Hg, int Wg, int64_t row0, bf16* __restrict__ dx,
    int64_t lddx, float* __restrict__ part0, float oscale) {
  __shared__ float red[2][RC_RB][RC_MAXT / 64];
  int nt, t;
  bool act;
  rc_cols<true>(C, nt, t, act);
  const int nw = (blockDim.x + 63) >> 6, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c0 = t * 8, c1 = (t + nt) * 8;
  const int pair0 = (c0 & 127) >> 1;
  float wr[16], p0[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) p0[r] = 0.f;
  if (act) {
    const f32x4 a0 = ldf4(w, c0), a1 = ldf4(w, c0 + 4), b0 = ldf4(w, c1), b1 = ldf4(w, c1 + 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      wr[r] = a0[r];
      wr[4 + r] = a1[r];
      wr[8 + r] = b0[r];
      wr[12 + r] = b1[r];
    }
  }
  // dy = the conj-rotated (dout * oscale) of one 8-element chunk
  auto rot8 = [&](const bf16x8& gq, bool rot, const float2 (&cs)[4], float (&g8)[8]) {
#pragma unroll
    for (int r = 0; r < 8; ++r) g8[r] = bf2f(gq[r]) * oscale;
    if (rot) {
#pragma unroll
      for (int pp = 0; pp < 4; ++pp) {
        const float ga = g8[2 * pp], gb = g8[2 * pp + 1];
        g8[2 * pp] = ga * cs[pp].x + gb * cs[pp].y;
        g8[2 * pp + 1] = gb * cs[pp].x - ga * cs[pp].y;
      }
    }
  };
  const int64_t rb = (int64_t)blockIdx.x * RC_ROWS;
  for (int it = 0; it < RC_ROWS / RC_RB; ++it) {
    const int buf = it & 1;
    bf16x8 gv[RC_RB][2], xv[RC_RB][2];     // the rows held (bf16) between the two passes
    float sp[RC_RB];
#pragma unroll
    for (int j = 0; j < RC_RB; ++j) {
      const int64_t row = rb + it * RC_RB + j;
      sp[j] = 0.f;
      if (act && row < L) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          gv[j][h] = *(const bf16x8*)(dout + row * lddo + (h ? c1 : c0));
          xv[j][h] = *(const bf16x8*)(x + row * ldx + (h ? c1 : c0));
        }
      }
    }
#pragma unroll
    for (int j = 0; j < RC_RB; ++j) {
      const int64_t row = rb + it * RC_RB + j;
      if (act && row < L) {
        const float rstd = rstd_in[row];
        int pf, ph, pw;
        bool rot;
        rope_pos(row0 + row, F, Hg, Wg, pf, ph, pw, rot);
        rot = rot && tab != nullptr;
        float2 cs[4];
        if (rot) rope_cs4(tab, pair0, pf, ph, pw, cs);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float g8[8];
          rot8(gv[j][h], rot, cs, g8);
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const int e = 8 * h + r;
            const float xhat = bf2f(xv[j][h][r]) * rstd;
            const float d = bfr(g8[r] * wr[e]);
            p0[e] += g8[r] * bfr(xhat);
            sp[j] += d * xhat;
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < RC_RB; ++j) {
      const float sw = wave_sum(sp[j]);
      if (lane == 0) red[buf][j][wv] = sw;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RC_RB; ++j) {
      const int64_t row = rb + it * RC_RB + j;
      if (!act || row >= L) continue;
      float tot = 0.f;
      for (int k = 0; k < nw; ++k) tot += red[buf][j][k];
      const float m = tot / C;
      const float rstd = rstd_in[row];
      int pf, ph, pw;
      bool rot;
      rope_pos(row0 + row, F, Hg, Wg, pf, ph, pw, rot);
      rot = rot && tab != nullptr;
      float2 cs[4];
      if (rot) rope_cs4(tab, pair0, pf, ph, pw, cs);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float g8[8];
        rot8(gv[j][h], rot, cs, g8);
        bf16x8 o;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int e = 8 * h + r;
          const float xhat = bf2f(xv[j][h][r]) * rstd;
          const float d = bfr(g8[r] * wr[e]);
          o[r] = f2bf(rstd * (d - xhat * m));
        }
        *(bf16x8*)(dx + row * lddx + (h ? c1 : c0)) = o;
      }
    }
  }
  if (act) {
    float* pr = part0 + (int64_t)blockIdx.x * C;
    *(f32x4*)(pr + c0) = (f32x4){p0[0], p0[1], p0[2], p0[3]};
    *(f32x4*)(pr + c0 + 4) = (f32x4){p0[4], p0[5], p0[6], p0[7]};
    *(f32x4*)(pr + c1) = (f32x4){p0[8], p0[9], p0[10], p0[11]};
    *(f32x4*)(pr + c1 + 4) = (f32x4){p0[12], p0[13], p0[14], p0[15]};
  }
}

// LN + modulate forward: one wave per row, the row (C <= 5120 -> 20 float4 chunks per lane) held
// in registers, both reductions wave shuffles (two-pass mean / variance); the per-column
// coefficients — (1 + scale, shift) or (w, b) — are staged once per workgroup in LDS and each wave
// normalises RPW rows in turn (re-reading them from L2 per row cost 8 B for every 4 B of x).
#ifndef LN_RPW
#define LN_RPW 4
#endif
// (the next row prefetched into a second register set, as RMS_WAVE_PF 2: 0.448 vs 0.449 ms at
// 720p, profiles/r06_ab_rms_prefetch.txt -- not kept)
constexpr int RPW = LN_RPW;   // rows per wave -> 16 rows per workgroup
__global__ __launch_bounds__(NT) void ln_mod_fwd_lds_kernel(
    const void* __restrict__ x, int x_bf16, int64_t ldx, int L, int C,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ w,
    const float* __restrict__ b, float eps, bf16* __restrict__ out, int64_t ldo,
    float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  __shared__ f32x4 cA[WV * 64], cB[WV * 64];
  const int nc = C / 4;
  for (int c = threadIdx.x; c < nc; c += NT) {
    if (w) {
      cA[c] = ldf4(w, c * 4);
      cB[c] = b ? ldf4(b, c * 4) : (f32x4){0, 0, 0, 0};
    } else {
      const f32x4 sc = ldf4(scale, c * 4);
      cA[c] = (f32x4){1.f + sc[0], 1.f + sc[1], 1.f + sc[2], 1.f + sc[3]};
      cB[c] = ldf4(shift, c * 4);
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t row0 = ((int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6)) * RPW;
  for (int rr = 0; rr < RPW; ++rr) {
    const int64_t row = row0 + rr;
    if (row >= L) return;
    f32x4 v[WV];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < WV; ++j) {
      const int c = lane + j * 64;
      if (c < nc) {
        v[j] = ld4(x, row * ldx + c * 4, x_bf16);
        s += v[j][0] + v[j][1] + v[j][2] + v[j][3];
      }
    }
    const float mean = wave_sum(s) / C;
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < WV; ++j) {
      const int c = lane + j * 64;
      if (c < nc) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = v[j][r] - mean;
          ss += d * d;
        }
      }
    }
    const float var = wave_sum(ss) / C;
    const float rstd = rsqrtf(var + eps);
#pragma unroll
    for (int j = 0; j < WV; ++j) {
      const int c = lane + j * 64;
      if (c < nc) {
        const f32x4 a = cA[c], bb = cB[c];
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float xh = (v[j][r] - mean) * rstd;
          if (!w && x_bf16) xh = bfr(xh);  // WanLayerNorm.type_as(x) for a bf16 input
          o[r] = f2bf(mul_rn(xh, a[r]) + bb[r]);
        }
        *(bf16x4*)(out + row * ldo + c * 4) = o;
      }
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

// ---- LN + modulate, column-fixed (round 6, LN_COLS) --------------------------------------------
// The layout of the column-fixed RMSNorm kernels: thread t of a C/16-thread workgroup owns columns
// [8t, 8t + 8) and [8(t + C/16), +8) of every row, its 16 (1 + scale | w) and (shift | b)
// coefficients in registers (no LDS staging), a block of LC_ROWS rows streamed LC_R at a time; the
// forward's two-pass mean / variance takes two cross-wave reductions per LC_R rows, the
// backward's two column sums (d scale | d w, d shift | d b) stay in registers over the block and
// its two row sums share one reduction.  Same per-element arithmetic as ln_mod_fwd_lds_kernel /
// ln_mod_bwd_kernel; the row sums add in another order.
#ifndef LN_COLS
#define LN_COLS 2           // bit 0: forward, bit 1: backward (forward 0.51 ms vs 0.46-0.49 ms for
#endif                      // ln_mod_fwd_lds_kernel; backward 1.13-1.15 ms either way)
constexpr int LC_R = 4;             // rows in flight (forward)
constexpr int LC_RB = 2;            // rows in flight (backward)

template <int N>
__device__ __forceinline__ void ld_cols(const void* p, int64_t off, int x_bf16, float (&v)[N]) {
  static_assert(N == 8, "8-element chunk");
  if (x_bf16) {
    const bf16x8 q = *(const bf16x8*)((const bf16*)p + off);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = bf2f(q[r]);
  } else {
    const f32x4 a = *(const f32x4*)((const float*)p + off), b = *(const f32x4*)((const float*)p + off + 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = a[r];
      v[r + 4] = b[r];
    }
  }
}

__global__ __launch_bounds__(RC_MAXT) void ln_mod_fwd_cols_kernel(
    const void* __restrict__ x, int x_bf16, int64_t ldx, int L, int C,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ w,
    const float* __restrict__ b, float eps, bf16* __restrict__ out, int64_t ldo,
    float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  __shared__ float red[2][2][LC_R][RC_MAXT / 64];
  const int nt = C / 16, t = threadIdx.x;
  const bool act = t < nt;
  const int nw = (blockDim.x + 63) >> 6, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c0 = t * 8, c1 = (t + nt) * 8;
  float ca[16], cb[16];
  if (act) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = h ? c1 : c0;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const f32x4 A = w ? ldf4(w, c + 4 * q) : ldf4(scale, c + 4 * q);
        const f32x4 Bv = w ? (b ? ldf4(b, c + 4 * q) : (f32x4){0, 0, 0, 0}) : ldf4(shift, c + 4 * q);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ca[8 * h + 4 * q + r] = w ? A[r] : 1.f + A[r];
          cb[8 * h + 4 * q + r] = Bv[r];
        }
      }
    }
  }
  const int64_t rb = (int64_t)blockIdx.x * RC_ROWS;
  for (int it = 0; it < RC_ROWS / LC_R; ++it) {
    const int buf = it & 1;
    float v[LC_R][16], ps[LC_R];
#pragma unroll
    for (int j = 0; j < LC_R; ++j) {
      const int64_t row = rb + it * LC_R + j;
      ps[j] = 0.f;
      if (act && row < L) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float q8[8];
          ld_cols(x, row * ldx + (h ? c1 : c0), x_bf16, q8);
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            v[j][8 * h + r] = q8[r];
            ps[j] += q8[r];
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < LC_R; ++j) {
      const float sw = wave_sum(ps[j]);
      if (lane == 0) red[buf][0][j][wv] = sw;
    }
    __syncthreads();
    float mean[LC_R];
#pragma unroll
    for (int j = 0; j < LC_R; ++j) {
      float tot = 0.f;
      for (int k = 0; k < nw; ++k) tot += red[buf][0][j][k];
      mean[j] = tot / C;
      float sq = 0.f;
      if (act) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float d = v[j][e] - mean[j];
          sq += d * d;
        }
      }
      const float sw = wave_sum(sq);
      if (lane == 0) red[buf][1][j][wv] = sw;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < LC_R; ++j) {
      const int64_t row = rb + it * LC_R + j;
      if (row >= L) break;
      float tot = 0.f;
      for (int k = 0; k < nw; ++k) tot += red[buf][1][j][k];
      const float rstd = rsqrtf(tot / C + eps);
      if (threadIdx.x == 0) {
        mean_out[row] = mean[j];
        rstd_out[row] = rstd;
      }
      if (!act) continue;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        bf16x8 o;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int e = 8 * h + r;
          float xh = (v[j][e] - mean[j]) * rstd;
          if (!w && x_bf16) xh = bfr(xh);  // WanLayerNorm.type_as(x) for a bf16 input
          o[r] = f2bf(mul_rn(xh, ca[e]) + cb[e]);
        }
        *(bf16x8*)(out + row * ldo + (h ? c1 : c0)) = o;
      }
    }
  }
}

__global__ __launch_bounds__(RC_MAXT) void ln_mod_bwd_cols_kernel(
    const bf16* __restrict__ dy, int64_t lddy, const void* __restrict__ x, int x_bf16, int64_t ldx,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, int L, int C,
    const float* __restrict__ scale, const float* __restrict__ w, float* __restrict__ dx,
    int64_t lddx, int dx_accumulate, float* __restrict__ part0, float* __restrict__ part1) {
  __shared__ float red[2][2][LC_RB][RC_MAXT / 64];
  const int nt = C / 16, t = threadIdx.x;
  const bool act = t < nt;
  const int nw = (blockDim.x + 63) >> 6, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c0 = t * 8, c1 = (t + nt) * 8;
  float m[16], p0[16], p1[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) p0[e] = p1[e] = 0.f;
  if (act) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const f32x4 A = w ? ldf4(w, (h ? c1 : c0) + 4 * q) : ldf4(scale, (h ? c1 : c0) + 4 * q);
#pragma unroll
        for (int r = 0; r < 4; ++r) m[8 * h + 4 * q + r] = w ? A[r] : 1.f + A[r];
      }
  }
  const int64_t rb = (int64_t)blockIdx.x * RC_ROWS;
  for (int it = 0; it < RC_ROWS / LC_RB; ++it) {
    const int buf = it & 1;
    bf16x8 dv[LC_RB][2];                  // (x is re-read in the second pass: L1 / L2)
    float s1[LC_RB], s2[LC_RB];
#pragma unroll
    for (int j = 0; j < LC_RB; ++j) {
      const int64_t row = rb + it * LC_RB + j;
      s1[j] = s2[j] = 0.f;
      if (act && row < L) {
        const float mean = mean_in[row], rstd = rstd_in[row];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float q8[8];
          ld_cols(x, row * ldx + (h ? c1 : c0), x_bf16, q8);
          dv[j][h] = *(const bf16x8*)(dy + row * lddy + (h ? c1 : c0));
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const int e = 8 * h + r;
            const float xhat = (q8[r] - mean) * rstd;
            const float d = bf2f(dv[j][h][r]);
            const float xu = (!w && x_bf16) ? bfr(xhat) : xhat;
            p0[e] += d * xu;
            p1[e] += d;
            const float gg = d * m[e];
            s1[j] += gg;
            s2[j] += gg * xhat;
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < LC_RB; ++j) {
      const float a = wave_sum(s1[j]), c = wave_sum(s2[j]);
      if (lane == 0) {
        red[buf][0][j][wv] = a;
        red[buf][1][j][wv] = c;
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < LC_RB; ++j) {
      const int64_t row = rb + it * LC_RB + j;
      if (!act || row >= L) continue;
      float t1 = 0.f, t2 = 0.f;
      for (int k = 0; k < nw; ++k) {
        t1 += red[buf][0][j][k];
        t2 += red[buf][1][j][k];
      }
      const float m1 = t1 / C, m2 = t2 / C;
      const float mean = mean_in[row], rstd = rstd_in[row];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float* dp = dx + row * lddx + (h ? c1 : c0);
        float q8[8];
        ld_cols(x, row * ldx + (h ? c1 : c0), x_bf16, q8);
        f32x4 o[2];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int e = 8 * h + r;
          const float xhat = (q8[r] - mean) * rstd;
          const float gg = bf2f(dv[j][h][r]) * m[e];
          o[r >> 2][r & 3] = rstd * (gg - m1 - xhat * m2);
        }
        if (dx_accumulate) {
          o[0] = o[0] + *(const f32x4*)dp;
          o[1] = o[1] + *(const f32x4*)(dp + 4);
        }
        *(f32x4*)dp = o[0];
        *(f32x4*)(dp + 4) = o[1];
      }
    }
  }
  if (act) {
    float* q0 = part0 + (int64_t)blockIdx.x * C;
    float* q1 = part1 + (int64_t)blockIdx.x * C;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = h ? c1 : c0;
      *(f32x4*)(q0 + c) = (f32x4){p0[8 * h], p0[8 * h + 1], p0[8 * h + 2], p0[8 * h + 3]};
      *(f32x4*)(q0 + c + 4) = (f32x4){p0[8 * h + 4], p0[8 * h + 5], p0[8 * h + 6], p0[8 * h + 7]};
      *(f32x4*)(q1 + c) = (f32x4){p1[8 * h], p1[8 * h + 1], p1[8 * h + 2], p1[8 * h + 3]};
      *(f32x4*)(q1 + c + 4) = (f32x4){p1[8 * h + 4], p1[8 * h + 5], p1[8 * h + 6], p1[8 * h + 7]};
    }
  }
}

constexpr int BWD_ROWS = 32;
bool bad_c(int64_t C) { return C <= 0 || (C % 4) != 0 || C > 4 * MAXV * NT; }
// the column-fixed RMSNorm+RoPE kernels: C / 16 threads, two 16-B chunks per thread per row
bool cols_ok(const void* a, int64_t lda, const void* b, int64_t ldb, int64_t C) {
  return C % 256 == 0 && C / 16 <= RC_MAXT && lda % 8 == 0 && ldb % 8 == 0 &&
         ((uintptr_t)a & 15) == 0 && ((uintptr_t)b & 15) == 0;
}
// the one-wave-per-row RMSNorm+RoPE kernels: 16-B chunks of both row-major operands
bool wave_ok(const void* a, int64_t lda, const void* b, int64_t ldb, int64_t C) {
  return C % 8 == 0 && C <= 64 * RW_NJ * 8 && lda % 8 == 0 && ldb % 8 == 0 &&
         ((uintptr_t)a & 15) == 0 && ((uintptr_t)b & 15) == 0;
}
}  // namespace

extern "C" int prfl_norm_rows_per_part(void) { return BWD_ROWS; }

extern "C" int prfl_ln_mod_fwd(const void* x, int x_bf16, int64_t ldx, int64_t L, int64_t C,
                               const float* scale, const float* shift, const float* w,
                               const float* b, float eps, void* out, int64_t ldo, float* mean,
                               float* rstd, void* stream) {
  if (L <= 0) return 0;
  if (bad_c(C) || (!w && (!scale || !shift))) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  prfl_prof::begin(KID_LN, s);
  if ((LN_COLS & 1) && cols_ok(x, ldx * (x_bf16 ? 1 : 2), out, ldo, C)) {
    hipLaunchKernelGGL(ln_mod_fwd_cols_kernel, dim3((L + RC_ROWS - 1) / RC_ROWS),
                       dim3(((C / 16) + 63) / 64 * 64), 0, s, x, x_bf16, ldx, (int)L, (int)C, scale,
                       shift, w, b, eps, (bf16*)out, ldo, mean, rstd);
  } else {
    hipLaunchKernelGGL(ln_mod_fwd_lds_kernel, dim3((L + NT / 64 * RPW - 1) / (NT / 64 * RPW)),
                       dim3(NT), 0, s, x, x_bf16, ldx, (int)L, (int)C, scale, shift, w, b, eps,
                       (bf16*)out, ldo, mean, rstd);
  }
  prfl_prof::set_work((double)L * C * ((x_bf16 ? 2 : 4) + 2));
  prfl_prof::end(KID_LN, s);
  PRFL_LAUNCH_CHECK();
  return 0;
}

extern "C" int prfl_ln_mod_bwd(const void* dy, int64_t lddy, const void* x, int x_bf16,
                               int64_t ldx, const float* mean, const float* rstd, int64_t L,
                               int64_t C, const float* scale, const float* w, float* dx,
                               int64_t lddx, int dx_accumulate, float* part0, float* part1,
                               void* stream) {
  if (L <= 0) return 0;
  if (bad_c(C) || (!w && !scale)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  prfl_prof::begin(KID_LN, s);
  if ((LN_COLS & 2) && cols_ok(x, ldx * (x_bf16 ? 1 : 2), dy, lddy, C) && cols_ok(dx, lddx * 2, dx, lddx * 2, C)) {
    hipLaunchKernelGGL(ln_mod_bwd_cols_kernel, dim3((L + RC_ROWS - 1) / RC_ROWS),
                       dim3(((C / 16) + 63) / 64 * 64), 0, s, (const bf16*)dy, lddy, x, x_bf16, ldx,
                       mean, rstd, (int)L, (int)C, scale, w, dx, lddx, dx_accumulate, part0, part1);
  } else {
    hipLaunchKernelGGL(ln_mod_bwd_kernel<BWD_ROWS>, dim3((L + BWD_ROWS - 1) / BWD_ROWS), dim3(NT),
                       0, s, (const bf16*)dy, lddy, x, x_bf16, ldx, mean, rstd, (int)L, (int)C, scale,
                       w, dx, lddx, dx_accumulate, part0, part1);
  }
  prfl_prof::set_work((double)L * C * (2 + (x_bf16 ? 2 : 4) + 4 + (dx_accumulate ? 4 : 0)));
  prfl_prof::end(KID_LN, s);
  PRFL_LAUNCH_CHECK();
  return 0;
}

extern "C" int prfl_rms_rope_fwd_pos(const void* x, int64_t ldx, int64_t L, int64_t C,
                                     const float* w, float eps, const float* rope_tab, int64_t F,
                                     int64_t Hg, int64_t Wg, int64_t row0, void* out, int64_t ldo,
                                     float* rstd, float out_scale, void* stream) {
  if (L <= 0) return 0;
  if (bad_c(C) || row0 < 0) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  prfl_prof::begin(KID_RMS, s);
  // (round 3: a one-wave-per-row form with the table loads hoisted ran 0.545 vs 0.456 ms at 720p,
  // profiles/r03_ab_rms_rope_wave.txt; round 6's RMS_WAVE form adds 16-B chunks, w in LDS and
  // several rows per wave: profiles/r06_ab_norms.txt)
  if ((RMS_COLS & 1) && cols_ok(x, ldx, out, ldo, C)) {
    hipLaunchKernelGGL(rms_rope_fwd_cols_kernel, dim3((L + RC_ROWS - 1) / RC_ROWS),
                       dim3(((C / 16) + 63) / 64 * 64), 0, s, (const bf16*)x, ldx, (int)L, (int)C, w,
                       eps, (const float2*)rope_tab, (int)F, (int)Hg, (int)Wg, row0, (bf16*)out, ldo,
                       rstd, out_scale);
  } else if (RMS_WAVE && wave_ok(x, ldx, out, ldo, C)) {
    const int64_t rows = NT / 64 * RW_RPW;
    hipLaunchKernelGGL(rms_rope_fwd_wave_kernel, dim3((L + rows - 1) / rows), dim3(NT), 0, s,
                       (const bf16*)x, ldx, (int)L, (int)C, w, eps, (const float2*)rope_tab, (int)F,
                       (int)Hg, (int)Wg, row0, (bf16*)out, ldo, rstd, out_scale);
  } else {
    hipLaunchKernelGGL(rms_rope_fwd_kernel, dim3(L), dim3(NT), 0, s, (const bf16*)x, ldx, (int)C,
                       w, eps, (const float2*)rope_tab, (int)F, (int)Hg, (int)Wg, row0, (bf16*)out,
                       ldo, rstd, out_scale);
  }
  prfl_prof::set_work((double)L * C * 4);
  prfl_prof::end(KID_RMS, s);
  PRFL_LAUNCH_CHECK();
  return 0;
}

extern "C" int prfl_rms_rope_bwd_pos(const void* dout, int64_t lddo, const void* x, int64_t ldx,
                                     const float* rstd, int64_t L, int64_t C, const float* w,
                                     const float* rope_tab, int64_t F, int64_t Hg, int64_t Wg,
                                     int64_t row0, void* dx, int64_t lddx, float* part0,
                                     float out_scale, void* stream) {
  if (L <= 0) return 0;
  if (bad_c(C) || row0 < 0) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  prfl_prof::begin(KID_RMS, s);
  if ((RMS_COLS & 2) && cols_ok(x, ldx, dx, lddx, C) && cols_ok(dout, lddo, dout, lddo, C)) {
    static_assert(RC_ROWS == BWD_ROWS, "one partial row per prfl_norm_rows_per_part rows");
    hipLaunchKernelGGL(rms_rope_bwd_cols_kernel, dim3((L + RC_ROWS - 1) / RC_ROWS),
                       dim3(((C / 16) + 63) / 64 * 64), 0, s, (const bf16*)dout, lddo, (const bf16*)x,
                       ldx, rstd, (int)L, (int)C, w, (const float2*)rope_tab, (int)F, (int)Hg,
                       (int)Wg, row0, (bf16*)dx, lddx, part0, out_scale);
  } else if (RMS_WAVE && wave_ok(x, ldx, dx, lddx, C) && wave_ok(dout, lddo, dout, lddo, C)) {
    hipLaunchKernelGGL(rms_rope_bwd_wave_kernel<BWD_ROWS>, dim3((L + BWD_ROWS - 1) / BWD_ROWS),
                       dim3(NT), 0, s, (const bf16*)dout, lddo, (const bf16*)x, ldx, rstd, (int)L,
                       (int)C, w, (const float2*)rope_tab, (int)F, (int)Hg, (int)Wg, row0,
                       (bf16*)dx, lddx, part0, out_scale);
  } else {
    hipLaunchKernelGGL(rms_rope_bwd_kernel<BWD_ROWS>, dim3((L + BWD_ROWS - 1) / BWD_ROWS),
                       dim3(NT), 0, s, (const bf16*)dout, lddo, (const bf16*)x, ldx, rstd, (int)L,
                       (int)C, w, (const float2*)rope_tab, (int)F, (int)Hg, (int)Wg, row0,
                       (bf16*)dx, lddx, part0, out_scale);
  }
  prfl_prof::set_work((double)L * C * 6);
  prfl_prof::end(KID_RMS, s);
  PRFL_LAUNCH_CHECK();
  return 0;
}

// the round-3 entries: positions counted from row 0
extern "C" int prfl_rms_rope_fwd_scaled(const void* x, int64_t ldx, int64_t L, int64_t C,
                                        const float* w, float eps, const float* rope_tab,
                                        int64_t F, int64_t Hg, int64_t Wg, void* out, int64_t ldo,
                                        float* rstd, float out_scale, void* stream) {
  return prfl_rms_rope_fwd_pos(x, ldx, L, C, w, eps, rope_tab, F, Hg, Wg, 0, out, ldo, rstd,
                               out_scale, stream);
}

extern "C" int prfl_rms_rope_bwd_scaled(const void* dout, int64_t lddo, const void* x,
                                        int64_t ldx, const float* rstd, int64_t L, int64_t C,
                                        const float* w, const float* rope_tab, int64_t F,
                                        int64_t Hg, int64_t Wg, void* dx, int64_t lddx,
                                        float* part0, float out_scale, void* stream) {
  return prfl_rms_rope_bwd_pos(dout, lddo, x, ldx, rstd, L, C, w, rope_tab, F, Hg, Wg, 0, dx, lddx,
                               part0, out_scale, stream);
}
