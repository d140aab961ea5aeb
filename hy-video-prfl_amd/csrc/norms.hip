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
constexpr int RW_RPW = 4;     // rows per wave in the forward (16 rows per workgroup)
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
  for (int c = threadIdx.x; c < C / 4; c += NT) ws[c] = ldf4(w, c * 4);
  __syncthreads();
  const int lane = threadIdx.x & 63, nc = C / 8, pair0 = ((lane * 8) & 127) >> 1;
  const int64_t rbase = ((int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6)) * RW_RPW;
  for (int rr = 0; rr < RW_RPW; ++rr) {
    const int64_t row = rbase + rr;
    if (row >= L) return;
    bf16x8 v[RW_NJ];
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < RW_NJ; ++j) {
      const int c = lane + 64 * j;
      if (c < nc) {
        v[j] = *(const bf16x8*)(x + row * ldx + c * 8);
#pragma unroll
        for (int r = 0; r < 8; ++r) ss += bf2f(v[j][r]) * bf2f(v[j][r]);
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
          y[r] = mul_rn(bfr(bf2f(v[j][r]) * rstd), w0[r]);
          y[r + 4] = mul_rn(bfr(bf2f(v[j][r + 4]) * rstd), w1[r]);
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

// LN + modulate forward: one wave per row, the row (C <= 5120 -> 20 float4 chunks per lane) held
// in registers, both reductions wave shuffles (two-pass mean / variance); the per-column
// coefficients — (1 + scale, shift) or (w, b) — are staged once per workgroup in LDS and each wave
// normalises RPW rows in turn (re-reading them from L2 per row cost 8 B for every 4 B of x).
#ifndef LN_RPW
#define LN_RPW 4
#endif
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

constexpr int BWD_ROWS = 32;
bool bad_c(int64_t C) { return C <= 0 || (C % 4) != 0 || C > 4 * MAXV * NT; }
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
  hipLaunchKernelGGL(ln_mod_fwd_lds_kernel, dim3((L + NT / 64 * RPW - 1) / (NT / 64 * RPW)),
                     dim3(NT), 0, s, x, x_bf16, ldx, (int)L, (int)C, scale, shift, w, b, eps,
                     (bf16*)out, ldo, mean, rstd);
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
  hipLaunchKernelGGL(ln_mod_bwd_kernel<BWD_ROWS>, dim3((L + BWD_ROWS - 1) / BWD_ROWS), dim3(NT),
                     0, s, (const bf16*)dy, lddy, x, x_bf16, ldx, mean, rstd, (int)L, (int)C, scale,
                     w, dx, lddx, dx_accumulate, part0, part1);
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
  if (RMS_WAVE && wave_ok(x, ldx, out, ldo, C)) {
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
  if (RMS_WAVE && wave_ok(x, ldx, dx, lddx, C) && wave_ok(dout, lddo, dout, lddo, C)) {
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
