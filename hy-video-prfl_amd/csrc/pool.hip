// Single-query attention pooling of the PAVRM / PRFL reward head (QueryAttention,
// `diffusers_lite/utils/network.py:80`: nn.MultiheadAttention with ONE learned query, 8 heads,
// E = 5120, over the L tokens of the latent reward model's block-8 features).
//
//   o_h = sum_l softmax_l(q_h . k_{l,h} * scale) v_{l,h}          (per sample, per head)
//
// K and V are the two halves of the MHA in-projection output kv [N][L][2E] (bf16, row stride
// ldkv), read once: the pooling is HBM-bound (2 * E * 2 B per token: 20 KB at E = 5120; 1.5 GB
// per sample at 720p x 81f).  Split over L (flash-decoding): workgroup (split, head, sample)
// streams a contiguous chunk of keys with 4 waves, each wave owning every 4th group of U keys;
// a lane holds 16-B pieces p = lane + 64 j of the head's hd = E / H elements (hd % 8 == 0,
// hd <= 1024), so one token-head row is read by one wave as full 16-B lanes.  Per key group:
// U dot products reduced across the wave (interleaved butterflies), an online-softmax update
// with P rounded to bf16 for P.V (flash-attention numerics, as the oracle and flash_attn use),
// fp32 row sum.  The workgroup's four waves merge in LDS; a second kernel merges the splits and
// writes o (bf16) and the log2-domain LSE.
//
// Backward (recomputation, no atomics): D_h = do_h . o_h with the fp32 o the forward also writes
// (NOT flash-attention's bf16 O: with one query over up to 74k nearly uniform keys, dp - D is a
// cancellation and D from a bf16-rounded o costs the key-side gradient several % — the
// reference's SDPA backward differentiates the unrounded output); per key p = exp2(s*sl2 - lse2),
// dp = do_h . v, ds = p (dp - D); dk = scale ds q_h and dv = p do_h are written straight into
// dkv [N][L][2E] (bf16, the in-projection's dY), dq_h += ds k accumulates per wave, merged per
// workgroup into a split partial, summed by the merge kernel.
#include "common.h"

namespace {
constexpr int PNT = 256;         // 4 waves
constexpr int PU = 4;            // keys per wave iteration
constexpr int PMAXJ = 2;         // pieces per lane: hd <= 64 * 8 * PMAXJ = 1024

struct PoolArgs {
  const bf16* q;   int64_t ldq;      // [N][E] row stride
  const bf16* kv;  int64_t ldkv, bkv;   // row stride (tokens), sample stride
  int N, L, H, hd, E;
  float sl2;                         // scale * log2(e)
  float scale;
  int nsplit, chunk;                 // keys per split
  float* part_m; float* part_l; float* part_o;   // [N][H][nsplit] (+ [hd])
};

__device__ __forceinline__ void load8(const bf16* p, float (&f)[8]) {
  const bf16x8 v = *(const bf16x8*)p;
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = bf2f(v[i]);
}

__global__ __launch_bounds__(PNT) void pool_fwd_kernel(PoolArgs a) {
  __shared__ float red[4][2 + 1024];
  const int split = blockIdx.x, h = blockIdx.y, n = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int npc = a.hd / 8;
  const int l0 = split * a.chunk, l1 = min(a.L, l0 + a.chunk);
  float qf[PMAXJ][8];
#pragma unroll
  for (int j = 0; j < PMAXJ; ++j) {
    const int pc = lane + 64 * j;
    if (pc < npc) load8(a.q + (int64_t)n * a.ldq + h * a.hd + pc * 8, qf[j]);
    else
#pragma unroll
      for (int i = 0; i < 8; ++i) qf[j][i] = 0.f;
  }
  float o[PMAXJ][8];
#pragma unroll
  for (int j = 0; j < PMAXJ; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) o[j][i] = 0.f;
  float m = -__builtin_huge_valf(), lsum = 0.f;
  const bf16* kb = a.kv + (int64_t)n * a.bkv + h * a.hd;
  const bf16* vb = kb + a.E;
  for (int g0 = l0 + w * PU; g0 < l1; g0 += 4 * PU) {
    float s[PU];
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      s[u] = 0.f;
      const int l = g0 + u;
      if (l < l1) {
#pragma unroll
        for (int j = 0; j < PMAXJ; ++j) {
          const int pc = lane + 64 * j;
          if (pc < npc) {
            float kf[8];
            load8(kb + (int64_t)l * a.ldkv + pc * 8, kf);
#pragma unroll
            for (int i = 0; i < 8; ++i) s[u] += qf[j][i] * kf[i];
          }
        }
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
      for (int u = 0; u < PU; ++u) s[u] += __shfl_xor(s[u], off, 64);
    float mx = m;
#pragma unroll
    for (int u = 0; u < PU; ++u)
      if (g0 + u < l1) mx = fmaxf(mx, s[u] * a.sl2);
    const float alpha = __builtin_amdgcn_exp2f(m - mx);
    m = mx;
    lsum *= alpha;
#pragma unroll
    for (int j = 0; j < PMAXJ; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) o[j][i] *= alpha;
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int l = g0 + u;
      if (l < l1) {
        const float p = __builtin_amdgcn_exp2f(s[u] * a.sl2 - m);
        lsum += p;
        const float pb = bfr(p);
#pragma unroll
        for (int j = 0; j < PMAXJ; ++j) {
          const int pc = lane + 64 * j;
          if (pc < npc) {
            float vf[8];
            load8(vb + (int64_t)l * a.ldkv + pc * 8, vf);
#pragma unroll
            for (int i = 0; i < 8; ++i) o[j][i] += pb * vf[i];
          }
        }
      }
    }
  }
  // merge the 4 waves of the workgroup
  if (lane == 0) {
    red[w][0] = m;
    red[w][1] = lsum;
  }
#pragma unroll
  for (int j = 0; j < PMAXJ; ++j) {
    const int pc = lane + 64 * j;
    if (pc < npc)
#pragma unroll
      for (int i = 0; i < 8; ++i) red[w][2 + pc * 8 + i] = o[j][i];
  }
  __syncthreads();
  float M = fmaxf(fmaxf(red[0][0], red[1][0]), fmaxf(red[2][0], red[3][0]));
  float f[4], Ls = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[k] = red[k][0] == -__builtin_huge_valf() ? 0.f : __builtin_amdgcn_exp2f(red[k][0] - M);
    Ls += red[k][1] * f[k];
  }
  const int64_t pidx = ((int64_t)n * a.H + h) * a.nsplit + split;
  if (threadIdx.x == 0) {
    a.part_m[pidx] = M;
    a.part_l[pidx] = Ls;
  }
  for (int d = threadIdx.x; d < a.hd; d += PNT) {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) acc += red[k][2 + d] * f[k];
    a.part_o[pidx * a.hd + d] = acc;
  }
}

// o[n][h*hd + d] = bf16(sum_s part_o * 2^(m_s - M) / sum_s part_l * 2^(m_s - M)); lse2 = M + log2 L;
// o32 (optional) = the same before the bf16 rounding
__global__ __launch_bounds__(PNT) void pool_merge_kernel(PoolArgs a, bf16* __restrict__ o,
                                                         int64_t ldo, float* __restrict__ lse2,
                                                         float* __restrict__ o32) {
  const int h = blockIdx.x, n = blockIdx.y;
  const int64_t base = ((int64_t)n * a.H + h) * a.nsplit;
  float M = -__builtin_huge_valf();
  for (int s = 0; s < a.nsplit; ++s) M = fmaxf(M, a.part_m[base + s]);
  float Ls = 0.f;
  for (int s = 0; s < a.nsplit; ++s)
    if (a.part_m[base + s] != -__builtin_huge_valf())
      Ls += a.part_l[base + s] * __builtin_amdgcn_exp2f(a.part_m[base + s] - M);
  const float inv = 1.f / Ls;
  for (int d = threadIdx.x; d < a.hd; d += PNT) {
    float acc = 0.f;
    for (int s = 0; s < a.nsplit; ++s)
      if (a.part_m[base + s] != -__builtin_huge_valf())
        acc += a.part_o[(base + s) * a.hd + d] * __builtin_amdgcn_exp2f(a.part_m[base + s] - M);
    o[(int64_t)n * ldo + h * a.hd + d] = f2bf(acc * inv);
    if (o32) o32[(int64_t)n * a.E + h * a.hd + d] = acc * inv;
  }
  if (threadIdx.x == 0) lse2[(int64_t)n * a.H + h] = M + log2f(Ls);
}

struct PoolBwdArgs {
  PoolArgs f;
  const bf16* dout; const float* o32;   // [N][E]
  const float* lse2;                 // [N][H]
  bf16* dkv; int64_t lddkv, bdkv;
};

__global__ __launch_bounds__(PNT) void pool_bwd_kernel(PoolBwdArgs b) {
  const PoolArgs& a = b.f;
  __shared__ float red[4][1024];
  const int split = blockIdx.x, h = blockIdx.y, n = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int npc = a.hd / 8;
  const int l0 = split * a.chunk, l1 = min(a.L, l0 + a.chunk);
  float qf[PMAXJ][8], df[PMAXJ][8], dq[PMAXJ][8];
  float dd = 0.f;
#pragma unroll
  for (int j = 0; j < PMAXJ; ++j) {
    const int pc = lane + 64 * j;
#pragma unroll
    for (int i = 0; i < 8; ++i) qf[j][i] = df[j][i] = dq[j][i] = 0.f;
    if (pc < npc) {
      const int64_t off = (int64_t)n * a.ldq + h * a.hd + pc * 8;
      load8(a.q + off, qf[j]);
      load8(b.dout + off, df[j]);
      const float* op = b.o32 + (int64_t)n * a.E + h * a.hd + pc * 8;
      const f32x4 o0 = *(const f32x4*)op, o1 = *(const f32x4*)(op + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) dd += df[j][i] * o0[i] + df[j][i + 4] * o1[i];
    }
  }
  dd = wave_sum(dd);                                   // D = rowsum(dO * O), fp32 O
  const float lse = b.lse2[(int64_t)n * a.H + h];
  const bf16* kb = a.kv + (int64_t)n * a.bkv + h * a.hd;
  const bf16* vb = kb + a.E;
  bf16* dkb = b.dkv + (int64_t)n * b.bdkv + h * a.hd;
  bf16* dvb = dkb + a.E;
  for (int g0 = l0 + w * PU; g0 < l1; g0 += 4 * PU) {
    float s[PU], dp[PU];
    float kf[PU][PMAXJ][8];
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      s[u] = dp[u] = 0.f;
      const int l = g0 + u;
#pragma unroll
      for (int j = 0; j < PMAXJ; ++j) {
        const int pc = lane + 64 * j;
        if (l < l1 && pc < npc) {
          float vf[8];
          load8(kb + (int64_t)l * a.ldkv + pc * 8, kf[u][j]);
          load8(vb + (int64_t)l * a.ldkv + pc * 8, vf);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            s[u] += qf[j][i] * kf[u][j][i];
            dp[u] += df[j][i] * vf[i];
          }
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) kf[u][j][i] = 0.f;
        }
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        s[u] += __shfl_xor(s[u], off, 64);
        dp[u] += __shfl_xor(dp[u], off, 64);
      }
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int l = g0 + u;
      if (l >= l1) continue;
      const float p = __builtin_amdgcn_exp2f(s[u] * a.sl2 - lse);
      const float ds = p * (dp[u] - dd);
#pragma unroll
      for (int j = 0; j < PMAXJ; ++j) {
        const int pc = lane + 64 * j;
        if (pc < npc) {
          bf16x8 dkv8, dvv8;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            dkv8[i] = f2bf(a.scale * ds * qf[j][i]);
            dvv8[i] = f2bf(p * df[j][i]);
            dq[j][i] += ds * kf[u][j][i];
          }
          *(bf16x8*)(dkb + (int64_t)l * b.lddkv + pc * 8) = dkv8;
          *(bf16x8*)(dvb + (int64_t)l * b.lddkv + pc * 8) = dvv8;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < PMAXJ; ++j) {
    const int pc = lane + 64 * j;
    if (pc < npc)
#pragma unroll
      for (int i = 0; i < 8; ++i) red[w][pc * 8 + i] = dq[j][i];
  }
  __syncthreads();
  const int64_t pidx = ((int64_t)n * a.H + h) * a.nsplit + split;
  for (int d = threadIdx.x; d < a.hd; d += PNT)
    a.part_o[pidx * a.hd + d] = red[0][d] + red[1][d] + red[2][d] + red[3][d];
}

// dq[n][h*hd + d] = scale * sum_s part
__global__ __launch_bounds__(PNT) void pool_dq_merge_kernel(PoolArgs a, float* __restrict__ dq,
                                                            int64_t lddq) {
  const int h = blockIdx.x, n = blockIdx.y;
  const int64_t base = ((int64_t)n * a.H + h) * a.nsplit;
  for (int d = threadIdx.x; d < a.hd; d += PNT) {
    float acc = 0.f;
    for (int s = 0; s < a.nsplit; ++s) acc += a.part_o[(base + s) * a.hd + d];
    dq[(int64_t)n * lddq + h * a.hd + d] = a.scale * acc;
  }
}

bool pool_shape_ok(int64_t N, int64_t L, int64_t H, int64_t E, int64_t ldq, int64_t ldkv,
                   const void* q, const void* kv) {
  if (N <= 0 || L <= 0 || H <= 0 || E % H) return false;
  const int64_t hd = E / H;
  if (hd % 8 || hd > 64 * 8 * PMAXJ || ldq % 8 || ldkv % 8 || ldkv < 2 * E) return false;
  if (((uintptr_t)q & 15) || ((uintptr_t)kv & 15)) return false;
  return N <= 65535 && H <= 65535 && L <= 0x7fffffff;
}
}  // namespace

extern "C" int prfl_query_pool_splits(int64_t N, int64_t L, int64_t H) {
  // ~2048 workgroups, >= 64 keys each
  const int64_t want = (2048 + N * H - 1) / (N * H);
  const int64_t maxs = (L + 63) / 64;
  return (int)(want < 1 ? 1 : (want > maxs ? maxs : want));
}

extern "C" int prfl_query_pool_fwd(const void* q, int64_t ldq, const void* kv, int64_t ldkv,
                                   int64_t bkv, int64_t N, int64_t L, int64_t H, int64_t E,
                                   float scale, void* o, int64_t ldo, float* lse2, float* o32,
                                   float* part_m, float* part_l, float* part_o, int64_t nsplit,
                                   void* stream) {
  if (!pool_shape_ok(N, L, H, E, ldq, ldkv, q, kv) || nsplit <= 0 || nsplit > L)
    return (int)hipErrorInvalidValue;
  PoolArgs a{(const bf16*)q, ldq, (const bf16*)kv, ldkv, bkv, (int)N, (int)L, (int)H,
             (int)(E / H), (int)E, scale * 1.4426950408889634f, scale, (int)nsplit,
             (int)((L + nsplit - 1) / nsplit), part_m, part_l, part_o};
  hipStream_t s = (hipStream_t)stream;
  prfl_prof::begin(KID_POOL, s);
  hipLaunchKernelGGL(pool_fwd_kernel, dim3(nsplit, H, N), dim3(PNT), 0, s, a);
  PRFL_LAUNCH_CHECK();
  hipLaunchKernelGGL(pool_merge_kernel, dim3(H, N), dim3(PNT), 0, s, a, (bf16*)o, ldo, lse2, o32);
  prfl_prof::set_work((double)N * L * 2 * E * 2);
  prfl_prof::end(KID_POOL, s);
  PRFL_LAUNCH_CHECK();
  return 0;
}

extern "C" int prfl_query_pool_bwd(const void* dout, const void* q, int64_t ldq, const void* kv,
                                   int64_t ldkv, int64_t bkv, const float* o32, const float* lse2,
                                   int64_t N, int64_t L, int64_t H, int64_t E, float scale,
                                   float* dq, int64_t lddq, void* dkv, int64_t lddkv, int64_t bdkv,
                                   float* part_o, int64_t nsplit, void* stream) {
  if (!pool_shape_ok(N, L, H, E, ldq, ldkv, q, kv) || nsplit <= 0 || nsplit > L ||
      lddkv % 8 || ((uintptr_t)dkv & 15) || ((uintptr_t)dout & 15) || ((uintptr_t)o32 & 15))
    return (int)hipErrorInvalidValue;
  PoolArgs a{(const bf16*)q, ldq, (const bf16*)kv, ldkv, bkv, (int)N, (int)L, (int)H,
             (int)(E / H), (int)E, scale * 1.4426950408889634f, scale, (int)nsplit,
             (int)((L + nsplit - 1) / nsplit), nullptr, nullptr, part_o};
  PoolBwdArgs b{a, (const bf16*)dout, o32, lse2, (bf16*)dkv, lddkv, bdkv};
  hipStream_t s = (hipStream_t)stream;
  prfl_prof::begin(KID_POOL, s);
  hipLaunchKernelGGL(pool_bwd_kernel, dim3(nsplit, H, N), dim3(PNT), 0, s, b);
  PRFL_LAUNCH_CHECK();
  hipLaunchKernelGGL(pool_dq_merge_kernel, dim3(H, N), dim3(PNT), 0, s, a, dq, lddq);
  prfl_prof::set_work((double)N * L * 2 * E * 4);
  prfl_prof::end(KID_POOL, s);
  PRFL_LAUNCH_CHECK();
  return 0;
}
