// Fused FlowUniPC (bh2, order <= 2, x0-prediction) sampler update and its backward.
//
// One pass over the latent replaces the ~25 element-wise torch ops of one
// FlowUniPCMultistepScheduler.step (diffusers_lite/wan/utils/fm_solvers_unipc.py:655-739):
//   convert_model_output  m_t = x - sigma * v                                   (:321)
//   UniC corrector        x_c = bf16(r*x_last - c1*m0 - aBh*(rho0*D1 + rhoL*(m_t - m0)))   (:486-626)
//   UniP predictor        prev = bf16(r'*x_c - c1'*m_t - aBh'*(0.5*D1'))       (:350-484)
// The scalar coefficients are host-side 0-dim fp32 values exactly as the reference computes
// them; every per-element operation below is one IEEE fp32 op in the reference's order and
// with its bf16 rounding points (a bf16 sample times a scalar rounds to bf16; everything that
// touches an fp32 model output stays fp32), so the result is bit-identical to the reference's
// torch chain on CPU.  No FMA contraction anywhere in this file.  `scalar * bf16_tensor` with the
// 0-dim scalar on the LEFT casts the scalar to the bf16 common dtype first (ATen's reduced-float
// scalar fast path only covers the right operand), hence bf16(bf16(r) * x); autograd's
// `grad * scalar` keeps the fp32 scalar.
//
// The backward is the transpose of that linear map as torch autograd evaluates it (same
// rounding of the gradient to bf16 where autograd casts it to a bf16 input's dtype, and the
// same accumulation order into m_t: D1 path, then c1 path, then the corrector path).
#include <string.h>

#include "common.h"

#pragma clang fp contract(off)

namespace {
constexpr int NT = 256;

struct UniPCCoef {
  float sig;                                     // sigma_i of convert_model_output
  int corr;                                      // 0: no corrector, 1/2: corrector order
  float c_r, c_c1, c_rk, c_rho0, c_rhoL, c_aBh;  // UniC: sig_t/sig_s0, alpha_t*h_phi_1, rk, rhos, alpha_t*B_h
  int pred;                                      // predictor order 1/2
  float p_r, p_c1, p_rk, p_aBh;                  // UniP
};

__device__ __forceinline__ float bfr_(float x) { return (float)(bf16)x; }

__device__ __forceinline__ void unipc_elem(const UniPCCoef& k, float s, float mo, float xl,
                                           float h1, float h2, float& mt, float& xc,
                                           float& pv) {
  const float t1 = k.sig * mo;
  mt = s - t1;
  float x = s;
  if (k.corr) {
    const float xr = bfr_(bfr_(k.c_r) * xl);
    const float q = k.c_c1 * h1;
    const float xt = xr - q;
    float w;
    if (k.corr == 2) {
      const float d1 = (h2 - h1) / k.c_rk;
      const float cr = k.c_rho0 * d1;
      const float v = k.c_rhoL * (mt - h1);
      w = cr + v;
    } else {
      const float v = k.c_rhoL * (mt - h1);
      w = 0.0f + v;
    }
    const float z = k.c_aBh * w;
    x = bfr_(xt - z);
  }
  xc = x;
  const float xr = bfr_(bfr_(k.p_r) * x);
  const float q = k.p_c1 * mt;
  float xt = xr - q;
  if (k.pred == 2) {
    const float d1 = (h1 - mt) / k.p_rk;
    const float s1 = 0.5f * d1;
    const float s2 = k.p_aBh * s1;
    xt = xt - s2;
  }
  pv = xt;
}

// d prev (bf16) -> d model_output (fp32)
__device__ __forceinline__ float unipc_elem_bwd(const UniPCCoef& k, float g) {
  float gm;
  const float g_q = -g;
  const float b = g_q * k.p_c1;
  if (k.pred == 2) {
    const float g_s1 = (-g) * k.p_aBh;
    const float g_d1 = g_s1 * 0.5f;
    const float a = -(g_d1 / k.p_rk);
    gm = a + b;
  } else {
    gm = b;
  }
  if (k.corr) {
    const float g_xr = bfr_(g);
    const float g_y = bfr_(g_xr * k.p_r);
    const float g_w = (-g_y) * k.c_aBh;
    const float c = g_w * k.c_rhoL;
    gm = gm + c;
  }
  return (-gm) * k.sig;
}

__global__ __launch_bounds__(NT) void unipc_fwd_kernel(
    UniPCCoef k, const bf16* __restrict__ sample, const float* __restrict__ mo,
    const bf16* __restrict__ last, const float* __restrict__ h1, const float* __restrict__ h2,
    float* __restrict__ mt_out, bf16* __restrict__ xc_out, bf16* __restrict__ prev, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * NT + threadIdx.x) * 4;
  if (i >= n) return;
  if (i + 4 <= n) {
    const bf16x4 s = *(const bf16x4*)(sample + i);
    const f32x4 m = *(const f32x4*)(mo + i);
    bf16x4 xl = s;
    f32x4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
    if (k.corr) {
      xl = *(const bf16x4*)(last + i);
      a = *(const f32x4*)(h1 + i);
      if (k.corr == 2) b = *(const f32x4*)(h2 + i);
    }
    if (k.pred == 2 && !k.corr) a = *(const f32x4*)(h1 + i);
    f32x4 mt;
    bf16x4 xc, pv;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x, p, t;
      unipc_elem(k, bf2f(s[r]), m[r], bf2f(xl[r]), a[r], b[r], t, x, p);
      mt[r] = t;
      xc[r] = f2bf(x);
      pv[r] = f2bf(p);
    }
    *(f32x4*)(mt_out + i) = mt;
    if (xc_out) *(bf16x4*)(xc_out + i) = xc;
    *(bf16x4*)(prev + i) = pv;
  } else {
    for (int64_t j = i; j < n; ++j) {
      const float xl = k.corr ? bf2f(last[j]) : 0.f;
      const float a = (k.corr || k.pred == 2) ? h1[j] : 0.f;
      const float b = k.corr == 2 ? h2[j] : 0.f;
      float mt, x, p;
      unipc_elem(k, bf2f(sample[j]), mo[j], xl, a, b, mt, x, p);
      mt_out[j] = mt;
      if (xc_out) xc_out[j] = f2bf(x);
      prev[j] = f2bf(p);
    }
  }
}

__global__ __launch_bounds__(NT) void unipc_bwd_kernel(UniPCCoef k, const bf16* __restrict__ gp,
                                                       float* __restrict__ gmo, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * NT + threadIdx.x) * 4;
  if (i >= n) return;
  if (i + 4 <= n) {
    const bf16x4 g = *(const bf16x4*)(gp + i);
    f32x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = unipc_elem_bwd(k, bf2f(g[r]));
    *(f32x4*)(gmo + i) = o;
  } else {
    for (int64_t j = i; j < n; ++j) gmo[j] = unipc_elem_bwd(k, bf2f(gp[j]));
  }
}

// host-side round-to-nearest-even to bf16 (the reference casts the solved rhos to the sample
// dtype, fm_solvers_unipc.py:612); NaN/inf pass through
float round_bf16(float x) {
  uint32_t u;
  memcpy(&u, &x, 4);
  if ((u & 0x7f800000u) != 0x7f800000u) u = (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u;
  float r;
  memcpy(&r, &u, 4);
  return r;
}

bool load_coef(const float* c, int corr, int pred, UniPCCoef& k) {
  if (corr < 0 || corr > 2 || pred < 1 || pred > 2 || !c) return false;
  k.sig = c[0];
  k.corr = corr;
  k.c_r = c[1]; k.c_c1 = c[2]; k.c_rk = c[3]; k.c_aBh = c[6];
  k.c_rho0 = round_bf16(c[4]);
  k.c_rhoL = round_bf16(c[5]);
  k.pred = pred;
  k.p_r = c[7]; k.p_c1 = c[8]; k.p_rk = c[9]; k.p_aBh = c[10];
  return true;
}

bool aligned(const void* p) { return ((uintptr_t)p & 15) == 0; }
}  // namespace

extern "C" int prfl_unipc_step(const void* sample, const float* model_output,
                               const void* last_sample, const float* hist1, const float* hist2,
                               float* m_t, void* sample_c, void* prev, int64_t n,
                               const float* coef, int corr_order, int pred_order, void* stream) {
  if (n <= 0) return 0;
  UniPCCoef k;
  if (!load_coef(coef, corr_order, pred_order, k)) return (int)hipErrorInvalidValue;
  if (!sample || !model_output || !m_t || !prev) return (int)hipErrorInvalidValue;
  if (corr_order && (!last_sample || !hist1)) return (int)hipErrorInvalidValue;
  if (corr_order == 2 && !hist2) return (int)hipErrorInvalidValue;
  if (pred_order == 2 && !hist1) return (int)hipErrorInvalidValue;
  // bf16 operands are read 8 B at a time, fp32 16 B at a time
  const void* ptrs[] = {model_output, hist1, hist2, m_t};
  for (const void* p : ptrs)
    if (p && !aligned(p)) return (int)hipErrorInvalidValue;
  const void* bptrs[] = {sample, last_sample, sample_c, prev};
  for (const void* p : bptrs)
    if (p && ((uintptr_t)p & 7)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  prfl_prof::begin(KID_ELTWISE, s);
  hipLaunchKernelGGL(unipc_fwd_kernel, dim3((n / 4 + NT) / NT), dim3(NT), 0, s, k,
                     (const bf16*)sample, model_output, (const bf16*)last_sample, hist1, hist2,
                     m_t, (bf16*)sample_c, (bf16*)prev, n);
  prfl_prof::set_work((double)n * (2 + 4 + 4 + 2 + (corr_order ? 2 + 4 : 0) +
                                   (corr_order == 2 ? 4 : 0) + (corr_order ? 2 : 0)));
  prfl_prof::end(KID_ELTWISE, s);
  PRFL_LAUNCH_CHECK();
  return 0;
}

extern "C" int prfl_unipc_step_bwd(const void* grad_prev, float* grad_model_output, int64_t n,
                                   const float* coef, int corr_order, int pred_order,
                                   void* stream) {
  if (n <= 0) return 0;
  UniPCCoef k;
  if (!load_coef(coef, corr_order, pred_order, k)) return (int)hipErrorInvalidValue;
  if (!grad_prev || !grad_model_output) return (int)hipErrorInvalidValue;
  if (((uintptr_t)grad_prev & 7) || !aligned(grad_model_output)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(unipc_bwd_kernel, dim3((n / 4 + NT) / NT), dim3(NT), 0, s, k,
                     (const bf16*)grad_prev, grad_model_output, n);
  PRFL_LAUNCH_CHECK();
  return 0;
}
