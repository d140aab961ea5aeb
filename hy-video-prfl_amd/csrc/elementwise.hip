// HBM-bound element-wise / reduction kernels of the PRFL step.
//
//  cast_f32_bf16   fp32 master weight -> bf16 GEMM operand (autocast weight cast)
//  gate_bwd        x_out = x_in + y*gate  ->  dy = bf16(dx*gate), partial sums of dx*y and dy
//  colsum_bf16     partial column sums of a bf16 matrix (bias gradients)
//  colsum_reduce   sum partial rows [P][N] -> out[N] (optionally accumulating)
//  sumsq           per-tensor sum of squares (grad-norm clipping, train_prfl.py:825)
//  scale           in-place x *= s[0] (clip coefficient lives on the device: no host sync)
//  adamw           torch.optim.AdamW (non-amsgrad, maximize=False) element update, fp32 state
#include "common.h"

namespace {
constexpr int NT = 256;

__global__ void cast_kernel(const float* __restrict__ src, bf16* __restrict__ dst, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * NT + threadIdx.x) * 8;
  if (i + 8 <= n) {
    const f32x4 a = *(const f32x4*)(src + i), b = *(const f32x4*)(src + i + 4);
    *(bf16x8*)(dst + i) = (bf16x8){f2bf(a[0]), f2bf(a[1]), f2bf(a[2]), f2bf(a[3]),
                                   f2bf(b[0]), f2bf(b[1]), f2bf(b[2]), f2bf(b[3])};
  } else {
    for (int64_t j = i; j < n; ++j) dst[j] = f2bf(src[j]);
  }
}

// fp32 W [N][K] (row stride ldw) -> bf16 W^T [K][N] (row stride ldo): a forward projection's
// weight as an MN-major GEMM operand (the four-wave GEMM runs 2-4 % faster on it than on the
// K-major W: its LDS-DMA pieces then fetch 256-B row runs instead of 64-B ones).  One workgroup
// per 64 x 64 tile through LDS: coalesced 16-B reads of W rows, 16-B writes of W^T rows.
__global__ __launch_bounds__(NT) void cast_t_kernel(const float* __restrict__ w, int64_t ldw,
                                                    bf16* __restrict__ out, int64_t ldo, int N, int K) {
  __shared__ float t[64][65];
  const int n0 = blockIdx.y * 64, k0 = blockIdx.x * 64, tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {                      // 64 rows (n) x 16 pieces of 4 k
    const int r = i * 16 + (tid >> 4), c = (tid & 15) * 4;
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    if (n0 + r < N && k0 + c + 3 < K) x = *(const f32x4*)(w + (int64_t)(n0 + r) * ldw + k0 + c);
    else
      for (int j = 0; j < 4; ++j)
        if (n0 + r < N && k0 + c + j < K) x[j] = w[(int64_t)(n0 + r) * ldw + k0 + c + j];
#pragma unroll
    for (int j = 0; j < 4; ++j) t[r][c + j] = x[j];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {                      // 64 rows (k) x 8 pieces of 8 n
    const int r = i * 32 + (tid >> 3), c = (tid & 7) * 8;
    if (k0 + r >= K) continue;
    bf16x8 y;
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = f2bf(t[c + j][r]);
    bf16* dst = out + (int64_t)(k0 + r) * ldo + n0 + c;
    if (n0 + c + 7 < N) *(bf16x8*)dst = y;
    else
      for (int j = 0; j < 8; ++j)
        if (n0 + c + j < N) dst[j] = y[j];
  }
}

// rows of ROWS per workgroup; thread t owns 4 columns (NT*4 = 1024 columns per workgroup)
template <int ROWS>
__global__ __launch_bounds__(NT) void gate_bwd_kernel(const float* __restrict__ dx, int64_t lddx,
                                                      const bf16* __restrict__ y, int64_t ldy,
                                                      const float* __restrict__ gate, int L, int N,
                                                      bf16* __restrict__ dy, int64_t lddy,
                                                      float* __restrict__ pgate,
                                                      float* __restrict__ pbias) {
  const int c = (blockIdx.x * NT + threadIdx.x) * 4;
  if (c >= N) return;
  const int r0 = blockIdx.y * ROWS;
  const f32x4 gt = gate ? *(const f32x4*)(gate + c) : (f32x4){1.f, 1.f, 1.f, 1.f};
  f32x4 sg = {0, 0, 0, 0}, sb = {0, 0, 0, 0};
  for (int rr = 0; rr < ROWS; ++rr) {
    const int64_t row = r0 + rr;
    if (row >= L) break;
    const f32x4 d = *(const f32x4*)(dx + row * lddx + c);
    bf16x4 o;
    if (y) {
      const bf16x4 yv = *(const bf16x4*)(y + row * ldy + c);
#pragma unroll
      for (int r = 0; r < 4; ++r) sg[r] += d[r] * bf2f(yv[r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      o[r] = f2bf(d[r] * gt[r]);
      sb[r] += bf2f(o[r]);
    }
    *(bf16x4*)(dy + row * lddy + c) = o;
  }
  if (pgate) *(f32x4*)(pgate + (int64_t)blockIdx.y * N + c) = sg;
  if (pbias) *(f32x4*)(pbias + (int64_t)blockIdx.y * N + c) = sb;
}

template <int ROWS>
__global__ __launch_bounds__(NT) void colsum_bf16_kernel(const bf16* __restrict__ x, int64_t ld,
                                                         int L, int N, float* __restrict__ part) {
  const int c = (blockIdx.x * NT + threadIdx.x) * 4;
  if (c >= N) return;
  const int r0 = blockIdx.y * ROWS;
  f32x4 s = {0, 0, 0, 0};
  for (int rr = 0; rr < ROWS; ++rr) {
    const int64_t row = r0 + rr;
    if (row >= L) break;
    const bf16x4 v = *(const bf16x4*)(x + row * ld + c);
#pragma unroll
    for (int r = 0; r < 4; ++r) s[r] += bf2f(v[r]);
  }
  *(f32x4*)(part + (int64_t)blockIdx.y * N + c) = s;
}

__global__ void colsum_reduce_kernel(const float* __restrict__ part, int P, int N,
                                     float* __restrict__ out, int accumulate) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= N) return;
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += part[(int64_t)p * N + c];
  out[c] = accumulate ? out[c] + s : s;
}

// 16 column lanes (4 columns each) x 16 row lanes per workgroup: a [P][N] partial-sum matrix is
// reduced with every workgroup streaming 64 columns of all P rows (16-B loads, 4 in flight per
// lane), then the 16 row-lane sums are added in a fixed order (deterministic).
__global__ __launch_bounds__(NT) void colsum_reduce4_kernel(const float* __restrict__ part, int P,
                                                            int N, float* __restrict__ out,
                                                            int accumulate) {
  __shared__ f32x4 red[16][16];
  const int cx = threadIdx.x & 15, ry = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + cx * 4;
  f32x4 s0 = {0, 0, 0, 0}, s1 = s0, s2 = s0, s3 = s0;
  if (c < N) {
    int p = ry;
    for (; p + 48 < P; p += 64) {
      s0 += *(const f32x4*)(part + (int64_t)p * N + c);
      s1 += *(const f32x4*)(part + (int64_t)(p + 16) * N + c);
      s2 += *(const f32x4*)(part + (int64_t)(p + 32) * N + c);
      s3 += *(const f32x4*)(part + (int64_t)(p + 48) * N + c);
    }
    for (; p < P; p += 16) s0 += *(const f32x4*)(part + (int64_t)p * N + c);
  }
  red[ry][cx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ry == 0 && c < N) {
    f32x4 t = red[0][cx];
#pragma unroll
    for (int r = 1; r < 16; ++r) t += red[r][cx];
    if (accumulate) t += *(const f32x4*)(out + c);
    *(f32x4*)(out + c) = t;
  }
}

__global__ void sumsq_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ out) {
  __shared__ float red[NT / 64];
  float s = 0.f;
  for (int64_t i = ((int64_t)blockIdx.x * NT + threadIdx.x) * 4; i < n;
       i += (int64_t)gridDim.x * NT * 4) {
    if (i + 4 <= n) {
      const f32x4 v = *(const f32x4*)(x + i);
      s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
    } else {
      for (int64_t j = i; j < n; ++j) s += x[j] * x[j];
    }
  }
  s = block_sum<NT>(s, red);
  if (threadIdx.x == 0) atomicAdd(out, s);
}

__global__ void scale_kernel(float* __restrict__ x, int64_t n, const float* __restrict__ sc) {
  const float f = sc[0];
  for (int64_t i = ((int64_t)blockIdx.x * NT + threadIdx.x) * 4; i < n;
       i += (int64_t)gridDim.x * NT * 4) {
    if (i + 4 <= n) {
      f32x4 v = *(f32x4*)(x + i);
      *(f32x4*)(x + i) = v * f;
    } else {
      for (int64_t j = i; j < n; ++j) x[j] *= f;
    }
  }
}

// torch/optim/adamw.py _single_tensor_adamw semantics (fp32):
//   p *= 1 - lr*wd ; m += (1-b1)(g-m) ; v = b2 v + (1-b2) g^2
//   p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
// ZG: the gradient is zeroed once read (optimizer.step() + zero_grad() in one pass, keeping the
// gradient buffers allocated for the next accumulation)
template <bool ZG>
__global__ void adamw_kernel(float* __restrict__ p, float* __restrict__ g,
                             float* __restrict__ m, float* __restrict__ v, int64_t n, float lr,
                             float b1, float b2, float eps, float wd, float step_size,
                             float bc2_sqrt) {
  for (int64_t i = ((int64_t)blockIdx.x * NT + threadIdx.x) * 4; i < n;
       i += (int64_t)gridDim.x * NT * 4) {
    const int cnt = (i + 4 <= n) ? 4 : (int)(n - i);
    f32x4 pv, gv, mv, vv;
    if (cnt == 4) {
      pv = *(f32x4*)(p + i); gv = *(const f32x4*)(g + i);
      mv = *(f32x4*)(m + i); vv = *(f32x4*)(v + i);
    } else {
      for (int j = 0; j < 4; ++j) {
        pv[j] = j < cnt ? p[i + j] : 0.f; gv[j] = j < cnt ? g[i + j] : 0.f;
        mv[j] = j < cnt ? m[i + j] : 0.f; vv[j] = j < cnt ? v[i + j] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float pp = pv[j] * (1.f - lr * wd);
      float mm = mv[j] + (1.f - b1) * (gv[j] - mv[j]);
      float vq = vv[j] * b2 + (1.f - b2) * gv[j] * gv[j];
      float den = sqrtf(vq) / bc2_sqrt + eps;
      pp = pp - step_size * (mm / den);
      pv[j] = pp; mv[j] = mm; vv[j] = vq;
    }
    if (cnt == 4) {
      *(f32x4*)(p + i) = pv; *(f32x4*)(m + i) = mv; *(f32x4*)(v + i) = vv;
      if (ZG) *(f32x4*)(g + i) = (f32x4){0.f, 0.f, 0.f, 0.f};
    } else {
      for (int j = 0; j < cnt; ++j) {
        p[i + j] = pv[j]; m[i + j] = mv[j]; v[i + j] = vv[j];
        if (ZG) g[i + j] = 0.f;
      }
    }
  }
}

constexpr int PROWS = 64;
int grid_for(int64_t n) {
  int64_t b = (n / 4 + NT - 1) / NT;
  return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}
}  // namespace

extern "C" int prfl_colsum_rows_per_part(void) { return PROWS; }

extern "C" int prfl_cast_f32_bf16(const float* src, void* dst, int64_t n, void* stream) {
  if (n <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(cast_kernel, dim3((n / 8 + NT) / NT), dim3(NT), 0, s, src, (bf16*)dst, n);
  PRFL_LAUNCH_CHECK();
  return 0;
}

extern "C" int prfl_cast_f32_bf16_t(const float* w, int64_t N, int64_t K, int64_t ldw, void* out,
                                    int64_t ldo, void* stream) {
  if (N <= 0 || K <= 0) return 0;
  if (ldw < K || ldo < N || ldw % 4 || ldo % 8 || ((uintptr_t)w & 15) || ((uintptr_t)out & 15) ||
      N > 0x7fffffff || K > 0x7fffffff || (K + 63) / 64 > 0x7fffffff || (N + 63) / 64 > 65535)
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(cast_t_kernel, dim3((unsigned)((K + 63) / 64), (unsigned)((N + 63) / 64)),
                     dim3(NT), 0, s, w, ldw, (bf16*)out, ldo, (int)N, (int)K);
  PRFL_LAUNCH_CHECK();
  return 0;
}

extern "C" int prfl_gate_bwd(const float* dx, int64_t lddx, const void* y, int64_t ldy,
                             const float* gate, int64_t L, int64_t N, void* dy, int64_t lddy,
                             float* pgate, float* pbias, void* stream) {
  if (L <= 0) return 0;
  if (N % 4) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((N / 4 + NT - 1) / NT, (L + PROWS - 1) / PROWS);
  prfl_prof::begin(KID_ELTWISE, s);
  hipLaunchKernelGGL(gate_bwd_kernel<PROWS>, grid, dim3(NT), 0, s, dx, lddx, (const bf16*)y, ldy,
                     gate, (int)L, (int)N, (bf16*)dy, lddy, pgate, pbias);
  prfl_prof::set_work((double)L * N * (4 + (y ? 2 : 0) + 2));
  prfl_prof::end(KID_ELTWISE, s);
  PRFL_LAUNCH_CHECK();
  return 0;
}

extern "C" int prfl_colsum_bf16(const void* x, int64_t ld, int64_t L, int64_t N, float* part,
                                void* stream) {
  if (L <= 0) return 0;
  if (N % 4) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((N / 4 + NT - 1) / NT, (L + PROWS - 1) / PROWS);
  hipLaunchKernelGGL(colsum_bf16_kernel<PROWS>, grid, dim3(NT), 0, s, (const bf16*)x, ld, (int)L,
                     (int)N, part);
  PRFL_LAUNCH_CHECK();
  return 0;
}

extern "C" int prfl_colsum_reduce(const float* part, int64_t P, int64_t N, float* out,
                                  int accumulate, void* stream) {
  if (N <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (N % 4 == 0 && ((uintptr_t)part & 15) == 0 && ((uintptr_t)out & 15) == 0)
    hipLaunchKernelGGL(colsum_reduce4_kernel, dim3((N + 63) / 64), dim3(NT), 0, s, part, (int)P,
                       (int)N, out, accumulate);
  else
    hipLaunchKernelGGL(colsum_reduce_kernel, dim3((N + NT - 1) / NT), dim3(NT), 0, s, part,
                       (int)P, (int)N, out, accumulate);
  PRFL_LAUNCH_CHECK();
  return 0;
}

extern "C" int prfl_sumsq(const float* x, int64_t n, float* out, void* stream) {
  if (n <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sumsq_kernel, dim3(grid_for(n)), dim3(NT), 0, s, x, n, out);
  PRFL_LAUNCH_CHECK();
  return 0;
}

extern "C" int prfl_scale(float* x, int64_t n, const float* factor, void* stream) {
  if (n <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n)), dim3(NT), 0, s, x, n, factor);
  PRFL_LAUNCH_CHECK();
  return 0;
}

namespace {
int adamw_launch(float* p, float* g, float* m, float* v, int64_t n, float lr, float beta1,
                 float beta2, float eps, float weight_decay, int64_t step, bool zero_grad,
                 void* stream) {
  if (n <= 0) return 0;
  if (step < 1) return (int)hipErrorInvalidValue;
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  hipStream_t s = (hipStream_t)stream;
  prfl_prof::begin(KID_ADAMW, s);
  if (zero_grad)
    hipLaunchKernelGGL(adamw_kernel<true>, dim3(grid_for(n)), dim3(NT), 0, s, p, g, m, v, n, lr,
                       beta1, beta2, eps, weight_decay, (float)(lr / bc1), (float)sqrt(bc2));
  else
    hipLaunchKernelGGL(adamw_kernel<false>, dim3(grid_for(n)), dim3(NT), 0, s, p, g, m, v, n, lr,
                       beta1, beta2, eps, weight_decay, (float)(lr / bc1), (float)sqrt(bc2));
  prfl_prof::set_work((double)n * (zero_grad ? 32.0 : 28.0));
  prfl_prof::end(KID_ADAMW, s);
  PRFL_LAUNCH_CHECK();
  return 0;
}
}  // namespace

extern "C" int prfl_adamw(float* p, const float* g, float* m, float* v, int64_t n, float lr,
                          float beta1, float beta2, float eps, float weight_decay, int64_t step,
                          void* stream) {
  return adamw_launch(p, const_cast<float*>(g), m, v, n, lr, beta1, beta2, eps, weight_decay,
                      step, false, stream);
}

extern "C" int prfl_adamw_zero_grad(float* p, float* g, float* m, float* v, int64_t n, float lr,
                                    float beta1, float beta2, float eps, float weight_decay,
                                    int64_t step, void* stream) {
  return adamw_launch(p, g, m, v, n, lr, beta1, beta2, eps, weight_decay, step, true, stream);
}
