// Shared device helpers for the MI355X (gfx950, CDNA4) PRFL kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }
// round an fp32 value to the nearest bf16 and back (an autocast cast point)
__device__ __forceinline__ float bfr(float x) { return (float)(bf16)x; }

// a*b rounded to fp32 on its own (the asm barrier stops contraction into an FMA with a later
// add), matching two separate torch ops such as `x + y * gate`.
__device__ __forceinline__ float mul_rn(float a, float b) {
  float p = a * b;
  asm volatile("" : "+v"(p));
  return p;
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// ds_read_b64_tr_b16: within each 16-lane group, lane 4q+p supplies the address of row q,
// columns 4p..4p+3 of a 4x16 block of 16-bit elements; lane i receives column i of the 4 rows.
__device__ __forceinline__ bf16x4 lds_read_tr(const void* lds_byte_addr) {
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(lds_byte_addr));
  return __builtin_bit_cast(bf16x4, v);
}

// LDS-DMA of one 16-B chunk per lane (global_load_lds_dwordx4) issued from inline asm, so the
// compiler's waitcnt bookkeeping does not see an LDS write it cannot disambiguate (hipcc would
// otherwise put vmcnt(0) before every ds_read_b64_tr_b16 and drain the prefetch).  The caller
// owns completion: counted `s_waitcnt vmcnt(N)` + barrier before any ds_read of the bytes.
// lds_dst is the wave-uniform LDS byte address of the 1-KiB piece (lane i lands at +16 i).
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
      : "memory");
}

// 4-B-per-lane variant (global_load_lds_dword): lane i lands at lds_dst + 4 i.
__device__ __forceinline__ void dma4(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
      : "memory");
}

// LDS-DMA through a buffer resource: global address = SRD base + voffset (per lane) + soffset
// (wave-uniform), so a loop that walks K moves only the SGPR soffset and keeps per-lane
// offsets that are computed once (no per-load 64-bit address arithmetic on the VALU).
typedef __attribute__((ext_vector_type(4))) int i32x4;
// raw buffer over [base, base + bytes): stride 0, dword3 = the gfx9 default data format
__device__ __forceinline__ i32x4 make_srd(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  return (i32x4){(int)__builtin_amdgcn_readfirstlane((uint32_t)a),
                 (int)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xffffu),
                 (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000};
}
__device__ __forceinline__ void dma16_buf(i32x4 srd, uint32_t voff, uint32_t soff, uint32_t lds_dst) {
  unsigned keep;     // m0 is reserved to the compiler: save / restore it around the DMA
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(srd), "s"(__builtin_amdgcn_readfirstlane(lds_dst)),
        "s"(__builtin_amdgcn_readfirstlane(soff))
      : "memory");
}

// Grouped form: m0 set once (saved) for several pieces at consecutive KiB of LDS, each piece then
// `buffer_load_dwordx4 ... offen offset:PIECE*1024 lds` (the instruction offset adds to both the
// LDS and the global address: the caller pre-subtracts it from voff), m0 restored after the group.
__device__ __forceinline__ void m0_set(uint32_t lds_base, unsigned& keep) {
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0"
               : "=&s"(keep) : "s"(__builtin_amdgcn_readfirstlane(lds_base)) : "memory");
}
__device__ __forceinline__ void m0_restore(unsigned keep) {
  asm volatile("s_mov_b32 m0, %0" :: "s"(keep) : "memory");
}
template <int PIECE>
__device__ __forceinline__ void dma16_buf_m0_(i32x4 srd, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2 offen offset:%3 lds"
               :: "v"(voff), "s"(srd), "s"(__builtin_amdgcn_readfirstlane(soff)), "i"(PIECE * 1024)
               : "memory");
}
__device__ __forceinline__ void dma16_buf_m0(i32x4 srd, uint32_t voff, uint32_t soff, int piece) {
  switch (piece) {
    case 0: dma16_buf_m0_<0>(srd, voff, soff); break;
    case 1: dma16_buf_m0_<1>(srd, voff, soff); break;
    case 2: dma16_buf_m0_<2>(srd, voff, soff); break;
    default: dma16_buf_m0_<3>(srd, voff, soff); break;
  }
}

// 4-B-per-lane buffer variant (buffer_load_dword ... lds): lane i lands at lds_dst + 4 i; a lane
// whose offset is past the SRD's num_records lands 0.
__device__ __forceinline__ void dma4_buf(i32x4 srd, uint32_t voff, uint32_t lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(srd), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
      : "memory");
}

// A wave-uniform pointer laundered through readfirstlane (SGPRs): `uniform_ptr(base + t * stride)
// + lane_offset` then cannot be re-associated into a per-lane 64-bit `base + lane_offset` that
// LICM hoists out of the tile loop (one VGPR pair per DMA stream -> spills at 256 VGPRs).
template <typename T>
__device__ __forceinline__ const T* uniform_ptr(const T* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const T*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ bf16x8 cat8(bf16x4 a, bf16x4 b) {
  return (bf16x8){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
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

// block-wide sum for blockDim.x == NT (multiple of 64); red must hold NT/64 floats
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += red[i];
  return s;
}

// GELU(tanh) (ATen GeluKernel.cpp, approximate='tanh': 0.5 x (1 + tanh(u)), u = sqrt(2/pi)
// (x + 0.044715 x^3)) in its sigmoid form 0.5 (1 + tanh(u)) = s = 1 / (1 + exp(-2u)): one v_exp
// and one v_rcp instead of the library tanhf (a branchy ~30-instruction sequence that cost the
// GEMM epilogue ~13 % of an FFN-up launch).  The two forms agree to a few fp32 ulp of the result
// (the sigmoid form has no 1 + tanh cancellation for u << 0); outputs are bf16.
__device__ __forceinline__ float gelu_sig(float x, float& x2) {
  const float kBeta = 0.7978845608028654f;   // sqrt(2/pi)
  const float kKappa = 0.044715f;
  x2 = x * x;
  const float u = kBeta * fmaf(kKappa * x2, x, x);
  const float e = __builtin_amdgcn_exp2f(-2.8853900817779268f * u);   // exp(-2u)
  return __builtin_amdgcn_rcpf(1.f + e);                                // exp overflow: s = 0
}
__device__ __forceinline__ float gelu_tanh(float x) {
  float x2;
  return x * gelu_sig(x, x2);
}
// d/dx: 0.5 (1 + t) + 0.5 x (1 - t^2) u'  with  1 + t = 2 s,  1 - t^2 = 4 s (1 - s)
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float kBeta = 0.7978845608028654f;
  const float kKappa = 0.044715f;
  float x2;
  const float s = gelu_sig(x, x2);
  const float du = kBeta * fmaf(3.f * kKappa, x2, 1.f);
  return fmaf(2.f * x * s * (1.f - s), du, s);
}

#define PRFL_LAUNCH_CHECK()                          \
  do {                                               \
    hipError_t _e = hipGetLastError();               \
    if (_e != hipSuccess) return (int)_e;            \
  } while (0)

// per-kernel timing hooks (bench.py roofline); defined in prof.hip
namespace prfl_prof {
void begin(int kid, hipStream_t s);
void end(int kid, hipStream_t s);
void set_work(double w);  // algorithmic FLOPs/bytes of the launch being timed
unsigned long long* clk_slot();  // (cycles, 100 MHz ticks) slot for the next launch, or null
}
enum {
  KID_GEMM = 0, KID_ATTN_FWD, KID_ATTN_FWD_SHORT, KID_ATTN_BWD_DKDV, KID_ATTN_BWD_DQ, KID_LN, KID_RMS,
  KID_ELTWISE, KID_ADAMW, KID_POOL, KID_ATTN_FWD_FP8,
  KID_COUNT
};
