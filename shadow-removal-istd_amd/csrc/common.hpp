// Shared device/host helpers for the gfx950 ST-CGAN kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <string>
#include <cstdio>
#include <cstdarg>

#include "../../include/stcgan_hip.h"

namespace stc {

using bf16 = __hip_bfloat16;
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef short shortx8 __attribute__((ext_vector_type(8)));
typedef short shortx4 __attribute__((ext_vector_type(4)));

// Diagnostic builds (scripts/diag_gemm.sh; never the shipped library): STC_EXP_NODMA drops the
// LDS-DMA operand loads, STC_EXP_NOMFMA replaces each MFMA by one VALU add that still consumes its
// fragments, STC_EXP_NOEPI ends the GEMM kernels after the K loop -- what each part of a tile costs.
#ifndef STC_EXP_NODMA
#define STC_EXP_NODMA 0
#endif
#ifndef STC_EXP_NOMFMA
#define STC_EXP_NOMFMA 0
#endif
#ifndef STC_EXP_NOEPI
#define STC_EXP_NOEPI 0
#endif
typedef __bf16 stc_bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ floatx4 exp_mfma(stc_bf16x8 a, stc_bf16x8 b, floatx4 c) {
#if STC_EXP_NOMFMA
  c[0] += (float)a[0] * (float)b[0];
  return c;
#else
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
#endif
}

// ---------------------------------------------------------------- errors
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);
// stc_time_next_main_kernel instrumentation: record around the main kernel of a call
void main_timer_begin(hipStream_t st);
void main_timer_end(hipStream_t st);

#define STC_CHECK_LAUNCH()                                                     \
  do {                                                                         \
    hipError_t e_ = hipGetLastError();                                         \
    if (e_ != hipSuccess)                                                      \
      return ::stc::fail((int)e_, "%s: launch failed: %s", __func__,          \
                         hipGetErrorString(e_));                               \
  } while (0)

#define STC_REQUIRE(cond, ...)                                                 \
  do {                                                                         \
    if (!(cond)) return ::stc::fail(-1, __VA_ARGS__);                          \
  } while (0)

// ---------------------------------------------------------------- bf16 helpers
__device__ __forceinline__ float bf2f(unsigned short u) {
  return __uint_as_float(((unsigned)u) << 16);
}
__device__ __forceinline__ unsigned short f2bf(float f) {
  // round-to-nearest-even; NaN kept NaN by the hardware convert
  bf16 b = __float2bfloat16(f);
  return *reinterpret_cast<unsigned short*>(&b);
}

// {lo, hi} -> one dword of two bf16 (round-to-nearest-even), a single v_cvt_pk_bf16_f32
typedef __bf16 stc_bf16x2 __attribute__((ext_vector_type(2)));
typedef float stc_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  const stc_f32x2 v = {lo, hi};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, stc_bf16x2));
}

// 4 consecutive elements <-> float4
template <typename T> struct Vec4;
template <> struct Vec4<float> {
  __device__ __forceinline__ static float4 load(const float* p) {
    return *reinterpret_cast<const float4*>(p);
  }
  __device__ __forceinline__ static void store(float* p, float4 v) {
    *reinterpret_cast<float4*>(p) = v;
  }
};
template <> struct Vec4<bf16> {
  __device__ __forceinline__ static float4 load(const bf16* p) {
    uint2 u = *reinterpret_cast<const uint2*>(p);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
  }
  __device__ __forceinline__ static void store(bf16* p, float4 v) {
    uint2 u;
    u.x = (unsigned)f2bf(v.x) | ((unsigned)f2bf(v.y) << 16);
    u.y = (unsigned)f2bf(v.z) | ((unsigned)f2bf(v.w) << 16);
    *reinterpret_cast<uint2*>(p) = u;
  }
};

template <typename T> __device__ __forceinline__ float ld1(const T* p);
template <> __device__ __forceinline__ float ld1<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld1<bf16>(const bf16* p) {
  return bf2f(*reinterpret_cast<const unsigned short*>(p));
}
template <typename T> __device__ __forceinline__ void st1(T* p, float v);
template <> __device__ __forceinline__ void st1<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void st1<bf16>(bf16* p, float v) {
  *reinterpret_cast<unsigned short*>(p) = f2bf(v);
}

// ---------------------------------------------------------------- views
struct View {  // device-side copy of stc_view
  char* p;
  int H, W;
  long long bs, rs;
  int ps, co, cs;
};
static inline View mkview(const stc_view& v) {
  View r;
  r.p = (char*)v.p; r.H = v.H; r.W = v.W; r.bs = v.bs; r.rs = v.rs;
  r.ps = v.ps; r.co = v.co; r.cs = v.cs;
  return r;
}
__device__ __forceinline__ long long vidx(const View& v, int b, int y, int x, int c) {
  return (long long)b * v.bs + (long long)y * v.rs + (long long)x * v.ps + (long long)(v.co + c) * v.cs;
}

__device__ __forceinline__ float act(float v, float slope) { return v > 0.f ? v : v * slope; }
__device__ __forceinline__ float dact(float n, float slope) { return n > 0.f ? 1.f : slope; }

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// q = n / d for 0 <= n < 2^24, d >= 1, with inv = 1.0f / d from the host: the float estimate is
// within one of the quotient, one integer correction makes it exact (≈6 VALU instead of the ≈35 of a
// 32-bit division by a runtime divisor)
__device__ __forceinline__ int fast_div(int n, int d, float inv) {
  int q = (int)((float)n * inv);
  const int r = n - q * d;
  return q + (r >= d) - (r < 0);
}

// Implicit-GEMM geometry of each conv kind (tap offsets are affine in the tap index).
struct Geometry {
  int taps_lg_tw;   // lg of taps per row (2 -> 4x4 taps, 1 -> 2x2 taps)
  int in_stride, os, nphase;
  int offy[4], offx[4];
  int stepy, stepx;
};

static inline Geometry geometry(int kind) {
  Geometry g{};
  switch (kind) {
    case STC_CONV_S2:
    case STC_CONV_S1:
      g.taps_lg_tw = 2; g.in_stride = kind == STC_CONV_S2 ? 2 : 1; g.os = 1; g.nphase = 1;
      g.offy[0] = -1; g.offx[0] = -1; g.stepy = 1; g.stepx = 1;
      break;
    case STC_CONV_S1_DGRAD:  // dx[i] = sum_k dy[i + 1 - k] w[k]
      g.taps_lg_tw = 2; g.in_stride = 1; g.os = 1; g.nphase = 1;
      g.offy[0] = 1; g.offx[0] = 1; g.stepy = -1; g.stepx = -1;
      break;
    case STC_CONVT_S2:  // out(2y+ph) = sum_t in(y + ph - t) w[(1-ph) + 2t]
      g.taps_lg_tw = 1; g.in_stride = 1; g.os = 2; g.nphase = 4;
      for (int z = 0; z < 4; ++z) { g.offy[z] = z >> 1; g.offx[z] = z & 1; }
      g.stepy = -1; g.stepx = -1;
      break;
  }
  return g;
}

// channel c's affine parameters and running statistics, loaded before the merge (off its latency chain)
struct BnPre {
  float g, bt, rm, rv;
};
__device__ __forceinline__ BnPre bn_pre(int c, const float* gamma, const float* beta, const float* rmean,
                                        const float* rvar) {
  return BnPre{gamma ? gamma[c] : 1.f, beta ? beta[c] : 0.f, rmean ? rmean[c] : 0.f, rvar ? rvar[c] : 0.f};
}

// mean / rstd / affine table / running statistics of channel c from the merged N, mean, M2
__device__ __forceinline__ void bn_finalize_store(int c, double N, double mu, double M2, const BnPre& q, float* rmean,
                                                  float* rvar, long long* nbt, float momentum, float eps,
                                                  float* mean_o, float* rstd_o, float* scale, float* shift) {
  const double var = N > 0 ? M2 / N : 0.0;
  const float rs = (float)(1.0 / sqrt(var + (double)eps));
  if (mean_o) mean_o[c] = (float)mu;
  if (rstd_o) rstd_o[c] = rs;
  const float sc = q.g * rs;
  scale[c] = sc;
  shift[c] = q.bt - (float)mu * sc;
  if (rmean) rmean[c] = (1.f - momentum) * q.rm + momentum * (float)mu;
  if (rvar) rvar[c] = (1.f - momentum) * q.rv + momentum * (float)(N > 1 ? M2 / (N - 1) : var);
  if (nbt && c == 0) nbt[0] += 1;
}
__device__ __forceinline__ void bn_finalize_store(int c, double N, double mu, double M2, const float* gamma,
                                                  const float* beta, float* rmean, float* rvar, long long* nbt,
                                                  float momentum, float eps, float* mean_o, float* rstd_o,
                                                  float* scale, float* shift) {
  bn_finalize_store(c, N, mu, M2, bn_pre(c, gamma, beta, rmean, rvar), rmean, rvar, nbt, momentum, eps, mean_o,
                    rstd_o, scale, shift);
}

}  // namespace stc
