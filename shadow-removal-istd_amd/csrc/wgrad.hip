// Weight gradient of the 4x4 conv / convT family as an implicit GEMM over pixels.
//
//   dW[r][ci][kh][kw] = sum_{b,oy,ox} D[b,oy,ox,r] * G[b, oy*s+kh-1, ox*s+kw-1, ci]
//   Conv2d s2/s1 : D = dy (output grid), G = x       (SURVEY.md a4/a5 backward)
//   ConvT  s2    : D = x  (input grid),  G = dy, s=2 (SURVEY.md a6 backward)
//
// GEMM view: C[R][16*Cg] = sum_p D[p][R]^T * Gcol[p][16*Cg]; both operands are
// pixel-major in HBM (channels contiguous), so each is staged into LDS as
// [pixel][channel] rows with 16-byte loads and 16-byte LDS stores, no transpose.
//   fp32: v_mfma_f32_32x32x2_f32 takes one k per lane half (lane l: A[i=l&31][k=l>>5]),
//         i.e. a plain ds_read_b32 across consecutive channels (conflict-free).
//   bf16: v_mfma_f32_32x32x16_bf16 needs 8 consecutive k (pixels) per lane: two
//         ds_read_b64_tr_b16 (hardware 4x16 transpose per 16-lane group) build each
//         operand from the [pixel][channel] image.  Rows are 320 B (256 B of data +
//         64 B pad): 320/4 = 80 = 16 mod 64 banks, so the four rows of a transposed
//         read land in disjoint 16-bank ranges (conflict-free per 32-lane half).
// The global loads of K-step s+1 are issued before step s's MFMAs and only consumed
// (prologue: BN affine + LeakyReLU/ReLU of the producer) when written to LDS.
// The pixel dimension is split over blockIdx.z into fp32 slabs that a second kernel
// sums in a fixed order (bitwise reproducible) while writing torch layout.
#include "common.hpp"

namespace stc {

struct WgradParams {
  const char* d;
  long long d_bs, d_rs;
  int d_ps, d_co;
  const char* g;
  long long g_bs, g_rs;
  int g_ps, g_co;
  int GH, GW;  // D grid (the reduction domain) -> P = B*GH*GW
  int IH, IW;  // G logical bounds
  int stride;
  int R, Cg, Ncol;  // Ncol = 16*Cg
  int P, pchunk, nsplit;
  const float *dsc, *dsh, *gsc, *gsh;
  int dact, gact;
  float dslope, gslope;
  float* ws;  // [nsplit][R][Ncol]
  float* dW;  // direct output when nsplit == 1 (torch layout), else nullptr
  int Cg_out;
  int mtiles, ntiles;
};

constexpr int WG_BM = 128, WG_BN = 128, WG_BK = 32;

template <typename T> struct WgCfg;
template <> struct WgCfg<float> {
  static constexpr int ROWB = (WG_BM + 4) * 4;  // 528 B: 16-byte aligned rows
};
template <> struct WgCfg<bf16> {
  static constexpr int ROWB = 320;  // 256 B data + 64 B pad (see header)
};

template <typename T>
__device__ __forceinline__ uint4 wg_pro(uint4 v, const float* sc, const float* sh, int act_on, float slope) {
  // sc/sh already offset to the chunk's first channel
  constexpr int VEC = 16 / sizeof(T);
  float f[VEC];
  if constexpr (sizeof(T) == 4) {
    f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y); f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
  } else {
    const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) { f[2 * q] = __uint_as_float(w[q] << 16); f[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u); }
  }
  if (sc) {
#pragma unroll
    for (int e = 0; e < VEC; ++e) f[e] = fmaf(f[e], sc[e], sh[e]);
  }
  if (act_on) {
#pragma unroll
    for (int e = 0; e < VEC; ++e) f[e] = f[e] > 0.f ? f[e] : f[e] * slope;
  }
  uint4 r;
  if constexpr (sizeof(T) == 4) {
    r.x = __float_as_uint(f[0]); r.y = __float_as_uint(f[1]); r.z = __float_as_uint(f[2]); r.w = __float_as_uint(f[3]);
  } else {
    unsigned w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = (unsigned)f2bf(f[2 * q]) | ((unsigned)f2bf(f[2 * q + 1]) << 16);
    r.x = w[0]; r.y = w[1]; r.z = w[2]; r.w = w[3];
  }
  return r;
}

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short v8i16 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ v4i16 lds_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(p));
}

template <typename T>
__global__ void __launch_bounds__(256)
wgrad_kernel(const WgradParams p) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int CPR = WG_BM * (int)sizeof(T) / 16;  // 16-byte chunks per staged row (32 fp32 / 16 bf16)
  constexpr int RPP = 256 / CPR;                     // rows per pass
  constexpr int NP = WG_BK / RPP;                    // passes per K-step (4 fp32 / 2 bf16)
  constexpr int ROWB = WgCfg<T>::ROWB;
  constexpr int TILEB = WG_BK * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILEB];  // [stage][A|B]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = p.mtiles * p.ntiles;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int mt = bid / p.ntiles, nt = bid % p.ntiles;
  const int r0 = mt * WG_BM, c0 = nt * WG_BN;
  const int split = blockIdx.z;
  const int pbeg = split * p.pchunk;
  const int pend = min(p.P, pbeg + p.pchunk);
  const int GHW = p.GH * p.GW;

  // staging map: row (pixel) kp = tid/CPR + RPP*i, chunk = tid%CPR (VEC channels)
  const int chunk = tid % CPR;
  const int rr = r0 + chunk * VEC;   // D channel of this chunk
  const int col = c0 + chunk * VEC;  // G column of this chunk
  const bool rval = rr < p.R;
  const bool cval = col < p.Ncol;
  const int t = col / p.Cg, ci = col - t * p.Cg;
  const int kh = t >> 2, kw = t & 3;
  const T* Dp = reinterpret_cast<const T*>(p.d);
  const T* Gp = reinterpret_cast<const T*>(p.g);
  const float* dsc = p.dsc ? p.dsc + rr : nullptr;
  const float* dsh = p.dsh ? p.dsh + rr : nullptr;
  const float* gsc = p.gsc ? p.gsc + ci : nullptr;
  const float* gsh = p.gsh ? p.gsh + ci : nullptr;
  const bool dpro = p.dsc != nullptr || p.dact;
  const bool gpro = p.gsc != nullptr || p.gact;

  uint4 va[NP], vb[NP];
  unsigned ma = 0, mb = 0;
  auto load = [&](int k0) {
    ma = 0; mb = 0;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int pix = k0 + tid / CPR + RPP * i;
      va[i] = make_uint4(0, 0, 0, 0);
      vb[i] = make_uint4(0, 0, 0, 0);
      if (pix < pend) {
        const int b = pix / GHW, rem = pix - b * GHW;
        const int oy = rem / p.GW, ox = rem - oy * p.GW;
        if (rval) {
          va[i] = *reinterpret_cast<const uint4*>(Dp + (long long)b * p.d_bs + (long long)oy * p.d_rs +
                                                  (long long)ox * p.d_ps + p.d_co + rr);
          ma |= 1u << i;
        }
        const int iy = oy * p.stride + kh - 1, ix = ox * p.stride + kw - 1;
        if (cval && (unsigned)iy < (unsigned)p.IH && (unsigned)ix < (unsigned)p.IW) {
          vb[i] = *reinterpret_cast<const uint4*>(Gp + (long long)b * p.g_bs + (long long)iy * p.g_rs +
                                                  (long long)ix * p.g_ps + p.g_co + ci);
          mb |= 1u << i;
        }
      }
    }
  };
  auto store = [&](int st) {
    char* sA = smem + st * 2 * TILEB;
    char* sB = sA + TILEB;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int kp = tid / CPR + RPP * i;
      uint4 a = va[i], b = vb[i];
      if (dpro && (ma >> i & 1u)) a = wg_pro<T>(a, dsc, dsh, p.dact, p.dslope);
      if (gpro && (mb >> i & 1u)) b = wg_pro<T>(b, gsc, gsh, p.gact, p.gslope);
      *reinterpret_cast<uint4*>(sA + kp * ROWB + chunk * 16) = a;
      *reinterpret_cast<uint4*>(sB + kp * ROWB + chunk * 16) = b;
    }
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nsteps = (pend - pbeg + WG_BK - 1) / WG_BK;
  if (nsteps > 0) {
    load(pbeg);
    store(0);
  }
  __syncthreads();
  const int li = lane & 31, lh = lane >> 5;
  // transposed-read addressing (bf16): 16-lane group g16, lane-in-group 4*trq + trp
  const int g16 = lane >> 4, lig = lane & 15;
  const int trq = lig >> 2, trp = lig & 3;
  const int trh = g16 >> 1, trc = 16 * (g16 & 1) + 4 * trp;
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    if (s + 1 < nsteps) load(pbeg + (s + 1) * WG_BK);
    const char* sA = smem + cur * 2 * TILEB;
    const char* sB = sA + TILEB;
    if constexpr (sizeof(T) == 4) {
#pragma unroll 4
      for (int kk = 0; kk < WG_BK / 2; ++kk) {
        const int k = 2 * kk + lh;
        const float* ra = reinterpret_cast<const float*>(sA + k * ROWB);
        const float* rb = reinterpret_cast<const float*>(sB + k * ROWB);
        const float a0 = ra[wm * 64 + li], a1 = ra[wm * 64 + 32 + li];
        const float b0 = rb[wn * 64 + li], b1 = rb[wn * 64 + 32 + li];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < WG_BK / 16; ++ks) {
        bf16x8 fa[2], fb[2];
        const int row = ks * 16 + 8 * trh + trq;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const char* pa = sA + row * ROWB + (wm * 64 + 32 * i + trc) * 2;
          const char* pb = sB + row * ROWB + (wn * 64 + 32 * i + trc) * 2;
          const v4i16 a_lo = lds_tr16(pa), a_hi = lds_tr16(pa + 4 * ROWB);
          const v4i16 b_lo = lds_tr16(pb), b_hi = lds_tr16(pb + 4 * ROWB);
          const v8i16 av = {a_lo[0], a_lo[1], a_lo[2], a_lo[3], a_hi[0], a_hi[1], a_hi[2], a_hi[3]};
          const v8i16 bv = {b_lo[0], b_lo[1], b_lo[2], b_lo[3], b_hi[0], b_hi[1], b_hi[2], b_hi[3]};
          fa[i] = __builtin_bit_cast(bf16x8, av);
          fb[i] = __builtin_bit_cast(bf16x8, bv);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
    if (s + 1 < nsteps) store(cur ^ 1);
    __syncthreads();
  }

  if (p.dW) {  // single pixel split: write torch layout dW[r][ci][kh][kw] directly
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = c0 + wn * 64 + 32 * j + li;
      const int tt = n / p.Cg, cc = n - tt * p.Cg;
      if (n >= p.Ncol || cc >= p.Cg_out) continue;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = r0 + wm * 64 + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * lh;
          if (m < p.R) p.dW[((long long)m * p.Cg_out + cc) * 16 + tt] = acc[i][j][e];
        }
    }
    return;
  }
  float* slab = p.ws + (long long)split * p.R * p.Ncol;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = c0 + wn * 64 + 32 * j + li;
      if (n >= p.Ncol) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = r0 + wm * 64 + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * lh;
        if (m < p.R) slab[(long long)m * p.Ncol + n] = acc[i][j][e];
      }
    }
}

// dW[r][ci][kh][kw] = sum_s ws[s][r][(kh*4+kw)*Cg + ci]: one thread per (r, tap, ci) with ci fastest
// (coalesced slab reads), the splits summed in a fixed order with 4 independent partial sums.
// Fixed-order sum of the split slabs (row-major [split][R][16*Cg], GEMM column n = tap*Cg + ci) into
// torch layout dW[R][Cg_out][16].  One thread = (r, ci, 4 consecutive taps): it reads each slab at
// columns tap*Cg + ci (consecutive threads -> consecutive ci, coalesced) and writes the 4 taps as one
// float4, so a warp's stores are one contiguous run of dW (the transposition costs no scattered stores).
__global__ void __launch_bounds__(128) wgrad_reduce_kernel(const float* __restrict__ ws, int nsplit, int R, int Cg,
                                                           int Cg_out, float* __restrict__ dW) {
  const long long total = (long long)R * Cg_out * 4;
  const long long Ncol = 16LL * Cg;
  const long long slab = (long long)R * Ncol;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int g = (int)(idx & 3);
    const long long rc = idx >> 2;
    const int ci = (int)(rc % Cg_out);
    const int r = (int)(rc / Cg_out);
    const float* src = ws + (long long)r * Ncol + (long long)(4 * g) * Cg + ci;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int sp = 0;
    for (; sp + 2 <= nsplit; sp += 2) {  // two slabs' loads in flight; the sum order stays split order
      const float* a = src + (long long)sp * slab;
      const float* b = a + slab;
      const float a0 = a[0], a1 = a[Cg], a2 = a[2 * Cg], a3 = a[3 * Cg];
      const float b0 = b[0], b1 = b[Cg], b2 = b[2 * Cg], b3 = b[3 * Cg];
      acc.x += a0; acc.y += a1; acc.z += a2; acc.w += a3;
      acc.x += b0; acc.y += b1; acc.z += b2; acc.w += b3;
    }
    for (; sp < nsplit; ++sp) {
      const float* a = src + (long long)sp * slab;
      acc.x += a[0]; acc.y += a[Cg]; acc.z += a[2 * Cg]; acc.w += a[3 * Cg];
    }
    *reinterpret_cast<float4*>(dW + ((long long)r * Cg_out + ci) * 16 + 4 * g) = acc;
  }
}

int64_t wgrad_reduce_blocks(int R, int Cg_out) {
  const long long total = (long long)R * Cg_out * 4;
  return std::min<long long>((total + 127) / 128, 16384);
}

// The same sum for small outputs over many slabs (the 3-8 channel first/last layers: P = B*256*256
// pixels split up to 256 ways, R*Cg_out*4 < 8192 output units): one wave per (r, ci, 4 taps) unit,
// lane l summing slabs l, l + 64, ... in order, then a fixed xor-butterfly across the lanes
// (deterministic; a thread per unit walking 256 slabs serially was latency-bound at 40-70 us).
__global__ void __launch_bounds__(256) wgrad_reduce_wide_kernel(const float* __restrict__ ws, int nsplit, int R, int Cg,
                                                                int Cg_out, float* __restrict__ dW) {
  const int lane = threadIdx.x & 63;
  const long long unit = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long long total = (long long)R * Cg_out * 4;
  if (unit >= total) return;
  const int g = (int)(unit & 3);
  const long long rc = unit >> 2;
  const int ci = (int)(rc % Cg_out);
  const int r = (int)(rc / Cg_out);
  const long long Ncol = 16LL * Cg;
  const long long slab = (long long)R * Ncol;
  const float* src = ws + (long long)r * Ncol + (long long)(4 * g) * Cg + ci;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int sp = lane; sp < nsplit; sp += 64) {
    const float* a = src + (long long)sp * slab;
    acc.x += a[0]; acc.y += a[Cg]; acc.z += a[2 * Cg]; acc.w += a[3 * Cg];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    acc.x += __shfl_xor(acc.x, o, 64); acc.y += __shfl_xor(acc.y, o, 64);
    acc.z += __shfl_xor(acc.z, o, 64); acc.w += __shfl_xor(acc.w, o, 64);
  }
  if (lane == 0) *reinterpret_cast<float4*>(dW + ((long long)r * Cg_out + ci) * 16 + 4 * g) = acc;
}

// The same fixed-order sum with more bytes in flight (the kernel above keeps 8 four-byte loads per
// thread outstanding and was latency-bound at ~17 us for 64 slabs of 512 KB): a block = one row r x
// 64 channels x 16 taps, a thread = (tap, 4 channels) reading one 16-byte vector per slab, 8 slabs
// loaded before they are added (in split order, so the result is bit-identical), then the tile is
// transposed through LDS into dW[r][ci][tap] and stored as contiguous 16-byte rows.
// Needs Cg % 4 == 0 and Cg_out >= 64.
__global__ void __launch_bounds__(256) wgrad_reduce_v4_kernel(const float* __restrict__ ws, int nsplit, int R, int Cg,
                                                              int Cg_out, float* __restrict__ dW) {
  __shared__ float tile[64 * 17];
  const int tid = threadIdx.x;
  const int r = blockIdx.x / ((Cg_out + 63) >> 6);
  const int c0 = (blockIdx.x - r * ((Cg_out + 63) >> 6)) * 64;
  const int tap = tid >> 4, c4 = tid & 15;
  const int ci = c0 + 4 * c4;
  const long long Ncol = 16LL * Cg;
  const long long slab = (long long)R * Ncol;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ci < Cg) {
    const float* src = ws + (long long)r * Ncol + (long long)tap * Cg + ci;
    int sp = 0;
    for (; sp + 8 <= nsplit; sp += 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(src + (long long)(sp + u) * slab);
#pragma unroll
      for (int u = 0; u < 8; ++u) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
    }
    for (; sp < nsplit; ++sp) {
      const float4 v = *reinterpret_cast<const float4*>(src + (long long)sp * slab);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  tile[(4 * c4 + 0) * 17 + tap] = acc.x;
  tile[(4 * c4 + 1) * 17 + tap] = acc.y;
  tile[(4 * c4 + 2) * 17 + tap] = acc.z;
  tile[(4 * c4 + 3) * 17 + tap] = acc.w;
  __syncthreads();
  const int cl = tid >> 2, t4 = (tid & 3) * 4;
  if (c0 + cl < Cg_out) {
    const float* q = tile + cl * 17 + t4;
    *reinterpret_cast<float4*>(dW + ((long long)r * Cg_out + c0 + cl) * 16 + t4) = make_float4(q[0], q[1], q[2], q[3]);
  }
}

// The same sum for small outputs over many slabs (the first layers' 256 splits of a 64|128 x 128 dW, the logits
// layer's 64 image parts): a block = one row r x 64 slab columns, thread = (float4 column cq, slab lane sl < 16): lane
// sl sums slabs sl, sl + 16, ... in order with 8 loads in flight, then the 16 lanes' partials are added in lane order
// through LDS; the wave-per-unit kernel above kept only 4 scalar loads per lane in flight (11-20 us for 256 slabs; this
// one 5-6 us, a 512-thread variant with 32 slab lanes no faster).
__global__ void __launch_bounds__(256) wgrad_reduce_many_kernel(const float* __restrict__ ws, int nsplit, int R, int Cg,
                                                                int Cg_out, float* __restrict__ dW) {
  __shared__ float4 part[16][16];
  const int tid = threadIdx.x, cq = tid & 15, sl = tid >> 4;
  const long long Ncol = 16LL * Cg;
  const int nchk = (int)((Ncol + 63) / 64);
  const int r = blockIdx.x / nchk;
  const long long c = (long long)(blockIdx.x - r * nchk) * 64 + 4 * cq;
  const long long slab = (long long)R * Ncol;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < Ncol) {  // (Ncol = 16 Cg is a multiple of 4: a float4 never straddles the end)
    const float* src = ws + (long long)r * Ncol + c;
    int sp = sl;
    for (; sp + 16 * 7 < nsplit; sp += 16 * 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(src + (long long)(sp + 16 * u) * slab);
#pragma unroll
      for (int u = 0; u < 8; ++u) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
    }
    for (; sp < nsplit; sp += 16) {
      const float4 v = *reinterpret_cast<const float4*>(src + (long long)sp * slab);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  part[sl][cq] = acc;
  __syncthreads();
  if (tid < 64) {  // column c0 + tid: the 16 lanes' partials in lane order
    const int q = tid >> 2, e = tid & 3;
    float t = 0.f;
#pragma unroll
    for (int l = 0; l < 16; ++l) {
      const float4 v = part[l][q];
      t += e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
    }
    const long long col = (long long)(blockIdx.x - r * nchk) * 64 + tid;
    if (col < Ncol) {
      const int tap = (int)(col / Cg), ci = (int)(col - (long long)tap * Cg);
      if (ci < Cg_out) dW[((long long)r * Cg_out + ci) * 16 + tap] = t;
    }
  }
}

void wgrad_reduce_launch(const float* ws, int nsplit, int R, int Cg, int Cg_out, float* dW, hipStream_t st) {
  const long long units = (long long)R * Cg_out * 4;
  if (Cg % 4 == 0 && Cg_out >= 64 && !(units < 8192 && nsplit >= 16))
    hipLaunchKernelGGL(wgrad_reduce_v4_kernel, dim3((unsigned)(R * ((Cg_out + 63) / 64))), dim3(256), 0, st, ws, nsplit,
                       R, Cg, Cg_out, dW);
  else if (units < 8192 && nsplit >= 16 && Cg % 4 == 0)
    hipLaunchKernelGGL(wgrad_reduce_many_kernel, dim3((unsigned)(R * ((16LL * Cg + 63) / 64))), dim3(256), 0, st, ws,
                       nsplit, R, Cg, Cg_out, dW);
  else if (units < 8192 && nsplit >= 16)
    hipLaunchKernelGGL(wgrad_reduce_wide_kernel, dim3((unsigned)((units + 3) / 4)), dim3(256), 0, st, ws, nsplit, R, Cg,
                       Cg_out, dW);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)wgrad_reduce_blocks(R, Cg_out)), dim3(128), 0, st, ws,
                       nsplit, R, Cg, Cg_out, dW);
}

struct WgPlan {
  int mtiles, ntiles, nsplit, pchunk;
};
static WgPlan wg_plan(int P, int R, int Cg) {
  WgPlan pl{};
  pl.mtiles = cdiv(R, WG_BM);
  pl.ntiles = cdiv(16LL * Cg, WG_BN);
  const long long tiles = (long long)pl.mtiles * pl.ntiles;
  int ns = 1;
  const int steps = cdiv(P, WG_BK);
  while (tiles * ns < 768 && ns * 2 <= 256 && steps / (ns * 2) >= 8) ns *= 2;
  pl.pchunk = cdiv(steps, ns) * WG_BK;
  pl.nsplit = cdiv(P, pl.pchunk);
  return pl;
}

}  // namespace stc

namespace stc {
bool wgrad_bf16_eligible(int B, const stc_view& D, int R, const stc_view& G, int Cg);
int64_t wgrad_bf16_workspace(int B, int Hd, int Wd, int R, int Cg, const int32_t* force);
void wgrad_bf16_plan(int B, int Hd, int Wd, int R, int Cg, const int32_t* force, int32_t* plan_out);
int wgrad_bf16(int B, int stride, stc_view D, int R, stc_view G, int Cg, int Cg_out, float* dW, void* workspace,
               int64_t workspace_bytes, hipStream_t st, const int32_t* force);
}  // namespace stc

namespace stc {

// ---- narrow-R weight gradient of a stride-1 4x4 conv (the PatchGAN logits layer, 512 -> 1 channel:
// STCGAN/networks.py:183-184).  With RO <= 2 real rows the GEMM form is all im2col traffic (16 taps
// of the 512-channel input, padded R); here each input pixel q is read ONCE and scattered into its 16
// taps: dW[r][ci][kh][kw] += G[q][ci] * D[qy-kh+1][qx-kw+1][r].
// Block = (image, 64-channel chunk, pixel split ps of 4), 256 threads = 16 channel quads x 16 pixel
// lanes: lane l takes the image's pixels 16 ps + l + 64 k; the image's D plane (RO channels, zero-padded by 2) sits in LDS and is
// read as broadcasts.  The 16 lanes' partials are summed in a fixed order (through LDS) into the
// slab [image][RO][16 * Cg] (column tap * Cg + ci), which the ordered wide reduce sums over images.
// One non-packed v_fma_f32.  The compiler otherwise pairs these accumulations into v_pk_fma_f32 with
// op_sel; in that form the kernel returned sporadically different low-half sums (one (tap, even
// channel) accumulator of a whole wave) when two processes shared the GPU (tests/test_gpu_dist.py).
// STC_ROWS_PACKED: diagnostic build only (scripts/rows_stress.py) -- the compiler's packed form.
__device__ __forceinline__ float fma_scalar(float a, float b, float c) {
#ifdef STC_ROWS_PACKED
  return __builtin_fmaf(a, b, c);
#else
  asm("v_fma_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
  return c;
#endif
}

template <typename T, int RO>
__global__ void __launch_bounds__(256) wgrad_rows_kernel(const char* __restrict__ dp, long long d_bs, long long d_rs,
                                                         int d_ps, int d_co, int OH, int OW, const char* __restrict__ gp,
                                                         long long g_bs, long long g_rs, int g_ps, int g_co, int IH,
                                                         int IW, int Cg, float* __restrict__ ws) {
  extern __shared__ float sm[];
  constexpr int PS = 4;  // pixel splits per (image, chunk): 4 blocks, lane stride 64
  const int nchunk = Cg / 64;
  const int ps = blockIdx.x % PS, bc = blockIdx.x / PS;
  const int b = bc / nchunk, cc = bc % nchunk;
  const float inv_iw = 1.0f / (float)IW;
  const int rows = OH + 4, cols = OW + 4;  // D plane with a 2-wide zero border
  float* dl = sm;                          // [RO][rows][cols]
  const T* D = reinterpret_cast<const T*>(dp);
  for (int i = threadIdx.x; i < RO * rows * cols; i += 256) {
    const int r = i / (rows * cols), rem = i - r * rows * cols, yy = rem / cols, xx = rem - yy * cols;
    const int oy = yy - 2, ox = xx - 2;
    float v = 0.f;
    if (oy >= 0 && oy < OH && ox >= 0 && ox < OW)
      v = ld1<T>(D + (long long)b * d_bs + (long long)oy * d_rs + (long long)ox * d_ps + d_co + r);
    dl[i] = v;
  }
  __syncthreads();
  const int quad = threadIdx.x & 15, plane = threadIdx.x >> 4;
  const int c0 = cc * 64 + quad * 4;
  float acc[RO][16][4];
#pragma unroll
  for (int r = 0; r < RO; ++r)
#pragma unroll
    for (int t = 0; t < 16; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[r][t][e] = 0.f;
  const T* G = reinterpret_cast<const T*>(gp) + (long long)b * g_bs + g_co + c0;
  const int npix = IH * IW;
  auto body = [&](int q, const float4 gq) {
    const int qy = fast_div(q, IW, inv_iw), qx = q - qy * IW;
    const float gv[4] = {gq.x, gq.y, gq.z, gq.w};
    // D[qy - kh + 1][qx - kw + 1] sits at LDS (qy - kh + 3, qx - kw + 3)
#pragma unroll
    for (int r = 0; r < RO; ++r)
#pragma unroll
      for (int kh = 0; kh < 4; ++kh)
#pragma unroll
        for (int kw = 0; kw < 4; ++kw) {
          const float dv = dl[(r * rows + qy - kh + 3) * cols + qx - kw + 3];
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[r][kh * 4 + kw][e] = fma_scalar(gv[e], dv, acc[r][kh * 4 + kw][e]);
        }
  };
  int q = plane + 16 * ps;
  for (; q + 64 * 3 < npix; q += 64 * 4) {  // four pixels' loads in flight
    float4 g4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int qq = q + 64 * u, qy = fast_div(qq, IW, inv_iw), qx = qq - qy * IW;
      g4[u] = Vec4<T>::load(G + (long long)qy * g_rs + (long long)qx * g_ps);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) body(q + 64 * u, g4[u]);
  }
  for (; q < npix; q += 64) {
    const int qy = fast_div(q, IW, inv_iw), qx = q - qy * IW;
    body(q, Vec4<T>::load(G + (long long)qy * g_rs + (long long)qx * g_ps));
  }
  // fixed-order sum over the 16 pixel planes (4 per wave), all through LDS: every plane stores its
  // partials (part[plane][r][t][64 channels], after the D plane), then each output is
  // ((p0 + p1) + (p2 + p3)) per wave and (w0 + w1) + (w2 + w3) across waves (the order of an xor
  // butterfly over the planes followed by a cross-wave sum).
  float* part = sm + ((RO * rows * cols + 3) & ~3);
  constexpr int PL = RO * 16 * 64;  // floats per plane
#pragma unroll
  for (int r = 0; r < RO; ++r)
#pragma unroll
    for (int t = 0; t < 16; ++t)
      *reinterpret_cast<float4*>(part + plane * PL + (r * 16 + t) * 64 + quad * 4) =
          make_float4(acc[r][t][0], acc[r][t][1], acc[r][t][2], acc[r][t][3]);
  __syncthreads();
  float* slab = ws + ((long long)b * PS + ps) * RO * 16 * Cg;
  for (int o = threadIdx.x; o < PL; o += 256) {  // o = (r * 16 + t) * 64 + c
    float w4[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float* pw = part + 4 * w * PL + o;
      w4[w] = (pw[0] + pw[PL]) + (pw[2 * PL] + pw[3 * PL]);
    }
    slab[(long long)(o >> 6) * Cg + cc * 64 + (o & 63)] = (w4[0] + w4[1]) + (w4[2] + w4[3]);
  }
}

// ---- the same weight gradient on MFMA (bf16): C[tap][ci] = sum_q Dpad[q - tap shift][r] * G[q][ci] is a 16-row
// GEMM (M = the 16 taps of one real D row, N = channels, K = the image's pixels), so v_mfma_f32_16x16x32_bf16 takes
// it whole.  K is laid out as image rows of 32 pixel slots (the input is <= 32 wide; slots past it are zero), so a
// K-step of 32 = one input row qy and a lane's 8 K values = 8 consecutive columns of one row:
//   A (16 taps x 32 slots): lane (tap = (kh, kw), kq) = D[qy - kh + 1][8 kq - kw + 1 ..] -- one 16-byte LDS read from
//     the kw-shifted copy of the zero-bordered D plane (4 copies, [row][40] bf16, built once per block);
//   B (32 slots x 16 channels): ds_read_b64_tr_b16 of the staged input.
// Block = (image, 64-channel chunk, 16-row part): its input part ([16 rows x 32 slots][64 ch] = 64 KiB, 16-byte chunk
// c of slot p in position c ^ 2((p >> 1) & 3): the 16 lanes of a transposed read hit 16 distinct 8-byte bank
// groups) is LDS-DMA'd in one go; wave w owns channels 16w .. +15.  Partial sums go to the slab
// [image * parts + part][RO][16 * Cg] (column tap * Cg + ci) for the ordered reduce, as in wgrad_rows_kernel.
constexpr int WRM_ROWS = 16;  // input rows per block (part)
constexpr int WRM_W = 32;     // pixel slots per input row
constexpr int WRM_PITCH = 40; // D-copy row pitch (bf16): 32 columns + pad, 16-byte rows
constexpr int WRM_DPT = 8;    // D values per thread (RO x OH x OW <= 2048)

template <int RO>
__global__ void __launch_bounds__(256) wgrad_rows_mfma_kernel(const char* __restrict__ dp, long long d_bs, long long d_rs,
                                                              int d_ps, int d_co, int OH, int OW, const char* __restrict__ gp,
                                                              unsigned g_bytes, int g_bs, int g_rs, int g_ps, int g_co,
                                                              int IH, int IW, int Cg, int parts, float* __restrict__ ws,
                                                              float* __restrict__ zdst, long long nzero) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* gs = smem;                                                          // [16 x 32 slots][128 B]
  unsigned short* dc = reinterpret_cast<unsigned short*>(smem + WRM_ROWS * WRM_W * 128);  // [RO][4 kw][OH + 5][40]
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nchunk = Cg / 64;
  int bid = blockIdx.x;
  const int part = bid % parts;
  bid /= parts;
  const int cc = bid % nchunk, b = bid / nchunk;
  const int y0 = part * WRM_ROWS;
  const int crow = OH + 5, cplane = crow * WRM_PITCH, ncopy = RO * 4 * cplane;
  // 1. the D plane's loads (RO x OH x OW <= 4 x 256 values), issued before the input DMA so that waiting for them
  //    does not wait for the DMA (VMEM completes in order)
  const unsigned short* D = reinterpret_cast<const unsigned short*>(dp);
  const int npl = OH * OW;
  unsigned short dv[WRM_DPT];
#pragma unroll
  for (int u = 0; u < WRM_DPT; ++u) {
    const int i = tid + 256 * u, r = i / npl, rem = i - r * npl, oy = rem / OW, ox = rem - oy * OW;
    const bool in = i < RO * npl;
    dv[u] = D[in ? (long long)b * d_bs + (long long)oy * d_rs + (long long)ox * d_ps + d_co + r : 0];
  }
  // 2. the input part by LDS-DMA: piece k (1 KiB) = slots 8k .. 8k+7, lane -> (slot 8k + (lane >> 3), position lane & 7)
  {
    const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)gp, (short)0, (int)g_bytes, 0x00020000);
    using lds_t = __attribute__((address_space(3))) void*;
#pragma unroll
    for (int k = 0; k < WRM_ROWS * WRM_W / 8 / 4; ++k) {
      const int pc = wave + 4 * k;
      const int px = 8 * pc + (lane >> 3), pos = lane & 7;
      const int c8 = pos ^ (((px >> 1) & 3) << 1);  // the 16-byte chunk stored in this position
      const int qy = y0 + px / WRM_W, qx = px % WRM_W;
      const bool ok = qy < IH && qx < IW;
      const unsigned off = (unsigned)(b * g_bs + qy * g_rs + qx * g_ps + g_co + cc * 64 + 8 * c8) * 2u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rg, (lds_t)(gs + pc * 1024), 16, ok ? off : 0x80000000u, 0, 0, 0);
    }
  }
  // 3. the kw-shifted D copies: copy[r][kw][row][x] = D[row - 2][x - kw + 1][r] (0 outside), x < 32 -- zeroed, then
  //    each D value written to its 4 positions
  for (int i = tid; i < ncopy / 8; i += 256) *reinterpret_cast<uint4*>(dc + 8 * i) = make_uint4(0u, 0u, 0u, 0u);
  // the padded D rows' weight gradient is zero: this block's share of dW[R_out .. R)
  for (long long z = (long long)blockIdx.x * 256 + tid; z < nzero; z += (long long)gridDim.x * 256) zdst[z] = 0.f;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int u = 0; u < WRM_DPT; ++u) {
    const int i = tid + 256 * u, r = i / npl, rem = i - r * npl, oy = rem / OW, ox = rem - oy * OW;
    if (i < RO * npl) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int x = ox + k - 1;
        if (x >= 0 && x < WRM_W) dc[(r * 4 + k) * cplane + (oy + 2) * WRM_PITCH + x] = dv[u];
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  // 3. K-steps = the part's input rows
  const int tap = lane & 15, kq = lane >> 4, kh = tap >> 2, kw = tap & 3;
  const int q4 = (lane & 15) >> 2, pcol = lane & 3;
  const int nrow = STC_EXP_NOEPI ? 0 : min(WRM_ROWS, IH - y0);  // (diagnostic builds: the loads alone)
  floatx4 acc[RO];
#pragma unroll
  for (int r = 0; r < RO; ++r) acc[r] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int col = 16 * wave + 4 * pcol;
  auto boff = [&](int px) { return px * 128 + 16 * ((col >> 3) ^ (((px >> 1) & 3) << 1)) + 2 * (col & 7); };
  const unsigned short* arow = dc + kw * cplane + 8 * kq;
  for (int s = 0; s < nrow; ++s) {
    const int pr = WRM_W * s + 8 * kq + q4;
    const v4i16 lo = lds_tr16(gs + boff(pr)), hi = lds_tr16(gs + boff(pr + 4));
    const v4i16 bv[2] = {lo, hi};
    const stc_bf16x8 bf = __builtin_bit_cast(stc_bf16x8, bv);
    const int arw = (y0 + s - kh + 3) * WRM_PITCH;
#pragma unroll
    for (int r = 0; r < RO; ++r) {
      const stc_bf16x8 a = *reinterpret_cast<const stc_bf16x8*>(arow + r * 4 * cplane + arw);
      acc[r] = exp_mfma(a, bf, acc[r]);
    }
  }
  // acc[r][e] = C[tap 4 kq + e][channel cc*64 + 16 wave + (lane & 15)] -> slab column tap * Cg + ci
  float* slab = ws + ((long long)b * parts + part) * RO * 16LL * Cg;
  const int ci = cc * 64 + 16 * wave + (lane & 15);
#pragma unroll
  for (int r = 0; r < RO; ++r)
#pragma unroll
    for (int e = 0; e < 4; ++e) slab[((long long)r * 16 + 4 * kq + e) * Cg + ci] = acc[r][e];
}

}  // namespace stc

using namespace stc;

extern "C" int64_t stc_conv_wgrad_rows_workspace(int B, int IH, int R_out, int Cg) {
  (void)IH;
  return (int64_t)B * 4 * R_out * 16LL * Cg * 4;  // a slab per (image, pixel split)
}

extern "C" int stc_conv_wgrad_rows(int dtype, int B, stc_view D, int R, int R_out, stc_view G, int Cg, int Cg_out,
                                   float* dW, void* workspace, int64_t workspace_bytes, void* stream) {
  STC_REQUIRE(dtype == STC_F32 || dtype == STC_BF16, "stc_conv_wgrad_rows: bad dtype");
  STC_REQUIRE(R_out >= 1 && R_out <= 2 && R_out <= R, "stc_conv_wgrad_rows: R_out=%d (1..2, <= R)", R_out);
  STC_REQUIRE(Cg % 64 == 0 && Cg_out <= Cg && G.cs == 1 && G.co % 4 == 0 && G.ps % 4 == 0 && D.cs == 1,
              "stc_conv_wgrad_rows: Cg=%d / views (NHWC, Cg a multiple of 64, 4-channel aligned)", Cg);
  STC_REQUIRE(D.H == G.H - 1 && D.W == G.W - 1, "stc_conv_wgrad_rows: stride-1 4x4 geometry needs D = G - 1 (%dx%d vs %dx%d)",
              D.H, D.W, G.H, G.W);
  hipStream_t st = (hipStream_t)stream;
  const int64_t need = stc_conv_wgrad_rows_workspace(B, G.H, R_out, Cg);
  // bf16 on MFMA (wgrad_rows_mfma_kernel): input <= 32 x 32 (rows of 32 slots), 16-byte aligned input channels
  const int parts = (G.H + WRM_ROWS - 1) / WRM_ROWS;
  const size_t lds_m = (size_t)WRM_ROWS * WRM_W * 128 + (size_t)R_out * 4 * (D.H + 5) * WRM_PITCH * 2;
  const long long g_bytes = (long long)B * G.bs * 2;
  if (dtype == STC_BF16 && G.ps % 8 == 0 && G.co % 8 == 0 && G.W <= WRM_W && G.H <= 32 && parts <= 4 &&
      R_out * D.H * D.W <= 256 * WRM_DPT &&
      lds_m <= 96 * 1024 && g_bytes < (1ll << 31)) {
    STC_REQUIRE(workspace && workspace_bytes >= need, "stc_conv_wgrad_rows: workspace %lld < %lld",
                (long long)workspace_bytes, (long long)need);
    float* ws = (float*)workspace;
    const dim3 grid((unsigned)(B * (Cg / 64) * parts));
    main_timer_begin(st);
#define STC_WRM(RO_)                                                                                               \
  hipLaunchKernelGGL((wgrad_rows_mfma_kernel<RO_>), grid, dim3(256), lds_m, st, (const char*)D.p, D.bs, D.rs, D.ps, \
                     D.co, D.H, D.W, (const char*)G.p, (unsigned)g_bytes, (int)G.bs, (int)G.rs, G.ps, G.co, G.H, G.W,  \
                     Cg, parts, ws, dW + (size_t)R_out * Cg_out * 16, (long long)(R - R_out) * Cg_out * 16)
    if (R_out == 1) STC_WRM(1);
    else STC_WRM(2);
#undef STC_WRM
    main_timer_end(st);
    STC_CHECK_LAUNCH();
    wgrad_reduce_launch(ws, B * parts, R_out, Cg, Cg_out, dW, st);
    STC_CHECK_LAUNCH();
    return 0;
  }
  const int blocks = B * (Cg / 64) * 4;
  STC_REQUIRE(workspace && workspace_bytes >= need, "stc_conv_wgrad_rows: workspace %lld < %lld",
              (long long)workspace_bytes, (long long)need);
  const size_t lds = ((((size_t)R_out * (D.H + 4) * (D.W + 4) + 3) & ~(size_t)3) + (size_t)16 * R_out * 16 * 64) * 4;
  STC_REQUIRE(lds <= 160 * 1024, "stc_conv_wgrad_rows: D plane too large for LDS (%dx%d)", D.H, D.W);
  float* ws = (float*)workspace;
  main_timer_begin(st);
#define STC_WR(T_, RO_)                                                                                          \
  hipLaunchKernelGGL((wgrad_rows_kernel<T_, RO_>), dim3(blocks), dim3(256), lds, st, (const char*)D.p, D.bs,    \
                     D.rs, D.ps, D.co, D.H, D.W, (const char*)G.p, G.bs, G.rs, G.ps, G.co, G.H, G.W, Cg, ws)
  if (dtype == STC_BF16) { if (R_out == 1) STC_WR(bf16, 1); else STC_WR(bf16, 2); }
  else { if (R_out == 1) STC_WR(float, 1); else STC_WR(float, 2); }
#undef STC_WR
  main_timer_end(st);
  STC_CHECK_LAUNCH();
  wgrad_reduce_launch(ws, B * 4, R_out, Cg, Cg_out, dW, st);
  STC_CHECK_LAUNCH();
  if (R > R_out) {  // the zero rows of the padded D channels
    (void)hipMemsetAsync(dW + (size_t)R_out * Cg_out * 16, 0, (size_t)(R - R_out) * Cg_out * 16 * 4, st);
    STC_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int stc_conv_wgrad_query(int dtype, int B, int Hd, int Wd, int R, int Cg, const int32_t* force_plan,
                                    int64_t* workspace_bytes, int32_t* plan_out) {
  const WgPlan pl = wg_plan(B * Hd * Wd, R, Cg);
  const int64_t ws_reg = pl.nsplit <= 1 ? 0 : (int64_t)pl.nsplit * R * 16LL * Cg * 4;  // 0: straight into dW
  // bf16 without prologues runs the LDS-DMA kernel (wgrad_bf16.hip); the prologue form the register-staged one
  const int64_t ws_dma = dtype == STC_BF16 ? wgrad_bf16_workspace(B, Hd, Wd, R, Cg, force_plan) : 0;
  if (workspace_bytes) *workspace_bytes = std::max(ws_reg, ws_dma);
  if (plan_out) {
    if (dtype == STC_BF16) {
      wgrad_bf16_plan(B, Hd, Wd, R, Cg, force_plan, plan_out);
    } else {
      plan_out[0] = -1; plan_out[1] = WG_BM; plan_out[2] = WG_BN; plan_out[3] = pl.nsplit; plan_out[4] = pl.nsplit > 1;
    }
  }
  return 0;
}

extern "C" int64_t stc_conv_wgrad_workspace(int dtype, int B, int Hd, int Wd, int R, int Cg) {
  int64_t ws = 0;
  stc_conv_wgrad_query(dtype, B, Hd, Wd, R, Cg, nullptr, &ws, nullptr);
  return ws;
}

extern "C" int stc_conv_wgrad(int dtype, int B, int stride, stc_view D, int R,
                              const float* d_scale, const float* d_shift, int d_act, float d_slope,
                              stc_view G, int Cg, int Cg_out,
                              const float* g_scale, const float* g_shift, int g_act, float g_slope,
                              float* dW, void* workspace, int64_t workspace_bytes, void* stream) {
  return stc_conv_wgrad_ex(dtype, B, stride, D, R, d_scale, d_shift, d_act, d_slope, G, Cg, Cg_out, g_scale, g_shift,
                           g_act, g_slope, dW, nullptr, workspace, workspace_bytes, stream);
}

extern "C" int stc_conv_wgrad_ex(int dtype, int B, int stride, stc_view D, int R,
                                 const float* d_scale, const float* d_shift, int d_act, float d_slope,
                                 stc_view G, int Cg, int Cg_out,
                                 const float* g_scale, const float* g_shift, int g_act, float g_slope,
                                 float* dW, const int32_t* force_plan, void* workspace, int64_t workspace_bytes,
                                 void* stream) {
  STC_REQUIRE(dtype == STC_F32 || dtype == STC_BF16, "stc_conv_wgrad: bad dtype");
  const int VEC = dtype == STC_F32 ? 4 : 8;
  STC_REQUIRE(Cg >= VEC && Cg % VEC == 0, "stc_conv_wgrad: Cg=%d must be a multiple of %d", Cg, VEC);
  STC_REQUIRE(R % VEC == 0, "stc_conv_wgrad: R=%d must be a multiple of %d", R, VEC);
  STC_REQUIRE(D.cs == 1 && G.cs == 1 && D.co % VEC == 0 && G.co % VEC == 0 && D.ps % VEC == 0 && G.ps % VEC == 0,
              "stc_conv_wgrad: views must be NHWC with %d-aligned channels", VEC);
  STC_REQUIRE(Cg_out <= Cg, "stc_conv_wgrad: Cg_out > Cg");
  WgradParams p{};
  p.d = (const char*)D.p; p.d_bs = D.bs; p.d_rs = D.rs; p.d_ps = D.ps; p.d_co = D.co;
  p.g = (const char*)G.p; p.g_bs = G.bs; p.g_rs = G.rs; p.g_ps = G.ps; p.g_co = G.co;
  p.GH = D.H; p.GW = D.W; p.IH = G.H; p.IW = G.W; p.stride = stride;
  p.R = R; p.Cg = Cg; p.Ncol = 16 * Cg;
  p.P = B * D.H * D.W;
  p.dsc = d_scale; p.dsh = d_shift; p.dact = d_act; p.dslope = d_slope;
  p.gsc = g_scale; p.gsh = g_shift; p.gact = g_act; p.gslope = g_slope;
  hipStream_t st = (hipStream_t)stream;
  if (p.P == 0) {
    (void)hipMemsetAsync(dW, 0, (size_t)R * Cg_out * 16 * 4, st);
    STC_CHECK_LAUNCH();
    return 0;
  }
  if (dtype == STC_BF16 && !d_scale && !d_act && !g_scale && !g_act && wgrad_bf16_eligible(B, D, R, G, Cg))
    return wgrad_bf16(B, stride, D, R, G, Cg, Cg_out, dW, workspace, workspace_bytes, st, force_plan);
  const WgPlan pl = wg_plan(p.P, R, Cg);
  p.mtiles = pl.mtiles; p.ntiles = pl.ntiles; p.nsplit = pl.nsplit; p.pchunk = pl.pchunk;
  p.Cg_out = Cg_out;
  dim3 grid(pl.mtiles * pl.ntiles, 1, pl.nsplit);
  if (pl.nsplit <= 1) {
    p.dW = dW;
    main_timer_begin(st);
    if (dtype == STC_F32) hipLaunchKernelGGL(wgrad_kernel<float>, grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL(wgrad_kernel<bf16>, grid, dim3(256), 0, st, p);
    main_timer_end(st);
    STC_CHECK_LAUNCH();
    return 0;
  }
  const int64_t need = (int64_t)pl.nsplit * R * 16LL * Cg * 4;
  STC_REQUIRE(workspace && workspace_bytes >= need, "stc_conv_wgrad: workspace %lld < %lld",
              (long long)workspace_bytes, (long long)need);
  p.ws = (float*)workspace;
  main_timer_begin(st);
  if (dtype == STC_F32) hipLaunchKernelGGL(wgrad_kernel<float>, grid, dim3(256), 0, st, p);
  else hipLaunchKernelGGL(wgrad_kernel<bf16>, grid, dim3(256), 0, st, p);
  main_timer_end(st);
  STC_CHECK_LAUNCH();
  wgrad_reduce_launch((const float*)p.ws, pl.nsplit, R, Cg, Cg_out, dW, st);
  STC_CHECK_LAUNCH();
  return 0;
}
