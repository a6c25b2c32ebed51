// Shared pieces of the bf16 LDS-DMA implicit-GEMM kernels (igemm_bf16.hip: the im2col tiles; halo_bf16.hip:
// the conv-s2 tiles with an LDS-resident input halo): the launch parameters, LDS-DMA helpers and the epilogue.
#pragma once
#include "common.hpp"

#ifndef STC_BNB_G  // rows per group of in-flight BN-input loads in the fused BN-backward epilogue (tuning builds)
#define STC_BNB_G 4
#endif

namespace stc {

struct GParams {
  const char* a;
  unsigned a_bytes;
  int a_bs, a_rs, a_ps, a_co;  // elements (a_bytes < 2^31, so 32-bit offsets suffice)
  int IH, IW, cin, lg_tw, in_stride;
  int offy[4], offx[4];
  int stepy, stepx;
  int GH, GW, M, N, K;
  float inv_ghw, inv_gw;  // 1/(GH*GW), 1/GW for fast_div (M < 2^24 is checked on the host)
  int ksplit, kchunk;
  const char* b;
  unsigned b_bytes;
  int b_phase_stride;
  char* c;
  long long c_bs, c_rs;
  int c_ps, c_co, c_cs;
  int os;
  int oy0[4], ox0[4];
  const float* bias;
  int tanh_, vec_out, out_f32;
  float* ws;
  float* stats;
  int nphase, mtiles, ntiles;
  // Fused BatchNorm-backward reduction (optional, NHWC bf16 output only): with this conv's output
  // v (the gradient reaching a BN's output through an activation) and the BN input x at the same
  // pixel, BN channel ch = n - bch_off:  nn = x*scale + shift,
  //   dn = v * act'(nn, bs_self) + g_other * act'(nn, bs_other),  xhat = (x - mean) * rstd,
  // part2[tile][ch] += {dn, dn * xhat} over the pixels inside the BN input extent.
  float* part2;
  const char* bx;
  long long bx_bs, bx_rs;
  int bx_ps, bx_co, bxH, bxW;
  const char* bg;
  long long bg_bs, bg_rs;
  int bg_ps, bg_co;
  const float *bsc, *bsh, *bmu, *brs;
  float bs_self, bs_other;
  int bC, bch_off;
  // bnb_act = 1 (stc_conv_bwd_act, layers with no BatchNorm): the BNB epilogue stores dn itself -- this conv's output
  // v (gradient reaching an activation) through the activation, nn = x (the activation's input), plus the second
  // gradient -- in place of v; no table, no sums (part2 unused).
  int bnb_act;
  int phase_major;  // grid linear over (tile, phase), phase fastest (set by the launcher)
  // Activation epilogue (layers with no BatchNorm: the first conv of G / D, STCGAN/networks.py:99,165-166):
  // act_n = 1 or 2 activated copies of the bf16-rounded output, out1 = act(v, act_s1) into c (instead of the
  // raw value), out2 = act(v, act_s2) into the c2 view -- what conv + stc_bn_apply(table = NULL) write, bit
  // for bit, without the raw tensor and its re-read.
  int act_n;
  float act_s1, act_s2;
  char* c2;
  long long c2_bs, c2_rs;
  int c2_ps, c2_co;
  // Padded GEMM grid (halo Conv2d k4 s1: the 31 x 31 output computed on its 32 x 32 input grid): vmask = 1 keeps
  // only the grid points y < vh, x < vw -- the others are neither stored nor counted in the statistics.
  int vmask, vh, vw;
  // In-launch split-K (igemm_bf16_body): each split stores its tile's fp32 accumulators to slab
  // [tile][ksplit][BM * BN] (write-through), takes the tile's ticket, and the last arriver sums the slabs in split
  // order and runs the epilogue -- no reduction launch.  tickets: one counter per tile, zero between launches.
  float* slab;
  unsigned* tickets;
  int acquire;  // the hand-off also takes the agent acquire (cdna_hip_programming.md Guideline 16)
};

// 8 bf16 (one uint4) -> act(v, slope) per element, rounded back to bf16 (as stc_bn_apply with no table)
__device__ __forceinline__ uint4 act_bf16x8(uint4 v, float slope) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
  unsigned o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    o[q] = pack_bf16x2(act(__uint_as_float(w[q] << 16), slope), act(__uint_as_float(w[q] & 0xffff0000u), slope));
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// {dn, dn*xhat} of 8 consecutive BN channels at one pixel (v: this conv's 8 output values)
__device__ __forceinline__ void bnb_accum(const GParams& p, int b, int oy, int ox, int ch, const float* v, float* sa,
                                          float* sb) {
  const bf16* xp = reinterpret_cast<const bf16*>(p.bx) + (long long)b * p.bx_bs + (long long)oy * p.bx_rs +
                   (long long)ox * p.bx_ps + p.bx_co + ch;
  const uint4 xr = *reinterpret_cast<const uint4*>(xp);
  float xv[8], gv[8];
  {
    const unsigned w[4] = {xr.x, xr.y, xr.z, xr.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) { xv[2 * q] = __uint_as_float(w[q] << 16); xv[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u); }
  }
  if (p.bg) {
    const bf16* gp = reinterpret_cast<const bf16*>(p.bg) + (long long)b * p.bg_bs + (long long)oy * p.bg_rs +
                     (long long)ox * p.bg_ps + p.bg_co + ch;
    const uint4 gr = *reinterpret_cast<const uint4*>(gp);
    const unsigned w[4] = {gr.x, gr.y, gr.z, gr.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) { gv[2 * q] = __uint_as_float(w[q] << 16); gv[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u); }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float nn = fmaf(xv[e], p.bsc[ch + e], p.bsh[ch + e]);
    float dn = v[e] * (nn > 0.f ? 1.f : p.bs_self);
    if (p.bg) dn += gv[e] * (nn > 0.f ? 1.f : p.bs_other);
    sa[e] += dn;
    sb[e] += dn * (xv[e] - p.bmu[ch + e]) * p.brs[ch + e];
  }
}

// 8 channels of the activation backward with no BatchNorm (stc_conv_bwd_act): dn = g * act'(x, s_other) +
// v * act'(x, s_self), summed in stc_bn_bwd_apply's order (second gradient first), rounded to bf16 -- the values
// conv + stc_bn_bwd_apply(no table) write, bit for bit
__device__ __forceinline__ uint4 act_bwd_bf16x8(uint4 v, uint4 x, uint4 g, bool has_g, float s_self, float s_other) {
  const unsigned wv[4] = {v.x, v.y, v.z, v.w}, wx[4] = {x.x, x.y, x.z, x.w}, wg[4] = {g.x, g.y, g.z, g.w};
  unsigned o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float d[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float vv = __uint_as_float(h ? (wv[q] & 0xffff0000u) : (wv[q] << 16));
      const float xx = __uint_as_float(h ? (wx[q] & 0xffff0000u) : (wx[q] << 16));
      float dn = 0.f;
      if (has_g) dn += __uint_as_float(h ? (wg[q] & 0xffff0000u) : (wg[q] << 16)) * dact(xx, s_other);
      dn += vv * dact(xx, s_self);
      d[h] = dn;
    }
    o[q] = pack_bf16x2(d[0], d[1]);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

// One in-launch hand-off to the last arriver of a counter (cdna_hip_programming.md Guideline 16, the write-through
// form): the payload is stored sc1 (write-through to memory, no release fence) and EVERY load of it is an sc1 load
// (past every L1 and L2, so no acquire); each wave drains its stores, the barrier joins them, lane 0 adds.
// Returns (to every thread) whether this block drew the last ticket.  The last arriver leaves the counter zero.
__device__ __forceinline__ bool last_arriver(unsigned* counter, unsigned total, unsigned* flag, bool acquire) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = old == total - 1 ? 1u : 0u;
    if (old == total - 1) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const bool last = *flag != 0u;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the sc1 loads below the ticket)
  if (last && acquire) {  // (more than one block per CU: the measured sc1 form covers one; the agent acquire too)
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
  return last;
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int SC1 = 16;  // buffer-op cache bits: sc1 (write-through stores, loads past the caches)
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, unsigned off, floatx4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, SC1);
}
__device__ __forceinline__ floatx4 ld_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, SC1));
}

// In-launch split-K combine of one tile (GParams::slab / tickets): this split's accumulators to its slab, the
// tile's ticket; the last arriver replaces acc by slab 0 + slab 1 + ... (split order -- the order of
// splitk_reduce_stats_kernel, so the sums are the same) and returns true, the others false.
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ bool splitk_combine(const GParams& p, floatx4 (&acc)[BM / WM / 16][BN / WN / 16], int tile,
                                               int split, char* smem) {
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.slab + (long long)tile * p.ksplit * (BM * BN)), (short)0, p.ksplit * BM * BN * 4, 0x00020000);
  auto off = [&](int s, int i, int j) { return (unsigned)((s * (BM * BN) + ((wave * FM + i) * FN + j) * 256 + lane * 4) * 4); };
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) st_sc1(rsl, off(split, i, j), acc[i][j]);
  if (!last_arriver(p.tickets + tile, (unsigned)p.ksplit, reinterpret_cast<unsigned*>(smem), p.acquire != 0))
    return false;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // every slab loaded (the own one too), groups of RG slabs in flight, summed in split order
  constexpr int RG = FM * FN <= 2 ? 8 : (FM * FN <= 4 ? 4 : 2);  // (<= 64 VGPRs in flight)
  const int S = p.ksplit;
  for (int s0 = 0; s0 < S; s0 += RG) {
    floatx4 v[RG][FM][FN];
#pragma unroll
    for (int g = 0; g < RG; ++g) {
      const int s = min(s0 + g, S - 1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) v[g][i][j] = ld_sc1(rsl, off(s, i, j));
    }
#pragma unroll
    for (int g = 0; g < RG; ++g) {
      if (s0 + g >= S) break;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] += v[g][i][j];
    }
  }
  return true;
}
using lds_vptr = __attribute__((address_space(3))) void*;

constexpr unsigned OOB = 0x80000000u;

#ifndef STC_IGEMM_INTERLEAVE
#define STC_IGEMM_INTERLEAVE 0
#endif
#ifndef STC_SETPRIO
#define STC_SETPRIO 0
#endif

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds_dst, unsigned voff) {
#if !STC_EXP_NODMA  // diagnostic builds only (common.hpp)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_vptr)lds_dst, 16, voff, 0, 0, 0);
#endif
}

// LDS swizzle of a K-row image: BK = 64 -> 128-B rows, chunk ^ (row & 7); BK = 32 -> 64-B rows,
// chunk ^ ((row >> 1) & 3).  Both make every ds_read_b128 lane group of the 16x16x32 operand
// read conflict-free for any 16-row-aligned fragment.
template <int BK>
__device__ __forceinline__ int kswz(int row) {
  if constexpr (BK == 64) return row & 7;
  else return (row >> 1) & 3;
}

// s_waitcnt that leaves the DMA pieces of the `ahead` youngest K-steps (P per step per wave) in
// flight: vmcnt takes an immediate, so one arm per ring depth (ahead <= NST - 2 <= 6).
template <int P>
__device__ __forceinline__ void wait_ahead(int ahead) {
  switch (ahead) {
    case 6: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(6 * P) : "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(5 * P) : "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(4 * P) : "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(3 * P) : "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * P) : "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(P) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); break;
  }
}

// In-range taps t in [0, nt) of one axis, input coordinate a + step * t (step = +-1) inside [0, I):
// an interval [lo, hi) in t, returned as a bit mask.
__device__ __forceinline__ unsigned tap_mask(int a, int I, int step, int nt) {
  const int a2 = step > 0 ? a : I - 1 - a;  // the step = -1 case mirrored onto step = +1
  const int lo = min(max(-a2, 0), nt), hi = min(max(I - a2, 0), nt);
  return ((1u << hi) - 1u) & ~((1u << lo) - 1u);
}
// Row mask (bit ty) -> bit ty << lg, the first tap of row ty in a 2-D tap set (the column mask is
// multiplied in: no carries, it has lg-bit width).
__device__ __forceinline__ unsigned tap_spread(unsigned r, int lg) {
  return (r & 1u) | (((r >> 1) & 1u) << (1 << lg)) | (((r >> 2) & 1u) << (2 << lg)) | (((r >> 3) & 1u) << (3 << lg));
}


// GEMM epilogue of one BM x BN tile (the compute waves' accumulators; LDS reused): split-K fp32 slab, or
// + bias -> (BatchNorm statistics) -> bf16 through LDS -> 16-byte NHWC row stores (+ activation copies, or the
// fused BatchNorm-backward sums); strided / fp32 outputs element-wise.  Rows m0.. are consecutive GEMM rows.
template <int BM, int BN, int WM, int WN, bool BNB>
__device__ __forceinline__ void igemm_epilogue(const GParams& p, floatx4 (&acc)[BM / WM / 16][BN / WN / 16], int m0,
                                               int n0, int ph, int mt, int z, char* smem) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int GHW = p.GH * p.GW;
  // accumulator element (i, j, r): row wm*TM + 16i + 4*(lane>>4) + r, column wn*TN + 16j + (lane&15)
  const int rq = 4 * (lane >> 4), cl = lane & 15;
  if (p.ws) {  // split-K / raw fp32 slab [z][M][N]
    float* slab = p.ws + (long long)z * p.M * p.N;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * TN + 16 * j + cl;
        if (n >= p.N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * TM + 16 * i + rq + r;
          if (m < p.M) slab[(long long)m * p.N + n] = acc[i][j][r];
        }
      }
    return;
  }

  if (p.bias) {  // (tanh epilogues only occur on narrow-N layers: narrow_bf16.hip)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * TN + 16 * j + cl;
      const float bz = n < p.N ? p.bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] += bz;
    }
  }

  __syncthreads();  // every wave is done with the stage buffers
  // BatchNorm batch statistics of the tile, one shifted pass per wave over its accumulators (shift = the column's
  // value in the wave's first row: S1 = sum(x - shift), S2 = sum((x - shift)^2)), then the WM row-waves merged
  // through LDS (at redp) into the tile's {count, 0, M2, mean} (Chan).  With 16-byte stores it runs after they are
  // issued (its LDS area past the staged tile), so the arithmetic and its barriers overlap the stores' drain.
  auto tile_stats = [&](char* redp) {
    int rows_w = min(TM, max(0, p.M - (m0 + wm * TM)));
    float* red = reinterpret_cast<float*>(redp);  // [WM][BN][4] {S1, S2, shift, rows}
    float sh[FN], s1[FN], s2[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      sh[j] = __shfl(acc[0][j][0], cl, 64);  // (the wave's first row: a kept grid point under vmask too)
      s1[j] = 0.f;
      s2[j] = 0.f;
    }
    if (p.vmask) {  // padded grid: only the kept points (the wave's rows are inside the grid: M is whole tiles)
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * TM + 16 * i + rq + r;
          const int b = fast_div(m, GHW, p.inv_ghw), rem = m - b * GHW;
          const int y = fast_div(rem, p.GW, p.inv_gw), x = rem - y * p.GW;
          const bool keep = y < p.vh && x < p.vw;
          cnt += keep ? 1 : 0;
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const float d = keep ? acc[i][j][r] - sh[j] : 0.f;
            s1[j] += d;
            s2[j] = fmaf(d, d, s2[j]);
          }
        }
      cnt += __shfl_xor(cnt, 16, 64);
      cnt += __shfl_xor(cnt, 32, 64);
      rows_w = cnt;
    } else if (rows_w == TM) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = acc[i][j][r] - sh[j];
            s1[j] += d;
            s2[j] = fmaf(d, d, s2[j]);
          }
    } else {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = 16 * i + rq + r < rows_w ? acc[i][j][r] - sh[j] : 0.f;
            s1[j] += d;
            s2[j] = fmaf(d, d, s2[j]);
          }
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      s1[j] += __shfl_xor(s1[j], 16, 64);
      s1[j] += __shfl_xor(s1[j], 32, 64);
      s2[j] += __shfl_xor(s2[j], 16, 64);
      s2[j] += __shfl_xor(s2[j], 32, 64);
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        float* q = red + (wm * BN + wn * TN + 16 * j + lane) * 4;
        q[0] = s1[j]; q[1] = s2[j]; q[2] = sh[j]; q[3] = (float)rows_w;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (LDS only: the stores stay in flight)
    __builtin_amdgcn_s_barrier();
    const long long tile = (long long)ph * p.mtiles + mt;
    for (int c = tid; c < BN; c += 64 * NW) {
      const int n = n0 + c;
      if (n >= p.N) continue;
      float cnt = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        const float* q = red + (w * BN + c) * 4;
        const float nw = q[3];
        if (nw <= 0.f) continue;
        const float mw = q[2] + q[0] / nw, m2w = fmaxf(q[1] - q[0] * (q[0] / nw), 0.f);
        const float nt = cnt + nw, dl = mw - mean;
        mean += dl * (nw / nt);
        m2 += m2w + dl * dl * (cnt * nw / nt);
        cnt = nt;
      }
      *reinterpret_cast<float4*>(p.stats + (tile * p.N + n) * 4) = make_float4(cnt, 0.f, m2, mean);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (LDS only: the stores stay in flight)
    __builtin_amdgcn_s_barrier();
  };
  if (p.stats && !p.vec_out) tile_stats(smem);
  if (p.vec_out) {
    // bf16 tile through LDS: [BM][BN] with a 16-byte row pad, then 16-byte row stores
    constexpr int PITCH = BN * 2 + 16;
    char* tl = smem;
    constexpr int CPR = BN / 8;  // 16-byte chunks per row (64*NW is a multiple of CPR: fixed cc per thread)
    constexpr int ITER = BM * CPR / (64 * NW);
    static_assert(ITER * 64 * NW == BM * CPR, "whole store iterations");
    const int cc = tid % CPR;
    const int n = n0 + cc * 8;
    // fused BatchNorm backward: the BN-input / second-gradient rows of a group of G output rows (addresses
    // independent of the GEMM result); the first group is issued before the tile staging below, so its
    // memory latency overlaps the accumulator shuffle and the barrier
    constexpr int G = ITER < STC_BNB_G ? ITER : STC_BNB_G;
    static_assert(ITER % G == 0, "whole groups");
    const int nch = n - p.bch_off;  // BN channel of this thread's chunk
    const bool bnb_on = nch >= 0 && nch < p.bC;
    const int nchc = bnb_on ? nch : 0;
    auto bnb_loads = [&](int it0, uint4* xr, uint4* gr, bool* ok) {
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int row = (tid + (it0 + u) * 64 * NW) / CPR;
        const int m = m0 + row;
        const bool in = m < p.M && n < p.N;
        const int mm = in ? m : m0;
        const int b = fast_div(mm, GHW, p.inv_ghw), rem = mm - b * GHW;
        const int y = fast_div(rem, p.GW, p.inv_gw), x = rem - y * p.GW;
        const int oy = y * p.os + p.oy0[ph], ox = x * p.os + p.ox0[ph];
        ok[u] = in && bnb_on && oy < p.bxH && ox < p.bxW && (!p.vmask || (y < p.vh && x < p.vw));
        const int oyc = ok[u] ? oy : 0, oxc = ok[u] ? ox : 0;
        xr[u] = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(p.bx) + (long long)b * p.bx_bs +
                                                (long long)oyc * p.bx_rs + (long long)oxc * p.bx_ps + p.bx_co + nchc);
        gr[u] = p.bg ? *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(p.bg) + (long long)b * p.bg_bs +
                                                       (long long)oyc * p.bg_rs + (long long)oxc * p.bg_ps + p.bg_co + nchc)
                     : make_uint4(0u, 0u, 0u, 0u);
      }
    };
    uint4 pxr[G], pgr[G];
    bool pok[G];
    if constexpr (BNB) bnb_loads(0, pxr, pgr, pok);
    // Column pairs: lanes l and l^1 hold columns c and c^1 of the same 4 rows; one DPP lane swap of two
    // values gives the even lane rows 0-1 and the odd lane rows 2-3 of the pair, each written as one
    // bf16x2 dword (half the LDS stores of per-element 16-bit writes)
    const unsigned em = (cl & 1) == 0 ? 0xffffffffu : 0u;  // even lane: all ones
    const int pcol = cl & ~1;
    // em ? u : v as one v_bfi_b32 (a ternary on the lane parity became a dynamically indexed
    // accumulator read -- a chain of compares and selects)
    auto sel = [em](float u, float v) { return __uint_as_float((em & __float_as_uint(u)) | (~em & __float_as_uint(v))); };
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const float a0 = acc[i][j][0], a1 = acc[i][j][1], a2 = acc[i][j][2], a3 = acc[i][j][3];
        // quad_perm [1,0,3,2]: every lane receives its neighbour's value
        const float x0 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(sel(a2, a0)), 0xB1, 0xF, 0xF, false));
        const float x1 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(sel(a3, a1)), 0xB1, 0xF, 0xF, false));
        const int row = wm * TM + 16 * i + rq + (em ? 0 : 2), col = wn * TN + 16 * j + pcol;
        char* dst = tl + row * PITCH + col * 2;
        *reinterpret_cast<unsigned*>(dst) = pack_bf16x2(sel(a0, x0), sel(x0, a2));
        *reinterpret_cast<unsigned*>(dst + PITCH) = pack_bf16x2(sel(a1, x1), sel(x1, a3));
      }
    __syncthreads();
    if constexpr (!BNB) {
      // rows r0 + RS*it of this thread: the pixel (b, y, x) is advanced incrementally (element
      // offsets < 2^31: vec_out is only set when the whole output view fits)
      constexpr int RS = 64 * NW / CPR;
      const int r0 = tid / CPR;
      int m = m0 + r0;
      int b = fast_div(m, GHW, p.inv_ghw), rem = m - b * GHW;
      int y = fast_div(rem, p.GW, p.inv_gw), x = rem - y * p.GW;
      const unsigned cbase = (unsigned)(p.c_co + n);
#pragma unroll 4
      for (int it = 0; it < ITER; ++it) {
        if (m >= p.M || n >= p.N) break;
        const int oy = y * p.os + p.oy0[ph], ox = x * p.os + p.ox0[ph];
        const unsigned off = (unsigned)b * (unsigned)p.c_bs + (unsigned)oy * (unsigned)p.c_rs + (unsigned)ox * (unsigned)p.c_ps +
                             cbase;
        const uint4 tv = *reinterpret_cast<const uint4*>(tl + (r0 + it * RS) * PITCH + cc * 16);
        if (p.vmask && (y >= p.vh || x >= p.vw)) {
          // (a padding point of the grid: not stored)
        } else if (p.act_n == 0) {
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.c) + off) = tv;
        } else {
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.c) + off) = act_bf16x8(tv, p.act_s1);
          if (p.act_n == 2) {
            const unsigned off2 = (unsigned)b * (unsigned)p.c2_bs + (unsigned)oy * (unsigned)p.c2_rs +
                                  (unsigned)ox * (unsigned)p.c2_ps + (unsigned)(p.c2_co + n);
            *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.c2) + off2) = act_bf16x8(tv, p.act_s2);
          }
        }
        m += RS;
        x += RS;
        while (x >= p.GW) {
          x -= p.GW;
          if (++y == p.GH) { y = 0; ++b; }
        }
      }
      if (p.stats) tile_stats(smem + BM * PITCH);
      return;
    }
    // fused BatchNorm-backward reduction: {sum dn, sum dn*xhat} of this thread's 8-channel chunk
    float sa[8], sb[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { sa[e] = 0.f; sb[e] = 0.f; }
    // groups of G rows: the BN-input / second-gradient loads of a group are in flight together
    // (one latency per group instead of one per row), then the reduction arithmetic
#pragma unroll
    for (int it0 = 0; it0 < ITER; it0 += G) {
      uint4 tv[G], xr[G], gr[G];
      bool ok[G];
      if (it0 == 0) {
#pragma unroll
        for (int u = 0; u < G; ++u) { xr[u] = pxr[u]; gr[u] = pgr[u]; ok[u] = pok[u]; }
      } else {
        bnb_loads(it0, xr, gr, ok);
      }
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int row = (tid + (it0 + u) * 64 * NW) / CPR;
        const int m = m0 + row;
        tv[u] = *reinterpret_cast<const uint4*>(tl + row * PITCH + cc * 16);
        if (m < p.M && n < p.N) {
          const int b = fast_div(m, GHW, p.inv_ghw), rem = m - b * GHW;
          const int y = fast_div(rem, p.GW, p.inv_gw), x = rem - y * p.GW;
          if (p.vmask && (y >= p.vh || x >= p.vw)) continue;
          const int oy = y * p.os + p.oy0[ph], ox = x * p.os + p.ox0[ph];
          const long long off = (long long)b * p.c_bs + (long long)oy * p.c_rs + (long long)ox * p.c_ps + p.c_co + n;
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.c) + off) =
              p.bnb_act && ok[u] ? act_bwd_bf16x8(tv[u], xr[u], gr[u], p.bg != nullptr, p.bs_self, p.bs_other) : tv[u];
        }
      }
      if (p.bnb_act) continue;  // (no BatchNorm: no sums)
#pragma unroll
      for (int u = 0; u < G; ++u) {
        if (!ok[u]) continue;
        const unsigned wt[4] = {tv[u].x, tv[u].y, tv[u].z, tv[u].w};
        const unsigned wx[4] = {xr[u].x, xr[u].y, xr[u].z, xr[u].w};
        const unsigned wg[4] = {gr[u].x, gr[u].y, gr[u].z, gr[u].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = __uint_as_float((e & 1) ? (wt[e >> 1] & 0xffff0000u) : (wt[e >> 1] << 16));
          const float xv = __uint_as_float((e & 1) ? (wx[e >> 1] & 0xffff0000u) : (wx[e >> 1] << 16));
          const float gv = __uint_as_float((e & 1) ? (wg[e >> 1] & 0xffff0000u) : (wg[e >> 1] << 16));
          const float nn = fmaf(xv, p.bsc[nch + e], p.bsh[nch + e]);
          const float dn = v * (nn > 0.f ? 1.f : p.bs_self) + gv * (nn > 0.f ? 1.f : p.bs_other);
          sa[e] += dn;
          sb[e] += dn * (xv - p.bmu[nch + e]) * p.brs[nch + e];
        }
      }
    }
    if (p.bnb_act) return;
    // per-tile reduction over the threads sharing a channel chunk (fixed order)
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [threads][16]
#pragma unroll
    for (int e = 0; e < 8; ++e) { red[tid * 16 + e] = sa[e]; red[tid * 16 + 8 + e] = sb[e]; }
    __syncthreads();
    if (tid < CPR) {
      const int ch0 = n0 + tid * 8 - p.bch_off;
      if (ch0 >= 0 && ch0 < p.bC) {
        float ta[8], tb[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) { ta[e] = 0.f; tb[e] = 0.f; }
        for (int t = tid; t < 64 * NW; t += CPR)
#pragma unroll
          for (int e = 0; e < 8; ++e) { ta[e] += red[t * 16 + e]; tb[e] += red[t * 16 + 8 + e]; }
        const long long tile = (long long)ph * p.mtiles + mt;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          *reinterpret_cast<float2*>(p.part2 + (tile * p.bC + ch0 + e) * 2) = make_float2(ta[e], tb[e]);
      }
    }
    return;
  }
  // general (strided / fp32) output: element stores
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * TM + 16 * i + rq + r;
      if (m >= p.M) continue;
      const int b = fast_div(m, GHW, p.inv_ghw), rem = m - b * GHW;
      const int y = fast_div(rem, p.GW, p.inv_gw), x = rem - y * p.GW;
      const int oy = y * p.os + p.oy0[ph], ox = x * p.os + p.ox0[ph];
      const long long ro = (long long)b * p.c_bs + (long long)oy * p.c_rs + (long long)ox * p.c_ps;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * TN + 16 * j + cl;
        if (n >= p.N) continue;
        const long long off = ro + (long long)(p.c_co + n) * p.c_cs;
        if (p.out_f32) reinterpret_cast<float*>(p.c)[off] = acc[i][j][r];
        else st1<bf16>(reinterpret_cast<bf16*>(p.c) + off, acc[i][j][r]);
      }
    }
}

}  // namespace stc
