// bf16 weight gradient of the 4x4 conv / convT family on MFMA, staged by LDS-DMA.
//
//   C[r][col] = sum_p D[p][r] * Gcol[p][col],   col = tap*Cg + ci,
//   Gcol[p][tap, ci] = G[b, oy*s + kh - 1, ox*s + kw - 1, ci]      (tap = kh*4 + kw)
//   Conv2d s2/s1 : D = dy (output grid), G = x (input);  ConvT s2 : D = x (input grid), G = dy.
// The reduction runs over pixels.  Both operands are pixel-major in HBM (channels contiguous),
// so each K-step (64 pixels) is DMA'd as [pixel][128 channels] 256-byte rows with the 16-byte
// chunk index XOR-swizzled by ((row&3)<<2 | (row>>2)&3) on the source side, and the MFMA
// operands (8 consecutive pixels of one channel per lane) come out of ds_read_b64_tr_b16
// (4 rows x 16 columns per 16-lane group, transposed by the LDS) -- conflict-free for the
// 16x16x32 operand with the two 4-row blocks of a 32-lane half 8 rows apart.
// Tile 128 (r) x 128 (col), 4 waves of 64x64, 2-stage ring (DMA of step s+1 under the
// MFMAs of step s).  The pixel range is split over blockIdx.z into fp32 slabs that
// wgrad_reduce_kernel sums in a fixed order; a single split writes torch layout directly.
#include "common.hpp"

namespace stc {

struct WbParams {
  const char* d;
  unsigned d_bytes;
  int d_bs, d_rs, d_ps, d_co;
  const char* g;
  unsigned g_bytes;
  int g_bs, g_rs, g_ps, g_co;
  int GH, GW, IH, IW, stride;
  int R, Cg, Ncol, Cg_out;
  int P, pchunk, nsplit;
  float inv_ghw, inv_gw;  // fast exact division by GH*GW and GW (p < 2^24)
  int mtiles, ntiles;
  float* ws;
  float* dW;
};

typedef short w4i16 __attribute__((ext_vector_type(4)));
typedef __bf16 wbf16x8 __attribute__((ext_vector_type(8)));
using wlds_ptr = __attribute__((address_space(3))) void*;

__device__ __forceinline__ void wdma16(__amdgpu_buffer_rsrc_t r, char* lds_dst, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (wlds_ptr)lds_dst, 16, voff, 0, 0, 0);
}
__device__ __forceinline__ w4i16 wtr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) w4i16*)(p));
}
// q = floor(n / d) for 0 <= n < 2^24: float estimate (exact n, |error| < 1) plus one correction
__device__ __forceinline__ int fdiv(int n, int d, float inv) {
  int q = (int)((float)n * inv);
  const int r = n - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

__device__ __forceinline__ int wswz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

constexpr int WB_BM = 128, WB_BN = 128, WB_BK = 64;
constexpr int WB_TILE = WB_BK * 256;  // bytes per operand per stage

__global__ void __launch_bounds__(256) wgrad_bf16_kernel(const WbParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = p.mtiles * p.ntiles;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int mt = bid / p.ntiles, nt = bid % p.ntiles;
  const int r0 = mt * WB_BM, c0 = nt * WB_BN;
  const int split = blockIdx.z;
  const int pbeg = split * p.pchunk;
  const int pend = min(p.P, pbeg + p.pchunk);
  const int nsteps = (pend - pbeg + WB_BK - 1) / WB_BK;
  const int GHW = p.GH * p.GW;

  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)p.d, (short)0, (int)p.d_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)p.g, (short)0, (int)p.g_bytes, 0x00020000);
  const unsigned OOBV = 0x80000000u;

  // DMA roles: a piece = 4 pixel rows x 256 B; lane -> row (lane>>4) of the piece, LDS slot lane&15.
  // Each wave issues pieces wave, wave+4, ... (4 per operand per step).
  const int prow = lane >> 4;
  // per-lane column roles (fixed over the K loop): the chunk this lane loads depends on its row's swizzle,
  // and rows 4*pc + prow have (row & 3) = prow and ((row >> 2) & 3) = pc & 3 -> per piece constant.
  int d_chunk_off[4], g_tap_dy[4], g_tap_dx[4], g_ci[4];
  unsigned d_pen[4], g_pen[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int pc = wave + 4 * i;  // piece index 0..15
    const int row = 4 * pc + prow;
    const int chunk = (lane & 15) ^ wswz(row);
    const int rr = r0 + chunk * 8;
    d_chunk_off[i] = p.d_co + rr;
    d_pen[i] = rr < p.R ? 0u : OOBV;
    const int col = c0 + chunk * 8;
    const int tap = col / p.Cg;
    g_ci[i] = p.g_co + col - tap * p.Cg;
    g_tap_dy[i] = (tap >> 2) - 1;
    g_tap_dx[i] = (tap & 3) - 1;
    g_pen[i] = col < p.Ncol ? 0u : OOBV;
  }

  auto issue = [&](int s, int stage) {
    char* sD = smem + stage * 2 * WB_TILE;
    char* sG = sD + WB_TILE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pc = wave + 4 * i;
      const int pix = pbeg + s * WB_BK + 4 * pc + prow;
      const unsigned ppen = pix < pend ? 0u : OOBV;
      const int pp = pix < pend ? pix : pbeg;
      const int b = fdiv(pp, GHW, p.inv_ghw), rem = pp - b * GHW;
      const int oy = fdiv(rem, p.GW, p.inv_gw), ox = rem - oy * p.GW;
      const unsigned doff = (((unsigned)b * (unsigned)p.d_bs + (unsigned)oy * (unsigned)p.d_rs +
                              (unsigned)ox * (unsigned)p.d_ps + (unsigned)d_chunk_off[i]) * 2u) | ppen | d_pen[i];
      wdma16(rd, sD + pc * 1024, doff);
      const int iy = oy * p.stride + g_tap_dy[i], ix = ox * p.stride + g_tap_dx[i];
      const unsigned ipen = ((unsigned)iy < (unsigned)p.IH && (unsigned)ix < (unsigned)p.IW) ? 0u : OOBV;
      const unsigned goff = (((unsigned)b * (unsigned)p.g_bs + (unsigned)iy * (unsigned)p.g_rs +
                              (unsigned)ix * (unsigned)p.g_ps + (unsigned)g_ci[i]) * 2u) | ppen | g_pen[i] | ipen;
      wdma16(rg, sG + pc * 1024, goff);
    }
  };

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // transposed-read addressing: lane 4q+p of 16-lane group g reads row (8g + q [+4]), columns 4p..4p+3
  // of the fragment's 16 columns.  Byte offset of (row, col) = 256*row + 16*((col>>3) ^ wswz(row)) + 2*(col&7).
  const int kq = lane >> 4;       // k-chunk: pixels 8*kq .. 8*kq+7 of the 32-pixel sub-step
  const int q = (lane & 15) >> 2, pcol = lane & 3;
  auto tr_off = [&](int row, int colbase) {
    const int col = colbase + 4 * pcol;
    return 256 * row + 16 * ((col >> 3) ^ wswz(row)) + 2 * (col & 7);
  };

  auto compute = [&](int stage) {
    const char* sD = smem + stage * 2 * WB_TILE;
    const char* sG = sD + WB_TILE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int rowa = kk * 32 + 8 * kq + q;  // rows rowa and rowa + 4
      wbf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int cb = wm * 64 + 16 * i;
        const w4i16 lo = wtr16(sD + tr_off(rowa, cb)), hi = wtr16(sD + tr_off(rowa + 4, cb));
        const w4i16 v8[2] = {lo, hi};
        fa[i] = __builtin_bit_cast(wbf16x8, v8);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cb = wn * 64 + 16 * j;
        const w4i16 lo = wtr16(sG + tr_off(rowa, cb)), hi = wtr16(sG + tr_off(rowa + 4, cb));
        const w4i16 v8[2] = {lo, hi};
        fb[j] = __builtin_bit_cast(wbf16x8, v8);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  };

  if (nsteps > 0) issue(0, 0);
  for (int s = 0; s < nsteps; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (s + 1 < nsteps) issue(s + 1, (s + 1) & 1);
    compute(s & 1);
  }

  // epilogue: acc[i][j][e] = C[r0 + wm*64 + 16i + 4*(lane>>4) + e][c0 + wn*64 + 16j + (lane&15)]
  const int rq = 4 * (lane >> 4), cl = lane & 15;
  if (p.dW) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = c0 + wn * 64 + 16 * j + cl;
      const int tt = n / p.Cg, cc = n - tt * p.Cg;
      if (n >= p.Ncol || cc >= p.Cg_out) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = r0 + wm * 64 + 16 * i + rq + e;
          if (m < p.R) p.dW[((long long)m * p.Cg_out + cc) * 16 + tt] = acc[i][j][e];
        }
    }
    return;
  }
  float* slab = p.ws + (long long)split * p.R * p.Ncol;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = c0 + wn * 64 + 16 * j + cl;
      if (n >= p.Ncol) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = r0 + wm * 64 + 16 * i + rq + e;
        if (m < p.R) slab[(long long)m * p.Ncol + n] = acc[i][j][e];
      }
    }
}

// ------------------------------------------------------------------------- host
struct WbPlan {
  int mtiles, ntiles, nsplit, pchunk;
};

static WbPlan wb_plan(int P, int R, int Cg) {
  WbPlan pl{};
  pl.mtiles = cdiv(R, WB_BM);
  pl.ntiles = cdiv(16LL * Cg, WB_BN);
  const long long tiles = (long long)pl.mtiles * pl.ntiles;
  const int steps = cdiv(P, WB_BK);
  int ns = 1;
  // ~2 blocks per CU, at least 8 K-steps (512 pixels) per split
  while (tiles * ns < 512 && ns * 2 <= 256 && steps / (ns * 2) >= 8) ns *= 2;
  pl.pchunk = cdiv(steps, ns) * WB_BK;
  pl.nsplit = cdiv(P, pl.pchunk);
  return pl;
}

bool wgrad_bf16_eligible(int B, const stc_view& D, int R, const stc_view& G, int Cg) {
  const long long dbytes = (long long)B * D.bs * 2, gbytes = (long long)B * G.bs * 2;
  const long long P = (long long)B * D.H * D.W;
  return R % 8 == 0 && Cg % 8 == 0 && D.cs == 1 && G.cs == 1 && D.co % 8 == 0 && G.co % 8 == 0 && D.ps % 8 == 0 &&
         G.ps % 8 == 0 && dbytes < (1ll << 31) && gbytes < (1ll << 31) && P < (1 << 24);
}

int64_t wgrad_bf16_workspace(int B, int Hd, int Wd, int R, int Cg) {
  const WbPlan pl = wb_plan(B * Hd * Wd, R, Cg);
  if (pl.nsplit <= 1) return 0;
  return (int64_t)pl.nsplit * R * 16LL * Cg * 4;
}

__global__ void wgrad_reduce_kernel(const float* ws, int nsplit, int R, int Cg, int Cg_out, float* dW);

int wgrad_bf16(int B, int stride, stc_view D, int R, stc_view G, int Cg, int Cg_out, float* dW, void* workspace,
               int64_t workspace_bytes, hipStream_t st) {
  WbParams p{};
  p.d = (const char*)D.p; p.d_bytes = (unsigned)((long long)B * D.bs * 2);
  p.d_bs = (int)D.bs; p.d_rs = (int)D.rs; p.d_ps = D.ps; p.d_co = D.co;
  p.g = (const char*)G.p; p.g_bytes = (unsigned)((long long)B * G.bs * 2);
  p.g_bs = (int)G.bs; p.g_rs = (int)G.rs; p.g_ps = G.ps; p.g_co = G.co;
  p.GH = D.H; p.GW = D.W; p.IH = G.H; p.IW = G.W; p.stride = stride;
  p.R = R; p.Cg = Cg; p.Ncol = 16 * Cg; p.Cg_out = Cg_out;
  p.P = B * D.H * D.W;
  p.inv_ghw = 1.0f / (float)(D.H * D.W);
  p.inv_gw = 1.0f / (float)D.W;
  const WbPlan pl = wb_plan(p.P, R, Cg);
  p.mtiles = pl.mtiles; p.ntiles = pl.ntiles; p.nsplit = pl.nsplit; p.pchunk = pl.pchunk;
  dim3 grid(pl.mtiles * pl.ntiles, 1, pl.nsplit);
  const size_t lds = 2 * 2 * WB_TILE;
  if (pl.nsplit <= 1) {
    p.dW = dW;
    hipLaunchKernelGGL(wgrad_bf16_kernel, grid, dim3(256), lds, st, p);
    STC_CHECK_LAUNCH();
    return 0;
  }
  const int64_t need = (int64_t)pl.nsplit * R * 16LL * Cg * 4;
  STC_REQUIRE(workspace && workspace_bytes >= need, "wgrad bf16: workspace %lld < %lld", (long long)workspace_bytes,
              (long long)need);
  p.ws = (float*)workspace;
  hipLaunchKernelGGL(wgrad_bf16_kernel, grid, dim3(256), lds, st, p);
  STC_CHECK_LAUNCH();
  const long long total = (long long)R * 16 * Cg_out;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, (const float*)p.ws, pl.nsplit, R, Cg, Cg_out,
                     dW);
  STC_CHECK_LAUNCH();
  return 0;
}

}  // namespace stc
