// bf16 weight gradient of the 4x4 conv / convT family on MFMA, staged by LDS-DMA.
//
//   C[r][col] = sum_p D[p][r] * Gcol[p][col],   col = tap*Cg + ci,
//   Gcol[p][tap, ci] = G[b, oy*s + kh - 1, ox*s + kw - 1, ci]      (tap = kh*4 + kw)
//   Conv2d s2/s1 : D = dy (output grid), G = x (input);  ConvT s2 : D = x (input grid), G = dy.
// The reduction runs over pixels.  Both operands are pixel-major in HBM (channels contiguous),
// so each K-step (64 pixels) is DMA'd as [pixel][BM or BN channels] rows with the 16-byte chunk
// index XOR-swizzled on the source side (wswz below), and the MFMA operands (8 consecutive
// pixels of one channel per lane) come out of ds_read_b64_tr_b16 (4 rows x 16 columns per
// 16-lane group, transposed by the LDS) -- conflict-free for the 16x16x32 operand with the two
// 4-row blocks of a 32-lane half 8 rows apart.
// Tiles: 128x128 (4 waves of 64x64), 64x128, a swapped 128x16 for R <= 16, and 8-wave
// 256x256 / 256x128 / 128x256 tiles for the large layers (half the DMA bytes per MFMA of the
// 128x128 tile: the L2->LDS stream, not the MFMA, bounds the small tiles).  2-stage ring (DMA of
// step s+1 under the MFMAs of step s).  The pixel range is split over blockIdx.z into fp32 slabs
// that wgrad_reduce_launch sums in a fixed order; a single split writes torch layout directly.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"

#ifndef STC_SETPRIO
#define STC_SETPRIO 0
#endif

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
  // pixel mapping of a 64-pixel K-step (host-chosen, wb_pmode): 0 general (per-lane division every
  // step); 1 a step stays inside one image row (GW % 64 == 0); 2 a step is whole rows of one image
  // (GW | 64, 64 | GH*GW); 3 a step is whole images (GH*GW | 64).  Modes 1-3: lane pixel = the step's
  // (b0, oy0, ox0), advanced in scalar registers, plus a per-lane constant -- no per-step VALU division.
  int pmode, lg_gw, lg_ghw;
  int mtiles, ntiles;
  // column order of the Gcol operand: 0 tap-major (col = tap*Cg + ci: a tile column range = one tap's channels);
  // 1 channel-group-major (col = (ci/8)*128 + tap*8 + ci%8: a 128-column tile = 8 channels x all 16 taps, whose
  // dW[r][ci][tap] rows are one contiguous 512-byte run -- stored from the tile, no transposing reduce)
  int cmajor;
  float* ws;
  float* dW;
};

typedef short w4i16 __attribute__((ext_vector_type(4)));
typedef __bf16 wbf16x8 __attribute__((ext_vector_type(8)));
using wlds_ptr = __attribute__((address_space(3))) void*;

__device__ __forceinline__ void wdma16(__amdgpu_buffer_rsrc_t r, char* lds_dst, unsigned voff) {
#if !STC_EXP_NODMA  // diagnostic builds only (common.hpp)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (wlds_ptr)lds_dst, 16, voff, 0, 0, 0);
#endif
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

// LDS image swizzle of a [pixel][W channels] operand row (W*2 bytes, CH = W/8 chunks):
//   CH = 16 (256-B rows): chunk ^ ((row&3)<<2 | (row>>2)&3)   (T10 image (b))
//   CH = 32 (512-B rows): the same XOR on the low 4 chunk bits -- the 64 banks span 256 B, so a
//                         512-B row is bank-equivalent to two 256-B rows at the same offsets
//   CH = 8  (128-B rows): chunk ^ (2*((row>>1)&1) + 4*((row>>3)&1))
//   CH = 2  (32-B rows) : none (2-way conflicts on a small operand)
// chosen so that the transposed 16x16x32 operand reads (rows 8g+q, g = 0/1 per 32-lane half) hit
// distinct bank slots.
template <int CH>
__device__ __forceinline__ int wswz(int row) {
  if constexpr (CH >= 16) return ((row & 3) << 2) | ((row >> 2) & 3);
  else if constexpr (CH == 8) return 2 * ((row >> 1) & 1) + 4 * ((row >> 3) & 1);
  else return 0;
}
__device__ __forceinline__ int wswz_rt(int ch, int row) {
  return ch >= 16 ? wswz<16>(row) : (ch == 8 ? wswz<8>(row) : 0);
}

constexpr int WB_BK = 64;

// Epilogue of one tile: acc[i][j][e] = C[a0 + wm*TM + 16i + 4*(lane>>4) + e][b0 + wn*TN + 16j + (lane&15)]
// (row, column) = (r, n) or, swapped, (n, r); n = tap*Cg + ci goes to dW[r][ci][tap] -- or the split's fp32 slab.
template <int BM, int BN, int WM, int WN, bool SWAP>
__device__ __forceinline__ void wgrad_store(const WbParams& p, floatx4 (&acc)[BM / WM / 16][BN / WN / 16], int a0, int b0,
                                            int split) {
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int rq = 4 * (lane >> 4), cl = lane & 15;
  float* slab = p.dW ? nullptr : p.ws + (long long)split * p.R * p.Ncol;
  auto put = [&](int r, int n, int tt, int cc, float v) {
    if (r >= p.R || n >= p.Ncol) return;
    if (slab) slab[(long long)r * p.Ncol + n] = v;
    else if (cc < p.Cg_out) p.dW[((long long)r * p.Cg_out + cc) * 16 + tt] = v;
  };
  if constexpr (!SWAP) {
    if (p.cmajor) {
      // channel-group-major columns (one split): the tile through LDS ([BM][BN + 4] fp32, the stages' space), then
      // every dW row's 512-byte runs as 16-byte stores: dest float 16 c8 + t of group g = tile column 128 g + 8 t + c8
      extern __shared__ __attribute__((aligned(16))) char smem[];
      float* tl = reinterpret_cast<float*>(smem);
      constexpr int PT = BN + 4, NT = 64 * WM * WN;
      __syncthreads();  // (the compute waves are done with the stages; loader waves have left)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) tl[(wm * TM + 16 * i + rq + e) * PT + wn * TN + 16 * j + cl] = acc[i][j][e];
      __syncthreads();
      for (int idx = (int)threadIdx.x; idx < BM * BN / 4; idx += NT) {
        const int row = idx / (BN / 4), d = (idx - row * (BN / 4)) * 4;  // d: dest float of the row's BN
        const int g = d >> 7, c8 = (d >> 4) & 7, t0 = d & 15;
        const int r = a0 + row, ch = ((b0 >> 7) + g) * 8 + c8;
        if (r >= p.R || ch >= p.Cg_out || b0 + 128 * g >= p.Ncol) continue;
        const float* q = tl + row * PT + 128 * g + 8 * t0 + c8;
        *reinterpret_cast<float4*>(p.dW + ((long long)r * p.Cg_out + ch) * 16 + t0) = make_float4(q[0], q[8], q[16], q[24]);
      }
      return;
    }
  }
  if (!SWAP && slab) {  // the common split case: plain row-major slab, no tap decomposition
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = b0 + wn * TN + 16 * j + cl;
      if (n >= p.Ncol) continue;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = a0 + wm * TM + 16 * i + rq + e;
          if (r < p.R) slab[(long long)r * p.Ncol + n] = acc[i][j][e];
        }
    }
    return;
  }
  if constexpr (!SWAP) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = b0 + wn * TN + 16 * j + cl;
      const int tt = p.cmajor ? (n >> 3) & 15 : n / p.Cg, cc = p.cmajor ? ((n >> 7) << 3) + (n & 7) : n - tt * p.Cg;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) put(a0 + wm * TM + 16 * i + rq + e, n, tt, cc, acc[i][j][e]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = a0 + wm * TM + 16 * i + rq + e;
        const int tt = n / p.Cg, cc = n - tt * p.Cg;
#pragma unroll
        for (int j = 0; j < FN; ++j) put(b0 + wn * TN + 16 * j + cl, n, tt, cc, acc[i][j][e]);
      }
  }
}

// Operand roles: the "row" operand (MFMA M) and the "column" operand (MFMA N) each come from either
// D (plain pixel-major channels r) or Gcol (im2col columns tap*Cg + ci).  SWAP = false: rows = D
// (r), columns = Gcol; SWAP = true (R <= 16): rows = Gcol, columns = D, so the tiny R dimension
// becomes a 16-wide MFMA N tile instead of wasting 7/8 of a 128-row tile.
// LD > 0: LD loader waves issue every LDS-DMA piece into an NST-stage ring, NST-1 steps ahead, and the
// WM*WN compute waves only read fragments and issue MFMAs (one barrier per step).
template <int BM, int BN, int WM, int WN, bool SWAP, bool FAST, int LD, int NST>
__device__ __forceinline__ void wgrad_bf16_body(const WbParams& p) {
  constexpr int NW = WM * WN;
  constexpr int NL = LD > 0 ? LD : NW;                 // waves that issue the DMA
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int CHA = BM / 8, CHB = BN / 8;            // 16-byte chunks per pixel row
  constexpr int ROWA = BM * 2, ROWB = BN * 2;          // bytes per pixel row
  constexpr int PA = WB_BK * ROWA / 1024, PB = WB_BK * ROWB / 1024;  // 1 KiB DMA pieces per step
  constexpr int TILEA = WB_BK * ROWA, TILEB = WB_BK * ROWB;
  constexpr int STAGE = TILEA + TILEB;
  constexpr int IA = (PA + NL - 1) / NL, IB = (PB + NL - 1) / NL;
  static_assert(LD == 0 || NST >= 3, "the loader ring runs at least two steps ahead");
  static_assert(FM >= 1 && FN >= 1 && PA >= 1 && PB >= 1, "tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int lw = LD > 0 ? wave - NW : wave;  // index among the loading waves
  // XCD-aware order over (split, tile): workgroups go round-robin to the 8 XCDs by linear id, so
  // remap the linear id to give every XCD a contiguous run of (split-major) work -- the tiles of one
  // pixel split then share their D / G rows in that XCD's L2 instead of every XCD streaming all splits.
  const int nwg = p.mtiles * p.ntiles;
  const int nlin = nwg * (int)gridDim.z;
  int bid = blockIdx.x + (int)blockIdx.z * nwg;
  {
    const int xcd = bid & 7, q = nlin >> 3, r = nlin & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int split = bid / nwg;
  bid -= split * nwg;
  const int mt = bid / p.ntiles, nt = bid % p.ntiles;
  const int a0 = mt * BM, b0 = nt * BN;  // first row / column of the tile
  const int pbeg = split * p.pchunk;
  const int pend = min(p.P, pbeg + p.pchunk);
  const int nsteps = (pend - pbeg + WB_BK - 1) / WB_BK;
  const int GHW = p.GH * p.GW;

  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)p.d, (short)0, (int)p.d_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)p.g, (short)0, (int)p.g_bytes, 0x00020000);
  const unsigned OOBV = 0x80000000u;

  // A piece of an operand with CH chunks per row covers 64/CH rows; lane -> (row lane/CH, slot lane%CH).
  struct Role {
    int chan_off;     // D: channel offset (co + r); G: co + ci
    int dy, dx;       // G tap offsets
    unsigned pen;     // column out of range
  };
  auto role = [&](bool is_g, int ch_per_row, int piece, int first) -> Role {
    const int rows_pp = 64 / ch_per_row;
    const int row = piece * rows_pp + lane / ch_per_row;
    const int chunk = (lane % ch_per_row) ^ wswz_rt(ch_per_row, row);
    Role ro{};
    if (!is_g) {
      const int r = first + chunk * 8;
      ro.chan_off = p.d_co + r;
      ro.pen = r < p.R ? 0u : OOBV;
    } else {
      const int col = first + chunk * 8;
      const int tap = p.cmajor ? (col >> 3) & 15 : col / p.Cg;
      ro.chan_off = p.g_co + (p.cmajor ? (col >> 7) << 3 : col - tap * p.Cg);
      ro.dy = (tap >> 2) - 1;
      ro.dx = (tap & 3) - 1;
      ro.pen = col < p.Ncol ? 0u : OOBV;
    }
    return ro;
  };
  Role ra_[IA], rb_[IB];
#pragma unroll
  for (int i = 0; i < IA; ++i) ra_[i] = role(SWAP, CHA, lw + NL * i, a0);
#pragma unroll
  for (int i = 0; i < IB; ++i) rb_[i] = role(!SWAP, CHB, lw + NL * i, b0);

  struct Pix {
    int b, oy, ox;
    unsigned pen;
  };
  auto pixel = [&](int rows_pp, int piece, int s) -> Pix {
    const int pix = pbeg + s * WB_BK + piece * rows_pp + lane / (64 / rows_pp);
    Pix px;
    px.pen = pix < pend ? 0u : OOBV;
    const int pp = pix < pend ? pix : pbeg;
    px.b = fdiv(pp, GHW, p.inv_ghw);
    const int rem = pp - px.b * GHW;
    px.oy = fdiv(rem, p.GW, p.inv_gw);
    px.ox = rem - px.oy * p.GW;
    return px;
  };
  auto dma_piece = [&](bool is_g, const Role& ro, const Pix& px, int piece, char* dst) {
    if (!is_g) {
      const unsigned off = (((unsigned)px.b * (unsigned)p.d_bs + (unsigned)px.oy * (unsigned)p.d_rs +
                             (unsigned)px.ox * (unsigned)p.d_ps + (unsigned)ro.chan_off) * 2u) | px.pen | ro.pen;
      wdma16(rd, dst + piece * 1024, off);
    } else {
      const int iy = px.oy * p.stride + ro.dy, ix = px.ox * p.stride + ro.dx;
      const unsigned ipen = ((unsigned)iy < (unsigned)p.IH && (unsigned)ix < (unsigned)p.IW) ? 0u : OOBV;
      const unsigned off = (((unsigned)px.b * (unsigned)p.g_bs + (unsigned)iy * (unsigned)p.g_rs +
                             (unsigned)ix * (unsigned)p.g_ps + (unsigned)ro.chan_off) * 2u) | px.pen | ro.pen | ipen;
      wdma16(rg, dst + piece * 1024, off);
    }
  };

  // ---- fast mapping (pmode 1..3): per-piece lane constants; the step base lives in scalar registers
  struct Lc {
    unsigned off;  // element offset of this lane's source relative to the step base (wraps mod 2^32)
    int cy, cx;    // G: tap-shifted pixel coordinates relative to (oy0*s, ox0*s); a column past Ncol
                   // gets cy = 2^30, so the bounds check that every G piece makes rejects it
    unsigned pen;  // D: the row penalty (r >= R)
  };
  auto lane_const = [&](bool is_g, const Role& ro, int rows_pp, int piece) -> Lc {
    const int d = piece * rows_pp + lane / (64 / rows_pp);
    int db = 0, doy = 0, dox = d;
    if (p.pmode == 2) { doy = d >> p.lg_gw; dox = d & (p.GW - 1); }
    else if (p.pmode == 3) { db = d >> p.lg_ghw; const int r = d & (GHW - 1); doy = r >> p.lg_gw; dox = r & (p.GW - 1); }
    Lc c;
    if (!is_g) {
      c.off = (unsigned)db * (unsigned)p.d_bs + (unsigned)doy * (unsigned)p.d_rs + (unsigned)dox * (unsigned)p.d_ps +
              (unsigned)ro.chan_off;
      c.cy = 0; c.cx = 0;
      c.pen = ro.pen;
    } else {
      c.cy = doy * p.stride + ro.dy;
      c.cx = dox * p.stride + ro.dx;
      c.off = (unsigned)db * (unsigned)p.g_bs + (unsigned)c.cy * (unsigned)p.g_rs + (unsigned)c.cx * (unsigned)p.g_ps +
              (unsigned)ro.chan_off;
      if (ro.pen) c.cy = 1 << 30;
      c.pen = 0;
    }
    return c;
  };
  Lc la_[IA], lb_[IB];
  if constexpr (FAST) {
#pragma unroll
    for (int i = 0; i < IA; ++i) la_[i] = lane_const(SWAP, ra_[i], 64 / CHA, lw + NL * i);
#pragma unroll
    for (int i = 0; i < IB; ++i) lb_[i] = lane_const(!SWAP, rb_[i], 64 / CHB, lw + NL * i);
  }
  // scalar step base (sb0, soy0, sox0) of pixel pbeg, advanced by 64 pixels per issued step
  int sb0 = 0, soy0 = 0, sox0 = 0;
  if constexpr (FAST) {
    sb0 = pbeg / GHW;
    const int r0 = pbeg - sb0 * GHW;
    soy0 = r0 / p.GW;
    sox0 = r0 - soy0 * p.GW;
  }
  auto fast_piece = [&](bool is_g, int rows_pp, const Lc& c, unsigned sbase, int sy, int sx, unsigned tail,
                        int piece, char* dst) {
    unsigned pen = is_g ? 0u : c.pen;
    if (tail) {  // only the last, partial step of the range
      const int d = piece * rows_pp + lane / (64 / rows_pp);
      pen |= (unsigned)d < tail ? 0u : OOBV;
    }
    if (!is_g) {
      wdma16(rd, dst + piece * 1024, ((sbase + c.off) * 2u) | pen);
    } else {
      const unsigned ipen = ((unsigned)(sy + c.cy) < (unsigned)p.IH && (unsigned)(sx + c.cx) < (unsigned)p.IW) ? 0u : OOBV;
      wdma16(rg, dst + piece * 1024, ((sbase + c.off) * 2u) | pen | ipen);
    }
  };

  auto issue = [&](int s, int stage) {
    char* sA = smem + stage * STAGE;
    char* sB = sA + TILEA;
    if constexpr (FAST) {
      const int p0 = pbeg + s * WB_BK;
      const unsigned tail = p0 + WB_BK > pend ? (unsigned)(pend - p0) : 0u;
      const int sy = soy0 * p.stride, sx = sox0 * p.stride;
      const unsigned sd = (unsigned)sb0 * (unsigned)p.d_bs + (unsigned)soy0 * (unsigned)p.d_rs + (unsigned)sox0 * (unsigned)p.d_ps;
      const unsigned sg = (unsigned)sb0 * (unsigned)p.g_bs + (unsigned)sy * (unsigned)p.g_rs + (unsigned)sx * (unsigned)p.g_ps;
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        const int pc = lw + NL * i;
        if (pc < PA) fast_piece(SWAP, 64 / CHA, la_[i], SWAP ? sg : sd, sy, sx, tail, pc, sA);
      }
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        const int pc = lw + NL * i;
        if (pc < PB) fast_piece(!SWAP, 64 / CHB, lb_[i], SWAP ? sd : sg, sy, sx, tail, pc, sB);
      }
      // advance the base by one step (64 pixels)
      if (p.pmode == 1) {
        sox0 += WB_BK;
        if (sox0 >= p.GW) { sox0 = 0; if (++soy0 >= p.GH) { soy0 = 0; ++sb0; } }
      } else if (p.pmode == 2) {
        soy0 += WB_BK >> p.lg_gw;
        if (soy0 >= p.GH) { soy0 = 0; ++sb0; }
      } else {
        sb0 += WB_BK >> p.lg_ghw;
      }
    } else if constexpr (CHA == CHB && IA == IB) {  // A and B pieces cover the same pixel rows
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        const int pc = lw + NL * i;
        if (pc < PA) {
          const Pix px = pixel(64 / CHA, pc, s);
          dma_piece(SWAP, ra_[i], px, pc, sA);
          dma_piece(!SWAP, rb_[i], px, pc, sB);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        const int pc = lw + NL * i;
        if (pc < PA) dma_piece(SWAP, ra_[i], pixel(64 / CHA, pc, s), pc, sA);
      }
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        const int pc = lw + NL * i;
        if (pc < PB) dma_piece(!SWAP, rb_[i], pixel(64 / CHB, pc, s), pc, sB);
      }
    }
  };

  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // transposed reads: lane 4q+p of 16-lane group kq reads row 8*kq + q (+4), columns 4p..4p+3 of the
  // fragment's 16 columns; byte offset of (row, col) = row*ROW + 16*((col>>3) ^ swz(row)) + 2*(col&7).
  const int kq = lane >> 4;
  const int q = (lane & 15) >> 2, pcol = lane & 3;
  auto tr_off = [&](int row, int colbase, int rowbytes, int ch) {
    const int col = colbase + 4 * pcol;
    return row * rowbytes + 16 * ((col >> 3) ^ wswz_rt(ch, row)) + 2 * (col & 7);
  };

  auto compute = [&](int stage) {
    const char* sA = smem + stage * STAGE;
    const char* sB = sA + TILEA;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int rowa = kk * 32 + 8 * kq + q;  // rows rowa and rowa + 4
      wbf16x8 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int cb = wm * TM + 16 * i;
        const w4i16 lo = wtr16(sA + tr_off(rowa, cb, ROWA, CHA)), hi = wtr16(sA + tr_off(rowa + 4, cb, ROWA, CHA));
        const w4i16 v8[2] = {lo, hi};
        fa[i] = __builtin_bit_cast(wbf16x8, v8);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int cb = wn * TN + 16 * j;
        const w4i16 lo = wtr16(sB + tr_off(rowa, cb, ROWB, CHB)), hi = wtr16(sB + tr_off(rowa + 4, cb, ROWB, CHB));
        const w4i16 v8[2] = {lo, hi};
        fb[j] = __builtin_bit_cast(wbf16x8, v8);
      }
#if STC_SETPRIO
      __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = exp_mfma(fa[i], fb[j], acc[i][j]);
#if STC_SETPRIO
      __builtin_amdgcn_s_setprio(0);
#endif
    }
  };

  if constexpr (LD > 0) {
    constexpr int P = IA + IB;  // pieces per loader wave per step (every wave issues all of its slots)
    static_assert(IA * NL == PA && IB * NL == PB, "loader pieces split evenly");
    if (wave >= NW) {  // loader: steps 0 .. NST-2 ahead, then one refill per step
#pragma unroll
      for (int i = 0; i < NST - 1; ++i)
        if (i < nsteps) issue(i, i);
      int nxt = NST - 1;
      for (int s = 0; s < nsteps; ++s) {
        const int ahead = min(NST - 2, nsteps - 1 - s);  // steps issued beyond s that may stay in flight
        if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * P) : "memory");
        else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (s + NST - 1 < nsteps) issue(s + NST - 1, nxt);  // into the stage step s - 1 used
        nxt = nxt == NST - 1 ? 0 : nxt + 1;
      }
      return;  // (a terminated wave no longer counts at barriers)
    }
    int cur = 0;
    for (int s = 0; s < nsteps; ++s) {
      __builtin_amdgcn_s_barrier();
      compute(cur);
      cur = cur == NST - 1 ? 0 : cur + 1;
    }
  } else {
    if (nsteps > 0) issue(0, 0);
    for (int s = 0; s < nsteps; ++s) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (s + 1 < nsteps) issue(s + 1, (s + 1) & 1);
      compute(s & 1);
    }
  }

#if STC_EXP_NOEPI
  {
    float s_ = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) s_ += acc[i][j][0] + acc[i][j][3];
    if (s_ == 1.2345f) p.ws[threadIdx.x] = s_;
    return;
  }
#endif
  wgrad_store<BM, BN, WM, WN, SWAP>(p, acc, a0, b0, split);
}

template <int BM, int BN, int WM, int WN, bool SWAP, bool FAST>
__global__ void __launch_bounds__(64 * WM * WN) wgrad_bf16_kernel(const WbParams p) {
  wgrad_bf16_body<BM, BN, WM, WN, SWAP, FAST, 0, 2>(p);
}

// loader-wave blocks (LD DMA-only waves, NST-stage ring), 2 waves per SIMD
template <int BM, int BN, int WM, int WN, bool SWAP, bool FAST, int LD, int NST>
__global__ void __launch_bounds__(64 * (WM * WN + LD), 2) wgrad_bf16_ld_kernel(const WbParams p) {
  wgrad_bf16_body<BM, BN, WM, WN, SWAP, FAST, LD, NST>(p);
}

// ---- halo weight gradient of the stride-2 geometry (Conv2d k4 s2: D = dy on the output grid, G = x; the
// ConvTranspose2d k4 s2 layers: D = x on the input grid, G = dy): dW[r][tap][ci] = sum_p D[p][r] * G[2p + tap offset][ci]
// with tap (ky, kx) at G row 2y + ky - 1, column 2x + kx - 1.  The im2col column operand stages every G pixel once per
// tap (16 times per K-step and 128 columns); here a tile owns 16 channels x all 16 taps (BN = 256) and a K-step of 64
// grid pixels (TR rows x TC columns) stages the G patch those pixels read once -- rows 2 y0 - 1 .. 2 y0 + 2 TR, both
// column parities as planes (plane 0: columns 2j - 1, plane 1: columns 2j, j = x0 .. x0 + TC) -- and every tap's
// fragment reads it: tap (ky, kx) of grid pixel (ty, tx) is patch row 2 ty + ky, plane kx & 1, position tx + kx / 2.
// A patch position is 32 B (16 channels); positions are permuted within 16-position groups (bit 2 ^= bit 3) so that
// the transposed reads of K rows q and q + 8 hit different banks.  Per K-step: D 64 px x 128 channels (16 KB) +
// the patch (<= 20 KB) against 128 x 256 x 64 MACs -- 2x the MACs per staged byte of the 128 x 128 im2col tile.
// Block: 4 compute waves (2 x 2, 64 x 128 each: 4 row x 8 tap fragments) + 4 loader waves, 4-stage ring (144 KiB).
// S1: the PatchGAN's Conv2d k4 s1 p1 (D = dy 31 x 31, G = x 32 x 32; STCGAN/networks.py:172-178) on a virtual 32 x 32
// D grid whose last row and column read as zeros: tap (ky, kx) at G row y + ky - 1, column x + kx - 1, one plane of
// patch columns x0 - 1 .. x0 + TC + 1, patch rows y0 - 1 .. y0 + TR + 1.
template <int TC, bool S1 = false>
struct WhGeom {
  static constexpr int TR = 64 / TC;                 // grid rows per K-step
  static constexpr int NR = S1 ? TR + 3 : 2 * TR + 2;  // patch rows
  static constexpr int NPL = S1 ? 1 : 2;             // column planes
  // positions per plane line: >= TC + 3, whole 16-groups -- TC = 8 (8 x 8 grids, a K-step = one whole image): 17, an
  // odd count, so that the transposed reads of K rows q and q + 8 (grid rows ty and ty + 1: two patch rows = 4 lines
  // apart) land 128 B apart mod 256 (different banks)
  static constexpr int NPOS = TC == 8 ? 17 : TC + 16;
  static constexpr int SLOTS = NR * NPL * NPOS;      // 32-B slots
  static constexpr int PBR = (SLOTS + 31) / 32;      // 1 KiB pieces of the patch
  static constexpr int PB = (PBR + 3) / 4 * 4;       // padded to whole pieces per loader wave
  static constexpr int TILEA = 64 * 128 * 2, TILEB = PB * 1024, STAGE = TILEA + TILEB;
};
static_assert(4 * WhGeom<64>::STAGE <= 163840 && 4 * WhGeom<32>::STAGE <= 163840 && 4 * WhGeom<16>::STAGE <= 163840 &&
                  4 * WhGeom<8>::STAGE <= 163840,
              "halo wgrad LDS");
__device__ __forceinline__ int wh_perm(int pos) { return pos ^ (((pos >> 3) & 1) << 2); }

template <int TC, bool S1>
__global__ void __launch_bounds__(512, 1) wgrad_halo_kernel(const WbParams p) {
  using G = WhGeom<TC, S1>;
  // (S1: p.GH / p.GW are the virtual grid, p.IH / p.IW the G image; D pixels outside D.H = GH - 1, D.W = GW - 1
  // are zeros)
  constexpr int BM = 128, NW = 4, NL = 4, NST = 4;
  constexpr int FM = 4, FN = 8;                      // compute wave tile 64 x 128 (8 taps x 16 channels)
  constexpr int CHA = 16, ROWA = 256;
  constexpr int IA = 16 / NL, IB = G::PB / NL, P = IA + IB;  // pieces per loader wave per step
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwg = p.mtiles * p.ntiles;
  const int nlin = nwg * (int)gridDim.z;
  int bid = blockIdx.x + (int)blockIdx.z * nwg;
  {  // XCD-aware order over (split, tile), as wgrad_bf16_body
    const int xcd = bid & 7, q = nlin >> 3, r = nlin & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int split = bid / nwg;
  bid -= split * nwg;
  const int mt = bid / p.ntiles, nt = bid % p.ntiles;
  const int a0 = mt * BM, c0 = nt * 16;  // D rows a0.., G channels c0 .. c0 + 15 (all 16 taps)
  const int pbeg = split * p.pchunk;
  const int pend = min(p.P, pbeg + p.pchunk);
  const int nsteps = (pend - pbeg + 63) / 64;

  if (wave >= NW) {  // ---- loader waves: steps 0 .. NST - 2 ahead, then one refill per step
    const int lw = wave - NW;
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)p.d, (short)0, (int)p.d_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)p.g, (short)0, (int)p.g_bytes, 0x00020000);
    const unsigned OOBV = 0x80000000u;
    // A (D) pieces: 4 pixel rows of 16 chunks; lane -> (row d, chunk), the chunk swizzled as the transposed reads expect
    unsigned aoff[IA], apen[IA];
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int pc = lw + NL * i;
      const int d = pc * 4 + lane / CHA;
      const int chunk = (lane % CHA) ^ wswz<16>(d);
      const int r = a0 + chunk * 8;
      aoff[i] = (unsigned)((d / TC) * p.d_rs + (d % TC) * p.d_ps + p.d_co + r);
      apen[i] = r < p.R && (!S1 || d % TC < p.GW - 1) ? 0u : OOBV;
    }
    // B (patch) pieces: slot -> (line = row * 2 + plane, position); lane & 1 = the 16-byte half of the 32-B slot
    unsigned boff[IB];
    int brow[IB], bcol[IB];  // G row / column offsets from (2 y0, 2 x0); row 1 << 20 = never valid
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int pc = lw + NL * i;
      const int slot = pc * 32 + (lane >> 1);
      const int line = slot / G::NPOS, pos = wh_perm(slot % G::NPOS);
      const int r = line / G::NPL, plane = line % G::NPL;
      const bool ok = line < G::NPL * G::NR && pos <= (S1 ? TC + 2 : TC);
      brow[i] = ok ? r - 1 : (1 << 20);
      bcol[i] = S1 ? pos - 1 : 2 * pos + plane - 1;
      boff[i] = (unsigned)(brow[i] * p.g_rs + bcol[i] * p.g_ps + p.g_co + c0 + 8 * (lane & 1));
    }
    // step base (b, y0, x0), advanced by 64 pixels per issued step
    const int GHW = p.GH * p.GW;
    int sb = pbeg / GHW;
    int sy = (pbeg - sb * GHW) / p.GW;
    int sx = pbeg - sb * GHW - sy * p.GW;
    auto issue = [&](int s, int stage) {
      char* sA = smem + stage * G::STAGE;
      char* sB = sA + G::TILEA;
      const int p0 = pbeg + s * 64;
      const unsigned tail = p0 + 64 > pend ? (unsigned)(pend - p0) : 64u;
      constexpr int SG = S1 ? 1 : 2;  // G pixels per grid step
      const unsigned bd = (unsigned)sb * (unsigned)p.d_bs + (unsigned)sy * (unsigned)p.d_rs + (unsigned)sx * (unsigned)p.d_ps;
      const unsigned bg = (unsigned)sb * (unsigned)p.g_bs + (unsigned)(SG * sy) * (unsigned)p.g_rs +
                          (unsigned)(SG * sx) * (unsigned)p.g_ps;
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        const int pc = lw + NL * i;
        const unsigned d = (unsigned)(pc * 4 + lane / CHA);
        const bool rowok = !S1 || sy + (int)d / TC < p.GH - 1;  // (S1: the virtual last grid row)
        wdma16(rd, sA + pc * 1024, ((bd + aoff[i]) * 2u) | apen[i] | (d < tail && rowok ? 0u : OOBV));
      }
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        const int pc = lw + NL * i;
        const bool in = (unsigned)(SG * sy + brow[i]) < (unsigned)p.IH && (unsigned)(SG * sx + bcol[i]) < (unsigned)p.IW;
        wdma16(rg, sB + pc * 1024, ((bg + boff[i]) * 2u) | (in ? 0u : OOBV));
      }
      sx += TC;
      if (sx >= p.GW) { sx = 0; sy += G::TR; if (sy >= p.GH) { sy = 0; ++sb; } }
    };
#pragma unroll
    for (int i = 0; i < NST - 1; ++i)
      if (i < nsteps) issue(i, i);
    int nxt = NST - 1;
    for (int s = 0; s < nsteps; ++s) {
      const int ahead = min(NST - 2, nsteps - 1 - s);
      if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * P) : "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (s + NST - 1 < nsteps) issue(s + NST - 1, nxt);
      nxt = nxt == NST - 1 ? 0 : nxt + 1;
    }
    return;
  }

  // ---- compute waves
  const int wm = wave >> 1, wn = wave & 1;
  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int kq = lane >> 4, q = (lane & 15) >> 2, pcol = lane & 3;
  // A (D) fragment offsets: row (pixel) rowa, columns wm*64 + 16 i + 4 pcol
  auto a_off = [&](int row, int i) {
    const int col = wm * 64 + 16 * i + 4 * pcol;
    return row * ROWA + 16 * ((col >> 3) ^ wswz<16>(row)) + 2 * (col & 7);
  };
  // B (patch) fragment offsets of K row d for the taps with column shift h (kx / 2; S1: kx): patch row 2 ty (+ ky)
  // (S1: ty + ky), position tx + h
  constexpr int NH = S1 ? 4 : 2;
  auto b_base = [&](int d, int h) {
    const int ty = d / TC, tx = d % TC;
    return ((S1 ? ty : 2 * ty) * G::NPL * G::NPOS + wh_perm(tx + h)) * 32 + 8 * pcol;
  };
  int bb[2][2][NH];  // [kk][lo/hi][h]
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int h = 0; h < NH; ++h) bb[kk][u][h] = b_base(kk * 32 + 8 * kq + q + 4 * u, h);
  int cur = 0;
  for (int s = 0; s < nsteps; ++s) {
    __builtin_amdgcn_s_barrier();
    const char* sA = smem + cur * G::STAGE;
    const char* sB = sA + G::TILEA;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int rowa = kk * 32 + 8 * kq + q;
      wbf16x8 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const w4i16 v8[2] = {wtr16(sA + a_off(rowa, i)), wtr16(sA + a_off(rowa + 4, i))};
        fa[i] = __builtin_bit_cast(wbf16x8, v8);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {  // tap t = wn * 8 + j: ky = t >> 2, kx = t & 3
        const int t = wn * 8 + j;      // (wn is wave-uniform: the two taps rows of this wave)
        const int ky = t >> 2, kx = t & 3;
        const int lineoff = (S1 ? ky : ky * 2 + (kx & 1)) * G::NPOS * 32;
        const int h = S1 ? kx : kx >> 1;
        const w4i16 v8[2] = {wtr16(sB + bb[kk][0][h] + lineoff), wtr16(sB + bb[kk][1][h] + lineoff)};
        fb[j] = __builtin_bit_cast(wbf16x8, v8);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = exp_mfma(fa[i], fb[j], acc[i][j]);
    }
    cur = cur == NST - 1 ? 0 : cur + 1;
  }
#if STC_EXP_NOEPI
  {
    float s_ = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) s_ += acc[i][j][0] + acc[i][j][3];
    if (s_ == 1.2345f) p.ws[threadIdx.x] = s_;
    return;
  }
#endif
  // epilogue: acc[i][j][e] = C[r = a0 + wm*64 + 16 i + 4 (lane >> 4) + e][tap wn*8 + j][ci = c0 + (lane & 15)]
  const int rq = 4 * (lane >> 4), cl = lane & 15, ci = c0 + cl;
  if (p.dW == nullptr) {  // the split's fp32 slab [R][16 Cg], column tap * Cg + ci
    float* slab = p.ws + (long long)split * p.R * p.Ncol;
    if (ci >= p.Cg) return;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = a0 + wm * 64 + 16 * i + rq + e;
        if (r >= p.R) continue;
#pragma unroll
        for (int j = 0; j < FN; ++j) slab[(long long)r * p.Ncol + (wn * 8 + j) * p.Cg + ci] = acc[i][j][e];
      }
    return;
  }
  if (ci >= p.Cg_out) return;  // torch layout dW[r][ci][tap]: this wave's 8 taps are contiguous
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = a0 + wm * 64 + 16 * i + rq + e;
      if (r >= p.R) continue;
      float* dst = p.dW + ((long long)r * p.Cg_out + ci) * 16 + wn * 8;
      *reinterpret_cast<float4*>(dst) = make_float4(acc[i][0][e], acc[i][1][e], acc[i][2][e], acc[i][3][e]);
      *reinterpret_cast<float4*>(dst + 4) = make_float4(acc[i][4][e], acc[i][5][e], acc[i][6][e], acc[i][7][e]);
    }
}

// ------------------------------------------------------------------------- host
// Tile configurations: {BM (rows), BN (columns), waves, swapped}
struct WbCfg {
  int BM, BN, waves;
  bool swap;
  int stages = 2, loaders = 0;
};
constexpr WbCfg kWbCfg[] = {
    {128, 128, 4, false},        // 0
    {64, 128, 4, false},         // 1: R <= 64
    {128, 16, 4, true},          // 2: R <= 16 (rows = im2col columns, columns = R)
    {256, 256, 8, false},        // 3
    {256, 128, 8, false},        // 4
    {128, 256, 8, false},        // 5
    {128, 128, 4, false, 4, 4},  // 6: + 4 loader waves, 4-stage ring
    {128, 128, 4, false, 3, 4},  // 7: + 4 loader waves, 3-stage ring
    {128, 256, 8, false, 4, 4},  // 8: halo (stride 2, 16 channels x 16 taps per tile; wgrad_halo_kernel)
};
constexpr int WB_HALO = 8;
constexpr int kNumWbCfg = sizeof(kWbCfg) / sizeof(kWbCfg[0]);


struct WbPlan {
  int cfg, BM, BN, mtiles, ntiles, nsplit, pchunk;
  bool slab;    // partial sums go to fp32 slabs + the ordered reduce (always when nsplit > 1)
  bool cmajor;  // channel-group-major columns (WbParams::cmajor): one split whose tiles store torch layout directly
};

// The halo tile (cfg WB_HALO) takes the stride-2 geometry on a D grid of width 16..128 (power of two; a K-step
// = whole grid rows or half a 128-wide row), 16-channel G groups and >= 96 D rows.  stride 0 = unknown (the
// query, which has no stride argument: it plans as stride 2 and sizes the workspace for either).
// Stride 1: a 31-wide D grid (the PatchGAN layer 4 at 256 x 256), run on the virtual 32 x 32 grid.
static bool wb_halo_s1(int GH, int GW, int stride) { return (stride == 1 || stride == 0) && GW == 31 && (GH + 1) % 2 == 0; }
static bool wb_halo_ok(int GH, int GW, int stride, int R, int Cg) {
  if (Cg % 16 != 0 || R < 96) return false;
  if (wb_halo_s1(GH, GW, stride)) return true;
  if (!(stride == 2 || stride == 0)) return false;
  if (!(GW == 8 || GW == 16 || GW == 32 || GW == 64 || GW == 128)) return false;
  return GH % (64 / std::min(GW, 64)) == 0;
}

// force (optional, per call: stc_conv_wgrad_ex / stc_conv_wgrad_query): {tile config, pixel splits (0 = auto; -1 =
// auto without the channel-group-major direct store)};
// NULL or an unknown config = the automatic plan (also the halo config where the geometry does not allow it)
static WbPlan wb_plan(int B, int GH, int GW, int stride, int R, int Cg, const int32_t* force) {
  WbPlan pl{};
  const long long ncol = 16LL * Cg;
  const bool halo = wb_halo_ok(GH, GW, stride, R, Cg);
  int cfg = force ? force[0] : -1;
  int force_ns = force ? std::max(force[1], 0) : 0;
  if (cfg == WB_HALO && !halo) cfg = -1;
  const bool s1v = halo && wb_halo_s1(GH, GW, stride) && (cfg < 0 || cfg >= kNumWbCfg || cfg == WB_HALO);
  const int P = s1v ? B * (GH + 1) * (GW + 1) : B * GH * GW;  // (the stride-1 halo: its virtual grid)
  const int steps = cdiv(P, WB_BK);
  if (cfg < 0 || cfg >= kNumWbCfg) {
    force_ns = 0;
    // (fitted to scripts/tune_wgrad.py over one train step: the 8-wave tiles pay off once each
    // split still has a long pixel loop; 128x128 stays best for the shorter reductions)
    if (R <= 16) cfg = 2;
    // (R <= 64: the 128 x 128 loader tile beats the 64 x 128 tile on the first layers' 524288-pixel problems even
    // with half its rows idle, 32-38 us against 40-45: profiles/r04/wgrad/tune_s1.log)
    else if (R <= 64 && P < 65536) cfg = 1;
    // (8 x 8 grids, P = 2048 at bs 32 -- the generator's 16 -> 8 conv and 8 -> 16 ConvT: the halo tile too, whose
    // patch stages each G pixel once instead of once per tap: profiles/r06/wgrad8/)
    else if (halo && (P >= 4096 || (GW == 8 && P >= 2048))) cfg = WB_HALO;
    else if (ncol >= 1024 && ((R >= 512 && P >= 16384) || (R >= 256 && P >= 65536))) cfg = 3;
    // 128x128 + 4 loader waves, 3-stage ring (96 KiB: a 64 KiB conv block still fits beside it): 5-13 % under
    // cfg 0 in isolation, -0.16 ms per train step in situ (profiles/r03/diag/plan_ab.log)
    else cfg = 7;
  }
  const WbCfg& c = kWbCfg[cfg];
  pl.cfg = cfg;
  pl.BM = c.BM;
  pl.BN = c.BN;
  if (c.swap) { pl.mtiles = (int)cdiv(ncol, c.BM); pl.ntiles = cdiv(R, c.BN); }
  else { pl.mtiles = cdiv(R, c.BM); pl.ntiles = (int)cdiv(ncol, c.BN); }
  if (cfg == WB_HALO) pl.ntiles = Cg / 16;
  const long long tiles = (long long)pl.mtiles * pl.ntiles;
  int ns = 1;
  if (force_ns > 0) {
    ns = std::min(force_ns, std::max(steps, 1));
  } else {
    // about 2 four-wave blocks (one eight-wave block; 4 of the short swapped tile) per CU, at least
    // 8 K-steps (512 pixels) per split
    const long long target = (c.waves == 8 || c.loaders) ? 256 : (c.swap ? 1024 : 512);
    while (tiles * ns < target && ns * 2 <= 256 && steps / (ns * 2) >= 8) ns *= 2;
  }
  pl.pchunk = cdiv(steps, ns) * WB_BK;
  pl.nsplit = cdiv(P, pl.pchunk);
  // A single split writes torch layout dW[r][ci][tap] from the tile directly only when a tile column
  // range covers every tap of its channels (16*Cg <= BN); otherwise those stores are 4-byte scatters at
  // a 64-byte stride (measured ~30 us for a 16.8 MB dW) and the slab + coalesced transposing reduce wins.
  pl.slab = pl.nsplit > 1 || (!c.swap && 16LL * Cg > c.BN && cfg != WB_HALO);
  // ... unless the tile width is a multiple of 128 columns = 8 channels x 16 taps: with the channel-group-major
  // column order each tile row is whole 512-byte runs of dW (the deep levels' single-split gradients: no reduce)
  pl.cmajor = pl.nsplit == 1 && pl.slab && !c.swap && cfg != WB_HALO && c.BN % 128 == 0 && Cg % 8 == 0 &&
              (long long)c.stages * WB_BK * (c.BM + c.BN) * 2 >= (long long)c.BM * (c.BN + 4) * 4 &&  // (LDS tile)
              !(force && force[1] < 0);  // (force {cfg, -1}: the tap-major slab + reduce -- tests / A/B)
  if (pl.cmajor) pl.slab = false;
  return pl;
}
static int64_t wb_ws(const WbPlan& pl, int R, int Cg) { return pl.slab ? (int64_t)pl.nsplit * R * 16LL * Cg * 4 : 0; }

bool wgrad_bf16_eligible(int B, const stc_view& D, int R, const stc_view& G, int Cg) {
  const long long dbytes = (long long)B * D.bs * 2, gbytes = (long long)B * G.bs * 2;
  const long long P = (long long)B * D.H * D.W;
  return R % 8 == 0 && Cg % 8 == 0 && D.cs == 1 && G.cs == 1 && D.co % 8 == 0 && G.co % 8 == 0 && D.ps % 8 == 0 &&
         G.ps % 8 == 0 && dbytes < (1ll << 31) && gbytes < (1ll << 31) && P < (1 << 24);
}

int64_t wgrad_bf16_workspace(int B, int Hd, int Wd, int R, int Cg, const int32_t* force) {
  // (no stride here: enough for the stride-2 plan and for the stride-1 one)
  return std::max(wb_ws(wb_plan(B, Hd, Wd, 0, R, Cg, force), R, Cg), wb_ws(wb_plan(B, Hd, Wd, 1, R, Cg, force), R, Cg));
}

void wgrad_reduce_launch(const float* ws, int nsplit, int R, int Cg, int Cg_out, float* dW, hipStream_t st);

// plan_out = {tile config, BM, BN, pixel splits, slab (1: slabs + reduce kernel)}
void wgrad_bf16_plan(int B, int Hd, int Wd, int R, int Cg, const int32_t* force, int32_t* plan_out) {
  const WbPlan pl = wb_plan(B, Hd, Wd, 0, R, Cg, force);  // (the stride-2 plan)
  plan_out[0] = pl.cfg; plan_out[1] = pl.BM; plan_out[2] = pl.BN; plan_out[3] = pl.nsplit; plan_out[4] = pl.slab;
}

int wgrad_bf16(int B, int stride, stc_view D, int R, stc_view G, int Cg, int Cg_out, float* dW, void* workspace,
               int64_t workspace_bytes, hipStream_t st, const int32_t* force) {
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
  {
    auto lg2 = [](int v) { int l = 0; while ((1 << l) < v) ++l; return (1 << l) == v ? l : -1; };
    const int ghw = D.H * D.W, lgw = lg2(D.W), lghw = lg2(ghw);
    p.pmode = 0;
    if (D.W % WB_BK == 0) p.pmode = 1;
    else if (lgw >= 0 && ghw % WB_BK == 0) p.pmode = 2;
    else if (lghw >= 0 && lgw >= 0 && WB_BK % ghw == 0) p.pmode = 3;
    p.lg_gw = lgw < 0 ? 0 : lgw;
    p.lg_ghw = lghw < 0 ? 0 : lghw;
  }
  // (the stride-2 halo tile needs G on exactly the doubled grid, the stride-1 one on the grid + 1)
  const bool g2x = G.H == 2 * D.H && G.W == 2 * D.W, g1x = G.H == D.H + 1 && G.W == D.W + 1;
  const WbPlan pl = wb_plan(B, D.H, D.W, stride == 2 ? (g2x ? 2 : -1) : (g1x ? 1 : -1), R, Cg, force);
  const bool hs1 = pl.cfg == WB_HALO && stride == 1;
  if (hs1) {  // the virtual grid
    p.GH = D.H + 1; p.GW = D.W + 1;
    p.P = B * p.GH * p.GW;
  }
  p.mtiles = pl.mtiles; p.ntiles = pl.ntiles; p.nsplit = pl.nsplit; p.pchunk = pl.pchunk;
  p.cmajor = pl.cmajor ? 1 : 0;
  dim3 grid(pl.mtiles * pl.ntiles, 1, pl.nsplit);
  const int htc = std::min(p.GW, 64);
  const size_t lds = pl.cfg == WB_HALO
                         ? (size_t)4 * (hs1 ? WhGeom<32, true>::STAGE : htc == 64 ? WhGeom<64>::STAGE
                                                                       : htc == 32 ? WhGeom<32>::STAGE
                                                                       : htc == 16 ? WhGeom<16>::STAGE : WhGeom<8>::STAGE)
                         : (size_t)kWbCfg[pl.cfg].stages * WB_BK * (pl.BM + pl.BN) * 2;
  if (!pl.slab) {
    p.dW = dW;
  } else {
    const int64_t need = (int64_t)pl.nsplit * R * 16LL * Cg * 4;
    STC_REQUIRE(workspace && workspace_bytes >= need, "wgrad bf16: workspace %lld < %lld", (long long)workspace_bytes,
                (long long)need);
    p.ws = (float*)workspace;
  }
  main_timer_begin(st);
#define STC_WB(BM_, BN_, WM_, WN_, SW_, T_)                                                                   \
  if (p.pmode) hipLaunchKernelGGL((wgrad_bf16_kernel<BM_, BN_, WM_, WN_, SW_, true>), grid, dim3(T_), lds, st, p); \
  else hipLaunchKernelGGL((wgrad_bf16_kernel<BM_, BN_, WM_, WN_, SW_, false>), grid, dim3(T_), lds, st, p);
  switch (pl.cfg) {
    case 0: STC_WB(128, 128, 2, 2, false, 256) break;
    case 1: STC_WB(64, 128, 1, 4, false, 256) break;
    case 2: STC_WB(128, 16, 4, 1, true, 256) break;
    case 3:  // (the fast addressing would spill this 256-VGPR kernel: it keeps the per-step division)
      hipLaunchKernelGGL((wgrad_bf16_kernel<256, 256, 2, 4, false, false>), grid, dim3(512), lds, st, p);
      break;
    case 4: STC_WB(256, 128, 4, 2, false, 512) break;
    case 5: STC_WB(128, 256, 2, 4, false, 512) break;
    case 6:
      if (p.pmode) hipLaunchKernelGGL((wgrad_bf16_ld_kernel<128, 128, 2, 2, false, true, 4, 4>), grid, dim3(512), lds, st, p);
      else hipLaunchKernelGGL((wgrad_bf16_ld_kernel<128, 128, 2, 2, false, false, 4, 4>), grid, dim3(512), lds, st, p);
      break;
    case WB_HALO:
      if (hs1) hipLaunchKernelGGL((wgrad_halo_kernel<32, true>), grid, dim3(512), lds, st, p);
      else if (htc == 64) hipLaunchKernelGGL((wgrad_halo_kernel<64, false>), grid, dim3(512), lds, st, p);
      else if (htc == 32) hipLaunchKernelGGL((wgrad_halo_kernel<32, false>), grid, dim3(512), lds, st, p);
      else if (htc == 16) hipLaunchKernelGGL((wgrad_halo_kernel<16, false>), grid, dim3(512), lds, st, p);
      else hipLaunchKernelGGL((wgrad_halo_kernel<8, false>), grid, dim3(512), lds, st, p);
      break;
    default:
      if (p.pmode) hipLaunchKernelGGL((wgrad_bf16_ld_kernel<128, 128, 2, 2, false, true, 4, 3>), grid, dim3(512), lds, st, p);
      else hipLaunchKernelGGL((wgrad_bf16_ld_kernel<128, 128, 2, 2, false, false, 4, 3>), grid, dim3(512), lds, st, p);
      break;
  }
#undef STC_WB
  main_timer_end(st);
  STC_CHECK_LAUNCH();
  if (!pl.slab) return 0;
  wgrad_reduce_launch((const float*)p.ws, pl.nsplit, R, Cg, Cg_out, dW, st);
  STC_CHECK_LAUNCH();
  return 0;
}

}  // namespace stc
