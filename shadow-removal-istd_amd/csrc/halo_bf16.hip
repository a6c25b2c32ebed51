// bf16 Conv2d k4 s2 p1 as an implicit GEMM whose A operand is an LDS-resident input halo (gfx950).
//
// The same problem as igemm_bf16.hip's conv-s2 geometry -- the forward of STCGAN/networks.py:104-105 (U-Net
// down convs) / :167-169,176-178 (PatchGAN convs), and the input gradient of the ConvTranspose2d layers
// (:112-114,119-121,126-128), which has this geometry -- but the im2col tile there stages each input pixel once
// per tap that reads it (4 of the 16 taps of a stride-2 4x4 kernel, per 128-row tile), so half of its L2 -> LDS
// stream is A bytes.  Here a block owns TH whole output rows of one image (BM = TH * GW = 256 GEMM rows) and
// stages, per 32 input channels, kernel row ky and input-column parity, the TH input rows that this (ky, parity)
// reads -- every staged pixel serves two taps (kx and kx + 2):
//
//   stage (ky, parity q) at LDS position P = r * GW + c holds input pixel (2 * (oy0 + r) + ky - 1, 2 * c + q);
//   tap kx of output (r, ox) reads position P = r * GW + ox + d with
//     kx = 0: q = 1, d = -1 (zero at ox = 0)       kx = 1: q = 0, d = 0
//     kx = 2: q = 1, d = 0                          kx = 3: q = 0, d = +1 (zero at ox = GW - 1)
//
// so a stage is exactly BM pixels x 64 B (position = GEMM row), filled by LDS-DMA (input rows outside the image:
// an out-of-range offset, read as zeros); the two edge cases zero the fragment of the lane that addressed the
// neighbouring row's pixel.  A bytes per GEMM row and 32 channels: 8 stages x 64 B against 16 x 64 B for the
// im2col tile -- and B (the packed weights [N][16 taps][Cin]) streams per tap as there.
//
// Block: 4 waves (2 x 2) of 128 x 64 (v_mfma_f32_16x16x32_bf16, 32 accumulator tiles per wave), 80 KiB of LDS,
// so two blocks share a CU and one block's stage waits, epilogue and prologue overlap the other's MFMAs.  LDS
// rows are 64 B with the 16-byte chunk XOR-ed by 2 * ((row >> 2) & 1): every ds_read_b128 lane group of a 16-row
// fragment is conflict-free for ANY first row (the d-shifted A fragments start at odd rows).
// Pipeline per super-step (one A stage + the two B K-steps of its taps, 64 MFMAs per wave): A is loaded two
// super-steps ahead into a 3-slot ring (first touch comes from HBM / the memory-side cache), B one ahead into a
// 2-pair ring (L2-resident); the 8 LDS-DMA pieces a wave issues per super-step are spread one per 8 MFMAs; one
// barrier per super-step.  K order: 64-channel chunk -> ky -> parity (odd, even) -> 32-channel half -> tap
// (0, 2 | 1, 3): fixed, but not the im2col tile's tap-major order, so the fp32 sums differ from it by rounding.
// Epilogue: igemm_bf16.hpp (bias, BatchNorm statistics, the fused BatchNorm-backward sums, 16-byte NHWC stores).
#include <type_traits>

#include "igemm_bf16.hpp"

namespace stc {

constexpr int HB_BM = 256, HB_BN = 128;  // block tile: 256 GEMM rows (whole output rows) x 128 output channels

// Two block shapes over one K loop (RB = bytes per LDS row = 2 x the channels of a stage):
//   RB = 64,  2 x 2 waves of 128 x 64, 80 KiB LDS: two blocks per CU (the default when the grid has >= 512 blocks)
//   RB = 128, 4 x 2 waves of 64 x 64, 160 KiB LDS: one 8-wave block per CU (grids of 256-511 blocks, where two
//             4-wave blocks per CU would leave half the CUs empty)
// LDS: [B pair 0][A slot 0][A slot 1][A slot 2][B pair 1].  The masked edge lanes of A slot 0 / 2 address one pixel
// before / after it: inside the neighbouring B pair, never outside the block's LDS.
template <int RB, int BN = HB_BN, int NB = 2> struct HaloGeom {  // NB: B K-steps per super-step (a pair / a quad)
  static constexpr int A = HB_BM * RB, B = BN * RB;
  static constexpr int A0 = NB * B, B1 = A0 + 3 * A, LDS = 2 * NB * B + 3 * A;
  static constexpr int CH = RB / 16;        // 16-byte chunks per row
  static constexpr int PR = 1024 / RB;      // rows per 1 KiB DMA piece
};
static_assert(HaloGeom<64>::LDS <= 81920 && HaloGeom<128>::LDS <= 163840, "LDS");
static_assert(HaloGeom<64, 64, 4>::LDS <= 81920, "LDS");

// chunk c of LDS row P sits in slot c ^ swz(P): RB = 128: P & 7; RB = 64: 2 * ((P >> 2) & 1) -- for both, every
// ds_read_b128 lane group of a 16-row fragment is conflict-free for ANY first row (the d-shifted A fragments)
template <int RB> __device__ __forceinline__ int hswz(int row) {
  if constexpr (RB == 128) return row & 7;
  else return ((row >> 2) & 1) << 1;
}

// GEOM 0: Conv2d k4 s2 (GEMM grid = output grid); GEOM 1: ConvTranspose2d k4 s2, one sub-pixel phase per block
// (GEMM grid = input grid): phase (py, px) tap (ty, tx) reads input (gy + py - ty, gx + px - tx), so the stage of
// ty holds the input rows gy0 + r + py - ty and its two taps tx read positions r * GW + gx + d, d = px - tx.
// GEOM 2: Conv2d k4 s1 p1 (the PatchGAN's stride-1 conv, STCGAN/networks.py:172-178) on the GEMM grid = its input
// grid (32 x 32; the output is 31 x 31: the last grid row and column are computed from zero padding and masked in
// the epilogue); GEOM 3: its input gradient (GEMM grid = the 32 x 32 output, A = the 31 x 31 output gradient).
// Tap (ky, kx) reads A row y + SG * ky + OF, column x + SG * kx + OF (SG, OF = 1, -1 / -1, 1): the stage of ky
// holds the rows oy0 + r + SG * ky + OF and its four taps read positions r * GW + x + d, d = SG * kx + OF, in two
// super-steps of two taps (every staged pixel serves four taps).
// GEOM 4: ConvTranspose2d k4 s2 with the TWO phases of one row parity per block, (py, 0) and (py, 1): they read the
// same input rows (gy + py - ty) and differ only in the column shift d = px - tx, so one A stage feeds both phases'
// taps -- four B K-steps (a quad) per super-step, two accumulator sets, half GEOM 1's A stream per output.
template <int GEOM, int GW, int BN, bool BNB, int RB, int WM, int WN>
__global__ void __launch_bounds__(64 * WM * WN, 8 / (WM * WN)) halo_conv_kernel(const GParams p) {
  constexpr bool T2 = GEOM == 4;                             // two ConvT phases per block
  constexpr int NB = T2 ? 4 : 2, NPH = T2 ? 2 : 1;           // B K-steps per super-step, accumulator sets
  using G = HaloGeom<RB, BN, NB>;
  constexpr int BM = HB_BM, NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;                  // wave tile: 128 x 64 / 64 x 64
  constexpr int FM = TM / 16, FN = TN / 16;                  // fragments of 16 x 16
  constexpr int KK = RB / 64;                                // 32-deep MFMA steps per K-step
  constexpr int AG = BM / (G::PR * NW), BG = BN / (G::PR * NW);  // DMA pieces per wave: A stage / B K-step
  constexpr int HALVES = 128 / RB;                           // stages per 64-channel chunk and (ky, parity) / ty
  constexpr bool S1 = GEOM == 2 || GEOM == 3;
  constexpr int SG = GEOM == 3 ? -1 : 1, OF = GEOM == 3 ? 1 : -1;
  constexpr int SPC = (GEOM == 1 || T2 ? 2 : 8) * HALVES;    // super-steps per 64-channel chunk
  constexpr int TH = BM / GW;
  constexpr int AH = S1 ? AG / 2 : AG;                       // A pieces per super-step (S1: a stage over two)
  constexpr int NP = NB * BG + AH, NG = NB * KK * FM / 2;    // DMA pieces / 8-MFMA groups per super-step and wave
  static_assert((GW % 16 == 0 || GW == 8) && BM % GW == 0 && TM % GW == 0 && FN == 4 && FM % 2 == 0 && BG >= 1,
                "whole output rows per tile and per wave; 16-row fragments inside an output row or two whole 8-wide rows");
  static_assert(S1 ? AG % 2 == 0 : (T2 || NP >= NG), "every MFMA group issues a piece (S1: whole halves of a stage)");
  static_assert(BM * (BN * 2 + 16) + WM * BN * 16 <= G::LDS, "epilogue tile + statistics merge area");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;

  // XCD-aware bijective remap (blocks b, b + 8, ... share an XCD): consecutive ids -- the 4 phases of a ConvT tile
  // (the same input rows), the N tiles of one A tile, vertically adjacent row tiles (overlapping stages) -- run on
  // one XCD's L2
  const int nwg = p.mtiles * p.ntiles * (GEOM == 1 ? 4 : (T2 ? 2 : 1));
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int ph = GEOM == 1 ? (bid & 3) : (T2 ? 2 * (bid & 1) : 0);  // phase (py, px) = (ph >> 1, ph & 1) (T2: px 0)
  if (GEOM == 1) bid >>= 2;
  if (T2) bid >>= 1;
  const int py = ph >> 1, px = ph & 1;
  const int mt = bid / p.ntiles, nt = bid % p.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  // (a tile = TH whole grid rows; an 8-wide grid's 32-row tile spans GH-row images: image and row per DMA row below)

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.a, (short)0, (int)p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.b, (short)0, (int)p.b_bytes, 0x00020000);

  // ---- DMA lane roles: lane -> (row prow of its piece, LDS slot lane % CH <- source chunk)
  const int prow = lane / G::CH;
  const int schunk = (lane % G::CH) ^ hswz<RB>(prow);  // (pieces are PR-row aligned: hswz(position) == hswz(prow))
  unsigned a_off[AG];
  // pieces whose grid row is the image's first / last: conv-s2 ky = 0 / 3 and ConvT row offset -1 / +1 read padding;
  // S1: the piece's grid row (a piece never straddles one), tested against each stage's row offset, and (GEOM 3) the
  // lanes of the grid column past the A image's last (read as zeros)
  unsigned top = 0, bot = 0, colpen = 0;
  int oyg[AG];
#pragma unroll
  for (int g = 0; g < AG; ++g) {
    const int pos = (wave * AG + g) * G::PR + prow;
    const int r = pos / GW, c = pos % GW;
    const int gr = mt * TH + r;  // grid row of the whole batch
    const int img = gr / p.GH, oy = gr - img * p.GH;
    const int s_ = GEOM == 0 ? 2 : 1;  // input rows / columns per grid step
    a_off[g] = (unsigned)(img * p.a_bs + p.a_co) + (unsigned)(s_ * oy) * (unsigned)p.a_rs +
               (unsigned)(s_ * c) * (unsigned)p.a_ps + (unsigned)(schunk * 8);
    top |= (oy == 0 ? 1u : 0u) << g;
    bot |= (GEOM == 0 ? 2 * oy + 2 >= p.IH : oy == p.GH - 1) ? (1u << g) : 0u;
    oyg[g] = oy;
    colpen |= (c >= p.IW ? 1u : 0u) << g;
  }
  unsigned b_off[BG];
#pragma unroll
  for (int h = 0; h < BG; ++h) {
    const int n = n0 + (wave * BG + h) * G::PR + prow;
    b_off[h] = n < p.N ? (unsigned)(ph * p.b_phase_stride + n * p.K + schunk * 8) : OOB;
  }
  const int cin = p.cin;

  // GEOM 0: super-step ss = ((chunk * 4 + ky) * 2 + q) * HALVES + half: parity q = 0 odd (taps 0, 2) / 1 even
  // (taps 1, 3); GEOM 1: ss = (chunk * 2 + ty) * HALVES + half (taps tx = 0, 1).  half = the 32-channel half of the
  // 64-channel chunk (RB = 64: the two halves of a pixel's 128-byte line back to back).  Its A stage goes to A slot
  // ss % 3, its two B K-steps to B pair ss & 1.
  // S1: stage st = ((chunk * 4 + ky) * HALVES + half) (super-steps 2 st, 2 st + 1: taps kx = 0, 1 | 2, 3)
  auto ss_terms = [&](int ss, int& half, int& odd, int& ky, int& ch) {
    half = HALVES == 2 ? (ss & 1) : 0;
    const int t = HALVES == 2 ? ss >> 1 : ss;
    if constexpr (GEOM == 0) {
      odd = (t & 1) ^ 1;
      ky = (t >> 1) & 3;
      ch = t >> 3;
    } else if constexpr (GEOM == 1 || T2) {  // (ky = ty)
      odd = 0;
      ky = t & 1;
      ch = t >> 1;
    } else {  // (ss = the stage)
      odd = 0;
      ky = t & 3;
      ch = t >> 2;
    }
  };
  auto a_terms = [&](int ss, unsigned& delta, unsigned& pen) {
    int half, odd, ky, ch;
    ss_terms(ss, half, odd, ky, ch);
    if constexpr (GEOM == 0) {
      delta = (unsigned)((ky - 1) * p.a_rs + odd * p.a_ps + ch * 64 + half * 32);
      pen = ky == 0 ? top : (ky == 3 ? bot : 0u);
    } else if constexpr (GEOM == 1 || T2) {
      const int dy = py - ky;
      delta = (unsigned)(dy * p.a_rs + ch * 64 + half * 32);
      pen = dy < 0 ? top : (dy > 0 ? bot : 0u);
    } else {  // (ss = the stage)
      const int dy = SG * ky + OF;
      delta = (unsigned)(dy * p.a_rs + ch * 64 + half * 32);
      pen = colpen;
#pragma unroll
      for (int g = 0; g < AG; ++g) pen |= ((unsigned)(oyg[g] + dy) >= (unsigned)p.IH ? 1u : 0u) << g;
    }
  };
  auto b_k0 = [&](int ss, int j) {
    int half, odd, ky, ch;
    ss_terms(S1 ? ss >> 1 : ss, half, odd, ky, ch);
    if constexpr (T2)  // K-step j = 2 px + tx of the quad: phase (py, px) (its weights one phase stride on), tap (ty, tx)
      return (unsigned)((j >> 1) * p.b_phase_stride + (2 * ky + (j & 1)) * cin + ch * 64 + half * 32);
    const int tap = GEOM == 0 ? 4 * ky + (odd ? 2 * j : 2 * j + 1) : (GEOM == 1 ? 2 * ky + j : 4 * ky + 2 * (ss & 1) + j);
    return (unsigned)(tap * cin + ch * 64 + half * 32);
  };
  auto piece_a = [&](char* sA, unsigned delta, unsigned pen, int g) {
    dma16(ra, sA + (wave * AG + g) * 1024, ((a_off[g] + delta) * 2u) | (((pen >> g) & 1u) << 31));
  };
  auto piece_b = [&](char* sB, unsigned k0, int j, int h) {
#if !STC_EXP_NOBDMA  // (diagnostic builds: the B stream compiled out)
    dma16(rb, sB + j * G::B + (wave * BG + h) * 1024, ((b_off[h] + k0) * 2u) | (b_off[h] & OOB));
#endif
  };
  auto issue_a = [&](int ss, int aslot) {
    unsigned delta, pen;
    a_terms(ss, delta, pen);
#pragma unroll
    for (int g = 0; g < AG; ++g) piece_a(smem + G::A0 + aslot * G::A, delta, pen, g);
  };
  auto issue_b = [&](int ss) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const unsigned k0 = b_k0(ss, j);
#pragma unroll
      for (int h = 0; h < BG; ++h) piece_b(smem + ((ss & 1) ? G::B1 : 0), k0, j, h);
    }
  };

  floatx4 acc[NPH][FM][FN];
#pragma unroll
  for (int h = 0; h < NPH; ++h)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[h][i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets: row (l & 15) of the fragment, chunk KK * 4 * kk... = 4 kk + (l >> 4); A rows shifted by
  // d = di - 2 (fragment i adds 16 i rows, which keeps hswz: 16 is a multiple of 8)
  const int rl = lane & 15, kq = lane >> 4;
  int a_rd[5][KK], b_rd[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
    for (int di = 0; di < 5; ++di) {
      const int pr = wm * TM + rl + di - 2;
      a_rd[di][kk] = pr * RB + (((4 * kk + kq) ^ hswz<RB>(pr)) * 16);
    }
    b_rd[kk] = (wn * TN + rl) * RB + (((4 * kk + kq) ^ hswz<RB>(rl)) * 16);
  }
  const bf16x8_t zero8 = {};
#if STC_EXP_NOBREAD
  bf16x8_t fb0[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) fb0[j] = reinterpret_cast<const bf16x8_t*>(p.b)[(lane + 64 * j) & 255];
#endif

  // one K-step (RB / 2 deep) from A stage sA / B K-step sBj, A rows shifted by D in [-2, 2]; dma(k) issues LDS-DMA
  // piece k of the future stages after each 8 MFMAs
  // D = DRT: the shift is the runtime value dr in [-1, 1] (the ConvT taps: d = px - tx, block-uniform), one code
  // path for both phase columns
  constexpr int DRT = 9;
  using P_0 = std::integral_constant<int, 0>;
  auto kstep = [&](const char* sA, const char* sBj, auto Dc, auto Pc, auto dma, int dr = 0) {
    constexpr int D = decltype(Dc)::value;
    constexpr int PH = decltype(Pc)::value;  // accumulator set (T2: the phase of the pair)
    constexpr bool RT = D == DRT;
    // edge lanes: the first -d (d < 0) / last d (d > 0) rows of an output row read padding
    // (GW = 8: a fragment is two grid rows -- lanes 0 / 8 start one, 7 / 15 end one)
    constexpr int RM = GW < 16 ? GW : 16;
    const bool mlo = RT ? (dr < 0 && rl % RM == 0) : (D < 0 && rl % RM < -D);
    const bool mhi = RT ? (dr > 0 && rl % RM == RM - 1) : (D > 0 && rl % RM >= RM - D);
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int ard = RT ? (dr < 0 ? a_rd[1][kk] : (dr > 0 ? a_rd[3][kk] : a_rd[2][kk])) : a_rd[(RT ? 0 : D) + 2][kk];
      bf16x8_t fa[FM], fb[FN];
#if STC_EXP_NOBREAD  // (diagnostic builds: B fragments from registers -- no LDS reads of B)
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = fb0[j];
#else
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = *reinterpret_cast<const bf16x8_t*>(sBj + b_rd[kk] + j * 16 * RB);
#endif
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        fa[i] = *reinterpret_cast<const bf16x8_t*>(sA + ard + i * 16 * RB);
        // the fragment's first (d = -1) / last (d = +1) row is an output row's left / right edge: that lane's
        // operand is the zero padding, not the neighbouring row's pixel it addressed
        if constexpr (RT || D < 0) {
          if (GW < 16 || (16 * i) % GW == 0) fa[i] = mlo ? zero8 : fa[i];
        }
        if constexpr (RT || D > 0) {
          if (GW < 16 || (16 * i + 16) % GW == 0) fa[i] = mhi ? zero8 : fa[i];
        }
      }
#pragma unroll
      for (int q = 0; q < FM / 2; ++q) {
#pragma unroll
        for (int i = 2 * q; i < 2 * q + 2; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[PH][i][j] = exp_mfma(fa[i], fb[j], acc[PH][i][j]);
        dma(kk * (FM / 2) + q);
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * FN, 0);  // these 8 MFMAs, then the group's pieces
        __builtin_amdgcn_sched_group_barrier(0x020, (NP + NG - 1) / NG, 0);
      }
    }
  };

  // Per super-step: wait for this wave's pieces of A(ss) and B(ss) -- A(ss + 1), issued after them, may stay in
  // flight -- then the barrier (every wave's pieces landed; every wave done with super-step ss - 1), then refill the
  // slots ss - 1 read, B(ss + 1) and A(ss + 2), one piece per 8 MFMAs of super-step ss (a burst of pieces after
  // the barrier holds the waves at the texture unit before their first MFMA).
  const int nss = (cin / 64) * SPC;  // super-steps (even)
  const int nst = S1 ? nss >> 1 : nss;  // A stages
  issue_a(0, 0);
  issue_b(0);
  issue_a(1, 1);
  int aslot = 0;
  // one super-step; U = q * HALVES + half (compile-time parity and B pair = U & 1); S1: U = half * 2 + tap pair
  auto super_step = [&](int s, auto Uc) {
    constexpr int U = decltype(Uc)::value;
    constexpr int TP = S1 ? (U & 1) : 0;
    const int st = S1 ? s >> 1 : s;  // this super-step's A stage
    if constexpr (S1)  // (the previous super-step's A pieces -- or the prologue's A(1) -- may stay in flight)
      wait_ahead<AH>(s == 0 ? 2 : (((s - 1) >> 1) + 2 < nst ? 1 : 0));
    else
      wait_ahead<AG>(s + 1 < nss ? 1 : 0);
    __builtin_amdgcn_s_barrier();
    const bool nb = s + 1 < nss, na = st + 2 < nst;
    const char* sA = smem + G::A0 + aslot * G::A;
    const char* sB = smem + ((U & 1) ? G::B1 : 0);
    char* rB = smem + ((U & 1) ? 0 : G::B1);  // B(s + 1): the other pair
    char* rA = smem + G::A0 + (aslot == 0 ? 2 : aslot - 1) * G::A;
    unsigned bk[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) bk[j] = b_k0(s + 1, j);
    unsigned adelta, apen;
    a_terms(st + 2, adelta, apen);
    // pieces per super-step and wave: B(s + 1) = NB K-steps x BG, then A(s + 2) = AG; MFMA group gi issues pieces
    // [gi * NP / NG, (gi + 1) * NP / NG)
    auto piece = [&](int k) {
      if (k < NB * BG) {
        if (nb) piece_b(rB, bk[k / BG], k / BG, k % BG);
      } else {
        if (na) piece_a(rA, adelta, apen, TP * AH + k - NB * BG);
      }
    };
    auto group = [&](int gi) {
      for (int k = gi * NP / NG; k < (gi + 1) * NP / NG; ++k) piece(k);
    };
    using D_m1 = std::integral_constant<int, -1>;
    using D_0 = std::integral_constant<int, 0>;
    using D_p1 = std::integral_constant<int, 1>;
    if constexpr (GEOM == 0) {
      if constexpr (U / HALVES == 0) {  // odd parity: taps 0 (d = -1), 2 (d = 0)
        kstep(sA, sB, D_m1{}, P_0{}, [&](int k) { group(k); });
        kstep(sA, sB + G::B, D_0{}, P_0{}, [&](int k) { group(NG / 2 + k); });
      } else {  // even parity: taps 1 (d = 0), 3 (d = +1)
        kstep(sA, sB, D_0{}, P_0{}, [&](int k) { group(k); });
        kstep(sA, sB + G::B, D_p1{}, P_0{}, [&](int k) { group(NG / 2 + k); });
      }
    } else if constexpr (GEOM == 1) {  // ConvT: taps tx = 0 (d = px), 1 (d = px - 1)
      using D_rt = std::integral_constant<int, DRT>;
      kstep(sA, sB, D_rt{}, P_0{}, [&](int k) { group(k); }, px);
      kstep(sA, sB + G::B, D_rt{}, P_0{}, [&](int k) { group(NG / 2 + k); }, px - 1);
    } else if constexpr (T2) {  // phase (py, 0): taps tx = 0 (d = 0), 1 (d = -1); phase (py, 1): d = +1, 0
      using P_1 = std::integral_constant<int, 1>;
      kstep(sA, sB, D_0{}, P_0{}, [&](int k) { group(k); });
      kstep(sA, sB + G::B, D_m1{}, P_0{}, [&](int k) { group(NG / 4 + k); });
      kstep(sA, sB + 2 * G::B, D_p1{}, P_1{}, [&](int k) { group(NG / 2 + k); });
      kstep(sA, sB + 3 * G::B, D_0{}, P_1{}, [&](int k) { group(3 * NG / 4 + k); });
    } else {  // S1: taps kx = 2 TP, 2 TP + 1
      using D_a = std::integral_constant<int, SG * (2 * TP) + OF>;
      using D_b = std::integral_constant<int, SG * (2 * TP + 1) + OF>;
      kstep(sA, sB, D_a{}, P_0{}, [&](int k) { group(k); });
      kstep(sA, sB + G::B, D_b{}, P_0{}, [&](int k) { group(NG / 2 + k); });
    }
    if (!S1 || TP == 1) aslot = aslot == 2 ? 0 : aslot + 1;
  };
  for (int ss = 0; ss < nss; ss += 2 * HALVES) {  // (GEOM 1: U / HALVES selects nothing; one or two ty per pass)
    super_step(ss, std::integral_constant<int, 0>{});
    super_step(ss + 1, std::integral_constant<int, 1>{});
    if constexpr (HALVES == 2) {
      super_step(ss + 2, std::integral_constant<int, 2>{});
      super_step(ss + 3, std::integral_constant<int, 3>{});
    }
  }

#if STC_EXP_NOEPI  // (diagnostic builds: the K loop alone, accumulators kept live)
  {
    float s_ = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) s_ += acc[0][i][j][0] + acc[NPH - 1][i][j][3];
    if (s_ == 1.2345f) p.ws[threadIdx.x] = s_;
    return;
  }
#endif
  igemm_epilogue<BM, BN, WM, WN, BNB>(p, acc[0], m0, n0, ph, mt, 0, smem);
  if constexpr (T2) igemm_epilogue<BM, BN, WM, WN, BNB>(p, acc[1], m0, n0, ph + 1, mt, 0, smem);
}

// ------------------------------------------------------------------------- host
// Eligible: Conv2d k4 s2 p1 on an even input (IH = 2 GH, IW = 2 GW) or ConvTranspose2d k4 s2 p1 (GEMM grid = the
// input grid), whole-row tiles of 256 grid points (GW in {16, 32, 64}, GH a multiple of 256 / GW), 64-channel
// chunks, 16-byte NHWC bf16 views (no split K).  N tile: 128 output channels, 64 for a ConvT with N <= 64.
// Conv2d k4 s1 p1 (kinds STC_CONV_S1 / STC_CONV_S1_DGRAD): a 32-wide GEMM grid only (the PatchGAN's 32 x 32 input
// at 256 x 256); the forward's GEMM grid is its input grid (output + 1 row and column).
// N tile: 64 channels for a ConvT with N <= 64, and for a conv-s2 grid whose 128-channel tiles leave the chip
// below 256 blocks while 64-channel ones fill it (the 16 x 16 level at bs 32: 128 -> 256 blocks of the 4-wave
// 256 x 64 block, 8 waves of 32 x 64); force shapes 3 / 4 take the 64-channel tile (4 / 8 waves) for any conv-s2
// layer (tests / A/B).
static int halo_bn(int kind, long long mtiles, int Cout, int shape) {
  // (ConvT: 64 channels for N <= 64, and where 128-channel tiles leave the chip below 256 blocks while 64-channel
  // ones fill it -- the 8 x 8 grid at bs 32: d4 and the input gradient of the 16 -> 8 conv)
  if (kind == STC_CONVT_S2)
    return Cout <= 64 || (mtiles * 4 * ((Cout + HB_BN - 1) / HB_BN) < 256 && mtiles * 4 * ((Cout + 63) / 64) >= 256) ? 64
                                                                                                                       : HB_BN;
  if (kind != STC_CONV_S2 || shape == 1 || shape == 2) return HB_BN;
  if (shape == 3 || shape == 4) return 64;
  return mtiles * ((Cout + HB_BN - 1) / HB_BN) < 256 && mtiles * ((Cout + 63) / 64) >= 256 ? 64 : HB_BN;
}
static void halo_grid(int kind, int& GH, int& GW) {
  if (kind == STC_CONV_S1) { ++GH; ++GW; }
}
int halo_plan_bn(int kind, int B, int GH, int GW, int Cout, int shape) {
  halo_grid(kind, GH, GW);
  return halo_bn(kind, (long long)B * GH * GW / HB_BM, Cout, shape);
}

bool halo_geometry_ok(int kind, int B, int GH, int GW, int Cin, int Cout) {
  if (kind != STC_CONV_S2 && kind != STC_CONVT_S2 && kind != STC_CONV_S1 && kind != STC_CONV_S1_DGRAD) return false;
  if (Cin % 64 != 0 || Cout % 8 != 0 || Cout > 2048) return false;
  halo_grid(kind, GH, GW);
  // (8-wide grids: a 256-row tile is 32 grid rows, spanning images -- the conv-s2 / ConvT geometries only)
  if (GW == 8) {
    if (kind != STC_CONV_S2 && kind != STC_CONVT_S2) return false;
    if ((long long)B * GH * GW % HB_BM != 0) return false;
  } else if (!(GW == 16 || GW == 32 || GW == 64) || GH % (HB_BM / GW) != 0) {
    return false;
  }
  if ((kind == STC_CONV_S1 || kind == STC_CONV_S1_DGRAD) && GW != 32) return false;
  return 16ll * Cin * Cout * 2 < (1ll << 31);
}

static long long halo_blocks(int kind, int B, int GH, int GW, int Cout) {
  halo_grid(kind, GH, GW);
  const long long mt = (long long)B * GH * GW / HB_BM;
  const int bn = halo_bn(kind, mt, Cout, 0);
  return mt * ((Cout + bn - 1) / bn) * (kind == STC_CONVT_S2 ? 4 : 1);
}

// The automatic plan takes the halo kernel when it fills the chip: >= 256 blocks (one 8-wave block per CU).
bool halo_auto(int kind, int B, int GH, int GW, int Cin, int Cout) {
#if STC_EXP_NOHALO  // diagnostic builds only: the im2col tiles everywhere
  return false;
#endif
  return halo_geometry_ok(kind, B, GH, GW, Cin, Cout) && halo_blocks(kind, B, GH, GW, Cout) >= 256;
}

bool halo_eligible(int kind, int B, const stc_view& x, int Cin, int Cout, const stc_view& y) {
  const bool convt = kind == STC_CONVT_S2;
  const int GH = convt ? x.H : y.H, GW = convt ? x.W : y.W;
  if (!halo_geometry_ok(kind, B, GH, GW, Cin, Cout)) return false;
  if (kind == STC_CONV_S2 && (x.H != 2 * GH || x.W != 2 * GW)) return false;
  if (kind == STC_CONV_S1 && (x.H != GH + 1 || x.W != GW + 1)) return false;
  if (kind == STC_CONV_S1_DGRAD && (x.H != GH - 1 || x.W != GW - 1)) return false;
  if (x.cs != 1 || x.co % 8 != 0 || x.ps % 8 != 0 || x.rs % 8 != 0 || x.bs % 8 != 0) return false;
  return (long long)B * x.bs * 2 < (1ll << 31);
}

int halo_chunks(int kind, int B, int GH, int GW) {
  halo_grid(kind, GH, GW);
  return B * GH * GW / HB_BM * (kind == STC_CONVT_S2 ? 4 : 1);
}

// p: filled by bf16_conv_fwd (geometry, operands, output, epilogue options; vec_out set).  shape: 0 automatic,
// 1 the 8-wave 160 KiB block, 2 the 4-wave 80 KiB block, 3 (conv-s2) the 4-wave 256 x 64 block (force_plan
// {HALO_CFG, shape}: tests / A/B; N <= 64 ConvTs always take the 4-wave 256 x 64 block), 4 the 8-wave 256 x 64
// block (the automatic conv-s2 N-64 block; grids 64 wide keep 4 waves), 5 (ConvT, N <= 64) one phase per block
// (GEOM 1) instead of the automatic phase pair (GEOM 4, the 4-wave 256 x 64 block; automatic when its grid has >= 256
// blocks), 6 (ConvT, N <= 64) the phase pair at any size.  (N = 128 ConvTs keep one phase per block: the phase pair
// needs 8 waves of 64 x 64 there -- two 4-wave accumulator sets of 128 x 64 do not fit -- and measured 75 us against
// 65 for d2 at bs 32, profiles/r05/halo_t2/.)
int halo_launch(GParams& p, hipStream_t st, int shape) {
  const bool convt = p.nphase == 4;
  const int geom = convt ? 1 : (p.in_stride == 2 ? 0 : (p.stepy > 0 ? 2 : 3));
  if (geom == 2) {  // the GEMM grid = the input grid; its last row and column (no output pixel) masked
    const int B = p.M / (p.GH * p.GW);
    p.vmask = 1; p.vh = p.GH; p.vw = p.GW;
    p.GH += 1; p.GW += 1;
    p.M = B * p.GH * p.GW;
    p.inv_ghw = 1.0f / (float)(p.GH * p.GW);
    p.inv_gw = 1.0f / (float)p.GW;
  }
  STC_REQUIRE(p.vec_out && !p.ws && (p.nphase == 1 || convt) && p.M % HB_BM == 0, "halo conv: bad launch parameters");
  p.mtiles = p.M / HB_BM;
  const int bn = halo_bn(convt ? STC_CONVT_S2 : (geom == 0 ? STC_CONV_S2 : STC_CONV_S1), p.mtiles, p.N, shape);
  p.ntiles = (p.N + bn - 1) / bn;
  p.ksplit = 1;
  p.kchunk = p.K;
  p.phase_major = 0;
  // ConvT: the two phases of a row parity per block (GEOM 4) when that still fills the chip (shape 5: one phase per
  // block, GEOM 1 -- tests / A/B)
  const bool t2 = convt && bn == 64 && (shape == 6 || (shape != 5 && p.mtiles * p.ntiles * 2 >= 256));
  const int blocks = p.mtiles * p.ntiles * (t2 ? 2 : p.nphase);
  const dim3 grid((unsigned)blocks);
  const bool bnb = p.part2 != nullptr || p.bnb_act;
  // >= 512 blocks: the 4-wave 80 KiB block, two per CU; fewer: the 8-wave block (one per CU, all CUs busy)
#ifndef STC_EXP_TWO_MIN
#define STC_EXP_TWO_MIN 512
#endif
  const bool two = shape == 2 || (shape != 1 && blocks >= STC_EXP_TWO_MIN) || bn == 64;
  // conv-s2 256 x 64: 8 waves of 32 x 64 in 128 KiB (automatic; e4 in the step 45 us against 59 for the 4-wave
  // 256 x 64 block (force shape 3) and 65 for the im2col tile, profiles/r04/halo/e4_in_step.txt)
  const bool n64_8w = shape != 3;
#define STC_HK(G_, GW_, BN_, B_, RB_, WM_, WN_)                                                               \
  hipLaunchKernelGGL((halo_conv_kernel<G_, GW_, BN_, B_, RB_, WM_, WN_>), grid, dim3(64 * WM_ * WN_),         \
                     (HaloGeom<RB_, BN_, (G_ == 4 ? 4 : 2)>::LDS), st, p)
#define STC_HB(G_, GW_, BN_, RB_, WM_, WN_) \
  if (bnb) STC_HK(G_, GW_, BN_, true, RB_, WM_, WN_); else STC_HK(G_, GW_, BN_, false, RB_, WM_, WN_);
#define STC_H(GW_)                                          \
  case GW_:                                                 \
    if (!convt) {                                           \
      if (bn == 64) {                                       \
        if (n64_8w) { STC_HB(0, GW_, 64, (GW_ <= 32 ? 128 : 64), (GW_ <= 32 ? 8 : 4), 1) } \
        else { STC_HB(0, GW_, 64, 64, 4, 1) }               \
      }                                                     \
      else if (two) { STC_HB(0, GW_, 128, 64, 2, 2) }       \
      else { STC_HB(0, GW_, 128, 128, 4, 2) }               \
    } else if (t2) {                                        \
      STC_HB(4, GW_, 64, 64, 4, 1)                          \
    } else if (bn == 64) {                                  \
      STC_HB(1, GW_, 64, 64, 4, 1)                          \
    } else {                                                \
      if (two) { STC_HB(1, GW_, 128, 64, 2, 2) }            \
      else { STC_HB(1, GW_, 128, 128, 4, 2) }               \
    }                                                       \
    break;
  main_timer_begin(st);
  if (geom >= 2) {
    STC_REQUIRE(p.GW == 32, "halo conv s1: grid width %d", p.GW);
    if (geom == 2) {
      if (two) { STC_HB(2, 32, 128, 64, 2, 2) }
      else { STC_HB(2, 32, 128, 128, 4, 2) }
    } else {
      if (two) { STC_HB(3, 32, 128, 64, 2, 2) }
      else { STC_HB(3, 32, 128, 128, 4, 2) }
    }
  } else {
    switch (p.GW) {
      STC_H(8)
      STC_H(16)
      STC_H(32)
      STC_H(64)
      default:
        return fail(-1, "halo conv: grid width %d", p.GW);
    }
  }
#undef STC_H
#undef STC_HB
#undef STC_HK
  main_timer_end(st);
  STC_CHECK_LAUNCH();
  return 0;
}

}  // namespace stc
