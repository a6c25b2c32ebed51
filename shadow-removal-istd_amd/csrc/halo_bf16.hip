// bf16 Conv2d k4 s2 p1 as an implicit GEMM whose A operand is an LDS-resident input halo (gfx950).
//
// The same problem as igemm_bf16.hip's conv-s2 geometry -- the forward of STCGAN/networks.py:104-105 (U-Net
// down convs) / :167-169,176-178 (PatchGAN convs), and the input gradient of the ConvTranspose2d layers
// (:112-114,119-121,126-128), which has this geometry -- but the im2col tile there stages each input pixel once
// per tap that reads it (4 of the 16 taps of a stride-2 4x4 kernel, per 128-row tile), so the L2 -> LDS stream
// is half A bytes.  Here a block owns TH whole output rows of one image (BM = TH * GW = 256 GEMM rows) and
// stages, per input-channel chunk of 64, kernel row ky and input-column parity, the TH input rows that this
// (ky, parity) reads -- every staged pixel serves two taps (kx and kx + 2):
//
//   stage (ky, parity q) at LDS position P = r * GW + c holds input pixel (2 * (oy0 + r) + ky - 1, 2 * c + q);
//   tap kx of output (r, ox) reads position P = r * GW + ox + d with
//     kx = 0: q = 1, d = -1 (zero at ox = 0)       kx = 1: q = 0, d = 0
//     kx = 2: q = 1, d = 0                          kx = 3: q = 0, d = +1 (zero at ox = GW - 1)
//
// so one stage = exactly BM pixels x 128 B in the same [row][128 B] XOR-swizzled image as the im2col A tile
// (position = GEMM row; the fragment of 16 consecutive rows shifted by d stays conflict-free), filled by
// LDS-DMA (input rows outside the image: an out-of-range offset, read as zeros).  The two edge cases read a
// zero pixel instead (a per-lane address redirect on the fragments that start / end an output row).
// A bytes per block: 8 stages x 32 KiB per 64 channels against 16 x 32 KiB (im2col, 128-row tile, per 128
// rows): 4x fewer A bytes per GEMM row.  B (the packed weights, [N][16 taps][Cin]) is streamed per tap as in
// igemm_bf16.hip.
//
// Pipeline: a super-step = one A stage (4 LDS-DMA pieces per wave) + the two B K-steps of its taps (2 x 2
// pieces), 64 KiB; a two-slot ring (the next super-step's DMA lands under the current one's 64 MFMAs per wave),
// one barrier per super-step; 8 waves (4 x 2) of 64 x 64, v_mfma_f32_16x16x32_bf16.  K order: chunk -> ky ->
// parity (odd, even) -> tap (0, 2 | 1, 3): a fixed order, but not the im2col tile's tap-major one, so the fp32
// sums differ from it by rounding only.  Epilogue: igemm_bf16.hpp (bias, BatchNorm statistics, the fused
// BatchNorm-backward sums, 16-byte NHWC stores).
#include <type_traits>

#include "igemm_bf16.hpp"

#ifndef STC_HALO_IL
#define STC_HALO_IL 1
#endif

namespace stc {

constexpr int HB_BM = 256, HB_BN = 128, HB_WM = 4, HB_WN = 2, HB_NW = HB_WM * HB_WN;
constexpr int HB_A = HB_BM * 128;             // A stage: BM pixels x 64 channels
constexpr int HB_B = HB_BN * 128;             // one B K-step: BN rows x 64 channels
// LDS: [B pair 0][A slot 0][A slot 1][A slot 2][B pair 1] = 160 KiB: one block (8 waves) per CU.  (The masked edge
// lanes of A slot 0 / 2 address one pixel before / after it: inside the neighbouring B pair, never outside LDS.)
constexpr int HB_A0 = 2 * HB_B;
constexpr int HB_LDS = 4 * HB_B + 3 * HB_A;
static_assert(HB_LDS <= 163840, "LDS");

template <int GW, bool BNB>
__global__ void __launch_bounds__(64 * HB_NW) halo_conv_s2_kernel(const GParams p) {
  constexpr int BM = HB_BM, BN = HB_BN, WN = HB_WN, NW = HB_NW;
  constexpr int FM = BM / HB_WM / 16, FN = BN / HB_WN / 16;  // 4 x 4 fragments of 16 x 16 per wave
  constexpr int AG = BM / (8 * NW), BG = BN / (8 * NW);      // DMA pieces per wave: 4 (A stage), 2 (B K-step)
  constexpr int TH = BM / GW;
  static_assert(GW >= 16 && GW <= 64 && BM % GW == 0, "whole output rows per tile, 16-row fragments inside a row");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;

  // XCD-aware bijective remap (blocks b, b + 8, ... share an XCD): consecutive tiles -- the N tiles of one A
  // tile, and vertically adjacent row tiles, whose stages overlap by one input row -- run on one XCD's L2
  const int nwg = p.mtiles * p.ntiles;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int mt = bid / p.ntiles, nt = bid % p.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int tiles_img = p.GH / TH;
  const int img = mt / tiles_img, oy0 = (mt - img * tiles_img) * TH;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.a, (short)0, (int)p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.b, (short)0, (int)p.b_bytes, 0x00020000);

  // ---- DMA lane roles: lane -> (pixel / row prow of its 8-row piece, LDS slot lane & 7 <- source chunk)
  const int prow = lane >> 3;
  const int schunk = (lane & 7) ^ prow;  // (position & 7 == prow: pieces are 8-row aligned)
  unsigned a_off[AG];
  unsigned top = 0, bot = 0;  // pieces whose output row is the image's first / last (ky = 0 / 3 read padding)
#pragma unroll
  for (int g = 0; g < AG; ++g) {
    const int pos = (wave * AG + g) * 8 + prow;
    const int r = pos / GW, c = pos % GW;
    const int oy = oy0 + r;
    a_off[g] = (unsigned)(img * p.a_bs + p.a_co) + (unsigned)(2 * oy) * (unsigned)p.a_rs + (unsigned)(2 * c) * (unsigned)p.a_ps +
               (unsigned)(schunk * 8);
    top |= (oy == 0 ? 1u : 0u) << g;
    bot |= (2 * oy + 2 >= p.IH ? 1u : 0u) << g;
  }
  unsigned b_off[BG];
#pragma unroll
  for (int h = 0; h < BG; ++h) {
    const int n = n0 + (wave * BG + h) * 8 + prow;
    b_off[h] = n < p.N ? (unsigned)(n * p.K + schunk * 8) : OOB;
  }
  const int cin = p.cin;

  // super-step ss: chunk ss >> 3, ky = (ss >> 1) & 3, parity odd (taps 0, 2) for even ss, even (taps 1, 3) for
  // odd ss.  Its A stage goes to A slot ss % 3 (issued two super-steps ahead: the input rows come from HBM / the
  // memory-side cache on first touch), its two B K-steps to B pair ss & 1 (one super-step ahead: the weights are
  // L2-resident).
  auto issue_a = [&](int ss, int aslot) {
    const int ch = ss >> 3, ky = (ss >> 1) & 3, odd = (ss & 1) ^ 1;
    char* sA = smem + HB_A0 + aslot * HB_A;
    const unsigned delta = (unsigned)((ky - 1) * p.a_rs + odd * p.a_ps + ch * 64);
    const unsigned pen = ky == 0 ? top : (ky == 3 ? bot : 0u);
#pragma unroll
    for (int g = 0; g < AG; ++g)
      dma16(ra, sA + (wave * AG + g) * 1024, ((a_off[g] + delta) * 2u) | (((pen >> g) & 1u) << 31));
  };
  auto issue_b = [&](int ss) {
    const int ch = ss >> 3, ky = (ss >> 1) & 3, odd = (ss & 1) ^ 1;
    char* sB = smem + ((ss & 1) ? HB_A0 + 3 * HB_A : 0);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kx = odd ? 2 * j : 2 * j + 1;
      const unsigned k0 = (unsigned)((4 * ky + kx) * cin + ch * 64);
#pragma unroll
      for (int h = 0; h < BG; ++h)
        dma16(rb, sB + j * HB_B + (wave * BG + h) * 1024, ((b_off[h] + k0) * 2u) | (b_off[h] & OOB));
    }
  };

  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets: row (l & 15) of the fragment, chunk 4 kk + (l >> 4); A rows shifted by d
  const int rl = lane & 15, kq = lane >> 4;
  int a_rd[3][2], b_rd[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
    for (int di = 0; di < 3; ++di) {
      const int pr = wm * 64 + rl + di - 1;  // fragment 0's row + d (fragment i adds 16 i rows)
      a_rd[di][kk] = pr * 128 + (((4 * kk + kq) ^ ((rl + di - 1) & 7)) * 16);
    }
    b_rd[kk] = (wn * 64 + rl) * 128 + (((4 * kk + kq) ^ (rl & 7)) * 16);
  }
  const bf16x8_t zero8 = {};

  // one K-step (64 deep) from A stage sA / B K-step sBj, A rows shifted by D; with STC_HALO_IL, dma(kk, half)
  // issues one LDS-DMA piece of the future stages after every 8 MFMAs (see below)
  auto kstep = [&](const char* sA, const char* sBj, auto Dc, auto dma) {
    constexpr int D = decltype(Dc)::value;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        fa[i] = *reinterpret_cast<const bf16x8_t*>(sA + a_rd[D + 1][kk] + i * 16 * 128);
        // the fragment's first (D = -1) / last (D = +1) row is an output row's left / right edge: that lane's
        // operand is the zero padding, not the neighbouring row's pixel it addressed
        if constexpr (D == -1) {
          if ((16 * i) % GW == 0) fa[i] = rl == 0 ? zero8 : fa[i];
        } else if constexpr (D == 1) {
          if ((16 * i + 16) % GW == 0) fa[i] = rl == 15 ? zero8 : fa[i];
        }
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = *reinterpret_cast<const bf16x8_t*>(sBj + b_rd[kk] + j * 16 * 128);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 2 * h; i < 2 * h + 2; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = exp_mfma(fa[i], fb[j], acc[i][j]);
#if STC_HALO_IL
        dma(kk, h);
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * FN, 0);  // these 8 MFMAs, then the piece
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
#endif
      }
    }
  };

  // Per super-step: wait for this wave's pieces of A(ss) and B(ss) -- A(ss + 1), issued after them, may stay
  // in flight -- then the barrier (every wave's pieces landed; every wave done with super-step ss - 1), then
  // refill the slots ss - 1 read: B(ss + 1), A(ss + 2).  STC_HALO_IL: the 8 pieces (per wave) of that refill are
  // spread over the super-step, one after every 8 of its 64 MFMAs, instead of issued as a burst after the barrier
  // (a burst of 64 one-KiB pieces per CU holds the waves at the texture unit before their first MFMA).
  const int nss = (cin / 64) * 8;  // super-steps (even)
  issue_a(0, 0);
  issue_b(0);
  issue_a(1, 1);
  int aslot = 0;
  char* const sB0 = smem;
  char* const sB1 = smem + HB_A0 + 3 * HB_A;
  for (int ss = 0; ss < nss; ss += 2) {
#pragma unroll
    for (int par = 0; par < 2; ++par) {  // even super-step: B pair 0, odd parity (taps 0, 2); odd: B pair 1, even
      const int s = ss + par;
      wait_ahead<AG>(s + 1 < nss ? 1 : 0);
      __builtin_amdgcn_s_barrier();
      const bool nb = s + 1 < nss, na = s + 2 < nss;
      const int na_slot = aslot == 0 ? 2 : aslot - 1;
      const char* sA = smem + HB_A0 + aslot * HB_A;
      const char* sB = par ? sB1 : sB0;
#if STC_HALO_IL
      // the refill's per-super-step terms (wave-uniform), then pieces k = 0..3 (B(s + 1)), 4..7 (A(s + 2))
      const int nch = (s + 1) >> 3, nky = ((s + 1) >> 1) & 3, nodd = ((s + 1) & 1) ^ 1;
      char* rB = smem + (((s + 1) & 1) ? HB_A0 + 3 * HB_A : 0);
      const int ach = (s + 2) >> 3, aky = ((s + 2) >> 1) & 3, aodd = ((s + 2) & 1) ^ 1;
      char* rA = smem + HB_A0 + na_slot * HB_A;
      const unsigned adelta = (unsigned)((aky - 1) * p.a_rs + aodd * p.a_ps + ach * 64);
      const unsigned apen = aky == 0 ? top : (aky == 3 ? bot : 0u);
      auto piece = [&](int k) {
        if (k < 4) {
          if (!nb) return;
          const int j = k >> 1, h = k & 1;
          const int kx = nodd ? 2 * j : 2 * j + 1;
          const unsigned k0 = (unsigned)((4 * nky + kx) * cin + nch * 64);
          dma16(rb, rB + j * HB_B + (wave * BG + h) * 1024, ((b_off[h] + k0) * 2u) | (b_off[h] & OOB));
        } else {
          if (!na) return;
          const int g = k - 4;
          dma16(ra, rA + (wave * AG + g) * 1024, ((a_off[g] + adelta) * 2u) | (((apen >> g) & 1u) << 31));
        }
      };
      if (par == 0) {
        kstep(sA, sB, std::integral_constant<int, -1>{}, [&](int kk, int h) { piece(2 * kk + h); });
        kstep(sA, sB + HB_B, std::integral_constant<int, 0>{}, [&](int kk, int h) { piece(4 + 2 * kk + h); });
      } else {
        kstep(sA, sB, std::integral_constant<int, 0>{}, [&](int kk, int h) { piece(2 * kk + h); });
        kstep(sA, sB + HB_B, std::integral_constant<int, 1>{}, [&](int kk, int h) { piece(4 + 2 * kk + h); });
      }
#else
      if (nb) issue_b(s + 1);
      if (na) issue_a(s + 2, na_slot);
      auto none = [](int, int) {};
      if (par == 0) {
        kstep(sA, sB, std::integral_constant<int, -1>{}, none);
        kstep(sA, sB + HB_B, std::integral_constant<int, 0>{}, none);
      } else {
        kstep(sA, sB, std::integral_constant<int, 0>{}, none);
        kstep(sA, sB + HB_B, std::integral_constant<int, 1>{}, none);
      }
#endif
      aslot = aslot == 2 ? 0 : aslot + 1;
    }
  }

#if STC_EXP_NOEPI  // (diagnostic builds: the K loop alone, accumulators kept live)
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
  igemm_epilogue<BM, BN, HB_WM, HB_WN, BNB>(p, acc, m0, n0, 0, mt, 0, smem);
}

// ------------------------------------------------------------------------- host
// Eligible: Conv2d k4 s2 p1 geometry on an even input (IH = 2 GH, IW = 2 GW), whole-row tiles of 256 rows
// (GW in {16, 32, 64}, GH a multiple of 256 / GW), 64-channel chunks, 16-byte NHWC bf16 views (no split K).
bool halo_geometry_ok(int kind, int B, int GH, int GW, int Cin, int Cout) {
  if (kind != STC_CONV_S2 || Cin % 64 != 0 || Cout % 8 != 0 || Cout > 2048) return false;
  if (!(GW == 16 || GW == 32 || GW == 64) || GH % (HB_BM / GW) != 0) return false;
  return 16ll * Cin * Cout * 2 < (1ll << 31);
}

// The automatic plan takes the halo kernel when it fills the chip: >= 256 blocks (one 8-wave block per CU).
bool halo_auto(int kind, int B, int GH, int GW, int Cin, int Cout) {
  if (!halo_geometry_ok(kind, B, GH, GW, Cin, Cout)) return false;
  return (long long)B * GH * GW / HB_BM * ((Cout + HB_BN - 1) / HB_BN) >= 256;
}

bool halo_eligible(int kind, int B, const stc_view& x, int Cin, int Cout, const stc_view& y) {
  const int GH = y.H, GW = y.W;
  if (!halo_geometry_ok(kind, B, GH, GW, Cin, Cout)) return false;
  if (x.H != 2 * GH || x.W != 2 * GW) return false;
  if (x.cs != 1 || x.co % 8 != 0 || x.ps % 8 != 0 || x.rs % 8 != 0 || x.bs % 8 != 0) return false;
  return (long long)B * x.bs * 2 < (1ll << 31);
}

int halo_chunks(int B, int GH, int GW) { return B * GH * GW / HB_BM; }

// p: filled by bf16_conv_fwd (geometry, operands, output, epilogue options; vec_out set).
int halo_launch(GParams& p, hipStream_t st) {
  STC_REQUIRE(p.vec_out && !p.ws && p.nphase == 1 && p.M % HB_BM == 0, "halo conv: bad launch parameters");
  p.mtiles = p.M / HB_BM;
  p.ntiles = (p.N + HB_BN - 1) / HB_BN;
  p.ksplit = 1;
  p.kchunk = p.K;
  p.phase_major = 0;
  const dim3 grid((unsigned)(p.mtiles * p.ntiles));
  const bool bnb = p.part2 != nullptr;
#define STC_H(GW_)                                                                                                \
  case GW_:                                                                                                       \
    if (bnb) hipLaunchKernelGGL((halo_conv_s2_kernel<GW_, true>), grid, dim3(64 * HB_NW), HB_LDS, st, p);       \
    else hipLaunchKernelGGL((halo_conv_s2_kernel<GW_, false>), grid, dim3(64 * HB_NW), HB_LDS, st, p);          \
    break;
  main_timer_begin(st);
  switch (p.GW) {
    STC_H(16)
    STC_H(32)
    STC_H(64)
    default:
      return fail(-1, "halo conv: output width %d", p.GW);
  }
#undef STC_H
  main_timer_end(st);
  STC_CHECK_LAUNCH();
  return 0;
}

}  // namespace stc
