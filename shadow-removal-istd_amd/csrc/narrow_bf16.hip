// Narrow-N bf16 convolutions on MFMA with an LDS halo tile (gfx950).
//
// The layers with N <= 8 output channels on the ST-CGAN path are HBM-bound on their input:
//   * the generator output ConvTranspose2d (128 -> 1|3 channels, 128^2 -> 256^2, + bias, tanh;
//     STCGAN/networks.py:112-116) and the input gradients of the first Conv2d layers (N = 8,
//     padded 3/4/7 channels) -- ConvT geometry, 4 sub-pixel phases;
//   * the PatchGAN logits Conv2d k4 s1 (512 -> 1, 31^2 -> 30^2, + bias; networks.py:183-184).
// An im2col GEMM would re-read each input element 9-16x through L2.  Here a block stages a
// (TY+halo) x (16+halo) pixel tile of one 64-channel chunk in LDS once (LDS-DMA, XOR-swizzled
// 128-B pixel rows), and every output grid point's whole 3x3 (ConvT) / 4x4 (conv s1)
// neighbourhood is read from that tile.  The reduction runs on v_mfma_f32_16x16x32_bf16 with
// the MFMA M dimension = 16 consecutive grid points of a row and the N dimension = all
// (phase, channel) outputs of a grid point (4N <= 32 for ConvT): per neighbour offset one
// MFMA, whose B fragment holds the weights of the (phase, tap) pairs that read that
// neighbour (zeros elsewhere).  Long reductions (the 8192-deep logits layer) split the
// channel chunks over blocks and reduce fp32 partials in a second pass.
// Two block organisations: narrow_halo_kernel splits the tile's rows over the 4 waves (every wave holds
// every B fragment), narrow_wk_kernel (the default) splits the K dimension over them (each fragment
// loaded once per block), sums the waves' partials through LDS in a fixed order and stores the output
// tile from LDS with row / pixel vector stores.
#include <type_traits>

#include "common.hpp"

namespace stc {

struct HParams {
  const char* a;
  unsigned a_bytes;
  int a_bs, a_rs, a_ps, a_co;  // elements
  int IH, IW, cin;
  int GH, GW, N, NP;           // grid (output grid for conv s1, input grid for ConvT); N' = columns
  const bf16* w;               // packed [phase][N][taps][cin]
  int w_phase_stride;
  char* c;
  long long c_bs, c_rs;
  int c_ps, c_co, c_cs;
  const float* bias;
  int tanh_, out_f32;
  int tiles_x, tiles_per_img;
  int chunks_per_split, nsplit;
  float* ws;  // [split][Mtot][NP] when nsplit > 1
  long long Mtot;  // B * GH * GW
  const char* frag;  // B fragment table (narrow_bfrag_kernel), in the workspace
  int smode;         // narrow_stream_kernel output stores: 0 scalar, 1 NHWC 16-byte pixels, 2 NCHW fp32 rows
};

typedef __bf16 bf16x8_h __attribute__((ext_vector_type(8)));
using lds_vptr_h = __attribute__((address_space(3))) void*;

__device__ __forceinline__ void hdma16(__amdgpu_buffer_rsrc_t r, char* lds_dst, unsigned voff) {
#if !STC_EXP_NODMA  // diagnostic builds only (common.hpp)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_vptr_h)lds_dst, 16, voff, 0, 0, 0);
#endif
}

__device__ __forceinline__ void store_out(const HParams& p, long long off, float v) {
  if (p.out_f32) reinterpret_cast<float*>(p.c)[off] = v;
  else st1<bf16>(reinterpret_cast<bf16*>(p.c) + off, v);
}

// B fragments in MFMA order: frag[((chunk * 2 + kk) * NBR + nb) * NB + j][lane] (16 B each), so that the
// main kernel loads them as whole 1 KiB wave rows with no address arithmetic.  Fragment (nb, j, kk)
// of lane l: column n' = 16j + (l & 15) -> (phase, channel) = (n' / N, n' % N), channels
// 8(l >> 4) .. +8 of the 32-channel half kk; zero where the (phase, neighbour) pair reads no tap.
template <int GEOM, int NB>
__global__ void __launch_bounds__(64) narrow_bfrag_kernel(const HParams p, uint4* __restrict__ frag) {
  constexpr int NBR = GEOM == 0 ? 9 : 16;
  const int f = blockIdx.x, lane = threadIdx.x;  // f = ((chunk * 2 + kk) * NBR + nb) * NB + j
  const int j = f % NB, nb = (f / NB) % NBR, kk = (f / (NB * NBR)) % 2, chunk = f / (NB * NBR * 2);
  const int np = 16 * j + (lane & 15);
  const int c = chunk * 64 + kk * 32 + 8 * (lane >> 4);
  int tap = -1, ph = 0, n = np;
  if (GEOM == 0) {
    const int dy = nb / 3 - 1, dx = nb % 3 - 1;
    ph = np / p.N;
    n = np - ph * p.N;
    const int ty = (ph >> 1) - dy, tx = (ph & 1) - dx;
    if (np < p.NP && ty >= 0 && ty <= 1 && tx >= 0 && tx <= 1) tap = ty * 2 + tx;
  } else {
    if (np < p.NP) tap = nb;  // tap index = (dy+1)*4 + (dx+1)
  }
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (tap >= 0)
    v = *reinterpret_cast<const uint4*>(p.w + (long long)ph * p.w_phase_stride +
                                        ((long long)n * (GEOM == 0 ? 4 : 16) + tap) * p.cin + c);
  frag[(long long)f * 64 + lane] = v;
}

// GEOM 0: ConvT k4 s2 (4 phases, 3x3 neighbourhood, NB column blocks of 16: N' = 4N <= 16*NB)
// GEOM 1: Conv k4 s1 (16 taps, 4x4 neighbourhood, N' = N <= 16)
// Tile: TY grid rows x 16*TXB grid columns; wave w owns rows [w*TY/4, (w+1)*TY/4) and all TXB
// 16-wide column blocks, so each B fragment (held in registers) feeds ROWS*TXB MFMAs.  The DMA of
// chunk c+1 is issued before chunk c's wait (counted vmcnt: the B fragments of chunk c are issued
// first, so they retire before it).
template <int GEOM, int NB, int TY, int TXB>
__global__ void __launch_bounds__(256) narrow_halo_kernel(const HParams p) {
  constexpr int TX = 16 * TXB;
  constexpr int HALO = GEOM == 0 ? 2 : 3;
  constexpr int RY = TY + HALO, RX = TX + HALO;
  constexpr int NPIX = RY * RX;
  constexpr int PIECES = (NPIX + 7) / 8;  // 1 KiB DMA pieces (8 pixels x 128 B)
  constexpr int STAGE = PIECES * 1024;
  constexpr int NBR = GEOM == 0 ? 9 : 16;  // neighbour offsets
  constexpr int ROWS = TY / 4;             // grid rows per wave
  constexpr int WP = (PIECES + 3) / 4;     // DMA pieces per wave (upper bound)
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int img = blockIdx.x / p.tiles_per_img, tix = blockIdx.x % p.tiles_per_img;
  const int y0 = (tix / p.tiles_x) * TY, x0 = (tix % p.tiles_x) * TX;
  const int split = blockIdx.y;
  const int nchunks = p.cin / 64;
  const int cbeg = split * p.chunks_per_split;
  const int cend = min(nchunks, cbeg + p.chunks_per_split);

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.a, (short)0, (int)p.a_bytes, 0x00020000);
  const unsigned OOBV = 0x80000000u;
  const int abase = img * p.a_bs + p.a_co;
  const int schunk = (lane & 7) ^ (lane >> 3);

  auto issue = [&](int chunk, int stage) {
    char* dst = smem + stage * STAGE;
    const int ci = chunk * 64 + schunk * 8;
#pragma unroll
    for (int k = 0; k < WP; ++k) {
      const int pc = wave + 4 * k;
      if (pc >= PIECES) break;
      const int pix = pc * 8 + (lane >> 3);
      const int py = pix / RX, px = pix - py * RX;
      const int iy = y0 - 1 + py, ix = x0 - 1 + px;
      const bool ok = pix < NPIX && (unsigned)iy < (unsigned)p.IH && (unsigned)ix < (unsigned)p.IW;
      const unsigned off = (((unsigned)abase + (unsigned)iy * (unsigned)p.a_rs + (unsigned)ix * (unsigned)p.a_ps +
                             (unsigned)ci) * 2u) | (ok ? 0u : OOBV);
      hdma16(ra, dst + pc * 1024, off);
    }
  };
  // this wave's DMA pieces per chunk (the count vmcnt leaves in flight while chunk c is consumed)
  const int my_pieces = (PIECES - wave + 3) / 4;

  // B fragment of (neighbour nb, column block j, half kk): one coalesced 16-byte load per lane from the
  // fragment table (narrow_bfrag_kernel)
  const uint4* frag = reinterpret_cast<const uint4*>(p.frag);
  auto load_b = [&](int chunk, int nb, int j, int kk) -> bf16x8_h {
    return __builtin_bit_cast(bf16x8_h, frag[((long long)((chunk * 2 + kk) * NBR + nb) * NB + j) * 64 + lane]);
  };

  floatx4 acc[ROWS][TXB][NB];
#pragma unroll
  for (int r = 0; r < ROWS; ++r)
#pragma unroll
    for (int cx = 0; cx < TXB; ++cx)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[r][cx][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int gx = lane & 15;
  if (cbeg < cend) issue(cbeg, 0);
  int stage = 0;
  for (int ch = cbeg; ch < cend; ++ch) {
    bf16x8_h bfr[2][NBR][NB];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int nb = 0; nb < NBR; ++nb)
#pragma unroll
        for (int j = 0; j < NB; ++j) bfr[kk][nb][j] = load_b(ch, nb, j, kk);
    // all waves finished reading stage^1 (chunk ch-1) before it is refilled with chunk ch+1
    if (ch > cbeg) __builtin_amdgcn_s_barrier();
    const bool pre = ch + 1 < cend;
    if (pre) issue(ch + 1, stage ^ 1);
    // chunk ch's pixels and B fragments landed; chunk ch+1's pieces may stay in flight
    if (pre) {
      switch (my_pieces) {  // vmcnt takes an immediate
#define STC_VM(n) case n: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory"); break;
        STC_VM(1) STC_VM(2) STC_VM(3) STC_VM(4) STC_VM(5) STC_VM(6) STC_VM(7) STC_VM(8) STC_VM(9) STC_VM(10)
        STC_VM(11) STC_VM(12) STC_VM(13) STC_VM(14) STC_VM(15) STC_VM(16) STC_VM(17) STC_VM(18) STC_VM(19) STC_VM(20)
        STC_VM(21) STC_VM(22) STC_VM(23) STC_VM(24) STC_VM(25) STC_VM(26) STC_VM(27) STC_VM(28) STC_VM(29) STC_VM(30)
#undef STC_VM
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const char* sT = smem + stage * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int cslot = kk * 4 + (lane >> 4);
#pragma unroll
      for (int nb = 0; nb < NBR; ++nb) {
        const int dy = GEOM == 0 ? nb / 3 - 1 : nb / 4 - 1;
        const int dx = GEOM == 0 ? nb % 3 - 1 : nb % 4 - 1;
#pragma unroll
        for (int r = 0; r < ROWS; ++r)
#pragma unroll
          for (int cx = 0; cx < TXB; ++cx) {
            const int py = wave * ROWS + r + dy + 1, px = 16 * cx + gx + dx + 1;
            const int pix = py * RX + px;
            const bf16x8_h af = *reinterpret_cast<const bf16x8_h*>(sT + pix * 128 + ((cslot ^ (pix & 7)) * 16));
#pragma unroll
            for (int j = 0; j < NB; ++j)
              acc[r][cx][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[kk][nb][j], acc[r][cx][j], 0, 0, 0);
          }
      }
    }
    stage ^= 1;
  }

  // ---- epilogue: acc[r][cx][j][e] = grid point (y0 + wave*ROWS + r, x0 + 16 cx + 4*(lane>>4) + e), column 16j + (lane&15)
  const int np_l = lane & 15;
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    const int gy = y0 + wave * ROWS + r;
    if (gy >= p.GH) continue;
#pragma unroll
    for (int cx = 0; cx < TXB; ++cx)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int gxx = x0 + 16 * cx + 4 * (lane >> 4) + e;
        if (gxx >= p.GW) continue;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const int np = 16 * j + np_l;
          if (np >= p.NP) continue;
          float v = acc[r][cx][j][e];
          if (p.nsplit > 1) {
            const long long m = ((long long)img * p.GH + gy) * p.GW + gxx;
            p.ws[((long long)split * p.Mtot + m) * p.NP + np] = v;
            continue;
          }
          int ph = 0, n = np;
          if (GEOM == 0) { ph = np / p.N; n = np - ph * p.N; }
          if (p.bias) v += p.bias[n];
          if (p.tanh_) v = tanhf(v);
          const int oy = GEOM == 0 ? 2 * gy + (ph >> 1) : gy;
          const int ox = GEOM == 0 ? 2 * gxx + (ph & 1) : gxx;
          store_out(p, (long long)img * p.c_bs + (long long)oy * p.c_rs + (long long)ox * p.c_ps +
                           (long long)(p.c_co + n) * p.c_cs, v);
        }
      }
  }
}

// The same reduction with the K dimension split over the block's waves instead of the rows: wave w owns
// column block j = w % NB and the 32-channel K-slices ks = w / NB + (4 / NB) t of the block's chunks, for
// every row of the tile.  Each B fragment is then loaded from L2 once per block -- in the row-split form
// above every wave loaded all of them, 3/4 of the block's L2 -> CU traffic for the N <= 16 layers.  All of
// the block's chunks are staged at once (one DMA wait, no ring); the partial sums of the waves of K group
// > 0 go through LDS (the A tile's space, after a barrier) to the K-group-0 wave of their column block,
// which adds them in wave order (deterministic) and stores.  3 waves per SIMD (<= 168 VGPRs): the LDS of
// 3 blocks per CU.
template <int GEOM, int NB, int TY, int TXB>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) narrow_wk_kernel(const HParams p) {
  constexpr int TX = 16 * TXB;
  constexpr int HALO = GEOM == 0 ? 2 : 3;
  constexpr int RY = TY + HALO, RX = TX + HALO;
  constexpr int NPIX = RY * RX;
  constexpr int PIECES = (NPIX + 7) / 8;  // 1 KiB DMA pieces per chunk image
  constexpr int CSTRIDE = PIECES * 1024;
  constexpr int NBR = GEOM == 0 ? 9 : 16;
  constexpr int KG = 4 / NB;  // waves per column block
  static_assert(NB == 1 || NB == 2, "NB");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = wave % NB, kg = wave / NB;
  const int img = blockIdx.x / p.tiles_per_img, tix = blockIdx.x % p.tiles_per_img;
  const int y0 = (tix / p.tiles_x) * TY, x0 = (tix % p.tiles_x) * TX;
  const int split = blockIdx.y;
  const int nchunks = p.cin / 64;
  const int cbeg = split * p.chunks_per_split;
  const int nch = min(nchunks, cbeg + p.chunks_per_split) - cbeg;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.a, (short)0, (int)p.a_bytes, 0x00020000);
  const unsigned OOBV = 0x80000000u;
  const int abase = img * p.a_bs + p.a_co;
  const int schunk = (lane & 7) ^ (lane >> 3);
  // every chunk image of the block: piece q = chunk * PIECES + pc, wave-strided
  for (int q = wave; q < nch * PIECES; q += 4) {
    const int c = q / PIECES, pc = q - c * PIECES;
    const int pix = pc * 8 + (lane >> 3);
    const int py = pix / RX, px = pix - py * RX;
    const int iy = y0 - 1 + py, ix = x0 - 1 + px;
    const bool ok = pix < NPIX && (unsigned)iy < (unsigned)p.IH && (unsigned)ix < (unsigned)p.IW;
    const unsigned off = (((unsigned)abase + (unsigned)iy * (unsigned)p.a_rs + (unsigned)ix * (unsigned)p.a_ps +
                           (unsigned)((cbeg + c) * 64 + schunk * 8)) * 2u) | (ok ? 0u : OOBV);
    hdma16(ra, smem + c * CSTRIDE + pc * 1024, off);
  }

  const uint4* frag = reinterpret_cast<const uint4*>(p.frag);
  floatx4 acc[TY][TXB];
#pragma unroll
  for (int r = 0; r < TY; ++r)
#pragma unroll
    for (int cx = 0; cx < TXB; ++cx) acc[r][cx] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int gx = lane & 15;
  const int KS = 2 * nch;
  bool first = true;
  for (int ks = kg; ks < KS || first; ks += KG) {
    const bool have = ks < KS;
    const int ch = cbeg + (ks >> 1), kk = ks & 1;
    bf16x8_h bfr[NBR];
    if (have) {
#pragma unroll
      for (int nb = 0; nb < NBR; ++nb)
        bfr[nb] = __builtin_bit_cast(bf16x8_h, frag[((long long)((ch * 2 + kk) * NBR + nb) * NB + j) * 64 + lane]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (first) {  // the chunk images (every wave's pieces) have landed
      __builtin_amdgcn_s_barrier();
      first = false;
    }
    if (!have) break;
    const char* sT = smem + (ks >> 1) * CSTRIDE;
    const int cslot = kk * 4 + (lane >> 4);
    // pixel pix = c + gx (c a compile-time offset per (row, neighbour, column block)) sits at byte
    // c*128 + lofs[c & 7]: eight per-lane bases, the rest an immediate offset of the read
    int lofs[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) lofs[m] = gx * 128 + ((cslot ^ ((m + gx) & 7)) * 16);
#pragma unroll
    for (int nb = 0; nb < NBR; ++nb) {
      const int dy = GEOM == 0 ? nb / 3 - 1 : nb / 4 - 1;
      const int dx = GEOM == 0 ? nb % 3 - 1 : nb % 4 - 1;
#pragma unroll
      for (int r = 0; r < TY; ++r)
#pragma unroll
        for (int cx = 0; cx < TXB; ++cx) {
          const int c = (r + dy + 1) * RX + 16 * cx + dx + 1;
          const bf16x8_h af = *reinterpret_cast<const bf16x8_h*>(sT + lofs[c & 7] + c * 128);
          acc[r][cx] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[nb], acc[r][cx], 0, 0, 0);
        }
      // one neighbour's reads at a time: hoisting all TY*TXB*NBR fragment reads spills
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // ---- partial sums through LDS: red[kg][j][r][cx][lane]; wave (j, kg) then sums rows
  // [kg*RPW, (kg+1)*RPW) of column block j over the K groups in order (deterministic)
  constexpr int RPW = TY / KG;
  __syncthreads();  // every wave is done with the chunk images
  floatx4* red = reinterpret_cast<floatx4*>(smem);
#pragma unroll
  for (int r = 0; r < TY; ++r)
#pragma unroll
    for (int cx = 0; cx < TXB; ++cx) red[(((kg * NB + j) * TY + r) * TXB + cx) * 64 + lane] = acc[r][cx];
  __syncthreads();
  floatx4 o[RPW][TXB];
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
    for (int cx = 0; cx < TXB; ++cx) o[rr][cx] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int g = 0; g < KG; ++g)
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
      for (int cx = 0; cx < TXB; ++cx) {
        const floatx4 v = red[(((g * NB + j) * TY + kg * RPW + rr) * TXB + cx) * 64 + lane];
        o[rr][cx][0] += v[0]; o[rr][cx][1] += v[1]; o[rr][cx][2] += v[2]; o[rr][cx][3] += v[3];
      }

  // ---- epilogue: o[rr][cx][e] = grid point (y0 + kg*RPW + rr, x0 + 16 cx + 4*(lane>>4) + e), column 16j + (lane&15)
  const int np = 16 * j + (lane & 15);
  const bool col_ok = np < p.NP;
  int ph = 0, n = np;
  if (GEOM == 0) { ph = np / p.N; n = np - ph * p.N; }
  if (p.nsplit > 1) {  // fp32 partials of this channel-chunk split, summed by narrow_reduce_kernel
    if (!col_ok) return;
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) {
      const int gy = y0 + kg * RPW + rr;
      if (gy >= p.GH) break;
#pragma unroll
      for (int cx = 0; cx < TXB; ++cx)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int gxx = x0 + 16 * cx + 4 * (lane >> 4) + e;
          if (gxx >= p.GW) continue;
          const long long m = ((long long)img * p.GH + gy) * p.GW + gxx;
          p.ws[((long long)split * p.Mtot + m) * p.NP + np] = o[rr][cx][e];
        }
    }
    return;
  }
  // the block's output tile staged in LDS as [oy][ox][n] (behind the partials),
  // then written with whole-row (NCHW fp32) or whole-pixel (NHWC bf16, 8 channels) vector stores
  constexpr int SC = GEOM == 0 ? 2 : 1;  // output pixels per grid point per axis
  constexpr int OYL = SC * TY, OXL = SC * TX;
  float* stg = reinterpret_cast<float*>(smem + (size_t)4 * TY * TXB * 1024);
  const int N = p.N;
  if (col_ok) {
    const float bz = p.bias ? p.bias[n] : 0.f;
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
      for (int cx = 0; cx < TXB; ++cx)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = o[rr][cx][e] + bz;
          if (p.tanh_) v = tanhf(v);
          const int ly = kg * RPW + rr, lx = 16 * cx + 4 * (lane >> 4) + e;
          const int oyl = GEOM == 0 ? 2 * ly + (ph >> 1) : ly, oxl = GEOM == 0 ? 2 * lx + (ph & 1) : lx;
          stg[(oyl * OXL + oxl) * N + n] = v;
        }
  }
  __syncthreads();
  const int OH = SC * p.GH, OW = SC * p.GW;
  const int oy0 = SC * y0, ox0 = SC * x0;
  const long long cbase = (long long)img * p.c_bs + (long long)p.c_co * p.c_cs;
  const bool f32_rows = p.out_f32 && p.c_ps == 1 && ((p.c_rs | p.c_cs | (int)(p.c_bs & 3) | p.c_co) & 3) == 0;
  const bool bf_pix = !p.out_f32 && N == 8 && p.c_cs == 1 && ((p.c_ps | p.c_rs | (int)(p.c_bs & 7) | p.c_co) & 7) == 0;
  if (f32_rows) {
    // (n, oy) rows of OXL floats: one float4 per thread-iteration
    for (int t = tid; t < N * OYL * (OXL / 4); t += 256) {
      const int xq = t % (OXL / 4), rest = t / (OXL / 4);
      const int oyl = rest % OYL, nn = rest / OYL;
      const int oy = oy0 + oyl, ox = ox0 + 4 * xq;
      if (oy >= OH || ox >= OW) continue;
      const float* sp = stg + (oyl * OXL + 4 * xq) * N + nn;
      float* dst = reinterpret_cast<float*>(p.c) + cbase + (long long)oy * p.c_rs + ox + (long long)nn * p.c_cs;
      if (ox + 4 <= OW) {
        *reinterpret_cast<float4*>(dst) = make_float4(sp[0], sp[N], sp[2 * N], sp[3 * N]);
      } else {
        for (int i = 0; i < OW - ox; ++i) dst[i] = sp[i * N];
      }
    }
  } else if (bf_pix) {
    // one pixel = 8 channels = one 16-byte store
    for (int t = tid; t < OYL * OXL; t += 256) {
      const int oxl = t % OXL, oyl = t / OXL;
      const int oy = oy0 + oyl, ox = ox0 + oxl;
      if (oy >= OH || ox >= OW) continue;
      const float* sp = stg + t * 8;
      uint4 u;
      u.x = pack_bf16x2(sp[0], sp[1]); u.y = pack_bf16x2(sp[2], sp[3]);
      u.z = pack_bf16x2(sp[4], sp[5]); u.w = pack_bf16x2(sp[6], sp[7]);
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.c) + cbase + (long long)oy * p.c_rs + (long long)ox * p.c_ps) = u;
    }
  } else {
    for (int t = tid; t < OYL * OXL * N; t += 256) {
      const int nn = t % N, pix = t / N;
      const int oxl = pix % OXL, oyl = pix / OXL;
      const int oy = oy0 + oyl, ox = ox0 + oxl;
      if (oy >= OH || ox >= OW) continue;
      store_out(p, cbase + (long long)oy * p.c_rs + (long long)ox * p.c_ps + (long long)nn * p.c_cs, stg[t]);
    }
  }
}

// ---- streaming ConvT (GEOM 0) for the HBM-bound full-resolution edges: the generator output layer (CIN 128, N 1|3)
// and the first convs' input gradients (CIN 64, N 8).  A block owns one image's strip of SR grid rows x 64 grid
// columns (16 per wave, all CIN channels); its SR + 2 input rows (66 pixels each: one halo column either side) flow
// through an NS-slot LDS ring by LDS-DMA, NS - 1 rows ahead of the MFMAs, so each input pixel crosses HBM once per
// strip (+2/SR for the halo rows) and ~50 KiB per block are in flight.  Grid row gy reads input rows gy-1, gy, gy+1:
// each staged row's A fragments (3 column shifts x CIN/32 K-steps) are read once and feed the three output rows it
// touches, accumulated in three rotating register tiles; a row is complete (and stored, + bias, tanh) two input rows
// after it started.  The whole CIN x 9 x N' B-fragment table lives in registers.  LDS rows: pixel-major, 16-byte
// channel chunks XOR-swizzled by pixel (conflict-free A reads).  Every wave's VMEM count per iteration is known
// (its DMA pieces per row + 4 NB stores per output row), so the ring waits are exact counted vmcnt.
constexpr int NS_SR = 16;  // grid rows per block strip
constexpr int NS_TW = 64;  // grid columns per block

__device__ __forceinline__ void vm_wait_dyn(int n) {
  switch (n) {
#define STC_VW(k) case k: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(k) : "memory"); return;
#define STC_VW8(k) STC_VW(k) STC_VW(k + 1) STC_VW(k + 2) STC_VW(k + 3) STC_VW(k + 4) STC_VW(k + 5) STC_VW(k + 6) STC_VW(k + 7)
    STC_VW8(0) STC_VW8(8) STC_VW8(16) STC_VW8(24) STC_VW8(32) STC_VW8(40) STC_VW8(48) STC_VW8(56)
#undef STC_VW8
#undef STC_VW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); return;
  }
}

template <int CIN, int NB, int NS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) narrow_stream_kernel(const HParams p) {
  constexpr int PXB = CIN * 2;                       // bytes per staged pixel
  constexpr int CH = CIN / 8;                        // 16-byte chunks per pixel
  constexpr int SH = CIN == 64 ? 1 : 0;              // swizzle: chunk ^ ((pixel >> SH) & (CH - 1))
  constexpr int RPX = NS_TW + 2;                     // staged pixels per row
  constexpr int PIECES = (RPX * PXB + 1023) / 1024;  // 1 KiB DMA pieces per row
  constexpr int SLOT = PIECES * 1024;
  constexpr int KK = CIN / 32;                       // MFMA K-steps per pixel
  constexpr int PD = NS - 1;                         // rows of DMA ahead
  constexpr int NROW = NS_SR + 2;                    // input rows per strip
  constexpr int PWMAX = (PIECES + 3) / 4;
  static_assert((PD - 1) * PWMAX + PD * 4 * NB <= 63, "narrow stream: vmcnt range");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int strips = p.GH / NS_SR, cols = p.GW / NS_TW;
  int bid = blockIdx.x;
  const int cb = bid % cols;
  bid /= cols;
  const int strip = bid % strips, img = bid / strips;
  const int y0 = strip * NS_SR, x0 = cb * NS_TW;
  const int pw = (PIECES - wave + 3) / 4;  // this wave's DMA pieces per row
  char* stg = smem + NS * SLOT + wave * 2048;  // the wave's output staging (smode 1 / 2)
  const int spr = STC_EXP_NOEPI ? 0 : (p.smode == 0 ? 4 * NB : 1);  // store instructions per output row

  // B fragments (K-step k = 64-channel chunk * 2 + half, neighbour nb = (dy+1)*3 + (dx+1), column block j)
  const uint4* frag = reinterpret_cast<const uint4*>(p.frag);
  bf16x8_h bfr[KK][9][NB];
#pragma unroll
  for (int k = 0; k < KK; ++k)
#pragma unroll
    for (int nb = 0; nb < 9; ++nb)
#pragma unroll
      for (int j = 0; j < NB; ++j) bfr[k][nb][j] = __builtin_bit_cast(bf16x8_h, frag[((k * 9 + nb) * NB + j) * 64 + lane]);
  // this lane's output column n' = 16 j + (lane & 15) -> (phase, channel), and its bias
  int ph[NB], nn[NB];
  float bz[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int np = 16 * j + (lane & 15);
    ph[j] = np / p.N;
    nn[j] = np - ph[j] * p.N;
    bz[j] = (p.bias && np < p.NP) ? p.bias[nn[j]] : 0.f;
  }

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.a, (short)0, (int)p.a_bytes, 0x00020000);
  const unsigned OOBV = 0x80000000u;
  auto issue = [&](int t) {  // input row y0 - 1 + t -> slot t % NS
    const int iy = y0 - 1 + t;
    const bool rok = (unsigned)iy < (unsigned)p.IH;
    char* dst = smem + (t % NS) * SLOT;
#pragma unroll
    for (int k = 0; k < PWMAX; ++k) {
      const int pc = wave + 4 * k;
      if (pc >= PIECES) break;
      const int o = pc * 1024 + lane * 16;
      const int pix = o / PXB, s = (o % PXB) >> 4;
      const int c = s ^ ((pix >> SH) & (CH - 1));
      const int ix = x0 - 1 + pix;
      const bool ok = rok && pix < RPX && (unsigned)ix < (unsigned)p.IW;
      const unsigned off = (((unsigned)(img * p.a_bs + iy * p.a_rs + ix * p.a_ps + p.a_co + 8 * c)) * 2u) |
                           (ok ? 0u : OOBV);
      hdma16(ra, dst + pc * 1024, ok ? off : OOBV);
    }
  };

  floatx4 acc[3][NB];
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[q][j] = floatx4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < PD; ++t) issue(t);

  const int rl = lane & 15, cq = lane >> 4;
  auto step = [&](int t, auto tm3) {
    constexpr int T3 = decltype(tm3)::value;  // t % 3
    // VMEM ops this wave issued after row t's DMA: rows t+1 .. t+PD-1 (those that exist) and the stores of the
    // iterations from row t's issue on (iterations >= 2 store)
    const int nrows = min(PD - 1, NROW - 1 - t);
    const int s0 = t < PD ? 0 : t - PD;
    const int nst = max(0, t - max(2, s0));
    vm_wait_dyn(nrows * pw + nst * spr);
    __builtin_amdgcn_s_barrier();
    if (t + PD < NROW) issue(t + PD);  // into the slot of row t - 1, which every wave finished before the barrier
    // row t: output rows q = t - 1 - dy (dy = -1, 0, 1) -> register tiles (t - 1 - dy) % 3
    constexpr int QA = T3, QB = (T3 + 2) % 3, QC = (T3 + 1) % 3;  // dy = -1, 0, +1
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[QA][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const char* row = smem + (t % NS) * SLOT;
#pragma unroll
    for (int k = 0; k < KK; ++k) {
      const int c = 4 * k + cq;
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int pix = 16 * wave + rl + dx;
        const bf16x8_h a = *reinterpret_cast<const bf16x8_h*>(row + pix * PXB + ((c ^ ((pix >> SH) & (CH - 1))) << 4));
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          acc[QA][j] = exp_mfma(a, bfr[k][0 * 3 + dx][j], acc[QA][j]);
          acc[QB][j] = exp_mfma(a, bfr[k][1 * 3 + dx][j], acc[QB][j]);
          acc[QC][j] = exp_mfma(a, bfr[k][2 * 3 + dx][j], acc[QC][j]);
        }
      }
    }
    // output row q = t - 2 is complete: acc[QC][j][e] = grid point (y0 + q, x0 + 16 wave + 4 cq + e), column n'
    if (!STC_EXP_NOEPI && t >= 2) {
      const int gy = y0 + t - 2;
      if (p.smode == 0) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const bool on = 16 * j + rl < p.NP;
          const int oy = 2 * gy + (ph[j] >> 1);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int gx = x0 + 16 * wave + 4 * cq + e;
            float v = acc[QC][j][e] + bz[j];
            if (p.tanh_) v = tanhf(v);
            const long long off = (long long)img * p.c_bs + (long long)oy * p.c_rs +
                                  (long long)(2 * gx + (ph[j] & 1)) * p.c_ps + (long long)(p.c_co + nn[j]) * p.c_cs;
            if (on) store_out(p, off, v);
          }
        }
      } else {
        // the wave's 2 x 32 output pixels x N channels through its LDS staging area, then one 16-byte store per
        // lane: smode 1 = [row][pixel][N] (a pixel's N channels are 16 bytes), smode 2 = [n][row][pixel] fp32
        const int esz = p.out_f32 ? 4 : 2;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          if (16 * j + rl >= p.NP) continue;
          const int row = ph[j] >> 1;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int px = 2 * (4 * cq + e) + (ph[j] & 1);
            float v = acc[QC][j][e] + bz[j];
            if (p.tanh_) v = tanhf(v);
            const int o = p.smode == 1 ? ((row * 32 + px) * p.N + nn[j]) * esz : ((nn[j] * 2 + row) * 32 + px) * 4;
            if (p.out_f32) *reinterpret_cast<float*>(stg + o) = v;
            else *reinterpret_cast<unsigned short*>(stg + o) = (unsigned short)(pack_bf16x2(v, 0.f) & 0xffffu);
          }
        }
        __builtin_amdgcn_wave_barrier();
        const int ox0 = 2 * (x0 + 16 * wave);
        if (p.smode == 1) {  // lane = (row, pixel)
          const int row = lane >> 5, px = lane & 31;
          const uint4 v = *reinterpret_cast<const uint4*>(stg + (row * 32 + px) * 16);
          const long long off = (long long)img * p.c_bs + (long long)(2 * gy + row) * p.c_rs +
                                (long long)(ox0 + px) * p.c_ps + p.c_co;
          *reinterpret_cast<uint4*>(p.c + off * esz) = v;
        } else if (lane < 16 * p.N) {  // lane = (n, row, 4-pixel quad)
          const int n = lane >> 4, row = (lane >> 3) & 1, qd = lane & 7;
          const uint4 v = *reinterpret_cast<const uint4*>(stg + ((n * 2 + row) * 32 + 4 * qd) * 4);
          const long long off = (long long)img * p.c_bs + (long long)(2 * gy + row) * p.c_rs + (ox0 + 4 * qd) +
                                (long long)(p.c_co + n) * p.c_cs;
          *reinterpret_cast<uint4*>(p.c + off * 4) = v;
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
  };
  // NROW = 18 = 6 x 3 iterations, unrolled by 3 so the register tiles rotate at compile time
  static_assert(NROW % 3 == 0, "narrow stream: strip rows + 2 must be a multiple of 3");
  for (int t = 0; t < NROW; t += 3) {
    step(t, std::integral_constant<int, 0>{});
    step(t + 1, std::integral_constant<int, 1>{});
    step(t + 2, std::integral_constant<int, 2>{});
  }
}

// ---- the PatchGAN logits layer (Conv2d k4 s1 p1, CIN -> 1; STCGAN/networks.py:183-184) in two passes: the 16 tap
// products of every input pixel, Y[q][tap] = sum_c x[q][c] w[tap][c] (an M = pixels, N = 16 taps, K = CIN GEMM on
// v_mfma_f32_16x16x32_bf16 with the A fragments loaded straight from HBM -- each input byte read once, no halo), then
// out[y][x] = bias + sum_taps Y[(y + ky - 1, x + kx - 1)][tap] (fixed tap order; out-of-image pixels contribute 0).
// The tiled kernel re-read the 4x16 tiles' halo (1.7x) and split the 8192-deep reduction over blocks.
template <int CIN>
__global__ void __launch_bounds__(256) logits_taps_kernel(const HParams p, float* __restrict__ Y) {
  constexpr int KS = CIN / 32;
  const int lane = threadIdx.x & 63;
  const long long Q = (long long)p.Mtot;                     // input pixels (B * IH * IW)
  const long long q0 = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
  if (q0 >= Q) return;
  const int rl = lane & 15, kq = lane >> 4;
  // B: tap rl, channels 32 k + 8 kq .. + 7
  bf16x8_h bw[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) bw[k] = *reinterpret_cast<const bf16x8_h*>(p.w + rl * CIN + 32 * k + 8 * kq);
  // A: pixel q0 + rl (clamped past the end), the same channels
  const long long q = min(q0 + rl, Q - 1);
  const int ihw = p.IH * p.IW;
  const int b = (int)(q / ihw), rem = (int)(q - (long long)b * ihw), iy = rem / p.IW, ix = rem - iy * p.IW;
  const bf16* xp = reinterpret_cast<const bf16*>(p.a) + (long long)b * p.a_bs + (long long)iy * p.a_rs +
                   (long long)ix * p.a_ps + p.a_co + 8 * kq;
  bf16x8_h av[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) av[k] = *reinterpret_cast<const bf16x8_h*>(xp + 32 * k);
  floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < KS; ++k) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[k], bw[k], acc, 0, 0, 0);
  // acc[e] = Y[q0 + 4 kq + e][tap rl]
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long long qq = q0 + 4 * kq + e;
    if (qq < Q) Y[qq * 16 + rl] = acc[e];
  }
}

// 4 lanes per output pixel (one kernel row each: its 4 taps' loads in flight together), summed in a fixed order
__global__ void __launch_bounds__(256) logits_gather_kernel(const HParams p, const float* __restrict__ Y) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long idx = t >> 2;
  const int ky = (int)(t & 3);
  const long long total = (long long)(p.Mtot / ((long long)p.IH * p.IW)) * p.GH * p.GW;
  const long long ic = idx < total ? idx : total - 1;
  const int ghw = p.GH * p.GW;
  const int b = (int)(ic / ghw), rem = (int)(ic - (long long)b * ghw), gy = rem / p.GW, gx = rem - gy * p.GW;
  const float* yb = Y + (long long)b * p.IH * p.IW * 16;
  const int iy = gy + ky - 1;
  float tv[4];
#pragma unroll
  for (int kx = 0; kx < 4; ++kx) {
    const int ix = gx + kx - 1;
    const bool ok = (unsigned)iy < (unsigned)p.IH && (unsigned)ix < (unsigned)p.IW;
    tv[kx] = ok ? yb[((long long)iy * p.IW + ix) * 16 + ky * 4 + kx] : 0.f;
  }
  float v = (tv[0] + tv[1]) + (tv[2] + tv[3]);
  v += __shfl_xor(v, 1, 64);  // (rows 0 + 1, 2 + 3), then the two pairs: the same order on every lane
  v += __shfl_xor(v, 2, 64);
  if (ky != 0 || idx >= total) return;
  if (p.bias) v += p.bias[0];
  if (p.tanh_) v = tanhf(v);
  store_out(p, (long long)b * p.c_bs + (long long)gy * p.c_rs + (long long)gx * p.c_ps + (long long)p.c_co * p.c_cs, v);
}

// split-K combine: out = epi(sum_s ws[s][m][n'])
template <int GEOM>
__global__ void narrow_reduce_kernel(const HParams p, int B) {
  const long long total = p.Mtot * p.NP;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int np = (int)(idx % p.NP);
    const long long m = idx / p.NP;
    float v = 0.f;
    for (int s = 0; s < p.nsplit; ++s) v += p.ws[(long long)s * total + idx];
    int ph = 0, n = np;
    if (GEOM == 0) { ph = np / p.N; n = np - ph * p.N; }
    if (p.bias) v += p.bias[n];
    if (p.tanh_) v = tanhf(v);
    const int img = (int)(m / ((long long)p.GH * p.GW));
    const int rem = (int)(m - (long long)img * p.GH * p.GW);
    const int gy = rem / p.GW, gx = rem - gy * p.GW;
    const int oy = GEOM == 0 ? 2 * gy + (ph >> 1) : gy;
    const int ox = GEOM == 0 ? 2 * gx + (ph & 1) : gx;
    store_out(p, (long long)img * p.c_bs + (long long)oy * p.c_rs + (long long)ox * p.c_ps +
                     (long long)(p.c_co + n) * p.c_cs, v);
  }
}

// ------------------------------------------------------------------------- host
static size_t halo_lds(int geom, int ty, int txb, int nstage) {
  const int halo = geom == 0 ? 2 : 3;
  const int npix = (ty + halo) * (16 * txb + halo);
  return (size_t)nstage * (size_t)((npix + 7) / 8) * 1024;
}

// K-split kernel LDS: all of the block's chunk images, or the partials + staged output tile if larger
static size_t wk_lds(int geom, int ty, int txb, int n_out, int nch) {
  const int halo = geom == 0 ? 2 : 3;
  const size_t img = (size_t)(((ty + halo) * (16 * txb + halo) + 7) / 8) * 1024;
  const int sc = geom == 0 ? 2 : 1;
  const size_t red = (size_t)4 * ty * txb * 1024;                         // every wave's partials
  const size_t stage = (size_t)(sc * ty) * (sc * 16 * txb) * n_out * 4;  // the output tile, fp32
  return std::max(img * (size_t)nch, red + stage);
}

// the streaming ConvT kernel's shapes: CIN 128 with N' <= 16 (the generator output layer) or CIN 64 with
// 16 < N' <= 32 (the N = 8 first-layer input gradients); whole strips and 64-column blocks
static bool narrow_stream_ok(int geom, int cin, int np_cols, int GH, int GW) {
  return geom == 0 && GH % NS_SR == 0 && GW % NS_TW == 0 &&
         ((cin == 128 && np_cols <= 16) || (cin == 64 && np_cols > 16 && np_cols <= 32));
}

// ring slots: 3 (CIN 128) / 4 (CIN 64), two blocks per CU (VGPR-bound); force {NS, 32} picks another depth (tuning).
// Measured (scripts/ab_narrow.py, bs=32 128^2 grids): 128 -> 1|3 37.7-38.2 us at NS 3, 40 us at 4, ~60 us at 6 / 8
// (one block per CU); 64 -> 8 32.4 us at 4, 35.4 at 6; the tiled K-split kernel 44.8 / 46.2 / 34.6 us.
static int stream_ns(int cin, const int32_t* force) {
  if (force && (force[1] & 32) && force[0] > 0) return force[0];
  return cin == 128 ? 3 : 4;
}

// the two-pass logits form: conv s1 with one output channel and 512 / 256 input channels
static bool logits_ok(int geom, int cin, int cout) { return geom == 1 && cout == 1 && (cin == 512 || cin == 256); }

static size_t stream_lds(int cin, int ns) {
  const int pieces = ((NS_TW + 2) * cin * 2 + 1023) / 1024;
  return (size_t)ns * pieces * 1024 + 4 * 2048;  // + the waves' output staging
}

// store mode of the streaming kernel's output (HParams::smode): 16-byte NHWC pixels (N x element = 16 B, 16-byte
// aligned views), NCHW fp32 rows (unit pixel stride, 16-byte aligned rows and planes), else scalar stores
static int stream_smode(const stc_view& y, int N, int out_f32) {
  const int esz = out_f32 ? 4 : 2;
  const int a = 16 / esz;  // elements per 16 bytes
  if (y.cs == 1 && N * esz == 16 && y.ps % a == 0 && y.co % a == 0 && y.rs % a == 0 && y.bs % a == 0) return 1;
  if (out_f32 && y.ps == 1 && N <= 4 && y.rs % 4 == 0 && y.cs % 4 == 0 && y.bs % 4 == 0 && (y.co * y.cs) % 4 == 0)
    return 2;
  return 0;
}

// Narrow plan: {ty, txb, nsplit, kernel}.  Kernel 2 (default where it applies): narrow_stream_kernel (force
// {0, 32} selects it explicitly; any other forced tile takes the tiled kernels).  Taller / wider tiles reuse each register-held B fragment over
// more MFMAs; the split over channel chunks keeps >= 1024 blocks on the long reductions.  Kernel 1 (default):
// narrow_wk_kernel, whose block stages all its chunks at once -- the split also keeps that under 56 KiB
// (3 blocks per CU).  force = {ty, txb (+16: the row-split narrow_halo_kernel)}.
static void narrow_plan(int geom, int B, int GH, int GW, int cin, int np_cols, const int32_t* force, int* ty,
                        int* txb, int* nsplit, int* kern, bool allow_stream = true) {
  // K-split kernel: 4 x 16 tiles (scripts/narrow_sweep.py, round 3: G output ConvT 128->1|3 41.6|43.7 us,
  // N = 8 input gradient 33.6 us, logits 21.1 us vs 60.7|60.3, 60.4, 24.7 us for the best row-split tiles)
  *ty = 4;
  *txb = 1;
  *kern = 1;
  if (allow_stream && narrow_stream_ok(geom, cin, np_cols, GH, GW) && (!force || (force[0] == 0 && force[1] == 0) || (force[1] & 32))) {
    *kern = 2;  // the streaming ConvT kernel: one strip per block, no split
    *nsplit = 1;
    return;
  }
  if (force && force[0] > 0) {
    *ty = force[0];
    *txb = (force[1] & 15) > 0 ? (force[1] & 15) : 1;
    if (force[1] & 16) *kern = 0;
  } else if (force && (force[1] & 16)) {  // the row-split kernel at its own default tile
    *kern = 0;
    *ty = 8;
    *txb = geom == 0 && np_cols > 16 ? 2 : 1;  // two column blocks per B fragment: -11 % on the N = 8 ConvT
  }
  const int nchunks = cin / 64;
  const int n_out = geom == 0 ? np_cols / 4 : np_cols;
  const long long blocks = (long long)B * cdiv(GH, *ty) * cdiv(GW, 16 * *txb);
  int ns = 1;
  while (blocks * ns < 1024 && ns * 2 <= nchunks) ns *= 2;
  if (*kern == 1)
    while (wk_lds(geom, *ty, *txb, n_out, cdiv(nchunks, ns)) > 56 * 1024 && ns * 2 <= nchunks) ns *= 2;
  *nsplit = ns;
}

// bytes of the B fragment table: chunks x 2 halves x neighbours x column blocks x 1 KiB (256-aligned)
static int64_t narrow_frag_bytes(int geom, int Cin, int Cout) {
  const int nbr = geom == 0 ? 9 : 16;
  const int np = geom == 0 ? 4 * Cout : Cout;
  const int nb = np <= 16 ? 1 : 2;
  return (int64_t)(Cin / 64) * 2 * nbr * nb * 1024;
}

bool bf16_narrow_eligible(int kind, int Cin, int Cout) {
  if (kind != STC_CONVT_S2 && kind != STC_CONV_S1) return false;
  if (Cin % 64 != 0) return false;
  return kind == STC_CONVT_S2 ? Cout <= 8 : Cout <= 16;
}

int64_t bf16_narrow_workspace(int kind, int B, int GH, int GW, int Cin, int Cout) {
  const int geom = kind == STC_CONVT_S2 ? 0 : 1;
  int ty, txb, ns, kern;
  const int np = geom == 0 ? 4 * Cout : Cout;
  narrow_plan(geom, B, GH, GW, Cin, np, nullptr, &ty, &txb, &ns, &kern, false);  // (a forced tiled plan's slab)
  const int64_t taps = logits_ok(geom, Cin, Cout) ? (int64_t)B * (GH + 1) * (GW + 1) * 16 * 4 : 0;  // (conv s1: IH = GH+1)
  return std::max<int64_t>((ns <= 1 ? 0 : (int64_t)ns * B * GH * GW * np * 4) + narrow_frag_bytes(geom, Cin, Cout), taps);
}

int bf16_narrow_fwd(int kind, int B, stc_view x, int Cin, const void* w_packed, int Cout, stc_view y,
                    const float* bias, int epi_tanh, int out_f32, void* ws, int64_t ws_bytes, hipStream_t st,
                    const int32_t* force) {
  const int geom = kind == STC_CONVT_S2 ? 0 : 1;
  HParams p{};
  p.a = (const char*)x.p;
  const long long a_bytes = (long long)B * x.bs * 2;
  STC_REQUIRE(a_bytes < (1ll << 31) && x.cs == 1 && x.ps % 8 == 0 && x.co % 8 == 0,
              "narrow bf16: input view must be NHWC, 16-byte aligned, < 2 GiB");
  p.a_bytes = (unsigned)a_bytes;
  p.a_bs = (int)x.bs; p.a_rs = (int)x.rs; p.a_ps = x.ps; p.a_co = x.co;
  p.IH = x.H; p.IW = x.W; p.cin = Cin;
  if (geom == 0) { p.GH = x.H; p.GW = x.W; }
  else { p.GH = y.H; p.GW = y.W; }
  p.N = Cout;
  p.NP = geom == 0 ? 4 * Cout : Cout;
  p.w = (const bf16*)w_packed;
  p.w_phase_stride = Cout * (geom == 0 ? 4 : 16) * Cin;
  p.c = (char*)y.p; p.c_bs = y.bs; p.c_rs = y.rs; p.c_ps = y.ps; p.c_co = y.co; p.c_cs = y.cs;
  p.bias = bias; p.tanh_ = epi_tanh; p.out_f32 = out_f32;
  p.Mtot = (long long)B * p.GH * p.GW;
  int ty, txb, ns, kern;
  narrow_plan(geom, B, p.GH, p.GW, Cin, p.NP, force, &ty, &txb, &ns, &kern);
  p.tiles_x = cdiv(p.GW, 16 * txb);
  p.tiles_per_img = p.tiles_x * cdiv(p.GH, ty);
  const int nchunks = Cin / 64;
  p.chunks_per_split = cdiv(nchunks, ns);
  p.nsplit = cdiv(nchunks, p.chunks_per_split);
  if (logits_ok(geom, Cin, Cout) && !(force && (force[0] > 0 || force[1] != 0))) {
    STC_REQUIRE(x.H == p.GH + 1 && x.W == p.GW + 1, "narrow bf16: logits geometry (%dx%d -> %dx%d)", x.H, x.W, p.GH, p.GW);
    const int64_t need = (int64_t)B * x.H * x.W * 16 * 4;
    STC_REQUIRE(ws && ws_bytes >= need, "narrow bf16: workspace %lld < %lld", (long long)ws_bytes, (long long)need);
    p.Mtot = (long long)B * x.H * x.W;  // (here: input pixels)
    if (p.Mtot == 0 || (long long)B * p.GH * p.GW == 0) return 0;
    float* Y = (float*)ws;
    const unsigned g1 = (unsigned)((p.Mtot + 63) / 64), g2 = (unsigned)((4LL * B * p.GH * p.GW + 255) / 256);
    main_timer_begin(st);
    if (Cin == 512) hipLaunchKernelGGL(logits_taps_kernel<512>, dim3(g1), dim3(256), 0, st, p, Y);
    else hipLaunchKernelGGL(logits_taps_kernel<256>, dim3(g1), dim3(256), 0, st, p, Y);
    main_timer_end(st);
    STC_CHECK_LAUNCH();
    hipLaunchKernelGGL(logits_gather_kernel, dim3(g2), dim3(256), 0, st, p, (const float*)Y);
    STC_CHECK_LAUNCH();
    return 0;
  }
  const int64_t slab_bytes = p.nsplit > 1 ? (int64_t)p.nsplit * B * p.GH * p.GW * p.NP * 4 : 0;
  const int64_t frag_bytes = narrow_frag_bytes(geom, Cin, Cout);
  STC_REQUIRE(ws && ws_bytes >= slab_bytes + frag_bytes, "narrow bf16: workspace %lld < %lld", (long long)ws_bytes,
              (long long)(slab_bytes + frag_bytes));
  if (p.nsplit > 1) p.ws = (float*)ws;
  p.frag = (const char*)ws + slab_bytes;
  if ((long long)B * p.GH * p.GW == 0) return 0;
  {
    const int nbr = geom == 0 ? 9 : 16, nb = p.NP <= 16 ? 1 : 2;
    const unsigned nfrag = (unsigned)((Cin / 64) * 2 * nbr * nb);
    if (geom == 0) {
      if (nb == 1) hipLaunchKernelGGL((narrow_bfrag_kernel<0, 1>), dim3(nfrag), dim3(64), 0, st, p, (uint4*)p.frag);
      else hipLaunchKernelGGL((narrow_bfrag_kernel<0, 2>), dim3(nfrag), dim3(64), 0, st, p, (uint4*)p.frag);
    } else {
      hipLaunchKernelGGL((narrow_bfrag_kernel<1, 1>), dim3(nfrag), dim3(64), 0, st, p, (uint4*)p.frag);
    }
    STC_CHECK_LAUNCH();
  }
  if (kern == 2) {
    STC_REQUIRE(p.nsplit == 1 && narrow_stream_ok(geom, Cin, p.NP, p.GH, p.GW), "narrow bf16: stream plan");
    const dim3 sgrid((unsigned)(B * (p.GH / NS_SR) * (p.GW / NS_TW)));
    p.smode = stream_smode(y, Cout, out_f32);
    STC_REQUIRE(p.smode == 0 || ((uintptr_t)y.p & 15) == 0, "narrow bf16: unaligned output");
    const int nsl = stream_ns(Cin, force);
    const size_t slds = stream_lds(Cin, nsl);
    main_timer_begin(st);
#define STC_NS(C_, NB_, S_) \
  else if (Cin == C_ && nsl == S_) hipLaunchKernelGGL((narrow_stream_kernel<C_, NB_, S_>), sgrid, dim3(256), slds, st, p)
    if (false) {}
    STC_NS(128, 1, 4); STC_NS(128, 1, 3); STC_NS(128, 1, 6); STC_NS(128, 1, 8);
    STC_NS(64, 2, 6); STC_NS(64, 2, 4);
    else return fail(-1, "narrow bf16: no stream kernel with %d slots", nsl);
#undef STC_NS
    main_timer_end(st);
    STC_CHECK_LAUNCH();
    return 0;
  }
  dim3 grid((unsigned)(B * p.tiles_per_img), (unsigned)p.nsplit);
  const size_t lds = kern == 1 ? wk_lds(geom, ty, txb, Cout, p.chunks_per_split)
                               : halo_lds(geom, ty, txb, p.chunks_per_split > 1 ? 2 : 1);
  STC_REQUIRE(lds <= 160 * 1024, "narrow bf16: tile %dx%d needs %zu B of LDS", ty, 16 * txb, lds);
  main_timer_begin(st);
  if (kern == 1) {
#define STC_NW(G_, NB_, TY_, TXB_) hipLaunchKernelGGL((narrow_wk_kernel<G_, NB_, TY_, TXB_>), grid, dim3(256), lds, st, p)
#define STC_NW_T(G_, NB_)                                                                  \
  if (ty == 8 && txb == 1) STC_NW(G_, NB_, 8, 1);                                          \
  else if (ty == 8 && txb == 2) STC_NW(G_, NB_, 8, 2);                                     \
  else if (ty == 16 && txb == 1) STC_NW(G_, NB_, 16, 1);                                   \
  else if (ty == 4 && txb == 1) STC_NW(G_, NB_, 4, 1);                                     \
  else if (ty == 4 && txb == 2) STC_NW(G_, NB_, 4, 2);                                     \
  else return fail(-1, "narrow bf16: no kernel for a %dx%d tile", ty, 16 * txb);
    if (geom == 0) {
      if (p.NP <= 16) { STC_NW_T(0, 1) }
      else { STC_NW_T(0, 2) }
    } else {
      STC_NW_T(1, 1)
    }
#undef STC_NW_T
#undef STC_NW
  } else {
#define STC_NH(G_, NB_, TY_, TXB_) hipLaunchKernelGGL((narrow_halo_kernel<G_, NB_, TY_, TXB_>), grid, dim3(256), lds, st, p)
#define STC_NH_T(G_, NB_)                                                                  \
  if (ty == 8 && txb == 1) STC_NH(G_, NB_, 8, 1);                                          \
  else if (ty == 8 && txb == 2) STC_NH(G_, NB_, 8, 2);                                     \
  else if (ty == 16 && txb == 1) STC_NH(G_, NB_, 16, 1);                                   \
  else if (ty == 16 && txb == 2) STC_NH(G_, NB_, 16, 2);                                   \
  else if (ty == 32 && txb == 1) STC_NH(G_, NB_, 32, 1);                                   \
  else return fail(-1, "narrow bf16: no kernel for a %dx%d tile", ty, 16 * txb);
    if (geom == 0) {
      if (p.NP <= 16) { STC_NH_T(0, 1) }
      else { STC_NH_T(0, 2) }
    } else {
      STC_NH_T(1, 1)
    }
#undef STC_NH_T
#undef STC_NH
  }
  main_timer_end(st);
  STC_CHECK_LAUNCH();
  if (p.nsplit > 1) {
    const long long total = (long long)B * p.GH * p.GW * p.NP;
    const int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
    if (geom == 0) hipLaunchKernelGGL(narrow_reduce_kernel<0>, dim3(blocks), dim3(256), 0, st, p, B);
    else hipLaunchKernelGGL(narrow_reduce_kernel<1>, dim3(blocks), dim3(256), 0, st, p, B);
    STC_CHECK_LAUNCH();
  }
  return 0;
}

}  // namespace stc
