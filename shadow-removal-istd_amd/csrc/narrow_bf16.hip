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
};

typedef __bf16 bf16x8_h __attribute__((ext_vector_type(8)));
using lds_vptr_h = __attribute__((address_space(3))) void*;

__device__ __forceinline__ void hdma16(__amdgpu_buffer_rsrc_t r, char* lds_dst, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_vptr_h)lds_dst, 16, voff, 0, 0, 0);
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

// Narrow plan: {ty, txb, nsplit}.  Taller / wider tiles reuse each register-held B fragment over more
// MFMAs; the split over channel chunks keeps >= 1024 blocks on the long reductions.
static void narrow_plan(int geom, int B, int GH, int GW, int cin, int np_cols, const int32_t* force, int* ty,
                        int* txb, int* nsplit) {
  *ty = 8;
  *txb = geom == 0 && np_cols > 16 ? 2 : 1;  // two column blocks per B fragment: -11 % on the N = 8 ConvT
  if (force && force[0] > 0) {
    *ty = force[0];
    *txb = force[1] > 0 ? force[1] : 1;
  }
  const int nchunks = cin / 64;
  const long long blocks = (long long)B * cdiv(GH, *ty) * cdiv(GW, 16 * *txb);
  int ns = 1;
  while (blocks * ns < 1024 && ns * 2 <= nchunks) ns *= 2;
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
  int ty, txb, ns;
  const int np = geom == 0 ? 4 * Cout : Cout;
  narrow_plan(geom, B, GH, GW, Cin, np, nullptr, &ty, &txb, &ns);
  return (ns <= 1 ? 0 : (int64_t)ns * B * GH * GW * np * 4) + narrow_frag_bytes(geom, Cin, Cout);
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
  int ty, txb, ns;
  narrow_plan(geom, B, p.GH, p.GW, Cin, p.NP, force, &ty, &txb, &ns);
  p.tiles_x = cdiv(p.GW, 16 * txb);
  p.tiles_per_img = p.tiles_x * cdiv(p.GH, ty);
  const int nchunks = Cin / 64;
  p.chunks_per_split = cdiv(nchunks, ns);
  p.nsplit = cdiv(nchunks, p.chunks_per_split);
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
  dim3 grid((unsigned)(B * p.tiles_per_img), (unsigned)p.nsplit);
  const size_t lds = halo_lds(geom, ty, txb, p.chunks_per_split > 1 ? 2 : 1);
  STC_REQUIRE(lds <= 160 * 1024, "narrow bf16: tile %dx%d needs %zu B of LDS", ty, 16 * txb, lds);
  main_timer_begin(st);
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
