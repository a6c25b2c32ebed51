// bf16 Conv2d k4 s2 p1 with 8 (padded) input channels: the K = 128 layers at the full-resolution edge of the
// generator and the discriminators, which are HBM-bound (their MFMA work is a few % of the time it takes to read the
// 16-byte input pixels once and write the output pixels once).
//   * forward of G's outermost down conv and D's first conv (STCGAN/networks.py:99, :165-166; 64 outputs, no
//     BatchNorm): the activation epilogue -- act(s1) [and act(s2)] of the bf16-rounded output, exactly as
//     stc_bn_apply with no table (MODE 1 / 2);
//   * the input gradient of G's output ConvTranspose2d (networks.py:112-116; dq, 8 channels -> the 128-channel
//     concat gradient) with the BatchNorm-backward sums of the up-path BN on its second half fused in (MODE 3, the
//     stc_conv_bwd_bn contract of igemm_bf16.hpp's BNB epilogue; one partial per block).
// The im2col GEMM tile re-stages every input pixel 4 times per 128-row tile and pays a load latency per tile; here a
// block owns a strip of 8 output rows of one image and streams its input rows through an 8-slot LDS ring by LDS-DMA
// (an input row = W x 16 B; output row oy reads input rows 2oy-1 .. 2oy+2, so each output row brings 2 new input
// rows), two output rows of loads ahead of the MFMAs.  Padding rows are out-of-range DMA offsets (zeros); the
// padding columns are zeroed in registers.
// MFMA v_mfma_f32_16x16x32_bf16, K-step = kernel row ky: a lane's 8 K values (tap (ky, kx = lane >> 4), 8 channels)
// are one input pixel, one ds_read_b128 (conflict-free: the 16 lanes of a group read 16 distinct pixels mod 16); the
// N x 128 weights live in registers.  A wave computes 16 output pixels x N channels per chunk and writes 16-byte NHWC
// rows through a per-wave LDS transpose.  Results equal the im2col tile's bit for bit (same K order, same MFMA).
#include <algorithm>

#include "igemm_bf16.hpp"

namespace stc {

// output rows per block: 8 for the activation modes, 16 for the BN-backward modes (scripts/ab_stem.py, bs = 32,
// profiles/r04/stem/strip_*.log: activation 25.8 / 29.9 us at 8 against 26.2 / 30.9 at 4 and 31.9 / 33.7 at 16; the
// output layer's input gradient + BN apply 113.1 us at 16 against 118.3 at 8, the logits layer's 45.8 against 51.7)
constexpr int STEM_RB = 8;
constexpr int STEM_RB_BNB = 16;
constexpr int S1D_RB = 16;
constexpr int STEM_NS = 8;   // input-row slots in the LDS ring

template <int WIN, int N, int MODE>
__global__ void __launch_bounds__(256) stem_conv_kernel(const GParams p) {
  constexpr int RB = MODE == 3 ? STEM_RB_BNB : STEM_RB;
  constexpr int WOUT = WIN / 2;
  constexpr int ROWB = WIN * 16;              // bytes of one input row (8 bf16 channels per pixel)
  constexpr int PPW = WIN / 256;              // 1 KiB DMA pieces per wave per input row
  constexpr int NCH = WOUT / 64;              // 64-pixel chunks per output row (16 per wave)
  constexpr int NF = N / 16;                  // MFMA N fragments
  constexpr int CPX = N / 8;                  // 16-byte chunks per output pixel
  constexpr int PXS = 64 / CPX;               // pixels per store pass of a wave
  constexpr int NPASS = 16 / PXS;             // store passes per chunk
  constexpr bool BNB = MODE == 3;
  // other VMEM ops per output row and wave: the stores, and (MODE 3) the BN input + second-gradient loads
  constexpr int OPW = NCH * NPASS * (MODE == 2 ? 2 : 1) + (BNB ? 2 * NCH * NPASS : 0);
  constexpr int PITCH = N * 2 + 16;           // output staging row (N bf16 + pad)
  static_assert(NPASS >= 1 && 4 * PPW <= 63 && 2 * PPW + 2 * OPW <= 63, "stem tile: vmcnt immediates");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  char* stg = smem + STEM_NS * ROWB + wave * 16 * PITCH;
  const int strips = p.GH / RB;
  const int img = blockIdx.x / strips, oy0 = (blockIdx.x - img * strips) * RB;
  const int rl = lane & 15, kq = lane >> 4;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.a, (short)0, (int)p.a_bytes, 0x00020000);
  // input row r (local: G row 2 oy0 - 1 + r) -> slot r % NS; piece w + 4 i of the row: pixels 64 (w + 4 i) + lane
  const int gy0 = 2 * oy0 - 1;
  auto load_row = [&](int r) {
    const int gy = gy0 + r;
    const bool ok = (unsigned)gy < (unsigned)p.IH;
    char* dst = ring + (r % STEM_NS) * ROWB;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave + 4 * i;
      const unsigned off = (unsigned)(img * p.a_bs + gy * p.a_rs + (64 * pc + lane) * p.a_ps + p.a_co);
      dma16(ra, dst + pc * 1024, ok ? off * 2u : OOB);
    }
  };

  // weights: B fragment (n-frag j, K-step ky) of lane (rl, kq) = w[16 j + rl][tap 4 ky + kq][0..7]
  bf16x8_t wf[NF][4];
#pragma unroll
  for (int j = 0; j < NF; ++j)
#pragma unroll
    for (int ky = 0; ky < 4; ++ky)
      wf[j][ky] = *reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const bf16*>(p.b) + (16 * j + rl) * 128 +
                                                     (4 * ky + kq) * 8);
  float bz[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) bz[j] = p.bias ? p.bias[16 * j + rl] : 0.f;
  const bf16x8_t zero8 = {};

  // store / BN-backward lane role: 16-byte chunk sc of pixels spx + PXS * h
  const int sc = lane % CPX, spx = lane / CPX;
  const int nb = sc * 8 - p.bch_off;  // BN channel of the chunk (MODE 3)
  const bool bn_lane = BNB && nb >= 0 && nb < p.bC;
  const int nbc = bn_lane ? nb : 0;
  float bsc[8], bsh[8], bmu[8], brs[8], sa[8], sb[8];
  if constexpr (BNB) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bsc[e] = p.bsc[nbc + e]; bsh[e] = p.bsh[nbc + e]; bmu[e] = p.bmu[nbc + e]; brs[e] = p.brs[nbc + e];
      sa[e] = 0.f; sb[e] = 0.f;
    }
  }

  // prologue: the 4 rows of output row 0 and the 2 new rows of output rows 1 and 2
#pragma unroll
  for (int r = 0; r < 8; ++r) load_row(r);
  for (int t = 0; t < RB; ++t) {
    // rows 2t .. 2t+3 must have landed; younger: this wave's other VMEM ops (stores, BN loads) of output rows t-2 and
    // t-1 and the loads of rows 2t+4 .. 2t+7 issued between them (t = 0: the loads of rows 4..7; t = 1: rows 6, 7
    // before the ops of row 0)
    if (t == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * PPW) : "memory");
    else if (t == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW + OPW) : "memory");
    else if (t + 1 < RB) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW + 2 * OPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * OPW) : "memory");
    __builtin_amdgcn_s_barrier();
    // refill rows 2t + 6, 2t + 7 into the slots of rows 2t - 2, 2t - 1, last read by output row t - 1, which every
    // wave finished before this barrier (the slots of rows 2t .. 2t + 3 are this row's)
    if (t >= 1 && 2 * t + 7 < 2 * RB + 2) {
      load_row(2 * t + 6);
      load_row(2 * t + 7);
    }
    const int oy = oy0 + t;
    const char* rows[4];
#pragma unroll
    for (int ky = 0; ky < 4; ++ky) rows[ky] = ring + ((2 * t + ky) % STEM_NS) * ROWB;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      // MODE 3: this chunk's BN inputs, loaded before the MFMAs
      uint4 bxv[NPASS], bgv[NPASS];
      if constexpr (BNB) {  // (the second gradient's loads always issue -- from the BN input when there is none --
                            // so that every wave's VMEM count per row is the compile-time OPW)
#pragma unroll
        for (int h = 0; h < NPASS; ++h) {
          const int oxs = ch * 64 + wave * 16 + spx + PXS * h;
          const bool in = oy < p.bxH && oxs < p.bxW;
          const int oyc = in ? oy : 0, oxc = in ? oxs : 0;
          const bf16* xq = reinterpret_cast<const bf16*>(p.bx) + (long long)img * p.bx_bs + (long long)oyc * p.bx_rs +
                           (long long)oxc * p.bx_ps + p.bx_co + nbc;
          const bf16* gq = p.bg ? reinterpret_cast<const bf16*>(p.bg) + (long long)img * p.bg_bs + (long long)oyc * p.bg_rs +
                                      (long long)oxc * p.bg_ps + p.bg_co + nbc
                                : xq;
          bxv[h] = *reinterpret_cast<const uint4*>(xq);
          bgv[h] = *reinterpret_cast<const uint4*>(gq);
        }
      }
      const int ox = ch * 64 + wave * 16 + rl;  // this lane's output pixel
      const int col = 2 * ox + kq - 1;          // input column of tap kx = kq
      const bool cok = (unsigned)col < (unsigned)WIN;
      floatx4 acc[NF];
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ky = 0; ky < 4; ++ky) {
        bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(rows[ky] + (cok ? col : 0) * 16);
        a = cok ? a : zero8;
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[j] = exp_mfma(a, wf[j][ky], acc[j]);
      }
      // acc[j][e] = out[pixel ch*64 + wave*16 + 4 kq + e][channel 16 j + rl]: + bias, bf16, staged [pixel][N]
#pragma unroll
      for (int j = 0; j < NF; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const unsigned u = pack_bf16x2(acc[j][e] + bz[j], 0.f) & 0xffffu;
          *reinterpret_cast<unsigned short*>(stg + (4 * kq + e) * PITCH + (16 * j + rl) * 2) = (unsigned short)u;
        }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int h = 0; h < NPASS; ++h) {
        const int px = spx + PXS * h;
        const uint4 tv = *reinterpret_cast<const uint4*>(stg + px * PITCH + sc * 16);
        const int oxs = ch * 64 + wave * 16 + px;
        const long long o1 = (long long)img * p.c_bs + (long long)oy * p.c_rs + (long long)oxs * p.c_ps + p.c_co + sc * 8;
        if constexpr (BNB) {
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.c) + o1) = tv;
          // {sum dn, sum dn * xhat} of the chunk's BN channels at this pixel (igemm_epilogue's BNB arithmetic)
          if (bn_lane && oy < p.bxH && oxs < p.bxW) {
            const unsigned wt[4] = {tv.x, tv.y, tv.z, tv.w};
            const unsigned wx[4] = {bxv[h].x, bxv[h].y, bxv[h].z, bxv[h].w};
            const unsigned wg[4] = {bgv[h].x, bgv[h].y, bgv[h].z, bgv[h].w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float v = __uint_as_float((e & 1) ? (wt[e >> 1] & 0xffff0000u) : (wt[e >> 1] << 16));
              const float xv = __uint_as_float((e & 1) ? (wx[e >> 1] & 0xffff0000u) : (wx[e >> 1] << 16));
              const float gv = __uint_as_float((e & 1) ? (wg[e >> 1] & 0xffff0000u) : (wg[e >> 1] << 16));
              const float nn = fmaf(xv, bsc[e], bsh[e]);
              float dn = v * (nn > 0.f ? 1.f : p.bs_self);
              if (p.bg) dn += gv * (nn > 0.f ? 1.f : p.bs_other);
              sa[e] += dn;
              sb[e] += dn * (xv - bmu[e]) * brs[e];
            }
          }
        } else {
#if STC_EXP_NOSTORE  // (diagnostic builds: the output stores compiled out -- what the stream of stores costs)
          if (tv.x == 0x12345678u) *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.c) + o1) = act_bf16x8(tv, p.act_s1);
          continue;
#endif
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.c) + o1) = act_bf16x8(tv, p.act_s1);
          if constexpr (MODE == 2) {
            const long long o2 = (long long)img * p.c2_bs + (long long)oy * p.c2_rs + (long long)oxs * p.c2_ps + p.c2_co +
                                 sc * 8;
            *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.c2) + o2) = act_bf16x8(tv, p.act_s2);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  if constexpr (BNB) {
    // the block's partial: threads sharing a chunk summed in thread order (fixed), through the ring's LDS
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [256][16]
#pragma unroll
    for (int e = 0; e < 8; ++e) { red[tid * 16 + e] = sa[e]; red[tid * 16 + 8 + e] = sb[e]; }
    __syncthreads();
    if (tid < CPX) {
      const int ch0 = tid * 8 - p.bch_off;
      if (ch0 >= 0 && ch0 < p.bC) {
        float ta[8], tb[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) { ta[e] = 0.f; tb[e] = 0.f; }
        for (int q = tid; q < 256; q += CPX)
#pragma unroll
          for (int e = 0; e < 8; ++e) { ta[e] += red[q * 16 + e]; tb[e] += red[q * 16 + 8 + e]; }
#pragma unroll
        for (int e = 0; e < 8; ++e)
          *reinterpret_cast<float2*>(p.part2 + ((long long)blockIdx.x * p.bC + ch0 + e) * 2) = make_float2(ta[e], tb[e]);
      }
    }
  }
}

// ---- the PatchGAN logits layer's input gradient (Conv2d k4 s1 p1, 512 -> 1 at 31 -> 30; STCGAN/networks.py:183-184):
// dy (30 x 30, the 1 real channel padded to 8) -> 31 x 31 x 512 with the layer-4 BatchNorm's backward sums fused in
// (stc_conv_bwd_bn, kind STC_CONV_S1_DGRAD).  out(y, x) = sum_{ky,kx} dy[y + 1 - ky][x + 1 - kx] w[ky][kx]: K = 128, so
// the launch is the 31.5 MB output + the 31.5 MB BN input.  A block = (image, 8-row strip, 128 output channels); the
// strip's 11 dy rows (5 KiB) are staged once; its 16 tasks (output row x 16-pixel half) go round-robin to the 4 waves,
// each task's BN-input loads issued one task ahead.
constexpr int S1D_W = 31, S1D_PAD = 32;
__global__ void __launch_bounds__(256) stem_s1d_kernel(const GParams p) {
  constexpr int NF = 8, CPX = 16, PXS = 4, NPASS = 4;  // 128 channels: 16-byte chunks per pixel, store passes
  constexpr int PITCH = 128 * 2 + 16;
  constexpr int NRW = S1D_RB + 3;                     // staged dy rows
  __shared__ __attribute__((aligned(16))) char dys[NRW * S1D_PAD * 16];
  __shared__ __attribute__((aligned(16))) char stgs[4 * 16 * PITCH];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  char* stg = stgs + wave * 16 * PITCH;
  const int nslices = p.N / 128, strips = (p.GH + S1D_RB - 1) / S1D_RB;
  int bid = blockIdx.x;
  const int ns = bid % nslices;
  bid /= nslices;
  const int strip = bid % strips, img = bid / strips;
  const int y0 = strip * S1D_RB, n0 = ns * 128;
  const int rl = lane & 15, kq = lane >> 4;
  // dy rows y0 - 2 .. y0 + 8 (local r), columns 0 .. 31 (>= IW: zero)
  for (int i = tid; i < NRW * S1D_PAD; i += 256) {
    const int r = i / S1D_PAD, c = i % S1D_PAD, gy = y0 - 2 + r;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if ((unsigned)gy < (unsigned)p.IH && c < p.IW)
      v = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(p.a) + (long long)img * p.a_bs +
                                          (long long)gy * p.a_rs + (long long)c * p.a_ps + p.a_co);
    *reinterpret_cast<uint4*>(dys + i * 16) = v;
  }
  bf16x8_t wf[NF][4];
#pragma unroll
  for (int j = 0; j < NF; ++j)
#pragma unroll
    for (int ky = 0; ky < 4; ++ky)
      wf[j][ky] = *reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const bf16*>(p.b) + (n0 + 16 * j + rl) * 128 +
                                                     (4 * ky + kq) * 8);
  const int sc = lane % CPX, spx = lane / CPX;
  const int nb = n0 + sc * 8 - p.bch_off;
  const bool bn_lane = nb >= 0 && nb < p.bC;
  const int nbc = bn_lane ? nb : 0;
  float bsc[8], bsh[8], bmu[8], brs[8], sa[8], sb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bsc[e] = p.bsc[nbc + e]; bsh[e] = p.bsh[nbc + e]; bmu[e] = p.bmu[nbc + e]; brs[e] = p.brs[nbc + e];
    sa[e] = 0.f; sb[e] = 0.f;
  }
  const bf16x8_t zero8 = {};
  __syncthreads();
  // task k of this wave: output row y0 + (k >> 1) within the image, pixels 16 (k & 1) .. + 15
  const int ntask = 2 * min(S1D_RB, p.GH - y0);
  auto bn_load = [&](int k, uint4 (&v)[NPASS]) {
    const int y = y0 + (k >> 1);
#pragma unroll
    for (int h = 0; h < NPASS; ++h) {
      const int x = 16 * (k & 1) + spx + PXS * h;
      const bool in = k < ntask && y < p.bxH && x < p.bxW;
      v[h] = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(p.bx) + (long long)img * p.bx_bs +
                                             (long long)(in ? y : 0) * p.bx_rs + (long long)(in ? x : 0) * p.bx_ps +
                                             p.bx_co + nbc);
    }
  };
  uint4 cur[NPASS], nxt[NPASS];
  bn_load(wave, cur);
  for (int k = wave; k < ntask; k += 4) {
    bn_load(k + 4, nxt);
    const int yl = k >> 1, y = y0 + yl;
    const int px = 16 * (k & 1) + rl;
    floatx4 acc[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ky = 0; ky < 4; ++ky) {
      const int col = px + 1 - kq;  // dy column of tap kx = kq; dy row y + 1 - ky = local row yl + 3 - ky
      const bool cok = (unsigned)col < (unsigned)S1D_PAD;
      bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(dys + ((yl + 3 - ky) * S1D_PAD + (cok ? col : 0)) * 16);
      a = cok ? a : zero8;
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[j] = exp_mfma(a, wf[j][ky], acc[j]);
    }
#pragma unroll
    for (int j = 0; j < NF; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const unsigned u = pack_bf16x2(acc[j][e], 0.f) & 0xffffu;
        *reinterpret_cast<unsigned short*>(stg + (4 * kq + e) * PITCH + (16 * j + rl) * 2) = (unsigned short)u;
      }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int h = 0; h < NPASS; ++h) {
      const int spix = spx + PXS * h;
      const int x = 16 * (k & 1) + spix;
      if (x >= p.GW) continue;  // (pixel 31 of the 32-wide task)
      const uint4 tv = *reinterpret_cast<const uint4*>(stg + spix * PITCH + sc * 16);
      const long long o = (long long)img * p.c_bs + (long long)y * p.c_rs + (long long)x * p.c_ps + p.c_co + n0 + sc * 8;
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.c) + o) = tv;
      if (bn_lane && y < p.bxH && x < p.bxW) {
        const unsigned wt[4] = {tv.x, tv.y, tv.z, tv.w};
        const unsigned wx[4] = {cur[h].x, cur[h].y, cur[h].z, cur[h].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = __uint_as_float((e & 1) ? (wt[e >> 1] & 0xffff0000u) : (wt[e >> 1] << 16));
          const float xv = __uint_as_float((e & 1) ? (wx[e >> 1] & 0xffff0000u) : (wx[e >> 1] << 16));
          const float nn = fmaf(xv, bsc[e], bsh[e]);
          const float dn = v * (nn > 0.f ? 1.f : p.bs_self);
          sa[e] += dn;
          sb[e] += dn * (xv - bmu[e]) * brs[e];
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int h = 0; h < NPASS; ++h) cur[h] = nxt[h];
  }
  // block partial of this slice's channels (threads sharing a chunk, thread order), through the staging LDS
  __syncthreads();
  float* red = reinterpret_cast<float*>(stgs);  // [256][16] = 16 KiB <= 17 KiB
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[tid * 16 + e] = sa[e]; red[tid * 16 + 8 + e] = sb[e]; }
  __syncthreads();
  if (tid < CPX) {
    const int ch0 = n0 + tid * 8 - p.bch_off;
    if (ch0 >= 0 && ch0 < p.bC) {
      float ta[8], tb[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { ta[e] = 0.f; tb[e] = 0.f; }
      for (int q = tid; q < 256; q += CPX)
#pragma unroll
        for (int e = 0; e < 8; ++e) { ta[e] += red[q * 16 + e]; tb[e] += red[q * 16 + 8 + e]; }
      const long long tile = (long long)img * strips + strip;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        *reinterpret_cast<float2*>(p.part2 + (tile * p.bC + ch0 + e) * 2) = make_float2(ta[e], tb[e]);
    }
  }
}

// Eligible: Conv2d k4 s2 p1, 8 input channels (a dense 16-byte bf16 pixel at channel offset 0), input width 256 or
// 512, output rows a multiple of 8, 16-byte NHWC output views; 64 outputs with the activation epilogue, or 128
// outputs with the fused BN-backward sums (input width 256).
static bool stem_sizes(int kind, int Cin, int Cout, int Hg, int Wg, bool bnb) {
  return kind == STC_CONV_S2 && Cin == 8 && Cout == (bnb ? 128 : 64) && (Wg == 128 || (Wg == 256 && !bnb)) &&
         Hg % (bnb ? STEM_RB_BNB : STEM_RB) == 0;
}

bool stem_eligible(int kind, int B, const stc_view& x, int Cin, int Cout, const stc_view& y, bool bnb) {
  if (!stem_sizes(kind, Cin, Cout, y.H, y.W, bnb) || y.H * 2 != x.H || y.W * 2 != x.W) return false;
  if (x.cs != 1 || x.ps != 8 || x.co != 0) return false;
  return (long long)B * x.bs * 2 < (1ll << 31);
}

// the logits layer's input gradient: 8 (padded) dy channels, 128-channel slices, the 31 x 31 grid
static bool s1d_sizes(int kind, int Cin, int Cout, int Hg, int Wg) {
  return kind == STC_CONV_S1_DGRAD && Cin == 8 && Cout % 128 == 0 && Hg == S1D_W && Wg == S1D_W;
}

// BN-backward partial count of the fused input gradient when it takes one of these kernels (0: it does not)
int stem_bnb_chunks(int kind, int B, int Hg, int Wg, int Cin, int Cout) {
  if (s1d_sizes(kind, Cin, Cout, Hg, Wg)) return B * ((Hg + S1D_RB - 1) / S1D_RB);
  return stem_sizes(kind, Cin, Cout, Hg, Wg, true) ? B * (Hg / STEM_RB_BNB) : 0;
}

bool stem_s1d_eligible(int kind, int B, const stc_view& dy, int Cin, int Cout, const stc_view& y) {
  return s1d_sizes(kind, Cin, Cout, y.H, y.W) && dy.H == y.H - 1 && dy.W == y.W - 1 && dy.cs == 1 && dy.ps % 8 == 0 &&
         dy.co % 8 == 0;
}

int stem_s1d_launch(GParams& p, hipStream_t st) {
  const int B = p.M / (p.GH * p.GW);
  const dim3 grid((unsigned)(B * ((p.GH + S1D_RB - 1) / S1D_RB) * (p.N / 128)));
  main_timer_begin(st);
  hipLaunchKernelGGL(stem_s1d_kernel, grid, dim3(256), 0, st, p);
  main_timer_end(st);
  STC_CHECK_LAUNCH();
  return 0;
}

int stem_launch(GParams& p, hipStream_t st) {
  const int B = p.M / (p.GH * p.GW);
  const bool bnb = p.part2 != nullptr;
  const dim3 grid((unsigned)(B * (p.GH / (bnb ? STEM_RB_BNB : STEM_RB))));
  const int n = bnb ? 128 : 64;
  const size_t lds = std::max((size_t)STEM_NS * p.IW * 16 + 4 * 16 * (n * 2 + 16), (size_t)256 * 16 * 4);
  main_timer_begin(st);
#define STEM_K(W_, N_, M_) hipLaunchKernelGGL((stem_conv_kernel<W_, N_, M_>), grid, dim3(256), lds, st, p)
  if (p.IW == 256) {
    if (bnb) STEM_K(256, 128, 3);
    else if (p.act_n == 2) STEM_K(256, 64, 2);
    else STEM_K(256, 64, 1);
  } else {
    if (p.act_n == 2) STEM_K(512, 64, 2);
    else STEM_K(512, 64, 1);
  }
#undef STEM_K
  main_timer_end(st);
  STC_CHECK_LAUNCH();
  return 0;
}

}  // namespace stc
