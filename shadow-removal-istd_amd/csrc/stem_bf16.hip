// bf16 first-layer Conv2d k4 s2 p1 with 8 (padded) input channels and 64 outputs + activation epilogue
// (G's outermost down conv, STCGAN/networks.py:99, and D's first conv, :165-166; no BatchNorm after either).
//
// The layer is HBM-bound: K = 16 taps x 8 channels = 128, so its MFMA work is 4 % of the time it takes to read
// the 16-byte input pixels once and write the 128-byte output pixels once or twice (the LeakyReLU copy for the next
// conv and, in G, the ReLU copy for the skip concat).  The im2col GEMM tile re-stages every input pixel 4 times per
// 128-row tile and pays a load latency per tile; here a block owns a strip of 8 output rows of one image and streams
// its input rows through an 8-slot LDS ring by LDS-DMA (an input row = W x 16 B; output row oy reads input rows
// 2oy-1 .. 2oy+2, so each output row brings 2 new input rows), two output rows of loads ahead of the MFMAs.  Padding
// rows are out-of-range DMA offsets (zeros); the padding columns are zeroed in registers.
//
// MFMA v_mfma_f32_16x16x32_bf16, K-step = kernel row ky: a lane's 8 K values (tap (ky, kx = lane >> 4), 8 channels)
// are one input pixel, one ds_read_b128 (conflict-free: the 16 lanes of a group read 16 distinct pixels mod 16);
// the 64 x 128 weights live in registers (16 fragments).  A wave computes 16 output pixels x 64 channels per chunk;
// the epilogue adds the bias, rounds to bf16, applies act(s1) [and act(s2)] to the rounded value exactly as
// stc_bn_apply with no table does, and writes 16-byte NHWC rows through a per-wave LDS transpose.
#include "igemm_bf16.hpp"

namespace stc {

constexpr int STEM_RB = 8;   // output rows per block
constexpr int STEM_NS = 8;   // input-row slots in the LDS ring

template <int WIN, int NOUT>
__global__ void __launch_bounds__(256) stem_conv_kernel(const GParams p) {
  constexpr int WOUT = WIN / 2;
  constexpr int ROWB = WIN * 16;              // bytes of one input row (8 bf16 channels per pixel)
  constexpr int PPW = WIN / 256;              // 1 KiB DMA pieces per wave per input row
  constexpr int NCH = WOUT / 64;              // 64-pixel chunks per output row (16 per wave)
  constexpr int SPW = NCH * 2 * NOUT;         // 16-byte stores per lane per output row
  constexpr int PITCH = 64 * 2 + 16;          // output staging row (64 bf16 + pad)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  char* stg = smem + STEM_NS * ROWB + wave * 16 * PITCH;
  const int strips = p.GH / STEM_RB;
  const int img = blockIdx.x / strips, oy0 = (blockIdx.x - img * strips) * STEM_RB;
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
  bf16x8_t wf[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int ky = 0; ky < 4; ++ky)
      wf[j][ky] = *reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const bf16*>(p.b) + (16 * j + rl) * 128 +
                                                     (4 * ky + kq) * 8);
  float bz[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bz[j] = p.bias ? p.bias[16 * j + rl] : 0.f;
  const bf16x8_t zero8 = {};

  // prologue: the 4 rows of output row 0 and the 2 new rows of output rows 1 and 2
#pragma unroll
  for (int r = 0; r < 8; ++r) load_row(r);
  for (int t = 0; t < STEM_RB; ++t) {
    // rows 2t .. 2t+3 must have landed; younger: this wave's stores of rows t-2 / t-1 and the loads of rows 2t+4.. 2t+7
    // issued between them (t = 0: the loads of rows 4..7; t = 1: rows 6, 7 after the stores of row 0)
    if (t == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * PPW) : "memory");
    else if (t == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW + SPW) : "memory");
    else if (t + 1 < STEM_RB) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW + 2 * SPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * SPW) : "memory");
    __builtin_amdgcn_s_barrier();
    // refill: rows 2t + 8, 2t + 9 into the slots of rows 2t, 2t + 1 ... read by THIS output row: so the refill for
    // output row t + 3 waits for the next barrier; here: rows 2t + 6, 2t + 7 (slots of rows 2t - 2, 2t - 1, last read
    // by output row t - 1, which every wave finished before this barrier)
    if (t >= 1 && 2 * t + 7 < 2 * STEM_RB + 2) {
      load_row(2 * t + 6);
      load_row(2 * t + 7);
    }
    const int oy = oy0 + t;
    const char* rows[4];
#pragma unroll
    for (int ky = 0; ky < 4; ++ky) rows[ky] = ring + ((2 * t + ky) % STEM_NS) * ROWB;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int ox = ch * 64 + wave * 16 + rl;  // this lane's output pixel
      const int col = 2 * ox + kq - 1;          // input column of tap kx = kq
      const bool cok = (unsigned)col < (unsigned)WIN;
      floatx4 acc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ky = 0; ky < 4; ++ky) {
        bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(rows[ky] + (cok ? col : 0) * 16);
        a = cok ? a : zero8;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = exp_mfma(a, wf[j][ky], acc[j]);
      }
      // acc[j][e] = out[pixel ch*64 + wave*16 + 4 kq + e][channel 16 j + rl]: + bias, bf16, staged [pixel][64 ch]
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = acc[j][e] + bz[j];
          const unsigned u = pack_bf16x2(v, 0.f) & 0xffffu;
          *reinterpret_cast<unsigned short*>(stg + (4 * kq + e) * PITCH + (16 * j + rl) * 2) = (unsigned short)u;
        }
      __builtin_amdgcn_wave_barrier();
      // 16 pixels x 8 chunks of 16 B: lane -> chunk lane & 7, pixels lane >> 3 and + 8
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int px = (lane >> 3) + 8 * h, c8 = lane & 7;
        const uint4 tv = *reinterpret_cast<const uint4*>(stg + px * PITCH + c8 * 16);
        const int oxs = ch * 64 + wave * 16 + px;
        const long long o1 = (long long)img * p.c_bs + (long long)oy * p.c_rs + (long long)oxs * p.c_ps + p.c_co + c8 * 8;
        *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.c) + o1) = act_bf16x8(tv, p.act_s1);
        if constexpr (NOUT == 2) {
          const long long o2 = (long long)img * p.c2_bs + (long long)oy * p.c2_rs + (long long)oxs * p.c2_ps + p.c2_co + c8 * 8;
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.c2) + o2) = act_bf16x8(tv, p.act_s2);
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// Eligible: Conv2d k4 s2 p1, 8 input channels (a 16-byte bf16 pixel, channel offset 0 of a dense pixel), 64 outputs,
// input width 256 or 512, output rows a multiple of 8, the activation epilogue (no statistics, no split), 16-byte
// NHWC output views.
bool stem_eligible(int kind, int B, const stc_view& x, int Cin, int Cout, const stc_view& y) {
  if (kind != STC_CONV_S2 || Cin != 8 || Cout != 64) return false;
  if (!(x.W == 256 || x.W == 512) || x.H % 2 != 0 || y.H * 2 != x.H || y.W * 2 != x.W || y.H % STEM_RB != 0) return false;
  if (x.cs != 1 || x.ps != 8 || x.co != 0) return false;
  return (long long)B * x.bs * 2 < (1ll << 31);
}

int stem_launch(GParams& p, hipStream_t st) {
  const int B = p.M / (p.GH * p.GW);
  const dim3 grid((unsigned)(B * (p.GH / STEM_RB)));
  const size_t lds = (size_t)STEM_NS * p.IW * 16 + 4 * 16 * (64 * 2 + 16);
  main_timer_begin(st);
  if (p.IW == 256) {
    if (p.act_n == 2) hipLaunchKernelGGL((stem_conv_kernel<256, 2>), grid, dim3(256), lds, st, p);
    else hipLaunchKernelGGL((stem_conv_kernel<256, 1>), grid, dim3(256), lds, st, p);
  } else {
    if (p.act_n == 2) hipLaunchKernelGGL((stem_conv_kernel<512, 2>), grid, dim3(256), lds, st, p);
    else hipLaunchKernelGGL((stem_conv_kernel<512, 1>), grid, dim3(256), lds, st, p);
  }
  main_timer_end(st);
  STC_CHECK_LAUNCH();
  return 0;
}

}  // namespace stc
