// First-layer convolutions (Cin = 8 after padding, Cout = 64, 4x4 stride 2 pad 1): the input layer of both
// generators and both discriminators, STCGAN/networks.py:99 (UnetSkipConnectionBlock outermost downconv) and
// :165 (NLayerDiscriminator's first Conv2d), each followed by LeakyReLU with no BatchNorm.
//
// K = 16 taps x 8 channels = 128, so the implicit GEMM has almost no reduction to hide its loads behind: the
// LDS-DMA tile (igemm_bf16.hip) gathers every 16-byte input pixel 4 times (the 2x2 output pixels whose 4x4
// windows cover it) and refills per 128-row tile, ~2.4 TB/s on ~100 MB of compulsory traffic.  Here a block
// owns whole output rows: the 4 input rows an output row reads are staged once in LDS (coalesced 16-byte
// loads, zero rows / columns for the padding), every MFMA A fragment is one ds_read_b128 of an input pixel
// (the 8 K values a lane holds in v_mfma_f32_16x16x32_bf16 are exactly one tap's 8 channels), and the
// weights (16 KiB) stay in registers for all the rows a persistent block visits.  Epilogue as the GEMM's
// activation epilogue: bias, bf16 rounding, act(v, slope) rounded again, one or two outputs, staged per wave
// through LDS into 16-byte NHWC stores.  The K order (4 steps of 32, tap-major, channels fastest) and the
// instruction are the GEMM tile's, so the outputs are bit-identical to it.
#include "common.hpp"

namespace stc {

struct H8Params {
  const char* x;  // NHWC bf16 input, 8 channels at x_co
  long long x_bs, x_rs;
  int x_ps, x_co;
  int B, IH, IW, OH, OW;
  const bf16* w;  // packed conv operand [64][128] (k = tap * 8 + c)
  const float* bias;
  char* y1;
  long long y1_bs, y1_rs;
  int y1_ps, y1_co;
  char* y2;  // second activated copy (act_n == 2)
  long long y2_bs, y2_rs;
  int y2_ps, y2_co;
  int act_n;
  float s1, s2;
};

constexpr int H8_T = 256;         // 4 waves
constexpr int H8_NF = 4;          // 64 output channels = 4 column fragments
constexpr int H8_CH = 16 * H8_NF;
constexpr int H8_STG = 16 * H8_CH * 2;  // one wave's staged 16 pixels x 64 channels, bf16 (per output)

__global__ void __launch_bounds__(H8_T) halo8_conv_kernel(const H8Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int RW = p.IW + 2;  // staged row: input columns -1 .. IW
  uint4* rows = reinterpret_cast<uint4*>(smem);
  char* stg = smem + (size_t)4 * RW * 16;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int cl = lane & 15, kq = lane >> 4;
  // B fragments: column fragment j, K step kk: W[16j + cl][32kk + 8kq .. +7]
  stc_bf16x8 fb[H8_NF][4];
#pragma unroll
  for (int j = 0; j < H8_NF; ++j)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      fb[j][kk] = *reinterpret_cast<const stc_bf16x8*>(p.w + (size_t)(16 * j + cl) * 128 + 32 * kk + 8 * kq);
  float bz[H8_NF];
#pragma unroll
  for (int j = 0; j < H8_NF; ++j) bz[j] = p.bias ? p.bias[16 * j + cl] : 0.f;
  const int groups = (p.OW + 15) / 16;  // 16-pixel groups of an output row
  const int gpw = (groups + 3) / 4;     // group iterations per wave (uniform: the barriers stay aligned)
  char* sw1 = stg + (size_t)wv * 2 * H8_STG;
  char* sw2 = sw1 + H8_STG;
  const int nrows = p.B * p.OH;
  for (int row = blockIdx.x; row < nrows; row += gridDim.x) {
    const int b = row / p.OH, oy = row - b * p.OH;
    __syncthreads();  // the previous row's fragment reads are done
    for (int q = tid; q < 4 * RW; q += H8_T) {
      const int r = q / RW, c = q - r * RW;
      const int iy = 2 * oy - 1 + r, ix = c - 1;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (iy >= 0 && iy < p.IH && ix >= 0 && ix < p.IW)
        v = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(p.x) + (long long)b * p.x_bs +
                                            (long long)iy * p.x_rs + (long long)ix * p.x_ps + p.x_co);
      rows[q] = v;
    }
    __syncthreads();
    for (int gi = 0; gi < gpw; ++gi) {
      const int g = wv + 4 * gi;
      if (g >= groups) continue;  // wave-uniform; no barrier below
      const int px = min(16 * g + cl, p.OW - 1);
      floatx4 acc[H8_NF];
#pragma unroll
      for (int j = 0; j < H8_NF; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        // tap (ky = kk, kx = kq) of output pixel px: input (2oy - 1 + kk, 2px - 1 + kq) = staged (kk, 2px + kq)
        const stc_bf16x8 fa = *reinterpret_cast<const stc_bf16x8*>(rows + kk * RW + 2 * px + kq);
#pragma unroll
        for (int j = 0; j < H8_NF; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[j][kk], acc[j], 0, 0, 0);
      }
      // acc[j][r]: pixel 16g + 4kq + r, channel 16j + cl -> staged [pixel][channel] bf16
#pragma unroll
      for (int j = 0; j < H8_NF; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[j][r] + bz[j];
          const float raw = __uint_as_float(pack_bf16x2(v, v) << 16);
          const int o = ((4 * kq + r) * H8_CH + 16 * j + cl) * 2;
          *reinterpret_cast<unsigned short*>(sw1 + o) = (unsigned short)(pack_bf16x2(act(raw, p.s1), 0.f) & 0xffffu);
          if (p.act_n == 2)
            *reinterpret_cast<unsigned short*>(sw2 + o) = (unsigned short)(pack_bf16x2(act(raw, p.s2), 0.f) & 0xffffu);
        }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // 16 pixels x 8 chunks of 16 bytes per output: 2 per lane
#pragma unroll
      for (int u = 0; u < 16 * (H8_CH / 8) / 64; ++u) {
        const int q = lane + 64 * u;
        const int pl = q / (H8_CH / 8), c8 = q - pl * (H8_CH / 8);
        const int gx = 16 * g + pl;
        if (gx >= p.OW) continue;
        const int so = (pl * H8_CH + 8 * c8) * 2;
        *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.y1) + (long long)b * p.y1_bs + (long long)oy * p.y1_rs +
                                  (long long)gx * p.y1_ps + p.y1_co + 8 * c8) = *reinterpret_cast<const uint4*>(sw1 + so);
        if (p.act_n == 2)
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.y2) + (long long)b * p.y2_bs + (long long)oy * p.y2_rs +
                                    (long long)gx * p.y2_ps + p.y2_co + 8 * c8) = *reinterpret_cast<const uint4*>(sw2 + so);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
}

static bool view16(const stc_view& v) {
  return v.p && v.cs == 1 && v.co % 8 == 0 && v.ps % 8 == 0 && v.rs % 8 == 0 && v.bs % 8 == 0 &&
         ((uintptr_t)v.p & 15) == 0;
}

// The halo kernel applies to the activation-epilogue conv_s2 with 8 input and 64 output channels whose input
// rows fit the LDS stage (STC_HALO8=1; otherwise the GEMM tile, for A/B and the bit-identity test).
bool halo8_ok(int kind, int B, const stc_view& x, int Cin, int Cout, const stc_view& y1, const stc_view* y2) {
  const char* e = getenv("STC_HALO8");
  if (!(e && e[0] == '1')) return false;  // opt-in: not faster than the GEMM tile
  if (kind != STC_CONV_S2 || Cin != 8 || Cout != H8_CH || B <= 0) return false;
  if (!view16(x) || !view16(y1) || (y2 && y2->p && (!view16(*y2) || y2->H != y1.H || y2->W != y1.W))) return false;
  if (x.W > 2048 || y1.W <= 0 || y1.H <= 0) return false;
  // the conv_s2 geometry of the output (k 4, s 2, p 1)
  return y1.H == x.H / 2 && y1.W == x.W / 2;
}

int halo8_conv_act(int B, const stc_view& x, const void* w_packed, const stc_view& y1, const stc_view* y2, int act_n,
                   float s1, float s2, const float* bias, hipStream_t st) {
  H8Params p{};
  p.x = (const char*)x.p; p.x_bs = x.bs; p.x_rs = x.rs; p.x_ps = x.ps; p.x_co = x.co;
  p.B = B; p.IH = x.H; p.IW = x.W; p.OH = y1.H; p.OW = y1.W;
  p.w = (const bf16*)w_packed; p.bias = bias;
  p.y1 = (char*)y1.p; p.y1_bs = y1.bs; p.y1_rs = y1.rs; p.y1_ps = y1.ps; p.y1_co = y1.co;
  if (act_n == 2) {
    STC_REQUIRE(y2 && y2->p, "halo8 conv: act_n = 2 needs a second output view");
    p.y2 = (char*)y2->p; p.y2_bs = y2->bs; p.y2_rs = y2->rs; p.y2_ps = y2->ps; p.y2_co = y2->co;
  }
  p.act_n = act_n; p.s1 = s1; p.s2 = s2;
  const long long nrows = (long long)B * p.OH;
  if (nrows == 0) return 0;
  STC_REQUIRE(nrows < (1ll << 31), "halo8 conv: too many output rows");
  const char* ge = getenv("STC_HALO8_GRID");  // (tuning hook: persistent blocks per CU)
  const long long per_cu = ge ? std::max(1, atoi(ge)) : 4;
  const unsigned grid = (unsigned)std::min<long long>(nrows, 256LL * per_cu);
  const size_t lds = (size_t)4 * (p.IW + 2) * 16 + (size_t)4 * 2 * H8_STG;
  main_timer_begin(st);
  hipLaunchKernelGGL(halo8_conv_kernel, dim3(grid), dim3(H8_T), lds, st, p);
  main_timer_end(st);
  STC_CHECK_LAUNCH();
  return 0;
}

}  // namespace stc
