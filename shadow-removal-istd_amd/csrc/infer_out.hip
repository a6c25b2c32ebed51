// Inference output stage of STCGAN.infer() (STCGAN/stcgan.py:351-377, STCGAN/utils.py:63-65):
//   v = net_out * 0.5 + 0.5                      (numpy float32, stcgan.py:355-357)
//   r = cv.resize(v_hwc, (OW, OH), INTER_LINEAR) (stcgan.py:367-368, 373-374)
//   u = (r * 255).astype(np.uint8)               (utils.float2uint: truncation, not rounding)
// from the generator's NCHW fp32 output straight to an HWC uint8 image batch [B][OH][OW][C]
// (the array cv.imwrite receives).  The bilinear resize restates OpenCV's generic float32
// INTER_LINEAR path: per-column source index / weights from (dx + 0.5) * scale - 0.5 in double
// rounded to float, the horizontal pass S[sx]*a0 + S[sx+1]*a1 (one term past the right edge),
// rows clamped to [0, H-1] and the vertical pass h0*b0 + h1*b1 -- every product and sum rounded
// separately (no fused multiply-add), as a non-FMA build of OpenCV computes them.  An exact 2x2
// downscale is the one case cv::resize reroutes INTER_LINEAR to INTER_AREA: the 2x2 block mean
// ((S00 + S01 + S10 + S11) summed in that order, times 0.25).
//
// HBM-bound: one thread per output pixel reads its 2x2 source neighbourhood of every channel
// (C <= 4) and writes C bytes; 4 * C * (input pixels touched) + C bytes per output pixel.
#include "common.hpp"

// every product / sum below is rounded on its own (OpenCV / numpy order): no FMA contraction
#pragma clang fp contract(off)

namespace stc {
// round-to-nearest float / double ops defined under contract(off) (HIP's mul_rn & co. are plain
// operators in headers compiled with -ffp-contract=fast, which LLVM may still fuse into an FMA)
__device__ __forceinline__ float mul_rn(float a, float b) { return a * b; }
__device__ __forceinline__ float add_rn(float a, float b) { return a + b; }
__device__ __forceinline__ float sub_rn(float a, float b) { return a - b; }
__device__ __forceinline__ double dmul_rn(double a, double b) { return a * b; }
__device__ __forceinline__ double dsub_rn(double a, double b) { return a - b; }
}  // namespace stc

namespace stc {

struct ResizeAxis {
  int s;     // first source index
  int two;   // 1: two-tap (s, s+1); 0: single tap s (right edge)
  float a0, a1;
};

// OpenCV resizeGeneric_ coefficient setup for INTER_LINEAR (ksize 2), one output index.
__device__ __forceinline__ ResizeAxis linear_axis_x(int d, double scale, int n) {
  float f = (float)dsub_rn(dmul_rn(d + 0.5, scale), 0.5);
  int s = (int)floorf(f);
  f = sub_rn(f, (float)s);
  ResizeAxis ax;
  ax.two = (s + 1 < n) ? 1 : 0;
  if (s < 0) { f = 0.f; s = 0; }
  if (s >= n - 1) { f = 0.f; s = n - 1; }
  ax.s = s;
  ax.a0 = sub_rn(1.f, f);
  ax.a1 = f;
  return ax;
}

__global__ void __launch_bounds__(256) infer_output_kernel(const float* __restrict__ src, int B, int C, int H, int W,
                                                           int OH, int OW, double scale_y, double scale_x,
                                                           int area2, unsigned char* __restrict__ dst) {
  const long long total = (long long)B * OH * OW;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int dx = (int)(i % OW);
    const long long t = i / OW;
    const int dy = (int)(t % OH);
    const int b = (int)(t / OH);
    unsigned char* o = dst + i * C;
    if (area2) {  // exact 2x2 downscale: OpenCV switches INTER_LINEAR to INTER_AREA (block mean)
      for (int c = 0; c < C; ++c) {
        const float* p0 = src + (((long long)b * C + c) * H + 2 * dy) * W + 2 * dx;
        float s = 0.f;
        const float q4[4] = {p0[0], p0[1], p0[W], p0[W + 1]};
#pragma unroll
        for (int k = 0; k < 4; ++k) s = add_rn(s, add_rn(mul_rn(q4[k], 0.5f), 0.5f));
        int q = (int)mul_rn(mul_rn(s, 0.25f), 255.f);
        o[c] = (unsigned char)(q < 0 ? 0 : (q > 255 ? 255 : q));
      }
      continue;
    }
    const ResizeAxis ax = linear_axis_x(dx, scale_x, W);
    // vertical: weights from the unclamped index, rows clamped (OpenCV clip(sy + k, 0, H))
    float fy = (float)dsub_rn(dmul_rn(dy + 0.5, scale_y), 0.5);
    const int sy = (int)floorf(fy);
    fy = sub_rn(fy, (float)sy);
    const float b0 = sub_rn(1.f, fy), b1 = fy;
    const int y0 = min(max(sy, 0), H - 1), y1 = min(max(sy + 1, 0), H - 1);
    const int x1 = ax.two ? ax.s + 1 : ax.s;
    for (int c = 0; c < C; ++c) {
      const float* plane = src + ((long long)b * C + c) * H * W;
      float h[2];
      const int ys[2] = {y0, y1};
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const float* row = plane + (long long)ys[k] * W;
        // v = x * 0.5 + 0.5 (x * 0.5 is exact, so one rounding either way)
        const float v0 = add_rn(mul_rn(row[ax.s], 0.5f), 0.5f);
        const float v1 = add_rn(mul_rn(row[x1], 0.5f), 0.5f);
        h[k] = ax.two ? add_rn(mul_rn(v0, ax.a0), mul_rn(v1, ax.a1)) : mul_rn(v0, ax.a0);
      }
      const float r = add_rn(mul_rn(h[0], b0), mul_rn(h[1], b1));
      // float2uint: (r * 255).astype(uint8) truncates toward zero; r is in [0, 1] up to rounding
      const float u = mul_rn(r, 255.f);
      int q = (int)u;
      q = q < 0 ? 0 : (q > 255 ? 255 : q);
      o[c] = (unsigned char)q;
    }
  }
}

}  // namespace stc

using namespace stc;

extern "C" int stc_infer_output(const float* src, int B, int C, int H, int W, int OH, int OW, unsigned char* dst,
                                void* stream) {
  STC_REQUIRE(B >= 0 && C >= 1 && C <= 4 && H >= 1 && W >= 1 && OH >= 1 && OW >= 1 && (B == 0 || (src && dst)),
              "stc_infer_output: bad arguments B=%d C=%d H=%d W=%d OH=%d OW=%d", B, C, H, W, OH, OW);
  if (B == 0) return 0;  // empty batch (null data pointers allowed)
  // cv::resize: inv_scale = dsize / ssize, scale = 1 / inv_scale (both double)
  const double scale_x = 1.0 / ((double)OW / W), scale_y = 1.0 / ((double)OH / H);
  const long long total = (long long)B * OH * OW;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 8192);
  const int area2 = (H == 2 * OH && W == 2 * OW) ? 1 : 0;  // cv::resize: INTER_LINEAR at scale 2x2 -> INTER_AREA
  hipLaunchKernelGGL(infer_output_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, src, B, C, H, W, OH, OW,
                     scale_y, scale_x, area2, dst);
  STC_CHECK_LAUNCH();
  return 0;
}
