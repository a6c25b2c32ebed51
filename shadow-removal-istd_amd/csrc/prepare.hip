// Training-batch preparation on the GPU (STCGAN/dataset.py:89-147 with the
// transforms of STCGAN/transform.py:103-156): from decoded uint8 HWC images to the fp32 NCHW
// tensors the trainer consumes,
//   v = u / 255                        (utils.uint2float, utils.py:58-60: float32 division)
//   v = (v - 0.5) * 2                  (dataset.py:122-124, the intended normalisation)
//   RandomHorizontalFlip               (np.fliplr when drawn, transform.py:103-116)
//   RandomCrop with zero padding       (cv.copyMakeBorder(BORDER_CONSTANT, 0) of the normalised
//                                       image when it is smaller than the crop, transform.py:119-156)
// in one pass: one thread per output element, reading its source byte (HBM-bound: 1 B read +
// 4 B written per element).  The random parameters are drawn on the host in the reference's
// call order and passed per image as {flip, row_offset, col_offset}.  Before it, as the reference
// composes them (transform.py:7-24): Resize (shrink in both axes: INTER_AREA, resize_area_kernel;
// otherwise INTER_LINEAR, resize_linear_kernel), RandomScale and RandomRotate (cv.warpAffine with
// getRotationMatrix2D about the image centre, INTER_LINEAR -- warpAffine turns RandomScale's
// INTER_AREA into INTER_LINEAR -- and BORDER_CONSTANT 0: warp_affine_kernel).
#include <cfloat>

#include "common.hpp"

#pragma clang fp contract(off)  // (u / 255 - 0.5) * 2 rounded step by step, as numpy does

namespace stc {

template <typename T>
__global__ void __launch_bounds__(256) prepare_kernel(const T* __restrict__ src, int B, int H, int W, int C,
                                                      const int* __restrict__ params, int pad_h, int pad_w, int OH,
                                                      int OW, float* __restrict__ dst) {
  const long long total = (long long)B * C * OH * OW;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(i % OW);
    long long t = i / OW;
    const int y = (int)(t % OH);
    t /= OH;
    const int c = (int)(t % C);
    const int b = (int)(t / C);
    const int flip = params[b * 3], oy = params[b * 3 + 1], ox = params[b * 3 + 2];
    const int Y = y + oy - pad_h, X = x + ox - pad_w;
    float v = 0.f;  // the constant border of the normalised image
    if (Y >= 0 && Y < H && X >= 0 && X < W) {
      const int sx = flip ? W - 1 - X : X;
      const T u = src[(((long long)b * H + Y) * W + sx) * C + c];
      if constexpr (sizeof(T) == 1) v = ((float)u / 255.f - 0.5f) * 2.f;
      else v = u;
    }
    dst[i] = v;
  }
}

// Resize (transform.py:159-181) on the normalised image when it shrinks in both dimensions:
// cv.resize INTER_AREA.  Generic scale: OpenCV's computeResizeAreaTab cells (partial first /
// whole / partial last source pixel, weights in double rounded to float) and ResizeArea_Invoker's
// order -- per source row of the cell a horizontal float sum buf = sum_k S[sx_k] * alpha_k, then
// sum = sum + beta * buf over the rows.  Integer scales in both axes: resizeAreaFast, the block sum
// in row-major order times float(1 / area).  Source = uint8, normalised on the fly exactly as the
// reference normalises before resizing ((u / 255 - 0.5) * 2 per pixel).
__device__ __forceinline__ int area_cells(int d, double scale, int ssize, int* sx, float* al) {
  const double fsx1 = d * scale, fsx2 = fsx1 + scale;
  const double cellWidth = fmin(scale, ssize - fsx1);
  int sx1 = (int)ceil(fsx1), sx2 = (int)floor(fsx2);
  sx2 = min(sx2, ssize - 1);
  sx1 = min(sx1, sx2);
  int k = 0;
  if (sx1 - fsx1 > 1e-3) { sx[k] = sx1 - 1; al[k++] = (float)((sx1 - fsx1) / cellWidth); }
  for (int s = sx1; s < sx2; ++s) { sx[k] = s; al[k++] = (float)(1.0 / cellWidth); }
  if (fsx2 - sx2 > 1e-3) { sx[k] = sx2; al[k++] = (float)(fmin(fmin(fsx2 - sx2, 1.0), cellWidth) / cellWidth); }
  return k;
}

constexpr int AREA_MAXK = 18;  // source pixels per cell (scale <= 16)

__global__ void __launch_bounds__(256) resize_area_kernel(const unsigned char* __restrict__ src, int B, int H, int W,
                                                          int C, int OH, int OW, double scale_y, double scale_x,
                                                          int fast_y, int fast_x, float* __restrict__ dst) {
  const long long total = (long long)B * OH * OW;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int dx = (int)(i % OW);
    const long long t = i / OW;
    const int dy = (int)(t % OH), b = (int)(t / OH);
    const unsigned char* img = src + (long long)b * H * W * C;
    for (int c = 0; c < C; ++c) {
      float out;
      if (fast_y > 0) {  // resizeAreaFast: integer scales in both axes
        float s = 0.f;
        for (int yy = 0; yy < fast_y; ++yy)
          for (int xx = 0; xx < fast_x; ++xx) {
            const float u = (float)img[((long long)(dy * fast_y + yy) * W + dx * fast_x + xx) * C + c];
            s = s + (u / 255.f - 0.5f) * 2.f;
          }
        out = s * (1.f / (float)(fast_y * fast_x));
      } else {
        int xs[AREA_MAXK], ys[AREA_MAXK];
        float ax[AREA_MAXK], ay[AREA_MAXK];
        const int kx = area_cells(dx, scale_x, W, xs, ax), ky = area_cells(dy, scale_y, H, ys, ay);
        float sum = 0.f;
        for (int j = 0; j < ky; ++j) {
          const unsigned char* row = img + (long long)ys[j] * W * C + c;
          float buf = 0.f;
          for (int k = 0; k < kx; ++k) {
            const float v = ((float)row[(long long)xs[k] * C] / 255.f - 0.5f) * 2.f;
            buf = buf + v * ax[k];
          }
          sum = sum + ay[j] * buf;
        }
        out = sum;
      }
      dst[i * C + c] = out;
    }
  }
}


// ---- src element: uint8 normalised on the fly ((u / 255 - 0.5) * 2, step by step) or fp32 as is
__device__ __forceinline__ float norm_src(const void* src, int u8, long long i) {
  if (u8) return ((float)reinterpret_cast<const unsigned char*>(src)[i] / 255.f - 0.5f) * 2.f;
  return reinterpret_cast<const float*>(src)[i];
}

// Resize (transform.py:173-178) when the image does not shrink in both axes: cv.resize INTER_LINEAR
// of the float32 image, OpenCV's generic path -- per output column the source index / weight from
// float((dx + 0.5) * scale - 0.5) (index clamped with weight 0 at the borders, one term past the
// right edge), per row the same with the rows clamped and the weights unclamped; horizontal
// S[sx]*a0 + S[sx+1]*a1, vertical h0*b0 + h1*b1, each product and sum rounded on its own.
__global__ void __launch_bounds__(256) resize_linear_kernel(const void* __restrict__ src, int u8, int B, int H, int W,
                                                            int C, int OH, int OW, double scale_y, double scale_x,
                                                            float* __restrict__ dst) {
  const long long total = (long long)B * OH * OW;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int dx = (int)(i % OW);
    const long long t = i / OW;
    const int dy = (int)(t % OH), b = (int)(t / OH);
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = (int)floorf(fx);
    fx = fx - (float)sx;
    const int two = sx + 1 < W ? 1 : 0;
    if (sx < 0) { fx = 0.f; sx = 0; }
    if (sx >= W - 1) { fx = 0.f; sx = W - 1; }
    const float a0 = 1.f - fx, a1 = fx;
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    const int sy = (int)floorf(fy);
    fy = fy - (float)sy;
    const float b0 = 1.f - fy, b1 = fy;
    const int y0 = min(max(sy, 0), H - 1), y1 = min(max(sy + 1, 0), H - 1);
    const int x1 = two ? sx + 1 : sx;
    const long long base = (long long)b * H * W * C;
    for (int c = 0; c < C; ++c) {
      float h[2];
      const int ys[2] = {y0, y1};
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const long long row = base + (long long)ys[k] * W * C + c;
        const float v0 = norm_src(src, u8, row + (long long)sx * C);
        const float v1 = norm_src(src, u8, row + (long long)x1 * C);
        h[k] = two ? v0 * a0 + v1 * a1 : v0 * a0;
      }
      dst[i * C + c] = h[0] * b0 + h[1] * b1;
    }
  }
}

// RandomScale / RandomRotate (transform.py:59-100): cv.warpAffine(x, M, (cols, rows), INTER_LINEAR,
// BORDER_CONSTANT 0) with M the per-image forward matrix (getRotationMatrix2D, float64).  OpenCV
// inverts M (warpAffine, no WARP_INVERSE_MAP), then maps each destination pixel in fixed point:
// X = (cvRound((M1*y + M2)*1024) + 16 + cvRound(M0*x*1024)) >> 5 (likewise Y), source pixel
// (X >> 5, Y >> 5), sub-pixel (X & 31, Y & 31) selecting the float weights of BilinearTab_f
// ((1 - fy)(1 - fx), (1 - fy) fx, fy (1 - fx), fy fx with f = k/32), and taps outside the image read
// the border value 0 (remapBilinear): D = ((S00*w0 + S01*w1) + S10*w2) + S11*w3.
__global__ void __launch_bounds__(256) warp_affine_kernel(const void* __restrict__ src, int u8, int B, int H, int W,
                                                          int C, const double* __restrict__ Mfwd,
                                                          float* __restrict__ dst) {
  const long long total = (long long)B * H * W;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(i % W);
    const long long t = i / W;
    const int y = (int)(t % H), b = (int)(t / H);
    double M[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) M[k] = Mfwd[b * 6 + k];
    {  // cv::warpAffine's inversion
      double D = M[0] * M[4] - M[1] * M[3];
      D = D != 0 ? 1. / D : 0;
      const double A11 = M[4] * D, A22 = M[0] * D;
      M[0] = A11; M[1] *= -D;
      M[3] *= -D; M[4] = A22;
      const double b1 = -M[0] * M[2] - M[1] * M[5];
      const double b2 = -M[3] * M[2] - M[4] * M[5];
      M[2] = b1; M[5] = b2;
    }
    const int X0 = __double2int_rn((M[1] * y + M[2]) * 1024.0) + 16;
    const int Y0 = __double2int_rn((M[4] * y + M[5]) * 1024.0) + 16;
    const int X = (X0 + __double2int_rn(M[0] * x * 1024.0)) >> 5;
    const int Y = (Y0 + __double2int_rn(M[3] * x * 1024.0)) >> 5;
    const int sx = X >> 5, sy = Y >> 5;
    const float fx = (float)(X & 31) * (1.f / 32.f), fy = (float)(Y & 31) * (1.f / 32.f);
    const float vx0 = 1.f - fx, vy0 = 1.f - fy;
    const float w0 = vy0 * vx0, w1 = vy0 * fx, w2 = fy * vx0, w3 = fy * fx;
    const bool in00 = sx >= 0 && sx < W && sy >= 0 && sy < H, in01 = sx + 1 >= 0 && sx + 1 < W && sy >= 0 && sy < H;
    const bool in10 = sx >= 0 && sx < W && sy + 1 >= 0 && sy + 1 < H;
    const bool in11 = sx + 1 >= 0 && sx + 1 < W && sy + 1 >= 0 && sy + 1 < H;
    const long long base = (long long)b * H * W * C;
    for (int c = 0; c < C; ++c) {
      const float s00 = in00 ? norm_src(src, u8, base + ((long long)sy * W + sx) * C + c) : 0.f;
      const float s01 = in01 ? norm_src(src, u8, base + ((long long)sy * W + sx + 1) * C + c) : 0.f;
      const float s10 = in10 ? norm_src(src, u8, base + ((long long)(sy + 1) * W + sx) * C + c) : 0.f;
      const float s11 = in11 ? norm_src(src, u8, base + ((long long)(sy + 1) * W + sx + 1) * C + c) : 0.f;
      dst[i * C + c] = ((s00 * w0 + s01 * w1) + s10 * w2) + s11 * w3;
    }
  }
}

}  // namespace stc

using namespace stc;

extern "C" int stc_prepare_batch(const unsigned char* src, int B, int H, int W, int C, const int* params, int pad_h,
                                 int pad_w, int OH, int OW, float* dst, void* stream) {
  STC_REQUIRE(B >= 0 && H >= 1 && W >= 1 && C >= 1 && OH >= 1 && OW >= 1 && pad_h >= 0 && pad_w >= 0,
              "stc_prepare_batch: bad shape B=%d H=%d W=%d C=%d OH=%d OW=%d", B, H, W, C, OH, OW);
  if (B == 0) return 0;
  STC_REQUIRE(src && params && dst, "stc_prepare_batch: null pointer");
  const long long total = (long long)B * C * OH * OW;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(prepare_kernel<unsigned char>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, src, B, H, W, C,
                     params, pad_h, pad_w, OH, OW, dst);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_prepare_batch_f32(const float* src, int B, int H, int W, int C, const int* params, int pad_h,
                                     int pad_w, int OH, int OW, float* dst, void* stream) {
  STC_REQUIRE(B >= 0 && H >= 1 && W >= 1 && C >= 1 && OH >= 1 && OW >= 1 && pad_h >= 0 && pad_w >= 0,
              "stc_prepare_batch_f32: bad shape B=%d H=%d W=%d C=%d OH=%d OW=%d", B, H, W, C, OH, OW);
  if (B == 0) return 0;
  STC_REQUIRE(src && params && dst, "stc_prepare_batch_f32: null pointer");
  const long long total = (long long)B * C * OH * OW;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(prepare_kernel<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, src, B, H, W, C, params,
                     pad_h, pad_w, OH, OW, dst);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_resize_area(const unsigned char* src, int B, int H, int W, int C, int OH, int OW, float* dst,
                               void* stream) {
  STC_REQUIRE(B >= 0 && C >= 1 && OH >= 1 && OW >= 1 && OH < H && OW < W,
              "stc_resize_area: INTER_AREA shrink only (B=%d %dx%d -> %dx%d)", B, H, W, OH, OW);
  if (B == 0) return 0;
  STC_REQUIRE(src && dst, "stc_resize_area: null pointer");
  const double scale_x = 1.0 / ((double)OW / W), scale_y = 1.0 / ((double)OH / H);
  const int iscale_x = (int)lround(scale_x), iscale_y = (int)lround(scale_y);
  const bool fast = fabs(scale_x - iscale_x) < DBL_EPSILON && fabs(scale_y - iscale_y) < DBL_EPSILON;
  STC_REQUIRE(fast || (scale_x < AREA_MAXK - 2 && scale_y < AREA_MAXK - 2), "stc_resize_area: scale too large");
  const long long total = (long long)B * OH * OW;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(resize_area_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, src, B, H, W, C, OH, OW,
                     scale_y, scale_x, fast ? iscale_y : 0, fast ? iscale_x : 0, dst);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_resize_linear(const void* src, int src_u8, int B, int H, int W, int C, int OH, int OW, float* dst,
                                 void* stream) {
  STC_REQUIRE(B >= 0 && H >= 1 && W >= 1 && C >= 1 && OH >= 1 && OW >= 1,
              "stc_resize_linear: bad shape B=%d %dx%d -> %dx%d", B, H, W, OH, OW);
  if (B == 0) return 0;
  STC_REQUIRE(src && dst, "stc_resize_linear: null pointer");
  const double scale_x = 1.0 / ((double)OW / W), scale_y = 1.0 / ((double)OH / H);
  const long long total = (long long)B * OH * OW;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(resize_linear_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, src, src_u8, B, H, W, C,
                     OH, OW, scale_y, scale_x, dst);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_warp_affine(const void* src, int src_u8, int B, int H, int W, int C, const double* M, float* dst,
                               void* stream) {
  STC_REQUIRE(B >= 0 && H >= 1 && W >= 1 && C >= 1 && H < 16384 && W < 16384,
              "stc_warp_affine: bad shape B=%d %dx%d", B, H, W);
  if (B == 0) return 0;
  STC_REQUIRE(src && M && dst, "stc_warp_affine: null pointer");
  const long long total = (long long)B * H * W;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(warp_affine_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, src, src_u8, B, H, W, C, M,
                     dst);
  STC_CHECK_LAUNCH();
  return 0;
}
