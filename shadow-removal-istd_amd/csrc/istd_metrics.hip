// ISTD evaluation errors and SSIM (src/eval.py:41-139 -- the step after the path):
// per image pair, the masked LAB errors and the squared error behind PSNR, from uint8 RGB images
// (the PNGs infer() writes and the ISTD ground truth, read as RGB as skimage.io.imread does):
//   v = u / 255                                   (util.img_as_float32, eval.py:66-69)
//   lab = rgb2lab(v)                              (skimage.color: sRGB gamma, D65/2-degree XYZ, CIE LAB)
//   shadow = mask_u8 / 255 >= 0.5                 (util.img_as_bool; no mask -> every pixel)
//   rmse_s += |lab1 - lab2|_2, mae_s += sum_c |lab1 - lab2|, n_s += 1   over shadow pixels
//   (the same over non-shadow pixels)             (eval.py:87-104, RMSE/MAE at :124-131)
//   sse += sum_c (v1 - v2)^2                      (PSNR = 10 log10(1 / (sse / (3 H W))), :134-136)
// One workgroup reduces a pixel range of one image to 7 fp64 sums (fixed order: lanes ->
// wave shuffles -> waves), a second launch adds the per-workgroup partials of each image in
// workgroup order (deterministic).  The colour conversion runs in fp32 (powf for the sRGB gamma,
// cbrtf for the LAB cube root), the sums in fp64.  stc_istd_errors / stc_istd_ssim take both images
// as img_as_float32 uint8 images; the typed entry points (stc_istd_errors_ex, stc_istd_ssim_ex,
// stc_image_resize_f64) follow all_metrics itself, where img2 and the mask are float64 after their
// transform.resize (and every image with ``size``), with skimage's dtype rules in rgb2lab.
#include "common.hpp"

namespace stc {

constexpr int ISTD_SUMS = 7;  // rmse_s, mae_s, n_s, rmse_n, mae_n, n_n, sse

__device__ __forceinline__ float srgb_lin(float c) {
  return c > 0.04045f ? powf((c + 0.055f) / 1.055f, 2.4f) : c / 12.92f;
}
__device__ __forceinline__ float lab_f(float t) { return t > 0.008856f ? cbrtf(t) : 7.787f * t + 16.f / 116.f; }

// skimage.color.rgb2lab (illuminant D65, observer 2): xyz = M * linear(rgb), lab from xyz / white
__device__ __forceinline__ void rgb2lab(float r, float g, float b, float* lab) {
  r = srgb_lin(r); g = srgb_lin(g); b = srgb_lin(b);
  const float x = 0.412453f * r + 0.357580f * g + 0.180423f * b;
  const float y = 0.212671f * r + 0.715160f * g + 0.072169f * b;
  const float z = 0.019334f * r + 0.119193f * g + 0.950227f * b;
  const float fx = lab_f(x / 0.95047f), fy = lab_f(y), fz = lab_f(z / 1.08883f);
  lab[0] = 116.f * fy - 16.f;
  lab[1] = 500.f * (fx - fy);
  lab[2] = 200.f * (fy - fz);
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(256) istd_errors_kernel(const unsigned char* __restrict__ img1,
                                                          const unsigned char* __restrict__ img2,
                                                          const unsigned char* __restrict__ mask, long long HW,
                                                          int pix_per_block, double* __restrict__ part) {
  const int b = blockIdx.y;
  const long long p0 = (long long)blockIdx.x * pix_per_block;
  const long long p1 = min(HW, p0 + pix_per_block);
  const unsigned char* a = img1 + (long long)b * HW * 3;
  const unsigned char* c = img2 + (long long)b * HW * 3;
  const unsigned char* m = mask ? mask + (long long)b * HW : nullptr;
  double s[ISTD_SUMS] = {0, 0, 0, 0, 0, 0, 0};
  constexpr float inv255 = 1.f / 255.f;
  for (long long p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
    const float r1 = a[p * 3] * inv255, g1 = a[p * 3 + 1] * inv255, b1 = a[p * 3 + 2] * inv255;
    const float r2 = c[p * 3] * inv255, g2 = c[p * 3 + 1] * inv255, b2 = c[p * 3 + 2] * inv255;
    float l1[3], l2[3];
    rgb2lab(r1, g1, b1, l1);
    rgb2lab(r2, g2, b2, l2);
    const double d0 = (double)l1[0] - l2[0], d1 = (double)l1[1] - l2[1], d2 = (double)l1[2] - l2[2];
    const double e2 = sqrt(d0 * d0 + d1 * d1 + d2 * d2), e1 = fabs(d0) + fabs(d1) + fabs(d2);
    const bool sh = m ? m[p] >= 128 : true;  // u / 255 >= 0.5
    s[sh ? 0 : 3] += e2;
    s[sh ? 1 : 4] += e1;
    s[sh ? 2 : 5] += 1.0;
    const double q0 = (double)r1 - r2, q1 = (double)g1 - g2, q2 = (double)b1 - b2;
    s[6] += q0 * q0 + q1 * q1 + q2 * q2;
  }
  __shared__ double red[ISTD_SUMS][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < ISTD_SUMS; ++k) {
    const double v = wave_sum_d(s[k]);
    if (lane == 0) red[k][wave] = v;
  }
  __syncthreads();
  if (threadIdx.x < ISTD_SUMS) {
    const int k = threadIdx.x;
    part[((long long)b * gridDim.x + blockIdx.x) * ISTD_SUMS + k] = ((red[k][0] + red[k][1]) + red[k][2]) + red[k][3];
  }
}

__global__ void istd_errors_final_kernel(const double* part, int nblk, int B, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * ISTD_SUMS) return;
  const int b = i / ISTD_SUMS, k = i % ISTD_SUMS;
  double v = 0.0;
  for (int j = 0; j < nblk; ++j) v += part[((long long)b * nblk + j) * ISTD_SUMS + k];
  out[i] = v;
}

// SSIM (skimage 0.17 structural_similarity(X, Y, multichannel=True), eval.py:137-139): 7x7
// uniform windows, sample covariance (49/48), data_range 2 (float dtype range), K1 0.01,
// K2 0.03, float64 statistics; the mean over the interior (the 3-pixel border is cropped, so
// no window leaves the image) of every channel, then over the channels.  One thread per
// interior pixel evaluates its three 7x7 windows directly.
__global__ void __launch_bounds__(256) istd_ssim_kernel(const unsigned char* __restrict__ img1,
                                                        const unsigned char* __restrict__ img2, int H, int W,
                                                        int pix_per_block, double* __restrict__ part) {
  const int b = blockIdx.y;
  const int IW = W - 6;
  const long long NI = (long long)(H - 6) * IW;
  const long long p0 = (long long)blockIdx.x * pix_per_block;
  const long long p1 = min(NI, p0 + pix_per_block);
  const unsigned char* a = img1 + (long long)b * H * W * 3;
  const unsigned char* c = img2 + (long long)b * H * W * 3;
  constexpr float inv255 = 1.f / 255.f;
  constexpr double R = 2.0, C1 = (0.01 * R) * (0.01 * R), C2 = (0.03 * R) * (0.03 * R);
  constexpr double NP = 49.0, cov_norm = NP / (NP - 1.0);
  double acc = 0.0;
  for (long long p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
    const int y = (int)(p / IW) + 3, x = (int)(p % IW) + 3;
    for (int ch = 0; ch < 3; ++ch) {
      double sx = 0, sy = 0, sxx = 0, syy = 0, sxy = 0;
      for (int dy = -3; dy <= 3; ++dy) {
        const long long row = ((long long)(y + dy) * W + (x - 3)) * 3 + ch;
#pragma unroll
        for (int dx = 0; dx < 7; ++dx) {
          const double X = (double)(a[row + dx * 3] * inv255), Y = (double)(c[row + dx * 3] * inv255);
          sx += X; sy += Y; sxx += X * X; syy += Y * Y; sxy += X * Y;
        }
      }
      const double ux = sx / NP, uy = sy / NP, uxx = sxx / NP, uyy = syy / NP, uxy = sxy / NP;
      const double vx = cov_norm * (uxx - ux * ux), vy = cov_norm * (uyy - uy * uy), vxy = cov_norm * (uxy - ux * uy);
      const double A1 = 2 * ux * uy + C1, A2 = 2 * vxy + C2, B1 = ux * ux + uy * uy + C1, B2 = vx + vy + C2;
      acc += (A1 * A2) / (B1 * B2);
    }
  }
  acc = wave_sum_d(acc);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[(long long)b * gridDim.x + blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ void istd_ssim_final_kernel(const double* part, int nblk, int B, double denom, double* out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double v = 0.0;
  for (int j = 0; j < nblk; ++j) v += part[(long long)b * nblk + j];
  out[b] = v / denom;
}


// ---------------------------------------------------------------------------------------------
// Typed images for the reference's resize branches (eval.py:64-81).  kind:
//   STC_IMG_U8F32 (0): uint8 [H][W][C] read as util.img_as_float32: float32(u) * float32(1/255)
//   STC_IMG_U8F64 (1): uint8 [H][W][C] read as util.img_as_float:   u * (1/255) in float64
//   STC_IMG_F64   (2): float64 [H][W][C]
// skimage keeps an image's float dtype through rgb2lab's sRGB gamma (float32 for img_as_float32
// images, float64 for transform.resize outputs) and computes in float64 from the xyz matrix product.
__device__ __forceinline__ double img_val(const void* p, int kind, long long i) {
  if (kind == 2) return reinterpret_cast<const double*>(p)[i];
  const unsigned u = reinterpret_cast<const unsigned char*>(p)[i];
  if (kind == 1) return (double)u * (1.0 / 255.0);
  return (double)((float)u * (1.f / 255.f));
}

// skimage rgb2lab with the gamma in float32 (f32 = true) or float64, float64 afterwards
__device__ __forceinline__ void rgb2lab_typed(double r, double g, double b, bool f32, double* lab) {
  double lin[3];
  const double v[3] = {r, g, b};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (f32) {
      const float c = (float)v[k];
      lin[k] = (double)(c > 0.04045f ? powf((c + 0.055f) / 1.055f, 2.4f) : c / 12.92f);
    } else {
      const double c = v[k];
      lin[k] = c > 0.04045 ? pow((c + 0.055) / 1.055, 2.4) : c / 12.92;
    }
  }
  // arr @ xyz_from_rgb.T (float64), / D65 white, cube root / linear segment
  const double x = (0.412453 * lin[0] + 0.357580 * lin[1]) + 0.180423 * lin[2];
  const double y = (0.212671 * lin[0] + 0.715160 * lin[1]) + 0.072169 * lin[2];
  const double z = (0.019334 * lin[0] + 0.119193 * lin[1]) + 0.950227 * lin[2];
  double t[3] = {x / 0.95047, y / 1.0, z / 1.08883};
#pragma unroll
  for (int k = 0; k < 3; ++k) t[k] = t[k] > 0.008856 ? cbrt(t[k]) : 7.787 * t[k] + 16.0 / 116.0;
  lab[0] = 116.0 * t[1] - 16.0;
  lab[1] = 500.0 * (t[0] - t[1]);
  lab[2] = 200.0 * (t[1] - t[2]);
}

__global__ void __launch_bounds__(256) istd_errors_typed_kernel(const void* __restrict__ img1, int k1,
                                                                const void* __restrict__ img2, int k2,
                                                                const double* __restrict__ mask, long long HW,
                                                                int pix_per_block, double* __restrict__ part) {
  const long long p0 = (long long)blockIdx.x * pix_per_block;
  const long long p1 = min(HW, p0 + pix_per_block);
  double s[ISTD_SUMS] = {0, 0, 0, 0, 0, 0, 0};
  for (long long p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
    const double r1 = img_val(img1, k1, p * 3), g1 = img_val(img1, k1, p * 3 + 1), b1 = img_val(img1, k1, p * 3 + 2);
    const double r2 = img_val(img2, k2, p * 3), g2 = img_val(img2, k2, p * 3 + 1), b2 = img_val(img2, k2, p * 3 + 2);
    double l1[3], l2[3];
    rgb2lab_typed(r1, g1, b1, k1 == 0, l1);
    rgb2lab_typed(r2, g2, b2, k2 == 0, l2);
    const double d0 = l1[0] - l2[0], d1 = l1[1] - l2[1], d2 = l1[2] - l2[2];
    const double e2 = sqrt((d0 * d0 + d1 * d1) + d2 * d2), e1 = (fabs(d0) + fabs(d1)) + fabs(d2);
    const bool sh = mask ? mask[p] > 0.5 : true;  // util.img_as_bool of a float mask
    s[sh ? 0 : 3] += e2;
    s[sh ? 1 : 4] += e1;
    s[sh ? 2 : 5] += 1.0;
    const double q0 = r1 - r2, q1 = g1 - g2, q2 = b1 - b2;
    s[6] += q0 * q0 + q1 * q1 + q2 * q2;
  }
  __shared__ double red[ISTD_SUMS][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < ISTD_SUMS; ++k) {
    const double v = wave_sum_d(s[k]);
    if (lane == 0) red[k][wave] = v;
  }
  __syncthreads();
  if (threadIdx.x < ISTD_SUMS) {
    const int k = threadIdx.x;
    part[(long long)blockIdx.x * ISTD_SUMS + k] = ((red[k][0] + red[k][1]) + red[k][2]) + red[k][3];
  }
}

__global__ void __launch_bounds__(256) istd_ssim_typed_kernel(const void* __restrict__ img1, int k1,
                                                              const void* __restrict__ img2, int k2, int H, int W,
                                                              int pix_per_block, double* __restrict__ part) {
  const int IW = W - 6;
  const long long NI = (long long)(H - 6) * IW;
  const long long p0 = (long long)blockIdx.x * pix_per_block;
  const long long p1 = min(NI, p0 + pix_per_block);
  constexpr double R = 2.0, C1 = (0.01 * R) * (0.01 * R), C2 = (0.03 * R) * (0.03 * R);
  constexpr double NP = 49.0, cov_norm = NP / (NP - 1.0);
  double acc = 0.0;
  for (long long p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
    const int y = (int)(p / IW) + 3, x = (int)(p % IW) + 3;
    for (int ch = 0; ch < 3; ++ch) {
      double sx = 0, sy = 0, sxx = 0, syy = 0, sxy = 0;
      for (int dy = -3; dy <= 3; ++dy) {
        const long long row = ((long long)(y + dy) * W + (x - 3)) * 3 + ch;
#pragma unroll
        for (int dx = 0; dx < 7; ++dx) {
          const double X = img_val(img1, k1, row + dx * 3), Y = img_val(img2, k2, row + dx * 3);
          sx += X; sy += Y; sxx += X * X; syy += Y * Y; sxy += X * Y;
        }
      }
      const double ux = sx / NP, uy = sy / NP, uxx = sxx / NP, uyy = syy / NP, uxy = sxy / NP;
      const double vx = cov_norm * (uxx - ux * ux), vy = cov_norm * (uyy - uy * uy), vxy = cov_norm * (uxy - ux * uy);
      const double A1 = 2 * ux * uy + C1, A2 = 2 * vxy + C2, B1 = ux * ux + uy * uy + C1, B2 = vx + vy + C2;
      acc += (A1 * A2) / (B1 * B2);
    }
  }
  acc = wave_sum_d(acc);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

// scipy.ndimage.gaussian_filter1d, mode 'nearest', along rows (axis 0) or columns (axis 1) of a
// float64 [H][W][C] image: the symmetric-kernel order of NI_Correlate1D,
//   out = in[0]*w[0] + sum_{j = r..1} (in[-j] + in[+j]) * w[j]   (outermost pair first)
__global__ void __launch_bounds__(256) gauss1d_kernel(const double* __restrict__ src, double* __restrict__ dst, int H,
                                                      int W, int C, int axis, const double* __restrict__ w,
                                                      int radius) {
  const long long n = (long long)H * W * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long pix = i / C;
    const int x = (int)(pix % W), y = (int)(pix / W);
    auto at = [&](int yy, int xx) {
      yy = min(max(yy, 0), H - 1);
      xx = min(max(xx, 0), W - 1);
      return src[((long long)yy * W + xx) * C + c];
    };
    double acc = at(y, x) * w[0];
    for (int j = radius; j >= 1; --j) {
      const double a = axis == 0 ? at(y - j, x) : at(y, x - j);
      const double b = axis == 0 ? at(y + j, x) : at(y, x + j);
      acc += (a + b) * w[j];
    }
    dst[i] = acc;
  }
}

// skimage transform.resize order 1, mode 'edge' (_warp_fast bilinear, float64): for output (r, c),
// row_in = s_r*r + (0.5*s_r - 0.5), col_in likewise, taps at floor / ceil clamped to the image
__global__ void __launch_bounds__(256) resize_bilinear_f64_kernel(const void* __restrict__ src, int kind, int H, int W,
                                                                  int C, int OH, int OW, double sr, double sc,
                                                                  double* __restrict__ dst) {
  const long long n = (long long)OH * OW * C;
  const double tr = 0.5 * sr - 0.5, tc = 0.5 * sc - 0.5;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(i % C);
    const long long pix = i / C;
    const int oc = (int)(pix % OW), orow = (int)(pix / OW);
    const double r = sr * orow + tr, c = sc * oc + tc;
    const double fr = floor(r), fc = floor(c);
    const int r0 = (int)fr, c0 = (int)fc, r1 = (int)ceil(r), c1 = (int)ceil(c);
    const double dr = r - fr, dc = c - fc;
    auto at = [&](int yy, int xx) {
      yy = min(max(yy, 0), H - 1);
      xx = min(max(xx, 0), W - 1);
      return img_val(src, kind, ((long long)yy * W + xx) * C + ch);
    };
    const double top = (1 - dc) * at(r0, c0) + dc * at(r0, c1);
    const double bottom = (1 - dc) * at(r1, c0) + dc * at(r1, c1);
    dst[i] = (1 - dr) * top + dr * bottom;
  }
}

__global__ void istd_sum_parts_kernel(const double* part, int nblk, int stride, int n, double* out, double scale) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  double v = 0.0;
  for (int j = 0; j < nblk; ++j) v += part[(long long)j * stride + k];
  out[k] = v * scale;
}

static int istd_blocks(long long HW, int* ppb) {
  const int nblk = (int)std::min<long long>(256, std::max<long long>(1, (HW + 1023) / 1024));
  *ppb = (int)((HW + nblk - 1) / nblk);
  return nblk;
}

}  // namespace stc

using namespace stc;

extern "C" int64_t stc_istd_errors_workspace(int B, int H, int W) {
  int ppb;
  const int nblk = istd_blocks((long long)H * W, &ppb);
  return (int64_t)B * nblk * ISTD_SUMS * (int64_t)sizeof(double);
}

extern "C" int stc_istd_errors(const unsigned char* img1, const unsigned char* img2, const unsigned char* mask, int B,
                               int H, int W, double* out, void* ws, int64_t ws_bytes, void* stream) {
  STC_REQUIRE(B >= 0 && H >= 1 && W >= 1, "stc_istd_errors: bad shape B=%d H=%d W=%d", B, H, W);
  if (B == 0) return 0;
  STC_REQUIRE(img1 && img2 && out && ws, "stc_istd_errors: null pointer");
  STC_REQUIRE(ws_bytes >= stc_istd_errors_workspace(B, H, W), "stc_istd_errors: workspace %lld < %lld",
              (long long)ws_bytes, (long long)stc_istd_errors_workspace(B, H, W));
  const long long HW = (long long)H * W;
  int ppb;
  const int nblk = istd_blocks(HW, &ppb);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(istd_errors_kernel, dim3(nblk, B), dim3(256), 0, st, img1, img2, mask, HW, ppb, (double*)ws);
  STC_CHECK_LAUNCH();
  hipLaunchKernelGGL(istd_errors_final_kernel, dim3((B * ISTD_SUMS + 255) / 256), dim3(256), 0, st,
                     (const double*)ws, nblk, B, out);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_istd_ssim(const unsigned char* img1, const unsigned char* img2, int B, int H, int W, double* out,
                             void* ws, int64_t ws_bytes, void* stream) {
  STC_REQUIRE(B >= 0 && H >= 7 && W >= 7, "stc_istd_ssim: bad shape B=%d H=%d W=%d (needs >= 7x7)", B, H, W);
  if (B == 0) return 0;
  STC_REQUIRE(img1 && img2 && out && ws, "stc_istd_ssim: null pointer");
  STC_REQUIRE(ws_bytes >= stc_istd_errors_workspace(B, H, W), "stc_istd_ssim: workspace %lld too small",
              (long long)ws_bytes);
  const long long NI = (long long)(H - 6) * (W - 6);
  int ppb;
  const int nblk = istd_blocks(NI, &ppb);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(istd_ssim_kernel, dim3(nblk, B), dim3(256), 0, st, img1, img2, H, W, ppb, (double*)ws);
  STC_CHECK_LAUNCH();
  hipLaunchKernelGGL(istd_ssim_final_kernel, dim3((B + 255) / 256), dim3(256), 0, st, (const double*)ws, nblk, B,
                     3.0 * (double)NI, out);
  STC_CHECK_LAUNCH();
  return 0;
}

// ---- typed entry points (eval.py:64-81 resize branches) ----------------------------------------

extern "C" int64_t stc_istd_typed_workspace(int H, int W) {
  int ppb;
  const int nblk = istd_blocks((long long)H * W, &ppb);
  const int64_t parts = (int64_t)nblk * ISTD_SUMS * (int64_t)sizeof(double);
  const int64_t img = (int64_t)H * W * 3 * (int64_t)sizeof(double);  // one float64 temporary (gaussian pass)
  return std::max(parts, img) + 64;
}

extern "C" int stc_istd_errors_ex(const void* img1, int kind1, const void* img2, int kind2, const double* mask, int H,
                                  int W, double* out, void* ws, int64_t ws_bytes, void* stream) {
  STC_REQUIRE(H >= 1 && W >= 1 && img1 && img2 && out && ws, "stc_istd_errors_ex: bad arguments");
  STC_REQUIRE((kind1 == 0 || kind1 == 2) && (kind2 == 0 || kind2 == 2),
              "stc_istd_errors_ex: images are STC_IMG_U8F32 or STC_IMG_F64");
  STC_REQUIRE(ws_bytes >= stc_istd_typed_workspace(H, W), "stc_istd_errors_ex: workspace too small");
  const long long HW = (long long)H * W;
  int ppb;
  const int nblk = istd_blocks(HW, &ppb);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(istd_errors_typed_kernel, dim3(nblk), dim3(256), 0, st, img1, kind1, img2, kind2, mask, HW, ppb,
                     (double*)ws);
  STC_CHECK_LAUNCH();
  hipLaunchKernelGGL(istd_sum_parts_kernel, dim3(1), dim3(64), 0, st, (const double*)ws, nblk, ISTD_SUMS, ISTD_SUMS,
                     out, 1.0);
  STC_CHECK_LAUNCH();
  return 0;
}

extern "C" int stc_istd_ssim_ex(const void* img1, int kind1, const void* img2, int kind2, int H, int W, double* out,
                                void* ws, int64_t ws_bytes, void* stream) {
  STC_REQUIRE(H >= 7 && W >= 7 && img1 && img2 && out && ws, "stc_istd_ssim_ex: bad arguments (needs >= 7x7)");
  STC_REQUIRE((kind1 == 0 || kind1 == 2) && (kind2 == 0 || kind2 == 2), "stc_istd_ssim_ex: bad image kind");
  STC_REQUIRE(ws_bytes >= stc_istd_typed_workspace(H, W), "stc_istd_ssim_ex: workspace too small");
  const long long NI = (long long)(H - 6) * (W - 6);
  int ppb;
  const int nblk = istd_blocks(NI, &ppb);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(istd_ssim_typed_kernel, dim3(nblk), dim3(256), 0, st, img1, kind1, img2, kind2, H, W, ppb,
                     (double*)ws);
  STC_CHECK_LAUNCH();
  hipLaunchKernelGGL(istd_sum_parts_kernel, dim3(1), dim3(64), 0, st, (const double*)ws, nblk, 1, 1, out,
                     1.0 / (3.0 * (double)NI));
  STC_CHECK_LAUNCH();
  return 0;
}

// transform.resize(img, (OH, OW), mode="edge", anti_aliasing=anti_alias) -> float64 [OH][OW][C].
// anti_alias: scipy gaussian_filter (sigma = max(0, (in/out - 1) / 2) per axis, mode 'nearest',
// truncate 4) before the bilinear warp; weights computed here as scipy's _gaussian_kernel1d does.
// ws: >= stc_image_resize_workspace(H, W, C) bytes.
extern "C" int64_t stc_image_resize_workspace(int H, int W, int C) {
  return 2 * (int64_t)H * W * C * (int64_t)sizeof(double) + 2 * 64 * (int64_t)sizeof(double) + 256;
}

extern "C" int stc_image_resize_f64(const void* src, int kind, int H, int W, int C, int OH, int OW, int anti_alias,
                                    double* dst, void* ws, int64_t ws_bytes, void* stream) {
  STC_REQUIRE(src && dst && H >= 1 && W >= 1 && C >= 1 && OH >= 1 && OW >= 1 && kind >= 0 && kind <= 2,
              "stc_image_resize_f64: bad arguments");
  const double sr = (double)H / OH, sc = (double)W / OW;
  hipStream_t st = (hipStream_t)stream;
  const void* in = src;
  int in_kind = kind;
  const double sig[2] = {std::max(0.0, (sr - 1) / 2), std::max(0.0, (sc - 1) / 2)};
  if (anti_alias && (sig[0] > 1e-15 || sig[1] > 1e-15)) {
    STC_REQUIRE(ws && ws_bytes >= stc_image_resize_workspace(H, W, C), "stc_image_resize_f64: workspace too small");
    const long long n = (long long)H * W * C;
    double* a = reinterpret_cast<double*>(ws);
    double* b = a + n;
    double* wdev = b + n;  // 2 x 64 weights
    // float64 copy of the source (kind conversion), then one pass per axis with sigma > 1e-15
    hipLaunchKernelGGL(resize_bilinear_f64_kernel, dim3((unsigned)std::min<long long>((n + 255) / 256, 4096)),
                       dim3(256), 0, st, src, kind, H, W, C, H, W, 1.0, 1.0, a);
    STC_CHECK_LAUNCH();
    double hw[2][64];
    int rad[2] = {0, 0};
    for (int ax = 0; ax < 2; ++ax) {
      if (sig[ax] <= 1e-15) continue;
      const int r = (int)(4.0 * sig[ax] + 0.5);
      STC_REQUIRE(r < 64, "stc_image_resize_f64: gaussian radius %d too large", r);
      rad[ax] = r;
      const double c2 = -0.5 / (sig[ax] * sig[ax]);
      double sum = 0;
      double phi[129];
      for (int x = -r; x <= r; ++x) { phi[x + r] = std::exp((c2 * x) * x); sum += phi[x + r]; }
      for (int j = 0; j <= r; ++j) hw[ax][j] = phi[r + j] / sum;
    }
    // (pageable source: the copy is staged before the call returns; stream-ordered before the passes)
    STC_REQUIRE(hipMemcpyAsync(wdev, hw, sizeof(hw), hipMemcpyHostToDevice, st) == hipSuccess,
                "stc_image_resize_f64: weight upload failed");
    double* cur = a;
    double* nxt = b;
    for (int ax = 0; ax < 2; ++ax) {
      if (sig[ax] <= 1e-15) continue;
      hipLaunchKernelGGL(gauss1d_kernel, dim3((unsigned)std::min<long long>((n + 255) / 256, 4096)), dim3(256), 0, st,
                         cur, nxt, H, W, C, ax, wdev + 64 * ax, rad[ax]);
      STC_CHECK_LAUNCH();
      std::swap(cur, nxt);
    }
    in = cur;
    in_kind = 2;
  }
  const long long m = (long long)OH * OW * C;
  hipLaunchKernelGGL(resize_bilinear_f64_kernel, dim3((unsigned)std::min<long long>((m + 255) / 256, 4096)), dim3(256),
                     0, st, in, in_kind, H, W, C, OH, OW, sr, sc, dst);
  STC_CHECK_LAUNCH();
  return 0;
}
