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
// cbrtf for the LAB cube root), the sums in fp64.
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
