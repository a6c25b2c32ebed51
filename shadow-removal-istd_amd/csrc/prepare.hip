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
// call order and passed per image as {flip, row_offset, col_offset}.  Resize / RandomScale /
// RandomRotate (cv.resize / cv.warpAffine) are not restated.
#include "common.hpp"

#pragma clang fp contract(off)  // (u / 255 - 0.5) * 2 rounded step by step, as numpy does

namespace stc {

__global__ void __launch_bounds__(256) prepare_kernel(const unsigned char* __restrict__ src, int B, int H, int W,
                                                      int C, const int* __restrict__ params, int pad_h, int pad_w,
                                                      int OH, int OW, float* __restrict__ dst) {
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
      const float u = (float)src[(((long long)b * H + Y) * W + sx) * C + c];
      v = (u / 255.f - 0.5f) * 2.f;
    }
    dst[i] = v;
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
  hipLaunchKernelGGL(prepare_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, src, B, H, W, C, params, pad_h,
                     pad_w, OH, OW, dst);
  STC_CHECK_LAUNCH();
  return 0;
}
