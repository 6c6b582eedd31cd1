// CLIP image preprocessing on the GPU (the image half of the data step).
//
// Replaces `processor(images=torch.stack(images), ...)` in the reference's prompt builders
// (cullavo/arch_cullavo.py:82,313,516): CLIPImageProcessor with do_resize (shortest edge 336,
// PIL bicubic), do_center_crop (336x336), do_rescale (1/255) and do_normalize (OpenAI CLIP mean /
// std), producing pixel_values [B, 3, 336, 336]. The arithmetic restated here is
//   * Pillow's separable resampler (third-party, installed here as Pillow 12.2; libImaging
//     Resample.c: precompute_coeffs, bicubic_filter with a = -0.5 and support 2, 22-bit
//     fixed-point coefficients, horizontal pass into a uint8 image, then the vertical pass);
//   * transformers' image_transforms: output size int(336 * long / short), center-crop offsets
//     (orig - crop) // 2, rescale float32(float64(u) * scale), normalize float32((x - mean) / std).
// The result is bit-identical to the CPU processor (tests/test_imageprep.py, fixtures made by
// tests/golden/make_golden_data.py with transformers' CLIPImageProcessorPil).
//
// Layout: images uint8 [B, C, H, W] with arbitrary element strides (CHW tensors as the
// reference's dataset mapper yields, or HWC numpy images); out [B, C, crop_h, crop_w] f32/bf16.
// Two HBM-bound passes. Pass 1 computes the horizontally resampled uint8 image only for the
// columns the crop keeps (all H source rows); pass 2 resamples vertically only the kept rows and
// writes the normalised value. Coefficient tables (a few KB) come from
// cullavo_resample_coeffs on the host, exactly as Pillow computes them.
#include "common.h"

#include <cmath>

namespace {

constexpr int kPrecisionBits = 32 - 8 - 2;  // Pillow Resample.c PRECISION_BITS

DEV uint8_t clip8(int32_t ss) {  // Pillow clip8: (ss >> 22) clamped to [0, 255]
  const int32_t v = ss >> kPrecisionBits;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// pass 1: tmp[b][c][y][ox] = horizontal resample of source row y at resized column left + ox
__global__ __launch_bounds__(256) void resample_h_k(const uint8_t* __restrict__ img, int64_t sb, int64_t sc,
                                                    int64_t sy, int64_t sx, int C, int H,
                                                    const int32_t* __restrict__ bounds,
                                                    const int32_t* __restrict__ kk, int ksize, int left,
                                                    int crop_w, uint8_t* __restrict__ tmp) {
  const int ox = blockIdx.x * 256 + threadIdx.x;
  const int64_t row = blockIdx.y;  // (b * C + c) * H + y
  if (ox >= crop_w) return;
  const int y = (int)(row % H);
  const int64_t bc = row / H;
  const int c = (int)(bc % C), b = (int)(bc / C);
  const int xx = left + ox;
  const int xmin = bounds[2 * xx], xn = bounds[2 * xx + 1];
  const int32_t* k = kk + (int64_t)xx * ksize;
  const uint8_t* src = img + b * sb + c * sc + y * sy + xmin * sx;
  int32_t ss = 1 << (kPrecisionBits - 1);
  for (int x = 0; x < xn; ++x) ss += (int32_t)src[x * sx] * k[x];
  tmp[row * crop_w + ox] = clip8(ss);
}

// pass 2: vertical resample of kept row top + oy, then rescale + normalise
template <typename TO>
__global__ __launch_bounds__(256) void resample_v_norm_k(const uint8_t* __restrict__ tmp, int C, int H,
                                                         const int32_t* __restrict__ bounds,
                                                         const int32_t* __restrict__ kk, int ksize, int top,
                                                         int crop_h, int crop_w, double rescale, float m0,
                                                         float m1, float m2, float s0, float s1, float s2,
                                                         TO* __restrict__ out) {
  const int ox = blockIdx.x * 256 + threadIdx.x;
  const int64_t orow = blockIdx.y;  // (b * C + c) * crop_h + oy
  if (ox >= crop_w) return;
  const int oy = (int)(orow % crop_h);
  const int64_t bc = orow / crop_h;
  const int c = (int)(bc % C);
  const int yy = top + oy;
  const int ymin = bounds[2 * yy], yn = bounds[2 * yy + 1];
  const int32_t* k = kk + (int64_t)yy * ksize;
  const uint8_t* src = tmp + (bc * H + ymin) * crop_w + ox;
  int32_t ss = 1 << (kPrecisionBits - 1);
  for (int y = 0; y < yn; ++y) ss += (int32_t)src[(int64_t)y * crop_w] * k[y];
  const uint8_t u = clip8(ss);
  // transformers rescale: float32(float64(u) * scale); normalize: float32 (x - mean) / std
  const float x = (float)((double)u * rescale);
  const float mean = c == 0 ? m0 : (c == 1 ? m1 : m2);
  const float stdv = c == 0 ? s0 : (c == 1 ? s1 : s2);
  const float v = __fdiv_rn(__fsub_rn(x, mean), stdv);
  Elt<TO>::st(out, orow * crop_w + ox, v);
}

#pragma clang fp contract(off)
// Pillow bicubic_filter (a = -0.5), evaluated in double without contraction like the C original
double bicubic(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

}  // namespace

extern "C" int cullavo_resample_coeffs(int in_size, int out_size, int32_t* bounds, int32_t* kk, int ksize_cap) {
  CV_REQUIRE(in_size > 0 && out_size > 0, CULLAVO_EINVAL, "resample sizes must be positive");
  // Pillow precompute_coeffs with in0 = 0, in1 = in_size (no box)
  const double scale = (double)((float)in_size - 0.0f) / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  const int ksize = (int)std::ceil(support) * 2 + 1;
  if (bounds == nullptr || kk == nullptr) return ksize;  // size query
  CV_REQUIRE(ksize <= ksize_cap, CULLAVO_EINVAL, "resample coefficient buffer too small");
  double w[1024];
  CV_REQUIRE(ksize <= 1024, CULLAVO_EUNSUPPORTED, "downscale factor too large for the resampler");
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = 0.0 + (xx + 0.5) * scale;
    double ww = 0.0;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    int x = 0;
    for (; x < xmax; ++x) {
      w[x] = bicubic((x + xmin - center + 0.5) * ss);
      ww += w[x];
    }
    for (x = 0; x < xmax; ++x)
      if (ww != 0.0) w[x] /= ww;
    for (; x < ksize; ++x) w[x] = 0;
    // Pillow normalize_coeffs_8bpc
    for (x = 0; x < ksize; ++x)
      kk[(int64_t)xx * ksize + x] = w[x] < 0 ? (int32_t)(-0.5 + w[x] * (1 << kPrecisionBits))
                                             : (int32_t)(0.5 + w[x] * (1 << kPrecisionBits));
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  return ksize;
}
#pragma clang fp contract(on)

extern "C" int cullavo_clip_image_preprocess(const uint8_t* images, int B, int C, int H, int W, int64_t sb,
                                             int64_t sc, int64_t sy, int64_t sx, int Hr, int Wr,
                                             const int32_t* h_bounds, const int32_t* h_kk, int h_ksize,
                                             const int32_t* v_bounds, const int32_t* v_kk, int v_ksize, int top,
                                             int left, int crop_h, int crop_w, double rescale, float mean0,
                                             float mean1, float mean2, float std0, float std1, float std2,
                                             uint8_t* tmp, void* out, int out_dtype, void* stream) {
  CV_REQUIRE(B >= 0 && H > 0 && W > 0 && C >= 1 && C <= 3, CULLAVO_EINVAL, "images must be [B, 1..3, H, W]");
  CV_REQUIRE(top >= 0 && left >= 0 && top + crop_h <= Hr && left + crop_w <= Wr && crop_h > 0 && crop_w > 0,
             CULLAVO_EINVAL, "crop window outside the resized image");
  CV_REQUIRE(out_dtype == CULLAVO_DT_F32 || out_dtype == CULLAVO_DT_BF16, CULLAVO_EUNSUPPORTED,
             "pixel_values dtype must be f32 or bf16");
  if (B == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  const dim3 g1((unsigned)cdiv(crop_w, 256), (unsigned)((int64_t)B * C * H));
  resample_h_k<<<g1, 256, 0, s>>>(images, sb, sc, sy, sx, C, H, h_bounds, h_kk, h_ksize, left, crop_w, tmp);
  const dim3 g2((unsigned)cdiv(crop_w, 256), (unsigned)((int64_t)B * C * crop_h));
  if (out_dtype == CULLAVO_DT_F32)
    resample_v_norm_k<float><<<g2, 256, 0, s>>>(tmp, C, H, v_bounds, v_kk, v_ksize, top, crop_h, crop_w, rescale,
                                                mean0, mean1, mean2, std0, std1, std2, (float*)out);
  else
    resample_v_norm_k<u16><<<g2, 256, 0, s>>>(tmp, C, H, v_bounds, v_kk, v_ksize, top, crop_h, crop_w, rescale,
                                              mean0, mean1, mean2, std0, std1, std2, (u16*)out);
  return cullavo_check_launch("clip_image_preprocess");
}
