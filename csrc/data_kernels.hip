// Training-data kernels: the per-sample resizes of the reference's SegmentationDataset on the GPU.
//
// /root/reference/scripts/train_segmenter.py:84-90 loads each colour image, converts BGR -> RGB and
// resizes it with cv2.INTER_AREA to 256x256, and resizes the mask with INTER_NEAREST -- per sample,
// on the host, every epoch. Here the decoded full-size u8 images are uploaded once and resized on the
// device into a device-resident u8 dataset (3 x 256 x 256 B = 192 KiB per sample: a million samples
// fit in 288 GB of HBM), so epochs gather batches on the GPU with no host work at all.
//
// resize_area_u8: separable INTER_AREA (area-overlap weights per output row / column, precomputed on
//   the host exactly as data/image_io.py:_area_weights), fp64 accumulation, round-half-even to u8
//   (numpy rint, the oracle's rounding), optional BGR -> RGB swap; C in {1, 3, 4}.
#include "common.h"

#define AREA_MAXTAP 32

__global__ __launch_bounds__(256) void resize_area_u8_kernel(const uint8_t* __restrict__ in, int h, int w, int C,
                                                             const int* __restrict__ ys, const int* __restrict__ yn,
                                                             const double* __restrict__ yw,
                                                             const int* __restrict__ xs, const int* __restrict__ xn,
                                                             const double* __restrict__ xw, int H, int W, int swap_rb,
                                                             uint8_t* __restrict__ out) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= H * W) return;
  const int oy = o / W, ox = o - oy * W;
  const int y0 = ys[oy], ny = yn[oy], x0 = xs[ox], nx = xn[ox];
  // rows first, then columns: the oracle's order (data/image_io.py:resize_area)
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int i = 0; i < nx; ++i) {
    const double wx = xw[(size_t)ox * AREA_MAXTAP + i];
    double col[4] = {0.0, 0.0, 0.0, 0.0};
    for (int j = 0; j < ny; ++j) {
      const double wy = yw[(size_t)oy * AREA_MAXTAP + j];
      const uint8_t* px = in + ((size_t)(y0 + j) * w + x0 + i) * C;
      for (int c = 0; c < C; ++c) col[c] += wy * (double)px[c];
    }
    for (int c = 0; c < C; ++c) acc[c] += wx * col[c];
  }
  uint8_t* dst = out + (size_t)o * C;
  for (int c = 0; c < C; ++c) {
    const int sc = (swap_rb && C >= 3 && c < 3) ? 2 - c : c;
    const double v = rint(acc[sc]);
    dst[c] = (uint8_t)(v < 0.0 ? 0.0 : (v > 255.0 ? 255.0 : v));
  }
}

extern "C" {
int rdp_area_maxtap() { return AREA_MAXTAP; }

int rdp_resize_area_u8(const void* in, int h, int w, int C, const int* ys, const int* yn, const double* yw,
                       const int* xs, const int* xn, const double* xw, int H, int W, int swap_rb, void* out,
                       hipStream_t s) {
  if (C < 1 || C > 4) return -1;
  const int n = H * W;
  hipLaunchKernelGGL(resize_area_u8_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const uint8_t*)in, h, w, C, ys,
                     yn, yw, xs, xn, xw, H, W, swap_rb, (uint8_t*)out);
  return 0;
}
}
