// Serving-path pre/post-processing kernels (per frame, graph-capturable).
//
// preprocess: replaces torchvision ToTensor() + Resize((256,256), antialias=True) + BGR->RGB (or RGB
//   input as decoded by the server, rgb = 1) of
//   /root/reference/services/vision_analysis/server.py:107-110,120-121: u8 BGR HWC -> /255 ->
//   antialiased bilinear (triangle filter, support = scale, normalized weights, torch
//   _upsample_bilinear2d_aa semantics; weight tables precomputed on the host) -> bf16 NHWC with
//   8 channels (3 RGB + 5 zero) = the packed first-layer input of the native U-Net.
// mask_upsample: replaces (sigmoid(logits) > 0.5) -> cv2.resize(INTER_NEAREST) -> count_nonzero
//   (server.py:124-125,133): u8 {0,1} mask at the camera resolution + coverage count (atomics).
#include "common.h"

#define AA_MAXTAP 16

struct AATable {  // per output index: first input index, number of taps, weights
  int start[256];
  int size[256];
  float w[256][AA_MAXTAP];
};

__global__ void preprocess_kernel(const uint8_t* __restrict__ bgr, int H, int W, const int* __restrict__ ystart,
                                  const int* __restrict__ ysize, const float* __restrict__ yw,
                                  const int* __restrict__ xstart, const int* __restrict__ xsize,
                                  const float* __restrict__ xw, int OH, int OW, int rgb, u16* __restrict__ out) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= OH * OW) return;
  const int oy = o / OW, ox = o - oy * OW;
  const int y0 = ystart[oy], ny = ysize[oy], x0 = xstart[ox], nx = xsize[ox];
  float r = 0.f, g = 0.f, b = 0.f;
  for (int j = 0; j < ny; ++j) {
    const float wy = yw[oy * AA_MAXTAP + j];
    const uint8_t* row = bgr + ((size_t)(y0 + j) * W + x0) * 3;
    float rr = 0.f, gg = 0.f, bb = 0.f;
    for (int i = 0; i < nx; ++i) {
      const float wx = xw[ox * AA_MAXTAP + i];
      bb += wx * (float)row[i * 3 + 0];
      gg += wx * (float)row[i * 3 + 1];
      rr += wx * (float)row[i * 3 + 2];
    }
    r += wy * rr;
    g += wy * gg;
    b += wy * bb;
  }
  if (rgb) {  // input already RGB (the server decodes JPEG straight to RGB): channels 0 / 2 swap roles
    const float t = r;
    r = b;
    b = t;
  }
  const float inv = 1.0f / 255.0f;
  uint4 v;
  v.x = pack2bf(r * inv, g * inv);
  v.y = pack2bf(b * inv, 0.f);
  v.z = 0u;
  v.w = 0u;
  *(uint4*)(out + (size_t)o * 8) = v;
}

// nearest upsample of the model-resolution mask to (H, W) + coverage count.
// src index = min(floor(dst * (in/out)), in-1) in double, like cv::resize INTER_NEAREST.
__global__ void mask_upsample_kernel(const uint8_t* __restrict__ m, int mh, int mw, uint8_t* __restrict__ out,
                                     int H, int W, double sy, double sx, unsigned* __restrict__ count) {
  __shared__ unsigned wc[4];
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned v = 0;
  if (p < H * W) {
    const int y = p / W, x = p - y * W;
    int iy = (int)floor((double)y * sy), ix = (int)floor((double)x * sx);
    iy = min(iy, mh - 1);
    ix = min(ix, mw - 1);
    v = m[iy * mw + ix];
    out[p] = (uint8_t)v;
  }
  // block count -> one atomic per block
  unsigned long long b = __ballot(v != 0);
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = (unsigned)__popcll(b);
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(count, wc[0] + wc[1] + wc[2] + wc[3]);
}

__global__ void zero_u32_kernel(unsigned* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0;
}

extern "C" {
int rdp_preprocess(const void* bgr, int H, int W, const int* ystart, const int* ysize, const float* yw,
                   const int* xstart, const int* xsize, const float* xw, int OH, int OW, int rgb, void* out,
                   hipStream_t s) {
  const int n = OH * OW;
  hipLaunchKernelGGL(preprocess_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const uint8_t*)bgr, H, W, ystart,
                     ysize, yw, xstart, xsize, xw, OH, OW, rgb, (u16*)out);
  return 0;
}

int rdp_mask_upsample(const void* m, int mh, int mw, void* out, int H, int W, unsigned* count, hipStream_t s) {
  hipLaunchKernelGGL(zero_u32_kernel, dim3(1), dim3(64), 0, s, count, 1);
  const double sy = 1.0 / ((double)H / (double)mh), sx = 1.0 / ((double)W / (double)mw);
  hipLaunchKernelGGL(mask_upsample_kernel, dim3((H * W + 255) / 256), dim3(256), 0, s, (const uint8_t*)m, mh, mw,
                     (uint8_t*)out, H, W, sy, sx, count);
  return 0;
}
}
