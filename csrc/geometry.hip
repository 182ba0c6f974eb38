// Curvature-profile geometry kernels: masked depth -> point cloud -> per-bin lower-edge points.
//
// Replaces the NumPy hot loop of /root/reference/pkg/geometry_utils.py:101-142:
//   * deproject: np.where(mask > 0) (row-major order), z = depth*scale, keep z > 0,
//     x = (u-cx) z / fx, y = (v-cy) z / fy in float64                               (:104-117)
//   * edge: x min/max, 50 bins of width (max-min)/50, idx = clip(floor((x-min)/w), 0, 49), per
//     non-empty bin the k = max(1, int(n*0.05)) points with the largest y            (:119-142)
// Determinism: compaction preserves row-major order (per-block counts -> exclusive offsets ->
// in-block ordered scan), and per-bin top-k ties on y are broken by the smaller point index (the
// order a stable descending sort gives), so the selected edge set is exactly defined.
//
// Kernels (all fixed-size launches, graph-capturable):
//   geo_count:   per row-block valid-pixel count + per-block x min/max (double)
//   geo_write:   each block derives its exclusive offset from the counts and writes its points
//   geo_edges:   one workgroup per bin: bin size, k, radix-select of the k-th largest y key,
//                then writes the bin's k points (x, y, z, index) into a per-bin output slab
#include "common.h"
#include <stdint.h>

#define GEO_ROWS_PER_BLOCK 4
#define GEO_THREADS 256

struct GeoCam {
  double fx, fy, cx, cy, scale;
};

RDP_DEV bool pix_valid(const uint8_t* mask, const uint16_t* depth, int p) { return mask[p] > 0 && depth[p] > 0; }

// block-wide exclusive scan of one int per thread (256 threads); returns total
RDP_DEV int block_scan_excl(int v, int* sh, int& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[wave] = x;
  __syncthreads();
  int wsum = 0;
  for (int w = 0; w < wave; ++w) wsum += sh[w];
  total = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return wsum + x - v;
}

__global__ __launch_bounds__(GEO_THREADS) void geo_count_kernel(const uint8_t* __restrict__ mask,
                                                                const uint16_t* __restrict__ depth, int H, int W,
                                                                GeoCam cam, int* __restrict__ counts,
                                                                double* __restrict__ xmin, double* __restrict__ xmax) {
  __shared__ double smin[GEO_THREADS / 64], smax[GEO_THREADS / 64];
  __shared__ int scnt[GEO_THREADS / 64];
  const int r0 = blockIdx.x * GEO_ROWS_PER_BLOCK;
  const int r1 = min(H, r0 + GEO_ROWS_PER_BLOCK);
  int cnt = 0;
  double lo = 1e300, hi = -1e300;
  for (int p = r0 * W + threadIdx.x; p < r1 * W; p += GEO_THREADS) {
    if (pix_valid(mask, depth, p)) {
      ++cnt;
      const int u = p % W;
      const double z = (double)depth[p] * cam.scale;
      const double x = ((double)u - cam.cx) * z / cam.fx;
      lo = fmin(lo, x);
      hi = fmax(hi, x);
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o, 64);
    lo = fmin(lo, __shfl_xor(lo, o, 64));
    hi = fmax(hi, __shfl_xor(hi, o, 64));
  }
  if (lane == 0) { scnt[wave] = cnt; smin[wave] = lo; smax[wave] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    int c = 0;
    double a = 1e300, b = -1e300;
    for (int w = 0; w < GEO_THREADS / 64; ++w) { c += scnt[w]; a = fmin(a, smin[w]); b = fmax(b, smax[w]); }
    counts[blockIdx.x] = c;
    xmin[blockIdx.x] = a;
    xmax[blockIdx.x] = b;
  }
}

// pts: [cap][4] doubles (x, y, z, index) ; npts[0] = total count (written by the last block's thread 0)
__global__ __launch_bounds__(GEO_THREADS) void geo_write_kernel(const uint8_t* __restrict__ mask,
                                                                const uint16_t* __restrict__ depth, int H, int W,
                                                                GeoCam cam, const int* __restrict__ counts,
                                                                int nblocks, double* __restrict__ pts, int cap,
                                                                int* __restrict__ npts) {
  __shared__ int sh[GEO_THREADS / 64];
  __shared__ int base_sh;
  if (threadIdx.x == 0) {
    int b = 0;
    for (int i = 0; i < (int)blockIdx.x; ++i) b += counts[i];
    base_sh = b;
    if (blockIdx.x == nblocks - 1) npts[0] = b + counts[blockIdx.x];
  }
  __syncthreads();
  int base = base_sh;
  const int r0 = blockIdx.x * GEO_ROWS_PER_BLOCK;
  const int r1 = min(H, r0 + GEO_ROWS_PER_BLOCK);
  for (int p0 = r0 * W; p0 < r1 * W; p0 += GEO_THREADS) {
    const int p = p0 + threadIdx.x;
    const int v = (p < r1 * W) && pix_valid(mask, depth, p);
    int total;
    const int off = block_scan_excl(v, sh, total);
    if (v) {
      const int idx = base + off;
      if (idx < cap) {
        const int u = p % W, row = p / W;
        const double z = (double)depth[p] * cam.scale;
        pts[(size_t)idx * 4 + 0] = ((double)u - cam.cx) * z / cam.fx;
        pts[(size_t)idx * 4 + 1] = ((double)row - cam.cy) * z / cam.fy;
        pts[(size_t)idx * 4 + 2] = z;
        pts[(size_t)idx * 4 + 3] = (double)idx;
      }
    }
    base += total;
  }
}

// order-preserving key of a double (larger double -> larger key)
RDP_DEV uint64_t dkey(double d) {
  const uint64_t b = (uint64_t)__double_as_longlong(d);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// One workgroup per bin. out: [nbins][kcap][4]; kout[b] = k written (0 if empty bin).
__global__ __launch_bounds__(GEO_THREADS) void geo_edges_kernel(const double* __restrict__ pts,
                                                                const int* __restrict__ npts_p,
                                                                const double* __restrict__ bxmin,
                                                                const double* __restrict__ bxmax, int nblk, int nbins,
                                                                double top, double* __restrict__ out, int kcap,
                                                                int* __restrict__ kout, int min_points) {
  __shared__ unsigned hist[256];
  __shared__ double s_lo, s_hi;
  __shared__ int s_tot[GEO_THREADS / 64];
  __shared__ uint64_t s_prefix;
  __shared__ int s_need;
  __shared__ int s_gt_cnt, s_eq_cnt;
  const int bin = blockIdx.x;
  const int n = npts_p[0];
  if (threadIdx.x == 0) {
    double a = 1e300, b = -1e300;
    for (int i = 0; i < nblk; ++i) { a = fmin(a, bxmin[i]); b = fmax(b, bxmax[i]); }
    s_lo = a;
    s_hi = b;
  }
  __syncthreads();
  const double lo = s_lo, hi = s_hi;
  const double width = (hi - lo) / (double)nbins;
  if (n < min_points || !(width > 0.0)) {
    if (threadIdx.x == 0) kout[bin] = 0;
    return;
  }
  auto bin_of = [&](double x) {
    double f = floor((x - lo) / width);
    int b = (int)fmin(fmax(f, 0.0), (double)(nbins - 1));
    return b;
  };
  // 1) bin size
  int c = 0;
  for (int i = threadIdx.x; i < n; i += GEO_THREADS) c += bin_of(pts[(size_t)i * 4]) == bin;
  int tot;
  (void)block_scan_excl(c, s_tot, tot);
  const int nb = tot;
  if (nb == 0) {
    if (threadIdx.x == 0) kout[bin] = 0;
    return;
  }
  int k = (int)((double)nb * top);
  if (k < 1) k = 1;
  if (k > kcap) k = kcap;
  // 2) radix select (8 passes x 8 bits, MSB first) of the k-th largest y key within the bin
  if (threadIdx.x == 0) { s_prefix = 0; s_need = k; }
  __syncthreads();
  for (int pass = 0; pass < 8; ++pass) {
    const int shift = 56 - 8 * pass;
    for (int i = threadIdx.x; i < 256; i += GEO_THREADS) hist[i] = 0;
    __syncthreads();
    const uint64_t prefix = s_prefix;
    const uint64_t pmask = pass == 0 ? 0ull : (~0ull << (64 - 8 * pass));
    for (int i = threadIdx.x; i < n; i += GEO_THREADS) {
      if (bin_of(pts[(size_t)i * 4]) != bin) continue;
      const uint64_t key = dkey(pts[(size_t)i * 4 + 1]);
      if ((key & pmask) != prefix) continue;
      atomicAdd(&hist[(key >> shift) & 255], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int need = s_need;
      int d = 255;
      for (; d > 0; --d) {  // walk from the largest digit down
        if ((int)hist[d] >= need) break;
        need -= hist[d];
      }
      s_need = need;
      s_prefix = prefix | ((uint64_t)d << shift);
    }
    __syncthreads();
  }
  const uint64_t kth = s_prefix;  // exact key of the k-th largest y
  // 3) write: every key > kth, plus the (need) smallest-index keys == kth
  if (threadIdx.x == 0) { s_gt_cnt = 0; s_eq_cnt = 0; }
  __syncthreads();
  const int need_eq = s_need;  // number of ties to take
  double* ob = out + (size_t)bin * kcap * 4;
  // keys > kth (order irrelevant: the host sorts the edge set)
  for (int i = threadIdx.x; i < n; i += GEO_THREADS) {
    if (bin_of(pts[(size_t)i * 4]) != bin) continue;
    if (dkey(pts[(size_t)i * 4 + 1]) > kth) {
      const int o = atomicAdd(&s_gt_cnt, 1);
      for (int j = 0; j < 4; ++j) ob[(size_t)o * 4 + j] = pts[(size_t)i * 4 + j];
    }
  }
  __syncthreads();
  // ties in ascending point index: ordered scan over the points
  int written = 0;
  const int gt = s_gt_cnt;
  for (int i0 = 0; i0 < n && written < need_eq; i0 += GEO_THREADS) {
    const int i = i0 + threadIdx.x;
    const int e = (i < n) && bin_of(pts[(size_t)i * 4]) == bin && dkey(pts[(size_t)i * 4 + 1]) == kth;
    int t;
    const int off = block_scan_excl(e, s_tot, t);
    if (e && written + off < need_eq) {
      const int o = gt + written + off;
      for (int j = 0; j < 4; ++j) ob[(size_t)o * 4 + j] = pts[(size_t)i * 4 + j];
    }
    written += t;
  }
  if (threadIdx.x == 0) kout[bin] = k;
}

// Pack the per-bin edge points contiguously: hdr[0] = E (total), edges[E][4].
__global__ void geo_pack_kernel(const double* __restrict__ out, int kcap, const int* __restrict__ kout, int nbins,
                                double* __restrict__ edges, int ecap, int* __restrict__ hdr) {
  __shared__ int offs[128];
  if (threadIdx.x == 0) {
    int o = 0;
    for (int b = 0; b < nbins; ++b) { offs[b] = o; o += kout[b]; }
    hdr[0] = o;
  }
  __syncthreads();
  for (int b = 0; b < nbins; ++b) {
    const int k = kout[b], o = offs[b];
    for (int i = threadIdx.x; i < k * 4; i += blockDim.x) {
      const int e = o * 4 + i;
      if (e < ecap * 4) edges[e] = out[(size_t)b * kcap * 4 + i];
    }
  }
}

extern "C" {
int rdp_geo_nblocks(int H) { return (H + GEO_ROWS_PER_BLOCK - 1) / GEO_ROWS_PER_BLOCK; }

// work: counts[nblk] ints, xmin/xmax[nblk] doubles (caller-provided); pts [cap][4]; out [nbins][kcap][4]
int rdp_geo_edges(const void* mask, const void* depth, int H, int W, double fx, double fy, double cx, double cy,
                  double scale, int* counts, double* xmin, double* xmax, double* pts, int cap, int* npts,
                  double* out, int kcap, int* kout, int nbins, double top, int min_points, double* edges,
                  int ecap, int* hdr, hipStream_t s) {
  if (nbins > 128 || nbins < 1) return -1;
  const int nblk = rdp_geo_nblocks(H);
  GeoCam cam{fx, fy, cx, cy, scale};
  hipLaunchKernelGGL(geo_count_kernel, dim3(nblk), dim3(GEO_THREADS), 0, s, (const uint8_t*)mask,
                     (const uint16_t*)depth, H, W, cam, counts, xmin, xmax);
  hipLaunchKernelGGL(geo_write_kernel, dim3(nblk), dim3(GEO_THREADS), 0, s, (const uint8_t*)mask,
                     (const uint16_t*)depth, H, W, cam, counts, nblk, pts, cap, npts);
  hipLaunchKernelGGL(geo_edges_kernel, dim3(nbins), dim3(GEO_THREADS), 0, s, pts, npts, xmin, xmax, nblk, nbins, top,
                     out, kcap, kout, min_points);
  hipLaunchKernelGGL(geo_pack_kernel, dim3(1), dim3(256), 0, s, out, kcap, kout, nbins, edges, ecap, hdr);
  return nblk;
}
}
