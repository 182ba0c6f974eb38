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
//   geo_write:   also bins every point by x (per-bin counts)
//   geo_bin_scatter: point indices grouped by bin
//   geo_select:  one workgroup per bin: bin size, k, radix-select of the k-th largest y key,
//                then writes the bin's k points (x, y, z, index) into a per-bin output slab, and
//                (serving) x-sorts them into the packed edge array (geo_sort.h)
#include "common.h"
#include "geo_sort.h"
#include <stdint.h>
#include <stdlib.h>

#define GEO_ROWS_PER_BLOCK 1  // 480 blocks at 480 rows (4 rows = 120 blocks left half the CUs idle: count + write 22 -> 11 us)
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

// Serving form (m256 != nullptr): the full-resolution mask is derived here from the model-resolution
// mask by cv2 INTER_NEAREST (src = min(floor(dst * in/out), in - 1), double math as the reference's
// cv2.resize, server.py:125) and written out (it is the PNG-encoded response mask), and the coverage
// count (nnz of the mask, server.py:133) is produced per row block -- no separate upsample kernel and
// no global atomics. Block 0 also zeroes the binning counters used two kernels later.
struct GeoSrc {
  const uint8_t* m256;  // nullptr: `mask` is an input
  int mh, mw;
  double sy, sx;
  uint8_t* mask_out;
  uint8_t* mask_host;  // optional second copy of mask_out in host memory (the serving read-back, zero-copy)
  int* cov;  // [nblk] coverage counts (serving form)
  int* zero;  // [nzero] ints zeroed by block 0
  int nzero;
};

RDP_DEV uint8_t src_mask(const GeoSrc& g, const uint8_t* mask, int p, int W) {
  if (!g.m256) return mask[p];
  const int y = p / W, x = p - y * W;
  const int iy = min((int)floor((double)y * g.sy), g.mh - 1), ix = min((int)floor((double)x * g.sx), g.mw - 1);
  return g.m256[iy * g.mw + ix];
}

RDP_DEV void geo_count_body(const uint8_t* __restrict__ mask,
                                                                const uint16_t* __restrict__ depth, int H, int W,
                                                                GeoCam cam, int* __restrict__ counts,
                                                                double* __restrict__ xmin, double* __restrict__ xmax,
                                                                GeoSrc gs) {
  __shared__ double smin[GEO_THREADS / 64], smax[GEO_THREADS / 64];
  __shared__ int scnt[GEO_THREADS / 64], scov[GEO_THREADS / 64];
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < gs.nzero; i += GEO_THREADS) gs.zero[i] = 0;
  const int r0 = blockIdx.x * GEO_ROWS_PER_BLOCK;
  const int r1 = min(H, r0 + GEO_ROWS_PER_BLOCK);
  int cnt = 0, cov = 0;
  double lo = 1e300, hi = -1e300;
  for (int p = r0 * W + threadIdx.x; p < r1 * W; p += GEO_THREADS) {
    const uint8_t mv = src_mask(gs, mask, p, W);
    if (gs.m256) {
      gs.mask_out[p] = mv;
      if (gs.mask_host) gs.mask_host[p] = mv;
    }
    cov += mv != 0;
    if (mv > 0 && depth[p] > 0) {
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
    cov += __shfl_xor(cov, o, 64);
    lo = fmin(lo, __shfl_xor(lo, o, 64));
    hi = fmax(hi, __shfl_xor(hi, o, 64));
  }
  if (lane == 0) { scnt[wave] = cnt; scov[wave] = cov; smin[wave] = lo; smax[wave] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    int c = 0, v = 0;
    double a = 1e300, b = -1e300;
    for (int w = 0; w < GEO_THREADS / 64; ++w) { c += scnt[w]; v += scov[w]; a = fmin(a, smin[w]); b = fmax(b, smax[w]); }
    counts[blockIdx.x] = c;
    xmin[blockIdx.x] = a;
    xmax[blockIdx.x] = b;
    if (gs.cov) gs.cov[blockIdx.x] = v;
  }
}

RDP_DEV void geo_range(const double* bxmin, const double* bxmax, int nblk, double* s_lo, double* s_hi);

// ---- binning: counting sort of point indices by x bin (bin computed once per point) ----
// bin = clip(floor((x - lo) / w), 0, nbins-1) with the reference's division (not a reciprocal
// multiply), so boundary points land in exactly the reference's bin.
struct GeoBins {
  int* bin_of;     // [cap]   bin of every point
  int* bidx;       // [cap]   point indices grouped by bin (order within a bin is arbitrary)
  int* cnt;        // [128]   points per bin
  int* cursor;     // [128]   scatter cursors
};

// pts: [cap][4] doubles (x, y, z, index) ; npts[0] = total count (written by the last block's thread 0)
// The x-bin of every written point and the per-bin counts are produced here too (the global x range
// is reduced from geo_count's per-block partials by every block): no separate counting launch.
RDP_DEV void geo_write_body(const uint8_t* __restrict__ mask,
                                                                const uint16_t* __restrict__ depth, int H, int W,
                                                                GeoCam cam, const int* __restrict__ counts,
                                                                int nblocks, double* __restrict__ pts, int cap,
                                                                int* __restrict__ npts, const double* __restrict__ bxmin,
                                                                const double* __restrict__ bxmax, int nbins,
                                                                GeoBins gb) {
  __shared__ int sh[GEO_THREADS / 64];
  __shared__ int base_sh;
  __shared__ unsigned lc[128];
  double lo, hi;
  geo_range(bxmin, bxmax, nblocks, &lo, &hi);
  const double width = (hi - lo) / (double)nbins;
  for (int i = threadIdx.x; i < nbins; i += GEO_THREADS) lc[i] = 0;
  {  // exclusive prefix of the earlier row blocks' counts: all threads load, wave sums, waves in order
    int b = 0;
    for (int i = threadIdx.x; i < (int)blockIdx.x; i += GEO_THREADS) b += counts[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) b += __shfl_xor(b, o, 64);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
      const int t = sh[0] + sh[1] + sh[2] + sh[3];
      base_sh = t;
      if (blockIdx.x == nblocks - 1) npts[0] = t + counts[blockIdx.x];
    }
    __syncthreads();
  }
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
        const double x = ((double)u - cam.cx) * z / cam.fx;
        pts[(size_t)idx * 4 + 0] = x;
        pts[(size_t)idx * 4 + 1] = ((double)row - cam.cy) * z / cam.fy;
        pts[(size_t)idx * 4 + 2] = z;
        pts[(size_t)idx * 4 + 3] = (double)idx;
        if (width > 0.0) {
          const double f = floor((x - lo) / width);
          const int b = (int)fmin(fmax(f, 0.0), (double)(nbins - 1));
          gb.bin_of[idx] = b;
          atomicAdd(&lc[b], 1u);
        }
      }
    }
    base += total;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nbins; i += GEO_THREADS)
    if (lc[i]) atomicAdd(&gb.cnt[i], (int)lc[i]);
}

// order-preserving key of a double (larger double -> larger key)
RDP_DEV uint64_t dkey(double d) {
  const uint64_t b = (uint64_t)__double_as_longlong(d);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

RDP_DEV void geo_range(const double* bxmin, const double* bxmax, int nblk, double* s_lo, double* s_hi) {
  // every block reduces the per-row-block partials itself (nblk ~ H/4 doubles)
  __shared__ double rlo[GEO_THREADS], rhi[GEO_THREADS];
  double a = 1e300, b = -1e300;
  for (int i = threadIdx.x; i < nblk; i += GEO_THREADS) { a = fmin(a, bxmin[i]); b = fmax(b, bxmax[i]); }
  rlo[threadIdx.x] = a;
  rhi[threadIdx.x] = b;
  __syncthreads();
  for (int o = GEO_THREADS / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      rlo[threadIdx.x] = fmin(rlo[threadIdx.x], rlo[threadIdx.x + o]);
      rhi[threadIdx.x] = fmax(rhi[threadIdx.x], rhi[threadIdx.x + o]);
    }
    __syncthreads();
  }
  *s_lo = rlo[0];
  *s_hi = rhi[0];
}

RDP_DEV void geo_bin_scatter_body(const int* __restrict__ npts_p, int nbins,
                                                                      GeoBins gb) {
  __shared__ int base[128];
  __shared__ unsigned lc[128], lbase[128];
  if (threadIdx.x == 0) {
    int o = 0;
    for (int b = 0; b < nbins; ++b) { base[b] = o; o += gb.cnt[b]; }
  }
  for (int i = threadIdx.x; i < nbins; i += GEO_THREADS) lc[i] = 0;
  __syncthreads();
  const int n = npts_p[0];
  // block-aggregated cursors: one global atomic per (block, bin)
  const int i0 = blockIdx.x * GEO_THREADS * 4;
  int bins[4], pos[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = i0 + u * GEO_THREADS + threadIdx.x;
    bins[u] = i < n ? gb.bin_of[i] : -1;
    pos[u] = bins[u] >= 0 ? (int)atomicAdd(&lc[bins[u]], 1u) : 0;
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nbins; b += GEO_THREADS)
    lbase[b] = lc[b] ? (unsigned)atomicAdd(&gb.cursor[b], (int)lc[b]) : 0u;
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = i0 + u * GEO_THREADS + threadIdx.x;
    if (bins[u] >= 0) gb.bidx[base[bins[u]] + (int)lbase[bins[u]] + pos[u]] = i;
  }
}

// Digit selection over a 256-bucket histogram by wave 0 (4 buckets per lane + a wave scan), instead
// of a serial walk by one thread. LARGEST = true: the largest digit d with #(digit >= d) >= need;
// false: the smallest d with #(digit <= d) >= need. Lane owning d stores d, the remaining need and
// the bucket count hist[d] (the number of candidates equal to the new prefix).
template <bool LARGEST>
RDP_DEV void geo_pick_digit(const unsigned* hist, int need, int* s_digit, int* s_need, int* s_eq) {
  const int l = threadIdx.x;  // wave 0 only
  int h[4], tot = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) { h[j] = (int)hist[4 * l + j]; tot += h[j]; }
  int sc = tot;  // LARGEST: inclusive suffix sum over lanes >= l; else inclusive prefix over lanes <= l
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = LARGEST ? __shfl_down(sc, off, 64) : __shfl_up(sc, off, 64);
    if (LARGEST ? l + off < 64 : l >= off) sc += o;
  }
  const int before = sc - tot;  // candidates strictly beyond this lane's buckets (in scan order)
  if (before < need && need <= sc) {
    int acc = before;
    if (LARGEST) {
#pragma unroll
      for (int j = 3; j >= 0; --j) {
        if (acc + h[j] >= need) { *s_digit = 4 * l + j; *s_need = need - acc; *s_eq = h[j]; break; }
        acc += h[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (acc + h[j] >= need) { *s_digit = 4 * l + j; *s_need = need - acc; *s_eq = h[j]; break; }
        acc += h[j];
      }
    }
  }
}

// Per-bin top-k by y (k = max(1, int(n_bin * top)), capped); ties at the k-th value go to the
// smallest point indices (= the reference's stable descending sort), by radix select (8 x 8 bits,
// MSB first) of the k-th largest y key, then -- only when the ties at that key are not all taken --
// radix select (4 x 8 bits) of the largest index among the ties to keep. One wave owns one bin, so the 8 + 4 radix passes and the bitonic x-sort need no workgroup
// barrier (a wave's LDS operations execute in issue order; the digit owner is found by ballot and
// broadcast by a lane shuffle). The k selected points are compacted in point-index order (ballot +
// popcount), so `out` is deterministic too. Bins beyond the LDS caches read / sort through global
// memory (vmcnt-ordered within the wave).
#define GEO_WLCAP 2048
#define GEO_WSORT 256
// cross-lane LDS hand-off inside one wave: drain this wave's LDS operations and keep the compiler
// from moving LDS accesses across (no workgroup barrier: other waves own other bins)
RDP_DEV void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}
template <bool LARGEST>
RDP_DEV void wave_pick_digit(const unsigned* hist, int need, int lane, int& digit, int& nneed, int& eq) {
  int h[4], tot = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) { h[j] = (int)hist[4 * lane + j]; tot += h[j]; }
  int sc = tot;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = LARGEST ? __shfl_down(sc, off, 64) : __shfl_up(sc, off, 64);
    if (LARGEST ? lane + off < 64 : lane >= off) sc += o;
  }
  const int before = sc - tot;
  int d = 0, nn = 0, e = 0;
  const bool own = before < need && need <= sc;
  if (own) {
    int acc = before;
    if (LARGEST) {
#pragma unroll
      for (int j = 3; j >= 0; --j) {
        if (acc + h[j] >= need) { d = 4 * lane + j; nn = need - acc; e = h[j]; break; }
        acc += h[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (acc + h[j] >= need) { d = 4 * lane + j; nn = need - acc; e = h[j]; break; }
        acc += h[j];
      }
    }
  }
  const int owner = __ffsll((unsigned long long)__ballot(own)) - 1;
  digit = __shfl(d, owner, 64);
  nneed = __shfl(nn, owner, 64);
  eq = __shfl(e, owner, 64);
}

RDP_DEV void geo_select_wave_body(const double* __restrict__ pts,
                                                              const int* __restrict__ npts_p, int nbins, double top,
                                                              GeoBins gb, double* __restrict__ out, int kcap,
                                                              int* __restrict__ kout, int min_points,
                                                              double* __restrict__ sorted, int* __restrict__ gperm,
                                                              int ecap) {
  __shared__ unsigned whist[4][256];
  __shared__ uint64_t wkey[4][GEO_WLCAP];
  __shared__ int wid[4][GEO_WLCAP];
  __shared__ double wsx[4][GEO_WSORT], wsy[4][GEO_WSORT], wsz[4][GEO_WSORT];
  __shared__ int wsi[4][GEO_WSORT], wperm[4][GEO_WSORT];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int bin = blockIdx.x * 4 + w;
  if (bin >= nbins) return;  // whole wave; no workgroup barriers below
  unsigned* hist = whist[w];
  uint64_t* skey = wkey[w];
  int* sid = wid[w];
  const int n = npts_p[0];
  const int nb = gb.cnt[bin];
  if (n < min_points || nb == 0) {
    if (lane == 0) kout[bin] = 0;
    return;
  }
  int start = 0, off = 0;  // first point of the bin in bidx; sum of the earlier bins' k
  for (int b = lane; b < bin; b += 64) {
    const int c = gb.cnt[b];
    start += c;
    int kb = (int)((double)c * top);
    if (kb < 1) kb = 1;
    if (kb > kcap) kb = kcap;
    off += c > 0 ? kb : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    start += __shfl_xor(start, o, 64);
    off += __shfl_xor(off, o, 64);
  }
  const int* ids = gb.bidx + start;
  int k = (int)((double)nb * top);
  if (k < 1) k = 1;
  if (k > kcap) k = kcap;
  for (int i = lane; i < nb && i < GEO_WLCAP; i += 64) {
    const int id = ids[i];
    sid[i] = id;
    skey[i] = dkey(pts[(size_t)id * 4 + 1]);
  }
  wave_lds_sync();
  auto key_at = [&](int i) -> uint64_t { return i < GEO_WLCAP ? skey[i] : dkey(pts[(size_t)ids[i] * 4 + 1]); };
  auto id_at = [&](int i) -> int { return i < GEO_WLCAP ? sid[i] : ids[i]; };
  // 1) k-th largest key (8 x 8-bit digits, MSB first)
  uint64_t prefix = 0;
  int need = k, eq = 0;
  for (int pass = 0; pass < 8; ++pass) {
    const int shift = 56 - 8 * pass;
#pragma unroll
    for (int j = 0; j < 4; ++j) hist[4 * lane + j] = 0;
    wave_lds_sync();
    const uint64_t pmask = pass == 0 ? 0ull : (~0ull << (64 - 8 * pass));
    for (int i = lane; i < nb; i += 64) {
      const uint64_t key = key_at(i);
      if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1u);
    }
    wave_lds_sync();
    int d, nn;
    wave_pick_digit<true>(hist, need, lane, d, nn, eq);
    prefix |= (uint64_t)d << shift;
    need = nn;
  }
  const uint64_t kth = prefix;
  // 2) ties at kth: the `need` smallest indices
  uint32_t last_id = 0xffffffffu;
  if (need < eq) {
    uint32_t ip = 0;
    for (int pass = 0; pass < 4; ++pass) {
      const int shift = 24 - 8 * pass;
#pragma unroll
      for (int j = 0; j < 4; ++j) hist[4 * lane + j] = 0;
      wave_lds_sync();
      const uint32_t pmask = pass == 0 ? 0u : (~0u << (32 - 8 * pass));
      for (int i = lane; i < nb; i += 64) {
        const uint32_t id = (uint32_t)id_at(i);
        if (key_at(i) == kth && (id & pmask) == ip) atomicAdd(&hist[(id >> shift) & 255], 1u);
      }
      wave_lds_sync();
      int d, nn, e2;
      wave_pick_digit<false>(hist, need, lane, d, nn, e2);
      ip |= (uint32_t)d << shift;
      need = nn;
    }
    last_id = ip;
  }
  // 3) compact the k points in bin order (ballot prefix): out slab + the sort caches
  double* ob = out + (size_t)bin * kcap * 4;
  const bool lsort = sorted != nullptr && k <= GEO_WSORT;
  int base = 0;
  for (int i0 = 0; i0 < nb; i0 += 64) {
    const int i = i0 + lane;
    bool sel = false;
    int id = 0;
    if (i < nb) {
      const uint64_t key = key_at(i);
      id = id_at(i);
      sel = key > kth || (key == kth && (uint32_t)id <= last_id);
    }
    const unsigned long long msk = __ballot(sel);
    const int pos = base + __popcll(msk & ((1ull << lane) - 1ull));
    if (sel && pos < kcap) {
      const double px = pts[(size_t)id * 4], py = pts[(size_t)id * 4 + 1], pz = pts[(size_t)id * 4 + 2];
      ob[(size_t)pos * 4] = px;
      ob[(size_t)pos * 4 + 1] = py;
      ob[(size_t)pos * 4 + 2] = pz;
      ob[(size_t)pos * 4 + 3] = pts[(size_t)id * 4 + 3];
      if (lsort) {
        wsx[w][pos] = px;
        wsy[w][pos] = py;
        wsz[w][pos] = pz;
        wsi[w][pos] = (int)pts[(size_t)id * 4 + 3];
      }
    }
    base += __popcll(msk);
  }
  wave_lds_sync();
  if (lane == 0) kout[bin] = k;
  if (!sorted) return;
  // 4) x-sort (x asc, y desc, index asc) of the k points into sorted[off ..] (as geo_sort_bin)
  if (off >= ecap) return;
  int kk = k;
  if (off + kk > ecap) kk = ecap - off;
  int P = 1;
  while (P < k) P <<= 1;
  int* perm = lsort ? wperm[w] : gperm + 2 * (size_t)off;
  if (!lsort) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's `out` stores, before re-reading
  for (int i = lane; i < P; i += 64) perm[i] = i;
  wave_lds_sync();
  auto after = [&](int a, int c) -> bool {
    if (a >= k) return c < k || a > c;
    if (c >= k) return false;
    double xa, xc, ya, yc;
    int ia, ic;
    if (lsort) {
      xa = wsx[w][a]; xc = wsx[w][c]; ya = wsy[w][a]; yc = wsy[w][c]; ia = wsi[w][a]; ic = wsi[w][c];
    } else {
      xa = ob[(size_t)a * 4]; xc = ob[(size_t)c * 4];
      ya = ob[(size_t)a * 4 + 1]; yc = ob[(size_t)c * 4 + 1];
      ia = (int)ob[(size_t)a * 4 + 3]; ic = (int)ob[(size_t)c * 4 + 3];
    }
    if (xa != xc) return xa > xc;
    if (ya != yc) return ya < yc;
    return ia > ic;
  };
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (!lsort) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // previous stage's perm stores
      for (int t = lane; t < P / 2; t += 64) {
        const int i = 2 * stride * (t / stride) + (t % stride), j = i + stride;
        const int a = perm[i], c = perm[j];
        const bool up = (i & size) == 0;
        if (up ? after(a, c) : after(c, a)) {
          perm[i] = c;
          perm[j] = a;
        }
      }
      wave_lds_sync();
    }
  }
  if (!lsort) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int i = lane; i < kk; i += 64) {
    const int sidx = perm[i];
    if (lsort) {
      sorted[(size_t)(off + i) * 3] = wsx[w][sidx];
      sorted[(size_t)(off + i) * 3 + 1] = wsy[w][sidx];
      sorted[(size_t)(off + i) * 3 + 2] = wsz[w][sidx];
    } else {
      for (int c = 0; c < 3; ++c) sorted[(size_t)(off + i) * 3 + c] = ob[(size_t)sidx * 4 + c];
    }
  }
}

// Pack the per-bin edge points contiguously (one block per bin): hdr[0] = E, edges[E][4].
__global__ void geo_pack_kernel(const double* __restrict__ out, int kcap, const int* __restrict__ kout, int nbins,
                                double* __restrict__ edges, int ecap, int* __restrict__ hdr) {
  __shared__ int s_off;
  const int b = blockIdx.x;
  if (threadIdx.x == 0) {
    int o = 0;
    for (int i = 0; i < b; ++i) o += kout[i];
    s_off = o;
    if (b == nbins - 1) hdr[0] = o + kout[b];
  }
  __syncthreads();
  const int k = kout[b], o = s_off;
  for (int i = threadIdx.x; i < k * 4; i += blockDim.x) {
    const int e = o * 4 + i;
    if (e < ecap * 4) edges[e] = out[(size_t)b * kcap * 4 + i];
  }
}

__global__ void geo_zero_kernel(int* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0;
}

// ---- kernels: one frame (the bodies above), or up to GEO_BATCH frames per launch (blockIdx.y = frame) ----
__global__ __launch_bounds__(GEO_THREADS) void geo_count_kernel(const uint8_t* __restrict__ mask,
                                                                const uint16_t* __restrict__ depth, int H, int W,
                                                                GeoCam cam, int* __restrict__ counts,
                                                                double* __restrict__ xmin, double* __restrict__ xmax,
                                                                GeoSrc gs) {
  geo_count_body(mask, depth, H, W, cam, counts, xmin, xmax, gs);
}
__global__ __launch_bounds__(GEO_THREADS) void geo_write_kernel(const uint8_t* __restrict__ mask,
                                                                const uint16_t* __restrict__ depth, int H, int W,
                                                                GeoCam cam, const int* __restrict__ counts, int nblocks,
                                                                double* __restrict__ pts, int cap, int* __restrict__ npts,
                                                                const double* __restrict__ bxmin,
                                                                const double* __restrict__ bxmax, int nbins, GeoBins gb) {
  geo_write_body(mask, depth, H, W, cam, counts, nblocks, pts, cap, npts, bxmin, bxmax, nbins, gb);
}
__global__ __launch_bounds__(GEO_THREADS) void geo_bin_scatter_kernel(const int* __restrict__ npts_p, int nbins,
                                                                      GeoBins gb) {
  geo_bin_scatter_body(npts_p, nbins, gb);
}
__global__ __launch_bounds__(256) void geo_select_wave_kernel(const double* __restrict__ pts,
                                                              const int* __restrict__ npts_p, int nbins, double top,
                                                              GeoBins gb, double* __restrict__ out, int kcap,
                                                              int* __restrict__ kout, int min_points,
                                                              double* __restrict__ sorted, int* __restrict__ gperm,
                                                              int ecap) {
  geo_select_wave_body(pts, npts_p, nbins, top, gb, out, kcap, kout, min_points, sorted, gperm, ecap);
}

// One frame's edge-stage arguments (rdp_geo_edges' launches, serving form: no packed edge list).
struct GeoFrame {
  const uint8_t* mask;
  const uint16_t* depth;
  int* counts;
  double *xmin, *xmax, *pts, *out, *sorted;
  int *npts, *kout, *gperm;
  int cap, kcap, secap;
  GeoSrc gs;
  GeoBins gb;
};
#define GEO_BATCH 4
struct GeoFrames {
  GeoFrame f[GEO_BATCH];
  GeoCam cam;
  int H, W, nblk, nbins, min_points;
  double top;
};
// (the frame index is wave-uniform: kernel-argument loads through it stay scalar)
__global__ __launch_bounds__(GEO_THREADS) void geo_count_batch_kernel(const GeoFrames g) {
  const GeoFrame& a = g.f[blockIdx.y];
  geo_count_body(a.mask, a.depth, g.H, g.W, g.cam, a.counts, a.xmin, a.xmax, a.gs);
}
__global__ __launch_bounds__(GEO_THREADS) void geo_write_batch_kernel(const GeoFrames g) {
  const GeoFrame& a = g.f[blockIdx.y];
  geo_write_body(a.mask, a.depth, g.H, g.W, g.cam, a.counts, g.nblk, a.pts, a.cap, a.npts, a.xmin, a.xmax, g.nbins,
                 a.gb);
}
__global__ __launch_bounds__(GEO_THREADS) void geo_bin_scatter_batch_kernel(const GeoFrames g) {
  const GeoFrame& a = g.f[blockIdx.y];
  geo_bin_scatter_body(a.npts, g.nbins, a.gb);
}
__global__ __launch_bounds__(256) void geo_select_wave_batch_kernel(const GeoFrames g) {
  const GeoFrame& a = g.f[blockIdx.y];
  geo_select_wave_body(a.pts, a.npts, g.nbins, g.top, a.gb, a.out, a.kcap, a.kout, g.min_points, a.sorted, a.gperm,
                       a.secap);
}

extern "C" {
int rdp_geo_nblocks(int H) { return (H + GEO_ROWS_PER_BLOCK - 1) / GEO_ROWS_PER_BLOCK; }

// int32 workspace needed beyond the per-row-block counts: bin_of + bidx [cap] each + 2 x 128
long rdp_geo_work_ints(int H, int W) { return (long)rdp_geo_nblocks(H) + 2L * H * W + 256; }

// work_i: [nblk] counts | [cap] bin_of | [cap] bidx | [128] cnt | [128] cursor ; work_d: xmin/xmax
// pts [cap][4]; out [nbins][kcap][4]
// m256 != nullptr (serving form): `mask` is an OUTPUT, derived from the mh x mw model mask by
// nearest upsampling, and cov[nblk] receives per-row-block coverage counts. edges == nullptr: no
// packed edge list (the on-device spline reads the per-bin slabs directly). sorted != nullptr: the
// x-sorted edge points [secap][3] are written too (gperm: 2*secap ints of sort scratch), so the
// spline stage runs with presorted = 1.
int rdp_geo_edges(const void* mask, const void* depth, int H, int W, double fx, double fy, double cx, double cy,
                  double scale, int* counts, double* xmin, double* xmax, double* pts, int cap, int* npts,
                  double* out, int kcap, int* kout, int nbins, double top, int min_points, double* edges,
                  int ecap, int* hdr, const void* m256, int mh, int mw, int* cov, double* sorted, int* gperm,
                  int secap, void* mask_host, hipStream_t s) {
  if (nbins > 128 || nbins < 1) return -1;
  const int nblk = rdp_geo_nblocks(H);
  GeoCam cam{fx, fy, cx, cy, scale};
  GeoBins gb;
  gb.bin_of = counts + nblk;
  gb.bidx = gb.bin_of + cap;
  gb.cnt = gb.bidx + cap;
  gb.cursor = gb.cnt + 128;
  GeoSrc gs;
  gs.m256 = (const uint8_t*)m256;
  gs.mh = mh;
  gs.mw = mw;
  gs.sy = m256 ? 1.0 / ((double)H / (double)mh) : 0.0;  // as cv::resize INTER_NEAREST (serve_kernels.hip)
  gs.sx = m256 ? 1.0 / ((double)W / (double)mw) : 0.0;
  gs.mask_out = (uint8_t*)mask;
  gs.mask_host = (uint8_t*)mask_host;
  gs.cov = cov;
  gs.zero = gb.cnt;  // cnt + cursor (256 ints), consumed two kernels later
  gs.nzero = 256;
  hipLaunchKernelGGL(geo_count_kernel, dim3(nblk), dim3(GEO_THREADS), 0, s, (const uint8_t*)mask,
                     (const uint16_t*)depth, H, W, cam, counts, xmin, xmax, gs);
  hipLaunchKernelGGL(geo_write_kernel, dim3(nblk), dim3(GEO_THREADS), 0, s, (const uint8_t*)mask,
                     (const uint16_t*)depth, H, W, cam, counts, nblk, pts, cap, npts, xmin, xmax, nbins, gb);
  const int pblocks = (cap + GEO_THREADS * 4 - 1) / (GEO_THREADS * 4);
  hipLaunchKernelGGL(geo_bin_scatter_kernel, dim3(pblocks), dim3(GEO_THREADS), 0, s, npts, nbins, gb);
  hipLaunchKernelGGL(geo_select_wave_kernel, dim3((nbins + 3) / 4), dim3(256), 0, s, pts, npts, nbins, top, gb, out,
                       kcap, kout, min_points, sorted, gperm, secap);
  if (edges) hipLaunchKernelGGL(geo_pack_kernel, dim3(nbins), dim3(256), 0, s, out, kcap, kout, nbins, edges, ecap, hdr);
  return nblk;
}

// The serving form of rdp_geo_edges for n <= GEO_BATCH frames of one camera in ONE launch per stage
// (blockIdx.y = frame): each frame's buffers as rdp_geo_edges takes them (array of n per field). The
// stages are latency-bound small grids, so n frames cost about what one does (a batch of 4 served frames:
// 4 x 48 us of geometry as per-frame launches, profiles/serve_batch.md).
int rdp_geo_edges_batch(int n, const void* const* mask, const void* const* depth, int H, int W, double fx, double fy,
                        double cx, double cy, double scale, int* const* counts, double* const* xmin,
                        double* const* xmax, double* const* pts, int cap, int* const* npts, double* const* out,
                        int kcap, int* const* kout, int nbins, double top, int min_points, const void* const* m256,
                        int mh, int mw, int* const* cov, double* const* sorted, int* const* gperm, int secap,
                        void* const* mask_host, hipStream_t s) {
  if (nbins > 128 || nbins < 1 || n < 1 || n > GEO_BATCH) return -1;
  GeoFrames g;
  g.cam = GeoCam{fx, fy, cx, cy, scale};
  g.H = H; g.W = W; g.nblk = rdp_geo_nblocks(H); g.nbins = nbins; g.min_points = min_points; g.top = top;
  for (int i = 0; i < GEO_BATCH; ++i) {
    const int j = i < n ? i : 0;  // (unused slots: a copy of frame 0's, never launched)
    GeoFrame& f = g.f[i];
    f.mask = (const uint8_t*)mask[j];
    f.depth = (const uint16_t*)depth[j];
    f.counts = counts[j]; f.xmin = xmin[j]; f.xmax = xmax[j]; f.pts = pts[j]; f.out = out[j]; f.sorted = sorted[j];
    f.npts = npts[j]; f.kout = kout[j]; f.gperm = gperm[j];
    f.cap = cap; f.kcap = kcap; f.secap = secap;
    f.gb.bin_of = counts[j] + g.nblk;
    f.gb.bidx = f.gb.bin_of + cap;
    f.gb.cnt = f.gb.bidx + cap;
    f.gb.cursor = f.gb.cnt + 128;
    f.gs.m256 = (const uint8_t*)m256[j];
    f.gs.mh = mh; f.gs.mw = mw;
    f.gs.sy = 1.0 / ((double)H / (double)mh);
    f.gs.sx = 1.0 / ((double)W / (double)mw);
    f.gs.mask_out = (uint8_t*)mask[j];
    f.gs.mask_host = mask_host ? (uint8_t*)mask_host[j] : nullptr;
    f.gs.cov = cov[j];
    f.gs.zero = f.gb.cnt;
    f.gs.nzero = 256;
  }
  const int pblocks = (cap + GEO_THREADS * 4 - 1) / (GEO_THREADS * 4);
  hipLaunchKernelGGL(geo_count_batch_kernel, dim3(g.nblk, n), dim3(GEO_THREADS), 0, s, g);
  hipLaunchKernelGGL(geo_write_batch_kernel, dim3(g.nblk, n), dim3(GEO_THREADS), 0, s, g);
  hipLaunchKernelGGL(geo_bin_scatter_batch_kernel, dim3(pblocks, n), dim3(GEO_THREADS), 0, s, g);
  hipLaunchKernelGGL(geo_select_wave_batch_kernel, dim3((nbins + 3) / 4, n), dim3(256), 0, s, g);
  return g.nblk;
}
}
