// Per-bin x-sort of selected edge points, shared by geo_sort_kernel (csrc/geo_spline.hip) and the
// fused select + sort path of geo_select_kernel (csrc/geometry.hip).
//
// The bins partition the x range monotonically, so the global order "x asc, y desc, point index asc"
// (the reference's argsort by x of the selected edge points, /root/reference/pkg/geometry_utils.py:
// 74-87, with deterministic ties) is the concatenation of per-bin sorts. One workgroup sorts one bin's
// k points: bitonic sort of a permutation (LDS for <= SORT_LCAP points, global scratch beyond),
// then writes the points packed as (x, y, z) at sorted[off ..].
#pragma once
#include "common.h"

#define SORT_LCAP 2048

// ob: the bin's k points as [k][4] (x, y, z, index); caller-provided LDS arrays of SORT_LCAP entries.
// Every thread of the workgroup calls it (barriers inside); k and off are workgroup-uniform.
RDP_DEV void geo_sort_bin(const double* ob, int k, int off, double* sorted, int* gperm, int ecap, double* sx,
                          double* sy, int* sid, int* sperm) {
  const int tid = threadIdx.x;
  if (k <= 0 || off >= ecap) return;
  if (off + k > ecap) k = ecap - off;
  int P = 1;
  while (P < k) P <<= 1;
  const bool lds = P <= SORT_LCAP;
  // global fallback: [2*off, 2*off + P) is private to this bin because P < 2k
  int* perm = lds ? sperm : gperm + 2 * (size_t)off;
  if (lds)
    for (int i = tid; i < k; i += blockDim.x) {
      sx[i] = ob[(size_t)i * 4];
      sy[i] = ob[(size_t)i * 4 + 1];
      sid[i] = (int)ob[(size_t)i * 4 + 3];
    }
  for (int i = tid; i < P; i += blockDim.x) perm[i] = i;
  __syncthreads();
  // a after c in the order (x asc, y desc, index asc); padding (>= k) sorts last
  auto after = [&](int a, int c) -> bool {
    if (a >= k) return c < k || a > c;
    if (c >= k) return false;
    double xa, xc, ya, yc;
    int ia, ic;
    if (lds) {
      xa = sx[a]; xc = sx[c]; ya = sy[a]; yc = sy[c]; ia = sid[a]; ic = sid[c];
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
      for (int t = tid; t < P / 2; t += blockDim.x) {
        const int i = 2 * stride * (t / stride) + (t % stride), j = i + stride;
        const int a = perm[i], c = perm[j];
        const bool up = (i & size) == 0;
        if (up ? after(a, c) : after(c, a)) {
          perm[i] = c;
          perm[j] = a;
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < k; i += blockDim.x) {
    const int s = perm[i];
    for (int c = 0; c < 3; ++c) sorted[(size_t)(off + i) * 3 + c] = ob[(size_t)s * 4 + c];
  }
}
