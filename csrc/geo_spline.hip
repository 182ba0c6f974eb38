// On-device B-spline stage of the curvature profile: x-sort of the edge points, FITPACK-equivalent
// parametric smoothing spline (splprep s, k), 100-sample splev of r, r', r'' and the curvature
// reduction -- so a served frame reads back 100 points + 6 scalars instead of the edge buffer.
//
// Replaces /root/reference/pkg/geometry_utils.py:74-87,144-162 (np.argsort by x, splprep([x,y,z],
// s=0.1, k=3), splev(der=0/1/2) at u = linspace(0, 1, 100), kappa = |r' x r''| / |r'|^3 on
// |r'| > 1e-6, mean / max). Semantics follow csrc/spline.cpp (the exact host port of FITPACK
// parcur/fppara, kept as the oracle and as the fallback for fits beyond the device capacity).
//
// Kernels:
//   geo_sort_kernel  one workgroup per x bin. The bins partition the x range monotonically, so
//                    the global order "x asc, y desc, point index asc" is the concatenation of
//                    per-bin sorts: bitonic sort of the bin's points (LDS for <= 2048 points,
//                    global scratch beyond), written packed as (x, y, z).
//   geo_fit_kernel   one workgroup (4 waves). Chord-length u by a block scan; then the FITPACK
//                    control flow (knot insertion fpknot, nplus heuristic, smoothing parameter
//                    iteration with fprati) on thread 0, with every O(points) pass data-parallel:
//                      * least squares for fixed knots via the banded normal equations: each wave
//                        accumulates B-spline outer products of its contiguous point range with
//                        wave reductions per knot interval into a private band copy (summed in a
//                        fixed order: deterministic), then a banded Cholesky solve on thread 0.
//                        R = chol(A^T A) has the diagonal of FITPACK's Givens R (both positive),
//                        so FITPACK's initial p = nk1 / sum(diag R) carries over exactly;
//                      * smoothing system (A^T A + p^-2 B^T B) c = A^T x with fpdisc's jump rows B
//                        (= the normal equations of FITPACK's rotated [A; B/p] system);
//                      * residual pass: fp and the per-interval residuals fpint with FITPACK's rule
//                        (the first point of an interval is split half / half).
//                    Finally 100 samples (one per thread), derivative coefficients as FITPACK's
//                    splder, curvature reduced in sample order on thread 0 (same order as the host).
// Results differ from the host Givens path only by rounding (normal equations in fp64 for a
// B-spline Gram matrix with <= 64 coefficients; tested against scipy and csrc/spline.cpp).
//
// res layout (doubles): [0] status (0 ok, 1 too few points, 2 too few edge points, 3 fit failed =
// FITPACK invalid input, 4 needs host: beyond the device knot capacity), [1] ier, [2] n knots,
// [3] fp, [4] mean kappa, [5] max kappa, [6] E edge points, [7] valid points, [8..] nsamp x 3 points,
// [8 + 3 nsamp] mask coverage count (serving form; -1 without coverage input).
#include "common.h"
#include "geo_sort.h"
#include <stdint.h>

#define SPL_THREADS 256
#define SPL_NK 64                   // max spline coefficients per dimension on the device
#define SPL_KMAX 5
#define SPL_NMAX (SPL_NK + SPL_KMAX + 1)  // max knots

enum { SPL_OK = 0, SPL_TOO_FEW_POINTS = 1, SPL_TOO_FEW_EDGES = 2, SPL_FIT_FAILED = 3, SPL_NEEDS_HOST = 4 };

// ------------------------------------------------------------------------------------------ sort
__global__ __launch_bounds__(256) void geo_sort_kernel(const double* __restrict__ out, int kcap,
                                                       const int* __restrict__ kout, double* __restrict__ sorted,
                                                       int* __restrict__ gperm, int ecap) {
  __shared__ double sx[SORT_LCAP], sy[SORT_LCAP];
  __shared__ int sid[SORT_LCAP], sperm[SORT_LCAP];
  __shared__ int s_off;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) {
    int o = 0;
    for (int i = 0; i < b; ++i) o += min(kout[i], kcap);
    s_off = o;
  }
  __syncthreads();
  geo_sort_bin(out + (size_t)b * kcap * 4, min(kout[b], kcap), s_off, sorted, gperm, ecap, sx, sy, sid, sperm);
}

// ------------------------------------------------------------------------------------------ fit
struct SplSh {
  double t[SPL_NMAX + 2];                  // knots, 1-based (t[1..n])
  double G[SPL_NK][SPL_KMAX + 1];          // band of A^T A: G[i][d] = (i, i + d), 0-based rows
  double Z[SPL_NK][3];                     // A^T x
  double A[SPL_NK][SPL_KMAX + 2];          // system being factored (band of A^T A [+ p^-2 B^T B])
  double R[SPL_NK][SPL_KMAX + 2];          // banded Cholesky factor (upper, bandwidth <= k + 2)
  double B[SPL_NK][SPL_KMAX + 2];          // fpdisc rows
  double c[3][SPL_NK];                     // coefficients
  double y[3][SPL_NK];                     // forward-substitution scratch
  double cd1[3][SPL_NK], cd2[3][SPL_NK];   // first / second derivative coefficients
  double fpint[SPL_NMAX + 2];              // 1-based
  int nrdata[SPL_NMAX + 2];                // 1-based
  double Gw[4][SPL_NK][SPL_KMAX + 1];      // per-wave partial sums
  double Zw[4][SPL_NK][3];
  double fpw[4][SPL_NK + 2];
  double fpsw[4];
  double scan[SPL_THREADS];
  double kap[SPL_THREADS];
  int kval[SPL_THREADS];
  double ev[9][SPL_THREADS];               // samples: r, r', r'' x 3 dims
  double fp, sumdiag;
  int n, phase, bad, smooth;
};

enum { PH_LSQ = 0, PH_SMOOTH = 1, PH_DONE = 2, PH_FAIL = 3, PH_HOST = 4 };

RDP_DEV double wsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);  // pairwise-commutative: same on all lanes
  return v;
}
RDP_DEV int wmin(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
RDP_DEV int wmax(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// FITPACK fpbspl: the K+1 non-zero B-splines of degree K at x, t1 1-based (t1[l] <= x < t1[l+1]);
// h[1..K+1]
template <int K>
RDP_DEV void bspl(const double* t1, double x, int l, double* h) {
  double hh[K + 2];
  h[1] = 1.0;
#pragma unroll
  for (int j = 1; j <= K; ++j) {
#pragma unroll
    for (int i = 1; i <= j; ++i) hh[i] = h[i];
    h[1] = 0.0;
#pragma unroll
    for (int i = 1; i <= j; ++i) {
      const int li = l + i, lj = li - j;
      const double a = t1[li], b = t1[lj];
      if (a == b) {
        h[i + 1] = 0.0;
        continue;
      }
      const double f = hh[i] / (a - b);
      h[i] = h[i] + f * (a - x);
      h[i + 1] = f * (x - b);
    }
  }
}

// largest l in [k1, nk1] with t1[l] <= u (FITPACK's interval of u, last interval closed)
RDP_DEV int find_l(const double* t1, int k1, int nk1, double u) {
  int lo = k1, hi = nk1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t1[mid] <= u) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// A^T A (band K+1) and A^T x for the current knots, deterministic (per-wave copies, fixed sum order)
template <int K>
RDP_DEV void gram_pass(SplSh& S, const double* __restrict__ P, const double* __restrict__ U, int m, int nk1) {
  constexpr int K1 = K + 1;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < 4 * SPL_NK; i += SPL_THREADS) {
    const int ww = i / SPL_NK, r = i % SPL_NK;
#pragma unroll
    for (int d = 0; d < K1; ++d) S.Gw[ww][r][d] = 0.0;
#pragma unroll
    for (int d = 0; d < 3; ++d) S.Zw[ww][r][d] = 0.0;
  }
  __syncthreads();
  const int per = (m + 3) / 4, b0 = w * per, b1 = min(m, b0 + per);
  for (int base = b0; base < b1; base += 64) {
    const int it = base + lane;
    const bool act = it < b1;
    double h[K1 + 1], x[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int a = 0; a <= K1; ++a) h[a] = 0.0;
    int l = 0;
    if (act) {
      const double u = U[it];
      l = find_l(S.t, K1, nk1, u);
      bspl<K>(S.t, u, l, h);
      x[0] = P[(size_t)it * 3];
      x[1] = P[(size_t)it * 3 + 1];
      x[2] = P[(size_t)it * 3 + 2];
    }
    const int lmin = wmin(act ? l : 0x7fffffff), lmax = wmax(act ? l : -1);
    constexpr int NG = K1 * (K1 + 1) / 2, NV = NG + 3 * K1;  // band products + right-hand sides
    for (int v = lmin; v <= lmax; ++v) {
      const bool sel = act && l == v;
      if (!__any(sel)) continue;
      const int r0 = v - K1;  // 0-based row of the interval's first coefficient
      // all NV products of this lane, then ONE step-major butterfly over them: the NV shuffle chains
      // are independent, so their LDS-permute latencies overlap (value-major wsums serialised them:
      // ~6.6 us per pass at 1 interval)
      double q[NV];
      {
        int k = 0;
#pragma unroll
        for (int a = 0; a < K1; ++a)
#pragma unroll
          for (int bb = a; bb < K1; ++bb) q[k++] = sel ? h[a + 1] * h[bb + 1] : 0.0;
#pragma unroll
        for (int a = 0; a < K1; ++a)
#pragma unroll
          for (int d = 0; d < 3; ++d) q[k++] = sel ? h[a + 1] * x[d] : 0.0;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int k = 0; k < NV; ++k) q[k] += __shfl_xor(q[k], o, 64);
      if (lane == 0) {
        int k = 0;
#pragma unroll
        for (int a = 0; a < K1; ++a)
#pragma unroll
          for (int bb = a; bb < K1; ++bb) S.Gw[w][r0 + a][bb - a] += q[k++];
#pragma unroll
        for (int a = 0; a < K1; ++a)
#pragma unroll
          for (int d = 0; d < 3; ++d) S.Zw[w][r0 + a][d] += q[k++];
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < nk1; i += SPL_THREADS) {
#pragma unroll
    for (int d = 0; d < K1; ++d) S.G[i][d] = ((S.Gw[0][i][d] + S.Gw[1][i][d]) + S.Gw[2][i][d]) + S.Gw[3][i][d];
#pragma unroll
    for (int d = 0; d < 3; ++d) S.Z[i][d] = ((S.Zw[0][i][d] + S.Zw[1][i][d]) + S.Zw[2][i][d]) + S.Zw[3][i][d];
  }
  __syncthreads();
}

// fp = sum of squared residuals of S.c; with fpint also FITPACK's per-interval residuals
template <int K>
RDP_DEV void resid_pass(SplSh& S, const double* __restrict__ P, const double* __restrict__ U, int m, int nk1,
                        bool want_fpint) {
  constexpr int K1 = K + 1;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nrint = nk1 - K;  // intervals
  for (int i = tid; i < 4 * (SPL_NK + 2); i += SPL_THREADS) S.fpw[i / (SPL_NK + 2)][i % (SPL_NK + 2)] = 0.0;
  if (tid < 4) S.fpsw[tid] = 0.0;
  __syncthreads();
  const int per = (m + 3) / 4, b0 = w * per, b1 = min(m, b0 + per);
  for (int base = b0; base < b1; base += 64) {
    const int it = base + lane;
    const bool act = it < b1;
    double term = 0.0;
    int iv = 0, newk = 0;
    if (act) {
      const double u = U[it];
      const int l = find_l(S.t, K1, nk1, u);
      double h[K1 + 1];
      bspl<K>(S.t, u, l, h);
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        double f = 0.0;
#pragma unroll
        for (int j = 1; j <= K1; ++j) f += S.c[d][l - K1 + j - 1] * h[j];
        const double r = f - P[(size_t)it * 3 + d];
        term += r * r;
      }
      iv = l - K1;
      if (want_fpint && it > 0) newk = find_l(S.t, K1, nk1, U[it - 1]) < l;
    }
    const double tsum = wsum(term);
    if (lane == 0) S.fpsw[w] += tsum;
    if (want_fpint) {
      const double w2 = newk ? term * 0.5 : 0.0, w1 = term - w2;
      const int lmin = wmin(act ? iv - 1 : 0x7fffffff), lmax = wmax(act ? iv : -1);
      for (int v = max(lmin, 0); v <= lmax; ++v) {
        const double q = wsum(act ? ((iv == v ? w1 : 0.0) + (iv - 1 == v ? w2 : 0.0)) : 0.0);
        if (lane == 0) S.fpw[w][v] += q;
      }
    }
  }
  __syncthreads();
  if (tid == 0) S.fp = ((S.fpsw[0] + S.fpsw[1]) + S.fpsw[2]) + S.fpsw[3];
  if (want_fpint)
    for (int i = tid; i < nrint; i += SPL_THREADS)
      S.fpint[i + 1] = ((S.fpw[0][i] + S.fpw[1][i]) + S.fpw[2][i]) + S.fpw[3][i];
  __syncthreads();
}

// Banded Cholesky + both triangular solves for the system A = G + p2i * BtB (band KB; G has band
// K1 <= KB, BtB = B^T B of the fpdisc rows when smoothing, p2i = p^-2), A c = Z for 3 right-hand
// sides; c -> S.c. Thread 0 only, but the row recurrences run in registers: a sliding window of the
// last KB rows of R (compile-time indexed) and of the forward-substitution values, so each row costs
// ~KB^2/2 register FMAs plus its KB loads of G / BtB / Z -- no LDS round trip inside the
// dependency chain (the LDS-latency-bound form took ~30 us per solve). R rows are stored once for
// the back substitution, which also keeps its c window in registers. false: non-positive pivot.
template <int KB, int K1>
RDP_DEV bool chol_solve(SplSh& S, int nk1, double p2i) {
  double win[KB][KB];  // win[q]: R row (i - (KB-1) + q), entries d = 0..KB-1 (rows < 0: zeros)
  double yw[3][KB];
#pragma unroll
  for (int q = 0; q < KB; ++q) {
#pragma unroll
    for (int d = 0; d < KB; ++d) win[q][d] = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) yw[k][q] = 0.0;
  }
  for (int i = 0; i < nk1; ++i) {
#pragma unroll
    for (int q = 0; q < KB - 1; ++q) {
#pragma unroll
      for (int d = 0; d < KB; ++d) win[q][d] = win[q + 1][d];
#pragma unroll
      for (int k = 0; k < 3; ++k) yw[k][q] = yw[k][q + 1];
    }
    double a[KB];
#pragma unroll
    for (int d = 0; d < KB; ++d) {
      const bool in = i + d < nk1;
      double v = (d < K1 && in) ? S.G[i][d] : 0.0;
      if (p2i != 0.0 && in) v += p2i * S.A[i][d];  // S.A holds B^T B while smoothing
      a[d] = v;
    }
    double r0 = 0.0, inv = 0.0;
#pragma unroll
    for (int d = 0; d < KB; ++d) {
      double sacc = a[d];
#pragma unroll
      for (int q = d; q < KB - 1; ++q) sacc -= win[q][KB - 1 - q] * win[q][KB - 1 - q + d];
      if (d == 0) {
        if (!(sacc > 0.0)) return false;
        r0 = sqrt(sacc);
        inv = 1.0 / r0;
        win[KB - 1][0] = r0;
      } else {
        win[KB - 1][d] = (i + d < nk1) ? sacc * inv : 0.0;
      }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      double sacc = S.Z[i][k];
#pragma unroll
      for (int q = 0; q < KB - 1; ++q) sacc -= win[q][KB - 1 - q] * yw[k][q];
      yw[k][KB - 1] = sacc * inv;
      S.y[k][i] = yw[k][KB - 1];
    }
#pragma unroll
    for (int d = 0; d < KB; ++d) S.R[i][d] = win[KB - 1][d];
  }
  double cw[3][KB];  // cw[k][d] = c_{i + 1 + d}
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int d = 0; d < KB; ++d) cw[k][d] = 0.0;
  for (int i = nk1 - 1; i >= 0; --i) {
    double r[KB];
#pragma unroll
    for (int d = 0; d < KB; ++d) r[d] = S.R[i][d];
    const double inv = 1.0 / r[0];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      double sacc = S.y[k][i];
#pragma unroll
      for (int d = 1; d < KB; ++d) sacc -= r[d] * cw[k][d - 1];
      const double ci = sacc * inv;
#pragma unroll
      for (int d = KB - 1; d > 0; --d) cw[k][d] = cw[k][d - 1];
      cw[k][0] = ci;
      S.c[k][i] = ci;
    }
  }
  return true;
}

// FITPACK fpknot (1-based arrays; x = u)
RDP_DEV void fpknot_dev(const double* __restrict__ U, double* t, int& n, double* fpint, int* nrdata, int& nrint,
                        int k) {
  double fpmax = 0.0;
  int number = 0, maxpt = 0, maxbeg = 0, jbegin = 1;
  for (int j = 1; j <= nrint; ++j) {
    const int jpoint = nrdata[j];
    if (!(fpmax >= fpint[j] || jpoint == 0)) {
      fpmax = fpint[j];
      number = j;
      maxpt = jpoint;
      maxbeg = jbegin;
    }
    jbegin = jbegin + jpoint + 1;
  }
  const int ihalf = maxpt / 2 + 1;
  const int nrx = maxbeg + ihalf;
  const int next = number + 1;
  if (next <= nrint) {
    for (int j = next; j <= nrint; ++j) {
      const int jj = next + nrint - j;
      fpint[jj + 1] = fpint[jj];
      nrdata[jj + 1] = nrdata[jj];
      const int jk = jj + k;
      t[jk + 1] = t[jk];
    }
  }
  nrdata[number] = ihalf - 1;
  nrdata[next] = maxpt - ihalf;
  const double am = maxpt;
  fpint[number] = fpmax * (double)nrdata[number] / am;
  fpint[next] = fpmax * (double)nrdata[next] / am;
  t[next + k] = U[nrx - 1];
  ++n;
  ++nrint;
}

// FITPACK fpdisc into S.B (0-based rows, K+2 columns)
template <int K>
RDP_DEV void fpdisc_dev(SplSh& S, int n) {
  constexpr int K1 = K + 1, K2 = K + 2;
  const double* t = S.t;
  const int nk1 = n - K1, nrint = nk1 - K;
  const double fac = (double)nrint / (t[nk1 + 1] - t[K1]);
  double h[2 * K2 + 2];
  for (int l = K2; l <= nk1; ++l) {
    const int lmk = l - K1;
    for (int j = 1; j <= K1; ++j) {
      const int ik = j + K1, lj = l + j, lk = lj - K2;
      h[j] = t[l] - t[lk];
      h[ik] = t[l] - t[lj];
    }
    int lp = lmk;
    for (int j = 1; j <= K2; ++j) {
      int jk = j;
      double prod = h[j];
      for (int i = 1; i <= K; ++i) {
        ++jk;
        prod = prod * h[jk] * fac;
      }
      const int lk = lp + K1;
      S.B[lmk - 1][j - 1] = (t[lk] - t[lp]) / prod;
      ++lp;
    }
  }
}

RDP_DEV double fprati_dev(double& p1, double& f1, double p2, double f2, double& p3, double& f3) {
  double p;
  if (p3 > 0.0) {
    const double h1 = f1 * (f2 - f3), h2 = f2 * (f3 - f1), h3 = f3 * (f1 - f2);
    p = -(p1 * p2 * h3 + p2 * p3 * h1 + p3 * p1 * h2) / (p1 * h1 + p2 * h2 + p3 * h3);
  } else {
    p = (p1 * (f1 - f3) * f2 - p2 * (f2 - f3) * f1) / ((f1 - f2) * f3);
  }
  if (f2 < 0.0) {
    p3 = p2;
    f3 = f2;
  } else {
    p1 = p2;
    f1 = f2;
  }
  return p;
}

// the three coordinates of a degree-KK spline (coefficients cd, knots t1 + lo, nn knots) at x: one
// interval search and basis, then per coordinate the arithmetic of rdp_splev1 (csrc/spline.cpp)
template <int KK>
RDP_DEV void splev3_dev(const double* t1, int lo, int nn, const double (*cd)[SPL_NK], int ncd, double x,
                        double (*out)[SPL_THREADS], int j) {
  const double* tt = t1 + lo;
  int l = KK;
  while (l < nn - KK - 2 && x >= tt[l + 2]) ++l;
  double h[KK + 2];
  bspl<KK>(tt, x, l + 1, h);
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    double s = 0.0;
#pragma unroll
    for (int jj = 1; jj <= KK + 1; ++jj) {
      const int ci = l - KK + jj - 1;
      if (ci >= 0 && ci < ncd) s += cd[d][ci] * h[jj];
    }
    out[d][j] = s;
  }
}

template <int K>
RDP_DEV void geo_fit_body(const double* __restrict__ P, double* __restrict__ U,
                                                              const int* __restrict__ kout, int nbins, int kcap,
                                                              const int* __restrict__ npts_p, int ecap, double s,
                                                              int nsamp, double eps, int min_points, int min_edge,
                                                              const int* __restrict__ cov, int ncov,
                                                              double* __restrict__ res, double* __restrict__ dbg,
                                                              const uint32_t* __restrict__ hsrc,
                                                              uint32_t* __restrict__ hdst, int hwords) {
  if (blockIdx.x > 0) {
    // blocks 1.. (serving): the frame mask's copy into host memory (4-B words) beside the one fit block,
    // on CUs it leaves idle -- written by geo_count it lengthened that kernel by ~4.5 us of its 9.4
    const int i = ((int)blockIdx.x - 1) * SPL_THREADS + (int)threadIdx.x;
    if (i < hwords) hdst[i] = hsrc[i];
    return;
  }
  constexpr int K1 = K + 1, K2 = K + 2, nmin = 2 * K1;
  constexpr int NCAP = SPL_NK + K1;  // max knots: nk1 = n - K1 <= SPL_NK coefficients
  __shared__ SplSh S;
  const int tid = threadIdx.x;
  // optional phase profile (dbg != nullptr, thread 0): 100 MHz realtime ticks per phase + counts.
  // [0] m [1] LSQ iterations [2] smoothing iterations [3] total [4] setup [5] gram [6] chol LSQ
  // [7] resid LSQ [8] knot control [9] BtB [10] chol smooth [11] resid smooth [12] eval [13] n
  // [14..18] eval sub-phases: derivative coefficients, samples, curvature, reductions, result write
  uint64_t t_last = 0;
  double prof[20] = {0.0};
  auto stamp = [&](int slot) {
    if (dbg != nullptr && tid == 0) {
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (slot >= 0) prof[slot] += (double)(now - t_last);
      t_last = now;
    }
  };
  stamp(-1);
  const uint64_t t_start = t_last;
  auto prof_flush = [&]() {
    if (dbg != nullptr && tid == 0) {
      stamp(12);
      prof[3] = (double)(t_last - t_start);
      for (int i = 0; i < 20; ++i) dbg[i] = prof[i];
    }
  };
  {  // edge-point count = the packed length of the per-bin slabs; coverage = sum of the row blocks
    int e = 0, c = 0;
    for (int b = tid; b < nbins; b += SPL_THREADS) e += min(kout[b], kcap);
    if (cov)
      for (int b = tid; b < ncov; b += SPL_THREADS) c += cov[b];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      e += __shfl_xor(e, o, 64);
      c += __shfl_xor(c, o, 64);
    }
    if ((tid & 63) == 0) {
      S.kval[tid >> 6] = e;
      S.kval[4 + (tid >> 6)] = c;
    }
    __syncthreads();
    if (tid == 0) {
      S.n = S.kval[0] + S.kval[1] + S.kval[2] + S.kval[3];
      res[8 + 3 * nsamp] = cov ? (double)(S.kval[4] + S.kval[5] + S.kval[6] + S.kval[7]) : -1.0;
    }
  }
  __syncthreads();
  const int m = min(S.n, ecap), np = npts_p[0];
  __syncthreads();
  auto finish_status = [&](int st, int ier, int n, double fp) {
    if (tid == 0) {
      res[0] = st; res[1] = ier; res[2] = n; res[3] = fp; res[4] = 0.0; res[5] = 0.0; res[6] = m; res[7] = np;
    }
  };
  if (np < min_points) { finish_status(SPL_TOO_FEW_POINTS, 0, 0, 0.0); return; }
  if (m < min_edge) { finish_status(SPL_TOO_FEW_EDGES, 0, 0, 0.0); return; }
  if (m <= K || s < 0.0) { finish_status(SPL_FIT_FAILED, 10, 0, 0.0); return; }
  // ---- chord-length parameters: contiguous chunk per thread, sequential scan of the chunk sums ----
  const int per = (m + SPL_THREADS - 1) / SPL_THREADS, c0 = min(m, tid * per), c1 = min(m, c0 + per);
  double run = 0.0;
  for (int i = c0; i < c1; ++i) {
    if (i > 0) {
      double d2 = 0.0;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const double d = P[(size_t)i * 3 + j] - P[(size_t)(i - 1) * 3 + j];
        d2 += d * d;
      }
      run += sqrt(d2);
    }
    U[i] = run;
  }
  {  // exclusive block scan of the chunk lengths: wave shfl scans + the 4 wave totals (fixed order)
    const int lane = tid & 63, w = tid >> 6;
    double incl = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) S.scan[w] = incl;
    if (tid == 0) S.bad = 0;
    __syncthreads();
    double wbase = 0.0;
    for (int q = 0; q < w; ++q) wbase += S.scan[q];
    const double total_all = ((S.scan[0] + S.scan[1]) + S.scan[2]) + S.scan[3];
    __syncthreads();
    S.scan[tid] = wbase + incl - run;  // exclusive prefix of this thread's chunk
    if (tid == 0) S.fp = total_all;    // total chord length
  }
  __syncthreads();
  const double base = S.scan[tid], total = S.fp;
  if (!(total > 0.0)) { finish_status(SPL_FIT_FAILED, 10, 0, 0.0); return; }
  for (int i = c0; i < c1; ++i) U[i] = (base + U[i]) / total;
  __syncthreads();  // one workgroup: its global writes are visible to it after the barrier
  {
    int bad = 0;
    for (int i = max(c0, 1); i < c1; ++i) bad |= U[i] <= U[i - 1];
    if (bad) S.bad = 1;  // benign race: every writer stores 1
  }
  __syncthreads();
  if (S.bad) { finish_status(SPL_FIT_FAILED, 10, 0, 0.0); return; }

  // ---- FITPACK fppara (iopt = 0, unit weights); scalar control on thread 0 ----
  const double tol = 0.001, con1 = 0.1, con9 = 0.9, con4 = 0.04, acc = tol * s;
  const int maxit = 20, nmax = m + K1, nest = m + 2 * K;
  const double ub = U[0], ue = U[m - 1];
  int ier = 0, nplus = 0;  // thread 0 only
  double fp0 = 0.0, fpold = 0.0, fpms = 0.0;
  stamp(4);
  if (tid == 0) {
    prof[0] = m;
    S.n = nmin;
    S.phase = PH_LSQ;
    S.nrdata[1] = m - 2;
    if (s == 0.0) {  // interpolating spline: knots at the data points
      S.n = nmax;
      if (nmax > NCAP) S.phase = PH_HOST;
      else
        for (int i = K2, j = K / 2 + 2; i <= m; ++i, ++j) S.t[i] = U[j - 1];
    }
  }
  __syncthreads();
  for (int iter = 1; iter <= m; ++iter) {
    if (S.phase != PH_LSQ) break;
    const int n = S.n, nk1 = n - K1;
    if (tid == 0) {
      if (n == nmin) ier = -2;
      for (int j = 1, i = n; j <= K1; ++j, --i) {
        S.t[j] = ub;
        S.t[i] = ue;
      }
    }
    __syncthreads();
    stamp(8);
    gram_pass<K>(S, P, U, m, nk1);
    stamp(5);
    if (tid == 0) {
      double sd = 0.0;
      if (!chol_solve<K1, K1>(S, nk1, 0.0)) S.phase = PH_HOST;
      for (int i = 0; i < nk1; ++i) sd += S.R[i][0];
      S.sumdiag = sd;
      prof[1] += 1.0;
    }
    __syncthreads();
    stamp(6);
    if (S.phase != PH_LSQ) break;
    resid_pass<K>(S, P, U, m, nk1, true);
    stamp(7);
    if (tid == 0) {
      const double fp = S.fp;
      int nn = n;
      if (ier == -2) fp0 = fp;
      fpms = fp - s;
      if (fabs(fpms) < acc) {
        S.phase = PH_DONE;
      } else if (fpms < 0.0) {
        S.phase = PH_SMOOTH;
      } else if (n == nmax) {
        ier = -1;
        S.phase = PH_DONE;
      } else if (n == nest) {
        ier = 1;
        S.phase = PH_DONE;
      } else {
        if (ier != 0) {
          nplus = 1;
          ier = 0;
        } else {
          int npl1 = nplus * 2;
          const double rn = nplus;
          if (fpold - fp > acc) npl1 = (int)(rn * fpms / (fpold - fp));
          nplus = min(nplus * 2, max(max(npl1, nplus / 2), 1));
        }
        fpold = fp;
        int nr = n - nmin + 1;
        for (int ll = 1; ll <= nplus; ++ll) {
          if (nn + 1 > NCAP) {
            S.phase = PH_HOST;
            break;
          }
          fpknot_dev(U, S.t, nn, S.fpint, S.nrdata, nr, K);
          if (nn == nmax || nn == nest) break;
        }
        if (nn == nmax && S.phase == PH_LSQ)
          for (int ii = K2, j = K / 2 + 2; ii <= m; ++ii, ++j) S.t[ii] = U[j - 1];
        S.n = nn;
      }
    }
    __syncthreads();
    stamp(8);
  }
  if (S.phase == PH_HOST) { finish_status(SPL_NEEDS_HOST, 0, S.n, 0.0); return; }

  // ier lives on thread 0: publish the block-uniform decision through LDS (a per-thread test here
  // sent threads 1..255 through 20 idle smoothing iterations, ~27 us, whenever the polynomial fit
  // already met s -- the common serving case)
  if (tid == 0) S.smooth = S.phase == PH_SMOOTH && ier != -2;
  __syncthreads();
  if (S.smooth) {
    // ---- smoothing spline: p with fp(p) = s by rational interpolation ----
    const int n = S.n, nk1 = n - K1, n8 = n - nmin;
    double p1 = 0.0, f1 = 0.0, p3 = -1.0, f3 = 0.0, p = 0.0;
    int ich1 = 0, ich3 = 0;
    if (tid == 0) {
      fpdisc_dev<K>(S, n);
      f1 = fp0 - s;
      f3 = fpms;
      p = (double)nk1 / S.sumdiag;
      S.phase = PH_SMOOTH;
    }
    __syncthreads();
    stamp(8);
    // B^T B (band K2) once for all p: A[i][d] = sum_a B[i-a][a] * B[i-a][a+d], in parallel
    for (int e = tid; e < nk1 * K2; e += SPL_THREADS) {
      const int i = e / K2, d = e - (e / K2) * K2;
      double v = 0.0;
      for (int a = 0; a + d < K2; ++a) {
        const int r = i - a;
        if (r >= 0 && r < n8 && i + d < nk1) v += S.B[r][a] * S.B[r][a + d];
      }
      S.A[i][d] = v;
    }
    __syncthreads();
    stamp(9);
    for (int iter = 1; iter <= maxit; ++iter) {
      if (tid == 0) {
        const double pinv = 1.0 / p, p2i = pinv * pinv;
        if (!chol_solve<K2, K1>(S, nk1, p2i)) S.phase = PH_HOST;
        prof[2] += 1.0;
      }
      __syncthreads();
      stamp(10);
      if (S.phase == PH_HOST) break;
      resid_pass<K>(S, P, U, m, nk1, false);
      stamp(11);
      if (tid == 0) {
        const double fp = S.fp;
        fpms = fp - s;
        bool stop = false;
        if (fabs(fpms) < acc) {
          ier = 0;
          stop = true;
        } else if (iter == maxit) {
          ier = 3;
          stop = true;
        } else {
          const double p2 = p, f2 = fpms;
          bool next = false;
          if (ich3 == 0) {
            if (!((f2 - f3) > acc)) {
              p3 = p2;
              f3 = f2;
              p = p * con4;
              if (p <= p1) p = p1 * con9 + p2 * con1;
              next = true;
            } else if (f2 < 0.0) {
              ich3 = 1;
            }
          }
          if (!next && ich1 == 0) {
            if (!((f1 - f2) > acc)) {
              p1 = p2;
              f1 = f2;
              p = p / con4;
              if (p3 >= 0.0 && p >= p3) p = p2 * con1 + p3 * con9;
              next = true;
            } else if (f2 > 0.0) {
              ich1 = 1;
            }
          }
          if (!next) {
            if (f2 >= f1 || f2 <= f3) {
              ier = 2;
              stop = true;
            } else {
              p = fprati_dev(p1, f1, p2, f2, p3, f3);
            }
          }
        }
        if (stop) S.phase = PH_DONE;
      }
      __syncthreads();
      stamp(8);
      if (S.phase != PH_SMOOTH) break;
    }
    if (S.phase == PH_HOST) { finish_status(SPL_NEEDS_HOST, 0, S.n, 0.0); return; }
  }

  // ---- evaluation: r, r', r'' at nsamp parameters; kappa = |r' x r''| / |r'|^3 ----
  const int n = S.n, nk1 = n - K1;
  if (tid == 0) prof[13] = n;
  for (int i = tid; i < 3 * nk1; i += SPL_THREADS) {  // first-derivative coefficients (splder)
    const int d = i / nk1, j = i % nk1;
    if (j < nk1 - 1) {
      const double den = S.t[j + K1 + 1] - S.t[j + 2];
      S.cd1[d][j] = den > 0.0 ? K * (S.c[d][j + 1] - S.c[d][j]) / den : 0.0;
    }
  }
  __syncthreads();
  stamp(14);
  for (int i = tid; i < 3 * nk1; i += SPL_THREADS) {  // second derivative
    const int d = i / nk1, j = i % nk1;
    if (j < nk1 - 2) {
      const double den = S.t[j + K1 + 1] - S.t[j + 3];
      S.cd2[d][j] = den > 0.0 ? (K - 1) * (S.cd1[d][j + 1] - S.cd1[d][j]) / den : 0.0;
    }
  }
  __syncthreads();
  stamp(14);
  // 3 x nsamp items (derivative order q, sample j): one interval search + basis per item for all three
  // coordinates, spread over the block. (One thread per sample running the 9 evaluations inline made
  // this phase ~30 us: a large cold code footprint executed once per launch.)
  for (int it = tid; it < 3 * nsamp; it += SPL_THREADS) {
    const int q = it / nsamp, j = it - q * nsamp;
    const double x = nsamp > 1 ? (double)j / (double)(nsamp - 1) : 0.0;
    if (q == 0) {
      splev3_dev<K>(S.t, 0, n, S.c, nk1, x, S.ev, j);
    } else if (q == 1) {
      splev3_dev<K - 1>(S.t, 1, n - 2, S.cd1, nk1 - 1, x, S.ev + 3, j);
    } else {
      if constexpr (K >= 2) splev3_dev<K - 2>(S.t, 2, n - 4, S.cd2, nk1 - 2, x, S.ev + 6, j);
      else S.ev[6][j] = S.ev[7][j] = S.ev[8][j] = 0.0;
    }
  }
  __syncthreads();
  stamp(15);
  if (tid < nsamp) {
    double d1[3], d2[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      res[8 + (size_t)tid * 3 + d] = S.ev[d][tid];
      d1[d] = S.ev[3 + d][tid];
      d2[d] = S.ev[6 + d][tid];
    }
    const double cx = d1[1] * d2[2] - d1[2] * d2[1], cy = d1[2] * d2[0] - d1[0] * d2[2],
                 cz = d1[0] * d2[1] - d1[1] * d2[0];
    const double nd = sqrt(d1[0] * d1[0] + d1[1] * d1[1] + d1[2] * d1[2]);
    S.kval[tid] = nd > eps;
    S.kap[tid] = nd > eps ? sqrt(cx * cx + cy * cy + cz * cz) / (nd * nd * nd) : 0.0;
  }
  __syncthreads();
  stamp(16);
  {  // mean / max over the samples with |r'| > eps: wave reductions, waves combined in order
    const bool v = tid < nsamp && S.kval[tid];
    double ks = v ? S.kap[tid] : 0.0, km = v ? S.kap[tid] : 0.0;
    int kc = v ? 1 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      ks += __shfl_xor(ks, o, 64);
      km = fmax(km, __shfl_xor(km, o, 64));
      kc += __shfl_xor(kc, o, 64);
    }
    __syncthreads();
    if ((tid & 63) == 0) {
      S.kap[tid >> 6] = ks;
      S.kap[4 + (tid >> 6)] = km;
      S.kval[tid >> 6] = kc;
    }
    __syncthreads();
  }
  stamp(17);
  if (tid == 0) {
    const double ksum = ((S.kap[0] + S.kap[1]) + S.kap[2]) + S.kap[3];
    const double kmax = fmax(fmax(S.kap[4], S.kap[5]), fmax(S.kap[6], S.kap[7]));
    const int cnt = S.kval[0] + S.kval[1] + S.kval[2] + S.kval[3];
    res[0] = SPL_OK;
    res[1] = ier;
    res[2] = n;
    res[3] = S.fp;
    res[4] = cnt ? ksum / cnt : 0.0;
    res[5] = cnt ? kmax : 0.0;
    res[6] = m;
    res[7] = np;
  }
  stamp(18);
  prof_flush();
}

template <int K>
__global__ __launch_bounds__(SPL_THREADS) void geo_fit_kernel(const double* __restrict__ P, double* __restrict__ U,
                                                              const int* __restrict__ kout, int nbins, int kcap,
                                                              const int* __restrict__ npts_p, int ecap, double s,
                                                              int nsamp, double eps, int min_points, int min_edge,
                                                              const int* __restrict__ cov, int ncov,
                                                              double* __restrict__ res, double* __restrict__ dbg,
                                                              const uint32_t* __restrict__ hsrc,
                                                              uint32_t* __restrict__ hdst, int hwords) {
  geo_fit_body<K>(P, U, kout, nbins, kcap, npts_p, ecap, s, nsamp, eps, min_points, min_edge, cov, ncov, res, dbg,
                  hsrc, hdst, hwords);
}

// up to 4 frames' fits in one launch (blockIdx.y = frame; blocks 1.. of each row copy that frame's mask)
struct FitFrame {
  const double* P;
  double* U;
  const int* kout;
  const int* npts;
  const int* cov;
  double* res;
  const uint32_t* hsrc;
  uint32_t* hdst;
};
struct FitFrames {
  FitFrame f[4];
  int nbins, kcap, ecap, nsamp, min_points, min_edge, ncov, hwords;
  double s, eps;
};
template <int K>
__global__ __launch_bounds__(SPL_THREADS) void geo_fit_batch_kernel(const FitFrames g) {
  const FitFrame& a = g.f[blockIdx.y];
  geo_fit_body<K>(a.P, a.U, a.kout, g.nbins, g.kcap, a.npts, g.ecap, g.s, g.nsamp, g.eps, g.min_points, g.min_edge,
                  a.cov, g.ncov, a.res, nullptr, a.hsrc, a.hdst, g.hwords);
}

extern "C" {
int rdp_geo_spline_res_len(int nsamp) { return 9 + 3 * nsamp; }

// rdp_geo_spline (presorted, serving) for n <= 4 frames in one launch: per-frame arrays of its buffers
int rdp_geo_spline_batch(int n, int nbins, int kcap, const int* const* kout, const int* const* npts,
                         double* const* sorted, double* const* u, int ecap, double s, int k, int nsamp, double eps,
                         int min_points, int min_edge, const int* const* cov, int ncov, double* const* res,
                         const void* const* mask, void* const* mask_host, long mask_bytes, hipStream_t st) {
  if (k < 1 || k > SPL_KMAX || nsamp < 1 || nsamp > SPL_THREADS || n < 1 || n > 4) return -1;
  if (mask_host && mask_bytes % 4) return -2;
  FitFrames g;
  g.nbins = nbins; g.kcap = kcap; g.ecap = ecap; g.nsamp = nsamp; g.min_points = min_points; g.min_edge = min_edge;
  g.ncov = ncov; g.s = s; g.eps = eps;
  g.hwords = mask_host ? (int)(mask_bytes / 4) : 0;
  for (int i = 0; i < 4; ++i) {
    const int j = i < n ? i : 0;
    FitFrame& f = g.f[i];
    f.P = sorted[j]; f.U = u[j]; f.kout = kout[j]; f.npts = npts[j]; f.cov = cov[j]; f.res = res[j];
    f.hsrc = mask_host ? (const uint32_t*)mask[j] : nullptr;
    f.hdst = mask_host ? (uint32_t*)mask_host[j] : nullptr;
    if (mask_host && ((((uintptr_t)mask[j]) | ((uintptr_t)mask_host[j])) & 3)) return -2;
  }
  const int grid = 1 + (g.hwords + SPL_THREADS - 1) / SPL_THREADS;
  switch (k) {
    case 1: hipLaunchKernelGGL(geo_fit_batch_kernel<1>, dim3(grid, n), dim3(SPL_THREADS), 0, st, g); break;
    case 2: hipLaunchKernelGGL(geo_fit_batch_kernel<2>, dim3(grid, n), dim3(SPL_THREADS), 0, st, g); break;
    case 3: hipLaunchKernelGGL(geo_fit_batch_kernel<3>, dim3(grid, n), dim3(SPL_THREADS), 0, st, g); break;
    case 4: hipLaunchKernelGGL(geo_fit_batch_kernel<4>, dim3(grid, n), dim3(SPL_THREADS), 0, st, g); break;
    default: hipLaunchKernelGGL(geo_fit_batch_kernel<5>, dim3(grid, n), dim3(SPL_THREADS), 0, st, g); break;
  }
  return 0;
}

// sort the per-bin edge points (out [nbins][kcap][4], kout) into sorted [ecap][3] and fit/evaluate.
int rdp_geo_spline(const double* out, int nbins, int kcap, const int* kout, const int* npts, double* sorted,
                   int* gperm, double* u, int ecap, double s, int k, int nsamp, double eps, int min_points,
                   int min_edge, const int* cov, int ncov, double* res, double* dbg, int presorted,
                   const void* mask, void* mask_host, long mask_bytes, hipStream_t st) {
  if (k < 1 || k > SPL_KMAX || nsamp < 1 || nsamp > SPL_THREADS) return -1;
  // presorted: rdp_geo_edges already wrote `sorted` (fused select + sort)
  if (!presorted)
    hipLaunchKernelGGL(geo_sort_kernel, dim3(nbins), dim3(256), 0, st, out, kcap, kout, sorted, gperm, ecap);
  // mask_host: copy `mask` (device) into it with blocks beside the fit (4-B words; mask_bytes % 4 == 0)
  if (mask_host && (mask_bytes % 4 || (((uintptr_t)mask | (uintptr_t)mask_host) & 3))) return -2;
  const int hwords = mask_host ? (int)(mask_bytes / 4) : 0;
  const int grid = 1 + (hwords + SPL_THREADS - 1) / SPL_THREADS;
#define RDP_FIT(KK)                                                                                                 \
  hipLaunchKernelGGL(geo_fit_kernel<KK>, dim3(grid), dim3(SPL_THREADS), 0, st, sorted, u, kout, nbins, kcap, npts, \
                     ecap, s, nsamp, eps, min_points, min_edge, cov, ncov, res, dbg, (const uint32_t*)mask,        \
                     (uint32_t*)mask_host, hwords)
  switch (k) {
    case 1: RDP_FIT(1); break;
    case 2: RDP_FIT(2); break;
    case 3: RDP_FIT(3); break;
    case 4: RDP_FIT(4); break;
    default: RDP_FIT(5); break;
  }
#undef RDP_FIT
  return 0;
}
}
