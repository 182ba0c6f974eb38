// Parametric smoothing B-spline fit (FITPACK parcur/fppara semantics) + evaluation + curvature.
//
// Replaces scipy.interpolate.splprep / splev (Fortran FITPACK) that the reference calls in
// /root/reference/pkg/geometry_utils.py:78,84,148-149: splprep([x, y, z], s=0.1, k=3) with
// chord-length parameters u in [0, 1], unit weights, then 100-sample evaluation of r, r', r''.
//
// Algorithm (Dierckx, "Curve and Surface Fitting with Splines", ch. 5; FITPACK fppara):
//   1. start with no interior knots (least-squares polynomial); if its residual fp0 <= s the
//      polynomial is returned (ier = -2; the common case for the reference's s = 0.1 m^2);
//   2. otherwise add knots (fpknot: at the middle data point of the interval with the largest
//      residual, nplus chosen from the residual decrease) and refit by Givens QR of the banded
//      observation matrix until fp(inf) < s;
//   3. then find the smoothing parameter p with f(p) = fp - s = 0 by rational interpolation
//      (fprati), rotating the k-th-derivative-jump rows (fpdisc) weighted by 1/p into the
//      triangular system; tol = 0.001*s, maxit = 20.
// Indices below are 1-based (Fortran style) through small accessor lambdas to keep the
// control flow identical to the published algorithm.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

namespace {

struct Banded {  // n x w row-major (1-based access)
  int n, w;
  std::vector<double> d;
  Banded(int n_, int w_) : n(n_), w(w_), d((size_t)n_ * w_, 0.0) {}
  double& operator()(int i, int j) { return d[(size_t)(i - 1) * w + (j - 1)]; }
};

void fpgivs(double piv, double& ww, double& cs, double& sn) {
  const double store = std::fabs(piv);
  double dd;
  if (store >= ww) dd = store * std::sqrt(1.0 + (ww / piv) * (ww / piv));
  else dd = ww * std::sqrt(1.0 + (piv / ww) * (piv / ww));
  cs = ww / dd;
  sn = piv / dd;
  ww = dd;
}

void fprota(double cs, double sn, double& a, double& b) {
  const double s1 = a, s2 = b;
  b = cs * s2 + sn * s1;
  a = cs * s1 - sn * s2;
}

// values of the k+1 non-zero B-splines at x, t(l) <= x < t(l+1); t 1-based via pointer offset
void fpbspl(const double* t, int k, double x, int l, double* h) {
  double hh[20];
  h[1] = 1.0;
  for (int j = 1; j <= k; ++j) {
    for (int i = 1; i <= j; ++i) hh[i] = h[i];
    h[1] = 0.0;
    for (int i = 1; i <= j; ++i) {
      const int li = l + i, lj = li - j;
      if (t[li] == t[lj]) {
        h[i + 1] = 0.0;
        continue;
      }
      const double f = hh[i] / (t[li] - t[lj]);
      h[i] = h[i] + f * (t[li] - x);
      h[i + 1] = f * (x - t[lj]);
    }
  }
}

// solve upper-triangular banded a (bandwidth kb) * c = z
void fpback(Banded& a, const double* z, int n, int kb, double* c) {
  const int k1 = kb - 1;
  c[n] = z[n] / a(n, 1);
  int i = n - 1;
  for (int j = 2; j <= n; ++j) {
    double store = z[i];
    const int i1 = (j <= k1) ? j - 1 : k1;
    int m = i;
    for (int l = 1; l <= i1; ++l) {
      ++m;
      store -= c[m] * a(i, l + 1);
    }
    c[i] = store / a(i, 1);
    --i;
  }
}

// discontinuity jumps of the k-th derivative of the B-splines at the interior knots
void fpdisc(const double* t, int n, int k2, Banded& b) {
  const int k1 = k2 - 1, k = k1 - 1, nk1 = n - k1, nrint = nk1 - k;
  const double fac = (double)nrint / (t[nk1 + 1] - t[k1]);
  double h[24];
  for (int l = k2; l <= nk1; ++l) {
    const int lmk = l - k1;
    for (int j = 1; j <= k1; ++j) {
      const int ik = j + k1, lj = l + j, lk = lj - k2;
      h[j] = t[l] - t[lk];
      h[ik] = t[l] - t[lj];
    }
    int lp = lmk;
    for (int j = 1; j <= k2; ++j) {
      int jk = j;
      double prod = h[j];
      for (int i = 1; i <= k; ++i) {
        ++jk;
        prod = prod * h[jk] * fac;
      }
      const int lk = lp + k1;
      b(lmk, j) = (t[lk] - t[lp]) / prod;
      ++lp;
    }
  }
}

double fprati(double& p1, double& f1, double p2, double f2, double& p3, double& f3) {
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

void fpknot(const double* x, double* t, int& n, double* fpint, int* nrdata, int& nrint, int istart) {
  const int k = (n - nrint - 1) / 2;
  double fpmax = 0.0;
  int number = 0, maxpt = 0, maxbeg = 0, jbegin = istart;
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
  double an = nrdata[number];
  fpint[number] = fpmax * an / am;
  an = nrdata[next];
  fpint[next] = fpmax * an / am;
  const int jk = next + k;
  t[jk] = x[nrx];
  ++n;
  ++nrint;
}

}  // namespace

extern "C" {

// FITPACK fppara for iopt = 0, unit weights, ub = u[0], ue = u[m-1].
//   x: m points x idim (point-major); t: >= nest knots; c: >= nest*idim coefficients (dim-major,
//   stride nest). Returns ier (-2 polynomial, 0 ok, 1..3 FITPACK warnings, 10 invalid input).
int rdp_parcur(int idim, int m, const double* u_in, const double* x_in, double s, int k, int nest, double* t_out,
               double* c_out, int* n_out, double* fp_out) {
  if (k < 1 || k > 5 || m <= k || s < 0.0 || idim < 1 || idim > 10 || nest < 2 * (k + 1)) return 10;
  for (int i = 1; i < m; ++i)
    if (u_in[i] <= u_in[i - 1]) return 10;  // FITPACK: u strictly increasing (scipy: "Invalid inputs")
  const double tol = 0.001, con1 = 0.1, con9 = 0.9, con4 = 0.04, half = 0.5;
  const int maxit = 20, k1 = k + 1, k2 = k + 2, nmin = 2 * k1, nmax = m + k1;
  // 1-based working arrays
  std::vector<double> u(m + 1), t(nest + 2, 0.0), fpint(nest + 2, 0.0), z((size_t)nest * idim + 2, 0.0),
      c((size_t)nest * idim + 2, 0.0), q((size_t)m * k1 + 1, 0.0);
  std::vector<int> nrdata(nest + 2, 0);
  for (int i = 1; i <= m; ++i) u[i] = u_in[i - 1];
  auto X = [&](int it, int j) { return x_in[(size_t)(it - 1) * idim + (j - 1)]; };
  auto Q = [&](int it, int j) -> double& { return q[(size_t)(it - 1) * k1 + j]; };
  const double ub = u[1], ue = u[m];
  const double acc = tol * s;
  int n = nmin, ier = 0, nplus = 0;
  double fp = 0.0, fp0 = 0.0, fpold = 0.0, fpms = 0.0;
  nrdata[1] = m - 2;
  if (s == 0.0) {  // interpolating spline: knots at the data points
    n = nmax;
    if (n > nest) return 1;
    for (int i = k2, j = k / 2 + 2; i <= m; ++i, ++j) t[i] = u[j];
  }
  Banded a(nest, k1);
  bool done = false, to_smooth = false;
  for (int iter = 1; iter <= m && !done; ++iter) {
    if (n == nmin) ier = -2;
    const int nrint = n - nmin + 1;
    const int nk1 = n - k1;
    for (int j = 1, i = n; j <= k1; ++j, --i) {
      t[j] = ub;
      t[i] = ue;
    }
    fp = 0.0;
    std::fill(a.d.begin(), a.d.end(), 0.0);
    std::fill(z.begin(), z.end(), 0.0);
    int l = k1;
    double h[12], xi[10];
    for (int it = 1; it <= m; ++it) {
      const double ui = u[it];
      while (!(ui < t[l + 1] || l == nk1)) ++l;
      fpbspl(t.data(), k, ui, l, h);
      for (int i = 1; i <= k1; ++i) Q(it, i) = h[i];
      for (int j = 1; j <= idim; ++j) xi[j - 1] = X(it, j);
      int j0 = l - k1;
      for (int i = 1; i <= k1; ++i) {
        ++j0;
        const double piv = h[i];
        if (piv == 0.0) continue;
        double cs, sn;
        fpgivs(piv, a(j0, 1), cs, sn);
        for (int j = 1; j <= idim; ++j) fprota(cs, sn, xi[j - 1], z[j0 + (size_t)(j - 1) * n]);
        if (i == k1) break;
        for (int i1 = i + 1, i2 = 1; i1 <= k1; ++i1) {
          ++i2;
          fprota(cs, sn, h[i1], a(j0, i2));
        }
      }
      for (int j = 1; j <= idim; ++j) fp += xi[j - 1] * xi[j - 1];
    }
    if (ier == -2) fp0 = fp;
    for (int j = 1; j <= idim; ++j) fpback(a, &z[(size_t)(j - 1) * n], nk1, k1, &c[(size_t)(j - 1) * n]);
    fpms = fp - s;
    if (std::fabs(fpms) < acc) { done = true; break; }
    if (fpms < 0.0) { to_smooth = true; break; }
    if (n == nmax) { ier = -1; done = true; break; }
    if (n == nest) { ier = 1; done = true; break; }
    if (ier != 0) {
      nplus = 1;
      ier = 0;
    } else {
      int npl1 = nplus * 2;
      const double rn = nplus;
      if (fpold - fp > acc) npl1 = (int)(rn * fpms / (fpold - fp));
      nplus = std::min(nplus * 2, std::max(std::max(npl1, nplus / 2), 1));
    }
    fpold = fp;
    // residual sum per knot interval (points on a knot split half / half)
    double fpart = 0.0;
    int i = 1, newk = 0;
    l = k2;
    for (int it = 1; it <= m; ++it) {
      if (!(u[it] < t[l] || l > nk1)) {
        newk = 1;
        ++l;
      }
      double term = 0.0;
      for (int j2 = 1; j2 <= idim; ++j2) {
        double fac = 0.0;
        int l0 = l - k2;
        for (int j = 1; j <= k1; ++j) {
          ++l0;
          fac += c[l0 + (size_t)(j2 - 1) * n] * Q(it, j);
        }
        term += (fac - X(it, j2)) * (fac - X(it, j2));
      }
      fpart += term;
      if (newk == 0) continue;
      const double store = term * half;
      fpint[i] = fpart - store;
      ++i;
      fpart = store;
      newk = 0;
    }
    fpint[nrint] = fpart;
    int nr = nrint;
    for (int ll = 1; ll <= nplus; ++ll) {
      // coefficients are stored with stride n; when n grows, re-pack is unnecessary because they
      // are recomputed at the next iteration
      fpknot(u.data(), t.data(), n, fpint.data(), nrdata.data(), nr, 1);
      if (n == nmax || n == nest) break;
    }
    if (n == nmax) {  // locate knots as for interpolation
      for (int ii = k2, j = k / 2 + 2; ii <= m; ++ii, ++j) t[ii] = u[j];
    }
  }
  if (to_smooth && ier != -2) {
    // part 2: smoothing spline with f(p) = s
    const int nk1 = n - k1, n8 = n - nmin;
    Banded b(nest, k2), g(nest, k2);
    fpdisc(t.data(), n, k2, b);
    double p1 = 0.0, f1 = fp0 - s, p3 = -1.0, f3 = fpms, p = 0.0;
    for (int i = 1; i <= nk1; ++i) p += a(i, 1);
    p = (double)nk1 / p;
    int ich1 = 0, ich3 = 0;
    std::vector<double> cc((size_t)n * idim + 2, 0.0), zz((size_t)n * idim + 2);
    for (int iter = 1; iter <= maxit; ++iter) {
      const double pinv = 1.0 / p;
      for (int j = 1; j <= idim; ++j)
        for (int i = 1; i <= nk1; ++i) zz[i + (size_t)(j - 1) * n] = z[i + (size_t)(j - 1) * n];
      for (int i = 1; i <= nk1; ++i) {
        g(i, k2) = 0.0;
        for (int j = 1; j <= k1; ++j) g(i, j) = a(i, j);
      }
      double h[12], xi[10];
      for (int it = 1; it <= n8; ++it) {
        for (int i = 1; i <= k2; ++i) h[i] = b(it, i) * pinv;
        for (int j = 1; j <= idim; ++j) xi[j - 1] = 0.0;
        for (int j = it; j <= nk1; ++j) {
          const double piv = h[1];
          double cs, sn;
          fpgivs(piv, g(j, 1), cs, sn);
          for (int j1 = 1; j1 <= idim; ++j1) fprota(cs, sn, xi[j1 - 1], zz[j + (size_t)(j1 - 1) * n]);
          if (j == nk1) break;
          const int i2 = (j > n8) ? nk1 - j : k1;
          for (int i = 1; i <= i2; ++i) {
            const int i1 = i + 1;
            fprota(cs, sn, h[i1], g(j, i1));
            h[i] = h[i1];
          }
          h[i2 + 1] = 0.0;
        }
      }
      for (int j = 1; j <= idim; ++j) fpback(g, &zz[(size_t)(j - 1) * n], nk1, k2, &cc[(size_t)(j - 1) * n]);
      fp = 0.0;
      int l = k2;
      for (int it = 1; it <= m; ++it) {
        if (!(u[it] < t[l] || l > nk1)) ++l;
        for (int j2 = 1; j2 <= idim; ++j2) {
          int l0 = l - k2;
          double term = 0.0;
          for (int j = 1; j <= k1; ++j) {
            ++l0;
            term += cc[l0 + (size_t)(j2 - 1) * n] * Q(it, j);
          }
          fp += (term - X(it, j2)) * (term - X(it, j2));
        }
      }
      for (size_t i = 0; i < cc.size() && i < c.size(); ++i) c[i] = cc[i];
      fpms = fp - s;
      if (std::fabs(fpms) < acc) { ier = 0; break; }
      if (iter == maxit) { ier = 3; break; }
      const double p2 = p, f2 = fpms;
      if (ich3 == 0) {
        if (!((f2 - f3) > acc)) {
          p3 = p2;
          f3 = f2;
          p = p * con4;
          if (p <= p1) p = p1 * con9 + p2 * con1;
          continue;
        }
        if (f2 < 0.0) ich3 = 1;
      }
      if (ich1 == 0) {
        if (!((f1 - f2) > acc)) {
          p1 = p2;
          f1 = f2;
          p = p / con4;
          if (p3 < 0.0) continue;
          if (p >= p3) p = p2 * con1 + p3 * con9;
          continue;
        }
        if (f2 > 0.0) ich1 = 1;
      }
      if (f2 >= f1 || f2 <= f3) { ier = 2; break; }
      p = fprati(p1, f1, p2, f2, p3, f3);
    }
  }
  *n_out = n;
  *fp_out = fp;
  for (int i = 1; i <= n; ++i) t_out[i - 1] = t[i];
  for (int j = 0; j < idim; ++j)
    for (int i = 1; i <= n; ++i) c_out[(size_t)j * nest + (i - 1)] = (i <= n - k1) ? c[i + (size_t)j * n] : 0.0;
  return ier;
}

// value / derivatives (der <= k) of a B-spline (t: n knots, c: n-k-1 coefficients) at x,
// extrapolating outside [t_k, t_{n-k-1}] like FITPACK splev(ext=0).
double rdp_splev1(const double* t, int n, const double* c, int k, double x, int der) {
  // derivative coefficients by repeated differencing (FITPACK splder)
  std::vector<double> cd(c, c + (n - k - 1));
  int kk = k, lo = 0;  // current coefficients live at t-index offset lo
  for (int d = 1; d <= der; ++d) {
    const int nc = (int)cd.size() - 1;
    std::vector<double> nd(std::max(nc, 0));
    for (int i = 0; i < nc; ++i) {
      const double den = t[i + lo + kk + 1] - t[i + lo + 1];
      nd[i] = den > 0.0 ? kk * (cd[i + 1] - cd[i]) / den : 0.0;
    }
    cd.swap(nd);
    --kk;
    ++lo;
  }
  // knot vector for the derivative spline: t[lo .. n-1-lo], degree kk
  const double* tt = t + lo;
  const int nn = n - 2 * lo;
  // locate interval tt[l] <= x < tt[l+1], kk <= l <= nn-kk-2 (0-based)
  int l = kk;
  while (l < nn - kk - 2 && x >= tt[l + 1]) ++l;
  double h[12];
  fpbspl(tt - 1, kk, x, l + 1, h);  // 1-based interface
  double s = 0.0;
  for (int j = 1; j <= kk + 1; ++j) {
    const int ci = l - kk + j - 1;
    if (ci >= 0 && ci < (int)cd.size()) s += cd[ci] * h[j];
  }
  return s;
}

// Full post-edge pipeline: chord-length u, parcur(s, k), 100-sample curvature + points.
//   pts: m x 3 (sorted by x); out_pts: nsamp x 3; out: [mean_k, max_k, fp, n]; returns ier
//   (-2/0/1/2/3 like FITPACK, 10 = invalid input -> caller returns the empty result).
int rdp_fit_curvature(const double* pts, int m, double s, int k, int nsamp, double eps, double* out_pts,
                      double* out) {
  if (m <= k) return 10;
  std::vector<double> u(m);
  u[0] = 0.0;
  for (int i = 1; i < m; ++i) {
    double d2 = 0.0;
    for (int j = 0; j < 3; ++j) {
      const double d = pts[(size_t)i * 3 + j] - pts[(size_t)(i - 1) * 3 + j];
      d2 += d * d;
    }
    u[i] = u[i - 1] + std::sqrt(d2);
  }
  if (!(u[m - 1] > 0.0)) return 10;
  for (int i = 0; i < m; ++i) u[i] /= u[m - 1];
  const int nest = m + 2 * k;
  std::vector<double> t(nest), c((size_t)nest * 3);
  int n = 0;
  double fp = 0.0;
  const int ier = rdp_parcur(3, m, u.data(), pts, s, k, nest, t.data(), c.data(), &n, &fp);
  if (ier == 10) return ier;
  double ksum = 0.0, kmax = 0.0;
  int cnt = 0;
  for (int i = 0; i < nsamp; ++i) {
    const double x = nsamp > 1 ? (double)i / (nsamp - 1) : 0.0;
    double r[3], d1[3], d2[3];
    for (int j = 0; j < 3; ++j) {
      const double* cj = c.data() + (size_t)j * nest;
      r[j] = rdp_splev1(t.data(), n, cj, k, x, 0);
      d1[j] = rdp_splev1(t.data(), n, cj, k, x, 1);
      d2[j] = k >= 2 ? rdp_splev1(t.data(), n, cj, k, x, 2) : 0.0;
      out_pts[(size_t)i * 3 + j] = r[j];
    }
    const double cx = d1[1] * d2[2] - d1[2] * d2[1], cy = d1[2] * d2[0] - d1[0] * d2[2],
                 cz = d1[0] * d2[1] - d1[1] * d2[0];
    const double nd = std::sqrt(d1[0] * d1[0] + d1[1] * d1[1] + d1[2] * d1[2]);
    if (nd > eps) {
      const double kap = std::sqrt(cx * cx + cy * cy + cz * cz) / (nd * nd * nd);
      ksum += kap;
      kmax = cnt ? std::max(kmax, kap) : kap;
      ++cnt;
    }
  }
  out[0] = cnt ? ksum / cnt : 0.0;
  out[1] = cnt ? kmax : 0.0;
  out[2] = fp;
  out[3] = n;
  return ier;
}

}  // extern "C"
