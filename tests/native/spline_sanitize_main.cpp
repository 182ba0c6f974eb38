// Host driver for the sanitizer build of csrc/spline.cpp (tests/test_sanitizers_cpu.py).
// Runs the FITPACK-equivalent fit + curvature over arcs, noisy clouds and degenerate inputs with
// exact-size heap buffers, so AddressSanitizer sees every out-of-bounds knot/coefficient access and
// UBSan every overflow / invalid shift.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" int rdp_parcur(int idim, int m, const double* u, const double* x, double s, int k, int nest, double* t,
                          double* c, int* n, double* fp);
extern "C" double rdp_splev1(const double* t, int n, const double* c, int k, double x, int der);
extern "C" int rdp_fit_curvature(const double* pts, int m, double s, int k, int nsamp, double eps, double* out_pts,
                                 double* out);

static unsigned long long g_state = 0x9e3779b97f4a7c15ull;
static double urand() {  // xorshift64*, deterministic
  g_state ^= g_state >> 12; g_state ^= g_state << 25; g_state ^= g_state >> 27;
  return (double)((g_state * 2685821657736338717ull) >> 11) / 9007199254740992.0;
}

static int run_fit(const std::vector<double>& p, double s, int k) {
  const int m = (int)p.size() / 3;
  std::vector<double> out_pts(100 * 3), out(4);
  const int ier = rdp_fit_curvature(p.data(), m, s, k, 100, 1e-6, out_pts.data(), out.data());
  if (ier != 10) {
    for (double v : out_pts)
      if (!std::isfinite(v)) { std::printf("non-finite spline point (m=%d s=%g k=%d)\n", m, s, k); return 1; }
    if (!std::isfinite(out[0]) || !std::isfinite(out[1]) || out[0] < 0 || out[1] < out[0] - 1e-12) {
      std::printf("bad curvature (m=%d s=%g k=%d): %g %g\n", m, s, k, out[0], out[1]);
      return 1;
    }
  }
  return 0;
}

int main() {
  int bad = 0, fits = 0;
  const double ss[] = {0.0, 1e-4, 1e-2, 0.1, 10.0};
  for (int trial = 0; trial < 60; ++trial) {
    const int m = 4 + (int)(urand() * 600);
    const double noise = trial % 3 == 0 ? 0.0 : (trial % 3 == 1 ? 0.005 : 0.08);
    std::vector<double> p((size_t)m * 3);
    for (int i = 0; i < m; ++i) {
      const double th = 1.6 * i / (m - 1);
      p[3 * i] = 0.2 * std::sin(th) + noise * (urand() - 0.5);
      p[3 * i + 1] = 0.2 * (1 - std::cos(th)) + noise * (urand() - 0.5);
      p[3 * i + 2] = 0.5 + 0.02 * th + noise * (urand() - 0.5);
    }
    for (double s : ss)
      for (int k = 1; k <= 5; k += 2) { bad += run_fit(p, s, k); ++fits; }
  }
  // degenerate inputs: too few points, all points identical (zero chord), two distinct points
  std::vector<double> tiny = {0, 0, 0, 1, 1, 1, 2, 2, 2};
  bad += run_fit(tiny, 0.1, 3);
  std::vector<double> same(30 * 3, 0.25);
  bad += run_fit(same, 0.1, 3);
  std::vector<double> dup(40 * 3);
  for (int i = 0; i < 40; ++i) { dup[3 * i] = i < 20 ? 0.0 : 1.0; dup[3 * i + 1] = 0.5; dup[3 * i + 2] = 1.0; }
  bad += run_fit(dup, 0.1, 3);
  // direct parcur + splev with the minimum legal nest (2k+2 .. m+k+1) and invalid arguments
  for (int k = 1; k <= 5; ++k) {
    const int m = 50;
    std::vector<double> u(m), x((size_t)m * 2);
    for (int i = 0; i < m; ++i) { u[i] = (double)i / (m - 1); x[2 * i] = std::cos(3 * u[i]); x[2 * i + 1] = u[i] * u[i]; }
    for (int nest : {2 * k + 2, m + k + 1}) {
      std::vector<double> t(nest), c((size_t)nest * 2);
      int n = 0;
      double fp = 0;
      const int ier = rdp_parcur(2, m, u.data(), x.data(), 0.01, k, nest, t.data(), c.data(), &n, &fp);
      if (ier <= 0 && n > 0)
        for (int der = 0; der <= k; ++der) {
          const double v = rdp_splev1(t.data(), n, c.data(), k, 0.37, der);
          if (!std::isfinite(v)) { std::printf("non-finite splev k=%d der=%d\n", k, der); ++bad; }
        }
    }
    int n = 0;
    double fp = 0, t[64], c[128];
    if (rdp_parcur(2, m, u.data(), x.data(), -1.0, k, 64, t, c, &n, &fp) != 10) { std::printf("s<0 accepted\n"); ++bad; }
  }
  std::printf("spline sanitizer driver: %d fits, %d failures\n", fits, bad);
  return bad ? 1 : 0;
}
