// Sanitizer driver (ASan + UBSan, host build) for the network-simplex EMD solver
// (dstagnn_drought_amd/csrc/emd_simplex.hpp via tests/native/emd_host.cpp): random cosine-cost
// and dense-cost problems (costs 1 - x.y in [0, 2]), T = 1..48, F = 1..4, balanced marginals
// with zero entries; checks that every solve terminates with status 0 and a finite
// non-negative cost (the values themselves are held to scipy linprog and the reference's
// goldens by tests/test_emd_solver_cpu.py).  Test infrastructure only
// (tests/test_sanitize_cpu.py builds and runs it); exit status 0 = clean.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

extern "C" double emd_host(const double* xh, const double* yh, const double* p, const double* q, const double* D,
                           int T, int F, int* status, long long* pivots);

static double urand(unsigned long long* s) {
  *s = *s * 6364136223846793005ULL + 1442695040888963407ULL;
  return (double)(*s >> 11) / 9007199254740992.0;
}

int main() {
  unsigned long long seed = 12345;
  int bad = 0, runs = 0;
  for (int T = 1; T <= 48; T += (T < 12 ? 1 : 7)) {
    for (int F = 1; F <= 4; ++F) {
      for (int rep = 0; rep < 6; ++rep) {
        double* xh = (double*)malloc(sizeof(double) * T * F);
        double* yh = (double*)malloc(sizeof(double) * T * F);
        double* p = (double*)malloc(sizeof(double) * T);
        double* q = (double*)malloc(sizeof(double) * T);
        double* D = (double*)malloc(sizeof(double) * T * T);
        double sp = 0, sq = 0;
        for (int t = 0; t < T; ++t) {
          double nx = 0, ny = 0;
          for (int f = 0; f < F; ++f) {
            xh[t * F + f] = urand(&seed) - 0.5;
            yh[t * F + f] = urand(&seed) - 0.5;
            nx += xh[t * F + f] * xh[t * F + f];
            ny += yh[t * F + f] * yh[t * F + f];
          }
          nx = sqrt(nx) > 0 ? sqrt(nx) : 1.0;
          ny = sqrt(ny) > 0 ? sqrt(ny) : 1.0;
          for (int f = 0; f < F; ++f) { xh[t * F + f] /= nx; yh[t * F + f] /= ny; }
          p[t] = (rep % 3 == 0 && t % 4 == 1) ? 0.0 : urand(&seed);  // some empty bins
          q[t] = (rep % 3 == 1 && t % 5 == 2) ? 0.0 : urand(&seed);
          sp += p[t];
          sq += q[t];
        }
        if (sp == 0) { p[0] = 1; sp = 1; }
        if (sq == 0) { q[0] = 1; sq = 1; }
        for (int t = 0; t < T; ++t) { p[t] /= sp; q[t] /= sq; }
        for (int i = 0; i < T; ++i)
          for (int j = 0; j < T; ++j) {
            double d = 0;
            for (int f = 0; f < F; ++f) d += xh[i * F + f] * yh[j * F + f];
            D[i * T + j] = 1.0 - d;
          }
        int st1 = -1, st2 = -1;
        long long pv1 = 0, pv2 = 0;
        const double r1 = emd_host(xh, yh, p, q, NULL, T, F, &st1, &pv1);
        const double r2 = emd_host(NULL, NULL, p, q, D, T, 0, &st2, &pv2);
        ++runs;
        if (st1 != 0 || st2 != 0 || !isfinite(r1) || !isfinite(r2) || r1 < -1e-12 || r2 < -1e-12) {
          fprintf(stderr, "T=%d F=%d rep=%d: status %d/%d cost %.17g / %.17g\n", T, F, rep, st1, st2, r1, r2);
          ++bad;
        }
        free(xh); free(yh); free(p); free(q); free(D);
      }
    }
  }
  printf("emd sanitize: %d problems, %d bad\n", runs, bad);
  return bad ? 1 : 0;
}
