// Host build of the network-simplex EMD solver (dstagnn_drought_amd/csrc/emd_simplex.hpp) for
// the CPU test suite only: it checks the algorithm against scipy linprog without a GPU.  The
// product path runs the same code in the gfx950 kernel (stag.hip); nothing in the package
// loads this library.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "../../dstagnn_drought_amd/csrc/emd_simplex.hpp"

// D null: cosine costs from xh / yh (T, F); else dense (T, T) costs (xh / yh unused).
extern "C" double emd_host(const double* xh, const double* yh, const double* p, const double* q, const double* D,
                           int T, int F, int* status, long long* pivots) {
  double sp = 0, sq = 0;
  for (int t = 0; t < T; ++t) { sp += p[t]; sq += q[t]; }
  if (pivots) *pivots = 0;
  if (!emd::balanced(sp, sq)) { *status = 1; return 1.0; }
  const long long bytes = emd::work_bytes(T, F);
  char* buf = (char*)aligned_alloc(64, (size_t)((bytes + 63) / 64 * 64));
  emd::Work w;
  emd::carve(w, buf, T, F);
  if (!D) {
    memcpy((void*)w.xh, xh, sizeof(double) * T * F);
    memcpy((void*)w.yh, yh, sizeof(double) * T * F);
  }
  memcpy((void*)w.p, p, sizeof(double) * T);
  memcpy((void*)w.q, q, sizeof(double) * T);
  double cmax = 1.0;
  if (D) {
    w.Dm = D;
    cmax = 0.0;
    for (long long i = 0; i < (long long)T * T; ++i) cmax = fmax(cmax, fabs(emd::clean_cost(D[i])));
  }
  int64_t piv = 0;
  double r = emd::solve<1>(w, 0, [](emd::Cand c) { return c; }, [] {}, cmax, status, &piv);
  if (pivots) *pivots = piv;
  free(buf);
  return r;
}
