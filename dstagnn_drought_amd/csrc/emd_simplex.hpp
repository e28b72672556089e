// emd_simplex.hpp — exact earth mover's distance of one STAG_gen node pair by a primal network
// simplex on the T x T transportation graph (replaces scipy linprog(method='highs') in
// data/STAG_gen.py:17-38, called from process_node_pair :40-59).
//
// Problem (the reference's LP with its dense 2T x T^2 A_eq):  min <D, P>  s.t.  P 1 = p,
// P^T 1 = q, P >= 0, with D_rc = clip(1 - xhat_r . yhat_c, 0, 1) (nan -> 1).  D is never stored:
// a cost is F fused multiply-adds on the unit-normalised series, recomputed wherever needed.
//
// Graph: rows 0..T-1 (supply p), cols T..2T-1 (demand q), artificial root 2T.  The basis is
// a spanning tree kept as parent pointers + doubly linked child lists; the tree arc of node v
// goes to parent[v] and carries flow[v].  Real arcs always point row -> col, the artificial
// arcs row -> root (cost 0) and root -> col (cost ART), so a row's tree arc points up and a
// col's points down.  Potentials: tree arcs have c + pi[tail] - pi[head] = 0, pi[root] = 0.
// Start: the all-artificial star (every flow > 0: strongly feasible).  Entering arc: block
// search over the T^2 real arcs (most negative reduced cost of the first block that has
// one, block = ceil64(max(T,64)) arcs, ties to the earliest arc in scan order).  Leaving arc:
// the strongly feasible rule (first blocking arc on the tail side with <, last on the head
// side with <=) which rules out cycling under degeneracy.  At the end the potentials are
// recomputed from the tree and a full pricing pass re-checks optimality (drift guard).
//
// Shared by the gfx950 kernel (stag.hip: one wave per pair, workspace in LDS, pricing split
// over the 64 lanes, tree updates executed redundantly by every lane) and a host build of
// the same code used only by the CPU tests (tests/native/emd_host.cpp).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define EMD_HD __host__ __device__ __forceinline__
#else
#define EMD_HD inline
#endif

namespace emd {

constexpr double kRcEps = 1e-11;       // enter only below -kRcEps * max(1, max|c|)
constexpr int kMaxPivotFactor = 64;    // give up (status 2) after 64 * T^2 pivots

// Per-pair workspace (node arrays sized n = 2T + 1).
struct Work {
  int T, F;
  const double* xh;   // (T, F) unit rows of node i (zero rows stay 0)
  const double* yh;   // (T, F) unit rows of node j
  const double* p;    // (T) supply
  const double* q;    // (T) demand
  double* flow;       // (n) flow on the tree arc to parent
  double* pi;         // (n) potentials
  int16_t* parent;    // (n)
  int16_t* fchild;    // (n) first child, -1 none
  int16_t* nsib;      // (n) next sibling, -1 none
  int16_t* psib;      // (n) previous sibling, -1 none
  int32_t* stamp;     // (n) ancestor marks for the join search
  const double* Dm;   // optional dense (T, T) cost (wasserstein_distance(p, q, D) entry); null: cosine
};

// The reference's LP has equality rows for p and columns for q; HiGHS declares it infeasible
// (linprog success False -> the 1.0 fallback, data/STAG_gen.py:37) once the totals differ by
// more than its 1e-7 feasibility tolerance (probed: 1e-7 boundary, sign dependent; 3e-7 always
// fails, 3e-8 never).  All-zero nodes hit this: their marginals sum to T / (T + 1).
constexpr double kBalanceTol = 1e-7;
EMD_HD bool balanced(double sum_p, double sum_q) {
  const double d = sum_p - sum_q;
  return d <= kBalanceTol && d >= -kBalanceTol;   // false for nan
}

// cost sanitising of wasserstein_distance (data/STAG_gen.py:33): nan -> 0, +-inf -> +-1e12
EMD_HD double clean_cost(double c) {
  if (c != c) return 0.0;
  if (c > 1e12) return 1e12;
  if (c < -1e12) return -1e12;
  return c;
}

// bytes of one Work for T, F (8-byte aligned pieces: doubles first)
EMD_HD int64_t work_bytes(int T, int F) {
  const int64_t n = 2 * (int64_t)T + 1;
  int64_t b = 8 * (2 * (int64_t)T * F + 2 * (int64_t)T + 2 * n);
  b += 2 * 4 * n;
  b = (b + 7) & ~7ll;
  b += 4 * n;
  return (b + 15) & ~15ll;
}

EMD_HD void carve(Work& w, char* base, int T, int F) {
  const int64_t n = 2 * (int64_t)T + 1;
  double* d = (double*)base;
  w.T = T; w.F = F;
  w.xh = d; d += (int64_t)T * F;
  w.yh = d; d += (int64_t)T * F;
  w.p = d; d += T;
  w.q = d; d += T;
  w.flow = d; d += n;
  w.pi = d; d += n;
  int16_t* s = (int16_t*)d;
  w.parent = s; s += n;
  w.fchild = s; s += n;
  w.nsib = s; s += n;
  w.psib = s; s += n;
  char* c = (char*)s;
  c = (char*)(((uintptr_t)c + 7) & ~(uintptr_t)7);
  w.stamp = (int32_t*)c;
  w.Dm = nullptr;
}

// D_rc of data/STAG_gen.py:50-57: 1 - cosine, nan -> 1, clipped to [0, 1]
EMD_HD double cost(const Work& w, int r, int c) {
  if (w.Dm) return clean_cost(w.Dm[(int64_t)r * w.T + c]);
  const double* a = w.xh + (int64_t)r * w.F;
  const double* b = w.yh + (int64_t)c * w.F;
  double s = 0.0;
  for (int f = 0; f < w.F; ++f) s += a[f] * b[f];
  double d = 1.0 - s;
  if (d != d) return 1.0;
  return d < 0.0 ? 0.0 : (d > 1.0 ? 1.0 : d);
}

// cost of the tree arc between v and parent[v]
EMD_HD double tree_cost(const Work& w, int v, int par, double art) {
  const int T = w.T;
  if (par == 2 * T) return v < T ? 0.0 : art;
  return v < T ? cost(w, v, par - T) : cost(w, par, v - T);
}

EMD_HD void unlink(Work& w, int v) {
  const int par = w.parent[v], a = w.psib[v], b = w.nsib[v];
  if (a >= 0) w.nsib[a] = (int16_t)b; else w.fchild[par] = (int16_t)b;
  if (b >= 0) w.psib[b] = (int16_t)a;
}

EMD_HD void link(Work& w, int v, int par) {
  const int h = w.fchild[par];
  w.parent[v] = (int16_t)par;
  w.psib[v] = -1;
  w.nsib[v] = (int16_t)h;
  if (h >= 0) w.psib[h] = (int16_t)v;
  w.fchild[par] = (int16_t)v;
}

// Candidate (reduced cost, scan offset) reduction across the lanes of a team.
struct Cand {
  double rc;
  int off;
};

// Recompute every potential from the tree (preorder walk from the root).
EMD_HD void potentials_from_tree(Work& w, double art) {
  const int root = 2 * w.T;
  w.pi[root] = 0.0;
  int u = w.fchild[root];
  while (u >= 0) {
    const int par = w.parent[u];
    const double c = tree_cost(w, u, par, art);
    w.pi[u] = u < w.T ? w.pi[par] - c : w.pi[par] + c;
    if (w.fchild[u] >= 0) { u = w.fchild[u]; continue; }
    while (u >= 0 && w.nsib[u] < 0) { u = w.parent[u]; if (u == root) { u = -1; break; } }
    if (u >= 0) u = w.nsib[u];
  }
}

// Solve; returns the optimal cost over the real arcs.  status: 0 ok, 2 pivot cap hit.
// Team: lane in [0, NL), reduce(Cand) -> the minimum over lanes (ties: smallest offset),
// identical on every lane; every lane runs the serial parts redundantly.
// cmax: largest |cost| (1 for the cosine costs).
// sync(): makes the lane-parallel initialisation visible to every lane before the serial part.
template <int NL, class Reduce, class Sync>
EMD_HD double solve(Work& w, int lane, Reduce reduce, Sync sync, double cmax, int* status, int64_t* pivots_out) {
  const int T = w.T;
  const int n = 2 * T + 1, root = 2 * T;
  const int64_t narcs = (int64_t)T * T;
  const double art = (cmax + 1.0) * n;   // > any path cost
  const double eps = kRcEps * (cmax > 1.0 ? cmax : 1.0);
  // the all-artificial start
  for (int v = lane; v < n; v += NL) {
    if (v < T) { w.flow[v] = w.p[v]; w.pi[v] = 0.0; }
    else if (v < root) { w.flow[v] = w.q[v - T]; w.pi[v] = art; }
    else { w.flow[v] = 0.0; w.pi[v] = 0.0; }
    w.parent[v] = (int16_t)(v < root ? root : -1);
    w.nsib[v] = (int16_t)(v + 1 < root ? v + 1 : -1);
    w.psib[v] = (int16_t)(v < root ? v - 1 : -1);
    w.fchild[v] = (int16_t)(v == root ? 0 : -1);
    w.stamp[v] = 0;
  }
  sync();
  int64_t blk = ((T > 64 ? T : 64) + 63) / 64 * 64;
  if (blk > narcs) blk = narcs;
  int64_t next = 0, piv = 0;
  const int64_t cap = (int64_t)kMaxPivotFactor * narcs + 16 * n;
  int32_t it = 0;
  bool rechecked = false;
  *status = 0;
  for (;;) {
    // ---- entering arc: block search ----
    Cand best{-eps, -1};
    int64_t scanned = 0, pos = next;
    while (scanned < narcs) {
      const int64_t len = blk < narcs - scanned ? blk : narcs - scanned;
      Cand mine{best.rc, -1};
      for (int64_t o = lane; o < len; o += NL) {
        int64_t a = pos + o;
        if (a >= narcs) a -= narcs;
        const int r = (int)(a / T), c = (int)(a - (int64_t)r * T);
        const double rc = cost(w, r, c) + w.pi[r] - w.pi[T + c];
        if (rc < mine.rc) { mine.rc = rc; mine.off = (int)o; }
      }
      mine = reduce(mine);
      scanned += len;
      pos += len;
      if (pos >= narcs) pos -= narcs;
      if (mine.off >= 0) {
        int64_t a = pos - len + mine.off;
        if (a < 0) a += narcs;
        if (a >= narcs) a -= narcs;
        best.rc = mine.rc;
        best.off = (int)a;
        break;
      }
    }
    if (best.off < 0) {
      if (rechecked) break;
      // drift guard: exact potentials, then one more full pass
      potentials_from_tree(w, art);
      rechecked = true;
      continue;
    }
    rechecked = false;
    if (++piv > cap) { *status = 2; break; }
    next = pos;
    const int r_in = best.off / T, c_in = best.off - r_in * T;
    const int first = r_in, second = T + c_in;
    const double rc_in = best.rc;
    // ---- join: lowest common ancestor ----
    ++it;
    for (int u = first;; u = w.parent[u]) { w.stamp[u] = it; if (u == root) break; }
    int join = second;
    while (w.stamp[join] != it) join = w.parent[join];
    // ---- leaving arc (strongly feasible rule) ----
    double delta = 1e300;
    int u_out = -1, side = 0;
    for (int u = first; u != join; u = w.parent[u])
      if (u < T && w.flow[u] < delta) { delta = w.flow[u]; u_out = u; side = 1; }
    for (int u = second; u != join; u = w.parent[u])
      if (u >= T && w.flow[u] <= delta) { delta = w.flow[u]; u_out = u; side = 2; }
    if (u_out < 0) { *status = 3; break; }   // impossible for a transportation problem
    // ---- augment around the cycle ----
    if (delta > 0.0) {
      for (int u = first; u != join; u = w.parent[u]) w.flow[u] += u < T ? -delta : delta;
      for (int u = second; u != join; u = w.parent[u]) w.flow[u] += u >= T ? -delta : delta;
    }
    // ---- re-hang the cut subtree from the entering arc ----
    const int e = side == 1 ? first : second, f = side == 1 ? second : first;
    const double sigma = side == 1 ? -rc_in : rc_in;
    {
      int prev = f, u = e;
      double pflow = delta;
      for (;;) {
        const int nxt = w.parent[u];
        const double fl = w.flow[u];
        unlink(w, u);
        link(w, u, prev);
        w.flow[u] = pflow;
        if (u == u_out) break;
        prev = u; pflow = fl; u = nxt;
      }
    }
    // ---- shift the potentials of the re-hung subtree ----
    {
      int u = e;
      for (;;) {
        w.pi[u] += sigma;
        if (w.fchild[u] >= 0) { u = w.fchild[u]; continue; }
        while (u != e && w.nsib[u] < 0) u = w.parent[u];
        if (u == e) break;
        u = w.nsib[u];
      }
    }
  }
  if (pivots_out) *pivots_out = piv;
  // objective over the real tree arcs (lane-strided; the caller sums across lanes)
  double obj = 0.0;
  for (int v = lane; v < root; v += NL) {
    const int par = w.parent[v];
    if (par != root) obj += w.flow[v] * tree_cost(w, v, par, art);
  }
  return obj;
}

}  // namespace emd
