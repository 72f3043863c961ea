/*
 * cgpc.c — plain-C restatement of the toolbox-equivalent GPC closed loop (oracle/toolbox_gpc.py),
 * TEST INFRASTRUCTURE ONLY: the timed CPU baseline ("port") of bench.py and a second, compiled
 * check of the numpy oracle.  Never linked into the product.
 *
 * Per candidate (closedloop_toolbox.m:36-100 semantics):
 *   G[(i,r),(n,c)] = s_in(n1_i + r - c)              MatG.m:64-67 (step table from the caller)
 *   H = G'QG + Lambda, Cholesky                       DTC_GPC_WW.m:98-100 (Q, Lambda squared
 *                                                     when the toolbox cost is selected)
 * per step t:
 *   y(t)        exact difference equations of every plant entry (lsim)
 *   f = Phi x   Phi = [F | Hp] rows, x = [y histories | du histories]   DTC_GPC_WW.m:139-146
 *   g = G'Q(f - r(t))                                   reference held flat (RefLookAhead off)
 *   dU = argmin 1/2 dU'H dU + g'dU s.t. rate/amplitude bounds: unconstrained Cholesky solve, then
 *        a Goldfarb-Idnani dual active-set method (same family as the toolbox's KWIK solver)
 *   u(t) = u(t-1) + dU(first move of every MV)
 * Costs: J1 (GAM_fun.m:219-220), j22 from inK (VNS2.m:173,177); open loop (uopt, ys, j21, Jnu)
 * restated as in closedloop_toolbox.m:85-100 / VNS2.m:172-191.
 *
 * Build: see oracle/Makefile (gcc -O3 -fopenmp -shared -fPIC).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
  int my, nu, nin, nit, n2max, tlen, nx, wsq, ink0;
  const int* n1;      /* [my] */
  const double* step; /* [my][nu][tlen] */
  const double* phi;  /* [my*n2max][nx] */
  const int* yoff;    /* [my] */
  const int* nyhi;    /* [my] */
  const int* upoff;   /* [nu] */
  const int* dum;     /* [nu] */
  int ne, pl_maxb, pl_maxa;
  const int* pl_nb;
  const int* pl_na;
  const double* pl_b; /* [ne][pl_maxb] */
  const double* pl_a; /* [ne][pl_maxa] */
  const double* bnd;  /* [4][nu] */
  const double* yref; /* [my][nit] */
} cg_scen;

#define CG_MAXM 64

static void chol(double* A, int n, int* ok) { /* lower, in place */
  *ok = 1;
  for (int k = 0; k < n; ++k) {
    double d = A[k * n + k];
    for (int j = 0; j < k; ++j) d -= A[k * n + j] * A[k * n + j];
    if (!(d > 0)) {
      *ok = 0;
      return;
    }
    d = sqrt(d);
    A[k * n + k] = d;
    for (int i = k + 1; i < n; ++i) {
      double s = A[i * n + k];
      for (int j = 0; j < k; ++j) s -= A[i * n + j] * A[k * n + j];
      A[i * n + k] = s / d;
    }
  }
}

/* H^-1 from the Cholesky factor */
static void chol_inv(const double* Lc, int n, double* Hi) {
  double* Li = (double*)calloc((size_t)n * n, sizeof(double));
  for (int j = 0; j < n; ++j)
    for (int i = j; i < n; ++i) {
      double s = (i == j) ? 1.0 : 0.0;
      for (int k = j; k < i; ++k) s -= Lc[i * n + k] * Li[k * n + j];
      Li[i * n + j] = s / Lc[i * n + i];
    }
  for (int a = 0; a < n; ++a)
    for (int b = 0; b < n; ++b) {
      int k0 = a > b ? a : b;
      double s = 0;
      for (int k = k0; k < n; ++k) s += Li[k * n + a] * Li[k * n + b];
      Hi[a * n + b] = s;
    }
  free(Li);
}

/* constraint p = 4*m + kind; see gpc_kernel.hip for the same convention */
static double slack(const double* x, int p, int Nu, const double* bnd, const double* up, int nu) {
  int m = p >> 2, kind = p & 3, n = m / Nu, l = m - n * Nu;
  double dmin = bnd[n], dmax = bnd[nu + n], umin = bnd[2 * nu + n], umax = bnd[3 * nu + n];
  if (l == 0) {
    if (kind == 0) return x[m] - fmax(dmin, umin - up[n]);
    if (kind == 1) return fmin(dmax, umax - up[n]) - x[m];
    return INFINITY;
  }
  if (kind == 0) return x[m] - dmin;
  if (kind == 1) return dmax - x[m];
  double pre = 0;
  for (int j = n * Nu; j <= m; ++j) pre += x[j];
  if (kind == 2) return pre - (umin - up[n]);
  return (umax - up[n]) - pre;
}

static void normal_range(int p, int Nu, int* j0, int* j1, double* sg) {
  int m = p >> 2, kind = p & 3;
  *sg = (kind & 1) ? -1.0 : 1.0;
  *j0 = kind < 2 ? m : (m / Nu) * Nu;
  *j1 = m;
}

/* Goldfarb-Idnani (Schur form), x holds the unconstrained minimiser on entry */
static int gi_qp(const double* Hi, int M, int Nu, int nu, const double* bnd, const double* up,
                 double* x, double tol, int maxit, int* st) {
  double Y[CG_MAXM * CG_MAXM], S[CG_MAXM * CG_MAXM], T[CG_MAXM * CG_MAXM];
  double v[CG_MAXM], z[CG_MAXM], r[CG_MAXM], u[CG_MAXM], sv[CG_MAXM];
  int W[CG_MAXM];
  unsigned char act[4 * CG_MAXM];
  memset(act, 0, sizeof(act));
  int q = 0, it = 0;
  for (;;) {
    double best = INFINITY;
    int p = -1;
    for (int c = 0; c < 4 * M; ++c) {
      if (act[c]) continue;
      double s = slack(x, c, Nu, bnd, up, nu);
      if (s < best) {
        best = s;
        p = c;
      }
    }
    if (!(best < -tol)) break;
    if (it >= maxit) {
      *st |= 1;
      break;
    }
    int j0, j1;
    double sg;
    normal_range(p, Nu, &j0, &j1, &sg);
    double sp = best, upm = 0.0;
    for (;;) {
      ++it;
      for (int m = 0; m < M; ++m) {
        double a = 0;
        for (int j = j0; j <= j1; ++j) a += Hi[j * M + m];
        v[m] = sg * a;
      }
      for (int w = 0; w < q; ++w) {
        int a0, a1;
        double sw;
        normal_range(W[w], Nu, &a0, &a1, &sw);
        double a = 0;
        for (int j = a0; j <= a1; ++j) a += v[j];
        sv[w] = sw * a;
      }
      for (int w = 0; w < q; ++w) {
        double a = 0;
        for (int k = 0; k < q; ++k) a += S[w * M + k] * sv[k];
        r[w] = a;
      }
      for (int m = 0; m < M; ++m) {
        double a = v[m];
        for (int w = 0; w < q; ++w) a -= Y[w * M + m] * r[w];
        z[m] = a;
      }
      double beta = 0, cpp = 0;
      for (int j = j0; j <= j1; ++j) {
        beta += z[j];
        cpp += v[j];
      }
      beta *= sg;
      cpp *= sg;
      double t1 = INFINITY;
      int kd = -1;
      for (int w = 0; w < q; ++w)
        if (r[w] > 0 && u[w] / r[w] < t1) {
          t1 = u[w] / r[w];
          kd = w;
        }
      double t2 = (beta > 1e-14 * cpp) ? -sp / beta : INFINITY;
      if (t1 == INFINITY && t2 == INFINITY) {
        *st |= 2;
        return it;
      }
      int full = t2 <= t1;
      double t = full ? t2 : t1;
      if (t2 != INFINITY)
        for (int m = 0; m < M; ++m) x[m] += t * z[m];
      for (int w = 0; w < q; ++w) u[w] -= t * r[w];
      upm += t;
      sp += t * beta;
      if (full) {
        for (int m = 0; m < M; ++m) Y[q * M + m] = v[m];
        double ib = 1.0 / beta;
        for (int a = 0; a <= q; ++a)
          for (int b = 0; b <= q; ++b) {
            double val;
            if (a < q && b < q)
              val = S[a * M + b] + r[a] * r[b] * ib;
            else if (a < q)
              val = -r[a] * ib;
            else if (b < q)
              val = -r[b] * ib;
            else
              val = ib;
            T[a * M + b] = val;
          }
        for (int a = 0; a <= q; ++a)
          for (int b = 0; b <= q; ++b) S[a * M + b] = T[a * M + b];
        u[q] = upm;
        W[q] = p;
        act[p] = 1;
        ++q;
        break;
      }
      /* drop kd */
      act[W[kd]] = 0;
      double ikk = 1.0 / S[kd * M + kd];
      for (int a = 0; a < q; ++a)
        for (int b = 0; b < q; ++b) {
          if (a == kd || b == kd) continue;
          int na = (a == q - 1) ? kd : a, nb = (b == q - 1) ? kd : b;
          T[na * M + nb] = S[a * M + b] - S[a * M + kd] * S[kd * M + b] * ikk;
        }
      for (int a = 0; a < q - 1; ++a)
        for (int b = 0; b < q - 1; ++b) S[a * M + b] = T[a * M + b];
      if (kd != q - 1) {
        for (int m = 0; m < M; ++m) Y[kd * M + m] = Y[(q - 1) * M + m];
        u[kd] = u[q - 1];
        W[kd] = W[q - 1];
      }
      --q;
      if (it >= maxit) {
        *st |= 1;
        break;
      }
    }
    if (it >= maxit) break;
  }
  return it;
}

/* one simulation; returns status */
static int simulate(const cg_scen* sc, int N2, int Nu, const double* delta, const double* lam,
                    const double* r, int open_loop, double* J1, double* j21, double* j22,
                    double* Jnu, int64_t* iters_out, double* ytraj, double* utraj, double* ystraj,
                    double* uopttraj) {
  const int my = sc->my, nu = sc->nu, nin = sc->nin, nit = sc->nit, nx = sc->nx;
  const int M = nu * Nu, P = my * N2;
  if (M > CG_MAXM || N2 > sc->n2max || Nu > N2 || Nu < 1) return 16;
  double* G = (double*)calloc((size_t)P * M, sizeof(double));
  double* QG = (double*)calloc((size_t)P * M, sizeof(double));
  double* H = (double*)calloc((size_t)M * M, sizeof(double));
  double* Hi = (double*)calloc((size_t)M * M, sizeof(double));
  double* f = (double*)calloc((size_t)P, sizeof(double));
  double* xs = (double*)calloc((size_t)nx, sizeof(double));
  double* U = (double*)calloc((size_t)2 * nin * nit, sizeof(double)); /* [copy][j][t] */
  double* Ye = (double*)calloc((size_t)2 * sc->ne * nit, sizeof(double));
  double qw[64], g[CG_MAXM], x[CG_MAXM], ucum[CG_MAXM];
  int st = 0;
  int64_t iters = 0;
  for (int i = 0; i < my; ++i) {
    double d = fabs(delta[i]);
    qw[i] = sc->wsq ? d * d : d;
  }
  for (int i = 0; i < my; ++i)
    for (int rr = 0; rr < N2; ++rr)
      for (int n = 0; n < nu; ++n)
        for (int c = 0; c < Nu; ++c) {
          int t = sc->n1[i] + rr - c;
          double gv = t >= 0 ? sc->step[((size_t)i * nu + n) * sc->tlen + t] : 0.0;
          G[(size_t)(i * N2 + rr) * M + n * Nu + c] = gv;
          QG[(size_t)(i * N2 + rr) * M + n * Nu + c] = qw[i] * gv;
        }
  for (int a = 0; a < M; ++a)
    for (int b = 0; b < M; ++b) {
      double s = 0;
      for (int k = 0; k < P; ++k) s += G[(size_t)k * M + a] * QG[(size_t)k * M + b];
      H[a * M + b] = s;
    }
  for (int a = 0; a < M; ++a)
    for (int b = 0; b < a; ++b) {
      double h = 0.5 * (H[a * M + b] + H[b * M + a]);
      H[a * M + b] = H[b * M + a] = h;
    }
  for (int n = 0; n < nu; ++n) {
    double l = fabs(lam[n]);
    double w = sc->wsq ? l * l : l;
    for (int c = 0; c < Nu; ++c) H[(n * Nu + c) * M + n * Nu + c] += w;
  }
  int ok;
  chol(H, M, &ok);
  if (!ok) {
    st |= 4;
    goto done;
  }
  chol_inv(H, M, Hi);
  {
    const double tol = 1e-10;
    const int maxit = 8 * M + 16;
    const double* bnd = sc->bnd;
    double uprev[64];
    memset(uprev, 0, sizeof(uprev));
    /* solve at the current xs with reference rv */
#define SOLVE(rv)                                                              \
  do {                                                                         \
    for (int i = 0; i < my; ++i)                                               \
      for (int rr = 0; rr < N2; ++rr) {                                        \
        const double* prow = sc->phi + (size_t)(i * sc->n2max + rr) * nx;     \
        double s = 0;                                                          \
        for (int k = 0; k < nx; ++k) s += prow[k] * xs[k];                     \
        f[i * N2 + rr] = s - (rv)[i];                                          \
      }                                                                        \
    for (int a = 0; a < M; ++a) {                                              \
      double s = 0;                                                            \
      for (int k = 0; k < P; ++k) s += QG[(size_t)k * M + a] * f[k];           \
      g[a] = s;                                                                \
    }                                                                          \
    for (int a = 0; a < M; ++a) {                                              \
      double s = 0;                                                            \
      for (int b = 0; b < M; ++b) s -= Hi[a * M + b] * g[b];                   \
      x[a] = s;                                                                \
    }                                                                          \
    iters += gi_qp(Hi, M, Nu, nu, bnd, uprev, x, tol, maxit, &st);             \
  } while (0)
    double jn[64];
    memset(jn, 0, sizeof(jn));
    if (open_loop) {
      double rend[64];
      for (int i = 0; i < my; ++i) rend[i] = r[i * nit + nit - 1];
      SOLVE(rend);
      for (int n = 0; n < nu; ++n) {
        double s = 0;
        for (int l = 0; l < Nu; ++l) {
          s += x[n * Nu + l];
          ucum[n * Nu + l] = s;
        }
        double u0 = fabs(ucum[n * Nu]);
        int nd_ = Nu - 1 < nit - 1 ? Nu - 1 : nit - 1;
        for (int t = 0; t < nd_; ++t) {
          double d = fabs(ucum[n * Nu + t + 1] - ucum[n * Nu + t]);
          double xr = u0 / d;
          if (isfinite(xr)) jn[n] += xr * xr;
        }
        for (int t = 0; t < nit; ++t) U[(size_t)(nin + n) * nit + t] = ucum[n * Nu + (t < Nu - 1 ? t : Nu - 1)];
      }
    }
    double sj1[64], sj21[64], sj22[64];
    memset(sj1, 0, sizeof(sj1));
    memset(sj21, 0, sizeof(sj21));
    memset(sj22, 0, sizeof(sj22));
    const int ncopy = open_loop ? 2 : 1;
    for (int t = 0; t < nit; ++t) {
      double ycl[64], yol[64];
      for (int i = 0; i < my; ++i) ycl[i] = yol[i] = 0;
      for (int cpy = 0; cpy < ncopy; ++cpy)
        for (int e = 0; e < sc->ne; ++e) {
          int j = e % nin, i = e / nin;
          const double* b = sc->pl_b + (size_t)e * sc->pl_maxb;
          const double* a = sc->pl_a + (size_t)e * sc->pl_maxa;
          const double* uu = U + (size_t)(cpy * nin + j) * nit;
          double* ye = Ye + (size_t)(cpy * sc->ne + e) * nit;
          double acc = 0;
          for (int l = 0; l < sc->pl_nb[e]; ++l)
            if (t - l >= 0 && !(cpy == 0 && l == 0 && j < nu)) acc += b[l] * uu[t - l];
          for (int l = 1; l < sc->pl_na[e]; ++l)
            if (t - l >= 0) acc -= a[l] * ye[t - l];
          ye[t] = acc;
          if (cpy == 0)
            ycl[i] += acc;
          else
            yol[i] += acc;
        }
      for (int i = 0; i < my; ++i) {
        int yo = sc->yoff[i], nh = sc->nyhi[i];
        for (int k = nh - 1; k > 0; --k) xs[yo + k] = xs[yo + k - 1];
        xs[yo] = ycl[i];
        double e1 = ycl[i] - sc->yref[i * nit + t];
        sj1[i] += e1 * e1;
        if (t >= sc->ink0) sj22[i] += e1 * e1;
        if (open_loop && t >= sc->ink0) sj21[i] += (ycl[i] - yol[i]) * (ycl[i] - yol[i]);
        if (ytraj) ytraj[(size_t)i * nit + t] = ycl[i];
        if (ystraj && open_loop) ystraj[(size_t)i * nit + t] = yol[i];
      }
      double rt[64];
      for (int i = 0; i < my; ++i) rt[i] = r[i * nit + t];
      SOLVE(rt);
      for (int n = 0; n < nu; ++n) {
        double du = x[n * Nu];
        double un = uprev[n] + du;
        int uo = sc->upoff[n], nh = sc->dum[n];
        for (int k = nh - 1; k > 0; --k) xs[uo + k] = xs[uo + k - 1];
        xs[uo] = du;
        U[(size_t)n * nit + t] = un;
        uprev[n] = un;
        if (utraj) utraj[(size_t)n * nit + t] = un;
        if (uopttraj && open_loop) uopttraj[(size_t)n * nit + t] = U[(size_t)(nin + n) * nit + t];
      }
    }
#undef SOLVE
    for (int i = 0; i < my; ++i) {
      if (J1) J1[i] = sj1[i];
      if (j22) j22[i] = sj22[i];
      if (j21) j21[i] = open_loop ? sj21[i] : NAN;
      if (!isfinite(sj1[i])) st |= 4;
    }
    for (int n = 0; n < nu; ++n)
      if (Jnu) Jnu[n] = open_loop ? jn[n] : NAN;
  }
done:
  if (iters_out) *iters_out = iters;
  free(G);
  free(QG);
  free(H);
  free(Hi);
  free(f);
  free(xs);
  free(U);
  free(Ye);
  return st;
}

/* Evaluate C candidates x nref references (same result layout as mpct_eval_batch). */
int cgpc_eval(const cg_scen* sc, int64_t C, const int* N2, const int* Nu, const double* delta,
              const double* lam, int nref, const double* r, int open_loop, int nthreads, double* J1,
              double* j21, double* j22, double* Jnu, int* status, int64_t* iters, double* ytraj,
              double* utraj, double* ystraj, double* uopttraj) {
  const int my = sc->my, nu = sc->nu, nit = sc->nit;
  const int64_t S = C * nref;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int64_t s = 0; s < S; ++s) {
    int64_t c = s / nref;
    int k = (int)(s - c * nref);
    status[s] = simulate(sc, N2[c], Nu[c], delta + c * my, lam + c * nu, r + (size_t)k * my * nit,
                         open_loop, J1 + s * my, j21 + s * my, j22 + s * my, Jnu + s * nu, iters + s,
                         ytraj ? ytraj + (size_t)s * my * nit : 0, utraj ? utraj + (size_t)s * nu * nit : 0,
                         ystraj ? ystraj + (size_t)s * my * nit : 0,
                         uopttraj ? uopttraj + (size_t)s * nu * nit : 0);
  }
  return 0;
}
