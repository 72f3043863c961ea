/*
 * cgpc.c — plain-C restatement of the toolbox-equivalent GPC closed loop (oracle/toolbox_gpc.py),
 * TEST INFRASTRUCTURE ONLY: the timed CPU baseline ("port") of bench.py and a second, compiled
 * check of the numpy oracle.  Never linked into the product.
 *
 * Per candidate (closedloop_toolbox.m:36-100 semantics):
 *   G[(i,r),(n,c)] = s_in(n1_i + r - c)              MatG.m:64-67 (step table from the caller)
 *   W = [Q^1/2 G; Lambda^1/2] = Q1 R by row-streamed Givens (R'R = H = G'QG + Lambda of
 *   DTC_GPC_WW.m:98-100, never formed: the normal equations lose ~cond(H)*eps)
 *   B = -R^-1 Q1'[Q^1/2; 0]                           (unconstrained minimiser dU = B (f - w))
 * per step t:
 *   y(t)        exact difference equations of every plant entry (lsim)
 *   f = Phi x   Phi = [F | Hp] rows, x = [y histories | du histories]   DTC_GPC_WW.m:139-146
 *   dU = B (f - r(t))                                   reference held flat (RefLookAhead off)
 *   dU = argmin 1/2 dU'H dU + g'dU s.t. rate/amplitude bounds: unconstrained minimiser, then
 *        a Goldfarb-Idnani dual active-set method (same family as the toolbox's KWIK solver)
 *   u(t) = u(t-1) + dU(first move of every MV)
 * Costs: J1 (GAM_fun.m:110-111), j22 from inK (VNS2.m:173,177); open loop (uopt, ys, j21, Jnu)
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

/* Goldfarb-Idnani dual active-set method in its numerically stable form (the toolbox's KWIK is
 * of this family).  With H = R'R (R from the QR of W) and B = R^-T N_W for the active normals:
 *   b_p = R^-T n_p,  [c; tail] = Qb' b_p (Householder QR of B, recomputed every iteration),
 *   r = Rb^-1 c (dual direction),  e = b_p - B r = Qb [0; tail],  z = R^-1 e (primal direction),
 *   beta = n_p' z = |tail|^2.
 * x holds the unconstrained minimiser on entry.  Rinv is upper triangular, row-major. */
static int gi_qp(const double* Rinv, int M, int Nu, int nu, const double* bnd, const double* up,
                 double* x, double tol, int maxit, int* st) {
  double Bc[CG_MAXM * CG_MAXM]; /* active b_w columns [w][m] */
  double Aw[CG_MAXM * (CG_MAXM + 1)]; /* work: column-major [col][m] */
  double V[CG_MAXM * CG_MAXM], vnv[CG_MAXM];
  double bp[CG_MAXM], e[CG_MAXM], z[CG_MAXM], r[CG_MAXM], u[CG_MAXM];
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
    if (it >= maxit) { /* q == M is legal: beta = 0, the step is a dual one (a drop) */
      *st |= 1;
      break;
    }
    int j0, j1;
    double sg;
    normal_range(p, Nu, &j0, &j1, &sg);
    double bpn = 0.0;
    for (int m = 0; m < M; ++m) {
      double a = 0;
      for (int j = j0; j <= j1; ++j) a += Rinv[j * M + m];
      bp[m] = sg * a;
      bpn += bp[m] * bp[m];
    }
    double sp = best, upm = 0.0;
    for (;;) {
      ++it;
      /* Householder QR of [B | b_p] */
      for (int w = 0; w < q; ++w) memcpy(Aw + w * M, Bc + w * M, sizeof(double) * M);
      memcpy(Aw + q * M, bp, sizeof(double) * M);
      for (int j = 0; j < q; ++j) {
        double* cj = Aw + j * M;
        double nrm = 0;
        for (int k = j; k < M; ++k) nrm += cj[k] * cj[k];
        nrm = sqrt(nrm);
        double alpha = cj[j] > 0 ? -nrm : nrm;
        double* v = V + j * M;
        for (int k = 0; k < M; ++k) v[k] = k < j ? 0.0 : cj[k];
        v[j] -= alpha;
        double vn = 0;
        for (int k = j; k < M; ++k) vn += v[k] * v[k];
        vnv[j] = vn;
        for (int w = j; w <= q; ++w) {
          double* cw = Aw + w * M;
          if (vn == 0.0) continue;
          double dt = 0;
          for (int k = j; k < M; ++k) dt += v[k] * cw[k];
          double f = 2.0 * dt / vn;
          for (int k = j; k < M; ++k) cw[k] -= f * v[k];
        }
      }
      double* cq = Aw + q * M;
      double beta = 0;
      for (int k = q; k < M; ++k) beta += cq[k] * cq[k];
      for (int k = 0; k < M; ++k) e[k] = k < q ? 0.0 : cq[k];
      for (int j = q - 1; j >= 0; --j) {
        const double* v = V + j * M;
        if (vnv[j] == 0.0) continue;
        double dt = 0;
        for (int k = j; k < M; ++k) dt += v[k] * e[k];
        double f = 2.0 * dt / vnv[j];
        for (int k = j; k < M; ++k) e[k] -= f * v[k];
      }
      for (int w = q - 1; w >= 0; --w) { /* Rb r = c */
        double a = cq[w];
        for (int k = w + 1; k < q; ++k) a -= Aw[k * M + w] * r[k];
        r[w] = a / Aw[w * M + w];
      }
      for (int m = 0; m < M; ++m) {
        double a = 0;
        for (int k = m; k < M; ++k) a += Rinv[m * M + k] * e[k];
        z[m] = a;
      }
      double t1 = INFINITY;
      int kd = -1;
      for (int w = 0; w < q; ++w)
        if (r[w] > 0 && u[w] / r[w] < t1) {
          t1 = u[w] / r[w];
          kd = w;
        }
      double t2 = (beta > 1e-14 * bpn) ? -sp / beta : INFINITY;
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
        memcpy(Bc + q * M, bp, sizeof(double) * M);
        u[q] = upm;
        W[q] = p;
        act[p] = 1;
        ++q;
        break;
      }
      /* drop kd (keep order) */
      act[W[kd]] = 0;
      for (int w = kd; w < q - 1; ++w) {
        memcpy(Bc + w * M, Bc + (w + 1) * M, sizeof(double) * M);
        u[w] = u[w + 1];
        W[w] = W[w + 1];
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
  double* RT = (double*)calloc((size_t)M * (M + P), sizeof(double)); /* [R | T] rows */
  double* B = (double*)calloc((size_t)M * P, sizeof(double));
  double* Hi = (double*)calloc((size_t)M * M, sizeof(double)); /* R^-1 */
  double* f = (double*)calloc((size_t)P, sizeof(double));
  double* xs = (double*)calloc((size_t)nx, sizeof(double));
  double* U = (double*)calloc((size_t)2 * nin * nit, sizeof(double)); /* [copy][j][t] */
  double* Ye = (double*)calloc((size_t)2 * sc->ne * nit, sizeof(double));
  double* row = (double*)calloc((size_t)(M + P), sizeof(double));
  double sqw[64], x[CG_MAXM], ucum[CG_MAXM];
  int st = 0;
  int64_t iters = 0;
  const int ncol = M + P;
  for (int i = 0; i < my; ++i) {
    double d = fabs(delta[i]);
    sqw[i] = sc->wsq ? d : sqrt(d); /* Q^1/2 */
  }
  for (int i = 0; i < my; ++i)
    for (int rr = 0; rr < N2; ++rr)
      for (int n = 0; n < nu; ++n)
        for (int c = 0; c < Nu; ++c) {
          int t = sc->n1[i] + rr - c;
          G[(size_t)(i * N2 + rr) * M + n * Nu + c] = t >= 0 ? sc->step[((size_t)i * nu + n) * sc->tlen + t] : 0.0;
        }
  /* QR of W = [Q^1/2 G; Lambda^1/2] by row-streamed Givens rotations, carrying the right-hand
   * block V = [diag(Q^1/2); 0]:  R starts as Lambda^1/2 (already triangular), T = Q1'V. */
  for (int n = 0; n < nu; ++n) {
    double l = fabs(lam[n]);
    double w = sc->wsq ? l : sqrt(l);
    for (int c = 0; c < Nu; ++c) RT[(size_t)(n * Nu + c) * ncol + n * Nu + c] = w;
  }
  for (int k = 0; k < P; ++k) {
    const double q = sqw[k / N2];
    memset(row, 0, sizeof(double) * ncol);
    for (int a = 0; a < M; ++a) row[a] = q * G[(size_t)k * M + a];
    row[M + k] = q;
    for (int a = 0; a < M; ++a) {
      double bb = row[a];
      if (bb == 0.0) continue;
      double aa = RT[(size_t)a * ncol + a];
      double rho = hypot(aa, bb), cs = aa / rho, sn = bb / rho;
      for (int j = a; j < ncol; ++j) {
        double rj = RT[(size_t)a * ncol + j], wj = row[j];
        RT[(size_t)a * ncol + j] = cs * rj + sn * wj;
        row[j] = -sn * rj + cs * wj;
      }
    }
  }
  for (int a = 0; a < M; ++a)
    if (!(RT[(size_t)a * ncol + a] > 0.0)) {
      st |= 4;
      goto done;
    }
  /* B = -R^-1 T  (M x P) */
  for (int k = 0; k < P; ++k)
    for (int a = M - 1; a >= 0; --a) {
      double acc = RT[(size_t)a * ncol + M + k];
      for (int j = a + 1; j < M; ++j) acc -= RT[(size_t)a * ncol + j] * (-B[(size_t)j * P + k]);
      B[(size_t)a * P + k] = -acc / RT[(size_t)a * ncol + a];
    }
  /* R^-1 (upper) for the active-set method */
  for (int j = 0; j < M; ++j)
    for (int a = j; a >= 0; --a) {
      double acc = (a == j) ? 1.0 : 0.0;
      for (int k = a + 1; k <= j; ++k) acc -= RT[(size_t)a * ncol + k] * Hi[(size_t)k * M + j];
      Hi[(size_t)a * M + j] = acc / RT[(size_t)a * ncol + a];
    }
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
      for (int k = 0; k < P; ++k) s += B[(size_t)a * P + k] * f[k];            \
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
  free(RT);
  free(B);
  free(row);
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
