/*
 * cband.c — plain-C restatement of the band-mode / measured-disturbance toolbox closed loop of
 * oracle/toolbox_band.py (config 3, Shell7x5.m:98-196; WoodBerry.m's toolbox MPC), TEST
 * INFRASTRUCTURE ONLY: it scores config-3 grids fast enough to pin the device's free-run costs
 * (tests/golden/make_config3_fixture.py) and replays device trajectories step by step.  Never
 * linked into the product.
 *
 * Per candidate (closedloop_toolbox.m:36-100 semantics, toolbox_band.py:326-386):
 *   S[i][n][k]  unit-step response of every model entry (MatG.m:51, toolbox_band.py:97)
 *   G[(i,k),(n,l)] = s_in(k+1-l), k = 0..N2-1 (toolbox window t+1..t+N2, toolbox_band.py:102)
 *   QP over x = [dU; eps]:  min 1/2 |W x + c|^2,  W = [sqrt(q_i) G_i; diag(sqrt(wl)); sqrt(rho)]
 *     s.t. MV rate/amplitude rows (toolbox_gpc.py:105 order), eps >= 0, and the soft bands
 *     -G_i dU + ecr^max_i s^y_i eps >= f_i - y^max_i,  G_i dU + ecr^min_i s^y_i eps >= y^min_i - f_i
 *   equilibrated (unit Hessian diagonal, unit constraint rows, toolbox_band.py:311-318) and solved
 *   by the textbook Goldfarb-Idnani dual method recomputed densely every iteration (no factor
 *   updates, no warm start; toolbox_band.py:170-246): Hs = L L' (Cholesky), rows Aw = As L^-T,
 *   a fresh Householder QR of the active rows per iteration, exact re-solve after every add.
 * per step t (toolbox_band.py:372-383):
 *   y(t)      exact difference equations of every entry (lsim; MV feed-through is zero)
 *   f         y(t+1..t+N2) with MVs held at u(t-1) and MDs held at v(t): each entry's own
 *             difference equation run forward from its actual history (the numpy oracle
 *             re-simulates the whole history with lfilter; same recursion)
 *   u(t) = u(t-1) + dU(first move of every MV)
 * Costs as cgpc.c: J1 (GAM_fun.m:110-111), j22 from inK, j21/Jnu from the open-loop leg
 * (closedloop_toolbox.m:85-100, VNS2.m:172-191).
 *
 * Build: oracle/Makefile (gcc -O3 -fopenmp -shared -fPIC, strict C11: no FP contraction).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
  int my, nu, nd, nit, wsq, ink0;
  int maxb, maxa;
  const int* nb;      /* [my*nin] numerator length (delay zeros included) */
  const int* na;      /* [my*nin] denominator length, a[0] = 1 */
  const double* b;    /* [my*nin][maxb] */
  const double* a;    /* [my*nin][maxa] */
  const double* bnd;  /* [4][nu]: du_min, du_max, u_min, u_max (+-inf allowed) */
  const double* ymin; /* [my] (+-inf allowed) */
  const double* ymax;
  const double* ecrmin;
  const double* ecrmax;
  const double* sy;   /* [my] OV ScaleFactor */
  const double* su;   /* [nu] MV ScaleFactor */
  double rho;         /* Weights.ECR */
  const double* yref; /* [my][nit] */
  int qp_warm;        /* 1: a second, equally valid QP path -- each step's dual method starts from
                         the previous step's final active set (re-solved exactly on it, negative
                         multipliers dropped) instead of from the unconstrained minimum.  The
                         C-vs-C floor of the config-3 parity (tools/config3_certify.py) */
} cb_scen;

/* status bits (same meaning as the device's) */
enum { CB_ST_MAXIT = 1, CB_ST_INFEAS = 2, CB_ST_NONFINITE = 4, CB_ST_BADH = 16, CB_ST_SLACK = 64 };

#define CB_MAXMP 128

/* ---------------------------------------------------------------------------------------- */
/* model entries: y_e(t) = sum_l b[l] u_j(t-l) - sum_{l>=1} a[l] y_e(t-l)                    */

typedef struct {
  int nb, na, b0; /* b0: first nonzero numerator tap */
  const double* b;
  const double* a;
} entry_t;

static void entries(const cb_scen* sc, entry_t* E) {
  const int nin = sc->nu + sc->nd, ne = sc->my * nin;
  for (int e = 0; e < ne; ++e) {
    E[e].nb = sc->nb[e];
    E[e].na = sc->na[e];
    E[e].b = sc->b + (size_t)e * sc->maxb;
    E[e].a = sc->a + (size_t)e * sc->maxa;
    int b0 = 0;
    while (b0 < E[e].nb && E[e].b[b0] == 0.0) ++b0;
    E[e].b0 = b0;
  }
}

/* unit-step response s(0..n-1) (lsim of ones, toolbox_band.py:97) */
static void step_resp(const entry_t* e, int n, double* s) {
  for (int t = 0; t < n; ++t) {
    double acc = 0.0;
    for (int l = e->b0; l < e->nb; ++l)
      if (t - l >= 0) acc += e->b[l];
    for (int l = 1; l < e->na; ++l)
      if (t - l >= 0) acc -= e->a[l] * s[t - l];
    s[t] = acc;
  }
}

/* ---------------------------------------------------------------------------------------- */
/* the dual method (toolbox_band.py:170-246), dense, on Aw w >= bw with Hessian I             */

typedef struct {
  int Mp, nrow;
  double* Aw;   /* [nrow][Mp] */
  double* bw;   /* [nrow] */
  double* gw;   /* [Mp] */
  double* s;    /* [nrow] work */
  int* act;     /* [Mp] */
  double* V;    /* [Mp][Mp] Householder vectors */
  double* vn;   /* [Mp] */
  double* Rq;   /* [Mp][Mp] R of the active rows, column-major [col][row] */
} dual_t;

/* Householder QR of the active rows' transposes (Mp x q); V, vn, Rq */
static void qr_active(dual_t* D, int q) {
  const int Mp = D->Mp;
  double* Aq = D->Rq;
  for (int w = 0; w < q; ++w) memcpy(Aq + (size_t)w * Mp, D->Aw + (size_t)D->act[w] * Mp, sizeof(double) * Mp);
  for (int j = 0; j < q; ++j) {
    double* cj = Aq + (size_t)j * Mp;
    double nrm = 0.0;
    for (int k = j; k < Mp; ++k) nrm += cj[k] * cj[k];
    nrm = sqrt(nrm);
    double alpha = cj[j] > 0 ? -nrm : nrm;
    double* v = D->V + (size_t)j * Mp;
    for (int k = 0; k < Mp; ++k) v[k] = k < j ? 0.0 : cj[k];
    v[j] -= alpha;
    double vv = 0.0;
    for (int k = j; k < Mp; ++k) vv += v[k] * v[k];
    D->vn[j] = vv;
    if (vv == 0.0) continue;
    for (int w = j; w < q; ++w) {
      double* cw = Aq + (size_t)w * Mp;
      double dt = 0.0;
      for (int k = j; k < Mp; ++k) dt += v[k] * cw[k];
      double f = 2.0 * dt / vv;
      for (int k = j; k < Mp; ++k) cw[k] -= f * v[k];
    }
  }
}

/* y <- Q' y (apply H_1 .. H_q) and y <- Q y (H_q .. H_1) */
static void apply_qt(const dual_t* D, int q, double* y) {
  const int Mp = D->Mp;
  for (int j = 0; j < q; ++j) {
    if (D->vn[j] == 0.0) continue;
    const double* v = D->V + (size_t)j * Mp;
    double dt = 0.0;
    for (int k = j; k < Mp; ++k) dt += v[k] * y[k];
    double f = 2.0 * dt / D->vn[j];
    for (int k = j; k < Mp; ++k) y[k] -= f * v[k];
  }
}

static void apply_q(const dual_t* D, int q, double* y) {
  const int Mp = D->Mp;
  for (int j = q - 1; j >= 0; --j) {
    if (D->vn[j] == 0.0) continue;
    const double* v = D->V + (size_t)j * Mp;
    double dt = 0.0;
    for (int k = j; k < Mp; ++k) dt += v[k] * y[k];
    double f = 2.0 * dt / D->vn[j];
    for (int k = j; k < Mp; ++k) y[k] -= f * v[k];
  }
}

#define RQ(D, r, c) ((D)->Rq[(size_t)(c) * (D)->Mp + (r)])

/* exact solve on the active set act[0..q): w = -gw + Q1 R^-T (b_A + Aw_A gw), u = R^-1 y (raw) */
static void resolve_active(dual_t* D, int q, double* w, double* u) {
  const int Mp = D->Mp;
  double y[CB_MAXMP], z[CB_MAXMP];
  qr_active(D, q);
  for (int j = 0; j < q; ++j) {
    const double* aj = D->Aw + (size_t)D->act[j] * Mp;
    double acc = D->bw[D->act[j]];
    for (int m = 0; m < Mp; ++m) acc += aj[m] * D->gw[m];
    for (int i = 0; i < j; ++i) acc -= RQ(D, i, j) * y[i];
    y[j] = acc / RQ(D, j, j);
  }
  memset(z, 0, sizeof(double) * Mp);
  memcpy(z, y, sizeof(double) * q);
  apply_q(D, q, z);
  for (int m = 0; m < Mp; ++m) w[m] = -D->gw[m] + z[m];
  for (int j = q - 1; j >= 0; --j) {
    double acc = y[j];
    for (int i = j + 1; i < q; ++i) acc -= RQ(D, j, i) * u[i];
    u[j] = acc / RQ(D, j, j);
  }
}

/* w solves min 1/2|w + gw|^2 s.t. Aw w >= bw.  Returns iterations; status bits in *st.
 * q0 > 0: warm start from the active rows D->act[0..q0) (cb_scen.qp_warm): exact solve on them,
 * the most negative multiplier dropped until none is, then the ordinary dual iterations.  *qout:
 * the final active-set size (D->act[0..*qout)) */
static int dual_solve(dual_t* D, double* w, double tol, int maxit, int* st, int q0, int* qout) {
  const int Mp = D->Mp, nrow = D->nrow;
  double u[CB_MAXMP + 1], up[CB_MAXMP + 1], z[CB_MAXMP], qn[CB_MAXMP], r[CB_MAXMP];
  unsigned char* isact = (unsigned char*)calloc((size_t)nrow, 1);
  int q = 0, it = 0;
  for (int m = 0; m < Mp; ++m) w[m] = -D->gw[m];
  if (q0 > 0) {
    q = q0;
    for (int j = 0; j < q; ++j) isact[D->act[j]] = 1;
    while (q > 0) {
      resolve_active(D, q, w, u);
      int k = -1;
      double umin = 0.0;
      for (int j = 0; j < q; ++j)
        if (u[j] < umin) {
          umin = u[j];
          k = j;
        }
      if (k < 0) break;
      ++it;
      isact[D->act[k]] = 0;
      for (int j = k; j < q - 1; ++j) D->act[j] = D->act[j + 1];
      --q;
    }
    if (q == 0)
      for (int m = 0; m < Mp; ++m) w[m] = -D->gw[m];
  }
  for (;;) {
    int p = -1;
    double best = INFINITY;
    for (int i = 0; i < nrow; ++i) {
      if (isact[i]) continue;
      const double* ai = D->Aw + (size_t)i * Mp;
      double s = 0.0;
      for (int m = 0; m < Mp; ++m) s += ai[m] * w[m];
      s -= D->bw[i];
      if (s < best) {
        best = s;
        p = i;
      }
    }
    if (p < 0 || !(best < -tol * fmax(1.0, fabs(D->bw[p])))) break;
    const double* n = D->Aw + (size_t)p * Mp;
    double nn = 0.0;
    for (int m = 0; m < Mp; ++m) nn += n[m] * n[m];
    for (int j = 0; j < q; ++j) up[j] = u[j];
    up[q] = 0.0;
    for (;;) {
      if (++it > maxit) {
        *st |= CB_ST_MAXIT;
        goto out;
      }
      if (q > 0) {
        qr_active(D, q);
        memcpy(qn, n, sizeof(double) * Mp);
        apply_qt(D, q, qn); /* [Q1'n; Q2'n] */
        for (int m = 0; m < Mp; ++m) z[m] = m < q ? 0.0 : qn[m];
        apply_q(D, q, z); /* z = Q2 Q2' n */
        for (int j = q - 1; j >= 0; --j) { /* r = R^-1 Q1' n */
          double acc = qn[j];
          for (int k = j + 1; k < q; ++k) acc -= RQ(D, j, k) * r[k];
          r[j] = acc / RQ(D, j, j);
        }
      } else {
        memcpy(z, n, sizeof(double) * Mp);
      }
      double zn = 0.0, nw = 0.0;
      for (int m = 0; m < Mp; ++m) {
        zn += z[m] * n[m];
        nw += n[m] * w[m];
      }
      double t2 = zn > 1e-20 * nn ? -(nw - D->bw[p]) / zn : INFINITY;
      double t1 = INFINITY;
      int k = -1;
      for (int j = 0; j < q; ++j)
        if (r[j] > 0) {
          double ra = up[j] / r[j];
          if (ra < t1) {
            t1 = ra;
            k = j;
          }
        }
      double t = t1 < t2 ? t1 : t2;
      if (!isfinite(t)) {
        *st |= CB_ST_INFEAS;
        goto out;
      }
      if (isfinite(t2))
        for (int m = 0; m < Mp; ++m) w[m] += t * z[m];
      for (int j = 0; j < q; ++j) up[j] -= t * r[j];
      up[q] += t;
      if (t2 <= t1) {
        D->act[q++] = p;
        isact[p] = 1;
        /* exact re-solve on the active set */
        resolve_active(D, q, w, u);
        for (int j = 0; j < q; ++j) u[j] = fmax(u[j], 0.0);
        break;
      }
      /* drop k (keep order) */
      isact[D->act[k]] = 0;
      for (int j = k; j < q - 1; ++j) {
        D->act[j] = D->act[j + 1];
        up[j] = up[j + 1];
      }
      up[q - 1] = up[q];
      --q;
    }
  }
out:
  /* feasibility of the returned point (the numpy oracle's KKT check raises on a slack < -1e-9) */
  {
    double smin = INFINITY;
    for (int i = 0; i < nrow; ++i) {
      const double* ai = D->Aw + (size_t)i * Mp;
      double s = 0.0;
      for (int m = 0; m < Mp; ++m) s += ai[m] * w[m];
      s -= D->bw[i];
      if (s < smin) smin = s;
    }
    if (smin < -1e-9) *st |= CB_ST_SLACK;
  }
  free(isact);
  if (qout) *qout = q;
  return it;
}

/* ---------------------------------------------------------------------------------------- */
/* one candidate                                                                              */

typedef struct {
  int my, nu, nd, nin, ne, N2, Nu, M, Mp, nrow;
  entry_t* E;
  double* G;      /* [my*N2][M] */
  double* Ls;     /* [Mp][Mp] lower Cholesky factor of Hs */
  double* dsc;    /* [Mp] */
  double* rn;     /* [nrow] row norms of A*dsc */
  int* rkind;     /* [nrow] 0 du_min, 1 du_max, 2 u_min, 3 u_max, 4 eps, 5 y_max, 6 y_min,
                     7 / 8 du_n(0) >= / <= a pinned value (replay-gap mode only, last 2 nu rows) */
  int* rarg;      /* [nrow] move index m (kinds 0-3, 7-8) or (i*N2 + k) (kinds 5-6) */
  double* wq;     /* [my] */
  double wl[64];  /* [nu] move weights */
  int warm, q_prev; /* qp_warm: the previous QP's final active-set size (D.act[0..q_prev)) */
  int pin_on;       /* pin rows enforce pin[] (else their bounds are -inf: never violated) */
  double pin[64];
  dual_t D;
} cand_t;

static void cand_free(cand_t* c) {
  free(c->E);
  free(c->G);
  free(c->Ls);
  free(c->dsc);
  free(c->rn);
  free(c->rkind);
  free(c->rarg);
  free(c->wq);
  free(c->D.Aw);
  free(c->D.bw);
  free(c->D.gw);
  free(c->D.s);
  free(c->D.act);
  free(c->D.V);
  free(c->D.vn);
  free(c->D.Rq);
}

/* A row (unscaled) of kind/arg into a[0..Mp-1] */
static void a_row(const cand_t* c, const cb_scen* sc, int kind, int arg, double* a) {
  const int M = c->M, Nu = c->Nu;
  memset(a, 0, sizeof(double) * c->Mp);
  if (kind >= 7) {
    a[arg] = kind == 7 ? 1.0 : -1.0;
  } else if (kind <= 3) {
    int n = arg / Nu;
    if (kind == 0) a[arg] = 1.0;
    else if (kind == 1) a[arg] = -1.0;
    else
      for (int j = n * Nu; j <= arg; ++j) a[j] = kind == 2 ? 1.0 : -1.0;
  } else if (kind == 4) {
    a[M] = 1.0;
  } else {
    int i = arg / c->N2;
    const double* g = c->G + (size_t)arg * M;
    double sg = kind == 5 ? -1.0 : 1.0;
    for (int m = 0; m < M; ++m) a[m] = sg * g[m];
    a[M] = (kind == 5 ? sc->ecrmax[i] : sc->ecrmin[i]) * sc->sy[i];
  }
}

static int cand_setup(cand_t* c, const cb_scen* sc, int N2, int Nu, const double* delta, const double* lam,
                      double* wl, int pin_rows) {
  const int my = sc->my, nu = sc->nu, nin = sc->nu + sc->nd;
  memset(c, 0, sizeof(*c));
  c->my = my;
  c->nu = nu;
  c->nd = sc->nd;
  c->nin = nin;
  c->ne = my * nin;
  c->N2 = N2;
  c->Nu = Nu;
  c->M = nu * Nu;
  c->Mp = c->M + 1;
  if (N2 < 1 || Nu < 1 || Nu > N2 || c->Mp > CB_MAXMP) return CB_ST_BADH;
  const int M = c->M, Mp = c->Mp;
  c->E = (entry_t*)malloc(sizeof(entry_t) * c->ne);
  entries(sc, c->E);
  c->wq = (double*)malloc(sizeof(double) * my);
  for (int i = 0; i < my; ++i) {
    double d = fabs(delta[i]) / sc->sy[i];
    c->wq[i] = sc->wsq ? d * d : d;
  }
  for (int n = 0; n < nu; ++n) {
    double l = fabs(lam[n]) / sc->su[n];
    wl[n] = sc->wsq ? l * l : l;
    c->wl[n] = wl[n];
  }
  c->warm = sc->qp_warm;
  /* step table and G (toolbox_band.py:97-113) */
  double* S = (double*)malloc(sizeof(double) * (N2 + 2));
  c->G = (double*)calloc((size_t)my * N2 * M, sizeof(double));
  for (int i = 0; i < my; ++i)
    for (int n = 0; n < nu; ++n) {
      step_resp(&c->E[i * nin + n], N2 + 2, S);
      for (int k = 0; k < N2; ++k)
        for (int l = 0; l < Nu; ++l)
          if (k + 1 - l >= 0) c->G[(size_t)(i * N2 + k) * M + n * Nu + l] = S[k + 1 - l];
    }
  free(S);
  /* H = W'W (dense), dsc = diag(H)^-1/2, Hs = D H D = Ls Ls' (toolbox_band.py:314, :189-191) */
  double* H = (double*)calloc((size_t)Mp * Mp, sizeof(double));
  for (int i = 0; i < my; ++i) {
    if (!(c->wq[i] > 0)) continue;
    double q = sqrt(c->wq[i]);
    for (int k = 0; k < N2; ++k) {
      const double* g = c->G + (size_t)(i * N2 + k) * M;
      for (int a = 0; a < M; ++a) {
        double ga = q * g[a];
        if (ga == 0.0) continue;
        for (int b = 0; b < M; ++b) H[a * Mp + b] += ga * (q * g[b]);
      }
    }
  }
  for (int n = 0; n < nu; ++n)
    for (int l = 0; l < Nu; ++l) {
      double sw = sqrt(wl[n]);
      H[(n * Nu + l) * Mp + n * Nu + l] += sw * sw;
    }
  {
    double sr = sqrt(sc->rho);
    H[M * Mp + M] += sr * sr;
  }
  c->dsc = (double*)malloc(sizeof(double) * Mp);
  for (int a = 0; a < Mp; ++a) c->dsc[a] = 1.0 / sqrt(H[a * Mp + a]);
  c->Ls = (double*)calloc((size_t)Mp * Mp, sizeof(double));
  for (int j = 0; j < Mp; ++j) {
    double d = H[j * Mp + j] * c->dsc[j] * c->dsc[j];
    for (int k = 0; k < j; ++k) d -= c->Ls[j * Mp + k] * c->Ls[j * Mp + k];
    if (!(d > 0)) {
      free(H);
      return CB_ST_BADH;
    }
    d = sqrt(d);
    c->Ls[j * Mp + j] = d;
    for (int i = j + 1; i < Mp; ++i) {
      double v = H[i * Mp + j] * c->dsc[i] * c->dsc[j];
      for (int k = 0; k < j; ++k) v -= c->Ls[i * Mp + k] * c->Ls[j * Mp + k];
      c->Ls[i * Mp + j] = v / d;
    }
  }
  free(H);
  /* constraint rows in toolbox_band.py:284-298 order */
  int cap = 4 * M + 1 + 2 * my * N2 + 2 * nu;
  c->rkind = (int*)malloc(sizeof(int) * cap);
  c->rarg = (int*)malloc(sizeof(int) * cap);
  int nr = 0;
  for (int n = 0; n < nu; ++n)
    for (int l = 0; l < Nu; ++l) {
      int m = n * Nu + l;
      for (int kind = 0; kind < 4; ++kind)
        if (isfinite(sc->bnd[kind * nu + n])) {
          c->rkind[nr] = kind;
          c->rarg[nr++] = m;
        }
    }
  c->rkind[nr] = 4;
  c->rarg[nr++] = 0;
  for (int i = 0; i < my; ++i) {
    if (isfinite(sc->ymax[i]))
      for (int k = 0; k < N2; ++k) {
        c->rkind[nr] = 5;
        c->rarg[nr++] = i * N2 + k;
      }
    if (isfinite(sc->ymin[i]))
      for (int k = 0; k < N2; ++k) {
        c->rkind[nr] = 6;
        c->rarg[nr++] = i * N2 + k;
      }
  }
  if (pin_rows)
    for (int n = 0; n < nu; ++n)
      for (int kind = 7; kind <= 8; ++kind) {
        c->rkind[nr] = kind;
        c->rarg[nr++] = n * Nu;
      }
  c->nrow = nr;
  /* Aw = (A D / rn) Ls^-T: row-wise forward substitution with Ls */
  c->rn = (double*)malloc(sizeof(double) * nr);
  dual_t* D = &c->D;
  D->Mp = Mp;
  D->nrow = nr;
  D->Aw = (double*)malloc(sizeof(double) * (size_t)nr * Mp);
  D->bw = (double*)malloc(sizeof(double) * nr);
  D->gw = (double*)malloc(sizeof(double) * Mp);
  D->s = (double*)malloc(sizeof(double) * nr);
  D->act = (int*)malloc(sizeof(int) * Mp);
  D->V = (double*)malloc(sizeof(double) * Mp * Mp);
  D->vn = (double*)malloc(sizeof(double) * Mp);
  D->Rq = (double*)malloc(sizeof(double) * Mp * Mp);
  double arow[CB_MAXMP];
  for (int r = 0; r < nr; ++r) {
    a_row(c, sc, c->rkind[r], c->rarg[r], arow);
    double nrm = 0.0;
    for (int m = 0; m < Mp; ++m) {
      arow[m] *= c->dsc[m];
      nrm += arow[m] * arow[m];
    }
    nrm = sqrt(nrm);
    if (nrm == 0.0) nrm = 1.0;
    c->rn[r] = nrm;
    double* aw = D->Aw + (size_t)r * Mp;
    for (int m = 0; m < Mp; ++m) {
      double acc = arow[m] / nrm;
      for (int k = 0; k < m; ++k) acc -= c->Ls[m * Mp + k] * aw[k];
      aw[m] = acc / c->Ls[m * Mp + m];
    }
  }
  return 0;
}

/* the toolbox QP at free response f (my*N2), reference rv (my), u(t-1) = up; x = [dU; eps] */
static int cand_qp(cand_t* c, const cb_scen* sc, const double* f, const double* rv, const double* up,
                   double* x, int* st) {
  const int M = c->M, Mp = c->Mp, N2 = c->N2, nu = c->nu;
  dual_t* D = &c->D;
  /* g = D W'c, c = [sqrt(q_i)(f_i - r_i); 0] (toolbox_band.py:270-283); gw = Ls^-1 g */
  double g[CB_MAXMP];
  memset(g, 0, sizeof(double) * Mp);
  for (int i = 0; i < c->my; ++i) {
    if (!(c->wq[i] > 0)) continue;
    double q = sqrt(c->wq[i]);
    for (int k = 0; k < N2; ++k) {
      double ck = q * (f[i * N2 + k] - rv[i]);
      const double* gr = c->G + (size_t)(i * N2 + k) * M;
      for (int m = 0; m < M; ++m) g[m] += (q * gr[m]) * ck;
    }
  }
  for (int m = 0; m < Mp; ++m) {
    double acc = g[m] * c->dsc[m];
    for (int k = 0; k < m; ++k) acc -= c->Ls[m * Mp + k] * D->gw[k];
    D->gw[m] = acc / c->Ls[m * Mp + m];
  }
  for (int r = 0; r < c->nrow; ++r) {
    int kind = c->rkind[r], arg = c->rarg[r];
    double b;
    int n = arg / c->Nu;
    switch (kind) {
      case 0: b = sc->bnd[n]; break;
      case 1: b = -sc->bnd[nu + n]; break;
      case 2: b = sc->bnd[2 * nu + n] - up[n]; break;
      case 3: b = -(sc->bnd[3 * nu + n] - up[n]); break;
      case 4: b = 0.0; break;
      case 5: b = f[arg] - sc->ymax[arg / N2]; break;
      case 6: b = sc->ymin[arg / N2] - f[arg]; break;
      case 7: b = c->pin_on ? c->pin[n] : -INFINITY; break;
      default: b = c->pin_on ? -c->pin[n] : -INFINITY; break;
    }
    D->bw[r] = b / c->rn[r];
  }
  double w[CB_MAXMP];
  int it = dual_solve(D, w, 1e-12, 5000, st, c->warm ? c->q_prev : 0, &c->q_prev);
  /* x = D Ls^-T w */
  for (int m = Mp - 1; m >= 0; --m) {
    double acc = w[m];
    for (int k = m + 1; k < Mp; ++k) acc -= c->Ls[k * Mp + m] * x[k];
    x[m] = acc / c->Ls[m * Mp + m];
  }
  for (int m = 0; m < Mp; ++m) x[m] *= c->dsc[m];
  (void)M;
  return it;
}

/* the QP objective 1/2 |W x + c|^2 at x = [dU; eps] (toolbox_band.py band_qp with_obj) */
static double cand_obj(const cand_t* c, const cb_scen* sc, const double* f, const double* rv, const double* x) {
  const int M = c->M, N2 = c->N2;
  double J = 0.0;
  for (int i = 0; i < c->my; ++i) {
    if (!(c->wq[i] > 0)) continue;
    for (int k = 0; k < N2; ++k) {
      const double* g = c->G + (size_t)(i * N2 + k) * M;
      double e = f[i * N2 + k] - rv[i];
      for (int m = 0; m < M; ++m) e += g[m] * x[m];
      J += c->wq[i] * e * e;
    }
  }
  for (int m = 0; m < M; ++m) J += c->wl[m / c->Nu] * x[m] * x[m];
  J += sc->rho * x[M] * x[M];
  return 0.5 * J;
}

/* history input of column j at time tau: before t the applied signal, from t on the held value */
static inline double u_at(const double* Uj, int tau, int t, double hold) {
  if (tau < 0) return 0.0;
  return tau < t ? Uj[tau] : hold;
}

/* free response f[i*N2 + k] = y_i(t+1+k), MVs held at up from t, MDs held at v(t); Ye holds the
 * actual entry outputs 0..t.  yq: scratch [N2+1] */
static void free_response(const cand_t* c, const double* U, const double* Ye, int t, int nT, const double* up,
                          const double* vt, double* f, double* yq) {
  const int N2 = c->N2, nin = c->nin, nu = c->nu;
  memset(f, 0, sizeof(double) * c->my * N2);
  for (int i = 0; i < c->my; ++i)
    for (int j = 0; j < nin; ++j) {
      const entry_t* e = &c->E[i * nin + j];
      if (e->b0 >= e->nb) continue;
      const double* Uj = U + (size_t)j * nT;
      const double* ye = Ye + (size_t)(i * nin + j) * nT;
      double hold = j < nu ? up[j] : vt[j - nu];
      yq[0] = ye[t];
      for (int k = 1; k <= N2; ++k) {
        int tau = t + k;
        double acc = 0.0;
        for (int l = e->b0; l < e->nb; ++l) acc += e->b[l] * u_at(Uj, tau - l, t, hold);
        for (int l = 1; l < e->na; ++l) {
          int s = tau - l;
          double yv = s < 0 ? 0.0 : (s <= t ? ye[s] : yq[s - t]);
          acc -= e->a[l] * yv;
        }
        yq[k] = acc;
        f[i * N2 + k - 1] += acc;
      }
    }
}

/* entry outputs at time t from the applied inputs U[:, < t] (MVs) and U[:, <= t] (MDs); the MV
 * feed-through b[0] is zero for every proper toolbox model (checked by the caller) */
static void step_plant(const cand_t* c, const double* U, double* Ye, int t, int nT, double* y) {
  const int nin = c->nin;
  for (int i = 0; i < c->my; ++i) y[i] = 0.0;
  for (int i = 0; i < c->my; ++i)
    for (int j = 0; j < nin; ++j) {
      const entry_t* e = &c->E[i * nin + j];
      double* ye = Ye + (size_t)(i * nin + j) * nT;
      const double* Uj = U + (size_t)j * nT;
      double acc = 0.0;
      for (int l = e->b0; l < e->nb; ++l)
        if (t - l >= 0) acc += e->b[l] * Uj[t - l];
      for (int l = 1; l < e->na; ++l)
        if (t - l >= 0) acc -= e->a[l] * ye[t - l];
      ye[t] = acc;
      y[i] += acc;
    }
}

/* one closed loop.  Uforce (nu x nit) != NULL: replay mode -- the applied MVs are Uforce and
 * du_o[n*T + t] receives the oracle's first move at each step t < T (toolbox_band.py:389-421). */
static int simulate(const cb_scen* sc, int N2, int Nu, const double* delta, const double* lam, const double* r,
                    const double* v, int open_loop, const double* Uforce, int T, double* du_o, double* J1,
                    double* j21, double* j22, double* Jnu, int64_t* iters_out, double* ytraj, double* utraj,
                    double* ystraj, double* uopttraj, double* gap_free, double* gap_pin) {
  const int my = sc->my, nu = sc->nu, nd = sc->nd, nin = nu + nd, nit = sc->nit;
  double wl[64];
  cand_t c;
  int st = cand_setup(&c, sc, N2, Nu, delta, lam, wl, gap_pin != NULL);
  int64_t iters = 0;
  if (st) {
    cand_free(&c);
    if (iters_out) *iters_out = 0;
    return st;
  }
  const int M = c.M, Mp = c.Mp, nT = nit + 1;
  double* U = (double*)calloc((size_t)2 * nin * nT, sizeof(double)); /* [copy][j][t] */
  double* Ye = (double*)calloc((size_t)2 * c.ne * nT, sizeof(double));
  double* f = (double*)malloc(sizeof(double) * my * N2);
  double* yq = (double*)malloc(sizeof(double) * (N2 + 1));
  double x[CB_MAXMP], up[64], vt[64], rv[64], ycl[64], yol[64];
  double sj1[64], sj21[64], sj22[64], jn[64];
  memset(sj1, 0, sizeof(sj1));
  memset(sj21, 0, sizeof(sj21));
  memset(sj22, 0, sizeof(sj22));
  memset(jn, 0, sizeof(jn));
  memset(up, 0, sizeof(up));
  for (int j = 0; j < nd; ++j)
    for (int t = 0; t < nit; ++t) U[(size_t)(nu + j) * nT + t] = v[(size_t)j * nit + t];
  if (open_loop) {
    /* closedloop_toolbox.m:85-100 / toolbox_band.py:354-364: the QP from rest with r(:,end) and
     * the MDs held at v(:,end) from time 0; uopt = cumulative moves, padded; ys = lsim([uopt v]) */
    double* U0 = (double*)calloc((size_t)nin * nT, sizeof(double));
    double* Y0 = (double*)calloc((size_t)c.ne * nT, sizeof(double));
    for (int j = 0; j < nd; ++j) vt[j] = v[(size_t)j * nit + nit - 1];
    for (int i = 0; i < my; ++i) rv[i] = r[(size_t)i * nit + nit - 1];
    for (int e = 0; e < c.ne; ++e) Y0[(size_t)e * nT] = 0.0;
    /* f0 = y(1..N2) from rest with the MDs held from time 0 (entry outputs at 0 use v_end) */
    for (int i = 0; i < my; ++i)
      for (int j = nu; j < nin; ++j) {
        const entry_t* e = &c.E[i * nin + j];
        Y0[(size_t)(i * nin + j) * nT] = e->b0 == 0 && e->nb > 0 ? e->b[0] * vt[j - nu] : 0.0;
      }
    free_response(&c, U0, Y0, 0, nT, up, vt, f, yq);
    iters += cand_qp(&c, sc, f, rv, up, x, &st);
    free(U0);
    free(Y0);
    double ucum[CB_MAXMP];
    for (int n = 0; n < nu; ++n) {
      double s = 0.0;
      for (int l = 0; l < Nu; ++l) {
        s += x[n * Nu + l];
        ucum[n * Nu + l] = s;
      }
      double u0 = fabs(ucum[n * Nu]);
      int ndf = Nu - 1 < nit - 1 ? Nu - 1 : nit - 1;
      for (int t = 0; t < ndf; ++t) {
        double d = fabs(ucum[n * Nu + t + 1] - ucum[n * Nu + t]);
        double xr = u0 / d;
        if (isfinite(xr)) jn[n] += xr * xr;
      }
      for (int t = 0; t < nit; ++t) U[(size_t)(nin + n) * nT + t] = ucum[n * Nu + (t < Nu - 1 ? t : Nu - 1)];
    }
    for (int j = 0; j < nd; ++j)
      for (int t = 0; t < nit; ++t) U[(size_t)(nin + nu + j) * nT + t] = v[(size_t)j * nit + t];
  }
  for (int t = 0; t < nit; ++t) {
    step_plant(&c, U, Ye, t, nT, ycl);
    if (open_loop) {
      /* ys = lsim(Pz, [uopt v]): the open-loop copy sees its own MV at t too */
      for (int i = 0; i < my; ++i) yol[i] = 0.0;
      for (int i = 0; i < my; ++i)
        for (int j = 0; j < nin; ++j) {
          const entry_t* e = &c.E[i * nin + j];
          double* ye = Ye + (size_t)(c.ne + i * nin + j) * nT;
          const double* Uj = U + (size_t)(nin + j) * nT;
          double acc = 0.0;
          for (int l = e->b0; l < e->nb; ++l)
            if (t - l >= 0) acc += e->b[l] * Uj[t - l];
          for (int l = 1; l < e->na; ++l)
            if (t - l >= 0) acc -= e->a[l] * ye[t - l];
          ye[t] = acc;
          yol[i] += acc;
        }
    }
    for (int i = 0; i < my; ++i) {
      double e1 = ycl[i] - sc->yref[(size_t)i * nit + t];
      sj1[i] += e1 * e1;
      if (t >= sc->ink0) sj22[i] += e1 * e1;
      if (open_loop && t >= sc->ink0) sj21[i] += (ycl[i] - yol[i]) * (ycl[i] - yol[i]);
      if (ytraj) ytraj[(size_t)i * nit + t] = ycl[i];
      if (ystraj && open_loop) ystraj[(size_t)i * nit + t] = yol[i];
    }
    if (Uforce && t >= T) break;
    for (int j = 0; j < nd; ++j) vt[j] = v[(size_t)j * nit + t];
    for (int i = 0; i < my; ++i) rv[i] = r[(size_t)i * nit + t];
    free_response(&c, U, Ye, t, nT, up, vt, f, yq);
    iters += cand_qp(&c, sc, f, rv, up, x, &st);
    if (Uforce && gap_pin) {
      /* replay gap (toolbox_band.py pinned_gap): the objective at the free optimum, and the
       * optimum with every MV's first move pinned to the applied one */
      double xp[CB_MAXMP];
      gap_free[t] = cand_obj(&c, sc, f, rv, x);
      for (int n = 0; n < nu; ++n) c.pin[n] = Uforce[(size_t)n * nit + t] - up[n];
      int stp = 0; /* a failed pinned QP marks its step (NaN), not the replay */
      c.pin_on = 1;
      cand_qp(&c, sc, f, rv, up, xp, &stp);
      c.pin_on = 0;
      gap_pin[t] = stp ? NAN : cand_obj(&c, sc, f, rv, xp);
    }
    for (int n = 0; n < nu; ++n) {
      double un;
      if (Uforce) {
        du_o[(size_t)n * T + t] = x[n * Nu];
        un = Uforce[(size_t)n * nit + t];
      } else {
        un = up[n] + x[n * Nu];
      }
      U[(size_t)n * nT + t] = un;
      up[n] = un;
      if (utraj) utraj[(size_t)n * nit + t] = un;
      if (uopttraj && open_loop) uopttraj[(size_t)n * nit + t] = U[(size_t)(nin + n) * nT + t];
    }
  }
  for (int i = 0; i < my; ++i) {
    if (J1) J1[i] = sj1[i];
    if (j22) j22[i] = sj22[i];
    if (j21) j21[i] = open_loop ? sj21[i] : NAN;
    if (!isfinite(sj1[i])) st |= CB_ST_NONFINITE;
  }
  for (int n = 0; n < nu; ++n)
    if (Jnu) Jnu[n] = open_loop ? jn[n] : NAN;
  (void)M;
  (void)Mp;
  free(U);
  free(Ye);
  free(f);
  free(yq);
  cand_free(&c);
  if (iters_out) *iters_out = iters;
  return st;
}

/* C candidates x nref reference sets (r [nref][my][nit], v [nref][nd][nit]); result layout as
 * mpct_eval_batch (simulation s = c*nref + k). */
int cband_eval(const cb_scen* sc, int64_t C, const int* N2, const int* Nu, const double* delta,
               const double* lam, int nref, const double* r, const double* v, int open_loop, int nthreads,
               double* J1, double* j21, double* j22, double* Jnu, int* status, int64_t* iters, double* ytraj,
               double* utraj, double* ystraj, double* uopttraj) {
  const int my = sc->my, nu = sc->nu, nd = sc->nd, nit = sc->nit;
  const int64_t S = C * nref;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int64_t s = 0; s < S; ++s) {
    int64_t c = s / nref;
    int k = (int)(s - c * nref);
    status[s] = simulate(sc, N2[c], Nu[c], delta + c * my, lam + c * nu, r + (size_t)k * my * nit,
                         v + (size_t)k * nd * nit, open_loop, NULL, 0, NULL, J1 + s * my, j21 + s * my,
                         j22 + s * my, Jnu + s * nu, iters + s, ytraj ? ytraj + (size_t)s * my * nit : 0,
                         utraj ? utraj + (size_t)s * nu * nit : 0, ystraj ? ystraj + (size_t)s * my * nit : 0,
                         uopttraj ? uopttraj + (size_t)s * nu * nit : 0, NULL, NULL);
  }
  return 0;
}

/* Per-step replay of C applied MV trajectories U [C][nu][nit] (one reference set r, v): the
 * oracle's first move at the state each trajectory actually reached, du_o [C][nu][T]. */
int cband_replay(const cb_scen* sc, int64_t C, const int* N2, const int* Nu, const double* delta,
                 const double* lam, const double* r, const double* v, const double* U, int T, int nthreads,
                 double* du_o, int* status) {
  const int my = sc->my, nu = sc->nu, nit = sc->nit;
  if (T < 0 || T > nit) return -1;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int64_t c = 0; c < C; ++c)
    status[c] = simulate(sc, N2[c], Nu[c], delta + c * my, lam + c * nu, r, v, 0, U + (size_t)c * nu * nit, T,
                         du_o + (size_t)c * nu * T, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL,
                         NULL, NULL);
  return 0;
}

/* The replay plus, at every step t < T, toolbox_band.py pinned_gap's two objectives: gap_free
 * [C][T] at the oracle's optimum of the state the trajectory reached, gap_pin [C][T] with every
 * MV's first move pinned to the applied one.  A move that differs from the oracle's yet attains
 * its optimal cost is an equally optimal solution of a flat QP. */
int cband_replay_gap(const cb_scen* sc, int64_t C, const int* N2, const int* Nu, const double* delta,
                     const double* lam, const double* r, const double* v, const double* U, int T, int nthreads,
                     double* du_o, double* gap_free, double* gap_pin, int* status) {
  const int my = sc->my, nu = sc->nu, nit = sc->nit;
  if (T < 0 || T > nit) return -1;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int64_t c = 0; c < C; ++c)
    status[c] = simulate(sc, N2[c], Nu[c], delta + c * my, lam + c * nu, r, v, 0, U + (size_t)c * nu * nit, T,
                         du_o + (size_t)c * nu * T, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL,
                         gap_free + (size_t)c * T, gap_pin + (size_t)c * T);
  return 0;
}
