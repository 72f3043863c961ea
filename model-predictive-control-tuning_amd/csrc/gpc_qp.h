// gpc_qp.h — the per-step QP of the linear closed-loop kernel (gpc_closed_loop_kernel):
// Goldfarb-Idnani on the box-constrained moves
// (rate / amplitude rows of MV blocks), warm-started from the previous step's active set
// (gi_core.h).  Runs on lanes 0..M-1 of the wave with wave-uniform control flow.
#pragma once
#include "gi_core.h"

// J (and R_A) are rebuilt from R^-1 after this many x M rotations.  M <= 16 class:
// 8 M was 5 % faster than 4 M, 32 M 1.5 % faster than 8 M (profiles/r02k_gib_rebuild_ab.txt), and
// with the register QP 128 M 3-4 % faster than 32 M at 4096 candidates with the same metric-grid
// parity (profiles/r03v_rebuild128_vptr_ab.txt).  DTC instances (config 4's mismatch draws) keep
// 32 M: 128 M was never measured where the interval actually fires on them.  The <32> / <64>
// classes keep 8 M (longer active sets apply more rotations per add).
constexpr int kGiRebuild16 = 128;
constexpr int kGiRebuild16Dtc = 32;
constexpr int kGiRebuildWide = 8;

namespace mpct {

// normal of constraint p = 4m + kind: rows j0..m of the MV block, sign
__device__ __forceinline__ void gi_normal(int p, const RowCons& rc, int& j0, int& mp, double& sg) {
  mp = p >> 2;
  const int kind = p & 3;
  j0 = kind < 2 ? mp : mp - __builtin_amdgcn_readlane(rc.l, mp);
  sg = (kind & 1) ? -1.0 : 1.0;
}

// the LDS arrays of one simulation's QP (lanes 0..M-1 are its rows)
struct QPBufs {
  const double* rinv;  // R^-1 (row-major)
  double *xc;          // in: -, out: the optimal moves (lanes < M)
  double *jt, *dv, *ra, *sl;
};

// the QP of one step: unconstrained minimiser xu (lanes < M), u(t-1) of the lane's MV up_row
template <int MAXM>
__device__ __forceinline__ int gi_qp(const QPBufs& Q, int M, int Nu, const RowCons& rc, double up_row,
                     double xu, double tol, int maxit, int* st, GIState<MAXM>& S
#ifdef MPCT_PROFILE
                     , ProfAccS& pacc, unsigned long long& pprev
#endif
                     ) {
  const int lane = qp_lane();
  const bool row = lane < M;
  const double* sRi = Q.rinv;
  double* sxc = Q.xc;
  double* sJT = Q.jt;
  double* sd = Q.dv;
  double* sRA = Q.ra;
  double* ssl = Q.sl;
  if (!row) up_row = 0.0;
  const int rl = rc.l;  // the lane's position in its MV block
  const double lo_box = fmax(rc.dmin, rc.umin - up_row), hi_box = fmin(rc.dmax, rc.umax - up_row);
  auto slacks = [&](double x, double s[4]) {
    const double pre = block_prefix<MAXM>(x, rl, Nu, row, sxc);
    if (rl == 0) {
      s[0] = x - lo_box;
      s[1] = hi_box - x;
      s[2] = INFINITY;
      s[3] = INFINITY;
    } else {
      s[0] = x - rc.dmin;
      s[1] = rc.dmax - x;
      s[2] = pre - (rc.umin - up_row);
      s[3] = (rc.umax - up_row) - pre;
    }
    if (!row) s[0] = s[1] = s[2] = s[3] = INFINITY;
  };
  int it = 0;
  double xm = xu;
  {
    // the unconstrained minimiser is optimal when it is feasible (the retained set is kept)
    double s[4];
    slacks(xu, s);
    const double smin = fmin(fmin(s[0], s[1]), fmin(s[2], s[3]));
    if (__ballot(smin < -tol) == 0) return 0;  // sxc already holds x_u (solve_step)
    if (S.q == 0) {
      S.jinit = false;  // nothing retained: restart from R^-1 when the first constraint enters
    } else {
      if (row) {
#pragma unroll
        for (int k = 0; k < 4; ++k) ssl[4 * lane + k] = s[k];
      }
      if (!S.jinit || S.nrot >= kGiRebuildWide * M) {
        // rebuild J (and R_A) for the retained set from R^-1, re-adding it in order
        const int qq = S.q;
        gi_load_rinv<MAXM>(S, sJT, sRi, M, row);
        S.q = 0;
        for (int v = 0; v < qq; ++v) {
          const int p = __builtin_amdgcn_readlane(S.ww, v);
          int j0, mp;
          double sg;
          gi_normal(p, rc, j0, mp, sg);
          const double dk = gi_dvec<MAXM>(sJT, sd, M, j0, mp, sg, row);
          const double beta = qsum<MAXM>(lane >= v ? dk * dk : 0.0);
          lds_sync();
          const double zm = gi_z(sJT, sd, v, M, row);
          const double uk = S.uw;
          gi_add<MAXM>(S, sJT, sRA, sd, M, p, dk, beta, zm, 0.0, row, BoxMark{});
          if (lane == v) S.uw = uk;
          ++it;
        }
        S.nrot = 0;
      }
      lds_sync();
      // equality-constrained solve on the retained set, dropping negative multipliers
      for (;;) {
        const int q = S.q;
        if (q == 0) {
          xm = xu;
          break;
        }
        double c = 0.0;
        if (lane < q) c = -ssl[S.ww];  // b_A - N_A'x_u
        double lam;
        xm = xu;
        {
          double wv = 0.0;
          for (int v = 0; v < q; ++v) {  // forward substitution R_A'w = c, x = x_u + J(:,0:q) w
            const double w = bcast(c * S.rdg, v);
            if (lane == v) wv = w;
            if (lane > v && lane < q) c -= sRA[v * M + lane] * w;
            if (row) xm += sJT[v * M + lane] * w;
          }
          lam = gi_backsub<MAXM>(S, sRA, M, wv);
        }
        if (lane < q) S.uw = lam;
        double lmin = lane < q ? lam : INFINITY;
        int kd = lane;
        qargmin<MAXM>(lmin, kd);
        if (!(lmin < 0.0)) break;
#ifdef MPCT_DIAG
        if (!(S.diag & kDiagSkipWarmDrop))
#endif
        gi_drop<MAXM>(S, sJT, sRA, M, kd, BoxMark{});
        if (++it >= maxit) {  // a drop shrinks the set: only a logic slip reaches the cap (gpc_qp16.h)
          *st |= MPCT_ST_QP_MAXITER_;
          break;
        }
      }
      if (!row) xm = 0.0;
    }
  }
  PSTAMP(PROF_QWARM);
  for (;;) {
    // ---- most violated inactive constraint
    double best = INFINITY;
    int bid = 0x7fffffff;
    {
      double s[4];
      slacks(xm, s);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (!((S.act >> k) & 1u) && s[k] < best) {
          best = s[k];
          bid = 4 * lane + k;
        }
    }
    qargmin<MAXM>(best, bid, 2);
    PSTAMP(PROF_QCHECK);
    if (!(best < -tol)) break;
    if (it >= maxit) {  // a full active set is legal (a dual step follows, gpc_qp16.h)
      *st |= MPCT_ST_QP_MAXITER_;
      break;
    }
    if (!S.jinit) gi_load_rinv<MAXM>(S, sJT, sRi, M, row);
    const int p = bid;
    int j0, mp;
    double sgp;
    gi_normal(p, rc, j0, mp, sgp);
    double sp = best;  // slack of p along the path
    double upm = 0.0;  // its multiplier
    bool infeas = false;
    for (;;) {
      ++it;
      const double dk = gi_dvec<MAXM>(sJT, sd, M, j0, mp, sgp, row);
      const double d2 = dk * dk;
      const double dn2 = qsum<MAXM>(d2);
      const double beta = qsum<MAXM>(lane >= S.q ? d2 : 0.0);
      lds_sync();
      const double zm = gi_z(sJT, sd, S.q, M, row);
      PSTAMP(PROF_QD);
      const double rk = gi_backsub<MAXM>(S, sRA, M, dk);
      // dual step over active constraints with r_w > 0
      double t1 = INFINITY;
      int kdrop = 0x7fffffff;
      if (lane < S.q && rk > 0.0) {
        t1 = qp_div(S.uw, rk);
        kdrop = lane;
      }
      qargmin<MAXM>(t1, kdrop, 0);
      PSTAMP(PROF_QR);
      const double t2 = (beta > 1e-14 * dn2) ? -qp_div(sp, beta) : INFINITY;
      if (t1 == INFINITY && t2 == INFINITY) {
        *st |= MPCT_ST_QP_INFEAS_;
        infeas = true;
        break;
      }
      const bool full = t2 <= t1;
      const double t = full ? t2 : t1;
      if (t2 != INFINITY) xm += t * zm;
      if (lane < S.q) S.uw -= t * rk;
      upm += t;
      sp += t * beta;
      if (full) {
        gi_add<MAXM>(S, sJT, sRA, sd, M, p, dk, beta, zm, upm, row, BoxMark{});
        PSTAMP(PROF_QADD);
        break;
      }
      if (kdrop >= S.q) {  // t1 or t2 NaN: no lane attains the ratio test (a non-finite state)
        *st |= MPCT_ST_NONFINITE_;
        infeas = true;
        break;
      }
      gi_drop<MAXM>(S, sJT, sRA, M, kdrop, BoxMark{});
      PSTAMP(PROF_QDROP);
      if (it >= maxit) {
        *st |= MPCT_ST_QP_MAXITER_;
        break;
      }
    }
    if (it >= maxit || infeas) break;
  }
  if (row) sxc[lane] = xm;
  lds_sync();
  return it;
}


}  // namespace mpct
