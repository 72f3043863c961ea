// gi_core.h — Goldfarb-Idnani dual active-set machinery in J-form, shared by the closed-loop
// kernels.  Lanes 0..M-1 are the QP rows (M = QP dimension <= MAXM <= 64).  The constraint
// bookkeeping (which ids are active) is the caller's: gi_add / gi_drop call mark(S, id, on).
#pragma once
#include "wave_ops.h"

namespace mpct {

// QP step lengths and the Householder / Givens scalars are divide-free: v_rcp_f64 / v_rsq_f64 plus
// two Newton steps (about 1 ulp; metric kernel 3.99 -> 3.87 ms, DESIGN.md §6 "Divide-free QP
// scalars", profiles/r02i_qp_fastdiv_ab.txt)
__device__ __forceinline__ double qp_div(double a, double b) { return a * rcp_nr(b); }
__device__ __forceinline__ double qp_rcp(double b) { return rcp_nr(b); }

// constraint p = 4*m + kind on move m = n*Nu + l:
//   kind 0:  du_m >= lo     kind 1: -du_m >= -hi      (l == 0: merged rate/amplitude box)
//   kind 2:  sum_{l'<=l} du_(n,l') >= u_min - u_prev    kind 3: -sum >= -(u_max - u_prev)
struct CInfo {
  int j0, j1;
  double sg;
};
__device__ __forceinline__ CInfo cinfo(int p, int Nu) {
  const int m = p >> 2, kind = p & 3;
  CInfo c;
  c.sg = (kind & 1) ? -1.0 : 1.0;
  c.j0 = kind < 2 ? m : (m / Nu) * Nu;
  c.j1 = m;
  return c;
}

// per-lane constraint data for QP row m (registers)
struct RowCons {
  double dmin, dmax, umin, umax;
  int n, l;
  const double* bnd;  // (gi_qp16<.., true>) the row's MV bounds dmin, dmax, umin, umax in LDS instead
};

// Goldfarb-Idnani dual active-set QP (Goldfarb & Idnani 1983; the toolbox's KWIK is of this
// family) in its factored, numerically stable form.  H = R'R;  J (M x M) with
// H^-1 = J J' starts as R^-1; the active normals N_A satisfy J'N_A = [R_A; 0].
// For the most violated constraint p:  d = J'n_p,  z = J(:,q:) d(q:) (primal direction),
// r = R_A^-1 d(0:q) (dual direction), beta = n_p'z = |d(q:)|^2.  Adding p applies ONE
// Householder reflector to J(:,q:) mapping d(q:) onto alpha e_q (its dot products are
// z - alpha J(:,q), so the add costs one sqrt) and appends [d(0:q); alpha] to R_A; dropping
// constraint k re-triangularises R_A with Givens rotations applied to J's columns.
//
// Warm start across the receding-horizon steps: the constraint normals do not depend on the
// step (only the bounds do), so the factorisation of the previous step's final active set is
// kept (J and R_A in LDS, multipliers and ids in lanes).  Each QP first solves the equality-constrained problem on
// that set from the unconstrained minimiser x_u (x = x_u + J_A w, R_A'w = b_A - N_A'x_u,
// lambda = R_A^-1 w), drops negative multipliers one at a time (x = EQP of the smaller set),
// and then runs ordinary GI iterations from that dual-feasible point: the optimum of a strictly
// convex QP is unique, so the result equals a cold start's up to rounding.  J is rebuilt from
// R^-1 (re-adding the set) after kGiRebuild* x M rotations (gpc_qp.h: 128 M in the M <= 16
// class, 32 M for its DTC instances, 8 M above), which bounds the orthogonality drift of the rotated J.  Without a rebuild
// the metric grid drifted to 3.5e-5 relative; the 7.5e-10 bound was measured at the original
// 4 M interval (C prototype).  At 32 M the metric grid's J1 still equals the C
// port to 3.2e-9 (the same figure as at 4 M and 8 M); the wider classes keep 8 M.
template <int MAXM>
struct GIState {
  double rdg;       // 1 / R_A(lane, lane)
  double uw;        // multiplier of active constraint `lane`
  int ww;           // id (4*m + kind) of active constraint `lane`
  unsigned act;     // active bits of this lane's 4 constraints (row m = lane)
  int q;            // active-set size (wave-uniform)
  int nrot;         // rotations applied to J since it was last built from R^-1 (uniform)
  bool jinit;       // J holds a factorisation consistent with the active set (uniform)
#ifdef MPCT_DIAG
  int diag = 0;     // planted faults of the diagnostic build (DevOpts::diag)
#endif
};

template <int MAXM>
__device__ __forceinline__ void gi_reset(GIState<MAXM>& S) {
  S.rdg = 0.0;
  S.uw = 0.0;
  S.ww = -1;
  S.act = 0;
  S.q = 0;
  S.nrot = 0;
  S.jinit = false;
}

template <int MAXM>
__device__ __forceinline__ void gi_load_rinv(GIState<MAXM>& S, double* sJT, const double* sRi, int M,
                                             bool row) {
  const int lane = qp_lane();
  // not unrolled: the x8 unroll hoists eight strided LDS pointers, the one VGPR over the 3-wave
  // budget of gpc_closed_loop_kernel<16>, spilled to scratch (~1 MiB of write-backs per metric
  // launch); the rebuild runs once per 32 updates so the loop overhead is noise
  if (row)
#pragma unroll 1
    for (int k = 0; k < M; ++k) sJT[k * M + lane] = sRi[lane * M + k];
  S.nrot = 0;
  S.jinit = true;
  lds_sync();
}

// d = J'n_p = sg * (sum of J's rows j0..mp): lane k sums column k of J (contiguous in JT); d -> sd
template <int MAXM>
__device__ __forceinline__ double gi_dvec(const double* sJT, double* sd, int M, int j0, int mp, double sg,
                                          bool row) {
  const int lane = qp_lane();
  double dk = 0.0;
  if (row) {
    for (int j = j0; j <= mp; ++j) dk += sJT[lane * M + j];
    dk *= sg;
    sd[lane] = dk;
  }
  return dk;
}

// z_i = sum_{k >= q} J(i,k) d_k  (d in sd, synchronised by the caller)
__device__ __forceinline__ double gi_z(const double* sJT, const double* sd, int q, int M, bool row) {
  const int lane = qp_lane();
  double z0 = 0.0, z1 = 0.0;
  if (row) {
    int k = q;
    for (; k + 3 < M; k += 4) {  // four terms' loads together, the two-term loop's order
      const double j0 = sJT[k * M + lane], j1 = sJT[(k + 1) * M + lane];
      const double j2 = sJT[(k + 2) * M + lane], j3 = sJT[(k + 3) * M + lane];
      const double d0 = sd[k], d1 = sd[k + 1], d2 = sd[k + 2], d3 = sd[k + 3];
      z0 += j0 * d0;
      z1 += j1 * d1;
      z0 += j2 * d2;
      z1 += j3 * d3;
    }
    for (; k + 1 < M; k += 2) {
      z0 += sJT[k * M + lane] * sd[k];
      z1 += sJT[(k + 1) * M + lane] * sd[k + 1];
    }
    if (k < M) z0 += sJT[k * M + lane] * sd[k];
  }
  return z0 + z1;
}

// R_A's place in LDS.  RAFull: row-major, row stride M (M x M).  RAPacked: column-major upper
// Hessenberg, column j holding rows 0..j+1 (the drop's shifted columns carry one subdiagonal entry
// until its Givens rotation clears it), M (M + 3) / 2 doubles: the band kernel's R_A at Mz = 46 is
// 8.6 KB smaller, which moves its heaviest simulations to a denser LDS tier.  Same arithmetic in
// both layouts; every index either layout forms stays inside its array.
struct RAFull {
  int M;
  static constexpr bool packed = false;
  static constexpr bool store = true;
  __device__ __forceinline__ int operator()(int i, int j) const { return i * M + j; }
};
struct RAPacked {
  static constexpr bool packed = true;
  static constexpr bool store = true;
  // 24-bit multiply (full rate; v_mul_lo_u32 is quarter rate): j <= 64
  __device__ __forceinline__ int operator()(int i, int j) const {
    return (int)(__umul24((unsigned)j, (unsigned)(j + 3)) >> 1) + i;
  }
};
__host__ __device__ constexpr int ra_packed_size(int M) { return (M * (M + 3)) / 2; }
// no R_A at all: the caller keeps B = R_A^-1 instead (the band kernel's widest class, which drops
// constraints with rotations derived from B); gi_add then writes no R_A entry
struct RANone {
  static constexpr bool packed = true;
  static constexpr bool store = false;
  __device__ __forceinline__ int operator()(int, int) const { return 0; }
};

// r = R_A^-1 c  (c_w in lane w < q): column back substitution, lane w ends with r_w
template <int MAXM, class RAL>
__device__ __forceinline__ double gi_backsub(const GIState<MAXM>& S, const double* sRA, int M, double c,
                                             const RAL& ra) {
  const int lane = qp_lane();
  double ck = lane < S.q ? c : 0.0, rk = 0.0;
  // R_A(lane, w) is loaded one step ahead, off the chain of broadcasts (LDS latency was exposed at
  // every step: config 3's q ~ 40 active sets)
  const bool in = lane < M;
  double a = in && S.q > 0 ? sRA[ra(lane, S.q - 1)] : 0.0;
  for (int w = S.q - 1; w >= 0; --w) {
    const double an = in && w > 0 ? sRA[ra(lane, w - 1)] : 0.0;
    const double rw = bcast(ck * S.rdg, w);
    if (lane == w) rk = rw;
    if (lane < w) ck -= a * rw;
    a = an;
  }
  return rk;
}
template <int MAXM>
__device__ __forceinline__ double gi_backsub(const GIState<MAXM>& S, const double* sRA, int M, double c) {
  return gi_backsub<MAXM>(S, sRA, M, c, RAFull{M});
}

// an extra factor a caller keeps in step with the active set (the band kernel's B = R_A^-1):
// gi_add calls add(q, 1 / alpha) for the new column q before the lds_sync that ends the add
struct GINoExt {
  __device__ __forceinline__ void add(int, double) const {}
};

// append constraint p (normal image d = J'n_p in dk / sd, beta = |d(q:)|^2, z = J(:,q:)d(q:))
template <int MAXM, class Mark, class RAL, class Ext = GINoExt>
__device__ __forceinline__ void gi_add(GIState<MAXM>& S, double* sJT, double* sRA, const double* sd, int M,
                                       int p, double dk, double beta, double zm, double upm, bool row,
                                       const Mark& mark, const RAL& ra, const Ext& ext = Ext{}) {
  const int lane = qp_lane();
  const int q = S.q;
  const double dq = bcast(dk, q);
  const double nrm = beta * rsq_nr(beta);  // beta > 0 on an add
  const double alpha = dq > 0.0 ? -nrm : nrm;
  const double vq = dq - alpha;
  const double two_vtv = qp_rcp(beta - alpha * dq);  // 2 / v'v
  if (row) {
    const double jq = sJT[q * M + lane];
    const double f = (zm - alpha * jq) * two_vtv;
    sJT[q * M + lane] = jq - f * vq;
    int k = q + 1;
    for (; k + 3 < M; k += 4) {  // independent columns: four loads in flight
      const double j0 = sJT[k * M + lane], j1 = sJT[(k + 1) * M + lane];
      const double j2 = sJT[(k + 2) * M + lane], j3 = sJT[(k + 3) * M + lane];
      const double d0 = sd[k], d1 = sd[k + 1], d2 = sd[k + 2], d3 = sd[k + 3];
      sJT[k * M + lane] = j0 - f * d0;
      sJT[(k + 1) * M + lane] = j1 - f * d1;
      sJT[(k + 2) * M + lane] = j2 - f * d2;
      sJT[(k + 3) * M + lane] = j3 - f * d3;
    }
    for (; k < M; ++k) sJT[k * M + lane] -= f * sd[k];
  }
  if constexpr (RAL::store) {
    if (lane < q) sRA[ra(lane, q)] = dk;  // new column q of R_A = [d(0:q-1); alpha]
  }
  const double ia = qp_rcp(alpha);
  if (lane == q) {
    if constexpr (RAL::store) sRA[ra(q, q)] = alpha;
    S.rdg = ia;
    S.uw = upm;
    S.ww = p;
  }
  ext.add(q, ia);
  mark(S, p, true);
  S.q = q + 1;
  S.nrot += 1;
  lds_sync();
}
template <int MAXM, class Mark>
__device__ __forceinline__ void gi_add(GIState<MAXM>& S, double* sJT, double* sRA, const double* sd, int M,
                                       int p, double dk, double beta, double zm, double upm, bool row,
                                       const Mark& mark) {
  gi_add<MAXM>(S, sJT, sRA, sd, M, p, dk, beta, zm, upm, row, mark, RAFull{M});
}

// remove active constraint kd: drop its column of R_A, re-triangularise with Givens on J
template <int MAXM, class Mark, class RAL>
__device__ __forceinline__ void gi_drop(GIState<MAXM>& S, double* sJT, double* sRA, int M, int kd,
                                        const Mark& mark, const RAL& ra) {
  const int lane = qp_lane();
  const int q = S.q;
  const int idk = __builtin_amdgcn_readlane(S.ww, kd);
  mark(S, idk, false);
  if (lane < q) {  // remove column kd (lanes = rows; rows below w + 1 of the new column w are
                   // never read, and the packed column w holds no more)
    for (int w = kd; w < q - 1; ++w)
      if (!RAL::packed || lane <= w + 1) sRA[ra(lane, w)] = sRA[ra(lane, w + 1)];
  }
  {
    const double un = lane_next<MAXM>(S.uw);
    const int wn = lane_next_i<MAXM>(S.ww);
    if (lane >= kd && lane < q - 1) {
      S.uw = un;
      S.ww = wn;
    }
  }
  lds_sync();
  // R_A is upper Hessenberg in columns kd..q-2: Givens on rows (jj, jj+1), lanes = columns
  for (int jj = kd; jj < q - 1; ++jj) {
    {
      const double a = sRA[ra(jj, jj)], b = sRA[ra(jj + 1, jj)];
      const double rr = a * a + b * b;
      if (rr != 0.0) {
        const double ri = rsq_nr(rr);
        const double cs = a * ri, sn = b * ri;
        if (lane >= jj && lane < q - 1) {
          const double r0 = sRA[ra(jj, lane)], r1 = sRA[ra(jj + 1, lane)];
          sRA[ra(jj, lane)] = cs * r0 + sn * r1;
          sRA[ra(jj + 1, lane)] = (lane == jj) ? 0.0 : -sn * r0 + cs * r1;
        }
        if (lane < M) {
          const double j0v = sJT[jj * M + lane], j1v = sJT[(jj + 1) * M + lane];
          sJT[jj * M + lane] = cs * j0v + sn * j1v;
          sJT[(jj + 1) * M + lane] = -sn * j0v + cs * j1v;
        }
        S.nrot += 1;
      }
      lds_sync();
    }
  }
  const int qn = q - 1;
  if (lane == qn) {
    S.uw = 0.0;
    S.ww = -1;
  }
  if (lane < qn) S.rdg = qp_rcp(sRA[ra(lane, lane)]);
  S.q = qn;
  lds_sync();
}
template <int MAXM, class Mark>
__device__ __forceinline__ void gi_drop(GIState<MAXM>& S, double* sJT, double* sRA, int M, int kd,
                                        const Mark& mark) {
  gi_drop<MAXM>(S, sJT, sRA, M, kd, mark, RAFull{M});
}


// active-flag bookkeeping of the box constraints p = 4m + kind: bit kind of lane m
struct BoxMark {
  template <class St>
  __device__ __forceinline__ void operator()(St& S, int p, bool on) const {
    if ((int)threadIdx.x == (p >> 2)) {
      if (on) S.act |= 1u << (p & 3);
      else S.act &= ~(1u << (p & 3));
    }
  }
};

}  // namespace mpct
