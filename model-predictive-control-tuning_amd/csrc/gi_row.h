// gi_row.h — the Goldfarb-Idnani primitives of gi_core.h for ONE simulation per 16-lane DPP row:
// four independent QPs (M <= 15 rows each) run side by side in one wavefront.  Same method and the
// same arithmetic order as gi_core.h's M <= 16 class (J-form, Householder add, Givens drop), but
// every quantity that gi_core keeps wave-uniform is row-uniform here: the active-set size q, the
// iteration decisions, the broadcasts (a row's lane k, by ds_bpermute: a row's four lanes read
// their own row) and the reductions (DPP within the row: row_sum / row_argmin, no readlane).  The
// LDS arrays are the row's own (RowQP pointers).  Lane gl = lane & 15 is the QP row index.
#pragma once
#include "gi_core.h"

namespace mpct {

__device__ __forceinline__ int rl_lane() { return (int)threadIdx.x & 15; }
__device__ __forceinline__ int rl_base() { return (int)threadIdx.x & ~15; }

// lane k (row-uniform, dynamic) of this lane's 16-lane row
__device__ __forceinline__ double rbcast(double v, int k) { return __shfl(v, rl_base() + k, 64); }
__device__ __forceinline__ int rbcast_i(int v, int k) { return __shfl(v, rl_base() + k, 64); }

// the row's sum / argmin on every lane of the row (lanes >= M hold 0 / INF: the callers)
__device__ __forceinline__ double rsum(double v) { return row_sum(v); }
__device__ __forceinline__ void rargmin(double& v, int& id) { row_argmin(v, id); }

// the LDS arrays of one row's QP (row-major / column-major as gi_core.h)
struct RowQP {
  double* JT;  // J column-major, JT[k*M + i] = J(i,k)
  double* RA;  // R_A row-major, stride M
  double* d;   // d = J'n
};

template <int MAXM>
__device__ __forceinline__ void gr_load_rinv(GIState<MAXM>& S, const RowQP& Q, const double* sRi, int M, bool row) {
  const int gl = rl_lane();
  if (row)
#pragma unroll 1
    for (int k = 0; k < M; ++k) Q.JT[k * M + gl] = sRi[gl * M + k];
  S.nrot = 0;
  S.jinit = true;
  lds_sync();
}

// d = J'n_p for box constraint rows j0..mp (sign sg): lane k sums column k of J
__device__ __forceinline__ double gr_dvec(const RowQP& Q, int M, int j0, int mp, double sg, bool row) {
  const int gl = rl_lane();
  double dk = 0.0;
  if (row) {
    for (int j = j0; j <= mp; ++j) dk += Q.JT[gl * M + j];
    dk *= sg;
    Q.d[gl] = dk;
  }
  return dk;
}

// z_i = sum_{k >= q} J(i,k) d_k (gi_z's order)
__device__ __forceinline__ double gr_z(const RowQP& Q, int q, int M, bool row) {
  const int gl = rl_lane();
  double z0 = 0.0, z1 = 0.0;
  if (row) {
    int k = q;
    for (; k + 3 < M; k += 4) {
      const double j0 = Q.JT[k * M + gl], j1 = Q.JT[(k + 1) * M + gl];
      const double j2 = Q.JT[(k + 2) * M + gl], j3 = Q.JT[(k + 3) * M + gl];
      const double d0 = Q.d[k], d1 = Q.d[k + 1], d2 = Q.d[k + 2], d3 = Q.d[k + 3];
      z0 += j0 * d0;
      z1 += j1 * d1;
      z0 += j2 * d2;
      z1 += j3 * d3;
    }
    for (; k + 1 < M; k += 2) {
      z0 += Q.JT[k * M + gl] * Q.d[k];
      z1 += Q.JT[(k + 1) * M + gl] * Q.d[k + 1];
    }
    if (k < M) z0 += Q.JT[k * M + gl] * Q.d[k];
  }
  return z0 + z1;
}

// r = R_A^-1 c (c_w in lane w < q), gi_backsub's order
template <int MAXM>
__device__ __forceinline__ double gr_backsub(const GIState<MAXM>& S, const RowQP& Q, int M, double c) {
  const int gl = rl_lane();
  double ck = gl < S.q ? c : 0.0, rk = 0.0;
  const bool in = gl < M;
  double a = in && S.q > 0 ? Q.RA[gl * M + S.q - 1] : 0.0;
  for (int w = S.q - 1; w >= 0; --w) {
    const double an = in && w > 0 ? Q.RA[gl * M + w - 1] : 0.0;
    const double rw = rbcast(ck * S.rdg, w);
    if (gl == w) rk = rw;
    if (gl < w) ck -= a * rw;
    a = an;
  }
  return rk;
}

template <int MAXM, class Mark>
__device__ __forceinline__ void gr_add(GIState<MAXM>& S, const RowQP& Q, int M, int p, double dk, double beta,
                                       double zm, double upm, bool row, const Mark& mark) {
  const int gl = rl_lane();
  const int q = S.q;
  const double dq = rbcast(dk, q);
  const double nrm = beta * rsq_nr(beta);
  const double alpha = dq > 0.0 ? -nrm : nrm;
  const double vq = dq - alpha;
  const double two_vtv = qp_rcp(beta - alpha * dq);
  if (row) {
    const double jq = Q.JT[q * M + gl];
    const double f = (zm - alpha * jq) * two_vtv;
    Q.JT[q * M + gl] = jq - f * vq;
    int k = q + 1;
    for (; k + 3 < M; k += 4) {
      const double j0 = Q.JT[k * M + gl], j1 = Q.JT[(k + 1) * M + gl];
      const double j2 = Q.JT[(k + 2) * M + gl], j3 = Q.JT[(k + 3) * M + gl];
      const double d0 = Q.d[k], d1 = Q.d[k + 1], d2 = Q.d[k + 2], d3 = Q.d[k + 3];
      Q.JT[k * M + gl] = j0 - f * d0;
      Q.JT[(k + 1) * M + gl] = j1 - f * d1;
      Q.JT[(k + 2) * M + gl] = j2 - f * d2;
      Q.JT[(k + 3) * M + gl] = j3 - f * d3;
    }
    for (; k < M; ++k) Q.JT[k * M + gl] -= f * Q.d[k];
  }
  if (gl < q) Q.RA[gl * M + q] = dk;
  const double ia = qp_rcp(alpha);
  if (gl == q) {
    Q.RA[q * M + q] = alpha;
    S.rdg = ia;
    S.uw = upm;
    S.ww = p;
  }
  mark(S, p, true);
  S.q = q + 1;
  S.nrot += 1;
  lds_sync();
}

template <int MAXM, class Mark>
__device__ __forceinline__ void gr_drop(GIState<MAXM>& S, const RowQP& Q, int M, int kd, const Mark& mark) {
  const int gl = rl_lane();
  const int q = S.q;
  const int idk = rbcast_i(S.ww, kd);
  mark(S, idk, false);
  if (gl < q)
    for (int w = kd; w < q - 1; ++w) Q.RA[gl * M + w] = Q.RA[gl * M + w + 1];
  {
    const double un = lane_next<16>(S.uw);
    const int wn = lane_next_i<16>(S.ww);
    if (gl >= kd && gl < q - 1) {
      S.uw = un;
      S.ww = wn;
    }
  }
  lds_sync();
  for (int jj = kd; jj < q - 1; ++jj) {
    const double a = Q.RA[jj * M + jj], b = Q.RA[(jj + 1) * M + jj];
    const double rr = a * a + b * b;
    if (rr != 0.0) {
      const double ri = rsq_nr(rr);
      const double cs = a * ri, sn = b * ri;
      if (gl >= jj && gl < q - 1) {
        const double r0 = Q.RA[jj * M + gl], r1 = Q.RA[(jj + 1) * M + gl];
        Q.RA[jj * M + gl] = cs * r0 + sn * r1;
        Q.RA[(jj + 1) * M + gl] = (gl == jj) ? 0.0 : -sn * r0 + cs * r1;
      }
      if (gl < M) {
        const double j0v = Q.JT[jj * M + gl], j1v = Q.JT[(jj + 1) * M + gl];
        Q.JT[jj * M + gl] = cs * j0v + sn * j1v;
        Q.JT[(jj + 1) * M + gl] = -sn * j0v + cs * j1v;
      }
      S.nrot += 1;
    }
    lds_sync();
  }
  const int qn = q - 1;
  if (gl == qn) {
    S.uw = 0.0;
    S.ww = -1;
  }
  if (gl < qn) S.rdg = qp_rcp(Q.RA[gl * M + gl]);
  S.q = qn;
  lds_sync();
}

// box-constraint active flags of the row's QP row gl (gi_core BoxMark with the row lane)
struct RowBoxMark {
  template <class St>
  __device__ __forceinline__ void operator()(St& S, int p, bool on) const {
    if (rl_lane() == (p >> 2)) {
      if (on) S.act |= 1u << (p & 3);
      else S.act &= ~(1u << (p & 3));
    }
  }
};

}  // namespace mpct
