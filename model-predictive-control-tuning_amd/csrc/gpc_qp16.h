// gpc_qp16.h — the per-step QP of the M <= 16 class of gpc_closed_loop_kernel with its factors in
// VGPRs across all 64 lanes (no LDS round trip on the Goldfarb-Idnani iteration's chain).
//
// Same method as gpc_qp.h / gi_core.h (dual active set in J-form, warm-started across steps,
// DESIGN.md §4-5), different data layout.  Lane l = i + 16 b (i = l & 15, b = l >> 4):
//   * QP-row quantities ("row vectors": x, slacks, multipliers, constraint ids, active flags) are
//     replicated: lane (i, b) holds entry i for every b, so the four 16-lane DPP rows compute the
//     same thing and no broadcast is ever needed between them;
//   * J (H^-1 = J J', 16 x 16) is held 4 entries per lane: lane (i, b) has J(i, 4b + r), r = 0..3
//     ("RB"); B = R_A^-1 (explicit, upper triangular on the active block) is in LDS with row
//     stride 16, so lane (i, b) reads its B(i, 4b..4b+3) with two 16-byte loads that do not depend
//     on the iteration's d and issue under d's DPP reduction;
//   * "column vectors" (d = J'n_p, w = B'c) come out of a 16-lane DPP reduction with entry 4b + r
//     in register r of every lane of row b.
// So y = X v (v a column vector) is 4 FMAs + one v_permlane16/32_swap reduction over b, and
// y = X'v (v a row vector) is 4 multiplies + one DPP reduction within the 16-lane rows.  Per
// iteration: d = J'n_p (DPP), then z = J(:,q:)d(q:), J(i,q), r = B d(0:q) and |d|^2, |d(q:)|^2 (one
// permlane reduction each, independent), the ratio test, and the add (Householder on J's
// registers, B's new column) or the drop.  R_A stays in LDS: only the drop's Givens chain reads it,
// and B's column rotations ride on that chain's LDS round trips.  The triangular solves of gi_qp
// (the warm start's R_A'w = c, lambda = R_A^-1 w, the dual direction r = R_A^-1 d) become products
// with B.  J and B in VGPRs both measured 190 VGPRs: the two
// waves per SIMD that allows lost more at 4096 candidates than the shorter chain won.
#pragma once
#include "gi_core.h"

namespace mpct {

// four doubles of one lane.  Every element access uses a compile-time index (FOR4 expands its body
// four times with a constexpr r), so SROA turns the arrays into registers before any other pass
// runs: a #pragma unroll loop left a variable index for InstCombine to fold the uniform-index
// selects into a dynamically indexed scratch load, and an ext_vector_type copied all 8 VGPRs of
// the vector at every branch merge
typedef double d4v[4];
#define FOR4(r, ...)             \
  do {                           \
    { constexpr int r = 0; __VA_ARGS__ } \
    { constexpr int r = 1; __VA_ARGS__ } \
    { constexpr int r = 2; __VA_ARGS__ } \
    { constexpr int r = 3; __VA_ARGS__ } \
  } while (0)

// J of one simulation (RB layout) and B = R_A^-1 in LDS (row-major, stride 16)
struct RegFactors {
  d4v J;
  double* sB;
};
// B's row stride.  Stride 16 has the column writes of an add 16-way, the drop's column reads 8-way
// and b_row4's row reads 4-way in LDS bank conflict (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
// 18.6 %); stride 18 halves that (13.7 %) but measured no faster, 1-2 % slower at 1024 and 8192
// candidates (profiles/r03n_bs_stride_ab.txt): the conflicts are not on the chain.  Round 6 rotated each
// row's 4-double blocks by (i >> 1) & 3 instead, and A's row reads in gpc_small.hip: conflicts 19.4 ->
// 7.4 % of LDS cycles, kernel 3-4 % slower (the index arithmetic sits on the QP chain; the A rotation
// alone was within noise), profiles/r06m_lds_banks_ab.txt
constexpr int kBS = 16;

// Drops keep R_A and its Givens chain: drops derived from B alone, as the band kernel's (DESIGN §11
// round 5), measured the same at 4096 candidates and 1 % slower on the heaviest 256 here (DESIGN §6
// round 5): the metric's drops average three rotations, and J's register rotations dominate them.
// Round 6 (profiles/r06a_drop_ab.txt): the column / row shifts as one parallel pass of the wave
// (all loads, then all stores) and the Givens chain with R_A's row and B's column carried in
// registers, (a, c) by readlane and no hand-off per rotation, were 3-12 % slower at 4096 candidates
// and on the heaviest 256: both add live values to a step loop at the 128-VGPR budget, whose
// allocator answers with 2-5 more step-loop invariants spilled and reloaded every step.  The same
// R_A(jj, jj) by readlane alone (loaded one rotation ahead otherwise) was 1-4 % slower as well,
// with or without the bounds in LDS (profiles/r06c_metric_ab.txt).  Once the bounds in LDS freed
// nine VGPRs, the chain without per-rotation hand-offs (fence only), with R_A(jj, jj) by readlane,
// and with R_A's row and B's column carried in registers fit without a spill, and none was faster
// (bitwise equal, within 1 % either way, profiles/r06f_drop_chain_ab.txt): the heaviest
// simulations' drops are not on a chain the hand-offs lengthen

// the lane id as an opaque value, re-derived at every use: the step loop's register budget cannot
// hold the dozens of lane-derived addresses and predicates the compiler would otherwise hoist out
// of it (three waves per SIMD = 168 VGPRs)
__device__ __forceinline__ int qlane() {
  int l = threadIdx.x;
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ int q16_i() { return qlane() & 15; }
__device__ __forceinline__ int q16_b() { return qlane() >> 4; }

// entry r (wave-uniform) of a lane's 4 registers.  The four values are passed by value: a
// selection between loads through a reference would be folded (in the callee, before inlining)
// into one load at a variable offset, which pins the caller's array to scratch
__device__ __forceinline__ double sel4u_v(double x0, double x1, double x2, double x3, int r) {
  double v = x0;
  if (r == 1) v = x1;
  if (r == 2) v = x2;
  if (r == 3) v = x3;
  return v;
}
#define sel4u(x, r) sel4u_v((x)[0], (x)[1], (x)[2], (x)[3], (r))
// entry r (per lane, 0..3) of a lane's 4 registers
__device__ __forceinline__ double sel4v_v(double x0, double x1, double x2, double x3, int r) {
  const double lo = (r & 1) ? x1 : x0;
  const double hi = (r & 1) ? x3 : x2;
  return (r & 2) ? hi : lo;
}
#define sel4v(x, r) sel4v_v((x)[0], (x)[1], (x)[2], (x)[3], (r))

// all-reduce of four values within every 16-lane row (four independent DPP chains)
__device__ __forceinline__ void row16_sum4(d4v& t) {
  FOR4(r, t[r] += dppd<kQx1>(t[r]););
  FOR4(r, t[r] += dppd<kQx2>(t[r]););
  FOR4(r, t[r] += dppd<kHalfMirror>(t[r]););
  FOR4(r, t[r] += dppd<kMirror>(t[r]););
}

// column vector entry k (wave-uniform) as a scalar: register k & 3 of row k >> 2
__device__ __forceinline__ double cvec_at(const d4v& c, int k) {
  return bcast(sel4u(c, k & 3), (k >> 2) * 16);
}

// B(i, 4b..4b+3) of lane (i, b)
__device__ __forceinline__ void b_row4(const double* sB, d4v& x) {
  const double2* p = reinterpret_cast<const double2*>(sB + q16_i() * kBS + 4 * q16_b());
  const double2 u = p[0], v = p[1];
  x[0] = u.x;
  x[1] = u.y;
  x[2] = v.x;
  x[3] = v.y;
}

// lane (i, b) receives lane (i, b + 1) / (i, b - 1): the rare Givens rotation across a register
// block boundary (columns 4b + 3 and 4b + 4)
__device__ __forceinline__ double rows_down(double v) { return __shfl(v, qlane() + 16, 64); }
__device__ __forceinline__ double rows_up(double v) { return __shfl(v, qlane() - 16, 64); }

// columns (jj, jj + 1) of J <- (c x_jj + s x_jj+1, -s x_jj + c x_jj+1).  jj is wave-uniform: a
// scalar switch picks the register pair (a branch-free form with selects on every register took 9
// more VGPRs)
__device__ __forceinline__ void rot_pair(double& a, double& c, bool on, double cs, double sn) {
  if (on) {
    const double a0 = a, c0 = c;
    a = cs * a0 + sn * c0;
    c = -sn * a0 + cs * c0;
  }
}
__device__ __forceinline__ void rb_rotate_cols(d4v& x, int jj, double cs, double sn) {
  const int b = q16_b(), b0 = jj >> 2;
  const bool on = b == b0;
  switch (jj & 3) {
    case 0: {
      double a = x[0], c = x[1];
      rot_pair(a, c, on, cs, sn);
      x[0] = a;
      x[1] = c;
      break;
    }
    case 1: {
      double a = x[1], c = x[2];
      rot_pair(a, c, on, cs, sn);
      x[1] = a;
      x[2] = c;
      break;
    }
    case 2: {
      double a = x[2], c = x[3];
      rot_pair(a, c, on, cs, sn);
      x[2] = a;
      x[3] = c;
      break;
    }
    default: {  // columns 4 b0 + 3 and 4 (b0 + 1): across two register blocks
      const double nx0 = rows_down(x[0]), pv3 = rows_up(x[3]);
      if (on) x[3] = cs * x[3] + sn * nx0;
      if (b == b0 + 1) x[0] = -sn * pv3 + cs * x[0];
      break;
    }
  }
}

// box-constraint active flags on the replicated rows: bit kind of row m = p >> 2
struct BoxMark16 {
  template <class St>
  __device__ __forceinline__ void operator()(St& S, int p, bool on) const {
    if (q16_i() == (p >> 2)) {
      if (on) S.act |= 1u << (p & 3);
      else S.act &= ~(1u << (p & 3));
    }
  }
};

// entry (i, k), k >= i, of the upper-triangular R^-1 in LDS: row-major M x M, or (PACKED) its
// upper triangle row by row (M (M + 1) / 2 doubles)
template <bool PACKED>
__device__ __forceinline__ int rinv_idx(int i, int k, int M) {
  return PACKED ? i * M - ((i * (i - 1)) >> 1) + (k - i) : i * M + k;
}

// J <- R^-1 (upper, in LDS), B <- 0 (rows i < M: B has M rows of stride kBS; lanes i >= M only
// ever read their own rows, whose products no QP row uses)
template <bool PACKED>
__device__ __forceinline__ void gi16_load_rinv(GIState<16>& S, RegFactors& F, const double* sRi, int M) {
  const int i = q16_i(), b = q16_b();
  FOR4(r, {
    const int k = 4 * b + r;
    F.J[r] = (i < M && k < M && k >= i) ? sRi[rinv_idx<PACKED>(i, k, M)] : 0.0;
  });
  if (i < M) {
    double2* p = reinterpret_cast<double2*>(F.sB + i * kBS + 4 * b);
    p[0] = make_double2(0.0, 0.0);
    p[1] = make_double2(0.0, 0.0);
  }
  S.nrot = 0;
  S.jinit = true;
}

// d = J'n_p for constraint p (rows j0..mp of J, sign sg) -> column vector.  A one-row normal (the
// rate rows, kinds 0/1) is row j0 of J itself: fetched by ds_bpermute (8 instructions) instead of
// the 16-lane sum of the masked rows (48), the same value
__device__ __forceinline__ void gi16_dvec(const RegFactors& F, int j0, int mp, double sg, d4v& d) {
  const int i = q16_i();
  if (j0 == mp) {
    const int src = j0 + 16 * q16_b();
    FOR4(r, d[r] = __shfl(F.J[r], src, kWave););
  } else {
    const bool in = i >= j0 && i <= mp;
    FOR4(r, d[r] = in ? F.J[r] : 0.0;);
    row16_sum4(d);
  }
  FOR4(r, d[r] *= sg;);
}

// the products an iteration needs from d (column vector), q = active-set size, Bl = the lane's
// B(i, 4b..4b+3):  z = J(:,q:)d(q:), jq = J(:,q), rk = B d(0:q) (row vectors), dn2 = |d|^2,
// beta = |d(q:)|^2
__device__ __forceinline__ void gi16_products(const RegFactors& F, const d4v& Bl, const d4v& d, int q,
                                              double& z, double& jq, double& rk, double& dn2, double& beta) {
  const int b = q16_b();
  double za = 0.0, ra = 0.0, s1 = 0.0, s2 = 0.0;
  FOR4(r, {
    const bool tail = 4 * b + r >= q;
    const double d2 = d[r] * d[r];
    s1 += d2;
    if (tail) {
      za = fma(F.J[r], d[r], za);
      s2 += d2;
    } else {
      ra = fma(Bl[r], d[r], ra);
    }
  });
  const double jl = (b == (q >> 2)) ? sel4u(F.J, q & 3) : 0.0;
  z = za;
  jq = jl;
  rk = ra;
  dn2 = s1;
  row4_sum4(z, jq, rk, dn2);  // bitwise the four row4_sums, 21 instructions instead of 40
  beta = row4_sum(s2);
}

// append constraint p: Householder on J(:,q:) mapping d(q:) to alpha e_q, B's column q and R_A's
// column q (LDS), the multiplier upm and the id
template <class Mark>
__device__ __forceinline__ void gi16_add(GIState<16>& S, RegFactors& F, double* sRA, int M, int p,
                                         const d4v& d, double beta, double z, double jq, double rk,
                                         double upm, const Mark& mark) {
  const int lane = qlane(), i = lane & 15, b = lane >> 4;
  const int q = S.q;
  const double dq = cvec_at(d, q);
  const double nrm = beta * rsq_nr(beta);  // beta > 0 on an add
  const double alpha = dq > 0.0 ? -nrm : nrm;
  const double vq = dq - alpha;
  const double two_vtv = qp_rcp(beta - alpha * dq);  // 2 / v'v
  const double f = (z - alpha * jq) * two_vtv;
  const double ia = qp_rcp(alpha);
  FOR4(r, {
    const int k = 4 * b + r;
    if (k >= q) F.J[r] = fma(-f, k == q ? vq : d[r], F.J[r]);
  });
  // B: column q = (-r / alpha; 1 / alpha), row q zero left of the diagonal (lanes = rows / columns)
  if (lane <= q) F.sB[lane * kBS + q] = lane < q ? -rk * ia : ia;
  if (lane < q) F.sB[q * kBS + lane] = 0.0;
  // R_A(w, q) = d_w (w < q), R_A(q, q) = alpha: lanes (i < 4, b) write entry 4b + i
  {
    const int w = 4 * b + i;
    if (i < 4 && w < q) sRA[w * M + q] = sel4v(d, i);
    if (lane == 0) sRA[q * M + q] = alpha;
  }
  if (i == q) {
    S.uw = upm;
    S.ww = p;
  }
  mark(S, p, true);
  S.q = q + 1;
  S.nrot += 1;
  lds_sync();  // B and R_A columns before the next read (ordering them only measured the same)
}

// remove active constraint kd: R_A loses column kd and is re-triangularised by Givens rotations
// (LDS, lanes = columns), applied to J's columns in registers and to B's columns in LDS (lanes =
// rows); B then loses row kd
template <class Mark>
__device__ __forceinline__ void gi16_drop(GIState<16>& S, RegFactors& F, double* sRA, int M, int kd,
                                          const Mark& mark) {
  const int lane = qlane(), i = lane & 15;
  const int q = S.q;
  double* sB = F.sB;
  const int idk = __builtin_amdgcn_readlane(S.ww, kd);
  mark(S, idk, false);
  lds_sync();  // R_A and B columns written by the adds
  // R_A loses column kd (lanes = rows) and B loses row kd (lanes = columns) in one loop, before the
  // rotations: removing a row of B commutes with rotating its columns (B G' minus row kd), so the
  // two serial shift chains run side by side instead of one after the other (round 6: 0.5 % on the
  // metric alone, 1.7 % with the bounds in LDS; bitwise the same; profiles/r06c_metric_ab.txt)
  if (lane < q) {
    for (int w = kd; w < q - 1; ++w) {
      sRA[lane * M + w] = sRA[lane * M + w + 1];
      sB[w * kBS + lane] = sB[(w + 1) * kBS + lane];
    }
  }
  {
    const double un = lane_next<16>(S.uw);
    const int wn = lane_next_i<16>(S.ww);
    if (i >= kd && i < q - 1) {
      S.uw = un;
      S.ww = wn;
    }
  }
  lds_sync();
#pragma nounroll
  for (int jj = kd; jj < q - 1; ++jj) {
    const double a = sRA[jj * M + jj], c = sRA[(jj + 1) * M + jj];
    const double rr = a * a + c * c;
    if (rr != 0.0) {
      const double ri = rsq_nr(rr);
      const double cs = a * ri, sn = c * ri;
      if (lane >= jj && lane < q - 1) {
        const double r0 = sRA[jj * M + lane], r1 = sRA[(jj + 1) * M + lane];
        sRA[jj * M + lane] = cs * r0 + sn * r1;
        sRA[(jj + 1) * M + lane] = (lane == jj) ? 0.0 : -sn * r0 + cs * r1;
      }
      if (lane < q) {  // B G': columns jj, jj + 1 (lanes = rows; row q - 1 is stale after the shift, unused)
        const double b0 = sB[lane * kBS + jj], b1 = sB[lane * kBS + jj + 1];
        sB[lane * kBS + jj] = cs * b0 + sn * b1;
        sB[lane * kBS + jj + 1] = -sn * b0 + cs * b1;
      }
      rb_rotate_cols(F.J, jj, cs, sn);
      S.nrot += 1;
    }
    lds_sync();
  }
  const int qn = q - 1;
  if (i == qn) {
    S.uw = 0.0;
    S.ww = -1;
  }
  S.q = qn;
  lds_sync();
}

// the QP of one step (M <= 16): unconstrained minimiser xu (row vector), u(t-1) of the row's MV
// up_row, the row's constraint data rc (both replicated over the four row blocks); the optimal
// moves come back in xout (row vector, registers; xu itself when it is feasible).  rebuild: the
// J rebuild interval in units of M rotations (gpc_qp.h); PACKED: R^-1's layout (rinv_idx)
template <bool PACKED = false, class PAcc = void, bool BLDS = false>
__device__ __forceinline__ int gi_qp16(const double* sRi, double* sRA, int M, int Nu,
                                       const RowCons& rc, double up_row, double xu, double tol, int maxit,
                                       int* st, GIState<16>& S, RegFactors& F, int rebuild, double& xout
#ifdef MPCT_PROFILE
                                       , PAcc& pacc, unsigned long long& pprev
#endif
                                       ) {
  const int lane = qlane(), i = lane & 15;
  const bool row = i < M;
  if (!row) up_row = 0.0;
  const int rl = rc.l;
  // BLDS (gpc_small_kernel): the row's bounds are read from LDS where a check needs them (the two
  // 16-byte loads issue under the block prefix's DPP chain) instead of living in eight VGPRs
  // across the whole step loop: the kernel's last VGPR spills go (2 -> 0, no scratch), and with
  // the merged drop shifts the metric is 1.7 % faster (profiles/r06c_metric_ab.txt)
  double lo_box = 0.0, hi_box = 0.0;
  if constexpr (!BLDS) {
    lo_box = fmax(rc.dmin, rc.umin - up_row);
    hi_box = fmin(rc.dmax, rc.umax - up_row);
  }
  auto slacks = [&](double x, double s[4]) {
    double dmin, dmax, umin, umax, lo, hi;
    if constexpr (BLDS) {
      const double2 a = reinterpret_cast<const double2*>(rc.bnd)[0], b = reinterpret_cast<const double2*>(rc.bnd)[1];
      dmin = a.x;
      dmax = a.y;
      umin = b.x;
      umax = b.y;
      lo = fmax(dmin, umin - up_row);
      hi = fmin(dmax, umax - up_row);
    } else {
      dmin = rc.dmin;
      dmax = rc.dmax;
      umin = rc.umin;
      umax = rc.umax;
      lo = lo_box;
      hi = hi_box;
    }
    const double pre = block_prefix<16>(x, rl, Nu, row, nullptr);
    if (rl == 0) {
      s[0] = x - lo;
      s[1] = hi - x;
      s[2] = INFINITY;
      s[3] = INFINITY;
    } else {
      s[0] = x - dmin;
      s[1] = dmax - x;
      s[2] = pre - (umin - up_row);
      s[3] = (umax - up_row) - pre;
    }
    if (!row) s[0] = s[1] = s[2] = s[3] = INFINITY;
  };
  const BoxMark16 mark{};
  auto add = [&](int p, const d4v& d, double beta, double z, double jq, double rk, double upm)
                 __attribute__((always_inline)) { gi16_add(S, F, sRA, M, p, d, beta, z, jq, rk, upm, mark); };
  int it = 0;
  double xm = xu;
  PSTAMP(PROF_QCHECK);
  {
    double s[4];
    slacks(xu, s);
    const double smin = fmin(fmin(s[0], s[1]), fmin(s[2], s[3]));
    if (__ballot(smin < -tol) == 0) {  // x_u is feasible: optimal (the retained set is kept)
      xout = xu;
      return 0;
    }
    PSTAMP(PROF_QWENTRY);
    if (S.q == 0) {
      S.jinit = false;  // nothing retained: restart from R^-1 when the first constraint enters
    } else {
      if (!S.jinit || S.nrot >= rebuild * M) {
        // rebuild J and B for the retained set from R^-1, re-adding it in order
        const int qq = S.q;
#ifdef MPCT_PROFILE
        pacc[PROF_QWREADD] += (unsigned long long)qq * kProfCount;
#endif
        gi16_load_rinv<PACKED>(S, F, sRi, M);
        S.q = 0;
        for (int v = 0; v < qq; ++v) {
          const int p = __builtin_amdgcn_readlane(S.ww, v);
          int j0, mp;
          double sg;
          gi_normal(p, rc, j0, mp, sg);
          d4v Bl, d;
          lds_sync();
          b_row4(F.sB, Bl);
          gi16_dvec(F, j0, mp, sg, d);
          double z, jq, rk, dn2, beta;
          gi16_products(F, Bl, d, v, z, jq, rk, dn2, beta);
          const double uk = S.uw;
          add(p, d, beta, z, jq, rk, 0.0);
          if (i == v) S.uw = uk;
          ++it;
        }
        S.nrot = 0;
      }
      PSTAMP(PROF_QWREB);
      lds_sync();
      // equality-constrained solve on the retained set, dropping negative multipliers:
      // w = R_A^-T c = B'c, x = x_u + J(:,0:q) w, lambda = R_A^-1 w = B w.
      // c = b_A - N_A'x_u: lane w < q gathers the slack at x_u of its constraint ww = 4 m + kind
      // from QP row m (ds_bpermute; no LDS buffer), once: a drop shifts c with the ids
      double c;
      {
        const int src = (S.ww >= 0 ? S.ww >> 2 : 0) + 16 * q16_b();
        const double g0 = __shfl(s[0], src, kWave), g1 = __shfl(s[1], src, kWave);
        const double g2 = __shfl(s[2], src, kWave), g3 = __shfl(s[3], src, kWave);
        c = i < S.q ? -sel4v_v(g0, g1, g2, g3, S.ww & 3) : 0.0;
      }
      PSTAMP(PROF_QWGATH);
      for (;;) {
        const int q = S.q;
        if (q == 0) {
          xm = xu;
          break;
        }
        d4v Bl, w;
        b_row4(F.sB, Bl);
        FOR4(r, w[r] = i < q ? Bl[r] * c : 0.0;);
        row16_sum4(w);
        const int b = q16_b();
        double xa = 0.0, la = 0.0;
        FOR4(r, {
          if (4 * b + r < q) {
            xa = fma(F.J[r], w[r], xa);
            la = fma(Bl[r], w[r], la);
          }
        });
        row4_sum2(xa, la);
        xm = xu + xa;
        const double lam = la;
        if (i < q) S.uw = lam;
        double lmin = i < q ? lam : INFINITY;
        int kd = i;
        qargmin<16>(lmin, kd, 0);
        PSTAMP(PROF_QWSOLVE);
        if (!(lmin < 0.0)) break;
#ifdef MPCT_PROFILE
        pacc[PROF_QWROT] += (unsigned long long)(S.q - 1 - kd) * kProfCount;
#endif
#ifdef MPCT_DIAG
        if (!(S.diag & kDiagSkipWarmDrop))
#endif
        {
          gi16_drop(S, F, sRA, M, kd, mark);
          {  // c follows the ids: entries kd + 1 .. q - 1 move down one lane
            const double cn = lane_next<16>(c);
            if (i >= kd && i < q - 1) c = cn;
            else if (i == q - 1) c = 0.0;
          }
        }
        PSTAMP(PROF_QWDROP);
        // every drop shrinks the set, so the loop ends within q passes; the cap turns a logic slip
        // that stops the shrinking into MPCT_ST_QP_MAXITER instead of a wave that never retires
        // (the release build of commit 0272c65 hung the GPU that way).  it <= 2M < maxit here
        if (++it >= maxit) {
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
          bid = 4 * i + k;
        }
    }
    qargmin<16>(best, bid, 2);
    PSTAMP(PROF_QCHECK);
    if (!(best < -tol)) break;
    // a full active set (S.q == M) is legal: beta = 0 there, so the step is a dual one (a drop).
    // Warm starts reach it whenever every move sits on a bound; bailing out there flagged QPs the
    // cold-started C port solves (tests/test_gpu_parity.py KEY_TEST_STATUS_MISMATCH)
    if (it >= maxit) {
      *st |= MPCT_ST_QP_MAXITER_;
      break;
    }
    if (!S.jinit) gi16_load_rinv<PACKED>(S, F, sRi, M);
    const int p = bid;
    int j0, mp;
    double sgp;
    gi_normal(p, rc, j0, mp, sgp);
    double sp = best;  // slack of p along the path
    double upm = 0.0;  // its multiplier
    bool infeas = false;
    for (;;) {
      ++it;
      d4v Bl, d;
      b_row4(F.sB, Bl);  // issues under d's reduction
      gi16_dvec(F, j0, mp, sgp, d);
      double zm, jq, rk, dn2, beta;
      gi16_products(F, Bl, d, S.q, zm, jq, rk, dn2, beta);
      PSTAMP(PROF_QD);
      // dual step over active constraints with r_w > 0
      double t1 = INFINITY;
      int kdrop = 0x7fffffff;
      if (i < S.q && rk > 0.0) {
        t1 = qp_div(S.uw, rk);
        kdrop = i;
      }
      qargmin<16>(t1, kdrop, 0);
      const double t2 = (beta > 1e-14 * dn2) ? -qp_div(sp, beta) : INFINITY;
      const bool t2inf = __builtin_amdgcn_readfirstlane((int)(t2 == INFINITY)) != 0;
      if (t1 == INFINITY && t2inf) {
        *st |= MPCT_ST_QP_INFEAS_;
        infeas = true;
        break;
      }
      const bool full = __builtin_amdgcn_readfirstlane((int)(t2 <= t1)) != 0;
      const double t = full ? t2 : t1;
      if (!t2inf) xm += t * zm;
      if (i < S.q) S.uw -= t * rk;
      upm += t;
      sp += t * beta;
      PSTAMP(PROF_QR);
      if (full) {
        add(p, d, beta, zm, jq, rk, upm);
        PSTAMP(PROF_QADD);
        break;
      }
      if (kdrop >= S.q) {  // t1 or t2 NaN: no lane attains the ratio test (a non-finite state)
        *st |= MPCT_ST_NONFINITE_;
        infeas = true;
        break;
      }
#ifdef MPCT_PROFILE
      pacc[PROF_QROT] += (unsigned long long)(S.q - 1 - kdrop) * kProfCount;
#endif
      gi16_drop(S, F, sRA, M, kdrop, mark);
      PSTAMP(PROF_QDROP);
      if (it >= maxit) {
        *st |= MPCT_ST_QP_MAXITER_;
        break;
      }
    }
    if (it >= maxit || infeas) break;
  }
  xout = xm;
  return it;
}

}  // namespace mpct
