// mdband_kernel.hip — batched closed loop of the toolbox MPC with measured-disturbance
// feed-forward and soft output bands, one wavefront (64 lanes) per simulation.
//
// Replaces, per simulation, closedloop_toolbox.m:36-100 for an mpc object with measured
// disturbances (setmpcsignals MV/MD, Shell7x5.m:171-172, WoodBerry.m:102), OV Min/Max softened by
// MinECR/MaxECR (Shell7x5.m:141-152), ScaleFactors (Shell7x5.m:155-168, rescaled by
// MPCTuning.m:175-199) and Weights.ECR (Shell7x5.m:191).  Semantics restated in
// oracle/toolbox_band.py and DESIGN.md §11:
//   prediction y(t+k|t), k = 1..N2, MVs u(t-1) + cumulative moves (blocked after Nu), MDs held at
//   v(t) (MDLookAhead 'off'); nominal model, so the toolbox estimator's prediction is exact;
//   cost sum (w_y/s_y)^2 (r - y)^2 + sum (w_du/s_u)^2 du^2 + rho eps^2;
//   MV amplitude / rate hard, ymin - eps V s_y <= y <= ymax + eps V s_y, eps >= 0.
//
// Free response without a Phi table (Shell 7x5 at N2 = 127 would need ~1.4 MB of it): the window
// F_t[k] = y(t+1+k | MVs held at u(t-1), MDs held at v(t)) is carried across steps,
//     F_t[k] = F_{t-1}[k+1] + sum_n s_in(k+2) du_n(t-1) + sum_m s_im(k+1) dv_m(t),
// and its new last element F_t[N2-1] is one exact step of every model entry's difference equation
// from that entry's own tail of the window (one lane per entry; the tail gets the same step
// corrections).  No truncation: the update is exact for any stable or unstable LTI entry.
// QP on z = [dU; eps] (Mz = M + 1 lanes): H = R'R with R from the row-streamed Givens QR of
// [Q^1/2 G; Lambda^1/2; rho^1/2 e_eps] (band mode, Q = 0: R is diagonal), g = G'Q(F - r);
// constraints: 4 box rows per move (gpc_kernel.hip's encoding), eps >= 0 (row M, kind 0) and
// 2*my*N2 output rows with normals -/+[G_ik, V s]; the warm-started Goldfarb-Idnani method of
// gi_core.h with general normals staged in LDS and an LDS bitmap of active output rows.
#include <hip/hip_runtime.h>
#include <math.h>


#include "gi_core.h"
#include "launch_fan.h"
#include "mpct_dev.h"

#ifndef MPCT_XP_POLISH_K
#define MPCT_XP_POLISH_K 1
#endif
// J is rebuilt and x re-centred after MPCT_XP_DRIFT_K x Mz rotations.  16 against 4 with the
// normalised constraint choice: config-3 grid 1.67 against 1.70 s, slowest simulation 189 against
// 198 ms, F beyond 1e-6 of the C port 2.04 against 2.19 % (profiles/r04f_config3_ab.jsonl); with
// the relative termination test 64 against 16: 1.54-1.55 against 1.57 s, 154-155 against 159 ms,
// F 1.34 against 1.40 %; 128, 256 and never rebuilding measured the same as 64 (the final polish
// re-solves long QPs anyway; profiles/r04w_*, r04x_config3_rebuild_interval_sweep.jsonl)
#ifndef MPCT_XP_DRIFT_K
#define MPCT_XP_DRIFT_K 64
#endif
// the QP stops when no constraint's normalised slack is below -kRelTol max(1, |normalised bound|):
// the oracle's own test (toolbox_band.py qp_dual_dense, oracle/cband.c dual_solve).  Against the
// absolute 1e-10 slack of round 3: F beyond 1e-6 of the C port 2.04 -> 1.39 %, per-output J1 of
// the stratified sample 12.5 -> 7.8 %, same time; 1e-11 3.26 %, 1e-13 one failed simulation
// (profiles/r04l_config3_reltol_ab.jsonl).  0 restores the absolute o.feas_tol test
#ifndef MPCT_BAND_RELTOL
#define MPCT_BAND_RELTOL 1e-12
#endif
constexpr double kRelTol = MPCT_BAND_RELTOL;
// the output rows' inverse norms |n o D|^-1 (the constraint choice and the termination test) in
// float, 4 B per row side: doubles, as the oracle computes them, measured no closer to the C port and
// slower (grid 1.22 against 0.96 s)
typedef float rn_t;
// The QP keeps B = R_A^-1 instead of R_A, in R_A's packed place (band_drop_b): the dual direction
// r = R_A^-1 d, the warm start's R_A'w = c and lambda = R_A^-1 w become products over the active set
// instead of serial substitutions (one broadcast per active constraint, q ~ 41 on config 3's
// slowest simulations), and a drop's rotations come from B's row instead of a chain of LDS round
// trips through R_A (grid 0.95 -> 0.89 s, slowest simulation 147 -> 117 ms).
// Measured and not kept there, all bitwise equal: an odd column stride for J, an LDS copy of the
// QP's step rows, eight taps per trip in the output-row scan

namespace mpct {

struct BandLayout {
  int ri, jt, ra, dv, nv, xc, gv, sl, ob, fr, bits, du, uprev, ucum, ye, yeh, uring, tail, sext, rn, plb, pla,
      mzb, mza, total;
  int yh, ur, ts;  // entry output ring, input ring (powers of two) and tail stride of this scenario
};

__host__ __device__ inline int pow2_at_least(int n) {
  int r = 1;
  while (r < n) r <<= 1;
  return r;
}

// LDS layout of one simulation; [fr, plb) holds the windows, the histories and the active-row
// bitmap (zeroed at start)
// LDS tiers of the class launches: 8/6/5/4/3/2/1 workgroups per CU (the last must be 160;
// tools/ab3.sh: 4 tiers 3.09 s, 6 tiers 2.88 s; after the round-4 LDS diet the 20 KB tier of
// 8 per CU, the 216-VGPR kernel's limit, took the grid 1.03-1.05 -> 0.98 s, and a 7-per-CU
// 22 KB tier or dropping the 26 or 32 KB tier were slower: profiles/r04zg_*, r04zh_*).  The QP
// reads the MV step table from global memory (L1/L2-resident, shared by every simulation)
// instead of an LDS copy: 21.5 KB less LDS at N2 = 127, 3.14 -> 3.09 s
constexpr long long kBandCapsKb[] = {20, 26, 32, 40, 53, 80, 160};


// full_ri: R^-1 is a full triangle (some OV weight > 0); in band mode R is diagonal and only its
// inverse diagonal is kept.  ncopy: 2 with the open-loop prediction (a second plant copy), else 1
__host__ __device__ inline BandLayout band_layout(const DevScenario& sc, int N2, int M, bool full_ri = true,
                                                  int ncopy = 2) {
  const int Mz = M + 1, my = sc.my, nu = sc.nu, nin = sc.nin, ne = sc.ne;
  BandLayout L;
  int o = 0;
  auto take = [&](int n) { int r = o; o += (n + 1) & ~1; return r; };
  L.ri = take(full_ri ? Mz * Mz : Mz);
  L.jt = take(Mz * Mz);  // J, column-major JT[k*Mz + i] = J(i,k)
  L.ra = take(ra_packed_size(Mz));  // B = R_A^-1, packed as R_A would be (gi_core.h RAPacked)
  L.dv = take(Mz);       // d = J'n
  L.nv = take(Mz);       // staged normal n_p
  L.xc = take(Mz);       // QP iterate
  L.gv = take(full_ri ? Mz : 0);  // linear term / triangular-solve scratch (tracking weights only)
  L.sl = take(4 * Mz);   // box slacks at the unconstrained minimiser
  L.ob = take(4 * my);   // y_min, y_max, V_min s_y, V_max s_y
  L.fr = take(my * N2);                    // free-response window, shifted in place every step
  L.bits = take((2 * my * N2 + 63) / 64);  // active output rows (32-bit words)
  L.du = take(nu);                         // du(t-1)
  L.uprev = take(nu);
  L.ucum = take(ncopy == 2 ? M : 0);  // open-loop Uopt only
  // the rings hold what the recursions read back: an entry's last pl_maxa outputs; the inputs of
  // the longest numerator (delay included) and the window tails' t - 1 (Shell 7x5: 2 and 16
  // instead of the general kernel's 8 and 32, 6.6 KB less LDS per simulation)
  const int nbmax = sc.pl_maxb > sc.mz_maxb ? sc.pl_maxb : sc.mz_maxb;
  L.yh = pow2_at_least(sc.pl_maxa);
  L.ur = pow2_at_least(nbmax > 2 ? nbmax : 2);
  L.ts = sc.mz_maxa > 2 ? sc.mz_maxa - 1 : 1;
  L.ye = take(ncopy * ne);
  L.yeh = take(ncopy * ne * L.yh);
  L.uring = take(ncopy * nin * L.ur);
  L.tail = take(ne * L.ts);  // model entry tails of the window (mz_na - 1 entries each)
  L.sext = take(ne);            // model entry window extensions
  L.rn = take(my * N2);  // output rows' inverse norms: 2 floats (upper, lower) per row
  L.plb = take(ne * sc.pl_maxbc);  // compact: taps from the first nonzero one
  L.pla = take(ne * sc.pl_maxa);
  L.mzb = take(ne * sc.mz_maxbc);
  L.mza = take(ne * sc.mz_maxa);
  L.total = (o + 1) & ~1;
  return L;
}

// B = R_A^-1 of the band kernel, in R_A's packed layout (gi_core.h RAPacked: column
// k holds rows 0..k+1).  Entry (k + 1, k) is kept zero on the active block, and bt_mul / bt_tmul
// read it in place of every entry below the stored ones.
__device__ __forceinline__ int bt_idx(int w, int k) { return (int)(__umul24((unsigned)k, (unsigned)(k + 3)) >> 1) + w; }
// gi_add's hook: column q = [-r / alpha; 1 / alpha] (r = R_A^-1 d(0:q), the iteration's dual
// direction), the stored entries below the diagonal next to it zeroed
struct BandBAdd {
  double* bt;
  double r;  // this lane's r_w
  __device__ __forceinline__ void add(int q, double ia) const {
    const int lane = threadIdx.x;
    if (lane < q) bt[bt_idx(lane, q)] = -r * ia;
    else if (lane == q) bt[bt_idx(q, q)] = ia;
    if (lane == q && q > 0) bt[bt_idx(q, q - 1)] = 0.0;
    if (lane == q + 1) bt[bt_idx(q + 1, q)] = 0.0;
  }
};
// lane w < q: sum_{k < q} B(w,k) c_k, c in LDS
__device__ __forceinline__ double bt_mul(const double* bt, const double* c, int q) {
  const int lane = threadIdx.x;
  double r0 = 0.0, r1 = 0.0;
  if (lane < q) {
    auto b = [&](int k) __attribute__((always_inline)) { return bt[bt_idx(min(lane, k + 1), k)]; };
    int k = 0;
    for (; k + 3 < q; k += 4) {
      const double b0 = b(k), b1 = b(k + 1), b2 = b(k + 2), b3 = b(k + 3);
      const double c0 = c[k], c1 = c[k + 1], c2 = c[k + 2], c3 = c[k + 3];
      r0 = fma(b0, c0, r0);
      r1 = fma(b1, c1, r1);
      r0 = fma(b2, c2, r0);
      r1 = fma(b3, c3, r1);
    }
    for (; k < q; ++k) r0 = fma(b(k), c[k], r0);
  }
  return r0 + r1;
}
// lane v < q: (B'c)_v = sum_{k < q} B(k,v) c_k, i.e. w with R_A'w = c
__device__ __forceinline__ double bt_tmul(const double* bt, const double* c, int q) {
  const int lane = threadIdx.x;
  double r0 = 0.0, r1 = 0.0;
  if (lane < q) {
    const double* col = bt + bt_idx(0, lane);
    auto b = [&](int k) __attribute__((always_inline)) { return col[min(k, lane + 1)]; };
    int k = 0;
    for (; k + 3 < q; k += 4) {
      const double b0 = b(k), b1 = b(k + 1), b2 = b(k + 2), b3 = b(k + 3);
      const double c0 = c[k], c1 = c[k + 1], c2 = c[k + 2], c3 = c[k + 3];
      r0 = fma(b0, c0, r0);
      r1 = fma(b1, c1, r1);
      r0 = fma(b2, c2, r0);
      r1 = fma(b3, c3, r1);
    }
    for (; k < q; ++k) r0 = fma(b(k), c[k], r0);
  }
  return r0 + r1;
}
// inclusive prefix sum over the wave's lanes: DPP row_shr within each 16-lane row, then the row
// totals (readlane) carried into the rows above
__device__ __forceinline__ double wave_prefix_sum(double v) {
  const int i = threadIdx.x & 15, b = threadIdx.x >> 4;
  double t;
  t = dppd<0x111>(v); if (i >= 1) v += t;
  t = dppd<0x112>(v); if (i >= 2) v += t;
  t = dppd<0x114>(v); if (i >= 4) v += t;
  t = dppd<0x118>(v); if (i >= 8) v += t;
  const double t0 = bcast(v, 15), t1 = bcast(v, 31), t2 = bcast(v, 47);
  if (b >= 1) v += t0;
  if (b >= 2) v += t1;
  if (b >= 3) v += t2;
  return v;
}
// remove active constraint kd with B alone.  R_A E (column kd removed) is re-triangularised by
// rotations G on rows (jj, jj + 1), jj = kd..q-2; then B_new = (B G')[rows != kd, columns < q-1],
// which is upper triangular exactly when G turns B's row kd into a multiple of e_{q-1} (row kd of
// B G' times R_new = row kd of E = 0).  So rotation jj zeroes the running entry x of row kd against
// y = B(kd, jj + 1): cs = y / r, sn = -x / r, r = |row kd (kd..jj+1)|, all from one prefix sum of
// B(kd, .)^2 -- no serial chain of LDS round trips (the R_A form's rsq + RMW + lds_sync per
// rotation).  The same rotations go to J's columns; each lane then sweeps its row of J and of B
// through them with the running entry in a register, writing B's rows kd + 1.. one row up.
// The same factorisation as the R_A form up to the signs of R_new's rows (Givens QR is unique up
// to them), which J and B carry consistently.  cs / sn are staged in sc_ / ss_ (Mz doubles each).
template <int MAXM, class Mark>
__device__ __forceinline__ void band_drop_b(GIState<MAXM>& S, double* sJT, double* bt, int Mz, int kd,
                                            const Mark& mark, double* sc_, double* ss_) {
  const int lane = threadIdx.x;
  const int q = S.q;
  const int idk = __builtin_amdgcn_readlane(S.ww, kd);
  mark(S, idk, false);
  {
    const double un = lane_next<MAXM>(S.uw);
    const int wn = lane_next_i<MAXM>(S.ww);
    if (lane >= kd && lane < q - 1) {
      S.uw = un;
      S.ww = wn;
    }
  }
  // rotation parameters: lane jj in [kd, q-2]
  const double y = (lane >= kd && lane < q) ? bt[bt_idx(kd, lane)] : 0.0;
  const double s2 = wave_prefix_sum(y * y);  // lane j: |B(kd, kd..j)|^2
  const double yn = lane_next<MAXM>(y), r2 = lane_next<MAXM>(s2);
  if (lane >= kd && lane < q - 1) {
    const double x = lane == kd ? y : (s2 > 0.0 ? s2 * rsq_nr(s2) : 0.0);
    double cs = 1.0, sn = 0.0;
    if (r2 > 0.0) {
      const double ri = rsq_nr(r2);
      cs = yn * ri;
      sn = -x * ri;
    }
    sc_[lane] = cs;
    ss_[lane] = sn;
  }
  lds_sync();
  // J's columns (lanes = rows of J) and B's rows by slot (lanes = rows w < q)
  const bool jrow = lane < Mz, brow = lane < q;
  double cj = jrow ? sJT[kd * Mz + lane] : 0.0;
  double cb = (brow && lane <= kd + 1) ? bt[bt_idx(lane, kd)] : 0.0;
  const int wdst = lane > kd ? lane - 1 : lane;  // B's row kd leaves: rows below move up one
  for (int jj = kd; jj < q - 1; ++jj) {
    const double cs = sc_[jj], sn = ss_[jj];
    const double nj = jrow ? sJT[(jj + 1) * Mz + lane] : 0.0;
    const double nb = (brow && lane <= jj + 2) ? bt[bt_idx(min(lane, jj + 2), jj + 1)] : 0.0;
    if (jrow) sJT[jj * Mz + lane] = cs * cj + sn * nj;
    const double vb = cs * cb + sn * nb;
    if (brow && lane != kd && wdst <= jj + 1) bt[bt_idx(wdst, jj)] = vb;
    cj = -sn * cj + cs * nj;
    cb = -sn * cb + cs * nb;
  }
  if (jrow) sJT[(q - 1) * Mz + lane] = cj;
  const int qn = q - 1;
  if (lane == qn) {
    S.uw = 0.0;
    S.ww = -1;
  }
  S.nrot += q - 1 - kd;
  S.q = qn;
  lds_sync();
}

// active flags: box rows (p < 4*Mz) in the lanes' act bits, output rows in the LDS bitmap
struct BandMark {
  unsigned* bits;
  int base;
  template <class St>
  __device__ __forceinline__ void operator()(St& S, int p, bool on) const {
    if (p < base) {
      BoxMark{}(S, p, on);
    } else if (threadIdx.x == 0) {
      const int q = p - base;
      if (on) bits[q >> 5] |= 1u << (q & 31);
      else bits[q >> 5] &= ~(1u << (q & 31));
    }
  }
};

template <int MAXM>
__global__ void __launch_bounds__(64, 1)
    mdband_closed_loop_kernel(const DevScenario sc, long long C, int nref, const int* __restrict__ N2v,
                              const int* __restrict__ Nuv, const double* __restrict__ deltav,
                              const double* __restrict__ lambdav, const double* __restrict__ rv,
                              const double* __restrict__ vv, const DevOpts o, const DevResult out,
                              int mz_lo, long long lds_lo, long long lds_hi, int first) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x;
  const long long sim = blockIdx.x;
  if (sim >= C * nref) return;
  const long long c = sim / nref;
  const int kref = (int)(sim - c * nref);
  const int my = sc.my, nu = sc.nu, nd = sc.nd, nin = sc.nin, nit = sc.nit, ne = sc.ne, tlen = sc.tlen;
  const int N2 = N2v[c], Nu = Nuv[c];
  const int M = nu * Nu, Mz = M + 1;
  const int P = my * N2;
  int st = 0;
#ifdef MPCT_PROFILE
  ProfAccS pacc;
  unsigned long long pprev = __builtin_amdgcn_s_memtime();
#endif

  auto write_nan = [&](int status) __attribute__((always_inline)) {
    if (lane < my) {
      if (out.J1) out.J1[sim * my + lane] = NAN;
      if (out.j21) out.j21[sim * my + lane] = NAN;
      if (out.j22) out.j22[sim * my + lane] = NAN;
    }
    if (lane < nu && out.Jnu) out.Jnu[sim * nu + lane] = NAN;
    if (lane == 0) {
      if (out.status) out.status[sim] = status;
      if (out.qp_iters) out.qp_iters[sim] = 0;
    }
  };
  if (N2 <= 0) {
    if (first) write_nan(MPCT_ST_SKIPPED_);
    return;
  }
  if (N2 > sc.n2max || Nu < 1 || Nu > sc.numax || Nu > N2) {
    if (first) write_nan(MPCT_ST_BADHORIZON_);
    return;
  }
  const double* dl = deltav + c * my;
  const double* lm = lambdav + c * nu;
  // toolbox weights over scale factors: q_i = (delta_i / s_y,i)^2, w_n = (lambda_n / s_u,n)^2
  auto qw = [&](int i) __attribute__((always_inline)) -> double {
    const double w = fabs(dl[i]) * sc.wscale[i];
    return sc.wsq ? w * w : w;
  };
  bool any_q = false;  // some OV tracked: R full; band mode: R (and J = R^-1) diagonal
  for (int i = 0; i < my; ++i) any_q = any_q || qw(i) > 0.0;
  const BandLayout L = band_layout(sc, N2, M, any_q, o.open_loop ? 2 : 1);
  // this launch serves one (QP size, LDS) class: the others' simulations leave at once
  if (Mz <= mz_lo || Mz > MAXM || (long long)L.total * 8 <= lds_lo || (long long)L.total * 8 > lds_hi) return;
  const int tls = sc.tlen;
  double* sRi = lds + L.ri;
  double* sJT = lds + L.jt;
  double* sRA = lds + L.ra;
  double* sBT = lds + L.ra;
  double* sd = lds + L.dv;
  double* snv = lds + L.nv;
  double* sxc = lds + L.xc;
  double* sgv = lds + L.gv;
  double* ssl = lds + L.sl;
  double* sob = lds + L.ob;
  double* sfr = lds + L.fr;
  unsigned* sbits = reinterpret_cast<unsigned*>(lds + L.bits);
  double* sdu = lds + L.du;
  double* suprev = lds + L.uprev;
  double* sucum = lds + L.ucum;
  double* sye = lds + L.ye;
  double* syeh = lds + L.yeh;
  double* sur = lds + L.uring;
  double* stail = lds + L.tail;
  const int umask = L.ur - 1, ymask = L.yh - 1;
  double* sext = lds + L.sext;
  double* splb = lds + L.plb;
  double* spla = lds + L.pla;
  double* smzb = lds + L.mzb;
  double* smza = lds + L.mza;
  const double* __restrict__ sstep = sc.step;  // global, L1/L2-resident

  // ------------------------------------------------------------------ prologue
  for (int e = lane; e < ne * sc.pl_maxbc; e += kWave) {
    const int en = e / sc.pl_maxbc, l = e - en * sc.pl_maxbc, off = sc.pl_off[en];
    splb[e] = off + l < sc.pl_nb[en] ? sc.pl_b[en * sc.pl_maxb + off + l] : 0.0;
  }
  for (int e = lane; e < ne * sc.pl_maxa; e += kWave) spla[e] = sc.pl_a[e];
  for (int e = lane; e < ne * sc.mz_maxbc; e += kWave) {
    const int en = e / sc.mz_maxbc, l = e - en * sc.mz_maxbc, off = sc.mz_off[en];
    smzb[e] = off + l < sc.mz_nb[en] ? sc.mz_b[en * sc.mz_maxb + off + l] : 0.0;
  }
  for (int e = lane; e < ne * sc.mz_maxa; e += kWave) smza[e] = sc.mz_a[e];
  for (int e = lane; e < 4 * my; e += kWave) sob[e] = sc.obnd[e];
  for (int e = lane; e < L.plb - L.fr; e += kWave) lds[L.fr + e] = 0.0;
  const bool row = lane < Mz;  // QP-row lanes: moves 0..M-1, eps at M
  RowCons rcn;
  rcn.n = lane < M ? lane / Nu : 0;
  rcn.l = lane < M ? lane - rcn.n * Nu : 0;
  rcn.dmin = sc.bnd[rcn.n];
  rcn.dmax = sc.bnd[nu + rcn.n];
  rcn.umin = sc.bnd[2 * nu + rcn.n];
  rcn.umax = sc.bnd[3 * nu + rcn.n];
  lds_sync();

  // QR of W = [Q^1/2 G (outputs with q_i > 0); Lambda^1/2; rho^1/2 e_eps] by row-streamed Givens
  // rotations (lane = column of R); rows of outputs with q_i = 0 are zero and skipped
  {
    double rcol[MAXM];
    {
      double w0 = 0.0;
      if (lane < M) {
        const double ln = fabs(lm[rcn.n]) * sc.wscale[my + rcn.n];
        w0 = sc.wsq ? ln : sqrt(ln);
      } else if (lane == M) {
        w0 = sqrt(sc.rho);
      }
#pragma unroll
      for (int k = 0; k < MAXM; ++k) rcol[k] = (k == lane) ? w0 : 0.0;
    }
    for (int i = 0; i < my; ++i) {
      const double qi = qw(i);
      if (!(qi > 0.0)) continue;
      const double sq = sqrt(qi);
      for (int r = 0; r < N2; ++r) {
        double w = 0.0;
        if (lane < M) {
          const int tt = 1 + r - rcn.l;
          w = tt >= 0 ? sq * sstep[(i * nu + rcn.n) * tls + tt] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < MAXM; ++k) {
          if (k < M) {  // the eps column never meets a G row
            const double b = bcast(w, k);
            const double a = bcast(rcol[k], k);
            const double rho = sqrt(a * a + b * b);
            const bool nz = b != 0.0;
            const double cs = nz ? a / rho : 1.0, sn = nz ? b / rho : 0.0;
            const double rk = rcol[k];
            rcol[k] = cs * rk + sn * w;
            w = -sn * rk + cs * w;
          }
        }
      }
    }
    double* sR = sJT;  // R parks in J's region until the QP starts
    double hmm = 0.0;  // H(m, m) = |column m of R|^2 (QR keeps W's column norms)
    if (row) {
#pragma unroll
      for (int k = 0; k < MAXM; ++k)
        if (k < Mz) {
          sR[k * Mz + lane] = rcol[k];
          hmm = fma(rcol[k], rcol[k], hmm);
        }
      snv[lane] = 1.0 / hmm;  // D^2 = diag(H)^-1 (the oracle's equilibration, toolbox_band.py band_qp)
    }
    lds_sync();
    bool spd = true;
    for (int k = 0; k < Mz; ++k)
      if (!(sR[k * Mz + k] > 0.0)) spd = false;
    if (!spd) {
      write_nan(MPCT_ST_NONFINITE_);
      return;
    }
    // R^-1 (upper, row-major): lane j solves R x = e_j in its own column; band mode: R is
    // diagonal, only 1/R_jj is kept
    if (row && !any_q) {
      sRi[lane] = 1.0 / sR[lane * Mz + lane];
    } else if (row) {
      for (int kk = lane; kk >= 0; --kk) {
        double a = (kk == lane) ? 1.0 : 0.0;
        for (int j = kk + 1; j <= lane; ++j) a -= sR[kk * Mz + j] * sRi[j * Mz + lane];
        sRi[kk * Mz + lane] = a / sR[kk * Mz + kk];
      }
      for (int kk = lane + 1; kk < Mz; ++kk) sRi[kk * Mz + lane] = 0.0;
    }
    lds_sync();
  }

  // the most violated constraint is chosen in the oracle's metric (toolbox_band.py band_qp,
  // oracle/cband.c): equilibrated variables D^-1 z, D = diag(H)^-1/2, and unit constraint rows,
  // i.e. the slack over |n o D|.  Raw slacks favour the output rows' large step-response
  // normals over the move bounds; the heaviest config-3 simulation took 3.5x the oracle's GI steps.
  // Box rows of lane m: kinds 0/1 (n = e_m), the cumulative kinds 2/3 (n = e_j0 + .. + e_m), eps >= 0
  // on lane M; output rows q = 2 g + side (upper, lower) from a float table (a selection weight only)
  double ib01 = 0.0, ib23 = 0.0;
  const rn_t* srn = reinterpret_cast<const rn_t*>(lds + L.rn);
  {
    const double d2 = row ? snv[lane] : 0.0;
    const double pre = block_prefix<MAXM>(d2, rcn.l, Nu, lane < M, sxc);
    if (row) {
      ib01 = rsq_nr(d2);
      ib23 = lane < M ? rsq_nr(pre) : 0.0;
    }
    rn_t* wrn = reinterpret_cast<rn_t*>(lds + L.rn);
    for (int g = lane; g < P; g += kWave) {
      const int i = g / N2, k = g - i * N2;
      const int lmax = min(Nu - 1, k + 1);
      double a = 0.0;
      for (int n = 0; n < nu; ++n) {
        const double* sp = sstep + (i * nu + n) * tls + (k + 1);
        for (int l = 0; l <= lmax; ++l) a = fma(sp[-l] * sp[-l], snv[n * Nu + l], a);
      }
      const double vu = sob[3 * my + i], vl = sob[2 * my + i], de = snv[M];
      // a zero normal (a hard bound inside the dead time) keeps norm 1, as the oracle's rn does
      // (toolbox_band.py band_qp, cband.c): its violation stays visible to the choice and the test
      const double nu2 = fma(vu * vu, de, a), nl2 = fma(vl * vl, de, a);
      wrn[2 * g] = nu2 > 0.0 ? (rn_t)rsq_nr(nu2) : (rn_t)1;
      wrn[2 * g + 1] = nl2 > 0.0 ? (rn_t)rsq_nr(nl2) : (rn_t)1;
    }
    lds_sync();
  }

  const double tol = o.feas_tol;
  // what the callers of most_violated accept as a violation: the winner itself under the
  // oracle's relative test (its raw slack is then negative), else the absolute tolerance
  const double tol_acc = kRelTol > 0.0 ? 0.0 : tol;
  const int maxit = o.max_qp_iter > 0 ? o.max_qp_iter : 200 * Mz + 1000;
  long long iters = 0;
  const double* rr = rv + (long long)kref * my * nit;
  const double* vvk = vv ? vv + (long long)kref * nd * nit : nullptr;
  const int base = 4 * Mz;  // first output-row constraint id
  const BandMark mark{sbits, base};
  GIState<MAXM> gis;
  gi_reset<MAXM>(gis);
#ifdef MPCT_DIAG
  gis.diag = o.diag;
#endif
#ifdef MPCT_DEBUG_BAND
  int dbg_t = -1, dbg_reb = 0, dbg_pol = 0, dbg_git = 0;
#endif

  // J = R^-1 (gi_load_rinv), or its diagonal in band mode
  auto load_j = [&]() __attribute__((always_inline)) {
    if (any_q) {
      gi_load_rinv<MAXM>(gis, sJT, sRi, Mz, row);
    } else {
      if (row) {
        const double dj = sRi[lane];
        for (int k = 0; k < Mz; ++k) sJT[k * Mz + lane] = k == lane ? dj : 0.0;
      }
      gis.nrot = 0;
      gis.jinit = true;
      lds_sync();
    }
  };
  // predicted output of row g = i*N2 + k at the iterate in sxc: F[g] + G_g dU
  auto yhat = [&](const double* F, int g) __attribute__((always_inline)) -> double {
    const int i = g / N2, k = g - i * N2;
    double a0 = F[g], a1 = 0.0;
    const int lmax = min(Nu - 1, k + 1);
    for (int n = 0; n < nu; ++n) {
      const double* sp = sstep + (i * nu + n) * tls + (k + 1);
      const double* xp = sxc + n * Nu;
      int l = 0;
      // four taps per trip, their loads issued together; the accumulation order (even taps into
      // a0, odd into a1) is the two-tap loop's
      for (; l + 3 <= lmax; l += 4) {
        const double s0 = sp[-l], s1 = sp[-l - 1], s2 = sp[-l - 2], s3 = sp[-l - 3];
        const double x0 = xp[l], x1 = xp[l + 1], x2 = xp[l + 2], x3 = xp[l + 3];
        a0 += s0 * x0;
        a1 += s1 * x1;
        a0 += s2 * x2;
        a1 += s3 * x3;
      }
      for (; l + 1 <= lmax; l += 2) {
        a0 += sp[-l] * xp[l];
        a1 += sp[-l - 1] * xp[l + 1];
      }
      if (l <= lmax) a0 += sp[-l] * xp[l];
    }
    return a0 + a1;
  };
  // slack of output-row constraint q = 2g + side at the iterate (eps = x_M)
  auto out_slack = [&](const double* F, int q, double eps) __attribute__((always_inline)) -> double {
    const int g = q >> 1, i = g / N2;
    const double yh = yhat(F, g);
    if (q & 1) return yh - sob[i] + sob[2 * my + i] * eps;        // lower: y + V s eps >= ymin
    return sob[my + i] + sob[3 * my + i] * eps - yh;              // upper: ymax + V s eps >= y
  };
  auto out_active = [&](int q) __attribute__((always_inline)) -> bool { return (sbits[q >> 5] >> (q & 31)) & 1u; };
  // stage the normal of constraint p in LDS and return this lane's d_k = (J'n_p)_k (also in sd)
  auto dvec = [&](int p) __attribute__((always_inline)) -> double {
    const int lpm = __builtin_amdgcn_readlane(rcn.l, p < base ? (p >> 2) : 0);  // uniform
    if (row) {
      double nvv = 0.0;
      if (p < base) {
        const int m = p >> 2, kind = p & 3;
        if (m == M) {
          nvv = lane == M ? 1.0 : 0.0;
        } else {
          const int j0 = kind < 2 ? m : m - lpm;
          nvv = (lane >= j0 && lane <= m) ? ((kind & 1) ? -1.0 : 1.0) : 0.0;
        }
      } else {
        const int q = p - base, g = q >> 1, i = g / N2, k = g - i * N2;
        if (lane < M) {
          const int tt = k + 1 - rcn.l;
          nvv = tt >= 0 ? sstep[(i * nu + rcn.n) * tls + tt] : 0.0;
          if (!(q & 1)) nvv = -nvv;
        } else {
          nvv = sob[((q & 1) ? 2 : 3) * my + i];
        }
      }
      snv[lane] = nvv;
    }
    lds_sync();
    double dk = 0.0;
    if (row) {
      const double* jc = sJT + lane * Mz;
      double d1 = 0.0;
      int r = 0;
      for (; r + 3 < Mz; r += 4) {  // four terms' loads together, the two-term loop's order
        const double j0 = jc[r], j1 = jc[r + 1], j2 = jc[r + 2], j3 = jc[r + 3];
        const double n0 = snv[r], n1 = snv[r + 1], n2 = snv[r + 2], n3 = snv[r + 3];
        dk += j0 * n0;
        d1 += j1 * n1;
        dk += j2 * n2;
        d1 += j3 * n3;
      }
      for (; r + 1 < Mz; r += 2) {
        dk += jc[r] * snv[r];
        d1 += jc[r + 1] * snv[r + 1];
      }
      if (r < Mz) dk += jc[r] * snv[r];
      dk += d1;
      sd[lane] = dk;
    }
    return dk;
  };

  // one toolbox QP at the window F, reference r (lane i < my holds r_i), MV u_prev in LDS;
  // result in sxc (moves 0..M-1, eps at M)
  auto solve = [&](const double* F, double r_i) __attribute__((always_inline)) {
    PSTAMP(PROF_PLANT);
    // ---- unconstrained minimiser x_u = -R^-1 R^-T g, g = G'Q(F - r)  (g = 0 in band mode)
    double xu = 0.0;
    if (any_q) {
      if (lane < my) sgv[lane] = r_i;
      lds_sync();
      double g = 0.0;
      if (lane < M) {
        for (int i = 0; i < my; ++i) {
          const double qi = qw(i);
          if (!(qi > 0.0)) continue;
          const double ri = sgv[i];
          const double* sp = sstep + (i * nu + rcn.n) * tls;
          for (int k = rcn.l > 0 ? rcn.l - 1 : 0; k < N2; ++k) g += qi * sp[k + 1 - rcn.l] * (F[i * N2 + k] - ri);
        }
      }
      lds_sync();
      if (row) sgv[lane] = g;
      lds_sync();
      double y = 0.0;
      if (row)
        for (int m = 0; m <= lane; ++m) y += sRi[m * Mz + lane] * sgv[m];
      lds_sync();
      if (row) sgv[lane] = y;
      lds_sync();
      if (row)
        for (int k = lane; k < Mz; ++k) xu -= sRi[lane * Mz + k] * sgv[k];
    }
    const double up_row = lane < M ? suprev[rcn.n] : 0.0;
    const double lo_box = fmax(rcn.dmin, rcn.umin - up_row), hi_box = fmin(rcn.dmax, rcn.umax - up_row);
    auto box_slacks = [&](double x, double s[4]) __attribute__((always_inline)) {
      const double pre = block_prefix<MAXM>(x, rcn.l, Nu, lane < M, sxc);
      s[0] = s[1] = s[2] = s[3] = INFINITY;
      if (lane < M) {
        if (rcn.l == 0) {
          s[0] = x - lo_box;
          s[1] = hi_box - x;
        } else {
          s[0] = x - rcn.dmin;
          s[1] = rcn.dmax - x;
          s[2] = pre - (rcn.umin - up_row);
          s[3] = (rcn.umax - up_row) - pre;
        }
      } else if (lane == M) {
        s[0] = x;  // eps >= 0
      }
    };
    // most violated constraint at the iterate x (this lane's component xm); all_rows: include the
    // active set (the entry test of x_u, which the retained set does not constrain)
    auto most_violated = [&](double xm, double& best, int& bid, double s[4], bool all_rows)
                             __attribute__((always_inline)) {
      box_slacks(xm, s);
      if (row) sxc[lane] = xm;
      lds_sync();
      // key = slack / |n o D| over the rows violated beyond tol; best = the winner's raw slack
      double key = INFINITY;
      double kraw = INFINITY;  // the raw slack of this lane's best row (handed to every lane below)
      bid = 0x7fffffff;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double ibk = k < 2 ? ib01 : ib23;
        // kRelTol > 0: the oracle's test, normalised slack below -tol max(1, |normalised bound|)
        double bk = 0.0;
        if (lane < M) {
          if (rcn.l == 0) bk = k == 0 ? lo_box : -hi_box;
          else bk = k == 0 ? rcn.dmin : (k == 1 ? -rcn.dmax : (k == 2 ? rcn.umin - up_row : up_row - rcn.umax));
        }
        const bool vk = kRelTol > 0.0 ? s[k] * ibk < -kRelTol * fmax(1.0, fabs(bk) * ibk) : s[k] < -tol;
        if ((all_rows || !((gis.act >> k) & 1u)) && vk) {
          const double kk = s[k] * ibk;
          if (kk < key) {
            key = kk;
            kraw = s[k];
            bid = 4 * lane + k;
          }
        }
      }
      const double eps = sxc[M];
      for (int g = lane; g < P; g += kWave) {
        const int i = g / N2;
        const double yh = yhat(F, g);
        if (isfinite(sob[my + i])) {
          const int q = 2 * g;
          const double s_up = sob[my + i] + sob[3 * my + i] * eps - yh;
          const bool vu = kRelTol > 0.0
                              ? s_up * (double)srn[q] < -kRelTol * fmax(1.0, fabs(F[g] - sob[my + i]) * (double)srn[q])
                              : s_up < -tol;
          if (vu && (all_rows || !out_active(q))) {
            const double kk = s_up * (double)srn[q];
            if (kk < key) {
              key = kk;
              kraw = s_up;
              bid = base + q;
            }
          }
        }
        if (isfinite(sob[i])) {
          const int q = 2 * g + 1;
          const double s_lo = yh - sob[i] + sob[2 * my + i] * eps;
          const bool vl = kRelTol > 0.0
                              ? s_lo * (double)srn[q] < -kRelTol * fmax(1.0, fabs(sob[i] - F[g]) * (double)srn[q])
                              : s_lo < -tol;
          if (vl && (all_rows || !out_active(q))) {
            const double kk = s_lo * (double)srn[q];
            if (kk < key) {
              key = kk;
              kraw = s_lo;
              bid = base + q;
            }
          }
        }
      }
      wave_argmin64(key, bid);
      // the winner's raw slack, from the lane that scanned it: box row 4 m + kind on lane m, output
      // row q = 2 g + side on lane g mod 64 (the scan's own value: no second prediction of that row)
      if (key == INFINITY) best = INFINITY;
      else best = bcast(kraw, bid < base ? (bid >> 2) : (((bid - base) >> 1) & (kWave - 1)));
    };
    int it = 0;   // all factorisation work (GI steps + rebuild re-adds + re-centring drops): qp_iters
    int git = 0;  // GI add/drop steps only: the iteration cap guards against cycling, not rebuilds
    // exact solve of the equality problem on the active set from x_u (needs sxc = x_u and this
    // lane's box slacks at x_u in s): J and R_A rebuilt from R^-1 when stale (or forced), then
    // x = x_u + J_A w with R_A'w = b_A - N_A'x_u, dropping negative multipliers one at a time.
    // Used for the warm start, and to re-centre long QPs whose incremental updates drift off the
    // active rows (the N2 = 127 search range runs ~450 iterations in one QP).
    auto eqp_from_xu = [&](const double s[4], bool force) __attribute__((always_inline)) -> double {
      if (row) {
#pragma unroll
        for (int k = 0; k < 4; ++k) ssl[4 * lane + k] = s[k];
      }
      lds_sync();
      if (force || !gis.jinit || gis.nrot >= MPCT_XP_DRIFT_K * Mz) {
        const int qq = gis.q;
        load_j();
        gis.q = 0;
        for (int v = 0; v < qq; ++v) {
          const int p = __builtin_amdgcn_readlane(gis.ww, v);
          const double dk = dvec(p);
          const double beta = qsum<MAXM>(lane >= v && row ? dk * dk : 0.0);
          lds_sync();
          const double zm = gi_z(sJT, sd, v, Mz, row);
          const double uk = gis.uw;
          gi_add<MAXM>(gis, sJT, sRA, sd, Mz, p, dk, beta, zm, 0.0, row, mark, RANone{},
                       BandBAdd{sBT, bt_mul(sBT, sd, v)});
          if (lane == v) gis.uw = uk;
          ++it;
        }
        gis.nrot = 0;
#ifdef MPCT_DEBUG_BAND
        ++dbg_reb;
#endif
      }
      lds_sync();
      double x = row ? xu : 0.0;
      int nd = 0;  // drops of this solve: each shrinks the set, so at most q <= Mz of them
      for (;;) {
        const int q = gis.q;
        if (q == 0) {
          x = row ? xu : 0.0;
          break;
        }
        double cc = 0.0;
        if (lane < q) {
          const int p = gis.ww;
          cc = p < base ? -ssl[p] : -out_slack(F, p - base, sxc[M]);
        }
        double wv = 0.0;
        x = row ? xu : 0.0;
        double lam;
        // w = B'c, then x = x_u + J(:,0:q) w and lambda = B w, three products (w staged in sd)
        if (row) snv[lane] = cc;
        lds_sync();
        wv = bt_tmul(sBT, snv, q);
        if (row) sd[lane] = lane < q ? wv : 0.0;
        lds_sync();
        if (row) {
          double x1 = 0.0;
          int v = 0;
          for (; v + 1 < q; v += 2) {
            x = fma(sJT[v * Mz + lane], sd[v], x);
            x1 = fma(sJT[(v + 1) * Mz + lane], sd[v + 1], x1);
          }
          if (v < q) x = fma(sJT[v * Mz + lane], sd[v], x);
          x += x1;
        }
        lam = bt_mul(sBT, sd, q);
        lds_sync();  // sd / snv are rewritten by the next dvec or pass
        if (lane < q) gis.uw = lam;
        double lmin = lane < q ? lam : INFINITY;
        int kd = lane;
        qargmin<MAXM>(lmin, kd);
        if (!(lmin < 0.0)) break;
#ifdef MPCT_DIAG
        if (!(gis.diag & kDiagSkipWarmDrop))
#endif
        band_drop_b(gis, sJT, sBT, Mz, kd, mark, snv, sd);
        ++it;
        if (++nd > Mz) {  // only a logic slip that stops the set shrinking gets here (gpc_qp16.h)
          st |= MPCT_ST_QP_MAXITER_;
          break;
        }
      }
      return row ? x : 0.0;
    };
    // re-centre at x_u's slacks (recomputed: sxc and ssl hold the current iterate's)
    auto recentre = [&](bool force) __attribute__((always_inline)) -> double {
      double b0, s0[4];
      int i0;
      most_violated(row ? xu : 0.0, b0, i0, s0, true);
      return eqp_from_xu(s0, force);
    };
    double xm = row ? xu : 0.0;
    {
      double best, s[4];
      int bid;
      most_violated(xm, best, bid, s, true);
#ifdef MPCT_DEBUG_BAND
      if (sim == 0 && lane == 0 && dbg_t < MPCT_DEBUG_BAND)
        printf("  entry t=%d best=%.3e bid=%d q=%d xu0=%.9e xuNu=%.9e\n", dbg_t, best, bid, gis.q, sxc[0], sxc[Nu]);
#endif
      if (!(best < -tol_acc)) return 0;  // x_u feasible: optimal (the retained set is kept)
      if (gis.q == 0) {
        gis.jinit = false;
      } else {
        xm = eqp_from_xu(s, false);
        PSTAMP(PROF_QWARM);
      }
    }
    int npolish = 0;
    for (;;) {
      double best, s[4];
      int bid;
      most_violated(xm, best, bid, s, false);
      PSTAMP(PROF_QCHECK);
      if (!(best < -tol_acc)) {
        // optimal up to the incremental updates: after a long QP re-solve the final active set
        // exactly from x_u (fresh J) and re-check every row before accepting
        if (gis.q > 0 && gis.nrot >= MPCT_XP_POLISH_K * Mz && npolish < 2) {
          ++npolish;
#ifdef MPCT_DEBUG_BAND
          ++dbg_pol;
#endif
          xm = recentre(true);
          PSTAMP(PROF_QWARM);
          continue;
        }
        break;
      }
      // a full active set (q == Mz) is legal here: beta = 0 forces dual steps (drops) first
      if (git >= maxit) {
        st |= MPCT_ST_QP_MAXITER_;
        break;
      }
      if (gis.q > 0 && gis.nrot >= MPCT_XP_DRIFT_K * Mz) {  // J has drifted: rebuild it and re-centre x
        xm = recentre(true);
        PSTAMP(PROF_QWARM);
        continue;
      }
      if (!gis.jinit) load_j();
      const int p = bid;
      double sp = best, upm = 0.0;
      bool infeas = false;
      for (;;) {
        ++it;
        ++git;
        const double dk = dvec(p);
        const double d2 = row ? dk * dk : 0.0;
        const double dn2 = qsum<MAXM>(d2);
        const double beta = qsum<MAXM>(lane >= gis.q ? d2 : 0.0);
        lds_sync();
        const double zm = gi_z(sJT, sd, gis.q, Mz, row);
        PSTAMP(PROF_QD);
        const double rk = bt_mul(sBT, sd, gis.q);
        double t1 = INFINITY;
        int kdrop = 0x7fffffff;
        if (lane < gis.q && rk > 0.0) {
          t1 = qp_div(gis.uw, rk);
          kdrop = lane;
        }
        qargmin<MAXM>(t1, kdrop);
        PSTAMP(PROF_QR);
        const double t2 = (beta > 1e-20 * dn2) ? -qp_div(sp, beta) : INFINITY;
        if (t1 == INFINITY && t2 == INFINITY) {
          st |= MPCT_ST_QP_INFEAS_;
          infeas = true;
          break;
        }
        const bool full = t2 <= t1;
        const double t = full ? t2 : t1;
        if (t2 != INFINITY) xm += t * zm;
        if (lane < gis.q) gis.uw -= t * rk;
        upm += t;
        sp += t * beta;
        if (full) {
          gi_add<MAXM>(gis, sJT, sRA, sd, Mz, p, dk, beta, zm, upm, row, mark, RANone{}, BandBAdd{sBT, rk});
          PSTAMP(PROF_QADD);
          break;
        }
        if (kdrop >= gis.q) {  // t1 or t2 NaN: no lane attains the ratio test (a non-finite state)
          st |= MPCT_ST_NONFINITE_;
          infeas = true;
          break;
        }
        band_drop_b(gis, sJT, sBT, Mz, kdrop, mark, snv, sd);
        PSTAMP(PROF_QDROP);
        if (git >= maxit) {
          st |= MPCT_ST_QP_MAXITER_;
          break;
        }
      }
      if (infeas) break;
      if (git >= maxit) {
        st |= MPCT_ST_QP_MAXITER_;
        break;
      }
    }
    if (row) sxc[lane] = xm;
    PSTAMP(PROF_QP);
    lds_sync();
#ifdef MPCT_DEBUG_BAND
    dbg_git = git;
#endif
    return it;
  };

  // ------------------------------------------------------------------ open-loop prediction
  // closedloop_toolbox.m:86-91: initial state, yo = 0, reference r(:,end), MD v(:,end) held from
  // time 0: the window is the MD step responses times v_end
  double jnu = 0.0;
  if (o.open_loop) {
    for (int g = lane; g < P; g += kWave) {
      const int i = g / N2, k = g - i * N2;
      double f = 0.0;
      for (int m = 0; m < nd; ++m) f += sc.step_md[(i * nd + m) * tlen + k + 1] * vvk[m * nit + nit - 1];
      sfr[g] = f;
    }
    lds_sync();
    iters += solve(sfr, lane < my ? rr[lane * nit + nit - 1] : 0.0);
    if (lane < M) {
      double s = 0.0;
      for (int j = lane - rcn.l; j <= lane; ++j) s += sxc[j];
      sucum[lane] = s;  // Uopt row l of MV n (held after Nu-1)
    }
    // the closed loop's first step shifts a zero window (the open-loop one is done with)
    for (int g = lane; g < P; g += kWave) sfr[g] = 0.0;
    lds_sync();
    if (lane < nu) {
      // VNS2.m:183-191: Xnu = |uopt(:,1)| ./ |diff(uopt)|, inf/NaN -> 0, Jnu = sum Xnu^2
      const double u0 = fabs(sucum[lane * Nu]);
      const int nd_ = Nu - 1 < nit - 1 ? Nu - 1 : nit - 1;
      for (int t = 0; t < nd_; ++t) {
        const double dd = fabs(sucum[lane * Nu + t + 1] - sucum[lane * Nu + t]);
        const double xr = u0 / dd;
        if (isfinite(xr)) jnu += xr * xr;
      }
    }
  }

  PSTAMP(PROF_PROLOGUE);
  // ------------------------------------------------------------------ closed loop
  double j1 = 0.0, j21 = 0.0, j22 = 0.0;
  const int ncopy = o.open_loop ? 2 : 1;
  double r_t = 0.0, yr_t = 0.0;
  if (lane < my) {
    r_t = rr[lane * nit];
    yr_t = sc.yref[lane * nit];
  }
  for (int t = 0; t < nit; ++t) {
    double r_n = 0.0, yr_n = 0.0;
    if (lane < my && t + 1 < nit) {
      r_n = rr[lane * nit + t + 1];
      yr_n = sc.yref[lane * nit + t + 1];
    }
    // inputs known at t: MDs v(t) (both copies); the open-loop copy's MVs uopt(t)
    for (int e = lane; e < ncopy * nd; e += kWave) {
      const int cpy = e / nd, j = e - cpy * nd;
      sur[(cpy * nin + nu + j) * L.ur + (t & umask)] = vvk[j * nit + t];
    }
    if (o.open_loop && lane < nu) {
      const int l = t < Nu - 1 ? t : Nu - 1;
      sur[(nin + lane) * L.ur + (t & umask)] = sucum[lane * Nu + l];
    }
    lds_sync();
    // plant entries y_e(t) (copy 0 closed loop, copy 1 open loop driven by uopt)
    for (int e = lane; e < ncopy * ne; e += kWave) {
      const int cpy = e / ne, ee = e - cpy * ne, j = ee % nin;
      const double* eb = splb + ee * sc.pl_maxbc - sc.pl_off[ee];  // tap l at eb[l], l >= off
      const double* ea = spla + ee * sc.pl_maxa;
      const double* eur = sur + (cpy * nin + j) * L.ur;
      double* eyh = syeh + e * L.yh;
      const int nb = sc.pl_nb[ee], na = sc.pl_na[ee], off = sc.pl_off[ee];
      double a0 = 0.0, a1 = 0.0;
      for (int l = off; l < nb; ++l) a0 += eb[l] * eur[(t - l) & umask];
      for (int l = 1; l < na; ++l) a1 -= ea[l] * eyh[(t - l) & ymask];
      const double acc = a0 + a1;
      eyh[t & ymask] = acc;
      sye[e] = acc;
    }
    lds_sync();
    if (lane < my) {
      const int i = lane;
      double y = 0.0;
      for (int j = 0; j < nin; ++j) y += sye[i * nin + j];
      const double e1 = y - yr_t;
      j1 += e1 * e1;
      if (t >= sc.ink0) j22 += e1 * e1;
      double ysv = 0.0;
      if (o.open_loop) {
        for (int j = 0; j < nin; ++j) ysv += sye[ne + i * nin + j];
        if (t >= sc.ink0) j21 += (y - ysv) * (y - ysv);
      }
      if (o.want_traj) {
        if (out.y) out.y[(sim * my + i) * nit + t] = y;
        if (o.open_loop && out.ys) out.ys[(sim * my + i) * nit + t] = ysv;
      }
    }
    // ---- free-response window F_{t-1} -> F_t
    // model entry tails: step corrections for du(t-1) and dv(t), then one difference-equation
    // step at tau = t + N2 (MVs u(min(tau', t-1)), MDs v(min(tau', t)))
    for (int e = lane; e < ne; e += kWave) {
      const int i = e / nin, j = e - i * nin;
      const double* mb = smzb + e * sc.mz_maxbc - sc.mz_off[e];  // tap l at mb[l], l >= off
      const double* ma = smza + e * sc.mz_maxa;
      const double* eur = sur + j * L.ur;
      double* tl = stail + e * L.ts;
      const int nb = sc.mz_nb[e], na = sc.mz_na[e] - 1, off = sc.mz_off[e];
      if (j < nu) {
        const double dlt = sdu[j];
        if (dlt != 0.0) {
          const double* sp = sstep + (i * nu + j) * tls;
          for (int l = 0; l < na; ++l)
            if (N2 - l >= 0) tl[l] += sp[N2 - l] * dlt;
        }
      } else {
        const double vt = eur[t & umask];
        const double dlt = vt - (t > 0 ? eur[(t - 1) & umask] : 0.0);
        if (dlt != 0.0) {
          const double* sp = sc.step_md + (i * nd + (j - nu)) * tlen;
          for (int l = 0; l < na; ++l)
            if (N2 - 1 - l >= 0) tl[l] += sp[N2 - 1 - l] * dlt;
        }
      }
      const int tcap = j < nu ? t - 1 : t;
      double a0 = 0.0, a1 = 0.0;
      for (int l = off; l < nb; ++l) {
        const int tau = min(t + N2 - l, tcap);
        if (tau >= 0) a0 += mb[l] * eur[tau & umask];
      }
      for (int l = 1; l <= na; ++l) a1 -= ma[l] * tl[l - 1];
      const double ext = a0 + a1;
      for (int l = na - 1; l > 0; --l) tl[l] = tl[l - 1];
      if (na > 0) tl[0] = ext;
      sext[e] = ext;
    }
    lds_sync();
    // F(t) = shifted F(t-1) + the step's increments, in place: entry g reads g + 1 of the same
    // output block before any lane stores g + 1 (one wave; the loads of a trip issue before its
    // stores, and the clobber keeps the next trip's store of g + 64 behind this trip's load of it)
    const double* Fp = sfr;
    double* Fc = sfr;
    bool any_dv = false;
    for (int m = 0; m < nd; ++m) {
      const double* vr = sur + (nu + m) * L.ur;
      any_dv = any_dv || (vr[t & umask] != (t > 0 ? vr[(t - 1) & umask] : 0.0));
    }
    for (int g = lane; g < P; g += kWave) {
      const int i = g / N2, k = g - i * N2;
      double f;
      if (k < N2 - 1) {
        f = Fp[g + 1];
        for (int n = 0; n < nu; ++n) f += sstep[(i * nu + n) * tls + k + 2] * sdu[n];
        if (any_dv) {
          for (int m = 0; m < nd; ++m) {
            const double* vr = sur + (nu + m) * L.ur;
            const double dv = vr[t & umask] - (t > 0 ? vr[(t - 1) & umask] : 0.0);
            f += sc.step_md[(i * nd + m) * tlen + k + 1] * dv;
          }
        }
      } else {
        f = 0.0;
        for (int j = 0; j < nin; ++j) f += sext[i * nin + j];
      }
      Fc[g] = f;
      asm volatile("" ::: "memory");
    }
    lds_sync();
#ifdef MPCT_DEBUG_BAND
    dbg_t = t;
    dbg_reb = dbg_pol = dbg_git = 0;
    const int it_dbg = solve(Fc, r_t);
    iters += it_dbg;
    if (sim == 0 && lane == 0 && t == MPCT_DEBUG_BAND - 3)
      for (int m = 0; m < Mz; ++m) printf("X %d %.17e\n", m, sxc[m]);
    if (sim == 0 && lane == 0 && t < MPCT_DEBUG_BAND)
      printf("t=%d it=%d git=%d reb=%d pol=%d q=%d eps=%.9e du=%.9e %.9e %.9e F0=%.9e Fend=%.9e y6=%.9e st=%d\n", t, it_dbg, dbg_git, dbg_reb, dbg_pol, gis.q,
             sxc[M], sxc[0], sxc[Nu], sxc[2 * Nu], Fc[0], Fc[N2 - 1], Fc[6 * N2], st);
#else
    iters += solve(Fc, r_t);
#endif
#ifdef MPCT_DEBUG_BAND_STEP
    // diagnostic build: the QP solution and active set of simulation 0 at one step
    if (sim == 0 && t == MPCT_DEBUG_BAND_STEP) {
      if (lane == 0) printf("STEP %d q=%d st=%d base=%d\n", t, gis.q, st, base);
      if (lane <= M) printf("X %d %.17e\n", lane, sxc[lane]);
      if (lane < gis.q) printf("A %d %d %.17e\n", lane, gis.ww, gis.uw);
    }
#endif
    if (lane < nu) {
      const int n = lane;
      const double du = sxc[n * Nu];
      const double un = suprev[n] + du;
      sdu[n] = du;
      sur[n * L.ur + (t & umask)] = un;
      if (o.want_traj) {
        if (out.u) out.u[(sim * nu + n) * nit + t] = un;
        if (o.open_loop && out.uopt) {
          const int l = t < Nu - 1 ? t : Nu - 1;
          out.uopt[(sim * nu + n) * nit + t] = sucum[n * Nu + l];
        }
      }
      suprev[n] = un;
    }
    lds_sync();
    r_t = r_n;
    yr_t = yr_n;
  }

#ifdef MPCT_PROFILE
  PSTAMP(PROF_PLANT);
  if (lane == 0 && out.prof)
    for (int k = 0; k < PROF_N; ++k) out.prof[sim * PROF_N + k] = pacc.get(k);
#endif
  // ------------------------------------------------------------------ results
  if (lane < my) {
    if (!isfinite(j1)) st |= MPCT_ST_NONFINITE_;
    if (out.J1) out.J1[sim * my + lane] = j1;
    if (out.j22) out.j22[sim * my + lane] = j22;
    if (out.j21) out.j21[sim * my + lane] = o.open_loop ? j21 : NAN;
  }
  if (lane < nu && out.Jnu) out.Jnu[sim * nu + lane] = o.open_loop ? jnu : NAN;
  const unsigned long long nf = __ballot(st & MPCT_ST_NONFINITE_);
  if (lane == 0) {
    const int s = st | (nf ? MPCT_ST_NONFINITE_ : 0);
    if (out.status) out.status[sim] = s;
    if (out.qp_iters) out.qp_iters[sim] = iters;
  }
}

}  // namespace mpct

// ------------------------------------------------------------------------------------------
// host-side launch
#include <algorithm>
#include <string>

#include "work_order.h"

namespace mpct {

long long mdband_lds_bytes(const DevScenario& sc, int N2, int Nu, int ncopy) {
  // the larger of the two R^-1 forms (full triangle / band-mode diagonal): the step-row copy of
  // band_layout depends on the rest of the layout, so neither total bounds the other
  const BandLayout Lf = band_layout(sc, N2, sc.nu * Nu, true, ncopy);
  const BandLayout Ld = band_layout(sc, N2, sc.nu * Nu, false, ncopy);
  return (long long)std::max(Lf.total, Ld.total) * 8;
}

// One launch per (QP size class MAXM, occupancy class): the dynamic LDS of a launch is what its
// class's largest simulation needs, so short-horizon candidates are not held to the occupancy of
// the scenario's (n2_max, nu_max) corner (one workgroup per CU at Shell 7x5's first 104 KiB).  Every
// launch spans the whole batch; a simulation runs in the one launch whose class holds its
// (Mz, LDS bytes) and leaves the others at once (no host round trip to bucket device-resident
// candidates).  Status-only outcomes (padding, bad horizons) are written by the first launch.
// Heaviest classes first, fanned over the caller's stream and the auxiliary streams of `fan`
// (launch_fan.h): light classes fill the SIMDs a 1-workgroup-per-CU class leaves idle.
template <int MAXM>
static int launch_band_t(const DevScenario& sc, long long C, int nref, const int* N2, const int* Nu,
                         const double* delta, const double* lambda, const double* r, const double* v,
                         const DevOpts& o, const DevResult& out, FanScope& fs, int& nl, int mz_lo, bool& first,
                         std::string* err) {
  const int nu_hi = std::min(sc.numax, (MAXM - 1) / sc.nu);
  if (nu_hi < 1) return 0;
  // the largest simulation of the class (over every N2 and Nu: no monotonicity assumed)
  long long lds_max = 0;
  for (int nu_c = 1; nu_c <= nu_hi; ++nu_c)
    for (int n2 = 1; n2 <= sc.n2max; ++n2)
      lds_max = std::max(lds_max, mdband_lds_bytes(sc, n2, nu_c, o.open_loop ? 2 : 1));
  if (lds_max > 160 * 1024) {
    *err = "scenario needs more than 160 KiB of LDS per simulation";
    return -4;
  }
  auto kern = mdband_closed_loop_kernel<MAXM>;
  const long long* capkb = kBandCapsKb;  // workgroups per CU: 160 KB / cap
  constexpr int kCaps = (int)(sizeof(kBandCapsKb) / sizeof(kBandCapsKb[0]));
  static_assert(kCaps <= 8, "at most 8 LDS tiers");
  long long lo[8], hi[8];
  int ncls = 0;
  for (long long l = 0; ncls < kCaps && l < lds_max; ++ncls) {
    lo[ncls] = l;
    hi[ncls] = std::min(capkb[ncls] * 1024, lds_max);
    l = hi[ncls];
  }
  for (int k = ncls - 1; k >= 0; --k) {
    const long long lds = hi[k];
    if (lds > 64 * 1024) {
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds) != hipSuccess) {
        *err = "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed";
        return -3;
      }
    }
    const hipStream_t ls = fs.stream(nl);
    if (!diag_drop_launch(nl++))
      hipLaunchKernelGGL(kern, dim3((unsigned)(C * nref)), dim3(kWave), (size_t)lds, ls, sc, C, nref, N2, Nu, delta,
                         lambda, r, v, o, out, mz_lo, lo[k], lds, first ? 1 : 0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      *err = std::string("kernel launch failed: ") + hipGetErrorString(e);
      return -3;
    }
    first = false;
  }
  return 0;
}

int launch_mdband(const DevScenario& sc, long long C, int nref, const int* N2, const int* Nu, const double* delta,
                  const double* lambda, const double* r, const double* v, const DevOpts& o, const DevResult& out,
                  hipStream_t stream, LaunchFan* fan, std::string* err) {
  const int Mz = sc.nu * sc.numax + 1;
  if (Mz > 64) {
    *err = "nu*nu_max + 1 > 64";
    return -4;
  }
  int rc = prefill_results(out, C * nref, sc.my, sc.nu, stream, err);
  if (rc) return rc;
  FanScope fs(fan, stream);
  bool first = true;
  int nl = 0;
  if (Mz > 32) rc = launch_band_t<64>(sc, C, nref, N2, Nu, delta, lambda, r, v, o, out, fs, nl, 32, first, err);
  if (rc == 0 && Mz > 16)
    rc = launch_band_t<32>(sc, C, nref, N2, Nu, delta, lambda, r, v, o, out, fs, nl, 16, first, err);
  if (rc == 0) rc = launch_band_t<16>(sc, C, nref, N2, Nu, delta, lambda, r, v, o, out, fs, nl, 0, first, err);
  fs.join();
  return rc;
}

}  // namespace mpct
