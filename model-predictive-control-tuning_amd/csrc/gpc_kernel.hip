// gpc_kernel.hip — batched closed-loop GPC simulation, one wavefront (64 lanes) per simulation.
//
// Replaces, per simulation, the body of closedloop_toolbox.m:36-100 (sim + mpcstate/mpcmove +
// lsim) with the toolbox-equivalent GPC of DESIGN.md:
//   prologue (once per candidate): G from the step table (MatG.m:64-67); QR of the weighted
//       least-squares matrix W = [Q^1/2 G; Lambda^1/2] by row-streamed Givens rotations carrying
//       V = [Q^1/2 Phi; 0] (Phi: Diophantine F | deltaUFree/cell2mat2 rows built on the host, on
//       a backward-difference basis); A = -R^-1 Q1'V (unconstrained gain), R^-1 for the QP.
//   per step t: plant output (exact difference equations of every (i,j) entry — lsim),
//       unconstrained minimiser dU = A x (x = [y-r, nabla y .. | du history]: the state of
//       DTC_GPC_WW.m:139-146 S*Yd + Hp*up), then the Goldfarb-Idnani dual active-set QP (the
//       toolbox's KWIK is of this family) when a rate / amplitude bound is violated; first move of
//       every MV applied; histories shifted.
// Latency design (one wave per simulation, the step loop is a serial recurrence):
//   * everything a step reads lives in LDS or registers (no global loads in the loop except the
//     prefetched r(t+1), Yref(t+1));
//   * scalars are broadcast with v_readlane (SGPR), QP-row reductions use DPP row operations when
//     M <= 16, the active-set QR runs lanes-as-rows entirely in registers;
//   * a workgroup is exactly one wave: LDS hand-offs between lanes need only lgkmcnt(0) and a
//     compiler fence (no s_barrier, no vmcnt drain of the prefetches).
// Small plants in cost-only batches (the metric) run gpc_small_kernel (gpc_small.hip) instead; this
// kernel is the general instance: any plant size, DTC mode, open-loop leg and trajectories.
#include <hip/hip_runtime.h>
#include <math.h>

#include "mpct_dev.h"
#include "gi_core.h"
#include "gpc_qp.h"
#include "gpc_qp16.h"
#include "gpc_prologue.h"
#include "gpc_record.h"

namespace mpct {

// waves per SIMD the VGPR budget allows: 168 VGPRs = 3 in the M <= 16 class (its LDS, 13.4 KB at
// Shell 3x3, allows that); the larger classes are LDS-bound at 1-2 workgroups per CU and uncapped
constexpr int kWaves16 = 3;

struct LdsLayout {
  int rinv, jt, dv, ra, sl, gb, A, x, xc, uprev, yprev, ucum, ye, yeh, uring, mzh, smz, frh, plb, pla, mzb,
      mza, frb, fra, total;
};

// LDS layout of one simulation; [x, plb) holds the state and every history (zeroed at start).
// ext: the EXT instance, whose open-loop leg needs a second copy of the plant state and Uopt; the
// cost-only instance leaves them out (13,440 -> 12,472 B at Shell 3x3: 12 instead of 11
// workgroups per CU at the 512-B LDS allocation granularity)
__host__ __device__ inline LdsLayout lds_layout(const DevScenario& sc, int M, bool ext) {
  const int nx = sc.nx, nu = sc.nu, nin = sc.nin, ne = sc.ne, my = sc.my;
  const int nmz = sc.dtc ? 2 * my * nu : 0;  // DTC predictor model entries (Pz, Gz)
  const int nfr = sc.dtc ? my : 0;           // DTC robustness filters
  const int ncp = ext ? 2 : 1;               // plant copies: closed loop (+ open loop)
  LdsLayout L;
  int o = 0;
  auto take = [&](int n) { int r = o; o += (n + 1) & ~1; return r; };
  const bool regqp = M <= 16;  // the M <= 16 class keeps J and d in VGPRs (gpc_qp16.h)
  L.rinv = take(M * M);
  L.jt = take(regqp ? 0 : M * M);  // J of the active-set method, column-major JT[k*M + i] = J(i,k)
  L.dv = take(regqp ? 0 : M);      // d = J'n_p
  L.ra = take(M * M);        // R_A of the active-set method (persists across steps)
  L.sl = take(regqp ? 0 : 4 * M);  // wide classes: slacks of the 4M constraints at x_u
  L.gb = take(regqp ? 16 * kBS : 0);  // M <= 16 class: B = R_A^-1 (row-major, stride kBS)
  L.A = take(((nx + 1) & ~1) * M);  // row-major A[m][s], rows padded to even length (16-B reads)
  L.x = take(nx + 1);
  L.xc = take(M);
  L.uprev = take(nu);
  L.yprev = take(my);
  L.ucum = take(ext ? M : 0);
  L.ye = take(ncp * ne);
  // plant entry output histories: the register path of the wide classes needs none; the M <= 16
  // class keeps them here (its row-packed plant holds only one tap per lane)
  L.yeh = take(sc.regpath && !regqp ? 0 : ncp * ne * kYeHist);
  L.uring = take(ncp * nin * kURing);
  L.mzh = take(nmz * kYeHist);   // DTC: model entry output histories
  L.smz = take(nmz);             // DTC: model entry outputs of the step
  L.frh = take(nfr * 2 * kYeHist);  // DTC: filter input (eM) and output histories
  L.plb = take(ne * sc.pl_maxb);
  L.pla = take(ne * sc.pl_maxa);
  L.mzb = take(nmz * (sc.dtc ? sc.mz_maxb : 0));
  L.mza = take(nmz * (sc.dtc ? sc.mz_maxa : 0));
  L.frb = take(nfr * (sc.dtc ? sc.fr_max : 0));
  L.fra = take(nfr * (sc.dtc ? sc.fr_max : 0));
  L.total = (o + 1) & ~1;
  return L;
}

// EXT: the open-loop prediction and/or trajectories may be requested; the EXT = false instance
// (GAM scoring: costs only) carries none of their state through the step loop
template <int MAXM, bool DTC, bool EXT>
__global__ void __launch_bounds__(64, MAXM <= 16 ? kWaves16 : 1)
    gpc_closed_loop_kernel(const DevScenario sc, long long C, int nref,
                           const int* __restrict__ N2v, const int* __restrict__ Nuv,
                           const double* __restrict__ deltav, const double* __restrict__ lambdav,
                           const double* __restrict__ rv, const double* __restrict__ vv,
                           const int* __restrict__ perm, const DevOpts o, const DevResult out, int mlo,
                           int first) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x;
  // workgroup slot -> candidate: perm (heaviest estimated work first, see order_candidates) or
  // identity; a candidate's nref simulations take consecutive slots, results stay in place
  const long long slot = blockIdx.x;
  if (slot >= C * nref) return;
  const long long cs = slot / nref;
  const int kref = (int)(slot - cs * nref);
  const long long c = perm ? (long long)perm[cs] : cs;
  const long long sim = c * nref + kref;
  const int my = sc.my, nu = sc.nu, nin = sc.nin, nit = sc.nit, nx = sc.nx, ne = sc.ne;
  const int N2 = N2v[c], Nu = Nuv[c];
  const int M = nu * Nu;
  int st = 0;
#ifdef MPCT_PROFILE
  ProfAccS pacc;
  unsigned long long pprev = __builtin_amdgcn_s_memtime();
#endif
#ifdef MPCT_TIMELINE
  // diagnostic build: when this workgroup ran and where (tools/diag/timeline.py)
  const unsigned long long tl_t0 = __builtin_amdgcn_s_memrealtime();
#endif

  // the cost record: caller's arrays at `sim`, or staging row xcd_row(slot) (ordered launches)
  auto put = [&](double j1v, double j21v, double j22v, double jnuv, int status, long long itv)
                 __attribute__((always_inline)) {
    put_record(out, slot, C * nref, sim, sc.my, sc.nu, lane, j1v, j21v, j22v, jnuv, status, itv);
  };
  auto write_nan = [&](int status) __attribute__((always_inline)) { put(NAN, NAN, NAN, NAN, status, 0); };
  if (N2 <= 0) {
    if (first) write_nan(MPCT_ST_SKIPPED_);
    return;
  }
  if (N2 > sc.n2max || Nu < 1 || Nu > sc.numax || Nu > N2) {
    if (first) write_nan(MPCT_ST_BADHORIZON_);
    return;
  }
  if (M <= mlo || M > MAXM) return;  // another QP-size class launch simulates it
  const LdsLayout L = lds_layout(sc, M, EXT);
  const int nxp = (nx + 1) & ~1;  // padded row length of A (x[nx] and the pad column are 0)
  double* sRi = lds + L.rinv;
  double* sA = lds + L.A;
  double* sx = lds + L.x;
  double* sxc = lds + L.xc;
  double* suprev = lds + L.uprev;
  double* syprev = lds + L.yprev;
  double* sucum = lds + L.ucum;
  double* sye = lds + L.ye;
  double* syeh = lds + L.yeh;
  double* sur = lds + L.uring;
  double* splb = lds + L.plb;
  double* spla = lds + L.pla;

  // ------------------------------------------------------------------ prologue
  // this simulation's plant variant (Monte-Carlo draw k % nvar)
  const int pvar = sc.nvar > 1 ? kref % sc.nvar : 0;
  const int pve = pvar * ne;
  for (int e = lane; e < ne * sc.pl_maxb; e += kWave) splb[e] = sc.pl_b[(long long)pve * sc.pl_maxb + e];
  for (int e = lane; e < ne * sc.pl_maxa; e += kWave) spla[e] = sc.pl_a[(long long)pve * sc.pl_maxa + e];
  if constexpr (DTC) {  // predictor model entries and filters (DTC_GPC_WW.m:40-46, mimofilter.m)
    const int nmz = 2 * my * nu;
    for (int e = lane; e < nmz * sc.mz_maxb; e += kWave) lds[L.mzb + e] = sc.mz_b[e];
    for (int e = lane; e < nmz * sc.mz_maxa; e += kWave) lds[L.mza + e] = sc.mz_a[e];
    for (int e = lane; e < my * sc.fr_max; e += kWave) {
      lds[L.frb + e] = sc.fr_b[e];
      lds[L.fra + e] = sc.fr_a[e];
    }
  }
  for (int e = lane; e < L.plb - L.x; e += kWave) lds[L.x + e] = 0.0;  // state + histories
  const double* dl = deltav + c * my;
  const double* lm = lambdav + c * nu;
  lds_sync();

  // prologue (gpc_prologue.h): A = -R^-1 Q1'V row-major with padded rows, R^-1; R parks in
  // J's region (R_A's in the M <= 16 class) until the QP starts
  double* sR = lds + (MAXM <= 16 ? L.ra : L.jt);
  if (!gpc_prologue<MAXM>(sc, lane, M, Nu, N2, dl, lm, sR, sRi, sA, nxp, nullptr)) {
    write_nan(MPCT_ST_NONFINITE_);
    return;
  }
  if (lane < M && nxp > nx) sA[lane * nxp + nx] = 0.0;  // pad column
  lds_sync();
  PSTAMP(PROF_PROLOGUE);

  // per-lane constants of the step loop, defined after the prologue so that they are not live
  // (and spilled) across its register-heavy QR
  const int yoff_i = lane < my ? sc.yoff[lane] : 0;
  const int nyh_i = lane < my ? sc.nyhi[lane] : 0;
  const int upoff_n = lane < nu ? sc.upoff[lane] : 0;
  const int dum_n = lane < nu ? sc.dum[lane] : 0;
  // QP row of the lane: in the M <= 16 class every 16-lane row block replicates the QP rows
  const int qrow = MAXM <= 16 ? (lane & 15) : lane;
  RowCons rcn;
  rcn.n = qrow < M ? qrow / Nu : 0;
  rcn.l = qrow < M ? qrow - rcn.n * Nu : 0;
  rcn.dmin = sc.bnd[rcn.n];
  rcn.dmax = sc.bnd[nu + rcn.n];
  rcn.umin = sc.bnd[2 * nu + rcn.n];
  rcn.umax = sc.bnd[3 * nu + rcn.n];
  // plant entry of the lane; the M <= 16 class packs the entries row-wise: lane (e, k) = e + 16 k
  // holds tap k of entry e (plant_packed below)
  const bool plant_packed = MAXM <= 16 && sc.regpath != 0 && ((EXT && o.open_loop) ? 2 : 1) * ne <= 16;
  const int elane = plant_packed ? (lane & 15) : lane;
  const int ecopy = elane / ne;
  const int ee = elane - ecopy * ne;
  const int ej = ee % nin;
  const int e_nb = (elane < ne * 2) ? sc.pl_nb[pve + ee] : 0;
  const int e_na = (elane < ne * 2) ? sc.pl_na[pve + ee] : 0;
  const int e_off = (elane < ne * 2) ? sc.pl_off[pve + ee] : 0;
  const double tol = o.feas_tol;
  const int maxit = o.max_qp_iter > 0 ? o.max_qp_iter : 8 * M + 16;
  long long iters = 0;
  const double* rr = rv + (long long)kref * my * nit;
  const double* vvk = vv ? vv + (long long)kref * sc.nd * nit : nullptr;

  GIState<MAXM> gis;  // active-set factorisation carried across the steps (warm start)
  gi_reset<MAXM>(gis);
#ifdef MPCT_DIAG
  gis.diag = o.diag;
#endif
  RegFactors rf;      // M <= 16 class: J in VGPRs, B = R_A^-1 in LDS (gpc_qp16.h), valid once gis.jinit
  FOR4(r, rf.J[r] = 0.0;);
  rf.sB = lds + L.gb;
  // unconstrained minimiser dU = A x, then the QP; result in sxc
  auto solve_step = [&]() __attribute__((always_inline)) {
    double xu = 0.0;
    if constexpr (MAXM <= 16) {
      // the four 16-lane rows split A's column pairs; row m of A on lanes m, m+16, m+32, m+48
      const int m = lane & 15, grp = lane >> 4;
      const int npair = nxp / 2, per = (npair + 3) >> 2;
      const int p0 = grp * per, p1 = min(npair, p0 + per);
      double a0 = 0.0, a1 = 0.0;
      if (m < M) {
        const double2* arow = reinterpret_cast<const double2*>(sA + m * nxp);
        const double2* xv = reinterpret_cast<const double2*>(sx);
        for (int q2 = p0; q2 < p1; ++q2) {
          const double2 av = arow[q2], xa = xv[q2];
          a0 += av.x * xa.x;
          a1 += av.y * xa.y;
        }
      }
      xu = row4_sum(a0 + a1);  // row m of A . x on lanes m, m+16, m+32, m+48
      if (m >= M) xu = 0.0;
    } else if (lane < M) {
      // 16-byte LDS reads: two A entries of this row and two x entries per load
      const double2* arow = reinterpret_cast<const double2*>(sA + lane * nxp);
      const double2* xv = reinterpret_cast<const double2*>(sx);
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      int s2 = 0;
      for (; s2 + 1 < nxp / 2; s2 += 2) {
        const double2 av = arow[s2], bv = arow[s2 + 1];
        const double2 xa = xv[s2], xb = xv[s2 + 1];
        a0 += av.x * xa.x;
        a1 += av.y * xa.y;
        a2 += bv.x * xb.x;
        a3 += bv.y * xb.y;
      }
      if (s2 < nxp / 2) {
        const double2 av = arow[s2], xa = xv[s2];
        a0 += av.x * xa.x;
        a1 += av.y * xa.y;
      }
      xu = (a0 + a1) + (a2 + a3);
      sxc[lane] = xu;
    }
    if constexpr (MAXM > 16) lds_sync();
    PSTAMP(PROF_UNC);
    if constexpr (MAXM <= 16) {
      double xq;
      iters += gi_qp16(lds + L.rinv, lds + L.ra, M, Nu, rcn, qrow < M ? suprev[rcn.n] : 0.0, xu,
                       tol, maxit, &st, gis, rf, DTC ? kGiRebuild16Dtc : kGiRebuild16, xq
#ifdef MPCT_PROFILE
                       , pacc, pprev
#endif
      );
      if (lane < M) sxc[lane] = xq;
      lds_sync();
    } else {
      const QPBufs qb{lds + L.rinv, lds + L.xc, lds + L.jt, lds + L.dv, lds + L.ra, lds + L.sl};
      iters += gi_qp<MAXM>(qb, M, Nu, rcn, lane < M ? suprev[rcn.n] : 0.0, xu, tol, maxit, &st, gis
#ifdef MPCT_PROFILE
                           , pacc, pprev
#endif
      );
    }
    PSTAMP(PROF_QP);
  };

  // ------------------------------------------------------------------ open-loop prediction
  double jnu = 0.0;
  if ((EXT && o.open_loop)) {
    // closedloop_toolbox.m:86-91: initial state (y = 0), reference r(:, end)
    if (lane < my) sx[yoff_i] = -rr[lane * nit + (nit - 1)];
    lds_sync();
    solve_step();
    if (lane < M) {
      double s = 0.0;
      for (int j = lane - rcn.l; j <= lane; ++j) s += sxc[j];
      sucum[lane] = s;  // Uopt row l for MV n (held after Nu-1)
    }
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
    if (lane < my) sx[yoff_i] = 0.0;
    lds_sync();
    PSTAMP(PROF_OPENLOOP);
  }

  // ------------------------------------------------------------------ closed loop
  double j1 = 0.0, j21 = 0.0, j22 = 0.0;
  const int ncopy = (EXT && o.open_loop) ? 2 : 1;
  const bool is_entry = elane < ncopy * ne;
  const double* eb = splb + ee * sc.pl_maxb;
  const double* ea = spla + ee * sc.pl_maxa;
  double* eyh = syeh + elane * kYeHist;
  const double* eur = sur + (ecopy * nin + ej) * kURing;
  // register-resident per-lane state (regpath, wide classes): plant entry taps / denominator /
  // output history
  constexpr int kRB = MAXM <= 16 ? 1 : kRegB, kRA = MAXM <= 16 ? 1 : kRegA;
  double bt[kRB], at[kRA], yh[kRA];
  // M <= 16 class (plant_packed): lane (e, k) holds numerator tap k and denominator a_(k+1) of
  // entry e; the output history stays in LDS, a step is one row4_sum over the four taps.  It holds
  // 4 instead of 24 plant VGPRs, which the register QP (gpc_qp16.h) needs for three waves per SIMD
  const int ktap = lane >> 4;
  if constexpr (MAXM <= 16) {
    bt[0] = (is_entry && ktap < e_nb - e_off) ? eb[e_off + ktap] : 0.0;
    at[0] = (is_entry && ktap + 1 < e_na) ? ea[ktap + 1] : 0.0;
    yh[0] = 0.0;
  } else {
#pragma unroll
    for (int k = 0; k < kRegB; ++k) bt[k] = (is_entry && k < e_nb - e_off) ? eb[e_off + k] : 0.0;
#pragma unroll
    for (int k = 0; k < kRegA; ++k) {
      at[k] = (is_entry && k + 1 < e_na) ? ea[k + 1] : 0.0;
      yh[k] = 0.0;
    }
  }
  const bool regpath = MAXM > 16 && sc.regpath != 0;
  // prefetched per-output signals
  double r_t = 0.0, yr_t = 0.0;
  if (lane < my) {
    r_t = rr[lane * nit];
    yr_t = sc.yref[lane * nit];
  }
  // u(t) = u(t-1) + du(t, first move) of MV n = lane: past-control state, plant input ring
  auto u_update = [&](int t, int ln) __attribute__((always_inline)) {
    if (ln < nu) {
      const int n = lane;
      const double du = sxc[n * Nu];
      const double un = suprev[n] + du;
      // past-control register shifted in LDS (kept in VGPRs it measured slower: register pressure)
      for (int k = dum_n - 1; k > 0; --k) sx[upoff_n + k] = sx[upoff_n + k - 1];
      sx[upoff_n] = du;
      sur[n * kURing + (t & (kURing - 1))] = un;
      if ((EXT && o.want_traj)) {
        if (out.u) out.u[(sim * nu + n) * nit + t] = un;
        if ((EXT && o.open_loop) && out.uopt) {
          const int l = t < Nu - 1 ? t : Nu - 1;
          // Info.Uopt has p+1 rows then the padding repeats the last row (:94-98)
          out.uopt[(sim * nu + n) * nit + t] = sucum[n * Nu + l];
        }
      }
      suprev[n] = un;
    }
  };
  // the per-lane constants and r(0), Yref(0) loaded above are waited for here, once.  Left
  // pending, their first use inside the step loop got an s_waitcnt vmcnt on every step (the
  // compiler's wait is placed at the use, inside the loop), which also waited for that step's
  // signal prefetch: its L2 latency was exposed every step
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  for (int t = 0; t < nit; ++t) {
    // the lane predicates of the step are re-derived from an opaque copy of the lane id every
    // step: hoisted out of the loop they are kept as SGPR-pair exec masks, which the kernel's
    // SGPR budget spills to VGPR lanes and reloads (v_readlane) several times per step
    int ln = lane;
    asm volatile("" : "+v"(ln));
    // inputs at time t that are already known: MDs v(t); open-loop uopt(t)
    if (sc.nd > 0) {
      for (int e = lane; e < ncopy * sc.nd; e += kWave) {
        const int cpy = e / sc.nd, j = e - cpy * sc.nd;
        sur[(cpy * nin + nu + j) * kURing + (t & (kURing - 1))] = vvk[j * nit + t];
      }
    }
    if ((EXT && o.open_loop) && lane < nu) {
      const int l = t < Nu - 1 ? t : Nu - 1;
      sur[(nin + lane) * kURing + (t & (kURing - 1))] = sucum[lane * Nu + l];
    }
    lds_sync();
    // plant entries y_e(t) (copy 0: closed loop, copy 1: open loop driven by uopt)
    if (plant_packed) {
      // tap k of every entry on row block k (histories are zero before t = 0: no bound tests)
      double pr = 0.0;
      if (is_entry) pr = bt[0] * eur[(t - e_off - ktap) & (kURing - 1)] - at[0] * eyh[(t - 1 - ktap) & (kYeHist - 1)];
      const double acc = row4_sum(pr);
      if (lane < ncopy * ne) {
        eyh[t & (kYeHist - 1)] = acc;
        sye[lane] = acc;
      }
    } else if (ln < ncopy * ne) {
      // histories are zero before t = 0, so no t - l >= 0 test: loads issue back to back
      // only the nonzero taps (the delay's leading zeros are skipped: pl_off)
      double acc;
      if (regpath) {
        double a0 = 0.0, a1 = 0.0;
#pragma unroll
        for (int k = 0; k < kRB; ++k) a0 += bt[k] * eur[(t - e_off - k) & (kURing - 1)];
#pragma unroll
        for (int k = 0; k < kRA; ++k) a1 -= at[k] * yh[k];
        acc = a0 + a1;
#pragma unroll
        for (int k = kRA - 1; k > 0; --k) yh[k] = yh[k - 1];
        yh[0] = acc;
      } else {
        double a0 = 0.0, a1 = 0.0;
        for (int l = e_off; l < e_nb; ++l) a0 += eb[l] * eur[(t - l) & (kURing - 1)];
        for (int l = 1; l < e_na; ++l) a1 -= ea[l] * eyh[(t - l) & (kYeHist - 1)];
        acc = a0 + a1;
        eyh[t & (kYeHist - 1)] = acc;
      }
      sye[lane] = acc;
    }
    lds_sync();
    PSTAMP(PROF_PLANT);
    if constexpr (DTC) {
      // predictor model entries on the controller's own input history (OptimalPredictor2.m:
      // lsim(Pz, u) and lsim(Gz, u) kept as recursions): lanes e < my*nu are Pz, the next my*nu Gz
      const int nmz = 2 * my * nu;
      if (lane < nmz) {
        const int j = lane % nu;
        const double* mb = lds + L.mzb + lane * sc.mz_maxb;
        const double* ma = lds + L.mza + lane * sc.mz_maxa;
        double* mh = lds + L.mzh + lane * kYeHist;
        const double* ur = sur + j * kURing;  // closed-loop input ring of MV j
        const int mnb = sc.mz_nb[lane], mna = sc.mz_na[lane], moff = sc.mz_off[lane];
        double a0 = 0.0, a1 = 0.0;
        for (int l = moff; l < mnb; ++l) a0 += mb[l] * ur[(t - l) & (kURing - 1)];
        for (int l = 1; l < mna; ++l) a1 -= ma[l] * mh[(t - l) & (kYeHist - 1)];
        const double am = a0 + a1;
        mh[t & (kYeHist - 1)] = am;
        lds[L.smz + lane] = am;
      }
      lds_sync();
    }
    if (ln < my) {
      const int i = lane;
      double y = 0.0;
      for (int j = 0; j < nin; ++j) y += sye[i * nin + j];
      // the measurement driving the free response: y, or the DTC predictor output
      // yp = Gz*u + Fr*(y - Pz*u)  (OptimalPredictor2.m:24-40, DTC_GPC_WW.m:133-142)
      double ym = y;
      if constexpr (DTC) {
        double ypz = 0.0, ygz = 0.0;
        for (int j = 0; j < nu; ++j) {
          ypz += lds[L.smz + i * nu + j];
          ygz += lds[L.smz + my * nu + i * nu + j];
        }
        double* eh = lds + L.frh + i * 2 * kYeHist;  // eM history, then yfr history
        double* fh = eh + kYeHist;
        const double* fb = lds + L.frb + i * sc.fr_max;
        const double* fa = lds + L.fra + i * sc.fr_max;
        eh[t & (kYeHist - 1)] = y - ypz;
        double yfr = 0.0;
        const int nf = sc.fr_n[i];
        for (int l = 0; l < nf; ++l) yfr += fb[l] * eh[(t - l) & (kYeHist - 1)];
        for (int l = 1; l < nf; ++l) yfr -= fa[l] * fh[(t - l) & (kYeHist - 1)];
        fh[t & (kYeHist - 1)] = yfr;
        ym = ygz + yfr;
      }
      // state: [y - r, nabla y, ..., nabla^na y]; nabla^k y(t) = nabla^{k-1} y(t) - nabla^{k-1} y(t-1)
      // backward differences shifted in LDS (kept in VGPRs they measured slower)
      double cur = ym, prev = syprev[i];
      for (int k = 1; k < nyh_i; ++k) {
        const double old = sx[yoff_i + k];
        const double nk = cur - prev;
        sx[yoff_i + k] = nk;
        cur = nk;
        prev = old;
      }
      syprev[i] = ym;
      sx[yoff_i] = ym - r_t;
      const double e1 = y - yr_t;
      j1 += e1 * e1;
      if (t >= sc.ink0) j22 += e1 * e1;
      double ysv = 0.0;
      if ((EXT && o.open_loop)) {
        for (int j = 0; j < nin; ++j) ysv += sye[ne + i * nin + j];
        if (t >= sc.ink0) j21 += (y - ysv) * (y - ysv);
      }
      if ((EXT && o.want_traj)) {
        if (out.y) out.y[(sim * my + i) * nit + t] = y;
        if ((EXT && o.open_loop) && out.ys) out.ys[(sim * my + i) * nit + t] = ysv;
      }
    }
    // prefetch r(t+1), Yref(t+1) (every lane loads, clamped address): issued after this step's
    // last use of r(t), Yref(t), so the compiler's wait for them lands in the next step's y update,
    // a whole step after the loads left
    double r_n, yr_n;
    {
      const int tn = t + 1 < nit ? t + 1 : t;
      const int si = lane < my ? lane : my - 1;
      r_n = rr[si * nit + tn];
      yr_n = sc.yref[si * nit + tn];
    }
    lds_sync();
    PSTAMP(PROF_YUPD);
    solve_step();
    u_update(t, ln);
    lds_sync();
    r_t = r_n;
    yr_t = yr_n;
    PSTAMP(PROF_UUPD);
  }
#ifdef MPCT_PROFILE
  if (lane == 0 && out.prof)
    for (int k = 0; k < PROF_N; ++k) out.prof[sim * PROF_N + k] = pacc.get(k);
#endif
#ifdef MPCT_TIMELINE
  if (lane == 0 && out.prof) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID: wave, SIMD, CU, SE
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    unsigned long long* tl = out.prof + slot * 4;
    tl[0] = tl_t0;
    tl[1] = __builtin_amdgcn_s_memrealtime();
    tl[2] = ((unsigned long long)hw << 32) | xcc;
    tl[3] = (unsigned long long)sim;
  }
#endif

  // ------------------------------------------------------------------ results
  if (lane < my && !isfinite(j1)) st |= MPCT_ST_NONFINITE_;
  const unsigned long long nf = __ballot(st & MPCT_ST_NONFINITE_);
  put(j1, (EXT && o.open_loop) ? j21 : NAN, j22, (EXT && o.open_loop) ? jnu : NAN,
      st | (nf ? MPCT_ST_NONFINITE_ : 0), iters);
}

}  // namespace mpct

// ------------------------------------------------------------------------------------------
// host-side launch
#include <string>

#include "work_order.h"
#include "launch_fan.h"

namespace mpct {

long long small_lds_bytes(const DevScenario& sc, int M);  // gpc_small.hip
int launch_small(const DevScenario& sc, long long C, int nref, const int* N2, const int* Nu, const double* delta,
                 const double* lambda, const double* r, const DevOpts& o, const DevResult& out, const int* perm,
                 int first, hipStream_t stream, std::string* err);
long long dtc_small_lds_bytes(const DevScenario& sc, int M);  // dtc_small.hip
int launch_dtc_small(const DevScenario& sc, int cls, long long C, int nref, const int* N2, const int* Nu,
                     const double* delta, const double* lambda, const double* r, const double* v, const DevOpts& o,
                     const DevResult& out, const int* perm, int mlo, int first, hipStream_t stream, std::string* err);

long long lds_bytes_for(const DevScenario& sc, int N2, int Nu, bool ext) {
  (void)N2;
  const int M = sc.nu * Nu;
  if (sc.small && !ext && M <= 16) return small_lds_bytes(sc, M);
  if (sc.small_dtc && !ext && M <= 32) return dtc_small_lds_bytes(sc, M);
  LdsLayout L = lds_layout(sc, M, ext);
  return (long long)L.total * 8;
}

// one QP-size class launch over the whole batch: simulations with mlo < M <= MAXM run here (first:
// this launch also writes the statuses of skipped / bad-horizon candidates)
template <int MAXM>
static int launch_t(const DevScenario& sc, long long C, int nref, const int* N2, const int* Nu,
                    const double* delta, const double* lambda, const double* r, const double* v,
                    const DevOpts& o, const DevResult& out, const int* perm, int mlo, int first,
                    hipStream_t stream, std::string* err) {
  const int nu_cls = sc.numax < MAXM / sc.nu ? sc.numax : MAXM / sc.nu;  // largest Nu of this class
  const bool ext = o.open_loop || o.want_traj;
  const long long lds = lds_bytes_for(sc, sc.n2max, nu_cls, ext);
  if (lds > 160 * 1024) {
    *err = "scenario needs more than 160 KiB of LDS per simulation";
    return -4;
  }
  auto kern = sc.dtc ? (ext ? gpc_closed_loop_kernel<MAXM, true, true> : gpc_closed_loop_kernel<MAXM, true, false>)
                     : (ext ? gpc_closed_loop_kernel<MAXM, false, true> : gpc_closed_loop_kernel<MAXM, false, false>);
  if (lds > 64 * 1024) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
      *err = "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed";
      return -3;
    }
  }
  const long long S = C * nref;
  hipLaunchKernelGGL(kern, dim3((unsigned)S), dim3(kWave), (size_t)lds, stream, sc, C, nref, N2, Nu,
                     delta, lambda, r, v, perm, o, out, mlo, first);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    *err = std::string("kernel launch failed: ") + hipGetErrorString(e);
    return -3;
  }
  return 0;
}

// QP-size classes a scenario launches: <16> for M <= 16, then <32>, <64> up to nu * nu_max (a
// batch with mixed Nu runs each simulation in the smallest class that holds it: the <16> instance
// has DPP reductions over one row and three waves per SIMD)
static int top_class(int maxM) { return maxM <= 16 ? 16 : maxM <= 32 ? 32 : 64; }

// the instance(s) launch_closed_loop picks (mpct_kernel_instance): QP size classes, DTC, EXT
std::string closed_loop_instance(const DevScenario& sc, int maxM, bool ext) {
  const std::string tail = std::string(sc.dtc ? ",true" : ",false") + (ext ? ",true>" : ",false>");
  std::string nm;
  for (int cls = 16; cls <= top_class(maxM); cls *= 2) {
    if (sc.nu > cls) continue;
    if (cls == 16 && sc.small && !ext) {
      nm = "gpc_small_kernel";
      continue;
    }
    if (cls <= 32 && sc.small_dtc && !ext) {
      nm += (nm.empty() ? "" : " + ") + std::string("dtc_small_kernel<") + std::to_string(cls) + ">";
      continue;
    }
    if (nm.empty()) nm = "gpc_closed_loop_kernel<" + std::to_string(cls) + tail;
    else if (nm.find("gpc_closed_loop_kernel") == std::string::npos)
      nm += " + gpc_closed_loop_kernel<" + std::to_string(cls) + tail;
    else nm += " + <" + std::to_string(cls) + tail;
  }
  return nm;
}

int launch_closed_loop(const DevScenario& sc, long long C, int nref, const int* N2, const int* Nu,
                       const double* delta, const double* lambda, const double* r,
                       const double* v, const DevOpts& o, const DevResult& out, int maxM,
                       WorkOrder* wo, LaunchFan* fan, hipStream_t stream, std::string* err) {
  if (maxM > 64) {
    *err = "nu*nu_max > 64";
    return -4;
  }
  // ordered launches stage their cost records XCD-major and gather them into the caller's order
  // afterwards (DevResult::stage): full-line writes instead of 24-B pieces from every L2.  The
  // staging rows are laid out before the dispatch-order key, whose launch prefills them
  const int* perm = nullptr;
  DevResult lo = out;
  bool prefilled = false;
  if (wo) {
    if (C >= kOrderMinC) {
      lo.srow = stage_row(out, sc.my, sc.nu);
      const int rs = lo.srow.w ? order_stage(*wo, C * nref, lo.srow.w, &lo.stage, err) : 0;
      if (rs) return rs;
    }
    const int rc = order_candidates(kOrderGpc, sc.my, sc.nu, C, N2, Nu, delta, lambda, *wo, &perm, stream, err,
                                    &sc, nref, r, &lo, &prefilled);
    if (rc) return rc;
  }
  if (!perm) {
    lo = out;
    prefilled = false;
  }
  int rc = prefilled ? 0 : prefill_results(lo, C * nref, sc.my, sc.nu, stream, err);
  if (rc) return rc;
  FanScope fs(top_class(maxM) > 16 ? fan : nullptr, stream);
  int k = 0, mlo = 0;
  for (int cls = 16; cls <= top_class(maxM) && rc == 0; cls *= 2) {
    if (sc.nu > cls) {  // no simulation fits this class
      mlo = cls;
      continue;
    }
    const hipStream_t st = fs.stream(k);
    const int first = k == 0;
    const bool ext = o.open_loop || o.want_traj;
    if (diag_drop_launch(k)) rc = 0;
    else if (cls == 16 && sc.small && !ext) rc = launch_small(sc, C, nref, N2, Nu, delta, lambda, r, o, lo, perm, first, st, err);
    else if (cls <= 32 && sc.small_dtc && !ext)
      rc = launch_dtc_small(sc, cls, C, nref, N2, Nu, delta, lambda, r, v, o, lo, perm, mlo, first, st, err);
    else if (cls == 16) rc = launch_t<16>(sc, C, nref, N2, Nu, delta, lambda, r, v, o, lo, perm, mlo, first, st, err);
    else if (cls == 32) rc = launch_t<32>(sc, C, nref, N2, Nu, delta, lambda, r, v, o, lo, perm, mlo, first, st, err);
    else rc = launch_t<64>(sc, C, nref, N2, Nu, delta, lambda, r, v, o, lo, perm, mlo, first, st, err);
    mlo = cls;
    ++k;
  }
  fs.join();
  if (rc == 0 && lo.stage) rc = unpermute_results(*wo, C, nref, sc.my, sc.nu, lo.srow, out, stream, err);
  if (perm) order_mark_used(*wo, stream);
  return rc;
}

}  // namespace mpct
