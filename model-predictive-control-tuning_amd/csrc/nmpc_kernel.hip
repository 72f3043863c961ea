// nmpc_kernel.hip — batched closed loop of the nonlinear MPC of VanDeVusse_NMPC.m (config 5), one
// wavefront (64 lanes) per simulation.
//
// Replaces, per simulation, closedloop_toolbox_nmpc.m:36-97: nlmpcmove at every step of an
// nit-step closed loop on the Van de Vusse reactor (nmpc_vandevusse_state.m:64-82), plus the
// open-loop prediction from (x0, u0) at r(:,end).  The closed-source parts are replaced as in
// oracle/nmpc_vdv.py: one fixed-step RK4 (nsub sub-steps per Ts) for plant and
// prediction; nlmpc's fmincon SQP by single-shooting Gauss-Newton SQP on the documented standard
// cost  sum (w_y/s_y)^2 (y - r)^2 + sum (w_du/s_u)^2 du^2  with hard MV bounds.
//
// Device formulation: decision variables are the move increments v = dU (lane m = n*Nu + l),
// so the rate term is diagonal and the MV bounds are gi_core's box rows (kind 0/1 at l = 0,
// cumulative kind 2/3 at l > 0).  Each Gauss-Newton iteration:
//   * lanes integrate the prediction x(k+1..k+N) redundantly and carry their own tangent
//     dx/dv_m through the RK4 stages (forward-mode sensitivities, exact for the RK4 map);
//   * every predicted output row (w_y dy/dv | w_y (y - r)) is streamed into a row-wise Givens QR
//     of the least-squares Jacobian as soon as it is produced (lanes = columns, lane M = the
//     residual column): no Jacobian is stored, and the QP never sees normal equations (the rate
//     weights span 1e-11..1 against the output rows' 1e2: cond(H) ~ 1e15, cond(R) ~ 3e7);
//   * the step solves the box QP with the Goldfarb-Idnani dual method of gi_core.h (J = R^-1);
//   * v += step (Armijo backtracking), or the Anderson-accelerated point (depth 1: a secant on the
//     last two Gauss-Newton points) when it meets the same decrease; stop when the largest
//     absolute-move change of the full step / s_u <= sqp_tol (the oracle's test).
#include <hip/hip_runtime.h>
#include <math.h>

#include "gi_core.h"
#include "launch_fan.h"
#include "mpct_dev.h"
#include "nmpc_model.h"

namespace mpct {

// lane groups of the multi-point prediction pass: the M <= 15 class runs up to four
// points of one controller call at once, one per 16-lane DPP row (the pass is bound by the FP64
// issue of one wave, not by its lanes); the M <= 32 class runs one (two points on 32-lane halves
// were measured slower: the half broadcasts cost more than the shared passes save)
template <int MAXM>
constexpr int kNmRows = MAXM <= 16 ? 4 : 1;

// active flags: box rows (p < base) in the lanes' act bits, state-bound rows in an LDS bitmap
struct StateMark {
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

// one wave per SIMD (342 VGPRs): capped at 2 or 3 waves the kernel spills and config 5 ran 27 %
// slower (profiles/r02i_nmpc_code_size.txt)
template <int MAXM>
__global__ void __launch_bounds__(64, 1)
    nmpc_closed_loop_kernel(const DevScenario sc, long long C, int nref, const int* __restrict__ Nv,
                            const int* __restrict__ Nuv, const double* __restrict__ deltav,
                            const double* __restrict__ lambdav, const double* __restrict__ rv,
                            const int* __restrict__ perm, const DevOpts o,
                            const DevResult out, int mz_lo, long long lds_lo, long long lds_hi, int first_) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x;
  // workgroup slot -> candidate (heaviest estimated work first, work_order.h) or identity
  const long long slot = blockIdx.x;
  if (slot >= C * nref) return;
  const long long cs = slot / nref;
  const int kref = (int)(slot - cs * nref);
  const long long c = perm ? (long long)perm[cs] : cs;
  const long long sim = c * nref + kref;
  const int ny = sc.my, nu = sc.nu, nit = sc.nit;
  const int N = Nv[c], Nu = Nuv[c];
  const int M = nu * Nu;
  int st = 0;
#ifdef MPCT_PROFILE
  // diagnostic build: section cycle sums (tools/nmpc_latency.py --profile; labels: mpct_host.cpp)
  ProfAccS pacc;
  unsigned long long pprev = __builtin_amdgcn_s_memtime();
#endif

  auto write_nan = [&](int status) __attribute__((always_inline)) {
    if (lane < ny) {
      if (out.J1) out.J1[sim * ny + lane] = NAN;
      if (out.j21) out.j21[sim * ny + lane] = NAN;
      if (out.j22) out.j22[sim * ny + lane] = NAN;
    }
    if (lane < nu && out.Jnu) out.Jnu[sim * nu + lane] = NAN;
    if (lane == 0) {
      if (out.status) out.status[sim] = status;
      if (out.qp_iters) out.qp_iters[sim] = 0;
    }
  };
  const bool first = first_ != 0;
  if (N <= 0) {
    if (first) write_nan(MPCT_ST_SKIPPED_);
    return;
  }
  if (N > sc.n2max || Nu < 1 || Nu > sc.numax || Nu > N) {
    if (first) write_nan(MPCT_ST_BADHORIZON_);
    return;
  }
  // another launch's QP size class: the M <= 15 class holds M + 1 lanes in one 16-lane row
  if (M <= mz_lo || M > (kNmRows<MAXM> > 1 ? 15 : MAXM)) return;
  const int G = kNmRows<MAXM> > 1 ? nm_groups(M, N) : 1;  // point buffers (uniform)
  const NmLayout L = nm_layout(M, N, G);
  if ((long long)L.total * 8 <= lds_lo || (long long)L.total * 8 > lds_hi) return;  // another LDS tier
  double* sRi = lds + L.ri;
  double* sJT = lds + L.jt;
  double* sRA = lds + L.ra;
  double* sd = lds + L.dv;
  double* sxc = lds + L.xc;
  double* sUo = lds + L.uo;
  double* snv = lds + L.nv;
  unsigned* sbits = reinterpret_cast<unsigned*>(lds + L.bits);
  // point buffer g, and the current point's pieces (the factorisation the QP uses)
  auto gbuf = [&](int g) __attribute__((always_inline)) -> double* { return lds + L.grp + g * L.gsz; };
  double *sR, *scv, *sU, *sxp, *ssx;
  auto setcur = [&](int g) __attribute__((always_inline)) {
    double* b = gbuf(g);
    sR = b + L.g_rr;
    scv = b + L.g_cv;
    sU = b + L.g_u;
    sxp = b + L.g_xp;
    ssx = b + L.g_sx;
  };
  setcur(0);

  const double* tab = sc.nm;  // [params][x0 3][u0 nu][lb nu][ub nu][xmin 3][xmax 3][sy ny][su nu]
  const VdV P = vdv_load(tab);
  const double* tx0 = tab + NM_NPAR;
  const double* tu0 = tx0 + 3;
  const double* tlb = tu0 + nu;
  const double* tub = tlb + nu;
  const double* txmin = tub + nu;
  const double* txmax = txmin + 3;
  const double* tsy = txmax + 3;
  const double* tsu = tsy + ny;
  const double h = sc.ts / sc.nsub;
  const int nsub = sc.nsub;

  const bool row = lane < M;
  const int bn = row ? lane / Nu : 0;     // MV of this lane's move
  const int bl = row ? lane - bn * Nu : 0;  // move index within the block
  const double lbn = tlb[bn], ubn = tub[bn], sun = tsu[bn];
  // toolbox weights over ScaleFactors, squared in the cost: residual rows carry w = |weight|/s
  const double* dl = deltav + c * ny;
  const double* lm = lambdav + c * nu;
  const double wu = fabs(lm[bn]) / sun;
  // the lane's place in the multi-point pass: 16-lane row grp, lane gl of the row (the whole
  // wave in the M <= 32 class); lanes gl < M carry tangent columns, gl = M the residual column
  constexpr int R4 = kNmRows<MAXM>;
  const int grp = R4 > 1 ? lane >> 4 : 0;
  const int gl = R4 > 1 ? lane & 15 : lane;
  const bool prow = gl < M;
  const int pbn = prow ? gl / Nu : 0, pbl = prow ? gl - pbn * Nu : 0;
  const double pwu = fabs(lm[pbn]) / tsu[pbn];
  int xc0 = sc.xc[0], xc1 = ny > 1 ? sc.xc[1] : 0;
  const double wy0 = fabs(dl[0]) / tsy[0], wy1 = ny > 1 ? fabs(dl[1]) / tsy[1] : 0.0;
  const double tol = o.feas_tol;
  const int maxit = o.max_qp_iter > 0 ? o.max_qp_iter : 200 * M + 1000;
  const double* rr = rv + (long long)kref * ny * nit;
  long long sqp_total = 0;

  // hard state bounds (VanDeVusse_NMPC.m:143-146), linearised along the prediction
  bool has_xb = false;
  for (int i = 0; i < 3; ++i) has_xb = has_xb || isfinite(txmin[i]) || isfinite(txmax[i]);
  const int nbits = (6 * N + 31) / 32;
  // d = J'n_p: box rows from gi_core's structure, state-bound rows from their staged normal
  auto dvec = [&](int p) __attribute__((always_inline)) -> double {
    if (p < 4 * M) {
      const CInfo ci = cinfo(p, Nu);
      return gi_dvec<MAXM>(sJT, sd, M, ci.j0, ci.j1, ci.sg, row);
    }
    const int q = p - 4 * M, r = q >> 1;
    if (row) snv[lane] = (q & 1) ? -ssx[r * M + lane] : ssx[r * M + lane];
    lds_sync();
    double dk = 0.0;
    if (row) {
      const double* jc = sJT + lane * M;
      for (int i = 0; i < M; ++i) dk += jc[i] * snv[i];
      sd[lane] = dk;
    }
    return dk;
  };

  // ---- one controller call (nlmpcmove restated): Gauss-Newton SQP from the warm start v
  // (this lane's increment), state x, last move ul[n], reference (r0, r1).  Returns v.
  // Speculation: a pass at a point this call may return also runs the next
  // calls' first passes from it, assuming each of them returns its warm start at once.  hq[0] >= 0:
  // point buffer hq[0] already holds this call's pass at v (speculated earlier), hq[1], hq[2] the
  // following calls' (-1: none), hqf their costs.  t: this call's closed-loop step, nf: the
  // future steps a speculation may reach (0..3).  sq / sqf: the chain for the returned point.
  auto controller = [&](const double x[3], const double ul[2], double r0, double r1, double v, const int* hq,
                        const double* hqf, int t, int nf, int* sq, double* sqf)
                        __attribute__((always_inline)) -> double {
    const double ulb = bn == 0 ? ul[0] : ul[1];
    // cost f(v') of increments v' by a tangent-free forward pass; xin: every predicted state
    // inside the hard state bounds
    auto trial = [&](double va, bool& xin) __attribute__((always_inline)) -> double {
      lds_sync();
      if (row) sxc[lane] = va;
      lds_sync();
      if (row) {
        double cum = 0.0;
        for (int j = lane - bl; j <= lane; ++j) cum += sxc[j];
        sU[lane] = ulb + cum;
      }
      lds_sync();
      double xa[3] = {x[0], x[1], x[2]};
      double fa = 0.0;
      bool inb = true;
      for (int i = 0; i < N; ++i) {
        const int li = i < Nu - 1 ? i : Nu - 1;
        const double u[2] = {sU[li], nu > 1 ? sU[Nu + li] : 0.0};
        vdv_rk4<false>(P, h, nsub, xa, u, nullptr, nullptr);
        const double e0 = wy0 * (sel3(xa, xc0) - r0);
        fa += e0 * e0;
        if (ny > 1) {
          const double e1 = wy1 * (sel3(xa, xc1) - r1);
          fa += e1 * e1;
        }
        if (has_xb)
          for (int s = 0; s < 3; ++s) inb = inb && xa[s] >= txmin[s] && xa[s] <= txmax[s];
      }
      xin = inb;
      return 0.5 * (fa + qsum<MAXM>(row ? (wu * va) * (wu * va) : 0.0));
    };
    // Anderson acceleration (depth 1) of the Gauss-Newton map v -> G(v) = v + d(v): the previous
    // iteration's absolute-move step (aa_f, this lane's entry) and G (aa_g, increments)
    bool aa_hist = false;
    double aa_f = 0.0, aa_g = 0.0;
    // the prediction with forward tangents at the points whose increments the caller wrote into
    // the point buffers, streamed into each point's Givens QR of the least-squares Jacobian
    // [rate rows; output rows] (R and c = Q'r), its linearised state rows and its cost.  Point g
    // runs on 16-lane row g (the whole wave in the M <= 32 class): the pass is bound by one wave's
    // FP64 issue, so up to four points cost what one does.  A point with bit g of `spec` set is
    // depth d_g = bits 2g..2g+1 of `dep` > 0 is the first point of the call d_g steps ahead from
    // point g's increments, each call between returning its warm start at once: d_g plant steps
    // with the first moves of the shifted increments, the increments shifted d_g moves (the closed
    // loop's own update), that step's reference.  fg[g]: the cost f, xg[g]: every predicted state
    // inside the hard bounds.
    auto mpass = [&](unsigned dep, double* fg, bool* xg) __attribute__((always_inline)) {
      lds_sync();  // the caller's increments
      const bool gact = grp < G;  // rows without a buffer recompute point 0 and write nothing
      double* gb = gbuf(gact ? grp : 0);
      double* gv = gb + L.g_v;
      double xs[3] = {x[0], x[1], x[2]};
      double ug0 = ul[0], ug1 = ul[1], gr0 = r0, gr1 = r1;
      double va = prow ? gv[gl] : 0.0;
      if (dep) {
        const int dg = gact ? (int)((dep >> (2 * grp)) & 3u) : 0;
        int dm = 0;
        for (int g = 0; g < 4; ++g) dm = max(dm, (int)((dep >> (2 * g)) & 3u));
        for (int j = 1; j <= dm; ++j) {
          // step j's applied moves: ul_(j-1) + the first moves of the increments shifted j - 1 times
          const double m0 = j - 1 < Nu ? gv[j - 1] : 0.0;
          const double m1 = nu > 1 && j - 1 < Nu ? gv[Nu + j - 1] : 0.0;
          const double u1[2] = {ug0 + m0, nu > 1 ? ug1 + m1 : 0.0};
          double xn[3] = {xs[0], xs[1], xs[2]};
          vdv_rk4<false>(P, h, nsub, xn, u1, nullptr, nullptr);
          if (j <= dg) {
            xs[0] = xn[0];
            xs[1] = xn[1];
            xs[2] = xn[2];
            ug0 = u1[0];
            ug1 = u1[1];
          }
        }
        if (dg > 0) {
          gr0 = rr[t + dg];
          gr1 = ny > 1 ? rr[nit + t + dg] : 0.0;
          va = (prow && pbl + dg < Nu) ? gv[gl + dg] : 0.0;
        }
        lds_sync();
        if (gact && prow) gv[gl] = va;
      }
      lds_sync();
      // absolute moves of the point: U[n][l] = ul[n] + sum_{l' <= l} v[n][l']
      double* gU = gb + L.g_u;
      double* grw = gb + L.g_rw;
      if (gact && prow) {
        double cum = 0.0;
        for (int j = gl - pbl; j <= gl; ++j) cum += gv[j];
        gU[gl] = (pbn == 0 ? ug0 : ug1) + cum;
        grw[gl] = pwu * va;
      }
      lds_sync();
      double rcol[MAXM];
#pragma unroll
      for (int k = 0; k < MAXM; ++k) {
        double e = 0.0;
        if (k < M) {
          if (gl == k) e = pwu;
          else if (gl == M) e = grw[k];  // rate residual w_u v_k
        }
        rcol[k] = e;
      }
      double* gxp = gb + L.g_xp;
      double* gsx = gb + L.g_sx;
      double td[3] = {0.0, 0.0, 0.0};
      double fo = 0.0;  // sum of squared output residuals (lane gl = M)
      bool inb = true;
      for (int i = 0; i < N; ++i) {
        const int li = i < Nu - 1 ? i : Nu - 1;
        const double u[2] = {gU[li], nu > 1 ? gU[Nu + li] : 0.0};
        double ud[2] = {0.0, 0.0};
        if (prow && pbl <= li) ud[pbn] = 1.0;
        vdv_rk4<true>(P, h, nsub, xs, u, td, ud);
        if (has_xb) {
          if (gact && prow) {
            gsx[(i * 3 + 0) * M + gl] = td[0];
            gsx[(i * 3 + 1) * M + gl] = td[1];
            gsx[(i * 3 + 2) * M + gl] = td[2];
          } else if (gact && gl == M) {
            gxp[i * 3 + 0] = xs[0];
            gxp[i * 3 + 1] = xs[1];
            gxp[i * 3 + 2] = xs[2];
          }
          for (int s3 = 0; s3 < 3; ++s3) inb = inb && xs[s3] >= txmin[s3] && xs[s3] <= txmax[s3];
        }
        for (int j = 0; j < ny; ++j) {
          const int xj = j == 0 ? xc0 : xc1;
          const double wy = j == 0 ? wy0 : wy1;
          if (!(wy > 0.0)) continue;
          double w = 0.0;
          if (prow) w = wy * sel3(td, xj);
          else if (gl == M) w = wy * (sel3(xs, xj) - (j == 0 ? gr0 : gr1));
          fo += w * w;
#pragma unroll
          for (int k = 0; k < MAXM; ++k) {
            if (k < M) {
              // the row's column-k entries: lane k of each 16-lane row (DPP row_newbcast), or of
              // the wave
              const double b = R4 > 1 ? row_bcast16(w, k) : bcast(w, k);
              const double a = R4 > 1 ? row_bcast16(rcol[k], k) : bcast(rcol[k], k);
              // 1/rho by v_rsq_f64 and two Newton steps (a divide-free chain, as gpc_kernel's QR)
              const double xx = a * a + b * b;
              double ri = __builtin_amdgcn_rsq(xx);
              const double hx = 0.5 * xx;
              ri = ri * fma(-hx * ri, ri, 1.5);
              ri = ri * fma(-hx * ri, ri, 1.5);
              const bool nz = b != 0.0;
              const double cs = nz ? a * ri : 1.0, sn = nz ? b * ri : 0.0;
              const double rk = rcol[k];
              rcol[k] = cs * rk + sn * w;
              w = -sn * rk + cs * w;
            }
          }
        }
      }
      // R (upper, lane j holds column j) and c = Q'r (lane M) -> the point's buffer
      if (gact && (prow || gl == M)) {
        double* gR = gb + L.g_rr;
        double* gc = gb + L.g_cv;
#pragma unroll
        for (int k = 0; k < MAXM; ++k)
          if (k < M) {
            if (prow) {
              if (k <= gl) gR[nm_up(k, gl, M)] = rcol[k];
            } else {
              gc[k] = rcol[k];
            }
          }
      }
      const double rv2 = prow ? (pwu * va) * (pwu * va) : 0.0;
      const double rs = R4 > 1 ? row_sum(rv2) : qsum<MAXM>(rv2);
      for (int g = 0; g < G; ++g) {
        fg[g] = 0.5 * (bcast(fo, 16 * g + M) + bcast(rs, 16 * g));
        xg[g] = __builtin_amdgcn_readlane((int)inb, 16 * g) != 0;
      }
    };
    // point g's increments (lanes < M hold them) -> its buffer
    auto put = [&](int g, double val) __attribute__((always_inline)) {
      if (row) gbuf(g)[L.g_v + lane] = val;
    };
    // cur: buffer of the pass at v (-1: none yet); ch[0..2]: the buffers of the next calls'
    // passes from v (-1: none), chf their costs
    int cur = hq[0], ch[3] = {hq[1], hq[2], -1};
    double fcur = hqf[0], chf[3] = {hqf[1], hqf[2], 0.0};
    double fg[4] = {0.0, 0.0, 0.0, 0.0};
    bool xg[4] = {true, true, true, true};
    for (int k = 0; k < 3; ++k) {
      sq[k] = -1;
      sqf[k] = 0.0;
    }
    // one point's pass on every buffer: the point, then the next calls' first points (G = 4:
    // three, G = 2: one), as far as the closed loop reaches
    const int ndep = min(nf, G - 1);
    const unsigned dchain = (ndep >= 1 ? 0x4u : 0u) | (ndep >= 2 ? 0x20u : 0u) | (ndep >= 3 ? 0xC0u : 0u);
    auto chain_of_solo = [&]() __attribute__((always_inline)) {
      for (int k = 0; k < 3; ++k) {
        ch[k] = k < ndep ? k + 1 : -1;
        chf[k] = k < ndep ? fg[k + 1] : 0.0;
      }
    };
#ifdef MPCT_PROFILE
    if (cur >= 0) pacc[PROF_NM_USED] += kProfCount;  // a speculated first point, ready
#define NM_COUNT_PASS(pts)                                         \
  do {                                                             \
    pacc[PROF_NM_NPASS] += kProfCount;                             \
    pacc[PROF_NM_POINTS] += (unsigned long long)(pts) * kProfCount; \
    pacc[PROF_NM_ROWS] += (unsigned long long)G * kProfCount;      \
  } while (0)
#define NM_COUNT_USED() pacc[PROF_NM_USED] += kProfCount
#else
#define NM_COUNT_PASS(pts) \
  do {                     \
  } while (0)
#define NM_COUNT_USED() \
  do {                  \
  } while (0)
#endif
    for (int it = 0; it < sc.sqp_max; ++it) {
      ++sqp_total;
      PSTAMP(PROF_NM_OTHER);
      if (cur < 0) {
        for (int g = 0; g < G; ++g) put(g, v);
        mpass(dchain, fg, xg);
        NM_COUNT_PASS(1 + ndep);
        NM_COUNT_USED();
        PSTAMP(PROF_NM_FULL);
        cur = 0;
        fcur = fg[0];
        chain_of_solo();
      }
      setcur(cur);
      const double f0 = fcur;
      lds_sync();
      // R^-1 (upper, packed by rows): lane j solves R x = e_j in its own column
      if (row) {
        for (int kk = lane; kk >= 0; --kk) {
          double a = (kk == lane) ? 1.0 : 0.0;
          for (int j = kk + 1; j <= lane; ++j) a -= sR[nm_up(kk, j, M)] * sRi[nm_up(j, lane, M)];
          sRi[nm_up(kk, lane, M)] = a / sR[nm_up(kk, kk, M)];
        }
      }
      lds_sync();
      // unconstrained Gauss-Newton step s_u = -R^-1 c
      double xm = 0.0;
      if (row)
        for (int k = lane; k < M; ++k) xm -= sRi[nm_up(lane, k, M)] * scv[k];
      PSTAMP(PROF_NM_RINV);
      // ---- box QP: lb <= U + cumulative step <= ub, Goldfarb-Idnani from s_u
      const double clo = row ? lbn - sU[lane] : 0.0, chi = row ? ubn - sU[lane] : 0.0;
      lds_sync();
      GIState<MAXM> gis;
      gi_reset<MAXM>(gis);
      for (int w = lane; w < nbits; w += kWave) sbits[w] = 0u;
      // J = R^-1 (gi_core's J'-in-LDS layout, sJT[k M + i] = J(i, k)) from the packed upper triangle
      if (row)
#pragma unroll 1
        for (int k = 0; k < M; ++k) sJT[k * M + lane] = k >= lane ? sRi[nm_up(lane, k, M)] : 0.0;
      gis.nrot = 0;
      gis.jinit = true;
      lds_sync();
      const StateMark mark{sbits, 4 * M};
      int git = 0;
      for (;;) {
        const double pre = block_prefix<MAXM>(xm, bl, Nu, row, sxc);
        double s4[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
        if (row) {
          if (bl == 0) {
            s4[0] = xm - clo;
            s4[1] = chi - xm;
          } else {
            s4[2] = pre - clo;
            s4[3] = chi - pre;
          }
        }
        double best = INFINITY;
        int bid = 0x7fffffff;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (!((gis.act >> k) & 1u) && s4[k] < best) {
            best = s4[k];
            bid = 4 * lane + k;
          }
        if (has_xb) {
          // linearised state rows  x_min <= x_i + dx_i/dv s <= x_max  at the iterate s
          if (row) sxc[lane] = xm;
          lds_sync();
          for (int q = lane; q < 6 * N; q += kWave) {
            if ((sbits[q >> 5] >> (q & 31)) & 1u) continue;
            const int r = q >> 1, si = r - (r / 3) * 3;
            const double bnd = (q & 1) ? txmax[si] : txmin[si];
            if (!isfinite(bnd)) continue;
            double dot = 0.0;
            for (int m = 0; m < M; ++m) dot += ssx[r * M + m] * sxc[m];
            const double xr = sxp[r] + dot;
            const double sl = (q & 1) ? bnd - xr : xr - bnd;
            if (sl < best) {
              best = sl;
              bid = 4 * M + q;
            }
          }
        }
        wave_argmin64(best, bid);
        if (!(best < -tol)) break;
        if (git >= maxit) {
          st |= MPCT_ST_QP_MAXITER_;
          break;
        }
        const int p = bid;
        double sp = best, upm = 0.0;
        bool infeas = false;
        for (;;) {
          ++git;
          const double dk = dvec(p);
          lds_sync();
          const double d2 = row ? dk * dk : 0.0;
          const double dn2 = qsum<MAXM>(d2);
          const double beta = qsum<MAXM>(lane >= gis.q ? d2 : 0.0);
          const double zm = gi_z(sJT, sd, gis.q, M, row);
          const double rk = gi_backsub<MAXM>(gis, sRA, M, dk, RAPacked{});
          double t1 = INFINITY;
          int kdrop = 0x7fffffff;
          if (lane < gis.q && rk > 0.0) {
            t1 = qp_div(gis.uw, rk);
            kdrop = lane;
          }
          qargmin<MAXM>(t1, kdrop);
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
            gi_add<MAXM>(gis, sJT, sRA, sd, M, p, dk, beta, zm, upm, row, mark, RAPacked{});
            break;
          }
          if (kdrop >= gis.q) {  // t1 or t2 NaN: no lane attains the ratio test (a non-finite state)
            st |= MPCT_ST_NONFINITE_;
            infeas = true;
            break;
          }
          gi_drop<MAXM>(gis, sJT, sRA, M, kdrop, mark, RAPacked{});
          if (git >= maxit) break;
        }
        if (infeas) break;
        if (git >= maxit) {
          st |= MPCT_ST_QP_MAXITER_;
          break;
        }
      }
      PSTAMP(PROF_NM_QP);
      // ---- convergence on the absolute-move change of the full step (oracle: max|d|/s_u); the
      // iterate itself is returned (its pass, and the next call's first pass from it, are done)
      const double dpre = block_prefix<MAXM>(xm, bl, Nu, row, sxc);
      double chg = row ? fabs(dpre) / sun : 0.0;
      if (!isfinite(chg)) chg = INFINITY;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) chg = fmax(chg, __shfl_xor(chg, off, 64));
      if (chg <= sc.sqp_tol) {
        for (int k = 0; k < 3; ++k) {
          sq[k] = ch[k];
          sqf[k] = chf[k];
        }
        return v;
      }
      if (!(chg < INFINITY)) {
        st |= MPCT_ST_NONFINITE_;
        return v;
      }
      // ---- directional derivative of the cost along the step: dd = r'J s = c'R s
      if (row) sxc[lane] = xm;
      lds_sync();
      double rs = 0.0;
      if (row)
        for (int j = lane; j < M; ++j) rs += sR[nm_up(lane, j, M)] * sxc[j];
      const double dd = qsum<MAXM>(row ? scv[lane] * rs : 0.0);
      // ---- Anderson step (oracle/nmpc_vdv.py AA_DEPTH = 1): gamma = <df, d>/<df, df> on the
      // absolute moves scaled by 1/s_u, candidate clip(G(v) - gamma (G(v) - G(v'))); taken when
      // it meets the Armijo decrease of the full step and respects the state bounds
      const double gv = v + (row ? xm : 0.0);
      bool have_aa = false;
      double vc = 0.0;
      if (aa_hist) {
        const double wdf = row ? (dpre - aa_f) / sun : 0.0;
        const double den = qsum<MAXM>(wdf * wdf);
        if (den > 0.0) {
          const double gam = qsum<MAXM>(row ? wdf * (dpre / sun) : 0.0) / den;
          const double vc0 = row ? gv - gam * (gv - aa_g) : 0.0;
          const double pc = block_prefix<MAXM>(vc0, bl, Nu, row, sxc);
          const double ucl = fmin(fmax(ulb + pc, lbn), ubn);
          const double upl = lane_prev<MAXM>(ucl);
          vc = row ? (bl == 0 ? ucl - ulb : ucl - upl) : 0.0;
          have_aa = true;
        }
      }
      aa_f = row ? dpre : 0.0;
      aa_g = gv;
      aa_hist = true;
      // ---- Armijo backtracking on the cost along the step (oracle/nmpc_vdv.py controller):
      // halve alpha until f(v + alpha s) <= f0 + c1 alpha dd or the cost change is below its own
      // rounding; the last alpha is taken regardless.  The Anderson candidate and the full step
      // (alpha = 1) share one pass when the point buffers allow (G > 1), with the next call's
      // first pass from each (G = 4)
      double alpha = 1.0;
      int ls0 = 0;        // first Armijo step still to try
      bool taken = false;
      if (have_aa) {
        PSTAMP(PROF_NM_OTHER);
        const double va1 = v + (row ? alpha * xm : 0.0);
        put(0, vc);
        if (G > 1) put(1, va1);
        if (G > 3) {
          put(2, vc);
          put(3, va1);
        }
        // G = 4: the Anderson candidate and the full step on rows 0, 1, the next call's first
        // point from each on rows 2, 3
        const bool sp4 = G > 3 && nf > 0;
        mpass(sp4 ? 0x50u : 0u, fg, xg);
        NM_COUNT_PASS((G > 1 ? 2 : 1) + (sp4 ? 2 : 0));
        PSTAMP(PROF_NM_AA);
        if (xg[0] && fg[0] <= f0 + kLsC1 * dd) {
          NM_COUNT_USED();
          v = vc;
          cur = 0;
          fcur = fg[0];
          ch[0] = sp4 ? 2 : -1;
          chf[0] = fg[2];
          ch[1] = ch[2] = -1;
          taken = true;
        } else if (G > 1) {
          const double f1 = fg[1];
          if (f1 <= f0 + kLsC1 * alpha * dd || f1 - f0 <= kLsFlat * f0) {
            NM_COUNT_USED();
            v = va1;
            cur = 1;
            fcur = f1;
            ch[0] = sp4 ? 3 : -1;
            chf[0] = fg[3];
            ch[1] = ch[2] = -1;
            taken = true;
          } else {
            alpha *= 0.5;
            ls0 = 1;
          }
        }
      }
      if (taken) continue;
      cur = -1;
      ch[0] = ch[1] = ch[2] = -1;
      for (int ls = ls0; ls < kLsMax; ++ls) {
        bool xin;
        // the full step's trial is a full pass (usually taken), shorter steps a tangent-free one
        const double va = v + (row ? alpha * xm : 0.0);
        PSTAMP(PROF_NM_OTHER);
        double f1;
        if (ls == 0) {
          for (int g = 0; g < G; ++g) put(g, va);
          mpass(dchain, fg, xg);
          NM_COUNT_PASS(1 + ndep);
          f1 = fg[0];
          PSTAMP(PROF_NM_LS0);
        } else {
          f1 = trial(va, xin);
          PSTAMP(PROF_NM_TRIAL);
        }
        if (f1 <= f0 + kLsC1 * alpha * dd || f1 - f0 <= kLsFlat * f0) {
          if (ls == 0) {
            NM_COUNT_USED();
            cur = 0;
            fcur = f1;
            chain_of_solo();
          }
          break;
        }
        alpha *= 0.5;
      }
      v += row ? alpha * xm : 0.0;
    }
    st |= MPCT_ST_SQP_MAXITER_;
    return v;
  };

  // ------------------------------------------------------------------ open-loop prediction
  // closedloop_toolbox_nmpc.m:79-95: one call at (x0, u0, r(:,end)); MVopt held after Nu
  double x0[3] = {tx0[0], tx0[1], tx0[2]};
  double u0[2] = {tu0[0], nu > 1 ? tu0[1] : 0.0};
  double vop = 0.0;
  double jnu = 0.0;
  if (o.open_loop) {
    const int hq0[3] = {-1, -1, -1};
    const double hqf0[3] = {0.0, 0.0, 0.0};
    int sq_[3];
    double sqf_[3];
    vop = controller(x0, u0, ny > 0 ? rr[nit - 1] : 0.0, ny > 1 ? rr[nit + nit - 1] : 0.0, 0.0, hq0, hqf0, 0, 0,
                     sq_, sqf_);
    // absolute moves -> sU (held in LDS for the open-loop simulation)
    if (row) sxc[lane] = vop;
    lds_sync();
    if (row) {
      double cum = 0.0;
      for (int j = lane - bl; j <= lane; ++j) cum += sxc[j];
      sUo[lane] = u0[bn] + cum;
    }
    lds_sync();
    if (lane < nu) {
      // VNS2.m:183-191: Xnu = |uopt(:,1)| ./ |diff(uopt)|, inf/NaN -> 0, Jnu = sum Xnu^2;
      // uopt(:,k) = MVopt row k (held after Nu - 1), k = 1..nit
      const double uf = fabs(sUo[lane * Nu]);
      for (int t = 0; t + 1 < nit; ++t) {
        const int l0 = t < Nu - 1 ? t : Nu - 1, l1 = t + 1 < Nu - 1 ? t + 1 : Nu - 1;
        const double dd = fabs(sUo[lane * Nu + l1] - sUo[lane * Nu + l0]);
        const double xr = uf / dd;
        if (isfinite(xr)) jnu += xr * xr;
      }
    }
  }

  // ------------------------------------------------------------------ closed loop
  double x[3] = {x0[0], x0[1], x0[2]};
  double xo[3] = {x0[0], x0[1], x0[2]};
  double ul[2] = {u0[0], u0[1]};
  double v = 0.0;  // warm start: moves held at u0
  // point buffers holding the next calls' first passes (speculated by earlier calls), their costs
  int hq[3] = {-1, -1, -1};
  double hqf[3] = {0.0, 0.0, 0.0};
  double j1 = 0.0, j21 = 0.0, j22 = 0.0;
  bool inb = true;
  const int ink0 = sc.ink0;
  for (int t = 0; t < nit; ++t) {
    if (t > 0) {
      const double r0 = rr[t], r1 = ny > 1 ? rr[nit + t] : 0.0;
      // this call also runs the first passes of up to three later calls (hq, hqf)
      int sq[3];
      double sqf[3];
      v = controller(x, ul, r0, r1, v, hq, hqf, t, min(3, nit - 1 - t), sq, sqf);
      for (int k = 0; k < 3; ++k) {
        hq[k] = sq[k];
        hqf[k] = sqf[k];
      }
      // the first move U(:,t) = u(t-1) + v[n][0]
      if (row) sxc[lane] = v;
      lds_sync();
      double un[2] = {ul[0] + sxc[0], nu > 1 ? ul[1] + sxc[Nu] : 0.0};
      lds_sync();
      PSTAMP(PROF_NM_OTHER);
      vdv_rk4<false>(P, h, nsub, x, un, nullptr, nullptr);
      PSTAMP(PROF_NM_PLANT);
      ul[0] = un[0];
      ul[1] = un[1];
      // warm start for the next step: the solution shifted by one move (last move repeated),
      // expressed against the new last move: v'[l] = v[l+1], v'[Nu-1] = 0
      const double vn = lane_next<64>(v);
      v = (row && bl < Nu - 1) ? vn : 0.0;
      if (o.open_loop) {
        const int l = t < Nu - 1 ? t : Nu - 1;
        const double uo[2] = {sUo[l], nu > 1 ? sUo[Nu + l] : 0.0};
        vdv_rk4<false>(P, h, nsub, xo, uo, nullptr, nullptr);
      }
    }
    for (int i = 0; i < 3; ++i) inb = inb && x[i] >= txmin[i] - 1e-9 && x[i] <= txmax[i] + 1e-9;
    if (lane < ny) {
      const double y = sel3(x, lane == 0 ? xc0 : xc1);
      const double e1 = y - sc.yref[lane * nit + t];
      j1 += e1 * e1;
      if (t >= ink0) j22 += e1 * e1;
      double ysv = 0.0;
      if (o.open_loop) {
        ysv = sel3(xo, lane == 0 ? xc0 : xc1);
        if (t >= ink0) j21 += (y - ysv) * (y - ysv);
      }
      if (o.want_traj) {
        if (out.y) out.y[(sim * ny + lane) * nit + t] = y;
        if (o.open_loop && out.ys) out.ys[(sim * ny + lane) * nit + t] = ysv;
      }
    }
    if (o.want_traj && lane < nu) {
      if (out.u) out.u[(sim * nu + lane) * nit + t] = ul[lane == 0 ? 0 : 1];
      if (o.open_loop && out.uopt) {
        const int l = t < Nu - 1 ? t : Nu - 1;
        out.uopt[(sim * nu + lane) * nit + t] = sUo[lane * Nu + l];
      }
    }
  }
  if (!inb) st |= MPCT_ST_BOUNDS_;
#ifdef MPCT_PROFILE
  PSTAMP(PROF_NM_OTHER);
  if (lane == 0 && out.prof)
    for (int k = 0; k < PROF_N; ++k) out.prof[sim * PROF_N + k] = pacc.get(k);
#endif
  // ------------------------------------------------------------------ results
  if (lane < ny) {
    if (!isfinite(j1)) st |= MPCT_ST_NONFINITE_;
    if (out.J1) out.J1[sim * ny + lane] = j1;
    if (out.j22) out.j22[sim * ny + lane] = j22;
    if (out.j21) out.j21[sim * ny + lane] = o.open_loop ? j21 : NAN;
  }
  if (lane < nu && out.Jnu) out.Jnu[sim * nu + lane] = o.open_loop ? jnu : NAN;
  const unsigned long long nf = __ballot(st & MPCT_ST_NONFINITE_);
  if (lane == 0) {
    const int s = st | (nf ? MPCT_ST_NONFINITE_ : 0);
    if (out.status) out.status[sim] = s;
    if (out.qp_iters) out.qp_iters[sim] = sqp_total;
  }
}

}  // namespace mpct

// ------------------------------------------------------------------------------------------
// host-side launch
#include <algorithm>
#include <string>

#include "work_order.h"

namespace mpct {


// LDS tiers (KB) of the class launches.  One wave per SIMD (384 / 434 VGPRs), so at most four
// workgroups per CU, which 40 KB still allows: the M <= 15 class sizes its point buffers to 40 KB
// (nm_groups), one tier; the M <= 32 class 40 KB, the rest above (a 32 KB first tier held the
// simulations between 32 and 40 KB to three per CU: config 5 21.7 k -> 22.0-22.3 k sims/s at 40,
// profiles/r06m_lds_banks_ab.txt; finer tiers measured slower)
constexpr long long kNmCap16Kb = 40, kNmCap32Kb = 40;

long long nmpc_lds_bytes(int M, int N) { return (long long)nm_layout(M, N, nm_groups(M, N)).total * 8; }

// one launch per (QP size class MAXM 16 / 32) x (LDS tier), heaviest first, fanned over the
// streams of launch_fan.h so the tiers overlap; a simulation runs in the launch of its class and
// tier, and the light tiers (short horizons) get the occupancy their own LDS allows instead of
// the n_max-sized allocation of the heaviest candidate
template <int MAXM>
static int launch_nmpc_t(const DevScenario& sc, long long C, int nref, const int* N, const int* Nu, const double* delta,
                         const double* lambda, const double* r, const int* perm, const DevOpts& o,
                         const DevResult& out, FanScope& fs, int& nl, int mz_lo, bool& first, std::string* err) {
  const int Mhi = std::min(sc.nu * sc.numax, kNmRows<MAXM> > 1 ? 15 : MAXM);
  long long lds_max = 0;  // the class's largest simulation (the point buffers depend on M and N)
  for (int m = mz_lo + 1; m <= Mhi; ++m)  // not monotone in N: the point buffers drop 4 -> 2 at 40 KB
    for (int n = 1; n <= sc.n2max; ++n) lds_max = std::max(lds_max, nmpc_lds_bytes(m, n));
  if (lds_max == 0) return 0;
  // LDS tiers (KB) of the class launches; the last one takes the rest up to lds_max
  static const long long c16[] = {kNmCap16Kb}, c32[] = {kNmCap32Kb};
  const long long* caps = MAXM <= 16 ? c16 : c32;
  const int ncap = 1;
  long long lo[8], hi[8];
  int ncls = 0;
  for (long long l = 0; ncls < 8 && l < lds_max; ++ncls) {
    lo[ncls] = l;
    hi[ncls] = ncls < ncap ? std::min(caps[ncls] * 1024, lds_max) : lds_max;
    l = hi[ncls];
  }
  for (int k = ncls - 1; k >= 0; --k) {
    const hipStream_t ls = fs.stream(nl);
    if (!diag_drop_launch(nl++))
      hipLaunchKernelGGL(nmpc_closed_loop_kernel<MAXM>, dim3((unsigned)(C * nref)), dim3(kWave), (size_t)hi[k], ls, sc,
                         C, nref, N, Nu, delta, lambda, r, perm, o, out, mz_lo, lo[k], hi[k], first ? 1 : 0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      *err = std::string("kernel launch failed: ") + hipGetErrorString(e);
      return -3;
    }
    first = false;
  }
  return 0;
}

int launch_nmpc(const DevScenario& sc, long long C, int nref, const int* N, const int* Nu, const double* delta,
                const double* lambda, const double* r, const DevOpts& o, const DevResult& out, hipStream_t stream,
                LaunchFan* fan, WorkOrder* wo, std::string* err) {
  const int Mmax = sc.nu * sc.numax;
  if (Mmax > 32) {
    *err = "nu*nu_max > 32";
    return -4;
  }
  // every (M, N) pair a candidate may use: the layout is not monotone in N (nm_groups)
  long long lds_all = 0;
  for (int m = 1; m <= Mmax; ++m)
    for (int n = 1; n <= sc.n2max; ++n) lds_all = std::max(lds_all, nmpc_lds_bytes(m, n));
  if (lds_all > 64 * 1024) {
    *err = "n_max x nu*nu_max needs more than 64 KiB of LDS per simulation";
    return -4;
  }
  const int* perm = nullptr;
  if (wo) {
    const int rc0 = order_candidates(kOrderNmpc, sc.my, sc.nu, C, N, Nu, delta, lambda, *wo, &perm, stream, err);
    if (rc0) return rc0;
  }
  int rc = prefill_results(out, C * nref, sc.my, sc.nu, stream, err);
  if (rc) return rc;
  FanScope fs(fan, stream);  // forks after the sort: every class launch waits for the permutation
  int nl = 0;
  bool first = true;  // the first launch also writes the padding / bad-horizon statuses
  if (Mmax > 15) rc = launch_nmpc_t<32>(sc, C, nref, N, Nu, delta, lambda, r, perm, o, out, fs, nl, 15, first, err);
  if (rc == 0) rc = launch_nmpc_t<16>(sc, C, nref, N, Nu, delta, lambda, r, perm, o, out, fs, nl, 0, first, err);
  fs.join();
  if (perm) order_mark_used(*wo, stream);  // after the join: every class launch has read it
  return rc;
}

}  // namespace mpct
