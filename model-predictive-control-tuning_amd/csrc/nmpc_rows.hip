// nmpc_rows.hip — throughput mode of the Van de Vusse NMPC closed loop (config 5): FOUR simulations
// per wavefront, one per 16-lane DPP row, for batches large enough to fill the chip
// (DESIGN.md §12).
//
// nmpc_kernel.hip runs one simulation per wave and spends the four 16-lane rows of its M <= 15 class
// on extra points of that one simulation (the Anderson candidate beside the full step, the next
// calls' first passes by speculation).  A pass is bound by the FP64 issue of its one wave, not by
// its lanes, so four points cost what one does; but speculated points are often wasted, and a
// 4096-candidate grid needs four rounds of 1024 waves.  Here each row carries its own simulation
// and every pass evaluates one point of each of the four: the batch runs in one round.
//
// Each row is a state machine over the same controller as nmpc_kernel.hip (oracle/nmpc_vdv.py
// controller, closedloop_nmpc): per tick the wave runs ONE joint prediction pass with forward
// tangents and the streamed Givens QR at every row's pending point, then every row takes the
// decision that point was evaluated for:
//   FIRST  the pass at the iterate v starts a Gauss-Newton iteration: R^-1, the unconstrained step,
//          the box / state-row QP (gi_row.h: row-local Goldfarb-Idnani), the convergence test, the
//          directional derivative, the Anderson candidate -> AA, else the full step -> LS
//   AA     the Anderson candidate: accepted (its pass is the next iteration's FIRST) or the full
//          step follows -> LS
//   LS     an Armijo trial at v + alpha s: accepted, or alpha halves (the last one is taken)
// A converged call applies its first moves (plant RK4 step), shifts the warm start and books the
// costs; the row's next call starts in the same tick.  The points evaluated, the decisions and the
// arithmetic of every point are the single-simulation kernel's (a tangent-free trial pass computes
// the same cost as a full one), so the results equal it; only the passes a simulation needs differ
// (no speculation).  Rows finish independently; a finished row idles until the wave's last row.
#include <hip/hip_runtime.h>
#include <math.h>

#include "gi_row.h"
#include "launch_fan.h"
#include "mpct_dev.h"
#include "nmpc_model.h"
#include "work_order.h"

namespace mpct {

// per-row sizes of the row kernel: one point buffer (G = 1)
__host__ __device__ inline long long nm_rows_bytes(int M, int N) { return (long long)nm_layout(M, N, 1).total * 8; }

// the row's decision modes
enum { NR_FIRST = 0, NR_AA = 1, NR_LS = 2, NR_DONE = 3 };

// row max over the 16 lanes of a row (every lane gets it)
__device__ __forceinline__ double row_max(double v) {
  v = fmax(v, dppd<kQx1>(v));
  v = fmax(v, dppd<kQx2>(v));
  v = fmax(v, dppd<kHalfMirror>(v));
  v = fmax(v, dppd<kMirror>(v));
  return v;
}

// active flags: box rows in the lanes' act bits, state-bound rows in the row's LDS bitmap
struct RowStateMark {
  unsigned* bits;
  int base;
  template <class St>
  __device__ __forceinline__ void operator()(St& S, int p, bool on) const {
    if (p < base) {
      RowBoxMark{}(S, p, on);
    } else if (rl_lane() == 0) {
      const int q = p - base;
      if (on) bits[q >> 5] |= 1u << (q & 31);
      else bits[q >> 5] &= ~(1u << (q & 31));
    }
  }
};

// One launch per LDS tier: a workgroup (one wave) takes the four consecutive dispatch slots
// 4 b .. 4 b + 3 (perm order, heaviest first), runs in the launch whose tier holds the four rows'
// LDS together, and only simulations with 1 <= M <= 15 (the M > 15 ones run nmpc_kernel.hip's M <= 32
// class; their rows idle here)
__global__ void __launch_bounds__(64, 1)
    nmpc_rows_kernel(const DevScenario sc, long long C, int nref, const int* __restrict__ Nv,
                     const int* __restrict__ Nuv, const double* __restrict__ deltav,
                     const double* __restrict__ lambdav, const double* __restrict__ rv,
                     const int* __restrict__ perm, const DevOpts o, const DevResult out, long long lds_lo,
                     long long lds_hi, int first_) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x, grp = lane >> 4, gl = lane & 15;
  const long long S = C * nref;
  const long long slot = 4LL * blockIdx.x + grp;
  const int ny = sc.my, nu = sc.nu, nit = sc.nit;
  // this row's simulation
  long long c = 0, sim = 0;
  int kref = 0, N = 0, Nu = 1, M = 0;
  bool live = slot < S;
  if (live) {
    const long long cs = slot / nref;
    kref = (int)(slot - cs * nref);
    c = perm ? (long long)perm[cs] : cs;
    sim = c * nref + kref;
    N = Nv[c];
    Nu = Nuv[c];
    M = nu * Nu;
    const bool bad = N <= 0 || N > sc.n2max || Nu < 1 || Nu > sc.numax || Nu > N;
    if (bad) {
      if (first_ && gl == 0) {
        if (out.status) out.status[sim] = N <= 0 ? MPCT_ST_SKIPPED_ : MPCT_ST_BADHORIZON_;
        if (out.qp_iters) out.qp_iters[sim] = 0;
      }
      if (first_ && gl < ny) {
        if (out.J1) out.J1[sim * ny + gl] = NAN;
        if (out.j21) out.j21[sim * ny + gl] = NAN;
        if (out.j22) out.j22[sim * ny + gl] = NAN;
      }
      if (first_ && gl < nu && out.Jnu) out.Jnu[sim * nu + gl] = NAN;
      live = false;
    } else if (M > 15) {
      live = false;  // nmpc_kernel.hip's M <= 32 class simulates it
    }
  }
  if (!live) {
    N = 0;
    Nu = 1;
    M = 0;
  }
  // the four rows' LDS, back to back; the group runs in the launch of its tier
  const NmLayout L = nm_layout(live ? M : 1, live ? N : 1, 1);
  const int mine = live ? L.total : 0;
  const int t0 = __shfl(mine, 0, 64), t1 = __shfl(mine, 16, 64), t2 = __shfl(mine, 32, 64),
            t3 = __shfl(mine, 48, 64);
  const long long gbytes = 8LL * (t0 + t1 + t2 + t3);
  if (gbytes == 0 || gbytes <= lds_lo || gbytes > lds_hi) return;  // no row here, or another tier
  const int roff = grp == 0 ? 0 : (grp == 1 ? t0 : (grp == 2 ? t0 + t1 : t0 + t1 + t2));
  double* base = lds + roff;
  double* sRi = base + L.ri;
  unsigned* sbits = reinterpret_cast<unsigned*>(base + L.bits);
  double* sxc = base + L.xc;
  double* sUo = base + L.uo;
  double* snv = base + L.nv;
  double* gb = base + L.grp;  // the row's one point buffer
  double* sR = gb + L.g_rr;
  double* scv = gb + L.g_cv;
  double* sU = gb + L.g_u;
  double* gv = gb + L.g_v;
  double* grw = gb + L.g_rw;
  double* sxp = gb + L.g_xp;
  double* ssx = gb + L.g_sx;
  const RowQP Q{base + L.jt, base + L.ra, base + L.dv};

  const double* tab = sc.nm;
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

  const bool row = live && gl < M;
  const int bn = row ? gl / Nu : 0;
  const int bl = row ? gl - bn * Nu : 0;
  const double lbn = tlb[bn], ubn = tub[bn], sun = tsu[bn];
  const double* dl = deltav + (live ? c : 0) * ny;
  const double* lm = lambdav + (live ? c : 0) * nu;
  const double wu = live ? fabs(lm[bn]) / sun : 0.0;
  const int xc0 = sc.xc[0], xc1 = ny > 1 ? sc.xc[1] : 0;
  const double wy0 = live ? fabs(dl[0]) / tsy[0] : 0.0, wy1 = live && ny > 1 ? fabs(dl[1]) / tsy[1] : 0.0;
  const double tol = o.feas_tol;
  const int maxit = o.max_qp_iter > 0 ? o.max_qp_iter : 200 * M + 1000;
  const double* rr = rv + (long long)kref * ny * nit;
  bool has_xb = false;
  for (int i = 0; i < 3; ++i) has_xb = has_xb || isfinite(txmin[i]) || isfinite(txmax[i]);
  const int nbits = (6 * N + 31) / 32;

  // ---- row state
  int st = 0;
  long long sqp_total = 0;
  int mode = live ? NR_FIRST : NR_DONE;
  int t = 0;             // closed-loop step of the running call (0: the open-loop call)
  bool olcall = false;   // the running call is the open-loop prediction (closedloop_toolbox_nmpc.m:79-95)
  double x[3] = {tx0[0], tx0[1], tx0[2]};
  double xo[3] = {tx0[0], tx0[1], tx0[2]};
  double ul[2] = {tu0[0], nu > 1 ? tu0[1] : 0.0};
  const double u0[2] = {tu0[0], nu > 1 ? tu0[1] : 0.0};
  double r0 = 0.0, r1 = 0.0;  // the running call's reference
  double v = 0.0;   // iterate (this lane's increment)
  double pt = 0.0;  // the pending point's increment (what the next pass evaluates)
  int it = 0;       // iterations of the running call
  double f0 = 0.0, dd = 0.0, alpha = 1.0, xm = 0.0, vc = 0.0;
  int ls = 0;
  bool aa_hist = false;
  double aa_f = 0.0, aa_g = 0.0;
  double j1 = 0.0, j21 = 0.0, j22 = 0.0, jnu = 0.0;
  bool inb_traj = true;
  const int ink0 = sc.ink0;

  // costs and trajectories of closed-loop step tt (state x, applied moves ul, open-loop state xo)
  auto book = [&](int tt) __attribute__((always_inline)) {
    for (int i = 0; i < 3; ++i) inb_traj = inb_traj && x[i] >= txmin[i] - 1e-9 && x[i] <= txmax[i] + 1e-9;
    if (gl < ny) {
      const double y = sel3(x, gl == 0 ? xc0 : xc1);
      const double e1 = y - sc.yref[gl * nit + tt];
      j1 += e1 * e1;
      if (tt >= ink0) j22 += e1 * e1;
      double ysv = 0.0;
      if (o.open_loop) {
        ysv = sel3(xo, gl == 0 ? xc0 : xc1);
        if (tt >= ink0) j21 += (y - ysv) * (y - ysv);
      }
      if (o.want_traj) {
        if (out.y) out.y[(sim * ny + gl) * nit + tt] = y;
        if (o.open_loop && out.ys) out.ys[(sim * ny + gl) * nit + tt] = ysv;
      }
    }
    if (o.want_traj && gl < nu) {
      if (out.u) out.u[(sim * nu + gl) * nit + tt] = ul[gl == 0 ? 0 : 1];
      if (o.open_loop && out.uopt) {
        const int l = tt < Nu - 1 ? tt : Nu - 1;
        out.uopt[(sim * nu + gl) * nit + tt] = sUo[gl * Nu + l];
      }
    }
  };
  // start a controller call from the warm start v at state x, last moves ul, reference (q0, q1)
  auto start_call = [&](double q0, double q1) __attribute__((always_inline)) {
    r0 = q0;
    r1 = q1;
    it = 0;
    aa_hist = false;
    aa_f = aa_g = 0.0;
    mode = NR_FIRST;
    pt = v;
  };
  // closed-loop step t of the running call is done: plant, warm start, costs; next call or done
  auto advance = [&]() __attribute__((always_inline)) {
    if (row) sxc[gl] = v;
    lds_sync();
    const double un[2] = {ul[0] + sxc[0], nu > 1 ? ul[1] + sxc[Nu] : 0.0};
    lds_sync();
    vdv_rk4<false>(P, h, nsub, x, un, nullptr, nullptr);
    ul[0] = un[0];
    ul[1] = un[1];
    const double vn = lane_next<16>(v);
    v = (row && bl < Nu - 1) ? vn : 0.0;
    if (o.open_loop) {
      const int l = t < Nu - 1 ? t : Nu - 1;
      const double uo[2] = {sUo[l], nu > 1 ? sUo[Nu + l] : 0.0};
      vdv_rk4<false>(P, h, nsub, xo, uo, nullptr, nullptr);
    }
    book(t);
    ++t;
    if (t >= nit) mode = NR_DONE;
    else start_call(rr[t], ny > 1 ? rr[nit + t] : 0.0);
  };
  // the open-loop call returned v: MVopt (held after Nu) and Jnu (VNS2.m:183-191); then the
  // closed loop starts: costs at t = 0, the first call at t = 1 from moves held at u0
  auto after_openloop = [&]() __attribute__((always_inline)) {
    if (row) sxc[gl] = v;
    lds_sync();
    if (row) {
      double cum = 0.0;
      for (int j = gl - bl; j <= gl; ++j) cum += sxc[j];
      sUo[gl] = u0[bn] + cum;
    }
    lds_sync();
    if (gl < nu) {
      const double uf = fabs(sUo[gl * Nu]);
      for (int tt = 0; tt + 1 < nit; ++tt) {
        const int l0 = tt < Nu - 1 ? tt : Nu - 1, l1 = tt + 1 < Nu - 1 ? tt + 1 : Nu - 1;
        const double d = fabs(sUo[gl * Nu + l1] - sUo[gl * Nu + l0]);
        const double xr = uf / d;
        if (isfinite(xr)) jnu += xr * xr;
      }
    }
    olcall = false;
    v = 0.0;
    book(0);
    t = 1;
    if (t >= nit) mode = NR_DONE;
    else start_call(rr[t], ny > 1 ? rr[nit + t] : 0.0);
  };
  // the running call returns v
  auto call_done = [&]() __attribute__((always_inline)) {
    if (olcall) after_openloop();
    else advance();
  };
  // the next iteration needs a fresh pass at v: or the call has used its sqp_max iterations
  auto next_first = [&]() __attribute__((always_inline)) {
    if (it >= sc.sqp_max) {
      st |= MPCT_ST_SQP_MAXITER_;
      call_done();
    } else {
      mode = NR_FIRST;
      pt = v;
    }
  };

  if (live) {
    for (int w = gl; w < (L.total - L.dv); w += 16) base[L.dv + w] = 0.0;  // vectors, bitmap, buffer
    if (o.open_loop) {
      olcall = true;
      v = 0.0;
      start_call(rr[nit - 1], ny > 1 ? rr[nit + nit - 1] : 0.0);
    } else {
      book(0);
      t = 1;
      if (t >= nit) mode = NR_DONE;
      else start_call(rr[t], ny > 1 ? rr[nit + t] : 0.0);
    }
  }
  lds_sync();

  while (__ballot(mode != NR_DONE) != 0) {
    const bool act = mode != NR_DONE;
    // ---------------------------------------------------------------- the joint pass
    // every active row's pending point pt: absolute moves, the prediction with forward tangents,
    // the streamed QR of [rate rows; output rows] (R, c = Q'r), the state rows, the cost f
    if (act && row) gv[gl] = pt;
    lds_sync();
    const bool prow = row;  // lane gl < M carries tangent column gl; lane gl = M the residual
    if (act && row) {
      double cum = 0.0;
      for (int j = gl - bl; j <= gl; ++j) cum += gv[j];
      sU[gl] = (bn == 0 ? ul[0] : ul[1]) + cum;
      grw[gl] = wu * pt;
    }
    lds_sync();
    double f = 0.0;
    bool inb = true;
    if (act) {
      double rcol[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        double e = 0.0;
        if (k < M) {
          if (gl == k) e = wu;
          else if (gl == M) e = grw[k];
        }
        rcol[k] = e;
      }
      double xs[3] = {x[0], x[1], x[2]};
      double td[3] = {0.0, 0.0, 0.0};
      double fo = 0.0;
      for (int i = 0; i < N; ++i) {
        const int li = i < Nu - 1 ? i : Nu - 1;
        const double u[2] = {sU[li], nu > 1 ? sU[Nu + li] : 0.0};
        double ud[2] = {0.0, 0.0};
        if (prow && bl <= li) ud[bn] = 1.0;
        vdv_rk4<true>(P, h, nsub, xs, u, td, ud);
        if (has_xb) {
          if (prow) {
            ssx[(i * 3 + 0) * M + gl] = td[0];
            ssx[(i * 3 + 1) * M + gl] = td[1];
            ssx[(i * 3 + 2) * M + gl] = td[2];
          } else if (gl == M) {
            sxp[i * 3 + 0] = xs[0];
            sxp[i * 3 + 1] = xs[1];
            sxp[i * 3 + 2] = xs[2];
          }
          for (int s3 = 0; s3 < 3; ++s3) inb = inb && xs[s3] >= txmin[s3] && xs[s3] <= txmax[s3];
        }
        for (int j = 0; j < ny; ++j) {
          const int xj = j == 0 ? xc0 : xc1;
          const double wy = j == 0 ? wy0 : wy1;
          if (!(wy > 0.0)) continue;
          double w = 0.0;
          if (prow) w = wy * sel3(td, xj);
          else if (gl == M) w = wy * (sel3(xs, xj) - (j == 0 ? r0 : r1));
          fo += w * w;
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            if (k < M) {
              const double b = row_bcast16(w, k);
              const double a = row_bcast16(rcol[k], k);
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
      if (prow || gl == M) {
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if (k < M) {
            if (prow) sR[k * M + gl] = rcol[k];
            else scv[k] = rcol[k];
          }
      }
      const double rv2 = prow ? (wu * pt) * (wu * pt) : 0.0;
      const double rs = row_sum(rv2);
      f = 0.5 * (rbcast(fo, M) + rs);
      // the state bounds of every predicted state, for the whole row (all lanes integrate it)
    }
    lds_sync();
    if (!act) continue;

    // ---------------------------------------------------------------- the row's decision
    bool iterate = false;  // this pass at v starts an iteration
    if (mode == NR_FIRST) {
      iterate = true;
    } else if (mode == NR_AA) {
      if (inb && f <= f0 + kLsC1 * dd) {
        v = vc;
        iterate = true;  // the candidate's pass is the next iteration's
        if (it >= sc.sqp_max) {
          st |= MPCT_ST_SQP_MAXITER_;
          iterate = false;
          call_done();
        }
      } else {
        alpha = 1.0;
        ls = 0;
        mode = NR_LS;
        pt = v + (row ? alpha * xm : 0.0);
      }
    } else {  // NR_LS: Armijo trial at v + alpha xm
      if (f <= f0 + kLsC1 * alpha * dd || f - f0 <= kLsFlat * f0) {
        const bool reuse = ls == 0;  // the full step's pass is the next iteration's
        v += row ? alpha * xm : 0.0;
        if (reuse) {
          iterate = true;
          if (it >= sc.sqp_max) {
            st |= MPCT_ST_SQP_MAXITER_;
            iterate = false;
            call_done();
          }
        } else {
          next_first();
        }
      } else {
        alpha *= 0.5;
        ++ls;
        if (ls >= kLsMax) {
          v += row ? alpha * xm : 0.0;
          next_first();
        } else {
          pt = v + (row ? alpha * xm : 0.0);
        }
      }
    }
    if (!iterate) continue;

    // ---------------------------------------------------------------- one Gauss-Newton iteration
    ++it;
    ++sqp_total;
    f0 = f;
    // R^-1 (upper, row-major): lane j solves R x = e_j in its own column
    if (row) {
      for (int kk = gl; kk >= 0; --kk) {
        double a = (kk == gl) ? 1.0 : 0.0;
        for (int j = kk + 1; j <= gl; ++j) a -= sR[kk * M + j] * sRi[j * M + gl];
        sRi[kk * M + gl] = a / sR[kk * M + kk];
      }
      for (int kk = gl + 1; kk < M; ++kk) sRi[kk * M + gl] = 0.0;
    }
    lds_sync();
    xm = 0.0;
    if (row)
      for (int k = gl; k < M; ++k) xm -= sRi[gl * M + k] * scv[k];
    // box QP lb <= U + cumulative step <= ub and the linearised state rows, Goldfarb-Idnani from s_u
    const double clo = row ? lbn - sU[gl] : 0.0, chi = row ? ubn - sU[gl] : 0.0;
    lds_sync();
    GIState<16> gis;
    gi_reset<16>(gis);
    for (int w = gl; w < nbits; w += 16) sbits[w] = 0u;
    gr_load_rinv<16>(gis, Q, sRi, M, row);
    const RowStateMark mark{sbits, 4 * M};
    int git = 0;
    for (;;) {
      const double pre = block_prefix<16>(xm, bl, Nu, row, nullptr);
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
          bid = 4 * gl + k;
        }
      if (has_xb) {
        if (row) sxc[gl] = xm;
        lds_sync();
        for (int q = gl; q < 6 * N; q += 16) {
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
      rargmin(best, bid);
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
        double dk;
        if (p < 4 * M) {
          const CInfo ci = cinfo(p, Nu);
          dk = gr_dvec(Q, M, ci.j0, ci.j1, ci.sg, row);
        } else {
          const int q = p - 4 * M, r = q >> 1;
          if (row) snv[gl] = (q & 1) ? -ssx[r * M + gl] : ssx[r * M + gl];
          lds_sync();
          dk = 0.0;
          if (row) {
            const double* jc = Q.JT + gl * M;
            for (int i = 0; i < M; ++i) dk += jc[i] * snv[i];
            Q.d[gl] = dk;
          }
        }
        lds_sync();
        const double d2 = row ? dk * dk : 0.0;
        const double dn2 = rsum(d2);
        const double beta = rsum(gl >= gis.q ? d2 : 0.0);
        const double zm = gr_z(Q, gis.q, M, row);
        const double rk = gr_backsub<16>(gis, Q, M, dk);
        double t1 = INFINITY;
        int kdrop = 0x7fffffff;
        if (gl < gis.q && rk > 0.0) {
          t1 = qp_div(gis.uw, rk);
          kdrop = gl;
        }
        rargmin(t1, kdrop);
        const double t2 = (beta > 1e-20 * dn2) ? -qp_div(sp, beta) : INFINITY;
        if (t1 == INFINITY && t2 == INFINITY) {
          st |= MPCT_ST_QP_INFEAS_;
          infeas = true;
          break;
        }
        const bool full = t2 <= t1;
        const double tt = full ? t2 : t1;
        if (t2 != INFINITY) xm += tt * zm;
        if (gl < gis.q) gis.uw -= tt * rk;
        upm += tt;
        sp += tt * beta;
        if (full) {
          gr_add<16>(gis, Q, M, p, dk, beta, zm, upm, row, mark);
          break;
        }
        gr_drop<16>(gis, Q, M, kdrop, mark);
        if (git >= maxit) break;
      }
      if (infeas) break;
      if (git >= maxit) {
        st |= MPCT_ST_QP_MAXITER_;
        break;
      }
    }
    // convergence on the absolute-move change of the full step (the iterate itself is returned)
    const double dpre = block_prefix<16>(xm, bl, Nu, row, nullptr);
    double chg = row ? fabs(dpre) / sun : 0.0;
    if (!isfinite(chg)) chg = INFINITY;
    chg = row_max(chg);
    if (chg <= sc.sqp_tol) {
      call_done();
      continue;
    }
    if (!(chg < INFINITY)) {
      st |= MPCT_ST_NONFINITE_;
      call_done();
      continue;
    }
    // directional derivative of the cost along the step: dd = c'R s
    if (row) sxc[gl] = xm;
    lds_sync();
    double rsv = 0.0;
    if (row)
      for (int j = gl; j < M; ++j) rsv += sR[gl * M + j] * sxc[j];
    dd = rsum(row ? scv[gl] * rsv : 0.0);
    // Anderson step (depth 1) on the absolute moves scaled by 1/s_u
    const double gvv = v + (row ? xm : 0.0);
    bool have_aa = false;
    if (aa_hist) {
      const double wdf = row ? (dpre - aa_f) / sun : 0.0;
      const double den = rsum(wdf * wdf);
      if (den > 0.0) {
        const double gam = rsum(row ? wdf * (dpre / sun) : 0.0) / den;
        const double vc0 = row ? gvv - gam * (gvv - aa_g) : 0.0;
        const double pc = block_prefix<16>(vc0, bl, Nu, row, nullptr);
        const double ulb = bn == 0 ? ul[0] : ul[1];
        const double ucl = fmin(fmax(ulb + pc, lbn), ubn);
        const double upl = lane_prev<16>(ucl);
        vc = row ? (bl == 0 ? ucl - ulb : ucl - upl) : 0.0;
        have_aa = true;
      }
    }
    aa_f = row ? dpre : 0.0;
    aa_g = gvv;
    aa_hist = true;
    if (have_aa) {
      mode = NR_AA;
      pt = vc;
    } else {
      alpha = 1.0;
      ls = 0;
      mode = NR_LS;
      pt = v + (row ? alpha * xm : 0.0);
    }
  }

  // ---------------------------------------------------------------- results
  if (!live) return;
  if (!inb_traj) st |= MPCT_ST_BOUNDS_;
  if (gl < ny) {
    if (!isfinite(j1)) st |= MPCT_ST_NONFINITE_;
    if (out.J1) out.J1[sim * ny + gl] = j1;
    if (out.j22) out.j22[sim * ny + gl] = j22;
    if (out.j21) out.j21[sim * ny + gl] = o.open_loop ? j21 : NAN;
  }
  if (gl < nu && out.Jnu) out.Jnu[sim * nu + gl] = o.open_loop ? jnu : NAN;
  // the row's status: lane 0 of the row ORs its lanes' non-finite flags
  const int nf = (int)row_max((st & MPCT_ST_NONFINITE_) ? 1.0 : 0.0);
  if (gl == 0) {
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

namespace mpct {

// LDS tiers (KB per workgroup of four rows) of the row launches: 4 / 3 / 2 / 1 workgroups per CU
constexpr long long kNmRowCapsKb[] = {40, 53, 80, 160};

long long nmpc_rows_group_max(const DevScenario& sc) {
  long long mx = 0;
  for (int m = 1; m <= std::min(15, sc.nu * sc.numax); ++m)
    for (int n = 1; n <= sc.n2max; ++n) mx = std::max(mx, nm_rows_bytes(m, n));
  return 4 * mx;
}

// the M <= 15 simulations of an NMPC batch, four per wave (one launch per LDS tier of the four
// rows' LDS together, fanned over `fs`); perm: the dispatch order (heaviest first, M > 15 first)
int launch_nmpc_rows(const DevScenario& sc, long long C, int nref, const int* N, const int* Nu, const double* delta,
                     const double* lambda, const double* r, const int* perm, const DevOpts& o,
                     const DevResult& out, FanScope& fs, int& nl, bool& first, std::string* err) {
  const long long gmax = nmpc_rows_group_max(sc);
  if (gmax == 0) return 0;
  if (gmax > 160 * 1024) {
    *err = "NMPC row mode: four rows need more than 160 KiB of LDS";
    return -4;
  }
  const long long S = C * nref;
  const unsigned groups = (unsigned)((S + 3) / 4);
  long long lo = 0;
  for (long long capkb : kNmRowCapsKb) {
    if (lo >= gmax) break;
    const long long hi = std::min(capkb * 1024, gmax);
    if (hi > lo) {
      if (hi > 64 * 1024 &&
          hipFuncSetAttribute(reinterpret_cast<const void*>(nmpc_rows_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)hi) != hipSuccess) {
        *err = "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed (NMPC rows)";
        return -3;
      }
      const hipStream_t ls = fs.stream(nl);
      if (!diag_drop_launch(nl++))
        hipLaunchKernelGGL(nmpc_rows_kernel, dim3(groups), dim3(kWave), (size_t)hi, ls, sc, C, nref, N, Nu, delta,
                           lambda, r, perm, o, out, lo, hi, first ? 1 : 0);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) {
        *err = std::string("kernel launch failed (NMPC rows): ") + hipGetErrorString(e);
        return -3;
      }
      first = false;
    }
    lo = hi;
  }
  if (lo < gmax) {
    *err = "NMPC row mode: LDS tiers do not cover the scenario";
    return -4;
  }
  return 0;
}

}  // namespace mpct
