// gpc_kernel.hip — batched closed-loop GPC simulation, one wavefront (64 lanes) per simulation.
//
// Replaces, per simulation, the body of closedloop_toolbox.m:36-100 (sim + mpcstate/mpcmove +
// lsim) with the toolbox-equivalent GPC of DESIGN.md:
//   prologue (once per candidate):  G from the step table (MatG.m:64-67), H = G'QG + Lambda,
//       K = G'Q*Phi with Phi = [F | Hp] (diophantine.m / deltaUFree.m / cell2mat2.m tables built
//       on the host), Kw = G'Q*E;  Cholesky -> H^-1;  A = [-H^-1 K | H^-1 Kw]
//   per step t:  plant output (exact difference equations of every (i,j) entry — lsim),
//       unconstrained minimiser dU = A [x; r(t)] (x = y histories | du histories, i.e. the
//       state S*Yd + Hp*up of DTC_GPC_WW.m:139-146 folded into A), then a Goldfarb-Idnani dual
//       active-set QP (the toolbox's KWIK is of this family) when a rate / amplitude bound is
//       violated, apply the first move of every MV, shift the histories.
// Lanes: rows of the QP (move index m = n*Nu + l) for the solver; plant entries for the plant;
// columns of [G | Phi | E] in the prologue.  All state lives in LDS (one wave per workgroup, so
// __syncthreads() is a single-wave barrier).  Arithmetic is IEEE f64 throughout.
#include <hip/hip_runtime.h>
#include <math.h>

#include "mpct_dev.h"

namespace mpct {

struct LdsLayout {
  int hinv, A, x, xc, v, z, r, u, sv, uprev, yprev, ucum, ye, yeh, uring, Y, sinv, tmp, step, wid, total;
};

__host__ __device__ inline LdsLayout lds_layout(int M, int nxa, int nu, int nin, int ne, int my,
                                                int tlen) {
  LdsLayout L;
  int o = 0;
  auto take = [&](int n) { int r = o; o += (n + 1) & ~1; return r; };
  L.hinv = take(M * M);
  L.A = take(nxa * M);
  L.x = take(nxa);
  L.xc = take(M);
  L.v = take(M);
  L.z = take(M);
  L.r = take(M);
  L.u = take(M);
  L.sv = take(M);
  L.uprev = take(nu);
  L.yprev = take(my);
  L.ucum = take(M);
  L.ye = take(2 * ne);
  L.yeh = take(2 * ne * kYeHist);
  L.uring = take(2 * nin * kURing);
  L.wid = take(M);
  // union: loop-only QP workspace | prologue step table
  int u0 = o;
  L.Y = u0;
  L.sinv = u0 + M * M;
  L.tmp = u0 + 2 * M * M;
  int loopsz = 3 * M * M;
  L.step = u0;
  int stepsz = my * nu * tlen;
  o = u0 + (loopsz > stepsz ? loopsz : stepsz);
  L.total = (o + 1) & ~1;
  return L;
}

__device__ __forceinline__ void wave_argmin(double& v, int& id) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    double ov = __shfl_xor(v, off, 64);
    int oid = __shfl_xor(id, off, 64);
    if (ov < v || (ov == v && oid < id)) {
      v = ov;
      id = oid;
    }
  }
}

// constraint p = 4*m + kind on move m = n*Nu + l:
//   kind 0:  du_m >= lo     kind 1: -du_m >= -hi      (l == 0: merged rate/amplitude box)
//   kind 2:  sum_{l'<=l} du_(n,l') >= u_min - u_prev    kind 3: -sum >= -(u_max - u_prev)
struct CInfo {
  int j0, j1;   // index range [j0, j1] of the normal's support
  double sg;    // sign of the normal
};
__device__ __forceinline__ CInfo cinfo(int p, int Nu) {
  int m = p >> 2, kind = p & 3;
  CInfo c;
  c.sg = (kind & 1) ? -1.0 : 1.0;
  if (kind < 2) {
    c.j0 = m;
    c.j1 = m;
  } else {
    c.j0 = (m / Nu) * Nu;
    c.j1 = m;
  }
  return c;
}

// Slacks of the 4 constraints owned by lane m (< M); +inf for disabled ones.
__device__ __forceinline__ void lane_slacks(const double* __restrict__ sxc, int m, int Nu,
                                            const double* bnd, const double* uprev, int nu,
                                            double s[4]) {
  int n = m / Nu, l = m - n * Nu;
  double dmin = bnd[n], dmax = bnd[nu + n], umin = bnd[2 * nu + n], umax = bnd[3 * nu + n];
  double up = uprev[n];
  double xm = sxc[m];
  if (l == 0) {
    double lo = fmax(dmin, umin - up), hi = fmin(dmax, umax - up);
    s[0] = xm - lo;
    s[1] = hi - xm;
    s[2] = INFINITY;
    s[3] = INFINITY;
  } else {
    double pre = 0.0;
    for (int j = n * Nu; j <= m; ++j) pre += sxc[j];
    s[0] = xm - dmin;
    s[1] = dmax - xm;
    s[2] = pre - (umin - up);
    s[3] = (umax - up) - pre;
  }
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Goldfarb-Idnani dual active-set QP, numerically stable form:
// with H = R'R (R from the QR of W = [Q^1/2 G; Lambda^1/2]) and B = R^-T N_W for the active
// normals, each iteration recomputes the Householder QR of [B | b_p] (lanes = columns):
//   [c; tail] = Qb' b_p,  r = Rb^-1 c,  e = Qb [0; tail],  z = R^-1 e,  beta = n_p'z = |tail|^2.
// Starts from the unconstrained minimiser in sxc[0..M).  R^-1 (upper, row-major) is in
// lds[L.hinv].  Returns inner iterations; sets *st bits.  Wave-uniform control flow.
template <int MAXM>
__device__ int gi_qp(double* __restrict__ lds, const LdsLayout& L, int M, int Nu, int nu,
                     const double* bnd, double tol, int maxit, int* st) {
  const int lane = threadIdx.x;
  const double* sRi = lds + L.hinv;
  double* sxc = lds + L.xc;
  double* sbp = lds + L.v;
  double* se = lds + L.z;
  double* sr = lds + L.r;
  double* su = lds + L.u;
  double* sc_ = lds + L.sv;
  double* sB = lds + L.Y;     // active b_w columns [w][m]
  double* sRb = lds + L.sinv; // Rb columns [w][k]
  double* sV = lds + L.tmp;   // reflectors [j][k]
  double* suprev = lds + L.uprev;
  int* sW = reinterpret_cast<int*>(lds + L.wid);
  unsigned act = 0;  // active bits of this lane's 4 constraints
  int q = 0, it = 0;
  double xm = lane < M ? sxc[lane] : 0.0;
  for (;;) {
    // ---- most violated inactive constraint
    double best = INFINITY;
    int bid = 0x7fffffff;
    if (lane < M) {
      double s[4];
      lane_slacks(sxc, lane, Nu, bnd, suprev, nu, s);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (!((act >> k) & 1u) && s[k] < best) {
          best = s[k];
          bid = 4 * lane + k;
        }
    }
    wave_argmin(best, bid);
    if (!(best < -tol)) break;
    if (it >= maxit || q >= M) {
      *st |= MPCT_ST_QP_MAXITER_;
      break;
    }
    const int p = bid;
    const CInfo cp = cinfo(p, Nu);
    // b_p = R^-T n_p:  b_p[m] = sg * sum_{j in S_p} Rinv[j][m]
    double bpm = 0.0;
    if (lane < M) {
      for (int j = cp.j0; j <= cp.j1; ++j) bpm += sRi[j * M + lane];
      bpm *= cp.sg;
      sbp[lane] = bpm;
    }
    const double bpn = wave_sum(bpm * bpm);
    double sp = best;  // current slack of p
    double up = 0.0;   // its multiplier
    __syncthreads();
    for (;;) {
      ++it;
      // ---- Householder QR of [B | b_p], lane w holds column w (w < q: b_w, w == q: b_p)
      double col[MAXM];
      const double* src = lane < q ? sB + lane * M : sbp;
#pragma unroll
      for (int k = 0; k < MAXM; ++k) col[k] = (lane <= q && k < M) ? src[k] : 0.0;
      for (int j = 0; j < q; ++j) {
        if (lane == j) {
          double nrm = 0.0, cj = 0.0;
#pragma unroll
          for (int k = 0; k < MAXM; ++k)
            if (k >= j && k < M) nrm += col[k] * col[k];
#pragma unroll
          for (int k = 0; k < MAXM; ++k)
            if (k == j) cj = col[k];
          nrm = sqrt(nrm);
          const double alpha = cj > 0.0 ? -nrm : nrm;
          double vn = 0.0;
#pragma unroll
          for (int k = 0; k < MAXM; ++k) {
            if (k < M) {
              double v = k < j ? 0.0 : (k == j ? col[k] - alpha : col[k]);
              sV[j * M + k] = v;
              vn += v * v;
              col[k] = k < j ? col[k] : (k == j ? alpha : 0.0);
            }
          }
          sc_[j] = vn;  // |v_j|^2 (sc_ reused: c is read from the b_p lane later)
        }
        __syncthreads();
        if (lane > j && lane <= q) {
          const double vn = sc_[j];
          if (vn != 0.0) {
            double dt = 0.0;
#pragma unroll
            for (int k = 0; k < MAXM; ++k)
              if (k >= j && k < M) dt += sV[j * M + k] * col[k];
            const double f = 2.0 * dt / vn;
#pragma unroll
            for (int k = 0; k < MAXM; ++k)
              if (k >= j && k < M) col[k] -= f * sV[j * M + k];
          }
        }
      }
      // Rb columns to LDS; lane q: c (k < q) and tail (k >= q)
      if (lane < q) {
#pragma unroll
        for (int k = 0; k < MAXM; ++k)
          if (k < M) sRb[lane * M + k] = col[k];
      }
      double beta_part = 0.0;
      if (lane == q) {
#pragma unroll
        for (int k = 0; k < MAXM; ++k)
          if (k < M) {
            se[k] = k < q ? 0.0 : col[k];
            if (k >= q) beta_part += col[k] * col[k];
            if (k < q) sr[k] = col[k];  // c, solved in place below
          }
      }
      const double beta = wave_sum(beta_part);
      __syncthreads();
      // e = H_0 ... H_{q-1} [0; tail]   (lanes = components)
      double ek = lane < M ? se[lane] : 0.0;
      for (int j = q - 1; j >= 0; --j) {
        const double vn = sc_[j];
        const double vk = (lane >= j && lane < M) ? sV[j * M + lane] : 0.0;
        const double dt = wave_sum(vk * ek);
        if (vn != 0.0) ek -= (2.0 * dt / vn) * vk;
      }
      // r = Rb^-1 c  (column-oriented back substitution, lane k holds c_k)
      double ck = lane < q ? sr[lane] : 0.0;
      double rk = 0.0;
      for (int w = q - 1; w >= 0; --w) {
        const double rw = __shfl(ck, w, 64) / sRb[w * M + w];
        if (lane == w) rk = rw;
        if (lane < w) ck -= sRb[w * M + lane] * rw;
      }
      if (lane < M) se[lane] = ek;
      __syncthreads();
      // z = R^-1 e
      double zm = 0.0;
      if (lane < M) {
        for (int k = lane; k < M; ++k) zm += sRi[lane * M + k] * se[k];
      }
      // dual step length t1 over active constraints with r_w > 0
      double t1 = INFINITY;
      int kdrop = 0x7fffffff;
      if (lane < q && rk > 0.0) {
        t1 = su[lane] / rk;
        kdrop = lane;
      }
      wave_argmin(t1, kdrop);
      const double t2 = (beta > 1e-14 * bpn) ? -sp / beta : INFINITY;
      if (t1 == INFINITY && t2 == INFINITY) {
        *st |= MPCT_ST_QP_INFEAS_;
        if (lane < M) sxc[lane] = xm;
        __syncthreads();
        return it;
      }
      const bool full = t2 <= t1;
      const double t = full ? t2 : t1;
      if (lane < M && t2 != INFINITY) {
        xm += t * zm;
        sxc[lane] = xm;
      }
      if (lane < q) su[lane] -= t * rk;
      up += t;
      sp += t * beta;
      __syncthreads();
      if (full) {
        if (lane < M) sB[q * M + lane] = sbp[lane];
        if (lane == 0) {
          su[q] = up;
          sW[q] = p;
        }
        if (lane == (p >> 2)) act |= 1u << (p & 3);
        ++q;
        __syncthreads();
        break;
      }
      // drop kdrop, keeping the order of the remaining columns
      {
        const int k = kdrop;
        const int idk = sW[k];
        if (lane == (idk >> 2)) act &= ~(1u << (idk & 3));
        __syncthreads();
        for (int w = k; w < q - 1; ++w) {
          if (lane < M) sB[w * M + lane] = sB[(w + 1) * M + lane];
          if (lane == 0) {
            su[w] = su[w + 1];
            sW[w] = sW[w + 1];
          }
        }
        --q;
        __syncthreads();
      }
      if (it >= maxit) {
        *st |= MPCT_ST_QP_MAXITER_;
        break;
      }
    }
    if (it >= maxit) break;
  }
  __syncthreads();
  return it;
}

template <int MAXM>
__global__ void __launch_bounds__(64)
    gpc_closed_loop_kernel(const DevScenario sc, long long C, int nref,
                           const int* __restrict__ N2v, const int* __restrict__ Nuv,
                           const double* __restrict__ deltav, const double* __restrict__ lambdav,
                           const double* __restrict__ rv, const double* __restrict__ vv,
                           const DevOpts o, const DevResult out) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x;
  const long long sim = blockIdx.x;
  if (sim >= C * nref) return;
  const long long c = sim / nref;
  const int kref = (int)(sim - c * nref);
  const int my = sc.my, nu = sc.nu, nin = sc.nin, nit = sc.nit, nx = sc.nx, ne = sc.ne;
  const int N2 = N2v[c], Nu = Nuv[c];
  const int M = nu * Nu;
  int st = 0;

  auto write_nan = [&](int status) {
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
    write_nan(MPCT_ST_SKIPPED_);
    return;
  }
  if (N2 > sc.n2max || Nu < 1 || Nu > sc.numax || Nu > N2 || M > MAXM) {
    write_nan(MPCT_ST_BADHORIZON_);
    return;
  }
  const LdsLayout L = lds_layout(M, nx, nu, nin, ne, my, sc.tlen);
  double* sH = lds + L.hinv;
  double* sA = lds + L.A;
  double* sx = lds + L.x;
  double* sxc = lds + L.xc;
  double* suprev = lds + L.uprev;
  double* sucum = lds + L.ucum;
  double* sye = lds + L.ye;
  double* syeh = lds + L.yeh;
  double* sur = lds + L.uring;
  double* sstep = lds + L.step;
  double* syprev = lds + L.yprev;  // raw y(t-1) per output

  // ------------------------------------------------------------------ prologue
  for (int e = lane; e < my * nu * sc.tlen; e += kWave) sstep[e] = sc.step[e];
  for (int e = lane; e < L.Y - L.x; e += kWave) lds[L.x + e] = 0.0;  // persistent state
  __syncthreads();
  const double* dl = deltav + c * my;
  const double* lm = lambdav + c * nu;

  // QR of the weighted least-squares matrix W = [Q^1/2 G; Lambda^1/2] by row-streamed Givens
  // rotations, carrying the right-hand block V = [Q^1/2 Phi_dev; 0]  (the
  // normal equations G'QG + Lambda reach cond 1e12 on the config-2 grid and lose ~1e-5).
  // Lane l owns column l of [R | T] (l < M: R, else T = Q1'V); rotation k is decided by lane k
  // and broadcast with a wave shuffle.  The Lambda^1/2 rows are already triangular: R0 = Lambda^1/2.
  const int ncol = M + nx;  // <= 64 (checked on the host)
  const int l = lane;
  double rc[MAXM];
  {
    double wl0 = 0.0;
    if (l < M) {
      const double ln = fabs(lm[l / Nu]);
      wl0 = sc.wsq ? ln : sqrt(ln);
    }
#pragma unroll
    for (int k = 0; k < MAXM; ++k) rc[k] = (k == l) ? wl0 : 0.0;
  }
  for (int i = 0; i < my; ++i) {
    const double di = fabs(dl[i]);
    const double sqi = sc.wsq ? di : sqrt(di);
    const int n1 = sc.n1[i];
    const double* stp = sstep + i * nu * sc.tlen;
    for (int r = 0; r < N2; ++r) {
      double w = 0.0;
      if (l < M) {
        const int n = l / Nu, cc = l - n * Nu, tt = n1 + r - cc;
        w = tt >= 0 ? stp[n * sc.tlen + tt] : 0.0;
      } else if (l < ncol) {
        w = sc.phi[(long long)(i * sc.n2max + r) * nx + (l - M)];
      }
      w *= sqi;
#pragma unroll
      for (int k = 0; k < MAXM; ++k) {
        if (k < M) {
          const double b = __shfl(w, k, 64);
          if (b != 0.0) {
            const double a = __shfl(rc[k], k, 64);
            const double rho = sqrt(a * a + b * b);
            const double cs = a / rho, sn = b / rho;
            const double rk = rc[k];
            rc[k] = cs * rk + sn * w;
            w = -sn * rk + cs * w;
          }
        }
      }
    }
  }
  // R to LDS (row-major, upper); singular R -> non-finite status
  if (l < M) {
#pragma unroll
    for (int k = 0; k < MAXM; ++k)
      if (k < M) sH[k * M + l] = rc[k];
  }
  __syncthreads();
  bool spd = true;
  for (int k = 0; k < M; ++k)
    if (!(sH[k * M + k] > 0.0)) spd = false;
  if (!spd) {
    write_nan(MPCT_ST_NONFINITE_);
    return;
  }
  // A = -R^-1 T (lanes M..M+nx-1, own column, back substitution), column-major [s][m]
  if (l >= M && l < ncol) {
#pragma unroll
    for (int kk = MAXM - 1; kk >= 0; --kk) {
      if (kk < M) {
        double a = rc[kk];
#pragma unroll
        for (int j = 0; j < MAXM; ++j)
          if (j > kk && j < M) a -= sH[kk * M + j] * rc[j];
        rc[kk] = a / sH[kk * M + kk];
      }
    }
#pragma unroll
    for (int m = 0; m < MAXM; ++m)
      if (m < M) sA[(l - M) * M + m] = -rc[m];
  }
  // R^-1 (upper) for the active-set method: lane j solves R x = e_j
  double* sRinv = lds + L.Y;  // temporary (union region; step table no longer needed)
  if (l < M) {
    double x[MAXM];
#pragma unroll
    for (int kk = 0; kk < MAXM; ++kk) x[kk] = 0.0;
#pragma unroll
    for (int kk = MAXM - 1; kk >= 0; --kk) {
      if (kk < M) {
        double a = (kk == l) ? 1.0 : 0.0;
#pragma unroll
        for (int j = 0; j < MAXM; ++j)
          if (j > kk && j < M) a -= sH[kk * M + j] * x[j];
        x[kk] = (kk <= l) ? a / sH[kk * M + kk] : 0.0;
      }
    }
#pragma unroll
    for (int kk = 0; kk < MAXM; ++kk)
      if (kk < M) sRinv[kk * M + l] = x[kk];
  }
  __syncthreads();
  for (int e = lane; e < M * M; e += kWave) sH[e] = sRinv[e];
  __syncthreads();

  const double* bnd = sc.bnd;
  const double tol = o.feas_tol;
  const int maxit = o.max_qp_iter > 0 ? o.max_qp_iter : 8 * M + 16;
  long long iters = 0;
  const double* rr = rv + (long long)kref * my * nit;
  const double* vvk = vv ? vv + (long long)kref * sc.nd * nit : nullptr;

  // unconstrained minimiser dU = A * state, then the QP; result in sxc
  auto solve_step = [&]() {
    if (lane < M) {
      double a0 = 0.0, a1 = 0.0;
      int s = 0;
      for (; s + 1 < nx; s += 2) {
        a0 += sA[s * M + lane] * sx[s];
        a1 += sA[(s + 1) * M + lane] * sx[s + 1];
      }
      if (s < nx) a0 += sA[s * M + lane] * sx[s];
      sxc[lane] = a0 + a1;
    }
    __syncthreads();
    iters += gi_qp<MAXM>(lds, L, M, Nu, nu, bnd, tol, maxit, &st);
  };

  // ------------------------------------------------------------------ open-loop prediction
  double jnu = 0.0;
  if (o.open_loop) {
    // closedloop_toolbox.m:86-91: initial state (y = 0), reference r(:, end)
    if (lane < my) sx[sc.yoff[lane]] = -rr[lane * nit + (nit - 1)];
    __syncthreads();
    solve_step();
    if (lane < M) {
      int n = lane / Nu, l = lane - n * Nu;
      double s = 0.0;
      for (int j = n * Nu; j <= n * Nu + l; ++j) s += sxc[j];
      sucum[lane] = s;  // Uopt row l for MV n (held after Nu-1)
    }
    __syncthreads();
    if (lane < nu) {
      // VNS2.m:183-191: Xnu = |uopt(:,1)| ./ |diff(uopt)|, inf/NaN -> 0, Jnu = sum Xnu^2
      double u0 = fabs(sucum[lane * Nu]);
      int nd_ = Nu - 1 < nit - 1 ? Nu - 1 : nit - 1;
      for (int t = 0; t < nd_; ++t) {
        double dd = fabs(sucum[lane * Nu + t + 1] - sucum[lane * Nu + t]);
        double xr = u0 / dd;
        if (isfinite(xr)) jnu += xr * xr;
      }
    }
    if (lane < my) sx[sc.yoff[lane]] = 0.0;
    __syncthreads();
  }

  // ------------------------------------------------------------------ closed loop
  double j1 = 0.0, j21 = 0.0, j22 = 0.0;
  const int ncopy = o.open_loop ? 2 : 1;
  for (int t = 0; t < nit; ++t) {
    // inputs at time t that are already known: MDs v(t); open-loop uopt(t)
    if (sc.nd > 0) {
      for (int e = lane; e < ncopy * sc.nd; e += kWave) {
        int cpy = e / sc.nd, j = e - cpy * sc.nd;
        sur[(cpy * nin + nu + j) * kURing + (t & (kURing - 1))] = vvk[j * nit + t];
      }
    }
    if (o.open_loop && lane < nu) {
      int l = t < Nu - 1 ? t : Nu - 1;
      sur[(nin + lane) * kURing + (t & (kURing - 1))] = sucum[lane * Nu + l];
    }
    __syncthreads();
    // plant entries y_e(t) (copy 0: closed loop, copy 1: open loop driven by uopt)
    for (int e = lane; e < ncopy * ne; e += kWave) {
      const int cpy = e / ne, ee = e - cpy * ne, j = ee % nin;
      const double* b = sc.pl_b + ee * sc.pl_maxb;
      const double* a = sc.pl_a + ee * sc.pl_maxa;
      const double* ur = sur + (cpy * nin + j) * kURing;
      double* yh = syeh + e * kYeHist;
      double acc = 0.0;
      const int nb = sc.pl_nb[ee], na = sc.pl_na[ee];
      for (int l = 0; l < nb; ++l)
        if (t - l >= 0) acc += b[l] * ur[(t - l) & (kURing - 1)];
      for (int l = 1; l < na; ++l)
        if (t - l >= 0) acc -= a[l] * yh[(t - l) & (kYeHist - 1)];
      yh[t & (kYeHist - 1)] = acc;
      sye[e] = acc;
    }
    __syncthreads();
    if (lane < my) {
      const int i = lane;
      double y = 0.0;
      for (int j = 0; j < nin; ++j) y += sye[i * nin + j];
      // state: [y - r, nabla y, ..., nabla^na y]; nabla^k y(t) = nabla^{k-1} y(t) - nabla^{k-1} y(t-1)
      const int yo = sc.yoff[i], nh = sc.nyhi[i];
      double cur = y, prev = syprev[i];
      for (int k = 1; k < nh; ++k) {
        const double old = sx[yo + k];
        const double nk = cur - prev;
        sx[yo + k] = nk;
        cur = nk;
        prev = old;
      }
      syprev[i] = y;
      sx[yo] = y - rr[i * nit + t];
      const double yr = sc.yref[i * nit + t];
      const double e1 = y - yr;
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
    __syncthreads();
    solve_step();
    if (lane < nu) {
      const int n = lane;
      const double du = sxc[n * Nu];
      const double un = suprev[n] + du;
      const int uo = sc.upoff[n], nh = sc.dum[n];
      for (int k = nh - 1; k > 0; --k) sx[uo + k] = sx[uo + k - 1];
      sx[uo] = du;
      sur[n * kURing + (t & (kURing - 1))] = un;
      if (o.want_traj) {
        if (out.u) out.u[(sim * nu + n) * nit + t] = un;
        if (o.open_loop && out.uopt) {
          int l = t < Nu - 1 ? t : Nu - 1;
          // Info.Uopt has p+1 rows then the padding repeats the last row (:94-98)
          out.uopt[(sim * nu + n) * nit + t] = sucum[n * Nu + l];
        }
      }
      suprev[n] = un;
    }
    __syncthreads();
  }

  // ------------------------------------------------------------------ results
  if (lane < my) {
    if (!isfinite(j1)) st |= MPCT_ST_NONFINITE_;
    if (out.J1) out.J1[sim * my + lane] = j1;
    if (out.j22) out.j22[sim * my + lane] = j22;
    if (out.j21) out.j21[sim * my + lane] = o.open_loop ? j21 : NAN;
  }
  if (lane < nu && out.Jnu) out.Jnu[sim * nu + lane] = o.open_loop ? jnu : NAN;
  unsigned long long nf = __ballot(st & MPCT_ST_NONFINITE_);
  if (lane == 0) {
    int s = st | (nf ? MPCT_ST_NONFINITE_ : 0);
    if (out.status) out.status[sim] = s;
    if (out.qp_iters) out.qp_iters[sim] = iters;
  }
}

}  // namespace mpct

// ------------------------------------------------------------------------------------------
// host-side launch
#include <string>

namespace mpct {

long long lds_bytes_for(const DevScenario& sc, int N2, int Nu) {
  (void)N2;
  const int M = sc.nu * Nu;
  LdsLayout L = lds_layout(M, sc.nx, sc.nu, sc.nin, sc.ne, sc.my, sc.tlen);
  return (long long)L.total * 8;
}

template <int MAXM>
static int launch_t(const DevScenario& sc, long long C, int nref, const int* N2, const int* Nu,
                    const double* delta, const double* lambda, const double* r, const double* v,
                    const DevOpts& o, const DevResult& out, hipStream_t stream, std::string* err) {
  const long long lds = lds_bytes_for(sc, sc.n2max, sc.numax);
  if (lds > 160 * 1024) {
    *err = "scenario needs more than 160 KiB of LDS per simulation";
    return -4;
  }
  auto kern = gpc_closed_loop_kernel<MAXM>;
  if (lds > 64 * 1024) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
      *err = "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed";
      return -3;
    }
  }
  const long long S = C * nref;
  hipLaunchKernelGGL(kern, dim3((unsigned)S), dim3(kWave), (size_t)lds, stream, sc, C, nref, N2, Nu,
                     delta, lambda, r, v, o, out);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    *err = std::string("kernel launch failed: ") + hipGetErrorString(e);
    return -3;
  }
  return 0;
}

int launch_closed_loop(const DevScenario& sc, long long C, int nref, const int* N2, const int* Nu,
                       const double* delta, const double* lambda, const double* r,
                       const double* v, const DevOpts& o, const DevResult& out, int maxM,
                       hipStream_t stream, std::string* err) {
  if (maxM <= 16) return launch_t<16>(sc, C, nref, N2, Nu, delta, lambda, r, v, o, out, stream, err);
  if (maxM <= 32) return launch_t<32>(sc, C, nref, N2, Nu, delta, lambda, r, v, o, out, stream, err);
  if (maxM <= 64) return launch_t<64>(sc, C, nref, N2, Nu, delta, lambda, r, v, o, out, stream, err);
  *err = "nu*nu_max > 64";
  return -4;
}

}  // namespace mpct
