// gpc_prologue.h — the once-per-candidate prologue of the linear closed-loop kernels
// (gpc_closed_loop_kernel, gpc_small_kernel): the dynamic matrix G (MatG.m:64-67) weighted and
// QR-factored together with the free-response rows, giving the unconstrained gain and R^-1.
//
// QR of W = [Q^1/2 G; Lambda^1/2] carrying V = [Q^1/2 Phi; 0], streaming W's rows in blocks of
// kHB (lane l < M owns column l of R, lane l >= M a column of T = Q1'V).  R's row k absorbs a
// block by one Householder reflection that annihilates the block's column k: x = [R_kk; w_.k],
// R_kk <- ||x|| (kept positive), v = x - ||x|| e1 with v_0 = -sigma / (R_kk + ||x||) (sigma =
// ||w_.k||^2: no cancellation), H = I - beta v v', beta = -1 / (||x|| v_0).  The reflection is
// decided by lane k and broadcast with v_readlane; per block of 8 rows it issues about half the
// VALU of 8 Givens rotations (one rsq / rcp chain per column instead of one per row).  When
// M + nx > 64 the V columns are processed in passes of 64 - M; every pass recomputes the same
// reflections (bitwise identical R), so T is exact.  Normal equations are never formed
// (cond(G'QG + Lambda) reaches 2e12 on the tuning grids).
#pragma once
#include "mpct_dev.h"
#include "wave_ops.h"

namespace mpct {

// Outputs in LDS: R (upper, row-major, M x M) in sR; R^-1 (upper: row-major M x M, or PACKED its
// upper triangle row by row, gpc_qp16.h rinv_idx) in sRi; the gain
// A = -R^-1 T with state column vc of row m at sA[m * astride + acol(vc)] (acol: host column map,
// nullptr = identity).  Returns false (uniformly) when R is not positive definite.
// RINV = false: no R^-1 (an unconstrained loop has no QP); FIRST = true: only the first-move rows
// m = n Nu of A, stored as row n (DTC_GPC_WW.m:105 Km: the unconstrained loop applies those alone)
template <int MAXM, bool PACKED = false, bool RINV = true, bool FIRST = false, int kHB = 8>
__device__ __forceinline__ bool gpc_prologue(const DevScenario& sc, int lane, int M, int Nu, int N2,
                                             const double* dl, const double* lm, double* sR, double* sRi,
                                             double* sA, int astride, const int* acol) {
  const int my = sc.my, nu = sc.nu, nx = sc.nx;
  const int vper = kWave - M;  // V columns per pass (host guarantees M < 64)
  const int npass = (nx + vper - 1) / vper;
  double rcol[MAXM];
  int gn = 0, gc = 0;
  if (lane < M) {
    gn = lane / Nu;
    gc = lane - gn * Nu;
  }
  double sqv = 0.0;  // lane i < my: the output weight's square root (broadcast per row)
  if (lane < my) {
    const double di = fabs(dl[lane]);
    sqv = sc.wsq ? di : sqrt(di);
  }
  for (int pass = 0; pass < npass; ++pass) {
    const int vc = pass * vper + (lane - M);  // this lane's V column in this pass
    const bool vlane = lane >= M && vc < nx;
    {
      double wl0 = 0.0;
      if (lane < M) {
        const double ln = fabs(lm[lane / Nu]);
        wl0 = sc.wsq ? ln : sqrt(ln);
      }
#pragma unroll
      for (int k = 0; k < MAXM; ++k) rcol[k] = (k == lane) ? wl0 : 0.0;
    }
    // lane's entry of the next weighted row (output fi, prediction step fr) of
    // [Q^1/2 G | Q^1/2 Phi]; zero rows past the end pad the last block
    int fi = 0, fr = 0;
    auto fetch = [&]() __attribute__((always_inline)) -> double {
      double v = 0.0;
      if (fi < my) {
        if (lane < M) {
          const int tt = sc.n1[fi] + fr - gc;
          v = tt >= 0 ? sc.step[(fi * nu + gn) * sc.tlen + tt] : 0.0;  // prologue only: global (L2)
        } else if (vlane) {
          v = sc.phi[(long long)(fi * sc.n2max + fr) * nx + vc];
        }
        v *= bcast(sqv, fi);
        if (++fr == N2) {
          fr = 0;
          ++fi;
        }
      }
      return v;
    };
    auto reflect = [&](double (&w)[kHB], int k) __attribute__((always_inline)) {
      double wk[kHB];
      double sg0 = 0.0, sg1 = 0.0;
#pragma unroll
      for (int i = 0; i < kHB; ++i) {
        wk[i] = bcast(w[i], k);
        if (i & 1) sg1 = fma(wk[i], wk[i], sg1);
        else sg0 = fma(wk[i], wk[i], sg0);
      }
      const double sig = sg0 + sg1;
      if (sig == 0.0) return;  // uniform: the block's column k is already zero
      const double x0 = bcast(rcol[k], k);
      const double rn = rsq_nr(fma(x0, x0, sig));  // 1 / ||x||
      const double rs = rcp_nr(sig);
      const double n = fma(x0, x0, sig) * rn;
      const double xpn = x0 + n;
      const double v0 = -sig * rcp_nr(xpn);
      const double beta = rn * xpn * rs;  // -1 / (||x|| v_0)
      double s0 = v0 * rcol[k], s1 = 0.0;
#pragma unroll
      for (int i = 0; i < kHB; ++i) {
        if (i & 1) s1 = fma(wk[i], w[i], s1);
        else s0 = fma(wk[i], w[i], s0);
      }
      const double f = beta * (s0 + s1);
      const bool own = lane == k;
      rcol[k] = own ? n : fma(-f, v0, rcol[k]);
      // lane k keeps its block entries' rounding residue instead of an exact 0: they only ever reach
      // lanes left of later pivots, i.e. R's lower triangle, which nothing reads, so R's upper
      // triangle and T are bitwise those of the select (round 6: 24 v_cndmask fewer per reflection,
      // the metric 1 % faster, profiles/r06z_prologue_nosel_ab.txt)
#pragma unroll
      for (int i = 0; i < kHB; ++i) w[i] = fma(-f, wk[i], w[i]);
    };
    const int P = my * N2;
    const int nblk = (P + kHB - 1) / kHB;
    double nb[kHB];
#pragma unroll
    for (int i = 0; i < kHB; ++i) nb[i] = fetch();
    for (int blk = 0; blk < nblk; ++blk) {
      double w[kHB];
#pragma unroll
      for (int i = 0; i < kHB; ++i) w[i] = nb[i];
      if (blk + 1 < nblk) {  // prefetch the next block (L2 latency under the reflections)
#pragma unroll
        for (int i = 0; i < kHB; ++i) nb[i] = fetch();
      }
#pragma unroll
      for (int k = 0; k < MAXM; ++k)
        if (k < M) reflect(w, k);
    }
    if (pass == 0) {  // R to LDS; singular R -> status
      lds_sync();
      // the lane id through an opaque copy: otherwise the compiler forms the M store addresses
      // before the QR and keeps them live across it, where a 12-row block spills them (round 6)
      int ln = lane;
      asm volatile("" : "+v"(ln));
      if (ln < M) {
#pragma unroll
        for (int k = 0; k < MAXM; ++k)
          if (k < M) sR[k * M + ln] = rcol[k];
      }
      lds_sync();
      bool spd = true;
      for (int k = 0; k < M; ++k)
        if (!(sR[k * M + k] > 0.0)) spd = false;
      if (!spd) return false;
    }
    // A = -R^-1 T: V lanes solve for their own column
    if (vlane) {
#pragma unroll
      for (int kk = MAXM - 1; kk >= 0; --kk) {
        if (kk < M) {
          double a = rcol[kk];
#pragma unroll
          for (int j = 0; j < MAXM; ++j)
            if (j > kk && j < M) a -= sR[kk * M + j] * rcol[j];
          rcol[kk] = a / sR[kk * M + kk];
        }
      }
      const int ac = acol ? acol[vc] : vc;
#pragma unroll
      for (int m = 0; m < MAXM; ++m) {
        if constexpr (FIRST) {
          if (m < M && m % Nu == 0) sA[(m / Nu) * astride + ac] = -rcol[m];
        } else {
          if (m < M) sA[m * astride + ac] = -rcol[m];
        }
      }
    }
  }
  // R^-1: lane j solves R x = e_j in its own LDS column (zeros below unless PACKED)
  auto ri = [&](int i, int k) __attribute__((always_inline)) -> int {
    return PACKED ? i * M - ((i * (i - 1)) >> 1) + (k - i) : i * M + k;
  };
  if (!RINV) {
    lds_sync();
    return true;
  }
  if (lane < M) {
    for (int kk = lane; kk >= 0; --kk) {
      double a = (kk == lane) ? 1.0 : 0.0;
      for (int j = kk + 1; j <= lane; ++j) a -= sR[kk * M + j] * sRi[ri(j, lane)];
      sRi[ri(kk, lane)] = a / sR[kk * M + kk];
    }
    if (!PACKED)
      for (int kk = lane + 1; kk < M; ++kk) sRi[kk * M + lane] = 0.0;
  }
  lds_sync();
  return true;
}

}  // namespace mpct
