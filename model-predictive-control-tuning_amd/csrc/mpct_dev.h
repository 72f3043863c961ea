// mpct_dev.h — device-side scenario layout shared by the host precompute (mpct_host.cpp) and
// the closed-loop kernel (gpc_kernel.hip).  Plain POD passed by value as a kernel argument.
#pragma once
#include <stdint.h>

namespace mpct {

// device buffers of the dispatch-order sort (keys, indices, hipcub temp), owned by a scenario
// The permutation is read by the launch that follows the sort; `used` is recorded after that
// launch so that the next call's sort (possibly on another stream) waits before rewriting it.
struct WorkOrder {
  void* buf = nullptr;
  size_t bytes = 0;
  const int* perm = nullptr;  // slot -> candidate (the last permutation), inside buf
  void* stage = nullptr;    // staging rows of the ordered launch's cost records (DevResult::stage)
  size_t stage_bytes = 0;
  hipEvent_t used = nullptr;
  bool pending = false;  // `used` has been recorded
};
constexpr long long kOrderMinC = 256;  // at most one workgroup per CU: a single round, order is moot
constexpr int kGramM = 16;                              // QP size of the dispatch-key Gram tables
constexpr int kGramOut = kGramM * kGramM + kGramM;      // doubles per output and (N2, Nu) block
constexpr long long kGramMaxBytes = 64ll << 20;         // larger tables are not built


constexpr int kMaxOut = 16;    // outputs (my)
constexpr int kMaxIn = 16;     // inputs (nu + nd)
constexpr int kURing = 32;     // plant input history ring (power of two)
constexpr int kMaxTaps = 16;   // longest plant numerator incl. delay (z^-1 taps)
constexpr int kYeHist = 8;     // plant entry output history ring (power of two)
constexpr int kMaxDum = 16;    // longest past-control register per MV (deltaUFree cp)
// register-resident per-lane state (DevScenario::regpath; larger scenarios use the LDS path)
constexpr int kRegB = 4;       // nonzero numerator taps per plant entry
constexpr int kRegA = 4;       // denominator coefficients a_1.. per plant entry
constexpr int kRegDu = 8;      // past-control register length per MV (regpath eligibility)
constexpr int kRegY = 6;       // y history (difference basis) length per output (regpath eligibility)
constexpr int kWave = 64;
// gpc_small_kernel (gpc_small.hip) layout constants, shared with the host tables it reads
constexpr int kSmY = 12;                   // y difference state: columns of A's quarter 0
constexpr int kSmR = 8;                    // past-control ring per MV: columns of quarters 1..3
constexpr int kSmA = kSmY + 3 * kSmR;      // A row stride
constexpr int kSmU = 16;                   // plant input ring per MV (power of two, > longest delay + taps)
constexpr int kSmE = 4;                    // longest plant entry output ring (power of two > denominator taps)
constexpr int kSmEOff = 3 * kSmU;          // entry output rings (4 my of them) after the input rings
constexpr int kDtcEOff = 4 * kSmU;         // dtc_small_kernel: 4 input rings (MVs + plant-only disturbances)

// per-simulation status bits (mirror of MPCT_ST_* in include/mpct.h)
constexpr int MPCT_ST_QP_MAXITER_ = 1;
constexpr int MPCT_ST_QP_INFEAS_ = 2;
constexpr int MPCT_ST_NONFINITE_ = 4;
constexpr int MPCT_ST_SKIPPED_ = 8;
constexpr int MPCT_ST_BADHORIZON_ = 16;
constexpr int MPCT_ST_SQP_MAXITER_ = 32;
constexpr int MPCT_ST_BOUNDS_ = 64;
constexpr int MPCT_ST_NOT_RUN_ = 128;

// NMPC model parameter table (mpct_nmpc_desc.params, nmpc_vandevusse_state.m:43-58 order)
enum { NM_K10 = 0, NM_K20, NM_K30, NM_E1, NM_E2, NM_E3, NM_DAB, NM_DBC, NM_DAD, NM_RHO, NM_CP, NM_KW, NM_AR,
       NM_V, NM_T0, NM_CA0, NM_NPAR };

struct DevScenario {
  int my, nu, nd, nin, nit;
  int n2max, numax, tlen;   // step table length per entry
  int nx;                   // free-response state: [y histories | du histories]
  int nyh, nup;             // sizes of the two parts
  int wsq;                  // weights squared
  int ink0;                 // VNS inK, 0-based
  int ne;                   // plant entries my*nin (nin = plant input columns incl. disturbances)
  int pl_maxb, pl_maxa;     // longest plant numerator (incl. delay) / denominator
  int regpath;              // every per-lane history / coefficient set fits the kReg* caps
  // small plants (gpc_small_kernel eligibility, mpct_host.cpp small_plant) and its lane tables:
  // plant term of lane L = 16 k + 4 i + j (coefficient, history ring offset in the kernel's history
  // region, delay, ring mask) and the state column -> A column map
  int small;
  int sm_ke;              // entry output ring length (DevScenario::small scenarios: 2 or 4)
  const double* sm_coef;  // [64]
  const int* sm_hoff;     // [64]
  const int* sm_hc;       // [64]
  const int* sm_hmask;    // [64]
  const int* sm_acol;     // [nx]
  // DTC-GPC small plants (dtc_small_kernel, dtc_small.hip; mpct_host.cpp dtc_small_plant): the sm_*
  // lane tables are [nvar][64] (plant variant k % nvar) and the filters Fr_i [my][8] (fb 0..3, fa 0..3)
  int small_dtc;
  const double* sm_fr;
  // tables (device pointers into one allocation)
  const double* step;   // [my][nu][tlen]   model step responses s_ij(t), t = 0..tlen-1
  // dispatch-key Gram tables (work_order.hip order_keys_gpc; nullptr when not built): block
  // (N2 - 1) numax + Nu - 1, output o at kGramOut o doubles: G_o'G_o (kGramM x kGramM, both
  // triangles) then G_o'1 (kGramM), G_o = the forced-response matrix of output o (MatG.m); only
  // for nu Nu <= kGramM and my <= 4
  const double* gram;
  const double* phi;    // [my*n2max][nx]   free response rows (Diophantine F | deltaUFree Hp)
  const int* n1;        // [my]   first predicted step
  const int* yoff;      // [my]   offset of y_i history (length na_i+1) in the state
  const int* nyhi;      // [my]   na_i + 1
  const int* upoff;     // [nu]   offset of du_n history (length duM_n) in the state
  const int* dum;       // [nu]   duM_n
  const int* pl_nb;     // [ne]   plant entry numerator length (z^-1, delay folded in)
  const int* pl_na;     // [ne]   plant entry denominator length
  const int* pl_off;    // [ne]   first nonzero numerator tap (the delay's leading zeros skipped)
  const double* pl_b;   // [ne][pl_maxb]
  const double* pl_a;   // [ne][pl_maxa]
  const double* bnd;    // [4][nu]  du_min, du_max, u_min, u_max
  const double* yref;   // [my][nit]
  // DTC-GPC predictor (dtc = 1): model entries Pz (e < my*nu) and Gz (e >= my*nu), z^-1 form,
  // and the robustness filters Fr_i, z^-1 form, delay 0
  int dtc;
  int nvar;               // plant variants: pl_* tables are [nvar][ne]; simulation k uses k % nvar
  int mz_maxb, mz_maxa, fr_max;
  const int* mz_nb;     // [2*my*nu]
  const int* mz_na;
  const int* mz_off;
  const double* mz_b;   // [2*my*nu][mz_maxb]
  const double* mz_a;   // [2*my*nu][mz_maxa]
  const int* fr_n;      // [my]
  const double* fr_b;   // [my][fr_max]
  const double* fr_a;   // [my][fr_max]
  // MD feed-forward + soft output bands (mdband = 1, mdband_kernel.hip): the model entries of all
  // nin = nu + nd columns are the mz_* tables ([my*nin], z^-1 form with delays)
  int mdband;
  double rho;             // Weights.ECR
  const double* step_md;  // [my][nd][tlen]  model MD step responses
  const double* obnd;     // [4][my]  y_min, y_max, MinECR*s_y, MaxECR*s_y (+-inf: no bound)
  const double* wscale;   // [my + nu]  1/s_y, 1/s_u (weights over ScaleFactors)
  int pl_maxbc, mz_maxbc; // longest run of numerator taps from the first nonzero one (compact LDS copies)
  // nonlinear MPC (nmpc = 1, nmpc_kernel.hip): my = outputs, nu = MVs, n2max = largest N
  int nmpc;
  int nsub, sqp_max;
  double ts, sqp_tol;
  const int* xc;          // [my] output states (0-based)
  const double* nm;       // [NM_NPAR][x0 3][u0 nu][u_min nu][u_max nu][x_min 3][x_max 3][s_y my][s_u nu]
};

struct DevOpts {
  int open_loop, want_traj, max_qp_iter;
  double feas_tol;
#ifdef MPCT_DIAG
  // diagnostic build only: planted kernel faults (kDiagSkipWarmDrop: the QPs' warm start computes
  // its drop but never applies it, so only the warm loop's own cap can end it)
  int diag;
#endif
};
#ifdef MPCT_DIAG
constexpr int kDiagSkipWarmDrop = 1;
#endif

// staging row of an ordered launch: the fields the caller asked for, in the order
// J1 [my] | j21 [my] | j22 [my] | Jnu [nu] | status | qp_iters (one double each); -1 = not staged
struct StageRow {
  int w, j1, j21, j22, jnu, st, it;
};

struct DevResult {
  double *J1, *j21, *j22, *Jnu;
  int32_t* status;
  int64_t* qp_iters;
  double *y, *u, *ys, *uopt;
  unsigned long long* prof;  // diagnostic builds only (-DMPCT_PROFILE): [sim][8] cycle sums
  // ordered launches: the cost record of workgroup slot k goes to staging row xcd_row(k) (layout
  // srow) instead of the caller's arrays, and unpermute_results gathers it back into the caller's
  // order.  The workgroups of a launch are dealt to the 8 XCDs round robin, so XCD x's slots fill
  // one contiguous block of rows and every 128-B line is written whole from one L2; written
  // straight to the caller's (permuted) index, a line collects 24-B pieces from up to 8 L2s and
  // each writes back its partial copy (2.6x the result bytes in WRITE_SIZE).
  double* stage = nullptr;
  StageRow srow = {0, -1, -1, -1, -1, -1, -1};
};

constexpr int kXcds = 8;
// staging row of workgroup slot k of an S-slot launch: XCD-major
__host__ __device__ inline long long xcd_row(long long k, long long S) {
  return (k % kXcds) * ((S + kXcds - 1) / kXcds) + k / kXcds;
}
inline StageRow stage_row(const DevResult& o, int my, int nu) {
  StageRow r = {0, -1, -1, -1, -1, -1, -1};
  auto put = [&r](bool on, int n, int& f) {
    if (on) {
      f = r.w;
      r.w += n;
    }
  };
  put(o.J1 != nullptr, my, r.j1);
  put(o.j21 != nullptr, my, r.j21);
  put(o.j22 != nullptr, my, r.j22);
  put(o.Jnu != nullptr, nu, r.jnu);
  put(o.status != nullptr, 1, r.st);
  put(o.qp_iters != nullptr, 1, r.it);
  return r;
}

// section ids of the diagnostic in-kernel stamps
enum { PROF_PROLOGUE = 0, PROF_PLANT, PROF_YUPD, PROF_UNC, PROF_QP, PROF_UUPD, PROF_OPENLOOP,
       PROF_QCHECK, PROF_QD, PROF_QR, PROF_QADD, PROF_QDROP, PROF_QWARM, PROF_QROT, PROF_QWENTRY, PROF_QWREB,
       PROF_QWGATH, PROF_QWSOLVE, PROF_QWDROP, PROF_QWROT, PROF_QWREADD, PROF_N = 21 };
// PROF_QROT: a count only (the drops' Givens rotations, gpc_qp16.h), no cycles.  The warm start of
// gpc_qp16.h: PROF_QWENTRY the entry test of an infeasible x_u, PROF_QWREB the
// J / B rebuild from R^-1, PROF_QWGATH the slacks' gather, PROF_QWSOLVE one pass of the equality
// solve, PROF_QWDROP one drop of a negative multiplier; PROF_QWARM closes what is left.
// PROF_QWROT / PROF_QWREADD: counts only (the warm drops' Givens rotations, the rebuild's re-adds)
// nmpc_kernel.hip's sections (same slots): the prediction with tangents and its streamed QR when
// it starts an iteration, R^-1 and the unconstrained step, the QP, the Anderson candidate's
// prediction, the full-step (alpha = 1) trial prediction, the shorter Armijo trials (tangent-free),
// the plant's RK4 step, everything else
enum { PROF_NM_FULL = 0, PROF_NM_RINV, PROF_NM_QP, PROF_NM_AA, PROF_NM_LS0, PROF_NM_TRIAL, PROF_NM_PLANT,
       PROF_NM_OTHER, PROF_NM_NPASS, PROF_NM_POINTS, PROF_NM_USED, PROF_NM_ROWS };
// counts only (tools/nmpc_fp64_split.py): PROF_NM_NPASS full passes (with
// tangents), PROF_NM_POINTS the points they were asked for (the iterate, the Anderson candidate, the
// alpha = 1 step, speculated first points of later calls), PROF_NM_USED the points whose
// linearisation an iteration went on to use (the iterate's first pass, the accepted Anderson /
// alpha = 1 point, a speculated point a later call started from), PROF_NM_ROWS the point rows each
// pass occupies (G: four 16-lane rows in the M <= 15 class, one whole wave above)

}  // namespace mpct
