// gpc_small.hip — closed-loop GPC scoring of small plants: one wavefront per simulation with every
// per-step quantity in a fixed lane layout, so the step loop has no data-dependent loops.
//
// Same simulation as gpc_closed_loop_kernel (closedloop_toolbox.m:36-50 restated as the
// toolbox-equivalent GPC of DESIGN.md §2, costs GAM_fun.m:110-111 J1 and VNS2.m:172-177 j22), for
// scenarios the host marks `small` (mpct_host.cpp small_plant): my <= 4 outputs, nu <= 3 MVs, no
// measured or plant-only disturbances, one plant, GPC (not DTC) mode, y difference state <= 12
// entries (<= 4 per output), past-control registers <= 8 per MV, <= 4 plant terms per entry, and
// cost-only batches (no open-loop leg, no trajectories).  The Shell 3x3 metric (BASELINE config 2)
// is such a scenario.  Others run the general kernel.
//
// Lane layout (lane L = 16 k + e, e = 4 i + j):
//   * plant: lane (k, e) holds term k of entry (output i, input j): a numerator tap b times a
//     delayed input u_j(t - c), or a denominator tap -a times the entry's own past output
//     y_e(t - c).  Each term is one LDS read from a history ring (the lane's ring, delay and
//     coefficient come from host tables), y_e = the sum over the four rows (v_permlane16/32_swap),
//     y_i = the sum over the quad (DPP quad_perm).  No per-entry loops.
//   * free-response state x = [y difference basis | past-control registers]: lane 4 i keeps output
//     i's backward differences in registers and stores them; each MV's past-control register is a
//     ring of 8 in LDS written twice per step (positions p and p + 8), so the window of the last 8
//     moves is contiguous at a rotating offset and nothing is shifted (ring buffers replace the
//     general kernel's serial LDS shifts).
//   * unconstrained minimiser dU = A x: lane (m, g) = QP row m, quarter g; quarter 0 holds the y
//     part (12 columns), quarters 1..3 the past-control ring of MV g - 1 (8 columns each; A's
//     columns are laid out the same way by the prologue's column map).  12 FMAs per lane, one
//     permlane reduction, and x_u arrives replicated over the four rows: the layout of the
//     register QP (gpc_qp16.h), which takes it without a hand-off.
//   * u update: the first moves come from the QP's register result by ds_bpermute.
// Per step: three LDS hand-offs (rings -> plant, y state -> product, and the QP's own), against
// five in the general kernel.
#include <hip/hip_runtime.h>
#include <math.h>

#include "mpct_dev.h"
#include "gi_core.h"
#include "gpc_qp.h"
#include "gpc_qp16.h"
#include "gpc_prologue.h"
#include "gpc_record.h"

namespace mpct {

// LDS layout of one simulation (doubles, 16-byte aligned pieces)
// (the Shell 3x3 metric, M = 15: 10,160 B, so 16 workgroups fit a CU's 160 KB)
struct SmallLayout {
  int rinv, ra, gb, A, xy, ring, hist, bnd, total;
};
__host__ __device__ inline SmallLayout small_layout(const DevScenario& sc, int M) {
  SmallLayout L;
  int o = 0;
  auto take = [&](int n) { int r = o; o += (n + 1) & ~1; return r; };
  L.rinv = take(M * (M + 1) / 2);   // R^-1, packed upper triangle (J rebuilds)
  L.ra = take(M * M);               // R_A (R during the prologue)
  L.gb = take(M * kBS);             // B = R_A^-1 (gpc_qp16.h), M rows
  L.A = take(M * kSmA);             // A, M rows x kSmA columns
  L.xy = take(kSmY);                // y part of x
  L.ring = take(3 * 2 * kSmR);      // past-control rings, two copies each
  L.hist = take(kSmEOff + 4 * sc.my * sc.sm_ke);  // input rings [3][kSmU] | entry output rings [4 my][ke]
  L.bnd = take(4 * 3);                            // MV bounds [nu][dmin, dmax, umin, umax] (96 B)
  L.total = (o + 1) & ~1;
  return L;
}

// opaque lane id: predicates derived from it are recomputed where used instead of being hoisted
// into SGPR-pair masks that the loop would have to keep live (and spill)
__device__ __forceinline__ int sm_lane() {
  int l = threadIdx.x;
  asm volatile("" : "+v"(l));
  return l;
}

// four waves per SIMD: 128 VGPRs (no spill since round 6: the QP rows' bounds live in LDS) and 10 KB of
// LDS, so 16 workgroups fit a CU and the metric's 4096 simulations run in one round.  Against three
// waves: bitwise the same results, 3.11-3.19 against 3.38-3.46 ms at 8192 candidates, the same
// 2.21-2.24 ms at 4096 (profiles/r04b_small_ab.txt)
__global__ void __launch_bounds__(64, 4)
    gpc_small_kernel(const DevScenario sc, long long C, int nref, const int* __restrict__ N2v,
                     const int* __restrict__ Nuv, const double* __restrict__ deltav,
                     const double* __restrict__ lambdav, const double* __restrict__ rv,
                     const int* __restrict__ perm, const DevOpts o, const DevResult out, int first) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x;
  const long long slot = blockIdx.x;
  const long long S = C * nref;
  if (slot >= S) return;
  const long long cs = slot / nref;
  const int kref = (int)(slot - cs * nref);
  const long long c = perm ? (long long)perm[cs] : cs;
  const long long sim = c * nref + kref;
  const int my = sc.my, nu = sc.nu, nit = sc.nit;
  const int N2 = N2v[c], Nu = Nuv[c];
  const int M = nu * Nu;
  auto write_nan = [&](int status) __attribute__((always_inline)) {
    put_record(out, slot, S, sim, my, nu, lane, NAN, NAN, NAN, NAN, status, 0);
  };
  if (N2 <= 0) {
    if (first) write_nan(MPCT_ST_SKIPPED_);
    return;
  }
  if (N2 > sc.n2max || Nu < 1 || Nu > sc.numax || Nu > N2) {
    if (first) write_nan(MPCT_ST_BADHORIZON_);
    return;
  }
  if (M > 16) return;  // the general kernel's wider class launches simulate it
#ifdef MPCT_PROFILE
  ProfAcc pacc;
  unsigned long long pprev = __builtin_amdgcn_s_memtime();
  using PAccT = ProfAcc;
#else
  using PAccT = void;
#endif
  const SmallLayout L = small_layout(sc, M);
  double* sA = lds + L.A;
  for (int e = lane; e < L.total - L.A; e += kWave) sA[e] = 0.0;  // A pads, state, rings
  lds_sync();

  // ------------------------------------------------------------------ prologue (gpc_prologue.h)
  // Householder blocks of 12 rows (round 6: 8 before; 12 fits 121 VGPRs once the R-store addresses
  // stop being hoisted across the QR, gpc_prologue.h): the heaviest 256 1.78-1.79 -> 1.76 ms, 8192
  // candidates 2.85 -> 2.78 ms, J1 within 1.8e-10 of the 8-row blocks (profiles/r06t_prologue_ab.txt)
  if (!gpc_prologue<16, true, true, false, 12>(sc, lane, M, Nu, N2, deltav + c * my, lambdav + c * nu, lds + L.ra, lds + L.rinv,
                              sA, kSmA, sc.sm_acol)) {
    write_nan(MPCT_ST_NONFINITE_);
    return;
  }
  PSTAMP(PROF_PROLOGUE);

  // per-lane constants of the step loop
  // plant term: coefficient, ring (LDS double index), delay, ring mask
  // the plant coefficient lives across the loop (round 5 spilled it to scratch and reloaded it at
  // the top of every step; re-reading it from the scenario table instead measured 2.5 % slower on
  // the heaviest 256; the bounds in LDS freed the registers in round 6)
  const double pcoef = sc.sm_coef[lane];
  const int pbase = L.hist + sc.sm_hoff[lane];
  const int pc = sc.sm_hc[lane], pmask = sc.sm_hmask[lane];
  const int ke = sc.sm_ke;
  // output lane 4 i (i < my): y difference state offset and length
  const int oi = (lane >> 2) & 3;
  const int yoff = oi < my ? sc.yoff[oi] : 0;
  const int nyh = oi < my ? sc.nyhi[oi] : 0;
  // product lane (m, g): A row segment and x segment
  const int qm = lane & 15, qg = lane >> 4;
  const int aoff = L.A + qm * kSmA + (qg ? kSmY + kSmR * (qg - 1) : 0);
  const int xoff = qg ? L.ring + 2 * kSmR * (qg - 1) : L.xy;
  // QP row of the lane (replicated over the four rows)
  RowCons rcn;
  rcn.n = qm < M ? qm / Nu : 0;
  rcn.l = qm < M ? qm - rcn.n * Nu : 0;
  // the row's MV bounds stay in LDS (gpc_qp16.h BLDS), stored before the loop's first lds_sync
  if (lane < 4 * nu) lds[L.bnd + lane] = sc.bnd[(lane & 3) * nu + (lane >> 2)];
  rcn.bnd = lds + L.bnd + 4 * rcn.n;
  const double tol = o.feas_tol;
  const int maxit = o.max_qp_iter > 0 ? o.max_qp_iter : 8 * M + 16;
  const int ink0 = sc.ink0;
  const double* rr = rv + (long long)kref * my * nit;
  const int si = oi < my ? oi : my - 1;  // signal row every lane loads (clamped)
  const double* psr = rr + (long long)si * nit;
  const double* psy = sc.yref + (long long)si * nit;
  GIState<16> gis;
  gi_reset<16>(gis);
#ifdef MPCT_DIAG
  gis.diag = o.diag;
#endif
  RegFactors rf;
  FOR4(r, rf.J[r] = 0.0;);
  rf.sB = lds + L.gb;
  long long iters = 0;
  int st = 0;
  double yd0 = 0.0;  // lane 4 i: y_i(t - 1)
  double uprev = 0.0;                                 // lane n < nu: u_n(t - 1)
  double j1 = 0.0, j22 = 0.0;
  double r_t = psr[0], yr_t = psy[0];
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): per-lane constants land before the loop

  for (int t = 0; t < nit; ++t) {
    lds_sync();  // rings of step t - 1 -> this step's plant terms and product
    // ---- plant (exact difference equations of every entry, lsim)
    const double hv = lds[pbase + ((t - pc) & pmask)];
    // the y update's reads of its own state (step t - 1's nabla y, nabla^2 y), issued with the ring
    // read so that their latency hides under the plant's reductions (every lane reads a valid slot)
    const double o1e = lds[L.xy + yoff + 1], o2e = lds[L.xy + yoff + 2];
    const double ye = row4_sum(pcoef * hv);  // y_e(t) on lane e of every row
    double yi = ye + dppd<kQx1>(ye);
    yi += dppd<kQx2>(yi);  // y_i(t) on every lane of quad i
    if (sm_lane() < 4 * my) lds[L.hist + kSmEOff + sm_lane() * ke + (t & (ke - 1))] = ye;
    PSTAMP(PROF_PLANT);
    // ---- y update and costs (lane 4 i): x = [y - r, nabla y, .., nabla^na y] (difference basis)
    {
      const int l = sm_lane();
      if ((l & ~12) == 0 && (l >> 2) < my) {
        // nabla^1,2 y(t-1) are the state's own entries of the last step (read before they are
        // overwritten); y(t-1) stays in a register
        double* xs = lds + L.xy + yoff;
        const double o1 = o1e, o2 = o2e;
        const double n1 = yi - yd0, n2 = n1 - o1, n3 = n2 - o2;
        xs[0] = yi - r_t;
        if (nyh > 1) xs[1] = n1;
        if (nyh > 2) xs[2] = n2;
        if (nyh > 3) xs[3] = n3;
        yd0 = yi;
        const double e1 = yi - yr_t;
        j1 = fma(e1, e1, j1);
        if (t >= ink0) j22 = fma(e1, e1, j22);
      }
    }
    // prefetch r(t+1), Yref(t+1): issued after this step's last use of r(t), Yref(t), so the
    // compiler's wait for them falls in the next step's y update
    const int tn = t + 1 < nit ? t + 1 : t;
    const double r_n = psr[tn], yr_n = psy[tn];
    lds_sync();  // y state -> product
    PSTAMP(PROF_YUPD);
    // ---- unconstrained minimiser dU = A x: quarter 0 the y part, quarters 1..3 the MV rings
    double xu;
    {
      const int h = (1 - t) & (kSmR - 1);  // ring window start: age-0 move
      const int xo = xoff + (sm_lane() >= 16 ? h : 0);
      const double2* av = reinterpret_cast<const double2*>(lds + aoff);
      const double* xv = lds + xo;
      double a0 = 0.0, a1 = 0.0;
      if ((sm_lane() & 15) < M) {  // A has M rows
#pragma unroll
        for (int p = 0; p < kSmR / 2; ++p) {
          const double2 a = av[p];
          a0 = fma(a.x, xv[2 * p], a0);
          a1 = fma(a.y, xv[2 * p + 1], a1);
        }
        if (sm_lane() < 16) {
#pragma unroll
          for (int p = kSmR / 2; p < kSmY / 2; ++p) {
            const double2 a = av[p];
            a0 = fma(a.x, xv[2 * p], a0);
            a1 = fma(a.y, xv[2 * p + 1], a1);
          }
        }
      }
      xu = row4_sum(a0 + a1);  // row m of A x on lanes m, m+16, m+32, m+48 (0 for m >= M)
    }
    PSTAMP(PROF_UNC);
    // ---- QP (gpc_qp16.h): u(t-1) of the row's MV from lane n
    double xq;
    const double up_row = __shfl(uprev, rcn.n, kWave);
    iters += gi_qp16<true, PAccT, true>(lds + L.rinv, lds + L.ra, M, Nu, rcn, up_row, xu, tol, maxit, &st, gis, rf,
                     kGiRebuild16, xq
#ifdef MPCT_PROFILE
                     , pacc, pprev
#endif
    );
    PSTAMP(PROF_QP);
    // ---- u update (lane n < nu): first move of MV n, plant input ring, past-control ring
    {
      const int l = sm_lane();
      const double du = __shfl(xq, l < nu ? l * Nu : 0, kWave);
      if (l < nu) {
        const double un = uprev + du;
        uprev = un;
        lds[L.hist + l * kSmU + (t & (kSmU - 1))] = un;
        double* ring = lds + L.ring + 2 * kSmR * l;
        const int p = (-t) & (kSmR - 1);
        ring[p] = du;
        ring[p + kSmR] = du;
      }
    }
    PSTAMP(PROF_UUPD);
    r_t = r_n;
    yr_t = yr_n;
  }
#ifdef MPCT_PROFILE
  if (lane == 0 && out.prof)
    for (int k = 0; k < PROF_N; ++k) out.prof[sim * PROF_N + k] = pacc.get(k);
#endif

  // ------------------------------------------------------------------ results (lane i <- lane 4 i)
  const double j1o = __shfl(j1, (lane & 3) * 4, kWave);
  const double j22o = __shfl(j22, (lane & 3) * 4, kWave);
  if (lane < my && !isfinite(j1o)) st |= MPCT_ST_NONFINITE_;
  const unsigned long long nf = __ballot(st & MPCT_ST_NONFINITE_);
  put_record(out, slot, S, sim, my, nu, lane, j1o, NAN, j22o, NAN, st | (nf ? MPCT_ST_NONFINITE_ : 0), iters);
}

}  // namespace mpct

// ------------------------------------------------------------------------------------------
// host-side launch
#include <string>

namespace mpct {

long long small_lds_bytes(const DevScenario& sc, int M) { return (long long)small_layout(sc, M).total * 8; }

// the M <= 16 class of a cost-only batch on a small scenario (launch_closed_loop); first: this
// launch also writes the statuses of skipped / bad-horizon candidates
int launch_small(const DevScenario& sc, long long C, int nref, const int* N2, const int* Nu, const double* delta,
                 const double* lambda, const double* r, const DevOpts& o, const DevResult& out, const int* perm,
                 int first, hipStream_t stream, std::string* err) {
  const int nu_cls = sc.numax < 16 / sc.nu ? sc.numax : 16 / sc.nu;
  const long long lds = small_lds_bytes(sc, sc.nu * nu_cls);
  const long long S = C * nref;
  hipLaunchKernelGGL(gpc_small_kernel, dim3((unsigned)S), dim3(kWave), (size_t)lds, stream, sc, C, nref, N2, Nu,
                     delta, lambda, r, perm, o, out, first);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    *err = std::string("kernel launch failed: ") + hipGetErrorString(e);
    return -3;
  }
  return 0;
}

}  // namespace mpct
