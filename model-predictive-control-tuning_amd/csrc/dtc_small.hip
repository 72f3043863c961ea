// dtc_small.hip — the DTC-GPC closed loop of small plants (WoodBerry
// with its plant-only disturbance and Monte-Carlo plant variants): one wavefront per simulation,
// every per-step quantity in a fixed lane layout, and no QP.
//
// DTC_GPC_WW.m is the unconstrained loop: deltaU = Km * (Ref - yf) (:149) with Km the first-move rows
// of K = (H'QH + W) \ H'Q (:98-105).  So a scenario in DTC mode whose move bounds are all infinite
// (what DTC_GPC_WW.m restates) needs, per step, only the nu first-move rows of the gain: no QP, no
// R^-1, no factor state.  The host marks such scenarios `small_dtc` (mpct_host.cpp dtc_small_plant):
// DTC mode, my <= 2 outputs, nu <= 2 MVs, nu + nq <= 4 plant inputs (MVs and plant-only
// disturbances, no measured disturbances), every plant variant's, Pz's and Gz's entry <= 4 terms,
// filters Fr_i of <= 4 taps, y difference state <= 4 per output, past-control registers <= 8 per
// MV, cost-only batches.  Everything else runs gpc_closed_loop_kernel<MAXM, true, ...> unchanged.
//
// Lane layout (lane L = 16 k + e, e = 4 q + p), the gpc_small.hip scheme extended by the predictor:
//   * quads q = i < my: term k of plant entry (output i, input p) of this simulation's plant variant
//     (Monte-Carlo draw kref % nvar): a numerator tap b u_p(t - c) or a denominator tap -a y_e(t - c),
//     one LDS read from a history ring; input p >= nu is a plant-only disturbance (its ring is fed
//     from v);
//   * quad q = 2 + i: p = 0, 1 the model entries Pz(i, p), p = 2, 3 the dead-time-free Gz(i, p - 2)
//     (OptimalPredictor2.m: lsim(Pz, u), lsim(Gz, u) as recursions on the controller's own inputs).
//   One v_permlane16/32_swap sum over the four term rows gives every entry's output; one DPP stage
//   pairs them (Pz_i, Gz_i on lanes 8 + 4i, 10 + 4i) and a second sums each plant quad (y_i).
//   Output lane 4 i fetches Pz_i and Gz_i by DPP row shifts, runs the robustness filter
//   yfr = Fr_i (y_i - Pz_i) (mimofilter.m, coefficients in LDS) and drives the free response with
//   the predictor output yp = Gz_i + yfr (OptimalPredictor2.m:24-40) while the costs use y_i.
//   * dU(first moves) = Km x: lane (n, g), n < nu, quarter g of row n of the gain (quarter 0 the y
//   part, quarters 1..3 MV g - 1's past-control ring), 12 FMAs, one permlane sum: row n on lane n.
#include <hip/hip_runtime.h>
#include <math.h>

#include "mpct_dev.h"
#include "wave_ops.h"
#include "gpc_prologue.h"
#include "gpc_record.h"

namespace mpct {

// LDS layout of one simulation (doubles): R (the prologue's M x M scratch), the first-move rows of
// the gain, the y part of x, the past-control rings (two copies each), the input rings [4][kSmU] |
// the entry output rings [16][ke] (from kDtcEOff), the filters' coefficients [my][8] (fb 0..3,
// fa 0..3) and their input / output rings [my][2][4]: 4.6 KB at M = 16 (Shell-sized plants)
struct DtcLayout {
  int R, A, xy, ring, hist, fr, frh, total;
};
__host__ __device__ inline DtcLayout dtc_layout(const DevScenario& sc, int M) {
  DtcLayout L;
  int o = 0;
  auto take = [&](int n) { int r = o; o += (n + 1) & ~1; return r; };
  L.R = take(M * M);
  L.A = take(2 * kSmA);
  L.xy = take(kSmY);
  L.ring = take(3 * 2 * kSmR);  // three MVs' worth: the product's quarter 3 reads zeros for nu = 2
  L.hist = take(kDtcEOff + 16 * sc.sm_ke);
  L.fr = take(2 * 8);
  L.frh = take(2 * 2 * 4);
  L.total = (o + 1) & ~1;
  return L;
}

// opaque lane id: predicates derived from it are recomputed where used, not kept live across the
// step loop (gpc_small.hip sm_lane)
__device__ __forceinline__ int dtc_lane() {
  int l = threadIdx.x;
  asm volatile("" : "+v"(l));
  return l;
}

// waves per SIMD the launch bounds ask for, and the prologue's Householder block (gpc_prologue.h
// kHB): unbounded the <16> instance needs 119 VGPRs (four waves; 22.9 ms for config 4's 320,000
// simulations); five waves with 8-row blocks spill 80 B per lane in the prologue (21.3 ms, but 1.33 GB
// of scratch write-backs per evaluation against 10 MB of records); four waves with 4-row blocks fit
// 103 VGPRs without a spill: 21.5 ms and 10.2 MB written (profiles/r06i_dtc_prologue_ab.txt)
#ifndef MPCT_DTC_HB
#define MPCT_DTC_HB 4
#endif
#ifndef MPCT_DTC_W16
#define MPCT_DTC_W16 4
#endif
#ifndef MPCT_DTC_W32
#define MPCT_DTC_W32 3
#endif
template <int MAXM>
__global__ void __launch_bounds__(64, MAXM <= 16 ? MPCT_DTC_W16 : MPCT_DTC_W32)
    dtc_small_kernel(const DevScenario sc, long long C, int nref, const int* __restrict__ N2v,
                     const int* __restrict__ Nuv, const double* __restrict__ deltav,
                     const double* __restrict__ lambdav, const double* __restrict__ rv,
                     const double* __restrict__ vv, const int* __restrict__ perm, const DevOpts o,
                     const DevResult out, int mlo, int first) {
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
  if (M <= mlo || M > MAXM) return;  // the other class launch simulates it
  const DtcLayout L = dtc_layout(sc, M);
  for (int e = lane; e < L.total - L.A; e += kWave) lds[L.A + e] = 0.0;  // gain pads, state, rings
  if (lane < 2 * 8) {  // filter coefficients: fb (taps 0..3), then fa (taps 0..3), zero-padded
    const int i = lane >> 3, k = lane & 7;
    lds[L.fr + lane] = i < my ? sc.sm_fr[i * 8 + k] : 0.0;
  }
  lds_sync();

  // ------------------------------------------------------------------ prologue (gpc_prologue.h):
  // the first-move rows of A only (row n = A row n Nu), no R^-1
  if (!gpc_prologue<MAXM, false, false, true, MPCT_DTC_HB>(sc, lane, M, Nu, N2, deltav + c * my, lambdav + c * nu, lds + L.R,
                                              nullptr, lds + L.A, kSmA, sc.sm_acol)) {
    write_nan(MPCT_ST_NONFINITE_);
    return;
  }

  // per-lane constants of the step loop: this lane's term of this simulation's plant variant
  const int pv = sc.nvar > 1 ? (kref % sc.nvar) * kWave : 0;
  const double pcoef = sc.sm_coef[pv + lane];
  const int pbase = L.hist + sc.sm_hoff[pv + lane];
  const int pc = sc.sm_hc[pv + lane], pmask = sc.sm_hmask[pv + lane];
  const int ke = sc.sm_ke;
  const int oi = (lane >> 2) & 3;  // output lane 4 i
  const int yoff = oi < my ? sc.yoff[oi] : 0;
  const int nyh = oi < my ? sc.nyhi[oi] : 0;
  const int qm = lane & 15, qg = lane >> 4;  // product lane (n, g)
  const int aoff = L.A + qm * kSmA + (qg ? kSmY + kSmR * (qg - 1) : 0);
  const int xoff = qg ? L.ring + 2 * kSmR * (qg - 1) : L.xy;
  const int ink0 = sc.ink0;
  const int nq = sc.nd;  // ring-fed plant inputs: the plant-only disturbances (no MDs here)
  const double* rr = rv + (long long)kref * my * nit;
  const int si = oi < my ? oi : my - 1;
  const double* psr = rr + (long long)si * nit;
  const double* psy = sc.yref + (long long)si * nit;
  // lane nu + k < nu + nq: disturbance k of this simulation's signal set
  const int qk = lane - nu < nq && lane >= nu ? lane - nu : 0;
  const double* psq = vv ? vv + ((long long)kref * nq + qk) * nit : nullptr;
  double yd0 = 0.0;    // lane 4 i: yp_i(t - 1)
  double uprev = 0.0;  // lane n < nu: u_n(t - 1)
  double j1 = 0.0, j22 = 0.0;
  double r_t = psr[0], yr_t = psy[0];
  double q_t = psq ? psq[0] : 0.0;
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): per-lane constants land before the loop

  for (int t = 0; t < nit; ++t) {
    // the disturbances known at t (DTC_GPC_WW.m:123-132: the plant sees q(t)), then the hand-off of
    // step t - 1's rings to this step's terms
    {
      const int l = dtc_lane();
      if (l >= nu && l < nu + nq) lds[L.hist + l * kSmU + (t & (kSmU - 1))] = q_t;
    }
    const int tn = t + 1 < nit ? t + 1 : t;
    const double q_n = psq ? psq[tn] : 0.0;
    lds_sync();
    // ---- plant entries, Pz and Gz: one term per lane, summed over the four term rows
    const double hv = lds[pbase + ((t - pc) & pmask)];
    const double o1e = lds[L.xy + yoff + 1], o2e = lds[L.xy + yoff + 2];
    const double ye = row4_sum(pcoef * hv);  // entry e's output on lane e of every row
    const double s1 = ye + dppd<kQx1>(ye);  // pair sums: Pz_i on lane 8 + 4i, Gz_i on lane 10 + 4i
    const double yq = s1 + dppd<kQx2>(s1);  // quad sums: y_i on the lanes of quad i < my
    const double pz = dppd<0x108>(s1);      // row_shl:8  -> lane 4i holds Pz_i
    const double gz = dppd<0x10A>(s1);      // row_shl:10 -> lane 4i holds Gz_i
    if (dtc_lane() < 16) lds[L.hist + kDtcEOff + dtc_lane() * ke + (t & (ke - 1))] = ye;
    // ---- predictor, y update and costs (lane 4 i)
    {
      const int l = dtc_lane();
      if ((l & ~12) == 0 && (l >> 2) < my) {
        const int i = l >> 2;
        // yfr = Fr_i (y - Pz_i): zero-padded taps, the general kernel's order (fb taps, then fa)
        const double* fb = lds + L.fr + i * 8;
        double* eh = lds + L.frh + i * 8;  // eM ring [4], then the filter output ring [4]
        double* fh = eh + 4;
        const double em = yq - pz;
        eh[t & 3] = em;
        double yfr = 0.0;
        yfr = fma(fb[0], em, yfr);
        yfr = fma(fb[1], eh[(t - 1) & 3], yfr);
        yfr = fma(fb[2], eh[(t - 2) & 3], yfr);
        yfr = fma(fb[3], eh[(t - 3) & 3], yfr);
        yfr = fma(-fb[5], fh[(t - 1) & 3], yfr);
        yfr = fma(-fb[6], fh[(t - 2) & 3], yfr);
        yfr = fma(-fb[7], fh[(t - 3) & 3], yfr);
        fh[t & 3] = yfr;
        const double ym = gz + yfr;
        double* xs = lds + L.xy + yoff;
        const double n1 = ym - yd0, n2 = n1 - o1e, n3 = n2 - o2e;
        xs[0] = ym - r_t;
        if (nyh > 1) xs[1] = n1;
        if (nyh > 2) xs[2] = n2;
        if (nyh > 3) xs[3] = n3;
        yd0 = ym;
        const double e1 = yq - yr_t;  // the costs use the plant output
        j1 = fma(e1, e1, j1);
        if (t >= ink0) j22 = fma(e1, e1, j22);
      }
    }
    const double r_n = psr[tn], yr_n = psy[tn];
    lds_sync();  // y state -> product
    // ---- first moves dU = Km x: quarter 0 the y part, quarters 1..3 the MV rings
    double du;
    {
      const int h = (1 - t) & (kSmR - 1);
      const int xo = xoff + (dtc_lane() >= 16 ? h : 0);
      const double2* av = reinterpret_cast<const double2*>(lds + aoff);
      const double* xv = lds + xo;
      double a0 = 0.0, a1 = 0.0;
      if ((dtc_lane() & 15) < nu) {
#pragma unroll
        for (int p = 0; p < kSmR / 2; ++p) {
          const double2 a = av[p];
          a0 = fma(a.x, xv[2 * p], a0);
          a1 = fma(a.y, xv[2 * p + 1], a1);
        }
        if (dtc_lane() < 16) {
#pragma unroll
          for (int p = kSmR / 2; p < kSmY / 2; ++p) {
            const double2 a = av[p];
            a0 = fma(a.x, xv[2 * p], a0);
            a1 = fma(a.y, xv[2 * p + 1], a1);
          }
        }
      }
      du = row4_sum(a0 + a1);  // first move of MV n on lane n
    }
    // ---- u update (lane n < nu): plant input ring, past-control ring
    {
      const int l = dtc_lane();
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
    r_t = r_n;
    yr_t = yr_n;
    q_t = q_n;
  }

  // ------------------------------------------------------------------ results (lane i <- lane 4 i)
  const double j1o = __shfl(j1, (lane & 3) * 4, kWave);
  const double j22o = __shfl(j22, (lane & 3) * 4, kWave);
  int st = 0;
  if (lane < my && !isfinite(j1o)) st |= MPCT_ST_NONFINITE_;
  const unsigned long long nf = __ballot(st & MPCT_ST_NONFINITE_);
  put_record(out, slot, S, sim, my, nu, lane, j1o, NAN, j22o, NAN, nf ? MPCT_ST_NONFINITE_ : 0, 0);
}

}  // namespace mpct

// ------------------------------------------------------------------------------------------
// host-side launch
#include <string>

namespace mpct {

long long dtc_small_lds_bytes(const DevScenario& sc, int M) { return (long long)dtc_layout(sc, M).total * 8; }

// one QP-size class (M <= 16 or 16 < M <= 32) of a cost-only batch on a small_dtc scenario
// (launch_closed_loop); first: this launch also writes the statuses of skipped / bad-horizon candidates
int launch_dtc_small(const DevScenario& sc, int cls, long long C, int nref, const int* N2, const int* Nu,
                     const double* delta, const double* lambda, const double* r, const double* v, const DevOpts& o,
                     const DevResult& out, const int* perm, int mlo, int first, hipStream_t stream, std::string* err) {
  const int nu_cls = sc.numax < cls / sc.nu ? sc.numax : cls / sc.nu;
  const long long lds = dtc_small_lds_bytes(sc, sc.nu * nu_cls);
  const long long S = C * nref;
  if (cls == 16)
    hipLaunchKernelGGL(dtc_small_kernel<16>, dim3((unsigned)S), dim3(kWave), (size_t)lds, stream, sc, C, nref, N2, Nu,
                       delta, lambda, r, v, perm, o, out, mlo, first);
  else
    hipLaunchKernelGGL(dtc_small_kernel<32>, dim3((unsigned)S), dim3(kWave), (size_t)lds, stream, sc, C, nref, N2, Nu,
                       delta, lambda, r, v, perm, o, out, mlo, first);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    *err = std::string("kernel launch failed: ") + hipGetErrorString(e);
    return -3;
  }
  return 0;
}

}  // namespace mpct
