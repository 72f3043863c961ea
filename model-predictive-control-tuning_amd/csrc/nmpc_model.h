// nmpc_model.h — the Van de Vusse reactor (nmpc_vandevusse_state.m:43-82) as the NMPC kernels
// integrate it: the model constants, the state derivative with its forward tangent, one sample of
// fixed-step RK4 (oracle/nmpc_vdv.py rk4), and the Gauss-Newton globalisation constants.  Shared by
// nmpc_kernel.hip (one simulation per wave) and nmpc_rows.hip (one simulation per 16-lane row).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include "mpct_dev.h"
#include "wave_ops.h"

namespace mpct {

// Van de Vusse model constants, derived once per wave from the parameter table
struct VdV {
  double k10, k20, k30, e1, e2, e3, dab, dbc, dad, a, b, T0, ca0;
};

__device__ __forceinline__ VdV vdv_load(const double* p) {
  VdV P;
  P.k10 = p[NM_K10];
  P.k20 = p[NM_K20];
  P.k30 = p[NM_K30];
  P.e1 = p[NM_E1];
  P.e2 = p[NM_E2];
  P.e3 = p[NM_E3];
  P.dab = p[NM_DAB];
  P.dbc = p[NM_DBC];
  P.dad = p[NM_DAD];
  P.a = 1.0 / (p[NM_RHO] * p[NM_CP]);
  P.b = p[NM_KW] * p[NM_AR] / (p[NM_RHO] * p[NM_CP] * p[NM_V]);
  P.T0 = p[NM_T0];
  P.ca0 = p[NM_CA0];
  return P;
}


// state derivative f(x, u) (nmpc_vandevusse_state.m:64-82) and, with TAN, its directional
// derivative along (xd, ud)
template <bool TAN>
__device__ __forceinline__ void vdv_rhs(const VdV& P, const double x[3], const double u[2], const double xd[3],
                                        const double ud[2], double f[3], double fd[3]) {
  const double ca = x[0], cb = x[1], T = x[2];
  const double th = T + 273.15;
  // 1/th by v_rcp_f64 + two Newton steps (config 5: 326 -> 293 ms, profiles/r02i_nmpc_rhs_ab.txt);
  // an Estrin-scheme exp measured 306 ms (more VALU than the libm exp) and is not kept
  const double ith = rcp_nr(th);
  // a table-driven exp (16 entries of 2^(j/16) in LDS, degree-7 expm1, within 1 ulp) took fewer
  // instructions than the library's but measured slower, config 5 24.1 -> 23.5 k sims/s and the N = 31
  // loop 30.2 -> 31.2 ms: its LDS load sits on the stage's chain (profiles/r06p_nmpc_ab.txt)
  const double ex1 = exp(P.e1 * ith);
  const double k1 = P.k10 * ex1;
  const double k2 = P.k20 * (P.e2 == P.e1 ? ex1 : exp(P.e2 * ith));  // E1 = E2 in the reference model
  const double k3 = P.k30 * exp(P.e3 * ith);
  const double fov = u[0], tk = u[1];
  f[0] = fov * (P.ca0 - ca) - k1 * ca - k3 * ca * ca;
  f[1] = -fov * cb + k1 * ca - k2 * cb;
  f[2] = P.a * (k1 * ca * P.dab + k2 * cb * P.dbc + k3 * ca * ca * P.dad) + fov * (P.T0 - T) + P.b * (tk - T);
  if (TAN) {
    const double ith2 = ith * ith;
    const double Td = xd[2];
    const double k1d = -P.e1 * ith2 * k1 * Td, k2d = -P.e2 * ith2 * k2 * Td, k3d = -P.e3 * ith2 * k3 * Td;
    const double cad = xd[0], cbd = xd[1];
    fd[0] = ud[0] * (P.ca0 - ca) - fov * cad - k1d * ca - k1 * cad - k3d * ca * ca - 2.0 * k3 * ca * cad;
    fd[1] = -ud[0] * cb - fov * cbd + k1d * ca + k1 * cad - k2d * cb - k2 * cbd;
    fd[2] = P.a * (k1d * ca * P.dab + k1 * cad * P.dab + k2d * cb * P.dbc + k2 * cbd * P.dbc + k3d * ca * ca * P.dad +
                   2.0 * k3 * ca * cad * P.dad) +
            ud[0] * (P.T0 - T) - fov * Td + P.b * (ud[1] - Td);
  }
}

// one sample Ts of classical RK4 with nsub sub-steps (oracle/nmpc_vdv.py rk4), tangent optional
template <bool TAN>
__device__ __forceinline__ void vdv_rk4(const VdV& P, double h, int nsub, double x[3], const double u[2],
                                        double xd[3], const double ud[2]) {
  for (int s = 0; s < nsub; ++s) {
    double k1[3], k2[3], k3[3], k4[3], K1[3], K2[3], K3[3], K4[3], xs[3], Xs[3];
    vdv_rhs<TAN>(P, x, u, xd, ud, k1, K1);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      xs[i] = x[i] + 0.5 * h * k1[i];
      if (TAN) Xs[i] = xd[i] + 0.5 * h * K1[i];
    }
    vdv_rhs<TAN>(P, xs, u, Xs, ud, k2, K2);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      xs[i] = x[i] + 0.5 * h * k2[i];
      if (TAN) Xs[i] = xd[i] + 0.5 * h * K2[i];
    }
    vdv_rhs<TAN>(P, xs, u, Xs, ud, k3, K3);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      xs[i] = x[i] + h * k3[i];
      if (TAN) Xs[i] = xd[i] + h * K3[i];
    }
    vdv_rhs<TAN>(P, xs, u, Xs, ud, k4, K4);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      x[i] = x[i] + (h / 6.0) * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
      if (TAN) xd[i] = xd[i] + (h / 6.0) * (K1[i] + 2.0 * K2[i] + 2.0 * K3[i] + K4[i]);
    }
  }
}

__device__ __forceinline__ double sel3(const double x[3], int i) { return i == 0 ? x[0] : (i == 1 ? x[1] : x[2]); }

// Gauss-Newton globalisation (oracle/nmpc_vdv.py LS_MAX, LS_C1, LS_FLAT)
constexpr int kLsMax = 12;
constexpr double kLsC1 = 1e-4;
constexpr double kLsFlat = 1e-14;

// LDS layout (doubles) of one simulation at QP size M with G point buffers
struct NmLayout {
  int ri, jt, ra, dv, xc, uo, nv, bits, grp, gsz, total;
  // offsets inside one point buffer: R, c = Q'r, absolute moves, increments, rate residuals,
  // predicted states, their sensitivities
  int g_rr, g_cv, g_u, g_v, g_rw, g_xp, g_sx;
};
// N: prediction horizon (the state-bound rows: predicted states x_i and dx_i/dv, i = 1..N).
// G: point buffers (nm_groups)
__host__ __device__ inline NmLayout nm_layout(int M, int N, int G) {
  NmLayout L;
  int o = 0;
  auto take = [&](int n) { int r = o; o += (n + 1) & ~1; return r; };
  L.ri = take(M * (M + 1) / 2);  // R^-1, upper triangle packed by rows (nm_up)
  L.jt = take(M * M);
  L.ra = take((M * (M + 3)) / 2);  // R_A, packed upper Hessenberg (gi_core.h RAPacked, ra_packed_size)
  L.dv = take(M + 1);
  L.xc = take(M + 1);
  L.uo = take(M + 1);  // absolute moves of the open-loop solution (Info.MVopt)
  L.nv = take(M + 1);  // staged normal of a state-bound row
  L.bits = take((6 * N + 63) / 64);  // active state-bound rows (32-bit words)
  const int w = G > 1 ? 16 : M + 1;  // per-lane vectors of a point (16-lane rows when grouped)
  int g = 0;
  auto gtake = [&](int n) { int r = g; g += (n + 1) & ~1; return r; };
  L.g_rr = gtake(M * (M + 1) / 2);  // R of the Gauss-Newton least-squares QR (upper, packed: nm_up)
  L.g_cv = gtake(w);
  L.g_u = gtake(w);
  L.g_v = gtake(w);
  L.g_rw = gtake(w);
  L.g_xp = gtake(3 * N);
  L.g_sx = gtake(3 * N * M);
  L.gsz = g;
  L.grp = o;
  o += G * g;
  L.total = (o + 1) & ~1;
  return L;
}

// entry (i, k), k >= i, of an upper-triangular M x M matrix packed row by row: R and R^-1 keep only
// their upper triangles (round 6: 3.4 KB less at M = 15 with four point buffers, 7 KB at M = 30, so
// more simulations fit the 40 KB of four workgroups per CU; the lower entries were never read)
__host__ __device__ inline int nm_up(int i, int k, int M) { return i * M - ((i * (i - 1)) >> 1) + (k - i); }

// point buffers of a simulation: four (one per 16-lane row) when they fit 40 KB, i.e. four
// workgroups per CU, the one-wave-per-SIMD occupancy of this kernel; else two while they fit the
// 64 KiB a launch may hold without the MaxDynamicSharedMemorySize opt-in; else one, the single-
// point pass of the M <= 32 class (long horizons: G = 2 doubles the 3 N M sensitivities, so at
// nu = 2, N = 127 the M <= 15 class would otherwise need 101 KB against 46 KB for G = 1)
__host__ __device__ inline int nm_groups(int M, int N) {
  if (M > 15) return 1;
  if (nm_layout(M, N, 4).total * 8 <= 40 * 1024) return 4;
  return nm_layout(M, N, 2).total * 8 <= 64 * 1024 ? 2 : 1;
}


}  // namespace mpct
