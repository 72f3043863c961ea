/* Plain-C client of the libmpct ABI (include/mpct.h), the way a MATLAB loadlibrary/calllib or MEX
 * host binds it: no torch, no C++ types.
 *   1. The linear Shell 3x3 scenario of Shell3x3.m (the BASELINE metric's plant) from the saved
 *      mpc object's scaled discrete tf (Shell3x3_Tuning_25Jul2023_12_06.mat: tfdata rows, IODelay)
 *      and its scaled MV bounds, with NO CARIMA tables (abi 5: the library derives them), the
 *      kernel-instance query, and -- with "eval" -- three candidates scored through
 *      mpct_eval_batch (J1 against yref = r = L*Xsp here).
 *   2. The Van de Vusse NMPC scenario of VanDeVusse_NMPC.m from plain arrays
 *      (mpct_nmpc_scenario_create), its argument errors, and -- with "eval" -- three candidates.
 * Prints status and J1 (GAM_fun.m:110-111) per candidate.
 *   usage: mpct_c_demo [eval]      exit 0 on success */
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "mpct.h"

#define NIT 60
#define LNIT 500

/* Shell3x3_Tuning_25Jul2023_12_06.mat: Tuning_Parameters.mpcobj.Model.Plant (L*Pz*R, c2d ZOH) */
static const double SH_NUM[9][2] = {
    {0.02313052619372795, 0.06667958558934375}, {0.0, 0.013710194313372143}, {0.02089018186516949, 0.06022122704814364},
    {0.058828715846932514, 0.0565220089046257}, {0.02173580108248058, 0.021023216763849436},
    {0.0294987546979058, 0.08419778882992246}, {0.0, 0.1963360266878832}, {0.032116113806741245, 0.03068897122230742},
    {0.0, 0.3338832924071783}};
static const double SH_DEN[9][2] = {
    {1.0, -0.9231163463866358}, {1.0, -0.9355069850316178}, {1.0, -0.9231163463866358},
    {1.0, -0.9231163463866358}, {1.0, -0.9355069850316178}, {1.0, -0.9048374180359595},
    {1.0, -0.8858460329277068}, {1.0, -0.9131007162822624}, {1.0, -0.8101577349324267}};
static const int32_t SH_DELAY[9] = {7, 7, 7, 5, 4, 4, 5, 6, 0};
static const double SH_L[3] = {0.43577812475231503, 0.4205588479390135, 0.5932860051199568};
static const double SH_UMIN[3] = {-1.510877401316376, -3.628338208043142, -2.4288171452857927};
static const double SH_UMAX[3] = {0.755438700658188, 1.814169104021571, 1.2144085726428964};
static const double SH_DUMAX[3] = {0.0755438700658188, 0.18141691040215713, 0.12144085726428963};

/* Xsp of Shell3x3.m:89-92 (1-based inclusive ranges, later ones overwrite), scaled by L */
static void shell_xsp(double* r) {
  const double lv[3][4] = {{0.2, 0.0, 0.1, 0.0}, {0.2, 0.4, 0.3, 0.0}, {0.2, 0.1, 0.0, 0.0}};
  for (int i = 0; i < 3; ++i)
    for (int t = 0; t < LNIT; ++t) {
      double x = 0.0;
      if (t >= 9 && t < 80) x = lv[i][0];
      if (t >= 79 && t < 200) x = lv[i][1];
      if (t >= 199 && t < 400) x = lv[i][2];
      if (t >= 399) x = lv[i][3];
      r[i * LNIT + t] = SH_L[i] * x;
    }
}

static int shell3x3_demo(int do_eval) {
  static double r[3 * LNIT];
  shell_xsp(r);
  mpct_dtf P[9];
  for (int e = 0; e < 9; ++e) {
    P[e].len = 2;
    P[e].num = SH_NUM[e];
    P[e].den = SH_DEN[e];
    P[e].delay = SH_DELAY[e];
  }
  double dumin[3];
  for (int n = 0; n < 3; ++n) dumin[n] = -SH_DUMAX[n];
  const int32_t n1[3] = {1, 1, 1};
  mpct_scenario_desc d;
  memset(&d, 0, sizeof d);
  d.abi_version = MPCT_ABI_VERSION;
  d.my = 3;
  d.nu = 3;
  d.nit = LNIT;
  d.n2_max = 30;
  d.nu_max = 5;
  d.weights_squared = 1;
  d.vns_ink = 10;
  d.n1 = n1;
  d.plant = P;
  d.model = P;
  d.du_min = dumin;
  d.du_max = SH_DUMAX;
  d.u_min = SH_UMIN;
  d.u_max = SH_UMAX;
  d.yref = r;  /* na / carima_A / nb / carima_B / dp stay NULL: derived by the library */
  mpct_scenario* s = NULL;
  if (mpct_scenario_create(&d, &s) != MPCT_OK || !s) {
    printf("linear create failed: %s\n", mpct_last_error());
    return 10;
  }
  char name[128];
  mpct_opts o = {0, 0, 0, -1, 0.0};
  if (mpct_kernel_instance(s, &o, name, (int32_t)sizeof name) < 0) return 11;
  printf("linear instance %s\n", name);
  if (do_eval) {
    const int32_t N[3] = {30, 30, 30}, Nu[3] = {5, 5, 5};
    const double delta[9] = {0.010659948215964849, 0.004019856475662751, 0.0007926546087416782, 0.5, 0.1, 0.01,
                             1.0, 1.0, 1.0};
    const double lambda[9] = {9.247457388705409e-05, 0.0005523146971406108, 0.0015219790494510478, 0.001, 0.01,
                              0.002, 0.1, 0.1, 0.1};
    double J1[9];
    int32_t status[3];
    mpct_result res;
    memset(&res, 0, sizeof res);
    res.J1 = J1;
    res.status = status;
    const int rc = mpct_eval_batch(s, 3, N, Nu, delta, lambda, 1, r, NULL, &o, &res);
    if (rc != MPCT_OK) {
      printf("linear eval failed (%d): %s\n", rc, mpct_last_error());
      mpct_scenario_destroy(s);
      return 12;
    }
    for (int c = 0; c < 3; ++c)
      printf("lin %d status %d J1 %.17g %.17g %.17g\n", c, status[c], J1[3 * c], J1[3 * c + 1], J1[3 * c + 2]);
  }
  mpct_scenario_destroy(s);
  return 0;
}

int main(int argc, char** argv) {
  const int do_eval = argc > 1 && strcmp(argv[1], "eval") == 0;
  printf("abi %d\n", mpct_abi_version());
  if (mpct_abi_version() != MPCT_ABI_VERSION) return 1;
  const int lrc = shell3x3_demo(do_eval);
  if (lrc) return lrc;
  /* VanDeVusse_NMPC.m:54-90: x0 = steady state at u0 (fsolve), bounds, scale factors, r */
  const double x0[3] = {1.246290177008599, 0.9052268854543595, 134.95095689423889};
  const double u0[2] = {20.0, 130.0}, umin[2] = {0.0, 40.0}, umax[2] = {150.0, 150.0};
  const double xmin[3] = {0.0, 0.0, 40.0}, xmax[3] = {6.0, 1.2, 150.0};
  const double ys[2] = {1.2, 110.0}, us[2] = {150.0, 110.0};
  const int32_t xc[2] = {2, 3};
  static double yref[2 * NIT], r[2 * NIT];
  for (int t = 0; t < NIT; ++t) {
    r[t] = t >= 9 ? 1.0 : x0[1];
    r[NIT + t] = t >= 40 ? 130.0 : x0[2];
    yref[t] = r[t];
    yref[NIT + t] = r[NIT + t];
  }
  mpct_nmpc_desc d;
  memset(&d, 0, sizeof d);
  d.abi_version = MPCT_ABI_VERSION;
  d.model = MPCT_NMPC_VANDEVUSSE;
  d.nx = 3;
  d.ny = 2;
  d.nu = 2;
  d.params = NULL; /* the reference's parameters */
  d.xc = xc;
  d.ts = 0.05;
  d.nsub = 10;
  d.x0 = x0;
  d.u0 = u0;
  d.u_min = umin;
  d.u_max = umax;
  d.x_min = xmin;
  d.x_max = xmax;
  d.y_scale = ys;
  d.u_scale = us;
  d.n_max = 31;
  d.nu_max = 15;
  d.nit = NIT;
  d.yref = yref;
  d.vns_ink = 10;
  mpct_scenario* s = NULL;
  /* argument errors come back as negative codes with a message, before anything is allocated */
  d.nu_max = 17;
  if (mpct_nmpc_scenario_create(&d, &s) != MPCT_ERANGE || s) return 2;
  printf("expected error: %s\n", mpct_last_error());
  d.nu_max = 15;
  d.abi_version = 3;
  if (mpct_nmpc_scenario_create(&d, &s) != MPCT_EINVAL) return 3;
  d.abi_version = MPCT_ABI_VERSION;
  int rc = mpct_nmpc_scenario_create(&d, &s);
  if (rc != MPCT_OK || !s) {
    printf("create failed: %s\n", mpct_last_error());
    return 4;
  }
  printf("lds bytes (N=31, Nu=15): %lld\n", (long long)mpct_lds_bytes(s, 31, 15));
  if (do_eval) {
    const int32_t N[3] = {3, 12, 25}, Nu[3] = {2, 4, 7};
    const double delta[6] = {0.09302224780430422, 0.11333840205801392, 1.0, 0.5, 0.3, 2.0};
    const double lambda[6] = {0.245996189227521, 0.12310801096548595, 0.05, 0.02, 0.1, 0.1};
    double J1[6];
    int32_t status[3];
    mpct_opts o = {0, 0, 0, -1, 0.0};
    mpct_result res;
    memset(&res, 0, sizeof res);
    res.J1 = J1;
    res.status = status;
    rc = mpct_eval_batch(s, 3, N, Nu, delta, lambda, 1, r, NULL, &o, &res);
    if (rc != MPCT_OK) {
      printf("eval failed (%d): %s\n", rc, mpct_last_error());
      mpct_scenario_destroy(s);
      return 5;
    }
    for (int c = 0; c < 3; ++c) printf("cand %d status %d J1 %.17g %.17g\n", c, status[c], J1[2 * c], J1[2 * c + 1]);
  }
  mpct_scenario_destroy(s);
  printf("ok\n");
  return 0;
}
