/* Plain-C client of the libmpct ABI (include/mpct.h), the way a MATLAB loadlibrary/calllib or MEX
 * host binds it: no torch, no C++ types.  Builds the Van de Vusse NMPC scenario of
 * VanDeVusse_NMPC.m from plain arrays (mpct_nmpc_scenario_create), checks the argument errors,
 * and -- with "eval" on a GPU host -- scores three candidates through mpct_eval_batch and prints
 * status and J1 (GAM_fun.m:110-111) per candidate.
 *   usage: mpct_c_demo [eval]      exit 0 on success */
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "mpct.h"

#define NIT 60

int main(int argc, char** argv) {
  const int do_eval = argc > 1 && strcmp(argv[1], "eval") == 0;
  printf("abi %d\n", mpct_abi_version());
  if (mpct_abi_version() != MPCT_ABI_VERSION) return 1;
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
