// gpc_record.h — one simulation's cost record (GAM_fun.m:110-111 J1, VNS2.m:172-191 j21 / j22 /
// Jnu, status, QP iterations), written by the linear closed-loop kernels either to the caller's
// arrays at index `sim` or, for ordered launches, to the XCD-major staging row of workgroup slot
// `slot` (DevResult::stage; unpermute_results gathers it back into the caller's order).
#pragma once
#include <hip/hip_runtime.h>

#include "mpct_dev.h"

namespace mpct {

// lanes i < my hold the output entries, lanes n < nu the MV entries, lane 0 status and iterations
__device__ __forceinline__ void put_record(const DevResult& out, long long slot, long long S, long long sim,
                                           int my, int nu, int lane, double j1v, double j21v, double j22v,
                                           double jnuv, int status, long long itv) {
  if (out.stage) {
    const StageRow& R = out.srow;
    double* row = out.stage + xcd_row(slot, S) * R.w;
    if (lane < my) {
      if (R.j1 >= 0) row[R.j1 + lane] = j1v;
      if (R.j21 >= 0) row[R.j21 + lane] = j21v;
      if (R.j22 >= 0) row[R.j22 + lane] = j22v;
    }
    if (lane < nu && R.jnu >= 0) row[R.jnu + lane] = jnuv;
    if (lane == 0) {
      if (R.st >= 0) row[R.st] = (double)status;
      if (R.it >= 0) row[R.it] = (double)itv;
    }
    return;
  }
  if (lane < my) {
    if (out.J1) out.J1[sim * my + lane] = j1v;
    if (out.j21) out.j21[sim * my + lane] = j21v;
    if (out.j22) out.j22[sim * my + lane] = j22v;
  }
  if (lane < nu && out.Jnu) out.Jnu[sim * nu + lane] = jnuv;
  if (lane == 0) {
    if (out.status) out.status[sim] = status;
    if (out.qp_iters) out.qp_iters[sim] = itv;
  }
}

}  // namespace mpct
