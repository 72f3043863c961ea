// work_order.hip — heaviest-first dispatch order of a candidate batch (see work_order.h).
#include <hipcub/hipcub.hpp>

#include "work_order.h"

namespace mpct {

// ---- dispatch order (longest-processing-time first).  The workgroups of a launch start in slot
// order and a batch larger than the resident slots (4096 simulations, 12 slots per CU at the
// metric) runs a second, partial round, so a long simulation that starts late sets the kernel
// time.  Simulation time grows with the QP size M and with the QP work, which the candidates'
// weights predict: the more the tracking weights dominate the move-rate weights, the more often
// the bounds bind.  Key (ascending = heavier first): ~(M << 20 | q(mean_j log2(max_i|delta_i| /
// |lambda_j|))); invalid candidates last.  Measured on the metric batch (tools/order_probe.py):
// grid order 5.36 ms, this key 3.9 ms, ideal (measured QP work, descending) 3.58 ms.
// NMPC (config 5, tools/order_probe5.py, tools/nmpc_key_ab.sh): the Gauss-Newton iteration count
// falls as the weight ratio grows (Spearman -0.54) while the work per iteration grows with the
// horizon N and the QP size; score log(N Nu) - 0.1 a.  Closed loop of the 4096 grid: grid order
// 506 ms, N Nu order 376 ms, this score 367 ms, ideal (measured work) 345 ms.
__global__ void order_keys(int kind, long long C, int my, int nu, const int* __restrict__ N2,
                           const int* __restrict__ Nu, const double* __restrict__ delta,
                           const double* __restrict__ lambda, unsigned* __restrict__ key, int* __restrict__ idx) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  unsigned k = 0xffffffffu;
  const int n2 = N2[c], nuc = Nu[c];
  if (n2 > 0 && nuc > 0 && nuc <= 64) {
    // a = mean_j log2(max_i |delta_i| / |lambda_j|): how much tracking dominates move suppression
    double dmax = 0.0;
    for (int i = 0; i < my; ++i) dmax = fmax(dmax, fabs(delta[c * my + i]));
    double a = 0.0;
    for (int j = 0; j < nu; ++j) a += log2(fmax(dmax, 1e-300) / fmax(fabs(lambda[c * nu + j]), 1e-300));
    a /= nu;
    if (kind == kOrderNmpc) {
      // heavier = larger score; map the float score to an order-preserving unsigned, inverted
      const float sc = (float)(log((double)n2 * nuc) - 0.1 * a);
      unsigned u = __float_as_uint(sc);
      u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
      k = ~u;
    } else {
      const double qd = fmin(fmax((a + 256.0) * 2048.0, 0.0), 1048575.0);
      const unsigned M = (unsigned)(nu * nuc);
      k = ~((M << 20) | (unsigned)qd);
    }
  }
  key[c] = k;
  idx[c] = (int)c;
}

int order_candidates(int kind, int my, int nu, long long C, const int* N2, const int* Nu, const double* delta,
                     const double* lambda, WorkOrder& wo, const int** perm, hipStream_t stream, std::string* err) {
  *perm = nullptr;
  if (C < kOrderMinC) return 0;  // one round of workgroups: the order cannot matter
  if (wo.pending && hipStreamWaitEvent(stream, wo.used, 0) != hipSuccess) {
    *err = "hipStreamWaitEvent failed (dispatch-order buffers)";
    return -3;
  }
  size_t temp = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (const unsigned*)nullptr, (unsigned*)nullptr,
                                         (const int*)nullptr, (int*)nullptr, (int)C) != hipSuccess) {
    *err = "hipcub::DeviceRadixSort::SortPairs (size query) failed";
    return -3;
  }
  const size_t arr = ((size_t)C * 4 + 255) & ~(size_t)255;
  const size_t need = 4 * arr + temp;
  if (!wo.used && hipEventCreateWithFlags(&wo.used, hipEventDisableTiming) != hipSuccess) {
    *err = "hipEventCreate failed (dispatch-order buffers)";
    return -3;
  }
  if (need > wo.bytes) {
    if (wo.buf) (void)hipFree(wo.buf);
    wo.buf = nullptr;
    wo.bytes = 0;
    if (hipMalloc(&wo.buf, need) != hipSuccess) {
      *err = "hipMalloc failed (dispatch-order buffers)";
      return -2;
    }
    wo.bytes = need;
  }
  char* b = static_cast<char*>(wo.buf);
  unsigned* kin = reinterpret_cast<unsigned*>(b);
  unsigned* kout = reinterpret_cast<unsigned*>(b + arr);
  int* iin = reinterpret_cast<int*>(b + 2 * arr);
  int* iout = reinterpret_cast<int*>(b + 3 * arr);
  hipLaunchKernelGGL(order_keys, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, stream, kind, C, my, nu, N2, Nu,
                     delta, lambda, kin, iin);
  if (hipcub::DeviceRadixSort::SortPairs(b + 4 * arr, temp, kin, kout, iin, iout, (int)C, 0, 32, stream) !=
      hipSuccess) {
    *err = "hipcub::DeviceRadixSort::SortPairs failed";
    return -3;
  }
  *perm = iout;
  return 0;
}

void order_release(WorkOrder& wo) {
  if (wo.buf) (void)hipFree(wo.buf);
  if (wo.used) (void)hipEventDestroy(wo.used);
  wo = WorkOrder{};
}

void order_mark_used(WorkOrder& wo, hipStream_t stream) {
  if (wo.used && hipEventRecord(wo.used, stream) == hipSuccess) wo.pending = true;
}

}  // namespace mpct
