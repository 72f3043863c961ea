// xlane_latency.hip — dependent-chain latency of the cross-lane and FP64 building blocks the QP
// loops of gpc_kernel.hip chain together (one wave alone on the GPU, so nothing hides latency).
// Each test runs ITERS iterations of  x = op(x) * a + b  on lanes 0..15 and reports shader-clock
// cycles per iteration (s_memtime).  Build: hipcc --offload-arch=gfx950 -O3 -o xlane_latency
// tools/diag/xlane_latency.hip ; run: ./xlane_latency
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITERS = 4096;

__device__ __forceinline__ double bcast_rl(double v, int src) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
  return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double row_sum(double v) {
  v += dppd<0xB1>(v);
  v += dppd<0x4E>(v);
  v += dppd<0x141>(v);
  v += dppd<0x140>(v);
  return v;
}
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  return fma(r, fma(-x, r, 1.0), r);
}

template <int TEST>
__global__ void chain(double* out, unsigned long long* cyc, double a, double b, int src) {
  __shared__ double lds[64];
  const int lane = threadIdx.x;
  double x = 1.0 + lane * 1e-3;
  lds[lane] = x;
  lds_sync();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; ++i) {
    if constexpr (TEST == 0) {  // FP64 FMA latency
      x = fma(x, a, b);
    } else if constexpr (TEST == 1) {  // v_readlane broadcast (uniform source lane) + FMA
      x = fma(bcast_rl(x, src), a, b);
    } else if constexpr (TEST == 2) {  // DPP row_newbcast:3 + FMA
      x = fma(dppd<0x153>(x), a, b);
    } else if constexpr (TEST == 3) {  // LDS store, fence, load of another lane's slot + FMA
      lds[lane] = x;
      lds_sync();
      x = fma(lds[src], a, b);
    } else if constexpr (TEST == 4) {  // DPP row_shr:1 + FMA
      x = fma(dppd<0x111>(x), a, b);
    } else if constexpr (TEST == 5) {  // 16-lane DPP row sum + FMA
      x = fma(row_sum(x), a, b) * 0.0625;
    } else if constexpr (TEST == 6) {  // row sum + readlane broadcast (qsum of gpc_qp.h)
      x = fma(bcast_rl(row_sum(x), 0), a, b) * 0.0625;
    } else if constexpr (TEST == 7) {  // reciprocal by v_rcp_f64 + two Newton steps
      x = rcp_nr(x) + b;
    } else if constexpr (TEST == 8) {  // IEEE FP64 divide
      x = a / x + b;
    } else if constexpr (TEST == 9) {  // ds_bpermute from lane src
      const int lo = __builtin_amdgcn_ds_bpermute(src * 4, __double2loint(x));
      const int hi = __builtin_amdgcn_ds_bpermute(src * 4, __double2hiint(x));
      x = fma(__hiloint2double(hi, lo), a, b);
    } else if constexpr (TEST == 10) {  // readlane of an int (index) + FMA with an LDS operand
      const int k = __builtin_amdgcn_readlane((int)x & 15, src);
      x = fma(lds[k], a, b) + x * 1e-9;
    } else if constexpr (TEST == 11) {  // LDS load with address from the previous value (pointer chase)
      const int k = ((int)(x * 8.0)) & 63;
      x = fma(lds[k], a, b);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[lane] = x;
  if (lane == 0) cyc[0] = t1 - t0;
}

template <int TEST>
static void run(const char* name, double* dout, unsigned long long* dcyc) {
  unsigned long long c = 0;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(chain<TEST>, dim3(1), dim3(64), 0, 0, dout, dcyc, 0.999, 1e-3, 3);
    (void)hipEventRecord(e1, 0);
    (void)hipDeviceSynchronize();
  }
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipMemcpy(&c, dcyc, sizeof c, hipMemcpyDeviceToHost);
  printf("%-44s %8.1f memtime-cycles/iter  %8.2f ns/iter (event)\n", name, (double)c / ITERS, ms * 1e6 / ITERS);
}

int main() {
  double* dout;
  unsigned long long* dcyc;
  (void)hipMalloc(&dout, 64 * sizeof(double));
  (void)hipMalloc(&dcyc, sizeof(unsigned long long));
  run<0>("fma_f64 chain", dout, dcyc);
  run<1>("readlane bcast + fma", dout, dcyc);
  run<2>("dpp row_newbcast + fma", dout, dcyc);
  run<3>("lds store/sync/load + fma", dout, dcyc);
  run<4>("dpp row_shr + fma", dout, dcyc);
  run<5>("dpp row_sum (4 steps) + fma", dout, dcyc);
  run<6>("row_sum + readlane bcast + fma", dout, dcyc);
  run<7>("rcp_nr (rcp + 2 newton)", dout, dcyc);
  run<8>("ieee f64 divide", dout, dcyc);
  run<9>("ds_bpermute + fma", dout, dcyc);
  run<10>("readlane idx + lds load + fma", dout, dcyc);
  run<11>("lds pointer chase + fma", dout, dcyc);
  return 0;
}
