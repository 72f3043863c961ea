// latency_probe.hip — dependent-chain latency of the one-wave primitives the closed-loop kernels are
// built from (wave_ops.h, gi_core.h, gpc_qp16.h), measured on the GPU with s_memtime around an
// unrolled chain of each, one wavefront alone on its CU (the latency roofline of
// the metric kernel, tools/latency_model.py).  Each probe repeats one dependent step kRep times per
// trip and kTrips trips; cycles per step = (stamp difference) / (kRep * kTrips), minus nothing: the
// loop overhead is one SALU compare and branch per kRep steps.  Built by hand (not part of build()):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DMPCT_PACKED_ARGMIN=1 -I model-predictive-control-tuning_amd/csrc \
//         tools/latency_probe.hip -o tools/latency_probe
// Usage: tools/latency_probe  -> one JSON object {probe: cycles per step}
#include <hip/hip_runtime.h>

#include <cstdio>

#include "wave_ops.h"

using namespace mpct;

constexpr int kRep = 64, kTrips = 64, kProbes = 21;

// keep a value live and opaque to the optimiser (no constant folding across steps)
__device__ __forceinline__ double opaque(double v) {
  asm volatile("" : "+v"(v));
  return v;
}

template <int P>
__device__ __forceinline__ double step(double x, double a, double* lds, int lane) {
  switch (P) {
    case 0:  // v_fma_f64, dependent
      return fma(x, a, 1e-3);
    case 1:  // v_add_f64, dependent
      return x + a;
    case 2:  // one DPP reduction stage: 2 x v_mov_b32_dpp + v_add_f64 (quad_perm)
      return x + dppd<kQx1>(x);
    case 3:  // row_sum: the 16-lane DPP reduction (4 stages)
      return row_sum(x) * a;
    case 4:  // row4_sum: v_permlane16_swap + v_permlane32_swap with the adds
      return row4_sum(x) * a;
    case 5:  // bcast: 2 x v_readlane (VALU -> SGPR) and a VALU use
      return bcast(x, 5) * a;
    case 6:  // __shfl (ds_bpermute) of a double, dependent
      return __shfl(x, (lane + 1) & 63, 64) * a;
    case 7: {  // LDS hand-off: store, lds_sync, load another lane's value
      lds[lane] = x;
      lds_sync();
      const double v = lds[(lane + 1) & 63];
      lds_sync();
      return v * a;
    }
    case 8:  // rsq_nr: v_rsq_f64 + two Newton steps
      return rsq_nr(x) * a + 0.25;
    case 9:  // rcp_nr: v_rcp_f64 + two Newton steps
      return rcp_nr(x) * a + 0.5;
    case 10:  // row_bcast16: DPP row_newbcast of lane k of each row
      return row_bcast16(x, 3) * a;
    case 11: {  // qargmin<16> with the packed key (the QP's most violated / ratio test)
      int id = lane;
      double v = x;
      qargmin<16>(v, id, 0);
      return v * a + (double)id * 1e-9;
    }
    case 12: {  // row_argmin over (value, id) pairs, 4 stages
      int id = lane;
      double v = x;
      row_argmin(v, id);
      return v * a;
    }
    case 13: {  // wave_argmin64: row_argmin + two pair_argmin (permlane swaps)
      int id = lane;
      double v = x;
      wave_argmin64(v, id);
      return v * a;
    }
    case 14:  // a wave-uniform branch on a VALU result (v_cmp -> readfirstlane / vcc -> s_cbranch)
      if (__builtin_amdgcn_readfirstlane((int)(x > 1e300)) != 0) return x * 0.5;
      return x * a;
    case 15:  // __ballot of a VALU compare feeding a uniform branch
      if (__ballot(x < -1e300) != 0) return x * 0.5;
      return x * a;
    case 16: {  // LDS read of a lane-dependent address computed from the previous step (pointer chase)
      const int i = ((int)(x * 0.0)) + lane;
      return lds[i & 63] * a + x * 0.0;
    }
    case 17:  // dppd<kQx1> alone (the 2 x v_mov_b32_dpp half of a stage)
      return dppd<kQx1>(x);
    case 18:  // block_prefix<16> at Nu = 5: three DPP row_shr stages with predicated adds
      return block_prefix<16>(x, lane & 7, 5, true, nullptr) * a;
    case 20: {  // qargmin<16> without the packed key: row_argmin and the lane-0 broadcast (gi_core)
      int id = lane;
      double v = x;
      qargmin<16>(v, id);
      return v * a + (double)id * 1e-9;
    }
    default:  // v_mul_f64, dependent
      return x * a;
  }
}

template <int P>
__global__ void probe(unsigned long long* out, double seed) {
  __shared__ double lds[64];
  const int lane = threadIdx.x;
  lds[lane] = 1.0 + lane * 1e-3;
  lds_sync();
  double x = opaque(seed + lane * 1e-6);
  const double a = opaque(0.9999999);
  unsigned long long t0 = 0, t1 = 0;
  for (int trip = -1; trip < kTrips; ++trip) {
    if (trip == 0) {
      __builtin_amdgcn_s_waitcnt(0);
      t0 = __builtin_amdgcn_s_memtime();
    }
#pragma unroll
    for (int r = 0; r < kRep; ++r) x = step<P>(x, a, lds, lane);
  }
  x = opaque(x);
  __builtin_amdgcn_s_waitcnt(0);
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    out[2 * P] = t1 - t0;
    out[2 * P + 1] = (unsigned long long)__double_as_longlong(x);  // keeps the chain live
  }
}

template <int P>
static void run(unsigned long long* d) {
  hipLaunchKernelGGL(probe<P>, dim3(1), dim3(64), 0, 0, d, 1.0);
}

// the shader clock during a busy FP64 loop: s_memtime ticks per s_memrealtime tick (100 MHz)
__global__ void clock_probe(unsigned long long* out) {
  double x = opaque(1.0 + threadIdx.x * 1e-9);
  const double a = opaque(0.9999999);
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 200000; ++i) x = fma(x, a, 1e-3);
  x = opaque(x);
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime(), t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = t1 - t0;
    out[1] = r1 - r0;
    out[2] = (unsigned long long)__double_as_longlong(x);
  }
}

int main() {
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, sizeof(unsigned long long) * 2 * kProbes) != hipSuccess) return 1;
  (void)hipMemset(d, 0, sizeof(unsigned long long) * 2 * kProbes);
  for (int rep = 0; rep < 2; ++rep) {  // the first round warms the clocks and the code
    run<0>(d); run<1>(d); run<2>(d); run<3>(d); run<4>(d); run<5>(d); run<6>(d); run<7>(d); run<8>(d);
    run<9>(d); run<10>(d); run<11>(d); run<12>(d); run<13>(d); run<14>(d); run<15>(d); run<16>(d);
    run<17>(d); run<18>(d); run<19>(d); run<20>(d);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
  }
  unsigned long long h[2 * kProbes];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 3;
  const char* names[kProbes] = {"fma_f64", "add_f64", "dpp_stage_f64", "row_sum16", "row4_sum_permlane",
                                "bcast_readlane", "shfl_bpermute", "lds_handoff", "rsq_nr", "rcp_nr",
                                "row_bcast16", "qargmin16_key", "row_argmin", "wave_argmin64",
                                "uniform_branch", "ballot_branch", "lds_read_chase", "dpp_mov_pair",
                                "block_prefix16_nu5", "mul_f64", "qargmin16_exact"};
  printf("{");
  for (int p = 0; p < kProbes; ++p)
    printf("%s\"%s\": %.2f", p ? ", " : "", names[p], (double)h[2 * p] / (kRep * kTrips));
  unsigned long long* dc = nullptr;
  if (hipMalloc(&dc, 3 * sizeof(unsigned long long)) != hipSuccess) return 4;
  hipLaunchKernelGGL(clock_probe, dim3(256), dim3(64), 0, 0, dc);  // every CU busy, like a launch
  unsigned long long hc[3];
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost) != hipSuccess)
    return 5;
  printf(", \"clock_mhz\": %.1f, \"steps_per_probe\": %d}\n", 100.0 * (double)hc[0] / (double)hc[1], kRep * kTrips);
  (void)hipFree(d);
  return 0;
}
