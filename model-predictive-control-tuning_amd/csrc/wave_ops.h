// wave_ops.h — one-wavefront building blocks shared by the closed-loop kernels (gpc_kernel.hip,
// mdband_kernel.hip): LDS hand-off fence, readlane broadcast, DPP / permlane reductions over the
// QP-row lanes, lane shifts and the per-MV-block prefix sum.  Every helper is force-inlined: the
// kernels rely on lds_sync() (lgkmcnt only), which is only correct when no helper is outlined
// into a FLAT-addressed call (checked on the ISA by __graft_entry__.kernel_isa()).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include "mpct_dev.h"

namespace mpct {

// ------------------------------------------------------------------------------------------
// wave helpers
__device__ __forceinline__ void lds_sync() {
  // one-wave workgroup: LDS requests of a wave complete in order; wait for this lane's and order
  // the compiler's memory operations around the hand-off.  The wait is not needed for
  // correctness (a fence-only build gave bitwise the same metric grid) and costs nothing
  // measurable (profiles/r04b_small_ab.txt), so it stays as the conservative form
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 1/x: v_rcp_f64 and two Newton steps (about 1 ulp, not correctly rounded): five dependent
// operations instead of the division's scale / rcp / refine / fixup sequence
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  return fma(r, fma(-x, r, 1.0), r);
}

// 1/sqrt(x), x > 0: v_rsq_f64 and two Newton steps (the Givens rotations' divide-free form)
__device__ __forceinline__ double rsq_nr(double x) {
  double r = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  r = r * fma(-h * r, r, 1.5);
  return r * fma(-h * r, r, 1.5);
}

// lane id for the QP helpers
__device__ __forceinline__ int qp_lane() {
  return threadIdx.x;
}

__device__ __forceinline__ double bcast(double v, int src) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
  return __hiloint2double(hi, lo);
}

// DPP moves.  Controls whose every lane has a source within its row (quad_perm, row_mirror,
// row_half_mirror, row_newbcast) use v_mov_b32_dpp without an `old` operand: the update_dpp(0, ..)
// form makes the compiler zero a fresh register before every move (two v_mov_b32 per double,
// ~60 per Goldfarb-Idnani step of the metric kernel; a double's move pair went from 32 to 13 cycles
// of dependent latency, tools/latency_probe.hip).  The row shifts (row_shl / row_shr: lanes at the
// row's edge have no source) set bound_ctrl, which writes 0 to those lanes as old = 0 would,
// without the zeroed register
template <int CTRL>
constexpr bool kDppAllLanes = CTRL < 0x100 || CTRL == 0x140 || CTRL == 0x141 || (CTRL >= 0x150 && CTRL <= 0x15F);
template <int CTRL>
__device__ __forceinline__ int dpp32(int v) {
  if constexpr (kDppAllLanes<CTRL>) return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
  else return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
  const int lo = dpp32<CTRL>(__double2loint(v));
  const int hi = dpp32<CTRL>(__double2hiint(v));
  return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
  return dpp32<CTRL>(v);
}
// DPP controls: quad_perm(1,0,3,2), quad_perm(2,3,0,1), row_half_mirror, row_mirror
constexpr int kQx1 = 0xB1, kQx2 = 0x4E, kHalfMirror = 0x141, kMirror = 0x140;

// sum over lanes 0..15 (every lane of row 0 gets it; callers zero inactive lanes)
__device__ __forceinline__ double row_sum(double v) {
  v += dppd<kQx1>(v);
  v += dppd<kQx2>(v);
  v += dppd<kHalfMirror>(v);
  v += dppd<kMirror>(v);
  return v;
}
// lane k (0..15, a compile-time constant after unrolling) of every 16-lane row, broadcast over its
// row: DPP row_newbcast (gfx950), no SGPR round trip; four rows give four independent broadcasts
__device__ __forceinline__ double row_bcast16(double v, int k) {
  switch (k & 15) {
    case 0: return dppd<0x150>(v);
    case 1: return dppd<0x151>(v);
    case 2: return dppd<0x152>(v);
    case 3: return dppd<0x153>(v);
    case 4: return dppd<0x154>(v);
    case 5: return dppd<0x155>(v);
    case 6: return dppd<0x156>(v);
    case 7: return dppd<0x157>(v);
    case 8: return dppd<0x158>(v);
    case 9: return dppd<0x159>(v);
    case 10: return dppd<0x15A>(v);
    case 11: return dppd<0x15B>(v);
    case 12: return dppd<0x15C>(v);
    case 13: return dppd<0x15D>(v);
    case 14: return dppd<0x15E>(v);
    default: return dppd<0x15F>(v);
  }
}
// min over the 16 lanes of each row, on every lane of the row (v_min_f64 on DPP-moved operands)
__device__ __forceinline__ double row_min(double v) {
  v = fmin(v, dppd<kQx1>(v));
  v = fmin(v, dppd<kQx2>(v));
  v = fmin(v, dppd<kHalfMirror>(v));
  return fmin(v, dppd<kMirror>(v));
}
__device__ __forceinline__ int row_min_i(int v) {
  v = min(v, dppi<kQx1>(v));
  v = min(v, dppi<kQx2>(v));
  v = min(v, dppi<kHalfMirror>(v));
  return min(v, dppi<kMirror>(v));
}
// (v, id) -> the row's smallest v and the smallest id attaining it, on every lane of the row: the
// lexicographic (value, id) minimum as two reductions -- the value by v_min_f64 stages, then the id
// among the lanes holding that value by 32-bit v_min_i32 stages -- instead of four stages of a
// (value, id) pair compare-and-select (measured: 485 cycles of dependent latency per call for the
// pair form, tools/latency_probe.hip; NaN values are never the minimum, as in the pair form's `<`)
__device__ __forceinline__ void row_argmin(double& v, int& id) {
  const double m = row_min(v);
  id = row_min_i(v == m ? id : 0x7fffffff);
  v = m;
}

// min of (v, id) with the partner half / row pair: v_permlane16/32_swap hand each lane its own and
// its partner's value (in either order), so the lexicographic min of the pair is symmetric
template <bool R32>
__device__ __forceinline__ void pair_argmin(double& v, int& id) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  auto l = R32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false) : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  auto h = R32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false) : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  auto k = R32 ? __builtin_amdgcn_permlane32_swap(id, id, false, false) : __builtin_amdgcn_permlane16_swap(id, id, false, false);
  double a = __hiloint2double(h[0], l[0]);
  const double b = __hiloint2double(h[1], l[1]);
  int ia = k[0];
  const int ib = k[1];
  if (b < a || (b == a && ib < ia)) {
    a = b;
    ia = ib;
  }
  v = a;
  id = ia;
}

// min of v / of an int with the partner row (R32: the partner half) by v_permlane16/32_swap
template <bool R32>
__device__ __forceinline__ double pair_min(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  auto l = R32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false) : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  auto h = R32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false) : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return fmin(__hiloint2double(h[0], l[0]), __hiloint2double(h[1], l[1]));
}
template <bool R32>
__device__ __forceinline__ int pair_min_i(int v) {
  auto k = R32 ? __builtin_amdgcn_permlane32_swap(v, v, false, false) : __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return min((int)k[0], (int)k[1]);
}

// reductions over the whole wave: DPP within the 16-lane rows, then the v_permlane16/32_swap
// exchanges between rows (gfx950) -- no LDS round trip.  A __shfl_xor butterfly costs six
// ds_bpermute round trips per value; the band kernel's M > 15 classes and the NMPC's M > 15
// class run several of these per QP iteration.  The lexicographic (value, id) minimum as two
// reductions (value, then the smallest id holding it): 757 cycles of dependent latency per call
// for the pair form (tools/latency_probe.hip)
__device__ __forceinline__ void wave_argmin64(double& v, int& id) {
  const double m = pair_min<true>(pair_min<false>(row_min(v)));
  id = pair_min_i<true>(pair_min_i<false>(row_min_i(v == m ? id : 0x7fffffff)));
  v = m;
}

// sum over the four 16-lane rows (lanes l, l+16, l+32, l+48), result in every row:
// v_permlane16_swap then v_permlane32_swap (gfx950), no LDS round trip
__device__ __forceinline__ double row4_sum(double v) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const double a = __hiloint2double(h16[0], l16[0]) + __hiloint2double(h16[1], l16[1]);
  lo = __double2loint(a);
  hi = __double2hiint(a);
  auto l32 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  auto h32 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double(h32[0], l32[0]) + __hiloint2double(h32[1], l32[1]);
}

// row4_sum of two / four values at once, bitwise equal to row4_sum of each ((v0 + v1) + (v2 + v3)):
// the first swaps pair different values, so they need no register copies (v_permlane*_swap
// overwrites both operands), and the partial sums travel together until one final broadcast.
// Two values: 12 instructions instead of 20; four: 21 instead of 40
__device__ __forceinline__ void permlane16_pair(double& x, double& y) {  // x, y <- rows (0 2 | 1 3) mix
  auto l = __builtin_amdgcn_permlane16_swap(__double2loint(x), __double2loint(y), false, false);
  auto h = __builtin_amdgcn_permlane16_swap(__double2hiint(x), __double2hiint(y), false, false);
  x = __hiloint2double(h[0], l[0]);
  y = __hiloint2double(h[1], l[1]);
}
__device__ __forceinline__ void permlane32_pair(double& x, double& y) {
  auto l = __builtin_amdgcn_permlane32_swap(__double2loint(x), __double2loint(y), false, false);
  auto h = __builtin_amdgcn_permlane32_swap(__double2hiint(x), __double2hiint(y), false, false);
  x = __hiloint2double(h[0], l[0]);
  y = __hiloint2double(h[1], l[1]);
}
__device__ __forceinline__ void row4_sum2(double& a, double& b) {
  permlane16_pair(a, b);  // a = [a0 b0 a2 b2], b = [a1 b1 a3 b3]
  double p = a + b;       // [a01 b01 a23 b23]
  double q = p;
  permlane32_pair(p, q);  // p = [a01 b01 a01 b01], q = [a23 b23 a23 b23]
  p += q;                 // [A B A B]
  q = p;
  permlane16_pair(p, q);  // p = [A A A A], q = [B B B B]
  a = p;
  b = q;
}
__device__ __forceinline__ void row4_sum4(double& a, double& b, double& c, double& d) {
  permlane16_pair(a, b);
  permlane16_pair(c, d);
  double p = a + b, q = c + d;  // p = [a01 b01 a23 b23], q = [c01 d01 c23 d23]
  permlane32_pair(p, q);        // p = [a01 b01 c01 d01], q = [a23 b23 c23 d23]
  double v = p + q;             // [A B C D]
  double w = v;
  permlane16_pair(v, w);        // v = [A A C C], w = [B B D D]
  double v2 = v, w2 = w;
  permlane32_pair(v, v2);       // v = [A A A A], v2 = [C C C C]
  permlane32_pair(w, w2);       // w = [B B B B], w2 = [D D D D]
  a = v;
  b = w;
  c = v2;
  d = w2;
}

__device__ __forceinline__ double wave_sum64(double v) { return row4_sum(row_sum(v)); }

// reductions over the QP-row lanes (0..M-1): DPP within row 0 when the template allows M <= 16
template <int MAXM>
__device__ __forceinline__ double qsum(double v) {
  if constexpr (MAXM <= 16) {
    return bcast(row_sum(v), 0);
  } else {
    return wave_sum64(v);
  }
}
// M <= 16 argmin on one order-preserving 64-bit key (value bits | id): (v, id) -> one unsigned key whose order is v's order, with v's low 6 mantissa bits replaced by
// id (< 64): one u64 compare per DPP step instead of the (value, id) pair.  The winner's exact
// value is re-read from its lane (ids are 4 * lane + k or lane: lane = id >> shift).
__device__ __forceinline__ unsigned long long argkey(double v, int id) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned long long u = (b >> 63) ? ~b : (b | 0x8000000000000000ull);
  return (u & ~63ull) | (unsigned long long)(id & 63);
}
template <int CTRL>
__device__ __forceinline__ unsigned long long dppu64(unsigned long long k) {
  const int lo = dpp32<CTRL>((int)(unsigned)k);
  const int hi = dpp32<CTRL>((int)(unsigned)(k >> 32));
  return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}
__device__ __forceinline__ unsigned long long row_minkey(unsigned long long k) {
  k = min(k, dppu64<kQx1>(k));
  k = min(k, dppu64<kQx2>(k));
  k = min(k, dppu64<kHalfMirror>(k));
  k = min(k, dppu64<kMirror>(k));
  return k;
}

// MPCT_PACKED_ARGMIN=1 restores the packed-key form for the callers that pass `shift` (round 2:
// five VALU instructions per stage against about ten for the (value, id) pair compare of the time).
// Measured per call as a dependent chain (tools/latency_probe.hip, r05): packed key 281 cycles,
// row_argmin (value min, then id min) plus the lane-0 broadcast 197 cycles, so the exact form is
// the default; it also selects exactly the lexicographic (value, id) minimum
#ifndef MPCT_PACKED_ARGMIN
#define MPCT_PACKED_ARGMIN 0
#endif
template <int MAXM>
__device__ __forceinline__ void qargmin(double& v, int& id, int shift = -1) {
  if constexpr (MAXM <= 16) {
    if (MPCT_PACKED_ARGMIN && shift >= 0) {
      // lanes >= 16 hold INF (callers), so row 0's minimum is the QP rows' minimum
      const unsigned long long k = row_minkey(argkey(v, id));
      const int kid = (int)(__builtin_amdgcn_readlane((int)(unsigned)k, 0) & 63);
      const double w = bcast(v, kid >> shift);
      if (w == INFINITY) {
        v = INFINITY;
        id = 0x7fffffff;
      } else {
        v = w;
        id = kid;
      }
      return;
    }
    row_argmin(v, id);
    v = bcast(v, 0);
    id = __builtin_amdgcn_readlane(id, 0);
  } else {
    wave_argmin64(v, id);
  }
}

#ifdef MPCT_PROFILE
// diagnostic build: section k's cycles in the low 40 bits of pacc[k] (1.1e12 cycles, minutes of one
// simulation), the number of times the section ended in the high 24 (tools/latency_model.py divides
// one by the other).  24 bits hold the band and NMPC kernels' counts too: a heavy config-3
// simulation ends its QP sections ~1e5 times, past the 16 bits of the first layout
constexpr int kProfCountShift = 40;
constexpr unsigned long long kProfCount = 1ull << kProfCountShift;
// ProfAcc: the section words live in one 64-bit VGPR pair, lane k holding word k.  The SGPR array
// of PROF_N words (ProfAccS, the first form) was copied whole at every loop back-edge of the metric
// kernel's step loop (28 s_mov per QP iteration), which inflated the sections it was measuring.
// A VALU add lands only in active lanes, so ProfAcc needs every stamp at a wave-uniform point (the
// metric kernel's are); the band, NMPC and general kernels stamp inside lane-divergent code and
// keep ProfAccS
struct ProfAccS {
  unsigned long long w[PROF_N] = {};
  __device__ __forceinline__ unsigned long long& operator[](int k) { return w[k]; }
  __device__ __forceinline__ unsigned long long get(int k) const { return w[k]; }
};
struct ProfAcc {
  unsigned long long v = 0;
  struct Ref {
    ProfAcc* a;
    int k;
    __device__ __forceinline__ void operator+=(unsigned long long d) { a->add(k, d); }
  };
  __device__ __forceinline__ Ref operator[](int k) { return Ref{this, k}; }
  __device__ __forceinline__ void add(int k, unsigned long long d) {
    int l = threadIdx.x;
    asm volatile("" : "+v"(l));
    v += (l == k) ? d : 0ull;
  }
  __device__ __forceinline__ unsigned long long get(int k) const {  // wave-uniform
    const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)v, k);
    const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(v >> 32), k);
    return ((unsigned long long)hi << 32) | lo;
  }
};
#define PSTAMP(k)                                              \
  do {                                                         \
    __builtin_amdgcn_sched_barrier(0);                         \
    asm volatile("; PSTAMP " #k);                              \
    unsigned long long now_ = __builtin_amdgcn_s_memtime();    \
    pacc[k] += now_ - pprev + kProfCount;                      \
    pprev = now_;                                              \
    __builtin_amdgcn_sched_barrier(0);                         \
  } while (0)
#else
#define PSTAMP(k) \
  do {            \
  } while (0)
#endif

// ------------------------------------------------------------------------------------------
// lane shifts by one within the QP rows: DPP row_shl/row_shr when the rows fit one DPP row
template <int MAXM>
__device__ __forceinline__ double lane_next(double v) {  // lane i receives lane i+1
  if constexpr (MAXM <= 16) return dppd<0x101>(v);
  else return __shfl_down(v, 1, 64);
}
template <int MAXM>
__device__ __forceinline__ double lane_prev(double v) {  // lane i receives lane i-1
  if constexpr (MAXM <= 16) return dppd<0x111>(v);
  else return __shfl_up(v, 1, 64);
}
template <int MAXM>
__device__ __forceinline__ int lane_next_i(int v) {
  if constexpr (MAXM <= 16) return dppi<0x101>(v);
  else return __shfl_down(v, 1, 64);
}

// inclusive prefix sum of x over the lanes of one MV block (lane position l within its block):
// the amplitude rows of the QP.  DPP row_shr Hillis-Steele scan when the rows fit one DPP row.
template <int MAXM>
__device__ __forceinline__ double block_prefix(double x, int l, int Nu, bool row, double* sxc) {
  if constexpr (MAXM <= 16) {
    // the first three stages run whatever Nu is (l < Nu masks them): their uniform Nu tests were
    // four SALU / VALU instructions and a branch each, more than the stage they skip
    double pre = x, t;
    t = dppd<0x111>(pre); if (l >= 1) pre += t;
    t = dppd<0x112>(pre); if (l >= 2) pre += t;
    t = dppd<0x114>(pre); if (l >= 4) pre += t;
    if (Nu > 8) { t = dppd<0x118>(pre); if (l >= 8) pre += t; }
    return pre;
  } else {
    const int lane = threadIdx.x;  // sxc holds the M QP rows only
    if (row) sxc[lane] = x;
    lds_sync();
    double pre = 0.0;
    if (row)
      for (int j = lane - l; j <= lane; ++j) pre += sxc[j];
    lds_sync();
    return pre;
  }
}

}  // namespace mpct
