// work_order.hip — heaviest-first dispatch order of a candidate batch (see work_order.h).
#include <hipcub/hipcub.hpp>

#include <cstdlib>

#include "wave_ops.h"
#include "work_order.h"


namespace mpct {

// NaN costs, status MPCT_ST_NOT_RUN, 0 iterations for simulation slot s (see prefill_kernel)
__device__ __forceinline__ void prefill_slot(const DevResult& out, long long s, long long S, int my, int nu) {
  const double nan = __longlong_as_double(0x7ff8000000000000ll);
  if (out.stage) {
    const StageRow& R = out.srow;
    double* row = out.stage + xcd_row(s, S) * R.w;
    for (int i = 0; i < my; ++i) {
      if (R.j1 >= 0) row[R.j1 + i] = nan;
      if (R.j21 >= 0) row[R.j21 + i] = nan;
      if (R.j22 >= 0) row[R.j22 + i] = nan;
    }
    if (R.jnu >= 0)
      for (int i = 0; i < nu; ++i) row[R.jnu + i] = nan;
    if (R.st >= 0) row[R.st] = (double)MPCT_ST_NOT_RUN_;
    if (R.it >= 0) row[R.it] = 0.0;
    return;
  }
  for (int i = 0; i < my; ++i) {
    if (out.J1) out.J1[s * my + i] = nan;
    if (out.j21) out.j21[s * my + i] = nan;
    if (out.j22) out.j22[s * my + i] = nan;
  }
  if (out.Jnu)
    for (int i = 0; i < nu; ++i) out.Jnu[s * nu + i] = nan;
  if (out.status) out.status[s] = MPCT_ST_NOT_RUN_;
  if (out.qp_iters) out.qp_iters[s] = 0;
}


// ---- dispatch order (longest-processing-time first).  The workgroups of a launch start in slot
// order and a batch larger than the resident slots (4096 simulations, 12 slots per CU at the
// metric) runs a second, partial round, so a long simulation that starts late sets the kernel
// time.  Simulation time grows with the QP size M and with the QP work, which the candidates'
// weights predict: the more the tracking weights dominate the move-rate weights, the more often
// the bounds bind.  Key (ascending = heavier first): ~(M << 20 | q(mean_j log2(max_i|delta_i| /
// |lambda_j|))); invalid candidates last.  Measured on the metric batch (tools/order_probe.py):
// grid order 5.36 ms, this key 3.9 ms, ideal (measured QP work, descending) 3.58 ms.  GPC and
// DTC-GPC batches now use the controller-based estimate of order_keys_gpc below; this weight-ratio
// key remains for NMPC and for scenarios whose H is too large to form per candidate.
// NMPC (config 5, tools/order_probe5.py, tools/diag/nmpc_order_ab.py): the work per Gauss-Newton
// iteration grows with the horizon N and the QP size.  Since the Anderson-accelerated iteration
// (round 2), N Nu alone orders the batch as well as the measured work (GAM mode: 267 ms for both,
// grid order 331 ms); the round-1 score log(N Nu) - 0.1 a, which also weighed the iteration
// count, measured 288 ms (tools/diag/nmpc_order_ab.py) and is not kept.
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
      k = ~((unsigned)(n2 * nuc) << 14);  // N * Nu: the prediction's length times the QP size

    } else {
      const double qd = fmin(fmax((a + 256.0) * 2048.0, 0.0), 1048575.0);
      const unsigned M = (unsigned)(nu * nuc);
      k = ~((M << 20) | (unsigned)qd);
    }
  }
  key[c] = k;
  idx[c] = (int)c;
}

// GPC / DTC-GPC key from the candidate's own controller: its unconstrained move demand for the
// scenario's setpoint jumps, in units of each MV's bounds.  H = G'QG + Lambda with the weights as
// the closed-loop kernel's QR applies them; w_i = H^-1 G'Q 1_i are the moves answering a unit
// step held on output i over the horizon, so a reference jump d asks for z = sum_i d_i w_i.  The
// more |z| exceeds the bounds, the more steps run active QP rows.  On the metric grid this
// estimate ranks the measured QP work with Spearman 0.93 (the weight-ratio key above: 0.58), and
// dispatching in its order takes 3.44 ms against the weight-ratio key's 3.90 ms and the measured-
// work order's 3.48 ms (tools/diag/order_key_probe.py).  One wave per candidate, lanes over the
// reference's time steps for the jumps.  H and the solves by QP size (round 5; the metric's key
// went 57 -> 45 us with the register Gauss-Jordan and -> 26 us with the Gram tables,
// profiles/r05_key_stages.txt):
//   * nu Nu <= 16, my <= 4 (the metric): H = sum_o q_o G_o'G_o + Lambda from the scenario's Gram
//     tables (mpct_host.cpp gram_tables), then Gauss-Jordan in registers (gj16).  Correlating the
//     step table in LDS per workgroup took 21 of the 45 us, the LDS Cholesky and solves 21 of 57;
//   * larger QPs: H by lanes over its entries (step-table correlations in LDS), Cholesky and the
//     my solves in LDS (the Gauss-Jordan where the tables were too large to build).
// [H | rhs_0..3] -> [I | H^-1 rhs] by Gauss-Jordan, lane m < M holding row m in registers, the
// pivot row broadcast by v_readlane (no LDS hand-off per column).  H is SPD, so the pivots need no
// exchange; false when a pivot is not positive
__device__ __forceinline__ bool gj16(double (&h)[kGramM], double (&g)[4], int M, int lane) {
#pragma unroll
  for (int j = 0; j < kGramM; ++j) {
    if (j < M) {
      const double piv = bcast(h[j], j);
      if (!(piv > 0.0)) return false;
      const double ip = 1.0 / piv;
      const bool pr = lane == j;
      const double f = h[j] * ip;
#pragma unroll
      for (int k = j + 1; k < kGramM; ++k) {
        const double pk = bcast(h[k], j);
        h[k] = pr ? pk * ip : fma(-f, pk, h[k]);
      }
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        const double po = bcast(g[o], j);
        g[o] = pr ? po * ip : fma(-f, po, g[o]);
      }
    }
  }
  return true;
}

// this lane's share of sum over (jump j, move m) of |z_jm| / b_n(m), z_j = sum_i d_ji w_i(m), for
// the nj jump vectors in sD (lanes over (jump, move) pairs; an unbounded MV adds nothing)
__device__ __forceinline__ double jump_demand(const double* sD, const double* sW, const double* sBn, int nj, int M,
                                              int my, int nuc, int lane) {
  double e = 0.0;
  for (int q = lane; q < nj * M; q += kWave) {
    const int j = q / M, m = q - j * M, n = m / nuc;
    const double bn = sBn[n];
    if (!(bn > 0.0 && bn < INFINITY)) continue;
    double z = 0.0;
    for (int i = 0; i < my; ++i) z += sD[j * my + i] * sW[i * M + m];
    e += fabs(z) / bn;
  }
  return e;
}

__global__ void __launch_bounds__(64) order_keys_gpc(const DevScenario sc, long long C, int nref,
                                                      const int* __restrict__ N2v, const int* __restrict__ Nuv,
                                                      const double* __restrict__ delta,
                                                      const double* __restrict__ lambda,
                                                      const double* __restrict__ r, unsigned* __restrict__ key,
                                                      int* __restrict__ idx, const DevResult pre, int do_pre) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const long long c = blockIdx.x;
  if (c >= C) return;
  const int lane = threadIdx.x;
  const int my = sc.my, nu = sc.nu, tlen = sc.tlen, nit = sc.nit;
  // the ordered launch's result prefill (prefill_kernel's records) rides on this launch: candidate
  // c's wave writes slots c nref .. c nref + nref - 1, so the C waves cover every slot once
  if (do_pre)
    for (int k = lane; k < nref; k += kWave) prefill_slot(pre, c * nref + k, C * nref, my, nu);
  const int n2 = N2v[c], nuc = Nuv[c];
  if (lane == 0) idx[c] = (int)c;
  if (!(n2 > 0 && n2 <= sc.n2max && nuc >= 1 && nuc <= sc.numax && nuc <= n2)) {
    if (lane == 0) key[c] = 0xffffffffu;
    return;
  }
  const int M = nu * nuc;
  const int Mp = sc.nu * sc.numax;
  double* sH = lds;             // H, then its Cholesky factor L (lower, row-major, stride M)
  double* sW = lds + Mp * Mp;   // w_i (row i, stride M)
  double* sQ = sW + my * Mp;    // q_i
  double* sS = sQ + my;         // the step table [my][nu][tlen]
  double* sD = sS + my * nu * tlen;  // jump vectors of one pass [64][my]
  double* sBn = sD + kWave * my;     // b_n per MV (read up front, off the jump passes' chain)
  double* sLw = sBn + nu;            // the move weight of each MV (H's diagonal)
  int* sN1 = reinterpret_cast<int*>(sLw + nu);
  // H and the right-hand sides from the scenario's Gram tables (mpct_host.cpp gram_tables) when
  // they cover this QP size; else correlated here from the step table
  const bool tab = sc.gram != nullptr && M <= kGramM && my <= 4;
  if (!tab)
    for (int e = lane; e < my * nu * tlen; e += kWave) sS[e] = sc.step[e];
  if (lane < my) {
    const double di = fabs(delta[c * my + lane]);
    const double sqi = sc.wsq ? di : sqrt(di);
    sQ[lane] = sqi * sqi;
    sN1[lane] = sc.n1[lane];
  }
  if (lane < nu) {
    sBn[lane] = 0.5 * fmin(sc.bnd[nu + lane] - sc.bnd[lane], sc.bnd[3 * nu + lane] - sc.bnd[2 * nu + lane]);
    const double ln = fabs(lambda[c * nu + lane]);
    const double wl = sc.wsq ? ln : sqrt(ln);
    sLw[lane] = wl * wl;
  }
  lds_sync();
  bool spd = true;
  if (tab) {
    // lane m < M: row m of H = sum_o q_o G_o'G_o + Lambda and rhs_o(m) = q_o G_o'1(m), straight
    // from the block of (N2, Nu) (rows are contiguous: 16 doubles per lane and output)
    const bool hr = lane < M;
    const int il = hr ? lane : 0;
    const double* gb = sc.gram + ((size_t)(n2 - 1) * sc.numax + (nuc - 1)) * my * kGramOut;
    double h[kGramM], g[4];
#pragma unroll
    for (int k = 0; k < kGramM; ++k) h[k] = 0.0;
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      g[o] = 0.0;
      if (o < my) {
        const double q = hr ? sQ[o] : 0.0;
        const double* go = gb + o * kGramOut;
#pragma unroll
        for (int k = 0; k < kGramM; ++k) h[k] = fma(q, go[il * kGramM + k], h[k]);
        g[o] = q * go[kGramM * kGramM + il];
      }
    }
    const double lw = hr ? sLw[il / nuc] : 0.0;
#pragma unroll
    for (int k = 0; k < kGramM; ++k)
      if (k == lane) h[k] += lw;
    spd = gj16(h, g, M, lane);
    if (spd && hr) {
#pragma unroll
      for (int o = 0; o < 4; ++o)
        if (o < my) sW[o * M + lane] = g[o];
    }
    lds_sync();
  } else {
    // H(a,b) = sum_i q_i sum_r G_i(r,a) G_i(r,b) + Lambda,  G_i(r, n*Nu + l) = s_in(n1_i + r - l)
    for (int e = lane; e < M * (M + 1) / 2; e += kWave) {  // lanes over the upper triangle
      int a = 0, b = e;
      while (b >= M - a) {
        b -= M - a;
        ++a;
      }
      b += a;
      const int na = a / nuc, la = a - na * nuc, nb = b / nuc, lb = b - nb * nuc;
      const int lm = la > lb ? la : lb;
      double h = 0.0;
      for (int i = 0; i < my; ++i) {
        const int n1 = sN1[i];
        const double* sa = sS + (i * nu + na) * tlen + n1 - la;  // sa[r] = s_i,na(n1 + r - la)
        const double* sb = sS + (i * nu + nb) * tlen + n1 - lb;
        int rr = lm - n1 > 0 ? lm - n1 : 0;  // first row where both step indices are >= 0
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        for (; rr + 3 < n2; rr += 4) {
          a0 += sa[rr] * sb[rr];
          a1 += sa[rr + 1] * sb[rr + 1];
          a2 += sa[rr + 2] * sb[rr + 2];
          a3 += sa[rr + 3] * sb[rr + 3];
        }
        for (; rr < n2; ++rr) a0 += sa[rr] * sb[rr];
        h += sQ[i] * ((a0 + a1) + (a2 + a3));
      }
      if (a == b) h += sLw[na];
      sH[a * M + b] = h;
      sH[b * M + a] = h;
    }
    // right-hand sides q_i G_i'1 (column sums of G_i); lane (i, m) keeps its entry in a register
    const bool wl = lane < my * M;
    const int wi = wl ? lane / M : 0, wm = wl ? lane - wi * M : 0;
    double w = 0.0;
    if (wl) {
      const int n = wm / nuc, l = wm - n * nuc, n1 = sN1[wi];
      const double* si = sS + (wi * nu + n) * tlen + n1 - l;
      for (int rr = l - n1 > 0 ? l - n1 : 0; rr < n2; ++rr) w += si[rr];
      w *= sQ[wi];
    }
    if (M <= kGramM && my <= 4) {
      // the Gram tables' size class without its tables (kGramMaxBytes): Gauss-Jordan on the
      // LDS-built H (a pivot <= 0 marks the candidate heaviest, as the Cholesky's does)
      if (wl) sW[wi * M + wm] = w;
      lds_sync();
      const bool hr = lane < M;
      double h[kGramM], g[4];
  #pragma unroll
      for (int k = 0; k < kGramM; ++k) h[k] = (hr && k < M) ? sH[lane * M + k] : 0.0;
  #pragma unroll
      for (int o = 0; o < 4; ++o) g[o] = (hr && o < my) ? sW[o * M + lane] : 0.0;
      spd = gj16(h, g, M, lane);
      if (spd && hr) {
  #pragma unroll
        for (int o = 0; o < 4; ++o)
          if (o < my) sW[o * M + lane] = g[o];
      }
      lds_sync();
    } else {
      lds_sync();
      // Cholesky H = L L': lane i owns row i (column k below the pivot, then its row of the
      // trailing block; no integer division in the loop)
      const bool hr = lane < M;
      for (int k = 0; k < M; ++k) {
        const double pk = sH[k * M + k];
        if (!(pk > 0.0)) {
          spd = false;
          break;
        }
        const double lk = sqrt(pk), il = 1.0 / lk;
        lds_sync();
        double lik = 0.0;
        if (lane == k) sH[k * M + k] = lk;
        if (hr && lane > k) {
          lik = sH[lane * M + k] * il;
          sH[lane * M + k] = lik;
        }
        lds_sync();
        if (hr && lane > k) {  // four columns' loads before their updates (the stores would otherwise
                               // hold each next load behind them: one LDS round trip per column)
          int j = k + 1;
          for (; j + 3 <= lane; j += 4) {
            const double h0 = sH[lane * M + j], h1 = sH[lane * M + j + 1];
            const double h2 = sH[lane * M + j + 2], h3 = sH[lane * M + j + 3];
            const double l0 = sH[j * M + k], l1 = sH[(j + 1) * M + k];
            const double l2 = sH[(j + 2) * M + k], l3 = sH[(j + 3) * M + k];
            sH[lane * M + j] = h0 - lik * l0;
            sH[lane * M + j + 1] = h1 - lik * l1;
            sH[lane * M + j + 2] = h2 - lik * l2;
            sH[lane * M + j + 3] = h3 - lik * l3;
          }
          for (; j <= lane; ++j) sH[lane * M + j] -= lik * sH[j * M + k];
        }
        lds_sync();
      }
      if (spd && my * M > kWave) {  // more right-hand side entries than lanes: one lane per output
        if (lane < my) {
          double* wr = sW + lane * M;
          for (int m = 0; m < M; ++m) {
            const int n = m / nuc, l = m - n * nuc, n1 = sN1[lane];
            const double* si = sS + (lane * nu + n) * tlen + n1 - l;
            double acc = 0.0;
            for (int rr = l - n1 > 0 ? l - n1 : 0; rr < n2; ++rr) acc += si[rr];
            wr[m] = sQ[lane] * acc;
          }
          for (int m = 0; m < M; ++m) {
            double a = wr[m];
            for (int j = 0; j < m; ++j) a -= sH[m * M + j] * wr[j];
            wr[m] = a / sH[m * M + m];
          }
          for (int m = M - 1; m >= 0; --m) {
            double a = wr[m];
            for (int j = m + 1; j < M; ++j) a -= sH[j * M + m] * wr[j];
            wr[m] = a / sH[m * M + m];
          }
        }
        lds_sync();
      } else if (spd) {
        // w_i = H^-1 rhs_i, lanes over (i, m): forward then backward substitution, the solved entry
        // of each step handed over in LDS
        for (int m = 0; m < M; ++m) {
          if (wl && wm == m) {
            w /= sH[m * M + m];
            sW[wi * M + m] = w;
          }
          lds_sync();
          if (wl && wm > m) w -= sH[wm * M + m] * sW[wi * M + m];
        }
        for (int m = M - 1; m >= 0; --m) {
          if (wl && wm == m) {
            w /= sH[m * M + m];
            sW[wi * M + m] = w;
          }
          lds_sync();
          if (wl && wm < m) w -= sH[m * M + wm] * sW[wi * M + m];
        }
        lds_sync();
      }
    }
  }
  double est = INFINITY;  // a factorisation that fails: treat as heaviest
  if (spd) {
    // jumps of every reference signal, 64 time steps per pass: lanes flag their step, the jump
    // vectors of the flagged steps are compacted into LDS (ballot prefix), then lanes over (jump,
    // move) pairs add |z| / b_n, b_n = half the tighter of MV n's rate and amplitude ranges (an
    // unbounded MV adds nothing)
    double e = 0.0;
    for (int k = 0; k < nref; ++k) {
      const double* rk = r + (long long)k * my * nit;
      for (int t0 = 1; t0 < nit; t0 += 8 * kWave) {
        // the jump flags of eight passes first: their loads are independent, so they are issued
        // together (one global-memory round trip per output instead of one per pass).  With my <= 4
        // the jump vectors stay in registers, and when the eight passes hold at most 64 jumps they
        // are compacted into LDS at once: one hand-off for the block instead of a global re-read
        // and two hand-offs per pass with a jump
        unsigned jm = 0;
        double dv[8][4];
        if (my <= 4) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const double* ri = rk + (i < my ? i : 0) * nit;
#pragma unroll
            for (int p = 0; p < 8; ++p) {
              const int t = t0 + p * kWave + lane;
              const int tc = t < nit ? t : nit - 1;
              const double a = ri[tc], b = ri[tc - 1];
              const bool j = i < my && t < nit && a != b;
              dv[p][i] = j ? a - b : 0.0;
              if (j) jm |= 1u << p;
            }
          }
        } else {
          for (int i = 0; i < my; ++i) {
            const double* ri = rk + i * nit;
#pragma unroll
            for (int p = 0; p < 8; ++p) {
              const int t = t0 + p * kWave + lane;
              const int tc = t < nit ? t : nit - 1;
              const double a = ri[tc], b = ri[tc - 1];
              if (t < nit && a != b) jm |= 1u << p;
            }
          }
        }
        unsigned long long bal[8];
        int nj = 0;
#pragma unroll
        for (int p = 0; p < 8; ++p) {
          bal[p] = __ballot((jm >> p) & 1u);
          nj += __popcll(bal[p]);
        }
        if (nj == 0) continue;
        if (my <= 4 && nj <= kWave) {
          int off = 0;
#pragma unroll
          for (int p = 0; p < 8; ++p) {
            if ((jm >> p) & 1u) {
              const int slot = off + __popcll(bal[p] & ((1ull << lane) - 1ull));
#pragma unroll
              for (int i = 0; i < 4; ++i)
                if (i < my) sD[slot * my + i] = dv[p][i];
            }
            off += __popcll(bal[p]);
          }
          lds_sync();
          e += jump_demand(sD, sW, sBn, nj, M, my, nuc, lane);
          lds_sync();
          continue;
        }
        for (int p = 0; p < 8; ++p) {
          const int t = t0 + p * kWave + lane;
          const bool jmp = (jm >> p) & 1u;
          if (!bal[p]) continue;
          if (jmp) {
            const int slot = __popcll(bal[p] & ((1ull << lane) - 1ull));
            for (int i = 0; i < my; ++i) sD[slot * my + i] = rk[i * nit + t] - rk[i * nit + t - 1];
          }
          lds_sync();
          e += jump_demand(sD, sW, sBn, __popcll(bal[p]), M, my, nuc, lane);
          lds_sync();
        }
      }
    }
    est = wave_sum64(e);
  }
  if (lane == 0) {
    const double lg = est > 0.0 ? log2(est) : -256.0;
    const double qd = fmin(fmax((lg + 256.0) * 2048.0, 0.0), 1048575.0);
    key[c] = ~(((unsigned)M << 20) | (unsigned)(isnan(qd) ? 1048575.0 : qd));
  }
}

// ---- rank by counting, for batches up to kCountRankMaxC: the stable ascending position of element
// i is the number of elements j with (key_j, j) < (key_i, i), so perm[position] = i is exactly the
// permutation of the stable radix sort.  One wave per two elements, lanes = (element e, chunk h of
// 32): a lane compares its element against one thirty-second of the keys (128 at the metric's 4096
// candidates, eight loads in flight), five xor shuffles add the chunks.  One launch instead of the
// radix sort's three (profiles/r05_key_stages.txt)
constexpr long long kCountRankMaxC = 8192;
template <class K>
__global__ void __launch_bounds__(64) count_rank(const K* __restrict__ keys, int n, int* __restrict__ perm) {
  const int lane = threadIdx.x;
  const int e = lane & 1, h = lane >> 1;
  const int i = blockIdx.x * 2 + e;
  const bool valid = i < n;
  const K ki = keys[valid ? i : 0];
  const int chunk = (n + 31) >> 5;
  const int j0 = h * chunk, j1 = j0 + chunk < n ? j0 + chunk : n;
  int cnt = 0;
#pragma unroll 8
  for (int j = j0; j < j1; ++j) {
    const K kj = keys[j];
    cnt += (kj < ki || (kj == ki && j < i)) ? 1 : 0;
  }
#pragma unroll
  for (int m = 2; m < kWave; m <<= 1) cnt += __shfl_xor(cnt, m, kWave);
  if (valid && h == 0) perm[cnt] = i;
}

int order_candidates(int kind, int my, int nu, long long C, const int* N2, const int* Nu, const double* delta,
                     const double* lambda, WorkOrder& wo, const int** perm, hipStream_t stream, std::string* err,
                     const DevScenario* sc, int nref, const double* r, const DevResult* pre, bool* prefilled) {
  *perm = nullptr;
  if (prefilled) *prefilled = false;
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
  // the controller-based estimate when its per-candidate cost (the upper half of H: one
  // step-table correlation over the horizon per output and entry) stays small; else weight ratio
  const double hcost = sc ? 0.5 * (double)(sc->nu * sc->numax) * (sc->nu * sc->numax) * sc->my * sc->n2max : 0.0;
  const int Mp = sc ? sc->nu * sc->numax : 0;
  const size_t lds = sc ? (size_t)(Mp * Mp + sc->my * Mp + sc->my + sc->my * sc->nu * sc->tlen + kWave * sc->my +
                                   2 * sc->nu) * sizeof(double) + (size_t)sc->my * sizeof(int)
                        : 0;
  if (kind == kOrderGpc && sc && r && !sc->mdband && !sc->nmpc && Mp <= 64 &&
      hcost <= kOrderEstMaxCost && lds <= 64 * 1024) {
    hipLaunchKernelGGL(order_keys_gpc, dim3((unsigned)C), dim3(kWave), lds, stream, *sc, C, nref, N2, Nu, delta,
                       lambda, r, kin, iin, pre ? *pre : DevResult{}, pre ? 1 : 0);
    if (prefilled) *prefilled = pre != nullptr;
  } else {
    hipLaunchKernelGGL(order_keys, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, stream, kind, C, my, nu, N2,
                       Nu, delta, lambda, kin, iin);
  }
  const hipError_t ke = hipGetLastError();
  if (ke != hipSuccess) {
    *err = std::string("dispatch-order key launch failed: ") + hipGetErrorString(ke);
    return -3;
  }
  if (C <= kCountRankMaxC) {
    hipLaunchKernelGGL(count_rank<unsigned>, dim3((unsigned)((C + 1) / 2)), dim3(kWave), 0, stream,
                       (const unsigned*)kin, (int)C, iout);
    if (hipGetLastError() != hipSuccess) {
      *err = "dispatch-order rank launch failed";
      return -3;
    }
  } else if (hipcub::DeviceRadixSort::SortPairs(b + 4 * arr, temp, kin, kout, iin, iout, (int)C, 0, 32, stream) !=
             hipSuccess) {
    *err = "hipcub::DeviceRadixSort::SortPairs failed";
    return -3;
  }
  wo.perm = iout;
  *perm = iout;
  return 0;
}

int order_stage(WorkOrder& wo, long long S, int width, double** stage, std::string* err) {
  const size_t need = (size_t)kXcds * ((S + kXcds - 1) / kXcds) * width * sizeof(double);
  if (need > wo.stage_bytes) {
    if (wo.stage) (void)hipFree(wo.stage);
    wo.stage = nullptr;
    wo.stage_bytes = 0;
    if (hipMalloc(&wo.stage, need) != hipSuccess) {
      *err = "hipMalloc failed (result staging)";
      return -2;
    }
    wo.stage_bytes = need;
  }
  *stage = static_cast<double*>(wo.stage);
  return 0;
}

// thread = staging slot (dispatch order): its row goes to the caller's index perm[c]*nref + k.  A
// scatter, so the sort's permutation serves as is (no inverse-permutation launch); the reads are
// coalesced, the few scattered writes (4096 records at the metric) cost the same
__global__ void unpermute_kernel(const double* __restrict__ stage, const int* __restrict__ perm, long long C,
                                 int nref, int my, int nu, StageRow R, DevResult out) {
  const long long slot = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long S = C * nref;
  if (slot >= S) return;
  const long long cs = slot / nref;
  const long long s = (long long)perm[cs] * nref + (slot - cs * nref);
  const double* row = stage + xcd_row(slot, S) * R.w;
  for (int i = 0; i < my; ++i) {
    if (R.j1 >= 0) out.J1[s * my + i] = row[R.j1 + i];
    if (R.j21 >= 0) out.j21[s * my + i] = row[R.j21 + i];
    if (R.j22 >= 0) out.j22[s * my + i] = row[R.j22 + i];
  }
  if (R.jnu >= 0)
    for (int i = 0; i < nu; ++i) out.Jnu[s * nu + i] = row[R.jnu + i];
  if (R.st >= 0) out.status[s] = (int)row[R.st];
  if (R.it >= 0) out.qp_iters[s] = (long long)row[R.it];
}

// one thread per simulation slot: NaN costs, status MPCT_ST_NOT_RUN, 0 iterations, in the staging
// row of the slot (ordered launches) or at the caller's index.  The slot's simulating launch
// overwrites the whole record; a slot no class launch claims keeps it (VNS2.m:151-163 treats a
// failed sim as an error, never as a value)
__global__ void prefill_kernel(DevResult out, long long S, int my, int nu) {
  const long long s = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  prefill_slot(out, s, S, my, nu);
}

#ifdef MPCT_DIAG
bool diag_drop_launch(int k) {
  const char* e = getenv("MPCT_DIAG_DROP_LAUNCH");
  return e && *e && atoi(e) == k;
}
#endif

int prefill_results(const DevResult& out, long long S, int my, int nu, hipStream_t stream, std::string* err) {
  if (S <= 0) return 0;
  hipLaunchKernelGGL(prefill_kernel, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, stream, out, S, my, nu);
  if (hipGetLastError() != hipSuccess) {
    *err = "result prefill launch failed";
    return -3;
  }
  return 0;
}

int unpermute_results(const WorkOrder& wo, long long C, int nref, int my, int nu, const StageRow& R,
                      const DevResult& out, hipStream_t stream, std::string* err) {
  const long long S = C * nref;
  hipLaunchKernelGGL(unpermute_kernel, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, stream,
                     static_cast<const double*>(wo.stage), wo.perm, C, nref, my, nu, R, out);
  if (hipGetLastError() != hipSuccess) {
    *err = "unpermute_results launch failed";
    return -3;
  }
  return 0;
}

// ---- ranking (mpct_rank_device): s_c = sum_j costs[c][j] w[j] in a fixed order, NaN -> +inf,
// -0 -> +0, mapped to an order-preserving unsigned 64-bit key; the radix sort is stable, so equal
// costs keep the candidate order
__device__ __forceinline__ unsigned long long rank_key(const double* __restrict__ costs, long long c, int k,
                                                       const double* __restrict__ w) {
  double s = 0.0;
  for (int j = 0; j < k; ++j) s = fma(costs[c * k + j], w[j], s);
  if (isnan(s)) s = INFINITY;
  s += 0.0;  // -0 -> +0 (round to nearest)
  const unsigned long long u = (unsigned long long)__double_as_longlong(s);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

__global__ void rank_keys(const double* __restrict__ costs, long long C, int k, const double* __restrict__ w,
                          unsigned long long* __restrict__ key, int* __restrict__ idx) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  key[c] = rank_key(costs, c, k, w);
  idx[c] = (int)c;
}

int rank_device(const double* costs, long long C, int k, const double* w, int* perm, hipStream_t stream,
                std::string* err) {
  if (C == 0) return 0;
  size_t temp = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (const unsigned long long*)nullptr,
                                         (unsigned long long*)nullptr, (const int*)nullptr, (int*)nullptr,
                                         (int)C) != hipSuccess) {
    *err = "hipcub::DeviceRadixSort::SortPairs (size query) failed";
    return -3;
  }
  const bool counting = C <= kCountRankMaxC;  // keys, then the counting rank (no sort buffers)
  const size_t arr8 = ((size_t)C * 8 + 255) & ~(size_t)255, arr4 = ((size_t)C * 4 + 255) & ~(size_t)255;
  void* buf = nullptr;
  if (hipMallocAsync(&buf, counting ? arr8 + arr4 : 2 * arr8 + arr4 + temp, stream) != hipSuccess) {
    *err = "hipMallocAsync failed (ranking buffers)";
    return -2;
  }
  char* b = static_cast<char*>(buf);
  unsigned long long* kin = reinterpret_cast<unsigned long long*>(b);
  unsigned long long* kout = reinterpret_cast<unsigned long long*>(b + arr8);
  int* iin = reinterpret_cast<int*>(b + (counting ? arr8 : 2 * arr8));
  hipLaunchKernelGGL(rank_keys, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, stream, costs, C, k, w, kin, iin);
  int rc = 0;
  if (hipGetLastError() != hipSuccess) {
    *err = "ranking key launch failed";
    rc = -3;
  } else if (counting) {
    hipLaunchKernelGGL(count_rank<unsigned long long>, dim3((unsigned)((C + 1) / 2)), dim3(kWave), 0, stream,
                       (const unsigned long long*)kin, (int)C, perm);
    if (hipGetLastError() != hipSuccess) {
      *err = "ranking launch failed";
      rc = -3;
    }
  } else if (hipcub::DeviceRadixSort::SortPairs(b + 2 * arr8 + arr4, temp, kin, kout, iin, perm, (int)C, 0, 64,
                                                stream) != hipSuccess) {
    *err = "hipcub::DeviceRadixSort::SortPairs failed (ranking)";
    rc = -3;
  }
  (void)hipFreeAsync(buf, stream);
  return rc;
}

void order_release(WorkOrder& wo) {
  if (wo.buf) (void)hipFree(wo.buf);
  if (wo.stage) (void)hipFree(wo.stage);
  if (wo.used) (void)hipEventDestroy(wo.used);
  wo = WorkOrder{};
}

void order_mark_used(WorkOrder& wo, hipStream_t stream) {
  if (wo.used && hipEventRecord(wo.used, stream) == hipSuccess) wo.pending = true;
}

}  // namespace mpct
