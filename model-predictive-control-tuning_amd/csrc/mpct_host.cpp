// mpct_host.cpp — C ABI of libmpct: scenario validation, host precompute of the candidate-
// independent GPC tables, device upload, launch wrappers.  See include/mpct.h.
//
// Host tables (restating the reference's setup functions, natively):
//   step[i][n][t]     step response of model entry (i,n), t = 0..tlen-1      (MatG.m:51 step)
//   F_i rows          Diophantine free-output polynomials for the window      (diophantine.m:35-65)
//   uG_in rows        past-control coefficients, ALL zeros removed, last cp    (deltaUFree.m:13-62)
//   phi[(i,r)][s]     = [F_i row r | uG_i* row r] laid out on the state vector
//                       x = [y_1(t..t-na_1) ... | du_1(t-1..t-duM_1) ...]     (cell2mat2.m,
//                       DTC_GPC_WW.m:139-146: yf = Hp*up + S*Yd)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>
#include <cstdio>
#include <thread>

#include "../../include/mpct.h"
#include "launch_fan.h"
#include "work_order.h"
#include "mpct_dev.h"

namespace mpct {
// defined in gpc_kernel_launch.hip
int launch_closed_loop(const DevScenario& sc, long long C, int nref, const int* N2, const int* Nu,
                       const double* delta, const double* lambda, const double* r,
                       const double* v, const DevOpts& o, const DevResult& out, int maxM,
                       WorkOrder* wo, LaunchFan* fan, hipStream_t stream, std::string* err);
long long lds_bytes_for(const DevScenario& sc, int N2, int Nu, bool ext);
std::string closed_loop_instance(const DevScenario& sc, int maxM, bool ext);
// defined in mdband_kernel.hip
int launch_mdband(const DevScenario& sc, long long C, int nref, const int* N2, const int* Nu, const double* delta,
                  const double* lambda, const double* r, const double* v, const DevOpts& o, const DevResult& out,
                  hipStream_t stream, LaunchFan* fan, std::string* err);
long long mdband_lds_bytes(const DevScenario& sc, int N2, int Nu, int ncopy);
// defined in nmpc_kernel.hip
int launch_nmpc(const DevScenario& sc, long long C, int nref, const int* N, const int* Nu, const double* delta,
                const double* lambda, const double* r, const DevOpts& o, const DevResult& out, hipStream_t stream,
                LaunchFan* fan, WorkOrder* wo, std::string* err);
long long nmpc_lds_bytes(int M, int N);
}  // namespace mpct

using namespace mpct;

// Everything a scenario keeps on one device.  The host-pointer entries run on the library-owned
// stream `stream` and synchronise only it (not the device), so other streams, host threads and
// the contexts of other devices proceed concurrently.
struct DevCtx {
  int dev = -1;
  void* dtab = nullptr;  // the scenario's tables, one 256-B-aligned blob
  DevScenario ds{};
  void* dscratch = nullptr;  // host-API input/result buffers (grow only)
  size_t dscratch_bytes = 0;
  // host-API reference / disturbance signals r | v: the last upload stays on the device and a
  // call whose signals are byte-identical skips the copy (the drop-in's scalar calls pass the
  // same Xsp every time: GAM_fun.m:81, VNS2.m:153)
  void* dsig = nullptr;
  size_t dsig_bytes = 0;
  std::vector<char> sig_host;  // bytes of the signals dsig holds
  hipStream_t stream = nullptr;
  LaunchFan fan;    // auxiliary streams of the class launches (band / NMPC kernels)
  WorkOrder order;  // dispatch-order sort buffers (GPC and NMPC kernels)
};

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

struct mpct_scenario {
  int my = 0, nu = 0, nd = 0, nin = 0, nit = 0, n2max = 0, numax = 0, wsq = 1, ink0 = 9;
  std::vector<int> n1;
  int tlen = 0;
  std::vector<double> step;  // [my][nu][tlen]
  int nx = 0, nyh = 0, nup = 0;
  std::vector<int> yoff, nyhi, upoff, dum;
  std::vector<double> phi;   // [my*n2max][nx]  reference layout (S | Hp)
  std::vector<double> phid;  // same rows on the device state basis (see create)
  int ne = 0, pl_maxb = 0, pl_maxa = 0;
  int npin = 0;  // plant input columns: nu MVs, nd MDs, nq plant-only disturbances
  int nvar = 1;  // plant variants (Monte-Carlo draws); tables are [nvar][ne]
  std::vector<int> pl_nb, pl_na, pl_off;
  std::vector<double> pl_b, pl_a;
  // DTC-GPC predictor (abi >= 2): Pz and Gz entries (2*my*nu, z^-1 form) and the filters Fr_i
  int dtc = 0, nq = 0;
  int mz_maxb = 1, mz_maxa = 1, fr_max = 1;
  std::vector<int> mz_nb, mz_na, mz_off;
  std::vector<double> mz_b, mz_a, fr_b, fr_a;
  std::vector<int> fr_n;
  std::vector<double> bnd;   // [4][nu]
  std::vector<double> yref;  // [my][nit]
  // MD feed-forward + soft output bands (abi >= 3): model entries of all nin columns in the mz_*
  // tables, MD step responses, output bounds, weight scales
  int mdband = 0;
  double rho = 0.0;
  std::vector<double> step_md;  // [my][nd][tlen]
  std::vector<double> obnd;     // [4][my]
  std::vector<double> wscale;   // [my + nu]
  // nonlinear MPC (abi >= 4, mpct_nmpc_scenario_create): my = ny outputs, nu MVs
  int nmpc = 0, nsub = 10, sqp_max = 100;
  double ts = 0.0, sqp_tol = 1e-8;
  std::vector<int> xc;      // [ny] 0-based output states
  std::vector<double> nm;   // see DevScenario::nm
  // device state, one context per device ordinal (created on first use, kept until destroy):
  // a scenario can be evaluated on several GPUs of one process (mpct_eval_batch_multi)
  std::vector<DevCtx*> ctx;
  // further contexts of a device listed more than once in one mpct_eval_batch_multi call:
  // extra[dev][j] serves its (j+2)-th occurrence (own stream, scratch and order buffers)
  std::vector<std::vector<DevCtx*>> extra;
};

extern "C" int32_t mpct_abi_version(void) { return MPCT_ABI_VERSION; }
extern "C" const char* mpct_last_error(void) { return g_err.c_str(); }

// ------------------------------------------------------------------------------------------
static std::vector<double> conv(const std::vector<double>& a, const std::vector<double>& b) {
  if (a.empty() || b.empty()) return {};
  std::vector<double> c(a.size() + b.size() - 1, 0.0);
  for (size_t i = 0; i < a.size(); ++i)
    for (size_t j = 0; j < b.size(); ++j) c[i + j] += a[i] * b[j];
  return c;
}

// direct-form discrete filter of a unit step: z^-delay num(z)/den(z) (tfdata form)
static void step_response(const mpct_dtf& d, int T, double* s) {
  const int len = d.len;
  std::vector<double> b(d.delay + len, 0.0), a(len);
  for (int k = 0; k < len; ++k) {
    b[d.delay + k] = d.num[k] / d.den[0];
    a[k] = d.den[k] / d.den[0];
  }
  std::vector<double> y(T, 0.0);
  for (int t = 0; t < T; ++t) {
    double acc = 0.0;
    for (int l = 0; l < (int)b.size(); ++l)
      if (t - l >= 0) acc += b[l];  // unit step input
    for (int l = 1; l < len; ++l)
      if (t - l >= 0) acc -= a[l] * y[t - l];
    y[t] = acc;
  }
  std::copy(y.begin(), y.end(), s);
}

// descompMPC.m:19-43 followed by the exact-LCM CARIMA form (BA_MIMO.m:20-71 with the row's
// DISTINCT denominator polynomials multiplied, instead of the rounded-roots LCM): what a host that
// passes na = carima_A = nb = carima_B = dp = NULL gets (abi >= 5; the MATLAB MEX host builds its
// descriptor from the mpc object's tfdata alone).  Same arithmetic as mpct/lti.py descomp + carima
// (exact=True), checked against it in tests/test_abi.py.
struct CarimaTables {
  std::vector<int32_t> na, nb, dp;
  std::vector<double> A, B;
};

static void derive_carima(const mpct_dtf* model, int my, int nin, CarimaTables& c) {
  c.na.assign(my, 0);
  c.nb.assign((size_t)my * nin, 0);
  c.dp.assign((size_t)my * nin, 0);
  c.A.clear();
  c.B.clear();
  std::vector<std::vector<double>> Bs((size_t)my * nin);
  for (int i = 0; i < my; ++i) {
    int dmax = 0;
    for (int j = 0; j < nin; ++j) dmax = std::max(dmax, model[i * nin + j].delay);
    for (int j = 0; j < nin; ++j) {
      const mpct_dtf& m = model[i * nin + j];
      std::vector<double> b(m.num, m.num + m.len);
      int dd = m.delay;
      if (b[0] != 0.0) {  // descompMPC.m:35-38: d = d - 1, B = [0 B]
        dd -= 1;
        b.insert(b.begin(), 0.0);
      }
      double sn = 0.0, sd = 0.0;
      for (int k = 0; k < m.len; ++k) {
        sn += m.num[k];
        sd += m.den[k];
      }
      if (sd != 0.0 && sn / sd == 0.0) dd = dmax;  // descompMPC.m:39-41: zero dcgain
      c.dp[i * nin + j] = dd;
      if (b[0] == 0.0) b.erase(b.begin());  // BA_MIMO.m:22-24: one leading zero stripped
      Bs[i * nin + j] = b;
    }
  }
  for (int i = 0; i < my; ++i) {
    std::vector<std::vector<double>> uniq;
    auto den = [&](int j) { return std::vector<double>(model[i * nin + j].den, model[i * nin + j].den + model[i * nin + j].len); };
    for (int j = 0; j < nin; ++j) {
      const std::vector<double> a = den(j);
      if (std::find(uniq.begin(), uniq.end(), a) == uniq.end()) uniq.push_back(a);
    }
    std::vector<double> Ai{1.0};
    for (const auto& u : uniq) Ai = conv(Ai, u);
    c.na[i] = (int)Ai.size() - 1;
    for (double x : Ai) c.A.push_back(x / Ai[0]);
    for (int j = 0; j < nin; ++j) {
      std::vector<double> b = Bs[i * nin + j];
      const std::vector<double> a = den(j);
      for (const auto& u : uniq)
        if (u != a) b = conv(b, u);
      c.nb[i * nin + j] = (int)b.size() - 1;
      for (double x : b) c.B.push_back(x / Ai[0]);
    }
  }
}

extern "C" int32_t mpct_scenario_create(const mpct_scenario_desc* d_in, mpct_scenario** out) {
  if (!d_in || !out) return fail(MPCT_EINVAL, "null argument");
  mpct_scenario_desc dcopy = *d_in;
  const mpct_scenario_desc* d = &dcopy;
  CarimaTables derived;
  if (d_in->abi_version >= 5 && !(d_in->mdband) && d_in->dtc == 0 && !d_in->na && !d_in->carima_A && !d_in->nb &&
      !d_in->carima_B && !d_in->dp && d_in->model && d_in->my >= 1 && d_in->nu >= 1 && d_in->nd >= 0 &&
      d_in->my <= kMaxOut && d_in->nu + d_in->nd <= kMaxIn) {
    const int nin = d_in->nu + d_in->nd;
    for (int e = 0; e < d_in->my * nin; ++e) {
      const mpct_dtf& m = d_in->model[e];
      if (m.len < 1 || !m.num || !m.den || m.den[0] == 0.0 || m.delay < 0) return fail(MPCT_EINVAL, "bad model entry");
    }
    derive_carima(d_in->model, d_in->my, nin, derived);
    dcopy.na = derived.na.data();
    dcopy.nb = derived.nb.data();
    dcopy.dp = derived.dp.data();
    dcopy.carima_A = derived.A.data();
    dcopy.carima_B = derived.B.data();
  }
  *out = nullptr;
  if (d->abi_version < 1 || d->abi_version > MPCT_ABI_VERSION) return fail(MPCT_EINVAL, "abi_version mismatch");
  const int dtc = d->abi_version >= 2 ? (d->dtc ? 1 : 0) : 0;
  const int nq = d->abi_version >= 2 ? d->nq : 0;
  const int nplant = (d->abi_version >= 2 && d->nplant > 1) ? d->nplant : 1;
  const int mdband = d->abi_version >= 3 ? (d->mdband ? 1 : 0) : 0;
  if (mdband && (dtc || nq > 0 || nplant > 1))
    return fail(MPCT_EINVAL, "mdband excludes dtc, plant-only disturbances and plant variants");
  if (mdband && (!d->y_min || !d->y_max || !d->ecr_min || !d->ecr_max))
    return fail(MPCT_EINVAL, "mdband needs y_min, y_max, ecr_min, ecr_max");
  if (nplant > 1 && !d->plant_var) return fail(MPCT_EINVAL, "nplant > 1 needs plant_var");
  if (nq < 0 || (nq > 0 && !d->dist)) return fail(MPCT_EINVAL, "nq > 0 needs dist");
  if (d->my < 1 || d->nu < 1 || d->nd < 0 || d->nit < 1 || d->n2_max < 1 || d->nu_max < 1)
    return fail(MPCT_EINVAL, "non-positive dimension");
  if (d->my > kMaxOut || d->nu + d->nd > kMaxIn) return fail(MPCT_ERANGE, "too many outputs/inputs");
  if (d->nd > 0 && !mdband)
    return fail(MPCT_ERANGE, "measured disturbances (nd > 0) need the mdband kernel (mdband = 1)");
  if (d->nu * d->nu_max + mdband > 64) return fail(MPCT_ERANGE, "nu*nu_max (+1 eps row) > 64 (one wavefront of QP rows)");
  if (!d->n1 || !d->plant || !d->model || !d->du_min || !d->du_max || !d->u_min || !d->u_max || !d->yref)
    return fail(MPCT_EINVAL, "null table pointer");
  if (!mdband && (!d->na || !d->carima_A || !d->nb || !d->carima_B || !d->dp))
    return fail(MPCT_EINVAL, "null CARIMA table pointer");
  auto* s = new mpct_scenario();
  s->my = d->my;
  s->nu = d->nu;
  s->nd = d->nd;
  s->nin = d->nu + d->nd;
  s->dtc = dtc;
  s->nq = nq;
  s->npin = s->nin + nq;
  s->nvar = nplant;
  s->mdband = mdband;
  if (s->npin > kMaxIn) {
    delete s;
    return fail(MPCT_ERANGE, "too many plant inputs");
  }
  s->nit = d->nit;
  s->n2max = d->n2_max;
  s->numax = d->nu_max;
  s->wsq = d->weights_squared ? 1 : 0;
  s->ink0 = d->vns_ink - 1;
  const int my = s->my, nu = s->nu, nin = s->nin, N = s->n2max;
  s->n1.assign(d->n1, d->n1 + my);
  int n1max = 0;
  for (int i = 0; i < my; ++i) {
    if (s->n1[i] < 1) {
      delete s;
      return fail(MPCT_EINVAL, "n1[i] must be >= 1");
    }
    n1max = std::max(n1max, s->n1[i]);
  }
  // ---- step table (MatG.m:51): enough samples for s(n1 + r - c), r < n2max
  s->tlen = n1max + N;
  s->step.assign((size_t)my * nu * s->tlen, 0.0);
  for (int i = 0; i < my; ++i)
    for (int n = 0; n < nu; ++n) {
      const mpct_dtf& m = d->model[i * nin + n];
      if (m.len < 1 || !m.num || !m.den || m.den[0] == 0.0 || m.delay < 0) {
        delete s;
        return fail(MPCT_EINVAL, "bad model entry");
      }
      step_response(m, s->tlen, &s->step[((size_t)i * nu + n) * s->tlen]);
    }
  if (mdband) {
    for (int i = 0; i < my; ++i)
      if (s->n1[i] != 1) {
        delete s;
        return fail(MPCT_EINVAL, "mdband predicts over the toolbox window: n1[i] must be 1");
      }
  } else {
  // ---- CARIMA offsets
  std::vector<int> aoff(my + 1, 0), boff(my * nin + 1, 0);
  for (int i = 0; i < my; ++i) {
    if (d->na[i] < 0) {
      delete s;
      return fail(MPCT_EINVAL, "na < 0");
    }
    aoff[i + 1] = aoff[i] + d->na[i] + 1;
  }
  for (int e = 0; e < my * nin; ++e) {
    if (d->nb[e] < 0 || d->dp[e] < 0) {
      delete s;
      return fail(MPCT_EINVAL, "nb/dp < 0");
    }
    boff[e + 1] = boff[e] + d->nb[e] + 1;
  }
  // ---- state layout
  s->yoff.resize(my);
  s->nyhi.resize(my);
  int o = 0;
  for (int i = 0; i < my; ++i) {
    s->yoff[i] = o;
    s->nyhi[i] = d->na[i] + 1;
    o += d->na[i] + 1;
  }
  s->nyh = o;
  // cp(i,n) = dp + length(B) - 1  (deltaUFree.m:25-29)
  std::vector<int> cp(my * nu);
  s->dum.assign(nu, 0);
  for (int i = 0; i < my; ++i)
    for (int n = 0; n < nu; ++n) {
      int c = d->dp[i * nin + n] + (d->nb[i * nin + n] + 1) - 1;
      if (c < 1) c = 1;
      cp[i * nu + n] = c;
      s->dum[n] = std::max(s->dum[n], c);
    }
  s->upoff.resize(nu);
  for (int n = 0; n < nu; ++n) {
    s->upoff[n] = o;
    o += s->dum[n];
  }
  s->nx = o;
  s->nup = o - s->nyh;
  if (s->nx + my > 256) {
    delete s;
    return fail(MPCT_ERANGE, "free-response state too large");
  }
  if (nu * s->numax > kWave - 1) {
    delete s;
    return fail(MPCT_ERANGE, "nu*nu_max must be < 64 (one QP row per lane)");
  }
  // ---- Diophantine + deltaUFree per output (window rows j = n1_i .. n1_i + N - 1)
  s->phi.assign((size_t)my * N * s->nx, 0.0);
  for (int i = 0; i < my; ++i) {
    const int na = d->na[i];
    const double* A = d->carima_A + aoff[i];
    if (A[0] != 1.0) {
      delete s;
      return fail(MPCT_EINVAL, "carima_A[i][0] must be 1");
    }
    // diophantine(A, N, d): N1 = d+1; DTC-GPC predicts from the delay-free yp (d = 0,
    // DTC_GPC_WW.m:80) while MatG keeps the dmin+1 window
    const int dd = s->dtc ? 0 : s->n1[i] - 1;
    std::vector<double> Ai(A, A + na + 1);
    std::vector<double> AD = conv(Ai, {1.0, -1.0});  // A~ = A*Delta (diophantine.m:35)
    const int nAD = (int)AD.size();                 // na + 2
    const int rows = dd + N + 1;
    std::vector<double> f((size_t)rows * (nAD - 1), 0.0);
    auto F = [&](int j, int k) -> double& { return f[(size_t)j * (nAD - 1) + k]; };
    F(0, 0) = 1.0;
    for (int j = 0; j < dd + N; ++j) {  // diophantine.m:55-63
      for (int k = 0; k < nAD - 2; ++k) F(j + 1, k) = F(j, k + 1) - F(j, 0) * AD[k + 1];
      F(j + 1, nAD - 2) = -F(j, 0) * AD[nAD - 1];
    }
    for (int r = 0; r < N; ++r) {
      const int j = dd + 1 + r;  // prediction step of this row (1-based)
      double* prow = &s->phi[((size_t)i * N + r) * s->nx];
      for (int k = 0; k <= na; ++k) prow[s->yoff[i] + k] = F(j, k);
      // E_j = [1, f(1,0), ..., f(j-1,0)]  (diophantine.m:69-77)
      std::vector<double> E(j);
      E[0] = 1.0;
      for (int k = 1; k < j; ++k) E[k] = F(k, 0);
      for (int n = 0; n < nu; ++n) {
        const int e = i * nin + n;
        std::vector<double> B(d->carima_B + boff[e], d->carima_B + boff[e + 1]);
        std::vector<double> aux = conv(E, B);
        std::vector<double> BE;
        for (double v : aux)
          if (v != 0.0) BE.push_back(v);  // deltaUFree.m:40-45: every zero removed
        const int c = cp[i * nu + n];
        const int lBE = (int)BE.size();
        double* dst = prow + s->upoff[n];  // left-aligned block (cell2mat2.m:56)
        if (lBE < c) {
          for (int k = 0; k < c - lBE; ++k) dst[k] = 0.0;
          for (int k = 0; k < lBE; ++k) dst[c - lBE + k] = BE[k];
        } else {
          for (int k = 0; k < c; ++k) dst[k] = BE[lBE - c + k];
        }
      }
    }
  }
  // ---- device copy of phi in a well-conditioned basis.  The F rows have
  // large alternating coefficients (|F| ~ 3e3 for Shell 3x3) that cancel on the slowly varying
  // y history; folded into the gain matrix they amplify rounding ~1e4x.  Rewrite the y part on
  // backward differences, y(t-l) = sum_k (-1)^k C(l,k) nabla^k y(t), and use the identity
  // F_j(1) = 1 (Atilde(1) = 0 in 1 = E_j Atilde + z^-j F_j) to make the nabla^0 column exactly
  // 1: the device state is [y_i(t) - r_i(t), nabla y_i(t), ..., nabla^na y_i(t) | du history].
  s->phid = s->phi;
  for (int i = 0; i < my; ++i) {
    const int n = d->na[i] + 1;
    std::vector<double> binom((size_t)n * n, 0.0);
    for (int l = 0; l < n; ++l) {
      binom[(size_t)l * n] = 1.0;
      for (int k = 1; k <= l; ++k) binom[(size_t)l * n + k] = binom[(size_t)(l - 1) * n + k - 1] +
                                                           (k <= l - 1 ? binom[(size_t)(l - 1) * n + k] : 0.0);
    }
    for (int r = 0; r < N; ++r) {
      const double* src = &s->phi[((size_t)i * N + r) * s->nx + s->yoff[i]];
      double* dst = &s->phid[((size_t)i * N + r) * s->nx + s->yoff[i]];
      for (int k = 0; k < n; ++k) {
        double a = 0.0;
        for (int l = k; l < n; ++l) a += src[l] * ((k & 1) ? -binom[(size_t)l * n + k] : binom[(size_t)l * n + k]);
        dst[k] = a;
      }
      dst[0] = 1.0;
    }
  }
  }  // !mdband
  // ---- plant entries in z^-1 form (delay folded into b); plant-only disturbance paths appended
  // as columns nin..npin-1 of each output row
  const int npin = s->npin;
  s->ne = my * npin;
  const int nve = s->nvar * s->ne;  // entries over all variants: ev = variant*ne + e
  s->pl_nb.resize(nve);
  s->pl_na.resize(nve);
  auto plant_entry = [&](int ev) -> const mpct_dtf& {
    const int v = ev / s->ne, e = ev % s->ne;
    const int i = e / npin, j = e % npin;
    if (j >= nin) return d->dist[i * nq + (j - nin)];
    return s->nvar > 1 ? d->plant_var[(size_t)v * my * nin + i * nin + j] : d->plant[i * nin + j];
  };
  for (int e = 0; e < nve; ++e) {
    const mpct_dtf& p = plant_entry(e);
    if (p.len < 1 || !p.num || !p.den || p.den[0] == 0.0 || p.delay < 0) {
      delete s;
      return fail(MPCT_EINVAL, "bad plant entry");
    }
    s->pl_nb[e] = p.delay + p.len;
    s->pl_na[e] = p.len;
    s->pl_maxb = std::max(s->pl_maxb, s->pl_nb[e]);
    s->pl_maxa = std::max(s->pl_maxa, s->pl_na[e]);
    const int j = (e % s->ne) % npin;
    if (j < nu && p.delay == 0 && p.num[0] != 0.0) {
      delete s;
      return fail(MPCT_EINVAL, "plant has direct feedthrough from an MV (algebraic loop)");
    }
  }
  for (int n = 0; n < (mdband ? 0 : nu); ++n)
    if (s->dum[n] > kMaxDum) {
      delete s;
      return fail(MPCT_ERANGE, "past-control register longer than the device supports (16)");
    }
  for (int i = 0; i < (mdband ? 0 : my); ++i)
    if (s->nyhi[i] > kYeHist) {
      delete s;
      return fail(MPCT_ERANGE, "CARIMA denominator order too high for the device (na <= 7)");
    }
  if (s->pl_maxb > kMaxTaps || s->pl_maxa > kYeHist) {
    delete s;
    return fail(MPCT_ERANGE, "plant entry too long for the device history rings");
  }
  s->pl_b.assign((size_t)nve * s->pl_maxb, 0.0);
  s->pl_a.assign((size_t)nve * s->pl_maxa, 0.0);
  for (int e = 0; e < nve; ++e) {
    const mpct_dtf& p = plant_entry(e);
    for (int k = 0; k < p.len; ++k) {
      s->pl_b[(size_t)e * s->pl_maxb + p.delay + k] = p.num[k] / p.den[0];
      s->pl_a[(size_t)e * s->pl_maxa + k] = p.den[k] / p.den[0];
    }
  }
  s->pl_off.assign(nve, 0);
  for (int e = 0; e < nve; ++e) {
    int o = 0;
    while (o < s->pl_nb[e] && s->pl_b[(size_t)e * s->pl_maxb + o] == 0.0) ++o;
    s->pl_off[e] = o;
  }
  if (s->dtc) {
    // Pz entries (e < my*nu, real delays) and Gz entries (delays minus dmin_i = n1_i - 1,
    // DTC_GPC_WW.m:40-46) in z^-1 form; filters Fr_i (mimofilter.m) with delay 0
    const int nm = 2 * my * nu;
    s->mz_nb.resize(nm);
    s->mz_na.resize(nm);
    s->mz_off.resize(nm);
    for (int e = 0; e < nm; ++e) {
      const int k = e % (my * nu), i = k / nu, j = k % nu;
      const mpct_dtf& m = d->model[i * nin + j];
      const int del = e < my * nu ? m.delay : m.delay - (s->n1[i] - 1);
      if (del < 0) {
        delete s;
        return fail(MPCT_EINVAL, "DTC: model delay below dmin (n1 - 1)");
      }
      s->mz_nb[e] = del + m.len;
      s->mz_na[e] = m.len;
      s->mz_maxb = std::max(s->mz_maxb, s->mz_nb[e]);
      s->mz_maxa = std::max(s->mz_maxa, s->mz_na[e]);
    }
    if (s->mz_maxb > kMaxTaps || s->mz_maxa > kYeHist) {
      delete s;
      return fail(MPCT_ERANGE, "DTC: model entry too long for the device history rings");
    }
    s->mz_b.assign((size_t)nm * s->mz_maxb, 0.0);
    s->mz_a.assign((size_t)nm * s->mz_maxa, 0.0);
    for (int e = 0; e < nm; ++e) {
      const int k = e % (my * nu), i = k / nu, j = k % nu;
      const mpct_dtf& m = d->model[i * nin + j];
      const int del = e < my * nu ? m.delay : m.delay - (s->n1[i] - 1);
      for (int q2 = 0; q2 < m.len; ++q2) {
        s->mz_b[(size_t)e * s->mz_maxb + del + q2] = m.num[q2] / m.den[0];
        s->mz_a[(size_t)e * s->mz_maxa + q2] = m.den[q2] / m.den[0];
      }
      int o2 = 0;
      while (o2 < s->mz_nb[e] && s->mz_b[(size_t)e * s->mz_maxb + o2] == 0.0) ++o2;
      s->mz_off[e] = o2;
    }
    s->fr_n.assign(my, 1);
    for (int i = 0; i < my; ++i)
      if (d->filter) s->fr_n[i] = d->filter[i].len;
    for (int i = 0; i < my; ++i) s->fr_max = std::max(s->fr_max, s->fr_n[i]);
    if (s->fr_max > kYeHist) {
      delete s;
      return fail(MPCT_ERANGE, "DTC: filter order too high (len <= 8)");
    }
    s->fr_b.assign((size_t)my * s->fr_max, 0.0);
    s->fr_a.assign((size_t)my * s->fr_max, 0.0);
    for (int i = 0; i < my; ++i) {
      if (!d->filter) {
        s->fr_b[(size_t)i * s->fr_max] = 1.0;
        s->fr_a[(size_t)i * s->fr_max] = 1.0;
        continue;
      }
      const mpct_dtf& f = d->filter[i];
      if (f.len < 1 || !f.num || !f.den || f.den[0] == 0.0 || f.delay != 0) {
        delete s;
        return fail(MPCT_EINVAL, "DTC: bad filter entry (delay must be 0)");
      }
      for (int q2 = 0; q2 < f.len; ++q2) {
        s->fr_b[(size_t)i * s->fr_max + q2] = f.num[q2] / f.den[0];
        s->fr_a[(size_t)i * s->fr_max + q2] = f.den[q2] / f.den[0];
      }
    }
  }
  if (mdband) {
    // the model of every column (MV and MD), z^-1 form with its delay: the window extension
    // (mdband_kernel.hip); plant == model (closedloop_toolbox.m:50 sims the controller's model)
    const int nm = my * nin;
    s->mz_nb.resize(nm);
    s->mz_na.resize(nm);
    s->mz_off.resize(nm);
    for (int e = 0; e < nm; ++e) {
      const mpct_dtf& m = d->model[e];
      const mpct_dtf& p = d->plant[e];
      if (m.len < 1 || !m.num || !m.den || m.den[0] == 0.0 || m.delay < 0) {
        delete s;
        return fail(MPCT_EINVAL, "bad model entry");
      }
      bool same = p.len == m.len && p.delay == m.delay;
      for (int k = 0; same && k < m.len; ++k) same = p.num[k] == m.num[k] && p.den[k] == m.den[k];
      if (!same) {
        delete s;
        return fail(MPCT_ERANGE, "mdband: plant must equal the model (the toolbox estimator is not restated)");
      }
      s->mz_nb[e] = m.delay + m.len;
      s->mz_na[e] = m.len;
      s->mz_maxb = std::max(s->mz_maxb, s->mz_nb[e]);
      s->mz_maxa = std::max(s->mz_maxa, s->mz_na[e]);
    }
    if (s->mz_maxb > kMaxTaps || s->mz_maxa > kYeHist) {
      delete s;
      return fail(MPCT_ERANGE, "mdband: model entry too long for the device history rings");
    }
    s->mz_b.assign((size_t)nm * s->mz_maxb, 0.0);
    s->mz_a.assign((size_t)nm * s->mz_maxa, 0.0);
    for (int e = 0; e < nm; ++e) {
      const mpct_dtf& m = d->model[e];
      for (int q2 = 0; q2 < m.len; ++q2) {
        s->mz_b[(size_t)e * s->mz_maxb + m.delay + q2] = m.num[q2] / m.den[0];
        s->mz_a[(size_t)e * s->mz_maxa + q2] = m.den[q2] / m.den[0];
      }
      int o2 = 0;
      while (o2 < s->mz_nb[e] && s->mz_b[(size_t)e * s->mz_maxb + o2] == 0.0) ++o2;
      s->mz_off[e] = o2;
    }
    const int nd = s->nd;
    s->step_md.assign((size_t)my * std::max(nd, 1) * s->tlen, 0.0);
    for (int i = 0; i < my; ++i)
      for (int j = 0; j < nd; ++j)
        step_response(d->model[i * nin + nu + j], s->tlen, &s->step_md[((size_t)i * nd + j) * s->tlen]);
    s->obnd.assign(4 * my, 0.0);
    s->wscale.assign(my + nu, 1.0);
    for (int i = 0; i < my; ++i) {
      const double sy = d->y_scale ? d->y_scale[i] : 1.0;
      if (!(sy > 0.0) || !(d->ecr_min[i] >= 0.0) || !(d->ecr_max[i] >= 0.0) || !(d->y_min[i] <= d->y_max[i])) {
        delete s;
        return fail(MPCT_EINVAL, "mdband: bad output bound / ECR / scale factor");
      }
      s->obnd[i] = d->y_min[i];
      s->obnd[my + i] = d->y_max[i];
      s->obnd[2 * my + i] = d->ecr_min[i] * sy;
      s->obnd[3 * my + i] = d->ecr_max[i] * sy;
      s->wscale[i] = 1.0 / sy;
    }
    for (int n = 0; n < nu; ++n) {
      const double su = d->u_scale ? d->u_scale[n] : 1.0;
      if (!(su > 0.0)) {
        delete s;
        return fail(MPCT_EINVAL, "mdband: bad MV scale factor");
      }
      s->wscale[my + n] = 1.0 / su;
    }
    s->rho = d->rho_ecr;
    if (!(s->rho > 0.0)) {
      delete s;
      return fail(MPCT_EINVAL, "mdband: rho_ecr must be > 0");
    }
  }
  s->bnd.resize(4 * nu);
  for (int n = 0; n < nu; ++n) {
    s->bnd[n] = d->du_min[n];
    s->bnd[nu + n] = d->du_max[n];
    s->bnd[2 * nu + n] = d->u_min[n];
    s->bnd[3 * nu + n] = d->u_max[n];
    if (!(s->bnd[n] <= 0.0 && s->bnd[nu + n] >= 0.0 && s->bnd[2 * nu + n] <= 0.0 &&
          s->bnd[3 * nu + n] >= 0.0)) {
      delete s;
      return fail(MPCT_EINVAL, "bounds must contain 0 (nominal u = 0 must be feasible)");
    }
  }
  s->yref.assign(d->yref, d->yref + (size_t)my * s->nit);
  *out = s;
  g_err.clear();
  return MPCT_OK;
}

// ------------------------------------------------------------------------------------------
// nonlinear MPC scenario (closedloop_toolbox_nmpc.m; VanDeVusse_NMPC.m)
static const double kVdvParams[NM_NPAR] = {  // nmpc_vandevusse_state.m:43-58
    1.287e12, 1.287e12, 9.043e9, -9758.3, -9758.3, -8560.0, -4.20, 11.00, 41.85,
    0.9342,   3.01,     4032.0,  0.215,   10.0,    130.00,  5.10};

extern "C" int32_t mpct_nmpc_scenario_create(const mpct_nmpc_desc* d, mpct_scenario** out) {
  if (!d || !out) return fail(MPCT_EINVAL, "null argument");
  *out = nullptr;
  if (d->abi_version < 4 || d->abi_version > MPCT_ABI_VERSION) return fail(MPCT_EINVAL, "abi_version mismatch");
  if (d->model != MPCT_NMPC_VANDEVUSSE) return fail(MPCT_EINVAL, "unknown NMPC model id");
  if (d->nx != 3 || d->nu != 2) return fail(MPCT_EINVAL, "the Van de Vusse model has nx = 3, nu = 2");
  if (d->ny < 1 || d->ny > 2) return fail(MPCT_ERANGE, "ny must be 1 or 2");
  if (d->nit < 1 || d->n_max < 1 || d->nu_max < 1) return fail(MPCT_EINVAL, "non-positive dimension");
  if (d->nu * d->nu_max > 32) return fail(MPCT_ERANGE, "nu*nu_max > 32");
  {
    // the LDS of every (M, N) a candidate may use (not monotone in N: nm_groups), as the launch checks
    long long lds_all = 0;
    for (int m = 1; m <= d->nu * d->nu_max; ++m)
      for (int n = 1; n <= d->n_max; ++n) lds_all = std::max(lds_all, nmpc_lds_bytes(m, n));
    if (lds_all > 64 * 1024)
      return fail(MPCT_ERANGE, "n_max x nu*nu_max needs more than 64 KiB of LDS per simulation");
  }
  if (!(d->ts > 0.0) || d->nsub < 1) return fail(MPCT_EINVAL, "ts must be > 0 and nsub >= 1");
  if (!d->xc || !d->x0 || !d->u0 || !d->u_min || !d->u_max || !d->x_min || !d->x_max || !d->y_scale ||
      !d->u_scale || !d->yref)
    return fail(MPCT_EINVAL, "null table pointer");
  for (int j = 0; j < d->ny; ++j)
    if (d->xc[j] < 1 || d->xc[j] > d->nx) return fail(MPCT_EINVAL, "xc out of range (1-based state index)");
  for (int n = 0; n < d->nu; ++n) {
    if (!(d->u_min[n] < d->u_max[n])) return fail(MPCT_EINVAL, "u_min must be < u_max");
    if (!(d->u_scale[n] > 0.0)) return fail(MPCT_EINVAL, "u_scale must be > 0");
  }
  for (int j = 0; j < d->ny; ++j)
    if (!(d->y_scale[j] > 0.0)) return fail(MPCT_EINVAL, "y_scale must be > 0");
  auto* s = new mpct_scenario();
  s->nmpc = 1;
  s->my = d->ny;
  s->nu = d->nu;
  s->nd = 0;
  s->npin = d->nu;
  s->nit = d->nit;
  s->n2max = d->n_max;
  s->numax = d->nu_max;
  s->ink0 = d->vns_ink > 0 ? d->vns_ink - 1 : 9;
  s->nsub = d->nsub;
  s->ts = d->ts;
  s->sqp_max = d->sqp_max > 0 ? d->sqp_max : 100;
  s->sqp_tol = d->sqp_tol > 0.0 ? d->sqp_tol : 1e-8;
  for (int j = 0; j < d->ny; ++j) s->xc.push_back(d->xc[j] - 1);
  const double* p = d->params ? d->params : kVdvParams;
  s->nm.assign(p, p + NM_NPAR);
  auto app = [&](const double* a, int n) { s->nm.insert(s->nm.end(), a, a + n); };
  app(d->x0, 3);
  app(d->u0, d->nu);
  app(d->u_min, d->nu);
  app(d->u_max, d->nu);
  app(d->x_min, 3);
  app(d->x_max, 3);
  app(d->y_scale, d->ny);
  app(d->u_scale, d->nu);
  s->yref.assign(d->yref, d->yref + (size_t)d->ny * d->nit);
  *out = s;
  g_err.clear();
  return MPCT_OK;
}

static void ctx_release(DevCtx* c) {
  (void)hipSetDevice(c->dev);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->dtab) (void)hipFree(c->dtab);
  if (c->dscratch) (void)hipFree(c->dscratch);
  if (c->dsig) (void)hipFree(c->dsig);
  order_release(c->order);
  c->fan.release();
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

extern "C" void mpct_scenario_destroy(mpct_scenario* s) {
  if (!s) return;
  int cur = -1;
  bool any = std::any_of(s->ctx.begin(), s->ctx.end(), [](DevCtx* c) { return c != nullptr; });
  for (auto& v : s->extra) any = any || !v.empty();
  if (any && hipGetDevice(&cur) != hipSuccess) cur = -1;
  for (DevCtx* c : s->ctx)
    if (c) ctx_release(c);
  for (auto& v : s->extra)
    for (DevCtx* c : v) ctx_release(c);
  if (cur >= 0) (void)hipSetDevice(cur);
  delete s;
}

extern "C" int64_t mpct_scenario_table(const mpct_scenario* s, int32_t which, double* buf, int64_t cap) {
  if (!s) return fail(MPCT_EINVAL, "null scenario");
  std::vector<double> dims;
  const std::vector<double>* src = nullptr;
  if (which == 0)
    src = &s->step;
  else if (which == 1)
    src = &s->phi;
  else if (which == 3)
    src = &s->phid;
  else if (which == 2) {
    dims = {(double)s->my, (double)s->nu, (double)s->nd, (double)s->n2max, (double)s->numax,
            (double)s->tlen, (double)s->nx, (double)s->nyh, (double)s->nup, (double)s->nit, (double)s->nq};
    src = &dims;
  } else
    return fail(MPCT_EINVAL, "unknown table");
  int64_t n = (int64_t)src->size();
  if (buf && cap > 0) std::memcpy(buf, src->data(), sizeof(double) * (size_t)std::min<int64_t>(n, cap));
  return n;
}

// ------------------------------------------------------------------------------------------
// every per-lane history / coefficient set fits gpc_kernel.hip's register caps (kReg*)
static int regpath(const mpct_scenario* s) {
  bool rp = !s->mdband && !s->nmpc && s->pl_maxa - 1 <= kRegA;  // gpc_kernel.hip only
  for (int e = 0; e < s->nvar * s->ne; ++e) rp = rp && (s->pl_nb[e] - s->pl_off[e] <= kRegB);
  for (int n = 0; rp && n < s->nu; ++n) rp = rp && (s->dum[n] <= kRegDu);
  for (int i = 0; rp && i < s->my; ++i) rp = rp && (s->nyhi[i] <= kRegY);
  return rp ? 1 : 0;
}

// gpc_small_kernel's lane tables (gpc_small.hip), or false when the scenario is not a small plant:
// my <= 4 outputs, nu <= 3 MVs, no MD / plant-only inputs, one plant, GPC mode, y difference state
// <= kSmY entries (<= 4 per output), past-control registers <= kSmR, <= 4 plant terms per entry
struct SmallTables {
  int ke = 2;
  std::vector<double> coef;
  std::vector<int> hoff, hc, hmask, acol;
};
static bool small_plant(const mpct_scenario* s, SmallTables* tb = nullptr) {
  if (s->mdband || s->nmpc || s->dtc || s->nd || s->nq || s->nvar != 1) return false;
  if (s->my > 4 || s->nu > 3 || s->npin != s->nu || s->nyh > kSmY) return false;
  for (int i = 0; i < s->my; ++i)
    if (s->nyhi[i] > 4) return false;
  for (int n = 0; n < s->nu; ++n)
    if (s->dum[n] > kSmR) return false;
  for (int e = 0; e < s->ne; ++e) {
    const int nbz = s->pl_nb[e] - s->pl_off[e], na1 = s->pl_na[e] - 1;
    if (nbz + na1 > 4 || na1 >= kSmE || s->pl_nb[e] > kSmU) return false;
  }
  if (!tb) return true;
  int na_max = 0;
  for (int e = 0; e < s->ne; ++e) na_max = std::max(na_max, s->pl_na[e] - 1);
  tb->ke = na_max < 2 ? 2 : 4;  // entry output ring: a power of two above the denominator taps
  tb->coef.assign(kWave, 0.0);
  tb->hoff.assign(kWave, 0);
  tb->hc.assign(kWave, 0);
  tb->hmask.assign(kWave, kSmU - 1);
  for (int L = 0; L < kWave; ++L) {
    const int k = L >> 4, ep = L & 15, i = ep >> 2, j = ep & 3;
    if (i >= s->my || j >= s->nu) continue;
    const int e = i * s->npin + j;
    const int off = s->pl_off[e], nbz = s->pl_nb[e] - off, na1 = s->pl_na[e] - 1;
    if (k < nbz) {  // b tap: u_j(t - off - k)
      tb->coef[L] = s->pl_b[(size_t)e * s->pl_maxb + off + k];
      tb->hoff[L] = j * kSmU;
      tb->hc[L] = off + k;
    } else if (k < nbz + na1) {  // a tap jj: -a_jj y_e(t - jj)
      const int jj = k - nbz + 1;
      tb->coef[L] = -s->pl_a[(size_t)e * s->pl_maxa + jj];
      tb->hoff[L] = kSmEOff + ep * tb->ke;
      tb->hc[L] = jj;
      tb->hmask[L] = tb->ke - 1;
    }
  }
  // A's columns: y part in state order, then MV n's past-control register (age k) at
  // kSmY + kSmR n + k
  tb->acol.assign(s->nx, 0);
  for (int c = 0; c < s->nyh; ++c) tb->acol[c] = c;
  for (int n = 0; n < s->nu; ++n)
    for (int k = 0; k < s->dum[n]; ++k) tb->acol[s->upoff[n] + k] = kSmY + kSmR * n + k;
  return true;
}

// dtc_small_kernel's lane tables (dtc_small.hip), or false when the scenario is not a DTC-GPC small
// plant: DTC mode with every move bound infinite (DTC_GPC_WW.m's unconstrained loop: no QP), my <= 2,
// nu <= 2, nu + nq <= 4 ring-fed inputs (no MDs), every entry of every plant variant, of Pz and of Gz
// <= 4 terms with rings the kernel holds, filters of <= 4 taps, y difference state <= 4 per output,
// past-control registers <= kSmR.  Tables: coef / hoff / hc / hmask [nvar][64] (lane L = 16 k + 4 q
// + p: quads q < my the plant entries (i = q, input p), quads 2 + i: p < 2 Pz(i, p), p >= 2
// Gz(i, p - 2)), the acol map as for gpc_small, filters fr [my][8] = fb 0..3 | fa 0..3
static bool dtc_small_plant(const mpct_scenario* s, SmallTables* tb = nullptr, std::vector<double>* fr = nullptr) {
  if (!s->dtc || s->mdband || s->nmpc || s->nd || s->my > 2 || s->nu > 2 || s->npin > 4) return false;
  for (int n = 0; n < s->nu; ++n)
    if (!(std::isinf(s->bnd[n]) && std::isinf(s->bnd[s->nu + n]) && std::isinf(s->bnd[2 * s->nu + n]) &&
          std::isinf(s->bnd[3 * s->nu + n])))
      return false;
  if (s->nyh > kSmY) return false;
  for (int i = 0; i < s->my; ++i)
    if (s->nyhi[i] > 4 || s->fr_n[i] > 4) return false;
  for (int n = 0; n < s->nu; ++n)
    if (s->dum[n] > kSmR) return false;
  int na_max = 0;
  auto fits = [&](int nb, int off, int na) {
    na_max = std::max(na_max, na - 1);
    return (nb - off) + (na - 1) <= 4 && na - 1 < kSmE && nb <= kSmU;
  };
  for (int e = 0; e < s->nvar * s->ne; ++e)
    if (!fits(s->pl_nb[e], s->pl_off[e], s->pl_na[e])) return false;
  for (int e = 0; e < 2 * s->my * s->nu; ++e)
    if (!fits(s->mz_nb[e], s->mz_off[e], s->mz_na[e])) return false;
  if (!tb) return true;
  tb->ke = na_max < 2 ? 2 : 4;
  const int V = s->nvar;
  tb->coef.assign((size_t)V * kWave, 0.0);
  tb->hoff.assign((size_t)V * kWave, 0);
  tb->hc.assign((size_t)V * kWave, 0);
  tb->hmask.assign((size_t)V * kWave, kSmU - 1);
  for (int v = 0; v < V; ++v)
    for (int L = 0; L < kWave; ++L) {
      const int k = L >> 4, ep = L & 15, q = ep >> 2, pp = ep & 3;
      int nb, off, na, j;
      const double *b, *a;
      if (q < 2) {  // plant entry (q, pp) of variant v
        if (q >= s->my || pp >= s->npin) continue;
        const int e = v * s->ne + q * s->npin + pp;
        nb = s->pl_nb[e], off = s->pl_off[e], na = s->pl_na[e], j = pp;
        b = &s->pl_b[(size_t)e * s->pl_maxb];
        a = &s->pl_a[(size_t)e * s->pl_maxa];
      } else {  // Pz (pp < 2) / Gz (pp >= 2) entry (q - 2, pp & 1): the controller's own inputs
        const int i = q - 2;
        j = pp & 1;
        if (i >= s->my || j >= s->nu) continue;
        const int e = (pp >= 2 ? s->my * s->nu : 0) + i * s->nu + j;
        nb = s->mz_nb[e], off = s->mz_off[e], na = s->mz_na[e];
        b = &s->mz_b[(size_t)e * s->mz_maxb];
        a = &s->mz_a[(size_t)e * s->mz_maxa];
      }
      const int nbz = nb - off, Li = v * kWave + L;
      if (k < nbz) {  // b tap: input j at t - off - k
        tb->coef[Li] = b[off + k];
        tb->hoff[Li] = j * kSmU;
        tb->hc[Li] = off + k;
      } else if (k < nbz + na - 1) {  // a tap jj: -a_jj y_e(t - jj)
        const int jj = k - nbz + 1;
        tb->coef[Li] = -a[jj];
        tb->hoff[Li] = kDtcEOff + ep * tb->ke;
        tb->hc[Li] = jj;
        tb->hmask[Li] = tb->ke - 1;
      }
    }
  tb->acol.assign(s->nx, 0);
  for (int c = 0; c < s->nyh; ++c) tb->acol[c] = c;
  for (int n = 0; n < s->nu; ++n)
    for (int k = 0; k < s->dum[n]; ++k) tb->acol[s->upoff[n] + k] = kSmY + kSmR * n + k;
  if (fr) {
    fr->assign((size_t)s->my * 8, 0.0);
    for (int i = 0; i < s->my; ++i)
      for (int l = 0; l < s->fr_n[i]; ++l) {
        (*fr)[(size_t)i * 8 + l] = s->fr_b[(size_t)i * s->fr_max + l];
        (*fr)[(size_t)i * 8 + 4 + l] = s->fr_a[(size_t)i * s->fr_max + l];
      }
  }
  return true;
}

// longest run of numerator taps from each entry's first nonzero one (mdband_kernel.hip keeps only
// those in LDS: the delay's leading zeros are skipped by pl_off / mz_off anyway)
static void compact_taps(const mpct_scenario* s, DevScenario& ds) {
  int pb = 1, mb = 1;
  for (size_t e = 0; e < s->pl_nb.size(); ++e) pb = std::max(pb, s->pl_nb[e] - s->pl_off[e]);
  for (size_t e = 0; e < s->mz_nb.size(); ++e) mb = std::max(mb, s->mz_nb[e] - s->mz_off[e]);
  ds.pl_maxbc = pb;
  ds.mz_maxbc = mb;
}

// the context of device want_dev (-1: the calling thread's current device), created and its
// tables uploaded on first use; makes that device current for the calling thread
static int build_ctx(mpct_scenario* s, int dev, DevCtx** out);

// occurrence j of device want_dev in one call (0: the primary context; j >= 1: extra[dev][j-1])
static int device_ctx(mpct_scenario* s, int want_dev, DevCtx** out, int occurrence = 0) {
  int dev = want_dev;
  if (dev < 0) {
    if (hipGetDevice(&dev) != hipSuccess) return fail(MPCT_EDEVICE, "hipGetDevice failed (no GPU?)");
  }
  int cnt = 0;
  if (hipGetDeviceCount(&cnt) != hipSuccess || cnt == 0) return fail(MPCT_EDEVICE, "no HIP device");
  if (dev >= cnt) return fail(MPCT_EINVAL, "device ordinal out of range");
  if (hipSetDevice(dev) != hipSuccess) return fail(MPCT_EDEVICE, "hipSetDevice failed");
  if ((int)s->ctx.size() < cnt) s->ctx.resize(cnt, nullptr);
  if ((int)s->extra.size() < cnt) s->extra.resize(cnt);
  DevCtx** slot = nullptr;
  if (occurrence == 0) {
    slot = &s->ctx[dev];
  } else {
    auto& ex = s->extra[dev];
    if ((int)ex.size() < occurrence) ex.resize(occurrence, nullptr);
    slot = &ex[occurrence - 1];
  }
  if (!*slot) {
    const int rc = build_ctx(s, dev, slot);
    if (rc) return rc;
  }
  *out = *slot;
  return MPCT_OK;
}

// the dispatch key's Gram tables (DevScenario::gram): for every horizon pair (N2, Nu) with
// nu Nu <= kGramM and every output o, G_o'G_o and G_o'1 of the forced-response matrix
// G_o(r, n Nu + l) = s_on(n1_o + r - l), r < N2 (MatG.m; zero where the step index is negative).
// They depend on the scenario alone, so the key forms H = sum_o q_o G_o'G_o + Lambda per candidate
// from them instead of re-correlating the step table in every workgroup.  Empty when the scenario
// has no step table, more than 4 outputs, or the tables would exceed kGramMaxBytes
static void gram_tables(const mpct_scenario* s, std::vector<double>& g) {
  g.clear();
  const int my = s->my, nu = s->nu, n2max = s->n2max, numax = s->numax, tlen = s->tlen;
  if (s->nmpc || s->mdband || my > 4 || nu < 1 || nu > kGramM || s->step.empty()) return;
  const size_t blk = (size_t)my * kGramOut;
  if ((long long)((size_t)n2max * numax * blk * 8) > kGramMaxBytes) return;
  g.assign((size_t)n2max * numax * blk, 0.0);
  for (int N2 = 1; N2 <= n2max; ++N2)
    for (int Nu = 1; Nu <= std::min(N2, numax) && nu * Nu <= kGramM; ++Nu) {
      const int M = nu * Nu;
      double* b = g.data() + ((size_t)(N2 - 1) * numax + (Nu - 1)) * blk;
      for (int o = 0; o < my; ++o) {
        double* go = b + (size_t)o * kGramOut;
        const int n1 = s->n1[o];
        const double* so = s->step.data() + (size_t)o * nu * tlen;
        for (int a = 0; a < M; ++a) {
          const int na = a / Nu, la = a - na * Nu;
          const double* sa = so + (size_t)na * tlen + n1 - la;  // sa[r] = s_o,na(n1 + r - la)
          double cs = 0.0;
          for (int r = std::max(la - n1, 0); r < N2; ++r) cs += sa[r];
          go[kGramM * kGramM + a] = cs;
          for (int bb = a; bb < M; ++bb) {
            const int nb = bb / Nu, lb = bb - nb * Nu;
            const double* sb = so + (size_t)nb * tlen + n1 - lb;
            double h = 0.0;
            for (int r = std::max(std::max(la, lb) - n1, 0); r < N2; ++r) h += sa[r] * sb[r];
            go[a * kGramM + bb] = h;
            go[bb * kGramM + a] = h;
          }
        }
      }
    }
}

// a new context on device dev (current): the scenario's tables uploaded, its own stream
static int build_ctx(mpct_scenario* s, int dev, DevCtx** out) {
  // pack all tables into one allocation, 256-B aligned pieces
  std::vector<char> blob;
  auto put = [&](const void* p, size_t bytes) -> size_t {
    size_t off = (blob.size() + 255) & ~(size_t)255;
    blob.resize(off + bytes);
    if (bytes) std::memcpy(blob.data() + off, p, bytes);
    return off;
  };
  size_t o_step = put(s->step.data(), s->step.size() * 8);
  size_t o_phi = put(s->phid.data(), s->phid.size() * 8);
  size_t o_n1 = put(s->n1.data(), s->n1.size() * 4);
  size_t o_yoff = put(s->yoff.data(), s->yoff.size() * 4);
  size_t o_nyhi = put(s->nyhi.data(), s->nyhi.size() * 4);
  size_t o_upoff = put(s->upoff.data(), s->upoff.size() * 4);
  size_t o_dum = put(s->dum.data(), s->dum.size() * 4);
  size_t o_plnb = put(s->pl_nb.data(), s->pl_nb.size() * 4);
  size_t o_plna = put(s->pl_na.data(), s->pl_na.size() * 4);
  size_t o_ploff = put(s->pl_off.data(), s->pl_off.size() * 4);
  size_t o_plb = put(s->pl_b.data(), s->pl_b.size() * 8);
  size_t o_pla = put(s->pl_a.data(), s->pl_a.size() * 8);
  size_t o_bnd = put(s->bnd.data(), s->bnd.size() * 8);
  size_t o_yref = put(s->yref.data(), s->yref.size() * 8);
  size_t o_mznb = put(s->mz_nb.data(), s->mz_nb.size() * 4);
  size_t o_mzna = put(s->mz_na.data(), s->mz_na.size() * 4);
  size_t o_mzoff = put(s->mz_off.data(), s->mz_off.size() * 4);
  size_t o_mzb = put(s->mz_b.data(), s->mz_b.size() * 8);
  size_t o_mza = put(s->mz_a.data(), s->mz_a.size() * 8);
  size_t o_frn = put(s->fr_n.data(), s->fr_n.size() * 4);
  size_t o_frb = put(s->fr_b.data(), s->fr_b.size() * 8);
  size_t o_fra = put(s->fr_a.data(), s->fr_a.size() * 8);
  size_t o_smd = put(s->step_md.data(), s->step_md.size() * 8);
  size_t o_obnd = put(s->obnd.data(), s->obnd.size() * 8);
  size_t o_wsc = put(s->wscale.data(), s->wscale.size() * 8);
  size_t o_xc = put(s->xc.data(), s->xc.size() * 4);
  size_t o_nm = put(s->nm.data(), s->nm.size() * 8);
  std::vector<double> gram;
  gram_tables(s, gram);
  size_t o_gram = put(gram.data(), gram.size() * 8);
  SmallTables smt;
  std::vector<double> sfr;
  const bool small = small_plant(s, &smt);
  const bool small_dtc = !small && dtc_small_plant(s, &smt, &sfr);
  size_t o_smc = put(smt.coef.data(), smt.coef.size() * 8);
  size_t o_smo = put(smt.hoff.data(), smt.hoff.size() * 4);
  size_t o_smh = put(smt.hc.data(), smt.hc.size() * 4);
  size_t o_smm = put(smt.hmask.data(), smt.hmask.size() * 4);
  size_t o_sma = put(smt.acol.data(), smt.acol.size() * 4);
  size_t o_sfr = put(sfr.data(), sfr.size() * 8);
  void* dp = nullptr;
  if (hipMalloc(&dp, blob.size()) != hipSuccess) return fail(MPCT_ENOMEM, "hipMalloc(tables) failed");
  if (hipMemcpy(dp, blob.data(), blob.size(), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(dp);
    return fail(MPCT_EDEVICE, "hipMemcpy(tables) failed");
  }
  DevCtx* cx = new DevCtx();
  if (hipStreamCreateWithFlags(&cx->stream, hipStreamNonBlocking) != hipSuccess) {
    (void)hipFree(dp);
    delete cx;
    return fail(MPCT_EDEVICE, "hipStreamCreate failed");
  }
  char* b = static_cast<char*>(dp);
  DevScenario& ds = cx->ds;
  ds.my = s->my;
  ds.nu = s->nu;
  ds.nd = s->nd + s->nq;  // ring-fed plant inputs (their signals are v's rows)
  ds.nin = s->npin;       // plant input columns
  ds.nit = s->nit;
  ds.n2max = s->n2max;
  ds.numax = s->numax;
  ds.tlen = s->tlen;
  ds.nx = s->nx;
  ds.nyh = s->nyh;
  ds.nup = s->nup;
  ds.wsq = s->wsq;
  ds.ink0 = s->ink0;
  ds.ne = s->ne;
  ds.pl_maxb = s->pl_maxb;
  ds.pl_maxa = s->pl_maxa;
  ds.regpath = regpath(s);
  ds.small = small ? 1 : 0;
  ds.sm_ke = smt.ke;
  ds.sm_coef = reinterpret_cast<const double*>(b + o_smc);
  ds.sm_hoff = reinterpret_cast<const int*>(b + o_smo);
  ds.sm_hc = reinterpret_cast<const int*>(b + o_smh);
  ds.sm_hmask = reinterpret_cast<const int*>(b + o_smm);
  ds.sm_acol = reinterpret_cast<const int*>(b + o_sma);
  ds.small_dtc = small_dtc ? 1 : 0;
  ds.sm_fr = reinterpret_cast<const double*>(b + o_sfr);
  ds.step = reinterpret_cast<const double*>(b + o_step);
  ds.gram = gram.empty() ? nullptr : reinterpret_cast<const double*>(b + o_gram);
  ds.phi = reinterpret_cast<const double*>(b + o_phi);
  ds.n1 = reinterpret_cast<const int*>(b + o_n1);
  ds.yoff = reinterpret_cast<const int*>(b + o_yoff);
  ds.nyhi = reinterpret_cast<const int*>(b + o_nyhi);
  ds.upoff = reinterpret_cast<const int*>(b + o_upoff);
  ds.dum = reinterpret_cast<const int*>(b + o_dum);
  ds.pl_nb = reinterpret_cast<const int*>(b + o_plnb);
  ds.pl_na = reinterpret_cast<const int*>(b + o_plna);
  ds.pl_off = reinterpret_cast<const int*>(b + o_ploff);
  ds.pl_b = reinterpret_cast<const double*>(b + o_plb);
  ds.pl_a = reinterpret_cast<const double*>(b + o_pla);
  ds.bnd = reinterpret_cast<const double*>(b + o_bnd);
  ds.yref = reinterpret_cast<const double*>(b + o_yref);
  ds.dtc = s->dtc;
  ds.nvar = s->nvar;
  ds.mz_maxb = s->mz_maxb;
  ds.mz_maxa = s->mz_maxa;
  ds.fr_max = s->fr_max;
  ds.mz_nb = reinterpret_cast<const int*>(b + o_mznb);
  ds.mz_na = reinterpret_cast<const int*>(b + o_mzna);
  ds.mz_off = reinterpret_cast<const int*>(b + o_mzoff);
  ds.mz_b = reinterpret_cast<const double*>(b + o_mzb);
  ds.mz_a = reinterpret_cast<const double*>(b + o_mza);
  ds.fr_n = reinterpret_cast<const int*>(b + o_frn);
  ds.fr_b = reinterpret_cast<const double*>(b + o_frb);
  ds.fr_a = reinterpret_cast<const double*>(b + o_fra);
  ds.mdband = s->mdband;
  ds.rho = s->rho;
  ds.step_md = reinterpret_cast<const double*>(b + o_smd);
  ds.obnd = reinterpret_cast<const double*>(b + o_obnd);
  ds.wscale = reinterpret_cast<const double*>(b + o_wsc);
  compact_taps(s, ds);
  ds.nmpc = s->nmpc;
  ds.nsub = s->nsub;
  ds.sqp_max = s->sqp_max;
  ds.ts = s->ts;
  ds.sqp_tol = s->sqp_tol;
  ds.xc = reinterpret_cast<const int*>(b + o_xc);
  ds.nm = reinterpret_cast<const double*>(b + o_nm);
  cx->dtab = dp;
  cx->dev = dev;
  if (!cx->fan.init(dev)) cx->fan.release();  // class launches over streams; no fan: one stream, still correct
  *out = cx;
  return MPCT_OK;
}

static DevOpts make_opts(const mpct_opts* o) {
  DevOpts d{};
  d.open_loop = o ? o->open_loop : 0;
  d.want_traj = o ? o->want_traj : 0;
  d.max_qp_iter = o ? o->max_qp_iter : 0;
  d.feas_tol = (o && o->feas_tol > 0) ? o->feas_tol : 1e-10;
#ifdef MPCT_DIAG
  const char* e = getenv("MPCT_DIAG_SKIP_WARM_DROP");
  d.diag = (e && *e && atoi(e) != 0) ? kDiagSkipWarmDrop : 0;
#endif
  return d;
}

static int check_args(mpct_scenario* s, int64_t C, int32_t nref, const int32_t* N2, const int32_t* Nu,
                      const double* delta, const double* lambda, const double* r, const double* v) {
  if (!s) return fail(MPCT_EINVAL, "null scenario");
  if (C < 0 || nref < 1) return fail(MPCT_EINVAL, "C < 0 or nref < 1");
  if (C * (int64_t)nref > 0x7fffffffLL) return fail(MPCT_ERANGE, "too many simulations in one call");
  if (C > 0 && (!N2 || !Nu || !delta || !lambda || !r)) return fail(MPCT_EINVAL, "null input pointer");
  if (s->nd + s->nq > 0 && !v) return fail(MPCT_EINVAL, "v required when nd + nq > 0");
  return MPCT_OK;
}

// enqueue one batch with device pointers on `stream` (ctx's device is current)
static int launch_batch(mpct_scenario* s, DevCtx* cx, int64_t C, const int32_t* N2, const int32_t* Nu,
                        const double* delta, const double* lambda, int32_t nref, const double* r, const double* v,
                        const mpct_opts* opts, const mpct_result* out, hipStream_t stream) {
  if (C == 0) return MPCT_OK;
  DevOpts dop = make_opts(opts);
  DevResult dr{out->J1, out->j21, out->j22, out->Jnu, out->status, out->qp_iters,
                out->y, out->u, out->ys, out->uopt, nullptr};
#ifdef MPCT_PROFILE
  // diagnostic build: per-simulation section cycle sums, summarised on stderr
  const long long S = C * nref;
  unsigned long long* dprof = nullptr;
  (void)hipMalloc(&dprof, sizeof(unsigned long long) * S * PROF_N);
  dr.prof = dprof;
#endif
#ifdef MPCT_TIMELINE
  // diagnostic build: [slot][t0, t1, HW_ID << 32 | XCC_ID, sim] -> $MPCT_TIMELINE_OUT
  const long long S = C * nref;
  unsigned long long* dprof = nullptr;
  (void)hipMalloc(&dprof, sizeof(unsigned long long) * S * 4);
  (void)hipMemset(dprof, 0, sizeof(unsigned long long) * S * 4);
  dr.prof = dprof;
#endif
  std::string err;
  int rc;
  if (s->nmpc)
    rc = launch_nmpc(cx->ds, C, nref, N2, Nu, delta, lambda, r, dop, dr, stream, &cx->fan, &cx->order, &err);
  else if (s->mdband)
    rc = launch_mdband(cx->ds, C, nref, N2, Nu, delta, lambda, r, v, dop, dr, stream, &cx->fan, &err);
  else
    rc = launch_closed_loop(cx->ds, C, nref, N2, Nu, delta, lambda, r, v, dop, dr, s->nu * s->numax, &cx->order, &cx->fan,
                            stream, &err);
  if (rc) return fail(rc, err);
#ifdef MPCT_TIMELINE
  {
    std::vector<unsigned long long> hp(S * 4);
    (void)hipStreamSynchronize(stream);
    (void)hipMemcpy(hp.data(), dprof, sizeof(unsigned long long) * S * 4, hipMemcpyDeviceToHost);
    (void)hipFree(dprof);
    const char* path = getenv("MPCT_TIMELINE_OUT");
    if (path) {
      FILE* f = fopen(path, "wb");
      if (f) {
        fwrite(hp.data(), sizeof(unsigned long long), hp.size(), f);
        fclose(f);
      }
    }
  }
#endif
#ifdef MPCT_PROFILE
  {
    std::vector<unsigned long long> hp(S * PROF_N);
    (void)hipStreamSynchronize(stream);
    (void)hipMemcpy(hp.data(), dprof, sizeof(unsigned long long) * S * PROF_N, hipMemcpyDeviceToHost);
    (void)hipFree(dprof);
    // low 40 bits: cycles, high 24: executions of the section (wave_ops.h PSTAMP, kProfCountShift)
    constexpr int kProfCountShift = 40;
    const unsigned long long cmask = (1ull << kProfCountShift) - 1;
    double sum[PROF_N] = {0}, mx[PROF_N] = {0}, cnt[PROF_N] = {0};
    for (long long i = 0; i < S; ++i)
      for (int k = 0; k < PROF_N; ++k) {
        sum[k] += (double)(hp[i * PROF_N + k] & cmask);
        cnt[k] += (double)(hp[i * PROF_N + k] >> kProfCountShift);
        mx[k] = std::max(mx[k], (double)(hp[i * PROF_N + k] & cmask));
      }
    if (const char* po = getenv("MPCT_PROF_OUT")) {  // per simulation, raw (tools/latency_model.py)
      FILE* f = fopen(po, "wb");
      if (f) {
        fwrite(hp.data(), sizeof(unsigned long long), hp.size(), f);
        fclose(f);
      }
    }
    const char* gpc_nm[PROF_N] = {"prologue", "plant", "y_update", "unconstrained", "qp(rest)", "u_update",
                                  "open_loop", "qp.check", "qp.d+z", "qp.r+t1", "qp.add", "qp.drop", "qp.warm",
                                  "qp.rotations", "qp.w.entry", "qp.w.rebuild", "qp.w.gather", "qp.w.solve",
                                  "qp.w.drop", "qp.w.rotations", "qp.w.readds"};
    const char* nmpc_nm[PROF_N] = {"full_pass", "rinv+step", "qp", "anderson_pass", "ls_full_pass", "ls_trials",
                                   "plant_rk4", "other", "n.passes", "n.points", "n.used", "n.rows", "-", "-", "-",
                                   "-", "-", "-", "-", "-", "-"};
    const char** nm = s->nmpc ? nmpc_nm : gpc_nm;
    fprintf(stderr, "[mpct profile] mean / max cycles and mean executions per simulation over %lld sims\n", S);
    for (int k = 0; k < PROF_N; ++k)
      fprintf(stderr, "  %-14s %12.0f %12.0f %10.1f\n", nm[k], sum[k] / (double)S, mx[k], cnt[k] / (double)S);
  }
#endif
  return MPCT_OK;
}

extern "C" int32_t mpct_eval_batch_device(mpct_scenario* s, int64_t C, const int32_t* N2, const int32_t* Nu,
                                          const double* delta, const double* lambda, int32_t nref,
                                          const double* r, const double* v, const mpct_opts* opts,
                                          mpct_result* out, void* stream) {
  int rc = check_args(s, C, nref, N2, Nu, delta, lambda, r, v);
  if (rc) return rc;
  if (!out) return fail(MPCT_EINVAL, "null result");
  if (s->dtc && opts && opts->open_loop) return fail(MPCT_EINVAL, "DTC mode has no open-loop prediction");
  DevCtx* cx = nullptr;
  rc = device_ctx(s, opts ? opts->device : -1, &cx);
  if (rc) return rc;
  return launch_batch(s, cx, C, N2, Nu, delta, lambda, nref, r, v, opts, out, static_cast<hipStream_t>(stream));
}

extern "C" int32_t mpct_rank_device(const double* costs, int64_t C, int32_t k, const double* w, int32_t* perm,
                                    void* stream) {
  if (C < 0 || C > 2147483647LL) return fail(MPCT_ERANGE, "C out of range for the ranking sort");
  if (k < 1) return fail(MPCT_EINVAL, "k < 1");
  if (C > 0 && (!costs || !w || !perm)) return fail(MPCT_EINVAL, "null pointer");
  std::string err;
  const int rc = rank_device(costs, C, k, w, perm, static_cast<hipStream_t>(stream), &err);
  if (rc) return fail(rc == -2 ? MPCT_ENOMEM : MPCT_EDEVICE, err);
  return MPCT_OK;
}

// host buffers in, host buffers out, on the context's own stream: H2D of the candidates and
// signals, the launch, D2H of the results, then a wait on that stream only
static int eval_host(mpct_scenario* s, DevCtx* cx, int64_t C, const int32_t* N2, const int32_t* Nu,
                     const double* delta, const double* lambda, int32_t nref, const double* r, const double* v,
                     const mpct_opts* opts, mpct_result* out) {
  if (hipSetDevice(cx->dev) != hipSuccess) return fail(MPCT_EDEVICE, "hipSetDevice failed");
  if (C == 0) return MPCT_OK;
  const int my = s->my, nu = s->nu, nd = s->nd, nit = s->nit;
  const int64_t S = C * nref;
  const bool traj = opts && opts->want_traj;
  const bool ol = opts && opts->open_loop;
  hipStream_t st = cx->stream;
  // device scratch layout
  size_t off = 0;
  auto slot = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  };
  size_t o_N2 = slot(C * 4), o_Nu = slot(C * 4), o_d = slot(C * my * 8), o_l = slot(C * nu * 8);
  size_t o_J1 = slot(S * my * 8), o_j21 = slot(S * my * 8), o_j22 = slot(S * my * 8), o_Jnu = slot(S * nu * 8);
  size_t o_st = slot(S * 4), o_it = slot(S * 8);
  size_t o_y = traj ? slot(S * my * nit * 8) : 0, o_u = traj ? slot(S * nu * nit * 8) : 0;
  size_t o_ys = (traj && ol) ? slot(S * my * nit * 8) : 0, o_uo = (traj && ol) ? slot(S * nu * nit * 8) : 0;
  if (off > cx->dscratch_bytes) {
    if (cx->dscratch) {
      (void)hipStreamSynchronize(st);
      (void)hipFree(cx->dscratch);
    }
    cx->dscratch = nullptr;
    cx->dscratch_bytes = 0;
    if (hipMalloc(&cx->dscratch, off) != hipSuccess) return fail(MPCT_ENOMEM, "hipMalloc(scratch) failed");
    cx->dscratch_bytes = off;
  }
  char* b = static_cast<char*>(cx->dscratch);
  auto h2d = [&](void* dst, const void* p, size_t bytes) {
    return bytes == 0 || hipMemcpyAsync(dst, p, bytes, hipMemcpyHostToDevice, st) == hipSuccess;
  };
  // signals r | v: uploaded only when they differ from what the context's signal buffer holds
  const size_t rb = (size_t)nref * my * nit * 8, vb = (size_t)nref * (nd + s->nq) * nit * 8;
  const bool same_sig = cx->sig_host.size() == rb + vb && std::memcmp(cx->sig_host.data(), r, rb) == 0 &&
                        (vb == 0 || std::memcmp(cx->sig_host.data() + rb, v, vb) == 0);
  if (!same_sig) {
    if (rb + vb > cx->dsig_bytes) {
      if (cx->dsig) {
        (void)hipStreamSynchronize(st);
        (void)hipFree(cx->dsig);
      }
      cx->dsig = nullptr;
      cx->dsig_bytes = 0;
      cx->sig_host.clear();
      if (hipMalloc(&cx->dsig, rb + vb) != hipSuccess) return fail(MPCT_ENOMEM, "hipMalloc(signals) failed");
      cx->dsig_bytes = rb + vb;
    }
    cx->sig_host.assign(reinterpret_cast<const char*>(r), reinterpret_cast<const char*>(r) + rb);
    if (vb) cx->sig_host.insert(cx->sig_host.end(), reinterpret_cast<const char*>(v), reinterpret_cast<const char*>(v) + vb);
  }
  char* sg = static_cast<char*>(cx->dsig);
  // the signals are copied from the context's own host copy (the caller's buffers may change
  // after the call returns; an earlier launch reading dsig is ordered before this copy on st)
  if (!h2d(b + o_N2, N2, C * 4) || !h2d(b + o_Nu, Nu, C * 4) || !h2d(b + o_d, delta, C * my * 8) ||
      !h2d(b + o_l, lambda, C * nu * 8) || (!same_sig && !h2d(sg, cx->sig_host.data(), rb + vb))) {
    // copies enqueued before the failing one may still read the caller's buffers
    (void)hipStreamSynchronize(st);
    cx->sig_host.clear();
    return fail(MPCT_EDEVICE, "hipMemcpyAsync(inputs) failed");
  }
  mpct_result dres{};
  dres.J1 = reinterpret_cast<double*>(b + o_J1);
  dres.j21 = reinterpret_cast<double*>(b + o_j21);
  dres.j22 = reinterpret_cast<double*>(b + o_j22);
  dres.Jnu = reinterpret_cast<double*>(b + o_Jnu);
  dres.status = reinterpret_cast<int32_t*>(b + o_st);
  dres.qp_iters = reinterpret_cast<int64_t*>(b + o_it);
  if (traj) {
    dres.y = reinterpret_cast<double*>(b + o_y);
    dres.u = reinterpret_cast<double*>(b + o_u);
    if (ol) {
      dres.ys = reinterpret_cast<double*>(b + o_ys);
      dres.uopt = reinterpret_cast<double*>(b + o_uo);
    }
  }
  int rc = launch_batch(s, cx, C, reinterpret_cast<const int32_t*>(b + o_N2), reinterpret_cast<const int32_t*>(b + o_Nu),
                        reinterpret_cast<const double*>(b + o_d), reinterpret_cast<const double*>(b + o_l), nref,
                        reinterpret_cast<const double*>(sg),
                        nd + s->nq > 0 ? reinterpret_cast<const double*>(sg + rb) : nullptr, opts, &dres, st);
  if (rc) {
    (void)hipStreamSynchronize(st);
    return rc;
  }
  auto d2h = [&](void* dst, const void* src, size_t bytes) {
    return !dst || bytes == 0 || hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st) == hipSuccess;
  };
  bool ok = d2h(out->J1, dres.J1, S * my * 8) && d2h(out->j21, dres.j21, S * my * 8) &&
            d2h(out->j22, dres.j22, S * my * 8) && d2h(out->Jnu, dres.Jnu, S * nu * 8) &&
            d2h(out->status, dres.status, S * 4) && d2h(out->qp_iters, dres.qp_iters, S * 8);
  if (traj) {
    ok = ok && d2h(out->y, dres.y, S * my * nit * 8) && d2h(out->u, dres.u, S * nu * nit * 8);
    if (ol) ok = ok && d2h(out->ys, dres.ys, S * my * nit * 8) && d2h(out->uopt, dres.uopt, S * nu * nit * 8);
  }
  const hipError_t se = hipStreamSynchronize(st);
  if (se != hipSuccess) return fail(MPCT_EDEVICE, std::string("kernel execution failed: ") + hipGetErrorString(se));
  if (!ok) return fail(MPCT_EDEVICE, "hipMemcpyAsync(results) failed");
  return MPCT_OK;
}

extern "C" int32_t mpct_eval_batch(mpct_scenario* s, int64_t C, const int32_t* N2, const int32_t* Nu,
                                   const double* delta, const double* lambda, int32_t nref, const double* r,
                                   const double* v, const mpct_opts* opts, mpct_result* out) {
  int rc = check_args(s, C, nref, N2, Nu, delta, lambda, r, v);
  if (rc) return rc;
  if (!out) return fail(MPCT_EINVAL, "null result");
  if (s->dtc && opts && opts->open_loop) return fail(MPCT_EINVAL, "DTC mode has no open-loop prediction");
  DevCtx* cx = nullptr;
  rc = device_ctx(s, opts ? opts->device : -1, &cx);
  if (rc) return rc;
  return eval_host(s, cx, C, N2, Nu, delta, lambda, nref, r, v, opts, out);
}

extern "C" int64_t mpct_shard_candidates(int64_t C, int32_t ndev, int32_t k, int64_t* idx, int64_t cap) {
  if (C < 0 || ndev < 1 || k < 0 || k >= ndev) return fail(MPCT_EINVAL, "bad shard arguments");
  const int64_t n = C > k ? (C - k + ndev - 1) / ndev : 0;
  if (idx)
    for (int64_t j = 0; j < std::min(n, cap); ++j) idx[j] = k + j * ndev;
  return n;
}

// copy `width` elements per simulation between the caller's order and a shard's packed order:
// simulation s = c*nref + q of candidate c = k + j*ndev <-> packed row j*nref + q
template <class T>
static void strided_copy(T* caller, T* packed, int64_t n, int32_t ndev, int32_t k, int32_t nref, int64_t width,
                         bool to_caller) {
  if (!caller || !packed) return;
  for (int64_t j = 0; j < n; ++j) {
    T* a = caller + (k + j * ndev) * (int64_t)nref * width;
    T* b = packed + j * (int64_t)nref * width;
    const size_t bytes = sizeof(T) * (size_t)nref * (size_t)width;
    if (to_caller)
      std::memcpy(a, b, bytes);
    else
      std::memcpy(b, a, bytes);
  }
}

extern "C" int32_t mpct_eval_batch_multi(mpct_scenario* s, int32_t ndev, const int32_t* devices, int64_t C,
                                         const int32_t* N2, const int32_t* Nu, const double* delta,
                                         const double* lambda, int32_t nref, const double* r, const double* v,
                                         const mpct_opts* opts, mpct_result* out) {
  int rc = check_args(s, C, nref, N2, Nu, delta, lambda, r, v);
  if (rc) return rc;
  if (!out) return fail(MPCT_EINVAL, "null result");
  if (ndev < 1 || ndev > 64 || !devices) return fail(MPCT_EINVAL, "ndev must be 1..64 with a device list");
  if (s->dtc && opts && opts->open_loop) return fail(MPCT_EINVAL, "DTC mode has no open-loop prediction");
  int cur = -1, cnt = 0;
  if (hipGetDevice(&cur) != hipSuccess || hipGetDeviceCount(&cnt) != hipSuccess || cnt == 0)
    return fail(MPCT_EDEVICE, "hipGetDevice failed (no GPU?)");
  // every ordinal is checked before any context exists or any device is made current
  for (int k = 0; k < ndev; ++k)
    if (devices[k] < 0 || devices[k] >= cnt) return fail(MPCT_EINVAL, "device ordinal out of range");
  // contexts (table uploads) serially on this thread, before any worker starts; a device listed
  // again gets a further context of its own
  std::vector<DevCtx*> cxs(ndev, nullptr);
  for (int k = 0; k < ndev; ++k) {
    int occ = 0;
    for (int j = 0; j < k; ++j) occ += devices[j] == devices[k];
    rc = device_ctx(s, devices[k], &cxs[k], occ);
    if (rc) {
      (void)hipSetDevice(cur);
      return rc;
    }
  }
  const int my = s->my, nu = s->nu, nit = s->nit;
  std::vector<int> rcs(ndev, MPCT_OK);
  std::vector<std::string> errs(ndev);
  auto shard = [&](int k) {
    const int64_t n = mpct_shard_candidates(C, ndev, k, nullptr, 0);
    if (n <= 0) {
      rcs[k] = hipSetDevice(cxs[k]->dev) == hipSuccess ? MPCT_OK : MPCT_EDEVICE;
      return;
    }
    if (ndev == 1) {  // the identity split: no gather / scatter
      rcs[k] = eval_host(s, cxs[k], C, N2, Nu, delta, lambda, nref, r, v, opts, out);
      if (rcs[k]) errs[k] = g_err;
      return;
    }
    // gather this slot's candidates (k, k+ndev, ...) and give it packed result buffers
    std::vector<int32_t> n2(n), nuv(n);
    std::vector<double> dl((size_t)n * my), lm((size_t)n * nu);
    strided_copy(const_cast<int32_t*>(N2), n2.data(), n, ndev, k, 1, 1, false);
    strided_copy(const_cast<int32_t*>(Nu), nuv.data(), n, ndev, k, 1, 1, false);
    strided_copy(const_cast<double*>(delta), dl.data(), n, ndev, k, 1, my, false);
    strided_copy(const_cast<double*>(lambda), lm.data(), n, ndev, k, 1, nu, false);
    const int64_t S = n * nref;
    auto buf = [&](const void* want, int64_t w) { return want ? std::vector<double>((size_t)(S * w)) : std::vector<double>(); };
    std::vector<double> J1 = buf(out->J1, my), j21 = buf(out->j21, my), j22 = buf(out->j22, my), Jnu = buf(out->Jnu, nu);
    std::vector<double> y = buf(out->y, (int64_t)my * nit), u = buf(out->u, (int64_t)nu * nit);
    std::vector<double> ys = buf(out->ys, (int64_t)my * nit), uo = buf(out->uopt, (int64_t)nu * nit);
    std::vector<int32_t> stv(out->status ? (size_t)S : 0);
    std::vector<int64_t> itv(out->qp_iters ? (size_t)S : 0);
    auto p = [](std::vector<double>& x) { return x.empty() ? nullptr : x.data(); };
    mpct_result o{};
    o.J1 = p(J1);
    o.j21 = p(j21);
    o.j22 = p(j22);
    o.Jnu = p(Jnu);
    o.status = stv.empty() ? nullptr : stv.data();
    o.qp_iters = itv.empty() ? nullptr : itv.data();
    o.y = p(y);
    o.u = p(u);
    o.ys = p(ys);
    o.uopt = p(uo);
    rcs[k] = eval_host(s, cxs[k], n, n2.data(), nuv.data(), dl.data(), lm.data(), nref, r, v, opts, &o);
    if (rcs[k]) {
      errs[k] = g_err;  // g_err is thread-local: carry it to the caller
      return;
    }
    // scatter into the caller's order (slots write disjoint candidates)
    strided_copy(out->J1, o.J1, n, ndev, k, nref, my, true);
    strided_copy(out->j21, o.j21, n, ndev, k, nref, my, true);
    strided_copy(out->j22, o.j22, n, ndev, k, nref, my, true);
    strided_copy(out->Jnu, o.Jnu, n, ndev, k, nref, nu, true);
    strided_copy(out->status, o.status, n, ndev, k, nref, 1, true);
    strided_copy(out->qp_iters, o.qp_iters, n, ndev, k, nref, 1, true);
    strided_copy(out->y, o.y, n, ndev, k, nref, (int64_t)my * nit, true);
    strided_copy(out->u, o.u, n, ndev, k, nref, (int64_t)nu * nit, true);
    strided_copy(out->ys, o.ys, n, ndev, k, nref, (int64_t)my * nit, true);
    strided_copy(out->uopt, o.uopt, n, ndev, k, nref, (int64_t)nu * nit, true);
  };
  if (ndev == 1) {
    shard(0);
  } else {
    std::vector<std::thread> th;
    for (int k = 1; k < ndev; ++k) th.emplace_back(shard, k);
    shard(0);
    for (auto& t : th) t.join();
  }
  (void)hipSetDevice(cur);
  for (int k = 0; k < ndev; ++k)
    if (rcs[k]) return fail(rcs[k], "device " + std::to_string(devices[k]) + ": " + errs[k]);
  return MPCT_OK;
}

extern "C" int32_t mpct_kernel_instance(const mpct_scenario* s, const mpct_opts* opts, char* buf, int32_t cap) {
  if (!s) return fail(MPCT_EINVAL, "null scenario");
  std::string nm;
  const bool ext = opts && (opts->open_loop || opts->want_traj);
  if (s->nmpc)
    nm = "nmpc_closed_loop_kernel (QP-size x LDS-tier class launches)";
  else if (s->mdband)
    nm = "mdband_closed_loop_kernel (QP-size x LDS-tier class launches)";
  else {
    DevScenario ds{};  // the fields the kernel choice reads
    ds.my = s->my;
    ds.nu = s->nu;
    ds.nd = s->nd + s->nq;
    ds.nin = s->npin;
    ds.nx = s->nx;
    ds.dtc = s->dtc;
    ds.regpath = regpath(s);
    ds.small = small_plant(s) ? 1 : 0;
    ds.small_dtc = !ds.small && dtc_small_plant(s) ? 1 : 0;
    nm = closed_loop_instance(ds, s->nu * s->numax, ext);
  }
  if (buf && cap > 0) {
    const size_t n = std::min<size_t>(nm.size(), (size_t)cap - 1);
    std::memcpy(buf, nm.data(), n);
    buf[n] = '\0';
  }
  return (int32_t)nm.size();
}

static int64_t lds_bytes_ext(const mpct_scenario* s, int32_t N2, int32_t Nu, bool ext) {
  if (!s) return fail(MPCT_EINVAL, "null scenario");
  if (s->nmpc) return nmpc_lds_bytes(s->nu * Nu, N2);
  DevScenario ds{};
  ds.my = s->my;
  ds.nu = s->nu;
  ds.nin = s->npin;
  ds.nx = s->nx;
  ds.ne = s->ne;
  ds.tlen = s->tlen;
  ds.pl_maxb = s->pl_maxb;
  ds.pl_maxa = s->pl_maxa;
  ds.dtc = s->dtc;
  ds.mz_maxb = s->mz_maxb;
  ds.mz_maxa = s->mz_maxa;
  ds.fr_max = s->fr_max;
  ds.mdband = s->mdband;
  ds.regpath = regpath(s);
  {
    SmallTables smt;
    ds.small = small_plant(s, &smt) ? 1 : 0;
    ds.small_dtc = !ds.small && dtc_small_plant(s, &smt) ? 1 : 0;
    ds.sm_ke = smt.ke;
  }
  ds.my = s->my;
  ds.nd = s->nd;
  compact_taps(s, ds);
  return s->mdband ? mdband_lds_bytes(ds, N2, Nu, ext ? 2 : 1) : lds_bytes_for(ds, N2, Nu, ext);
}

extern "C" int64_t mpct_lds_bytes(const mpct_scenario* s, int32_t N2, int32_t Nu) {
  return lds_bytes_ext(s, N2, Nu, true);
}

extern "C" int64_t mpct_lds_bytes_opts(const mpct_scenario* s, const mpct_opts* opts, int32_t N2, int32_t Nu) {
  return lds_bytes_ext(s, N2, Nu, opts && (opts->open_loop || opts->want_traj));
}
