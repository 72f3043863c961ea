/*
 * mpct.h — C ABI of the MI355X batched closed-loop GPC scoring engine (libmpct.so).
 *
 * Drop-in boundary for the reference's per-candidate closed-loop seam
 *   function [y,u,t,ys,uopt] = closedloop_toolbox(mpc_toolbox,r,v,N,Nu,delta,lambda,nit)
 *   (MPC-Tuning/MPC_Tuning/closedloop_toolbox.m:1), called once per candidate (and once per
 *   output for square plants) by VNS2.m:153,168 and GAM_fun.m:81.
 * Here one call scores a whole BATCH of candidates (N2, Nu, delta, lambda) on the GPU.  A
 * MATLAB host binds it with loadlibrary('libmpct','mpct.h') / calllib, or through the MEX
 * shim in INTEGRATION.md; the Python host mirror (mpct/) binds it with ctypes.
 *
 * Conventions
 *   - plain C types only; every matrix is row-major double; "row signals" are [row][t].
 *   - the caller owns every input/output buffer; the library owns the scenario (host tables
 *     and their device copies) until mpct_scenario_destroy.
 *   - negative return codes are argument / shape / device errors (message in
 *     mpct_last_error(), thread-local); per-candidate numerical trouble never fails the call:
 *     it is reported in mpct_result.status[] with NaN costs (the reference swallows such
 *     errors with fprintf and continues: VNS2.m:161-163, GAM_fun.m:82-84).
 *   - threading: one scenario per host thread, or external synchronisation.  All device work
 *     of a call is complete when mpct_eval_batch returns.  A scenario keeps one context per GPU
 *     it has been evaluated on (table copies, sort buffers, a library-owned stream); the
 *     host-pointer entries synchronise that stream only, never the whole device.
 */
#ifndef MPCT_H
#define MPCT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPCT_ABI_VERSION 7 /* 7: every simulation slot is prefilled with MPCT_ST_NOT_RUN and NaN costs
                              before the class launches (a slot no launch simulates stays so).
                              6: strided multi-device shards (mpct_shard_candidates replaces the
                              contiguous mpct_shard_range), a device may appear more than once in
                              mpct_eval_batch_multi's list; dims table carries nit, nq.
                              5: one scenario on several GPUs of one process (mpct_eval_batch_multi),
                              kernel-instance query; the host-pointer entries wait on
                              their own stream only.  4: nonlinear MPC scenarios (mpct_nmpc_scenario_create); 3: MD feed-forward +
                              soft output bands; 2: DTC-GPC predictor + plant-only disturbances + plant
                              variants; v1..v3 descriptors accepted */

/* error codes */
#define MPCT_OK 0
#define MPCT_EINVAL (-1)   /* bad argument / shape                                  */
#define MPCT_ENOMEM (-2)   /* host or device allocation failed                      */
#define MPCT_EDEVICE (-3)  /* HIP runtime error (no device, launch failure, ...)    */
#define MPCT_ERANGE (-4)   /* a size exceeds what the compiled kernels support       */

/* per-simulation status bits (mpct_result.status) */
#define MPCT_ST_OK 0
#define MPCT_ST_QP_MAXITER 1   /* active-set iteration cap hit at some step          */
#define MPCT_ST_QP_INFEAS 2    /* QP infeasible at some step (dual unbounded)        */
#define MPCT_ST_NONFINITE 4    /* a non-finite value appeared in the state           */
#define MPCT_ST_SKIPPED 8      /* padding / sentinel candidate (N2 <= 0)             */
#define MPCT_ST_BADHORIZON 16  /* N2/Nu outside the scenario's range or Nu > N2      */
#define MPCT_ST_SQP_MAXITER 32 /* NMPC: a Gauss-Newton SQP hit sqp_max at some step  */
#define MPCT_ST_BOUNDS 64      /* NMPC: the closed loop left the state/OV bounds     */
#define MPCT_ST_NOT_RUN 128    /* no kernel launch simulated this slot (an internal
                                  dispatch fault; costs NaN).  Every slot is prefilled
                                  with it before the class launches, which overwrite it */

/* One SISO discrete transfer function  y = z^-delay * num(z)/den(z) u  in the form tfdata(.,'v')
 * returns it (descending powers of z, numerator padded to the denominator's length, den[0]=1)
 * — the representation descompMPC.m:19 reads.  len = number of coefficients of each. */
typedef struct mpct_dtf {
  int32_t len;
  const double* num;
  const double* den;
  int32_t delay;
} mpct_dtf;

/* Scenario: everything that does not depend on the candidate.
 *   plant[i*(nu+nd)+j]  : simulated plant entries (the toolbox's sim simulates the model
 *                         itself unless options.Model is set: closedloop_toolbox.m:50)
 *   model[i*(nu+nd)+j]  : prediction model entries, used for the MatG step responses
 *                         (MatG.m:51 step(Ps(i,j),...))
 *   carima_A / carima_B : the CARIMA form after descompMPC + BA_MIMO (DTC_GPC_WW.m:79):
 *                         A_i (na[i]+1 coeffs, z^-1 powers, A_i[0]=1) concatenated over i;
 *                         B_ij (nb[i*(nu+nd)+j]+1 coeffs) concatenated row-major over (i,j);
 *                         dp[i*(nu+nd)+j] the descompMPC delays.  abi >= 5, dtc == 0, mdband == 0:
 *                         na, carima_A, nb, carima_B and dp may ALL be NULL; the library then
 *                         derives them from `model` (descompMPC.m:19-43, then the exact LCM of
 *                         each row's distinct denominators: the toolbox-equivalent CARIMA form).
 *   n1[i]               : first predicted step of output i: 1 = toolbox window t+1..t+N2
 *                         (PredictionHorizon semantics), dmin_i+1 = GPC window (MatG.m:64,
 *                         diophantine.m:44 N1 = d+1)
 *   weights_squared     : 1 = toolbox cost (Weights enter squared), 0 = DTC_GPC_WW.m:67-76
 *   du_min..u_max[nu]   : MV rate / amplitude bounds (already scaled, MPCTuning.m:170-178);
 *                         +-INFINITY disables a bound
 *   n2_max, nu_max      : largest horizons any candidate of this scenario may use
 *   nit                 : closed-loop length (Par.nit);  vns_ink: VNS2.m:43 inK (1-based)
 *   yref[my*nit]        : GAM/VNS reference trajectory Par.Yref (MPCTuning.m:188,320)      */
typedef struct mpct_scenario_desc {
  int32_t abi_version; /* = MPCT_ABI_VERSION */
  int32_t my, nu, nd;
  int32_t nit;
  int32_t n2_max, nu_max;
  int32_t weights_squared;
  int32_t vns_ink;
  const int32_t* n1;
  const mpct_dtf* plant;
  const mpct_dtf* model;
  const int32_t* na;
  const double* carima_A;
  const int32_t* nb;
  const double* carima_B;
  const int32_t* dp;
  const double* du_min;
  const double* du_max;
  const double* u_min;
  const double* u_max;
  const double* yref;
  /* ---- abi_version >= 2 (ignored for version 1 descriptors) -------------------------------
   * dtc      1: DTC-GPC (DTC_GPC_WW.m:126-164): the free response is driven by the predictor
   *             yp = Gz*u + Fr*(y - Pz*u) (OptimalPredictor2.m:24-40) instead of the measured y.
   *             The caller passes the model with its real delays (MatG window n1 = dmin+1),
   *             dp = dnz = descompMPC delays minus dmin (deltaUFree.m / DTC_GPC_WW.m:91-93) and
   *             the Diophantine window starts at d = 0 (DTC_GPC_WW.m:80).  Requires open_loop 0.
   * filter   [my] Fr_i(z) (mimofilter.m / filtro_siso.m), delay 0; NULL -> Fr = 1
   * nq       plant-only disturbance inputs: they drive the simulated plant through dist and are
   *             never seen by the controller's model (DTC_GPC_WW.m:29-30 Pq, :128-129)
   * dist     [my*nq] disturbance paths; their signals are the rows of eval's v: [nref][nd+nq][nit] */
  int32_t dtc;
  const mpct_dtf* filter;
  int32_t nq;
  const mpct_dtf* dist;
  /* nplant     number of simulated-plant variants (plant-mismatch Monte-Carlo draws, SURVEY
   *            §8d config 4); 0 or 1 -> the single plant above.  Simulation s = c*nref + k runs
   *            variant k % nplant (the draws ride on the reference dimension)
   * plant_var  [nplant][my*(nu+nd)] variant plants (replace plant when nplant > 1)           */
  int32_t nplant;
  const mpct_dtf* plant_var;
  /* ---- abi_version >= 3 --------------------------------------------------------------------
   * mdband   1: the toolbox MPC with measured-disturbance feed-forward and soft output bands
   *             (Shell7x5.m:112-196, WoodBerry.m:102-148; mdband_kernel.hip).  MD
   *             columns nu..nu+nd-1 of plant/model enter the prediction held at v(t)
   *             (mpcsimopt MDLookAhead 'off'); OV Min/Max are softened by MinECR/MaxECR with ONE
   *             slack eps >= 0 weighted by rho_ecr (Weights.ECR); Weights.OV / Weights.MVRate act
   *             over the ScaleFactors.  Requires plant == model (closedloop_toolbox.m:50 sims the
   *             model), n1[i] == 1 (PredictionHorizon window), dtc == 0, nq == 0, nplant <= 1 and
   *             nu*nu_max + 1 <= 64.  na/carima_A/nb/carima_B/dp may be NULL (no Diophantine tables).
   * y_min, y_max [my]      OV Min / Max, already scaled (MPCTuning.m:180-181); +-INFINITY: none
   * ecr_min, ecr_max [my]  OV MinECR / MaxECR (0: hard output bound)
   * y_scale [my], u_scale [nu]  OV / MV ScaleFactor after MPCTuning.m:175-184 (NULL: all 1)
   * rho_ecr                Weights.ECR (Shell7x5.m:191, MPCTuning.m:354)                       */
  int32_t mdband;
  const double* y_min;
  const double* y_max;
  const double* ecr_min;
  const double* ecr_max;
  const double* y_scale;
  const double* u_scale;
  double rho_ecr;
} mpct_scenario_desc;

typedef struct mpct_scenario mpct_scenario;

/* Nonlinear MPC scenario (config 5): the seam
 *   function [y,u,yopt,uopt] = closedloop_toolbox_nmpc(nmpcobj,model,init,r,N,Nu,delta,lambda,nit)
 *   (Matlab-Toolbox/NMPC/closedloop_toolbox_nmpc.m:1; callers VNS2.m:155, GAM_fun.m:87,
 *   MPC-Tuning/VanDeVusse_NMPC.m:244).  MATLAB passes the model as a function handle; a C ABI
 *   cannot carry one to the GPU, so the model is chosen from the library's built-in families by id
 *   with its parameters:
 *     model  MPCT_NMPC_VANDEVUSSE: nmpc_vandevusse_state.m (nx = 3, nu = 2), params[16] in the
 *            order of nmpc_vandevusse_state.m:43-58 (k10 k20 k30 E1 E2 E3 dHab dHbc dHad rho cp
 *            Kw Ar V T0 Ca0); NULL = the reference's values
 *   xc[ny]          output states, 1-based as init.xc (VanDeVusse_NMPC.m:82: [2 3]); ny <= 2
 *   ts, nsub        Ts and the fixed RK4 sub-steps per Ts that replace ode15s / the toolbox's
 *                   discretisation (plant and prediction use the same integrator)
 *   x0[nx], u0[nu]  init.x0, init.u0
 *   u_min/u_max[nu] MV Min/Max (hard); x_min/x_max[nx] hard state bounds, linearised in
 *                   every SQP subproblem (+-inf = none; a closed loop whose states still leave
 *                   them is flagged MPCT_ST_BOUNDS); y_scale[ny], u_scale[nu] OV / MV ScaleFactor
 *   n_max, nu_max   largest prediction / control horizon any candidate uses (nu*nu_max <= 32)
 *   nit, yref[ny*nit], vns_ink  as in mpct_scenario_desc
 *   sqp_max, sqp_tol  Gauss-Newton iteration cap per controller call and the stopping test
 *                   max |change of an absolute move| / u_scale <= sqp_tol (0: 100 and 1e-8); each
 *                   step is globalised by Armijo backtracking on the cost
 * Evaluate with mpct_eval_batch(_device) exactly like a linear scenario: N2[] holds N, delta[] the
 * OV weights, lambda[] the MVRate weights, r[] the reference sets (ny rows), v = NULL; ys / uopt
 * are yopt / uopt; qp_iters counts Gauss-Newton iterations. */
#define MPCT_NMPC_VANDEVUSSE 1
typedef struct mpct_nmpc_desc {
  int32_t abi_version; /* >= 4 */
  int32_t model;
  int32_t nx, ny, nu;
  const double* params;
  const int32_t* xc;
  double ts;
  int32_t nsub;
  const double* x0;
  const double* u0;
  const double* u_min;
  const double* u_max;
  const double* x_min;
  const double* x_max;
  const double* y_scale;
  const double* u_scale;
  int32_t n_max, nu_max;
  int32_t nit;
  const double* yref;
  int32_t vns_ink;
  int32_t sqp_max;
  double sqp_tol;
} mpct_nmpc_desc;

/* Build a nonlinear MPC scenario (no device needed).  Returns MPCT_OK. */
int32_t mpct_nmpc_scenario_create(const mpct_nmpc_desc* desc, mpct_scenario** out);

/* Evaluation options. */
typedef struct mpct_opts {
  int32_t open_loop;   /* 1: also compute the open-loop first-move prediction (uopt, ys) and
                          the VNS terms j21/Jnu (closedloop_toolbox.m:85-100); 0: closed loop
                          + J1/j22 only (all GAM_fun needs, GAM_fun.m:81)                  */
  int32_t want_traj;   /* 1: write y/u (and ys/uopt if open_loop) trajectories             */
  int32_t max_qp_iter; /* active-set iteration cap per step (0 = default 8*M)              */
  int32_t device;      /* HIP device ordinal (-1 = current)                               */
  double feas_tol;     /* constraint feasibility tolerance (0 = default 1e-10)            */
} mpct_opts;

/* Results, one row per SIMULATION s = c*nref + k (candidate c, reference k).  Any pointer may
 * be NULL to skip that output.  Sizes: J1/j21/j22 [S*my], Jnu [S*nu], status/qp_iters [S],
 * y/ys [S*my*nit], u/uopt [S*nu*nit].
 *   J1[i]  = sum_t (y_i - yref_i)^2                       GAM_fun.m:110-111
 *   j21[i] = sum_{t>=inK} (y_i - ys_i)^2                   VNS2.m:172,176
 *   j22[i] = sum_{t>=inK} (y_i - yref_i)^2                 VNS2.m:173,177
 *   Jnu[n] = sum_t (|uopt_n(1)| / |diff(uopt_n)|)^2, inf/NaN -> 0   VNS2.m:183-191           */
typedef struct mpct_result {
  double* J1;
  double* j21;
  double* j22;
  double* Jnu;
  int32_t* status;
  int64_t* qp_iters;
  double* y;
  double* u;
  double* ys;
  double* uopt;
} mpct_result;

/* Version / capability query (no device needed). */
int32_t mpct_abi_version(void);
const char* mpct_last_error(void);

/* Build a scenario: validates the description, precomputes the candidate-independent tables on
 * the host (step responses s_ij(t), Diophantine F rows, deltaUFree/cell2mat2 past-control
 * rows; see DESIGN.md §Data layout).  Does NOT touch the GPU (device copies are made on first
 * evaluation), so it is usable on a CPU-only host for inspection.  Returns MPCT_OK. */
int32_t mpct_scenario_create(const mpct_scenario_desc* desc, mpct_scenario** out);
void mpct_scenario_destroy(mpct_scenario* s);

/* Host-table inspection (testing / MATLAB-side debugging; no device needed).
 *   which: 0 = MV step table [my][nu][tlen], 1 = free-response table Phi [my*n2_max][nx],
 *          2 = dims {my, nu, nd, n2_max, nu_max, tlen, nx, nyh, nup, nit, nq},
 *          3 = Phi on the device state basis [y-r, backward differences of y | du history]
 * Copies at most cap doubles into buf; returns the number of doubles the table holds, or <0. */
int64_t mpct_scenario_table(const mpct_scenario* s, int32_t which, double* buf, int64_t cap);

/* Score C candidates x nref references.  Host pointers (MATLAB / ctypes callers).
 *   N2[C], Nu[C]      horizons used by the toolbox: max(N), max(Nu) (closedloop_toolbox.m:38-40)
 *   delta[C*my], lambda[C*nu]   Weights.OV, Weights.MVRate (closedloop_toolbox.m:42-43)
 *   r[nref*my*nit]    reference sets (row signals; VNS passes one unit step per output,
 *                     VNS2.m:148-150; GAM passes Xsp)
 *   v[nref*(nd+nq)*nit] disturbance signals per reference set (NULL when nd + nq == 0)     */
int32_t mpct_eval_batch(mpct_scenario* s, int64_t C, const int32_t* N2, const int32_t* Nu,
                        const double* delta, const double* lambda, int32_t nref, const double* r,
                        const double* v, const mpct_opts* opts, mpct_result* out);

/* Same, all pointers DEVICE pointers (inputs already resident in HBM; results written to
 * device memory), enqueued on `stream` (a hipStream_t, NULL = default stream) and NOT
 * synchronised — the caller synchronises.  Used by multi-GPU sharding and the benchmark.
 * Batches of 256 or more candidates are dispatched heaviest-first (an a-priori work key and a
 * device radix sort on `stream`, ~20 us; results stay in the caller's order).  The sort buffers
 * belong to the scenario.  Back-to-back calls on one scenario from different streams are safe:
 * each sort waits for the launch that read the previous permutation. */
int32_t mpct_eval_batch_device(mpct_scenario* s, int64_t C, const int32_t* N2, const int32_t* Nu,
                               const double* delta, const double* lambda, int32_t nref,
                               const double* r, const double* v, const mpct_opts* opts,
                               mpct_result* out, void* stream);

/* Score C candidates on ndev GPUs of this process at once (host pointers, like mpct_eval_batch).
 * The candidates are independent (VNS2.m:148-169, GAM_fun.m:79-91 score each one in isolation),
 * so they are split into strided shards: slot k scores candidates k, k+ndev, k+2*ndev, ...
 * (mpct_shard_candidates) on devices[k].  Tuning grids are built cell by cell (all lambda draws of
 * one (N2, Nu) pair together), so a contiguous split would hand one slot all the heavy horizons;
 * the strided one gives every slot the same mix.  Each slot gets its own scenario context (a copy
 * of the tables, its own stream and scratch), one host thread per slot gathers its candidates,
 * drives the H2D copies, launch and D2H copies and scatters the results back, and the call returns
 * when every shard is done.  Results land in the caller's order (simulation s = c*nref + k), so a
 * single-threaded MATLAB host drives all GPUs of a node with one call.  A device ordinal may
 * appear more than once (each occurrence gets its own context and stream on that device).
 * ndev = 1 is exactly mpct_eval_batch on devices[0].  opts->device is ignored.  Every ordinal is
 * checked before any work starts.  Errors: the first failing slot's code, its message prefixed
 * with "device <ordinal>: ". */
int32_t mpct_eval_batch_multi(mpct_scenario* s, int32_t ndev, const int32_t* devices, int64_t C,
                              const int32_t* N2, const int32_t* Nu, const double* delta, const double* lambda,
                              int32_t nref, const double* r, const double* v, const mpct_opts* opts,
                              mpct_result* out);

/* The strided shard of C candidates that device slot k of ndev scores (the split of
 * mpct_eval_batch_multi and of the torch.distributed ranks, mpct.dist.shard_indices): candidates
 * k, k+ndev, ... < C.  Writes at most cap indices into idx (idx may be NULL); returns the shard's
 * size ceil((C - k) / ndev), or <0. */
int64_t mpct_shard_candidates(int64_t C, int32_t ndev, int32_t k, int64_t* idx, int64_t cap);

/* The ranking every rank computes after the cost all-gather (Shell3x3.m:161 ranks by
 * the Pareto-weighted cost): perm[0..C) = candidate indices by ascending s_c = sum_j costs[c*k+j] *
 * w[j], ties by candidate index, NaN costs (failed / sentinel candidates) last.  All pointers are
 * DEVICE pointers; enqueued on `stream` (NULL = default), not synchronised.  One key kernel and a
 * device radix sort (stable).  Returns MPCT_OK or <0. */
int32_t mpct_rank_device(const double* costs, int64_t C, int32_t k, const double* w, int32_t* perm, void* stream);

/* Name of the kernel instance mpct_eval_batch(_device) launches for this scenario and options,
 * e.g. "gpc_closed_loop_kernel<16,false,false>" (QP-size class, DTC mode, open-loop/trajectory
 * state).  Copies at most cap-1 characters plus a NUL into buf; returns the name's length, or <0.
 * No device needed (tests pin the instance a benchmark times). */
int32_t mpct_kernel_instance(const mpct_scenario* s, const mpct_opts* opts, char* buf, int32_t cap);

/* Bytes of dynamic LDS one simulation's workgroup uses for this scenario at (N2, Nu) with the
 * open-loop leg / trajectories on (the cost-only instance of a linear scenario needs less); <0 on
 * error.  Lets a host check occupancy before launching. */
int64_t mpct_lds_bytes(const mpct_scenario* s, int32_t N2, int32_t Nu);

/* The same for the instance a call with these options launches (opts NULL = costs only: the
 * GAM_fun.m:81 call, which the tuning-grid benchmark times). */
int64_t mpct_lds_bytes_opts(const mpct_scenario* s, const mpct_opts* opts, int32_t N2, int32_t Nu);

#ifdef __cplusplus
}
#endif
#endif /* MPCT_H */
