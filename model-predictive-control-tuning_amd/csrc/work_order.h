// work_order.h — heaviest-first dispatch order of a batch of candidates (host side).
//
// The closed-loop kernels run one simulation per workgroup and their batches overfill the
// resident slots, so the last round of workgroups starts as slots free up; a long simulation that
// starts late sets the kernel time.  order_candidates sorts the candidates by an a-priori work
// key (longest-processing-time first) and hands the kernels a permutation slot -> candidate; the
// results stay in the caller's order.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "mpct_dev.h"

namespace mpct {

enum OrderKind {
  kOrderGpc = 0,   // GPC / DTC-GPC: QP size M, then the unconstrained move demand (or the weight ratio)
  kOrderNmpc = 1,  // NMPC: horizon N and the weight ratio (fewer Gauss-Newton iterations)
};

// per-candidate work bound of the controller-based GPC key (multiply-adds for H); above it the
// weight-ratio key is used
constexpr double kOrderEstMaxCost = 1 << 20;

// perm = nullptr when the batch is too small for the order to matter (kOrderMinC).  kOrderGpc with
// the scenario and its reference signals (sc, nref, r: device [nref][my][nit]) keys on the
// candidate's unconstrained move demand (order_keys_gpc); without them, on the weight ratio.
int order_candidates(int kind, int my, int nu, long long C, const int* N2, const int* Nu, const double* delta,
                     const double* lambda, WorkOrder& wo, const int** perm, hipStream_t stream, std::string* err,
                     const DevScenario* sc = nullptr, int nref = 0, const double* r = nullptr,
                     const DevResult* pre = nullptr, bool* prefilled = nullptr);

// ascending weighted-cost order of C candidates (mpct_rank_device): device pointers, on `stream`
int rank_device(const double* costs, long long C, int k, const double* w, int* perm, hipStream_t stream,
                std::string* err);

// staging rows for the cost records of an ordered launch of S simulations (DevResult::stage), and
// the gather of those rows back into the caller's order (one thread per simulation, contiguous
// writes); enqueue the gather after every launch of the batch
int order_stage(WorkOrder& wo, long long S, int width, double** stage, std::string* err);
int unpermute_results(const WorkOrder& wo, long long C, int nref, int my, int nu, const StageRow& R,
                      const DevResult& out, hipStream_t stream, std::string* err);

// every simulation slot of `out` (its staging rows when out.stage is set) <- NaN costs, status
// MPCT_ST_NOT_RUN, 0 iterations; enqueue before the class launches, which overwrite the records
// of the slots they simulate, so a slot that no launch claims cannot pass for a result
int prefill_results(const DevResult& out, long long S, int my, int nu, hipStream_t stream, std::string* err);
// diagnostic build only (-DMPCT_DIAG, csrc/libmpct_diag.so): with MPCT_DIAG_DROP_LAUNCH=k in the
// environment the k-th class launch of every batch is not issued (tests plant the dispatch fault
// that the prefill must expose).  The release library has no fault hook: always false
#ifdef MPCT_DIAG
bool diag_drop_launch(int k);
#else
inline bool diag_drop_launch(int) { return false; }
#endif

// after the launch(es) that read *perm: later sorts wait for them before rewriting the buffer
void order_mark_used(WorkOrder& wo, hipStream_t stream);
void order_release(WorkOrder& wo);

}  // namespace mpct
