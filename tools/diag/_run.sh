#!/bin/bash
# r06ad (diagnostic): the metric QP's drops split into setup + shifts (the open_loop slot of the profile build,
# unused by the metric) and rotations, over the heaviest 256 simulations; the plain profile build beside it
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; T=${1:-r06ad}; O="gpurun_out/$T"; mkdir -p "$O"
C=$R/model-predictive-control-tuning_amd/csrc
bash tools/gpu_steps.sh "$O" \
  "120 kprof_ds env MPCT_LIB=$C/libmpct_profds.so MPCT_PROF_OUT=$O/ds.bin python3 tools/kprof.py 256 heavy" \
  "120 kprof env MPCT_LIB=$C/libmpct_prof.so MPCT_PROF_OUT=$O/base.bin python3 tools/kprof.py 256 heavy"
