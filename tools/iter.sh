#!/bin/bash
# GPU iteration: parity tests, A/B kernel time against libmpct_old.so, section profile.
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; C=model-predictive-control-tuning_amd/csrc
mkdir -p gpurun_out
timeout -k 10 400 python3 -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
grep -h "full grid" gpurun_out/pytest_gpu.log || true
for lib in libmpct_old.so libmpct.so; do
  [ -f $C/$lib ] && MPCT_LIB=$R/$C/$lib timeout -k 10 120 python3 tools/ab.py 2>&1 | grep -v amdgpu.ids
done
[ -f $C/libmpct_prof.so ] && timeout -k 10 200 python3 tools/kprof.py 4096 2>&1 | grep -v amdgpu.ids | tail -14
