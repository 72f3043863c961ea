#!/bin/bash
# Build a libmpct variant with extra defines for one kernel unit (default gpc_kernel.hip; K=gpc_small.hip,
# K=mdband_kernel.hip or K=nmpc_kernel.hip for the others, K=all for every kernel unit) and the host unit:
#   [K=unit.hip] bash tools/variant.sh NAME -DFOO=1 ...
set -e
C=/root/repo/model-predictive-control-tuning_amd/csrc; NAME=$1; shift
K=${K:-gpc_kernel.hip}
OBJS=""
for u in gpc_kernel gpc_small dtc_small mdband_kernel nmpc_kernel work_order; do
  if [ "$u.hip" = "$K" ] || { [ "$K" = all ] && [ $u != work_order ]; }; then
    UF=""; [ $u = gpc_small ] && UF="-mllvm -amdgpu-sched-strategy=max-ilp -mllvm -misched-prera-direction=topdown"  # __graft_entry__.UNIT_FLAGS
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $UF "$@" -c $C/$u.hip -o /tmp/${u}_$NAME.o
    OBJS="$OBJS /tmp/${u}_$NAME.o"
  else
    OBJS="$OBJS $C/$u.o"
  fi
done
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result "$@" -c $C/mpct_host.cpp -o /tmp/host_$NAME.o
hipcc --offload-arch=gfx950 -shared -fPIC $OBJS /tmp/host_$NAME.o -o $C/libmpct_$NAME.so
echo built $C/libmpct_$NAME.so
