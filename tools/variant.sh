#!/bin/bash
# Build a libmpct variant with extra defines for the gpc kernel:  bash tools/variant.sh NAME -DFOO=1 ...
set -e
C=/root/repo/model-predictive-control-tuning_amd/csrc; NAME=$1; shift
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result "$@" -c $C/gpc_kernel.hip -o /tmp/gpc_$NAME.o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result "$@" -c $C/mpct_host.cpp -o /tmp/host_$NAME.o
hipcc --offload-arch=gfx950 -shared -fPIC /tmp/gpc_$NAME.o $C/mdband_kernel.o $C/nmpc_kernel.o $C/work_order.o /tmp/host_$NAME.o -o $C/libmpct_$NAME.so
echo built $C/libmpct_$NAME.so
