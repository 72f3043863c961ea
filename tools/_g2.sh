set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
C=model-predictive-control-tuning_amd/csrc
for v in base w4 nowait w4nw base w4 nowait w4nw; do
  lib=$C/libmpct.so; [ $v = base ] || lib=$C/libmpct_$v.so
  MPCT_LIB=$lib QAB_DUMP=$O/$v.npz timeout -k 10 120 python3 tools/qab.py 1024 4096 8192 h256 2>&1 | grep -v amdgpu.ids | tee -a $O/qab.log || exit 1
done
python3 -c "
import numpy as np
a=np.load('$O/base.npz')
for v in ('w4','nowait','w4nw'):
    b=np.load('$O/%s.npz'%v)
    print(v, 'bitwise J1 equal:', np.array_equal(a['J1'], b['J1']), 'iters equal:', np.array_equal(a['it'], b['it']), 'max rel', np.max(np.abs(a['J1']-b['J1'])/np.abs(a['J1'])))
" | tee $O/cmp.txt
MPCT_LIB=$C/libmpct_prof.so timeout -k 10 120 python3 tools/kprof.py 256 heavy > $O/kprof_h256.txt 2>&1 || exit 1
MPCT_LIB=$C/libmpct_prof.so timeout -k 10 120 python3 tools/kprof.py 4096 > $O/kprof_4096.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/kprof_h256.txt $O/kprof_4096.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_band.py tests/test_dtc.py tests/test_gpu_tuning.py -x -v -s --timeout 300 --timeout-method thread -k "metric or config3_grid or full_size or row1 or engine_evaluators" > $O/pytest_new.log 2>&1; rc=$?
grep -E "config3:|config 4 full|metric instance|PASS|FAIL|Error|error" $O/pytest_new.log | head -30
echo rc=$rc
MPCT_LIB=$C/libmpct_nprof.so timeout -k 10 200 python3 tools/nmpc_latency.py > $O/nmpc_prof.txt 2>&1
grep -v amdgpu.ids $O/nmpc_prof.txt | head -80
for v in base pol4 nopol d8p4 polall; do
  lib=$C/libmpct.so; [ $v = base ] || lib=$C/libmpct_$v.so
  MPCT_LIB=$lib C3_DUMP=$O/c3_$v.npz timeout -k 10 200 python3 tools/config3_ab.py 2>&1 | grep -v amdgpu.ids | tee -a $O/config3_ab.txt
done
