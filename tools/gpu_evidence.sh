#!/bin/bash
# One end-of-round evidence pass on the GPU box (repo root): the -m gpu suite, smoke(), the bench
# line, a rocprofv3 --kernel-trace --stats pass, separate FETCH_SIZE and WRITE_SIZE passes (for
# roofline.traffic, keyed to this libmpct.so's sha256), and one SQ pass with the LDS bank-conflict
# counters plus a second SQ pass (FP64 ADD / MUL / TRANS, SALU, wait states) for
# roofline.fp64_counter_tflops.  Each GPU step has its own time limit; the first failure ends the script.
# Usage: bash tools/gpu_evidence.sh TAG   -> gpurun_out/TAG/
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
TAG="${1:-r03}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
sha256sum "$R/model-predictive-control-tuning_amd/csrc/libmpct.so" > "$O/lib_sha256.txt"
timeout -k 10 540 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
timeout -k 10 300 python3 bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
export TMPDIR=/tmp
cd /tmp
BENCH=(python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- "${BENCH[@]}" > "$O/kt.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o fetch -- "${BENCH[@]}" > "$O/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o write -- "${BENCH[@]}" > "$O/write.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FMA_F64 \
  --output-format csv -d "$O/sq" -o sq -- python3 "$R/tools/ab.py" > "$O/sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  --output-format csv -d "$O/sq2" -o sq2 -- python3 "$R/tools/ab.py" > "$O/sq2.log" 2>&1
echo evidence done
