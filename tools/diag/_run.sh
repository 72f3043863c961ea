#!/bin/bash
# GPU suite on the max-ILP / top-down metric build, then scheduler variants of the other kernel units
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r05j2"; mkdir -p "$O"; C="$R/model-predictive-control-tuning_amd/csrc"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 200 python3 bench.py --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || exit 1; cut -c1-260 "$O/bench.json"
run() {  # W L rep
  MPCT_LIB=$C/$2 timeout -k 10 200 python3 bench.py --workload $1 --no-cpu-baseline > "$O/$1.$2.$3.json" 2> "$O/$1.$2.$3.err" || { tail -5 "$O/$1.$2.$3.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['value']), round(d['ms_per_step'],3), d.get('top_candidate'))" "$O/$1.$2.$3.json" $1 $2
}
for rep in 1 2; do
  for L in libmpct.so libmpct_mtd.so libmpct_mmc.so libmpct_mii.so; do run shell7x5 $L $rep; done
  for L in libmpct.so libmpct_gtd.so; do run dtc-mc $L $rep; done
  for L in libmpct.so libmpct_ntd.so; do run vandevusse $L $rep; done
done
