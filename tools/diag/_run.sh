set -o pipefail
O=gpurun_out/r04zk; mkdir -p $O
timeout -k 10 600 python3 -u tools/shard_balance.py --only shell7x5 --out $O/shard_balance.json > $O/shard_balance.log 2>&1 || { tail -20 $O/shard_balance.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/shard_balance.json'))
for k,v in d['shell7x5'].items(): print(k, [round(x) for x in v['shard_ms']], round(max(v['shard_ms'])), round(v['max_over_mean'],3))"
echo diag done
