set -o pipefail
python -u -c "
import sys,json; sys.path.insert(0,'.')
from dpu_operator_amd.utils import cpuquota
print(json.dumps({'cpu_share': cpuquota.cpu_share()}))" >> gpurun_out/r6_s3_live_full.jsonl
for c in "8 0 8" "8 0 6" "7 0 7" "6 0 6" "8 0 8"; do
  set -- $c
  timeout -k 10 120 python -u tools/live_bench.py --queues $1 --tx-workers $2 --threads $3 --trials 3 --duration 1.0 >> gpurun_out/r6_s3_live_full.jsonl 2>> gpurun_out/r6_s3_live_full.err || exit $?
done
