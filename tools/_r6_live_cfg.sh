#!/bin/bash
# live pod->pod: queues x pod threads near the 16-CPU grant, full runs (saturated trials, idle, 90 %, half load)
cd "$(dirname "$0")/.."
for cfg in "7 8" "8 7" "8 8" "7 7" "6 8"; do
  set -- $cfg
  timeout -k 10 150 python -u tools/live_bench.py --device cuda:0 --queues $1 --threads $2 --trials 3 --duration 1.0 \
    > gpurun_out/r6_s25_live_q$1_g$2.json 2> gpurun_out/r6_s25_live_q$1_g$2.err || exit $?
  echo "q$1 g$2 done"
done
