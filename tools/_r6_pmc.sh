#!/bin/bash
# round-6 PMC passes over the headline fused kernel (tools/pmc_fused.py), one counter group per run,
# then the ring A/B.  Stops at the first timeout / abort.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "stop: rc $rc ($2)"; exit $rc; fi; }
n=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE TCC_ATOMIC" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_LEVEL_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INST_LEVEL_VMEM"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/r6_pmc/p$n -o pmc --output-format csv -- python3 tools/pmc_fused.py \
    > gpurun_out/r6_pmc_p$n.log 2>&1; ok $? "pass $n"
done
timeout -k 10 300 python -u tools/ring_ab.py --trials 5 > gpurun_out/r6_s9_ring_ab.json 2> gpurun_out/r6_s9_ring_ab.err; ok $? ring_ab
echo done
