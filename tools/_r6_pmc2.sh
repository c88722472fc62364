#!/bin/bash
# PMC passes over the final headline kernel (buffer-load bucket fetch) and the ClassBench-style set
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "stop: rc $rc ($2)"; exit $rc; fi; }
n=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE TCC_ATOMIC" "TCC_HIT_sum TCC_MISS_sum"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/r6_pmc2/p$n -o pmc --output-format csv -- python3 tools/pmc_fused.py \
    > gpurun_out/r6_pmc2_p$n.log 2>&1; ok $? "pass $n"
done
PMC_WILD=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS \
  -d gpurun_out/r6_pmc2/wild -o pmc --output-format csv -- python3 tools/pmc_fused.py > gpurun_out/r6_pmc2_wild.log 2>&1; ok $? wild
echo done
