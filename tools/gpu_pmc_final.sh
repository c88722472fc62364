#!/bin/bash
# PMC counter passes over the 1-GPU headline bench (fused kernel), one rocprofv3 run per group;
# every group within the per-block limits (<= 8 SQ, <= 4 TCC with FETCH_SIZE = 3 / WRITE_SIZE = 2,
# <= 4 TCP, <= 2 TA / TD / GRBM).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/pmc_final
mkdir -p $out
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" -d $out/$name -o $name --output-format csv \
    -- python3 bench.py --steps 5 --warmup 1 --no-lowlat --no-variants --rotate 1 > $out/$name.log 2>&1
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES && echo p1 ok && \
run p2 SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE && echo p2 ok && \
run p3 FETCH_SIZE TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum && echo p3 ok && \
run p4 WRITE_SIZE TCC_HIT_sum TCC_MISS_sum && echo p4 ok
rc=$?
python3 tools/pmc_summary.py $out fused_kernel > $out/summary.txt 2>&1
cat $out/summary.txt
exit $rc
