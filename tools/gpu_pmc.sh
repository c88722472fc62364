#!/bin/bash
# PMC counter passes over the 1-GPU bench (fused kernel), one rocprofv3 run per counter group
# (each within the per-block limits: <= 8 SQ, <= 4 TCC counters per run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc2/$name -o $name --output-format csv \
    -- python3 bench.py --steps 5 --warmup 1 --no-lowlat --rotate 1 > gpurun_out/pmc2/$name.log 2>&1
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH && echo p1 ok && \
run p2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS && echo p2 ok && \
run p3 SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VSKIPPED SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE && echo p3 ok && \
run p4 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum && echo p4 ok && \
run p5 TCC_EA0_WRREQ_sum TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_DRAM_sum && echo p5 ok
rc=$?
python3 tools/pmc_summary.py gpurun_out/pmc2 fused_kernel
exit $rc
