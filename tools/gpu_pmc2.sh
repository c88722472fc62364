#!/bin/bash
# PMC passes over the fused kernel, each its own rocprofv3 run within the per-block limits
# (SQ <= 8, TCC <= 4 with FETCH_SIZE = 3 / WRITE_SIZE = 2, TA/TD/GRBM <= 2, TCP <= 4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/${PMC_DIR:-pmc3}
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "import torch; print(torch.cuda.is_available())" > /dev/null 2>&1
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/${PMC_DIR:-pmc3}/$name -o $name --output-format csv \
    -- python3 tools/pmc_fused.py > gpurun_out/${PMC_DIR:-pmc3}/$name.log 2>&1
}
run fetch FETCH_SIZE GRBM_GUI_ACTIVE && echo fetch ok && \
run write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum && echo write ok && \
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU && echo sq ok && \
run ta TA_TA_BUSY_sum TA_BUSY_avr TD_TD_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum TCP_PENDING_STALL_CYCLES_sum && echo ta ok
rc=$?
python3 tools/pmc_summary.py gpurun_out/${PMC_DIR:-pmc3} fused_kernel
exit $rc
