#!/bin/bash
# PMC passes over the ESP kernels (tools/esp_bench.py, 1404-B frames): L1/TA pressure vs VALU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/${PMC_DIR:-pmc_esp}
mkdir -p $D
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" -d $D/$name -o $name --output-format csv -- \
    python3 tools/esp_bench.py --sizes 1400 --n 65536 --steps 2 > $D/$name.log 2>&1
}
run ta TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum && echo "ta ok" && \
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE && echo "sq ok" && \
run lds SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_COUNT && echo "lds ok" || exit 1
mkdir -p $D/sum && cp -r $D/ta $D/sq $D/lds $D/sum/ && python3 tools/pmc_summary.py $D/sum esp_kernel
