#!/bin/bash
# PMC A/B of the early bucket fetch on the 1024-rule ACL: the fused kernel with (flags 0) and
# without (flags 256 = kFlagNoEarly) the early-fetch instance, one rocprofv3 run per counter group.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/${PMC_DIR:-pmc_early}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "import torch; print(torch.cuda.is_available())" > /dev/null 2>&1
run() {
  local name=$1 flags=$2; shift 2
  PMC_ACL=1024 PMC_FLAGS=$flags timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" -d $D/$name -o $name \
    --output-format csv -- python3 tools/pmc_fused.py > $D/$name.log 2>&1
}
for cfg in "early 0" "late 256"; do
  set -- $cfg
  run ${1}_ta $2 TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum && echo "$1 ta ok" && \
  run ${1}_sq $2 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE && echo "$1 sq ok" || exit 1
done
for cfg in early late; do
  echo "== $cfg"
  mkdir -p $D/sum_$cfg && cp -r $D/${cfg}_ta $D/${cfg}_sq $D/sum_$cfg/ && python3 tools/pmc_summary.py $D/sum_$cfg fused_kernel
done
