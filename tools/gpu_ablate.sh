#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 500 python tools/ablate.py > gpurun_out/ablate.log 2>&1 && echo "ablate ok" && \
(rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true) && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/pmc/p1 -o p1 --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-lowlat --rotate 1 > gpurun_out/pmc/p1.log 2>&1 && echo "pmc1 ok" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc/p2 -o p2 --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-lowlat --rotate 1 > gpurun_out/pmc/p2.log 2>&1 && echo "pmc2 ok"
rc=$?
cat gpurun_out/ablate.log | grep -v amdgpu.ids
exit $rc
