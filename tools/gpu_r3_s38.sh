set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3_s38_prof -o prof --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-live > $GRAFT_REPO_ROOT/gpurun_out/r3_s38_prof.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAIT_INST_ANY -d $GRAFT_REPO_ROOT/gpurun_out/r3_s38_pmc -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --variant-steps 3 --no-lowlat --no-live --rotate 1 > $GRAFT_REPO_ROOT/gpurun_out/r3_s38_pmc.log 2>&1
