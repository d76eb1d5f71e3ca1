set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1 || true
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc1 -o run -- python $GRAFT_REPO_ROOT/tools/conv_one.py l3 6 > $GRAFT_REPO_ROOT/gpurun_out/pmc1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_WAVE32 --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc2 -o run -- python $GRAFT_REPO_ROOT/tools/conv_one.py l3 6 > $GRAFT_REPO_ROOT/gpurun_out/pmc2.log 2>&1
