set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" gpurun_out/counters_list.txt | sort -u > gpurun_out/sq_counters.txt || true
bash tools/pmc_join.sh "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES" > gpurun_out/pmc_slot.txt 2>&1
cat gpurun_out/pmc_slot.txt
