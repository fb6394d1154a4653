#!/usr/bin/env bash
# Counter passes over the cold top-k filter (topk_x3_kernel, DBP15K zh_en).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${PMC_DIR:-r6ae}; mkdir -p $O
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_WAVE32_LDS SQ_INSTS_SENDMSG"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/pmc$i -o run -- python tools/micro/topk_cold.py 2 > $O/pmc$i.log 2>&1 || { tail -5 $O/pmc$i.log; exit 1; }
  f=$(find $O/pmc$i -name '*counter_collection.csv' | head -1); python tools/pmc_summary.py $f topk_x3 > $O/pmc_topk_$i.txt || exit 1
  rm -rf $O/pmc$i
  cut -c1-500 $O/pmc_topk_$i.txt
done
