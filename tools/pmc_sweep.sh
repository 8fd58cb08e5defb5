set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_$tag -o run -- python tools/ba_once.py > gpurun_out/pmc_$tag.log 2>&1
done
echo ok
