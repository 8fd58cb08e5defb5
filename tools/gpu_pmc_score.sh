# PMC passes over the cfg2 one-shot F score: the round-4 kernel (abso/head) and the tree's.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"
for d in abso/head structure-from-motion-_amd abso/v4p1; do
  n=$(basename $d)
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc/kt_$n -o kt --output-format csv -- python3 tools/score_once.py $d > gpurun_out/pmc/kt_$n.log 2>&1 || { echo "kt $n failed"; exit 1; }
  i=1
  for P in "$P1" "$P2"; do
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc/p${i}_$n -o pmc --output-format csv -- python3 tools/score_once.py $d > gpurun_out/pmc/p${i}_$n.log 2>&1 || { echo "pmc $i $n failed"; tail -3 gpurun_out/pmc/p${i}_$n.log; exit 1; }
    i=$((i+1))
  done
done
find gpurun_out/pmc -name "*.csv" | head -20
