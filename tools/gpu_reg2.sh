set -o pipefail
export TMPDIR=/tmp
: > gpurun_out/rab2.txt
for d in structure-from-motion-_amd abso/p1 abso/p2 abso/s5 abso/s3; do
  timeout -k 10 120 python tools/ransac_ab.py $d 1 >> gpurun_out/rab2.txt 2>&1 || { echo "fail $d"; exit 1; }
done
grep -E "package|oneshot_score|call_kernels" gpurun_out/rab2.txt | sed 's#.*/repo/##'
mkdir -p gpurun_out/pmc2
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"
i=1
for P in "$P1" "$P2"; do
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc2/p$i -o pmc --output-format csv -- python3 tools/score_once.py > gpurun_out/pmc2/p$i.log 2>&1 || { echo "pmc $i failed"; tail -3 gpurun_out/pmc2/p$i.log; exit 1; }
  i=$((i+1))
done
echo pmc done
