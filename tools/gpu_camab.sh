# GPU session: camera LDS stride variants (abso/l*): BA kernel split alternated,
# then one PMC pass (LDS bank conflicts) per variant on cfg5.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cam
: > gpurun_out/cam/ab.txt
for r in 1 2; do
  for d in abso/l12b30 abso/l13b31 abso/l14b33; do
    echo "== $d" >> gpurun_out/cam/ab.txt
    timeout -k 10 200 python tools/gj_ab.py SFM_AB_DUMMY 0 1 $d >> gpurun_out/cam/ab.txt 2>&1 || { echo "fail $d"; exit 1; }
  done
done
grep -E "^==|^round" gpurun_out/cam/ab.txt | sed -E 's/ (point_prep|schur_blocks|allreduce|cholesky) [0-9.]+//g'
for d in abso/l12b30 abso/l13b31 abso/l14b33; do
  n=$(basename $d)
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES -d gpurun_out/cam/p_$n -o pmc --output-format csv -- python3 tools/gj_ab.py SFM_AB_DUMMY 0 1 $d > gpurun_out/cam/p_$n.log 2>&1 || { echo "pmc $n failed"; tail -3 gpurun_out/cam/p_$n.log; exit 1; }
done
echo done
