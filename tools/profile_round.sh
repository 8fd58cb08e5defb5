#!/bin/bash
# On the GPU box: bench line, rocprofv3 kernel trace + stats of bench.py, and
# per workload (cfg4, cfg5) the PMC passes (separate runs, --kernel-trace
# only, as the microarch guide prescribes) of tools/ba_once.py (20 fixed LM
# iterations = bench's timed region): HBM FETCH/WRITE, L2 hit, and the FP64
# VALU / MFMA instruction counters.  Output under gpurun_out/$1.  Every GPU
# step is time-limited; the bench and the traces stop the chain on a
# failure, a counter pass that fails is recorded and skipped.
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 800 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kernel_trace -o run --output-format csv -- python bench.py --no-cpu-baseline --no-next-rows > $OUT/prof.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || echo "list-avail failed" >> $OUT/passes.log
for W in cfg4 cfg5; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$W/kernel_trace -o run --output-format csv -- python tools/ba_once.py $W 20 > $OUT/kt_$W.log 2>&1 || exit 1
  for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64" \
           "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_WAVES" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
    tag=$(echo $C | tr ' ' '_')
    if timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/$W/$tag -o run -- python tools/ba_once.py $W 20 > $OUT/pmc_${W}_$tag.log 2>&1; then
      echo "$W $tag ok" >> $OUT/passes.log
    else
      echo "$W $tag FAILED $?" >> $OUT/passes.log
    fi
  done
done
# RANSAC (cfg2 drop-in calls): kernel trace and the FP64 / VALU counters of
# k_fit_samples and k_ransac_score (the executed-flop count behind bench's
# algorithmic-equivalent score rate)
W=ransac
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$W/kernel_trace -o run --output-format csv -- python tools/ransac_once.py > $OUT/kt_$W.log 2>&1 || exit 1
for C in "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64" \
         "SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" FETCH_SIZE; do
  tag=$(echo $C | tr ' ' '_')
  if timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/$W/$tag -o run -- python tools/ransac_once.py > $OUT/pmc_${W}_$tag.log 2>&1; then
    echo "$W $tag ok" >> $OUT/passes.log
  else
    echo "$W $tag FAILED $?" >> $OUT/passes.log
  fi
done
echo DONE
