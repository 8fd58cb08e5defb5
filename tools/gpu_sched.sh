set -o pipefail
for S in "" "2048,7168,7168" "1024,5120,5120,5120" "2048,4096,4096,4096,2048" "1536,6144,6144,2560" "1024,3072,6144,6144"; do
  echo "sched=[$S]"
  SFM_RP_SCHEDULE="$S" timeout -k 10 120 python tools/ransac_ab.py - 1 | grep -E "dropin|call_kernels|call  " || exit 1
done
for d in abso/p2 abso/p3 abso/p4; do TAG=$d timeout -k 10 60 python tools/score_sizes.py $d || exit 1; done
