set -o pipefail
for r in 1 2; do
for S in "" "1024,4096,4096,4096,2048,1024" "1024,3072,4096,4096,3072,1024" "512,2048,4096,4096,4096,1024,512" "1024,4096,4096,4096,3072"; do
  echo "[$S] $(SFM_RP_SCHEDULE="$S" timeout -k 10 120 python tools/dropin_phases.py)"
done; done
