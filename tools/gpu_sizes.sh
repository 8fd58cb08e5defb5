set -o pipefail
for E in "TAG=wgs512 SFM_EPI_WGS=512" "TAG=wgs384 SFM_EPI_WGS=384" "TAG=wgs256 SFM_EPI_WGS=256" "TAG=wgs512hb2 SFM_EPI_WGS=512 SFM_EPI_HB_MIN=2"; do
  env $E timeout -k 10 60 python tools/score_sizes.py || exit 1
done
for E in "SFM_EPI_WGS=512" "SFM_EPI_WGS=384" "SFM_EPI_WGS=256"; do echo "$E"; env $E timeout -k 10 120 python tools/ransac_ab.py - 1 | grep -E "dropin|call_kernels"; done
