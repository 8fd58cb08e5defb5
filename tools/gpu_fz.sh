set -o pipefail
bash tools/trace_ransac2.sh rtl11 "SFM_RANSAC_FUSED=0"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rtl11/f1
cp tools/ransac_once.py /tmp/ro.py
sed -i 's#sys.path\[:0\] = \[#sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "abso", "f1"), #' tools/ransac_once.py
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rtl11/f1/trace -o run -- python tools/ransac_once.py > gpurun_out/rtl11/f1/trace.log 2>&1
cp /tmp/ro.py tools/ransac_once.py
echo DONE2
