L=structure-from-motion-_amd/libsfmcore.so
cp $L abso/cur.so
for V in a b a b; do
  [ -f abso/$V.so ] || break
  cp abso/$V.so $L
  echo "== $V" >> gpurun_out/so_ab.log
  timeout -k 10 200 python tools/gj_ab.py SFM_GJ_X 0 1 >> gpurun_out/so_ab.log 2>&1 || break
  [ -f abso/$V.so ] || break
done
cp abso/cur.so $L
