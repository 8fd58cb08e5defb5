#!/bin/bash
# Dev helper: the package built with extra compile flags into abso/NAME
# (python files + libsfmcore.so), for same-box A/B runs.
#   tools/build_variant.sh NAME "-DFOO=1 -DBAR=2" [GIT_REV]
set -e
NAME=$1; FLAGS=$2; REV=$3
W=/tmp/bv_$NAME
rm -rf $W && mkdir -p $W
if [ -n "$REV" ]; then
  git -C /root/repo archive $REV structure-from-motion-_amd include | tar -x -C $W
else
  cp -r /root/repo/structure-from-motion-_amd /root/repo/include $W/
  rm -rf $W/structure-from-motion-_amd/build $W/structure-from-motion-_amd/libsfmcore.so
fi
make -s -C $W/structure-from-motion-_amd -j8 HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-result $FLAGS" >/dev/null
mkdir -p /root/repo/abso/$NAME
cp $W/structure-from-motion-_amd/*.py $W/structure-from-motion-_amd/libsfmcore.so /root/repo/abso/$NAME/
echo built abso/$NAME
