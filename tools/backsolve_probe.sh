#!/bin/bash
# Builds tools/backsolve_probe (on the CPU side, in-tree under tools/bin).
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -c tools/backsolve_probe.hip -o tools/bin/backsolve_probe.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -o tools/bin/backsolve_probe tools/bin/backsolve_probe.o \
  structure-from-motion-_amd/build/sfm_api.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
