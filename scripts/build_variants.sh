#!/bin/bash
# build libtorj_hip variants for A/B timing: NAME:DEFINES ...
set -e
cd "$(dirname "$0")/../torj.jl_amd/csrc"
mkdir -p ../build/variants
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -fopenmp -shared $defs -o ../build/variants/libtorj_hip_$name.so torj_hip.hip &
done
wait
ls -la ../build/variants
