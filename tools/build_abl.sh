#!/bin/bash
# Builds LSMB_ABL timing-ablation variants of the library (tools/abl.sh).
set -e
cd "$(dirname "$0")/../storage-engine_amd"
make -j8 >/dev/null
for v in "$@"; do
  mkdir -p build/abl$v
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -DLSMB_ABL=$v \
    -c csrc/bloom_build.hip -o build/abl$v/bloom_build.o 2>/dev/null &
done
wait
for v in "$@"; do
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/liblsmbloom_abl$v.so build/abl$v/bloom_build.o build/bloom_probe.o build/capi.o
done
