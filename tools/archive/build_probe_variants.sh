#!/bin/bash
# Measurement variants of the probe kernels (tools only, never the product):
#   tools/build_probe_variants.sh pabl1="-DLSMB_PROBE_ABL=1" ...
# -> storage-engine_amd/lib/liblsmbloom_<name>.so (bloom_probe.hip recompiled
# with the flags).  Run with LSMB_LIB=... python bench.py ...
set -e
cd "$(dirname "$0")/../storage-engine_amd"
make -j8 >/dev/null
for nv in "$@"; do
  name=${nv%%=*}; flags=${nv#*=}
  mkdir -p build/var_$name
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics $flags \
    -c csrc/bloom_probe.hip -o build/var_$name/bloom_probe.o &
done
wait
for nv in "$@"; do
  name=${nv%%=*}
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/liblsmbloom_$name.so \
    build/var_$name/bloom_probe.o $(ls build/*.o | grep -v '/bloom_probe.o$')
done
echo built: "$@"
