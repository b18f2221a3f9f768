#!/bin/bash
# Builds measurement variants of the library (tools only, never the product):
#   [VSRC=bloom_probe] tools/build_variants.sh name1="-DLSMB_ABL=1" name2="-DLSMB_PIPE=1" ...
# -> storage-engine_amd/lib/liblsmbloom_<name>.so (csrc/$VSRC.hip, default
# bloom_build, recompiled with the flags; the other objects shared).  Run them
# with tools/run_variants.sh.
set -e
cd "$(dirname "$0")/../storage-engine_amd"
make -j8 >/dev/null
for nv in "$@"; do
  name=${nv%%=*}; flags=${nv#*=}
  mkdir -p build/var_$name
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics $flags \
    -Wno-unused-value -c csrc/${VSRC:-bloom_build}.hip -o build/var_$name/${VSRC:-bloom_build}.o &
done
wait
for nv in "$@"; do
  name=${nv%%=*}
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/liblsmbloom_$name.so \
    build/var_$name/${VSRC:-bloom_build}.o $(ls build/*.o | grep -v "/${VSRC:-bloom_build}.o\$")
done
echo built: "$@"
