#!/bin/bash
# Build an experimental variant of libtic.so with extra compile flags for the stride-1 / chain
# kernels (e.g. -DW4_SCHED=2): tools/build_variant.sh NAME FLAGS...  ->  tf_image_compression_amd/libtic_NAME.so
# (select it with TIC_LIB=...; the other objects are the default build's; KERNELS="conv_s2 ..."
# picks which kernel objects get the flags)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
make -s -j8 >/dev/null
mkdir -p build/v_$name
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude -Itf_image_compression_amd/csrc"
for k in ${KERNELS:-conv_s1 conv_chain}; do
  /opt/rocm/bin/hipcc $F "$@" -c tf_image_compression_amd/csrc/$k.hip -o build/v_$name/$k.o &
done
wait
objs=""
for o in build/*.o; do b=$(basename $o); if [ -f build/v_$name/$b ]; then objs="$objs build/v_$name/$b"; else objs="$objs $o"; fi; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tf_image_compression_amd/libtic_$name.so $objs -Wl,-rpath,/opt/rocm/lib
echo built tf_image_compression_amd/libtic_$name.so
