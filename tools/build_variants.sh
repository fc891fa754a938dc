#!/bin/bash
# Builds A/B variants of libbdpt_amd.so: VARIANTS="name:FLAGS name2:FLAGS2 ..." -> build_var_<name>.so
# (common translation units compiled once, bdpt_hip.hip once per variant, in parallel).
cd "$(dirname "$0")/.." || exit 1
CS=bidirectional-pathtracing_amd/csrc
FL="--offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -fPIC -Iinclude -I$CS"
mkdir -p build/var
# a common unit is rebuilt when its source or any header (bdpt_ctx.h's Ctx layout included) is newer
newest_h=$(ls -t $CS/*.h include/bdpt/*.h | head -1)
for u in bdpt_wavefront.hip bdpt_scene.cpp dae_loader.cpp exr_loader.cpp; do
  [ build/var/$u.o -nt $CS/$u ] && [ build/var/$u.o -nt "$newest_h" ] || hipcc $FL -c $CS/$u -o build/var/$u.o &
done
for v in $VARIANTS; do
  name=${v%%:*}; flags=${v#*:}; flags=${flags//,/ }
  hipcc $FL $flags -c $CS/bdpt_hip.hip -o build/var/hip_$name.o &
done
wait
for v in $VARIANTS; do
  name=${v%%:*}
  hipcc $FL -shared -o build_var_$name.so build/var/hip_$name.o build/var/bdpt_wavefront.hip.o build/var/bdpt_scene.cpp.o \
    build/var/dae_loader.cpp.o build/var/exr_loader.cpp.o -lz || exit 1
done
ls -la build_var_*.so
