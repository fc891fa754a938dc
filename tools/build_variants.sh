#!/bin/bash
# Builds A/B variants of libbdpt_amd.so: VARIANTS="name:FLAGS name2:FLAGS2 ..." -> build_var_<name>.so
# (a flag -DBDPT_ONLY_MAXV=5 compiles one depth class only: m <= 5, a quarter of the compile time)
# Every translation unit of a variant is compiled with that variant's flags into its own
# directory (build/var/<name>/): a variant never links objects built with other macro settings or
# against an older bdpt_ctx.h (round 1's phase-profile run linked a stale bdpt_wavefront.hip.o whose
# Ctx layout predated the last Ctx change; bdpt_destroy -> wf_free then read c->wf at the wrong
# offset and the process crashed on its way out).
cd "$(dirname "$0")/.." || exit 1
CS=bidirectional-pathtracing_amd/csrc
FL="--offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -fPIC -Iinclude -I$CS"
UNITS="bdpt_hip.hip bdpt_reduce.hip bdpt_scene.cpp dae_loader.cpp exr_loader.cpp"
for v in $VARIANTS; do
  name=${v%%:*}; flags=${v#*:}; flags=${flags//,/ }
  mkdir -p build/var/$name
  for u in $UNITS; do
    hipcc $FL $flags -c $CS/$u -o build/var/$name/$u.o &
  done
done
wait
for v in $VARIANTS; do
  name=${v%%:*}
  objs=""
  for u in $UNITS; do objs="$objs build/var/$name/$u.o"; done
  hipcc $FL -shared -o build_var_$name.so $objs -lz -ldl || exit 1
done
ls -la build_var_*.so
