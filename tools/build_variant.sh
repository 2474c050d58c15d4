#!/bin/bash
# Build lib/libilqg_amd_<name>.so: one translation unit recompiled with extra
# -D flags, linked with the standard objects (A/B runs via ILQG_LIB=...).
#   tools/build_variant.sh NAME TU(kernels_rollout|kernels_fd|riccati) "-DFLAG=0 ..."
set -e
# (run `make -C ilqg-mujoco_amd` first: a variant carries the sources' digest, build/srcsha.o,
# which ilqg_amd.lib() checks)
cd "$(dirname "$0")/../ilqg-mujoco_amd"
name=$1; tu=$2; defs=$3
ROCM=/opt/rocm
FLAGS="-std=c++20 -O3 -fPIC -ffp-contract=off -fno-fast-math -I../include -Icsrc -Icsrc/device -Icsrc/model --offload-arch=gfx950 -munsafe-fp-atomics"
mkdir -p build/var
$ROCM/bin/hipcc $FLAGS $defs -x hip -c csrc/device/$tu.hip -o build/var/${tu}_$name.o
objs=""
for o in kernels_fd kernels_fd32 kernels_rollout riccati; do
  if [ "$o" = "$tu" ]; then objs="$objs build/var/${tu}_$name.o"; else objs="$objs build/$o.o"; fi
done
$ROCM/bin/hipcc $FLAGS -shared -Wl,--version-script=csrc/exports.map -Wl,-Bsymbolic -o lib/libilqg_amd_$name.so \
  $objs build/capi.o build/mjcf.o build/setconst.o build/srcsha.o
echo "built lib/libilqg_amd_$name.so"
