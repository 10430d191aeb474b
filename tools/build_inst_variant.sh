#!/bin/bash
# Rebuild one instantiation unit with extra flags and link it with the standard objects:
#   tools/build_inst_variant.sh <name> <pf_inst_xxx> "<flags>"  ->  build/libpf_hip_<name>.so
set -e
cd "$(dirname "$0")/../particle_filters_amd/csrc"
B=../../build/csrc
name=$1; unit=$2; flags=$3
OTHERS=""
for o in pf_diag pf_engine pf_inst_linear pf_inst_l96 pf_inst_mat pf_inst_sv pf_inst_dyn pf_ledh; do
  [ "$o" = "$unit" ] || OTHERS="$OTHERS $B/$o.o"
done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-pass-failed $flags \
  -c $unit.hip -o $B/v_${name}_$unit.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ../../build/libpf_hip_$name.so $B/v_${name}_$unit.o $OTHERS
echo "built $name"
