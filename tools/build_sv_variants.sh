#!/bin/bash
# Builds resident-kernel experiment libraries: only pf_inst_sv (k_resident) is
# recompiled with the variant's flags and linked with the standard objects.
#   tools/build_sv_variants.sh name1:"-DFLAG ..." name2:"..."   -> build/libpf_hip_<name>.so
set -e
cd "$(dirname "$0")/../particle_filters_amd/csrc"
B=../../build/csrc
OTHERS="$B/pf_diag.o $B/pf_engine.o $B/pf_inst_linear.o $B/pf_inst_l96.o $B/pf_inst_mat.o $B/pf_inst_dyn.o $B/pf_ledh.o"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-pass-failed $flags \
      -c pf_inst_sv.hip -o $B/sv_$name.o &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ../../build/libpf_hip_$name.so $B/sv_$name.o $OTHERS &&
    echo "built $name" ) &
done
wait
