#!/bin/bash
# Ablation builds of libgnk.so (tooling only): tools/_abl/libgnk_<mask>.so with -DGNK_SDBG=<mask>.
# Use with GNK_LIB=tools/_abl/libgnk_<mask>.so python tools/kbench.py ...
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$R/tools/_abl"
for m in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DGNK_SDBG=$m \
    -I"$R/include" -o "$R/tools/_abl/libgnk_$m.so" "$R/gauss_newton_via_generalized_krylov_subspaces_amd/csrc/gnk_kernels.hip" &
done
wait
