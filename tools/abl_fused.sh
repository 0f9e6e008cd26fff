#!/bin/bash
# Ablation builds of the fused pass (tooling only): tools/_ablf/libgnk_f<mask>.so with -DGNK_FDBG=<mask>.
# Use with GNK_LIB=tools/_ablf/libgnk_f<mask>.so python tools/kbench.py --kernels fused ...
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$R/tools/_ablf"
for m in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DGNK_FDBG=$m \
    -I"$R/include" -o "$R/tools/_ablf/libgnk_f$m.so" "$R/gauss_newton_via_generalized_krylov_subspaces_amd/csrc/gnk_kernels.hip" &
done
wait
