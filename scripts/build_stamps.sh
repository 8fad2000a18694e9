#!/bin/bash
# Timing-diagnostic build of the halo conv (gemm2.hip with -DIRX_HALO_STAMPS: in-kernel s_memtime segment sums in the
# HALO == 4 loop, read back by irx_debug_halo_stamps) linked with the regular objects into
# scripts/_skdbg/libirx_stamps.so (git-ignored and listed in .gpurunignore: drop that line for a stamps run).  Used by
# scripts/halo_diag.py --stamps.
set -eu
cd "$(dirname "$0")/.."
python3 -m image_restoration_and_enhancement_amd.build > /dev/null
B=image_restoration_and_enhancement_amd/build
mkdir -p scripts/_skdbg
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -DIRX_HALO_STAMPS -c \
  image_restoration_and_enhancement_amd/csrc/gemm2.hip -o /tmp/gemm2_stamps.o
objs=$(ls $B/*.o | grep -v gemm2.hip.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs /tmp/gemm2_stamps.o -o scripts/_skdbg/libirx_stamps.so
ls -la scripts/_skdbg
