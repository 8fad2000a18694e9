#!/bin/bash
# Timing-diagnostic build of gemm2.hip (-DIRX_HALO_STAMPS: the option gemm_dbg knock-outs of every gemm2 loop, which the
# product library compiles out, and in-kernel s_memtime segment sums in the
# HALO == 4 loop, read back by irx_debug_halo_stamps) linked with the regular objects into
# scripts/_skdbg/libirx_stamps.so (git-ignored and listed in .gpurunignore: drop that line for a stamps run).  Used by
# scripts/halo_diag.py --stamps and, with IRX_LIB=scripts/_skdbg/libirx_stamps.so, kbench.py dbg1/dbg2/dbg3.
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
