#!/bin/bash
# Timing-diagnostic builds of the K = 320 streaming GEMM (gemm_sk.hip with IRX_SK_DBG = 1 / 2 / 3 / 4 / 5 / 6 / 7, see
# the kernel) linked with the regular objects into scripts/_skdbg/libirx_skdbgN.so (git-ignored; travels to the GPU box).
# Used only by scripts/kprof.py --lib; results of these libraries are wrong by design.
set -eu
cd "$(dirname "$0")/.."
python3 -m image_restoration_and_enhancement_amd.build > /dev/null
B=image_restoration_and_enhancement_amd/build
mkdir -p scripts/_skdbg
for d in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -DIRX_SK_DBG=$d -c \
    image_restoration_and_enhancement_amd/csrc/gemm_sk.hip -o /tmp/gemm_sk_dbg$d.o
  objs=$(ls $B/*.o | grep -v gemm_sk.hip.o)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs /tmp/gemm_sk_dbg$d.o -o scripts/_skdbg/libirx_skdbg$d.so
done
ls -la scripts/_skdbg
