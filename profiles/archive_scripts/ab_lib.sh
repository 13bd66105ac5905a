#!/bin/bash
# Build one kernel source file at a given git revision into ab/lib<name>_<rev>.so, for
# same-box A/B microbenchmarks that load two builds of one kernel side by side
# (scripts/bench_fused_attn.py --lib). Usage: scripts/ab_lib.sh <rev> <kernel basename>
set -euo pipefail
rev=$1; name=$2
mkdir -p ab/src_$rev
git show "$rev:csrc/kernels/$name.hip" > ab/src_$rev/$name.hip
git show "$rev:csrc/kernels/common.h" > ab/src_$rev/common.h
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-gpu-rdc -shared \
  -I ab/src_$rev ab/src_$rev/$name.hip -o ab/lib${name}_$rev.so
echo ab/lib${name}_$rev.so
