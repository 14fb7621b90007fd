#!/bin/bash
# same-box A/B of the Cholesky solve: tools/ab_chol.sh <name> [N ...]  (ab/<name> from tools/ab_build.sh)
name=$1; shift
for r in 1 2; do
  echo "== ab/$name"; RTI_PKG_DIR=ab/$name/smartphone-based-rti_amd timeout -k 10 120 python -u tools/sweep_chol.py "$@" 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== tree"; timeout -k 10 120 python -u tools/sweep_chol.py "$@" 2>&1 | grep -v amdgpu.ids || exit 1
done
