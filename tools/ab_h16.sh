#!/bin/bash
# same-box A/B of the 8-bit h16 fit: tools/ab_h16.sh <name> <config> (ab/<name> from tools/ab_build.sh)
name=$1; cfg=$2
for r in 1 2; do
  echo "== ab/$name"; RTI_PKG_DIR=ab/$name/smartphone-based-rti_amd timeout -k 10 120 python -u tools/sweep_h16.py --config $cfg --batches 4 2>&1 | grep -v "amdgpu.ids\|^{" || exit 1
  echo "== tree"; timeout -k 10 120 python -u tools/sweep_h16.py --config $cfg --batches 4 2>&1 | grep -v "amdgpu.ids\|^{" || exit 1
done
