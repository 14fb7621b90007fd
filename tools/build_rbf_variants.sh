#!/bin/bash
# Build librti.so variants of the per-pixel RBF kernel with phases disabled, for timing
# splits (tools/time_rbf_perpixel.py with RTI_LIBRARY=...).  Not used by the product.
#   tools/build_rbf_variants.sh   ->  tools/probe/librti_<name>.so
set -e
cd "$(dirname "$0")/../smartphone-based-rti_amd"
make -j8 >/dev/null
OUT=../tools/probe
OBJS="build/rti_host.cpp.o build/rti_fit.hip.o build/rti_perpixel.hip.o build/rti_relight.hip.o build/rti_operator.hip.o"
build() {  # name, defines...
  name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function "$@" -c csrc/rti_rbf.hip -o build/rbf_$name.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/librti_$name.so $OBJS build/rbf_$name.o
}
build norefine -DRBF_MAX_REFINE=0
build nolu -DRBF_MAX_REFINE=0 -DRBF_PROBE_NO_LU
build refine1 -DRBF_MAX_REFINE=1
build exacteval -DRBF_EXACT_EVAL
build timing -DRBF_TIMING
