#!/bin/bash
# SQ stall / instruction-mix and FETCH passes for one bench workload (each pass its own run; gfx950 slot
# limits: 8 SQ, FETCH_SIZE alone).  tools/pmc_sq.sh KEY KERNEL_REGEX "bench args"
key=$1; kre=$2; bargs=$3
d=gpurun_out/pmcsq_$key
rm -rf $d; mkdir -p $d
export TMPDIR=/tmp
a="--no-cpu --no-parity --steps 5 --warmup 1 $bargs"
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex "$kre" --output-format csv -d $d/$name -o run -- \
    python3 bench.py $a > $d/$name.log 2>&1 || { echo "pass $name failed rc=$?"; exit 1; }
}
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES
run sq2 SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
echo "pmc $key done"
