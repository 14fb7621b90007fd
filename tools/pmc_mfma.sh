#!/bin/bash
# Matrix-core utilisation of one bench workload: one --pmc pass with the MFMA busy
# counter and the GRBM active clock (1 SQ + 1 GRBM counter: well inside one pass),
# a kernel-trace pass for the duration, then summarise into gpurun_out/mfma.json.
#   tools/pmc_mfma.sh KEY "bench args" KERNEL_REGEX N_MFMA_PER_LAUNCH CYCLES_PER_MFMA
key=$1; bargs=$2; kre=$3; nmfma=$4; cyc=$5
d=gpurun_out/mfma_$key
rm -rf $d; mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d/trace -o run -- python3 bench.py --no-cpu --steps 10 --warmup 3 $bargs > $d/trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$kre" --output-format csv -d $d/pmc -o run -- python3 bench.py --no-cpu --steps 5 --warmup 1 $bargs > $d/pmc.log 2>&1 || exit $?
python3 tools/summarize_mfma.py --trace $d/trace --pmc $d/pmc --kernel "$kre" --key "$key" \
    --n-mfma $nmfma --cycles-per-mfma $cyc --out gpurun_out/mfma.json
