#!/bin/bash
# Traffic profile of one workload: kernel-trace pass + one --pmc pass per counter
# (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950), then summarise.
#   [LAUNCHES=L] tools/pmc_pass.sh KEY "args" KERNEL_REGEX ALG_BYTES_PER_STEP [SCRIPT]
# SCRIPT defaults to bench.py (run with --no-cpu --steps/--warmup); any other script gets "args" only.
key=$1; bargs=$2; kre=$3; alg=$4; script=${5:-bench.py}
d=gpurun_out/pmc_$key
rm -rf $d; mkdir -p $d
export TMPDIR=/tmp
if [ "$script" = bench.py ]; then
  a1="--no-cpu --steps 10 --warmup 3 $bargs"; a2="--no-cpu --steps 5 --warmup 1 $bargs"
else
  a1="$bargs"; a2="$bargs"
fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d/trace -o run -- python3 $script $a1 > $d/trace.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$kre" --output-format csv -d $d/fetch -o run -- python3 $script $a2 > $d/fetch.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$kre" --output-format csv -d $d/write -o run -- python3 $script $a2 > $d/write.log 2>&1 || exit $?
python3 tools/summarize_prof.py --trace $d/trace --fetch $d/fetch --write $d/write --kernel "$kre" --key "$key" --alg-bytes $alg --launches-per-step ${LAUNCHES:-1} --out gpurun_out/traffic.json
