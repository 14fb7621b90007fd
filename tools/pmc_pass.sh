#!/bin/bash
# Traffic profile of one bench workload: kernel-trace pass + one --pmc pass per counter
# (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950), then summarise.
#   tools/pmc_pass.sh KEY "bench args" KERNEL_REGEX ALG_BYTES
key=$1; bargs=$2; kre=$3; alg=$4
d=gpurun_out/pmc_$key
rm -rf $d; mkdir -p $d
export TMPDIR=/tmp
rocprofv3 --kernel-trace --stats --output-format csv -d $d/trace -o run -- python3 bench.py --no-cpu --steps 10 --warmup 3 $bargs > $d/trace.log 2>&1 || exit $?
rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$kre" --output-format csv -d $d/fetch -o run -- python3 bench.py --no-cpu --steps 5 --warmup 1 $bargs > $d/fetch.log 2>&1 || exit $?
rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$kre" --output-format csv -d $d/write -o run -- python3 bench.py --no-cpu --steps 5 --warmup 1 $bargs > $d/write.log 2>&1 || exit $?
python3 tools/summarize_prof.py --trace $d/trace --fetch $d/fetch --write $d/write --kernel "$kre" --key "$key" --alg-bytes $alg --out gpurun_out/traffic.json
