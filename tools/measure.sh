#!/bin/bash
# Measurement pass (TAG=rNN) on one MI355X box: every bench config under
# rocprofv3 --kernel-trace --stats (bench line + kernel stats of the same command),
# the L3-resident relight for comparison, and PMC traffic passes.
# Output under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03}
mkdir -p $out
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 $secs "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 $out/$name.log
  case $rc in 124|134|137|139) echo "fatal rc=$rc"; exit $rc;; esac
  return 0
}
for c in ${CONFIGS:-c3 c2 c4 c10 c5 c9 c6 c7 c8 c8n200}; do
  budget=8; [ $c = c3 ] && budget=16; extra=""; case $c in c8n200) extra="--no-cpu";; esac
  run bench_$c$SUFFIX 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$c$SUFFIX -o run -- \
      python3 bench.py --config $c --cpu-budget $budget $extra $BENCH_ARGS
done
if [ -z "$SKIP_EXTRA" ]; then
  run bench_c5_hot 200 python3 bench.py --config c5 --map-sets 1 --no-cpu
  run bench_c9_hot 200 python3 bench.py --config c9 --map-sets 1 --no-cpu
fi
exit 0
