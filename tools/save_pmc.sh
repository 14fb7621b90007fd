#!/bin/bash
# Copy one PMC pass's summaries (tools/pmc_pass.sh output under gpurun_out/pmc_KEY) into profiles/ as
# TAG_pmc_KEY_{fetch_size,write_size,trace_kernel_stats}.csv (the counter CSVs filtered to the profiled kernel).
#   tools/save_pmc.sh TAG KEY...
tag=$1; shift
for key in "$@"; do
  d=gpurun_out/pmc_$key
  [ -d "$d" ] || { echo "no $d"; continue; }
  cp "$d/trace/run_kernel_stats.csv" "profiles/${tag}_pmc_${key}_trace_kernel_stats.csv"
  cp "$d/fetch/run_counter_collection.csv" "profiles/${tag}_pmc_${key}_fetch_size.csv"
  cp "$d/write/run_counter_collection.csv" "profiles/${tag}_pmc_${key}_write_size.csv"
done
