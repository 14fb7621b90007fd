#!/bin/bash
# Print per-kernel VGPR/SGPR/scratch/occupancy for a HIP source (gfx950).
# usage: tools/resource_usage.sh file.hip [extra hipcc flags]
src=$1; shift
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c "$src" -o /dev/null -Rpass-analysis=kernel-resource-usage "$@" 2>&1 \
 | grep -E "Function Name|VGPRs:|TotalSGPRs|ScratchSize|Occupancy" \
 | sed -E 's/.*remark: [^ ]+ +//; s/ \[-Rpass.*//' \
 | paste - - - - - | c++filt | sed -E 's/\(anonymous namespace\):://g'
