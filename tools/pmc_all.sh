#!/bin/bash
# PMC traffic passes (tools/pmc_pass.sh: kernel trace + separate FETCH_SIZE / WRITE_SIZE passes) for every
# bench config whose line carries roofline.traffic; merged afterwards into profiles/traffic.json by
# tools/merge_traffic.py (which stamps the commit and refuses entries whose kernel sources changed).
set -o pipefail
export TMPDIR=/tmp
rm -f gpurun_out/traffic.json
run() {  # key "bench args" kernel-regex alg-bytes-per-step launches-per-step
  echo "=== pmc $1"
  LAUNCHES=$5 timeout -k 10 400 tools/pmc_pass.sh "$1" "$2" "$3" "$4" > gpurun_out/pmc_$1.log 2>&1
  local rc=$?
  echo "=== pmc $1 rc=$rc"; tail -2 gpurun_out/pmc_$1.log
  case $rc in 124|134|137|139) echo "fatal rc=$rc"; exit $rc;; esac
  return 0
}
for k in ${KEYS:-c3 c2 c4 c3u8 c4u8 c10 c6 c7 c5 c9}; do
  case $k in
    c3) run c3-auto-pixel "--config c3" fit_shared_valu 3516825600 4;;
    c2) run c2-auto-pixel "--config c2" fit_shared_valu 464486400 1;;
    c4) run c4-auto-pixel "--config c4" fit_shared_tile_w 21499084800 6;;
    c3u8) run c3-auto-pixel-u8 "--config c3 --in-dtype u8" fit_h16 1028505600 1;;
    c4u8) run c4-auto-pixel-u8 "--config c4 --in-dtype u8" fit_h16 6569164800 1;;
    c3q8) run c3-q8-pixel-u8 "--config c3 --in-dtype u8 --kernel q8" fit_q8 1028505600 1;;
    c4q8) run c4-q8-pixel-u8 "--config c4 --in-dtype u8 --kernel q8" fit_q8 6569164800 1;;
    c10) run c10 "--config c10" fit_shared_residual_k 3550003200 8;;
    c6) run c6 "--config c6" fit_perpixel_cam 3516825600 1;;
    c7) run c7-split16 "--config c7" apply_op 6464000000 1;;
    c3pm) run c3-auto-pixel-pm "--config c3 --stack pixel" fit_pm_vgen 3516825600 4;;
    c4pm) run c4-auto-pixel-pm "--config c4 --stack pixel" fit_pm_direct 21499084800 1;;
    c8n400) LAUNCHES=1 timeout -k 10 600 tools/pmc_pass.sh c8n400-chol "400" rbf_solve_chol 1792000000 \
              tools/sweep_chol.py > gpurun_out/pmc_c8n400-chol.log 2>&1
            echo "=== pmc c8n400-chol rc=$?"; tail -2 gpurun_out/pmc_c8n400-chol.log;;
    c5) run c5 "--config c5" relight_eval_major 232243200 1;;
    c9) run c9 "--config c9" relight_frame_k 248832000 1;;
  esac
done
exit 0
