set -e
mkdir -p gpurun_out/r05m
for cfg in "512 32 1" "512 16 1" "256 16 2" "256 8 2" "256 32 1" "512 32 1"; do
  set -- $cfg
  echo "TH=$1 NB=$2 WPC=$3"
  RTI_RBF_CHOL_TH=$1 RTI_RBF_CHOL_NB=$2 RTI_RBF_CHOL_WPC=$3 timeout -k 10 120 python -u tools/sweep_chol.py 400 2>&1 | grep -v amdgpu.ids
done
