# A/B of two library builds on one box: kbench of one op/level under PWC_HOTPATH_LIB=$1 and the
# in-tree library, alternating.  usage: bash tools/gpu_ab_lib.sh OTHER_LIB "kbench args"
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  PWC_HOTPATH_LIB=$1 timeout -k 10 120 python tools/kbench.py $2 > gpurun_out/ab_a.log 2>&1 || exit 1; echo "other: $(grep corr_fwd gpurun_out/ab_a.log | tr '\n' ' ')"
  timeout -k 10 120 python tools/kbench.py $2 > gpurun_out/ab_b.log 2>&1 || exit 1; echo "tree:  $(grep corr_fwd gpurun_out/ab_b.log | tr '\n' ' ')"
done
