set -o pipefail
for a in 3 7 11 15; do
  if [ $a = 0 ]; then L=""; else L=$PWD/scratch/abl$a/libpwc_hotpath.so; fi
  PWC_HOTPATH_LIB=$L PWC_GRP_CFG=C timeout -k 10 120 python tools/kbench.py --levels 0,1,2,3 --iters 40 2>/dev/null | grep corr_fwd | sed "s/^/abl$a /" || exit 1
done
