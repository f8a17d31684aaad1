set -o pipefail
mkdir -p gpurun_out/wb_batch
for B in 4 6 7 8 10 12 16; do
  timeout -k 10 200 python tools/kbench.py --batch $B --levels 3,4 --ops none --backward > gpurun_out/wb_batch/b$B.txt 2>&1 || { tail gpurun_out/wb_batch/b$B.txt; exit 1; }
  echo "B=$B: $(grep -o '"level": [0-9], "op": "warp_bwd", "shape": [^]]*], "us": [0-9.]*' gpurun_out/wb_batch/b$B.txt | sed 's/"shape": \[[^]]*\], //;s/"level": //;s/"op": //;s/"us": //' | tr '\n' ' ')"
done
