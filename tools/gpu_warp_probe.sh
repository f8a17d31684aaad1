set -o pipefail
mkdir -p gpurun_out/wp
for fs in 0 0.5 2 8; do
timeout -k 10 120 python tools/kbench.py --ops warp --levels 2,3,4 --flow-scale $fs --tag "fs$fs" 2>/dev/null >> gpurun_out/wp/kb.txt || exit 1
done
timeout -k 10 200 python tools/kbench.py --ops none --backward --levels 0,1,2,3,4 --tag bwd 2>/dev/null >> gpurun_out/wp/kb.txt || exit 1
cat gpurun_out/wp/kb.txt
