# per-kernel split of the backward (rocprofv3 kernel stats over kbench --backward)
set -o pipefail
mkdir -p gpurun_out/bwdp
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for l in 0 2 4; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/bwdp/l$l -o run --output-format csv -- python tools/kbench.py --ops none --backward --levels $l --iters 20 > gpurun_out/bwdp/l$l.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/bwdp/l$l/run_kernel_stats.csv')):
    print('l$l', r['Name'][:70], r['Calls'], r['AverageNs'])"
done
