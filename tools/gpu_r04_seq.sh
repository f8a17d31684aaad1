# round 4: the l4 strip correlation behind the l4 warp (the bench step's order) vs alone
set -o pipefail
mkdir -p gpurun_out/seq
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/kbench.py --levels 4 --ops corr,warp,seq > gpurun_out/seq/kb.txt 2>&1 || exit 1; grep level gpurun_out/seq/kb.txt
PWC_DEBUG=strip=0 timeout -k 10 120 python tools/kbench.py --levels 4 --ops corr,seq > gpurun_out/seq/kb_stream.txt 2>&1 || exit 1; grep level gpurun_out/seq/kb_stream.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/seq/t_corr -o run --output-format csv -- python tools/kbench.py --levels 4 --ops corr > /dev/null 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/seq/t_seq -o run --output-format csv -- python tools/kbench.py --levels 4 --ops seq > /dev/null 2>&1 || exit 1
for f in gpurun_out/seq/t_corr/run_kernel_stats.csv gpurun_out/seq/t_seq/run_kernel_stats.csv; do echo $f; grep -E "corr_fwd_strip|warp_fwd_kernel" $f | cut -d, -f1-4 | cut -c1-40,150-; done
timeout -k 10 60 tools/strip_bench 300 | tail -1
