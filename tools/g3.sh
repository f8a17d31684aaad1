set -o pipefail
mkdir -p gpurun_out/g3
# warm the clocks first (2 s of back-to-back launches), then the probe
timeout -k 10 60 ./tools/sbench 2000 > /dev/null 2>&1
timeout -k 10 60 ./tools/issue_probe > gpurun_out/g3/issue.txt 2>&1 || exit 1
cat gpurun_out/g3/issue.txt
cd /tmp && export TMPDIR=/tmp
for abl in 0 14; do
  PWC_DEBUG=stream_abl=$abl timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT -d $GRAFT_REPO_ROOT/gpurun_out/g3/pmc$abl -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/sbench 50 > $GRAFT_REPO_ROOT/gpurun_out/g3/pmc$abl.log 2>&1 || { tail $GRAFT_REPO_ROOT/gpurun_out/g3/pmc$abl.log; exit 1; }
done
echo ok
