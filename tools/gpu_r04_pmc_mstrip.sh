# round 4: PMC counters of the matrix-core strip kernel at config-4 l4 / l3 / l2 (one pass each)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_ms
run() {  # $1 tag, $2 counters
  timeout -s KILL 90 rocprofv3 --pmc $2 --kernel-include-regex "corr_fwd_mstrip16" -d gpurun_out/pmc_ms/$1 -o run --output-format csv -- python tools/kbench.py --batch 16 --height 448 --width 1024 --dtype fp16 --levels 2,3,4 --ops corr --iters 5 > gpurun_out/pmc_ms/$1.log 2>&1 || { tail -5 gpurun_out/pmc_ms/$1.log; return 1; }
}
run sq "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE" || exit 1
run fetch "FETCH_SIZE" || exit 1
run write "WRITE_SIZE" || exit 1
python - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc_ms/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        geo = k[k.find("Geo<"):k.find(">")+1] if "Geo<" in k else k[:40]
        acc[(geo, r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k, round(sum(v) / len(v)), len(v))
PY
