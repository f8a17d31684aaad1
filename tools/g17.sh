set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/g17; : > gpurun_out/g17/pmc.txt
for LV in 2 3; do
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAVES" "GRBM_GUI_ACTIVE"; do
OUT=gpurun_out/g17/l${LV}_$(echo $CTRS | cut -c1-12 | tr ' ' '_'); mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-include-regex "corr_fwd_rows" -d $OUT -o run --output-format csv -- python tools/variants.py --op corr --level $LV --iters 5 > $OUT/log.txt 2>&1 || { tail $OUT/log.txt; exit 1; }
python - >> gpurun_out/g17/pmc.txt <<PY
import csv, glob, collections
f = glob.glob("$OUT/**/run_counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    acc[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print("l$LV", k, round(sum(v)/len(v)))
PY
done; done
cat gpurun_out/g17/pmc.txt
