# round 4: matrix-core strip output stores, nontemporal (tree) vs plain (build/ab_plain):
# WRITE_SIZE per launch and kbench time at config-4 l2..l4, alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mss
K="--batch 16 --height 448 --width 1024 --dtype fp16 --levels 2,3,4 --ops corr"
for v in tree plain; do
  if [ $v = plain ]; then export PWC_HOTPATH_LIB=build/ab_plain/libpwc_hotpath.so; else unset PWC_HOTPATH_LIB; fi
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "corr_fwd_mstrip16" -d gpurun_out/mss/$v -o run --output-format csv -- python tools/kbench.py $K --iters 5 > gpurun_out/mss/$v.log 2>&1 || { tail -5 gpurun_out/mss/$v.log; exit 1; }
done
unset PWC_HOTPATH_LIB
python - <<'PY'
import csv, glob, collections
for v in ("tree", "plain"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/mss/{v}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]; acc[k[k.find("Geo<"):k.find(">")+1]].append(float(r["Counter_Value"]))
    print(v, {k: round(sum(x) / len(x)) for k, x in sorted(acc.items())})
PY
for i in 1 2; do
  PWC_HOTPATH_LIB=build/ab_plain/libpwc_hotpath.so timeout -k 10 120 python tools/kbench.py $K > gpurun_out/mss/a.log 2>&1 || { tail gpurun_out/mss/a.log; exit 1; }
  echo "plain: $(grep -o '"level": [0-9], "op": "corr_fwd".*"us": [0-9.]*' gpurun_out/mss/a.log | sed 's/"op".*"us"/us/' | tr '\n' ' ')"
  timeout -k 10 120 python tools/kbench.py $K > gpurun_out/mss/b.log 2>&1 || { tail gpurun_out/mss/b.log; exit 1; }
  echo "nt:    $(grep -o '"level": [0-9], "op": "corr_fwd".*"us": [0-9.]*' gpurun_out/mss/b.log | sed 's/"op".*"us"/us/' | tr '\n' ' ')"
done
