set -o pipefail
mkdir -p gpurun_out/fin
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fin/pytest.log 2>&1 || { tail -30 gpurun_out/fin/pytest.log; exit 1; }
tail -1 gpurun_out/fin/pytest.log
for l in 4 3 2 1 0; do timeout -k 10 200 python tools/variants.py --op corr_bwd --level $l 2>&1 | grep us | cut -c1-110 || exit 1; done
timeout -k 10 300 python tools/train_bench.py > gpurun_out/fin/train.json 2> gpurun_out/fin/train.err || { tail gpurun_out/fin/train.err; exit 1; }
python -c "import json; t=json.load(open('gpurun_out/fin/train.json')); print('train', t['value'], t['ms_per_step'], t['checks']['self_check']['ok'])"
