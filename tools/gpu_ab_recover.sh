#!/bin/bash
# recovery A/B on one box: the recovery GPU tests, then ecrecover / notary legs alternating between the
# in-tree library ("new") and variants/<variant>/libgsv.so, two repetitions.  Usage: <variant> <tag>
set -o pipefail
export PYTHONUNBUFFERED=1
V=$1; T=${2:-ab}
timeout -k 10 600 python -u -m pytest tests/test_gpu_secp256k1.py tests/test_gpu_notary.py tests/test_gpu_configs.py tests/test_gpu_collation.py tests/test_gpu_boundary.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2; do
  for lib in new $V; do
    if [ $lib = new ]; then L=""; else L="GSV_LIB_PATH=variants/$lib/libgsv.so"; fi
    env $L timeout -k 10 200 python bench.py --legs ecrecover,notary --steps 10 --no-cpu-baseline > gpurun_out/${T}_${lib}_$rep.json 2> gpurun_out/${T}_$lib.err || { tail -5 gpurun_out/${T}_$lib.err; exit 1; }
    python -c "
import json;d=json.loads([l for l in open('gpurun_out/${T}_${lib}_$rep.json') if l.startswith('{')][0])
n=d.get('notary',{}); r=d['roofline']
print('$lib rep $rep: ecrecover', round(d['value']/1e6,3), 'M/s kernel', r['kernel_avg_ms'], 'ms | notary', n.get('shards_per_s'), 'shards/s tx', n.get('tx_kernels_ms_per_step'))"
  done
done
