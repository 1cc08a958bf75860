#!/bin/bash
# round 4: secp256k1 column form 2 (unmasked high columns) -- parity, then ecrecover / notary A/B
# against form 1 (variants/fe9c1) and the r03 library; then the pairing same-bytes A/B
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_secp256k1.py tests/test_gpu_notary.py tests/test_gpu_configs.py tests/test_gpu_collation.py -x -q --timeout 300 --timeout-method thread > gpurun_out/g4_tests.log 2>&1 || { tail -30 gpurun_out/g4_tests.log; exit 1; }
tail -1 gpurun_out/g4_tests.log
for rep in 1 2; do
  for lib in new fe9c1 base_r03; do
    if [ $lib = new ]; then L=""; else L="GSV_LIB_PATH=variants/$lib/libgsv.so"; fi
    env $L timeout -k 10 200 python bench.py --legs ecrecover,notary --steps 10 --no-cpu-baseline > gpurun_out/g4_$lib.json 2> gpurun_out/g4_$lib.err || { tail -5 gpurun_out/g4_$lib.err; exit 1; }
    python -c "
import json;d=json.loads([l for l in open('gpurun_out/g4_$lib.json') if l.startswith('{')][0])
n=d.get('notary',{}); r=d['roofline']
print('$lib rep $rep: ecrecover', round(d['value']/1e6,3), 'M/s kernel', r['kernel_avg_ms'], 'ms | notary', n.get('shards_per_s'), 'shards/s tx', n.get('tx_kernels_ms_per_step'))"
  done
done
bash tools/gpu_r04_miller.sh
