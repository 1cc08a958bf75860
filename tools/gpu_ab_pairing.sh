#!/bin/bash
# pairing-leg A/B on one box: the in-tree library ("new") against variants/<variant>/libgsv.so, two
# interleaved repetitions of the bench's pairing leg.  Usage: <variant> <tag>
set -o pipefail
V=$1; T=${2:-abp}
timeout -k 10 300 python -u -m pytest tests/test_gpu_bn256.py -x -q --timeout 250 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -20 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2; do
  for lib in new $V; do
    if [ $lib = new ]; then L=""; else L="GSV_LIB_PATH=variants/$lib/libgsv.so"; fi
    env $L timeout -k 10 200 python bench.py --legs pairing --steps 6 --no-cpu-baseline > gpurun_out/${T}_${lib}_$rep.json 2> gpurun_out/${T}_$lib.err || { tail -5 gpurun_out/${T}_$lib.err; exit 1; }
    python -c "
import json;d=json.loads([l for l in open('gpurun_out/${T}_${lib}_$rep.json') if l.startswith('{')][0])
p=d['bn256_pairing']
print('$lib rep $rep:', p['checks_per_s'], 'lines/miller/final', p['prepare_kernel_ms'], p['miller_kernel_ms'], p['final_exp_kernel_ms'])"
  done
done
