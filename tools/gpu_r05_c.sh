#!/bin/bash
# r05 call C: recovery / notary GPU tests on the tree with the shifted comb digits and the notary's LDS
# chunk staging; A/B of the ecrecover + notary legs against variants/comb0 (r04 comb digits) and
# variants/ntst0 (notary without staging), interleaved twice; the N = 8 pairing batch re-swept with a
# proper warm-up
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05c; mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests/test_gpu_secp256k1.py tests/test_gpu_notary.py tests/test_gpu_configs.py \
   tests/test_gpu_collation.py tests/test_gpu_boundary.py tests/test_gpu_partition.py tests/test_gpu_bn256.py \
   -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for lib in new comb0 ntst0; do
    if [ $lib = new ]; then L=""; else L="GSV_LIB_PATH=variants/$lib/libgsv.so"; fi
    env $L $T 240 python bench.py --legs ecrecover,notary --steps 10 --no-cpu-baseline > $O/ab_${lib}_$rep.json 2> $O/ab_$lib.err || { tail -5 $O/ab_$lib.err; exit 1; }
    python -c "
import json;d=json.loads([l for l in open('$O/ab_${lib}_$rep.json') if l.startswith('{')][0])
n=d.get('notary',{}); r=d['roofline']
print('$lib rep $rep: ecrecover', round(d['value']/1e6,3), 'M/s kernel', r['kernel_avg_ms'], 'ms | notary', n.get('shards_per_s'), 'shards/s tx', n.get('tx_kernels_ms_per_step'))"
  done
done
for k in 1 2 4; do
  GSV_BN_PAIRS_PER_LANE=$k SWEEP_KEEP_LAYOUT=1 SWEEP_PIPELINE="3,4" $T 240 python -u tools/pairing_sweep.py 8192 > $O/sweep8192_k$k.txt 2>&1 || { echo sweep $k failed; tail $O/sweep8192_k$k.txt; exit 1; }
  grep checks $O/sweep8192_k$k.txt | sed "s/^/k=$k /"
done
SWEEP_PIPELINE="3,4" $T 240 python -u tools/pairing_sweep.py 8192 > $O/sweep8192_auto.txt 2>&1 && grep checks $O/sweep8192_auto.txt | sed "s/^/auto /"
