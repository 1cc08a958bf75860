#!/bin/bash
# r05 call D: pairing GPU tests with the two-wave lines kernel (default) and the one-wave one; configs[4]
# sweeps lines w2 on/off; the N = 8 rank batch at depths 3/4 repeated in one process; the notary leg's
# tx-kernel time with and without the chunk roots forked beside it (variants/nfork0)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05d; mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests/test_gpu_bn256.py "tests/test_gpu_configs.py::test_configs4_full_batch_verdicts" \
   tests/test_gpu_stream_contract.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lw in 1 0; do
  GSV_BN_LINES_W2=$lw SWEEP_CASES="0,,;2,," $T 240 python -u tools/pairing_sweep.py 65536 16384 8192 > $O/sweep_lw$lw.txt 2>&1 || { echo sweep $lw failed; tail $O/sweep_lw$lw.txt; exit 1; }
  GSV_BN_LINES_W2=$lw SWEEP_PIPELINE="2,3,2,3" $T 300 python -u tools/pairing_sweep.py 65536 >> $O/sweep_lw$lw.txt 2>&1 || { echo pipe $lw failed; tail $O/sweep_lw$lw.txt; exit 1; }
  GSV_BN_LINES_W2=$lw SWEEP_PIPELINE="3,4,3,4" $T 300 python -u tools/pairing_sweep.py 8192 >> $O/sweep_lw$lw.txt 2>&1 || { echo pipe8k $lw failed; tail $O/sweep_lw$lw.txt; exit 1; }
  grep checks $O/sweep_lw$lw.txt | sed "s/^/lines_w2=$lw /"
done
for lib in new nfork0; do
  if [ $lib = new ]; then L=""; else L="GSV_LIB_PATH=variants/$lib/libgsv.so"; fi
  env $L $T 240 python bench.py --legs notary --steps 10 --no-cpu-baseline > $O/notary_$lib.json 2> $O/notary_$lib.err || { tail -5 $O/notary_$lib.err; exit 1; }
  python -c "
import json;d=json.loads([l for l in open('$O/notary_$lib.json') if l.startswith('{')][0])
n=d.get('notary',{}); print('$lib notary', n.get('shards_per_s'), 'shards/s tx kernels', n.get('tx_kernels_ms_per_step'), 'ms/step')"
done
