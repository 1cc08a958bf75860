#!/bin/bash
# round 4: final-exponentiation machine (no private segment) -- GPU tests, then new/base timing
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_bn256.py tests/test_gpu_configs.py tests/test_gpu_partition.py -k "pairing or g2 or synth or precompile or configs4 or partition or ranks" -x -v --timeout 400 --timeout-method thread > gpurun_out/g1_tests.log 2>&1 || { tail -40 gpurun_out/g1_tests.log; exit 1; }
tail -3 gpurun_out/g1_tests.log
SWEEP_CASES="0,,;0,0,;0,1," timeout -k 10 300 python tools/pairing_sweep.py 65536 8192 > gpurun_out/g1_sweep_new.txt 2>&1 && cat gpurun_out/g1_sweep_new.txt || exit 1
GSV_LIB_PATH=variants/base_r03/libgsv.so SWEEP_CASES="0,,;0,0,;0,1," timeout -k 10 300 python tools/pairing_sweep.py 65536 8192 > gpurun_out/g1_sweep_base.txt 2>&1 && cat gpurun_out/g1_sweep_base.txt || exit 1
SWEEP_PIPELINE=2,3 timeout -k 10 300 python tools/pairing_sweep.py 65536 8192 > gpurun_out/g1_pipe_new.txt 2>&1 && cat gpurun_out/g1_pipe_new.txt || exit 1
GSV_LIB_PATH=variants/base_r03/libgsv.so SWEEP_PIPELINE=2,3 timeout -k 10 300 python tools/pairing_sweep.py 65536 8192 > gpurun_out/g1_pipe_base.txt 2>&1 && cat gpurun_out/g1_pipe_base.txt
# fused trie top at wave priority 3 (GSV_TOP_PRIO) beside the notary's recovery and the pipelined chunk roots
for pr in 0 1; do
  GSV_TOP_PRIO=$pr timeout -k 10 300 python bench.py --legs chunk_root,notary --steps 10 --no-cpu-baseline > gpurun_out/g1_prio$pr.json 2> gpurun_out/g1_prio$pr.err || { tail gpurun_out/g1_prio$pr.err; exit 1; }
  python -c "
import json;d=json.loads([l for l in open('gpurun_out/g1_prio$pr.json') if l.startswith('{')][0])
c=d.get('chunk_root',{}); n=d.get('notary',{})
print('prio $pr chunk', c.get('collation_GBps'), c.get('ms_per_step'), 'notary', n.get('shards_per_s'), n.get('ms_per_step'), n.get('tx_kernels_ms_per_step'))"
  GSV_TOP_PRIO=$pr timeout -k 10 300 python tools/notary_sweep.py 13 100 > gpurun_out/g1_nsweep_prio$pr.txt 2>&1 && cat gpurun_out/g1_nsweep_prio$pr.txt || exit 1
done
# prepare at the one-wave budget (k_bn_lines, no spills) for every batch size
GSV_BN_CONC=1 SWEEP_CASES="0,," timeout -k 10 300 python tools/pairing_sweep.py 65536 > gpurun_out/g1_conc1.txt 2>&1 && cat gpurun_out/g1_conc1.txt
