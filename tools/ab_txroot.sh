#!/bin/bash
# A/B of the generic DeriveSha (tx root) leg: in-tree library vs variants/oldleaf (tests, then the bench tx_root leg).
set -o pipefail
for v in base oldleaf base oldleaf; do
  if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
  GSV_LIB_PATH=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_chunk_root.py tests/test_gpu_collation.py tests/test_gpu_keccak.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$v.log 2>&1 || { echo "$v tests failed"; tail -5 gpurun_out/t_$v.log; exit 1; }
  GSV_LIB_PATH=$L timeout -k 10 200 python bench.py --legs tx_root,keccak --no-cpu-baseline --steps 20 > gpurun_out/tb_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/tb_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['collation_extras']; print('$v', d['tx_root']['txs_per_s'], d['tx_root']['ms_per_step'], d['keccak256']['hashes_per_s'])"
done
