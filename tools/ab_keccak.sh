#!/bin/bash
# A/B of the Keccak-256 batch kernel: in-tree library vs variants/oldkec (tests, then the bench keccak leg).
set -o pipefail
for v in base oldkec base oldkec; do
  if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
  GSV_LIB_PATH=$L timeout -k 10 200 python -u -m pytest tests/test_gpu_keccak.py tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k_$v.log 2>&1 || { echo "$v tests failed"; tail -5 gpurun_out/k_$v.log; exit 1; }
  GSV_LIB_PATH=$L timeout -k 10 200 python bench.py --legs keccak --no-cpu-baseline --steps 20 > gpurun_out/kb_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/kb_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['collation_extras']['keccak256']; print('$v', d['hashes_per_s'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
done
