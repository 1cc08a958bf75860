#!/bin/bash
# the round-end checks on one box: every -m gpu test, smoke(), then the default bench line
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-full}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -40 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/$T/bench.log 2>&1 || { tail -20 gpurun_out/$T/bench.log; exit 1; }
python - <<'PY'
import json,sys
T=sys.argv[1] if len(sys.argv)>1 else None
PY
python -c "
import json
d=json.loads([l for l in open('gpurun_out/$T/bench.log') if l.startswith('{')][-1])
print('value', d['value'], 'frac', d['roofline']['frac'], 'kernel', d['roofline']['kernel_avg_ms'])
print('chunk', d['chunk_root']['collation_GBps'], 'pairing', d['bn256_pairing']['checks_per_s'], 'notary', d['notary']['shards_per_s'], d['notary']['tx_kernels_ms_per_step'])
"
