#!/bin/bash
# r05 call AX: GPU suite, smoke and the driver's bench command on the build with the Keccak launch knob
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05ax; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
echo smoke ok
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); print('value', d['value'], 'chunk', d['chunk_root']['ms_per_step'], 'pairing', d['bn256_pairing']['ms_per_step'], 'notary', d['notary']['ms_per_step'], 'keccak', d['collation_extras']['keccak256']['ms_per_step'])"
