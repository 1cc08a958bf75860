#!/bin/bash
# r05 call I: round profile part B (pairing / notary PMC passes, then the default bench reading
# profiles/r05), plus the first-run artifact of the pipelined 8,192-check batch: the same streams re-used
# vs fresh streams, and the bench's own pairing leg at the N = 8 per-rank batch
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05i; mkdir -p $O
T="timeout -k 10"
SWEEP_REUSE_STREAMS=1 SWEEP_PIPELINE="3,3,3" $T 300 python -u tools/pairing_sweep.py 8192 > $O/pipe_reuse.txt 2>&1 || { echo pipe failed; tail $O/pipe_reuse.txt; exit 1; }
grep checks $O/pipe_reuse.txt | sed 's/^/reuse /'
$T 300 python bench.py --legs pairing --pairing-checks 8192 --no-cpu-baseline > $O/bench_pairing8192.json 2> $O/bench_pairing8192.err || { tail -5 $O/bench_pairing8192.err; exit 1; }
python -c "
import json;d=json.loads([l for l in open('$O/bench_pairing8192.json') if l.startswith('{')][0])
p=d['bn256_pairing']; print('bench pairing 8192/rank:', p['ms_per_step'], 'ms per batch, depth', p['pipeline_depth'], p['checks_per_s'])"
bash tools/round_profile_b.sh r05
