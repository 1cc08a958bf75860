#!/bin/bash
# r05 call N: pipelines on dedicated-queue streams (gsv_stream_create) - stream-contract / pipeline GPU
# tests, the pairing sweep at 8,192, the bench's pairing leg at the N = 8 per-rank batch, the notary
# sweep with side streams on shared / own queues, the default bench, and a clean exit under rocprofv3
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05n; mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
SWEEP_PIPELINE="3,3,4,3" $T 300 python -u tools/pairing_sweep.py 8192 > $O/sweep_dedicated.txt 2>&1 && grep checks $O/sweep_dedicated.txt && \
$T 300 python bench.py --legs pairing --pairing-checks 8192 --no-cpu-baseline > $O/bench_pairing8192.json 2> $O/bench_pairing8192.err && python3 -c "
import json; d=json.load(open('$O/bench_pairing8192.json'))['bn256_pairing']; print('bench pairing 8192/rank:', d['ms_per_step'], 'ms per batch, depth', d['pipeline_depth'])" && \
$T 300 python -u tools/notary_sweep.py 100 > $O/notary_sweep.txt 2>&1 && cat $O/notary_sweep.txt | grep -v amdgpu.ids && \
GSV_SIDE_OWN_QUEUE=1 $T 300 python -u tools/notary_sweep.py 100 > $O/notary_sweep_ownside.txt 2>&1 && cat $O/notary_sweep_ownside.txt | grep -v amdgpu.ids && \
$T 300 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err && python3 -c "
import json; d=json.load(open('$O/bench_default.json')); print('default bench', d['value'], d['collation_GBps'], d['bn256_pairing']['checks_per_s'], d['notary']['shards_per_s'])" && \
GSV_SIDE_OWN_QUEUE=1 $T 300 python bench.py --no-cpu-baseline --legs notary > $O/bench_notary_ownside.json 2> $O/bench_notary_ownside.err && python3 -c "
import json; d=json.load(open('$O/bench_notary_ownside.json')); print('notary own side queues', d['notary']['shards_per_s'])" && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
$T 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --legs chunk_root,pairing,notary --no-cpu-baseline > $O/bench_traced.json 2> $O/bench_traced.err && echo "traced exit ok"
