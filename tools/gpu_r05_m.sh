#!/bin/bash
# r05 call M: queue lanes (gsv_api.hip shape_run) - GPU tests of the pipelined / stream paths, the
# stream-set experiment with lanes on and off, the bench's pairing leg at the N = 8 per-rank batch, and
# a clean exit under rocprofv3
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05m; mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
SWEEP_STREAM_SETS="0,1,2;1,2,3;0,4,8;0,1,2,3;4,5,6,7" $T 300 python -u tools/pairing_sweep.py 8192 > $O/sets_lanes.txt 2>&1 && grep streams $O/sets_lanes.txt && \
GSV_LANES=0 SWEEP_STREAM_SETS="0,1,2;1,2,3;0,4,8;0,1,2,3;4,5,6,7" $T 300 python -u tools/pairing_sweep.py 8192 > $O/sets_nolanes.txt 2>&1 && grep streams $O/sets_nolanes.txt && \
$T 300 python bench.py --legs pairing --pairing-checks 8192 --no-cpu-baseline > $O/bench_pairing8192.json 2> $O/bench_pairing8192.err && python3 -c "
import json; d=json.load(open('$O/bench_pairing8192.json'))['bn256_pairing']; print('bench pairing 8192/rank lanes:', round(1e3*d['checks_per_rank']/d['checks_per_s']*d['checks']/d['checks_per_rank'],3), 'ms per batch, depth', d['pipeline_depth'])" && \
GSV_LANES=0 $T 300 python bench.py --legs pairing --pairing-checks 8192 --no-cpu-baseline > $O/bench_pairing8192_nolanes.json 2>> $O/bench_pairing8192.err && python3 -c "
import json; d=json.load(open('$O/bench_pairing8192_nolanes.json'))['bn256_pairing']; print('bench pairing 8192/rank no lanes:', round(1e3*d['checks_per_rank']/d['checks_per_s']*d['checks']/d['checks_per_rank'],3), 'ms per batch')" && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
$T 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --legs pairing,notary --no-cpu-baseline > $O/bench_traced.json 2> $O/bench_traced.err && echo "traced exit ok" && \
$T 300 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err && python3 -c "
import json; d=json.load(open('$O/bench_default.json')); print('default bench', d['value'], d['collation_GBps'], d['bn256_pairing']['checks_per_s'], d['notary']['shards_per_s'])"
