#!/bin/bash
# (Record of the r06 run; k_generic_lane was not kept: profiles/r06/ab/generic_lane.txt.)
# A/B of the generic-only heights' kernel (k_generic_lane: a branch's child loads issued together) (run through gpurun from the repo root):
#   base  = in-tree: k_generic_lane for heights of generic nodes only, in lane mode
#   gold  = the library before it (those heights in k_chunk_level, one child's loads after another), variants/gold
# Collation / boundary / chunk-root GPU tests on the in-tree library, then the bench's tx-root leg for
# each library twice in alternation, then one kernel trace per library for the level kernels' durations.
set -o pipefail
O=gpurun_out/gl; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_collation.py tests/test_gpu_boundary.py tests/test_gpu_chunk_root.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in base gold; do
    if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
    GSV_LIB_PATH=$L timeout -k 10 300 python3 bench.py --legs tx_root --no-cpu-baseline > $O/bench_${v}_r$rep.log 2>&1 || { echo "$v bench failed"; tail -5 $O/bench_${v}_r$rep.log; exit 1; }
    tail -1 $O/bench_${v}_r$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['collation_extras']['tx_root']; print('$v leg', d['txs_per_s'], 'txs/s', d['ms_per_step'], 'ms/step')"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base gold; do
  if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
  GSV_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/tr_$v -o run -- python3 bench.py --legs tx_root --no-cpu-baseline --steps 3 --warmup 1 > $O/tr_$v.log 2>&1 || { echo "$v trace failed"; tail -5 $O/tr_$v.log; exit 1; }
  python3 - $O/tr_$v $v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "derive_leaf" in r["Name"] or "chunk_level" in r["Name"] or "generic_lane" in r["Name"]:
            print(sys.argv[2], "rocprofv3", r["Name"].split("(")[0], r["Calls"], "calls, avg", round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
