#!/bin/bash
# (Record of the r06 run; the change it measured was not kept: profiles/r06/ab/notary_lead_bytes.txt.)
# A/B of k_notary_tx's integer-item lead bytes and V read as dwords together (run through gpurun from the repo root):
#   base = in-tree: the seven integer items' lead bytes read together, V as two dwords
#   dold = the library before it (dependent byte reads), variants/dold
# Notary / partition GPU tests on the in-tree library; then per library, twice in alternation: the
# 100- and 13-shard steps one at a time (no side streams), the 13-shard step four deep (the N = 8 share)
# and the bench's notary leg; and one kernel trace per library for k_blob_index's own duration.
set -o pipefail
O=gpurun_out/di; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_notary.py tests/test_gpu_partition.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in base dold; do
    if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
    GSV_LIB_PATH=$L GSV_MAX_SIDE_STREAMS=0 NOTARY_DEPTHS=1 NOTARY_STEPS=12 timeout -k 10 300 python3 tools/notary_sweep.py 100 13 > $O/${v}_d1_r$rep.txt 2>&1 || { echo "$v sweep failed"; tail $O/${v}_d1_r$rep.txt; exit 1; }
    grep shards $O/${v}_d1_r$rep.txt | sed "s/^/$v /"
    GSV_LIB_PATH=$L NOTARY_DEPTHS=4 timeout -k 10 300 python3 tools/notary_sweep.py 13 > $O/${v}_d4_r$rep.txt 2>&1 || { echo "$v sweep4 failed"; tail $O/${v}_d4_r$rep.txt; exit 1; }
    grep shards $O/${v}_d4_r$rep.txt | sed "s/^/$v /"
    GSV_LIB_PATH=$L timeout -k 10 300 python3 bench.py --legs notary --no-cpu-baseline > $O/bench_${v}_r$rep.log 2>&1 || { echo "$v bench failed"; tail -5 $O/bench_${v}_r$rep.log; exit 1; }
    tail -1 $O/bench_${v}_r$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['notary']; print('$v leg', d['shards_per_s'], 'shards/s', d.get('ms_per_step'), 'ms/step')"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base dold; do
  if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
  GSV_LIB_PATH=$L GSV_MAX_SIDE_STREAMS=0 NOTARY_DEPTHS=1 NOTARY_STEPS=6 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/tr_$v -o run -- python3 tools/notary_sweep.py 100 > $O/tr_$v.log 2>&1 || { echo "$v trace failed"; tail -5 $O/tr_$v.log; exit 1; }
  find $O/tr_$v -name "*kernel_stats.csv" -exec grep -h "k_blob_index" {} \; | cut -d, -f1-4 | sed "s/^/$v /"
done
