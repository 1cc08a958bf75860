#!/bin/bash
# A/B of k_chunk_level<BOTTOM>'s payload length (run through gpurun from the repo root):
#   base = in-tree: per-byte class compares (16 x two selects and an add)
#   pl   = variants/pl: counted four bytes at a time (popcount of high bits and of zero-byte flags)
#          (within noise and not kept: the change is quoted in profiles/r06/ab/bottom_payload.txt)
# Chunk-root / configs / collation GPU tests on the variant, the bench's chunk-root leg for each library
# four times in alternation, then one kernel trace per library (--pipeline 1).
set -o pipefail
O=gpurun_out/pl; mkdir -p $O
export PYTHONUNBUFFERED=1
GSV_LIB_PATH=variants/pl/libgsv.so timeout -k 10 500 python -u -m pytest tests/test_gpu_chunk_root.py tests/test_gpu_configs.py tests/test_gpu_collation.py -x -q --timeout 200 --timeout-method thread > $O/tests_pl.log 2>&1 || { echo "tests failed"; tail -30 $O/tests_pl.log; exit 1; }
tail -1 $O/tests_pl.log
for rep in 1 2 3 4; do
  for v in base pl; do
    if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
    GSV_LIB_PATH=$L timeout -k 10 300 python3 bench.py --legs chunk_root --no-cpu-baseline > $O/bench_${v}_r$rep.log 2>&1 || { echo "$v bench failed"; tail -5 $O/bench_${v}_r$rep.log; exit 1; }
    tail -1 $O/bench_${v}_r$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['chunk_root']
print('$v r$rep chunk_root', c['ms_per_step'], 'ms/step', round(100*2**20/c['ms_per_step']/1e6,1), 'GB/s, bottom', c['roofline']['kernel_avg_ms'], 'ms')"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base pl; do
  if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
  GSV_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/tr_$v -o run -- python3 bench.py --legs chunk_root --no-cpu-baseline --steps 6 --warmup 2 --pipeline 1 > $O/tr_$v.log 2>&1 || { echo "$v trace failed"; tail -5 $O/tr_$v.log; exit 1; }
  python3 - $O/tr_$v $v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "chunk_level" in r["Name"] or "chunk_top" in r["Name"]:
            print(sys.argv[2], "rocprofv3", r["Name"].split("(")[0], r["Calls"], "calls, avg", round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
