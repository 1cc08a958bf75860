#!/bin/bash
# A/B of the digest permutation (keccak_dev.cuh keccakf_split_digest: the last round computes only the
# four digest words) in k_keccak256, the chunk-root levels and the header hash (run through gpurun
# from the repo root):
#   base  = in-tree
#   kold  = the library before it, variants/kold
# Keccak / chunk-root / collation GPU tests on the in-tree library, then the bench's keccak and
# chunk-root legs for each library twice in alternation, then one kernel trace per library.
set -o pipefail
O=gpurun_out/kd; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_keccak.py tests/test_gpu_chunk_root.py tests/test_gpu_collation.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in base kold; do
    if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
    GSV_LIB_PATH=$L timeout -k 10 300 python3 bench.py --legs chunk_root,keccak --no-cpu-baseline > $O/bench_${v}_r$rep.log 2>&1 || { echo "$v bench failed"; tail -5 $O/bench_${v}_r$rep.log; exit 1; }
    tail -1 $O/bench_${v}_r$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['chunk_root']; k=d['collation_extras']['keccak256']
print('$v chunk_root', c['ms_per_step'], 'ms/step', c['level_kernels_ms_per_step'], 'level ms', 'frac', c['roofline']['frac'],
      '| keccak', k['permutations_per_s'], 'perm/s frac', k['roofline']['frac'], 'pipelined', k['roofline'].get('frac_pipelined'))"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base kold; do
  if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
  GSV_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/tr_$v -o run -- python3 bench.py --legs chunk_root,keccak --no-cpu-baseline --steps 6 --warmup 2 --pipeline 1 > $O/tr_$v.log 2>&1 || { echo "$v trace failed"; tail -5 $O/tr_$v.log; exit 1; }
  python3 - $O/tr_$v $v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "keccak" in r["Name"] or "chunk_level" in r["Name"] or "chunk_top" in r["Name"]:
            print(sys.argv[2], "rocprofv3", r["Name"].split("(")[0], r["Calls"], "calls, avg", round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
