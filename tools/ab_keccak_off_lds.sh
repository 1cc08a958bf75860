#!/bin/bash
# (Record of the r06 run; the LDS form and its GSV_KECCAK_OFF_LDS switch were not kept: profiles/r06/ab/keccak_off_lds.txt.)
# A/B of k_keccak256's message bounds after the block-count reordering (run through gpurun from the
# repo root): base = carried through LDS with the reordering; koff0 = re-loaded from HBM by the sorted
# lane (variants/koff0, GSV_KECCAK_OFF_LDS=0).  Keccak / boundary tests on base, then keccak_scale and
# the bench's keccak leg per library, twice in alternation.
set -o pipefail
O=gpurun_out/ko; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_keccak.py tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in base koff0; do
    if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
    GSV_LIB_PATH=$L timeout -k 10 120 python tools/keccak_scale.py 400000 1600000 > $O/scale_${v}_$r.txt 2>&1 || { echo "$v scale failed"; tail -5 $O/scale_${v}_$r.txt; exit 1; }
    grep messages $O/scale_${v}_$r.txt | sed "s/^/$v /"
    GSV_LIB_PATH=$L timeout -k 10 200 python bench.py --legs keccak --no-cpu-baseline --steps 20 > $O/bench_${v}_$r.log 2>&1 || { echo "$v bench failed"; tail -5 $O/bench_${v}_$r.log; exit 1; }
    tail -1 $O/bench_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['collation_extras']['keccak256']; print('$v leg', d['hashes_per_s'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])"
  done
done
