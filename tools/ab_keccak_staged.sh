#!/bin/bash
# (Record of the r06 run: the staged kernel and the GSV_KECCAK_STAGED switch were removed after it; profiles/r06/ab/keccak_staged_lds.txt.)
# A/B of the Keccak-256 batch kernel (run through gpurun from the repo root):
#   base  = in-tree: k_keccak256_staged (two messages per lane, next block staged in LDS by
#           global_load_lds_dwordx4 while the current one is permuted)
#   ktail = k_keccak256 with the whole-group final-block loader (variants/ktail, GSV_KECCAK_STAGED=0)
# Keccak / boundary / collation tests on the in-tree library, then keccak_scale (400 k / 1.6 M / 6.4 M
# messages) and the bench's keccak leg for each, twice in alternation.
set -o pipefail
O=gpurun_out/ks; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_keccak.py tests/test_gpu_boundary.py tests/test_gpu_collation.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in base ktail; do
    if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
    GSV_LIB_PATH=$L timeout -k 10 120 python tools/keccak_scale.py 400000 1600000 6400000 > $O/scale_${v}_$r.txt 2>&1 || { echo "$v scale failed"; tail -5 $O/scale_${v}_$r.txt; exit 1; }
    grep messages $O/scale_${v}_$r.txt | sed "s/^/$v /"
    GSV_LIB_PATH=$L timeout -k 10 200 python bench.py --legs keccak --no-cpu-baseline --steps 20 > $O/bench_${v}_$r.log 2>&1 || { echo "$v bench failed"; tail -5 $O/bench_${v}_$r.log; exit 1; }
    tail -1 $O/bench_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['collation_extras']['keccak256']; print('$v leg', d['hashes_per_s'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])"
  done
done
